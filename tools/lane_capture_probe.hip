// Probe (GPU box): multi-stream hipGraph capture with N lanes, the pattern of
// yxh_graph_create_lanes (runtime.cpp): fork event on lane 0, every other lane waits on it, ops
// on their lanes with cross-lane event waits, every lane joined back into lane 0, end capture,
// instantiate, replay twice, check the counts.  Usage: lane_capture_probe NLANES EMPTY_LANES
// (EMPTY_LANES: how many of the last lanes get no op at all -- their only captured work is the
// fork wait).  Prints one line and exits 0 on success; a failing HIP call exits 1.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                      \
    do {                                                                           \
        hipError_t e_ = (x);                                                       \
        if (e_ != hipSuccess) {                                                    \
            printf("FAIL %s: %s\n", #x, hipGetErrorString(e_));                    \
            fflush(stdout);                                                        \
            return 1;                                                              \
        }                                                                          \
    } while (0)

__global__ void bump(int* p, int i) {
    if (threadIdx.x == 0 && blockIdx.x == 0) p[i] += 1;
}

int main(int argc, char** argv) {
    const int nl = argc > 1 ? atoi(argv[1]) : 4, empty = argc > 2 ? atoi(argv[2]) : 0;
    const int per = 3, n = nl * per;
    int* d = nullptr;
    CK(hipMalloc(&d, n * sizeof(int)));
    CK(hipMemset(d, 0, n * sizeof(int)));
    std::vector<hipStream_t> st(nl);
    for (auto& s : st) CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipEvent_t fork;
    CK(hipEventCreateWithFlags(&fork, hipEventDisableTiming));
    std::vector<hipEvent_t> ev(n), join(nl);
    for (auto& e : ev) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    for (auto& e : join) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    CK(hipStreamBeginCapture(st[0], hipStreamCaptureModeThreadLocal));
    CK(hipEventRecord(fork, st[0]));
    for (int l = 1; l < nl; ++l) CK(hipStreamWaitEvent(st[l], fork, 0));
    // op i on lane i % nl (lanes >= nl - empty get none); op i also waits on op i - nl - 1's event
    // when that one ran on another lane (a cross-lane edge per op, as the planner's deps)
    std::vector<int> lane_of(n, -1);
    int want = 0;
    for (int i = 0; i < n; ++i) {
        const int l = i % nl;
        if (l >= nl - empty) continue;
        const int j = i - nl - 1;
        if (j >= 0 && lane_of[j] >= 0 && lane_of[j] != l) CK(hipStreamWaitEvent(st[l], ev[j], 0));
        hipLaunchKernelGGL(bump, dim3(1), dim3(64), 0, st[l], d, i);
        CK(hipGetLastError());
        CK(hipEventRecord(ev[i], st[l]));
        lane_of[i] = l;
        ++want;
    }
    for (int l = 1; l < nl; ++l) {
        CK(hipEventRecord(join[l], st[l]));
        CK(hipStreamWaitEvent(st[0], join[l], 0));
    }
    hipGraph_t g;
    CK(hipStreamEndCapture(st[0], &g));
    hipGraphExec_t ge;
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    CK(hipGraphLaunch(ge, st[0]));
    CK(hipGraphLaunch(ge, st[0]));
    CK(hipStreamSynchronize(st[0]));
    std::vector<int> h(n);
    CK(hipMemcpy(h.data(), d, n * sizeof(int), hipMemcpyDeviceToHost));
    int got = 0, bad = 0;
    for (int i = 0; i < n; ++i) {
        got += h[i] / 2;
        bad += lane_of[i] >= 0 ? h[i] != 2 : h[i] != 0;
    }
    printf("lanes %d empty %d: ops %d, replayed ok %d, bad %d\n", nl, empty, want, got, bad);
    fflush(stdout);
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(g));
    return bad ? 1 : 0;
}
