// Fused optimizer step of the training hot path: torch.optim.SGD (momentum, nesterov,
// per-group weight decay; reference config.py:307-333 via core/trainer.py:124
// `self.scaler.step(self.optimizer)`) and ModelEMA.update (reference utils/ema.py:46-58,
// trainer.py:127) in ONE HBM pass over the parameters, instead of ~10 torch foreach
// kernels (+ one per BN buffer).  Per element, the arithmetic follows torch's
// _multi_tensor_sgd / the EMA's mul_/add_ op by op (one rounding each):
//   g  = g + wd * p                  (_foreach_add(grads, params, alpha=wd))
//   b  = first ? g : b * m + g       (_foreach_mul_(bufs, m); _foreach_add_(bufs, grads))
//   g' = nesterov ? g + m * b : b    (_foreach_add_(grads, bufs, alpha=m))
//   p  = p - lr * g'                 (_foreach_add_(params, grads, alpha=-lr))
//   e  = e * d + (1 - d) * p         (ema: v *= d; v += (1 - d) * msd[k])
// EMA-only segments (param == NULL) carry the BN running statistics.
#include "yxh_common.hpp"
#include "yoloxhip.h"

namespace yxh {

constexpr int kOptPer = 4;                // elements per thread (loads issued together)
constexpr int kOptChunk = 256 * kOptPer;  // elements per workgroup

__global__ __launch_bounds__(256) void sgd_ema_step(const yxh_opt_seg* __restrict__ segs,
                                                    const int32_t* __restrict__ chunks, yxh_opt_hparams h) {
    const int seg = chunks[2 * blockIdx.x], ci = chunks[2 * blockIdx.x + 1];
    const yxh_opt_seg s = segs[seg];
    const long long base = (long long)ci * kOptChunk + threadIdx.x;
    long long idx[kOptPer];
    bool ok[kOptPer];
#pragma unroll
    for (int k = 0; k < kOptPer; ++k) {
        idx[k] = base + k * 256;
        ok[k] = idx[k] < s.n;
    }
    const bool ema = h.do_ema && s.ema;
    if (s.param) {
        float p[kOptPer], g[kOptPer], b[kOptPer], e[kOptPer];
#pragma unroll
        for (int k = 0; k < kOptPer; ++k) {
            p[k] = ok[k] ? s.param[idx[k]] : 0.0f;
            g[k] = ok[k] ? s.grad[idx[k]] : 0.0f;
            b[k] = ok[k] && !h.first_step ? s.buf[idx[k]] : 0.0f;
            e[k] = ok[k] && ema ? s.ema[idx[k]] : 0.0f;
        }
        const float lr = h.lr[s.group & 3], m = h.momentum;
#pragma unroll
        for (int k = 0; k < kOptPer; ++k) {
            float gg = s.weight_decay != 0.0f ? __builtin_fmaf(s.weight_decay, p[k], g[k]) : g[k];
            const float bb = h.first_step ? gg : __fadd_rn(__fmul_rn(b[k], m), gg);
            gg = h.nesterov ? __builtin_fmaf(m, bb, gg) : bb;
            p[k] = __builtin_fmaf(-lr, gg, p[k]);
            b[k] = bb;
            e[k] = __builtin_fmaf(h.ema_omd, p[k], __fmul_rn(e[k], h.ema_d));
        }
#pragma unroll
        for (int k = 0; k < kOptPer; ++k) {
            if (!ok[k]) continue;
            s.param[idx[k]] = p[k];
            s.buf[idx[k]] = b[k];
            if (ema) s.ema[idx[k]] = e[k];
        }
    } else if (ema) {
        float v[kOptPer], e[kOptPer];
#pragma unroll
        for (int k = 0; k < kOptPer; ++k) {
            v[k] = ok[k] ? s.src[idx[k]] : 0.0f;
            e[k] = ok[k] ? s.ema[idx[k]] : 0.0f;
        }
#pragma unroll
        for (int k = 0; k < kOptPer; ++k)
            if (ok[k]) s.ema[idx[k]] = __builtin_fmaf(h.ema_omd, v[k], __fmul_rn(e[k], h.ema_d));
    }
}

}  // namespace yxh

int yxh_opt_chunk_elems(void) { return yxh::kOptChunk; }

int yxh_sgd_ema_step(const yxh_opt_seg* segs, const int32_t* chunks, int32_t nchunks,
                     const yxh_opt_hparams* hp, void* stream) {
    if (!segs || !chunks || !hp || nchunks < 0) {
        yxh::set_error("sgd_ema_step: null table / hyper-parameters");
        return YXH_EINVAL;
    }
    if (nchunks == 0) return YXH_OK;
    hipLaunchKernelGGL(yxh::sgd_ema_step, dim3(nchunks), dim3(256), 0, (hipStream_t)stream, segs, chunks, *hp);
    return yxh::check_hip(hipGetLastError(), "sgd_ema_step launch");
}
