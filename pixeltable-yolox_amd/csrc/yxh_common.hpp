// Shared device/host helpers for libyoloxhip (gfx950 only).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "yoloxhip.h"

namespace yxh {

typedef __bf16 bf16;
typedef _Float16 f16;
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

// Wavefront width on CDNA4 (never 32).
constexpr int kWave = 64;

template <typename T> __device__ __forceinline__ float to_f32(T v) { return (float)v; }
template <typename T> __device__ __forceinline__ T from_f32(float v) { return (T)v; }

// 16-byte chunk of T (8 bf16/f16, 4 f32): the unit of every global/LDS move.
template <typename T> struct Chunk { static constexpr int N = 16 / sizeof(T); };

// PRECISE: the fp32 parity path uses the correctly-rounded-ish expf and an IEEE
// divide; the bf16/f16 paths (outputs rounded to 8/11 bits) use the hardware exp and
// one v_rcp_f32 (~1 ulp) -- the IEEE divide sequence alone was ~10 VALU ops per output
// and the SiLU epilogue up to ~25% of a wide 1x1 conv's time (tools/pw_probe.py).
template <bool PRECISE>
__device__ __forceinline__ float silu(float v) {
    if (PRECISE) return v / (1.0f + expf(-v));
    // one v_mul + v_exp_f32 (2^x) + v_add + v_rcp_f32 + v_mul; exp2 overflow -> rcp(inf) = 0
    return v * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(v * -1.4426950408889634f));
}

// SiLU of 4 values: the operations of silu<false> (so bit-identical results) on a vector, which
// gfx950 issues as packed-fp32 pairs (v_pk_mul_f32 / v_pk_add_f32): half the non-transcendental
// issue slots of four scalar silu calls -- the epilogues of the 1x1 / stem kernels are VALU-heavy
__device__ __forceinline__ f32x4 silu4(f32x4 v) {
    const f32x4 t = v * -1.4426950408889634f;
    f32x4 e = {__builtin_amdgcn_exp2f(t.x), __builtin_amdgcn_exp2f(t.y), __builtin_amdgcn_exp2f(t.z),
               __builtin_amdgcn_exp2f(t.w)};
    e = e + 1.0f;
    const f32x4 r = {__builtin_amdgcn_rcpf(e.x), __builtin_amdgcn_rcpf(e.y), __builtin_amdgcn_rcpf(e.z),
                     __builtin_amdgcn_rcpf(e.w)};
    return v * r;
}

// four fp32 values -> four 16-bit values packed in two dwords by two v_cvt_pk_{bf16,f16}_f32 (the same
// round-to-nearest-even as from_f32; written per element, the compiler sometimes converted each value
// alone and re-packed the halves with v_perm / shifts)
template <typename T>
__device__ __forceinline__ uint2 pack4(f32x4 v) {
    typedef float f32x2 __attribute__((ext_vector_type(2)));
    typedef T t16x2 __attribute__((ext_vector_type(2)));
    const t16x2 a = __builtin_convertvector((f32x2{v[0], v[1]}), t16x2);
    const t16x2 b = __builtin_convertvector((f32x2{v[2], v[3]}), t16x2);
    return make_uint2(__builtin_bit_cast(uint32_t, a), __builtin_bit_cast(uint32_t, b));
}

template <bool PRECISE = false>
__device__ __forceinline__ float apply_act(float v, int act) {
    switch (act) {
        case YXH_ACT_SILU: return silu<PRECISE>(v);
        case YXH_ACT_RELU: return v > 0.0f ? v : 0.0f;
        case YXH_ACT_LRELU: return v > 0.0f ? v : 0.1f * v;
        default: return v;
    }
}

// Host-side error channel (thread-local message, see runtime.cpp).
void set_error(const char* fmt, ...);
int check_hip(hipError_t e, const char* what);
// compute units of the GPU (queried once per process; 256 on MI355X): persistent grids
// are sized from it, one block (or BPC blocks) per CU
int device_cus();

}  // namespace yxh

#define YXH_CHECK_ARG(cond, ...)              \
    do {                                      \
        if (!(cond)) {                        \
            ::yxh::set_error(__VA_ARGS__);    \
            return YXH_EINVAL;                \
        }                                     \
    } while (0)

#define YXH_CHECK_LAUNCH(what) \
    do { int _rc = ::yxh::check_hip(hipGetLastError(), what); if (_rc) return _rc; } while (0)
