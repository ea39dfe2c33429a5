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
//
// With a GradScaler (--fp16, trainer.py:111-114) the whole scaler.step / scaler.update
// sequence runs on the device with no host sync (torch's GradScaler reads found_inf with
// .item() before deciding to step):
//   amp_found_inf : any non-finite scaled gradient -> found_inf = 1
//                   (_amp_foreach_non_finite_check_and_unscale_'s check)
//   sgd_ema_step  : g = g * inv_scale, inv_scale = float(1 / double(scale)), written back
//                   like torch's in-place unscale; the SGD update is skipped when
//                   found_inf (params and momentum untouched); the EMA update always runs
//                   (the reference calls ema_model.update after every scaler.step)
//   amp_update    : _amp_update_scale_ (backoff on inf, growth every `interval` steps)
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
        const bool amp = h.amp_scale != nullptr;
        const bool skip = amp && *h.amp_found_inf != 0.0f;  // scaler.step skips the optimizer
        const float inv_scale = amp ? (float)(1.0 / (double)*h.amp_scale) : 1.0f;
        float p[kOptPer], g[kOptPer], b[kOptPer], e[kOptPer];
#pragma unroll
        for (int k = 0; k < kOptPer; ++k) {
            p[k] = ok[k] ? s.param[idx[k]] : 0.0f;
            g[k] = ok[k] ? s.grad[idx[k]] : 0.0f;
            b[k] = ok[k] && !h.first_step ? s.buf[idx[k]] : 0.0f;
            e[k] = ok[k] && ema ? s.ema[idx[k]] : 0.0f;
        }
        if (amp) {
#pragma unroll
            for (int k = 0; k < kOptPer; ++k) {
                if (inv_scale != 1.0f) g[k] = __fmul_rn(g[k], inv_scale);
                if (ok[k]) const_cast<float*>(s.grad)[idx[k]] = g[k];  // unscaled gradient stays in .grad
            }
        }
        const float lr = h.lr[s.group & 3], m = h.momentum;
        if (!skip) {
#pragma unroll
            for (int k = 0; k < kOptPer; ++k) {
                float gg = s.weight_decay != 0.0f ? __builtin_fmaf(s.weight_decay, p[k], g[k]) : g[k];
                const float bb = h.first_step ? gg : __fadd_rn(__fmul_rn(b[k], m), gg);
                gg = h.nesterov ? __builtin_fmaf(m, bb, gg) : bb;
                p[k] = __builtin_fmaf(-lr, gg, p[k]);
                b[k] = bb;
            }
        }
#pragma unroll
        for (int k = 0; k < kOptPer; ++k) e[k] = __builtin_fmaf(h.ema_omd, p[k], __fmul_rn(e[k], h.ema_d));
#pragma unroll
        for (int k = 0; k < kOptPer; ++k) {
            if (!ok[k]) continue;
            if (!skip) {
                s.param[idx[k]] = p[k];
                s.buf[idx[k]] = b[k];
            }
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

// found_inf = 1 if any parameter gradient holds a non-finite value (found_inf zeroed by
// the launcher first).  Plain vector stores of the same value: idempotent, no atomics.
__global__ __launch_bounds__(256) void amp_found_inf(const yxh_opt_seg* __restrict__ segs,
                                                     const int32_t* __restrict__ chunks, float* found_inf) {
    const int seg = chunks[2 * blockIdx.x], ci = chunks[2 * blockIdx.x + 1];
    const yxh_opt_seg s = segs[seg];
    if (!s.param) return;
    const long long base = (long long)ci * kOptChunk + threadIdx.x;
    bool bad = false;
#pragma unroll
    for (int k = 0; k < kOptPer; ++k) {
        const long long i = base + k * 256;
        if (i < s.n) bad |= !__builtin_isfinite(s.grad[i]);
    }
    if (__any(bad) && (threadIdx.x & 63) == 0) *found_inf = 1.0f;
}

// torch._amp_update_scale_ (one thread)
__global__ void amp_update(float* scale, int32_t* tracker, const float* found_inf, double growth, double backoff,
                           int interval) {
    if (*found_inf != 0.0f) {
        *scale = (float)((double)*scale * backoff);
        *tracker = 0;
    } else {
        const int ok = *tracker + 1;
        if (ok == interval) {
            const float ns = (float)((double)*scale * growth);
            if (__builtin_isfinite(ns)) *scale = ns;
            *tracker = 0;
        } else {
            *tracker = ok;
        }
    }
}

__global__ void zero_flag(float* f) { *f = 0.f; }

}  // namespace yxh

int yxh_opt_chunk_elems(void) { return yxh::kOptChunk; }

int yxh_amp_found_inf(const yxh_opt_seg* segs, const int32_t* chunks, int32_t nchunks, float* found_inf,
                      void* stream) {
    if (!segs || !chunks || !found_inf || nchunks < 0) {
        yxh::set_error("amp_found_inf: null table / output");
        return YXH_EINVAL;
    }
    // a kernel, not hipMemsetAsync: memset nodes in a captured step broke later replays (train.py)
    hipLaunchKernelGGL(yxh::zero_flag, dim3(1), dim3(1), 0, (hipStream_t)stream, found_inf);
    int rc = yxh::check_hip(hipGetLastError(), "zero found_inf");
    if (rc || nchunks == 0) return rc;
    hipLaunchKernelGGL(yxh::amp_found_inf, dim3(nchunks), dim3(256), 0, (hipStream_t)stream, segs, chunks,
                       found_inf);
    return yxh::check_hip(hipGetLastError(), "amp_found_inf launch");
}

int yxh_amp_update_scale(float* scale, int32_t* growth_tracker, const float* found_inf, double growth_factor,
                         double backoff_factor, int32_t growth_interval, void* stream) {
    if (!scale || !growth_tracker || !found_inf || growth_interval <= 0) {
        yxh::set_error("amp_update_scale: bad arguments");
        return YXH_EINVAL;
    }
    hipLaunchKernelGGL(yxh::amp_update, dim3(1), dim3(1), 0, (hipStream_t)stream, scale, growth_tracker, found_inf,
                       growth_factor, backoff_factor, (int)growth_interval);
    return yxh::check_hip(hipGetLastError(), "amp_update_scale launch");
}

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
