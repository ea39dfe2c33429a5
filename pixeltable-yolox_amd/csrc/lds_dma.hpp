// LDS-DMA helpers shared by the buffer-descriptor conv kernels (conv_r3.hip, conv_ws.hip).
//
// Every DMA is `buffer_load_dwordx4 ... offen lds` through a raw buffer descriptor: the
// per-lane byte offset is range-checked by the hardware, so an offset beyond the
// descriptor's range (kDmaOob) lands zeros in LDS -- zero padding without a branch.
// The instruction is issued from inline asm because hipcc's own buffer/global_load_lds
// builtins make it put `s_waitcnt vmcnt(0)` in front of every later ds_read; kernels
// order LDS reads behind the DMA with counted vmcnt waits + raw s_barrier instead.
#pragma once

#include "yxh_common.hpp"

namespace yxh {
namespace dma {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr uint32_t kOob = 0x80000000u;  // beyond any descriptor range: reads 0

template <int N>
__device__ __forceinline__ void wait_vm() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// all of this wave's LDS traffic done, then the workgroup barrier
__device__ __forceinline__ void barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

// raw buffer descriptor (stride 0, byte-range checked): out-of-range loads return 0
__device__ __forceinline__ u32x4 srd(const void* base, uint32_t bytes) {
    const uint64_t a = (uint64_t)base;
    u32x4 r;
    r.x = __builtin_amdgcn_readfirstlane((uint32_t)a);
    r.y = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32) & 0xffffu);
    r.z = __builtin_amdgcn_readfirstlane(bytes);
    r.w = 0x00020000u;
    return r;
}

// one wave-load: lane l's 16 bytes at srd + voff + soff land at LDS byte lds + 16 l
__device__ __forceinline__ void load16(u32x4 rsrc, uint32_t voff, uint32_t soff, uint32_t lds) {
    uint32_t saved;  // M0 is reserved to the compiler: save and restore it around the DMA
    asm volatile(
        "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %4\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %3 offen lds\n\t"
        "s_mov_b32 m0, %0"
        : "=&s"(saved)
        : "v"(voff), "s"(rsrc), "s"(soff), "s"(lds)
        : "memory");
}

__device__ __forceinline__ uint32_t lds_addr(const void* p) {
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}

// block id -> id such that consecutive ids run on one XCD (blocks are dealt to the 8 XCDs
// round-robin by hardware id)
__device__ __forceinline__ int xcd_remap(int id, int nblk) {
    const int q = nblk / 8, r = nblk % 8, xcd = id % 8;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + id / 8;
}

}  // namespace dma
}  // namespace yxh
