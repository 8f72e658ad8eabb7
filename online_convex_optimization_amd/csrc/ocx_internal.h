// ocx_internal.h — shared device helpers for the gfx950 kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cstdlib>

#include "../../include/ocx.h"

#define OCX_WAVE 64
#define OCX_BLOCK 256  // 4 wave-groups per workgroup
#define OCX_WAVES_PER_BLOCK (OCX_BLOCK / OCX_WAVE)

// Wave-group index of the calling wave: blocks hold blockDim.x / 64 waves (see
// ocx_block_waves; kernels are compiled for OCX_BLOCK threads and launched with 64,
// 128 or 256).
__device__ __forceinline__ int64_t ocx_wave_id() {
    return (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
}

// Waves per workgroup for a launch of G independent wave-groups.  Four-wave blocks pack a
// CU's four SIMDs, but a launch of few waves (capacity-limited long horizons, d = 1024)
// then lands on G/4 CUs and leaves the rest idle: below 8 waves per CU use one-wave
// blocks, which the dispatcher spreads over every CU.  OCX_BLOCK_WAVES=1|2|4 forces it.
inline int ocx_block_waves(int64_t G) {
    // read once, thread-safe (host threads of ocx_gT_sweep_devices launch concurrently):
    // a function-local static's initialiser runs exactly once (C++11 magic statics)
    static const int forced = [] {
        const char* e = std::getenv("OCX_BLOCK_WAVES");
        const int v = e ? std::atoi(e) : 0;
        return (v == 1 || v == 2 || v == 4) ? v : 0;
    }();
    if (forced) return forced;
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        cus = 256;
    return G >= 8 * (int64_t)cus ? OCX_WAVES_PER_BLOCK : 1;
}
inline dim3 ocx_grid(int64_t G, int wpb) { return dim3((unsigned)((G + wpb - 1) / wpb)); }

// ---------------------------------------------------------------------------
// Cross-lane fp64 reductions over the P lanes that own one sequence.
// All steps are symmetric butterflies (lane i: a+b, its partner: b+a), so every
// lane of a sequence ends with the bit-identical total and takes the same
// branch (norm > 1, sign of q - y) — the per-sequence control flow stays uniform.
// ---------------------------------------------------------------------------
template <int CTRL>
__device__ __forceinline__ double ocx_dpp(double v) {
    int lo = __double2loint(v), hi = __double2hiint(v);
    // old = the value itself: a lane without a source (lane 0 under wave_shr) keeps its
    // own value, which no caller reads, and the move needs no zeroed destination first
    lo = __builtin_amdgcn_update_dpp(lo, lo, CTRL, 0xF, 0xF, false);
    hi = __builtin_amdgcn_update_dpp(hi, hi, CTRL, 0xF, 0xF, false);
    return __hiloint2double(hi, lo);
}

// DPP move for the full-source patterns (quad_perm, row_half_mirror, row_mirror: every lane
// has a source lane): bound_ctrl, so no copy of the old value is made first (two v_mov
// fewer per 64-bit move than ocx_dpp); the data moved are the same.
template <int CTRL>
__device__ __forceinline__ double ocx_dpp_all(double v) {
    int lo = __double2loint(v), hi = __double2hiint(v);
    lo = __builtin_amdgcn_mov_dpp(lo, CTRL, 0xF, 0xF, true);
    hi = __builtin_amdgcn_mov_dpp(hi, CTRL, 0xF, 0xF, true);
    return __hiloint2double(hi, lo);
}

__device__ __forceinline__ double ocx_readlane(double v, int src) {
    const int lo = __builtin_amdgcn_readlane(__double2loint(v), src);
    const int hi = __builtin_amdgcn_readlane(__double2hiint(v), src);
    return __hiloint2double(hi, lo);
}

__device__ __forceinline__ double ocx_swz_xor16(double v) {
    // ds_swizzle bit-mode: and 0x1F, or 0, xor 0x10 (within 32-lane halves)
    int lo = __double2loint(v), hi = __double2hiint(v);
    lo = __builtin_amdgcn_ds_swizzle(lo, 0x401F);
    hi = __builtin_amdgcn_ds_swizzle(hi, 0x401F);
    return __hiloint2double(hi, lo);
}

__device__ __forceinline__ double ocx_xor32(double v) {
    int addr = ((int)(threadIdx.x & 63) ^ 32) << 2;
    int lo = __double2loint(v), hi = __double2hiint(v);
    lo = __builtin_amdgcn_ds_bpermute(addr, lo);
    hi = __builtin_amdgcn_ds_bpermute(addr, hi);
    return __hiloint2double(hi, lo);
}

template <int P>
__device__ __forceinline__ double ocx_seq_sum(double v) {
    if constexpr (P >= 2) v = v + ocx_dpp_all<0xB1>(v);   // quad_perm [1,0,3,2]  (xor 1)
    if constexpr (P >= 4) v = v + ocx_dpp_all<0x4E>(v);   // quad_perm [2,3,0,1]  (xor 2)
    if constexpr (P >= 8) v = v + ocx_dpp_all<0x141>(v);  // row_half_mirror (quads are uniform)
    if constexpr (P >= 16) v = v + ocx_dpp_all<0x140>(v); // row_mirror (half-rows are uniform)
    if constexpr (P >= 32) v = v + ocx_swz_xor16(v);
    if constexpr (P >= 64) v = v + ocx_xor32(v);
    return v;
}

// Index of element (g, t, j-chunk pair k, lane L, e) in the tiled z layout.
__host__ __device__ __forceinline__ int64_t ocx_ztile_base(int64_t g, int64_t T, int64_t t,
                                                          int C) {
    return (g * T + t) * (int64_t)(64 * C);
}

// Native 2 x f64 vector (one dwordx4 per lane); HIP's double2 is a struct, which
// __builtin_nontemporal_load does not accept.
typedef double ocx_d2 __attribute__((ext_vector_type(2)));
