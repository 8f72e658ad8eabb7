// hbm_probe.hip — diagnostic read-bandwidth ceilings on this MI355X (not product code).
// Each wave streams one contiguous region (the FTRL kernel's access shape) with U
// outstanding 1 KiB dwordx4 loads per wave, or a grid-stride pattern.
#include <hip/hip_runtime.h>
#include <stdint.h>
typedef double d2 __attribute__((ext_vector_type(2)));

template <int U, bool NT>
__global__ __launch_bounds__(256) void probe_region(const d2* __restrict__ p, int64_t n2_per_wave,
                                                    int64_t nwaves, double* out) {
    const int lane = threadIdx.x & 63;
    const int64_t w = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (w >= nwaves) return;
    const d2* q = p + w * n2_per_wave + lane;
    d2 acc = {0.0, 0.0};
    for (int64_t i = 0; i < n2_per_wave; i += 64 * U) {
        d2 v[U];
#pragma unroll
        for (int k = 0; k < U; ++k) v[k] = NT ? __builtin_nontemporal_load(q + i + k * 64) : q[i + k * 64];
#pragma unroll
        for (int k = 0; k < U; ++k) acc += v[k];
    }
    if (acc.x + acc.y == 12345.678) out[w] = acc.x;  // keep loads alive
}

__global__ __launch_bounds__(256) void probe_stride(const d2* __restrict__ p, int64_t n2,
                                                    double* out) {
    const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t nth = (int64_t)gridDim.x * blockDim.x;
    d2 acc = {0.0, 0.0};
    for (int64_t i = tid; i < n2; i += nth * 4) {
        d2 v[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) v[k] = (i + k * nth < n2) ? __builtin_nontemporal_load(p + i + k * nth) : d2{0.0, 0.0};
#pragma unroll
        for (int k = 0; k < 4; ++k) acc += v[k];
    }
    if (acc.x + acc.y == 12345.678) out[tid & 1023] = acc.x;
}

template <int U, bool NT>
static void launch_region(const void* p, int64_t n2, int64_t nwaves, double* out, hipStream_t st) {
    const int64_t per = (n2 / nwaves) / (64 * U) * (64 * U);
    hipLaunchKernelGGL((probe_region<U, NT>), dim3((unsigned)((nwaves + 3) / 4)), dim3(256), 0, st,
                       (const d2*)p, per, nwaves, out);
}

// kind 0: region U=8 nt; 1: stride; 2: region U=16 nt; 3: region U=32 nt; 4: region U=16 plain
extern "C" int probe_run(int kind, const void* p, int64_t bytes, int64_t nwaves, double* out,
                         void* stream) {
    hipStream_t st = (hipStream_t)stream;
    const int64_t n2 = bytes / 16;
    switch (kind) {
        case 0: launch_region<8, true>(p, n2, nwaves, out, st); break;
        case 1: hipLaunchKernelGGL(probe_stride, dim3(256 * 8), dim3(256), 0, st, (const d2*)p, n2, out); break;
        case 2: launch_region<16, true>(p, n2, nwaves, out, st); break;
        case 3: launch_region<32, true>(p, n2, nwaves, out, st); break;
        case 4: launch_region<16, false>(p, n2, nwaves, out, st); break;
    }
    return (int)hipGetLastError();
}
