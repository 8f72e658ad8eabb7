// hbm_probe.hip — diagnostic read-bandwidth ceilings on this MI355X (not product code).
// Two access shapes over the same buffer the FTRL kernel streams:
//   per-wave contiguous region (what ocx_alg_kernel does, one region per wave)
//   grid-stride (the textbook streaming pattern)
#include <hip/hip_runtime.h>
#include <stdint.h>
typedef double d2 __attribute__((ext_vector_type(2)));

__global__ __launch_bounds__(256) void probe_region(const d2* __restrict__ p, int64_t n2_per_wave,
                                                    int64_t nwaves, double* out, int unroll_dummy) {
    const int lane = threadIdx.x & 63;
    const int64_t w = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (w >= nwaves) return;
    const d2* q = p + w * n2_per_wave + lane;
    d2 acc = {0.0, 0.0};
    for (int64_t i = 0; i < n2_per_wave; i += 64 * 8) {
        d2 v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = __builtin_nontemporal_load(q + i + k * 64);
#pragma unroll
        for (int k = 0; k < 8; ++k) acc += v[k];
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

extern "C" int probe_run(int kind, const void* p, int64_t bytes, int64_t nwaves, double* out,
                         void* stream) {
    hipStream_t st = (hipStream_t)stream;
    const int64_t n2 = bytes / 16;
    if (kind == 0) {
        const int64_t per = (n2 / nwaves) / 512 * 512;
        hipLaunchKernelGGL(probe_region, dim3((unsigned)((nwaves + 3) / 4)), dim3(256), 0, st,
                           (const d2*)p, per, nwaves, out, 0);
    } else {
        hipLaunchKernelGGL(probe_stride, dim3(256 * 8), dim3(256), 0, st, (const d2*)p, n2, out);
    }
    return (int)hipGetLastError();
}
