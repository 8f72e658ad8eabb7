// wprobe.hip — WRITE_SIZE calibration for the generator's 8-B-per-lane store shapes
// (diagnostic, not product code).  Each launch writes a known number of bytes:
//   mode 0: each wave writes its own contiguous region, 8 B per lane (512 B per store);
//   mode 1: the g(T) generator's z-tile map at d = 64, P = 4 (one wave per sequence, lane j
//           writes coordinate j of each row: 8 planes x one 64-B segment per store);
//   mode 2: mode 1's map with 16-B-per-lane stores (32 lanes, two coordinates each);
//   mode 3: mode 1 with plain (write-back) stores instead of nontemporal ones.
// Run under rocprofv3 --pmc WRITE_SIZE; the byte count is printed per launch.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

__global__ __launch_bounds__(256) void w_contig(double* p, int64_t n_per_wave, int64_t nw) {
    const int lane = threadIdx.x & 63;
    const int64_t w = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (w >= nw) return;
    double* q = p + w * n_per_wave + lane;
    for (int64_t i = 0; i < n_per_wave; i += 64) __builtin_nontemporal_store((double)i, q + i);
}

// z tile of the (P = 4, C = 16) layout: element (plane k, group g, step t, slot 2(sP+c)+e)
__global__ __launch_bounds__(256) void w_tile(double* zt, int64_t G, int64_t T, int64_t nseq,
                                              int64_t nw, int wide) {
    const int lane = threadIdx.x & 63;
    const int64_t w = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (w >= nw) return;
    for (int64_t b = w; b < nseq; b += nw) {
        const int64_t g = b / 16;
        const int s = (int)(b % 16);
        if (wide != 1) {
            const int j = lane, c = j / 16, kl = (j % 16) >> 1, el = j & 1;
            double* zp = zt + ((int64_t)kl * G + g) * T * 128 + (s * 4 + c) * 2 + el;
            if (wide == 2) {
                for (int64_t t = 0; t < T; ++t) zp[t * 128] = (double)t;
            } else {
                for (int64_t t = 0; t < T; ++t) __builtin_nontemporal_store((double)t, zp + t * 128);
            }
        } else if (lane < 32) {  // wide == 1
            typedef double d2 __attribute__((ext_vector_type(2)));
            const int c = lane / 8, kl = lane % 8;
            d2* zp = (d2*)(zt + ((int64_t)kl * G + g) * T * 128 + (s * 4 + c) * 2);
            for (int64_t t = 0; t < T; ++t) {
                d2 v = {(double)t, (double)t};
                __builtin_nontemporal_store(v, zp + t * 64);
            }
        }
    }
}

int main(int argc, char** argv) {
    const int mode = argc > 1 ? atoi(argv[1]) : 0;
    const int64_t G = 2048, T = argc > 2 ? atoll(argv[2]) : 1000, nseq = G * 16;
    const int64_t n = 8 * G * T * 128;  // doubles
    double* p = nullptr;
    if (hipMalloc(&p, n * 8) != hipSuccess) return 2;
    const int64_t nw = 4096;
    for (int rep = 0; rep < 2; ++rep) {
        if (mode == 0)
            hipLaunchKernelGGL(w_contig, dim3(nw / 4), dim3(256), 0, 0, p, n / nw, nw);
        else
            hipLaunchKernelGGL(w_tile, dim3(nw / 4), dim3(256), 0, 0, p, G, T, nseq, nw, mode == 2 ? 1 : (mode == 3 ? 2 : 0));
        if (hipDeviceSynchronize() != hipSuccess) return 3;
    }
    printf("mode %d: %lld bytes per launch\n", mode, (long long)(n * 8));
    hipFree(p);
    return 0;
}
