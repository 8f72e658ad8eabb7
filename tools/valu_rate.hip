// Issue cost of the generator's integer multiply instructions on gfx950.
// Each wave runs ITER iterations of 8 independent chains of one instruction; the grid fills
// every SIMD with W waves.  Prints ns per launch and SIMD cycles per wave-instruction.
//   hipcc --offload-arch=gfx950 -O2 -o tools/valu_rate tools/valu_rate.hip && tools/valu_rate
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

constexpr int ITER = 4096;

template <int OP>
__global__ __launch_bounds__(256) void rate_kernel(uint64_t* out, uint32_t sb) {
    uint64_t c[8];
    uint32_t a[8];
    double f[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        c[i] = threadIdx.x + i;
        a[i] = threadIdx.x * 7 + i;
        f[i] = (double)(threadIdx.x + i);
    }
    for (int it = 0; it < ITER; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            if constexpr (OP == 0) {  // v_mad_u64_u32 (VGPR, SGPR, VGPR pair)
                uint64_t cy;
                asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(c[i]), "=s"(cy) : "v"(a[i]), "s"(sb));
            } else if constexpr (OP == 1) {  // v_mul_lo_u32
                asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a[i]) : "s"(sb));
            } else if constexpr (OP == 2) {  // v_add_co_u32 (full-rate reference)
                uint64_t cy;
                asm volatile("v_add_co_u32_e64 %0, %1, %0, %2" : "+v"(a[i]), "=s"(cy) : "v"(a[(i + 1) & 7]));
            } else if constexpr (OP == 3) {  // v_fma_f64
                asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(f[i]) : "v"(f[(i + 1) & 7]), "v"(f[(i + 2) & 7]));
            } else if constexpr (OP == 4) {  // v_mul_hi_u32
                asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(a[i]) : "s"(sb));
            } else if constexpr (OP == 5) {  // v_alignbit_b32
                asm volatile("v_alignbit_b32 %0, %0, %1, 7" : "+v"(a[i]) : "v"(a[(i + 3) & 7]));
            } else if constexpr (OP == 6) {  // v_lshrrev_b64
                asm volatile("v_lshrrev_b64 %0, 9, %0" : "+v"(c[i]));
            } else if constexpr (OP == 7) {  // v_cvt_f64_u32
                asm volatile("v_cvt_f64_u32 %0, %1" : "=v"(f[i]) : "v"(a[i]));
                asm volatile("v_add_u32 %0, %0, 1" : "+v"(a[i]));
            }
        }
    }
    uint64_t s = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) s += c[i] + a[i] + (uint64_t)f[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int OP>
void run(const char* name, int ninst_per_iter, int waves_per_simd, int ncu) {
    const int blocks = ncu * waves_per_simd;  // 256 threads = 4 waves = one per SIMD
    uint64_t* out;
    hipMalloc(&out, (size_t)blocks * 256 * 8);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    rate_kernel<OP><<<blocks, 256>>>(out, 0x9E3779B9u);
    hipDeviceSynchronize();
    hipEventRecord(e0);
    for (int r = 0; r < 5; ++r) rate_kernel<OP><<<blocks, 256>>>(out, 0x9E3779B9u);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    ms /= 5;
    // per SIMD: waves_per_simd waves x ITER x 8 x ninst instructions
    const double inst = (double)waves_per_simd * ITER * 8 * ninst_per_iter;
    const double cyc = ms * 1e-3 * 2.4e9;  // nominal clock
    printf("{\"op\": \"%s\", \"waves_per_simd\": %d, \"ms\": %.4f, \"cycles_per_wave_inst\": %.3f}\n", name,
           waves_per_simd, ms, cyc / inst);
    hipFree(out);
}

int main() {
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, 0);
    const int ncu = p.multiProcessorCount;
    for (int w : {1, 4, 8}) {
        run<0>("v_mad_u64_u32", 1, w, ncu);
        run<1>("v_mul_lo_u32", 1, w, ncu);
        run<4>("v_mul_hi_u32", 1, w, ncu);
        run<2>("v_add_co_u32", 1, w, ncu);
        run<3>("v_fma_f64", 1, w, ncu);
        run<5>("v_alignbit_b32", 1, w, ncu);
        run<6>("v_lshrrev_b64", 1, w, ncu);
        run<7>("v_cvt_f64_u32+v_add_u32", 2, w, ncu);
    }
    return 0;
}
