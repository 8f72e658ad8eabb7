// gen_probe.hip — where does the on-device g(T) generator spend its time?
//
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off tools/gen_probe.hip \
//         -I online_convex_optimization_amd/csrc -o build/gen_probe && build/gen_probe
//
// Each variant runs `lanes` independent NumPy streams (one per lane) and draws N values
// per lane; it prints one JSON line with the draws per second.  Diagnostic only: not
// part of the product path.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#include "ocx_rng.h"

#define CHECK(x)                                                                     \
    do {                                                                             \
        hipError_t e_ = (x);                                                         \
        if (e_ != hipSuccess) {                                                      \
            fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, \
                    __LINE__);                                                       \
            exit(1);                                                                 \
        }                                                                            \
    } while (0)

struct Tables {
    uint64_t ki[256];
    double wi[256];
    double fi[256];
};

__device__ __forceinline__ void load_tables(Tables& tb) {
    for (int i = threadIdx.x; i < 256; i += blockDim.x) {
        tb.ki[i] = OCX_ZIG_KI[i];
        tb.wi[i] = __longlong_as_double((long long)OCX_ZIG_WI_BITS[i]);
        tb.fi[i] = __longlong_as_double((long long)OCX_ZIG_FI_BITS[i]);
    }
}

// 0: raw PCG64 next64
template <int PAD>
__global__ __launch_bounds__(64) void k_pcg(int64_t n, double* outd) {
    uint64_t* out = reinterpret_cast<uint64_t*>(outd);
    __shared__ double pad[PAD];
    ocx_pcg64 g;
    ocx_rng_init3(&g, 0, 10000, blockIdx.x * 64 + threadIdx.x);
    uint64_t acc = 0;
    for (int64_t i = 0; i < n; ++i) acc ^= ocx_pcg_next64(&g);
    if (PAD > 1) pad[threadIdx.x] = (double)acc;
    if (acc == 0x1234567) out[0] = acc + (PAD > 1 ? (uint64_t)pad[(threadIdx.x + 1) % 64] : 0);
    else out[blockIdx.x * 64 + threadIdx.x] = acc;
}

// 1: full NumPy standard_normal (ziggurat, LDS tables); PAD doubles of extra LDS
// emulate the staged kernel's occupancy.
template <int PAD>
__global__ __launch_bounds__(64) void k_normal(int64_t n, double* out) {
    __shared__ Tables tb;
    __shared__ double pad[PAD];
    load_tables(tb);
    __syncthreads();
    auto ki = [&](int i) { return tb.ki[i]; };
    auto wi = [&](int i) { return tb.wi[i]; };
    auto fi = [&](int i) { return tb.fi[i]; };
    ocx_pcg64 g;
    ocx_rng_init3(&g, 0, 10000, blockIdx.x * 64 + threadIdx.x);
    double acc = 0.0;
    for (int64_t i = 0; i < n; ++i) acc += ocx_standard_normal(&g, ki, wi, fi);
    if (PAD > 1) pad[threadIdx.x] = acc;
    out[blockIdx.x * 64 + threadIdx.x] = acc + (PAD > 1 ? pad[(threadIdx.x + 1) % 64] : 0.0);
}

// 2: fast path only (every draw accepted: wrong values, measures the common path)
template <int PAD>
__global__ __launch_bounds__(64) void k_fast(int64_t n, double* out) {
    __shared__ Tables tb;
    __shared__ double pad[PAD];
    load_tables(tb);
    __syncthreads();
    ocx_pcg64 g;
    ocx_rng_init3(&g, 0, 10000, blockIdx.x * 64 + threadIdx.x);
    double acc = 0.0;
    for (int64_t i = 0; i < n; ++i) {
        uint64_t r = ocx_pcg_next64(&g);
        int idx = (int)(r & 0xff);
        r >>= 8;
        uint64_t rabs = (r >> 1) & 0x000fffffffffffffULL;
        double x = (double)rabs * tb.wi[idx];
        if (r & 1) x = -x;
        acc += (rabs < tb.ki[idx]) ? x : 0.0;
    }
    if (PAD > 1) pad[threadIdx.x] = acc;
    out[blockIdx.x * 64 + threadIdx.x] = acc + (PAD > 1 ? pad[(threadIdx.x + 1) % 64] : 0.0);
}

// 3: two independent streams per lane, interleaved
template <int PAD>
__global__ __launch_bounds__(64) void k_normal2(int64_t n, double* out) {
    __shared__ Tables tb;
    __shared__ double pad[PAD];
    load_tables(tb);
    __syncthreads();
    auto ki = [&](int i) { return tb.ki[i]; };
    auto wi = [&](int i) { return tb.wi[i]; };
    auto fi = [&](int i) { return tb.fi[i]; };
    ocx_pcg64 g0, g1;
    ocx_rng_init3(&g0, 0, 10000, 2 * (blockIdx.x * 64 + threadIdx.x));
    ocx_rng_init3(&g1, 0, 10000, 2 * (blockIdx.x * 64 + threadIdx.x) + 1);
    double a0 = 0.0, a1 = 0.0;
    for (int64_t i = 0; i < n; i += 2) {
        a0 += ocx_standard_normal(&g0, ki, wi, fi);
        a1 += ocx_standard_normal(&g1, ki, wi, fi);
    }
    if (PAD > 1) pad[threadIdx.x] = a0;
    out[blockIdx.x * 64 + threadIdx.x] = a0 + a1 + (PAD > 1 ? pad[(threadIdx.x + 1) % 64] : 0.0);
}

// 4: one step of a uniform per-draw state machine (every lane consumes exactly one raw
// draw per iteration; a lane emits a normal when its draw completes one).
template <int PAD>
__global__ __launch_bounds__(64) void k_machine(int64_t n, double* out) {
    __shared__ Tables tb;
    __shared__ double pad[PAD];
    load_tables(tb);
    __syncthreads();
    ocx_pcg64 g;
    ocx_rng_init3(&g, 0, 10000, blockIdx.x * 64 + threadIdx.x);
    double acc = 0.0;
    int64_t emitted = 0;
    // state: 0 new draw; 1 wedge uniform for (idx, x); 2 tail xx; 3 tail yy
    int state = 0, idx = 0, sign = 0;
    double x = 0.0, xx = 0.0;
    while (true) {
        // uniform exit: all lanes have emitted n
        if (emitted >= n) break;
        const uint64_t r = ocx_pcg_next64(&g);
        if (state == 0) {
            idx = (int)(r & 0xff);
            const uint64_t r8 = r >> 8;
            sign = (int)(r8 & 1);
            const uint64_t rabs = (r8 >> 1) & 0x000fffffffffffffULL;
            x = (double)rabs * tb.wi[idx];
            if (sign) x = -x;
            if (rabs < tb.ki[idx]) {
                acc += x;
                ++emitted;
            } else {
                state = (idx == 0) ? 2 : 1;
            }
        } else if (state == 1) {
            const double u = (double)(r >> 11) * (1.0 / 9007199254740992.0);
            if (((tb.fi[idx - 1] - tb.fi[idx]) * u + tb.fi[idx]) < exp(-0.5 * x * x)) {
                acc += x;
                ++emitted;
            }
            state = 0;
        } else if (state == 2) {
            const double u = (double)(r >> 11) * (1.0 / 9007199254740992.0);
            xx = -OCX_ZIG_NOR_INV_R * ocx_log1p(-u);
            state = 3;
        } else {
            const double u = (double)(r >> 11) * (1.0 / 9007199254740992.0);
            const double yy = -ocx_log1p(-u);
            if (yy + yy > xx * xx) {
                acc += sign ? -(OCX_ZIG_NOR_R + xx) : OCX_ZIG_NOR_R + xx;
                ++emitted;
                state = 0;
            } else {
                state = 2;
            }
        }
    }
    if (PAD > 1) pad[threadIdx.x] = acc;
    out[blockIdx.x * 64 + threadIdx.x] = acc + (PAD > 1 ? pad[(threadIdx.x + 1) % 64] : 0.0);
}

template <class F>
static double time_ms(F f, int reps) {
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    f();
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(a));
    for (int i = 0; i < reps; ++i) f();
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, a, b));
    return ms / reps;
}

int main(int argc, char** argv) {
    const int64_t lanes = argc > 1 ? atoll(argv[1]) : 262144;
    const int64_t n = argc > 2 ? atoll(argv[2]) : 2048;
    double* out;
    CHECK(hipMalloc(&out, lanes * 2 * sizeof(double)));
    const dim3 grid((unsigned)(lanes / 64)), blk(64);
    auto report = [&](const char* name, int pad, double ms, double per_lane) {
        printf("{\"what\": \"gen_probe\", \"variant\": \"%s\", \"pad_doubles\": %d, \"lanes\": %lld, "
               "\"n\": %lld, \"ms\": %.4f, \"draws_per_s\": %.4e}\n",
               name, pad, (long long)lanes, (long long)n, ms, lanes * per_lane / (ms * 1e-3));
        fflush(stdout);
    };
#define RUN(KER, NAME, PAD, PER)                                                            \
    {                                                                                      \
        double ms = time_ms([&] { hipLaunchKernelGGL((KER<PAD>), grid, blk, 0, 0, n, out); }, 3); \
        CHECK(hipGetLastError());                                                          \
        report(NAME, PAD, ms, PER);                                                        \
    }
    // PAD 1 → occupancy set by registers; PAD 4224 → 64 rows × 66 doubles, as the staged kernel
    RUN(k_pcg, "pcg_next64", 1, (double)n)
    RUN(k_pcg, "pcg_next64", 4224, (double)n)
    RUN(k_fast, "ziggurat_fast_path", 1, (double)n)
    RUN(k_fast, "ziggurat_fast_path", 4224, (double)n)
    RUN(k_normal, "standard_normal", 1, (double)n)
    RUN(k_normal, "standard_normal", 4224, (double)n)
    RUN(k_normal2, "standard_normal_2streams", 1, (double)n)
    RUN(k_normal2, "standard_normal_2streams", 4224, (double)n)
    RUN(k_machine, "standard_normal_machine", 1, (double)n)
    RUN(k_machine, "standard_normal_machine", 4224, (double)n)
    CHECK(hipFree(out));
    return 0;
}
