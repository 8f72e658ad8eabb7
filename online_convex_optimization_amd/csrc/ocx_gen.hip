// ocx_gen.hip — on-device g(T) adversary (fast_algorithms.py:231-239), one lane per
// sequence, writing straight into the tiled layout the simulation kernels stream.
//
// Sequence b of the batch is the stream _rng(base_seed, T, run0 + b): SeedSequence
// mixing, PCG64 XSL-RR and NumPy's ziggurat run in-lane (ocx_rng.h), so the z/y the
// GPU simulates are the reference's own sequences, never copied from the host.
// Row clipping needs ‖z_t‖ before any coordinate is scaled:
//   staged kernel (padded row <= 64): the row goes to an LDS slot while its squares
//     stream through NumPy's pairwise order; the wave then writes each finished
//     step's tiles with coalesced 1 KiB dwordx4 stores;
//   regen kernel (wider rows): the lane saves the PCG state at the row start, sums
//     the squares, rewinds and regenerates the row to scale and store it.
#include "ocx_internal.h"
#include "ocx_rng.h"
#include "ocx_sim_kernels.h"

#define OCX_GEN_ROW 66  // LDS doubles per staged row (64 + pad keeps b128 reads aligned)

namespace {

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

}  // namespace

// One wavefront (64 threads) = 64 consecutive sequences = P groups of the layout.
__global__ __launch_bounds__(64) void ocx_gen_staged_kernel(
    uint64_t base_seed, int64_t T, int64_t run0, int64_t B, int d, int P, int C, int64_t G,
    double* __restrict__ zt, double* __restrict__ ytl) {
    __shared__ Tables tb;
    __shared__ __attribute__((aligned(16))) double rows[64 * OCX_GEN_ROW];
    __shared__ double scale[64];
    load_tables(tb);
    const int lane = threadIdx.x;
    const int S = 64 / P;
    const int Dp = P * C;
    const int64_t seq0 = (int64_t)blockIdx.x * 64;  // first sequence of this wave
    const int64_t b = seq0 + lane;
    double* row = rows + lane * OCX_GEN_ROW;
    for (int j = 0; j < OCX_GEN_ROW; ++j) row[j] = 0.0;  // padding coordinates stay 0
    __syncthreads();
    auto ki = [&](int i) { return tb.ki[i]; };
    auto wi = [&](int i) { return tb.wi[i]; };
    auto fi = [&](int i) { return tb.fi[i]; };

    const bool live = b < B;
    ocx_pcg64 rng;
    ocx_rng_init3(&rng, base_seed, (uint64_t)T, (uint64_t)(run0 + (live ? b : 0)));
    ocx_pw_plan plan;
    ocx_pw_build(&plan, d);
    const int64_t tile = 64 * (int64_t)C;
    const int64_t g0 = seq0 / S;  // first group of this wave

    for (int64_t t = 0; t < T; ++t) {
        if (live) {
            const double sumsq = ocx_row_sumsq(
                d, plan, [&]() { return ocx_standard_normal(&rng, ki, wi, fi); },
                [&](int j, double v) { row[j] = v; });
            const double nrm = sqrt(sumsq);
            scale[lane] = 1.0 / (nrm > 1.0 ? nrm : 1.0);  // 1.0 / np.maximum(norms, 1.0)
        } else {
            scale[lane] = 0.0;
        }
        __syncthreads();
        // cooperative store: group gi of this wave, pair k → one 1 KiB dwordx4 store
        for (int gi = 0; gi < P; ++gi) {
            const int64_t g = g0 + gi;
            if (g >= G) break;
            const int sl = gi * S + lane / P;  // wave-local sequence of this lane's slot
            const int c = lane % P;
            const double sc = scale[sl];
            const double* src = rows + sl * OCX_GEN_ROW + c * C;
            ocx_d2* dst = reinterpret_cast<ocx_d2*>(zt + (g * T + t) * tile) + lane;
            for (int k = 0; k < C / 2; ++k) {
                ocx_d2 v = *reinterpret_cast<const ocx_d2*>(src + 2 * k);
                v.x *= sc;
                v.y *= sc;
                __builtin_nontemporal_store(v, dst + k * 64);
            }
        }
        __syncthreads();
    }
    // labels: choice([-1.0, 1.0], size=T) → integers(0, 2) → top bit of next_uint32
    const int64_t g = b / S;
    if (g < G) {
        double* yrow = ytl + g * T * S + (b - g * S);
        for (int64_t t = 0; t < T; ++t) {
            double yv = 0.0;
            if (live) yv = (ocx_pcg_next32(&rng) >> 31) ? 1.0 : -1.0;
            yrow[t * S] = yv;
        }
    }
    (void)Dp;
}

// General rows (padded width > 64): one lane per sequence, regenerate-to-scale.
__global__ __launch_bounds__(OCX_BLOCK) void ocx_gen_regen_kernel(
    uint64_t base_seed, int64_t T, int64_t run0, int64_t B, int64_t d, int P, int C,
    int64_t nlanes, double* __restrict__ zt, double* __restrict__ ytl) {
    __shared__ Tables tb;
    load_tables(tb);
    __syncthreads();
    auto ki = [&](int i) { return tb.ki[i]; };
    auto wi = [&](int i) { return tb.wi[i]; };
    auto fi = [&](int i) { return tb.fi[i]; };

    const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= nlanes) return;
    const int S = 64 / P;
    const int64_t g = b / S;
    const int s = (int)(b - g * S);
    const int64_t tile = 64 * (int64_t)C;
    const int64_t Dp = (int64_t)P * C;
    auto zidx = [&](int64_t t, int64_t j) -> int64_t {
        const int c = (int)(j / C);
        const int r = (int)(j - (int64_t)c * C);
        const int L = s * P + c;
        return (g * T + t) * tile + (r >> 1) * 128 + L * 2 + (r & 1);
    };
    double* yrow = ytl + g * T * S + s;

    if (b >= B) {  // padding sequence: zeros
        for (int64_t t = 0; t < T; ++t) {
            for (int64_t j = 0; j < Dp; ++j) zt[zidx(t, j)] = 0.0;
            yrow[t * S] = 0.0;
        }
        return;
    }

    ocx_pcg64 rng;
    ocx_rng_init3(&rng, base_seed, (uint64_t)T, (uint64_t)(run0 + b));
    ocx_pw_plan plan;
    ocx_pw_build(&plan, (int)d);
    auto normal = [&]() { return ocx_standard_normal(&rng, ki, wi, fi); };

    for (int64_t t = 0; t < T; ++t) {
        const ocx_pcg64 row_start = rng;
        const double sumsq = ocx_row_sumsq((int)d, plan, normal, [](int, double) {});
        const double nrm = sqrt(sumsq);
        const double scale = 1.0 / (nrm > 1.0 ? nrm : 1.0);  // 1.0 / np.maximum(norms, 1.0)
        rng = row_start;
        for (int64_t jj = 0; jj < d; ++jj) zt[zidx(t, jj)] = normal() * scale;
        for (int64_t jj = d; jj < Dp; ++jj) zt[zidx(t, jj)] = 0.0;
    }
    for (int64_t t = 0; t < T; ++t) yrow[t * S] = (ocx_pcg_next32(&rng) >> 31) ? 1.0 : -1.0;
}

hipError_t ocx_launch_gen_gT(const ocx_layout* L, uint64_t base_seed, int64_t run0, double* zt,
                             double* ytl, hipStream_t st) {
    const int64_t nlanes = L->G * L->S;
    if (nlanes == 0 || L->T == 0) return hipSuccess;
    if ((int64_t)L->P * L->C <= 64) {
        const unsigned grid = (unsigned)((nlanes + 63) / 64);
        hipLaunchKernelGGL(ocx_gen_staged_kernel, dim3(grid), dim3(64), 0, st, base_seed, L->T,
                           run0, L->B, (int)L->d, L->P, L->C, L->G, zt, ytl);
    } else {
        const unsigned grid = (unsigned)((nlanes + OCX_BLOCK - 1) / OCX_BLOCK);
        hipLaunchKernelGGL(ocx_gen_regen_kernel, dim3(grid), dim3(OCX_BLOCK), 0, st, base_seed,
                           L->T, run0, L->B, L->d, L->P, L->C, nlanes, zt, ytl);
    }
    return hipGetLastError();
}
