// ocx_gen.hip — on-device g(T) adversary (fast_algorithms.py:231-239), one lane per
// sequence, writing straight into the tiled layout the simulation kernels stream.
//
// Sequence b of the batch is the stream _rng(base_seed, T, run0 + b): SeedSequence
// mixing, PCG64 XSL-RR and NumPy's ziggurat run in-lane (ocx_rng.h), so the z/y the
// GPU simulates are the reference's own sequences, never copied from the host.
// Row clipping needs ‖z_t‖ before any coordinate is scaled: the lane saves the PCG
// state at the row start, streams the d squares through NumPy's pairwise-sum order,
// then rewinds and regenerates the row to scale and store it (regeneration costs
// ALU, not HBM bytes).
#include "ocx_internal.h"
#include "ocx_rng.h"
#include "ocx_sim_kernels.h"

struct ocx_lds_tables {
    const uint64_t* ki;
    const double* wi;
    const double* fi;
};

__global__ __launch_bounds__(OCX_BLOCK) void ocx_gen_gT_kernel(
    uint64_t base_seed, int64_t T, int64_t run0, int64_t B, int64_t d, int P, int C,
    int64_t nlanes, double* __restrict__ zt, double* __restrict__ ytl) {
    __shared__ uint64_t s_ki[256];
    __shared__ double s_wi[256];
    __shared__ double s_fi[256];
    for (int i = threadIdx.x; i < 256; i += blockDim.x) {
        s_ki[i] = OCX_ZIG_KI[i];
        s_wi[i] = __longlong_as_double((long long)OCX_ZIG_WI_BITS[i]);
        s_fi[i] = __longlong_as_double((long long)OCX_ZIG_FI_BITS[i]);
    }
    __syncthreads();
    auto ki = [&](int i) { return s_ki[i]; };
    auto wi = [&](int i) { return s_wi[i]; };
    auto fi = [&](int i) { return s_fi[i]; };

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

    for (int64_t t = 0; t < T; ++t) {
        const ocx_pcg64 row_start = rng;
        // pass 1: ‖z_t‖² in NumPy's pairwise order (np.linalg.norm(axis=1))
        double stack[16];
        int sp = 0;
        int64_t j = 0;
        for (int op = 0; op < plan.nops; ++op) {
            const int code = plan.ops[op];
            if (code >= 0) {
                ocx_pw_leaf leaf;
                ocx_pw_leaf_begin(&leaf, plan.leaf_len[code]);
                for (int i = 0; i < plan.leaf_len[code]; ++i, ++j) {
                    const double v = ocx_standard_normal(&rng, ki, wi, fi);
                    ocx_pw_leaf_add(&leaf, v * v);
                }
                stack[sp++] = leaf.res;
            } else {
                const double rgt = stack[--sp];
                const double lft = stack[--sp];
                stack[sp++] = lft + rgt;
            }
        }
        const double sumsq = (d > 0) ? stack[0] : 0.0;
        const double nrm = sqrt(sumsq);
        const double scale = 1.0 / (nrm > 1.0 ? nrm : 1.0);  // 1.0 / np.maximum(norms, 1.0)
        // pass 2: rewind, regenerate, scale, store
        rng = row_start;
        for (int64_t jj = 0; jj < d; ++jj) {
            const double v = ocx_standard_normal(&rng, ki, wi, fi);
            zt[zidx(t, jj)] = v * scale;
        }
        for (int64_t jj = d; jj < Dp; ++jj) zt[zidx(t, jj)] = 0.0;
    }
    // labels: choice([-1.0, 1.0], size=T) → integers(0, 2) → top bit of next_uint32
    for (int64_t t = 0; t < T; ++t) {
        const uint32_t u = ocx_pcg_next32(&rng);
        yrow[t * S] = (u >> 31) ? 1.0 : -1.0;
    }
}

hipError_t ocx_launch_gen_gT(const ocx_layout* L, uint64_t base_seed, int64_t run0, double* zt,
                             double* ytl, hipStream_t st) {
    const int64_t nlanes = L->G * L->S;
    if (nlanes == 0 || L->T == 0) return hipSuccess;
    const unsigned grid = (unsigned)((nlanes + OCX_BLOCK - 1) / OCX_BLOCK);
    hipLaunchKernelGGL(ocx_gen_gT_kernel, dim3(grid), dim3(OCX_BLOCK), 0, st, base_seed, L->T,
                       run0, L->B, L->d, L->P, L->C, nlanes, zt, ytl);
    return hipGetLastError();
}
