// ocx_gen.hip — on-device sequence families of sequence_generation.py, one lane per
// sequence, writing straight into the tiled layout the simulation kernels stream.
//
// The g(T) adversary itself (fast_algorithms.py:231-239) is generated one wavefront
// per stream in ocx_gen_wave.hip.  Here: the fp32 random families (IID, Massart; a
// row goes to an LDS slot, is clipped, labelled, and the wave then writes each
// finished step's tiles with coalesced 1 KiB dwordx4 stores) and the deterministic
// ones (label flips, switching leaders).
#include <algorithm>

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

// Row recipes of the staged kernel (template FAM):
//   OCX_FAM_IID     make_random_iid_stream (sequence_generation.py:54-69): fp32 rows,
//                   y = sign(z·u) with u from _rng(run_seed, 0, 11);
//   OCX_FAM_MASSART make_noisy_iid_stream (:72-89): as IID with u from stream 21, then
//                   y flipped where gen.random(T) < p.
// fp32 arithmetic restates NumPy/OpenBLAS on the host CPU: row norms are NumPy's fp32
// pairwise sums; u's norm is cblas_sdot (fp32 products summed in fp64); z @ u is
// cblas_sgemv (four fma lanes, ((l0+l1)+(l2+l3)), fma tail) — verified bit-exact for
// d = 4, 5 (the reference's families use d = 5), an approximation for other d.
enum { OCX_FAM_IID = 1, OCX_FAM_MASSART = 2 };

__device__ __forceinline__ float ocx_f32_pairwise_sq(const double* row, int d) {
    // np.linalg.norm(z32, axis=1)**2: fp32 squares, fp32 pairwise sum (d <= 128)
    if (d < 8) {
        float r = 0.0f;
        for (int j = 0; j < d; ++j) {
            const float v = (float)row[j];
            r += v * v;
        }
        return r;
    }
    float a[8] = {0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f};
    const int n8 = d - (d % 8);
    for (int i0 = 0; i0 < n8; i0 += 8) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const float v = (float)row[i0 + k];
            a[k] += v * v;
        }
    }
    float r = ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
    for (int j = n8; j < d; ++j) {
        const float v = (float)row[j];
        r += v * v;
    }
    return r;
}

__device__ __forceinline__ float ocx_sgemv_dot(const double* row, const float* u, int d) {
    float l[4] = {0.0f, 0.0f, 0.0f, 0.0f};
    const int d4 = d - (d % 4);
    for (int j0 = 0; j0 < d4; j0 += 4) {
#pragma unroll
        for (int k = 0; k < 4; ++k) l[k] = fmaf((float)row[j0 + k], u[j0 + k], l[k]);
    }
    float h = (d4 > 0) ? ((l[0] + l[1]) + (l[2] + l[3])) : 0.0f;
    for (int j = d4; j < d; ++j) h = fmaf((float)row[j], u[j], h);
    return h;
}

// One wavefront (64 threads) = 64 consecutive sequences = P groups of the layout:
// sequence b = _rng(run_seed[b], T, stream_id[b]) with u from _rng(run_seed[b], 0, 11 | 21).
template <int FAM>
__global__ __launch_bounds__(64) void ocx_gen_staged_kernel(
    int64_t T, int64_t B, int d, int P, int C, int64_t G, const uint64_t* __restrict__ run_seeds,
    const uint64_t* __restrict__ stream_ids, double p, double* __restrict__ zt,
    double* __restrict__ ytl) {
    __shared__ Tables tb;
    __shared__ __attribute__((aligned(16))) double rows[64 * OCX_GEN_ROW];
    __shared__ float us[64 * 65];
    load_tables(tb);
    const int lane = threadIdx.x;
    const int S = 64 / P;
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
    float* u = us + lane * 65;
    const uint64_t rs = live ? run_seeds[b] : 0;
    // u: _rng(run_seed, 0, 11 | 21).standard_normal(d) as fp32, / ||u|| (sdot)
    ocx_rng_init3(&rng, rs, 0, FAM == OCX_FAM_IID ? 11 : 21);
    {
        double sq = 0.0;
        for (int j = 0; j < d; ++j) {
            const float v = (float)ocx_standard_normal(&rng, ki, wi, fi);
            u[j] = v;
            sq += (double)(v * v);
        }
        const float n = sqrtf((float)sq);
        if (n > 0.0f)
            for (int j = 0; j < d; ++j) u[j] = u[j] / n;
    }
    ocx_rng_init3(&rng, rs, (uint64_t)T, live ? stream_ids[b] : 0);
    const int64_t kst = G * T * 64;  // plane stride in ocx_d2 (pair k of a step)
    const int64_t g0 = seq0 / S;  // first group of this wave
    const int64_t gb = b / S;
    double* yrow = ytl + gb * T * S + (b - gb * S);

    for (int64_t t = 0; t < T; ++t) {
        if (live) {
            for (int j = 0; j < d; ++j) row[j] = (double)(float)ocx_standard_normal(&rng, ki, wi, fi);
            const float nrm = sqrtf(ocx_f32_pairwise_sq(row, d));
            const float sc = 1.0f / (nrm > 1.0f ? nrm : 1.0f);  // np.maximum, 1.0 / norms
            for (int j = 0; j < d; ++j) row[j] = (double)((float)row[j] * sc);
            const float q = ocx_sgemv_dot(row, u, d);
            yrow[t * S] = (q < 0.0f) ? -1.0 : 1.0;  // np.sign, then y[y == 0] = 1
        } else if (gb < G) {
            yrow[t * S] = 0.0;
        }
        __syncthreads();
        // cooperative store: group gi of this wave, pair k → one 1 KiB dwordx4 store
        for (int gi = 0; gi < P; ++gi) {
            const int64_t g = g0 + gi;
            if (g >= G) break;
            const int sl = gi * S + lane / P;  // wave-local sequence of this lane's slot
            const int c = lane % P;
            const double* src = rows + sl * OCX_GEN_ROW + c * C;
            ocx_d2* dst = reinterpret_cast<ocx_d2*>(zt) + (g * T + t) * 64 + lane;
            for (int k = 0; k < C / 2; ++k)
                __builtin_nontemporal_store(*reinterpret_cast<const ocx_d2*>(src + 2 * k),
                                            dst + k * kst);
        }
        __syncthreads();
    }
    if (FAM == OCX_FAM_MASSART && gb < G && live) {
        // flips = gen.random(T) < p; y[flips] *= -1.0
        for (int64_t t = 0; t < T; ++t)
            if (ocx_pcg_next_double(&rng) < p) yrow[t * S] = -yrow[t * S];
    }
}

// Label flips / switching leaders (sequence_generation.py:24-47): z = e1, y patterned.
__global__ void ocx_gen_fixed_kernel(int family, int64_t block_len, int64_t B, int64_t T,
                                     int P, int C, int64_t G, int64_t zn, int64_t yn,
                                     double* __restrict__ zt, double* __restrict__ ytl) {
    const int S = 64 / P;
    for (int64_t o = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; o < zn;
         o += (int64_t)gridDim.x * blockDim.x) {
        // o = ((k*G + g)*T + t)*128 + 2L + e
        const int64_t row = o >> 7;
        const int L = (int)((o & 127) >> 1), e = (int)(o & 1);
        const int64_t kg = row / T;
        const int64_t k = kg / G, g = kg - k * G;
        const int64_t b = g * S + L / P;
        const int64_t j = (int64_t)(L % P) * C + 2 * k + e;
        zt[o] = (b < B && j == 0) ? 1.0 : 0.0;
    }
    for (int64_t o = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; o < yn;
         o += (int64_t)gridDim.x * blockDim.x) {
        const int64_t tix = o / S;
        const int64_t b = (tix / T) * S + (o - tix * S);
        const int64_t t = tix - (tix / T) * T;
        double yv;
        if (family == 3) yv = (t % 2 == 0) ? 1.0 : -1.0;               // t+1 odd → +1
        else yv = ((t / block_len) % 2 == 0) ? 1.0 : -1.0;              // blocks of +1, -1
        ytl[o] = (b < B) ? yv : 0.0;
    }
}

hipError_t ocx_launch_gen_family(const ocx_layout* L, int family, const uint64_t* run_seeds,
                                 const uint64_t* stream_ids, double p, int64_t block_len,
                                 double* zt, double* ytl, hipStream_t st) {
    const int64_t nlanes = L->G * L->S;
    if (nlanes == 0 || L->T == 0) return hipSuccess;
    if (family == 3 || family == 4) {
        const int64_t n = std::max(L->z_elems, L->y_elems);
        const unsigned grid = (unsigned)std::min<int64_t>((n + 255) / 256, 65536);
        hipLaunchKernelGGL(ocx_gen_fixed_kernel, dim3(grid), dim3(256), 0, st, family, block_len,
                           L->B, L->T, L->P, L->C, L->G, L->z_elems, L->y_elems, zt, ytl);
        return hipGetLastError();
    }
    if ((int64_t)L->P * L->C > 64) return hipErrorNotSupported;
    const unsigned grid = (unsigned)((nlanes + 63) / 64);
    if (family == 1)
        hipLaunchKernelGGL(ocx_gen_staged_kernel<OCX_FAM_IID>, dim3(grid), dim3(64), 0, st, L->T,
                           L->B, (int)L->d, L->P, L->C, L->G, run_seeds, stream_ids, p, zt, ytl);
    else if (family == 2)
        hipLaunchKernelGGL(ocx_gen_staged_kernel<OCX_FAM_MASSART>, dim3(grid), dim3(64), 0, st,
                           L->T, L->B, (int)L->d, L->P, L->C, L->G, run_seeds, stream_ids, p, zt,
                           ytl);
    else
        return hipErrorInvalidValue;
    return hipGetLastError();
}
