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

// Saved PCG64 stream state in HBM: 6 x u64 per sequence
// [state lo, state hi, inc lo, inc hi, buf32 | has32 << 32, 0].
__device__ __forceinline__ void load_state(ocx_pcg64* g, const uint64_t* p) {
    g->state = ((ocx_u128)p[1] << 64) | p[0];
    g->inc = ((ocx_u128)p[3] << 64) | p[2];
    g->buf32 = (uint32_t)p[4];
    g->has32 = (int)(p[4] >> 32);
}

__device__ __forceinline__ void save_state(const ocx_pcg64* g, uint64_t* p) {
    p[0] = (uint64_t)g->state;
    p[1] = (uint64_t)(g->state >> 64);
    p[2] = (uint64_t)g->inc;
    p[3] = (uint64_t)(g->inc >> 64);
    p[4] = (uint64_t)g->buf32 | ((uint64_t)(uint32_t)g->has32 << 32);
    p[5] = 0;
}

}  // namespace

// Per-family row recipes (template FAM of the staged kernel):
//   OCX_FAM_GT      g(T) sampler, fast_algorithms.py:231-239 (fp64 rows, ±1 labels drawn
//                   after the rows);
//   OCX_FAM_IID     make_random_iid_stream (sequence_generation.py:54-69): fp32 rows,
//                   y = sign(z·u) with u from _rng(run_seed, 0, 11);
//   OCX_FAM_MASSART make_noisy_iid_stream (:72-89): as IID with u from stream 21, then
//                   y flipped where gen.random(T) < p.
// fp32 arithmetic restates NumPy/OpenBLAS on the host CPU: row norms are NumPy's fp32
// pairwise sums; u's norm is cblas_sdot (fp32 products summed in fp64); z @ u is
// cblas_sgemv (four fma lanes, ((l0+l1)+(l2+l3)), fma tail) — verified bit-exact for
// d = 4, 5 (the reference's families use d = 5), an approximation for other d.
enum { OCX_FAM_GT = 0, OCX_FAM_IID = 1, OCX_FAM_MASSART = 2 };

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

// One wavefront (64 threads) = 64 consecutive sequences = P groups of the layout.
// GT: sequence b = _rng(base_seed, T, run0 + b).  IID/MASSART: sequence b =
// _rng(run_seed[b], T, stream_id[b]) with u from _rng(run_seed[b], 0, 11 | 21).
template <int FAM>
__global__ __launch_bounds__(64) void ocx_gen_staged_kernel(
    uint64_t base_seed, int64_t T, int64_t run0, int64_t B, int d, int P, int C, int64_t G,
    const uint64_t* __restrict__ run_seeds, const uint64_t* __restrict__ stream_ids, double p,
    double* __restrict__ zt, double* __restrict__ ytl, int64_t T_seed,
    const uint64_t* __restrict__ st_in, uint64_t* __restrict__ st_out,
    const uint64_t* __restrict__ lab_in, uint64_t* __restrict__ lab_out) {
    // GT chunk mode (st_in != nullptr): rows resume from st_in[b], T is the chunk length
    // and T_seed the horizon the streams were seeded with; labels come from a second
    // saved cursor lab_in[b] (the stream position after all T_seed·d normals).
    __shared__ Tables tb;
    __shared__ __attribute__((aligned(16))) double rows[64 * OCX_GEN_ROW];
    __shared__ float us[FAM == OCX_FAM_GT ? 1 : 64 * 65];
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
    float* u = us + (FAM == OCX_FAM_GT ? 0 : lane * 65);
    if constexpr (FAM == OCX_FAM_GT) {
        if (st_in != nullptr && live) load_state(&rng, st_in + 6 * b);
        else ocx_rng_init3(&rng, base_seed, (uint64_t)T_seed, (uint64_t)(run0 + (live ? b : 0)));
    } else {
        const uint64_t rs = live ? run_seeds[b] : 0;
        // u: _rng(run_seed, 0, 11 | 21).standard_normal(d) as fp32, / ||u|| (sdot)
        ocx_rng_init3(&rng, rs, 0, FAM == OCX_FAM_IID ? 11 : 21);
        double sq = 0.0;
        for (int j = 0; j < d; ++j) {
            const float v = (float)ocx_standard_normal(&rng, ki, wi, fi);
            u[j] = v;
            sq += (double)(v * v);
        }
        const float n = sqrtf((float)sq);
        if (n > 0.0f)
            for (int j = 0; j < d; ++j) u[j] = u[j] / n;
        ocx_rng_init3(&rng, rs, (uint64_t)T, live ? stream_ids[b] : 0);
    }
    ocx_pw_plan plan;
    ocx_pw_build(&plan, d);
    const int64_t kst = G * T * 64;  // plane stride in ocx_d2 (pair k of a step)
    const int64_t g0 = seq0 / S;  // first group of this wave
    const int64_t gb = b / S;
    double* yrow = ytl + gb * T * S + (b - gb * S);

    for (int64_t t = 0; t < T; ++t) {
        if (live) {
            if constexpr (FAM == OCX_FAM_GT) {
                const double sumsq = ocx_row_sumsq(
                    d, plan, [&]() { return ocx_standard_normal(&rng, ki, wi, fi); },
                    [&](int j, double v) { row[j] = v; });
                const double nrm = sqrt(sumsq);
                const double sc = 1.0 / (nrm > 1.0 ? nrm : 1.0);  // 1.0 / np.maximum(norms, 1.0)
                for (int j = 0; j < d; ++j) row[j] *= sc;
            } else {
                for (int j = 0; j < d; ++j)
                    row[j] = (double)(float)ocx_standard_normal(&rng, ki, wi, fi);
                const float nrm = sqrtf(ocx_f32_pairwise_sq(row, d));
                const float sc = 1.0f / (nrm > 1.0f ? nrm : 1.0f);  // np.maximum, 1.0 / norms
                for (int j = 0; j < d; ++j) row[j] = (double)((float)row[j] * sc);
                const float q = ocx_sgemv_dot(row, u, d);
                yrow[t * S] = (q < 0.0f) ? -1.0 : 1.0;  // np.sign, then y[y == 0] = 1
            }
        } else if (FAM != OCX_FAM_GT && gb < G) {
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
    if (FAM == OCX_FAM_GT && st_out != nullptr && live) save_state(&rng, st_out + 6 * b);
    if (gb >= G) return;
    if constexpr (FAM == OCX_FAM_GT) {
        // labels: choice([-1.0, 1.0], size=T) → integers(0, 2) → top bit of next_uint32
        if (lab_in != nullptr && live) load_state(&rng, lab_in + 6 * b);
        for (int64_t t = 0; t < T; ++t) {
            double yv = 0.0;
            if (live) yv = (ocx_pcg_next32(&rng) >> 31) ? 1.0 : -1.0;
            yrow[t * S] = yv;
        }
        if (lab_out != nullptr && live) save_state(&rng, lab_out + 6 * b);
    } else if constexpr (FAM == OCX_FAM_MASSART) {
        // flips = gen.random(T) < p; y[flips] *= -1.0
        if (live)
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

// Stream positions for chunked generation: st_out[b] = the fresh stream
// _rng(base_seed, T_seed, run0 + b); lab_out[b] = the same stream after the T_seed·d
// standard normals, i.e. where choice(T) starts drawing labels (fast_algorithms.py:234,239).
// The ziggurat consumes a data-dependent number of raw draws, so the only way there is
// to run it.
__global__ __launch_bounds__(OCX_BLOCK) void ocx_gen_seek_kernel(
    uint64_t base_seed, int64_t T_seed, int64_t run0, int64_t B, int64_t d,
    uint64_t* __restrict__ st_out, uint64_t* __restrict__ lab_out) {
    __shared__ Tables tb;
    load_tables(tb);
    __syncthreads();
    auto ki = [&](int i) { return tb.ki[i]; };
    auto wi = [&](int i) { return tb.wi[i]; };
    auto fi = [&](int i) { return tb.fi[i]; };
    const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= B) return;
    ocx_pcg64 rng;
    ocx_rng_init3(&rng, base_seed, (uint64_t)T_seed, (uint64_t)(run0 + b));
    save_state(&rng, st_out + 6 * b);
    double sink = 0.0;
    const int64_t n = T_seed * d;
    int64_t i = 0;
    for (; i + 4 <= n; i += 4) {
#pragma unroll
        for (int k = 0; k < 4; ++k) sink += ocx_standard_normal(&rng, ki, wi, fi);
    }
    for (; i < n; ++i) sink += ocx_standard_normal(&rng, ki, wi, fi);
    save_state(&rng, lab_out + 6 * b);
    if (sink == 1.2345e300) st_out[6 * b + 5] = 1;  // keep the draws alive (never true)
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
    const int64_t Dp = (int64_t)P * C;
    const int64_t G = nlanes / S;
    auto zidx = [&](int64_t t, int64_t j) -> int64_t {
        const int c = (int)(j / C);
        const int r = (int)(j - (int64_t)c * C);
        const int L = s * P + c;
        return (((int64_t)(r >> 1) * G + g) * T + t) * 128 + L * 2 + (r & 1);
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
        hipLaunchKernelGGL(ocx_gen_staged_kernel<OCX_FAM_GT>, dim3(grid), dim3(64), 0, st,
                           base_seed, L->T, run0, L->B, (int)L->d, L->P, L->C, L->G, nullptr,
                           nullptr, 0.0, zt, ytl, L->T, nullptr, nullptr, nullptr, nullptr);
    } else {
        const unsigned grid = (unsigned)((nlanes + OCX_BLOCK - 1) / OCX_BLOCK);
        hipLaunchKernelGGL(ocx_gen_regen_kernel, dim3(grid), dim3(OCX_BLOCK), 0, st, base_seed,
                           L->T, run0, L->B, L->d, L->P, L->C, nlanes, zt, ytl);
    }
    return hipGetLastError();
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
        hipLaunchKernelGGL(ocx_gen_staged_kernel<OCX_FAM_IID>, dim3(grid), dim3(64), 0, st,
                           (uint64_t)0, L->T, (int64_t)0, L->B, (int)L->d, L->P, L->C, L->G,
                           run_seeds, stream_ids, p, zt, ytl, L->T, nullptr, nullptr, nullptr,
                           nullptr);
    else if (family == 2)
        hipLaunchKernelGGL(ocx_gen_staged_kernel<OCX_FAM_MASSART>, dim3(grid), dim3(64), 0, st,
                           (uint64_t)0, L->T, (int64_t)0, L->B, (int)L->d, L->P, L->C, L->G,
                           run_seeds, stream_ids, p, zt, ytl, L->T, nullptr, nullptr, nullptr,
                           nullptr);
    else
        return hipErrorInvalidValue;
    return hipGetLastError();
}

hipError_t ocx_launch_gen_seek(uint64_t base_seed, int64_t T_seed, int64_t run0, int64_t B,
                               int64_t d, uint64_t* st_out, uint64_t* lab_out, hipStream_t st) {
    if (B == 0) return hipSuccess;
    hipLaunchKernelGGL(ocx_gen_seek_kernel, dim3((unsigned)((B + OCX_BLOCK - 1) / OCX_BLOCK)),
                       dim3(OCX_BLOCK), 0, st, base_seed, T_seed, run0, B, d, st_out, lab_out);
    return hipGetLastError();
}

hipError_t ocx_launch_gen_gT_chunk(const ocx_layout* L, int64_t T_seed, const uint64_t* st_in,
                                   uint64_t* st_out, const uint64_t* lab_in, uint64_t* lab_out,
                                   double* zt, double* ytl, hipStream_t st) {
    const int64_t nlanes = L->G * L->S;
    if (nlanes == 0 || L->T == 0) return hipSuccess;
    if ((int64_t)L->P * L->C > 64) return hipErrorNotSupported;
    const unsigned grid = (unsigned)((nlanes + 63) / 64);
    hipLaunchKernelGGL(ocx_gen_staged_kernel<OCX_FAM_GT>, dim3(grid), dim3(64), 0, st,
                       (uint64_t)0, L->T, (int64_t)0, L->B, (int)L->d, L->P, L->C, L->G, nullptr,
                       nullptr, 0.0, zt, ytl, T_seed, st_in, st_out, lab_in, lab_out);
    return hipGetLastError();
}
