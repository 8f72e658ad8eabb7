// ocx_twin32.hip — the float32 NumPy twin that driver.py imports (algorithms.py:10-171):
// FTRL / FTL (simulate_alg :28-54), single-switch SMART (simulate_SMART_like :65-120) and
// the g(T) sampler's float32 row clip (:157-163), in NumPy 2's float32 arithmetic.
//
// What the twin's NumPy calls compute (probed on this image's NumPy 2.2 / OpenBLAS 0.3.29,
// pinned by tests/golden/twin32.npz):
// * float32 state, Python-float (double) scalars: f32(s) * theta (NEP 50: the Python scalar
//   takes the array's dtype), cum_loss in double, f32(f32(cum) - comp) returned;
// * np.dot / np.linalg.norm / z[t] @ x (OpenBLAS sdot, n < 32): each product rounded to
//   float, the products summed in double, the sum rounded to float;
// * z @ x (the comparator, SMART's prefix test; OpenBLAS sgemv): rows in blocks of four
//   take a float fma chain over the columns, the n mod 4 tail rows a plain float chain,
//   a one-row matrix the sdot rule (exactly the host kernel's for d = 5, the reference's d);
// * np.sum of a float32 vector: NumPy's pairwise sum (leaves of <= 128 elements with eight
//   accumulators) over buffers of 8192 elements, the buffers added in order;
// * np.linalg.norm(z, axis=1): sqrt of the pairwise leaf sum of the row's squares.
// One lane per sequence (layout P = 1, d <= 32): the twin's sequences are short (driver.py:
// T <= 1000, d = 5) and its SMART re-reads the whole prefix every step (:109-111); rows
// are read in blocks of up to 8 steps so their loads are in flight together.
#include <algorithm>
#include <cstdlib>

#include "ocx_internal.h"
#include "ocx_sim_kernels.h"

namespace {

constexpr int kPwBuf = 8192;   // NumPy's reduction buffer: one pairwise sum per buffer
constexpr int kPwBlock = 128;  // PW_BLOCKSIZE: the leaves of the pairwise recursion

// correctly rounded float sqrt and division, through double: 53 >= 2*24 + 2 bits, so the
// second rounding never changes the result (the float intrinsics here are not all rte)
__device__ __forceinline__ float t32_sqrt(float x) { return (float)sqrt((double)x); }
__device__ __forceinline__ float t32_div(float a, float b) { return (float)((double)a / (double)b); }

__device__ __forceinline__ float t32_tree8(const float (&r)[8]) {
    return ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
}

// sdot, n < 32: float products summed in double (padding coordinates add +0)
template <int C>
__device__ __forceinline__ float t32_sdot(const float (&a)[C], const float (&b)[C]) {
    double acc = 0.0;
#pragma unroll
    for (int j = 0; j < C; ++j) acc += (double)(a[j] * b[j]);
    return (float)acc;
}

// row i of an n-row sgemv z @ x
template <int C>
__device__ __forceinline__ float t32_gemv_row(const float (&z)[C], const float (&x)[C], int64_t i,
                                              int64_t n) {
    if (n == 1) return t32_sdot<C>(z, x);
    float a = 0.0f;
    if (i < (n & ~(int64_t)3)) {
#pragma unroll
        for (int j = 0; j < C; ++j) a = fmaf(z[j], x[j], a);
    } else {
#pragma unroll
        for (int j = 0; j < C; ++j) a = a + z[j] * x[j];
    }
    return a;
}

// _action_ftl (algorithms.py:13-15)
template <int C>
__device__ __forceinline__ void t32_ftl(const float (&th)[C], float (&x)[C]) {
    const float n = t32_sqrt(t32_sdot<C>(th, th));
    const float s = n == 0.0f ? 0.0f : -t32_div(1.0f, n);
#pragma unroll
    for (int j = 0; j < C; ++j) x[j] = n == 0.0f ? 0.0f : s * th[j];
}

// _action_ftrl (algorithms.py:17-21)
template <int C>
__device__ __forceinline__ void t32_ftrl(const float (&th)[C], int64_t t, double eta0,
                                         float (&x)[C]) {
    const float sc = (float)(-(eta0 / sqrt((double)(t > 1 ? t : 1))));
#pragma unroll
    for (int j = 0; j < C; ++j) x[j] = sc * th[j];
    const float n = t32_sqrt(t32_sdot<C>(x, x));
    if (n > 1.0f) {
        const float inv = t32_div(1.0f, n);
#pragma unroll
        for (int j = 0; j < C; ++j) x[j] = x[j] * inv;
    }
}

__device__ __forceinline__ double t32_grad(double diff) {
    return diff > 0.0 ? 0.5 : (diff < 0.0 ? -0.5 : 0.0);
}

// z *= 1 / max(||z||, 1) in float32 (algorithms.py:159-160)
template <int C>
__device__ __forceinline__ void t32_clip(float (&z)[C], int d) {
    float sq[C];
#pragma unroll
    for (int j = 0; j < C; ++j) sq[j] = z[j] * z[j];
    float ss = -0.0f;
    if (d < 8) {
#pragma unroll
        for (int j = 0; j < C; ++j)
            if (j < d) ss = ss + sq[j];
    } else {
        if constexpr (C >= 8) {
            float r[8];
#pragma unroll
            for (int q = 0; q < 8; ++q) r[q] = sq[q];
            const int m = d - (d & 7);
#pragma unroll
            for (int j = 8; j < C; ++j)
                if (j < m) r[j & 7] = r[j & 7] + sq[j];
            ss = t32_tree8(r);
#pragma unroll
            for (int j = 8; j < C; ++j)
                if (j >= m && j < d) ss = ss + sq[j];
        }
    }
    const float nrm = t32_sqrt(ss);
    const float inv = t32_div(1.0f, nrm > 1.0f ? nrm : 1.0f);
#pragma unroll
    for (int j = 0; j < C; ++j) z[j] = z[j] * inv;
}

constexpr int t32_nb(int C) { return C <= 8 ? 8 : (C <= 16 ? 4 : 2); }

// one lane's sequence in the P = 1 tiled layout
struct T32Seq {
    const ocx_d2* z;  // pair 0 of step 0
    const double* y;  // step 0
    int64_t kst;      // plane stride (pairs)
    int d;
    int clip;
};

// rows [t0, t0 + NB) below n as the twin sees them (float32; clipped for the g(T) sampler)
template <int C, int NB>
__device__ __forceinline__ void t32_rows(const T32Seq& q, int64_t t0, int64_t n,
                                         float (&zb)[NB][C], float (&yb)[NB]) {
    ocx_d2 raw[NB][C / 2];
#pragma unroll
    for (int u = 0; u < NB; ++u)
        if (t0 + u < n) {
#pragma unroll
            for (int k = 0; k < C / 2; ++k) raw[u][k] = q.z[(t0 + u) * 64 + k * q.kst];
            yb[u] = (float)q.y[(t0 + u) * 64];
        }
#pragma unroll
    for (int u = 0; u < NB; ++u)
        if (t0 + u < n) {
#pragma unroll
            for (int k = 0; k < C / 2; ++k) {
                zb[u][2 * k] = (float)raw[u][k].x;
                zb[u][2 * k + 1] = (float)raw[u][k].y;
            }
            if (q.clip) t32_clip<C>(zb[u], q.d);
        }
}

// 0.5 * |row i of z @ x - y_i| in float32, rows [s, s + NB) below e
template <int C, int NB>
__device__ __forceinline__ void t32_block_losses(const T32Seq& q, const float (&x)[C], int64_t n,
                                                 int64_t s, int64_t e, float (&l)[NB]) {
    float zb[NB][C], yb[NB];
    t32_rows<C, NB>(q, s, e, zb, yb);
#pragma unroll
    for (int u = 0; u < NB; ++u)
        l[u] = s + u < e ? 0.5f * fabsf(t32_gemv_row<C>(zb[u], x, s + u, n) - yb[u]) : 0.0f;
}

// One leaf of NumPy's pairwise sum: m losses from row s (every leaf of a buffer longer
// than 7 starts at a multiple of 8, since the recursion cuts at multiples of 8): eight
// accumulators over the whole groups of 8, their tree, then the tail one by one
template <int C>
__device__ __forceinline__ float t32_leaf(const T32Seq& q, const float (&x)[C], int64_t n,
                                          int64_t s, int m) {
    float l[8];
    if (m < 8) {
        t32_block_losses<C, 8>(q, x, n, s, s + m, l);
        float res = -0.0f;
#pragma unroll
        for (int u = 0; u < 8; ++u)
            if (u < m) res = res + l[u];
        return res;
    }
    const int mfull = m - (m & 7);
    float r[8];
    t32_block_losses<C, 8>(q, x, n, s, s + 8, r);
    for (int i = 8; i < mfull; i += 8) {
        t32_block_losses<C, 8>(q, x, n, s + i, s + i + 8, l);
#pragma unroll
        for (int u = 0; u < 8; ++u) r[u] = r[u] + l[u];
    }
    float res = t32_tree8(r);
    if (m & 7) {
        t32_block_losses<C, 8>(q, x, n, s + mfull, s + m, l);
#pragma unroll
        for (int u = 0; u < 8; ++u)
            if (u < (m & 7)) res = res + l[u];
    }
    return res;
}

// NumPy's pairwise sum of one buffer of nb <= 8192 losses from row s0: pw(m) = m <= 128 ?
// leaf(m) : pw(m2) + pw(m - m2), m2 = m/2 cut down to a multiple of 8, walked in post
// order with a frame per pending right half (the frames are touched once per leaf)
template <int C>
__device__ float t32_pw_buffer(const T32Seq& q, const float (&x)[C], int64_t n, int64_t s0,
                               int nb) {
    int fr_len[8];
    float fr_val[8];
    bool fr_has[8];
    int sp = 0, m = nb;
    int64_t pos = s0;
    for (;;) {
        while (m > kPwBlock) {
            int m2 = m / 2;
            m2 -= m2 % 8;
            fr_len[sp] = m - m2;
            fr_has[sp] = false;
            ++sp;
            m = m2;
        }
        float v = t32_leaf<C>(q, x, n, pos, m);
        pos += m;
        while (sp > 0 && fr_has[sp - 1]) {
            v = fr_val[sp - 1] + v;
            --sp;
        }
        if (sp == 0) return v;
        fr_val[sp - 1] = v;
        fr_has[sp - 1] = true;
        m = fr_len[sp - 1];
    }
}

// np.sum(0.5 * np.abs(z[:n] @ x - y[:n])) (algorithms.py:52-53, :110-111, :117-118):
// one pairwise sum per 8192-element buffer, the buffers added in order
template <int C>
__device__ __attribute__((noinline)) float t32_loss_sum(const T32Seq& q, const float (&x)[C],
                                                        int64_t n) {
    float total = 0.0f;
    for (int64_t s0 = 0; s0 < n; s0 += kPwBuf) {
        const int nb = (int)(n - s0 < kPwBuf ? n - s0 : kPwBuf);
        const float p = t32_pw_buffer<C>(q, x, n, s0, nb);
        total = s0 == 0 ? p : total + p;
    }
    return total;
}

template <int C>
__global__ __launch_bounds__(64) void ocx_twin32_kernel(
    const double* __restrict__ zt, const double* __restrict__ yt, int64_t B, int64_t T,
    int64_t G, int d, int algo, double eta0, const double* __restrict__ thresh, int clip,
    float* __restrict__ result, double* __restrict__ cum_out, float* __restrict__ comp_out,
    int64_t* __restrict__ sw_out) {
    constexpr int NB = t32_nb(C);
    const int64_t g = blockIdx.x;
    const int s = threadIdx.x;
    const int64_t b = g * 64 + s;
    const bool live = b < B;
    T32Seq q;
    q.z = reinterpret_cast<const ocx_d2*>(zt) + g * T * 64 + s;
    q.y = yt + g * T * 64 + s;
    q.kst = G * T * 64;
    q.d = d;
    q.clip = clip;

    float th[C], x[C];
#pragma unroll
    for (int j = 0; j < C; ++j) th[j] = 0.0f;
    double cum = 0.0;
    int64_t sw = -1;
    if (algo != 2) {
        // simulate_alg (algorithms.py:28-50)
        for (int64_t t0 = 0; t0 < T; t0 += NB) {
            float zb[NB][C], yb[NB];
            t32_rows<C, NB>(q, t0, T, zb, yb);
#pragma unroll
            for (int u = 0; u < NB; ++u)
                if (t0 + u < T) {
                    if (algo == 0)
                        t32_ftrl<C>(th, t0 + u + 1, eta0, x);
                    else
                        t32_ftl<C>(th, x);
                    const double qv = (double)t32_sdot<C>(zb[u], x);
                    const double yv = (double)yb[u];
                    cum += 0.5 * fabs(qv - yv);
                    const float gq = (float)t32_grad(qv - yv);
#pragma unroll
                    for (int j = 0; j < C; ++j) th[j] = th[j] + gq * zb[u][j];
                }
        }
    } else {
        // simulate_SMART_like (algorithms.py:65-120): FTL until its regret against the best
        // constant action so far reaches the threshold, FTRL from the next step on.  One
        // step at a time: the prefix test re-reads rows 0..t every step before the switch.
        float thr[C], sx[C];
#pragma unroll
        for (int j = 0; j < C; ++j) thr[j] = 0.0f;
        const float th32 = live ? (float)thresh[b] : 0.0f;
        bool switched = false;
        double ftl_loss = 0.0;
        for (int64_t t = 0; t < T; ++t) {
            float zb[1][C], yb[1];
            t32_rows<C, 1>(q, t, T, zb, yb);
            const float(&zr)[C] = zb[0];
            const double yv = (double)yb[0];
            t32_ftl<C>(th, x);
            const double pf = (double)t32_sdot<C>(zr, x);
            const float gf = (float)t32_grad(pf - yv);
#pragma unroll
            for (int j = 0; j < C; ++j) th[j] = th[j] + gf * zr[j];
            const double lf = 0.5 * fabs(pf - yv);
            ftl_loss += lf;
            if (switched) {
                t32_ftrl<C>(thr, t + 1, eta0, x);
                const double pr = (double)t32_sdot<C>(zr, x);
                cum += 0.5 * fabs(pr - yv);
                const float gr = (float)t32_grad(pr - yv);
#pragma unroll
                for (int j = 0; j < C; ++j) thr[j] = thr[j] + gr * zr[j];
            } else {
                cum += lf;
                t32_ftl<C>(th, sx);
                const float sl = t32_loss_sum<C>(q, sx, t + 1);
                if ((float)ftl_loss - sl >= th32) {
                    switched = true;
                    sw = t;
                }
            }
        }
    }
    t32_ftl<C>(th, x);  // the comparator: FTL on the whole sequence (:51-53, :116-118)
    const float comp = t32_loss_sum<C>(q, x, T);
    if (live) {
        result[b] = (float)cum - comp;
        if (cum_out) cum_out[b] = cum;
        if (comp_out) comp_out[b] = comp;
        if (sw_out) sw_out[b] = sw;
    }
}

// ---- SMART, one wavefront per sequence --------------------------------------------------
// simulate_SMART_like re-sums its whole prefix every step before the switch (:109-111):
// O(T^2) work per sequence, latency-bound in a lane of its own (T = 1000: 0.3 s for one
// sequence, against ~20 ms for NumPy).  Here the sequence's rows sit in LDS as float and
// the wave splits each prefix sum the way NumPy's pairwise recursion does: its leaves (of
// <= 128 losses, all starting at multiples of 8) and their eight accumulator chains are
// independent, so lane 8*i + k runs chain k of leaf i; lane 8*i then folds the chains
// (tree of 8) and the leaf's tail, and the leaf sums are combined in the recursion's post
// order.  The scalar part of the step (actions, theta updates) runs on every lane alike.
constexpr int kWaveLeaves = 128;  // leaves of an 8192-element buffer: at most 8192/64

struct T32Wave {
    const float* z;  // LDS rows [T][C]
    const float* y;  // LDS labels [T]
    float* red;      // [64]
    int* lstart;     // [kWaveLeaves]
    int* llen;
    float* lsum;
};

template <int C>
__device__ __forceinline__ float t32_wave_loss(const T32Wave& w, const float (&x)[C], int i, int n) {
    float zr[C];
#pragma unroll
    for (int j = 0; j < C; ++j) zr[j] = w.z[i * C + j];
    return 0.5f * fabsf(t32_gemv_row<C>(zr, x, i, n) - w.y[i]);
}

// np.sum(0.5 * np.abs(z[:n] @ x - y[:n])), n <= 8192 (one NumPy buffer), on the whole wave
template <int C>
__device__ float t32_wave_loss_sum(const T32Wave& w, const float (&x)[C], int n, int lane) {
    if (n == 0) return 0.0f;
    // the leaves, in order
    int nl = 0;
    {
        int stk[8];
        int sp = 0, m = n, pos = 0;
        for (;;) {
            while (m > kPwBlock) {
                int m2 = m / 2;
                m2 -= m2 % 8;
                stk[sp++] = m - m2;
                m = m2;
            }
            if (lane == 0) {
                w.lstart[nl] = pos;
                w.llen[nl] = m;
            }
            ++nl;
            pos += m;
            if (sp == 0) break;
            m = stk[--sp];
        }
    }
    __syncthreads();
    for (int base = 0; base < nl; base += 8) {
        const int leaf = base + (lane >> 3), k = lane & 7;
        int s = 0, m = 0;
        if (leaf < nl) {
            s = w.lstart[leaf];
            m = w.llen[leaf];
        }
        const int mfull = m - (m & 7);
        float r = 0.0f;
        if (m >= 8) {
            r = t32_wave_loss<C>(w, x, s + k, n);
            for (int i = s + k + 8; i < s + mfull; i += 8) r = r + t32_wave_loss<C>(w, x, i, n);
        }
        w.red[lane] = r;
        __syncthreads();
        if (k == 0 && leaf < nl) {
            float res;
            int i0;
            if (m >= 8) {
                float rr[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) rr[u] = w.red[lane + u];
                res = t32_tree8(rr);
                i0 = s + mfull;
            } else {
                res = -0.0f;
                i0 = s;
            }
            for (int i = i0; i < s + m; ++i) res = res + t32_wave_loss<C>(w, x, i, n);
            w.lsum[leaf] = res;
        }
        __syncthreads();
    }
    // the recursion's post order over the leaf sums
    int fr_len[8];
    float fr_val[8];
    bool fr_has[8];
    int sp = 0, m = n, li = 0;
    for (;;) {
        while (m > kPwBlock) {
            int m2 = m / 2;
            m2 -= m2 % 8;
            fr_len[sp] = m - m2;
            fr_has[sp] = false;
            ++sp;
            m = m2;
        }
        float v = w.lsum[li++];
        while (sp > 0 && fr_has[sp - 1]) {
            v = fr_val[sp - 1] + v;
            --sp;
        }
        if (sp == 0) {
            __syncthreads();  // leaf arrays are rewritten by the next call
            return v;
        }
        fr_val[sp - 1] = v;
        fr_has[sp - 1] = true;
        m = fr_len[sp - 1];
    }
}

template <int C>
__global__ __launch_bounds__(64) void ocx_twin32_smart_wave_kernel(
    const double* __restrict__ zt, const double* __restrict__ yt, int64_t B, int64_t T,
    int64_t G, double eta0, const double* __restrict__ thresh, float* __restrict__ result,
    double* __restrict__ cum_out, float* __restrict__ comp_out, int64_t* __restrict__ sw_out) {
    extern __shared__ float t32_lds[];
    __shared__ float red[64];
    __shared__ int lstart[kWaveLeaves], llen[kWaveLeaves];
    __shared__ float lsum[kWaveLeaves];
    const int lane = threadIdx.x;
    const int64_t b = blockIdx.x;
    const int n = (int)T;
    float* zs = t32_lds;
    float* ys = t32_lds + (int64_t)n * C;
    {
        // stage the sequence (lane L of wave-group g in the P = 1 layout) as float rows
        const int64_t g = b / 64;
        const int sl = (int)(b % 64);
        const ocx_d2* zp = reinterpret_cast<const ocx_d2*>(zt) + g * T * 64 + sl;
        const int64_t kst = G * T * 64;
        for (int t = lane; t < n; t += 64) {
#pragma unroll
            for (int k = 0; k < C / 2; ++k) {
                const ocx_d2 v = zp[(int64_t)t * 64 + k * kst];
                zs[t * C + 2 * k] = (float)v.x;
                zs[t * C + 2 * k + 1] = (float)v.y;
            }
            ys[t] = (float)yt[(g * T + t) * 64 + sl];
        }
    }
    __syncthreads();
    T32Wave w{zs, ys, red, lstart, llen, lsum};
    float th[C], thr[C], x[C], sx[C];
#pragma unroll
    for (int j = 0; j < C; ++j) th[j] = thr[j] = 0.0f;
    const float th32 = (float)thresh[b];
    bool switched = false;
    double ftl_loss = 0.0, cum = 0.0;
    int64_t sw = -1;
    for (int t = 0; t < n; ++t) {
        float zr[C];
#pragma unroll
        for (int j = 0; j < C; ++j) zr[j] = zs[t * C + j];
        const double yv = (double)ys[t];
        t32_ftl<C>(th, x);
        const double pf = (double)t32_sdot<C>(zr, x);
        const float gf = (float)t32_grad(pf - yv);
#pragma unroll
        for (int j = 0; j < C; ++j) th[j] = th[j] + gf * zr[j];
        const double lf = 0.5 * fabs(pf - yv);
        ftl_loss += lf;
        if (switched) {
            t32_ftrl<C>(thr, t + 1, eta0, x);
            const double pr = (double)t32_sdot<C>(zr, x);
            cum += 0.5 * fabs(pr - yv);
            const float gr = (float)t32_grad(pr - yv);
#pragma unroll
            for (int j = 0; j < C; ++j) thr[j] = thr[j] + gr * zr[j];
        } else {
            cum += lf;
            t32_ftl<C>(th, sx);
            const float sl = t32_wave_loss_sum<C>(w, sx, t + 1, lane);
            if ((float)ftl_loss - sl >= th32) {
                switched = true;
                sw = t;
            }
        }
    }
    t32_ftl<C>(th, x);
    const float comp = t32_wave_loss_sum<C>(w, x, n, lane);
    if (lane == 0) {
        result[b] = (float)cum - comp;
        if (cum_out) cum_out[b] = cum;
        if (comp_out) comp_out[b] = comp;
        if (sw_out) sw_out[b] = sw;
    }
}

constexpr int64_t kWaveLdsBytes = 60 * 1024;  // rows of one sequence staged in LDS (<= 64 KB with the static arrays)

template <int C>
hipError_t launch_t32(const ocx_layout* L, const double* zt, const double* yt, int algo,
                      double eta0, const double* thresh, int clip, float* result, double* cum,
                      float* comp, int64_t* sw, hipStream_t st) {
    const int64_t lds = L->T * (C + 1) * 4;
    // OCX_TWIN32_SMART_LANES=1 (tests): the lane-per-sequence kernel for SMART as well
    static const bool lanes_only = [] {
        const char* e = std::getenv("OCX_TWIN32_SMART_LANES");
        return e != nullptr && e[0] == '1';
    }();
    if (algo == 2 && !clip && lds <= kWaveLdsBytes && !lanes_only) {
        // SMART: a wavefront per sequence wherever the rows fit the LDS (T <= 2340 at d = 5)
        hipLaunchKernelGGL((ocx_twin32_smart_wave_kernel<C>), dim3((unsigned)L->B), dim3(64),
                           (size_t)lds, st, zt, yt, L->B, L->T, L->G, eta0, thresh, result, cum,
                           comp, sw);
        return hipGetLastError();
    }
    hipLaunchKernelGGL((ocx_twin32_kernel<C>), dim3((unsigned)L->G), dim3(64), 0, st, zt, yt, L->B,
                       L->T, L->G, (int)L->d, algo, eta0, thresh, clip, result, cum, comp, sw);
    return hipGetLastError();
}

__global__ void ocx_pack32_z_kernel(const float* __restrict__ z, double* __restrict__ zt,
                                    int64_t B, int64_t T, int64_t d, int64_t G, int64_t total) {
    for (int64_t o = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; o < total;
         o += (int64_t)gridDim.x * blockDim.x) {
        // o = ((k*G + g)*T + t)*128 + 2s + e, coordinate 2k + e of sequence 64g + s
        const int64_t row = o >> 7;
        const int s = (int)((o & 127) >> 1), e = (int)(o & 1);
        const int64_t kg = row / T;
        const int64_t t = row - kg * T;
        const int64_t k = kg / G, g = kg - k * G;
        const int64_t b = g * 64 + s;
        const int64_t j = 2 * k + e;
        zt[o] = (b < B && j < d) ? (double)z[(b * T + t) * d + j] : 0.0;
    }
}

__global__ void ocx_pack32_y_kernel(const float* __restrict__ y, double* __restrict__ ytl,
                                    int64_t B, int64_t T, int64_t total) {
    for (int64_t o = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; o < total;
         o += (int64_t)gridDim.x * blockDim.x) {
        const int64_t tix = o >> 6;
        const int s = (int)(o & 63);
        const int64_t g = tix / T, t = tix - g * T;
        const int64_t b = g * 64 + s;
        ytl[o] = b < B ? (double)y[b * T + t] : 0.0;
    }
}

}  // namespace

hipError_t ocx_launch_twin32(const ocx_layout* L, const double* zt, const double* yt, int algo,
                             double eta0, const double* thresh, int clip, float* result,
                             double* cum, float* comp, int64_t* sw, hipStream_t st) {
    if (L->G == 0) return hipSuccess;
    if (L->P != 1 || L->S != 64) return hipErrorInvalidValue;
    switch (L->C) {
        case 2: return launch_t32<2>(L, zt, yt, algo, eta0, thresh, clip, result, cum, comp, sw, st);
        case 4: return launch_t32<4>(L, zt, yt, algo, eta0, thresh, clip, result, cum, comp, sw, st);
        case 6: return launch_t32<6>(L, zt, yt, algo, eta0, thresh, clip, result, cum, comp, sw, st);
        case 8: return launch_t32<8>(L, zt, yt, algo, eta0, thresh, clip, result, cum, comp, sw, st);
        case 12: return launch_t32<12>(L, zt, yt, algo, eta0, thresh, clip, result, cum, comp, sw, st);
        case 16: return launch_t32<16>(L, zt, yt, algo, eta0, thresh, clip, result, cum, comp, sw, st);
        case 24: return launch_t32<24>(L, zt, yt, algo, eta0, thresh, clip, result, cum, comp, sw, st);
        case 32: return launch_t32<32>(L, zt, yt, algo, eta0, thresh, clip, result, cum, comp, sw, st);
        default: return hipErrorInvalidValue;
    }
}

hipError_t ocx_launch_pack32(const ocx_layout* L, const float* z, const float* y, double* zt,
                             double* ytl, hipStream_t st) {
    if (L->P != 1) return hipErrorInvalidValue;
    const int64_t zn = L->z_elems, yn = L->y_elems;
    if (zn > 0) {
        const unsigned grid = (unsigned)std::min<int64_t>((zn + 255) / 256, 65536);
        hipLaunchKernelGGL(ocx_pack32_z_kernel, dim3(grid), dim3(256), 0, st, z, zt, L->B, L->T,
                           L->d, L->G, zn);
    }
    if (yn > 0) {
        const unsigned grid = (unsigned)std::min<int64_t>((yn + 255) / 256, 65536);
        hipLaunchKernelGGL(ocx_pack32_y_kernel, dim3(grid), dim3(256), 0, st, y, ytl, L->B, L->T, yn);
    }
    return hipGetLastError();
}
