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

// np.sum of a float32 vector whose elements arrive one at a time (every lane of the wave
// sums a vector of the same length, so the recursion is uniform).  The recursion
// pw(n) = n <= 128 ? leaf(n) : pw(n2) + pw(n - n2), n2 = n/2 rounded down to a multiple of
// 8, is walked in post order: a frame per pending right half, holding the left half's sum.
struct Pw32 {
    int64_t left;  // elements still to come
    float total;
    bool any;
    int sp, ln, li;  // frames in use; current leaf's length and position
    int fr_len[8];
    float fr_val[8];
    bool fr_has[8];
    float r[8];
    float res;

    __device__ void begin(int64_t n) {
        left = n;
        total = 0.0f;
        any = false;
        if (n > 0) buffer();
    }
    __device__ void buffer() {
        sp = 0;
        descend(left < kPwBuf ? (int)left : kPwBuf);
    }
    __device__ void descend(int n) {
        while (n > kPwBlock) {
            int n2 = n / 2;
            n2 -= n2 % 8;
            fr_len[sp] = n - n2;
            fr_has[sp] = false;
            ++sp;
            n = n2;
        }
        ln = n;
        li = 0;
        res = -0.0f;
    }
    __device__ void push(float v) {
        if (ln < 8) {
            res = res + v;
        } else {
            const int m = ln - (ln & 7);
            if (li < m) {
                const int k = li & 7;
                const bool first = li < 8;
#pragma unroll
                for (int q = 0; q < 8; ++q)
                    if (q == k) r[q] = first ? v : r[q] + v;
            } else {
                if (li == m) res = t32_tree8(r);
                res = res + v;
            }
        }
        ++li;
        --left;
        if (li == ln) done((ln >= 8 && (ln & 7) == 0) ? t32_tree8(r) : res);
    }
    __device__ void done(float v) {
        for (;;) {
            if (sp == 0) {  // a buffer's sum
                total = any ? total + v : v;
                any = true;
                if (left > 0) buffer();
                return;
            }
            const int top = sp - 1;
            if (!fr_has[top]) {  // left half done: walk the right half
                fr_val[top] = v;
                fr_has[top] = true;
                descend(fr_len[top]);
                return;
            }
            v = fr_val[top] + v;
            --sp;
        }
    }
    __device__ float value() const { return any ? total : 0.0f; }
};

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

// np.sum(0.5 * np.abs(z[:n] @ x - y[:n])) (algorithms.py:52-53, :110-111, :117-118)
template <int C>
__device__ __attribute__((noinline)) float t32_loss_sum(const T32Seq& q, const float (&x)[C],
                                                        int64_t n) {
    constexpr int NB = t32_nb(C);
    Pw32 pw;
    pw.begin(n);
    for (int64_t i0 = 0; i0 < n; i0 += NB) {
        float zb[NB][C], yb[NB];
        t32_rows<C, NB>(q, i0, n, zb, yb);
#pragma unroll
        for (int u = 0; u < NB; ++u)
            if (i0 + u < n) {
                const float qv = t32_gemv_row<C>(zb[u], x, i0 + u, n);
                pw.push(0.5f * fabsf(qv - yb[u]));
            }
    }
    return pw.value();
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

template <int C>
hipError_t launch_t32(const ocx_layout* L, const double* zt, const double* yt, int algo,
                      double eta0, const double* thresh, int clip, float* result, double* cum,
                      float* comp, int64_t* sw, hipStream_t st) {
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
