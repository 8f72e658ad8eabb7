// ocx_smart_wave.hip — SMART (fast_algorithms.py:118-164) with one wavefront per
// sequence, for batches too small to fill the GPU with the lane-group kernel.
//
// SMART's cost is the prefix re-scan before the switch: at every step t it sums
// ½|z_i·s_t − y_i| over i = 0..t in order, O(T²) dependent additions per sequence.
// The lane-group kernel (ocx_sim.hip) walks that prefix with one lane group per
// sequence, so a driver-sized batch (a few hundred sequences) leaves the GPU idle on
// the latency of every term.  Here the 64 lanes compute 64 terms of the prefix at
// once (their dot products are independent) and the wave adds them to the running
// sum in order from LDS, so only the additions themselves stay sequential — the
// reference's own summation order, bit for bit.  Lane j < d keeps coordinate j of the
// FTL and FTRL states; the d-term sums of the actions use the same ordered adder.
#include "ocx_internal.h"
#include "ocx_sim_kernels.h"

namespace {

constexpr int kSmartBlock = 256;
constexpr int kSpec = 4;  // pre-switch steps whose prefix re-scans run side by side

// acc + v_0 + v_1 + ... + v_{n-1}, left to right (v_k = lane k's value), n <= 64.
// The values go through the wave's LDS slot `buf`; every lane returns the same sum.
__device__ __forceinline__ double ordered_sum(double acc, double v, int n, double* buf,
                                              int lane) {
    buf[lane] = v;
    __builtin_amdgcn_wave_barrier();
    int k = 0;
    for (; k + 8 <= n; k += 8) {
        double t[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) t[u] = buf[k + u];
#pragma unroll
        for (int u = 0; u < 8; ++u) acc += t[u];
    }
    for (; k < n; ++k) acc += buf[k];
    __builtin_amdgcn_wave_barrier();
    return acc;
}

__device__ __forceinline__ double grad(double diff) {
    return diff > 0.0 ? 0.5 : (diff < 0.0 ? -0.5 : 0.0);
}

}  // namespace

template <int DMAX>
__global__ __launch_bounds__(kSmartBlock) void ocx_smart_wave_kernel(
    const double* __restrict__ zt, const double* __restrict__ yt, int64_t B, int64_t T, int d,
    int P, int C, int64_t G, const double* __restrict__ thresh, double eta0,
    double* __restrict__ regret, int64_t* __restrict__ switch_step) {
    __shared__ double bufs[kSmartBlock * kSpec];
    const int lane = threadIdx.x & 63;
    double* buf = bufs + (threadIdx.x & ~63) * kSpec;  // kSpec x 64 doubles per wave
    const int64_t b = (int64_t)blockIdx.x * (kSmartBlock / 64) + (threadIdx.x >> 6);
    if (b >= B) return;
    const int S = 64 / P;
    const int64_t g = b / S;
    const int s = (int)(b - g * S);
    const bool own = lane < d;  // this lane's coordinate j = lane exists
    // tile offset of coordinate `lane` of this sequence at step 0 (+ t·128 for step t)
    int64_t zoff = 0;
    if (own) {
        const int c = lane / C, rr = lane - c * C;
        zoff = ((int64_t)(rr >> 1) * G + g) * T * 128 + (s * P + c) * 2 + (rr & 1);
    }
    const double* __restrict__ yp = yt + g * T * S + s;  // y_t = yp[t * S]
    const double th_sw = thresh[b];

    // ½|z_i·sv − y_i| summed over rows i < n in order: lane ℓ forms the terms of rows
    // i0 + ℓ (coordinates read from the lanes that own them), the wave adds them.  With
    // DMAX > 0 (d <= DMAX) the next chunk's rows are loaded while this chunk is summed.
    auto offset_of = [&](int j) -> int64_t {
        return ((int64_t)__builtin_amdgcn_readlane((int)(zoff >> 32), j) << 32) |
               (uint32_t)__builtin_amdgcn_readlane((int)zoff, j);
    };
    auto coord_of = [&](double v, int j) -> double {
        return __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(v), j),
                                __builtin_amdgcn_readlane(__double2loint(v), j));
    };
    auto prefix_loss = [&](double sv, int64_t n) -> double {
        double tot = 0.0;
        if constexpr (DMAX > 0) {
            double zc[DMAX], yc = 0.0;
            auto load = [&](int64_t i0, double (&zb)[DMAX], double& yb) {
                const int64_t i = (i0 + lane < n) ? i0 + lane : 0;
#pragma unroll
                for (int j = 0; j < DMAX; ++j) zb[j] = (j < d) ? zt[offset_of(j) + i * 128] : 0.0;
                yb = yp[i * S];
            };
            if (n > 0) load(0, zc, yc);
            for (int64_t i0 = 0; i0 < n; i0 += 64) {
                const int m = (int)((n - i0) < 64 ? (n - i0) : 64);
                double zn[DMAX], yn = 0.0;
                if (i0 + 64 < n) load(i0 + 64, zn, yn);
                double q = 0.0;
#pragma unroll
                for (int j = 0; j < DMAX; ++j)
                    if (j < d) q += zc[j] * coord_of(sv, j);
                const double h = 0.5 * fabs(q - yc);
                tot = ordered_sum(tot, h, m, buf, lane);
#pragma unroll
                for (int j = 0; j < DMAX; ++j) zc[j] = zn[j];
                yc = yn;
            }
        } else {
            for (int64_t i0 = 0; i0 < n; i0 += 64) {
                const int m = (int)((n - i0) < 64 ? (n - i0) : 64);
                const int64_t i = i0 + (lane < m ? lane : 0);
                double q = 0.0;
                for (int j = 0; j < d; ++j) q += zt[offset_of(j) + i * 128] * coord_of(sv, j);
                const double h = 0.5 * fabs(q - yp[i * S]);
                tot = ordered_sum(tot, h, m, buf, lane);
            }
        }
        return tot;
    };
    // The prefix losses of kSpec consecutive steps t..t+K-1 at once: sv[k] = s_{t+k}, rows
    // 0..t+k each.  The chunk's rows are shared; a row beyond t+k contributes +0.0 to
    // chain k, which leaves that sum unchanged.  The K ordered chains interleave.
    auto prefix_loss_multi = [&](const double (&sv)[kSpec], int64_t t, int K,
                                 double (&out)[kSpec]) {
#pragma unroll
        for (int k = 0; k < kSpec; ++k) out[k] = 0.0;
        const int64_t n = t + K;
        auto chunk = [&](int64_t i0, const double* zr, double yr) {
            const int m = (int)((n - i0) < 64 ? (n - i0) : 64);
            const int64_t i = i0 + lane;
#pragma unroll
            for (int k = 0; k < kSpec; ++k) {
                double q = 0.0;
                if constexpr (DMAX > 0) {
#pragma unroll
                    for (int j = 0; j < DMAX; ++j)
                        if (j < d) q += zr[j] * coord_of(sv[k], j);
                } else {
                    const int64_t ii = (i < n) ? i : 0;
                    for (int j = 0; j < d; ++j) q += zt[offset_of(j) + ii * 128] * coord_of(sv[k], j);
                }
                buf[k * 64 + lane] = (k < K && i <= t + k) ? 0.5 * fabs(q - yr) : 0.0;
            }
            __builtin_amdgcn_wave_barrier();
            int u = 0;
            for (; u + 4 <= m; u += 4) {
#pragma unroll
                for (int v = 0; v < 4; ++v)
#pragma unroll
                    for (int k = 0; k < kSpec; ++k) out[k] += buf[k * 64 + u + v];
            }
            for (; u < m; ++u)
#pragma unroll
                for (int k = 0; k < kSpec; ++k) out[k] += buf[k * 64 + u];
            __builtin_amdgcn_wave_barrier();
        };
        if constexpr (DMAX > 0) {
            double zc[DMAX], yc = 0.0;
            auto load = [&](int64_t i0, double (&zb)[DMAX], double& yb) {
                const int64_t i = (i0 + lane < n) ? i0 + lane : 0;
#pragma unroll
                for (int j = 0; j < DMAX; ++j) zb[j] = (j < d) ? zt[offset_of(j) + i * 128] : 0.0;
                yb = yp[i * S];
            };
            load(0, zc, yc);
            for (int64_t i0 = 0; i0 < n; i0 += 64) {
                double zn[DMAX], yn = 0.0;
                if (i0 + 64 < n) load(i0 + 64, zn, yn);
                chunk(i0, zc, yc);
#pragma unroll
                for (int j = 0; j < DMAX; ++j) zc[j] = zn[j];
                yc = yn;
            }
        } else {
            for (int64_t i0 = 0; i0 < n; i0 += 64) {
                const int64_t i = (i0 + lane < n) ? i0 + lane : 0;
                chunk(i0, nullptr, yp[i * S]);
            }
        }
    };
    // FTL action (fast_algorithms.py:37-49) of the state held in `th`, coordinate `lane`
    auto action_ftl = [&](double th) -> double {
        const double n2 = ordered_sum(0.0, own ? th * th : 0.0, d, buf, lane);
        if (n2 == 0.0) return 0.0;
        const double scale = -(1.0 / sqrt(n2));
        return scale * th;
    };

    double tf = 0.0, tr = 0.0;  // theta_ftl, theta_ftrl (coordinate `lane`)
    bool switched = false;
    int64_t sw = -1;
    double ftl_loss = 0.0, total_loss = 0.0;
    // post-switch step t (:140-154): FTL still updated, FTRL played with its own theta
    auto post_switch_step = [&](int64_t t) {
        const double z = own ? zt[zoff + t * 128] : 0.0;
        const double yv = yp[t * S];
        const double xf = action_ftl(tf);
        const double pf = ordered_sum(0.0, own ? z * xf : 0.0, d, buf, lane);
        const double dfl = pf - yv;
        tf += grad(dfl) * z;
        ftl_loss += 0.5 * fabs(dfl);
        const double sc = -(eta0 / sqrt((double)(t + 1)));
        double xr = sc * tr;
        const double n2 = ordered_sum(0.0, own ? xr * xr : 0.0, d, buf, lane);
        if (n2 > 1.0) xr *= 1.0 / sqrt(n2);
        const double pr = ordered_sum(0.0, own ? z * xr : 0.0, d, buf, lane);
        const double dr = pr - yv;
        total_loss += 0.5 * fabs(dr);
        tr += grad(dr) * z;
    };
    // Pre-switch steps go kSpec at a time: the FTL part of each step (which never depends
    // on the switch) runs ahead, the kSpec prefix re-scans run side by side, and the
    // switch test is then applied in step order.  Steps after a switch inside the group
    // already have their FTL update and are replayed as FTRL steps.
    double xf_next = 0.0;  // FTL(theta_ftl) as it stands: FTL(0) = 0
    int64_t t = 0;
    while (t < T) {
        if (switched) {
            post_switch_step(t);
            ++t;
            continue;
        }
        const int K = (T - t) < kSpec ? (int)(T - t) : kSpec;
        double sv[kSpec], lf[kSpec], fl[kSpec];
#pragma unroll
        for (int k = 0; k < kSpec; ++k) {
            sv[k] = 0.0;
            lf[k] = fl[k] = 0.0;
            if (k < K) {
                const double z = own ? zt[zoff + (t + k) * 128] : 0.0;
                const double yv = yp[(t + k) * S];
                const double pf = ordered_sum(0.0, own ? z * xf_next : 0.0, d, buf, lane);
                const double dfl = pf - yv;
                tf += grad(dfl) * z;
                lf[k] = 0.5 * fabs(dfl);
                ftl_loss += lf[k];
                fl[k] = ftl_loss;
                sv[k] = action_ftl(tf);  // s_{t+k} (:157); also the next step's FTL action
                xf_next = sv[k];
            }
        }
        double sl[kSpec];
        prefix_loss_multi(sv, t, K, sl);
        int ks = -1;
#pragma unroll
        for (int k = 0; k < kSpec; ++k) {
            if (k < K && ks < 0) {
                total_loss += lf[k];  // :156
                if (fl[k] - sl[k] >= th_sw) ks = k;
            }
        }
        if (ks >= 0) {
            switched = true;
            sw = t + ks;
            for (int k = ks + 1; k < K; ++k) {  // FTRL on the group's later steps
                const int64_t tk = t + k;
                const double z = own ? zt[zoff + tk * 128] : 0.0;
                const double yv = yp[tk * S];
                const double sc = -(eta0 / sqrt((double)(tk + 1)));
                double xr = sc * tr;
                const double n2 = ordered_sum(0.0, own ? xr * xr : 0.0, d, buf, lane);
                if (n2 > 1.0) xr *= 1.0 / sqrt(n2);
                const double pr = ordered_sum(0.0, own ? z * xr : 0.0, d, buf, lane);
                const double dr = pr - yv;
                total_loss += 0.5 * fabs(dr);
                tr += grad(dr) * z;
            }
        }
        t += K;
    }
    // final comparator = FTL(theta_ftl) (:162-163)
    const double comp = prefix_loss(action_ftl(tf), T);
    if (lane == 0) {
        regret[b] = total_loss - comp;
        if (switch_step) switch_step[b] = sw;
    }
}

hipError_t ocx_launch_smart_wave(const ocx_layout* L, const double* zt, const double* yt,
                                 const double* th, double eta0, double* reg, int64_t* sw,
                                 hipStream_t st) {
    if (L->B == 0) return hipSuccess;
    if (L->d > 64) return hipErrorNotSupported;
    const unsigned grid = (unsigned)((L->B + (kSmartBlock / 64) - 1) / (kSmartBlock / 64));
    if (L->d <= 8)
        hipLaunchKernelGGL(ocx_smart_wave_kernel<8>, dim3(grid), dim3(kSmartBlock), 0, st, zt, yt,
                           L->B, L->T, (int)L->d, L->P, L->C, L->G, th, eta0, reg, sw);
    else
        hipLaunchKernelGGL(ocx_smart_wave_kernel<0>, dim3(grid), dim3(kSmartBlock), 0, st, zt, yt,
                           L->B, L->T, (int)L->d, L->P, L->C, L->G, th, eta0, reg, sw);
    return hipGetLastError();
}
