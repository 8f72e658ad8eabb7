// ocx_device_math.h — per-step device arithmetic shared by the simulation kernels:
// tile loads, per-sequence totals (tree / chained), FTRL & FTL actions, z·x.
// Every function follows the reference's operation order (fast_algorithms.py:11-66).
#pragma once
#include "ocx_internal.h"

// Register-ring depth (steps in flight per wave) by coordinates per lane; tuned on
// MI355X with tools/tune.py (the -D overrides build the tuning variants).
#ifndef OCX_NB_LE8
#define OCX_NB_LE8 4
#endif
#ifndef OCX_NB_16
#define OCX_NB_16 3
#endif
#ifndef OCX_NB_GE32
#define OCX_NB_GE32 2
#endif
#ifndef OCX_LOAD_NT
#define OCX_LOAD_NT 1
#endif

constexpr int nb_for(int C) { return C <= 8 ? OCX_NB_LE8 : (C <= 16 ? OCX_NB_16 : OCX_NB_GE32); }

template <int C>
__device__ __forceinline__ void ocx_load_tile(ocx_d2 (&dst)[C / 2], const ocx_d2* __restrict__ p,
                                              int64_t kst) {
    // pair k of this lane's step lives in plane k, kst = G*T*64 ocx_d2 further on
#pragma unroll
    for (int k = 0; k < C / 2; ++k) {
#if OCX_LOAD_NT
        dst[k] = __builtin_nontemporal_load(p + k * kst);
#else
        dst[k] = p[k * kst];
#endif
    }
}

__device__ __forceinline__ double ocx_zj(const ocx_d2* zb, int j) {
    return (j & 1) ? zb[j >> 1].y : zb[j >> 1].x;
}


// ---------------------------------------------------------------------------
// Per-sequence totals of C per-lane products p[j] (coordinate c*C + j).
//   tree  (CHAIN=false): lane-local sequential sum, then the P-lane butterfly;
//   chain (CHAIN=true):  the running sum visits lanes 0..P-1 in order and each
//         lane adds its products one by one → exactly the reference's sequential
//         order over all d coordinates (exact mode, P > 1).
// ---------------------------------------------------------------------------
template <int C, int P, bool CHAIN>
__device__ __forceinline__ double ocx_total(const double (&p)[C], int lane) {
    if constexpr (!CHAIN || P == 1) {
        double acc = 0.0;
#pragma unroll
        for (int j = 0; j < C; ++j) acc += p[j];
        return ocx_seq_sum<P>(acc);
    } else {
        // the running sum moves one lane up per hop (DPP wave_shr:1, lane i <- lane i-1:
        // a VALU move, no LDS round trip); the group's last lane then holds the total,
        // which one bpermute hands to all P lanes
        const int c = lane % P;
        double acc = 0.0;
        for (int cc = 0; cc < P; ++cc) {
            if (c == cc) {
#pragma unroll
                for (int j = 0; j < C; ++j) acc += p[j];
            }
            if (cc + 1 < P) acc = ocx_dpp<0x138>(acc);
        }
        return __shfl(acc, lane - c + P - 1, 64);
    }
}

// Two independent totals at once (same order as two ocx_total calls): their chains /
// butterflies interleave, so the second one rides on the first one's latency.
template <int C, int P, bool CHAIN>
__device__ __forceinline__ void ocx_total2(const double (&p)[C], const double (&q)[C], double& a,
                                           double& b, int lane) {
    if constexpr (!CHAIN || P == 1) {
        double x = 0.0, y = 0.0;
#pragma unroll
        for (int j = 0; j < C; ++j) {
            x += p[j];
            y += q[j];
        }
        a = ocx_seq_sum<P>(x);
        b = ocx_seq_sum<P>(y);
    } else {
        const int c = lane % P;
        double x = 0.0, y = 0.0;
        for (int cc = 0; cc < P; ++cc) {
            if (c == cc) {
#pragma unroll
                for (int j = 0; j < C; ++j) {
                    x += p[j];
                    y += q[j];
                }
            }
            if (cc + 1 < P) {
                x = ocx_dpp<0x138>(x);
                y = ocx_dpp<0x138>(y);
            }
        }
        a = __shfl(x, lane - c + P - 1, 64);
        b = __shfl(y, lane - c + P - 1, 64);
    }
}

__device__ __forceinline__ double ocx_grad(double diff) {  // fast_algorithms.py:27-34
    return diff > 0.0 ? 0.5 : (diff < 0.0 ? -0.5 : 0.0);
}

// FTRL action (fast_algorithms.py:52-66): x = (s*theta) * f, f = 1/||s*theta|| if > 1
template <int C, int P, bool CHAIN>
__device__ __forceinline__ void ocx_action_ftrl(const double (&th)[C], int64_t t1, double eta0,
                                                double (&x)[C], int lane) {
    const double sc = -(eta0 / sqrt((double)t1));
    double p[C];
#pragma unroll
    for (int j = 0; j < C; ++j) {
        x[j] = sc * th[j];
        p[j] = x[j] * x[j];
    }
    const double nsq = ocx_total<C, P, CHAIN>(p, lane);
    const double f = 1.0 / sqrt(nsq > 1.0 ? nsq : 1.0);  // nsq <= 1: f == 1.0 exactly
#pragma unroll
    for (int j = 0; j < C; ++j) x[j] *= f;
}

// FTL action (fast_algorithms.py:37-49): x = -(1/||theta||) * theta, or 0
template <int C, int P, bool CHAIN>
__device__ __forceinline__ void ocx_action_ftl(const double (&th)[C], double (&x)[C], int lane) {
    double p[C];
#pragma unroll
    for (int j = 0; j < C; ++j) p[j] = th[j] * th[j];
    const double nsq = ocx_total<C, P, CHAIN>(p, lane);
    const double sc = -(1.0 / sqrt(nsq));
#pragma unroll
    for (int j = 0; j < C; ++j) x[j] = (nsq == 0.0) ? 0.0 : sc * th[j];
}

template <int C, int P, bool CHAIN>
__device__ __forceinline__ double ocx_zdot(const ocx_d2* z, const double (&x)[C], int lane) {
    double p[C];
#pragma unroll
    for (int j = 0; j < C; ++j) p[j] = ocx_zj(z, j) * x[j];
    return ocx_total<C, P, CHAIN>(p, lane);
}

// FTRL action and q = z_t·x in one pass (fast_algorithms.py:52-66, :105).  ‖sθ‖² and
// z·(sθ) are summed side by side; when ‖sθ‖² <= 1 the action is sθ itself (the
// reference's rescale does not happen) and that q is the answer.  Otherwise x is
// rescaled and q summed again.  Every sum keeps the reference's order.
template <int C, int P, bool CHAIN>
__device__ __forceinline__ double ocx_ftrl_act_dot(const double (&th)[C], const ocx_d2* z,
                                                   int64_t t1, double eta0, double (&x)[C],
                                                   int lane) {
    const double sc = -(eta0 / sqrt((double)t1));
#pragma unroll
    for (int j = 0; j < C; ++j) x[j] = sc * th[j];
    // products formed where they are summed: no p[]/pq[] arrays held across the sums
    double nsq, q;
    if constexpr (!CHAIN || P == 1) {
        double a = 0.0, b = 0.0;
#pragma unroll
        for (int j = 0; j < C; ++j) {
            a += x[j] * x[j];
            b += ocx_zj(z, j) * x[j];
        }
        nsq = ocx_seq_sum<P>(a);
        q = ocx_seq_sum<P>(b);
    } else {
        const int c = lane % P;
        double a = 0.0, b = 0.0;
        for (int cc = 0; cc < P; ++cc) {
            if (c == cc) {
#pragma unroll
                for (int j = 0; j < C; ++j) {
                    a += x[j] * x[j];
                    b += ocx_zj(z, j) * x[j];
                }
            }
            if (cc + 1 < P) {
                a = ocx_dpp<0x138>(a);
                b = ocx_dpp<0x138>(b);
            }
        }
        nsq = __shfl(a, lane - c + P - 1, 64);
        q = __shfl(b, lane - c + P - 1, 64);
    }
    if (nsq > 1.0) {
        const double f = 1.0 / sqrt(nsq);
#pragma unroll
        for (int j = 0; j < C; ++j) x[j] *= f;
        q = ocx_zdot<C, P, CHAIN>(z, x, lane);
    }
    return q;
}


