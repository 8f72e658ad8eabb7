// ocx_device_math.h — per-step device arithmetic shared by the simulation kernels:
// tile loads, per-sequence totals (tree / chained), FTRL & FTL actions, z·x.
// Every function follows the reference's operation order (fast_algorithms.py:11-66).
#pragma once
#include "ocx_internal.h"

// Register-ring depth (steps in flight per wave) by coordinates per lane; tuned on
// MI355X with tools/tune.py (the -D overrides build the tuning variants).
#ifndef OCX_NB_LE8
#define OCX_NB_LE8 8
#endif
#ifndef OCX_NB_16
#define OCX_NB_16 3
#endif
#ifndef OCX_NB_GE32
#define OCX_NB_GE32 2
#endif
// steps in flight in the paired comparator pass (ocx_comp_pass2) for C <= 8 (4 above):
// the pair in use and OCX_NB_PASS2 - 2 prefetched
#ifndef OCX_NB_PASS2
#define OCX_NB_PASS2 8
#endif
#ifndef OCX_LOAD_NT
#define OCX_LOAD_NT 1
#endif
// Chained (exact) sums with at least this many lanes per sequence form the FTRL step's
// products with full-lane instructions before the chain (shorter chains form them
// inside it, saving registers), and with <= 16 coordinates per lane sum the comparator
// pass two steps at a time (ocx_comp_pass2): a long chain leaves issue slots idle.
#ifndef OCX_CHAIN_WIDE_P
#define OCX_CHAIN_WIDE_P 8
#endif

// C <= 8: 8 steps (few-wave exact batches are latency-bound: d=64, T=1e5, 8 lanes
// measured 126 -> 116 ms with 8 here and in the paired comparator pass), except where
// the ring would not stay in registers (chains of 32+ lanes, the 4-total fused kernel).
constexpr int nb_for(int C, int P = 1, bool deep = true) {
    return C <= 8 ? ((deep && P < 32) ? OCX_NB_LE8 : 4) : (C <= 16 ? OCX_NB_16 : OCX_NB_GE32);
}

// The register-ring loop of the streaming kernels: steps t in [0, T) with NB-1 steps of
// loads in flight.  load(slot, t) issues step t's loads into ring slot `slot`; step(u, t)
// consumes slot u (u is a compile-time constant once the loop is unrolled).  Every full
// block of NB steps issues its loads unconditionally — a look-ahead past the end re-reads
// step T-1, harmless — so the compiler's s_waitcnt pass sees a fixed sequence of loads and
// waits only for the slot about to be used.  (With the loads behind `if (t + NB - 1 < T)`
// it could not count them, and waited at every step for nearly every load in flight,
// including the look-ahead just issued: the ring hid no latency.)  The last block's steps
// past T are skipped; its loads are still issued (clamped), so the count stays fixed.
// Ring cycles per loop iteration (tuning knob): the compiler's wait at the loop header
//  then drains the look-ahead once per OCX_RING_UNROLL * NB steps.
#ifndef OCX_RING_UNROLL
#define OCX_RING_UNROLL 1
#endif
// LATE = true issues each block step's look-ahead load after the step instead of before it
// (NB-2 steps in flight instead of NB-1): for a step that still reads the slot the early
// load would overwrite (ocx_alg_pipe_kernel's z_{t-1}), which otherwise makes the register
// allocator rotate the ring with copies at the loop's back edge — and every copy of an
// in-flight slot is a wait for its load.
// IT: the step counter's type.  int (callers that guarantee T < 2^31, checked on the host)
// keeps the loop's bound and clamp tests on the scalar unit: the ISA has no 64-bit signed
// scalar compare, so an int64_t counter costs two VALU compares per step whose results the
// scalar unit then waits for.
// T_load (>= T_arg; default T_arg): the rows that exist for the loads — a chunk of a longer
// horizon (ocx_alg_pipe_kernel's chunked runs) looks ahead into the next chunk's rows, and
// only the horizon's last row clamps.
template <int NB, bool LATE = false, class IT = int64_t, class Load, class Step>
__device__ __forceinline__ void ocx_ring_loop(int64_t T_arg, Load&& load, Step&& step,
                                              int64_t T_load = -1) {
    static_assert(NB >= (LATE ? 3 : 2), "a ring with at least one step in flight");
    constexpr int BL = NB * OCX_RING_UNROLL;  // steps per loop iteration
    if (T_arg <= 0) return;
    const IT T = (IT)T_arg;
    const IT TL = T_load < T_arg ? T : (IT)T_load;
#pragma unroll
    for (int u = 0; u < NB - 1; ++u) {
        load(u, (int64_t)(u < TL ? (IT)u : TL - 1));
        // keep the prologue's loads in slot order: the loop header merges this order with
        // the back edge's, and a slot the scheduler loaded last here would be waited for
        // as if it were the newest load on every pass (a drain once per ring cycle)
        __builtin_amdgcn_sched_barrier(0);
    }
    for (IT t0 = 0; t0 < T; t0 += BL) {
#pragma unroll
        for (int u = 0; u < BL; ++u) {
            const IT tp = t0 + u + NB - 1;
            if (!LATE) load((u + NB - 1) % NB, (int64_t)(tp < TL ? tp : TL - 1));  // unconditional: above
            if (t0 + u < T) step(u % NB, (int64_t)(t0 + u));  // the last block may be short
            if (LATE) load((u + NB - 1) % NB, (int64_t)(tp < TL ? tp : TL - 1));
        }
    }
}

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

// Lane-local part of a tree total: the sequential sum of a lane's C products (with P = 1
// the reference's order).  In-lane pairwise sums for P > 1 measured 1.5 % on the few-wave
// T = 1e5 batch (round 2; the record is in git history): not taken.
template <int C>
__device__ __forceinline__ double ocx_lane_sum(const double (&p)[C]) {
    double acc = 0.0;
#pragma unroll
    for (int j = 0; j < C; ++j) acc += p[j];
    return acc;
}


// ---------------------------------------------------------------------------
// Per-sequence totals of C per-lane products p[j] (coordinate c*C + j).
//   tree  (CHAIN=false): lane-local sequential sum, then the P-lane butterfly;
//   chain (CHAIN=true):  the running sum visits lanes 0..P-1 in order and each
//         lane adds its products one by one → exactly the reference's sequential
//         order over all d coordinates (exact mode, P > 1).
// ---------------------------------------------------------------------------
//
// The chain is a diagonal: every hop, EVERY lane adds its C products to the value it
// holds and then takes its left neighbour's (DPP wave_shr:1, a VALU move).  Lane c's
// value is the true running sum at hop c (it received lane c-1's sum of hop c-1; lane 0
// starts from 0.0), and the group's last lane ends with the total; what the other
// lanes compute is never read.  No exec-mask changes: the chain is one basic block the
// scheduler interleaves with independent work, with no DPP-after-exec wait states.
// Long chains (P >= OCX_CHAIN_WIDE_P) use it, with the DPP/readlane broadcast and the
// comparator's totals left in the last lane; short chains (the bench's P = 4) keep the
// exec-masked hop and a bpermute, measured 2-9 % faster there.

// hops unrolled per loop iteration (full unroll up to 128 adds per chain)
constexpr int ocx_chain_unroll(int P, int C) { return P * C <= 128 ? P : (C >= 32 ? 1 : 2); }

// The group's last lane (c = P-1) holds a chained total: hand it to all P lanes.  DPP
// within a row for P <= 16 (quad_perm / row_half_mirror / row_mirror), readlane for
// P >= 32 (one or two sequences per wave).
template <int P>
__device__ __forceinline__ double ocx_bcast_last(double v, int lane) {
    if constexpr (P == 1) {
        return v;
    } else if constexpr (P == 2) {
        return ocx_dpp_all<0xF5>(v);  // quad_perm [1,1,3,3]
    } else if constexpr (P == 4) {
        return ocx_dpp_all<0xFF>(v);  // quad_perm [3,3,3,3]
    } else if constexpr (P == 8) {
        const double s1 = ocx_dpp_all<0xFF>(v);    // lanes 4-7 of the half-row: lane 7's value
        const double s2 = ocx_dpp_all<0x141>(s1);  // half-row mirror: lanes 0-3 <- lanes 7-4
        return (lane & 4) ? s1 : s2;
    } else if constexpr (P == 16) {
        const int r = lane & 15;
        const double s1 = ocx_dpp_all<0xFF>(v);    // lanes 12-15: lane 15's value
        const double s2 = ocx_dpp_all<0x140>(s1);  // row mirror: lanes 0-3 <- lanes 15-12
        const double m = r >= 12 ? s1 : s2;        // right in lanes 0-3 and 12-15
        const double s3 = ocx_dpp_all<0x141>(m);   // half mirrors: 4-7 <- 3-0, 8-11 <- 15-12
        return (r < 4 || r >= 12) ? m : s3;
    } else if constexpr (P == 32) {
        const double lo = ocx_readlane(v, 31), hi = ocx_readlane(v, 63);
        return lane < 32 ? lo : hi;
    } else {
        return ocx_readlane(v, 63);
    }
}

// Chained total of p over the group, valid in the group's LAST lane only.
template <int C, int P>
__device__ __forceinline__ double ocx_chain_last(const double (&p)[C]) {
    double acc = 0.0;
#pragma unroll ocx_chain_unroll(P, C)
    for (int cc = 0; cc + 1 < P; ++cc) {
#pragma unroll
        for (int j = 0; j < C; ++j) acc += p[j];
        acc = ocx_dpp<0x138>(acc);
    }
#pragma unroll
    for (int j = 0; j < C; ++j) acc += p[j];
    return acc;
}

// Two chained totals side by side, valid in the group's last lane only.
template <int C, int P>
__device__ __forceinline__ void ocx_chain2_last(const double (&p)[C], const double (&q)[C],
                                                double& a, double& b) {
    double x = 0.0, y = 0.0;
#pragma unroll ocx_chain_unroll(P, C)
    for (int cc = 0; cc + 1 < P; ++cc) {
#pragma unroll
        for (int j = 0; j < C; ++j) {
            x += p[j];
            y += q[j];
        }
        x = ocx_dpp<0x138>(x);
        y = ocx_dpp<0x138>(y);
    }
#pragma unroll
    for (int j = 0; j < C; ++j) {
        x += p[j];
        y += q[j];
    }
    a = x;
    b = y;
}

template <int C, int P, bool CHAIN>
__device__ __forceinline__ double ocx_total(const double (&p)[C], int lane) {
    if constexpr (!CHAIN || P == 1) {
        return ocx_seq_sum<P>(ocx_lane_sum<C>(p));
    } else if constexpr (P < OCX_CHAIN_WIDE_P) {
        // short chain: the hop's lane adds (exec-masked), one bpermute hands the total out
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
    } else {
        return ocx_bcast_last<P>(ocx_chain_last<C, P>(p), lane);
    }
}

// The total where the comparator pass needs it: the group's last lane (chain) or
// every lane (tree).  A running sum of such values is read with ocx_comp_lane_value.
template <int C, int P, bool CHAIN>
__device__ __forceinline__ double ocx_total_last(const double (&p)[C], int lane) {
    if constexpr (!CHAIN || P < OCX_CHAIN_WIDE_P) {
        return ocx_total<C, P, CHAIN>(p, lane);
    } else {
        return ocx_chain_last<C, P>(p);
    }
}

template <int P, bool CHAIN>
__device__ __forceinline__ double ocx_comp_lane_value(double comp, int lane) {
    if constexpr (!CHAIN || P < OCX_CHAIN_WIDE_P) {
        return comp;
    } else {
        return ocx_bcast_last<P>(comp, lane);
    }
}

// Two independent totals at once (same order as two ocx_total calls): their chains /
// butterflies interleave, so the second one rides on the first one's latency.
template <int C, int P, bool CHAIN>
__device__ __forceinline__ void ocx_total2(const double (&p)[C], const double (&q)[C], double& a,
                                           double& b, int lane) {
    if constexpr (!CHAIN || P == 1) {
        a = ocx_seq_sum<P>(ocx_lane_sum<C>(p));
        b = ocx_seq_sum<P>(ocx_lane_sum<C>(q));
    } else if constexpr (P < OCX_CHAIN_WIDE_P) {
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
    } else {
        ocx_chain2_last<C, P>(p, q, a, b);
        a = ocx_bcast_last<P>(a, lane);
        b = ocx_bcast_last<P>(b, lane);
    }
}

// ocx_total2 with the totals where ocx_total_last leaves them.
template <int C, int P, bool CHAIN>
__device__ __forceinline__ void ocx_total2_last(const double (&p)[C], const double (&q)[C],
                                                double& a, double& b, int lane) {
    if constexpr (!CHAIN || P < OCX_CHAIN_WIDE_P) {
        ocx_total2<C, P, CHAIN>(p, q, a, b, lane);
    } else {
        ocx_chain2_last<C, P>(p, q, a, b);
    }
}

// The one-pass comparator's `onepass` argument: 0 the streamed second pass; 1 the closed form
// where certified, every row checked to lie in the ball; 2 the same for rows clipped by
// construction (the engine's own g(T) sampler: z_t = x_t / max(1, ||x_t||), NumPy's rows bit for
// bit), whose per-row check is skipped (OCX_CLIPPED_SKIP=0 keeps it: tuning A/B).
#ifndef OCX_CLIPPED_SKIP
#define OCX_CLIPPED_SKIP 1
#endif
__host__ __device__ __forceinline__ bool ocx_check_rows(int onepass) {
    return onepass == 1 || (onepass == 2 && !OCX_CLIPPED_SKIP);
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

// ---------------------------------------------------------------------------
// Exact FTL over the l1 and linf unit balls (exact_ftl.py:83-105 norm='l1' / 'linf') in
// the closed form of their linear regime (see ocx_sim.hip, algo 2): with theta = −S_t
// the prefix minimiser maximises x·S_t over the ball:
//   l1   x = sign(S_j*) e_j*, j* = the first coordinate of largest |S_j| (0 if S = 0);
//   linf x_j = sign(S_j) (0 where S_j = 0).
// Ties (several j*, or S_j = 0 under linf) leave the SOCP/LP solution non-unique; the
// engine's choice is the one above.  norm codes: 0 l2, 1 l1, 2 linf.
// ---------------------------------------------------------------------------
template <int C, int P>
__device__ __forceinline__ void ocx_action_exact_poly(const double (&th)[C], double (&x)[C],
                                                      int norm, int lane) {
    if (norm == 2) {
#pragma unroll
        for (int j = 0; j < C; ++j) x[j] = th[j] > 0.0 ? -1.0 : (th[j] < 0.0 ? 1.0 : 0.0);
        return;
    }
    const int c = lane % P;
    double best = -1.0;
    int bj = 0;
#pragma unroll
    for (int j = 0; j < C; ++j) {
        const double v = fabs(th[j]);
        if (v > best) {  // strict: the first of equal values
            best = v;
            bj = c * C + j;
        }
    }
#pragma unroll
    for (int m = 1; m < P; m <<= 1) {  // (value, index) max over the P lanes, lowest index
        const double ob = __shfl_xor(best, m, 64);
        const int oj = __shfl_xor(bj, m, 64);
        if (ob > best || (ob == best && oj < bj)) {
            best = ob;
            bj = oj;
        }
    }
#pragma unroll
    for (int j = 0; j < C; ++j)
        x[j] = (best > 0.0 && c * C + j == bj) ? (th[j] > 0.0 ? -1.0 : 1.0) : 0.0;
}

// Prefixes where the closed form's maximiser of x·S_t is not unique AND the general solver's
// answer — the central path's limit, the analytic centre of the optimal face
// (ocx_exact_ball.hip), what interior-point cvxpy backends approach — is not the closed
// form's point:
//   l1    two or more coordinates attain max_j |S_j| > 0 (the face is their simplex; the
//         rows' slack terms place its centre);
//   linf  S_j = 0 in a coordinate some row of the prefix has touched (`touch`, bit j: the
//         face is free there, and the rows pull its centre off 0).
// S_t = 0 is not such a case: the centre is then x = 0 (the rows' barrier has gradient −S_t
// = 0 there), which is the closed forms' answer.  Callers leave the regime on a tie, so the
// general solver answers those sequences.  Whole wave active (lane exchanges).
template <int C, int P>
__device__ __forceinline__ bool ocx_exact_poly_tie(const double (&th)[C], uint64_t touch, int norm) {
    if (norm == 1) {
        double best = 0.0;
#pragma unroll
        for (int j = 0; j < C; ++j) best = fmax(best, fabs(th[j]));
#pragma unroll
        for (int m = 1; m < P; m <<= 1) best = fmax(best, __shfl_xor(best, m, 64));
        double cnt = 0.0;
#pragma unroll
        for (int j = 0; j < C; ++j) cnt += (best > 0.0 && fabs(th[j]) == best) ? 1.0 : 0.0;
        return ocx_seq_sum<P>(cnt) >= 2.0;
    }
    if (norm == 2) {
        double f = 0.0;
#pragma unroll
        for (int j = 0; j < C; ++j) f += (th[j] == 0.0 && ((touch >> j) & 1ull)) ? 1.0 : 0.0;
        return ocx_seq_sum<P>(f) > 0.0;
    }
    return false;
}
template <int C>
__device__ __forceinline__ uint64_t ocx_touch(uint64_t touch, const ocx_d2* z) {
#pragma unroll
    for (int j = 0; j < C; ++j) touch |= (ocx_zj(z, j) != 0.0 ? 1ull : 0ull) << j;
    return touch;
}

// Is row z inside the regime of the `norm` ball's closed form: its dual norm <= 1
// (l2: ||z||_2^2 <= 1 + 1e-6, the bar of round 1; l1 ball: max_j |z_j| <= 1 + 1e-12;
// linf ball: sum_j |z_j| <= 1 + 1e-12)?  Every lane of the sequence gets the answer.
template <int C, int P, bool CHAIN>
__device__ __forceinline__ bool ocx_dual_ok(const ocx_d2* z, int norm, int lane);

// Certification test of the closed-form comparators (ocx_alg_kernel onepass,
// ocx_alg_chunk_kernel): is ||z_t||_2^2 <= 1 + 1e-12 for this row?  Not part of the
// reference's arithmetic, so any summation order does (fused lane sums, butterfly); the
// 1e-12 slack admits rows clipped in floating point (np.linalg.norm ∘ z / max(n, 1)
// leaves ||z_t|| within a few ulps of 1).  Every lane of the sequence gets the answer; call
// it with the whole wave active (the butterfly reads neighbouring lanes).
template <int C, int P>
__device__ __forceinline__ bool ocx_row_in_ball(const ocx_d2* z) {
    double acc = 0.0;
#pragma unroll
    for (int j = 0; j < C; ++j) acc = __builtin_fma(ocx_zj(z, j), ocx_zj(z, j), acc);
    return ocx_seq_sum<P>(acc) <= 1.0 + 1e-12;
}

template <int C, int P, bool CHAIN>
__device__ __forceinline__ double ocx_zdot(const ocx_d2* z, const double (&x)[C], int lane) {
    double p[C];
#pragma unroll
    for (int j = 0; j < C; ++j) p[j] = ocx_zj(z, j) * x[j];
    return ocx_total<C, P, CHAIN>(p, lane);
}

// FTRL scales s_t = −(η0/√t) of 64 consecutive steps, one per lane, refreshed every 64
// steps (fast_algorithms.py:58): the sqrt/div sequence costs one lane-parallel pass per 64
// steps instead of one per step, and step t reads its value with a readlane.  The same
// expression per t as the per-step form, so bit for bit the same scale.
struct OcxScaleTable {
    double v = 0.0;
    int64_t base = INT64_MIN / 2;  // 1-based step of lane 0's entry (none yet)
};
__device__ __forceinline__ double ocx_ftrl_scale(OcxScaleTable& tb, int64_t t1, double eta0,
                                                 int lane) {
    if (t1 - tb.base >= 64 || t1 < tb.base) {
        tb.base = t1;
        tb.v = -(eta0 / sqrt((double)(t1 + lane)));
    }
    return ocx_readlane(tb.v, (int)(t1 - tb.base));
}

// FTRL action and q = z_t·x in one pass (fast_algorithms.py:52-66, :105).  ‖sθ‖² and
// z·(sθ) are summed side by side; when ‖sθ‖² <= 1 the action is sθ itself (the
// reference's rescale does not happen) and that q is the answer.  Otherwise x is
// rescaled and q summed again.  Every sum keeps the reference's order.
//
// Long chains (ocx_ftrl_q_sc): `sc` = −(η0/√t) comes from the caller, computed a step
// ahead (off the chain's critical path); products by every lane at once, then the
// diagonal chain.  Returns q and the rescale factor f (1.0 when none): the action is
// x_j = (sc·θ_j)·f, bit for bit what the reference holds, formed only where needed.
template <int C, int P, bool CHAIN>
__device__ __forceinline__ double ocx_ftrl_q_sc(const double (&th)[C], const ocx_d2* z, double sc,
                                                double& f, int lane) {
    static_assert(CHAIN && P >= OCX_CHAIN_WIDE_P, "long chains only");
    double pa[C], pb[C];
#pragma unroll
    for (int j = 0; j < C; ++j) {
        const double xj = sc * th[j];
        pa[j] = xj * xj;
        pb[j] = ocx_zj(z, j) * xj;
    }
    double nsq, q;
    ocx_chain2_last<C, P>(pa, pb, nsq, q);
    nsq = ocx_bcast_last<P>(nsq, lane);
    q = ocx_bcast_last<P>(q, lane);
    f = 1.0;
    if (nsq > 1.0) {
        f = 1.0 / sqrt(nsq);
        double x[C];
#pragma unroll
        for (int j = 0; j < C; ++j) x[j] = (sc * th[j]) * f;
        q = ocx_zdot<C, P, CHAIN>(z, x, lane);
    }
    return q;
}

// `sc` = −(η0/√t) (ocx_ftrl_scale: one sqrt/div per 64 steps instead of one per step)
template <int C, int P, bool CHAIN>
__device__ __forceinline__ double ocx_ftrl_act_dot_sc(const double (&th)[C], const ocx_d2* z,
                                                      double sc, double (&x)[C], int lane) {
    if constexpr (CHAIN && P >= OCX_CHAIN_WIDE_P) {
        double f;
        const double q = ocx_ftrl_q_sc<C, P, CHAIN>(th, z, sc, f, lane);
#pragma unroll
        for (int j = 0; j < C; ++j) x[j] = (sc * th[j]) * f;
        return q;
    }
#pragma unroll
    for (int j = 0; j < C; ++j) x[j] = sc * th[j];
    // products formed where they are summed: no p[]/pq[] arrays held across the sums
    double nsq, q;
    if constexpr (!CHAIN || P == 1) {
        double pa[C], pb[C];
#pragma unroll
        for (int j = 0; j < C; ++j) {
            pa[j] = x[j] * x[j];
            pb[j] = ocx_zj(z, j) * x[j];
        }
        nsq = ocx_seq_sum<P>(ocx_lane_sum<C>(pa));
        q = ocx_seq_sum<P>(ocx_lane_sum<C>(pb));
    } else {
        // short chain: the hop's lane adds (exec-masked), one bpermute hands the totals out
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

template <int C, int P, bool CHAIN>
__device__ __forceinline__ double ocx_ftrl_act_dot(const double (&th)[C], const ocx_d2* z,
                                                   int64_t t1, double eta0, double (&x)[C],
                                                   int lane) {
    return ocx_ftrl_act_dot_sc<C, P, CHAIN>(th, z, -(eta0 / sqrt((double)t1)), x, lane);
}

// Comparator loss Σ_t ½|z_t·xs − y_t| over steps [0, T) of one tile region, added to
// `comp` in step order (fast_algorithms.py:69-76).  The steps' dot products are
// independent, so two are summed side by side (ocx_total2): in a long lane chain the
// second chain fills the issue slots the first one leaves idle.  NBC steps in flight:
// the pair in use and NBC-2 prefetched.
template <int C, int P, bool CHAIN, int NBC>
__device__ __forceinline__ double ocx_comp_pass2(const ocx_d2* __restrict__ zp,
                                                 const double* __restrict__ yp, int64_t T,
                                                 int64_t kst, int S, const double (&xs)[C],
                                                 double comp, int lane) {
    static_assert(NBC >= 4 && NBC % 2 == 0, "a pair in use and at least a pair in flight");
    constexpr int K = C / 2;
    constexpr int64_t tstride = 64;  // ocx_d2 per step within a plane
    ocx_d2 zb[NBC][K];
    double yb[NBC];
#pragma unroll
    for (int u = 0; u < NBC - 2; ++u)
        if (u < T) {
            ocx_load_tile<C>(zb[u], zp + u * tstride, kst);
            yb[u] = yp[u * S];
        }
    for (int64_t t0 = 0; t0 < T; t0 += NBC) {
#pragma unroll
        for (int u = 0; u < NBC; u += 2) {
            const int64_t t = t0 + u;
            if (t < T) {
#pragma unroll
                for (int v = 0; v < 2; ++v) {
                    const int64_t tp = t + NBC - 2 + v;
                    if (tp < T) {
                        ocx_load_tile<C>(zb[(u + NBC - 2 + v) % NBC], zp + tp * tstride, kst);
                        yb[(u + NBC - 2 + v) % NBC] = yp[tp * S];
                    }
                }
                const bool two = t + 1 < T;
                double p0[C], p1[C];
#pragma unroll
                for (int j = 0; j < C; ++j) {
                    p0[j] = ocx_zj(zb[u], j) * xs[j];
                    p1[j] = two ? ocx_zj(zb[u + 1], j) * xs[j] : 0.0;
                }
                double q0, q1;
                ocx_total2_last<C, P, CHAIN>(p0, p1, q0, q1, lane);
                comp += 0.5 * fabs(q0 - yb[u]);
                if (two) comp += 0.5 * fabs(q1 - yb[u + 1]);
            }
        }
    }
    return ocx_comp_lane_value<P, CHAIN>(comp, lane);
}



template <int C, int P, bool CHAIN>
__device__ __forceinline__ bool ocx_dual_ok(const ocx_d2* z, int norm, int lane) {
    double p[C];
    if (norm == 1) {
        double m = 0.0;
#pragma unroll
        for (int j = 0; j < C; ++j) m = fmax(m, fabs(ocx_zj(z, j)));
#pragma unroll
        for (int k = 1; k < P; k <<= 1) m = fmax(m, __shfl_xor(m, k, 64));
        return m <= 1.0 + 1e-12;
    }
#pragma unroll
    for (int j = 0; j < C; ++j) p[j] = norm == 0 ? ocx_zj(z, j) * ocx_zj(z, j) : fabs(ocx_zj(z, j));
    const double t = ocx_total<C, P, CHAIN>(p, lane);
    return norm == 0 ? t <= 1.0 + 1e-6 : t <= 1.0 + 1e-12;
}
