// ocx_sim.hip — gfx950 kernels for the per-timestep FTRL/FTL/SMART loops.
//
// One wavefront owns S = 64/P independent sequences; the P lanes of a sequence
// hold C coordinates each of theta (registers), so the sequential T-step
// recurrence runs entirely on chip and HBM sees only the streamed z_t / y_t tiles
// (layout: include/ocx.h, ocx_layout).  Each step a wave loads one 512*C-byte tile
// with C/2 coalesced 1 KiB dwordx4 loads, issued NB-1 steps ahead through a
// register ring so the HBM latency hides behind the on-chip arithmetic.
//
// Arithmetic follows the reference's operation order per lane (sequential sums
// from 0.0, IEEE sqrt/div, no contraction: built with -ffp-contract=off); with
// P = 1 every sum is the reference's sequential sum and results are bit-identical
// to fast_algorithms.py; with P > 1 the per-lane partial sums are combined by a
// butterfly (ocx_seq_sum).
#include <algorithm>

#include <cstdlib>
#include <cstring>

#include "ocx_device_math.h"
#include "ocx_dispatch.h"
#include "ocx_internal.h"
#include "ocx_sim_kernels.h"

// ---------------------------------------------------------------------------
// fast_algorithms.py:88-115 `_simulate_alg_core` (+ exact_ftl.py:230-277 outputs)
//   algo 0 FTRL, 1 FTL (the reference's alg_flag 0 / non-zero);
//   algo 2 exact FTL over the unit ball of `norm` (0 l2, 1 l1, 2 linf; exact_ftl.py:83-105,
//          :280-333 compute_prefix_actions + replay) in its linear regime: when every row's
//          dual norm is <= 1 and y_t = ±1, |z_i·x| <= 1 on the ball and
//          ½Σ|z_i·x − y_i| = ½(t − x·S_t), so the prefix minimiser maximises x·S_t,
//          S_t = Σ_{i<t} y_i z_i: S_t/||S_t|| for l2 (0 if S_t = 0; the FTL action of
//          theta = −S_t), ocx_action_exact_poly for l1 / linf.  regime_out[b] reports
//          whether the data were in that regime (ocx_dual_ok and |y_t| == 1); the caller
//          rejects otherwise.
// cmp_out [B][d] (nullable) receives the comparator action of the second pass.
// ---------------------------------------------------------------------------
// Waves per SIMD the register allocation of the FTRL kernel must allow (tuning knob:
// -DOCX_ALG_MIN_WAVES=2 asks for 2 waves/SIMD when C <= 16).
#ifndef OCX_ALG_MIN_WAVES
#define OCX_ALG_MIN_WAVES 1
#endif
// MINW > 0: the register budget of MINW waves per SIMD (the small-d pipeline's FTRL side asks for
// 4: <= 128 VGPRs, one wave beside four 96-VGPR generator waves)
template <int C, int P, bool CHAIN, int NB, int MINW = 0>
__global__ __launch_bounds__(OCX_BLOCK, (MINW > 0 ? MINW : (C <= 16 ? OCX_ALG_MIN_WAVES : 1))) void ocx_alg_kernel(
    const double* __restrict__ zt, const double* __restrict__ yt, int64_t B, int64_t T,
    int64_t d, int64_t G, int algo, double eta0, const double* __restrict__ comparator,
    double* __restrict__ regret, double* __restrict__ cum_out, double* __restrict__ comp_out,
    double* __restrict__ x_last, double* __restrict__ cmp_out, int* __restrict__ regime_out,
    int onepass, int norm, int64_t g0, int64_t gn, unsigned long long* __restrict__ gmax) {
    constexpr int S = 64 / P;
    constexpr int K = C / 2;
    const int lane = threadIdx.x & 63;
    // wave-groups [g0, g0 + gn) of the layout (a sub-batch of the overlapped pipeline; the
    // whole layout otherwise), G the layout's groups (the plane stride)
    const int64_t wv = ocx_wave_id();
    if (wv >= gn) return;
    const int64_t g = g0 + wv;
#ifdef OCX_ALG_PRIO  // tuning: issue priority over waves of a kernel running beside it
    __builtin_amdgcn_s_setprio(OCX_ALG_PRIO);
#endif
    const int s = lane / P;
    const int c = lane % P;
    const int64_t b = g * S + s;
    const int64_t tstride = 64;  // ocx_d2 per step within a plane
    const ocx_d2* __restrict__ zp = reinterpret_cast<const ocx_d2*>(zt) + g * T * tstride + lane;
    const int64_t kst = G * T * 64;  // plane stride (pairs k)
    const double* __restrict__ yp = yt + g * T * S + s;
    const bool ftl = (algo != 0);
    const bool exact = (algo == 2);
    bool linear = true;  // algo 2: data inside the closed form's regime so far
    uint64_t touch = 0;  // algo 2, linf: coordinates some row has touched (ocx_exact_poly_tie)
    bool clean = true;   // onepass: every sub-gradient so far was −y_t/2 (see below)

    double th[C];
#pragma unroll
    for (int j = 0; j < C; ++j) th[j] = 0.0;

    ocx_d2 zb[NB][K];
    double yb[NB];
    auto load = [&](int slot, int64_t tl) {
        ocx_load_tile<C>(zb[slot], zp + tl * tstride, kst);
        yb[slot] = yp[tl * S];
    };

    double cum = 0.0;
    OcxScaleTable sct;  // FTRL scales, 64 steps at a time (long chains)
    ocx_ring_loop<NB>(T, load, [&](int u, int64_t t) {
                double x[C];
                double q;  // :105
                if (!ftl) {
                    if constexpr (CHAIN && P >= OCX_CHAIN_WIDE_P) {
                        const double sc = ocx_ftrl_scale(sct, t + 1, eta0, lane);
                        double fr;
                        q = ocx_ftrl_q_sc<C, P, CHAIN>(th, zb[u], sc, fr, lane);
#pragma unroll
                        for (int j = 0; j < C; ++j) x[j] = (sc * th[j]) * fr;
                    } else {
#ifdef OCX_ALG_STEP_SCALE  // tuning A/B: the scale's sqrt/div every step
                        q = ocx_ftrl_act_dot<C, P, CHAIN>(th, zb[u], t + 1, eta0, x, lane);
#else
                        const double sc = ocx_ftrl_scale(sct, t + 1, eta0, lane);
                        q = ocx_ftrl_act_dot_sc<C, P, CHAIN>(th, zb[u], sc, x, lane);
#endif
                    }
                } else {
                    if (exact && norm != 0) {
                        ocx_action_exact_poly<C, P>(th, x, norm, lane);
                        linear = linear && !ocx_exact_poly_tie<C, P>(th, touch, norm);
                    } else {
                        ocx_action_ftl<C, P, CHAIN>(th, x, lane);
                    }
                    q = ocx_zdot<C, P, CHAIN>(zb[u], x, lane);
                }
                if (x_last != nullptr && t == T - 1 && b < B) {
#pragma unroll
                    for (int j = 0; j < C; ++j) {
                        const int64_t jj = (int64_t)c * C + j;
                        if (jj < d) x_last[b * d + jj] = x[j];
                    }
                }
                const double diff = q - yb[u];  // :106-111
                cum += 0.5 * fabs(diff);
                double gq = ocx_grad(diff);
                // the closed form needs ||z_t|| <= 1 too: certified here, row by row,
                // whatever the caller asserts (whole wave active: the test sums across lanes)
                if (ocx_check_rows(onepass)) clean = clean & ocx_row_in_ball<C, P>(zb[u]);
                clean = clean && fabs(yb[u]) == 1.0 && gq == -0.5 * yb[u];
                if (exact) {  // theta = −S_t: accumulate −y_t z_t; check the regime
                    linear = linear && ocx_dual_ok<C, P, CHAIN>(zb[u], norm, lane) &&
                             fabs(yb[u]) == 1.0;
                    if (norm == 2) touch = ocx_touch<C>(touch, zb[u]);
                    gq = -yb[u];
                }
#pragma unroll
                for (int j = 0; j < C; ++j) th[j] += gq * ocx_zj(zb[u], j);  // gq*z is exact
    });

    // ---- closed-form comparator (onepass) ----
    // For rows with ||z_t|| <= 1 (the g(T) sampler's clipped rows; certified per row in
    // the loop above, ocx_row_in_ball) and x* = FTL(theta_T) in the unit ball, |z_t.x* − y_t| = 1 − y_t z_t.x* when y_t = ±1,
    // so the comparator loss is ½(T − x*.S_T), S_T = Σ y_t z_t.  If every step's
    // sub-gradient was −y_t/2 (no tie, y_t = ±1: `clean`), theta_T = −½ S_T exactly
    // (powers of two), x* = −theta/||theta|| and the loss is T/2 − ||theta_T||: no second
    // pass over z.  It equals the reference's sequential sum up to rounding (≈1e-13
    // relative on the regret, tests/test_gpu_parity.py).  A wave with an unclean
    // sequence streams the second pass for it; every clean sequence keeps the closed
    // form, so a sequence's result never depends on the wave it shares.
    const bool closed = onepass && comparator == nullptr && !exact && (clean || b >= B);
    const bool pass2 = __ballot(!closed) != 0;  // wave-uniform

    // ---- comparator action (fast_algorithms.py:113 FTL of theta, or the caller's) ----
    double xs[C];
    if (!pass2 && cmp_out == nullptr) {
#pragma unroll
        for (int j = 0; j < C; ++j) xs[j] = 0.0;
    } else if (comparator != nullptr) {
#pragma unroll
        for (int j = 0; j < C; ++j) {
            const int64_t jj = (int64_t)c * C + j;
            xs[j] = (b < B && jj < d) ? comparator[b * d + jj] : 0.0;
        }
    } else if (exact && norm != 0) {
        ocx_action_exact_poly<C, P>(th, xs, norm, lane);
        linear = linear && !ocx_exact_poly_tie<C, P>(th, touch, norm);
    } else {
        ocx_action_ftl<C, P, CHAIN>(th, xs, lane);
    }
    if (cmp_out != nullptr && b < B) {
#pragma unroll
        for (int j = 0; j < C; ++j) {
            const int64_t jj = (int64_t)c * C + j;
            if (jj < d) cmp_out[b * d + jj] = xs[j];
        }
    }

    // ---- second streaming pass: comparator loss (fast_algorithms.py:69-76) ----
    double comp = 0.0;
#ifdef OCX_TUNE_SKIP_COMP  // tuning only: time the FTRL pass alone (regrets are wrong)
    if (true) {
    } else
#endif
    if (!pass2) {
    } else if constexpr (CHAIN && P >= OCX_CHAIN_WIDE_P && P <= 16 && C <= 16) {
        comp = ocx_comp_pass2<C, P, CHAIN, (C <= 8 ? OCX_NB_PASS2 : 4)>(zp, yp, T, kst, S, xs, 0.0, lane);
    } else {
        ocx_ring_loop<NB>(T, load, [&](int u, int64_t) {
            double p[C];
#pragma unroll
            for (int j = 0; j < C; ++j) p[j] = ocx_zj(zb[u], j) * xs[j];
            const double q = ocx_total_last<C, P, CHAIN>(p, lane);
            comp += 0.5 * fabs(q - yb[u]);
        });
        comp = ocx_comp_lane_value<P, CHAIN>(comp, lane);
    }
    if (__ballot(closed) != 0) {  // wave-uniform: the sum below crosses lanes
        double p[C];
#pragma unroll
        for (int j = 0; j < C; ++j) p[j] = th[j] * th[j];
        const double nrm = sqrt(ocx_total<C, P, CHAIN>(p, lane));
        if (closed) comp = 0.5 * (double)T - nrm;
    }

    // g(T) folded in (the small-d pipeline's FTRL launches; ocx_alg_pipe.hip does the same): a
    // max over the wave's sequences, one 64-bit atomic max of the bit pattern per wave —
    // positive doubles order as their bits and a NaN never passes `>`, so this selects what
    // ocx_max_fold_kernel and the host's loop select
    if (gmax != nullptr && __ballot(b < B) != 0) {  // wave-uniform
        const double rg = cum - comp;
        double mv = (c == 0 && b < B && rg > 0.0) ? rg : 0.0;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            const double u = __shfl_xor(mv, o, 64);
            if (u > mv) mv = u;
        }
        if (lane == 0 && mv > 0.0) atomicMax(gmax, (unsigned long long)__double_as_longlong(mv));
    }
    if (c == 0 && b < B) {
        if (regret) regret[b] = cum - comp;
        if (cum_out) cum_out[b] = cum;
        if (comp_out) comp_out[b] = comp;
        // algo 2: the exact closed form's regime; algo 0/1: whether the closed-form
        // comparator was taken (onepass)
        if (regime_out) regime_out[b] = (exact ? linear : closed) ? 1 : 0;
    }
}

// ---------------------------------------------------------------------------
// fast_algorithms.py:118-164 `_simulate_SMART_like_core`
// ---------------------------------------------------------------------------
template <int C, int P, bool CHAIN>
__global__ __launch_bounds__(OCX_BLOCK) void ocx_smart_kernel(
    const double* __restrict__ zt, const double* __restrict__ yt, int64_t B, int64_t T,
    int64_t G, const double* __restrict__ thresh, double eta0, double* __restrict__ regret,
    int64_t* __restrict__ switch_step) {
    constexpr int S = 64 / P;
    constexpr int K = C / 2;
    const int lane = threadIdx.x & 63;
    const int64_t g = ocx_wave_id();
    if (g >= G) return;
    const int s = lane / P;
    const int c = lane % P;
    const int64_t b = g * S + s;
    const int64_t tstride = 64;  // ocx_d2 per step within a plane
    const ocx_d2* __restrict__ zp = reinterpret_cast<const ocx_d2*>(zt) + g * T * tstride + lane;
    const int64_t kst = G * T * 64;  // plane stride (pairs k)
    const double* __restrict__ yp = yt + g * T * S + s;
    const double th_sw = (b < B) ? thresh[b] : 0.0;

    double tf[C], tr[C];
#pragma unroll
    for (int j = 0; j < C; ++j) tf[j] = tr[j] = 0.0;
    bool switched = (b >= B);  // padding sequences never scan
    int64_t sw = -1;
    double ftl_loss = 0.0, total_loss = 0.0;

    for (int64_t t = 0; t < T; ++t) {
        ocx_d2 z[K];
        ocx_load_tile<C>(z, zp + t * tstride, kst);
        const double yv = yp[t * S];
        // FTL is always run and updated (:140-146)
        double x[C];
        ocx_action_ftl<C, P, CHAIN>(tf, x, lane);
        const double pf = ocx_zdot<C, P, CHAIN>(z, x, lane);
        const double dfl = pf - yv;
        const double gfl = ocx_grad(dfl);
#pragma unroll
        for (int j = 0; j < C; ++j) tf[j] += gfl * ocx_zj(z, j);
        const double loss_ftl = 0.5 * fabs(dfl);
        ftl_loss += loss_ftl;
        if (switched) {
            // post-switch: FTRL with its own theta and the global t (:148-154)
            ocx_action_ftrl<C, P, CHAIN>(tr, t + 1, eta0, x, lane);
            const double pr = ocx_zdot<C, P, CHAIN>(z, x, lane);
            const double dr = pr - yv;
            total_loss += 0.5 * fabs(dr);
            const double gr = ocx_grad(dr);
#pragma unroll
            for (int j = 0; j < C; ++j) tr[j] += gr * ocx_zj(z, j);
        } else {
            total_loss += loss_ftl;  // :156
            // s_t = FTL(theta_ftl) after the update; loss of s_t over rows 0..t (:157-160)
            double sv[C];
            ocx_action_ftl<C, P, CHAIN>(tf, sv, lane);
            double s_loss = 0.0;
            for (int64_t i = 0; i <= t; ++i) {
                ocx_d2 zi[K];
                ocx_load_tile<C>(zi, zp + i * tstride, kst);
                const double q = ocx_zdot<C, P, CHAIN>(zi, sv, lane);
                s_loss += 0.5 * fabs(q - yp[i * S]);
            }
            if (ftl_loss - s_loss >= th_sw) {
                switched = true;
                sw = t;
            }
        }
    }
    // final comparator = FTL(theta_ftl) (:162-163)
    double sv[C];
    ocx_action_ftl<C, P, CHAIN>(tf, sv, lane);
    double comp = 0.0;
    for (int64_t t = 0; t < T; ++t) {
        ocx_d2 z[K];
        ocx_load_tile<C>(z, zp + t * tstride, kst);
        const double q = ocx_zdot<C, P, CHAIN>(z, sv, lane);
        comp += 0.5 * fabs(q - yp[t * S]);
    }
    if (c == 0 && b < B) {
        regret[b] = total_loss - comp;
        if (switch_step) switch_step[b] = sw;
    }
}

// ---------------------------------------------------------------------------
// exact_ftl.py:306-333 `replay_exact_ftl`: loss of given actions a_t, comparator a_T
// ---------------------------------------------------------------------------
template <int C, int P, bool CHAIN>
__global__ __launch_bounds__(OCX_BLOCK) void ocx_replay_kernel(
    const double* __restrict__ zt, const double* __restrict__ yt, const double* __restrict__ at,
    int64_t B, int64_t T, int64_t G, double* __restrict__ cum_out, double* __restrict__ comp_out) {
    constexpr int S = 64 / P;
    constexpr int K = C / 2;
    const int lane = threadIdx.x & 63;
    const int64_t g = ocx_wave_id();
    if (g >= G) return;
    const int s = lane / P;
    const int c = lane % P;
    const int64_t b = g * S + s;
    const int64_t tstride = 64;  // ocx_d2 per step within a plane
    const ocx_d2* __restrict__ zp = reinterpret_cast<const ocx_d2*>(zt) + g * T * tstride + lane;
    const int64_t kst = G * T * 64;  // plane stride (pairs k)
    const ocx_d2* __restrict__ ap =
        reinterpret_cast<const ocx_d2*>(at) + g * (T + 1) * tstride + lane;
    const int64_t kst_a = G * (T + 1) * 64;
    const double* __restrict__ yp = yt + g * T * S + s;
    double aT[C];
    {
        ocx_d2 a2[K];
        ocx_load_tile<C>(a2, ap + T * tstride, kst_a);
#pragma unroll
        for (int j = 0; j < C; ++j) aT[j] = ocx_zj(a2, j);
    }
    double cum = 0.0, comp = 0.0;
    for (int64_t t = 0; t < T; ++t) {
        ocx_d2 z[K], a2[K];
        ocx_load_tile<C>(z, zp + t * tstride, kst);
        ocx_load_tile<C>(a2, ap + t * tstride, kst_a);
        const double yv = yp[t * S];
        double a[C];
#pragma unroll
        for (int j = 0; j < C; ++j) a[j] = ocx_zj(a2, j);
        const double q = ocx_zdot<C, P, CHAIN>(z, a, lane);
        const double qc = ocx_zdot<C, P, CHAIN>(z, aT, lane);
        cum += 0.5 * fabs(q - yv);
        comp += 0.5 * fabs(qc - yv);
    }
    if (c == 0 && b < B) {
        cum_out[b] = cum;
        comp_out[b] = comp;
    }
}

// ---------------------------------------------------------------------------
// exact_ftl.py:280-303 `compute_prefix_actions` for the l2 ball, in the closed form of
// the exact SOCP solution (regime as ocx_alg_kernel algo 2): actions[b][t] = FTL of
// theta_t = −S_t = −Σ_{i<t} y_i z_i for t = 0..T, row-major [B][T+1][d].  The same step
// arithmetic as algo 2, so replaying these actions reproduces ocx_ftl_exact's losses bit
// for bit.  Writes are per-sequence rows (d contiguous doubles per lane group): this is
// the drivers' small-batch API, not a bandwidth path.
// ---------------------------------------------------------------------------
template <int C, int P, bool CHAIN>
__global__ __launch_bounds__(OCX_BLOCK) void ocx_prefix_actions_kernel(
    const double* __restrict__ zt, const double* __restrict__ yt, int64_t B, int64_t T,
    int64_t d, int64_t G, double* __restrict__ actions, int* __restrict__ regime_out, int norm) {
    constexpr int S = 64 / P;
    constexpr int K = C / 2;
    const int lane = threadIdx.x & 63;
    const int64_t g = ocx_wave_id();
    if (g >= G) return;
    const int s = lane / P;
    const int c = lane % P;
    const int64_t b = g * S + s;
    const int64_t tstride = 64;
    const ocx_d2* __restrict__ zp = reinterpret_cast<const ocx_d2*>(zt) + g * T * tstride + lane;
    const int64_t kst = G * T * 64;
    const double* __restrict__ yp = yt + g * T * S + s;
    double* __restrict__ arow = actions + (b < B ? b : 0) * (T + 1) * d + (int64_t)c * C;
    const int jn = (int)std::max<int64_t>(0, std::min<int64_t>(C, d - (int64_t)c * C));

    double th[C];
#pragma unroll
    for (int j = 0; j < C; ++j) th[j] = 0.0;
    bool linear = true;
    uint64_t touch = 0;
    for (int64_t t = 0; t <= T; ++t) {
        double x[C];
        if (norm != 0) {
            ocx_action_exact_poly<C, P>(th, x, norm, lane);
            linear = linear && !ocx_exact_poly_tie<C, P>(th, touch, norm);
        } else {
            ocx_action_ftl<C, P, CHAIN>(th, x, lane);
        }
        if (b < B) {
#pragma unroll
            for (int j = 0; j < C; ++j)
                if (j < jn) arow[t * d + j] = x[j];
        }
        if (t == T) break;
        ocx_d2 z[K];
        ocx_load_tile<C>(z, zp + t * tstride, kst);
        const double yv = yp[t * S];
        linear = linear && ocx_dual_ok<C, P, CHAIN>(z, norm, lane) && fabs(yv) == 1.0;
        if (norm == 2) touch = ocx_touch<C>(touch, z);
        const double gq = -yv;
#pragma unroll
        for (int j = 0; j < C; ++j) th[j] += gq * ocx_zj(z, j);
    }
    if (c == 0 && b < B && regime_out) regime_out[b] = linear ? 1 : 0;
}

// ---------------------------------------------------------------------------
// Layout packing and small reductions
// ---------------------------------------------------------------------------
__global__ void ocx_pack_z_kernel(const double* __restrict__ z, double* __restrict__ zt,
                                  int64_t B, int64_t T, int64_t d, int P, int C, int64_t G,
                                  int64_t total) {
    const int S = 64 / P;
    for (int64_t o = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; o < total;
         o += (int64_t)gridDim.x * blockDim.x) {
        // o = ((k*G + g)*T + t)*128 + 2L + e
        const int64_t row = o >> 7;
        const int L = (int)((o & 127) >> 1), e = (int)(o & 1);
        const int64_t kg = row / T;
        const int64_t t = row - kg * T;
        const int64_t k = kg / G, g = kg - k * G;
        const int64_t b = g * S + L / P;
        const int64_t j = (int64_t)(L % P) * C + 2 * k + e;
        zt[o] = (b < B && j < d) ? z[(b * T + t) * d + j] : 0.0;
    }
}

__global__ void ocx_pack_y_kernel(const double* __restrict__ y, double* __restrict__ ytl,
                                  int64_t B, int64_t T, int S, int64_t total) {
    for (int64_t o = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; o < total;
         o += (int64_t)gridDim.x * blockDim.x) {
        const int64_t tix = o / S;
        const int s = (int)(o - tix * S);
        const int64_t g = tix / T, t = tix - (tix / T) * T;
        const int64_t b = g * S + s;
        ytl[o] = (b < B) ? y[b * T + t] : 0.0;
    }
}

// max over runs starting from 0.0 with `reg > max` (fast_algorithms.py:228, :242-243)
__global__ void ocx_max_kernel(const double* __restrict__ r, int64_t B, double* __restrict__ out) {
    __shared__ double sm[OCX_BLOCK];
    double m = 0.0;
    for (int64_t i = threadIdx.x; i < B; i += blockDim.x) {
        const double v = r[i];
        if (v > m) m = v;
    }
    sm[threadIdx.x] = m;
    __syncthreads();
    for (int w = OCX_BLOCK / 2; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w && sm[threadIdx.x + w] > sm[threadIdx.x])
            sm[threadIdx.x] = sm[threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x == 0) *out = sm[0];
}

// ---------------------------------------------------------------------------
// Launchers: runtime (C, P) → template instance
// ---------------------------------------------------------------------------
namespace {

// (grid, block) of a launch over G wave-groups (ocx_block_waves)
#define OCX_SHAPE(G) ocx_grid((G), ocx_block_waves(G)), dim3(64 * ocx_block_waves(G))

template <int C, int P, bool CH>
hipError_t launch_alg_cp(const ocx_layout* L, const double* zt, const double* yt, int algo,
                         double eta0, const double* cmp, double* reg, double* cum, double* comp,
                         double* xl, double* cmp_out, int* regime, int onepass, int norm,
                         hipStream_t st) {
    hipLaunchKernelGGL((ocx_alg_kernel<C, P, CH, nb_for(C, P)>), OCX_SHAPE(L->G), 0, st, zt, yt,
                       L->B, L->T, L->d, L->G, algo, eta0, cmp, reg, cum, comp, xl, cmp_out,
                       regime, onepass, norm, (int64_t)0, L->G, (unsigned long long*)nullptr);
    return hipGetLastError();
}

// FTRL over wave-groups [g0, g0 + gn) of L with g(T) folded into gmax (nullable): the small-d
// pipeline's FTRL side (ocx_pipeline.hip), the g(T) layouts of 16 <= d < 64 (butterfly, 8 lanes)
template <int C, int P, bool CH>
hipError_t launch_alg_range_cp(const ocx_layout* L, const double* zt, const double* yt,
                               double eta0, double* reg, int onepass, int64_t g0, int64_t gn,
                               unsigned long long* gmax, hipStream_t st) {
    if constexpr (CH) {
        return hipErrorInvalidValue;
    } else {
        // one-wave blocks: the dispatcher spreads them over the SIMDs the generator leaves room on
        hipLaunchKernelGGL((ocx_alg_kernel<C, P, false, nb_for(C, P), 4>), ocx_grid(gn, 1), dim3(64), 0,
                           st, zt, yt, L->B, L->T, L->d, L->G, 0, eta0, (const double*)nullptr, reg,
                           (double*)nullptr, (double*)nullptr, (double*)nullptr, (double*)nullptr,
                           (int*)nullptr, onepass, 0, g0, gn, gmax);
        return hipGetLastError();
    }
}

template <int C, int P, bool CH>
hipError_t launch_smart_cp(const ocx_layout* L, const double* zt, const double* yt,
                           const double* th, double eta0, double* reg, int64_t* sw,
                           hipStream_t st) {
    hipLaunchKernelGGL((ocx_smart_kernel<C, P, CH>), OCX_SHAPE(L->G), 0, st,
                       zt, yt, L->B, L->T, L->G, th, eta0, reg, sw);
    return hipGetLastError();
}

template <int C, int P, bool CH>
hipError_t launch_replay_cp(const ocx_layout* L, const double* zt, const double* yt,
                            const double* at, double* cum, double* comp, hipStream_t st) {
    hipLaunchKernelGGL((ocx_replay_kernel<C, P, CH>), OCX_SHAPE(L->G), 0,
                       st, zt, yt, at, L->B, L->T, L->G, cum, comp);
    return hipGetLastError();
}

template <int C, int P, bool CH>
hipError_t launch_prefix_cp(const ocx_layout* L, const double* zt, const double* yt,
                            double* actions, int* regime, int norm, hipStream_t st) {
    hipLaunchKernelGGL((ocx_prefix_actions_kernel<C, P, CH>), OCX_SHAPE(L->G), 0, st, zt, yt,
                       L->B, L->T, L->d, L->G, actions, regime, norm);
    return hipGetLastError();
}

}  // namespace

bool ocx_supported_C(int C) {
    return C == 2 || C == 4 || C == 6 || C == 8 || C == 12 || C == 16 || C == 24 || C == 32 ||
           C == 48 || C == 64;
}

hipError_t ocx_launch_alg(const ocx_layout* L, const double* zt, const double* yt, int algo,
                          double eta0, const double* cmp, double* reg, double* cum, double* comp,
                          double* xl, hipStream_t st, double* cmp_out, int* regime, int onepass,
                          int norm) {
    if (L->G == 0) return hipSuccess;
    // butterfly layouts: the pipelined step (ocx_alg_pipe.hip) unless an input comparator,
    // x_last or the comparator action is asked for (OCX_ALG_NO_PIPE=1: the plain kernel,
    // for A/B measurements)
    static const bool no_pipe = [] {
        const char* e = std::getenv("OCX_ALG_NO_PIPE");
        return e && std::atoi(e) != 0;
    }();
    if ((algo == 0 || algo == 1) && !cmp && !xl && !cmp_out && !no_pipe && ocx_pipe_supported(L))
        return ocx_launch_alg_pipe(L, zt, yt, algo, eta0, reg, cum, comp, regime, onepass, st);
    OCX_DISPATCH(launch_alg_cp, L, zt, yt, algo, eta0, cmp, reg, cum, comp, xl, cmp_out, regime,
                 onepass, norm, st)
}

hipError_t ocx_launch_alg_range(const ocx_layout* L, const double* zt, const double* yt,
                                double eta0, double* reg, int onepass, int64_t g0, int64_t gn,
                                unsigned long long* gmax, hipStream_t st) {
    if (gn <= 0) return hipSuccess;
    if (g0 < 0 || g0 + gn > L->G || L->chain) return hipErrorInvalidValue;
    // d = 16's g(T) layout: 8 lanes of 2 coordinates (8 x 4 runs the pipelined kernel's lean form)
    if (L->P == 8 && L->C == 2)
        return launch_alg_range_cp<2, 8, false>(L, zt, yt, eta0, reg, onepass, g0, gn, gmax, st);
    return hipErrorInvalidValue;
}

hipError_t ocx_launch_smart(const ocx_layout* L, const double* zt, const double* yt,
                            const double* th, double eta0, double* reg, int64_t* sw,
                            hipStream_t st) {
    if (L->G == 0) return hipSuccess;
    // Small batches (the drivers' few hundred sequences) cannot hide the prefix
    // re-scan's latency with lane groups: one wavefront per sequence instead.
    // OCX_SMART_KERNEL=wave|lanes forces a path (tests, tuning).
    bool wave = L->d <= 64 && L->B <= 32768;  // measured: wave 0.22 s vs lanes 0.30 s at 32768 (d = 5)
    if (const char* e = std::getenv("OCX_SMART_KERNEL"))
        wave = std::strcmp(e, "wave") == 0 && L->d <= 64;
    if (wave) return ocx_launch_smart_wave(L, zt, yt, th, eta0, reg, sw, st);
    OCX_DISPATCH(launch_smart_cp, L, zt, yt, th, eta0, reg, sw, st)
}

hipError_t ocx_launch_replay(const ocx_layout* L, const double* zt, const double* yt,
                             const double* at, double* cum, double* comp, hipStream_t st) {
    if (L->G == 0) return hipSuccess;
    OCX_DISPATCH(launch_replay_cp, L, zt, yt, at, cum, comp, st)
}
hipError_t ocx_launch_prefix_actions(const ocx_layout* L, const double* zt, const double* yt,
                                     double* actions, int* regime, hipStream_t st, int norm) {
    if (L->G == 0) return hipSuccess;
    OCX_DISPATCH(launch_prefix_cp, L, zt, yt, actions, regime, norm, st)
}

hipError_t ocx_launch_pack(const ocx_layout* L, const double* z, const double* y, double* zt,
                           double* ytl, hipStream_t st) {
    const int64_t zn = L->z_elems, yn = L->y_elems;
    if (zn > 0) {
        const unsigned grid = (unsigned)std::min<int64_t>((zn + 255) / 256, 65536);
        hipLaunchKernelGGL(ocx_pack_z_kernel, dim3(grid), dim3(256), 0, st, z, zt, L->B, L->T,
                           L->d, L->P, L->C, L->G, zn);
    }
    if (yn > 0) {
        const unsigned grid = (unsigned)std::min<int64_t>((yn + 255) / 256, 65536);
        hipLaunchKernelGGL(ocx_pack_y_kernel, dim3(grid), dim3(256), 0, st, y, ytl, L->B, L->T,
                           L->S, yn);
    }
    return hipGetLastError();
}

hipError_t ocx_launch_max(const double* r, int64_t B, double* out, hipStream_t st) {
    hipLaunchKernelGGL(ocx_max_kernel, dim3(1), dim3(OCX_BLOCK), 0, st, r, B, out);
    return hipGetLastError();
}
