// ocx_alg_pipe.hip — FTRL/FTL (fast_algorithms.py:88-115) for the butterfly-sum layouts
// (P >= 2 lanes per sequence, chain = 0) with the step's dependency chain cut short.
//
// In the plain kernel (ocx_sim.hip) step t waits for g_{t-1}, then forms x = sθ_t, sums
// ||x||² and z_t·x lane by lane (C dependent adds each), crosses the P lanes, and — when
// the FTRL action is rescaled, which on the g(T) adversary is most steps — sums z_t·x a
// second time: about 60 dependent fp64 operations, ≈1 100 cycles per step.  A few-wave
// batch (capacity-limited long horizons: d = 64, T = 1e5, ≈4 900 sequences, one wave per
// SIMD) cannot hide that, so its time is T × that latency.
//
// Here every lane-local product of step t is formed BEFORE g_{t-1} is known, from the
// lagging state θ' = θ_{t-1} (θ_t = θ' + g_{t-1} z_{t-1}):
//     A = z_t·θ',  Bz = z_t·z_{t-1},  U = θ'·θ',  V = θ'·z_{t-1},  W = z_{t-1}·z_{t-1}
// (per lane, over its C coordinates), so that once g = g_{t-1} arrives
//     z_t·θ_t = A + g·Bz,   ||θ_t||² = U + g·(2V + g·W)
// are one or two fma per lane, then the P-lane butterflies; FTRL's action follows as
//     s_abs = |s_t|·sqrt(||θ_t||²),  f = 1/s_abs if s_abs > 1 else 1,  q = (s_t·(z_t·θ_t))·f
// and FTL's as q = (−1/sqrt(||θ_t||²))·(z_t·θ_t) (0 when θ_t = 0).  The chain is ≈25
// dependent operations; the C-wide products run beside it.  θ itself is updated exactly
// as the reference does (θ += g·z, g a power of two), so the trajectory is the
// reference's; each step's q carries the butterfly layouts' usual ~1e-16 relative
// rounding difference (tests/test_gpu_parity.py: 1e-12 bar).  For rows with a single
// nonzero coordinate (the flip / switching families, exact ties) every quantity above
// is exact and equal to the reference's (sqrt of an exact square is exact; s_abs =
// |fl(s θ_j)| and f = fl(1/s_abs) then reproduce the reference's rescale bit for bit).
// FTL near θ = 0, where ||θ_t||² = U + g(2V + gW) would lose relative accuracy to
// cancellation, re-sums ||θ_t||² directly (||θ_t||² < 0.25: early steps, returns to the
// origin).  The comparator pass / closed form are those of ocx_alg_kernel.
#include <cstdlib>
#include <type_traits>

#include "ocx_device_math.h"
// tuning switches (A/B through _build.build_variant; bit-identical either way)
#ifndef OCX_PIPE_Y_SADDR
#define OCX_PIPE_Y_SADDR 0
#endif
#ifndef OCX_PIPE_FTL_NOBRANCH
#define OCX_PIPE_FTL_NOBRANCH 0
#endif
// FTL's near-origin test decided a step early: ||θ_{t+1}||² = ||θ_t||² + g(2 z_t·θ_t + g||z_t||²)
// >= ||θ_t||² − |z_t·θ_t| for every g in {−½, 0, ½}, so a sequence whose ||θ_t||² − |z_t·θ_t|
// clears 0.25 (with a margin far above the running update's rounding) cannot need the
// re-sum at t+1.  The step then tests one wave-uniform mask formed a step earlier (a scalar
// branch off the chain) instead of an exec-mask branch on ||θ_t||² itself; lanes of a wave
// that may need it run the per-lane test as before.  Bit-identical.
// The step counter's type (ocx_ring_loop): int keeps the loop tests on the scalar unit; used
// for C <= OCX_PIPE_IT32_MAXC coordinates per lane.  Measured (r04_pipe_ab.jsonl): the 16 x 4
// few-wave batch 35.5 -> 32.4 ms with it, while the 8 x 8 kernel's loads were scheduled with
// shallower waits and it ran 40.2 -> 42.0 ms, so 8 x 8 keeps the int64_t counter.
#ifndef OCX_PIPE_WAVE_CLOCK  // diagnostic: per-wave clocks instead of cum / comp (see below)
#define OCX_PIPE_WAVE_CLOCK 0
#endif
#ifndef OCX_PIPE_IT32_MAXC
#define OCX_PIPE_IT32_MAXC 4
#endif
#ifndef OCX_PIPE_FTL_EARLY
#define OCX_PIPE_FTL_EARLY 0
#endif
// FTRL: the rescale's sqrt only in waves where a sequence may need the rescale (RT, see the
// step): 0 never, 1 where measured faster (pipe_rt), 2 in every kernel (tuning)
#ifndef OCX_PIPE_RESCALE_TEST
#define OCX_PIPE_RESCALE_TEST 1
#endif
// FTRL's rescale as q = a · (1 / max(s_abs, 1)) on every lane instead of an exec-mask branch
// on s_abs > 1: where s_abs <= 1 the factor is exactly 1.0 and q = a, bit for bit.
#ifndef OCX_PIPE_FTRL_NOBRANCH
#define OCX_PIPE_FTRL_NOBRANCH 0
#endif

// The correctly rounded sqrt and reciprocal as the compiler expands them, without the parts
// for extreme operands: sqrt(n) is v_rsq_f64 and the Goldschmidt iteration the compiler
// emits, minus its scaling of n < 2^-767 and its class fix-up of 0 and inf; 1/s is v_rcp_f64,
// two Newton steps and the remainder correction, i.e. div_scale / div_fmas / div_fixup with
// nothing to scale or fix.  Same operations in the same order, so the same bits, for
// 2^-500 <= n <= 2^500 (the caller checks the range for the whole wave and otherwise takes
// sqrt() and the division).  OCX_PIPE_FAST_SQRT (tuning until measured).
#ifndef OCX_PIPE_FAST_SQRT
#define OCX_PIPE_FAST_SQRT 0
#endif
__device__ __forceinline__ double ocx_sqrt_mid(double n) {
    const double r = __builtin_amdgcn_rsq(n);
    double g = n * r, h = r * 0.5;
    const double e = __builtin_fma(-h, g, 0.5);
    g = __builtin_fma(g, e, g);
    h = __builtin_fma(h, e, h);
    double d = __builtin_fma(-g, g, n);
    g = __builtin_fma(d, h, g);
    d = __builtin_fma(-g, g, n);
    return __builtin_fma(d, h, g);
}
__device__ __forceinline__ double ocx_div_mid(double a, double b) {  // a / b, |a| = 1
    double r = __builtin_amdgcn_rcp(b);
    double e = __builtin_fma(-b, r, 1.0);
    r = __builtin_fma(r, e, r);
    e = __builtin_fma(-b, r, 1.0);
    r = __builtin_fma(r, e, r);
    const double q = a * r;
    const double rem = __builtin_fma(-b, q, a);
    return __builtin_fma(rem, r, q);
}
__device__ __forceinline__ bool ocx_mid_range(double n) { return n >= 0x1p-500 && n <= 0x1p500; }

// 1/sqrt(n) for n > 0: v_rsq_f64 and two Newton steps (r <- r + r(1 - n r²)/2), within a
// few ulp — the fast action (FQ) below, never where the reference's rounding is promised.
__device__ __forceinline__ double ocx_rsq_nr(double n) {
    double r = __builtin_amdgcn_rsq(n);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const double e = __builtin_fma(-n * r, r, 1.0);
        r = __builtin_fma(0.5 * r, e, r);
    }
    return r;
}
// The sub-gradient the SPEC step assumes for step t: fast_algorithms.py:27-34 with q_t
// strictly inside (−1, 1), i.e. sign(q − y)/2 = −sign(y)/2 (y = 0: 0, checked like the rest).
__device__ __forceinline__ double ocx_spec_grad(double y) {
    return y > 0.0 ? -0.5 : (y < 0.0 ? 0.5 : 0.0);
}
#include "ocx_internal.h"
#include "ocx_sim_kernels.h"

// Wave-group of this wave when gn groups run in blocks of W waves.  A plain blockIdx * W +
// wave mapping leaves the nblk * W − gn spare slots in the last block, so a few-wave launch
// ends with a block of one or two waves, alone on its CU — and a lone FTL wave measured
// ≈10 % slower than its neighbours in full blocks, setting the launch's time
// (profiles/r04_wave_clock*.jsonl).  Here the last `idle` blocks hold W − 1 groups each
// instead (W = 4: at least three waves per CU); a spare slot gets gn and exits.
__device__ __forceinline__ int64_t ocx_pipe_wave_id(int64_t gn) {
    const int64_t W = blockDim.x >> 6, blk = blockIdx.x, w = threadIdx.x >> 6;
    const int64_t idle = (int64_t)gridDim.x * W - gn;
    const int64_t full = (int64_t)gridDim.x - idle;  // blocks of W groups
    if (idle <= 0 || full < 0 || blk < full) return blk * W + w;
    return w < W - 1 ? full * W + (blk - full) * (W - 1) + w : gn;
}

// MINW: waves per SIMD the register allocation must allow (1: the whole file; 4: at most
// 128 VGPRs, the lean form the overlapped pipeline runs beside the generator,
// ocx_pipeline.hip).  The launch covers wave-groups [g0, g0 + gn) of the layout.
// FQ (the fast action, g(T) rows only: the caller's OCX_ALG_CLIPPED_ROWS batches): the step's
// 1/sqrt and division — ≈30 of its ≈160 VALU instructions, and most of its dependency chain —
// become one v_rsq_f64 refined by two Newton steps, so q_t = s_t (z_t·θ_t) · min(1, rsqrt(||θ_t||²)
// / |s_t|) (FTRL; 1/|s_t| from the same 64-step table as s_t) or −(z_t·θ_t) · rsqrt(||θ_t||²)
// (FTL), a few ulp from the reference's fl(1/fl(sqrt(·))).  Only a sub-gradient can turn on
// an ulp: wherever |q_t − y_t| <= 1e-12 |q_t| (an exact tie is possible there) the step
// recomputes q_t in the reference's rounding before the hinge and the sub-gradient, so ties
// and their g = 0 are the reference's.  The regrets are then within the butterfly layouts'
// 1e-12 bar, not bit-identical to the exact-rounding form (FQ = false).
template <int C, int P, int NB, bool FTL, bool CAND, bool FQ = false, bool RT = false,
          bool SPEC = false>
__device__ __forceinline__ void alg_pipe_body(
    const double* __restrict__ zt, const double* __restrict__ yt, int64_t B, int64_t T,
    int64_t G, double eta0, double* __restrict__ regret, double* __restrict__ cum_out,
    double* __restrict__ comp_out, int* __restrict__ closed_out, int onepass, int64_t g0,
    int64_t gn) {
    static_assert(P >= 2 && NB >= 4, "butterfly layouts, a ring holding z_{t-1} .. z_{t+1}");
    using IT = typename std::conditional<(C <= OCX_PIPE_IT32_MAXC), int, int64_t>::type;
    constexpr int S = 64 / P;
    constexpr int K = C / 2;
    const int lane = threadIdx.x & 63;
    // wave-uniform, provably (readfirstlane): the tile bases live in SGPRs and every load
    // is an SGPR base + the lane's constant offset, with no per-load address arithmetic
    const int64_t wv = (int64_t)__builtin_amdgcn_readfirstlane((int)ocx_pipe_wave_id(gn));
    if (wv >= gn) return;
    const int64_t g = g0 + wv;
#if OCX_PIPE_WAVE_CLOCK  // diagnostic build only: see the end of the body
    const uint64_t clk0 = __builtin_amdgcn_s_memrealtime();
#endif
#ifdef OCX_ALG_PRIO  // tuning: issue priority over waves of a kernel running beside it
    __builtin_amdgcn_s_setprio(OCX_ALG_PRIO);
#endif
    const int s = lane / P;
    const int c = lane % P;
    const int64_t b = g * S + s;
    // The layout's padding sequences (b >= B, the last wave-group's spare slots) have all-zero
    // rows, so their θ stays 0 and FTL's near-origin re-sum below would run for them at every
    // step — in the one wave that holds them, which then set the launch's time (a 47.6 ms
    // straggler among 41–42 ms waves on the 4 900 x 1e5 batch, profiles/r04_wave_clock*.jsonl).
    // Their results are never written, so they skip it.
    const bool live = b < B;
    const int64_t tstride = 64;  // ocx_d2 per step within a plane
    const ocx_d2* __restrict__ zg = reinterpret_cast<const ocx_d2*>(zt) + g * T * tstride;
    const int64_t kst = G * T * 64;  // plane stride (pairs k)
    const double* __restrict__ yg = yt + g * T * S;
    bool clean = true;  // onepass: rows in the ball, every sub-gradient −y_t/2

    double th[C];  // θ_{t-1} (lagging one update)
#pragma unroll
    for (int j = 0; j < C; ++j) th[j] = 0.0;
    double gp = 0.0;                                   // g_{t-1}
    double A = 0.0, Bz = 0.0, U = 0.0, V = 0.0, W = 0.0;  // step t's lane partials

    // z_{t-1} is read where it lies, in the slot before step t's: the late loads
    // (ocx_ring_loop<NB, true>) refill that slot only after step t.  At t = 0 that slot is
    // the zeroed one below (g_{-1} = 0 multiplies it).
    ocx_d2 zb[NB][K];
    double yb[NB];
#pragma unroll
    for (int k = 0; k < K; ++k) zb[NB - 1][k] = ocx_d2{0.0, 0.0};
    auto load = [&](int slot, int64_t tl) {
        const ocx_d2* __restrict__ row = zg + tl * tstride;  // uniform
#pragma unroll
        for (int k = 0; k < K; ++k) {
#if OCX_LOAD_NT
            zb[slot][k] = __builtin_nontemporal_load(row + k * kst + lane);
#else
            zb[slot][k] = row[k * kst + lane];
#endif
        }
#if OCX_PIPE_Y_SADDR
        yb[slot] = (yg + tl * S)[s];  // uniform row base (SGPRs) + the lane's constant offset
#else
        yb[slot] = yg[tl * S + s];
#endif
    };
    double cum = 0.0;
    double scv = 0.0;  // −η0/√(t+1+lane) for the 64 steps from the last multiple of 64
    double iscv = 0.0;  // FQ: 1/|scv|
#if OCX_PIPE_FTL_EARLY
    uint64_t near_m = ~0ULL;  // FTL: lanes whose step may need the near-origin re-sum (θ_0 = 0)
#endif

    // ---- CAND: the step's action for every value g_{t-1} can take, formed a step early.
    // g is −½, 0 or +½, so z_t·θ_t = A + g·Bz and ||θ_t||² = U + g(2V + gW) have three
    // possible values; their butterflies, sqrt and division — everything the plain pipelined
    // step does after g_{t-1} arrives — are formed for g = ±½ at the end of step t−1 (beside
    // step t−1's own chain), and step t only selects.  The selected values are the ones the
    // plain step computes from the same lane partials, bit for bit.  g = 0 (an exact tie) is
    // formed when it happens (a wave-uniform branch on the chain, rare outside the flip /
    // switching families).
    double qq_m = 0.0, qq_p = 0.0;  // step t's q_t for g_{t-1} = −½ / +½
    double zl_m = 0.0, zl_p = 0.0, tl_m = 0.0, tl_p = 0.0;  // their lane partials
    // q from the lane partials of z_t·θ_t (zl) and ||θ_t||² (tl) at step t1; FTL near the
    // origin re-sums ||θ_t||² directly from θ_t = th + g·zc (as the plain step does)
    auto q_of = [&](double zl, double& tl, double g, const ocx_d2* zc, int64_t t1) -> double {
        const double q_raw = ocx_seq_sum<P>(zl);
        double n_raw = ocx_seq_sum<P>(tl);
        if constexpr (!FTL) {
            const double sc = ocx_readlane(scv, (int)(t1 & 63));
            const double a = sc * q_raw;
            const double s_abs = fabs(sc) * sqrt(n_raw > 0.0 ? n_raw : 0.0);
            return s_abs > 1.0 ? a * (1.0 / s_abs) : a;
        } else {
            if (__ballot(n_raw < 0.25 && live) != 0) {  // wave-uniform; per sequence below
                double p[C];
#pragma unroll
                for (int j = 0; j < C; ++j) {
                    const double tj = __builtin_fma(g, ocx_zj(zc, j), th[j]);
                    p[j] = tj * tj;
                }
                const double tld = ocx_lane_sum<C>(p);
                const double nd = ocx_seq_sum<P>(tld);
                if (n_raw < 0.25 && live) {
                    tl = tld;
                    n_raw = nd;
                }
            }
            return n_raw == 0.0 ? 0.0 : (-(1.0 / sqrt(n_raw))) * q_raw;
        }
    };
    auto make_cand = [&](const ocx_d2* zc, int64_t t1) {
        const double v2 = 2.0 * V;
        zl_m = __builtin_fma(-0.5, Bz, A);
        zl_p = __builtin_fma(0.5, Bz, A);
        tl_m = __builtin_fma(-0.5, __builtin_fma(-0.5, W, v2), U);
        tl_p = __builtin_fma(0.5, __builtin_fma(0.5, W, v2), U);
        qq_m = q_of(zl_m, tl_m, -0.5, zc, t1);
        qq_p = q_of(zl_p, tl_p, 0.5, zc, t1);
    };
    if constexpr (CAND) {
        if constexpr (!FTL) scv = -(eta0 / sqrt((double)(1 + lane)));
        make_cand(zb[NB - 1], 0);  // θ_0 = 0 whatever g_{-1}: every candidate is q_0
    }

    if constexpr (CAND) ocx_ring_loop<NB, true, IT>(T, load, [&](int u, int64_t t) {
        const ocx_d2* zp1 = zb[(u + NB - 1) % NB];  // z_{t-1}
        // ---- chain: g_{t-1} → select q_t → g_t
        double q = gp > 0.0 ? qq_p : qq_m;
        double zth = gp > 0.0 ? zl_p : zl_m;
        double tth = gp > 0.0 ? tl_p : tl_m;
        if (__ballot(gp == 0.0) != 0) {  // an exact tie last step: θ_t = θ_{t-1}
            double tl0 = U;
            const double q0 = q_of(A, tl0, 0.0, zp1, t);
            if (gp == 0.0) {
                q = q0;
                zth = A;
                tth = tl0;
            }
        }
        const double yv = yb[u];
        const double diff = q - yv;  // :106-111
        cum += 0.5 * fabs(diff);
        const double gq = ocx_grad(diff);
        clean = clean && fabs(yv) == 1.0 && gq == -0.5 * yv;

        // ---- beside the chain: θ_t, step t+1's lane partials and its candidates
#pragma unroll
        for (int j = 0; j < C; ++j) th[j] = __builtin_fma(gp, ocx_zj(zp1, j), th[j]);
        const ocx_d2* zc = zb[u];
        const ocx_d2* zn = zb[(u + 1) % NB];
        double w = 0.0, an = 0.0, bn = 0.0;
#pragma unroll
        for (int j = 0; j < C; ++j) {
            const double zj = ocx_zj(zc, j);
            w = __builtin_fma(zj, zj, w);
            an = __builtin_fma(ocx_zj(zn, j), th[j], an);
            bn = __builtin_fma(ocx_zj(zn, j), zj, bn);
        }
        if (onepass) clean = clean & (ocx_seq_sum<P>(w) <= 1.0 + 1e-12);
        V = zth;
        W = w;
        A = an;
        Bz = bn;
        gp = gq;
        if (((t + 1) & 63) == 0) {  // as the plain step's refresh at the top of step t+1
            if constexpr (!FTL) scv = -(eta0 / sqrt((double)(t + 2 + lane)));
            double uu = 0.0;
#pragma unroll
            for (int j = 0; j < C; ++j) uu = __builtin_fma(th[j], th[j], uu);
            U = uu;
        } else {
            U = tth;
        }
        make_cand(zc, t + 1);
    });
    if constexpr (CAND) {
        if (T > 0) {
            ocx_d2 zl[K];
            ocx_load_tile<C>(zl, zg + (T - 1) * tstride + lane, kst);
#pragma unroll
            for (int j = 0; j < C; ++j) th[j] = __builtin_fma(gp, ocx_zj(zl, j), th[j]);
        }
    }
    auto run_plain = [&]() {
    ocx_ring_loop<NB, true, IT>(T, load, [&](int u, int64_t t) {
        // every 64 steps: the FTRL scales of the next 64 steps (one per lane, one sqrt/div
        // per lane instead of one per step) and ||θ||²'s lane part summed afresh, so the
        // running update below drifts for at most 64 steps
        if ((t & 63) == 0) {
            if constexpr (!FTL) {
                scv = -(eta0 / sqrt((double)(t + 1 + lane)));
                if constexpr (FQ) iscv = 1.0 / fabs(scv);
            }
            double uu = 0.0;
#pragma unroll
            for (int j = 0; j < C; ++j) uu = __builtin_fma(th[j], th[j], uu);
            U = uu;
        }
        // ---- chain: g_{t-1} → z_t·θ_t, ||θ_t||² → q_t → g_t
        const double zth = __builtin_fma(gp, Bz, A);
        double tth = __builtin_fma(gp, __builtin_fma(gp, W, 2.0 * V), U);
        // θ_t = θ_{t-1} + g_{t-1} z_{t-1} (exact: g is a power of two or 0)
        const ocx_d2* zp1 = zb[(u + NB - 1) % NB];
#pragma unroll
        for (int j = 0; j < C; ++j) th[j] = __builtin_fma(gp, ocx_zj(zp1, j), th[j]);
        const double q_raw = ocx_seq_sum<P>(zth);
        double n_raw = ocx_seq_sum<P>(tth);
        double q;
        if constexpr (!FTL) {
            const double sc = ocx_readlane(scv, (int)(t & 63));  // −η0/√(t+1)
            const double a = sc * q_raw;
            if constexpr (FQ) {
                const double isc = ocx_readlane(iscv, (int)(t & 63));
                const double r = ocx_rsq_nr(n_raw > 1e-300 ? n_raw : 1e-300);
                q = a * fmin(r * isc, 1.0);  // exactly a where s_abs <= 1
                if (__ballot(fabs(q - yb[u]) <= 1e-12 * fabs(q)) != 0) {  // near a tie
                    const double s_abs = fabs(sc) * sqrt(n_raw > 0.0 ? n_raw : 0.0);
                    if (fabs(q - yb[u]) <= 1e-12 * fabs(q)) q = s_abs > 1.0 ? a * (1.0 / s_abs) : a;
                }
            } else {
            // RT: no sequence of the wave near the rescale (s²||θ||² < 1 − 1e-12, far outside
            // the rounding of the test below): q = s·(z·θ), without the sqrt the test below
            // needs — what the test below would give, bit for bit.  On the g(T) rows ||sθ||
            // stays near 0.71 and the rescale is rare.
            if (RT && __ballot(sc * sc * n_raw >= 1.0 - 1e-12) == 0) {
                q = a;
            } else {
#if OCX_PIPE_FAST_SQRT
            double s_abs;
            if (__ballot(!ocx_mid_range(n_raw)) == 0) s_abs = fabs(sc) * ocx_sqrt_mid(n_raw);
            else s_abs = fabs(sc) * sqrt(n_raw > 0.0 ? n_raw : 0.0);
#else
            const double s_abs = fabs(sc) * sqrt(n_raw > 0.0 ? n_raw : 0.0);
#endif
#if OCX_PIPE_FTRL_NOBRANCH
            q = a * (1.0 / fmax(s_abs, 1.0));
#else
            q = s_abs > 1.0 ? a * (1.0 / s_abs) : a;
#endif
            }
            }
        } else {
#if OCX_PIPE_FTL_EARLY
            if (near_m != 0)  // wave-uniform, formed at step t-1
#endif
            if (n_raw < 0.25 && live) {  // near θ = 0: re-sum directly (see above)
                double p[C];
#pragma unroll
                for (int j = 0; j < C; ++j) p[j] = th[j] * th[j];
                tth = ocx_lane_sum<C>(p);
                n_raw = ocx_seq_sum<P>(tth);
            }
#if OCX_PIPE_FTL_EARLY
            near_m = __ballot(live && !(n_raw - fabs(q_raw) >= 0.25 + 1e-9 * n_raw));
#endif
            if constexpr (FQ) {
                const double r = ocx_rsq_nr(n_raw > 0.0 ? n_raw : 1.0);
                q = n_raw == 0.0 ? 0.0 : -(q_raw * r);
                if (__ballot(fabs(q - yb[u]) <= 1e-12 * fabs(q)) != 0) {  // near a tie
                    if (fabs(q - yb[u]) <= 1e-12 * fabs(q))
                        q = n_raw == 0.0 ? 0.0 : (-(1.0 / sqrt(n_raw))) * q_raw;
                }
            } else {
#if OCX_PIPE_FTL_NOBRANCH
            // the sqrt and division on every lane (no exec-mask branch around them); where
            // θ_t = 0 they run on 1.0 and the select keeps the reference's 0
            const double ns = n_raw > 0.0 ? n_raw : 1.0;
            const double rs = -(1.0 / sqrt(ns));
            q = n_raw == 0.0 ? 0.0 : rs * q_raw;
#elif OCX_PIPE_FAST_SQRT
            if (__ballot(!ocx_mid_range(n_raw) && n_raw != 0.0) == 0)
                q = n_raw == 0.0 ? 0.0 : (-ocx_div_mid(1.0, ocx_sqrt_mid(n_raw > 0.0 ? n_raw : 1.0))) * q_raw;
            else
                q = n_raw == 0.0 ? 0.0 : (-(1.0 / sqrt(n_raw))) * q_raw;
#else
            q = n_raw == 0.0 ? 0.0 : (-(1.0 / sqrt(n_raw))) * q_raw;
#endif
            }
        }
        const double yv = yb[u];
        const double diff = q - yv;  // :106-111
        cum += 0.5 * fabs(diff);
        const double gq = ocx_grad(diff);
        clean = clean && fabs(yv) == 1.0 && gq == -0.5 * yv;

        // ---- off the chain: step t+1's lane partials (θ_t is known, g_t is not)
        const ocx_d2* zc = zb[u];
        const ocx_d2* zn = zb[(u + 1) % NB];  // z_{t+1}, in flight since NB-2 steps
        double w = 0.0, an = 0.0, bn = 0.0;
#pragma unroll
        for (int j = 0; j < C; ++j) {
            const double zj = ocx_zj(zc, j);
            w = __builtin_fma(zj, zj, w);
            an = __builtin_fma(ocx_zj(zn, j), th[j], an);
            bn = __builtin_fma(ocx_zj(zn, j), zj, bn);
        }
        if (onepass) clean = clean & (ocx_seq_sum<P>(w) <= 1.0 + 1e-12);  // row t in ball
        // (at t = T-1, zn is the clamped look-ahead: A and Bz are then never used)
        V = zth;
        W = w;
        U = tth;  // ||θ_t||²'s lane part, by the running update
        A = an;
        Bz = bn;
        gp = gq;
    });
    // θ_T = θ_{T-1} + g_{T-1} z_{T-1} (z_{T-1} loaded again: its ring slot is not known at
    // compile time)
    if (T > 0) {
        ocx_d2 zl[K];
        ocx_load_tile<C>(zl, zg + (T - 1) * tstride + lane, kst);
#pragma unroll
        for (int j = 0; j < C; ++j) th[j] = __builtin_fma(gp, ocx_zj(zl, j), th[j]);
    }
    };

    // ---- SPEC: the sub-gradient taken as known.  On rows in the unit ball with labels ±1
    // (the g(T) adversary: the caller's onepass batches) |q_t| <= 1, so q_t − y_t has the
    // sign of −y_t and g_t = −y_t/2 whatever q_t is — the `clean` condition the closed-form
    // comparator already certifies.  θ's trajectory then does not wait for q: step t takes
    // ĝ_{t−1} = −y_{t−1}/2 (ocx_spec_grad) from the label ring, and step t−1's q (its sqrt and
    // division for FTL, FTRL's rare rescale), hinge loss and sub-gradient are finished in
    // step t's block, beside step t's butterflies, instead of on a chain between the steps.
    // Every step checks the g it computes against the ĝ it assumed; the arithmetic is the
    // plain step's, so where every check holds the results are the plain kernel's bit for
    // bit, and a wave where one fails runs the plain loop over again (run_plain).  The rare
    // branches (FTL near θ = 0, FTRL's rescale) are wave-uniform and decided by masks formed
    // a step early, at the top of the step, outside the block the scheduler interleaves.
    auto run_spec = [&]() -> bool {
        bool ok = true;
        double qr_p = 0.0, nr_p = 0.0, tth_p = 0.0, qa_p = 0.0, sc_p = 0.0;
        // the pending step before step 0: q = 0 against y = 1 (loss ½, cancelled by cum's start,
        // sub-gradient −½ = ĝ_{-1}, which multiplies the zeroed z_{-1})
        double y_p = 1.0;
        yb[NB - 1] = 1.0;
        cum = T > 0 ? -0.5 : 0.0;
        uint64_t fix_m = 0;  // lanes whose pending step needs its rare branch
        auto fix_pending = [&]() {  // θ = th = θ_{t-1}, the pending step's
            if (fix_m != 0) {  // wave-uniform
                if constexpr (FTL) {
                    if (nr_p < 0.25 && live) {  // the plain step's near-origin re-sum
                        double p[C];
#pragma unroll
                        for (int j = 0; j < C; ++j) p[j] = th[j] * th[j];
                        tth_p = ocx_lane_sum<C>(p);
                        nr_p = ocx_seq_sum<P>(tth_p);
                    }
                } else {  // the plain step's rescale
                    const double s_abs = fabs(sc_p) * sqrt(nr_p > 0.0 ? nr_p : 0.0);
                    if (s_abs > 1.0) qa_p = qa_p * (1.0 / s_abs);
                }
            }
        };
        auto finish_pending = [&](double gs) {  // q, hinge loss, sub-gradient check
            double qp;
            if constexpr (FTL) qp = nr_p == 0.0 ? 0.0 : (-(1.0 / sqrt(nr_p))) * qr_p;
            else qp = qa_p;
            const double diff = qp - y_p;  // :106-111
            cum += 0.5 * fabs(diff);
            const double gq = ocx_grad(diff);
            ok = ok & (gq == gs);
            clean = clean & (fabs(y_p) == 1.0) & (gq == -0.5 * y_p);
        };
        ocx_ring_loop<NB, true, IT>(T, load, [&](int u, int64_t t) {
            fix_pending();
            U = tth_p;
            if ((t & 63) == 0) {  // as the plain step
                if constexpr (!FTL) scv = -(eta0 / sqrt((double)(t + 1 + lane)));
                double uu = 0.0;
#pragma unroll
                for (int j = 0; j < C; ++j) uu = __builtin_fma(th[j], th[j], uu);
                U = uu;
            }
            // ---- one block: step t's sums (θ_t from ĝ_{t-1}) beside step t−1's finish
            const double gs = ocx_spec_grad(yb[(u + NB - 1) % NB]);  // ĝ_{t-1}
            const double zth = __builtin_fma(gs, Bz, A);
            const double tth = __builtin_fma(gs, __builtin_fma(gs, W, 2.0 * V), U);
            const ocx_d2* zp1 = zb[(u + NB - 1) % NB];
#pragma unroll
            for (int j = 0; j < C; ++j) th[j] = __builtin_fma(gs, ocx_zj(zp1, j), th[j]);
            const double q_raw = ocx_seq_sum<P>(zth);
            const double n_raw = ocx_seq_sum<P>(tth);
            finish_pending(gs);
            const ocx_d2* zc = zb[u];
            const ocx_d2* zn = zb[(u + 1) % NB];
            double w = 0.0, an = 0.0, bn = 0.0;
#pragma unroll
            for (int j = 0; j < C; ++j) {
                const double zj = ocx_zj(zc, j);
                w = __builtin_fma(zj, zj, w);
                an = __builtin_fma(ocx_zj(zn, j), th[j], an);
                bn = __builtin_fma(ocx_zj(zn, j), zj, bn);
            }
            clean = clean & (ocx_seq_sum<P>(w) <= 1.0 + 1e-12);  // SPEC runs onepass only
            V = zth;
            W = w;
            A = an;
            Bz = bn;
            qr_p = q_raw;
            nr_p = n_raw;
            tth_p = tth;
            y_p = yb[u];
            if constexpr (FTL) {
                fix_m = __ballot(n_raw < 0.25 && live);
            } else {
                sc_p = ocx_readlane(scv, (int)(t & 63));  // −η0/√(t+1)
                qa_p = sc_p * q_raw;
                fix_m = __ballot(sc_p * sc_p * n_raw >= 1.0 - 1e-12);  // RT's test
            }
        });
        if (T > 0) {
            fix_pending();
            const double gs = ocx_spec_grad(y_p);  // ĝ_{T-1}
            finish_pending(gs);
            ocx_d2 zl[K];
            ocx_load_tile<C>(zl, zg + (T - 1) * tstride + lane, kst);
#pragma unroll
            for (int j = 0; j < C; ++j) th[j] = __builtin_fma(gs, ocx_zj(zl, j), th[j]);
        }
        return ok;
    };
    if constexpr (CAND) {
        // ran its own loop and θ_T above
    } else if constexpr (SPEC) {
        if (__ballot(!run_spec()) != 0) {  // wave-uniform: a check failed, start again
#pragma unroll
            for (int j = 0; j < C; ++j) th[j] = 0.0;
            gp = A = Bz = U = V = W = 0.0;
            cum = scv = iscv = 0.0;
            clean = true;
#pragma unroll
            for (int k = 0; k < K; ++k) zb[NB - 1][k] = ocx_d2{0.0, 0.0};
#if OCX_PIPE_FTL_EARLY
            near_m = ~0ULL;
#endif
            run_plain();
        }
    } else {
        run_plain();
    }

    // ---- comparator: closed form where certified (ocx_alg_kernel onepass), else the
    // reference's second streaming pass with x* = FTL(θ_T) (fast_algorithms.py:113-114)
    const bool closed = onepass && (clean || b >= B);
    double comp = 0.0;
    if (__ballot(!closed) != 0) {  // wave-uniform
        double xs[C];
        ocx_action_ftl<C, P, false>(th, xs, lane);
        ocx_ring_loop<NB, false, IT>(T, load, [&](int u, int64_t) {
            double p[C];
#pragma unroll
            for (int j = 0; j < C; ++j) p[j] = ocx_zj(zb[u], j) * xs[j];
            const double qq = ocx_total<C, P, false>(p, lane);
            comp += 0.5 * fabs(qq - yb[u]);
        });
    }
    if (__ballot(closed) != 0) {
        double p[C];
#pragma unroll
        for (int j = 0; j < C; ++j) p[j] = th[j] * th[j];
        const double nrm = sqrt(ocx_total<C, P, false>(p, lane));
        if (closed) comp = 0.5 * (double)T - nrm;
    }
    if (c == 0 && b < B) {
        if (regret) regret[b] = cum - comp;
#if OCX_PIPE_WAVE_CLOCK
        // diagnostic build (tools/wave_clock_probe.py): the wave's duration in ticks of the
        // 100 MHz real-time clock, and where it ran (HW_ID, XCC_ID) — not results
        const uint64_t clk1 = __builtin_amdgcn_s_memrealtime();
        if (cum_out) cum_out[b] = (double)(clk1 - clk0);
        if (comp_out) comp_out[b] = (double)clk0;
        if (closed_out)
            closed_out[b] = (int)((__builtin_amdgcn_s_getreg((31 << 11) | 4) & 0xffffu) |
                                  ((__builtin_amdgcn_s_getreg((31 << 11) | 20) & 0xfu) << 16));
#else
        if (cum_out) cum_out[b] = cum;
        if (comp_out) comp_out[b] = comp;
        if (closed_out) closed_out[b] = closed ? 1 : 0;
#endif
    }
}

// The rescale test (RT) per kernel: measured (profiles/r04_pipe_ab3.jsonl) 3 328 x 1e5 at
// 16 x 4: 32.5 -> 28.7 ms; the pipeline's lean 8 x 8 form: 66.7 -> 64.3 ms per batch; but the
// 8 x 8 full form (the T = 1e5 batch): 40.8 -> 43.6 ms, which keeps the sqrt.
template <int C, int P, int MINW>
constexpr bool pipe_rt() {
    return OCX_PIPE_RESCALE_TEST == 2 || (OCX_PIPE_RESCALE_TEST == 1 && !(C == 8 && P == 8 && MINW == 1));
}
template <int C, int P, int NB, bool FTL, bool CAND, int MINW = 1, bool FQ = false,
          bool SPEC = false>
__global__ __launch_bounds__(OCX_BLOCK, MINW) void ocx_alg_pipe_kernel(
    const double* __restrict__ zt, const double* __restrict__ yt, int64_t B, int64_t T,
    int64_t G, double eta0, double* __restrict__ regret, double* __restrict__ cum_out,
    double* __restrict__ comp_out, int* __restrict__ closed_out, int onepass, int64_t g0,
    int64_t gn) {
    alg_pipe_body<C, P, NB, FTL, CAND, FQ, pipe_rt<C, P, MINW>(), SPEC>(
        zt, yt, B, T, G, eta0, regret, cum_out, comp_out, closed_out, onepass, g0, gn);
}

namespace {
// CAND (candidate actions formed a step early): bit-identical, and measured SLOWER on every
// batch it was meant for (profiles/r04_pipe_probe.jsonl): 4 900 x 1e5 x 64 FTRL 40.4 ->
// 67.8 ms, FTL 45.8 -> 95.1 ms; 3 328 x 1e5 (16 x 4) FTRL 35.5 -> 56.4 ms; d = 1024 and the
// bench batch unchanged or 2-3 % slower.  At 0.6 waves per SIMD the step is bound by the
// wave's instruction issue, not by its dependency chain: the two candidates' butterflies,
// sqrt and division per step cost more issue slots than the shorter chain saves.  Off by
// default; OCX_PIPE_CAND=1 selects it (tuning, tests; read at every launch).
bool pipe_cand(const ocx_layout* L) {
    // read per launch (a getenv per kernel launch is noise), so one process can A/B both
    if (const char* e = std::getenv("OCX_PIPE_CAND")) return std::atoi(e) != 0;
    return false;
}
// The fast action (FQ, see alg_pipe_body) on g(T) rows (onepass: the caller's
// OCX_ALG_CLIPPED_ROWS).  OCX_PIPE_FASTQ=0/1 overrides the default (read per launch).
#ifndef OCX_PIPE_FASTQ_DEFAULT
#define OCX_PIPE_FASTQ_DEFAULT 0
#endif
bool pipe_fastq(int onepass) {
    if (!onepass) return false;
    if (const char* e = std::getenv("OCX_PIPE_FASTQ")) return std::atoi(e) != 0;
    return OCX_PIPE_FASTQ_DEFAULT != 0;
}
// The SPEC step (see alg_pipe_body) on onepass batches: OCX_PIPE_SPEC=0/1 overrides the
// default per algorithm (read per launch).  Measured bit-identical and no faster on the
// few-wave batches (profiles/r04_pipe_spec_ab.jsonl: 4 900 x 1e5 x 64 FTRL 40.2 -> 42.9 ms,
// FTL 45.9 -> 46.3), so off.  The full form only: in the pipeline's 128-VGPR lean form its
// fallback loop spilled, and it measured no faster there either (65.9 / 65.8 vs 65.8 /
// 65.6 ms per batch, profiles/r04_overlap_spec_ab.jsonl).
#ifndef OCX_PIPE_SPEC_FTL
#define OCX_PIPE_SPEC_FTL 0
#endif
#ifndef OCX_PIPE_SPEC_FTRL
#define OCX_PIPE_SPEC_FTRL 0
#endif
// Waves per block of the full-form launch: four (one wave per SIMD of a CU, the last blocks
// three, ocx_pipe_wave_id) unless OCX_BLOCK_WAVES forces another shape or the launch has
// fewer than four groups.  The few-wave batches measured one-wave blocks (which the plain
// kernels keep below eight waves per CU) slower: profiles/r04_pipe_bw_ab.jsonl,
// r04_wave_clock*.jsonl.
int pipe_block_waves(int64_t G) {
    if (std::getenv("OCX_BLOCK_WAVES")) return ocx_block_waves(G);
    return G >= 4 ? 4 : 1;
}
bool pipe_spec(int onepass, bool ftl) {
    if (!onepass) return false;
    if (const char* e = std::getenv("OCX_PIPE_SPEC")) return std::atoi(e) != 0;
    return (ftl ? OCX_PIPE_SPEC_FTL : OCX_PIPE_SPEC_FTRL) != 0;
}

template <int C, int P, bool FTL, bool CAND>
hipError_t launch_pipe_k(const ocx_layout* L, const double* zt, const double* yt, double eta0,
                         double* reg, double* cum, double* comp, int* closed_out, int onepass,
                         hipStream_t st) {
    // z_{t-1} .. z_{t+1} must be in the ring, and the late loads (ocx_ring_loop) keep NB-2
    // steps in flight: one slot more than the plain kernel's ring
    constexpr int NB = nb_for(C, P) + 1 < 4 ? 4 : nb_for(C, P) + 1;
    const int bw = pipe_block_waves(L->G);
    const dim3 grid = ocx_grid(L->G, bw), block(64 * bw);
    if (!CAND && pipe_fastq(onepass))
        hipLaunchKernelGGL((ocx_alg_pipe_kernel<C, P, NB, FTL, false, 1, true>), grid, block, 0,
                           st, zt, yt, L->B, L->T, L->G, eta0, reg, cum, comp, closed_out, onepass,
                           (int64_t)0, L->G);
    else if (!CAND && pipe_spec(onepass, FTL))
        hipLaunchKernelGGL((ocx_alg_pipe_kernel<C, P, NB, FTL, false, 1, false, true>), grid,
                           block, 0, st, zt, yt, L->B, L->T, L->G, eta0, reg, cum, comp,
                           closed_out, onepass, (int64_t)0, L->G);
    else
        hipLaunchKernelGGL((ocx_alg_pipe_kernel<C, P, NB, FTL, CAND>), grid, block, 0, st, zt, yt,
                           L->B, L->T, L->G, eta0, reg, cum, comp, closed_out, onepass, (int64_t)0,
                           L->G);
    return hipGetLastError();
}

template <int C, int P>
hipError_t launch_pipe_cp(const ocx_layout* L, const double* zt, const double* yt, int ftl,
                          double eta0, double* reg, double* cum, double* comp, int* closed_out,
                          int onepass, hipStream_t st) {
    const bool cand = pipe_cand(L);
    if (ftl)
        return cand ? launch_pipe_k<C, P, true, true>(L, zt, yt, eta0, reg, cum, comp, closed_out, onepass, st)
                    : launch_pipe_k<C, P, true, false>(L, zt, yt, eta0, reg, cum, comp, closed_out, onepass, st);
    return cand ? launch_pipe_k<C, P, false, true>(L, zt, yt, eta0, reg, cum, comp, closed_out, onepass, st)
                : launch_pipe_k<C, P, false, false>(L, zt, yt, eta0, reg, cum, comp, closed_out, onepass, st);
}

template <int C>
hipError_t launch_pipe_c(const ocx_layout* L, const double* zt, const double* yt, int ftl,
                         double eta0, double* reg, double* cum, double* comp, int* closed_out,
                         int onepass, hipStream_t st) {
    switch (L->P) {
        case 8: return launch_pipe_cp<C, 8>(L, zt, yt, ftl, eta0, reg, cum, comp, closed_out, onepass, st);
        case 16: return launch_pipe_cp<C, 16>(L, zt, yt, ftl, eta0, reg, cum, comp, closed_out, onepass, st);
        case 32: return launch_pipe_cp<C, 32>(L, zt, yt, ftl, eta0, reg, cum, comp, closed_out, onepass, st);
        default: return hipErrorInvalidValue;
    }
}
}  // namespace

// The pipelined step pays where one wave's step latency sets the batch time: the few-wave
// butterfly layouts OCX_LANES_BEST chooses (8 x 8, 16 x 4 at d = 64; 16 x 16; 32 x 32 at
// d = 1024) and their neighbours.  Other butterfly layouts keep the plain kernel.
bool ocx_pipe_supported(const ocx_layout* L) {
    // T < 2^30: the step counter is a 32-bit int (ocx_ring_loop<..., int>)
    return !L->chain && L->T < ((int64_t)1 << 30) && (L->P == 8 || L->P == 16 || L->P == 32) &&
           (L->C == 4 || L->C == 8 || L->C == 16 || L->C == 32);
}

hipError_t ocx_launch_alg_pipe(const ocx_layout* L, const double* zt, const double* yt, int ftl,
                               double eta0, double* reg, double* cum, double* comp,
                               int* closed_out, int onepass, hipStream_t st) {
    if (L->G == 0) return hipSuccess;
    switch (L->C) {
        case 4: return launch_pipe_c<4>(L, zt, yt, ftl, eta0, reg, cum, comp, closed_out, onepass, st);
        case 8: return launch_pipe_c<8>(L, zt, yt, ftl, eta0, reg, cum, comp, closed_out, onepass, st);
        case 16: return launch_pipe_c<16>(L, zt, yt, ftl, eta0, reg, cum, comp, closed_out, onepass, st);
        case 32: return launch_pipe_c<32>(L, zt, yt, ftl, eta0, reg, cum, comp, closed_out, onepass, st);
        default: return hipErrorInvalidValue;
    }
}

// The lean form over wave-groups [g0, g0 + gn) (ocx_pipeline.hip): at most 128 VGPRs, so one
// wave fits on a SIMD beside three generator waves; a shorter ring (OCX_PIPE_LEAN_NB8 / _NB4
// slots at 8 / 4 coordinates per lane) is what makes it fit.  FTRL only, the pipeline's
// algorithm; 8 x 8 and 16 x 4 layouts.
#ifndef OCX_PIPE_LEAN_NB8
#define OCX_PIPE_LEAN_NB8 4
#endif
#ifndef OCX_PIPE_LEAN_NB4
#define OCX_PIPE_LEAN_NB4 8
#endif
#ifndef OCX_PIPE_LEAN168_NB
#define OCX_PIPE_LEAN168_NB 7
#endif
namespace {
template <int C, int P>
hipError_t launch_lean(const ocx_layout* L, const double* zt, const double* yt, double eta0,
                       double* reg, int onepass, int64_t g0, int64_t gn, int cand,
                       hipStream_t st) {
    constexpr int NB = C >= 8 ? OCX_PIPE_LEAN_NB8 : OCX_PIPE_LEAN_NB4;
    const dim3 grid = ocx_grid(gn, 1), block(64);
    if (cand)
        hipLaunchKernelGGL((ocx_alg_pipe_kernel<C, P, NB, false, true, 4>), grid, block, 0, st, zt,
                           yt, L->B, L->T, L->G, eta0, reg, (double*)nullptr, (double*)nullptr,
                           (int*)nullptr, onepass, g0, gn);
    else if (pipe_fastq(onepass))
        hipLaunchKernelGGL((ocx_alg_pipe_kernel<C, P, NB, false, false, 4, true>), grid, block, 0,
                           st, zt, yt, L->B, L->T, L->G, eta0, reg, (double*)nullptr,
                           (double*)nullptr, (int*)nullptr, onepass, g0, gn);
    else
        hipLaunchKernelGGL((ocx_alg_pipe_kernel<C, P, NB, false, false, 4>), grid, block, 0, st, zt,
                           yt, L->B, L->T, L->G, eta0, reg, (double*)nullptr, (double*)nullptr,
                           (int*)nullptr, onepass, g0, gn);
    return hipGetLastError();
}
}  // namespace

bool ocx_pipe_lean_supported(const ocx_layout* L) {
    return !L->chain && L->T < ((int64_t)1 << 30) && ((L->P == 8 && L->C == 8) || (L->P == 16 && L->C == 4));
}

hipError_t ocx_launch_alg_pipe_lean(const ocx_layout* L, const double* zt, const double* yt,
                                    double eta0, double* reg, int onepass, int64_t g0,
                                    int64_t gn, int cand, hipStream_t st, int vgpr_budget) {
    if (gn <= 0) return hipSuccess;
    if (g0 < 0 || g0 + gn > L->G) return hipErrorInvalidValue;
    if (vgpr_budget >= 168 && L->P == 8 && L->C == 8 && !cand) {
        // the 168-VGPR form (three waves per SIMD's budget) and a seven-slot ring: beside
        // three generator waves of the 96-VGPR form (3 x 96 + 168 <= 512)
        hipLaunchKernelGGL((ocx_alg_pipe_kernel<8, 8, OCX_PIPE_LEAN168_NB, false, false, 3>),
                           ocx_grid(gn, 1), dim3(64), 0, st, zt, yt, L->B, L->T, L->G, eta0, reg,
                           (double*)nullptr, (double*)nullptr, (int*)nullptr, onepass, g0, gn);
        return hipGetLastError();
    }
    if (L->P == 8 && L->C == 8)
        return launch_lean<8, 8>(L, zt, yt, eta0, reg, onepass, g0, gn, cand, st);
    if (L->P == 16 && L->C == 4)
        return launch_lean<4, 16>(L, zt, yt, eta0, reg, onepass, g0, gn, cand, st);
    return hipErrorInvalidValue;
}
