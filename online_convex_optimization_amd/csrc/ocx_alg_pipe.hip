// ocx_alg_pipe.hip — FTRL/FTL (fast_algorithms.py:88-115) for the butterfly-sum layouts
// (P >= 2 lanes per sequence, chain = 0) with the step's dependency chain cut short.
//
// In the plain kernel (ocx_sim.hip) step t waits for g_{t-1}, then forms x = sθ_t, sums
// ||x||² and z_t·x lane by lane (C dependent adds each), crosses the P lanes, and — when
// the FTRL action is rescaled — sums z_t·x a second time: about 60 dependent fp64
// operations, ≈1 100 cycles per step.  A few-wave batch (capacity-limited long horizons:
// d = 64, T = 1e5, ≈4 900 sequences, one wave per SIMD) cannot hide that, so its time is
// T × that latency.
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
//
// Chunked runs (the trailing pipeline, ocx_pipeline.hip): a launch may cover steps
// [t0, t0 + tn) of the horizon only (t0 a multiple of 64), carrying the step's whole state —
// θ_{t-1}, z_{t-1}, the lane partials A, Bz, V, W, g_{t-1}, the loss and the `clean` flag —
// through HBM between launches.  U and the FTRL scales are re-formed at the chunk's first
// step (a multiple of 64: their periodic refresh), so a chunked run is the whole run, bit for
// bit.  The rows before t0 may already hold the next batch, so a chunked run never streams
// the second comparator pass: a sequence the closed form cannot certify gets a NaN regret
// and raises *bad (the caller runs its batch again in the sequential path).
#include <cmath>
#include <cstdlib>
#include <type_traits>

#include "ocx_device_math.h"
#include "ocx_internal.h"
#include "ocx_sim_kernels.h"

// The step counter's type (ocx_ring_loop): int keeps the loop tests on the scalar unit; used
// for C <= OCX_PIPE_IT32_MAXC coordinates per lane.  Measured (r04_pipe_ab1.jsonl): the 16 x 4
// few-wave batch 35.5 -> 32.4 ms with it, while the 8 x 8 kernel's loads were scheduled with
// shallower waits and it ran 40.2 -> 42.0 ms, so 8 x 8 keeps the int64_t counter.
#ifndef OCX_PIPE_IT32_MAXC
#define OCX_PIPE_IT32_MAXC 4
#endif
#ifndef OCX_PIPE_WAVE_CLOCK  // diagnostic build: per-wave clocks instead of cum / comp (below)
#define OCX_PIPE_WAVE_CLOCK 0
#endif

// Per-lane state words of a chunked run (see the header): θ_{t-1} [C], z_{t-1} [C], then
// A, Bz, V, W, g_{t-1}, cum, clean.  Stored word-major per wave-group: word i of lane l of
// group g at state[(g·NS + i)·64 + l], so each word is one coalesced 512-B access.
constexpr int pipe_state_words(int C) { return 2 * C + 7; }

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

// Launch arguments of the kernel (one struct: the launchers below forward it unchanged).
struct PipeArgs {
    const double* zt;
    const double* yt;
    int64_t B, T, G;
    double eta0;
    double* regret;
    double* cum_out;
    double* comp_out;
    int* closed_out;
    int onepass;
    int64_t g0, gn;  // wave-groups [g0, g0 + gn) of the layout
    int64_t t0, tn;  // steps [t0, t0 + tn) (a whole run: 0, T)
    double* state;   // chunked runs: the carried state (nullable: whole run)
    int* bad;        // chunked runs: set when a sequence needs the second pass
    unsigned long long* gmax;  // nullable: g(T) = max(0, max regret) folded in (bit pattern)
};

// RT (FTRL): the rescale's sqrt only in waves where a sequence may need the rescale (see the
// step).  CHUNK: a chunked run (t0, tn, state); the whole-run kernels compile without it, so
// its bookkeeping costs them no registers (the lean form spilled with it: 148 B per lane).
template <int C, int P, int NB, bool FTL, bool RT, bool CHUNK = false>
__device__ __forceinline__ void alg_pipe_body(const PipeArgs& a) {
    static_assert(P >= 2 && NB >= 4, "butterfly layouts, a ring holding z_{t-1} .. z_{t+1}");
    using IT = typename std::conditional<(C <= OCX_PIPE_IT32_MAXC), int, int64_t>::type;
    constexpr int S = 64 / P;
    constexpr int K = C / 2;
    constexpr int NS = pipe_state_words(C);
    const int lane = threadIdx.x & 63;
    // wave-uniform, provably (readfirstlane): the tile bases live in SGPRs and every load
    // is an SGPR base + the lane's constant offset, with no per-load address arithmetic
    const int64_t wv = (int64_t)__builtin_amdgcn_readfirstlane((int)ocx_pipe_wave_id(a.gn));
    if (wv >= a.gn) return;
    const int64_t g = a.g0 + wv;
    const int64_t T = a.T, t0 = CHUNK ? a.t0 : 0, tn = CHUNK ? a.tn : T;
    const bool first = !CHUNK || t0 == 0, last = !CHUNK || t0 + tn >= T;
    const double eta0 = a.eta0;
#if OCX_PIPE_WAVE_CLOCK  // diagnostic build only: see the end of the body
    const uint64_t clk0 = __builtin_amdgcn_s_memrealtime();
#endif
    const int s = lane / P;
    const int c = lane % P;
    const int64_t b = g * S + s;
    // The layout's padding sequences (b >= B, the last wave-group's spare slots) have all-zero
    // rows, so their θ stays 0 and FTL's near-origin re-sum below would run for them at every
    // step — in the one wave that holds them, which then set the launch's time (a 47.6 ms
    // straggler among 41–42 ms waves on the 4 900 x 1e5 batch, profiles/r04_wave_clock*.jsonl).
    // Their results are never written, so they skip it.
    const bool live = b < a.B;
    const int64_t tstride = 64;  // ocx_d2 per step within a plane
    // this chunk's first row
    const ocx_d2* __restrict__ zg = reinterpret_cast<const ocx_d2*>(a.zt) + (g * T + t0) * tstride;
    const int64_t kst = a.G * T * 64;  // plane stride (pairs k)
    const double* __restrict__ yg = a.yt + (g * T + t0) * S;
    // word i of this lane's carried state (formed where used: nothing stays live over the loop)
    auto stw = [&](int i) -> double& { return a.state[(g * NS + i) * 64 + lane]; };

    double th[C];  // θ_{t-1} (lagging one update)
    double gp = 0.0;                                   // g_{t-1}
    double A = 0.0, Bz = 0.0, U = 0.0, V = 0.0, W = 0.0;  // step t's lane partials
    double cum = 0.0;
    bool clean = true;  // onepass: rows in the ball, every sub-gradient −y_t/2

    // z_{t-1} is read where it lies, in the slot before step t's: the late loads
    // (ocx_ring_loop<NB, true>) refill that slot only after step t.  At t = 0 that slot is
    // zero (g_{-1} = 0 multiplies it); a later chunk restores z_{t0-1} there.
    ocx_d2 zb[NB][K];
    double yb[NB];
    if (first) {
#pragma unroll
        for (int j = 0; j < C; ++j) th[j] = 0.0;
#pragma unroll
        for (int k = 0; k < K; ++k) zb[NB - 1][k] = ocx_d2{0.0, 0.0};
    } else if constexpr (CHUNK) {
#pragma unroll
        for (int j = 0; j < C; ++j) th[j] = stw(j);
#pragma unroll
        for (int k = 0; k < K; ++k) zb[NB - 1][k] = ocx_d2{stw(C + 2 * k), stw(C + 2 * k + 1)};
        A = stw(2 * C);
        Bz = stw(2 * C + 1);
        V = stw(2 * C + 2);
        W = stw(2 * C + 3);
        gp = stw(2 * C + 4);
        cum = stw(2 * C + 5);
        clean = stw(2 * C + 6) != 0.0;
    }
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
        yb[slot] = yg[tl * S + s];
    };
    double scv = 0.0;  // −η0/√(t+1+lane) for the 64 steps from the last multiple of 64

    ocx_ring_loop<NB, true, IT>(tn, load, [&](int u, int64_t tl) {
        const int64_t t = t0 + tl;
        // every 64 steps: the FTRL scales of the next 64 steps (one per lane, one sqrt/div
        // per lane instead of one per step) and ||θ||²'s lane part summed afresh, so the
        // running update below drifts for at most 64 steps
        if ((tl & 63) == 0) {
            if constexpr (!FTL) scv = -(eta0 / sqrt((double)(t + 1 + lane)));
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
            const double sc = ocx_readlane(scv, (int)(tl & 63));  // −η0/√(t+1)
            const double qa = sc * q_raw;
            // RT: no sequence of the wave near the rescale (s²||θ||² < 1 − 1e-12, far outside
            // the rounding of the test below): q = s·(z·θ), without the sqrt the test below
            // needs — what the test below would give, bit for bit.  On the g(T) rows ||sθ||
            // stays near 0.71 and the rescale is rare.
            if (RT && __ballot(sc * sc * n_raw >= 1.0 - 1e-12) == 0) {
                q = qa;
            } else {
                const double s_abs = fabs(sc) * sqrt(n_raw > 0.0 ? n_raw : 0.0);
                q = s_abs > 1.0 ? qa * (1.0 / s_abs) : qa;
            }
        } else {
            if (n_raw < 0.25 && live) {  // near θ = 0: re-sum directly (see above)
                double p[C];
#pragma unroll
                for (int j = 0; j < C; ++j) p[j] = th[j] * th[j];
                tth = ocx_lane_sum<C>(p);
                n_raw = ocx_seq_sum<P>(tth);
            }
            q = n_raw == 0.0 ? 0.0 : (-(1.0 / sqrt(n_raw))) * q_raw;
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
        if (ocx_check_rows(a.onepass)) clean = clean & (ocx_seq_sum<P>(w) <= 1.0 + 1e-12);  // row t in ball
        // (at t = T-1, zn is the clamped look-ahead: A and Bz are then never used)
        V = zth;
        W = w;
        U = tth;  // ||θ_t||²'s lane part, by the running update
        A = an;
        Bz = bn;
        gp = gq;
    }, CHUNK ? T - t0 : T);
    // the chunk's last row: z_{t1-1} for the next chunk, or z_{T-1} for θ_T (loaded again:
    // its ring slot is not known at compile time)
    ocx_d2 zl[K];
    if (tn > 0) ocx_load_tile<C>(zl, zg + (tn - 1) * tstride + lane, kst);
    if constexpr (CHUNK) if (!last) {
#pragma unroll
        for (int j = 0; j < C; ++j) stw(j) = th[j];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            stw(C + 2 * k) = zl[k].x;
            stw(C + 2 * k + 1) = zl[k].y;
        }
        stw(2 * C) = A;
        stw(2 * C + 1) = Bz;
        stw(2 * C + 2) = V;
        stw(2 * C + 3) = W;
        stw(2 * C + 4) = gp;
        stw(2 * C + 5) = cum;
        stw(2 * C + 6) = clean ? 1.0 : 0.0;
        return;
    }
    // θ_T = θ_{T-1} + g_{T-1} z_{T-1}
    if (tn > 0) {
#pragma unroll
        for (int j = 0; j < C; ++j) th[j] = __builtin_fma(gp, ocx_zj(zl, j), th[j]);
    }

    // ---- comparator: closed form where certified (ocx_alg_kernel onepass), else the
    // reference's second streaming pass with x* = FTL(θ_T) (fast_algorithms.py:113-114) —
    // which a chunked run (t0 > 0: the early rows may hold the next batch) cannot stream
    const bool closed = a.onepass && (clean || !live);
    double comp = 0.0;
    if (__ballot(!closed) != 0) {  // wave-uniform
        if (first) {  // zg, yg: row 0
            double xs[C];
            ocx_action_ftl<C, P, false>(th, xs, lane);
            ocx_ring_loop<NB, false, IT>(T, load, [&](int u, int64_t) {
                double p[C];
#pragma unroll
                for (int j = 0; j < C; ++j) p[j] = ocx_zj(zb[u], j) * xs[j];
                const double qq = ocx_total<C, P, false>(p, lane);
                comp += 0.5 * fabs(qq - yb[u]);
            });
        } else if constexpr (CHUNK) {
            comp = __builtin_nan("");
            if (!closed && c == 0 && a.bad) *a.bad = 1;
        }
    }
    if (__ballot(closed) != 0) {
        double p[C];
#pragma unroll
        for (int j = 0; j < C; ++j) p[j] = th[j] * th[j];
        const double nrm = sqrt(ocx_total<C, P, false>(p, lane));
        if (closed) comp = 0.5 * (double)T - nrm;
    }
    // g(T) folded in here (the pipelines' FTRL launches): a max over the wave's sequences,
    // then one 64-bit atomic max of the bit pattern per wave — positive doubles order as
    // their bits, every candidate that can win is > +0.0 and a NaN never passes `>`, so this
    // is ocx_max_fold_kernel's selection, bit-identical to the host's loop, without a
    // separate launch that would wait for a free slot beside the generator (2-3 ms each).
    if (a.gmax && __ballot(live) != 0) {  // wave-uniform
        const double rg = cum - comp;
        double mv = (c == 0 && live && rg > 0.0) ? rg : 0.0;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            const double u = __shfl_xor(mv, o, 64);
            if (u > mv) mv = u;
        }
        if (lane == 0 && mv > 0.0) atomicMax(a.gmax, (unsigned long long)__double_as_longlong(mv));
    }
    if (c == 0 && live) {
        if (a.regret) a.regret[b] = cum - comp;
#if OCX_PIPE_WAVE_CLOCK
        // diagnostic build (tools/wave_clock_probe.py): the wave's duration in ticks of the
        // 100 MHz real-time clock, and where it ran (HW_ID, XCC_ID) — not results
        const uint64_t clk1 = __builtin_amdgcn_s_memrealtime();
        if (a.cum_out) a.cum_out[b] = (double)(clk1 - clk0);
        if (a.comp_out) a.comp_out[b] = (double)clk0;
        if (a.closed_out)
            a.closed_out[b] = (int)((__builtin_amdgcn_s_getreg((31 << 11) | 4) & 0xffffu) |
                                    ((__builtin_amdgcn_s_getreg((31 << 11) | 20) & 0xfu) << 16));
#else
        if (a.cum_out) a.cum_out[b] = cum;
        if (a.comp_out) a.comp_out[b] = comp;
        if (a.closed_out) a.closed_out[b] = closed ? 1 : 0;
#endif
    }
}

// The rescale test (RT) per kernel: measured (profiles/r04_pipe_ab3.jsonl) 3 328 x 1e5 at
// 16 x 4: 32.5 -> 28.7 ms; the pipeline's lean 8 x 8 form: 66.7 -> 64.3 ms per batch; but the
// 8 x 8 full form (the T = 1e5 batch): 40.8 -> 43.6 ms, which keeps the sqrt.
template <int C, int P, int MINW>
constexpr bool pipe_rt() {
    return !(C == 8 && P == 8 && MINW == 1);
}
template <int C, int P, int NB, bool FTL, int MINW = 1, bool CHUNK = false>
__global__ __launch_bounds__(OCX_BLOCK, MINW) void ocx_alg_pipe_kernel(PipeArgs a) {
    alg_pipe_body<C, P, NB, FTL, pipe_rt<C, P, MINW>(), CHUNK>(a);
}

namespace {
// Waves per block of the full-form launch: four (one wave per SIMD of a CU, the last blocks
// three, ocx_pipe_wave_id) unless OCX_BLOCK_WAVES forces another shape or the launch has
// fewer than four groups.  The few-wave batches measured one-wave blocks (which the plain
// kernels keep below eight waves per CU) slower: profiles/r04_pipe_bw_ab.jsonl,
// r04_wave_clock*.jsonl.
int pipe_block_waves(int64_t G) {
    if (std::getenv("OCX_BLOCK_WAVES")) return ocx_block_waves(G);
    return G >= 4 ? 4 : 1;
}

template <int C>
constexpr int pipe_nb(int P) {
    // z_{t-1} .. z_{t+1} must be in the ring, and the late loads (ocx_ring_loop) keep NB-2
    // steps in flight: one slot more than the plain kernel's ring
    return nb_for(C, P) + 1 < 4 ? 4 : nb_for(C, P) + 1;
}

template <int C, int P>
hipError_t launch_pipe_cp(const PipeArgs& a, int ftl, hipStream_t st) {
    constexpr int NB = pipe_nb<C>(P);
    const int bw = pipe_block_waves(a.gn);
    const dim3 grid = ocx_grid(a.gn, bw), block(64 * bw);
    if (a.state)  // a chunked run (FTRL: the trailing pipeline's algorithm)
        hipLaunchKernelGGL((ocx_alg_pipe_kernel<C, P, NB, false, 1, true>), grid, block, 0, st, a);
    else if (ftl)
        hipLaunchKernelGGL((ocx_alg_pipe_kernel<C, P, NB, true>), grid, block, 0, st, a);
    else
        hipLaunchKernelGGL((ocx_alg_pipe_kernel<C, P, NB, false>), grid, block, 0, st, a);
    return hipGetLastError();
}

template <int C>
hipError_t launch_pipe_c(int P, const PipeArgs& a, int ftl, hipStream_t st) {
    switch (P) {
        case 8: return launch_pipe_cp<C, 8>(a, ftl, st);
        case 16: return launch_pipe_cp<C, 16>(a, ftl, st);
        case 32: return launch_pipe_cp<C, 32>(a, ftl, st);
        case 64:  // one sequence per wave: d = 1024 at 16 coordinates per lane only
            if constexpr (C == 16) return launch_pipe_cp<16, 64>(a, ftl, st);
            return hipErrorInvalidValue;
        default: return hipErrorInvalidValue;
    }
}

hipError_t launch_pipe(const ocx_layout* L, const PipeArgs& a, int ftl, hipStream_t st) {
    if (a.gn <= 0) return hipSuccess;
    switch (L->C) {
        case 4: return launch_pipe_c<4>(L->P, a, ftl, st);
        case 8: return launch_pipe_c<8>(L->P, a, ftl, st);
        case 16: return launch_pipe_c<16>(L->P, a, ftl, st);
        case 32: return launch_pipe_c<32>(L->P, a, ftl, st);
        default: return hipErrorInvalidValue;
    }
}

PipeArgs pipe_args(const ocx_layout* L, const double* zt, const double* yt, double eta0,
                   double* reg, double* cum, double* comp, int* closed_out, int onepass) {
    PipeArgs a{};
    a.zt = zt;
    a.yt = yt;
    a.B = L->B;
    a.T = L->T;
    a.G = L->G;
    a.eta0 = eta0;
    a.regret = reg;
    a.cum_out = cum;
    a.comp_out = comp;
    a.closed_out = closed_out;
    a.onepass = onepass;
    a.g0 = 0;
    a.gn = L->G;
    a.t0 = 0;
    a.tn = L->T;
    return a;
}
}  // namespace

// The pipelined step pays where one wave's step latency sets the batch time: the few-wave
// butterfly layouts OCX_LANES_BEST chooses (8 x 8, 16 x 4 at d = 64; 16 x 16; 32 x 32 at
// d = 1024) and their neighbours, and 64 x 16 at d = 1024 (lanes_per_seq = 64: 17.4 vs 19.2-19.7 ms
// for the 32 x 32 layout's pass over 2 688 x 5 000 steps, profiles/r05_genscale.jsonl).  Other
// butterfly layouts keep the plain kernel.
bool ocx_pipe_supported(const ocx_layout* L) {
    // T < 2^30: the step counter is a 32-bit int (ocx_ring_loop<..., int>)
    return !L->chain && L->T < ((int64_t)1 << 30) &&
           (((L->P == 8 || L->P == 16 || L->P == 32) &&
             (L->C == 4 || L->C == 8 || L->C == 16 || L->C == 32)) ||
            (L->P == 64 && L->C == 16));
}

hipError_t ocx_launch_alg_pipe(const ocx_layout* L, const double* zt, const double* yt, int ftl,
                               double eta0, double* reg, double* cum, double* comp,
                               int* closed_out, int onepass, hipStream_t st) {
    if (L->G == 0) return hipSuccess;
    return launch_pipe(L, pipe_args(L, zt, yt, eta0, reg, cum, comp, closed_out, onepass), ftl, st);
}

int64_t ocx_pipe_state_doubles(const ocx_layout* L) {
    return L->G * 64 * (int64_t)pipe_state_words(L->C);
}

// The lean form (ocx_pipeline.hip: the FTRL side of both pipelines): at most 128 VGPRs, so
// one wave fits on a SIMD beside four generator waves of the 96-VGPR form (the sub-batch
// pipeline) or four of the 80-VGPR few-stream form (the trailing pipeline); a shorter ring
// (OCX_PIPE_LEAN_NB8 / _NB4 slots at 8 / 4 coordinates per lane) is what makes it fit.  FTRL
// only, the pipelines' algorithm; 8 x 8 and 16 x 4 layouts.  One-wave blocks: the dispatcher
// spreads them over the SIMDs the generator leaves room on.
#ifndef OCX_PIPE_LEAN_NB8
#define OCX_PIPE_LEAN_NB8 4
#endif
#ifndef OCX_PIPE_LEAN_NB4
#define OCX_PIPE_LEAN_NB4 8
#endif
bool ocx_pipe_lean_supported(const ocx_layout* L) {
    return !L->chain && L->T < ((int64_t)1 << 30) && ((L->P == 8 && L->C == 8) || (L->P == 16 && L->C == 4));
}

// The layouts the lean form is built for beyond the trailing pipeline's: 8 x 4 (d = 32's
// g(T) layout in the sub-batch pipeline, round 6).
bool ocx_pipe_lean_launchable(const ocx_layout* L) {
    return ocx_pipe_lean_supported(L) || (!L->chain && L->T < ((int64_t)1 << 30) && L->P == 8 && L->C == 4);
}

namespace {
hipError_t launch_lean(const ocx_layout* L, const PipeArgs& a, hipStream_t st) {
    const dim3 grid = ocx_grid(a.gn, 1), block(64);
    if (L->P == 8 && L->C == 4 && !a.state) {
        hipLaunchKernelGGL((ocx_alg_pipe_kernel<4, 8, OCX_PIPE_LEAN_NB4, false, 4>), grid, block, 0, st, a);
    } else if (L->P == 8 && L->C == 8) {
        if (a.state)
            hipLaunchKernelGGL((ocx_alg_pipe_kernel<8, 8, OCX_PIPE_LEAN_NB8, false, 4, true>), grid, block, 0, st, a);
        else
            hipLaunchKernelGGL((ocx_alg_pipe_kernel<8, 8, OCX_PIPE_LEAN_NB8, false, 4>), grid, block, 0, st, a);
    } else if (L->P == 16 && L->C == 4) {
        if (a.state)
            hipLaunchKernelGGL((ocx_alg_pipe_kernel<4, 16, OCX_PIPE_LEAN_NB4, false, 4, true>), grid, block, 0, st, a);
        else
            hipLaunchKernelGGL((ocx_alg_pipe_kernel<4, 16, OCX_PIPE_LEAN_NB4, false, 4>), grid, block, 0, st, a);
    } else {
        return hipErrorInvalidValue;
    }
    return hipGetLastError();
}
}  // namespace

hipError_t ocx_launch_alg_pipe_lean(const ocx_layout* L, const double* zt, const double* yt,
                                    double eta0, double* reg, int onepass, int64_t g0,
                                    int64_t gn, unsigned long long* gmax, hipStream_t st) {
    if (gn <= 0) return hipSuccess;
    if (g0 < 0 || g0 + gn > L->G) return hipErrorInvalidValue;
    PipeArgs a = pipe_args(L, zt, yt, eta0, reg, nullptr, nullptr, nullptr, onepass);
    a.g0 = g0;
    a.gn = gn;
    a.gmax = gmax;
    return launch_lean(L, a, st);
}

// Chunked runs take the lean form where the layout has one (the trailing pipeline's
// layouts: it runs beside the generator), the full form otherwise (tests of other layouts).
hipError_t ocx_launch_alg_pipe_chunk(const ocx_layout* L, const double* zt, const double* yt,
                                     double eta0, double* reg, int onepass, int64_t t0,
                                     int64_t tn, double* state, int* bad,
                                     unsigned long long* gmax, hipStream_t st) {
    if (L->G == 0 || tn <= 0) return hipSuccess;
    // onepass only: a chunk after the first cannot stream the second comparator pass
    if (t0 < 0 || t0 % 64 != 0 || t0 + tn > L->T || !state || !onepass || !ocx_pipe_supported(L))
        return hipErrorInvalidValue;
    PipeArgs a = pipe_args(L, zt, yt, eta0, reg, nullptr, nullptr, nullptr, onepass);
    a.t0 = t0;
    a.tn = tn;
    a.state = state;
    a.bad = bad;
    a.gmax = t0 + tn >= L->T ? gmax : nullptr;  // the chunk that writes the regrets
    return ocx_pipe_lean_supported(L) ? launch_lean(L, a, st) : launch_pipe(L, a, 0, st);
}
