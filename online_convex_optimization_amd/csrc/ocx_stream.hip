// ocx_stream.hip — long-horizon (T-chunked) FTRL/FTL for sweeps whose sequences do not
// fit in HBM at once (configs[3]: T up to 1e5 with 1e6 runs).
//
// The horizon is cut into chunks of Tc steps.  Pass A walks the chunks in order:
// the generator writes chunk c's rows and labels (resuming each stream from its saved
// PCG state) and ocx_alg_chunk_kernel advances theta and the cumulative loss, which
// live in HBM between launches.  Pass B regenerates every chunk from the same saved
// states and accumulates the comparator loss of FTL(theta_T) (fast_algorithms.py:113-114).
// The per-step arithmetic is the same ocx_device_math.h code as ocx_alg_kernel, so the
// regrets are identical to a single-launch run.
#include "ocx_device_math.h"
#include "ocx_dispatch.h"
#include "ocx_internal.h"
#include "ocx_sim_kernels.h"

// mode 0: loop steps [t0, t0+Tc) of fast_algorithms.py:99-111, theta/cum in & out;
//         unclean[b] (nullable) is set to 1 when a step's sub-gradient is not −y_t/2
//         or its row is not inside the unit ball (ocx_row_in_ball).
// mode 1: comparator loss of those steps with x* = FTL(theta_state); when regret_out
//         is non-null (last chunk) also regret = cum - comp (only where unclean[b] != 0
//         when unclean is given: the clean sequences took the closed form in mode 2).
// mode 2: no rows read; for every sequence with unclean[b] == 0 the closed-form
//         comparator loss (ocx_alg_kernel, onepass) t0/2 − ||theta_T|| (t0 = T here)
//         and regret; unclean[B] (one past the sequences) = 1 when any sequence needs
//         the second pass.
template <int C, int P, bool CHAIN, int NB>
__global__ __launch_bounds__(OCX_BLOCK) void ocx_alg_chunk_kernel(
    const double* __restrict__ zt, const double* __restrict__ yt, int64_t B, int64_t Tc,
    int64_t G, int64_t t0, int alg_flag, double eta0, int mode, double* __restrict__ theta_state,
    int64_t Dp, double* __restrict__ cum_state, double* __restrict__ comp_state,
    double* __restrict__ regret_out, double* __restrict__ unclean) {
    constexpr int S = 64 / P;
    constexpr int K = C / 2;
    const int lane = threadIdx.x & 63;
    const int64_t g = ocx_wave_id();
    if (g >= G) return;
    const int s = lane / P;
    const int c = lane % P;
    const int64_t b = g * S + s;
    const bool live = b < B;
    const int64_t tstride = 64;  // ocx_d2 per step within a plane
    const ocx_d2* __restrict__ zp = reinterpret_cast<const ocx_d2*>(zt) + g * Tc * tstride + lane;
    const int64_t kst = G * Tc * 64;  // plane stride (pairs k)
    const double* __restrict__ yp = yt + g * Tc * S + s;
    double* th_row = theta_state + (live ? b : 0) * Dp + (int64_t)c * C;

    double th[C];
#pragma unroll
    for (int j = 0; j < C; ++j) th[j] = live ? th_row[j] : 0.0;

    if (mode == 2) {
        double p[C];
#pragma unroll
        for (int j = 0; j < C; ++j) p[j] = th[j] * th[j];
        const double nrm = sqrt(ocx_total<C, P, CHAIN>(p, lane));
        if (live && c == 0) {
            if (unclean[b] == 0.0) {
                const double comp = 0.5 * (double)t0 - nrm;
                comp_state[b] = comp;
                regret_out[b] = cum_state[b] - comp;
            } else {
                unclean[B] = 1.0;  // plain store of the same value by every writer
            }
        }
        return;
    }

    ocx_d2 zb[NB][K];
    double yb[NB];
#pragma unroll
    for (int u = 0; u < NB - 1; ++u)
        if (u < Tc) {
            ocx_load_tile<C>(zb[u], zp + u * tstride, kst);
            yb[u] = yp[u * S];
        }

    if (mode == 0) {
        const bool ftl = (alg_flag != 0);
        bool clean = true;
        double cum = live ? cum_state[b] : 0.0;
        OcxScaleTable sct;  // FTRL scales, 64 steps at a time (long chains)
        for (int64_t u0 = 0; u0 < Tc; u0 += NB) {
#pragma unroll
            for (int u = 0; u < NB; ++u) {
                const int64_t t = u0 + u;
                if (t < Tc) {
                    const int64_t tp = t + NB - 1;
                    if (tp < Tc) {
                        ocx_load_tile<C>(zb[(u + NB - 1) % NB], zp + tp * tstride, kst);
                        yb[(u + NB - 1) % NB] = yp[tp * S];
                    }
                    double x[C];
                    double q;
                    if (!ftl) {
                        if constexpr (CHAIN && P >= OCX_CHAIN_WIDE_P) {
                            const double sc = ocx_ftrl_scale(sct, t0 + t + 1, eta0, lane);
                            double fr;
                            q = ocx_ftrl_q_sc<C, P, CHAIN>(th, zb[u], sc, fr, lane);
                        } else {
                            const double sc = ocx_ftrl_scale(sct, t0 + t + 1, eta0, lane);
                            q = ocx_ftrl_act_dot_sc<C, P, CHAIN>(th, zb[u], sc, x, lane);
                        }
                    } else {
                        ocx_action_ftl<C, P, CHAIN>(th, x, lane);
                        q = ocx_zdot<C, P, CHAIN>(zb[u], x, lane);
                    }
                    const double diff = q - yb[u];
                    cum += 0.5 * fabs(diff);
                    const double gq = ocx_grad(diff);
                    // closed form: rows certified inside the unit ball (ocx_row_in_ball)
                    if (unclean != nullptr) clean = clean & ocx_row_in_ball<C, P>(zb[u]);
                    clean = clean && fabs(yb[u]) == 1.0 && gq == -0.5 * yb[u];
#pragma unroll
                    for (int j = 0; j < C; ++j) th[j] += gq * ocx_zj(zb[u], j);
                }
            }
        }
        if (live) {
#pragma unroll
            for (int j = 0; j < C; ++j) th_row[j] = th[j];
            if (c == 0) cum_state[b] = cum;
            if (c == 0 && unclean != nullptr && !clean) unclean[b] = 1.0;
        }
    } else {
        double xs[C];
        ocx_action_ftl<C, P, CHAIN>(th, xs, lane);
        double comp = live ? comp_state[b] : 0.0;
        if constexpr (CHAIN && P >= OCX_CHAIN_WIDE_P && P <= 16 && C <= 16) {
            // pairs of steps (its own ring; the one preloaded above goes unused)
            comp = ocx_comp_pass2<C, P, CHAIN, (C <= 8 ? OCX_NB_PASS2 : 4)>(zp, yp, Tc, kst, S, xs, comp, lane);
        } else {
            for (int64_t u0 = 0; u0 < Tc; u0 += NB) {
#pragma unroll
                for (int u = 0; u < NB; ++u) {
                    const int64_t t = u0 + u;
                    if (t < Tc) {
                        const int64_t tp = t + NB - 1;
                        if (tp < Tc) {
                            ocx_load_tile<C>(zb[(u + NB - 1) % NB], zp + tp * tstride, kst);
                            yb[(u + NB - 1) % NB] = yp[tp * S];
                        }
                        double p[C];
#pragma unroll
                        for (int j = 0; j < C; ++j) p[j] = ocx_zj(zb[u], j) * xs[j];
                        const double q = ocx_total_last<C, P, CHAIN>(p, lane);
                        comp += 0.5 * fabs(q - yb[u]);
                    }
                }
            }
            comp = ocx_comp_lane_value<P, CHAIN>(comp, lane);
        }
        if (live && c == 0) {
            comp_state[b] = comp;
            if (regret_out && (unclean == nullptr || unclean[b] != 0.0))
                regret_out[b] = cum_state[b] - comp;
        }
    }
}

namespace {
template <int C, int P, bool CH>
hipError_t launch_chunk_cp(const ocx_layout* L, const double* zt, const double* yt, int64_t t0,
                           int alg_flag, double eta0, int mode, double* th, double* cum,
                           double* comp, double* reg, double* unclean, hipStream_t st) {
    hipLaunchKernelGGL((ocx_alg_chunk_kernel<C, P, CH, nb_for(C, P)>),
                       ocx_grid(L->G, ocx_block_waves(L->G)), dim3(64 * ocx_block_waves(L->G)), 0,
                       st, zt, yt, L->B, L->T, L->G, t0, alg_flag, eta0, mode, th, L->Dp, cum,
                       comp, reg, unclean);
    return hipGetLastError();
}
}  // namespace

hipError_t ocx_launch_alg_chunk(const ocx_layout* L, const double* zt, const double* yt,
                                int64_t t0, int alg_flag, double eta0, int mode, double* theta,
                                double* cum, double* comp, double* regret, hipStream_t st,
                                double* unclean) {
    if (L->G == 0 || (L->T == 0 && mode != 2)) return hipSuccess;
    OCX_DISPATCH(launch_chunk_cp, L, zt, yt, t0, alg_flag, eta0, mode, theta, cum, comp, regret,
                 unclean, st)
}
