// ocx_smart_closed.hip — SMART (fast_algorithms.py:118-164) in O(T·d) per sequence.
//
// The reference's SMART re-scans the whole prefix before the switch: at every step t it
// sums ½|z_i·s_t − y_i| over i = 0..t (`_comparator_loss_prefix`, :79-85, called at
// :158), O(T²·d) per sequence, and compares ftl_loss − s_loss with the threshold (:159).
// On the reference's own data that prefix loss has a closed form.  When every row so far
// lies in the unit ball (||z_i|| <= 1: the g(T) sampler and the random families clip
// them) and every label is ±1, |z_i·s_t| <= 1 for the unit-norm FTL action s_t, so
// ½|z_i·s_t − y_i| = ½(1 − y_i z_i·s_t) and
//
//     s_loss_t = (t+1)/2 − ½ s_t·S_t,   S_t = Σ_{i<=t} y_i z_i,
//
// one dot product per step with S_t kept beside theta in registers.  The closed form
// differs from the reference's sequential sum only by rounding, so it DECIDES the switch
// only where ftl_loss − s_loss is farther from the threshold than a bound on that
// rounding (`guard` below); inside the band, or once a row leaves the ball or a label is
// not ±1, the step re-scans its prefix exactly as the reference does.  The switch step
// is therefore the reference's (bit-identical decisions in the exact layouts), and the
// regret — total_loss minus the comparator loss, both summed as the reference does —
// is unchanged.
//
// Guard (u = 2^-53): the reference's prefix sum differs from the exact value of
// Σ ½|z_i·s_t − y_i| by at most (t+1)·u·(t + d/2 + 2) (d-term dot products, t+1 ordered
// adds of terms <= 1); that value differs from the closed form's exact value by at most
// (t+1)·(5e-13 + (d/2 + 4)·u) (rows certified to ||z||² <= 1 + 1e-12, ||s_t|| <= 1 + a few
// u); the computed closed form differs from its exact value by at most (t+1)·u·(t + d + 1)
// (S_t's sums, the dot, the final subtraction); the decision's own subtractions add
// 2u·(|ftl_loss| + |s| + |thresh|).  The band below is about twice their sum.
//
// The final comparator FTL(theta_ftl) (:162-163) is streamed as the reference does, or —
// closed_comp, not in the bit-exact APIs — taken in closed form T/2 − ||theta_ftl|| where
// every FTL sub-gradient was −y_t/2 (then theta_ftl = −½ S_T; see ocx_alg_kernel's
// onepass comparator), which makes the whole kernel one HBM pass.
#include "ocx_device_math.h"
#include "ocx_dispatch.h"
#include "ocx_internal.h"
#include "ocx_sim_kernels.h"

template <int C, int P, bool CHAIN, int NB>
__global__ __launch_bounds__(OCX_BLOCK) void ocx_smart_closed_kernel(
    const double* __restrict__ zt, const double* __restrict__ yt, int64_t B, int64_t T,
    int64_t d, int64_t G, const double* __restrict__ thresh, double eta0,
    double* __restrict__ regret, int64_t* __restrict__ switch_step, int closed_prefix,
    int closed_comp, unsigned long long* __restrict__ stats) {
    constexpr int S = 64 / P;
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

    // theta_ftl, theta_ftrl, S_t = Σ y_i z_i, and FTL(theta_ftl) as it stands (the next
    // step's FTL action and this step's s_t)
    double tf[C], tr[C], sv[C], xf[C];
#pragma unroll
    for (int j = 0; j < C; ++j) tf[j] = tr[j] = sv[j] = xf[j] = 0.0;
    bool switched = (b >= B);  // padding sequences never scan
    int64_t sw = -1;
    bool regime = true;  // every row so far in the unit ball, every label ±1
    bool clean = true;   // ... and every FTL sub-gradient −y_t/2 (closed comparator)
    double ftl_loss = 0.0, total_loss = 0.0;
    unsigned long long rescans = 0;

    ocx_d2 zb[NB][C / 2];
    double yb[NB];
#pragma unroll
    for (int u = 0; u < NB - 1; ++u)
        if (u < T) {
            ocx_load_tile<C>(zb[u], zp + u * tstride, kst);
            yb[u] = yp[u * S];
        }

    for (int64_t t0 = 0; t0 < T; t0 += NB) {
#pragma unroll
        for (int u = 0; u < NB; ++u) {
            const int64_t t = t0 + u;
            if (t < T) {
                const int64_t tp = t + NB - 1;
                if (tp < T) {
                    ocx_load_tile<C>(zb[(u + NB - 1) % NB], zp + tp * tstride, kst);
                    yb[(u + NB - 1) % NB] = yp[tp * S];
                }
                const double yv = yb[u];
                // FTL is always run and updated (:140-146)
                const double pf = ocx_zdot<C, P, CHAIN>(zb[u], xf, lane);
                const double dfl = pf - yv;
                const double gfl = ocx_grad(dfl);
#pragma unroll
                for (int j = 0; j < C; ++j) tf[j] += gfl * ocx_zj(zb[u], j);
                const double lf = 0.5 * fabs(dfl);
                ftl_loss += lf;
                // whole wave active: the certification sums across lanes
                const bool rowok = ocx_row_in_ball<C, P>(zb[u]) && fabs(yv) == 1.0;
                regime = regime && rowok;
                clean = clean && rowok && gfl == -0.5 * yv;
#pragma unroll
                for (int j = 0; j < C; ++j) sv[j] += yv * ocx_zj(zb[u], j);  // exact: y = ±1
                ocx_action_ftl<C, P, CHAIN>(tf, xf, lane);                 // s_t (:157)
                if (switched) {
                    // post-switch: FTRL with its own theta and the global t (:148-154); the
                    // scale per step (ocx_ftrl_scale's table is wave-wide, this branch is not)
                    const double sc = -(eta0 / sqrt((double)(t + 1)));
                    double x[C];
                    const double pr = ocx_ftrl_act_dot_sc<C, P, CHAIN>(tr, zb[u], sc, x, lane);
                    const double dr = pr - yv;
                    total_loss += 0.5 * fabs(dr);
                    const double gr = ocx_grad(dr);
#pragma unroll
                    for (int j = 0; j < C; ++j) tr[j] += gr * ocx_zj(zb[u], j);
                } else {
                    total_loss += lf;  // :156
                    bool decided = false, fire = false;
                    if (closed_prefix && ftl_loss < th_sw) {
                        // s_loss >= 0, so fl(ftl_loss - s_loss) <= ftl_loss < thresh: the
                        // reference's test is false whatever the prefix (any thresh, +inf too)
                        decided = true;
                    } else if (closed_prefix && regime) {
                        double p[C];
#pragma unroll
                        for (int j = 0; j < C; ++j) p[j] = xf[j] * sv[j];
                        const double dot = ocx_total<C, P, CHAIN>(p, lane);
                        const double n1 = (double)(t + 1);
                        const double s_cl = 0.5 * n1 - 0.5 * dot;
                        const double D = ftl_loss - s_cl - th_sw;
                        // an infinite threshold must not widen the band (+inf: never fires,
                        // D = -inf; -inf: fires at once, D = +inf), and a NaN one never fires
                        // (`>= NaN` is false, :159) — decided here, not by O(t) re-scans
                        const double tha = __builtin_isfinite(th_sw) ? fabs(th_sw) : 0.0;
                        const double guard =
                            n1 * (1e-12 + 2.5e-16 * (2.0 * n1 + 2.0 * (double)d + 8.0)) +
                            4e-16 * (fabs(ftl_loss) + n1 + tha);
                        if (th_sw != th_sw) {
                            decided = true;
                            fire = false;
                        } else if (fabs(D) > guard) {
                            decided = true;
                            fire = D > 0.0;
                        }
                    }
                    if (!decided) {
                        // the reference's prefix re-scan (:157-160, :79-85)
                        ++rescans;
                        double s_loss = 0.0;
                        for (int64_t i = 0; i <= t; ++i) {
                            ocx_d2 zi[C / 2];
                            ocx_load_tile<C>(zi, zp + i * tstride, kst);
                            const double q = ocx_zdot<C, P, CHAIN>(zi, xf, lane);
                            s_loss += 0.5 * fabs(q - yp[i * S]);
                        }
                        fire = ftl_loss - s_loss >= th_sw;
                    }
                    if (fire) {
                        switched = true;
                        sw = t;
                    }
                }
            }
        }
    }

    // final comparator = FTL(theta_ftl) (:162-163) = xf
    const bool closed = closed_comp && (clean || b >= B);
    double comp = 0.0;
    if (__ballot(!closed) != 0) {  // wave-uniform: stream the second pass
#pragma unroll
        for (int u = 0; u < NB - 1; ++u)
            if (u < T) {
                ocx_load_tile<C>(zb[u], zp + u * tstride, kst);
                yb[u] = yp[u * S];
            }
        for (int64_t t0 = 0; t0 < T; t0 += NB) {
#pragma unroll
            for (int u = 0; u < NB; ++u) {
                const int64_t t = t0 + u;
                if (t < T) {
                    const int64_t tp = t + NB - 1;
                    if (tp < T) {
                        ocx_load_tile<C>(zb[(u + NB - 1) % NB], zp + tp * tstride, kst);
                        yb[(u + NB - 1) % NB] = yp[tp * S];
                    }
                    double p[C];
#pragma unroll
                    for (int j = 0; j < C; ++j) p[j] = ocx_zj(zb[u], j) * xf[j];
                    const double q = ocx_total_last<C, P, CHAIN>(p, lane);
                    comp += 0.5 * fabs(q - yb[u]);
                }
            }
        }
        comp = ocx_comp_lane_value<P, CHAIN>(comp, lane);
    }
    if (__ballot(closed) != 0) {
        double p[C];
#pragma unroll
        for (int j = 0; j < C; ++j) p[j] = tf[j] * tf[j];
        const double nrm = sqrt(ocx_total<C, P, CHAIN>(p, lane));
        if (closed) comp = 0.5 * (double)T - nrm;
    }
    if (c == 0 && b < B) {
        regret[b] = total_loss - comp;
        if (switch_step) switch_step[b] = sw;
        if (stats) {
            if (rescans) atomicAdd(&stats[0], rescans);
            if (closed) atomicAdd(&stats[1], 1ULL);
        }
    }
}

namespace {
template <int C, int P, bool CH>
hipError_t launch_smart_closed_cp(const ocx_layout* L, const double* zt, const double* yt,
                                  const double* th, double eta0, double* reg, int64_t* sw,
                                  int closed_prefix, int closed_comp, unsigned long long* stats,
                                  hipStream_t st) {
    hipLaunchKernelGGL((ocx_smart_closed_kernel<C, P, CH, nb_for(C, P, false)>),
                       ocx_grid(L->G, ocx_block_waves(L->G)), dim3(64 * ocx_block_waves(L->G)), 0,
                       st, zt, yt, L->B, L->T, L->d, L->G, th, eta0, reg, sw, closed_prefix,
                       closed_comp, stats);
    return hipGetLastError();
}
}  // namespace

hipError_t ocx_launch_smart_closed(const ocx_layout* L, const double* zt, const double* yt,
                                   const double* th, double eta0, double* reg, int64_t* sw,
                                   int closed_prefix, int closed_comp, unsigned long long* stats,
                                   hipStream_t st) {
    if (L->G == 0) return hipSuccess;
    OCX_DISPATCH(launch_smart_closed_cp, L, zt, yt, th, eta0, reg, sw, closed_prefix, closed_comp,
                 stats, st)
}
