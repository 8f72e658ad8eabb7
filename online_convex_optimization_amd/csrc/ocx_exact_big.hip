// ocx_exact_big.hip — the general exact-FTL comparator (ExactFTLNoClip, exact_ftl.py:83-105,
// solved by cvxpy at :119-128) for 64 < d <= 256: the path of ocx_exact_wide.hip (same
// barrier, schedule, damping, certificate and certificate polish) for a Newton system that no
// longer fits LDS (DP = 256: 514 KB).
//
// One wavefront per problem (sequence b, prefix n), persistent over the problems (block k
// takes p = k, k + grid, ...), DP = 64·Q padded coordinates (Q = 2, 4):
//   * coordinate vectors live Q per lane: coordinate lane + 64 q in slot q;
//   * rows are staged through LDS RC = 32 at a time; the Hessian Σ_i h_i a_i a_iᵀ is formed one
//     64 × 64 tile at a time (lane 8·bj + bk owning an 8 × 8 block, the DP = 64 grid of
//     ocx_exact_wide.hip), one pass over the prefix's rows per lower tile, into the block's
//     scratch matrix in HBM: DP × (DP + 1) doubles, column-major (element (i, j), i >= j, at
//     j·LD + i), so a column — what the factorisation and the forward sweep walk — is one
//     coalesced access across the lanes;
//   * the system is factorised there (Jacobi-scaled right-looking Cholesky, pivots floored at
//     1e-13, lane i owning rows i + 64 q) and solved by column sweeps.
// Padded coordinates (d <= j < DP) carry x_j = 0, a unit diagonal and no barrier term.  The
// reference's exact callers use d = 5 and 10 (exact_ftl_driver.py:86, exact_ftl.py:460-475):
// this kernel is for the rare wide problem, bound by L2 latency in the factorisation
// (DESIGN.md §3.6), and it only has to certify, not to be fast.
#include <algorithm>

#include "ocx_exact_src.h"
#include "ocx_internal.h"
#include "ocx_sim_kernels.h"

namespace {

// the barrier path's constants: ocx_exact_wide.hip's (and ocx_exact_ball.hip's)
constexpr int kMaxIter = 1000;  // the l1 path needs more steps as d grows
constexpr double kMu0 = 1.0;
constexpr double kMuEnd = 1e-10;
constexpr double kKappa = 10.0;
constexpr double kTolCenter = 1.0;
constexpr double kTolFinal = 1e-6;
constexpr int kFinalSteps = 6;
constexpr double kPivotFloor = 1e-13;
constexpr double kBreakdown = 1e8;
constexpr double kKeepRtol = 1e-9;  // the polish's keep bar (ocx_exact_wide.hip)
constexpr int kSweeps = 11;         // the polish's threshold sweeps (ocx_exact_wide.hip)
constexpr int RC = 32;              // rows per staged chunk

__device__ __forceinline__ void lds_sync() { __syncthreads(); }

// Σ over a lane's Q slots, then over the wave
template <int Q>
__device__ __forceinline__ double qsum(const double (&v)[Q]) {
    double s = v[0];
#pragma unroll
    for (int q = 1; q < Q; ++q) s += v[q];
    return ocx_seq_sum<64>(s);
}

// slot q (wave-uniform) of a per-lane vector
template <int Q>
__device__ __forceinline__ double qpick(const double (&v)[Q], int q) {
    double t = v[0];
#pragma unroll
    for (int k = 1; k < Q; ++k)
        if (q == k) t = v[k];
    return t;
}

template <int Q>
__device__ __forceinline__ double qmax_abs(const double (&v)[Q]) {
    double m = fabs(v[0]);
#pragma unroll
    for (int q = 1; q < Q; ++q) m = fmax(m, fabs(v[q]));
    for (int o = 32; o > 0; o >>= 1) m = fmax(m, __shfl_xor(m, o, 64));
    return m;
}

// S (DP × DP SPD, lower triangle, column-major: (i, j) at S[j·LD + i]) ← its Cholesky factor
// after Jacobi scaling (scales into sc[] and si).  Right-looking, eight columns per panel: the
// panel's columns (rows i + 64 q in registers) are factorised among themselves, then the
// trailing columns take the panel's eight updates in one read and one write, k in order —
// every element sees the same fma(−L_ik, L_jk, ·) sequence, k = 0, 1, ..., as one column at a
// time (ocx_exact_wide.hip's LDS factorisation), so the factor is that one's, bit for bit,
// with an eighth of the passes over the trailing matrix.  cl: LDS [8][DP], the panel's factor
// columns.
constexpr int kPanel = 8;
template <int Q>
__device__ void big_factor(double* S, double* sc, double* cl, int lane, double (&si)[Q]) {
    constexpr int DP = 64 * Q, LD = DP + 1, NP = kPanel;
#pragma unroll
    for (int q = 0; q < Q; ++q) {
        const int i = lane + 64 * q;
        const double dg = S[(int64_t)i * LD + i];
        si[q] = 1.0 / sqrt(dg > 0.0 ? dg : kPivotFloor);
        sc[i] = si[q];
    }
    lds_sync();
    for (int j = 0; j < DP; ++j) {
        const double sj = sc[j];
        double* col = S + (int64_t)j * LD;
#pragma unroll
        for (int q = 0; q < Q; ++q) {
            const int i = lane + 64 * q;
            if (i >= j) col[i] *= si[q] * sj;
        }
    }
    lds_sync();
    for (int k0 = 0; k0 < DP; k0 += NP) {
        // the panel's columns k0 .. k0 + 7, rows i >= k0 (the others are never read)
        double pc[NP][Q];
#pragma unroll
        for (int u = 0; u < NP; ++u)
#pragma unroll
            for (int q = 0; q < Q; ++q) {
                const int i = lane + 64 * q;
                pc[u][q] = i >= k0 + u ? S[(int64_t)(k0 + u) * LD + i] : 0.0;
            }
#pragma unroll
        for (int u = 0; u < NP; ++u) {
            const int k = k0 + u;
            double s = ocx_readlane(qpick(pc[u], k >> 6), k & 63);
            s = s > kPivotFloor ? s : kPivotFloor;
            const double l = sqrt(s), rd = 1.0 / l;
#pragma unroll
            for (int q = 0; q < Q; ++q) {
                const int i = lane + 64 * q;
                const double lik = i > k ? pc[u][q] * rd : 0.0;
                pc[u][q] = i == k ? l : lik;  // the factor's column (0 above the diagonal)
                cl[u * DP + i] = lik;
            }
            lds_sync();  // column k of the factor published
            // the panel's later columns: fma(−L_ik, L_jk, S_ij), j = k0 + u2
#pragma unroll
            for (int u2 = u + 1; u2 < NP; ++u2) {
                const double ljk = cl[u * DP + k0 + u2];
#pragma unroll
                for (int q = 0; q < Q; ++q) {
                    const int i = lane + 64 * q;
                    if (i >= k0 + u2) pc[u2][q] = __builtin_fma(-(i > k ? pc[u][q] : 0.0), ljk, pc[u2][q]);
                }
            }
        }
#pragma unroll
        for (int u = 0; u < NP; ++u)
#pragma unroll
            for (int q = 0; q < Q; ++q) {
                const int i = lane + 64 * q;
                if (i >= k0 + u) S[(int64_t)(k0 + u) * LD + i] = pc[u][q];
            }
        // the trailing columns j >= k0 + 8 take the panel's eight updates, k in order; four
        // columns' loads in flight
        for (int j0 = k0 + NP; j0 < DP; j0 += 4) {
            double v[4][Q];
#pragma unroll
            for (int w = 0; w < 4; ++w) {
                const int j = j0 + w;
                const double* col = S + (int64_t)j * LD;
#pragma unroll
                for (int q = 0; q < Q; ++q) {
                    const int i = lane + 64 * q;
                    v[w][q] = (j < DP && i >= j) ? col[i] : 0.0;
                }
            }
#pragma unroll
            for (int w = 0; w < 4; ++w) {
                const int j = j0 + w;
                if (j >= DP) break;
                double* col = S + (int64_t)j * LD;
#pragma unroll
                for (int u = 0; u < NP; ++u) {
                    const double ljk = cl[u * DP + j];
#pragma unroll
                    for (int q = 0; q < Q; ++q) v[w][q] = __builtin_fma(-pc[u][q], ljk, v[w][q]);
                }
#pragma unroll
                for (int q = 0; q < Q; ++q) {
                    const int i = lane + 64 * q;
                    if (i >= j) col[i] = v[w][q];
                }
            }
        }
        lds_sync();  // the trailing matrix and cl are done with before the next panel
    }
}

// out = K⁻¹ rhs for the factor big_factor left in S (si its scales): L w = rhs·sc, Lᵀ c = w
template <int Q>
__device__ void big_solve(const double* S, int lane, const double (&si)[Q], const double (&rhs)[Q],
                          double (&out)[Q]) {
    constexpr int DP = 64 * Q, LD = DP + 1;
    double v[Q], w[Q];
#pragma unroll
    for (int q = 0; q < Q; ++q) {
        v[q] = rhs[q] * si[q];
        w[q] = 0.0;
    }
    for (int k = 0; k < DP; ++k) {
        const double* ck = S + (int64_t)k * LD;
        const double wk = ocx_readlane(qpick(v, k >> 6), k & 63) / ck[k];
#pragma unroll
        for (int q = 0; q < Q; ++q) {
            const int i = lane + 64 * q;
            if (i == k) w[q] = wk;
            if (i > k) v[q] = __builtin_fma(-ck[i], wk, v[q]);
        }
    }
    double c[Q];
#pragma unroll
    for (int q = 0; q < Q; ++q) c[q] = 0.0;
    for (int k = DP - 1; k >= 0; --k) {
        const double dk = ocx_readlane(qpick(w, k >> 6), k & 63) / S[(int64_t)k * LD + k];
#pragma unroll
        for (int q = 0; q < Q; ++q) {
            const int i = lane + 64 * q;
            if (i == k) c[q] = dk;
            if (i < k) w[q] = __builtin_fma(-S[(int64_t)i * LD + k], dk, w[q]);
        }
    }
#pragma unroll
    for (int q = 0; q < Q; ++q) out[q] = c[q] * si[q];
}

// LDS of both kernels: RC staged rows, then DP-vectors, the row weights and the factor's
// panel (barrier kernel: 3 vectors, polish: 5)
template <int Q>
constexpr size_t big_lds_bytes() {
    return (size_t)(RC * (64 * Q + 1) + (5 + kPanel) * 64 * Q + 2 * 64) * sizeof(double) +
           (size_t)64 * Q * sizeof(int);
}

// stage rows [c0, c0 + rows) of problem b into R (zero past d); y into yv (lane r) if wanted
template <int DP>
__device__ __forceinline__ void big_stage(const WideSrc& rs, int64_t b, double* R, int lane,
                                          int64_t c0, int rows, double* yv) {
    constexpr int LD = DP + 1;
    const int d = rs.d;
    lds_sync();  // the previous chunk's readers are done with R
    for (int f = lane; f < rows * DP; f += 64) {
        const int r = f / DP, j = f - r * DP;
        R[r * LD + j] = j < d ? rs.zat(b, c0 + r, j) : 0.0;
    }
    if (yv) *yv = lane < rows ? rs.yat(b, c0 + lane) : 0.0;
    lds_sync();
}

template <int Q, int NORM>
__global__ __launch_bounds__(64) void ocx_exact_big_kernel(
    WideSrc rs, int64_t B, int64_t NP, double* __restrict__ scratch, int64_t sstride,
    double* __restrict__ actions, double* __restrict__ obj_out, double* __restrict__ gap_out,
    double* __restrict__ step_loss, int32_t* __restrict__ info_out) {
    constexpr int DP = 64 * Q, LD = DP + 1;
    extern __shared__ double lds[];
    double* R = lds;             // [RC][LD] staged rows
    double* xs = R + RC * LD;    // x (then the direction vector of a rank-1 term)
    double* vv = xs + DP;        // diagonal terms of the ball barrier
    double* sc = vv + DP;        // Jacobi scales
    double* gw = sc + DP;        // row weights r/s
    double* hw = gw + 64;        // row weights μ/(s·rt)
    double* cl = hw + 64;        // the factor's panel columns [8][DP]
    double* S = scratch + (int64_t)blockIdx.x * sstride;  // the system [DP][LD]
    double* W = S + (int64_t)DP * LD;                     // μ/(s·rt) of every row [T]

    const int lane = threadIdx.x & 63;
    const int bj = lane >> 3, bk = lane & 7;
    const int d = rs.d;
    const int64_t T = rs.T;
    for (int64_t p = blockIdx.x; p < B * NP; p += gridDim.x) {
        const int64_t b = p % B;
        const int64_t n = T - p / B;  // longest problems first
        const int64_t slot = NP == 1 ? 0 : n;
        bool cj[Q];
        double x[Q], u[Q];
#pragma unroll
        for (int q = 0; q < Q; ++q) {
            cj[q] = lane + 64 * q < d;
            x[q] = 0.0;
            u[q] = (NORM == 1 && cj[q]) ? 0.5 / d : 0.0;
        }
        double mu = kMu0;
        int it = 0, kend = 0;
        bool conv = n == 0, broke = false;
        // row r's residual z_r·x − y_r (lane r), in _dot's order from −y
        auto residual = [&](int r, double yv) {
            double rr = -yv;
            for (int j = 0; j < d; ++j) rr = __builtin_fma(R[r * LD + j], xs[j], rr);
            return rr;
        };

        while (!conv && it < kMaxIter) {
            ++it;
            lds_sync();  // the last pass's readers of xs are done
#pragma unroll
            for (int q = 0; q < Q; ++q) xs[lane + 64 * q] = x[q];
            // ---- rows: gradient Σ (r/s) a_i and the weights μ/(s·rt) into W
            double Gj[Q];
#pragma unroll
            for (int q = 0; q < Q; ++q) Gj[q] = 0.0;
            for (int64_t c0 = 0; c0 < n; c0 += RC) {
                const int rows = (int)(n - c0 < RC ? n - c0 : RC);
                double yv;
                big_stage<DP>(rs, b, R, lane, c0, rows, &yv);
                double g1 = 0.0;
                if (lane < rows) {
                    const double r = residual(lane, yv);
                    const double rt = sqrt(__builtin_fma(mu, mu, r * r));
                    const double s = mu + rt;
                    const double inv = 1.0 / (s * rt);
                    g1 = r * rt * inv;      // r / s
                    W[c0 + lane] = mu * inv;  // μ / (s·rt)
                }
                gw[lane] = g1;
                lds_sync();
                for (int r = 0; r < rows; ++r) {
                    const double g = gw[r];
#pragma unroll
                    for (int q = 0; q < Q; ++q) Gj[q] = __builtin_fma(g, R[r * LD + lane + 64 * q], Gj[q]);
                }
            }
            const double im = 1.0 / mu;
#pragma unroll
            for (int q = 0; q < Q; ++q) Gj[q] = cj[q] ? Gj[q] * im : 0.0;

            // ---- the ball's barrier: gradient, diagonal (vv) and a rank-1 term (xs, c1)
            double c1 = 0.0, gam = 0.0;
            double gu[Q], ia[Q], be[Q], rhs_g[Q];
#pragma unroll
            for (int q = 0; q < Q; ++q) gu[q] = ia[q] = be[q] = 0.0;
            lds_sync();  // the residuals' reads of xs are done
            if constexpr (NORM == 0) {
                double t[Q];
#pragma unroll
                for (int q = 0; q < Q; ++q) t[q] = cj[q] ? x[q] * x[q] : 0.0;
                const double iq = 1.0 / (1.0 - qsum(t));
#pragma unroll
                for (int q = 0; q < Q; ++q) {
                    Gj[q] = cj[q] ? __builtin_fma(2.0 * iq, x[q], Gj[q]) : 0.0;
                    vv[lane + 64 * q] = cj[q] ? 2.0 * iq : 1.0;  // padded coordinates: unit diagonal
                    xs[lane + 64 * q] = cj[q] ? x[q] : 0.0;
                    rhs_g[q] = Gj[q];
                }
                c1 = 4.0 * iq * iq;
            } else if constexpr (NORM == 2) {
#pragma unroll
                for (int q = 0; q < Q; ++q) {
                    const double iq = cj[q] ? 1.0 / __builtin_fma(-x[q], x[q], 1.0) : 0.0;
                    Gj[q] = cj[q] ? __builtin_fma(2.0 * x[q], iq, Gj[q]) : 0.0;
                    vv[lane + 64 * q] = cj[q] ? 2.0 * __builtin_fma(x[q], x[q], 1.0) * iq * iq : 1.0;
                    xs[lane + 64 * q] = 0.0;
                    rhs_g[q] = Gj[q];
                }
            } else {
                double t[Q];
#pragma unroll
                for (int q = 0; q < Q; ++q) t[q] = cj[q] ? u[q] : 0.0;
                const double iw = 1.0 / (1.0 - qsum(t)), c = iw * iw;
                double al[Q];
#pragma unroll
                for (int q = 0; q < Q; ++q) {
                    al[q] = 1.0;
                    if (cj[q]) {
                        const double ip = 1.0 / (u[q] - x[q]), ipp = 1.0 / (u[q] + x[q]);
                        Gj[q] += ip - ipp;
                        gu[q] = iw - ip - ipp;
                        al[q] = __builtin_fma(ip, ip, ipp * ipp);
                        be[q] = (ipp - ip) * (ipp + ip);
                        ia[q] = 1.0 / al[q];
                    }
                }
                gam = c / __builtin_fma(c, qsum(ia), 1.0);
#pragma unroll
                for (int q = 0; q < Q; ++q) t[q] = gu[q] * ia[q];
                const double tt = qsum(t);
#pragma unroll
                for (int q = 0; q < Q; ++q) {
                    const double hg = (gu[q] - gam * tt) * ia[q];
                    rhs_g[q] = cj[q] ? __builtin_fma(-be[q], hg, Gj[q]) : 0.0;
                    const double v = be[q] * ia[q];
                    vv[lane + 64 * q] = cj[q] ? __builtin_fma(-be[q], v, al[q]) : 1.0;
                    xs[lane + 64 * q] = v;
                }
                c1 = gam;
            }
            // (vv, xs are published by the first staging's barrier below)

            // ---- H/μ + diag(vv) + c1·xs xsᵀ into S, one lower 64 × 64 tile per pass
            for (int ti = 0; ti < Q; ++ti)
                for (int tk = 0; tk <= ti; ++tk) {
                    double H[8][8];
#pragma unroll
                    for (int i = 0; i < 8; ++i)
#pragma unroll
                        for (int k = 0; k < 8; ++k) H[i][k] = 0.0;
                    const int ci = ti * 64 + bj * 8, ck = tk * 64 + bk * 8;
                    for (int64_t c0 = 0; c0 < n; c0 += RC) {
                        const int rows = (int)(n - c0 < RC ? n - c0 : RC);
                        big_stage<DP>(rs, b, R, lane, c0, rows, nullptr);
                        hw[lane] = lane < rows ? W[c0 + lane] : 0.0;
                        lds_sync();
                        for (int r = 0; r < rows; ++r) {
                            const double h = hw[r];
                            double a1[8], a2[8];
#pragma unroll
                            for (int i = 0; i < 8; ++i) {
                                a1[i] = h * R[r * LD + ci + i];
                                a2[i] = R[r * LD + ck + i];
                            }
#pragma unroll
                            for (int i = 0; i < 8; ++i)
#pragma unroll
                                for (int k = 0; k < 8; ++k) H[i][k] = __builtin_fma(a1[i], a2[k], H[i][k]);
                        }
                    }
                    lds_sync();  // vv, xs published (n = 0 runs no staging)
#pragma unroll
                    for (int i = 0; i < 8; ++i) {
                        const int gi = ci + i;
#pragma unroll
                        for (int k = 0; k < 8; ++k) {
                            const int gk = ck + k;
                            if (gi < gk) continue;
                            double h = gi < d && gk < d ? H[i][k] * im : 0.0;
                            h = __builtin_fma(c1 * xs[gi], xs[gk], h);
                            if (gi == gk) h += vv[gi];
                            S[(int64_t)gk * LD + gi] = h;
                        }
                    }
                }
            lds_sync();  // the system is complete
            double si[Q], sol[Q], dx[Q];
            big_factor<Q>(S, sc, cl, lane, si);
            big_solve<Q>(S, lane, si, rhs_g, sol);
#pragma unroll
            for (int q = 0; q < Q; ++q) dx[q] = cj[q] ? -sol[q] : 0.0;
            double du[Q], lam2;
#pragma unroll
            for (int q = 0; q < Q; ++q) du[q] = 0.0;
            if constexpr (NORM == 1) {
                double rh[Q], t[Q];
#pragma unroll
                for (int q = 0; q < Q; ++q) {
                    rh[q] = cj[q] ? __builtin_fma(-be[q], dx[q], -gu[q]) : 0.0;
                    t[q] = rh[q] * ia[q];
                }
                const double tr = qsum(t);
#pragma unroll
                for (int q = 0; q < Q; ++q) {
                    du[q] = cj[q] ? (rh[q] - gam * tr) * ia[q] : 0.0;
                    t[q] = __builtin_fma(-Gj[q], dx[q], -gu[q] * du[q]);
                }
                lam2 = qsum(t);
            } else {
                double t[Q];
#pragma unroll
                for (int q = 0; q < Q; ++q) t[q] = -Gj[q] * dx[q];
                lam2 = qsum(t);
            }
            const double lam = sqrt(lam2 > 0.0 ? lam2 : 0.0);
            if (lam > kBreakdown) {  // μ has outrun fp64 (see ocx_exact_ball.hip)
                broke = true;
                break;
            }
            double step = lam > 0.25 ? 1.0 / (1.0 + lam) : 1.0;
            for (int h = 0; h < 60; ++h) {
                double xn[Q], un[Q], t[Q];
                bool bad = false;
#pragma unroll
                for (int q = 0; q < Q; ++q) {
                    xn[q] = __builtin_fma(step, dx[q], x[q]);
                    un[q] = NORM == 1 ? __builtin_fma(step, du[q], u[q]) : 0.0;
                }
                bool ok;
                if constexpr (NORM == 0) {
#pragma unroll
                    for (int q = 0; q < Q; ++q) t[q] = cj[q] ? xn[q] * xn[q] : 0.0;
                    ok = qsum(t) < 1.0;
                } else if constexpr (NORM == 2) {
#pragma unroll
                    for (int q = 0; q < Q; ++q) bad = bad || (cj[q] && !(fabs(xn[q]) < 1.0));
                    ok = __ballot(bad) == 0;
                } else {
#pragma unroll
                    for (int q = 0; q < Q; ++q) {
                        bad = bad || (cj[q] && !(fabs(xn[q]) < un[q]));
                        t[q] = cj[q] ? un[q] : 0.0;
                    }
                    ok = __ballot(bad) == 0 && qsum(t) < 1.0;
                }
                if (ok) {
#pragma unroll
                    for (int q = 0; q < Q; ++q) {
                        x[q] = xn[q];
                        u[q] = un[q];
                    }
                    break;
                }
                step *= 0.5;
            }
            if (mu > kMuEnd) {
                if (lam < kTolCenter) mu = fmax(mu / kKappa, kMuEnd);
            } else if (lam < kTolFinal || ++kend >= kFinalSteps) {
                conv = true;
                break;
            }
        }

        // ---- certificate (as ocx_exact_wide.hip): obj, dual bounds of λ_a = r/(2s) and λ_b
        lds_sync();
#pragma unroll
        for (int q = 0; q < Q; ++q) xs[lane + 64 * q] = x[q];
        double P = 0.0, Ya = 0.0, Yb = 0.0, Wa[Q], Wb[Q];
#pragma unroll
        for (int q = 0; q < Q; ++q) Wa[q] = Wb[q] = 0.0;
        for (int64_t c0 = 0; c0 < n; c0 += RC) {
            const int rows = (int)(n - c0 < RC ? n - c0 : RC);
            double yv;
            big_stage<DP>(rs, b, R, lane, c0, rows, &yv);
            double la = 0.0, lb = 0.0;
            if (lane < rows) {
                const double r = residual(lane, yv);
                P += 0.5 * fabs(r);
                const double s = mu + sqrt(__builtin_fma(mu, mu, r * r));
                la = 0.5 * r / s;
                lb = fabs(r) > 1e3 * mu ? (r > 0.0 ? 0.5 : -0.5) : la;
                Ya = __builtin_fma(la, yv, Ya);
                Yb = __builtin_fma(lb, yv, Yb);
            }
            gw[lane] = la;
            hw[lane] = lb;
            lds_sync();
            for (int r = 0; r < rows; ++r) {
#pragma unroll
                for (int q = 0; q < Q; ++q) {
                    const double a = R[r * LD + lane + 64 * q];
                    Wa[q] = __builtin_fma(gw[r], a, Wa[q]);
                    Wb[q] = __builtin_fma(hw[r], a, Wb[q]);
                }
            }
        }
        P = ocx_seq_sum<64>(P);
        Ya = ocx_seq_sum<64>(Ya);
        Yb = ocx_seq_sum<64>(Yb);
#pragma unroll
        for (int q = 0; q < Q; ++q)
            if (!cj[q]) Wa[q] = Wb[q] = 0.0;
        double na, nb;
        if constexpr (NORM == 0) {
            double ta[Q], tb[Q];
#pragma unroll
            for (int q = 0; q < Q; ++q) {
                ta[q] = Wa[q] * Wa[q];
                tb[q] = Wb[q] * Wb[q];
            }
            na = sqrt(qsum(ta));
            nb = sqrt(qsum(tb));
        } else if constexpr (NORM == 2) {
            double ta[Q], tb[Q];
#pragma unroll
            for (int q = 0; q < Q; ++q) {
                ta[q] = fabs(Wa[q]);
                tb[q] = fabs(Wb[q]);
            }
            na = qsum(ta);
            nb = qsum(tb);
        } else {
            na = qmax_abs(Wa);
            nb = qmax_abs(Wb);
        }
        const double bound = fmax(fmax(-Ya - na, -Yb - nb), 0.0);
#pragma unroll
        for (int q = 0; q < Q; ++q)
            if (cj[q]) actions[(b * NP + slot) * d + lane + 64 * q] = x[q];
        if (lane == 0) {
            if (obj_out) obj_out[b * NP + slot] = P;
            if (gap_out) gap_out[b * NP + slot] = fmax(P - bound, 0.0);
            if (info_out)
                info_out[b * NP + slot] = broke ? (OCX_EXACT_INFO_BREAKDOWN | it) : (conv ? it : -it);
            if (step_loss) {
                // FTL's loss at step n (replay_exact_ftl :318-323: _dot's sequential sum)
                double lo = 0.0;
                if (n < T) {
                    double qq = 0.0;
                    for (int j = 0; j < d; ++j) qq = qq + rs.zat(b, n, j) * xs[j];
                    lo = 0.5 * fabs(qq - rs.yat(b, n));
                }
                step_loss[b * NP + slot] = lo;
            }
        }
    }
}

// ---------------------------------------------------------------------------------------------
// Certificate polish for 64 < d <= 256: ocx_exact_wide.hip's ocx_exact_polish_kernel (eleven
// threshold pairs; active set, primal purification, KKT dual; see there) with at most DP
// active rows (one fewer beside the cone row).  The active rows sit row-major in the block's
// second scratch matrix A; their Gram systems in S, factorised by big_factor.
template <int Q, int NORM>
__global__ __launch_bounds__(64) void ocx_exact_big_polish_kernel(
    WideSrc rs, int64_t B, int64_t NP, double* __restrict__ scratch, int64_t sstride,
    double* __restrict__ actions, double* __restrict__ obj, double* __restrict__ gap,
    double* __restrict__ step_loss) {
    constexpr int DP = 64 * Q, LD = DP + 1;
    extern __shared__ double lds[];
    double* R = lds;             // [RC][LD] staged rows
    double* xs = R + RC * LD;    // x, then x'
    double* gs = xs + DP;        // g = Σ_{i∉A} λ_i z_i
    double* em = gs + DP;        // 1.0 where coordinate j's stationarity equation holds
    double* sc = em + DP;        // δ on fixed coordinates / the solve's scales / λ_A
    double* ra = sc + DP;        // active rows' residuals at x, then their y
    double* wv = ra + DP;        // per-row weights of a staged chunk
    double* cl = wv + 128;       // the factor's panel columns [8][DP]
    int* act = reinterpret_cast<int*>(cl + kPanel * DP);  // active row indices [DP]
    double* S = scratch + (int64_t)blockIdx.x * sstride;  // the Gram systems [DP][LD]
    double* A = S + (int64_t)DP * LD;                      // active rows (+ cone row) [DP][LD]

    const int lane = threadIdx.x & 63;
    const int d = rs.d;
    const int64_t T = rs.T;
    for (int64_t p = blockIdx.x; p < B * NP; p += gridDim.x) {
        const int64_t b = p % B;
        const int64_t n = T - p / B;
        const int64_t o = b * NP + (NP == 1 ? 0 : n);
        const double g0 = gap[o], f0 = obj[o];
        if (n == 0 || !(g0 > 0.0)) continue;  // exact already (or a NaN the caller reports)
        bool cj[Q];
        double x[Q], xbest[Q];
#pragma unroll
        for (int q = 0; q < Q; ++q) {
            cj[q] = lane + 64 * q < d;
            x[q] = cj[q] ? actions[o * d + lane + 64 * q] : 0.0;
            xbest[q] = x[q];
        }
        double best = g0, pbest = f0;
        bool improved = false;
        double bestx = g0, P0x = f0;
        auto resid = [&](int r, double yv) {  // staged row r at xs, in _dot's order from −y
            double rr = -yv;
            for (int j = 0; j < d; ++j) rr = __builtin_fma(R[r * LD + j], xs[j], rr);
            return rr;
        };
        // S ← Σ_j em_j A_l,j A_l',j over the first mr rows (+ ridge), identity past mr
        auto gram = [&](int mr) {
#pragma unroll
            for (int q = 0; q < Q; ++q) {
                const int l = lane + 64 * q;
                for (int l2 = 0; l2 <= l; ++l2) {
                    double s2;
                    if (l < mr) {
                        s2 = 0.0;
                        for (int j = 0; j < d; ++j)
                            s2 = __builtin_fma(em[j] * A[(int64_t)l * LD + j], A[(int64_t)l2 * LD + j], s2);
                    } else {
                        s2 = l2 == l ? 1.0 : 0.0;
                    }
                    S[(int64_t)l2 * LD + l] = s2;
                }
            }
            lds_sync();
            double t[Q];
#pragma unroll
            for (int q = 0; q < Q; ++q) {
                const int l = lane + 64 * q;
                t[q] = l < mr ? S[(int64_t)l * LD + l] : 0.0;
            }
            const double tr = qsum(t);
#pragma unroll
            for (int q = 0; q < Q; ++q) {
                const int l = lane + 64 * q;
                if (l < mr) S[(int64_t)l * LD + l] += 1e-13 * (tr / (mr > 0 ? mr : 1)) + 1e-300;
            }
            lds_sync();
        };

        for (int sweep = 0; sweep < kSweeps; ++sweep) {
            const double tsc = sweep == 0 ? 1.0 : (sweep == 1 ? 1e3 : (sweep == 2 ? 1e2 : (sweep == 3 ? 10.0 :
                               (sweep == 4 ? 1e4 : (sweep == 5 ? 0.1 : 0.01)))));
            // sweeps 7..10 scale the coordinates' and the rows' thresholds apart (a near-degenerate
            // bound sits ~μ/ν from x while every row is still tight at 1e-7)
            const double tx = sweep < 7 ? tsc : (sweep == 7 ? 1e2 : (sweep == 8 ? 1e4 : 1.0));
            const double tr = sweep < 7 ? tsc : (sweep == 9 ? 1e2 : (sweep == 10 ? 1e4 : 1.0));
            const double kTight = 1e-8 * tx, kZero = 1e-7 * tx, kZeroR = 1e-7 * tr;
            // ---- 1. the ball's constraints at x
            bool cone = false, fixed[Q];
            double tgt[Q], crow[Q], t[Q];
#pragma unroll
            for (int q = 0; q < Q; ++q) {
                fixed[q] = false;
                tgt[q] = crow[q] = 0.0;
            }
            if constexpr (NORM == 0) {
#pragma unroll
                for (int q = 0; q < Q; ++q) {
                    t[q] = x[q] * x[q];
                    crow[q] = 2.0 * x[q];
                }
                cone = qsum(t) >= 1.0 - kTight;
            } else if constexpr (NORM == 2) {
#pragma unroll
                for (int q = 0; q < Q; ++q) {
                    fixed[q] = cj[q] && fabs(x[q]) >= 1.0 - kTight;
                    tgt[q] = x[q] > 0.0 ? 1.0 : -1.0;
                }
            } else {
#pragma unroll
                for (int q = 0; q < Q; ++q) t[q] = fabs(x[q]);
                cone = qsum(t) >= 1.0 - kTight;
                if (cone) {
#pragma unroll
                    for (int q = 0; q < Q; ++q) {
                        fixed[q] = cj[q] && fabs(x[q]) <= kZero;
                        crow[q] = (cj[q] && !fixed[q]) ? (x[q] > 0.0 ? 1.0 : -1.0) : 0.0;
                    }
                }
            }
            bool freec[Q];
#pragma unroll
            for (int q = 0; q < Q; ++q) freec[q] = cj[q] && !fixed[q];
            const int AM = DP - (cone ? 1 : 0);
            lds_sync();
#pragma unroll
            for (int q = 0; q < Q; ++q) {
                xs[lane + 64 * q] = x[q];
                em[lane + 64 * q] = freec[q] ? 1.0 : 0.0;
            }
            // ---- pass 1 at x: ½Σ|r|, the active set and its residuals
            double P0 = 0.0;
            int m = 0;
            bool over = false;
            for (int64_t c0 = 0; c0 < n; c0 += RC) {
                const int rows = (int)(n - c0 < RC ? n - c0 : RC);
                double yv;
                big_stage<DP>(rs, b, R, lane, c0, rows, &yv);
                bool a = false;
                double rr = 0.0;
                if (lane < rows) {
                    rr = resid(lane, yv);
                    P0 += 0.5 * fabs(rr);
                    a = fabs(rr) <= kZeroR * (1.0 + fabs(yv));
                }
                const uint64_t am = __ballot(a);
                const int pos = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(am >> 32),
                                                               __builtin_amdgcn_mbcnt_lo((uint32_t)am, 0u));
                if (a && m + pos < AM) {
                    act[m + pos] = (int)(c0 + lane);
                    ra[m + pos] = rr;
                }
                m += __builtin_popcountll(am);
                over = over || m > AM;
            }
            if (over) continue;  // wave-uniform: too many active rows at this scale
            P0 = ocx_seq_sum<64>(P0);
            P0x = P0;
            const int mr = m + (cone ? 1 : 0);
            lds_sync();
            // ---- 2. primal purification: rows of the active set (+ the cone row) into A
            for (int f = lane; f < m * DP; f += 64) {
                const int k = f / DP, j = f - k * DP;
                A[(int64_t)k * LD + j] = j < d ? rs.zat(b, act[k], j) : 0.0;
            }
#pragma unroll
            for (int q = 0; q < Q; ++q) {
                if (cone) A[(int64_t)m * LD + lane + 64 * q] = cj[q] ? crow[q] : 0.0;
                sc[lane + 64 * q] = fixed[q] ? tgt[q] - x[q] : 0.0;  // δ_j on a fixed coordinate
            }
            lds_sync();
            // right-hand sides: −r_k minus the fixed coordinates' part; the cone row's defect
            double defect;
            if constexpr (NORM == 0) {
#pragma unroll
                for (int q = 0; q < Q; ++q) t[q] = x[q] * x[q];
            } else {
#pragma unroll
                for (int q = 0; q < Q; ++q) t[q] = freec[q] ? fabs(x[q]) : 0.0;
            }
            defect = 1.0 - qsum(t);
            double rhs[Q];
#pragma unroll
            for (int q = 0; q < Q; ++q) {
                const int k = lane + 64 * q;
                rhs[q] = 0.0;
                if (k < m) {
                    double r2 = -ra[k];
                    for (int j = 0; j < d; ++j) r2 = __builtin_fma(-A[(int64_t)k * LD + j], sc[j], r2);
                    rhs[q] = r2;
                }
                if (cone && k == m) rhs[q] = defect;
            }
            gram(mr);
            double si[Q], uu[Q];
            big_factor<Q>(S, sc, cl, lane, si);
            big_solve<Q>(S, lane, si, rhs, uu);
            lds_sync();
#pragma unroll
            for (int q = 0; q < Q; ++q) sc[lane + 64 * q] = lane + 64 * q < mr ? uu[q] : 0.0;
            lds_sync();
            double xn[Q];
#pragma unroll
            for (int q = 0; q < Q; ++q) {
                xn[q] = x[q];
                if (cj[q]) {
                    if (fixed[q]) {
                        xn[q] = tgt[q];
                    } else {
                        double dl = 0.0;
                        for (int k = 0; k < mr; ++k)
                            dl = __builtin_fma(A[(int64_t)k * LD + lane + 64 * q], sc[k], dl);
                        xn[q] = x[q] + dl;
                    }
                }
            }
            // into the ball
            if constexpr (NORM == 0) {
#pragma unroll
                for (int q = 0; q < Q; ++q) t[q] = xn[q] * xn[q];
                const double nn = sqrt(qsum(t));
                if (nn > 1.0)
#pragma unroll
                    for (int q = 0; q < Q; ++q) xn[q] = xn[q] / nn;
            } else if constexpr (NORM == 2) {
#pragma unroll
                for (int q = 0; q < Q; ++q) xn[q] = fmin(fmax(xn[q], -1.0), 1.0);
            } else {
#pragma unroll
                for (int q = 0; q < Q; ++q) t[q] = fabs(xn[q]);
                const double s1 = qsum(t);
                if (s1 > 1.0)
#pragma unroll
                    for (int q = 0; q < Q; ++q) xn[q] = xn[q] / s1;
            }
            lds_sync();
#pragma unroll
            for (int q = 0; q < Q; ++q) xs[lane + 64 * q] = xn[q];
            // ---- pass 2 at x': ½Σ|r'|, λ_i = ½ sign(r'_i) off the active set into g and λ·y
            double P1 = 0.0, Y = 0.0, gj[Q];
#pragma unroll
            for (int q = 0; q < Q; ++q) gj[q] = 0.0;
            int ia = 0;  // next entry of act[] (the active rows come in increasing order)
            for (int64_t c0 = 0; c0 < n; c0 += RC) {
                const int rows = (int)(n - c0 < RC ? n - c0 : RC);
                double yv;
                big_stage<DP>(rs, b, R, lane, c0, rows, &yv);
                double lam = 0.0;
                bool isact = false;
                if (lane < rows) {
                    const double rr = resid(lane, yv);
                    P1 += 0.5 * fabs(rr);
                    for (int k = ia; k < m && act[k] <= (int)(c0 + lane); ++k)
                        if (act[k] == (int)(c0 + lane)) isact = true;
                    lam = isact ? 0.0 : (rr > 0.0 ? 0.5 : (rr < 0.0 ? -0.5 : 0.0));
                    Y = __builtin_fma(lam, yv, Y);
                }
                while (ia < m && act[ia] < (int)(c0 + rows)) ++ia;
                wv[lane] = lam;
                lds_sync();
                for (int r = 0; r < rows; ++r) {
                    const double wr = wv[r];
#pragma unroll
                    for (int q = 0; q < Q; ++q)
                        if (cj[q]) gj[q] = __builtin_fma(wr, R[r * LD + lane + 64 * q], gj[q]);
                }
            }
            P1 = ocx_seq_sum<64>(P1);
            Y = ocx_seq_sum<64>(Y);
            if (!(P1 <= P0)) continue;  // the purified point is no better: keep x's certificate
            lds_sync();
#pragma unroll
            for (int q = 0; q < Q; ++q) {
                gs[lane + 64 * q] = gj[q];
                if (lane + 64 * q < m) ra[lane + 64 * q] = rs.yat(b, act[lane + 64 * q]);
            }
            lds_sync();
            // ---- 3. dual: least squares for λ_A (and ν) on the free coordinates' equations
            double hk[Q];
#pragma unroll
            for (int q = 0; q < Q; ++q) {
                const int l = lane + 64 * q;
                hk[q] = 0.0;
                if (l < mr)
                    for (int j = 0; j < d; ++j) hk[q] = __builtin_fma(em[j] * A[(int64_t)l * LD + j], gs[j], hk[q]);
                rhs[q] = l < mr ? -hk[q] : 0.0;
            }
            gram(mr);
            double cc[Q];
            big_factor<Q>(S, sc, cl, lane, si);
            big_solve<Q>(S, lane, si, rhs, cc);
            double la[Q];
#pragma unroll
            for (int q = 0; q < Q; ++q) {
                const int k = lane + 64 * q;
                la[q] = k < m ? fmin(fmax(cc[q], -0.5), 0.5) : 0.0;
                t[q] = k < m ? la[q] * ra[k] : 0.0;
            }
            Y += qsum(t);
            lds_sync();
#pragma unroll
            for (int q = 0; q < Q; ++q) sc[lane + 64 * q] = la[q];
            lds_sync();
            double wj[Q];
#pragma unroll
            for (int q = 0; q < Q; ++q) {
                wj[q] = gj[q];
                if (cj[q])
                    for (int k = 0; k < m; ++k) wj[q] = __builtin_fma(sc[k], A[(int64_t)k * LD + lane + 64 * q], wj[q]);
                else
                    wj[q] = 0.0;
            }
            double nw;
            if constexpr (NORM == 0) {
#pragma unroll
                for (int q = 0; q < Q; ++q) t[q] = wj[q] * wj[q];
                nw = sqrt(qsum(t));
            } else if constexpr (NORM == 2) {
#pragma unroll
                for (int q = 0; q < Q; ++q) t[q] = fabs(wj[q]);
                nw = qsum(t);
            } else {
                nw = qmax_abs(wj);
            }
            const double gn = fmax(P1 - (-Y - nw), 0.0);
            bestx = fmin(bestx, fmax(P0 - (-Y - nw), 0.0));
            if (gn < best) {
                best = gn;
                pbest = P1;
#pragma unroll
                for (int q = 0; q < Q; ++q) xbest[q] = xn[q];
                improved = true;
            }
            if (best <= 1e-14 * (1.0 + pbest) && bestx <= kKeepRtol * (1.0 + fabs(P0x))) break;
        }
        if (bestx < g0 && bestx <= kKeepRtol * (1.0 + fabs(P0x))) {
            // x certifies on its own: keep it (and its step loss), report its objective and gap
            if (lane == 0) {
                obj[o] = P0x;
                gap[o] = bestx;
            }
            continue;
        }
        if (!improved) continue;
#pragma unroll
        for (int q = 0; q < Q; ++q)
            if (cj[q]) actions[o * d + lane + 64 * q] = xbest[q];
        lds_sync();
#pragma unroll
        for (int q = 0; q < Q; ++q) xs[lane + 64 * q] = xbest[q];
        lds_sync();
        if (lane == 0) {
            obj[o] = pbest;
            gap[o] = best;
            if (step_loss && NP > 1) {
                // FTL's loss at step n with this action (replay_exact_ftl :318-323: _dot's order)
                double lo = 0.0;
                if (n < T) {
                    double qq = 0.0;
                    for (int j = 0; j < d; ++j) qq = qq + rs.zat(b, n, j) * xs[j];
                    lo = 0.5 * fabs(qq - rs.yat(b, n));
                }
                step_loss[o] = lo;
            }
        }
    }
}

template <int Q, int NORM>
hipError_t launch_big_qn(const WideSrc& rs, int64_t B, int64_t NP, double* actions, double* obj,
                         double* gap, double* step_loss, int32_t* info, hipStream_t st) {
    constexpr int DP = 64 * Q, LD = DP + 1;
    const int64_t total = B * NP;
    // persistent blocks: about what the LDS lets stay resident (81 KB at Q = 4, 42 KB at Q = 2)
    const int blocks = (int)std::min<int64_t>(total, Q == 2 ? 512 : 256);
    // per block: the system and (polish) the active rows, or the system and a weight per row
    int64_t sstride = std::max<int64_t>(2 * (int64_t)DP * LD, (int64_t)DP * LD + rs.T);
    sstride = (sstride + 63) / 64 * 64;
    double* scratch = nullptr;
    hipError_t e = hipMallocAsync(reinterpret_cast<void**>(&scratch), (size_t)blocks * sstride * 8, st);
    if (e != hipSuccess) return e;
    const size_t lds = big_lds_bytes<Q>();
    hipLaunchKernelGGL((ocx_exact_big_kernel<Q, NORM>), dim3(blocks), dim3(64), lds, st, rs, B, NP,
                       scratch, sstride, actions, obj, gap, step_loss, info);
    e = hipGetLastError();
    if (e == hipSuccess && gap && obj) {
        hipLaunchKernelGGL((ocx_exact_big_polish_kernel<Q, NORM>), dim3(blocks), dim3(64), lds, st,
                           rs, B, NP, scratch, sstride, actions, obj, gap, step_loss);
        e = hipGetLastError();
    }
    const hipError_t ef = hipFreeAsync(scratch, st);
    return e != hipSuccess ? e : ef;
}

template <int Q>
hipError_t launch_big_q(const WideSrc& rs, int64_t B, int64_t NP, int norm, double* actions,
                        double* obj, double* gap, double* step_loss, int32_t* info, hipStream_t st) {
    switch (norm) {
        case 0: return launch_big_qn<Q, 0>(rs, B, NP, actions, obj, gap, step_loss, info, st);
        case 1: return launch_big_qn<Q, 1>(rs, B, NP, actions, obj, gap, step_loss, info, st);
        case 2: return launch_big_qn<Q, 2>(rs, B, NP, actions, obj, gap, step_loss, info, st);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace

// 64 < d <= 256: the solve and its certificate polish, row-major (tiled = 0) or the tiled layout
hipError_t ocx_launch_exact_big(const double* z, const double* y, int64_t B, int64_t T, int64_t d,
                                int tiled, int P, int C, int S, int64_t G, int norm,
                                int all_prefixes, double* actions, double* obj, double* gap,
                                double* step_loss, int32_t* info, hipStream_t st) {
    const int64_t NP = all_prefixes ? T + 1 : 1;
    if (B == 0 || NP == 0) return hipSuccess;
    if (d <= 64 || d > 256 || T > (int64_t)1 << 30 ||
        B > ((int64_t)1 << 40) / std::max<int64_t>(NP, 1))
        return hipErrorInvalidValue;
    const WideSrc rs{z, y, T, G, (int)d, P, C, S, tiled};
    if (d <= 128) return launch_big_q<2>(rs, B, NP, norm, actions, obj, gap, step_loss, info, st);
    return launch_big_q<4>(rs, B, NP, norm, actions, obj, gap, step_loss, info, st);
}
