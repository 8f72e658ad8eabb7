// ocx_exact_ball.hip — the general exact-FTL comparator: ExactFTLNoClip's problem
// (exact_ftl.py:83-105, solved by cvxpy at :119-128)
//     min_x  ½ Σ_{i<n} |z_i·x − y_i|   s.t.  ||x||_p <= 1,   p ∈ {2, 1, ∞}
// for ANY rows and labels — where the closed forms of ocx_ftl_exact_batch do not apply
// (rows whose dual norm exceeds 1: the linf ball on the reference's ||z||_2 <= 1 rows,
// unclipped caller data, labels other than ±1).
//
// Method: a primal log-barrier path with the slacks eliminated in closed form.  For the
// epigraph form  min Σ s_i, s_i >= |r_i|, r = Zx − y,  the barrier
//     F_μ(x, s) = (1/μ) Σ s_i − Σ log(s_i − r_i) − Σ log(s_i + r_i) + β(x)
// is minimised over s by  s_i = μ + sqrt(μ² + r_i²), leaving a self-concordant F_μ(x) with
//     ∂F/∂r_i = r_i / (μ s_i),   ∂²F/∂r_i² = 1 / (s_i sqrt(μ² + r_i²))
// and the ball's barrier β (l2: −log(1 − ||x||²); linf: −Σ log(1 − x_j²); l1: variables
// (x, u), −Σ log(u_j − x_j) − Σ log(u_j + x_j) − log(1 − Σ u_j), u eliminated from each
// Newton system by a Schur complement, so every system is d × d).  Damped Newton
// (step 1/(1+λ) while the decrement λ > 1/4: in the domain by self-concordance) follows
// the central path from μ = 1 down to 1e-10 (μ /= 10 once λ < 1); the path's limit is the
// analytic centre of the optimal face — the point interior-point solvers such as the ECOS /
// Clarabel backends cvxpy picks approach — so where the minimiser is not unique this
// returns that point.
//
// One wavefront per problem (sequence b, prefix length n): lanes stride the rows of a
// Newton pass (gradient and Hessian sums; the rows stay in L2 across the ≈50 passes), a
// butterfly gives every lane the same totals, and every lane solves the small system
// redundantly (Jacobi-scaled Cholesky, pivots floored at 1e-13 for the μ → 0
// ill-conditioning), so the control flow stays wave-uniform.  Problems are issued longest
// first.  A final pass certifies each answer: obj = ½Σ|r_i| and a dual bound
// −λ·y − ||Zᵀλ||_* for three feasible duals (|λ_i| <= ½: the barrier's λ_i = r_i/(2 s_i),
// that one with the clearly inactive rows rounded to ±½, and 0); gap = obj − best bound >= 0
// bounds obj − optimum.  This is a compute kernel (≈50 passes over each prefix), not a
// streaming one: its bound is the VALU, and the answer's accuracy (≈1e-9) is set by μ_end.
#include "ocx_internal.h"
#include "ocx_sim_kernels.h"

namespace {

constexpr int kMaxIter = 300;
constexpr double kMu0 = 1.0;
constexpr double kMuEnd = 1e-10;
constexpr double kKappa = 10.0;
constexpr double kTolCenter = 1.0;  // λ below which μ decreases
constexpr double kTolFinal = 1e-6;  // λ at μ_end that ends the solve
constexpr int kFinalSteps = 6;      // or this many Newton steps at μ_end
constexpr double kPivotFloor = 1e-13;
constexpr double kBreakdown = 1e8;  // a Newton decrement no centred step produces

// packed lower triangle, row by row: (i, j), j <= i
__host__ __device__ constexpr int tri(int i, int j) { return i * (i + 1) / 2 + j; }

__device__ __forceinline__ double wave_total(double v) { return ocx_seq_sum<64>(v); }

// Solve H dx = -g (H SPD, packed lower) by Jacobi-scaled Cholesky; returns dx.
template <int D>
__device__ __forceinline__ void spd_solve(double (&H)[D * (D + 1) / 2], const double (&g)[D],
                                          double (&dx)[D]) {
    double sc[D], w[D];
#pragma unroll
    for (int i = 0; i < D; ++i) sc[i] = 1.0 / sqrt(H[tri(i, i)] > 0.0 ? H[tri(i, i)] : kPivotFloor);
#pragma unroll
    for (int i = 0; i < D; ++i)
#pragma unroll
        for (int j = 0; j <= i; ++j) H[tri(i, j)] *= sc[i] * sc[j];
    double rd[D];  // reciprocal diagonal of L
#pragma unroll
    for (int j = 0; j < D; ++j) {
        double s = H[tri(j, j)];
#pragma unroll
        for (int k = 0; k < j; ++k) s = __builtin_fma(-H[tri(j, k)], H[tri(j, k)], s);
        s = s > kPivotFloor ? s : kPivotFloor;
        const double l = sqrt(s);
        H[tri(j, j)] = l;
        rd[j] = 1.0 / l;
#pragma unroll
        for (int i = j + 1; i < D; ++i) {
            double v = H[tri(i, j)];
#pragma unroll
            for (int k = 0; k < j; ++k) v = __builtin_fma(-H[tri(i, k)], H[tri(j, k)], v);
            H[tri(i, j)] = v * rd[j];
        }
    }
#pragma unroll
    for (int i = 0; i < D; ++i) {  // L w = g_scaled
        double v = g[i] * sc[i];
#pragma unroll
        for (int k = 0; k < i; ++k) v = __builtin_fma(-H[tri(i, k)], w[k], v);
        w[i] = v * rd[i];
    }
#pragma unroll
    for (int i = D - 1; i >= 0; --i) {  // Lᵀ v = −w
        double v = -w[i];
#pragma unroll
        for (int k = i + 1; k < D; ++k) v = __builtin_fma(-H[tri(k, i)], dx[k], v);
        dx[i] = v * rd[i];
    }
#pragma unroll
    for (int i = 0; i < D; ++i) dx[i] *= sc[i];
}

template <int D, int NORM>
__device__ __forceinline__ bool in_domain(const double (&x)[D], const double (&u)[D]) {
    if constexpr (NORM == 0) {
        double q = 0.0;
#pragma unroll
        for (int j = 0; j < D; ++j) q = __builtin_fma(x[j], x[j], q);
        return q < 1.0;
    } else if constexpr (NORM == 2) {
        bool ok = true;
#pragma unroll
        for (int j = 0; j < D; ++j) ok = ok && fabs(x[j]) < 1.0;
        return ok;
    } else {
        bool ok = true;
        double su = 0.0;
#pragma unroll
        for (int j = 0; j < D; ++j) {
            ok = ok && fabs(x[j]) < u[j];
            su += u[j];
        }
        return ok && su < 1.0;
    }
}

// Where row i of sequence b lives: row-major z [B][T][D], y [B][T], or the tiled layout
// (ocx_layout, ocx_pack_z_kernel's inverse: element j of row t in plane k = (j%C)/2, lane
// (b%S)·P + j/C, half (j%C)&1; y at (g·T + t)·S + b%S).
struct RowSrc {
    const double* z;
    const double* y;
    int64_t T, G;
    int P, C, S, tiled;
};

template <int D>
__device__ __forceinline__ void load_row(const RowSrc& rs, int64_t b, int64_t i, double (&a)[D],
                                         double& yi) {
    if (!rs.tiled) {
#pragma unroll
        for (int j = 0; j < D; ++j) a[j] = rs.z[(b * rs.T + i) * D + j];
        yi = rs.y[b * rs.T + i];
        return;
    }
    const int64_t g = b / rs.S;
    const int s = (int)(b - g * rs.S);
#pragma unroll
    for (int j = 0; j < D; ++j) {
        const int jl = j / rs.C, jj = j - jl * rs.C;
        const int64_t k = jj >> 1;
        a[j] = rs.z[((k * rs.G + g) * rs.T + i) * 128 + 2 * (s * rs.P + jl) + (jj & 1)];
    }
    yi = rs.y[(g * rs.T + i) * rs.S + s];
}

template <int D, int NORM>
__global__ __launch_bounds__(OCX_BLOCK) void ocx_exact_ball_kernel(
    RowSrc rs, int64_t B, int64_t NP, double* __restrict__ actions, double* __restrict__ obj_out,
    double* __restrict__ gap_out, double* __restrict__ step_loss, int32_t* __restrict__ info_out) {
    constexpr int NH = D * (D + 1) / 2;
    const int lane = threadIdx.x & 63;
    const int64_t p = ocx_wave_id();
    if (p >= B * NP) return;
    const int64_t T = rs.T;
    const int64_t b = p % B;
    const int64_t n = T - p / B;  // longest problems first: T, T-1, …, T-NP+1
    const int64_t slot = NP == 1 ? 0 : n;

    double x[D], u[D];
#pragma unroll
    for (int j = 0; j < D; ++j) {
        x[j] = 0.0;
        u[j] = NORM == 1 ? 0.5 / D : 0.0;
    }
    double mu = kMu0;
    int it = 0, kend = 0;
    bool conv = n == 0, broke = false;  // the empty prefix: x = 0, as compute_prefix_actions (:296-298) sets it
    while (!conv && it < kMaxIter) {
        ++it;
        double G[D], H[NH];
#pragma unroll
        for (int j = 0; j < D; ++j) G[j] = 0.0;
#pragma unroll
        for (int j = 0; j < NH; ++j) H[j] = 0.0;
        for (int64_t i = lane; i < n; i += 64) {
            double a[D], yi;
            load_row<D>(rs, b, i, a, yi);
            double r = -yi;
#pragma unroll
            for (int j = 0; j < D; ++j) r = __builtin_fma(a[j], x[j], r);
            const double rt = sqrt(__builtin_fma(mu, mu, r * r));
            const double s = mu + rt;
            const double inv = 1.0 / (s * rt);
            const double g1 = r * rt * inv;  // r / s
            const double h1 = mu * inv;      // μ / (s·rt)
#pragma unroll
            for (int j = 0; j < D; ++j) G[j] = __builtin_fma(g1, a[j], G[j]);
#pragma unroll
            for (int j = 0; j < D; ++j) {
                const double w = h1 * a[j];
#pragma unroll
                for (int k = 0; k <= j; ++k) H[tri(j, k)] = __builtin_fma(w, a[k], H[tri(j, k)]);
            }
        }
        const double im = 1.0 / mu;
#pragma unroll
        for (int j = 0; j < D; ++j) G[j] = wave_total(G[j]) * im;
#pragma unroll
        for (int j = 0; j < NH; ++j) H[j] = wave_total(H[j]) * im;

        // ball barrier, Newton direction, decrement
        double dx[D], du[D], lam2 = 0.0;
        if constexpr (NORM == 0) {
            double q = 1.0;
#pragma unroll
            for (int j = 0; j < D; ++j) q = __builtin_fma(-x[j], x[j], q);
            const double iq = 1.0 / q, c2 = 2.0 * iq, c4 = 4.0 * iq * iq;
#pragma unroll
            for (int j = 0; j < D; ++j) {
                G[j] = __builtin_fma(c2, x[j], G[j]);
#pragma unroll
                for (int k = 0; k <= j; ++k) H[tri(j, k)] += c4 * x[j] * x[k] + (j == k ? c2 : 0.0);
            }
            spd_solve<D>(H, G, dx);
#pragma unroll
            for (int j = 0; j < D; ++j) lam2 = __builtin_fma(-G[j], dx[j], lam2);
        } else if constexpr (NORM == 2) {
#pragma unroll
            for (int j = 0; j < D; ++j) {
                const double iq = 1.0 / __builtin_fma(-x[j], x[j], 1.0);
                G[j] = __builtin_fma(2.0 * x[j], iq, G[j]);
                H[tri(j, j)] += 2.0 * __builtin_fma(x[j], x[j], 1.0) * iq * iq;
            }
            spd_solve<D>(H, G, dx);
#pragma unroll
            for (int j = 0; j < D; ++j) lam2 = __builtin_fma(-G[j], dx[j], lam2);
        } else {
            // l1: (x, u) with p = u − x, pp = u + x, w = 1 − Σu.  Huu = diag(α) + c 11ᵀ,
            // Hxu = diag(β); Schur complement S = Hxx − Hxu Huu⁻¹ Hxu (Sherman–Morrison).
            double su = 0.0;
#pragma unroll
            for (int j = 0; j < D; ++j) su += u[j];
            const double iw = 1.0 / (1.0 - su), c = iw * iw;
            double al[D], be[D], gu[D], ia[D];
            double sia = 0.0;
#pragma unroll
            for (int j = 0; j < D; ++j) {
                const double ip = 1.0 / (u[j] - x[j]), ipp = 1.0 / (u[j] + x[j]);
                G[j] += ip - ipp;
                gu[j] = iw - ip - ipp;
                al[j] = __builtin_fma(ip, ip, ipp * ipp);
                be[j] = (ipp - ip) * (ipp + ip);  // exactly 0 where x_j = 0
                ia[j] = 1.0 / al[j];
                sia += ia[j];
            }
            const double gam = c / __builtin_fma(c, sia, 1.0);
            // Huu⁻¹ gu = gu/α − γ (Σ gu_j/α_j) / α
            double t = 0.0;
#pragma unroll
            for (int j = 0; j < D; ++j) t = __builtin_fma(gu[j], ia[j], t);
            double gt[D], v[D];
#pragma unroll
            for (int j = 0; j < D; ++j) {
                const double hg = (gu[j] - gam * t) * ia[j];
                gt[j] = __builtin_fma(-be[j], hg, G[j]);
                v[j] = be[j] * ia[j];
            }
#pragma unroll
            for (int j = 0; j < D; ++j) {
                H[tri(j, j)] += __builtin_fma(-be[j], v[j], al[j]);
#pragma unroll
                for (int k = 0; k <= j; ++k) H[tri(j, k)] += gam * v[j] * v[k];
            }
            spd_solve<D>(H, gt, dx);
            // du = Huu⁻¹ (−gu − β∘dx)
            double rhs[D];
            double tr = 0.0;
#pragma unroll
            for (int j = 0; j < D; ++j) {
                rhs[j] = __builtin_fma(-be[j], dx[j], -gu[j]);
                tr = __builtin_fma(rhs[j], ia[j], tr);
            }
#pragma unroll
            for (int j = 0; j < D; ++j) du[j] = (rhs[j] - gam * tr) * ia[j];
#pragma unroll
            for (int j = 0; j < D; ++j) {
                lam2 = __builtin_fma(-G[j], dx[j], lam2);
                lam2 = __builtin_fma(-gu[j], du[j], lam2);
            }
        }
        const double lam = sqrt(lam2 > 0.0 ? lam2 : 0.0);
        if (lam > kBreakdown) {
            // μ has outrun fp64: with the optimal face's directions pinned only by the
            // O(1) ball barrier and the active rows' curvature ~1/μ², the floored Cholesky
            // returns garbage (λ ~1e19).  The iterate is the last centre, accurate to that
            // μ (the certificate below says how well): stop there, marked as such
            // (OCX_EXACT_INFO_BREAKDOWN) — not a converged solve.
            broke = true;
            break;
        }
        double step = lam > 0.25 ? 1.0 / (1.0 + lam) : 1.0;
        // damped Newton stays in the domain in exact arithmetic; the floored pivots do
        // not promise it, so check and halve
        for (int h = 0; h < 60; ++h) {
            double xn[D], un[D];
#pragma unroll
            for (int j = 0; j < D; ++j) {
                xn[j] = __builtin_fma(step, dx[j], x[j]);
                un[j] = NORM == 1 ? __builtin_fma(step, du[j], u[j]) : 0.0;
            }
            if (in_domain<D, NORM>(xn, un)) {
#pragma unroll
                for (int j = 0; j < D; ++j) {
                    x[j] = xn[j];
                    u[j] = un[j];
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

    // certificate: obj = ½Σ|r|, dual bounds of λ_a = r/(2s) and λ_b (inactive rows ±½)
    double P = 0.0, Ya = 0.0, Yb = 0.0, Wa[D], Wb[D];
#pragma unroll
    for (int j = 0; j < D; ++j) Wa[j] = Wb[j] = 0.0;
    for (int64_t i = lane; i < n; i += 64) {
        double a[D], yi;
        load_row<D>(rs, b, i, a, yi);
        double r = -yi;
#pragma unroll
        for (int j = 0; j < D; ++j) r = __builtin_fma(a[j], x[j], r);
        P += 0.5 * fabs(r);
        const double s = mu + sqrt(__builtin_fma(mu, mu, r * r));
        const double la = 0.5 * r / s;
        const double lb = fabs(r) > 1e3 * mu ? (r > 0.0 ? 0.5 : -0.5) : la;
        Ya = __builtin_fma(la, yi, Ya);
        Yb = __builtin_fma(lb, yi, Yb);
#pragma unroll
        for (int j = 0; j < D; ++j) {
            Wa[j] = __builtin_fma(la, a[j], Wa[j]);
            Wb[j] = __builtin_fma(lb, a[j], Wb[j]);
        }
    }
    P = wave_total(P);
    Ya = wave_total(Ya);
    Yb = wave_total(Yb);
    double na = 0.0, nb = 0.0;  // dual norms of Zᵀλ
#pragma unroll
    for (int j = 0; j < D; ++j) {
        const double wa = wave_total(Wa[j]), wb = wave_total(Wb[j]);
        if constexpr (NORM == 0) {
            na = __builtin_fma(wa, wa, na);
            nb = __builtin_fma(wb, wb, nb);
        } else if constexpr (NORM == 2) {
            na += fabs(wa);
            nb += fabs(wb);
        } else {
            na = fmax(na, fabs(wa));
            nb = fmax(nb, fabs(wb));
        }
    }
    if constexpr (NORM == 0) {
        na = sqrt(na);
        nb = sqrt(nb);
    }
    // λ = 0 is feasible too (bound 0): it certifies the zero-loss prefixes (n < d rows
    // interpolated exactly) where a solve stopped early leaves the barrier's λ far off
    const double bound = fmax(fmax(-Ya - na, -Yb - nb), 0.0);
    if (lane == 0) {
        double* xo = actions + (b * NP + slot) * D;
#pragma unroll
        for (int j = 0; j < D; ++j) xo[j] = x[j];
        if (obj_out) obj_out[b * NP + slot] = P;
        if (gap_out) gap_out[b * NP + slot] = fmax(P - bound, 0.0);
        if (info_out)
            info_out[b * NP + slot] = broke ? (OCX_EXACT_INFO_BREAKDOWN | it) : (conv ? it : -it);
        if (step_loss) {
            // FTL's loss at step n with this action (replay_exact_ftl, exact_ftl.py:318-323:
            // _dot's sequential sum, then the normalized hinge); 0 for the full prefix
            double lo = 0.0;
            if (n < T) {
                double a[D], yi;
                load_row<D>(rs, b, n, a, yi);
                double q = 0.0;
#pragma unroll
                for (int j = 0; j < D; ++j) q = q + a[j] * x[j];
                lo = 0.5 * fabs(q - yi);
            }
            step_loss[b * NP + slot] = lo;
        }
    }
}

template <int D, int NORM>
hipError_t launch_dn(const RowSrc& rs, int64_t B, int64_t NP, double* actions, double* obj,
                     double* gap, double* step_loss, int32_t* info, hipStream_t st) {
    const int64_t G = B * NP;
    const int wpb = ocx_block_waves(G);
    hipLaunchKernelGGL((ocx_exact_ball_kernel<D, NORM>), ocx_grid(G, wpb), dim3(64 * wpb), 0, st, rs,
                       B, NP, actions, obj, gap, step_loss, info);
    return hipGetLastError();
}

template <int D>
hipError_t launch_d(const RowSrc& rs, int64_t B, int64_t NP, int norm, double* actions,
                    double* obj, double* gap, double* step_loss, int32_t* info, hipStream_t st) {
    switch (norm) {
        case 0: return launch_dn<D, 0>(rs, B, NP, actions, obj, gap, step_loss, info, st);
        case 1: return launch_dn<D, 1>(rs, B, NP, actions, obj, gap, step_loss, info, st);
        case 2: return launch_dn<D, 2>(rs, B, NP, actions, obj, gap, step_loss, info, st);
        default: return hipErrorInvalidValue;
    }
}

hipError_t solve(const RowSrc& rs, int64_t B, int64_t d, int norm, int all_prefixes,
                 double* actions, double* obj, double* gap, double* step_loss, int32_t* info,
                 hipStream_t st) {
    const int64_t NP = all_prefixes ? rs.T + 1 : 1;
    if (B == 0 || NP == 0) return hipSuccess;
    switch (d) {
#define OCX_EB_CASE(D) \
    case D: return launch_d<D>(rs, B, NP, norm, actions, obj, gap, step_loss, info, st);
        OCX_EB_CASE(1) OCX_EB_CASE(2) OCX_EB_CASE(3) OCX_EB_CASE(4) OCX_EB_CASE(5)
        OCX_EB_CASE(6) OCX_EB_CASE(7) OCX_EB_CASE(8) OCX_EB_CASE(9) OCX_EB_CASE(10)
#undef OCX_EB_CASE
        default:
            // 64 < d <= 256: the system in HBM scratch, the solve and its polish
            // (ocx_exact_big.hip)
            if (d > 64)
                return ocx_launch_exact_big(rs.z, rs.y, B, rs.T, d, rs.tiled, rs.P, rs.C, rs.S,
                                            rs.G, norm, all_prefixes, actions, obj, gap,
                                            step_loss, info, st);
            // 10 < d <= 64: the system in LDS, one coordinate per lane (ocx_exact_wide.hip)
            return ocx_launch_exact_wide(rs.z, rs.y, B, rs.T, d, rs.tiled, rs.P, rs.C, rs.S, rs.G,
                                         norm, all_prefixes, actions, obj, gap, step_loss, info,
                                         st);
    }
}

// the solve, then its certificate polished (ocx_launch_exact_polish)
hipError_t launch(const RowSrc& rs, int64_t B, int64_t d, int norm, int all_prefixes,
                  double* actions, double* obj, double* gap, double* step_loss, int32_t* info,
                  hipStream_t st) {
    const hipError_t e = solve(rs, B, d, norm, all_prefixes, actions, obj, gap, step_loss, info, st);
    if (e != hipSuccess || d > 64) return e;  // ocx_launch_exact_big polishes its own solves
    return ocx_launch_exact_polish(rs.z, rs.y, B, rs.T, d, rs.tiled, rs.P, rs.C, rs.S, rs.G, norm,
                                   all_prefixes, actions, obj, gap, step_loss, st);
}

}  // namespace

hipError_t ocx_launch_exact_ball(const double* z, const double* y, int64_t B, int64_t T,
                                 int64_t d, int norm, int all_prefixes, double* actions,
                                 double* obj, double* gap, double* step_loss, int32_t* info,
                                 hipStream_t st) {
    const RowSrc rs{z, y, T, 0, 1, 1, 1, 0};
    return launch(rs, B, d, norm, all_prefixes, actions, obj, gap, step_loss, info, st);
}

hipError_t ocx_launch_exact_ball_tiled(const ocx_layout* L, const double* zt, const double* yt,
                                       int norm, int all_prefixes, double* actions, double* obj,
                                       double* gap, double* step_loss, int32_t* info,
                                       hipStream_t st) {
    const RowSrc rs{zt, yt, L->T, L->G, L->P, L->C, L->S, 1};
    return launch(rs, L->B, L->d, norm, all_prefixes, actions, obj, gap, step_loss, info, st);
}
