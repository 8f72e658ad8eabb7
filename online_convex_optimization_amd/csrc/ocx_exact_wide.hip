// ocx_exact_wide.hip — the general exact-FTL comparator (ExactFTLNoClip, exact_ftl.py:83-105,
// solved by cvxpy at :119-128) for 10 < d <= 64: the same primal log-barrier path as
// ocx_exact_ball.hip (same barrier, schedule, damping, certificate; see that file), laid out
// for a d × d Newton system that no longer fits one lane's registers.
//
// One wavefront per problem (sequence b, prefix n), DP = 16 / 32 / 64 padded coordinates:
//   * coordinate vectors (x, u, the gradient, the step) live one coordinate per lane;
//   * the Hessian Σ_i h_i a_i a_iᵀ is accumulated as an 8 × 8 grid of (DP/8)² blocks, lane
//     8·bj + bk owning rows bj·DP/8.., columns bk·DP/8.. — (DP/8)² fp64 FMAs per row and lane;
//   * rows are staged through LDS 64 at a time (one coalesced read of the chunk; lane r then
//     forms row r's residual and barrier weights, which reach the other lanes through LDS);
//   * the system is factorised in LDS (Jacobi-scaled right-looking Cholesky, pivots floored
//     at 1e-13; lane i owns row i) and solved by column sweeps.
// Padded coordinates (d <= j < DP) carry x_j = 0, a unit diagonal and no barrier term, so
// their steps are 0.  This is a compute kernel: ≈50–100 Newton passes over each prefix's
// rows (from L2), bound by the VALU.
#include <algorithm>

#include "ocx_exact_src.h"
#include "ocx_internal.h"
#include "ocx_sim_kernels.h"

namespace {

constexpr int kMaxIter = 300;
constexpr double kMu0 = 1.0;
constexpr double kMuEnd = 1e-10;
constexpr double kKappa = 10.0;
constexpr double kTolCenter = 1.0;
constexpr double kTolFinal = 1e-6;
constexpr int kFinalSteps = 6;
constexpr double kPivotFloor = 1e-13;
constexpr double kBreakdown = 1e8;
constexpr int RC = 64;  // rows per staged chunk

__device__ __forceinline__ double wsum(double v) { return ocx_seq_sum<64>(v); }

// Lanes hand values to each other through LDS (staged rows, row weights, the system and its
// factor): every publish is followed by a barrier.  The block is one wave, so s_barrier
// costs little; it orders the LDS traffic for the compiler as the memory model requires,
// instead of relying on the wave's lockstep.
__device__ __forceinline__ void lds_sync() { __syncthreads(); }

template <int DP, int NORM>
__global__ __launch_bounds__(64) void ocx_exact_wide_kernel(
    WideSrc rs, int64_t B, int64_t NP, int64_t p0, double* __restrict__ actions,
    double* __restrict__ obj_out, double* __restrict__ gap_out, double* __restrict__ step_loss,
    int32_t* __restrict__ info_out) {
    constexpr int BS = DP / 8;       // block edge per lane
    constexpr int LD = DP + 1;       // LDS row stride (odd: conflict-free columns and rows)
    extern __shared__ double lds[];
    double* M = lds;                 // [RC][LD] row chunk, then [DP][LD] the system
    double* xs = M + RC * LD;        // x (then the direction vector of a rank-1 term)
    double* gw = xs + 64;            // row weights r/s
    double* hw = gw + 64;            // row weights μ/(s·rt)
    double* vv = hw + 64;            // rank-1 / diagonal terms of the ball barrier
    double* sc = vv + 64;            // Jacobi scales

    const int lane = threadIdx.x & 63;
    const int64_t p = p0 + blockIdx.x;
    if (p >= B * NP) return;
    const int d = rs.d;
    const int64_t T = rs.T;
    const int64_t b = p % B;
    const int64_t n = T - p / B;  // longest problems first
    const int64_t slot = NP == 1 ? 0 : n;
    const bool cj = lane < d;     // this lane's coordinate is real
    const int bj = lane >> 3, bk = lane & 7;

    double x = 0.0, u = (NORM == 1 && cj) ? 0.5 / d : 0.0;
    double mu = kMu0;
    int it = 0, kend = 0;
    bool conv = n == 0, broke = false;

    // Stage rows [c0, c0 + rows) into M (zero-padded to DP columns) and y into yv (lane r).
    auto stage = [&](int64_t c0, int rows, double& yv) {
        lds_sync();  // the previous chunk's readers are done with M
        const int tot = rows * d;
        for (int f = lane; f < tot; f += 64) {
            const int r = f / d, j = f - r * d;
            M[r * LD + j] = rs.zat(b, c0 + r, j);
        }
        if (DP > d)
            for (int f = lane; f < rows * (DP - d); f += 64) {
                const int r = f / (DP - d), j = d + (f - r * (DP - d));
                M[r * LD + j] = 0.0;
            }
        yv = lane < rows ? rs.yat(b, c0 + lane) : 0.0;
        lds_sync();
    };
    // row r's residual z_r·x − y_r (lane r), in _dot's order from −y
    auto residual = [&](int r, double yv) {
        double rr = -yv;
        for (int j = 0; j < d; ++j) rr = __builtin_fma(M[r * LD + j], xs[j], rr);
        return rr;
    };

    while (!conv && it < kMaxIter) {
        ++it;
        lds_sync();  // the last pass's readers of xs are done
        xs[lane] = x;
        double Gj = 0.0;
        double H[BS][BS];
#pragma unroll
        for (int i = 0; i < BS; ++i)
#pragma unroll
            for (int k = 0; k < BS; ++k) H[i][k] = 0.0;
        for (int64_t c0 = 0; c0 < n; c0 += RC) {
            const int rows = (int)(n - c0 < RC ? n - c0 : RC);
            double yv;
            stage(c0, rows, yv);
            double g1 = 0.0, h1 = 0.0;
            if (lane < rows) {
                const double r = residual(lane, yv);
                const double rt = sqrt(__builtin_fma(mu, mu, r * r));
                const double s = mu + rt;
                const double inv = 1.0 / (s * rt);
                g1 = r * rt * inv;  // r / s
                h1 = mu * inv;      // μ / (s·rt)
            }
            gw[lane] = g1;
            hw[lane] = h1;
            lds_sync();
            for (int r = 0; r < rows; ++r) {
                Gj = __builtin_fma(gw[r], M[r * LD + (lane < DP ? lane : 0)], Gj);
                double a1[BS], a2[BS];
#pragma unroll
                for (int i = 0; i < BS; ++i) {
                    a1[i] = hw[r] * M[r * LD + bj * BS + i];
                    a2[i] = M[r * LD + bk * BS + i];
                }
#pragma unroll
                for (int i = 0; i < BS; ++i)
#pragma unroll
                    for (int k = 0; k < BS; ++k) H[i][k] = __builtin_fma(a1[i], a2[k], H[i][k]);
            }
        }
        const double im = 1.0 / mu;
        Gj = cj ? Gj * im : 0.0;
#pragma unroll
        for (int i = 0; i < BS; ++i)
#pragma unroll
            for (int k = 0; k < BS; ++k) H[i][k] *= im;

        // ---- the ball's barrier: gradient (lane j), diagonal (vv) and a rank-1 term
        // (xs = its vector, c1 its weight), then the system into M
        double c1 = 0.0, gu = 0.0, ia = 0.0, be = 0.0, gam = 0.0;
        double rhs_g;  // right-hand side of the x system
        if constexpr (NORM == 0) {
            const double q = 1.0 - wsum(cj ? x * x : 0.0);
            const double iq = 1.0 / q;
            Gj = cj ? __builtin_fma(2.0 * iq, x, Gj) : 0.0;
            vv[lane] = cj ? 2.0 * iq : 1.0;  // padded coordinates: unit diagonal
            c1 = 4.0 * iq * iq;
            xs[lane] = cj ? x : 0.0;
            rhs_g = Gj;
        } else if constexpr (NORM == 2) {
            const double iq = cj ? 1.0 / __builtin_fma(-x, x, 1.0) : 0.0;
            Gj = cj ? __builtin_fma(2.0 * x, iq, Gj) : 0.0;
            vv[lane] = cj ? 2.0 * __builtin_fma(x, x, 1.0) * iq * iq : 1.0;
            xs[lane] = 0.0;
            rhs_g = Gj;
        } else {
            const double su = wsum(cj ? u : 0.0);
            const double iw = 1.0 / (1.0 - su), c = iw * iw;
            double al = 1.0;
            if (cj) {
                const double ip = 1.0 / (u - x), ipp = 1.0 / (u + x);
                Gj += ip - ipp;
                gu = iw - ip - ipp;
                al = __builtin_fma(ip, ip, ipp * ipp);
                be = (ipp - ip) * (ipp + ip);
                ia = 1.0 / al;
            }
            gam = c / __builtin_fma(c, wsum(ia), 1.0);
            const double t = wsum(gu * ia);
            const double hg = (gu - gam * t) * ia;
            rhs_g = cj ? __builtin_fma(-be, hg, Gj) : 0.0;
            const double v = be * ia;
            vv[lane] = cj ? __builtin_fma(-be, v, al) : 1.0;
            xs[lane] = v;
            c1 = gam;
        }
        lds_sync();  // vv, xs published; the last chunk's reads of M are done
        // H + diag(vv) + c1·xs xsᵀ into M (full matrix)
#pragma unroll
        for (int i = 0; i < BS; ++i) {
            const int gi = bj * BS + i;
#pragma unroll
            for (int k = 0; k < BS; ++k) {
                const int gk = bk * BS + k;
                double h = gi < d && gk < d ? H[i][k] : 0.0;
                h = __builtin_fma(c1 * xs[gi], xs[gk], h);
                if (gi == gk) h += vv[gi];
                M[gi * LD + gk] = h;
            }
        }
        lds_sync();
        // Jacobi scaling, then Cholesky (lane i owns row i)
        const int ri = lane < DP ? lane : DP - 1;
        const double dg = M[ri * LD + ri];
        const double sci = 1.0 / sqrt(dg > 0.0 ? dg : kPivotFloor);
        sc[lane] = sci;
        lds_sync();
        if (lane < DP)
            for (int j = 0; j <= lane; ++j) M[lane * LD + j] *= sci * sc[j];
        lds_sync();
        for (int k = 0; k < DP; ++k) {
            double s = M[k * LD + k];
            s = s > kPivotFloor ? s : kPivotFloor;
            const double l = sqrt(s), rd = 1.0 / l;
            double lik = 0.0;
            if (lane > k && lane < DP) lik = M[lane * LD + k] * rd;
            lds_sync();  // every lane has read row k's diagonal before lane k rewrites it
            if (lane == k) M[k * LD + k] = l;
            if (lane > k && lane < DP) M[lane * LD + k] = lik;
            lds_sync();  // column k of the factor published
            if (lane > k && lane < DP)
                for (int j = k + 1; j <= lane; ++j)
                    M[lane * LD + j] = __builtin_fma(-lik, M[j * LD + k], M[lane * LD + j]);
        }
        lds_sync();
        // L w = rhs·sc ; Lᵀ v = −w ; dx = v·sc
        double vcur = lane < DP ? rhs_g * sci : 0.0, w = 0.0;
        for (int k = 0; k < DP; ++k) {
            const double wk = ocx_readlane(vcur, k) / M[k * LD + k];
            if (lane == k) w = wk;
            if (lane > k && lane < DP) vcur = __builtin_fma(-M[lane * LD + k], wk, vcur);
        }
        double vb = -w, dx = 0.0;
        for (int k = DP - 1; k >= 0; --k) {
            const double dk = ocx_readlane(vb, k) / M[k * LD + k];
            if (lane == k) dx = dk;
            if (lane < k) vb = __builtin_fma(-M[k * LD + lane], dk, vb);
        }
        dx = cj ? dx * sci : 0.0;
        double du = 0.0, lam2;
        if constexpr (NORM == 1) {
            const double rhs = cj ? __builtin_fma(-be, dx, -gu) : 0.0;
            const double tr = wsum(rhs * ia);
            du = cj ? (rhs - gam * tr) * ia : 0.0;
            lam2 = wsum(__builtin_fma(-Gj, dx, -gu * du));
        } else {
            lam2 = wsum(-Gj * dx);
        }
        const double lam = sqrt(lam2 > 0.0 ? lam2 : 0.0);
        if (lam > kBreakdown) {  // μ has outrun fp64 (see ocx_exact_ball.hip)
            broke = true;
            break;
        }
        double step = lam > 0.25 ? 1.0 / (1.0 + lam) : 1.0;
        for (int h = 0; h < 60; ++h) {
            const double xn = __builtin_fma(step, dx, x);
            const double un = NORM == 1 ? __builtin_fma(step, du, u) : 0.0;
            bool ok;
            if constexpr (NORM == 0) {
                ok = wsum(cj ? xn * xn : 0.0) < 1.0;
            } else if constexpr (NORM == 2) {
                ok = __ballot(cj && !(fabs(xn) < 1.0)) == 0;
            } else {
                ok = __ballot(cj && !(fabs(xn) < un)) == 0 && wsum(cj ? un : 0.0) < 1.0;
            }
            if (ok) {
                x = xn;
                u = un;
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

    // ---- certificate (as ocx_exact_ball.hip): obj, dual bounds of λ_a = r/(2s) and λ_b
    lds_sync();
    xs[lane] = x;
    double P = 0.0, Ya = 0.0, Yb = 0.0, Wa = 0.0, Wb = 0.0;
    for (int64_t c0 = 0; c0 < n; c0 += RC) {
        const int rows = (int)(n - c0 < RC ? n - c0 : RC);
        double yv;
        stage(c0, rows, yv);
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
            const double a = M[r * LD + (lane < DP ? lane : 0)];
            Wa = __builtin_fma(gw[r], a, Wa);
            Wb = __builtin_fma(hw[r], a, Wb);
        }
    }
    P = wsum(P);
    Ya = wsum(Ya);
    Yb = wsum(Yb);
    if (!cj) Wa = Wb = 0.0;
    double na, nb;
    if constexpr (NORM == 0) {
        na = sqrt(wsum(Wa * Wa));
        nb = sqrt(wsum(Wb * Wb));
    } else if constexpr (NORM == 2) {
        na = wsum(fabs(Wa));
        nb = wsum(fabs(Wb));
    } else {
        double ma = fabs(Wa), mb = fabs(Wb);
        for (int o = 32; o > 0; o >>= 1) {
            ma = fmax(ma, __shfl_xor(ma, o, 64));
            mb = fmax(mb, __shfl_xor(mb, o, 64));
        }
        na = ma;
        nb = mb;
    }
    const double bound = fmax(fmax(-Ya - na, -Yb - nb), 0.0);
    if (cj) actions[(b * NP + slot) * d + lane] = x;
    if (lane == 0) {
        if (obj_out) obj_out[b * NP + slot] = P;
        if (gap_out) gap_out[b * NP + slot] = fmax(P - bound, 0.0);
        if (info_out)
            info_out[b * NP + slot] = broke ? (OCX_EXACT_INFO_BREAKDOWN | it) : (conv ? it : -it);
        if (step_loss) {
            // FTL's loss at step n (replay_exact_ftl :318-323: _dot's sequential sum)
            double lo = 0.0;
            if (n < T) {
                double q = 0.0;
                for (int j = 0; j < d; ++j) q = q + rs.zat(b, n, j) * xs[j];
                lo = 0.5 * fabs(q - rs.yat(b, n));
            }
            step_loss[b * NP + slot] = lo;
        }
    }
}

template <int DP, int NORM>
hipError_t launch_wide_dn(const WideSrc& rs, int64_t B, int64_t NP, double* actions, double* obj,
                          double* gap, double* step_loss, int32_t* info, hipStream_t st) {
    const size_t lds = (size_t)(RC * (DP + 1) + 5 * 64) * sizeof(double);
    // one 64-thread block per problem, launched in slices: a launch may hold at most 2^32 - 1
    // threads along x
    const int64_t total = B * NP, slice = (int64_t)1 << 24;
    for (int64_t p0 = 0; p0 < total; p0 += slice) {
        hipLaunchKernelGGL((ocx_exact_wide_kernel<DP, NORM>), dim3((unsigned)std::min(slice, total - p0)),
                           dim3(64), lds, st, rs, B, NP, p0, actions, obj, gap, step_loss, info);
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

template <int DP>
hipError_t launch_wide_d(const WideSrc& rs, int64_t B, int64_t NP, int norm, double* actions,
                         double* obj, double* gap, double* step_loss, int32_t* info,
                         hipStream_t st) {
    switch (norm) {
        case 0: return launch_wide_dn<DP, 0>(rs, B, NP, actions, obj, gap, step_loss, info, st);
        case 1: return launch_wide_dn<DP, 1>(rs, B, NP, actions, obj, gap, step_loss, info, st);
        case 2: return launch_wide_dn<DP, 2>(rs, B, NP, actions, obj, gap, step_loss, info, st);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace

// 10 < d <= 64, row-major (tiled = 0) or the tiled layout (P, C, S, G of it)
hipError_t ocx_launch_exact_wide(const double* z, const double* y, int64_t B, int64_t T,
                                 int64_t d, int tiled, int P, int C, int S, int64_t G, int norm,
                                 int all_prefixes, double* actions, double* obj, double* gap,
                                 double* step_loss, int32_t* info, hipStream_t st) {
    const int64_t NP = all_prefixes ? T + 1 : 1;
    if (B == 0 || NP == 0) return hipSuccess;
    if (d < 1 || d > 64 || B > ((int64_t)1 << 40) / std::max<int64_t>(NP, 1)) return hipErrorInvalidValue;
    const WideSrc rs{z, y, T, G, (int)d, P, C, S, tiled};
    if (d <= 16) return launch_wide_d<16>(rs, B, NP, norm, actions, obj, gap, step_loss, info, st);
    if (d <= 32) return launch_wide_d<32>(rs, B, NP, norm, actions, obj, gap, step_loss, info, st);
    return launch_wide_d<64>(rs, B, NP, norm, actions, obj, gap, step_loss, info, st);
}

namespace {

// ---------------------------------------------------------------------------------------------
// Certificate polish (both general solvers, d <= 64): the solver's x purified onto the face its
// active constraints define, and a dual rebuilt from the KKT system there, so the gap
// certifies the objective to rounding.
//
// The barrier path stops at μ_end = 1e-10: its x sits about μ_end/|slope| inside the optimal
// face, and its multipliers λ_i = r_i/(2 s_i) are exact for the rows the optimum does not
// interpolate (±½) but only as good as μ_end for the ones it does.  Where the optimum
// interpolates rows (n > d real-valued rows: an LAD vertex; n < d rows fitted exactly) the
// barrier certificate stayed near 1e-5 relative, and a zero-loss prefix kept ½Σ|r_i| ≈ 5e-8.
// For each of eleven threshold pairs (τ_x, τ_r) = (1e-8·s, 1e-7·s) for seven scales s, then
// four with the coordinates' and the rows' scales apart — a near-degenerate bound (normal-cone
// multiplier ν ≪ 1) leaves x about μ_end/ν = 1e-6 inside it while every interpolated row is
// tight to 1e-9, so no joint scale finds both (round 6, d = 100 linf) — the best is kept and
// every bound is valid:
//   1. active set at x: rows with |r_i| <= τ_r (1 + |y_i|) (at most 64, 63 beside the cone
//      row), and the ball's
//      constraints that hold: l2 ||x|| = 1; linf |x_j| = 1 (those coordinates fixed at ±1);
//      l1 ||x||_1 = 1 (the zero coordinates fixed at 0, the others keep their signs);
//   2. primal purification: the least-change step δ (minimum norm over the free coordinates)
//      that makes the active rows' residuals and the tight constraint (l2: linearised) hold
//      exactly, x' = x + δ projected into the ball, kept only if ½Σ|r| does not grow;
//   3. dual at x': λ_i = ½ sign(r_i) off the active set, and on it the least-squares solution
//      of stationarity Σ_A λ_i z_i = −g − w (g the other rows' part, w in the ball's normal
//      cone: l2 ν x, l1 ν sign(x) on the support, linf free on the fixed coordinates), clipped
//      to [−½, ½]; D = −λ·y − ||Zᵀλ||_* (weak duality: a bound whatever the λ in the box).
// If the best scale certifies a smaller gap than the solver's, x', its objective, the gap and
// the prefix's step loss replace the solver's.  One wave per problem; the small systems by
// the solver's LDS Cholesky.
__device__ void polish_cholesky_solve(double* K, double* sc, int lane, double rhs, double& out) {
    // K: [64][65] SPD (identity past the system), rhs on lane k; out = K⁻¹ rhs on lane k
    constexpr int DP = 64, LD = 65;
    const double dg = K[lane * LD + lane];
    const double sci = 1.0 / sqrt(dg > 0.0 ? dg : kPivotFloor);
    sc[lane] = sci;
    lds_sync();
    for (int j = 0; j <= lane; ++j) K[lane * LD + j] *= sci * sc[j];
    lds_sync();
    for (int k = 0; k < DP; ++k) {
        double s = K[k * LD + k];
        s = s > kPivotFloor ? s : kPivotFloor;
        const double l = sqrt(s), rd = 1.0 / l;
        double lik = 0.0;
        if (lane > k) lik = K[lane * LD + k] * rd;
        lds_sync();
        if (lane == k) K[k * LD + k] = l;
        if (lane > k) K[lane * LD + k] = lik;
        lds_sync();
        if (lane > k)
            for (int j = k + 1; j <= lane; ++j)
                K[lane * LD + j] = __builtin_fma(-lik, K[j * LD + k], K[lane * LD + j]);
    }
    lds_sync();
    double vcur = rhs * sci, w = 0.0;
    for (int k = 0; k < DP; ++k) {
        const double wk = ocx_readlane(vcur, k) / K[k * LD + k];
        if (lane == k) w = wk;
        if (lane > k) vcur = __builtin_fma(-K[lane * LD + k], wk, vcur);
    }
    double vb = w, ck = 0.0;
    for (int k = DP - 1; k >= 0; --k) {
        const double dk = ocx_readlane(vb, k) / K[k * LD + k];
        if (lane == k) ck = dk;
        if (lane < k) vb = __builtin_fma(-K[k * LD + lane], dk, vb);
    }
    out = ck * sci;
    lds_sync();
}

// The bar under which the polish keeps the solver's own x: a decade inside the host's
// acceptance bar (engine.EXACT_GAP_RTOL = 1e-8), so a kept x always passes it.
constexpr double kKeepRtol = 1e-9;
// threshold sweeps: seven joint scales, then four with the coordinates' and rows' apart
constexpr int kSweeps = 11;

template <int NORM>
__global__ __launch_bounds__(64) void ocx_exact_polish_kernel(
    WideSrc rs, int64_t B, int64_t NP, int64_t p0, double* __restrict__ actions,
    double* __restrict__ obj, double* __restrict__ gap, double* __restrict__ step_loss) {
    constexpr int DP = 64, LD = DP + 1;
    extern __shared__ double lds[];
    double* M = lds;             // [64][LD] the active rows (+ the cone row)
    double* K = M + DP * LD;     // [64][LD] staged rows during passes; the small systems
    double* xs = K + DP * LD;    // x, then x'
    double* wv = xs + 64;        // per-row weights of a staged chunk
    double* gs = wv + 64;        // g = Σ_{i∉A} λ_i z_i
    double* em = gs + 64;        // 1.0 where coordinate j's stationarity equation holds
    double* sc = em + 64;        // Jacobi scales / λ_A
    double* ra = sc + 64;        // active rows' residuals at x, then their y
    int* act = reinterpret_cast<int*>(ra + 64);  // active row indices

    const int lane = threadIdx.x & 63;
    const int64_t p = p0 + blockIdx.x;
    if (p >= B * NP) return;
    const int d = rs.d;
    const int64_t T = rs.T;
    const int64_t b = p % B;
    const int64_t n = T - p / B;
    const int64_t o = b * NP + (NP == 1 ? 0 : n);
    const double g0 = gap[o], f0 = obj[o];
    if (n == 0 || !(g0 > 0.0)) return;  // exact already (or a NaN the caller reports)
    const bool cj = lane < d;
    const double x = cj ? actions[o * d + lane] : 0.0;
    double best = g0, pbest = f0, xbest = x;
    bool improved = false;
    // the certificate of the solver's own x (P(x) - D, valid for any dual of the box): where it
    // passes, x — the path's analytic-centre limit ocx.h promises — is kept, not x'
    double bestx = g0, P0x = f0;

    // stage rows [c0, c0 + rows) into K; y into yv (lane r)
    auto stage = [&](int64_t c0, int rows, double& yv) {
        lds_sync();
        for (int f = lane; f < rows * d; f += 64) {
            const int r = f / d, j = f - r * d;
            K[r * LD + j] = rs.zat(b, c0 + r, j);
        }
        yv = lane < rows ? rs.yat(b, c0 + lane) : 0.0;
        lds_sync();
    };
    auto resid = [&](int r, double yv) {  // staged row r at xs, in _dot's order from −y
        double rr = -yv;
        for (int j = 0; j < d; ++j) rr = __builtin_fma(K[r * LD + j], xs[j], rr);
        return rr;
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
        bool cone = false, fixed = false;
        double tgt = 0.0, crow = 0.0;  // fixed coordinate's value; the cone row's entry
        if constexpr (NORM == 0) {
            cone = wsum(x * x) >= 1.0 - kTight;
            crow = 2.0 * x;
        } else if constexpr (NORM == 2) {
            fixed = cj && fabs(x) >= 1.0 - kTight;
            tgt = x > 0.0 ? 1.0 : -1.0;
        } else {
            cone = wsum(fabs(x)) >= 1.0 - kTight;
            if (cone) {
                fixed = cj && fabs(x) <= kZero;
                tgt = 0.0;
                crow = (cj && !fixed) ? (x > 0.0 ? 1.0 : -1.0) : 0.0;
            }
        }
        const bool freec = cj && !fixed;
        // active rows the [64][65] systems hold: 64, one fewer beside the cone row (d = 64: an
        // LAD vertex inside the ball interpolates 64 rows)
        const int AM = DP - (cone ? 1 : 0);
        const double vfix = fixed ? tgt - x : 0.0;  // δ_j on a fixed coordinate
        lds_sync();
        xs[lane] = x;
        em[lane] = freec ? 1.0 : 0.0;  // stationarity holds on the free coordinates
        // ---- pass 1 at x: ½Σ|r|, the active set and its residuals
        double P0 = 0.0;
        int m = 0;
        bool over = false;
        for (int64_t c0 = 0; c0 < n; c0 += RC) {
            const int rows = (int)(n - c0 < RC ? n - c0 : RC);
            double yv;
            stage(c0, rows, yv);
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
        P0 = wsum(P0);
        P0x = P0;
        const int mr = m + (cone ? 1 : 0);
        lds_sync();
        // ---- 2. primal purification: rows of the active set (+ the cone row) into M
        for (int f = lane; f < m * d; f += 64) {
            const int k = f / d, j = f - k * d;
            M[k * LD + j] = rs.zat(b, act[k], j);
        }
        if (cone) M[m * LD + lane] = cj ? crow : 0.0;
        sc[lane] = vfix;
        lds_sync();
        // right-hand sides: −r_k minus the fixed coordinates' part; the cone row's defect
        double rhs = 0.0;
        if (lane < m) {
            rhs = -ra[lane];
            for (int j = 0; j < d; ++j) rhs = __builtin_fma(-M[lane * LD + j], sc[j], rhs);
        }
        double defect;
        if constexpr (NORM == 0) defect = 1.0 - wsum(x * x);
        else defect = 1.0 - wsum(freec ? fabs(x) : 0.0);
        if (cone && lane == m) rhs = defect;
        // K = R_F R_Fᵀ over the free coordinates (+ ridge), identity past mr
        if (lane < mr)
            for (int l = 0; l < mr; ++l) {
                double s2 = 0.0;
                for (int j = 0; j < d; ++j) s2 = __builtin_fma(em[j] * M[lane * LD + j], M[l * LD + j], s2);
                K[lane * LD + l] = s2;
            }
        for (int l = (lane < mr ? mr : 0); l < DP; ++l) K[lane * LD + l] = (l == lane) ? 1.0 : 0.0;
        lds_sync();
        const double trK = wsum(lane < mr ? K[lane * LD + lane] : 0.0);
        if (lane < mr) K[lane * LD + lane] += 1e-13 * (trK / (mr > 0 ? mr : 1)) + 1e-300;
        lds_sync();
        double u = 0.0;
        polish_cholesky_solve(K, sc, lane, lane < mr ? rhs : 0.0, u);
        sc[lane] = lane < mr ? u : 0.0;
        lds_sync();
        double xn = x;
        if (cj) {
            if (fixed) {
                xn = tgt;
            } else {
                double dl = 0.0;
                for (int k = 0; k < mr; ++k) dl = __builtin_fma(M[k * LD + lane], sc[k], dl);
                xn = x + dl;
            }
        }
        // into the ball
        if constexpr (NORM == 0) {
            const double nn = sqrt(wsum(xn * xn));
            if (nn > 1.0) xn = xn / nn;
        } else if constexpr (NORM == 2) {
            xn = fmin(fmax(xn, -1.0), 1.0);
        } else {
            const double s1 = wsum(fabs(xn));
            if (s1 > 1.0) xn = xn / s1;
        }
        lds_sync();
        xs[lane] = xn;
        gs[lane] = 0.0;
        // ---- pass 2 at x': ½Σ|r'|, λ_i = ½ sign(r'_i) off the active set into g and λ·y
        double P1 = 0.0, Y = 0.0, gj = 0.0;
        int ia = 0;  // next entry of act[] (the active rows come in increasing order)
        for (int64_t c0 = 0; c0 < n; c0 += RC) {
            const int rows = (int)(n - c0 < RC ? n - c0 : RC);
            double yv;
            stage(c0, rows, yv);
            double lam = 0.0;
            bool isact = false;
            if (lane < rows) {
                const double rr = resid(lane, yv);
                P1 += 0.5 * fabs(rr);
                // membership of row c0 + lane in act[ia ..) (sorted)
                for (int k = ia; k < m && act[k] <= (int)(c0 + lane); ++k)
                    if (act[k] == (int)(c0 + lane)) isact = true;
                lam = isact ? 0.0 : (rr > 0.0 ? 0.5 : (rr < 0.0 ? -0.5 : 0.0));
                Y = __builtin_fma(lam, yv, Y);
            }
            while (ia < m && act[ia] < (int)(c0 + rows)) ++ia;
            wv[lane] = lam;
            lds_sync();
            if (cj)
                for (int r = 0; r < rows; ++r) gj = __builtin_fma(wv[r], K[r * LD + lane], gj);
        }
        P1 = wsum(P1);
        Y = wsum(Y);
        if (!(P1 <= P0)) continue;  // the purified point is no better: keep x's certificate
        lds_sync();
        gs[lane] = gj;
        if (lane < m) ra[lane] = rs.yat(b, act[lane]);
        lds_sync();
        // ---- 3. dual: least squares for λ_A (and ν) on the free coordinates' equations
        double hk = 0.0;
        if (lane < mr)
            for (int j = 0; j < d; ++j) hk = __builtin_fma(em[j] * M[lane * LD + j], gs[j], hk);
        if (lane < mr)
            for (int l = 0; l < mr; ++l) {
                double s2 = 0.0;
                for (int j = 0; j < d; ++j) s2 = __builtin_fma(em[j] * M[lane * LD + j], M[l * LD + j], s2);
                K[lane * LD + l] = s2;
            }
        for (int l = (lane < mr ? mr : 0); l < DP; ++l) K[lane * LD + l] = (l == lane) ? 1.0 : 0.0;
        lds_sync();
        const double trG = wsum(lane < mr ? K[lane * LD + lane] : 0.0);
        if (lane < mr) K[lane * LD + lane] += 1e-13 * (trG / (mr > 0 ? mr : 1)) + 1e-300;
        lds_sync();
        double c = 0.0;
        polish_cholesky_solve(K, sc, lane, lane < mr ? -hk : 0.0, c);
        const double la = lane < m ? fmin(fmax(c, -0.5), 0.5) : 0.0;
        Y += wsum(lane < m ? la * ra[lane] : 0.0);
        sc[lane] = la;
        lds_sync();
        double wj = gj;
        if (cj)
            for (int k = 0; k < m; ++k) wj = __builtin_fma(sc[k], M[k * LD + lane], wj);
        if (!cj) wj = 0.0;
        double nw;
        if constexpr (NORM == 0) {
            nw = sqrt(wsum(wj * wj));
        } else if constexpr (NORM == 2) {
            nw = wsum(fabs(wj));
        } else {
            double mx = fabs(wj);
            for (int s2 = 32; s2 > 0; s2 >>= 1) mx = fmax(mx, __shfl_xor(mx, s2, 64));
            nw = mx;
        }
        const double gn = fmax(P1 - (-Y - nw), 0.0);
        bestx = fmin(bestx, fmax(P0 - (-Y - nw), 0.0));
        if (gn < best) {
            best = gn;
            pbest = P1;
            xbest = xn;
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
        return;
    }
    if (!improved) return;
    if (cj) actions[o * d + lane] = xbest;
    lds_sync();
    xs[lane] = xbest;
    lds_sync();
    if (lane == 0) {
        obj[o] = pbest;
        gap[o] = best;
        if (step_loss && NP > 1) {
            // FTL's loss at step n with this action (replay_exact_ftl :318-323: _dot's order)
            double lo = 0.0;
            if (n < T) {
                double q = 0.0;
                for (int j = 0; j < d; ++j) q = q + rs.zat(b, n, j) * xs[j];
                lo = 0.5 * fabs(q - rs.yat(b, n));
            }
            step_loss[o] = lo;
        }
    }
}

template <int NORM>
hipError_t launch_polish_n(const WideSrc& rs, int64_t B, int64_t NP, double* actions, double* obj,
                           double* gap, double* step_loss, hipStream_t st) {
    const size_t lds = (size_t)(2 * 64 * 65 + 7 * 64) * sizeof(double) + 64 * sizeof(int);
    const int64_t total = B * NP, slice = (int64_t)1 << 24;
    for (int64_t p0 = 0; p0 < total; p0 += slice) {
        hipLaunchKernelGGL((ocx_exact_polish_kernel<NORM>), dim3((unsigned)std::min(slice, total - p0)),
                           dim3(64), lds, st, rs, B, NP, p0, actions, obj, gap, step_loss);
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

}  // namespace

hipError_t ocx_launch_exact_polish(const double* z, const double* y, int64_t B, int64_t T,
                                   int64_t d, int tiled, int P, int C, int S, int64_t G, int norm,
                                   int all_prefixes, double* actions, double* obj, double* gap,
                                   double* step_loss, hipStream_t st) {
    const int64_t NP = all_prefixes ? T + 1 : 1;
    if (B == 0 || NP == 0 || !gap || !obj || !actions) return hipSuccess;
    if (d < 1 || d > 64) return hipErrorInvalidValue;
    const WideSrc rs{z, y, T, G, (int)d, P, C, S, tiled};
    switch (norm) {
        case 0: return launch_polish_n<0>(rs, B, NP, actions, obj, gap, step_loss, st);
        case 1: return launch_polish_n<1>(rs, B, NP, actions, obj, gap, step_loss, st);
        case 2: return launch_polish_n<2>(rs, B, NP, actions, obj, gap, step_loss, st);
        default: return hipErrorInvalidValue;
    }
}
