/*
 * ocx_oracle.c — CPU restatement of the reference's FTRL/FTL/SMART hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the parity checker ("oracle") for the
 * MI355X engine in online_convex_optimization_amd/.  Only tests/, the smoke()
 * entry point and bench.py's cpu_baseline leg may load it.  The product path
 * never links, loads or falls back to it.
 *
 * Every function restates one function of the reference
 * (/root/reference/fast_algorithms.py, exact_ftl.py) in the SAME floating-point
 * operation order: sequential sums starting from 0.0, IEEE sqrt and division,
 * no FMA contraction (built with -ffp-contract=off, no -ffast-math).  With that
 * order it is bit-identical to numba's default (non-fastmath) compilation of
 * the reference, which is pinned by tests/golden/ (fixtures produced by running
 * the reference itself in the build container, see tests/golden/make_golden.py).
 *
 * Parity status: pinned (tests/test_oracle_golden.py checks every golden vector
 * bit-for-bit).
 */
#include <math.h>
#include <stddef.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#ifdef _OPENMP
#include <omp.h>
#endif

/* fast_algorithms.py:11-16 `_dot` */
static double oc_dot(const double *a, const double *b, int64_t n) {
    double total = 0.0;
    for (int64_t i = 0; i < n; ++i) total += a[i] * b[i];
    return total;
}

/* fast_algorithms.py:19-24 `_normalized_hinge` */
static double oc_normalized_hinge(double q, double y) {
    double diff = q - y;
    if (diff < 0.0) diff = -diff;
    return 0.5 * diff;
}

/* fast_algorithms.py:27-34 `_compute_gradient` (exact ties give 0) */
static double oc_compute_gradient(double q, double y) {
    double diff = q - y;
    if (diff > 0.0) return 0.5;
    if (diff < 0.0) return -0.5;
    return 0.0;
}

/* fast_algorithms.py:37-49 `_action_ftl` */
static void oc_action_ftl(const double *theta, int64_t d, double *out) {
    double norm_sq = 0.0;
    for (int64_t j = 0; j < d; ++j) norm_sq += theta[j] * theta[j];
    if (norm_sq == 0.0) {
        for (int64_t j = 0; j < d; ++j) out[j] = 0.0;
        return;
    }
    double scale = -(1.0 / sqrt(norm_sq));
    for (int64_t j = 0; j < d; ++j) out[j] = scale * theta[j];
}

/* fast_algorithms.py:52-66 `_action_ftrl` (t is 1-based) */
static void oc_action_ftrl(const double *theta, int64_t d, int64_t t, double eta0, double *out) {
    double scale = -(eta0 / sqrt((double)(t > 1 ? t : 1)));
    for (int64_t j = 0; j < d; ++j) out[j] = scale * theta[j];
    double norm_sq = 0.0;
    for (int64_t j = 0; j < d; ++j) norm_sq += out[j] * out[j];
    if (norm_sq <= 1.0) return;
    double norm = sqrt(norm_sq);
    double factor = 1.0 / norm;
    for (int64_t j = 0; j < d; ++j) out[j] *= factor;
}

/* fast_algorithms.py:69-76 `_total_comparator_loss` / :79-85 `_comparator_loss_prefix` */
static double oc_comparator_loss_prefix(const double *z, const double *y, int64_t d,
                                        const double *action, int64_t length) {
    double total = 0.0;
    for (int64_t i = 0; i < length; ++i)
        total += oc_normalized_hinge(oc_dot(z + i * d, action, d), y[i]);
    return total;
}

/*
 * fast_algorithms.py:88-115 `_simulate_alg_core` (alg_flag==0 → FTRL, else FTL).
 * Extra outputs serve exact_ftl.py:230-277 `_simulate_ftrl`: when `comparator`
 * is non-NULL the final FTL action is replaced by it (exact_ftl.py:266-269);
 * x_last (nullable) receives the last played action (exact_ftl.py:276).
 */
int oc_simulate_alg(const double *z, const double *y, int64_t T, int64_t d, int alg_flag,
                    double eta0, const double *comparator, double *regret, double *cum_loss_out,
                    double *comp_loss_out, double *x_last) {
    double *theta = (double *)calloc((size_t)(d > 0 ? d : 1), sizeof(double));
    double *x = (double *)calloc((size_t)(d > 0 ? d : 1), sizeof(double));
    if (!theta || !x) { free(theta); free(x); return -1; }
    double cum_loss = 0.0;
    for (int64_t t = 0; t < T; ++t) {
        if (alg_flag == 0) oc_action_ftrl(theta, d, t + 1, eta0, x);
        else oc_action_ftl(theta, d, x);
        const double *zt = z + t * d;
        double q = oc_dot(zt, x, d);
        double yt = y[t];
        cum_loss += oc_normalized_hinge(q, yt);
        double g = oc_compute_gradient(q, yt);
        for (int64_t j = 0; j < d; ++j) theta[j] += g * zt[j];
    }
    if (x_last) memcpy(x_last, x, (size_t)d * sizeof(double));
    const double *act = comparator;
    if (!act) { oc_action_ftl(theta, d, x); act = x; }
    double comp = oc_comparator_loss_prefix(z, y, d, act, T);
    if (regret) *regret = cum_loss - comp;
    if (cum_loss_out) *cum_loss_out = cum_loss;
    if (comp_loss_out) *comp_loss_out = comp;
    free(theta); free(x);
    return 0;
}

/* fast_algorithms.py:118-164 `_simulate_SMART_like_core` */
int oc_simulate_smart(const double *z, const double *y, int64_t T, int64_t d, double theta_thresh,
                      double eta0, double *regret, int64_t *switch_step) {
    size_t n = (size_t)(d > 0 ? d : 1);
    double *theta_ftl = (double *)calloc(n, sizeof(double));
    double *theta_ftrl = (double *)calloc(n, sizeof(double));
    double *x = (double *)calloc(n, sizeof(double));
    double *s = (double *)calloc(n, sizeof(double));
    if (!theta_ftl || !theta_ftrl || !x || !s) {
        free(theta_ftl); free(theta_ftrl); free(x); free(s); return -1;
    }
    int switched = 0;
    int64_t sw = -1;
    double ftl_loss = 0.0, total_loss = 0.0;
    for (int64_t t = 0; t < T; ++t) {
        const double *zt = z + t * d;
        double yt = y[t];
        oc_action_ftl(theta_ftl, d, x);
        double pred_ftl = oc_dot(zt, x, d);
        double grad_ftl = oc_compute_gradient(pred_ftl, yt);
        for (int64_t j = 0; j < d; ++j) theta_ftl[j] += grad_ftl * zt[j];
        double loss_ftl = oc_normalized_hinge(pred_ftl, yt);
        ftl_loss += loss_ftl;
        if (switched) {
            oc_action_ftrl(theta_ftrl, d, t + 1, eta0, x);
            double pred = oc_dot(zt, x, d);
            total_loss += oc_normalized_hinge(pred, yt);
            double grad = oc_compute_gradient(pred, yt);
            for (int64_t j = 0; j < d; ++j) theta_ftrl[j] += grad * zt[j];
        } else {
            total_loss += loss_ftl;
            oc_action_ftl(theta_ftl, d, s);
            double s_loss = oc_comparator_loss_prefix(z, y, d, s, t + 1);
            if (ftl_loss - s_loss >= theta_thresh) { switched = 1; sw = t; }
        }
    }
    oc_action_ftl(theta_ftl, d, s);
    double comp = oc_comparator_loss_prefix(z, y, d, s, T);
    if (regret) *regret = total_loss - comp;
    if (switch_step) *switch_step = sw;
    free(theta_ftl); free(theta_ftrl); free(x); free(s);
    return 0;
}

/* exact_ftl.py:280-333 (compute_prefix_actions + replay_exact_ftl, l2 ball) in closed
 * form.  When every ||z_t|| <= 1 and y_t = +-1 the objective 0.5*sum|z_i.x - y_i| equals
 * 0.5*(t - x.S_t) on the unit ball, so the prefix minimiser is S_t/||S_t|| (0 if S_t = 0),
 * S_t = sum_{i<t} y_i z_i: the FTL action (fast_algorithms.py:37-49) of theta = -S_t.
 * The reference obtains the same points from cvxpy (absent here; parity unpinned): this
 * restatement is checked against an independent scipy solver in tests/. */
int oc_ftl_exact(const double *z, const double *y, int64_t T, int64_t d, double *cum_out,
                 double *comp_out, double *cmp_action, int *regime) {
    double *theta = (double *)calloc((size_t)(d > 0 ? d : 1), sizeof(double));
    double *x = (double *)calloc((size_t)(d > 0 ? d : 1), sizeof(double));
    if (!theta || !x) { free(theta); free(x); return -1; }
    int linear = 1;
    double cum = 0.0;
    for (int64_t t = 0; t < T; ++t) {
        const double *zt = z + t * d;
        oc_action_ftl(theta, d, x);
        cum += oc_normalized_hinge(oc_dot(zt, x, d), y[t]);
        double zz = 0.0;
        for (int64_t j = 0; j < d; ++j) zz += zt[j] * zt[j];
        if (!(zz <= 1.0 + 1e-6 && fabs(y[t]) == 1.0)) linear = 0;
        for (int64_t j = 0; j < d; ++j) theta[j] += (-y[t]) * zt[j];
    }
    oc_action_ftl(theta, d, x);
    double comp = oc_comparator_loss_prefix(z, y, d, x, T);
    if (cum_out) *cum_out = cum;
    if (comp_out) *comp_out = comp;
    if (cmp_action) memcpy(cmp_action, x, (size_t)d * sizeof(double));
    if (regime) *regime = linear;
    free(theta); free(x);
    return 0;
}

/* exact_ftl.py:280-303 `compute_prefix_actions` for the l2 ball in the closed form of
 * oc_ftl_exact: actions [T+1][d], actions[t] = FTL(theta_t), theta_t = -S_t. */
int oc_ftl_prefix_actions(const double *z, const double *y, int64_t T, int64_t d,
                          double *actions, int *regime) {
    double *theta = (double *)calloc((size_t)(d > 0 ? d : 1), sizeof(double));
    if (!theta) return -1;
    int linear = 1;
    for (int64_t t = 0; t <= T; ++t) {
        oc_action_ftl(theta, d, actions + t * d);
        if (t == T) break;
        const double *zt = z + t * d;
        double zz = 0.0;
        for (int64_t j = 0; j < d; ++j) zz += zt[j] * zt[j];
        if (!(zz <= 1.0 + 1e-6 && fabs(y[t]) == 1.0)) linear = 0;
        for (int64_t j = 0; j < d; ++j) theta[j] += (-y[t]) * zt[j];
    }
    if (regime) *regime = linear;
    free(theta);
    return 0;
}

/* exact_ftl.py:306-333 `replay_exact_ftl` loop: actions is [T+1][d]. */
int oc_replay(const double *z, const double *y, int64_t T, int64_t d, const double *actions,
              double *cum_loss_out) {
    double cum = 0.0;
    for (int64_t t = 0; t < T; ++t)
        cum += oc_normalized_hinge(oc_dot(z + t * d, actions + t * d, d), y[t]);
    *cum_loss_out = cum;
    return 0;
}

/* Batched drivers over B independent sequences (z: [B][T][d], y: [B][T]).
 * nthreads <= 0 → all OpenMP threads.  Used for the bench's CPU baseline. */
int oc_simulate_alg_batch(const double *z, const double *y, int64_t B, int64_t T, int64_t d,
                          int alg_flag, double eta0, const double *comparator, double *regret,
                          double *cum_loss, double *comp_loss, double *x_last, int nthreads) {
    int err = 0;
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 1) reduction(| : err)
#endif
    for (int64_t b = 0; b < B; ++b) {
        err |= oc_simulate_alg(z + b * T * d, y + b * T, T, d, alg_flag, eta0,
                               comparator ? comparator + b * d : NULL, regret ? regret + b : NULL,
                               cum_loss ? cum_loss + b : NULL, comp_loss ? comp_loss + b : NULL,
                               x_last ? x_last + b * d : NULL);
    }
    (void)nthreads;
    return err;
}

int oc_simulate_smart_batch(const double *z, const double *y, int64_t B, int64_t T, int64_t d,
                            const double *thresh, double eta0, double *regret, int64_t *switch_step,
                            int nthreads) {
    int err = 0;
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 1) reduction(| : err)
#endif
    for (int64_t b = 0; b < B; ++b)
        err |= oc_simulate_smart(z + b * T * d, y + b * T, T, d, thresh[b], eta0, regret + b,
                                 switch_step ? switch_step + b : NULL);
    (void)nthreads;
    return err;
}

int oc_max_threads(void) {
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}
