/*
 * ocx.h — C ABI of the MI355X online-convex-optimization engine (libocx.so).
 *
 * Drop-in boundary for the reference's per-timestep FTRL/FTL hot path
 * (revvu/online_convex_optimization, /root/reference).  The reference is pure
 * Python: its "operator API" is the module-level functions that the drivers
 * select by import (fast_driver.py:23-28 vs driver.py:22-27).  Every entry point
 * below names the reference function it replaces; the ctypes binding a maintainer
 * adds on the reference side is shown in INTEGRATION.md and implemented in
 * online_convex_optimization_amd/_lib.py.
 *
 * Conventions
 *   - extern "C", plain pointers and sizes, no torch types.
 *   - Every function returns 0 on success or a negative ocx_status; the message
 *     of the last failure on the calling thread is available via ocx_last_error().
 *   - "host" entry points take host (numpy) pointers, copy to device `device`, run
 *     the HIP kernels and copy results back (synchronous).
 *   - "dev" entry points take device pointers in the engine's tiled HBM layout
 *     (see ocx_layout) and a hipStream_t passed as void* (NULL = default stream);
 *     they are asynchronous and capture-safe (no allocation, no sync) — except
 *     ocx_dev_exact_ball_solve / _tiled at d > 64, which take their Newton systems' scratch
 *     stream-ordered (hipMallocAsync / hipFreeAsync on the caller's stream; no sync).
 *   - All arithmetic is IEEE binary64 (dtype "f64").
 *   - lanes_per_seq selects how a sequence's d coordinates map onto lanes:
 *       0      auto: the fewest lanes that fill the GPU; partial sums combined by a
 *              butterfly (~1e-16 relative to the reference's sequential sums);
 *       k >= 2 k lanes (power of two), butterfly sums;
 *       1      exact, auto lanes (<= 16 coordinates per lane, <= 32 from d = 512 on;
 *              <= 4 lanes unless d needs more): every sum in the reference's
 *              sequential order, so results are bit-identical;
 *       -k     exact with k lanes; for k > 1 the running sum is handed from lane to
 *              lane (layout.chain = 1);
 *       OCX_LANES_BEST (128)  the fastest certified mode, the default of the batched
 *              APIs: the exact layout's sums (value 1) wherever its lane chains are short
 *              (fewer than 8 lanes per sequence) and d < 64; butterfly sums otherwise —
 *              d >= 512 and few-wave batches such as the capacity-limited T = 1e5 g(T)
 *              batch, where a chain of 8+ lanes leaves the kernel latency-bound, and
 *              batches of >= 4096 sequences at 64 <= d <= 128, where the pipelined 8 x 8
 *              butterfly kernel beats the 4-lane chain and the generator writes whole
 *              128-B lines of its tile.  The g(T) and FTRL-vs-exact entry points also
 *              take the closed-form comparator losses in this mode wherever the kernel
 *              certifies them (ocx_dev_simulate_alg_ex), so their results are NOT
 *              bit-identical to the reference: the loops keep the sums above, the
 *              comparator loss differs from the reference's sequential sum by that sum's
 *              rounding (about 1e-13 relative on the regret at T = 1e4).  Use 1 (or -k)
 *              for bit-identical results: every drop-in module does.
 */
#ifndef OCX_H_
#define OCX_H_

#define OCX_LANES_BEST 128
/* ocx_version() == OCX_VERSION = 10000 * major + 100 * minor + patch (400 = 0.4.0).  0.2.0:
 * ocx_ftrl_vs_exact_batch has its round-1 signature again (the `norm` argument moved to
 * ocx_ftrl_vs_exact_batch_ex); callers built against 0.1.x check ocx_version() >= 200.
 * 0.3.0 adds the general exact-FTL solver (ocx_exact_ball_solve, ocx_dev_exact_ball_solve,
 * ocx_dev_exact_ball_solve_tiled); nothing existing changed.  0.4.0 adds
 * ocx_dev_gen_simulate (generation overlapped with FTRL); nothing existing changed.
 *
 * Checking the ABI: one intermediate 0.1.x tree exported ocx_ftrl_vs_exact_batch WITH a
 * `norm` argument under the same symbol and the same version number as the release without
 * it, so a version number alone cannot tell those two apart and a C linker will not either.
 * A C caller must therefore require EXACT equality, ocx_version() == the OCX_VERSION it was
 * compiled with (OCX_ABI_MATCHES() below), not ocx_version() >= some minimum, and must take
 * `norm` through ocx_ftrl_vs_exact_batch_ex only.  The Python binding (_lib.py) checks
 * equality the same way. */
#define OCX_VERSION 400

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum ocx_status {
    OCX_OK = 0,
    OCX_E_INVALID = -1,   /* bad argument / shape */
    OCX_E_HIP = -2,       /* HIP runtime error (no device, launch failure, OOM) */
    OCX_E_UNSUPPORTED = -3
} ocx_status;

/* Tiled HBM layout shared by the generators and the simulation kernels.
 * A wave-group is 64 lanes = S sequences x P lanes; lane L = s*P + c owns
 * coordinates [c*C, (c+1)*C) of sequence b = g*S + s.  Coordinate pair k of every
 * lane lives in "plane" k (k < C/2): per (g, t) one contiguous 1 KiB row
 * [lane 0..63][2].  A wave therefore streams C/2 independent contiguous regions
 * (one per plane) with fully coalesced 1 KiB dwordx4 loads, which keeps more HBM
 * streams open than one region per wave:
 *   z_tiled[((k*G + g)*T + t)*128 + L*2 + e] = z[b][t][c*C + 2k + e]
 *   y_tiled[(g*T + t)*S + s]                 = y[b][t]
 * Padding (coordinates j >= d, sequences b >= B) holds zeros. */
typedef struct ocx_layout {
    int64_t B, T, d;  /* logical sizes */
    int32_t P;        /* lanes per sequence (1..64, power of two) */
    int32_t C;        /* coordinates per lane (even) */
    int32_t S;        /* sequences per wave-group = 64 / P */
    int32_t chain;    /* 1: exact mode with P > 1 (running sum passed lane to lane) */
    int64_t Dp;       /* padded dimension P*C >= d */
    int64_t G;        /* wave-groups = ceil(B / S) */
    int64_t z_elems;  /* doubles in z_tiled = G*T*64*C */
    int64_t y_elems;  /* doubles in y_tiled = G*T*S */
} ocx_layout;

/* ---- library / device ---------------------------------------------------- */
int ocx_version(void);
/* 1 when the loaded library implements exactly the ABI this header describes. */
#define OCX_ABI_MATCHES() (ocx_version() == OCX_VERSION)
int ocx_last_error(char* buf, size_t len);
int ocx_device_count(int* count);
/* Free the HBM the library caches per device for its host entry points and g(T) sweeps
 * (grown on demand, kept between calls).  Safe between calls; the next call regrows it.
 * Use before allocating large device buffers of one's own (engine.DeviceBatch). */
int ocx_release_buffers(int device);
/* Fill *out for (B, T, d) and a lanes_per_seq request (see Conventions). */
int ocx_layout_init(int64_t B, int64_t T, int64_t d, int lanes_per_seq, ocx_layout* out);

/* ---- host entry points (numpy buffers in, results out) ------------------- */

/* fast_algorithms.py:171-177 simulate_alg (→ _simulate_alg_core :88-115), batched
 * over B independent sequences; also exact_ftl.py:230-277 _simulate_ftrl when
 * `comparator` ([B][d], nullable) replaces the final FTL action.
 *   z [B][T][d], y [B][T] (C-contiguous f64); alg_flag 0 = FTRL, else FTL.
 *   regret/cum_loss/comp_loss [B] (each nullable); x_last [B][d] nullable =
 *   the last action played (exact_ftl.py:276). */
int ocx_simulate_alg_batch(const double* z, const double* y, int64_t B, int64_t T, int64_t d,
                           int alg_flag, double eta0, const double* comparator, double* regret,
                           double* cum_loss, double* comp_loss, double* x_last,
                           int lanes_per_seq, int device);

/* fast_algorithms.py:184-195 simulate_SMART_like (→ :118-164), batched; thresh [B].
 * switch_step [B] nullable: the t at which the switch fired, or -1.  In the bit-exact modes
 * (lanes_per_seq 1 or -k) the reference's O(T²·d) prefix re-scan and streamed comparator;
 * otherwise the O(T·d) kernel of ocx_dev_simulate_smart_ex with both flags (the same
 * switch steps; the comparator loss within its rounding). */
int ocx_simulate_smart_batch(const double* z, const double* y, int64_t B, int64_t T, int64_t d,
                             const double* thresh, double eta0, double* regret,
                             int64_t* switch_step, int lanes_per_seq, int device);

/* exact_ftl.py:423-453 run_ftl_exact (compute_prefix_actions :280-303 + replay
 * :306-333) over the unit ball of `norm` (0 l2, 1 l1, 2 linf; ExactFTLNoClip :83-105),
 * batched, in the closed form that is exact when every row's dual norm is <= 1 and
 * y_t = ±1 (then |z_i·x| <= 1 on the ball and ½Σ|z_i·x − y_i| = ½(t − x·S_t),
 * S_t = Σ_{i<t} y_i z_i): the prefix minimiser maximises x·S_t over the ball:
 *   l2   S_t/||S_t|| (0 if S_t = 0)            regime ||z_t||_2^2 <= 1 + 1e-6
 *   l1   sign(S_j*) e_j*, j* = first argmax |S_j|  regime max_j |z_tj| <= 1 + 1e-12
 *   linf sign(S_t) componentwise (0 where S_tj = 0)  regime sum_j |z_tj| <= 1 + 1e-12
 * regime [B] (int32, 1 = the data were in that regime); outside it the returned numbers
 * are not the SOCP/LP solution and callers must reject them.  Where the maximiser is not
 * unique (S_t = 0, ties in |S_j|, zero coordinates under linf) the solver's choice is
 * arbitrary; the engine returns the point above.  cmp_action [B][d] nullable = actions[T]
 * (the exact comparator of the whole sequence).  The reference solves an SOCP / LP with
 * cvxpy, absent here: parity unpinned, validated against scipy's solvers. */
int ocx_ftl_exact_batch(const double* z, const double* y, int64_t B, int64_t T, int64_t d,
                        int norm, double* cum_loss, double* comp_loss, double* cmp_action,
                        int32_t* regime, int lanes_per_seq, int device);

/* exact_ftl.py:280-303 compute_prefix_actions (ExactFTLNoClip, `norm` as above), batched:
 * actions [B][T+1][d] row-major, actions[b][t] = the exact FTL solution of prefix length
 * t, in the closed form of ocx_ftl_exact_batch (S_t/||S_t||, 0 for S_t = 0), with the
 * same regime flags (int32 [B], required).  Replaying these actions (ocx_replay_batch)
 * gives ocx_ftl_exact_batch's cum_loss bit for bit.  Parity vs cvxpy: unpinned. */
int ocx_ftl_prefix_actions_batch(const double* z, const double* y, int64_t B, int64_t T,
                                 int64_t d, int norm, double* actions, int32_t* regime,
                                 int lanes_per_seq, int device);

/* exact_ftl_driver.py:157-186 per sequence, batched, in one read of the data: exact FTL
 * (as ocx_ftl_exact_batch over the `norm` ball) and FTRL (fast_algorithms.py:88-111 order,
 * eta0) against the exact comparator actions[T] (exact_ftl.py:399-420 run_ftrl with
 * comparator_action).  Outputs [B]: cum_ftrl, cum_exact, comp_exact (the loss of
 * actions[T], shared by both regrets: FTRL = cum_ftrl - comp_exact, exact FTL =
 * cum_exact - comp_exact), comp_ftl (nullable: the loss of FTL(theta_ftrl), the
 * comparator simulate_alg itself would use), cmp_action [B][d] (nullable) and regime
 * (int32, required; see ocx_ftl_exact_batch). */
int ocx_ftrl_vs_exact_batch(const double* z, const double* y, int64_t B, int64_t T, int64_t d,
                            double eta0, double* cum_ftrl, double* cum_exact, double* comp_exact,
                            double* comp_ftl, double* cmp_action, int32_t* regime,
                            int lanes_per_seq, int device);
/* ocx_ftrl_vs_exact_batch over the unit ball of `norm` (0 l2 — what the plain entry point
 * uses —, 1 l1, 2 linf), as ocx_ftl_exact_batch.  (Version 200 restored the plain entry
 * point's round-1 signature; `norm` lives here.) */
int ocx_ftrl_vs_exact_batch_ex(const double* z, const double* y, int64_t B, int64_t T, int64_t d,
                               double eta0, double* cum_ftrl, double* cum_exact,
                               double* comp_exact, double* comp_ftl, double* cmp_action,
                               int32_t* regime, int norm, int lanes_per_seq, int device);

/* The general exact-FTL comparator: ExactFTLNoClip's problem (exact_ftl.py:83-105,
 * solved with cvxpy at :119-128)
 *     min_x ½ Σ_{i<n} |z_i·x − y_i|   s.t.  ||x||_norm <= 1   (norm 0 l2, 1 l1, 2 linf)
 * for any rows and labels (no regime: where the closed forms above do not apply), on device
 * by a primal log-barrier path (damped Newton, μ from 1 to 1e-10), then a
 * polish: the active rows and face found at several thresholds, x purified onto them and the
 * dual rebuilt from the KKT system.  The path's own x is kept whenever that dual certifies it
 * (gap <= 1e-9·(1 + obj)); the purified x replaces it only where x alone does not certify and
 * the purified point tightens the certificate.  So where the minimiser is not unique the
 * path's limit, the analytic centre of the optimal face, is returned.  Problems: each sequence's prefixes n = 0..T (all_prefixes = 1, actions
 * [B][T+1][d] as compute_prefix_actions :280-303 returns; actions[b][0] = 0) or n = T only
 * (all_prefixes = 0, [B][1][d]: the comparator).  obj [B][NP] (nullable) = ½Σ|r| at x
 * (for n = T: the comparator loss, exact_ftl.py:224-227, in butterfly order); gap [B][NP]
 * (nullable) = obj minus a dual lower bound (a certificate: obj − optimum <= gap);
 * step_loss [B][NP] (nullable) = ½|z_n·x_n − y_n|, what FTL pays at step n with the prefix-n
 * action (replay_exact_ftl :318-323; 0 for n = T), so Σ_n step_loss is exact FTL's cumulative
 * loss; info [B][NP] (int32, nullable) = the solve's status and Newton steps:
 *   info >= 0, bit OCX_EXACT_INFO_BREAKDOWN clear: converged (steps; 0: the empty prefix);
 *   info < 0: the step cap (300 steps; 1000 for d > 64) ended the solve (-steps);
 *   bit OCX_EXACT_INFO_BREAKDOWN set: stopped where μ outran fp64 (a Newton decrement no
 *     centred step produces) at the last centre, after (info & 0xFFFFF) steps — accurate to
 *     that μ only.
 * Only a converged solve is an answer by itself; for the other two the certificate decides
 * (the engine accepts a solve iff info >= 0 and gap <= 1e-8·(1 + |obj|), and raises
 * otherwise, as exact_ftl.py:125-126 does on a solver failure).  1 <= d <=
 * OCX_EXACT_BALL_MAX_D (else OCX_E_UNSUPPORTED).  Parity vs cvxpy: unpinned (validated
 * against scipy's HiGHS LPs and by the certificate). */
#define OCX_EXACT_INFO_BREAKDOWN (1 << 20)
#define OCX_EXACT_BALL_MAX_D 256
int ocx_exact_ball_solve(const double* z, const double* y, int64_t B, int64_t T, int64_t d,
                         int norm, int all_prefixes, double* actions, double* obj, double* gap,
                         double* step_loss, int32_t* info, int device);

/* exact_ftl.py:306-333 replay_exact_ftl, batched: actions [B][T+1][d].
 * cum_loss = sum_{t<T} 0.5|z_t.a_t - y_t|; comp_loss = sum_t 0.5|z_t.a_T - y_t|. */
int ocx_replay_batch(const double* z, const double* y, const double* actions, int64_t B,
                     int64_t T, int64_t d, double* cum_loss, double* comp_loss, int device);

/* fast_algorithms.py:230-241 (the body of empirical_worst_case_thresholds for one T):
 * regenerates on device the R sequences _rng(base_seed, T, run0 + r), r < R, with
 * `d` coordinates (the reference hard-codes d = 5), runs FTRL(eta0) on each and
 * returns the R regrets (host array).  Only the regrets leave the GPU. */
int ocx_gT_regrets(uint64_t base_seed, int64_t T, int64_t run0, int64_t R, int64_t d,
                   double eta0, double* regrets, int lanes_per_seq, int device);
/* ocx_gT_regrets with the regrets written to device memory: regrets_dev [R] lives on
 * `device`.  Nothing crosses PCIe (the FTRL kernel writes each batch's regrets in place);
 * the call returns when they are complete, so any stream or collective (an RCCL all-gather
 * of every rank's shard, parallel.gT_sweep_distributed) may read them afterwards. */
int ocx_gT_regrets_dev(uint64_t base_seed, int64_t T, int64_t run0, int64_t R, int64_t d,
                       double eta0, double* regrets_dev, int lanes_per_seq, int device);
/* ocx_gT_regrets reduced on device: *gmax = max(0.0, max over the R regrets) as
 * fast_algorithms.py:228, :242-243 (bit-identical to the max of ocx_gT_regrets' output);
 * only 8 bytes leave the GPU.  What empirical_worst_case_thresholds needs per T. */
int ocx_gT_max(uint64_t base_seed, int64_t T, int64_t run0, int64_t R, int64_t d, double eta0,
               int lanes_per_seq, int device, double* gmax);
/* In the bit-exact modes (lanes_per_seq 1 or -k) the comparator pass is the reference's
 * sequential sum; in the others the closed form of ocx_dev_simulate_alg_ex applies where
 * the kernel certifies it (the sampler's rows satisfy it by construction). */

/* fast_algorithms.py:211-247 empirical_worst_case_thresholds with `d` coordinates, over
 * several GPUs of this process: for every T of T_grid [nT], the runs [0, runs) are split
 * into contiguous shards, one per device, each generated and simulated on its own GPU by a
 * host thread (ocx_gT_regrets).  gmax [nT] = max(0.0, max over runs) as :228,:242-243;
 * regrets [nT][runs] (nullable: then each shard's max is reduced on its GPU, ocx_gT_max)
 * in run order.  ngpus <= 0: every visible device. */
int ocx_gT_sweep(const int64_t* T_grid, int nT, int64_t runs, uint64_t base_seed, int64_t d,
                 double eta0, int ngpus, double* gmax, double* regrets);
/* ocx_gT_sweep over an explicit device list (a device may repeat: its shards then share
 * that device's stream) and a lanes_per_seq mode. */
int ocx_gT_sweep_devices(const int64_t* T_grid, int nT, int64_t runs, uint64_t base_seed,
                         int64_t d, double eta0, const int* devices, int ndev, int lanes_per_seq,
                         double* gmax, double* regrets);

/* exact_ftl.py:224-227 `_comparator_loss` (0.5 * sum |z @ x - y|) for B sequences in the
 * reference's own operation order: OpenBLAS dgemv_t's row sums and NumPy's pairwise sum
 * (DESIGN.md §4).  z [B][T][d], y [B][T] row-major, x [B][d] the comparator actions.
 * The exact_ftl drop-in uses it for every RunResult.comp_loss. */
int ocx_comparator_loss_blas_batch(const double* z, const double* y, const double* x, int64_t B,
                                   int64_t T, int64_t d, double* comp_loss, int device);

/* ---- float32 twin (algorithms.py, the module driver.py imports) ----------- */
/* algorithms.py:28-54 simulate_alg (algo 0 FTRL, 1 FTL) and :65-120 simulate_SMART_like
 * (algo 2, thresh[B] = theta_thresh per sequence), batched over B sequences of float32 rows
 * z[B][T][d], y[B][T], d <= 32, in NumPy 2's float32 arithmetic:
 * result[b] = the twin's np.float32 return value; cum_loss (double, the Python float
 * accumulator), comp_loss (float32) and switch_step (SMART: step of the switch, -1 if none)
 * are optional. */
int ocx_twin32_batch(const float* z, const float* y, int64_t B, int64_t T, int64_t d, int algo,
                     double eta0, const double* thresh, float* result, double* cum_loss,
                     float* comp_loss, int64_t* switch_step, int device);
/* ocx_twin32_batch on a device-resident batch in a one-lane layout (lanes_per_seq = -1);
 * thresh (SMART) is a device array [B]; result / comp_loss are float32. */
int ocx_dev_twin32(const ocx_layout* L, const double* z_tiled, const double* y_tiled, int algo,
                   double eta0, const double* thresh, float* result, double* cum_loss,
                   float* comp_loss, int64_t* switch_step, void* stream);
/* The float32 twin's g(T) inner loop (algorithms.py:150-169): the regrets of runs
 * run0 .. run0+R-1 of _rng(base_seed, T, run), rows rounded to float32 and clipped in
 * float32, FTRL with eta0; on device (generator + twin kernel), nothing but the regrets
 * crosses PCIe. */
int ocx_twin32_gT_regrets(uint64_t base_seed, int64_t T, int64_t run0, int64_t R, int64_t d,
                          double eta0, float* regrets, int device);

/* ---- device entry points (tiled layout, caller-owned device memory) ------ */

/* Re-tile device arrays z [B][T][d], y [B][T] into the layout. */
int ocx_dev_pack(const ocx_layout* L, const double* z, const double* y, double* z_tiled,
                 double* y_tiled, void* stream);

/* fast_algorithms.py:231-239 sampler on device: sequence b of the layout is
 * _rng(base_seed, T, run0 + b) → clipped N(0, I_d) rows and ±1 labels. */
int ocx_dev_gen_gT(const ocx_layout* L, uint64_t base_seed, int64_t run0, double* z_tiled,
                   double* y_tiled, void* stream);

/* sequence_generation.py families on device, sequence b of the layout:
 *   family 1  make_random_iid_stream (:54-69): _rng(run_seeds[b], T, stream_ids[b]),
 *             u from _rng(run_seeds[b], 0, 11); fp32 rows, y = sign(z.u) (0 → +1);
 *   family 2  make_noisy_iid_stream (:72-89): u from stream 21, labels flipped where
 *             gen.random(T) < p;
 *   family 3  flip_sequence (:24-28);  family 4  switching_two_leaders_sequence
 *             (:36-47) with block_len.  Families 3/4 ignore the seed arrays.
 * run_seeds / stream_ids are device uint64 [B].  The float32 rows are stored as the
 * float64 values simulate_alg's np.ascontiguousarray(z, float64) would see. */
int ocx_dev_gen_family(const ocx_layout* L, int family, const uint64_t* run_seeds,
                       const uint64_t* stream_ids, double p, int64_t block_len, double* z_tiled,
                       double* y_tiled, void* stream);

/* fast_algorithms.py:88-115 on device.  comparator [B][d] device, nullable.
 * Outputs are device arrays [B] (nullable) and x_last [B][d] (nullable). */
int ocx_dev_simulate_alg(const ocx_layout* L, const double* z_tiled, const double* y_tiled,
                         int alg_flag, double eta0, const double* comparator, double* regret,
                         double* cum_loss, double* comp_loss, double* x_last, void* stream);

/* ocx_dev_simulate_alg with options.  flags (bitwise or):
 *   OCX_ALG_CLIPPED_ROWS (or its synonym OCX_ALG_CLOSED_COMPARATOR)  closed-form comparator
 *     loss where the kernel certifies it.  With comparator == NULL, the loss of
 *     FTL(theta_T) over the sequence is T/2 - ||theta_T|| whenever every row is inside the
 *     unit ball (||z_t||^2 <= 1 + 1e-12, as the g(T) sampler's clipped rows are,
 *     fast_algorithms.py:234-237) and every step's sub-gradient was -y_t/2 (y_t = +-1, no
 *     exact tie), because |z_t.x* - y_t| = 1 - y_t z_t.x* on the unit ball and
 *     theta_T = -S_T/2.  The kernel checks BOTH conditions itself, row by row and step by
 *     step, for every sequence: the flag is a request, never a trusted assertion, and is
 *     safe on any data.  A wave whose sequences all pass skips the second pass over z: one
 *     HBM pass instead of two.  The comparator loss then equals the reference's sequential
 *     sum up to that sum's rounding (about 1e-12 relative on the regret at T = 1e4; the
 *     loop itself keeps the layout's summation order); a sequence failing the check gets
 *     the streamed second pass, bit-identical to flags 0.
 * closed_out [B] (int32, nullable): 1 where the closed form was taken. */
#define OCX_ALG_CLIPPED_ROWS 1
int ocx_dev_simulate_alg_ex(const ocx_layout* L, const double* z_tiled, const double* y_tiled,
                            int alg_flag, double eta0, const double* comparator, double* regret,
                            double* cum_loss, double* comp_loss, double* x_last, int flags,
                            int32_t* closed_out, void* stream);

/* ocx_ftl_exact_batch on device (`norm` 0 l2, 1 l1, 2 linf). */
int ocx_dev_ftl_exact(const ocx_layout* L, const double* z_tiled, const double* y_tiled, int norm,
                      double* cum_loss, double* comp_loss, double* cmp_action, int32_t* regime,
                      void* stream);

/* ocx_ftl_prefix_actions_batch on device: actions [B][T+1][d] row-major (device). */
int ocx_dev_ftl_prefix_actions(const ocx_layout* L, const double* z_tiled,
                               const double* y_tiled, int norm, double* actions,
                               int32_t* regime, void* stream);

/* ocx_ftrl_vs_exact_batch on device: both loops in one pass, both comparator losses in
 * a second (two HBM passes instead of four). */
int ocx_dev_ftrl_vs_exact(const ocx_layout* L, const double* z_tiled, const double* y_tiled,
                          double eta0, double* cum_ftrl, double* cum_exact, double* comp_exact,
                          double* comp_ftl, double* cmp_action, int32_t* regime, void* stream);

/* ocx_dev_ftrl_vs_exact with options: `norm` of the exact side (0 l2, 1 l1, 2 linf, as
 * ocx_ftl_exact_batch), and flags OCX_ALG_CLOSED_COMPARATOR (or OCX_ALG_CLIPPED_ROWS):
 * for l2 and every sequence whose rows the kernel finds inside the unit ball
 * (||z_t||^2 <= 1 + 1e-12, summed in the step anyway) with labels +-1, both comparator
 * losses take their closed form T/2 + x.theta_e/2 (every loss is linear on the ball and
 * theta_e = -S_T is in registers), so such waves read z once instead of twice; the rest
 * stream the second pass.  Equal to the sequential sums up to their rounding. */
#define OCX_ALG_CLOSED_COMPARATOR 2
/* OCX_ALG_TREE_SUMS (ocx_dev_ftrl_vs_exact_ex): butterfly sums even when the layout chains
 * (the tiling is the same): the fused kernel's four chained totals per step leave it
 * latency-bound where the plain FTRL kernel streams (32768 x 1e4 x 64, one pass: 43 ms
 * chained vs 28 ms butterfly); about 1e-16 relative instead of the sequential order.
 * ocx_ftrl_vs_exact_batch applies it for lanes_per_seq = OCX_LANES_BEST. */
#define OCX_ALG_TREE_SUMS 4
int ocx_dev_ftrl_vs_exact_ex(const ocx_layout* L, const double* z_tiled, const double* y_tiled,
                             double eta0, double* cum_ftrl, double* cum_exact, double* comp_exact,
                             double* comp_ftl, double* cmp_action, int32_t* regime, int norm,
                             int flags, void* stream);

/* fast_algorithms.py:118-164 on device; thresh [B] device. */
int ocx_dev_simulate_smart(const ocx_layout* L, const double* z_tiled, const double* y_tiled,
                           const double* thresh, double eta0, double* regret,
                           int64_t* switch_step, void* stream);

/* ocx_dev_simulate_smart with options.  flags (bitwise or):
 *   OCX_SMART_CLOSED_PREFIX  O(T·d): the pre-switch prefix loss (:157-160) in closed form,
 *     (t+1)/2 − ½ s_t·S_t with S_t = Σ_{i<=t} y_i z_i, valid while every row is in the unit
 *     ball (||z_i||² <= 1 + 1e-12) and every label is ±1 (the kernel checks both).  It only
 *     decides the switch where ftl_loss − s_loss is farther from the threshold than a bound
 *     on the rounding that separates it from the reference's sequential sum; inside that
 *     band, or outside the regime, the step re-scans its prefix as the reference does.  The
 *     switch steps, hence the regrets, are the reference's.
 *   OCX_ALG_CLOSED_COMPARATOR  the final comparator loss of FTL(theta_ftl) as T/2 −
 *     ||theta_ftl|| where certified (as ocx_dev_simulate_alg_ex): one HBM pass in all, the
 *     regret then within the comparator sum's rounding of the reference's.
 * stats (nullable, device uint64 [2]): += steps that re-scanned, += sequences that took the
 * closed comparator. */
#define OCX_SMART_CLOSED_PREFIX 8
int ocx_dev_simulate_smart_ex(const ocx_layout* L, const double* z_tiled, const double* y_tiled,
                              const double* thresh, double eta0, double* regret,
                              int64_t* switch_step, int flags, unsigned long long* stats,
                              void* stream);

/* exact_ftl.py:306-333 on device; a_tiled is the actions [B][T+1][d] tiled with a
 * layout of T+1 steps (z/y use L, actions use La with La->T == L->T + 1). */
int ocx_dev_replay(const ocx_layout* L, const ocx_layout* La, const double* z_tiled,
                   const double* y_tiled, const double* a_tiled, double* cum_loss,
                   double* comp_loss, void* stream);

/* ocx_exact_ball_solve on device: z [B][T][d], y [B][T] row-major (device), outputs as
 * there (device); runs on `stream`, does not synchronise. */
int ocx_dev_exact_ball_solve(const double* z, const double* y, int64_t B, int64_t T, int64_t d,
                             int norm, int all_prefixes, double* actions, double* obj, double* gap,
                             double* step_loss, int32_t* info, void* stream);
/* The same on a resident batch in the tiled layout L. */
int ocx_dev_exact_ball_solve_tiled(const ocx_layout* L, const double* z_tiled,
                                   const double* y_tiled, int norm, int all_prefixes,
                                   double* actions, double* obj, double* gap, double* step_loss,
                                   int32_t* info, void* stream);

/* Max over runs of regrets[B] (device) into *gmax (device), starting from 0.0
 * as fast_algorithms.py:228,242-243 does. */
int ocx_dev_max_regret(const double* regrets, int64_t B, double* gmax, void* stream);

/* fast_algorithms.py:230-247's inner loop over resident batches: for k < nbatch, the runs
 * run0 + k*B .. run0 + (k+1)*B - 1 are generated on device into z_tiled / y_tiled
 * (ocx_dev_gen_gT) and simulated by FTRL (alg_flag 0, eta0; the certified closed-form
 * comparator unless OCX_GENSIM_TWO_PASS, as ocx_gT_regrets does).  regret [B] (device,
 * required: every batch's regrets pass through it) holds the last batch's regrets; gmax (device double, nullable) receives
 * max(0, max over every batch's regrets), bit-identical to the host loop.  Queued on
 * `stream`; complete when the stream reaches this point.
 *   Pipelined (the default where supported: d = 64 with the 8 x 8 or 16 x 4 butterfly
 * layout, d = 16 / 32 with 8 lanes of 2 / 4 coordinates — the g(T) layouts — and a batch of
 * at least four generator rounds unless sub_seqs > 0 asks for it): the batch is cut into
 * sub-batches of sequences (sub_seqs, <= 0: generator rounds making about 64 000 normals per
 * stream, one to four) and sub-batch i+1 is generated while the FTRL kernel reads
 * sub-batch i, the sub-batches alternating over two library streams per side (forked from
 * and joined to `stream` by events), the generator at four 96-VGPR waves per SIMD and the
 * FTRL kernel in a 128-VGPR form so both stay resident (csrc/ocx_pipeline.hip); consecutive
 * batches overlap the same way.  On a stream under graph capture the sequential loop runs
 * instead.  Same kernels and arithmetic as the sequential path: the regrets are
 * bit-identical to it.
 *   OCX_GENSIM_SEQUENTIAL: generate, then simulate, batch by batch on `stream` (any layout).
 *   OCX_GENSIM_TWO_PASS: the reference's streamed comparator pass instead of the certified
 *     closed form (what the bit-exact layouts ask for; the regrets are then bit-identical to
 *     fast_algorithms.py in those layouts). */
#define OCX_GENSIM_SEQUENTIAL 1u
#define OCX_GENSIM_TWO_PASS 2u
int ocx_dev_gen_simulate(const ocx_layout* L, uint64_t base_seed, int64_t run0, int64_t nbatch,
                         double* z_tiled, double* y_tiled, double eta0, double* regret,
                         double* gmax, uint32_t flags, int64_t sub_seqs, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* OCX_H_ */
