// ocx_sim_kernels.h — host-side launchers for the gfx950 kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/ocx.h"

bool ocx_supported_C(int C);
// algo: 0 FTRL, 1 FTL, 2 exact FTL (l2 ball, linear regime; see ocx_sim.hip).
// onepass: rows are known to satisfy ||z_t|| <= 1 (g(T) sampler): the comparator loss of
// FTL(theta_T) in closed form where the kernel can certify it (ocx_alg_kernel)
hipError_t ocx_launch_alg(const ocx_layout* L, const double* zt, const double* yt, int algo,
                          double eta0, const double* cmp, double* reg, double* cum, double* comp,
                          double* xl, hipStream_t st, double* cmp_out = nullptr,
                          int* regime = nullptr, int onepass = 0, int norm = 0);
// FTRL / FTL for butterfly layouts (chain = 0, P >= 2, C <= 32) with the step's dependency
// chain cut short (ocx_alg_pipe.hip); no comparator input, x_last or comparator output
bool ocx_pipe_supported(const ocx_layout* L);
hipError_t ocx_launch_alg_pipe(const ocx_layout* L, const double* zt, const double* yt, int ftl,
                               double eta0, double* reg, double* cum, double* comp,
                               int* closed_out, int onepass, hipStream_t st);
// the lean form over wave-groups [g0, g0 + gn) (<= 128 VGPRs; FTRL, 8 x 8 and 16 x 4 layouts),
// the FTRL side of the overlapped pipeline (ocx_pipeline.hip)
bool ocx_pipe_lean_supported(const ocx_layout* L);
// gmax (nullable, device): g(T)'s bit pattern, max-folded in the kernel (ocx_max_fold's rule)
hipError_t ocx_launch_alg_pipe_lean(const ocx_layout* L, const double* zt, const double* yt,
                                    double eta0, double* reg, int onepass, int64_t g0,
                                    int64_t gn, unsigned long long* gmax, hipStream_t st);
// FTRL over steps [t0, t0 + tn) of every sequence (t0 a multiple of 64), the step's state
// carried in `state` (ocx_pipe_state_doubles(L) doubles) from the chunk before; the chunk that
// ends at T writes the regrets (closed-form comparator only: onepass; a sequence it cannot
// certify gets NaN and sets *bad).  Bit-identical to one whole-horizon launch.
int64_t ocx_pipe_state_doubles(const ocx_layout* L);
hipError_t ocx_launch_alg_pipe_chunk(const ocx_layout* L, const double* zt, const double* yt,
                                     double eta0, double* reg, int onepass, int64_t t0,
                                     int64_t tn, double* state, int* bad,
                                     unsigned long long* gmax, hipStream_t st);
// g(T) sampler over sequences [b_off, b_off + nseq) of a d = 64 layout, at most wps waves per
// SIMD (four-wave blocks; ocx_gen_wave.hip)
// (wps >= 4: the 96-VGPR form, which spills a little; below: the 128-VGPR form)
hipError_t ocx_launch_gen_gT_range(const ocx_layout* L, uint64_t base_seed, int64_t run0,
                                   int64_t b_off, int64_t nseq, int wps, double* zt, double* ytl,
                                   hipStream_t st);
// generation overlapped with FTRL (ocx_pipeline.hip): nbatch batches of L->B runs from run0,
// regret = the last batch's; gmax (nullable, device) max-folds g(T) over every batch
bool ocx_pipeline_supported(const ocx_layout* L);
bool ocx_pipeline_worth(const ocx_layout* L, int wps);
// the multi-stream paths may fork from st (not under graph capture on HIP runtimes < 7.2)
bool ocx_stream_fork_ok(hipStream_t st);
hipError_t ocx_launch_gen_gT_range_lr(const ocx_layout* L, uint64_t base_seed, int64_t run0,
                                      int64_t b_off, int64_t nseq, double* zt, double* ytl,
                                      hipStream_t st);
// generation alone in rounds over two streams (ocx_pipeline.hip)
hipError_t ocx_run_gen_rounds(const ocx_layout* L, uint64_t base_seed, int64_t run0, double* zt,
                              double* yt, hipStream_t st);
hipError_t ocx_run_gen_sim_pipelined(const ocx_layout* L, uint64_t base_seed, int64_t run0,
                                     int64_t nbatch, double* zt, double* yt, double eta0,
                                     double* regret, int onepass, unsigned long long* gmax,
                                     int wps, int64_t sub_seqs, hipStream_t st);
// generation of batch k+1 trailing the chunked FTRL pass over batch k in one z buffer
// (ocx_pipeline.hip: the capacity-limited batches); see there for the buffers
bool ocx_pipe_lean_launchable(const ocx_layout* L);  // ocx_launch_alg_pipe_lean's layouts
bool ocx_trailing_supported(const ocx_layout* L);
// the largest batch whose generator waves all fit beside the FTRL chunks' waves
int64_t ocx_trailing_max_batch(const ocx_layout* L);
int64_t ocx_trailing_batches_run();  // batches through ocx_run_gen_sim_trailing so far
hipError_t ocx_run_gen_sim_trailing(const ocx_layout* L, uint64_t base_seed, int64_t run0,
                                    int64_t nbatch, double* zt, double* yt0, double* yt1,
                                    uint64_t* gst, double* fst, int* bad, double eta0,
                                    double* regret, int64_t last_B, unsigned long long* gmax,
                                    int nchunks, hipStream_t st);
// rows [t_off, t_off + nrows) of L's full-horizon tile, streams fresh (st_in null) or resumed
// from st_in, saved to st_out (nullable, not st_in); labels: then the T labels (ocx_gen_wave.hip)
hipError_t ocx_launch_gen_gT_rows(const ocx_layout* L, uint64_t base_seed, int64_t run0,
                                  int64_t t_off, int64_t nrows, const uint64_t* st_in,
                                  uint64_t* st_out, int labels, double* zt, double* ytl,
                                  hipStream_t st);
// the general exact comparator for 10 < d <= 64 (ocx_exact_wide.hip): row-major z/y
// (tiled = 0) or a tiled layout's (P, C, S, G)
hipError_t ocx_launch_exact_wide(const double* z, const double* y, int64_t B, int64_t T,
                                 int64_t d, int tiled, int P, int C, int S, int64_t G, int norm,
                                 int all_prefixes, double* actions, double* obj, double* gap,
                                 double* step_loss, int32_t* info, hipStream_t st);
// the general solvers' certificate polish (ocx_exact_wide.hip): the actions purified onto
// their active face and a dual rebuilt from the KKT system there; where that certifies a
// smaller gap, actions, obj, gap and step_loss are replaced.  d <= 64
hipError_t ocx_launch_exact_polish(const double* z, const double* y, int64_t B, int64_t T,
                                   int64_t d, int tiled, int P, int C, int S, int64_t G, int norm,
                                   int all_prefixes, double* actions, double* obj, double* gap,
                                   double* step_loss, hipStream_t st);
// the general exact comparator for 64 < d <= 256 (ocx_exact_big.hip): the solve and its
// certificate polish, the system in a per-block HBM scratch matrix
hipError_t ocx_launch_exact_big(const double* z, const double* y, int64_t B, int64_t T, int64_t d,
                                int tiled, int P, int C, int S, int64_t G, int norm,
                                int all_prefixes, double* actions, double* obj, double* gap,
                                double* step_loss, int32_t* info, hipStream_t st);
hipError_t ocx_launch_smart(const ocx_layout* L, const double* zt, const double* yt,
                            const double* th, double eta0, double* reg, int64_t* sw,
                            hipStream_t st);
// SMART in O(T·d) (ocx_smart_closed.hip): closed_prefix decides the switch from the
// closed-form prefix loss outside a rounding guard band (re-scan inside it: the reference's
// decisions); closed_comp takes the final comparator loss in closed form where certified.
// stats (nullable, device [2]): += re-scanned steps, += sequences with the closed comparator
hipError_t ocx_launch_smart_closed(const ocx_layout* L, const double* zt, const double* yt,
                                   const double* th, double eta0, double* reg, int64_t* sw,
                                   int closed_prefix, int closed_comp, unsigned long long* stats,
                                   hipStream_t st);
// SMART with one wavefront per sequence (ocx_smart_wave.hip), d <= 64
hipError_t ocx_launch_smart_wave(const ocx_layout* L, const double* zt, const double* yt,
                                 const double* th, double eta0, double* reg, int64_t* sw,
                                 hipStream_t st);
hipError_t ocx_launch_replay(const ocx_layout* L, const double* zt, const double* yt,
                             const double* at, double* cum, double* comp, hipStream_t st);
// exact FTL prefix actions [B][T+1][d] (closed form, l2 ball; ocx_sim.hip)
hipError_t ocx_launch_prefix_actions(const ocx_layout* L, const double* zt, const double* yt,
                                     double* actions, int* regime, hipStream_t st, int norm = 0);
hipError_t ocx_launch_pack(const ocx_layout* L, const double* z, const double* y, double* zt,
                           double* ytl, hipStream_t st);
hipError_t ocx_launch_max(const double* r, int64_t B, double* out, hipStream_t st);
int64_t ocx_gen_resident_waves(int64_t d, int dev);  // streams the generator runs in one round
// FTRL over wave-groups [g0, g0 + gn) of the 8 x 2 tree layout (the small-d pipeline's FTRL side
// at d = 16), g(T) folded into gmax (nullable)
hipError_t ocx_launch_alg_range(const ocx_layout* L, const double* zt, const double* yt,
                                double eta0, double* reg, int onepass, int64_t g0, int64_t gn,
                                unsigned long long* gmax, hipStream_t st);
hipError_t ocx_launch_gen_gT(const ocx_layout* L, uint64_t base_seed, int64_t run0, double* zt,
                             double* ytl, hipStream_t st);
// the g(T) sampler's normals unclipped (the float32 twin clips them itself)
hipError_t ocx_launch_gen_gT_raw(const ocx_layout* L, uint64_t base_seed, int64_t run0, double* zt,
                                 double* ytl, hipStream_t st);
hipError_t ocx_launch_gen_family(const ocx_layout* L, int family, const uint64_t* run_seeds,
                                 const uint64_t* stream_ids, double p, int64_t block_len,
                                 double* zt, double* ytl, hipStream_t st);
hipError_t ocx_launch_gen_seek(uint64_t base_seed, int64_t T_seed, int64_t run0, int64_t B,
                               int64_t d, uint64_t* st_out, uint64_t* lab_out, hipStream_t st);
hipError_t ocx_launch_gen_gT_chunk(const ocx_layout* L, int64_t T_seed, const uint64_t* st_in,
                                   uint64_t* st_out, const uint64_t* lab_in, uint64_t* lab_out,
                                   double* zt, double* ytl, hipStream_t st);
// mode 0 pass A, 1 pass B, 2 closed-form comparator (ocx_stream.hip); unclean [B + 1]
hipError_t ocx_launch_alg_chunk(const ocx_layout* L, const double* zt, const double* yt,
                                int64_t t0, int alg_flag, double eta0, int mode, double* theta,
                                double* cum, double* comp, double* regret, hipStream_t st,
                                double* unclean = nullptr);
// FTRL and exact FTL in one pass (ocx_ftrl_exact.hip)
hipError_t ocx_launch_ftrl_exact(const ocx_layout* L, const double* zt, const double* yt,
                                 double eta0, double* cum_r, double* cum_e, double* comp_e,
                                 double* comp_f, double* cmp_out, int* regime, hipStream_t st,
                                 int onepass = 0, int norm = 0);
// float32 twin (algorithms.py, ocx_twin32.hip): P = 1 layouts, d <= 32
// algo 0 FTRL, 1 FTL, 2 SMART (thresh[B]); clip: rows are raw g(T) normals to round to
// float and clip in float32 (algorithms.py:157-160)
hipError_t ocx_launch_twin32(const ocx_layout* L, const double* zt, const double* yt, int algo,
                             double eta0, const double* thresh, int clip, float* result,
                             double* cum, float* comp, int64_t* sw, hipStream_t st);
hipError_t ocx_launch_pack32(const ocx_layout* L, const float* z, const float* y, double* zt,
                             double* ytl, hipStream_t st);
// exact_ftl.py:224-227 `_comparator_loss` in OpenBLAS / NumPy order (ocx_comp_blas.hip):
// z [B][T][d] and y [B][T] row-major, x [B][d]; absr scratch [B][T]
hipError_t ocx_launch_comp_blas(const double* z, const double* y, const double* x, int64_t B,
                                int64_t T, int64_t d, double* absr, double* comp, hipStream_t st);
// The general exact-FTL comparator (ocx_exact_ball.hip): z [B][T][d], y [B][T] row-major;
// problems (b, n) for n = T … T-NP+1 (NP = all_prefixes ? T+1 : 1); actions [B][NP][d],
// obj / gap [B][NP] and info [B][NP] (Newton steps, negative at the iteration cap).
// d in 1..10.
// step_loss [B][NP] (nullable): ½|z_n·x_n − y_n|, the loss FTL pays at step n with the
// prefix-n action (0 for n = T).  The tiled form reads z / y in L's layout.
hipError_t ocx_launch_exact_ball(const double* z, const double* y, int64_t B, int64_t T,
                                 int64_t d, int norm, int all_prefixes, double* actions,
                                 double* obj, double* gap, double* step_loss, int32_t* info,
                                 hipStream_t st);
hipError_t ocx_launch_exact_ball_tiled(const ocx_layout* L, const double* zt, const double* yt,
                                       int norm, int all_prefixes, double* actions, double* obj,
                                       double* gap, double* step_loss, int32_t* info,
                                       hipStream_t st);
