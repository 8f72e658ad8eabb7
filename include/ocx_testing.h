/*
 * ocx_testing.h — test-only entry points of libocx.so (not part of the drop-in boundary).
 *
 * They exercise paths that correct inputs never reach, so the test suite can check them
 * without a process-wide switch in the product entry points.
 */
#ifndef OCX_TESTING_H_
#define OCX_TESTING_H_

#include <stdint.h>

#include "ocx.h"

#ifdef __cplusplus
extern "C" {
#endif

/* ocx_gT_regrets, but on the streamed (T-chunked) path every run r0 + b of a streamed
 * batch with b % unclean_every == 0 is treated as if it had failed the closed-form
 * comparator's check, so it takes the regenerated second pass (bit-identical to the
 * two-pass kernel); on the trailing path (resident batches of generation behind a chunked
 * FTRL pass) every batch k with k % unclean_every == 0 runs again whole, as a batch with a
 * NaN-flagged sequence does.  unclean_every >= 1. */
int ocx_test_gT_regrets_unclean(uint64_t base_seed, int64_t T, int64_t run0, int64_t R,
                                int64_t d, double eta0, double* regrets, int lanes_per_seq,
                                int device, int64_t unclean_every);

/* The trailing pipeline's FTRL side on a resident batch: the pipelined FTRL kernel run in
 * launches of chunk_steps steps (a multiple of 64), its state carried through device memory
 * between them, closed-form comparator.  regret [B] (device): bit-identical to one launch
 * for every sequence the closed form certifies; NaN for the others, and *bad (device int,
 * zeroed by the caller) set to 1.  Synchronises `stream`.  Butterfly layouts the pipelined
 * kernel takes (P in {8, 16, 32}, C in {4, 8, 16, 32}). */
int ocx_test_alg_pipe_chunked(const ocx_layout* L, const double* z_tiled, const double* y_tiled,
                              double eta0, int64_t chunk_steps, double* regret, int* bad,
                              void* stream);

/* Batches that have entered the trailing pipeline (ocx_run_gen_sim_trailing) in this process
 * so far: lets a test assert that a call took that path rather than the sequential loop. */
int64_t ocx_test_trailing_batches(void);

#ifdef __cplusplus
}
#endif
#endif /* OCX_TESTING_H_ */
