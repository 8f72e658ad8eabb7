/*
 * ocx_testing.h — test-only entry points of libocx.so (not part of the drop-in boundary).
 *
 * They exercise paths that correct inputs never reach, so the test suite can check them
 * without a process-wide switch in the product entry points.
 */
#ifndef OCX_TESTING_H_
#define OCX_TESTING_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ocx_gT_regrets, but on the streamed (T-chunked) path every run r0 + b of a streamed
 * batch with b % unclean_every == 0 is treated as if it had failed the closed-form
 * comparator's check, so it takes the regenerated second pass (bit-identical to the
 * two-pass kernel).  The resident path ignores it.  unclean_every >= 1. */
int ocx_test_gT_regrets_unclean(uint64_t base_seed, int64_t T, int64_t run0, int64_t R,
                                int64_t d, double eta0, double* regrets, int lanes_per_seq,
                                int device, int64_t unclean_every);

#ifdef __cplusplus
}
#endif
#endif /* OCX_TESTING_H_ */
