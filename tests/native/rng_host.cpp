// Host build of online_convex_optimization_amd/csrc/ocx_rng.h for CPU unit tests:
// the same source the generator kernel runs, checked against NumPy on the host.
#include <math.h>
#include <stdint.h>
#include <string.h>

#include "../../online_convex_optimization_amd/csrc/ocx_rng.h"

static double bits2d(uint64_t b) { double d; memcpy(&d, &b, 8); return d; }
struct Ki { uint64_t operator()(int i) const { return OCX_ZIG_KI[i]; } };
struct Wi { double operator()(int i) const { return bits2d(OCX_ZIG_WI_BITS[i]); } };
struct Fi { double operator()(int i) const { return bits2d(OCX_ZIG_FI_BITS[i]); } };

extern "C" {
void h_log1p(const double* x, int64_t n, double* out) { for (int64_t i = 0; i < n; ++i) out[i] = ocx_log1p(x[i]); }

void h_seedseq_state4(const uint32_t* words, int n, uint64_t* out) { ocx_seedseq_state4(words, n, out); }

void h_raw(uint64_t w0, uint64_t w1, uint64_t w2, int64_t n, uint64_t* out) {
    ocx_pcg64 g; ocx_rng_init3(&g, w0, w1, w2);
    for (int64_t i = 0; i < n; ++i) out[i] = ocx_pcg_next64(&g);
}

void h_normals(uint64_t w0, uint64_t w1, uint64_t w2, int64_t n, double* out) {
    ocx_pcg64 g; ocx_rng_init3(&g, w0, w1, w2);
    Ki ki; Wi wi; Fi fi;
    for (int64_t i = 0; i < n; ++i) out[i] = ocx_standard_normal(&g, ki, wi, fi);
}

// the g(T) sampler (fast_algorithms.py:231-239) for one sequence, row-major z[T][d], y[T]
void h_gT(uint64_t seed, int64_t T, int64_t run, int64_t d, double* z, double* y) {
    ocx_pcg64 g; ocx_rng_init3(&g, seed, (uint64_t)T, (uint64_t)run);
    Ki ki; Wi wi; Fi fi;
    ocx_pw_plan plan; ocx_pw_build(&plan, (int)d);
    for (int64_t t = 0; t < T; ++t) {
        double* row = z + t * d;
        double sumsq = ocx_row_sumsq((int)d, plan, [&]() { return ocx_standard_normal(&g, ki, wi, fi); },
                                     [&](int j, double v) { row[j] = v; });
        double nrm = sqrt(sumsq);
        double sc = 1.0 / (nrm > 1.0 ? nrm : 1.0);
        for (int64_t k = 0; k < d; ++k) row[k] *= sc;
    }
    for (int64_t t = 0; t < T; ++t) y[t] = (ocx_pcg_next32(&g) >> 31) ? 1.0 : -1.0;
}
}
