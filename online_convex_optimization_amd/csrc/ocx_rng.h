// ocx_rng.h — NumPy-stream-compatible RNG for the g(T) adversary, host+device.
//
// Restates, for one lane = one independent stream, what the reference's `_rng`
// (fast_algorithms.py:254-257, algorithms.py:177-180) builds through NumPy 2.x:
//   Generator(PCG64(SeedSequence([base_seed, T, run])))
// and the draws the g(T) sampler makes from it (fast_algorithms.py:234-239):
//   standard_normal  → NumPy's 256-layer ziggurat (random_standard_normal),
//   choice([-1,1])   → integers(0, 2) → buffered Lemire uint32 = top bit of each
//                      32-bit half of a raw draw, low half first.
// The same source compiles with g++ (tests/test_rng_host.py checks it against NumPy
// on the CPU) and with hipcc for gfx950 (the generator kernel).
#pragma once
#include <stdint.h>

#include "zig_tables.h"

#if defined(__HIPCC__)
#define OCX_HD __host__ __device__ __forceinline__
#define OCX_HD_NOINLINE __host__ __device__ __noinline__
#else
#define OCX_HD static inline
#define OCX_HD_NOINLINE static __attribute__((noinline))
#include <math.h>
#endif

typedef unsigned __int128 ocx_u128;

// ---------------------------------------------------------------------------
// SeedSequence (numpy/random/bit_generator.pyx): pool_size 4, uint32 arithmetic.
// ---------------------------------------------------------------------------
#define OCX_SS_INIT_A 0x43b0d7e5u
#define OCX_SS_MULT_A 0x931e8875u
#define OCX_SS_INIT_B 0x8b51f9ddu
#define OCX_SS_MULT_B 0x58f38dedu
#define OCX_SS_MIX_L 0xca01f9ddu
#define OCX_SS_MIX_R 0x4973f715u
#define OCX_SS_MAX_WORDS 12

OCX_HD uint32_t ocx_ss_hashmix(uint32_t value, uint32_t* hash_const) {
    value ^= *hash_const;
    *hash_const *= OCX_SS_MULT_A;
    value *= *hash_const;
    value ^= value >> 16;
    return value;
}

OCX_HD uint32_t ocx_ss_mix(uint32_t x, uint32_t y) {
    uint32_t r = OCX_SS_MIX_L * x - OCX_SS_MIX_R * y;
    r ^= r >> 16;
    return r;
}

// entropy: the concatenated uint32 words of every entropy integer (each integer
// contributes ⌈bits/32⌉ words, little-endian, and 0 contributes one word 0).
// Writes the 4 uint64 words of generate_state(4, np.uint64).
OCX_HD void ocx_seedseq_state4(const uint32_t* entropy, int n, uint64_t out[4]) {
    uint32_t pool[4];
    uint32_t hc = OCX_SS_INIT_A;
    for (int i = 0; i < 4; ++i) pool[i] = ocx_ss_hashmix(i < n ? entropy[i] : 0u, &hc);
    for (int s = 0; s < 4; ++s)
        for (int d = 0; d < 4; ++d)
            if (s != d) pool[d] = ocx_ss_mix(pool[d], ocx_ss_hashmix(pool[s], &hc));
    for (int s = 4; s < n; ++s)
        for (int d = 0; d < 4; ++d) pool[d] = ocx_ss_mix(pool[d], ocx_ss_hashmix(entropy[s], &hc));
    uint32_t w[8];
    uint32_t hb = OCX_SS_INIT_B;
    for (int i = 0; i < 8; ++i) {
        uint32_t v = pool[i & 3];
        v ^= hb;
        hb *= OCX_SS_MULT_B;
        v *= hb;
        v ^= v >> 16;
        w[i] = v;
    }
    for (int i = 0; i < 4; ++i) out[i] = (uint64_t)w[2 * i] | ((uint64_t)w[2 * i + 1] << 32);
}

// Append the uint32 words of a non-negative integer (numpy _int_to_uint32_array).
OCX_HD int ocx_ss_push_int(uint32_t* words, int n, uint64_t v) {
    if (v == 0) {
        words[n++] = 0u;
        return n;
    }
    while (v != 0) {
        words[n++] = (uint32_t)v;
        v >>= 32;
    }
    return n;
}

// ---------------------------------------------------------------------------
// PCG64 (XSL-RR 128/64), as numpy/random/src/pcg64: step, then output.
// ---------------------------------------------------------------------------
struct ocx_pcg64 {
    ocx_u128 state;
    ocx_u128 inc;
    uint32_t buf32;   // buffered high half for next_uint32
    int has32;
};

#define OCX_PCG_MULT ((((ocx_u128)0x2360ED051FC65DA4ULL) << 64) | (ocx_u128)0x4385DF649FCCF645ULL)

OCX_HD void ocx_pcg_seed(ocx_pcg64* g, const uint64_t st4[4]) {
    ocx_u128 s = (((ocx_u128)st4[0]) << 64) | st4[1];
    ocx_u128 i = (((ocx_u128)st4[2]) << 64) | st4[3];
    g->state = 0;
    g->inc = (i << 1) | 1u;
    g->state = g->state * OCX_PCG_MULT + g->inc;
    g->state += s;
    g->state = g->state * OCX_PCG_MULT + g->inc;
    g->buf32 = 0;
    g->has32 = 0;
}

OCX_HD uint64_t ocx_pcg_next64(ocx_pcg64* g) {
    g->state = g->state * OCX_PCG_MULT + g->inc;
    uint64_t hi = (uint64_t)(g->state >> 64);
    uint64_t lo = (uint64_t)g->state;
    unsigned rot = (unsigned)(g->state >> 122);
    uint64_t x = hi ^ lo;
    return (x >> rot) | (x << ((0u - rot) & 63u));
}

OCX_HD uint32_t ocx_pcg_next32(ocx_pcg64* g) {
    if (g->has32) {
        g->has32 = 0;
        return g->buf32;
    }
    uint64_t v = ocx_pcg_next64(g);
    g->has32 = 1;
    g->buf32 = (uint32_t)(v >> 32);
    return (uint32_t)v;
}

OCX_HD double ocx_pcg_next_double(ocx_pcg64* g) {
    return (double)(ocx_pcg_next64(g) >> 11) * (1.0 / 9007199254740992.0);
}

// Seed one stream exactly as _rng(w0, w1, w2) = SeedSequence([w0, w1, w2]).
OCX_HD void ocx_rng_init3(ocx_pcg64* g, uint64_t w0, uint64_t w1, uint64_t w2) {
    uint32_t words[OCX_SS_MAX_WORDS];
    int n = 0;
    n = ocx_ss_push_int(words, n, w0);
    n = ocx_ss_push_int(words, n, w1);
    n = ocx_ss_push_int(words, n, w2);
    uint64_t st[4];
    ocx_seedseq_state4(words, n, st);
    ocx_pcg_seed(g, st);
}

// ---------------------------------------------------------------------------
// log1p exactly as the host libm computes it (glibc 2.35, dbl-64/s_log1p.c: the
// fdlibm algorithm with glibc's Estrin-form polynomial).  NumPy's ziggurat tail
// (npy_log1p → libm log1p) turns its result straight into a normal deviate, so the
// device must reproduce libm bit for bit, not merely to 1 ulp; tests/test_rng_host.py
// checks this restatement against math.log1p on millions of inputs.
// Algorithm and constants: fdlibm, Copyright (C) 1993 by Sun Microsystems, Inc.
// Permission to use, copy, modify, and distribute this software is freely granted,
// provided that this notice is preserved.
// ---------------------------------------------------------------------------
OCX_HD int32_t ocx_hiword(double x) {
    return (int32_t)(__builtin_bit_cast(uint64_t, x) >> 32);
}
OCX_HD double ocx_with_hiword(double x, int32_t h) {
    const uint64_t lo = __builtin_bit_cast(uint64_t, x) & 0xffffffffULL;
    return __builtin_bit_cast(double, ((uint64_t)(uint32_t)h << 32) | lo);
}

OCX_HD double ocx_log1p(double x) {
    const double ln2_hi = 6.93147180369123816490e-01, ln2_lo = 1.90821492927058770002e-10,
                 two54 = 1.80143985094819840000e+16;
    const double Lp1 = 6.666666666666735130e-01, Lp2 = 3.999999999940941908e-01,
                 Lp3 = 2.857142874366239149e-01, Lp4 = 2.222219843214978396e-01,
                 Lp5 = 1.818357216161805012e-01, Lp6 = 1.531383769920937332e-01,
                 Lp7 = 1.479819860511658591e-01;
    double hfsq, f = 0.0, c = 0.0, s, z, R, u;
    int32_t k, hu = 0;
    const int32_t hx = ocx_hiword(x);
    const int32_t ax = hx & 0x7fffffff;
    k = 1;
    if (hx < 0x3FDA827A) {                     /* x < 0.41422 */
        if (ax >= 0x3ff00000) {                /* x <= -1.0 */
            if (x == -1.0) return -two54 / 0.0;
            return (x - x) / (x - x);
        }
        if (ax < 0x3e200000) {                 /* |x| < 2**-29 */
            if (ax < 0x3c900000) return x;     /* |x| < 2**-54 */
            return x - x * x * 0.5;
        }
        if (hx > 0 || hx <= (int32_t)0xbfd2bec3) { /* -0.2929 < x < 0.41422 */
            k = 0;
            f = x;
            hu = 1;
        }
    }
    if (hx >= 0x7ff00000) return x + x;
    if (k != 0) {
        if (hx < 0x43400000) {
            u = 1.0 + x;
            hu = ocx_hiword(u);
            k = (hu >> 20) - 1023;
            c = (k > 0) ? 1.0 - (u - x) : x - (u - 1.0); /* correction term */
            c /= u;
        } else {
            u = x;
            hu = ocx_hiword(u);
            k = (hu >> 20) - 1023;
            c = 0.0;
        }
        hu &= 0x000fffff;
        if (hu < 0x6a09e) {
            u = ocx_with_hiword(u, hu | 0x3ff00000); /* normalize u */
        } else {
            k += 1;
            u = ocx_with_hiword(u, hu | 0x3fe00000); /* normalize u/2 */
            hu = (0x00100000 - hu) >> 2;
        }
        f = u - 1.0;
    }
    hfsq = 0.5 * f * f;
    if (hu == 0) { /* |f| < 2**-20 */
        if (f == 0.0) {
            if (k == 0) return 0.0;
            c += k * ln2_lo;
            return k * ln2_hi + c;
        }
        R = hfsq * (1.0 - 0.66666666666666666 * f);
        if (k == 0) return f - R;
        return k * ln2_hi - ((R - (k * ln2_lo + c)) - f);
    }
    s = f / (2.0 + f);
    z = s * s;
    const double R1 = z * Lp1, z2 = z * z;
    const double R2 = Lp2 + z * Lp3, z4 = z2 * z2;
    const double R3 = Lp4 + z * Lp5, z6 = z4 * z2;
    const double R4 = Lp6 + z * Lp7;
    R = R1 + z2 * R2 + z4 * R3 + z6 * R4;
    if (k == 0) return f - (hfsq - s * (hfsq + R));
    return k * ln2_hi - ((hfsq - (s * (hfsq + R) + (k * ln2_lo + c))) - f);
}

// ---------------------------------------------------------------------------
// Ziggurat standard normal (NumPy random_standard_normal).  The three tables are
// passed in so the device kernel can serve them from LDS.
// ---------------------------------------------------------------------------
#define OCX_ZIG_NOR_R 3.6541528853610087963519472518
#define OCX_ZIG_NOR_INV_R 0.27366123732975827203338247596

// Rejection part of the ziggurat (≈0.7 % of draws), continuing NumPy's for(;;) loop
// from a rejected draw.  Inlined: an out-of-line call would take the PCG state's
// address and pin it in scratch memory for the whole kernel.
template <class KiT, class WiT, class FiT>
OCX_HD double ocx_standard_normal_slow(ocx_pcg64* g, const KiT& ki, const WiT& wi,
                                                const FiT& fi, int idx, uint64_t rabs, double x) {
    for (;;) {
        if (idx == 0) {
            for (;;) {
                double xx = -OCX_ZIG_NOR_INV_R * ocx_log1p(-ocx_pcg_next_double(g));
                double yy = -ocx_log1p(-ocx_pcg_next_double(g));
                if (yy + yy > xx * xx)
                    return ((rabs >> 8) & 0x1) ? -(OCX_ZIG_NOR_R + xx) : OCX_ZIG_NOR_R + xx;
            }
        } else {
            if (((fi(idx - 1) - fi(idx)) * ocx_pcg_next_double(g) + fi(idx)) < exp(-0.5 * x * x))
                return x;
        }
        uint64_t r = ocx_pcg_next64(g);
        idx = (int)(r & 0xff);
        r >>= 8;
        int sign = (int)(r & 0x1);
        rabs = (r >> 1) & 0x000fffffffffffffULL;
        x = (double)rabs * wi(idx);
        if (sign & 0x1) x = -x;
        if (rabs < ki(idx)) return x;
    }
}

template <class KiT, class WiT, class FiT>
OCX_HD double ocx_standard_normal(ocx_pcg64* g, const KiT& ki, const WiT& wi, const FiT& fi) {
    uint64_t r = ocx_pcg_next64(g);
    int idx = (int)(r & 0xff);
    r >>= 8;
    int sign = (int)(r & 0x1);
    uint64_t rabs = (r >> 1) & 0x000fffffffffffffULL;
    double x = (double)rabs * wi(idx);
    if (sign & 0x1) x = -x;
    if (rabs < ki(idx)) return x; /* 99.3% of the time */
    return ocx_standard_normal_slow(g, ki, wi, fi, idx, rabs, x);
}

// NumPy pairwise_sum order for a row of n squares (numpy/_core/src/umath/loops_utils.h):
// n < 8 sequential; 8 <= n <= 128 eight strided accumulators combined
// ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)) then the n%8 tail sequentially; n > 128 split
// at n2 = n/2 - (n/2)%8 and recurse.  ocx_pw_* evaluate that order while values
// stream in one at a time: `ocx_pw_plan` lists the leaves (≤128-element blocks) in
// order and the post-order combine program.
#define OCX_PW_MAX_LEAVES 64
struct ocx_pw_plan {
    int nleaf;
    int leaf_len[OCX_PW_MAX_LEAVES];
    // program: sequence of ops; op >= 0 → push leaf #op; op == -1 → pop b, pop a, push a+b
    int nops;
    int ops[2 * OCX_PW_MAX_LEAVES];
};

OCX_HD void ocx_pw_build_rec(ocx_pw_plan* p, int n) {
    if (n <= 128) {
        p->ops[p->nops++] = p->nleaf;
        p->leaf_len[p->nleaf++] = n;
        return;
    }
    int n2 = n / 2;
    n2 -= n2 % 8;
    ocx_pw_build_rec(p, n2);
    ocx_pw_build_rec(p, n - n2);
    p->ops[p->nops++] = -1;
}

OCX_HD void ocx_pw_build(ocx_pw_plan* p, int n) {
    p->nleaf = 0;
    p->nops = 0;
    ocx_pw_build_rec(p, n);
}

// Sum of one leaf block of `n` (≤128) values in NumPy's order.
struct ocx_pw_leaf {
    double r[8];
    double res;
    int i, n, n8;
};

OCX_HD void ocx_pw_leaf_begin(ocx_pw_leaf* L, int n) {
    for (int k = 0; k < 8; ++k) L->r[k] = 0.0;
    L->res = 0.0;
    L->i = 0;
    L->n = n;
    L->n8 = n - (n % 8);
}

OCX_HD void ocx_pw_leaf_add(ocx_pw_leaf* L, double v) {  // host reference form
    if (L->n < 8) {
        L->res += v;
    } else if (L->i < L->n8) {
        L->r[L->i & 7] += v;  // r[k] = a[k] + a[k+8] + ... (0.0 + a[k] is exact)
        if (L->i + 1 == L->n8)
            L->res = ((L->r[0] + L->r[1]) + (L->r[2] + L->r[3])) +
                     ((L->r[4] + L->r[5]) + (L->r[6] + L->r[7]));
    } else {
        L->res += v;
    }
    L->i++;
}

// One row of the g(T) sampler: draws d normals in order (NumPy's C order), hands each
// to store(j, v) and returns their sum of squares in NumPy's pairwise order
// (np.linalg.norm(z, axis=1)**2).  Leaves are consumed 8 values at a time so the
// eight accumulators have static indices (registers, not scratch).
template <class NormalFn, class StoreFn>
OCX_HD double ocx_row_sumsq(int d, const ocx_pw_plan& plan, NormalFn&& normal, StoreFn&& store) {
    double stack[16];
    int sp = 0;
    int j = 0;
    for (int op = 0; op < plan.nops; ++op) {
        const int code = plan.ops[op];
        if (code < 0) {
            const double rr = stack[--sp];
            const double ll = stack[--sp];
            stack[sp++] = ll + rr;
            continue;
        }
        const int n = plan.leaf_len[code];
        double res = 0.0;
        if (n < 8) {
            for (int i = 0; i < n; ++i) {
                const double v = normal();
                store(j++, v);
                res += v * v;
            }
        } else {
            double r[8] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
            const int n8 = n - (n % 8);
            for (int i0 = 0; i0 < n8; i0 += 8) {
#if defined(__HIPCC__)
#pragma unroll
#endif
                for (int k = 0; k < 8; ++k) {
                    const double v = normal();
                    store(j++, v);
                    r[k] += v * v;
                }
            }
            res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
            for (int i = n8; i < n; ++i) {
                const double v = normal();
                store(j++, v);
                res += v * v;
            }
        }
        if (plan.nops == 1) return res;
        stack[sp++] = res;
    }
    return d > 0 ? stack[0] : 0.0;
}
