// ocx_gen_wave.hip — the g(T) adversary (fast_algorithms.py:231-239) with one
// wavefront per NumPy stream.
//
// NumPy's ziggurat is sequential per stream, but 98.5 % of its draws are accepted on
// the fast path, so a wave speculates: lane k computes raw draw k of the stream by
// PCG64 jump-ahead (state_{n+k+1} = A^{k+1} state_n + inc·(A^k + … + 1)), runs the
// fast test, and the wave then parses the 64 draws in stream order.  A rejected draw
// k consumes draw k+1 as its wedge uniform (a lane-parallel test; exp() is only
// evaluated exactly when a float estimate is too close to call), a tail draw falls
// back to NumPy's sequential loop, and the accepted normals are appended to a
// per-wave LDS ring with mbcnt.  Whole rows leave the ring: their sum of squares in
// NumPy's pairwise order (8 strided accumulators, combined by the DPP butterfly
// of ocx_seq_sum<8>, which reproduces ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)) bit for
// bit), the clip scale 1/max(‖z_t‖, 1), and a store into the tiled layout.  The
// ±1 labels (choice → top bit of each buffered uint32) follow, 128 per round.
//
// Compared with one lane per stream (ocx_gen.hip's row staging, 33 KB of LDS per
// wave): no per-lane rows, so occupancy is set by registers, every lane works on
// every round, and a batch of a few thousand sequences already fills the GPU.
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <type_traits>
#include <utility>

#include "ocx_internal.h"
#include "ocx_rng.h"
#include "ocx_sim_kernels.h"

namespace {

constexpr uint64_t kMask52 = 0x000fffffffffffffULL;

// Float fast path of the ziggurat's wedge test (see zig_round; 0 = the double form).
// Measured no faster (d = 64, 32768 x 1e4: 71.5 vs 71.1 ms, profiles/r03_gen_ab.jsonl):
// off by default, kept as a tuning knob.
#ifndef OCX_GEN_WEDGE_F32
#define OCX_GEN_WEDGE_F32 0
#endif
// WU (zig_round): the wedge test of a rejection round on every lane, its outcome read off
// ballots (no exec-mask branches, no per-lane bool carried into the parse).  Bit-identical;
// the d = 1024 rows take it (2 048 x 1e4: 77.2 / 77.5 -> 76.2 / 76.0 ms), the d = 64 rows
// measured slower with it (58.9 -> 60.5 ms; profiles/r03_gen_wu_ab.jsonl).

// The fast path's table lookup (ki[idx], wi[idx] for a random layer idx per lane) is one
// ds_read_b128 of an interleaved {ki, wi} entry: the two separate tables read as a
// ds_read2_b64, which banks on (a/4) mod 32 in 16-lane groups, so 16 random layers fall
// into 16 slots per access and pass twice; a b128 read banks on (a/4) mod 64 and passes
// once.  Bit-identical and time-neutral (32 768 x 1e4 x 64: 59.76 vs 59.76 ms; 2 048 x 1e4
// x 1024: 77.47 vs 77.52; profiles/r03_gen_kw_ab.jsonl): the LDS is not what bounds the
// generator.
// KD: ki stored as a double.  ki < 2^53 and rabs < 2^52 are both exact doubles, so rabs < ki
// is decided on the double the draw is converted to anyway and the integer rabs need not
// stay live beside it (the tail path re-derives it from r): one VALU less per round.  Kept
// for the d = 64 rows (32 768 x 1e4: 58.6 / 58.5 vs 58.9 / 58.9 ms); the d = 1024 kernel,
// already at 128 VGPRs, spills more with it (76.7 / 76.8 vs 75.0 / 75.2 ms;
// profiles/r03_gen_kid_ab.jsonl).
#ifndef OCX_GEN_KI_DOUBLE
#define OCX_GEN_KI_DOUBLE 1
#endif
// Copies of the {ki, wi} table in the d = 64 (KD) kernels.  A ds_read_b128 of a random layer
// lands on slot idx mod 16 of the 256-B bank row, so a 16-lane group of random layers has
// ~3 lanes on its busiest slot.  With K copies entry (idx, c) lives at idx·K + c and lane l
// reads copy c = l mod K: each b128 group holds every c twice (its lanes mod 8 are 0..7
// twice), so at K = 8 a group's busiest slot holds 2 lanes.  1 = a single table.
// Measured at K = 8 (round 4; profiles/r04_gen_kw_ab.jsonl, r04_pmc_gen_lds_*.txt): bit-
// identical, SQ_LDS_BANK_CONFLICT 7.87e9 -> 5.38e9 cycles per 32 768 x 1e4 x 64 launch
// (2.6 -> 1.8 per LDS instruction), and the time unchanged (57.84 vs 57.99 ms): the conflicts
// are not on the generator's critical path, which is VALU issue.  The 32 KB table costs the
// six-wave few-stream form its occupancy (4 900 x 1e5: 89.3 -> 118.1 ms).  Off.
#ifndef OCX_GEN_KW_COPIES
#define OCX_GEN_KW_COPIES 1
#endif
template <bool KD>
struct ZigTables {
    static constexpr int kCopies = KD ? OCX_GEN_KW_COPIES : 1;
    struct alignas(16) Entry {
        typename std::conditional<KD, double, uint64_t>::type ki;
        double wi;
    } kw[256 * kCopies];
    double fi[256];
};
template <bool KD>
__device__ __forceinline__ void zig_lookup(const ZigTables<KD>& tb, int idx,
                                           typename std::conditional<KD, double, uint64_t>::type& ki,
                                           double& wi) {
    if constexpr (KD) {
        typedef double f64x2 __attribute__((ext_vector_type(2)));
        constexpr int K = ZigTables<KD>::kCopies;
        const f64x2 v = *reinterpret_cast<const f64x2*>(
            &tb.kw[K == 1 ? idx : idx * K + (int)(threadIdx.x & (K - 1))]);
        ki = v.x;
        wi = v.y;
    } else {
        typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
        const u32x4 v = *reinterpret_cast<const u32x4*>(&tb.kw[idx]);
        ki = ((uint64_t)v.y << 32) | v.x;
        wi = __hiloint2double((int)v.w, (int)v.z);
    }
}

__device__ __forceinline__ uint32_t rl32(uint32_t v, int lane) {
    return (uint32_t)__builtin_amdgcn_readlane((int)v, lane);
}
__device__ __forceinline__ uint64_t rl64(uint64_t v, int lane) {
    return ((uint64_t)rl32((uint32_t)(v >> 32), lane) << 32) | rl32((uint32_t)v, lane);
}
__device__ __forceinline__ ocx_u128 rl128(ocx_u128 v, int lane) {
    return ((ocx_u128)rl64((uint64_t)(v >> 64), lane) << 64) | rl64((uint64_t)v, lane);
}
// lane k gets lane k+1's value (DPP wave_shl:1, a VALU move; lane 63 gets 0 (bound_ctrl,
// no copy of the old value first), which no caller reads: a rejected lane 63 is redrawn
// next round)
__device__ __forceinline__ uint64_t shfl_down1(uint64_t v) {
    int lo = (int)(uint32_t)v, hi = (int)(uint32_t)(v >> 32);
    lo = __builtin_amdgcn_mov_dpp(lo, 0x130, 0xF, 0xF, true);
    hi = __builtin_amdgcn_mov_dpp(hi, 0x130, 0xF, 0xF, true);
    return ((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo;
}
__device__ __forceinline__ double shfl_double(double v, int src) {
    const int addr = src << 2;
    const int lo = __builtin_amdgcn_ds_bpermute(addr, __double2loint(v));
    const int hi = __builtin_amdgcn_ds_bpermute(addr, __double2hiint(v));
    return __hiloint2double(hi, lo);
}
__device__ __forceinline__ uint64_t ballot(bool p) { return __ballot(p); }
__device__ __forceinline__ int mbcnt(uint64_t m) {
    return (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                         __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}
__device__ __forceinline__ uint64_t lowmask(int n) {
    return n >= 64 ? ~0ULL : ((1ULL << n) - 1ULL);
}
__device__ __forceinline__ uint64_t xsl_rr(ocx_u128 s) {
    // rotr64(hi ^ lo, hi >> 58) as two funnel shifts (v_alignbit_b32)
    const uint64_t hi = (uint64_t)(s >> 64), lo = (uint64_t)s;
    const uint32_t rot = (uint32_t)(hi >> 58);
    const uint64_t x = hi ^ lo;
    const uint32_t xl = (uint32_t)x, xh = (uint32_t)(x >> 32);
    const bool sw = rot & 32;
    const uint32_t a = sw ? xh : xl, b = sw ? xl : xh;
    const uint32_t rl = __builtin_amdgcn_alignbit(b, a, rot);
    const uint32_t rh = __builtin_amdgcn_alignbit(a, b, rot);
    return ((uint64_t)rh << 32) | rl;
}
// (double)v for v < 2^52, exactly: the bits of 2^52 + v, minus 2^52
__device__ __forceinline__ double u52_to_double(uint64_t v) {
    return __longlong_as_double((long long)(0x4330000000000000ULL | v)) - 4503599627370496.0;
}
__device__ __forceinline__ double u53(uint64_t r) {
    return (double)(r >> 11) * (1.0 / 9007199254740992.0);
}

// Rare paths, kept out of line so their constants do not occupy registers of the
// round loop: the exact wedge comparison (float estimate too close to call, ~1e-5 of
// wedge tests) and NumPy's tail loop (≈3e-4 of draws).
__device__ __noinline__ bool wedge_exact(double lhs, double a) { return lhs < exp(a); }

struct TailOut {
    double v;
    uint64_t lo, hi;
};

__device__ __noinline__ TailOut zig_tail(uint64_t st_lo, uint64_t st_hi, uint64_t inc_lo,
                                        uint64_t inc_hi, uint64_t rabs) {
    ocx_pcg64 g;
    g.state = ((ocx_u128)st_hi << 64) | st_lo;
    g.inc = ((ocx_u128)inc_hi << 64) | inc_lo;
    g.buf32 = 0;
    g.has32 = 0;
    double xx, yy;
    for (;;) {
        xx = -OCX_ZIG_NOR_INV_R * ocx_log1p(-ocx_pcg_next_double(&g));
        yy = -ocx_log1p(-ocx_pcg_next_double(&g));
        if (yy + yy > xx * xx) break;
    }
    TailOut o;
    o.v = ((rabs >> 8) & 0x1) ? -(OCX_ZIG_NOR_R + xx) : OCX_ZIG_NOR_R + xx;
    o.lo = (uint64_t)g.state;
    o.hi = (uint64_t)(g.state >> 64);
    return o;
}

// Lane states (OCX_GEN_LANE_STATE): the round loop carries each lane's state for its next
// draw instead of the uniform base.  After a round that consumed all 64 draws, state k + 64
// = A^64·(state k) + C64 in every lane at once — the same 128-bit multiply-add as the jump
// from the base, with a constant multiplier — so no readlanes of lane 63's state (nor the
// wait for them) sit between one round and the next; a round that stops short rebuilds the
// states from its last consumed draw (readlanes + the jump, as before).  The d = 64 rows
// only (FLAT rounds): 62.4 -> 61.1 ms at 32 768 x 1e4, while the d = 1024 rows measured
// 78.8 -> 80.5 ms (profiles/r03_gen_lanestate_ab.jsonl).
#ifndef OCX_GEN_LANE_STATE
#define OCX_GEN_LANE_STATE 1
#endif

// One stream, as a wave sees it: the uniform state and increment, and this lane's
// jump-ahead pair (state after draw k of a round = Ak * base + Dk).  spec: this lane's
// state of the NEXT round, formed ahead from lane 63's state (valid when `have_spec`, i.e.
// the round consumed all 64 draws, which 99 % of rounds do).
struct WaveStream {
    ocx_u128 base, inc;
    ocx_u128 Ak, Dk;
    ocx_u128 C64;  // inc·(A^63 + … + A + 1): the 64-draw jump's additive part (uniform)
    ocx_u128 spec;
    bool have_spec;
    ocx_u128 s;     // OCX_GEN_LANE_STATE: this lane's state for the next round's draw
    ocx_u128 C64v;  // C64 in every lane (a VGPR operand of the advance)
};

// Next round's base after a round that consumed all 64 draws: lane 63's state, which is
// also A^64·base + C64.  OCX_GEN_SCALAR_NEXT computes it that way from the uniform base — a
// 128-bit multiply on the scalar unit, beside the round's vector work and independent of it —
// instead of four readlanes that wait for lane 63's vector multiply.  Bit-identical, and
// measured slower (d = 64, 32768 x 1e4: 83.0 vs 70.5 ms, profiles/r03_gen_scalar_ab.jsonl:
// the kernel already runs out of SGPRs, and the jump's temporaries add spills through VGPR
// lanes): off by default, kept as a tuning knob.
#ifndef OCX_GEN_SCALAR_NEXT
#define OCX_GEN_SCALAR_NEXT 0
#endif
constexpr ocx_u128 pcg_pow(int n) {
    ocx_u128 a = 1;
    for (int i = 0; i < n; ++i) a = a * OCX_PCG_MULT;
    return a;
}
constexpr ocx_u128 pcg_gsum(int n) {  // A^(n-1) + … + A + 1
    ocx_u128 g = 0;
    for (int i = 0; i < n; ++i) g = g * OCX_PCG_MULT + 1;
    return g;
}
// Per-lane jump-ahead constants, lane k: A^(k+1) and A^k + ... + A + 1 (low / high 64 bits),
// computed at compile time: a wave used to form them in a 64-trip loop of two 128-bit
// multiplies per lane (≈2 000 VALU per wave), which at T = 100 rivals a stream's rows.
struct JumpTable {
    uint64_t w[64][4];
};
constexpr JumpTable make_jump_table() {
    JumpTable t{};
    ocx_u128 a = 1, g = 0;
    for (int k = 0; k < 64; ++k) {
        g = g * OCX_PCG_MULT + 1;
        a = a * OCX_PCG_MULT;
        t.w[k][0] = (uint64_t)a;
        t.w[k][1] = (uint64_t)(a >> 64);
        t.w[k][2] = (uint64_t)g;
        t.w[k][3] = (uint64_t)(g >> 64);
    }
    return t;
}
__constant__ JumpTable kJumpTable = make_jump_table();
constexpr ocx_u128 kA64 = pcg_pow(64);
constexpr ocx_u128 kG64 = pcg_gsum(64);
constexpr ocx_u128 inv_u128(ocx_u128 a) {  // a^-1 mod 2^128 (a odd): Newton, 3 -> 384 bits
    ocx_u128 x = a;
    for (int i = 0; i < 7; ++i) x = x * (2 - a * x);
    return x;
}
constexpr ocx_u128 kAinv = inv_u128(OCX_PCG_MULT);
static_assert(kAinv * OCX_PCG_MULT == 1, "PCG multiplier inverse");

// ---- (a * b + d) mod 2^128 with a, d per lane and b wave-uniform (SGPRs) --------------
// Ten 32x32 partial products: six v_mad_u64_u32 (the 64-bit columns, each keeping its
// carry-out in an SGPR pair instead of re-deriving it), four v_mul_lo_u32 for the top
// column, and the carries folded in with v_addc: 18 VALU instructions where the
// compiler's __int128 lowering spends 25 (it zero-extends every 32-bit carry into a
// VGPR pair with v_mov).  Operand order keeps one scalar source per VOP3.
__device__ __forceinline__ uint64_t mad64c(uint32_t a, uint32_t b, uint64_t c, uint64_t& cy) {
    uint64_t r;
    asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %4" : "=&v"(r), "=s"(cy) : "v"(a), "s"(b), "v"(c));
    return r;
}
__device__ __forceinline__ uint64_t mad64z(uint32_t a, uint32_t b) {
    uint64_t r, cy;
    asm volatile("v_mad_u64_u32 %0, %1, %2, %3, 0" : "=&v"(r), "=s"(cy) : "v"(a), "s"(b));
    return r;
}
__device__ __forceinline__ uint32_t add32c(uint32_t a, uint32_t b, uint64_t& cy) {
    uint32_t r;
    asm volatile("v_add_co_u32_e64 %0, %1, %2, %3" : "=v"(r), "=s"(cy) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ uint32_t addc32(uint32_t a, uint32_t b, uint64_t cin, uint64_t& cy) {
    uint32_t r;
    asm volatile("v_addc_co_u32_e64 %0, %1, %2, %3, %4" : "=v"(r), "=s"(cy) : "v"(a), "v"(b), "s"(cin));
    return r;
}
__device__ __forceinline__ uint32_t addc32z(uint32_t a, uint64_t cin) {
    uint32_t r;
    uint64_t cy;
    asm volatile("v_addc_co_u32_e64 %0, %1, %2, 0, %3" : "=v"(r), "=s"(cy) : "v"(a), "s"(cin));
    return r;
}
__device__ __forceinline__ ocx_u128 mul_add_u128(ocx_u128 a, ocx_u128 b, ocx_u128 d) {
#if defined(OCX_GEN_TUNE_CHEAP_MUL)  // tuning only: no multiply (wrong normals)
    return (a ^ b) + d;
#elif defined(OCX_GEN_INT128_MUL)  // reference form (tuning A/B)
    return a * b + d;
#else
    const uint32_t a0 = (uint32_t)a, a1 = (uint32_t)(a >> 32), a2 = (uint32_t)(a >> 64),
                   a3 = (uint32_t)(a >> 96);
    const uint32_t b0 = (uint32_t)b, b1 = (uint32_t)(b >> 32), b2 = (uint32_t)(b >> 64),
                   b3 = (uint32_t)(b >> 96);
    uint64_t ca, cb, cc, c1, c3, cx;
    const uint64_t T = mad64c(a0, b0, (uint64_t)d, ca);               // a0b0 + d_lo
    const uint64_t M = mad64c(a1, b0, mad64z(a0, b1), cb);            // a0b1 + a1b0 (cb: 2^96)
    const uint32_t l1 = add32c((uint32_t)(T >> 32), (uint32_t)M, cc);  // bits 32..63
    uint64_t H = mad64c(a0, b2, (uint64_t)(d >> 64), cx);             // bits 64..127, mod 2^64
    H = mad64c(a1, b1, H, cx);
    H = mad64c(a2, b0, H, cx);
    const uint32_t X = a0 * b3 + a1 * b2 + a2 * b1 + a3 * b0;          // bits 96..127
    uint32_t hl = addc32((uint32_t)H, (uint32_t)(M >> 32), cc, c1);
    hl = addc32(hl, 0u, ca, c3);
    uint32_t hh = addc32((uint32_t)(H >> 32), X, c1, cx);
    hh = addc32z(hh, c3);
    hh = addc32z(hh, cb);
    const uint64_t lo = ((uint64_t)l1 << 32) | (uint32_t)T;
    const uint64_t hi = ((uint64_t)hh << 32) | hl;
    return ((ocx_u128)hi << 64) | lo;
#endif
}

// a copy the compiler cannot prove uniform: it stays in VGPRs (no per-round SGPR → VGPR moves)
__device__ __forceinline__ ocx_u128 vcopy128(ocx_u128 v) {
    uint32_t q[4] = {(uint32_t)v, (uint32_t)(v >> 32), (uint32_t)(v >> 64), (uint32_t)(v >> 96)};
#pragma unroll
    for (int i = 0; i < 4; ++i) asm volatile("v_mov_b32 %0, %1" : "=v"(q[i]) : "v"(q[i]));
    return ((ocx_u128)q[3] << 96) | ((ocx_u128)q[2] << 64) | ((ocx_u128)q[1] << 32) | q[0];
}

template <bool LS>
__device__ __forceinline__ void ws_set(WaveStream& w, const ocx_pcg64& g, ocx_u128 Gk) {
    // every lane holds the same state; reading it from lane 0 makes it provably uniform,
    // so the round loop keeps the base in SGPRs (the multiply's scalar operand)
    w.base = rl128(g.state, 0);
    w.inc = g.inc;
    w.Dk = g.inc * Gk;
    w.C64 = rl128(g.inc, 0) * kG64;
    w.have_spec = false;
    if constexpr (LS) {
        w.C64v = vcopy128(w.C64);
        w.s = mul_add_u128(w.Ak, w.base, w.Dk);
    }
}

// The base of the stream (the state of the last draw consumed) from the lane states:
// lane 0's state is A·base + inc.  Only where something reads the base (the labels, saved
// states) — the round loop itself carries the lane states.
template <bool LS>
__device__ __forceinline__ void ws_sync_base(WaveStream& w) {
    if constexpr (LS) w.base = rl128(kAinv * (rl128(w.s, 0) - rl128(w.inc, 0)), 0);
}

// One round: speculate 64 draws, parse them in stream order, append at most `need`
// normals to the ring at `head` (when RING).  Returns the number appended and advances
// the stream past exactly the draws those normals consumed (NumPy random_standard_normal).
// FULL: need == 64 is known (every round of a d = 64 row stream but the last): a rejection
// round then appends at most 63 normals, so the need-capping tail below drops out.
// Speculative next-round state (OCX_GEN_SPEC_NEXT): the next round's multiply-add is
// issued right after this round's, from lane 63's state, so it could overlap this round's
// table lookup, test and parse; a round that stops short of draw 63 (a rejected lane 63, a
// tail draw, the last round) drops it.  Measured slower (74.9 vs 71.1 ms at d = 64,
// 32768 x 1e4, profiles/r03_gen_ab.jsonl: the kernel is VALU-bound, not latency-bound, and
// the extra state costs registers): off by default, kept as a tuning knob.
#ifndef OCX_GEN_SPEC_NEXT
#define OCX_GEN_SPEC_NEXT 0
#endif
#ifndef OCX_GEN_FAST_REJ
#define OCX_GEN_FAST_REJ 1
#endif
// the single-rejection shortcut below in the d = 64 rows' flat rounds too, with lane states.
// Re-measured in round 6 on the current form: bit-identical, 49.66 -> 50.83 ms at 32 768 x 1e4
// x 64, 90.07 -> 90.50 ms at 4 900 x 1e5 (profiles/r06_gen_fastrej_flat_ab.jsonl).  Off.
#ifndef OCX_GEN_FAST_REJ_FLAT
#define OCX_GEN_FAST_REJ_FLAT 0
#endif
// d = 64 row loop: an inner loop of full rounds while a whole batch is still to draw
#ifndef OCX_GEN_INNER
#define OCX_GEN_INNER 1
#endif
// The d = 64 inner do-while of full rounds, two rounds per trip: the lane states alternate
// between two register sets instead of being copied at the back edge (32 768 x 1e4 x 64:
// 59.9 -> 59.4 ms, 58.7 -> 58.1 on a second box; the d = 1024 rows, without lane states,
// measured slower: 77.5 -> 78.8 ms; profiles/r03_gen_swz_ab.jsonl, r03_gen_variants4_ab.jsonl)
#ifndef OCX_GEN_UNROLL
#define OCX_GEN_UNROLL 2
#endif
// d = 1024 rows with the d = 64 form's round (FLAT: unmasked ring, lane states): measured
// 80.4 vs 77.2 ms (profiles/r03_gen_variants4_ab.jsonl); off, a tuning knob
#ifndef OCX_GEN_1K_FLAT
#define OCX_GEN_1K_FLAT 0
#endif
// lane states: the next round's states formed before this round's table lookup, to overlap
// the lookup's latency: 60.6 vs 58.1 ms at 32 768 x 1e4 x 64 (r03_gen_variants4_ab.jsonl:
// four more live VGPRs, no latency to hide); off, a tuning knob
#ifndef OCX_GEN_LS_EARLY
#define OCX_GEN_LS_EARLY 0
#endif
// labels through LDS, one 32-B segment per step and block (see the kernel)
#ifndef OCX_GEN_STAGE_Y
#define OCX_GEN_STAGE_Y 1
#endif
// Swizzled ring of the d = 1024 rows (OCX_GEN_SWZ1K).  The row's epilogue reads the ring
// with strides that put a whole 32-lane half on one LDS bank pair: the 32 x 32 store map
// reads slot 32·(l/2) + (l%2) + 2i (16-way) and the pairwise sum slot 128·(l/8) + l%8 + 8q
// (4-way; ds_read_b64 banks repeat every 32 doubles).  Slot i lives at i ^ (bits 5..8 of i
// moved to bits 1..4): a permutation inside each aligned 32-double block, so the round's
// contiguous writes stay conflict-free and both epilogue reads hit 32 distinct bank pairs.
// Bit-identical; 2 048 x 1e4 x 1024: 79.2 -> 77.5 ms, SQ_LDS_BANK_CONFLICT 1.82e10 -> 7.55e9
// cycles (profiles/r03_gen_swz_ab.jsonl, r03_pmc_gen1k_lds.json).
#ifndef OCX_GEN_SWZ1K
#define OCX_GEN_SWZ1K 1
#endif
template <int SW>
__device__ __forceinline__ unsigned rix(unsigned i) {
    if constexpr (SW == 1) return i ^ ((i >> 4) & 30u);
    else return i;
}

// FLAT: the ring is never wrapped (the caller keeps head + 64 within it and moves what is
// left to the front itself): ring indices go unmasked.  SW: the ring's slot map (rix).
// DF (deferred wedges, the d = 64 rows' full rounds; OCX_GEN_DEFER): a round does not run
// the wedge test of its rejected draws.  Whatever the test decides, a rejected draw k < 63
// consumes draw k+1 as its uniform, so the draws a full round consumes — and the stream
// state — do not depend on it; only whether x_k is emitted does.  The round emits every
// candidate tentatively and appends {ring slot, layer, next draw} to the wave's pending list;
// resolve_wedges() runs the tests of the whole list at once (one wave instruction per
// operation for all of them, instead of one per rejected draw) and compacts the ring where a
// test rejects, before anything reads the ring's rows.  Bit-identical, and measured slower:
// 32 768 x 1e4 x 64 took 69.6 vs 58.9 ms (profiles/r03_gen_defer_ab.jsonl).  With NumPy's
// tables 46 % of wedge tests reject, so nearly every batch compacts its ring (~3.6 slots),
// and the compaction's read -> ballot -> write chain per 64-slot chunk is latency the four
// waves per SIMD do not hide; the ~22 VALU per rejection round it saves are less.  Off; a
// tuning knob.
#ifndef OCX_GEN_DEFER
#define OCX_GEN_DEFER 0
#endif
// A round's candidates are attempts, never adjacent draws (an attempt consumes the next draw)
// and never draw 63: at most 32 per round.  Resolving once 32 are pending keeps the list
// within one wavefront (<= 63 entries).
constexpr int kPendMax = 64;    // pending entries per wave
constexpr int kPendFlush = 32;  // resolve once this many are pending

template <bool RING, bool FULL = false, bool FLAT = false, int SW = 0, bool WU = false,
          bool DF = false, bool KD = false>
__device__ __attribute__((always_inline)) int zig_round(WaveStream& w, int need, const ZigTables<KD>& tb, double* ring, int rmask,
                         unsigned head, int lane, uint64_t* pend = nullptr, int* npend = nullptr) {
    static_assert(!DF || (FULL && FLAT), "deferred wedges: full rounds of the flat ring only");
    const unsigned fmask = FLAT ? ~0u : (unsigned)rmask;
    constexpr bool LS = FLAT && OCX_GEN_LANE_STATE;  // lane states (d = 64 rows)
#if OCX_GEN_SPEC_NEXT
    ocx_u128 s;
    if (w.have_spec) {  // wave-uniform
        s = w.spec;
    } else {
        s = mul_add_u128(w.Ak, w.base, w.Dk);
    }
    const ocx_u128 s63 = rl128(s, 63);
    w.spec = mul_add_u128(w.Ak, s63, w.Dk);
#else
    const ocx_u128 s = LS ? w.s : mul_add_u128(w.Ak, w.base, w.Dk);
#endif
#if OCX_GEN_LS_EARLY
    const ocx_u128 s64 = LS ? mul_add_u128(s, kA64, w.C64v) : s;  // next round's, if m == 64
#endif
    const uint64_t r = xsl_rr(s);
    const int idx = (int)(r & 0xff);
    const uint64_t r8 = r >> 8;
    const uint64_t rabs = (r8 >> 1) & kMask52;
    typename std::conditional<KD, double, uint64_t>::type kidx;
    double widx;
    zig_lookup(tb, idx, kidx, widx);
    const double xa = u52_to_double(rabs);  // (double)rabs, exactly
    double x = xa * widx;
    // sign bit 8 of the draw → the sign of x (x = -x, -0.0 included), one xor
    x = __hiloint2double(__double2hiint(x) ^ (int)(((uint32_t)r & 0x100u) << 23),
                         __double2loint(x));
#ifdef OCX_GEN_TUNE_NO_PARSE  // tuning only: every draw accepted (wrong normals)
    const bool fast = true;
#else
    bool fast;
    if constexpr (KD) fast = xa < kidx;
    else fast = rabs < kidx;
#endif
    const uint64_t rej = ballot(!fast);
    if (rej == 0 && (FULL || need == 64)) {  // every draw accepted (38 % of rounds)
        if (RING) ring[rix<SW>((head + (unsigned)lane) & fmask)] = x;
#if OCX_GEN_SPEC_NEXT
        w.base = s63;
        w.have_spec = true;
#elif OCX_GEN_SCALAR_NEXT
        w.base = w.base * kA64 + w.C64;
#else
#if OCX_GEN_LS_EARLY
        if constexpr (LS) w.s = s64;
#else
        if constexpr (LS) w.s = mul_add_u128(s, kA64, w.C64v);
#endif
        else w.base = rl128(s, 63);
#endif
        return 64;
    }
#if OCX_GEN_FAST_REJ
    if constexpr (FULL && (!FLAT || OCX_GEN_FAST_REJ_FLAT)) {
        // The common rejection round (≈3/4 of them): one rejected draw k < 63 that is not a
        // tail draw.  Its wedge test runs on every lane (no exec-mask branch; lanes other than
        // k compute values nobody reads), the outcome is read off two ballots, and the
        // emission is a lane shift: lanes below k keep their slot, draw k+1 is its uniform,
        // lanes above it move down by one (wedge accepted) or two.  The arithmetic of lane k
        // is the general path's below, so the normals are the same; a wedge too close to
        // call, and every other pattern, take the general path.  Bit-identical; measured
        // (profiles/r03_gen_rej_ab.jsonl) 91.7 → 88.8 ms on the d = 1024 rows (2048 x 1e4),
        // but 70.7 → 73.9 ms on the d = 64 form (FLAT), which keeps the general path.
        const uint64_t zidx = ballot(idx == 0);
        if ((rej & (rej - 1)) == 0 && (rej >> 63) == 0 && (rej & zidx) == 0) {
            const int k = __builtin_ctzll(rej);
            const uint64_t rn = shfl_down1(r);
            const int i1 = idx ? idx : 1;  // lane k has idx != 0; the others any valid row
            const double lhs = (tb.fi[i1 - 1] - tb.fi[i1]) * u53(rn) + tb.fi[i1];
            const double e = (double)__expf((float)(-0.5 * x * x));
            const uint64_t sure_acc = ballot(lhs < e * (1.0 - 1e-5));
            const uint64_t sure_rej = ballot(lhs > e * (1.0 + 1e-5));
            const uint64_t kb = 1ULL << k;
            if ((sure_acc | sure_rej) & kb) {
                const bool wa = (sure_acc & kb) != 0;
                const unsigned sh = wa ? 1u : 2u;
                const bool skip = lane == k + 1 || (!wa && lane == k);
                if (RING && !skip)
                    ring[rix<SW>((head + (unsigned)lane - (lane > k + 1 ? sh : 0u)) & fmask)] = x;
                // the round consumed all 64 draws (k < 63 takes draw k + 1 as its uniform)
                if constexpr (LS) w.s = mul_add_u128(s, kA64, w.C64v);
                else w.base = rl128(s, 63);
                return wa ? 63 : 62;
            }
        }
    }
#endif
    uint64_t cons = 0, wacc = 0;
    int limit = 64, tail_k = -1;
    uint64_t rn = 0;
    if (rej) {
        // wedge test of a rejected draw k uses draw k+1 (next_double) as its uniform
        rn = shfl_down1(r);
        uint64_t tailm;
        if constexpr (DF) {
            // every wedge candidate tentatively accepted (resolve_wedges decides)
            const uint64_t zidx = ballot(idx == 0);
            tailm = rej & zidx;
            wacc = rej & ~zidx;
        } else if constexpr (WU && !OCX_GEN_WEDGE_F32) {
            // the same double arithmetic on every lane; lanes that are not wedge candidates
            // compute values nobody reads, from a valid table row
            const uint64_t zidx = ballot(idx == 0);
            const uint64_t cm = rej & ~zidx;  // wedge candidates
            tailm = rej & zidx;               // tail draws (layer 0)
            const int i1 = idx ? idx : 1;
            const double lhs = (tb.fi[i1 - 1] - tb.fi[i1]) * u53(rn) + tb.fi[i1];
            const double a = -0.5 * x * x;
            const double e = (double)__expf((float)a);  // |rel err| < 1e-6 for a in [-7, 0]
            wacc = cm & ballot(lhs < e * (1.0 - 1e-5));
            const uint64_t unsure = cm & ~wacc & ~ballot(lhs > e * (1.0 + 1e-5));
            if (unsure) {  // ~1e-5 of wedge tests: NumPy's exact comparison
                bool ex = false;
                if ((unsure >> lane) & 1) ex = wedge_exact(lhs, a);
                wacc |= ballot(ex);
            }
        } else {
        bool wa = false;
#ifdef OCX_GEN_TUNE_NO_WEDGE  // tuning only: no wedge test (wrong normals)
        if (false) {
#else
        if (!fast && idx != 0) {
#endif
#if OCX_GEN_WEDGE_F32
        }
        {
            // Every lane evaluates a float estimate of both sides (no exec-mask branch; the
            // rejected lanes' results are kept): lhs = (fi[idx-1] − fi[idx])·u + fi[idx]
            // with u from the top 32 bits of the next draw, and exp(−x²/2) by v_exp_f32,
            // each within 3e-6 relative, decided with a 1e-5 margin; a lane too close to
            // call (~1e-5 of wedge tests) takes NumPy's double arithmetic below.
            const int i1 = idx ? idx : 1;
            const float f1 = (float)tb.fi[i1 - 1], f0 = (float)tb.fi[i1];
            const float u = (float)(uint32_t)(rn >> 32) * 2.3283064365386963e-10f;  // 2^-32
            const float lhs_f = fmaf(f1 - f0, u, f0);
            const float xf = (float)x;
            const float e = __expf(-0.5f * xf * xf);
            const bool cand = !fast && idx != 0;
            wa = cand && lhs_f < e * (1.0f - 1e-5f);
            const bool unsure = cand && !wa && !(lhs_f > e * (1.0f + 1e-5f));
            if (ballot(unsure) != 0 && unsure) {
                const double lhs = (tb.fi[idx - 1] - tb.fi[idx]) * u53(rn) + tb.fi[idx];
                wa = wedge_exact(lhs, -0.5 * x * x);
            }
        }
#else
            const double lhs = (tb.fi[idx - 1] - tb.fi[idx]) * u53(rn) + tb.fi[idx];
            const double a = -0.5 * x * x;
            const double e = (double)__expf((float)a);  // |rel err| < 1e-6 for a in [-7, 0]
            if (lhs < e * (1.0 - 1e-5)) wa = true;
            else if (lhs > e * (1.0 + 1e-5)) wa = false;
            else wa = wedge_exact(lhs, a);
        }
#endif
        wacc = ballot(wa);
        tailm = ballot(!fast && idx == 0);
        }
        // Usual case: no tail draw and no two rejected draws side by side, so every
        // rejected draw k takes draw k+1 as its uniform and a rejected draw 63 is redone
        // next round: the walk below reduces to two bit operations.
        uint64_t rem = rej;
        if (tailm == 0 && (rej & (rej << 1)) == 0) {
            cons = rej << 1;
            limit = (rej >> 63) ? 63 : 64;
            rem = 0;
        }
        while (rem) {
            const int k = __builtin_ctzll(rem);
            rem &= rem - 1;
            if ((cons >> k) & 1) continue;  // this draw is an earlier wedge's uniform
            if ((tailm >> k) & 1) {
                limit = k;
                tail_k = k;
                break;
            }
            if (k == 63) {  // its uniform is not in this round: redo it next round
                limit = 63;
                break;
            }
            cons |= 1ULL << (k + 1);
        }
    }
    uint64_t emit = (~rej | (rej & wacc)) & ~cons & lowmask(limit);
    int n = __builtin_popcountll(emit);
    int m = limit;  // draws consumed
    if (!FULL && n >= need) {
        int p;  // lane of the need-th normal
        if (n == need) {
            p = 63 - __builtin_clzll(emit);
        } else {  // only in the last round of a sequence or chunk
            uint64_t e = emit;
            for (int i = 1; i < need; ++i) e &= e - 1;
            p = __builtin_ctzll(e);
        }
        emit &= lowmask(p + 1);
        m = ((rej >> p) & 1) ? p + 2 : p + 1;
        n = need;
        tail_k = -1;
    }
    if (RING && ((emit >> lane) & 1)) ring[rix<SW>((head + mbcnt(emit)) & fmask)] = x;
    if constexpr (DF) {
        const uint64_t pc = emit & rej;  // tentatively emitted wedge candidates
        if (pc) {
            if ((pc >> lane) & 1) {
                uint64_t* e = pend + 2 * (*npend + mbcnt(pc));
                e[0] = (uint64_t)(head + (unsigned)mbcnt(emit)) | ((uint64_t)(uint32_t)idx << 32);
                e[1] = rn;
            }
            *npend += __builtin_popcountll(pc);
        }
    }
    if (tail_k >= 0) {
        // NumPy's tail loop, sequential from the state after the tail draw
        const ocx_u128 st = rl128(s, tail_k);
        const TailOut o = zig_tail((uint64_t)st, (uint64_t)(st >> 64), (uint64_t)w.inc,
                                   (uint64_t)(w.inc >> 64),
                                   KD ? (rl64(r, tail_k) >> 9) & kMask52 : rl64(rabs, tail_k));
        if (RING && lane == 0) ring[rix<SW>((head + n) & fmask)] = o.v;
        w.base = rl128(((ocx_u128)o.hi << 64) | o.lo, 0);  // uniform (see ws_set)
        if constexpr (LS) w.s = mul_add_u128(w.Ak, w.base, w.Dk);
#if OCX_GEN_SPEC_NEXT
        w.have_spec = false;
#endif
        return n + 1;
    }
#if OCX_GEN_SPEC_NEXT
    if (m == 64) {  // the next round starts from lane 63's state: the speculation holds
        w.base = s63;
        w.have_spec = true;
    } else {
        w.base = rl128(s, m - 1);
        w.have_spec = false;
    }
#elif OCX_GEN_SCALAR_NEXT
    w.base = m == 64 ? w.base * kA64 + w.C64 : rl128(s, m - 1);
#else
    w.base = rl128(s, m - 1);
#endif
    if constexpr (LS)
#if OCX_GEN_LS_EARLY
        w.s = m == 64 ? s64 : mul_add_u128(w.Ak, rl128(s, m - 1), w.Dk);
#else
        w.s = m == 64 ? mul_add_u128(s, kA64, w.C64v) : mul_add_u128(w.Ak, rl128(s, m - 1), w.Dk);
#endif
    return n;
}

// Double rounds of the d = 1024 rows (round 6, measured and removed; git history keeps the
// form): each lane drew draws k and 64 + k (A^64 times the first state plus C64) and the wave
// parsed all 128 with zig_round's bit trick over a 128-bit mask, falling back to a single
// round for a tail draw or two adjacent rejections.  Bit-identical; 1 024 / 2 048 / 3 072 x
// 5 000 streams (1 / 2 / 3 waves per SIMD, 168 VGPRs): 29.7 / 36.5 / 49.4 ms against 32.8 /
// 37.7 / 49.3 ms — the latency it hides is gone by three waves per SIMD, which is where every
// d = 1024 batch runs (profiles/r06_gen1k_double_ab.jsonl).

// The wedge tests of the pending list (see DF above), all at once: lane i tests entry i, in
// NumPy's double arithmetic (the 1e-5 float-estimate margin, the exact comparison where too
// close to call).  Each rejected entry's slot is removed from the flat ring (flags in `gone`,
// one byte per slot: every later normal moves down by the removed slots before it), and
// head / produced drop by the count.  Pending entries are in stream order, so are slots.
template <bool KD>
__device__ __forceinline__ void resolve_wedges(double* ring, const uint64_t* pend, unsigned char* gone,
                                               int& npend, unsigned& head, uint32_t& produced,
                                               const ZigTables<KD>& tb, int lane) {
    if (npend == 0) return;
    const bool act = lane < npend;
    uint64_t w0 = 1ULL << 32, rn = 0;  // inactive lanes: layer 1, slot 0 (read, never used)
    if (act) {
        w0 = pend[2 * lane];
        rn = pend[2 * lane + 1];
    }
    const unsigned pos = (unsigned)w0;
    const int idx = (int)(w0 >> 32);
    const double x = ring[pos];
    const double lhs = (tb.fi[idx - 1] - tb.fi[idx]) * u53(rn) + tb.fi[idx];
    const double a = -0.5 * x * x;
    const double e = (double)__expf((float)a);  // |rel err| < 1e-6 for a in [-7, 0]
    const uint64_t am = lowmask(npend);
    uint64_t accm = am & ballot(lhs < e * (1.0 - 1e-5));
    const uint64_t un = am & ~accm & ~ballot(lhs > e * (1.0 + 1e-5));
    if (un) {  // ~1e-5 of wedge tests
        bool ex = false;
        if ((un >> lane) & 1) ex = wedge_exact(lhs, a);
        accm |= ballot(ex);
    }
    npend = 0;
    const uint64_t rejm = am & ~accm;
    if (rejm == 0) return;
    const bool rj = (rejm >> lane) & 1;
    if (rj) gone[pos] = 1;
    const unsigned first = (unsigned)__builtin_amdgcn_readlane((int)pos, __builtin_ctzll(rejm));
    unsigned before = 0;  // removed slots below the current chunk
    for (unsigned c = first & ~63u; c < head; c += 64) {
        const unsigned j = c + (unsigned)lane;
        const bool in = j < head;
        const double v = in ? ring[j] : 0.0;
        const uint64_t gm = ballot(in && gone[j] != 0);
        if (in && !((gm >> lane) & 1)) ring[j - before - (unsigned)mbcnt(gm)] = v;
        before += (unsigned)__builtin_popcountll(gm);
    }
    if (rj) gone[pos] = 0;
    head -= before;
    produced -= before;
}

// NumPy pairwise sum of v*v over one leaf of n <= 128 ring values starting at o.
// Lane k (mod 8) keeps accumulator r_k = v_k² + v_{k+8}² + ... in order; the loads of
// a lane are issued together (NF > 0: n known at compile time).
template <int NF>
__device__ __forceinline__ double leaf_sumsq(const double* ring, int rmask, unsigned o, int n_arg,
                                             int lane) {
    const int n = NF ? NF : n_arg;
    double res = 0.0;
    int i = 0;
    if (n >= 8) {
        const int n8 = n - (n % 8);
        const unsigned ok = o + (unsigned)(lane & 7);
        double acc;
        if constexpr (NF == 64) {
            // rows of 64 start at multiples of 64 in a ring of a multiple of 64: a row
            // never wraps, so one masked base and immediate offsets (ds_read2_b64 pairs)
            const double* rp = ring + (o & (unsigned)rmask) + (lane & 7);
            double v[8];
#pragma unroll
            for (int q = 0; q < 8; ++q) v[q] = rp[8 * q];
            acc = v[0] * v[0];
#pragma unroll
            for (int q = 1; q < 8; ++q) acc += v[q] * v[q];
        } else if constexpr (NF >= 8) {
            constexpr int M = (NF - NF % 8) / 8;
            double v[M];
#pragma unroll
            for (int q = 0; q < M; ++q) v[q] = ring[(ok + 8u * q) & rmask];
            acc = v[0] * v[0];
#pragma unroll
            for (int q = 1; q < M; ++q) acc += v[q] * v[q];
        } else {
            double v = ring[ok & rmask];
            acc = v * v;
            for (int j = 8; j < n8; j += 8) {
                v = ring[(ok + (unsigned)j) & rmask];
                acc += v * v;
            }
        }
        res = ocx_seq_sum<8>(acc);  // ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)) in every lane
        i = n8;
    }
    for (; i < n; ++i) {
        const double v = ring[(o + i) & rmask];
        res += v * v;
    }
    return res;
}

// The sums of squares of a batch of 512 ring normals = 512/DF rows of DF = 16 or 32 normals
// (the small-d rows, rows r at ring[r·DF, (r+1)·DF)): DF/8 lanes per row, every lane keeping
// 8/(DF/8) of NumPy's eight accumulators r_k = Σ_q v_{k+8q}² (8 loads per lane), summed in the
// lane as the left or right part of ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)) and combined across
// the row's lanes by the butterfly ocx_seq_sum<DF/8>: the pairwise order of a leaf of DF <= 128
// elements, bit for bit.  Lane l serves row l / (DF/8); every lane of the row gets the sum.
template <int DF>
__device__ __forceinline__ double batch_sumsq_small(const double* ring, int lane) {
    static_assert(DF == 16 || DF == 32, "small-d batch rows");
    constexpr int LPR = DF / 8;   // lanes per row
    constexpr int K = 8 / LPR;    // accumulators per lane
    constexpr int Q = DF / 8;     // terms per accumulator
    const int row = lane / LPR, c = lane % LPR;
    const double* rp = ring + row * DF + c * K;
    double r[K];
#pragma unroll
    for (int i = 0; i < K; ++i) {
        const double v0 = rp[i];
        r[i] = v0 * v0;
#pragma unroll
        for (int q = 1; q < Q; ++q) {
            const double v = rp[i + 8 * q];
            r[i] += v * v;
        }
    }
    double part;
    if constexpr (K == 4) part = (r[0] + r[1]) + (r[2] + r[3]);
    else part = r[0] + r[1];
    return ocx_seq_sum<LPR>(part);
}

// np.linalg.norm(z, axis=1)**2 for one row of d values (pairwise_sum recursion above
// 128 elements: split at n/2 rounded down to a multiple of 8, left + right).  The
// post-order walk of that recursion keeps its (uniform) stack in the wave's LDS slot
// `stk` so no register array is indexed dynamically.
struct PwFrame {
    unsigned o;
    int n, state;
    double val;
};

__device__ double row_sumsq(const double* ring, int rmask, unsigned o, int d, int lane,
                            PwFrame* stk) {
    if (d <= 128) return leaf_sumsq<0>(ring, rmask, o, d, lane);
    int sp = 0;
    if (lane == 0) stk[0] = PwFrame{o, d, 0, 0.0};
    double ret = 0.0;
    for (;;) {
        __builtin_amdgcn_wave_barrier();
        const PwFrame f = stk[sp];
        if (f.n <= 128) {
            ret = leaf_sumsq<0>(ring, rmask, f.o, f.n, lane);
        } else if (f.state < 2) {
            int n2 = f.n / 2;
            n2 -= n2 % 8;
            if (lane == 0) {
                stk[sp].state = f.state + 1;
                if (f.state == 1) stk[sp].val = ret;
                stk[sp + 1] = (f.state == 0) ? PwFrame{f.o, n2, 0, 0.0}
                                             : PwFrame{f.o + (unsigned)n2, f.n - n2, 0, 0.0};
            }
            ++sp;
            continue;
        } else {
            ret = f.val + ret;
        }
        if (sp == 0) return ret;
        --sp;
    }
}

__device__ __forceinline__ void save_state6(uint64_t* p, ocx_u128 state, ocx_u128 inc,
                                            uint32_t buf32, int has32) {
    p[0] = (uint64_t)state;
    p[1] = (uint64_t)(state >> 64);
    p[2] = (uint64_t)inc;
    p[3] = (uint64_t)(inc >> 64);
    p[4] = (uint64_t)buf32 | ((uint64_t)(uint32_t)has32 << 32);
    p[5] = 0;
}

__device__ __forceinline__ void load_state6(const uint64_t* p, ocx_u128& state, ocx_u128& inc,
                                            uint32_t& buf32, int& has32) {
    state = ((ocx_u128)p[1] << 64) | p[0];
    inc = ((ocx_u128)p[3] << 64) | p[2];
    buf32 = (uint32_t)p[4];
    has32 = (int)(p[4] >> 32);
}

// Waves per block of the default d = 64 form (OCX_GEN_NW64): a block's waves hold
// consecutive sequences, so the staged labels (see the kernel) leave as NW·8-B segments per
// step (up to a whole 128-B line of the y tile at S = 16).  32 768 x 1e4 at d = 64: 63.9 /
// 62.6 / 65.5 ms with 4 / 8 / 16 waves per block (profiles/r03_gen_nw_ab.jsonl; 16 makes
// every label round wait for the slowest of 16 waves).  The other forms keep 4 (their LDS
// then still admits their occupancy).
#ifndef OCX_GEN_NW64
#define OCX_GEN_NW64 8
#endif
// OV (the overlapped pipeline, ocx_pipeline.hip): four-wave blocks of the default d = 64
// form, so the launcher can cap the generator at three blocks (waves) per CU (SIMD) through
// its LDS request and leave each SIMD room for one FTRL wave beside it.
__host__ __device__ constexpr int gen_block(int DF, bool LR, int OV = 0) {
    return 64 * ((DF == 64 && !LR && !OV) ? OCX_GEN_NW64 : 4);
}
#ifdef OCX_GEN_TUNE_NO_STORE  // tuning only: rows computed, not written
#define OCX_GEN_STORE(v, p) do { if ((v) == 1234.5) *(p) = (v); } while (0)
#elif defined(OCX_GEN_PLAIN_STORE)  // tuning: write-back z stores
#define OCX_GEN_STORE(v, p) (*(p) = (v))
#else
#define OCX_GEN_STORE(v, p) __builtin_nontemporal_store((v), (p))
#endif
// Waves per SIMD the register allocation must allow.  The d = 64 kernels' rings (4.6 KB per
// wave) and tables (6 KB per block) admit six waves per SIMD in LDS; the default form keeps
// the four-wave register budget (no spills), the few-stream form (LR) asks for six.
#ifndef OCX_GENW_MIN_WAVES
#define OCX_GENW_MIN_WAVES_FOR(DF, LR) ((DF) == 64 ? ((LR) ? 6 : 4) : (((DF) == 1024 || (DF) == 16 || (DF) == 32) ? 4 : 1))
#else
#define OCX_GENW_MIN_WAVES_FOR(DF, LR) OCX_GENW_MIN_WAVES
#endif

// rows per batch leaving the ring (see the kernel)
#ifndef OCX_GEN_ROWS64
// rows per batch at 32 < d <= 64: 8 rows use all 64 lanes for the 8-accumulator sums of
// squares and share one sqrt/div sequence (d = 64, 32768 x 1e4: 84.8 ms vs 92.9 at 4 rows,
// profiles/r02_gen_variants.jsonl)
#define OCX_GEN_ROWS64 8
#endif
__host__ __device__ __forceinline__ int batch_rows(int d) {
    if (d < 8) return 32;
    if (d <= 128) return d <= 32 ? 8 : (d <= 64 ? OCX_GEN_ROWS64 : 2);
    return 1;
}
constexpr int kStackDoubles = 16 * sizeof(PwFrame) / 8;  // pairwise recursion depth <= 16
// rows per batch of the d = 64 kernels (both forms; 8 rows use all 64 lanes for the
// 8-accumulator sums of squares and share one sqrt/div sequence)
constexpr int kRows64 = 8;

}  // namespace

// MODE 0 (generate): rows [t_off, t_off + nrows) of the tiled layout (z_t clipped,
//   fast_algorithms.py:234-237; a whole launch: [0, T)) and then, if `labels`, the T labels
//   (:239).  Fresh streams _rng(base_seed, T_seed, run0+b), or, in chunk mode (st_in !=
//   nullptr), rows resume from st_in[b]; the stream after the rows is saved to st_out[b]
//   (nullable), and the labels resume from lab_in[b] (saved to lab_out[b]) when given.
// MODE 1 (seek): st_out[b] = the fresh stream, lab_out[b] = the stream after its
//   T_seed·d normals, i.e. where choice(T) starts.
// DF = 64: the d = 64, P·C = 64 rows of every configs[] workload, with the row shape
// known at compile time; DF = 1024: configs[4]'s d = 1024 rows (P·C = 1024, any P):
// the ring holds exactly one row (rounds stop at the row's end), the pairwise sum of
// squares uses all 64 lanes (8 leaves of 128, 8 accumulators each: the leaf and tree
// order of NumPy's recursion is the 64-lane butterfly) and every store instruction
// writes whole contiguous plane segments; DF = 0: any d.
// LR (DF = 64 only): the few-stream form: the same rows, compiled for six waves per SIMD
// (a register budget of 80 VGPRs, a few cold spills) where the default form keeps four.
// RAW (DF = 0 only): rows left unclipped, for the float32 twin (ocx_twin32.hip), which
// rounds them to float and clips them in float32 itself (algorithms.py:157-160).
// b_off: the launch covers sequences [b_off, b_off + nseq) of the layout (a sub-batch of the
// overlapped pipeline; 0 otherwise), a multiple of the block's waves.
// OV: 0, or the overlapped form's register budget in waves per SIMD (4: 128 VGPRs, beside an
// FTRL wave at three generator waves per SIMD; 5: 96 VGPRs, four generator waves beside one)
template <int MODE, int DF, bool LR = false, bool RAW = false, int OV = 0>
__global__ __launch_bounds__(gen_block(DF, LR, OV), OV ? OV : OCX_GENW_MIN_WAVES_FOR(DF, LR)) void ocx_gen_wave_kernel(
    uint64_t base_seed, int64_t T_seed, int64_t run0, int64_t B, int64_t nseq, int64_t T,
    int d_arg, int P, int C, int64_t G, double* __restrict__ zt, double* __restrict__ ytl,
    const uint64_t* __restrict__ st_in, uint64_t* __restrict__ st_out,
    const uint64_t* __restrict__ lab_in, uint64_t* __restrict__ lab_out, int rb,
    int64_t nwaves, int64_t b_off, int64_t t_off, int64_t nrows, int labels) {
    constexpr int kBlock = gen_block(DF, LR, OV);
    constexpr int kNW = kBlock / 64;
    // lane states in the round loop: the d = 64 row loop's FLAT rounds (see zig_round)
    constexpr bool kSmall = DF == 16 || DF == 32;  // the small-d rows (the d = 64 loop's form)
    constexpr bool kLS = OCX_GEN_LANE_STATE && MODE == 0 &&
                         (DF == 64 || kSmall || (DF == 1024 && OCX_GEN_1K_FLAT));
    constexpr bool kKD = OCX_GEN_KI_DOUBLE && (DF == 64 || kSmall);  // ki as doubles (see ZigTables)
    constexpr bool kDF = OCX_GEN_DEFER && MODE == 0 && DF == 64 && !LR && OCX_GEN_INNER;  // deferred wedges
    __shared__ ZigTables<kKD> tb;
    extern __shared__ double rings[];
    for (int i = threadIdx.x; i < 256 * ZigTables<kKD>::kCopies; i += blockDim.x) {
        const int e = i / ZigTables<kKD>::kCopies;
        tb.kw[i].ki = (decltype(tb.kw[i].ki))OCX_ZIG_KI[e];  // < 2^53: exact as a double
        tb.kw[i].wi = __longlong_as_double((long long)OCX_ZIG_WI_BITS[e]);
        if (i < 256) tb.fi[i] = __longlong_as_double((long long)OCX_ZIG_FI_BITS[i]);
    }
    __syncthreads();
    const int lane = threadIdx.x & 63;
    // wave-uniform by construction; readfirstlane makes it provably so, and with it the
    // stream index b: the per-stream SeedSequence hashing then runs on the scalar unit
    // beside other waves' VALU work instead of on 64 identical lanes
    const int64_t wave = __builtin_amdgcn_readfirstlane(
        (int)(blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6)));
    if (wave >= nwaves) return;
    const int slot = rb + (DF == 0 && d_arg > 128 ? kStackDoubles : 0);  // ring (+ pairwise stack)
    double* ring = rings + (threadIdx.x >> 6) * slot;
    PwFrame* stk = reinterpret_cast<PwFrame*>(ring + rb);
    const int rmask = rb - 1;
    if constexpr (kDF) {  // the removed-slot flags start clear (resolve_wedges clears its own)
        unsigned char* gone = reinterpret_cast<unsigned char*>(ring + kRows64 * 64 + 64 + 8 + 2 * kPendMax);
        for (int i = lane; i < kRows64 * 64 + 64; i += 64) gone[i] = 0;
    }

    // jump-ahead constants of this lane: A^(k+1) and A^k + ... + A + 1 (kJumpTable)
    WaveStream w;
    const ocx_u128 Gk = ((ocx_u128)kJumpTable.w[lane][3] << 64) | kJumpTable.w[lane][2];
    w.Ak = ((ocx_u128)kJumpTable.w[lane][1] << 64) | kJumpTable.w[lane][0];
    const int d = DF ? DF : d_arg;
    const int S = 64 / P;
    const int Dp = (DF == 64 || kSmall) ? DF : P * C;
    // DF = 1024 store map: flat index f = i*64 + lane of the row → plane k = f / (2P),
    // offset w = f % (2P) of the sequence's segment in that plane, coordinate
    // j = (w/2)*C + 2k + (w%2)
    const int lg2P = __builtin_ctz((unsigned)(2 * P));
    // P <= 32: store i of a row goes to plane k0 + i*kstep, offset w0, from ring slot
    // j0 + i*jstep (see the DF = 1024 epilogue)
    struct {
        int w0, k0, kstep, j0, jstep;
    } st1k;
    st1k.w0 = lane & (2 * P - 1);
    st1k.k0 = lane >> lg2P;
    st1k.kstep = 64 >> lg2P;
    st1k.j0 = (st1k.w0 >> 1) * C + 2 * st1k.k0 + (st1k.w0 & 1);
    st1k.jstep = 2 * st1k.kstep;
    // rows leave the ring in batches of R: the sums of squares of a batch run side by
    // side (8 lanes per row for 8 <= d <= 128, one lane per row for d < 8)
    const int R = batch_rows(d);
    // store map for Dp <= 64: lane → (row of the pass, coordinate j), RP rows per pass
    const int RP = Dp <= 64 ? 64 / Dp : 1;
    const int jl = Dp <= 64 ? lane % Dp : lane;
    const int rl = Dp <= 64 ? lane / Dp : 0;
    const int cl = jl / C, kl = (jl - cl * C) >> 1, el = (jl - cl * C) & 1;

    // Labels through LDS (stage_y): the kNW waves of a block hold kNW consecutive sequences,
    // so each step's labels of the block are min(kNW, S) contiguous, aligned doubles of the y
    // tile.  Each wave leaves a round's 128 labels at the front of its own ring and the block
    // stores them together, kNW lanes per step, instead of each wave's 8-B stores each costing
    // a whole write granule (WRITE_SIZE 1.052x the algorithmic bytes at d = 64, ~35 B per
    // 8-B label; profiles/r02_traffic_gen_final.json, r03_gen_ystage_*).  Every wave of a
    // block runs the same number of sequences and label rounds (fresh streams only: the chunk
    // mode's buffered half-draw makes rounds differ per sequence; nseq and nwaves multiples of
    // kNW, checked here and arranged by the launcher).
    const bool stage_y = OCX_GEN_STAGE_Y && MODE == 0 && lab_in == nullptr &&
                         nwaves % kNW == 0 && nseq % kNW == 0 && b_off % kNW == 0;
    // b0: the block's first sequence of this pass (the block's waves hold b0 .. b0 + kNW - 1)
    auto store_y_round = [&](int64_t tl, int64_t b0) {
        __syncthreads();  // every wave's round is in its ring
        const int tid = (int)threadIdx.x;
        const int64_t left = T - tl;
        const int Sq = 64 / P;
#pragma unroll
        for (int i = 0; i < 2; ++i) {  // 128 steps x kNW waves over kBlock threads
            const int q = i * kBlock + tid;
            const int tt = q / kNW, wv = q % kNW;
            const int64_t bw = b0 + wv;
            const int64_t gw = bw / Sq;
            if (tt < left)
                __builtin_nontemporal_store(rings[wv * slot + tt],
                                            ytl + (gw * T + tl + tt) * Sq + (bw - gw * Sq));
        }
        __syncthreads();  // the rings are free again
    };
    for (int64_t b = b_off + wave; b < b_off + nseq; b += nwaves) {
        const int64_t g = b / S;
        const int s = (int)(b - g * S);
        double* yrow = ytl + g * T * S + s;
        // tile offset of (t = 0, j = jl) for this sequence (Dp <= 64)
        const int64_t zoff = ((int64_t)kl * G + g) * T * 128 + (s * P + cl) * 2 + el;
        auto zaddr = [&](int64_t t, int j) -> double* {  // general j (Dp > 64)
            const int c = j / C, rr = j - c * C;
            return zt + (((int64_t)(rr >> 1) * G + g) * T + t) * 128 + (s * P + c) * 2 + (rr & 1);
        };
        if (MODE == 0 && (b >= B || d == 0)) {  // padding sequence / empty rows: zeros
            for (int64_t t = t_off; t < t_off + nrows; ++t)
                for (int j = lane; j < Dp; j += 64) *zaddr(t, j) = 0.0;
            if (b >= B && !labels) continue;
            if (b >= B) {
                if (stage_y) {
                    // the block's label rounds (and barriers) with zeros for this sequence
                    for (int64_t tl = 0; tl < T; tl += 128) {
                        ring[2 * lane] = 0.0;
                        ring[2 * lane + 1] = 0.0;
                        store_y_round(tl, b - (b % kNW));
                    }
                } else {
                    for (int64_t t = lane; t < T; t += 64) yrow[t * S] = 0.0;
                }
                continue;
            }
        }
        ocx_pcg64 g0;
        if (MODE == 0 && st_in != nullptr) {
            load_state6(st_in + 6 * b, g0.state, g0.inc, g0.buf32, g0.has32);
        } else {
            ocx_rng_init3(&g0, base_seed, (uint64_t)T_seed, (uint64_t)(run0 + b));
            if (MODE == 1 && lane == 0) save_state6(st_out + 6 * b, g0.state, g0.inc, 0, 0);
        }
        ws_set<kLS>(w, g0, Gk);

        // ---- rows
        if constexpr (MODE == 0 && (DF == 64 || DF == 32 || DF == 16)) {
            // DF = 16 / 32 (round 6): the same loop over batches of 512 normals = 512/DF rows
            // (32 / 16), their sums of squares by batch_sumsq_small (DF/8 lanes per row), the
            // stores 64/DF rows per pass.  The notes below are the d = 64 form's.
            // d = 64, a front-moving ring of R rows + one round (kRows64 * 64 + 64 doubles):
            // rows always start at ring[0], so no index is ever masked and every ring access
            // is a fixed base + an immediate offset.  A batch of R rows leaves as soon as the
            // ring holds it (at most one per round) and the <= 63 normals drawn past it then
            // move to the front (LDS operations of a wave run in order: the batch's reads come
            // first); the last batch may be shorter.  The batch's row scales reach the store
            // lanes through LDS (`scl`, one broadcast read per row) instead of readlanes.
            constexpr int RR = DF == 64 ? kRows64 : 512 / DF;  // rows per batch (512 normals)
            constexpr int kRP = 64 / DF;                      // rows per store pass
            const uint32_t total = (uint32_t)(nrows * DF);
            uint32_t produced = 0;
            unsigned head = 0;  // normals in the ring
            int64_t t = t_off;
            double* scl = ring + RR * DF + 64;  // the batch's row scales
            // deferred wedges (the default form): the pending list and the removed-slot flags
            // follow the scales in the wave's slot (ring_doubles)
            uint64_t* pend = reinterpret_cast<uint64_t*>(ring + RR * DF + 64 + 8);
            unsigned char* gone = reinterpret_cast<unsigned char*>(ring + RR * DF + 64 + 8 + 2 * kPendMax);
            int npend = 0;
            // (head > 0 once everything is drawn: at DF < 64 the <= 63 normals left over from a
            // batch can hold the last rows whole)
            while (produced < total || head > 0) {
#if OCX_GEN_INNER
                if (produced == total) {
                    // only the rows left in the ring to write
                } else if (total - produced >= (uint32_t)(RR * DF + 64)) {
                    // a whole batch still to draw: full rounds until the ring holds it, with
                    // one loop test per round (no per-round need / last-round / batch tests;
                    // every round here has 64 or more normals left to draw — with deferred
                    // wedges `produced` may count tentative normals, so the true remainder is
                    // larger still)
                    do {
                        const int n = zig_round<true, true, true, 0, false, kDF>(w, 64, tb, ring, 0, head,
                                                                                lane, pend, &npend);
                        produced += (uint32_t)n;
                        head += (unsigned)n;
#if OCX_GEN_UNROLL == 2
                        // two rounds per trip: the state alternates between two register sets
                        // (no back-edge copies of the 128-bit lane states)
                        if (head >= (unsigned)(RR * DF) || (kDF && npend >= kPendFlush)) break;
                        const int n2 = zig_round<true, true, true, 0, false, kDF>(w, 64, tb, ring, 0, head,
                                                                                 lane, pend, &npend);
                        produced += (uint32_t)n2;
                        head += (unsigned)n2;
#endif
                    } while (head < (unsigned)(RR * DF) && !(kDF && npend >= kPendFlush));
                    if constexpr (kDF) resolve_wedges(ring, pend, gone, npend, head, produced, tb, lane);
                } else
#endif
                if (produced < total) {
                    const uint32_t left = total - produced;
                    const int n =
                        left >= 64u ? zig_round<true, true, true>(w, 64, tb, ring, 0, head, lane)
                                    : zig_round<true, false, true>(w, (int)left, tb, ring, 0, head,
                                                                   lane);
                    produced += (uint32_t)n;
                    head += (unsigned)n;
                }
                if (head >= (unsigned)(RR * DF) || (produced == total && head > 0)) {
                    const int nrows = (int)(head / DF) < RR ? (int)(head / DF) : RR;
                    // lanes 8r..8r+7 (DF/8 lanes per row at DF < 64): row r's NumPy pairwise sum
                    // of squares, its clip scale
                    double ss;
                    if constexpr (DF == 64) ss = leaf_sumsq<64>(ring, -1, (unsigned)((lane >> 3) * 64), 64, lane);
                    else ss = batch_sumsq_small<DF>(ring, lane);
                    const double nrm = sqrt(ss);
                    const double sc = 1.0 / (nrm > 1.0 ? nrm : 1.0);  // 1.0 / np.maximum(norms, 1.0)
                    scl[lane / (DF / 8)] = sc;  // the lanes of a row write the same value
                    double* zp = zt + zoff + t * 128;
                    if constexpr (DF == 64) {
                        // lane j stores coordinate j of each row
                        if (nrows == RR) {
#pragma unroll
                            for (int r = 0; r < RR; ++r)
                                OCX_GEN_STORE(ring[64 * r + lane] * scl[r], zp + r * 128);
                        } else {
                            for (int r = 0; r < nrows; ++r)
                                OCX_GEN_STORE(ring[64 * r + lane] * scl[r], zp + r * 128);
                        }
                    } else {
                        // pass i: lane l stores coordinate l % DF of row i·kRP + l / DF
                        zp += rl * 128;
                        if (nrows == RR) {
#pragma unroll
                            for (int i = 0; i < 8; ++i)
                                OCX_GEN_STORE(ring[64 * i + lane] * scl[i * kRP + rl], zp + i * kRP * 128);
                        } else {
                            for (int i = 0; i * kRP < nrows; ++i)
                                if (i * kRP + rl < nrows)
                                    OCX_GEN_STORE(ring[64 * i + lane] * scl[i * kRP + rl], zp + i * kRP * 128);
                        }
                    }
                    const unsigned used = (unsigned)(nrows * DF);
                    ring[lane] = ring[used + lane];  // the next rows' first normals to the front
                    head -= used;
                    t += nrows;
                }
            }
        } else if constexpr (MODE == 0 && DF == 1024) {
            // d = 1024: full rounds (no need cap at the row's end).  The row always starts
            // at ring[0]; a round that completes it spills at most 63 normals of the next
            // row into ring[1024, 1087), which move to the front once the row has left.
            // (The ring is 1088 doubles: 4 waves' rings and the tables fill 160 KiB of LDS
            // with four 256-thread blocks, so the occupancy of the 1024 ring is kept.)
            constexpr int kFlat = 2047;  // every ring index is < 1088: masking is a no-op
            constexpr int kSW = OCX_GEN_SWZ1K ? 1 : 0;
            constexpr bool kF1k = OCX_GEN_1K_FLAT;
            const uint32_t total = (uint32_t)(nrows * 1024);
            uint32_t produced = 0;
            unsigned head = 0;
            int64_t t = t_off;
            const int64_t kst = G * T * 128;
            const double* rp = ring + st1k.j0;
            const int64_t pstep = st1k.kstep * kst;
            while (produced < total) {
#if OCX_GEN_INNER
                if (total - produced >= 1024u + 64u) {  // a whole row still to draw
                    do {
                        const int n = zig_round<true, true, kF1k, kSW, true>(w, 64, tb, ring, kFlat, head, lane);
                        produced += (uint32_t)n;
                        head += (unsigned)n;
                    } while (head < 1024u);
                } else
#endif
                {
                    const uint32_t left = total - produced;
                    const int n = left >= 64u
                                      ? zig_round<true, true, kF1k, kSW, true>(w, 64, tb, ring, kFlat, head, lane)
                                      : zig_round<true, false, kF1k, kSW, true>(w, (int)left, tb, ring,
                                                                         kFlat, head, lane);
                    produced += (uint32_t)n;
                    head += (unsigned)n;
                }
                if (head >= 1024u) {
                    // NumPy's pairwise sum of squares: lanes 8l..8l+7 keep leaf l's eight
                    // accumulators (16 values each), the 64 partials combine in its order
                    // slot 128a + b + 8q (a = lane/8, b = lane%8): its fields are disjoint, so
                    // rix of it is (128a + b + 8(a%4)) ^ (8q + 2((q/4)%4)), a lane base xor a
                    // constant
                    const unsigned o = (unsigned)((lane >> 3) * 128 + (lane & 7));
                    const unsigned osw = kSW ? (o | (unsigned)(((lane >> 3) & 3) << 3)) : o;
                    double v[16];
#pragma unroll
                    for (int q = 0; q < 16; ++q)
                        v[q] = ring[kSW ? (osw ^ (8u * q + 2u * ((q >> 2) & 3))) : o + 8u * q];
                    double acc = v[0] * v[0];
#pragma unroll
                    for (int q = 1; q < 16; ++q) acc += v[q] * v[q];
                    const double nrm = sqrt(ocx_seq_sum<64>(acc));
                    const double scr = 1.0 / (nrm > 1.0 ? nrm : 1.0);
                    double* zrow = zt + (int64_t)g * T * 128 + t * 128 + (int64_t)s * 2 * P;
                    if (kSW && P == 32) {
                        // the 32 x 32 layout: slot 32·(l/2) + l%2 + 2i, rix = base ^ 2i with
                        // base = 32·(l/2) + l%2 + 2·((l/2) % 16)
                        double* zp = zrow + st1k.w0;
                        const unsigned jb = (unsigned)st1k.j0 | (unsigned)(((lane >> 1) & 15) << 1);
#pragma unroll
                        for (int i = 0; i < 16; ++i)
                            __builtin_nontemporal_store(ring[jb ^ (2u * i)] * scr, zp + i * kst);
                    } else if (kSW && P == 64) {
                        // the 64 x 16 layout (one sequence per wave): store i fills half i%2 of
                        // plane i/2; its slot (l/2)·16 + l%2 + 2(i/2) + 512(i%2) maps to
                        // rix = base ^ 2(i/2) + 512(i%2), base = ((l/2)·16 + l%2) ^ ((l/2) & 30):
                        // no per-store index arithmetic, and the 32 lanes of each half read 32
                        // distinct bank pairs
                        const unsigned jb = ((unsigned)(lane >> 1) * 16u + (unsigned)(lane & 1)) ^
                                            ((unsigned)(lane >> 1) & 30u);
                        double* zp = zrow + lane;
#pragma unroll
                        for (int i = 0; i < 16; ++i)
                            __builtin_nontemporal_store(ring[(jb ^ (2u * (unsigned)(i >> 1))) + 512u * (unsigned)(i & 1)] * scr,
                                                        zp + (i >> 1) * kst + (i & 1) * 64);
                    } else if (P <= 32) {
                        double* zp = zrow + st1k.k0 * kst + st1k.w0;
#pragma unroll
                        for (int i = 0; i < 16; ++i)
                            __builtin_nontemporal_store(
                                ring[rix<kSW>((unsigned)(st1k.j0 + i * st1k.jstep))] * scr,
                                zp + i * pstep);
                    } else {
#pragma unroll 4
                        for (int i = 0; i < 16; ++i) {
                            const int f = i * 64 + lane;
                            const int k = f >> lg2P, wo = f & (2 * P - 1);
                            const int j = (wo >> 1) * C + 2 * k + (wo & 1);
                            __builtin_nontemporal_store(ring[rix<kSW>((unsigned)j)] * scr,
                                                        zrow + k * kst + wo);
                        }
                    }
                    // the spill moves to the front (LDS operations of a wave run in order:
                    // the row's reads above complete before these writes)
                    const unsigned ov = head - 1024u;
                    const double sp = ring[rix<kSW>(1024u + (lane < 63 ? lane : 63))];
                    if ((unsigned)lane < ov) ring[rix<kSW>((unsigned)lane)] = sp;
                    head = ov;
                    ++t;
                }
            }
        } else {
        const int64_t rows = (MODE == 0) ? nrows : T_seed;
        uint32_t remaining = (uint32_t)(rows * d);  // normals still to draw (< 2^32, host-checked)
        unsigned head = 0, tailp = 0;  // ring counters (mod 2^32; masked on use)
        unsigned partial = 0;          // normals of the row being filled
        int ready = 0;                 // whole rows waiting in the ring
        int64_t t = t_off;
        while (remaining > 0) {
            int need = remaining < 64 ? (int)remaining : 64;
            const int n = zig_round<MODE == 0>(w, need, tb, ring, rmask, head, lane);
            head += n;
            remaining -= (uint32_t)n;
            if (MODE != 0) continue;
            partial += (unsigned)n;
            while (partial >= (unsigned)d) {
                partial -= (unsigned)d;
                ++ready;
            }
            while (ready >= R || (remaining == 0 && ready > 0)) {
                const int nrows = ready < R ? ready : R;
                // this lane's row of the batch and its clip scale
                double sc = 1.0;
#ifdef OCX_GEN_TUNE_NO_NORM  // tuning only: no row norms (unclipped rows)
                if (false) {
#else
                if (!RAW && d <= 128) {
#endif
                    const int r = d < 8 ? lane : (lane >> 3);
                    const unsigned o = tailp + (unsigned)(r * d);
                    double ss = 0.0;
                    if (d < 8) {
                        for (int i = 0; i < d; ++i) {
                            const double v = ring[(o + i) & rmask];
                            ss += v * v;
                        }
                    } else {
                        ss = leaf_sumsq<DF>(ring, rmask, o, d, lane);
                    }
                    const double nrm = sqrt(ss);
                    sc = 1.0 / (nrm > 1.0 ? nrm : 1.0);  // 1.0 / np.maximum(norms, 1.0)
                }
                const int sc_stride = d < 8 ? 1 : 8;
                if (Dp <= 64 && d <= 128 && RP == 1) {
                    for (int r = 0; r < nrows; ++r) {
                        const double scr = __hiloint2double(
                            __builtin_amdgcn_readlane(__double2hiint(sc), r * sc_stride),
                            __builtin_amdgcn_readlane(__double2loint(sc), r * sc_stride));
                        if (rl == 0) {
                            const double v =
                                jl < d ? ring[(tailp + (unsigned)(r * d + jl)) & rmask] * scr : 0.0;
                            OCX_GEN_STORE(v, zt + zoff + (t + r) * 128);
                        }
                    }
                } else if (Dp <= 64 && d <= 128) {
                    for (int r0 = 0; r0 < nrows; r0 += RP) {
                        const int r = r0 + rl;
                        const double scr = shfl_double(sc, (r < 64 / sc_stride ? r : 0) * sc_stride);
                        if (rl < RP && r < nrows) {
                            const double v =
                                jl < d ? ring[(tailp + (unsigned)(r * d + jl)) & rmask] * scr : 0.0;
                            OCX_GEN_STORE(v, zt + zoff + (t + r) * 128);
                        }
                    }
                } else {
                    for (int r = 0; r < nrows; ++r) {
                        const unsigned o = tailp + (unsigned)(r * d);
                        double scr;
                        if (RAW) {
                            scr = 1.0;
                        } else if (d > 128) {
                            const double nrm = sqrt(row_sumsq(ring, rmask, o, d, lane, stk));
                            scr = 1.0 / (nrm > 1.0 ? nrm : 1.0);
                        } else {
                            scr = shfl_double(sc, r * sc_stride);
                        }
                        for (int j = lane; j < Dp; j += 64) {
                            const double v = j < d ? ring[(o + (unsigned)j) & rmask] * scr : 0.0;
                            __builtin_nontemporal_store(v, zaddr(t + r, j));
                        }
                    }
                }
                tailp += (unsigned)(nrows * d);
                t += nrows;
                ready -= nrows;
            }
        }
        }  // generic row loop
        ws_sync_base<kLS>(w);
        if (MODE == 1) {
            if (lane == 0) save_state6(lab_out + 6 * b, w.base, w.inc, 0, 0);
            continue;
        }
        if (st_out != nullptr && lane == 0) save_state6(st_out + 6 * b, w.base, w.inc, 0, 0);
        if (!labels) continue;

        // ---- labels: choice([-1., 1.], T) = top bit of each buffered uint32, low half first
        uint32_t buf32 = 0;
        int has32 = 0;
        if (lab_in != nullptr) {
            ocx_u128 ls, li;
            load_state6(lab_in + 6 * b, ls, li, buf32, has32);
            w.base = rl128(ls, 0);
        }
        int64_t tl = 0;
        if (has32 && T > 0) {  // (chunk mode only: never with stage_y)
            if (lane == 0) yrow[0] = (buf32 >> 31) ? 1.0 : -1.0;
            has32 = 0;
            tl = 1;
        }
        while (tl < T) {
            const int64_t left = T - tl;
            const int ndraw = left >= 128 ? 64 : (int)((left + 1) / 2);
            const ocx_u128 st = mul_add_u128(w.Ak, w.base, w.Dk);
            const uint64_t r = xsl_rr(st);
            const int64_t t0 = tl + 2 * lane;
            if (stage_y) {
                ring[2 * lane] = (((uint32_t)r) >> 31) ? 1.0 : -1.0;
                ring[2 * lane + 1] = (((uint32_t)(r >> 32)) >> 31) ? 1.0 : -1.0;
                store_y_round(tl, b - (b % kNW));
            } else if (lane < ndraw) {
                yrow[t0 * S] = (((uint32_t)r) >> 31) ? 1.0 : -1.0;
                if (t0 + 1 < T) yrow[(t0 + 1) * S] = (((uint32_t)(r >> 32)) >> 31) ? 1.0 : -1.0;
            }
            if (left < 128 && (left & 1)) {  // the last draw's high half stays buffered
                has32 = 1;
                buf32 = (uint32_t)(rl64(r, ndraw - 1) >> 32);
            }
            w.base = rl128(st, ndraw - 1);
            tl += 2 * (int64_t)ndraw;
        }
        if (lab_out != nullptr && lane == 0) save_state6(lab_out + 6 * b, w.base, w.inc, buf32, has32);
    }
}

namespace {

int ring_doubles(int64_t d, int DF, bool LR = false) {
    if (DF == 1024) return 1024 + 64;  // one row + the next row's first round (ocx_gen_wave_kernel)
    // R rows + one round, the R row scales; the default form also the deferred-wedge list
    // (kPendMax 16-B entries) and one flag byte per ring slot
    if (DF == 64)
        return kRows64 * 64 + 64 + 8 + ((OCX_GEN_DEFER && !LR) ? 2 * kPendMax + (kRows64 * 64 + 64) / 8 : 0);
    if (DF == 16 || DF == 32) return 512 + 64 + 512 / DF;  // a 512-normal batch + one round, the scales
    // a full batch of rows plus one round of normals
    int rb = 128;
    while (rb < (int64_t)batch_rows((int)d) * d + 65) rb *= 2;
    return rb;
}

template <int MODE, int DF, bool LR = false, bool RAW = false>
hipError_t launch_wave_df(uint64_t base_seed, int64_t T_seed, int64_t run0, int64_t B,
                          int64_t nseq, int64_t T, int64_t d, int P, int C, int64_t G, double* zt,
                          double* ytl, const uint64_t* st_in, uint64_t* st_out,
                          const uint64_t* lab_in, uint64_t* lab_out, hipStream_t st,
                          int64_t t_off = 0, int64_t nrows = -1, int labels = 1) {
    constexpr int kBlock = gen_block(DF, LR);
    const int rb = (MODE == 0) ? ring_doubles(d, DF, LR) : 0;
    const size_t lds =
        (MODE == 0) ? (size_t)(rb + (DF == 0 && d > 128 ? kStackDoubles : 0)) * 8 * (kBlock / 64) : 0;
    // resident waves: fill the GPU once, sequences spread evenly over the waves
    int dev = 0, cus = 256, per_cu = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (e != hipSuccess) return e;
    // OCX_GEN_CUS: CUs the launch may use (a stream restricted to a CU mask)
    if (const char* ev = std::getenv("OCX_GEN_CUS")) {
        const int n = std::atoi(ev);
        if (n > 0 && n < cus) cus = n;
    }
    {
        // the occupancy of this instance on a device depends only on its LDS size: query
        // once per (device, LDS size) — a device list may mix GPUs, and host threads of
        // ocx_gT_sweep_devices launch concurrently
        static std::mutex mu;
        static std::map<std::pair<int, size_t>, int> cache;
        std::lock_guard<std::mutex> lk(mu);
        const auto key = std::make_pair(dev, lds);
        auto it = cache.find(key);
        if (it == cache.end()) {
            int q = 0;
            e = hipOccupancyMaxActiveBlocksPerMultiprocessor(
                &q, ocx_gen_wave_kernel<MODE, DF, LR, RAW>, kBlock, lds);
            if (e != hipSuccess) return e;
            it = cache.emplace(key, q).first;
        }
        per_cu = it->second;
    }
    int64_t waves_per_cu = (int64_t)std::max(per_cu, 1) * (kBlock / 64);
    // OCX_GEN_WAVES_PER_SIMD caps the resident generator waves (leaves registers free for
    // a kernel running beside it on another stream)
    if (const char* ev = std::getenv("OCX_GEN_WAVES_PER_SIMD")) {
        const int64_t cap = std::atoll(ev);
        if (cap > 0) waves_per_cu = std::min<int64_t>(waves_per_cu, 4 * cap);
    }
    const int64_t resident = std::max<int64_t>(1, (int64_t)cus * waves_per_cu);
    const int64_t per_wave = (nseq + resident - 1) / resident;
    const unsigned blocks =
        (unsigned)(((nseq + per_wave - 1) / per_wave + (kBlock / 64) - 1) / (kBlock / 64));
    // every block full (a multiple of 4 waves: the staged label stores, see the kernel); the
    // waves past the last sequence run no sequence
    const int64_t nwaves = (int64_t)blocks * (kBlock / 64);
    hipLaunchKernelGGL((ocx_gen_wave_kernel<MODE, DF, LR, RAW>), dim3(blocks), dim3(kBlock), lds, st,
                       base_seed, T_seed, run0, B, nseq, T, (int)d, P, C, G, zt, ytl, st_in,
                       st_out, lab_in, lab_out, rb, nwaves, (int64_t)0, t_off, nrows < 0 ? T : nrows,
                       labels);
    return hipGetLastError();
}

// The overlapped pipeline's generator (ocx_pipeline.hip): the d = 64 default form in four-wave
// blocks over sequences [b_off, b_off + nseq) of L, at most `wps` waves per SIMD.  The cap is
// set through the LDS request (each block asks for a CU's LDS / wps, so no CU takes more than
// wps blocks) and leaves every SIMD the registers of one more wave for the FTRL kernel running
// beside it on another stream.  One wave per stream (nseq <= the cap's resident waves makes a
// single round).
struct OvGeom {
    size_t lds = 0;
    int per_cu = 0;
};
template <int DF, int OV>
OvGeom ov_geometry(int dev, int wps) {
    static std::mutex mu;
    static std::map<std::pair<int, int>, OvGeom> cache;
    std::lock_guard<std::mutex> lk(mu);
    const auto key = std::make_pair(dev, wps);
    auto it = cache.find(key);
    if (it != cache.end()) return it->second;
    OvGeom gm;
    int lds_cu = 0;
    if (hipDeviceGetAttribute(&lds_cu, hipDeviceAttributeMaxSharedMemoryPerMultiprocessor, dev) !=
            hipSuccess || lds_cu <= 0)
        lds_cu = 160 * 1024;
    const size_t base = (size_t)ring_doubles(DF, DF) * 8 * 4;  // four waves' rings
    size_t lds = base;
    int q = 0;
    for (; lds <= (size_t)lds_cu; lds += 512) {
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&q, ocx_gen_wave_kernel<0, DF, false, false, OV>,
                                                         256, lds) != hipSuccess)
            break;
        if (q <= wps) break;
    }
    gm.lds = lds;
    gm.per_cu = q;
    cache.emplace(key, gm);
    return gm;
}

}  // namespace

namespace {
template <int DF>
hipError_t launch_gen_range_df(const ocx_layout* L, uint64_t base_seed, int64_t run0, int64_t b_off,
                               int64_t nseq, int wps, double* zt, double* ytl, hipStream_t st) {
    int dev = 0, cus = 256;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (e != hipSuccess) return e;
    // up to three waves per SIMD the 128-VGPR form (one FTRL wave of <= 128 VGPRs fits
    // beside it); four or more: the 96-VGPR form (a few spills)
    const bool w4 = wps >= 4;
    const OvGeom gm = w4 ? ov_geometry<DF, 5>(dev, wps) : ov_geometry<DF, 4>(dev, wps);
    const int64_t resident = (int64_t)cus * 4 * std::max(1, std::min(gm.per_cu, wps));
    const int64_t per_wave = (nseq + resident - 1) / resident;
    const unsigned blocks = (unsigned)(((nseq + per_wave - 1) / per_wave + 3) / 4);
    const int64_t nwaves = (int64_t)blocks * 4;
    if (w4)
        hipLaunchKernelGGL((ocx_gen_wave_kernel<0, DF, false, false, 5>), dim3(blocks), dim3(256),
                           gm.lds, st, base_seed, L->T, run0, L->B, nseq, L->T, (int)L->d,
                           (int)L->P, (int)L->C, L->G, zt, ytl, (const uint64_t*)nullptr,
                           (uint64_t*)nullptr, (const uint64_t*)nullptr, (uint64_t*)nullptr,
                           ring_doubles(DF, DF), nwaves, b_off, (int64_t)0, L->T, 1);
    else
        hipLaunchKernelGGL((ocx_gen_wave_kernel<0, DF, false, false, 4>), dim3(blocks), dim3(256),
                           gm.lds, st, base_seed, L->T, run0, L->B, nseq, L->T, (int)L->d,
                           (int)L->P, (int)L->C, L->G, zt, ytl, (const uint64_t*)nullptr,
                           (uint64_t*)nullptr, (const uint64_t*)nullptr, (uint64_t*)nullptr,
                           ring_doubles(DF, DF), nwaves, b_off, (int64_t)0, L->T, 1);
    return hipGetLastError();
}
}  // namespace

// The overlapped pipeline's generator: rows of d = 16 / 32 / 64 filling their lanes (P·C = d), in
// four-wave blocks over sequences [b_off, b_off + nseq) of L, at most `wps` waves per SIMD (see
// ov_geometry).
hipError_t ocx_launch_gen_gT_range(const ocx_layout* L, uint64_t base_seed, int64_t run0,
                                   int64_t b_off, int64_t nseq, int wps, double* zt, double* ytl,
                                   hipStream_t st) {
    if (nseq <= 0 || L->T == 0) return hipSuccess;
    if ((L->d != 64 && L->d != 32 && L->d != 16) || L->P * L->C != L->d || b_off % 4 || nseq % 4)
        return hipErrorInvalidValue;
    if (L->T * L->d >= ((int64_t)1 << 32)) return hipErrorInvalidValue;
    if (L->d == 16) return launch_gen_range_df<16>(L, base_seed, run0, b_off, nseq, wps, zt, ytl, st);
    if (L->d == 32) return launch_gen_range_df<32>(L, base_seed, run0, b_off, nseq, wps, zt, ytl, st);
    return launch_gen_range_df<64>(L, base_seed, run0, b_off, nseq, wps, zt, ytl, st);
}

// The few-stream (LR) form over sequences [b_off, b_off + nseq) of L, one wave per stream,
// six waves per SIMD (80 VGPRs): a generator round for ocx_run_gen_rounds' tuning forms.
hipError_t ocx_launch_gen_gT_range_lr(const ocx_layout* L, uint64_t base_seed, int64_t run0,
                                      int64_t b_off, int64_t nseq, double* zt, double* ytl,
                                      hipStream_t st) {
    if (nseq <= 0 || L->T == 0) return hipSuccess;
    if (L->d != 64 || L->P * L->C != 64 || b_off % 4 || nseq % 4) return hipErrorInvalidValue;
    if (L->T * L->d >= ((int64_t)1 << 32)) return hipErrorInvalidValue;
    constexpr int kBlock = gen_block(64, true);
    const int rb = ring_doubles(64, 64, true);
    const size_t lds = (size_t)rb * 8 * (kBlock / 64);
    const unsigned blocks = (unsigned)(nseq / (kBlock / 64));
    hipLaunchKernelGGL((ocx_gen_wave_kernel<0, 64, true, false, 0>), dim3(blocks), dim3(kBlock), lds,
                       st, base_seed, L->T, run0, L->B, nseq, L->T, (int)L->d, (int)L->P,
                       (int)L->C, L->G, zt, ytl, (const uint64_t*)nullptr, (uint64_t*)nullptr,
                       (const uint64_t*)nullptr, (uint64_t*)nullptr, rb, (int64_t)blocks * (kBlock / 64),
                       b_off, (int64_t)0, L->T, 1);
    return hipGetLastError();
}

namespace {

template <int MODE>
hipError_t launch_wave(uint64_t base_seed, int64_t T_seed, int64_t run0, int64_t B, int64_t nseq,
                       int64_t T, int64_t d, int P, int C, int64_t G, double* zt, double* ytl,
                       const uint64_t* st_in, uint64_t* st_out, const uint64_t* lab_in,
                       uint64_t* lab_out, hipStream_t st, int64_t t_off = 0, int64_t nrows = -1,
                       int labels = 1) {
    // the kernel counts a sequence's normals in 32 bits
    if ((MODE == 0 ? T : T_seed) * d >= ((int64_t)1 << 32)) return hipErrorInvalidValue;
    if (d == 64 && (MODE == 1 || (int64_t)P * C == 64)) {
        // Two forms: the default (4 waves per SIMD's register budget) and the few-stream one
        // (6 waves per SIMD; round 2 measured these with a 7-row, 4 KB ring for the latter
        // and an 8 KB ring for the former: both now share the 4.6 KB ring).  Every wave takes
        // ceil(streams / slots) whole streams, so a form's makespan is that count times the
        // waves of its busiest SIMD; the low-LDS form wins where that is smaller, or equal
        // within the ~6 % its extra waves buy per stream when it really runs more waves per
        // SIMD (1e6 x T=100: 23.9 vs 25.3 ms; 131072 x 1e3: 30.4 vs 31.4; 4900 x 1e5: 117 vs
        // 161), and loses where its rounding is worse (32768 x 1e4: 78.9 vs 75.6 ms;
        // profiles/r02_gen_forms.jsonl).
        int dev = 0, cus = 256;
        hipError_t e = hipGetDevice(&dev);
        if (e != hipSuccess) return e;
        e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        if (e != hipSuccess) return e;
        const int64_t simds = 4 * (int64_t)cus;
        auto load = [&](int64_t w, int64_t& wps) {  // makespan in stream units, waves/SIMD
            const int64_t per_wave = (nseq + w * simds - 1) / (w * simds);
            const int64_t nw = (nseq + per_wave - 1) / per_wave;
            wps = (nw + simds - 1) / simds;
            return per_wave * wps;
        };
        int64_t wps4 = 0, wps6 = 0;
        const int64_t l4 = load(4, wps4), l6 = load(6, wps6);
        bool lr = l6 < l4 || (wps6 > wps4 && (double)l6 <= 1.06 * (double)l4);
        // OCX_GEN_FORM=default|lr forces the form (tests, tuning and counter probes: the
        // few-stream form's four-wave blocks place one wave per SIMD per 1 024 streams)
        if (const char* ev = std::getenv("OCX_GEN_FORM")) {
            if (!std::strcmp(ev, "lr")) lr = true;
            else if (!std::strcmp(ev, "default")) lr = false;
        }
        if (MODE == 0 && lr)
            return launch_wave_df<MODE, 64, true>(base_seed, T_seed, run0, B, nseq, T, d, P, C, G,
                                                  zt, ytl, st_in, st_out, lab_in, lab_out, st,
                                                  t_off, nrows, labels);
        return launch_wave_df<MODE, 64>(base_seed, T_seed, run0, B, nseq, T, d, P, C, G, zt, ytl,
                                        st_in, st_out, lab_in, lab_out, st, t_off, nrows, labels);
    }
    // d = 16 / 32 rows that fill their lanes (P·C = d): the d = 64 loop's form over 512-normal
    // batches (OCX_GEN_SMALL=0: the generic loop, tuning)
    if constexpr (MODE == 0) {
        const char* gs = std::getenv("OCX_GEN_SMALL");
        if ((d == 16 || d == 32) && (int64_t)P * C == d && (!gs || std::atoi(gs) != 0)) {
            if (d == 16)
                return launch_wave_df<MODE, 16>(base_seed, T_seed, run0, B, nseq, T, d, P, C, G, zt,
                                                ytl, st_in, st_out, lab_in, lab_out, st, t_off, nrows,
                                                labels);
            return launch_wave_df<MODE, 32>(base_seed, T_seed, run0, B, nseq, T, d, P, C, G, zt, ytl,
                                            st_in, st_out, lab_in, lab_out, st, t_off, nrows, labels);
        }
    }
    if (MODE == 0 && d == 1024 && (int64_t)P * C == 1024 && P <= 64)
        return launch_wave_df<MODE, 1024>(base_seed, T_seed, run0, B, nseq, T, d, P, C, G, zt,
                                          ytl, st_in, st_out, lab_in, lab_out, st, t_off, nrows,
                                          labels);
    return launch_wave_df<MODE, 0>(base_seed, T_seed, run0, B, nseq, T, d, P, C, G, zt, ytl,
                                   st_in, st_out, lab_in, lab_out, st, t_off, nrows, labels);
}

}  // namespace

namespace {
template <int DF>
int64_t resident_waves_df(int64_t d, int dev) {
    constexpr int kBlock = gen_block(DF, false);
    const size_t lds = (size_t)(ring_doubles(d, DF) + (DF == 0 && d > 128 ? kStackDoubles : 0)) * 8 *
                       (kBlock / 64);
    int q = 0, cus = 256;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&q, ocx_gen_wave_kernel<0, DF>, kBlock, lds) !=
            hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        return 0;
    return (int64_t)q * (kBlock / 64) * cus;
}
}  // namespace

// Streams the g(T) generator runs at once (one wave each) for rows of d on device `dev`: the
// batch size below which it runs a single round (gT_run's batch sizing).
int64_t ocx_gen_resident_waves(int64_t d, int dev) {
    if (d == 1024) return resident_waves_df<1024>(d, dev);
    if (d == 16) return resident_waves_df<16>(d, dev);
    if (d == 32) return resident_waves_df<32>(d, dev);
    if (d == 64) return resident_waves_df<64>(d, dev);
    return resident_waves_df<0>(d, dev);
}

hipError_t ocx_launch_gen_gT(const ocx_layout* L, uint64_t base_seed, int64_t run0, double* zt,
                             double* ytl, hipStream_t st) {
    const int64_t nseq = L->G * L->S;
    if (nseq == 0 || L->T == 0) return hipSuccess;
    // d = 64 batches of four or more generator rounds: one round per launch over two streams
    // (ocx_run_gen_rounds), bit-identical; OCX_GEN_ROUNDS=0 keeps the single launch (tuning),
    // and so does a stream whose capture cannot fork (ocx_stream_fork_ok)
    const char* gr = std::getenv("OCX_GEN_ROUNDS");
    if ((!gr || std::atoi(gr) != 0) && L->d == 64 && ocx_pipeline_supported(L) &&
        ocx_pipeline_worth(L, 4) && ocx_stream_fork_ok(st))
        return ocx_run_gen_rounds(L, base_seed, run0, zt, ytl, st);
    return launch_wave<0>(base_seed, L->T, run0, L->B, nseq, L->T, L->d, L->P, L->C, L->G, zt,
                          ytl, nullptr, nullptr, nullptr, nullptr, st);
}

hipError_t ocx_launch_gen_gT_raw(const ocx_layout* L, uint64_t base_seed, int64_t run0, double* zt,
                                 double* ytl, hipStream_t st) {
    const int64_t nseq = L->G * L->S;
    if (nseq == 0 || L->T == 0) return hipSuccess;
    if (L->T * L->d >= ((int64_t)1 << 32)) return hipErrorInvalidValue;
    return launch_wave_df<0, 0, false, true>(base_seed, L->T, run0, L->B, nseq, L->T, L->d, L->P,
                                             L->C, L->G, zt, ytl, nullptr, nullptr, nullptr,
                                             nullptr, st);
}

hipError_t ocx_launch_gen_seek(uint64_t base_seed, int64_t T_seed, int64_t run0, int64_t B,
                               int64_t d, uint64_t* st_out, uint64_t* lab_out, hipStream_t st) {
    if (B == 0) return hipSuccess;
    return launch_wave<1>(base_seed, T_seed, run0, B, B, 0, d, 1, 2, 0, nullptr, nullptr,
                          nullptr, st_out, nullptr, lab_out, st);
}

hipError_t ocx_launch_gen_gT_chunk(const ocx_layout* L, int64_t T_seed, const uint64_t* st_in,
                                   uint64_t* st_out, const uint64_t* lab_in, uint64_t* lab_out,
                                   double* zt, double* ytl, hipStream_t st) {
    const int64_t nseq = L->G * L->S;
    if (nseq == 0 || L->T == 0) return hipSuccess;
    return launch_wave<0>(0, T_seed, 0, L->B, nseq, L->T, L->d, L->P, L->C, L->G, zt, ytl, st_in,
                          st_out, lab_in, lab_out, st);
}

// Rows [t_off, t_off + nrows) of every sequence of L's full-horizon tile (the trailing
// pipeline, ocx_pipeline.hip): fresh streams _rng(base_seed, L->T, run0 + b) when st_in is
// null, else resumed from st_in[b]; the stream after the rows is saved to st_out[b]
// (nullable; a buffer other than st_in).  labels: the last row range of a horizon also draws the T
// labels that follow its normals (fast_algorithms.py:239), as a whole-horizon launch does.
hipError_t ocx_launch_gen_gT_rows(const ocx_layout* L, uint64_t base_seed, int64_t run0,
                                  int64_t t_off, int64_t nrows, const uint64_t* st_in,
                                  uint64_t* st_out, int labels, double* zt, double* ytl,
                                  hipStream_t st) {
    const int64_t nseq = L->G * L->S;
    if (nseq == 0 || L->T == 0 || nrows <= 0) return hipSuccess;
    if (t_off < 0 || t_off + nrows > L->T) return hipErrorInvalidValue;
    return launch_wave<0>(base_seed, L->T, run0, L->B, nseq, L->T, L->d, L->P, L->C, L->G, zt, ytl,
                          st_in, st_out, nullptr, nullptr, st, t_off, nrows, labels);
}
