// ocx_pipeline.hip — generation of the g(T) adversary overlapped with the FTRL pass
// (fast_algorithms.py:230-247: each run's z, y drawn, then simulated).
//
// The two kernels are bound by different units: the generator (ocx_gen_wave.hip) by the
// VALU — a 128-bit LCG and the ziggurat per normal, ≈74 VALU + 39 SALU instructions per
// 64-normal row, writing at ≈3 TB/s — and the FTRL kernel by HBM reads (one pass, 6.3–6.5
// TB/s).  Run one after the other they take gen + FTRL (57.4 + 26.1 ms per 32 768 × 1e4 × 64
// batch).  Here a resident batch is cut into sub-batches of sequences; sub-batch i+1 is
// generated while the FTRL kernel reads sub-batch i on other streams.  Three things make
// the kernels share the CUs instead of queueing behind each other:
//   * the generator runs in four-wave blocks whose LDS request admits at most `wps` (4)
//     blocks per CU, i.e. 4 of its 96-VGPR waves per SIMD (ocx_launch_gen_gT_range);
//   * the FTRL kernel runs in its lean form (<= 128 VGPRs, ocx_launch_alg_pipe_lean), so one
//     FTRL wave fits on every SIMD beside them whenever its sub-batch is ready;
//   * consecutive sub-batches alternate between two streams per side (see below).
// A sub-batch is one round of generator waves (one stream per wave), so no generator wave
// idles at a sub-batch's end.  Sub-batch i of batch k+1 is generated into the region FTRL
// read for sub-batch i of batch k, after that read (events), so consecutive batches overlap
// too.  The kernels, and so every regret, are the sequential path's, bit for bit.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <vector>

#include "ocx_internal.h"
#include "ocx_sim_kernels.h"

namespace {

struct PipeCtx {
    std::mutex mu;
    bool init = false;
    hipStream_t sim = nullptr;
    hipStream_t gen2 = nullptr, sim2 = nullptr;  // the second generator / FTRL streams
    // fork: the caller's work so far (every library stream waits on it); join_*: each library
    // stream's last work, waited on by the caller's stream.  One event per role, so no event
    // is re-recorded within a call (a captured call then has one producer per event)
    hipEvent_t fork = nullptr, join_gen2 = nullptr, join_sim = nullptr, join_sim2 = nullptr;
    std::vector<hipEvent_t> ev_gen, ev_sim;
    std::vector<char> sim_recorded;
};
PipeCtx g_pipe[64];

hipError_t ensure_events(PipeCtx& c, size_t n) {
    while (c.ev_gen.size() < n) {
        hipEvent_t a, b;
        hipError_t e = hipEventCreateWithFlags(&a, hipEventDisableTiming);
        if (e != hipSuccess) return e;
        e = hipEventCreateWithFlags(&b, hipEventDisableTiming);
        if (e != hipSuccess) return e;
        c.ev_gen.push_back(a);
        c.ev_sim.push_back(b);
        c.sim_recorded.push_back(0);
    }
    return hipSuccess;
}

hipError_t pipe_init(PipeCtx& c) {  // under c.mu
    if (c.init) return hipSuccess;
    hipError_t e;
    if ((e = hipStreamCreateWithFlags(&c.sim, hipStreamNonBlocking)) != hipSuccess) return e;
    if ((e = hipStreamCreateWithFlags(&c.gen2, hipStreamNonBlocking)) != hipSuccess) return e;
    if ((e = hipStreamCreateWithFlags(&c.sim2, hipStreamNonBlocking)) != hipSuccess) return e;
    if ((e = hipEventCreateWithFlags(&c.join_gen2, hipEventDisableTiming)) != hipSuccess) return e;
    if ((e = hipEventCreateWithFlags(&c.join_sim, hipEventDisableTiming)) != hipSuccess) return e;
    if ((e = hipEventCreateWithFlags(&c.join_sim2, hipEventDisableTiming)) != hipSuccess) return e;
    if ((e = hipEventCreateWithFlags(&c.fork, hipEventDisableTiming)) != hipSuccess) return e;
    c.init = true;
    return hipSuccess;
}

int64_t lcm64(int64_t a, int64_t b) {
    int64_t x = a, y = b;
    while (y) {
        const int64_t t = x % y;
        x = y;
        y = t;
    }
    return a / x * b;
}

#define OCX_PIPE_TRY(expr)                    \
    do {                                      \
        hipError_t e_ = (expr);               \
        if (e_ != hipSuccess) return e_;      \
    } while (0)

}  // namespace

// Whether the multi-stream paths (the sub-batch pipeline, the generator rounds) may fork to
// the library streams from `st`: always outside graph capture; under capture only on a HIP
// runtime whose capture of a fork / join survives hipStreamEndCapture.  HIP 7.0 (the runtime
// torch 2.10+rocm7.0 ships, which the package's processes load) segfaults there on a plain
// three-stream fork / join with no library code at all (tools/capture_repro.hip stage 1 on
// torch's libamdhip64: profiles/r05_capture_repro_torchhip.log; the same pattern in torch
// alone, tools/capture_torch_repro.py, likewise), while ROCm 7.2's runtime captures it and
// this library's overlapped pipeline bit for bit (stages 1-3, r05_capture_repro.log).  On
// the older runtimes a captured call keeps to `st` (the sequential loop, same results).
bool ocx_stream_fork_ok(hipStream_t st) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(st, &cs) != hipSuccess || cs == hipStreamCaptureStatusNone) return true;
    int v = 0;
    return hipRuntimeGetVersion(&v) == hipSuccess && v >= 70200000;
}

// The layouts the sub-batch pipeline runs: d = 64 in the lean pipelined FTRL form's layouts
// (8 x 8, 16 x 4), and (round 6) the g(T) layouts of d = 16 / 32 (butterfly lanes of 2 / 4
// coordinates, P·C = d), whose FTRL side is the plain kernel over a group range
// (ocx_launch_alg_range).
bool ocx_pipeline_supported(const ocx_layout* L) {
    if (L->T <= 0 || L->T * L->d >= ((int64_t)1 << 32) || L->P * L->C != L->d) return false;
    if (L->d == 64) return ocx_pipe_lean_supported(L);
    // the FTRL side must be the arithmetic the sequential loop runs (ocx_launch_alg): the
    // pipelined kernel's lean form where that loop takes the pipelined kernel (8 x 4), the
    // plain kernel over group ranges otherwise (8 x 2)
    return (L->d == 16 || L->d == 32) && !L->chain && L->P == 8 &&
           (ocx_pipe_supported(L) ? ocx_pipe_lean_launchable(L) : L->C == 2);
}

// Whether cutting L's batch into generator rounds of `wps` waves per SIMD pays: at least four
// sub-batches (one round each).  A batch of a round or two (the capacity-limited T = 1e5
// batches of ~4 900 streams) would leave the generator's last round nearly empty, and one
// round at full occupancy (ocx_launch_gen_gT) beats two at four waves per SIMD.
bool ocx_pipeline_worth(const ocx_layout* L, int wps) {
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        cus = 256;
    return L->G * L->S >= 4 * (int64_t)cus * 4 * std::max(1, wps);
}

// Generation alone in rounds (ocx_launch_gen_gT for the d = 64 batches of four or more
// generator rounds): one round of four-wave blocks per launch, one stream per wave, the
// launches alternating between the caller's stream and a second one so that no round drains
// before the next starts, joined back on `st`.  The normals and labels are the one-launch
// generator's, bit for bit (the same kernel body).
hipError_t ocx_run_gen_rounds(const ocx_layout* L, uint64_t base_seed, int64_t run0, double* zt,
                              double* yt, hipStream_t st) {
    // The round's form (OCX_GEN_ROUNDS_FORM overrides, tuning): "lr6", the default, the
    // few-stream form (80 VGPRs) at six waves per SIMD; "ov5" / "ov4" the 96-VGPR four-wave-
    // block form at five / four.  32 768 x 1e4 x 64: 49.7 / 50.2 / 52.3 ms, one launch 58.1
    // ms, all bit-identical (profiles/r04_gen_rounds_forms.jsonl).  Alone, more waves per SIMD
    // pay; beside the FTRL kernel (the pipeline) the generator keeps four.
    const char* fe = std::getenv("OCX_GEN_ROUNDS_FORM");
    const bool lr6 = !fe || std::strcmp(fe, "lr6") == 0;
    const int wps = (fe && std::strcmp(fe, "ov5") == 0) ? 5 : (lr6 ? 6 : 4);
    if (!ocx_pipeline_supported(L) || L->d != 64) return hipErrorInvalidValue;
    int dev = 0, cus = 256;
    OCX_PIPE_TRY(hipGetDevice(&dev));
    OCX_PIPE_TRY(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    if (dev < 0 || dev >= 64) return hipErrorInvalidDevice;
    PipeCtx& c = g_pipe[dev];
    std::lock_guard<std::mutex> lk(c.mu);
    OCX_PIPE_TRY(pipe_init(c));
    const int64_t Bp = L->G * L->S;
    const int64_t unit = lcm64(L->S, 4);
    int64_t sub = (int64_t)cus * 4 * wps;
    sub = std::max(unit, (sub + unit - 1) / unit * unit);
    OCX_PIPE_TRY(hipEventRecord(c.fork, st));
    OCX_PIPE_TRY(hipStreamWaitEvent(c.gen2, c.fork, 0));
    int64_t j = 0;
    for (int64_t b0 = 0; b0 < Bp; b0 += sub, ++j)
        OCX_PIPE_TRY(lr6 ? ocx_launch_gen_gT_range_lr(L, base_seed, run0, b0, std::min(sub, Bp - b0),
                                                      zt, yt, (j & 1) ? c.gen2 : st)
                         : ocx_launch_gen_gT_range(L, base_seed, run0, b0, std::min(sub, Bp - b0),
                                                   wps, zt, yt, (j & 1) ? c.gen2 : st));
    OCX_PIPE_TRY(hipEventRecord(c.join_gen2, c.gen2));
    OCX_PIPE_TRY(hipStreamWaitEvent(st, c.join_gen2, 0));
    return hipSuccess;
}

// nbatch batches of L->B runs each (runs run0 + k·B, k < nbatch) through one z/y buffer of
// layout L; regret[] holds the last batch's regrets, gmax (nullable, device) folds the max
// over all of them in the FTRL kernel (bit pattern of g(T) = max(0, max regret)).  sub_seqs <= 0:
// one generator round per sub-batch (up to four below T = 1000).  Returns with the work queued
// on `st` (joined).
hipError_t ocx_run_gen_sim_pipelined(const ocx_layout* L, uint64_t base_seed, int64_t run0,
                                     int64_t nbatch, double* zt, double* yt, double eta0,
                                     double* regret, int onepass, unsigned long long* gmax,
                                     int wps, int64_t sub_seqs, hipStream_t st) {
    if (!ocx_pipeline_supported(L)) return hipErrorInvalidValue;
    int dev = 0, cus = 256;
    OCX_PIPE_TRY(hipGetDevice(&dev));
    OCX_PIPE_TRY(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    if (dev < 0 || dev >= 64) return hipErrorInvalidDevice;
    PipeCtx& c = g_pipe[dev];
    std::lock_guard<std::mutex> lk(c.mu);
    OCX_PIPE_TRY(pipe_init(c));
    // Two streams per side: consecutive sub-batches alternate between them, so one launch's
    // last waves need not drain before the next launch's first waves start (launches on one
    // stream are ordered).  A sub-batch is one round of generator waves, and a round whose
    // blocks the dispatcher does not spread evenly leaves part of the chip idle until its
    // slowest CU is done: 32 768 x 1e4 x 64, generation alone 64.1 -> 51.0 ms, the FTRL side
    // alone 31.1 -> 25.6 ms, pipelined 72.4 -> 66.9 ms per batch (profiles/r04_overlap2.jsonl).
    // Sub-batches write and read disjoint regions; only the gen(i) -> FTRL(i) and
    // FTRL(i, batch k) -> gen(i, batch k+1) events order them.  OCX_PIPE_GEN_STREAMS /
    // OCX_PIPE_SIM_STREAMS = 1 select one stream per side (tuning).
    const char* gs_env = std::getenv("OCX_PIPE_GEN_STREAMS");
    const char* ss_env = std::getenv("OCX_PIPE_SIM_STREAMS");
    const int ngs = (gs_env && std::atoi(gs_env) == 1) ? 1 : 2;
    const int nss = (ss_env && std::atoi(ss_env) == 1) ? 1 : 2;
    // the library streams start after the work already queued on the caller's stream: each
    // waits on the fork (under graph capture that wait is what makes it join the capture)
    OCX_PIPE_TRY(hipEventRecord(c.fork, st));
    OCX_PIPE_TRY(hipStreamWaitEvent(c.gen2, c.fork, 0));
    OCX_PIPE_TRY(hipStreamWaitEvent(c.sim, c.fork, 0));
    OCX_PIPE_TRY(hipStreamWaitEvent(c.sim2, c.fork, 0));
    const int64_t S = L->S;
    const int64_t Bp = L->G * S;  // sequences of the layout, padding included
    // sub-batch: whole wave-groups and whole four-wave generator blocks
    const int64_t unit = lcm64(S, 4);
    // sub_seqs <= 0: `rounds` generator rounds per sub-batch.  Short horizons take up to
    // four, so a launch holds at least ≈1 000 steps per stream's worth of rounds: the g(T)
    // sweep at T = 100 (1e6 runs) ran 3.70e9 -> 3.98e9 timesteps/s (g(T) alone 4.23e9 ->
    // 4.59e9) with four, T = 1e3 the same with one or four, and 16 was slower at T = 1e3
    // (profiles/r04_sweep_subrounds.jsonl).  OCX_PIPE_SUB_ROUNDS overrides (tuning).
    // (round 6: by normals per stream, T·d, rather than T: d = 16 / 32 rows are short, and
    // configs[1]'s 65 536 x 1e3 x 16 batch ran 5.60 / 5.13 / 5.01 ms with 1 / 2 / 4 rounds per
    // sub-batch against 5.42 ms sequential; d = 32: 7.98 / 7.94 / 8.10 vs 9.66 ms,
    // profiles/r06_small_pipe.jsonl.  d = 64 keeps 1000 / T.)
    int64_t rounds = std::max<int64_t>(1, std::min<int64_t>(4, 64000 / std::max<int64_t>(L->T * L->d, 1)));
    if (const char* e = std::getenv("OCX_PIPE_SUB_ROUNDS")) rounds = std::max<int64_t>(1, std::atoll(e));
    int64_t sub = sub_seqs > 0 ? sub_seqs : (int64_t)cus * 4 * std::max(1, wps) * rounds;
    sub = std::max(unit, (sub + unit - 1) / unit * unit);
    const int64_t nsub = (Bp + sub - 1) / sub;
    OCX_PIPE_TRY(ensure_events(c, (size_t)nsub));
    std::fill(c.sim_recorded.begin(), c.sim_recorded.end(), 0);
#ifdef OCX_PIPE_TUNE_SKIP
    // tuning builds only (wrong outputs): time one side of the pipeline alone
    const char* sk = std::getenv("OCX_PIPE_SKIP");
    const bool skip_gen = sk && sk[0] == 'g', skip_sim = sk && sk[0] == 's';
#else
    constexpr bool skip_gen = false, skip_sim = false;
#endif
    int64_t j = 0;  // sub-batch launches so far (stream alternation)
    for (int64_t k = 0; k < nbatch; ++k) {
        const int64_t r0 = run0 + k * L->B;
        for (int64_t i = 0; i < nsub; ++i, ++j) {
            const int64_t b0 = i * sub, nb = std::min(sub, Bp - b0);
            hipStream_t gs = (ngs == 2 && (j & 1)) ? c.gen2 : st;
            hipStream_t ss = (nss == 2 && (j & 1)) ? c.sim2 : c.sim;
            // this region's previous reader (sub-batch i of batch k-1) must be done
            if (c.sim_recorded[(size_t)i]) OCX_PIPE_TRY(hipStreamWaitEvent(gs, c.ev_sim[(size_t)i], 0));
            if (!skip_gen)
                OCX_PIPE_TRY(ocx_launch_gen_gT_range(L, base_seed, r0, b0, nb, wps, zt, yt, gs));
            OCX_PIPE_TRY(hipEventRecord(c.ev_gen[(size_t)i], gs));
            OCX_PIPE_TRY(hipStreamWaitEvent(ss, c.ev_gen[(size_t)i], 0));
            if (!skip_sim)
                OCX_PIPE_TRY(ocx_pipe_supported(L)
                                 ? ocx_launch_alg_pipe_lean(L, zt, yt, eta0, regret, onepass, b0 / S,
                                                            nb / S, gmax, ss)
                                 : ocx_launch_alg_range(L, zt, yt, eta0, regret, onepass, b0 / S,
                                                        nb / S, gmax, ss));
            OCX_PIPE_TRY(hipEventRecord(c.ev_sim[(size_t)i], ss));
            c.sim_recorded[(size_t)i] = 1;
        }
    }
    // the caller's stream sees every generator launch, FTRL pass and fold done (each stream
    // runs in order: its last event covers it)
    OCX_PIPE_TRY(hipEventRecord(c.join_gen2, c.gen2));
    OCX_PIPE_TRY(hipEventRecord(c.join_sim, c.sim));
    OCX_PIPE_TRY(hipEventRecord(c.join_sim2, c.sim2));
    OCX_PIPE_TRY(hipStreamWaitEvent(st, c.join_gen2, 0));
    OCX_PIPE_TRY(hipStreamWaitEvent(st, c.join_sim, 0));
    OCX_PIPE_TRY(hipStreamWaitEvent(st, c.join_sim2, 0));
    return hipSuccess;
}

// ---------------------------------------------------------------------------------------------
// The trailing pipeline: generation of batch k+1 overlapped with the FTRL pass over batch k
// INSIDE ONE z buffer, for the batches the HBM budget caps (d = 64 at T = 1e5: ≈4 900 streams;
// d = 1024 at T = 1e4: ≈2 700), where a double buffer would halve the batch and the sub-batch
// pipeline above has too few generator rounds to cut.  The horizon is cut into n chunks of
// whole 64-step blocks.  FTRL over batch k runs chunk by chunk (ocx_launch_alg_pipe_chunk:
// the step's state carried through HBM, bit-identical to one launch), and the generator of
// batch k+1 writes chunk c's rows (ocx_launch_gen_gT_rows: the stream resumed from the state
// chunk c−1 left) as soon as FTRL k has read them — an event per chunk orders that — so the
// generator trails the reader through the same rows.  NumPy draws a sequence's labels after
// all of its T·d normals (fast_algorithms.py:234-239), so the last chunk's launch draws them,
// into the other of two label tiles (y is 1/d of z); FTRL k+1 starts when that is done.
// Per batch the FTRL pass then hides behind generation except for its first chunk.
//
// z, y[2]: the layout's tiles; gst: 2·(G·S)·6 words of generator states (ping-pong);
// fst: ocx_pipe_state_doubles(L); bad[nbatch]: set for a batch with a sequence the closed-form
// comparator could not certify (its regret is NaN: the caller reruns that batch whole);
// regret: nbatch·B doubles, batch k's at regret + k·B; gmax (nullable): g(T) folded in by
// each batch's last FTRL chunk.  The last batch may hold fewer runs (last_B <= B): it keeps the
// layout's tiles, its spare sequences are padding.
//
// Registers decide where it pays.  The FTRL chunks run in the lean form (<= 128 VGPRs) beside
// generator waves of the few-stream form (80 VGPRs: six per SIMD alone, four beside an FTRL
// wave), so a batch is capped where every generator wave still fits beside the FTRL waves
// (ocx_trailing_max_batch; 8 x 8 at d = 64: ≈4 900 streams).  d = 1024 keeps the sequential
// loop: its generator waves take 128 VGPRs and no 1 024-coordinate FTRL wave fits in 128, and
// the pairings that do fit measured slower than sequential (2.22e8 timesteps/s): the 32 x 32
// full form 2.15e8; a 64 x 16 grid-stride form (one FTRL wave of 256 VGPRs beside two generator
// waves per SIMD) 1.98e8, and beside three 80-VGPR generator waves 2.17e8 — the generator's
// chunks ran 9–13 ms beside the FTRL chunks against 7.3 ms alone (profiles/r05_trail_c4*.jsonl,
// DESIGN.md §3.8).
bool ocx_trailing_supported(const ocx_layout* L) {
    return ocx_pipe_lean_supported(L) && L->T >= 128 && L->T * L->d < ((int64_t)1 << 32);
}

int64_t ocx_trailing_max_batch(const ocx_layout* L) {
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        cus = 256;
    const int64_t simds = 4 * (int64_t)cus, S = L->S;
    // generator waves that fit: 4 on a SIMD beside an FTRL wave, 6 on one without
    int64_t b = simds * 6;
    while (b > S) {
        const int64_t nf = std::min(simds, (b + S - 1) / S);
        if (nf * 4 + (simds - nf) * 6 >= b) break;
        b -= S;
    }
    return b;
}

// batches that have entered the trailing pipeline in this process (ocx_test_trailing_batches)
static std::atomic<int64_t> g_trailing_batches{0};
int64_t ocx_trailing_batches_run() { return g_trailing_batches.load(); }

hipError_t ocx_run_gen_sim_trailing(const ocx_layout* L, uint64_t base_seed, int64_t run0,
                                    int64_t nbatch, double* zt, double* yt0, double* yt1,
                                    uint64_t* gst, double* fst, int* bad, double eta0,
                                    double* regret, int64_t last_B, unsigned long long* gmax,
                                    int nchunks, hipStream_t st) {
    if (!ocx_trailing_supported(L) || nbatch <= 0 || !regret || !gst || !fst || !bad ||
        last_B < 1 || last_B > L->B)
        return hipErrorInvalidValue;
    g_trailing_batches += nbatch;
    ocx_layout Ll = *L;  // the last batch: same tiles, last_B runs
    Ll.B = last_B;
    auto lay = [&](int64_t k) { return k + 1 == nbatch ? &Ll : L; };
    int dev = 0;
    OCX_PIPE_TRY(hipGetDevice(&dev));
    if (dev < 0 || dev >= 64) return hipErrorInvalidDevice;
    PipeCtx& c = g_pipe[dev];
    std::lock_guard<std::mutex> lk(c.mu);
    OCX_PIPE_TRY(pipe_init(c));
    // chunks of whole 64-step blocks (the FTRL state's refresh points), at least two.  Each
    // batch's FTRL pass can start only once the generator has drawn the batch's labels (after
    // all its normals), and the next batch's first generator chunk only once that pass has read
    // chunk 0: with equal chunks the generator idled for one FTRL chunk per batch (≈5 ms of a
    // ≈120 ms period at T = 1e5, profiles/r05_trail_kernel_trace.csv).  So the horizon starts
    // with a ramp (round 6): chunks of `ramp` blocks, doubling up to the standard size — the
    // reader, ≈2.3× faster per row than the writer, stays a chunk ahead from the first one.
    // OCX_TRAIL_RAMP (blocks, default 4; 0 = equal chunks) is a tuning knob.
    const int64_t blocks = (L->T + 63) / 64;
    const int64_t n = std::max<int64_t>(2, std::min<int64_t>(nchunks, blocks));
    const int64_t std_blocks = (blocks + n - 1) / n;
    int64_t ramp = 4;
    if (const char* e = std::getenv("OCX_TRAIL_RAMP")) ramp = std::max<int64_t>(0, std::atoll(e));
    std::vector<int64_t> cstart;  // first step of each chunk; cstart.back() == T
    for (int64_t b = 0, r = ramp > 0 ? ramp : std_blocks; b < blocks; r *= 2) {
        cstart.push_back(b * 64);
        b += std::min(std::min(r, std_blocks), blocks - b);
    }
    cstart.push_back(L->T);
    const int64_t nch = (int64_t)cstart.size() - 1;
    OCX_PIPE_TRY(ensure_events(c, (size_t)nch));
    const int64_t words = L->G * L->S * 6;
    double* yts[2] = {yt0, yt1};
    hipStream_t F = c.sim;
    OCX_PIPE_TRY(hipMemsetAsync(bad, 0, (size_t)nbatch * sizeof(int), st));
    // batch 0 in one launch (the plain one: ocx_launch_gen_gT's rounds would take this lock);
    // the FTRL stream starts after it and after the caller's work
    OCX_PIPE_TRY(ocx_launch_gen_gT_rows(lay(0), base_seed, run0, 0, L->T, nullptr, nullptr, 1, zt, yt0, st));
    for (int64_t k = 0; k < nbatch; ++k) {
        // FTRL k: batch k is generated (its last launch was queued on st just before)
        OCX_PIPE_TRY(hipEventRecord(c.fork, st));
        OCX_PIPE_TRY(hipStreamWaitEvent(F, c.fork, 0));
        double* yk = yts[k & 1];
        const bool next = k + 1 < nbatch;
        const int64_t rk = run0 + (k + 1) * L->B;
        for (int64_t ci = 0; ci < nch; ++ci) {
            const int64_t t0 = cstart[(size_t)ci], tn = cstart[(size_t)ci + 1] - t0;
            OCX_PIPE_TRY(ocx_launch_alg_pipe_chunk(lay(k), zt, yk, eta0, regret + k * L->B, 1, t0, tn,
                                                   fst, bad + k, gmax, F));
            OCX_PIPE_TRY(hipEventRecord(c.ev_sim[(size_t)ci], F));
            if (!next) continue;
            // batch k+1's chunk ci, behind FTRL k's; its labels with the last chunk
            const bool lastc = ci + 1 == nch;
            OCX_PIPE_TRY(hipStreamWaitEvent(st, c.ev_sim[(size_t)ci], 0));
            OCX_PIPE_TRY(ocx_launch_gen_gT_rows(lay(k + 1), base_seed, rk, t0, tn,
                                                ci == 0 ? nullptr : gst + ((ci - 1) & 1) * words,
                                                lastc ? nullptr : gst + (ci & 1) * words,
                                                lastc ? 1 : 0, zt, yts[(k + 1) & 1], st));
        }
    }
    OCX_PIPE_TRY(hipEventRecord(c.join_sim, F));
    OCX_PIPE_TRY(hipStreamWaitEvent(st, c.join_sim, 0));
    return hipSuccess;
}
