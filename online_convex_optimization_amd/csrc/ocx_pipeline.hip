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
    hipEvent_t join_gen2 = nullptr, join_sim2 = nullptr, fork = nullptr;
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

bool ocx_stream_capturing(hipStream_t st) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    return hipStreamIsCapturing(st, &cs) == hipSuccess && cs != hipStreamCaptureStatusNone;
}

bool ocx_pipeline_supported(const ocx_layout* L) {
    return L->d == 64 && L->P * L->C == 64 && ocx_pipe_lean_supported(L) && L->T > 0 &&
           L->T * L->d < ((int64_t)1 << 32);
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
    if (!ocx_pipeline_supported(L)) return hipErrorInvalidValue;
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
                                                   wps, zt, yt, (j & 1) ? c.gen2 : st, 1));
    OCX_PIPE_TRY(hipEventRecord(c.join_gen2, c.gen2));
    OCX_PIPE_TRY(hipStreamWaitEvent(st, c.join_gen2, 0));
    return hipSuccess;
}

// nbatch batches of L->B runs each (runs run0 + k·B, k < nbatch) through one z/y buffer of
// layout L; regret[] holds the last batch's regrets, dmax (nullable, device) folds the max
// over all of them (ocx_max_fold: bit pattern of g(T) = max(0, max regret)).  sub_seqs <= 0:
// one generator round per sub-batch (up to four below T = 1000).  Returns with the work queued
// on `st` (joined).
hipError_t ocx_run_gen_sim_pipelined(const ocx_layout* L, uint64_t base_seed, int64_t run0,
                                     int64_t nbatch, double* zt, double* yt, double eta0,
                                     double* regret, int onepass,
                                     hipError_t (*fold)(const double*, int64_t, void*, hipStream_t),
                                     void* fold_arg, int wps, int64_t sub_seqs, int cand,
                                     hipStream_t st) {
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
    // the extra streams start after the work already queued on the caller's stream
    OCX_PIPE_TRY(hipEventRecord(c.fork, st));
    OCX_PIPE_TRY(hipStreamWaitEvent(c.gen2, c.fork, 0));
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
    int64_t rounds = std::max<int64_t>(1, std::min<int64_t>(4, 1000 / std::max<int64_t>(L->T, 1)));
    if (const char* e = std::getenv("OCX_PIPE_SUB_ROUNDS")) rounds = std::max<int64_t>(1, std::atoll(e));
    int64_t sub = sub_seqs > 0 ? sub_seqs : (int64_t)cus * 4 * std::max(1, wps) * rounds;
    sub = std::max(unit, (sub + unit - 1) / unit * unit);
    const int64_t nsub = (Bp + sub - 1) / sub;
    OCX_PIPE_TRY(ensure_events(c, (size_t)nsub));
    std::fill(c.sim_recorded.begin(), c.sim_recorded.end(), 0);
    // tuning only (wrong outputs): time one side of the pipeline alone
    const char* sk = std::getenv("OCX_PIPE_SKIP");
    const bool skip_gen = sk && sk[0] == 'g', skip_sim = sk && sk[0] == 's';
    // the FTRL side's register budget (tuning, OCX_PIPE_LEAN): 128 VGPRs beside three
    // generator waves of the 128-VGPR form or four of the 96-VGPR one; 168 beside three of
    // the 96-VGPR form
    const char* lb = std::getenv("OCX_PIPE_LEAN");
    const int sim_budget = lb ? std::atoi(lb) : 128;
    // the generator's register form: 96 VGPRs when the FTRL side takes 168 (or at wps 4)
    const int gen96 = sim_budget >= 168 ? 1 : 0;
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
                OCX_PIPE_TRY(ocx_launch_gen_gT_range(L, base_seed, r0, b0, nb, wps, zt, yt, gs, gen96));
            OCX_PIPE_TRY(hipEventRecord(c.ev_gen[(size_t)i], gs));
            OCX_PIPE_TRY(hipStreamWaitEvent(ss, c.ev_gen[(size_t)i], 0));
            if (!skip_sim)
                OCX_PIPE_TRY(ocx_launch_alg_pipe_lean(L, zt, yt, eta0, regret, onepass, b0 / S, nb / S,
                                                      cand, ss, sim_budget));
            const int64_t nreal = std::min(nb, L->B - b0);
            if (fold && nreal > 0) OCX_PIPE_TRY(fold(regret + b0, nreal, fold_arg, ss));
            OCX_PIPE_TRY(hipEventRecord(c.ev_sim[(size_t)i], ss));
            c.sim_recorded[(size_t)i] = 1;
        }
    }
    // the caller's stream sees every generator launch, FTRL pass and fold done (each stream
    // runs in order: its last event covers it)
    if (nsub > 0 && nbatch > 0) {
        OCX_PIPE_TRY(hipEventRecord(c.join_gen2, c.gen2));
        OCX_PIPE_TRY(hipEventRecord(c.join_sim2, c.sim2));
        OCX_PIPE_TRY(hipStreamWaitEvent(st, c.join_gen2, 0));
        OCX_PIPE_TRY(hipStreamWaitEvent(st, c.join_sim2, 0));
        OCX_PIPE_TRY(hipEventRecord(c.fork, c.sim));
        OCX_PIPE_TRY(hipStreamWaitEvent(st, c.fork, 0));
    }
    return hipSuccess;
}
