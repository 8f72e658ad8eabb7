// ocx_capi.hip — the extern "C" boundary (include/ocx.h): layout planning, per-device
// workspaces for the host entry points, argument checking and error reporting.
// Host code, plus the g(T) max fold below; the other kernels live in ocx_sim.hip /
// ocx_gen*.hip.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/ocx.h"
#include "../../include/ocx_testing.h"
#include "ocx_sim_kernels.h"


namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}

#define OCX_HIP(expr)                                                                     \
    do {                                                                                  \
        hipError_t e_ = (expr);                                                           \
        if (e_ != hipSuccess)                                                             \
            return fail(OCX_E_HIP, std::string(#expr) + ": " + hipGetErrorString(e_));   \
    } while (0)

constexpr int kMaxDevices = 64;

// Grow-only device buffers for the host entry points (one set per device).
struct DevBuf {
    void* p = nullptr;
    size_t cap = 0;
    hipError_t release() {
        hipError_t e = p ? hipFree(p) : hipSuccess;
        p = nullptr;
        cap = 0;
        return e;
    }
    // Growing frees and maps again, which for the budget-sized batches (~250 GB) costs seconds.
    // Buffers of a GiB or more therefore get a little slack (1/8, at most 4 GiB, in 256-MiB
    // granules) when it fits, so the batches of successive calls — whose sizes differ by a few
    // streams' bytes as T changes — reuse the allocation (tools/full_configs.py).
    hipError_t ensure(size_t n) {
        if (n <= cap) return hipSuccess;
        if (p) {
            hipError_t e = hipFree(p);
            if (e != hipSuccess) return e;
            p = nullptr;
            cap = 0;
        }
        size_t want = n ? n : 16;
        if (n >= ((size_t)1 << 30)) {
            constexpr size_t kGran = (size_t)256 << 20;
            const size_t pad = std::min(n / 8, (size_t)4 << 30);
            want = (n + pad + kGran - 1) / kGran * kGran;
        }
        hipError_t e = hipMalloc(&p, want);
        if (e != hipSuccess && want != n) {  // no room for the slack: the exact size
            (void)hipGetLastError();
            want = n;
            e = hipMalloc(&p, want);
        }
        if (e == hipSuccess) cap = want;
        return e;
    }
    template <class T>
    T* as() const { return static_cast<T*>(p); }
};

struct DevCtx {
    std::mutex mu;
    bool init = false;
    hipStream_t stream = nullptr;
    DevBuf zraw, yraw, zt, yt, at, araw, cmp, thr, out, sw;
    DevBuf rstate, lstate, theta, acc;  // long-horizon (T-chunked) g(T) sweep
    DevBuf gmax;                        // ocx_gT_max: the running max's bit pattern
    DevBuf yt2, gst, fst, bad;          // the trailing pipeline (second label tile, states)
};

DevCtx g_ctx[kMaxDevices];

int ctx_enter(int device, DevCtx** out) {
    int n = 0;
    OCX_HIP(hipGetDeviceCount(&n));
    if (device < 0 || device >= n || device >= kMaxDevices)
        return fail(OCX_E_INVALID, "device " + std::to_string(device) + " out of range (count " +
                                       std::to_string(n) + ")");
    OCX_HIP(hipSetDevice(device));
    DevCtx* c = &g_ctx[device];
    {
        // one stream per device even when threads enter concurrently (gT_sweep over
        // several devices, or two host calls on one device)
        static std::mutex init_mu;
        std::lock_guard<std::mutex> lk(init_mu);
        if (!c->init) {
            OCX_HIP(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
            c->init = true;
        }
    }
    *out = c;
    return OCX_OK;
}

int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

// g(T) = max over runs of the regrets, starting from 0.0 with `reg > max`
// (fast_algorithms.py:228, :242-243).  Every candidate that can win is > +0.0 (a NaN never
// passes `>`), and positive doubles order as their bit patterns, so blocks and batches fold
// into *acc (initialised to +0.0) by a 64-bit unsigned atomic max: a selection, bit-identical
// to the host's loop over the same regrets.
__global__ void ocx_max_fold_kernel(const double* __restrict__ r, int64_t n,
                                    unsigned long long* __restrict__ acc) {
    double m = 0.0;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const double v = r[i];
        if (v > m) m = v;
    }
    for (int o = 32; o > 0; o >>= 1) {
        const double u = __shfl_down(m, o, 64);
        if (u > m) m = u;
    }
    if ((threadIdx.x & 63) == 0 && m > 0.0)
        atomicMax(acc, (unsigned long long)__double_as_longlong(m));
}

// acc = +0.0 by a one-lane kernel: an 8-byte hipMemsetAsync captured into a HIP graph
// replayed as 0xb8 bytes under HIP 7 (test_pipeline_captures_into_a_graph)
__global__ void ocx_zero_u64_kernel(unsigned long long* acc) { *acc = 0ULL; }

hipError_t launch_zero_u64(unsigned long long* acc, hipStream_t st) {
    hipLaunchKernelGGL(ocx_zero_u64_kernel, dim3(1), dim3(1), 0, st, acc);
    return hipGetLastError();
}

hipError_t launch_max_fold(const double* r, int64_t n, unsigned long long* acc, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    const unsigned grid = (unsigned)std::min<int64_t>((n + 255) / 256, 1024);
    hipLaunchKernelGGL(ocx_max_fold_kernel, dim3(grid), dim3(256), 0, st, r, n, acc);
    return hipGetLastError();
}

// The ocx_dev_* entry points take a stream, not a device: the stream's device is made
// current for the call (the launchers size their grids from the current device, and
// ocx_pipeline.hip's library streams and events belong to it) and the caller's restored
// afterwards.  The null stream is the caller's current device's.
struct StreamDevice {
    int prev = -1;
    explicit StreamDevice(void* stream) {
        if (!stream) return;
        int dev = -1, cur = -1;
        if (hipStreamGetDevice((hipStream_t)stream, &dev) != hipSuccess ||
            hipGetDevice(&cur) != hipSuccess || dev == cur)
            return;
        if (hipSetDevice(dev) == hipSuccess) prev = cur;
    }
    ~StreamDevice() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
    StreamDevice(const StreamDevice&) = delete;
    StreamDevice& operator=(const StreamDevice&) = delete;
};

int even_supported_C(int64_t need) {
    static const int Cs[] = {2, 4, 6, 8, 12, 16, 24, 32, 48, 64};
    for (int c : Cs)
        if (c >= need) return c;
    return -1;
}

}  // namespace

extern "C" {

int ocx_version(void) { return OCX_VERSION; }

int ocx_last_error(char* buf, size_t len) {
    if (buf && len) {
        std::snprintf(buf, len, "%s", g_err.c_str());
    }
    return (int)g_err.size();
}

int ocx_device_count(int* count) {
    if (!count) return fail(OCX_E_INVALID, "count is NULL");
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess) {
        *count = 0;
        return fail(OCX_E_HIP, std::string("hipGetDeviceCount: ") + hipGetErrorString(e));
    }
    *count = n;
    return OCX_OK;
}

int ocx_release_buffers(int device) {
    DevCtx* cx;
    if (int rc = ctx_enter(device, &cx)) return rc;
    std::lock_guard<std::mutex> lk(cx->mu);
    OCX_HIP(hipStreamSynchronize(cx->stream));
    for (DevBuf* b : {&cx->zraw, &cx->yraw, &cx->zt, &cx->yt, &cx->at, &cx->araw, &cx->cmp,
                      &cx->thr, &cx->out, &cx->sw, &cx->rstate, &cx->lstate, &cx->theta,
                      &cx->acc, &cx->gmax, &cx->yt2, &cx->gst, &cx->fst, &cx->bad})
        OCX_HIP(b->release());
    return OCX_OK;
}

int ocx_layout_init(int64_t B, int64_t T, int64_t d, int lanes_per_seq, ocx_layout* L) {
    if (!L) return fail(OCX_E_INVALID, "layout is NULL");
    if (B < 0 || T < 0 || d < 0) return fail(OCX_E_INVALID, "negative size");
    if (d > 4096) return fail(OCX_E_UNSUPPORTED, "d > 4096 not supported");
    // lanes_per_seq: 0 = auto (tree sums), k >= 2 = k lanes (tree sums),
    // 1 = exact with auto lanes, -k = exact with k lanes.  Exact mode keeps every sum
    // in the reference's sequential order; with P > 1 the running sum is handed from
    // lane to lane (chain = 1).
    // OCX_LANES_BEST: the exact-auto layout unless it chains 8+ lanes (d >= 512, or a
    // few-wave batch), then butterfly sums with at least 4 coordinates per lane: d = 64,
    // T = 1e5, 3328 sequences measured 69 ms at 16 x 4 (62 % of 8 TB/s) against 75 ms at
    // 8 x 8, 82 ms at 32 x 2 and 104 ms for the exact 8-lane chain; d = 1024: 52 ms
    // (81 %) against 102 ms exact (profiles/r02_fewwave_block_shapes.jsonl)
    // Since round 3 the pipelined butterfly kernel (ocx_alg_pipe.hip) also wins on the big
    // resident batches at 64 <= d <= 128 from 4096 sequences on: d = 64, 32 768 x 1e4, one
    // pass over z: 26.6 ms at 8 x 8 against 27.05 ms for the exact 4 x 16 chain, and the
    // generator writes whole 128-B lines of the 8 x 8 tile (59.5 vs 60.8 ms; WRITE_SIZE
    // 1.00002x vs 1.024x; profiles/r03_e2e_layout.jsonl, r03_traffic_gen_p8.json).
    bool best_tree = false;  // OCX_LANES_BEST fell back to butterfly sums
    if (lanes_per_seq == OCX_LANES_BEST) {
        ocx_layout Le;
        if (int rc = ocx_layout_init(B, T, d, 1, &Le)) return rc;
        if (Le.P < 8 && !(d >= 64 && d <= 128 && B >= 4096)) {
            *L = Le;
            return OCX_OK;
        }
        best_tree = true;
        lanes_per_seq = 0;
    }
    const bool exact = (lanes_per_seq == 1 || lanes_per_seq < 0);
    int P = lanes_per_seq < 0 ? -lanes_per_seq : lanes_per_seq;
    // auto: fewest lanes with <= 16 coordinates each (more coordinates per lane cost
    // registers, hence occupancy: d = 1024 measured 7.5e7 g(T) timesteps/s at 64 or 32
    // lanes and 4.7e7 at 16 x 64); most lanes keeping >= 2 coordinates
    int64_t p_min = 1;
    while (p_min < 64 && ceil_div(d, p_min) > 16) p_min *= 2;
    int64_t p_max = 1;
    const int64_t c_min = 2;  // fewest coordinates per lane
    while (p_max < 64 && ceil_div(d, p_max * 2) >= c_min) p_max *= 2;
    if (best_tree) {
        // OCX_LANES_BEST where exact chains would be latency-bound: butterfly lanes of 8
        // coordinates up to d = 128 from 4096 sequences on (their 8-step register ring;
        // d = 64, T = 1e5, 4900 sequences, one pass over z: 52 ms at 8 x 8 vs 59 at 16 x 4
        // and 71 at 4 x 16), 4 below (3328: 46 ms at 16 x 4 vs 52 at 8 x 8: twice the
        // waves), 32 from d = 512 (d = 1024, 3400 sequences: 44 ms at 32 x 32 vs 46 at
        // 64 x 16), 16 between (profiles/r02_fewwave_lanes_onepass.jsonl, r02_best2_probe.jsonl)
        const int64_t ct = d >= 512 ? 32 : (d <= 128 ? (B >= 4096 ? 8 : 4) : 16);
        int64_t p = 1;
        while (p < 64 && ceil_div(d, p) > ct) p *= 2;
        P = (int)p;
    } else if (lanes_per_seq == 0) {
        // auto: enough lanes for ~8 wavefronts per CU (131072 lanes on
        // 256 CUs) when B allows.
        int64_t p_lanes = 1;
        while (p_lanes < 64 && p_lanes * B < 131072) p_lanes *= 2;
        P = (int)std::max(p_min, std::min(p_lanes, p_max));
    } else if (lanes_per_seq == 1) {
        // exact auto: at most 16 coordinates per lane (register budget of the chained
        // sums; 32 from d = 512 on, where the chain's hop count costs more than the
        // registers: d = 1024 measured 1.6x faster at 32 lanes x 32 than 64 x 16), then
        // up to 4 lanes while that is needed to reach 65536 lanes.
        const int64_t cmax = d >= 512 ? 32 : 16;
        int64_t p = 1;
        while (p < 64 && ceil_div(d, p) > cmax) p *= 2;
        while (p < 4 && p * B < 65536 && ceil_div(d, 2 * p) >= 2) p *= 2;
        // few-wave batches (capacity-limited, e.g. the resident g(T) batch at T = 1e5) are
        // latency-bound: 8 lanes keeping >= 8 coordinates each (d = 64, T = 1e5, 3328
        // sequences measured 137 ms at 8 lanes, 172 ms at 4, 146 ms at 16)
        while (p < 8 && p * B < 32768 && ceil_div(d, 2 * p) >= 8) p *= 2;
        P = (int)p;
    }
    if (P < 1 || P > 64 || (P & (P - 1)) != 0)
        return fail(OCX_E_INVALID, "lanes_per_seq must be 0, 1, or +/- a power of two <= 64");
    const int chain = (exact && P > 1) ? 1 : 0;
    int C;
    const int64_t need = std::max<int64_t>(ceil_div(d, P), 1);
    if (need > 64)
        return fail(OCX_E_UNSUPPORTED,
                    "d / lanes_per_seq > 64 coordinates per lane; use more lanes");
    if (chain) {
        C = 2;
        while (C < need) C *= 2;
    } else {
        C = even_supported_C(need);
    }
    std::memset(L, 0, sizeof(*L));
    L->B = B;
    L->T = T;
    L->d = d;
    L->P = P;
    L->C = C;
    L->chain = chain;
    L->S = 64 / P;
    L->Dp = (int64_t)P * C;
    L->G = ceil_div(B, L->S);
    L->z_elems = L->G * T * 64 * (int64_t)C;
    L->y_elems = L->G * T * L->S;
    return OCX_OK;
}

// ---------------------------------------------------------------- device API
static int check_layout(const ocx_layout* L) {
    if (!L) return fail(OCX_E_INVALID, "layout is NULL");
    if (!ocx_supported_C(L->C) || L->P < 1 || L->P > 64 || L->S * L->P != 64)
        return fail(OCX_E_INVALID, "corrupt layout");
    if (L->chain && (L->C & (L->C - 1)) != 0)
        return fail(OCX_E_INVALID, "corrupt layout (chain needs a power-of-two C)");
    return OCX_OK;
}

int ocx_dev_pack(const ocx_layout* L, const double* z, const double* y, double* z_tiled,
                 double* y_tiled, void* stream) {
    StreamDevice sd_(stream);
    if (int rc = check_layout(L)) return rc;
    if (L->z_elems && (!z_tiled || (L->B * L->T * L->d > 0 && !z)))
        return fail(OCX_E_INVALID, "NULL z buffer");
    if (L->y_elems && (!y_tiled || !y)) return fail(OCX_E_INVALID, "NULL y buffer");
    OCX_HIP(ocx_launch_pack(L, z, y, z_tiled, y_tiled, (hipStream_t)stream));
    return OCX_OK;
}

int ocx_dev_gen_gT(const ocx_layout* L, uint64_t base_seed, int64_t run0, double* z_tiled,
                   double* y_tiled, void* stream) {
    StreamDevice sd_(stream);
    if (int rc = check_layout(L)) return rc;
    if (run0 < 0) return fail(OCX_E_INVALID, "run0 < 0");
    if (L->z_elems && (!z_tiled || !y_tiled)) return fail(OCX_E_INVALID, "NULL buffer");
    OCX_HIP(ocx_launch_gen_gT(L, base_seed, run0, z_tiled, y_tiled, (hipStream_t)stream));
    return OCX_OK;
}

int ocx_dev_gen_family(const ocx_layout* L, int family, const uint64_t* run_seeds,
                       const uint64_t* stream_ids, double p, int64_t block_len, double* z_tiled,
                       double* y_tiled, void* stream) {
    StreamDevice sd_(stream);
    if (int rc = check_layout(L)) return rc;
    if (family < 1 || family > 4) return fail(OCX_E_INVALID, "family must be 1..4");
    if (L->z_elems && (!z_tiled || !y_tiled)) return fail(OCX_E_INVALID, "NULL buffer");
    if ((family == 1 || family == 2) && L->B > 0 && (!run_seeds || !stream_ids))
        return fail(OCX_E_INVALID, "NULL seed arrays");
    if ((family == 1 || family == 2) && (int64_t)L->P * L->C > 64)
        return fail(OCX_E_UNSUPPORTED, "random families need a padded row <= 64 coordinates");
    if (family == 4 && block_len < 1) return fail(OCX_E_INVALID, "block_len < 1");
    OCX_HIP(ocx_launch_gen_family(L, family, run_seeds, stream_ids, p, block_len, z_tiled,
                                  y_tiled, (hipStream_t)stream));
    return OCX_OK;
}

int ocx_dev_simulate_alg(const ocx_layout* L, const double* z_tiled, const double* y_tiled,
                         int alg_flag, double eta0, const double* comparator, double* regret,
                         double* cum_loss, double* comp_loss, double* x_last, void* stream) {
    StreamDevice sd_(stream);
    if (int rc = check_layout(L)) return rc;
    if (L->z_elems && (!z_tiled || !y_tiled)) return fail(OCX_E_INVALID, "NULL input buffer");
    OCX_HIP(ocx_launch_alg(L, z_tiled, y_tiled, alg_flag != 0 ? 1 : 0, eta0, comparator, regret,
                           cum_loss, comp_loss, x_last, (hipStream_t)stream));
    return OCX_OK;
}

int ocx_dev_simulate_alg_ex(const ocx_layout* L, const double* z_tiled, const double* y_tiled,
                            int alg_flag, double eta0, const double* comparator, double* regret,
                            double* cum_loss, double* comp_loss, double* x_last, int flags,
                            int32_t* closed_out, void* stream) {
    StreamDevice sd_(stream);
    if (int rc = check_layout(L)) return rc;
    if (L->z_elems && (!z_tiled || !y_tiled)) return fail(OCX_E_INVALID, "NULL input buffer");
    if (flags & ~(OCX_ALG_CLIPPED_ROWS | OCX_ALG_CLOSED_COMPARATOR))
        return fail(OCX_E_INVALID, "unknown flags");
    // the two flags are one request: the kernel certifies every row and sub-gradient itself
    OCX_HIP(ocx_launch_alg(L, z_tiled, y_tiled, alg_flag != 0 ? 1 : 0, eta0, comparator, regret,
                           cum_loss, comp_loss, x_last, (hipStream_t)stream, nullptr, closed_out,
                           (flags & (OCX_ALG_CLIPPED_ROWS | OCX_ALG_CLOSED_COMPARATOR)) ? 1 : 0));
    return OCX_OK;
}

int ocx_dev_ftl_exact(const ocx_layout* L, const double* z_tiled, const double* y_tiled, int norm,
                      double* cum_loss, double* comp_loss, double* cmp_action, int32_t* regime,
                      void* stream) {
    StreamDevice sd_(stream);
    if (int rc = check_layout(L)) return rc;
    if (norm < 0 || norm > 2) return fail(OCX_E_INVALID, "norm must be 0 (l2), 1 (l1) or 2 (linf)");
    if (L->z_elems && (!z_tiled || !y_tiled)) return fail(OCX_E_INVALID, "NULL input buffer");
    if (L->B && !regime) return fail(OCX_E_INVALID, "regime output is required");
    OCX_HIP(ocx_launch_alg(L, z_tiled, y_tiled, 2, 0.0, nullptr, nullptr, cum_loss, comp_loss,
                           nullptr, (hipStream_t)stream, cmp_action, regime, 0, norm));
    return OCX_OK;
}

int ocx_dev_ftl_prefix_actions(const ocx_layout* L, const double* z_tiled,
                               const double* y_tiled, int norm, double* actions,
                               int32_t* regime, void* stream) {
    StreamDevice sd_(stream);
    if (int rc = check_layout(L)) return rc;
    if (norm < 0 || norm > 2) return fail(OCX_E_INVALID, "norm must be 0 (l2), 1 (l1) or 2 (linf)");
    if (L->z_elems && (!z_tiled || !y_tiled)) return fail(OCX_E_INVALID, "NULL input buffer");
    if (L->B && (!regime || (L->d > 0 && !actions)))
        return fail(OCX_E_INVALID, "NULL output buffer");
    OCX_HIP(ocx_launch_prefix_actions(L, z_tiled, y_tiled, actions, regime, (hipStream_t)stream,
                                      norm));
    return OCX_OK;
}

int ocx_dev_ftrl_vs_exact(const ocx_layout* L, const double* z_tiled, const double* y_tiled,
                          double eta0, double* cum_ftrl, double* cum_exact, double* comp_exact,
                          double* comp_ftl, double* cmp_action, int32_t* regime, void* stream) {
    StreamDevice sd_(stream);
    if (int rc = check_layout(L)) return rc;
    if (L->z_elems && (!z_tiled || !y_tiled)) return fail(OCX_E_INVALID, "NULL input buffer");
    if (L->B && (!cum_ftrl || !cum_exact || !comp_exact || !regime))
        return fail(OCX_E_INVALID, "NULL output buffer");
    OCX_HIP(ocx_launch_ftrl_exact(L, z_tiled, y_tiled, eta0, cum_ftrl, cum_exact, comp_exact,
                                  comp_ftl, cmp_action, regime, (hipStream_t)stream));
    return OCX_OK;
}

int ocx_dev_ftrl_vs_exact_ex(const ocx_layout* L, const double* z_tiled, const double* y_tiled,
                             double eta0, double* cum_ftrl, double* cum_exact, double* comp_exact,
                             double* comp_ftl, double* cmp_action, int32_t* regime, int norm,
                             int flags, void* stream) {
    StreamDevice sd_(stream);
    if (norm < 0 || norm > 2) return fail(OCX_E_INVALID, "norm must be 0 (l2), 1 (l1) or 2 (linf)");
    if (int rc = check_layout(L)) return rc;
    if (L->z_elems && (!z_tiled || !y_tiled)) return fail(OCX_E_INVALID, "NULL input buffer");
    if (L->B && (!cum_ftrl || !cum_exact || !comp_exact || !regime))
        return fail(OCX_E_INVALID, "NULL output buffer");
    if (flags & ~(OCX_ALG_CLIPPED_ROWS | OCX_ALG_CLOSED_COMPARATOR | OCX_ALG_TREE_SUMS))
        return fail(OCX_E_INVALID, "unknown flags");
    ocx_layout Lt = *L;
    if (flags & OCX_ALG_TREE_SUMS) Lt.chain = 0;  // same tiling, butterfly sums
    OCX_HIP(ocx_launch_ftrl_exact(&Lt, z_tiled, y_tiled, eta0, cum_ftrl, cum_exact, comp_exact,
                                  comp_ftl, cmp_action, regime, (hipStream_t)stream,
                                  (flags & (OCX_ALG_CLIPPED_ROWS | OCX_ALG_CLOSED_COMPARATOR)) ? 1
                                                                                             : 0,
                                  norm));
    return OCX_OK;
}

int ocx_dev_simulate_smart(const ocx_layout* L, const double* z_tiled, const double* y_tiled,
                           const double* thresh, double eta0, double* regret,
                           int64_t* switch_step, void* stream) {
    StreamDevice sd_(stream);
    if (int rc = check_layout(L)) return rc;
    if (L->B && (!thresh || !regret)) return fail(OCX_E_INVALID, "NULL thresh/regret");
    if (L->z_elems && (!z_tiled || !y_tiled)) return fail(OCX_E_INVALID, "NULL input buffer");
    OCX_HIP(ocx_launch_smart(L, z_tiled, y_tiled, thresh, eta0, regret, switch_step,
                             (hipStream_t)stream));
    return OCX_OK;
}

int ocx_dev_simulate_smart_ex(const ocx_layout* L, const double* z_tiled, const double* y_tiled,
                              const double* thresh, double eta0, double* regret,
                              int64_t* switch_step, int flags, unsigned long long* stats,
                              void* stream) {
    StreamDevice sd_(stream);
    if (int rc = check_layout(L)) return rc;
    if (L->B && (!thresh || !regret)) return fail(OCX_E_INVALID, "NULL thresh/regret");
    if (L->z_elems && (!z_tiled || !y_tiled)) return fail(OCX_E_INVALID, "NULL input buffer");
    if (flags & ~(OCX_SMART_CLOSED_PREFIX | OCX_ALG_CLOSED_COMPARATOR | OCX_ALG_CLIPPED_ROWS))
        return fail(OCX_E_INVALID, "unknown flags");
    const int prefix = (flags & OCX_SMART_CLOSED_PREFIX) ? 1 : 0;
    const int comp = (flags & (OCX_ALG_CLOSED_COMPARATOR | OCX_ALG_CLIPPED_ROWS)) ? 1 : 0;
    if (!prefix && !comp && !stats) {
        OCX_HIP(ocx_launch_smart(L, z_tiled, y_tiled, thresh, eta0, regret, switch_step,
                                 (hipStream_t)stream));
    } else {
        OCX_HIP(ocx_launch_smart_closed(L, z_tiled, y_tiled, thresh, eta0, regret, switch_step,
                                        prefix, comp, stats, (hipStream_t)stream));
    }
    return OCX_OK;
}

int ocx_dev_replay(const ocx_layout* L, const ocx_layout* La, const double* z_tiled,
                   const double* y_tiled, const double* a_tiled, double* cum_loss,
                   double* comp_loss, void* stream) {
    StreamDevice sd_(stream);
    if (int rc = check_layout(L)) return rc;
    if (int rc = check_layout(La)) return rc;
    if (La->T != L->T + 1 || La->B != L->B || La->P != L->P || La->C != L->C ||
        La->chain != L->chain)
        return fail(OCX_E_INVALID, "actions layout must match z layout with T+1 steps");
    if (L->B && (!a_tiled || !cum_loss || !comp_loss)) return fail(OCX_E_INVALID, "NULL buffer");
    OCX_HIP(ocx_launch_replay(L, z_tiled, y_tiled, a_tiled, cum_loss, comp_loss,
                              (hipStream_t)stream));
    return OCX_OK;
}

int ocx_dev_max_regret(const double* regrets, int64_t B, double* gmax, void* stream) {
    StreamDevice sd_(stream);
    if (!gmax || (B > 0 && !regrets)) return fail(OCX_E_INVALID, "NULL buffer");
    OCX_HIP(ocx_launch_max(regrets, B, gmax, (hipStream_t)stream));
    return OCX_OK;
}

}  // extern "C"

namespace {

// ocx_pipeline.hip's knob (tuning; the default is the measured best): generator waves per
// SIMD beside the FTRL kernel
int pipe_wps() {
    // 4: four generator waves per SIMD in the 96-VGPR form beside one 128-VGPR FTRL wave;
    // 32 768 x 1e4 x 64 with two streams per side measured 64.3-66.9 ms per batch, vs
    // 69.6-72.9 at 3 waves of the 128-VGPR form and 69.9-73.0 with a 168-VGPR FTRL form beside
    // 3 (profiles/r04_overlap3.jsonl, r04_overlap4.jsonl)
    const char* e = std::getenv("OCX_PIPE_WPS");
    const int v = e ? std::atoi(e) : 4;
    return v >= 1 && v <= 8 ? v : 4;
}
}  // namespace

extern "C" {

int ocx_dev_gen_simulate(const ocx_layout* L, uint64_t base_seed, int64_t run0, int64_t nbatch,
                         double* z_tiled, double* y_tiled, double eta0, double* regret,
                         double* gmax, uint32_t flags, int64_t sub_seqs, void* stream) {
    StreamDevice sd_(stream);
    if (int rc = check_layout(L)) return rc;
    if (run0 < 0 || nbatch < 0) return fail(OCX_E_INVALID, "negative run0 / nbatch");
    if (flags & ~(OCX_GENSIM_SEQUENTIAL | OCX_GENSIM_TWO_PASS))
        return fail(OCX_E_INVALID, "unknown flags");
    if (L->B > 0 && !regret) return fail(OCX_E_INVALID, "NULL regret");
    if (L->z_elems && (!z_tiled || !y_tiled)) return fail(OCX_E_INVALID, "NULL buffer");
    const hipStream_t st = (hipStream_t)stream;
    unsigned long long* acc = reinterpret_cast<unsigned long long*>(gmax);
    if (acc) OCX_HIP(launch_zero_u64(acc, st));  // +0.0
    if (nbatch == 0 || L->B == 0 || L->T == 0) return OCX_OK;
    // the sampler's rows are clipped (by construction: no per-row check, ocx_check_rows): the
    // closed-form comparator unless the caller asks for the reference's streamed pass (the
    // bit-exact modes)
    const int onepass = (flags & OCX_GENSIM_TWO_PASS) ? 0 : 2;
    if (!(flags & OCX_GENSIM_SEQUENTIAL) && ocx_pipeline_supported(L) && ocx_stream_fork_ok(st) &&
        (sub_seqs > 0 || ocx_pipeline_worth(L, pipe_wps()))) {
        OCX_HIP(ocx_run_gen_sim_pipelined(L, base_seed, run0, nbatch, z_tiled, y_tiled, eta0,
                                          regret, onepass, acc,
                                          pipe_wps(), sub_seqs, st));
        return OCX_OK;
    }
    for (int64_t k = 0; k < nbatch; ++k) {
        OCX_HIP(ocx_launch_gen_gT(L, base_seed, run0 + k * L->B, z_tiled, y_tiled, st));
        OCX_HIP(ocx_launch_alg(L, z_tiled, y_tiled, 0, eta0, nullptr, regret, nullptr, nullptr,
                               nullptr, st, nullptr, nullptr, onepass));
        if (acc) OCX_HIP(launch_max_fold(regret, L->B, acc, st));
    }
    return OCX_OK;
}

// ---------------------------------------------------------------- host API
int ocx_simulate_alg_batch(const double* z, const double* y, int64_t B, int64_t T, int64_t d,
                           int alg_flag, double eta0, const double* comparator, double* regret,
                           double* cum_loss, double* comp_loss, double* x_last,
                           int lanes_per_seq, int device) {
    ocx_layout L;
    if (int rc = ocx_layout_init(B, T, d, lanes_per_seq, &L)) return rc;
    if (B == 0) return OCX_OK;
    if ((T * d > 0 && !z) || (T > 0 && !y)) return fail(OCX_E_INVALID, "NULL z/y");
    DevCtx* cx;
    if (int rc = ctx_enter(device, &cx)) return rc;
    std::lock_guard<std::mutex> lk(cx->mu);
    hipStream_t st = cx->stream;
    const size_t nz = (size_t)(B * T * d), ny = (size_t)(B * T);
    OCX_HIP(cx->zraw.ensure(nz * 8));
    OCX_HIP(cx->yraw.ensure(ny * 8));
    OCX_HIP(cx->zt.ensure((size_t)L.z_elems * 8));
    OCX_HIP(cx->yt.ensure((size_t)L.y_elems * 8));
    OCX_HIP(cx->out.ensure((size_t)B * (3 + d) * 8));
    if (nz) OCX_HIP(hipMemcpyAsync(cx->zraw.p, z, nz * 8, hipMemcpyHostToDevice, st));
    if (ny) OCX_HIP(hipMemcpyAsync(cx->yraw.p, y, ny * 8, hipMemcpyHostToDevice, st));
    const double* dcmp = nullptr;
    if (comparator) {
        OCX_HIP(cx->cmp.ensure((size_t)B * d * 8 + 8));
        if (B * d)
            OCX_HIP(hipMemcpyAsync(cx->cmp.p, comparator, (size_t)B * d * 8,
                                   hipMemcpyHostToDevice, st));
        dcmp = cx->cmp.as<double>();
    }
    OCX_HIP(ocx_launch_pack(&L, cx->zraw.as<double>(), cx->yraw.as<double>(), cx->zt.as<double>(),
                            cx->yt.as<double>(), st));
    double* o = cx->out.as<double>();
    double* dxl = x_last ? o + 3 * B : nullptr;
    if (dxl && B * d) OCX_HIP(hipMemsetAsync(dxl, 0, (size_t)B * d * 8, st));
    OCX_HIP(ocx_launch_alg(&L, cx->zt.as<double>(), cx->yt.as<double>(), alg_flag != 0 ? 1 : 0,
                           eta0, dcmp, o, o + B, o + 2 * B, dxl, st));
    std::vector<double> h((size_t)B * (3 + (x_last ? d : 0)));
    OCX_HIP(hipMemcpyAsync(h.data(), o, h.size() * 8, hipMemcpyDeviceToHost, st));
    OCX_HIP(hipStreamSynchronize(st));
    if (regret) std::memcpy(regret, h.data(), B * 8);
    if (cum_loss) std::memcpy(cum_loss, h.data() + B, B * 8);
    if (comp_loss) std::memcpy(comp_loss, h.data() + 2 * B, B * 8);
    if (x_last && d) std::memcpy(x_last, h.data() + 3 * B, (size_t)B * d * 8);
    return OCX_OK;
}

int ocx_simulate_smart_batch(const double* z, const double* y, int64_t B, int64_t T, int64_t d,
                             const double* thresh, double eta0, double* regret,
                             int64_t* switch_step, int lanes_per_seq, int device) {
    ocx_layout L;
    if (int rc = ocx_layout_init(B, T, d, lanes_per_seq, &L)) return rc;
    if (B == 0) return OCX_OK;
    if ((T * d > 0 && !z) || (T > 0 && !y) || !thresh || !regret)
        return fail(OCX_E_INVALID, "NULL argument");
    DevCtx* cx;
    if (int rc = ctx_enter(device, &cx)) return rc;
    std::lock_guard<std::mutex> lk(cx->mu);
    hipStream_t st = cx->stream;
    const size_t nz = (size_t)(B * T * d), ny = (size_t)(B * T);
    OCX_HIP(cx->zraw.ensure(nz * 8));
    OCX_HIP(cx->yraw.ensure(ny * 8));
    OCX_HIP(cx->zt.ensure((size_t)L.z_elems * 8));
    OCX_HIP(cx->yt.ensure((size_t)L.y_elems * 8));
    OCX_HIP(cx->thr.ensure((size_t)B * 8));
    OCX_HIP(cx->out.ensure((size_t)B * 8));
    OCX_HIP(cx->sw.ensure((size_t)B * 8));
    if (nz) OCX_HIP(hipMemcpyAsync(cx->zraw.p, z, nz * 8, hipMemcpyHostToDevice, st));
    if (ny) OCX_HIP(hipMemcpyAsync(cx->yraw.p, y, ny * 8, hipMemcpyHostToDevice, st));
    OCX_HIP(hipMemcpyAsync(cx->thr.p, thresh, (size_t)B * 8, hipMemcpyHostToDevice, st));
    OCX_HIP(ocx_launch_pack(&L, cx->zraw.as<double>(), cx->yraw.as<double>(), cx->zt.as<double>(),
                            cx->yt.as<double>(), st));
    if (lanes_per_seq == 1 || lanes_per_seq < 0) {
        // bit-exact modes: the reference's prefix re-scan and streamed comparator
        OCX_HIP(ocx_launch_smart(&L, cx->zt.as<double>(), cx->yt.as<double>(),
                                 cx->thr.as<double>(), eta0, cx->out.as<double>(),
                                 cx->sw.as<int64_t>(), st));
    } else {
        // O(T·d): guarded closed-form prefix, certified closed-form comparator
        OCX_HIP(ocx_launch_smart_closed(&L, cx->zt.as<double>(), cx->yt.as<double>(),
                                        cx->thr.as<double>(), eta0, cx->out.as<double>(),
                                        cx->sw.as<int64_t>(), 1, 1, nullptr, st));
    }
    OCX_HIP(hipMemcpyAsync(regret, cx->out.p, (size_t)B * 8, hipMemcpyDeviceToHost, st));
    if (switch_step)
        OCX_HIP(hipMemcpyAsync(switch_step, cx->sw.p, (size_t)B * 8, hipMemcpyDeviceToHost, st));
    OCX_HIP(hipStreamSynchronize(st));
    return OCX_OK;
}

int ocx_ftl_exact_batch(const double* z, const double* y, int64_t B, int64_t T, int64_t d,
                        int norm, double* cum_loss, double* comp_loss, double* cmp_action,
                        int32_t* regime, int lanes_per_seq, int device) {
    ocx_layout L;
    if (int rc = ocx_layout_init(B, T, d, lanes_per_seq, &L)) return rc;
    if (norm < 0 || norm > 2) return fail(OCX_E_INVALID, "norm must be 0 (l2), 1 (l1) or 2 (linf)");
    if (B == 0) return OCX_OK;
    if ((T * d > 0 && !z) || (T > 0 && !y) || !regime) return fail(OCX_E_INVALID, "NULL argument");
    DevCtx* cx;
    if (int rc = ctx_enter(device, &cx)) return rc;
    std::lock_guard<std::mutex> lk(cx->mu);
    hipStream_t st = cx->stream;
    const size_t nz = (size_t)(B * T * d), ny = (size_t)(B * T);
    OCX_HIP(cx->zraw.ensure(nz * 8));
    OCX_HIP(cx->yraw.ensure(ny * 8));
    OCX_HIP(cx->zt.ensure((size_t)L.z_elems * 8));
    OCX_HIP(cx->yt.ensure((size_t)L.y_elems * 8));
    OCX_HIP(cx->out.ensure((size_t)B * (2 + d) * 8 + (size_t)B * 4));
    if (nz) OCX_HIP(hipMemcpyAsync(cx->zraw.p, z, nz * 8, hipMemcpyHostToDevice, st));
    if (ny) OCX_HIP(hipMemcpyAsync(cx->yraw.p, y, ny * 8, hipMemcpyHostToDevice, st));
    OCX_HIP(ocx_launch_pack(&L, cx->zraw.as<double>(), cx->yraw.as<double>(), cx->zt.as<double>(),
                            cx->yt.as<double>(), st));
    double* o = cx->out.as<double>();
    int* rg = reinterpret_cast<int*>(o + B * (2 + d));
    OCX_HIP(ocx_launch_alg(&L, cx->zt.as<double>(), cx->yt.as<double>(), 2, 0.0, nullptr, nullptr,
                           o, o + B, nullptr, st, o + 2 * B, rg, 0, norm));
    std::vector<double> h((size_t)B * (2 + d));
    OCX_HIP(hipMemcpyAsync(h.data(), o, h.size() * 8, hipMemcpyDeviceToHost, st));
    OCX_HIP(hipMemcpyAsync(regime, rg, (size_t)B * 4, hipMemcpyDeviceToHost, st));
    OCX_HIP(hipStreamSynchronize(st));
    if (cum_loss) std::memcpy(cum_loss, h.data(), B * 8);
    if (comp_loss) std::memcpy(comp_loss, h.data() + B, B * 8);
    if (cmp_action && d) std::memcpy(cmp_action, h.data() + 2 * B, (size_t)B * d * 8);
    return OCX_OK;
}

int ocx_ftl_prefix_actions_batch(const double* z, const double* y, int64_t B, int64_t T,
                                 int64_t d, int norm, double* actions, int32_t* regime,
                                 int lanes_per_seq, int device) {
    ocx_layout L;
    if (int rc = ocx_layout_init(B, T, d, lanes_per_seq, &L)) return rc;
    if (norm < 0 || norm > 2) return fail(OCX_E_INVALID, "norm must be 0 (l2), 1 (l1) or 2 (linf)");
    if (B == 0) return OCX_OK;
    if ((T * d > 0 && !z) || (T > 0 && !y) || !regime || (d > 0 && !actions))
        return fail(OCX_E_INVALID, "NULL argument");
    DevCtx* cx;
    if (int rc = ctx_enter(device, &cx)) return rc;
    std::lock_guard<std::mutex> lk(cx->mu);
    hipStream_t st = cx->stream;
    const size_t nz = (size_t)(B * T * d), ny = (size_t)(B * T), na = (size_t)(B * (T + 1) * d);
    OCX_HIP(cx->zraw.ensure(nz * 8));
    OCX_HIP(cx->yraw.ensure(ny * 8));
    OCX_HIP(cx->zt.ensure((size_t)L.z_elems * 8));
    OCX_HIP(cx->yt.ensure((size_t)L.y_elems * 8));
    OCX_HIP(cx->araw.ensure(na * 8));
    OCX_HIP(cx->out.ensure((size_t)B * 4));
    if (nz) OCX_HIP(hipMemcpyAsync(cx->zraw.p, z, nz * 8, hipMemcpyHostToDevice, st));
    if (ny) OCX_HIP(hipMemcpyAsync(cx->yraw.p, y, ny * 8, hipMemcpyHostToDevice, st));
    OCX_HIP(ocx_launch_pack(&L, cx->zraw.as<double>(), cx->yraw.as<double>(), cx->zt.as<double>(),
                            cx->yt.as<double>(), st));
    int* rg = cx->out.as<int>();
    OCX_HIP(ocx_launch_prefix_actions(&L, cx->zt.as<double>(), cx->yt.as<double>(),
                                      cx->araw.as<double>(), rg, st, norm));
    if (na) OCX_HIP(hipMemcpyAsync(actions, cx->araw.p, na * 8, hipMemcpyDeviceToHost, st));
    OCX_HIP(hipMemcpyAsync(regime, rg, (size_t)B * 4, hipMemcpyDeviceToHost, st));
    OCX_HIP(hipStreamSynchronize(st));
    return OCX_OK;
}

int ocx_ftrl_vs_exact_batch(const double* z, const double* y, int64_t B, int64_t T, int64_t d,
                            double eta0, double* cum_ftrl, double* cum_exact, double* comp_exact,
                            double* comp_ftl, double* cmp_action, int32_t* regime,
                            int lanes_per_seq, int device) {
    return ocx_ftrl_vs_exact_batch_ex(z, y, B, T, d, eta0, cum_ftrl, cum_exact, comp_exact,
                                      comp_ftl, cmp_action, regime, 0, lanes_per_seq, device);
}

int ocx_ftrl_vs_exact_batch_ex(const double* z, const double* y, int64_t B, int64_t T, int64_t d,
                               double eta0, double* cum_ftrl, double* cum_exact,
                               double* comp_exact, double* comp_ftl, double* cmp_action,
                               int32_t* regime, int norm, int lanes_per_seq, int device) {
    ocx_layout L;
    if (int rc = ocx_layout_init(B, T, d, lanes_per_seq, &L)) return rc;
    if (norm < 0 || norm > 2) return fail(OCX_E_INVALID, "norm must be 0 (l2), 1 (l1) or 2 (linf)");
    if (B == 0) return OCX_OK;
    if ((T * d > 0 && !z) || (T > 0 && !y) || !cum_ftrl || !cum_exact || !comp_exact || !regime)
        return fail(OCX_E_INVALID, "NULL argument");
    DevCtx* cx;
    if (int rc = ctx_enter(device, &cx)) return rc;
    std::lock_guard<std::mutex> lk(cx->mu);
    hipStream_t st = cx->stream;
    const size_t nz = (size_t)(B * T * d), ny = (size_t)(B * T);
    OCX_HIP(cx->zraw.ensure(nz * 8));
    OCX_HIP(cx->yraw.ensure(ny * 8));
    OCX_HIP(cx->zt.ensure((size_t)L.z_elems * 8));
    OCX_HIP(cx->yt.ensure((size_t)L.y_elems * 8));
    OCX_HIP(cx->out.ensure((size_t)B * (4 + d) * 8 + (size_t)B * 4));
    if (nz) OCX_HIP(hipMemcpyAsync(cx->zraw.p, z, nz * 8, hipMemcpyHostToDevice, st));
    if (ny) OCX_HIP(hipMemcpyAsync(cx->yraw.p, y, ny * 8, hipMemcpyHostToDevice, st));
    OCX_HIP(ocx_launch_pack(&L, cx->zraw.as<double>(), cx->yraw.as<double>(), cx->zt.as<double>(),
                            cx->yt.as<double>(), st));
    double* o = cx->out.as<double>();
    int* rg = reinterpret_cast<int*>(o + B * (4 + d));
    // outside the bit-exact modes the comparator losses take their closed form where the
    // kernel certifies the regime, and OCX_LANES_BEST sums with the butterfly
    // (ocx_dev_ftrl_vs_exact_ex, OCX_ALG_TREE_SUMS)
    const int onepass = (lanes_per_seq == 1 || lanes_per_seq < 0) ? 0 : 1;
    if (lanes_per_seq == OCX_LANES_BEST) L.chain = 0;
    OCX_HIP(ocx_launch_ftrl_exact(&L, cx->zt.as<double>(), cx->yt.as<double>(), eta0, o, o + B,
                                  o + 2 * B, comp_ftl ? o + 3 * B : nullptr, o + 4 * B, rg, st,
                                  onepass, norm));
    std::vector<double> h((size_t)B * (4 + d));
    OCX_HIP(hipMemcpyAsync(h.data(), o, h.size() * 8, hipMemcpyDeviceToHost, st));
    OCX_HIP(hipMemcpyAsync(regime, rg, (size_t)B * 4, hipMemcpyDeviceToHost, st));
    OCX_HIP(hipStreamSynchronize(st));
    std::memcpy(cum_ftrl, h.data(), B * 8);
    std::memcpy(cum_exact, h.data() + B, B * 8);
    std::memcpy(comp_exact, h.data() + 2 * B, B * 8);
    if (comp_ftl) std::memcpy(comp_ftl, h.data() + 3 * B, B * 8);
    if (cmp_action && d) std::memcpy(cmp_action, h.data() + 4 * B, (size_t)B * d * 8);
    return OCX_OK;
}

int ocx_replay_batch(const double* z, const double* y, const double* actions, int64_t B,
                     int64_t T, int64_t d, double* cum_loss, double* comp_loss, int device) {
    ocx_layout L, La;
    if (int rc = ocx_layout_init(B, T, d, 1, &L)) return rc;
    if (int rc = ocx_layout_init(B, T + 1, d, 1, &La)) return rc;
    if (B == 0) return OCX_OK;
    if ((T * d > 0 && !z) || (T > 0 && !y) || (d > 0 && !actions) || !cum_loss || !comp_loss)
        return fail(OCX_E_INVALID, "NULL argument");
    DevCtx* cx;
    if (int rc = ctx_enter(device, &cx)) return rc;
    std::lock_guard<std::mutex> lk(cx->mu);
    hipStream_t st = cx->stream;
    const size_t nz = (size_t)(B * T * d), ny = (size_t)(B * T), na = (size_t)(B * (T + 1) * d);
    OCX_HIP(cx->zraw.ensure(nz * 8));
    OCX_HIP(cx->yraw.ensure(ny * 8));
    OCX_HIP(cx->araw.ensure(na * 8));
    OCX_HIP(cx->zt.ensure((size_t)L.z_elems * 8));
    OCX_HIP(cx->yt.ensure((size_t)L.y_elems * 8));
    OCX_HIP(cx->at.ensure((size_t)La.z_elems * 8));
    OCX_HIP(cx->out.ensure((size_t)B * 2 * 8));
    if (nz) OCX_HIP(hipMemcpyAsync(cx->zraw.p, z, nz * 8, hipMemcpyHostToDevice, st));
    if (ny) OCX_HIP(hipMemcpyAsync(cx->yraw.p, y, ny * 8, hipMemcpyHostToDevice, st));
    if (na) OCX_HIP(hipMemcpyAsync(cx->araw.p, actions, na * 8, hipMemcpyHostToDevice, st));
    OCX_HIP(ocx_launch_pack(&L, cx->zraw.as<double>(), cx->yraw.as<double>(), cx->zt.as<double>(),
                            cx->yt.as<double>(), st));
    // actions are tiled like z with T+1 steps (no label part)
    ocx_layout Lz = La;
    Lz.y_elems = 0;
    OCX_HIP(ocx_launch_pack(&Lz, cx->araw.as<double>(), nullptr, cx->at.as<double>(), nullptr, st));
    double* o = cx->out.as<double>();
    OCX_HIP(ocx_launch_replay(&L, cx->zt.as<double>(), cx->yt.as<double>(), cx->at.as<double>(), o,
                              o + B, st));
    OCX_HIP(hipMemcpyAsync(cum_loss, o, (size_t)B * 8, hipMemcpyDeviceToHost, st));
    OCX_HIP(hipMemcpyAsync(comp_loss, o + B, (size_t)B * 8, hipMemcpyDeviceToHost, st));
    OCX_HIP(hipStreamSynchronize(st));
    return OCX_OK;
}

int ocx_dev_exact_ball_solve(const double* z, const double* y, int64_t B, int64_t T, int64_t d,
                             int norm, int all_prefixes, double* actions, double* obj, double* gap,
                             double* step_loss, int32_t* info, void* stream) {
    StreamDevice sd_(stream);
    if (B < 0 || T < 0 || d < 1) return fail(OCX_E_INVALID, "need B >= 0, T >= 0, d >= 1");
    if (d > OCX_EXACT_BALL_MAX_D)
        return fail(OCX_E_UNSUPPORTED, "the general exact-FTL solver takes d <= " +
                                           std::to_string(OCX_EXACT_BALL_MAX_D));
    if (norm < 0 || norm > 2) return fail(OCX_E_INVALID, "norm must be 0 (l2), 1 (l1) or 2 (linf)");
    if (B == 0) return OCX_OK;
    if ((T > 0 && (!z || !y)) || !actions) return fail(OCX_E_INVALID, "NULL argument");
    OCX_HIP(ocx_launch_exact_ball(z, y, B, T, d, norm, all_prefixes, actions, obj, gap, step_loss,
                                  info, (hipStream_t)stream));
    return OCX_OK;
}

int ocx_dev_exact_ball_solve_tiled(const ocx_layout* L, const double* z_tiled,
                                   const double* y_tiled, int norm, int all_prefixes,
                                   double* actions, double* obj, double* gap, double* step_loss,
                                   int32_t* info, void* stream) {
    StreamDevice sd_(stream);
    if (int rc = check_layout(L)) return rc;
    if (L->d < 1) return fail(OCX_E_INVALID, "need d >= 1");
    if (L->d > OCX_EXACT_BALL_MAX_D)
        return fail(OCX_E_UNSUPPORTED, "the general exact-FTL solver takes d <= " +
                                           std::to_string(OCX_EXACT_BALL_MAX_D));
    if (norm < 0 || norm > 2) return fail(OCX_E_INVALID, "norm must be 0 (l2), 1 (l1) or 2 (linf)");
    if (L->B == 0) return OCX_OK;
    if ((L->z_elems && (!z_tiled || !y_tiled)) || !actions) return fail(OCX_E_INVALID, "NULL argument");
    OCX_HIP(ocx_launch_exact_ball_tiled(L, z_tiled, y_tiled, norm, all_prefixes, actions, obj, gap,
                                        step_loss, info, (hipStream_t)stream));
    return OCX_OK;
}

int ocx_exact_ball_solve(const double* z, const double* y, int64_t B, int64_t T, int64_t d,
                         int norm, int all_prefixes, double* actions, double* obj, double* gap,
                         double* step_loss, int32_t* info, int device) {
    if (B < 0 || T < 0 || d < 1) return fail(OCX_E_INVALID, "need B >= 0, T >= 0, d >= 1");
    if (d > OCX_EXACT_BALL_MAX_D)
        return fail(OCX_E_UNSUPPORTED, "the general exact-FTL solver takes d <= " +
                                           std::to_string(OCX_EXACT_BALL_MAX_D));
    if (norm < 0 || norm > 2) return fail(OCX_E_INVALID, "norm must be 0 (l2), 1 (l1) or 2 (linf)");
    if (B == 0) return OCX_OK;
    if ((T > 0 && (!z || !y)) || !actions) return fail(OCX_E_INVALID, "NULL argument");
    DevCtx* cx;
    if (int rc = ctx_enter(device, &cx)) return rc;
    std::lock_guard<std::mutex> lk(cx->mu);
    hipStream_t st = cx->stream;
    const int64_t NP = all_prefixes ? T + 1 : 1;
    const size_t nz = (size_t)(B * T * d), ny = (size_t)(B * T), na = (size_t)(B * NP * d);
    const size_t np = (size_t)(B * NP);
    OCX_HIP(cx->zraw.ensure(nz * 8));
    OCX_HIP(cx->yraw.ensure(ny * 8));
    OCX_HIP(cx->araw.ensure(na * 8));
    OCX_HIP(cx->out.ensure(np * 28));
    if (nz) OCX_HIP(hipMemcpyAsync(cx->zraw.p, z, nz * 8, hipMemcpyHostToDevice, st));
    if (ny) OCX_HIP(hipMemcpyAsync(cx->yraw.p, y, ny * 8, hipMemcpyHostToDevice, st));
    double* o = cx->out.as<double>();
    int32_t* inf = reinterpret_cast<int32_t*>(o + 3 * np);
    OCX_HIP(ocx_launch_exact_ball(cx->zraw.as<double>(), cx->yraw.as<double>(), B, T, d, norm,
                                  all_prefixes, cx->araw.as<double>(), o, o + np, o + 2 * np, inf,
                                  st));
    OCX_HIP(hipMemcpyAsync(actions, cx->araw.p, na * 8, hipMemcpyDeviceToHost, st));
    if (obj) OCX_HIP(hipMemcpyAsync(obj, o, np * 8, hipMemcpyDeviceToHost, st));
    if (gap) OCX_HIP(hipMemcpyAsync(gap, o + np, np * 8, hipMemcpyDeviceToHost, st));
    if (step_loss)
        OCX_HIP(hipMemcpyAsync(step_loss, o + 2 * np, np * 8, hipMemcpyDeviceToHost, st));
    if (info) OCX_HIP(hipMemcpyAsync(info, inf, np * 4, hipMemcpyDeviceToHost, st));
    OCX_HIP(hipStreamSynchronize(st));
    return OCX_OK;
}

}  // extern "C"

namespace {

// fast_algorithms.py:230-243 for one T: the regrets of runs [run0, run0 + R) to the host
// (`regrets`), or only their max (`gmax`: the regrets never leave the GPU).
// test_unclean_every (ocx_test_gT_regrets_unclean only, 0 elsewhere): on the streamed path,
// mark every k-th run as failing the closed form's check, so the fallback pass is exercised;
// on the trailing path, run every k-th batch again whole, as a NaN-flagged batch is.
// regrets_on_device: `regrets` is device memory of `device` (ocx_gT_regrets_dev): the FTRL
// kernel writes each batch's regrets straight into it and nothing crosses PCIe.
int gT_run(uint64_t base_seed, int64_t T, int64_t run0, int64_t R, int64_t d, double eta0,
           double* regrets, double* gmax, int lanes_per_seq, int device,
           int64_t test_unclean_every = 0, bool regrets_on_device = false) {
    if (R < 0 || run0 < 0 || T < 0 || d < 0) return fail(OCX_E_INVALID, "negative argument");
    if (gmax) *gmax = 0.0;
    if (R == 0) return OCX_OK;
    if (!regrets && !gmax) return fail(OCX_E_INVALID, "NULL regrets");
    // the sampler's rows are clipped (by construction: no per-row check, ocx_check_rows):
    // outside the bit-exact modes the comparator loss takes the closed form
    // (ocx_dev_simulate_alg_ex), one HBM pass instead of two
    const int onepass = (lanes_per_seq == 1 || lanes_per_seq < 0) ? 0 : 2;
    // These batches are generated on device, and for 8 <= d < 64 the exact layout's one or
    // two lanes per sequence leave each generator wave (one stream) writing 16- or 32-B
    // pieces of a row into C/2 planes of the tile.  OCX_LANES_BEST takes butterfly lanes of
    // two coordinates here, up to 8 lanes (128-B row pieces): 65 536 x 1e3, generation +
    // FTRL: d = 16 27.6 -> 7.5 ms, d = 32 21.7 -> 12.7, d = 8 14.1 -> 4.8, d = 5 (two
    // lanes) 10.6 -> 7.9 (the FTRL kernel alone 1.36 -> 1.60 ms at d = 16;
    // profiles/r03_config1_layouts.jsonl, r03_gt_small_d.jsonl).
    if (lanes_per_seq == OCX_LANES_BEST && d >= 4 && d < 64) lanes_per_seq = d >= 16 ? 8 : (d >= 8 ? 4 : 2);
    DevCtx* cx;
    if (int rc = ctx_enter(device, &cx)) return rc;
    std::lock_guard<std::mutex> lk(cx->mu);
    hipStream_t st = cx->stream;
    unsigned long long* dmax = nullptr;
    if (!regrets) {
        OCX_HIP(cx->gmax.ensure(8));
        dmax = cx->gmax.as<unsigned long long>();
        OCX_HIP(hipMemsetAsync(dmax, 0, 8, st));  // +0.0
    }
    // the max leaves the GPU once, after the last batch; device-resident regrets are
    // complete when the call returns (any stream may read them then)
    auto finish = [&]() -> int {
        if (dmax) OCX_HIP(hipMemcpyAsync(gmax, dmax, 8, hipMemcpyDeviceToHost, st));
        if (dmax || regrets_on_device) OCX_HIP(hipStreamSynchronize(st));
        return OCX_OK;
    };
    // HBM budget for the z/y tiles of one batch (OCX_HBM_BUDGET_GB): by default 90 % of
    // what is free plus what this context already holds, at most 240 GiB.  d = 64, T = 1e5
    // measured 1.62e9 timesteps/s at 192 GiB and 1.91e9 at 240 GiB (round 1, FTRL-bound);
    // since round 3 the generator (VALU-bound: its time grows with the streams) dominates
    // those batches, and 272 GiB measured no faster at T = 1e5 (3.82 vs 3.80 s) and 4 %
    // slower for configs[4] (d = 1024 batches of 3 277 put four generator waves on some
    // SIMDs where 2 979 put three; profiles/r03_sweep_budget272.jsonl).
    int64_t budget;
    if (const char* e = std::getenv("OCX_HBM_BUDGET_GB")) {
        budget = (int64_t)(std::atof(e) * (1 << 30));
    } else {
        size_t fr = 0, tot = 0;
        OCX_HIP(hipMemGetInfo(&fr, &tot));
        const double avail = (double)fr + (double)cx->zt.cap + (double)cx->yt.cap;
        budget = std::min<int64_t>((int64_t)240 << 30, (int64_t)(0.9 * avail));
    }
    const int64_t kBatch = 131072;   // streams per batch of the streamed path
    // Resident batches (one generation pass) win over the streamed path (seek + two
    // generation passes) from ~1024 sequences per batch on (OCX_MIN_RESIDENT): d = 1024,
    // T = 1e4 measured 1.1e8 timesteps/s resident at 2600 per batch vs 7.5e7 streamed;
    // d = 64, T = 1e5: 1.37e9 resident at 4100 per batch vs 1.13e9 streamed.
    int64_t kMinResident = 1024;
    if (const char* e = std::getenv("OCX_MIN_RESIDENT")) kMinResident = std::max<int64_t>(1, std::atoll(e));
    ocx_layout L1;
    if (int rc = ocx_layout_init(std::min<int64_t>(R, kBatch), std::max<int64_t>(T, 1), d,
                                 lanes_per_seq, &L1))
        return rc;
    const int64_t step_bytes = (L1.z_elems + L1.y_elems) * 8 / std::max<int64_t>(T, 1);
    // whole horizon of one sequence, resident
    const int64_t per_seq = std::max<int64_t>(step_bytes * T / std::max<int64_t>(L1.B, 1), 8);
    // Resident batches (generate once, simulate once) while a batch still holds enough
    // sequences; otherwise stream the horizon (seek + two generation passes).
    const bool streamed = budget / per_seq < std::min<int64_t>(R, kMinResident);
    if (!streamed) {
        // whole horizon resident: as many runs per batch as the budget holds
        int64_t chunk = std::max<int64_t>(64, std::min<int64_t>(budget / per_seq, R));
        int64_t nbat = (R + chunk - 1) / chunk;
        chunk = (R + nbat - 1) / nbat;  // equal batches: no small, under-filled last one
        {
            // A batch of between one and two rounds of resident FTRL waves (one wave per
            // SIMD at C >= 16) would run its second round nearly empty: cut it to one
            // round (d = 1024: 2731 sequences per batch measured 11 % slower overall
            // than 2048).
            int dev = 0, cus = 256;
            OCX_HIP(hipGetDevice(&dev));
            OCX_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
            const int64_t wmax = (int64_t)cus * 4;
            ocx_layout Lc;
            if (int rc = ocx_layout_init(chunk, T, d, lanes_per_seq, &Lc)) return rc;
            // (two-pass only: with the closed-form comparator the generator's throughput,
            // which grows with the streams per batch, dominates: d = 1024, T = 1e4
            // measured 1.68e8 timesteps/s at 3400 per batch vs 1.50e8 at 2048)
            if (!onepass && Lc.G > wmax && Lc.G < 2 * wmax && Lc.C >= 16) {
                chunk = wmax * Lc.S;
                nbat = (R + chunk - 1) / chunk;
                chunk = (R + nbat - 1) / nbat;
            }
            // Whole generator rounds: with many streams per generator wave (a batch over
            // twice the generator's resident waves, 16 per CU) the streams of a batch
            // spread as ceil(batch / waves) per wave, and the part of the last round left
            // empty is lost.  One batch more is taken when it wastes less (by more than
            // the ~1 % an extra batch costs): d = 64, T = 1e4, 131 072 runs as three
            // batches of 43 691 (11 streams per wave, 3 % idle) took 398.8 ms, as four of
            // 32 768 (8 per wave) 386.5 ms; T = 1e3, 1e6 runs keeps its three
            // (round 2; the record is in git history).
            const int64_t rs = (int64_t)cus * 16;
            auto idle = [rs](int64_t c) {
                return (double)(((c + rs - 1) / rs) * rs) / (double)c - 1.0;
            };
            if (nbat >= 2 && chunk > 2 * rs) {
                const int64_t c2 = (R + nbat) / (nbat + 1);  // ceil(R / (nbat + 1))
                if (idle(c2) + 0.01 < idle(chunk)) {
                    ++nbat;
                    chunk = c2;
                }
            }
        }
        // Full generator waves (round 6): where the generator runs one wave per stream in a
        // single round (d = 1024: the HBM budget holds ~3 000 streams, the form 4 096 resident
        // waves) a batch takes as long as its busiest SIMD's waves, ceil(chunk / SIMDs), and
        // the d = 1024 and d = 64 forms cost the same per row at equal waves per SIMD (1 / 2 / 3
        // waves: 988 / 567 / 495 vs 1 106 / 610 / 495 cycles per 64-normal row,
        // profiles/r06_genwaves.jsonl).  So batches of whole waves per SIMD (a multiple of the
        // SIMDs, the last one the remainder) replace equal ones when that needs fewer waves in
        // all: 32 768 runs as 10 x 3 072 + 2 048 (32 waves per SIMD) instead of 12 x 2 731 (36).
        // OCX_BATCH_WAVES=0: equal batches (tuning).
        if (d != 64 && R > chunk) {
            const char* bw = std::getenv("OCX_BATCH_WAVES");
            int dev = 0, cus = 256;
            OCX_HIP(hipGetDevice(&dev));
            OCX_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
            const int64_t simds = 4 * (int64_t)cus;
            const int64_t cap = std::max<int64_t>(64, std::min<int64_t>(budget / per_seq, R));
            const int64_t cw = cap / simds * simds;
            if ((!bw || std::atoi(bw) != 0) && cw >= simds && cw <= ocx_gen_resident_waves(d, dev)) {
                auto waves = [simds](int64_t n) { return (n + simds - 1) / simds; };
                const int64_t nb = (R + chunk - 1) / chunk;
                const int64_t eq = (nb - 1) * waves(chunk) + waves(R - (nb - 1) * chunk);
                const int64_t full = (R / cw) * (cw / simds) + waves(R % cw);
                if (full < eq) chunk = cw;
            }
        }
        OCX_HIP(cx->out.ensure((size_t)chunk * 8));
        // Generation overlapped with FTRL (ocx_pipeline.hip) where the layout allows it
        // (OCX_PIPELINE=0: the sequential loop below).  For g(T) alone the equal batches go
        // through one call, so batch k+1's generation overlaps batch k's last FTRL pass too.
        ocx_layout Lp;
        if (int rc = ocx_layout_init(chunk, T, d, lanes_per_seq, &Lp)) return rc;
        const char* pe = std::getenv("OCX_PIPELINE");
        const bool pipe = (!pe || std::atoi(pe) != 0) && ocx_pipeline_supported(&Lp) &&
                          ocx_pipeline_worth(&Lp, pipe_wps());
        // A call of several batches holds its z tile at the whole budget (less two label
        // tiles), not at its own batch: the batches of successive calls (a sweep over T at 1e6
        // runs: 171 / 247 / 257 GB) differ, and growing an allocation of that size frees it and
        // maps it again — a 3.7 s hipMalloc after the free, against 0.48 s for the first one
        // (tools/batch_probe.py, profiles/r06_alloc_regrow.jsonl).
        if (R > chunk) {
            const int64_t zb = (int64_t)Lp.z_elems * 8, yb = (int64_t)Lp.y_elems * 8;
            OCX_HIP(cx->zt.ensure((size_t)std::max<int64_t>(zb, budget - 2 * yb)));
        }
        int64_t done = 0;
        // The batches the sub-batch pipeline leaves — capacity-limited (too few generator
        // rounds to cut: d = 64 at T = 1e5) or d != 64 (configs[4]'s d = 1024) — take the
        // trailing pipeline (ocx_pipeline.hip): batch k+1 generated chunk by chunk behind the
        // chunked FTRL pass over batch k, in the same z buffer (OCX_TRAILING=0: the sequential
        // loop below).  Its second label tile comes out of the budget.
        const char* te = std::getenv("OCX_TRAILING");
        bool trail = !pipe && onepass && (!te || std::atoi(te) != 0) &&
                     ocx_trailing_supported(&Lp) && R > chunk;
        if (trail) {
            const int64_t per_trail = per_seq + 8 * T + 64 * 8 * (2 * (int64_t)Lp.C + 7);
            int64_t c2 = std::max<int64_t>(64, std::min<int64_t>(budget / per_trail, R));
            const int64_t nb2 = (R + c2 - 1) / c2;
            c2 = (R + nb2 - 1) / nb2;
            // and no more streams than fit beside the FTRL waves in one generator round
            const int64_t cap = ocx_trailing_max_batch(&Lp);
            if (c2 > cap) {
                const int64_t nb3 = (R + cap - 1) / cap;
                c2 = (R + nb3 - 1) / nb3;
            }
            if (c2 < chunk) {
                chunk = c2;
                if (int rc = ocx_layout_init(chunk, T, d, lanes_per_seq, &Lp)) return rc;
                OCX_HIP(cx->out.ensure((size_t)chunk * 8));
            }
            trail = ocx_trailing_supported(&Lp) && R > chunk;
        }
        if (trail) {
            // every batch, the last one holding the remainder in the same tiles
            const int64_t nfull = (R + chunk - 1) / chunk, last_B = R - (nfull - 1) * chunk;
            OCX_HIP(cx->zt.ensure((size_t)Lp.z_elems * 8));
            OCX_HIP(cx->yt.ensure((size_t)Lp.y_elems * 8));
            OCX_HIP(cx->yt2.ensure((size_t)Lp.y_elems * 8));
            OCX_HIP(cx->gst.ensure((size_t)2 * Lp.G * Lp.S * 6 * 8));
            OCX_HIP(cx->fst.ensure((size_t)ocx_pipe_state_doubles(&Lp) * 8));
            OCX_HIP(cx->bad.ensure((size_t)nfull * sizeof(int)));
            double* rdst = regrets_on_device ? regrets : nullptr;
            if (!rdst) {
                OCX_HIP(cx->out.ensure((size_t)(nfull * chunk) * 8));
                rdst = cx->out.as<double>();
            }
            // FTRL chunks per horizon (OCX_TRAIL_CHUNKS, tuning): 4 900 x 1e5 x 64 batches,
            // 131 072 runs: 8 -> 4.06-4.08e9, 12 -> 4.13-4.17e9, 16 -> 4.06e9 timesteps/s; making
            // FTRL chunk c wait for the generator's chunk c - 2, 3 or 4 (so the reader does not
            // run ahead) measured no better (profiles/r05_trail_pace.jsonl, r05_trail_chunks.jsonl)
            // round 6, with the ramp (ocx_run_gen_sim_trailing): 8 chunks 4.20e9, 12 4.16e9
            // (profiles/r06_trail.jsonl)
            int nch = 8;
            if (const char* e = std::getenv("OCX_TRAIL_CHUNKS")) nch = std::max(2, std::atoi(e));
            OCX_HIP(ocx_run_gen_sim_trailing(&Lp, base_seed, run0, nfull, cx->zt.as<double>(),
                                             cx->yt.as<double>(), cx->yt2.as<double>(),
                                             cx->gst.as<uint64_t>(), cx->fst.as<double>(),
                                             cx->bad.as<int>(), eta0, rdst, last_B,
                                             dmax, nch, st));
            // a batch with a sequence the closed-form comparator could not certify (its regret
            // NaN, never the max) runs again whole: the kernel streams its second pass
            std::vector<int> hb((size_t)nfull, 0);
            OCX_HIP(hipMemcpyAsync(hb.data(), cx->bad.p, (size_t)nfull * sizeof(int),
                                   hipMemcpyDeviceToHost, st));
            OCX_HIP(hipStreamSynchronize(st));
            if (test_unclean_every > 0)  // test hook: these batches run again as if marked
                for (int64_t k = 0; k < nfull; k += test_unclean_every) hb[(size_t)k] = 1;
            for (int64_t k = 0; k < nfull; ++k) {
                if (!hb[(size_t)k]) continue;
                ocx_layout Lk = Lp;  // the last batch: same tiles, last_B runs
                if (k + 1 == nfull) Lk.B = last_B;
                OCX_HIP(ocx_launch_gen_gT(&Lk, base_seed, run0 + k * chunk, cx->zt.as<double>(),
                                          cx->yt.as<double>(), st));
                OCX_HIP(ocx_launch_alg(&Lk, cx->zt.as<double>(), cx->yt.as<double>(), 0, eta0,
                                       nullptr, rdst + k * chunk, nullptr, nullptr, nullptr, st,
                                       nullptr, nullptr, onepass));
                if (dmax) OCX_HIP(launch_max_fold(rdst + k * chunk, Lk.B, dmax, st));
            }
            if (!dmax && !regrets_on_device) {
                OCX_HIP(hipMemcpyAsync(regrets, rdst, (size_t)R * 8, hipMemcpyDeviceToHost, st));
                OCX_HIP(hipStreamSynchronize(st));
            }
            done = R;
        }
        if (pipe && dmax) {
            const int64_t nfull = R / chunk;
            OCX_HIP(cx->zt.ensure((size_t)Lp.z_elems * 8));
            OCX_HIP(cx->yt.ensure((size_t)Lp.y_elems * 8));
            OCX_HIP(ocx_run_gen_sim_pipelined(&Lp, base_seed, run0, nfull, cx->zt.as<double>(),
                                              cx->yt.as<double>(), eta0, cx->out.as<double>(),
                                              onepass, dmax, pipe_wps(), 0, st));
            done = nfull * chunk;
        }
        for (int64_t r0 = done; r0 < R; r0 += chunk) {
            const int64_t nb = std::min(chunk, R - r0);
            ocx_layout L;
            if (int rc = ocx_layout_init(nb, T, d, lanes_per_seq, &L)) return rc;
            OCX_HIP(cx->zt.ensure((size_t)L.z_elems * 8));
            OCX_HIP(cx->yt.ensure((size_t)L.y_elems * 8));
            double* rdst = regrets_on_device ? regrets + r0 : cx->out.as<double>();
            if (pipe && ocx_pipeline_supported(&L) && ocx_pipeline_worth(&L, pipe_wps())) {
                OCX_HIP(ocx_run_gen_sim_pipelined(&L, base_seed, run0 + r0, 1, cx->zt.as<double>(),
                                                  cx->yt.as<double>(), eta0, rdst, onepass,
                                                  nullptr, pipe_wps(), 0, st));
            } else {
                OCX_HIP(ocx_launch_gen_gT(&L, base_seed, run0 + r0, cx->zt.as<double>(),
                                          cx->yt.as<double>(), st));
                OCX_HIP(ocx_launch_alg(&L, cx->zt.as<double>(), cx->yt.as<double>(), 0, eta0,
                                       nullptr, rdst, nullptr, nullptr, nullptr, st, nullptr,
                                       nullptr, onepass));
            }
            if (dmax) {
                OCX_HIP(launch_max_fold(cx->out.as<double>(), nb, dmax, st));
            } else if (!regrets_on_device) {
                OCX_HIP(hipMemcpyAsync(regrets + r0, cx->out.p, (size_t)nb * 8,
                                       hipMemcpyDeviceToHost, st));
                OCX_HIP(hipStreamSynchronize(st));
            }
        }
        return finish();
    }
    // streamed: batches of kBatch runs, horizon cut into chunks of Tc steps
    // (ocx_stream.hip): seek → pass A (generate chunk, advance theta) → pass B
    // (regenerate chunk, comparator loss) with the PCG states saved at chunk starts.
    const int64_t Tc = std::max<int64_t>(1, budget / std::max<int64_t>(step_bytes, 1));
    const int64_t nch = (T + Tc - 1) / Tc;
    const int64_t Bc = L1.B;
    OCX_HIP(cx->rstate.ensure((size_t)(nch + 1) * Bc * 48));
    OCX_HIP(cx->lstate.ensure((size_t)(nch + 1) * Bc * 48));
    // theta rows are Dp wide, and Dp follows each batch's own layout (the lane rule
    // depends on the batch size, so a short last batch can have more, narrower lanes):
    // size for the widest batch and zero each batch with its own Dp
    ocx_layout Ltail;
    if (int rc = ocx_layout_init(R % Bc ? R % Bc : Bc, 1, d, lanes_per_seq, &Ltail)) return rc;
    OCX_HIP(cx->theta.ensure((size_t)std::max(Bc * L1.Dp, Ltail.B * Ltail.Dp) * 8));
    OCX_HIP(cx->acc.ensure((size_t)(Bc * 4 + 1) * 8));
    const int64_t unclean_every = test_unclean_every;
    for (int64_t r0 = 0; r0 < R; r0 += Bc) {
        const int64_t nb = std::min(Bc, R - r0);
        ocx_layout Lb;
        if (int rc = ocx_layout_init(nb, 1, d, lanes_per_seq, &Lb)) return rc;
        uint64_t* rs = cx->rstate.as<uint64_t>();
        uint64_t* ls = cx->lstate.as<uint64_t>();
        double* th = cx->theta.as<double>();
        double* cum = cx->acc.as<double>();
        double* comp = cum + Bc;
        double* reg = comp + Bc;
        double* unclean = onepass ? reg + Bc : nullptr;  // [nb + 1]
        OCX_HIP(ocx_launch_gen_seek(base_seed, T, run0 + r0, nb, d, rs, ls, st));
        OCX_HIP(hipMemsetAsync(th, 0, (size_t)nb * Lb.Dp * 8, st));
        OCX_HIP(hipMemsetAsync(cum, 0, (size_t)Bc * 2 * 8, st));
        if (unclean) OCX_HIP(hipMemsetAsync(unclean, 0, (size_t)(nb + 1) * 8, st));
        if (unclean && unclean_every > 0) {
            // test hook (ocx_test_gT_regrets_unclean, k): mark runs r0 + b with b % k == 0 as if a
            // step had failed the closed form's check, so the second pass serves them
            std::vector<double> mk((size_t)nb, 0.0);
            for (int64_t i = 0; i < nb; i += unclean_every) mk[(size_t)i] = 1.0;
            OCX_HIP(hipMemcpyAsync(unclean, mk.data(), (size_t)nb * 8, hipMemcpyHostToDevice, st));
            OCX_HIP(hipStreamSynchronize(st));
        }
        for (int pass = 0; pass < 2; ++pass) {
            if (pass == 1 && unclean) {
                // closed-form comparator for the clean sequences (no regeneration); the
                // second pass only when a sequence needs it
                OCX_HIP(ocx_launch_alg_chunk(&Lb, nullptr, nullptr, T, 0, eta0, 2, th, cum, comp,
                                             reg, st, unclean));
                double any = 0.0;
                OCX_HIP(hipMemcpyAsync(&any, unclean + nb, 8, hipMemcpyDeviceToHost, st));
                OCX_HIP(hipStreamSynchronize(st));
                if (any == 0.0) break;
            }
            for (int64_t c = 0; c < nch; ++c) {
                const int64_t t0 = c * Tc, tl = std::min(Tc, T - t0);
                ocx_layout L;
                if (int rc = ocx_layout_init(nb, tl, d, lanes_per_seq, &L)) return rc;
                OCX_HIP(cx->zt.ensure((size_t)L.z_elems * 8));
                OCX_HIP(cx->yt.ensure((size_t)L.y_elems * 8));
                uint64_t* rin = rs + (size_t)c * Bc * 6;
                uint64_t* lin = ls + (size_t)c * Bc * 6;
                OCX_HIP(ocx_launch_gen_gT_chunk(&L, T, rin, pass == 0 ? rin + Bc * 6 : nullptr, lin,
                                                pass == 0 ? lin + Bc * 6 : nullptr,
                                                cx->zt.as<double>(), cx->yt.as<double>(), st));
                OCX_HIP(ocx_launch_alg_chunk(&L, cx->zt.as<double>(), cx->yt.as<double>(), t0, 0,
                                             eta0, pass, th, cum, comp,
                                             (pass == 1 && c == nch - 1) ? reg : nullptr, st,
                                             unclean));
            }
        }
        if (dmax) {
            OCX_HIP(launch_max_fold(reg, nb, dmax, st));
        } else if (regrets_on_device) {
            OCX_HIP(hipMemcpyAsync(regrets + r0, reg, (size_t)nb * 8, hipMemcpyDeviceToDevice, st));
        } else {
            OCX_HIP(hipMemcpyAsync(regrets + r0, reg, (size_t)nb * 8, hipMemcpyDeviceToHost, st));
            OCX_HIP(hipStreamSynchronize(st));
        }
    }
    return finish();
}

}  // namespace

extern "C" {

int ocx_gT_regrets(uint64_t base_seed, int64_t T, int64_t run0, int64_t R, int64_t d,
                   double eta0, double* regrets, int lanes_per_seq, int device) {
    if (!regrets && R > 0) return fail(OCX_E_INVALID, "NULL regrets");
    return gT_run(base_seed, T, run0, R, d, eta0, regrets, nullptr, lanes_per_seq, device);
}

int ocx_gT_regrets_dev(uint64_t base_seed, int64_t T, int64_t run0, int64_t R, int64_t d,
                       double eta0, double* regrets_dev, int lanes_per_seq, int device) {
    if (!regrets_dev && R > 0) return fail(OCX_E_INVALID, "NULL regrets");
    return gT_run(base_seed, T, run0, R, d, eta0, regrets_dev, nullptr, lanes_per_seq, device, 0,
                  true);
}

int ocx_test_alg_pipe_chunked(const ocx_layout* L, const double* z_tiled, const double* y_tiled,
                              double eta0, int64_t chunk_steps, double* regret, int* bad,
                              void* stream) {
    StreamDevice sd_(stream);
    if (int rc = check_layout(L)) return rc;
    if (!ocx_pipe_supported(L)) return fail(OCX_E_UNSUPPORTED, "not a pipelined butterfly layout");
    if (chunk_steps <= 0 || chunk_steps % 64) return fail(OCX_E_INVALID, "chunk_steps: a multiple of 64");
    if (L->B > 0 && (!regret || !bad || !z_tiled || !y_tiled)) return fail(OCX_E_INVALID, "NULL buffer");
    const hipStream_t st = (hipStream_t)stream;
    double* state = nullptr;
    OCX_HIP(hipMalloc(&state, (size_t)std::max<int64_t>(ocx_pipe_state_doubles(L), 1) * 8));
    hipError_t e = hipSuccess;
    for (int64_t t0 = 0; t0 < L->T && e == hipSuccess; t0 += chunk_steps)
        e = ocx_launch_alg_pipe_chunk(L, z_tiled, y_tiled, eta0, regret, 1, t0,
                                      std::min(chunk_steps, L->T - t0), state, bad, nullptr, st);
    const hipError_t es = hipStreamSynchronize(st);
    (void)hipFree(state);
    OCX_HIP(e);
    OCX_HIP(es);
    return OCX_OK;
}

int64_t ocx_test_trailing_batches(void) { return ocx_trailing_batches_run(); }

int ocx_test_gT_regrets_unclean(uint64_t base_seed, int64_t T, int64_t run0, int64_t R,
                                int64_t d, double eta0, double* regrets, int lanes_per_seq,
                                int device, int64_t unclean_every) {
    if (!regrets && R > 0) return fail(OCX_E_INVALID, "NULL regrets");
    if (unclean_every < 1) return fail(OCX_E_INVALID, "unclean_every must be >= 1");
    return gT_run(base_seed, T, run0, R, d, eta0, regrets, nullptr, lanes_per_seq, device,
                  unclean_every);
}

int ocx_gT_max(uint64_t base_seed, int64_t T, int64_t run0, int64_t R, int64_t d, double eta0,
               int lanes_per_seq, int device, double* gmax) {
    if (!gmax) return fail(OCX_E_INVALID, "NULL gmax");
    return gT_run(base_seed, T, run0, R, d, eta0, nullptr, gmax, lanes_per_seq, device);
}

int ocx_gT_sweep_devices(const int64_t* T_grid, int nT, int64_t runs, uint64_t base_seed,
                         int64_t d, double eta0, const int* devices, int ndev, int lanes_per_seq,
                         double* gmax, double* regrets) {
    if (nT < 0 || runs < 0 || d < 0) return fail(OCX_E_INVALID, "negative argument");
    if (nT == 0) return OCX_OK;
    if (!T_grid || !gmax || !devices || ndev < 1) return fail(OCX_E_INVALID, "NULL argument");
    for (int i = 0; i < nT; ++i)
        if (T_grid[i] < 0) return fail(OCX_E_INVALID, "negative T");
    for (int i = 0; i < nT; ++i) {
        // without `regrets` each shard reduces its max on its GPU and only that leaves it
        double* row = regrets ? regrets + (size_t)i * runs : nullptr;
        std::vector<double> smax(ndev, 0.0);
        // contiguous shards [runs*k/ndev, runs*(k+1)/ndev), one host thread per shard
        std::vector<int> rc(ndev, OCX_OK);
        std::vector<std::string> err(ndev);
        auto work = [&](int k) {
            const int64_t lo = runs * k / ndev, hi = runs * (k + 1) / ndev;
            rc[k] = gT_run(base_seed, T_grid[i], lo, hi - lo, d, eta0, row ? row + lo : nullptr,
                           row ? nullptr : &smax[k], lanes_per_seq, devices[k]);
            if (rc[k]) err[k] = g_err;  // the message is thread-local
        };
        std::vector<std::thread> th;
        for (int k = 1; k < ndev; ++k) th.emplace_back(work, k);
        work(0);
        for (auto& t : th) t.join();
        for (int k = 0; k < ndev; ++k)
            if (rc[k]) return fail(rc[k], "device " + std::to_string(devices[k]) + ": " + err[k]);
        double m = 0.0;  // fast_algorithms.py:228, :242-243
        if (row) {
            for (int64_t r = 0; r < runs; ++r)
                if (row[r] > m) m = row[r];
        } else {
            for (int k = 0; k < ndev; ++k)
                if (smax[k] > m) m = smax[k];
        }
        gmax[i] = m;
    }
    return OCX_OK;
}

int ocx_gT_sweep(const int64_t* T_grid, int nT, int64_t runs, uint64_t base_seed, int64_t d,
                 double eta0, int ngpus, double* gmax, double* regrets) {
    int n = 0;
    OCX_HIP(hipGetDeviceCount(&n));
    if (ngpus <= 0) ngpus = n;
    if (ngpus > n) return fail(OCX_E_INVALID, "ngpus " + std::to_string(ngpus) +
                                                  " > device count " + std::to_string(n));
    std::vector<int> devs(ngpus);
    for (int k = 0; k < ngpus; ++k) devs[k] = k;
    return ocx_gT_sweep_devices(T_grid, nT, runs, base_seed, d, eta0, devs.data(), ngpus,
                                OCX_LANES_BEST, gmax, regrets);
}

int ocx_comparator_loss_blas_batch(const double* z, const double* y, const double* x, int64_t B,
                                   int64_t T, int64_t d, double* comp_loss, int device) {
    if (B < 0 || T < 0 || d < 0) return fail(OCX_E_INVALID, "negative size");
    if (B == 0) return OCX_OK;
    if ((T * d > 0 && !z) || (T > 0 && !y) || (d > 0 && !x) || !comp_loss)
        return fail(OCX_E_INVALID, "NULL argument");
    DevCtx* cx;
    if (int rc = ctx_enter(device, &cx)) return rc;
    std::lock_guard<std::mutex> lk(cx->mu);
    hipStream_t st = cx->stream;
    const size_t nz = (size_t)(B * T * d), ny = (size_t)(B * T), nx = (size_t)(B * d);
    OCX_HIP(cx->zraw.ensure(nz * 8));
    OCX_HIP(cx->yraw.ensure(ny * 8));
    OCX_HIP(cx->cmp.ensure(nx * 8 + 8));
    OCX_HIP(cx->at.ensure(ny * 8 + 8));
    OCX_HIP(cx->out.ensure((size_t)B * 8));
    if (nz) OCX_HIP(hipMemcpyAsync(cx->zraw.p, z, nz * 8, hipMemcpyHostToDevice, st));
    if (ny) OCX_HIP(hipMemcpyAsync(cx->yraw.p, y, ny * 8, hipMemcpyHostToDevice, st));
    if (nx) OCX_HIP(hipMemcpyAsync(cx->cmp.p, x, nx * 8, hipMemcpyHostToDevice, st));
    OCX_HIP(ocx_launch_comp_blas(cx->zraw.as<double>(), cx->yraw.as<double>(), cx->cmp.as<double>(),
                                 B, T, d, cx->at.as<double>(), cx->out.as<double>(), st));
    OCX_HIP(hipMemcpyAsync(comp_loss, cx->out.p, (size_t)B * 8, hipMemcpyDeviceToHost, st));
    OCX_HIP(hipStreamSynchronize(st));
    return OCX_OK;
}

// ---------------------------------------------------------------- float32 twin
int ocx_twin32_batch(const float* z, const float* y, int64_t B, int64_t T, int64_t d, int algo,
                     double eta0, const double* thresh, float* result, double* cum_loss,
                     float* comp_loss, int64_t* switch_step, int device) {
    if (algo < 0 || algo > 2) return fail(OCX_E_INVALID, "algo must be 0 (FTRL), 1 (FTL) or 2 (SMART)");
    if (B < 0 || T < 0 || d < 0) return fail(OCX_E_INVALID, "negative size");
    if (d > 32) return fail(OCX_E_UNSUPPORTED, "the float32 twin supports d <= 32");
    ocx_layout L;
    if (int rc = ocx_layout_init(B, T, d, -1, &L)) return rc;  // one lane per sequence
    if (B == 0) return OCX_OK;
    if ((T * d > 0 && !z) || (T > 0 && !y) || !result || (algo == 2 && !thresh))
        return fail(OCX_E_INVALID, "NULL argument");
    DevCtx* cx;
    if (int rc = ctx_enter(device, &cx)) return rc;
    std::lock_guard<std::mutex> lk(cx->mu);
    hipStream_t st = cx->stream;
    const size_t nz = (size_t)(B * T * d), ny = (size_t)(B * T);
    OCX_HIP(cx->zraw.ensure(nz * 4));
    OCX_HIP(cx->yraw.ensure(ny * 4));
    OCX_HIP(cx->zt.ensure((size_t)L.z_elems * 8));
    OCX_HIP(cx->yt.ensure((size_t)L.y_elems * 8));
    OCX_HIP(cx->out.ensure((size_t)B * 16));
    OCX_HIP(cx->sw.ensure((size_t)B * 8));
    if (nz) OCX_HIP(hipMemcpyAsync(cx->zraw.p, z, nz * 4, hipMemcpyHostToDevice, st));
    if (ny) OCX_HIP(hipMemcpyAsync(cx->yraw.p, y, ny * 4, hipMemcpyHostToDevice, st));
    const double* dthr = nullptr;
    if (algo == 2) {
        OCX_HIP(cx->thr.ensure((size_t)B * 8));
        OCX_HIP(hipMemcpyAsync(cx->thr.p, thresh, (size_t)B * 8, hipMemcpyHostToDevice, st));
        dthr = cx->thr.as<double>();
    }
    OCX_HIP(ocx_launch_pack32(&L, cx->zraw.as<float>(), cx->yraw.as<float>(), cx->zt.as<double>(),
                              cx->yt.as<double>(), st));
    double* cum = cx->out.as<double>();
    float* res = reinterpret_cast<float*>(cum + B);
    float* comp = res + B;
    OCX_HIP(ocx_launch_twin32(&L, cx->zt.as<double>(), cx->yt.as<double>(), algo, eta0, dthr, 0,
                              res, cum, comp, cx->sw.as<int64_t>(), st));
    OCX_HIP(hipMemcpyAsync(result, res, (size_t)B * 4, hipMemcpyDeviceToHost, st));
    if (cum_loss) OCX_HIP(hipMemcpyAsync(cum_loss, cum, (size_t)B * 8, hipMemcpyDeviceToHost, st));
    if (comp_loss) OCX_HIP(hipMemcpyAsync(comp_loss, comp, (size_t)B * 4, hipMemcpyDeviceToHost, st));
    if (switch_step)
        OCX_HIP(hipMemcpyAsync(switch_step, cx->sw.p, (size_t)B * 8, hipMemcpyDeviceToHost, st));
    OCX_HIP(hipStreamSynchronize(st));
    return OCX_OK;
}

int ocx_dev_twin32(const ocx_layout* L, const double* z_tiled, const double* y_tiled, int algo,
                   double eta0, const double* thresh, float* result, double* cum_loss,
                   float* comp_loss, int64_t* switch_step, void* stream) {
    StreamDevice sd_(stream);
    if (int rc = check_layout(L)) return rc;
    if (L->P != 1) return fail(OCX_E_INVALID, "the float32 twin needs a one-lane layout (lanes_per_seq = -1)");
    if (L->d > 32) return fail(OCX_E_UNSUPPORTED, "the float32 twin supports d <= 32");
    if (algo < 0 || algo > 2) return fail(OCX_E_INVALID, "algo must be 0 (FTRL), 1 (FTL) or 2 (SMART)");
    if (L->B > 0 && (!result || (algo == 2 && !thresh)))
        return fail(OCX_E_INVALID, "NULL result / thresh");
    if (L->z_elems && (!z_tiled || !y_tiled)) return fail(OCX_E_INVALID, "NULL input buffer");
    OCX_HIP(ocx_launch_twin32(L, z_tiled, y_tiled, algo, eta0, algo == 2 ? thresh : nullptr, 0,
                              result, cum_loss, comp_loss, switch_step, (hipStream_t)stream));
    return OCX_OK;
}

int ocx_twin32_gT_regrets(uint64_t base_seed, int64_t T, int64_t run0, int64_t R, int64_t d,
                          double eta0, float* regrets, int device) {
    if (R < 0 || run0 < 0 || T < 0 || d < 0) return fail(OCX_E_INVALID, "negative argument");
    if (d > 32) return fail(OCX_E_UNSUPPORTED, "the float32 twin supports d <= 32");
    if (T * d >= ((int64_t)1 << 32)) return fail(OCX_E_UNSUPPORTED, "T * d >= 2^32");
    if (R == 0) return OCX_OK;
    if (!regrets) return fail(OCX_E_INVALID, "NULL regrets");
    DevCtx* cx;
    if (int rc = ctx_enter(device, &cx)) return rc;
    std::lock_guard<std::mutex> lk(cx->mu);
    hipStream_t st = cx->stream;
    ocx_layout L1;
    if (int rc = ocx_layout_init(1, T, d, -1, &L1)) return rc;
    // batches of <= 4 GiB of tiles (raw float64 normals, rounded to float in the kernel)
    const int64_t per_seq = std::max<int64_t>(8, T * (L1.C + 1) * 8);
    const int64_t chunk = std::max<int64_t>(64, std::min<int64_t>(R, ((int64_t)4 << 30) / per_seq));
    OCX_HIP(cx->out.ensure((size_t)chunk * 16));
    for (int64_t r0 = 0; r0 < R; r0 += chunk) {
        const int64_t nb = std::min(chunk, R - r0);
        ocx_layout L;
        if (int rc = ocx_layout_init(nb, T, d, -1, &L)) return rc;
        OCX_HIP(cx->zt.ensure((size_t)L.z_elems * 8));
        OCX_HIP(cx->yt.ensure((size_t)L.y_elems * 8));
        OCX_HIP(ocx_launch_gen_gT_raw(&L, base_seed, run0 + r0, cx->zt.as<double>(),
                                      cx->yt.as<double>(), st));
        float* res = reinterpret_cast<float*>(cx->out.as<double>() + chunk);
        OCX_HIP(ocx_launch_twin32(&L, cx->zt.as<double>(), cx->yt.as<double>(), 0, eta0, nullptr, 1,
                                  res, nullptr, nullptr, nullptr, st));
        OCX_HIP(hipMemcpyAsync(regrets + r0, res, (size_t)nb * 4, hipMemcpyDeviceToHost, st));
        OCX_HIP(hipStreamSynchronize(st));
    }
    return OCX_OK;
}

}  // extern "C"
