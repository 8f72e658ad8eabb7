// capture_repro.hip — does HIP graph capture of a multi-stream fork/join crash without torch?
//
// tests/test_gpu_pipeline.py::test_pipeline_captures_into_a_graph captures
// ocx_dev_gen_simulate (ocx_pipeline.hip: the caller's stream forks to three library streams
// through one event, sub-batches ordered by per-sub-batch events, joined back by one event per
// stream) with torch.cuda.graph, and the process segfaults in capture_end.  This program takes
// torch out of the picture, in three stages, each printed before it runs:
//   1. the same fork / event / join pattern with stand-in kernels, pure HIP: a warm-up run
//      on the same streams and events, then hipStreamBeginCapture (global mode, as
//      torch.cuda.graph's default), hipStreamEndCapture, hipGraphInstantiate, two replays;
//   2. libocx's ocx_dev_gen_simulate itself captured the same way (no torch in the process),
//      the replays checked against an eager call bit for bit;
//   3. stage 2 in thread-local capture mode.
// Build (CPU):  hipcc --offload-arch=gfx950 -O2 tools/capture_repro.hip -o tools/capture_repro \
//                  -Lonline_convex_optimization_amd -locx -Wl,-rpath,'$ORIGIN/../online_convex_optimization_amd'
// Run (GPU):    timeout -k 10 120 tools/capture_repro
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../include/ocx.h"

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            std::printf("FAIL %s: %s (line %d)\n", #x, hipGetErrorString(e_), __LINE__);  \
            std::fflush(stdout);                                                           \
            std::exit(2);                                                                  \
        }                                                                                  \
    } while (0)

__global__ void produce(double* buf, int64_t n, double v) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) buf[i] = v + (double)i;
}
__global__ void consume(const double* buf, double* out, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = 2.0 * buf[i];
}

struct Pattern {
    hipStream_t gen2, sim, sim2;
    hipEvent_t fork, jg2, js, js2;
    std::vector<hipEvent_t> eg, es;
};

// ocx_run_gen_sim_pipelined's schedule: nb batches x ns sub-batches, generator launches
// alternating st / gen2, consumer launches alternating sim / sim2
void enqueue(Pattern& p, hipStream_t st, double* buf, double* out, int64_t per, int nb, int ns) {
    CK(hipEventRecord(p.fork, st));
    CK(hipStreamWaitEvent(p.gen2, p.fork, 0));
    CK(hipStreamWaitEvent(p.sim, p.fork, 0));
    CK(hipStreamWaitEvent(p.sim2, p.fork, 0));
    std::vector<char> rec(ns, 0);
    int j = 0;
    for (int k = 0; k < nb; ++k)
        for (int i = 0; i < ns; ++i, ++j) {
            hipStream_t gs = (j & 1) ? p.gen2 : st, ss = (j & 1) ? p.sim2 : p.sim;
            if (rec[i]) CK(hipStreamWaitEvent(gs, p.es[i], 0));
            hipLaunchKernelGGL(produce, dim3((per + 255) / 256), dim3(256), 0, gs, buf + i * per, per,
                               (double)k);
            CK(hipGetLastError());
            CK(hipEventRecord(p.eg[i], gs));
            CK(hipStreamWaitEvent(ss, p.eg[i], 0));
            hipLaunchKernelGGL(consume, dim3((per + 255) / 256), dim3(256), 0, ss, buf + i * per,
                               out + i * per, per);
            CK(hipGetLastError());
            CK(hipEventRecord(p.es[i], ss));
            rec[i] = 1;
        }
    CK(hipEventRecord(p.jg2, p.gen2));
    CK(hipEventRecord(p.js, p.sim));
    CK(hipEventRecord(p.js2, p.sim2));
    CK(hipStreamWaitEvent(st, p.jg2, 0));
    CK(hipStreamWaitEvent(st, p.js, 0));
    CK(hipStreamWaitEvent(st, p.js2, 0));
}

int stage1() {
    std::printf("stage 1: pure HIP fork/join pattern under capture (global mode)\n");
    std::fflush(stdout);
    const int nb = 2, ns = 6;
    const int64_t per = 1 << 16;
    double *buf, *out;
    CK(hipMalloc(&buf, ns * per * 8));
    CK(hipMalloc(&out, ns * per * 8));
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    Pattern p;
    CK(hipStreamCreateWithFlags(&p.gen2, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&p.sim, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&p.sim2, hipStreamNonBlocking));
    for (hipEvent_t* e : {&p.fork, &p.jg2, &p.js, &p.js2}) CK(hipEventCreateWithFlags(e, hipEventDisableTiming));
    p.eg.resize(ns);
    p.es.resize(ns);
    for (int i = 0; i < ns; ++i) {
        CK(hipEventCreateWithFlags(&p.eg[i], hipEventDisableTiming));
        CK(hipEventCreateWithFlags(&p.es[i], hipEventDisableTiming));
    }
    enqueue(p, st, buf, out, per, nb, ns);  // warm-up, eager
    CK(hipStreamSynchronize(st));
    std::vector<double> ref(ns * per), got(ns * per);
    CK(hipMemcpy(ref.data(), out, ns * per * 8, hipMemcpyDeviceToHost));
    CK(hipMemset(out, 0, ns * per * 8));
    CK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
    enqueue(p, st, buf, out, per, nb, ns);
    hipGraph_t g;
    std::printf("  end capture\n");
    std::fflush(stdout);
    CK(hipStreamEndCapture(st, &g));
    hipGraphExec_t ge;
    std::printf("  instantiate\n");
    std::fflush(stdout);
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    for (int r = 0; r < 2; ++r) {
        CK(hipMemsetAsync(out, 0, ns * per * 8, st));
        CK(hipGraphLaunch(ge, st));
        CK(hipStreamSynchronize(st));
        CK(hipMemcpy(got.data(), out, ns * per * 8, hipMemcpyDeviceToHost));
        if (std::memcmp(got.data(), ref.data(), ns * per * 8) != 0) {
            std::printf("  replay %d: WRONG output\n", r);
            return 1;
        }
    }
    std::printf("stage 1 ok: captured, instantiated, replayed twice, output equal\n");
    std::fflush(stdout);
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(g));
    CK(hipFree(buf));
    CK(hipFree(out));
    return 0;
}

int stage_ocx(hipStreamCaptureMode mode, const char* name) {
    std::printf("%s: ocx_dev_gen_simulate under capture\n", name);
    std::fflush(stdout);
    ocx_layout L;
    const int64_t B = 3000, T = 120, d = 64;
    if (ocx_layout_init(B, T, d, 8, &L) != 0) {
        std::printf("FAIL layout\n");
        return 2;
    }
    double *z, *y, *reg, *gm;
    CK(hipMalloc(&z, L.z_elems * 8));
    CK(hipMalloc(&y, L.y_elems * 8));
    CK(hipMalloc(&reg, B * 8));
    CK(hipMalloc(&gm, 8));
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    auto call = [&]() {
        const int rc = ocx_dev_gen_simulate(&L, 7, 0, 2, z, y, 1.4142135623730951, reg, gm, 0u, 512, st);
        if (rc != 0) {
            char msg[512];
            ocx_last_error(msg, sizeof msg);
            std::printf("FAIL ocx_dev_gen_simulate rc=%d: %s\n", rc, msg);
            std::exit(2);
        }
    };
    call();  // eager
    CK(hipStreamSynchronize(st));
    std::vector<double> ref(B), got(B);
    double gref = 0, gg = 0;
    CK(hipMemcpy(ref.data(), reg, B * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(&gref, gm, 8, hipMemcpyDeviceToHost));
    CK(hipStreamBeginCapture(st, mode));
    call();
    hipGraph_t g;
    std::printf("  end capture\n");
    std::fflush(stdout);
    CK(hipStreamEndCapture(st, &g));
    hipGraphExec_t ge;
    std::printf("  instantiate\n");
    std::fflush(stdout);
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    for (int r = 0; r < 2; ++r) {
        CK(hipMemsetAsync(reg, 0, B * 8, st));
        CK(hipMemsetAsync(gm, 0, 8, st));
        CK(hipGraphLaunch(ge, st));
        CK(hipStreamSynchronize(st));
        CK(hipMemcpy(got.data(), reg, B * 8, hipMemcpyDeviceToHost));
        CK(hipMemcpy(&gg, gm, 8, hipMemcpyDeviceToHost));
        if (std::memcmp(got.data(), ref.data(), B * 8) != 0 || gg != gref) {
            std::printf("  replay %d: WRONG regrets / g(T)\n", r);
            return 1;
        }
    }
    std::printf("%s ok: replayed twice, regrets and g(T) bit-identical to the eager call\n", name);
    std::fflush(stdout);
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(g));
    return 0;
}

int main() {
    int rc = stage1();
    if (rc) return rc;
    rc = stage_ocx(hipStreamCaptureModeGlobal, "stage 2 (global mode)");
    if (rc) return rc;
    return stage_ocx(hipStreamCaptureModeThreadLocal, "stage 3 (thread-local mode)");
}
