// Where do the waves of a CU-masked stream run?  For a few masks given to
// hipExtStreamCreateWithCUMask, launch many short one-wave blocks and record each block's
// XCC_ID and HW_ID (SE, CU), then print the distinct CUs used per XCC.  Decides which mask
// bits to give the FTRL side of a CU split (tools/cumask_probe.py) so that it spreads over
// the XCDs' memory paths.
//
//   hipcc --offload-arch=gfx950 -O2 -o tools/cumask_map tools/cumask_map.cpp && tools/cumask_map
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <set>
#include <string>
#include <tuple>
#include <vector>

#define CHECK(x)                                                                      \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            std::exit(1);                                                             \
        }                                                                             \
    } while (0)

__global__ void where(unsigned* out, long spin) {
    if (threadIdx.x != 0) return;
    const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);   // HW_ID
    const unsigned xcc = __builtin_amdgcn_s_getreg((15 << 11) | 20); // XCC_ID [3:0]
    const long t0 = (long)__builtin_amdgcn_s_memrealtime();
    while ((long)__builtin_amdgcn_s_memrealtime() - t0 < spin) {
    }
    out[blockIdx.x] = (xcc & 0xfu) << 16 | ((hw >> 13) & 7u) << 8 | ((hw >> 8) & 0xfu);
}

int main() {
    int ncu = 0;
    CHECK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
    const int nblk = 8192;
    unsigned* d = nullptr;
    CHECK(hipMalloc(&d, nblk * sizeof(unsigned)));
    std::vector<unsigned> h(nblk);
    struct M {
        std::string name;
        std::vector<int> bits;
    };
    std::vector<M> masks;
    auto add = [&](std::string n, int first, int count, int step) {
        M m{n, {}};
        for (int i = 0; i < count; ++i) m.bits.push_back(first + i * step);
        masks.push_back(m);
    };
    add("all", 0, ncu, 1);
    add("contig0-31", 0, 32, 1);
    add("stride8x32", 0, 32, 8);
    add("contig0-7", 0, 8, 1);
    add("stride32x8", 0, 8, 32);
    add("contig0-63", 0, 64, 1);
    add("stride4x64", 0, 64, 4);
    add("stride2x128", 0, 128, 2);
    for (const M& m : masks) {
        std::vector<uint32_t> w((ncu + 31) / 32, 0u);
        for (int b : m.bits) w[b / 32] |= 1u << (b % 32);
        hipStream_t s;
        CHECK(hipExtStreamCreateWithCUMask(&s, (uint32_t)w.size(), w.data()));
        CHECK(hipMemsetAsync(d, 0xff, nblk * sizeof(unsigned), s));
        hipLaunchKernelGGL(where, dim3(nblk), dim3(64), 0, s, d, 2000L);  // 20 us each
        CHECK(hipGetLastError());
        CHECK(hipStreamSynchronize(s));
        CHECK(hipMemcpy(h.data(), d, nblk * sizeof(unsigned), hipMemcpyDeviceToHost));
        CHECK(hipStreamDestroy(s));
        std::set<unsigned> cus;
        std::vector<std::set<unsigned>> per_xcc(16);
        for (unsigned v : h) {
            cus.insert(v);
            per_xcc[(v >> 16) & 15].insert(v & 0xffffu);
        }
        std::printf("%-12s bits=%3zu distinct_cus=%3zu per_xcc:", m.name.c_str(), m.bits.size(), cus.size());
        for (int x = 0; x < 8; ++x) std::printf(" %zu", per_xcc[x].size());
        std::printf("  first:");
        int k = 0;
        for (unsigned v : cus) {
            if (k++ >= 6) break;
            std::printf(" x%u/se%u/cu%u", v >> 16, (v >> 8) & 0xff, v & 0xff);
        }
        std::printf("\n");
    }
    CHECK(hipFree(d));
    return 0;
}
