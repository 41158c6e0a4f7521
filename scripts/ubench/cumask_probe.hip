// Where the chunker's overlap-mode streams run (RC_PIPELINED, capi.cpp setup_overlap).
// Two streams with complementary CU masks -- the first R bits (the chain's) and the rest (the
// tile kernel's) -- each run a kernel of many short workgroups that record the CU they ran on
// (HW_ID: CU / SH / SE, XCC_ID).  Prints, per mask, the distinct CUs used per XCD and whether
// the two sets are disjoint; then runs a 1024-thread 144 KiB-LDS persistent kernel (the tile
// kernel's footprint) on the tile stream beside a short-wave kernel on the chain stream and
// prints both kernels' spans (s_memrealtime, 100 MHz): the chain kernel must finish inside.
//   ./cumask_probe [R=16]
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <set>
#include <tuple>
#include <vector>

#define CHECK(x)                                                                   \
    do {                                                                           \
        hipError_t e_ = (x);                                                       \
        if (e_ != hipSuccess) {                                                    \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                \
            exit(1);                                                               \
        }                                                                          \
    } while (0)

// HW_ID (hwreg 4, 32 bits) and XCC_ID (hwreg 20, low 16 bits)
__global__ void where(uint32_t *out, int spin) {
    const uint32_t hw = __builtin_amdgcn_s_getreg(4 | (31 << 11));
    const uint32_t xcc = __builtin_amdgcn_s_getreg(20 | (15 << 11));
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < (uint64_t)spin) __builtin_amdgcn_s_sleep(2);
    if (threadIdx.x == 0) {
        out[2 * blockIdx.x] = hw;
        out[2 * blockIdx.x + 1] = xcc;
    }
}

// a persistent 1024-thread workgroup per CU with 144 KiB of LDS, spinning `spin` ticks
__global__ void __launch_bounds__(1024) hold(uint64_t *span, int spin) {
    extern __shared__ uint32_t lds[];
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    lds[threadIdx.x] = threadIdx.x;
    __syncthreads();
    while (__builtin_amdgcn_s_memrealtime() - t0 < (uint64_t)spin) __builtin_amdgcn_s_sleep(8);
    const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) {
        span[2 * blockIdx.x] = t0 + lds[blockIdx.x & 1023] * 0;
        span[2 * blockIdx.x + 1] = t1;
    }
}

__global__ void small(uint64_t *span, int spin) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < (uint64_t)spin) __builtin_amdgcn_s_sleep(2);
    if (threadIdx.x == 0) {
        span[2 * blockIdx.x] = t0;
        span[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime();
    }
}

typedef std::tuple<uint32_t, uint32_t, uint32_t, uint32_t> Cu;  // xcc, se, sh, cu

std::set<Cu> run_where(hipStream_t s, int blocks) {
    uint32_t *d = nullptr;
    CHECK(hipMalloc(&d, 8 * (size_t)blocks));
    hipLaunchKernelGGL(where, dim3(blocks), dim3(64), 0, s, d, 2000);  // 20 us each
    CHECK(hipGetLastError());
    CHECK(hipStreamSynchronize(s));
    std::vector<uint32_t> h(2 * (size_t)blocks);
    CHECK(hipMemcpy(h.data(), d, 8 * (size_t)blocks, hipMemcpyDeviceToHost));
    CHECK(hipFree(d));
    std::set<Cu> cus;
    for (int b = 0; b < blocks; ++b) {
        const uint32_t hw = h[2 * b], xcc = h[2 * b + 1] & 15;
        cus.insert(Cu(xcc, (hw >> 13) & 7, (hw >> 12) & 1, (hw >> 8) & 15));
    }
    return cus;
}

void report(const char *name, const std::set<Cu> &s) {
    int per[16] = {0};
    for (auto &c : s) per[std::get<0>(c) & 15]++;
    printf("%s: %zu CUs; per XCD:", name, s.size());
    for (int x = 0; x < 8; ++x) printf(" %d", per[x]);
    printf("\n");
}

int main(int argc, char **argv) {
    const int R = argc > 1 ? atoi(argv[1]) : 16;
    int cus = 0;
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    std::vector<uint32_t> tm((cus + 31) / 32, 0), xm((cus + 31) / 32, 0);
    for (int i = 0; i < cus; ++i) (i < R ? xm : tm)[i / 32] |= 1u << (i % 32);
    hipStream_t ts, xs, all;
    CHECK(hipExtStreamCreateWithCUMask(&ts, (uint32_t)tm.size(), tm.data()));
    CHECK(hipExtStreamCreateWithCUMask(&xs, (uint32_t)xm.size(), xm.data()));
    CHECK(hipStreamCreateWithFlags(&all, hipStreamNonBlocking));
    printf("device CUs %d, reserved (chain) %d\n", cus, R);
    const auto a = run_where(all, 16 * cus), t = run_where(ts, 16 * cus), x = run_where(xs, 16 * cus);
    report("unmasked", a);
    report("tile mask", t);
    report("chain mask", x);
    size_t both = 0;
    for (auto &c : x) both += t.count(c);
    printf("CUs in both masks: %zu (expect 0); tile + chain = %zu (expect %zu)\n", both,
           t.size() + x.size(), a.size());

    // co-residency: the tile footprint on the tile stream, short waves on the chain stream
    const int tile_grid = cus - R;
    uint64_t *dh = nullptr, *dsm = nullptr;
    const int sm_blocks = 64 * R;
    CHECK(hipMalloc(&dh, 16 * (size_t)tile_grid));
    CHECK(hipMalloc(&dsm, 16 * (size_t)sm_blocks));
    CHECK(hipFuncSetAttribute((const void *)hold, hipFuncAttributeMaxDynamicSharedMemorySize, 144 << 10));
    hipLaunchKernelGGL(hold, dim3(tile_grid), dim3(1024), 144 << 10, ts, dh, 200000);  // 2 ms
    CHECK(hipGetLastError());
    hipLaunchKernelGGL(small, dim3(sm_blocks), dim3(256), 0, xs, dsm, 10000);  // 100 us each
    CHECK(hipGetLastError());
    CHECK(hipDeviceSynchronize());
    std::vector<uint64_t> h(2 * (size_t)tile_grid), g(2 * (size_t)sm_blocks);
    CHECK(hipMemcpy(h.data(), dh, h.size() * 8, hipMemcpyDeviceToHost));
    CHECK(hipMemcpy(g.data(), dsm, g.size() * 8, hipMemcpyDeviceToHost));
    uint64_t h0 = ~0ull, h1 = 0, g0 = ~0ull, g1 = 0;
    for (int i = 0; i < tile_grid; ++i) h0 = std::min(h0, h[2 * i]), h1 = std::max(h1, h[2 * i + 1]);
    for (int i = 0; i < sm_blocks; ++i) g0 = std::min(g0, g[2 * i]), g1 = std::max(g1, g[2 * i + 1]);
    printf("tile-footprint kernel (%d WGs): %.1f .. %.1f us; chain-side kernel (%d WGs): %.1f .. %.1f us "
           "(relative to the first start)\n",
           tile_grid, 0.01 * (h0 - std::min(h0, g0)), 0.01 * (h1 - std::min(h0, g0)), sm_blocks,
           0.01 * (g0 - std::min(h0, g0)), 0.01 * (g1 - std::min(h0, g0)));
    printf("%s\n", g1 < h1 && g0 < h1 ? "OVERLAP: the chain-side kernel ran beside the persistent one"
                                      : "NO OVERLAP");
    return 0;
}
