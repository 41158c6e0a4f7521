// Cache policy of the tile ring's loads: the tile kernel's streaming pattern (persistent
// 1024-thread workgroups, one per CU; each wave a contiguous share of 16 KiB tiles, read through a
// 16-slot register ring of 16-byte buffer loads, each slot re-issued for the next tile as it is
// consumed) with every cache-policy bit combination of the buffer load (gfx950: sc0 = 1, nt = 2,
// sc1 = 16), over a 64 GiB arena.  The product uses nt (kernels.hip kStreamAux = 2).
// Then the ring's depth against the waves per CU at the product's policy: W waves per CU, each
// with S 1 KiB slots in flight (the product: 16 waves x 16 slots, 256 KiB per CU).
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/ubench/ring_policy.hip -o diag/ring_policy
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// S slots of 1 KiB per wave (a "tile" of S KiB), W waves per workgroup, one workgroup per CU
template <int AUX, int S = 16, int W = 16>
__global__ __launch_bounds__(W * 64) void ring(const uint8_t *__restrict__ a, uint64_t n_kib,
                                               uint32_t *__restrict__ out) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t n_tiles = n_kib / S;
    const uint64_t nw = (uint64_t)gridDim.x * W;
    const uint64_t gw = (uint64_t)blockIdx.x * W + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t per = (n_tiles + nw - 1) / nw;
    const uint64_t t0 = gw * per, t1 = std::min(n_tiles, t0 + per);
    if (t0 >= t1) return;
    u32x4 x[S];
    __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint8_t *>(a + t0 * S * 1024), 0, 0xffffffffu, 0x00020000);
#pragma unroll
    for (int it = 0; it < S; ++it) {
        x[it] = __builtin_amdgcn_raw_buffer_load_b128(r, lane * 16, it * 1024, AUX);
        __builtin_amdgcn_sched_barrier(0);
    }
    uint32_t acc = 0;
    for (uint64_t t = t0; t < t1; ++t) {
        const uint64_t tn = t + 1 < t1 ? t + 1 : t;
        const __amdgpu_buffer_rsrc_t rn = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<uint8_t *>(a + tn * S * 1024), 0, 0xffffffffu, 0x00020000);
#pragma unroll
        for (int it = 0; it < S; ++it) {
            const u32x4 w = x[it];
            acc ^= w.x ^ w.y ^ w.z ^ w.w;
            x[it] = __builtin_amdgcn_raw_buffer_load_b128(rn, lane * 16, it * 1024, AUX);
        }
    }
#pragma unroll
    for (int it = 0; it < S; ++it) acc ^= x[it].x;
    out[(uint64_t)blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

typedef void (*Kern)(const uint8_t *, uint64_t, uint32_t *);

int main() {
    const uint64_t bytes = 64ull << 30, n_kib = bytes / 1024;
    uint8_t *a;
    uint32_t *out;
    if (hipMalloc(&a, bytes) != hipSuccess || hipMalloc(&out, 16ull << 20) != hipSuccess) {
        printf("alloc failed\n");
        return 1;
    }
    if (hipMemset(a, 0x5a, bytes) != hipSuccess) return 1;
    int cus = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    struct V {
        const char *name;
        Kern k;
        int waves;
    };
    const V vs[] = {{"plain", ring<0>, 16}, {"sc0", ring<1>, 16}, {"nt (product)", ring<2>, 16},
                    {"sc0 nt", ring<3>, 16}, {"sc1", ring<16>, 16}, {"sc0 sc1", ring<17>, 16},
                    {"nt sc1", ring<18>, 16}, {"sc0 nt sc1", ring<19>, 16},
                    {"nt W8 S32", ring<2, 32, 8>, 8}, {"nt W8 S16", ring<2, 16, 8>, 8},
                    {"nt W16 S8", ring<2, 8, 16>, 16}, {"nt W4 S64", ring<2, 64, 4>, 4},
                    {"nt W12 S16", ring<2, 16, 12>, 12}, {"nt W16 S24", ring<2, 24, 16>, 16}};
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    printf("CUs %d, arena %.1f GB\n", cus, bytes / 1e9);
    std::vector<std::vector<float>> ms(sizeof vs / sizeof vs[0]);
    for (int round = 0; round < 4; ++round) {  // variants interleaved, round after round
        for (size_t i = 0; i < sizeof vs / sizeof vs[0]; ++i) {
            for (int r = 0; r < 3; ++r) {
                (void)hipEventRecord(e0, 0);
                hipLaunchKernelGGL(vs[i].k, dim3(cus), dim3(vs[i].waves * 64), 0, 0, a, n_kib, out);
                (void)hipEventRecord(e1, 0);
                if (hipEventSynchronize(e1) != hipSuccess) {
                    printf("%s: launch failed\n", vs[i].name);
                    return 1;
                }
                float t = 0;
                (void)hipEventElapsedTime(&t, e0, e1);
                if (r > 0) ms[i].push_back(t);
            }
        }
    }
    for (size_t i = 0; i < sizeof vs / sizeof vs[0]; ++i) {
        std::sort(ms[i].begin(), ms[i].end());
        printf("%-14s best %.3f ms %.0f GB/s, median %.3f ms %.0f GB/s\n", vs[i].name, ms[i].front(),
               bytes / ms[i].front() / 1e6, ms[i][ms[i].size() / 2], bytes / ms[i][ms[i].size() / 2] / 1e6);
    }
    return 0;
}
