// Streaming-read ceiling of one MI355X over a 64 GiB arena (the config-2 footprint), with the
// simplest load patterns, to place rc_read_probe_kernel (the tile kernel's own pattern) against
// them.  Every variant XOR-folds the 16-byte loads it issues and writes one word per thread, so
// nothing is optimised away; 6 timed launches after 2 warm-up ones, hipEvent timing.
//
//   gs<T, U, NT>   grid-stride: T threads per block, 8 blocks' worth of waves per CU, U independent
//                  16-byte loads in flight per thread per iteration; NT: nontemporal loads
//   ch<T, U, NT>   contiguous: block b reads its own 1/grid of the arena, U loads per iteration
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/ubench/read_ceiling.hip -o diag/read_ceiling
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <bool NT>
__device__ __forceinline__ u32x4 ld(const u32x4 *p) {
    if constexpr (NT) return __builtin_nontemporal_load(p);
    return *p;
}

template <int U, bool NT>
__global__ void gs(const u32x4 *__restrict__ a, uint64_t n, uint32_t *__restrict__ out) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t acc = 0;
    for (; i + (U - 1) * stride < n; i += U * stride) {
        u32x4 v[U];
#pragma unroll
        for (int k = 0; k < U; ++k) v[k] = ld<NT>(a + i + k * stride);
#pragma unroll
        for (int k = 0; k < U; ++k) acc ^= v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
    }
    for (; i < n; i += stride) {
        const u32x4 v = ld<NT>(a + i);
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    out[(uint64_t)blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

template <int U, bool NT>
__global__ void ch(const u32x4 *__restrict__ a, uint64_t n, uint32_t *__restrict__ out) {
    const uint64_t per = (n + gridDim.x - 1) / gridDim.x;
    const uint64_t b = (uint64_t)blockIdx.x * per, e = std::min(n, b + per);
    uint32_t acc = 0;
    uint64_t i = b + threadIdx.x;
    for (; i + (U - 1) * blockDim.x < e; i += (uint64_t)U * blockDim.x) {
        u32x4 v[U];
#pragma unroll
        for (int k = 0; k < U; ++k) v[k] = ld<NT>(a + i + k * blockDim.x);
#pragma unroll
        for (int k = 0; k < U; ++k) acc ^= v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
    }
    for (; i < e; i += blockDim.x) {
        const u32x4 v = ld<NT>(a + i);
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    out[(uint64_t)blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

typedef void (*Kern)(const u32x4 *, uint64_t, uint32_t *);

int main() {
    const uint64_t bytes = 64ull << 30, n = bytes / 16;
    u32x4 *a;
    uint32_t *out;
    if (hipMalloc(&a, bytes) != hipSuccess || hipMalloc(&out, 64ull << 20) != hipSuccess) {
        printf("alloc failed\n");
        return 1;
    }
    if (hipMemset(a, 0x5a, bytes) != hipSuccess) return 1;
    int cus = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    struct V {
        const char *name;
        Kern k;
        int threads, blocks_per_cu;
    };
    const V vs[] = {
        {"gs T256 U4 nt", gs<4, true>, 256, 8},   {"gs T256 U8 nt", gs<8, true>, 256, 8},
        {"gs T256 U8 plain", gs<8, false>, 256, 8}, {"gs T256 U16 nt", gs<16, true>, 256, 8},
        {"gs T1024 U8 nt", gs<8, true>, 1024, 2}, {"gs T512 U8 nt", gs<8, true>, 512, 4},
        {"gs T256 U8 nt x16", gs<8, true>, 256, 16},
        {"ch T1024 U16 nt", ch<16, true>, 1024, 1}, {"ch T256 U16 nt", ch<16, true>, 256, 4},
        {"ch T256 U8 nt x8", ch<8, true>, 256, 8}, {"ch T256 U16 plain", ch<16, false>, 256, 4},
    };
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    printf("CUs %d, arena %.1f GB\n", cus, bytes / 1e9);
    for (const V &v : vs) {
        const int grid = cus * v.blocks_per_cu;
        std::vector<float> ms;
        for (int r = 0; r < 8; ++r) {
            (void)hipEventRecord(e0, 0);
            hipLaunchKernelGGL(v.k, dim3(grid), dim3(v.threads), 0, 0, a, n, out);
            (void)hipEventRecord(e1, 0);
            if (hipEventSynchronize(e1) != hipSuccess) {
                printf("%s: launch failed\n", v.name);
                return 1;
            }
            float t = 0;
            (void)hipEventElapsedTime(&t, e0, e1);
            if (r >= 2) ms.push_back(t);
        }
        std::sort(ms.begin(), ms.end());
        printf("%-20s grid %6d: best %.3f ms %.0f GB/s, median %.3f ms %.0f GB/s\n", v.name, grid,
               ms.front(), bytes / ms.front() / 1e6, ms[ms.size() / 2], bytes / ms[ms.size() / 2] / 1e6);
        fflush(stdout);
    }
    return 0;
}
