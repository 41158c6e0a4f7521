// Dependent-load latency by access spread (diagnostic for the lane-per-stream chain).
// Every lane walks a chain of `iters` dependent 16-byte loads; lane g of the grid reads at
// base + (g * lane_stride + k * step) mod size, the next address depending on the loaded value
// (the buffer is zero, so the offsets do not change, but each load waits for the last).
//   lane_stride 16      : a wave reads one 1 KiB run            (one page per wave)
//   lane_stride 1 MiB   : every lane a different MiB             (the lane chain on 1 MiB streams)
//   lane_stride 64 KiB  : lanes 64 KiB apart                      (records of 64 streams)
// Prints ns per dependent load (s_memrealtime, 100 MHz) for 1024 waves (one per SIMD).
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__global__ void chase(const uint8_t *base, uint64_t size, uint64_t lane_stride, uint64_t step,
                      int iters, uint64_t *out) {
    const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint64_t off = (g * lane_stride) % size;
    uint32_t acc = 0;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    for (int k = 0; k < iters; ++k) {
        const u32x4 v = *reinterpret_cast<const u32x4 *>(base + (off & ~15ull));
        acc += v.x;
        off = (off + step + v.x) % size;
    }
    const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
    if ((threadIdx.x & 63) == 0) out[g / 64] = t1 - t0;
    if (acc == 12345) out[1 << 20] = acc;
}

int main() {
    const uint64_t size = 16ull << 30;
    uint8_t *buf;
    uint64_t *out;
    if (hipMalloc(&buf, size) != hipSuccess || hipMalloc(&out, (2 << 20) * 8) != hipSuccess) return 1;
    (void)hipMemset(buf, 0, size);
    const int iters = 200;
    const uint64_t strides[] = {16, 4096, 65536, 1 << 20, 4 << 20};
    const uint64_t steps[] = {80000, 1 << 20};
    static uint64_t h[1024];
    for (uint64_t step : steps)
        for (uint64_t st : strides) {
            for (int rep = 0; rep < 2; ++rep) {
                hipLaunchKernelGGL(chase, dim3(256), dim3(256), 0, 0, buf, size, st, step, iters, out);
                (void)hipDeviceSynchronize();
            }
            (void)hipMemcpy(h, out, sizeof h, hipMemcpyDeviceToHost);
            double s = 0;
            for (int w = 0; w < 1024; ++w) s += h[w];
            printf("lane_stride %8llu step %8llu: %.0f ns per dependent 16-B load\n",
                   (unsigned long long)st, (unsigned long long)step, s / 1024 * 10.0 / iters);
        }
    return 0;
}
