// VALU issue/latency microbenchmark for gfx950 (the instructions the BLAKE2b quad kernel uses).
// For each instruction: 8 independent chains (throughput) and 1 dependent chain (latency),
// 1 and 2 waves per SIMD.  Cycles from s_memtime (core clock), wall from s_memrealtime (100 MHz).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define REP8(x) x x x x x x x x
#define REP64(x) REP8(REP8(x))

template <int OP, bool DEP>
__global__ void kern(uint64_t *out, int iters) {
    uint64_t t0 = __builtin_amdgcn_s_memtime();
    uint64_t r0 = __builtin_amdgcn_s_memrealtime();
    uint64_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5,
             a6 = a0 + 6, a7 = a0 + 7, b = a0 * 3;
    for (int i = 0; i < iters; ++i) {
        if constexpr (OP == 0) {  // v_lshl_add_u64
            if constexpr (DEP) { REP64(asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(a0) : "v"(b));) }
            else { REP8(asm volatile("v_lshl_add_u64 %0, %0, 0, %8\n v_lshl_add_u64 %1, %1, 0, %8\n v_lshl_add_u64 %2, %2, 0, %8\n v_lshl_add_u64 %3, %3, 0, %8\n v_lshl_add_u64 %4, %4, 0, %8\n v_lshl_add_u64 %5, %5, 0, %8\n v_lshl_add_u64 %6, %6, 0, %8\n v_lshl_add_u64 %7, %7, 0, %8" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b));) }
        } else if constexpr (OP == 1) {  // v_xor_b32
            uint32_t x0 = a0, x1 = a1, x2 = a2, x3 = a3, x4 = a4, x5 = a5, x6 = a6, x7 = a7, y = b;
            if constexpr (DEP) { REP64(asm volatile("v_xor_b32 %0, %0, %1" : "+v"(x0) : "v"(y));) }
            else { REP8(asm volatile("v_xor_b32 %0, %0, %8\n v_xor_b32 %1, %1, %8\n v_xor_b32 %2, %2, %8\n v_xor_b32 %3, %3, %8\n v_xor_b32 %4, %4, %8\n v_xor_b32 %5, %5, %8\n v_xor_b32 %6, %6, %8\n v_xor_b32 %7, %7, %8" : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3), "+v"(x4), "+v"(x5), "+v"(x6), "+v"(x7) : "v"(y));) }
            a0 = x0 ^ x1 ^ x2 ^ x3 ^ x4 ^ x5 ^ x6 ^ x7;
        } else if constexpr (OP == 2) {  // v_alignbit_b32
            uint32_t x0 = a0, x1 = a1, x2 = a2, x3 = a3, x4 = a4, x5 = a5, x6 = a6, x7 = a7, y = b;
            if constexpr (DEP) { REP64(asm volatile("v_alignbit_b32 %0, %0, %1, 24" : "+v"(x0) : "v"(y));) }
            else { REP8(asm volatile("v_alignbit_b32 %0, %0, %8, 24\n v_alignbit_b32 %1, %1, %8, 24\n v_alignbit_b32 %2, %2, %8, 24\n v_alignbit_b32 %3, %3, %8, 24\n v_alignbit_b32 %4, %4, %8, 24\n v_alignbit_b32 %5, %5, %8, 24\n v_alignbit_b32 %6, %6, %8, 24\n v_alignbit_b32 %7, %7, %8, 24" : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3), "+v"(x4), "+v"(x5), "+v"(x6), "+v"(x7) : "v"(y));) }
            a0 = x0 ^ x1 ^ x2 ^ x3 ^ x4 ^ x5 ^ x6 ^ x7;
        } else if constexpr (OP == 3) {  // v_mov_b32_dpp quad_perm
            uint32_t x0 = a0, x1 = a1, x2 = a2, x3 = a3, x4 = a4, x5 = a5, x6 = a6, x7 = a7;
            if constexpr (DEP) { REP64(asm volatile("s_nop 1\n v_mov_b32_dpp %0, %0 quad_perm:[1,2,3,0] row_mask:0xf bank_mask:0xf" : "+v"(x0));) }
            else { REP8(asm volatile("v_mov_b32_dpp %0, %0 quad_perm:[1,2,3,0] row_mask:0xf bank_mask:0xf\n v_mov_b32_dpp %1, %1 quad_perm:[1,2,3,0] row_mask:0xf bank_mask:0xf\n v_mov_b32_dpp %2, %2 quad_perm:[1,2,3,0] row_mask:0xf bank_mask:0xf\n v_mov_b32_dpp %3, %3 quad_perm:[1,2,3,0] row_mask:0xf bank_mask:0xf\n v_mov_b32_dpp %4, %4 quad_perm:[1,2,3,0] row_mask:0xf bank_mask:0xf\n v_mov_b32_dpp %5, %5 quad_perm:[1,2,3,0] row_mask:0xf bank_mask:0xf\n v_mov_b32_dpp %6, %6 quad_perm:[1,2,3,0] row_mask:0xf bank_mask:0xf\n v_mov_b32_dpp %7, %7 quad_perm:[1,2,3,0] row_mask:0xf bank_mask:0xf" : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3), "+v"(x4), "+v"(x5), "+v"(x6), "+v"(x7));) }
            a0 = x0 ^ x1 ^ x2 ^ x3 ^ x4 ^ x5 ^ x6 ^ x7;
        } else if constexpr (OP == 4) {  // v_add_co_u32 + v_addc_co_u32 (64-bit add in 2)
            uint32_t l0 = a0, h0 = a0 >> 7, l1 = a1, h1 = a1 >> 3, l2 = a2, h2 = 5, l3 = a3, h3 = 9, y = b, z = b >> 5;
            if constexpr (DEP) { REP64(asm volatile("v_add_co_u32 %0, vcc, %0, %2\n v_addc_co_u32 %1, vcc, %1, %3, vcc" : "+v"(l0), "+v"(h0) : "v"(y), "v"(z) : "vcc");) }
            else { REP8(asm volatile("v_add_co_u32 %0, vcc, %0, %8\n v_addc_co_u32 %1, vcc, %1, %9, vcc\n v_add_co_u32 %2, vcc, %2, %8\n v_addc_co_u32 %3, vcc, %3, %9, vcc\n v_add_co_u32 %4, vcc, %4, %8\n v_addc_co_u32 %5, vcc, %5, %9, vcc\n v_add_co_u32 %6, vcc, %6, %8\n v_addc_co_u32 %7, vcc, %7, %9, vcc" : "+v"(l0), "+v"(h0), "+v"(l1), "+v"(h1), "+v"(l2), "+v"(h2), "+v"(l3), "+v"(h3) : "v"(y), "v"(z) : "vcc");) }
            a0 = l0 ^ h0 ^ l1 ^ h1 ^ l2 ^ h2 ^ l3 ^ h3;
        } else if constexpr (OP == 5) {  // v_xor3_b32
            uint32_t x0 = a0, x1 = a1, x2 = a2, x3 = a3, x4 = a4, x5 = a5, x6 = a6, x7 = a7, y = b;
            if constexpr (DEP) { REP64(asm volatile("v_xad_u32 %0, %0, %1, %1" : "+v"(x0) : "v"(y));) }
            else { REP8(asm volatile("v_xad_u32 %0, %0, %8, %8\n v_xad_u32 %1, %1, %8, %8\n v_xad_u32 %2, %2, %8, %8\n v_xad_u32 %3, %3, %8, %8\n v_xad_u32 %4, %4, %8, %8\n v_xad_u32 %5, %5, %8, %8\n v_xad_u32 %6, %6, %8, %8\n v_xad_u32 %7, %7, %8, %8" : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3), "+v"(x4), "+v"(x5), "+v"(x6), "+v"(x7) : "v"(y));) }
            a0 = x0 ^ x1 ^ x2 ^ x3 ^ x4 ^ x5 ^ x6 ^ x7;
        } else if constexpr (OP == 6) {  // v_pk_add_u32? not on gfx950: use v_add3_u32
            uint32_t x0 = a0, x1 = a1, x2 = a2, x3 = a3, x4 = a4, x5 = a5, x6 = a6, x7 = a7, y = b;
            if constexpr (DEP) { REP64(asm volatile("v_add3_u32 %0, %0, %1, %1" : "+v"(x0) : "v"(y));) }
            else { REP8(asm volatile("v_add3_u32 %0, %0, %8, %8\n v_add3_u32 %1, %1, %8, %8\n v_add3_u32 %2, %2, %8, %8\n v_add3_u32 %3, %3, %8, %8\n v_add3_u32 %4, %4, %8, %8\n v_add3_u32 %5, %5, %8, %8\n v_add3_u32 %6, %6, %8, %8\n v_add3_u32 %7, %7, %8, %8" : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3), "+v"(x4), "+v"(x5), "+v"(x6), "+v"(x7) : "v"(y));) }
            a0 = x0 ^ x1 ^ x2 ^ x3 ^ x4 ^ x5 ^ x6 ^ x7;
        } else if constexpr (OP == 7) {  // v_mov_b64 (64-bit move)
            if constexpr (DEP) { REP64(asm volatile("v_mov_b64 %0, %1\n" : "=v"(a0) : "v"(a0));) }
            else { REP8(asm volatile("v_mov_b64 %0, %4\n v_mov_b64 %1, %4\n v_mov_b64 %2, %4\n v_mov_b64 %3, %4\n v_mov_b64 %0, %4\n v_mov_b64 %1, %4\n v_mov_b64 %2, %4\n v_mov_b64 %3, %4" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3) : "v"(b));) }
        }
    }
    uint64_t t1 = __builtin_amdgcn_s_memtime();
    uint64_t r1 = __builtin_amdgcn_s_memrealtime();
    if ((threadIdx.x & 63) == 0) {
        out[(blockIdx.x * blockDim.x + threadIdx.x) / 64 * 2] = t1 - t0;
        out[(blockIdx.x * blockDim.x + threadIdx.x) / 64 * 2 + 1] = r1 - r0;
    }
    if (a0 == 12345 && a1 == 7) out[1 << 20] = a2 + a3 + a4 + a5 + a6 + a7;
}

template <int OP, bool DEP>
void run(const char *name, uint64_t *d, int threads) {
    const int iters = 2000;
    kern<OP, DEP><<<256, threads>>>(d, iters);
    hipDeviceSynchronize();
    kern<OP, DEP><<<256, threads>>>(d, iters);
    hipDeviceSynchronize();
    uint64_t h[2];
    hipMemcpy(h, d, 16, hipMemcpyDeviceToHost);
    const double instrs = 64.0 * iters * (OP == 4 ? 2 : 1);
    printf("%-22s %-4s waves/SIMD=%d  cycles/instr(per wave)=%.2f  clock=%.2f GHz\n", name,
           DEP ? "dep" : "ind", threads / 256, h[0] / instrs, h[0] / (h[1] * 10.0));
}

int main() {
    uint64_t *d;
    hipMalloc(&d, (2 << 20) * 8);
    for (int th : {256, 512}) {
        run<0, false>("v_lshl_add_u64", d, th);
        run<0, true>("v_lshl_add_u64", d, th);
        run<1, false>("v_xor_b32", d, th);
        run<1, true>("v_xor_b32", d, th);
        run<2, false>("v_alignbit_b32", d, th);
        run<2, true>("v_alignbit_b32", d, th);
        run<3, false>("v_mov_b32_dpp", d, th);
        run<3, true>("v_mov_b32_dpp+s_nop1", d, th);
        run<4, false>("v_add_co+v_addc", d, th);
        run<4, true>("v_add_co+v_addc", d, th);
        run<5, false>("v_xad_u32", d, th);
        run<5, true>("v_xad_u32", d, th);
        run<6, false>("v_add3_u32", d, th);
        run<6, true>("v_add3_u32", d, th);
        run<7, false>("v_mov_b64", d, th);
        run<7, true>("v_mov_b64", d, th);
    }
    return 0;
}
