// diag.h -- the diagnostic builds' instrumentation of kernels.hip, as one macro layer.
//
// The product library defines none of the RC_DIAG_* / RC_PLAIN_LOADS macros: everything below
// then expands to nothing (or to the product's choice), and the kernels carry no diagnostic code
// and no #ifdef.  A diagnostic library is a separate build under diag/ loaded through
// RC_LIB_PATH by the measurement scripts only:
//     python -m replicat_amd.build --variant STAMPS -DRC_DIAG_STAMPS          (chain stamps)
//     python -m replicat_amd.build --variant TSTAMPS -DRC_DIAG_TILE_STAMPS    (tile-kernel waves)
//     python -m replicat_amd.build --variant PLAIN -DRC_PLAIN_LOADS           (cache policy A/B)
// (scripts/diag_stamps.py, scripts/tile_stamps.py read the stamps back.)
#pragma once

// ---- streamed-byte cache policy: nontemporal (the product) or the default policy
#ifdef RC_PLAIN_LOADS
#define RC_STREAM_LOAD(p) (*(p))
#define RC_DIAG_STREAM_AUX 0
#else
#define RC_STREAM_LOAD(p) __builtin_nontemporal_load(p)
#define RC_DIAG_STREAM_AUX 2  // nt
#endif

// ---- the tile scan's 16 lookups per slice: issued together behind a scheduling fence (the
// product), or in the compiler's own order (-DRC_DIAG_NO_SLICE_FENCE, the round-4 code)
#ifdef RC_DIAG_NO_SLICE_FENCE
#define RC_DIAG_SLICE_FENCE false
#else
#define RC_DIAG_SLICE_FENCE true
#endif

// ---- a forced fail-safe stop of the tile kernel (-DRC_DIAG_GRAB_FAULT, diag/lib_GRABFAULT.so):
// wave 1 of workgroup 0 stops at its first workgroup grab -- the unit it took is never run --
// and sets the fail-safe flag, as a wave whose slot was never published would (UnitGrab::next).
// Every launch with tiles faults; tests/test_gpu_fault.py checks that every product surface
// reports it instead of returning cuts.
#ifdef RC_DIAG_GRAB_FAULT
#define RC_DIAG_FORCE_GRAB_STOP() (blockIdx.x == 0 && (threadIdx.x >> 6) == 1)
#else
#define RC_DIAG_FORCE_GRAB_STOP() false
#endif

// ---- per-wave stamps of the tile kernel: s_memrealtime (100 MHz) when a wave's first tile
// starts and when its last record is stored, and its tile count
#ifdef RC_DIAG_TILE_STAMPS
__device__ uint64_t g_tile_stamp[3 * 8192];
#define RC_TILE_STAMP_BEGIN()                                                   \
    const uint64_t diag_stamp0_ = __builtin_amdgcn_s_memrealtime();             \
    uint64_t diag_done_ = 0
#define RC_TILE_STAMP_TILE() (++diag_done_)
#define RC_TILE_STAMP_END(gw)                                                   \
    do {                                                                        \
        if ((gw) < 8192) {                                                      \
            g_tile_stamp[3 * (gw)] = diag_stamp0_;                              \
            g_tile_stamp[3 * (gw) + 1] = __builtin_amdgcn_s_memrealtime();      \
            g_tile_stamp[3 * (gw) + 2] = diag_done_;                            \
        }                                                                       \
    } while (0)
extern "C" int rc_diag_tile_read(uint64_t *out, uint32_t waves) {
    if (waves > 8192) waves = 8192;
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_tile_stamp), 3 * 8 * (size_t)waves) != hipSuccess) return 1;
    static uint64_t zero[3 * 8192];
    return hipMemcpyToSymbol(HIP_SYMBOL(g_tile_stamp), zero, sizeof zero) != hipSuccess;
}
#else
#define RC_TILE_STAMP_BEGIN() \
    do {                      \
    } while (0)
#define RC_TILE_STAMP_TILE() \
    do {                     \
    } while (0)
#define RC_TILE_STAMP_END(gw) \
    do {                      \
    } while (0)
#endif

// ---- per-step stamps of one chain walker (stream 0's): RC_STAMP inside chain_step (its
// ChainStream `st` carries the diag flag), RC_LSTAMP in the lane / quad chains (a local `diag`)
#ifdef RC_DIAG_STAMPS
#define RC_DIAG_ONLY(...) __VA_ARGS__
__device__ uint64_t g_diag[4096];
__device__ uint32_t g_diag_n;
#define RC_STAMP(tag)                                                                      \
    do {                                                                                   \
        if (st.diag && (threadIdx.x & 63) == 0 && g_diag_n < 4000) {                       \
            g_diag[g_diag_n++] = ((uint64_t)(tag) << 56) | __builtin_amdgcn_s_memrealtime(); \
        }                                                                                  \
    } while (0)
#define RC_LSTAMP(tag)                                                                     \
    do {                                                                                   \
        if (diag && (threadIdx.x & 63) == 0 && g_diag_n < 4000) {                          \
            g_diag[g_diag_n++] = ((uint64_t)(tag) << 56) | __builtin_amdgcn_s_memrealtime(); \
        }                                                                                  \
    } while (0)
extern "C" int rc_diag_read(uint64_t *out, uint32_t cap, uint32_t *n) {
    uint32_t k = 0;
    if (hipMemcpyFromSymbol(&k, HIP_SYMBOL(g_diag_n), 4) != hipSuccess) return 1;
    if (k > cap) k = cap;
    if (k && hipMemcpyFromSymbol(out, HIP_SYMBOL(g_diag), k * 8) != hipSuccess) return 1;
    *n = k;
    const uint32_t z = 0;
    return hipMemcpyToSymbol(HIP_SYMBOL(g_diag_n), &z, 4) != hipSuccess;
}
#else
#define RC_DIAG_ONLY(...)
#define RC_STAMP(tag) \
    do {              \
    } while (0)
#define RC_LSTAMP(tag) \
    do {               \
    } while (0)
#endif
