// kernels.hip -- gfx950 kernels of the content-defined chunker.
//
// Replaces the scan of /root/reference/src/adapters.cpp:42-77 (next_cut's argmax over key())
// with two launches per batch of streams:
//
//   phase A  tile kernel   (HBM-bound, one pass over every input byte)
//            Every wave owns 4096-key tiles (16 KiB of stream) and reduces each to one
//            TileRecord = (first maximal 64-bit key, its index).  Bytes stream straight from
//            HBM into registers with coalesced 16-byte loads (1 KiB per wave instruction).
//            Per key it evaluates only the top 16 bits of the hash: 4 conflict-free LDS
//            lookups per 32-bit word (replicated prefilter tables, see gclmul.h) + DPP for the
//            neighbour word.  Each lane keeps the first and the last index of its largest
//            top-16 value; the exact 64-bit key is computed once per lane, the wave reduces
//            (key desc, index asc).  A lane whose top-16 maximum occurs twice and could be the
//            tile maximum sends the tile down the exact path (rare on random data).
//
//   phase B  chain kernel  (latency-bound, tiny)
//            One wave per stream walks the cut chain exactly as replicat's adapter loop does
//            (tail rules of adapters.cpp:48-57 under the piece framing of adapters.py:290-305):
//            the argmax window [s+4, s+max) is the maximum over the tile records fully inside
//            it plus the exact keys of the two partial edge tiles.
//
// No MFMA anywhere: this is integer byte work.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "gclmul.h"

using namespace rc;

namespace {

thread_local char g_launch_err[256];

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t lane_id() { return threadIdx.x & 63; }

__device__ __forceinline__ uint32_t ld_u32(const uint8_t *p) {
    return *reinterpret_cast<const uint32_t *>(p);
}

// Exact 64-bit key of (w[j-1], w[j]) from the byte tables (gclmul.h), k1 included.
__device__ __forceinline__ uint64_t full_key(const uint64_t *__restrict__ tl,
                                             const uint64_t *__restrict__ th, uint32_t wlo,
                                             uint32_t whi) {
    return tl[wlo & 255] ^ tl[256 + ((wlo >> 8) & 255)] ^ tl[512 + ((wlo >> 16) & 255)] ^
           tl[768 + (wlo >> 24)] ^ th[whi & 255] ^ th[256 + ((whi >> 8) & 255)] ^
           th[512 + ((whi >> 16) & 255)] ^ th[768 + (whi >> 24)];
}

__device__ __forceinline__ uint64_t key_at(const uint64_t *tl, const uint64_t *th,
                                           const uint8_t *base, uint64_t j) {
    const uint8_t *p = base + 4 * j;
    return full_key(tl, th, ld_u32(p - 4), ld_u32(p));
}

// (key desc, index asc) maximum over the wave; every lane gets the result.
__device__ __forceinline__ void wave_best(uint64_t &k, uint64_t &j) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        const uint64_t ko = __shfl_xor(k, off);
        const uint64_t jo = __shfl_xor(j, off);
        if (ko > k || (ko == k && jo < j)) {
            k = ko;
            j = jo;
        }
    }
}

// ------------------------------------------------------------------ phase A: tile kernel

__shared__ __attribute__((aligned(16))) uint32_t s_tile_lds[kTileLdsBytes / 4];

__device__ __forceinline__ uint32_t pf_lds(uint32_t byte_addr) {
    return *reinterpret_cast<const uint32_t *>(reinterpret_cast<const char *>(s_tile_lds) +
                                               byte_addr);
}

// 32-bit prefilter entry of a word: top16(Lmap(w)) << 16 | top16(Hmap(w)).
// v_perm builds each table address (v << 8 | lane's bank column | table half) in one op.
__device__ __forceinline__ uint32_t pf_entry(uint32_t w, uint32_t lb_a, uint32_t lb_b) {
    const uint32_t a0 = __builtin_amdgcn_perm(w, lb_a, 0x0c020400u);
    const uint32_t a1 = __builtin_amdgcn_perm(w, lb_a, 0x0c020500u);
    const uint32_t a2 = __builtin_amdgcn_perm(w, lb_b, 0x0c020600u);
    const uint32_t a3 = __builtin_amdgcn_perm(w, lb_b, 0x0c020700u);
    return pf_lds(a0) ^ pf_lds(a1 + 128) ^ pf_lds(a2) ^ pf_lds(a3 + 128);
}

// Exact per-key path over keys [ja, jb] of the tile starting at key j0 (edge tiles, tie
// fallback, unaligned streams).  Same key -> lane mapping as the fast path.
__device__ void tile_exact(const uint64_t *tl, const uint64_t *th, const uint8_t *base,
                           uint64_t j0, uint64_t ja, uint64_t jb, uint64_t &bk, uint64_t &bj) {
    const uint32_t lane = lane_id();
    bk = 0;
    bj = ~0ull;
    for (int m = 0; m < 64; ++m) {
        const uint64_t j = j0 + (uint64_t)(m >> 2) * 256 + lane * 4 + (m & 3);
        if (j >= ja && j <= jb) {
            const uint64_t k = key_at(tl, th, base, j);
            if (k > bk) {
                bk = k;
                bj = j;
            }
        }
    }
    wave_best(bk, bj);
}

__device__ __forceinline__ void tile_fast(const uint64_t *tl, const uint64_t *th,
                                          const uint8_t *base, uint64_t j0, uint32_t lb_a,
                                          uint32_t lb_b, uint64_t &bk, uint64_t &bj) {
    const uint32_t lane = lane_id();
    const u32x4 *src = reinterpret_cast<const u32x4 *>(base + 4 * j0);
    u32x4 x[kTileIters];
#pragma unroll
    for (int it = 0; it < kTileIters; ++it) x[it] = __builtin_nontemporal_load(src + it * 64 + lane);

    uint32_t carry = pf_entry(ld_u32(base + 4 * j0 - 4), lb_a, lb_b);
    uint32_t acc_first = 0, acc_last = 0;
#pragma unroll
    for (int it = 0; it < kTileIters; ++it) {
        const uint32_t e0 = pf_entry(x[it].x, lb_a, lb_b);
        const uint32_t e1 = pf_entry(x[it].y, lb_a, lb_b);
        const uint32_t e2 = pf_entry(x[it].z, lb_a, lb_b);
        const uint32_t e3 = pf_entry(x[it].w, lb_a, lb_b);
        // previous word's entry for key 0 of this lane: lane-1's e3 (wave_ror:1); lane 0 takes
        // the carry = lane 63's e3 of the previous iteration (or the word before the tile).
        const uint32_t rot = __builtin_amdgcn_update_dpp(0u, e3, 0x13C, 0xf, 0xf, false);
        const uint32_t ep = lane == 0 ? carry : rot;
        carry = rot;
        const uint32_t b0 = (ep & 0xffff0000u) ^ (e0 << 16);
        const uint32_t b1 = (e0 & 0xffff0000u) ^ (e1 << 16);
        const uint32_t b2 = (e1 & 0xffff0000u) ^ (e2 << 16);
        const uint32_t b3 = (e2 & 0xffff0000u) ^ (e3 << 16);
        // local key index l = 4*it + k;  "first" packs 63 - l, "last" packs l
        const uint32_t inv = 60u - 4u * it, idx = 4u * it;
        acc_first = max(acc_first, max(b0 | inv | 3u, b1 | inv | 2u));
        acc_first = max(acc_first, max(b2 | inv | 1u, b3 | inv));
        acc_last = max(acc_last, max(b0 | idx, b1 | idx | 1u));
        acc_last = max(acc_last, max(b2 | idx | 2u, b3 | idx | 3u));
    }
    const uint32_t top = acc_first >> 16;
    const uint32_t first = 63u - (acc_first & 0xffffu);
    const uint32_t last = acc_last & 0xffffu;
    const uint64_t j = j0 + (uint64_t)(first >> 2) * 256 + lane * 4 + (first & 3);
    bk = key_at(tl, th, base, j);
    bj = j;
    wave_best(bk, bj);
    const bool tie = top == (uint32_t)(bk >> 48) && first != last;
    if (__any(tie)) tile_exact(tl, th, base, j0, j0, j0 + kTileKeys - 1, bk, bj);
}

__global__ __launch_bounds__(1024) void rc_tile_kernel(const KeyTables *__restrict__ tab,
                                                       StreamDesc d, uint64_t n_streams,
                                                       uint64_t n_tiles,
                                                       TileRecord *__restrict__ rec) {
    // stage the replicated prefilter tables and the exact tables into LDS
    for (uint32_t i = threadIdx.x; i < 1024u * 32u; i += blockDim.x) {
        const uint32_t e = i >> 5, c = i & 31, b = e >> 8, v = e & 255;
        s_tile_lds[((b >> 1) * 65536u + v * 256u + (b & 1) * 128u) / 4 + c] = tab->pf[b][v];
    }
    uint64_t *full = reinterpret_cast<uint64_t *>(s_tile_lds + kFullOff / 4);
    const uint64_t *gfull = &tab->tl[0][0];
    for (uint32_t i = threadIdx.x; i < 2048u; i += blockDim.x) full[i] = gfull[i];
    __syncthreads();
    const uint64_t *tl = full, *th = full + 1024;

    const uint32_t lane = lane_id();
    const uint32_t lb_a = (lane & 31) * 4, lb_b = lb_a | 0x10000u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t gw = (uint64_t)blockIdx.x * (blockDim.x >> 6) + wave;
    const uint64_t nw = (uint64_t)gridDim.x * (blockDim.x >> 6);
    uint64_t t = n_tiles * gw / nw;
    const uint64_t t_end = n_tiles * (gw + 1) / nw;
    if (t >= t_end) return;

    // stream of tile t: largest s with tile_base[s] <= t
    uint64_t lo = 0, hi = n_streams;
    while (hi - lo > 1) {
        const uint64_t mid = (lo + hi) >> 1;
        if (d.tile_base[mid] <= t) lo = mid;
        else hi = mid;
    }
    uint64_t s = lo, cur = d.tile_base[s], next = d.tile_base[s + 1];
    for (; t < t_end; ++t) {
        while (t >= next) {
            ++s;
            cur = next;
            next = d.tile_base[s + 1];
        }
        const uint8_t *base = d.ptr[s];
        const uint64_t jneed = d.jneed[s];
        const uint64_t j0 = (t - cur) * kTileKeys;
        uint64_t bk, bj;
        const bool fast = j0 >= kTileKeys && j0 + kTileKeys - 1 <= jneed &&
                          (reinterpret_cast<uintptr_t>(base) & 15) == 0;
        if (fast) {
            tile_fast(tl, th, base, j0, lb_a, lb_b, bk, bj);
        } else {
            const uint64_t jb = min(j0 + kTileKeys - 1, jneed);
            tile_exact(tl, th, base, j0, max(j0, (uint64_t)1), jb, bk, bj);
        }
        if (lane == 0) {
            rec[t].key = bk;
            rec[t].j = bj;
        }
    }
}

// ----------------------------------------------------------------- phase B: chain kernel

// best (key desc, index asc) over the exact keys [a, b] of one stream, lanes strided
__device__ __forceinline__ void scan_exact(const uint64_t *tl, const uint64_t *th,
                                           const uint8_t *base, uint64_t a, uint64_t b,
                                           uint64_t &bk, uint64_t &bj) {
    for (uint64_t j = a + lane_id(); j <= b; j += 64) {
        const uint64_t k = key_at(tl, th, base, j);
        if (k > bk) {
            bk = k;
            bj = j;
        }
    }
}

__global__ __launch_bounds__(256) void rc_chain_kernel(const KeyTables *__restrict__ tab,
                                                       StreamDesc d, uint64_t n_streams,
                                                       ChainParams prm,
                                                       const TileRecord *__restrict__ rec,
                                                       uint64_t *__restrict__ cuts,
                                                       int64_t *__restrict__ counts) {
    __shared__ __attribute__((aligned(16))) uint64_t s_full[2048];
    const uint64_t *gfull = &tab->tl[0][0];
    for (uint32_t i = threadIdx.x; i < 2048u; i += blockDim.x) s_full[i] = gfull[i];
    __syncthreads();
    const uint64_t *tl = s_full, *th = s_full + 1024;

    const uint32_t lane = lane_id();
    const uint64_t s = (uint64_t)blockIdx.x * (blockDim.x >> 6) +
                       __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (s >= n_streams) return;

    const uint8_t *base = d.ptr[s];
    const uint64_t L = d.len[s], P = d.last[s], tb0 = d.tile_base[s];
    const uint64_t cbase = d.cut_base[s], cap = d.cut_cap[s];
    const uint64_t minl = prm.min_length, maxl = prm.max_length, T = prm.window;
    const uint64_t jmax = L >= 8 ? (L - 4) / 4 : 0;
    const uint64_t forced = (minl + 3) & ~3ull;
    const bool single = prm.max_steps == 0;  // raw next_cut: one argmax, result even if 0

    uint64_t pos = 0, n = 0;
    bool overflow = false;
    auto emit = [&](uint64_t c) {
        if (n >= cap) {
            overflow = true;
            return;
        }
        if (lane == 0) cuts[cbase + n] = c;
        ++n;
    };
    const uint64_t steps = single ? 1 : prm.max_steps;

    while (pos < L && n < steps && !overflow) {
        const uint64_t rem = L - pos;
        const bool argmax = single || (P >= pos && P - pos >= maxl) || rem >= 2 * maxl;
        if (prm.open && !argmax) break;  // a non-final next_cut returns 0: wait for more bytes
        if (argmax) {
            // window keys j in [pos/4 + 1, pos/4 + T]  (i = 4 .. < max, adapters.cpp:59)
            const uint64_t s4 = pos >> 2;
            const uint64_t ja = s4 + 1, jb = min(s4 + T, jmax);
            uint64_t bk = 0, bj = ~0ull;
            if (T > 0 && ja <= jb) {
                const uint64_t t_lo = (ja + kTileKeys - 1) / kTileKeys;
                const uint64_t t_hi = (jb + 1) / kTileKeys;
                if (t_lo < t_hi) {
                    scan_exact(tl, th, base, ja, t_lo * kTileKeys - 1, bk, bj);
                    for (uint64_t t = t_lo + lane; t < t_hi; t += 64) {
                        const TileRecord r = rec[tb0 + t];
                        if (r.key > bk) {
                            bk = r.key;
                            bj = r.j;
                        }
                    }
                    scan_exact(tl, th, base, t_hi * kTileKeys, jb, bk, bj);
                } else {
                    scan_exact(tl, th, base, ja, jb, bk, bj);
                }
                wave_best(bk, bj);
            }
            uint64_t idx = bk > 0 ? 4 * (bj - s4) : 0;
            if (idx < minl) idx = forced;  // adapters.cpp:66-67
            if (single) {
                emit(idx);
                break;
            }
            if (idx != 0) {
                pos += idx;
                emit(pos);
                continue;
            }
            if (rem >= 2 * maxl || prm.open) break;  // min_length == 0, no positive key (S7 UB)
        }
        // tail rule of a final buffer < 2*max (adapters.cpp:48-55): one or two chunks
        uint64_t c;
        if (rem <= maxl) c = rem;
        else if (rem < maxl + minl) c = rem / 2;
        else c = maxl;
        if (c == 0) break;
        emit(pos + c);
        if (c < rem) emit(L);
        break;
    }
    if (lane == 0) counts[s] = overflow ? -1 : (int64_t)n;
}

// ---------------------------------------------------------------------- synthetic bytes

__global__ void rc_fill_kernel(uint8_t *__restrict__ dst, uint64_t nbytes, uint64_t base) {
    const uint64_t nwords = nbytes / 8;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    uint64_t *w = reinterpret_cast<uint64_t *>(dst);
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nwords; i += stride)
        w[i] = splitmix64(base ^ i);
    if (blockIdx.x == 0 && threadIdx.x < (nbytes & 7)) {
        const uint64_t v = splitmix64(base ^ nwords);
        dst[nwords * 8 + threadIdx.x] = (uint8_t)(v >> (8 * threadIdx.x));
    }
}

int launch_status(const char *what) {
    const hipError_t e = hipGetLastError();
    if (e == hipSuccess) return 0;
    snprintf(g_launch_err, sizeof g_launch_err, "%s: %s", what, hipGetErrorString(e));
    return 1;
}

int cu_count() {
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 256;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        cus <= 0)
        return 256;
    return cus;
}

}  // namespace

extern "C" {

const char *rc_launch_error(void) { return g_launch_err; }

int rc_launch_tiles(const KeyTables *d_tables, StreamDesc desc, uint64_t n_streams,
                    uint64_t n_tiles, TileRecord *d_records, void *stream) {
    if (n_tiles == 0) return 0;
    const uint64_t waves_per_wg = 1024 / kWaveSize;
    uint64_t grid = (n_tiles + waves_per_wg - 1) / waves_per_wg;
    const uint64_t cus = (uint64_t)cu_count();
    if (grid > cus) grid = cus;  // persistent: one 144 KiB-LDS workgroup per CU
    hipLaunchKernelGGL(rc_tile_kernel, dim3((unsigned)grid), dim3(1024), 0,
                       (hipStream_t)stream, d_tables, desc, n_streams, n_tiles, d_records);
    return launch_status("rc_tile_kernel");
}

int rc_launch_chain(const KeyTables *d_tables, StreamDesc desc, uint64_t n_streams,
                    ChainParams prm, const TileRecord *d_records, uint64_t *d_cuts,
                    int64_t *d_counts, void *stream) {
    if (n_streams == 0) return 0;
    const uint64_t grid = (n_streams + kChainWaves - 1) / kChainWaves;
    hipLaunchKernelGGL(rc_chain_kernel, dim3((unsigned)grid), dim3(kChainWaves * kWaveSize), 0,
                       (hipStream_t)stream, d_tables, desc, n_streams, prm, d_records, d_cuts,
                       d_counts);
    return launch_status("rc_chain_kernel");
}

int rc_launch_fill(uint8_t *d_dst, uint64_t nbytes, uint64_t seed, uint64_t stream_id,
                   void *stream) {
    if (nbytes == 0) return 0;
    const uint64_t base = (seed * 0x9E3779B97F4A7C15ull) ^ (stream_id << 34);
    uint64_t grid = (nbytes / 8 + 255) / 256;
    if (grid > 8192) grid = 8192;
    if (grid == 0) grid = 1;
    hipLaunchKernelGGL(rc_fill_kernel, dim3((unsigned)grid), dim3(256), 0, (hipStream_t)stream,
                       d_dst, nbytes, base);
    return launch_status("rc_fill_kernel");
}

}  // extern "C"
