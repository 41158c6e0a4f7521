// kernels.hip -- gfx950 kernels of the content-defined chunker.
//
// Replaces the scan of /root/reference/src/adapters.cpp:42-77 (next_cut's argmax over key())
// with, per batch of streams:
//
//   tile kernel  (HBM-bound, one pass over every needed input byte)  rc_tile_kernel<G>
//            Persistent: one 1024-thread workgroup per CU, each wave a contiguous range of
//            4096-key tiles (16 KiB of stream, kTileKeys in gclmul.h), reduced to one
//            TileRecord = (first maximal 64-bit key, its index).  Bytes stream straight from
//            HBM into a register ring (16 x 16-byte buffer loads per lane in flight).  Per key
//            only the top 16 bits of the hash are evaluated: 4 conflict-free LDS lookups per
//            32-bit word (32x replicated prefilter tables, see gclmul.h), one v_bitop3 fold, DPP
//            for the neighbour word.  The wave's candidate lanes (their top-16 maximum is the
//            tile's) get the exact 64-bit key one tile later.  A candidate lane whose maximum
//            occurs twice makes the tile a marker record, resolved by rc_edge_kernel from the
//            candidate lanes.  G = 4 also stores per-quarter group bounds (small windows).
//
//   edge kernel  rc_edge_kernel: marker tiles and the tiles that run past a stream's end.
//
//   chain        (latency-bound)  the cut chain exactly as replicat's adapter loop cuts
//            (tail rules of adapters.cpp:48-57 under the piece framing of adapters.py:290-305):
//            each argmax window [s+4, s+max) is the maximum over the records of the tiles fully
//            inside it plus its two partial edge ranges.  Default for batches of >= 256 small-
//            window streams: a QUAD of lanes per stream (rc_quad_chain_kernel); otherwise one
//            wave per segment (rc_spec_kernel: speculative chains over segments of long
//            streams, spliced by rc_join_kernel / rc_merge / rc_scan / rc_copy).
//
// No MFMA anywhere: this is integer byte work.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "gclmul.h"
#include "diag.h"

using namespace rc;

namespace {

thread_local char g_launch_err[256];

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
// Stream bytes are global memory; the pointers come out of descriptor arrays, so say so
// explicitly -- a flat (generic) load also counts against lgkmcnt and would make every LDS
// wait drain the whole in-flight HBM stream.
typedef __attribute__((address_space(1))) const u32x4 gu32x4;
typedef __attribute__((address_space(1))) const uint32_t gu32;

constexpr int kStreamAux = RC_DIAG_STREAM_AUX;  // the streamed bytes' cache policy (nt)

// The tile ring reads through a buffer resource based at the tile: the lane offset stays in one
// VGPR for the whole kernel and the slot offset is an SGPR, so a reissue costs no address VALU
// (a 64-bit global address would need a v_add_co/v_addc pair per 4 KiB of immediate range).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t tile_rsrc(const uint8_t *base,
                                                             uint32_t bytes = 0xffffffffu) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(base), 0, bytes, 0x00020000);
}
__device__ __forceinline__ u32x4 ring_load(__amdgpu_buffer_rsrc_t r, uint32_t lane_off, int it) {
    return __builtin_amdgcn_raw_buffer_load_b128(r, lane_off, it * 1024, kStreamAux);
}

__device__ __forceinline__ uint32_t lane_id() { return threadIdx.x & 63; }

// v_max3_u32 as an opaque step: left to itself LLVM reassociates the running maxima of the
// unrolled tile loop into one tree at the end, keeping every intermediate alive (spills).
__device__ __forceinline__ uint32_t max3_u32(uint32_t a, uint32_t b, uint32_t c) {
    uint32_t r;
    asm("v_max3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}


// Lane l's 64-bit value (readlane returns int: keep both halves unsigned).
__device__ __forceinline__ uint64_t lane_u64(uint64_t v, int l) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((uint32_t)v, l);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((uint32_t)(v >> 32), l);
    return ((uint64_t)hi << 32) | lo;
}

// Descriptor words through the SCALAR cache (constant address space -> s_load): a vector load
// would sit in the in-order vmcnt queue behind the stream prefetch and its wait would drain it.
typedef __attribute__((address_space(4))) const uint64_t cu64;
__device__ __forceinline__ uint64_t sload(const uint64_t *p) { return *(cu64 *)(p); }
__device__ __forceinline__ const uint8_t *sload_ptr(const uint8_t *const *p) {
    return reinterpret_cast<const uint8_t *>(sload(reinterpret_cast<const uint64_t *>(p)));
}

__device__ __forceinline__ uint32_t ld_u32(const uint8_t *p) {
    return *(gu32 *)(p);
}
__device__ __forceinline__ gu32x4 *as_global_x4(const uint8_t *p) { return (gu32x4 *)(p); }

// Exact 64-bit key of (w[j-1], w[j]) from the byte tables (gclmul.h), k1 included.
__device__ __forceinline__ uint64_t full_key(const uint64_t *__restrict__ tl,
                                             const uint64_t *__restrict__ th, uint32_t wlo,
                                             uint32_t whi) {
    return tl[wlo & 255] ^ tl[256 + ((wlo >> 8) & 255)] ^ tl[512 + ((wlo >> 16) & 255)] ^
           tl[768 + (wlo >> 24)] ^ th[whi & 255] ^ th[256 + ((whi >> 8) & 255)] ^
           th[512 + ((whi >> 16) & 255)] ^ th[768 + (whi >> 24)];
}

// 64-bit DPP move; lanes without a source (bound_ctrl off, masked rows) keep their own value,
// which the lexicographic maximum below absorbs.
template <int kCtrl, int kRowMask>
__device__ __forceinline__ uint64_t dpp_u64(uint64_t v) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp((int)(uint32_t)v, (int)(uint32_t)v,
                                                              kCtrl, kRowMask, 0xf, false);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp((int)(uint32_t)(v >> 32),
                                                              (int)(uint32_t)(v >> 32), kCtrl,
                                                              kRowMask, 0xf, false);
    return ((uint64_t)hi << 32) | lo;
}

template <int kCtrl, int kRowMask>
__device__ __forceinline__ void best_step(uint64_t &k, uint64_t &j) {
    const uint64_t ko = dpp_u64<kCtrl, kRowMask>(k), jo = dpp_u64<kCtrl, kRowMask>(j);
    if (ko > k || (ko == k && jo < j)) {
        k = ko;
        j = jo;
    }
}

// (key desc, index asc) maximum over the wave; every lane gets the result.  DPP row shifts
// 1/2/4/8 leave each row's maximum in its lane 15, row broadcasts 15 and 31 carry it to lane
// 63, read back as a scalar: no LDS round trips (ds_bpermute) on the chain's critical path.
__device__ __forceinline__ void wave_best(uint64_t &k, uint64_t &j) {
    best_step<0x111, 0xf>(k, j);  // row_shr:1
    best_step<0x112, 0xf>(k, j);  // row_shr:2
    best_step<0x114, 0xf>(k, j);  // row_shr:4
    best_step<0x118, 0xf>(k, j);  // row_shr:8
    best_step<0x142, 0xa>(k, j);  // row_bcast:15 into rows 1 and 3
    best_step<0x143, 0xc>(k, j);  // row_bcast:31 into rows 2 and 3
    k = lane_u64(k, 63);
    j = lane_u64(j, 63);
}

// ------------------------------------------------------------------ phase A: tile kernel

__shared__ __attribute__((aligned(16))) uint32_t s_tile_lds[kTileLdsBytes / 4];

__device__ __forceinline__ uint32_t pf_lds(uint32_t byte_addr) {
    return *reinterpret_cast<const uint32_t *>(reinterpret_cast<const char *>(s_tile_lds) +
                                               byte_addr);
}

__device__ __forceinline__ void pf_addrs(uint32_t w, uint32_t lb_a, uint32_t lb_b, uint32_t *a) {
    a[0] = __builtin_amdgcn_perm(w, lb_a, 0x0c020400u);
    a[1] = __builtin_amdgcn_perm(w, lb_a, 0x0c020500u) + 128;
    a[2] = __builtin_amdgcn_perm(w, lb_b, 0x0c020600u);
    a[3] = __builtin_amdgcn_perm(w, lb_b, 0x0c020700u) + 128;
}
// the four lookups of a word folded in two VALU: gfx950's v_bitop3_b32 (truth table 0x96) is a
// three-input XOR (left to itself the compiler XORs them pairwise as the loads land)
__device__ __forceinline__ uint32_t pf_gather(const uint32_t *a) {
    return __builtin_amdgcn_bitop3_b32(pf_lds(a[0]), pf_lds(a[1]), pf_lds(a[2]), 0x96) ^ pf_lds(a[3]);
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

// The chain kernels' tables: the prefilter entries PF[4][256] once (no replication: the chain
// scans an edge range only when the tile records cannot settle it, a few % of ranges), then
// the exact TL/TH tables -- 20 KiB instead of 144 KiB, so several chain workgroups share a CU.
__shared__ __attribute__((aligned(16))) uint32_t s_chain_lds[1024 + 4096];

__device__ __forceinline__ uint32_t pfc_entry(const uint32_t *pf, uint32_t w) {
    return pf[w & 255] ^ pf[256 + ((w >> 8) & 255)] ^ pf[512 + ((w >> 16) & 255)] ^
           pf[768 + (w >> 24)];
}

__device__ __forceinline__ void stage_chain_tables(const KeyTables *tab) {
    const uint32_t nt = blockDim.x;
    const uint32_t *gpf = &tab->pf[0][0];
    for (uint32_t i = threadIdx.x; i < 1024u; i += nt) s_chain_lds[i] = gpf[i];
    uint64_t *full = reinterpret_cast<uint64_t *>(s_chain_lds + 1024);
    const uint64_t *gfull = &tab->tl[0][0];
    for (uint32_t i = threadIdx.x; i < 2048u; i += nt) full[i] = gfull[i];
    __syncthreads();
}

// (key desc, index asc) improvement test: the lexicographic order makes the merge of ranges
// and records independent of the order in which a lane visits them.
__device__ __forceinline__ void take_best(uint64_t k, uint64_t j, uint64_t &bk, uint64_t &bj) {
    if (k > bk || (k == bk && j < bj)) {
        bk = k;
        bj = j;
    }
}

// Best exact key over the two key ranges [a0, b0] and [a1, b1] of one stream (either may be
// empty: a > b).  Lanes take consecutive keys (coalesced 256-B loads).  Every round first
// issues all of the lane's loads -- unconditionally, at indices clamped into the range, so
// the compiler cannot serialise them behind divergent branches -- then evaluates, so a round
// costs one memory latency.
constexpr int kScanUnroll = 16;  // edge kernel: a whole tile per wave
#ifndef RC_CHAIN_SCAN_UNROLL
#define RC_CHAIN_SCAN_UNROLL 4
#endif
constexpr int kChainScanUnroll = RC_CHAIN_SCAN_UNROLL;  // chain steps' rare exact fallback

template <int kScanUnroll>
__device__ __forceinline__ void scan_ranges(const uint64_t *tl, const uint64_t *th,
                                            const uint8_t *base, uint64_t a0, uint64_t b0,
                                            uint64_t a1, uint64_t b1, uint64_t &bk,
                                            uint64_t &bj) {
    const bool e0 = a0 <= b0, e1 = a1 <= b1;
    if (!e0 && !e1) return;
    if (!e0) a0 = b0 = a1;  // a valid dummy key, never taken
    if (!e1) a1 = b1 = a0;
    const uint64_t lane = lane_id();
    for (uint64_t r = 0;; r += 64 * kScanUnroll) {
        const bool live0 = e0 && a0 + r <= b0, live1 = e1 && a1 + r <= b1;
        if (!live0 && !live1) break;
        uint2 w0[kScanUnroll], w1[kScanUnroll];
#pragma unroll
        for (int u = 0; u < kScanUnroll; ++u) {
            const uint64_t j0 = min(a0 + r + 64 * u + lane, b0);
            const uint64_t j1 = min(a1 + r + 64 * u + lane, b1);
            w0[u].x = ld_u32(base + 4 * j0 - 4);
            w0[u].y = ld_u32(base + 4 * j0);
            w1[u].x = ld_u32(base + 4 * j1 - 4);
            w1[u].y = ld_u32(base + 4 * j1);
        }
#pragma unroll
        for (int u = 0; u < kScanUnroll; ++u) {
            const uint64_t j0 = a0 + r + 64 * u + lane, j1 = a1 + r + 64 * u + lane;
            if (e0 && j0 <= b0) take_best(full_key(tl, th, w0[u].x, w0[u].y), j0, bk, bj);
            if (e1 && j1 <= b1) take_best(full_key(tl, th, w1[u].x, w1[u].y), j1, bk, bj);
        }
    }
}

// Best record over tiles [t_lo, t_hi) of one stream, loads issued up front per round.
#ifndef RC_REC_UNROLL
#define RC_REC_UNROLL 4
#endif
constexpr int kRecUnroll = RC_REC_UNROLL;

__device__ __forceinline__ void scan_records(const TileRecord *rec, uint64_t t_lo, uint64_t t_hi,
                                             uint64_t &bk, uint64_t &bj) {
    const uint64_t lane = lane_id();
    for (uint64_t r = t_lo; r < t_hi; r += 64 * kRecUnroll) {
        TileRecord v[kRecUnroll];
#pragma unroll
        for (int u = 0; u < kRecUnroll; ++u) v[u] = rec[min(r + 64 * u + lane, t_hi - 1)];
#pragma unroll
        for (int u = 0; u < kRecUnroll; ++u)
            if (r + 64 * u + lane < t_hi && v[u].key != 0) take_best(v[u].key, v[u].j, bk, bj);
    }
}

// Where a wave's tile lives.  `fast` = every key j0 .. j0+4095 has its 8 bytes inside the
// stream (tile_fast below): the tile kernel's register ring reads exactly those 16 KiB.
// Tile 0 is fast too (its key 0, which would need the word before the stream, is masked out of
// the scan), and so is a stream's last tile when it ends inside the data: its keys past `jneed`
// are real keys no argmax window reaches, so its record is the first maximum over a superset of
// the keys the chain asks about -- which the chain only ever uses as that tile's exact answer
// when the record's index lies inside the asked range, and otherwise as an upper bound (see
// chain_step), both of which hold for a superset.  Only a last tile that runs past the stream's
// final word goes to the edge kernel (it happens when jneed is within 4096 keys of the end).
struct TileRef {  // 24 bytes, no padding: a padded copy left two 7-byte allocas in the group-
                  // grab kernels, which the backend promoted to LDS (14 KiB per workgroup, a
                  // struct copy through LDS at every tile)
    const uint8_t *base;
    uint64_t j0;
    uint32_t s;     // its stream (< 2^31, checked by the host)
    uint32_t fast;  // 0: not fast; else the 256-key slices to read (kTileIters; fewer: kClip)
};

// j0 + 4095 <= jmax, with jmax = (L - 4) / 4 the last key whose 8 bytes exist (adapters.cpp:73)
__device__ __forceinline__ bool tile_fast(uint64_t j0, uint64_t L) {
    return L >= 8 && j0 + kTileKeys - 1 <= (L - 4) / 4;
}

// Last key index of a tile's record: the whole tile on the fast path, else clipped to jneed.
__device__ __forceinline__ uint64_t tile_key_end(uint64_t j0, uint64_t L, uint64_t jneed) {
    return tile_fast(j0, L) ? j0 + kTileKeys - 1 : min(j0 + kTileKeys - 1, jneed);
}

// TileRecord.j of a tile left to the exact path: ~stream index (its key: the candidate lanes;
// streams are numbered below 2^31 here, checked by the host)
constexpr uint64_t kTieMark = ~0ull;

// (hi16(a) ^ lo16(b)) << 16 in ONE VALU (SDWA: src0 WORD_1, src1 WORD_0, dst WORD_1, low half
// zero): the top 16 bits of key j from the prefilter entries of words j-1 (a, its Lmap half) and
// j (b, its Hmap half).  Round 6: replaces the split of every entry into a masked high half and
// a shifted low half (two VALU per word) and the per-key index packing (below).
__device__ __forceinline__ uint32_t key_top16(uint32_t a, uint32_t b) {
    uint32_t r;
    asm("v_xor_b32_sdwa %0, %1, %2 dst_sel:WORD_1 dst_unused:UNUSED_PAD src0_sel:WORD_1 "
        "src1_sel:WORD_0"
        : "=v"(r) : "v"(a), "v"(b));
    return r;
}
// an opaque v_max_u32 (as max3_u32: keeps LLVM from re-associating the running maxima)
__device__ __forceinline__ uint32_t max_u32_op(uint32_t a, uint32_t b) {
    uint32_t r;
    asm("v_max_u32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}

// Fast path over a tile whose kTileIters loads are in flight in x[].  As iteration `it` consumes
// x[it] it re-issues x[it] for the wave's NEXT fast tile (if any), so every wave keeps
// 8 KiB of HBM reads in flight through its compute phase (a register ring: no extra VGPRs,
// the in-order vmcnt does the bookkeeping).
//
// Returns the lane's largest top-16 value `top` and the first and last SLICE (iteration) of the
// lane holding it, fs and ls (round 6; until round 5 the first and last key, packed per key: two
// fused XOR-ORs per key).  Per 16-byte slice: 16 table addresses (v_perm), 16 lookups, 4 three-
// input XOR folds + 4 XORs (the words' entries), the neighbour entry by DPP, 4 SDWA XORs (the
// keys' top 16 bits), the slice maximum, and the slice index ORed into the two running maxima:
// 36 VALU instead of 43.  The key inside the slice is found exactly at retire (rc_tile_kernel:
// the 4 keys of a candidate lane's first slice get exact keys), and a lane whose maximum is in
// two slices makes the tile a marker, as a key-level tie did.
// `prev_word` holds the word before the tile (key j0's low half) and is refilled with the next
// tile's, issued with the ring.
//
// G > 1 (chunkers with small windows, see rc_launch_tiles): the tile's keys also fall into G
// groups of kTileKeys / G consecutive keys (iterations it * G / kTileIters), and the lane's
// largest top-16 value per group comes back packed two per word in gpk (group g in half g & 1
// of gpk[g / 2]): one more v_max per slice.
template <int G>
__device__ __forceinline__ void tile_scan(const TileRef &tr, const TileRef &nx,
                                          u32x4 (&x)[kTileIters], uint32_t &prev_word,
                                          uint32_t lb_a, uint32_t lb_b, uint32_t &top,
                                          uint32_t &fs, uint32_t &ls,
                                          uint32_t (&gpk)[(G + 1) / 2]) {
    static_assert(G == 1 || (G % 2 == 0 && kTileIters % G == 0), "groups: 1 or an even divisor");
    static_assert(kTileIters <= 16, "slice indices: 4 bits");
    constexpr int kPer = kTileIters / G;  // iterations per group
    const uint32_t lane = lane_id();
    // no next fast tile (end of the wave's range): harmlessly re-read this tile instead, so
    // the ring loads stay unconditional
    const uint8_t *nbase = nx.fast ? nx.base + 4 * nx.j0 : tr.base + 4 * tr.j0;
    // G > 1: a stream's last tile reads only its slices up to the last needed key (TileCursor
    // kClip); loads past the resource's range return zeros without touching memory
    const __amdgpu_buffer_rsrc_t nsrc =
        G > 1 ? tile_rsrc(nbase, (nx.fast ? nx.fast : tr.fast) * 1024u) : tile_rsrc(nbase);
    uint32_t carry = pf_entry(prev_word, lb_a, lb_b);
    // the word before the next tile; a stream's tile 0 has none (its key 0 is masked below),
    // so it re-reads its own first word rather than the 4 bytes before the stream.  Round 6: a
    // next tile that follows this one in its stream takes it from the ring instead (this tile's
    // last word: lane 63 of slice 15), and the load reads nothing -- a buffer resource of range 0
    // keeps it one vector-memory instruction, so every tile issues the same sequence (a third of
    // the kernel's auxiliary requests: those cost the scan ~1 %, profiles/r06/aux_loads/)
    const uint64_t nj0 = nx.fast ? nx.j0 : tr.j0;
    const bool consec = nx.fast && nx.s == tr.s && nx.j0 == tr.j0 + kTileKeys;
    const uint32_t pw_loaded = __builtin_amdgcn_raw_buffer_load_b32(
        tile_rsrc(nj0 ? nbase - 4 : nbase, consec ? 0u : 4u), 0, 0, 0);
    uint32_t last_w = 0;
    // key 0 of a stream (local index 0 of lane 0 in tile 0) does not exist: i starts at 4
    // (adapters.cpp:59).  Its top-16 value is zeroed, so it never raises a slice maximum.
    const uint32_t key0_mask = (tr.j0 == 0 && lane == 0) ? 0u : ~0u;
    uint32_t acc_first = 0, acc_last = 0, acc_grp = 0;
#pragma unroll
    for (int it = 0; it < kTileIters; ++it) {
        // the 16 table addresses of this 16-byte slice; then the slot is free for the next
        // tile's slice (same registers: no copies when the loop wraps)
        uint32_t a[16], r[16];
        pf_addrs(x[it].x, lb_a, lb_b, a + 0);
        pf_addrs(x[it].y, lb_a, lb_b, a + 4);
        pf_addrs(x[it].z, lb_a, lb_b, a + 8);
        pf_addrs(x[it].w, lb_a, lb_b, a + 12);
        if (it == kTileIters - 1) last_w = (uint32_t)__builtin_amdgcn_readlane(x[it].w, 63);
        x[it] = ring_load(nsrc, lane * 16, it);
        // the slice's 16 lookups issued together, then folded (round 5): left to itself the
        // scheduler gave every variant but rc_tile_kernel<1, false> a low-pressure order -- 3-4
        // lookups, then lgkmcnt(0), ~83 full LDS drains per tile (the ISA of <4>, the small-
        // window kernel, had it in round 4 too); the fence makes the order the same in all
        // four kernels (16 lookups in flight, 128 VGPRs, no spills)
        uint32_t e0, e1, e2, e3;
        if constexpr (RC_DIAG_SLICE_FENCE) {
#pragma unroll
            for (int q = 0; q < 16; ++q) r[q] = pf_lds(a[q]);
            __builtin_amdgcn_sched_barrier(0);
            e0 = __builtin_amdgcn_bitop3_b32(r[0], r[1], r[2], 0x96) ^ r[3];
            e1 = __builtin_amdgcn_bitop3_b32(r[4], r[5], r[6], 0x96) ^ r[7];
            e2 = __builtin_amdgcn_bitop3_b32(r[8], r[9], r[10], 0x96) ^ r[11];
            e3 = __builtin_amdgcn_bitop3_b32(r[12], r[13], r[14], 0x96) ^ r[15];
        } else {  // the compiler's order (round 4)
            e0 = pf_gather(a + 0);
            e1 = pf_gather(a + 4);
            e2 = pf_gather(a + 8);
            e3 = pf_gather(a + 12);
        }
        // previous word's entry for key 0 of this lane: lane-1's e3 (wave_ror:1); lane 0 takes
        // the carry = lane 63's e3 of the previous iteration (or the word before the tile).
        const uint32_t rot = __builtin_amdgcn_mov_dpp(e3, 0x13C, 0xf, 0xf, false);
        const uint32_t ep = lane == 0 ? carry : rot;
        carry = rot;
        uint32_t b0 = key_top16(ep, e0);
        if (it == 0) b0 &= key0_mask;
        const uint32_t b1 = key_top16(e0, e1), b2 = key_top16(e1, e2), b3 = key_top16(e2, e3);
        // the slice's maximum; its index ORed in low: "first" prefers the earliest slice
        // (15 - it), "last" the latest (it)
        uint32_t sm = max_u32_op(max3_u32(b0, b1, b2), b3);
        if constexpr (G > 1) sm &= (uint32_t)it < tr.fast ? ~0u : 0u;  // a clipped slice: no keys
        acc_first = max_u32_op(acc_first, sm | (uint32_t)(kTileIters - 1 - it));
        acc_last = max_u32_op(acc_last, sm | (uint32_t)it);
        if constexpr (G > 1) {
            acc_grp = max_u32_op(acc_grp, sm);
            if ((it + 1) % kPer == 0) {  // compile-time after the unroll
                const int g = it / kPer;
                if (g % 2 == 0) gpk[g / 2] = acc_grp >> 16;
                else gpk[g / 2] |= acc_grp & 0xffff0000u;
                acc_grp = 0;
            }
        }
    }
    top = acc_first >> 16;
    fs = (uint32_t)(kTileIters - 1) - (acc_first & 0xffffu);
    ls = acc_last & 0xffffu;
    prev_word = consec ? last_w : pw_loaded;
}

// Maximum over the wave, returned in SGPRs: DPP shifts within each 16-lane row, then the
// four row maxima (lanes 15, 31, 47, 63) through readlane.
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false));
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false));
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false));
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false));
    const uint32_t r0 = __builtin_amdgcn_readlane(v, 15), r1 = __builtin_amdgcn_readlane(v, 31);
    const uint32_t r2 = __builtin_amdgcn_readlane(v, 47), r3 = __builtin_amdgcn_readlane(v, 63);
    return max(max(r0, r1), max(r2, r3));
}

__device__ __forceinline__ uint32_t pk_max_u16(uint32_t a, uint32_t b) {
    uint32_t r;
    asm("v_pk_max_u16 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ uint32_t pk_max_u16_s(uint32_t a, uint32_t b) {  // uniform values
    return max(a & 0xffffu, b & 0xffffu) | (max(a >> 16, b >> 16) << 16);
}

// Per-half maximum of two packed u16 values over the wave (uniform result): DPP row shifts,
// then the four row maxima through readlane, as wave_max_u32.
__device__ __forceinline__ uint32_t wave_max_pk16(uint32_t v) {
    v = pk_max_u16(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false));
    v = pk_max_u16(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false));
    v = pk_max_u16(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false));
    v = pk_max_u16(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false));
    const uint32_t r0 = __builtin_amdgcn_readlane(v, 15), r1 = __builtin_amdgcn_readlane(v, 31);
    const uint32_t r2 = __builtin_amdgcn_readlane(v, 47), r3 = __builtin_amdgcn_readlane(v, 63);
    return pk_max_u16_s(pk_max_u16_s(r0, r1), pk_max_u16_s(r2, r3));
}

// Walks a wave's tile range across stream boundaries (all state wave-uniform).  kCache: the
// stream's pointer and fast-tile count are loaded when the cursor enters it, not per tile (scalar
// loads share lgkmcnt with the LDS reads, so each one in flight is a wait the next LDS use pays
// for); round 6: on for rc_tile_kernel<4> too (its SGPRs fit since the SDWA scan).
// kClip (round 6, rc_tile_kernel<4>): TileRef.fast of a stream's LAST tile is the number of its
// 256-key slices up to the stream's last needed key, not 16: the ring reads only those (the
// buffer resource's range ends there) and the scan masks the rest -- config 3 (iii)'s 1 MiB
// streams need 2 of their last tile's 16 slices, 1.5 % of the bytes the kernel read before.
template <bool kCache, bool kClip = false>
struct TileCursor {
    StreamDesc d;
    uint64_t s, cur, next;
    const uint8_t *base;
    uint32_t nfast;  // the stream's tiles 0 .. nfast - 1 are on the fast path (tile_fast)
    uint32_t nlast;  // kClip: the slices of the stream's last tile holding needed keys
    __device__ void enter() {
        if constexpr (!kCache) return;
        base = sload_ptr(d.ptr + s);
        const uint64_t L = sload(d.len + s);
        // tile_fast(j0, L) for j0 = i * kTileKeys  <=>  i < nfast
        nfast = L >= 8 && (L - 4) / 4 >= kTileKeys - 1
                    ? (uint32_t)(((L - 4) / 4 - (kTileKeys - 1)) / kTileKeys + 1) : 0u;
        if constexpr (kClip) {
            const uint64_t jl = sload(d.jneed + s) - (next - cur - 1) * kTileKeys;
            nlast = jl < (uint64_t)kTileKeys ? (uint32_t)(jl >> 8) + 1u : (uint32_t)kTileIters;
        }
    }
    __device__ void init(const StreamDesc &dd, uint64_t n_streams, uint64_t t) {
        d = dd;
        uint64_t lo = 0, hi = n_streams;  // largest s with tile_base[s] <= t
        while (hi - lo > 1) {
            const uint64_t mid = (lo + hi) >> 1;
            if (sload(d.tile_base + mid) <= t) lo = mid;
            else hi = mid;
        }
        s = lo;
        cur = sload(d.tile_base + s);
        next = sload(d.tile_base + s + 1);
        enter();
    }
    __device__ TileRef at(uint64_t t) {  // t must not decrease between calls
        if (t >= next) {
            do {
                ++s;
                cur = next;
                next = sload(d.tile_base + s + 1);
            } while (t >= next);
            enter();
        }
        TileRef r;
        r.j0 = (t - cur) * kTileKeys;
        r.s = (uint32_t)s;
        if constexpr (kCache) {
            r.base = base;
            r.fast = t - cur < nfast ? (kClip && t + 1 == next ? nlast : (uint32_t)kTileIters) : 0u;
        } else {
            r.base = sload_ptr(d.ptr + s);
            r.fast = __builtin_amdgcn_readfirstlane((uint32_t)tile_fast(r.j0, sload(d.len + s))) != 0;
        }
        return r;
    }
};

__device__ __forceinline__ void stage_tile_tables_nb(const KeyTables *tab) {
    // the 32x replicated prefilter tables and the exact tables.  Each thread loads its table
    // entries once (all loads in flight together), then writes the 32 copies, starting at a
    // lane-dependent copy so that a wave's stores spread over the banks.
    const uint32_t nt = blockDim.x;
    for (uint32_t e0 = 0; e0 < 1024u; e0 += 4 * nt) {
        uint32_t v[4];
        uint32_t ent[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            ent[k] = e0 + k * nt + threadIdx.x;
            v[k] = ent[k] < 1024u ? (&tab->pf[0][0])[ent[k]] : 0u;
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            if (ent[k] >= 1024u) continue;
            const uint32_t b = ent[k] >> 8, vv = ent[k] & 255;
            uint32_t *row = s_tile_lds + ((b >> 1) * 65536u + vv * 256u + (b & 1) * 128u) / 4;
            for (uint32_t c = 0; c < 32; ++c) row[(c + threadIdx.x) & 31] = v[k];
        }
    }
    uint64_t *full = reinterpret_cast<uint64_t *>(s_tile_lds + kFullOff / 4);
    const uint64_t *gfull = &tab->tl[0][0];
    for (uint32_t i = threadIdx.x; i < 2048u; i += nt) full[i] = gfull[i];
}

// Group bounds of one tile from the lanes' packed per-group top-16 maxima (gpk: group 2i in the
// low half of gpk[i], 2i + 1 in the high half): the group maxima (one packed wave maximum per
// pair of groups) and the lanes whose maximum reaches the hot threshold (one ballot per group).
template <int G>
__device__ __forceinline__ GroupRecord tile_groups(const uint32_t (&gpk)[(G + 1) / 2], uint32_t hot) {
    GroupRecord r;
    r.max = 0;
    r.pad = 0;
#pragma unroll
    for (int i = 0; i < (G + 1) / 2; ++i) {
        const uint32_t v = gpk[i];
        r.max |= (uint64_t)wave_max_pk16(v) << (32 * i);
        r.hot[2 * i] = __ballot((v & 0xffffu) >= hot);
        r.hot[2 * i + 1] = __ballot((v >> 16) >= hot);
    }
    return r;
}

// The tile kernel's work units (round 3): wave w first takes the static unit w, tiles
// [w s0, (w + 1) s0); the rest of the tiles, from dyn0 = nw s0 on, are dynamic units of `chunk`
// tiles that waves grab from a counter (one atomic per unit) when they run out of work.  Round 2
// gave every wave the same static share and measured (RC_DIAG_TILE_STAMPS) the waves of one
// launch ending between 52 % and 100 % of its time: the slowest waves' tail was ~23 % of the
// kernel.  Small launches (fewer than TileSched::dyn_min tiles per wave) stay fully static.
// Static share 25 % and 32-tile units: 10-11 % faster on configs 2, 3 (iii) and 4 than fully
// static on the same allocation; late in round 3, 10 % and 12-tile units took ~4 % more off
// (tile_units).
struct TileUnits {  // tile indices fit 32 bits (the tie lists store them as u32)
    uint32_t n_tiles, nw, s0, chunk, dyn0, n_units;
    uint32_t gshift;    // group grabs (UnitGrab): 2^gshift dynamic units per global grab
    uint32_t n_groups;  // group grabs: global grab values below this hold units; 0: per-wave grabs
    __device__ __host__ void range(uint32_t u, uint32_t &b, uint32_t &e) const {
        if (u < nw) {
            b = u * s0;
            e = b + s0;
        } else {
            b = dyn0 + (u - nw) * chunk;
            e = b + chunk;
        }
        if (b > n_tiles) b = n_tiles;
        if (e > n_tiles) e = n_tiles;
    }
};

// Units of a launch over n_tiles tiles by nw waves (sched: knobs.h RC_TILE_STATIC, per mille:
// the share of the tiles handed out statically; RC_TILE_CHUNK: dynamic unit size;
// RC_TILE_DYN_MIN: fewer tiles per wave stay fully static; RC_TILE_GROUP: units per workgroup
// grab).  Defaults since round 5: 0 / 3 / 0 / 64 -- every tile in 3-tile units, 64 units per
// workgroup grab (config 2 tile kernel -3 to -4 %, the harness -5 %, 3 ii / 3 iii / config 4
// -2 to -4 % against the round-4 schedule on one allocation each, profiles/r05/sched/).
// Round 3/4 defaults were 100 / 12 / 128 / 0, measured so:  Both
// measured on one allocation per config (scripts/tile_sched_ab.py, profiles/r03/sched): tile
// kernel vs the round-2 fully static schedule, config 2 11.06 -> 9.88 ms, 3 (iii) 11.46 -> 10.32,
// config 4 23.87 -> 21.23; the harness (76 tiles per wave) is fastest fully static.  Units were
// 32 tiles until a later sweep went below (scripts/overlap_ab.py, profiles/r03/sched_units*):
// the last units are the launch's tail, and on two allocations config 2's tile kernel took
// 10.17 / 10.21 ms with 32, 9.87 / 9.89 with 12, 9.82 with 10, 9.90 / 9.87 with 8 -- and 10.51
// with 6: every grab is a device-scope atomic on one counter, and ~480 k of them in a 10 ms
// launch saturate it.  12 keeps half that rate (3 ii 10.65 -> 10.41 ms, 3 iii and config 4 ~1 %).
// With 12-tile units a 10 % static share beat 25 % (config 2 9.77 -> 9.68 ms pipelined, 9.78 ->
// 9.68 sequential, 3 iii 9.98 -> 9.94; 0 %: 9.72; profiles/r03/sched_static/): ~290 k grabs.
// RC_TILE_GROUP (sched.group, rounded down to a power of two): the units come in groups of that
// many, one global grab per group, dealt to the workgroup's waves through LDS (UnitGrab).
constexpr uint64_t kDynChunkMin = 2;    // units of at least 2 tiles
constexpr uint32_t kGrabMinShift = 4;   // groups of at least 16 units (UnitGrab's LDS ring)
__host__ inline TileUnits tile_units(uint64_t n_tiles, uint64_t nw, TileSched sched) {
    TileUnits U;
    U.n_tiles = (uint32_t)n_tiles;
    U.nw = (uint32_t)nw;
    U.gshift = 0;
    U.n_groups = 0;
    uint64_t permille = sched.permille, chunk = sched.chunk, dyn_min = sched.dyn_min;
    if (permille > 1000) permille = 1000;
    if (chunk < kDynChunkMin) chunk = kDynChunkMin;
    if (n_tiles < dyn_min * nw || permille == 1000) {  // fully static
        U.s0 = (uint32_t)((n_tiles + nw - 1) / nw);
        U.chunk = 1;
        U.dyn0 = (uint32_t)n_tiles;
        U.n_units = (uint32_t)nw;
        return U;
    }
    U.s0 = (uint32_t)(n_tiles * permille / 1000 / nw);
    // at least ~4 dynamic units per wave: a unit is the granularity of the launch's tail
    const uint64_t dyn = n_tiles - nw * U.s0, fit = dyn / (4 * nw);
    if (chunk > fit) chunk = fit > kDynChunkMin ? fit : kDynChunkMin;
    U.chunk = (uint32_t)chunk;
    U.dyn0 = (uint32_t)(nw * U.s0);
    U.n_units = (uint32_t)(nw + (n_tiles - U.dyn0 + chunk - 1) / chunk);
    if (sched.group) {
        // at least 2^kGrabMinShift units per group: the LDS ring's margin (UnitGrab)
        uint32_t sh = 0;
        while ((2u << sh) <= sched.group && sh < 8) ++sh;
        if (sh < kGrabMinShift) sh = kGrabMinShift;
        U.gshift = sh;
        U.n_groups = (uint32_t)(((uint64_t)(U.n_units - U.nw) + (1u << sh) - 1) >> sh);
    }
    return U;
}

// How a wave gets its next dynamic unit.
//
// Per-wave grabs (kGroup false, the round-3 schedule): lane 0's global atomic on the one
// counter, issued when the wave enters a unit and read when it leaves it.  One counter hands the
// units out in address order (the chip sweeps the bytes as one front), but it serves only ~45
// grabs per microsecond, so the units cannot be short: 12 tiles, ~0.1 ms of a wave, which is 1 %
// of a config-2 launch but an eighth of the reference harness's (0.85 ms).
//
// Group grabs (kGroup, round 5): one global grab per GROUP of 2^gshift consecutive units, dealt
// to the workgroup's waves through LDS.  A wave takes an ordinal o from the workgroup's LDS
// counter; o's slot k = o >> gshift is the workgroup's k-th group, its sub-unit o & (2^gshift-1).
// Slot k's global group index is published in s_grab_slot[k % kGrabSlots] as (k << 32 | g):
//   * slot 0 is grabbed by thread 0 while the workgroup stages its tables (before the barrier);
//   * the wave that takes sub-unit 0 of slot k grabs slot k + 1 right after it has read slot k
//     -- so the workgroup's grabs return increasing values -- waits for the atomic and publishes
//     it at once (past the end: g = ~0, without a grab).  Waiting drains that wave's loads once
//     per group; nothing is carried from unit to unit, so the tile loop keeps its registers;
//   * a wave whose slot is not published yet waits on LDS (s_sleep) -- for the publisher of
//     its slot, which holds the slot before it and never waits before it publishes, so the
//     waits end (tests/test_grab_model.py runs the protocol under random interleavings).
// A wave stops at the first unit past the end; every later ordinal of its workgroup is past the
// end too (the grabs increase), and every earlier one was taken by a wave that runs it: each
// unit is run exactly once.  Global grabs drop by 2^gshift, so units can be short.
// The ring holds kGrabSlots groups: slot k + kGrabSlots overwrites slot k once the other waves
// have taken ~15 * 2^gshift more ordinals (tile_units keeps gshift >= 4: 240 units, ~0.45 ms of
// 15 waves' work, between a wave's ordinal and its next LDS read).  A wave that finds a later
// tag in its slot lagged that far: its group index is lost, so it takes the fail-safe stop at
// once instead of waiting for a tag that never comes back.
constexpr uint32_t kGrabSlots = 16;
constexpr uint32_t kGrabSpinLimit = 1u << 24;  // ~1-2 s of s_sleep waits
__shared__ uint32_t s_grab_ord;
__shared__ uint32_t s_grab_cfg[2];  // gshift, n_groups: read from LDS at a switch, so the tile
                                    // loop holds no SGPRs for them (it is at its SGPR limit)
__shared__ uint64_t s_grab_slot[kGrabSlots];

// the fail-safe flag's word in the tile kernel's counter buffer (gclmul.h kCtrErrWord)
constexpr uint32_t kGrabErrWord = kCtrErrWord;

template <bool kGroup>
struct UnitGrab {
    uint32_t v;  // per-wave grabs: lane 0's pending global grab; group: thread 0's slot-0 grab

    // The first global grab, issued before the workgroup stages its tables (per-wave: this
    // wave's; group: thread 0's, for slot 0, written to LDS by seed()).
    __device__ void start(const TileUnits &U, uint32_t *ctr) {
        v = 0;
        if (U.n_units <= U.nw) return;
        if (kGroup ? threadIdx.x == 0 : lane_id() == 0) v = atomicAdd(ctr, 1u);
    }
    // Group grabs: slot 0 and the ordinal counter, before the workgroup's first barrier (which
    // makes them visible to every wave).
    __device__ void seed(const TileUnits &U) {
        if (!kGroup || U.n_units <= U.nw || threadIdx.x != 0) return;
        s_grab_ord = 0;
        s_grab_cfg[0] = U.gshift;
        s_grab_cfg[1] = U.n_groups;
        s_grab_slot[0] = (uint64_t)v;  // tag 0
        for (uint32_t i = 1; i < kGrabSlots; ++i) s_grab_slot[i] = ~0ull;
    }
    // The wave's next dynamic unit; U.n_units or more: none left.
    // err (may be NULL): set to 1 if a slot stayed unpublished for ~kGrabSpinLimit waits or was
    // overwritten before this wave read it (a protocol failure: the wave then stops as if the
    // units had run out, so the launch ends with incomplete records instead of hanging the GPU;
    // the edge kernel turns the flag into the call's fault stamp and every stream's count into
    // RC_COUNT_FAULT, so no caller receives those cuts as results).
    __device__ uint32_t next(const TileUnits &U, uint32_t *ctr, uint32_t *err) {
        if (U.n_units <= U.nw) return U.n_units;
        if constexpr (!kGroup) {
            const uint32_t u = U.nw + (uint32_t)__builtin_amdgcn_readfirstlane(v);
            if (u < U.n_units && lane_id() == 0) v = atomicAdd(ctr, 1u);
            return u;
        }
        uint32_t o = 0;
        if (lane_id() == 0)
            o = __hip_atomic_fetch_add(&s_grab_ord, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        o = (uint32_t)__builtin_amdgcn_readfirstlane(o);
        const uint32_t gshift = (uint32_t)__builtin_amdgcn_readfirstlane(s_grab_cfg[0]);
        const uint32_t n_groups = (uint32_t)__builtin_amdgcn_readfirstlane(s_grab_cfg[1]);
        const uint32_t k = o >> gshift, sub = o & ((1u << gshift) - 1);
        uint32_t g = ~0u;
        for (uint32_t spins = 0;; ++spins) {
            const uint64_t e = __hip_atomic_load(&s_grab_slot[k % kGrabSlots], __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_WORKGROUP);
            const uint32_t tag = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(e >> 32));
            if (tag == k) {
                g = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)e);
                break;
            }
            // fail-safe (never seen): a later group in the slot (this wave lagged a whole ring)
            // or ~1 s without a publisher -- stop, flag it, no hang.  ~0 tags: not yet written
            if ((tag != ~0u && (int32_t)(tag - k) > 0) || spins == kGrabSpinLimit) {
                if (err && lane_id() == 0) atomicOr(err, 1u);
                break;
            }
            __builtin_amdgcn_s_sleep(2);
        }
        const bool live = g < n_groups;
        if (sub == 0) {  // this wave grabs and publishes slot k + 1
            uint32_t nv = ~0u;
            if (live && lane_id() == 0) nv = atomicAdd(ctr, 1u);
            nv = (uint32_t)__builtin_amdgcn_readfirstlane(nv);
            if (lane_id() == 0)
                __hip_atomic_store(&s_grab_slot[(k + 1) % kGrabSlots], ((uint64_t)(k + 1) << 32) | nv,
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        if (RC_DIAG_FORCE_GRAB_STOP() && err) {  // diagnostic build: this unit is never run
            if (lane_id() == 0) atomicOr(err, 1u);
            return U.n_units;
        }
        return live ? U.nw + (g << gshift) + sub : U.n_units;
    }
};

// Persistent: one 1024-thread workgroup per CU, each wave its static unit, then dynamic units.
// G > 1: also grp[t] = the tile's group bounds (GroupRecord: the top-16 maximum of each of its
// G key groups, keys that do not exist counting as 0, and the maximum outside the lane holding
// it), upper bounds the chains use to leave most of an edge range unscanned (chain_step,
// rc_lane_chain_kernel).
//
// Tiles the fast path cannot settle -- a candidate lane holding its top-16 maximum twice --
// are listed per unit for the edge kernel: xlist[b + i] (i < xcount[u], b the unit's first
// tile).  Every tile stores its index at its unit's next slot and only a tie advances the count,
// so the store is unconditional and every tile keeps the same vector-memory sequence.
//
// The grab for a wave's next unit is issued when it enters a unit and read when it leaves it,
// so the atomic's latency hides behind the unit's tiles.  ctr must be 0 at launch.
template <int G, bool kGroup>
__global__ __launch_bounds__(1024) void rc_tile_kernel(const KeyTables *__restrict__ tab,
                                                       StreamDesc d, uint64_t n_streams,
                                                       TileUnits U,
                                                       TileRecord *__restrict__ rec,
                                                       GroupRecord *__restrict__ grp,
                                                       uint32_t hot,
                                                       uint32_t *__restrict__ xlist,
                                                       uint32_t *__restrict__ xcount,
                                                       uint32_t *__restrict__ ctr) {
    UnitGrab<kGroup> grab;
    grab.start(U, ctr);
    stage_tile_tables_nb(tab);
    grab.seed(U);
    __syncthreads();
    const uint64_t *full = reinterpret_cast<const uint64_t *>(s_tile_lds + kFullOff / 4);
    const uint64_t *tl = full, *th = full + 1024;
    const uint64_t n_tiles = U.n_tiles;

    const uint32_t lane = lane_id();
    const uint32_t lb_a = (lane & 31) * 4, lb_b = lb_a | 0x10000u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t gw = (uint64_t)blockIdx.x * (blockDim.x >> 6) + wave;
    uint32_t u = (uint32_t)gw, ub, ue;
    U.range(u, ub, ue);
    uint32_t n_ties = 0;
    RC_TILE_STAMP_BEGIN();

    // the first fast tile, possibly in a later unit (units without one list no ties)
    TileCursor<true, (G > 1)> cursor;
    TileRef cur;
    uint64_t t = ub;
    bool seek = true;
    for (;;) {
        if (t < ue) {
            if (seek) cursor.init(d, n_streams, t);
            seek = false;
            cur = cursor.at(t);
            if (cur.fast) break;
            ++t;
            continue;
        }
        if (lane == 0) xcount[u] = 0;
        u = grab.next(U, ctr, ctr + kGrabErrWord);
        if (u >= U.n_units) return;
        U.range(u, ub, ue);
        t = ub;
        seek = true;
    }
    u32x4 x[kTileIters];
    // the word before the first tile (tile 0 of a stream has none: key 0 is masked)
    uint32_t prev_word = ld_u32(cur.base + 4 * cur.j0 - (cur.j0 ? 4 : 0));
    {
        const __amdgpu_buffer_rsrc_t src = tile_rsrc(cur.base + 4 * cur.j0);
#pragma unroll
        for (int it = 0; it < kTileIters; ++it) {
            x[it] = ring_load(src, lane * 16, it);
            __builtin_amdgcn_sched_barrier(0);  // issue in ring order: the waits count on it
        }
    }
    // Records are produced one tile late: a tile's candidate words are loaded when it ends and
    // its exact keys are evaluated (and its record stored) at the end of the next tile, when the
    // loads have long landed.  Every tile issues the same vector-memory sequence (ring loads,
    // neighbour word, candidate words, one record store) so the compiler's in-order vmcnt
    // waits stay exact; the first store goes to the spare record at n_tiles.
    uint64_t pend_t = n_tiles;  // SGPRs: the pending tile,
    uint64_t pend_jm = 0;       // its first key | its top-16 maximum M << 48 (j0 < 2^44),
    uint64_t pend_mask = 0;     // a marker's candidate lanes, else the lanes holding a key
    uint32_t pend_st = 0;       // bit 31: a marker record, low bits: the stream
    uint32_t pend_lo = 0, pend_hi = 0, pend_jl = 0;  // per lane: its key's words and index

    // retire the pending tile: the first maximal exact key over the keys the lanes hold (those
    // whose top 16 bits are M), or the marker the edge kernel resolves
    auto retire = [&]() {
        const uint64_t k = full_key(tl, th, pend_lo, pend_hi);
        const bool ptie = pend_st >> 31;
        const uint64_t pj0 = pend_jm & ((1ull << 48) - 1);
        const uint32_t pm = (uint32_t)(pend_jm >> 48);
        const uint64_t hold = ptie ? 0 : pend_mask;
        // a marker carries what the edge kernel needs: candidate lanes, ~stream
        uint64_t bk = ptie ? pend_mask : 0, bj = kTieMark ^ (pend_st & 0x7fffffffu);
        const bool win = ((hold >> lane) & 1) && (uint32_t)(k >> 48) == pm &&
                         pj0 + pend_jl != 0;  // key 0 of a stream does not exist
        const uint64_t wm = __ballot(win);
        for (uint64_t m = wm; m; m &= m - 1) {  // usually one lane
            const int l = __builtin_ctzll(m);
            const uint64_t kl = lane_u64(k, l);
            const uint64_t jl = pj0 + (uint32_t)__builtin_amdgcn_readlane(pend_jl, l);
            if (m == wm || kl > bk || (kl == bk && jl < bj)) {
                bk = kl;
                bj = jl;
            }
        }
        if (lane == 0) {
            rec[pend_t].key = bk;
            rec[pend_t].j = bj;
        }
    };

    for (;;) {
        // the next fast tile: in this unit, else in the next units (grabbed ones)
        TileRef nx = cur;
        nx.fast = false;
        uint64_t tn = t + 1;
        uint32_t nu = u, nub = ub, nue = ue;
        for (;;) {
            if (tn < nue) {
                nx = cursor.at(tn);
                if (nx.fast) break;
                ++tn;
                continue;
            }
            if (nu != u && lane == 0) xcount[nu] = 0;  // a grabbed unit without a fast tile
            nu = grab.next(U, ctr, ctr + kGrabErrWord);
            if (nu >= U.n_units) {
                nu = u;  // no more work: cur is the wave's last tile
                break;
            }
            U.range(nu, nub, nue);
            tn = nub;
            if (tn < nue) cursor.init(d, n_streams, tn);
        }
        uint32_t top, fs, ls;
        uint32_t gpk[(G + 1) / 2];
        tile_scan<G>(cur, nx, x, prev_word, lb_a, lb_b, top, fs, ls, gpk);
        if constexpr (G > 1) {  // this tile's group bounds, stored now (no exact key needed)
            const GroupRecord g = tile_groups<G>(gpk, hot);
            if (lane == 0) grp[t] = g;
        }

        retire();

        // this tile: its largest top-16 value M; the lanes holding it are the candidates, and
        // every key that can reach M lies in a candidate lane's first slice holding M -- unless
        // a candidate holds M in two slices, or there are more than 16 candidates: then the
        // tile becomes a marker record and the edge kernel recomputes it from the candidate
        // lanes.  Otherwise lane 4q + k takes key k of the q-th candidate's slice; its exact key
        // is evaluated one tile later.
        const uint32_t M = wave_max_u32(top);
        const bool cand = top == M;
        const uint64_t cmask = __ballot(cand);
        const uint32_t nc = (uint32_t)__builtin_popcountll(cmask);
        const bool tie = __ballot(cand && fs != ls) != 0 || nc > 16;
        const uint32_t c0 = (uint32_t)__builtin_ctzll(cmask);
        const uint32_t f0 = (uint32_t)__builtin_amdgcn_readlane(fs, c0);
        uint32_t jl = f0 * 256 + c0 * 4 + (lane & 3);  // lanes past the last candidate: a copy
        if (!tie) {
            uint64_t m = cmask & (cmask - 1);
            for (uint32_t q = 1; m; m &= m - 1, ++q) {  // the other candidates (rare)
                const uint32_t c = (uint32_t)__builtin_ctzll(m);
                const uint32_t f = (uint32_t)__builtin_amdgcn_readlane(fs, c);
                if ((lane >> 2) == q) jl = f * 256 + c * 4 + (lane & 3);
            }
        }
        if (lane == 0) xlist[ub + n_ties] = (uint32_t)t;  // kept only if it is a tie
        n_ties += tie ? 1u : 0u;
        pend_t = t;
        pend_jm = cur.j0 | ((uint64_t)M << 48);
        pend_mask = tie ? cmask : (nc >= 16 ? ~0ull : (1ull << (4 * nc)) - 1);
        pend_st = (tie ? 0x80000000u : 0u) | (uint32_t)cur.s;
        pend_jl = jl;
        const uint8_t *q = cur.base + 4 * (cur.j0 + pend_jl);
        pend_lo = ld_u32(q - (cur.j0 + pend_jl ? 4 : 0));  // no read before the stream
        pend_hi = ld_u32(q);
        RC_TILE_STAMP_TILE();
        if (nu != u) {  // cur was its unit's last fast tile: close the unit's tie list
            if (lane == 0) xcount[u] = n_ties;
            n_ties = 0;
            u = nu;
            ub = nub;
            ue = nue;
        }
        if (!nx.fast) break;
        t = tn;
        cur = nx;
    }
    retire();
    if (lane == 0) {
        xcount[u] = n_ties;
        RC_TILE_STAMP_END(gw);
    }
}

__device__ __forceinline__ uint64_t stream_of_tile(const StreamDesc &d, uint64_t n_streams,
                                                   uint64_t t) {
    uint64_t lo = 0, hi = n_streams;
    while (hi - lo > 1) {
        const uint64_t mid = (lo + hi) >> 1;
        if (sload(d.tile_base + mid) <= t) lo = mid;
        else hi = mid;
    }
    return lo;
}

__device__ __forceinline__ void exact_tile(const uint64_t *tl, const uint64_t *th,
                                           const StreamDesc &d, uint64_t s, uint64_t t,
                                           TileRecord *rec, GroupRecord *grp) {
    const uint64_t j0 = (t - sload(d.tile_base + s)) * kTileKeys;
    const uint64_t jb = tile_key_end(j0, sload(d.len + s), sload(d.jneed + s));
    uint64_t bk = 0, bj = ~0ull;
    scan_ranges<kScanUnroll>(tl, th, sload_ptr(d.ptr + s), max(j0, (uint64_t)1), jb, 1, 0, bk, bj);
    wave_best(bk, bj);
    if (lane_id() == 0) {
        rec[t].key = bk;
        rec[t].j = bj;
        if (grp) grp[t] = GroupRecord{~0ull, {~0ull, ~0ull, ~0ull, ~0ull}, 0ull};  // no bounds
    }
}

// A tie tile of the fast path, from its marker: the first maximal exact key lies in one of the
// candidate lanes (lanes whose top-16 maximum is the tile's, i.e. every key that can reach the
// tile's maximum), so the wave evaluates those lanes' 64 keys each (edge lane i takes the
// lane's key k = i & 3 of iteration i >> 2: local index 256 (i >> 2) + 4 c + (i & 3)), loads of
// all (at most kTieLanes) candidates in flight together.  Key 0 of a stream does not exist.
constexpr int kTieLanes = 4;
__device__ __forceinline__ void exact_lanes(const uint64_t *tl, const uint64_t *th,
                                            const StreamDesc &d, uint64_t s, uint64_t t,
                                            uint64_t lanes, TileRecord *rec) {
    const uint64_t j0 = (t - sload(d.tile_base + s)) * kTileKeys;
    const uint8_t *base = sload_ptr(d.ptr + s);
    const uint32_t i = lane_id();
    const uint64_t local = (i >> 2) * 256 + (i & 3);
    uint32_t lo[kTieLanes], hi[kTieLanes];
    uint64_t jj[kTieLanes];
    uint64_t m = lanes;
#pragma unroll
    for (int q = 0; q < kTieLanes; ++q) {
        const uint32_t c = m ? (uint32_t)__builtin_ctzll(m) : 0u;
        const uint64_t j = j0 + local + 4 * c;
        const uint8_t *p = base + 4 * j;
        lo[q] = ld_u32(j ? p - 4 : p);  // never a read before the stream
        hi[q] = ld_u32(p);
        jj[q] = (m && j) ? j : ~0ull;
        m &= m - 1;
    }
    uint64_t bk = 0, bj = ~0ull;
#pragma unroll
    for (int q = 0; q < kTieLanes; ++q)
        if (jj[q] != ~0ull) take_best(full_key(tl, th, lo[q], hi[q]), jj[q], bk, bj);
    wave_best(bk, bj);
    if (lane_id() == 0) {
        rec[t].key = bk;
        rec[t].j = bj;
    }
}

// Exact tiles, one wave per item, grid-strided: items 0 .. n_waves - 1 are the tie lists of
// the tile kernel's waves (xlist / xcount), the rest the host's list of tiles the fast path
// does not take (tile_fast: the stream ends inside the tile; d.xtiles).  Each is recomputed
// over the same key range the fast path would have covered (tile_key_end).
__global__ __launch_bounds__(256) void rc_edge_kernel(const KeyTables *__restrict__ tab,
                                                      StreamDesc d, uint64_t n_streams,
                                                      TileUnits U,
                                                      TileRecord *__restrict__ rec,
                                                      GroupRecord *__restrict__ grp,
                                                      const uint32_t *__restrict__ xlist,
                                                      const uint32_t *__restrict__ xcount,
                                                      uint32_t *__restrict__ ctr, uint64_t epoch) {
    __shared__ __attribute__((aligned(16))) uint64_t s_full[2048];
    __shared__ uint32_t s_fault;
    // The tile kernel is done with its grab counter: zero it for the workspace's next launch
    // (round 3: replaces a hipMemsetAsync between consecutive tile kernels).  Its fail-safe flag
    // (UnitGrab::next) becomes this call's fault stamp -- which the chain kernels read -- and
    // the flag is cleared: workgroup 0 stores the stamp, counts the fault, then clears the flag
    // with release order, so a workgroup that reads the flag (acquire) either sees it set or
    // sees the stamp.  A faulted call's tie lists may be stale (units no wave ran never wrote
    // their counts), so then nothing is recomputed.
    if (threadIdx.x == 0) {
        uint32_t *err = ctr + kCtrErrWord;
        uint64_t *stamp = reinterpret_cast<uint64_t *>(ctr + kCtrStampWord);
        uint32_t f = __hip_atomic_load(err, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
        if (blockIdx.x == 0) {
            *ctr = 0u;
            if (f) {
                __hip_atomic_store(stamp, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                atomicAdd(ctr + kCtrFaultsWord, 1u);
                __hip_atomic_store(err, 0u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
            }
        } else if (!f) {
            f = __hip_atomic_load(stamp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == epoch;
        }
        s_fault = f;
    }
    __syncthreads();
    if (s_fault) return;
    const uint64_t gw = (uint64_t)blockIdx.x * (blockDim.x >> 6) +
                        __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t nw = (uint64_t)gridDim.x * (blockDim.x >> 6);
    const uint64_t n_host = sload(d.xtiles);
    const uint64_t n_units = U.n_units;
    const uint64_t n_items = n_units + n_host;
    const uint32_t lane = lane_id();
    // Items (tie lists of the units, then the host's tiles) in runs of 64: the wave takes runs
    // gw, gw + nw, ...; lane l loads the count of item 64 c + l (one coalesced 256-byte load
    // per run) and one ballot says which have work (round 3: ~23 units per wave on config 2 --
    // one dependent load each was 10 us; round 5: ~1.4 M 3-tile units per config-2 launch,
    // so the loads must be coalesced -- a lane-strided run touched 64 cache lines).
    const uint64_t n_runs = (n_items + 63) / 64;
    auto needs = [&](uint64_t c) -> uint64_t {
        const uint64_t e = c * 64 + lane;
        const bool w = e < n_items && (e >= n_units || xcount[e] != 0);
        return __ballot(w);
    };
    // almost every workgroup has nothing to recompute: it leaves before staging the tables
    bool work = false;
    for (uint64_t c = gw; c < n_runs && !work; c += nw) work = needs(c) != 0;
    if (!__syncthreads_or(work)) return;
    const uint64_t *gfull = &tab->tl[0][0];
    for (uint32_t i = threadIdx.x; i < 2048u; i += blockDim.x) s_full[i] = gfull[i];
    __syncthreads();
    const uint64_t *tl = s_full, *th = s_full + 1024;
    for (uint64_t c = gw; c < n_runs; c += nw) {
        for (uint64_t m = needs(c); m; m &= m - 1) {
            const uint64_t e = c * 64 + (uint64_t)__builtin_ctzll(m);
            if (e < n_units) {
                uint32_t t0, t1;
                U.range((uint32_t)e, t0, t1);
                const uint32_t c = (uint32_t)__builtin_amdgcn_readfirstlane(xcount[e]);
                for (uint32_t i = 0; i < c; ++i) {
                    const uint64_t t = (uint32_t)__builtin_amdgcn_readfirstlane(xlist[t0 + i]);
                    // the marker the tile kernel left: candidate lanes, ~stream
                    const uint64_t lanes = sload(&rec[t].key), s = ~sload(&rec[t].j) & 0x7fffffffu;
                    if (__builtin_popcountll(lanes) <= kTieLanes)
                        exact_lanes(tl, th, d, s, t, lanes, rec);  // its group record stays valid
                    else  // e.g. constant data: every lane a candidate
                        exact_tile(tl, th, d, s, t, rec, grp);
                }
            } else {
                const uint64_t t = sload(d.xtiles + 1 + (e - n_units));
                exact_tile(tl, th, d, stream_of_tile(d, n_streams, t), t, rec, grp);
            }
        }
    }
}

// ----------------------------------------------------------------- phase B: chain kernels
//
// The cut chain is sequential (each chunk starts at the previous cut), but the transition
// next(s) depends on the position s only.  A stream whose argmax region spans several
// segments of `seg_bytes` is walked segment-parallel (SURVEY.md §8 e): every segment runs a
// SPECULATIVE chain from its own start g_i (4-aligned) through its segment and `ext_steps`
// chunks beyond; the join kernel then follows the true chain (segment 0's) and hops onto
// segment i's list at the first position both chains share -- from there the two are the
// same chain.  Chains normally meet within a chunk; if a list runs out first, the join kernel
// computes the missing steps itself, so the result is exact in every case.

// The call's fault stamp (rc_edge_kernel): its tile kernel took the fail-safe stop, so its
// records are incomplete.  Read once per wave at the start of every chain kernel (uniform over
// the grid: written before the launch); the kernels then walk nothing and every stream's count
// becomes kCountFault (fault_counts), which every host path reports as an error.
__device__ __forceinline__ bool call_faulted(const ChainParams &prm) {
    return prm.fault != nullptr && sload(prm.fault) == prm.epoch;
}
__device__ __forceinline__ void fault_counts(int64_t *counts, uint64_t n_streams) {
    for (uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; s < n_streams;
         s += (uint64_t)gridDim.x * blockDim.x)
        counts[s] = kCountFault;
}

struct ChainStream {
    const uint8_t *base;
    uint64_t L, P, tb0, nt, jmax;
    RC_DIAG_ONLY(bool diag;)
};

__device__ __forceinline__ ChainStream chain_stream(const StreamDesc &d, uint64_t s) {
    ChainStream st;
    st.base = sload_ptr(d.ptr + s);
    st.L = sload(d.len + s);
    st.P = sload(d.last + s);
    st.tb0 = sload(d.tile_base + s);
    st.nt = sload(d.tile_base + s + 1) - st.tb0;
    st.jmax = st.L >= 8 ? (st.L - 4) / 4 : 0;
    RC_DIAG_ONLY(st.diag = s == 0;)
    return st;
}

// Top-16 scan of the window's two partial edge tiles, keys [a0, b0] then [a1, b1] (either
// may be empty), with the conflict-free prefilter tables -- the tile kernel's inner loop on an
// unaligned key range: each lane takes 4 consecutive words per 256-key iteration, the word
// before a lane's first key comes from the previous lane by DPP.  Per lane: running maxima of
// (top16 << 16 | valid 0x8000 | order) for the first and the last occurrence; the order is the
// lane-local key index (0-255 head, 256-511 tail; a range holds at most 8190 keys).
#ifndef RC_EDGE_ITERS
#define RC_EDGE_ITERS 2
#endif
constexpr int kEdgeIters = RC_EDGE_ITERS;  // 256-key iterations whose loads are issued together

// One edge range [a, b] of keys scanned at top-16 precision in batches of kEdgeIters 256-key
// iterations: load() issues a batch's words, compute() folds them into the lane's running
// maxima.  Splitting the two lets a chain step put the record loads and both ranges' first
// batches in flight together (one memory round trip for a typical step).
struct EdgeRange {
    const uint8_t *p;     // word q0 of the stream
    uint64_t a, q0;       // first key, first word of iteration 0 (a & ~3)
    uint32_t nk, wlast;   // last key offset from q0, last existing word from q0
    uint32_t lo, span;    // valid key offsets: lo = a - q0 (0-3) .. nk, as off - lo <= span
    uint32_t it0;         // next iteration to load
    uint32_t carry;       // entry of the word before the next iteration's lane 0 key
    uint32_t carry_word;
    uint32_t R;           // 0 head / 1 tail (lane-local order 256*R + 4*it + k)
    bool live;

    __device__ void init(const uint8_t *base, uint64_t wmax, uint64_t a_, uint64_t b_, uint32_t R_) {
        R = R_;
        live = a_ <= b_;
        a = a_;
        q0 = a_ & ~3ull;
        nk = live ? (uint32_t)(b_ - q0) : 0;
        lo = (uint32_t)(a_ - q0);
        span = nk - lo;  // live: b >= a, so nk >= lo
        p = base + 4 * q0;
        wlast = live ? (uint32_t)(wmax - q0) : 0;
        it0 = 0;
        carry_word = 0;  // loaded with the first batch
        carry = 0;
    }
    __device__ bool more() const { return live && it0 * 256 <= nk; }
    // One 16-byte load per lane and iteration (1 KiB per wave instruction).  A lane's block is
    // clamped to the aligned block holding the last existing word: past the stream's end the
    // lane's keys are invalid anyway, and a 16-byte block that holds a stream byte cannot
    // cross a page, so the read is safe even with no padding after the stream.
    __device__ void load(uint32_t (&w)[kEdgeIters][4]) {
        const uint32_t lane = lane_id();
        if (it0 == 0) carry_word = ld_u32(q0 ? p - 4 : p);
#pragma unroll
        for (int i = 0; i < kEdgeIters; ++i) {
            const uint32_t o = min((it0 + i) * 256 + lane * 4, wlast & ~3u);
            const u32x4 v = *as_global_x4(p + 4 * o);
            w[i][0] = v.x;
            w[i][1] = v.y;
            w[i][2] = v.z;
            w[i][3] = v.w;
        }
    }
    // kCompact: entries from the chain kernels' single PF copy at `pf`; otherwise from the
    // tile kernel's 32x-replicated, conflict-free image
    template <bool kCompact>
    __device__ void compute(const uint32_t (&w)[kEdgeIters][4], uint32_t lb_a, uint32_t lb_b,
                            const uint32_t *pf, uint32_t &acc_first, uint32_t &acc_last) {
        const uint32_t lane = lane_id();
        if (it0 == 0) carry = kCompact ? pfc_entry(pf, carry_word) : pf_entry(carry_word, lb_a, lb_b);
#pragma unroll
        for (int i = 0; i < kEdgeIters; ++i) {
            const uint32_t it = it0 + i;
            uint32_t e0, e1, e2, e3;
            if constexpr (kCompact) {
                e0 = pfc_entry(pf, w[i][0]);
                e1 = pfc_entry(pf, w[i][1]);
                e2 = pfc_entry(pf, w[i][2]);
                e3 = pfc_entry(pf, w[i][3]);
            } else {
                uint32_t ad[16];
                pf_addrs(w[i][0], lb_a, lb_b, ad + 0);
                pf_addrs(w[i][1], lb_a, lb_b, ad + 4);
                pf_addrs(w[i][2], lb_a, lb_b, ad + 8);
                pf_addrs(w[i][3], lb_a, lb_b, ad + 12);
                e0 = pf_gather(ad + 0);
                e1 = pf_gather(ad + 4);
                e2 = pf_gather(ad + 8);
                e3 = pf_gather(ad + 12);
            }
            const uint32_t rot = __builtin_amdgcn_mov_dpp(e3, 0x13C, 0xf, 0xf, false);
            const uint32_t ep = lane == 0 ? carry : rot;
            carry = rot;
            const uint32_t t[4] = {(ep & 0xffff0000u) ^ (e0 << 16), (e0 & 0xffff0000u) ^ (e1 << 16),
                                   (e1 & 0xffff0000u) ^ (e2 << 16), (e2 & 0xffff0000u) ^ (e3 << 16)};
            // an iteration whose 256 keys are all in range (every one but the first and the
            // last, as a rule) skips the per-key test and folds two keys per v_max3
            const uint32_t it_lo = it * 256u, it_hi = it * 256u + 255u;
            if (it_lo >= lo && it_hi <= nk) {
                const uint32_t lf = 511u - 256u * R - it * 4u, ll = 256u * R + it * 4u;
                acc_first = max3_u32(acc_first, t[0] | 0x8000u | lf, t[1] | 0x8000u | (lf - 1u));
                acc_first = max3_u32(acc_first, t[2] | 0x8000u | (lf - 2u), t[3] | 0x8000u | (lf - 3u));
                acc_last = max3_u32(acc_last, t[0] | 0x8000u | ll, t[1] | 0x8000u | (ll + 1u));
                acc_last = max3_u32(acc_last, t[2] | 0x8000u | (ll + 2u), t[3] | 0x8000u | (ll + 3u));
                continue;
            }
            // one 32-bit compare per key: off < lo wraps above span
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const uint32_t off = it * 256 + lane * 4 + k;  // key q0 + off
                const bool valid = off - lo <= span;
                const uint32_t local = 256u * R + it * 4 + k;
                acc_first = max3_u32(acc_first, valid ? (t[k] | 0x8000u | (511u - local)) : 0u, 0u);
                acc_last = max3_u32(acc_last, valid ? (t[k] | 0x8000u | local) : 0u, 0u);
            }
        }
        it0 += kEdgeIters;
    }
};

enum : int { kStepStop = 0, kStepCut = 1, kStepTail1 = 2, kStepTail2 = 3 };

// Trim the key range [a, b] inside tile `te` to the groups whose top-16 maximum (gm: u16 per
// group) reaches tb16; an empty result becomes a > b.  Returns whether the range changed.
__device__ __forceinline__ bool trim_groups(uint64_t gm, uint64_t te, uint32_t tb16, uint64_t &a,
                                            uint64_t &b) {
    const uint64_t tj0 = te * kTileKeys;
    uint32_t ga = (uint32_t)((a - tj0) / kGroupKeys), gb = (uint32_t)((b - tj0) / kGroupKeys);
    const uint32_t ga0 = ga, gb0 = gb;
    while (ga <= gb && ((gm >> (16 * ga)) & 0xffffu) < tb16) ++ga;
    while (gb > ga && ((gm >> (16 * gb)) & 0xffffu) < tb16) --gb;
    if (ga > gb) {
        a = 1;
        b = 0;
        return true;
    }
    if (ga == ga0 && gb == gb0) return false;
    a = max(a, tj0 + (uint64_t)ga * kGroupKeys);
    b = min(b, tj0 + (uint64_t)(gb + 1) * kGroupKeys - 1);
    return true;
}

// A walker's window onto its stream's tile records, held in registers across chain steps:
// lane l of row u holds the record of stream tile c0 + 64u + l.  Consecutive windows overlap
// (a chunk advances by less than a window), so while the next step's tiles lie inside the
// cached span the step reads no memory at all for its records -- with windows of a few tiles
// (small max_length) a whole stream of up to 64R tiles is loaded once.  A step that needs
// tiles outside it reloads the span from its first needed tile (one round trip, as before).
template <int R>
struct RecCache {
    uint32_t c0 = 0, n = 0;  // cached stream tiles [c0, c0 + n) (a stream has < 2^32 tiles)
    TileRecord v[R];
    uint64_t g[R];           // group maxima of the same tiles (when the tile kernel made them)

    __device__ bool has(uint64_t t) const { return t >= c0 && t - c0 < n; }
    __device__ void load(const TileRecord *rec, const GroupRecord *grp, const ChainStream &st,
                         uint64_t lo) {
        c0 = (uint32_t)lo;
        n = (uint32_t)min(st.nt - lo, (uint64_t)64 * R);
        const uint64_t lane = lane_id();
#pragma unroll
        for (int u = 0; u < R; ++u)
            if ((uint64_t)64 * u < n) {
                const uint64_t t = st.tb0 + lo + min((uint64_t)64 * u + lane, n - 1);
                v[u] = rec[t];
                if (grp) g[u] = grp[t].max;
            }
    }
    __device__ TileRecord get(uint64_t t, uint64_t &gm) const {  // t uniform and cached
        const uint64_t off = t - c0;
        const int row = (int)(off >> 6), l = (int)(off & 63);
        TileRecord r = {0, 0};
        gm = ~0ull;
#pragma unroll
        for (int u = 0; u < R; ++u)
            if (u == row) {
                r.key = lane_u64(v[u].key, l);
                r.j = lane_u64(v[u].j, l);
                gm = lane_u64(g[u], l);
            }
        return r;
    }
    // (key desc, index asc) best of the cached records of tiles [t_lo, t_hi), per lane
    __device__ void reduce(uint64_t t_lo, uint64_t t_hi, uint64_t &bk, uint64_t &bj) const {
        const uint64_t lane = lane_id();
#pragma unroll
        for (int u = 0; u < R; ++u) {
            const uint64_t t = c0 + 64 * u + lane;
            if ((uint64_t)64 * u < n && t - c0 < n && t >= t_lo && t < t_hi && v[u].key != 0)
                take_best(v[u].key, v[u].j, bk, bj);
        }
    }
};


// One chain step from chunk start `pos` (< L): an argmax cut (adapters.cpp:59-69), or the tail
// rule's one or two final cuts (adapters.cpp:48-55), or stop (non-final wait / S7 UB).
// prm.max_steps == 0 is the raw single next_cut: c1 = the argmax offset, whatever its value.
template <int R>
__device__ int chain_step(const uint64_t *tl, const uint64_t *th, const uint32_t *pf,
                          const TileRecord *rec, const ChainStream &st, const ChainParams &prm,
                          RecCache<R> &cache, uint64_t pos, uint32_t lb_a, uint32_t lb_b,
                          uint64_t &c1, uint64_t &c2) {
    const uint64_t minl = prm.min_length, maxl = prm.max_length, T = prm.window;
    const bool single = prm.max_steps == 0;
    const uint64_t rem = st.L - pos;
    const bool argmax = single || (st.P >= pos && st.P - pos >= maxl) || rem >= 2 * maxl;
    if (prm.open && !argmax) return kStepStop;  // a non-final next_cut returns 0: wait
    if (argmax) {
        // window keys j in [pos/4 + 1, pos/4 + T]  (i = 4 .. < max, adapters.cpp:59): the full
        // tiles inside it come from their records (exact keys); the two partial edge tiles are
        // scanned at top-16 precision and only their candidates get exact keys -- and only if
        // they can beat the records (the records hold ~99 % of a default-size window).
        const uint64_t s4 = pos >> 2;
        const uint64_t ja = s4 + 1, jb = min(s4 + T, st.jmax);
        uint64_t bk = 0, bj = ~0ull;
        RC_STAMP(1);
        if (T > 0 && ja <= jb) {
            const uint64_t t_lo = (ja + kTileKeys - 1) / kTileKeys;
            const uint64_t t_hi = (jb + 1) / kTileKeys;
            uint64_t a0 = ja, b0 = jb, a1 = 1, b1 = 0;
            const bool have_rec = t_lo < t_hi;
            if (have_rec) {
                b0 = t_lo * kTileKeys - 1;
                a1 = t_hi * kTileKeys;
                b1 = jb;
            }
            // one round trip: the window's records and both edge tiles' records in flight
            EdgeRange r0, r1;
            r0.init(st.base, st.L / 4 - 1, a0, b0, 0);
            r1.init(st.base, st.L / 4 - 1, a1, b1, 1);
            uint32_t w0[kEdgeIters][4], w1[kEdgeIters][4];
            uint32_t acc_first = 0, acc_last = 0;
            // An edge range inside one tile needs no scan when that tile's record -- its FIRST
            // maximal key -- lies in the range (the first maximum of a set is the first maximum
            // of every subset holding it), or when the tile's keys are all 0 (never taken,
            // adapters.cpp:60-63).
            const bool one0 = r0.live && a0 / kTileKeys == b0 / kTileKeys;
            const bool one1 = r1.live && a1 / kTileKeys == b1 / kTileKeys;
            const uint64_t te0 = a0 / kTileKeys, te1 = a1 / kTileKeys;
            // the tiles this step reads records of: the window's full tiles and the edge tiles
            uint64_t need_lo = ~0ull, need_hi = 0;
            if (have_rec) {
                need_lo = t_lo;
                need_hi = t_hi - 1;
            }
            if (one0) {
                need_lo = min(need_lo, te0);
                need_hi = max(need_hi, te0);
            }
            if (one1) {
                need_lo = min(need_lo, te1);
                need_hi = max(need_hi, te1);
            }
            if (need_lo <= need_hi && !(cache.has(need_lo) && cache.has(need_hi)))
                cache.load(rec, prm.grp, st, need_lo);  // one round trip, edge records included
            // edge tiles past the span (windows wider than 64R tiles) come from memory, issued
            // together with the reload
            TileRecord er0 = {}, er1 = {};
            uint64_t gm0 = ~0ull, gm1 = ~0ull;
            const bool g0 = one0 && !cache.has(te0), g1 = one1 && !cache.has(te1);
            if (g0) {
                er0 = rec[st.tb0 + te0];
                if (prm.grp) gm0 = prm.grp[st.tb0 + te0].max;
            }
            if (g1) {
                er1 = rec[st.tb0 + te1];
                if (prm.grp) gm1 = prm.grp[st.tb0 + te1].max;
            }
            if (have_rec) {
                cache.reduce(t_lo, t_hi, bk, bj);
                if (t_hi > cache.c0 + cache.n)  // a window wider than the span
                    scan_records(rec, st.tb0 + max(cache.c0 + cache.n, t_lo), st.tb0 + t_hi, bk, bj);
            }
            if (one0 && !g0) er0 = cache.get(te0, gm0);
            if (one1 && !g1) er1 = cache.get(te1, gm1);
            wave_best(bk, bj);
            // Otherwise the record still bounds the range from above: the head range (indices
            // below every full tile's) cannot win when its bound is below the records' best,
            // the tail range (indices above) not even when it equals it (index asc breaks the
            // tie) -- and the final best is at least the records' best.
            if (one0 && (er0.key == 0 || (er0.j >= a0 && er0.j <= b0) || er0.key < bk)) {
                if (er0.key != 0 && er0.j >= a0 && er0.j <= b0) take_best(er0.key, er0.j, bk, bj);
                r0.live = false;
            }
            if (one1 && (er1.key == 0 || (er1.j >= a1 && er1.j <= b1) || er1.key <= bk)) {
                if (er1.key != 0 && er1.j >= a1 && er1.j <= b1) take_best(er1.key, er1.j, bk, bj);
                r1.live = false;
            }
            // With group maxima (small windows): a key group whose top-16 maximum is below bk's
            // top 16 bits holds no key >= bk, so it cannot win, head or tail; the range left to
            // scan is trimmed to its groups from the first to the last one that can.  The head
            // tile always holds the previous cut's key -- the maximum of the previous window --
            // so its record rarely settles the head; its groups after that key usually do.
            if (prm.grp) {
                const uint32_t tb16 = (uint32_t)(bk >> 48);
                if (one0 && r0.live && trim_groups(gm0, te0, tb16, a0, b0))
                    r0.init(st.base, st.L / 4 - 1, a0, b0, 0);
                if (one1 && r1.live && trim_groups(gm1, te1, tb16, a1, b1))
                    r1.init(st.base, st.L / 4 - 1, a1, b1, 1);
            }
            // the few ranges left are scanned: their first batches only now (a second round
            // trip for them; none at all for the rest)
            if (r0.more()) r0.load(w0);
            if (r1.more()) r1.load(w1);
            RC_STAMP(2);
            // a range's next batch is issued as soon as its registers are consumed, so the
            // other range's compute covers its latency
            for (;;) {
                const bool m0 = r0.more(), m1 = r1.more();
                if (!m0 && !m1) break;
                if (m0) {
                    r0.template compute<true>(w0, lb_a, lb_b, pf, acc_first, acc_last);
                    if (r0.more()) r0.load(w0);
                }
                if (m1) {
                    r1.template compute<true>(w1, lb_a, lb_b, pf, acc_first, acc_last);
                    if (r1.more()) r1.load(w1);
                }
            }
            RC_STAMP(3);
            const uint32_t m = wave_max_u32(acc_first);
            if ((m & 0x8000u) && (m >> 16) >= (uint32_t)(bk >> 48)) {
                const bool cand = (acc_first >> 16) == (m >> 16) && (acc_first & 0x8000u);
                const uint32_t fl = 511u - (acc_first & 0x1ffu), ll = acc_last & 0x1ffu;
                if (__any(cand && fl != ll)) {
                    // a candidate lane holds its top-16 maximum twice: exact scan of the edges
                    uint64_t ek = 0, ej = ~0ull;
                    scan_ranges<kChainScanUnroll>(tl, th, st.base, a0, b0, a1, b1, ek, ej);
                    take_best(ek, ej, bk, bj);
                    wave_best(bk, bj);
                } else {
                    const uint32_t lo = fl & 255u;  // lane-local index within its range
                    const uint64_t jc = ((fl < 256 ? a0 : a1) & ~3ull) + 256ull * (lo >> 2) +
                                        4ull * lane_id() + (lo & 3);
                    const uint64_t jl = cand ? jc : (uint64_t)a0;  // any valid index
                    const uint64_t k = full_key(tl, th, ld_u32(st.base + 4 * jl - 4),
                                                ld_u32(st.base + 4 * jl));
                    for (uint64_t cm = __ballot(cand); cm; cm &= cm - 1) {
                        const int l = __builtin_ctzll(cm);
                        take_best(lane_u64(k, l), lane_u64(jl, l), bk, bj);
                    }
                }
            }
        }
        RC_STAMP(4);
        uint64_t idx = bk > 0 ? 4 * (bj - s4) : 0;
        if (idx < minl) idx = (minl + 3) & ~3ull;  // adapters.cpp:66-67
        if (single) {
            c1 = idx;
            return kStepCut;
        }
        if (idx != 0) {
            c1 = pos + idx;
            return kStepCut;
        }
        if (rem >= 2 * maxl || prm.open) return kStepStop;  // min_length == 0 (S7 UB)
    }
    uint64_t c;
    if (rem <= maxl) c = rem;
    else if (rem < maxl + minl) c = rem / 2;
    else c = maxl;
    if (c == 0) return kStepStop;
    c1 = pos + c;
    if (c < rem) {
        c2 = st.L;
        return kStepTail2;
    }
    return kStepTail1;
}

// ---- the chain step for small windows (prm.lean): the same decisions as chain_step, with the
// window's tiles in the one cached record row and key indices in 32 bits (streams below
// 16 GiB).  chain_step's 64-bit uniform compares are VALU instructions on gfx950 (there is no
// 64-bit SALU compare) and its live ranges spill SGPRs to VGPR lanes; at ~25 steps per 1 MiB
// stream that overhead, not memory, set the chain's time (rocprofv3 SQ counters,
// profiles/r02/chain_pmc_3iii_groups.txt).

__device__ __forceinline__ bool ge64(uint64_t a, uint32_t b) {  // a >= b with SALU compares
    return (uint32_t)(a >> 32) != 0u || (uint32_t)a >= b;
}

__device__ __forceinline__ void take_best32(uint64_t k, uint32_t j, uint64_t &bk, uint32_t &bj) {
    if (k > bk || (k == bk && j < bj)) {
        bk = k;
        bj = j;
    }
}

// trim_groups on 32-bit indices: the range [a, b] inside tile te, emptied as a > b
__device__ __forceinline__ void trim_groups32(uint64_t gm, uint32_t te, uint32_t tb16,
                                              uint32_t &a, uint32_t &b) {
    const uint32_t tj0 = te * kTileKeys;
    uint32_t ga = (a - tj0) / kGroupKeys, gb = (b - tj0) / kGroupKeys;
    while (ga <= gb && ((gm >> (16 * ga)) & 0xffffu) < tb16) ++ga;
    while (gb > ga && ((gm >> (16 * gb)) & 0xffffu) < tb16) --gb;
    if (ga > gb) {
        a = 1;
        b = 0;
        return;
    }
    a = max(a, tj0 + ga * kGroupKeys);
    b = min(b, tj0 + (gb + 1) * kGroupKeys - 1);
}

__device__ int chain_step_small(const uint64_t *tl, const uint64_t *th, const uint32_t *pf,
                                const TileRecord *rec, const ChainStream &st,
                                const ChainParams &prm, RecCache<1> &cache, uint64_t pos,
                                uint32_t lb_a, uint32_t lb_b, uint64_t &c1, uint64_t &c2) {
    const uint32_t minl = (uint32_t)prm.min_length, maxl = (uint32_t)prm.max_length;
    const uint32_t T = (uint32_t)prm.window;
    const bool single = prm.max_steps == 0;
    const uint64_t rem = st.L - pos;
    const bool argmax = single || (st.P >= pos && ge64(st.P - pos, maxl)) || ge64(rem, 2 * maxl);
    if (prm.open && !argmax) return kStepStop;
    if (argmax) {
        const uint32_t s4 = (uint32_t)(pos >> 2), jmax = (uint32_t)st.jmax;
        const uint32_t ja = s4 + 1, jb = min(s4 + T, jmax);
        uint64_t bk = 0;
        uint32_t bj = ~0u;
        if (T > 0 && ja <= jb) {
            const uint32_t t_lo = (ja + kTileKeys - 1) / kTileKeys, t_hi = (jb + 1) / kTileKeys;
            const bool have_rec = t_lo < t_hi;
            uint32_t a0 = ja, b0 = jb, a1 = 1, b1 = 0;
            if (have_rec) {
                b0 = t_lo * kTileKeys - 1;
                a1 = t_hi * kTileKeys;
                b1 = jb;
            }
            const bool one0 = a0 <= b0 && a0 / kTileKeys == b0 / kTileKeys;
            const bool one1 = a1 <= b1 && a1 / kTileKeys == b1 / kTileKeys;
            const uint32_t te0 = a0 / kTileKeys, te1 = a1 / kTileKeys;
            uint32_t need_lo = have_rec ? t_lo : ~0u, need_hi = have_rec ? t_hi - 1 : 0u;
            if (one0) {
                need_lo = min(need_lo, te0);
                need_hi = max(need_hi, te0);
            }
            if (one1) {
                need_lo = min(need_lo, te1);
                need_hi = max(need_hi, te1);
            }
            if (need_lo <= need_hi && !(cache.has(need_lo) && cache.has(need_hi)))
                cache.load(rec, prm.grp, st, need_lo);  // covers them all: window + 2 <= 64 tiles
            const uint32_t lane = lane_id();
            const uint64_t key = cache.v[0].key;
            // the full tiles' best record: the lanes' key high words, then (on a tie) the low
            // words, then the lowest lane -- the lowest tile, hence the lowest index
            if (have_rec) {
                const uint32_t t = cache.c0 + lane;
                const bool inr = lane < cache.n && t >= t_lo && t < t_hi && key != 0;
                const uint32_t hi = inr ? (uint32_t)(key >> 32) : 0u;
                const uint32_t mhi = wave_max_u32(hi);
                const bool top = inr && hi == mhi;
                uint64_t m = __ballot(top);
                if (m & (m - 1)) {
                    const uint32_t lo = top ? (uint32_t)key : 0u;
                    const uint32_t mlo = wave_max_u32(lo);
                    m = __ballot(top && lo == mlo);
                }
                if (m) {
                    const int w = __builtin_ctzll(m);
                    bk = lane_u64(key, w);
                    bj = (uint32_t)__builtin_amdgcn_readlane((uint32_t)cache.v[0].j, w);
                }
            }
            uint64_t ek0 = 0, ek1 = 0, gm0 = ~0ull, gm1 = ~0ull;
            uint32_t ej0 = 0, ej1 = 0;
            if (one0) {
                const int l = (int)(te0 - cache.c0);
                ek0 = lane_u64(key, l);
                ej0 = (uint32_t)__builtin_amdgcn_readlane((uint32_t)cache.v[0].j, l);
                if (prm.grp) gm0 = lane_u64(cache.g[0], l);
            }
            if (one1) {
                const int l = (int)(te1 - cache.c0);
                ek1 = lane_u64(key, l);
                ej1 = (uint32_t)__builtin_amdgcn_readlane((uint32_t)cache.v[0].j, l);
                if (prm.grp) gm1 = lane_u64(cache.g[0], l);
            }
            // settle the edge ranges by their tiles' records, then trim them by the group
            // maxima (chain_step explains both rules)
            bool live0 = a0 <= b0, live1 = a1 <= b1;
            if (one0 && (ek0 == 0 || (ej0 >= a0 && ej0 <= b0) || ek0 < bk)) {
                if (ek0 != 0 && ej0 >= a0 && ej0 <= b0) take_best32(ek0, ej0, bk, bj);
                live0 = false;
            }
            if (one1 && (ek1 == 0 || (ej1 >= a1 && ej1 <= b1) || ek1 <= bk)) {
                if (ek1 != 0 && ej1 >= a1 && ej1 <= b1) take_best32(ek1, ej1, bk, bj);
                live1 = false;
            }
            if (prm.grp) {
                const uint32_t tb16 = (uint32_t)(bk >> 48);
                if (one0 && live0) {
                    trim_groups32(gm0, te0, tb16, a0, b0);
                    live0 = a0 <= b0;
                }
                if (one1 && live1) {
                    trim_groups32(gm1, te1, tb16, a1, b1);
                    live1 = a1 <= b1;
                }
            }
            if (live0 || live1) {
                if (!live0) {
                    a0 = 1;
                    b0 = 0;
                }
                if (!live1) {
                    a1 = 1;
                    b1 = 0;
                }
                EdgeRange r0, r1;
                r0.init(st.base, st.L / 4 - 1, a0, b0, 0);
                r1.init(st.base, st.L / 4 - 1, a1, b1, 1);
                uint32_t w0[kEdgeIters][4], w1[kEdgeIters][4];
                uint32_t acc_first = 0, acc_last = 0;
                if (r0.more()) r0.load(w0);
                if (r1.more()) r1.load(w1);
                for (;;) {
                    const bool m0 = r0.more(), m1 = r1.more();
                    if (!m0 && !m1) break;
                    if (m0) {
                        r0.template compute<true>(w0, lb_a, lb_b, pf, acc_first, acc_last);
                        if (r0.more()) r0.load(w0);
                    }
                    if (m1) {
                        r1.template compute<true>(w1, lb_a, lb_b, pf, acc_first, acc_last);
                        if (r1.more()) r1.load(w1);
                    }
                }
                const uint32_t m = wave_max_u32(acc_first);
                if ((m & 0x8000u) && (m >> 16) >= (uint32_t)(bk >> 48)) {
                    const bool cand = (acc_first >> 16) == (m >> 16) && (acc_first & 0x8000u);
                    const uint32_t fl = 511u - (acc_first & 0x1ffu), ll = acc_last & 0x1ffu;
                    if (__any(cand && fl != ll)) {
                        // a candidate lane holds its top-16 maximum twice: exact scan
                        uint64_t ek = 0, ej = ~0ull;
                        scan_ranges<kChainScanUnroll>(tl, th, st.base, a0, b0, a1, b1, ek, ej);
                        uint64_t bj64 = bj == ~0u ? ~0ull : bj;
                        take_best(ek, ej, bk, bj64);
                        wave_best(bk, bj64);
                        bj = (uint32_t)bj64;
                    } else {
                        const uint32_t lo = fl & 255u;  // lane-local index within its range
                        const uint32_t jc = ((fl < 256 ? a0 : a1) & ~3u) + 256u * (lo >> 2) +
                                            4u * lane + (lo & 3);
                        const uint32_t jl = cand ? jc : a0 <= b0 ? a0 : a1;  // any valid index
                        const uint64_t k = full_key(tl, th, ld_u32(st.base + 4ull * jl - 4),
                                                    ld_u32(st.base + 4ull * jl));
                        for (uint64_t cm = __ballot(cand); cm; cm &= cm - 1) {
                            const int l = __builtin_ctzll(cm);
                            take_best32(lane_u64(k, l),
                                        (uint32_t)__builtin_amdgcn_readlane(jl, l), bk, bj);
                        }
                    }
                }
            }
        }
        uint32_t idx = bk > 0 ? 4u * (bj - s4) : 0u;
        if (idx < minl) idx = (minl + 3) & ~3u;  // adapters.cpp:66-67
        if (single) {
            c1 = idx;
            return kStepCut;
        }
        if (idx != 0) {
            c1 = pos + idx;
            return kStepCut;
        }
        if (ge64(rem, 2 * maxl) || prm.open) return kStepStop;  // min_length == 0 (S7 UB)
    }
    uint64_t c;
    if (rem <= maxl) c = rem;
    else if (rem < (uint64_t)maxl + minl) c = rem / 2;
    else c = maxl;
    if (c == 0) return kStepStop;
    c1 = pos + c;
    if (c < rem) {
        c2 = st.L;
        return kStepTail2;
    }
    return kStepTail1;
}

__device__ __forceinline__ uint64_t find_index(const uint64_t *base_arr, uint64_t n, uint64_t v) {
    uint64_t lo = 0, hi = n;  // largest i with base_arr[i] <= v
    while (hi - lo > 1) {
        const uint64_t mid = (lo + hi) >> 1;
        if (sload(base_arr + mid) <= v) lo = mid;
        else hi = mid;
    }
    return lo;
}

// Spec kernel: one wave per segment.  A one-segment stream writes its final cuts directly;
// segment i of a longer stream writes its list to the scratch and its count (bit 63 set if the
// chain ended inside the list: tail rule or stop).
// Workgroups of kChainWaves walkers on 20 KiB of LDS.  R = rows of the record cache: 1 for
// windows of up to ~60 tiles (max_length below ~1 MB: a 1 MiB stream's records load once),
// 4 otherwise (a default window spans 313 tiles and reloads every step, as it must).
template <int R, bool kLean>
__global__ __launch_bounds__(kChainWaves * 64) void rc_spec_kernel(const KeyTables *__restrict__ tab,
                                                      StreamDesc d, uint64_t n_streams,
                                                      ChainParams prm, uint64_t n_segs,
                                                      const TileRecord *__restrict__ rec,
                                                      uint64_t *__restrict__ cuts,
                                                      int64_t *__restrict__ counts,
                                                      uint64_t *__restrict__ scratch,
                                                      uint64_t *__restrict__ seg_counts,
                                                      uint64_t *__restrict__ seg_rcount) {
    if (call_faulted(prm)) {  // the merge / scan / mark kernels after it return too
        fault_counts(counts, n_streams);
        return;
    }
    stage_chain_tables(tab);
    const uint32_t *pf = s_chain_lds;
    const uint64_t *full = reinterpret_cast<const uint64_t *>(s_chain_lds + 1024);
    const uint64_t *tl = full, *th = full + 1024;
    const uint32_t lane = lane_id();
    const uint32_t lb_a = (lane & 31) * 4, lb_b = lb_a | 0x10000u;
    const uint64_t q = (uint64_t)blockIdx.x * (blockDim.x >> 6) +
                       __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (q >= n_segs) return;
    const uint64_t s = find_index(d.seg_base, n_streams + 1, q);
    const uint64_t sb = sload(d.seg_base + s), nseg = sload(d.seg_base + s + 1) - sb;
    const uint64_t i = q - sb;
    ChainStream st = chain_stream(d, s);
    RC_DIAG_ONLY(st.diag = st.diag && i == (nseg > 8 ? 7 : 0);)  // one walker of stream 0 (mid)
    const bool direct = nseg == 1;
    uint64_t *out = direct ? cuts + sload(d.cut_base + s) : scratch + sload(d.scratch_base + s) + i * prm.seg_cap;
    const uint64_t cap = direct ? sload(d.cut_cap + s) : prm.seg_cap;
    const uint64_t seg_end = (i + 1) * prm.seg_bytes;
    const uint64_t steps = prm.max_steps == 0 ? 1 : prm.max_steps;

    uint64_t pos = i * prm.seg_bytes, n = 0, ext = 0;
    bool overflow = false, term = false;
    RecCache<R> cache;
    auto emit = [&](uint64_t c) {
        if (n >= cap) {
            overflow = true;
            return;
        }
        if (lane == 0) out[n] = c;
        ++n;
    };
    for (;;) {
        if (pos >= st.L || n >= steps) {
            term = true;
            break;
        }
        if (!direct && pos >= seg_end && ext++ >= prm.ext_steps) break;
        uint64_t c1 = 0, c2 = 0;
        int kind;
        if constexpr (kLean) {
            static_assert(R == 1, "the lean step works on the one-row cache");
            kind = chain_step_small(tl, th, pf, rec, st, prm, cache, pos, lb_a, lb_b, c1, c2);
        } else {
            kind = chain_step<R>(tl, th, pf, rec, st, prm, cache, pos, lb_a, lb_b, c1, c2);
        }
        if (kind == kStepStop) {
            term = true;
            break;
        }
        emit(c1);
        if (kind == kStepTail2) emit(c2);
        if (kind != kStepCut) {
            term = true;
            break;
        }
        if (overflow) break;
        pos = c1;
    }
    if (lane == 0) {
        if (direct) {
            counts[s] = overflow ? -1 : (int64_t)n;
        } else {
            // the count the scan reads, unless the merge kernel repairs (extends) this list
            const uint64_t v = overflow ? ~0ull : (n | (term ? (1ull << 63) : 0));
            seg_counts[q] = v;
            seg_rcount[q] = v;
        }
    }
}

// ---- the lane-per-stream chain (small windows, many single-segment streams)
//
// rc_spec_kernel walks one stream per WAVE: a step's decisions are scalar and its edge ranges
// are scanned by the whole wave.  With 1 MiB streams and an 80 KB max_length (config 3 iii:
// 65,536 streams x 22 steps) that is ~250 VALU + ~300 SALU per step and ~1.1 ms of a 13 ms
// batch, almost all of it the scan of the head range -- the rest of the previous cut's group,
// whose top-16 maximum is that cut's own key.  Here every LANE walks its own stream, and the
// group bounds (GroupRecord) settle the edge ranges without a scan:
//   * the window's full tiles come from their records (16-byte loads, all in flight together);
//   * a partial edge range is settled by its tile's record when the record lies in it, or
//     excluded when the record is below the best (head) or at most the best (tail) -- as in
//     chain_step;
//   * otherwise each group the range overlaps is excluded when its top-16 maximum is below
//     the best so far; when only the maximum's own lane l0 can reach it (the other lanes'
//     bound is below), the walking lane evaluates the keys of lane l0 in the range itself:
//     kTileIters / G iterations of 4 keys, one 16-byte load and the word before each;
//   * a group in which two lanes reach the bound (the window's maximum shares the previous
//     cut's group: ~2 % of steps) is scanned exactly by the whole wave, lane after lane.
// A key whose top 16 bits are below the best's cannot be >= it, so every rule is exact.
constexpr int kLaneFull = 8;  // widest window of the lane chain: window keys / kTileKeys <= 8
constexpr int kLaneIters = kTileIters / kTileGroups;  // tile-kernel iterations per group

// Group classification of one edge range [a, b] inside tile te: mk[q] = the lanes of group q
// whose keys the walking lane evaluates (its hot lanes, when the best so far reaches the hot
// threshold, at most kLaneHotMax of them), sc = the groups left to an exact scan (below the
// threshold, or more hot lanes); a group whose top-16 maximum is below the best needs neither.
constexpr uint32_t kLaneHotMax = 4;
constexpr int kLaneTasks = 2;  // (group, lane) tasks per round of the lane chain (even; 4: slower,
                               // every slot's scan is paid whether a lane has a task or not)

__device__ __forceinline__ void lane_groups(bool live, const GroupRecord &g, uint32_t te,
                                            uint32_t a, uint32_t b, uint32_t t16, uint32_t hot,
                                            uint64_t (&mk)[kTileGroups], uint32_t &sc) {
    sc = 0;
#pragma unroll
    for (int q = 0; q < kTileGroups; ++q) mk[q] = 0;
    if (!live) return;
    const uint32_t tj0 = te * kTileKeys;
    const uint32_t qa = (a - tj0) / kGroupKeys, qb = (b - tj0) / kGroupKeys;
#pragma unroll
    for (int q = 0; q < kTileGroups; ++q) {
        if ((uint32_t)q < qa || (uint32_t)q > qb) continue;
        if (((uint32_t)(g.max >> (16 * q)) & 0xffffu) < t16) continue;  // nothing reaches the best
        const uint32_t nh = (uint32_t)__popcll(g.hot[q]);
        if (t16 < hot || nh > kLaneHotMax || nh == 0) sc |= 1u << q;  // (nh 0: an exact tile's max)
        else mk[q] = g.hot[q];
    }
}

// top-16 of key j from the prefilter entries of its two words (gclmul.h)
__device__ __forceinline__ uint32_t top16_of(uint32_t e_lo_word, uint32_t e_hi_word) {
    return ((e_lo_word & 0xffff0000u) ^ (e_hi_word << 16)) >> 16;
}

// One lane's keys in one group: keys jq + 256 i .. jq + 256 i + 3 (i < kLaneIters), jq =
// the group's first key + 4 l -- one 16-byte block per iteration and the word before it.
struct LaneQuarter {
    uint32_t w[kLaneIters][5];  // the word before each block, then the block's 4 words
};

// Loads only the iterations holding a key of [a, b] (none when a > b).  A loaded block holds
// a key <= b <= jmax, hence a stream byte: it cannot cross a page.
__device__ __forceinline__ void lq_load(const uint8_t *base, uint32_t jq, uint32_t a, uint32_t b,
                                        LaneQuarter &x) {
#pragma unroll
    for (int i = 0; i < kLaneIters; ++i) {
        const uint32_t j4 = jq + 256 * i;
        u32x4 v = u32x4{0u, 0u, 0u, 0u};
        uint32_t p = 0;
        if (j4 <= b && j4 + 3 >= a) {
            v = *as_global_x4(base + 4ull * j4);
            p = ld_u32(base + 4ull * j4 - (j4 ? 4 : 0));
        }
        x.w[i][0] = p;
        x.w[i][1] = v.x;
        x.w[i][2] = v.y;
        x.w[i][3] = v.z;
        x.w[i][4] = v.w;
    }
}

// The candidate among the keys of x in [a, b]: the one with the largest top-16 value (from the
// prefilter) that reaches t16 -- a key with a smaller top-16 value is smaller -- and whether
// another key shares that value (then every key of the lane is evaluated exactly: rare).
struct LaneCand {
    bool have, tie;
    uint32_t ct, cj;
};

__device__ __forceinline__ LaneCand lq_scan(const uint32_t *pf, const LaneQuarter &x, uint32_t jq,
                                            uint32_t a, uint32_t b, uint32_t t16) {
    bool have = false, tie = false;
    uint32_t ct = 0, cj = 0;
#pragma unroll
    for (int i = 0; i < kLaneIters; ++i) {
        const uint32_t j4 = jq + 256 * i;
        if (!(j4 <= b && j4 + 3 >= a)) continue;
        uint32_t e[5];
#pragma unroll
        for (int k = 0; k < 5; ++k) e[k] = pfc_entry(pf, x.w[i][k]);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t j = j4 + k, t = top16_of(e[k], e[k + 1]);
            if (j >= a && j <= b && t >= t16) {
                if (!have || t > ct) {
                    have = true;
                    tie = false;
                    ct = t;
                    cj = j;
                } else if (t == ct) {
                    tie = true;
                }
            }
        }
    }
    return LaneCand{have, tie, ct, cj};
}

// Every key of lane jq's blocks in [a, b] exactly, its words read again (rolled: rare, small code)
__device__ __forceinline__ void lq_all(const uint64_t *tl, const uint64_t *th, const uint8_t *base,
                                       uint32_t jq, uint32_t a, uint32_t b, uint64_t &bk,
                                       uint32_t &bj) {
#pragma unroll 1
    for (uint32_t i = 0; i < 4 * kLaneIters; ++i) {
        const uint32_t j = jq + 256 * (i >> 2) + (i & 3);
        if (j >= a && j <= b)
            take_best32(full_key(tl, th, ld_u32(base + 4ull * j - 4), ld_u32(base + 4ull * j)), j, bk, bj);
    }
}

// Two lanes' candidates folded into (bk, bj): their words read again (cache hits, both in
// flight together) -- cheaper than carrying each candidate's words through the scan.
__device__ __forceinline__ void lq_fold(const uint64_t *tl, const uint64_t *th, const uint8_t *base,
                                        const LaneCand &c0, uint32_t jq0, uint32_t a0, uint32_t b0,
                                        const LaneCand &c1, uint32_t jq1, uint32_t a1, uint32_t b1,
                                        uint64_t &bk, uint32_t &bj) {
    uint32_t w00 = 0, w01 = 0, w10 = 0, w11 = 0;
    if (c0.have) {
        w00 = ld_u32(base + 4ull * c0.cj - 4);
        w01 = ld_u32(base + 4ull * c0.cj);
    }
    if (c1.have) {
        w10 = ld_u32(base + 4ull * c1.cj - 4);
        w11 = ld_u32(base + 4ull * c1.cj);
    }
    if (c0.have) take_best32(full_key(tl, th, w00, w01), c0.cj, bk, bj);
    if (c1.have) take_best32(full_key(tl, th, w10, w11), c1.cj, bk, bj);
    if (c0.tie) lq_all(tl, th, base, jq0, a0, b0, bk, bj);
    if (c1.tie) lq_all(tl, th, base, jq1, a1, b1, bk, bj);
}

// Best exact key over [a, b] of one stream by the whole wave, 64 * U keys per memory round trip.
template <int U>
__device__ __forceinline__ void scan_range(const uint64_t *tl, const uint64_t *th,
                                           const uint8_t *base, uint64_t a, uint64_t b,
                                           uint64_t &bk, uint64_t &bj) {
    const uint64_t lane = lane_id();
    for (uint64_t r = a; r <= b; r += 64 * U) {
        uint2 w[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t j = min(r + 64 * u + lane, b);
            w[u].x = ld_u32(base + 4 * j - 4);
            w[u].y = ld_u32(base + 4 * j);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t j = r + 64 * u + lane;
            if (j <= b) take_best(full_key(tl, th, w[u].x, w[u].y), j, bk, bj);
        }
    }
}

template <int F>  // full tiles per window held in flight (window keys / kTileKeys <= F)
__global__ __launch_bounds__(256) void rc_lane_chain_kernel(const KeyTables *__restrict__ tab,
                                                            StreamDesc d, uint64_t n_streams,
                                                            ChainParams prm,
                                                            const TileRecord *__restrict__ rec,
                                                            uint64_t *__restrict__ cuts,
                                                            int64_t *__restrict__ counts) {
    if (call_faulted(prm)) {
        fault_counts(counts, n_streams);
        return;
    }
    stage_chain_tables(tab);
    const uint32_t *pf = s_chain_lds;
    const uint64_t *full = reinterpret_cast<const uint64_t *>(s_chain_lds + 1024);
    const uint64_t *tl = full, *th = full + 1024;
    const uint32_t lane = lane_id();
    const uint64_t gid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (gid - lane >= n_streams) return;  // the whole wave is past the last stream
    const bool mine = gid < n_streams;
    const uint64_t s = mine ? gid : n_streams - 1;  // surplus lanes shadow the last stream, silent
    const GroupRecord *grp = prm.grp;
    const uint8_t *base = d.ptr[s];
    const uint64_t L = d.len[s], P = d.last[s];
    const uint64_t tb0 = d.tile_base[s], nt = d.tile_base[s + 1] - tb0;
    uint64_t *out = cuts + d.cut_base[s];
    const uint64_t cap = d.cut_cap[s];
    const uint32_t jmax = L >= 8 ? (uint32_t)((L - 4) / 4) : 0u;
    const uint32_t minl = (uint32_t)prm.min_length, maxl = (uint32_t)prm.max_length;
    const uint32_t T = (uint32_t)prm.window;
    // a stream tile's global index; the spare record at n_tiles for anything else (a safe
    // address for loads whose values are not used)
    auto gtile = [&](bool use, uint32_t t) -> uint64_t { return use && t < nt ? tb0 + t : prm.n_tiles; };

    uint64_t pos = 0, n = 0;
    bool walking = mine && L > 0 && prm.max_steps > 0, overflow = false;
    RC_DIAG_ONLY(const bool diag = gid < 64;)  // wave 0: per-phase stamps
    for (;;) {
        if (!__any(walking)) break;
        RC_LSTAMP(1);
        const uint64_t rem = L - pos;
        const bool argmax = (P >= pos && P - pos >= maxl) || rem >= 2ull * maxl;
        const uint32_t s4 = (uint32_t)(pos >> 2);
        const uint32_t ja = s4 + 1, jb = min(s4 + T, jmax);
        const bool win = walking && argmax && T > 0 && ja <= jb;
        // full tiles [t_lo, t_hi); head [a0, b0] inside tile te0, tail [a1, b1] inside tile te1
        const uint32_t t_lo = (ja + kTileKeys - 1) / kTileKeys, t_hi = (jb + 1) / kTileKeys;
        const uint32_t nf = win && t_hi > t_lo ? t_hi - t_lo : 0u;
        const uint32_t a0 = ja, b0 = min(jb, t_lo * kTileKeys - 1), te0 = ja / kTileKeys;
        const uint32_t a1 = t_hi * kTileKeys, b1 = jb, te1 = t_hi;
        bool live0 = win && ja < t_lo * kTileKeys;
        bool live1 = win && t_hi >= t_lo && jb >= a1;

        TileRecord fr[F];
#pragma unroll
        for (int i = 0; i < F; ++i) fr[i] = rec[gtile((uint32_t)i < nf, t_lo + i)];
        const TileRecord r0 = rec[gtile(live0, te0)], r1 = rec[gtile(live1, te1)];
        const GroupRecord g0 = grp[gtile(live0, te0)], g1 = grp[gtile(live1, te1)];
        // with them, the words of the previous cut's lane in the rest of its group (key s4 is
        // in tile te0 whenever the head range is not empty)
        const bool spec = live0;
        const uint32_t lc = (s4 & 255u) >> 2, qc = (s4 & (kTileKeys - 1)) / kGroupKeys;
        const uint32_t jqc = (s4 & ~(uint32_t)(kGroupKeys - 1)) + 4 * lc;
        LaneQuarter x[kLaneTasks];
        lq_load(base, jqc, spec ? a0 : 1u, spec ? b0 : 0u, x[0]);

        uint64_t bk = 0;
        uint32_t bj = ~0u;
#pragma unroll
        for (int i = 0; i < F; ++i)
            if ((uint32_t)i < nf && fr[i].key != 0) take_best32(fr[i].key, (uint32_t)fr[i].j, bk, bj);
        if (live0) {
            const uint32_t rj = (uint32_t)r0.j;
            const bool inr = r0.key != 0 && rj >= a0 && rj <= b0;
            if (inr) take_best32(r0.key, rj, bk, bj);
            if (r0.key == 0 || inr || r0.key < bk) live0 = false;
        }
        if (live1) {
            const uint32_t rj = (uint32_t)r1.j;
            const bool inr = r1.key != 0 && rj >= a1 && rj <= b1;
            if (inr) take_best32(r1.key, rj, bk, bj);
            if (r1.key == 0 || inr || r1.key <= bk) live1 = false;
        }
        uint32_t sc0, sc1;
        RC_LSTAMP(2);
        // tasks: the (group, lane) pairs to evaluate, as lane masks per group of the head's tile
        // (h) and the tail's (t), popped head first
        uint64_t h[kTileGroups], t[kTileGroups];
        lane_groups(live0, g0, te0, a0, b0, (uint32_t)(bk >> 48), prm.hot, h, sc0);
        lane_groups(live1, g1, te1, a1, b1, (uint32_t)(bk >> 48), prm.hot, t, sc1);
        static_assert(kTileGroups == 4, "the task queue below spells out four groups");
        auto any_task = [&]() { return (h[0] | h[1] | h[2] | h[3] | t[0] | t[1] | t[2] | t[3]) != 0; };
        // pops the next task as its lane's first key block jq and range [a, b] (a > b: none)
        auto task = [&](uint32_t &jq, uint32_t &a, uint32_t &b) {
            int r = -1;
            uint32_t q = 0, l = 0;
#define RC_POP(M, R, Q)                            \
    if (r < 0 && M) {                              \
        l = (uint32_t)__builtin_ctzll(M);          \
        M &= M - 1;                                \
        r = R;                                     \
        q = Q;                                     \
    }
            RC_POP(h[0], 0, 0) RC_POP(h[1], 0, 1) RC_POP(h[2], 0, 2) RC_POP(h[3], 0, 3)
            RC_POP(t[0], 1, 0) RC_POP(t[1], 1, 1) RC_POP(t[2], 1, 2) RC_POP(t[3], 1, 3)
#undef RC_POP
            a = 1, b = 0;
            if (r < 0) return;
            jq = (r ? te1 : te0) * kTileKeys + q * kGroupKeys + 4 * l;
            a = r ? a1 : a0;
            b = r ? b1 : b0;
        };

        // the lanes' keys, kLaneTasks tasks per round with their loads in flight together.
        // The first is, as a rule, the previous cut's own group and lane (that cut's key is the
        // maximum of the previous window): its words came with the records.
        bool first = false;
#define RC_FIRST(Q)                                              \
    if (spec && qc == Q && (h[Q] >> lc & 1u)) {                  \
        h[Q] &= ~(1ull << lc);                                   \
        first = true;                                            \
    }
        RC_FIRST(0) RC_FIRST(1) RC_FIRST(2) RC_FIRST(3)
#undef RC_FIRST
        uint32_t jq[kLaneTasks], ra[kLaneTasks], rb[kLaneTasks];
        jq[0] = jqc, ra[0] = first ? a0 : 1u, rb[0] = first ? b0 : 0u;
        for (;;) {
            if (!__any(first || any_task())) break;
#pragma unroll
            for (int k = 0; k < kLaneTasks; ++k) {
                if (k == 0 && first) continue;  // x[0] holds the previous cut's lane already
                task(jq[k], ra[k], rb[k]);
                lq_load(base, jq[k], ra[k], rb[k], x[k]);
            }
            const uint32_t t16 = (uint32_t)(bk >> 48);
            LaneCand c[kLaneTasks];
#pragma unroll
            for (int k = 0; k < kLaneTasks; ++k) c[k] = lq_scan(pf, x[k], jq[k], ra[k], rb[k], t16);
#pragma unroll
            for (int k = 0; k < kLaneTasks; k += 2)
                lq_fold(tl, th, base, c[k], jq[k], ra[k], rb[k], c[k + 1], jq[k + 1], ra[k + 1],
                        rb[k + 1], bk, bj);
            first = false;
            RC_LSTAMP(3);
        }
        RC_LSTAMP(4);

        // groups with too many hot lanes, or a best below the threshold: exact scans by the whole
        // wave, one lane's range at a time
        // (from the first to the last such group of the range), a group per memory round trip
#pragma unroll 1
        for (int r = 0; r < 2; ++r) {
            const uint32_t sv = r == 0 ? +sc0 : +sc1;  // values, not a select of addresses
            const uint32_t te = r == 0 ? +te0 : +te1, ra = r == 0 ? +a0 : +a1, rb = r == 0 ? +b0 : +b1;
            uint32_t sa = 1, sb = 0;
            if (sv) {
                const uint32_t qlo = (uint32_t)__builtin_ctz(sv), qhi = 31u - (uint32_t)__builtin_clz(sv);
                sa = max(ra, te * kTileKeys + qlo * kGroupKeys);
                sb = min(rb, te * kTileKeys + (qhi + 1) * kGroupKeys - 1);
            }
            for (uint64_t m = __ballot(sa <= sb); m; m &= m - 1) {
                const int l = __builtin_ctzll(m);
                const uint32_t la = (uint32_t)__builtin_amdgcn_readlane(sa, l);
                const uint32_t lb = (uint32_t)__builtin_amdgcn_readlane(sb, l);
                const uint8_t *lbase = reinterpret_cast<const uint8_t *>(lane_u64((uint64_t)base, l));
                uint64_t ek = 0, ej = ~0ull;
                scan_range<kGroupKeys / 64>(tl, th, lbase, la, lb, ek, ej);
                wave_best(ek, ej);
                if (lane == (uint32_t)l && ek != 0) take_best32(ek, (uint32_t)ej, bk, bj);
                RC_LSTAMP(5);
            }
        }
        RC_LSTAMP(6);

        // the step's cut(s): chain_step_small's decisions (adapters.cpp:48-69)
        if (walking) {
            int kind = kStepStop;
            uint64_t c1 = 0, c2 = 0;
            if (argmax) {
                uint32_t idx = bk > 0 ? 4u * (bj - s4) : 0u;
                if (idx < minl) idx = (minl + 3) & ~3u;  // adapters.cpp:66-67
                if (idx != 0) {
                    c1 = pos + idx;
                    kind = kStepCut;
                }
            }
            if (kind != kStepCut && !prm.open && !(argmax && rem >= 2ull * maxl)) {
                uint64_t c;  // the tail rule (adapters.cpp:48-55); argmax with idx 0 is S7 UB
                if (rem <= maxl) c = rem;
                else if (rem < (uint64_t)maxl + minl) c = rem / 2;
                else c = maxl;
                if (c != 0) {
                    c1 = pos + c;
                    kind = kStepTail1;
                    if (c < rem) {
                        c2 = L;
                        kind = kStepTail2;
                    }
                }
            }
            if (kind != kStepStop) {
                if (n < cap) out[n++] = c1;
                else overflow = true;
                if (kind == kStepTail2) {
                    if (n < cap) out[n++] = c2;
                    else overflow = true;
                }
            }
            if (kind != kStepCut || overflow) walking = false;
            pos = c1;
            if (pos >= L || n >= prm.max_steps) walking = false;
        }
    }
    if (mine) counts[s] = overflow ? -1 : (int64_t)n;
}

// ---- the quad-per-stream chain: the lane chain with four lanes per stream
//
// The lane chain runs one wave per SIMD on config 3 (iii) (65,536 lanes), so a step is ~14 us
// of mostly dependent instructions with nothing to overlap them.  Here a QUAD of lanes walks
// each stream: the steps are the same, but lane q of the quad loads the window's full-tile
// record q (and q + 4) and takes iteration q of every (group, lane) task -- one 16-byte block,
// the word before it and 4 keys, not 4 of each -- and the quad reduces records and candidates
// with two DPP quad_perm exchanges.  Four waves per SIMD hide each other's latency.
template <int kCtrl>
__device__ __forceinline__ uint32_t qperm32(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, kCtrl, 0xf, 0xf, true);
}
template <int kCtrl>
__device__ __forceinline__ uint64_t qperm64(uint64_t v) {
    return (uint64_t)qperm32<kCtrl>((uint32_t)(v >> 32)) << 32 | qperm32<kCtrl>((uint32_t)v);
}
// (key desc, index asc) best over the quad, in every lane of it
__device__ __forceinline__ void quad_best32(uint64_t &k, uint32_t &j) {
    {
        const uint64_t ko = qperm64<0xB1>(k);  // quad_perm [1, 0, 3, 2]
        const uint32_t jo = qperm32<0xB1>(j);
        if (ko > k || (ko == k && jo < j)) k = ko, j = jo;
    }
    {
        const uint64_t ko = qperm64<0x4E>(k);  // quad_perm [2, 3, 0, 1]
        const uint32_t jo = qperm32<0x4E>(j);
        if (ko > k || (ko == k && jo < j)) k = ko, j = jo;
    }
}

// One quad lane's iteration of a task: keys j4 .. j4 + 3 of the task's lane, j4 = jq + 256 q.
struct QuadIter {
    u32x4 v;     // the block
    uint32_t p;  // the word before it
};

__device__ __forceinline__ QuadIter qi_load(const uint8_t *base, uint32_t j4, uint32_t a,
                                            uint32_t b) {
    QuadIter x = {u32x4{0u, 0u, 0u, 0u}, 0u};
    if (j4 <= b && j4 + 3 >= a) {  // a block holding a key <= b <= jmax cannot cross a page
        x.v = *as_global_x4(base + 4ull * j4);
        x.p = ld_u32(base + 4ull * j4 - (j4 ? 4 : 0));
    }
    return x;
}

// Folds the iteration's keys in [a, b] whose top-16 value reaches t16 into (lk, lj): the exact
// key of the one with the largest top-16 value, or of all of them when two share it (rare).
__device__ __forceinline__ void qi_eval(const uint32_t *pf, const uint64_t *tl, const uint64_t *th,
                                        const uint8_t *base, const QuadIter &x, uint32_t j4,
                                        uint32_t a, uint32_t b, uint32_t t16, uint64_t &lk,
                                        uint32_t &lj) {
    if (!(j4 <= b && j4 + 3 >= a)) return;
    const uint32_t wd[5] = {x.p, x.v.x, x.v.y, x.v.z, x.v.w};
    uint32_t e[5];
#pragma unroll
    for (int k = 0; k < 5; ++k) e[k] = pfc_entry(pf, wd[k]);
    bool have = false, tie = false;
    uint32_t ct = 0, cj = 0, clo = 0, chi = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint32_t j = j4 + k, t = top16_of(e[k], e[k + 1]);
        const bool in = j >= a && j <= b && t >= t16;
        const bool take = in && (!have || t > ct);
        tie = take ? false : (tie || (in && t == ct));
        ct = take ? t : ct;
        cj = take ? j : cj;
        clo = take ? wd[k] : clo;
        chi = take ? wd[k + 1] : chi;
        have = have || in;
    }
    if (have) take_best32(full_key(tl, th, clo, chi), cj, lk, lj);
    if (tie) {
#pragma unroll 1
        for (uint32_t k = 0; k < 4; ++k) {
            const uint32_t j = j4 + k;
            if (j >= a && j <= b)
                take_best32(full_key(tl, th, ld_u32(base + 4ull * j - 4), ld_u32(base + 4ull * j)), j, lk, lj);
        }
    }
}

constexpr int kQuadTasks = 4;  // (group, lane) tasks per round of the quad chain

template <int F>  // full tiles per window (window keys / kTileKeys <= F; F / 4 records per lane)
__global__ __launch_bounds__(256) void rc_quad_chain_kernel(const KeyTables *__restrict__ tab,
                                                            StreamDesc d, uint64_t n_streams,
                                                            ChainParams prm,
                                                            const TileRecord *__restrict__ rec,
                                                            uint64_t *__restrict__ cuts,
                                                            int64_t *__restrict__ counts) {
    static_assert(F % 4 == 0 && kLaneIters == 4, "a quad lane per record row and per iteration");
    if (call_faulted(prm)) {
        fault_counts(counts, n_streams);
        return;
    }
    stage_chain_tables(tab);
    const uint32_t *pf = s_chain_lds;
    const uint64_t *full = reinterpret_cast<const uint64_t *>(s_chain_lds + 1024);
    const uint64_t *tl = full, *th = full + 1024;
    const uint32_t lane = lane_id(), q = lane & 3u;
    const uint64_t gid = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 2;  // the stream
    if (gid - (lane >> 2) >= n_streams) return;  // the whole wave is past the last stream
    const bool mine = gid < n_streams;
    const uint64_t s = mine ? gid : n_streams - 1;  // surplus quads shadow the last stream, silent
    const GroupRecord *grp = prm.grp;
    const uint8_t *base = d.ptr[s];
    const uint64_t L = d.len[s], P = d.last[s];
    const uint64_t tb0 = d.tile_base[s], nt = d.tile_base[s + 1] - tb0;
    uint64_t *out = cuts + d.cut_base[s];
    const uint64_t cap = d.cut_cap[s];
    const uint32_t jmax = L >= 8 ? (uint32_t)((L - 4) / 4) : 0u;
    const uint32_t minl = (uint32_t)prm.min_length, maxl = (uint32_t)prm.max_length;
    const uint32_t T = (uint32_t)prm.window;
    auto gtile = [&](bool use, uint32_t t) -> uint64_t { return use && t < nt ? tb0 + t : prm.n_tiles; };

    uint64_t pos = 0, n = 0;
    bool walking = mine && L > 0 && prm.max_steps > 0, overflow = false;
    RC_DIAG_ONLY(const bool diag = gid < 16 && q == 0;)  // wave 0
    for (;;) {
        if (!__any(walking)) break;
        RC_LSTAMP(1);
        const uint64_t rem = L - pos;
        const bool argmax = (P >= pos && P - pos >= maxl) || rem >= 2ull * maxl;
        const uint32_t s4 = (uint32_t)(pos >> 2);
        const uint32_t ja = s4 + 1, jb = min(s4 + T, jmax);
        const bool win = walking && argmax && T > 0 && ja <= jb;
        const uint32_t t_lo = (ja + kTileKeys - 1) / kTileKeys, t_hi = (jb + 1) / kTileKeys;
        const uint32_t nf = win && t_hi > t_lo ? t_hi - t_lo : 0u;
        const uint32_t a0 = ja, b0 = min(jb, t_lo * kTileKeys - 1), te0 = ja / kTileKeys;
        const uint32_t a1 = t_hi * kTileKeys, b1 = jb, te1 = t_hi;
        bool live0 = win && ja < t_lo * kTileKeys;
        bool live1 = win && t_hi >= t_lo && jb >= a1;

        TileRecord fr[F / 4];
#pragma unroll
        for (int i = 0; i < F / 4; ++i) {
            const uint32_t t = 4 * i + q;
            fr[i] = rec[gtile(t < nf, t_lo + t)];
        }
        const TileRecord r0 = rec[gtile(live0, te0)], r1 = rec[gtile(live1, te1)];
        const GroupRecord g0 = grp[gtile(live0, te0)], g1 = grp[gtile(live1, te1)];
        // the previous cut's lane in its group: iteration q of it
        const bool spec = live0;
        const uint32_t lc = (s4 & 255u) >> 2, qc = (s4 & (kTileKeys - 1)) / kGroupKeys;
        const uint32_t jqc = (s4 & ~(uint32_t)(kGroupKeys - 1)) + 4 * lc;
        QuadIter x[kQuadTasks];
        x[0] = qi_load(base, jqc + 256 * q, spec ? a0 : 1u, spec ? b0 : 0u);

        uint64_t bk = 0;
        uint32_t bj = ~0u;
#pragma unroll
        for (int i = 0; i < F / 4; ++i)
            if (4 * (uint32_t)i + q < nf && fr[i].key != 0) take_best32(fr[i].key, (uint32_t)fr[i].j, bk, bj);
        quad_best32(bk, bj);
        if (live0) {
            const uint32_t rj = (uint32_t)r0.j;
            const bool inr = r0.key != 0 && rj >= a0 && rj <= b0;
            if (inr) take_best32(r0.key, rj, bk, bj);
            if (r0.key == 0 || inr || r0.key < bk) live0 = false;
        }
        if (live1) {
            const uint32_t rj = (uint32_t)r1.j;
            const bool inr = r1.key != 0 && rj >= a1 && rj <= b1;
            if (inr) take_best32(r1.key, rj, bk, bj);
            if (r1.key == 0 || inr || r1.key <= bk) live1 = false;
        }
        uint32_t sc0, sc1;
        RC_LSTAMP(2);
        uint64_t h[kTileGroups], t[kTileGroups];
        lane_groups(live0, g0, te0, a0, b0, (uint32_t)(bk >> 48), prm.hot, h, sc0);
        lane_groups(live1, g1, te1, a1, b1, (uint32_t)(bk >> 48), prm.hot, t, sc1);
        static_assert(kTileGroups == 4, "the task queue below spells out four groups");
        auto any_task = [&]() { return (h[0] | h[1] | h[2] | h[3] | t[0] | t[1] | t[2] | t[3]) != 0; };
        auto task = [&](uint32_t &jq, uint32_t &a, uint32_t &b) {
            int r = -1;
            uint32_t g = 0, l = 0;
#define RC_POP(M, R, Q)                            \
    if (r < 0 && M) {                              \
        l = (uint32_t)__builtin_ctzll(M);          \
        M &= M - 1;                                \
        r = R;                                     \
        g = Q;                                     \
    }
            RC_POP(h[0], 0, 0) RC_POP(h[1], 0, 1) RC_POP(h[2], 0, 2) RC_POP(h[3], 0, 3)
            RC_POP(t[0], 1, 0) RC_POP(t[1], 1, 1) RC_POP(t[2], 1, 2) RC_POP(t[3], 1, 3)
#undef RC_POP
            a = 1, b = 0;
            if (r < 0) return;
            jq = (r ? te1 : te0) * kTileKeys + g * kGroupKeys + 4 * l;
            a = r ? a1 : a0;
            b = r ? b1 : b0;
        };
        bool first = false;
#define RC_FIRST(Q)                                              \
    if (spec && qc == Q && (h[Q] >> lc & 1u)) {                  \
        h[Q] &= ~(1ull << lc);                                   \
        first = true;                                            \
    }
        RC_FIRST(0) RC_FIRST(1) RC_FIRST(2) RC_FIRST(3)
#undef RC_FIRST
        uint32_t jq[kQuadTasks], ra[kQuadTasks], rb[kQuadTasks];
        jq[0] = jqc, ra[0] = first ? a0 : 1u, rb[0] = first ? b0 : 0u;
        for (;;) {
            if (!__any(first || any_task())) break;
            bool used[kQuadTasks];  // wave-uniform: a slot no quad of the wave fills is skipped
#pragma unroll
            for (int k = 0; k < kQuadTasks; ++k) {
                if (!(k == 0 && first)) {  // x[0] may hold the previous cut's lane already
                    task(jq[k], ra[k], rb[k]);
                    x[k] = qi_load(base, jq[k] + 256 * q, ra[k], rb[k]);
                }
                used[k] = __any(ra[k] <= rb[k]);
            }
            const uint32_t t16 = (uint32_t)(bk >> 48);
            uint64_t lk = 0;
            uint32_t lj = ~0u;
#pragma unroll
            for (int k = 0; k < kQuadTasks; ++k)
                if (used[k]) qi_eval(pf, tl, th, base, x[k], jq[k] + 256 * q, ra[k], rb[k], t16, lk, lj);
            quad_best32(lk, lj);
            if (lk != 0) take_best32(lk, lj, bk, bj);
            first = false;
            RC_LSTAMP(3);
        }
        RC_LSTAMP(4);

        // groups with too many hot lanes, or a best below the threshold: exact scans by the whole
        // wave, one stream's range at a time (ballot over the quads' first lanes)
#pragma unroll 1
        for (int r = 0; r < 2; ++r) {
            const uint32_t sv = r == 0 ? +sc0 : +sc1;
            const uint32_t te = r == 0 ? +te0 : +te1, ra_ = r == 0 ? +a0 : +a1, rb_ = r == 0 ? +b0 : +b1;
            uint32_t sa = 1, sb = 0;
            if (sv) {
                const uint32_t qlo = (uint32_t)__builtin_ctz(sv), qhi = 31u - (uint32_t)__builtin_clz(sv);
                sa = max(ra_, te * kTileKeys + qlo * kGroupKeys);
                sb = min(rb_, te * kTileKeys + (qhi + 1) * kGroupKeys - 1);
            }
            for (uint64_t m = __ballot(q == 0 && sa <= sb); m; m &= m - 1) {
                const int l = __builtin_ctzll(m);
                const uint32_t la = (uint32_t)__builtin_amdgcn_readlane(sa, l);
                const uint32_t lb = (uint32_t)__builtin_amdgcn_readlane(sb, l);
                const uint8_t *lbase = reinterpret_cast<const uint8_t *>(lane_u64((uint64_t)base, l));
                uint64_t ek = 0, ej = ~0ull;
                scan_range<kGroupKeys / 64>(tl, th, lbase, la, lb, ek, ej);
                wave_best(ek, ej);
                if ((lane >> 2) == ((uint32_t)l >> 2) && ek != 0) take_best32(ek, (uint32_t)ej, bk, bj);
                RC_LSTAMP(5);
            }
        }
        RC_LSTAMP(6);

        // the step's cut(s), the same in the four lanes; lane 0 of the quad stores them
        if (walking) {
            int kind = kStepStop;
            uint64_t c1 = 0, c2 = 0;
            if (argmax) {
                uint32_t idx = bk > 0 ? 4u * (bj - s4) : 0u;
                if (idx < minl) idx = (minl + 3) & ~3u;  // adapters.cpp:66-67
                if (idx != 0) {
                    c1 = pos + idx;
                    kind = kStepCut;
                }
            }
            if (kind != kStepCut && !prm.open && !(argmax && rem >= 2ull * maxl)) {
                uint64_t c;  // the tail rule (adapters.cpp:48-55); argmax with idx 0 is S7 UB
                if (rem <= maxl) c = rem;
                else if (rem < (uint64_t)maxl + minl) c = rem / 2;
                else c = maxl;
                if (c != 0) {
                    c1 = pos + c;
                    kind = kStepTail1;
                    if (c < rem) {
                        c2 = L;
                        kind = kStepTail2;
                    }
                }
            }
            if (kind != kStepStop) {
                if (n < cap) {
                    if (q == 0) out[n] = c1;
                    ++n;
                } else {
                    overflow = true;
                }
                if (kind == kStepTail2) {
                    if (n < cap) {
                        if (q == 0) out[n] = c2;
                        ++n;
                    } else {
                        overflow = true;
                    }
                }
            }
            if (kind != kStepCut || overflow) walking = false;
            pos = c1;
            if (pos >= L || n >= prm.max_steps) walking = false;
        }
    }
    if (mine && q == 0) counts[s] = overflow ? -1 : (int64_t)n;
}

// ---- parallel join of the speculative lists (multi-segment streams)
//
// Three small launches instead of one wave walking every segment of a stream in turn (one
// dependent memory round trip per hop: milliseconds for the ~800 segments of a 64 GiB
// stream):
//   merge  one wave per boundary k: the first position p >= g_k of list k-1 that is g_k itself
//          or an entry of list k -- where segment k-1's chain becomes segment k's;
//   scan   one wave per stream: the true chain is list 0 up to its merge point, then list 1
//          from there up to its own merge point, ...; slice lengths, prefix offsets, count;
//   copy   one wave per segment: its slice to the stream's cut array.
// Whenever that structure does not hold (no merge inside a list, a list that ends without the
// chain ending, merge points out of order) the stream is marked kNeedJoin and the sequential
// join below computes it exactly.
constexpr uint64_t kNoMerge = ~0ull;
constexpr int64_t kNeedJoin = -2;

// Repair (round 3): a boundary whose lists do not meet -- segment k-1's chain ran its
// extension steps past g_k without landing on a cut of segment k's -- is no longer a reason to
// walk the whole stream in sequence: the boundary's wave runs chain k-1 on from its last cut,
// appending to list k-1 (its capacity is sized for min-length chunks, far more than a chain
// needs), until a cut is g_k or one of list k's first 64 entries, or the chain ends or passes
// list k's last entry (tests/test_join_model.py restates the whole splice on the CPU).  Boundaries
// repair in parallel: each touches only its own list k-1 and writes the extended count to
// seg_rcount[q - 1] (merge and repair of other boundaries read the original seg_counts).
// Without a meeting within kRepairSteps the stream still takes the sequential join.
constexpr int kRepairSteps = 64;

template <int R>
__global__ __launch_bounds__(256) void rc_merge_kernel(const KeyTables *__restrict__ tab,
                                                       StreamDesc d, uint64_t n_streams,
                                                       ChainParams prm, uint64_t n_segs,
                                                       const TileRecord *__restrict__ rec,
                                                       uint64_t *__restrict__ scratch,
                                                       const uint64_t *__restrict__ seg_counts,
                                                       uint64_t *__restrict__ seg_merge,
                                                       uint64_t *__restrict__ seg_rcount,
                                                       bool repair) {
    if (call_faulted(prm)) return;  // the spec lists were never written (rc_spec_kernel)
    const uint32_t lane = lane_id();
    const uint64_t q = (uint64_t)blockIdx.x * (blockDim.x >> 6) +
                       __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    // no early return before the workgroup's barrier below: inactive waves just take part
    bool active = q < n_segs;
    uint64_t s = 0, k = 0, na = 0, nb = 0, g = 0, ca = ~0ull;
    uint64_t *A = nullptr;
    uint64_t bv = ~0ull, b_last = 0;
    uint64_t result = kNoMerge;
    if (active) {
        s = find_index(d.seg_base, n_streams + 1, q);
        const uint64_t sb = sload(d.seg_base + s), nseg = sload(d.seg_base + s + 1) - sb;
        k = q - sb;
        active = nseg > 1 && k > 0;
    }
    if (active) {
        A = scratch + sload(d.scratch_base + s) + (k - 1) * prm.seg_cap;
        const uint64_t *B = A + prm.seg_cap;
        ca = seg_counts[q - 1];
        const uint64_t cb = seg_counts[q];
        if (ca != ~0ull && cb != ~0ull) {
            na = ca & ~(1ull << 63);
            nb = cb & ~(1ull << 63);
            g = k * prm.seg_bytes;
            // list k-1's entries at or past g are its last few (the chain's extension)
            const uint64_t a0 = na > 64 ? na - 64 : 0;
            const uint64_t ai = a0 + lane;
            const uint64_t av = ai < na ? A[ai] : 0;
            bv = lane < nb ? B[lane] : ~0ull;
            b_last = lane_u64(bv, 63);
            uint64_t cm = __ballot(ai < na && av >= g);
            const bool whole = a0 == 0 || !(cm & 1ull);  // every entry >= g is in this window
            for (; whole && cm; cm &= cm - 1) {
                const int l = __builtin_ctzll(cm);
                const uint64_t p = lane_u64(av, l);
                if (p == g) {
                    result = (a0 + l + 1) | (0ull << 32);
                    break;
                }
                const uint64_t hit = __ballot(bv == p);
                if (hit) {
                    result = (a0 + l + 1) | ((uint64_t)(__builtin_ctzll(hit) + 1) << 32);
                    break;
                }
                if (nb > 64 && p > b_last) break;  // beyond the first 64 entries: let the walk do it
            }
        }
    }
    // repair only a live chain (not ended in list k-1) with a last cut to go on from, whose
    // meeting can be seen in list k's first 64 entries
    const bool need = active && result == kNoMerge && ca != ~0ull && (ca >> 63) == 0 && na > 0 &&
                      nb <= 64 && repair;
    if (__syncthreads_or(need)) {
        stage_chain_tables(tab);
        if (need) {
            const uint32_t *pf = s_chain_lds;
            const uint64_t *full = reinterpret_cast<const uint64_t *>(s_chain_lds + 1024);
            const uint64_t *tl = full, *th = full + 1024;
            const uint32_t lb_a = (lane & 31) * 4, lb_b = lb_a | 0x10000u;
            const ChainStream st = chain_stream(d, s);
            RecCache<R> cache;
            uint64_t n = na, pos = A[na - 1];
            // past list k's last entry the meeting is beyond what list k holds: give up there
            // (the sequential join takes the stream)
            const uint64_t b_end = nb ? lane_u64(bv, (int)nb - 1) : 0;
            bool term = false, over = false, past = false;
            for (int step = 0; step < kRepairSteps && result == kNoMerge && !over; ++step) {
                if (pos >= st.L) {
                    term = true;
                    break;
                }
                uint64_t c[2] = {0, 0};
                const int kind = chain_step<R>(tl, th, pf, rec, st, prm, cache, pos, lb_a, lb_b,
                                               c[0], c[1]);
                if (kind == kStepStop) {
                    term = true;
                    break;
                }
                const int nc = kind == kStepTail2 ? 2 : 1;
                for (int e = 0; e < nc && result == kNoMerge; ++e) {
                    if (n >= prm.seg_cap) {
                        over = true;
                        break;
                    }
                    if (lane == 0) A[n] = c[e];
                    ++n;
                    if (c[e] == g) {
                        result = n;
                        break;
                    }
                    const uint64_t hit = __ballot(bv == c[e]);
                    if (hit) result = n | ((uint64_t)(__builtin_ctzll(hit) + 1) << 32);
                    else if (c[e] > b_end) past = true;
                }
                if (past) break;
                if (kind != kStepCut) {
                    term = result == kNoMerge;  // the chain ended before the lists met
                    break;
                }
                pos = c[0];
            }
            if (lane == 0 && !over) seg_rcount[q - 1] = n | (term ? (1ull << 63) : 0);
            if (over) result = kNoMerge;
        }
    }
    if (active && lane == 0) seg_merge[q] = result;
}

__global__ __launch_bounds__(256) void rc_scan_kernel(StreamDesc d, uint64_t n_streams,
                                                      ChainParams prm,
                                                      const uint64_t *__restrict__ seg_counts,
                                                      const uint64_t *__restrict__ seg_merge,
                                                      const uint64_t *__restrict__ seg_rcount,
                                                      uint64_t *__restrict__ seg_off,
                                                      uint64_t *__restrict__ seg_slice,
                                                      int64_t *__restrict__ counts) {
    if (call_faulted(prm)) return;  // counts hold kCountFault (rc_spec_kernel): copy and join skip
    const uint32_t lane = lane_id();
    const uint64_t s = (uint64_t)blockIdx.x * (blockDim.x >> 6) +
                       __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (s >= n_streams) return;
    const uint64_t sb = sload(d.seg_base + s), nseg = sload(d.seg_base + s + 1) - sb;
    if (nseg <= 1) return;
    const uint64_t cap = sload(d.cut_cap + s);
    uint64_t carry = 0;
    int64_t entry = 0;  // the true chain's entry index into the last segment of the previous 64
    bool fail = false, ended = false;
    constexpr int64_t kNeg = INT64_MIN / 4;
    // every segment's slice is written (~0 past the chain's end): the copy kernel trusts it
    for (uint64_t k0 = 0; k0 < nseg; k0 += 64) {
        const uint64_t k = k0 + lane, q = sb + k;
        const bool valid = k < nseg;
        // a repaired list's extended count (its original count otherwise, see rc_spec_kernel)
        const uint64_t c = valid ? seg_rcount[q] : 0;
        const uint64_t m_in = valid && k > 0 ? seg_merge[q] : 0;
        const uint64_t m_out = k + 1 < nseg ? seg_merge[q + 1] : kNoMerge;
        const uint64_t n_k = c & ~(1ull << 63);
        const bool term = (c >> 63) != 0 && c != ~0ull;
        const bool ends = m_out == kNoMerge;
        const uint64_t hi = ends ? n_k : (m_out & 0xffffffffu);
        // Round 3: the entry into list k.  Boundary k says list k-1's first a_k entries lead to
        // list k's entry b_k; a chain that enters list k-1 at e >= a_k is past that meeting, where
        // the two lists are one chain, so it enters list k at b_k + (e - a_k) and takes nothing
        // from list k-1 (a speculative chain whose extension ran past the next segment's merge).
        // entry_k = max(b_k, entry_{k-1} + b_k - a_k): a max-plus recurrence, composed over the
        // wave as pairs (P, Q) meaning x -> max(P, x + Q).
        int64_t P = 0, Q = kNeg;  // segment 0: entry 0
        if (valid && k > 0 && m_in != kNoMerge) {
            P = (int64_t)(m_in >> 32);
            Q = P - (int64_t)(m_in & 0xffffffffu);
        }
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const int64_t pp = __shfl_up(P, off), qp = __shfl_up(Q, off);
            if (lane >= (uint32_t)off) {  // self after prev: x -> max(P, max(pp, x + qp) + Q)
                P = max(P, pp + Q);
                Q = max(qp + Q, kNeg);
            }
        }
        const int64_t e_k = max(P, entry + Q);
        const uint64_t lo = (uint64_t)e_k;
        bool bad = valid && (c == ~0ull || (k > 0 && m_in == kNoMerge) ||
                             (ends && (!term || lo > n_k)));
        // the chain reaches segment k only if no earlier segment ended it
        const uint64_t end_mask = ended ? 0 : __ballot(valid && ends && !bad);
        const uint64_t first_end = end_mask ? __builtin_ctzll(end_mask) : 64;
        const bool active = valid && !ended && lane <= first_end;
        const uint64_t bad_mask = __ballot(active && bad);
        if (bad_mask) {
            fail = true;
            break;
        }
        uint64_t len = active && hi > lo ? hi - lo : 0, x = len;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {  // inclusive prefix sum over the wave
            const uint64_t y = __shfl_up(x, off);
            if (lane >= (uint32_t)off) x += y;
        }
        if (active) {
            seg_off[q] = carry + x - len;
            seg_slice[q] = len ? (lo | (hi << 32)) : ~0ull;
        } else if (valid) {
            seg_slice[q] = ~0ull;
        }
        carry += lane_u64(x, 63);
        entry = (int64_t)lane_u64((uint64_t)e_k, 63);
        if (end_mask) ended = true;
    }
    if (lane == 0) counts[s] = fail ? kNeedJoin : carry > cap ? -1 : (int64_t)carry;
}

__global__ __launch_bounds__(256) void rc_copy_kernel(StreamDesc d, uint64_t n_streams,
                                                      ChainParams prm, uint64_t n_segs,
                                                      const uint64_t *__restrict__ scratch,
                                                      const uint64_t *__restrict__ seg_off,
                                                      const uint64_t *__restrict__ seg_slice,
                                                      uint64_t *__restrict__ cuts,
                                                      const int64_t *__restrict__ counts) {
    const uint32_t lane = lane_id();
    const uint64_t q = (uint64_t)blockIdx.x * (blockDim.x >> 6) +
                       __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (q >= n_segs) return;
    const uint64_t s = find_index(d.seg_base, n_streams + 1, q);
    const uint64_t sb = sload(d.seg_base + s), nseg = sload(d.seg_base + s + 1) - sb;
    if (nseg <= 1 || counts[s] < 0) return;
    const uint64_t sl = seg_slice[q];
    if (sl == ~0ull) return;
    const uint64_t lo = sl & 0xffffffffu, hi = sl >> 32;
    const uint64_t *src = scratch + sload(d.scratch_base + s) + (q - sb) * prm.seg_cap;
    uint64_t *dst = cuts + sload(d.cut_base + s) + seg_off[q];
    for (uint64_t i = lo + lane; i < hi; i += 64) dst[i - lo] = src[i];
}

// RC_JOIN_WALK=1 (tests, diagnostics): every multi-segment stream takes the sequential walk.
__global__ __launch_bounds__(256) void rc_mark_kernel(StreamDesc d, uint64_t n_streams,
                                                      ChainParams prm, int64_t *__restrict__ counts) {
    if (call_faulted(prm)) return;
    const uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (s < n_streams && sload(d.seg_base + s + 1) - sload(d.seg_base + s) > 1)
        counts[s] = kNeedJoin;
}

// Join kernel: one wave per multi-segment stream, following the true chain across the
// speculative lists (see above).  Only streams the scan marked kNeedJoin.
template <int R>
__global__ __launch_bounds__(256) void rc_join_kernel(const KeyTables *__restrict__ tab,
                                                      StreamDesc d, uint64_t n_streams,
                                                      ChainParams prm,
                                                      const TileRecord *__restrict__ rec,
                                                      uint64_t *__restrict__ cuts,
                                                      int64_t *__restrict__ counts,
                                                      const uint64_t *__restrict__ scratch,
                                                      const uint64_t *__restrict__ seg_counts) {
    const uint64_t s = (uint64_t)blockIdx.x * (blockDim.x >> 6) +
                       __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const bool need = s < n_streams && counts[s] == kNeedJoin;
    if (!__syncthreads_or(need)) return;  // the usual case: nothing to walk in this group
    stage_chain_tables(tab);
    if (!need) return;
    const uint32_t *pf = s_chain_lds;
    const uint64_t *full = reinterpret_cast<const uint64_t *>(s_chain_lds + 1024);
    const uint64_t *tl = full, *th = full + 1024;
    const uint32_t lane = lane_id();
    const uint32_t lb_a = (lane & 31) * 4, lb_b = lb_a | 0x10000u;
    const uint64_t sb = sload(d.seg_base + s), nseg = sload(d.seg_base + s + 1) - sb;
    const ChainStream st = chain_stream(d, s);
    uint64_t *out = cuts + sload(d.cut_base + s);
    const uint64_t cap = sload(d.cut_cap + s);
    const uint64_t *lists = scratch + sload(d.scratch_base + s);
    const uint64_t S = prm.seg_bytes;

    auto list_of = [&](uint64_t k) { return lists + k * prm.seg_cap; };
    auto count_of = [&](uint64_t k, bool &term, bool &bad) {
        const uint64_t c = seg_counts[sb + k];
        bad = c == ~0ull;
        term = (c >> 63) != 0;
        return c & ~(1ull << 63);
    };

    uint64_t pos = 0, n = 0, src = 0, idx = 0;
    bool overflow = false, src_term, bad;
    RecCache<R> cache;
    uint64_t src_cnt = count_of(0, src_term, bad);
    overflow |= bad;
    while (!overflow) {
        // bulk: the source list's entries below the next segment's start need no checks
        const uint64_t g_next = src + 1 < nseg ? (src + 1) * S : ~0ull;
        const uint64_t *lst = list_of(src);
        for (;;) {
            const uint64_t k = idx + lane;
            const uint64_t v = k < src_cnt ? lst[k] : ~0ull;
            const uint64_t take = __ballot(v < g_next);
            const uint32_t m = __popcll(take);  // sorted list: a prefix
            if (m == 0) break;
            if (n + m > cap) {
                overflow = true;
                break;
            }
            if (v < g_next) out[n + lane] = v;
            n += m;
            idx += m;
            pos = lane_u64(v, m - 1);
            if (m < 64) break;
        }
        if (overflow) break;
        if (idx >= src_cnt && src_term) break;  // the true chain ended inside this list
        // hop: is `pos` a position of a later segment's speculative chain?
        bool hopped = false;
        const uint64_t kmax = min(pos / S, nseg - 1);
        for (uint64_t k = src + 1; k <= kmax && !hopped; ++k) {
            bool kt, kb;
            const uint64_t kc = count_of(k, kt, kb);
            if (kb) {
                overflow = true;
                break;
            }
            if (pos == k * S) {  // the speculative start itself
                hopped = true;
                src = k;
                idx = 0;
                src_cnt = kc;
                src_term = kt;
                break;
            }
            const uint64_t *kl = list_of(k);
            for (uint64_t w = 0; w < kc; w += 64) {
                const uint64_t v = w + lane < kc ? kl[w + lane] : ~0ull;
                const uint64_t hit = __ballot(v == pos);
                if (hit) {
                    hopped = true;
                    src = k;
                    idx = w + __builtin_ctzll(hit) + 1;
                    src_cnt = kc;
                    src_term = kt;
                    break;
                }
                if (lane_u64(v, 63) > pos || w + 64 >= kc) break;  // sorted: no later match
            }
        }
        if (overflow) break;
        if (hopped) continue;
        // no hop: follow the current list one entry, or compute the step when it ran out
        if (idx < src_cnt) {
            const uint64_t v = lst[idx++];
            if (n >= cap) {
                overflow = true;
                break;
            }
            if (lane == 0) out[n] = v;
            ++n;
            pos = v;
            if (idx >= src_cnt && src_term) break;
            continue;
        }
        if (pos >= st.L) break;
        uint64_t c1 = 0, c2 = 0;
        const int kind = chain_step<R>(tl, th, pf, rec, st, prm, cache, pos, lb_a, lb_b, c1, c2);
        if (kind == kStepStop) break;
        if (n + (kind == kStepTail2 ? 2 : 1) > cap) {
            overflow = true;
            break;
        }
        if (lane == 0) {
            out[n] = c1;
            if (kind == kStepTail2) out[n + 1] = c2;
        }
        n += kind == kStepTail2 ? 2 : 1;
        if (kind != kStepCut) break;
        pos = c1;
        src_cnt = idx;  // nothing left to follow in the current list
    }
    if (lane == 0) counts[s] = overflow ? -1 : (int64_t)n;
}

// ---------------------------------------------------------------- read-bandwidth probe
//
// Calibration only (bench.py --calibrate): streams `nbytes` with exactly the tile kernel's
// access pattern -- persistent 1024-thread workgroups, each wave reading 16 KiB tiles through
// a 16-slot register ring of 16-byte nontemporal loads -- and XORs them.  Its rate is the
// streaming-read ceiling the tile kernel is compared against on the same box.
//
// block > 0 (diagnostics: the tile order): instead of one contiguous range per wave, the waves
// take runs of `block` consecutive tiles in turn (wave w: runs w, w + nw, ...), so at any moment
// the whole grid reads one window of nw * block tiles -- far fewer distinct pages in flight.
__device__ __forceinline__ uint64_t probe_tile(uint64_t k, uint64_t gw, uint64_t nw,
                                               uint64_t block) {
    return (k / block * nw + gw) * block + k % block;  // the k-th tile of wave gw
}

template <bool kGroup>
__global__ __launch_bounds__(1024) void rc_read_probe_kernel(const uint8_t *__restrict__ src,
                                                             uint64_t n_tiles,
                                                             uint32_t *__restrict__ out,
                                                             uint64_t block, TileUnits U,
                                                             uint32_t *__restrict__ ctr) {
    const uint32_t lane = lane_id();
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t gw = (uint64_t)blockIdx.x * (blockDim.x >> 6) + wave;
    const uint64_t nw = (uint64_t)gridDim.x * (blockDim.x >> 6);
    uint32_t acc = 0;
    if (block == 0) {
        // the tile kernel's schedule (TileUnits): the static unit, then grabbed units; the next
        // tile is known one tile ahead, so the ring never drains at a unit switch
        UnitGrab<kGroup> grab;
        grab.start(U, ctr);
        grab.seed(U);
        __syncthreads();
        uint32_t u = (uint32_t)gw, ub, ue;
        U.range(u, ub, ue);
        auto next_unit = [&]() -> bool {  // the wave's next non-empty unit, or false
            for (;;) {
                u = grab.next(U, ctr, nullptr);
                if (u >= U.n_units) return false;
                U.range(u, ub, ue);
                if (ub < ue) return true;
            }
        };
        if (ub >= ue && !next_unit()) return;
        uint64_t t = ub;
        u32x4 x[kTileIters];
        gu32x4 *p = as_global_x4(src + t * (uint64_t)kTileKeys * 4) + lane;
#pragma unroll
        for (int it = 0; it < kTileIters; ++it) {
            x[it] = RC_STREAM_LOAD(p + it * 64);
            __builtin_amdgcn_sched_barrier(0);
        }
        for (;;) {
            uint64_t tn = t + 1;
            bool more = true;
            if (tn >= ue) {
                more = next_unit();
                tn = more ? ub : t;
            }
            gu32x4 *q = as_global_x4(src + tn * (uint64_t)kTileKeys * 4) + lane;
#pragma unroll
            for (int it = 0; it < kTileIters; ++it) {
                const u32x4 w = x[it];
                acc = max3_u32(acc, w.x ^ w.y, w.z ^ w.w);
                x[it] = RC_STREAM_LOAD(q + it * 64);
            }
            if (!more) break;
            t = tn;
        }
        if (acc == 0x9E3779B9u) out[0] = acc;  // keeps the loads alive
        return;
    }
    uint64_t t = 0, t_end = 0;  // block > 0: k-th tile of this wave; tiles past n_tiles dropped
    while (probe_tile(t_end, gw, nw, block) < n_tiles) ++t_end;  // short: n_tiles / nw
    if (t >= t_end) return;
    u32x4 x[kTileIters];
    gu32x4 *p = as_global_x4(src + probe_tile(t, gw, nw, block) * (uint64_t)kTileKeys * 4) + lane;
#pragma unroll
    for (int it = 0; it < kTileIters; ++it) {
        x[it] = RC_STREAM_LOAD(p + it * 64);
        __builtin_amdgcn_sched_barrier(0);
    }
    for (; t < t_end; ++t) {
        const uint64_t tn = t + 1 < t_end ? t + 1 : t;
        gu32x4 *q = as_global_x4(src + probe_tile(tn, gw, nw, block) * (uint64_t)kTileKeys * 4) + lane;
#pragma unroll
        for (int it = 0; it < kTileIters; ++it) {
            const u32x4 w = x[it];
            acc = max3_u32(acc, w.x ^ w.y, w.z ^ w.w);
            x[it] = RC_STREAM_LOAD(q + it * 64);
        }
    }
    if (acc == 0x9E3779B9u) out[0] = acc;  // keeps the loads alive
}

// ---------------------------------------------------------------------- synthetic bytes

__global__ void rc_fill_kernel(uint8_t *__restrict__ dst, uint64_t nbytes, uint64_t base,
                               uint64_t word0) {
    const uint64_t nwords = nbytes / 8;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    uint64_t *w = reinterpret_cast<uint64_t *>(dst);
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nwords; i += stride)
        w[i] = splitmix64(base ^ (word0 + i));
    if (blockIdx.x == 0 && threadIdx.x < (nbytes & 7)) {
        const uint64_t v = splitmix64(base ^ (word0 + nwords));
        dst[nwords * 8 + threadIdx.x] = (uint8_t)(v >> (8 * threadIdx.x));
    }
}

// n streams of nbytes each, `slot` bytes apart (slot % 8 == 0, slot >= nbytes rounded up to 8:
// a stream's last word is written whole, into its slot's slack), stream k has id id0 + k*id_step
__global__ void rc_fill_streams_kernel(uint8_t *__restrict__ dst, uint64_t n, uint64_t nbytes,
                                       uint64_t slot, uint64_t seed, uint64_t id0,
                                       uint64_t id_step) {
    const uint64_t wps = (nbytes + 7) / 8, total = n * wps;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
        const uint64_t k = i / wps, w = i - k * wps;
        const uint64_t base = (seed * 0x9E3779B97F4A7C15ull) ^ ((id0 + k * id_step) << 34);
        reinterpret_cast<uint64_t *>(dst + k * slot)[w] = splitmix64(base ^ w);
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
                    uint64_t n_tiles, TileRecord *d_records, GroupRecord *d_grp,
                    uint32_t hot, uint32_t *d_xlist, uint32_t *d_ctr, uint64_t epoch,
                    void *stream, void *mid_event, uint32_t tile_cus, void *edge_stream,
                    void *tiled, TileSched sched) {
    hipStream_t st = (hipStream_t)stream;
    hipStream_t est = edge_stream ? (hipStream_t)edge_stream : st;
    // the edge kernel's stream follows the tile kernel (also when there are no tiles)
    auto hand_over = [&]() -> int {
        if (est == st) return 0;
        // `tiled` may be mid_event itself, already recorded after the tile kernel
        if ((tiled != mid_event && hipEventRecord((hipEvent_t)tiled, st) != hipSuccess) ||
            hipStreamWaitEvent(est, (hipEvent_t)tiled, 0) != hipSuccess) {
            snprintf(g_launch_err, sizeof g_launch_err, "edge stream hand-over failed");
            return 1;
        }
        return 0;
    };
    if (n_tiles == 0) {
        if (mid_event && hipEventRecord((hipEvent_t)mid_event, st) != hipSuccess) return 1;
        return hand_over();
    }
    const uint64_t waves_per_wg = 1024 / kWaveSize;
    uint64_t grid = (n_tiles + waves_per_wg - 1) / waves_per_wg;
    const uint64_t cus = tile_cus ? (uint64_t)tile_cus : (uint64_t)cu_count();
    if (grid > cus) grid = cus;  // persistent: one 144 KiB-LDS workgroup per CU
    const uint64_t n_waves = grid * waves_per_wg;
    const TileUnits U = tile_units(n_tiles, n_waves, sched);
    // the tie lists: n_tiles slots, one count per unit; d_ctr is 0 (the edge kernel re-zeros it)
    uint32_t *d_xcount = d_xlist + n_tiles;
    // workgroup grabs (RC_TILE_GROUP) are a kernel of their own: the per-wave kernel keeps
    // the round-4 code (the group protocol's registers cost the static harness 3.5 %,
    // profiles/r05/grab/)
    const bool grp = U.n_groups != 0;
    if (d_grp && grp)
        hipLaunchKernelGGL((rc_tile_kernel<kTileGroups, true>), dim3((unsigned)grid), dim3(1024), 0,
                           st, d_tables, desc, n_streams, U, d_records, d_grp, hot, d_xlist,
                           d_xcount, d_ctr);
    else if (d_grp)
        hipLaunchKernelGGL((rc_tile_kernel<kTileGroups, false>), dim3((unsigned)grid), dim3(1024),
                           0, st, d_tables, desc, n_streams, U, d_records, d_grp, hot, d_xlist,
                           d_xcount, d_ctr);
    else if (grp)
        hipLaunchKernelGGL((rc_tile_kernel<1, true>), dim3((unsigned)grid), dim3(1024), 0, st,
                           d_tables, desc, n_streams, U, d_records, d_grp, hot, d_xlist, d_xcount,
                           d_ctr);
    else
        hipLaunchKernelGGL((rc_tile_kernel<1, false>), dim3((unsigned)grid), dim3(1024), 0, st,
                           d_tables, desc, n_streams, U, d_records, d_grp, hot, d_xlist, d_xcount,
                           d_ctr);
    if (launch_status("rc_tile_kernel")) return 1;
    if (mid_event && hipEventRecord((hipEvent_t)mid_event, st) != hipSuccess) {
        snprintf(g_launch_err, sizeof g_launch_err, "hipEventRecord failed");
        return 1;
    }
    if (hand_over()) return 1;
    // one wave per tie list (almost always empty) and per host-listed tile, grid-strided
    uint64_t egrid = (U.n_units + 3) / 4;
    if (egrid > 4 * cus) egrid = 4 * cus;
    if (egrid == 0) egrid = 1;
    hipLaunchKernelGGL(rc_edge_kernel, dim3((unsigned)egrid), dim3(256), 0, est, d_tables, desc,
                       n_streams, U, d_records, d_grp, (const uint32_t *)d_xlist,
                       (const uint32_t *)d_xcount, d_ctr, epoch);
    return launch_status("rc_edge_kernel");
}

int rc_tile_schedule(uint64_t n_tiles, uint32_t waves, uint32_t permille, uint32_t chunk,
                     uint32_t dyn_min, uint32_t *ranges, uint64_t cap, uint64_t *n_units) {
    if (!n_units || waves == 0 || n_tiles >= (1ull << 32)) return 1;
    TileSched sched;
    sched.permille = permille;
    sched.chunk = chunk;
    sched.dyn_min = dyn_min;
    const TileUnits U = tile_units(n_tiles, waves, sched);
    *n_units = U.n_units;
    for (uint32_t u = 0; u < U.n_units && u < cap && ranges; ++u) U.range(u, ranges[2 * u], ranges[2 * u + 1]);
    return 0;
}

uint64_t rc_tie_list_words(uint64_t n_tiles) {
    // n_tiles list slots + one count per unit (static units: at most n_tiles + 15 waves;
    // dynamic: at most n_tiles / kDynChunkMin + 1)
    return 2 * n_tiles + n_tiles / kDynChunkMin + 64;
}

int rc_launch_chain(const KeyTables *d_tables, StreamDesc desc, uint64_t n_streams,
                    ChainParams prm, uint64_t n_segs, const TileRecord *d_records,
                    uint64_t *d_cuts, int64_t *d_counts, uint64_t *d_scratch,
                    uint64_t *d_seg_counts, bool any_multi, uint32_t join, void *stream) {
    if (n_streams == 0) return 0;
    hipStream_t st = (hipStream_t)stream;
    // many single-segment streams with small windows and group bounds: one lane per stream
    if (prm.lane && prm.lean && prm.grp && !any_multi && n_segs == n_streams &&
        prm.max_steps != 0 && prm.window / kTileKeys <= (uint64_t)kLaneFull) {
        const bool narrow = prm.window / kTileKeys <= 4;
        if (prm.lane == 3) {  // RC_LANE_CHAIN=lane: one lane per stream (comparison)
            const uint64_t grid = (n_streams + 255) / 256;
            if (narrow)
                hipLaunchKernelGGL(rc_lane_chain_kernel<4>, dim3((unsigned)grid), dim3(256), 0, st,
                                   d_tables, desc, n_streams, prm, d_records, d_cuts, d_counts);
            else
                hipLaunchKernelGGL(rc_lane_chain_kernel<kLaneFull>, dim3((unsigned)grid), dim3(256),
                                   0, st, d_tables, desc, n_streams, prm, d_records, d_cuts, d_counts);
            return launch_status("rc_lane_chain_kernel");
        }
        const uint64_t grid = (n_streams + 63) / 64;  // a quad of lanes per stream
        if (narrow)
            hipLaunchKernelGGL(rc_quad_chain_kernel<4>, dim3((unsigned)grid), dim3(256), 0, st,
                               d_tables, desc, n_streams, prm, d_records, d_cuts, d_counts);
        else
            hipLaunchKernelGGL(rc_quad_chain_kernel<kLaneFull>, dim3((unsigned)grid), dim3(256), 0,
                               st, d_tables, desc, n_streams, prm, d_records, d_cuts, d_counts);
        return launch_status("rc_quad_chain_kernel");
    }
    // 4-wave workgroups on 20 KiB of LDS (compact tables)
    const bool small = prm.window / kTileKeys + 3 <= 64;  // window + both edge tiles in one row
    const uint64_t grid = (n_segs + kChainWaves - 1) / kChainWaves;
    // d_seg_counts holds 5 arrays of n_segs: counts, merge points, slice offsets, slices and
    // the repaired counts
    uint64_t *seg_merge = d_seg_counts + n_segs, *seg_off = seg_merge + n_segs;
    uint64_t *seg_slice = seg_off + n_segs, *seg_rcount = seg_slice + n_segs;
    if (small && prm.lean)
        hipLaunchKernelGGL((rc_spec_kernel<1, true>), dim3((unsigned)grid),
                           dim3(kChainWaves * kWaveSize), 0, st, d_tables, desc, n_streams, prm,
                           n_segs, d_records, d_cuts, d_counts, d_scratch, d_seg_counts, seg_rcount);
    else if (small)
        hipLaunchKernelGGL((rc_spec_kernel<1, false>), dim3((unsigned)grid),
                           dim3(kChainWaves * kWaveSize), 0, st, d_tables, desc, n_streams, prm,
                           n_segs, d_records, d_cuts, d_counts, d_scratch, d_seg_counts, seg_rcount);
    else
        hipLaunchKernelGGL((rc_spec_kernel<kRecUnroll, false>), dim3((unsigned)grid),
                           dim3(kChainWaves * kWaveSize), 0, st, d_tables, desc, n_streams, prm,
                           n_segs, d_records, d_cuts, d_counts, d_scratch, d_seg_counts, seg_rcount);
    if (launch_status("rc_spec_kernel")) return 1;
    if (!any_multi) return 0;
    const uint64_t sgrid = (n_segs + 3) / 4, jgrid = (n_streams + kChainWaves - 1) / kChainWaves;
    if (!(join & RC_JOIN_WALK_ONLY)) {
        const bool repair = (join & RC_JOIN_REPAIR) != 0;
        if (small)
            hipLaunchKernelGGL(rc_merge_kernel<1>, dim3((unsigned)sgrid), dim3(256), 0, st,
                               d_tables, desc, n_streams, prm, n_segs, d_records, d_scratch,
                               (const uint64_t *)d_seg_counts, seg_merge, seg_rcount, repair);
        else
            hipLaunchKernelGGL(rc_merge_kernel<kRecUnroll>, dim3((unsigned)sgrid), dim3(256), 0,
                               st, d_tables, desc, n_streams, prm, n_segs, d_records, d_scratch,
                               (const uint64_t *)d_seg_counts, seg_merge, seg_rcount, repair);
        if (launch_status("rc_merge_kernel")) return 1;
        hipLaunchKernelGGL(rc_scan_kernel, dim3((unsigned)jgrid), dim3(kChainWaves * kWaveSize), 0,
                           st, desc, n_streams, prm, (const uint64_t *)d_seg_counts,
                           (const uint64_t *)seg_merge, (const uint64_t *)seg_rcount, seg_off,
                           seg_slice, d_counts);
        if (launch_status("rc_scan_kernel")) return 1;
        hipLaunchKernelGGL(rc_copy_kernel, dim3((unsigned)sgrid), dim3(256), 0, st, desc,
                           n_streams, prm, n_segs, (const uint64_t *)d_scratch,
                           (const uint64_t *)seg_off, (const uint64_t *)seg_slice, d_cuts,
                           (const int64_t *)d_counts);
        if (launch_status("rc_copy_kernel")) return 1;
    } else {
        hipLaunchKernelGGL(rc_mark_kernel, dim3((unsigned)jgrid), dim3(kChainWaves * kWaveSize), 0,
                           st, desc, n_streams, prm, d_counts);
        if (launch_status("rc_mark_kernel")) return 1;
    }
    if (small)
        hipLaunchKernelGGL(rc_join_kernel<1>, dim3((unsigned)jgrid), dim3(kChainWaves * kWaveSize),
                           0, st, d_tables, desc, n_streams, prm, d_records, d_cuts, d_counts,
                           (const uint64_t *)d_scratch, (const uint64_t *)d_seg_counts);
    else
        hipLaunchKernelGGL(rc_join_kernel<kRecUnroll>, dim3((unsigned)jgrid),
                           dim3(kChainWaves * kWaveSize), 0, st, d_tables, desc, n_streams, prm,
                           d_records, d_cuts, d_counts, (const uint64_t *)d_scratch,
                           (const uint64_t *)d_seg_counts);
    return launch_status("rc_join_kernel");
}

int rc_launch_read_probe(const uint8_t *d_src, uint64_t nbytes, uint32_t *d_out, uint32_t block,
                         TileSched sched, void *stream) {
    const uint64_t n_tiles = nbytes / ((uint64_t)kTileKeys * 4);
    if (n_tiles == 0) return 0;
    uint64_t grid = (n_tiles + 15) / 16;
    const uint64_t cus = (uint64_t)cu_count();
    if (grid > cus) grid = cus;
    // block (RC_PROBE_BLOCK, diagnostics): interleaved runs of tiles, static; otherwise the tile
    // kernel's schedule `sched` (d_out[1] is the grab counter)
    const TileUnits U = tile_units(n_tiles, grid * (1024 / kWaveSize), sched);
    if (block == 0 && U.n_units > U.nw &&
        hipMemsetAsync(d_out + 1, 0, sizeof(uint32_t), (hipStream_t)stream) != hipSuccess) {
        snprintf(g_launch_err, sizeof g_launch_err, "hipMemsetAsync failed");
        return 1;
    }
    if (U.n_groups)
        hipLaunchKernelGGL(rc_read_probe_kernel<true>, dim3((unsigned)grid), dim3(1024), 0,
                           (hipStream_t)stream, d_src, n_tiles, d_out, (uint64_t)block, U, d_out + 1);
    else
        hipLaunchKernelGGL(rc_read_probe_kernel<false>, dim3((unsigned)grid), dim3(1024), 0,
                           (hipStream_t)stream, d_src, n_tiles, d_out, (uint64_t)block, U, d_out + 1);
    return launch_status("rc_read_probe_kernel");
}

int rc_launch_fill_streams(uint8_t *d_dst, uint64_t n, uint64_t nbytes, uint64_t slot,
                           uint64_t seed, uint64_t id0, uint64_t id_step, void *stream) {
    if (n == 0 || nbytes == 0) return 0;
    const uint64_t words = n * ((nbytes + 7) / 8);
    uint64_t grid = (words + 255) / 256;
    if (grid > 65536) grid = 65536;
    hipLaunchKernelGGL(rc_fill_streams_kernel, dim3((unsigned)grid), dim3(256), 0,
                       (hipStream_t)stream, d_dst, n, nbytes, slot, seed, id0, id_step);
    return launch_status("rc_fill_streams_kernel");
}

int rc_launch_fill(uint8_t *d_dst, uint64_t nbytes, uint64_t seed, uint64_t stream_id,
                   uint64_t word0, void *stream) {
    if (nbytes == 0) return 0;
    const uint64_t base = (seed * 0x9E3779B97F4A7C15ull) ^ (stream_id << 34);
    uint64_t grid = (nbytes / 8 + 255) / 256;
    if (grid > 8192) grid = 8192;
    if (grid == 0) grid = 1;
    hipLaunchKernelGGL(rc_fill_kernel, dim3((unsigned)grid), dim3(256), 0, (hipStream_t)stream,
                       d_dst, nbytes, base, word0);
    return launch_status("rc_fill_kernel");
}

}  // extern "C"
