// blake2b.hip -- BLAKE2b digests of chunks on gfx950.
//
// What it replaces: the per-chunk `self.props.hash_digest(output_chunk)` of replicat's snapshot
// loop (/root/reference/replicat/repository.py:1462), i.e. `blake2b(length).digest(data)` =
// `hashlib.blake2b(data, digest_size=length).digest()` (replicat/utils/adapters.py:195-225;
// default length 64, repository.py:217).  hashlib's BLAKE2b is RFC 7693: unkeyed, no salt or
// personalisation, parameter block word 0 = 0x01010000 ^ digest_size.
//
// Shape of the work.  BLAKE2b is a chain over 128-byte blocks: one chunk's compressions are
// strictly sequential, so a chunk's latency is (#blocks) x (one compression's dependent
// instruction stream).  The only parallelism inside a compression is the four G functions of a
// column (or diagonal) step, so a QUAD of lanes hashes one chunk: lane q owns state column q
// (v[q], v[4+q], v[8+q], v[12+q]) and chaining words h[q], h[q+4].  The diagonal step rotates
// rows b/c/d by 1/2/3 lanes inside the quad with DPP quad_perm moves and back again -- 12 moves
// per round, no LDS.  A compression is ~600 VALU per lane instead of ~1900 for one lane per
// chunk, which is what bounds a 5 MB chunk (the critical path of config 2).
//
// The message schedule sigma makes lane q read word sigma[r][2q] (lane-dependent) in round r,
// so the block is staged in LDS (two ds_write_b128 per lane: lane q writes bytes 32q..32q+31)
// and each lane reads its four words per round through 40 precomputed LDS pointers.
//
// Loads: chunk starts are 4-aligned inside a stream except a stream's tail chunk, so every
// lane loads 9 dwords from its 4-aligned base and funnels them with v_alignbyte (a no-op shift
// when aligned).  Two blocks are kept in flight (one being hashed, the next two loaded).  The
// final block clamps its dword addresses to the last dword holding chunk bytes and masks the
// bytes past the chunk end: nothing beyond a chunk's last dword is ever read.
//
// Roofline: VALU issue, not HBM (64 GiB of chunks is ~1 TB/s of reads at the rates reached).

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "digest_kernels.h"

namespace {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
// chunk bytes are read through global-address-space pointers: flat loads would also count
// against lgkmcnt and make every LDS message read wait for the blocks in flight
#define GLOBAL __attribute__((address_space(1)))
typedef const GLOBAL uint8_t *gbytes;

constexpr uint64_t kIV[8] = {0x6a09e667f3bcc908ull, 0xbb67ae8584caa73bull, 0x3c6ef372fe94f82bull,
                             0xa54ff53a5f1d36f1ull, 0x510e527fade682d1ull, 0x9b05688c2b3e6c1full,
                             0x1f83d9abfb41bd6bull, 0x5be0cd19137e2179ull};

constexpr uint8_t kSigma[10][16] = {
    {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15},
    {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3},
    {11, 8, 12, 0, 5, 2, 15, 13, 10, 14, 3, 6, 7, 1, 9, 4},
    {7, 9, 3, 1, 13, 12, 11, 14, 2, 6, 5, 10, 4, 0, 15, 8},
    {9, 0, 5, 7, 2, 4, 10, 15, 14, 1, 11, 12, 6, 8, 3, 13},
    {2, 12, 6, 10, 0, 11, 8, 3, 4, 13, 7, 5, 15, 14, 1, 9},
    {12, 5, 1, 15, 14, 13, 4, 10, 0, 7, 6, 3, 9, 2, 8, 11},
    {13, 11, 7, 14, 12, 1, 3, 9, 5, 0, 15, 4, 8, 6, 2, 10},
    {6, 15, 14, 9, 11, 3, 0, 8, 12, 2, 13, 7, 1, 4, 10, 5},
    {10, 2, 8, 4, 7, 6, 1, 5, 15, 11, 9, 14, 3, 12, 13, 0}};

// word that lane q reads as message input k (0,1: column step; 2,3: diagonal step) in round r,
// packed 4 bits per lane so that one v_bfe per (r, k) extracts it
constexpr uint32_t sigma_pack(int r, int k) {
    uint32_t p = 0;
    for (int q = 0; q < 4; ++q) {
        const int idx = k < 2 ? 2 * q + k : 8 + 2 * q + (k - 2);
        p |= uint32_t(kSigma[r][idx]) << (4 * q);
    }
    return p;
}

// quad_perm controls: output lane j takes input lane perm[j]
constexpr int kRot1 = 0x39;  // [1,2,3,0]
constexpr int kRot2 = 0x4E;  // [2,3,0,1]
constexpr int kRot3 = 0x93;  // [3,0,1,2]

template <int C>
__device__ __forceinline__ uint64_t quad_perm(uint64_t x) {
    const uint32_t lo = __builtin_amdgcn_mov_dpp(static_cast<int>(x), C, 0xF, 0xF, true);
    const uint32_t hi = __builtin_amdgcn_mov_dpp(static_cast<int>(x >> 32), C, 0xF, 0xF, true);
    return (uint64_t(hi) << 32) | lo;
}

template <int N>
__device__ __forceinline__ uint64_t rotr(uint64_t x) {
    const uint32_t lo = static_cast<uint32_t>(x), hi = static_cast<uint32_t>(x >> 32);
    uint32_t rl, rh;
    if constexpr (N == 32) {
        rl = hi;
        rh = lo;
    } else if constexpr (N < 32) {
        rl = __builtin_amdgcn_alignbit(hi, lo, N);
        rh = __builtin_amdgcn_alignbit(lo, hi, N);
    } else {
        rl = __builtin_amdgcn_alignbit(lo, hi, N - 32);
        rh = __builtin_amdgcn_alignbit(hi, lo, N - 32);
    }
    return (uint64_t(rh) << 32) | rl;
}

__device__ __forceinline__ void g_mix(uint64_t &a, uint64_t &b, uint64_t &c, uint64_t &d,
                                      uint64_t x, uint64_t y) {
    a = a + b + x;
    d = rotr<32>(d ^ a);
    c = c + d;
    b = rotr<24>(b ^ c);
    a = a + b + y;
    d = rotr<16>(d ^ a);
    c = c + d;
    b = rotr<63>(b ^ c);
}

struct LaneCtx {
    const uint64_t *mp[10][4];  // this lane's message words, per round row and input
    uint64_t iv_c, iv_d;        // IV[q], IV[q+4]
    uint64_t t_mask, f_mask;    // ~0 on lane 0 (counter word v12) / lane 2 (final flag v14)
};

// One BLAKE2b compression of the quad's staged block; lane q updates h[q] (h0) and h[q+4] (h1).
__device__ __forceinline__ void compress(uint64_t &h0, uint64_t &h1, const LaneCtx &cx, uint64_t t,
                                         bool final) {
    // all 40 message words of the lane up front: one LDS latency per block, not one per round
    uint64_t m[10][4];
#pragma unroll
    for (int s = 0; s < 10; ++s)
#pragma unroll
        for (int k = 0; k < 4; ++k) m[s][k] = *cx.mp[s][k];
    __builtin_amdgcn_sched_barrier(0);
    uint64_t a = h0, b = h1, c = cx.iv_c;
    uint64_t d = cx.iv_d ^ (t & cx.t_mask) ^ (final ? cx.f_mask : 0ull);
#pragma unroll
    for (int r = 0; r < 12; ++r) {
        const int s = r % 10;
        const uint64_t m0 = m[s][0], m1 = m[s][1], m2 = m[s][2], m3 = m[s][3];
        g_mix(a, b, c, d, m0, m1);  // column q
        b = quad_perm<kRot1>(b);
        c = quad_perm<kRot2>(c);
        d = quad_perm<kRot3>(d);
        g_mix(a, b, c, d, m2, m3);  // diagonal q
        b = quad_perm<kRot3>(b);
        c = quad_perm<kRot2>(c);
        d = quad_perm<kRot1>(d);
    }
    h0 ^= a ^ c;
    h1 ^= b ^ d;
}

struct Raw {
    u32x4 x, y;
    uint32_t z;
};

// 36 bytes from a 4-aligned address (the lane's 32 bytes plus the funnel spill)
__device__ __forceinline__ Raw load_raw(gbytes a4) {
    Raw r;
    r.x = *reinterpret_cast<const GLOBAL u32x4 *>(a4);
    r.y = *reinterpret_cast<const GLOBAL u32x4 *>(a4 + 16);
    r.z = *reinterpret_cast<const GLOBAL uint32_t *>(a4 + 32);
    return r;
}

__device__ __forceinline__ void stage(uint64_t *qb, int q, const Raw &w, uint32_t sh) {
    const uint32_t sb = sh * 8;  // v_alignbyte takes the byte count; alignbit on bits is the same
    u32x4 o0, o1;
    o0.x = __builtin_amdgcn_alignbit(w.x.y, w.x.x, sb);
    o0.y = __builtin_amdgcn_alignbit(w.x.z, w.x.y, sb);
    o0.z = __builtin_amdgcn_alignbit(w.x.w, w.x.z, sb);
    o0.w = __builtin_amdgcn_alignbit(w.y.x, w.x.w, sb);
    o1.x = __builtin_amdgcn_alignbit(w.y.y, w.y.x, sb);
    o1.y = __builtin_amdgcn_alignbit(w.y.z, w.y.y, sb);
    o1.z = __builtin_amdgcn_alignbit(w.y.w, w.y.z, sb);
    o1.w = __builtin_amdgcn_alignbit(w.z, w.y.w, sb);
    *reinterpret_cast<u32x4 *>(qb + 4 * q) = o0;
    *reinterpret_cast<u32x4 *>(qb + 4 * q + 2) = o1;
}

__device__ __forceinline__ uint32_t byte_mask(int64_t valid) {
    return valid >= 4 ? 0xFFFFFFFFu : valid <= 0 ? 0u : (1u << (8 * valid)) - 1u;
}

}  // namespace

namespace {

// Lane q's message pointers and constants; qb is the quad's 128-byte block in LDS.
__device__ __forceinline__ LaneCtx make_ctx(int q, uint64_t *qb) {
    LaneCtx cx;
#pragma unroll
    for (int r = 0; r < 10; ++r)
#pragma unroll
        for (int k = 0; k < 4; ++k) cx.mp[r][k] = qb + ((sigma_pack(r, k) >> (4 * q)) & 15u);
    cx.iv_c = q == 0 ? kIV[0] : q == 1 ? kIV[1] : q == 2 ? kIV[2] : kIV[3];
    cx.iv_d = q == 0 ? kIV[4] : q == 1 ? kIV[5] : q == 2 ? kIV[6] : kIV[7];
    cx.t_mask = q == 0 ? ~0ull : 0ull;
    cx.f_mask = q == 2 ? ~0ull : 0ull;
    return cx;
}

// Compress blocks 0 .. nfull-1 of a message (non-final; counter t0 + 128 (b + 1)).  a4/sh: the
// lane's 4-aligned base (p + 32 q rounded down) and its byte shift.
__device__ __forceinline__ void body_blocks(uint64_t &h0, uint64_t &h1, const LaneCtx &cx,
                                            uint64_t *qb, int q, gbytes a4, uint32_t sh,
                                            uint64_t nfull, uint64_t t0) {
    // blocks b >= nfull are not loaded by the loop: clamp to block 0 (always readable when
    // nfull > 0) so that every iteration issues the same loads
    auto blk = [&](uint64_t b) { return a4 + 128 * (b < nfull ? b : 0); };
    Raw A, B;
    if (nfull) {
        A = load_raw(blk(0));
        B = load_raw(blk(1));
    }
    // two blocks per iteration with fixed register roles: copying A = B would make the
    // compiler wait for B's loads (vmcnt(0)) and collapse the prefetch distance
    uint64_t b = 0;
    for (; b + 2 <= nfull; b += 2) {
        stage(qb, q, A, sh);
        A = load_raw(blk(b + 2));
        compress(h0, h1, cx, t0 + (b + 1) * 128, false);
        stage(qb, q, B, sh);
        B = load_raw(blk(b + 3));
        compress(h0, h1, cx, t0 + (b + 2) * 128, false);
    }
    if (b < nfull) {  // odd count: A holds block b
        stage(qb, q, A, sh);
        compress(h0, h1, cx, t0 + (b + 1) * 128, false);
    }
}

// Stage block nfull -- the last 1..128 bytes of a len-byte message at p (0 bytes only for an
// empty one) -- into qb, zero past the message end.  Nothing beyond its last dword is read.
__device__ __forceinline__ void stage_last(uint64_t *qb, int q, gbytes p, gbytes a4, uint32_t sh,
                                           uint64_t nfull, uint64_t len) {
    const int64_t rem = static_cast<int64_t>(len - nfull * 128);
    Raw F;
    if (len) {
        const uintptr_t last = (reinterpret_cast<uintptr_t>(p) + len - 1) & ~uintptr_t(3);
        const uintptr_t f4 = reinterpret_cast<uintptr_t>(a4) + 128 * nfull;
        uint32_t w[9];
#pragma unroll
        for (int i = 0; i < 9; ++i) {
            uintptr_t a = f4 + 4 * i;
            a = a < last ? a : last;
            w[i] = *reinterpret_cast<const GLOBAL uint32_t *>(a);
        }
        F.x = u32x4{w[0], w[1], w[2], w[3]};
        F.y = u32x4{w[4], w[5], w[6], w[7]};
        F.z = w[8];
    } else {
        F.x = F.y = u32x4{0u, 0u, 0u, 0u};
        F.z = 0;
    }
    // funnel, then zero the bytes at or past the message end
    const uint32_t sb = sh * 8;
    const int64_t v0 = rem - 32 * q;
    u32x4 o0, o1;
    o0.x = __builtin_amdgcn_alignbit(F.x.y, F.x.x, sb) & byte_mask(v0);
    o0.y = __builtin_amdgcn_alignbit(F.x.z, F.x.y, sb) & byte_mask(v0 - 4);
    o0.z = __builtin_amdgcn_alignbit(F.x.w, F.x.z, sb) & byte_mask(v0 - 8);
    o0.w = __builtin_amdgcn_alignbit(F.y.x, F.x.w, sb) & byte_mask(v0 - 12);
    o1.x = __builtin_amdgcn_alignbit(F.y.y, F.y.x, sb) & byte_mask(v0 - 16);
    o1.y = __builtin_amdgcn_alignbit(F.y.z, F.y.y, sb) & byte_mask(v0 - 20);
    o1.z = __builtin_amdgcn_alignbit(F.y.w, F.y.z, sb) & byte_mask(v0 - 24);
    o1.w = __builtin_amdgcn_alignbit(F.z, F.y.w, sb) & byte_mask(v0 - 28);
    *reinterpret_cast<u32x4 *>(qb + 4 * q) = o0;
    *reinterpret_cast<u32x4 *>(qb + 4 * q + 2) = o1;
}

// digest bytes [8q, 8q+8) = h[q] and [32+8q, 40+8q) = h[q+4]; bytes >= outlen are zero
__device__ __forceinline__ void write_digest(uint8_t *slot, int q, uint64_t h0, uint64_t h1,
                                             uint32_t outlen) {
    auto keep = [&](uint64_t h, int byte0) -> uint64_t {
        const int v = static_cast<int>(outlen) - byte0;
        return v >= 8 ? h : v <= 0 ? 0ull : h & ((1ull << (8 * v)) - 1);
    };
    uint64_t *o = reinterpret_cast<uint64_t *>(slot);
    o[q] = keep(h0, 8 * q);
    o[4 + q] = keep(h1, 32 + 8 * q);
}

}  // namespace

namespace {

// ---- one LANE per chunk (round 3): the throughput form for many short chunks.
//
// A quad spends ~720 VALU per lane on a compression (2,880 lane-instructions per block, 20 %
// of it the diagonal step's DPP moves); one lane holding the whole 16-word state needs ~1,900
// and no cross-lane moves, so a batch of many short chunks -- where the VALU throughput, not one
// chain, sets the time -- hashes faster this way (config 3 iii's 1.45 M chunks: 46.3 -> 37.7 ms).
// A single chain is ~3x slower than a quad's, so only chunks short enough to finish well inside
// the batch's time go to lanes (lane_max, rc_b2_lane_max in digest_kernels.h).

__device__ __forceinline__ void g_lane(uint64_t &a, uint64_t &b, uint64_t &c, uint64_t &d,
                                       uint64_t x, uint64_t y) {
    a = a + b + x;
    d = rotr<32>(d ^ a);
    c = c + d;
    b = rotr<24>(b ^ c);
    a = a + b + y;
    d = rotr<16>(d ^ a);
    c = c + d;
    b = rotr<63>(b ^ c);
}

// RFC 7693 F: h ^= the 12-round mix of (h, IV ^ (t, 0, final, 0)) over message m.
__device__ __forceinline__ void compress_lane(uint64_t (&h)[8], const uint64_t (&m)[16], uint64_t t,
                                              bool final) {
    uint64_t v[16];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        v[i] = h[i];
        v[8 + i] = kIV[i];
    }
    v[12] ^= t;
    if (final) v[14] = ~v[14];
#pragma unroll
    for (int r = 0; r < 12; ++r) {
        const uint8_t *sg = kSigma[r % 10];
        g_lane(v[0], v[4], v[8], v[12], m[sg[0]], m[sg[1]]);
        g_lane(v[1], v[5], v[9], v[13], m[sg[2]], m[sg[3]]);
        g_lane(v[2], v[6], v[10], v[14], m[sg[4]], m[sg[5]]);
        g_lane(v[3], v[7], v[11], v[15], m[sg[6]], m[sg[7]]);
        g_lane(v[0], v[5], v[10], v[15], m[sg[8]], m[sg[9]]);
        g_lane(v[1], v[6], v[11], v[12], m[sg[10]], m[sg[11]]);
        g_lane(v[2], v[7], v[8], v[13], m[sg[12]], m[sg[13]]);
        g_lane(v[3], v[4], v[9], v[14], m[sg[14]], m[sg[15]]);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) h[i] ^= v[i] ^ v[8 + i];
}

struct LaneRaw {  // 132 bytes from a 4-aligned address: one block plus the funnel spill
    u32x4 q[8];
    uint32_t z;
};

__device__ __forceinline__ LaneRaw lane_load(gbytes a4) {
    LaneRaw r;
#pragma unroll
    for (int i = 0; i < 8; ++i) r.q[i] = *reinterpret_cast<const GLOBAL u32x4 *>(a4 + 16 * i);
    r.z = *reinterpret_cast<const GLOBAL uint32_t *>(a4 + 128);
    return r;
}

// the block's 16 little-endian words, funnelled by sh bytes (a no-op shift when aligned)
__device__ __forceinline__ void lane_words(const LaneRaw &r, uint32_t sh, uint64_t (&m)[16]) {
    const uint32_t sb = sh * 8;
    uint32_t w[33];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        w[4 * i] = r.q[i].x;
        w[4 * i + 1] = r.q[i].y;
        w[4 * i + 2] = r.q[i].z;
        w[4 * i + 3] = r.q[i].w;
    }
    w[32] = r.z;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const uint32_t lo = __builtin_amdgcn_alignbit(w[2 * i + 1], w[2 * i], sb);
        const uint32_t hi = __builtin_amdgcn_alignbit(w[2 * i + 2], w[2 * i + 1], sb);
        m[i] = (uint64_t(hi) << 32) | lo;
    }
}

// hash_digest of one message (len bytes at p) by one lane into out (outlen bytes of 64, the
// rest zero).  Nothing beyond the message's last dword is read.
__device__ __forceinline__ void lane_hash(gbytes p, uint64_t len, uint32_t outlen, uint8_t *out) {
    uint64_t h[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) h[i] = kIV[i];
    h[0] ^= 0x01010000ull | outlen;
    const uint64_t nfull = len ? (len - 1) / 128 : 0;  // non-final blocks
    const uint32_t sh = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(p) & 3);
    gbytes a4 = p - sh;
    uint64_t m[16];
    if (nfull) {
        LaneRaw nxt = lane_load(a4);
#pragma unroll 1
        for (uint64_t b = 0; b < nfull; ++b) {
            const LaneRaw cur = nxt;
            // the next block's loads go out before this block's compression; the last full
            // block re-reads itself (always readable) so every iteration issues the same loads
            nxt = lane_load(a4 + 128 * (b + 1 < nfull ? b + 1 : b));
            lane_words(cur, sh, m);
            compress_lane(h, m, 128 * (b + 1), false);
        }
    }
    // the last 1..128 bytes (none for an empty message), zero past the end
    const int64_t rem = static_cast<int64_t>(len - nfull * 128);
    uint32_t w[33];
    if (len) {
        const uintptr_t last = (reinterpret_cast<uintptr_t>(p) + len - 1) & ~uintptr_t(3);
        const uintptr_t f4 = reinterpret_cast<uintptr_t>(a4) + 128 * nfull;
#pragma unroll
        for (int i = 0; i < 33; ++i) {
            uintptr_t a = f4 + 4 * i;
            a = a < last ? a : last;
            w[i] = *reinterpret_cast<const GLOBAL uint32_t *>(a);
        }
    } else {
#pragma unroll
        for (int i = 0; i < 33; ++i) w[i] = 0;
    }
    {
        const uint32_t sb = sh * 8;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const uint32_t lo = __builtin_amdgcn_alignbit(w[2 * i + 1], w[2 * i], sb) & byte_mask(rem - 8 * i);
            const uint32_t hi = __builtin_amdgcn_alignbit(w[2 * i + 2], w[2 * i + 1], sb) &
                                byte_mask(rem - 8 * i - 4);
            m[i] = (uint64_t(hi) << 32) | lo;
        }
    }
    compress_lane(h, m, len, true);
    uint64_t *o = reinterpret_cast<uint64_t *>(out);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const int v = static_cast<int>(outlen) - 8 * i;
        o[i] = v >= 8 ? h[i] : v <= 0 ? 0ull : h[i] & ((1ull << (8 * v)) - 1);
    }
}

// first index of the longest-first list whose length is at most lane_max (binary search)
__device__ __forceinline__ uint64_t lane_split(const B2Item *items, uint64_t total, uint64_t lane_max) {
    uint64_t lo = 0, hi = total;
    while (lo < hi) {
        const uint64_t mid = (lo + hi) >> 1;
        if (items[mid].len <= lane_max) hi = mid;
        else lo = mid + 1;
    }
    return lo;
}

// Items [first, all) one per lane, dealt round-robin over the lanes of `groups` workgroups
// (this one is `group`): neighbouring lanes take neighbouring items of the longest-first list.
__device__ __forceinline__ void lane_items(const B2Item *items, uint64_t first, uint64_t all,
                                           uint64_t group, uint64_t groups, uint32_t outlen,
                                           uint8_t *out) {
    const uint64_t nl = groups * kB2Threads;
    for (uint64_t g = first + group * kB2Threads + threadIdx.x; g < all; g += nl) {
        const B2Item it = items[g];
        lane_hash(reinterpret_cast<gbytes>(it.ptr), it.len, outlen, out + it.slot * kB2Slot);
    }
}

}  // namespace

// Every item one per lane: the launch for batches whose items are all short enough for lanes
// (rc_b2_lane_max).  It holds 114 VGPRs against the quad kernel's 238, so four waves share a
// SIMD instead of two -- the lane form is VALU-throughput bound, and one wave issues a VALU
// instruction only every ~5-6 cycles.
__global__ __launch_bounds__(kB2Threads) void rc_b2_lane_kernel(const B2Item *__restrict__ items,
                                                                const uint64_t *__restrict__ d_total,
                                                                uint64_t n_static, uint32_t outlen,
                                                                uint8_t *__restrict__ out) {
    const uint64_t all = d_total ? *d_total : n_static;
    lane_items(items, 0, all, blockIdx.x, gridDim.x, outlen, out);
}

// One quad per chunk; a workgroup is kB2Threads / 4 quads.  Items g = quad, quad + Q, ...
// Workgroups [0, quad_groups) hash the list's items [0, k) by quads; the rest hash items
// [k, total) one per lane, where k is the first item of at most lane_max bytes (the list is
// longest first; lane_max 0: every item by quads).
__global__ __launch_bounds__(kB2Threads) void rc_b2_kernel(const B2Item *__restrict__ items,
                                                           const uint64_t *__restrict__ d_total,
                                                           uint64_t n_static, uint32_t outlen,
                                                           uint8_t *__restrict__ out,
                                                           uint64_t lane_max, uint32_t quad_groups) {
    __shared__ uint64_t blocks[kB2Threads / 4 * 16];
    const uint64_t all = d_total ? *d_total : n_static;
    const uint64_t k = lane_max ? lane_split(items, all, lane_max) : all;
    if (blockIdx.x >= quad_groups) {  // lane role: items k + i, k + i + NL, ..
        lane_items(items, k, all, blockIdx.x - quad_groups, gridDim.x - quad_groups, outlen, out);
        return;
    }
    const int q = threadIdx.x & 3;
    const int quad = threadIdx.x >> 2;
    uint64_t *qb = blocks + quad * 16;

    const LaneCtx cx = make_ctx(q, qb);
    const uint64_t h0_init = (q == 0 ? kIV[0] ^ (0x01010000ull | outlen) : cx.iv_c);
    const uint64_t h1_init = cx.iv_d;

    // One wave per SIMD (256 groups) unless items are plentiful: a BLAKE2b compression is
    // VALU-issue bound, so a second wave on a SIMD halves the speed of the first -- and the
    // longest chunk's wave sets the end of the launch.  Every group computes the same count.
    const uint64_t total = k;
    const uint64_t per_group = kB2Threads / 4;
    uint64_t groups = total >= kB2TwoWaveItems ? kB2MaxGroups : kB2OneWaveGroups;
    groups = groups < quad_groups ? groups : quad_groups;
    const uint64_t need = (total + per_group - 1) / per_group;
    groups = need < groups ? (need ? need : 1) : groups;
    if (blockIdx.x >= groups) return;
    const uint64_t nq = groups * per_group;
    // Snake deal over the longest-first list: round r takes items [r nq, (r+1) nq), in quad order
    // on even rounds and reversed on odd ones, so the quad that got the longest item of one
    // round gets the shortest of the next (a wave's 16 quads stay on 16 neighbouring items).
    const uint64_t gq = uint64_t(blockIdx.x) * per_group + quad;
    for (uint64_t r0 = 0; r0 < total; r0 += 2 * nq)
#pragma unroll 1
    for (int odd = 0; odd < 2; ++odd) {
        const uint64_t g = r0 + odd * nq + (odd ? nq - 1 - gq : gq);
        if (g >= total) continue;
        const B2Item it = items[g];
        gbytes p = reinterpret_cast<gbytes>(it.ptr);
        const uint64_t len = it.len;
        uint64_t h0 = h0_init, h1 = h1_init;
        const uint64_t nfull = len ? (len - 1) / 128 : 0;  // non-final blocks
        // lane base of block b: p + 128 b + 32 q, funnelled from its 4-aligned dword
        gbytes lb = p + 32 * q;
        const uint32_t sh = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(lb) & 3);
        gbytes a4 = lb - sh;
        body_blocks(h0, h1, cx, qb, q, a4, sh, nfull, 0);
        stage_last(qb, q, p, a4, sh, nfull, len);
        compress(h0, h1, cx, len, true);
        write_digest(out + it.slot * kB2Slot, q, h0, h1, outlen);
    }
}

// Incremental / keyed BLAKE2b: one quad per (state, buffer) item.  The state holds the chaining
// value, the byte counter and the last 1..128 message bytes not yet compressed (BLAKE2b may
// compress a block only once it knows whether the block is the last).  A keyed state starts
// with the zero-padded key as its pending block (RFC 7693 §3.3), so a keyed or salted hash is
// the same walk.  Non-final items write the state back; final items write the digest (to `out`)
// only, so one read-only state may serve many final items.
__device__ __forceinline__ void b2_update(uint64_t *qb, int q, const LaneCtx &cx,
                                          rc_blake2b_state *st, gbytes p, uint64_t len, bool final,
                                          uint8_t *out) {
    uint8_t *qbb = reinterpret_cast<uint8_t *>(qb);
    uint64_t h0 = st->h[q], h1 = st->h[q + 4];
    uint64_t t = st->t;
    const uint64_t buflen = st->buflen;
    const uint32_t outlen = st->digest_size;
    const uint64_t tot = buflen + len;
    if (!final && tot <= 128) {  // still one pending block: append
        for (uint64_t j = q; j < len; j += 4) st->buf[buflen + j] = p[j];
        if (q == 0) st->buflen = tot;
        return;
    }
    if (buflen) {  // pending bytes + the first bytes of p form the next block
#pragma unroll 4
        for (int i = 0; i < 32; ++i) {
            const uint64_t j = 32 * q + i;
            uint8_t v = 0;
            if (j < buflen)
                v = st->buf[j];
            else if (j - buflen < len)
                v = p[j - buflen];
            qbb[j] = v;
        }
        if (tot <= 128) {  // final and short: this is the last block
            compress(h0, h1, cx, t + tot, true);
            write_digest(out, q, h0, h1, outlen);
            return;
        }
        compress(h0, h1, cx, t + 128, false);
        t += 128;
        p += 128 - buflen;
        len -= 128 - buflen;
    }
    const uint64_t nfull = len ? (len - 1) / 128 : 0;
    gbytes lb = p + 32 * q;
    const uint32_t sh = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(lb) & 3);
    gbytes a4 = lb - sh;
    body_blocks(h0, h1, cx, qb, q, a4, sh, nfull, t);
    stage_last(qb, q, p, a4, sh, nfull, len);
    if (final) {
        compress(h0, h1, cx, t + len, true);
        write_digest(out, q, h0, h1, outlen);
    } else {  // keep the last 1..128 bytes pending
        u32x4 *dst = reinterpret_cast<u32x4 *>(st->buf + 32 * q);
        dst[0] = *reinterpret_cast<const u32x4 *>(qb + 4 * q);
        dst[1] = *reinterpret_cast<const u32x4 *>(qb + 4 * q + 2);
        st->h[q] = h0;
        st->h[q + 4] = h1;
        if (q == 0) {
            st->t = t + 128 * nfull;
            st->buflen = len - 128 * nfull;
        }
    }
}

__global__ __launch_bounds__(kB2Threads) void rc_b2_update_kernel(const B2UItem *__restrict__ items,
                                                                  uint64_t total,
                                                                  uint8_t *__restrict__ out) {
    __shared__ uint64_t blocks[kB2Threads / 4 * 16];
    const int q = threadIdx.x & 3;
    const int quad = threadIdx.x >> 2;
    uint64_t *qb = blocks + quad * 16;
    const LaneCtx cx = make_ctx(q, qb);

    const uint64_t nq = uint64_t(gridDim.x) * (kB2Threads / 4);
    for (uint64_t g = uint64_t(blockIdx.x) * (kB2Threads / 4) + quad; g < total; g += nq) {
        const B2UItem it = items[g];
        b2_update(qb, q, cx, reinterpret_cast<rc_blake2b_state *>(it.state),
                  reinterpret_cast<gbytes>(it.ptr), it.len, it.final != 0, out + it.slot * kB2Slot);
    }
}

// Per-chunk subkeys: `derive_shared_subkey(digest)` of every cut slot (repository.py:132-137,
// 1470-1472; adapters.py:205-213 = hashlib.blake2b(digest, salt=params, key=shared_key,
// digest_size=key bytes)).  The KDF state (key pending, salt in the parameter block) absorbs the
// first msg_len bytes of digest slot s and finalises into keys + 64 s.  One quad per chunk; the
// state is only read.
struct DeriveLists {
    const uint64_t *cut_base;
    const int64_t *counts;
    uint64_t n, spw;  // streams, streams per workgroup
};

__global__ __launch_bounds__(kB2Threads) void rc_b2_derive_kernel(DeriveLists c,
                                                                  rc_blake2b_state *kdf,
                                                                  uint64_t digests, uint32_t msg_len,
                                                                  uint8_t *__restrict__ keys) {
    __shared__ uint64_t blocks[kB2Threads / 4 * 16];
    const int q = threadIdx.x & 3;
    const int quad = threadIdx.x >> 2;
    uint64_t *qb = blocks + quad * 16;
    const LaneCtx cx = make_ctx(q, qb);
    const uint64_t s0 = blockIdx.x * c.spw, s1 = s0 + c.spw < c.n ? s0 + c.spw : c.n;
    for (uint64_t s = s0; s < s1; ++s) {
        const int64_t cnt = c.counts[s];
        const uint64_t base = c.cut_base[s];
        for (int64_t k = quad; k < cnt; k += kB2Threads / 4) {
            const uint64_t slot = base + uint64_t(k);
            b2_update(qb, q, cx, kdf, reinterpret_cast<gbytes>(digests + kB2Slot * slot), msg_len,
                      true, keys + kB2Slot * slot);
        }
    }
}

// Work list of the chunks rc_chunk_device wrote, longest first.
//
// The digest kernel hands items out round-robin in list order (quad g of the grid takes items
// g, g + Q, ..): with the list sorted by decreasing length, the 16 quads of a wave get items of
// about the same length (a wave runs as long as its longest item) and the grid gets the longest
// items first (LPT), so no wave is left holding a 5 MB chunk at the end.  The order is a bucket
// sort on (floor(log2(len+1)), next two bits): 256 buckets, exact enough for scheduling.

__device__ __forceinline__ uint32_t len_bucket(uint64_t len) {
    const uint64_t x = len + 1;
    const int e = 63 - __clzll(static_cast<long long>(x));
    const uint32_t m = e >= 2 ? static_cast<uint32_t>(x >> (e - 2)) & 3u : (e == 1 ? (x & 1u) << 1 : 0u);
    return 255u - (4u * static_cast<uint32_t>(e) + m);  // 0 = longest
}

// Pass 1 (one workgroup): exclusive prefix of the per-stream chunk counts into chunk_off[0..n],
// total at chunk_off[n].
__global__ __launch_bounds__(1024) void rc_b2_scan_kernel(const int64_t *__restrict__ counts,
                                                          uint64_t n,
                                                          uint64_t *__restrict__ chunk_off) {
    __shared__ uint64_t part[1024];
    const uint64_t per = (n + 1023) / 1024;
    const uint64_t lo = threadIdx.x * per, hi = lo + per < n ? lo + per : n;
    uint64_t s = 0;
    for (uint64_t i = lo; i < hi; ++i) s += counts[i] > 0 ? uint64_t(counts[i]) : 0;
    part[threadIdx.x] = s;
    __syncthreads();
    for (int off = 1; off < 1024; off <<= 1) {  // inclusive Hillis-Steele scan
        const uint64_t v = threadIdx.x >= off ? part[threadIdx.x - off] : 0;
        __syncthreads();
        part[threadIdx.x] += v;
        __syncthreads();
    }
    uint64_t acc = part[threadIdx.x] - s;
    for (uint64_t i = lo; i < hi; ++i) {
        chunk_off[i] = acc;
        acc += counts[i] > 0 ? uint64_t(counts[i]) : 0;
    }
    if (threadIdx.x == 1023) chunk_off[n] = part[1023];
}

struct ChunkLists {
    const uint64_t *ptrs, *cut_base, *cuts;
    const int64_t *counts;
    uint64_t n, spw;  // streams, streams per workgroup
};

// Pass 2: per workgroup (a run of spw streams) a histogram of its chunks' buckets, stored
// bucket-major: hist[b * G + g].
__global__ __launch_bounds__(256) void rc_b2_hist_kernel(ChunkLists c, uint32_t *__restrict__ hist) {
    __shared__ uint32_t h[kB2Buckets];
    for (int b = threadIdx.x; b < kB2Buckets; b += 256) h[b] = 0;
    __syncthreads();
    const uint64_t s0 = blockIdx.x * c.spw, s1 = s0 + c.spw < c.n ? s0 + c.spw : c.n;
    for (uint64_t s = s0; s < s1; ++s) {
        const int64_t cnt = c.counts[s];
        const uint64_t *e = c.cuts + c.cut_base[s];
        for (int64_t k = threadIdx.x; k < cnt; k += 256)
            atomicAdd(&h[len_bucket(e[k] - (k ? e[k - 1] : 0))], 1u);
    }
    __syncthreads();
    for (int b = threadIdx.x; b < kB2Buckets; b += 256) hist[uint64_t(b) * gridDim.x + blockIdx.x] = h[b];
}

// Pass 3 (one workgroup): exclusive scan of hist in place (bucket-major = longest first).
__global__ __launch_bounds__(1024) void rc_b2_hscan_kernel(uint32_t *__restrict__ hist, uint64_t m) {
    __shared__ uint64_t part[1024];
    const uint64_t per = (m + 1023) / 1024;
    const uint64_t lo = threadIdx.x * per, hi = lo + per < m ? lo + per : m;
    uint64_t s = 0;
    for (uint64_t i = lo; i < hi; ++i) s += hist[i];
    part[threadIdx.x] = s;
    __syncthreads();
    for (int off = 1; off < 1024; off <<= 1) {
        const uint64_t v = threadIdx.x >= off ? part[threadIdx.x - off] : 0;
        __syncthreads();
        part[threadIdx.x] += v;
        __syncthreads();
    }
    uint64_t acc = part[threadIdx.x] - s;
    for (uint64_t i = lo; i < hi; ++i) {
        const uint32_t v = hist[i];
        hist[i] = static_cast<uint32_t>(acc);
        acc += v;
    }
}

// Pass 4: scatter every chunk to its sorted position (start address, length, cut slot).
__global__ __launch_bounds__(256) void rc_b2_scatter_kernel(ChunkLists c,
                                                            const uint32_t *__restrict__ off,
                                                            B2Item *__restrict__ items) {
    __shared__ uint32_t cur[kB2Buckets];
    for (int b = threadIdx.x; b < kB2Buckets; b += 256) cur[b] = off[uint64_t(b) * gridDim.x + blockIdx.x];
    __syncthreads();
    const uint64_t s0 = blockIdx.x * c.spw, s1 = s0 + c.spw < c.n ? s0 + c.spw : c.n;
    for (uint64_t s = s0; s < s1; ++s) {
        const int64_t cnt = c.counts[s];
        const uint64_t base = c.cut_base[s], p = c.ptrs[s];
        const uint64_t *e = c.cuts + base;
        for (int64_t k = threadIdx.x; k < cnt; k += 256) {
            const uint64_t start = k ? e[k - 1] : 0, len = e[k] - start;
            const uint32_t pos = atomicAdd(&cur[len_bucket(len)], 1u);
            items[pos] = B2Item{p + start, len, base + k};
        }
    }
}

namespace {
thread_local char g_b2_err[256];

int b2_status(const char *what) {
    const hipError_t e = hipGetLastError();
    if (e == hipSuccess) return 0;
    snprintf(g_b2_err, sizeof g_b2_err, "%s: %s", what, hipGetErrorString(e));
    return 1;
}

unsigned b2_grid(uint64_t upper) {
    const uint64_t quads = kB2Threads / 4;
    uint64_t wg = (upper + quads - 1) / quads;
    if (wg > kB2MaxGroups) wg = kB2MaxGroups;
    return static_cast<unsigned>(wg ? wg : 1);
}
}  // namespace

const char *rc_b2_launch_error(void) { return g_b2_err; }

// lane-role workgroups for up to `upper` items: two waves per SIMD at most (kB2MaxGroups)
static unsigned b2_lane_grid(uint64_t upper, uint64_t lane_max) {
    if (!lane_max) return 0;
    uint64_t wg = (upper + kB2Threads - 1) / kB2Threads;
    if (wg > kB2MaxGroups) wg = kB2MaxGroups;
    return static_cast<unsigned>(wg);
}

// lane-only workgroups for up to `upper` items: four waves per SIMD at most
static unsigned b2_lane_only_grid(uint64_t upper) {
    uint64_t wg = (upper + kB2Threads - 1) / kB2Threads;
    if (wg > kB2LaneGroups) wg = kB2LaneGroups;
    return static_cast<unsigned>(wg ? wg : 1);
}

int rc_b2_launch_items(const B2Item *d_items, uint64_t n, uint32_t outlen, uint8_t *d_out,
                       uint64_t lane_max, bool lane_only, hipStream_t stream) {
    if (!n) return 0;
    if (lane_only) {
        rc_b2_lane_kernel<<<b2_lane_only_grid(n), kB2Threads, 0, stream>>>(d_items, nullptr, n,
                                                                           outlen, d_out);
        return b2_status("rc_b2_lane_kernel");
    }
    const unsigned qg = b2_grid(n);
    rc_b2_kernel<<<qg + b2_lane_grid(n, lane_max), kB2Threads, 0, stream>>>(d_items, nullptr, n, outlen,
                                                                          d_out, lane_max, qg);
    return b2_status("rc_b2_kernel");
}

int rc_b2_launch_chunks(uint64_t n, const uint64_t *d_ptrs, const uint64_t *d_cut_base,
                        const uint64_t *d_cuts, const int64_t *d_counts, uint64_t *d_chunk_off,
                        uint32_t *d_hist, B2Item *d_items, uint64_t items_cap, uint32_t outlen,
                        uint8_t *d_out, uint64_t lane_max, bool lane_only, hipStream_t stream) {
    if (!n) return 0;
    rc_b2_scan_kernel<<<1, 1024, 0, stream>>>(d_counts, n, d_chunk_off);
    if (b2_status("rc_b2_scan_kernel")) return 1;
    const ChunkLists c{d_ptrs, d_cut_base, d_cuts, d_counts, n, rc_b2_streams_per_group(n)};
    const unsigned groups = static_cast<unsigned>((n + c.spw - 1) / c.spw);
    rc_b2_hist_kernel<<<groups, 256, 0, stream>>>(c, d_hist);
    if (b2_status("rc_b2_hist_kernel")) return 1;
    rc_b2_hscan_kernel<<<1, 1024, 0, stream>>>(d_hist, uint64_t(kB2Buckets) * groups);
    if (b2_status("rc_b2_hscan_kernel")) return 1;
    rc_b2_scatter_kernel<<<groups, 256, 0, stream>>>(c, d_hist, d_items);
    if (b2_status("rc_b2_scatter_kernel")) return 1;
    if (lane_only) {
        rc_b2_lane_kernel<<<b2_lane_only_grid(items_cap), kB2Threads, 0, stream>>>(
            d_items, d_chunk_off + n, 0, outlen, d_out);
        return b2_status("rc_b2_lane_kernel");
    }
    const unsigned qg = b2_grid(items_cap);
    rc_b2_kernel<<<qg + b2_lane_grid(items_cap, lane_max), kB2Threads, 0, stream>>>(
        d_items, d_chunk_off + n, 0, outlen, d_out, lane_max, qg);
    return b2_status("rc_b2_kernel");
}

int rc_b2_launch_update(const B2UItem *d_items, uint64_t n, uint8_t *d_out, hipStream_t stream) {
    if (!n) return 0;
    rc_b2_update_kernel<<<b2_grid(n), kB2Threads, 0, stream>>>(d_items, n, d_out);
    return b2_status("rc_b2_update_kernel");
}

int rc_b2_launch_scan(const int64_t *d_counts, uint64_t n, uint64_t *d_chunk_off, hipStream_t stream) {
    if (!n) return 0;
    rc_b2_scan_kernel<<<1, 1024, 0, stream>>>(d_counts, n, d_chunk_off);
    return b2_status("rc_b2_scan_kernel");
}

int rc_b2_launch_derive(uint64_t n, const uint64_t *d_cut_base, const int64_t *d_counts,
                        const rc_blake2b_state *d_kdf, const uint8_t *d_digests, uint32_t msg_len,
                        uint8_t *d_keys, hipStream_t stream) {
    if (!n) return 0;
    const DeriveLists c{d_cut_base, d_counts, n, rc_b2_streams_per_group(n)};
    const unsigned groups = static_cast<unsigned>((n + c.spw - 1) / c.spw);
    rc_b2_derive_kernel<<<groups, kB2Threads, 0, stream>>>(c, const_cast<rc_blake2b_state *>(d_kdf),
                                                           reinterpret_cast<uint64_t>(d_digests),
                                                           msg_len, d_keys);
    return b2_status("rc_b2_derive_kernel");
}
