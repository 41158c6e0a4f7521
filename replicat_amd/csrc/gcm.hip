// gcm.hip -- AES-GCM encryption / decryption of chunks on gfx950.
//
// What it replaces: the per-chunk `self.props.encrypt(output_chunk, subkey)` of replicat's
// snapshot loop (/root/reference/replicat/repository.py:1470-1473) with the default cipher
// `aes_gcm(key_bits=256, nonce_bits=96)` (replicat/utils/adapters.py:117-158; repository.py:216):
// nonce = os.urandom(nonce_bytes); nonce || AESGCM(key).encrypt(nonce, chunk, None) = nonce || C || T,
// and `decrypt`, its inverse with the tag check (InvalidTag -> DecryptionError, :136-144).
// AES per FIPS 197, GCM per NIST SP 800-38D, no associated data.
//
// Shape of the work.  CTR mode is parallel over 16-byte blocks; GHASH is the polynomial
// S = (sum_i C_i H^(m-i) + L) H over the ciphertext blocks C_0..C_(m-1) and the length block L.
// One workgroup (1024 threads) per chunk: thread t owns blocks t, t+1024, .. (each
// row of 1024 blocks is one coalesced 16 KiB read and write) and folds its blocks by Horner with
// M = H^1024.  The chunk is virtually left-padded with zero blocks to a whole number of rows
// (leading zeros do not change a GHASH that starts at 0), so all 1024 chains end in the last row
// and their results Z_t form a 1024-block GHASH themselves: 32 lanes fold 32 each with H, one lane
// folds the 32 results with H^32, adds L and multiplies by H.
//
// AES: T-tables in LDS.  All four T_k = rotl(8k) T0 are replicated 32x in two 64 KiB regions,
// row e (256 B) of region A holding [T0[e] x 32 | T1[e] x 32] and of region B [T2[e] x 32 |
// T3[e] x 32], so lane l of a ds_read_b32 half-wave always reads bank l: random lookups without
// bank conflicts, and the address 65536 R + 256 e + 4 (l mod 32) (+128 for T1 / T3) is ONE
// v_perm_b32 of the state word and a per-lane constant (the chunker's prefilter trick,
// kernels.hip:pf_entry): per round 16 v_perm + 8 VALU (two three-input XORs per column) + 16
// ds_read_b32.  Until round 5 only T0 / T1 were in LDS and T2 / T3 came from one rot16 of
// T0[c] ^ T1[d] ^ rot16(k) per column (12 VALU per round): 128 KiB of T-tables now fit because
// the GHASH tables of H^32 and the chain results live in the AES region once the rounds are done
// (LDS map below).  Round keys are expanded per chunk by one lane and then held in SGPRs.
//
// GHASH: the product by a fixed field element Y uses 32 nibble tables T[j][v] = Y . E(j, v)
// (16 entries of 16 B per nibble position: the 16 lanes of a ds_read_b128 quarter-wave hit
// distinct 4-bank groups), 8 KiB per Y, built per chunk for H, H^32 and H^1024 from H = E_K(0).
// Squaring is GF(2)-linear, so H^32 and H^1024 take ten lookups in a constant squaring table.
//
// Roofline: LDS issue (16 ds_read_b32 per AES round, 32 ds_read_b128 per GHASH step), not HBM.

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "cipher_kernels.h"

#ifdef RC_GCM_TRACE  // diagnostic build (scripts/gcm_diag.cpp): progress word of workgroup 0
__device__ unsigned long long g_gcm_trace[4];
#define GCM_MARK(code, val)                                                                      \
    do {                                                                                         \
        if (blockIdx.x == 0 && threadIdx.x == 0) {                                               \
            __hip_atomic_store(&g_gcm_trace[0], (unsigned long long)(code), __ATOMIC_RELAXED,    \
                               __HIP_MEMORY_SCOPE_SYSTEM);                                       \
            __hip_atomic_store(&g_gcm_trace[1], (unsigned long long)(val), __ATOMIC_RELAXED,     \
                               __HIP_MEMORY_SCOPE_SYSTEM);                                       \
        }                                                                                        \
    } while (0)
#else
#define GCM_MARK(code, val) do { } while (0)
#endif

namespace {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4a4 __attribute__((ext_vector_type(4), aligned(4)));
#define GLOBAL __attribute__((address_space(1)))
typedef const GLOBAL uint8_t *gcbytes;
typedef GLOBAL uint8_t *gbytes;

// LDS map (bytes).  The AES regions are dead once every wave has left the CTR loop (E_K(J0) is
// computed before it): the fold's chain results and the table of H^32 reuse them then.
constexpr uint32_t kAes = 0;          // region A: 256 rows x 256 B (T0 | T1); region B at +64 KiB (T2 | T3)
constexpr uint32_t kZ = 0;            // after the CTR loop: 1024 chain results (16 KiB)
constexpr uint32_t kTab32 = 16384;    // after the CTR loop: GHASH table of H^32
constexpr uint32_t kTabM = 131072;    // GHASH table of M = H^1024
constexpr uint32_t kTab1 = 139264;    // of H (setup for non-96-bit nonces, and the fold)
constexpr uint32_t kMisc = 147456;
constexpr uint32_t kRk = kMisc;      // expanded key, <= 60 words
constexpr uint32_t kH = kMisc + 256;
constexpr uint32_t kH32 = kMisc + 272;
constexpr uint32_t kHM = kMisc + 288;
constexpr uint32_t kJ0 = kMisc + 304;
constexpr uint32_t kEJ0 = kMisc + 320;
constexpr uint32_t kP = kMisc + 512;  // 32 partial sums
constexpr uint32_t kSq = kMisc + 1024;  // squaring table (constant, setup only)
constexpr uint32_t kLds = kSq + 8192;   // 153 KiB of the 160
static_assert(kTab32 + 8192 <= 131072 && kTabM >= 131072 && kLds <= 163840, "LDS map overlaps");

__shared__ __attribute__((aligned(16))) uint8_t s_gcm[kLds];

template <typename T>
__device__ __forceinline__ T &lds(uint32_t off) {
    return *reinterpret_cast<T *>(s_gcm + off);
}

__device__ __forceinline__ uint32_t rotl8(uint32_t x) { return (x << 8) | (x >> 24); }
__device__ __forceinline__ uint32_t rot16(uint32_t x) { return __builtin_amdgcn_alignbit(x, x, 16); }
__device__ __forceinline__ uint32_t bswap(uint32_t x) { return __builtin_bswap32(x); }
// a ^ b ^ c in one VALU (gfx950 v_bitop3_b32, truth table 0x96): the rounds and GHASH are
// VALU-co-bound with the LDS, and half their XORs fold away
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

// ------------------------------------------------------------------------------ AES

// v_perm selector: byte 0 <- lo.byte0 (lane column, +128 for T1 / T3), byte 1 <- state byte k
// (table row), byte 2 <- lo.byte2 (the region: 0 for T0 / T1, 1 for T2 / T3), byte 3 <- 0
constexpr uint32_t sel(int k) { return 0x0C020000u | ((4u + uint32_t(k)) << 8); }

__device__ __forceinline__ uint32_t tl(uint32_t w, uint32_t lo, uint32_t s) {
    return lds<uint32_t>(__builtin_amdgcn_perm(w, lo, s));
}

// the S-box is byte 1 of T0 (T0[x] = 2s | s << 8 | s << 16 | 3s << 24)
__device__ __forceinline__ uint32_t sbox(uint32_t x) { return (lds<uint32_t>(kAes + x * 256) >> 8) & 0xFFu; }
__device__ __forceinline__ uint32_t subword(uint32_t t) {
    return sbox(t & 0xFFu) | (sbox((t >> 8) & 0xFFu) << 8) | (sbox((t >> 16) & 0xFFu) << 16) |
           (sbox(t >> 24) << 24);
}

// One block.  State words are little-endian columns (byte r of word c = row r of column c), so a
// 16-byte block loads straight into them.  lo0 .. lo3: the lane's address constants of T0 .. T3.
template <int NR>
__device__ __forceinline__ u32x4 aes_encrypt(u32x4 in, const uint32_t *rk, uint32_t lo0, uint32_t lo1,
                                             uint32_t lo2, uint32_t lo3) {
    uint32_t s0 = in.x ^ rk[0], s1 = in.y ^ rk[1], s2 = in.z ^ rk[2], s3 = in.w ^ rk[3];
#pragma unroll
    for (int r = 1; r < NR; ++r) {
        // column c takes row k from column c + k (ShiftRows); T_k = rotl(8k) T0 (MixColumns)
        const uint32_t n0 = xor3(tl(s0, lo0, sel(0)), tl(s1, lo1, sel(1)),
                                 xor3(tl(s2, lo2, sel(2)), tl(s3, lo3, sel(3)), rk[4 * r]));
        const uint32_t n1 = xor3(tl(s1, lo0, sel(0)), tl(s2, lo1, sel(1)),
                                 xor3(tl(s3, lo2, sel(2)), tl(s0, lo3, sel(3)), rk[4 * r + 1]));
        const uint32_t n2 = xor3(tl(s2, lo0, sel(0)), tl(s3, lo1, sel(1)),
                                 xor3(tl(s0, lo2, sel(2)), tl(s1, lo3, sel(3)), rk[4 * r + 2]));
        const uint32_t n3 = xor3(tl(s3, lo0, sel(0)), tl(s0, lo1, sel(1)),
                                 xor3(tl(s1, lo2, sel(2)), tl(s2, lo3, sel(3)), rk[4 * r + 3]));
        s0 = n0;
        s1 = n1;
        s2 = n2;
        s3 = n3;
    }
    // last round (no MixColumns): S[x] is byte 1 or 2 of T0[x] and byte 3 of T1[x]
    auto last = [&](uint32_t a, uint32_t b, uint32_t c, uint32_t d, uint32_t k) {
        return (((tl(a, lo0, sel(0)) >> 8) & 0xFFu) | (tl(b, lo0, sel(1)) & 0xFF00u) |
                (tl(c, lo0, sel(2)) & 0xFF0000u) | (tl(d, lo1, sel(3)) & 0xFF000000u)) ^ k;
    };
    u32x4 o;
    o.x = last(s0, s1, s2, s3, rk[4 * NR]);
    o.y = last(s1, s2, s3, s0, rk[4 * NR + 1]);
    o.z = last(s2, s3, s0, s1, rk[4 * NR + 2]);
    o.w = last(s3, s0, s1, s2, rk[4 * NR + 3]);
    return o;
}

// FIPS 197 §5.2 in little-endian words (RotWord = rotr8), one lane; the schedule goes to kRk.
template <int NR>
__device__ __forceinline__ void expand_key(gcbytes key) {
    constexpr int NK = NR - 6, NW = 4 * (NR + 1);
    uint32_t w[NW];
#pragma unroll
    for (int i = 0; i < NK; ++i)
        w[i] = uint32_t(key[4 * i]) | (uint32_t(key[4 * i + 1]) << 8) |
               (uint32_t(key[4 * i + 2]) << 16) | (uint32_t(key[4 * i + 3]) << 24);
    uint32_t rcon = 1;
#pragma unroll
    for (int i = NK; i < NW; ++i) {
        uint32_t t = w[i - 1];
        if (i % NK == 0) {
            t = subword((t >> 8) | (t << 24)) ^ rcon;
            rcon = ((rcon << 1) ^ ((rcon & 0x80u) ? 0x1Bu : 0u)) & 0xFFu;
        } else if (NK > 6 && i % NK == 4) {
            t = subword(t);
        }
        w[i] = w[i - NK] ^ t;
    }
#pragma unroll
    for (int i = 0; i < NW; ++i) lds<uint32_t>(kRk + 4 * i) = w[i];
}

// ---------------------------------------------------------------------------- GHASH

// x . Y for the Y whose nibble tables sit at BASE: nibble j of x (j = 2 b: the high nibble of
// byte b; j = 2 b + 1: the low one) with value v selects the 16 bytes at BASE + 256 j + 16 v.
// Tables past 56 KiB (kTabM and the setup tables since round 5): a DS instruction's offset field
// holds 16 bits, so BASE + 256 j would be OR-ed into every address by its own VALU; with BASE in
// an opaque register each address is ONE v_and_or_b32 (nibble | BASE) and 256 j the offset.
template <uint32_t BASE>
__device__ __forceinline__ u32x4 tab_mul(u32x4 x) {
    u32x4 acc = {0u, 0u, 0u, 0u};
    uint32_t base = BASE;
    if constexpr (BASE + 32 * 256 > 65536) asm("" : "+v"(base));
#pragma unroll
    for (int d = 0; d < 4; ++d) {
        const uint32_t w = x[d];
        const uint32_t hi = w & 0xF0F0F0F0u, lo = (w << 4) & 0xF0F0F0F0u;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t j = 2 * (4 * d + k);
            const u32x4 p = lds<u32x4>((((hi >> (8 * k)) & 0xF0u) | base) + j * 256);
            const u32x4 q = lds<u32x4>((((lo >> (8 * k)) & 0xF0u) | base) + (j + 1) * 256);
            acc = u32x4{xor3(acc.x, p.x, q.x), xor3(acc.y, p.y, q.y), xor3(acc.z, p.z, q.z),
                        xor3(acc.w, p.w, q.w)};
        }
    }
    return acc;
}

// Field elements as big-endian words (w0 = bytes 0..3): SP 800-38D bit i is integer bit 127 - i,
// so multiplying by x is a right shift with the reduction 0xE1 || 0^120.
struct Be {
    uint32_t w0, w1, w2, w3;
};
__device__ __forceinline__ Be be_xor(Be a, Be b) { return {a.w0 ^ b.w0, a.w1 ^ b.w1, a.w2 ^ b.w2, a.w3 ^ b.w3}; }
__device__ __forceinline__ Be mulx(Be b) {
    const uint32_t c = b.w3 & 1u;
    return {(b.w0 >> 1) ^ ((0u - c) & 0xE1000000u), __builtin_amdgcn_alignbit(b.w0, b.w1, 1),
            __builtin_amdgcn_alignbit(b.w1, b.w2, 1), __builtin_amdgcn_alignbit(b.w2, b.w3, 1)};
}
// . x^4: the four dropped bits l come back as clmul(l, 0xE1) << 117
__device__ __forceinline__ Be mulx4(Be b) {
    const uint32_t l = b.w3 & 15u;
    return {(b.w0 >> 4) ^ ((l ^ (l << 5) ^ (l << 6) ^ (l << 7)) << 21),
            __builtin_amdgcn_alignbit(b.w0, b.w1, 4), __builtin_amdgcn_alignbit(b.w1, b.w2, 4),
            __builtin_amdgcn_alignbit(b.w2, b.w3, 4)};
}

// Lane j (< 32) writes the 16 entries of nibble position j of Y's table at base:
// T[j][v] = xor over the set bits (3 - m) of v of Y . x^(4 j + m).
__device__ __forceinline__ void build_table(uint32_t base, u32x4 y, int j) {
    Be b = {bswap(y.x), bswap(y.y), bswap(y.z), bswap(y.w)};
    for (int i = 0; i < j; ++i) b = mulx4(b);
    const Be b0 = b, b1 = mulx(b0), b2 = mulx(b1), b3 = mulx(b2);
#pragma unroll
    for (int v = 0; v < 16; ++v) {
        Be e = {0u, 0u, 0u, 0u};
        if (v & 8) e = be_xor(e, b0);
        if (v & 4) e = be_xor(e, b1);
        if (v & 2) e = be_xor(e, b2);
        if (v & 1) e = be_xor(e, b3);
        lds<u32x4>(base + uint32_t(j) * 256 + uint32_t(v) * 16) =
            u32x4{bswap(e.w0), bswap(e.w1), bswap(e.w2), bswap(e.w3)};
    }
}

// ------------------------------------------------------------------------ byte access

__device__ __forceinline__ u32x4 load_bytes(gcbytes p, uint32_t n) {
    uint32_t w[4] = {0u, 0u, 0u, 0u};
#pragma unroll
    for (int i = 0; i < 16; ++i)
        if (uint32_t(i) < n) w[i >> 2] |= uint32_t(p[i]) << (8 * (i & 3));
    return u32x4{w[0], w[1], w[2], w[3]};
}

__device__ __forceinline__ void store_bytes(gbytes p, u32x4 v, uint32_t n) {
#pragma unroll
    for (int i = 0; i < 16; ++i)
        if (uint32_t(i) < n) p[i] = static_cast<uint8_t>(v[i >> 2] >> (8 * (i & 3)));
}

__device__ __forceinline__ u32x4 keep_bytes(u32x4 v, uint32_t n) {
    auto m = [&](uint32_t d) -> uint32_t {
        return n >= 4 * d + 4 ? 0xFFFFFFFFu : n <= 4 * d ? 0u : (1u << (8 * (n - 4 * d))) - 1u;
    };
    return u32x4{v.x & m(0), v.y & m(1), v.z & m(2), v.w & m(3)};
}

}  // namespace

// ----------------------------------------------------------------------------- kernel

template <int NR, bool DEC>
__global__ __launch_bounds__(kGcmThreads) void rc_gcm_kernel(GcmArgs a) {
    constexpr int NW = 4 * (NR + 1);
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    // one workgroup per message, straight-line (no work-queue loop: barriers inside a loop whose
    // exit the compiler could not prove uniform were structurized into a hang)
    const uint64_t idx = blockIdx.x;
    if (a.d_total && idx >= *a.d_total) return;
    GCM_MARK(2, idx);

    // constant tables: region A [T0 x 32 | T1 x 32] per row, region B [T2 x 32 | T3 x 32]
    for (int i = tid; i < 256 * 64; i += kGcmThreads) {
        const int e = i >> 6, c = i & 63;
        const uint32_t t0 = a.te0[e], t = c < 32 ? t0 : rotl8(t0);
        lds<uint32_t>(kAes + e * 256 + c * 4) = t;
        lds<uint32_t>(kAes + 65536 + e * 256 + c * 4) = rot16(t);
    }
    for (int i = tid; i < 512; i += kGcmThreads)
        lds<u32x4>(kSq + i * 16) = reinterpret_cast<const u32x4 *>(a.sq)[i];
    const uint32_t lo0 = kAes | (uint32_t(lane & 31) << 2), lo1 = lo0 | 128u;
    const uint32_t lo2 = lo0 | 0x10000u, lo3 = lo1 | 0x10000u;
    const uint32_t nbytes = a.nonce_bytes;
    {
        const GcmItem it = a.items[idx];
        gcbytes nonce = reinterpret_cast<gcbytes>(DEC ? it.in : it.nonce);

        // ---- A: key schedule (one lane)
        __syncthreads();  // the tables
        if (tid == 0) expand_key<NR>(reinterpret_cast<gcbytes>(it.key));
        __syncthreads();
        GCM_MARK(3, idx);
        uint32_t rk[NW];
#pragma unroll
        for (int i = 0; i < NW; ++i) rk[i] = __builtin_amdgcn_readfirstlane(lds<uint32_t>(kRk + 4 * i));

        // ---- B: H = E_K(0) and its powers H^32, H^1024 (lane 0); for 96-bit nonces (lane 1)
        // J0 = IV || 0^31 || 1 and E_K(J0)
        if (wave == 0 && lane < 2) {
            u32x4 blk = {0u, 0u, 0u, 0u};
            if (lane == 1 && nbytes == 12) {
                const u32x4 iv = load_bytes(nonce, 12);
                blk = u32x4{iv.x, iv.y, iv.z, 0x01000000u};
            }
            const u32x4 e = aes_encrypt<NR>(blk, rk, lo0, lo1, lo2, lo3);
            if (lane == 0) {
                lds<u32x4>(kH) = e;
                u32x4 p = e;
#pragma unroll 1
                for (int k = 1; k <= 10; ++k) {
                    p = tab_mul<kSq>(p);
                    if (k == 5) lds<u32x4>(kH32) = p;
                }
                lds<u32x4>(kHM) = p;
            } else if (nbytes == 12) {
                lds<u32x4>(kJ0) = blk;
                lds<u32x4>(kEJ0) = e;
            }
        }
        __syncthreads();

        GCM_MARK(4, idx);
        // ---- C: the nibble tables of H and H^1024 (32 lanes each; H^32's is built after the CTR
        // loop, in the AES region)
        if (wave < 2 && lane < 32) {
            const uint32_t src = wave == 0 ? kH : kHM;
            const uint32_t dst = wave == 0 ? kTab1 : kTabM;
            build_table(dst, lds<u32x4>(src), lane);
        }
        __syncthreads();

        GCM_MARK(5, idx);
        // ---- D: other nonce lengths: J0 = GHASH_H(IV || 0-pad || 0^64 || [len(IV)]_64)
        if (nbytes != 12) {
            if (tid == 0) {
                u32x4 y = {0u, 0u, 0u, 0u};
                for (uint32_t off = 0; off < nbytes; off += 16)
                    y = tab_mul<kTab1>(y ^ load_bytes(nonce + off, nbytes - off < 16 ? nbytes - off : 16));
                y = tab_mul<kTab1>(y ^ u32x4{0u, 0u, 0u, bswap(nbytes * 8u)});
                lds<u32x4>(kJ0) = y;
                lds<u32x4>(kEJ0) = aes_encrypt<NR>(y, rk, lo0, lo1, lo2, lo3);
            }
            __syncthreads();
        }

        // ---- E: CTR over the blocks; 1024 GHASH chains folded with M = H^1024
        const u32x4 j0 = lds<u32x4>(kJ0);
        const uint32_t j0x = __builtin_amdgcn_readfirstlane(j0.x);
        const uint32_t j0y = __builtin_amdgcn_readfirstlane(j0.y);
        const uint32_t j0z = __builtin_amdgcn_readfirstlane(j0.z);
        const uint32_t ctr0 = bswap(__builtin_amdgcn_readfirstlane(j0.w));
        const uint64_t len = it.len;
        const uint64_t src_a = it.in + (DEC ? nbytes : 0), dst_a = it.out + (DEC ? 0 : nbytes);
        gcbytes src = reinterpret_cast<gcbytes>(src_a);
        gbytes dst = reinterpret_cast<gbytes>(dst_a);
        if (!DEC && uint32_t(tid) < nbytes) reinterpret_cast<gbytes>(it.out)[tid] = nonce[tid];
        const uint64_t nb = (len + 15) >> 4, nfull = len >> 4;
        const uint64_t pad = (uint64_t(kGcmThreads) - (nb & (kGcmThreads - 1))) & (kGcmThreads - 1);
        const uint64_t rows = (nb + pad) / kGcmThreads;
        const bool fast = ((src_a | dst_a) & 3) == 0;
        u32x4 acc = {0u, 0u, 0u, 0u};
        GCM_MARK(6, rows);
        for (uint64_t r = 0; r < rows; ++r) {
            const int64_t b = int64_t(r * kGcmThreads + uint64_t(tid)) - int64_t(pad);
            u32x4 x = {0u, 0u, 0u, 0u};
            if (b >= 0) {
                const uint64_t off = uint64_t(b) * 16;
                const bool whole = uint64_t(b) < nfull;
                const uint32_t n = whole ? 16u : uint32_t(len - off);
                // the data load goes out before the AES rounds that hide its latency
                const u32x4 d = whole && fast ? *reinterpret_cast<const GLOBAL u32x4a4 *>(src + off)
                                              : load_bytes(src + off, n);
                const uint32_t ctr = ctr0 + 1u + uint32_t(b);  // inc32 from J0, mod 2^32
                const u32x4 ks = aes_encrypt<NR>(u32x4{j0x, j0y, j0z, bswap(ctr)}, rk, lo0, lo1, lo2, lo3);
                const u32x4 c = keep_bytes(d ^ ks, n);
                if (whole && fast)
                    *reinterpret_cast<GLOBAL u32x4a4 *>(dst + off) = c;
                else
                    store_bytes(dst + off, c, n);
                x = DEC ? d : c;
            }
            acc = r == 0 ? x : (tab_mul<kTabM>(acc) ^ x);
        }
        __syncthreads();  // every wave is past its last AES round: the T-tables are dead
        lds<u32x4>(kZ + 16 * tid) = acc;
        if (wave == 1 && lane < 32) build_table(kTab32, lds<u32x4>(kH32), lane);
        __syncthreads();
        GCM_MARK(7, rows);

        // ---- F: fold the chains: P_j = sum_i Z_(32j+i) H^(32-i); D = sum_j P_j H^(32(31-j))
        if (wave == 0 && lane < 32) {
            u32x4 p = {0u, 0u, 0u, 0u};
#pragma unroll 1
            for (int i = 0; i < 32; ++i) p = tab_mul<kTab1>(p ^ lds<u32x4>(kZ + 16 * (32 * lane + i)));
            lds<u32x4>(kP + 16 * lane) = p;
        }
        __syncthreads();
        GCM_MARK(8, idx);
        if (tid == 0) {
            u32x4 d = lds<u32x4>(kP);
#pragma unroll 1
            for (int j = 1; j < 32; ++j) d = tab_mul<kTab32>(d) ^ lds<u32x4>(kP + 16 * j);
            const uint64_t bits = len * 8;  // [len(A)]_64 = 0 || [len(C)]_64
            const u32x4 lb = {0u, 0u, bswap(uint32_t(bits >> 32)), bswap(uint32_t(bits))};
            const u32x4 tag = tab_mul<kTab1>(d ^ lb) ^ lds<u32x4>(kEJ0);
            if (DEC) {
                const u32x4 t = load_bytes(src + len, 16) ^ tag;
                a.ok[it.slot] = (t.x | t.y | t.z | t.w) == 0u ? 1 : 0;
            } else {
                store_bytes(dst + len, tag, 16);
            }
        }
        GCM_MARK(10, idx);
    }
}

// Work list of the chunks rc_chunk_device wrote: one workgroup per run of spw streams.
__global__ __launch_bounds__(256) void rc_gcm_items_kernel(GcmChunkLists c, GcmItem *__restrict__ items) {
    const uint64_t s0 = blockIdx.x * c.spw, s1 = s0 + c.spw < c.n ? s0 + c.spw : c.n;
    const uint64_t over = c.nonce_bytes + 16;
    for (uint64_t s = s0; s < s1; ++s) {
        const int64_t cnt = c.counts[s];
        const uint64_t base = c.cut_base[s], p = c.ptrs[s], ob = c.out_base[s], o = c.chunk_off[s];
        const uint64_t *e = c.cuts + base;
        for (int64_t k = threadIdx.x; k < cnt; k += 256) {
            const uint64_t start = k ? e[k - 1] : 0, len = e[k] - start, slot = base + uint64_t(k);
            items[o + uint64_t(k)] = GcmItem{p + start, len, c.out + ob + start + uint64_t(k) * over,
                                             c.keys + 64 * slot, c.nonces + c.nonce_bytes * slot, slot};
        }
    }
}

namespace {
thread_local char g_gcm_err[256];

int gcm_status(const char *what) {
    const hipError_t e = hipGetLastError();
    if (e == hipSuccess) return 0;
    snprintf(g_gcm_err, sizeof g_gcm_err, "%s: %s", what, hipGetErrorString(e));
    return 1;
}

template <int NR>
int launch_nr(bool decrypt, const GcmArgs &args, unsigned groups, hipStream_t stream) {
    if (decrypt)
        rc_gcm_kernel<NR, true><<<groups, kGcmThreads, 0, stream>>>(args);
    else
        rc_gcm_kernel<NR, false><<<groups, kGcmThreads, 0, stream>>>(args);
    return gcm_status("rc_gcm_kernel");
}
}  // namespace

const char *rc_gcm_launch_error(void) { return g_gcm_err; }

#ifdef RC_GCM_TRACE
int rc_gcm_trace_read(unsigned long long *out, hipStream_t st) {
    if (hipMemcpyFromSymbolAsync(out, HIP_SYMBOL(g_gcm_trace), sizeof g_gcm_trace, 0,
                                 hipMemcpyDeviceToHost, st) != hipSuccess)
        return 1;
    return hipStreamSynchronize(st) != hipSuccess;
}
int rc_gcm_trace_reset(void) {
    const unsigned long long z[4] = {0, 0, 0, 0};
    return hipMemcpyToSymbol(HIP_SYMBOL(g_gcm_trace), z, sizeof z) != hipSuccess;
}
#endif

int rc_gcm_launch(uint32_t key_bytes, bool decrypt, const GcmArgs &args, unsigned groups,
                  hipStream_t stream) {
    if (!groups) return 0;
    switch (key_bytes) {
        case 16: return launch_nr<10>(decrypt, args, groups, stream);
        case 24: return launch_nr<12>(decrypt, args, groups, stream);
        case 32: return launch_nr<14>(decrypt, args, groups, stream);
        default:
            snprintf(g_gcm_err, sizeof g_gcm_err, "bad AES key size %u", key_bytes);
            return 1;
    }
}

int rc_gcm_launch_chunk_items(const GcmChunkLists &c, GcmItem *items, hipStream_t stream) {
    if (!c.n) return 0;
    const unsigned groups = static_cast<unsigned>((c.n + c.spw - 1) / c.spw);
    rc_gcm_items_kernel<<<groups, 256, 0, stream>>>(c, items);
    return gcm_status("rc_gcm_items_kernel");
}
