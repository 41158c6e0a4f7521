/*
 * blake2b_oracle.c -- TEST INFRASTRUCTURE ONLY: plain-C restatement of the digest replicat's
 * snapshot loop takes of every chunk.
 *
 * Reference call sites: /root/reference/replicat/repository.py:1462
 * (`digest = self.props.hash_digest(output_chunk)`), the default hashing adapter
 * repository.py:217 (`DEFAULT_HASHER_NAME = 'blake2b'`) and
 * replicat/utils/adapters.py:195-197,224-225 (`blake2b(length=64).digest(data)` =
 * `hashlib.blake2b(data, digest_size=self.digest_size).digest()`).
 *
 * The algorithm lives in a dependency that is not in /root/reference: CPython's hashlib
 * (its bundled BLAKE2 reference code; the interpreter here and on the GPU box is 3.10.12).
 * hashlib's blake2b is RFC 7693 BLAKE2b; this file restates RFC 7693 §3.2 (compression F,
 * mixing G) and Appendix C's unkeyed hash for digest sizes 1..64.
 * Parity pin: tests/test_digest_oracle.py checks it against RFC 7693 Appendix A
 * (BLAKE2b-512("abc")) and against hashlib itself on random messages of every length class.
 *
 * Imported only by tests/ and bench.py's cpu_baseline leg; never by replicat_amd/.
 */
#include <stdint.h>
#include <string.h>

static const uint64_t IV[8] = {0x6a09e667f3bcc908ULL, 0xbb67ae8584caa73bULL, 0x3c6ef372fe94f82bULL,
                               0xa54ff53a5f1d36f1ULL, 0x510e527fade682d1ULL, 0x9b05688c2b3e6c1fULL,
                               0x1f83d9abfb41bd6bULL, 0x5be0cd19137e2179ULL};

/* RFC 7693 §2.7 message schedule SIGMA */
static const uint8_t SIGMA[12][16] = {
    {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15},
    {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3},
    {11, 8, 12, 0, 5, 2, 15, 13, 10, 14, 3, 6, 7, 1, 9, 4},
    {7, 9, 3, 1, 13, 12, 11, 14, 2, 6, 5, 10, 4, 0, 15, 8},
    {9, 0, 5, 7, 2, 4, 10, 15, 14, 1, 11, 12, 6, 8, 3, 13},
    {2, 12, 6, 10, 0, 11, 8, 3, 4, 13, 7, 5, 15, 14, 1, 9},
    {12, 5, 1, 15, 14, 13, 4, 10, 0, 7, 6, 3, 9, 2, 8, 11},
    {13, 11, 7, 14, 12, 1, 3, 9, 5, 0, 15, 4, 8, 6, 2, 10},
    {6, 15, 14, 9, 11, 3, 0, 8, 12, 2, 13, 7, 1, 4, 10, 5},
    {10, 2, 8, 4, 7, 6, 1, 5, 15, 11, 9, 14, 3, 12, 13, 0},
    {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15},
    {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3}};

static uint64_t rotr64(uint64_t x, unsigned n) { return (x >> n) | (x << (64 - n)); }

static uint64_t le64(const uint8_t *p) {
    uint64_t v = 0;
    for (int i = 7; i >= 0; --i) v = (v << 8) | p[i];
    return v;
}

/* RFC 7693 §3.1 mixing function G (R1..R4 = 32, 24, 16, 63) */
#define G(a, b, c, d, x, y)                \
    do {                                   \
        v[a] = v[a] + v[b] + (x);          \
        v[d] = rotr64(v[d] ^ v[a], 32);    \
        v[c] = v[c] + v[d];                \
        v[b] = rotr64(v[b] ^ v[c], 24);    \
        v[a] = v[a] + v[b] + (y);          \
        v[d] = rotr64(v[d] ^ v[a], 16);    \
        v[c] = v[c] + v[d];                \
        v[b] = rotr64(v[b] ^ v[c], 63);    \
    } while (0)

/* RFC 7693 §3.2 compression F; t < 2^64 here (t's high word is 0) */
static void compress(uint64_t h[8], const uint8_t block[128], uint64_t t, int last) {
    uint64_t v[16], m[16];
    for (int i = 0; i < 16; ++i) m[i] = le64(block + 8 * i);
    for (int i = 0; i < 8; ++i) {
        v[i] = h[i];
        v[i + 8] = IV[i];
    }
    v[12] ^= t;
    if (last) v[14] = ~v[14];
    for (int r = 0; r < 12; ++r) {
        const uint8_t *s = SIGMA[r];
        G(0, 4, 8, 12, m[s[0]], m[s[1]]);
        G(1, 5, 9, 13, m[s[2]], m[s[3]]);
        G(2, 6, 10, 14, m[s[4]], m[s[5]]);
        G(3, 7, 11, 15, m[s[6]], m[s[7]]);
        G(0, 5, 10, 15, m[s[8]], m[s[9]]);
        G(1, 6, 11, 12, m[s[10]], m[s[11]]);
        G(2, 7, 8, 13, m[s[12]], m[s[13]]);
        G(3, 4, 9, 14, m[s[14]], m[s[15]]);
    }
    for (int i = 0; i < 8; ++i) h[i] ^= v[i] ^ v[i + 8];
}

/* Unkeyed BLAKE2b of data[0..len) with an outlen-byte digest (1..64), RFC 7693 Appendix C.
 * Returns 0, or -1 for a bad outlen. */
int oc_blake2b(const uint8_t *data, uint64_t len, uint32_t outlen, uint8_t *out) {
    if (outlen < 1 || outlen > 64) return -1;
    uint64_t h[8];
    memcpy(h, IV, sizeof h);
    h[0] ^= 0x01010000ULL ^ outlen; /* parameter block: fanout 1, depth 1, no key */
    uint8_t block[128];
    uint64_t done = 0;
    while (len - done > 128) {
        compress(h, data + done, done + 128, 0);
        done += 128;
    }
    memset(block, 0, sizeof block);
    if (len > done) memcpy(block, data + done, len - done);
    compress(h, block, len, 1);
    for (uint32_t i = 0; i < outlen; ++i) out[i] = (uint8_t)(h[i / 8] >> (8 * (i % 8)));
    return 0;
}

/* Digests of the chunks of one stream: chunk k = [ends[k-1], ends[k]) (from 0), into
 * out + 64 * k (first outlen bytes; the rest of each slot zeroed). */
int oc_blake2b_chunks(const uint8_t *stream, const uint64_t *ends, uint64_t n, uint32_t outlen,
                      uint8_t *out) {
    uint64_t s = 0;
    for (uint64_t k = 0; k < n; ++k) {
        memset(out + 64 * k, 0, 64);
        if (oc_blake2b(stream + s, ends[k] - s, outlen, out + 64 * k)) return -1;
        s = ends[k];
    }
    return 0;
}
