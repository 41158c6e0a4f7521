/*
 * aesgcm_oracle.c -- TEST INFRASTRUCTURE ONLY: plain-C restatement of the AES-GCM chunk
 * encryption of replicat's encrypted snapshots.
 *
 * What the reference does (/root/reference):
 *   replicat/repository.py:1470-1473   encrypted_contents = encrypt(chunk, derive_shared_subkey(digest))
 *   replicat/repository.py:132-137     derive_shared_subkey = shared_kdf.derive(shared_key,
 *                                      context=digest, params=shared_kdf_params)
 *   replicat/utils/adapters.py:205-213 blake2b.derive = hashlib.blake2b(context, salt=params,
 *                                      digest_size=length, key=key_material); length = the
 *                                      cipher's key bytes (repository.py:623-627)
 *   replicat/utils/adapters.py:131-144 AEADCipherAdapterMixin.encrypt: nonce = os.urandom(nonce_bytes);
 *                                      return nonce + AESGCM(key).encrypt(nonce, data, None);
 *                                      decrypt splits the nonce off, InvalidTag -> DecryptionError
 *   replicat/utils/adapters.py:151-158 aes_gcm(key_bits=256, nonce_bits=96), key_bits in {128,192,256}
 *
 * AESGCM comes from the third-party `cryptography` package (not vendored under /root/reference and
 * not installed here), a binding of OpenSSL's EVP AES-GCM.  Its published algorithm is restated:
 * FIPS 197 (AES: key expansion §5.2, cipher §5.1) and NIST SP 800-38D (GCM: GHASH §6.4, GCTR §6.5,
 * J0 §7.1 for any IV length, tag = GCTR(J0, S), no associated data).  encrypt returns C || T.
 *
 * Deliberately the slow textbook form (byte-wise rounds, bit-serial GF(2^128) multiply): nothing
 * here is shared with the HIP kernels.  Pinned by tests/test_gcm_oracle.py against FIPS 197 /
 * SP 800-38D known answers and against fixtures made with the host's OpenSSL libcrypto
 * (tests/golden/make_gcm_golden.py -> tests/golden/gcm.json).
 */
#include <stdint.h>
#include <string.h>

/* ------------------------------------------------------------------ AES (FIPS 197) */

static uint8_t xtime(uint8_t a) { return (uint8_t)((a << 1) ^ ((a & 0x80) ? 0x1b : 0)); }

static uint8_t gmul8(uint8_t a, uint8_t b) { /* §4.2 */
    uint8_t p = 0;
    while (b) {
        if (b & 1) p ^= a;
        a = xtime(a);
        b >>= 1;
    }
    return p;
}

static uint8_t sbox_entry(uint8_t x) { /* §5.1.1: multiplicative inverse, then the affine map */
    uint8_t inv = 0;
    if (x)
        for (int c = 1; c < 256; ++c)
            if (gmul8(x, (uint8_t)c) == 1) {
                inv = (uint8_t)c;
                break;
            }
    uint8_t s = inv;
    for (int i = 1; i <= 4; ++i) s ^= (uint8_t)((inv << i) | (inv >> (8 - i)));
    return s ^ 0x63;
}

static uint8_t SBOX[256];
static int sbox_ready;

static void init_sbox(void) {
    if (sbox_ready) return;
    for (int i = 0; i < 256; ++i) SBOX[i] = sbox_entry((uint8_t)i);
    sbox_ready = 1;
}

/* §5.2: Nk = key_bytes / 4, Nr = Nk + 6; w holds 4 (Nr + 1) words as bytes */
static int key_expansion(const uint8_t *key, int key_bytes, uint8_t w[240]) {
    const int nk = key_bytes / 4, nr = nk + 6, total = 4 * (nr + 1);
    uint8_t rcon = 1;
    memcpy(w, key, (size_t)key_bytes);
    for (int i = nk; i < total; ++i) {
        uint8_t t[4];
        memcpy(t, w + 4 * (i - 1), 4);
        if (i % nk == 0) {
            const uint8_t t0 = t[0];
            t[0] = SBOX[t[1]] ^ rcon;
            t[1] = SBOX[t[2]];
            t[2] = SBOX[t[3]];
            t[3] = SBOX[t0];
            rcon = xtime(rcon);
        } else if (nk > 6 && i % nk == 4) {
            for (int j = 0; j < 4; ++j) t[j] = SBOX[t[j]];
        }
        for (int j = 0; j < 4; ++j) w[4 * i + j] = w[4 * (i - nk) + j] ^ t[j];
    }
    return nr;
}

/* §5.1: state s[r + 4c] = in[r + 4c] */
static void aes_block(const uint8_t *w, int nr, const uint8_t in[16], uint8_t out[16]) {
    uint8_t s[16], t[16];
    for (int i = 0; i < 16; ++i) s[i] = in[i] ^ w[i];
    for (int round = 1; round <= nr; ++round) {
        for (int i = 0; i < 16; ++i) s[i] = SBOX[s[i]];                      /* SubBytes */
        for (int r = 0; r < 4; ++r)                                          /* ShiftRows */
            for (int c = 0; c < 4; ++c) t[r + 4 * c] = s[r + 4 * ((c + r) % 4)];
        if (round != nr) {                                                   /* MixColumns */
            for (int c = 0; c < 4; ++c) {
                const uint8_t *a = t + 4 * c;
                s[4 * c + 0] = gmul8(a[0], 2) ^ gmul8(a[1], 3) ^ a[2] ^ a[3];
                s[4 * c + 1] = a[0] ^ gmul8(a[1], 2) ^ gmul8(a[2], 3) ^ a[3];
                s[4 * c + 2] = a[0] ^ a[1] ^ gmul8(a[2], 2) ^ gmul8(a[3], 3);
                s[4 * c + 3] = gmul8(a[0], 3) ^ a[1] ^ a[2] ^ gmul8(a[3], 2);
            }
        } else {
            memcpy(s, t, 16);
        }
        for (int i = 0; i < 16; ++i) s[i] ^= w[16 * round + i];             /* AddRoundKey */
    }
    memcpy(out, s, 16);
}

/* ------------------------------------------------------------------ GCM (SP 800-38D) */

/* §6.3 Algorithm 1: Z = X . Y in GF(2^128); bit 0 = MSB of byte 0; R = 11100001 || 0^120 */
static void gf_mul(const uint8_t X[16], const uint8_t Y[16], uint8_t Z[16]) {
    uint8_t V[16], acc[16] = {0};
    memcpy(V, Y, 16);
    for (int i = 0; i < 128; ++i) {
        if (X[i / 8] & (0x80 >> (i % 8)))
            for (int j = 0; j < 16; ++j) acc[j] ^= V[j];
        const int lsb = V[15] & 1;
        for (int j = 15; j > 0; --j) V[j] = (uint8_t)((V[j] >> 1) | (V[j - 1] << 7));
        V[0] >>= 1;
        if (lsb) V[0] ^= 0xe1;
    }
    memcpy(Z, acc, 16);
}

/* §6.4: continue Y = GHASH_H over the zero-padded 16-byte blocks of data */
static void ghash_update(const uint8_t H[16], uint8_t Y[16], const uint8_t *data, uint64_t len) {
    for (uint64_t off = 0; off < len; off += 16) {
        uint8_t blk[16] = {0};
        const uint64_t n = len - off < 16 ? len - off : 16;
        memcpy(blk, data + off, (size_t)n);
        for (int j = 0; j < 16; ++j) blk[j] ^= Y[j];
        gf_mul(blk, H, Y);
    }
}

static void put_be64(uint8_t *p, uint64_t v) {
    for (int i = 7; i >= 0; --i) {
        p[i] = (uint8_t)v;
        v >>= 8;
    }
}

static void inc32(uint8_t cb[16]) { /* §6.2: the last 32 bits, big-endian, mod 2^32 */
    for (int i = 15; i >= 12; --i)
        if (++cb[i]) break;
}

struct gcm_ctx {
    uint8_t w[240];
    int nr;
    uint8_t H[16], J0[16];
};

static int gcm_setup(struct gcm_ctx *g, const uint8_t *key, uint32_t key_bytes, const uint8_t *iv,
                     uint64_t iv_len) {
    if (key_bytes != 16 && key_bytes != 24 && key_bytes != 32) return 1;
    if (iv_len == 0) return 2;
    init_sbox();
    g->nr = key_expansion(key, (int)key_bytes, g->w);
    const uint8_t zero[16] = {0};
    aes_block(g->w, g->nr, zero, g->H);
    if (iv_len == 12) { /* §7.1 step 2: J0 = IV || 0^31 || 1 */
        memcpy(g->J0, iv, 12);
        g->J0[12] = g->J0[13] = g->J0[14] = 0;
        g->J0[15] = 1;
    } else { /* J0 = GHASH_H(IV || 0^(s+64) || [len(IV)]_64) */
        uint8_t Y[16] = {0}, lb[16] = {0};
        ghash_update(g->H, Y, iv, iv_len);
        put_be64(lb + 8, iv_len * 8);
        ghash_update(g->H, Y, lb, 16);
        memcpy(g->J0, Y, 16);
    }
    return 0;
}

/* §6.5 GCTR from ICB = inc32(J0) */
static void gctr(const struct gcm_ctx *g, const uint8_t *in, uint64_t len, uint8_t *out) {
    uint8_t cb[16], ks[16];
    memcpy(cb, g->J0, 16);
    for (uint64_t off = 0; off < len; off += 16) {
        inc32(cb);
        aes_block(g->w, g->nr, cb, ks);
        const uint64_t n = len - off < 16 ? len - off : 16;
        for (uint64_t j = 0; j < n; ++j) out[off + j] = in[off + j] ^ ks[j];
    }
}

/* §7.1 steps 5-6 with A empty (adapters.py:134 passes associated_data=None) */
static void tag_of(const struct gcm_ctx *g, const uint8_t *ct, uint64_t len, uint8_t T[16]) {
    uint8_t S[16] = {0}, lb[16] = {0}, ej[16];
    ghash_update(g->H, S, ct, len);
    put_be64(lb + 8, len * 8);
    ghash_update(g->H, S, lb, 16);
    aes_block(g->w, g->nr, g->J0, ej);
    for (int j = 0; j < 16; ++j) T[j] = S[j] ^ ej[j];
}

/* AES-{128,192,256} of one block (FIPS 197 Appendix C) */
int oc_aes_block(const uint8_t *key, uint32_t key_bytes, const uint8_t *in, uint8_t *out) {
    if (key_bytes != 16 && key_bytes != 24 && key_bytes != 32) return 1;
    init_sbox();
    uint8_t w[240];
    const int nr = key_expansion(key, (int)key_bytes, w);
    aes_block(w, nr, in, out);
    return 0;
}

/* out (len + 16 bytes) = C || T = AESGCM(key).encrypt(iv, pt, None) */
int oc_gcm_encrypt(const uint8_t *key, uint32_t key_bytes, const uint8_t *iv, uint64_t iv_len,
                   const uint8_t *pt, uint64_t len, uint8_t *out) {
    struct gcm_ctx g;
    const int rc = gcm_setup(&g, key, key_bytes, iv, iv_len);
    if (rc) return rc;
    gctr(&g, pt, len, out);
    tag_of(&g, out, len, out + len);
    return 0;
}

/* in = C || T (len + 16 bytes) -> pt (len bytes); 3 when the tag does not verify
 * (cryptography's InvalidTag -> replicat's DecryptionError) */
int oc_gcm_decrypt(const uint8_t *key, uint32_t key_bytes, const uint8_t *iv, uint64_t iv_len,
                   const uint8_t *in, uint64_t len, uint8_t *pt) {
    struct gcm_ctx g;
    const int rc = gcm_setup(&g, key, key_bytes, iv, iv_len);
    if (rc) return rc;
    uint8_t T[16];
    tag_of(&g, in, len, T);
    gctr(&g, in, len, pt);
    uint8_t diff = 0;
    for (int j = 0; j < 16; ++j) diff |= (uint8_t)(T[j] ^ in[len + j]);
    return diff ? 3 : 0;
}

/* the field product, for tests of the device's table construction */
void oc_gf_mul(const uint8_t *X, const uint8_t *Y, uint8_t *Z) { gf_mul(X, Y, Z); }
