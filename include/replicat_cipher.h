/*
 * replicat_cipher.h -- C ABI of the MI355X (gfx950) AES-GCM chunk encryption.
 *
 * Replaces, for the snapshot path of encrypted repositories, the per-chunk
 *     encrypted_contents = self.props.encrypt(output_chunk, self.props.derive_shared_subkey(digest))
 * of /root/reference/replicat/repository.py:1470-1473 with replicat's default cipher
 * `aes_gcm(key_bits=256, nonce_bits=96)` (replicat/utils/adapters.py:151-158; default name
 * repository.py:216), i.e. AEADCipherAdapterMixin (adapters.py:117-148):
 *     encrypt(data, key) = nonce || AESGCM(key).encrypt(nonce, data, None), nonce = os.urandom(nonce_bytes)
 *     decrypt(blob, key) = AESGCM(key).decrypt(blob[:nonce_bytes], blob[nonce_bytes:], None),
 *                          InvalidTag -> DecryptionError
 * AESGCM (the `cryptography` package) is AES (FIPS 197) in GCM (NIST SP 800-38D) with the 16-byte
 * tag appended to the ciphertext and no associated data.  Nonces are the caller's: the adapter
 * draws them from os.urandom, and so does the Python layer (replicat_amd/cipher.py).
 *
 * The per-chunk subkeys come from rc_blake2b_derive_chunks (replicat_digest.h).  Implemented by
 * replicat_amd/csrc/{capi_cipher.cpp,gcm.hip} in replicat_amd/libreplicat_chunker.so.
 */
#ifndef REPLICAT_CIPHER_H
#define REPLICAT_CIPHER_H

#include <stdint.h>

#include "replicat_chunker.h"

#ifdef __cplusplus
extern "C" {
#endif

#define RC_ERR_KEY_SIZE 6   /* "Invalid key size": aes_gcm's ValueError for key_bits (adapters.py:155-156) */
#define RC_ERR_NONCE_SIZE 7 /* "Nonce must be between 8 and 128 bytes": AESGCM's ValueError */
#define RC_ERR_TAG 8        /* a tag did not verify: InvalidTag -> DecryptionError (adapters.py:141-144) */

typedef struct rc_gcm rc_gcm;

/* `aes_gcm(key_bits=, nonce_bits=)` (adapters.py:154-158) bound to HIP device `device`: key_bits
 * 128 / 192 / 256; nonce_bytes = nonce_bits / 8 must lie in 8..128 (96 bits is the direct J0 case,
 * other lengths take J0 = GHASH(IV || pad || [len(IV)]_64)). */
int rc_gcm_create(uint32_t key_bits, uint32_t nonce_bits, int device, rc_gcm **out);
void rc_gcm_destroy(rc_gcm *g);
uint32_t rc_gcm_key_bytes(const rc_gcm *g);
uint32_t rc_gcm_nonce_bytes(const rc_gcm *g);

/* encrypt (adapters.py:131-134) of n DEVICE buffers d_in[i] (lens[i] bytes) with the key at
 * d_keys[i] (key_bytes) and the nonce at d_nonces[i] (nonce_bytes): d_out[i] receives
 * nonce || C || T (nonce_bytes + lens[i] + 16 bytes).  Enqueued on hip_stream. */
int rc_gcm_encrypt_device(rc_gcm *g, uint64_t n, const uint8_t *const *d_in, const uint64_t *lens,
                          const uint8_t *const *d_keys, const uint8_t *const *d_nonces,
                          uint8_t *const *d_out, void *hip_stream);

/* decrypt (adapters.py:136-144) of n DEVICE blobs nonce || C || T of lens[i] bytes: d_out[i]
 * receives lens[i] - nonce_bytes - 16 bytes of plaintext and d_ok[i] = 1 when the tag verifies,
 * else 0 (also for a blob too short to hold nonce and tag).  Enqueued on hip_stream. */
int rc_gcm_decrypt_device(rc_gcm *g, uint64_t n, const uint8_t *const *d_in, const uint64_t *lens,
                          const uint8_t *const *d_keys, uint8_t *const *d_out, uint8_t *d_ok,
                          void *hip_stream);

/* The same over HOST buffers (copied in, processed, copied back; blocking).  decrypt fills ok[i]
 * and returns RC_ERR_TAG when any of them is 0. */
int rc_gcm_encrypt_host(rc_gcm *g, uint64_t n, const uint8_t *const *in, const uint64_t *lens,
                        const uint8_t *const *keys, const uint8_t *const *nonces,
                        uint8_t *const *out);
int rc_gcm_decrypt_host(rc_gcm *g, uint64_t n, const uint8_t *const *in, const uint64_t *lens,
                        const uint8_t *const *keys, uint8_t *const *out, uint8_t *ok);

/* Output layout of rc_gcm_encrypt_chunks for n streams of lens[i] bytes: stream i's region starts
 * at out_base[i] (16-byte aligned; room for nonce_bytes + 16 more bytes per cut slot of
 * rc_cut_capacity).  Returns the total bytes.  Host-only. */
uint64_t rc_gcm_chunks_layout(const rc_gcm *g, const rc_chunker *layout, uint64_t n,
                              const uint64_t *lens, uint64_t *out_base);

/* encrypt(chunk, subkey) of every chunk rc_chunk_device wrote for the same streams
 * (repository.py:1470-1473): chunk k of stream i, cut range [s, e), cut slot c = cut_base[i] + k,
 * is encrypted with the key at d_keys + 64 c (where rc_blake2b_derive_chunks leaves it) and the
 * nonce at d_nonces + nonce_bytes * c into d_out + out_base[i] + s + k * (nonce_bytes + 16) as
 * nonce || C || T.  Counts are read on the device (no host sync).  Enqueued on hip_stream. */
int rc_gcm_encrypt_chunks(rc_gcm *g, const rc_chunker *layout, uint64_t n,
                          const uint8_t *const *d_streams, const uint64_t *lens,
                          const uint64_t *d_cuts, const int64_t *d_counts, const uint8_t *d_keys,
                          const uint8_t *d_nonces, uint8_t *d_out, void *hip_stream);

/* Kernel timing for benchmarks: while enabled, each enqueue records HIP events around its kernels
 * on the launch stream; read returns the summed milliseconds and clears. */
int rc_gcm_timing_enable(rc_gcm *g, int enable);
int rc_gcm_timing_read(rc_gcm *g, double *ms, uint64_t *calls);

#ifdef __cplusplus
}
#endif

#endif /* REPLICAT_CIPHER_H */
