/*
 * replicat_digest.h -- C ABI of the MI355X (gfx950) BLAKE2b chunk digests.
 *
 * Replaces, for the snapshot path, the per-chunk `self.props.hash_digest(output_chunk)` of
 * /root/reference/replicat/repository.py:1462, i.e. replicat's default hashing adapter
 * `blake2b(length=64)` (replicat/utils/adapters.py:195-197,224-225; default name
 * repository.py:217): hashlib.blake2b(data, digest_size=length).digest(), which is RFC 7693
 * BLAKE2b, unkeyed, without salt or personalisation.
 *
 * The incremental and keyed entries (rc_blake2b_state_*, rc_blake2b_update_device) cover the
 * rest of that adapter: `incremental_hasher()` (adapters.py:227-228 -> HashlibIncrementalHasher
 * :106-114, the per-file digest of repository.py:1433-1446), `derive(key_material, params,
 * context)` (the shared-subkey KDF of encrypted repositories, adapters.py:203-211,
 * repository.py:132-137) and `mac(message, params)` (adapters.py:217-221): hashlib.blake2b
 * with key / salt / person set, which RFC 7693 defines as the parameter block XORed into the IV
 * and the zero-padded key prepended as a first block.
 *
 * Digests live in 64-byte slots: the digest of message i (or of cut slot s) is the first
 * digest_size bytes of slot i (s); the rest of the slot is zero.  Implemented by
 * replicat_amd/csrc/{capi_digest.cpp,blake2b.hip} in replicat_amd/libreplicat_chunker.so.
 */
#ifndef REPLICAT_DIGEST_H
#define REPLICAT_DIGEST_H

#include <stdint.h>

#include "replicat_chunker.h"

#ifdef __cplusplus
extern "C" {
#endif

#define RC_DIGEST_SLOT 64
#define RC_ERR_DIGEST_SIZE 4 /* "digest_size must be between 1 and 64 bytes": hashlib.blake2b's
                                ValueError for the adapter's `length` (adapters.py:196-197) */

#define RC_ERR_B2_PARAM 5   /* "maximum key length is 64 bytes" / "maximum salt length is 16 bytes"
                              / "maximum person length is 16 bytes": hashlib's ValueErrors */

typedef struct rc_hasher rc_hasher;

/* An incremental BLAKE2b in DEVICE memory (256 bytes, 16-byte aligned): chaining value, bytes
 * compressed so far, and the last 1..128 message bytes not yet compressed.  Built on the host
 * by rc_blake2b_state_init, copied to the device, advanced by rc_blake2b_update_device. */
typedef struct rc_blake2b_state {
    uint64_t h[8];
    uint64_t t;           /* bytes compressed */
    uint64_t buflen;      /* pending bytes in buf, 0..128 */
    uint8_t buf[128];
    uint32_t digest_size; /* 1..64 */
    uint32_t reserved0;
    uint64_t reserved[5];
} rc_blake2b_state;

/* `blake2b(length=digest_size)` (adapters.py:196-197) bound to HIP device `device`. */
int rc_blake2b_create(uint32_t digest_size, int device, rc_hasher **out);
void rc_blake2b_destroy(rc_hasher *h);
uint32_t rc_blake2b_digest_size(const rc_hasher *h);

/* `digest(data)` (adapters.py:224-225) of n DEVICE buffers d_ptrs[i] of lens[i] bytes (any
 * alignment; NULL allowed for an empty buffer) into d_out + 64 * i.  Enqueued on hip_stream;
 * returns without synchronising. */
int rc_blake2b_device(rc_hasher *h, uint64_t n, const uint8_t *const *d_ptrs,
                      const uint64_t *lens, uint8_t *d_out, void *hip_stream);

/* The same for n HOST buffers into host out + 64 * i: copies in, hashes, copies back; blocking. */
int rc_blake2b_host(rc_hasher *h, uint64_t n, const uint8_t *const *ptrs, const uint64_t *lens,
                    uint8_t *out);

/* `hash_digest` of every chunk that rc_chunk_device wrote for the same streams (repository.py
 * :1455-1462): chunk k of stream i is [cuts[cut_base[i]+k-1], cuts[cut_base[i]+k]) (from 0
 * for k = 0), where cut_base is the capacity prefix of rc_cut_capacity(layout, ...).  Its digest
 * goes to d_digests + 64 * (cut_base[i] + k).  Counts are read on the device (no host sync).
 * Enqueued on hip_stream. */
int rc_blake2b_chunks(rc_hasher *h, const rc_chunker *layout, uint64_t n,
                      const uint8_t *const *d_streams, const uint64_t *lens,
                      const uint64_t *d_cuts, const int64_t *d_counts, uint8_t *d_digests,
                      void *hip_stream);

/* rc_chunk_host (replicat_chunker.h) plus the digest of every chunk, the snapshot loop's
 * chunkify + hash_digest over host streams: digests[64 * (cut_base[i] + k)].  Blocking. */
int rc_chunk_digest_host(rc_chunker *ch, rc_hasher *h, uint64_t n, const uint8_t *const *streams,
                         const uint64_t *lens, const uint64_t *last_piece, uint32_t flags,
                         uint64_t *cuts, int64_t *counts, uint8_t *digests);

/* hashlib.blake2b(digest_size=, key=, salt=, person=) before any data (RFC 7693 §2.8, §3.3):
 * host-only, no device work.  Lengths above 64 / 16 / 16 bytes fail with RC_ERR_B2_PARAM;
 * shorter salt / person are zero-padded as hashlib does.  NULL pointers mean empty. */
int rc_blake2b_state_init(uint32_t digest_size, const uint8_t *key, uint32_t keylen,
                          const uint8_t *salt, uint32_t saltlen, const uint8_t *person,
                          uint32_t personlen, rc_blake2b_state *out);

/* n incremental updates (HashlibIncrementalHasher.feed / .digest, adapters.py:106-114): item i
 * feeds the DEVICE buffer d_ptrs[i] (lens[i] bytes) into the DEVICE state d_states[i]; when
 * finals[i] is non-zero it also finalises, writing the digest into d_out + 64 * i and leaving
 * the state untouched (so one read-only state -- e.g. a KDF or MAC key -- may serve many final
 * items).  A state may appear in at most one non-final item per call.  Enqueued on hip_stream. */
int rc_blake2b_update_device(rc_hasher *h, uint64_t n, rc_blake2b_state *const *d_states,
                             const uint8_t *const *d_ptrs, const uint64_t *lens,
                             const uint8_t *finals, uint8_t *d_out, void *hip_stream);

/* `derive_shared_subkey(digest)` of every chunk rc_blake2b_chunks digested for the same streams
 * (repository.py:132-137, 1470-1472 -> adapters.py:205-213: hashlib.blake2b(digest,
 * salt=shared_kdf_params, key=shared_key, digest_size=cipher key bytes)).  For cut slot s the
 * DEVICE state d_kdf_state -- rc_blake2b_state_init(key_bytes, shared_key, salt=shared_kdf_params);
 * only read -- absorbs the first msg_len bytes of d_digests + 64 s, and its digest goes to
 * d_keys + 64 s, where rc_gcm_encrypt_chunks (replicat_cipher.h) takes it.  Counts are read on the
 * device.  Enqueued on hip_stream. */
int rc_blake2b_derive_chunks(rc_hasher *h, const rc_chunker *layout, uint64_t n,
                             const uint64_t *lens, const int64_t *d_counts,
                             const rc_blake2b_state *d_kdf_state, const uint8_t *d_digests,
                             uint32_t msg_len, uint8_t *d_keys, void *hip_stream);

/* Kernel timing for bench.py: while enabled, each rc_blake2b_* enqueue records HIP events around
 * its kernels on the launch stream; read returns the summed milliseconds and clears. */
int rc_blake2b_timing_enable(rc_hasher *h, int enable);
int rc_blake2b_timing_read(rc_hasher *h, double *ms, uint64_t *calls);

#ifdef __cplusplus
}
#endif

#endif /* REPLICAT_DIGEST_H */
