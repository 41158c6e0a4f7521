// cipher_kernels.h -- internal interface between gcm.hip (kernels) and capi_cipher.cpp.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

// One message: device addresses of its input, output, key (key_bytes) and nonce (nonce_bytes),
// its plaintext (= ciphertext) length, and the slot of its decrypt verdict.
//   encrypt: reads len bytes at in and the nonce; writes nonce || C || T at out
//            (nonce_bytes + len + 16 bytes), as AEADCipherAdapterMixin.encrypt returns them
//   decrypt: reads nonce || C || T at in (nonce field unused); writes len bytes of plaintext at
//            out and ok[slot] = 1 if the tag verifies, else 0
struct GcmItem {
    uint64_t in, len, out, key, nonce, slot;
};

struct GcmArgs {
    const GcmItem *items;
    const uint64_t *d_total;   // item count on the device (chunk path; the grid covers its bound)
    const uint32_t *te0;       // AES T0 table (256 words)
    const uint32_t *sq;        // GF(2^128) squaring nibble table (512 x 16 bytes)
    uint8_t *ok;               // decrypt verdicts
    uint32_t nonce_bytes;
};

constexpr int kGcmThreads = 1024;  // 16 waves: one workgroup per CU (153 KiB of LDS)

const char *rc_gcm_launch_error(void);

// AES-GCM over a work list (key_bytes 16 / 24 / 32): workgroup i takes item i; groups = the item
// count (or, with d_total, its bound).
int rc_gcm_launch(uint32_t key_bytes, bool decrypt, const GcmArgs &args, unsigned groups,
                  hipStream_t stream);

// Chunk lists as rc_chunk_device left them, with the per-stream output regions.
struct GcmChunkLists {
    const uint64_t *ptrs, *cut_base, *out_base, *cuts, *chunk_off;
    const int64_t *counts;
    uint64_t n, spw;             // streams, streams per workgroup
    uint64_t keys, nonces, out;  // device addresses: 64-byte key slots, nonce_bytes per cut slot
    uint32_t nonce_bytes;
};

// Work list of the chunks: item chunk_off[i] + k = chunk k of stream i.
int rc_gcm_launch_chunk_items(const GcmChunkLists &c, GcmItem *items, hipStream_t stream);
