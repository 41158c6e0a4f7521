// capi_internal.h -- what capi.cpp (chunker) and capi_digest.cpp (BLAKE2b) share.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/replicat_digest.h"

// Sets the calling thread's rc_last_error() message and returns `code`.
int rc_fail(int code, const char *fmt, ...);

// Live handles (chunkers, hashers, ciphers): every *_create registers its handle with the
// destroy function that releases it, every *_destroy unregisters it.  The first registration
// installs an atexit hook that destroys whatever is still registered when the process exits --
// after the caller's own teardown (Python's finalisation included) and BEFORE the HIP runtime's
// static destructors, which ran later than a leaked CU-masked stream's teardown can (round 3:
// a process that exited with a pipelined chunker alive died in __cxa_finalize).
void rc_track(void *handle, void (*destroy)(void *));
void rc_untrack(void *handle);

#define RC_HIP_TRY(expr)                                                                 \
    do {                                                                                 \
        const hipError_t e_ = (expr);                                                    \
        if (e_ != hipSuccess)                                                            \
            return rc_fail(RC_ERR_HIP, "%s failed: %s", #expr, hipGetErrorString(e_));   \
    } while (0)

// Enqueue on `st` the digests of the chunks of n device streams (d_ptrs: HOST array of device
// pointers) whose cut lists sit at d_cuts[cut_base[i] ..] with d_counts[i] entries, into
// d_out + 64 * (cut_base[i] + k).  total_cap = sum of the cut capacities (>= the chunk count);
// bytes = the streams' total length, longest = a bound on one chunk's length (they set the
// lane / quad split, rc_b2_lane_max).
int rc_hasher_enqueue_chunks(rc_hasher *h, uint64_t n, const uint8_t *const *d_ptrs,
                             const uint64_t *cut_base, const uint64_t *d_cuts,
                             const int64_t *d_counts, uint64_t total_cap, uint64_t bytes,
                             uint64_t longest, uint8_t *d_out, hipStream_t st);
