// digest_kernels.h -- internal interface between blake2b.hip (kernels) and capi_digest.cpp.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "../../include/replicat_digest.h"

// One message to hash: device address, length in bytes, output slot (digest at out + 64 * slot).
struct B2Item {
    uint64_t ptr, len, slot;
};

// One (state, buffer) pair of an incremental / keyed update: state is a device rc_blake2b_state.
struct B2UItem {
    uint64_t ptr, len, slot, state;
    uint32_t final, pad;
};

constexpr int kB2Threads = 256;       // 4 waves, 64 quads per workgroup
constexpr uint64_t kB2MaxGroups = 512;  // 2 waves per SIMD on 256 CUs; items beyond loop
constexpr uint64_t kB2OneWaveGroups = 256;   // one wave per SIMD
constexpr uint64_t kB2TwoWaveItems = 65536;  // from this many items on, two waves per SIMD
constexpr uint64_t kB2LaneGroups = 1024;     // lane-only launches: four waves per SIMD
constexpr int kB2Buckets = 256;       // length classes of the longest-first work list
constexpr uint64_t kB2Slot = 64;      // bytes per digest slot (BLAKE2b's largest digest)

const char *rc_b2_launch_error(void);

// Digests of n items (host-built work list, already on the device).
// lane_max: items of at most this many bytes are hashed one per lane, longer ones by quads
// (rc_b2_lane_max); 0: every item by quads.  lane_only: every item by lanes, in the lane
// kernel (four waves per SIMD) -- for batches whose items are all at most lane_max bytes.
int rc_b2_launch_items(const B2Item *d_items, uint64_t n, uint32_t outlen, uint8_t *d_out,
                       uint64_t lane_max, bool lane_only, hipStream_t stream);

// Incremental updates of n (state, buffer) items; finals write the digest at d_out + 64 * slot.
int rc_b2_launch_update(const B2UItem *d_items, uint64_t n, uint8_t *d_out, hipStream_t stream);

// Streams per workgroup of the work-list passes, and the size (u32 words) of their histogram.
inline uint64_t rc_b2_streams_per_group(uint64_t n) { return n ? (n + 1023) / 1024 : 1; }
inline uint64_t rc_b2_hist_words(uint64_t n) {
    const uint64_t spw = rc_b2_streams_per_group(n);
    return uint64_t(kB2Buckets) * ((n + spw - 1) / spw + 1);
}

// Digests of the chunks of n streams as rc_chunk_device wrote them: d_cuts at d_cut_base[i],
// d_counts[i] chunks.  d_chunk_off has n + 1 entries, d_hist rc_b2_hist_words(n); d_items holds
// items_cap (>= sum of counts) entries.  The work list is sorted longest first on the device.
int rc_b2_launch_chunks(uint64_t n, const uint64_t *d_ptrs, const uint64_t *d_cut_base,
                        const uint64_t *d_cuts, const int64_t *d_counts, uint64_t *d_chunk_off,
                        uint32_t *d_hist, B2Item *d_items, uint64_t items_cap, uint32_t outlen,
                        uint8_t *d_out, uint64_t lane_max, bool lane_only, hipStream_t stream);

// The lane/quad split for a batch of `bytes` message bytes whose longest message is at most
// `longest` bytes.  Lanes pay off only when the batch is throughput-bound: its ALU time
// (~bytes / 1.7 TB/s) well above the longest quad chain (~longest / 128 x 1.4 us), i.e.
// bytes >= longest << 16; otherwise every item goes to quads (config 2: its 5 MB chunks' chains
// set the time, and lanes sharing their SIMDs only lengthen them).  Within a throughput-bound
// batch a message goes to a lane when its chain (~3x a quad's) ends well inside the batch time:
// len <= bytes >> 17.  knob_max (RC_B2_LANE_MAX, knobs.h: -1 = the rule) overrides the whole
// rule, 0 turning lanes off.
inline uint64_t rc_b2_lane_max(uint64_t bytes, uint64_t longest, int64_t knob_max) {
    if (knob_max >= 0) return (uint64_t)knob_max;
    return longest > (bytes >> 16) ? 0 : bytes >> 17;
}
// Whether a batch whose messages are at most `longest` bytes goes to the lane kernel alone
// (never_only, RC_B2_LANE_ONLY=0: the fused kernel's lane role instead, for A/B runs).
inline bool rc_b2_lane_only(uint64_t lane_max, uint64_t longest, bool never_only) {
    if (never_only) return false;
    return lane_max != 0 && longest <= lane_max;
}

// Exclusive prefix of the per-stream chunk counts into d_chunk_off[0..n] (the total at [n]).
int rc_b2_launch_scan(const int64_t *d_counts, uint64_t n, uint64_t *d_chunk_off, hipStream_t stream);

// derive_shared_subkey of every cut slot (rc_b2_derive_kernel): the read-only KDF state absorbs
// msg_len bytes of digest slot s and finalises into d_keys + 64 s.  d_cut_base has n entries.
int rc_b2_launch_derive(uint64_t n, const uint64_t *d_cut_base, const int64_t *d_counts,
                        const rc_blake2b_state *d_kdf, const uint8_t *d_digests, uint32_t msg_len,
                        uint8_t *d_keys, hipStream_t stream);
