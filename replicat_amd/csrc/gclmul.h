// gclmul.h -- layouts shared by the gfx950 kernels (kernels.hip) and the host side (capi.cpp).
//
// Key algebra (replaces the PCLMULQDQ pair of /root/reference/src/adapters.cpp:72-77).
// gfx950 has no carry-less multiply, but for a fixed key the chunker hash is GF(2)-affine
// in the 8 data bytes:  key(d) = k1 ^ M d,  M a 64x64 bit matrix fixed by k0.  Key j of a
// stream covers bytes [4j-4, 4j+4) = LE32 words w[j-1] (low half) and w[j] (high half), so
//     key(j) = k1 ^ Lmap(w[j-1]) ^ Hmap(w[j])
// with Lmap/Hmap the two 32-column halves of M.  Each is evaluated one byte at a time from
// 256-entry tables:   TL[b][v] = Lmap(v << 8b),  TH[b][v] = Hmap(v << 8b)  (k1 folded into TH[0]).
// The streaming kernel needs only the TOP 16 bits of every key to find each lane's candidate
// (the exact 64-bit key is evaluated once per lane and tile), so it uses 32-bit
// "prefilter" entries  PF[b][v] = top16(TL[b][v]) << 16 | top16(TH[b][v]).
#pragma once
#include <stdint.h>

namespace rc {

#ifndef RC_TILE_ITERS
#define RC_TILE_ITERS 16
#endif
constexpr int kTileIters = RC_TILE_ITERS;  // 16-byte loads per lane per tile (16 KiB in flight per wave)
constexpr int kTileKeys = 64 * 4 * kTileIters;  // keys per tile = one wave: 64 lanes x 4 keys
constexpr int kWaveSize = 64;
constexpr int kTileWaves = 16;       // waves per workgroup of the tile kernel (1024 threads)
constexpr int kChainWaves = 4;       // waves (= streams) per workgroup of the chain kernel
#ifndef RC_TILE_GROUPS
#define RC_TILE_GROUPS 4
#endif
constexpr int kTileGroups = RC_TILE_GROUPS;  // key groups per tile with group maxima (<= 4: one u64)
constexpr int kGroupKeys = kTileKeys / kTileGroups;

// ---- LDS image of the tile kernel -------------------------------------------------------
// Prefilter tables replicated 32x so that the 32 lanes of each ds_read_b32 lane group each own
// one bank (bank = dword address mod 32 = lane mod 32): conflict-free random lookups.
//   byte address of PF[b][v] for lane l:  (b>>1)*65536 + v*256 + (b&1)*128 + (l&31)*4
constexpr uint32_t kPfBytes = 131072;
constexpr uint32_t kFullOff = kPfBytes;                 // TL[4][256], then TH[4][256] (u64)
constexpr uint32_t kFullBytes = 2 * 4 * 256 * 8;        // 16 KiB
constexpr uint32_t kTileLdsBytes = kPfBytes + kFullBytes;

// Key tables of one chunker, built on the host, uploaded once, staged into LDS per workgroup.
struct KeyTables {
    uint64_t tl[4][256];
    uint64_t th[4][256];   // k1 folded into th[0][*]
    uint32_t pf[4][256];
};

// Per-call stream descriptors (structure of arrays in one device buffer).
struct StreamDesc {
    const uint8_t *const *ptr;  // device pointers
    const uint64_t *len;        // L
    const uint64_t *last;       // P
    const uint64_t *jneed;      // last key any window can reach (0 = none)
    const uint64_t *tile_base;  // n+1 entries, exclusive prefix sum of tiles per stream
    const uint64_t *cut_base;   // n entries
    const uint64_t *cut_cap;    // n entries
    const uint64_t *seg_base;   // n+1 entries, exclusive prefix sum of chain segments per stream
    const uint64_t *scratch_base;  // n entries: offset of the stream's speculative lists
    const uint64_t *xtiles;        // count, then the tiles that are not fast (tile_fast), global
};

// One record per tile: first maximal key of the tile and its key index in the stream.
struct TileRecord {
    uint64_t key;
    uint64_t j;
};

// Per-tile group bounds of the small-window tile kernel (kTileGroups groups of kGroupKeys keys;
// group g = the tile kernel's iterations g*kTileIters/G .., in which lane l holds keys
// 256*it + 4l .. 256*it + 4l + 3):
//   max:     u16 g = the top-16 maximum of group g (keys that do not exist count as 0);
//   hot[g]:  bit l = lane l's own top-16 maximum in group g is >= the chunker's hot threshold
//            (group_hot_threshold: low enough that a window's best almost always reaches it,
//            high enough that a group rarely has more than one such lane).
// So when the best so far reaches the threshold, only the lanes in hot[g] can hold a key of the
// group that reaches it.  A tile computed exactly (rc_edge_kernel) has max = ~0 and every lane
// hot: no bound at all.
struct GroupRecord {
    uint64_t max;
    uint64_t hot[kTileGroups];
    uint64_t pad;  // 48 bytes: three 16-byte stores / loads
};
static_assert(kTileGroups % 2 == 0 && sizeof(GroupRecord) % 16 == 0, "group record layout");

// Hot threshold of a chunker whose argmax window holds `window` keys: 10 / window of the
// 16-bit range below the top.  The best of the window's full tiles (>= 0.6 window keys) falls
// below it with probability ~e^-6 or less, and a group of kGroupKeys keys has ~10 kGroupKeys /
// window hot lanes besides its maximum's (0.5 for config 3 iii's 20,000-key windows).  0 for
// windows of under a tile (nothing is excluded: the chain scans).
__host__ __device__ inline uint32_t group_hot_threshold(uint64_t window) {
    if (window < (uint64_t)kTileKeys) return 0;
    const uint64_t below = (10 * 65536 + window - 1) / window;
    return below >= 65536 ? 0u : (uint32_t)(65536 - below);
}

struct ChainParams {
    uint64_t min_length;
    uint64_t max_length;
    uint64_t window;      // T = (max_length - 1) / 4 keys per argmax window (0 if max < 5)
    uint64_t max_steps;   // stop after this many cuts per stream (~0 = unbounded; 0 = one raw
                          // argmax whatever its value: the single-buffer next_cut)
    uint64_t seg_bytes;   // chain segment length (multiple of 4)
    uint64_t seg_cap;     // entries per speculative list
    uint64_t ext_steps;   // steps a speculative chain runs past its segment end
    const GroupRecord *grp;  // per-tile group bounds (rc_launch_tiles), or NULL
    uint64_t n_tiles;     // tiles of the call (records and group bounds hold n_tiles + 1)
    uint32_t open;        // RC_OPEN: non-final prefix, no tail rule
    uint32_t lean;        // small windows and every stream < 16 GiB: 32-bit chain steps
    uint32_t lane;        // lane-per-stream chain allowed (rc_lane_chain_kernel; 2 = forced)
    uint32_t hot;         // the group records' hot threshold (group_hot_threshold)
    // the call's fault stamp (the workspace counter buffer's kCtrStampWord, written by the
    // edge kernel) and this call's epoch: equal = the tile kernel took its fail-safe stop, the
    // records are incomplete, and the chain kernels write RC_COUNT_FAULT instead of cuts
    const uint64_t *fault;
    uint64_t epoch;
};

// The tile kernel's counter buffer (256 bytes per workspace, capi.cpp ensure_ctr), in u32 words:
//   0            the dynamic units' grab counter (the edge kernel re-zeroes it for the next launch)
//   kCtrErrWord  the fail-safe flag: set by a tile-kernel wave that stopped (UnitGrab::next);
//                the edge kernel moves it into the stamp below and clears it
//   kCtrStampWord (u64) the epoch of the last call whose tile kernel set the flag
//   kCtrFaultsWord how many calls set it since the last rc_chunker_check
constexpr uint32_t kCtrErrWord = 32, kCtrStampWord = 34, kCtrFaultsWord = 36;
// Count written for every stream of a faulted call (include/replicat_chunker.h RC_COUNT_FAULT;
// -1 is a capacity overflow, -2 the chain kernels' internal kNeedJoin)
constexpr int64_t kCountFault = -3;

// The tile kernel's work schedule (kernels.hip tile_units; knobs.h RC_TILE_STATIC / CHUNK /
// DYN_MIN): the share of the tiles handed out statically (per mille), the dynamic unit size and
// the tiles per wave from which a launch hands out dynamic units at all.
// Defaults since round 5: every tile in 3-tile units, 64 units per workgroup grab (knobs.h).
struct TileSched {
    uint32_t permille = 0;
    uint32_t chunk = 3;
    uint32_t dyn_min = 0;
    uint32_t group = 64;  // units per workgroup grab (kernels.hip UnitGrab); 0: per-wave grabs
};

// splitmix64 finaliser (replicat_amd/synth.py)
__host__ __device__ inline uint64_t splitmix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

}  // namespace rc

// Launchers implemented in kernels.hip (host-callable, enqueue only).
extern "C" {
// d_records: n_tiles + 1 entries (the last is scratch for the tile kernel's pipeline)
// d_grp (may be NULL): n_tiles + 1 group records (per-group top-16 bounds, GroupRecord) --
// the chain's bounds for small windows.  mid_event (a hipEvent_t, may be NULL):
// recorded between the tile and the edge kernel.
// d_xlist: rc_tie_list_words(n_tiles) u32 of scratch: the tile kernel's tie lists (n_tiles
// slots) and one count per work unit.  d_ctr: the counter buffer (kCtrErrWord above): the grab
// counter is 0 at the call and the edge kernel zeros it again for the next launch; `epoch`
// (this call's, never 0) is what the edge kernel stamps when the tile kernel took its fail-safe
// stop, and the edge kernel then recomputes nothing (the tie lists may be stale).
// cus: the CUs the tile kernel's stream may use (its persistent grid; 0 = every CU of the
// device).  edge_stream (may be NULL = stream): where the edge kernel runs; when it differs,
// `tiled` (a hipEvent_t) is recorded after the tile kernel and edge_stream waits for it.
// sched: the chunker's schedule knobs.
int rc_launch_tiles(const rc::KeyTables *d_tables, rc::StreamDesc desc, uint64_t n_streams,
                    uint64_t n_tiles, rc::TileRecord *d_records, rc::GroupRecord *d_grp,
                    uint32_t hot, uint32_t *d_xlist, uint32_t *d_ctr, uint64_t epoch,
                    void *stream, void *mid_event, uint32_t cus, void *edge_stream, void *tiled,
                    rc::TileSched sched);
uint64_t rc_tie_list_words(uint64_t n_tiles);
// (exported for tests: include/replicat_chunker.h rc_tile_schedule)
// join: RC_JOIN_* bits -- how multi-segment streams are spliced
enum : uint32_t { RC_JOIN_WALK_ONLY = 1, RC_JOIN_REPAIR = 2 };
int rc_launch_chain(const rc::KeyTables *d_tables, rc::StreamDesc desc, uint64_t n_streams,
                    rc::ChainParams prm, uint64_t n_segs, const rc::TileRecord *d_records,
                    uint64_t *d_cuts, int64_t *d_counts, uint64_t *d_scratch,
                    uint64_t *d_seg_counts, bool any_multi, uint32_t join, void *stream);
int rc_launch_fill(uint8_t *d_dst, uint64_t nbytes, uint64_t seed, uint64_t stream_id,
                   uint64_t word0, void *stream);
int rc_launch_fill_streams(uint8_t *d_dst, uint64_t n, uint64_t nbytes, uint64_t slot,
                           uint64_t seed, uint64_t id0, uint64_t id_step, void *stream);
// block: 0 = the tile kernel's schedule `sched`, else interleaved static runs of `block` tiles
int rc_launch_read_probe(const uint8_t *d_src, uint64_t nbytes, uint32_t *d_out, uint32_t block,
                         rc::TileSched sched, void *stream);
const char *rc_launch_error(void);
}
