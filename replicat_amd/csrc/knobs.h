// knobs.h -- every environment setting the library reads, in one table.
//
// Nothing else in the library calls getenv.  A handle reads the table ONCE, when it is created
// (rc_chunker_create, rc_blake2b_create, rc_gcm_create; the free functions rc_read_probe once per
// process), and keeps the values for its lifetime: a setting can no longer change a schedule
// from one call to the next.  A value that is not a legal word or an integer inside the knob's
// range fails the creation with RC_ERR_ARGUMENT naming the variable -- a typo is an error, not a
// silent default.  Every knob is a measurement or test switch: the defaults are the measured
// schedule (DESIGN.md cites the runs), and a service sets none of them.
#pragma once
#include <stdint.h>

#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cstring>

namespace rc {

enum Knob : int {
    knPipeAll,        // RC_PIPE_ALL
    knOverlapCus,     // RC_OVERLAP_CUS
    knLaneChain,      // RC_LANE_CHAIN
    knTileGroups,     // RC_TILE_GROUPS
    knChainLean,      // RC_CHAIN_LEAN
    knSegmentBytes,   // RC_SEGMENT_BYTES
    knSegmentExt,     // RC_SEGMENT_EXT
    knSegmentFloor,   // RC_SEGMENT_FLOOR
    knTileStatic,     // RC_TILE_STATIC
    knTileChunk,      // RC_TILE_CHUNK
    knTileDynMin,     // RC_TILE_DYN_MIN
    knJoinWalk,       // RC_JOIN_WALK
    knRepair,         // RC_REPAIR
    knB2LaneMax,      // RC_B2_LANE_MAX
    knB2LaneOnly,     // RC_B2_LANE_ONLY
    knProbeBlock,     // RC_PROBE_BLOCK
    knGcmDebug,       // RC_GCM_DEBUG
    knTileStreams,    // RC_TILE_STREAMS
    knTileGroup,      // RC_TILE_GROUP
    knTileMask,       // RC_TILE_MASK
    kKnobCount
};

// words: "w0|w1|..." -- the knob takes exactly those words, as values 0, 1, ...; nullptr: an
// integer in [lo, hi] (decimal or 0x-hex).
struct KnobSpec {
    const char *name;
    int64_t def, lo, hi;
    const char *words;
    const char *doc;
};

// clang-format off
inline constexpr KnobSpec kKnobTable[kKnobCount] = {
    {"RC_PIPE_ALL", 0, 0, 1, "0|1",
     "1: every RC_PIPELINED request overlaps (otherwise small-window chunkers and requests "
     "under a tile per tile-kernel wave run in sequence, capi.cpp rc_chunk_device)"},
    {"RC_OVERLAP_CUS", 32, 1, 1024, nullptr,
     "CUs reserved for the chain kernels of pipelined calls (rc_chunker_overlap overrides; "
     "must be below the device's CU count)"},
    {"RC_LANE_CHAIN", 0, 0, 3, "auto|0|1|lane",
     "chain kernel of small-window batches: auto (quads for >= 256 streams), 0 wave per "
     "stream, 1 quads whatever the count, lane one lane per stream"},
    {"RC_TILE_GROUPS", 0, 0, 2, "auto|0|1",
     "per-quarter group records of the tile kernel: auto (small windows), 0 never, 1 always"},
    {"RC_CHAIN_LEAN", 0, 0, 1, "auto|0",
     "32-bit chain steps for small windows: auto, 0 never (comparison)"},
    {"RC_SEGMENT_BYTES", 0, 0, int64_t(1) << 50, nullptr,
     "chain segment length in bytes (0: sized per call for ~4096 walkers)"},
    {"RC_SEGMENT_EXT", 2, 0, 64, nullptr,
     "steps a speculative chain runs past its segment end"},
    {"RC_SEGMENT_FLOOR", 2, 1, 64, nullptr,
     "shortest automatic segment, in max_lengths"},
    {"RC_TILE_STATIC", 0, 0, 1000, nullptr,
     "share of the tiles handed out statically, per mille (1000: fully static)"},
    {"RC_TILE_CHUNK", 3, 2, 4096, nullptr,
     "tiles per dynamic unit of the tile kernel"},
    {"RC_TILE_DYN_MIN", 0, 0, int64_t(1) << 20, nullptr,
     "tiles per wave from which a launch hands out dynamic units"},
    {"RC_JOIN_WALK", 0, 0, 1, "0|1",
     "1: every multi-segment stream through the sequential join (comparison)"},
    {"RC_REPAIR", 1, 0, 1, "0|1",
     "0: no boundary repair in the merge kernel (a miss walks the stream)"},
    {"RC_B2_LANE_MAX", -1, -1, int64_t(1) << 62, nullptr,
     "BLAKE2b: longest message hashed by one lane (-1: the throughput rule, 0: quads only)"},
    {"RC_B2_LANE_ONLY", 0, 0, 2, "auto|0|1",
     "BLAKE2b: 0 never uses the lane-only kernel (the fused kernel's lane role instead); "
     "auto and 1 use it when every message fits a lane"},
    {"RC_PROBE_BLOCK", 0, 0, int64_t(1) << 20, nullptr,
     "read probe: interleaved static runs of this many tiles (0: the tile kernel's schedule)"},
    {"RC_GCM_DEBUG", 0, 0, 1, "0|1",
     "1: stamp every host step of an AES-GCM call on stderr"},
    {"RC_TILE_STREAMS", 1, 1, 2, nullptr,
     "CU-masked tile streams of pipelined calls: 2 alternates them, so a call's tile kernel "
     "may start on CUs the previous one has left"},
    {"RC_TILE_GROUP", 64, 0, 256, nullptr,
     "dynamic units per workgroup grab of the tile kernel (a power of two: the workgroup's "
     "waves take that many units from one global grab through LDS; below 16 runs as 16, the "
     "LDS ring's margin); 0: one grab per unit"},
    {"RC_TILE_MASK", 0, 0, 2, "masked|full|plain",
     "tile stream of pipelined calls: masked (the CUs the chain stream does not reserve), full "
     "(its own queue with every CU in its mask) or plain (a non-blocking stream on the shared "
     "queues); with full / plain the tile kernel's workgroups take every CU the chain kernels "
     "leave (measurement switch)"},
};
// clang-format on

struct Knobs {
    int64_t v[kKnobCount];
    int64_t operator[](Knob k) const { return v[k]; }
};

// Parses one setting; false when it is not a legal value.
inline bool parse_knob(const KnobSpec &s, const char *text, int64_t &out) {
    if (s.words) {
        int64_t idx = 0;
        for (const char *w = s.words; *w; ++idx) {
            const char *bar = std::strchr(w, '|');
            const size_t n = bar ? size_t(bar - w) : std::strlen(w);
            if (std::strlen(text) == n && std::strncmp(text, w, n) == 0) {
                out = idx;
                return true;
            }
            w += n + (bar ? 1 : 0);
        }
        return false;
    }
    if (!*text) return false;
    char *end = nullptr;
    errno = 0;
    const long long x = std::strtoll(text, &end, 0);
    if (errno || *end || x < s.lo || x > s.hi) return false;
    out = x;
    return true;
}

// Reads the whole table from the environment.  Returns 0, or the failing knob's index + 1 with
// a message in err.
inline int read_knobs(Knobs &k, char *err, size_t err_len) {
    for (int i = 0; i < kKnobCount; ++i) {
        const KnobSpec &s = kKnobTable[i];
        k.v[i] = s.def;
        const char *e = std::getenv(s.name);
        if (!e) continue;
        if (!parse_knob(s, e, k.v[i])) {
            if (s.words)
                std::snprintf(err, err_len, "%s=%s: not one of %s", s.name, e, s.words);
            else
                std::snprintf(err, err_len, "%s=%s: not an integer in [%lld, %lld]", s.name, e,
                              (long long)s.lo, (long long)s.hi);
            return i + 1;
        }
    }
    return 0;
}

// The process-wide table, read on first use (free functions without a handle: the read probe,
// the AES-GCM debug stamps).  A bad value there falls back to the defaults.
inline const Knobs &process_knobs() {
    static const Knobs k = [] {
        Knobs r;
        char err[160];
        if (read_knobs(r, err, sizeof err))
            for (int i = 0; i < kKnobCount; ++i) r.v[i] = kKnobTable[i].def;
        return r;
    }();
    return k;
}

}  // namespace rc
