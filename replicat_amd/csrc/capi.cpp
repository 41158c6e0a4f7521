// capi.cpp -- host side of the C ABI in include/replicat_chunker.h.
//
// Owns the per-key lookup tables (built here from k0/k1, see gclmul.h), per-call stream
// descriptors, the tile-record workspace, and the blocking single-buffer `next_cut`
// (the drop-in for /root/reference/src/adapters.cpp:42-70).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <vector>

#include "../../include/replicat_chunker.h"
#include "capi_internal.h"
#include "gclmul.h"
#include "knobs.h"

using namespace rc;

static_assert(kCountFault == RC_COUNT_FAULT && kCtrFaultsWord * 4 < 256, "counter buffer layout");

constexpr uint64_t kDigestSlot = RC_DIGEST_SLOT;

namespace {

thread_local char g_err[512];

int vfail(int code, const char *fmt, va_list ap) {
    vsnprintf(g_err, sizeof g_err, fmt, ap);
    return code;
}

int fail(int code, const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vfail(code, fmt, ap);
    va_end(ap);
    return code;
}

#define HIP_TRY(expr)                                                                  \
    do {                                                                               \
        const hipError_t e_ = (expr);                                                  \
        if (e_ != hipSuccess)                                                          \
            return fail(RC_ERR_HIP, "%s failed: %s", #expr, hipGetErrorString(e_));    \
    } while (0)

// Carry-less 64x64 -> 128 product.
void clmul64(uint64_t a, uint64_t b, uint64_t &lo, uint64_t &hi) {
    lo = hi = 0;
    for (int i = 0; i < 64; ++i)
        if ((b >> i) & 1) {
            lo ^= a << i;
            if (i) hi ^= a >> (64 - i);
        }
}

// The linear part of the key map (adapters.cpp:72-77 without the k1 term).
uint64_t key_linear(uint64_t k0, uint64_t d) {
    uint64_t lo, hi, rlo, rhi;
    clmul64(k0, d, lo, hi);
    clmul64(0x1B, hi, rlo, rhi);  // single partial fold; the overflow bits rhi are dropped
    return lo ^ rlo;
}

void build_tables(uint64_t k0, uint64_t k1, KeyTables &t) {
    uint64_t col[64];
    for (int c = 0; c < 64; ++c) col[c] = key_linear(k0, 1ull << c);
    for (int b = 0; b < 4; ++b)
        for (int v = 0; v < 256; ++v) {
            uint64_t l = 0, h = 0;
            for (int i = 0; i < 8; ++i)
                if ((v >> i) & 1) {
                    l ^= col[8 * b + i];
                    h ^= col[32 + 8 * b + i];
                }
            if (b == 0) h ^= k1;
            t.tl[b][v] = l;
            t.th[b][v] = h;
            t.pf[b][v] = (uint32_t)((l >> 48) << 16) | (uint32_t)(h >> 48);
        }
}

uint64_t load_le64(const uint8_t *p) {
    uint64_t v = 0;
    for (int i = 7; i >= 0; --i) v = (v << 8) | p[i];
    return v;
}

uint64_t window_keys(uint64_t max_length) { return max_length >= 1 ? (max_length - 1) / 4 : 0; }

struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != dev) (void)hipSetDevice(dev);
    }
    ~DeviceGuard() {
        int cur = -1;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
    }
};

// growable device buffer
struct DevBuf {
    void *p = nullptr;
    size_t n = 0;
    int ensure(size_t bytes) {
        if (bytes <= n) return 0;
        if (p) {
            HIP_TRY(hipDeviceSynchronize());
            HIP_TRY(hipFree(p));
            p = nullptr;
            n = 0;
        }
        size_t want = std::max<size_t>(bytes, 4096);
        want = (want + 4095) & ~(size_t)4095;
        HIP_TRY(hipMalloc(&p, want));
        n = want;
        return 0;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
    }
};

struct HostBuf {  // growable pinned host buffer
    void *p = nullptr;
    size_t n = 0;
    int ensure(size_t bytes) {
        if (bytes <= n) return 0;
        if (p) HIP_TRY(hipHostFree(p));
        p = nullptr;
        n = 0;
        size_t want = std::max<size_t>(bytes, 4096);
        HIP_TRY(hipHostMalloc(&p, want, hipHostMallocDefault));
        n = want;
        return 0;
    }
    void release() {
        if (p) (void)hipHostFree(p);
        p = nullptr;
        n = 0;
    }
};

}  // namespace

int rc_fail(int code, const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vfail(code, fmt, ap);
    va_end(ap);
    return code;
}

namespace {

// The live-handle registry (capi_internal.h).  Heap-allocated and never freed: a static
// container would have a destructor of its own in the exit sequence.
struct LiveHandle {
    void *h;
    void (*destroy)(void *);
};
std::mutex g_live_mu;
std::vector<LiveHandle> *g_live = nullptr;
bool g_exiting = false;

void destroy_live_at_exit() {
    std::vector<LiveHandle> left;
    {
        std::lock_guard<std::mutex> lock(g_live_mu);
        g_exiting = true;
        if (g_live) left.swap(*g_live);
    }
    for (auto it = left.rbegin(); it != left.rend(); ++it) it->destroy(it->h);
}

}  // namespace

void rc_track(void *handle, void (*destroy)(void *)) {
    std::lock_guard<std::mutex> lock(g_live_mu);
    if (!g_live) {
        g_live = new std::vector<LiveHandle>();
        // registered after the HIP runtime initialised (the caller created a device object
        // first), so it runs before the runtime's own exit-time teardown
        std::atexit(destroy_live_at_exit);
    }
    g_live->push_back({handle, destroy});
}

void rc_untrack(void *handle) {
    std::lock_guard<std::mutex> lock(g_live_mu);
    if (!g_live || g_exiting) return;
    for (size_t i = 0; i < g_live->size(); ++i)
        if ((*g_live)[i].h == handle) {
            (*g_live)[i] = g_live->back();
            g_live->pop_back();
            return;
        }
}

struct rc_chunker {
    uint64_t min_length = 0, max_length = 0, window = 0;
    bool small = false;   // window + 2 edge tiles within 64 tiles (the chain's one-row cache)
    bool groups = false;  // small windows: the tile kernel also writes per-group maxima
    uint64_t seg_force = 0, ext_steps = 2;  // segment-parallel chains (see stage_descriptors)
    uint64_t seg_floor = 2;                 // shortest segment, in max_lengths
    uint64_t k0 = 0, k1 = 0;
    int device = 0;
    Knobs knobs;      // knobs.h, read once at creation
    TileSched sched;  // the tile kernel's schedule (from knobs)
    KeyTables tables;
    KeyTables *d_tables = nullptr;
    std::mutex mu;  // one call at a time per chunker (the reference is used by one thread)

    // per-call workspaces, used alternately so that two calls can be in flight
    struct Workspace {
        HostBuf h_desc;     // pinned staging of the descriptor arrays
        DevBuf d_desc;      // device copy
        DevBuf d_records;   // one TileRecord per tile
        DevBuf d_scratch;   // speculative chain lists of multi-segment streams
        DevBuf d_seg_counts;  // one count (+ termination bit) per chain segment
        DevBuf d_ctr;         // the tile kernel's counter buffer (gclmul.h kCtrErrWord): grab
                              // counter, fail-safe flag, fault stamp and count
        bool ctr_dirty = false;  // a launch failed between the tile and the edge kernel: re-zero it
        uint64_t epoch = 0;      // this workspace's last launch (the edge kernel's fault stamp)
        std::vector<uint64_t> xtiles;  // host list of the tiles the fast path does not take
        hipEvent_t done = nullptr;  // the call that last used this workspace has finished
        bool pending = false;
        bool piped = false;  // that call's chain ran on a pipelined stream, not the caller's
    } ws[2];
    unsigned next_ws = 0;

    // single-buffer next_cut scratch
    DevBuf d_buf, d_out;
    HostBuf h_out;

    // host-stream path scratch
    DevBuf d_stage[2], d_hcuts[2], d_hcounts[2], d_hdig[2];
    hipStream_t hstream[2] = {nullptr, nullptr};

    // descriptor uploads run on their own stream, so that a call's upload overlaps the
    // previous call's kernels (the workspace alternation keeps the two apart)
    hipStream_t cstream = nullptr;
    hipEvent_t uploaded[2] = {nullptr, nullptr};

    // RC_PIPELINED calls (overlap mode): the tile kernel on `tstream`, whose CU mask leaves out
    // `reserve` CUs, the edge and chain kernels on `xstream`, masked to exactly those CUs, so
    // that one call's chain runs beside the next call's tile kernel
    uint32_t reserve_req = 0;  // rc_chunker_overlap (0: RC_OVERLAP_CUS, default 32)
    uint32_t reserve = 0, tile_cus = 0;  // of the streams below (0: not created)
    hipStream_t tstream = nullptr, xstream = nullptr;
    hipStream_t tstream2 = nullptr;  // RC_TILE_STREAMS=2: the odd workspace's tile kernels
    hipStream_t fstream = nullptr;  // RC_PIPELINE_END calls' edge and chain kernels: every CU
    hipEvent_t in_ev[2] = {nullptr, nullptr}, tiled[2] = {nullptr, nullptr};
    uint64_t pipelined_calls = 0;  // RC_PIPELINED requests that ran on the two streams
    bool overlap_failed = false;   // the masked streams could not be created (calls run in sequence)

    // timing: events before the tile kernel, after it, after the edge kernel, after the chain
    bool timing = false;
    // rc_timing_enable's per-call events: ev[0], ev[2], ev[3] only time (no system-scope fence,
    // hipEventDisableSystemFence); ev[1] also hands the tile kernel's records to the chain
    // stream in pipelined calls, so it is an ordinary event (ev_pool_sync)
    std::vector<hipEvent_t> ev_pool, ev_pool_sync;
    std::vector<std::array<hipEvent_t, 4>> ev_rec;
};

namespace {

struct Plan {
    uint64_t n = 0, n_tiles = 0, total_cap = 0, max_len = 0;
    uint64_t n_segs = 0, scratch_entries = 0;
    uint64_t seg_bytes = 0, seg_cap = 0;
    bool any_multi = false;
    size_t bytes = 0;
};

// Layout of the descriptor buffer: ptr[n] len[n] last[n] jneed[n] tile_base[n+1] cut_base[n]
// cut_cap[n] seg_base[n+1] scratch_base[n] xtiles[1 + k], all u64 (xtiles: the count k, then
// the global indices of the tiles the fast path does not take).
StreamDesc desc_view(void *base, uint64_t n) {
    uint64_t *u = static_cast<uint64_t *>(base);
    StreamDesc d;
    d.ptr = reinterpret_cast<const uint8_t *const *>(u);
    d.len = u + n;
    d.last = u + 2 * n;
    d.jneed = u + 3 * n;
    d.tile_base = u + 4 * n;
    d.cut_base = u + 5 * n + 1;
    d.cut_cap = u + 6 * n + 1;
    d.seg_base = u + 7 * n + 1;
    d.scratch_base = u + 8 * n + 2;
    d.xtiles = u + 9 * n + 2;
    return d;
}

// Largest chunk start at which an argmax happens (S4), if any.
bool argmax_bound(uint64_t max_length, uint64_t L, uint64_t P, uint64_t &bound) {
    bool any = false;
    bound = 0;
    if (P >= max_length) {
        any = true;
        bound = P - max_length;
    }
    if (L >= 2 * max_length) {
        const uint64_t b2 = L - 2 * max_length;
        if (!any || b2 > bound) bound = b2;
        any = true;
    }
    return any;
}

uint64_t cut_cap_of(uint64_t min_length, uint64_t L) {
    const uint64_t step = std::max<uint64_t>(4, (min_length + 3) & ~3ull);
    return L / step + 3;
}

int validate_streams(uint64_t n, const uint8_t *const *ptrs, const uint64_t *lens,
                     const uint64_t *last, bool device_aligned) {
    if (n && (!ptrs || !lens)) return fail(RC_ERR_ARGUMENT, "null stream arrays");
    if (n >= (1ull << 31))  // tie markers carry the stream index in 31 bits (kernels.hip)
        return fail(RC_ERR_ARGUMENT, "too many streams in one call: %llu", (unsigned long long)n);
    for (uint64_t i = 0; i < n; ++i) {
        const uint64_t P = last ? last[i] : 0;
        if (P > lens[i]) return fail(RC_ERR_ARGUMENT, "stream %llu: last piece start %llu > length %llu",
                                     (unsigned long long)i, (unsigned long long)P,
                                     (unsigned long long)lens[i]);
        if (lens[i] && !ptrs[i]) return fail(RC_ERR_ARGUMENT, "stream %llu: null pointer", (unsigned long long)i);
        if (device_aligned && lens[i] && (reinterpret_cast<uintptr_t>(ptrs[i]) & 15))
            return fail(RC_ERR_ALIGN, "stream %llu: device pointer not 16-byte aligned",
                        (unsigned long long)i);
    }
    return 0;
}

// Fill the pinned descriptor staging and return the plan.  Waits for the previous upload
// from the same staging to have been consumed.
using Workspace = rc_chunker::Workspace;

Workspace &acquire_ws(rc_chunker *ch) {
    Workspace &w = ch->ws[ch->next_ws & 1];
    ++ch->next_ws;
    return w;
}

int stage_descriptors(rc_chunker *ch, Workspace &ws, uint64_t n, const uint8_t *const *ptrs,
                      const uint64_t *lens, const uint64_t *last, Plan &plan, bool open = false,
                      bool single = false, uint64_t walkers = 0) {
    plan.n = n;
    if (ws.pending) {  // the call that used this workspace before must be done with it
        HIP_TRY(hipEventSynchronize(ws.done));
        ws.pending = false;
    }
    // tiles the fast path does not take (kernels.hip tile_fast): a stream's tile 0 when the
    // stream is shorter than a tile, and its last tile when the stream ends inside it
    std::vector<uint64_t> &xt = ws.xtiles;
    xt.clear();
    {
        uint64_t tiles = 0;
        for (uint64_t i = 0; i < n; ++i) {
            const uint64_t L = lens[i], P = open ? L : (last ? last[i] : 0);
            const uint64_t jneed = rc_keys_needed(ch->max_length, L, P);
            const uint64_t nt = jneed ? jneed / kTileKeys + 1 : 0;
            const uint64_t jmax = L >= 8 ? (L - 4) / 4 : 0;
            auto fast = [&](uint64_t t) { return L >= 8 && t * kTileKeys + kTileKeys - 1 <= jmax; };
            if (nt && !fast(0)) xt.push_back(tiles);
            if (nt > 1 && !fast(nt - 1)) xt.push_back(tiles + nt - 1);  // the tiles between are fast
            tiles += nt;
        }
    }
    plan.bytes = (9 * n + 3 + xt.size()) * sizeof(uint64_t);
    if (int rc = ws.h_desc.ensure(plan.bytes)) return rc;
    uint64_t *u = static_cast<uint64_t *>(ws.h_desc.p);
    u[9 * n + 2] = xt.size();
    std::copy(xt.begin(), xt.end(), u + 9 * n + 3);
    // Chain segments.  The chain of a stream is one wave walking ~(bound / chunk) steps; split
    // a stream only when the batch has too few streams to keep ~kChainWalkers waves busy, and
    // never below seg_floor (2) * max_length per segment (speculative chains meet within a few
    // chunks; the merge kernel repairs a boundary where they do not).  4096
    // walkers (4 waves per SIMD): a walker is latency-bound, so shorter chains on more waves
    // finish sooner even with the extension steps and the join (round 2, same box: config 2
    // 0.19 -> 0.15 ms, 3 (ii) 0.31 -> 0.20, config 4 0.47 -> 0.24; 1024 walkers before).
    // Pipelined calls walk on the reserved CUs only (16 walkers per CU, as 4096 on 256): there
    // the chain must fit beside the next tile kernel, and fewer segments are less work.
    {
        const uint64_t kChainWalkers = walkers ? walkers : 4096;
        uint64_t total = 0;
        for (uint64_t i = 0; i < n; ++i) {
            uint64_t b = 0;
            const uint64_t P = open ? lens[i] : (last ? last[i] : 0);
            if (argmax_bound(ch->max_length, lens[i], P, b)) total += b;
        }
        // a stream gets floor(bound / seg) + 1 segments: size them with headroom so that a
        // batch of equal streams lands on one walker each when it already has enough streams
        uint64_t seg = ch->seg_force ? ch->seg_force
                                     : std::max<uint64_t>(total / kChainWalkers / 4 * 5 + 4, 1);
        const uint64_t floor_len =
            ch->max_length < (1ull << 60) ? ch->seg_floor * ch->max_length : ~0ull >> 2;
        if (!ch->seg_force) seg = std::max(seg, std::max<uint64_t>(floor_len, 4ull << 20));
        seg = std::max<uint64_t>((seg + 3) & ~3ull, 4);
        const uint64_t step = std::max<uint64_t>(4, (ch->min_length + 3) & ~3ull);
        plan.seg_bytes = seg;
        plan.seg_cap = seg / step + ch->ext_steps + 4;
    }
    uint64_t tiles = 0, cuts = 0, segs = 0, scratch = 0;
    plan.any_multi = false;
    for (uint64_t i = 0; i < n; ++i) {
        const uint64_t L = lens[i], P = open ? L : (last ? last[i] : 0);
        uint64_t bound = 0, nseg = 1;
        if (!single && argmax_bound(ch->max_length, L, P, bound)) nseg = bound / plan.seg_bytes + 1;
        u[7 * n + 1 + i] = segs;
        u[8 * n + 2 + i] = scratch;
        segs += nseg;
        if (nseg > 1) {
            scratch += nseg * plan.seg_cap;
            plan.any_multi = true;
        }
        const uint64_t jneed = rc_keys_needed(ch->max_length, L, P);
        plan.max_len = std::max(plan.max_len, L);
        u[i] = reinterpret_cast<uint64_t>(ptrs[i]);
        u[n + i] = L;
        u[2 * n + i] = P;
        u[3 * n + i] = jneed;
        u[4 * n + i] = tiles;
        tiles += jneed ? jneed / kTileKeys + 1 : 0;
        const uint64_t cap = cut_cap_of(ch->min_length, L);
        u[5 * n + 1 + i] = cuts;
        u[6 * n + 1 + i] = cap;
        cuts += cap;
    }
    u[5 * n] = tiles;
    u[8 * n + 1] = segs;
    // tile indices are 32-bit in the tile kernel's units and tie lists (kernels.hip TileUnits):
    // 2^32 tiles = 64 TiB of stream per call
    if (tiles >= (1ull << 32) - (1ull << 20))
        return fail(RC_ERR_ARGUMENT, "too many bytes in one call: %llu tiles", (unsigned long long)tiles);
    plan.n_tiles = tiles;
    plan.total_cap = cuts;
    plan.n_segs = segs;
    plan.scratch_entries = scratch;
    return 0;
}

GroupRecord *group_records(Workspace &ws, const Plan &plan) {
    return reinterpret_cast<GroupRecord *>(static_cast<char *>(ws.d_records.p) +
                                           (plan.n_tiles + 1) * sizeof(TileRecord));
}

// the tile kernel's tie lists: n_tiles slots, one count per work unit, the grab counter
uint32_t *tie_lists(Workspace &ws, const Plan &plan) {
    return reinterpret_cast<uint32_t *>(group_records(ws, plan) + plan.n_tiles + 1);
}

size_t records_bytes(const Plan &plan) {
    return (plan.n_tiles + 1) * (sizeof(TileRecord) + sizeof(GroupRecord)) +
           rc_tie_list_words(plan.n_tiles) * 4;
}

// the grab counter: allocated and zeroed once per workspace; every edge kernel leaves it 0.  A
// launch that failed after its tile kernel was queued leaves it dirty (abandon_launch): it is
// zeroed again on the stream of the next tile kernel, after the host has waited for the orphan.
// The first zeroing goes on that stream too (round 5): hipMemset runs on the legacy NULL
// stream, which a caller's non-blocking stream does not wait for, and since round 5 every
// launch grabs its units from this counter -- a tile kernel that started before the memset had
// landed read whatever the fresh allocation held (a GPU test saw a fresh chunker's first call
// come back with garbage counts once).
// A dirty buffer is re-zeroed up to the fault stamp: the fault count (kCtrFaultsWord) is kept
// for rc_chunker_check.
int ensure_ctr(Workspace &ws, hipStream_t st) {
    size_t zero = kCtrFaultsWord * 4;
    if (!ws.d_ctr.p) {
        if (int rc = ws.d_ctr.ensure(256)) return rc;
        ws.ctr_dirty = true;
        zero = 256;
    }
    if (ws.ctr_dirty) {
        HIP_TRY(hipMemsetAsync(ws.d_ctr.p, 0, zero, st));
        ws.ctr_dirty = false;
    }
    return 0;
}

const char kFaultMsg[] =
    "tile kernel fail-safe stop: a workgroup grab was never published, so the launch's records "
    "are incomplete and its cuts are not the reference's";

// Did the workspace's last launch take the tile kernel's fail-safe stop (kernels.hip
// UnitGrab::next; the edge kernel stamps the launch's epoch)?  Blocking read; the caller has
// synchronised.
int grab_fault(Workspace &ws) {
    if (!ws.d_ctr.p || !ws.epoch) return 0;
    uint64_t stamp = 0;
    HIP_TRY(hipMemcpy(&stamp, static_cast<uint32_t *>(ws.d_ctr.p) + kCtrStampWord, 8,
                      hipMemcpyDeviceToHost));
    return stamp == ws.epoch ? fail(RC_ERR_DEVICE_FAULT, "%s", kFaultMsg) : 0;
}

// The faults the workspace's launches counted since the last call (rc_chunker_check), reset.
int take_faults(Workspace &ws, uint32_t &n) {
    n = 0;
    if (!ws.d_ctr.p) return 0;
    uint32_t *w = static_cast<uint32_t *>(ws.d_ctr.p) + kCtrFaultsWord;
    HIP_TRY(hipMemcpy(&n, w, 4, hipMemcpyDeviceToHost));
    if (n) HIP_TRY(hipMemset(w, 0, 4));
    return 0;
}

// A launch sequence that failed after its tile kernel was queued: wait for whatever it queued
// (this workspace's buffers are reused by the call after next) and leave the grab counter to be
// re-zeroed -- its edge kernel, which zeroes it, may never have been queued.  Returns `rc`.
int abandon_launch(Workspace &ws, hipStream_t ts, hipStream_t xs, int rc) {
    (void)hipStreamSynchronize(ts);
    if (xs != ts) (void)hipStreamSynchronize(xs);
    ws.ctr_dirty = true;
    ws.pending = false;
    return rc;
}

// batches of at least this many streams walk their chains one lane per stream (when the
// windows are small and every stream is one segment: kernels.hip rc_lane_chain_kernel)
constexpr uint64_t kLaneMinStreams = 256;

int upload_and_launch(rc_chunker *ch, Workspace &ws, const Plan &plan, ChainParams prm,
                      uint64_t *d_cuts, int64_t *d_counts, hipStream_t stream,
                      bool pipelined = false, bool end = false) {
    if (int rc = ws.d_desc.ensure(plan.bytes)) return rc;
    // records, then (small windows) the group maxima of every tile, then the tie lists
    if (int rc = ws.d_records.ensure(records_bytes(plan))) return rc;
    if (int rc = ws.d_scratch.ensure(std::max<uint64_t>(plan.scratch_entries, 1) * 8)) return rc;
    // counts, merge points, slice offsets, slices and repaired counts of the parallel join
    // (kernels.hip)
    if (int rc = ws.d_seg_counts.ensure(std::max<uint64_t>(plan.n_segs, 1) * 40)) return rc;
    // The upload goes on the copy stream: stage_descriptors already waited for the call that
    // last used this workspace, so its device buffer is free now, while the previous call's
    // kernels may still be running on `stream`.  `stream` waits for the upload only.
    const int wi = &ws == &ch->ws[0] ? 0 : 1;
    if (!ch->cstream) HIP_TRY(hipStreamCreateWithFlags(&ch->cstream, hipStreamNonBlocking));
    if (!ch->uploaded[wi]) HIP_TRY(hipEventCreateWithFlags(&ch->uploaded[wi], hipEventDisableTiming));
    HIP_TRY(hipMemcpyAsync(ws.d_desc.p, ws.h_desc.p, plan.bytes, hipMemcpyHostToDevice, ch->cstream));
    HIP_TRY(hipEventRecord(ch->uploaded[wi], ch->cstream));
    // ts: the tile kernel's stream, xs: the edge and chain kernels'.  A pipelined call's tile
    // kernel waits for what the caller queued on `stream` before the call (its inputs); the
    // caller's stream waits for nothing (rc_chunk_wait)
    hipStream_t ts = stream, xs = stream;
    if (pipelined) {
        ts = wi == 1 && ch->tstream2 ? ch->tstream2 : ch->tstream;
        // RC_PIPELINE_END: nothing follows for this chain to overlap, so it runs on every CU
        xs = end ? ch->fstream : ch->xstream;
        // the inputs: nothing to wait for when the caller's stream has no work pending (each
        // event record and wait is a packet between two tile kernels)
        if (hipStreamQuery(stream) != hipSuccess) {
            HIP_TRY(hipEventRecord(ch->in_ev[wi], stream));
            HIP_TRY(hipStreamWaitEvent(ts, ch->in_ev[wi], 0));
        }
        // the chain kernels of consecutive calls stay in call order whichever stream they
        // are on (calls may share output arrays): wait for the previous call's
        HIP_TRY(hipStreamWaitEvent(xs, ch->ws[wi ^ 1].done, 0));
    }
    HIP_TRY(hipStreamWaitEvent(ts, ch->uploaded[wi], 0));
    if (int rc = ensure_ctr(ws, ts)) return rc;
    // the call's epoch: its chain kernels compare it with the edge kernel's fault stamp
    prm.fault = reinterpret_cast<const uint64_t *>(static_cast<uint32_t *>(ws.d_ctr.p) + kCtrStampWord);
    prm.epoch = ++ws.epoch;
    const StreamDesc d = desc_view(ws.d_desc.p, plan.n);
    std::array<hipEvent_t, 4> ev{};
    if (ch->timing) {
        // round 5: timing events with the default system-scope fence cost a harness step
        // ~20 us (0.808 vs 0.829 ms per step with and without them on one box,
        // profiles/r05/warmup/ab_harness*.log)
        for (int k = 0; k < 4; ++k) {
            std::vector<hipEvent_t> &pool = k == 1 ? ch->ev_pool_sync : ch->ev_pool;
            if (pool.empty()) {
                HIP_TRY(k == 1 ? hipEventCreate(&ev[k])
                               : hipEventCreateWithFlags(&ev[k], hipEventDisableSystemFence));
            } else {
                ev[k] = pool.back();
                pool.pop_back();
            }
        }
        HIP_TRY(hipEventRecord(ev[0], ts));
    }
    GroupRecord *grp = ch->groups ? group_records(ws, plan) : nullptr;
    prm.grp = grp;
    prm.n_tiles = plan.n_tiles;
    // lane-per-stream chain (kernels.hip rc_lane_chain_kernel) for batches of many streams;
    // RC_LANE_CHAIN: auto, 0 never, 1 whatever the count, lane one lane per stream (not a quad)
    switch (ch->knobs[knLaneChain]) {
    case 1: prm.lane = 0u; break;
    case 2: prm.lane = 2u; break;
    case 3: prm.lane = 3u; break;
    default: prm.lane = plan.n >= kLaneMinStreams ? 1u : 0u;
    }
    // 32-bit chain steps: small windows (the one-row record cache) and key indices < 2^32
    prm.lean = ch->small && plan.max_len < (16ull << 30) ? 1u : 0u;
    prm.hot = group_hot_threshold(ch->window);
    if (rc_launch_tiles(ch->d_tables, d, plan.n, plan.n_tiles,
                        static_cast<TileRecord *>(ws.d_records.p), grp, prm.hot, tie_lists(ws, plan),
                        static_cast<uint32_t *>(ws.d_ctr.p), prm.epoch, ts,
                        ch->timing ? ev[1] : nullptr,
                        pipelined ? ch->tile_cus : 0u, xs,
                        // the timing event after the tile kernel doubles as the hand-over event
                        !pipelined ? nullptr : ch->timing ? ev[1] : ch->tiled[wi], ch->sched))
        return abandon_launch(ws, ts, xs, fail(RC_ERR_HIP, "%s", rc_launch_error()));
    // A call in sequence after a pipelined one: that call's chain runs on another stream and
    // may still be writing cuts and counts that this call's chain writes too (calls may share
    // output arrays), so this chain waits for it.  (Pipelined calls wait above.)
    const Workspace &prev = ch->ws[wi ^ 1];
    if (!pipelined && prev.piped && hipStreamWaitEvent(xs, prev.done, 0) != hipSuccess)
        return abandon_launch(ws, ts, xs, fail(RC_ERR_HIP, "hipStreamWaitEvent failed"));
    if (ch->timing && hipEventRecord(ev[2], xs) != hipSuccess)
        return abandon_launch(ws, ts, xs, fail(RC_ERR_HIP, "hipEventRecord failed"));
    const uint32_t join = (ch->knobs[knJoinWalk] ? RC_JOIN_WALK_ONLY : 0u) |
                          (ch->knobs[knRepair] ? RC_JOIN_REPAIR : 0u);
    if (rc_launch_chain(ch->d_tables, d, plan.n, prm, plan.n_segs,
                        static_cast<const TileRecord *>(ws.d_records.p), d_cuts, d_counts,
                        static_cast<uint64_t *>(ws.d_scratch.p),
                        static_cast<uint64_t *>(ws.d_seg_counts.p), plan.any_multi, join, xs))
        return abandon_launch(ws, ts, xs, fail(RC_ERR_HIP, "%s", rc_launch_error()));
    if (hipEventRecord(ws.done, xs) != hipSuccess)
        return abandon_launch(ws, ts, xs, fail(RC_ERR_HIP, "hipEventRecord failed"));
    ws.pending = true;
    ws.piped = pipelined;
    if (ch->timing) {
        HIP_TRY(hipEventRecord(ev[3], xs));
        ch->ev_rec.push_back(ev);
    }
    return 0;
}

// CUs reserved for the edge and chain kernels of pipelined calls when rc_chunker_overlap does
// not say (RC_OVERLAP_CUS, knobs.h, default 32): one per shader engine (4 per XCD).  Measured on one allocation
// (scripts/overlap_ab.py, profiles/r03/overlap/): reserving 8 or 16 CUs left the shader
// engines of an XCD unequal and the persistent tile kernel 15 % slower (config 2: 11.3 and
// 11.7 ms against 9.87 unpipelined -- a workgroup the dispatcher sends to a full engine waits
// for the end of the launch); 32 keeps every engine at 7 CUs and the tile kernel at 9.84 ms.
// The two streams of overlap mode.  KFD spreads the bits of a queue's CU mask over the XCDs
// first (bit i -> XCD i % 8), then over that XCD's shader engines (bits 0-7 engine 0, 8-15
// engine 1, ...), so the first `reserve` bits take reserve / 8 CUs of every XCD and, for a
// multiple of 32, the same number of every engine (scripts/ubench/cumask_probe.hip reads the
// CUs each mask runs on: disjoint, 2 or 4 per XCD).
int setup_overlap(rc_chunker *ch) {
    const uint32_t want = ch->reserve_req ? ch->reserve_req : (uint32_t)ch->knobs[knOverlapCus];
    if (ch->tstream && ch->reserve == want) return 0;
    int cus = 0;
    HIP_TRY(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, ch->device));
    if (want == 0 || (int)want >= cus)
        return fail(RC_ERR_ARGUMENT, "overlap: %u reserved CUs of %d", want, cus);
    if (ch->tstream) {  // a different split: retire the old pair
        if (ch->tstream2) {
            HIP_TRY(hipStreamSynchronize(ch->tstream2));
            (void)hipStreamDestroy(ch->tstream2);
            ch->tstream2 = nullptr;
        }
        HIP_TRY(hipStreamSynchronize(ch->tstream));
        HIP_TRY(hipStreamSynchronize(ch->xstream));
        (void)hipStreamDestroy(ch->tstream);
        (void)hipStreamDestroy(ch->xstream);
        ch->tstream = ch->xstream = nullptr;
    }
    std::vector<uint32_t> tm((cus + 31) / 32, 0u), xm((cus + 31) / 32, 0u);
    for (int i = 0; i < cus; ++i) ((uint32_t)i < want ? xm : tm)[i / 32] |= 1u << (i % 32);
    // RC_TILE_MASK (measurement switch): full -- the tile stream's mask holds every CU; plain --
    // an ordinary non-blocking stream.  Either way its workgroups may take any CU the chain
    // kernels leave (they cannot share one: 144 KiB of LDS); dynamic units make a late one harmless
    const int64_t tmask = ch->knobs[knTileMask];
    if (tmask == 1)
        for (int i = 0; i < cus; ++i) tm[i / 32] |= 1u << (i % 32);
    if (tmask == 2)
        HIP_TRY(hipStreamCreateWithFlags(&ch->tstream, hipStreamNonBlocking));
    else
        HIP_TRY(hipExtStreamCreateWithCUMask(&ch->tstream, (uint32_t)tm.size(), tm.data()));
    const hipError_t ex = hipExtStreamCreateWithCUMask(&ch->xstream, (uint32_t)xm.size(), xm.data());
    if (ex != hipSuccess) {  // both streams or neither (a call checks tstream only)
        (void)hipStreamDestroy(ch->tstream);
        ch->tstream = ch->xstream = nullptr;
        return fail(RC_ERR_HIP, "hipExtStreamCreateWithCUMask failed: %s", hipGetErrorString(ex));
    }
    // RC_TILE_STREAMS=2: odd calls' tile kernels on a second stream with the same mask (a queue
    // of its own), so that a call's tile kernel is not held behind the previous one's last
    // workgroups: its workgroups take the CUs the previous launch leaves (their workspaces are
    // distinct; a call's chain still follows its own tile kernel and the previous chain)
    if (ch->knobs[knTileStreams] == 2 &&
        (tmask == 2 ? hipStreamCreateWithFlags(&ch->tstream2, hipStreamNonBlocking)
                    : hipExtStreamCreateWithCUMask(&ch->tstream2, (uint32_t)tm.size(), tm.data())) !=
            hipSuccess)
        ch->tstream2 = nullptr;  // one tile stream: still correct
    if (!ch->fstream) HIP_TRY(hipStreamCreateWithFlags(&ch->fstream, hipStreamNonBlocking));
    for (int i = 0; i < 2; ++i) {
        if (!ch->in_ev[i]) HIP_TRY(hipEventCreateWithFlags(&ch->in_ev[i], hipEventDisableTiming));
        if (!ch->tiled[i]) HIP_TRY(hipEventCreateWithFlags(&ch->tiled[i], hipEventDisableTiming));
    }
    ch->reserve = want;
    ch->tile_cus = (uint32_t)cus - (tmask ? 0u : want);
    return 0;
}

ChainParams chain_params(const rc_chunker *ch, const Plan &plan, uint64_t max_steps,
                         uint32_t flags = 0) {
    ChainParams p;
    p.open = (flags & RC_OPEN) ? 1u : 0u;
    p.min_length = ch->min_length;
    p.max_length = ch->max_length;
    p.window = ch->window;
    p.max_steps = max_steps;
    p.seg_bytes = plan.seg_bytes;
    p.seg_cap = plan.seg_cap;
    p.ext_steps = ch->ext_steps;
    p.grp = nullptr;  // set per launch (upload_and_launch)
    p.n_tiles = 0;
    p.lean = 0;
    p.lane = 0;
    p.hot = 0;
    p.fault = nullptr;  // set per launch (upload_and_launch)
    p.epoch = 0;
    return p;
}

}  // namespace

extern "C" {

int rc_version(void) { return 300; }

#ifndef RC_BUILD_ID
#define RC_BUILD_ID "unknown"
#endif
// "RC_BUILD_ID:" + the hash replicat_amd/build.py computes over the sources and flags; the
// marker lets build.py read it from the .so file without loading it
static const char kBuildId[] = "RC_BUILD_ID:" RC_BUILD_ID;
const char *rc_build_id(void) { return kBuildId + 12; }

const char *rc_last_error(void) { return g_err; }

uint32_t rc_group_hot_threshold(const rc_chunker *ch) { return ch ? group_hot_threshold(ch->window) : 0u; }

uint64_t rc_keys_needed(uint64_t max_length, uint64_t L, uint64_t P) {
    // S4: at chunk start s an argmax happens iff P - s >= max or L - s >= 2*max; the window of
    // start s reaches key s/4 + T (adapters.cpp:59).  Largest such s -> largest key.
    const uint64_t T = window_keys(max_length);
    if (T == 0 || L < 8) return 0;
    bool any = false;
    uint64_t bound = 0;
    if (P >= max_length) {
        any = true;
        bound = P - max_length;
    }
    if (L >= 2 * max_length) {
        const uint64_t b2 = L - 2 * max_length;
        if (!any || b2 > bound) bound = b2;
        any = true;
    }
    if (!any) return 0;
    const uint64_t jneed = bound / 4 + T, jmax = (L - 4) / 4;
    return std::min(jneed, jmax);
}

int rc_chunker_create(uint64_t min_length, uint64_t max_length, const uint8_t *key,
                      uint64_t key_len, int device, rc_chunker **out) {
    if (!out) return fail(RC_ERR_ARGUMENT, "null output handle");
    *out = nullptr;
    // adapters.cpp:21-29, in the reference's order
    if (key_len != 16 || !key) return fail(RC_ERR_KEY_LENGTH, "key must contain exactly 16 characters");
    if (min_length > max_length)
        return fail(RC_ERR_MIN_GT_MAX, "Minimum length is greater than the maximum one");
    const uint64_t k0 = load_le64(key), k1 = load_le64(key + 8);
    if (k0 == 0) return fail(RC_ERR_BAD_KEY, "Bad key contents");
    // the environment knobs (knobs.h), once: a malformed one is an error, not a silent default
    Knobs knobs;
    if (read_knobs(knobs, g_err, sizeof g_err)) return RC_ERR_ARGUMENT;

    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0)
        return fail(RC_ERR_NO_DEVICE, "no HIP device available (the chunker runs on MI355X only)");
    if (device < 0 || device >= ndev) return fail(RC_ERR_NO_DEVICE, "device %d out of range", device);
    hipDeviceProp_t prop;
    HIP_TRY(hipGetDeviceProperties(&prop, device));
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return fail(RC_ERR_NO_DEVICE, "device %d is %s, not gfx950", device, prop.gcnArchName);

    rc_chunker *ch = new rc_chunker();
    ch->min_length = min_length;
    ch->max_length = max_length;
    ch->window = window_keys(max_length);
    // a window (plus its two edge tiles) within one 64-tile row of the chain's record cache:
    // the chain's edge ranges are then a large part of its work, and group maxima trim them
    ch->knobs = knobs;
    ch->small = ch->window / kTileKeys + 3 <= 64;
    // RC_TILE_GROUPS=1: group records for large windows too (the chains trim their edge ranges
    // with them, chain_step; measured slower); =0: never
    ch->groups = knobs[knTileGroups] == 0 ? ch->small : knobs[knTileGroups] == 2;
    if (knobs[knChainLean] == 1) ch->small = false;  // RC_CHAIN_LEAN=0
    ch->sched.permille = (uint32_t)knobs[knTileStatic];
    ch->sched.chunk = (uint32_t)knobs[knTileChunk];
    ch->sched.dyn_min = (uint32_t)knobs[knTileDynMin];
    ch->sched.group = (uint32_t)knobs[knTileGroup];
    ch->k0 = k0;
    ch->k1 = k1;
    ch->device = device;
    build_tables(k0, k1, ch->tables);
    // chain segmentation (RC_SEGMENT_BYTES forces a segment length; the per-call choice is made
    // in stage_descriptors).  2 extension steps past the segment end, segments of at least 2 x
    // max (round 3, with boundary repair in the merge kernel: a boundary whose chains miss is
    // continued where it is, where before one miss sent the whole stream to the sequential join,
    // so round 2 ran 4 steps over 3 x max).  One allocation each (scripts/chain_ab.py,
    // profiles/r03/repair/): the harness's chain 0.108 -> 0.091 ms, 3 (ii) 0.241 -> 0.231, config
    // 4 0.268 -> 0.253, config 2 0.159 -> 0.152; 1 x max segments with 1 step miss past the next
    // list and fall back (1.76 ms on the harness)
    ch->seg_force = (uint64_t)knobs[knSegmentBytes];
    ch->ext_steps = (uint64_t)knobs[knSegmentExt];
    ch->seg_floor = (uint64_t)knobs[knSegmentFloor];
    {
        DeviceGuard g(device);
        hipError_t e = hipMalloc(&ch->d_tables, sizeof(KeyTables));
        if (e == hipSuccess)
            e = hipMemcpy(ch->d_tables, &ch->tables, sizeof(KeyTables), hipMemcpyHostToDevice);
        for (auto &w : ch->ws)
            if (e == hipSuccess) e = hipEventCreateWithFlags(&w.done, hipEventDisableTiming);
        if (e != hipSuccess) {
            rc_chunker_destroy(ch);
            return fail(RC_ERR_HIP, "device setup failed: %s", hipGetErrorString(e));
        }
    }
    rc_track(ch, [](void *h) { rc_chunker_destroy(static_cast<rc_chunker *>(h)); });
    *out = ch;
    return RC_OK;
}

void rc_chunker_destroy(rc_chunker *ch) {
    if (!ch) return;
    rc_untrack(ch);
    {
        // a call still running on another thread (a daemon thread when the exit hook runs)
        // finishes first: its buffers and streams go only after it
        std::lock_guard<std::mutex> lock(ch->mu);
        DeviceGuard g(ch->device);
        (void)hipDeviceSynchronize();
        if (ch->d_tables) (void)hipFree(ch->d_tables);
        for (auto &w : ch->ws) {
            w.d_desc.release();
            w.d_records.release();
            w.d_scratch.release();
            w.d_seg_counts.release();
            w.d_ctr.release();
            w.h_desc.release();
            if (w.done) (void)hipEventDestroy(w.done);
        }
        ch->d_buf.release();
        ch->d_out.release();
        for (int i = 0; i < 2; ++i) {
            ch->d_stage[i].release();
            ch->d_hcuts[i].release();
            ch->d_hcounts[i].release();
            ch->d_hdig[i].release();
            if (ch->hstream[i]) (void)hipStreamDestroy(ch->hstream[i]);
        }
        ch->h_out.release();
        if (ch->cstream) (void)hipStreamDestroy(ch->cstream);
        if (ch->tstream) (void)hipStreamDestroy(ch->tstream);
        if (ch->tstream2) (void)hipStreamDestroy(ch->tstream2);
        if (ch->xstream) (void)hipStreamDestroy(ch->xstream);
        if (ch->fstream) (void)hipStreamDestroy(ch->fstream);
        for (auto e : ch->uploaded)
            if (e) (void)hipEventDestroy(e);
        for (int i = 0; i < 2; ++i) {
            if (ch->in_ev[i]) (void)hipEventDestroy(ch->in_ev[i]);
            if (ch->tiled[i]) (void)hipEventDestroy(ch->tiled[i]);
        }
        for (auto &r : ch->ev_rec)
            for (auto e : r) (void)hipEventDestroy(e);
        for (auto e : ch->ev_pool) (void)hipEventDestroy(e);
        for (auto e : ch->ev_pool_sync) (void)hipEventDestroy(e);
    }
    delete ch;
}

uint64_t rc_chunker_min_length(const rc_chunker *ch) { return ch ? ch->min_length : 0; }
uint64_t rc_chunker_max_length(const rc_chunker *ch) { return ch ? ch->max_length : 0; }

uint64_t rc_host_key(const rc_chunker *ch, uint64_t d) {
    const uint32_t lo = (uint32_t)d, hi = (uint32_t)(d >> 32);
    uint64_t k = 0;
    for (int b = 0; b < 4; ++b) k ^= ch->tables.tl[b][(lo >> (8 * b)) & 255] ^ ch->tables.th[b][(hi >> (8 * b)) & 255];
    return k;
}

int rc_tables_key(const uint8_t *key16, uint64_t n, const uint64_t *ds, uint64_t *out,
                  uint32_t *top16) {
    if (!key16 || (n && (!ds || !out))) return fail(RC_ERR_ARGUMENT, "null argument");
    KeyTables *t = new KeyTables;
    build_tables(load_le64(key16), load_le64(key16 + 8), *t);
    for (uint64_t i = 0; i < n; ++i) {
        const uint32_t lo = (uint32_t)ds[i], hi = (uint32_t)(ds[i] >> 32);
        uint64_t k = 0;
        uint32_t el = 0, eh = 0;
        for (int b = 0; b < 4; ++b) {
            k ^= t->tl[b][(lo >> (8 * b)) & 255] ^ t->th[b][(hi >> (8 * b)) & 255];
            el ^= t->pf[b][(lo >> (8 * b)) & 255];
            eh ^= t->pf[b][(hi >> (8 * b)) & 255];
        }
        out[i] = k;
        // the kernel's combination: (e(w[j-1]) & 0xffff0000) ^ (e(w[j]) << 16)
        if (top16) top16[i] = ((el & 0xffff0000u) ^ (eh << 16)) >> 16;
    }
    delete t;
    return RC_OK;
}

uint64_t rc_cut_capacity(const rc_chunker *ch, uint64_t n, const uint64_t *lens, uint64_t *caps) {
    uint64_t total = 0;
    for (uint64_t i = 0; i < n; ++i) {
        const uint64_t c = cut_cap_of(ch->min_length, lens[i]);
        if (caps) caps[i] = c;
        total += c;
    }
    return total;
}

int rc_next_cut(rc_chunker *ch, const uint8_t *buffer, uint64_t size, int final, uint64_t *out_cut) {
    if (!ch || !out_cut) return fail(RC_ERR_ARGUMENT, "null argument");
    if (size && !buffer) return fail(RC_ERR_ARGUMENT, "null buffer");
    const uint64_t mn = ch->min_length, mx = ch->max_length;
    // adapters.cpp:48-57
    if (final && size < 2 * mx) {
        *out_cut = size <= mx ? size : (size < mx + mn ? size / 2 : mx);
        return RC_OK;
    }
    if (!final && size < mx) {
        *out_cut = 0;
        return RC_OK;
    }
    if (ch->window == 0) {  // no key offsets below max: adapters.cpp:66-67 directly
        *out_cut = (mn + 3) & ~3ull;
        return RC_OK;
    }
    std::lock_guard<std::mutex> lock(ch->mu);
    DeviceGuard g(ch->device);
    // keys 1..T read bytes [0, 4T+4); never more than the buffer holds
    const uint64_t ncopy = std::min<uint64_t>(size, 4 * ch->window + 4);
    if (int rc = ch->d_buf.ensure(ncopy + 16)) return rc;
    if (int rc = ch->d_out.ensure(64)) return rc;
    if (int rc = ch->h_out.ensure(64)) return rc;
    hipStream_t stream = nullptr;
    HIP_TRY(hipMemcpyAsync(ch->d_buf.p, buffer, ncopy, hipMemcpyHostToDevice, stream));
    const uint8_t *ptr = static_cast<const uint8_t *>(ch->d_buf.p);
    const uint64_t L = ncopy, P = ncopy;
    Plan plan;
    Workspace &ws = acquire_ws(ch);
    if (int rc = stage_descriptors(ch, ws, 1, &ptr, &L, &P, plan, false, true)) return rc;
    uint64_t *d_cut = static_cast<uint64_t *>(ch->d_out.p);
    int64_t *d_count = reinterpret_cast<int64_t *>(d_cut + 1);
    const bool timing = ch->timing;
    ch->timing = false;
    int rc = upload_and_launch(ch, ws, plan, chain_params(ch, plan, 0), d_cut, d_count, stream);
    ch->timing = timing;
    if (rc) return rc;
    HIP_TRY(hipMemcpyAsync(ch->h_out.p, d_cut, 16, hipMemcpyDeviceToHost, stream));
    HIP_TRY(hipStreamSynchronize(stream));
    const uint64_t *h = static_cast<const uint64_t *>(ch->h_out.p);
    if ((int64_t)h[1] == kCountFault) return fail(RC_ERR_DEVICE_FAULT, "%s", kFaultMsg);
    if ((int64_t)h[1] != 1) return fail(RC_ERR_OVERFLOW, "device chain returned %lld cuts", (long long)h[1]);
    *out_cut = h[0];
    return RC_OK;
}

int rc_chunk_device(rc_chunker *ch, uint64_t n, const uint8_t *const *d_streams,
                    const uint64_t *lens, const uint64_t *last_piece, uint32_t flags,
                    uint64_t *d_cuts, int64_t *d_counts, void *hip_stream) {
    if (!ch) return fail(RC_ERR_ARGUMENT, "null chunker");
    if (n == 0) return RC_OK;
    if (!d_cuts || !d_counts) return fail(RC_ERR_ARGUMENT, "null output arrays");
    const bool open = (flags & RC_OPEN) != 0;
    if (int rc = validate_streams(n, d_streams, lens, open ? nullptr : last_piece, true)) return rc;
    // Small-window chunkers (group records, lane / quad chains: config 3 iii) run a pipelined
    // request in sequence on the caller's stream -- a legal schedule of the flag (inputs and
    // outputs in that stream's order): their quad chain takes 2.8 ms on 32 CUs and their
    // VALU-heavier tile kernel lost 3 % on 224 CUs (scripts/overlap_ab.py, profiles/r03/overlap/).
    // Round 4 re-measured launches on the static schedule (the harness: one 5.12 GB stream,
    // 76 tiles per wave), which round 3 also ran in sequence: on one allocation the tile kernel
    // takes 0.833 ms on 224 CUs as on 256, and pipelined steps 0.876 ms against 0.950 in sequence
    // (profiles/r04/harness/harness_sched.log), so they pipeline now -- when the request has at
    // least a tile per wave (below).  RC_PIPE_ALL=1 pipelines every call (tests, measurements).
    std::lock_guard<std::mutex> lock(ch->mu);
    DeviceGuard g(ch->device);
    const bool all = ch->knobs[knPipeAll] != 0;
    bool pipelined = (flags & RC_PIPELINED) != 0 && (all || !ch->groups);
    // no CU-masked streams on this device / runtime: the request runs in sequence (the call
    // stays correct; rc_chunker_overlap reports the error, rc_chunker_overlap_cus stays 0)
    if (pipelined && !ch->overlap_failed && setup_overlap(ch) != 0) {
        ch->overlap_failed = true;
        fprintf(stderr, "replicat_amd: pipelined calls run in sequence: %s\n", g_err);
    }
    if (ch->overlap_failed && !ch->tstream) pipelined = false;
    // A request with fewer tiles than the masked tile launch has waves has next to nothing to
    // overlap its chain with, and that chain would run on the reserved CUs only: config 3 (i)
    // (65,536 x 1 MiB at the defaults: no key is ever needed) took 0.78 ms per step pipelined
    // against 0.43 in sequence (profiles/r04/final/configs.log).  It runs in sequence.
    if (pipelined && !all) {
        uint64_t tiles = 0;
        for (uint64_t i = 0; i < n; ++i) {
            const uint64_t P = open ? lens[i] : (last_piece ? last_piece[i] : 0);
            const uint64_t j = rc_keys_needed(ch->max_length, lens[i], P);
            tiles += j ? j / kTileKeys + 1 : 0;
        }
        if (tiles < 16ull * ch->tile_cus) pipelined = false;
    }
    ch->pipelined_calls += pipelined ? 1 : 0;
    Plan plan;
    Workspace &ws = acquire_ws(ch);
    if (int rc = stage_descriptors(ch, ws, n, d_streams, lens, last_piece, plan, open, false,
                                   pipelined ? 16ull * ch->reserve : 0))
        return rc;
    return upload_and_launch(ch, ws, plan, chain_params(ch, plan, ~0ull, flags), d_cuts, d_counts,
                             static_cast<hipStream_t>(hip_stream), pipelined,
                             (flags & RC_PIPELINE_END) != 0);
}

int rc_stream_create(int device, void **out_stream) {
    if (!out_stream) return fail(RC_ERR_ARGUMENT, "null output stream");
    *out_stream = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev)
        return fail(RC_ERR_NO_DEVICE, "no HIP device %d", device);
    DeviceGuard g(device);
    int cus = 0;
    HIP_TRY(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device));
    std::vector<uint32_t> mask((cus + 31) / 32, 0u);
    for (int i = 0; i < cus; ++i) mask[i / 32] |= 1u << (i % 32);
    hipStream_t s = nullptr;
    HIP_TRY(hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size(), mask.data()));
    rc_track(s, [](void *h) { rc_stream_destroy(h); });
    *out_stream = s;
    return RC_OK;
}

void rc_stream_destroy(void *stream) {
    if (!stream) return;
    rc_untrack(stream);
    (void)hipStreamSynchronize(static_cast<hipStream_t>(stream));
    (void)hipStreamDestroy(static_cast<hipStream_t>(stream));
}

int rc_chunker_overlap(rc_chunker *ch, uint32_t reserve_cus) {
    if (!ch) return fail(RC_ERR_ARGUMENT, "null chunker");
    std::lock_guard<std::mutex> lock(ch->mu);
    DeviceGuard g(ch->device);
    ch->reserve_req = reserve_cus;
    const int rc = setup_overlap(ch);
    ch->overlap_failed = rc != 0 && !ch->tstream;
    return rc;
}

uint32_t rc_chunker_overlap_cus(const rc_chunker *ch) { return ch ? ch->reserve : 0u; }

uint64_t rc_chunker_pipelined_calls(const rc_chunker *ch) { return ch ? ch->pipelined_calls : 0; }

int rc_chunker_check(rc_chunker *ch) {
    if (!ch) return fail(RC_ERR_ARGUMENT, "null chunker");
    std::lock_guard<std::mutex> lock(ch->mu);
    DeviceGuard g(ch->device);
    uint32_t faults = 0;
    for (auto &w : ch->ws) {
        if (w.pending) HIP_TRY(hipEventSynchronize(w.done));
        uint32_t n = 0;
        if (int rc = take_faults(w, n)) return rc;
        faults += n;
    }
    if (faults)
        return fail(RC_ERR_DEVICE_FAULT, "%s (%u call(s) since the last check)", kFaultMsg, faults);
    return RC_OK;
}

int rc_chunk_wait(rc_chunker *ch, void *hip_stream) {
    if (!ch) return fail(RC_ERR_ARGUMENT, "null chunker");
    std::lock_guard<std::mutex> lock(ch->mu);
    DeviceGuard g(ch->device);
    // a workspace's `done` was recorded by its last call, after the host had waited for the
    // call before that one on the same workspace: the two events cover every call so far
    for (auto &w : ch->ws)
        HIP_TRY(hipStreamWaitEvent(static_cast<hipStream_t>(hip_stream), w.done, 0));
    return RC_OK;
}

}  // extern "C"

namespace {

// rc_chunk_host, and with a hasher rc_chunk_digest_host: batches of whole streams go through
// pinned double-buffered copies; each batch's kernels (and digests) run on one of two streams.
int chunk_host_impl(rc_chunker *ch, rc_hasher *hasher, uint64_t n, const uint8_t *const *streams,
                    const uint64_t *lens, const uint64_t *last_piece, uint32_t flags,
                    uint64_t *cuts, int64_t *counts, uint8_t *digests) {
    if (!ch) return fail(RC_ERR_ARGUMENT, "null chunker");
    if (n == 0) return RC_OK;
    if (!cuts || !counts) return fail(RC_ERR_ARGUMENT, "null output arrays");
    if (hasher && !digests) return fail(RC_ERR_ARGUMENT, "null digest array");
    const bool open = (flags & RC_OPEN) != 0;
    if (int rc = validate_streams(n, streams, lens, open ? nullptr : last_piece, false)) return rc;
    std::lock_guard<std::mutex> lock(ch->mu);
    DeviceGuard g(ch->device);
    for (int i = 0; i < 2; ++i)
        if (!ch->hstream[i]) HIP_TRY(hipStreamCreateWithFlags(&ch->hstream[i], hipStreamNonBlocking));

    // batches of whole streams, each up to `budget` bytes (one stream may exceed it alone)
    const uint64_t budget = 1ull << 30;
    std::vector<uint64_t> cut_base(n + 1, 0);
    for (uint64_t i = 0; i < n; ++i) cut_base[i + 1] = cut_base[i] + cut_cap_of(ch->min_length, lens[i]);

    struct Batch {
        uint64_t first = 0, count = 0;
    } inflight[2];
    bool busy[2] = {false, false};
    std::vector<const uint8_t *> dptr;
    std::vector<uint64_t> off;

    auto finish = [&](int slot) -> int {
        if (!busy[slot]) return 0;
        HIP_TRY(hipStreamSynchronize(ch->hstream[slot]));
        busy[slot] = false;
        const Batch &b = inflight[slot];
        for (uint64_t i = 0; i < b.count; ++i) {
            if (counts[b.first + i] == kCountFault) return fail(RC_ERR_DEVICE_FAULT, "%s", kFaultMsg);
            if (counts[b.first + i] < 0)
                return fail(RC_ERR_OVERFLOW, "stream %llu overflowed its cut capacity",
                            (unsigned long long)(b.first + i));
        }
        return 0;
    };

    uint64_t i = 0;
    int slot = 0;
    while (i < n) {
        uint64_t j = i, bytes = 0;
        while (j < n && (j == i || bytes + ((lens[j] + 15) & ~15ull) <= budget)) {
            bytes += (lens[j] + 15) & ~15ull;
            ++j;
        }
        if (int rc = finish(slot)) return rc;  // slot's previous batch done: buffers free
        const uint64_t nb = j - i;
        if (int rc = ch->d_stage[slot].ensure(bytes + 16)) return rc;
        const uint64_t ncut = cut_base[j] - cut_base[i];
        if (int rc = ch->d_hcuts[slot].ensure(ncut * 8)) return rc;
        if (int rc = ch->d_hcounts[slot].ensure(nb * 8)) return rc;
        hipStream_t st = ch->hstream[slot];
        dptr.resize(nb);
        uint64_t o = 0;
        for (uint64_t k = 0; k < nb; ++k) {
            uint8_t *dst = static_cast<uint8_t *>(ch->d_stage[slot].p) + o;
            dptr[k] = dst;
            if (lens[i + k]) HIP_TRY(hipMemcpyAsync(dst, streams[i + k], lens[i + k], hipMemcpyHostToDevice, st));
            o += (lens[i + k] + 15) & ~15ull;
        }
        Plan plan;
        Workspace &ws = acquire_ws(ch);
        if (int rc = stage_descriptors(ch, ws, nb, dptr.data(), lens + i,
                                       last_piece ? last_piece + i : nullptr, plan, open))
            return rc;
        uint64_t *dc = static_cast<uint64_t *>(ch->d_hcuts[slot].p);
        int64_t *dn = static_cast<int64_t *>(ch->d_hcounts[slot].p);
        if (int rc = upload_and_launch(ch, ws, plan, chain_params(ch, plan, ~0ull, flags), dc, dn, st))
            return rc;
        if (hasher) {
            if (int rc = ch->d_hdig[slot].ensure(ncut * kDigestSlot)) return rc;
            uint8_t *dd = static_cast<uint8_t *>(ch->d_hdig[slot].p);
            std::vector<uint64_t> cb(nb);
            for (uint64_t k = 0; k < nb; ++k) cb[k] = cut_base[i + k] - cut_base[i];
            uint64_t bytes = 0, longest = 0;
            for (uint64_t k = 0; k < nb; ++k) {
                bytes += lens[i + k];
                longest = std::max(longest, lens[i + k]);
            }
            if (int rc = rc_hasher_enqueue_chunks(hasher, nb, dptr.data(), cb.data(), dc, dn, ncut,
                                                  bytes, std::min(longest, ch->max_length), dd, st))
                return rc;
            HIP_TRY(hipMemcpyAsync(digests + cut_base[i] * kDigestSlot, dd, ncut * kDigestSlot,
                                   hipMemcpyDeviceToHost, st));
        }
        HIP_TRY(hipMemcpyAsync(cuts + cut_base[i], dc, ncut * 8, hipMemcpyDeviceToHost, st));
        HIP_TRY(hipMemcpyAsync(counts + i, dn, nb * 8, hipMemcpyDeviceToHost, st));
        inflight[slot] = {i, nb};
        busy[slot] = true;
        i = j;
        slot ^= 1;
    }
    if (int rc = finish(0)) return rc;
    if (int rc = finish(1)) return rc;
    return RC_OK;
}

}  // namespace

extern "C" {

int rc_chunk_host(rc_chunker *ch, uint64_t n, const uint8_t *const *streams, const uint64_t *lens,
                  const uint64_t *last_piece, uint32_t flags, uint64_t *cuts, int64_t *counts) {
    return chunk_host_impl(ch, nullptr, n, streams, lens, last_piece, flags, cuts, counts, nullptr);
}

int rc_chunk_digest_host(rc_chunker *ch, rc_hasher *h, uint64_t n, const uint8_t *const *streams,
                         const uint64_t *lens, const uint64_t *last_piece, uint32_t flags,
                         uint64_t *cuts, int64_t *counts, uint8_t *digests) {
    if (!h) return fail(RC_ERR_ARGUMENT, "null hasher");
    return chunk_host_impl(ch, h, n, streams, lens, last_piece, flags, cuts, counts, digests);
}

uint64_t rc_tile_keys(void) { return kTileKeys; }

int rc_tile_records(rc_chunker *ch, uint64_t n, const uint8_t *const *d_streams,
                    const uint64_t *lens, const uint64_t *last_piece, uint64_t *keys,
                    uint64_t *js, uint64_t *gmax, uint64_t *ghot, uint64_t cap,
                    uint64_t *n_tiles) {
    if (!ch || !n_tiles) return fail(RC_ERR_ARGUMENT, "null argument");
    if (int rc = validate_streams(n, d_streams, lens, last_piece, true)) return rc;
    std::lock_guard<std::mutex> lock(ch->mu);
    DeviceGuard g(ch->device);
    Plan plan;
    Workspace &ws = acquire_ws(ch);
    if (int rc = stage_descriptors(ch, ws, n, d_streams, lens, last_piece, plan)) return rc;
    if (int rc = ws.d_desc.ensure(plan.bytes)) return rc;
    if (int rc = ws.d_records.ensure(records_bytes(plan))) return rc;
    HIP_TRY(hipMemcpy(ws.d_desc.p, ws.h_desc.p, plan.bytes, hipMemcpyHostToDevice));
    if (int rc = ensure_ctr(ws, nullptr)) return rc;
    GroupRecord *d_grp = ch->groups ? group_records(ws, plan) : nullptr;
    // poison the records first: a tile the schedule never ran shows as 0xabab.. keys
    if (plan.n_tiles)
        HIP_TRY(hipMemset(ws.d_records.p, 0xab, (plan.n_tiles + 1) * sizeof(TileRecord)));
    if (rc_launch_tiles(ch->d_tables, desc_view(ws.d_desc.p, n), n, plan.n_tiles,
                        static_cast<TileRecord *>(ws.d_records.p), d_grp,
                        group_hot_threshold(ch->window), tie_lists(ws, plan),
                        static_cast<uint32_t *>(ws.d_ctr.p), ++ws.epoch, nullptr, nullptr, 0u,
                        nullptr, nullptr, ch->sched))
        return abandon_launch(ws, nullptr, nullptr, fail(RC_ERR_HIP, "%s", rc_launch_error()));
    HIP_TRY(hipDeviceSynchronize());
    if (int rc = grab_fault(ws)) return rc;
    std::vector<TileRecord> h(plan.n_tiles);
    std::vector<GroupRecord> hg(plan.n_tiles, GroupRecord{~0ull, {~0ull, ~0ull, ~0ull, ~0ull}, 0ull});
    if (plan.n_tiles) {
        HIP_TRY(hipMemcpy(h.data(), ws.d_records.p, plan.n_tiles * sizeof(TileRecord),
                          hipMemcpyDeviceToHost));
        if (d_grp)
            HIP_TRY(hipMemcpy(hg.data(), d_grp, plan.n_tiles * sizeof(GroupRecord), hipMemcpyDeviceToHost));
    }
    *n_tiles = plan.n_tiles;
    for (uint64_t t = 0; t < plan.n_tiles && t < cap; ++t) {
        keys[t] = h[t].key;
        js[t] = h[t].j;
        if (gmax) gmax[t] = hg[t].max;
        if (ghot)
            for (int g = 0; g < kTileGroups; ++g) ghot[kTileGroups * t + g] = hg[t].hot[g];
    }
    return RC_OK;
}

int rc_timing_enable(rc_chunker *ch, int enable) {
    if (!ch) return fail(RC_ERR_ARGUMENT, "null chunker");
    ch->timing = enable != 0;
    return RC_OK;
}

int rc_timing_read_kernels(rc_chunker *ch, double *tile_ms, double *edge_ms, double *chain_ms,
                           uint64_t *calls) {
    if (!ch) return fail(RC_ERR_ARGUMENT, "null chunker");
    std::lock_guard<std::mutex> lock(ch->mu);
    DeviceGuard g(ch->device);
    double t[3] = {0, 0, 0};
    for (auto &r : ch->ev_rec) {
        HIP_TRY(hipEventSynchronize(r[3]));
        for (int k = 0; k < 3; ++k) {
            float x = 0;
            HIP_TRY(hipEventElapsedTime(&x, r[k], r[k + 1]));
            t[k] += x;
        }
        for (int k = 0; k < 4; ++k) (k == 1 ? ch->ev_pool_sync : ch->ev_pool).push_back(r[k]);
    }
    if (tile_ms) *tile_ms = t[0];
    if (edge_ms) *edge_ms = t[1];
    if (chain_ms) *chain_ms = t[2];
    if (calls) *calls = ch->ev_rec.size();
    ch->ev_rec.clear();
    return RC_OK;
}

int rc_timing_read(rc_chunker *ch, double *phase_a_ms, double *phase_b_ms, uint64_t *calls) {
    double tile = 0, edge = 0, chain = 0;
    if (int rc = rc_timing_read_kernels(ch, &tile, &edge, &chain, calls)) return rc;
    if (phase_a_ms) *phase_a_ms = tile + edge;
    if (phase_b_ms) *phase_b_ms = chain;
    return RC_OK;
}

int rc_read_probe(const uint8_t *d_src, uint64_t nbytes, uint32_t *d_out, void *hip_stream) {
    if (nbytes && (!d_src || !d_out)) return fail(RC_ERR_ARGUMENT, "null argument");
    if (reinterpret_cast<uintptr_t>(d_src) & 15) return fail(RC_ERR_ALIGN, "source not 16-byte aligned");
    // the tile kernel's schedule as a chunker created now would run it (the process's knobs)
    const Knobs &k = process_knobs();
    TileSched sched;
    sched.permille = (uint32_t)k[knTileStatic];
    sched.chunk = (uint32_t)k[knTileChunk];
    sched.dyn_min = (uint32_t)k[knTileDynMin];
    sched.group = (uint32_t)k[knTileGroup];
    if (rc_launch_read_probe(d_src, nbytes, d_out, (uint32_t)k[knProbeBlock], sched, hip_stream))
        return fail(RC_ERR_HIP, "%s", rc_launch_error());
    return RC_OK;
}

int rc_chunker_read_probe(rc_chunker *ch, const uint8_t *d_src, uint64_t nbytes, uint32_t *d_out,
                          void *hip_stream) {
    if (!ch) return fail(RC_ERR_ARGUMENT, "null chunker");
    if (nbytes && (!d_src || !d_out)) return fail(RC_ERR_ARGUMENT, "null argument");
    if (reinterpret_cast<uintptr_t>(d_src) & 15) return fail(RC_ERR_ALIGN, "source not 16-byte aligned");
    DeviceGuard g(ch->device);
    if (rc_launch_read_probe(d_src, nbytes, d_out, 0, ch->sched, hip_stream))
        return fail(RC_ERR_HIP, "%s", rc_launch_error());
    return RC_OK;
}

int rc_fill_splitmix(uint8_t *d_dst, uint64_t nbytes, uint64_t seed, uint64_t stream, void *hip_stream) {
    if (nbytes && !d_dst) return fail(RC_ERR_ARGUMENT, "null destination");
    if (rc_launch_fill(d_dst, nbytes, seed, stream, 0, hip_stream)) return fail(RC_ERR_HIP, "%s", rc_launch_error());
    return RC_OK;
}

int rc_fill_splitmix_streams(uint8_t *d_dst, uint64_t n, uint64_t nbytes, uint64_t slot,
                             uint64_t seed, uint64_t first_stream, uint64_t stream_step,
                             void *hip_stream) {
    if (n && nbytes && !d_dst) return fail(RC_ERR_ARGUMENT, "null destination");
    if (slot % 8 || slot < ((nbytes + 7) & ~7ull))
        return fail(RC_ERR_ARGUMENT, "slot %llu must be a multiple of 8 holding %llu bytes",
                    (unsigned long long)slot, (unsigned long long)nbytes);
    if (reinterpret_cast<uintptr_t>(d_dst) & 7) return fail(RC_ERR_ALIGN, "destination not 8-byte aligned");
    if (rc_launch_fill_streams(d_dst, n, nbytes, slot, seed, first_stream, stream_step, hip_stream))
        return fail(RC_ERR_HIP, "%s", rc_launch_error());
    return RC_OK;
}

int rc_fill_splitmix_at(uint8_t *d_dst, uint64_t nbytes, uint64_t seed, uint64_t stream,
                        uint64_t word0, void *hip_stream) {
    if (nbytes && !d_dst) return fail(RC_ERR_ARGUMENT, "null destination");
    if (rc_launch_fill(d_dst, nbytes, seed, stream, word0, hip_stream)) return fail(RC_ERR_HIP, "%s", rc_launch_error());
    return RC_OK;
}

}  // extern "C"
