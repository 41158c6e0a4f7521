// capi_digest.cpp -- host side of include/replicat_digest.h: BLAKE2b digests on the device.
//
// The hasher mirrors replicat's `blake2b(length)` hashing adapter (replicat/utils/adapters.py
// :195-225): its digest_size, and `digest(data)` = hashlib.blake2b(data, digest_size).digest()
// over many buffers per call.  Work lists are built here (buffers) or on the device (chunk
// lists left in HBM by rc_chunk_device), then blake2b.hip hashes them one quad of lanes per
// message.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <cstring>
#include <mutex>
#include <vector>

#include "capi_internal.h"
#include "knobs.h"
#include "digest_kernels.h"

static_assert(sizeof(rc_blake2b_state) == 256, "rc_blake2b_state is a 256-byte device record");

namespace {

struct DevMem {
    void *p = nullptr;
    size_t n = 0;
    int ensure(size_t bytes) {
        if (bytes <= n) return 0;
        if (p) {
            RC_HIP_TRY(hipDeviceSynchronize());
            RC_HIP_TRY(hipFree(p));
            p = nullptr;
            n = 0;
        }
        const size_t want = (std::max<size_t>(bytes, 4096) + 4095) & ~size_t(4095);
        RC_HIP_TRY(hipMalloc(&p, want));
        n = want;
        return 0;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
    }
};

struct PinnedMem {
    void *p = nullptr;
    size_t n = 0;
    int ensure(size_t bytes) {
        if (bytes <= n) return 0;
        if (p) RC_HIP_TRY(hipHostFree(p));
        p = nullptr;
        n = 0;
        RC_HIP_TRY(hipHostMalloc(&p, std::max<size_t>(bytes, 4096), hipHostMallocDefault));
        n = std::max<size_t>(bytes, 4096);
        return 0;
    }
    void release() {
        if (p) (void)hipHostFree(p);
        p = nullptr;
        n = 0;
    }
};

struct Guard {
    int prev = -1;
    explicit Guard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != dev) (void)hipSetDevice(dev);
    }
    ~Guard() {
        int cur = -1;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
    }
};

}  // namespace

struct rc_hasher {
    uint32_t digest_size = 64;
    int device = 0;
    rc::Knobs knobs;  // knobs.h, read once at creation (the lane / quad split)
    std::mutex mu;
    struct Workspace {
        PinnedMem h_stage;   // host-built descriptors / items
        DevMem d_stage;      // their device copy
        DevMem d_items;      // work list of the chunk path
        hipEvent_t done = nullptr;
        bool pending = false;
    } ws[2];
    unsigned next_ws = 0;
    // blocking host path
    DevMem d_data, d_out;
    // timing
    bool timing = false;
    std::vector<hipEvent_t> ev_pool;
    std::vector<std::array<hipEvent_t, 2>> ev_rec;
};

namespace {

using Workspace = rc_hasher::Workspace;

int acquire(rc_hasher *h, Workspace *&out) {
    Workspace &w = h->ws[h->next_ws++ & 1];
    if (w.pending) {  // its previous call must have consumed the staging
        RC_HIP_TRY(hipEventSynchronize(w.done));
        w.pending = false;
    }
    out = &w;
    return 0;
}

int timing_begin(rc_hasher *h, hipStream_t st, std::array<hipEvent_t, 2> &ev) {
    if (!h->timing) return 0;
    for (auto &e : ev) {
        if (h->ev_pool.empty()) {
            RC_HIP_TRY(hipEventCreate(&e));
        } else {
            e = h->ev_pool.back();
            h->ev_pool.pop_back();
        }
    }
    RC_HIP_TRY(hipEventRecord(ev[0], st));
    return 0;
}

int timing_end(rc_hasher *h, hipStream_t st, std::array<hipEvent_t, 2> &ev) {
    if (!h->timing) return 0;
    RC_HIP_TRY(hipEventRecord(ev[1], st));
    h->ev_rec.push_back(ev);
    return 0;
}

int finish(rc_hasher *h, Workspace &w, hipStream_t st) {
    RC_HIP_TRY(hipEventRecord(w.done, st));
    w.pending = true;
    (void)h;
    return 0;
}

// digest of n device buffers: items built on the host
int enqueue_items(rc_hasher *h, uint64_t n, const uint8_t *const *d_ptrs, const uint64_t *lens,
                  uint8_t *d_out, hipStream_t st) {
    Workspace *w = nullptr;
    if (int rc = acquire(h, w)) return rc;
    const size_t bytes = n * sizeof(B2Item);
    if (int rc = w->h_stage.ensure(bytes)) return rc;
    if (int rc = w->d_stage.ensure(bytes)) return rc;
    B2Item *it = static_cast<B2Item *>(w->h_stage.p);
    for (uint64_t i = 0; i < n; ++i) it[i] = B2Item{reinterpret_cast<uint64_t>(d_ptrs[i]), lens[i], i};
    // longest first: the kernel deals items round-robin (see blake2b.hip)
    std::stable_sort(it, it + n, [](const B2Item &x, const B2Item &y) { return x.len > y.len; });
    RC_HIP_TRY(hipMemcpyAsync(w->d_stage.p, w->h_stage.p, bytes, hipMemcpyHostToDevice, st));
    std::array<hipEvent_t, 2> ev{};
    if (int rc = timing_begin(h, st, ev)) return rc;
    uint64_t msg_bytes = 0;
    for (uint64_t i = 0; i < n; ++i) msg_bytes += lens[i];
    const uint64_t lane_max = rc_b2_lane_max(msg_bytes, it[0].len, h->knobs[rc::knB2LaneMax]);
    if (rc_b2_launch_items(static_cast<const B2Item *>(w->d_stage.p), n, h->digest_size, d_out,
                           lane_max, rc_b2_lane_only(lane_max, it[0].len, h->knobs[rc::knB2LaneOnly] == 1),
                           st))
        return rc_fail(RC_ERR_HIP, "%s", rc_b2_launch_error());
    if (int rc = timing_end(h, st, ev)) return rc;
    return finish(h, *w, st);
}

// incremental updates: items built on the host
int enqueue_update(rc_hasher *h, uint64_t n, rc_blake2b_state *const *d_states,
                   const uint8_t *const *d_ptrs, const uint64_t *lens, const uint8_t *finals,
                   uint8_t *d_out, hipStream_t st) {
    Workspace *w = nullptr;
    if (int rc = acquire(h, w)) return rc;
    const size_t bytes = n * sizeof(B2UItem);
    if (int rc = w->h_stage.ensure(bytes)) return rc;
    if (int rc = w->d_stage.ensure(bytes)) return rc;
    B2UItem *it = static_cast<B2UItem *>(w->h_stage.p);
    for (uint64_t i = 0; i < n; ++i)
        it[i] = B2UItem{reinterpret_cast<uint64_t>(d_ptrs[i]), lens[i], i,
                        reinterpret_cast<uint64_t>(d_states[i]), finals && finals[i] ? 1u : 0u, 0u};
    std::stable_sort(it, it + n, [](const B2UItem &x, const B2UItem &y) { return x.len > y.len; });
    RC_HIP_TRY(hipMemcpyAsync(w->d_stage.p, w->h_stage.p, bytes, hipMemcpyHostToDevice, st));
    std::array<hipEvent_t, 2> ev{};
    if (int rc = timing_begin(h, st, ev)) return rc;
    if (rc_b2_launch_update(static_cast<const B2UItem *>(w->d_stage.p), n, d_out, st))
        return rc_fail(RC_ERR_HIP, "%s", rc_b2_launch_error());
    if (int rc = timing_end(h, st, ev)) return rc;
    return finish(h, *w, st);
}

int check_buffers(uint64_t n, const uint8_t *const *ptrs, const uint64_t *lens) {
    if (n && (!ptrs || !lens)) return rc_fail(RC_ERR_ARGUMENT, "null buffer arrays");
    for (uint64_t i = 0; i < n; ++i)
        if (lens[i] && !ptrs[i])
            return rc_fail(RC_ERR_ARGUMENT, "buffer %llu: null pointer", (unsigned long long)i);
    return 0;
}

}  // namespace

int rc_hasher_enqueue_chunks(rc_hasher *h, uint64_t n, const uint8_t *const *d_ptrs,
                             const uint64_t *cut_base, const uint64_t *d_cuts,
                             const int64_t *d_counts, uint64_t total_cap, uint64_t bytes,
                             uint64_t longest, uint8_t *d_out, hipStream_t st) {
    if (!n) return 0;
    std::lock_guard<std::mutex> lock(h->mu);
    Guard g(h->device);
    Workspace *w = nullptr;
    if (int rc = acquire(h, w)) return rc;
    // staging: ptr[n] cut_base[n] | device also: chunk_off[n+1], the sort histogram
    const size_t up = 2 * n * sizeof(uint64_t);
    const size_t hist_off = up + (n + 1) * sizeof(uint64_t);
    if (int rc = w->h_stage.ensure(up)) return rc;
    if (int rc = w->d_stage.ensure(hist_off + rc_b2_hist_words(n) * sizeof(uint32_t))) return rc;
    if (int rc = w->d_items.ensure(std::max<uint64_t>(total_cap, 1) * sizeof(B2Item))) return rc;
    uint64_t *u = static_cast<uint64_t *>(w->h_stage.p);
    for (uint64_t i = 0; i < n; ++i) {
        u[i] = reinterpret_cast<uint64_t>(d_ptrs[i]);
        u[n + i] = cut_base[i];
    }
    RC_HIP_TRY(hipMemcpyAsync(w->d_stage.p, w->h_stage.p, up, hipMemcpyHostToDevice, st));
    const uint64_t *d = static_cast<const uint64_t *>(w->d_stage.p);
    uint64_t *chunk_off = static_cast<uint64_t *>(w->d_stage.p) + 2 * n;
    std::array<hipEvent_t, 2> ev{};
    if (int rc = timing_begin(h, st, ev)) return rc;
    uint32_t *hist = reinterpret_cast<uint32_t *>(static_cast<uint8_t *>(w->d_stage.p) + hist_off);
    const uint64_t lane_max = rc_b2_lane_max(bytes, longest, h->knobs[rc::knB2LaneMax]);
    if (rc_b2_launch_chunks(n, d, d + n, d_cuts, d_counts, chunk_off, hist,
                            static_cast<B2Item *>(w->d_items.p), total_cap, h->digest_size, d_out,
                            lane_max, rc_b2_lane_only(lane_max, longest, h->knobs[rc::knB2LaneOnly] == 1),
                            st))
        return rc_fail(RC_ERR_HIP, "%s", rc_b2_launch_error());
    if (int rc = timing_end(h, st, ev)) return rc;
    return finish(h, *w, st);
}

namespace {
thread_local char g_knob_err[256];
}

extern "C" {

int rc_blake2b_create(uint32_t digest_size, int device, rc_hasher **out) {
    if (!out) return rc_fail(RC_ERR_ARGUMENT, "null output handle");
    *out = nullptr;
    if (digest_size < 1 || digest_size > 64)
        return rc_fail(RC_ERR_DIGEST_SIZE, "digest_size must be between 1 and 64 bytes");
    rc::Knobs knobs;
    if (rc::read_knobs(knobs, g_knob_err, sizeof g_knob_err))
        return rc_fail(RC_ERR_ARGUMENT, "%s", g_knob_err);
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || device < 0 || device >= count)
        return rc_fail(RC_ERR_NO_DEVICE, "no HIP device %d", device);
    Guard g(device);
    rc_hasher *h = new rc_hasher;
    h->knobs = knobs;
    h->digest_size = digest_size;
    h->device = device;
    for (auto &w : h->ws) {
        const hipError_t e = hipEventCreateWithFlags(&w.done, hipEventDisableTiming);
        if (e != hipSuccess) {
            rc_blake2b_destroy(h);
            return rc_fail(RC_ERR_HIP, "hipEventCreate failed: %s", hipGetErrorString(e));
        }
    }
    rc_track(h, [](void *p) { rc_blake2b_destroy(static_cast<rc_hasher *>(p)); });
    *out = h;
    return RC_OK;
}

void rc_blake2b_destroy(rc_hasher *h) {
    if (!h) return;
    rc_untrack(h);
    {
        // a call still running on another thread (a daemon thread when the exit hook runs)
        // finishes first: its buffers and streams go only after it
        std::lock_guard<std::mutex> lock(h->mu);
        Guard g(h->device);
        (void)hipDeviceSynchronize();
        for (auto &w : h->ws) {
            w.h_stage.release();
            w.d_stage.release();
            w.d_items.release();
            if (w.done) (void)hipEventDestroy(w.done);
        }
        h->d_data.release();
        h->d_out.release();
        for (auto &r : h->ev_rec)
            for (auto e : r) (void)hipEventDestroy(e);
        for (auto e : h->ev_pool) (void)hipEventDestroy(e);
    }
    delete h;
}

uint32_t rc_blake2b_digest_size(const rc_hasher *h) { return h ? h->digest_size : 0; }

int rc_blake2b_device(rc_hasher *h, uint64_t n, const uint8_t *const *d_ptrs, const uint64_t *lens,
                      uint8_t *d_out, void *hip_stream) {
    if (!h) return rc_fail(RC_ERR_ARGUMENT, "null hasher");
    if (n == 0) return RC_OK;
    if (!d_out) return rc_fail(RC_ERR_ARGUMENT, "null output");
    if (int rc = check_buffers(n, d_ptrs, lens)) return rc;
    std::lock_guard<std::mutex> lock(h->mu);
    Guard g(h->device);
    return enqueue_items(h, n, d_ptrs, lens, d_out, static_cast<hipStream_t>(hip_stream));
}

int rc_blake2b_host(rc_hasher *h, uint64_t n, const uint8_t *const *ptrs, const uint64_t *lens,
                    uint8_t *out) {
    if (!h) return rc_fail(RC_ERR_ARGUMENT, "null hasher");
    if (n == 0) return RC_OK;
    if (!out) return rc_fail(RC_ERR_ARGUMENT, "null output");
    if (int rc = check_buffers(n, ptrs, lens)) return rc;
    std::lock_guard<std::mutex> lock(h->mu);
    Guard g(h->device);
    std::vector<uint64_t> off(n);
    uint64_t total = 0;
    for (uint64_t i = 0; i < n; ++i) {
        off[i] = total;
        total += (lens[i] + 15) & ~15ull;
    }
    if (int rc = h->d_data.ensure(total + 16)) return rc;
    if (int rc = h->d_out.ensure(n * kB2Slot)) return rc;
    std::vector<const uint8_t *> dp(n);
    uint8_t *base = static_cast<uint8_t *>(h->d_data.p);
    for (uint64_t i = 0; i < n; ++i) {
        dp[i] = base + off[i];
        if (lens[i]) RC_HIP_TRY(hipMemcpyAsync(base + off[i], ptrs[i], lens[i], hipMemcpyHostToDevice, nullptr));
    }
    if (int rc = enqueue_items(h, n, dp.data(), lens, static_cast<uint8_t *>(h->d_out.p), nullptr)) return rc;
    RC_HIP_TRY(hipMemcpyAsync(out, h->d_out.p, n * kB2Slot, hipMemcpyDeviceToHost, nullptr));
    RC_HIP_TRY(hipStreamSynchronize(nullptr));
    return RC_OK;
}

int rc_blake2b_chunks(rc_hasher *h, const rc_chunker *layout, uint64_t n,
                      const uint8_t *const *d_streams, const uint64_t *lens, const uint64_t *d_cuts,
                      const int64_t *d_counts, uint8_t *d_digests, void *hip_stream) {
    if (!h || !layout) return rc_fail(RC_ERR_ARGUMENT, "null hasher or chunker");
    if (n == 0) return RC_OK;
    if (!d_cuts || !d_counts || !d_digests) return rc_fail(RC_ERR_ARGUMENT, "null device arrays");
    if (int rc = check_buffers(n, d_streams, lens)) return rc;
    std::vector<uint64_t> caps(n), base(n);
    const uint64_t total = rc_cut_capacity(layout, n, lens, caps.data());
    uint64_t acc = 0;
    for (uint64_t i = 0; i < n; ++i) {
        base[i] = acc;
        acc += caps[i];
    }
    uint64_t bytes = 0, longest = 0;
    for (uint64_t i = 0; i < n; ++i) {
        bytes += lens[i];
        longest = std::max(longest, lens[i]);
    }
    if (const uint64_t m = rc_chunker_max_length(layout)) longest = std::min(longest, m);
    return rc_hasher_enqueue_chunks(h, n, d_streams, base.data(), d_cuts, d_counts, total, bytes,
                                    longest, d_digests, static_cast<hipStream_t>(hip_stream));
}

int rc_blake2b_state_init(uint32_t digest_size, const uint8_t *key, uint32_t keylen,
                          const uint8_t *salt, uint32_t saltlen, const uint8_t *person,
                          uint32_t personlen, rc_blake2b_state *out) {
    static const uint64_t iv[8] = {0x6a09e667f3bcc908ull, 0xbb67ae8584caa73bull,
                                   0x3c6ef372fe94f82bull, 0xa54ff53a5f1d36f1ull,
                                   0x510e527fade682d1ull, 0x9b05688c2b3e6c1full,
                                   0x1f83d9abfb41bd6bull, 0x5be0cd19137e2179ull};
    if (!out) return rc_fail(RC_ERR_ARGUMENT, "null state");
    if (digest_size < 1 || digest_size > 64)
        return rc_fail(RC_ERR_DIGEST_SIZE, "digest_size must be between 1 and 64 bytes");
    if (keylen > 64) return rc_fail(RC_ERR_B2_PARAM, "maximum key length is 64 bytes");
    if (saltlen > 16) return rc_fail(RC_ERR_B2_PARAM, "maximum salt length is 16 bytes");
    if (personlen > 16) return rc_fail(RC_ERR_B2_PARAM, "maximum person length is 16 bytes");
    if ((keylen && !key) || (saltlen && !salt) || (personlen && !person))
        return rc_fail(RC_ERR_ARGUMENT, "null key / salt / person");
    // parameter block (RFC 7693 §2.8): digest length, key length, fanout 1, depth 1; salt at
    // byte 32, personalisation at byte 48; everything else zero (sequential mode)
    uint8_t pb[64] = {};
    pb[0] = static_cast<uint8_t>(digest_size);
    pb[1] = static_cast<uint8_t>(keylen);
    pb[2] = 1;
    pb[3] = 1;
    if (saltlen) std::memcpy(pb + 32, salt, saltlen);
    if (personlen) std::memcpy(pb + 48, person, personlen);
    std::memset(out, 0, sizeof *out);
    for (int i = 0; i < 8; ++i) {
        uint64_t w;
        std::memcpy(&w, pb + 8 * i, 8);  // little-endian host (x86-64)
        out->h[i] = iv[i] ^ w;
    }
    out->digest_size = digest_size;
    if (keylen) {  // the key, zero-padded to a block, is the first (pending) block (§3.3)
        std::memcpy(out->buf, key, keylen);
        out->buflen = 128;
    }
    return RC_OK;
}

int rc_blake2b_update_device(rc_hasher *h, uint64_t n, rc_blake2b_state *const *d_states,
                             const uint8_t *const *d_ptrs, const uint64_t *lens,
                             const uint8_t *finals, uint8_t *d_out, void *hip_stream) {
    if (!h) return rc_fail(RC_ERR_ARGUMENT, "null hasher");
    if (n == 0) return RC_OK;
    if (!d_states) return rc_fail(RC_ERR_ARGUMENT, "null state array");
    if (int rc = check_buffers(n, d_ptrs, lens)) return rc;
    bool any_final = false;
    for (uint64_t i = 0; i < n; ++i) {
        if (!d_states[i] || (reinterpret_cast<uintptr_t>(d_states[i]) & 15))
            return rc_fail(RC_ERR_ARGUMENT, "state %llu: null or not 16-byte aligned",
                           (unsigned long long)i);
        any_final = any_final || (finals && finals[i]);
    }
    if (any_final && !d_out) return rc_fail(RC_ERR_ARGUMENT, "null output");
    std::lock_guard<std::mutex> lock(h->mu);
    Guard g(h->device);
    return enqueue_update(h, n, d_states, d_ptrs, lens, finals, d_out,
                          static_cast<hipStream_t>(hip_stream));
}

int rc_blake2b_derive_chunks(rc_hasher *h, const rc_chunker *layout, uint64_t n,
                             const uint64_t *lens, const int64_t *d_counts,
                             const rc_blake2b_state *d_kdf_state, const uint8_t *d_digests,
                             uint32_t msg_len, uint8_t *d_keys, void *hip_stream) {
    if (!h || !layout) return rc_fail(RC_ERR_ARGUMENT, "null hasher or chunker");
    if (n == 0) return RC_OK;
    if (!lens || !d_counts || !d_kdf_state || !d_digests || !d_keys)
        return rc_fail(RC_ERR_ARGUMENT, "null arrays");
    if (msg_len > kB2Slot) return rc_fail(RC_ERR_ARGUMENT, "msg_len above the 64-byte digest slot");
    if (reinterpret_cast<uintptr_t>(d_kdf_state) & 15)
        return rc_fail(RC_ERR_ARGUMENT, "KDF state not 16-byte aligned");
    std::vector<uint64_t> caps(n);
    rc_cut_capacity(layout, n, lens, caps.data());
    std::lock_guard<std::mutex> lock(h->mu);
    Guard g(h->device);
    const hipStream_t st = static_cast<hipStream_t>(hip_stream);
    Workspace *w = nullptr;
    if (int rc = acquire(h, w)) return rc;
    const size_t bytes = n * sizeof(uint64_t);
    if (int rc = w->h_stage.ensure(bytes)) return rc;
    if (int rc = w->d_stage.ensure(bytes)) return rc;
    uint64_t *u = static_cast<uint64_t *>(w->h_stage.p);
    uint64_t acc = 0;
    for (uint64_t i = 0; i < n; ++i) {
        u[i] = acc;
        acc += caps[i];
    }
    RC_HIP_TRY(hipMemcpyAsync(w->d_stage.p, u, bytes, hipMemcpyHostToDevice, st));
    std::array<hipEvent_t, 2> ev{};
    if (int rc = timing_begin(h, st, ev)) return rc;
    if (rc_b2_launch_derive(n, static_cast<const uint64_t *>(w->d_stage.p), d_counts, d_kdf_state,
                            d_digests, msg_len, d_keys, st))
        return rc_fail(RC_ERR_HIP, "%s", rc_b2_launch_error());
    if (int rc = timing_end(h, st, ev)) return rc;
    return finish(h, *w, st);
}

int rc_blake2b_timing_enable(rc_hasher *h, int enable) {
    if (!h) return rc_fail(RC_ERR_ARGUMENT, "null hasher");
    h->timing = enable != 0;
    return RC_OK;
}

int rc_blake2b_timing_read(rc_hasher *h, double *ms, uint64_t *calls) {
    if (!h) return rc_fail(RC_ERR_ARGUMENT, "null hasher");
    std::lock_guard<std::mutex> lock(h->mu);
    Guard g(h->device);
    double a = 0;
    for (auto &r : h->ev_rec) {
        RC_HIP_TRY(hipEventSynchronize(r[1]));
        float x = 0;
        RC_HIP_TRY(hipEventElapsedTime(&x, r[0], r[1]));
        a += x;
        for (auto e : r) h->ev_pool.push_back(e);
    }
    if (ms) *ms = a;
    if (calls) *calls = h->ev_rec.size();
    h->ev_rec.clear();
    return RC_OK;
}

}  // extern "C"
