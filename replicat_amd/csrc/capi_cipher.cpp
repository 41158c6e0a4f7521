// capi_cipher.cpp -- host side of include/replicat_cipher.h: AES-GCM on the device.
//
// A handle mirrors replicat's `aes_gcm(key_bits, nonce_bits)` cipher adapter
// (replicat/utils/adapters.py:117-158): encrypt = nonce || C || T, decrypt with the tag check.
// Work lists are built here (buffers) or on the device (the chunk lists rc_chunk_device left in
// HBM); gcm.hip runs them one workgroup per message.  The constant tables the kernel stages into
// LDS -- the AES T0 table and the GF(2^128) squaring table -- are computed here per handle.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <vector>

#include "../../include/replicat_cipher.h"
#include "capi_internal.h"
#include "knobs.h"
#include "cipher_kernels.h"
#include "digest_kernels.h"

static_assert(sizeof(GcmItem) == 48, "GcmItem is a 48-byte device record");

namespace {

// RC_GCM_DEBUG=1 (knobs.h): every host step of a call is stamped on stderr (hang diagnosis)
bool debug_on() { return rc::process_knobs()[rc::knGcmDebug] != 0; }
#define GCM_DBG(...)                                      \
    do {                                                  \
        if (debug_on()) {                                 \
            std::fprintf(stderr, "rc_gcm: " __VA_ARGS__); \
            std::fputc('\n', stderr);                     \
            std::fflush(stderr);                          \
        }                                                 \
    } while (0)

struct DevBuf {
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
        GCM_DBG("hipMalloc %zu", want);
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

// Staging memory: pinned when the runtime grants it, else pageable (copies from pageable memory
// are synchronous, which every user of these buffers tolerates).
struct HostBuf {
    void *p = nullptr;
    size_t n = 0;
    bool pinned = false;
    int ensure(size_t bytes) {
        if (bytes <= n) return 0;
        release();
        const size_t want = std::max<size_t>(bytes, 4096);
        GCM_DBG("hipHostMalloc %zu", want);
        if (hipHostMalloc(&p, want, hipHostMallocDefault) == hipSuccess) {
            pinned = true;
        } else {
            GCM_DBG("hipHostMalloc refused: pageable staging");
            (void)hipGetLastError();  // clear the failed allocation's status
            p = std::malloc(want);
            pinned = false;
            if (!p) return rc_fail(RC_ERR_HIP, "host staging: %zu bytes unavailable", want);
        }
        n = want;
        return 0;
    }
    void release() {
        if (p) {
            if (pinned)
                (void)hipHostFree(p);
            else
                std::free(p);
        }
        p = nullptr;
        n = 0;
    }
};

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

uint64_t up16(uint64_t x) { return (x + 15) & ~uint64_t(15); }
uint64_t addr(const void *p) { return reinterpret_cast<uint64_t>(p); }

// ------------------------------------------------------------------ constant tables

uint8_t xt(uint8_t a) { return static_cast<uint8_t>((a << 1) ^ ((a & 0x80) ? 0x1B : 0)); }
uint8_t gm(uint8_t a, uint8_t b) {
    uint8_t p = 0;
    for (; b; b >>= 1, a = xt(a))
        if (b & 1) p ^= a;
    return p;
}

// FIPS 197 S-box (§5.1.1: inverse in GF(2^8), then the affine map) and T0[x] = {2s, s, s, 3s}:
// the first column of MixColumns applied to s = S[x], as a little-endian word
void make_te0(uint32_t *te0) {
    uint8_t inv[256] = {0};
    for (int x = 1; x < 256; ++x)
        for (int c = 1; c < 256; ++c)
            if (gm(static_cast<uint8_t>(x), static_cast<uint8_t>(c)) == 1) {
                inv[x] = static_cast<uint8_t>(c);
                break;
            }
    for (int x = 0; x < 256; ++x) {
        const uint8_t b = inv[x];
        uint8_t s = b;
        for (int i = 1; i <= 4; ++i) s ^= static_cast<uint8_t>((b << i) | (b >> (8 - i)));
        s ^= 0x63;
        te0[x] = uint32_t(gm(s, 2)) | (uint32_t(s) << 8) | (uint32_t(s) << 16) | (uint32_t(gm(s, 3)) << 24);
    }
}

// SP 800-38D §6.3 product; bit 0 = the MSB of byte 0
void gf_mul(const uint8_t *X, const uint8_t *Y, uint8_t *Z) {
    uint8_t V[16], acc[16] = {0};
    std::memcpy(V, Y, 16);
    for (int i = 0; i < 128; ++i) {
        if (X[i / 8] & (0x80 >> (i % 8)))
            for (int j = 0; j < 16; ++j) acc[j] ^= V[j];
        const int lsb = V[15] & 1;
        for (int j = 15; j > 0; --j) V[j] = static_cast<uint8_t>((V[j] >> 1) | (V[j - 1] << 7));
        V[0] >>= 1;
        if (lsb) V[0] ^= 0xE1;
    }
    std::memcpy(Z, acc, 16);
}

// Squaring is GF(2)-linear: entry (j, v) = E(j, v)^2 for the element whose nibble j (the high
// nibble of byte j / 2 for even j, the low one for odd j) is v; bytes in memory order.
void make_sq(uint32_t *sq) {
    for (int j = 0; j < 32; ++j)
        for (int v = 0; v < 16; ++v) {
            uint8_t e[16] = {0}, z[16];
            e[j / 2] = static_cast<uint8_t>(j & 1 ? v : v << 4);
            gf_mul(e, e, z);
            std::memcpy(sq + 4 * (16 * j + v), z, 16);
        }
}

constexpr size_t kTe0Words = 256, kSqWords = 2048;

}  // namespace

struct rc_gcm {
    uint32_t key_bytes = 32, nonce_bytes = 12;
    int device = 0;
    std::mutex mu;
    DevBuf d_consts;  // te0 | sq
    struct Workspace {
        HostBuf h_stage;  // [header 16 B] [host-built staging]
        DevBuf d_stage;   // its device copy (+ device-built lists)
        hipEvent_t done = nullptr;
        bool pending = false;
    } ws[2];
    unsigned next_ws = 0;
    // blocking host paths
    HostBuf h_in, h_out;
    DevBuf d_in, d_out, d_ok;
    // timing
    bool timing = false;
    std::vector<hipEvent_t> ev_pool;
    std::vector<std::array<hipEvent_t, 2>> ev_rec;
};

namespace {

using Workspace = rc_gcm::Workspace;

int acquire(rc_gcm *g, Workspace *&out) {
    Workspace &w = g->ws[g->next_ws++ & 1];
    if (w.pending) {  // its previous call must have consumed the staging
        GCM_DBG("wait for workspace %u", (g->next_ws - 1) & 1);
        RC_HIP_TRY(hipEventSynchronize(w.done));
        w.pending = false;
    }
    out = &w;
    return 0;
}

int timing_begin(rc_gcm *g, hipStream_t st, std::array<hipEvent_t, 2> &ev) {
    if (!g->timing) return 0;
    for (auto &e : ev) {
        if (g->ev_pool.empty()) {
            RC_HIP_TRY(hipEventCreate(&e));
        } else {
            e = g->ev_pool.back();
            g->ev_pool.pop_back();
        }
    }
    RC_HIP_TRY(hipEventRecord(ev[0], st));
    return 0;
}

int timing_end(rc_gcm *g, hipStream_t st, std::array<hipEvent_t, 2> &ev) {
    if (!g->timing) return 0;
    RC_HIP_TRY(hipEventRecord(ev[1], st));
    g->ev_rec.push_back(ev);
    return 0;
}

int finish(Workspace &w, hipStream_t st) {
    RC_HIP_TRY(hipEventRecord(w.done, st));
    w.pending = true;
    return 0;
}

GcmArgs base_args(const rc_gcm *g) {
    GcmArgs a{};
    a.te0 = static_cast<const uint32_t *>(g->d_consts.p);
    a.sq = a.te0 + kTe0Words;
    a.nonce_bytes = g->nonce_bytes;
    return a;
}

// n host-built items, longest first (the kernel hands them out in list order)
int enqueue_items(rc_gcm *g, bool dec, std::vector<GcmItem> &items, uint8_t *d_ok, hipStream_t st) {
    const uint64_t n = items.size();
    if (!n) return 0;
    std::stable_sort(items.begin(), items.end(),
                     [](const GcmItem &x, const GcmItem &y) { return x.len > y.len; });
    Workspace *w = nullptr;
    if (int rc = acquire(g, w)) return rc;
    const size_t bytes = 16 + n * sizeof(GcmItem);
    if (int rc = w->h_stage.ensure(bytes)) return rc;
    if (int rc = w->d_stage.ensure(bytes)) return rc;
    uint8_t *h = static_cast<uint8_t *>(w->h_stage.p);
    std::memset(h, 0, 16);  // header (reserved)
    std::memcpy(h + 16, items.data(), n * sizeof(GcmItem));
    RC_HIP_TRY(hipMemcpyAsync(w->d_stage.p, h, bytes, hipMemcpyHostToDevice, st));
    uint8_t *d = static_cast<uint8_t *>(w->d_stage.p);
    GcmArgs a = base_args(g);
    a.items = reinterpret_cast<const GcmItem *>(d + 16);
    a.ok = d_ok;
    std::array<hipEvent_t, 2> ev{};
    if (int rc = timing_begin(g, st, ev)) return rc;
    if (n > 0x7FFFFFFFull) return rc_fail(RC_ERR_ARGUMENT, "%llu messages in one call", (unsigned long long)n);
    const unsigned groups = static_cast<unsigned>(n);
    GCM_DBG("launch %s n=%llu groups=%u", dec ? "decrypt" : "encrypt", (unsigned long long)n, groups);
    if (rc_gcm_launch(g->key_bytes, dec, a, groups, st))
        return rc_fail(RC_ERR_HIP, "%s", rc_gcm_launch_error());
    if (int rc = timing_end(g, st, ev)) return rc;
    return finish(*w, st);
}

int check_handle(const rc_gcm *g) { return g ? 0 : rc_fail(RC_ERR_ARGUMENT, "null cipher"); }

}  // namespace

extern "C" {

int rc_gcm_create(uint32_t key_bits, uint32_t nonce_bits, int device, rc_gcm **out) {
    if (!out) return rc_fail(RC_ERR_ARGUMENT, "null output handle");
    *out = nullptr;
    if (key_bits != 128 && key_bits != 192 && key_bits != 256)
        return rc_fail(RC_ERR_KEY_SIZE, "Invalid key size");
    const uint32_t nonce_bytes = nonce_bits / 8;
    if (nonce_bytes < 8 || nonce_bytes > 128)
        return rc_fail(RC_ERR_NONCE_SIZE, "Nonce must be between 8 and 128 bytes");
    {  // the environment knobs (knobs.h): a malformed one fails every handle's creation
        rc::Knobs knobs;
        char err[256];
        if (rc::read_knobs(knobs, err, sizeof err)) return rc_fail(RC_ERR_ARGUMENT, "%s", err);
    }
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || device < 0 || device >= count)
        return rc_fail(RC_ERR_NO_DEVICE, "no HIP device %d", device);
    DeviceGuard guard(device);
    rc_gcm *g = new rc_gcm;
    g->key_bytes = key_bits / 8;
    g->nonce_bytes = nonce_bytes;
    g->device = device;
    std::vector<uint32_t> consts(kTe0Words + kSqWords);
    make_te0(consts.data());
    make_sq(consts.data() + kTe0Words);
    int rc = g->d_consts.ensure(consts.size() * sizeof(uint32_t));
    if (!rc) {
        const hipError_t e = hipMemcpy(g->d_consts.p, consts.data(), consts.size() * sizeof(uint32_t),
                                       hipMemcpyHostToDevice);
        if (e != hipSuccess) rc = rc_fail(RC_ERR_HIP, "hipMemcpy failed: %s", hipGetErrorString(e));
    }
    for (auto &w : g->ws) {
        if (rc) break;
        const hipError_t e = hipEventCreateWithFlags(&w.done, hipEventDisableTiming);
        if (e != hipSuccess) rc = rc_fail(RC_ERR_HIP, "hipEventCreate failed: %s", hipGetErrorString(e));
    }
    if (rc) {
        rc_gcm_destroy(g);
        return rc;
    }
    rc_track(g, [](void *p) { rc_gcm_destroy(static_cast<rc_gcm *>(p)); });
    *out = g;
    return RC_OK;
}

void rc_gcm_destroy(rc_gcm *g) {
    if (!g) return;
    rc_untrack(g);
    {
        // a call still running on another thread (a daemon thread when the exit hook runs)
        // finishes first: its buffers and streams go only after it
        std::lock_guard<std::mutex> lock(g->mu);
        DeviceGuard guard(g->device);
        (void)hipDeviceSynchronize();
        for (auto &w : g->ws) {
            w.h_stage.release();
            w.d_stage.release();
            if (w.done) (void)hipEventDestroy(w.done);
        }
        g->d_consts.release();
        g->h_in.release();
        g->h_out.release();
        g->d_in.release();
        g->d_out.release();
        g->d_ok.release();
        for (auto &r : g->ev_rec)
            for (auto e : r) (void)hipEventDestroy(e);
        for (auto e : g->ev_pool) (void)hipEventDestroy(e);
    }
    delete g;
}

uint32_t rc_gcm_key_bytes(const rc_gcm *g) { return g ? g->key_bytes : 0; }
uint32_t rc_gcm_nonce_bytes(const rc_gcm *g) { return g ? g->nonce_bytes : 0; }

int rc_gcm_encrypt_device(rc_gcm *g, uint64_t n, const uint8_t *const *d_in, const uint64_t *lens,
                          const uint8_t *const *d_keys, const uint8_t *const *d_nonces,
                          uint8_t *const *d_out, void *hip_stream) {
    if (int rc = check_handle(g)) return rc;
    if (n == 0) return RC_OK;
    if (!d_in || !lens || !d_keys || !d_nonces || !d_out) return rc_fail(RC_ERR_ARGUMENT, "null arrays");
    std::vector<GcmItem> items(n);
    for (uint64_t i = 0; i < n; ++i) {
        if ((lens[i] && !d_in[i]) || !d_keys[i] || !d_nonces[i] || !d_out[i])
            return rc_fail(RC_ERR_ARGUMENT, "item %llu: null pointer", (unsigned long long)i);
        items[i] = GcmItem{addr(d_in[i]), lens[i], addr(d_out[i]), addr(d_keys[i]), addr(d_nonces[i]), i};
    }
    std::lock_guard<std::mutex> lock(g->mu);
    DeviceGuard guard(g->device);
    return enqueue_items(g, false, items, nullptr, static_cast<hipStream_t>(hip_stream));
}

int rc_gcm_decrypt_device(rc_gcm *g, uint64_t n, const uint8_t *const *d_in, const uint64_t *lens,
                          const uint8_t *const *d_keys, uint8_t *const *d_out, uint8_t *d_ok,
                          void *hip_stream) {
    if (int rc = check_handle(g)) return rc;
    if (n == 0) return RC_OK;
    if (!d_in || !lens || !d_keys || !d_out || !d_ok) return rc_fail(RC_ERR_ARGUMENT, "null arrays");
    const uint64_t over = g->nonce_bytes + 16;
    std::vector<GcmItem> items;
    items.reserve(n);
    for (uint64_t i = 0; i < n; ++i) {
        if (lens[i] < over) continue;  // too short to hold nonce and tag: ok stays 0 (InvalidTag)
        const uint64_t len = lens[i] - over;
        if (!d_in[i] || !d_keys[i] || (len && !d_out[i]))
            return rc_fail(RC_ERR_ARGUMENT, "item %llu: null pointer", (unsigned long long)i);
        items.push_back(GcmItem{addr(d_in[i]), len, addr(d_out[i]), addr(d_keys[i]), 0, i});
    }
    std::lock_guard<std::mutex> lock(g->mu);
    DeviceGuard guard(g->device);
    const hipStream_t st = static_cast<hipStream_t>(hip_stream);
    RC_HIP_TRY(hipMemsetAsync(d_ok, 0, n, st));
    return enqueue_items(g, true, items, d_ok, st);
}

int rc_gcm_encrypt_host(rc_gcm *g, uint64_t n, const uint8_t *const *in, const uint64_t *lens,
                        const uint8_t *const *keys, const uint8_t *const *nonces, uint8_t *const *out) {
    if (int rc = check_handle(g)) return rc;
    if (n == 0) return RC_OK;
    if (!in || !lens || !keys || !nonces || !out) return rc_fail(RC_ERR_ARGUMENT, "null arrays");
    for (uint64_t i = 0; i < n; ++i)
        if ((lens[i] && !in[i]) || !keys[i] || !nonces[i] || !out[i])
            return rc_fail(RC_ERR_ARGUMENT, "item %llu: null pointer", (unsigned long long)i);
    std::lock_guard<std::mutex> lock(g->mu);
    DeviceGuard guard(g->device);
    const uint64_t kb = g->key_bytes, nb = g->nonce_bytes;
    // input image: messages (16-aligned) | keys (64 B each) | nonces (128 B each)
    std::vector<uint64_t> in_off(n), out_off(n);
    uint64_t a = 0, b = 0;
    for (uint64_t i = 0; i < n; ++i) {
        in_off[i] = a;
        a += up16(lens[i]);
        out_off[i] = b;
        b += up16(nb + lens[i] + 16);
    }
    const uint64_t key_off = a, nonce_off = a + 64 * n, in_total = nonce_off + 128 * n;
    if (int rc = g->h_in.ensure(in_total)) return rc;
    if (int rc = g->d_in.ensure(in_total)) return rc;
    if (int rc = g->h_out.ensure(b)) return rc;
    if (int rc = g->d_out.ensure(b)) return rc;
    uint8_t *hi = static_cast<uint8_t *>(g->h_in.p), *ho = static_cast<uint8_t *>(g->h_out.p);
    for (uint64_t i = 0; i < n; ++i) {
        if (lens[i]) std::memcpy(hi + in_off[i], in[i], lens[i]);
        std::memcpy(hi + key_off + 64 * i, keys[i], kb);
        std::memcpy(hi + nonce_off + 128 * i, nonces[i], nb);
    }
    GCM_DBG("encrypt_host: upload %llu bytes", (unsigned long long)in_total);
    RC_HIP_TRY(hipMemcpyAsync(g->d_in.p, hi, in_total, hipMemcpyHostToDevice, nullptr));
    const uint64_t D = addr(g->d_in.p), O = addr(g->d_out.p);
    std::vector<GcmItem> items(n);
    for (uint64_t i = 0; i < n; ++i)
        items[i] = GcmItem{D + in_off[i], lens[i], O + out_off[i], D + key_off + 64 * i,
                           D + nonce_off + 128 * i, i};
    if (int rc = enqueue_items(g, false, items, nullptr, nullptr)) return rc;
    GCM_DBG("encrypt_host: download %llu bytes", (unsigned long long)b);
    RC_HIP_TRY(hipMemcpyAsync(ho, g->d_out.p, b, hipMemcpyDeviceToHost, nullptr));
    GCM_DBG("encrypt_host: synchronize");
    RC_HIP_TRY(hipStreamSynchronize(nullptr));
    GCM_DBG("encrypt_host: done");
    for (uint64_t i = 0; i < n; ++i) std::memcpy(out[i], ho + out_off[i], nb + lens[i] + 16);
    return RC_OK;
}

int rc_gcm_decrypt_host(rc_gcm *g, uint64_t n, const uint8_t *const *in, const uint64_t *lens,
                        const uint8_t *const *keys, uint8_t *const *out, uint8_t *ok) {
    if (int rc = check_handle(g)) return rc;
    if (n == 0) return RC_OK;
    if (!in || !lens || !keys || !out || !ok) return rc_fail(RC_ERR_ARGUMENT, "null arrays");
    std::lock_guard<std::mutex> lock(g->mu);
    DeviceGuard guard(g->device);
    const uint64_t kb = g->key_bytes, over = g->nonce_bytes + 16;
    std::vector<uint64_t> in_off(n), out_off(n);
    uint64_t a = 0, b = 0;
    for (uint64_t i = 0; i < n; ++i) {
        if ((lens[i] && !in[i]) || !keys[i] || (lens[i] > over && !out[i]))
            return rc_fail(RC_ERR_ARGUMENT, "item %llu: null pointer", (unsigned long long)i);
        in_off[i] = a;
        a += up16(lens[i]);
        out_off[i] = b;
        b += up16(lens[i] >= over ? lens[i] - over : 0);
    }
    const uint64_t key_off = a, in_total = a + 64 * n;
    if (int rc = g->h_in.ensure(in_total)) return rc;
    if (int rc = g->d_in.ensure(in_total)) return rc;
    if (int rc = g->h_out.ensure(b + 16)) return rc;
    if (int rc = g->d_out.ensure(b + 16)) return rc;
    if (int rc = g->d_ok.ensure(n)) return rc;
    uint8_t *hi = static_cast<uint8_t *>(g->h_in.p), *ho = static_cast<uint8_t *>(g->h_out.p);
    for (uint64_t i = 0; i < n; ++i) {
        if (lens[i]) std::memcpy(hi + in_off[i], in[i], lens[i]);
        std::memcpy(hi + key_off + 64 * i, keys[i], kb);
    }
    const hipStream_t st = nullptr;
    RC_HIP_TRY(hipMemcpyAsync(g->d_in.p, hi, in_total, hipMemcpyHostToDevice, st));
    uint8_t *d_ok = static_cast<uint8_t *>(g->d_ok.p);
    RC_HIP_TRY(hipMemsetAsync(d_ok, 0, n, st));
    const uint64_t D = addr(g->d_in.p), O = addr(g->d_out.p);
    std::vector<GcmItem> items;
    items.reserve(n);
    for (uint64_t i = 0; i < n; ++i)
        if (lens[i] >= over)
            items.push_back(GcmItem{D + in_off[i], lens[i] - over, O + out_off[i], D + key_off + 64 * i, 0, i});
    if (int rc = enqueue_items(g, true, items, d_ok, st)) return rc;
    if (b) RC_HIP_TRY(hipMemcpyAsync(ho, g->d_out.p, b, hipMemcpyDeviceToHost, st));
    RC_HIP_TRY(hipMemcpyAsync(ok, d_ok, n, hipMemcpyDeviceToHost, st));
    RC_HIP_TRY(hipStreamSynchronize(st));
    bool all = true;
    for (uint64_t i = 0; i < n; ++i) {
        if (lens[i] > over) std::memcpy(out[i], ho + out_off[i], lens[i] - over);
        all = all && ok[i];
    }
    return all ? RC_OK : rc_fail(RC_ERR_TAG, "tag mismatch (InvalidTag)");
}

uint64_t rc_gcm_chunks_layout(const rc_gcm *g, const rc_chunker *layout, uint64_t n,
                              const uint64_t *lens, uint64_t *out_base) {
    if (!g || !layout || !lens || !n) return 0;
    std::vector<uint64_t> caps(n);
    rc_cut_capacity(layout, n, lens, caps.data());
    const uint64_t over = g->nonce_bytes + 16;
    uint64_t acc = 0;
    for (uint64_t i = 0; i < n; ++i) {
        if (out_base) out_base[i] = acc;
        acc = up16(acc + lens[i] + caps[i] * over);  // 16-aligned regions keep the fast path
    }
    return acc;
}

int rc_gcm_encrypt_chunks(rc_gcm *g, const rc_chunker *layout, uint64_t n,
                          const uint8_t *const *d_streams, const uint64_t *lens,
                          const uint64_t *d_cuts, const int64_t *d_counts, const uint8_t *d_keys,
                          const uint8_t *d_nonces, uint8_t *d_out, void *hip_stream) {
    if (!g || !layout) return rc_fail(RC_ERR_ARGUMENT, "null cipher or chunker");
    if (n == 0) return RC_OK;
    if (!d_streams || !lens || !d_cuts || !d_counts || !d_keys || !d_nonces || !d_out)
        return rc_fail(RC_ERR_ARGUMENT, "null arrays");
    for (uint64_t i = 0; i < n; ++i)
        if (lens[i] && !d_streams[i])
            return rc_fail(RC_ERR_ARGUMENT, "stream %llu: null pointer", (unsigned long long)i);
    std::vector<uint64_t> caps(n), out_base(n);
    const uint64_t total_cap = rc_cut_capacity(layout, n, lens, caps.data());
    rc_gcm_chunks_layout(g, layout, n, lens, out_base.data());
    std::lock_guard<std::mutex> lock(g->mu);
    DeviceGuard guard(g->device);
    const hipStream_t st = static_cast<hipStream_t>(hip_stream);
    Workspace *w = nullptr;
    if (int rc = acquire(g, w)) return rc;
    // staging: [header 16 B] ptrs[n] cut_base[n] out_base[n] | device only: chunk_off[n + 1], items
    const size_t up = 16 + 3 * n * sizeof(uint64_t);
    const size_t items_off = up16(up + (n + 1) * sizeof(uint64_t));
    if (int rc = w->h_stage.ensure(up)) return rc;
    if (int rc = w->d_stage.ensure(items_off + std::max<uint64_t>(total_cap, 1) * sizeof(GcmItem))) return rc;
    uint8_t *h = static_cast<uint8_t *>(w->h_stage.p);
    std::memset(h, 0, 16);
    uint64_t *u = reinterpret_cast<uint64_t *>(h + 16);
    uint64_t acc = 0;
    for (uint64_t i = 0; i < n; ++i) {
        u[i] = addr(d_streams[i]);
        u[n + i] = acc;
        acc += caps[i];
        u[2 * n + i] = out_base[i];
    }
    RC_HIP_TRY(hipMemcpyAsync(w->d_stage.p, h, up, hipMemcpyHostToDevice, st));
    uint8_t *d = static_cast<uint8_t *>(w->d_stage.p);
    const uint64_t *du = reinterpret_cast<const uint64_t *>(d + 16);
    uint64_t *chunk_off = reinterpret_cast<uint64_t *>(d + up);
    GcmItem *items = reinterpret_cast<GcmItem *>(d + items_off);
    std::array<hipEvent_t, 2> ev{};
    if (int rc = timing_begin(g, st, ev)) return rc;
    if (rc_b2_launch_scan(d_counts, n, chunk_off, st)) return rc_fail(RC_ERR_HIP, "%s", rc_b2_launch_error());
    GcmChunkLists c{};
    c.ptrs = du;
    c.cut_base = du + n;
    c.out_base = du + 2 * n;
    c.cuts = d_cuts;
    c.chunk_off = chunk_off;
    c.counts = d_counts;
    c.n = n;
    c.spw = rc_b2_streams_per_group(n);
    c.keys = addr(d_keys);
    c.nonces = addr(d_nonces);
    c.out = addr(d_out);
    c.nonce_bytes = g->nonce_bytes;
    if (rc_gcm_launch_chunk_items(c, items, st)) return rc_fail(RC_ERR_HIP, "%s", rc_gcm_launch_error());
    GcmArgs a = base_args(g);
    a.items = items;
    a.d_total = chunk_off + n;
    if (total_cap > 0x7FFFFFFFull)
        return rc_fail(RC_ERR_ARGUMENT, "%llu chunk slots in one call", (unsigned long long)total_cap);
    const unsigned groups = static_cast<unsigned>(std::max<uint64_t>(total_cap, 1));
    if (rc_gcm_launch(g->key_bytes, false, a, groups, st))
        return rc_fail(RC_ERR_HIP, "%s", rc_gcm_launch_error());
    if (int rc = timing_end(g, st, ev)) return rc;
    return finish(*w, st);
}

int rc_gcm_timing_enable(rc_gcm *g, int enable) {
    if (int rc = check_handle(g)) return rc;
    g->timing = enable != 0;
    return RC_OK;
}

int rc_gcm_timing_read(rc_gcm *g, double *ms, uint64_t *calls) {
    if (int rc = check_handle(g)) return rc;
    std::lock_guard<std::mutex> lock(g->mu);
    DeviceGuard guard(g->device);
    double t = 0;
    for (auto &r : g->ev_rec) {
        RC_HIP_TRY(hipEventSynchronize(r[1]));
        float x = 0;
        RC_HIP_TRY(hipEventElapsedTime(&x, r[0], r[1]));
        t += x;
        for (auto e : r) g->ev_pool.push_back(e);
    }
    if (ms) *ms = t;
    if (calls) *calls = g->ev_rec.size();
    g->ev_rec.clear();
    return RC_OK;
}

}  // extern "C"
