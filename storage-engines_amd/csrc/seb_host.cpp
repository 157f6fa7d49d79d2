// seb_host.cpp — the C ABI (include/seb_bloom.h): device-resident entry points, host-buffer
// batched entry points with a chunked H2D -> kernel -> D2H pipeline, and the handle API that
// mirrors lsm/bloom.go method for method.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cctype>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/seb_bloom.h"
#include "seb_kernels.h"

namespace seb {
int params(int64_t n, double p, uint64_t *m_out, uint32_t *k_out);
}

using namespace seb;

// ------------------------------------------------------------------ errors ------------------

static thread_local std::string t_err;

static int fail(int code, const char *fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    t_err = buf;
    return code;
}

// The status a failed HIP call maps to.  Only genuine unavailability is SEB_ERR_DEVICE (no device,
// no driver, no code object for it, a runtime that is not up) and only an allocation failure is
// SEB_ERR_NOMEM: those two are what the Go API mirror's CPU fallback absorbs.  Everything else (a
// rejected launch, parameters the library computed wrong, a kernel fault) is SEB_ERR_INTERNAL,
// which is reported and never absorbed, so a library bug cannot hide behind the fallback.
static int hip_status(hipError_t e) {
    switch (e) {
    case hipErrorOutOfMemory:
        return SEB_ERR_NOMEM;
    case hipErrorNoDevice:
    case hipErrorInvalidDevice:
    case hipErrorInsufficientDriver:
    case hipErrorNoBinaryForGpu:
    case hipErrorNotInitialized:
    case hipErrorDeinitialized:
        return SEB_ERR_DEVICE;
    default:
        return SEB_ERR_INTERNAL;
    }
}

// A failed HIP call is reported through the return code, and HIP's last-error state is cleared so
// it does not surface again in the caller's own later checks (torch's hipGetLastError, say).
#define HIP_OR_FAIL(expr)                                                                              \
    do {                                                                                               \
        hipError_t e_ = (expr);                                                                        \
        if (e_ != hipSuccess) {                                                                        \
            (void)hipGetLastError();                                                                   \
            return fail(hip_status(e_), "%s: %s", #expr, hipGetErrorString(e_));                       \
        }                                                                                              \
    } while (0)

// Makes `device` current for one call and restores the caller's device when it returns.
struct DeviceGuard {
    int saved = -1;
    int set(int device) {
        HIP_OR_FAIL(hipGetDevice(&saved));
        if (saved != device) HIP_OR_FAIL(hipSetDevice(device));
        return SEB_OK;
    }
    ~DeviceGuard() {
        int cur = -1;
        if (saved >= 0 && hipGetDevice(&cur) == hipSuccess && cur != saved) (void)hipSetDevice(saved);
    }
};

extern "C" const char *seb_last_error(void) { return t_err.c_str(); }
extern "C" int seb_abi_version(void) { return SEB_ABI_VERSION; }

// ------------------------------------------------------------------ helpers -----------------

extern "C" uint64_t seb_num_bytes(uint64_t m) { return m / 8 + (m % 8 != 0); }
extern "C" uint64_t seb_words_bytes(uint64_t m) { return (m / 128 + (m % 128 != 0)) * 16; }

extern "C" int seb_params(int64_t n, double p, uint64_t *m, uint32_t *k) {
    if (!m || !k) return fail(SEB_ERR_INVALID, "seb_params: null output");
    if (seb::params(n, p, m, k) != 0)
        return fail(SEB_ERR_RANGE, "seb_params: n=%lld p=%g outside the reference's defined range", (long long)n, p);
    return SEB_OK;
}

static ModArg mod_arg(uint64_t m, uint32_t k) {
    ModArg a{};
    a.m = m;
    a.k = k;
    a.mu = UINT64_MAX / m;
    a.c = (UINT64_MAX % m + 1) % m;  // 2^64 mod m
    return a;
}

static int check_filter_args(uint64_t m, uint32_t k, const char *who) {
    if (m == 0) return fail(SEB_ERR_INVALID, "%s: numBits == 0 (the reference panics: integer divide by zero)", who);
    if (k > 4096) return fail(SEB_ERR_INVALID, "%s: numHashes %u > 4096", who, k);
    return SEB_OK;
}

static int check_keys(const seb_keys *kb, const char *who) {
    if (!kb) return fail(SEB_ERR_INVALID, "%s: null keys", who);
    if (kb->reserved != 0) return fail(SEB_ERR_INVALID, "%s: keys.reserved must be 0", who);
    if (kb->n > 0 && !kb->data && (kb->offsets || kb->stride != 0))
        return fail(SEB_ERR_INVALID, "%s: null key data", who);
    return SEB_OK;
}

static KeyBatch key_batch(const seb_keys *kb) {
    return KeyBatch{kb->data, kb->offsets, kb->n, kb->stride};
}

static bool env_flag(const char *name, long *out) {
    const char *v = getenv(name);
    if (!v || !*v) return false;
    *out = strtol(v, nullptr, 0);
    return true;
}

// Every knob of seb_set_option: name, field, accepted range.  SEB_<NAME> in the environment sets
// its initial value.
struct OptionDesc {
    const char *name;
    int64_t lo, hi;
    int64_t (*get)(const Options &);
    void (*set)(Options &, int64_t);
};
#define SEB_OPT(field, lo, hi)                                                              \
    OptionDesc {                                                                            \
        #field, lo, hi, [](const Options &o) { return (int64_t)o.field; },                   \
            [](Options &o, int64_t v) { o.field = (decltype(o.field))v; }                    \
    }
static const OptionDesc kOptions[] = {
    SEB_OPT(build_algo, 0, 4),
    SEB_OPT(multi_interleave, 0, 1),
    SEB_OPT(multiget_order, 0, 2),
    SEB_OPT(multiget_l0_group, 0, 1),
    SEB_OPT(multiget_xcd, 0, 1),
    SEB_OPT(varlen_prehash_min_keys, 0, INT64_MAX),
    SEB_OPT(bucket_min_keys, 0, INT64_MAX),
    SEB_OPT(lds_min_keys, 0, INT64_MAX),
    SEB_OPT(many_splits, 0, 64),
    SEB_OPT(probe_phases, 0, 64),
    SEB_OPT(probe_compact, 0, 1),
    SEB_OPT(scatter_bins, 0, 1),
    SEB_OPT(grid_cap, 1, 1 << 30),
    SEB_OPT(workspace_limit_mib, 0, 1 << 30),
    SEB_OPT(multiget_piece_mib, 1, 1 << 20),
    SEB_OPT(varlen_tail, 0, 3),
    SEB_OPT(cpu_fallback, 0, 1),
    SEB_OPT(fault_inject, 0, 2),
};
#undef SEB_OPT

static const OptionDesc *find_option(const char *name) {
    for (const OptionDesc &d : kOptions)
        if (!strcmp(d.name, name)) return &d;
    return nullptr;
}

static std::once_flag g_env_once;
static void load_env() {
    Options &o = options();
    for (const OptionDesc &d : kOptions) {
        char var[64] = "SEB_";
        size_t j = 4;
        for (const char *c = d.name; *c && j + 1 < sizeof var; ++c) var[j++] = (char)toupper((unsigned char)*c);
        var[j] = 0;
        long v;
        if (env_flag(var, &v) && v >= d.lo && v <= d.hi) d.set(o, v);
    }
}

// Entry of a call that launches kernels: the knobs are loaded, and HIP's last-error state is
// cleared, so a failed HIP call made earlier on this thread (the caller's, or an allocation the
// library recovered from) is not reported by this call's post-launch hipGetLastError.
static void enter() {
    std::call_once(g_env_once, load_env);
    (void)hipGetLastError();
}

extern "C" int seb_set_option(const char *name, int64_t value) {
    std::call_once(g_env_once, load_env);
    if (!name) return fail(SEB_ERR_INVALID, "seb_set_option: null name");
    const OptionDesc *d = find_option(name);
    if (!d || value < d->lo || value > d->hi)
        return fail(SEB_ERR_INVALID, "seb_set_option: bad option %s=%lld", name, (long long)value);
    d->set(options(), value);
    return SEB_OK;
}

extern "C" int seb_get_option(const char *name, int64_t *value) {
    std::call_once(g_env_once, load_env);
    if (!name || !value) return fail(SEB_ERR_INVALID, "seb_get_option: null argument");
    const OptionDesc *d = find_option(name);
    if (!d) return fail(SEB_ERR_INVALID, "seb_get_option: unknown option %s", name);
    *value = d->get(options());
    return SEB_OK;
}

extern "C" int seb_device_check(int device) {
    std::call_once(g_env_once, load_env);
    int count = 0;
    hipError_t e = hipGetDeviceCount(&count);
    if (e != hipSuccess || count == 0)
        return fail(SEB_ERR_DEVICE, "no HIP device (%s)", e != hipSuccess ? hipGetErrorString(e) : "count 0");
    if (device < 0 || device >= count) return fail(SEB_ERR_DEVICE, "device %d out of range (count %d)", device, count);
    hipDeviceProp_t prop;
    HIP_OR_FAIL(hipGetDeviceProperties(&prop, device));
    if (strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return fail(SEB_ERR_DEVICE, "device %d is %s; this library is built for gfx950 only", device, prop.gcnArchName);
    return SEB_OK;
}

// ------------------------------------------------------- device-resident entry points --------

extern "C" int seb_dev_clear(uint32_t *words, uint64_t m, void *stream) {
    enter();
    if (!words && m) return fail(SEB_ERR_INVALID, "seb_dev_clear: null words");
    if (m == 0) return SEB_OK;
    if (((uintptr_t)words & 15) == 0)
        HIP_OR_FAIL(launch_clear_words(words, seb_words_bytes(m), (hipStream_t)stream));
    else
        HIP_OR_FAIL(hipMemsetAsync(words, 0, seb_words_bytes(m), (hipStream_t)stream));
    return SEB_OK;
}

// Library-owned scratch: grow-only buffers, one set per (device, stream), so concurrent streams
// never share one.  Calls on ONE stream are ordered by the stream, but their enqueue phases can
// overlap across host threads; so an ABI call holds its stream's slot (a recursive lock) from its
// first workspace request until it returns (WsCall at the entry point).  A second thread's call
// on the same stream therefore enqueues after the first call's launches, and a grow (stream sync
// + free) can never free a buffer that another thread has been handed but not yet launched on.
struct WsEntry {
    int tag;  // 0: build / key preparation; 1: packed residues; 2: compacted probe rows; 3: MultiGet key-range order;
              // 4: the fresh build's overflow bitmap (kept all zero)
    void *p;
    uint64_t bytes;
};
struct WsSlot {
    int device;
    hipStream_t stream;
    bool dead = false;  // its stream was destroyed (ws_drop_stream); reusable for a new one
    std::recursive_mutex mu;  // held by the call enqueueing against this slot's buffers
    std::vector<WsEntry> bufs;
};
static std::mutex g_ws_mu;  // guards the slot list; each slot's buffers are guarded by slot->mu
static std::vector<std::unique_ptr<WsSlot>> g_ws;
static thread_local int t_ws_depth = 0;
static thread_local std::vector<std::unique_lock<std::recursive_mutex>> t_ws_held;

// Scope of one ABI call that may use library scratch: slots locked inside it stay locked until
// the call returns (its last launch is enqueued by then).
struct WsCall {
    size_t mark;
    WsCall() : mark(t_ws_held.size()) {
        if (t_ws_depth++ == 0) (void)hipGetLastError();  // as enter(): no stale error from before this call
    }
    ~WsCall() {
        while (t_ws_held.size() > mark) t_ws_held.pop_back();
        --t_ws_depth;
    }
    WsCall(const WsCall &) = delete;
    WsCall &operator=(const WsCall &) = delete;
};

static WsSlot *ws_slot(int dev, hipStream_t s) {
    std::lock_guard<std::mutex> g(g_ws_mu);
    for (auto &sl : g_ws)
        if (!sl->dead && sl->device == dev && sl->stream == s) return sl.get();
    for (auto &sl : g_ws)
        if (sl->dead) {  // buffers already freed; nobody holds a dead slot's lock
            sl->dead = false;
            sl->device = dev;
            sl->stream = s;
            return sl.get();
        }
    g_ws.emplace_back(new WsSlot());
    g_ws.back()->device = dev;
    g_ws.back()->stream = s;
    return g_ws.back().get();
}

// A failed hipMalloc is answered with SEB_ERR_NOMEM and HIP's error state is cleared, so a caller
// that falls back (MultiGet's batch order) does not find it again in a later hipGetLastError.
static int ws_alloc(void **p, uint64_t bytes) {
    const uint64_t lim = options().workspace_limit_mib;
    if (lim && bytes > (lim << 20))
        return fail(SEB_ERR_NOMEM, "workspace %llu B > workspace_limit_mib %llu", (unsigned long long)bytes,
                    (unsigned long long)lim);
    hipError_t a = hipMalloc(p, bytes);
    if (a != hipSuccess) {
        *p = nullptr;
        (void)hipGetLastError();
        return fail(SEB_ERR_NOMEM, "workspace hipMalloc(%llu): %s", (unsigned long long)bytes, hipGetErrorString(a));
    }
    return SEB_OK;
}

// zero: a new (or regrown) buffer is cleared on the stream before first use (the fresh build's
// overflow bitmap, which its users leave all zero).
static int cached_workspace(hipStream_t s, uint64_t bytes, void **out, int tag = 0, bool zero = false) {
    if (t_ws_depth == 0) return fail(SEB_ERR_INVALID, "internal: library scratch requested outside a WsCall scope");
    int dev = 0;
    HIP_OR_FAIL(hipGetDevice(&dev));
    WsSlot *sl = ws_slot(dev, s);
    t_ws_held.emplace_back(sl->mu);  // released when the outermost WsCall of this thread returns
    for (auto &e : sl->bufs)
        if (e.tag == tag) {
            if (e.bytes >= bytes) {
                *out = e.p;
                return SEB_OK;
            }
            HIP_OR_FAIL(hipStreamSynchronize(s));  // earlier launches on this stream may still read it
            HIP_OR_FAIL(hipFree(e.p));
            e.p = nullptr;
            e.bytes = 0;
            int rc = ws_alloc(&e.p, bytes);
            if (rc) return rc;
            e.bytes = bytes;
            if (zero) HIP_OR_FAIL(hipMemsetAsync(e.p, 0, bytes, s));
            *out = e.p;
            return SEB_OK;
        }
    void *p = nullptr;
    int rc = ws_alloc(&p, bytes);
    if (rc) return rc;
    sl->bufs.push_back({tag, p, bytes});
    if (zero) HIP_OR_FAIL(hipMemsetAsync(p, 0, bytes, s));
    *out = p;
    return SEB_OK;
}

// A stream about to be destroyed (a context's) gives its scratch back first: otherwise its slot
// would keep a dead handle that a later seb_workspace_release would synchronise on.
static void ws_drop_stream(int dev, hipStream_t s) {
    WsSlot *sl = nullptr;
    {
        std::lock_guard<std::mutex> g(g_ws_mu);
        for (auto &x : g_ws)
            if (!x->dead && x->device == dev && x->stream == s) sl = x.get();
    }
    if (!sl) return;
    std::lock_guard<std::recursive_mutex> g2(sl->mu);  // a call still enqueueing on it finishes first
    if (!sl->bufs.empty()) {
        (void)hipStreamSynchronize(s);
        for (auto &b : sl->bufs) (void)hipFree(b.p);
        sl->bufs.clear();
    }
    (void)hipGetLastError();
    std::lock_guard<std::mutex> g(g_ws_mu);
    sl->dead = true;
}

// Drop this stream's scratch buffer `tag` (after a failed call that may have left it dirty, such as
// the fresh build's overflow bitmap); the next request allocates (and zeroes) a new one.
static void ws_discard(hipStream_t s, int tag) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return (void)hipGetLastError();
    WsSlot *sl = ws_slot(dev, s);
    std::lock_guard<std::recursive_mutex> g(sl->mu);
    for (auto &e : sl->bufs)
        if (e.tag == tag && e.p) {
            (void)hipStreamSynchronize(s);
            (void)hipFree(e.p);
            e.p = nullptr;
            e.bytes = 0;
        }
    (void)hipGetLastError();
}

// Slots are never deleted, so the pointers stay valid after g_ws_mu is dropped (a call holding a
// slot's lock may take g_ws_mu for another request, so the two are never held in that order here).
static std::vector<WsSlot *> ws_slots_snapshot() {
    std::lock_guard<std::mutex> g(g_ws_mu);
    std::vector<WsSlot *> v;
    for (auto &sl : g_ws) v.push_back(sl.get());
    return v;
}

extern "C" uint64_t seb_workspace_bytes(void) {
    uint64_t total = 0;
    for (WsSlot *sl : ws_slots_snapshot()) {
        std::lock_guard<std::recursive_mutex> g(sl->mu);
        for (auto &e : sl->bufs) total += e.bytes;
    }
    return total;
}

extern "C" int seb_workspace_release(void) {
    int saved = 0;
    HIP_OR_FAIL(hipGetDevice(&saved));
    int rc = SEB_OK;
    for (WsSlot *sl : ws_slots_snapshot()) {
        std::lock_guard<std::recursive_mutex> g2(sl->mu);  // waits for a call still enqueueing on it
        if (sl->bufs.empty()) continue;
        hipError_t e = hipSetDevice(sl->device);
        if (e == hipSuccess) e = hipStreamSynchronize(sl->stream);
        for (auto &b : sl->bufs)
            if (e == hipSuccess) e = hipFree(b.p);
        if (e != hipSuccess) {
            rc = fail(hip_status(e), "seb_workspace_release: %s", hipGetErrorString(e));
            break;
        }
        sl->bufs.clear();
    }
    (void)hipSetDevice(saved);
    return rc;
}

static bool want_prehash(const KeyBatch &kb) {
    return kb.offsets && !kb.hashes && kb.n >= options().varlen_prehash_min_keys;
}
static uint64_t prehash_bytes(const KeyBatch &kb) { return want_prehash(kb) ? ((kb.n * 16 + 255) & ~255ull) : 0; }
// Pre-hash straight to packed residues (8 B per key) when the filter allows them (k == 7,
// m < 2^29): the bucketed build and the phased probe then read half the bytes per key and skip
// re-deriving the residues.
static bool want_prehash_packed(const KeyBatch &kb, const ModArg &md) {
    return want_prehash(kb) && md.k == 7 && md.m < (1ull << kPackBits);
}

// Build dispatcher: bucketed (LDS, no global atomics), LDS-resident or device-scope atomics;
// large variable-length batches are pre-hashed first.  `ws` / `ws_bytes` may be null/0, in which
// case `grow` supplies scratch.
// fresh: `words` holds nothing yet (a new filter); the image build then writes it without a clear,
// and so does the bucketed build given `ovf` (an all-zero overflow bitmap of seb_words_bytes(m));
// every other path clears it first.
template <typename Grow>
static int build_dispatch(KeyBatch kb, uint32_t *words, const ModArg &md, hipStream_t s, void *ws, uint64_t ws_bytes,
                          Grow &&grow, bool fresh = false, uint32_t *ovf = nullptr) {
    // The clear kernel and the image build's OR kernel store 16 B per lane: word arrays that are
    // only 4-B aligned are cleared by hipMemsetAsync and built by the LDS-filter build instead.
    const bool a16 = ((uintptr_t)words & 15) == 0;
    auto clear = [&]() -> hipError_t {
        return a16 ? launch_clear_words(words, seb_words_bytes(md.m), s)
                   : hipMemsetAsync(words, 0, seb_words_bytes(md.m), s);
    };
    if (kb.n == 0 || md.k == 0) {
        if (fresh) HIP_OR_FAIL(clear());
        return SEB_OK;
    }
    int algo = choose_build_algo(kb.n, md.m, md.k);
    if (algo == 4 && !a16) algo = 3;
    const bool bucketed = algo == 2;
    if (!(fresh && bucketed)) ovf = nullptr;
    if (fresh && algo != 4 && !ovf) HIP_OR_FAIL(clear());
    if (bucketed && want_prehash_packed(kb, md)) {  // scratch: [packed residues | bucketed]
        const uint64_t pack_b = (kb.n * 8 + 255) & ~255ull;
        const uint64_t need = pack_b + bucketed_workspace_bytes(kb.n, md.m, md.k);
        if (need > ws_bytes) {
            int rc = grow(need, &ws);
            if (rc) return rc;
            ws_bytes = need;
        }
        HIP_OR_FAIL(launch_hash_varlen_packed(kb, md, (uint64_t *)ws, s));
        HIP_OR_FAIL(launch_build_bucketed_packed((const uint64_t *)ws, kb.n, words, md, (uint8_t *)ws + pack_b,
                                                 ws_bytes - pack_b, s, ovf));
        return SEB_OK;
    }
    const uint64_t head = prehash_bytes(kb);
    const uint64_t need = head + (bucketed ? bucketed_workspace_bytes(kb.n, md.m, md.k)
                                  : algo == 4 ? image_workspace_bytes(kb.n, md.m) : 0);
    if (need > ws_bytes) {
        int rc = grow(need, &ws);
        if (rc) return rc;
        ws_bytes = need;
    }
    if (head) {
        HIP_OR_FAIL(launch_hash_varlen(kb, (uint4 *)ws, s));
        kb.hashes = (const uint4 *)ws;
    }
    if (bucketed) {
        HIP_OR_FAIL(launch_build_bucketed(kb, words, md, (uint8_t *)ws + head, ws_bytes - head, s, ovf));
        return SEB_OK;
    }
    if (algo == 4) {
        HIP_OR_FAIL(launch_build_images(kb, words, md, (uint8_t *)ws + head, ws_bytes - head, fresh, s));
        return SEB_OK;
    }
    if (algo == 3) {  // the whole filter in one CU's LDS, the keys split over workgroups (build_many's kernel)
        ManyArg ma;
        memset(&ma, 0, sizeof ma);
        ma.nf = 1;
        ma.f[0].words = words;
        ma.f[0].nwords = seb_words_bytes(md.m) / 4;
        ma.f[0].key_begin = 0;
        ma.f[0].key_end = kb.n;
        ma.f[0].md = md;
        HIP_OR_FAIL(launch_build_many_lds(kb, ma, (uint32_t)seb_words_bytes(md.m), s));
        return SEB_OK;
    }
    HIP_OR_FAIL(launch_build(kb, words, md, s));
    return SEB_OK;
}

// Variable-length probe batches: pre-hash into the per-(device, stream) scratch cache first.
// `extra` bytes at the front of the scratch are the caller's.
static int prepare_probe_keys(KeyBatch &kb, hipStream_t s, uint64_t extra, void **ws_out) {
    const uint64_t pre_b = prehash_bytes(kb);
    *ws_out = nullptr;
    if (extra + pre_b == 0) return SEB_OK;
    void *ws = nullptr;
    int rc = cached_workspace(s, extra + pre_b, &ws);
    if (rc) return rc;
    *ws_out = ws;
    if (pre_b) {
        HIP_OR_FAIL(launch_hash_varlen(kb, (uint4 *)((uint8_t *)ws + extra), s));
        kb.hashes = (const uint4 *)((uint8_t *)ws + extra);
    }
    return SEB_OK;
}

// The phased probe applies to k == 7, m < 2^29 filters spanning more than one phase, with a
// 4-byte aligned answer array.
static bool want_phased(uint64_t n, const ModArg &md, const uint8_t *out) {
    if (md.k != 7 || md.m >= (1ull << kPackBits)) return false;
    return probe_phase_count(md.m) > 1 && ((uintptr_t)out & 3) == 0 && n > 0;
}

static int probe_dispatch(KeyBatch kb, const uint32_t *words, const ModArg &md, uint8_t *out, hipStream_t s) {
    void *ws;
    int rc;
    if (want_phased(kb.n, md, out) && want_prehash_packed(kb, md) && options().probe_compact) {
        // the pre-hash with phase 0 fused in: compacted rows (tag 2) only, no dense packed batch
        void *rows;
        if ((rc = cached_workspace(s, probe_compact_bytes(kb.n), &rows, 2))) return rc;
        HIP_OR_FAIL(launch_probe_compact_varlen(kb, words, md, out, rows, s));
        return SEB_OK;
    }
    if (want_phased(kb.n, md, out) && want_prehash_packed(kb, md)) {  // pre-hash to packed, all phases from it
        void *packed;
        if ((rc = cached_workspace(s, kb.n * 8, &packed, 1))) return rc;
        HIP_OR_FAIL(launch_hash_varlen_packed(kb, md, (uint64_t *)packed, s));
        if (options().probe_compact) {  // compacted rows (tag 2) from the packed words
            void *rows;
            if ((rc = cached_workspace(s, probe_compact_bytes(kb.n), &rows, 2))) return rc;
            HIP_OR_FAIL(launch_probe_compact_packed((const uint64_t *)packed, kb.n, words, md, out, rows, s));
        } else {
            HIP_OR_FAIL(launch_probe_phased(nullptr, kb.n, words, md, out, (uint64_t *)packed, s));
        }
        return SEB_OK;
    }
    if ((rc = prepare_probe_keys(kb, s, 0, &ws))) return rc;
    if (want_phased(kb.n, md, out) && options().probe_compact) {  // compacted rows in their own scratch (tag 1)
        void *rows;
        if ((rc = cached_workspace(s, probe_compact_bytes(kb.n), &rows, 1))) return rc;
        HIP_OR_FAIL(launch_probe_compact(kb, words, md, out, rows, s));
        return SEB_OK;
    }
    if (want_phased(kb.n, md, out)) {  // packed residues in their own scratch (tag 1)
        void *packed;
        if ((rc = cached_workspace(s, kb.n * 8, &packed, 1))) return rc;
        HIP_OR_FAIL(launch_probe_phased(&kb, kb.n, words, md, out, (uint64_t *)packed, s));
        return SEB_OK;
    }
    HIP_OR_FAIL(launch_probe(kb, words, md, out, s));
    return SEB_OK;
}

extern "C" uint64_t seb_dev_build_workspace_size(uint64_t n, uint64_t m, uint32_t k) {
    enter();
    if (m == 0 || n == 0) return 0;
    // conservative: assumes a variable-length batch (pre-hashed) as well
    const uint64_t pre_b = n >= options().varlen_prehash_min_keys ? ((n * 16 + 255) & ~255ull) : 0;
    const int algo = choose_build_algo(n, m, k);
    return pre_b + (algo == 2 ? bucketed_workspace_bytes(n, m, k) : algo == 4 ? image_workspace_bytes(n, m) : 0);
}

extern "C" int seb_dev_build_ws(const seb_keys *keys, uint32_t *words, uint64_t m, uint32_t k, void *ws,
                                uint64_t ws_bytes, void *stream) {
    enter();
    int rc;
    if ((rc = check_keys(keys, "seb_dev_build_ws")) || (rc = check_filter_args(m, k, "seb_dev_build_ws"))) return rc;
    if (!words) return fail(SEB_ERR_INVALID, "seb_dev_build_ws: null words");
    return build_dispatch(key_batch(keys), words, mod_arg(m, k), (hipStream_t)stream, ws, ws_bytes,
                          [&](uint64_t need, void **) -> int {
                              return fail(SEB_ERR_INVALID, "seb_dev_build_ws: workspace %llu B < %llu B",
                                          (unsigned long long)ws_bytes, (unsigned long long)need);
                          });
}

extern "C" int seb_dev_build(const seb_keys *keys, uint32_t *words, uint64_t m, uint32_t k, void *stream) {
    WsCall ws_call;
    enter();
    int rc;
    if ((rc = check_keys(keys, "seb_dev_build")) || (rc = check_filter_args(m, k, "seb_dev_build"))) return rc;
    if (!words) return fail(SEB_ERR_INVALID, "seb_dev_build: null words");
    hipStream_t s = (hipStream_t)stream;
    return build_dispatch(key_batch(keys), words, mod_arg(m, k), s, nullptr, 0,
                          [&](uint64_t need, void **out) { return cached_workspace(s, need, out); });
}

extern "C" int seb_dev_build_fresh(const seb_keys *keys, uint32_t *words, uint64_t m, uint32_t k, void *stream) {
    WsCall ws_call;
    enter();
    int rc;
    if ((rc = check_keys(keys, "seb_dev_build_fresh")) || (rc = check_filter_args(m, k, "seb_dev_build_fresh")))
        return rc;
    if (!words) return fail(SEB_ERR_INVALID, "seb_dev_build_fresh: null words");
    hipStream_t s = (hipStream_t)stream;
    const KeyBatch kb = key_batch(keys);
    const ModArg md = mod_arg(m, k);
    void *ovf = nullptr;
    if (kb.n && choose_build_algo(kb.n, md.m, md.k) == 2 &&
        (rc = cached_workspace(s, seb_words_bytes(m), &ovf, 4, true)))
        return rc;
    rc = build_dispatch(kb, words, md, s, nullptr, 0,
                        [&](uint64_t need, void **out) { return cached_workspace(s, need, out); }, true,
                        (uint32_t *)ovf);
    if (rc && ovf) ws_discard(s, 4);  // the bitmap may no longer be all zero
    return rc;
}

extern "C" int seb_dev_probe(const seb_keys *keys, const uint32_t *words, uint64_t m, uint32_t k, uint8_t *out,
                             void *stream) {
    WsCall ws_call;
    enter();
    int rc;
    if ((rc = check_keys(keys, "seb_dev_probe")) || (rc = check_filter_args(m, k, "seb_dev_probe"))) return rc;
    if (!words || (!out && keys->n)) return fail(SEB_ERR_INVALID, "seb_dev_probe: null words/out");
    return probe_dispatch(key_batch(keys), words, mod_arg(m, k), out, (hipStream_t)stream);
}

// Packed residues: one 8-byte word per key (r0, b, carry flags) for k == 7 and m < 2^29.
static int check_packed_args(uint64_t m, uint32_t k, const char *who) {
    int rc = check_filter_args(m, k, who);
    if (rc) return rc;
    if (k != 7 || m >= (1ull << kPackBits))
        return fail(SEB_ERR_INVALID, "%s: packed residues need k == 7 and m < 2^%u (k=%u m=%llu)", who, kPackBits, k,
                    (unsigned long long)m);
    return SEB_OK;
}

extern "C" int seb_dev_pack_residues(const seb_keys *keys, uint64_t m, uint32_t k, uint64_t *packed, void *stream) {
    WsCall ws_call;
    enter();
    int rc;
    if ((rc = check_keys(keys, "seb_dev_pack_residues")) || (rc = check_packed_args(m, k, "seb_dev_pack_residues")))
        return rc;
    if (!packed && keys->n) return fail(SEB_ERR_INVALID, "seb_dev_pack_residues: null packed");
    KeyBatch kb = key_batch(keys);
    if (want_prehash_packed(kb, mod_arg(m, k))) {
        HIP_OR_FAIL(launch_hash_varlen_packed(kb, mod_arg(m, k), packed, (hipStream_t)stream));
        return SEB_OK;
    }
    void *ws;
    if ((rc = prepare_probe_keys(kb, (hipStream_t)stream, 0, &ws))) return rc;
    HIP_OR_FAIL(launch_pack_residues(kb, mod_arg(m, k), packed, (hipStream_t)stream));
    return SEB_OK;
}

extern "C" int seb_dev_probe_packed(const uint64_t *packed, uint64_t n, const uint32_t *words, uint64_t m, uint32_t k,
                                    uint8_t *out, void *stream) {
    WsCall ws_call;
    enter();
    int rc = check_packed_args(m, k, "seb_dev_probe_packed");
    if (rc) return rc;
    if (n && (!packed || !words || !out)) return fail(SEB_ERR_INVALID, "seb_dev_probe_packed: null pointer");
    const ModArg md = mod_arg(m, k);
    if (want_phased(n, md, out) && options().probe_compact) {
        void *rows;
        if ((rc = cached_workspace((hipStream_t)stream, probe_compact_bytes(n), &rows, 2))) return rc;
        HIP_OR_FAIL(launch_probe_compact_packed(packed, n, words, md, out, rows, (hipStream_t)stream));
    } else if (want_phased(n, md, out))
        HIP_OR_FAIL(launch_probe_phased(nullptr, n, words, md, out, const_cast<uint64_t *>(packed), (hipStream_t)stream));
    else
        HIP_OR_FAIL(launch_probe_packed(packed, n, words, md, out, (hipStream_t)stream));
    return SEB_OK;
}

// Narrow packed residues: 6 bytes per key in 64-key blocks, for k == 7 and m < 2^21.
static int check_packed6_args(uint64_t m, uint32_t k, const char *who) {
    int rc = check_filter_args(m, k, who);
    if (rc) return rc;
    if (k != 7 || m >= (1ull << kPack6Bits))
        return fail(SEB_ERR_INVALID, "%s: 6-byte packed residues need k == 7 and m < 2^%u (k=%u m=%llu)", who,
                    kPack6Bits, k, (unsigned long long)m);
    return SEB_OK;
}

extern "C" uint64_t seb_packed6_bytes(uint64_t n) { return packed6_bytes(n); }

extern "C" int seb_dev_pack_residues6(const seb_keys *keys, uint64_t m, uint32_t k, void *packed6, void *stream) {
    WsCall ws_call;
    enter();
    int rc;
    if ((rc = check_keys(keys, "seb_dev_pack_residues6")) || (rc = check_packed6_args(m, k, "seb_dev_pack_residues6")))
        return rc;
    if (!packed6 && keys->n) return fail(SEB_ERR_INVALID, "seb_dev_pack_residues6: null packed6");
    if (((uintptr_t)packed6 & 3) != 0) return fail(SEB_ERR_INVALID, "seb_dev_pack_residues6: packed6 not 4-byte aligned");
    KeyBatch kb = key_batch(keys);
    void *ws;
    if ((rc = prepare_probe_keys(kb, (hipStream_t)stream, 0, &ws))) return rc;
    HIP_OR_FAIL(launch_pack_residues6(kb, mod_arg(m, k), (uint8_t *)packed6, (hipStream_t)stream));
    return SEB_OK;
}

extern "C" int seb_dev_probe_emit_packed(const seb_keys *keys, const uint32_t *words, uint64_t m, uint32_t k,
                                         uint8_t *out, uint64_t *packed, void *stream) {
    WsCall ws_call;
    enter();
    int rc;
    if ((rc = check_keys(keys, "seb_dev_probe_emit_packed")) ||
        (rc = check_packed_args(m, k, "seb_dev_probe_emit_packed")))
        return rc;
    if (keys->n && (!words || !out || !packed)) return fail(SEB_ERR_INVALID, "seb_dev_probe_emit_packed: null pointer");
    KeyBatch kb = key_batch(keys);
    const ModArg md = mod_arg(m, k);
    if (want_phased(kb.n, md, out) && want_prehash_packed(kb, md)) {
        HIP_OR_FAIL(launch_hash_varlen_packed(kb, md, packed, (hipStream_t)stream));
        HIP_OR_FAIL(launch_probe_phased(nullptr, kb.n, words, md, out, packed, (hipStream_t)stream));
        return SEB_OK;
    }
    void *ws;
    if ((rc = prepare_probe_keys(kb, (hipStream_t)stream, 0, &ws))) return rc;
    if (want_phased(kb.n, md, out))  // phase 0 writes the packed residues anyway
        HIP_OR_FAIL(launch_probe_phased(&kb, kb.n, words, md, out, packed, (hipStream_t)stream));
    else
        HIP_OR_FAIL(launch_probe_emit(kb, words, md, out, packed, (hipStream_t)stream));
    return SEB_OK;
}

static int fill_multi(const seb_filter_ref *filters, uint32_t nf, uint32_t mask_bytes, MultiArg *ma,
                      const char *who) {
    if (!filters || nf == 0) return fail(SEB_ERR_INVALID, "%s: no filters", who);
    if (nf > (uint32_t)kMaxMulti) return fail(SEB_ERR_INVALID, "%s: %u filters > %d", who, nf, kMaxMulti);
    if (!(mask_bytes == 1 || mask_bytes == 2 || mask_bytes == 4 || mask_bytes == 8) || nf > 8 * mask_bytes)
        return fail(SEB_ERR_INVALID, "%s: mask_bytes %u cannot hold %u filters", who, mask_bytes, nf);
    memset(ma, 0, sizeof *ma);
    ma->nf = nf;
    for (uint32_t f = 0; f < nf; ++f) {
        int rc = check_filter_args(filters[f].num_bits, filters[f].num_hashes, who);
        if (rc) return rc;
        if (!filters[f].bits || filters[f].reserved) return fail(SEB_ERR_INVALID, "%s: bad filter %u", who, f);
        ma->f[f].words = (const uint32_t *)filters[f].bits;
        ma->f[f].md = mod_arg(filters[f].num_bits, filters[f].num_hashes);
    }
    return SEB_OK;
}

extern "C" int seb_dev_probe_multi(const seb_keys *keys, const seb_filter_ref *filters, uint32_t nf, void *mask,
                                   uint32_t mask_bytes, void *stream) {
    WsCall ws_call;
    enter();
    int rc;
    MultiArg ma;
    if ((rc = check_keys(keys, "seb_dev_probe_multi")) ||
        (rc = fill_multi(filters, nf, mask_bytes, &ma, "seb_dev_probe_multi")))
        return rc;
    if (!mask && keys->n) return fail(SEB_ERR_INVALID, "seb_dev_probe_multi: null mask");
    hipStream_t s = (hipStream_t)stream;
    KeyBatch kb = key_batch(keys);
    const uint64_t tb = options().multi_interleave && keys->n >= 65536 ? interleaved_bytes(ma, mask_bytes) : 0;
    void *ws = nullptr;
    if ((rc = prepare_probe_keys(kb, s, (tb + 255) & ~255ull, &ws))) return rc;
    if (tb) {
        HIP_OR_FAIL(launch_probe_interleaved(kb, ma, mask, mask_bytes, ws, s));
        return SEB_OK;
    }
    HIP_OR_FAIL(launch_probe_multi(kb, ma, mask, mask_bytes, s));
    return SEB_OK;
}

extern "C" int seb_dev_probe_multi_packed(const uint64_t *packed, uint64_t n, const seb_filter_ref *filters,
                                          uint32_t nf, void *mask, uint32_t mask_bytes, void *stream) {
    WsCall ws_call;
    enter();
    int rc;
    MultiArg ma;
    if ((rc = fill_multi(filters, nf, mask_bytes, &ma, "seb_dev_probe_multi_packed"))) return rc;
    for (uint32_t f = 0; f < nf; ++f)
        if (ma.f[f].md.m != ma.f[0].md.m || ma.f[f].md.k != ma.f[0].md.k)
            return fail(SEB_ERR_INVALID, "seb_dev_probe_multi_packed: filters must share (num_bits, num_hashes)");
    if ((rc = check_packed_args(ma.f[0].md.m, ma.f[0].md.k, "seb_dev_probe_multi_packed"))) return rc;
    if (n && (!packed || !mask)) return fail(SEB_ERR_INVALID, "seb_dev_probe_multi_packed: null pointer");
    if (n == 0) return SEB_OK;
    hipStream_t s = (hipStream_t)stream;
    const uint64_t tb = ((ma.f[0].md.m + 31) / 32) * 32 * mask_bytes;
    void *ws = nullptr;
    if ((rc = cached_workspace(s, (tb + 255) & ~255ull, &ws))) return rc;
    HIP_OR_FAIL(launch_probe_interleaved_packed(packed, n, ma, mask, mask_bytes, ws, s));
    return SEB_OK;
}

extern "C" int seb_dev_probe_multi_packed6(const void *packed6, uint64_t n, const seb_filter_ref *filters,
                                           uint32_t nf, void *mask, uint32_t mask_bytes, void *stream) {
    WsCall ws_call;
    enter();
    int rc;
    MultiArg ma;
    if ((rc = fill_multi(filters, nf, mask_bytes, &ma, "seb_dev_probe_multi_packed6"))) return rc;
    for (uint32_t f = 0; f < nf; ++f)
        if (ma.f[f].md.m != ma.f[0].md.m || ma.f[f].md.k != ma.f[0].md.k)
            return fail(SEB_ERR_INVALID, "seb_dev_probe_multi_packed6: filters must share (num_bits, num_hashes)");
    if ((rc = check_packed6_args(ma.f[0].md.m, ma.f[0].md.k, "seb_dev_probe_multi_packed6"))) return rc;
    if (n && (!packed6 || !mask)) return fail(SEB_ERR_INVALID, "seb_dev_probe_multi_packed6: null pointer");
    if (((uintptr_t)packed6 & 3) != 0)
        return fail(SEB_ERR_INVALID, "seb_dev_probe_multi_packed6: packed6 not 4-byte aligned");
    if (n == 0) return SEB_OK;
    hipStream_t s = (hipStream_t)stream;
    const uint64_t tb = ((ma.f[0].md.m + 31) / 32) * 32 * mask_bytes;
    void *ws = nullptr;
    if ((rc = cached_workspace(s, (tb + 255) & ~255ull, &ws))) return rc;
    HIP_OR_FAIL(launch_probe_interleaved_packed6((const uint8_t *)packed6, n, ma, mask, mask_bytes, ws, s));
    return SEB_OK;
}

extern "C" int seb_dev_or_slices(const uint32_t *slices, uint32_t num_slices, uint64_t slice_words, uint32_t *out,
                                 void *stream) {
    enter();
    if (slice_words && num_slices && (!slices || !out)) return fail(SEB_ERR_INVALID, "seb_dev_or_slices: null pointer");
    HIP_OR_FAIL(launch_or_slices(slices, num_slices, slice_words, out, (hipStream_t)stream));
    return SEB_OK;
}

static const uint32_t kLdsMax = 160 * 1024;

extern "C" int seb_dev_build_many(const seb_keys *keys, const uint64_t *key_begin, const seb_filter_ref *filters,
                                  uint32_t nf, void *stream) {
    enter();
    int rc;
    if ((rc = check_keys(keys, "seb_dev_build_many"))) return rc;
    if (!key_begin || (!filters && nf)) return fail(SEB_ERR_INVALID, "seb_dev_build_many: null arrays");
    hipStream_t s = (hipStream_t)stream;
    KeyBatch kb = key_batch(keys);
    ManyArg ma;
    memset(&ma, 0, sizeof ma);
    uint32_t lds = 0;
    auto flush = [&]() -> int {
        if (ma.nf == 0) return SEB_OK;
        HIP_OR_FAIL(launch_build_many_lds(kb, ma, lds, s));
        memset(&ma, 0, sizeof ma);
        lds = 0;
        return SEB_OK;
    };
    for (uint32_t f = 0; f < nf; ++f) {
        const uint64_t m = filters[f].num_bits;
        const uint32_t k = filters[f].num_hashes;
        if ((rc = check_filter_args(m, k, "seb_dev_build_many"))) return rc;
        if (!filters[f].bits || key_begin[f + 1] < key_begin[f] || key_begin[f + 1] > keys->n)
            return fail(SEB_ERR_INVALID, "seb_dev_build_many: bad filter %u", f);
        const uint64_t wb = seb_words_bytes(m);
        if (wb <= kLdsMax) {
            ManyFilter &F = ma.f[ma.nf++];
            F.words = (uint32_t *)filters[f].bits;
            F.nwords = wb / 4;
            F.key_begin = key_begin[f];
            F.key_end = key_begin[f + 1];
            F.md = mod_arg(m, k);
            lds = std::max<uint32_t>(lds, (uint32_t)wb);
            if (ma.nf == (uint32_t)kMaxMany && (rc = flush())) return rc;
        } else {  // too large for one CU's LDS: grid-wide atomics over this filter's key range
            KeyBatch sub = kb;
            sub.n = key_begin[f + 1] - key_begin[f];
            if (kb.offsets)
                sub.offsets = kb.offsets + key_begin[f];
            else
                sub.data = kb.data + key_begin[f] * (uint64_t)kb.stride;
            HIP_OR_FAIL(launch_build(sub, (uint32_t *)filters[f].bits, mod_arg(m, k), s));
        }
    }
    return flush();
}

extern "C" int seb_dev_alloc(void **ptr, uint64_t bytes) {
    if (!ptr) return fail(SEB_ERR_INVALID, "seb_dev_alloc: null");
    hipError_t e = hipMalloc(ptr, bytes ? bytes : 16);
    if (e != hipSuccess) return (void)hipGetLastError(), fail(SEB_ERR_NOMEM, "hipMalloc(%llu): %s", (unsigned long long)bytes, hipGetErrorString(e));
    return SEB_OK;
}
extern "C" int seb_dev_free(void *ptr) {
    HIP_OR_FAIL(hipFree(ptr));
    return SEB_OK;
}
extern "C" int seb_host_alloc(void **ptr, uint64_t bytes) {
    if (!ptr) return fail(SEB_ERR_INVALID, "seb_host_alloc: null");
    hipError_t e = hipHostMalloc(ptr, bytes ? bytes : 16, hipHostMallocDefault);
    if (e != hipSuccess) return (void)hipGetLastError(), fail(SEB_ERR_NOMEM, "hipHostMalloc(%llu): %s", (unsigned long long)bytes, hipGetErrorString(e));
    return SEB_OK;
}
extern "C" int seb_host_free(void *ptr) {
    HIP_OR_FAIL(hipHostFree(ptr));
    return SEB_OK;
}
extern "C" int seb_memcpy_h2d(void *dst, const void *src, uint64_t bytes, void *stream) {
    HIP_OR_FAIL(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, (hipStream_t)stream));
    return SEB_OK;
}
extern "C" int seb_memcpy_d2h(void *dst, const void *src, uint64_t bytes, void *stream) {
    HIP_OR_FAIL(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, (hipStream_t)stream));
    return SEB_OK;
}
extern "C" int seb_stream_sync(void *stream) {
    HIP_OR_FAIL(hipStreamSynchronize((hipStream_t)stream));
    return SEB_OK;
}

// Timing events without the system-scope fence a default HIP event performs when it completes:
// that fence writes back and invalidates L2 and costs ~15 us between two kernels on gfx950
// (profiles/r02_event_gaps), which would inflate the very step it measures.
extern "C" int seb_timer_create(void **ev) {
    if (!ev) return fail(SEB_ERR_INVALID, "seb_timer_create: null");
    hipEvent_t e;
    HIP_OR_FAIL(hipEventCreateWithFlags(&e, hipEventDisableSystemFence));
    *ev = (void *)e;
    return SEB_OK;
}

extern "C" int seb_timer_record(void *ev, void *stream) {
    HIP_OR_FAIL(hipEventRecord((hipEvent_t)ev, (hipStream_t)stream));
    return SEB_OK;
}

extern "C" int seb_timer_elapsed_ms(void *start, void *end, float *ms) {
    if (!ms) return fail(SEB_ERR_INVALID, "seb_timer_elapsed_ms: null");
    HIP_OR_FAIL(hipEventSynchronize((hipEvent_t)end));
    HIP_OR_FAIL(hipEventElapsedTime(ms, (hipEvent_t)start, (hipEvent_t)end));
    return SEB_OK;
}

extern "C" int seb_timer_destroy(void *ev) {
    if (ev) HIP_OR_FAIL(hipEventDestroy((hipEvent_t)ev));
    return SEB_OK;
}

// ------------------------------------------------------- contexts (host-buffer API) ----------

struct DevBuf {
    void *p = nullptr;
    uint64_t cap = 0;
    // limited: scratch that workspace_limit_mib caps (a context's build scratch)
    int reserve(uint64_t bytes, bool limited = false) {
        if (bytes <= cap) return SEB_OK;
        const uint64_t lim = options().workspace_limit_mib;
        if (limited && lim && bytes > (lim << 20))
            return fail(SEB_ERR_NOMEM, "workspace %llu B > workspace_limit_mib %llu", (unsigned long long)bytes,
                        (unsigned long long)lim);
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
        uint64_t want = std::max<uint64_t>(bytes, 4096);
        hipError_t e = hipMalloc(&p, want);
        if (e != hipSuccess) return (void)hipGetLastError(), fail(SEB_ERR_NOMEM, "hipMalloc(%llu): %s", (unsigned long long)want, hipGetErrorString(e));
        cap = want;
        return SEB_OK;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
    }
};

// Grow-only host-pinned buffer (device-accessible), for the small builds' zero-copy path.
struct PinBuf {
    void *p = nullptr;
    void *dev = nullptr;  // the device's address of p
    uint64_t cap = 0;
    int reserve(uint64_t bytes) {
        if (bytes <= cap) return SEB_OK;
        release();
        uint64_t want = std::max<uint64_t>(bytes, 1 << 20);
        hipError_t e = hipHostMalloc(&p, want, hipHostMallocDefault);
        if (e != hipSuccess) {
            p = nullptr;
            return (void)hipGetLastError(), fail(SEB_ERR_NOMEM, "hipHostMalloc(%llu): %s", (unsigned long long)want,
                                                 hipGetErrorString(e));
        }
        if ((e = hipHostGetDevicePointer(&dev, p, 0)) != hipSuccess) {
            release();
            return (void)hipGetLastError(), fail(hip_status(e), "hipHostGetDevicePointer: %s", hipGetErrorString(e));
        }
        cap = want;
        return SEB_OK;
    }
    void release() {
        if (p) (void)hipHostFree(p);
        p = dev = nullptr;
        cap = 0;
    }
};

struct seb_ctx {
    int device = 0;
    std::mutex mu;
    hipStream_t s_h2d = nullptr, s_comp = nullptr, s_d2h = nullptr;
    hipEvent_t ev_h2d[2] = {}, ev_comp[2] = {}, ev_d2h[2] = {};
    DevBuf keys[2], offs[2], out[2], words, filt, ws;
    PinBuf hkeys, hbits;  // small filter builds: keys in, bits out, read and written by the kernels
    uint64_t chunk_bytes = 64ull << 20;
    std::vector<uint64_t> off_tmp[2];
};

extern "C" int seb_ctx_create(int device, seb_ctx **out) {
    if (!out) return fail(SEB_ERR_INVALID, "seb_ctx_create: null out");
    int rc = seb_device_check(device);
    if (rc) return rc;
    HIP_OR_FAIL(hipSetDevice(device));
    seb_ctx *c = new seb_ctx();
    c->device = device;
    long cb;
    if (env_flag("SEB_CHUNK_BYTES", &cb) && cb > 0) c->chunk_bytes = (uint64_t)cb;
    hipError_t e = hipSuccess;
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&c->s_h2d, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&c->s_comp, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&c->s_d2h, hipStreamNonBlocking);
    for (int b = 0; b < 2 && e == hipSuccess; ++b) {
        e = hipEventCreateWithFlags(&c->ev_h2d[b], hipEventDisableTiming);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&c->ev_comp[b], hipEventDisableTiming);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&c->ev_d2h[b], hipEventDisableTiming);
    }
    if (e != hipSuccess) {
        seb_ctx_destroy(c);
        return fail(hip_status(e), "seb_ctx_create: %s", hipGetErrorString(e));
    }
    *out = c;
    return SEB_OK;
}

extern "C" void seb_ctx_destroy(seb_ctx *c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->s_comp) (void)hipStreamSynchronize(c->s_comp);
    for (int b = 0; b < 2; ++b) {
        c->keys[b].release();
        c->offs[b].release();
        c->out[b].release();
        if (c->ev_h2d[b]) (void)hipEventDestroy(c->ev_h2d[b]);
        if (c->ev_comp[b]) (void)hipEventDestroy(c->ev_comp[b]);
        if (c->ev_d2h[b]) (void)hipEventDestroy(c->ev_d2h[b]);
    }
    c->words.release();
    c->filt.release();
    c->ws.release();
    c->hkeys.release();
    c->hbits.release();
    for (hipStream_t st : {c->s_h2d, c->s_comp, c->s_d2h})
        if (st) ws_drop_stream(c->device, st);
    if (c->s_h2d) (void)hipStreamDestroy(c->s_h2d);
    if (c->s_comp) (void)hipStreamDestroy(c->s_comp);
    if (c->s_d2h) (void)hipStreamDestroy(c->s_d2h);
    delete c;
}

// Host key batch -> sequence of chunks [i0, i1) whose key bytes fit the chunk budget.
struct Chunk {
    uint64_t i0, i1, byte0, byte1;
};

static void plan_chunks(const seb_keys *kb, uint64_t budget, std::vector<Chunk> &out) {
    out.clear();
    const uint64_t n = kb->n;
    if (n == 0) return;
    if (!kb->offsets) {
        uint64_t per = kb->stride ? std::max<uint64_t>(1, budget / kb->stride) : n;
        for (uint64_t i = 0; i < n; i += per) {
            uint64_t j = std::min(n, i + per);
            out.push_back({i, j, i * kb->stride, j * kb->stride});
        }
        return;
    }
    const uint64_t *o = kb->offsets;
    uint64_t i = 0;
    while (i < n) {
        // largest j with o[j] - o[i] <= budget (at least one key)
        uint64_t lo = i + 1, hi = n;
        while (lo < hi) {
            uint64_t mid = lo + (hi - lo + 1) / 2;
            if (o[mid] - o[i] <= budget) lo = mid; else hi = mid - 1;
        }
        out.push_back({i, lo, o[i], o[lo]});
        i = lo;
    }
}

static int validate_offsets(const seb_keys *kb, const char *who) {
    if (!kb->offsets) return SEB_OK;
    for (uint64_t i = 0; i < kb->n; ++i)
        if (kb->offsets[i + 1] < kb->offsets[i]) return fail(SEB_ERR_INVALID, "%s: offsets decrease at %llu", who, (unsigned long long)i);
    return SEB_OK;
}

// Stage one chunk of host keys into buffer b on s_h2d; returns the device KeyBatch for it.  A batch
// of one chunk is copied on s_comp itself: nothing to overlap, and a cross-stream event wait
// costs ~17 us before the kernel may start (profiles/r03_flush_trace.txt).
static int stage_chunk(seb_ctx *c, const seb_keys *kb, const Chunk &ch, int b, KeyBatch *dk, bool single) {
    int rc;
    const uint64_t bytes = ch.byte1 - ch.byte0;
    if ((rc = c->keys[b].reserve(bytes + 16))) return rc;
    hipStream_t cs = single ? c->s_comp : c->s_h2d;
    if (!single) HIP_OR_FAIL(hipStreamWaitEvent(c->s_h2d, c->ev_comp[b], 0));  // buffer b no longer read
    if (bytes) HIP_OR_FAIL(hipMemcpyAsync(c->keys[b].p, kb->data + ch.byte0, bytes, hipMemcpyHostToDevice, cs));
    dk->n = ch.i1 - ch.i0;
    dk->stride = kb->stride;
    if (kb->offsets) {
        const uint64_t cnt = dk->n + 1;
        if ((rc = c->offs[b].reserve(cnt * 8))) return rc;
        HIP_OR_FAIL(hipMemcpyAsync(c->offs[b].p, kb->offsets + ch.i0, cnt * 8, hipMemcpyHostToDevice, cs));
        dk->offsets = (const uint64_t *)c->offs[b].p;
        dk->data = (const uint8_t *)c->keys[b].p - ch.byte0;  // offsets are absolute
    } else {
        dk->offsets = nullptr;
        dk->data = (const uint8_t *)c->keys[b].p;
    }
    if (single) return SEB_OK;
    HIP_OR_FAIL(hipEventRecord(c->ev_h2d[b], c->s_h2d));
    HIP_OR_FAIL(hipStreamWaitEvent(c->s_comp, c->ev_h2d[b], 0));
    return SEB_OK;
}

// OR host keys into device words (all on c->s_comp ordering), chunked + double buffered.
static int build_device_from_host(seb_ctx *c, const seb_keys *kb, uint32_t *dwords, const ModArg &md,
                                  bool fresh = false) {
    std::vector<Chunk> chunks;
    plan_chunks(kb, c->chunk_bytes, chunks);
    for (size_t j = 0; j < chunks.size(); ++j) {
        const int b = (int)(j & 1);
        KeyBatch dk{};
        int rc = stage_chunk(c, kb, chunks[j], b, &dk, chunks.size() == 1);
        if (rc) return rc;
        rc = build_dispatch(dk, dwords, md, c->s_comp, c->ws.p, c->ws.cap, [&](uint64_t need, void **out) -> int {
            HIP_OR_FAIL(hipStreamSynchronize(c->s_comp));  // previous chunks may still use it
            int r = c->ws.reserve(need, true);
            *out = c->ws.p;
            return r;
        }, fresh && j == 0);
        if (rc) return rc;
        HIP_OR_FAIL(hipEventRecord(c->ev_comp[b], c->s_comp));
    }
    return SEB_OK;
}

static int probe_device_to_host(seb_ctx *c, const seb_keys *kb, const uint32_t *dwords, const ModArg &md,
                                uint8_t *out) {
    std::vector<Chunk> chunks;
    plan_chunks(kb, c->chunk_bytes, chunks);
    for (size_t j = 0; j < chunks.size(); ++j) {
        const int b = (int)(j & 1);
        KeyBatch dk{};
        const bool single = chunks.size() == 1;  // copy in, probe, copy out on s_comp alone
        int rc = stage_chunk(c, kb, chunks[j], b, &dk, single);
        if (rc) return rc;
        const uint64_t cnt = dk.n;
        if ((rc = c->out[b].reserve(cnt))) return rc;
        if (!single) HIP_OR_FAIL(hipStreamWaitEvent(c->s_comp, c->ev_d2h[b], 0));  // out[b] drained
        if ((rc = probe_dispatch(dk, dwords, md, (uint8_t *)c->out[b].p, c->s_comp))) return rc;
        if (single) {
            HIP_OR_FAIL(hipMemcpyAsync(out + chunks[j].i0, c->out[b].p, cnt, hipMemcpyDeviceToHost, c->s_comp));
            HIP_OR_FAIL(hipStreamSynchronize(c->s_comp));
            return SEB_OK;
        }
        HIP_OR_FAIL(hipEventRecord(c->ev_comp[b], c->s_comp));
        HIP_OR_FAIL(hipStreamWaitEvent(c->s_d2h, c->ev_comp[b], 0));
        HIP_OR_FAIL(hipMemcpyAsync(out + chunks[j].i0, c->out[b].p, cnt, hipMemcpyDeviceToHost, c->s_d2h));
        HIP_OR_FAIL(hipEventRecord(c->ev_d2h[b], c->s_d2h));
    }
    HIP_OR_FAIL(hipStreamSynchronize(c->s_d2h));
    return SEB_OK;
}

extern "C" int seb_build(seb_ctx *c, const seb_keys *kb, uint8_t *bits, uint64_t m, uint32_t k, uint32_t flags) {
    int rc;
    if (!c) return fail(SEB_ERR_INVALID, "seb_build: null ctx");
    if ((rc = check_keys(kb, "seb_build")) || (rc = check_filter_args(m, k, "seb_build")) ||
        (rc = validate_offsets(kb, "seb_build")))
        return rc;
    if (!bits) return fail(SEB_ERR_INVALID, "seb_build: null bits");
    std::lock_guard<std::mutex> g(c->mu);
    HIP_OR_FAIL(hipSetDevice(c->device));
    const uint64_t wb = seb_words_bytes(m), nb = seb_num_bytes(m);
    if ((rc = c->words.reserve(wb))) return rc;
    uint32_t *dw = (uint32_t *)c->words.p;
    HIP_OR_FAIL(hipMemsetAsync(dw, 0, wb, c->s_comp));
    if (!(flags & SEB_BUILD_FRESH)) HIP_OR_FAIL(hipMemcpyAsync(dw, bits, nb, hipMemcpyHostToDevice, c->s_comp));
    if ((rc = build_device_from_host(c, kb, dw, mod_arg(m, k)))) return rc;
    HIP_OR_FAIL(hipMemcpyAsync(bits, dw, nb, hipMemcpyDeviceToHost, c->s_comp));
    HIP_OR_FAIL(hipStreamSynchronize(c->s_comp));
    return SEB_OK;
}

extern "C" int seb_probe(seb_ctx *c, const seb_keys *kb, const uint8_t *bits, uint64_t m, uint32_t k, uint8_t *out) {
    WsCall ws_call;
    int rc;
    if (!c) return fail(SEB_ERR_INVALID, "seb_probe: null ctx");
    if ((rc = check_keys(kb, "seb_probe")) || (rc = check_filter_args(m, k, "seb_probe")) ||
        (rc = validate_offsets(kb, "seb_probe")))
        return rc;
    if (!bits || (!out && kb->n)) return fail(SEB_ERR_INVALID, "seb_probe: null bits/out");
    std::lock_guard<std::mutex> g(c->mu);
    HIP_OR_FAIL(hipSetDevice(c->device));
    const uint64_t wb = seb_words_bytes(m), nb = seb_num_bytes(m);
    if ((rc = c->words.reserve(wb))) return rc;
    uint32_t *dw = (uint32_t *)c->words.p;
    HIP_OR_FAIL(hipMemsetAsync(dw, 0, wb, c->s_comp));
    HIP_OR_FAIL(hipMemcpyAsync(dw, bits, nb, hipMemcpyHostToDevice, c->s_comp));
    return probe_device_to_host(c, kb, dw, mod_arg(m, k), out);
}

extern "C" int seb_probe_multi(seb_ctx *c, const seb_keys *kb, const seb_filter_ref *filters, uint32_t nf,
                               uint64_t *mask) {
    int rc;
    if (!c) return fail(SEB_ERR_INVALID, "seb_probe_multi: null ctx");
    if ((rc = check_keys(kb, "seb_probe_multi")) || (rc = validate_offsets(kb, "seb_probe_multi"))) return rc;
    if (!mask && kb->n) return fail(SEB_ERR_INVALID, "seb_probe_multi: null mask");
    if (!filters || nf == 0 || nf > (uint32_t)kMaxMulti) return fail(SEB_ERR_INVALID, "seb_probe_multi: bad filter count");
    std::lock_guard<std::mutex> g(c->mu);
    HIP_OR_FAIL(hipSetDevice(c->device));
    uint64_t total = 0;
    std::vector<uint64_t> at(nf);
    for (uint32_t f = 0; f < nf; ++f) {
        if ((rc = check_filter_args(filters[f].num_bits, filters[f].num_hashes, "seb_probe_multi"))) return rc;
        if (!filters[f].bits) return fail(SEB_ERR_INVALID, "seb_probe_multi: null bits %u", f);
        at[f] = total;
        total += seb_words_bytes(filters[f].num_bits);
    }
    if ((rc = c->filt.reserve(total))) return rc;
    HIP_OR_FAIL(hipMemsetAsync(c->filt.p, 0, total, c->s_comp));
    std::vector<seb_filter_ref> dref(filters, filters + nf);
    for (uint32_t f = 0; f < nf; ++f) {
        uint8_t *d = (uint8_t *)c->filt.p + at[f];
        HIP_OR_FAIL(hipMemcpyAsync(d, filters[f].bits, seb_num_bytes(filters[f].num_bits), hipMemcpyHostToDevice, c->s_comp));
        dref[f].bits = d;
    }
    MultiArg ma;
    if ((rc = fill_multi(dref.data(), nf, 8, &ma, "seb_probe_multi"))) return rc;
    std::vector<Chunk> chunks;
    plan_chunks(kb, c->chunk_bytes, chunks);
    for (size_t j = 0; j < chunks.size(); ++j) {
        const int b = (int)(j & 1);
        KeyBatch dk{};
        if ((rc = stage_chunk(c, kb, chunks[j], b, &dk, false))) return rc;
        if ((rc = c->out[b].reserve(dk.n * 8))) return rc;
        HIP_OR_FAIL(hipStreamWaitEvent(c->s_comp, c->ev_d2h[b], 0));
        HIP_OR_FAIL(launch_probe_multi(dk, ma, c->out[b].p, 8, c->s_comp));
        HIP_OR_FAIL(hipEventRecord(c->ev_comp[b], c->s_comp));
        HIP_OR_FAIL(hipStreamWaitEvent(c->s_d2h, c->ev_comp[b], 0));
        HIP_OR_FAIL(hipMemcpyAsync(mask + chunks[j].i0, c->out[b].p, dk.n * 8, hipMemcpyDeviceToHost, c->s_d2h));
        HIP_OR_FAIL(hipEventRecord(c->ev_d2h[b], c->s_d2h));
    }
    HIP_OR_FAIL(hipStreamSynchronize(c->s_d2h));
    return SEB_OK;
}

// ------------------------------------------------ Go API mirror (lsm/bloom.go handles) -------

static std::mutex g_pool_mu;
static std::vector<seb_ctx *> g_pool;

static int default_device() {
    long d;
    return env_flag("SEB_DEVICE", &d) ? (int)d : 0;
}

struct CtxLease {  // borrow a context from the process pool (concurrent filters do not serialise)
    seb_ctx *c = nullptr;
    int rc = SEB_OK;
    explicit CtxLease(int device) {
        {
            std::lock_guard<std::mutex> g(g_pool_mu);
            for (size_t i = 0; i < g_pool.size(); ++i)
                if (g_pool[i]->device == device) {
                    c = g_pool[i];
                    g_pool.erase(g_pool.begin() + i);
                    break;
                }
        }
        if (!c) rc = seb_ctx_create(device, &c);
    }
    ~CtxLease() {
        if (c) {
            std::lock_guard<std::mutex> g(g_pool_mu);
            g_pool.push_back(c);
        }
    }
};

static inline void cpu_relax() {
#if defined(__x86_64__) || defined(__i386__)
    __builtin_ia32_pause();
#endif
}

// A lock for the filter handle: one atomic exchange to take it uncontended (Add takes it once per
// key, so a pthread mutex's call + fence pair showed in the per-key cost), a bounded spin, then
// yields (a waiter may be waiting on a GPU build that takes milliseconds).
struct FilterLock {
    std::atomic<bool> held{false};
    void lock() {
        for (int spin = 0; held.exchange(true, std::memory_order_acquire); ++spin) {
            while (held.load(std::memory_order_relaxed)) {
                if (++spin > 64) std::this_thread::yield();
                else cpu_relax();
            }
        }
    }
    void unlock() { held.store(false, std::memory_order_release); }
};
using FilterGuard = std::lock_guard<FilterLock>;

// Freed filters' device word arrays, kept per device for the next filter of a similar size
// (flushes and compactions create filters of a few sizes over and over); at most 256 MiB.
struct DevWordsPool {
    std::mutex mu;
    struct Buf {
        int device;
        void *p;
        uint64_t bytes;
    };
    std::vector<Buf> free;
    uint64_t total = 0;
    static constexpr uint64_t kCap = 256ull << 20;
    void *take(int device, uint64_t bytes, uint64_t *got) {
        std::lock_guard<std::mutex> g(mu);
        size_t best = free.size();
        for (size_t i = 0; i < free.size(); ++i)
            if (free[i].device == device && free[i].bytes >= bytes && free[i].bytes <= 2 * bytes &&
                (best == free.size() || free[i].bytes < free[best].bytes))
                best = i;
        if (best == free.size()) return nullptr;
        void *p = free[best].p;
        *got = free[best].bytes;
        total -= free[best].bytes;
        free.erase(free.begin() + best);
        return p;
    }
    bool give(int device, void *p, uint64_t bytes) {
        std::lock_guard<std::mutex> g(mu);
        if (total + bytes > kCap) return false;
        free.push_back({device, p, bytes});
        total += bytes;
        return true;
    }
};
static DevWordsPool g_words_pool;

// A filter handle.  Writers (Add, flush, Encode's host sync) hold `mu`.  A single-key MayContain
// does not: once the host copy reflects every Add (no pending keys, host_ok) and the filter is
// usable, `readable` is published (release) and MayContain answers from `host` with no lock, as
// the reference's MayContain runs lock-free from many goroutines (lsm/lsm.go:166 drops the RLock
// before the SSTable loop).  `host` is sized once, at New/Decode, and never reallocated, so a
// reader can never see freed memory; a reader racing an Add on the same filter sees bits of
// either state, which is the reference's own contract (an unsynchronised Go Add/MayContain pair
// is a data race there).
//
// Deferred Adds go to a host arena.  While every key has one length (the reference's SSTable keys
// usually do) the arena is a fixed-stride batch and no offsets are kept: the build reads it as
// such (16-B keys take the vector path), and the H2D copy carries the key bytes only.  The first
// key of another length materialises the offsets.
constexpr uint64_t kNoLen = UINT64_MAX, kMixedLen = UINT64_MAX - 1;
struct seb_filter {
    FilterLock mu;
    uint64_t m = 0;
    uint32_t k = 0;
    uint64_t mu_m = 0, c_m = 0;  // floor((2^64-1)/m), 2^64 mod m: the host MayContain's reductions
    uint64_t nbytes = 0;  // len(bits): ceil(m/8) for New, len(data)-12 for Decode
    int device = 0;
    uint32_t *dwords = nullptr;  // HBM copy, authoritative once allocated
    uint64_t dbytes = 0;
    std::vector<uint8_t> host;  // host copy (valid when host_ok); nbytes long for the handle's life
    bool host_ok = true;
    bool host_zero = false;     // New, nothing built yet: the device copy starts as a memset
    std::atomic<bool> readable{false};  // host_ok, nothing pending, usable: lock-free MayContain
    std::unique_ptr<uint8_t[]> pend; // deferred Add arena: pend_bytes of pend_capb used
    uint64_t pend_bytes = 0, pend_capb = 0;
    std::vector<uint64_t> pend_off;  // n+1 offsets into pend, only once lengths differ
    uint64_t pend_n = 0;
    uint64_t pend_len = kNoLen;      // the common key length, or kMixedLen
    uint64_t pend_cap = 64ull << 20;
};

static void set_moduli(seb_filter *f) {
    if (f->m) {
        f->mu_m = UINT64_MAX / f->m;
        f->c_m = (0 - f->m) % f->m;
    }
}

static bool usable_quiet(const seb_filter *f) {
    return f->m != 0 && f->k <= 4096 && f->nbytes >= seb_num_bytes(f->m);
}

static void publish_locked(seb_filter *f) {
    f->readable.store(f->host_ok && f->pend_n == 0 && usable_quiet(f), std::memory_order_release);
}

// x mod m with mu = floor((2^64-1)/m): the Barrett estimate is at most 2 low.
static inline uint64_t host_mod(uint64_t x, uint64_t m, uint64_t mu) {
    const uint64_t q = (uint64_t)(((unsigned __int128)x * mu) >> 64);
    uint64_t r = x - q * m;
    if (r >= m) r -= m;
    if (r >= m) r -= m;
    return r;
}

// lsm/bloom.go:82-92 for one key on the host copy: hash1 = FNV-1a 64, hash2 = FNV-1 64
// (:44-54), positions (h1 + i*h2) mod m with u64 wraparound (:58-67), LSB-first bit test
// (:87), false at the first clear bit.  The positions are stepped incrementally: with
// r = (h1 + i*h2) mod m and b = h2 mod m, the next residue is r + b mod m, less 2^64 mod m when
// the u64 sum h1 + (i+1)*h2 wrapped: two Barrett reductions per key instead of k divisions.
static int host_may_contain(const seb_filter *f, const uint8_t *key, uint64_t len) {
    const uint8_t *bits = f->host.data();
    const uint64_t m = f->m, c = f->c_m;
    const uint32_t k = f->k;
    uint64_t h1 = 0xcbf29ce484222325ull, h2 = 0xcbf29ce484222325ull;
    const uint64_t P = 0x100000001b3ull;
    for (uint64_t i = 0; i < len; ++i) {
        h1 = (h1 ^ key[i]) * P;
        h2 = (h2 * P) ^ key[i];
    }
    if (k == 0) return 1;  // no positions: the reference's loop never returns false
    uint64_t r = host_mod(h1, m, f->mu_m);
    const uint64_t b = host_mod(h2, m, f->mu_m);
    uint64_t s = h1;
    for (uint32_t i = 0;;) {
        if (!(bits[r >> 3] & (1u << (r & 7)))) return 0;
        if (++i >= k) return 1;
        const uint64_t s2 = s + h2;
        const bool wrap = s2 < s;
        s = s2;
        uint64_t t = r + b;
        if (t < r || t >= m) t -= m;  // r, b < m: one subtract, also when r + b overflowed
        if (wrap) t = t >= c ? t - c : t + (m - c);
        r = t;
    }
}

// The device word array, on `s`: a pooled or new buffer, zeroed, then the host bits unless the
// filter is a fresh New (all zero).
static int ensure_device_copy(seb_filter *f, hipStream_t s, bool clear = true) {
    if (f->dwords) return SEB_OK;
    HIP_OR_FAIL(hipSetDevice(f->device));
    uint64_t want = std::max<uint64_t>(seb_words_bytes(f->m), (f->nbytes + 15) / 16 * 16);
    if (want == 0) want = 16;
    uint64_t got = 0;
    void *p = g_words_pool.take(f->device, want, &got);
    if (!p) {
        hipError_t e = hipMalloc(&p, want);
        if (e != hipSuccess) {
            (void)hipGetLastError();
            return fail(SEB_ERR_NOMEM, "filter: hipMalloc(%llu): %s", (unsigned long long)want, hipGetErrorString(e));
        }
        got = want;
    }
    f->dwords = (uint32_t *)p;
    f->dbytes = got;
    if (f->host_zero) {
        if (clear) HIP_OR_FAIL(hipMemsetAsync(f->dwords, 0, f->dbytes, s));
    } else {
        const uint64_t tail = f->nbytes & ~15ull;  // zero the padding past the copied bytes
        HIP_OR_FAIL(hipMemsetAsync((uint8_t *)f->dwords + tail, 0, f->dbytes - tail, s));
        if (f->nbytes) HIP_OR_FAIL(hipMemcpyAsync(f->dwords, f->host.data(), f->nbytes, hipMemcpyHostToDevice, s));
    }
    return SEB_OK;
}

static int usable(seb_filter *f, const char *who) {
    int rc = check_filter_args(f->m, f->k, who);
    if (rc) return rc;
    if (f->nbytes < seb_num_bytes(f->m))
        return fail(SEB_ERR_SHORT, "%s: decoded bits (%llu B) shorter than ceil(numBits/8) (%llu B); the reference "
                    "panics (index out of range)", who, (unsigned long long)f->nbytes,
                    (unsigned long long)seb_num_bytes(f->m));
    return SEB_OK;
}

// OR host keys into the filter's device words on a pooled context; returns when the build is done.
// `fresh`: the filter is a New with nothing built, and its device words are taken without a clear
// (the build writes them whole or clears them itself); host_zero stays set until the build
// succeeded (build_into_filter drops such a device copy on failure, so a retry starts clean).
static int build_into_filter_device_on(seb_ctx *c, seb_filter *f, const seb_keys *kb, bool fresh);

// On failure the context's stream is drained before the lease goes back, so nothing queued by this
// build can still write the filter's device words when drop_device_copy hands them to the pool;
// only this stream is waited for (no device-wide synchronisation, which would stall other threads'
// work and break their stream captures).
static int build_into_filter_device(seb_filter *f, const seb_keys *kb, bool fresh) {
    if (options().fault_inject)
        return fail(options().fault_inject == 2 ? SEB_ERR_INTERNAL : SEB_ERR_DEVICE,
                    "BloomFilter build: injected %s (fault_inject)",
                    options().fault_inject == 2 ? "internal error" : "device fault");
    CtxLease L(f->device);
    if (L.rc) return L.rc;
    std::lock_guard<std::mutex> g(L.c->mu);
    HIP_OR_FAIL(hipSetDevice(f->device));
    const int rc = build_into_filter_device_on(L.c, f, kb, fresh);
    if (rc != SEB_OK) {
        (void)hipStreamSynchronize(L.c->s_comp);
        (void)hipGetLastError();
    }
    return rc;
}

static int build_into_filter_device_on(seb_ctx *c, seb_filter *f, const seb_keys *kb, bool fresh) {
    int rc;
    // a new filter's first build writes its words whole (image build) or clears them first: no
    // separate memset of the device copy
    if ((rc = ensure_device_copy(f, c->s_comp, !fresh))) return rc;
    f->host_ok = false;  // the device copy is about to move ahead of the host copy
    f->readable.store(false, std::memory_order_relaxed);
    // Small builds skip the DMA engine, whose copies started ~8 us (keys in) and ~16 us (bits out)
    // after the work before them ended (profiles/r03_flush_trace.txt).  Keys: a device-scope-atomic
    // build (flush sizes, one thread per key, hundreds of workgroups) reads them straight from
    // host-pinned staging over PCIe; the LDS builds (a dozen workgroups) read too few at a time for
    // that and get a DMA copy.  Bits: a kernel writes filters up to 16 MiB into pinned memory.
    const ModArg md = mod_arg(f->m, f->k);
    const uint64_t kbytes = kb->offsets ? kb->offsets[kb->n] - kb->offsets[0] : kb->n * (uint64_t)kb->stride;
    const uint64_t obytes = kb->offsets ? (kb->n + 1) * 8 : 0;
    const bool zc_keys = choose_build_algo(kb->n, f->m, f->k) == 1 && kbytes <= (16ull << 20) &&
                         obytes <= (8ull << 20) && !(kb->offsets && kb->n >= options().varlen_prehash_min_keys);
    const bool zc_bits = f->nbytes <= (16ull << 20);
    const bool mirror = f->nbytes <= (64ull << 20);
    if (zc_keys) {
        const uint64_t kpad = (kbytes + 15) & ~15ull;
        if ((rc = c->hkeys.reserve(kpad + obytes + 16))) return rc;
        uint8_t *hk = (uint8_t *)c->hkeys.p;
        if (kbytes) memcpy(hk, kb->data + (kb->offsets ? kb->offsets[0] : 0), kbytes);
        KeyBatch dk{(const uint8_t *)c->hkeys.dev, nullptr, kb->n, kb->stride};
        if (kb->offsets) {
            uint64_t *ho = (uint64_t *)(hk + kpad);
            const uint64_t o0 = kb->offsets[0];
            for (uint64_t i = 0; i <= kb->n; ++i) ho[i] = kb->offsets[i] - o0;
            dk.offsets = (const uint64_t *)((uint8_t *)c->hkeys.dev + kpad);
        }
        rc = build_dispatch(dk, f->dwords, md, c->s_comp, c->ws.p, c->ws.cap,
                            [&](uint64_t need, void **out) -> int {
                                HIP_OR_FAIL(hipStreamSynchronize(c->s_comp));
                                int r = c->ws.reserve(need, true);
                                *out = c->ws.p;
                                return r;
                            }, fresh);
        if (rc) return rc;
    } else if ((rc = build_device_from_host(c, kb, f->dwords, md, fresh))) {
        return rc;
    }
    // the host copy follows in the same stream (Encode or a first MayContain comes next on the
    // flush path): one synchronisation for build and copy
    if (zc_bits) {
        if ((rc = c->hbits.reserve(f->nbytes + 16))) return rc;
        HIP_OR_FAIL(launch_copy_out(f->dwords, (uint8_t *)c->hbits.dev, f->nbytes, c->s_comp));
    } else if (mirror && f->nbytes) {
        HIP_OR_FAIL(hipMemcpyAsync(f->host.data(), f->dwords, f->nbytes, hipMemcpyDeviceToHost, c->s_comp));
    }
    HIP_OR_FAIL(hipStreamSynchronize(c->s_comp));
    if (zc_bits && f->nbytes) memcpy(f->host.data(), c->hbits.p, f->nbytes);
    f->host_ok = mirror;
    f->host_zero = false;
    return SEB_OK;
}

// The boundary's CPU fallback (SURVEY.md 8(b) error row): the Go API has no error returns
// (lsm/bloom.go:19-41,70-77,96-102 never fail on valid input), so a build or batched probe whose
// device path fails for want of a device or of memory is done on the filter's host copy instead,
// with the same arithmetic as host_may_contain.  Every use is counted (seb_fallback_count); the
// GPU tests and smoke() assert that the count stays 0, so the parity they show is the HIP path's.
static std::atomic<uint64_t> g_fallbacks{0};

extern "C" uint64_t seb_fallback_count(void) { return g_fallbacks.load(std::memory_order_relaxed); }

static bool device_failure(int rc) { return rc == SEB_ERR_DEVICE || rc == SEB_ERR_NOMEM; }

// Counts a fallback; the first one in the process is also written to stderr with its cause (the
// failing call's seb_last_error), so a deployment sees it without reading the counter.
static void note_fallback(const char *who) {
    if (g_fallbacks.fetch_add(1, std::memory_order_relaxed) == 0)
        fprintf(stderr, "seb_bloom: %s fell back to the host copy (CPU) after a device failure: %s\n", who,
                t_err.c_str());
}

// lsm/bloom.go:70-77 for one key on the host copy: positions stepped as in host_may_contain
// ((h1 + i*h2) mod m with u64 wraparound, :58-67), LSB-first byte ORs (:73-75).
static void host_add_key(seb_filter *f, const uint8_t *key, uint64_t len) {
    uint8_t *bits = f->host.data();
    const uint64_t m = f->m, c = f->c_m;
    const uint32_t k = f->k;
    uint64_t h1 = 0xcbf29ce484222325ull, h2 = 0xcbf29ce484222325ull;
    const uint64_t P = 0x100000001b3ull;
    for (uint64_t i = 0; i < len; ++i) {
        h1 = (h1 ^ key[i]) * P;
        h2 = (h2 * P) ^ key[i];
    }
    uint64_t r = host_mod(h1, m, f->mu_m);
    const uint64_t b = host_mod(h2, m, f->mu_m);
    uint64_t s = h1;
    for (uint32_t i = 0; i < k; ++i) {
        bits[r >> 3] |= (uint8_t)(1u << (r & 7));
        const uint64_t s2 = s + h2;
        const bool wrap = s2 < s;
        s = s2;
        uint64_t t = r + b;
        if (t < r || t >= m) t -= m;
        if (wrap) t = t >= c ? t - c : t + (m - c);
        r = t;
    }
}

static const uint8_t *host_key(const seb_keys *kb, uint64_t i, uint64_t *len) {
    if (kb->offsets) {
        *len = kb->offsets[i + 1] - kb->offsets[i];
        return kb->data + kb->offsets[i];
    }
    *len = kb->stride;
    return kb->data + i * (uint64_t)kb->stride;
}

// Give the device word array back: a copy that is garbage (a fresh build that failed) or stale
// (the host copy moved ahead in a fallback).  Its only writer, the failed build's stream, was
// drained before that build's lease ended (build_into_filter_device).  The next device use
// uploads the host copy again (ensure_device_copy).
static void drop_device_copy(seb_filter *f) {
    if (!f->dwords) return;
    (void)hipSetDevice(f->device);
    if (!g_words_pool.give(f->device, f->dwords, f->dbytes)) (void)hipFree(f->dwords);
    (void)hipGetLastError();
    f->dwords = nullptr;
    f->dbytes = 0;
}

static int build_into_filter(seb_filter *f, const seb_keys *kb) {
    const bool fresh = f->host_zero && !f->dwords;
    const bool host_was_ok = f->host_ok;
    int rc = build_into_filter_device(f, kb, fresh);
    if (rc == SEB_OK) return SEB_OK;
    if (fresh) {  // its device words were never cleared: back to a New's state, so a retry starts from zeros
        drop_device_copy(f);
        if (f->nbytes) memset(f->host.data(), 0, f->nbytes);
        f->host_ok = true;
    }
    // Otherwise the device copy (authoritative while host_ok is false) holds the old bits ORed with
    // part of this batch at most, and the batch stays pending: a retry ORs it whole.
    if (!device_failure(rc) || !options().cpu_fallback || !(fresh || host_was_ok) || f->nbytes < seb_num_bytes(f->m))
        return rc;  // no usable host copy to fall back on (a large filter whose device copy is ahead)
    // The host copy holds the bits before this build, or (a D2H that ran before the failure) those
    // ORed with some of this batch's: OR-ing the whole batch into it gives the right filter.
    for (uint64_t i = 0; i < kb->n; ++i) {
        uint64_t len;
        const uint8_t *key = host_key(kb, i, &len);
        host_add_key(f, key, len);
    }
    drop_device_copy(f);
    f->host_ok = true;
    f->host_zero = false;
    note_fallback("BloomFilter build");
    (void)hipGetLastError();
    return SEB_OK;
}

static int flush_locked(seb_filter *f) {
    if (f->pend_n == 0) return SEB_OK;
    int rc = usable(f, "BloomFilter.Add");
    if (rc) return rc;
    const bool uniform = f->pend_len != kMixedLen;
    seb_keys kb{f->pend.get(), uniform ? nullptr : f->pend_off.data(), f->pend_n,
                uniform ? (uint32_t)f->pend_len : 0u, 0};
    if ((rc = build_into_filter(f, &kb))) return rc;
    f->pend_bytes = 0;
    f->pend_off.clear();
    f->pend_n = 0;
    f->pend_len = kNoLen;
    publish_locked(f);
    return SEB_OK;
}

// Room for `more` bytes in the Add arena (doubling); false when memory runs out.
static bool arena_reserve(seb_filter *f, uint64_t more) {
    if (f->pend_bytes + more <= f->pend_capb) return true;
    uint64_t cap = std::max<uint64_t>({f->pend_bytes + more, 2 * f->pend_capb, 4096});
    uint8_t *p = new (std::nothrow) uint8_t[cap];
    if (!p) return false;
    if (f->pend_bytes) memcpy(p, f->pend.get(), f->pend_bytes);
    f->pend.reset(p);
    f->pend_capb = cap;
    return true;
}

extern "C" seb_filter *seb_filter_new(int64_t n, double p) {
    uint64_t m;
    uint32_t k;
    if (seb_params(n, p, &m, &k) != SEB_OK) return nullptr;
    seb_filter *f = new (std::nothrow) seb_filter();
    if (!f) return nullptr;
    f->m = m;
    f->k = k;
    set_moduli(f);
    f->nbytes = seb_num_bytes(m);
    f->device = default_device();
    f->host.assign(f->nbytes, 0);
    f->host_zero = true;
    long cap;
    if (env_flag("SEB_PENDING_CAP", &cap) && cap > 0) f->pend_cap = (uint64_t)cap;
    // the caller's expectedKeys: room for that many 16-B keys (the arena still grows past it)
    if (n > 0) (void)arena_reserve(f, std::min<uint64_t>((uint64_t)n * 16, f->pend_cap));
    publish_locked(f);  // an empty filter answers false everywhere
    return f;
}

extern "C" void seb_filter_free(seb_filter *f) {
    if (!f) return;
    if (f->dwords && !g_words_pool.give(f->device, f->dwords, f->dbytes)) {
        (void)hipSetDevice(f->device);
        (void)hipFree(f->dwords);
    }
    delete f;
}

extern "C" int seb_filter_add(seb_filter *f, const uint8_t *key, uint64_t len) {
    if (!f || (!key && len)) return fail(SEB_ERR_INVALID, "BloomFilter.Add: null argument");
    FilterGuard g(f->mu);
    if (__builtin_expect(!usable_quiet(f), 0)) return usable(f, "BloomFilter.Add");
    f->readable.store(false, std::memory_order_relaxed);  // pending keys: MayContain must flush first
    if (len != f->pend_len) {
        if (f->pend_len == kNoLen && len <= 0xffffffffull) {
            f->pend_len = len;
        } else if (f->pend_len != kMixedLen) {  // the first key of another length: keep offsets from here
            f->pend_off.resize(f->pend_n + 1);
            for (uint64_t i = 0; i <= f->pend_n; ++i) f->pend_off[i] = i * f->pend_len;
            f->pend_len = kMixedLen;
        }
    }
    if (!arena_reserve(f, len)) return fail(SEB_ERR_NOMEM, "BloomFilter.Add: arena of %llu B", (unsigned long long)len);
    uint8_t *dst = f->pend.get() + f->pend_bytes;
    if (len == 16)
        memcpy(dst, key, 16);  // the reference's fixed-size keys: one 16-B move
    else if (len)
        memcpy(dst, key, len);
    f->pend_bytes += len;
    ++f->pend_n;
    if (f->pend_len == kMixedLen) f->pend_off.push_back(f->pend_bytes);
    if (f->pend_bytes >= f->pend_cap || f->pend_n >= (1ull << 32)) return flush_locked(f);
    return SEB_OK;
}

extern "C" int seb_filter_add_batch(seb_filter *f, const seb_keys *kb) {
    if (!f) return fail(SEB_ERR_INVALID, "BloomFilter.Add: null filter");
    int rc;
    if ((rc = check_keys(kb, "BloomFilter.Add")) || (rc = validate_offsets(kb, "BloomFilter.Add"))) return rc;
    FilterGuard g(f->mu);
    if ((rc = usable(f, "BloomFilter.Add"))) return rc;
    if ((rc = flush_locked(f))) return rc;  // keep Add order: earlier single Adds first
    if (kb->n == 0) return SEB_OK;
    if ((rc = build_into_filter(f, kb))) return rc;
    publish_locked(f);
    return SEB_OK;
}

static int probe_filter_device(seb_filter *f, const seb_keys *kb, uint8_t *out) {
    if (options().fault_inject)
        return fail(options().fault_inject == 2 ? SEB_ERR_INTERNAL : SEB_ERR_DEVICE,
                    "BloomFilter probe: injected %s (fault_inject)",
                    options().fault_inject == 2 ? "internal error" : "device fault");
    CtxLease L(f->device);
    if (L.rc) return L.rc;
    std::lock_guard<std::mutex> g2(L.c->mu);
    HIP_OR_FAIL(hipSetDevice(f->device));
    int rc;
    if ((rc = ensure_device_copy(f, L.c->s_comp))) return rc;
    return probe_device_to_host(L.c, kb, f->dwords, mod_arg(f->m, f->k), out);
}

extern "C" int seb_filter_may_contain_batch(seb_filter *f, const seb_keys *kb, uint8_t *out) {
    WsCall ws_call;
    if (!f) return fail(SEB_ERR_INVALID, "BloomFilter.MayContain: null filter");
    int rc;
    if ((rc = check_keys(kb, "BloomFilter.MayContain")) || (rc = validate_offsets(kb, "BloomFilter.MayContain")))
        return rc;
    if (!out && kb->n) return fail(SEB_ERR_INVALID, "BloomFilter.MayContain: null out");
    FilterGuard g(f->mu);
    if ((rc = usable(f, "BloomFilter.MayContain"))) return rc;
    if ((rc = flush_locked(f))) return rc;
    rc = probe_filter_device(f, kb, out);
    if (rc == SEB_OK || !device_failure(rc) || !options().cpu_fallback || !f->host_ok) return rc;
    for (uint64_t i = 0; i < kb->n; ++i) {  // the boundary's CPU fallback (see build_into_filter)
        uint64_t len;
        const uint8_t *key = host_key(kb, i, &len);
        out[i] = (uint8_t)host_may_contain(f, key, len);
    }
    note_fallback("BloomFilter.MayContain batch");
    (void)hipGetLastError();
    return SEB_OK;
}

static int sync_host_locked(seb_filter *f);

// MayContain(key) (lsm/bloom.go:82-92), called once per Get per candidate SSTable
// (lsm/sstable.go:206): answered on the host copy, lock-free once the filter is readable.  A GPU
// launch costs microseconds against ~100 ns for this; batches go to the GPU
// (seb_filter_may_contain_batch).
extern "C" int seb_filter_may_contain(seb_filter *f, const uint8_t *key, uint64_t len) {
    if (!f) return fail(SEB_ERR_INVALID, "BloomFilter.MayContain: null filter");
    if (!key && len) return fail(SEB_ERR_INVALID, "BloomFilter.MayContain: null key");
    if (!f->readable.load(std::memory_order_acquire)) {
        FilterGuard g(f->mu);
        int rc;
        if ((rc = usable(f, "BloomFilter.MayContain")) || (rc = flush_locked(f)) || (rc = sync_host_locked(f)))
            return rc;
        publish_locked(f);
    }
    return host_may_contain(f, key, len);
}

static int sync_host_locked(seb_filter *f) {
    if (f->host_ok) return SEB_OK;
    HIP_OR_FAIL(hipSetDevice(f->device));
    if (f->nbytes) HIP_OR_FAIL(hipMemcpy(f->host.data(), f->dwords, f->nbytes, hipMemcpyDeviceToHost));
    f->host_ok = true;
    publish_locked(f);
    return SEB_OK;
}

extern "C" uint64_t seb_filter_encoded_size(seb_filter *f) { return f ? 12 + f->nbytes : 0; }

extern "C" int seb_filter_encode(seb_filter *f, uint8_t *out, uint64_t cap) {
    if (!f || !out) return fail(SEB_ERR_INVALID, "BloomFilter.Encode: null argument");
    FilterGuard g(f->mu);
    if (cap < 12 + f->nbytes) return fail(SEB_ERR_INVALID, "BloomFilter.Encode: buffer too small");
    int rc;
    if ((rc = flush_locked(f)) || (rc = sync_host_locked(f))) return rc;
    for (int b = 0; b < 8; ++b) out[b] = (uint8_t)(f->m >> (8 * b));  // binary.LittleEndian
    for (int b = 0; b < 4; ++b) out[8 + b] = (uint8_t)(f->k >> (8 * b));
    if (f->nbytes) memcpy(out + 12, f->host.data(), f->nbytes);
    return SEB_OK;
}

extern "C" seb_filter *seb_filter_decode(const uint8_t *data, uint64_t len) {
    if (!data || len < 12) {
        fail(SEB_ERR_INVALID, "DecodeBloomFilter: %llu bytes < 12 (Go returns nil)", (unsigned long long)len);
        return nullptr;
    }
    seb_filter *f = new (std::nothrow) seb_filter();
    if (!f) return nullptr;
    for (int b = 0; b < 8; ++b) f->m |= (uint64_t)data[b] << (8 * b);
    for (int b = 0; b < 4; ++b) f->k |= (uint32_t)data[8 + b] << (8 * b);
    f->nbytes = len - 12;
    set_moduli(f);
    f->device = default_device();
    f->host.assign(data + 12, data + len);
    publish_locked(f);  // immutable from here unless Add is called on it
    return f;
}

extern "C" uint64_t seb_filter_num_bits(const seb_filter *f) { return f ? f->m : 0; }
extern "C" uint32_t seb_filter_num_hashes(const seb_filter *f) { return f ? f->k : 0; }
extern "C" uint64_t seb_filter_pending(seb_filter *f) {
    if (!f) return 0;
    FilterGuard g(f->mu);
    return f->pend_n;
}
extern "C" int seb_filter_flush(seb_filter *f) {
    if (!f) return fail(SEB_ERR_INVALID, "flush: null filter");
    FilterGuard g(f->mu);
    return flush_locked(f);
}

// --------------------------------- device-resident filter registry + batched MultiGet --------
// SURVEY.md §8(f) rows 1-2.  Each SSTable's bloom block (its Encode() bytes, read at
// lsm/sstable.go:121-129) is decoded straight into HBM once; the level layout mirrors
// lsm/levels.go: level 0 in insertion order (AddSSTable appends, :53), levels 1..4 sorted by
// MinKey (:56-60; ties keep insertion order).  seb_registry_multiget answers, for a whole key
// batch, which registered files LSM.Get would consult and which of their filters may contain the
// key (lsm/lsm.go:168-198).

struct RegEntry {
    uint64_t file_num = 0, seq = 0;
    int level = 0;
    uint32_t slot = 0;
    uint64_t m = 0;
    uint32_t k = 0;
    uint32_t *dwords = nullptr;
    std::string min_key, max_key;
};

struct seb_registry {
    std::mutex mu;
    int device = 0;
    std::vector<RegEntry> entries;
    uint64_t seq = 0;
    bool dirty = true;
    DevBuf dslots, dranges;
    DevBuf dl0;                    // the L0 group's interleaved table (RegLayout::l0tab)
    DevBuf dbrange;                // per partition bucket, each disjoint level's bisection range (MgSeg::brange)
    bool has_brange = false;
    uint32_t nslots = 0;
    uint32_t max_cand = 0;         // longest Get walk: every L0 file + one file per non-empty level 1..4
    uint32_t max_slot = 0;         // 1 + the largest slot id in use (the mask form needs <= 64)
    uint32_t part_lo = 0, part_hi = 0;  // multiget_order's partition level: lookup-ordered slots [lo, hi)
    RegLayout layout{};
    seb_ctx *ctx = nullptr;
};

static void be_prefix(const std::string &s, uint64_t out[2]) {  // first 16 bytes, big-endian, zero padded
    for (int w = 0; w < 2; ++w) {
        uint64_t v = 0;
        for (int i = 0; i < 8; ++i) {
            const size_t at = (size_t)w * 8 + i;
            v = (v << 8) | (at < s.size() ? (uint8_t)s[at] : 0u);
        }
        out[w] = v;
    }
}

extern "C" seb_registry *seb_registry_new(int device) {
    seb_registry *r = new (std::nothrow) seb_registry();
    if (!r) return nullptr;
    r->device = device;
    return r;
}

extern "C" void seb_registry_free(seb_registry *r) {
    if (!r) return;
    (void)hipSetDevice(r->device);
    for (auto &e : r->entries) (void)hipFree(e.dwords);
    r->dslots.release();
    r->dranges.release();
    r->dl0.release();
    if (r->ctx) seb_ctx_destroy(r->ctx);
    delete r;
}

extern "C" int seb_registry_put(seb_registry *r, uint64_t file_num, int level, const uint8_t *bloom, uint64_t bloom_len,
                                const uint8_t *min_key, uint64_t min_len, const uint8_t *max_key, uint64_t max_len) {
    if (!r || !bloom || (!min_key && min_len) || (!max_key && max_len))
        return fail(SEB_ERR_INVALID, "seb_registry_put: null argument");
    if (level < 0 || level > 4) return fail(SEB_ERR_INVALID, "seb_registry_put: level %d outside 0..4", level);
    if (bloom_len < 12) return fail(SEB_ERR_INVALID, "seb_registry_put: bloom block < 12 bytes (DecodeBloomFilter: nil)");
    uint64_t m = 0;
    uint32_t k = 0;
    for (int b = 0; b < 8; ++b) m |= (uint64_t)bloom[b] << (8 * b);
    for (int b = 0; b < 4; ++b) k |= (uint32_t)bloom[8 + b] << (8 * b);
    int rc = check_filter_args(m, k, "seb_registry_put");
    if (rc) return rc;
    if (bloom_len - 12 < seb_num_bytes(m)) return fail(SEB_ERR_SHORT, "seb_registry_put: bits shorter than ceil(m/8)");
    std::lock_guard<std::mutex> g(r->mu);
    for (auto &e : r->entries)
        if (e.file_num == file_num) return fail(SEB_ERR_INVALID, "seb_registry_put: file %llu already registered",
                                                (unsigned long long)file_num);
    if (r->entries.size() >= kRegMaxFiles)
        return fail(SEB_ERR_INVALID, "seb_registry_put: registry holds at most %u files", kRegMaxFiles);
    std::vector<char> used(kRegMaxFiles, 0);
    for (auto &e : r->entries) used[e.slot] = 1;
    uint32_t slot = 0;  // lowest free slot: a registry of <= 64 files keeps every slot < 64 (mask form)
    while (used[slot]) ++slot;
    HIP_OR_FAIL(hipSetDevice(r->device));
    RegEntry e;
    e.file_num = file_num;
    e.seq = r->seq++;
    e.level = level;
    e.slot = slot;
    e.m = m;
    e.k = k;
    e.min_key.assign((const char *)min_key, min_len);
    e.max_key.assign((const char *)max_key, max_len);
    const uint64_t wb = seb_words_bytes(m);
    hipError_t a = hipMalloc((void **)&e.dwords, wb);
    if (a != hipSuccess) return (void)hipGetLastError(), fail(SEB_ERR_NOMEM, "seb_registry_put: hipMalloc: %s", hipGetErrorString(a));
    HIP_OR_FAIL(hipMemset(e.dwords, 0, wb));
    HIP_OR_FAIL(hipMemcpy(e.dwords, bloom + 12, seb_num_bytes(m), hipMemcpyHostToDevice));
    r->entries.push_back(std::move(e));
    r->dirty = true;
    return (int)slot;
}

extern "C" int seb_registry_remove(seb_registry *r, uint64_t file_num) {
    if (!r) return fail(SEB_ERR_INVALID, "seb_registry_remove: null registry");
    std::lock_guard<std::mutex> g(r->mu);
    for (size_t i = 0; i < r->entries.size(); ++i)
        if (r->entries[i].file_num == file_num) {
            HIP_OR_FAIL(hipSetDevice(r->device));
            HIP_OR_FAIL(hipDeviceSynchronize());  // no multiget may still read it
            HIP_OR_FAIL(hipFree(r->entries[i].dwords));
            r->entries.erase(r->entries.begin() + i);
            r->dirty = true;
            return SEB_OK;
        }
    return fail(SEB_ERR_INVALID, "seb_registry_remove: file %llu not registered", (unsigned long long)file_num);
}

// Lookup order: level 0 by insertion, then each level 1..4 by (MinKey, insertion).
static std::vector<const RegEntry *> lookup_order(const seb_registry *r) {
    std::vector<const RegEntry *> v;
    for (auto &e : r->entries) v.push_back(&e);
    std::stable_sort(v.begin(), v.end(), [](const RegEntry *a, const RegEntry *b) {
        if (a->level != b->level) return a->level < b->level;
        if (a->level > 0 && a->min_key != b->min_key) return a->min_key < b->min_key;
        return a->seq < b->seq;
    });
    return v;
}

static int sync_registry_locked(seb_registry *r) {
    if (!r->dirty) return SEB_OK;
    HIP_OR_FAIL(hipSetDevice(r->device));
    auto order = lookup_order(r);
    std::vector<RegSlot> slots;
    std::string ranges;
    RegLayout lay{};
    lay.all_k7_m32 = 1;
    for (int L = 0; L < 5; ++L) lay.lo[L] = lay.hi[L] = 0;
    for (size_t i = 0; i < order.size(); ++i) {
        const int L = order[i]->level;
        if (i == 0 || order[i - 1]->level != L) lay.lo[L] = (uint32_t)i;
        lay.hi[L] = (uint32_t)i + 1;
        if (order[i]->k != 7 || order[i]->m >= kM32Limit) lay.all_k7_m32 = 0;
    }
    for (int L = 0; L < 5; ++L)
        if (lay.hi[L] == 0) lay.lo[L] = lay.hi[L] = (uint32_t)order.size();  // empty level
    for (int L = 1; L < 5; ++L) {  // disjoint, MinKey-ordered level: bisection finds the first cover
        bool ok = true;
        for (uint32_t i = lay.lo[L]; i + 1 < lay.hi[L]; ++i)
            ok &= order[i]->min_key <= order[i]->max_key && order[i]->max_key < order[i + 1]->min_key;
        if (lay.hi[L] > lay.lo[L]) ok &= order[lay.hi[L] - 1]->min_key <= order[lay.hi[L] - 1]->max_key;
        if (ok) lay.nonoverlap |= 1u << L;
    }
    for (const RegEntry *e : order) {
        RegSlot s{};
        s.words = e->dwords;
        s.md = mod_arg(e->m, e->k);
        s.min_off = (uint32_t)ranges.size();
        s.min_len = (uint32_t)e->min_key.size();
        ranges += e->min_key;
        s.max_off = (uint32_t)ranges.size();
        s.max_len = (uint32_t)e->max_key.size();
        ranges += e->max_key;
        s.level = e->level;
        s.slot = e->slot;
        s.gbit = -1;
        be_prefix(e->min_key, s.min_be);
        be_prefix(e->max_key, s.max_be);
        slots.push_back(s);
    }
    // L0 group: the largest set of L0 files sharing (m, k) (flushes of equal-sized memtables do;
    // MaxL0Files = 4, lsm/levels.go:9), at most kL0GroupMax, tested through one interleaved table
    std::vector<uint32_t> grp;
    for (uint32_t i = lay.lo[0]; i < lay.hi[0]; ++i) {
        std::vector<uint32_t> same;
        for (uint32_t j = lay.lo[0]; j < lay.hi[0] && same.size() < kL0GroupMax; ++j)
            if (order[j]->m == order[i]->m && order[j]->k == order[i]->k) same.push_back(j);
        if (same.size() > grp.size()) grp = same;
    }
    if (grp.size() < 2) grp.clear();
    uint32_t gbits = 2;
    while (gbits < grp.size()) gbits *= 2;
    int rc;
    if ((rc = r->dslots.reserve(sizeof(RegSlot) * (slots.size() + 1))) ||
        (rc = r->dranges.reserve(ranges.size() + 16)) ||
        (!grp.empty() && (rc = r->dl0.reserve(4 * l0_table_words(order[grp[0]]->m, gbits) + 16))))
        return rc;
    HIP_OR_FAIL(hipDeviceSynchronize());  // previous multigets may still read the tables
    lay.l0g = 0;
    if (!grp.empty()) {
        L0Members mem{};
        for (uint32_t f = 0; f < grp.size(); ++f) {
            mem.w[f] = order[grp[f]]->dwords;
            slots[grp[f]].gbit = (int32_t)f;
        }
        const RegEntry *g0 = order[grp[0]];
        HIP_OR_FAIL(launch_l0_table(mem, (uint32_t)grp.size(), gbits, g0->m, (uint32_t *)r->dl0.p, nullptr));
        HIP_OR_FAIL(hipStreamSynchronize(nullptr));  // MultiGets run on other (non-blocking) streams
        lay.l0tab = (const uint32_t *)r->dl0.p;
        lay.l0md = mod_arg(g0->m, g0->k);
        lay.l0g = (uint32_t)grp.size();
        lay.l0b = gbits;
    }
    if (!slots.empty()) HIP_OR_FAIL(hipMemcpy(r->dslots.p, slots.data(), sizeof(RegSlot) * slots.size(), hipMemcpyHostToDevice));
    if (!ranges.empty()) HIP_OR_FAIL(hipMemcpy(r->dranges.p, ranges.data(), ranges.size(), hipMemcpyHostToDevice));
    r->nslots = (uint32_t)slots.size();
    r->layout = lay;
    r->max_cand = lay.hi[0] - lay.lo[0];
    for (int L = 1; L < 5; ++L) r->max_cand += lay.hi[L] > lay.lo[L] ? 1u : 0u;
    r->max_slot = 0;
    for (const RegEntry *e : order) r->max_slot = std::max(r->max_slot, e->slot + 1);
    r->part_lo = r->part_hi = 0;  // the disjoint level with the most files orders MultiGet batches
    for (int L = 1; L < 5; ++L)
        if ((lay.nonoverlap >> L & 1u) && lay.hi[L] - lay.lo[L] >= 2 && lay.hi[L] - lay.lo[L] < kMgMaxBuckets &&
            lay.hi[L] - lay.lo[L] > r->part_hi - r->part_lo) {
            r->part_lo = lay.lo[L];
            r->part_hi = lay.hi[L];
        }
    // Per bucket b (keys K with MinKey_P[b-1] <= K < MinKey_P[b] of the partition files P) and
    // disjoint level L: A = its files with MinKey <= MinKey_P[b-1], B = those with MinKey <
    // MinKey_P[b]; K's bisection result lies in [A, B].
    r->has_brange = false;
    if (r->part_hi > r->part_lo) {
        const uint32_t nb = r->part_hi - r->part_lo + 1;
        std::vector<uint32_t> br((size_t)nb * 4, 0u);
        for (uint32_t b = 0; b < nb; ++b) {
            const std::string *low = b ? &order[r->part_lo + b - 1]->min_key : nullptr;
            const std::string *high = b + 1 < nb ? &order[r->part_lo + b]->min_key : nullptr;
            for (int L = 1; L < 5; ++L) {
                uint32_t A = 0, B = lay.hi[L] - lay.lo[L];
                if ((lay.nonoverlap >> L & 1u) && lay.hi[L] > lay.lo[L]) {  // MinKey-ordered files
                    const auto f0 = order.begin() + lay.lo[L], f1 = order.begin() + lay.hi[L];
                    if (low)
                        A = (uint32_t)(std::partition_point(f0, f1, [&](const RegEntry *e) { return e->min_key <= *low; }) - f0);
                    if (high)
                        B = (uint32_t)(std::partition_point(f0, f1, [&](const RegEntry *e) { return e->min_key < *high; }) - f0);
                }
                br[(size_t)b * 4 + L - 1] = A | B << 16;
            }
        }
        int brc;
        if ((brc = r->dbrange.reserve(br.size() * 4))) return brc;
        HIP_OR_FAIL(hipMemcpy(r->dbrange.p, br.data(), br.size() * 4, hipMemcpyHostToDevice));
        r->has_brange = true;
    }
    r->dirty = false;
    return SEB_OK;
}

extern "C" int seb_registry_slots(seb_registry *r, uint64_t *file_nums, int32_t *levels, uint32_t cap) {
    if (!r) return fail(SEB_ERR_INVALID, "seb_registry_slots: null registry");
    std::lock_guard<std::mutex> g(r->mu);
    for (uint32_t s = 0; s < cap; ++s) {
        if (file_nums) file_nums[s] = UINT64_MAX;
        if (levels) levels[s] = -1;
    }
    for (auto &e : r->entries)
        if (e.slot < cap) {
            if (file_nums) file_nums[e.slot] = e.file_num;
            if (levels) levels[e.slot] = e.level;
        }
    return (int)r->entries.size();
}

// The layout a MultiGet launches with: the L0 group table only while multiget_l0_group is on.
static RegLayout mg_layout(const seb_registry *r) {
    RegLayout l = r->layout;
    if (!options().multiget_l0_group) l.l0g = 0;
    return l;
}

// multiget_order: the batch's key-range order over the registry's partition level, in the
// stream's scratch (tag 3); mo->active false when off, too small a batch or no disjoint level of
// >= 2 files.  On success kb reads the moved keys, if they were moved.
static std::atomic<uint64_t> g_mg_batch_order{0};
extern "C" uint64_t seb_multiget_order_fallbacks(void) { return g_mg_batch_order.load(std::memory_order_relaxed); }

static bool multiget_ordered(const seb_registry *r, uint64_t n) {
    return options().multiget_order && r->part_hi > r->part_lo && n >= 65536 && n <= 0xffffffffull;
}

static int multiget_order(seb_registry *r, KeyBatch &kb, uint64_t answer_bytes, hipStream_t s, MgOrder *mo) {
    *mo = MgOrder{};
    if (!multiget_ordered(r, kb.n)) return SEB_OK;
    void *ws = nullptr;
    int rc = cached_workspace(s, multiget_order_bytes(kb, answer_bytes, r->part_hi - r->part_lo + 1), &ws, 3);
    if (rc == SEB_ERR_NOMEM) {  // the order is only a speed-up: batch order needs no scratch
        t_err.clear();
        g_mg_batch_order.fetch_add(1, std::memory_order_relaxed);  // seb_multiget_order_fallbacks
        return SEB_OK;
    }
    if (rc) return rc;
    HIP_OR_FAIL(launch_multiget_order(kb, (const RegSlot *)r->dslots.p, r->part_lo, r->part_hi,
                                      (const uint8_t *)r->dranges.p, ws, mo, s));
    if (mo->keys) kb.data = mo->keys;  // the MultiGet streams the moved keys
    return SEB_OK;
}

// One MultiGet launch (mask form: maybe; list form: cand rows of cap u16) over kb, in key-range
// order when the registry has a partition level (answers in sorted rows, then unpermuted into the
// output), else in batch order.
// Largest ordered piece: the order's scratch (bucket ids, tables, sorted keys, sorted-row answers)
// stays near multiget_piece_mib (1 GiB) however large the batch or its rows; a larger batch is
// walked in pieces of whole 2048-key chunks, each in key-range order.

static int multiget_piece(seb_registry *r, KeyBatch kb, uint64_t *maybe, uint16_t *cand, uint32_t cap, hipStream_t s);

static int multiget_launch(seb_registry *r, KeyBatch kb, uint64_t *maybe, uint16_t *cand, uint32_t cap,
                           hipStream_t s) {
    const uint64_t answer_bytes = maybe ? 8 : 2ull * cap;
    const uint64_t scratch = (uint64_t)options().multiget_piece_mib << 20;
    const uint64_t piece = std::max<uint64_t>(65536, (scratch / (answer_bytes + 40)) & ~2047ull);
    if (!multiget_ordered(r, kb.n) || kb.n <= piece) return multiget_piece(r, kb, maybe, cand, cap, s);
    for (uint64_t off = 0; off < kb.n; off += piece) {
        KeyBatch p = kb;
        p.n = std::min(piece, kb.n - off);
        if (kb.offsets)
            p.offsets = kb.offsets + off;  // absolute offsets into the same data
        else
            p.data = kb.data + off * kb.stride;
        if (kb.hashes) p.hashes = kb.hashes + off;
        const int rc = multiget_piece(r, p, maybe ? maybe + off : nullptr, cand ? cand + off * cap : nullptr, cap, s);
        if (rc) return rc;
    }
    return SEB_OK;
}

static int multiget_piece(seb_registry *r, KeyBatch kb, uint64_t *maybe, uint16_t *cand, uint32_t cap,
                          hipStream_t s) {
    const uint64_t answer_bytes = maybe ? 8 : 2ull * cap;
    MgOrder mo;
    int rc;
    if ((rc = multiget_order(r, kb, answer_bytes, s, &mo))) return rc;
    // masks of a registry whose slots are all < 32 travel through the sorted rows as u32 (40 MB
    // less written and read per 10M keys), list rows of 2/4/6/8 slots all < 255 as u8 (6-slot rows:
    // 60 MB); the caller's output keeps its u64 masks / u16 rows
    if (mo.active && maybe && r->max_slot <= 32 && ((uintptr_t)maybe & 7) == 0) mo.narrow = 1;
    if (mo.seg.seg && r->has_brange) mo.seg.brange = (const uint32_t *)r->dbrange.p;
    if (mo.active && !maybe && r->max_slot <= 255 && cap <= 8 && cap % 2 == 0 &&
        ((uintptr_t)cand & (cap == 6 ? 3 : 2 * cap - 1)) == 0)
        mo.narrow = 2;
    HIP_OR_FAIL(launch_multiget(kb, (const RegSlot *)r->dslots.p, r->nslots, mg_layout(r), (const uint8_t *)r->dranges.p,
                                mo.active ? (maybe ? (uint64_t *)mo.answers : nullptr) : maybe,
                                mo.active ? (maybe ? nullptr : (uint16_t *)mo.answers) : cand, cap, s, mo.key_order,
                                mo.seg, mo.narrow != 0));
    if (mo.active)
        HIP_OR_FAIL(launch_multiget_unpermute(mo, maybe ? (void *)maybe : (void *)cand, answer_bytes, s));
    return SEB_OK;
}

// Mask form (maybe != null) or list form (cand, cap u16 per key); called with r->mu held and the
// registry synced.
static int check_multiget_out(seb_registry *r, uint64_t *maybe, uint16_t *cand, uint32_t cap, uint64_t n,
                              const char *who) {
    if (!maybe && !cand && n) return fail(SEB_ERR_INVALID, "%s: null output", who);
    if (maybe && r->max_slot > 64)
        return fail(SEB_ERR_INVALID, "%s: slot %u >= 64 does not fit a u64 mask; use seb_registry_multiget_list",
                    who, r->max_slot - 1);
    if (cand && cap < r->max_cand)
        return fail(SEB_ERR_INVALID, "%s: cap %u < %u candidates a key can have", who, cap, r->max_cand);
    return SEB_OK;
}

static int registry_multiget_dev(seb_registry *r, const seb_keys *keys, uint64_t *maybe, uint16_t *cand, uint32_t cap,
                                 void *stream, const char *who) {
    enter();
    int rc;
    if (!r) return fail(SEB_ERR_INVALID, "%s: null registry", who);
    if ((rc = check_keys(keys, who))) return rc;
    DeviceGuard dg;  // the registry's tables, and so the stream and its scratch, are on r->device
    if ((rc = dg.set(r->device))) return rc;
    WsCall ws_call;
    std::lock_guard<std::mutex> g(r->mu);
    if ((rc = sync_registry_locked(r)) || (rc = check_multiget_out(r, maybe, cand, cap, keys->n, who))) return rc;
    return multiget_launch(r, key_batch(keys), maybe, cand, cap, (hipStream_t)stream);
}

static int registry_multiget_host_locked(seb_registry *r, const seb_keys *kb, uint64_t *maybe, uint16_t *cand,
                                         uint32_t cap);

static int registry_multiget_host(seb_registry *r, const seb_keys *kb, uint64_t *maybe, uint16_t *cand, uint32_t cap,
                                  const char *who) {
    int rc;
    if (!r) return fail(SEB_ERR_INVALID, "%s: null registry", who);
    if ((rc = check_keys(kb, who)) || (rc = validate_offsets(kb, who))) return rc;
    std::lock_guard<std::mutex> g(r->mu);
    if ((rc = sync_registry_locked(r)) || (rc = check_multiget_out(r, maybe, cand, cap, kb->n, who))) return rc;
    return registry_multiget_host_locked(r, kb, maybe, cand, cap);
}

// Host keys through the registry's own context; r->mu held, registry synced, outputs checked.
static int registry_multiget_host_locked(seb_registry *r, const seb_keys *kb, uint64_t *maybe, uint16_t *cand,
                                         uint32_t cap) {
    WsCall ws_call;
    int rc;
    if (!r->ctx && (rc = seb_ctx_create(r->device, &r->ctx))) return rc;
    seb_ctx *c = r->ctx;
    std::lock_guard<std::mutex> g2(c->mu);
    HIP_OR_FAIL(hipSetDevice(c->device));
    const uint64_t per_key = maybe ? 8 : 2ull * cap;
    std::vector<Chunk> chunks;
    plan_chunks(kb, c->chunk_bytes, chunks);
    for (size_t j = 0; j < chunks.size(); ++j) {
        const int b = (int)(j & 1);
        KeyBatch dk{};
        if ((rc = stage_chunk(c, kb, chunks[j], b, &dk, false))) return rc;
        if ((rc = c->out[b].reserve(dk.n * per_key))) return rc;
        HIP_OR_FAIL(hipStreamWaitEvent(c->s_comp, c->ev_d2h[b], 0));
        if ((rc = multiget_launch(r, dk, maybe ? (uint64_t *)c->out[b].p : nullptr,
                                  maybe ? nullptr : (uint16_t *)c->out[b].p, cap, c->s_comp)))
            return rc;
        HIP_OR_FAIL(hipEventRecord(c->ev_comp[b], c->s_comp));
        HIP_OR_FAIL(hipStreamWaitEvent(c->s_d2h, c->ev_comp[b], 0));
        uint8_t *dst = maybe ? (uint8_t *)(maybe + chunks[j].i0) : (uint8_t *)(cand + chunks[j].i0 * cap);
        HIP_OR_FAIL(hipMemcpyAsync(dst, c->out[b].p, dk.n * per_key, hipMemcpyDeviceToHost, c->s_d2h));
        HIP_OR_FAIL(hipEventRecord(c->ev_d2h[b], c->s_d2h));
    }
    HIP_OR_FAIL(hipStreamSynchronize(c->s_d2h));
    return SEB_OK;
}

extern "C" int seb_registry_multiget_dev(seb_registry *r, const seb_keys *keys, uint64_t *maybe, void *stream) {
    if (!maybe && keys && keys->n) return fail(SEB_ERR_INVALID, "seb_registry_multiget: null output");
    return registry_multiget_dev(r, keys, maybe, nullptr, 0, stream, "seb_registry_multiget");
}

extern "C" int seb_registry_multiget(seb_registry *r, const seb_keys *kb, uint64_t *maybe) {
    if (!maybe && kb && kb->n) return fail(SEB_ERR_INVALID, "seb_registry_multiget: null output");
    return registry_multiget_host(r, kb, maybe, nullptr, 0, "seb_registry_multiget");
}

extern "C" int seb_registry_max_candidates(seb_registry *r) {
    if (!r) return fail(SEB_ERR_INVALID, "seb_registry_max_candidates: null registry");
    std::lock_guard<std::mutex> g(r->mu);
    int rc = sync_registry_locked(r);
    return rc ? rc : (int)r->max_cand;
}

extern "C" int seb_registry_multiget_list(seb_registry *r, const seb_keys *kb, uint16_t *cand, uint32_t cap) {
    if (!cand && kb && kb->n) return fail(SEB_ERR_INVALID, "seb_registry_multiget_list: null output");
    return registry_multiget_host(r, kb, nullptr, cand, cap, "seb_registry_multiget_list");
}

// The list form translated to file numbers under ONE hold of the registry lock, so a Put or
// Remove between sizing the rows, running the lookup and mapping slots to files cannot make the
// rows overflow or a freed-and-reused slot name the wrong file (the three-call sequence
// max_candidates / multiget_list / slots is not atomic).
extern "C" int seb_registry_multiget_files(seb_registry *r, const seb_keys *kb, uint64_t *files, uint32_t cap,
                                           uint32_t *need) {
    const char *who = "seb_registry_multiget_files";
    int rc;
    if (!r) return fail(SEB_ERR_INVALID, "%s: null registry", who);
    if ((rc = check_keys(kb, who)) || (rc = validate_offsets(kb, who))) return rc;
    if (!files && kb->n) return fail(SEB_ERR_INVALID, "%s: null output", who);
    std::lock_guard<std::mutex> g(r->mu);
    if ((rc = sync_registry_locked(r))) return rc;
    const uint32_t want = std::max<uint32_t>(r->max_cand, 1);
    if (need) *need = want;
    if (cap < want)
        return fail(SEB_ERR_RANGE, "%s: cap %u < %u candidates a key can have now; retry with *need", who, cap, want);
    if (kb->n == 0) return SEB_OK;
    std::vector<uint16_t> cand(kb->n * (uint64_t)cap);
    if ((rc = registry_multiget_host_locked(r, kb, nullptr, cand.data(), cap))) return rc;
    std::vector<uint64_t> by_slot(kRegMaxFiles, UINT64_MAX);
    for (auto &e : r->entries) by_slot[e.slot] = e.file_num;
    for (uint64_t i = 0; i < cand.size(); ++i) files[i] = cand[i] == 0xFFFF ? UINT64_MAX : by_slot[cand[i]];
    return SEB_OK;
}

extern "C" int seb_registry_multiget_list_dev(seb_registry *r, const seb_keys *keys, uint16_t *cand, uint32_t cap,
                                              void *stream) {
    if (!cand && keys && keys->n) return fail(SEB_ERR_INVALID, "seb_registry_multiget_list: null output");
    return registry_multiget_dev(r, keys, nullptr, cand, cap, stream, "seb_registry_multiget_list");
}

// ------------------------------------------------ shard routing + WAL checksums (§8(f) row 4)

extern "C" int seb_dev_shard_route(const seb_keys *keys, uint32_t bits, uint16_t *shard, uint32_t *hash,
                                   void *stream) {
    enter();
    int rc;
    if ((rc = check_keys(keys, "seb_dev_shard_route"))) return rc;
    if (bits > 16) return fail(SEB_ERR_INVALID, "seb_dev_shard_route: shard_bits %u > 16", bits);
    HIP_OR_FAIL(launch_route(key_batch(keys), bits, shard, hash, (hipStream_t)stream));
    return SEB_OK;
}

extern "C" uint64_t seb_dev_shard_partition_workspace_size(uint64_t n, uint32_t bits) {
    return bits > 12 ? 0 : route_workspace_bytes(n, bits);
}

extern "C" int seb_dev_shard_partition(const seb_keys *keys, uint32_t bits, uint32_t *perm, uint64_t *shard_begin,
                                       uint16_t *shard, void *ws, uint64_t ws_bytes, void *stream) {
    enter();
    int rc;
    if ((rc = check_keys(keys, "seb_dev_shard_partition"))) return rc;
    if (bits > 12) return fail(SEB_ERR_INVALID, "seb_dev_shard_partition: shard_bits %u > 12", bits);
    if (keys->n >= (1ull << 32)) return fail(SEB_ERR_INVALID, "seb_dev_shard_partition: n >= 2^32");
    if (keys->n && (!perm || !ws)) return fail(SEB_ERR_INVALID, "seb_dev_shard_partition: null perm/workspace");
    if (ws_bytes < route_workspace_bytes(keys->n, bits))
        return fail(SEB_ERR_INVALID, "seb_dev_shard_partition: workspace %llu < %llu bytes",
                    (unsigned long long)ws_bytes, (unsigned long long)route_workspace_bytes(keys->n, bits));
    HIP_OR_FAIL(launch_route_partition(key_batch(keys), bits, perm, shard_begin, shard, ws, ws_bytes,
                                       (hipStream_t)stream));
    return SEB_OK;
}

extern "C" int seb_dev_wal_crc(uint8_t *data, const uint64_t *rec_off, uint64_t n, int mode, uint32_t *crc,
                               uint8_t *ok, void *stream) {
    enter();
    if (mode < SEB_WAL_CRC || mode > SEB_WAL_VERIFY) return fail(SEB_ERR_INVALID, "seb_dev_wal_crc: bad mode %d", mode);
    if (n && (!data || !rec_off)) return fail(SEB_ERR_INVALID, "seb_dev_wal_crc: null data/offsets");
    if (n && mode == SEB_WAL_VERIFY && !ok) return fail(SEB_ERR_INVALID, "seb_dev_wal_crc: VERIFY needs ok[]");
    HIP_OR_FAIL(launch_wal_crc(data, rec_off, n, mode, crc, ok, (hipStream_t)stream));
    return SEB_OK;
}

// ReadAll's framing walk (lsm/wal.go:98-121): a 21-byte header, then keySize + valueSize bytes.
extern "C" int seb_wal_scan(const uint8_t *data, uint64_t bytes, uint64_t *rec_off, uint64_t cap, uint64_t *n) {
    if (!n || (bytes && !data)) return fail(SEB_ERR_INVALID, "seb_wal_scan: null argument");
    *n = 0;
    if (cap < 1 || !rec_off) return fail(SEB_ERR_INVALID, "seb_wal_scan: offsets capacity 0");
    uint64_t at = 0, cnt = 0;
    rec_off[0] = 0;
    while (at < bytes) {
        if (bytes - at < 21) {
            *n = cnt;
            return fail(SEB_ERR_SHORT, "seb_wal_scan: truncated header at byte %llu", (unsigned long long)at);
        }
        uint32_t ks, vs;
        memcpy(&ks, data + at + 12, 4);
        memcpy(&vs, data + at + 16, 4);
        const uint64_t len = 21ull + ks + vs;
        if (bytes - at < len) {
            *n = cnt;
            return fail(SEB_ERR_SHORT, "seb_wal_scan: truncated record at byte %llu", (unsigned long long)at);
        }
        if (cnt + 2 > cap) {
            *n = cnt;
            return fail(SEB_ERR_INVALID, "seb_wal_scan: more than %llu records", (unsigned long long)(cap - 1));
        }
        at += len;
        rec_off[++cnt] = at;
    }
    *n = cnt;
    return SEB_OK;
}
