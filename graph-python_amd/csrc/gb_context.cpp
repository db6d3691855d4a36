#include <algorithm>
#include <chrono>
#include <cstdio>
// gb_context.cpp -- library context: init/finalize, the HIP stream, the
// stream-ordered device memory pool, error plumbing, descriptors, builtin
// object lookup.  (Replaces SuiteSparse's GrB_init / GxB_Global / GrB_Descriptor
// surface used by reference graphblas/__init__.py:118-197 and
// core/descriptor.py:92-156.)
#include <cstdio>
#include <cstdlib>
#include <atomic>
#include <map>
#include <mutex>
#include <unordered_map>
#include <vector>

#include <cstring>
#include <dlfcn.h>

#include "gb_internal.h"

namespace {
bool g_init = false;
int g_device = 0;
hipStream_t g_own_stream = nullptr;
hipStream_t g_user_stream = nullptr;
bool g_user_stream_set = false;
std::mutex g_knob_mu;
std::map<std::string, int64_t> g_knobs;
std::atomic<bool> g_any_knob{false};  // no knob ever set: every lookup is 0 without the lock
}  // namespace

static const GrB_Index GB_ALL_SENTINEL = 0;
extern "C" {
const GrB_Index *GrB_ALL = &GB_ALL_SENTINEL;
}

[[noreturn]] void gb_throw(GrB_Info info, const std::string &msg) { throw gb_exception{info, msg}; }

void gb_hip_check(hipError_t e, const char *what) {
    if (e == hipSuccess) return;
    if (e == hipErrorOutOfMemory || e == hipErrorMemoryAllocation) {
        (void)hipGetLastError();
        gb_throw(GrB_OUT_OF_MEMORY, std::string("device out of memory: ") + what);
    }
    gb_throw(GrB_PANIC, std::string("HIP error ") + hipGetErrorString(e) + " in " + what);
}

static void gb_do_init() {
    if (g_init) return;
    const char *dev = getenv("GRAPHBLAS_AMD_DEVICE");
    if (dev) g_device = atoi(dev);
    GB_HIP(hipSetDevice(g_device));
    GB_HIP(hipStreamCreateWithFlags(&g_own_stream, hipStreamNonBlocking));
    // keep freed blocks in the pool (no release to the OS between calls)
    hipMemPool_t pool;
    if (hipDeviceGetDefaultMemPool(&pool, g_device) == hipSuccess) {
        uint64_t thr = UINT64_MAX;
        (void)hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &thr);
    }
    g_init = true;
}

void gb_require_init() {
    if (!g_init) gb_do_init();  // lazy init, like python-graphblas's auto-init
}

static std::atomic<uint64_t> g_epoch{1};
uint64_t gb_epoch() { return g_epoch.load(std::memory_order_relaxed); }

hipStream_t gb_stream() {
    gb_require_init();
    g_epoch.fetch_add(1, std::memory_order_relaxed);  // every caller is about to enqueue work
    return g_user_stream_set ? g_user_stream : g_own_stream;
}
hipStream_t gb_stream_peek() {
    gb_require_init();
    return g_user_stream_set ? g_user_stream : g_own_stream;
}

// ---- host mailboxes (see gb_internal.h)
namespace {
std::mutex g_slot_mu;
std::vector<gb_host_slot *> g_slot_free;
std::vector<std::pair<gb_host_slot *, gb_host_slot *>> g_slot_slabs;  // (host base, device base)
std::atomic<uint64_t> g_pub_seq{0};
const int kSlotsPerSlab = 1024;
}  // namespace

gb_host_slot *gb_host_slot_alloc() {
    std::lock_guard<std::mutex> lk(g_slot_mu);
    if (g_slot_free.empty()) {
        gb_require_init();
        gb_host_slot *h = nullptr, *d = nullptr;
        GB_HIP(hipHostMalloc((void **)&h, kSlotsPerSlab * sizeof(gb_host_slot),
                             hipHostMallocCoherent | hipHostMallocMapped));
        GB_HIP(hipHostGetDevicePointer((void **)&d, h, 0));
        memset(h, 0, kSlotsPerSlab * sizeof(gb_host_slot));
        g_slot_slabs.push_back({h, d});
        for (int i = kSlotsPerSlab - 1; i >= 0; i--) g_slot_free.push_back(h + i);
    }
    gb_host_slot *s = g_slot_free.back();
    g_slot_free.pop_back();
    __atomic_store_n(&s->seq, 0LL, __ATOMIC_RELEASE);  // no word of a previous owner can match
    s->host_last = 0;
    return s;
}

void gb_host_slot_release(gb_host_slot *s) {
    if (!s) return;
    std::lock_guard<std::mutex> lk(g_slot_mu);
    __atomic_store_n(&s->seq, 0LL, __ATOMIC_RELEASE);
    s->host_last = 0;
    g_slot_free.push_back(s);
}

gb_host_slot *gb_host_slot_device(gb_host_slot *s) {
    std::lock_guard<std::mutex> lk(g_slot_mu);
    for (auto &sl : g_slot_slabs)
        if (s >= sl.first && s < sl.first + kSlotsPerSlab) return sl.second + (s - sl.first);
    return nullptr;
}

// A tagged one-word publish carries 31 bits of the sequence number, so a word a slot kept
// from a publish 2^30 or more numbers ago could alias a later one: such a word is cleared before
// the slot's next publish is issued (that old publish has completed: all library work is on one
// stream, and 2^30 launches have been issued behind it).  host_last holds, on the host only, the
// last number issued to the slot (a field no kernel writes: pad[0] carries a device hint).
uint64_t gb_next_pub_seq(gb_host_slot *s) {
    const uint64_t seq = g_pub_seq.fetch_add(1, std::memory_order_relaxed) + 1;
    if (s) {
        const uint64_t last = (uint64_t)s->host_last;
        if (last && seq - last >= (1ULL << 30)) __atomic_store_n(&s->seq, 0LL, __ATOMIC_RELEASE);
        s->host_last = (long long)seq;
    }
    return seq;
}

static inline bool slot_match(gb_host_slot *s, uint64_t seq, int64_t *value) {
    const uint64_t w = (uint64_t)__atomic_load_n(&s->seq, __ATOMIC_ACQUIRE);
    if (w == seq) {
        *value = __atomic_load_n(&s->value, __ATOMIC_RELAXED);
        return true;
    }
    if ((w & GB_PUB_TAG) && ((w >> 32) & 0x7fffffffULL) == (seq & 0x7fffffffULL)) {
        *value = (int64_t)(w & 0xffffffffULL);  // tagged one-word publish
        return true;
    }
    return false;
}

// The stream is asked whether it drained (a publish that never lands: a failed launch) only once
// the wait has lasted `slot_query_us` (default 2000 us, longer than any level's kernel): each
// hipStreamQuery on a busy stream makes the runtime put a marker into the queue behind the
// enqueued kernels, and the GPU then idles ~3.5 us between them (tools/iso_gaps.py: the BFS
// levels after a long wait started 6 us after the previous one ended instead of 2.5 us when the
// query ran every 1024 spins, i.e. on every wait longer than ~40 us).
bool gb_host_slot_wait(gb_host_slot *s, uint64_t seq, int64_t *value) {
    int64_t t0 = 0, query_ns = 0;
    for (uint64_t i = 1;; i++) {
        if (slot_match(s, seq, value)) return true;
        if ((i & 1023) == 0) {
            const int64_t now = std::chrono::duration_cast<std::chrono::nanoseconds>(
                                    std::chrono::steady_clock::now().time_since_epoch()).count();
            if (!t0) {
                t0 = now;
                const int64_t k = gb_knob("slot_query_us");
                query_ns = (k > 0 ? k : 2000) * 1000;
            }
            if (now - t0 >= query_ns) {
                hipError_t q = hipStreamQuery(gb_stream_peek());
                if (q != hipErrorNotReady) return slot_match(s, seq, value);  // drained (or failed): one last look
            }
        }
        __builtin_ia32_pause();
    }
}

void gb_sync() { GB_HIP(hipStreamSynchronize(gb_stream())); }

unsigned long long *gb_device_state() {
    static std::mutex mu;
    static unsigned long long *st = nullptr;
    std::lock_guard<std::mutex> lk(mu);
    if (!st) {
        gb_require_init();
        GB_HIP(hipMalloc(&st, GB_STATE_WORDS * sizeof(unsigned long long)));
        GB_HIP(hipMemset(st, 0, GB_STATE_WORDS * sizeof(unsigned long long)));
        GB_HIP(hipDeviceSynchronize());
    }
    return st;
}

// ---- host-time probes (gb_internal.h)
bool g_hprof_on = getenv("GRAPHBLAS_AMD_HPROF") != nullptr;

// ---- roctx ranges (gb_internal.h: gb_roctx_range)
namespace {
int (*p_roctx_push)(const char *) = nullptr;
int (*p_roctx_pop)() = nullptr;
bool roctx_init() {
    const char *e = getenv("GRAPHBLAS_AMD_ROCTX");
    if (!e || strcmp(e, "1") != 0) return false;
    void *h = dlopen("librocprofiler-sdk-roctx.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) h = dlopen("librocprofiler-sdk-roctx.so", RTLD_NOW | RTLD_GLOBAL);
    if (!h) {
        fprintf(stderr, "graphblas_amd: GRAPHBLAS_AMD_ROCTX=1 but the roctx library is not loadable\n");
        return false;
    }
    p_roctx_push = (int (*)(const char *))dlsym(h, "roctxRangePushA");
    p_roctx_pop = (int (*)())dlsym(h, "roctxRangePop");
    return p_roctx_push && p_roctx_pop;
}
}  // namespace
bool g_roctx_on = roctx_init();
void gb_roctx_push(const char *name) { p_roctx_push(name); }
void gb_roctx_pop() { p_roctx_pop(); }
namespace {
struct hprof_slot {
    std::atomic<int64_t> ns{0}, calls{0};
    const char *name = nullptr;
    std::mutex mu;
    std::vector<int64_t> samples;  // the first 1M durations (median / p10 at exit)
};
hprof_slot g_hprof[32];
struct hprof_print {
    ~hprof_print() {
        if (!g_hprof_on) return;
        for (auto &s : g_hprof)
            if (s.name && s.calls.load()) {
                std::vector<int64_t> v = s.samples;
                std::sort(v.begin(), v.end());
                const double med = v.empty() ? 0.0 : v[v.size() / 2] / 1e3, p10 = v.empty() ? 0.0 : v[v.size() / 10] / 1e3;
                fprintf(stderr, "[hprof] %-28s calls %9lld  mean %8.2f us  median %8.2f  p10 %8.2f\n", s.name,
                        (long long)s.calls.load(), s.ns.load() / 1e3 / (double)s.calls.load(), med, p10);
            }
    }
} g_hprof_print;
}  // namespace
int64_t gb_hprof_now() {
    return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
        .count();
}
void gb_hprof_add(int slot, const char *name, int64_t ns) {
    g_hprof[slot].name = name;
    g_hprof[slot].ns += ns;
    g_hprof[slot].calls += 1;
    std::lock_guard<std::mutex> lk(g_hprof[slot].mu);
    if (g_hprof[slot].samples.size() < (1u << 20)) g_hprof[slot].samples.push_back(ns);
}

namespace {
std::mutex g_named_stat_mu;
std::map<std::string, int64_t> g_named_stats;
}  // namespace
void gb_stat_add(const char *name, int64_t v) {
    std::lock_guard<std::mutex> lk(g_named_stat_mu);
    g_named_stats[name] += v;
}
bool gb_stat_get(const char *name, int64_t *v) {
    std::lock_guard<std::mutex> lk(g_named_stat_mu);
    auto it = g_named_stats.find(name);
    if (it == g_named_stats.end()) return false;
    *v = it->second;
    return true;
}

int64_t gb_knob(const char *key) {
    if (!g_any_knob.load(std::memory_order_acquire)) return 0;
    std::lock_guard<std::mutex> lk(g_knob_mu);
    auto it = g_knobs.find(key);
    return it == g_knobs.end() ? 0 : it->second;
}

// ---- device memory: a size-class cache over the stream-ordered pool.
// Every library kernel runs on one stream, so a block returned to the cache
// can be handed to later work on that stream without any synchronisation
// (stream order retires the old uses first).  This keeps hipFreeAsync (about
// 10 us of host time each, measured in profiles/) off the per-call path.
namespace {
std::mutex g_mem_mu;
struct gb_cached {
    void *p;
    uint64_t seq;  // free order (eviction oldest first)
};
std::unordered_map<void *, size_t> g_live;                    // ptr -> class size
std::unordered_map<size_t, std::vector<gb_cached>> g_cache;  // class size -> idle blocks
std::map<uint64_t, std::pair<void *, size_t>> g_lru;          // seq -> (ptr, class)
uint64_t g_free_seq = 0;
size_t g_cached_bytes = 0;
// Idle bytes kept (of 288 GB HBM).  A block freed over the limit evicts the
// oldest idle blocks rather than being dropped itself: the blocks of the work
// that is running now are the ones the next call asks for again (a 42 GB
// SpGEMM output handed back to the pool and requested again after a run of
// other sizes was split by them and re-mapped fresh: ~2 s per call).
const size_t kCacheLimit = (size_t)96 << 30;
void *g_pinned = nullptr;  // pinned staging for small device->host reads
const size_t kPinned = 1 << 16;
std::mutex g_pin_mu;

size_t size_class(size_t b) {
    if (b < 256) b = 256;
    if (b <= ((size_t)64 << 20)) {
        size_t c = 256;
        while (c < b) c <<= 1;
        return c;
    }
    const size_t g = (size_t)2 << 20;
    return (b + g - 1) / g * g;
}

void release_cache_locked() {
    for (auto &kv : g_cache)
        for (const gb_cached &c : kv.second) (void)hipFreeAsync(c.p, gb_stream());
    g_cache.clear();
    g_lru.clear();
    g_cached_bytes = 0;
}

void evict_oldest_locked() {
    auto it = g_lru.begin();
    void *p = it->second.first;
    const size_t cls = it->second.second;
    g_lru.erase(it);
    auto &v = g_cache[cls];
    for (size_t i = 0; i < v.size(); i++)
        if (v[i].p == p) {
            v.erase(v.begin() + (std::ptrdiff_t)i);
            break;
        }
    g_cached_bytes -= cls;
    (void)hipFreeAsync(p, gb_stream());
}
}  // namespace

void *gb_malloc(size_t bytes) {
    const size_t cls = size_class(bytes);
    std::lock_guard<std::mutex> lk(g_mem_mu);
    auto it = g_cache.find(cls);
    if (it != g_cache.end() && !it->second.empty()) {
        const gb_cached c = it->second.back();
        it->second.pop_back();
        g_lru.erase(c.seq);
        g_cached_bytes -= cls;
        g_live[c.p] = cls;
        return c.p;
    }
    void *p = nullptr;
    hipError_t e = hipMallocAsync(&p, cls, gb_stream());
    if (e != hipSuccess || !p) {
        (void)hipGetLastError();
        release_cache_locked();  // give idle blocks back and retry once
        (void)hipStreamSynchronize(gb_stream());
        e = hipMallocAsync(&p, cls, gb_stream());
        if (e != hipSuccess || !p) {
            (void)hipGetLastError();
            gb_throw(GrB_OUT_OF_MEMORY, "device allocation of " + std::to_string(bytes) + " bytes failed");
        }
    }
    g_live[p] = cls;
    return p;
}

void gb_free(void *p) {
    if (!p) return;
    std::lock_guard<std::mutex> lk(g_mem_mu);
    auto it = g_live.find(p);
    if (it == g_live.end()) {
        (void)hipFreeAsync(p, gb_stream());
        return;
    }
    size_t cls = it->second;
    g_live.erase(it);
    if (cls > kCacheLimit) {
        (void)hipFreeAsync(p, gb_stream());
        return;
    }
    while (g_cached_bytes + cls > kCacheLimit && !g_lru.empty()) evict_oldest_locked();
    const uint64_t seq = ++g_free_seq;
    g_cache[cls].push_back(gb_cached{p, seq});
    g_lru.emplace(seq, std::make_pair(p, cls));
    g_cached_bytes += cls;
}

void gb_memset(void *p, int v, size_t bytes) {
    if (bytes) GB_HIP(hipMemsetAsync(p, v, bytes, gb_stream()));
}
void gb_copy_d2d(void *dst, const void *src, size_t bytes) {
    if (bytes) GB_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, gb_stream()));
}
void gb_copy_h2d(void *dst, const void *src, size_t bytes) {
    if (bytes) GB_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, gb_stream()));
}
void gb_copy_d2h(void *dst, const void *src, size_t bytes) {
    if (bytes && bytes <= kPinned) {
        std::lock_guard<std::mutex> lk(g_pin_mu);
        if (!g_pinned) GB_HIP(hipHostMalloc(&g_pinned, kPinned, hipHostMallocDefault));
        GB_HIP(hipMemcpyAsync(g_pinned, src, bytes, hipMemcpyDeviceToHost, gb_stream()));
        gb_sync();
        memcpy(dst, g_pinned, bytes);
        return;
    }
    if (bytes) GB_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, gb_stream()));
    gb_sync();
}
int64_t gb_read_i64(const int64_t *dptr) {
    int64_t v = 0;
    gb_copy_d2h(&v, dptr, sizeof(v));
    return v;
}

int64_t gb_iso_ts_dump();  // gb_mxv.hip (diagnostics)

static const char *k_type_names[] = {"BOOL", "INT8", "UINT8", "INT16", "UINT16", "INT32",
                                     "UINT32", "INT64", "UINT64", "FP32", "FP64"};
static const size_t k_type_sizes[] = {1, 1, 1, 2, 2, 4, 4, 8, 8, 4, 8};
const char *gb_type_name(int code) { return k_type_names[code]; }
size_t gb_type_size(int code) { return k_type_sizes[code]; }
GrB_Type gb_type_of(int code) {
    switch (code) {
    case GBAMD_T_BOOL: return GrB_BOOL;
    case GBAMD_T_INT8: return GrB_INT8;
    case GBAMD_T_UINT8: return GrB_UINT8;
    case GBAMD_T_INT16: return GrB_INT16;
    case GBAMD_T_UINT16: return GrB_UINT16;
    case GBAMD_T_INT32: return GrB_INT32;
    case GBAMD_T_UINT32: return GrB_UINT32;
    case GBAMD_T_INT64: return GrB_INT64;
    case GBAMD_T_UINT64: return GrB_UINT64;
    case GBAMD_T_FP32: return GrB_FP32;
    default: return GrB_FP64;
    }
}

gb_desc gb_read_desc(const GrB_Descriptor d) {
    gb_desc r;
    if (!d) return r;
    GB_REQUIRE(d->magic == GB_MAGIC, GrB_UNINITIALIZED_OBJECT, "invalid descriptor");
    r.replace = d->outp == GrB_REPLACE;
    r.comp = (d->mask & GrB_COMP) != 0;
    r.structure = (d->mask & GrB_STRUCTURE) != 0;
    r.tran0 = d->inp0 == GrB_TRAN;
    r.tran1 = d->inp1 == GrB_TRAN;
    return r;
}

extern "C" {

static int32_t g_mode = GrB_NONBLOCKING;

GrB_Info GrB_init(GrB_Mode mode) {
    return gb_api(nullptr, [&] {
        GB_REQUIRE(!g_init, GrB_INVALID_VALUE, "GrB_init called twice");
        GB_REQUIRE(mode == GrB_BLOCKING || mode == GrB_NONBLOCKING, GrB_INVALID_VALUE, "invalid mode");
        gb_do_init();
        g_mode = mode;
    });
}

GrB_Info GxB_Global_Option_get_INT32(GxB_Option_Field field, int32_t *value) {
    if (!value) return GrB_NULL_POINTER;
    if (field != GxB_MODE) return GrB_INVALID_VALUE;
    *value = g_mode;
    return GrB_SUCCESS;
}

GrB_Info GrB_finalize(void) {
    return gb_api(nullptr, [&] {
        if (!g_init) return;
        GB_HIP(hipDeviceSynchronize());
    });
}

GrB_Info GrB_getVersion(unsigned int *version, unsigned int *subversion) {
    if (!version || !subversion) return GrB_NULL_POINTER;
    *version = GRB_VERSION;
    *subversion = GRB_SUBVERSION;
    return GrB_SUCCESS;
}

GrB_Info GxB_Context_set_stream(void *hip_stream) {
    return gb_api(nullptr, [&] {
        gb_require_init();
        // cached device blocks are reused in stream order: drain the old stream first
        GB_HIP(hipStreamSynchronize(gb_stream()));
        g_user_stream = (hipStream_t)hip_stream;
        g_user_stream_set = hip_stream != nullptr;
    });
}

GrB_Info GxB_Context_get_stream(void **hip_stream) {
    if (!hip_stream) return GrB_NULL_POINTER;
    return gb_api(nullptr, [&] { *hip_stream = (void *)gb_stream(); });
}

GrB_Info GxB_Context_set_device(int device) {
    if (g_init) return GrB_INVALID_VALUE;
    g_device = device;
    return GrB_SUCCESS;
}

GrB_Info GxB_Global_set_int(const char *key, int64_t value) {
    if (!key) return GrB_NULL_POINTER;
    std::lock_guard<std::mutex> lk(g_knob_mu);
    g_knobs[key] = value;
    g_any_knob.store(true, std::memory_order_release);
    return GrB_SUCCESS;
}

GrB_Info GxB_Global_get_int(const char *key, int64_t *value) {
    if (!key || !value) return GrB_NULL_POINTER;
    // statistics (read-only): BFS level speculation (gb_ops.hip)
    if (!strcmp(key, "stat_bfs_spec_adopted")) {
        *value = g_stat_spec_adopted.load(std::memory_order_relaxed);
        return GrB_SUCCESS;
    }
    if (!strcmp(key, "stat_bfs_spec_rollbacks")) {
        *value = g_stat_spec_rollbacks.load(std::memory_order_relaxed);
        return GrB_SUCCESS;
    }
    // vector counts read with a device copy (stream sync) instead of the kernel's mailbox
    if (!strcmp(key, "stat_spmv_host_push")) {
        *value = g_stat_host_push.load(std::memory_order_relaxed);
        return GrB_SUCCESS;
    }
    if (!strcmp(key, "stat_nvals_copy")) {
        *value = g_stat_nvals_copy.load(std::memory_order_relaxed);
        return GrB_SUCCESS;
    }
    if (!strcmp(key, "iso_ts_dump")) {  // diagnostics: GRAPHBLAS_AMD_ISO_TS (gb_mxv.hip)
        return gb_api(nullptr, [&] { *value = gb_iso_ts_dump(); });
    }
    // named kernel-class counters (gb_stat_add): "stat_" + name; 0 before the first count
    if (!strncmp(key, "stat_", 5)) {
        if (!gb_stat_get(key + 5, value)) *value = 0;
        return GrB_SUCCESS;
    }
    *value = gb_knob(key);
    return GrB_SUCCESS;
}

GrB_Info GxB_builtin_lookup(void **handle, int *kind, const char *name) {
    if (!handle || !kind || !name) return GrB_NULL_POINTER;
    static std::map<std::string, const GB_builtin_entry *> *idx = nullptr;
    static std::mutex mu;
    {
        std::lock_guard<std::mutex> lk(mu);
        if (!idx) {
            idx = new std::map<std::string, const GB_builtin_entry *>();
            for (const GB_builtin_entry *e = GB_builtin_registry; e->name; e++) (*idx)[e->name] = e;
        }
    }
    auto it = idx->find(name);
    if (it == idx->end()) return GrB_INVALID_VALUE;
    *handle = it->second->obj;
    *kind = it->second->kind;
    return GrB_SUCCESS;
}

GrB_Info GxB_name(const char **name, const void *obj) {
    if (!name || !obj) return GrB_NULL_POINTER;
    // every builtin struct starts with magic; the name field position differs per kind
    for (const GB_builtin_entry *e = GB_builtin_registry; e->name; e++) {
        if (e->obj == obj) {
            *name = e->name;
            return GrB_SUCCESS;
        }
    }
    return GrB_INVALID_VALUE;
}

// builtin types/ops are static: freeing is a no-op (as for SuiteSparse builtins)
GrB_Info GrB_Type_free(GrB_Type *t) {
    (void)t;
    return GrB_SUCCESS;
}
GrB_Info GrB_BinaryOp_free(GrB_BinaryOp *op) {
    (void)op;
    return GrB_SUCCESS;
}
GrB_Info GrB_Monoid_free(GrB_Monoid *m) {
    (void)m;
    return GrB_SUCCESS;
}
GrB_Info GrB_Semiring_free(GrB_Semiring *s) {
    if (s && *s && (*s)->magic == GB_MAGIC && (*s)->user) {
        (*s)->magic = GB_FREED;
        delete *s;
        *s = nullptr;
    }
    return GrB_SUCCESS;
}
GrB_Info GrB_UnaryOp_free(GrB_UnaryOp *op) {
    (void)op;
    return GrB_SUCCESS;
}
GrB_Info GxB_Semiring_add(GrB_Monoid *add, GrB_Semiring s) {
    if (!add || !s) return GrB_NULL_POINTER;
    *add = s->add;
    return GrB_SUCCESS;
}
GrB_Info GxB_Semiring_multiply(GrB_BinaryOp *mul, GrB_Semiring s) {
    if (!mul || !s) return GrB_NULL_POINTER;
    *mul = s->mul;
    return GrB_SUCCESS;
}

GrB_Info GrB_Descriptor_new(GrB_Descriptor *desc) {
    if (!desc) return GrB_NULL_POINTER;
    GB_Descriptor_opaque *d = new (std::nothrow) GB_Descriptor_opaque{GB_MAGIC, 0, 0, 0, 0, false, "desc"};
    if (!d) return GrB_OUT_OF_MEMORY;
    *desc = d;
    return GrB_SUCCESS;
}

GrB_Info GrB_Descriptor_set(GrB_Descriptor d, GrB_Desc_Field field, GrB_Desc_Value val) {
    if (!d) return GrB_NULL_POINTER;
    if (d->magic != GB_MAGIC) return GrB_UNINITIALIZED_OBJECT;
    if (d->builtin) return GrB_INVALID_VALUE;  // predefined descriptors are read-only
    switch (field) {
    case GrB_OUTP:
        if (val != GxB_DEFAULT && val != GrB_REPLACE) return GrB_INVALID_VALUE;
        d->outp = val;
        break;
    case GrB_MASK:
        if (val == GxB_DEFAULT) d->mask = 0;
        else if (val == GrB_COMP || val == GrB_STRUCTURE || val == GrB_COMP_STRUCTURE) d->mask |= val;
        else return GrB_INVALID_VALUE;
        break;
    case GrB_INP0:
        if (val != GxB_DEFAULT && val != GrB_TRAN) return GrB_INVALID_VALUE;
        d->inp0 = val;
        break;
    case GrB_INP1:
        if (val != GxB_DEFAULT && val != GrB_TRAN) return GrB_INVALID_VALUE;
        d->inp1 = val;
        break;
    default: return GrB_INVALID_VALUE;
    }
    return GrB_SUCCESS;
}

GrB_Info GrB_Descriptor_free(GrB_Descriptor *desc) {
    if (!desc) return GrB_NULL_POINTER;
    if (*desc && !(*desc)->builtin) {
        (*desc)->magic = GB_FREED;
        delete *desc;
    }
    *desc = nullptr;
    return GrB_SUCCESS;
}

}  // extern "C"
