// gb_peer.hip -- device-initiated frontier exchange of the 1-D row-sharded level BFS
// (SURVEY §8(e)): the per-level all-gather of the ranks' frontier slices
// without a host-issued collective.
//
// Reference loop: notebooks/Example B.1 -- Level BFS.ipynb cell 8 (`q(~v.S, replace) <<
// q.vxm(A, lor_land)` per level), reached through core/matrix.py:2163-2204 (mxv) /
// core/vector.py:1298 (vxm).  Sharded by rows of A^T, each rank computes its slice qloc of
// the next frontier; every rank then needs the whole frontier q.  Round 5 moved that
// exchange as a torch.distributed all-gather issued by the host each level, plus a recount
// launch.  Here every rank owns a *peer window* -- one hipMalloc'd block (IPC-exportable):
//
//     buf[2][words]   the assembled frontier bitmap, double-buffered by exchange parity
//     cnt[2][R]       each source rank's slice count, per parity
//     flag[R]         per source rank: the last exchange number whose slice and count landed
//     arrive, err     the local put's arrival counter; the wait's timeout flag
//
// mapped into every peer's address space (hipIpcOpenMemHandle over xGMI; or, for several
// shards driven from one process, the other window's own address).  Per level:
//   put  (k_peer_put):  every block copies its words of qloc into buf[par] of EVERY window at
//        the rank's word offset (system-scope stores), counts them, fences, and arrives; the
//        last arriving block writes the rank's count into every window's cnt[par][rank],
//        fences, and release-stores flag[rank] = seq in every window;
//   wait (k_peer_wait): every block acquires the R flags of its own window (spinning, with a
//        wall-clock timeout that ends the kernel and raises the window's error word instead of
//        hanging), then copies buf[par] into q's bitmap with cache-bypassing loads; block 0
//        sums cnt[par][*] into q's device count and publishes it to q's host mailbox.
// Two buffers suffice for the pipelined loop (graphblas_amd/dist.py: pipelined_levels): a peer
// can only start exchange seq + 2 after its wait for seq + 1, which needs this rank's put of
// seq + 1, which the stream orders after this rank's wait for seq has read buf[seq % 2].
#include <cstring>
#include <vector>

#include "gb_internal.h"

#define GB_PEER_MAX 16
#define GB_PEER_MAGIC 0x77696e6450656572ULL

namespace {

struct peer_layout {
    int64_t words;   // frontier bitmap words
    int64_t o_buf;   // byte offsets inside a window
    int64_t o_cnt;
    int64_t o_flag;
    int64_t o_arrive;
    int64_t o_err;
    int64_t bytes;
};

peer_layout make_layout(int64_t words) {
    peer_layout L;
    auto a256 = [](int64_t x) { return (x + 255) / 256 * 256; };
    L.words = words;
    L.o_buf = 0;
    L.o_cnt = a256(2 * words * 8);
    L.o_flag = a256(L.o_cnt + 2 * GB_PEER_MAX * 8);
    L.o_arrive = a256(L.o_flag + GB_PEER_MAX * 8);
    L.o_err = L.o_arrive + 64;
    L.bytes = a256(L.o_err + 64);
    return L;
}

struct peer_bases {
    char *p[GB_PEER_MAX];
};

__device__ __forceinline__ void st_sys(unsigned long long *p, unsigned long long v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ unsigned long long ld_sys(const unsigned long long *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// put: the rank's slice (nw words of src) into buf[par] of every window at word lo_w
__global__ __launch_bounds__(256) void k_peer_put(const uint64_t *__restrict__ src, int64_t nw, int64_t lo_w,
                                                  peer_bases pb, int nranks, int rank, unsigned long long seq,
                                                  peer_layout L) {
    const int par = (int)(seq & 1);
    long long c = 0;
    for (int64_t w = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; w < nw; w += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t x = src[w];
        c += __popcll(x);
        for (int p = 0; p < nranks; p++)
            st_sys((unsigned long long *)(pb.p[p] + L.o_buf) + (int64_t)par * L.words + lo_w + w, x);
    }
    // block count, then one arrival per block on the local window's counter (count << 24 | blocks)
    __shared__ long long part[4];
    for (int off = 32; off > 0; off >>= 1) c += __shfl_xor(c, off, 64);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x != 0) return;
    c = part[0] + part[1] + part[2] + part[3];
    __threadfence_system();  // this block's slice stores are visible system-wide before it arrives
    unsigned long long *arrive = (unsigned long long *)(pb.p[rank] + L.o_arrive);
    const unsigned long long old = atomicAdd(arrive, ((unsigned long long)c << 24) + 1ULL);
    if ((unsigned)(old & 0xFFFFFF) + 1 != gridDim.x) return;
    __hip_atomic_store(arrive, 0ULL, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __threadfence_system();  // every block's stores (ordered before their arrivals) before the flags
    const unsigned long long tot = (old >> 24) + (unsigned long long)c;
    for (int p = 0; p < nranks; p++)
        st_sys((unsigned long long *)(pb.p[p] + L.o_cnt) + par * GB_PEER_MAX + rank, tot);
    __threadfence_system();
    for (int p = 0; p < nranks; p++)
        __hip_atomic_store((unsigned long long *)(pb.p[p] + L.o_flag) + rank, seq, __ATOMIC_RELEASE,
                           __HIP_MEMORY_SCOPE_SYSTEM);
}

// wait: acquire every source rank's flag for seq, assemble q, count and publish
__global__ __launch_bounds__(256) void k_peer_wait(char *win, int nranks, unsigned long long seq, peer_layout L,
                                                   uint64_t *__restrict__ qbits, int64_t *__restrict__ qcount,
                                                   void *qiso, int qiso_size, gb_host_slot *pub,
                                                   long long pub_seq, long long timeout_ticks) {
    const int par = (int)(seq & 1);
    __shared__ int ok;
    if (threadIdx.x == 0) {
        const unsigned long long *flag = (const unsigned long long *)(win + L.o_flag);
        const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();  // 100 MHz wall clock
        int all = 0;
        while (true) {
            all = 1;
            for (int p = 0; p < nranks; p++)
                if (__hip_atomic_load(flag + p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) < seq) all = 0;
            if (all) break;
            if ((long long)__builtin_amdgcn_s_memrealtime() - t0 > timeout_ticks) break;
            __builtin_amdgcn_s_sleep(2);
        }
        ok = all;
        if (!all) st_sys((unsigned long long *)(win + L.o_err), 1ULL);  // a peer never arrived
    }
    __syncthreads();
    const unsigned long long *buf = (const unsigned long long *)(win + L.o_buf) + (int64_t)par * L.words;
    if (ok)
        for (int64_t w = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; w < L.words;
             w += (int64_t)gridDim.x * blockDim.x)
            qbits[w] = ld_sys(buf + w);  // bypasses the caches: the words were written by peers
    if (blockIdx.x != 0 || threadIdx.x != 0) return;
    long long tot = 0;
    if (ok) {
        const unsigned long long *cnt = (const unsigned long long *)(win + L.o_cnt) + par * GB_PEER_MAX;
        for (int p = 0; p < nranks; p++) tot += (long long)ld_sys(cnt + p);
    } else {
        for (int64_t w = 0; w < L.words; w++) qbits[w] = 0;  // a failed exchange yields an empty frontier
    }
    *qcount = tot;
    switch (qiso_size) {  // the frontier's entries are true (iso)
    case 1: *(uint8_t *)qiso = 1; break;
    case 2: *(uint16_t *)qiso = 1; break;
    case 4: *(uint32_t *)qiso = 1; break;
    default: *(uint64_t *)qiso = 1; break;
    }
    if (pub) {
        const long long w = (long long)(GB_PUB_TAG | (((unsigned long long)pub_seq & 0x7fffffffULL) << 32) |
                                        ((unsigned long long)tot & 0xffffffffULL));
        __hip_atomic_store(&pub->seq, w, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

}  // namespace

struct GB_PeerWindow_opaque {
    uint64_t magic = 0;
    int nranks = 0, rank = 0;
    int64_t n = 0;
    std::vector<int64_t> bounds;  // nranks + 1 word offsets
    peer_layout L{};
    char *base = nullptr;  // own window (hipMalloc: IPC-exportable)
    char *peer[GB_PEER_MAX] = {};
    bool opened[GB_PEER_MAX] = {};  // mapped by hipIpcOpenMemHandle (closed at free)
    uint64_t put_seq = 0, wait_seq = 0;
};

static GB_PeerWindow_opaque *peer_check(GxB_PeerWindow w) {
    GB_REQUIRE(w && w->magic == GB_PEER_MAGIC, GrB_UNINITIALIZED_OBJECT, "invalid peer window");
    return w;
}

static void peer_require_connected(GB_PeerWindow_opaque *w) {
    for (int p = 0; p < w->nranks; p++)
        GB_REQUIRE(w->peer[p], GrB_INVALID_OBJECT, "peer window " + std::to_string(p) + " not connected");
}

extern "C" {

GrB_Info GxB_PeerWindow_new(GxB_PeerWindow *w, GrB_Index n, int nranks, int rank, const GrB_Index *bounds) {
    if (!w) return GrB_NULL_POINTER;
    return gb_api(nullptr, [&] {
        GB_REQUIRE(nranks >= 1 && nranks <= GB_PEER_MAX, GrB_INVALID_VALUE, "nranks must be in [1, 16]");
        GB_REQUIRE(rank >= 0 && rank < nranks, GrB_INVALID_VALUE, "rank out of range");
        gb_require_init();
        const int64_t words = gb_words((int64_t)n);
        auto *o = new GB_PeerWindow_opaque();
        o->nranks = nranks;
        o->rank = rank;
        o->n = (int64_t)n;
        o->bounds.resize(nranks + 1);
        if (bounds) {
            for (int k = 0; k <= nranks; k++) o->bounds[k] = (int64_t)bounds[k];
        } else {  // equal slots of ceil(words / nranks) words (graphblas_amd/dist.py: partition)
            const int64_t slot = (words + nranks - 1) / nranks;
            for (int k = 0; k <= nranks; k++) o->bounds[k] = std::min<int64_t>(words, k * slot);
        }
        bool okb = o->bounds[0] == 0 && o->bounds[nranks] == words;
        for (int k = 0; k < nranks; k++) okb = okb && o->bounds[k] <= o->bounds[k + 1];
        if (!okb) {
            delete o;
            gb_throw(GrB_INVALID_VALUE, "bounds must rise from 0 to the bitmap's word count");
        }
        o->L = make_layout(words);
        hipError_t e = hipMalloc((void **)&o->base, (size_t)o->L.bytes);
        if (e != hipSuccess) {
            (void)hipGetLastError();
            delete o;
            gb_throw(GrB_OUT_OF_MEMORY, "peer window allocation failed");
        }
        GB_HIP(hipMemset(o->base, 0, (size_t)o->L.bytes));
        GB_HIP(hipDeviceSynchronize());
        o->peer[rank] = o->base;
        o->magic = GB_PEER_MAGIC;
        *w = o;
    });
}

GrB_Info GxB_PeerWindow_handle(void *handle, GxB_PeerWindow w) {
    if (!handle) return GrB_NULL_POINTER;
    return gb_api(nullptr, [&] {
        GB_PeerWindow_opaque *o = peer_check(w);
        static_assert(sizeof(hipIpcMemHandle_t) <= GxB_PEER_HANDLE_BYTES, "IPC handle size");
        hipIpcMemHandle_t h;
        GB_HIP(hipIpcGetMemHandle(&h, o->base));
        memset(handle, 0, GxB_PEER_HANDLE_BYTES);
        memcpy(handle, &h, sizeof(h));
    });
}

GrB_Info GxB_PeerWindow_open(GxB_PeerWindow w, int peer, const void *handle) {
    if (!handle) return GrB_NULL_POINTER;
    return gb_api(nullptr, [&] {
        GB_PeerWindow_opaque *o = peer_check(w);
        GB_REQUIRE(peer >= 0 && peer < o->nranks && peer != o->rank, GrB_INVALID_VALUE, "peer out of range");
        GB_REQUIRE(!o->peer[peer], GrB_INVALID_VALUE, "peer already connected");
        hipIpcMemHandle_t h;
        memcpy(&h, handle, sizeof(h));
        void *p = nullptr;
        GB_HIP(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess));
        o->peer[peer] = (char *)p;
        o->opened[peer] = true;
    });
}

GrB_Info GxB_PeerWindow_attach(GxB_PeerWindow w, int peer, GxB_PeerWindow other) {
    return gb_api(nullptr, [&] {
        GB_PeerWindow_opaque *o = peer_check(w), *t = peer_check(other);
        GB_REQUIRE(peer >= 0 && peer < o->nranks && peer != o->rank && t->rank == peer && t->nranks == o->nranks &&
                       t->n == o->n && t->bounds == o->bounds,
                   GrB_INVALID_VALUE, "the other window is not this exchange's rank `peer`");
        o->peer[peer] = t->base;
        o->opened[peer] = false;
    });
}

GrB_Info GxB_PeerWindow_put(GxB_PeerWindow w, const GrB_Vector qloc) {
    return gb_api(OBJ(qloc), [&] {
        GB_PeerWindow_opaque *o = peer_check(w);
        peer_require_connected(o);
        GB_Obj *v = gb_obj_check(qloc);
        GB_REQUIRE(v->kind != GB_KIND_MATRIX, GrB_INVALID_OBJECT, "qloc is not a vector");
        const int64_t lo_w = o->bounds[o->rank], hi_w = o->bounds[o->rank + 1];
        const int64_t lo = lo_w * 64, hi = std::min<int64_t>(o->n, hi_w * 64);
        GB_REQUIRE(v->nrows == hi - lo, GrB_DIMENSION_MISMATCH,
                   "qloc must hold the rank's rows [lo, hi) of the frontier");
        const int64_t nw = gb_words(v->nrows);
        peer_bases pb;
        for (int p = 0; p < GB_PEER_MAX; p++) pb.p[p] = p < o->nranks ? o->peer[p] : nullptr;
        const unsigned long long seq = ++o->put_seq;
        unsigned g = (unsigned)std::max<int64_t>(1, std::min<int64_t>((nw + 255) / 256, 1024));
        hipLaunchKernelGGL(k_peer_put, dim3(g), dim3(256), 0, gb_stream(), v->bits, nw, lo_w, pb, o->nranks,
                           o->rank, seq, o->L);
        GB_LAUNCH_CHECK();
    });
}

GrB_Info GxB_PeerWindow_wait(GrB_Vector q, GxB_PeerWindow w) {
    return gb_api(OBJ(q), [&] {
        GB_PeerWindow_opaque *o = peer_check(w);
        GB_Obj *v = gb_obj_check(q);
        GB_REQUIRE(v->kind != GB_KIND_MATRIX, GrB_INVALID_OBJECT, "q is not a vector");
        GB_REQUIRE(v->nrows == o->n, GrB_DIMENSION_MISMATCH, "q must hold the whole frontier");
        GB_REQUIRE(o->wait_seq < o->put_seq, GrB_INVALID_VALUE, "wait without a put of this exchange");
        const unsigned long long seq = ++o->wait_seq;
        const size_t ts = v->type->size;
        if (!v->dense || !v->iso) {
            gb_free(v->dense);
            v->dense = gb_malloc(ts);
        }
        v->iso = true;
        if (!v->pub) v->pub = gb_host_slot_alloc();
        const uint64_t pseq = gb_next_pub_seq(v->pub);
        // a peer that never arrives ends the wait after ~5 s (GxB_PeerWindow_error reports it)
        const long long timeout = gb_knob("peer_timeout_ms") > 0 ? gb_knob("peer_timeout_ms") * 100000LL : 500000000LL;
        unsigned g = (unsigned)std::max<int64_t>(1, std::min<int64_t>((o->L.words + 255) / 256, 128));  // few spinning blocks
        hipLaunchKernelGGL(k_peer_wait, dim3(g), dim3(256), 0, gb_stream(), o->base, o->nranks, seq, o->L, v->bits,
                           v->d_nvals, v->dense, (int)ts, gb_host_slot_device(v->pub), (long long)pseq, timeout);
        GB_LAUNCH_CHECK();
        v->nvals_valid = false;
        v->hint_valid = false;
        v->pub_seq = pseq;
        v->pub_epoch = gb_epoch();
    });
}

GrB_Info GxB_PeerWindow_error(int64_t *code, GxB_PeerWindow w) {
    if (!code) return GrB_NULL_POINTER;
    return gb_api(nullptr, [&] {
        GB_PeerWindow_opaque *o = peer_check(w);
        unsigned long long e = 0;
        gb_copy_d2h(&e, o->base + o->L.o_err, sizeof(e));
        *code = (int64_t)e;
    });
}

GrB_Info GxB_PeerWindow_free(GxB_PeerWindow *w) {
    if (!w) return GrB_NULL_POINTER;
    if (!*w) return GrB_SUCCESS;
    GB_PeerWindow_opaque *o = *w;
    if (o->magic != GB_PEER_MAGIC) return GrB_SUCCESS;
    GrB_Info info = gb_api(nullptr, [&] {
        GB_HIP(hipStreamSynchronize(gb_stream()));
        for (int p = 0; p < o->nranks; p++)
            if (o->opened[p]) (void)hipIpcCloseMemHandle(o->peer[p]);
        (void)hipFree(o->base);
    });
    o->magic = 0;
    delete o;
    *w = nullptr;
    return info;
}

}  // extern "C"
