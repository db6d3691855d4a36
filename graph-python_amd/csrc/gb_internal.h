// gb_internal.h -- object model and host-side helpers of libgraphblas_amd.so.
//
// One object struct backs GrB_Matrix, GrB_Vector and GrB_Scalar, so the pointer
// casts python-graphblas performs ((GrB_Matrix)v in Vector.inner/outer,
// reference core/vector.py:1643,1686; Vector._as_matrix core/vector.py:186-205;
// Scalar._as_vector core/scalar.py:555-573) are legal: the operation looks at
// the object's kind and converts storage on the fly.
#pragma once
#include <atomic>
#include <utility>
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/gbamd_codes.h"
#include "gb_state.h"
#include "../../include/graphblas_amd.h"

#define GB_MAGIC 0x6d614d424731ULL   // live object
#define GB_FREED 0x646565724642ULL   // freed object

struct GB_Type_opaque {
    uint64_t magic;
    int code;
    size_t size;
    const char *name;
};
struct GB_BinaryOp_opaque {
    uint64_t magic;
    int opcode;
    GrB_Type xtype, ytype, ztype;  // xtype == nullptr: positional op
    const char *name;
};
struct GB_UnaryOp_opaque {
    uint64_t magic;
    int opcode;
    GrB_Type xtype, ztype;
    const char *name;
};
struct GB_Monoid_opaque {
    uint64_t magic;
    int mcode;
    GrB_Type type;
    GrB_BinaryOp op;
    const char *name;
};
struct GB_Semiring_opaque {
    uint64_t magic;
    GrB_Monoid add;
    GrB_BinaryOp mul;
    const char *name;
    bool user;  // created by GrB_Semiring_new (heap), freed by GrB_Semiring_free
};
struct GB_Descriptor_opaque {
    uint64_t magic;
    int outp, mask, inp0, inp1;
    bool builtin;
    const char *name;
};

struct GB_builtin_entry {
    const char *name;
    int kind;
    void *obj;
};
extern const GB_builtin_entry GB_builtin_registry[];

enum { GB_KIND_MATRIX = 0, GB_KIND_VECTOR = 1, GB_KIND_SCALAR = 2 };

// Device storage.  CSR for matrices; bitmap + dense values for vectors/scalars.
struct GB_Matrix_opaque {
    uint64_t magic;
    int kind;
    GrB_Type type;
    int64_t nrows, ncols;
    bool iso;            // values hold one element that applies to every entry
    // ---- CSR (kind == MATRIX)
    int64_t nvals;       // exact, host-known for CSR
    int64_t *rowptr;     // [nrows+1]
    int32_t *colidx;     // [nvals]
    void *vals;          // [nvals] or [1] when iso
    // cached transpose (CSC), built lazily by gb_csc()
    bool t_valid;
    int64_t *t_rowptr;
    int32_t *t_colidx;
    void *t_vals;
    int64_t *t_perm;     // CSC position -> CSR position of the same entry
    // cached hub-chunk tables of the CSR (0) and CSC (1) orientation, built by
    // gb_view_hubs (gb_mxv.hip); dropped with the transpose
    int32_t *hub_tab[2];
    int64_t hub_n[2], hub_H[2];
    // cached bitmaps of the non-empty rows of the CSR (0) / CSC (1)
    uint64_t *rows_ne[2];
    // cached pull heads of the CSR (0) / CSC (1) orientation (gb_view_pullfirst, gb_mxv.hip):
    // per row 4 int32 -- its neighbours with the most entries in the other orientation
    // first, the whole row when it has at most 4 (padding -1), else 3 of them and -2 -- and
    // the row's own length in the other orientation (saturated to 32 bits)
    int32_t *phead[2];
    uint32_t *pdeg[2];
    int64_t maxdeg[2];   // longest row of each orientation (host), built with the hub tables; -1 unknown
    // cached long-row chunk tables (general SpMV, gb_mxv.hip)
    int32_t *long_tab[2];
    int64_t long_n[2];
    // cached hot-column relabel (general SpMV with a dense input, gb_prim.hip gb_view_hot):
    // colidx with the hot_n most frequent columns replaced by INT32_MIN | rank (rank in
    // descending frequency), and the hot columns' original ids in rank order
    int32_t *hot_ci[2];
    int32_t *hot_cols[2];
    int64_t hot_n[2];
    // cached narrow copy of the integer values of the CSR (0) / CSC (1) orientation, when every
    // value fits fewer bytes (gb_prim.hip gb_view_narrow): nar_k = 1/2/4 unsigned, -1/-2/-4
    // signed bytes per value, 0 not narrowable; nar_done: computed
    void *nar_vx[2];
    int nar_k[2];
    bool nar_done[2];
    // ---- bitmap (kind == VECTOR / SCALAR); length n = nrows (ncols == 1)
    uint64_t *bits;      // [ceil(n/64)]
    void *dense;         // [n] or [1] when iso
    int64_t *d_nvals;    // device counter kept current by every writer
    bool nvals_valid;    // host copy in `nvals` is current
    // host-visible copy of d_nvals published by the kernel that produced it
    // (valid while pub_epoch == gb_epoch(): nothing enqueued since)
    struct gb_host_slot *pub;
    uint64_t pub_seq, pub_epoch;
    // d_nvals[2 .. 2 + GB_HINT_PARTS) hold (in parts) the edge count of this vector's entries in the rows of the
    // push-orientation CSR whose rowptr is hint_key (written by the BFS SpMV that
    // produced it; a stale hint only affects the push/pull choice, never results)
    bool hint_valid;
    const void *hint_key;
    std::string err;
    // ---- column-word bitmap (kind == MATRIX, 1 <= nrows <= 64): the batched-frontier
    // format of gb_colbits.hip.  cw != nullptr: the matrix is held as cw[ncols]
    // presence words (bit r of cw[j] = entry (r, j)) and values cw_vals[j * nrows + r]
    // (or [1] when iso); rowptr/colidx/vals are empty, the count lives in cw_stat[0]
    // (+ the pub mailbox, like a vector's), cw_stat[1] holds the edge hint keyed by
    // hint_key.  Every API entry point outside gb_colbits.hip sees CSR: gb_obj_check
    // converts back (gb_cw_to_csr).
    uint64_t *cw;
    void *cw_vals;
    int64_t *cw_stat;
    // set when a deferred operation on this object failed after its call returned
    // (GrB_INVALID_OBJECT from then on, C API 2.0 nonblocking execution errors)
    GrB_Info invalid = GrB_SUCCESS;
};
typedef GB_Matrix_opaque GB_Obj;

inline GB_Obj *OBJ(const void *p) { return (GB_Obj *)p; }

// ------------------------------------------------------------------ errors
struct gb_exception {
    GrB_Info info;
    std::string msg;
};
[[noreturn]] void gb_throw(GrB_Info info, const std::string &msg);
#define GB_REQUIRE(cond, info, msg) \
    do {                            \
        if (!(cond)) gb_throw(info, msg); \
    } while (0)
void gb_hip_check(hipError_t e, const char *what);
#define GB_HIP(x) gb_hip_check((x), #x)
#define GB_LAUNCH_CHECK() gb_hip_check(hipGetLastError(), "kernel launch")

// API-boundary wrapper: runs body, converts exceptions to GrB_Info and stores
// the message on the error object (reference core/exceptions.py:124-155 reads
// it back with GrB_<Type>_error on the call's output argument).
// a deferred assign (gb_asg, gb_ops.hip) is carried out before any API call
// other than the SpMV that may fuse it
extern std::atomic<bool> g_pending_active;
void gb_pending_flush();
// a speculatively enqueued next BFS level (gb_ops.hip): rolled back before any API call that
// could observe it, unless the caller resolves it itself (g_spec_hold > 0); gb_spec_resolve(obj)
// leaves it in place when obj is a read-only target the speculation does not touch
extern std::atomic<bool> g_spec_active;
extern thread_local int g_spec_hold;
void gb_spec_resolve(const void *keep);
extern std::atomic<int64_t> g_stat_spec_adopted, g_stat_spec_rollbacks;  // GxB_Global_get_int("stat_...")
extern std::atomic<int64_t> g_stat_nvals_copy;
extern std::atomic<int64_t> g_stat_host_push;  // SpMV launches whose push direction the host proved
// named counters of which kernel classes a call used (host-side, off the per-level BFS path):
// GxB_Global_get_int("stat_<name>") reads them; tests assert that a workload reached a class
void gb_stat_add(const char *name, int64_t v);
bool gb_stat_get(const char *name, int64_t *v);
struct gb_spec_hold_guard {
    gb_spec_hold_guard() { g_spec_hold++; }
    ~gb_spec_hold_guard() { g_spec_hold--; }
};
// A pending root (gb_object.hip): `GrB_Vector_setElement_BOOL(q, true, i)` on an empty BOOL vector
// -- the BFS start, notebooks/Example B.1 cell 8 -- is recorded instead of launched; the level
// SpMV of the notebook shape that reads q consumes it (its kernel pushes from vertex i, gb_mxv.hip
// gb_push_root), and the deferred stamp `v<q> = 1` before it keeps it pending (g_root_hold); any
// other API call materialises it first (gb_root_flush: the single-thread set launch it replaced).
extern std::atomic<bool> g_root_active;
extern thread_local int g_root_hold;
void gb_root_flush();
bool gb_root_pending(const GB_Obj *v);
int64_t gb_root_take(GB_Obj *v);  // the root index, the record cleared; -1 when v holds none
const void *gb_bool_true_dev();   // one device byte holding true (a consumed root's iso value)
struct gb_root_hold_guard {
    gb_root_hold_guard() { g_root_hold++; }
    ~gb_root_hold_guard() { g_root_hold--; }
};

// roctx ranges named by the API entry point around each library call (environment
// GRAPHBLAS_AMD_ROCTX=1; the roctx library is loaded then, never otherwise), so a rocprofv3
// trace with --marker-trace attributes every kernel to the GrB_* / GxB_* call that launched
// it -- the kernel-level counterpart of the reference's Recorder (core/recorder.py:34-178).
extern bool g_roctx_on;
void gb_roctx_push(const char *name);
void gb_roctx_pop();
struct gb_roctx_range {
    bool on;
    explicit gb_roctx_range(const char *name) : on(g_roctx_on && name) {
        if (on) gb_roctx_push(name);
    }
    ~gb_roctx_range() {
        if (on) gb_roctx_pop();
    }
};

template <bool FLUSH = true, class F>
GrB_Info gb_api_impl(GB_Obj *errobj, F &&body, const char *name = nullptr) {
    gb_roctx_range range(name);
    try {
        if (FLUSH && !g_spec_hold && g_spec_active.load(std::memory_order_acquire)) gb_spec_resolve(nullptr);
        if (FLUSH && !g_root_hold && g_root_active.load(std::memory_order_acquire)) gb_root_flush();
        if (FLUSH && g_pending_active.load(std::memory_order_acquire)) gb_pending_flush();
        body();
        if (errobj && errobj->magic == GB_MAGIC) errobj->err.clear();
        return GrB_SUCCESS;
    } catch (const gb_exception &e) {
        if (errobj && errobj->magic == GB_MAGIC) errobj->err = e.msg;
        return e.info;
    } catch (const std::bad_alloc &) {
        if (errobj && errobj->magic == GB_MAGIC) errobj->err = "out of host memory";
        return GrB_OUT_OF_MEMORY;
    } catch (...) {
        return GrB_PANIC;
    }
}
template <class F>
GrB_Info gb_api_named(const char *name, GB_Obj *errobj, F &&body) {
    return gb_api_impl<true>(errobj, std::forward<F>(body), name);
}
// GrB_mxv / GrB_vxm: the deferred assign is fused or flushed inside (do_spmv)
template <class F>
GrB_Info gb_api_keep_pending_named(const char *name, GB_Obj *errobj, F &&body) {
    return gb_api_impl<false>(errobj, std::forward<F>(body), name);
}
// the entry point's own name (__func__) names its trace range
#define gb_api(obj, ...) gb_api_named(__func__, obj, __VA_ARGS__)
#define gb_api_keep_pending(obj, ...) gb_api_keep_pending_named(__func__, obj, __VA_ARGS__)

// ------------------------------------------------------------------ host-time probes
// Diagnostics of the per-call host path (environment GRAPHBLAS_AMD_HPROF=1): cumulative
// nanoseconds per named section, printed at exit.  A disabled probe costs one load.
extern bool g_hprof_on;
void gb_hprof_add(int slot, const char *name, int64_t ns);
int64_t gb_hprof_now();
struct gb_hprof_scope {
    int slot;
    const char *name;
    int64_t t0;
    gb_hprof_scope(int s, const char *n) : slot(s), name(n), t0(g_hprof_on ? gb_hprof_now() : 0) {}
    ~gb_hprof_scope() {
        if (g_hprof_on) gb_hprof_add(slot, name, gb_hprof_now() - t0);
    }
};
#define GB_HPROF(slot, name) gb_hprof_scope gb_hprof_##slot(slot, name)

// ------------------------------------------------------------------ context
hipStream_t gb_stream();
void gb_require_init();
void gb_sync();
int64_t gb_knob(const char *key);
// persistent zeroed device words (layout: gb_state.h), allocated on first use
unsigned long long *gb_device_state();

// Host-visible mailboxes in pinned coherent memory: a kernel publishes a
// device count with a sequence number (system-scope store); the host spins on
// it instead of a copy + stream synchronisation.
struct gb_host_slot {
    long long seq;
    long long value;
    long long pad[5];  // pad[0]: the column-word kernels' device-written hint (gb_colbits.hip)
    long long host_last;  // host only, never written by a device: the last sequence number issued
};
gb_host_slot *gb_host_slot_alloc();
void gb_host_slot_release(gb_host_slot *s);
gb_host_slot *gb_host_slot_device(gb_host_slot *s);  // device address of the same slot
uint64_t gb_next_pub_seq(gb_host_slot *s);  // the next publish number for slot s
// count of work enqueued through gb_stream() (a published value is current only
// while no later work has been enqueued)
uint64_t gb_epoch();
hipStream_t gb_stream_peek();  // the library stream, without counting an enqueue
// wait for slot->seq == seq; false if the stream drained without it (caller falls back).
// A publisher may instead store one tagged word into seq: bit 63 | (seq & 0x7fffffff) << 32 |
// the 32-bit count (GB_PUB_TAG; a plain seq never has bit 63 set)
#define GB_PUB_TAG (1ULL << 63)
bool gb_host_slot_wait(gb_host_slot *s, uint64_t seq, int64_t *value);
// zero nw bitmap words and (if given) the count, in one launch
void gb_zero_bitmap(uint64_t *bits, int64_t nw, int64_t *d_count);
// count the set bits into *d_count (one launch); publish to the host mailbox when given
void gb_bitmap_count_pub(const uint64_t *bits, int64_t n, int64_t *d_count, gb_host_slot *pub_host, uint64_t seq);  // tuning knobs (0 = auto)

// device memory (stream-ordered pool on the library stream)
void *gb_malloc(size_t bytes);        // throws GrB_OUT_OF_MEMORY
void gb_free(void *p);
template <class T>
T *gb_malloc_n(size_t n) {
    return (T *)gb_malloc(n * sizeof(T));
}
void gb_memset(void *p, int v, size_t bytes);
void gb_copy_d2d(void *dst, const void *src, size_t bytes);
void gb_copy_h2d(void *dst, const void *src, size_t bytes);
void gb_copy_d2h(void *dst, const void *src, size_t bytes);  // synchronises

// scratch owner: frees device buffers at scope exit (stream ordered)
struct gb_scratch {
    void *ptrs[32];
    int n = 0;
    template <class T>
    T *get(size_t count) {
        T *p = gb_malloc_n<T>(count ? count : 1);
        ptrs[n++] = p;
        return p;
    }
    ~gb_scratch() {
        for (int i = 0; i < n; i++) gb_free(ptrs[i]);
    }
};

// ------------------------------------------------------------------ objects
GB_Obj *gb_obj_check(const void *p, bool allow_null = false);      // CSR for matrices
GB_Obj *gb_obj_check_raw(const void *p, bool allow_null = false);  // any internal format
// column-word bitmap matrices (gb_colbits.hip)
void gb_cw_to_csr(GB_Obj *A);    // back to CSR (device work; reads the count)
void gb_cw_release(GB_Obj *A);   // drop the column-word storage without converting
void gb_cw_materialize(GB_Obj *A);  // carry out pending level-stamp layers (values)
GB_Obj *gb_new_object(int kind, GrB_Type type, int64_t nrows, int64_t ncols);
extern "C" void gb_vec_recount(GB_Obj *v);  // a vector's bitmap changed on the device: recount + publish
void gb_obj_free_storage(GB_Obj *A);
void gb_drop_transpose(GB_Obj *A);
int64_t gb_nvals(GB_Obj *A);           // exact (may synchronise for bitmaps)
inline int64_t gb_words(int64_t n) { return (n + 63) >> 6; }
inline bool gb_is_bitmap(const GB_Obj *A) { return A->kind != GB_KIND_MATRIX; }

// Typecast a device array (n elements, or the single iso value).
void gb_cast_array(void *dst, int dst_code, const void *src, int src_code, int64_t n);

// Read-only CSR view of any object (a vector becomes an n x 1 CSR temporary).
struct gb_csr_view {
    int64_t nrows = 0, ncols = 0, nvals = 0;
    const int64_t *rowptr = nullptr;
    const int32_t *colidx = nullptr;
    const void *vals = nullptr;
    bool iso = false;
    int tcode = 0;
    // hub chunks (rows longer than hub_H cut into hub_H-edge pieces): pairs (row, piece)
    const int32_t *hubs = nullptr;
    int64_t nhubs = 0, hub_H = 0;
    const uint64_t *nonempty = nullptr;  // bitmap of rows with entries (when attached)
    const int32_t *phead = nullptr;      // pull head per row, 4 int32 (when attached; see GB_Obj)
    const uint32_t *pdeg = nullptr;      // row length in the other orientation (when attached)
    int64_t maxdeg = -1;                 // longest row (host; attached with the hub chunks, -1 unknown)
    const int32_t *lchunks = nullptr;    // long-row chunks (row, piece) of the general SpMV (when attached)
    int64_t nlchunks = -1;
    const void *nvx = nullptr;           // narrow copy of vals (when attached; see GB_Obj::nar_vx)
    int nvk = 0;                         // its kind: 1/2/4 unsigned, -1/-2/-4 signed bytes, 0 none
    const int32_t *hcolidx = nullptr;    // hot-column relabelled colidx (when attached; see GB_Obj::hot_ci)
    const int32_t *hcols = nullptr;      // the hot columns' original ids, rank order
    int64_t nhot = 0;
    gb_scratch own;
};
void gb_get_csr(gb_csr_view &v, GB_Obj *A);
// attach the cached hub-chunk table of matrix A's orientation (0 CSR, 1 CSC) to v
void gb_view_hubs(gb_csr_view &v, GB_Obj *A, int orient, int64_t H);
// attach the cached non-empty-rows bitmap of matrix A's orientation to v
void gb_view_nonempty(gb_csr_view &v, GB_Obj *A, int orient);
// attach the cached pull heads of A's orientation (other_rowptr: the other orientation's row
// pointers, other_n rows) -- the iso pull tests a row's best-connected neighbours first, and
// rows of at most 4 entries without reading their bounds or edges
void gb_view_pullfirst(gb_csr_view &v, GB_Obj *A, int orient, const int64_t *other_rowptr, int64_t other_n);
void gb_view_long_rows(gb_csr_view &v, GB_Obj *A, int orient);
// attach the cached narrow copy of matrix A's orientation's integer values (built on first use:
// one min/max pass, then a cast) when they fit fewer bytes; v.nvx stays null otherwise
void gb_view_narrow(gb_csr_view &v, GB_Obj *A, int orient);
// attach (building on first use) the hot-column relabel of matrix A's orientation, when the
// matrix is large enough for the x gathers of a dense-input SpMV to miss in L2
void gb_view_hot(gb_csr_view &v, GB_Obj *A, int orient);
// CSC of A (i.e. CSR of A^T), cached on the object when A is a matrix.
void gb_get_csc(gb_csr_view &v, GB_Obj *A);
// the cached CSC of a matrix and, per CSC entry, its CSR position (built on first use)
const int64_t *gb_csc_perm(GB_Obj *A);
// Values of a CSR view cast to type `code` (returns the view's own pointer if same type).
const void *gb_view_vals_as(gb_csr_view &v, int code, gb_scratch &s);

// Read-only bitmap view of any object (an n x 1 matrix becomes a bitmap temporary).
struct gb_bitmap_view {
    int64_t n = 0;
    const uint64_t *bits = nullptr;
    const void *vals = nullptr;
    bool iso = false;
    int tcode = 0;
    const int64_t *count = nullptr;      // device count of entries (nullptr: unknown)
    const long long *mf_hint = nullptr;  // device edge count of the entries (see GB_Obj::hint_key)
    const void *hint_key = nullptr;
    bool full = false;                   // every entry present, known on the host
    int64_t h_nvals = -1;                // entries, when known on the host (-1: not known)
    gb_scratch own;
};
void gb_get_bitmap(gb_bitmap_view &v, GB_Obj *A);
const void *gb_bitmap_vals_as(gb_bitmap_view &v, int code, gb_scratch &s);

// Install freshly computed storage into an object (takes ownership).
void gb_install_csr(GB_Obj *C, int64_t nrows, int64_t ncols, int64_t nvals, int64_t *rowptr,
                    int32_t *colidx, void *vals, bool iso);
void gb_install_bitmap(GB_Obj *C, int64_t n, uint64_t *bits, void *dense, bool iso,
                       int64_t *d_nvals /* may be null: recomputed */);

// bitmap helpers (device work on the library stream)
void gb_bitmap_count(const uint64_t *bits, int64_t n, int64_t *d_count);
void gb_bitmap_to_csr(const uint64_t *bits, const void *dense, bool iso, int64_t n, size_t tsize,
                      int64_t **rowptr, int32_t **colidx, void **vals, int64_t *nvals);
void gb_csr_col_to_bitmap(const gb_csr_view &v, size_t tsize, uint64_t **bits, void **dense,
                          int64_t **d_nvals);

// COO build (sort + duplicate fold) into an empty object; extract tuples to host
void gb_build(GB_Obj *C, const GrB_Index *I, const GrB_Index *J, const void *X, int xcode, bool x_iso,
              int64_t n, GrB_BinaryOp dup);
void gb_extract_tuples(GB_Obj *A, GrB_Index *I, GrB_Index *J, void *X, int xcode, GrB_Index *nvals);

// expand iso values to a full array of n elements
void *gb_expand_iso(const void *one_value, size_t tsize, int64_t n);

// transpose CSR -> CSR of the transpose (values optional)
// tperm (optional): receives the CSC position -> CSR position map (caller frees)
void gb_transpose_csr(int64_t nrows, int64_t ncols, int64_t nvals, const int64_t *rowptr,
                      const int32_t *colidx, const void *vals, size_t tsize, bool iso,
                      int64_t **trowptr, int32_t **tcolidx, void **tvals, int64_t **tperm = nullptr);

// ------------------------------------------------------------------ index lists
// GrB_ALL, an explicit list, or the GxB_RANGE / GxB_STRIDE / GxB_BACKWARDS encodings
// (gb_extract.hip), expanded on the host and checked against n
struct gb_index_list {
    bool all = false;          // GrB_ALL: idx is empty, the list is 0 .. n-1
    int64_t n = 0;             // length of the list
    std::vector<int64_t> idx;  // explicit indices (all == false)
};
void gb_expand_indices(gb_index_list &L, const GrB_Index *I, GrB_Index ni, int64_t n);

// ------------------------------------------------------------------ ops
struct gb_desc {
    bool replace = false, comp = false, structure = false, tran0 = false, tran1 = false;
};
gb_desc gb_read_desc(const GrB_Descriptor d);
// batched-frontier fast paths (gb_colbits.hip): C<M> = A lor.land B with A of at most 64
// rows, and C<M> = x over all indices; false when the call is not of that shape (the
// caller then runs the general path on CSR operands)
bool gb_colbits_mxm(GB_Obj *C, GB_Obj *M, GrB_BinaryOp accum, GrB_Semiring sr, GB_Obj *A, GB_Obj *B,
                    const gb_desc &d);
bool gb_colbits_assign_scalar(GB_Obj *C, GB_Obj *M, GrB_BinaryOp accum, const void *x, int xcode,
                              const GrB_Index *I, const GrB_Index *J, const gb_desc &d);

// Effective mask: bitmap of positions where the mask is true (value masks cast
// to bool), for vector outputs; CSR (structure only) for matrix outputs.
struct gb_vmask {
    const uint64_t *bits = nullptr;  // nullptr: no mask
    bool comp = false;
    const int64_t *count = nullptr;  // device count of set mask bits, when known
    int64_t h_count = -1;            // the same count known on the host (-1: not known)
    // value mask of an iso vector, left unmaterialised (only when the caller allows it):
    // the mask is `bits` if the device value *iso_val is nonzero, else empty
    const void *iso_val = nullptr;
    int iso_code = -1;
    gb_scratch own;
};
void gb_make_vmask(gb_vmask &m, GB_Obj *M, const gb_desc &d, int64_t n, bool allow_iso_value = false);

struct gb_mmask {
    bool present = false, comp = false;
    GB_Obj *obj = nullptr;   // the mask matrix when rowptr/colidx are its own CSR (structural)
    gb_csr_view view;        // structure of the mask
    const int64_t *rowptr = nullptr;
    const int32_t *colidx = nullptr;
    int64_t nvals = 0;
    gb_scratch own;
};
void gb_make_mmask(gb_mmask &m, GB_Obj *M, const gb_desc &d, int64_t nrows, int64_t ncols);

// Result of a computation before the write-back into C.
struct gb_vec_result {  // bitmap, type code ztype
    int64_t n = 0;
    uint64_t *bits = nullptr;
    void *dense = nullptr;
    bool iso = false;
    int tcode = 0;
    int64_t *d_nvals = nullptr;
    gb_host_slot *pub = nullptr;  // if set, the producing kernel publishes nvals here
    uint64_t pub_seq = 0;
    bool published = false;       // set by the producer when it did publish
    const void *hint_key = nullptr;  // set when d_nvals[2..] hold the edge-count hint parts
};
struct gb_mat_result {  // CSR
    int64_t nrows = 0, ncols = 0, nvals = 0;
    int64_t *rowptr = nullptr;
    int32_t *colidx = nullptr;
    void *vals = nullptr;
    bool iso = false;
    int tcode = 0;
    bool within_mask = false;  // T already restricted to the (non-complemented) mask
};

// C<M,replace> = C accum T  (takes ownership of T's buffers)
// returns true when T was installed into C as is (no merge)
bool gb_writeback_vector(GB_Obj *C, gb_vec_result &T, GB_Obj *M, const gb_desc &d,
                         GrB_BinaryOp accum, bool t_within_mask);
void gb_writeback_matrix(GB_Obj *C, gb_mat_result &T, GB_Obj *M, const gb_desc &d,
                         GrB_BinaryOp accum);

// kernels of the hot path (gb_mxv.hip, gb_mxm.hip)
// A: rows = output positions (pull); Apush: the other orientation (rows = u's
// positions) or nullptr; the device picks push or pull per call.
// A deferred `w<q>(:) = x` (GrB_Vector_assign with a value or structural mask q,
// no accum / replace, all indices) carried out by the iso SpMV kernel whose input
// is q and whose mask is w's structure (the BFS level loop: v<q> = d;
// q<!v.S> = q lor.land A).  gb_ops.hip defers such assigns; every other API call
// performs them first (gb_pending_flush, called by gb_api).
struct gb_asg {
    uint64_t *bits = nullptr;  // w's bitmap (read as the call's mask, OR q)
    void *vals = nullptr;      // w's dense values
    int size = 0;              // value size in bytes
    unsigned long long x = 0;  // the value's bytes
    const void *q_iso = nullptr;  // q's iso value when q is a value mask (nullptr: structure)
    int q_iso_code = -1;
    int64_t *count = nullptr;  // w's device count
    int64_t h_count = -1;      // w's count before the assign, when the host knew it (-1: not known)
    // u's device count is exact (written by the kernel that produced u, earlier on the stream):
    // an empty u ends the launch early (the speculated level after a BFS's last one)
    bool u_count_exact = false;
    // u is a pending root (gb_root_take): the frontier is {root}; u's storage does not hold it
    int64_t root = -1;
};
void gb_spmv(gb_vec_result &T, const gb_csr_view &A, const gb_csr_view *Apush, gb_bitmap_view &u,
             const gb_vmask &mask, GrB_Semiring sr, bool flip, const gb_asg *asg = nullptr);
bool gb_spmv_result_iso(GrB_Semiring sr, bool a_iso, bool u_iso, bool flip);
void gb_spgemm(gb_mat_result &T, gb_csr_view &A, gb_csr_view &B, gb_csr_view *BT,
               gb_mmask &mask, GrB_Semiring sr);
// Vector clears without a launch (gb_mxv.hip): a cleared vector takes a pre-zeroed bitmap and
// count from a small pool; its old bitmap is zeroed by the next iso SpMV launch and returns to
// the pool.  Returns false (nothing changed but the old bitmap possibly taken) when the pool
// has nothing of this size: the caller then allocates and zeroes as usual.
bool gb_zpool_clear_vector(GB_Obj *v);

// hash Gustavson C = A*B (gb_spgemm_hash.hip): flops = per-row product counts
void gb_spgemm_hash(gb_mat_result &T, gb_csr_view &A, gb_csr_view &B, GrB_Semiring sr, bool iso,
                    const void *av, const void *bv, const int64_t *flops);

// scans / sorts (gb_prim.hip)
void gb_exclusive_scan_i64(const int64_t *in, int64_t *out, int64_t n);  // out[n] = total
void gb_exclusive_scan_u8(const uint8_t *in, int64_t *out, int64_t n);  // 0/1 flags, int64 prefixes
void gb_exclusive_scan_i32(const int32_t *in, int64_t add_each, int64_t *out, int64_t n);  // of in[i] + add_each
void gb_sort_pairs_u64(uint64_t *keys, int64_t *vals, int64_t n, int end_bit);
void gb_sort_pairs_i32(int32_t *keys, int64_t *vals, int64_t n, int end_bit);
int64_t gb_read_i64(const int64_t *dptr);

const char *gb_type_name(int code);
size_t gb_type_size(int code);
GrB_Type gb_type_of(int code);
