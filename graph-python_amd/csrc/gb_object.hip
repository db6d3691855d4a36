// gb_object.hip -- GrB_Matrix / GrB_Vector / GrB_Scalar objects on the device.
//
// Lifecycle, build (COO ingest with duplicate handling), extractTuples,
// import/export (CSR / CSC / COO), element access, dup/clear/resize, and the
// storage views (CSR view, cached CSC, bitmap view) the kernels consume.
// Replaces the SuiteSparse calls behind reference core/matrix.py:178-213
// (new/free), :643-697 (build), :543-611 (to_coo), :1057-1133 (_from_csx),
// :1658-1702 (_to_csx) and core/vector.py:152-184, 482, 538.
#include <algorithm>
#include <vector>

#include "gb_device.cuh"
#include <mutex>

#include "gb_internal.h"

#define GB_BLOCK 256
static inline unsigned grid_for(int64_t n, unsigned cap = 8192) {
    int64_t g = (n + GB_BLOCK - 1) / GB_BLOCK;
    if (g < 1) g = 1;
    if (g > cap) g = cap;
    return (unsigned)g;
}
#define GRID_STRIDE(i, n) \
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < (n); i += (int64_t)gridDim.x * blockDim.x)

// dispatch a functor templated on the C type of a type code
template <class F>
static void with_type(int code, F &&f) {
    switch (code) {
    case GBAMD_T_BOOL: f((bool)0); break;
    case GBAMD_T_INT8: f((int8_t)0); break;
    case GBAMD_T_UINT8: f((uint8_t)0); break;
    case GBAMD_T_INT16: f((int16_t)0); break;
    case GBAMD_T_UINT16: f((uint16_t)0); break;
    case GBAMD_T_INT32: f((int32_t)0); break;
    case GBAMD_T_UINT32: f((uint32_t)0); break;
    case GBAMD_T_INT64: f((int64_t)0); break;
    case GBAMD_T_UINT64: f((uint64_t)0); break;
    case GBAMD_T_FP32: f((float)0); break;
    default: f((double)0); break;
    }
}

// ================================================================== object basics
GB_Obj *gb_obj_check(const void *p, bool allow_null) {
    GB_Obj *A = gb_obj_check_raw(p, allow_null);
    if (A && A->cw) gb_cw_to_csr(A);
    return A;
}

GB_Obj *gb_obj_check_raw(const void *p, bool allow_null) {
    if (!p) {
        if (allow_null) return nullptr;
        gb_throw(GrB_NULL_POINTER, "required object is NULL");
    }
    GB_Obj *A = OBJ(p);
    if (A->magic == GB_FREED) gb_throw(GrB_INVALID_OBJECT, "object has been freed");
    if (A->magic != GB_MAGIC) gb_throw(GrB_UNINITIALIZED_OBJECT, "object is not initialized");
    if (A->invalid != GrB_SUCCESS) gb_throw(GrB_INVALID_OBJECT, A->err);
    return A;
}

static void alloc_empty_storage(GB_Obj *A) {
    if (A->kind == GB_KIND_MATRIX) {
        A->rowptr = gb_malloc_n<int64_t>(A->nrows + 1);
        gb_memset(A->rowptr, 0, (A->nrows + 1) * sizeof(int64_t));
        A->colidx = nullptr;
        A->vals = nullptr;
        A->nvals = 0;
    } else {
        int64_t nw = gb_words(A->nrows);
        A->bits = gb_malloc_n<uint64_t>(nw);
        A->dense = nullptr;
        if (!A->d_nvals) A->d_nvals = gb_malloc_n<int64_t>(1);
        gb_zero_bitmap(A->bits, nw, A->d_nvals);  // one launch: bits and count
        A->nvals = 0;
        A->nvals_valid = true;
        A->hint_valid = false;
        A->pub_seq = 0;
    }
    A->iso = false;
}

GB_Obj *gb_new_object(int kind, GrB_Type type, int64_t nrows, int64_t ncols) {
    gb_require_init();
    GB_REQUIRE(type && type->magic == GB_MAGIC, GrB_UNINITIALIZED_OBJECT, "invalid type");
    GB_REQUIRE(nrows >= 0 && ncols >= 0, GrB_INVALID_VALUE, "negative dimension");
    GB_REQUIRE(nrows <= (int64_t)GrB_INDEX_MAX && ncols <= (int64_t)GrB_INDEX_MAX, GrB_INVALID_VALUE,
               "dimension too large");
    if (kind == GB_KIND_MATRIX) {
        // device column indices are int32: matrices up to 2^31 - 1 columns
        GB_REQUIRE(ncols < (1LL << 31), GrB_OUT_OF_MEMORY,
                   "matrix with >= 2^31 columns exceeds the device index width");
    }
    GB_Obj *A = new GB_Obj();
    A->magic = GB_MAGIC;
    A->kind = kind;
    A->type = type;
    A->nrows = nrows;
    A->ncols = ncols;
    try {
        alloc_empty_storage(A);
    } catch (...) {
        gb_free(A->rowptr);
        gb_free(A->bits);
        gb_free(A->d_nvals);
        A->magic = GB_FREED;
        delete A;
        throw;
    }
    return A;
}

void gb_drop_transpose(GB_Obj *A) {
    if (A->t_valid) {
        gb_free(A->t_rowptr);
        gb_free(A->t_colidx);
        gb_free(A->t_vals);
        gb_free(A->t_perm);
    }
    A->t_perm = nullptr;
    A->t_rowptr = nullptr;
    A->t_colidx = nullptr;
    A->t_vals = nullptr;
    A->t_valid = false;
    for (int o = 0; o < 2; o++) {
        gb_free(A->hub_tab[o]);
        A->hub_tab[o] = nullptr;
        A->hub_n[o] = A->hub_H[o] = 0;
        A->maxdeg[o] = 0;
        gb_free(A->rows_ne[o]);
        A->rows_ne[o] = nullptr;
        gb_free(A->phead[o]);
        gb_free(A->pdeg[o]);
        A->phead[o] = nullptr;
        A->pdeg[o] = nullptr;
        gb_free(A->long_tab[o]);
        A->long_tab[o] = nullptr;
        gb_free(A->hot_ci[o]);
        gb_free(A->hot_cols[o]);
        A->hot_ci[o] = nullptr;
        A->hot_cols[o] = nullptr;
        A->hot_n[o] = 0;
        A->long_n[o] = 0;
        gb_free(A->nar_vx[o]);
        A->nar_vx[o] = nullptr;
        A->nar_k[o] = 0;
        A->nar_done[o] = false;
    }
}

void gb_obj_free_storage(GB_Obj *A) {
    gb_cw_release(A);
    gb_drop_transpose(A);
    gb_free(A->rowptr);
    gb_free(A->colidx);
    gb_free(A->vals);
    gb_free(A->bits);
    gb_free(A->dense);
    A->rowptr = nullptr;
    A->colidx = nullptr;
    A->vals = nullptr;
    A->bits = nullptr;
    A->dense = nullptr;
}

std::atomic<int64_t> g_stat_nvals_copy{0};
std::atomic<int64_t> g_stat_host_push{0};

int64_t gb_nvals(GB_Obj *A) {
    if (A->kind == GB_KIND_MATRIX && !A->cw) return A->nvals;
    if (!A->nvals_valid) {
        int64_t v;
        if (A->pub && A->pub_seq && A->pub_epoch == gb_epoch() && gb_host_slot_wait(A->pub, A->pub_seq, &v)) {
            A->nvals = v;  // published by the kernel that produced d_nvals
        } else {
            g_stat_nvals_copy.fetch_add(1, std::memory_order_relaxed);
            A->nvals = gb_read_i64(A->cw ? A->cw_stat : A->d_nvals);
        }
        A->nvals_valid = true;
    }
    return A->nvals;
}

void gb_install_csr(GB_Obj *C, int64_t nrows, int64_t ncols, int64_t nvals, int64_t *rowptr,
                    int32_t *colidx, void *vals, bool iso) {
    if (C->kind == GB_KIND_MATRIX) {
        gb_cw_release(C);
        gb_drop_transpose(C);
        gb_free(C->rowptr);
        gb_free(C->colidx);
        gb_free(C->vals);
        C->nrows = nrows;
        C->ncols = ncols;
        C->nvals = nvals;
        C->rowptr = rowptr;
        C->colidx = colidx;
        C->vals = vals;
        C->iso = iso && nvals > 0;
        if (nvals == 0 && iso) C->iso = false;
        return;
    }
    // vector target: n x 1 CSR -> bitmap
    GB_REQUIRE(ncols == 1, GrB_DIMENSION_MISMATCH, "vector result must have one column");
    gb_csr_view v;
    v.nrows = nrows;
    v.ncols = 1;
    v.nvals = nvals;
    v.rowptr = rowptr;
    v.colidx = colidx;
    v.vals = vals;
    v.iso = iso;
    v.tcode = C->type->code;
    uint64_t *bits;
    void *dense;
    int64_t *cnt;
    gb_csr_col_to_bitmap(v, C->type->size, &bits, &dense, &cnt);
    gb_free(rowptr);
    gb_free(colidx);
    gb_free(vals);
    gb_install_bitmap(C, nrows, bits, dense, iso, cnt);
}

void gb_install_bitmap(GB_Obj *C, int64_t n, uint64_t *bits, void *dense, bool iso, int64_t *d_nvals) {
    if (C->kind != GB_KIND_MATRIX) {
        gb_free(C->bits);
        gb_free(C->dense);
        C->nrows = n;
        C->ncols = 1;
        C->bits = bits;
        C->dense = dense;
        C->iso = iso;
        if (d_nvals) {
            gb_free(C->d_nvals);
            C->d_nvals = d_nvals;
        } else {
            if (!C->d_nvals) C->d_nvals = gb_malloc_n<int64_t>(1);
            gb_bitmap_count(bits, n, C->d_nvals);
        }
        C->nvals_valid = false;
        C->pub_seq = 0;
        C->hint_valid = false;
        return;
    }
    // matrix target (n x 1): bitmap -> CSR
    GB_REQUIRE(C->ncols == 1, GrB_DIMENSION_MISMATCH, "matrix output of a vector op must be n x 1");
    int64_t *rp;
    int32_t *ci;
    void *vx;
    int64_t nz;
    gb_bitmap_to_csr(bits, dense, iso, n, C->type->size, &rp, &ci, &vx, &nz);
    gb_free(bits);
    gb_free(dense);
    gb_free(d_nvals);
    gb_install_csr(C, n, 1, nz, rp, ci, vx, iso);
}

// ================================================================== views
void gb_get_csr(gb_csr_view &v, GB_Obj *A) {
    v.tcode = A->type->code;
    if (A->kind == GB_KIND_MATRIX) {
        v.nrows = A->nrows;
        v.ncols = A->ncols;
        v.nvals = A->nvals;
        v.rowptr = A->rowptr;
        v.colidx = A->colidx;
        v.vals = A->vals;
        v.iso = A->iso;
        return;
    }
    int64_t *rp;
    int32_t *ci;
    void *vx;
    int64_t nz;
    if (!A->dense) {  // no entries were ever written
        rp = gb_malloc_n<int64_t>(A->nrows + 1);
        gb_memset(rp, 0, (A->nrows + 1) * sizeof(int64_t));
        ci = gb_malloc_n<int32_t>(1);
        vx = gb_malloc(A->type->size);
        nz = 0;
    } else {
        gb_bitmap_to_csr(A->bits, A->dense, A->iso, A->nrows, A->type->size, &rp, &ci, &vx, &nz);
    }
    v.own.ptrs[v.own.n++] = rp;
    v.own.ptrs[v.own.n++] = ci;
    v.own.ptrs[v.own.n++] = vx;
    v.nrows = A->nrows;
    v.ncols = 1;
    v.nvals = nz;
    v.rowptr = rp;
    v.colidx = ci;
    v.vals = vx;
    v.iso = A->iso;
}

void gb_get_csc(gb_csr_view &v, GB_Obj *A) {
    v.tcode = A->type->code;
    if (A->kind == GB_KIND_MATRIX) {
        if (!A->t_valid) {
            gb_transpose_csr(A->nrows, A->ncols, A->nvals, A->rowptr, A->colidx, A->vals,
                             A->type->size, A->iso, &A->t_rowptr, &A->t_colidx, &A->t_vals);
            A->t_valid = true;
        }
        v.nrows = A->ncols;
        v.ncols = A->nrows;
        v.nvals = A->nvals;
        v.rowptr = A->t_rowptr;
        v.colidx = A->t_colidx;
        v.vals = A->t_vals;
        v.iso = A->iso;
        return;
    }
    gb_csr_view c;
    gb_get_csr(c, A);
    int64_t *trp;
    int32_t *tci;
    void *tvx;
    gb_transpose_csr(c.nrows, c.ncols, c.nvals, c.rowptr, c.colidx, c.vals, A->type->size, c.iso,
                     &trp, &tci, &tvx);
    v.own.ptrs[v.own.n++] = trp;
    v.own.ptrs[v.own.n++] = tci;
    v.own.ptrs[v.own.n++] = tvx;
    v.nrows = c.ncols;
    v.ncols = c.nrows;
    v.nvals = c.nvals;
    v.rowptr = trp;
    v.colidx = tci;
    v.vals = tvx;
    v.iso = c.iso;
}

// perm[q] = CSR position of the CSC entry q: a wave per CSC row j, each lane binary-searches
// column j in the CSR row of its entry (built on first use; only the two-sided masked dot
// reads it, for a matrix used as a structural mask)
__global__ __launch_bounds__(256) void k_csc_perm(int64_t ncols, const int64_t *__restrict__ trp,
                                                  const int32_t *__restrict__ tci, const int64_t *__restrict__ rp,
                                                  const int32_t *__restrict__ ci, int64_t *__restrict__ perm) {
    const int lane = threadIdx.x & 63;
    const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
    for (int64_t j = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6; j < ncols; j += nwaves) {
        for (int64_t q = trp[j] + lane; q < trp[j + 1]; q += 64) {
            const int64_t i = tci[q];
            int64_t lo = rp[i], hi = rp[i + 1];
            while (lo < hi) {
                const int64_t mid = (lo + hi) >> 1;
                if (ci[mid] < j) lo = mid + 1;
                else hi = mid;
            }
            perm[q] = lo;
        }
    }
}

const int64_t *gb_csc_perm(GB_Obj *A) {
    GB_REQUIRE(A->kind == GB_KIND_MATRIX, GrB_INVALID_VALUE, "CSC position map of a non-matrix");
    gb_csr_view v;
    gb_get_csc(v, A);
    if (!A->t_perm) {
        A->t_perm = gb_malloc_n<int64_t>(A->nvals ? A->nvals : 1);
        if (A->nvals) {
            int64_t blocks = (A->ncols + 3) / 4;
            if (blocks > 65535) blocks = 65535;
            hipLaunchKernelGGL(k_csc_perm, dim3((unsigned)blocks), dim3(256), 0, gb_stream(), A->ncols, A->t_rowptr,
                               A->t_colidx, A->rowptr, A->colidx, A->t_perm);
            GB_LAUNCH_CHECK();
        }
    }
    return A->t_perm;
}

const void *gb_view_vals_as(gb_csr_view &v, int code, gb_scratch &s) {
    if (code == v.tcode) return v.vals;
    int64_t n = v.iso ? 1 : v.nvals;
    void *d = s.get<char>(n * gb_type_size(code));
    gb_cast_array(d, code, v.vals, v.tcode, n);
    return d;
}

void gb_get_bitmap(gb_bitmap_view &v, GB_Obj *A) {
    v.tcode = A->type->code;
    if (A->kind != GB_KIND_MATRIX) {
        v.n = A->nrows;
        v.bits = A->bits;
        v.iso = A->iso;
        v.count = A->d_nvals;
        if (!A->dense) {  // empty vector: give kernels a valid value pointer
            void *d = v.own.get<char>(A->type->size);
            gb_memset(d, 0, A->type->size);
            v.vals = d;
            v.iso = true;
        } else {
            v.vals = A->dense;
        }
        return;
    }
    GB_REQUIRE(A->ncols == 1, GrB_DIMENSION_MISMATCH, "matrix used as a vector must be n x 1");
    gb_csr_view c;
    gb_get_csr(c, A);
    uint64_t *bits;
    void *dense;
    int64_t *cnt;
    gb_csr_col_to_bitmap(c, A->type->size, &bits, &dense, &cnt);
    v.own.ptrs[v.own.n++] = bits;
    v.own.ptrs[v.own.n++] = dense;
    v.own.ptrs[v.own.n++] = cnt;
    v.count = cnt;
    v.n = A->nrows;
    v.bits = bits;
    v.vals = dense;
    v.iso = A->iso;
}

const void *gb_bitmap_vals_as(gb_bitmap_view &v, int code, gb_scratch &s) {
    if (code == v.tcode) return v.vals;
    int64_t n = v.iso ? 1 : v.n;
    void *d = s.get<char>(n * gb_type_size(code));
    gb_cast_array(d, code, v.vals, v.tcode, n);
    return d;
}

// ================================================================== kernels for build
__global__ void k_check_and_key(const uint64_t *__restrict__ I, const uint64_t *__restrict__ J,
                                int64_t n, uint64_t nrows, uint64_t ncols,
                                uint64_t *__restrict__ keys, int64_t *__restrict__ perm,
                                int *__restrict__ bad) {
    GRID_STRIDE(q, n) {
        uint64_t i = I[q], j = J ? J[q] : 0;
        if (i >= nrows || j >= ncols) {
            *bad = 1;
            i = 0;
            j = 0;
        }
        keys[q] = (i << 32) | j;
        perm[q] = q;
    }
}

__global__ void k_heads(const uint64_t *__restrict__ keys, int64_t n, int64_t *__restrict__ head) {
    GRID_STRIDE(q, n) head[q] = (q == 0 || keys[q] != keys[q - 1]) ? 1 : 0;
}

// one thread per run: fold duplicates in input order with the dup operator
// (dup < 0: keep the last occurrence).
template <class T>
__global__ void k_fold_runs(const uint64_t *__restrict__ keys, const int64_t *__restrict__ perm,
                            const int64_t *__restrict__ pos, int64_t n, const T *__restrict__ X,
                            bool x_iso, int dup, uint64_t *__restrict__ ukeys, T *__restrict__ uvals) {
    GRID_STRIDE(q, n) {
        if (q != 0 && keys[q] == keys[q - 1]) continue;
        T v = X[x_iso ? 0 : perm[q]];
        int64_t r = q + 1;
        for (; r < n && keys[r] == keys[q]; r++) {
            T x = X[x_iso ? 0 : perm[r]];
            v = (dup < 0) ? x : gb_binop<T>(dup, v, x);
        }
        int64_t o = pos[q];
        ukeys[o] = keys[q];
        if (uvals) uvals[o] = v;
    }
}

__global__ void k_rows_hist(const uint64_t *__restrict__ ukeys, int64_t nu,
                            unsigned long long *__restrict__ cnt, int32_t *__restrict__ colidx) {
    GRID_STRIDE(q, nu) {
        atomicAdd(&cnt[ukeys[q] >> 32], 1ULL);
        colidx[q] = (int32_t)(ukeys[q] & 0xffffffffULL);
    }
}

template <class T>
__global__ void k_scatter_vec(const uint64_t *__restrict__ ukeys, const T *__restrict__ uvals,
                              int64_t nu, unsigned long long *__restrict__ bits, T *__restrict__ dense) {
    GRID_STRIDE(q, nu) {
        uint64_t i = ukeys[q] >> 32;
        atomicOr(&bits[i >> 6], 1ULL << (i & 63));
        if (dense) dense[i] = uvals[q];
    }
}

// Sort + dedupe COO tuples on the device.  Returns unique keys (row<<32|col)
// and folded values (already in `code`), count in *nu.
static void coo_sort_fold(const GrB_Index *I, const GrB_Index *J, const void *X_dev, bool x_iso,
                          int64_t n, int64_t nrows, int64_t ncols, int code, int dup_opcode,
                          uint64_t **ukeys_out, void **uvals_out, int64_t *nu_out) {
    gb_scratch s;
    uint64_t *dI = s.get<uint64_t>(n), *dJ = J ? s.get<uint64_t>(n) : nullptr;
    gb_copy_h2d(dI, I, n * sizeof(uint64_t));
    if (J) gb_copy_h2d(dJ, J, n * sizeof(uint64_t));
    uint64_t *keys = s.get<uint64_t>(n);
    int64_t *perm = s.get<int64_t>(n);
    int *bad = s.get<int>(1);
    gb_memset(bad, 0, sizeof(int));
    hipLaunchKernelGGL(k_check_and_key, dim3(grid_for(n)), dim3(GB_BLOCK), 0, gb_stream(), dI, dJ, n,
                       (uint64_t)nrows, (uint64_t)ncols, keys, perm, bad);
    GB_LAUNCH_CHECK();
    int hbad = 0;
    gb_copy_d2h(&hbad, bad, sizeof(int));
    GB_REQUIRE(!hbad, GrB_INDEX_OUT_OF_BOUNDS, "index out of bounds in build");
    int rbits = 1;
    while (rbits < 31 && (1LL << rbits) < nrows) rbits++;
    gb_sort_pairs_u64(keys, perm, n, 32 + rbits);
    int64_t *head = s.get<int64_t>(n), *pos = s.get<int64_t>(n + 1);
    hipLaunchKernelGGL(k_heads, dim3(grid_for(n)), dim3(GB_BLOCK), 0, gb_stream(), keys, n, head);
    GB_LAUNCH_CHECK();
    gb_exclusive_scan_i64(head, pos, n);
    int64_t nu = gb_read_i64(pos + n);
    uint64_t *ukeys = gb_malloc_n<uint64_t>(nu);
    void *uvals = X_dev ? gb_malloc(nu * gb_type_size(code)) : nullptr;
    with_type(code, [&](auto z) {
        using T = decltype(z);
        hipLaunchKernelGGL(k_fold_runs<T>, dim3(grid_for(n)), dim3(GB_BLOCK), 0, gb_stream(), keys, perm,
                           pos, n, (const T *)X_dev, x_iso, dup_opcode, ukeys, (T *)uvals);
    });
    GB_LAUNCH_CHECK();
    *ukeys_out = ukeys;
    *uvals_out = uvals;
    *nu_out = nu;
}

void gb_build(GB_Obj *C, const GrB_Index *I, const GrB_Index *J, const void *X, int xcode,
                         bool x_iso, int64_t n, GrB_BinaryOp dup) {
    GB_REQUIRE(C->kind == GB_KIND_MATRIX || C->ncols == 1, GrB_INVALID_OBJECT, "bad build target");
    GB_REQUIRE(gb_nvals(C) == 0, GrB_OUTPUT_NOT_EMPTY, "output is not empty");
    if (n == 0) return;
    GB_REQUIRE(I && (J || C->kind != GB_KIND_MATRIX) && X, GrB_NULL_POINTER, "NULL build array");
    int code = C->type->code;
    size_t ts = C->type->size;
    gb_scratch s;
    int64_t nx = x_iso ? 1 : n;
    void *Xraw = s.get<char>(nx * gb_type_size(xcode));
    gb_copy_h2d(Xraw, X, nx * gb_type_size(xcode));
    void *Xc = Xraw;
    if (xcode != code) {
        Xc = s.get<char>(nx * ts);
        gb_cast_array(Xc, code, Xraw, xcode, nx);
    }
    int dupop = dup ? dup->opcode : -1;
    uint64_t *ukeys;
    void *uvals;
    int64_t nu;
    bool is_vec = C->kind != GB_KIND_MATRIX;
    coo_sort_fold(I, is_vec ? nullptr : J, Xc, x_iso, n, C->nrows, is_vec ? 1 : C->ncols, code, dupop,
                  &ukeys, &uvals, &nu);
    if (x_iso) {  // every folded value equals the scalar unless a dup op changed it
        if (dup == nullptr || dup->opcode == GBAMD_OP_FIRST || dup->opcode == GBAMD_OP_SECOND ||
            dup->opcode == GBAMD_OP_ANY || dup->opcode == GBAMD_OP_MIN || dup->opcode == GBAMD_OP_MAX ||
            dup->opcode == GBAMD_OP_LOR || dup->opcode == GBAMD_OP_LAND) {
            gb_free(uvals);
            uvals = gb_malloc(ts);
            gb_copy_d2d(uvals, Xc, ts);
        } else {
            x_iso = false;
        }
    }
    if (!is_vec) {
        int64_t *cnt = s.get<int64_t>(C->nrows + 1);
        gb_memset(cnt, 0, (C->nrows + 1) * sizeof(int64_t));
        int32_t *colidx = gb_malloc_n<int32_t>(nu);
        hipLaunchKernelGGL(k_rows_hist, dim3(grid_for(nu)), dim3(GB_BLOCK), 0, gb_stream(), ukeys, nu,
                           (unsigned long long *)cnt, colidx);
        GB_LAUNCH_CHECK();
        int64_t *rowptr = gb_malloc_n<int64_t>(C->nrows + 1);
        gb_exclusive_scan_i64(cnt, rowptr, C->nrows);
        gb_free(ukeys);
        gb_install_csr(C, C->nrows, C->ncols, nu, rowptr, colidx, uvals, x_iso);
    } else {
        int64_t nw = gb_words(C->nrows);
        uint64_t *bits = gb_malloc_n<uint64_t>(nw);
        gb_memset(bits, 0, nw * sizeof(uint64_t));
        void *dense = x_iso ? uvals : gb_malloc(C->nrows * ts);
        with_type(code, [&](auto z) {
            using T = decltype(z);
            hipLaunchKernelGGL(k_scatter_vec<T>, dim3(grid_for(nu)), dim3(GB_BLOCK), 0, gb_stream(), ukeys,
                               (const T *)uvals, nu, (unsigned long long *)bits, x_iso ? nullptr : (T *)dense);
        });
        GB_LAUNCH_CHECK();
        gb_free(ukeys);
        if (!x_iso) gb_free(uvals);
        int64_t *cnt = gb_malloc_n<int64_t>(1);
        gb_copy_h2d(cnt, &nu, sizeof(int64_t));
        gb_sync();
        gb_install_bitmap(C, C->nrows, bits, dense, x_iso, cnt);
        C->nvals = nu;
        C->nvals_valid = true;
    }
}

// ================================================================== extract
__global__ void k_rows_of(const int64_t *__restrict__ rowptr, int64_t nrows, uint64_t *__restrict__ I) {
    int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
    int lane = threadIdx.x & 63;
    int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
    for (int64_t i = wave; i < nrows; i += nw)
        for (int64_t p = rowptr[i] + lane; p < rowptr[i + 1]; p += 64) I[p] = (uint64_t)i;
}
__global__ void k_i32_to_u64(const int32_t *__restrict__ a, int64_t n, uint64_t *__restrict__ b) {
    GRID_STRIDE(q, n) b[q] = (uint64_t)(uint32_t)a[q];
}
__global__ void k_word_pop2(const uint64_t *__restrict__ bits, int64_t nw, int64_t *__restrict__ pop) {
    GRID_STRIDE(w, nw) pop[w] = __popcll(bits[w]);
}
template <class T>
__global__ void k_bitmap_compact(const uint64_t *__restrict__ bits, const T *__restrict__ dense, bool iso,
                                 int64_t n, const int64_t *__restrict__ woff, uint64_t *__restrict__ idx,
                                 T *__restrict__ vals) {
    GRID_STRIDE(i, n) {
        uint64_t w = bits[i >> 6];
        int b = i & 63;
        if ((w >> b) & 1ULL) {
            int64_t r = woff[i >> 6] + __popcll(b ? (w & (~0ULL >> (64 - b))) : 0ULL);
            idx[r] = (uint64_t)i;
            if (vals) vals[r] = iso ? dense[0] : dense[i];
        }
    }
}

// copy (cast) device values to a host array of type `code`
static void values_to_host(void *host, int code, const void *dvals, int src_code, bool iso, int64_t n) {
    if (n == 0) return;
    gb_scratch s;
    const void *src = dvals;
    int64_t m = iso ? 1 : n;
    if (code != src_code) {
        void *t = s.get<char>(m * gb_type_size(code));
        gb_cast_array(t, code, dvals, src_code, m);
        src = t;
    }
    if (iso) {
        char one[16];
        gb_copy_d2h(one, src, gb_type_size(code));
        for (int64_t q = 0; q < n; q++) memcpy((char *)host + q * gb_type_size(code), one, gb_type_size(code));
    } else {
        gb_copy_d2h(host, src, n * gb_type_size(code));
    }
}

void gb_extract_tuples(GB_Obj *A, GrB_Index *I, GrB_Index *J, void *X, int xcode, GrB_Index *nvals) {
    GB_REQUIRE(nvals, GrB_NULL_POINTER, "nvals is NULL");
    int64_t nz = gb_nvals(A);
    GB_REQUIRE((int64_t)*nvals >= nz, GrB_INSUFFICIENT_SPACE, "output arrays too small");
    *nvals = nz;
    if (nz == 0) return;
    gb_scratch s;
    if (A->kind == GB_KIND_MATRIX) {
        if (I) {
            uint64_t *dI = s.get<uint64_t>(nz);
            hipLaunchKernelGGL(k_rows_of, dim3(grid_for(A->nrows * 64)), dim3(GB_BLOCK), 0, gb_stream(),
                               A->rowptr, A->nrows, dI);
            GB_LAUNCH_CHECK();
            gb_copy_d2h(I, dI, nz * sizeof(uint64_t));
        }
        if (J) {
            uint64_t *dJ = s.get<uint64_t>(nz);
            hipLaunchKernelGGL(k_i32_to_u64, dim3(grid_for(nz)), dim3(GB_BLOCK), 0, gb_stream(), A->colidx,
                               nz, dJ);
            GB_LAUNCH_CHECK();
            gb_copy_d2h(J, dJ, nz * sizeof(uint64_t));
        }
        if (X) values_to_host(X, xcode, A->vals, A->type->code, A->iso, nz);
        return;
    }
    int64_t n = A->nrows, nw = gb_words(n);
    int64_t *pop = s.get<int64_t>(nw), *woff = s.get<int64_t>(nw + 1);
    hipLaunchKernelGGL(k_word_pop2, dim3(grid_for(nw)), dim3(GB_BLOCK), 0, gb_stream(), A->bits, nw, pop);
    GB_LAUNCH_CHECK();
    gb_exclusive_scan_i64(pop, woff, nw);
    uint64_t *dI = s.get<uint64_t>(nz);
    void *dX = (X && !A->iso) ? s.get<char>(nz * A->type->size) : nullptr;
    with_type(A->type->code, [&](auto z) {
        using T = decltype(z);
        hipLaunchKernelGGL(k_bitmap_compact<T>, dim3(grid_for(n)), dim3(GB_BLOCK), 0, gb_stream(), A->bits,
                           (const T *)A->dense, A->iso, n, woff, dI, (T *)dX);
    });
    GB_LAUNCH_CHECK();
    if (I) gb_copy_d2h(I, dI, nz * sizeof(uint64_t));
    if (J) memset(J, 0, nz * sizeof(GrB_Index));
    if (X) {
        if (A->iso) values_to_host(X, xcode, A->dense, A->type->code, true, nz);
        else values_to_host(X, xcode, dX, A->type->code, false, nz);
    }
}

// ================================================================== element access
// binary search of (i, j) in CSR; result: pos (or insertion point) and found flag
__global__ void k_find(const int64_t *__restrict__ rowptr, const int32_t *__restrict__ colidx, int64_t i,
                       int32_t j, int64_t *__restrict__ out) {
    int64_t lo = rowptr[i], hi = rowptr[i + 1];
    while (lo < hi) {
        int64_t mid = (lo + hi) >> 1;
        if (colidx[mid] < j) lo = mid + 1;
        else hi = mid;
    }
    out[0] = lo;
    out[1] = (lo < rowptr[i + 1] && colidx[lo] == j) ? 1 : 0;
}

template <class T>
__global__ void k_insert(const int64_t *__restrict__ rp, const int32_t *__restrict__ ci, const T *__restrict__ vx,
                         int64_t nrows, int64_t nvals, int64_t row, int64_t pos, int32_t col, T val,
                         int64_t *__restrict__ rp2, int32_t *__restrict__ ci2, T *__restrict__ vx2) {
    GRID_STRIDE(q, nvals + 1) {
        if (q < pos) {
            ci2[q] = ci[q];
            vx2[q] = vx[q];
        } else if (q == pos) {
            ci2[q] = col;
            vx2[q] = val;
        } else {
            ci2[q] = ci[q - 1];
            vx2[q] = vx[q - 1];
        }
    }
    GRID_STRIDE(r, nrows + 1) rp2[r] = rp[r] + (r > row ? 1 : 0);
}

template <class T>
__global__ void k_delete(const int64_t *__restrict__ rp, const int32_t *__restrict__ ci, const T *__restrict__ vx,
                         int64_t nrows, int64_t nvals, int64_t row, int64_t pos, int64_t *__restrict__ rp2,
                         int32_t *__restrict__ ci2, T *__restrict__ vx2, bool iso) {
    GRID_STRIDE(q, nvals - 1) {
        int64_t src = q < pos ? q : q + 1;
        ci2[q] = ci[src];
        if (!iso) vx2[q] = vx[src];
    }
    GRID_STRIDE(r, nrows + 1) rp2[r] = rp[r] - (r > row ? 1 : 0);
}

static void matrix_de_iso(GB_Obj *A) {
    if (!A->iso) return;
    void *full = gb_expand_iso(A->vals, A->type->size, A->nvals);
    gb_free(A->vals);
    A->vals = full;
    A->iso = false;
    gb_drop_transpose(A);
}

static void vector_de_iso(GB_Obj *v) {
    if (!v->iso) return;
    void *full = gb_expand_iso(v->dense, v->type->size, v->nrows);
    gb_free(v->dense);
    v->dense = full;
    v->iso = false;
}

template <class T>
static void matrix_set_element(GB_Obj *A, T x, int64_t i, int64_t j) {
    GB_REQUIRE(i >= 0 && i < A->nrows && j >= 0 && j < A->ncols, GrB_INVALID_INDEX, "index out of range");
    gb_scratch s;
    int64_t *res = s.get<int64_t>(2);
    hipLaunchKernelGGL(k_find, dim3(1), dim3(1), 0, gb_stream(), A->rowptr, A->colidx, i, (int32_t)j, res);
    GB_LAUNCH_CHECK();
    int64_t h[2];
    gb_copy_d2h(h, res, sizeof(h));
    if (h[1]) {
        if (A->iso) {
            T cur;
            gb_copy_d2h(&cur, A->vals, sizeof(T));
            if (memcmp(&cur, &x, sizeof(T)) == 0) return;
            matrix_de_iso(A);
        }
        gb_copy_h2d((T *)A->vals + h[0], &x, sizeof(T));
        gb_sync();
        gb_drop_transpose(A);
        return;
    }
    matrix_de_iso(A);
    int64_t nz = A->nvals;
    int64_t *rp2 = gb_malloc_n<int64_t>(A->nrows + 1);
    int32_t *ci2 = gb_malloc_n<int32_t>(nz + 1);
    T *vx2 = gb_malloc_n<T>(nz + 1);
    const T *vx = (const T *)(A->vals ? A->vals : (void *)vx2);
    hipLaunchKernelGGL(k_insert<T>, dim3(grid_for(std::max(nz + 1, A->nrows + 1))), dim3(GB_BLOCK), 0, gb_stream(),
                       A->rowptr, A->colidx ? A->colidx : ci2, vx, A->nrows, nz, i, h[0], (int32_t)j, x, rp2,
                       ci2, vx2);
    GB_LAUNCH_CHECK();
    gb_sync();
    gb_install_csr(A, A->nrows, A->ncols, nz + 1, rp2, ci2, vx2, false);
}

template <class T>
__global__ void k_vec_set(unsigned long long *__restrict__ bits, T *__restrict__ dense, int64_t i, T x,
                          unsigned long long *__restrict__ cnt, T *__restrict__ iso_init) {
    unsigned long long m = 1ULL << (i & 63);
    unsigned long long old = atomicOr(&bits[i >> 6], m);
    if (dense) dense[i] = x;
    if (iso_init) *iso_init = x;  // first entry of an empty vector: its iso value
    if (!(old & m)) atomicAdd(cnt, 1ULL);
}
__global__ void k_vec_clear(unsigned long long *__restrict__ bits, int64_t i, unsigned long long *__restrict__ cnt) {
    unsigned long long m = 1ULL << (i & 63);
    unsigned long long old = atomicAnd(&bits[i >> 6], ~m);
    if (old & m) atomicAdd(cnt, (unsigned long long)-1LL);
}

// ---- the pending root (gb_internal.h)
std::atomic<bool> g_root_active{false};
thread_local int g_root_hold = 0;
static std::mutex g_root_mu;
static GB_Obj *g_root_v = nullptr;
static int64_t g_root_i = -1;

void gb_root_flush() {
    std::lock_guard<std::mutex> lk(g_root_mu);
    GB_Obj *v = g_root_v;
    g_root_v = nullptr;
    g_root_active.store(false, std::memory_order_release);
    if (!v || v->magic != GB_MAGIC) return;
    hipLaunchKernelGGL(k_vec_set<bool>, dim3(1), dim3(1), 0, gb_stream(), (unsigned long long *)v->bits, nullptr,
                       g_root_i, true, (unsigned long long *)v->d_nvals, (bool *)v->dense);
    GB_LAUNCH_CHECK();
}
bool gb_root_pending(const GB_Obj *v) {
    if (!g_root_active.load(std::memory_order_acquire)) return false;
    std::lock_guard<std::mutex> lk(g_root_mu);
    return v && v == g_root_v;
}
int64_t gb_root_take(GB_Obj *v) {
    std::lock_guard<std::mutex> lk(g_root_mu);
    if (!v || v != g_root_v) return -1;
    g_root_v = nullptr;
    g_root_active.store(false, std::memory_order_release);
    return g_root_i;
}
const void *gb_bool_true_dev() {
    static std::mutex mu;
    static bool *p = nullptr;
    std::lock_guard<std::mutex> lk(mu);
    if (!p) {
        GB_HIP(hipMalloc((void **)&p, 16));
        const unsigned char one[16] = {1};
        GB_HIP(hipMemcpy(p, one, sizeof(one), hipMemcpyHostToDevice));
    }
    return p;
}

template <class T>
static void vector_set_element(GB_Obj *v, T x, int64_t i) {
    GB_REQUIRE(i >= 0 && i < v->nrows, GrB_INVALID_INDEX, "index out of range");
    if constexpr (std::is_same<T, bool>::value) {
        // the first entry of an empty BOOL vector, true: deferred (the BFS root; gb_internal.h)
        if (x && v->kind == GB_KIND_VECTOR && v->type->code == GBAMD_T_BOOL && v->nvals_valid && v->nvals == 0 &&
            !v->dense && v->bits && v->invalid == GrB_SUCCESS && gb_knob("root_defer") != 1) {
            if (g_root_active.load(std::memory_order_acquire)) gb_root_flush();  // one record at a time
            v->dense = gb_malloc(sizeof(bool));  // written when the root materialises (or never read)
            v->iso = true;
            v->nvals = 1;  // known on the host
            v->hint_valid = false;
            std::lock_guard<std::mutex> lk(g_root_mu);
            g_root_v = v;
            g_root_i = i;
            g_root_active.store(true, std::memory_order_release);
            return;
        }
    }
    T *iso_init = nullptr;
    if (!v->dense) {
        // first value: store it as an iso vector (the set kernel writes the value)
        v->dense = gb_malloc(sizeof(T));
        iso_init = (T *)v->dense;
        v->iso = true;
    } else if (v->iso) {
        T cur;
        gb_copy_d2h(&cur, v->dense, sizeof(T));
        if (memcmp(&cur, &x, sizeof(T)) != 0 || gb_nvals(v) == 0) {
            if (gb_nvals(v) == 0) {
                gb_copy_h2d(v->dense, &x, sizeof(T));
                gb_sync();
            } else {
                vector_de_iso(v);
            }
        }
    }
    const bool was_empty = v->nvals_valid && v->nvals == 0;
    hipLaunchKernelGGL(k_vec_set<T>, dim3(1), dim3(1), 0, gb_stream(), (unsigned long long *)v->bits,
                       v->iso ? nullptr : (T *)v->dense, i, x, (unsigned long long *)v->d_nvals, iso_init);
    GB_LAUNCH_CHECK();
    // the count stays known on the host when the vector was known to be empty
    v->nvals_valid = was_empty;
    v->nvals = was_empty ? 1 : v->nvals;
    v->hint_valid = false;
}

template <class T>
static GrB_Info vector_extract_element(T *x, GB_Obj *v, int64_t i) {
    GB_REQUIRE(x, GrB_NULL_POINTER, "x is NULL");
    GB_REQUIRE(i >= 0 && i < v->nrows, GrB_INVALID_INDEX, "index out of range");
    uint64_t w;
    gb_copy_d2h(&w, v->bits + (i >> 6), sizeof(w));
    if (!((w >> (i & 63)) & 1ULL)) return GrB_NO_VALUE;
    char buf[16];
    int code = v->type->code;
    gb_copy_d2h(buf, (const char *)v->dense + (v->iso ? 0 : i * v->type->size), v->type->size);
    with_type(code, [&](auto z) {
        using S = decltype(z);
        S sv;
        memcpy(&sv, buf, sizeof(S));
        *x = gb_cast<T, S>(sv);
    });
    return GrB_SUCCESS;
}

template <class T>
static GrB_Info matrix_extract_element(T *x, GB_Obj *A, int64_t i, int64_t j) {
    GB_REQUIRE(x, GrB_NULL_POINTER, "x is NULL");
    GB_REQUIRE(i >= 0 && i < A->nrows && j >= 0 && j < A->ncols, GrB_INVALID_INDEX, "index out of range");
    gb_scratch s;
    int64_t *res = s.get<int64_t>(2);
    hipLaunchKernelGGL(k_find, dim3(1), dim3(1), 0, gb_stream(), A->rowptr, A->colidx, i, (int32_t)j, res);
    GB_LAUNCH_CHECK();
    int64_t h[2];
    gb_copy_d2h(h, res, sizeof(h));
    if (!h[1]) return GrB_NO_VALUE;
    char buf[16];
    gb_copy_d2h(buf, (const char *)A->vals + (A->iso ? 0 : h[0] * A->type->size), A->type->size);
    with_type(A->type->code, [&](auto z) {
        using S = decltype(z);
        S sv;
        memcpy(&sv, buf, sizeof(S));
        *x = gb_cast<T, S>(sv);
    });
    return GrB_SUCCESS;
}

static void matrix_remove_element(GB_Obj *A, int64_t i, int64_t j) {
    GB_REQUIRE(i >= 0 && i < A->nrows && j >= 0 && j < A->ncols, GrB_INVALID_INDEX, "index out of range");
    gb_scratch s;
    int64_t *res = s.get<int64_t>(2);
    hipLaunchKernelGGL(k_find, dim3(1), dim3(1), 0, gb_stream(), A->rowptr, A->colidx, i, (int32_t)j, res);
    GB_LAUNCH_CHECK();
    int64_t h[2];
    gb_copy_d2h(h, res, sizeof(h));
    if (!h[1]) return;
    int64_t nz = A->nvals;
    int64_t *rp2 = gb_malloc_n<int64_t>(A->nrows + 1);
    int32_t *ci2 = gb_malloc_n<int32_t>(nz - 1);
    size_t ts = A->type->size;
    void *vx2 = A->iso ? gb_malloc(ts) : gb_malloc((nz - 1) * ts);
    if (A->iso) gb_copy_d2d(vx2, A->vals, ts);
    with_type(A->type->code, [&](auto z) {
        using T = decltype(z);
        hipLaunchKernelGGL(k_delete<T>, dim3(grid_for(std::max(nz, A->nrows + 1))), dim3(GB_BLOCK), 0, gb_stream(),
                           A->rowptr, A->colidx, (const T *)A->vals, A->nrows, nz, i, h[0], rp2, ci2, (T *)vx2,
                           A->iso);
    });
    GB_LAUNCH_CHECK();
    gb_install_csr(A, A->nrows, A->ncols, nz - 1, rp2, ci2, vx2, A->iso);
}

// ================================================================== import / export
__global__ void k_u64_to_i32_check(const uint64_t *__restrict__ a, int64_t n, uint64_t bound,
                                   int32_t *__restrict__ b, int *__restrict__ bad) {
    GRID_STRIDE(q, n) {
        uint64_t x = a[q];
        if (x >= bound) {
            *bad = 1;
            x = 0;
        }
        b[q] = (int32_t)x;
    }
}
// rows must be strictly increasing in column index (sorted, no duplicates)
__global__ void k_check_sorted(const int64_t *__restrict__ rowptr, const int32_t *__restrict__ ci, int64_t nrows,
                               int *__restrict__ jumbled) {
    GRID_STRIDE(i, nrows) {
        for (int64_t p = rowptr[i] + 1; p < rowptr[i + 1]; p++)
            if (ci[p] <= ci[p - 1]) {
                *jumbled = 1;
                break;
            }
    }
}

static void import_csr(GB_Obj *A, const GrB_Index *Ap, const GrB_Index *Ai, const void *Ax, int xcode,
                       int64_t nrows, int64_t ncols, int64_t nvals, bool x_iso) {
    gb_scratch s;
    int64_t *rp = gb_malloc_n<int64_t>(nrows + 1);
    gb_copy_h2d(rp, Ap, (nrows + 1) * sizeof(int64_t));
    uint64_t *ai = s.get<uint64_t>(nvals);
    gb_copy_h2d(ai, Ai, nvals * sizeof(uint64_t));
    int32_t *ci = gb_malloc_n<int32_t>(nvals);
    int *flags = s.get<int>(2);
    gb_memset(flags, 0, 2 * sizeof(int));
    hipLaunchKernelGGL(k_u64_to_i32_check, dim3(grid_for(nvals)), dim3(GB_BLOCK), 0, gb_stream(), ai, nvals,
                       (uint64_t)ncols, ci, flags);
    hipLaunchKernelGGL(k_check_sorted, dim3(grid_for(nrows)), dim3(GB_BLOCK), 0, gb_stream(), rp, ci, nrows,
                       flags + 1);
    GB_LAUNCH_CHECK();
    int h[2];
    gb_copy_d2h(h, flags, sizeof(h));
    if (h[0]) {
        gb_free(rp);
        gb_free(ci);
        gb_throw(GrB_INDEX_OUT_OF_BOUNDS, "column index out of bounds in import");
    }
    int64_t nx = x_iso ? 1 : nvals;
    void *vx = gb_malloc(nx * A->type->size);
    {
        void *raw = s.get<char>(nx * gb_type_size(xcode));
        gb_copy_h2d(raw, Ax, nx * gb_type_size(xcode));
        gb_cast_array(vx, A->type->code, raw, xcode, nx);
    }
    if (!h[1]) {
        gb_sync();
        gb_install_csr(A, nrows, ncols, nvals, rp, ci, vx, x_iso);
        return;
    }
    // jumbled rows: go through the COO build path (sorts; duplicates keep the last)
    std::vector<GrB_Index> I(nvals), Ap_h(nrows + 1);
    memcpy(Ap_h.data(), Ap, (nrows + 1) * sizeof(GrB_Index));
    for (int64_t r = 0; r < nrows; r++)
        for (GrB_Index p = Ap_h[r]; p < Ap_h[r + 1]; p++) I[p] = r;
    gb_free(rp);
    gb_free(ci);
    std::vector<char> Xh(nx * A->type->size);
    gb_copy_d2h(Xh.data(), vx, Xh.size());
    gb_free(vx);
    A->nrows = nrows;
    A->ncols = ncols;
    gb_obj_free_storage(A);
    alloc_empty_storage(A);
    gb_build(A, I.data(), Ai, Xh.data(), A->type->code, x_iso, nvals, nullptr);
}

static void export_matrix(GB_Obj *A, GrB_Index *Ap, GrB_Index *Ai, void *Ax, int xcode, GrB_Index *Ap_len,
                          GrB_Index *Ai_len, GrB_Index *Ax_len, GrB_Format format) {
    GB_REQUIRE(Ap_len && Ai_len && Ax_len, GrB_NULL_POINTER, "NULL length");
    int64_t nz = A->nvals;
    gb_csr_view v;
    int64_t np;
    if (format == GrB_CSR_FORMAT) {
        gb_get_csr(v, A);
        np = A->nrows + 1;
    } else if (format == GrB_CSC_FORMAT) {
        gb_get_csc(v, A);
        np = A->ncols + 1;
    } else {
        gb_get_csr(v, A);
        np = nz;
    }
    GB_REQUIRE((int64_t)*Ap_len >= np && (int64_t)*Ai_len >= nz && (int64_t)*Ax_len >= nz,
               GrB_INSUFFICIENT_SPACE, "export arrays too small");
    gb_scratch s;
    if (format == GrB_COO_FORMAT) {
        uint64_t *dI = s.get<uint64_t>(nz);
        if (nz) {
            hipLaunchKernelGGL(k_rows_of, dim3(grid_for(v.nrows * 64)), dim3(GB_BLOCK), 0, gb_stream(), v.rowptr,
                               v.nrows, dI);
            GB_LAUNCH_CHECK();
        }
        gb_copy_d2h(Ap, dI, nz * sizeof(uint64_t));
    } else {
        gb_copy_d2h(Ap, v.rowptr, np * sizeof(int64_t));
    }
    if (nz) {
        uint64_t *dJ = s.get<uint64_t>(nz);
        hipLaunchKernelGGL(k_i32_to_u64, dim3(grid_for(nz)), dim3(GB_BLOCK), 0, gb_stream(), v.colidx, nz, dJ);
        GB_LAUNCH_CHECK();
        gb_copy_d2h(Ai, dJ, nz * sizeof(uint64_t));
        values_to_host(Ax, xcode, v.vals, A->type->code, v.iso, nz);
    }
    *Ap_len = np;
    *Ai_len = nz;
    *Ax_len = nz;
}

// ================================================================== resize
__global__ void k_resize_rows(const int64_t *__restrict__ rp, const int32_t *__restrict__ ci, int64_t nrows_keep,
                              int64_t ncols, int64_t *__restrict__ cnt) {
    GRID_STRIDE(i, nrows_keep) {
        int64_t c = 0;
        for (int64_t p = rp[i]; p < rp[i + 1]; p++) c += ci[p] < ncols;
        cnt[i] = c;
    }
}
template <class T>
__global__ void k_resize_fill(const int64_t *__restrict__ rp, const int32_t *__restrict__ ci, const T *__restrict__ vx,
                              int64_t nrows_keep, int64_t ncols, const int64_t *__restrict__ rp2,
                              int32_t *__restrict__ ci2, T *__restrict__ vx2) {
    GRID_STRIDE(i, nrows_keep) {
        int64_t o = rp2[i];
        for (int64_t p = rp[i]; p < rp[i + 1]; p++)
            if (ci[p] < ncols) {
                ci2[o] = ci[p];
                if (vx2) vx2[o] = vx[p];
                o++;
            }
    }
}

static void matrix_resize(GB_Obj *A, int64_t nrows, int64_t ncols) {
    GB_REQUIRE(ncols < (1LL << 31), GrB_OUT_OF_MEMORY, "too many columns");
    int64_t keep = std::min(nrows, A->nrows);
    gb_scratch s;
    int64_t *cnt = s.get<int64_t>(nrows + 1);
    gb_memset(cnt, 0, (nrows + 1) * sizeof(int64_t));
    if (keep && A->nvals) {
        hipLaunchKernelGGL(k_resize_rows, dim3(grid_for(keep)), dim3(GB_BLOCK), 0, gb_stream(), A->rowptr,
                           A->colidx, keep, ncols, cnt);
        GB_LAUNCH_CHECK();
    }
    int64_t *rp2 = gb_malloc_n<int64_t>(nrows + 1);
    gb_exclusive_scan_i64(cnt, rp2, nrows);
    int64_t nz = gb_read_i64(rp2 + nrows);
    int32_t *ci2 = gb_malloc_n<int32_t>(nz);
    size_t ts = A->type->size;
    void *vx2 = A->iso ? gb_malloc(ts) : gb_malloc(nz * ts);
    if (A->iso) gb_copy_d2d(vx2, A->vals, ts);
    if (nz) {
        with_type(A->type->code, [&](auto z) {
            using T = decltype(z);
            hipLaunchKernelGGL(k_resize_fill<T>, dim3(grid_for(keep)), dim3(GB_BLOCK), 0, gb_stream(), A->rowptr,
                               A->colidx, (const T *)A->vals, keep, ncols, rp2, ci2, A->iso ? nullptr : (T *)vx2);
        });
        GB_LAUNCH_CHECK();
    }
    gb_install_csr(A, nrows, ncols, nz, rp2, ci2, vx2, A->iso);
}

__global__ void k_bits_truncate(uint64_t *__restrict__ bits, int64_t nw_new, int64_t n_new) {
    GRID_STRIDE(w, nw_new) {
        int64_t lo = w << 6;
        if (lo + 64 > n_new) {
            int keep = (int)(n_new - lo);
            bits[w] &= keep <= 0 ? 0ULL : (keep >= 64 ? ~0ULL : ((1ULL << keep) - 1));
        }
    }
}

static void vector_resize(GB_Obj *v, int64_t n) {
    int64_t nw_old = gb_words(v->nrows), nw = gb_words(n);
    uint64_t *bits = gb_malloc_n<uint64_t>(nw);
    gb_memset(bits, 0, nw * sizeof(uint64_t));
    gb_copy_d2d(bits, v->bits, std::min(nw, nw_old) * sizeof(uint64_t));
    if (n < v->nrows && nw) {
        hipLaunchKernelGGL(k_bits_truncate, dim3(grid_for(nw)), dim3(GB_BLOCK), 0, gb_stream(), bits, nw, n);
        GB_LAUNCH_CHECK();
    }
    void *dense = nullptr;
    size_t ts = v->type->size;
    if (v->dense) {
        if (v->iso) {
            dense = gb_malloc(ts);
            gb_copy_d2d(dense, v->dense, ts);
        } else {
            dense = gb_malloc(n * ts);
            gb_copy_d2d(dense, v->dense, std::min(n, v->nrows) * ts);
        }
    }
    bool iso = v->iso;
    gb_free(v->bits);
    gb_free(v->dense);
    v->bits = nullptr;
    v->dense = nullptr;
    v->nrows = n;
    v->bits = bits;
    v->dense = dense;
    v->iso = iso;
    gb_bitmap_count(bits, n, v->d_nvals);
    v->nvals_valid = false;
    v->hint_valid = false;
}

// ================================================================== dup
static GB_Obj *dup_object(GB_Obj *A) {
    GB_Obj *C = gb_new_object(A->kind, A->type, A->nrows, A->ncols);
    size_t ts = A->type->size;
    if (A->kind == GB_KIND_MATRIX) {
        gb_copy_d2d(C->rowptr, A->rowptr, (A->nrows + 1) * sizeof(int64_t));
        C->nvals = A->nvals;
        C->iso = A->iso;
        C->colidx = gb_malloc_n<int32_t>(A->nvals);
        gb_copy_d2d(C->colidx, A->colidx, A->nvals * sizeof(int32_t));
        int64_t nv = A->iso ? 1 : A->nvals;
        C->vals = gb_malloc(nv * ts);
        if (A->vals) gb_copy_d2d(C->vals, A->vals, nv * ts);
    } else {
        gb_copy_d2d(C->bits, A->bits, gb_words(A->nrows) * sizeof(uint64_t));
        gb_copy_d2d(C->d_nvals, A->d_nvals, sizeof(int64_t));
        C->nvals = A->nvals;
        C->nvals_valid = A->nvals_valid;
        C->iso = A->iso;
        if (A->dense) {
            int64_t nv = A->iso ? 1 : A->nrows;
            C->dense = gb_malloc(nv * ts);
            gb_copy_d2d(C->dense, A->dense, nv * ts);
        }
    }
    return C;
}

// ================================================================== C API
extern "C" {

// ---------------- Matrix
GrB_Info GrB_Matrix_new(GrB_Matrix *A, GrB_Type type, GrB_Index nrows, GrB_Index ncols) {
    if (!A) return GrB_NULL_POINTER;
    return gb_api(nullptr, [&] { *A = (GrB_Matrix)gb_new_object(GB_KIND_MATRIX, type, nrows, ncols); });
}
GrB_Info GrB_Matrix_dup(GrB_Matrix *C, const GrB_Matrix A) {
    if (!C) return GrB_NULL_POINTER;
    return gb_api(nullptr, [&] { *C = (GrB_Matrix)dup_object(gb_obj_check(A)); });
}
GrB_Info GrB_Matrix_clear(GrB_Matrix A) {
    GB_HPROF(6, "GrB_*_clear");
    GB_Obj *o = OBJ(A);
    return gb_api(o, [&] {
        gb_obj_check_raw(A);
        if (o->kind != GB_KIND_MATRIX && gb_zpool_clear_vector(o)) return;  // no launch
        gb_obj_free_storage(o);
        alloc_empty_storage(o);
    });
}
GrB_Info GrB_Matrix_nrows(GrB_Index *n, const GrB_Matrix A) {
    if (!n) return GrB_NULL_POINTER;
    return gb_api(OBJ(A), [&] { *n = gb_obj_check_raw(A)->nrows; });
}
GrB_Info GrB_Matrix_ncols(GrB_Index *n, const GrB_Matrix A) {
    if (!n) return GrB_NULL_POINTER;
    return gb_api(OBJ(A), [&] { *n = gb_obj_check_raw(A)->ncols; });
}
GrB_Info GrB_Matrix_nvals(GrB_Index *n, const GrB_Matrix A) {
    if (!n) return GrB_NULL_POINTER;
    GB_HPROF(7, "GrB_*_nvals (incl. wait)");
    // a speculated BFS level (gb_ops.hip) changes only its stamp target: counts of anything else
    // are read without rolling it back
    if (g_spec_active.load(std::memory_order_acquire)) {
        GrB_Info e = gb_api_impl<false>(OBJ(A), [&] { gb_spec_resolve(A); });
        if (e != GrB_SUCCESS) return e;
    }
    gb_spec_hold_guard hold;
    return gb_api(OBJ(A), [&] { *n = gb_nvals(gb_obj_check_raw(A)); });
}
GrB_Info GrB_Matrix_resize(GrB_Matrix A, GrB_Index nrows, GrB_Index ncols) {
    return gb_api(OBJ(A), [&] {
        GB_Obj *o = gb_obj_check(A);
        if (o->kind == GB_KIND_MATRIX) matrix_resize(o, nrows, ncols);
        else {
            GB_REQUIRE(ncols == 1, GrB_INVALID_VALUE, "vector must keep one column");
            vector_resize(o, nrows);
        }
    });
}
GrB_Info GrB_Matrix_free(GrB_Matrix *A) {
    if (!A) return GrB_NULL_POINTER;
    if (!*A) return GrB_SUCCESS;
    GB_Obj *o = OBJ(*A);
    if (o->magic != GB_MAGIC) return GrB_SUCCESS;
    GrB_Info info = gb_api(nullptr, [&] {
        gb_obj_free_storage(o);
        gb_free(o->d_nvals);
        gb_host_slot_release(o->pub);
        o->pub = nullptr;
    });
    o->magic = GB_FREED;
    delete o;
    *A = nullptr;
    return info;
}
GrB_Info GrB_Matrix_wait(GrB_Matrix A, GrB_WaitMode mode) {
    (void)mode;
    return gb_api(OBJ(A), [&] {
        gb_cw_materialize(gb_obj_check_raw(A));  // pending column-word value layers
        gb_sync();
    });
}
GrB_Info GrB_Matrix_error(const char **error, const GrB_Matrix A) {
    if (!error) return GrB_NULL_POINTER;
    static const char *empty = "";
    *error = (A && OBJ(A)->magic == GB_MAGIC) ? OBJ(A)->err.c_str() : empty;
    return GrB_SUCCESS;
}
GrB_Info GxB_Matrix_type(GrB_Type *type, const GrB_Matrix A) {
    if (!type) return GrB_NULL_POINTER;
    return gb_api(OBJ(A), [&] { *type = gb_obj_check_raw(A)->type; });
}
GrB_Info GrB_Matrix_removeElement(GrB_Matrix A, GrB_Index i, GrB_Index j) {
    return gb_api(OBJ(A), [&] {
        GB_Obj *o = gb_obj_check(A);
        if (o->kind != GB_KIND_MATRIX) {
            GB_REQUIRE(j == 0, GrB_INVALID_INDEX, "index out of range");
            GB_REQUIRE(i < (GrB_Index)o->nrows, GrB_INVALID_INDEX, "index out of range");
            hipLaunchKernelGGL(k_vec_clear, dim3(1), dim3(1), 0, gb_stream(), (unsigned long long *)o->bits,
                               (int64_t)i, (unsigned long long *)o->d_nvals);
            GB_LAUNCH_CHECK();
            o->nvals_valid = false;
            o->hint_valid = false;
            return;
        }
        matrix_remove_element(o, i, j);
    });
}
GrB_Info GrB_Matrix_exportSize(GrB_Index *Ap_len, GrB_Index *Ai_len, GrB_Index *Ax_len, GrB_Format format,
                               GrB_Matrix A) {
    if (!Ap_len || !Ai_len || !Ax_len) return GrB_NULL_POINTER;
    return gb_api(OBJ(A), [&] {
        GB_Obj *o = gb_obj_check(A);
        int64_t nz = gb_nvals(o);
        int64_t ncols = o->kind == GB_KIND_MATRIX ? o->ncols : 1;
        *Ap_len = format == GrB_CSR_FORMAT ? o->nrows + 1 : format == GrB_CSC_FORMAT ? ncols + 1 : nz;
        *Ai_len = nz;
        *Ax_len = nz;
    });
}
GrB_Info GrB_Matrix_exportHint(GrB_Format *format, GrB_Matrix A) {
    if (!format) return GrB_NULL_POINTER;
    *format = GrB_CSR_FORMAT;
    (void)A;
    return GrB_SUCCESS;
}

// ---------------- Vector
GrB_Info GrB_Vector_new(GrB_Vector *v, GrB_Type type, GrB_Index n) {
    if (!v) return GrB_NULL_POINTER;
    return gb_api(nullptr, [&] { *v = (GrB_Vector)gb_new_object(GB_KIND_VECTOR, type, n, 1); });
}
GrB_Info GrB_Vector_dup(GrB_Vector *w, const GrB_Vector u) {
    if (!w) return GrB_NULL_POINTER;
    return gb_api(nullptr, [&] { *w = (GrB_Vector)dup_object(gb_obj_check(u)); });
}
GrB_Info GrB_Vector_clear(GrB_Vector v) { return GrB_Matrix_clear((GrB_Matrix)v); }
GrB_Info GrB_Vector_size(GrB_Index *n, const GrB_Vector v) { return GrB_Matrix_nrows(n, (GrB_Matrix)v); }
GrB_Info GrB_Vector_nvals(GrB_Index *n, const GrB_Vector v) { return GrB_Matrix_nvals(n, (GrB_Matrix)v); }
GrB_Info GrB_Vector_resize(GrB_Vector v, GrB_Index n) {
    return gb_api(OBJ(v), [&] {
        GB_Obj *o = gb_obj_check(v);
        if (o->kind == GB_KIND_MATRIX) matrix_resize(o, n, 1);
        else vector_resize(o, n);
    });
}
GrB_Info GrB_Vector_free(GrB_Vector *v) { return GrB_Matrix_free((GrB_Matrix *)v); }
GrB_Info GrB_Vector_wait(GrB_Vector v, GrB_WaitMode mode) { return GrB_Matrix_wait((GrB_Matrix)v, mode); }
GrB_Info GrB_Vector_error(const char **error, const GrB_Vector v) {
    return GrB_Matrix_error(error, (GrB_Matrix)v);
}
GrB_Info GxB_Vector_type(GrB_Type *type, const GrB_Vector v) { return GxB_Matrix_type(type, (GrB_Matrix)v); }
GrB_Info GrB_Vector_removeElement(GrB_Vector v, GrB_Index i) {
    return GrB_Matrix_removeElement((GrB_Matrix)v, i, 0);
}

// ---------------- Scalar (a 1-element vector)
GrB_Info GrB_Scalar_new(GrB_Scalar *s, GrB_Type type) {
    if (!s) return GrB_NULL_POINTER;
    return gb_api(nullptr, [&] { *s = (GrB_Scalar)gb_new_object(GB_KIND_SCALAR, type, 1, 1); });
}
GrB_Info GrB_Scalar_dup(GrB_Scalar *s, const GrB_Scalar t) {
    if (!s) return GrB_NULL_POINTER;
    return gb_api(nullptr, [&] { *s = (GrB_Scalar)dup_object(gb_obj_check(t)); });
}
GrB_Info GrB_Scalar_clear(GrB_Scalar s) { return GrB_Matrix_clear((GrB_Matrix)s); }
GrB_Info GrB_Scalar_nvals(GrB_Index *n, const GrB_Scalar s) { return GrB_Matrix_nvals(n, (GrB_Matrix)s); }
GrB_Info GrB_Scalar_free(GrB_Scalar *s) { return GrB_Matrix_free((GrB_Matrix *)s); }
GrB_Info GrB_Scalar_wait(GrB_Scalar s, GrB_WaitMode mode) { return GrB_Matrix_wait((GrB_Matrix)s, mode); }
GrB_Info GrB_Scalar_error(const char **error, const GrB_Scalar s) {
    return GrB_Matrix_error(error, (GrB_Matrix)s);
}

// ---------------- typed entry points
#define GB_DEFINE_TYPED(T, ctype)                                                                              \
    GrB_Info GrB_Matrix_build_##T(GrB_Matrix C, const GrB_Index *I, const GrB_Index *J, const ctype *X,      \
                                  GrB_Index nvals, const GrB_BinaryOp dup) {                                 \
        return gb_api(OBJ(C), [&] {                                                                          \
            gb_build(gb_obj_check(C), I, J, X, GBAMD_T_##T, false, (int64_t)nvals, dup);                 \
        });                                                                                                  \
    }                                                                                                        \
    GrB_Info GxB_Matrix_build_Scalar_##T(GrB_Matrix C, const GrB_Index *I, const GrB_Index *J, ctype x,     \
                                         GrB_Index nvals) {                                                  \
        return gb_api(OBJ(C), [&] {                                                                          \
            gb_build(gb_obj_check(C), I, J, &x, GBAMD_T_##T, true, (int64_t)nvals, GrB_FIRST_##T);       \
        });                                                                                                  \
    }                                                                                                        \
    GrB_Info GrB_Matrix_setElement_##T(GrB_Matrix C, ctype x, GrB_Index i, GrB_Index j) {                    \
        return gb_api(OBJ(C), [&] {                                                                          \
            GB_Obj *o = gb_obj_check(C);                                                                     \
            with_type(o->type->code, [&](auto z) {                                                           \
                using S = decltype(z);                                                                       \
                if (o->kind == GB_KIND_MATRIX) matrix_set_element<S>(o, gb_cast<S, ctype>(x), i, j);         \
                else {                                                                                       \
                    GB_REQUIRE(j == 0, GrB_INVALID_INDEX, "index out of range");                             \
                    vector_set_element<S>(o, gb_cast<S, ctype>(x), i);                                       \
                }                                                                                            \
            });                                                                                              \
        });                                                                                                  \
    }                                                                                                        \
    GrB_Info GrB_Matrix_extractElement_##T(ctype *x, const GrB_Matrix A, GrB_Index i, GrB_Index j) {         \
        GrB_Info r = GrB_SUCCESS;                                                                            \
        GrB_Info e = gb_api(OBJ(A), [&] {                                                                    \
            GB_Obj *o = gb_obj_check(A);                                                                     \
            if (o->kind == GB_KIND_MATRIX) r = matrix_extract_element<ctype>(x, o, i, j);                    \
            else {                                                                                           \
                GB_REQUIRE(j == 0, GrB_INVALID_INDEX, "index out of range");                                 \
                r = vector_extract_element<ctype>(x, o, i);                                                  \
            }                                                                                                \
        });                                                                                                  \
        return e != GrB_SUCCESS ? e : r;                                                                     \
    }                                                                                                        \
    GrB_Info GrB_Matrix_extractTuples_##T(GrB_Index *I, GrB_Index *J, ctype *X, GrB_Index *nvals,            \
                                          const GrB_Matrix A) {                                              \
        return gb_api(OBJ(A), [&] { gb_extract_tuples(gb_obj_check(A), I, J, X, GBAMD_T_##T, nvals); });       \
    }                                                                                                        \
    GrB_Info GrB_Matrix_import_##T(GrB_Matrix *A, GrB_Type type, GrB_Index nrows, GrB_Index ncols,           \
                                   const GrB_Index *Ap, const GrB_Index *Ai, const ctype *Ax,                \
                                   GrB_Index Ap_len, GrB_Index Ai_len, GrB_Index Ax_len, GrB_Format fmt) {   \
        if (!A) return GrB_NULL_POINTER;                                                                     \
        return gb_api(nullptr, [&] {                                                                         \
            GB_Obj *o = gb_new_object(GB_KIND_MATRIX, type, nrows, ncols);                                   \
            try {                                                                                            \
                if (fmt == GrB_CSR_FORMAT) {                                                                 \
                    GB_REQUIRE(Ap_len >= nrows + 1, GrB_INVALID_VALUE, "Ap too short");                      \
                    int64_t nz = (int64_t)Ap[nrows];                                                         \
                    GB_REQUIRE((int64_t)Ai_len >= nz && (int64_t)Ax_len >= nz, GrB_INVALID_VALUE, "short"); \
                    import_csr(o, Ap, Ai, Ax, GBAMD_T_##T, nrows, ncols, nz, false);                         \
                } else if (fmt == GrB_CSC_FORMAT) {                                                          \
                    GB_REQUIRE(Ap_len >= ncols + 1, GrB_INVALID_VALUE, "Ap too short");                      \
                    int64_t nz = (int64_t)Ap[ncols];                                                         \
                    GB_REQUIRE((int64_t)Ai_len >= nz && (int64_t)Ax_len >= nz, GrB_INVALID_VALUE, "short"); \
                    GB_Obj *t = gb_new_object(GB_KIND_MATRIX, type, ncols, nrows);                           \
                    import_csr(t, Ap, Ai, Ax, GBAMD_T_##T, ncols, nrows, nz, false);                         \
                    gb_csr_view cv;                                                                          \
                    gb_get_csc(cv, t);                                                                       \
                    int64_t *rp = gb_malloc_n<int64_t>(nrows + 1);                                           \
                    int32_t *ci = gb_malloc_n<int32_t>(nz);                                                  \
                    void *vx = gb_malloc(nz * type->size);                                                   \
                    gb_copy_d2d(rp, cv.rowptr, (nrows + 1) * sizeof(int64_t));                               \
                    gb_copy_d2d(ci, cv.colidx, nz * sizeof(int32_t));                                        \
                    gb_copy_d2d(vx, cv.vals, nz * type->size);                                               \
                    gb_install_csr(o, nrows, ncols, nz, rp, ci, vx, false);                                  \
                    GrB_Matrix tm = (GrB_Matrix)t;                                                           \
                    GrB_Matrix_free(&tm);                                                                    \
                } else {                                                                                     \
                    GB_REQUIRE(Ap_len == Ai_len && Ai_len <= Ax_len, GrB_INVALID_VALUE, "bad COO lengths");  \
                    gb_build(o, Ap, Ai, Ax, GBAMD_T_##T, false, (int64_t)Ai_len, nullptr);               \
                }                                                                                            \
            } catch (...) {                                                                                  \
                GrB_Matrix m = (GrB_Matrix)o;                                                                \
                GrB_Matrix_free(&m);                                                                         \
                throw;                                                                                       \
            }                                                                                                \
            *A = (GrB_Matrix)o;                                                                              \
        });                                                                                                  \
    }                                                                                                        \
    GrB_Info GrB_Matrix_export_##T(GrB_Index *Ap, GrB_Index *Ai, ctype *Ax, GrB_Index *Ap_len,               \
                                   GrB_Index *Ai_len, GrB_Index *Ax_len, GrB_Format fmt, GrB_Matrix A) {     \
        return gb_api(OBJ(A), [&] {                                                                          \
            export_matrix(gb_obj_check(A), Ap, Ai, Ax, GBAMD_T_##T, Ap_len, Ai_len, Ax_len, fmt);            \
        });                                                                                                  \
    }                                                                                                        \
    GrB_Info GrB_Vector_build_##T(GrB_Vector w, const GrB_Index *I, const ctype *X, GrB_Index nvals,         \
                                  const GrB_BinaryOp dup) {                                                  \
        return gb_api(OBJ(w), [&] {                                                                          \
            gb_build(gb_obj_check(w), I, nullptr, X, GBAMD_T_##T, false, (int64_t)nvals, dup);           \
        });                                                                                                  \
    }                                                                                                        \
    GrB_Info GxB_Vector_build_Scalar_##T(GrB_Vector w, const GrB_Index *I, ctype x, GrB_Index nvals) {      \
        return gb_api(OBJ(w), [&] {                                                                          \
            gb_build(gb_obj_check(w), I, nullptr, &x, GBAMD_T_##T, true, (int64_t)nvals, GrB_FIRST_##T); \
        });                                                                                                  \
    }                                                                                                        \
    GrB_Info GrB_Vector_setElement_##T(GrB_Vector w, ctype x, GrB_Index i) {                                 \
        GB_HPROF(9, "GrB_Vector_setElement");                                                                \
        return GrB_Matrix_setElement_##T((GrB_Matrix)w, x, i, 0);                                           \
    }                                                                                                        \
    GrB_Info GrB_Vector_extractElement_##T(ctype *x, const GrB_Vector v, GrB_Index i) {                      \
        return GrB_Matrix_extractElement_##T(x, (GrB_Matrix)v, i, 0);                                        \
    }                                                                                                        \
    GrB_Info GrB_Vector_extractTuples_##T(GrB_Index *I, ctype *X, GrB_Index *nvals, const GrB_Vector v) {    \
        return gb_api(OBJ(v), [&] { gb_extract_tuples(gb_obj_check(v), I, nullptr, X, GBAMD_T_##T, nvals); }); \
    }                                                                                                        \
    GrB_Info GrB_Scalar_setElement_##T(GrB_Scalar s, ctype x) {                                              \
        return GrB_Matrix_setElement_##T((GrB_Matrix)s, x, 0, 0);                                            \
    }                                                                                                        \
    GrB_Info GrB_Scalar_extractElement_##T(ctype *x, const GrB_Scalar s) {                                   \
        return GrB_Matrix_extractElement_##T(x, (GrB_Matrix)s, 0, 0);                                        \
    }

GB_FOR_EACH_TYPE(GB_DEFINE_TYPED)

// ---------------- device views
GrB_Info GxB_Matrix_device_view(GxB_DeviceView *view, const GrB_Matrix A) {
    if (!view) return GrB_NULL_POINTER;
    return gb_api(OBJ(A), [&] {
        GB_Obj *o = gb_obj_check(A);
        memset(view, 0, sizeof(*view));
        view->type_code = o->type->code;
        view->iso = o->iso;
        view->nrows = o->nrows;
        view->ncols = o->ncols;
        view->nvals = gb_nvals(o);
        if (o->kind == GB_KIND_MATRIX) {
            view->format = 0;
            view->rowptr = o->rowptr;
            view->colidx = o->colidx;
            view->values = o->vals;
        } else {
            view->format = 1;
            view->bitmap = o->bits;
            view->values = o->dense;
        }
    });
}
// CSR from device buffers (copied on the library stream): the receiving side of
// an all-gather of row panels (graphblas_amd.dist.gather_row_panels).  The caller
// guarantees a valid CSR (rowptr[0] == 0, sorted unique columns per row), the
// contract of GxB_Matrix_import_CSR with jumbled = false.
GrB_Info GxB_Matrix_import_device(GrB_Matrix *A, GrB_Type type, GrB_Index nrows, GrB_Index ncols,
                                  const void *rowptr, const void *colidx, const void *values,
                                  GrB_Index nvals, bool iso) {
    if (!A) return GrB_NULL_POINTER;
    return gb_api(nullptr, [&] {
        GB_REQUIRE(type && type->magic == GB_MAGIC, GrB_UNINITIALIZED_OBJECT, "type");
        GB_REQUIRE(rowptr && (nvals == 0 || colidx) && (nvals == 0 || values), GrB_NULL_POINTER,
                   "device buffers");
        GB_REQUIRE(ncols <= (GrB_Index)INT32_MAX, GrB_INVALID_VALUE, "ncols exceeds the 32-bit column index");
        GB_Obj *o = gb_new_object(GB_KIND_MATRIX, type, (int64_t)nrows, (int64_t)ncols);
        try {
            const size_t zs = gb_type_size(type->code);
            int64_t *rp = gb_malloc_n<int64_t>(nrows + 1);
            int32_t *ci = gb_malloc_n<int32_t>(nvals ? nvals : 1);
            const bool is = iso && nvals > 0;
            void *vx = gb_malloc((is ? 1 : (nvals ? nvals : 1)) * zs);
            gb_copy_d2d(rp, rowptr, (nrows + 1) * sizeof(int64_t));
            if (nvals) {
                gb_copy_d2d(ci, colidx, nvals * sizeof(int32_t));
                gb_copy_d2d(vx, values, (is ? 1 : nvals) * zs);
            }
            gb_install_csr(o, (int64_t)nrows, (int64_t)ncols, (int64_t)nvals, rp, ci, vx, is);
        } catch (...) {
            GrB_Matrix m = (GrB_Matrix)o;
            GrB_Matrix_free(&m);
            throw;
        }
        *A = (GrB_Matrix)o;
    });
}
GrB_Info GxB_Vector_device_view(GxB_DeviceView *view, const GrB_Vector v) {
    return GxB_Matrix_device_view(view, (GrB_Matrix)v);
}
// recount a vector whose bitmap was rewritten on the device; the count is
// published to the host mailbox, so a following nvals spins instead of copying
static void vec_recount_published(GB_Obj *o) {
    if (!o->pub) o->pub = gb_host_slot_alloc();
    const uint64_t seq = gb_next_pub_seq(o->pub);
    gb_bitmap_count_pub(o->bits, o->nrows, o->d_nvals, o->pub, seq);
    o->nvals_valid = false;
    o->hint_valid = false;
    o->pub_seq = seq;
    o->pub_epoch = gb_epoch();
}
void gb_vec_recount(GB_Obj *o) { vec_recount_published(o); }
GrB_Info GxB_Vector_device_touch(GrB_Vector v) {
    return gb_api(OBJ(v), [&] {
        GB_Obj *o = gb_obj_check(v);
        GB_REQUIRE(o->kind != GB_KIND_MATRIX, GrB_INVALID_OBJECT, "not a vector");
        vec_recount_published(o);
    });
}
// The ticket of v's last device publish and a wait on it (include/graphblas_amd.h): the count
// v had at that publish, read from the host mailbox even after later work that does not write
// v has been enqueued (nvals itself trusts a mailbox only while nothing was enqueued since).
GrB_Info GxB_Vector_publish_ticket(uint64_t *ticket, GrB_Vector v) {
    if (!ticket) return GrB_NULL_POINTER;
    return gb_api(OBJ(v), [&] {
        GB_Obj *o = gb_obj_check(v);
        GB_REQUIRE(o->kind != GB_KIND_MATRIX, GrB_INVALID_OBJECT, "not a vector");
        *ticket = o->pub ? o->pub_seq : 0;
    });
}
GrB_Info GxB_Vector_wait_ticket(GrB_Index *nvals, GrB_Vector v, uint64_t ticket) {
    if (!nvals) return GrB_NULL_POINTER;
    return gb_api(OBJ(v), [&] {
        GB_Obj *o = gb_obj_check(v);
        GB_REQUIRE(o->kind != GB_KIND_MATRIX, GrB_INVALID_OBJECT, "not a vector");
        GB_REQUIRE(o->pub && ticket, GrB_INVALID_VALUE, "no device publish to wait for");
        int64_t c = 0;
        if (!gb_host_slot_wait(o->pub, ticket, &c)) {
            // the stream drained without the word: a later publish of v overwrote it (superseded),
            // or the publishing launch failed or never ran (lost) -- told apart by the slot's
            // last issued number, which only the host writes
            GB_REQUIRE((uint64_t)o->pub->host_last == ticket, GrB_INVALID_VALUE,
                       "the publish was superseded by a later one of the same vector");
            gb_sync();  // a failed launch surfaces here as GrB_PANIC
            GB_REQUIRE(o->pub_seq == ticket, GrB_PANIC, "the publish never landed and v changed since");
            c = gb_nvals(o);  // nothing published since: v's count is the ticket's (synchronous read)
        }
        *nvals = (GrB_Index)c;
    });
}
GrB_Info GxB_Vector_bitmap_export(GrB_Vector v, void *dst, GrB_Index nwords) {
    return gb_api(OBJ(v), [&] {
        GB_Obj *o = gb_obj_check(v);
        GB_REQUIRE(o->kind != GB_KIND_MATRIX, GrB_INVALID_OBJECT, "not a vector");
        GB_REQUIRE((int64_t)nwords <= gb_words(o->nrows), GrB_INVALID_VALUE, "too many words");
        gb_copy_d2d(dst, o->bits, nwords * sizeof(uint64_t));
    });
}
GrB_Info GxB_Vector_bitmap_import(GrB_Vector v, const void *src, GrB_Index nwords) {
    return gb_api(OBJ(v), [&] {
        GB_Obj *o = gb_obj_check(v);
        GB_REQUIRE(o->kind != GB_KIND_MATRIX, GrB_INVALID_OBJECT, "not a vector");
        GB_REQUIRE((int64_t)nwords == gb_words(o->nrows), GrB_INVALID_VALUE, "word count mismatch");
        gb_copy_d2d(o->bits, src, nwords * sizeof(uint64_t));
        // every imported entry carries the value 1 (true): an iso vector
        size_t ts = o->type->size;
        char one[16] = {0};
        with_type(o->type->code, [&](auto z) {
            using T = decltype(z);
            T x = (T)1;
            memcpy(one, &x, sizeof(T));
        });
        if (!o->dense || !o->iso) {
            gb_free(o->dense);
            o->dense = gb_malloc(ts);
        }
        gb_copy_h2d(o->dense, one, ts);
        o->iso = true;
        vec_recount_published(o);
    });
}
// builds the cached transpose and, for integer values that fit fewer bytes, both orientations'
// narrow value copies (gb_view_narrow: a min/max pass and a blocking read) -- the one-time work a
// first masked GrB_mxm would otherwise do inside its call
GrB_Info GxB_Matrix_prepare_transpose(GrB_Matrix A) {
    return gb_api(OBJ(A), [&] {
        GB_Obj *o = gb_obj_check(A);
        if (o->kind != GB_KIND_MATRIX) return;
        gb_csr_view v, vt;
        gb_get_csr(v, o);
        gb_view_narrow(v, o, 0);
        gb_get_csc(vt, o);
        gb_view_narrow(vt, o, 1);
    });
}

}  // extern "C"
