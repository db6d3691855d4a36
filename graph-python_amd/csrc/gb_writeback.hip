// gb_writeback.hip -- C<M,replace> = C accum T, the GraphBLAS output rule
// (C API 2.0 §3.5; SURVEY.md §8(a) rules 2-5) applied after every operation.
//
// Most hot-path calls never launch a merge: with no accumulator and either no
// mask or a mask the kernel already applied under `replace` (BFS:
// q<!v.S, replace> = ...), T simply becomes C's new storage.  Otherwise a
// word-parallel (vectors) or entry-parallel (matrices) merge runs.
//
// Mixed-type accumulators (accum type != C type) are evaluated by casting C
// and T into the accumulator type, merging there and casting back; entries
// present only in C therefore make a round trip through the accumulator type.
#include "gb_dispatch.cuh"
#include "gb_internal.h"

#define WB_BLOCK 256
static inline unsigned wb_grid(int64_t n, unsigned cap = 16384) {
    int64_t g = (n + WB_BLOCK - 1) / WB_BLOCK;
    if (g < 1) g = 1;
    if (g > cap) g = cap;
    return (unsigned)g;
}
#define WB_STRIDE(i, n) \
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < (n); i += (int64_t)gridDim.x * blockDim.x)

// ================================================================== masks
template <class T>
__global__ void k_vmask_values(const uint64_t *__restrict__ bits, const T *__restrict__ vals, bool iso, int64_t n,
                               uint64_t *__restrict__ out) {
    WB_STRIDE(w, (n + 63) >> 6) {
        uint64_t word = bits[w], r = 0;
        while (word) {
            int b = __ffsll((unsigned long long)word) - 1;
            word &= word - 1;
            int64_t i = (w << 6) + b;
            if (gb_cast<bool, T>(iso ? vals[0] : vals[i])) r |= 1ULL << b;
        }
        out[w] = r;
    }
}

void gb_make_vmask(gb_vmask &m, GB_Obj *M, const gb_desc &d, int64_t n, bool allow_iso_value) {
    m.comp = d.comp;
    if (!M) {
        if (d.comp) {  // ~NULL: nothing is selected
            uint64_t *z = m.own.get<uint64_t>(gb_words(n));
            gb_memset(z, 0, gb_words(n) * sizeof(uint64_t));
            m.bits = z;
            m.comp = false;
        }
        return;
    }
    GB_REQUIRE(M->nrows == n && (M->kind != GB_KIND_MATRIX || M->ncols == 1), GrB_DIMENSION_MISMATCH,
               "mask dimensions do not match the output");
    gb_bitmap_view *bv = new gb_bitmap_view();  // owned by m.own through a small holder below
    gb_get_bitmap(*bv, M);
    if (d.structure) {
        // copy only when the view owns temporaries (matrix-typed mask)
        if (bv->own.n) {
            uint64_t *c = m.own.get<uint64_t>(gb_words(n));
            gb_copy_d2d(c, bv->bits, gb_words(n) * sizeof(uint64_t));
            m.bits = c;
        } else {
            m.bits = bv->bits;
            m.count = M->d_nvals;  // kept current by every writer of M
        }
    } else if (allow_iso_value && bv->iso && !bv->own.n) {
        m.bits = bv->bits;
        m.iso_val = bv->vals;
        m.iso_code = bv->tcode;
    } else {
        uint64_t *c = m.own.get<uint64_t>(gb_words(n));
        gb_with_type(bv->tcode, [&](auto z) {
            using T = decltype(z);
            hipLaunchKernelGGL(k_vmask_values<T>, dim3(wb_grid(gb_words(n))), dim3(WB_BLOCK), 0, gb_stream(), bv->bits,
                               (const T *)bv->vals, bv->iso, n, c);
        });
        GB_LAUNCH_CHECK();
        m.bits = c;
    }
    delete bv;  // stream-ordered frees of its temporaries happen after the copies above
}

template <class T>
__global__ void k_mmask_count(const int64_t *__restrict__ rp, const T *__restrict__ vals, bool iso, int64_t nrows,
                              int64_t *__restrict__ cnt) {
    WB_STRIDE(i, nrows) {
        int64_t c = 0;
        for (int64_t p = rp[i]; p < rp[i + 1]; p++) c += gb_cast<bool, T>(iso ? vals[0] : vals[p]);
        cnt[i] = c;
    }
}
template <class T>
__global__ void k_mmask_fill(const int64_t *__restrict__ rp, const int32_t *__restrict__ ci, const T *__restrict__ vals,
                             bool iso, int64_t nrows, const int64_t *__restrict__ rp2, int32_t *__restrict__ ci2) {
    WB_STRIDE(i, nrows) {
        int64_t o = rp2[i];
        for (int64_t p = rp[i]; p < rp[i + 1]; p++)
            if (gb_cast<bool, T>(iso ? vals[0] : vals[p])) ci2[o++] = ci[p];
    }
}

void gb_make_mmask(gb_mmask &m, GB_Obj *M, const gb_desc &d, int64_t nrows, int64_t ncols) {
    m.comp = d.comp;
    if (!M) {
        if (d.comp) {  // ~NULL: an empty structure, not complemented = nothing selected
            m.present = true;
            m.comp = false;
            int64_t *rp = m.own.get<int64_t>(nrows + 1);
            gb_memset(rp, 0, (nrows + 1) * sizeof(int64_t));
            m.rowptr = rp;
            m.colidx = m.own.get<int32_t>(1);
            m.nvals = 0;
        }
        return;
    }
    int64_t mcols = M->kind == GB_KIND_MATRIX ? M->ncols : 1;
    GB_REQUIRE(M->nrows == nrows && mcols == ncols, GrB_DIMENSION_MISMATCH, "mask dimensions do not match the output");
    m.present = true;
    gb_get_csr(m.view, M);
    if (d.structure) {
        m.rowptr = m.view.rowptr;
        m.colidx = m.view.colidx;
        m.nvals = m.view.nvals;
        if (M->kind == GB_KIND_MATRIX) m.obj = M;
        return;
    }
    int64_t *cnt = m.own.get<int64_t>(nrows + 1);
    int64_t *rp2 = m.own.get<int64_t>(nrows + 1);
    gb_memset(cnt, 0, (nrows + 1) * sizeof(int64_t));
    gb_with_type(m.view.tcode, [&](auto z) {
        using T = decltype(z);
        if (nrows)
            hipLaunchKernelGGL(k_mmask_count<T>, dim3(wb_grid(nrows)), dim3(WB_BLOCK), 0, gb_stream(), m.view.rowptr,
                               (const T *)m.view.vals, m.view.iso, nrows, cnt);
    });
    GB_LAUNCH_CHECK();
    gb_exclusive_scan_i64(cnt, rp2, nrows);
    int64_t nz = gb_read_i64(rp2 + nrows);
    int32_t *ci2 = m.own.get<int32_t>(nz);
    gb_with_type(m.view.tcode, [&](auto z) {
        using T = decltype(z);
        if (nrows)
            hipLaunchKernelGGL(k_mmask_fill<T>, dim3(wb_grid(nrows)), dim3(WB_BLOCK), 0, gb_stream(), m.view.rowptr,
                               m.view.colidx, (const T *)m.view.vals, m.view.iso, nrows, rp2, ci2);
    });
    GB_LAUNCH_CHECK();
    m.rowptr = rp2;
    m.colidx = ci2;
    m.nvals = nz;
}

// ================================================================== vectors
template <class CT>
__global__ __launch_bounds__(WB_BLOCK) void k_vec_merge(
    int64_t n, const uint64_t *__restrict__ cbits, const CT *__restrict__ cvals, bool c_iso,
    const uint64_t *__restrict__ tbits, const CT *__restrict__ tvals, bool t_iso, const uint64_t *__restrict__ mbits,
    bool mcomp, bool replace, int accum, uint64_t *__restrict__ obits, CT *__restrict__ ovals,
    unsigned long long *__restrict__ count, unsigned long long *__restrict__ gst) {
    unsigned long long mine = 0;
    // 64 consecutive elements per wave -> one output word per wave
    for (int64_t base = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) & ~63LL; base < n;
         base += (int64_t)gridDim.x * blockDim.x) {
        int64_t i = base + (threadIdx.x & 63);
        bool inr = i < n;
        bool c = inr && gb_bit(cbits, i);
        bool t = inr && gb_bit(tbits, i);
        bool m = inr && (mbits ? (gb_bit(mbits, i) != mcomp) : !mcomp);
        bool have = false;
        CT v = CT();
        if (m) {
            if (accum >= 0 && c && t) {
                v = gb_binop<CT>(accum, cvals[c_iso ? 0 : i], tvals[t_iso ? 0 : i]);
                have = true;
            } else if (t) {
                v = tvals[t_iso ? 0 : i];
                have = true;
            } else if (accum >= 0 && c) {
                v = cvals[c_iso ? 0 : i];
                have = true;
            }
        } else if (!replace && c) {
            v = cvals[c_iso ? 0 : i];
            have = true;
        }
        if (have) ovals[i] = v;
        unsigned long long word = __ballot(have);
        if ((threadIdx.x & 63) == 0) {
            obits[base >> 6] = word;
            mine += __popcll(word);
        }
    }
    gb_grid_add((long long)mine, count, gst);
}

static void cast_vec_result(gb_vec_result &T, int code) {
    if (T.tcode == code) return;
    int64_t nv = T.iso ? 1 : T.n;
    void *d = gb_malloc(nv * gb_type_size(code));
    gb_cast_array(d, code, T.dense, T.tcode, nv);
    gb_free(T.dense);
    T.dense = d;
    T.tcode = code;
}

static void free_vec_result(gb_vec_result &T) {
    gb_free(T.bits);
    gb_free(T.dense);
    gb_free(T.d_nvals);
    T.bits = nullptr;
    T.dense = nullptr;
    T.d_nvals = nullptr;
}

bool gb_writeback_vector(GB_Obj *C, gb_vec_result &T, GB_Obj *M, const gb_desc &d, GrB_BinaryOp accum,
                         bool t_within_mask) {
    const int ct = C->type->code;
    const int64_t n = T.n;
    GB_REQUIRE(C->nrows == n, GrB_DIMENSION_MISMATCH, "output size mismatch");
    bool no_mask = (M == nullptr && !d.comp);
    if (!accum && (no_mask || (t_within_mask && d.replace))) {
        cast_vec_result(T, ct);
        gb_install_bitmap(C, n, T.bits, T.dense, T.iso, T.d_nvals);
        T.bits = nullptr;
        T.dense = nullptr;
        T.d_nvals = nullptr;
        return true;
    }
    // general merge
    int wcode = ct;
    if (accum) {
        GB_REQUIRE(accum->magic == GB_MAGIC, GrB_UNINITIALIZED_OBJECT, "invalid accum");
        GB_REQUIRE(accum->xtype != nullptr, GrB_DOMAIN_MISMATCH, "positional accumulator");
        wcode = accum->xtype->code;
    }
    gb_vmask mask;
    gb_make_vmask(mask, M, d, n);
    gb_bitmap_view cv;
    gb_get_bitmap(cv, C);
    gb_scratch s;
    const void *cvals = cv.vals;
    bool c_iso = cv.iso;
    if (wcode != ct) {
        cvals = gb_bitmap_vals_as(cv, wcode, s);
    }
    cast_vec_result(T, wcode);
    uint64_t *obits = gb_malloc_n<uint64_t>(gb_words(n));
    void *ovals = gb_malloc(n * gb_type_size(wcode));
    int64_t *cnt = gb_malloc_n<int64_t>(1);
    gb_memset(cnt, 0, sizeof(int64_t));
    if (n) {
        gb_with_type(wcode, [&](auto z) {
            using W = decltype(z);
            hipLaunchKernelGGL(k_vec_merge<W>, dim3(wb_grid(n, 1024)), dim3(WB_BLOCK), 0, gb_stream(), n, cv.bits,
                               (const W *)cvals, c_iso, T.bits, (const W *)T.dense, T.iso, mask.bits, mask.comp,
                               d.replace, accum ? accum->opcode : -1, obits, (W *)ovals,
                               (unsigned long long *)cnt, gb_device_state());
        });
        GB_LAUNCH_CHECK();
    }
    free_vec_result(T);
    if (wcode != ct) {
        void *o2 = gb_malloc(n * gb_type_size(ct));
        gb_cast_array(o2, ct, ovals, wcode, n);
        gb_free(ovals);
        ovals = o2;
    }
    gb_install_bitmap(C, n, obits, ovals, false, cnt);
    return false;
}

// ================================================================== matrices
// Entry-parallel merge of C and T under the mask (one thread per stored entry,
// so R-MAT hub rows with 10^4-10^5 entries do not serialise a thread):
//   1. flag every entry of C and of T that survives (k_merge_flag_c / _t);
//   2. exclusive scans of both (byte) flag arrays into int64 offsets (sc, st);
//   3. row r of the output starts at sc[crp[r]] + st[trp[r]];
//   4. a surviving C entry (r, j) lands at sc[e] + st[lower_bound of j in T's row r],
//      a surviving T entry at st[e] + sc[lower_bound of j in C's row r]
//      (both rows sorted, so this is their merge order).
// A C entry survives where the mask is false (unless replace) or where it is true,
// accum is set and T has no entry; a T entry survives where the mask is true and
// carries accum(C, T) when C has the entry too.
__device__ __forceinline__ int64_t wb_row_of(const int64_t *__restrict__ rp, int64_t nrows, int64_t e) {
    int64_t lo = 0, hi = nrows;  // last r with rp[r] <= e
    while (hi - lo > 1) {
        int64_t mid = (lo + hi) >> 1;
        if (rp[mid] <= e) lo = mid;
        else hi = mid;
    }
    return lo;
}
__device__ __forceinline__ int64_t wb_lower_bound(const int32_t *__restrict__ ci, int64_t lo, int64_t hi, int32_t j) {
    while (lo < hi) {
        int64_t mid = (lo + hi) >> 1;
        if (ci[mid] < j) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}
__device__ __forceinline__ bool wb_mask_at(const int64_t *__restrict__ mrp, const int32_t *__restrict__ mci,
                                          bool has_mask, bool mcomp, int64_t r, int32_t j) {
    if (!has_mask) return !mcomp;
    int64_t a = mrp[r], b = mrp[r + 1];
    int64_t p = wb_lower_bound(mci, a, b, j);
    return (p < b && mci[p] == j) != mcomp;
}

__global__ __launch_bounds__(WB_BLOCK) void k_merge_flag_c(
    int64_t nrows, int64_t cnz, const int64_t *__restrict__ crp, const int32_t *__restrict__ cci,
    const int64_t *__restrict__ trp, const int32_t *__restrict__ tci, const int64_t *__restrict__ mrp,
    const int32_t *__restrict__ mci, bool has_mask, bool mcomp, bool replace, bool accum,
    uint8_t *__restrict__ flag) {
    WB_STRIDE(e, cnz) {
        const int64_t r = wb_row_of(crp, nrows, e);
        const int32_t j = cci[e];
        bool keep;
        if (wb_mask_at(mrp, mci, has_mask, mcomp, r, j)) {
            if (accum) {
                int64_t a = trp[r], b = trp[r + 1];
                int64_t p = wb_lower_bound(tci, a, b, j);
                keep = !(p < b && tci[p] == j);
            } else {
                keep = false;
            }
        } else {
            keep = !replace;
        }
        flag[e] = keep;
    }
}

__global__ __launch_bounds__(WB_BLOCK) void k_merge_flag_t(
    int64_t nrows, int64_t tnz, const int64_t *__restrict__ trp, const int32_t *__restrict__ tci,
    const int64_t *__restrict__ mrp, const int32_t *__restrict__ mci, bool has_mask, bool mcomp, bool within_mask,
    uint8_t *__restrict__ flag) {
    WB_STRIDE(e, tnz) {
        bool keep = true;
        if (!within_mask) {
            const int64_t r = wb_row_of(trp, nrows, e);
            keep = wb_mask_at(mrp, mci, has_mask, mcomp, r, tci[e]);
        }
        flag[e] = keep;
    }
}

__global__ void k_merge_rowptr(int64_t nrows, const int64_t *__restrict__ crp, const int64_t *__restrict__ trp,
                               const int64_t *__restrict__ sc, const int64_t *__restrict__ st,
                               int64_t *__restrict__ orp) {
    WB_STRIDE(r, nrows + 1) orp[r] = sc[crp[r]] + st[trp[r]];
}

template <class CT>
__global__ __launch_bounds__(WB_BLOCK) void k_merge_place_c(
    int64_t nrows, int64_t cnz, const int64_t *__restrict__ crp, const int32_t *__restrict__ cci,
    const CT *__restrict__ cvx, bool c_iso, const int64_t *__restrict__ trp, const int32_t *__restrict__ tci,
    const int64_t *__restrict__ sc, const int64_t *__restrict__ st, int32_t *__restrict__ oci,
    CT *__restrict__ ovx) {
    WB_STRIDE(e, cnz) {
        if (sc[e + 1] == sc[e]) continue;
        const int64_t r = wb_row_of(crp, nrows, e);
        const int32_t j = cci[e];
        const int64_t p = wb_lower_bound(tci, trp[r], trp[r + 1], j);
        const int64_t o = sc[e] + st[p];
        oci[o] = j;
        ovx[o] = cvx[c_iso ? 0 : e];
    }
}

template <class CT>
__global__ __launch_bounds__(WB_BLOCK) void k_merge_place_t(
    int64_t nrows, int64_t tnz, const int64_t *__restrict__ trp, const int32_t *__restrict__ tci,
    const CT *__restrict__ tvx, bool t_iso, const int64_t *__restrict__ crp, const int32_t *__restrict__ cci,
    const CT *__restrict__ cvx, bool c_iso, int accum, const int64_t *__restrict__ sc,
    const int64_t *__restrict__ st, int32_t *__restrict__ oci, CT *__restrict__ ovx) {
    WB_STRIDE(e, tnz) {
        if (st[e + 1] == st[e]) continue;
        const int64_t r = wb_row_of(trp, nrows, e);
        const int32_t j = tci[e];
        const int64_t a = crp[r], b = crp[r + 1];
        const int64_t p = wb_lower_bound(cci, a, b, j);
        CT v = tvx[t_iso ? 0 : e];
        if (accum >= 0 && p < b && cci[p] == j) v = gb_binop<CT>(accum, cvx[c_iso ? 0 : p], v);
        const int64_t o = st[e] + sc[p];
        oci[o] = j;
        ovx[o] = v;
    }
}

static void cast_mat_result(gb_mat_result &T, int code) {
    if (T.tcode == code) return;
    int64_t nv = T.iso ? 1 : T.nvals;
    void *d = gb_malloc(nv * gb_type_size(code));
    gb_cast_array(d, code, T.vals, T.tcode, nv);
    gb_free(T.vals);
    T.vals = d;
    T.tcode = code;
}

void gb_writeback_matrix(GB_Obj *C, gb_mat_result &T, GB_Obj *M, const gb_desc &d, GrB_BinaryOp accum) {
    const int ct = C->type->code;
    const int64_t nrows = T.nrows, ncols = T.ncols;
    int64_t cncols = C->kind == GB_KIND_MATRIX ? C->ncols : 1;
    GB_REQUIRE(C->nrows == nrows && cncols == ncols, GrB_DIMENSION_MISMATCH, "output dimensions mismatch");
    bool no_mask = (M == nullptr && !d.comp);
    int64_t cnv = gb_nvals(C);
    bool fast = false;
    if (no_mask && (!accum || cnv == 0)) fast = true;                  // C = T  (or C empty: C = T)
    if (T.within_mask && !d.comp && M && (d.replace || cnv == 0) && (!accum || cnv == 0)) fast = true;
    if (fast) {
        cast_mat_result(T, ct);
        gb_install_csr(C, nrows, ncols, T.nvals, T.rowptr, T.colidx, T.vals, T.iso);
        T.rowptr = nullptr;
        T.colidx = nullptr;
        T.vals = nullptr;
        return;
    }
    int wcode = ct;
    if (accum) {
        GB_REQUIRE(accum->magic == GB_MAGIC, GrB_UNINITIALIZED_OBJECT, "invalid accum");
        GB_REQUIRE(accum->xtype != nullptr, GrB_DOMAIN_MISMATCH, "positional accumulator");
        wcode = accum->xtype->code;
    }
    gb_mmask mask;
    gb_make_mmask(mask, M, d, nrows, ncols);
    gb_csr_view cv;
    gb_get_csr(cv, C);
    gb_scratch s;
    const void *cvals = (wcode != ct) ? gb_view_vals_as(cv, wcode, s) : cv.vals;
    cast_mat_result(T, wcode);
    const bool has_mask = mask.present;
    const int64_t cnz = cv.nvals, tnz = T.nvals;
    // 0/1 byte flags (scratch: 1 + 8 bytes per entry; the scans run in < 2^31-item chunks)
    uint8_t *fc = s.get<uint8_t>(std::max<int64_t>(cnz, 1));
    uint8_t *ft = s.get<uint8_t>(std::max<int64_t>(tnz, 1));
    int64_t *sc = s.get<int64_t>(cnz + 1);
    int64_t *st = s.get<int64_t>(tnz + 1);
    if (cnz)
        hipLaunchKernelGGL(k_merge_flag_c, dim3(wb_grid(cnz)), dim3(WB_BLOCK), 0, gb_stream(), nrows, cnz, cv.rowptr,
                           cv.colidx, T.rowptr, T.colidx, mask.rowptr, mask.colidx, has_mask, mask.comp, d.replace,
                           accum != nullptr, fc);
    if (tnz)
        hipLaunchKernelGGL(k_merge_flag_t, dim3(wb_grid(tnz)), dim3(WB_BLOCK), 0, gb_stream(), nrows, tnz, T.rowptr,
                           T.colidx, mask.rowptr, mask.colidx, has_mask, mask.comp,
                           T.within_mask && has_mask && !mask.comp, ft);
    GB_LAUNCH_CHECK();
    gb_exclusive_scan_u8(fc, sc, cnz);
    gb_exclusive_scan_u8(ft, st, tnz);
    int64_t *orp = gb_malloc_n<int64_t>(nrows + 1);
    hipLaunchKernelGGL(k_merge_rowptr, dim3(wb_grid(nrows + 1)), dim3(WB_BLOCK), 0, gb_stream(), nrows, cv.rowptr,
                       T.rowptr, sc, st, orp);
    GB_LAUNCH_CHECK();
    int64_t nz = gb_read_i64(orp + nrows);
    int32_t *oci = gb_malloc_n<int32_t>(std::max<int64_t>(nz, 1));
    void *ovx = gb_malloc(std::max<int64_t>(nz, 1) * gb_type_size(wcode));
    gb_with_type(wcode, [&](auto z) {
        using W = decltype(z);
        if (cnz)
            hipLaunchKernelGGL((k_merge_place_c<W>), dim3(wb_grid(cnz)), dim3(WB_BLOCK), 0, gb_stream(), nrows, cnz,
                               cv.rowptr, cv.colidx, (const W *)cvals, cv.iso, T.rowptr, T.colidx, sc, st, oci,
                               (W *)ovx);
        if (tnz)
            hipLaunchKernelGGL((k_merge_place_t<W>), dim3(wb_grid(tnz)), dim3(WB_BLOCK), 0, gb_stream(), nrows, tnz,
                               T.rowptr, T.colidx, (const W *)T.vals, T.iso, cv.rowptr, cv.colidx, (const W *)cvals,
                               cv.iso, accum ? accum->opcode : -1, sc, st, oci, (W *)ovx);
    });
    GB_LAUNCH_CHECK();
    gb_free(T.rowptr);
    gb_free(T.colidx);
    gb_free(T.vals);
    T.rowptr = nullptr;
    T.colidx = nullptr;
    T.vals = nullptr;
    if (wcode != ct) {
        void *o2 = gb_malloc(nz * gb_type_size(ct));
        gb_cast_array(o2, ct, ovx, wcode, nz);
        gb_free(ovx);
        ovx = o2;
    }
    gb_install_csr(C, nrows, ncols, nz, orp, oci, ovx, false);
}
