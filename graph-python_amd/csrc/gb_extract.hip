// gb_extract.hip -- index lists and the extract family of the C ABI:
//   GrB_Matrix_extract  C<M> = accum(C, A'(I, J))   (reference core/matrix.py:2868, cfunc "GrB_Matrix_extract")
//   GrB_Col_extract     w<m> = accum(w, A'(I, j))   (reference core/matrix.py:2903,2917, cfunc "GrB_Col_extract")
//   GrB_Vector_extract  w<m> = accum(w, u(I))       (reference core/vector.py:1026, cfunc "GrB_Vector_extract")
// and the SuiteSparse index-list encodings python-graphblas passes for slices
// (reference core/slice.py:10-49): ni == GxB_RANGE with I = [begin, end] (inclusive),
// ni == GxB_STRIDE with I = [begin, end, inc], ni == GxB_BACKWARDS with I = [begin, end, dec].
//
// Device work: the submatrix is produced row-parallel (a wave per output row); columns
// are mapped through an inverse of J (count per source column, prefix sum, positions),
// so duplicated or unsorted J are handled; output rows come out sorted by a radix sort of
// (row, position) keys unless J is all columns (then they are sorted already).
#include <algorithm>
#include <vector>

#include "gb_dispatch.cuh"
#include "gb_internal.h"

#define EXT_BLOCK 256

void gb_expand_indices(gb_index_list &L, const GrB_Index *I, GrB_Index ni, int64_t n) {
    L.idx.clear();
    L.all = false;
    if (I == GrB_ALL) {
        L.all = true;
        L.n = n;
        return;
    }
    GB_REQUIRE(I != nullptr, GrB_NULL_POINTER, "index list is NULL");
    auto check = [&](int64_t i) {
        GB_REQUIRE(i >= 0 && i < n, GrB_INDEX_OUT_OF_BOUNDS, "index out of bounds");
    };
    if (ni == (GrB_Index)GxB_RANGE || ni == (GrB_Index)GxB_STRIDE) {
        int64_t b = (int64_t)I[GxB_BEGIN], e = (int64_t)I[GxB_END];
        int64_t inc = ni == (GrB_Index)GxB_STRIDE ? (int64_t)I[GxB_INC] : 1;
        GB_REQUIRE(inc > 0, GrB_INVALID_VALUE, "stride must be positive");
        for (int64_t i = b; i <= e; i += inc) {
            check(i);
            L.idx.push_back(i);
        }
    } else if (ni == (GrB_Index)GxB_BACKWARDS) {
        int64_t b = (int64_t)I[GxB_BEGIN], e = (int64_t)I[GxB_END], dec = (int64_t)I[GxB_INC];
        GB_REQUIRE(dec > 0, GrB_INVALID_VALUE, "stride must be positive");
        for (int64_t i = b; i >= e; i -= dec) {
            check(i);
            L.idx.push_back(i);
        }
    } else {
        GB_REQUIRE(ni < (GrB_Index)(1LL << 40), GrB_INVALID_VALUE, "index list too long");
        L.idx.resize(ni);
        for (GrB_Index q = 0; q < ni; q++) {
            check((int64_t)I[q]);
            L.idx[q] = (int64_t)I[q];
        }
    }
    L.n = (int64_t)L.idx.size();
}

// ------------------------------------------------------------------ kernels
static inline unsigned ext_grid(int64_t items, int64_t per_block, unsigned cap = 65535) {
    int64_t g = (items + per_block - 1) / per_block;
    return (unsigned)std::max<int64_t>(1, std::min<int64_t>(g, cap));
}

// jcnt[c] = number of positions p with J[p] == c
__global__ void k_ext_jcount(int64_t nj, const int64_t *__restrict__ J, int32_t *__restrict__ jcnt) {
    for (int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; p < nj; p += (int64_t)gridDim.x * blockDim.x)
        atomicAdd(&jcnt[J[p]], 1);
}
// jpos[jptr[c] ...] = the positions p with J[p] == c (any order: the output sort fixes it)
__global__ void k_ext_jfill(int64_t nj, const int64_t *__restrict__ J, int64_t *__restrict__ cursor,
                            int32_t *__restrict__ jpos) {
    for (int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; p < nj; p += (int64_t)gridDim.x * blockDim.x)
        jpos[atomicAdd((unsigned long long *)&cursor[J[p]], 1ULL)] = (int32_t)p;
}

// A wave per output row r (source row I[r], or r): FILL == false counts the row's outputs
// into cnt[r]; FILL == true writes key = (r << 32 | output column) and the source entry
// position for each output at outp[r] + rank.
template <bool JALL, bool FILL>
__global__ __launch_bounds__(EXT_BLOCK) void k_ext_rows(int64_t ni, const int64_t *__restrict__ I,
                                                        const int64_t *__restrict__ rp, const int32_t *__restrict__ ci,
                                                        const int64_t *__restrict__ jptr,
                                                        const int32_t *__restrict__ jpos, int64_t *__restrict__ cnt,
                                                        const int64_t *__restrict__ outp, uint64_t *__restrict__ okey,
                                                        int64_t *__restrict__ osrc) {
    const int lane = threadIdx.x & 63;
    const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
    const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
    for (int64_t r = wave; r < ni; r += nwaves) {
        const int64_t src = I ? I[r] : r;
        const int64_t e0 = rp[src], e1 = rp[src + 1];
        int64_t run = FILL ? outp[r] : 0;  // wave-uniform output cursor
        for (int64_t base = e0; base < e1; base += 64) {
            const int64_t e = base + lane;
            int64_t m = 0, c = 0;
            if (e < e1) {
                c = ci[e];
                m = JALL ? 1 : jptr[c + 1] - jptr[c];
            }
            // inclusive wave scan of m
            int64_t incl = m;
#pragma unroll
            for (int off = 1; off < 64; off <<= 1) {
                int64_t t = __shfl_up(incl, off, 64);
                if (lane >= off) incl += t;
            }
            const int64_t total = __shfl(incl, 63, 64);
            if (FILL && m) {
                int64_t pos = run + incl - m;
                if (JALL) {
                    okey[pos] = ((uint64_t)r << 32) | (uint64_t)c;
                    osrc[pos] = e;
                } else {
                    for (int64_t k = 0; k < m; k++) {
                        okey[pos + k] = ((uint64_t)r << 32) | (uint64_t)(uint32_t)jpos[jptr[c] + k];
                        osrc[pos + k] = e;
                    }
                }
            }
            run += total;
        }
        if (!FILL && lane == 0) cnt[r] = run;
    }
}

// colidx / values of the output from the (sorted) keys and source positions
template <class V>
__global__ void k_ext_finish(int64_t nz, const uint64_t *__restrict__ key, const int64_t *__restrict__ src,
                             const V *__restrict__ vin, int32_t *__restrict__ colidx, V *__restrict__ vout) {
    for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < nz; t += (int64_t)gridDim.x * blockDim.x) {
        colidx[t] = (int32_t)(key[t] & 0xffffffffULL);
        if (vout) vout[t] = vin[src[t]];
    }
}

// w(k) = u(I[k]) on bitmaps: a wave per output word
template <class V>
__global__ __launch_bounds__(EXT_BLOCK) void k_ext_vec(int64_t nk, const int64_t *__restrict__ I,
                                                       const uint64_t *__restrict__ ubits, const V *__restrict__ uvals,
                                                       uint64_t *__restrict__ wbits, V *__restrict__ wvals) {
    const int lane = threadIdx.x & 63;
    for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; (k & ~63LL) < nk;
         k += (int64_t)gridDim.x * blockDim.x) {
        bool hit = false;
        if (k < nk) {
            const int64_t i = I[k];
            hit = (ubits[i >> 6] >> (i & 63)) & 1ULL;
            if (hit && wvals) wvals[k] = uvals[i];
        }
        const uint64_t word = __ballot(hit);
        if (lane == 0) wbits[k >> 6] = word;
    }
}

// w(k) = V(j, I[k]) (I == nullptr: k itself): binary search in row j of V's sorted columns
template <class V>
__global__ __launch_bounds__(EXT_BLOCK) void k_ext_col(int64_t nk, const int64_t *__restrict__ I,
                                                       const int32_t *__restrict__ ci, int64_t e0, int64_t e1,
                                                       const V *__restrict__ vin, uint64_t *__restrict__ wbits,
                                                       V *__restrict__ wvals) {
    const int lane = threadIdx.x & 63;
    for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; (k & ~63LL) < nk;
         k += (int64_t)gridDim.x * blockDim.x) {
        bool hit = false;
        if (k < nk) {
            const int64_t c = I ? I[k] : k;
            int64_t lo = e0, hi = e1;
            while (lo < hi) {
                const int64_t mid = (lo + hi) >> 1;
                if (ci[mid] < c) lo = mid + 1;
                else hi = mid;
            }
            hit = lo < e1 && ci[lo] == c;
            if (hit && wvals) wvals[k] = vin[lo];
        }
        const uint64_t word = __ballot(hit);
        if (lane == 0) wbits[k >> 6] = word;
    }
}

template <class F>
static void with_size(size_t ts, F &&f) {
    switch (ts) {
    case 1: f(uint8_t()); break;
    case 2: f(uint16_t()); break;
    case 4: f(uint32_t()); break;
    case 8: f(uint64_t()); break;
    default: gb_throw(GrB_NOT_IMPLEMENTED, "value size");
    }
}

static int64_t *upload_list(const gb_index_list &L, gb_scratch &s) {
    if (L.all || L.n == 0) return nullptr;
    int64_t *d = s.get<int64_t>(L.n);
    gb_copy_h2d(d, L.idx.data(), L.n * sizeof(int64_t));
    return d;
}

// T = V(I, J) for a CSR view V
static void extract_csr(gb_mat_result &T, const gb_csr_view &v, const gb_index_list &LI, const gb_index_list &LJ) {
    gb_scratch s;
    const int64_t ni = LI.n, nj = LJ.n;
    GB_REQUIRE(ni < (1LL << 31) && nj < (1LL << 31), GrB_NOT_IMPLEMENTED, "extract of more than 2^31 rows/columns");
    const int64_t *dI = upload_list(LI, s);
    const int64_t *dJ = upload_list(LJ, s);
    T.nrows = ni;
    T.ncols = nj;
    T.tcode = v.tcode;
    T.iso = v.iso;
    const size_t ts = gb_type_size(v.tcode);
    T.rowptr = gb_malloc_n<int64_t>(ni + 1);
    const int64_t *jptr = nullptr;
    int32_t *jpos = nullptr;
    if (!LJ.all) {
        int32_t *jcnt = s.get<int32_t>(v.ncols);
        gb_memset(jcnt, 0, v.ncols * sizeof(int32_t));
        if (nj) hipLaunchKernelGGL(k_ext_jcount, dim3(ext_grid(nj, EXT_BLOCK, 4096)), dim3(EXT_BLOCK), 0, gb_stream(),
                                   nj, dJ, jcnt);
        int64_t *jp = s.get<int64_t>(v.ncols + 1);
        gb_exclusive_scan_i32(jcnt, 0, jp, v.ncols);
        int64_t *cursor = s.get<int64_t>(v.ncols + 1);
        gb_copy_d2d(cursor, jp, (v.ncols + 1) * sizeof(int64_t));
        jpos = s.get<int32_t>(nj);
        if (nj) hipLaunchKernelGGL(k_ext_jfill, dim3(ext_grid(nj, EXT_BLOCK, 4096)), dim3(EXT_BLOCK), 0, gb_stream(),
                                   nj, dJ, cursor, jpos);
        jptr = jp;
    }
    int64_t *cnt = s.get<int64_t>(ni + 1);
    const unsigned grid = ext_grid(ni, EXT_BLOCK / 64, 16384);
    if (ni) {
        if (LJ.all)
            hipLaunchKernelGGL((k_ext_rows<true, false>), dim3(grid), dim3(EXT_BLOCK), 0, gb_stream(), ni, dI,
                               v.rowptr, v.colidx, jptr, jpos, cnt, nullptr, nullptr, nullptr);
        else
            hipLaunchKernelGGL((k_ext_rows<false, false>), dim3(grid), dim3(EXT_BLOCK), 0, gb_stream(), ni, dI,
                               v.rowptr, v.colidx, jptr, jpos, cnt, nullptr, nullptr, nullptr);
        GB_LAUNCH_CHECK();
    }
    gb_exclusive_scan_i64(cnt, T.rowptr, ni);
    const int64_t nz = gb_read_i64(T.rowptr + ni);
    T.nvals = nz;
    T.colidx = gb_malloc_n<int32_t>(nz);
    T.vals = gb_malloc((v.iso ? 1 : nz) * ts);
    if (v.iso) gb_copy_d2d(T.vals, v.vals, ts);
    if (nz) {
        uint64_t *key = s.get<uint64_t>(nz);
        int64_t *src = s.get<int64_t>(nz);
        if (LJ.all)
            hipLaunchKernelGGL((k_ext_rows<true, true>), dim3(grid), dim3(EXT_BLOCK), 0, gb_stream(), ni, dI,
                               v.rowptr, v.colidx, jptr, jpos, nullptr, T.rowptr, key, src);
        else
            hipLaunchKernelGGL((k_ext_rows<false, true>), dim3(grid), dim3(EXT_BLOCK), 0, gb_stream(), ni, dI,
                               v.rowptr, v.colidx, jptr, jpos, nullptr, T.rowptr, key, src);
        GB_LAUNCH_CHECK();
        if (!LJ.all) {
            int bits = 32;
            while (bits < 64 && (1LL << (bits - 32)) < ni) bits++;
            gb_sort_pairs_u64(key, src, nz, bits);
        }
        with_size(ts, [&](auto z) {
            using V = decltype(z);
            hipLaunchKernelGGL((k_ext_finish<V>), dim3(ext_grid(nz, EXT_BLOCK, 16384)), dim3(EXT_BLOCK), 0,
                               gb_stream(), nz, key, src, (const V *)v.vals, T.colidx, v.iso ? nullptr : (V *)T.vals);
        });
        GB_LAUNCH_CHECK();
    }
}

static gb_vec_result empty_vec_result(int64_t n, int code, bool iso) {
    gb_vec_result T;
    T.n = n;
    T.tcode = code;
    T.iso = iso;
    T.bits = gb_malloc_n<uint64_t>(gb_words(n) ? gb_words(n) : 1);
    T.dense = gb_malloc((iso ? 1 : std::max<int64_t>(n, 1)) * gb_type_size(code));
    T.d_nvals = gb_malloc_n<int64_t>(1);
    return T;
}

extern "C" {

GrB_Info GrB_Matrix_extract(GrB_Matrix C, const GrB_Matrix Mask, const GrB_BinaryOp accum, const GrB_Matrix A,
                            const GrB_Index *I, GrB_Index ni, const GrB_Index *J, GrB_Index nj,
                            const GrB_Descriptor desc) {
    return gb_api(OBJ(C), [&] {
        GB_Obj *Co = gb_obj_check(C), *Ao = gb_obj_check(A), *Mo = gb_obj_check(Mask, true);
        GB_REQUIRE(!accum || accum->magic == GB_MAGIC, GrB_UNINITIALIZED_OBJECT, "invalid accum");
        gb_desc d = gb_read_desc(desc);
        gb_csr_view v;
        if (d.tran0) gb_get_csc(v, Ao);
        else gb_get_csr(v, Ao);
        gb_index_list LI, LJ;
        gb_expand_indices(LI, I, ni, v.nrows);
        gb_expand_indices(LJ, J, nj, v.ncols);
        const int64_t cc = Co->kind == GB_KIND_MATRIX ? Co->ncols : 1;
        GB_REQUIRE(Co->nrows == LI.n && cc == LJ.n, GrB_DIMENSION_MISMATCH,
                   "output dimensions do not match the index lists");
        gb_mat_result T;
        extract_csr(T, v, LI, LJ);
        gb_writeback_matrix(Co, T, Mo, d, accum);
    });
}

GrB_Info GrB_Col_extract(GrB_Vector w, const GrB_Vector mask, const GrB_BinaryOp accum, const GrB_Matrix A,
                         const GrB_Index *I, GrB_Index ni, GrB_Index j, const GrB_Descriptor desc) {
    return gb_api(OBJ(w), [&] {
        GB_Obj *W = gb_obj_check(w), *Ao = gb_obj_check(A), *Mo = gb_obj_check(mask, true);
        GB_REQUIRE(!accum || accum->magic == GB_MAGIC, GrB_UNINITIALIZED_OBJECT, "invalid accum");
        gb_desc d = gb_read_desc(desc);
        // A'(I, j) = row j of A'^T: the CSC of A, or A's CSR when INP0 is transposed
        gb_csr_view v;
        if (d.tran0) gb_get_csr(v, Ao);
        else gb_get_csc(v, Ao);
        GB_REQUIRE(j < (GrB_Index)v.nrows, GrB_INVALID_INDEX, "column index out of bounds");
        gb_index_list LI;
        gb_expand_indices(LI, I, ni, v.ncols);
        GB_REQUIRE(W->nrows == LI.n, GrB_DIMENSION_MISMATCH, "output size does not match the index list");
        gb_scratch s;
        const int64_t *dI = upload_list(LI, s);
        int64_t e[2];
        gb_copy_d2h(e, v.rowptr + j, 2 * sizeof(int64_t));
        gb_vec_result T = empty_vec_result(LI.n, v.tcode, v.iso);
        const size_t ts = gb_type_size(v.tcode);
        if (v.iso) gb_copy_d2d(T.dense, v.vals, ts);
        if (LI.n) {
            with_size(ts, [&](auto z) {
                using V = decltype(z);
                hipLaunchKernelGGL((k_ext_col<V>), dim3(ext_grid(LI.n, EXT_BLOCK, 16384)), dim3(EXT_BLOCK), 0,
                                   gb_stream(), LI.n, dI, v.colidx, e[0], e[1], (const V *)v.vals, T.bits,
                                   v.iso ? nullptr : (V *)T.dense);
            });
            GB_LAUNCH_CHECK();
        }
        gb_bitmap_count(T.bits, LI.n, T.d_nvals);
        gb_writeback_vector(W, T, Mo, d, accum, false);
    });
}

GrB_Info GrB_Vector_extract(GrB_Vector w, const GrB_Vector mask, const GrB_BinaryOp accum, const GrB_Vector u,
                            const GrB_Index *I, GrB_Index ni, const GrB_Descriptor desc) {
    return gb_api(OBJ(w), [&] {
        GB_Obj *W = gb_obj_check(w), *U = gb_obj_check(u), *Mo = gb_obj_check(mask, true);
        GB_REQUIRE(!accum || accum->magic == GB_MAGIC, GrB_UNINITIALIZED_OBJECT, "invalid accum");
        gb_desc d = gb_read_desc(desc);
        gb_bitmap_view uv;
        gb_get_bitmap(uv, U);
        gb_index_list LI;
        gb_expand_indices(LI, I, ni, uv.n);
        GB_REQUIRE(W->nrows == LI.n, GrB_DIMENSION_MISMATCH, "output size does not match the index list");
        gb_scratch s;
        std::vector<int64_t> ident;
        const int64_t *dI = upload_list(LI, s);
        if (LI.all && LI.n) {
            int64_t *d = s.get<int64_t>(LI.n);
            ident.resize(LI.n);
            for (int64_t k = 0; k < LI.n; k++) ident[k] = k;
            gb_copy_h2d(d, ident.data(), LI.n * sizeof(int64_t));
            dI = d;
        }
        gb_vec_result T = empty_vec_result(LI.n, uv.tcode, uv.iso);
        const size_t ts = gb_type_size(uv.tcode);
        if (uv.iso) gb_copy_d2d(T.dense, uv.vals, ts);
        if (LI.n) {
            with_size(ts, [&](auto z) {
                using V = decltype(z);
                hipLaunchKernelGGL((k_ext_vec<V>), dim3(ext_grid(LI.n, EXT_BLOCK, 16384)), dim3(EXT_BLOCK), 0,
                                   gb_stream(), LI.n, dI, uv.bits, (const V *)uv.vals, T.bits,
                                   uv.iso ? nullptr : (V *)T.dense);
            });
            GB_LAUNCH_CHECK();
        }
        gb_bitmap_count(T.bits, LI.n, T.d_nvals);
        gb_writeback_vector(W, T, Mo, d, accum, false);
    });
}

}  // extern "C"
