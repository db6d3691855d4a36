// gb_ops.hip -- the GraphBLAS operations exported by the C ABI:
//   GrB_mxm / GrB_mxv / GrB_vxm                      (the hot path)
//   eWiseMult / eWiseAdd, assign, reduce, transpose  (loop companions used by
//   python-graphblas's isequal (reference core/matrix.py:391-398) and the
//   BFS/SSSP notebook loops)
// Each call: validate -> views of the inputs (casting values to the operator's
// input type) -> compute T on the device -> C<M,replace> = C accum T.
#include <algorithm>
#include <atomic>
#include <mutex>
#include <vector>

#include "gb_dispatch.cuh"
#include "gb_internal.h"

#define OPS_BLOCK 256
static inline unsigned ops_grid(int64_t n, unsigned cap = 16384) {
    int64_t g = (n + OPS_BLOCK - 1) / OPS_BLOCK;
    if (g < 1) g = 1;
    if (g > cap) g = cap;
    return (unsigned)g;
}
#define OPS_STRIDE(i, n) \
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < (n); i += (int64_t)gridDim.x * blockDim.x)

static void check_semiring(GrB_Semiring sr) {
    GB_REQUIRE(sr, GrB_NULL_POINTER, "semiring is NULL");
    GB_REQUIRE(sr->magic == GB_MAGIC, GrB_UNINITIALIZED_OBJECT, "invalid semiring");
}
static void check_binop(GrB_BinaryOp op, bool allow_null) {
    if (!op) {
        GB_REQUIRE(allow_null, GrB_NULL_POINTER, "operator is NULL");
        return;
    }
    GB_REQUIRE(op->magic == GB_MAGIC, GrB_UNINITIALIZED_OBJECT, "invalid operator");
}
static int64_t ncols_of(GB_Obj *A) { return A->kind == GB_KIND_MATRIX ? A->ncols : 1; }

static bool take_pending_assign(gb_asg &asg, GB_Obj *w, GB_Obj *mask, GB_Obj *A, GB_Obj *u, const gb_desc &d,
                                bool iso_result);

// ================================================================== mxv / vxm
// The operand views of one SpMV: A' along the pulled rows (+ the other orientation for the
// push direction of iso results), u's bitmap (+ its next-frontier edge hint), the mask.
struct spmv_views {
    gb_csr_view av, pv;
    const gb_csr_view *push = nullptr;
    gb_bitmap_view uv;
    gb_vmask m;
    bool iso_result = false;
};

static void spmv_build_views(spmv_views &V, GB_Obj *mask, GrB_Semiring sr, GB_Obj *A, GB_Obj *u, const gb_desc &d,
                             bool vxm, int64_t a_rows, const gb_asg *asg) {
    const bool use_csc = vxm ? !d.tran1 : d.tran0;
    if (use_csc) gb_get_csc(V.av, A);
    else gb_get_csr(V.av, A);
    gb_view_nonempty(V.av, A, use_csc ? 1 : 0);
    gb_get_bitmap(V.uv, u);
    if (u->kind != GB_KIND_MATRIX && u->hint_valid) {
        V.uv.mf_hint = (const long long *)(u->d_nvals + 2);  // GB_HINT_PARTS parts
        V.uv.hint_key = u->hint_key;
    }
    if (u->kind != GB_KIND_MATRIX && u->nvals_valid) V.uv.h_nvals = u->nvals;
    gb_make_vmask(V.m, mask, d, a_rows);
    // an empty mask vector: its count is known on the host (value or structure alike)
    if (V.m.bits && mask && mask->kind != GB_KIND_MATRIX && mask->nvals_valid && mask->nvals == 0) V.m.h_count = 0;
    // the fused assign's target is the mask (take_pending_assign): its count before this call's
    // assign, as the host knew it when the assign was deferred (a BFS's first level after
    // clearing v: 0), lets gb_spmv pick push on the host without the prep launch
    // -- a stored-entry count equals the set-bit count only for a structural mask; for a value
    // mask it is an upper bound, which still bounds the open rows of a complemented mask from
    // below but says nothing for a plain one
    if (asg && V.m.bits && V.m.h_count < 0 && asg->h_count >= 0 && (d.structure || d.comp))
        V.m.h_count = asg->h_count;
    // the other orientation (cached on matrices) enables the push direction for iso results
    V.iso_result = gb_spmv_result_iso(sr, A->iso, V.uv.iso, vxm);
    if (!V.iso_result) gb_view_long_rows(V.av, A, use_csc ? 1 : 0);
    V.uv.full = u->kind != GB_KIND_MATRIX && u->nvals_valid && u->nvals == u->nrows && u->nrows > 0;
    if (!V.iso_result && V.uv.full && !V.uv.iso && A->kind == GB_KIND_MATRIX && !gb_sr_describe(sr).positional)
        gb_view_hot(V.av, A, use_csc ? 1 : 0);
    if (A->kind == GB_KIND_MATRIX && gb_knob("spmv_direction") != 1 && V.iso_result) {
        if (use_csc) gb_get_csr(V.pv, A);
        else gb_get_csc(V.pv, A);
        int64_t H = gb_knob("push_heavy");
        gb_view_hubs(V.pv, A, use_csc ? 0 : 1, H > 0 ? H : 512);
        V.push = &V.pv;
        if (gb_knob("pull_first") != 1) gb_view_pullfirst(V.av, A, use_csc ? 1 : 0, V.pv.rowptr, V.pv.nrows);
    }
}

static bool spec_try_adopt(GB_Obj *w, GB_Obj *mask, GrB_BinaryOp accum, GrB_Semiring sr, GB_Obj *A, GB_Obj *u,
                           const gb_desc &d, bool vxm);
static void spec_after_level(GB_Obj *w, GB_Obj *mask, GrB_BinaryOp accum, GrB_Semiring sr, GB_Obj *A, GB_Obj *u,
                             const gb_desc &d, bool vxm, const gb_asg &asg, bool direct, bool published);

static void do_spmv(GB_Obj *w, GB_Obj *mask, GrB_BinaryOp accum, GrB_Semiring sr, GB_Obj *A, GB_Obj *u,
                    const gb_desc &d, bool vxm) {
    GB_HPROF(1, "do_spmv total");
    check_semiring(sr);
    check_binop(accum, true);
    // rows of the operand matrix the kernel pulls along:
    //   mxv:  w = A' u    -> rows of A'          (A' = A: CSR, A' = A^T: CSC)
    //   vxm:  w = u' A'   -> rows of A'^T        (A' = A: CSC, A' = A^T: CSR)
    int64_t a_rows = (vxm ? (d.tran1 ? A->nrows : ncols_of(A)) : (d.tran0 ? ncols_of(A) : A->nrows));
    int64_t a_cols = (vxm ? (d.tran1 ? ncols_of(A) : A->nrows) : (d.tran0 ? A->nrows : ncols_of(A)));
    GB_REQUIRE(u->nrows == a_cols && ncols_of(u) == 1, GrB_DIMENSION_MISMATCH, "u size does not match A");
    GB_REQUIRE(w->nrows == a_rows && ncols_of(w) == 1, GrB_DIMENSION_MISMATCH, "w size does not match A");
    // the next BFS level, launched speculatively by the previous call (below): adopted when this
    // call is the one predicted, rolled back otherwise
    if (g_spec_active.load(std::memory_order_acquire) && spec_try_adopt(w, mask, accum, sr, A, u, d, vxm)) return;
    // a deferred `mask<u> = x` (the BFS level stamp) is fused into this call's kernel, or done now
    gb_asg asg;
    bool fused = false;
    if (g_pending_active.load(std::memory_order_acquire)) {
        fused = A->kind == GB_KIND_MATRIX && u->kind != GB_KIND_MATRIX &&
                take_pending_assign(asg, w, mask, A, u, d, gb_spmv_result_iso(sr, A->iso, u->iso, vxm));
        if (!fused) {
            if (g_root_active.load(std::memory_order_acquire)) gb_root_flush();  // the assign may read it
            gb_pending_flush();
        }
    }
    const int64_t hp_t0 = g_hprof_on ? gb_hprof_now() : 0;
    spmv_views V;
    spmv_build_views(V, mask, sr, A, u, d, vxm, a_rows, fused ? &asg : nullptr);
    if (g_hprof_on) gb_hprof_add(2, "do_spmv views+mask", gb_hprof_now() - hp_t0);
    // a pending root (the BFS start): consumed by the notebook level shape -- q<!v.S, replace> =
    // q (+).(x) A with the stamp v<q> = x fused, iso result, push orientation at hand -- whose kernel
    // pushes from it; materialised before any other SpMV
    if (g_root_active.load(std::memory_order_acquire)) {
        const bool shape = fused && u == w && !accum && d.replace && d.comp && d.structure && V.iso_result &&
                           V.push && V.push->nrows == u->nrows && V.push->hubs && gb_knob("spmv_direction") != 1;
        if (shape) asg.root = gb_root_take(u);
        if (asg.root >= 0) {
            // u's storage does not hold the root: its iso value (true) and count come from the host
            V.uv.vals = gb_bool_true_dev();
            V.uv.count = nullptr;
            if (asg.q_iso) asg.q_iso = gb_bool_true_dev();
        } else {
            gb_root_flush();
        }
    }
    gb_vec_result T;
    if (w->kind != GB_KIND_MATRIX) {
        if (!w->pub) w->pub = gb_host_slot_alloc();
        T.pub = w->pub;
        T.pub_seq = gb_next_pub_seq(T.pub);
    }
    {
        GB_HPROF(3, "gb_spmv (host+launch)");
        gb_spmv(T, V.av, V.push, V.uv, V.m, sr, vxm, fused ? &asg : nullptr);
    }
    const void *hint_key = T.hint_key;
    const bool published = T.published;
    GB_HPROF(4, "writeback+epilogue");
    const bool direct = gb_writeback_vector(w, T, mask, d, accum, true);
    if (direct && published) {
        // w's count is the one the kernel published; valid until more work is enqueued
        w->pub_seq = T.pub_seq;
        w->pub_epoch = gb_epoch();
    }
    if (direct && hint_key && w->kind != GB_KIND_MATRIX) {
        w->hint_valid = true;
        w->hint_key = hint_key;
    }
    if (fused) spec_after_level(w, mask, accum, sr, A, u, d, vxm, asg, direct, published);
}

// ================================================================== mxm
static void do_mxm(GB_Obj *C, GB_Obj *M, GrB_BinaryOp accum, GrB_Semiring sr, GB_Obj *A, GB_Obj *B,
                   const gb_desc &d) {
    check_semiring(sr);
    check_binop(accum, true);
    int64_t ar = d.tran0 ? ncols_of(A) : A->nrows, ac = d.tran0 ? A->nrows : ncols_of(A);
    int64_t br = d.tran1 ? ncols_of(B) : B->nrows, bc = d.tran1 ? B->nrows : ncols_of(B);
    GB_REQUIRE(ac == br, GrB_DIMENSION_MISMATCH, "inner dimensions of A and B do not match");
    GB_REQUIRE(C->nrows == ar && ncols_of(C) == bc, GrB_DIMENSION_MISMATCH, "C dimensions do not match A*B");
    gb_csr_view av, bv, btv;
    if (d.tran0) gb_get_csc(av, A);
    else gb_get_csr(av, A);
    if (d.tran1) gb_get_csc(bv, B);
    else gb_get_csr(bv, B);
    gb_mmask m;
    gb_make_mmask(m, M, d, ar, bc);
    gb_csr_view *btp = nullptr;
    int64_t method = gb_knob("mxm_method");  // 0 auto, 1 dot, 2 gustavson
    if (m.present && !m.comp && method != 2) {
        // B'^T: rows are the columns of B'
        if (d.tran1) gb_get_csr(btv, B);
        else gb_get_csc(btv, B);
        btp = &btv;
        // the masked dot reads one value per matching key: narrow copies of integer values
        if (gb_sr_describe(sr).reads_values) {
            gb_view_narrow(av, A, d.tran0 ? 1 : 0);
            gb_view_narrow(btv, B, d.tran1 ? 0 : 1);
        }
    }
    gb_mat_result T;
    gb_spgemm(T, av, bv, btp, m, sr);
    gb_writeback_matrix(C, T, M, d, accum);
}

// ================================================================== eWise
template <class X, class Z>
__global__ void k_ewise_vec(int64_t n, int op, bool add, const uint64_t *__restrict__ ub, const X *__restrict__ ux,
                            bool u_iso, const uint64_t *__restrict__ vb, const X *__restrict__ vx, bool v_iso,
                            uint64_t *__restrict__ ob, Z *__restrict__ oz, unsigned long long *__restrict__ cnt,
                            unsigned long long *__restrict__ gst) {
    unsigned long long mine = 0;
    for (int64_t base = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) & ~63LL; base < n;
         base += (int64_t)gridDim.x * blockDim.x) {
        int64_t i = base + (threadIdx.x & 63);
        bool a = i < n && gb_bit(ub, i), b = i < n && gb_bit(vb, i);
        bool have = add ? (a || b) : (a && b);
        if (have) {
            if (a && b) oz[i] = gb_binop_z<X, Z>(op, ux[u_iso ? 0 : i], vx[v_iso ? 0 : i], i, 0, 0);
            else if (a) oz[i] = gb_cast<Z, X>(ux[u_iso ? 0 : i]);
            else oz[i] = gb_cast<Z, X>(vx[v_iso ? 0 : i]);
        }
        unsigned long long w = __ballot(have);
        if ((threadIdx.x & 63) == 0) {
            ob[base >> 6] = w;
            mine += __popcll(w);
        }
    }
    gb_grid_add((long long)mine, cnt, gst);
}

template <class X, class Z, bool FILL>
__global__ void k_ewise_mat(int64_t nrows, int op, bool add, const int64_t *__restrict__ arp,
                            const int32_t *__restrict__ aci, const X *__restrict__ ax, bool a_iso,
                            const int64_t *__restrict__ brp, const int32_t *__restrict__ bci, const X *__restrict__ bx,
                            bool b_iso, int64_t *__restrict__ orp, int32_t *__restrict__ oci, Z *__restrict__ oz) {
    OPS_STRIDE(i, nrows) {
        int64_t pa = arp[i], ea = arp[i + 1], pb = brp[i], eb = brp[i + 1];
        int64_t o = FILL ? orp[i] : 0;
        while (pa < ea || pb < eb) {
            int32_t ja = pa < ea ? aci[pa] : INT32_MAX, jb = pb < eb ? bci[pb] : INT32_MAX;
            int32_t j = ja < jb ? ja : jb;
            bool a = ja == j, b = jb == j;
            bool have = add ? true : (a && b);
            if (have) {
                if (FILL) {
                    oci[o] = j;
                    if (a && b) oz[o] = gb_binop_z<X, Z>(op, ax[a_iso ? 0 : pa], bx[b_iso ? 0 : pb], i, j, j);
                    else if (a) oz[o] = gb_cast<Z, X>(ax[a_iso ? 0 : pa]);
                    else oz[o] = gb_cast<Z, X>(bx[b_iso ? 0 : pb]);
                }
                o++;
            }
            if (a) pa++;
            if (b) pb++;
        }
        if (!FILL) orp[i] = o;
    }
}

template <class F>
static void dispatch_xz(int xcode, int zcode, F &&f) {
    if (xcode == zcode) {
        gb_with_type(xcode, [&](auto x) {
            using X = decltype(x);
            f(X{}, X{});
        });
    } else if (zcode == GBAMD_T_BOOL) {
        gb_with_type(xcode, [&](auto x) {
            using X = decltype(x);
            f(X{}, bool{});
        });
    } else {
        gb_throw(GrB_NOT_IMPLEMENTED, "operator type combination not supported");
    }
}

static void do_ewise(GB_Obj *C, GB_Obj *M, GrB_BinaryOp accum, GrB_BinaryOp op, GB_Obj *A, GB_Obj *B,
                     const gb_desc &d, bool add) {
    check_binop(op, false);
    check_binop(accum, true);
    GB_REQUIRE(op->xtype != nullptr, GrB_NOT_IMPLEMENTED, "positional eWise operator");
    int xcode = op->xtype->code, zcode = op->ztype->code;
    bool vec = C->kind != GB_KIND_MATRIX;
    if (vec) {
        int64_t n = C->nrows;
        GB_REQUIRE(A->nrows == n && B->nrows == n && ncols_of(A) == 1 && ncols_of(B) == 1, GrB_DIMENSION_MISMATCH,
                   "vector sizes do not match");
        gb_bitmap_view ua, ub;
        gb_get_bitmap(ua, A);
        gb_get_bitmap(ub, B);
        gb_scratch s;
        const void *xa = gb_bitmap_vals_as(ua, xcode, s), *xb = gb_bitmap_vals_as(ub, xcode, s);
        gb_vec_result T;
        T.n = n;
        T.tcode = zcode;
        T.bits = gb_malloc_n<uint64_t>(gb_words(n));
        T.dense = gb_malloc(n * gb_type_size(zcode));
        T.d_nvals = gb_malloc_n<int64_t>(1);
        gb_memset(T.d_nvals, 0, sizeof(int64_t));
        dispatch_xz(xcode, zcode, [&](auto x, auto z) {
            using X = decltype(x);
            using Z = decltype(z);
            if (n)
                hipLaunchKernelGGL((k_ewise_vec<X, Z>), dim3(ops_grid(n, 1024)), dim3(OPS_BLOCK), 0, gb_stream(), n,
                                   op->opcode, add, ua.bits, (const X *)xa, ua.iso, ub.bits, (const X *)xb, ub.iso,
                                   T.bits, (Z *)T.dense, (unsigned long long *)T.d_nvals, gb_device_state());
        });
        GB_LAUNCH_CHECK();
        gb_writeback_vector(C, T, M, d, accum, false);
        return;
    }
    int64_t nr = C->nrows, nc = C->ncols;
    GB_Obj *A2 = A, *B2 = B;
    gb_csr_view av, bv;
    if (d.tran0) gb_get_csc(av, A2);
    else gb_get_csr(av, A2);
    if (d.tran1) gb_get_csc(bv, B2);
    else gb_get_csr(bv, B2);
    GB_REQUIRE(av.nrows == nr && av.ncols == nc && bv.nrows == nr && bv.ncols == nc, GrB_DIMENSION_MISMATCH,
               "matrix dimensions do not match");
    gb_scratch s;
    const void *xa = gb_view_vals_as(av, xcode, s), *xb = gb_view_vals_as(bv, xcode, s);
    gb_mat_result T;
    T.nrows = nr;
    T.ncols = nc;
    T.tcode = zcode;
    int64_t *cnt = s.get<int64_t>(nr + 1);
    T.rowptr = gb_malloc_n<int64_t>(nr + 1);
    dispatch_xz(xcode, zcode, [&](auto x, auto z) {
        using X = decltype(x);
        using Z = decltype(z);
        if (nr)
            hipLaunchKernelGGL((k_ewise_mat<X, Z, false>), dim3(ops_grid(nr)), dim3(OPS_BLOCK), 0, gb_stream(), nr,
                               op->opcode, add, av.rowptr, av.colidx, (const X *)xa, av.iso, bv.rowptr, bv.colidx,
                               (const X *)xb, bv.iso, cnt, nullptr, nullptr);
        GB_LAUNCH_CHECK();
        gb_exclusive_scan_i64(cnt, T.rowptr, nr);
        T.nvals = gb_read_i64(T.rowptr + nr);
        T.colidx = gb_malloc_n<int32_t>(T.nvals);
        T.vals = gb_malloc(T.nvals * sizeof(Z));
        if (nr)
            hipLaunchKernelGGL((k_ewise_mat<X, Z, true>), dim3(ops_grid(nr)), dim3(OPS_BLOCK), 0, gb_stream(), nr,
                               op->opcode, add, av.rowptr, av.colidx, (const X *)xa, av.iso, bv.rowptr, bv.colidx,
                               (const X *)xb, bv.iso, T.rowptr, T.colidx, (Z *)T.vals);
        GB_LAUNCH_CHECK();
    });
    gb_writeback_matrix(C, T, M, d, accum);
}

// ================================================================== reduce
template <class T>
__global__ void k_reduce_partial(int mon, const T *__restrict__ vals, bool iso, int64_t nvals,
                                 const uint64_t *__restrict__ bits, int64_t n, T *__restrict__ part,
                                 int *__restrict__ pfound) {
    // bits == nullptr: reduce vals[0..nvals); else reduce vals[i] for set bits i < n
    __shared__ T sv[256];
    __shared__ int sf[256];
    T acc = T();
    bool found = false;
    int64_t total = bits ? n : nvals;
    OPS_STRIDE(i, total) {
        if (bits && !gb_bit(bits, i)) continue;
        T v = vals[iso ? 0 : i];
        acc = found ? gb_monoid<T>(mon, acc, v) : v;
        found = true;
    }
    sv[threadIdx.x] = acc;
    sf[threadIdx.x] = found;
    __syncthreads();
    if (threadIdx.x == 0) {
        T a = T();
        bool f = false;
        for (int t = 0; t < blockDim.x; t++)
            if (sf[t]) {
                a = f ? gb_monoid<T>(mon, a, sv[t]) : sv[t];
                f = true;
            }
        part[blockIdx.x] = a;
        pfound[blockIdx.x] = f;
    }
}

// returns true if any entry; value in *out (monoid type)
static bool reduce_values(GB_Obj *A, GrB_Monoid monoid, void *out) {
    GB_REQUIRE(monoid && monoid->magic == GB_MAGIC, GrB_UNINITIALIZED_OBJECT, "invalid monoid");
    int code = monoid->type->code;
    gb_scratch s;
    const void *vals;
    bool iso;
    const uint64_t *bits = nullptr;
    int64_t n, nvals;
    gb_bitmap_view bv;
    gb_csr_view cv;
    if (A->kind == GB_KIND_MATRIX) {
        gb_get_csr(cv, A);
        vals = gb_view_vals_as(cv, code, s);
        iso = cv.iso;
        nvals = cv.nvals;
        n = nvals;
    } else {
        gb_get_bitmap(bv, A);
        vals = gb_bitmap_vals_as(bv, code, s);
        iso = bv.iso;
        bits = bv.bits;
        n = bv.n;
        nvals = n;
    }
    const int nb = (int)std::max<int64_t>(1, std::min<int64_t>(256, (n + 255) / 256));
    bool any = false;
    gb_with_type(code, [&](auto z) {
        using T = decltype(z);
        T *part = s.get<T>(nb);
        int *pf = s.get<int>(nb);
        hipLaunchKernelGGL(k_reduce_partial<T>, dim3(nb), dim3(256), 0, gb_stream(), monoid->mcode, (const T *)vals,
                           iso, nvals, bits, n, part, pf);
        GB_LAUNCH_CHECK();
        std::vector<char> hpb(nb * sizeof(T));
        std::vector<int> hf(nb);
        gb_copy_d2h(hpb.data(), part, nb * sizeof(T));
        gb_copy_d2h(hf.data(), pf, nb * sizeof(int));
        T acc = T();
        for (int b = 0; b < nb; b++)
            if (hf[b]) {
                T hv;
                memcpy(&hv, hpb.data() + b * sizeof(T), sizeof(T));
                acc = any ? gb_monoid<T>(monoid->mcode, acc, hv) : hv;
                any = true;
            }
        memcpy(out, &acc, sizeof(T));
    });
    return any;
}

// identity of a monoid (value written to *out)
static void monoid_identity(GrB_Monoid monoid, void *out) {
    int m = monoid->mcode;
    gb_with_type(monoid->type->code, [&](auto z) {
        using T = decltype(z);
        T v = T();
        switch (m) {
        case GBAMD_MON_TIMES: v = (T)1; break;
        case GBAMD_MON_MIN: v = gb_tmax<T>(); break;
        case GBAMD_MON_MAX: v = gb_tmin<T>(); break;
        case GBAMD_MON_LAND: case GBAMD_MON_LXNOR: v = (T)1; break;
        case GBAMD_MON_BAND: case GBAMD_MON_BXNOR:
            if constexpr (gb_traits<T>::is_int) v = (T)~(T)0;
            break;
        default: v = T(); break;
        }
        memcpy(out, &v, sizeof(T));
    });
}

// ================================================================== transpose
static void do_transpose(GB_Obj *C, GB_Obj *M, GrB_BinaryOp accum, GB_Obj *A, const gb_desc &d) {
    check_binop(accum, true);
    gb_csr_view v;
    if (d.tran0) gb_get_csr(v, A);  // transpose of the transpose
    else gb_get_csc(v, A);
    gb_mat_result T;
    T.nrows = v.nrows;
    T.ncols = v.ncols;
    T.nvals = v.nvals;
    T.tcode = v.tcode;
    T.iso = v.iso;
    size_t ts = gb_type_size(v.tcode);
    T.rowptr = gb_malloc_n<int64_t>(v.nrows + 1);
    gb_copy_d2d(T.rowptr, v.rowptr, (v.nrows + 1) * sizeof(int64_t));
    T.colidx = gb_malloc_n<int32_t>(v.nvals);
    gb_copy_d2d(T.colidx, v.colidx, v.nvals * sizeof(int32_t));
    int64_t nv = v.iso ? 1 : v.nvals;
    T.vals = gb_malloc(nv * ts);
    gb_copy_d2d(T.vals, v.vals, nv * ts);
    gb_writeback_matrix(C, T, M, d, accum);
}

// ================================================================== assign
// T for "x assigned at every index of I (GrB_ALL: all)": iso bitmap vector
static void scalar_vec_T(gb_vec_result &T, int64_t n, const GrB_Index *I, int64_t ni, const void *x, int code) {
    T.n = n;
    T.tcode = code;
    T.iso = true;
    int64_t nw = gb_words(n);
    T.bits = gb_malloc_n<uint64_t>(nw);
    T.dense = gb_malloc(gb_type_size(code));
    gb_copy_h2d(T.dense, x, gb_type_size(code));
    T.d_nvals = gb_malloc_n<int64_t>(1);
    if (I == GrB_ALL) {
        std::vector<uint64_t> hb(nw, ~0ULL);
        if (n & 63) hb[nw - 1] = (1ULL << (n & 63)) - 1;
        gb_copy_h2d(T.bits, hb.data(), nw * sizeof(uint64_t));
        int64_t nn = n;
        gb_copy_h2d(T.d_nvals, &nn, sizeof(int64_t));
        gb_sync();
        return;
    }
    std::vector<uint64_t> hb(nw, 0);
    int64_t c = 0;
    gb_index_list L;
    gb_expand_indices(L, I, (GrB_Index)ni, n);
    for (int64_t i : L.idx) {
        uint64_t &w = hb[i >> 6];
        uint64_t b = 1ULL << (i & 63);
        if (!(w & b)) c++;
        w |= b;
    }
    gb_copy_h2d(T.bits, hb.data(), nw * sizeof(uint64_t));
    gb_copy_h2d(T.d_nvals, &c, sizeof(int64_t));
    gb_sync();
}

static GrB_BinaryOp second_of(int code) {
    void *h;
    int kind;
    std::string name = std::string("GrB_SECOND_") + gb_type_name(code);
    GxB_builtin_lookup(&h, &kind, name.c_str());
    return (GrB_BinaryOp)h;
}

// w<M, replace>(:) = x with no accumulator, in place: one pass over the bitmap,
// values written only where the mask selects (BFS level stamping,
// notebooks/Example B.1 cell 8: v[:](mask=q.V) << d).  Waves whose 64 mask bits
// select nothing (and do not replace) leave their word untouched.
template <class T>
__global__ __launch_bounds__(OPS_BLOCK) void k_assign_all_scalar(
    int64_t n, uint64_t *__restrict__ cbits, T *__restrict__ cvals, const uint64_t *__restrict__ mbits, bool mcomp,
    const void *miso, int miso_code, bool replace, T x, unsigned long long *__restrict__ count,
    unsigned long long *__restrict__ gst) {
    // value mask over an iso vector: the mask is its structure if the value is true, else empty
    const bool iso_true = miso ? gb_dyn_nonzero(miso, miso_code) : true;
    long long delta = 0;  // change of nvals(C); added to the count C already holds
    for (int64_t base = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) & ~63LL; base < n;
         base += (int64_t)gridDim.x * blockDim.x) {
        const int lane = threadIdx.x & 63;
        const int64_t w = base >> 6;
        const int64_t i = base + lane;
        uint64_t mword = (mbits && iso_true) ? mbits[w] : 0;
        if (mbits && !mcomp && mword == 0 && !replace) continue;
        const uint64_t cword = cbits[w];
        bool inr = i < n;
        bool m = inr && (mbits ? ((((mword >> lane) & 1ULL) != 0) != mcomp) : !mcomp);
        bool c = (cword >> lane) & 1ULL;
        if (m) cvals[i] = x;
        bool have = m || (!replace && c && inr);
        unsigned long long word = __ballot(have);
        if (lane == 0) {
            if (word != cword) cbits[w] = word;
            delta += (long long)__popcll(word) - (long long)__popcll(cword);
        }
    }
    gb_grid_add(delta, count, gst);
}

// w<M>(:) = x, M a plain (non-complemented) mask, no replace: a wave takes 16
// mask words per step, one per lane (each lane updates its presence word);
// then the selected values of each non-zero word are written by the whole
// wave, one lane per position (coalesced stores).
template <class T>
__global__ __launch_bounds__(OPS_BLOCK) void k_assign_mask_words(int64_t nwords, uint64_t *__restrict__ cbits,
                                                                 T *__restrict__ cvals,
                                                                 const uint64_t *__restrict__ mbits, const void *miso,
                                                                 int miso_code, T x,
                                                                 unsigned long long *__restrict__ count,
                                                                 unsigned long long *__restrict__ gst) {
    const bool iso_true = miso ? gb_dyn_nonzero(miso, miso_code) : true;
    const int lane = threadIdx.x & 63;
    const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
    const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
    long long delta = 0;
    if (iso_true) {
        for (int64_t base = wave * 16; base < nwords; base += nwaves * 16) {
            const int64_t w = base + lane;
            const uint64_t m = (lane < 16 && w < nwords) ? mbits[w] : 0;
            if (m) {
                const uint64_t c = cbits[w], nwd = c | m;
                if (nwd != c) cbits[w] = nwd;
                delta += (long long)__popcll(nwd) - (long long)__popcll(c);
            }
            unsigned long long nz = __ballot(m != 0);
            while (nz) {
                const int l = __ffsll(nz) - 1;
                nz &= nz - 1;
                const uint64_t mw = __shfl(m, l, 64);
                if ((mw >> lane) & 1ULL) cvals[((base + l) << 6) + lane] = x;
            }
        }
    }
    gb_grid_add(delta, count, gst);
}

// make a vector's value array writable in place (non-iso, allocated) and its count present
static void make_values_writable(GB_Obj *w) {
    const int64_t n = w->nrows;
    const size_t ts = w->type->size;
    if (!w->dense) {
        w->dense = gb_malloc(n * ts);
        w->iso = false;
    } else if (w->iso) {
        void *full = gb_expand_iso(w->dense, ts, n);
        gb_free(w->dense);
        w->dense = full;
        w->iso = false;
    }
    if (!w->d_nvals) {
        w->d_nvals = gb_malloc_n<int64_t>(1);
        gb_memset(w->d_nvals, 0, sizeof(int64_t));
    }
}

static bool assign_all_scalar_fast(GB_Obj *w, GB_Obj *mask, const char *xc, const gb_desc &d) {
    if (w->kind == GB_KIND_MATRIX) return false;
    const int64_t n = w->nrows;
    const size_t ts = w->type->size;
    gb_vmask m;
    gb_make_vmask(m, mask, d, n, true);
    if (!m.bits && !m.comp) {
        // no mask: w becomes full and iso x
        int64_t nw = gb_words(n);
        uint64_t *bits = gb_malloc_n<uint64_t>(nw);
        gb_memset(bits, 0xff, nw * sizeof(uint64_t));
        if (n & 63) {
            uint64_t last = (1ULL << (n & 63)) - 1;
            gb_copy_h2d(bits + nw - 1, &last, sizeof(last));
        }
        void *dense = gb_malloc(ts);
        gb_copy_h2d(dense, xc, ts);
        int64_t *cnt = gb_malloc_n<int64_t>(1);
        gb_copy_h2d(cnt, &n, sizeof(int64_t));
        gb_sync();  // the host-side sources above live on this stack frame
        gb_install_bitmap(w, n, bits, dense, true, cnt);
        return true;
    }
    make_values_writable(w);
    unsigned grid = (unsigned)std::min<int64_t>((n + OPS_BLOCK - 1) / OPS_BLOCK, 1024);
    gb_with_type(w->type->code, [&](auto z) {
        using T = decltype(z);
        T xv;
        memcpy(&xv, xc, sizeof(T));
        if (n && m.bits && !m.comp && !d.replace)
            hipLaunchKernelGGL(k_assign_mask_words<T>,
                               dim3((unsigned)std::max<int64_t>(1, std::min<int64_t>((gb_words(n) + 63) / 64, 2048))),
                               dim3(OPS_BLOCK), 0, gb_stream(), gb_words(n), w->bits, (T *)w->dense, m.bits, m.iso_val,
                               m.iso_code, xv, (unsigned long long *)w->d_nvals, gb_device_state());
        else if (n)
            hipLaunchKernelGGL(k_assign_all_scalar<T>, dim3(grid), dim3(OPS_BLOCK), 0, gb_stream(), n, w->bits,
                               (T *)w->dense, m.bits, m.comp, m.iso_val, m.iso_code, d.replace, xv,
                               (unsigned long long *)w->d_nvals, gb_device_state());
    });
    GB_LAUNCH_CHECK();
    w->nvals_valid = false;
    w->hint_valid = false;
    return true;
}

// ---- deferred masked scalar assign (gb_asg): `w<q>(:) = x` is recorded instead of
// launched; the next GrB_mxv / GrB_vxm whose input is q and whose mask is w's
// structure performs it inside its kernel (the BFS level loop, notebooks/Example
// B.1 cell 8: v[:](mask=q.V) << d; q(~v.S, replace) << q.vxm(A)); any other API
// call performs it first (gb_api -> gb_pending_flush), so the deferral is never
// observable.  Knob fuse_assign = 1 disables it.
std::atomic<bool> g_pending_active{false};
static std::mutex g_pend_mu;
static struct {
    GB_Obj *w = nullptr, *mask = nullptr;
    char x[16];
    gb_desc d;
    int64_t w_count = -1;  // w's count before the deferral, when the host knew it
} g_pend;

// A failure of the deferred assign is an execution error of `w`, not of the call that
// triggered the flush: it is recorded on w (message + GrB_INVALID_OBJECT from then on,
// as the C API 2.0 prescribes for nonblocking execution errors) and the triggering call
// goes on.  The pending record is cleared only once the assign has been issued or has
// failed and been recorded.
void gb_pending_flush() {
    // the assign reads its mask's (or writes its target's) storage: a pending root there is materialised
    if (g_root_active.load(std::memory_order_acquire)) gb_root_flush();
    std::lock_guard<std::mutex> lk(g_pend_mu);
    GB_Obj *w = g_pend.w, *m = g_pend.mask;
    if (w && w->magic == GB_MAGIC && m && m->magic == GB_MAGIC && w->invalid == GrB_SUCCESS) {
        try {
            // fault injection for the tests (knob inject_flush_fail = 1)
            GB_REQUIRE(gb_knob("inject_flush_fail") != 1, GrB_OUT_OF_MEMORY, "injected failure");
            assign_all_scalar_fast(w, m, g_pend.x, g_pend.d);
        } catch (const gb_exception &e) {
            w->invalid = e.info;
            w->err = "deferred GrB_Vector_assign failed: " + e.msg;
        } catch (const std::bad_alloc &) {
            w->invalid = GrB_OUT_OF_MEMORY;
            w->err = "deferred GrB_Vector_assign failed: out of host memory";
        }
    }
    g_pend.w = g_pend.mask = nullptr;
    g_pending_active.store(false, std::memory_order_release);
}

static bool try_defer_assign(GB_Obj *w, GB_Obj *mask, const char *xc, const gb_desc &d) {
    if (gb_knob("fuse_assign") == 1) return false;
    if (!mask || mask == w || w->kind == GB_KIND_MATRIX || mask->kind == GB_KIND_MATRIX) return false;
    if (d.comp || d.replace || w->type->size > 8 || mask->nrows != w->nrows || !w->bits) return false;
    if (!d.structure && !(mask->iso && mask->dense)) return false;  // per-entry values: assign now
    make_values_writable(w);
    std::lock_guard<std::mutex> lk(g_pend_mu);
    g_pend.w = w;
    g_pend.mask = mask;
    memcpy(g_pend.x, xc, sizeof(g_pend.x));
    g_pend.d = d;
    g_pend.w_count = w->nvals_valid ? w->nvals : -1;
    g_pending_active.store(true, std::memory_order_release);
    w->nvals_valid = false;
    w->hint_valid = false;
    return true;
}

// take the pending assign into `asg` when this SpMV can carry it out (see above)
static bool take_pending_assign(gb_asg &asg, GB_Obj *w, GB_Obj *mask, GB_Obj *A, GB_Obj *u, const gb_desc &d,
                                bool iso_result) {
    std::lock_guard<std::mutex> lk(g_pend_mu);
    GB_Obj *pw = g_pend.w;
    if (!pw || pw != mask || g_pend.mask != u || !d.structure || w == pw || A == pw || !iso_result ||
        u->kind == GB_KIND_MATRIX || pw->nrows != u->nrows)
        return false;
    asg.bits = pw->bits;
    asg.vals = pw->dense;
    asg.size = (int)pw->type->size;
    memcpy(&asg.x, g_pend.x, sizeof(asg.x));
    asg.q_iso = g_pend.d.structure ? nullptr : u->dense;
    asg.q_iso_code = u->type->code;
    asg.count = pw->d_nvals;
    asg.h_count = g_pend.w_count;
    g_pend.w = g_pend.mask = nullptr;
    g_pending_active.store(false, std::memory_order_release);
    return true;
}

// ---- BFS level speculation (knob bfs_spec = 1 disables).  The notebook's level loop
// (reference notebooks/Example B.1 cell 8) is
//     v[:](mask=q.V) << d ;  q(~v.S, replace) << q.vxm(A) ;  if q.nvals == 0: break ;  d += 1
// and each level's launch waits on the host: the previous level's count reaches the host's
// nvals, then the host issues the next assign and vxm (≈ 12 µs of idle GPU per level, measured
// with rocprofv3 kernel traces).  After a level of exactly this shape (the
// deferred stamp `v<q> = x` fused into `q<!v.S, replace> = q (+).(x) A`, integer x), the next
// level -- stamp x + 1, then the same SpMV on the q just produced -- is enqueued right behind
// it, into a result of its own with a mailbox of its own.  When the host then issues exactly
// that assign and that vxm, the assign is absorbed and the vxm installs the speculative result
// (and enqueues the level after it): the GPU runs the levels back to back.  Anything else --
// another call touching v, q or A, a different stamp value, descriptor or semiring -- rolls the
// speculation back first: the speculative stamp only added q's bits to v (q and v are disjoint:
// q was produced under the mask !v.S), so clearing q's bits in v and subtracting q's count
// restores v exactly (nothing to undo when q is empty, the loop's normal exit), the speculative
// result is dropped, and an absorbed assign is re-issued.  Reads that the speculation leaves
// alone (nvals of any object but v) go through.  No call ever observes a speculative state.
std::atomic<bool> g_spec_active{false};
thread_local int g_spec_hold = 0;
std::atomic<int64_t> g_stat_spec_adopted{0}, g_stat_spec_rollbacks{0};
static void vector_assign_scalar(GB_Obj *w, GB_Obj *mask, GrB_BinaryOp accum, const void *x, int xcode,
                                 const GrB_Index *I, int64_t ni, const gb_desc &d);
static std::mutex g_spec_mu;
static struct {
    bool active = false;
    GB_Obj *q = nullptr, *v = nullptr, *A = nullptr;  // w == u == q, mask == the stamp's target v
    GrB_Semiring sr = nullptr;
    gb_desc d;                     // the SpMV's descriptor
    bool vxm = false;
    bool stamp_struct = false;     // the stamp's mask: q.S (true) or q's value (iso q)
    unsigned long long x = 0;      // the predicted stamp value (v's type, its bytes)
    gb_vec_result T;               // the speculative next q
    gb_host_slot *slot = nullptr;  // its mailbox (swapped with q's on adoption)
    uint64_t *q_bits = nullptr;    // the q the speculative kernel read (and stamped into v)
    int64_t *q_dn = nullptr;
    const void *q_iso = nullptr;   // its iso value (a value-mask stamp happens only when nonzero)
    int q_iso_code = 0;
    bool assign_matched = false;   // the host has issued the predicted stamp (absorbed)
} g_spec;

// q_iso: q's iso value when the stamp's mask was q's values (nullptr: q.S) -- an iso-false q
// stamped nothing, so there is nothing to take back
__global__ void k_spec_unstamp(int64_t nw, uint64_t *__restrict__ vbits, const uint64_t *__restrict__ qbits,
                               int64_t *__restrict__ vcount, const int64_t *__restrict__ qcount, const void *q_iso,
                               int q_iso_code) {
    if (q_iso && !gb_dyn_nonzero(q_iso, q_iso_code)) return;
    OPS_STRIDE(k, nw) {
        const uint64_t qb = qbits[k];
        if (qb) vbits[k] &= ~qb;
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) vcount[0] -= qcount[0];
}

static bool spec_int_type(int code) { return code >= GBAMD_T_INT8 && code <= GBAMD_T_UINT64; }

static unsigned long long spec_next(unsigned long long x, size_t size) {
    const unsigned long long m = size >= 8 ? ~0ULL : ((1ULL << (8 * size)) - 1);
    return (x + 1) & m;  // two's complement wrap in v's width
}

static void spec_drop_result() {
    gb_free(g_spec.T.bits);
    gb_free(g_spec.T.dense);
    gb_free(g_spec.T.d_nvals);
    g_spec.T = gb_vec_result{};
}

// undo the speculative level (g_spec_mu held); see above.  Never throws: the rollback runs on
// behalf of whichever call found the speculation in its way, so a failure of the unstamp or of
// the re-issued absorbed stamp is an execution error of v -- recorded on v (GrB_INVALID_OBJECT
// from then on, like a failed deferred assign in gb_pending_flush), not of the calling API.
static void spec_rollback_locked() {
    if (!g_spec.active) return;
    GB_Obj *q = g_spec.q, *v = g_spec.v;
    g_spec.active = false;
    g_spec_active.store(false, std::memory_order_release);
    g_stat_spec_rollbacks.fetch_add(1, std::memory_order_relaxed);
    const bool matched = g_spec.assign_matched;
    g_spec.assign_matched = false;
    auto record = [&](GrB_Info info, const std::string &msg) {
        if (v->magic != GB_MAGIC) return;
        v->invalid = info;
        v->err = "speculative BFS level rollback failed: " + msg;
    };
    try {
        const bool q_empty = q->nvals_valid && q->nvals == 0 && q->bits == g_spec.q_bits;
        if (!q_empty) {
            const int64_t nw = gb_words(v->nrows);
            hipLaunchKernelGGL(k_spec_unstamp, dim3(ops_grid(nw, 1024)), dim3(OPS_BLOCK), 0, gb_stream(), nw,
                               v->bits, g_spec.q_bits, v->d_nvals, g_spec.q_dn,
                               g_spec.stamp_struct ? nullptr : g_spec.q_iso, g_spec.q_iso_code);
            GB_LAUNCH_CHECK();
        }
        v->nvals_valid = false;
        v->hint_valid = false;
        if (matched) {
            // the host issued the predicted stamp; it was absorbed: issue it now
            // (fault injection for the tests: knob inject_spec_fail = 1)
            GB_REQUIRE(gb_knob("inject_spec_fail") != 1, GrB_OUT_OF_MEMORY, "injected failure");
            gb_desc ad;
            ad.structure = g_spec.stamp_struct;
            char xc[16] = {0};
            memcpy(xc, &g_spec.x, sizeof(g_spec.x));
            vector_assign_scalar(v, q, nullptr, xc, v->type->code, GrB_ALL, v->nrows, ad);
        }
    } catch (const gb_exception &e) {
        record(e.info, e.msg);
    } catch (const std::bad_alloc &) {
        record(GrB_OUT_OF_MEMORY, "out of host memory");
    } catch (...) {
        record(GrB_PANIC, "unknown error");
    }
    try {
        spec_drop_result();
    } catch (...) {
        // freeing goes back to the caching allocator; nothing to record
    }
}

void gb_spec_resolve(const void *keep) {
    std::lock_guard<std::mutex> lk(g_spec_mu);
    if (!g_spec.active) return;
    if (keep && OBJ(keep) != g_spec.v) return;  // a read the speculation leaves alone
    spec_rollback_locked();
}

// enqueue the level after the one just issued (g_spec_mu held): stamp v<q> = x, then
// q' = q (+).(x) A under !v.S into a result of its own
static void spec_launch_locked(GB_Obj *q, GB_Obj *v, GB_Obj *A, GrB_Semiring sr, const gb_desc &d, bool vxm,
                               unsigned long long x, bool stamp_struct) {
    gb_asg asg;
    asg.bits = v->bits;
    asg.vals = v->dense;
    asg.size = (int)v->type->size;
    asg.x = x;
    asg.q_iso = stamp_struct ? nullptr : q->dense;
    asg.q_iso_code = q->type->code;
    asg.count = v->d_nvals;
    asg.h_count = -1;
    asg.u_count_exact = true;  // q was just produced by the kernel before this one
    spmv_views V;
    spmv_build_views(V, v, sr, A, q, d, vxm, q->nrows, &asg);
    if (!V.iso_result) return;
    if (!g_spec.slot) g_spec.slot = gb_host_slot_alloc();
    gb_vec_result T;
    T.pub = g_spec.slot;
    T.pub_seq = gb_next_pub_seq(T.pub);
    gb_spmv(T, V.av, V.push, V.uv, V.m, sr, vxm, &asg);
    g_spec.T = T;
    g_spec.q = q;
    g_spec.v = v;
    g_spec.A = A;
    g_spec.sr = sr;
    g_spec.d = d;
    g_spec.vxm = vxm;
    g_spec.stamp_struct = stamp_struct;
    g_spec.x = x;
    g_spec.q_bits = q->bits;
    g_spec.q_dn = q->d_nvals;
    g_spec.q_iso = q->dense;
    g_spec.q_iso_code = q->type->code;
    g_spec.assign_matched = false;
    g_spec.active = true;
    g_spec_active.store(true, std::memory_order_release);
}

static bool same_desc(const gb_desc &a, const gb_desc &b) {
    return a.replace == b.replace && a.comp == b.comp && a.structure == b.structure && a.tran0 == b.tran0 &&
           a.tran1 == b.tran1;
}

// after a level whose stamp was fused (do_spmv): speculate the next one when the call has the
// notebook loop's shape
static void spec_after_level(GB_Obj *w, GB_Obj *mask, GrB_BinaryOp accum, GrB_Semiring sr, GB_Obj *A, GB_Obj *u,
                             const gb_desc &d, bool vxm, const gb_asg &asg, bool direct, bool published) {
    if (gb_knob("bfs_spec") == 1 || (gb_knob("iso_dbg") & ~(128 | 512)) != 0) return;  // 128, 512: A/B orders, exact
    if (!direct || !published || accum || w != u || !mask || !d.replace || !d.comp || !d.structure) return;
    if (w->kind == GB_KIND_MATRIX || mask->kind == GB_KIND_MATRIX || A->kind != GB_KIND_MATRIX || A->cw) return;
    if (!spec_int_type(mask->type->code) || asg.bits != mask->bits || asg.vals != mask->dense) return;
    std::lock_guard<std::mutex> lk(g_spec_mu);
    if (g_spec.active) spec_rollback_locked();  // cannot happen (do_spmv adopted or rolled back)
    try {
        spec_launch_locked(w, mask, A, sr, d, vxm, spec_next(asg.x, mask->type->size), asg.q_iso == nullptr);
    } catch (...) {
        // a speculation that could not be set up is simply not made (the level itself is done);
        // if its kernel did run, undo it like any other
        if (g_spec.active) spec_rollback_locked();
        return;
    }
    // the level's own count stays readable from its mailbox: the speculative launch does not touch w
    if (w->pub_seq) w->pub_epoch = gb_epoch();
}

// the host issues `w<mask> = x` (all indices, no accum): absorbed when it is the predicted stamp
// Absorbs only what the normal path would carry out without error: GrB_ALL with ni == n, a
// valid (not execution-failed) target and mask; anything else rolls back and takes gb_api.
static bool spec_match_assign(GB_Obj *w, GB_Obj *mask, GrB_BinaryOp accum, const void *x, int xcode,
                              const GrB_Index *I, int64_t ni, GrB_Descriptor desc) {
    std::lock_guard<std::mutex> lk(g_spec_mu);
    if (!g_spec.active) return false;
    bool ok = !g_spec.assign_matched && w == g_spec.v && mask == g_spec.q && !accum && I == GrB_ALL &&
              !g_pending_active.load(std::memory_order_acquire) && w->magic == GB_MAGIC &&
              ni == w->nrows && w->invalid == GrB_SUCCESS && mask && mask->magic == GB_MAGIC &&
              mask->invalid == GrB_SUCCESS;
    if (ok) {
        gb_desc ad;
        try {
            ad = gb_read_desc(desc);
        } catch (...) {
            ok = false;
        }
        ok = ok && !ad.replace && !ad.comp && ad.structure == g_spec.stamp_struct && !ad.tran0 && !ad.tran1;
    }
    if (ok) {
        unsigned long long xv = 0;
        gb_with_type(w->type->code, [&](auto z) {
            using D = decltype(z);
            gb_with_type(xcode, [&](auto y) {
                using S = decltype(y);
                S sv;
                memcpy(&sv, x, sizeof(S));
                D dv = gb_cast<D, S>(sv);
                memcpy(&xv, &dv, sizeof(D));
            });
        });
        ok = xv == g_spec.x;
    }
    if (!ok) {
        spec_rollback_locked();
        return false;
    }
    g_spec.assign_matched = true;
    w->err.clear();
    w->nvals_valid = false;
    w->hint_valid = false;
    return true;
}

// the host issues the predicted SpMV: install the speculative result and speculate again
static bool spec_try_adopt(GB_Obj *w, GB_Obj *mask, GrB_BinaryOp accum, GrB_Semiring sr, GB_Obj *A, GB_Obj *u,
                           const gb_desc &d, bool vxm) {
    std::lock_guard<std::mutex> lk(g_spec_mu);
    if (!g_spec.active) return false;
    const bool ok = g_spec.assign_matched && w == g_spec.q && u == g_spec.q && mask == g_spec.v && A == g_spec.A &&
                    sr == g_spec.sr && !accum && vxm == g_spec.vxm && same_desc(d, g_spec.d) &&
                    w->bits == g_spec.q_bits && g_spec.T.published && gb_knob("bfs_spec") != 1 &&
                    !g_pending_active.load(std::memory_order_acquire);
    if (!ok) {
        spec_rollback_locked();
        return false;
    }
    GB_Obj *q = w, *v = mask;
    gb_vec_result T = g_spec.T;
    g_spec.T = gb_vec_result{};
    g_spec.active = false;
    g_spec_active.store(false, std::memory_order_release);
    g_stat_spec_adopted.fetch_add(1, std::memory_order_relaxed);
    std::swap(q->pub, g_spec.slot);  // the result's mailbox becomes q's; q's old one, the next speculation's
    const void *hk = T.hint_key;
    const uint64_t seq = T.pub_seq;
    gb_writeback_vector(q, T, v, d, nullptr, true);  // replace, T within the mask: installed as is
    q->pub_seq = seq;
    q->hint_valid = hk != nullptr;
    q->hint_key = hk;
    v->nvals_valid = false;
    v->hint_valid = false;
    try {
        spec_launch_locked(q, v, A, sr, d, vxm, spec_next(g_spec.x, v->type->size), g_spec.stamp_struct);
    } catch (...) {
        if (g_spec.active) spec_rollback_locked();
    }
    q->pub_epoch = gb_epoch();
    return true;
}

static void vector_assign_scalar(GB_Obj *w, GB_Obj *mask, GrB_BinaryOp accum, const void *x, int xcode,
                                 const GrB_Index *I, int64_t ni, const gb_desc &d) {
    check_binop(accum, true);
    GB_REQUIRE(w->kind != GB_KIND_MATRIX || w->ncols == 1, GrB_DIMENSION_MISMATCH, "not a vector");
    int ct = w->type->code;
    // cast the scalar to C's type on the host
    char xc[16];
    gb_with_type(ct, [&](auto z) {
        using D = decltype(z);
        gb_with_type(xcode, [&](auto y) {
            using S = decltype(y);
            S sv;
            memcpy(&sv, x, sizeof(S));
            D dv = gb_cast<D, S>(sv);
            memcpy(xc, &dv, sizeof(D));
        });
    });
    // a pending root stays pending only under the deferred stamp whose mask it is (gb_internal.h)
    if (g_root_active.load(std::memory_order_acquire) &&
        !(I == GrB_ALL && !accum && mask && gb_root_pending(mask) && !gb_root_pending(w)))
        gb_root_flush();
    if (I == GrB_ALL && !accum && try_defer_assign(w, mask, xc, d)) return;
    if (g_root_active.load(std::memory_order_acquire)) gb_root_flush();  // not deferred: the assign reads it
    if (I == GrB_ALL && !accum && assign_all_scalar_fast(w, mask, xc, d)) return;
    gb_vec_result T;
    scalar_vec_T(T, w->nrows, I, ni, xc, ct);
    GrB_BinaryOp acc = accum;
    if (I != GrB_ALL && !acc) acc = second_of(ct);  // outside I, C is kept
    gb_writeback_vector(w, T, mask, d, acc, false);
}

static void matrix_assign_scalar(GB_Obj *C, GB_Obj *M, GrB_BinaryOp accum, const void *x, int xcode,
                                 const GrB_Index *I, int64_t ni, const GrB_Index *J, int64_t nj, const gb_desc &d) {
    check_binop(accum, true);
    int ct = C->type->code;
    char xc[16];
    gb_with_type(ct, [&](auto z) {
        using D = decltype(z);
        gb_with_type(xcode, [&](auto y) {
            using S = decltype(y);
            S sv;
            memcpy(&sv, x, sizeof(S));
            D dv = gb_cast<D, S>(sv);
            memcpy(xc, &dv, sizeof(D));
        });
    });
    int64_t nr = C->nrows, nc = ncols_of(C);
    gb_index_list LI, LJ;
    gb_expand_indices(LI, I, (GrB_Index)ni, nr);
    gb_expand_indices(LJ, J, (GrB_Index)nj, nc);
    std::vector<int64_t> rows, cols;
    if (LI.all) {
        rows.resize(nr);
        for (int64_t i = 0; i < nr; i++) rows[i] = i;
    } else rows = LI.idx;
    if (LJ.all) {
        cols.resize(nc);
        for (int64_t j = 0; j < nc; j++) cols[j] = j;
    } else cols = LJ.idx;
    std::sort(rows.begin(), rows.end());
    rows.erase(std::unique(rows.begin(), rows.end()), rows.end());
    std::sort(cols.begin(), cols.end());
    cols.erase(std::unique(cols.begin(), cols.end()), cols.end());
    int64_t nz = (int64_t)rows.size() * (int64_t)cols.size();
    std::vector<int64_t> rp(nr + 1, 0);
    for (auto r : rows) rp[r + 1] = (int64_t)cols.size();
    for (int64_t i = 0; i < nr; i++) rp[i + 1] += rp[i];
    std::vector<int32_t> ci(nz);
    for (size_t a = 0; a < rows.size(); a++)
        for (size_t b = 0; b < cols.size(); b++) ci[a * cols.size() + b] = (int32_t)cols[b];
    gb_mat_result T;
    T.nrows = nr;
    T.ncols = nc;
    T.nvals = nz;
    T.tcode = ct;
    T.iso = true;
    T.rowptr = gb_malloc_n<int64_t>(nr + 1);
    T.colidx = gb_malloc_n<int32_t>(nz);
    T.vals = gb_malloc(gb_type_size(ct));
    gb_copy_h2d(T.rowptr, rp.data(), (nr + 1) * sizeof(int64_t));
    gb_copy_h2d(T.colidx, ci.data(), nz * sizeof(int32_t));
    gb_copy_h2d(T.vals, xc, gb_type_size(ct));
    gb_sync();
    GrB_BinaryOp acc = accum;
    if ((I != GrB_ALL || J != GrB_ALL) && !acc) acc = second_of(ct);
    gb_writeback_matrix(C, T, M, d, acc);
}

// ================================================================== C API
// ================================================================== apply
// z = op(x) (kind 0), op(s, x) (kind 1, BinaryOp1st), op(x, s) (kind 2, BinaryOp2nd)
// over the n stored values (n = 1 for iso inputs): structure is not touched.
template <class X, class Z>
__global__ void k_apply(int64_t n, int kind, int op, const X *__restrict__ in, X s, Z *__restrict__ out) {
    OPS_STRIDE(i, n) {
        X x = in[i];
        if (kind == 0) out[i] = gb_cast<Z, X>(gb_unop<X>(op, x));
        else if (kind == 1) out[i] = gb_binop_z<X, Z>(op, s, x, 0, 0, 0);
        else out[i] = gb_binop_z<X, Z>(op, x, s, 0, 0, 0);
    }
}

// kind 0: uop; kind 1/2: bop with the bound scalar *sval (type scode)
static void do_apply(GB_Obj *C, GB_Obj *M, GrB_BinaryOp accum, int kind, GrB_UnaryOp uop, GrB_BinaryOp bop,
                     const void *sval, int scode, GB_Obj *A, const gb_desc &d) {
    check_binop(accum, true);
    int xcode, zcode, opcode;
    if (kind == 0) {
        GB_REQUIRE(uop, GrB_NULL_POINTER, "operator is NULL");
        GB_REQUIRE(uop->magic == GB_MAGIC, GrB_UNINITIALIZED_OBJECT, "invalid operator");
        xcode = uop->xtype->code;
        zcode = uop->ztype->code;
        opcode = uop->opcode;
    } else {
        check_binop(bop, false);
        GB_REQUIRE(bop->xtype != nullptr, GrB_NOT_IMPLEMENTED, "positional operator in apply");
        xcode = bop->xtype->code;
        zcode = bop->ztype->code;
        opcode = bop->opcode;
    }
    // the bound scalar, cast to the operator's input type
    char sx[16] = {0};
    if (kind != 0) {
        gb_with_type(scode, [&](auto sv) {
            using S = decltype(sv);
            S v;
            memcpy(&v, sval, sizeof(S));
            gb_with_type(xcode, [&](auto xv) {
                using X = decltype(xv);
                X c = gb_cast<X, S>(v);
                memcpy(sx, &c, sizeof(X));
            });
        });
    }
    auto launch = [&](int64_t n, const void *in, void *out) {
        dispatch_xz(xcode, zcode, [&](auto x, auto z) {
            using X = decltype(x);
            using Z = decltype(z);
            X s;
            memcpy(&s, sx, sizeof(X));
            if (n)
                hipLaunchKernelGGL((k_apply<X, Z>), dim3(ops_grid(n)), dim3(OPS_BLOCK), 0, gb_stream(), n, kind,
                                   opcode, (const X *)in, s, (Z *)out);
        });
        GB_LAUNCH_CHECK();
    };
    const size_t zs = gb_type_size(zcode);
    if (C->kind != GB_KIND_MATRIX) {
        GB_REQUIRE(A->nrows == C->nrows && ncols_of(A) == 1, GrB_DIMENSION_MISMATCH, "vector sizes do not match");
        gb_bitmap_view uv;
        gb_get_bitmap(uv, A);
        gb_scratch s;
        const void *xin = gb_bitmap_vals_as(uv, xcode, s);
        gb_vec_result T;
        T.n = uv.n;
        T.tcode = zcode;
        T.iso = uv.iso;
        const int64_t nw = gb_words(uv.n);
        T.bits = gb_malloc_n<uint64_t>(std::max<int64_t>(nw, 1));
        if (nw) gb_copy_d2d(T.bits, uv.bits, nw * sizeof(uint64_t));
        const int64_t nv = uv.iso ? 1 : uv.n;
        T.dense = gb_malloc(std::max<int64_t>(nv, 1) * zs);
        launch(nv, xin, T.dense);
        T.d_nvals = gb_malloc_n<int64_t>(1);
        if (uv.count) gb_copy_d2d(T.d_nvals, uv.count, sizeof(int64_t));
        else gb_bitmap_count(T.bits, T.n, T.d_nvals);
        gb_writeback_vector(C, T, M, d, accum, false);
        return;
    }
    gb_csr_view v;
    if (d.tran0) gb_get_csc(v, A);
    else gb_get_csr(v, A);
    GB_REQUIRE(v.nrows == C->nrows && v.ncols == C->ncols, GrB_DIMENSION_MISMATCH, "matrix dimensions do not match");
    gb_scratch s;
    const void *xin = gb_view_vals_as(v, xcode, s);
    gb_mat_result T;
    T.nrows = v.nrows;
    T.ncols = v.ncols;
    T.nvals = v.nvals;
    T.tcode = zcode;
    T.iso = v.iso;
    T.rowptr = gb_malloc_n<int64_t>(v.nrows + 1);
    gb_copy_d2d(T.rowptr, v.rowptr, (v.nrows + 1) * sizeof(int64_t));
    T.colidx = gb_malloc_n<int32_t>(std::max<int64_t>(v.nvals, 1));
    if (v.nvals) gb_copy_d2d(T.colidx, v.colidx, v.nvals * sizeof(int32_t));
    const int64_t nv = v.iso ? (v.nvals ? 1 : 0) : v.nvals;
    T.vals = gb_malloc(std::max<int64_t>(nv, 1) * zs);
    launch(nv, xin, T.vals);
    gb_writeback_matrix(C, T, M, d, accum);
}

// ================================================================== reduce to vector
static GrB_BinaryOp first_of(int code) {
    void *h;
    int kind;
    std::string name = std::string("GrB_FIRST_") + gb_type_name(code);
    GxB_builtin_lookup(&h, &kind, name.c_str());
    return (GrB_BinaryOp)h;
}

static void do_reduce_rows(GB_Obj *w, GB_Obj *mask, GrB_BinaryOp accum, GrB_Monoid monoid, GB_Obj *A,
                           const gb_desc &d) {
    GB_REQUIRE(monoid, GrB_NULL_POINTER, "monoid is NULL");
    GB_REQUIRE(monoid->magic == GB_MAGIC, GrB_UNINITIALIZED_OBJECT, "invalid monoid");
    GB_REQUIRE(A->kind == GB_KIND_MATRIX, GrB_INVALID_OBJECT, "reduce input must be a matrix");
    const int code = monoid->type->code;
    // w = A' (monoid.FIRST) ones: the product is A'(i,k); the iso-full vector only supplies structure
    GB_Semiring_opaque sr{GB_MAGIC, monoid, first_of(code), "reduce", false};
    const int64_t k = d.tran0 ? A->nrows : A->ncols;
    GrB_Vector u = nullptr;
    GrB_Info info = GrB_Vector_new(&u, monoid->type, (GrB_Index)k);
    GB_REQUIRE(info == GrB_SUCCESS, info, "cannot allocate the reduction vector");
    struct Free {
        GrB_Vector *u;
        ~Free() { GrB_Vector_free(u); }
    } fr{&u};
    char one[16] = {0};
    gb_with_type(code, [&](auto z) {
        using Z = decltype(z);
        Z v = (Z)1;
        memcpy(one, &v, sizeof(Z));
    });
    vector_assign_scalar(OBJ(u), nullptr, nullptr, one, code, GrB_ALL, k, gb_desc());
    gb_desc dd = d;
    dd.tran1 = false;
    do_spmv(w, mask, accum, &sr, A, OBJ(u), dd, false);
}

static GrB_Monoid monoid_of_binop(GrB_BinaryOp op) {
    check_binop(op, false);
    GB_REQUIRE(op->xtype != nullptr && op->xtype == op->ztype, GrB_DOMAIN_MISMATCH,
               "reduce requires a BinaryOp that is a monoid");
    static const struct {
        int opcode;
        const char *pre, *mid;
    } tab[] = {{GBAMD_OP_PLUS, "GrB_PLUS_MONOID_", nullptr},   {GBAMD_OP_TIMES, "GrB_TIMES_MONOID_", nullptr},
               {GBAMD_OP_MIN, "GrB_MIN_MONOID_", nullptr},     {GBAMD_OP_MAX, "GrB_MAX_MONOID_", nullptr},
               {GBAMD_OP_ANY, "GxB_ANY_", "_MONOID"},          {GBAMD_OP_LOR, "GrB_LOR_MONOID_", nullptr},
               {GBAMD_OP_LAND, "GrB_LAND_MONOID_", nullptr},   {GBAMD_OP_LXOR, "GrB_LXOR_MONOID_", nullptr},
               {GBAMD_OP_LXNOR, "GrB_LXNOR_MONOID_", nullptr}, {GBAMD_OP_BOR, "GxB_BOR_", "_MONOID"},
               {GBAMD_OP_BAND, "GxB_BAND_", "_MONOID"},        {GBAMD_OP_BXOR, "GxB_BXOR_", "_MONOID"},
               {GBAMD_OP_BXNOR, "GxB_BXNOR_", "_MONOID"}};
    for (auto &t : tab) {
        if (t.opcode != op->opcode) continue;
        std::string name = std::string(t.pre) + gb_type_name(op->ztype->code) + (t.mid ? t.mid : "");
        void *h = nullptr;
        int kind = -1;
        if (GxB_builtin_lookup(&h, &kind, name.c_str()) == GrB_SUCCESS && kind == 2) return (GrB_Monoid)h;
    }
    gb_throw(GrB_DOMAIN_MISMATCH, "reduce requires a BinaryOp that is a monoid");
    return nullptr;
}

extern "C" {

GrB_Info GrB_mxm(GrB_Matrix C, const GrB_Matrix Mask, const GrB_BinaryOp accum, const GrB_Semiring op,
                 const GrB_Matrix A, const GrB_Matrix B, const GrB_Descriptor desc) {
    return gb_api(OBJ(C), [&] {
        const gb_desc d = gb_read_desc(desc);
        if (gb_colbits_mxm(gb_obj_check_raw(C), gb_obj_check_raw(Mask, true), accum, op, gb_obj_check_raw(A),
                           gb_obj_check_raw(B), d))
            return;
        do_mxm(gb_obj_check(C), gb_obj_check(Mask, true), accum, op, gb_obj_check(A), gb_obj_check(B), d);
    });
}

GrB_Info GrB_mxv(GrB_Vector w, const GrB_Vector mask, const GrB_BinaryOp accum, const GrB_Semiring op,
                 const GrB_Matrix A, const GrB_Vector u, const GrB_Descriptor desc) {
    return gb_api_keep_pending(OBJ(w), [&] {
        do_spmv(gb_obj_check(w), gb_obj_check(mask, true), accum, op, gb_obj_check(A), gb_obj_check(u),
                gb_read_desc(desc), false);
    });
}

GrB_Info GrB_vxm(GrB_Vector w, const GrB_Vector mask, const GrB_BinaryOp accum, const GrB_Semiring op,
                 const GrB_Vector u, const GrB_Matrix A, const GrB_Descriptor desc) {
    GB_HPROF(0, "GrB_vxm total");
    return gb_api_keep_pending(OBJ(w), [&] {
        do_spmv(gb_obj_check(w), gb_obj_check(mask, true), accum, op, gb_obj_check(A), gb_obj_check(u),
                gb_read_desc(desc), true);
    });
}

GrB_Info GrB_Matrix_eWiseMult_BinaryOp(GrB_Matrix C, const GrB_Matrix Mask, const GrB_BinaryOp accum,
                                       const GrB_BinaryOp op, const GrB_Matrix A, const GrB_Matrix B,
                                       const GrB_Descriptor desc) {
    return gb_api(OBJ(C), [&] {
        do_ewise(gb_obj_check(C), gb_obj_check(Mask, true), accum, op, gb_obj_check(A), gb_obj_check(B),
                 gb_read_desc(desc), false);
    });
}
GrB_Info GrB_Vector_eWiseMult_BinaryOp(GrB_Vector w, const GrB_Vector mask, const GrB_BinaryOp accum,
                                       const GrB_BinaryOp op, const GrB_Vector u, const GrB_Vector v,
                                       const GrB_Descriptor desc) {
    return gb_api(OBJ(w), [&] {
        do_ewise(gb_obj_check(w), gb_obj_check(mask, true), accum, op, gb_obj_check(u), gb_obj_check(v),
                 gb_read_desc(desc), false);
    });
}
GrB_Info GrB_Matrix_eWiseAdd_BinaryOp(GrB_Matrix C, const GrB_Matrix Mask, const GrB_BinaryOp accum,
                                      const GrB_BinaryOp op, const GrB_Matrix A, const GrB_Matrix B,
                                      const GrB_Descriptor desc) {
    return gb_api(OBJ(C), [&] {
        do_ewise(gb_obj_check(C), gb_obj_check(Mask, true), accum, op, gb_obj_check(A), gb_obj_check(B),
                 gb_read_desc(desc), true);
    });
}
GrB_Info GrB_Vector_eWiseAdd_BinaryOp(GrB_Vector w, const GrB_Vector mask, const GrB_BinaryOp accum,
                                      const GrB_BinaryOp op, const GrB_Vector u, const GrB_Vector v,
                                      const GrB_Descriptor desc) {
    return gb_api(OBJ(w), [&] {
        do_ewise(gb_obj_check(w), gb_obj_check(mask, true), accum, op, gb_obj_check(u), gb_obj_check(v),
                 gb_read_desc(desc), true);
    });
}

GrB_Info GrB_transpose(GrB_Matrix C, const GrB_Matrix Mask, const GrB_BinaryOp accum, const GrB_Matrix A,
                       const GrB_Descriptor desc) {
    return gb_api(OBJ(C), [&] {
        do_transpose(gb_obj_check(C), gb_obj_check(Mask, true), accum, gb_obj_check(A), gb_read_desc(desc));
    });
}

// w(I) = u without accum replaces the region: entries of w at I (where the mask selects)
// that u does not hold are deleted.  Clears those bits before the merge with accum SECOND.
__global__ void k_clear_region(int64_t nw, uint64_t *__restrict__ wbits, const uint64_t *__restrict__ rbits,
                               const uint64_t *__restrict__ mbits, bool mcomp) {
    OPS_STRIDE(k, nw) {
        uint64_t sel = mbits ? (mcomp ? ~mbits[k] : mbits[k]) : ~0ULL;
        wbits[k] &= ~(rbits[k] & sel);
    }
}

static void vector_clear_region(GB_Obj *W, const gb_index_list &L, GB_Obj *M, const gb_desc &d) {
    const int64_t n = W->nrows, nw = gb_words(n);
    GB_REQUIRE(W->kind != GB_KIND_MATRIX, GrB_NOT_IMPLEMENTED, "index-list assign into an n x 1 matrix");
    if (nw == 0) return;
    std::vector<uint64_t> hr(nw, 0);
    for (int64_t i : L.idx) hr[i >> 6] |= 1ULL << (i & 63);
    gb_scratch s;
    uint64_t *r = s.get<uint64_t>(nw);
    gb_copy_h2d(r, hr.data(), nw * sizeof(uint64_t));
    gb_vmask m;
    gb_make_vmask(m, M, d, n);
    hipLaunchKernelGGL(k_clear_region, dim3(ops_grid(nw)), dim3(OPS_BLOCK), 0, gb_stream(), nw, W->bits, r, m.bits,
                       m.comp);
    GB_LAUNCH_CHECK();
    gb_vec_recount(W);
    gb_sync();
}

GrB_Info GrB_Vector_assign(GrB_Vector w, const GrB_Vector mask, const GrB_BinaryOp accum, const GrB_Vector u,
                           const GrB_Index *I, GrB_Index ni, const GrB_Descriptor desc) {
    return gb_api(OBJ(w), [&] {
        GB_Obj *W = gb_obj_check(w), *U = gb_obj_check(u);
        gb_desc d = gb_read_desc(desc);
        check_binop(accum, true);
        int64_t n = W->nrows;
        gb_vec_result T;
        T.n = n;
        T.tcode = U->type->code;
        if (I == GrB_ALL) {
            GB_REQUIRE(U->nrows == n, GrB_DIMENSION_MISMATCH, "u size does not match w");
            gb_bitmap_view uv;
            gb_get_bitmap(uv, U);
            T.iso = uv.iso;
            T.bits = gb_malloc_n<uint64_t>(gb_words(n));
            gb_copy_d2d(T.bits, uv.bits, gb_words(n) * sizeof(uint64_t));
            size_t ts = gb_type_size(uv.tcode);
            T.dense = gb_malloc((uv.iso ? 1 : n) * ts);
            gb_copy_d2d(T.dense, uv.vals, (uv.iso ? 1 : n) * ts);
            T.d_nvals = gb_malloc_n<int64_t>(1);
            gb_bitmap_count(T.bits, n, T.d_nvals);
            gb_writeback_vector(W, T, gb_obj_check(mask, true), d, accum, false);
            return;
        }
        // index list: w(I[k]) = u(k)
        gb_index_list L;
        gb_expand_indices(L, I, ni, n);
        GB_REQUIRE(U->nrows == L.n, GrB_DIMENSION_MISMATCH, "u size does not match the index list");
        int64_t unv = gb_nvals(U);
        std::vector<GrB_Index> ui(unv);
        std::vector<char> ux(unv * U->type->size);
        {
            GrB_Index nv = unv;
            gb_extract_tuples(U, ui.data(), nullptr, ux.data(), U->type->code, &nv);
        }
        GB_Obj *Tv = gb_new_object(GB_KIND_VECTOR, U->type, n, 1);
        std::vector<GrB_Index> wi(unv);
        for (int64_t q = 0; q < unv; q++) {
            GB_REQUIRE(ui[q] < (GrB_Index)L.n, GrB_INDEX_OUT_OF_BOUNDS, "index out of bounds");
            wi[q] = (GrB_Index)L.idx[ui[q]];
        }
        try {
            gb_build(Tv, wi.data(), nullptr, ux.data(), U->type->code, false, unv, nullptr);
        } catch (...) {
            GrB_Vector tv = (GrB_Vector)Tv;
            GrB_Vector_free(&tv);
            throw;
        }
        gb_bitmap_view tvw;
        gb_get_bitmap(tvw, Tv);
        T.iso = tvw.iso;
        T.bits = gb_malloc_n<uint64_t>(gb_words(n));
        gb_copy_d2d(T.bits, tvw.bits, gb_words(n) * sizeof(uint64_t));
        size_t ts = gb_type_size(tvw.tcode);
        T.dense = gb_malloc((tvw.iso ? 1 : n) * ts);
        gb_copy_d2d(T.dense, tvw.vals, (tvw.iso ? 1 : n) * ts);
        T.d_nvals = gb_malloc_n<int64_t>(1);
        gb_bitmap_count(T.bits, n, T.d_nvals);
        GrB_Vector tv = (GrB_Vector)Tv;
        GrB_Vector_free(&tv);
        GB_Obj *Mo = gb_obj_check(mask, true);
        // w(w.S)[I] = u / w(w.V)[I] = u: the region clear below edits w's bitmap, which IS the
        // mask; the writeback must see the mask as it was before the clear, so take a copy
        struct mask_copy {
            GrB_Vector h = nullptr;
            ~mask_copy() { if (h) GrB_Vector_free(&h); }
        } mc;
        if (!accum && Mo == W) {
            GB_REQUIRE(GrB_Vector_dup(&mc.h, mask) == GrB_SUCCESS, GrB_OUT_OF_MEMORY, "mask copy");
            Mo = gb_obj_check(mc.h);
        }
        if (!accum) vector_clear_region(W, L, Mo, d);
        gb_writeback_vector(W, T, Mo, d, accum ? accum : second_of(W->type->code), false);
    });
}

GrB_Info GrB_Matrix_assign(GrB_Matrix C, const GrB_Matrix Mask, const GrB_BinaryOp accum, const GrB_Matrix A,
                           const GrB_Index *I, GrB_Index ni, const GrB_Index *J, GrB_Index nj,
                           const GrB_Descriptor desc) {
    return gb_api(OBJ(C), [&] {
        GB_Obj *Co = gb_obj_check(C), *Ao = gb_obj_check(A);
        gb_desc d = gb_read_desc(desc);
        GB_REQUIRE(I == GrB_ALL && J == GrB_ALL, GrB_NOT_IMPLEMENTED, "Matrix_assign supports GrB_ALL only");
        gb_csr_view v;
        if (d.tran0) gb_get_csc(v, Ao);
        else gb_get_csr(v, Ao);
        GB_REQUIRE(v.nrows == Co->nrows && v.ncols == ncols_of(Co), GrB_DIMENSION_MISMATCH, "dimension mismatch");
        gb_mat_result T;
        T.nrows = v.nrows;
        T.ncols = v.ncols;
        T.nvals = v.nvals;
        T.tcode = v.tcode;
        T.iso = v.iso;
        size_t ts = gb_type_size(v.tcode);
        T.rowptr = gb_malloc_n<int64_t>(v.nrows + 1);
        gb_copy_d2d(T.rowptr, v.rowptr, (v.nrows + 1) * sizeof(int64_t));
        T.colidx = gb_malloc_n<int32_t>(v.nvals);
        gb_copy_d2d(T.colidx, v.colidx, v.nvals * sizeof(int32_t));
        T.vals = gb_malloc((v.iso ? 1 : v.nvals) * ts);
        gb_copy_d2d(T.vals, v.vals, (v.iso ? 1 : v.nvals) * ts);
        gb_writeback_matrix(Co, T, gb_obj_check(Mask, true), d, accum);
    });
}

GrB_Info GrB_Matrix_reduce_Monoid_Scalar(GrB_Scalar s, const GrB_BinaryOp accum, const GrB_Monoid monoid,
                                         const GrB_Matrix A, const GrB_Descriptor desc) {
    (void)desc;
    return gb_api(OBJ(s), [&] {
        GB_Obj *S = gb_obj_check(s);
        char v[16];
        bool any = reduce_values(gb_obj_check(A), monoid, v);
        gb_vec_result T;
        T.n = 1;
        T.tcode = monoid->type->code;
        T.iso = true;
        T.bits = gb_malloc_n<uint64_t>(1);
        uint64_t b = any ? 1 : 0;
        gb_copy_h2d(T.bits, &b, sizeof(b));
        T.dense = gb_malloc(16);
        gb_copy_h2d(T.dense, v, gb_type_size(T.tcode));
        T.d_nvals = gb_malloc_n<int64_t>(1);
        int64_t nn = any ? 1 : 0;
        gb_copy_h2d(T.d_nvals, &nn, sizeof(nn));
        gb_sync();
        gb_writeback_vector(S, T, nullptr, gb_desc(), accum, false);
    });
}
GrB_Info GrB_Vector_reduce_Monoid_Scalar(GrB_Scalar s, const GrB_BinaryOp accum, const GrB_Monoid monoid,
                                         const GrB_Vector u, const GrB_Descriptor desc) {
    return GrB_Matrix_reduce_Monoid_Scalar(s, accum, monoid, (GrB_Matrix)u, desc);
}
GrB_Info GrB_Matrix_reduce_Monoid(GrB_Vector w, const GrB_Vector mask, const GrB_BinaryOp accum,
                                  const GrB_Monoid monoid, const GrB_Matrix A, const GrB_Descriptor desc) {
    return gb_api(OBJ(w), [&] {
        do_reduce_rows(gb_obj_check(w), gb_obj_check(mask, true), accum, monoid, gb_obj_check(A),
                       gb_read_desc(desc));
    });
}
GrB_Info GrB_Matrix_reduce_BinaryOp(GrB_Vector w, const GrB_Vector mask, const GrB_BinaryOp accum,
                                    const GrB_BinaryOp op, const GrB_Matrix A, const GrB_Descriptor desc) {
    return gb_api(OBJ(w), [&] {
        do_reduce_rows(gb_obj_check(w), gb_obj_check(mask, true), accum, monoid_of_binop(op), gb_obj_check(A),
                       gb_read_desc(desc));
    });
}
GrB_Info GrB_Vector_apply(GrB_Vector w, const GrB_Vector mask, const GrB_BinaryOp accum, const GrB_UnaryOp op,
                          const GrB_Vector u, const GrB_Descriptor desc) {
    return gb_api(OBJ(w), [&] {
        do_apply(gb_obj_check(w), gb_obj_check(mask, true), accum, 0, op, nullptr, nullptr, 0, gb_obj_check(u),
                 gb_read_desc(desc));
    });
}
GrB_Info GrB_Matrix_apply(GrB_Matrix C, const GrB_Matrix Mask, const GrB_BinaryOp accum, const GrB_UnaryOp op,
                          const GrB_Matrix A, const GrB_Descriptor desc) {
    return gb_api(OBJ(C), [&] {
        do_apply(gb_obj_check(C), gb_obj_check(Mask, true), accum, 0, op, nullptr, nullptr, 0, gb_obj_check(A),
                 gb_read_desc(desc));
    });
}
GrB_Info GrB_Semiring_new(GrB_Semiring *semiring, GrB_Monoid add, GrB_BinaryOp multiply) {
    if (!semiring || !add || !multiply) return GrB_NULL_POINTER;
    if (add->magic != GB_MAGIC || multiply->magic != GB_MAGIC) return GrB_UNINITIALIZED_OBJECT;
    if (multiply->ztype != add->type) return GrB_DOMAIN_MISMATCH;
    GB_Semiring_opaque *s = new (std::nothrow) GB_Semiring_opaque{GB_MAGIC, add, multiply, "user_semiring", true};
    if (!s) return GrB_OUT_OF_MEMORY;
    *semiring = s;
    return GrB_SUCCESS;
}

#define GB_DEFINE_TYPED_OPS(T, ctype)                                                                          \
    GrB_Info GrB_Vector_assign_##T(GrB_Vector w, const GrB_Vector mask, const GrB_BinaryOp accum, ctype x,   \
                                   const GrB_Index *I, GrB_Index ni, const GrB_Descriptor desc) {            \
        GB_HPROF(8, "GrB_Vector_assign scalar");                                                             \
        gb_root_hold_guard root_hold; /* a deferred stamp whose mask is a pending root keeps it pending */   \
        if (g_spec_active.load(std::memory_order_acquire) && w && OBJ(w)->magic == GB_MAGIC) {             \
            /* the predicted level stamp, already carried out (BFS speculation); the match runs   \
               inside the API wrapper so that nothing it raises crosses the C boundary */          \
            bool absorbed = false;                                                                           \
            const GrB_Info mi = gb_api_impl<false>(OBJ(w), [&] {                                             \
                absorbed = spec_match_assign(OBJ(w), mask ? OBJ(mask) : nullptr, accum, &x, GBAMD_T_##T, I, \
                                             (int64_t)ni, desc);                                             \
            });                                                                                              \
            if (mi != GrB_SUCCESS) return mi;                                                                \
            if (absorbed) return GrB_SUCCESS;                                                                \
        }                                                                                                    \
        return gb_api(OBJ(w), [&] {                                                                          \
            vector_assign_scalar(gb_obj_check(w), gb_obj_check(mask, true), accum, &x, GBAMD_T_##T, I,       \
                                 (int64_t)ni, gb_read_desc(desc));                                           \
        });                                                                                                  \
    }                                                                                                        \
    GrB_Info GrB_Matrix_assign_##T(GrB_Matrix C, const GrB_Matrix Mask, const GrB_BinaryOp accum, ctype x,   \
                                   const GrB_Index *I, GrB_Index ni, const GrB_Index *J, GrB_Index nj,       \
                                   const GrB_Descriptor desc) {                                              \
        return gb_api(OBJ(C), [&] {                                                                          \
            const gb_desc d = gb_read_desc(desc);                                                            \
            if (gb_colbits_assign_scalar(gb_obj_check_raw(C), gb_obj_check_raw(Mask, true), accum, &x,       \
                                         GBAMD_T_##T, I, J, d))                                              \
                return;                                                                                      \
            GB_Obj *Co = gb_obj_check(C);                                                                    \
            if (Co->kind != GB_KIND_MATRIX)                                                                  \
                vector_assign_scalar(Co, gb_obj_check(Mask, true), accum, &x, GBAMD_T_##T, I, (int64_t)ni,   \
                                     gb_read_desc(desc));                                                    \
            else                                                                                             \
                matrix_assign_scalar(Co, gb_obj_check(Mask, true), accum, &x, GBAMD_T_##T, I, (int64_t)ni, J, \
                                     (int64_t)nj, gb_read_desc(desc));                                       \
        });                                                                                                  \
    }                                                                                                        \
    GrB_Info GrB_Vector_reduce_##T(ctype *c, const GrB_BinaryOp accum, const GrB_Monoid monoid,              \
                                   const GrB_Vector u, const GrB_Descriptor desc) {                          \
        (void)desc;                                                                                          \
        if (!c) return GrB_NULL_POINTER;                                                                     \
        return gb_api(OBJ(u), [&] {                                                                          \
            char v[16];                                                                                      \
            GB_REQUIRE(monoid && monoid->magic == GB_MAGIC, GrB_UNINITIALIZED_OBJECT, "invalid monoid");     \
            if (!reduce_values(gb_obj_check(u), monoid, v)) monoid_identity(monoid, v);                      \
            ctype r;                                                                                         \
            gb_with_type(monoid->type->code, [&](auto z) {                                                   \
                using S = decltype(z);                                                                       \
                S sv;                                                                                        \
                memcpy(&sv, v, sizeof(S));                                                                   \
                r = gb_cast<ctype, S>(sv);                                                                   \
            });                                                                                              \
            if (accum) {                                                                                     \
                check_binop(accum, false);                                                                   \
                r = gb_binop<ctype>(accum->opcode, *c, r);                                                   \
            }                                                                                                \
            *c = r;                                                                                          \
        });                                                                                                  \
    }                                                                                                        \
    GrB_Info GrB_Matrix_reduce_##T(ctype *c, const GrB_BinaryOp accum, const GrB_Monoid monoid,              \
                                   const GrB_Matrix A, const GrB_Descriptor desc) {                          \
        return GrB_Vector_reduce_##T(c, accum, monoid, (GrB_Vector)A, desc);                                 \
    }                                                                                                        \
    GrB_Info GrB_Vector_apply_BinaryOp1st_##T(GrB_Vector w, const GrB_Vector mask, const GrB_BinaryOp accum,  \
                                              const GrB_BinaryOp op, ctype x, const GrB_Vector u,            \
                                              const GrB_Descriptor desc) {                                   \
        return gb_api(OBJ(w), [&] {                                                                          \
            do_apply(gb_obj_check(w), gb_obj_check(mask, true), accum, 1, nullptr, op, &x, GBAMD_T_##T,      \
                     gb_obj_check(u), gb_read_desc(desc));                                                   \
        });                                                                                                  \
    }                                                                                                        \
    GrB_Info GrB_Vector_apply_BinaryOp2nd_##T(GrB_Vector w, const GrB_Vector mask, const GrB_BinaryOp accum,  \
                                              const GrB_BinaryOp op, const GrB_Vector u, ctype y,            \
                                              const GrB_Descriptor desc) {                                   \
        return gb_api(OBJ(w), [&] {                                                                          \
            do_apply(gb_obj_check(w), gb_obj_check(mask, true), accum, 2, nullptr, op, &y, GBAMD_T_##T,      \
                     gb_obj_check(u), gb_read_desc(desc));                                                   \
        });                                                                                                  \
    }                                                                                                        \
    GrB_Info GrB_Matrix_apply_BinaryOp1st_##T(GrB_Matrix C, const GrB_Matrix Mask, const GrB_BinaryOp accum,  \
                                              const GrB_BinaryOp op, ctype x, const GrB_Matrix A,            \
                                              const GrB_Descriptor desc) {                                   \
        return gb_api(OBJ(C), [&] {                                                                          \
            do_apply(gb_obj_check(C), gb_obj_check(Mask, true), accum, 1, nullptr, op, &x, GBAMD_T_##T,      \
                     gb_obj_check(A), gb_read_desc(desc));                                                   \
        });                                                                                                  \
    }                                                                                                        \
    GrB_Info GrB_Matrix_apply_BinaryOp2nd_##T(GrB_Matrix C, const GrB_Matrix Mask, const GrB_BinaryOp accum,  \
                                              const GrB_BinaryOp op, const GrB_Matrix A, ctype y,            \
                                              const GrB_Descriptor desc) {                                   \
        return gb_api(OBJ(C), [&] {                                                                          \
            do_apply(gb_obj_check(C), gb_obj_check(Mask, true), accum, 2, nullptr, op, &y, GBAMD_T_##T,      \
                     gb_obj_check(A), gb_read_desc(desc));                                                   \
        });                                                                                                  \
    }

GB_FOR_EACH_TYPE(GB_DEFINE_TYPED_OPS)

}  // extern "C"
