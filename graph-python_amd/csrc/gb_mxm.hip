// gb_mxm.hip -- SpGEMM over a semiring: the kernels behind GrB_mxm
// (replaces SuiteSparse's GB_AxB_dot3 / saxpy3 reached from reference
// core/matrix.py:2241 and core/vector.py:1686).
//
// Two methods, chosen per call:
//  * masked dot product (mask present, not complemented): T(i,j) is computed
//    only for (i,j) in M, by merging row i of A' with row j of B'^T (the
//    cached CSC).  Each entry folds its terms in ascending k.
//  * Gustavson as expand-sort-compress (no mask / complemented mask): every
//    product A'(i,k) B'(k,j) is written at a position ordered by (i, k, j),
//    a stable radix sort on (i, j) groups the terms of each output entry
//    without disturbing their k order, and one pass folds each run.  Rows are
//    processed in chunks so the expanded products stay within a memory budget.
// The masked dot kernels and expand-sort-compress fold every output entry in
// ascending k, so their floating-point results do not depend on scheduling.
// The default Gustavson kernel is the hash method of gb_spgemm_hash.hip, which
// folds fp PLUS/TIMES with atomics in arrival order: fp64 plus_times results
// can differ between runs in the last bits (exact monoids -- min/max/integer
// plus/times/lor/land/any_pair -- stay bit-exact).  Knob spgemm_method=1
// (GxB_set_knob, graphblas_amd.set_knob("spgemm_method", 1)) selects
// expand-sort-compress: the deterministic, bit-reproducible mode.
#include <algorithm>
#include <vector>

#include "gb_dispatch.cuh"
#include "gb_internal.h"

#define MXM_BLOCK 256
static inline unsigned mxm_grid(int64_t n, unsigned cap = 16384) {
    int64_t g = (n + MXM_BLOCK - 1) / MXM_BLOCK;
    if (g < 1) g = 1;
    if (g > cap) g = cap;
    return (unsigned)g;
}
#define MXM_STRIDE(i, n) \
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < (n); i += (int64_t)gridDim.x * blockDim.x)

__global__ void k_rowof(const int64_t *__restrict__ rowptr, int64_t r0, int64_t r1, int64_t pbase,
                        int64_t *__restrict__ rowof) {
    int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
    int lane = threadIdx.x & 63;
    int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
    for (int64_t i = r0 + wave; i < r1; i += nw)
        for (int64_t p = rowptr[i] + lane; p < rowptr[i + 1]; p += 64) rowof[p - pbase] = i;
}

// ================================================================== masked dot
template <class SR, class X, class Z>
__global__ __launch_bounds__(MXM_BLOCK) void k_dot_masked(
    SR sr, int64_t nm, const int64_t *__restrict__ mrowof, const int32_t *__restrict__ mci,
    const int64_t *__restrict__ arp, const int32_t *__restrict__ aci, const X *__restrict__ avx, bool a_iso,
    const int64_t *__restrict__ brp, const int32_t *__restrict__ bci, const X *__restrict__ bvx, bool b_iso,
    Z *__restrict__ tval, uint8_t *__restrict__ tflag) {
    MXM_STRIDE(q, nm) {
        const int64_t i = mrowof[q];
        const int32_t j = mci[q];
        const int64_t pa0 = arp[i], ea = arp[i + 1], pb0 = brp[j], eb = brp[j + 1];
        // walk the shorter list in ascending k; find each k in the longer one by
        // galloping from the last match (exponential then binary search)
        const bool a_short = (ea - pa0) <= (eb - pb0);
        const int32_t *__restrict__ sci = a_short ? aci : bci;
        const int32_t *__restrict__ lci = a_short ? bci : aci;
        int64_t ps = a_short ? pa0 : pb0, es = a_short ? ea : eb;
        int64_t pl = a_short ? pb0 : pa0, el = a_short ? eb : ea;
        bool found = false;
        Z acc = Z();
        for (; ps < es && pl < el; ps++) {
            const int32_t k = sci[ps];
            if (lci[pl] < k) {
                int64_t lo = pl, step = 1;  // lci[lo] < k
                while (lo + step < el && lci[lo + step] < k) {
                    lo += step;
                    step <<= 1;
                }
                int64_t hi = lo + step < el ? lo + step : el;  // lci[hi] >= k or hi == el
                while (hi - lo > 1) {
                    const int64_t mid = (lo + hi) >> 1;
                    if (lci[mid] < k) lo = mid;
                    else hi = mid;
                }
                pl = hi;
                if (pl >= el) break;
            }
            if (lci[pl] != k) continue;
            const int64_t pa = a_short ? ps : pl, pb = a_short ? pl : ps;
            X a = X(), b = X();
            if (SR::reads_values && avx && bvx) {
                a = avx[a_iso ? 0 : pa];
                b = bvx[b_iso ? 0 : pb];
            }
            Z z = sr.mult(a, b, i, k, j);
            acc = found ? sr.add(acc, z) : z;
            found = true;
            if (sr.terminal(acc)) break;
            pl++;
        }
        tflag[q] = found ? 1 : 0;
        if (found) tval[q] = acc;
    }
}

// Masked dot with G lanes per mask entry, for monoids that are exactly
// associative and commutative on Z (MIN/MAX/logical/bitwise, integer
// PLUS/TIMES): the lanes split the shorter of the two lists and binary-search
// each k in the longer one (independent loads, no serial merge), then fold
// their partials across the group.
template <class SR, class X, class Z, int G>
__global__ __launch_bounds__(MXM_BLOCK) void k_dot_masked_group(
    SR sr, int64_t nm, const int64_t *__restrict__ mrowof, const int32_t *__restrict__ mci,
    const int64_t *__restrict__ arp, const int32_t *__restrict__ aci, const X *__restrict__ avx, bool a_iso,
    const int64_t *__restrict__ brp, const int32_t *__restrict__ bci, const X *__restrict__ bvx, bool b_iso,
    Z *__restrict__ tval, uint8_t *__restrict__ tflag, const int64_t *__restrict__ qlist) {
    const int64_t tid = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    const int gl = (int)(tid & (G - 1));
    const int64_t ngroups = ((int64_t)gridDim.x * blockDim.x) / G;
    for (int64_t qq = tid / G; qq < nm; qq += ngroups) {
        const int64_t q = qlist ? qlist[qq] : qq;  // a list of mask positions, or all of them
        const int64_t i = mrowof[q];
        const int32_t j = mci[q];
        const int64_t pa0 = arp[i], ea = arp[i + 1], pb0 = brp[j], eb = brp[j + 1];
        const bool a_short = (ea - pa0) <= (eb - pb0);
        const int32_t *__restrict__ sci = a_short ? aci : bci;
        const int32_t *__restrict__ lci = a_short ? bci : aci;
        const int64_t ps0 = a_short ? pa0 : pb0, es = a_short ? ea : eb;
        const int64_t pl0 = a_short ? pb0 : pa0, el = a_short ? eb : ea;
        bool found = false;
        Z acc = Z();
        const int64_t L = el - pl0;
        if (G == 64 && L >= 256) {
            // a wave per entry: 64 evenly spaced samples of the long list (one load per
            // lane) narrow every search to one 1/64 bucket by shuffles, before any
            // dependent global load
            const int32_t samp = lci[pl0 + (((int64_t)gl * L) >> 6)];
            for (int64_t base = 0; base < es - ps0; base += 64) {
                const int64_t ps = ps0 + base + gl;
                const bool act = ps < es;
                const int32_t k = act ? sci[ps] : 0x7fffffff;
                int bk = 0;
#pragma unroll
                for (int st = 32; st > 0; st >>= 1)
                    if (__shfl(samp, bk + st, 64) <= k) bk += st;
                if (!act) continue;
                int64_t a = pl0 + (((int64_t)bk * L) >> 6);
                int64_t b = bk == 63 ? el : pl0 + (((int64_t)(bk + 1) * L) >> 6) + 1;
                if (b > el) b = el;
                while (a < b) {
                    const int64_t mid = (a + b) >> 1;
                    if (lci[mid] < k) a = mid + 1;
                    else b = mid;
                }
                if (a < el && lci[a] == k) {
                    const int64_t pa = a_short ? ps : a, pb = a_short ? a : ps;
                    X av = X(), bv = X();
                    if (SR::reads_values && avx && bvx) {
                        av = avx[a_iso ? 0 : pa];
                        bv = bvx[b_iso ? 0 : pb];
                    }
                    const Z z = sr.mult(av, bv, i, k, j);
                    acc = found ? sr.add(acc, z) : z;
                    found = true;
                }
            }
        }
        int64_t lo = pl0;  // this lane's k values increase: the search window only shrinks
        for (int64_t ps = ps0 + gl; !(G == 64 && L >= 256) && ps < es && lo < el; ps += G) {
            const int32_t k = sci[ps];
            int64_t a = lo, b = el;  // first position with lci >= k
            while (a < b) {
                const int64_t mid = (a + b) >> 1;
                if (lci[mid] < k) a = mid + 1;
                else b = mid;
            }
            lo = a;
            if (a < el && lci[a] == k) {
                const int64_t pa = a_short ? ps : a, pb = a_short ? a : ps;
                X av = X(), bv = X();
                if (SR::reads_values && avx && bvx) {
                    av = avx[a_iso ? 0 : pa];
                    bv = bvx[b_iso ? 0 : pb];
                }
                const Z z = sr.mult(av, bv, i, k, j);
                acc = found ? sr.add(acc, z) : z;
                found = true;
            }
        }
#pragma unroll
        for (int off = G >> 1; off > 0; off >>= 1) {
            const bool of = __shfl_xor((int)found, off, G);
            const Z oz = gb_shfl_xor(acc, off, G);
            if (of) {
                acc = found ? sr.add(acc, oz) : oz;
                found = true;
            }
        }
        if (gl == 0) {
            tflag[q] = found ? 1 : 0;
            if (found) tval[q] = acc;
        }
    }
}

static bool exact_monoid(int mon, int zcode) {
    switch (mon) {
    case GBAMD_MON_MIN: case GBAMD_MON_MAX: case GBAMD_MON_LOR: case GBAMD_MON_LAND: case GBAMD_MON_LXOR:
    case GBAMD_MON_LXNOR: case GBAMD_MON_BOR: case GBAMD_MON_BAND: case GBAMD_MON_BXOR: case GBAMD_MON_BXNOR:
        return true;
    case GBAMD_MON_PLUS: case GBAMD_MON_TIMES: return zcode != GBAMD_T_FP32 && zcode != GBAMD_T_FP64;
    default: return false;  // ANY keeps the first k: the sequential merge does that
    }
}

__global__ void k_gather_rowptr(const int64_t *__restrict__ mrp, const int64_t *__restrict__ pos, int64_t nrows,
                                int64_t *__restrict__ trp) {
    MXM_STRIDE(i, nrows + 1) trp[i] = pos[mrp[i]];
}

template <class Z>
__global__ void k_compact_dot(int64_t nm, const uint8_t *__restrict__ flag, const int64_t *__restrict__ pos,
                              const int32_t *__restrict__ mci, const Z *__restrict__ tval, int32_t *__restrict__ oci,
                              Z *__restrict__ ovx) {
    MXM_STRIDE(q, nm) {
        if (flag[q]) {
            int64_t o = pos[q];
            oci[o] = mci[q];
            if (ovx) ovx[o] = tval[q];
        }
    }
}

// ================================================================== Gustavson (ESC)
__global__ void k_row_flops(const int64_t *__restrict__ arp, const int32_t *__restrict__ aci, int64_t nrows,
                            const int64_t *__restrict__ brp, int64_t *__restrict__ fl) {
    int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
    int lane = threadIdx.x & 63;
    int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
    for (int64_t i = wave; i < nrows; i += nw) {
        int64_t s = 0;
        for (int64_t p = arp[i] + lane; p < arp[i + 1]; p += 64) {
            int32_t k = aci[p];
            s += brp[k + 1] - brp[k];
        }
        for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
        if (lane == 0) fl[i] = s;
    }
}

__global__ void k_entry_counts(const int32_t *__restrict__ aci, int64_t p0, int64_t np, const int64_t *__restrict__ brp,
                               int64_t *__restrict__ cnt) {
    MXM_STRIDE(q, np) {
        int32_t k = aci[p0 + q];
        cnt[q] = brp[k + 1] - brp[k];
    }
}

// one wave per A' entry: the B' row is streamed by 64 lanes (coalesced)
template <class SR, class X, class Z>
__global__ __launch_bounds__(MXM_BLOCK) void k_expand(
    SR sr, int64_t p0, int64_t np, int64_t r0, const int64_t *__restrict__ rowof, const int32_t *__restrict__ aci,
    const X *__restrict__ avx, bool a_iso, const int64_t *__restrict__ brp, const int32_t *__restrict__ bci,
    const X *__restrict__ bvx, bool b_iso, const int64_t *__restrict__ eoff, uint64_t *__restrict__ keys,
    int64_t *__restrict__ perm, Z *__restrict__ vals) {
    int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
    int lane = threadIdx.x & 63;
    int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
    for (int64_t q = wave; q < np; q += nw) {
        int64_t p = p0 + q;
        int64_t i = rowof[q];
        int32_t k = aci[p];
        X a = X();
        const bool rv = SR::reads_values && avx && bvx;
        if (rv) a = avx[a_iso ? 0 : p];
        int64_t base = eoff[q], b0 = brp[k], b1 = brp[k + 1];
        for (int64_t pb = b0 + lane; pb < b1; pb += 64) {
            int32_t j = bci[pb];
            X b = X();
            if (rv) b = bvx[b_iso ? 0 : pb];
            int64_t o = base + (pb - b0);
            keys[o] = ((uint64_t)(i - r0) << 32) | (uint32_t)j;
            perm[o] = o;
            if (vals) vals[o] = sr.mult(a, b, i, k, j);
        }
    }
}

__global__ void k_run_heads(const uint64_t *__restrict__ keys, int64_t n, int64_t *__restrict__ head) {
    MXM_STRIDE(q, n) head[q] = (q == 0 || keys[q] != keys[q - 1]) ? 1 : 0;
}

template <class SR, class Z>
__global__ void k_fold(SR sr, const uint64_t *__restrict__ keys, const int64_t *__restrict__ perm,
                       const int64_t *__restrict__ pos, int64_t n, const Z *__restrict__ vals, int64_t r0,
                       unsigned long long *__restrict__ rowcnt, int32_t *__restrict__ oci, Z *__restrict__ ovx) {
    MXM_STRIDE(q, n) {
        if (q != 0 && keys[q] == keys[q - 1]) continue;
        int64_t o = pos[q];
        oci[o] = (int32_t)(keys[q] & 0xffffffffULL);
        atomicAdd(&rowcnt[r0 + (int64_t)(keys[q] >> 32)], 1ULL);
        if (ovx) {
            Z acc = vals[perm[q]];
            for (int64_t r = q + 1; r < n && keys[r] == keys[q]; r++) {
                if (sr.terminal(acc)) break;
                acc = sr.add(acc, vals[perm[r]]);
            }
            ovx[o] = acc;
        }
    }
}

static bool idempotent(int m) {
    return m == GBAMD_MON_ANY || m == GBAMD_MON_MIN || m == GBAMD_MON_MAX || m == GBAMD_MON_LOR ||
           m == GBAMD_MON_LAND || m == GBAMD_MON_BOR || m == GBAMD_MON_BAND;
}

template <class SR, class X, class Z>
__global__ void k_iso_value2(SR sr, const X *avals, const X *bvals, Z *out) {
    X a = avals ? avals[0] : X(), b = bvals ? bvals[0] : X();
    *out = sr.mult(a, b, 0, 0, 0);
}

// gb_dot.hip: masked dot, two-sided LDS method (exact monoids)
int64_t gb_dot_two_sided(const gb_csr_view &A, const gb_csr_view &BT, gb_mmask &mask, const gb_sr_info &info,
                         const void *av, const void *btv, void *tval, uint8_t *tflag, int64_t **huge);

void gb_spgemm(gb_mat_result &T, gb_csr_view &A, gb_csr_view &B, gb_csr_view *BT, gb_mmask &mask,
               GrB_Semiring sr) {
    gb_sr_info info = gb_sr_describe(sr);
    gb_scratch s;
    const void *av = info.reads_values ? gb_view_vals_as(A, info.xcode, s) : nullptr;
    const int64_t nrows = A.nrows, ncols = B.ncols;
    const size_t zs = gb_type_size(info.zcode);
    bool reads_a = info.reads_values, reads_b = info.reads_values;
    if (info.mul == GBAMD_OP_FIRST) reads_b = false;
    if (info.mul == GBAMD_OP_SECOND) reads_a = false;
    bool iso = !info.positional && idempotent(info.mon) && (!reads_a || A.iso) && (!reads_b || B.iso);
    if (info.mul == GBAMD_OP_PAIR) iso = idempotent(info.mon);
    T.nrows = nrows;
    T.ncols = ncols;
    T.tcode = info.zcode;
    T.iso = iso;

    const bool use_dot = mask.present && !mask.comp && BT != nullptr;
    if (use_dot) {
        const void *btv = info.reads_values ? gb_view_vals_as(*BT, info.xcode, s) : nullptr;
        const int64_t nm = mask.nvals;
        uint8_t *flag = s.get<uint8_t>(nm);
        int64_t *pos = s.get<int64_t>(nm + 1);
        void *tval = s.get<char>(nm * zs);
        int64_t *mrowof = nullptr;
        auto rowof = [&]() {
            mrowof = s.get<int64_t>(nm);
            hipLaunchKernelGGL(k_rowof, dim3(mxm_grid(std::min<int64_t>(nrows * 64, 1LL << 22))), dim3(MXM_BLOCK), 0,
                               gb_stream(), mask.rowptr, (int64_t)0, nrows, (int64_t)0, mrowof);
        };
        gb_dispatch_sr(info, [&](auto srf, auto x, auto z) {
            using SRT = decltype(srf);
            using X = decltype(x);
            using Z = decltype(z);
            int64_t gsel = gb_knob("dot_group");  // 0 auto (a wave per entry), 1 thread per entry, else lanes
            if (gsel == 0) gsel = 64;
            const bool exact = exact_monoid(info.mon, info.zcode);
            // the two-sided LDS method (gb_dot.hip) folds into monoid identities: not for
            // float MIN/MAX, whose NaN-ignoring fold of only-NaN terms differs from the identity's
            const bool float_minmax = (info.zcode == GBAMD_T_FP32 || info.zcode == GBAMD_T_FP64) &&
                                      (info.mon == GBAMD_MON_MIN || info.mon == GBAMD_MON_MAX);
            const bool any_pair = info.mon == GBAMD_MON_ANY && info.mul == GBAMD_OP_PAIR;
            const bool two_sided = nm && (exact || any_pair) && !float_minmax && gb_knob("dot_method") != 1;
            if (nm) gb_memset(flag, 0, nm);
            if (two_sided) {
                int64_t *hq = nullptr;
                const int64_t nh = gb_dot_two_sided(A, *BT, mask, info, av, btv, tval, flag, &hq);
                if (nh) {
                    rowof();
                    const unsigned g = mxm_grid(std::min<int64_t>(nh * 64, 1LL << 24));
                    hipLaunchKernelGGL((k_dot_masked_group<SRT, X, Z, 64>), dim3(g), dim3(MXM_BLOCK), 0, gb_stream(),
                                       srf, nh, mrowof, mask.colidx, A.rowptr, A.colidx, (const X *)av, A.iso,
                                       BT->rowptr, BT->colidx, (const X *)btv, BT->iso, (Z *)tval, flag, hq);
                    GB_LAUNCH_CHECK();
                    gb_free(hq);
                }
            } else if (nm && gsel > 1 && exact) {
                rowof();
                const unsigned g = mxm_grid(std::min<int64_t>(nm * gsel, 1LL << 24));
#define GB_DOT_GROUP(GG)                                                                                 \
    hipLaunchKernelGGL((k_dot_masked_group<SRT, X, Z, GG>), dim3(g), dim3(MXM_BLOCK), 0, gb_stream(), srf, nm, \
                       mrowof, mask.colidx, A.rowptr, A.colidx, (const X *)av, A.iso, BT->rowptr, BT->colidx, \
                       (const X *)btv, BT->iso, (Z *)tval, flag, (const int64_t *)nullptr)
                if (gsel <= 4) GB_DOT_GROUP(4);
                else if (gsel <= 8) GB_DOT_GROUP(8);
                else if (gsel <= 16) GB_DOT_GROUP(16);
                else if (gsel <= 32) GB_DOT_GROUP(32);
                else GB_DOT_GROUP(64);
#undef GB_DOT_GROUP
            } else if (nm) {
                rowof();
                hipLaunchKernelGGL((k_dot_masked<SRT, X, Z>), dim3(mxm_grid(nm)), dim3(MXM_BLOCK), 0, gb_stream(),
                                   srf, nm, mrowof, mask.colidx, A.rowptr, A.colidx, (const X *)av, A.iso,
                                   BT->rowptr, BT->colidx, (const X *)btv, BT->iso, (Z *)tval, flag);
            }
            GB_LAUNCH_CHECK();
            gb_exclusive_scan_u8(flag, pos, nm);
            int64_t nz = gb_read_i64(pos + nm);
            T.rowptr = gb_malloc_n<int64_t>(nrows + 1);
            hipLaunchKernelGGL(k_gather_rowptr, dim3(mxm_grid(nrows + 1)), dim3(MXM_BLOCK), 0, gb_stream(),
                               mask.rowptr, pos, nrows, T.rowptr);
            T.colidx = gb_malloc_n<int32_t>(nz);
            T.vals = gb_malloc((iso ? 1 : nz) * zs);
            if (nm)
                hipLaunchKernelGGL(k_compact_dot<Z>, dim3(mxm_grid(nm)), dim3(MXM_BLOCK), 0, gb_stream(), nm, flag,
                                   pos, mask.colidx, (const Z *)tval, T.colidx, iso ? nullptr : (Z *)T.vals);
            if (iso)
                hipLaunchKernelGGL((k_iso_value2<SRT, X, Z>), dim3(1), dim3(1), 0, gb_stream(), srf, (const X *)av,
                                   (const X *)btv, (Z *)T.vals);
            GB_LAUNCH_CHECK();
            T.nvals = nz;
        });
        T.within_mask = true;
        return;
    }

    // ---------------- Gustavson, expand-sort-compress in row chunks
    const void *bv = info.reads_values ? gb_view_vals_as(B, info.xcode, s) : nullptr;
    int64_t *fl = s.get<int64_t>(nrows + 1);
    int64_t *flp = s.get<int64_t>(nrows + 1);
    if (nrows)
        hipLaunchKernelGGL(k_row_flops, dim3(mxm_grid(std::min<int64_t>(nrows * 64, 1LL << 22))), dim3(MXM_BLOCK), 0,
                           gb_stream(), A.rowptr, A.colidx, nrows, B.rowptr, fl);
    GB_LAUNCH_CHECK();
    if (gb_knob("spgemm_method") != 1) {
        // default: hash Gustavson (gb_spgemm_hash.hip)
        gb_spgemm_hash(T, A, B, sr, iso, av, bv, fl);
        if (iso)
            gb_dispatch_sr(info, [&](auto srf, auto x, auto z) {
                using SRT = decltype(srf);
                using X = decltype(x);
                using Z = decltype(z);
                hipLaunchKernelGGL((k_iso_value2<SRT, X, Z>), dim3(1), dim3(1), 0, gb_stream(), srf, (const X *)av,
                                   (const X *)bv, (Z *)T.vals);
                GB_LAUNCH_CHECK();
            });
        T.within_mask = false;
        return;
    }
    gb_exclusive_scan_i64(fl, flp, nrows);
    const int64_t F = gb_read_i64(flp + nrows);
    int64_t budget = gb_knob("esc_budget");
    if (budget <= 0) budget = 1LL << 27;
    // chunk boundaries (host)
    std::vector<int64_t> bounds;
    bounds.push_back(0);
    if (F > budget) {
        std::vector<int64_t> hp(nrows + 1);
        gb_copy_d2h(hp.data(), flp, (nrows + 1) * sizeof(int64_t));
        int64_t r = 0;
        while (r < nrows) {
            int64_t lim = hp[r] + budget;
            int64_t e = std::upper_bound(hp.begin() + r + 1, hp.end(), lim) - hp.begin() - 1;
            if (e <= r) e = r + 1;  // a single row larger than the budget
            if (e > nrows) e = nrows;
            bounds.push_back(e);
            r = e;
        }
    } else {
        bounds.push_back(nrows);
    }
    // row pointers of A' (host copy of the chunk boundaries' entry offsets)
    std::vector<int64_t> chunk_nz;
    std::vector<int32_t *> chunk_ci;
    std::vector<void *> chunk_vx;
    unsigned long long *rowcnt = s.get<unsigned long long>(nrows + 1);
    gb_memset(rowcnt, 0, (nrows + 1) * sizeof(unsigned long long));
    gb_dispatch_sr(info, [&](auto srf, auto x, auto z) {
        using SRT = decltype(srf);
        using X = decltype(x);
        using Z = decltype(z);
        for (size_t c = 0; c + 1 < bounds.size(); c++) {
            const int64_t r0 = bounds[c], r1 = bounds[c + 1];
            int64_t pr[2];
            gb_copy_d2h(&pr[0], A.rowptr + r0, sizeof(int64_t));
            gb_copy_d2h(&pr[1], A.rowptr + r1, sizeof(int64_t));
            const int64_t p0 = pr[0], np = pr[1] - pr[0];
            gb_scratch cs;
            int64_t *cnt = cs.get<int64_t>(np + 1);
            int64_t *eoff = cs.get<int64_t>(np + 1);
            int64_t *rowof = cs.get<int64_t>(np);
            if (np) {
                hipLaunchKernelGGL(k_entry_counts, dim3(mxm_grid(np)), dim3(MXM_BLOCK), 0, gb_stream(), A.colidx, p0,
                                   np, B.rowptr, cnt);
                hipLaunchKernelGGL(k_rowof, dim3(mxm_grid(std::min<int64_t>((r1 - r0) * 64, 1LL << 22))),
                                   dim3(MXM_BLOCK), 0, gb_stream(), A.rowptr, r0, r1, p0, rowof);
                GB_LAUNCH_CHECK();
            }
            gb_exclusive_scan_i64(cnt, eoff, np);
            const int64_t fc = gb_read_i64(eoff + np);
            if (fc == 0) {
                chunk_nz.push_back(0);
                chunk_ci.push_back(nullptr);
                chunk_vx.push_back(nullptr);
                continue;
            }
            uint64_t *keys = cs.get<uint64_t>(fc);
            int64_t *perm = cs.get<int64_t>(fc);
            Z *vals = iso ? nullptr : cs.get<Z>(fc);
            hipLaunchKernelGGL((k_expand<SRT, X, Z>), dim3(mxm_grid(std::min<int64_t>(np * 64, 1LL << 24))),
                               dim3(MXM_BLOCK), 0, gb_stream(), srf, p0, np, r0, rowof, A.colidx, (const X *)av, A.iso,
                               B.rowptr, B.colidx, (const X *)bv, B.iso, eoff, keys, perm, vals);
            GB_LAUNCH_CHECK();
            int rbits = 1;
            while (rbits < 31 && (1LL << rbits) < (r1 - r0)) rbits++;
            gb_sort_pairs_u64(keys, perm, fc, 32 + rbits);
            int64_t *head = cs.get<int64_t>(fc);
            int64_t *pos = cs.get<int64_t>(fc + 1);
            hipLaunchKernelGGL(k_run_heads, dim3(mxm_grid(fc)), dim3(MXM_BLOCK), 0, gb_stream(), keys, fc, head);
            GB_LAUNCH_CHECK();
            gb_exclusive_scan_i64(head, pos, fc);
            const int64_t nu = gb_read_i64(pos + fc);
            int32_t *oci = gb_malloc_n<int32_t>(nu);
            Z *ovx = iso ? nullptr : gb_malloc_n<Z>(nu);
            hipLaunchKernelGGL((k_fold<SRT, Z>), dim3(mxm_grid(fc)), dim3(MXM_BLOCK), 0, gb_stream(), srf, keys, perm,
                               pos, fc, (const Z *)vals, r0, rowcnt, oci, ovx);
            GB_LAUNCH_CHECK();
            chunk_nz.push_back(nu);
            chunk_ci.push_back(oci);
            chunk_vx.push_back(ovx);
        }
        int64_t nz = 0;
        for (int64_t c : chunk_nz) nz += c;
        T.rowptr = gb_malloc_n<int64_t>(nrows + 1);
        gb_exclusive_scan_i64((const int64_t *)rowcnt, T.rowptr, nrows);
        if (chunk_nz.size() == 1) {
            T.colidx = chunk_ci[0] ? chunk_ci[0] : gb_malloc_n<int32_t>(1);
            T.vals = iso ? gb_malloc(zs) : (chunk_vx[0] ? chunk_vx[0] : gb_malloc(zs));
        } else {
            T.colidx = gb_malloc_n<int32_t>(nz);
            T.vals = gb_malloc((iso ? 1 : nz) * zs);
            int64_t off = 0;
            for (size_t c = 0; c < chunk_nz.size(); c++) {
                if (chunk_nz[c]) {
                    gb_copy_d2d(T.colidx + off, chunk_ci[c], chunk_nz[c] * sizeof(int32_t));
                    if (!iso) gb_copy_d2d((char *)T.vals + off * zs, chunk_vx[c], chunk_nz[c] * zs);
                }
                off += chunk_nz[c];
                gb_free(chunk_ci[c]);
                gb_free(chunk_vx[c]);
            }
        }
        if (iso)
            hipLaunchKernelGGL((k_iso_value2<SRT, X, Z>), dim3(1), dim3(1), 0, gb_stream(), srf, (const X *)av,
                               (const X *)bv, (Z *)T.vals);
        GB_LAUNCH_CHECK();
        T.nvals = nz;
    });
    T.within_mask = false;
}
