// gb_spmv_sliced.hip -- general (non-iso) SpMV with a dense input, column-sliced by
// XCD: the kernel behind GrB_mxv / GrB_vxm with u full (reference
// core/matrix.py:2196, core/vector.py:1298; SURVEY §8d config 2, and the
// aggregators' A @ iso-full lowering, agg.py:207-279).
//
// Why: every product gathers u[k] at a random k.  On MI355X each of the 8 XCDs
// has its own 4 MiB L2; with the output rows spread over all XCDs every XCD
// gathers from all of u (32 MB fp64 at R-MAT s22), so most gathers miss L2 and
// are served by the Infinity Cache / HBM in 64-128 B lines (measured: 37 % L2
// hit rate, ~3 GB fetched per SpMV against 0.88 GB of algorithmic bytes).
// The matrix's columns are cut into 8 slices of ncols/8 and the entries copied
// once into slice-major CSRs (cached on the matrix per orientation, like the
// CSC).  A launch gives slice c to the blocks b with b % 8 == c -- blocks are
// dispatched round-robin over the XCDs, so each XCD gathers only from its own
// 1/8 of u, which its L2 holds.  Each slice folds its rows' products (a lane per
// short row, long rows in chunks over all waves) into a partial row vector; a
// second kernel folds the 8 partials in slice order, applies the mask and writes
// the result bitmap, values and count.  Extra traffic: the slice row pointers
// (8 x 4 B per row) and the partials (8 x (8 B + 1 bit) per row).
// Measured at R-MAT s22 (plus_times fp64 vxm): L2 hit rate of the gathers 37 % ->
// 71-78 %, fetched bytes 2.9 -> 0.9-1.3 GB per call -- but 1.15 ms against the
// words kernel's 0.92 ms: a row's ~16 entries become 8 runs of ~2, and the
// per-run work (row pointers, lane-per-row loads that no longer coalesce, or the
// words kernel's segmented scans) outweighs the saved misses.  Kept opt-in
// (knob spmv_sliced = 2) with its parity tests.
// Folds run in a fixed order (k within a slice's row, then slices): results
// are deterministic; for fp plus they differ from the unsliced order only by
// association (rtol 1e-12 in the tests).
#include <algorithm>

#include "gb_dispatch.cuh"
#include "gb_internal.h"

namespace {

constexpr int SL_N = 8;        // slices = XCDs
constexpr int SL_BLOCK = 256;  // 4 waves
constexpr int SL_U = 4;        // entries per lane per step

// ---------------------------------------------------------------- build
// per row: the start of each slice's run inside the row (columns are sorted), found by
// lane c's binary search for the slice's first column; counts[c][r] = run length
__global__ void k_sl_count(const int64_t *__restrict__ rowptr, const int32_t *__restrict__ colidx, int64_t nrows,
                           int64_t width, int32_t *__restrict__ cnt) {
    const int lane = threadIdx.x & 63;
    const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
    for (int64_t r = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6; r < nrows; r += nw) {
        const int64_t a = rowptr[r], b = rowptr[r + 1];
        int64_t off = 0;
        if (lane <= SL_N) {
            const int64_t key = lane * width;
            int64_t lo = a, hi = b;
            while (lo < hi) {
                const int64_t mid = (lo + hi) >> 1;
                if (colidx[mid] < key) lo = mid + 1;
                else hi = mid;
            }
            off = lane == SL_N ? b : lo;
        }
        const int64_t nxt = __shfl_down(off, 1, 64);
        if (lane < SL_N) cnt[(int64_t)lane * nrows + r] = (int32_t)(nxt - off);
    }
}

// copy each row's slice runs to their slice CSR (a wave per row)
template <class V>
__global__ void k_sl_fill(const int64_t *__restrict__ rowptr, const int32_t *__restrict__ colidx,
                          const V *__restrict__ vals, int64_t nrows, const int64_t *__restrict__ sp,
                          const int64_t *__restrict__ sbase, int32_t *__restrict__ scol, V *__restrict__ sval) {
    const int lane = threadIdx.x & 63;
    const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
    for (int64_t r = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6; r < nrows; r += nw) {
        int64_t src = rowptr[r];
        for (int c = 0; c < SL_N; c++) {
            const int64_t d0 = sp[(int64_t)c * (nrows + 1) + r], d1 = sp[(int64_t)c * (nrows + 1) + r + 1];
            const int64_t len = d1 - d0, dst = sbase[c] + d0;
            for (int64_t i = lane; i < len; i += 64) {
                scol[dst + i] = colidx[src + i];
                if (vals) sval[dst + i] = vals[src + i];
            }
            src += len;
        }
    }
}

constexpr int SL_SHORT = 8;   // rows with at most this many entries in a slice: a lane each
constexpr int SL_CH = 256;    // longer rows: chunks of SL_CH entries spread over the waves

// chunks per (slice, row): rows longer than SL_SHORT in the slice
__global__ void k_sl_lcount(const int32_t *__restrict__ cnt, int64_t total, int32_t *__restrict__ lc) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
        const int32_t d = cnt[i];
        lc[i] = d > SL_SHORT ? (d + SL_CH - 1) / SL_CH : 0;
    }
}
__global__ void k_sl_lfill(const int32_t *__restrict__ lc, const int64_t *__restrict__ loff, int64_t nrows,
                           int64_t total, int32_t *__restrict__ tab) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
        const int32_t c = lc[i];
        const int64_t o = loff[i];
        for (int32_t h = 0; h < c; h++) {
            tab[2 * (o + h)] = (int32_t)(i % nrows);
            tab[2 * (o + h) + 1] = h;
        }
    }
}

__global__ void k_i64_to_i32(const int64_t *__restrict__ in, int32_t *__restrict__ out, int64_t n) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        out[i] = (int32_t)in[i];
}

// ---------------------------------------------------------------- SpMV
template <class T>
__device__ __forceinline__ T sl_stream_load(const T *p) {
    return *p;
}

// slice c = blockIdx.x % SL_N; a wave per 64-row word of the slice's CSR, a lane per
// row.  A slice holds ~1/8 of a row's entries: rows of at most SL_SHORT entries are
// folded by their own lane in ascending k (all their loads and gathers issued at
// once); longer rows are taken one at a time by the whole wave (lanes stride the
// row, fold their share in order, then a butterfly in lane order).  No per-entry
// cross-lane traffic: the segmented scans of the words kernel would cost more than
// the gathers they organise at ~2 entries per row and slice.  Rows longer than
// SL_SHORT in the slice are cut into SL_CH-entry chunks (a table cached with the
// slices) that every wave of the slice takes in turn -- R-MAT's hubs sit in the first
// rows, so a word of them would otherwise hold one wave for milliseconds; each
// chunk's fold (lane shares in order, then a butterfly in lane order) goes to
// cpart, and k_spmv_slice_chunks folds a row's chunks in order into its partial.

template <class SR, class X, class Z, bool FLIP>
__global__ __launch_bounds__(SL_BLOCK) void k_spmv_slice(
    SR sr, int64_t nrows, const int32_t *__restrict__ srp, const int32_t *__restrict__ scol,
    const X *__restrict__ sval, bool a_iso, const X *__restrict__ uvals, bool u_iso, const int64_t *__restrict__ sbase,
    const int32_t *__restrict__ ltab, Z *__restrict__ cpart, int8_t *__restrict__ cfound, Z *__restrict__ part,
    uint64_t *__restrict__ pbits) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int c = blockIdx.x % SL_N;
    const int64_t wave = (int64_t)(blockIdx.x / SL_N) * (SL_BLOCK / 64) + wid;
    const int64_t nwaves = (int64_t)(gridDim.x / SL_N) * (SL_BLOCK / 64);
    const int64_t nwords = (nrows + 63) >> 6;
    const int32_t *rp = srp + (int64_t)c * (nrows + 1);
    const int64_t base = sbase[c];
    const int32_t *ci = scol + base;
    const X *vx = (sval && !a_iso) ? sval + base : nullptr;
    const bool rv = SR::reads_values && uvals && (vx || a_iso);
    X a0 = X(), u0 = X();
    if (rv) {
        if (a_iso) a0 = sval[0];
        if (u_iso) u0 = uvals[0];
    }
    Z *pc = part + (int64_t)c * nrows;
    uint64_t *bc = pbits + (int64_t)c * nwords;
    // long rows' chunks of this slice
    for (int64_t t = sbase[SL_N + 1 + c] + wave; t < sbase[SL_N + 2 + c]; t += nwaves) {
        const int32_t rr = ltab[2 * t], h = ltab[2 * t + 1];
        const int q1 = rp[rr + 1];
        const int q0 = rp[rr] + h * SL_CH;
        const int ql = min(SL_CH, q1 - q0);
        bool g = false;
        Z y = Z();
        int kk[SL_CH / 64];
        X aa[SL_CH / 64], bb[SL_CH / 64];
#pragma unroll
        for (int u = 0; u < SL_CH / 64; u++) {
            const int e = u * 64 + lane;
            kk[u] = e < ql ? sl_stream_load(ci + q0 + e) : 0;
            aa[u] = X();
            if (rv && e < ql) aa[u] = a_iso ? a0 : sl_stream_load(vx + q0 + e);
        }
#pragma unroll
        for (int u = 0; u < SL_CH / 64; u++) {
            bb[u] = X();
            if (rv && u * 64 + lane < ql) bb[u] = u_iso ? u0 : uvals[kk[u]];
        }
#pragma unroll
        for (int u = 0; u < SL_CH / 64; u++) {
            if (u * 64 + lane < ql) {
                const Z m = FLIP ? sr.mult(bb[u], aa[u], 0, kk[u], rr) : sr.mult(aa[u], bb[u], rr, kk[u], 0);
                y = g ? sr.add(y, m) : m;
                g = true;
            }
        }
        // fold the lanes' shares in lane order: lane i absorbs lane i + off
        for (int off = 1; off < 64; off <<= 1) {
            const bool og = __shfl_down((int)g, off, 64);
            const Z oy = gb_shfl_down(y, off, 64);
            if (lane + off < 64 && (lane & (2 * off - 1)) == 0 && og) {
                y = g ? sr.add(y, oy) : oy;
                g = true;
            }
        }
        if (lane == 0) {
            cfound[t] = g ? 1 : 0;
            if (g) cpart[t] = y;
        }
    }
    for (int64_t w = wave; w < nwords; w += nwaves) {
        const int64_t r = (w << 6) + lane;
        int p0 = 0, len = 0;
        if (r < nrows) {
            p0 = rp[r];
            len = rp[r + 1] - p0;
        }
        // short rows: the lane's own fold, loads first (long rows: their chunks, above)
        const bool shortr = len <= SL_SHORT;
        int k[SL_SHORT];
        X av[SL_SHORT], bv[SL_SHORT];
#pragma unroll
        for (int t = 0; t < SL_SHORT; t++) {
            const bool ok = shortr && t < len;
            k[t] = ok ? sl_stream_load(ci + p0 + t) : 0;
            av[t] = X();
            if (rv && ok) av[t] = a_iso ? a0 : sl_stream_load(vx + p0 + t);
        }
#pragma unroll
        for (int t = 0; t < SL_SHORT; t++) {
            bv[t] = X();
            if (rv && shortr && t < len) bv[t] = u_iso ? u0 : uvals[k[t]];
        }
        bool f = false;
        Z z = Z();
#pragma unroll
        for (int t = 0; t < SL_SHORT; t++) {
            if (shortr && t < len) {
                const Z m = FLIP ? sr.mult(bv[t], av[t], 0, k[t], r) : sr.mult(av[t], bv[t], r, k[t], 0);
                z = f ? sr.add(z, m) : m;
                f = true;
            }
        }
        const unsigned long long fmask = __ballot(f);
        if (f) pc[r] = z;
        if (lane == 0) bc[w] = fmask;
    }
}

// a long row's chunks (consecutive in the table) folded in order into its slice partial
template <class SR, class Z>
__global__ void k_spmv_slice_chunks(SR sr, int64_t nrows, const int32_t *__restrict__ ltab,
                                    const int64_t *__restrict__ sbase, int64_t ltotal, const Z *__restrict__ cpart,
                                    const int8_t *__restrict__ cfound, Z *__restrict__ part,
                                    uint64_t *__restrict__ pbits) {
    const int64_t nwords = (nrows + 63) >> 6;
    for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < ltotal; t += (int64_t)gridDim.x * blockDim.x) {
        if (ltab[2 * t + 1] != 0) continue;
        int c = 0;
        while (c + 1 < SL_N && sbase[SL_N + 2 + c] <= t) c++;
        const int32_t r = ltab[2 * t];
        const int64_t tend = sbase[SL_N + 2 + c];
        bool f = false;
        Z z = Z();
        for (int64_t h = t; h < tend && ltab[2 * h] == r && (h == t || ltab[2 * h + 1] != 0); h++) {
            if (!cfound[h]) continue;
            z = f ? sr.add(z, cpart[h]) : cpart[h];
            f = true;
        }
        if (f) {
            part[(int64_t)c * nrows + r] = z;
            atomicOr((unsigned long long *)&pbits[(int64_t)c * nwords + (r >> 6)], 1ULL << (r & 63));
        }
    }
}

// the result: fold the slices' partials in slice order, apply the mask, count
template <class SR, class Z>
__global__ __launch_bounds__(SL_BLOCK) void k_spmv_slice_combine(
    SR sr, int64_t nrows, const Z *__restrict__ part, const uint64_t *__restrict__ pbits,
    const uint64_t *__restrict__ mbits, bool mcomp, uint64_t *__restrict__ tbits, Z *__restrict__ tvals,
    unsigned long long *__restrict__ tcount, unsigned long long *__restrict__ gst) {
    const int lane = threadIdx.x & 63;
    const int64_t nwords = (nrows + 63) >> 6;
    const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
    long long cnt = 0;
    for (int64_t w = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6; w < nwords; w += nw) {
        const int64_t r = (w << 6) + lane;
        uint64_t allow = ~0ULL;
        if (mbits) allow = mcomp ? ~mbits[w] : mbits[w];
        bool found = false;
        Z acc = Z();
#pragma unroll
        for (int c = 0; c < SL_N; c++) {
            const uint64_t b = pbits[(int64_t)c * nwords + w] & allow;
            if ((b >> lane) & 1ULL) {
                const Z v = part[(int64_t)c * nrows + r];
                acc = found ? sr.add(acc, v) : v;
                found = true;
            }
        }
        const unsigned long long word = __ballot(found);
        if (found) tvals[r] = acc;
        if (lane == 0) {
            tbits[w] = word;
            cnt += __popcll(word);
        }
    }
    long long tot;
    if (gb_grid_sum(cnt, gst, &tot)) *tcount = (unsigned long long)tot;
}

}  // namespace

// slice-major copy of a matrix orientation (cached, like the CSC); v is the orientation's view
void gb_view_slices(gb_csr_view &v, GB_Obj *A, int orient) {
    if (A->kind != GB_KIND_MATRIX || v.nrows >= (1LL << 31) || v.nvals >= (1LL << 31)) return;
    if (!A->sl_colidx[orient]) {
        const int64_t n = v.nrows;
        int64_t width = (v.ncols + SL_N - 1) / SL_N;
        width = (width + 63) & ~63LL;
        gb_scratch s;
        int32_t *cnt = s.get<int32_t>((size_t)SL_N * n);
        const unsigned g = (unsigned)std::max<int64_t>(1, std::min<int64_t>((n * 64 + 255) / 256, 1 << 16));
        hipLaunchKernelGGL(k_sl_count, dim3(g), dim3(256), 0, gb_stream(), v.rowptr, v.colidx, n, width, cnt);
        GB_LAUNCH_CHECK();
        int64_t *sp = s.get<int64_t>((size_t)SL_N * (n + 1));
        int64_t base[SL_N + 1];
        base[0] = 0;
        for (int c = 0; c < SL_N; c++) {
            gb_exclusive_scan_i32(cnt + (int64_t)c * n, 0, sp + (int64_t)c * (n + 1), n);
            base[c + 1] = base[c] + gb_read_i64(sp + (int64_t)c * (n + 1) + n);
        }
        int64_t *dbase = s.get<int64_t>(SL_N + 1);
        gb_copy_h2d(dbase, base, sizeof(base));  // for the fill below
        int32_t *srp = gb_malloc_n<int32_t>((size_t)SL_N * (n + 1));
        hipLaunchKernelGGL(k_i64_to_i32, dim3(std::min<int64_t>(((int64_t)SL_N * (n + 1) + 255) / 256, 1 << 16)),
                           dim3(256), 0, gb_stream(), sp, srp, (int64_t)SL_N * (n + 1));
        int32_t *scol = gb_malloc_n<int32_t>(std::max<int64_t>(v.nvals, 1));
        const size_t ts = gb_type_size(v.tcode);
        void *sval = v.iso ? nullptr : gb_malloc(std::max<int64_t>(v.nvals, 1) * ts);
        gb_with_type(v.tcode, [&](auto z) {
            using V = decltype(z);
            hipLaunchKernelGGL((k_sl_fill<V>), dim3(g), dim3(256), 0, gb_stream(), v.rowptr, v.colidx,
                               v.iso ? nullptr : (const V *)v.vals, n, sp, dbase, scol, (V *)sval);
        });
        GB_LAUNCH_CHECK();
        // long rows of the slices: (row, chunk) table, slices in order, rows ascending
        int32_t *lc = s.get<int32_t>((size_t)SL_N * n);
        const unsigned g2 = (unsigned)std::max<int64_t>(1, std::min<int64_t>(((int64_t)SL_N * n + 255) / 256, 1 << 16));
        hipLaunchKernelGGL(k_sl_lcount, dim3(g2), dim3(256), 0, gb_stream(), cnt, (int64_t)SL_N * n, lc);
        GB_LAUNCH_CHECK();
        int64_t *loff = s.get<int64_t>((size_t)SL_N * n + 1);
        gb_exclusive_scan_i32(lc, 0, loff, (int64_t)SL_N * n);
        int64_t lbase[SL_N + 1];
        for (int c = 0; c <= SL_N; c++) lbase[c] = gb_read_i64(loff + (int64_t)c * n);
        const int64_t ltotal = lbase[SL_N];
        int32_t *ltab = gb_malloc_n<int32_t>(2 * ltotal + 2);
        hipLaunchKernelGGL(k_sl_lfill, dim3(g2), dim3(256), 0, gb_stream(), lc, loff, n, (int64_t)SL_N * n, ltab);
        GB_LAUNCH_CHECK();
        A->sl_rowptr[orient] = srp;
        A->sl_colidx[orient] = scol;
        A->sl_vals[orient] = sval;
        for (int c = 0; c <= SL_N; c++) A->sl_base[orient][c] = base[c];
        int64_t both[2 * (SL_N + 1)];
        for (int c = 0; c <= SL_N; c++) {
            both[c] = base[c];
            both[SL_N + 1 + c] = lbase[c];
        }
        A->sl_dbase[orient] = gb_malloc_n<int64_t>(2 * (SL_N + 1));
        gb_copy_h2d(A->sl_dbase[orient], both, sizeof(both));
        A->sl_ltab[orient] = ltab;
        A->sl_lcount[orient] = ltotal;
    }
    v.sl_rowptr = A->sl_rowptr[orient];
    v.sl_colidx = A->sl_colidx[orient];
    v.sl_vals = A->sl_vals[orient] ? A->sl_vals[orient] : v.vals;  // iso: the one value
    v.sl_base = A->sl_dbase[orient];
    v.sl_ltab = A->sl_ltab[orient];
    v.sl_lcount = A->sl_lcount[orient];
}

// y = A' u (or u' A') with u full, not iso in the result; false if not applicable
bool gb_spmv_sliced(gb_vec_result &T, const gb_csr_view &A, const void *uv, bool u_iso, const gb_vmask &mask,
                    GrB_Semiring sr, bool flip) {
    if (!A.sl_colidx) return false;
    gb_sr_info info = gb_sr_describe(sr);
    if (info.reads_values && A.tcode != info.xcode && !A.iso) return false;  // the copy holds A's own type
    const int64_t n = A.nrows;
    const int64_t nw = gb_words(n);
    gb_scratch s;
    const size_t zs = gb_type_size(info.zcode);
    void *part = s.get<char>((size_t)SL_N * n * zs);
    uint64_t *pbits = s.get<uint64_t>((size_t)SL_N * nw);
    const int64_t lt = A.sl_lcount;
    void *cpart = s.get<char>((size_t)(lt + 1) * zs);
    int8_t *cfound = s.get<int8_t>(lt + 1);
    unsigned long long *gst = gb_device_state();
    gb_dispatch_sr(info, [&](auto srf, auto x, auto z) {
        using SRT = decltype(srf);
        using X = decltype(x);
        using Z = decltype(z);
        int64_t per = gb_knob("spmv_slice_blocks");
        if (per <= 0) per = 512;  // blocks per slice (x 8 slices)
        per = std::max<int64_t>(1, std::min<int64_t>(per, (nw + 3) / 4));
        const unsigned grid = (unsigned)(per * SL_N);
        const X *av = info.reads_values ? (const X *)A.sl_vals : nullptr;
        if (flip)
            hipLaunchKernelGGL((k_spmv_slice<SRT, X, Z, true>), dim3(grid), dim3(SL_BLOCK), 0, gb_stream(), srf, n,
                               A.sl_rowptr, A.sl_colidx, av, A.iso, (const X *)uv, u_iso, A.sl_base, A.sl_ltab,
                               (Z *)cpart, cfound, (Z *)part, pbits);
        else
            hipLaunchKernelGGL((k_spmv_slice<SRT, X, Z, false>), dim3(grid), dim3(SL_BLOCK), 0, gb_stream(), srf, n,
                               A.sl_rowptr, A.sl_colidx, av, A.iso, (const X *)uv, u_iso, A.sl_base, A.sl_ltab,
                               (Z *)cpart, cfound, (Z *)part, pbits);
        GB_LAUNCH_CHECK();
        if (lt > 0) {
            const unsigned fg = (unsigned)std::max<int64_t>(1, std::min<int64_t>((lt + 255) / 256, 4096));
            hipLaunchKernelGGL((k_spmv_slice_chunks<SRT, Z>), dim3(fg), dim3(256), 0, gb_stream(), srf, n, A.sl_ltab,
                               A.sl_base, lt, (const Z *)cpart, cfound, (Z *)part, pbits);
            GB_LAUNCH_CHECK();
        }
        const unsigned cg = (unsigned)std::max<int64_t>(1, std::min<int64_t>((nw + 3) / 4, 4096));
        hipLaunchKernelGGL((k_spmv_slice_combine<SRT, Z>), dim3(cg), dim3(SL_BLOCK), 0, gb_stream(), srf, n,
                           (const Z *)part, pbits, mask.bits, mask.comp, T.bits, (Z *)T.dense,
                           (unsigned long long *)T.d_nvals, gst);
        GB_LAUNCH_CHECK();
    });
    return true;
}
