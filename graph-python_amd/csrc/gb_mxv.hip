// gb_mxv.hip -- masked SpMV over a semiring: the kernels behind GrB_mxv and
// GrB_vxm (replaces SuiteSparse's GB_AxB dot/saxpy kernels reached from
// reference core/matrix.py:2196 and core/vector.py:1298).
//
// Pull (bottom-up): output position r reads row r of A' (CSR for mxv, the
// cached CSC for vxm), tests the bitmap of u for each column k and folds the
// products with the monoid.  Masked-out rows are skipped before any of their
// entries are read (the BFS `~v.S` mask removes every visited vertex).
// Monoids with a terminal value (LOR, ANY, MIN on integers, ...) stop a row as
// soon as any lane of its group reaches it.
// Layout: a 256-thread block owns tiles of 256 consecutive output rows
// (4 bitmap words).  G lanes (G = 1..64, from the average row length) share a
// row; their column-index loads are coalesced.  Output presence bits are
// assembled in LDS and written as whole 64-bit words (no global atomics); the
// popcount of the block's words goes to the device nvals counter with one
// atomic per block.
//
// Push (top-down), for results whose value is iso (BFS lor_land / any_pair):
// every frontier vertex k streams its row of the other orientation of A'
// and sets the output bits of the unmasked targets with atomicOr.  The choice
// between the two is made on the device from the frontier's edge count
// (Beamer's direction-optimizing rule), so no host round trip is needed.
#include "gb_dispatch.cuh"
#include "gb_internal.h"

#define SPMV_BLOCK 256
#define SPMV_TILE 256

struct gb_dir_state {
    unsigned long long mf;  // frontier edges in the push orientation
    unsigned long long nf;  // frontier vertices
};

__device__ __forceinline__ bool gb_choose_push(const gb_dir_state *st, const int64_t *mask_count, bool mcomp,
                                               int64_t n_out, int64_t nnz, int64_t alpha) {
    int64_t open = n_out;  // rows the pull kernel would have to visit
    if (mask_count) {
        int64_t mc = *mask_count;
        open = mcomp ? (n_out - mc) : mc;
    }
    double avg = n_out ? (double)nnz / (double)n_out : 0.0;
    return (double)st->mf * (double)alpha < (double)open * avg;
}

template <class SR, class X, class Z, bool FLIP>
__global__ __launch_bounds__(SPMV_BLOCK) void k_spmv_pull(
    SR sr, int64_t nrows, const int64_t *__restrict__ rowptr, const int32_t *__restrict__ colidx,
    const X *__restrict__ avals, bool a_iso, const uint64_t *__restrict__ ubits,
    const X *__restrict__ uvals, bool u_iso, const uint64_t *__restrict__ mbits, bool mcomp, int lg,
    uint64_t *__restrict__ tbits, Z *__restrict__ tvals, unsigned long long *__restrict__ tcount,
    const gb_dir_state *__restrict__ st, const int64_t *__restrict__ mask_count, int64_t nnz, int64_t alpha) {
    if (st && gb_choose_push(st, mask_count, mcomp, nrows, nnz, alpha)) return;
    __shared__ unsigned long long words[SPMV_TILE / 64];
    const int G = 1 << lg;
    const int gid = threadIdx.x >> lg;
    const int gl = threadIdx.x & (G - 1);
    const int ngroups = SPMV_BLOCK >> lg;
    const int lane = threadIdx.x & 63;
    const unsigned long long gmask = (G == 64) ? ~0ULL : (((1ULL << G) - 1) << (lane & ~(G - 1)));
    const int64_t nwords = (nrows + 63) >> 6;
    const bool rv = SR::reads_values && avals && uvals;
    X a0 = X(), u0 = X();
    if (rv) {
        if (a_iso) a0 = avals[0];
        if (u_iso) u0 = uvals[0];
    }
    unsigned long long mycount = 0;
    for (int64_t tile = blockIdx.x; tile * SPMV_TILE < nrows; tile += gridDim.x) {
        if (threadIdx.x < SPMV_TILE / 64) words[threadIdx.x] = 0;
        __syncthreads();
        const int64_t base = tile * SPMV_TILE;
        for (int rr = gid; rr < SPMV_TILE; rr += ngroups) {
            const int64_t r = base + rr;
            bool active = r < nrows;
            if (active && mbits) active = gb_bit(mbits, r) != mcomp;
            bool found = false;
            Z acc = Z();
            if (active) {
                const int64_t p1 = rowptr[r + 1];
                for (int64_t p = rowptr[r] + gl; p < p1; p += G) {
                    const int k = colidx[p];
                    bool term = false;
                    if (gb_bit(ubits, k)) {
                        X a = X(), b = X();
                        if (rv) {
                            a = a_iso ? a0 : avals[p];
                            b = u_iso ? u0 : uvals[k];
                        }
                        Z z = FLIP ? sr.mult(b, a, 0, k, r) : sr.mult(a, b, r, k, 0);
                        acc = found ? sr.add(acc, z) : z;
                        found = true;
                        term = sr.terminal(acc);
                    }
                    if (__ballot(term) & gmask) break;
                }
            }
            // reduce the group's partial results (all lanes reconverged here)
            for (int off = G >> 1; off > 0; off >>= 1) {
                bool of = __shfl_xor((int)found, off, 64);
                Z oa = gb_shfl_xor(acc, off, 64);
                if (of) {
                    acc = found ? ((gl & off) ? sr.add(oa, acc) : sr.add(acc, oa)) : oa;
                    found = true;
                }
            }
            if (gl == 0 && found) {
                if (tvals) tvals[r] = acc;
                atomicOr(&words[rr >> 6], 1ULL << (rr & 63));
            }
        }
        __syncthreads();
        if (threadIdx.x < SPMV_TILE / 64) {
            const int64_t w = (base >> 6) + threadIdx.x;
            if (w < nwords) {
                unsigned long long bitsw = words[threadIdx.x];
                tbits[w] = bitsw;
                mycount += __popcll(bitsw);
            }
        }
    }
    if (threadIdx.x < SPMV_TILE / 64 && mycount) atomicAdd(tcount, mycount);
}

// frontier size and edge count (push orientation) for the direction choice
__global__ void k_frontier_edges(const uint64_t *__restrict__ ubits, int64_t nwords, const int64_t *__restrict__ prow,
                                 gb_dir_state *__restrict__ st) {
    unsigned long long mf = 0, nf = 0;
    for (int64_t w = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; w < nwords;
         w += (int64_t)gridDim.x * blockDim.x) {
        uint64_t word = ubits[w];
        nf += __popcll(word);
        while (word) {
            int b = __ffsll((unsigned long long)word) - 1;
            word &= word - 1;
            int64_t k = (w << 6) + b;
            mf += prow[k + 1] - prow[k];
        }
    }
    for (int off = 32; off > 0; off >>= 1) {
        mf += __shfl_xor(mf, off, 64);
        nf += __shfl_xor(nf, off, 64);
    }
    if ((threadIdx.x & 63) == 0 && (mf || nf)) {
        atomicAdd(&st->mf, mf);
        atomicAdd(&st->nf, nf);
    }
}

// T(j) exists iff some k in u has A'(j,k): presence bits only (iso results).
// Work unit = (frontier word, part): P waves share each 64-vertex word and
// split every row of its set bits into strides of 64*P edges, so hub rows are
// spread over P waves.
__global__ __launch_bounds__(SPMV_BLOCK) void k_spmv_push_bits(
    int64_t nwords_u, const uint64_t *__restrict__ ubits, const int64_t *__restrict__ prow,
    const int32_t *__restrict__ pcol, const uint64_t *__restrict__ mbits, bool mcomp,
    unsigned long long *__restrict__ tbits, unsigned long long *__restrict__ tcount, int P,
    const gb_dir_state *__restrict__ st, const int64_t *__restrict__ mask_count, int64_t n_out, int64_t nnz,
    int64_t alpha) {
    if (st && !gb_choose_push(st, mask_count, mcomp, n_out, nnz, alpha)) return;
    const int lane = threadIdx.x & 63;
    const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
    const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
    unsigned long long added = 0;
    for (int64_t unit = wave; unit < nwords_u * P; unit += nwaves) {
        const int64_t w = unit / P;
        const int part = (int)(unit - w * P);
        uint64_t word = ubits[w];
        while (word) {
            const int b = __ffsll((unsigned long long)word) - 1;
            word &= word - 1;
            const int64_t k = (w << 6) + b;
            const int64_t p1 = prow[k + 1];
            for (int64_t p = prow[k] + (int64_t)part * 64 + lane; p < p1; p += (int64_t)P * 64) {
                const int32_t j = pcol[p];
                if (mbits && (gb_bit(mbits, j) == mcomp)) continue;
                const unsigned long long m = 1ULL << (j & 63);
                if (!(tbits[j >> 6] & m)) {
                    unsigned long long old = atomicOr(&tbits[j >> 6], m);
                    if (!(old & m)) added++;
                }
            }
        }
    }
    for (int off = 32; off > 0; off >>= 1) added += __shfl_xor(added, off, 64);
    if (lane == 0 && added) atomicAdd(tcount, added);
}

// constant value of an iso result: mult(a0, u0) (positional ops are never iso)
template <class SR, class X, class Z, bool FLIP>
__global__ void k_iso_value(SR sr, const X *avals, const X *uvals, Z *out) {
    X a = avals ? avals[0] : X(), b = uvals ? uvals[0] : X();
    *out = FLIP ? sr.mult(b, a, 0, 0, 0) : sr.mult(a, b, 0, 0, 0);
}

static bool idempotent_monoid(int m) {
    return m == GBAMD_MON_ANY || m == GBAMD_MON_MIN || m == GBAMD_MON_MAX || m == GBAMD_MON_LOR ||
           m == GBAMD_MON_LAND || m == GBAMD_MON_BOR || m == GBAMD_MON_BAND;
}

bool gb_spmv_result_iso(GrB_Semiring sr, bool a_iso, bool u_iso, bool flip) {
    gb_sr_info info = gb_sr_describe(sr);
    bool reads_a = info.reads_values, reads_u = info.reads_values;
    if (info.mul == GBAMD_OP_FIRST) (flip ? reads_a : reads_u) = false;
    if (info.mul == GBAMD_OP_SECOND) (flip ? reads_u : reads_a) = false;
    if (info.mul == GBAMD_OP_PAIR) return idempotent_monoid(info.mon);
    return !info.positional && idempotent_monoid(info.mon) && (!reads_a || a_iso) && (!reads_u || u_iso);
}

void gb_spmv(gb_vec_result &T, const gb_csr_view &A, const gb_csr_view *Apush, gb_bitmap_view &u,
             const gb_vmask &mask, GrB_Semiring sr, bool flip) {
    gb_sr_info info = gb_sr_describe(sr);
    gb_scratch s;
    gb_csr_view &Av = const_cast<gb_csr_view &>(A);
    const void *av = info.reads_values ? gb_view_vals_as(Av, info.xcode, s) : nullptr;
    const void *uv = info.reads_values ? gb_bitmap_vals_as(u, info.xcode, s) : nullptr;
    // which operand does the multiplier read?  (mxv: mult(A, u); vxm: mult(u, A))
    bool reads_a = info.reads_values, reads_u = info.reads_values;
    if (info.mul == GBAMD_OP_FIRST) (flip ? reads_a : reads_u) = false;
    if (info.mul == GBAMD_OP_SECOND) (flip ? reads_u : reads_a) = false;
    bool iso = !info.positional && idempotent_monoid(info.mon) && (!reads_a || A.iso) && (!reads_u || u.iso);
    if (info.mul == GBAMD_OP_PAIR) iso = idempotent_monoid(info.mon);

    const int64_t n = A.nrows;
    const size_t zs = gb_type_size(info.zcode);
    T.n = n;
    T.tcode = info.zcode;
    T.iso = iso;
    T.bits = gb_malloc_n<uint64_t>(gb_words(n));
    T.dense = gb_malloc((iso ? 1 : n) * zs);
    T.d_nvals = gb_malloc_n<int64_t>(1);
    gb_memset(T.d_nvals, 0, sizeof(int64_t));
    if (n == 0) return;

    int64_t avg = A.nrows ? (A.nvals + A.nrows - 1) / A.nrows : 1;
    int lg = 0;
    while (lg < 6 && (1LL << lg) < avg) lg++;
    int64_t forced = gb_knob("spmv_lg");
    if (forced > 0) lg = (int)(forced - 1);
    int64_t tiles = (n + SPMV_TILE - 1) / SPMV_TILE;
    unsigned grid = (unsigned)std::min<int64_t>(tiles, 2048);

    // direction-optimizing path: iso (presence-only) results with the other orientation available
    const int64_t dir_knob = gb_knob("spmv_direction");  // 0 auto, 1 pull only, 2 push only
    const bool can_push = iso && Apush && Apush->nrows == u.n && dir_knob != 1;
    gb_dir_state *st = nullptr;
    int64_t alpha = gb_knob("push_alpha");
    if (alpha <= 0) alpha = 14;
    if (can_push) {
        gb_memset(T.bits, 0, gb_words(n) * sizeof(uint64_t));
        if (dir_knob != 2) {
            st = s.get<gb_dir_state>(1);
            gb_memset(st, 0, sizeof(gb_dir_state));
            int64_t uw = gb_words(u.n);
            unsigned g = (unsigned)std::max<int64_t>(1, std::min<int64_t>((uw + 255) / 256, 1024));
            hipLaunchKernelGGL(k_frontier_edges, dim3(g), dim3(256), 0, gb_stream(), u.bits, uw, Apush->rowptr, st);
            GB_LAUNCH_CHECK();
        }
        int P = (int)gb_knob("push_parts");
        if (P <= 0) P = 8;
        int64_t units = gb_words(u.n) * P;
        unsigned pg = (unsigned)std::max<int64_t>(1, std::min<int64_t>((units + 3) / 4, 8192));
        hipLaunchKernelGGL(k_spmv_push_bits, dim3(pg), dim3(SPMV_BLOCK), 0, gb_stream(), gb_words(u.n), u.bits,
                           Apush->rowptr, Apush->colidx, mask.bits, mask.comp, (unsigned long long *)T.bits,
                           (unsigned long long *)T.d_nvals, P, st, mask.count, n, A.nvals, alpha);
        GB_LAUNCH_CHECK();
    }

    gb_dispatch_sr(info, [&](auto srf, auto x, auto z) {
        using SRT = decltype(srf);
        using X = decltype(x);
        using Z = decltype(z);
        Z *tvals = iso ? nullptr : (Z *)T.dense;
        if (!can_push || dir_knob != 2) {
            // with a push path enqueued, the pull kernel runs only if the device picks it
            const gb_dir_state *pst = can_push ? st : nullptr;
            if (flip)
                hipLaunchKernelGGL((k_spmv_pull<SRT, X, Z, true>), dim3(grid), dim3(SPMV_BLOCK), 0, gb_stream(), srf,
                                   n, A.rowptr, A.colidx, (const X *)av, A.iso, u.bits, (const X *)uv, u.iso,
                                   mask.bits, mask.comp, lg, T.bits, tvals, (unsigned long long *)T.d_nvals, pst,
                                   mask.count, A.nvals, alpha);
            else
                hipLaunchKernelGGL((k_spmv_pull<SRT, X, Z, false>), dim3(grid), dim3(SPMV_BLOCK), 0, gb_stream(), srf,
                                   n, A.rowptr, A.colidx, (const X *)av, A.iso, u.bits, (const X *)uv, u.iso,
                                   mask.bits, mask.comp, lg, T.bits, tvals, (unsigned long long *)T.d_nvals, pst,
                                   mask.count, A.nvals, alpha);
            GB_LAUNCH_CHECK();
        }
        if (iso) {
            if (flip)
                hipLaunchKernelGGL((k_iso_value<SRT, X, Z, true>), dim3(1), dim3(1), 0, gb_stream(), srf,
                                   (const X *)av, (const X *)uv, (Z *)T.dense);
            else
                hipLaunchKernelGGL((k_iso_value<SRT, X, Z, false>), dim3(1), dim3(1), 0, gb_stream(), srf,
                                   (const X *)av, (const X *)uv, (Z *)T.dense);
            GB_LAUNCH_CHECK();
        }
    });
}
