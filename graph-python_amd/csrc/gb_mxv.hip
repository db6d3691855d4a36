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
// (4 bitmap words).  G lanes (G = 1..64) share a row; their column-index loads
// are coalesced.  Output presence bits are assembled in LDS and written as
// whole 64-bit words; one counter atomic per block.
//
// Iso results (BFS lor_land / any_pair: only presence is computed) take the
// direction-optimised path, three launches per call:
//   k_dir_prep  frontier edge count m_f (block partials; the last block applies
//               Beamer's rule m_f * alpha < m_u on the device), hub chunks,
//               zeroed output, iso value;
//   k_push      top-down: each frontier row of the other orientation of A'
//               sets the bits of its unmasked targets with atomicOr; rows with
//               more than H edges are split into H-edge chunks over many waves;
//   k_pull_iso  bottom-up: one lane per output row, stop at the first k in u.
// The direction not chosen returns at once; no host round trip.
#include <mutex>

#include "gb_dispatch.cuh"
#include "gb_internal.h"

#define SPMV_BLOCK 256
#define SPMV_TILE 256
#define PREP_BLOCKS 256

template <class SR, class X, class Z, bool FLIP>
__global__ __launch_bounds__(SPMV_BLOCK) void k_spmv_pull(
    SR sr, int64_t nrows, const int64_t *__restrict__ rowptr, const int32_t *__restrict__ colidx,
    const X *__restrict__ avals, bool a_iso, const uint64_t *__restrict__ ubits,
    const X *__restrict__ uvals, bool u_iso, const uint64_t *__restrict__ mbits, bool mcomp, int lg,
    uint64_t *__restrict__ tbits, Z *__restrict__ tvals, unsigned long long *__restrict__ tcount) {
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
    gb_block_add(threadIdx.x < SPMV_TILE / 64 ? mycount : 0, tcount);
}

// ---------------------------------------------------------------- iso results (BFS)
// Persistent per-process state of the direction-optimised path (zeroed once;
// every gb_spmv leaves it as it found it):
//   [0] prep-block ticket (the last prep block resets it)
//   [1] chosen direction: 1 push, 0 pull (written by the last prep block)
//   [2] number of hub chunks listed by prep (reset by the pull kernel)
enum { ST_TICKET = 0, ST_PUSH = 1, ST_NCHUNKS = 2, ST_WORDS = 8 };

struct gb_dir_rule {
    const int64_t *mask_count;  // device count of set mask bits (nullptr: unknown)
    bool mcomp;
    int64_t n_out, nnz, alpha;
    int force_push;
};

// Prep: per-block (m_f, n_f) of the frontier in the push orientation; hub rows
// (more than H edges) are cut into H-edge chunks listed in `chunks`; zeroes the
// output bitmap and count; writes the iso result value.  The last block to
// finish sums the partials and applies Beamer's rule m_f * alpha < m_u.
template <class SR, class X, class Z, bool FLIP>
__global__ __launch_bounds__(SPMV_BLOCK) void k_dir_prep(
    SR sr, const uint64_t *__restrict__ ubits, int64_t nwords_u, const int64_t *__restrict__ prow, int64_t H,
    int64_t *__restrict__ chunks, unsigned long long *__restrict__ part, unsigned long long *__restrict__ state,
    uint64_t *__restrict__ tbits, int64_t nwords_out, unsigned long long *__restrict__ tcount, const X *avals,
    const X *uvals, Z *iso_out, gb_dir_rule rule) {
    unsigned long long mf = 0;
    const int64_t tid = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    const int64_t nthr = (int64_t)gridDim.x * blockDim.x;
    for (int64_t w = tid; w < nwords_u; w += nthr) {
        uint64_t word = ubits[w];
        while (word) {
            const int b = __ffsll((unsigned long long)word) - 1;
            word &= word - 1;
            const int64_t k = (w << 6) + b;
            const int64_t deg = prow[k + 1] - prow[k];
            mf += deg;
            if (deg > H) {
                const int64_t c = (deg + H - 1) / H;
                const int64_t base = (int64_t)atomicAdd(&state[ST_NCHUNKS], (unsigned long long)c);
                for (int64_t i = 0; i < c; i++) {
                    chunks[2 * (base + i)] = k;
                    chunks[2 * (base + i) + 1] = i;
                }
            }
        }
    }
    for (int64_t w = tid; w < nwords_out; w += nthr) tbits[w] = 0;
    if (tid == 0) {
        *tcount = 0;
        if (iso_out) {
            X a = avals ? avals[0] : X(), b = uvals ? uvals[0] : X();
            *iso_out = FLIP ? sr.mult(b, a, 0, 0, 0) : sr.mult(a, b, 0, 0, 0);
        }
    }
    __shared__ unsigned long long red[SPMV_BLOCK / 64];
    __shared__ int s_last;
    for (int off = 32; off > 0; off >>= 1) mf += __shfl_xor(mf, off, 64);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = mf;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long a = 0;
        for (int i = 0; i < SPMV_BLOCK / 64; i++) a += red[i];
        part[blockIdx.x] = a;
        __threadfence();
        s_last = atomicAdd(&state[ST_TICKET], 1ULL) == gridDim.x - 1;
    }
    __syncthreads();
    if (!s_last) return;
    // last block: every partial is visible (each was fenced before its ticket)
    __threadfence();
    unsigned long long v = 0;
    for (int i = threadIdx.x; i < (int)gridDim.x; i += blockDim.x) v += ((volatile unsigned long long *)part)[i];
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long total = 0;
        for (int i = 0; i < SPMV_BLOCK / 64; i++) total += red[i];
        int64_t open = rule.n_out;  // rows the pull kernel would visit
        if (rule.mask_count) {
            const int64_t mc = *rule.mask_count;
            open = rule.mcomp ? (rule.n_out - mc) : mc;
        }
        const double avg = rule.n_out ? (double)rule.nnz / (double)rule.n_out : 0.0;
        const bool push = rule.force_push || ((double)total * (double)rule.alpha < (double)open * avg);
        state[ST_PUSH] = push ? 1ULL : 0ULL;
        state[ST_TICKET] = 0;
    }
}

// set output bits for edges [p0, p1) of one row; 4 loads in flight per lane
__device__ __forceinline__ unsigned long long gb_push_range(int64_t p0, int64_t p1, int lane,
                                                            const int32_t *__restrict__ pcol,
                                                            const uint64_t *__restrict__ mbits, bool mcomp,
                                                            unsigned long long *__restrict__ tbits) {
    unsigned long long added = 0;
    for (int64_t p = p0 + lane; p < p1; p += 256) {
        int32_t j[4];
        bool ok[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const int64_t q = p + 64 * u;
            ok[u] = q < p1;
            j[u] = ok[u] ? pcol[q] : 0;
        }
        if (mbits) {
#pragma unroll
            for (int u = 0; u < 4; u++)
                if (ok[u]) ok[u] = gb_bit(mbits, j[u]) != mcomp;
        }
        unsigned long long cur[4];
#pragma unroll
        for (int u = 0; u < 4; u++) cur[u] = ok[u] ? tbits[j[u] >> 6] : ~0ULL;
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const unsigned long long m = 1ULL << (j[u] & 63);
            if (ok[u] && !(cur[u] & m)) {
                unsigned long long old = atomicOr(&tbits[j[u] >> 6], m);
                if (!(old & m)) added++;
            }
        }
    }
    return added;
}

// Push (top-down): units [0, nchunks) are hub chunks, then one unit per
// frontier word (its rows of at most H edges).  One wave per unit.
__global__ __launch_bounds__(SPMV_BLOCK) void k_push(
    int64_t nwords_u, const uint64_t *__restrict__ ubits, const int64_t *__restrict__ prow,
    const int32_t *__restrict__ pcol, const uint64_t *__restrict__ mbits, bool mcomp,
    unsigned long long *__restrict__ tbits, unsigned long long *__restrict__ tcount,
    const int64_t *__restrict__ chunks, const unsigned long long *__restrict__ state, int64_t H) {
    if (!state[ST_PUSH]) return;
    const int lane = threadIdx.x & 63;
    const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
    const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
    const int64_t nch = (int64_t)state[ST_NCHUNKS];
    unsigned long long added = 0;
    for (int64_t unit = wave; unit < nch + nwords_u; unit += nwaves) {
        if (unit < nch) {
            const int64_t k = chunks[2 * unit], c = chunks[2 * unit + 1];
            const int64_t p0 = prow[k] + c * H, pe = prow[k + 1];
            added += gb_push_range(p0, (p0 + H < pe) ? p0 + H : pe, lane, pcol, mbits, mcomp, tbits);
            continue;
        }
        const int64_t w = unit - nch;
        uint64_t word = ubits[w];
        while (word) {
            const int b = __ffsll((unsigned long long)word) - 1;
            word &= word - 1;
            const int64_t k = (w << 6) + b;
            const int64_t p0 = prow[k], p1 = prow[k + 1];
            if (p1 - p0 > H) continue;  // a hub: done by its chunks
            added += gb_push_range(p0, p1, lane, pcol, mbits, mcomp, tbits);
        }
    }
    gb_block_add(added, tcount);
}

// Pull (bottom-up) for iso results: only presence is computed.  One wave per
// 64-row bitmap word, one lane per row: a lane walks its own row two edges a
// step (neighbouring rows are neighbouring in colidx, so the loads coalesce),
// stopping at the first k present in u; rows still open after 8 edges are
// finished by the whole wave, one row at a time, 256 edges a step.
__global__ __launch_bounds__(SPMV_BLOCK) void k_pull_iso(
    int64_t nrows, const int64_t *__restrict__ rowptr, const int32_t *__restrict__ colidx,
    const uint64_t *__restrict__ ubits, const uint64_t *__restrict__ mbits, bool mcomp, uint64_t *__restrict__ tbits,
    unsigned long long *__restrict__ tcount, unsigned long long *__restrict__ state) {
    if (state) {
        if (blockIdx.x == 0 && threadIdx.x == 0) state[ST_NCHUNKS] = 0;  // k_push is done with it
        if (state[ST_PUSH]) return;
    }
    const int lane = threadIdx.x & 63;
    const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
    const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
    const int64_t nwords = (nrows + 63) >> 6;
    unsigned long long cnt = 0;
    for (int64_t w = wave; w < nwords; w += nwaves) {
        uint64_t act = ~0ULL;
        if (mbits) act = mcomp ? ~mbits[w] : mbits[w];
        if (w == nwords - 1 && (nrows & 63)) act &= (1ULL << (nrows & 63)) - 1;
        if (act == 0) {
            if (lane == 0) tbits[w] = 0;
            continue;
        }
        const int64_t r = (w << 6) + lane;
        const bool live = (act >> lane) & 1ULL;
        int64_t p = 0, p1 = 0;
        if (live) {
            p = rowptr[r];
            p1 = rowptr[r + 1];
        }
        bool found = false;
        for (int it = 0; it < 4; it++) {
            const bool go = live && !found && p < p1;
            if (!__ballot(go)) break;
            if (go) {
                const int k0 = colidx[p];
                const int k1 = (p + 1 < p1) ? colidx[p + 1] : k0;
                found = (gb_bit(ubits, k0) + gb_bit(ubits, k1)) != 0;
                p += 2;
            }
        }
        unsigned long long pend = __ballot(live && !found && p < p1);
        while (pend) {
            const int l = __ffsll(pend) - 1;
            pend &= pend - 1;
            const int64_t q0 = __shfl(p, l, 64), q1 = __shfl(p1, l, 64);
            bool f = false;
            for (int64_t q = q0 + lane; q < q1; q += 256) {
                int j[4];
#pragma unroll
                for (int u = 0; u < 4; u++) j[u] = (q + 64 * u < q1) ? colidx[q + 64 * u] : -1;
#pragma unroll
                for (int u = 0; u < 4; u++) f = f || (j[u] >= 0 && gb_bit(ubits, j[u]));
                if (__ballot(f)) break;
            }
            if (__ballot(f) && lane == l) found = true;
        }
        const unsigned long long word = __ballot(found);
        if (lane == 0) {
            tbits[w] = word;
            cnt += __popcll(word);
        }
    }
    gb_block_add(cnt, tcount);
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

// the persistent direction state (see k_dir_prep), allocated and zeroed once
static std::mutex g_dir_mu;
static unsigned long long *gb_dir_state() {
    static unsigned long long *st = nullptr;
    if (!st) {
        GB_HIP(hipMalloc(&st, ST_WORDS * sizeof(unsigned long long)));
        GB_HIP(hipMemset(st, 0, ST_WORDS * sizeof(unsigned long long)));
        GB_HIP(hipDeviceSynchronize());
    }
    return st;
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
    const bool iso = gb_spmv_result_iso(sr, A.iso, u.iso, flip);

    const int64_t n = A.nrows;
    const size_t zs = gb_type_size(info.zcode);
    T.n = n;
    T.tcode = info.zcode;
    T.iso = iso;
    T.bits = gb_malloc_n<uint64_t>(gb_words(n));
    T.dense = gb_malloc((iso ? 1 : n) * zs);
    T.d_nvals = gb_malloc_n<int64_t>(1);
    if (n == 0) {
        gb_memset(T.d_nvals, 0, sizeof(int64_t));
        return;
    }

    const int64_t dir_knob = gb_knob("spmv_direction");  // 0 auto, 1 pull only, 2 push only
    const bool can_push = iso && Apush && Apush->nrows == u.n && dir_knob != 1;
    int64_t alpha = gb_knob("push_alpha");
    if (alpha <= 0) alpha = 14;
    int64_t H = gb_knob("push_heavy");
    if (H <= 0) H = 2048;
    const int64_t nw = gb_words(n);
    const unsigned iso_grid = (unsigned)std::min<int64_t>((nw + 3) / 4, 8192);

    gb_dispatch_sr(info, [&](auto srf, auto x, auto z) {
        using SRT = decltype(srf);
        using X = decltype(x);
        using Z = decltype(z);
        if (can_push) {
            // prep -> push -> pull, one direction doing the work; the other returns at once
            std::lock_guard<std::mutex> lk(g_dir_mu);  // keeps the three launches adjacent
            unsigned long long *state = gb_dir_state();
            const int64_t uw = gb_words(u.n);
            unsigned long long *part = s.get<unsigned long long>(PREP_BLOCKS);
            int64_t *chunks = s.get<int64_t>(2 * (2 * (Apush->nvals / H) + 2));
            gb_dir_rule rule{mask.count, mask.comp, n, A.nvals, alpha, dir_knob == 2};
            if (flip)
                hipLaunchKernelGGL((k_dir_prep<SRT, X, Z, true>), dim3(PREP_BLOCKS), dim3(SPMV_BLOCK), 0, gb_stream(),
                                   srf, u.bits, uw, Apush->rowptr, H, chunks, part, state, T.bits, nw,
                                   (unsigned long long *)T.d_nvals, (const X *)av, (const X *)uv, (Z *)T.dense,
                                   rule);
            else
                hipLaunchKernelGGL((k_dir_prep<SRT, X, Z, false>), dim3(PREP_BLOCKS), dim3(SPMV_BLOCK), 0,
                                   gb_stream(), srf, u.bits, uw, Apush->rowptr, H, chunks, part, state, T.bits, nw,
                                   (unsigned long long *)T.d_nvals, (const X *)av, (const X *)uv, (Z *)T.dense,
                                   rule);
            GB_LAUNCH_CHECK();
            const unsigned pgrid = (unsigned)std::max<int64_t>(1, std::min<int64_t>((uw + 3) / 4, 2048));
            hipLaunchKernelGGL(k_push, dim3(pgrid), dim3(SPMV_BLOCK), 0, gb_stream(), uw, u.bits, Apush->rowptr,
                               Apush->colidx, mask.bits, mask.comp, (unsigned long long *)T.bits,
                               (unsigned long long *)T.d_nvals, chunks, state, H);
            GB_LAUNCH_CHECK();
            hipLaunchKernelGGL(k_pull_iso, dim3(iso_grid), dim3(SPMV_BLOCK), 0, gb_stream(), n, A.rowptr, A.colidx,
                               u.bits, mask.bits, mask.comp, T.bits, (unsigned long long *)T.d_nvals, state);
            GB_LAUNCH_CHECK();
            return;
        }
        gb_memset(T.d_nvals, 0, sizeof(int64_t));
        if (iso) {
            hipLaunchKernelGGL(k_pull_iso, dim3(iso_grid), dim3(SPMV_BLOCK), 0, gb_stream(), n, A.rowptr, A.colidx,
                               u.bits, mask.bits, mask.comp, T.bits, (unsigned long long *)T.d_nvals,
                               (unsigned long long *)nullptr);
            GB_LAUNCH_CHECK();
            if (flip)
                hipLaunchKernelGGL((k_iso_value<SRT, X, Z, true>), dim3(1), dim3(1), 0, gb_stream(), srf,
                                   (const X *)av, (const X *)uv, (Z *)T.dense);
            else
                hipLaunchKernelGGL((k_iso_value<SRT, X, Z, false>), dim3(1), dim3(1), 0, gb_stream(), srf,
                                   (const X *)av, (const X *)uv, (Z *)T.dense);
            GB_LAUNCH_CHECK();
            return;
        }
        // general semiring: G lanes per row, G from the average row length
        const int64_t avg = (A.nvals + n - 1) / n;
        int lg = 0;
        while (lg < 6 && (1LL << lg) < avg) lg++;
        const int64_t forced = gb_knob("spmv_lg");
        if (forced > 0) lg = (int)(forced - 1);
        const unsigned grid = (unsigned)std::min<int64_t>((n + SPMV_TILE - 1) / SPMV_TILE, 2048);
        if (flip)
            hipLaunchKernelGGL((k_spmv_pull<SRT, X, Z, true>), dim3(grid), dim3(SPMV_BLOCK), 0, gb_stream(), srf, n,
                               A.rowptr, A.colidx, (const X *)av, A.iso, u.bits, (const X *)uv, u.iso, mask.bits,
                               mask.comp, lg, T.bits, (Z *)T.dense, (unsigned long long *)T.d_nvals);
        else
            hipLaunchKernelGGL((k_spmv_pull<SRT, X, Z, false>), dim3(grid), dim3(SPMV_BLOCK), 0, gb_stream(), srf, n,
                               A.rowptr, A.colidx, (const X *)av, A.iso, u.bits, (const X *)uv, u.iso, mask.bits,
                               mask.comp, lg, T.bits, (Z *)T.dense, (unsigned long long *)T.d_nvals);
        GB_LAUNCH_CHECK();
    });
}
