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
// direction-optimised path, two launches per call:
//   k_dir_prep  frontier edge count m_f (grid-wide sum; the block completing it
//               applies Beamer's rule m_f * alpha < m_u on the device), zeroed
//               output, iso value;
//   k_iso_work  the chosen direction --
//     push (top-down): each frontier row of the other orientation of A' sets
//       the bits of its unmasked targets with atomicOr; a wave spreads the
//       rows of one frontier word over its lanes; rows longer than H are cut
//       into H-edge chunks (a table cached on the matrix) spread over waves;
//     pull (bottom-up): one lane per output row, stop at the first k in u.
// No host round trip is needed for the choice.
#include <mutex>

#include "gb_dispatch.cuh"
#include "gb_internal.h"

#define SPMV_BLOCK 256
#define SPMV_TILE 256

template <class SR, class X, class Z, bool FLIP>
__global__ __launch_bounds__(SPMV_BLOCK) void k_spmv_pull(
    SR sr, int64_t nrows, const int64_t *__restrict__ rowptr, const int32_t *__restrict__ colidx,
    const X *__restrict__ avals, bool a_iso, const uint64_t *__restrict__ ubits,
    const X *__restrict__ uvals, bool u_iso, const uint64_t *__restrict__ mbits, bool mcomp, int lg,
    uint64_t *__restrict__ tbits, Z *__restrict__ tvals, unsigned long long *__restrict__ tcount,
    unsigned long long *__restrict__ gst) {
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
    gb_grid_add(threadIdx.x < SPMV_TILE / 64 ? (long long)mycount : 0, tcount, gst);
}

// ---------------------------------------------------------------- iso results (BFS)
// Direction state words (gb_state.h, GB_DIR_STATE_OFFSET; zero between calls
// except ST_PUSH, which every prep rewrites):
//   [ST_PUSH]     chosen direction: 1 push, 0 pull (written by the last prep block)
enum { ST_PUSH = 0 };
#define PULL_U 4  // bitmap words per wave step (independent loads in flight)

struct gb_dir_rule {
    const int64_t *mask_count;  // device count of set mask bits (nullptr: unknown)
    const int64_t *extra_count; // entries a fused assign adds to the mask (upper bound; nullptr: none)
    bool mcomp;
    int64_t n_out, nnz, alpha;
    int force_push;
};

// Beamer's rule: push while the frontier's edges m_f (times alpha) are fewer
// than the edges the pull would examine, estimated as open rows x average degree
__device__ __forceinline__ bool gb_dir_decide(long long mf, const gb_dir_rule &rule) {
    int64_t open = rule.n_out;  // rows the pull kernel would visit
    if (rule.mask_count) {
        int64_t mc = *rule.mask_count;
        if (rule.extra_count) mc += *rule.extra_count;
        if (mc > rule.n_out) mc = rule.n_out;
        open = rule.mcomp ? (rule.n_out - mc) : mc;
    }
    const double avg = rule.n_out ? (double)rule.nnz / (double)rule.n_out : 0.0;
    return rule.force_push || ((double)mf * (double)rule.alpha < (double)open * avg);
}

// Prep: m_f = edges of the frontier in the push orientation (one lane per
// frontier bit); zeroes the output bitmap and count; writes the iso result
// value.  The block that completes the grid-wide sum of m_f applies
// Beamer's rule m_f * alpha < m_u and stores the direction.
template <class SR, class X, class Z, bool FLIP>
__global__ __launch_bounds__(SPMV_BLOCK) void k_dir_prep(
    SR sr, const uint64_t *__restrict__ ubits, int64_t nwords_u, const int64_t *__restrict__ prow,
    unsigned long long *__restrict__ gst, unsigned long long *__restrict__ dst,
    uint64_t *__restrict__ tbits, int64_t nwords_out, unsigned long long *__restrict__ tcount, const X *avals,
    const X *uvals, Z *iso_out, gb_dir_rule rule) {
    const int lane = threadIdx.x & 63;
    const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
    const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
    long long mf = 0;
    // 16 frontier words per wave step (lanes 0-15 load them); the non-zero ones
    // are expanded one lane per bit, four words at a time
    for (int64_t base = wave * 16; base < nwords_u; base += nwaves * 16) {
        const int64_t wl = base + (lane & 15);
        const uint64_t mine = wl < nwords_u ? ubits[wl] : 0;
        unsigned long long nz = __ballot(mine != 0) & 0xFFFFULL;
        while (nz) {
            int64_t deg[4];
#pragma unroll
            for (int u = 0; u < 4; u++) {
                deg[u] = 0;
                if (nz) {
                    const int l = __ffsll(nz) - 1;
                    nz &= nz - 1;
                    const uint64_t word = __shfl(mine, l, 64);
                    if ((word >> lane) & 1ULL) {
                        const int64_t k = ((base + l) << 6) + lane;
                        deg[u] = prow[k + 1] - prow[k];
                    }
                }
            }
#pragma unroll
            for (int u = 0; u < 4; u++) mf += deg[u];
        }
    }
    const int64_t tid = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    for (int64_t w = tid; w < nwords_out; w += (int64_t)gridDim.x * blockDim.x) tbits[w] = 0;
    if (tid == 0) {
        *tcount = 0;
        if (iso_out) {
            X a = avals ? avals[0] : X(), b = uvals ? uvals[0] : X();
            *iso_out = FLIP ? sr.mult(b, a, 0, 0, 0) : sr.mult(a, b, 0, 0, 0);
        }
    }
    long long total;
    if (gb_grid_sum(mf, gst, &total)) dst[ST_PUSH] = gb_dir_decide(total, rule) ? 1ULL : 0ULL;
}

// set the output bits of up to 4 targets per lane (unmasked, not yet set);
// returns how many bits this lane turned on
__device__ __forceinline__ long long gb_push_targets(const int32_t (&j)[4], bool (&ok)[4],
                                                     const uint64_t *__restrict__ mbits, bool mcomp,
                                                     unsigned long long *__restrict__ tbits,
                                                     const int64_t *__restrict__ hprow, long long &mfn,
                                                     const uint64_t *__restrict__ qbits, bool serial = false,
                                                     int64_t qroot = -1) {
    unsigned long long cur[4];
    if (serial) {  // diagnostics (iso_dbg 128): the round-4 order, each read behind the one before
        if (mbits) {
#pragma unroll
            for (int u = 0; u < 4; u++)
                if (ok[u]) ok[u] = (gb_bit(mbits, j[u]) || (qbits && gb_bit(qbits, j[u]))) != mcomp;
        }
#pragma unroll
        for (int u = 0; u < 4; u++) cur[u] = ok[u] ? tbits[j[u] >> 6] : ~0ULL;
    } else {
        // the mask words (w's and the fused stamp's q) and the output word of every target
        // are read at once: one round trip instead of three dependent ones
        uint64_t mw[4], qw[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            mw[u] = qw[u] = 0;
            cur[u] = ~0ULL;
            if (ok[u]) {
                if (mbits) mw[u] = mbits[j[u] >> 6];
                if (mbits && qbits) qw[u] = qbits[j[u] >> 6];
                cur[u] = tbits[j[u] >> 6];
            }
        }
        if (mbits) {
            // qroot: the fused stamp's frontier is one pending vertex (gb_push_root), not q's bits
#pragma unroll
            for (int u = 0; u < 4; u++)
                if (ok[u]) ok[u] = (((((mw[u] | qw[u]) >> (j[u] & 63)) & 1ULL) != 0) || j[u] == qroot) != mcomp;
        }
    }
    long long added = 0;
#pragma unroll
    for (int u = 0; u < 4; u++) {
        const unsigned long long m = 1ULL << (j[u] & 63);
        if (ok[u] && !(cur[u] & m)) {
            const unsigned long long old = atomicOr(&tbits[j[u] >> 6], m);
            if (!(old & m)) {
                added++;
                if (hprow) mfn += hprow[j[u] + 1] - hprow[j[u]];  // edges of the next frontier
            }
        }
    }
    return added;
}

// ------------------------------------------------ wave-level segment lists (LDS)
// A wave gathers up to WL_MAX row segments (start, length) into its own LDS
// area, takes a prefix sum of the lengths and then walks the concatenated
// edges 256 at a time, four independent loads per lane; a lane finds the
// segment of its edge by binary search over the prefix.  This keeps every lane
// busy whatever the mix of row lengths (no lane-per-row tail, no wave per row).
#define WL_MAX 256
#define WAVES_PER_BLOCK (SPMV_BLOCK / 64)
struct gb_wlist {
    int64_t p[WL_MAX];    // next edge position of the segment
    int32_t rem[WL_MAX];  // edges left in the row
    int32_t pref[WL_MAX]; // inclusive prefix of this round's lengths
    int16_t id[WL_MAX];   // u * 64 + lane of the row (pull)
    int8_t hit[WL_MAX];   // a k present in u was found this round
    unsigned long long hitw[PULL_U];  // pull: rows of the unit's words found through the list
};

// this round takes min(rem[i], cap) edges of segment i; hit[i] = 0; pref = inclusive
// prefix of the taken lengths; returns the total
__device__ __forceinline__ int gb_wlist_round(gb_wlist &L, int n, int cap, int lane) {
    int v[4], sum = 0;
#pragma unroll
    for (int t = 0; t < 4; t++) {
        const int i = lane * 4 + t;
        v[t] = 0;
        if (i < n) {
            v[t] = L.rem[i] < cap ? L.rem[i] : cap;
            L.hit[i] = 0;
        }
        sum += v[t];
    }
    int incl = sum;
    for (int off = 1; off < 64; off <<= 1) {
        const int y = __shfl_up(incl, off, 64);
        if (lane >= off) incl += y;
    }
    int run = incl - sum;
#pragma unroll
    for (int t = 0; t < 4; t++) {
        const int i = lane * 4 + t;
        run += v[t];
        if (i < n) L.pref[i] = run;
    }
    gb_wave_sync();
    return __shfl(incl, 63, 64);
}

// start of segment i's edges in the concatenated stream
__device__ __forceinline__ int gb_wlist_start(const gb_wlist &L, int i) { return i ? L.pref[i - 1] : 0; }

// segment of concatenated edge e: first i with pref[i] > e (n <= WL_MAX)
__device__ __forceinline__ int gb_wlist_find(const gb_wlist &L, int n, int e) {
    int lo = 0;
#pragma unroll
    for (int st = WL_MAX / 2; st > 0; st >>= 1)
        if (lo + st <= n && L.pref[lo + st - 1] <= e) lo += st;
    return lo;
}

// The fused assign (gb_asg) for the 4 words w0..w0+3 of q (lanes 0-3 hold word
// w0 + (lane & 3) in qw): w's presence words |= q, w's value at each q bit = x
// (one lane per position: coalesced stores); returns the entries added to w.
struct gb_asg_dev {
    uint64_t *bits;
    void *vals;
    int size;
    unsigned long long x;
};
__device__ __forceinline__ void gb_store_sized(void *base, int64_t i, int size, unsigned long long x) {
    switch (size) {
    case 1: ((uint8_t *)base)[i] = (uint8_t)x; break;
    case 2: ((uint16_t *)base)[i] = (uint16_t)x; break;
    case 4: ((uint32_t *)base)[i] = (uint32_t)x; break;
    default: ((unsigned long long *)base)[i] = x; break;
    }
}
// cpre: w's word already read by the caller (nullptr: read it here)
__device__ __forceinline__ long long gb_asg_words(const gb_asg_dev &g, int64_t w0, int64_t nwords, uint64_t qw,
                                                 int lane, const uint64_t *cpre = nullptr) {
    long long added = 0;
    const int64_t wl = w0 + (lane & 3);
    if (lane < 4 && wl < nwords && qw) {
        const uint64_t c = cpre ? *cpre : g.bits[wl], nwd = c | qw;
        if (nwd != c) g.bits[wl] = nwd;
        added = (long long)__popcll(nwd) - (long long)__popcll(c);
    }
#pragma unroll
    for (int u = 0; u < 4; u++) {
        const uint64_t word = __shfl(qw, u, 64);
        if ((word >> lane) & 1ULL) gb_store_sized(g.vals, ((w0 + u) << 6) + lane, g.size, g.x);
    }
    return added;
}

// Push (top-down).  First the matrix's hub chunks (rows longer than H cut into
// H-edge pieces, a static table; a wave tests 16 strided entries against the
// frontier at once and expands the hits, 256 edges a step).  Then the frontier
// words, 4 per wave step: the rows of their frontier vertices (at most H edges
// each) go into the wave's segment list and are walked as one edge stream.
__device__ __forceinline__ long long gb_push_phase(int64_t nwords_u, const uint64_t *__restrict__ ubits,
                                                  const int64_t *__restrict__ prow, const int32_t *__restrict__ pcol,
                                                  const int32_t *__restrict__ hubs, int64_t nhubs, int64_t H,
                                                  const uint64_t *__restrict__ mbits, bool mcomp,
                                                  unsigned long long *__restrict__ tbits, gb_wlist &L,
                                                  const int64_t *__restrict__ hprow, long long &mfn,
                                                  const uint64_t *__restrict__ qbits, const gb_asg_dev &g,
                                                  long long &adelta, bool serial = false, bool prefetch = true) {
    const int lane = threadIdx.x & 63;
    const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
    const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
    const unsigned long long lt = (1ULL << lane) - 1;
    long long added = 0;
    // the frontier words of this wave's first 16 steps, loaded before the hub chunks (round 5):
    // lane l holds step l / 4's word l % 4, so a small frontier's scan costs one load round trip
    // (overlapped with the hub test's) instead of one per step -- with one wave of workgroups a
    // wave takes nwords / (4 * waves) steps, 4 at s22
    uint64_t pre = 0;
    {
        const int64_t wl = wave * 4 + (int64_t)(lane >> 2) * nwaves * 4 + (lane & 3);
        if (wl < nwords_u) pre = ubits[wl];
    }
    // hub chunks: lane l of wave w tests table entry w + l * nwaves (a hub's
    // consecutive chunks land on different waves); hits are expanded in turn
    for (int64_t base = wave; base < nhubs; base += nwaves * 16) {
        const int64_t h = base + (int64_t)lane * nwaves;
        int k = 0, cc = 0;
        bool act = false;
        if (lane < 16 && h < nhubs) {
            k = hubs[2 * h];
            cc = hubs[2 * h + 1];
            act = gb_bit(ubits, k);
        }
        unsigned long long b = __ballot(act);
        while (b) {
            const int l = __ffsll(b) - 1;
            b &= b - 1;
            const int64_t kk = __shfl(k, l, 64);
            const int64_t c = __shfl(cc, l, 64);
            const int64_t p0 = prow[kk] + c * H, pe = prow[kk + 1];
            const int64_t p1 = (p0 + H < pe) ? p0 + H : pe;
            for (int64_t p = p0 + lane; p < p1; p += 256) {
                int32_t j[4];
                bool ok[4];
#pragma unroll
                for (int u = 0; u < 4; u++) {
                    ok[u] = p + 64 * u < p1;
                    j[u] = ok[u] ? pcol[p + 64 * u] : 0;
                }
                added += gb_push_targets(j, ok, mbits, mcomp, tbits, hprow, mfn, qbits, serial);
            }
        }
    }
    // frontier words, 4 per wave step (lanes 0-3 load them; the first 16 steps' came above)
    int step = 0;
    for (int64_t w0 = wave * 4; w0 < nwords_u; w0 += nwaves * 4, step++) {
        const int64_t wl = w0 + (lane & 3);
        uint64_t mine;
        if (prefetch && step < 16) {
            mine = __shfl(pre, (step << 2) | (lane & 3), 64);
        } else {
            mine = wl < nwords_u ? ubits[wl] : 0;
        }
        if (!__ballot(mine != 0)) continue;
        if (qbits) adelta += gb_asg_words(g, w0, nwords_u, mine, lane);
        int64_t p0[4], d[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const uint64_t word = __shfl(mine, u, 64);
            p0[u] = d[u] = 0;
            if ((word >> lane) & 1ULL) {
                const int64_t k = ((w0 + u) << 6) + lane;
                p0[u] = prow[k];
                d[u] = prow[k + 1] - p0[u];
            }
        }
        int n = 0;
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const bool in = d[u] > 0 && d[u] <= H;  // hubs: done by their chunks
            const unsigned long long bb = __ballot(in);
            if (in) {
                const int i = n + __popcll(bb & lt);
                L.p[i] = p0[u];
                L.rem[i] = (int32_t)d[u];
            }
            n += __popcll(bb);
        }
        if (!n) continue;
        gb_wave_sync();
        const int total = gb_wlist_round(L, n, 1 << 30, lane);
        for (int e0 = 0; e0 < total; e0 += 256) {
            int32_t j[4];
            bool ok[4];
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const int e = e0 + lane + 64 * u;
                ok[u] = e < total;
                j[u] = 0;
                if (ok[u]) {
                    const int s = gb_wlist_find(L, n, e);
                    j[u] = pcol[L.p[s] + (e - gb_wlist_start(L, s))];
                }
            }
            added += gb_push_targets(j, ok, mbits, mcomp, tbits, hprow, mfn, qbits, serial);
        }
        gb_wave_sync();
    }
    return added;
}

// Push from a single pending vertex (the BFS root, gb_internal.h g_root_active): the host knows
// the frontier is {root}, so the kernel neither tests the hub table against the frontier nor
// scans its bitmap words (which do not hold the root) -- the root's edges are spread over the
// whole grid, 4 per lane per step, and block 0 carries out the fused stamp v<q> = x for it.
// Replaces the single-thread set launch and the first level's two scan round trips.
__device__ __forceinline__ long long gb_push_root(int64_t root, const int64_t *__restrict__ prow,
                                                 const int32_t *__restrict__ pcol,
                                                 const uint64_t *__restrict__ mbits, bool mcomp,
                                                 unsigned long long *__restrict__ tbits,
                                                 const int64_t *__restrict__ hprow, long long &mfn, bool stamp,
                                                 const gb_asg_dev &g, long long &adelta) {
    const int lane = threadIdx.x & 63;
    const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
    const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
    if (stamp && blockIdx.x == 0 && threadIdx.x == 0) {
        const unsigned long long m = 1ULL << (root & 63);
        const unsigned long long old = atomicOr((unsigned long long *)&g.bits[root >> 6], m);
        gb_store_sized(g.vals, root, g.size, g.x);
        if (!(old & m)) adelta += 1;
    }
    const int64_t p0 = prow[root], p1 = prow[root + 1];
    long long added = 0;
    for (int64_t p = p0 + wave * 256 + lane; p < p1; p += nwaves * 256) {
        int32_t j[4];
        bool ok[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            ok[u] = p + 64 * u < p1;
            j[u] = ok[u] ? pcol[p + 64 * u] : 0;
        }
        added += gb_push_targets(j, ok, mbits, mcomp, tbits, hprow, mfn, nullptr, false, stamp ? root : -1);
    }
    return added;
}

// Pull (bottom-up) for iso results: only presence is computed.  A wave takes
// PULL_U 64-row bitmap words at a time, one lane per row of each: a lane walks
// its own rows four edges a step (neighbouring rows are neighbouring in colidx,
// so the loads coalesce), stopping at the first k present in u.  Rows still
// open after 8 edges go into the wave's segment list and are walked as one
// edge stream in rounds (at most `cap` edges per row per round, cap doubling),
// dropping the rows that found a k after each round.
__device__ __forceinline__ long long gb_pull_iso_phase(int64_t nrows, const int64_t *__restrict__ rowptr,
                                                      const int32_t *__restrict__ colidx,
                                                      const uint64_t *__restrict__ ubits,
                                                      const uint64_t *__restrict__ mbits, bool mcomp,
                                                      uint64_t *__restrict__ tbits, gb_wlist &L,
                                                      const int64_t *__restrict__ hprow, long long &mfn,
                                                      int p1_steps, int cap0, const uint64_t *__restrict__ rne,
                                                      const uint64_t *__restrict__ qbits, const gb_asg_dev &g,
                                                      long long &adelta, int dbg = 0,
                                                      const int32_t *__restrict__ ph = nullptr,
                                                      const uint32_t *__restrict__ pdeg = nullptr) {
    const int lane = threadIdx.x & 63;
    const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
    const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
    const int64_t nwords = (nrows + 63) >> 6;
    const uint64_t tail = (nrows & 63) ? ((1ULL << (nrows & 63)) - 1) : ~0ULL;
    const unsigned long long lt = (1ULL << lane) - 1;
    long long cnt = 0;
    for (int64_t w0 = wave * PULL_U; w0 < nwords; w0 += nwaves * PULL_U) {
        const int64_t wl = w0 + (lane & (PULL_U - 1));
        const bool inr = wl < nwords;
        // the step's words read together (the stamp's q, the mask, the rows with entries): the
        // stamp's store no longer orders the mask read behind it
        const uint64_t qw = (qbits && inr) ? qbits[wl] : 0;
        const uint64_t mw = (mbits && inr) ? mbits[wl] : 0;
        const uint64_t rw = (rne && inr) ? rne[wl] : ~0ULL;
        uint64_t mine = ~0ULL;
        if (qbits) {  // fused assign: w |= q; the mask is w's structure after it
            adelta += gb_asg_words(g, w0, nwords, qw, lane, g.bits == mbits ? &mw : nullptr);
            if (mbits) mine = inr ? (mcomp ? ~(mw | qw) : (mw | qw)) : 0;
        } else if (mbits) {
            mine = inr ? (mcomp ? ~mw : mw) : 0;
        }
        if (rne && inr) mine &= rw;  // rows without entries produce nothing
        if (wl == nwords - 1) mine &= tail;
        if (wl >= nwords) mine = 0;
        if (!__ballot(mine != 0)) {  // nothing open in these words
            if (lane < PULL_U && wl < nwords) tbits[wl] = 0;
            continue;
        }
        bool live[PULL_U], found[PULL_U];
        int64_t p[PULL_U], p1[PULL_U];
        int64_t dg[PULL_U];
#pragma unroll
        for (int u = 0; u < PULL_U; u++) {
            live[u] = (__shfl(mine, u, 64) >> lane) & 1ULL;
            found[u] = false;
        }
        if (ph) {
            // pull heads: each open row first tests its best-connected neighbours (one coalesced
            // 16-byte load per row); rows they settle, and rows of at most 4 entries, never read
            // their bounds or edges -- the dependent row-pointer / edge round trips are left to
            // the long rows that found nothing
            int4 hv[PULL_U];
#pragma unroll
            for (int u = 0; u < PULL_U; u++) {
                hv[u] = make_int4(-1, -1, -1, -1);
                if (live[u]) hv[u] = reinterpret_cast<const int4 *>(ph)[((w0 + u) << 6) + lane];
            }
            if (dbg & 128) {  // diagnostics: the round-4 short-circuit probes (A/B)
#pragma unroll
                for (int u = 0; u < PULL_U; u++)
                    found[u] = (hv[u].x >= 0 && gb_bit(ubits, hv[u].x)) ||
                               (hv[u].y >= 0 && gb_bit(ubits, hv[u].y)) ||
                               (hv[u].z >= 0 && gb_bit(ubits, hv[u].z)) ||
                               (hv[u].w >= 0 && gb_bit(ubits, hv[u].w));
            } else {
                // the probes in two rounds, each with every load in flight at once: the first
                // head of every open row, then the other three for the rows it missed (a
                // short-circuit test makes each probe wait for the one before it: up to 16
                // dependent frontier reads per wave step)
                const uint32_t *ub32 = reinterpret_cast<const uint32_t *>(ubits);
                uint32_t w1[PULL_U];
#pragma unroll
                for (int u = 0; u < PULL_U; u++) {
                    w1[u] = 0;
                    if (hv[u].x >= 0) w1[u] = ub32[hv[u].x >> 5];
                }
#pragma unroll
                for (int u = 0; u < PULL_U; u++) found[u] = hv[u].x >= 0 && ((w1[u] >> (hv[u].x & 31)) & 1u);
                uint32_t wy[PULL_U], wz[PULL_U], ww[PULL_U];
#pragma unroll
                for (int u = 0; u < PULL_U; u++) {
                    wy[u] = wz[u] = ww[u] = 0;
                    if (!found[u]) {
                        if (hv[u].y >= 0) wy[u] = ub32[hv[u].y >> 5];
                        if (hv[u].z >= 0) wz[u] = ub32[hv[u].z >> 5];
                        if (hv[u].w >= 0) ww[u] = ub32[hv[u].w >> 5];
                    }
                }
#pragma unroll
                for (int u = 0; u < PULL_U; u++)
                    found[u] = found[u] || (hv[u].y >= 0 && ((wy[u] >> (hv[u].y & 31)) & 1u)) ||
                               (hv[u].z >= 0 && ((wz[u] >> (hv[u].z & 31)) & 1u)) ||
                               (hv[u].w >= 0 && ((ww[u] >> (hv[u].w & 31)) & 1u));
            }
#pragma unroll
            for (int u = 0; u < PULL_U; u++) {
                const int64_t r = ((w0 + u) << 6) + lane;
                p[u] = p1[u] = 0;
                if (live[u] && !found[u] && hv[u].w == -2 && r < nrows) {  // a long row: walk it
                    p[u] = rowptr[r];
                    p1[u] = rowptr[r + 1];
                }
                dg[u] = (hprow && found[u]) ? (int64_t)pdeg[r] : p1[u] - p[u];
            }
        } else {
            // row bounds are loaded for every row, independently of the mask word
#pragma unroll
            for (int u = 0; u < PULL_U; u++) {
                const int64_t r = ((w0 + u) << 6) + lane;
                p[u] = p1[u] = 0;
                if (r < nrows) {
                    p[u] = rowptr[r];
                    p1[u] = rowptr[r + 1];
                }
                dg[u] = p1[u] - p[u];
            }
        }
        for (int it = 0; it < p1_steps; it++) {
            bool go[PULL_U], any = false;
#pragma unroll
            for (int u = 0; u < PULL_U; u++) {
                go[u] = live[u] && !found[u] && p[u] < p1[u];
                any = any || go[u];
            }
            if (!__ballot(any)) break;
            int k[PULL_U][4];
#pragma unroll
            for (int u = 0; u < PULL_U; u++) {
#pragma unroll
                for (int t = 0; t < 4; t++) k[u][t] = -1;
                if (go[u]) {
#pragma unroll
                    for (int t = 0; t < 4; t++)
                        if (p[u] + t < p1[u]) k[u][t] = colidx[p[u] + t];
                }
            }
#pragma unroll
            for (int u = 0; u < PULL_U; u++) {
                if (go[u]) {
                    int f = 0;
                    if (dbg & 32) {  // diagnostics: no frontier probes in the steps
#pragma unroll
                        for (int t = 0; t < 4; t++) f += k[u][t] == 0x7fffffff;
                    } else {
#pragma unroll
                        for (int t = 0; t < 4; t++) f += k[u][t] >= 0 && gb_bit(ubits, k[u][t]);
                    }
                    found[u] = f != 0;
                    p[u] += 4;
                }
            }
        }
        // rows still open -> segment list
        int n = 0;
#pragma unroll
        for (int u = 0; u < PULL_U; u++) {
            const bool pd = live[u] && !found[u] && p[u] < p1[u];
            const unsigned long long bb = __ballot(pd);
            if (pd) {
                const int i = n + __popcll(bb & lt);
                L.p[i] = p[u];
                L.rem[i] = (int32_t)(p1[u] - p[u]);
                L.id[i] = (int16_t)(u * 64 + lane);
            }
            n += __popcll(bb);
        }
        if (lane < PULL_U) L.hitw[lane] = 0;
        if (dbg & 16) n = 0;  // diagnostics: rows left after the steps are dropped
        int cap = cap0;
        while (n) {
            gb_wave_sync();
            const int total = gb_wlist_round(L, n, cap, lane);
            for (int e0 = 0; e0 < total; e0 += 256) {
                int k[4], s[4];
                bool ok[4];
#pragma unroll
                for (int u = 0; u < 4; u++) {
                    const int e = e0 + lane + 64 * u;
                    ok[u] = e < total;
                    s[u] = 0;
                    k[u] = 0;
                    if (ok[u]) {
                        s[u] = gb_wlist_find(L, n, e);
                        k[u] = colidx[L.p[s[u]] + (e - gb_wlist_start(L, s[u]))];
                    }
                }
#pragma unroll
                for (int u = 0; u < 4; u++)
                    if (ok[u] && gb_bit(ubits, k[u])) L.hit[s[u]] = 1;
            }
            gb_wave_sync();
            // survivors of the round, compacted in place (chunks of 64, in order)
            int m = 0;
            for (int c0 = 0; c0 < n; c0 += 64) {
                const int i = c0 + lane;
                bool alive = false, hit = false;
                int64_t np = 0;
                int32_t nr = 0;
                int16_t id = 0;
                if (i < n) {
                    const int32_t taken = L.pref[i] - gb_wlist_start(L, i);
                    hit = L.hit[i] != 0;
                    id = L.id[i];
                    np = L.p[i] + taken;
                    nr = L.rem[i] - taken;
                    alive = !hit && nr > 0;
                }
                if (hit) atomicOr(&L.hitw[id >> 6], 1ULL << (id & 63));
                const unsigned long long ab = __ballot(alive);
                gb_wave_sync();
                if (alive) {
                    const int j = m + __popcll(ab & lt);
                    L.p[j] = np;
                    L.rem[j] = nr;
                    L.id[j] = id;
                }
                m += __popcll(ab);
                gb_wave_sync();
            }
            n = m;
            cap = cap < (1 << 20) ? cap * 2 : cap;
        }
        gb_wave_sync();
#pragma unroll
        for (int u = 0; u < PULL_U; u++) {
            if ((L.hitw[u] >> lane) & 1ULL) found[u] = true;
            const unsigned long long word = __ballot(found[u]);
            if (lane == 0 && w0 + u < nwords) {
                tbits[w0 + u] = word;
                cnt += __popcll(word);
            }
        }
        if (hprow) {
            // edges of the next frontier, estimated by the rows' pull-orientation
            // length (already loaded; exact for symmetric matrices): a hint for the
            // next call's push/pull choice only
#pragma unroll
            for (int u = 0; u < PULL_U; u++)
                if (found[u]) mfn += dg[u];
        }
    }
    return cnt;
}

// z = mult(a0, u0) for an iso result, types known only at run time (z is x's
// type or bool: the builtin semirings' z types)
template <class X>
__device__ void gb_iso_eval_x(int mul, bool zbool, bool flip, const void *a0, const void *u0, void *out) {
    const X a = a0 ? *(const X *)a0 : X(), b = u0 ? *(const X *)u0 : X();
    const X x = flip ? b : a, y = flip ? a : b;
    if (zbool) *(bool *)out = gb_binop_z<X, bool>(mul, x, y, 0, 0, 0);
    else *(X *)out = gb_binop_z<X, X>(mul, x, y, 0, 0, 0);
}
__device__ void gb_iso_eval(int mul, int xcode, int zcode, bool flip, const void *a0, const void *u0, void *out) {
    const bool zb = zcode == GBAMD_T_BOOL && xcode != GBAMD_T_BOOL;
    switch (xcode) {
    case GBAMD_T_BOOL: gb_iso_eval_x<bool>(mul, zb, flip, a0, u0, out); break;
    case GBAMD_T_INT8: gb_iso_eval_x<int8_t>(mul, zb, flip, a0, u0, out); break;
    case GBAMD_T_UINT8: gb_iso_eval_x<uint8_t>(mul, zb, flip, a0, u0, out); break;
    case GBAMD_T_INT16: gb_iso_eval_x<int16_t>(mul, zb, flip, a0, u0, out); break;
    case GBAMD_T_UINT16: gb_iso_eval_x<uint16_t>(mul, zb, flip, a0, u0, out); break;
    case GBAMD_T_INT32: gb_iso_eval_x<int32_t>(mul, zb, flip, a0, u0, out); break;
    case GBAMD_T_UINT32: gb_iso_eval_x<uint32_t>(mul, zb, flip, a0, u0, out); break;
    case GBAMD_T_INT64: gb_iso_eval_x<int64_t>(mul, zb, flip, a0, u0, out); break;
    case GBAMD_T_UINT64: gb_iso_eval_x<uint64_t>(mul, zb, flip, a0, u0, out); break;
    case GBAMD_T_FP32: gb_iso_eval_x<float>(mul, zb, flip, a0, u0, out); break;
    case GBAMD_T_FP64: gb_iso_eval_x<double>(mul, zb, flip, a0, u0, out); break;
    default: break;
    }
}

#define GB_ZP_MAX 4  // pooled cleared-vector storages zeroed per iso SpMV launch

struct gb_iso_args {
    // direction: from the frontier's edge-count hint (the vector's producer
    // computed it), else from k_dir_prep's decision, else pull
    const long long *mf_hint;
    gb_dir_rule rule;
    const unsigned long long *dst;
    // next-frontier hint: edges of the output's entries in rows of hprow
    const int64_t *hprow;
    long long *mf_out;
    // iso value of the result (nullptr: written elsewhere)
    int mul, xcode, zcode;
    bool flip;
    const void *a0, *u0;
    void *iso_out;
    // host mailbox for the count; pub_form (knob iso_pub): 0 one tagged word (GB_PUB_TAG) stored
    // relaxed, 1 value + system fence + release seq (round 4), 2 the tagged word stored release
    gb_host_slot *pub;
    long long pub_seq;
    int pub_form;
    // u's exact device count (gb_asg::u_count_exact; nullptr: not known): 0 ends the launch early
    const int64_t *u_exit;
    bool out_zeroed;  // T's bitmap came zeroed (the spare)
    // a bitmap to zero for the next call's push output
    uint64_t *spare;
    int64_t spare_words;
    // pull shape: lane-per-row steps of 4 edges, then the first per-row cap of the list rounds
    int p1_steps, cap0;
    int dbg;                        // diagnostics (knob iso_dbg): 1 no mailbox, 2 no hint sum, 4 no work, 8 empty,
                                    // 16 pull without its segment list, 32 pull steps without probes (wrong results),
                                    // 64 no finish, 128 the round-4 dependent read order (exact; A/B),
                                    // 512 push without the frontier-word prefetch (exact; A/B)
    bool packed;                    // one-round finish (iso_finish_packed): n < 2^27
    const uint64_t *rows_nonempty;  // pull rows with entries (nullptr: all)
    const int32_t *phead;           // pull head per row, 4 int32 (nullptr: none; gb_view_pullfirst)
    const uint32_t *pdeg;           // push-orientation length per pull row (the hint of found rows)
    int host_dir;                   // 1: push, decided on the host (small frontier of known size)
    // storage of cleared vectors zeroed by this launch (gb_zpool_*): bitmaps of zb_words words,
    // counts of 2 + GB_HINT_PARTS words
    uint64_t *zb[GB_ZP_MAX];
    int64_t *zc[GB_ZP_MAX];
    int nzb, nzc;
    int64_t zb_words;
    // fused deferred assign (gb_asg): w<q>(:) = x with q = u (asg.bits nullptr: none)
    gb_asg_dev asg;
    const void *asg_qiso;
    int asg_qiso_code;
    unsigned long long *asg_count;
    int64_t root;  // >= 0: the frontier is this one pending vertex (gb_push_root); u's bits do not hold it
    // diagnostics (environment GRAPHBLAS_AMD_ISO_TS): wall-clock stamps (s_memrealtime, 100 MHz) of
    // each launch's start (block 0) and end (the finishing block), ts[0] / ts[1] launch counters,
    // pairs from ts[2] -- kernel gaps without a profiler (tools/iso_gaps.py)
    unsigned long long *ts;
};

// ------------------------------------------------ general SpMV: balanced words
// One wave per 64-row output word (a bitmap word): the entries of the word's
// rows (rows of at most LONG entries) are concatenated and walked 256 at a
// time, four independent gathers per lane; products of one row sit in
// consecutive lanes, so a segmented scan across the wave folds them and the
// last lane of each segment adds the run to the row's accumulator in LDS (row
// order = ascending k: deterministic).  Rows longer than LONG are cut into
// CH-entry chunks (a table cached on the matrix) whose partial folds are
// combined in chunk order by k_spmv_fold.
#define SPMV_LONG 128
#define SPMV_CH 1024
#define SPMV_WU 8  // entries per lane per step of the words kernel (gathers in flight)

template <class SR, class X, class Z, bool FLIP>
__device__ __forceinline__ void gb_spmv_product(SR &sr, bool rv, const X *__restrict__ avals, bool a_iso, X a0,
                                                const X *__restrict__ uvals, bool u_iso, X u0, int64_t p, int k,
                                                int64_t r, Z &z, const X *__restrict__ uhot, bool nt = false) {
    X a = X(), b = X();
    if (rv) {
        // nt: the streamed A values bypass L2 retention (the hot x values stay resident)
        a = a_iso ? a0 : (nt ? __builtin_nontemporal_load(&avals[p]) : avals[p]);
        // k < 0: a hot column (relabelled colidx, gb_view_hot): its value from the packed copy
        b = u_iso ? u0 : (k < 0 ? uhot[k & 0x7fffffff] : uvals[k]);
    }
    z = FLIP ? sr.mult(b, a, 0, k, r) : sr.mult(a, b, r, k, 0);
}

// Merge-path word (general SpMV, mode 1): the word's concatenated entries are
// cut into 64 equal contiguous runs, one per lane; a lane folds its run
// sequentially (row changes read from LDS, four entries' loads issued ahead),
// rows wholly inside one run are finished by that lane, and rows crossing runs
// are folded by their owner lane from the runs' carries in lane order.
template <class Z>
struct gb_mp_lds {
    int incl[64];
    int64_t p0[64];
    Z pa[64], pb[64];  // carry of the row continuing from the previous run / into the next
    int fa[64], fb[64];
};

template <class SR, class X, class Z, bool FLIP>
__device__ __forceinline__ long long gb_spmv_words_mp(
    SR &sr, int64_t nrows, const int64_t *__restrict__ rowptr, const int32_t *__restrict__ colidx,
    const X *__restrict__ avals, bool a_iso, X a0, const uint64_t *__restrict__ ubits, const X *__restrict__ uvals,
    bool u_iso, X u0, const uint64_t *__restrict__ mbits, bool mcomp, bool ufull, bool rv,
    uint64_t *__restrict__ tbits, Z *__restrict__ tvals, Z *acc, int *fl, gb_mp_lds<Z> &M,
    const X *__restrict__ uhot) {
    const int lane = threadIdx.x & 63;
    const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
    const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
    const int64_t nwords = (nrows + 63) >> 6;
    long long cnt = 0;
    for (int64_t w = wave; w < nwords; w += nwaves) {
        const int64_t r = (w << 6) + lane;
        bool open = r < nrows;
        if (open && mbits) open = gb_bit(mbits, r) != mcomp;
        int64_t p0 = 0;
        int len = 0;
        if (open) {
            p0 = rowptr[r];
            const int64_t d = rowptr[r + 1] - p0;
            len = d > SPMV_LONG ? 0 : (int)d;  // long rows: chunks + k_spmv_fold
        }
        int incl = len;
        for (int off = 1; off < 64; off <<= 1) {
            const int y = __shfl_up(incl, off, 64);
            if (lane >= off) incl += y;
        }
        const int total = __shfl(incl, 63, 64);
        M.incl[lane] = incl;
        M.p0[lane] = p0;
        M.fa[lane] = 0;
        M.fb[lane] = 0;
        gb_wave_sync();
        if (total > 0) {
            const int c = (total + 63) >> 6;
            const int s0 = lane * c;
            const int e1 = s0 + c < total ? s0 + c : total;
            if (s0 < e1) {
                int row = 0;  // first row with incl > s0
#pragma unroll
                for (int st = 32; st > 0; st >>= 1)
                    if (M.incl[row + st - 1] <= s0) row += st;
                int rbeg = row ? M.incl[row - 1] : 0, rend = M.incl[row];
                bool before = rbeg < s0;
                int64_t pbase = M.p0[row] - rbeg;
                bool f = false;
                Z z = Z();
                for (int e = s0; e < e1; e += 4) {
                    int rw[4];
                    int64_t pos[4];
                    bool ok[4];
                    // positions of the next four entries (row changes from LDS)
                    int trow = row, tbeg = rbeg, tend = rend;
                    int64_t tbase = pbase;
#pragma unroll
                    for (int t = 0; t < 4; t++) {
                        const int et = e + t;
                        ok[t] = et < e1;
                        if (ok[t]) {
                            while (et >= tend) {
                                trow++;
                                tbeg = tend;
                                tend = M.incl[trow];
                                tbase = M.p0[trow] - tbeg;
                            }
                        }
                        rw[t] = trow;
                        pos[t] = tbase + et;
                    }
                    int k[4];
#pragma unroll
                    for (int t = 0; t < 4; t++) k[t] = ok[t] ? colidx[pos[t]] : 0;
                    bool hit[4];
                    Z zt[4];
#pragma unroll
                    for (int t = 0; t < 4; t++) {
                        hit[t] = ok[t] && (ufull || gb_bit(ubits, k[t]));
                        zt[t] = Z();
                        if (hit[t])
                            gb_spmv_product<SR, X, Z, FLIP>(sr, rv, avals, a_iso, a0, uvals, u_iso, u0, pos[t], k[t],
                                                            (w << 6) + rw[t], zt[t], uhot);
                    }
#pragma unroll
                    for (int t = 0; t < 4; t++) {
                        if (!ok[t]) break;
                        if (rw[t] != row) {  // the current row closed inside this run
                            if (before) {
                                M.pa[lane] = z;
                                M.fa[lane] = f;
                            } else if (f) {
                                acc[row] = z;
                                fl[row] = 1;
                            }
                            row = rw[t];
                            before = false;
                            f = false;
                        }
                        if (hit[t]) {
                            z = f ? sr.add(z, zt[t]) : zt[t];
                            f = true;
                        }
                    }
                    row = trow;
                    rbeg = tbeg;
                    rend = tend;
                    pbase = tbase;
                }
                // the row open at the end of the run
                const bool cont = rend > e1;
                if (before) {
                    M.pa[lane] = z;
                    M.fa[lane] = f;
                } else if (cont) {
                    M.pb[lane] = z;
                    M.fb[lane] = f;
                } else if (f) {
                    acc[row] = z;
                    fl[row] = 1;
                }
            }
            gb_wave_sync();
            // rows crossing runs: the owner lane folds the carries in lane order
            if (len > 0) {
                const int ex = incl - len;
                const int k0 = ex / c, k1 = (incl - 1) / c;
                if (k1 > k0) {
                    bool f = M.fb[k0] != 0;
                    Z z = M.pb[k0];
                    for (int k = k0 + 1; k <= k1; k++) {
                        if (!M.fa[k]) continue;
                        z = f ? sr.add(z, M.pa[k]) : M.pa[k];
                        f = true;
                    }
                    if (f) {
                        acc[lane] = z;
                        fl[lane] = 1;
                    }
                }
            }
            gb_wave_sync();
        }
        const bool hitrow = fl[lane] != 0;
        const unsigned long long fmask = __ballot(hitrow);
        if (hitrow) tvals[r] = acc[lane];
        if (lane == 0) {
            tbits[w] = fmask;
            cnt += __popcll(fmask);
        }
        fl[lane] = 0;
        gb_wave_sync();
    }
    return cnt;
}

template <class SR, class X, class Z, bool FLIP>
__global__ __launch_bounds__(SPMV_BLOCK) void k_spmv_words(
    SR sr, int64_t nrows, const int64_t *__restrict__ rowptr, const int32_t *__restrict__ colidx,
    const X *__restrict__ avals, bool a_iso, const uint64_t *__restrict__ ubits,
    const X *__restrict__ uvals, bool u_iso, const uint64_t *__restrict__ mbits, bool mcomp,
    const int32_t *__restrict__ chunks, int64_t nchunks, Z *__restrict__ cpart, int8_t *__restrict__ cfound,
    uint64_t *__restrict__ tbits, Z *__restrict__ tvals, unsigned long long *__restrict__ tcount,
    unsigned long long *__restrict__ gst, const int64_t *__restrict__ ucount, int64_t un, int mode,
    const X *__restrict__ uhot) {
    __shared__ Z accs[WAVES_PER_BLOCK][64];
    __shared__ int fls[WAVES_PER_BLOCK][64];
    __shared__ gb_mp_lds<Z> mps[WAVES_PER_BLOCK];
    Z *acc = accs[threadIdx.x >> 6];
    int *fl = fls[threadIdx.x >> 6];  // row has at least one product
    const int lane = threadIdx.x & 63;
    const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
    const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
    const int64_t nwords = (nrows + 63) >> 6;
    const bool rv = SR::reads_values && avals && uvals;
    X a0 = X(), u0 = X();
    if (rv) {
        if (a_iso) a0 = avals[0];
        if (u_iso) u0 = uvals[0];
    }
    // u has every entry: no presence tests (a relabelled colidx, uhot, is used only then)
    const bool ufull = uhot || (ucount && *ucount == un);
    const bool nt = (mode & 2) != 0;  // non-temporal loads of the streamed colidx / values
    mode &= 1;
    fl[lane] = 0;
    gb_wave_sync();
    long long cnt = 0;
    // long-row chunks: lane-sequential folds in ascending k, then a wave fold in lane order
    for (int64_t c = wave; c < nchunks; c += nwaves) {
        const int64_t r = chunks[2 * c], piece = chunks[2 * c + 1];
        bool f = false;
        Z z = Z();
        if (!mbits || gb_bit(mbits, r) != mcomp) {
            const int64_t pe = rowptr[r + 1];
            const int64_t p0 = rowptr[r] + piece * SPMV_CH;
            const int64_t p1 = p0 + SPMV_CH < pe ? p0 + SPMV_CH : pe;
            for (int64_t q = p0 + lane; q < p1; q += 256) {
                int kk[4];
                bool ok[4];
#pragma unroll
                for (int u = 0; u < 4; u++) {
                    ok[u] = q + 64 * u < p1;
                    kk[u] = ok[u] ? (nt ? __builtin_nontemporal_load(&colidx[q + 64 * u]) : colidx[q + 64 * u]) : 0;
                }
#pragma unroll
                for (int u = 0; u < 4; u++) {
                    if (!ok[u] || (!ufull && !gb_bit(ubits, kk[u]))) continue;
                    Z t;
                    gb_spmv_product<SR, X, Z, FLIP>(sr, rv, avals, a_iso, a0, uvals, u_iso, u0, q + 64 * u, kk[u],
                                                    r, t, uhot, nt);
                    z = f ? sr.add(z, t) : t;
                    f = true;
                }
            }
        }
        for (int off = 1; off < 64; off <<= 1) {  // fold lanes in order: lane l absorbs l+off
            const bool of = __shfl_down((int)f, off, 64);
            const Z oz = gb_shfl_down(z, off, 64);
            if (lane + off < 64 && (lane & (2 * off - 1)) == 0 && of) {
                z = f ? sr.add(z, oz) : oz;
                f = true;
            }
        }
        if (lane == 0) {
            cfound[c] = f ? 1 : 0;
            if (f) cpart[c] = z;
        }
    }
    // output words
    if (mode == 1) {
        cnt += gb_spmv_words_mp<SR, X, Z, FLIP>(sr, nrows, rowptr, colidx, avals, a_iso, a0, ubits, uvals, u_iso, u0,
                                                mbits, mcomp, ufull, rv, tbits, tvals, acc, fl, mps[threadIdx.x >> 6],
                                                uhot);
        long long tot;
        if (gb_grid_sum(cnt, gst, &tot)) *tcount = (unsigned long long)tot;
        return;
    }
    for (int64_t w = wave; w < nwords; w += nwaves) {
        const int64_t r = (w << 6) + lane;
        bool open = r < nrows;
        if (open && mbits) open = gb_bit(mbits, r) != mcomp;
        int64_t p0 = 0;
        int len = 0;
        if (open) {
            p0 = rowptr[r];
            const int64_t d = rowptr[r + 1] - p0;
            len = d > SPMV_LONG ? 0 : (int)d;  // long rows: chunks + k_spmv_fold
        }
        int incl = len;
        for (int off = 1; off < 64; off <<= 1) {
            const int y = __shfl_up(incl, off, 64);
            if (lane >= off) incl += y;
        }
        const int excl = incl - len;
        const int total = __shfl(incl, 63, 64);
        for (int e0 = 0; e0 < total; e0 += 64 * SPMV_WU) {
            // all SPMV_WU gathers of the step are issued before the first fold waits on one
            int k[SPMV_WU], own[SPMV_WU];
            int64_t pos[SPMV_WU];
            bool ok[SPMV_WU];
#pragma unroll
            for (int u = 0; u < SPMV_WU; u++) {
                const int e = e0 + lane + 64 * u;
                int lo = 0;
#pragma unroll
                for (int st = 32; st > 0; st >>= 1)
                    if (__shfl(incl, lo + st - 1, 64) <= e) lo += st;
                own[u] = lo;
                pos[u] = __shfl(p0, lo, 64) + (e - __shfl(excl, lo, 64));
                ok[u] = e < total;
                k[u] = ok[u] ? (nt ? __builtin_nontemporal_load(&colidx[pos[u]]) : colidx[pos[u]]) : 0;
            }
            bool fu[SPMV_WU];
            Z zu[SPMV_WU];
#pragma unroll
            for (int u = 0; u < SPMV_WU; u++) {
                fu[u] = ok[u] && (ufull || gb_bit(ubits, k[u]));
                zu[u] = Z();
                if (fu[u])
                    gb_spmv_product<SR, X, Z, FLIP>(sr, rv, avals, a_iso, a0, uvals, u_iso, u0, pos[u], k[u],
                                                    (w << 6) + own[u], zu[u], uhot, nt);
            }
#pragma unroll
            for (int u = 0; u < SPMV_WU; u++) {
                bool f = fu[u];
                Z z = zu[u];
                // segmented inclusive scan over lanes of the same row; the segments and the
                // products' presence travel as two ballots, so each step shuffles only z:
                // before step off, lane l holds [max(seg, l-off+1), l]
                const int row = ok[u] ? own[u] : 64 + lane;  // idle lanes: own segment
                const int prow = __shfl_up(row, 1, 64);  // all lanes shuffle (not under ||)
                const unsigned long long heads = __ballot(lane == 0 || prow != row);
                const unsigned long long fmask = __ballot(f);
                const int seg = 63 - __clzll(heads & ((2ULL << lane) - 1ULL));  // this row's first lane
                for (int off = 1; off < 64; off <<= 1) {
                    const Z oz = gb_shfl_up(z, off, 64);
                    const int hi = lane - off;
                    if (hi >= seg) {
                        const int lo = hi - off + 1 > seg ? hi - off + 1 : seg;
                        if ((fmask >> lo) & ((2ULL << (hi - lo)) - 1ULL)) {  // lane hi's range holds a product
                            z = f ? sr.add(oz, z) : oz;
                            f = true;
                        }
                    }
                }
                const bool last = ok[u] && (lane == 63 || ((heads >> (lane + 1)) & 1ULL));
                // a row's runs arrive in order (earlier batches first): fold into its accumulator
                if (last && f) {
                    acc[row] = fl[row] ? sr.add(acc[row], z) : z;
                    fl[row] = 1;
                }
                gb_wave_sync();
            }
        }
        const bool hit = fl[lane] != 0;
        const unsigned long long fmask = __ballot(hit);
        if (hit) tvals[r] = acc[lane];
        if (lane == 0) {
            tbits[w] = fmask;
            cnt += __popcll(fmask);
        }
        fl[lane] = 0;
        gb_wave_sync();
    }
    long long tot;
    if (gb_grid_sum(cnt, gst, &tot)) *tcount = (unsigned long long)tot;  // k_spmv_fold adds the long rows
}

// the hot columns' values of a dense u, packed in rank order (gb_view_hot)
template <class X>
__global__ void k_hot_gather(const X *__restrict__ uvals, const int32_t *__restrict__ hcols, int64_t nh,
                             X *__restrict__ uhot) {
    for (int64_t h = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; h < nh; h += (int64_t)gridDim.x * blockDim.x)
        uhot[h] = uvals[hcols[h]];
}

// long rows: fold their chunks' partials in chunk order (one thread per row)
template <class SR, class Z>
__global__ void k_spmv_fold(SR sr, const int32_t *__restrict__ chunks, int64_t nchunks, const Z *__restrict__ cpart,
                            const int8_t *__restrict__ cfound, uint64_t *__restrict__ tbits, Z *__restrict__ tvals,
                            unsigned long long *__restrict__ tcount, unsigned long long *__restrict__ gst) {
    long long cnt = 0;
    for (int64_t c = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; c < nchunks;
         c += (int64_t)gridDim.x * blockDim.x) {
        if (chunks[2 * c + 1] != 0) continue;
        const int64_t r = chunks[2 * c];
        bool f = false;
        Z z = Z();
        for (int64_t h = c; h < nchunks && chunks[2 * h] == r; h++) {
            if (!cfound[h]) continue;
            z = f ? sr.add(z, cpart[h]) : cpart[h];
            f = true;
        }
        if (f) {
            tvals[r] = z;
            atomicOr((unsigned long long *)&tbits[r >> 6], 1ULL << (r & 63));
            cnt++;
        }
    }
    gb_grid_add(cnt, tcount, gst);
}

// The result's finish in one round of atomics (n < 2^27): the block sums of the
// count and of the fused assign's count delta travel packed in one 64-bit word
// (arrival 10 bits | count 27 | delta 27) through the sharded grid sum, and the
// next-frontier hint needs no root at all -- each shard's last block stores the
// shard's total in the output's hint parts, which the hint's reader adds up.  All
// of a block's atomics are issued together (one round trip instead of the six of
// three separate grid sums: ~5 us per BFS level).
#define ISO_ARR_BITS 10
#define ISO_VAL_BITS 27

// hand the count to the host without a copy (gb_host_slot_wait)
#define ISO_TS_PAIRS (1 << 20)
__device__ __forceinline__ void iso_ts_mark(const gb_iso_args &a, int which) {
    if (!a.ts) return;
    const unsigned long long t = __builtin_amdgcn_s_memrealtime();
    const unsigned long long k = atomicAdd(&a.ts[which], 1ULL);
    if (k < ISO_TS_PAIRS) a.ts[2 + 2 * k + which] = t;
}

__device__ __forceinline__ void iso_publish(const gb_iso_args &a, long long tot) {
    iso_ts_mark(a, 1);
    if (!a.pub || (a.dbg & 1)) return;
    if (a.pub_form == 1) {
        __hip_atomic_store(&a.pub->value, tot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __threadfence_system();
        __hip_atomic_store(&a.pub->seq, a.pub_seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        return;
    }
    const long long w = (long long)(GB_PUB_TAG | (((unsigned long long)a.pub_seq & 0x7fffffffULL) << 32) |
                                    ((unsigned long long)tot & 0xffffffffULL));
    if (a.pub_form == 0) __hip_atomic_store(&a.pub->seq, w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    else __hip_atomic_store(&a.pub->seq, w, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void iso_finish_packed(long long cnt, long long mfn, long long adelta,
                                                  unsigned long long *__restrict__ tcount,
                                                  unsigned long long *__restrict__ gst, const gb_iso_args &a) {
    __shared__ long long part[3][SPMV_BLOCK / 64];
    for (int off = 32; off > 0; off >>= 1) {
        cnt += __shfl_xor(cnt, off, 64);
        mfn += __shfl_xor(mfn, off, 64);
        adelta += __shfl_xor(adelta, off, 64);
    }
    const int wid = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        part[0][wid] = cnt;
        part[1][wid] = mfn;
        part[2][wid] = adelta;
    }
    __syncthreads();
    if (threadIdx.x != 0) return;
    cnt = mfn = adelta = 0;
    for (int w = 0; w < SPMV_BLOCK / 64; w++) {
        cnt += part[0][w];
        mfn += part[1][w];
        adelta += part[2][w];
    }
    const unsigned nb = gridDim.x;
    const unsigned s = blockIdx.x % GB_GRID_SHARDS;
    const unsigned in_shard = (nb - s + GB_GRID_SHARDS - 1) / GB_GRID_SHARDS;
    const unsigned long long AM = (1ULL << ISO_ARR_BITS) - 1, VM = (1ULL << ISO_VAL_BITS) - 1;
    unsigned long long *cs = gst + (size_t)s * GB_GRID_STRIDE;
    unsigned long long *hs = gst + GB_GRID2_OFFSET + (size_t)s * GB_GRID_STRIDE;
    const unsigned long long pk =
        ((unsigned long long)adelta << (ISO_ARR_BITS + ISO_VAL_BITS)) | ((unsigned long long)cnt << ISO_ARR_BITS) | 1ULL;
    unsigned long long oh = 0;
    if (a.mf_out) {
        oh = atomicAdd(hs, ((unsigned long long)mfn << 12) + 1ULL);
        if (blockIdx.x == 0)  // the parts of shards no block maps to
            for (unsigned i = nb; i < GB_HINT_PARTS; i++) a.mf_out[i] = 0;
    }
    const unsigned long long oc = atomicAdd(cs, pk);
    if (a.mf_out && (unsigned)(oh & 0xFFF) + 1 == in_shard) {
        a.mf_out[s] = (long long)(oh >> 12) + mfn;  // this shard's part of the hint
        atomicExch(hs, 0ULL);
    }
    if ((unsigned)(oc & AM) + 1 != in_shard) return;
    atomicExch(cs, 0ULL);
    const unsigned long long scnt = ((oc >> ISO_ARR_BITS) & VM) + (unsigned long long)cnt;
    const unsigned long long sadd = (oc >> (ISO_ARR_BITS + ISO_VAL_BITS)) + (unsigned long long)adelta;
    const unsigned nshards = nb < GB_GRID_SHARDS ? nb : GB_GRID_SHARDS;
    unsigned long long *root = gst + (size_t)GB_GRID_SHARDS * GB_GRID_STRIDE;
    const unsigned long long o2 =
        atomicAdd(root, (sadd << (ISO_ARR_BITS + ISO_VAL_BITS)) | (scnt << ISO_ARR_BITS) | 1ULL);
    if ((unsigned)(o2 & AM) + 1 != nshards) return;
    const long long tot = (long long)(((o2 >> ISO_ARR_BITS) & VM) + scnt);
    const long long add = (long long)((o2 >> (ISO_ARR_BITS + ISO_VAL_BITS)) + sadd);
    *tcount = (unsigned long long)tot;
    iso_publish(a, tot);
    // after the publish (off the host's critical path; the next launch on the stream starts
    // only after this kernel has ended): the root reset and the fused assign's count
    atomicExch(root, 0ULL);
    if (a.asg.bits && add) atomicAdd(a.asg_count, (unsigned long long)add);
}

// One launch does the chosen direction and finishes the result: count
// (stored, no prior zeroing needed), next-frontier hint, iso value, mailbox.
__global__ __launch_bounds__(SPMV_BLOCK) void k_iso_work(
    int64_t nrows, const int64_t *__restrict__ rowptr, const int32_t *__restrict__ colidx,
    int64_t nwords_u, const uint64_t *__restrict__ ubits, const int64_t *__restrict__ prow,
    const int32_t *__restrict__ pcol, const int32_t *__restrict__ hubs, int64_t nhubs, int64_t H,
    const uint64_t *__restrict__ mbits, bool mcomp, uint64_t *__restrict__ tbits,
    unsigned long long *__restrict__ tcount, unsigned long long *__restrict__ gst, gb_iso_args a) {
    __shared__ gb_wlist lists[WAVES_PER_BLOCK];
    gb_wlist &L = lists[threadIdx.x >> 6];
    if (a.ts && blockIdx.x == 0 && threadIdx.x == 0) iso_ts_mark(a, 0);
    if (a.dbg & 8) return;  // diagnostics: the launch alone
    bool push = false;
    if (a.host_dir == 1) {
        push = true;
    } else if (a.mf_hint) {
        long long mf = 0;  // the hint's parts (one per grid-sum shard of its producer)
        for (int i = 0; i < GB_HINT_PARTS; i++) mf += a.mf_hint[i];
        push = gb_dir_decide(mf, a.rule);
    }
    else if (a.dst) push = a.dst[ST_PUSH] != 0;
    if (a.spare && !(a.dbg & 32)) {  // dbg 32: diagnostics, no zeroing
        for (int64_t w = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; w < a.spare_words;
             w += (int64_t)gridDim.x * blockDim.x)
            a.spare[w] = 0;
    }
    for (int j = 0; j < ((a.dbg & 32) ? 0 : a.nzb); j++)  // cleared vectors' bitmaps, back to the pool zeroed
        for (int64_t w = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; w < a.zb_words;
             w += (int64_t)gridDim.x * blockDim.x)
            a.zb[j][w] = 0;
    if (blockIdx.x == 0)
        for (int j = 0; j < a.nzc; j++)
            for (int w = threadIdx.x; w < 2 + GB_HINT_PARTS; w += blockDim.x) a.zc[j][w] = 0;
    // the result's iso value does not depend on the work: evaluated here, off the finish's path
    if (a.packed && a.iso_out && blockIdx.x == 0 && threadIdx.x == 0)
        gb_iso_eval(a.mul, a.xcode, a.zcode, a.flip, a.a0, a.u0, a.iso_out);
    if (a.u_exit && *a.u_exit == 0) {
        // an empty u (the speculated level after a BFS's last): no products, an empty stamp, so
        // no grid-wide finish -- block 0 stores the zero count and hint and publishes
        if (!a.out_zeroed)
            for (int64_t w = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; w < ((nrows + 63) >> 6);
                 w += (int64_t)gridDim.x * blockDim.x)
                tbits[w] = 0;
        if (blockIdx.x == 0) {
            if (a.mf_out)
                for (int i = threadIdx.x; i < GB_HINT_PARTS; i += blockDim.x) a.mf_out[i] = 0;
            if (threadIdx.x == 0) {
                *tcount = 0ULL;
                if (!a.packed && a.iso_out) gb_iso_eval(a.mul, a.xcode, a.zcode, a.flip, a.a0, a.u0, a.iso_out);
                iso_publish(a, 0);
            }
        }
        return;
    }
    // fused assign: q's value mask is empty when q is iso with a false value
    const uint64_t *qbits = nullptr;
    if (a.asg.bits && (!a.asg_qiso || gb_dyn_nonzero(a.asg_qiso, a.asg_qiso_code))) qbits = ubits;
    long long mfn = 0, cnt = 0, adelta = 0;
    if (a.dbg & 4)
        ;
    else if (a.root >= 0)
        cnt = gb_push_root(a.root, prow, pcol, mbits, mcomp, (unsigned long long *)tbits, a.hprow, mfn,
                           a.asg.bits != nullptr, a.asg, adelta);
    else if (push)
        cnt = gb_push_phase(nwords_u, ubits, prow, pcol, hubs, nhubs, H, mbits, mcomp,
                            (unsigned long long *)tbits, L, a.hprow, mfn, qbits, a.asg, adelta, (a.dbg & 128) != 0,
                            (a.dbg & 512) == 0);
    else
        cnt = gb_pull_iso_phase(nrows, rowptr, colidx, ubits, mbits, mcomp, tbits, L, a.hprow, mfn, a.p1_steps,
                                a.cap0, a.rows_nonempty, qbits, a.asg, adelta, a.dbg,
                                (a.phead && (!a.hprow || a.pdeg)) ? a.phead : nullptr, a.pdeg);
    if (a.dbg & 64) return;  // diagnostics: no finish (count, hint, mailbox)
    if (a.packed) {
        iso_finish_packed(cnt, mfn, adelta, tcount, gst, a);
        return;
    }
    long long tot;
    if (gb_grid_sum(cnt, gst, &tot)) {
        *tcount = (unsigned long long)tot;
        if (a.iso_out) gb_iso_eval(a.mul, a.xcode, a.zcode, a.flip, a.a0, a.u0, a.iso_out);
        iso_publish(a, tot);
    }
    if (a.mf_out && !(a.dbg & 2)) {
        long long m;
        if (gb_grid_sum(mfn, gst + GB_GRID2_OFFSET, &m)) {
            a.mf_out[0] = m;
            for (int i = 1; i < GB_HINT_PARTS; i++) a.mf_out[i] = 0;
        }
    }
    if (a.asg.bits) gb_grid_add(adelta, a.asg_count, gst + GB_GRID3_OFFSET);
}

// hub-chunk table of a CSR: pieces per row, then (row, piece) pairs
__global__ void k_hub_count(const int64_t *__restrict__ rowptr, int64_t n, int64_t thresh, int64_t H,
                            int64_t *__restrict__ cnt) {
    for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < n; r += (int64_t)gridDim.x * blockDim.x) {
        const int64_t d = rowptr[r + 1] - rowptr[r];
        cnt[r] = d > thresh ? (d + H - 1) / H : 0;
    }
}
__global__ void k_hub_fill(const int64_t *__restrict__ cnt, const int64_t *__restrict__ off, int64_t n,
                           int32_t *__restrict__ tab) {
    for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < n; r += (int64_t)gridDim.x * blockDim.x) {
        const int64_t c = cnt[r], o = off[r];
        for (int64_t i = 0; i < c; i++) {
            tab[2 * (o + i)] = (int32_t)r;
            tab[2 * (o + i) + 1] = (int32_t)i;
        }
    }
}

// (row, piece) table of the rows of v longer than thresh, cut into H-entry pieces
static int32_t *gb_build_chunk_table(const gb_csr_view &v, int64_t thresh, int64_t H, int64_t *total_out) {
    const int64_t n = v.nrows;
    gb_scratch s;
    int64_t *cnt = s.get<int64_t>(n + 1);
    int64_t *off = s.get<int64_t>(n + 1);
    const unsigned g = (unsigned)std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, 8192));
    hipLaunchKernelGGL(k_hub_count, dim3(g), dim3(256), 0, gb_stream(), v.rowptr, n, thresh, H, cnt);
    GB_LAUNCH_CHECK();
    gb_exclusive_scan_i64(cnt, off, n);
    const int64_t total = gb_read_i64(off + n);
    int32_t *tab = gb_malloc_n<int32_t>(2 * total + 2);
    hipLaunchKernelGGL(k_hub_fill, dim3(g), dim3(256), 0, gb_stream(), cnt, off, n, tab);
    GB_LAUNCH_CHECK();
    *total_out = total;
    return tab;
}

__global__ void k_row_maxlen(const int64_t *__restrict__ rowptr, int64_t n, unsigned long long *__restrict__ mx) {
    unsigned long long m = 0;
    for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < n; r += (int64_t)gridDim.x * blockDim.x) {
        const unsigned long long d = (unsigned long long)(rowptr[r + 1] - rowptr[r]);
        m = d > m ? d : m;
    }
    for (int off = 32; off > 0; off >>= 1) {
        const unsigned long long o = __shfl_xor(m, off, 64);
        m = o > m ? o : m;
    }
    if ((threadIdx.x & 63) == 0 && m) atomicMax(mx, m);
}

void gb_view_hubs(gb_csr_view &v, GB_Obj *A, int orient, int64_t H) {
    if (A->kind != GB_KIND_MATRIX) return;
    if (!A->hub_tab[orient] || A->hub_H[orient] != H) {
        gb_free(A->hub_tab[orient]);
        A->hub_tab[orient] = gb_build_chunk_table(v, H, H, &A->hub_n[orient]);
        A->hub_H[orient] = H;
        // the longest row, for host-side direction decisions on small frontiers (gb_spmv)
        gb_scratch s;
        unsigned long long *mx = s.get<unsigned long long>(1);
        gb_memset(mx, 0, sizeof(unsigned long long));
        const unsigned g = (unsigned)std::max<int64_t>(1, std::min<int64_t>((v.nrows + 255) / 256, 2048));
        hipLaunchKernelGGL(k_row_maxlen, dim3(g), dim3(256), 0, gb_stream(), v.rowptr, v.nrows, mx);
        GB_LAUNCH_CHECK();
        unsigned long long h = 0;
        gb_copy_d2h(&h, mx, sizeof(h));
        A->maxdeg[orient] = (int64_t)h + 1;  // stored + 1: 0 means not built
    }
    v.hubs = A->hub_tab[orient];
    v.nhubs = A->hub_n[orient];
    v.hub_H = H;
    v.maxdeg = A->maxdeg[orient] - 1;
}

void gb_view_long_rows(gb_csr_view &v, GB_Obj *A, int orient) {
    if (A->kind != GB_KIND_MATRIX) return;
    if (!A->long_tab[orient]) A->long_tab[orient] = gb_build_chunk_table(v, SPMV_LONG, SPMV_CH, &A->long_n[orient]);
    v.lchunks = A->long_tab[orient];
    v.nlchunks = A->long_n[orient];
}

__global__ void k_rows_nonempty(const int64_t *__restrict__ rowptr, int64_t n, uint64_t *__restrict__ ne) {
    const int lane = threadIdx.x & 63;
    const int64_t nw = (n + 63) >> 6;
    for (int64_t w = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6; w < nw;
         w += ((int64_t)gridDim.x * blockDim.x) >> 6) {
        const int64_t r = (w << 6) + lane;
        const unsigned long long b = __ballot(r < n && rowptr[r + 1] > rowptr[r]);
        if (lane == 0) ne[w] = b;
    }
}

void gb_view_nonempty(gb_csr_view &v, GB_Obj *A, int orient) {
    if (A->kind != GB_KIND_MATRIX) return;
    if (!A->rows_ne[orient]) {
        const int64_t nw = gb_words(v.nrows);
        A->rows_ne[orient] = gb_malloc_n<uint64_t>(nw);
        const unsigned g = (unsigned)std::max<int64_t>(1, std::min<int64_t>((nw + 3) / 4, 8192));
        hipLaunchKernelGGL(k_rows_nonempty, dim3(g), dim3(256), 0, gb_stream(), v.rowptr, v.nrows,
                           A->rows_ne[orient]);
        GB_LAUNCH_CHECK();
    }
    v.nonempty = A->rows_ne[orient];
}

// pull heads: a wave per row picks its neighbours with the longest rows in the other
// orientation (ties: the smaller index) -- in a level BFS those are the ones most likely to
// be in the frontier, so most rows the pull settles are settled by them -- 3 of them for a
// row longer than 4 (4th slot -2: "walk the row"), the whole row otherwise (padding -1), and
// stores the row's own length in the other orientation (the next-frontier hint of a row
// settled without reading its bounds)
__device__ __forceinline__ void pf_better(int64_t &bd, int32_t &bi, int64_t d, int32_t i) {
    if (i >= 0 && (d > bd || (d == bd && (bi < 0 || i < bi)))) {
        bd = d;
        bi = i;
    }
}
__global__ __launch_bounds__(256) void k_pull_head(int64_t n, const int64_t *__restrict__ rp,
                                                   const int32_t *__restrict__ ci,
                                                   const int64_t *__restrict__ orp, int64_t on,
                                                   int4 *__restrict__ head, uint32_t *__restrict__ pdeg) {
    const int lane = threadIdx.x & 63;
    const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
    for (int64_t j = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6; j < n; j += nwaves) {
        const int64_t e0 = rp[j], e1 = rp[j + 1], d = e1 - e0;
        int32_t pick[4] = {-1, -1, -1, -1};
        const int rounds = d <= 4 ? (int)d : 3;
        for (int r = 0; r < rounds; r++) {
            int64_t bd = -1;
            int32_t bi = -1;
            for (int64_t e = e0 + lane; e < e1; e += 64) {
                const int32_t i = ci[e];
                bool taken = false;
                for (int q = 0; q < r; q++) taken = taken || pick[q] == i;
                if (!taken) pf_better(bd, bi, orp[i + 1] - orp[i], i);
            }
            for (int off = 32; off > 0; off >>= 1) {
                const int64_t od = __shfl_xor(bd, off, 64);
                const int32_t oi = __shfl_xor(bi, off, 64);
                pf_better(bd, bi, od, oi);
            }
            pick[r] = bi;  // identical on every lane
        }
        if (d > 4) pick[3] = -2;
        if (lane == 0) {
            head[j] = make_int4(pick[0], pick[1], pick[2], pick[3]);
            if (pdeg) {
                const int64_t od = j < on ? orp[j + 1] - orp[j] : 0;
                pdeg[j] = (uint32_t)(od < 0xFFFFFFFFLL ? od : 0xFFFFFFFFLL);
            }
        }
    }
}

void gb_view_pullfirst(gb_csr_view &v, GB_Obj *A, int orient, const int64_t *other_rowptr, int64_t other_n) {
    if (A->kind != GB_KIND_MATRIX || v.nrows == 0) return;
    if (!A->phead[orient]) {
        A->phead[orient] = gb_malloc_n<int32_t>(4 * v.nrows);
        A->pdeg[orient] = gb_malloc_n<uint32_t>(v.nrows);
        const unsigned g = (unsigned)std::max<int64_t>(1, std::min<int64_t>((v.nrows + 3) / 4, 65535));
        hipLaunchKernelGGL(k_pull_head, dim3(g), dim3(256), 0, gb_stream(), v.nrows, v.rowptr, v.colidx,
                           other_rowptr, other_n, reinterpret_cast<int4 *>(A->phead[orient]), A->pdeg[orient]);
        GB_LAUNCH_CHECK();
    }
    v.phead = A->phead[orient];
    v.pdeg = A->pdeg[orient];
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

static std::mutex g_dir_mu;
static unsigned long long *g_iso_ts = nullptr;  // GRAPHBLAS_AMD_ISO_TS diagnostics buffer
static unsigned long long *iso_ts_buffer() {
    static const bool on = getenv("GRAPHBLAS_AMD_ISO_TS") != nullptr;
    if (!on) return nullptr;
    if (!g_iso_ts) {
        GB_HIP(hipMalloc((void **)&g_iso_ts, (2 + 2 * (size_t)ISO_TS_PAIRS) * sizeof(unsigned long long)));
        GB_HIP(hipMemset(g_iso_ts, 0, (2 + 2 * (size_t)ISO_TS_PAIRS) * sizeof(unsigned long long)));
        GB_HIP(hipDeviceSynchronize());
    }
    return g_iso_ts;
}
// writes the stamps to the file GRAPHBLAS_AMD_ISO_TS names (raw u64: starts, ends, pairs); returns the
// launch count (GxB_Global_get_int("iso_ts_dump"))
int64_t gb_iso_ts_dump() {
    const char *path = getenv("GRAPHBLAS_AMD_ISO_TS");
    if (!path || !g_iso_ts) return 0;
    GB_HIP(hipStreamSynchronize(gb_stream()));
    unsigned long long c[2];
    GB_HIP(hipMemcpy(c, g_iso_ts, sizeof(c), hipMemcpyDeviceToHost));
    const size_t k = std::min<unsigned long long>(std::min(c[0], c[1]), ISO_TS_PAIRS);
    std::vector<unsigned long long> buf(2 + 2 * k);
    GB_HIP(hipMemcpy(buf.data(), g_iso_ts, buf.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost));
    FILE *f = fopen(path, "wb");
    if (!f) return -1;
    fwrite(buf.data(), sizeof(unsigned long long), buf.size(), f);
    fclose(f);
    return (int64_t)k;
}
static uint64_t *g_spare = nullptr;  // zeroed bitmap for the next iso SpMV's output (under g_dir_mu)
static int64_t g_spare_words = 0;

// ---- pool of zeroed vector storage (under g_dir_mu): bitmaps of one size (g_zp_words) and
// counts; `dirty` ones are zeroed by the next k_iso_work launch, then become `ready`
static std::vector<uint64_t *> g_zp_ready_b, g_zp_dirty_b;
static std::vector<int64_t *> g_zp_ready_c, g_zp_dirty_c;
static int64_t g_zp_words = 0;

bool gb_zpool_clear_vector(GB_Obj *v) {
    if (gb_knob("zero_pool") == 1) return false;
    std::lock_guard<std::mutex> lk(g_dir_mu);
    const int64_t nw = gb_words(v->nrows);
    if (nw != g_zp_words) {  // a new size: the pool follows the most recent one
        for (auto *p : g_zp_ready_b) gb_free(p);
        for (auto *p : g_zp_dirty_b) gb_free(p);
        g_zp_ready_b.clear();
        g_zp_dirty_b.clear();
        g_zp_words = nw;
    }
    if (v->bits && (int)g_zp_dirty_b.size() < GB_ZP_MAX) {  // the old bitmap, to be zeroed later
        g_zp_dirty_b.push_back(v->bits);
        v->bits = nullptr;
    }
    if (g_zp_ready_b.empty() || g_zp_ready_c.empty()) return false;
    gb_cw_release(v);
    gb_free(v->bits);
    gb_free(v->dense);
    gb_free(v->d_nvals);
    v->bits = g_zp_ready_b.back();
    g_zp_ready_b.pop_back();
    v->d_nvals = g_zp_ready_c.back();
    g_zp_ready_c.pop_back();
    v->dense = nullptr;
    v->iso = false;
    v->nvals = 0;
    v->nvals_valid = true;
    v->hint_valid = false;
    v->pub_seq = 0;
    return true;
}

// blocks of k_iso_work the device holds at once (the work grid is sized to one wave of blocks)
static int64_t iso_work_resident_blocks() {
    static int64_t cap = 0;
    if (!cap) {
        int dev = 0, cus = 0, per = 0;
        GB_HIP(hipGetDevice(&dev));
        GB_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
        GB_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k_iso_work, SPMV_BLOCK, 0));
        cap = std::max<int64_t>(1, (int64_t)cus * std::max(per, 1));
    }
    return cap;
}  // keeps the prep/push/pull launches of one call adjacent

bool gb_spmv_result_iso(GrB_Semiring sr, bool a_iso, bool u_iso, bool flip) {
    gb_sr_info info = gb_sr_describe(sr);
    bool reads_a = info.reads_values, reads_u = info.reads_values;
    if (info.mul == GBAMD_OP_FIRST) (flip ? reads_a : reads_u) = false;
    if (info.mul == GBAMD_OP_SECOND) (flip ? reads_u : reads_a) = false;
    if (info.mul == GBAMD_OP_PAIR) return idempotent_monoid(info.mon);
    return !info.positional && idempotent_monoid(info.mon) && (!reads_a || a_iso) && (!reads_u || u_iso);
}

void gb_spmv(gb_vec_result &T, const gb_csr_view &A, const gb_csr_view *Apush, gb_bitmap_view &u,
             const gb_vmask &mask, GrB_Semiring sr, bool flip, const gb_asg *asg) {
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
    // [0] count; [2 .. 2 + GB_HINT_PARTS): next-frontier edge hint in parts (iso path)
    T.d_nvals = gb_malloc_n<int64_t>(2 + GB_HINT_PARTS);
    if (n == 0) {
        gb_memset(T.d_nvals, 0, sizeof(int64_t));
        return;
    }

    const int64_t dir_knob = gb_knob("spmv_direction");  // 0 auto, 1 pull only, 2 push only
    const bool can_push = iso && Apush && Apush->nrows == u.n && Apush->hubs && dir_knob != 1;
    int64_t alpha = gb_knob("push_alpha");
    // Beamer's alpha, swept with tools/ab_bfs.py (s22, 16 roots, 8 interleaved rounds; two boxes):
    // 14 -> 0.312 / 0.328 ms per BFS, 36 -> 0.299 / 0.318, 48 -> 0.2985, 64 -> 0.314, 96 -> 0.323
    if (alpha <= 0) alpha = 48;
    const int64_t nw = gb_words(n);
    unsigned long long *gst = gb_device_state();
    unsigned long long *dst = gst + GB_DIR_STATE_OFFSET;

    gb_dispatch_sr(info, [&](auto srf, auto x, auto z) {
        using SRT = decltype(srf);
        using X = decltype(x);
        using Z = decltype(z);
        if (iso) {
            const int64_t uw = gb_words(u.n);
            int64_t units = (nw + PULL_U - 1) / PULL_U;  // waves the pull wants
            std::lock_guard<std::mutex> lk(g_dir_mu);  // the spare bitmap and the direction state
            gb_iso_args args{};
            args.rule = gb_dir_rule{mask.count, asg ? u.count : nullptr, mask.comp, n, A.nvals, alpha, dir_knob == 2};
            if (asg) {
                GB_REQUIRE(u.n == n, GrB_INVALID_VALUE, "fused assign needs u and w of one size");
                args.asg = gb_asg_dev{asg->bits, asg->vals, asg->size, asg->x};
                args.asg_qiso = asg->q_iso;
                args.asg_qiso_code = asg->q_iso_code;
                args.asg_count = (unsigned long long *)asg->count;
            }
            args.dbg = (int)gb_knob("iso_dbg");
            args.ts = iso_ts_buffer();
            args.root = asg ? asg->root : -1;
            GB_REQUIRE(args.root < 0 || can_push, GrB_PANIC, "a pending root needs the push orientation");
            args.packed = n < (1LL << ISO_VAL_BITS) && u.n < (1LL << ISO_VAL_BITS) && gb_knob("iso_packed") != 1;
            if (args.dbg & 1) T.pub = nullptr;  // diagnostics: the host reads the count by a copy
            // lane-per-row steps after the pull heads: none by default (tools/gpu_ab2.sh, s22
            // any_pair: 0.340 ms/BFS without, 0.356 with 2, 0.350 with 1)
            args.p1_steps = (int)gb_knob("pull_steps");
            if (args.p1_steps < 0) args.p1_steps = 0;
            // first per-row cap of the pull's segment-list rounds: tools/ab_bfs.py (s22, 6 interleaved
            // rounds, after the two-round head probes): 16 -> 0.2285, 32 -> 0.2266, 64 -> 0.2260 ms/BFS
            args.cap0 = (int)gb_knob("pull_cap");
            if (args.cap0 <= 0) args.cap0 = 64;
            args.rows_nonempty = A.nonempty;
            args.phead = A.phead;
            args.pdeg = A.pdeg;
            // the result's iso value: evaluated by the finishing block when z is x's type or bool
            const bool eval_ok = info.zcode == info.xcode || info.zcode == GBAMD_T_BOOL;
            if (eval_ok) {
                args.mul = info.mul;
                args.xcode = info.xcode;
                args.zcode = info.zcode;
                args.flip = flip;
                args.a0 = av;
                args.u0 = uv;
                args.iso_out = T.dense;
            }
            args.pub = T.pub ? gb_host_slot_device(T.pub) : nullptr;
            args.pub_seq = (long long)T.pub_seq;
            // the count travels in one tagged word stored without a fence: the host needs only the
            // count, and the kernel's end orders everything else for the next launch.  With the
            // BFS speculation on, tools/ab_bfs.py (s22, 8 interleaved rounds): 0.2298 ms per BFS
            // vs 0.2325 with value + system fence + release seq (round 3 had measured the reverse
            // without speculation, when the host waited on every mailbox)
            args.pub_form = n < (1LL << 31) ? (int)std::max<int64_t>(0, std::min<int64_t>(2, gb_knob("iso_pub"))) : 1;
            // a zeroed output bitmap left by the previous call (push may write into it directly)
            bool spare_taken = false;
            if (g_spare && g_spare_words == nw) {
                gb_free(T.bits);
                T.bits = g_spare;
                spare_taken = true;
            } else if (g_spare) {
                gb_free(g_spare);
            }
            g_spare = nullptr;
            g_spare_words = 0;
            args.out_zeroed = spare_taken;
            if (asg && asg->u_count_exact && u.count && asg->root < 0 && gb_knob("spec_empty_exit") != 1)
                args.u_exit = u.count;
            bool need_prep = false;
            if (can_push) {
                units = std::max<int64_t>(units, std::max<int64_t>((Apush->nhubs + 15) / 16, (uw + 3) / 4));
                if (n == u.n) {  // outputs index the same vertex space as u: they can seed the next call
                    args.hprow = Apush->rowptr;
                    args.mf_out = (long long *)(T.d_nvals + 2);
                    T.hint_key = Apush->rowptr;
                }
                const bool hint_ok = u.mf_hint && u.hint_key == Apush->rowptr;
                // no hint (a frontier set by the host, e.g. a BFS root): push is certain when even
                // every frontier vertex having the longest row stays under the pull's least work
                bool push_sure = false;
                if (!hint_ok && spare_taken && eval_ok && u.h_nvals >= 0 && Apush->maxdeg >= 0 &&
                    gb_knob("host_dir") != 1) {
                    // open rows (where the output may be written) from below.  mask.h_count is the
                    // mask's set-bit count; do_spmv fills it from a stored-entry count (an upper
                    // bound on the set bits of a value mask, whose stored entries may be false)
                    // only for structural or complemented masks, or when the mask is empty -- so
                    // for a plain value mask it is never an over-estimate (tests/test_gpu_parity.py::
                    // test_value_mask_false_entries_no_host_push)
                    int64_t open_lo = -1;
                    if (!mask.bits) {
                        open_lo = n;
                    } else if (mask.h_count >= 0) {
                        const int64_t mc_hi = std::min<int64_t>(n, mask.h_count + (asg ? u.h_nvals : 0));
                        open_lo = mask.comp ? n - mc_hi : mask.h_count;
                    }
                    const double avg = n ? (double)A.nvals / (double)n : 0.0;
                    push_sure = open_lo >= 0 &&
                                (double)u.h_nvals * (double)Apush->maxdeg * (double)alpha < (double)open_lo * avg;
                }
                if (args.root >= 0) {
                    // the frontier is one vertex the host knows; the push writes T's bitmap directly, so
                    // it must start zeroed (the spare usually is; a first call zeroes it here)
                    if (!spare_taken) gb_memset(T.bits, 0, nw * sizeof(uint64_t));
                    args.out_zeroed = true;
                    args.host_dir = 1;
                    g_stat_host_push.fetch_add(1, std::memory_order_relaxed);
                    gb_stat_add("bfs_root_push", 1);
                } else if (hint_ok && spare_taken) {
                    args.mf_hint = u.mf_hint;  // decide in the work kernel: one launch
                } else if (push_sure) {
                    args.host_dir = 1;  // one launch, no prep
                    g_stat_host_push.fetch_add(1, std::memory_order_relaxed);
                } else {
                    need_prep = true;
                }
            }
            if (need_prep || (!eval_ok && can_push)) {
                // prep (frontier edges -> direction, zeroed output, iso value), then the work launch
                int64_t pcap = gb_knob("prep_grid");
                if (pcap <= 0) pcap = 1024;
                const unsigned prep_grid =
                    (unsigned)std::max<int64_t>(1, std::min<int64_t>((uw + 63) / 64, pcap));
                if (flip)
                    hipLaunchKernelGGL((k_dir_prep<SRT, X, Z, true>), dim3(prep_grid), dim3(SPMV_BLOCK), 0,
                                       gb_stream(), srf, u.bits, uw, Apush->rowptr, gst, dst, T.bits, nw,
                                       (unsigned long long *)T.d_nvals, (const X *)av, (const X *)uv, (Z *)T.dense,
                                       args.rule);
                else
                    hipLaunchKernelGGL((k_dir_prep<SRT, X, Z, false>), dim3(prep_grid), dim3(SPMV_BLOCK), 0,
                                       gb_stream(), srf, u.bits, uw, Apush->rowptr, gst, dst, T.bits, nw,
                                       (unsigned long long *)T.d_nvals, (const X *)av, (const X *)uv, (Z *)T.dense,
                                       args.rule);
                GB_LAUNCH_CHECK();
                args.mf_hint = nullptr;
                args.dst = dst;
            } else if (!eval_ok) {
                if (flip)
                    hipLaunchKernelGGL((k_iso_value<SRT, X, Z, true>), dim3(1), dim3(1), 0, gb_stream(), srf,
                                       (const X *)av, (const X *)uv, (Z *)T.dense);
                else
                    hipLaunchKernelGGL((k_iso_value<SRT, X, Z, false>), dim3(1), dim3(1), 0, gb_stream(), srf,
                                       (const X *)av, (const X *)uv, (Z *)T.dense);
                GB_LAUNCH_CHECK();
            }
            if (can_push) {  // zeroed by this launch, for the next call's push output
                args.spare = gb_malloc_n<uint64_t>(nw);
                args.spare_words = nw;
            }
            // cleared vectors' storage (gb_zpool_clear_vector): zeroed by this launch, then ready
            while ((int)(g_zp_ready_c.size() + g_zp_dirty_c.size()) < GB_ZP_MAX)
                g_zp_dirty_c.push_back(gb_malloc_n<int64_t>(2 + GB_HINT_PARTS));
            args.nzb = (int)std::min<size_t>(g_zp_dirty_b.size(), GB_ZP_MAX);
            for (int j = 0; j < args.nzb; j++) args.zb[j] = g_zp_dirty_b[j];
            args.zb_words = g_zp_words;
            args.nzc = (int)std::min<size_t>(g_zp_dirty_c.size(), GB_ZP_MAX);
            for (int j = 0; j < args.nzc; j++) args.zc[j] = g_zp_dirty_c[j];
            if (args.dbg & (8 | 32)) {
                // diagnostics that return before (8) or skip (32) the zeroing: nothing handed to this
                // launch may be treated as zeroed afterwards
                args.nzb = args.nzc = 0;
                if (args.spare) gb_free(args.spare);
                args.spare = nullptr;
                args.spare_words = 0;
            }
            int64_t gcap = gb_knob("iso_work_grid");
            if (gcap <= 0) gcap = iso_work_resident_blocks();
            // a frontier the host knows to be tiny (the BFS loop reads nvals every level): a small
            // grid -- the work is a few rows, and the finish's grid-wide sum and the drain of
            // fewer blocks are what the level costs
            const int64_t small_n = gb_knob("iso_small_n");
            if (small_n > 0 && u.h_nvals >= 0 && u.h_nvals <= small_n) {
                int64_t sg = gb_knob("iso_small_grid");
                if (sg <= 0) sg = 64;
                gcap = std::min<int64_t>(gcap, sg);
            }
            const unsigned grid = (unsigned)std::max<int64_t>(1, std::min<int64_t>((units + 3) / 4, gcap));
            if (grid >= GB_GRID_SHARDS * ((1u << ISO_ARR_BITS) - 1)) args.packed = false;  // arrival field
            GB_HPROF(5, "k_iso_work launch");
            hipLaunchKernelGGL(k_iso_work, dim3(grid), dim3(SPMV_BLOCK), 0, gb_stream(), n, A.rowptr, A.colidx, uw,
                               u.bits, can_push ? Apush->rowptr : nullptr, can_push ? Apush->colidx : nullptr,
                               can_push ? Apush->hubs : nullptr, can_push ? Apush->nhubs : 0,
                               can_push ? Apush->hub_H : 1, mask.bits, mask.comp, T.bits,
                               (unsigned long long *)T.d_nvals, gst, args);
            GB_LAUNCH_CHECK();
            g_spare = args.spare;
            g_spare_words = args.spare ? nw : 0;
            for (int j = 0; j < args.nzb; j++) g_zp_ready_b.push_back(args.zb[j]);
            g_zp_dirty_b.erase(g_zp_dirty_b.begin(), g_zp_dirty_b.begin() + args.nzb);
            for (int j = 0; j < args.nzc; j++) g_zp_ready_c.push_back(args.zc[j]);
            g_zp_dirty_c.erase(g_zp_dirty_c.begin(), g_zp_dirty_c.begin() + args.nzc);
            T.published = T.pub != nullptr;
            return;
        }
        if (A.nlchunks >= 0 && gb_knob("spmv_general") != 1) {
            // general semiring: balanced words + long-row chunks (+ their fold)
            Z *cpart = s.get<Z>(A.nlchunks + 1);
            int8_t *cfound = s.get<int8_t>(A.nlchunks + 1);
            const int64_t units = std::max<int64_t>(nw, A.nlchunks);
            const bool u_iso_k = u.iso || gb_knob("spmv_timing_no_x_gather") == 1;  // timing experiment only
            int spmv_mode = gb_knob("spmv_words") == 2 ? 1 : 0;  // 0: segmented scan (default), 2: merge path
            if (gb_knob("spmv_nt") == 1) spmv_mode |= 2;
            const unsigned grid = (unsigned)std::max<int64_t>(1, std::min<int64_t>((units + 3) / 4, 4096));
            // dense u on a relabelled matrix: the hot columns' values packed first (gb_view_hot);
            // positional multipliers need the true column, so they keep the plain colidx
            const int32_t *ci = A.colidx;
            X *uhot = nullptr;
            if (A.hcolidx && u.full && !u_iso_k && uv && !info.positional && info.reads_values) {
                uhot = s.get<X>(A.nhot);
                const unsigned hg = (unsigned)std::max<int64_t>(1, std::min<int64_t>((A.nhot + 255) / 256, 2048));
                hipLaunchKernelGGL((k_hot_gather<X>), dim3(hg), dim3(256), 0, gb_stream(), (const X *)uv, A.hcols,
                                   A.nhot, uhot);
                GB_LAUNCH_CHECK();
                ci = A.hcolidx;
            }
            if (flip)
                hipLaunchKernelGGL((k_spmv_words<SRT, X, Z, true>), dim3(grid), dim3(SPMV_BLOCK), 0, gb_stream(), srf,
                                   n, A.rowptr, ci, (const X *)av, A.iso, u.bits, (const X *)uv, u_iso_k,
                                   mask.bits, mask.comp, A.lchunks, A.nlchunks, cpart, cfound, T.bits, (Z *)T.dense,
                                   (unsigned long long *)T.d_nvals, gst, u.count, u.n, spmv_mode, (const X *)uhot);
            else
                hipLaunchKernelGGL((k_spmv_words<SRT, X, Z, false>), dim3(grid), dim3(SPMV_BLOCK), 0, gb_stream(),
                                   srf, n, A.rowptr, ci, (const X *)av, A.iso, u.bits, (const X *)uv, u_iso_k,
                                   mask.bits, mask.comp, A.lchunks, A.nlchunks, cpart, cfound, T.bits, (Z *)T.dense,
                                   (unsigned long long *)T.d_nvals, gst, u.count, u.n, spmv_mode, (const X *)uhot);
            GB_LAUNCH_CHECK();
            if (A.nlchunks > 0) {
                const unsigned fg = (unsigned)std::max<int64_t>(1, std::min<int64_t>((A.nlchunks + 255) / 256, 1024));
                hipLaunchKernelGGL((k_spmv_fold<SRT, Z>), dim3(fg), dim3(256), 0, gb_stream(), srf, A.lchunks,
                                   A.nlchunks, cpart, cfound, T.bits, (Z *)T.dense, (unsigned long long *)T.d_nvals,
                                   gst);
                GB_LAUNCH_CHECK();
            }
            return;
        }
        // fallback (no long-row table: the operand is not a matrix object): G lanes per row
        gb_memset(T.d_nvals, 0, sizeof(int64_t));
        const int64_t avg = (A.nvals + n - 1) / n;
        int lg = 0;
        while (lg < 6 && (1LL << lg) < avg) lg++;
        const int64_t forced = gb_knob("spmv_lg");
        if (forced > 0) lg = (int)(forced - 1);
        const unsigned grid = (unsigned)std::min<int64_t>((n + SPMV_TILE - 1) / SPMV_TILE, 2048);
        if (flip)
            hipLaunchKernelGGL((k_spmv_pull<SRT, X, Z, true>), dim3(grid), dim3(SPMV_BLOCK), 0, gb_stream(), srf, n,
                               A.rowptr, A.colidx, (const X *)av, A.iso, u.bits, (const X *)uv, u.iso, mask.bits,
                               mask.comp, lg, T.bits, (Z *)T.dense, (unsigned long long *)T.d_nvals, gst);
        else
            hipLaunchKernelGGL((k_spmv_pull<SRT, X, Z, false>), dim3(grid), dim3(SPMV_BLOCK), 0, gb_stream(), srf, n,
                               A.rowptr, A.colidx, (const X *)av, A.iso, u.bits, (const X *)uv, u.iso, mask.bits,
                               mask.comp, lg, T.bits, (Z *)T.dense, (unsigned long long *)T.d_nvals, gst);
        GB_LAUNCH_CHECK();
    });
}
