// gb_dot.hip -- masked dot-product SpGEMM, two-sided LDS method: the kernel
// behind GrB_mxm with a non-complemented mask (replaces SuiteSparse's
// GB_AxB_dot3, reached from reference core/matrix.py:2241 via core/base.py:483)
// for monoids whose fold order cannot change the result (exact_monoid in
// gb_mxm.hip: min/max on integers, integer plus/times, logical/bitwise, any_pair).
//
// T(i,j) for (i,j) in M intersects the sorted lists A'(i,:) and B'^T(j,:).  The
// cost of an intersection is set by the shorter list when the longer one can be
// searched cheaply, and the longer list is shared by every mask entry of its row
// (A' side) or column (B'^T side).  So every mask entry is given to the side
// that owns its longer list:
//   phase R: entries with |A'(i,:)| >= |B'^T(j,:)|, grouped by mask row i
//            (the mask's CSR);
//   phase C: entries with |B'^T(j,:)| > |A'(i,:)|, grouped by mask column j
//            (the mask's CSC, whose position map gives each entry's CSR slot).
// Per group g (row or column) the longer list X(g,:) is loaded once; each
// entry's shorter list Y(o,:) is streamed (coalesced) and every key is searched
// in X(g,:):
//   * |X(g,:)| <= 64: a wave per group, X's keys and values held one per lane,
//     membership by a 6-step shuffle search (k_dot_small);
//   * |X(g,:)| <= 16384: a workgroup per task, X's keys in LDS (64 KB) behind a
//     hashed membership bitmap (32 KB: one LDS read rejects most keys), binary
//     search for the rest; tasks are runs of one group's entries cut at fixed
//     windows of streamed work (<= 256 entries), so R-MAT hub rows are spread over
//     many workgroups; one flat stream over the task's entries keeps every lane
//     busy for short and long Y lists alike (k_dot_task);
//   * longer (R-MAT's largest hubs): the per-entry wave kernel of gb_mxm.hip.
// Work is sum over mask entries of min(|A'(i,:)|, |B'^T(j,:)|) streamed keys
// plus one LDS search each -- instead of a search in global memory per key.
#include <algorithm>
#include <climits>
#include <cstdio>

#include "gb_dispatch.cuh"
#include "gb_internal.h"

namespace {

constexpr int DT_BLOCK = 256;
constexpr int DT_SMALL = 64;      // long side <= 64: k_dot_small, keys one per lane
constexpr int DT_MID = 256;       // long side <= 256: k_dot_small, four keys per lane
constexpr int DT_CAP = 8191;      // long side <= DT_CAP: k_dot_task (keys in LDS, a 13-level Eytzinger tree)
constexpr int DT_OVH = 64;        // per-entry cost added to the streamed length (task windows)
constexpr int DT_OVH_MIN = 64;    // the least per-entry cost (knob dot_ovh): sizes the task's entry arrays
constexpr int DT_WIN = 32768;     // task window: <= DT_WIN / ovh entries start in one
constexpr int DT_MAXE = DT_WIN / DT_OVH_MIN;

static inline unsigned dt_grid(int64_t n, int per_block = DT_BLOCK, int64_t cap = 1 << 16) {
    int64_t g = (n + per_block - 1) / per_block;
    if (g < 1) g = 1;
    if (g > cap) g = cap;
    return (unsigned)g;
}

// one phase's view: groups (rows of the mask for R, its columns for C), the
// longer lists X (indexed by group) and the shorter lists Y (indexed by the
// entry's other index)
struct dt_side {
    const int64_t *grp_rp;  // [ng+1] entries of group g: [grp_rp[g], grp_rp[g+1])
    const int32_t *grp_oi;  // [nm]   other index of each entry
    const int64_t *perm;    // [nm]   entry -> CSR position of the mask (nullptr: identity)
    int64_t ng;
    const int64_t *xrp;
    const int32_t *xci;
    const int64_t *yrp;
    const int32_t *yci;
};

// the entry belongs to this phase: R takes |X| >= |Y|, C takes |X| > |Y|
template <bool SWAP>
__device__ __forceinline__ bool dt_side_of(int64_t a, int64_t b) {
    return SWAP ? a > b : a >= b;
}

// a list side's values: full width, one iso value, or the cached narrow copy (gb_view_narrow:
// integer values that all fit 1-4 bytes, widened on load -- a hit's value read then touches a
// fraction of the cache lines)
template <class X>
struct dt_vals {
    const X *v;
    const void *nv;
    int nk;
    bool iso;
    __device__ __forceinline__ X operator[](int64_t i) const {
        if (iso) return v[0];
        if constexpr (std::is_integral<X>::value && !std::is_same<X, bool>::value && sizeof(X) > 1) {
            switch (nk) {
            case 1: return (X)((const uint8_t *)nv)[i];
            case -1: return (X)((const int8_t *)nv)[i];
            case 2: if constexpr (sizeof(X) > 2) return (X)((const uint16_t *)nv)[i]; break;
            case -2: if constexpr (sizeof(X) > 2) return (X)((const int16_t *)nv)[i]; break;
            case 4: if constexpr (sizeof(X) > 4) return (X)((const uint32_t *)nv)[i]; break;
            case -4: if constexpr (sizeof(X) > 4) return (X)((const int32_t *)nv)[i]; break;
            default: break;
            }
        }
        return v[i];
    }
};

// ---------------------------------------------------------------- classify
// flags (pre-zeroed): tflag[p] = 1 for this phase's entries of task-sized groups
// (G order); entries whose longer list exceeds the cap: hg[p] = 1 (G order) when
// they run as pieces, else hflag[q] = 1 (CSR order, the per-entry wave kernel)
template <bool SWAP>
__global__ __launch_bounds__(DT_BLOCK) void k_dt_classify(dt_side s, int cap, uint8_t *__restrict__ tflag,
                                                         uint8_t *__restrict__ hflag, uint8_t *__restrict__ hg,
                                                         bool hubs_chunked) {
    const int lane = threadIdx.x & 63;
    const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
    for (int64_t g = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6; g < s.ng; g += nw) {
        const int64_t a = s.xrp[g + 1] - s.xrp[g];
        if (a <= DT_MID) continue;  // k_dot_small (or nothing to match)
        if (hubs_chunked && a > cap) continue;  // k_dt_hub_classify
        for (int64_t p = s.grp_rp[g] + lane; p < s.grp_rp[g + 1]; p += 64) {
            const int32_t o = s.grp_oi[p];
            const int64_t b = s.yrp[o + 1] - s.yrp[o];
            if (b == 0 || !dt_side_of<SWAP>(a, b)) continue;  // an empty Y list matches nothing
            if (a <= cap) tflag[p] = 1;
            else if (hg) hg[p] = 1;  // pieces (G order)
            else hflag[s.perm ? s.perm[p] : p] = 1;
        }
    }
}

// compacted task entries in G order: group, Y start and length, other index, CSR slot
// (huge: the entries of groups longer than the cap, and the longest such group in *amax)
template <bool SWAP>
__global__ __launch_bounds__(DT_BLOCK) void k_dt_compact(dt_side s, int cap, const uint8_t *__restrict__ tflag,
                                                        const int64_t *__restrict__ pos, int32_t *__restrict__ eG,
                                                        int64_t *__restrict__ eYS, int32_t *__restrict__ eO,
                                                        int32_t *__restrict__ eB, int64_t *__restrict__ eQ, bool huge,
                                                        unsigned long long *__restrict__ amax) {
    const int lane = threadIdx.x & 63;
    const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
    for (int64_t g = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6; g < s.ng; g += nw) {
        const int64_t a = s.xrp[g + 1] - s.xrp[g];
        if (huge ? a <= cap : (a <= DT_MID || a > cap)) continue;
        if (huge && lane == 0) atomicMax(amax, (unsigned long long)a);
        for (int64_t p = s.grp_rp[g] + lane; p < s.grp_rp[g + 1]; p += 64) {
            if (!tflag[p]) continue;
            const int32_t o = s.grp_oi[p];
            const int64_t e = pos[p];
            const int64_t ys = s.yrp[o];
            eG[e] = (int32_t)g;
            eYS[e] = ys;
            eO[e] = o;
            eB[e] = (int32_t)(s.yrp[o + 1] - ys);
            eQ[e] = s.perm ? s.perm[p] : p;
        }
    }
}

// Hub groups (longer list X(g,:) above the cap) hold most of the entries of a few groups --
// an R-MAT hub row's group has up to ~10^5 entries -- so a wave per group leaves their entries
// to a handful of waves (round 4: the hub compaction took 1.8-2.2 ms per phase, latency-bound
// on those waves).  They are classified and compacted in chunks of DT_HCH entries instead, a
// workgroup per chunk: k_dt_hub_count sizes the chunks per group (0 for other groups), a scan
// numbers them, and the chunk kernels find their group by a binary search over that scan.
constexpr int DT_HCH = 2048;

__global__ void k_dt_hub_count(dt_side s, int cap, int32_t *__restrict__ nch, unsigned long long *__restrict__ amax) {
    for (int64_t g = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; g < s.ng; g += (int64_t)gridDim.x * blockDim.x) {
        const int64_t a = s.xrp[g + 1] - s.xrp[g], ne = s.grp_rp[g + 1] - s.grp_rp[g];
        const bool hub = a > cap && ne > 0;
        nch[g] = hub ? (int32_t)((ne + DT_HCH - 1) / DT_HCH) : 0;
        if (hub) atomicMax(amax, (unsigned long long)a);
    }
}

__device__ __forceinline__ int64_t dt_chunk_group(const int64_t *__restrict__ cp, int64_t ng, int64_t c) {
    int64_t lo = 0, hi = ng;  // last g with cp[g] <= c
    while (hi - lo > 1) {
        const int64_t m = (lo + hi) >> 1;
        if (cp[m] <= c) lo = m;
        else hi = m;
    }
    return lo;
}

// flags of the hub groups' entries: hg[p] = 1 (G order) when they run as pieces, else hflag[q] = 1
template <bool SWAP>
__global__ __launch_bounds__(DT_BLOCK) void k_dt_hub_classify(dt_side s, const int64_t *__restrict__ cp,
                                                             int64_t nchunk, uint8_t *__restrict__ hflag,
                                                             uint8_t *__restrict__ hg) {
    for (int64_t c = blockIdx.x; c < nchunk; c += gridDim.x) {
        const int64_t g = dt_chunk_group(cp, s.ng, c);
        const int64_t a = s.xrp[g + 1] - s.xrp[g];
        const int64_t p0 = s.grp_rp[g] + (c - cp[g]) * DT_HCH, pe = s.grp_rp[g + 1];
        const int64_t p1 = p0 + DT_HCH < pe ? p0 + DT_HCH : pe;
        for (int64_t p = p0 + threadIdx.x; p < p1; p += blockDim.x) {
            const int32_t o = s.grp_oi[p];
            const int64_t b = s.yrp[o + 1] - s.yrp[o];
            if (b == 0 || !dt_side_of<SWAP>(a, b)) continue;
            if (hg) hg[p] = 1;
            else hflag[s.perm ? s.perm[p] : p] = 1;
        }
    }
}

template <bool SWAP>
__global__ __launch_bounds__(DT_BLOCK) void k_dt_hub_compact(dt_side s, const int64_t *__restrict__ cp,
                                                            int64_t nchunk, const uint8_t *__restrict__ hg,
                                                            const int64_t *__restrict__ pos, int32_t *__restrict__ eG,
                                                            int64_t *__restrict__ eYS, int32_t *__restrict__ eO,
                                                            int32_t *__restrict__ eB, int64_t *__restrict__ eQ) {
    for (int64_t c = blockIdx.x; c < nchunk; c += gridDim.x) {
        const int64_t g = dt_chunk_group(cp, s.ng, c);
        const int64_t p0 = s.grp_rp[g] + (c - cp[g]) * DT_HCH, pe = s.grp_rp[g + 1];
        const int64_t p1 = p0 + DT_HCH < pe ? p0 + DT_HCH : pe;
        for (int64_t p = p0 + threadIdx.x; p < p1; p += blockDim.x) {
            if (!hg[p]) continue;
            const int32_t o = s.grp_oi[p];
            const int64_t e = pos[p];
            const int64_t ys = s.yrp[o];
            eG[e] = (int32_t)g;
            eYS[e] = ys;
            eO[e] = o;
            eB[e] = (int32_t)(s.yrp[o + 1] - ys);
            eQ[e] = s.perm ? s.perm[p] : p;
        }
    }
}

// Pieces of the longest lists (> cap keys): piece j of X(g,:) is its keys
// [j * cap, (j + 1) * cap).  An entry's work in piece j is the run of its Y keys
// inside the piece's key range (found by two binary searches), cut into sub-entries
// of at most cap keys (the task kernel's flat-space bound); cnt[i] = number of them.
__device__ __forceinline__ int64_t dt_lower(const int32_t *__restrict__ v, int64_t lo, int64_t hi, int32_t k) {
    while (lo < hi) {
        const int64_t m = (lo + hi) >> 1;
        if (v[m] < k) lo = m + 1;
        else hi = m;
    }
    return lo;
}

// The hub entries come in G order (hG ascending); the hub entries of group g are [h0, h1).
// Pairs (entry, piece) are numbered group by group, piece-major inside a group -- pair
// (i, j) = P[h0] + j * (h1 - h0) + (i - h0), P the exclusive scan of the entries' piece
// counts -- so a group's entries of one piece are consecutive (its tasks share that piece's
// keys in LDS) and the pair space is exactly the pieces the entries have (the
// round-4 piece-major layout was nh x the longest list's piece count).
// The span comes from the hub flags' exclusive scan `pos` (hub entry numbers in G order) at the
// group's entry bounds: two loads (a binary search over hG cost 44 dependent loads per entry).
__device__ __forceinline__ void dt_group_span(const dt_side &s, const int64_t *__restrict__ pos, int64_t g,
                                              int64_t &h0, int64_t &h1) {
    h0 = pos[s.grp_rp[g]];
    h1 = pos[s.grp_rp[g + 1]];
}

__global__ void k_dt_piece_count(dt_side s, int64_t nh, int cap, const int32_t *__restrict__ hG,
                                 int64_t *__restrict__ npc) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nh; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t g = hG[i], a = s.xrp[g + 1] - s.xrp[g];
        npc[i] = (a + cap - 1) / cap;
    }
}

// per pair: the entry's run of Y keys inside the piece's key range, cut into sub-entries of at
// most cap keys (the task kernel's flat-space bound).  Piece j's range is [X[j cap], X[(j+1) cap])
// (the last: to the end): the Y keys between a piece's last key and the next piece's first are
// in no piece of X, so they match nothing wherever they go, and one lower bound per piece start
// sizes every piece (round 4 searched both ends of each piece: 2 np searches per entry, now
// np + 1 per batch).  All of an entry's searches run in lockstep -- the branchless lower bound's
// length sequence depends only on the Y list's length -- so a batch of DT_PB pieces advances its
// DT_PB + 1 searches together with their loads in flight.
constexpr int DT_PB = 8;

__global__ void k_dt_piece_flags(dt_side s, int64_t nh, int cap, const int32_t *__restrict__ hG,
                                 const int64_t *__restrict__ hYS, const int32_t *__restrict__ hB,
                                 const int64_t *__restrict__ P, const int64_t *__restrict__ hpos,
                                 int32_t *__restrict__ cnt, int64_t *__restrict__ pys, int32_t *__restrict__ pb) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nh; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t g = hG[i], xs = s.xrp[g];
        int64_t h0, h1;
        dt_group_span(s, hpos, g, h0, h1);
        const int64_t base = P[h0] + (i - h0), m = h1 - h0, np = P[i + 1] - P[i];
        const int64_t ys = hYS[i], ye = ys + hB[i];
        for (int64_t j0 = 0; j0 < np; j0 += DT_PB) {
            int32_t key[DT_PB + 1];
            int64_t bp[DT_PB + 1];
            bool end[DT_PB + 1];
#pragma unroll
            for (int u = 0; u <= DT_PB; u++) {
                const int64_t j = j0 + u < np ? j0 + u : np;  // j == np: the end of the list
                end[u] = j == np;
                key[u] = end[u] ? INT32_MAX : s.xci[xs + j * cap];
                bp[u] = ys;
            }
            int64_t n = ye - ys;
            while (n > 1) {
                const int64_t half = n >> 1;
#pragma unroll
                for (int q = 0; q <= DT_PB; q++)
                    if (s.yci[bp[q] + half - 1] < key[q]) bp[q] += half;
                n -= half;
            }
            int64_t lb[DT_PB + 1];
#pragma unroll
            for (int q = 0; q <= DT_PB; q++) {
                // bp is the last candidate: the lower bound is bp or bp + 1
                lb[q] = (n == 1 && s.yci[bp[q]] < key[q]) ? bp[q] + 1 : bp[q];
                if (end[q]) lb[q] = ye;
            }
#pragma unroll
            for (int u = 0; u < DT_PB; u++) {
                const int64_t j = j0 + u;
                if (j >= np) break;
                const int64_t lo = lb[u], hi = lb[u + 1] > lo ? lb[u + 1] : lo;
                const int64_t q = base + j * m;
                pys[q] = lo;
                pb[q] = (int32_t)(hi - lo);
                cnt[q] = (int32_t)((hi - lo + cap - 1) / cap);
            }
        }
    }
}

// every pair's sub-entries at its scanned position; ePc[e] = the piece
__global__ void k_dt_piece_compact(dt_side s, int64_t nh, int cap, const int32_t *__restrict__ hG,
                                   const int32_t *__restrict__ hO, const int64_t *__restrict__ hQ,
                                   const int64_t *__restrict__ P, const int64_t *__restrict__ hpos,
                                   const int32_t *__restrict__ cnt, const int64_t *__restrict__ ppos,
                                   const int64_t *__restrict__ pys, const int32_t *__restrict__ pb,
                                   int32_t *__restrict__ eG, int64_t *__restrict__ eYS, int32_t *__restrict__ eO,
                                   int32_t *__restrict__ eB, int64_t *__restrict__ eQ, uint16_t *__restrict__ ePc) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nh; i += (int64_t)gridDim.x * blockDim.x) {
        const int32_t g = hG[i], o = hO[i];
        int64_t h0, h1;
        dt_group_span(s, hpos, g, h0, h1);
        const int64_t base = P[h0] + (i - h0), m = h1 - h0, np = P[i + 1] - P[i];
        const int64_t qq = hQ[i];
        for (int64_t j = 0; j < np; j++) {
            const int64_t q = base + j * m;
            for (int c = 0; c < cnt[q]; c++) {
                const int64_t e = ppos[q] + c;
                const int64_t o0 = (int64_t)c * cap;
                eG[e] = g;
                eYS[e] = pys[q] + o0;
                eO[e] = o;
                eB[e] = (int32_t)(pb[q] - o0 < cap ? pb[q] - o0 : cap);
                eQ[e] = qq;
                ePc[e] = (uint16_t)j;
            }
        }
    }
}

// Y-blocked task order (knob dot_yblk = K > 1): the task entries are stably partitioned by
// which K-th of the Y matrix's entries their Y list starts in, so that at any time the
// workgroups stream Y lists (keys and values) from one K-th of Y -- a working set the
// Infinity Cache / L2 can hold -- instead of from all of it.  X lists are reloaded once
// per block they have entries in.
__global__ void k_dt_ykey(int64_t ne, int K, int64_t ytot, const int64_t *__restrict__ eYS, int32_t *__restrict__ key,
                          int64_t *__restrict__ idx) {
    for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < ne; e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t b = ytot > 0 ? (int64_t)(((__int128)eYS[e] * K) / ytot) : 0;
        key[e] = (int32_t)(b < K ? b : K - 1);
        idx[e] = e;
    }
}

template <class T>
__global__ void k_dt_gather(int64_t ne, const int64_t *__restrict__ idx, const T *__restrict__ src, T *__restrict__ dst) {
    for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < ne; e += (int64_t)gridDim.x * blockDim.x)
        dst[e] = src[idx[e]];
}

// huge entries left to the per-entry kernel: G-order flags -> CSR-order flags
__global__ void k_dt_huge_to_csr(int64_t nm, const uint8_t *__restrict__ hg, const int64_t *__restrict__ perm,
                                 uint8_t *__restrict__ hflag) {
    for (int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; p < nm; p += (int64_t)gridDim.x * blockDim.x)
        if (hg[p]) hflag[perm ? perm[p] : p] = 1;
}

// the huge entries' outputs start at the monoid identity (pieces fold into them)
template <class Z>
__global__ void k_dt_ident(int64_t nh, const int64_t *__restrict__ hQ, Z *__restrict__ tval, Z ident) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nh; i += (int64_t)gridDim.x * blockDim.x)
        tval[hQ[i]] = ident;
}

// a task starts where the group changes or the cost prefix enters a new window
__global__ void k_dt_task_flags(int64_t ne, int64_t win, const int32_t *__restrict__ eG,
                                const uint16_t *__restrict__ ePc, const int64_t *__restrict__ cum,
                                uint8_t *__restrict__ ts) {
    for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < ne; e += (int64_t)gridDim.x * blockDim.x)
        ts[e] = (e == 0 || eG[e] != eG[e - 1] || (ePc && ePc[e] != ePc[e - 1]) || cum[e] / win != cum[e - 1] / win)
                    ? 1 : 0;
}

__global__ void k_dt_task_fill(int64_t ne, const uint8_t *__restrict__ ts, const int64_t *__restrict__ tpos,
                               int64_t *__restrict__ tstart) {
    for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < ne; e += (int64_t)gridDim.x * blockDim.x)
        if (ts[e]) tstart[tpos[e]] = e;
    if (blockIdx.x == 0 && threadIdx.x == 0) tstart[tpos[ne]] = ne;
}

// one task's descriptor, built before the task kernel (k_dt_task_desc) so that a workgroup
// starting a task issues one load instead of the tstart -> eG -> row-pointer chain of
// dependent loads (round 5)
struct dt_task {
    int64_t e0;     // first entry (task order)
    int64_t xs;     // X(g,:)'s (piece's) first key
    int32_t ne;     // entries
    int32_t g;      // group
    int32_t a;      // X keys (of the piece)
    int32_t piece;  // -1, or the piece of a list longer than the cap
};

__global__ void k_dt_task_desc(int64_t nt, const int64_t *__restrict__ tstart, const int32_t *__restrict__ eG,
                               const uint16_t *__restrict__ ePc, const int64_t *__restrict__ xrp, int pcap,
                               dt_task *__restrict__ td) {
    for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < nt; t += (int64_t)gridDim.x * blockDim.x) {
        const int64_t e0 = tstart[t];
        const int32_t g = eG[e0];
        const int piece = ePc ? (int)ePc[e0] : -1;
        int64_t xs = xrp[g], alen = xrp[g + 1] - xs;
        if (piece >= 0) {
            xs += (int64_t)piece * pcap;
            alen -= (int64_t)piece * pcap;
            if (alen > pcap) alen = pcap;
        }
        dt_task d;
        d.e0 = e0;
        d.xs = xs;
        d.ne = (int32_t)(tstart[t + 1] - e0);
        d.g = g;
        d.a = (int32_t)alen;
        d.piece = piece;
        td[t] = d;
    }
}

__global__ void k_dt_positions(int64_t n, const uint8_t *__restrict__ flag, const int64_t *__restrict__ pos,
                               int64_t *__restrict__ out) {
    for (int64_t q = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; q < n; q += (int64_t)gridDim.x * blockDim.x)
        if (flag[q]) out[pos[q]] = q;
}

// ---------------------------------------------------------------- folds
// fold z into a 64-bit LDS slot holding a Z (monoid with identity; exact, so any
// arrival order gives the same result)
template <class SR, class Z>
__device__ __forceinline__ void dt_lds_fold(const SR &sr, unsigned long long *slot, Z z) {
    if constexpr (std::is_same<SR, gb_sr_min_plus<int64_t>>::value) {
        atomicMin((long long *)slot, (long long)z);
    } else if constexpr (std::is_same<SR, gb_sr_plus_times<int64_t>>::value) {
        atomicAdd(slot, (unsigned long long)z);
    } else {
        unsigned long long old = *(volatile unsigned long long *)slot;
        while (true) {
            Z cur;
            __builtin_memcpy(&cur, &old, sizeof(Z));
            const Z nv = sr.add(cur, z);
            unsigned long long nb = old;
            __builtin_memcpy(&nb, &nv, sizeof(Z));
            if (nb == old) return;
            const unsigned long long prev = atomicCAS(slot, old, nb);
            if (prev == old) return;
            old = prev;
        }
    }
}

// fold z into an LDS slot; ANY stores (any term is the result)
template <class SR, class Z>
__device__ __forceinline__ void dt_slot_fold(const SR &sr, bool any_store, unsigned long long *slot, Z z) {
    if (any_store) {
        unsigned long long v = 0;
        __builtin_memcpy(&v, &z, sizeof(Z));
        *slot = v;
    } else {
        dt_lds_fold(sr, slot, z);
    }
}

extern "C" __device__ __attribute__((const)) long long __ockl_wfred_min_i64(long long);
extern "C" __device__ __attribute__((const)) long long __ockl_wfred_add_i64(long long);

// wave fold of (found, acc) into every lane (butterfly; exact monoids).  Callers reach it only when
// some lane found a term.  Integer MIN and PLUS monoids use the device library's wavefront reduction
// (DPP row operations, no LDS traffic) over the lanes' terms with the monoid's identity in the lanes
// that found none (round 6): the butterfly's 6 steps x 3 ds_bpermute (a flag and two 32-bit halves)
// were most of k_dot_small's LDS instructions
template <class SR, class Z>
__device__ __forceinline__ void dt_wave_fold(const SR &sr, bool &found, Z &acc) {
    if constexpr (std::is_same<SR, gb_sr_min_plus<int64_t>>::value) {
        acc = (Z)__ockl_wfred_min_i64(found ? (long long)acc : LLONG_MAX);
        found = true;
        return;
    } else if constexpr (std::is_same<SR, gb_sr_min_plus<int32_t>>::value) {
        acc = (Z)__ockl_wfred_min_i32(found ? (int)acc : INT_MAX);
        found = true;
        return;
    } else if constexpr (std::is_same<SR, gb_sr_plus_times<int64_t>>::value) {
        acc = (Z)__ockl_wfred_add_i64(found ? (long long)acc : 0LL);
        found = true;
        return;
    } else if constexpr (std::is_same<SR, gb_sr_plus_times<int32_t>>::value) {
        acc = (Z)__ockl_wfred_add_i32(found ? (int)acc : 0);
        found = true;
        return;
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        const bool of = __shfl_xor((int)found, off, 64);
        const Z oz = gb_shfl_xor(acc, off, 64);
        if (of) {
            acc = found ? sr.add(acc, oz) : oz;
            found = true;
        }
    }
}

template <class SR, class X, class Z, bool SWAP>
__device__ __forceinline__ Z dt_mult(const SR &sr, X xv, X yv, int64_t g, int32_t k, int64_t o) {
    // R: x = A'(i,k), y = B'(k,j), i = g, j = o;  C: x = B'(k,j), y = A'(i,k), i = o, j = g
    if constexpr (SWAP) return sr.mult(yv, xv, o, k, g);
    else return sr.mult(xv, yv, g, k, o);
}

// ---------------------------------------------------------------- small groups
// a wave per group with 1 <= |X(g,:)| <= 64*KPL: lane l holds X's keys
// [l*KPL, l*KPL + KPL) (and, for KPL = 1, its value); the group's entries are read
// 64 at a time (other index, Y bounds) and taken one after the other: lanes load
// Y's keys 64 at a time (|Y| <= |X|) and find each among X's keys by shuffles --
// 6 steps over the lanes' first keys, then the KPL keys of the lane found.
// position of key yk among the wave's X keys (lane l holds X[l*KPL, l*KPL + KPL)), or -1
template <int KPL>
__device__ __forceinline__ int dt_small_find(const int32_t (&xk)[KPL], int32_t yk, bool act) {
    int pos = -1;
    if constexpr (KPL == 1) {
        int lo = 0;
#pragma unroll
        for (int st = 32; st > 0; st >>= 1)
            if (__shfl(xk[0], lo + st - 1, 64) < yk) lo += st;
        // every lane takes part in the shuffle (a lane outside |Y| still serves its key)
        const int32_t xl = __shfl(xk[0], lo, 64);
        if (act && xl == yk) pos = lo;
    } else {
        int L = 0;  // last lane whose first key <= yk
#pragma unroll
        for (int st = 32; st > 0; st >>= 1) {
            const int c = L + st;
            const int32_t v = __shfl(xk[0], c < 64 ? c : 63, 64);
            if (c < 64 && v <= yk) L = c;
        }
#pragma unroll
        for (int j = 0; j < KPL; j++) {
            const int32_t v = __shfl(xk[j], L, 64);
            if (act && v == yk) pos = L * KPL + j;
        }
    }
    return pos;
}



// Flat entries (round 6, the default): a batch's entries' Y lists are one flat run of keys, 64 per
// lane-step and DT_FU steps at a time -- a lane finds its element's entry by a shuffle search over
// the entries' prefix -- so short Y lists no longer leave most of a wave idle; a hit (a few % of
// the keys in these classes) folds into its entry's LDS slot by an atomic, so there is no
// segmented scan (round 6: it replaced a loop taking four entries at a time, each a whole 64-lane
// pass).  seq 1: one entry at a time (A/B).
constexpr int DT_FU = 2;  // steps of 64 keys in flight (4: 96 VGPRs; 2 measured 4 % faster at s20)

template <class SR, class X, class Z, bool SWAP, int KPL>
__global__ __launch_bounds__(DT_BLOCK) void k_dot_small(SR sr, int mon, dt_side s, dt_vals<X> xvx, dt_vals<X> yvx,
                                                       Z *__restrict__ tval, uint8_t *__restrict__ tflag, int seq) {
    const int lane = threadIdx.x & 63;
    const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
    const bool rv = SR::reads_values && xvx.v && yvx.v;
    constexpr int AMIN = KPL == 1 ? 1 : DT_SMALL + 1;
    __shared__ unsigned long long f_slot[DT_BLOCK / 64][64];
    __shared__ unsigned long long f_found[DT_BLOCK / 64];
    unsigned long long *fslot = f_slot[threadIdx.x >> 6];
    unsigned long long *ffound = &f_found[threadIdx.x >> 6];
    const bool ANY = std::is_same<SR, gb_sr_any_pair<Z>>::value || mon == GBAMD_MON_ANY;
    const Z ident = ANY ? Z() : gb_monoid_identity<Z>(mon);
    unsigned long long identb = 0;
    __builtin_memcpy(&identb, &ident, sizeof(Z));
    for (int64_t g = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6; g < s.ng; g += nw) {
        const int64_t xs = s.xrp[g];
        const int a = __builtin_amdgcn_readfirstlane((int)(s.xrp[g + 1] - xs));
        const int64_t p0 = s.grp_rp[g], p1 = s.grp_rp[g + 1];
        const int cnt_e = __builtin_amdgcn_readfirstlane((int)(p1 - p0));
        if (a < AMIN || a > 64 * KPL || cnt_e == 0) continue;  // before any cross-lane operation
        int32_t xk[KPL];
#pragma unroll
        for (int j = 0; j < KPL; j++) xk[j] = lane * KPL + j < a ? s.xci[xs + lane * KPL + j] : 0x7fffffff;
        // X's values: read on a hit from the row just loaded (an L2 hit); round 4 held them in
        // registers beside the keys and shuffled KPL of them (two 32-bit shuffles each for 8-byte
        // values) for every 64 Y keys -- the kernel is bound by its shuffles, not by these loads
        // flat entries for both classes (X of 1..64 and 65..256 keys; 64 / 72 VGPRs)
        if (!seq) {
            for (int64_t pb = p0; pb < p1; pb += 64) {
                const int nb = __builtin_amdgcn_readfirstlane((int)std::min<int64_t>(64, p1 - pb));
                int32_t o_l = 0;
                int64_t ys_l = 0;
                int b_l = 0;
                if (lane < nb) {
                    o_l = s.grp_oi[pb + lane];
                    ys_l = s.yrp[o_l];
                    b_l = (int)(s.yrp[o_l + 1] - ys_l);
                }
                const int bl = (lane < nb && b_l > 0 && dt_side_of<SWAP>(a, b_l)) ? b_l : 0;
                int inc = bl;
#pragma unroll
                for (int off = 1; off < 64; off <<= 1) {
                    const int y = __shfl_up(inc, off, 64);
                    if (lane >= off) inc += y;
                }
                const int T = __builtin_amdgcn_readlane(inc, 63);
                if (T == 0) continue;  // wave-uniform
                const int64_t yoff_l = ys_l - (inc - bl);  // entry e's flat element f sits at Y position yoff_e + f
                fslot[lane] = identb;
                if (lane == 0) *ffound = 0ULL;
                gb_wave_sync();
                for (int f0 = 0; f0 < T; f0 += 64 * DT_FU) {
                    int ee[DT_FU];
                    int64_t py[DT_FU];
                    int32_t yk[DT_FU];
#pragma unroll
                    for (int u = 0; u < DT_FU; u++) {
                        const int f = f0 + u * 64 + lane;
                        int lo = 0;  // the first entry whose inclusive prefix exceeds f
#pragma unroll
                        for (int st = 32; st > 0; st >>= 1)
                            if (__shfl(inc, lo + st - 1, 64) <= f) lo += st;
                        ee[u] = lo;
                        py[u] = gb_shfl(yoff_l, lo < 64 ? lo : 63) + f;
                        yk[u] = f < T ? s.yci[py[u]] : -1;
                    }
                    int pos[DT_FU];
#pragma unroll
                    for (int u = 0; u < DT_FU; u++) pos[u] = dt_small_find<KPL>(xk, yk[u], f0 + u * 64 + lane < T);
#pragma unroll
                    for (int u = 0; u < DT_FU; u++) {
                        const int32_t o = __shfl(o_l, ee[u] < 64 ? ee[u] : 63, 64);  // every lane shuffles
                        if (pos[u] >= 0) {
                            X xm = X(), yv = X();
                            if (rv) {
                                xm = xvx[xs + pos[u]];
                                yv = yvx[py[u]];
                            }
                            const Z z = dt_mult<SR, X, Z, SWAP>(sr, xm, yv, g, yk[u], o);
                            dt_slot_fold(sr, ANY, &fslot[ee[u]], z);
                            atomicOr(ffound, 1ULL << ee[u]);
                        }
                    }
                }
                gb_wave_sync();
                if (lane < nb && ((*ffound >> lane) & 1ULL)) {
                    const int64_t p = pb + lane;
                    const int64_t q = s.perm ? s.perm[p] : p;
                    Z v;
                    const unsigned long long raw = fslot[lane];
                    __builtin_memcpy(&v, &raw, sizeof(Z));
                    tval[q] = v;
                    tflag[q] = 1;
                }
                gb_wave_sync();  // the slots are rewritten by the next batch
            }
            continue;
        }
        for (int64_t pb = p0; pb < p1; pb += 64) {
            const int nb = __builtin_amdgcn_readfirstlane((int)std::min<int64_t>(64, p1 - pb));
            int32_t o_l = 0;
            int64_t ys_l = 0;
            int b_l = 0;
            if (lane < nb) {
                o_l = s.grp_oi[pb + lane];
                ys_l = s.yrp[o_l];
                b_l = (int)(s.yrp[o_l + 1] - ys_l);
            }
            for (int t = 0; t < nb; t++) {
                // (no `continue` in this loop: its body holds cross-lane operations)
                const int b = __builtin_amdgcn_readlane(b_l, t);
                if (b > 0 && dt_side_of<SWAP>(a, b)) {
                    const int32_t o = __builtin_amdgcn_readlane(o_l, t);
                    const int64_t ys = gb_shfl(ys_l, t);
                    bool found = false;
                    Z acc = Z();
                    for (int f0 = 0; f0 < b; f0 += 64) {
                        const bool act = f0 + lane < b;
                        const int32_t yk = act ? s.yci[ys + f0 + lane] : -1;
                        int pos = -1;
                        X xm = X();
                        if constexpr (KPL == 1) {
                            int lo = 0;
#pragma unroll
                            for (int st = 32; st > 0; st >>= 1)
                                if (__shfl(xk[0], lo + st - 1, 64) < yk) lo += st;
                            // every lane takes part in the shuffle (a lane outside |Y| still serves its key)
                            const int32_t xl = __shfl(xk[0], lo, 64);
                            if (act && xl == yk) pos = lo;
                        } else {
                            int L = 0;  // last lane whose first key <= yk
#pragma unroll
                            for (int st = 32; st > 0; st >>= 1) {
                                const int c = L + st;
                                const int32_t v = __shfl(xk[0], c < 64 ? c : 63, 64);
                                if (c < 64 && v <= yk) L = c;
                            }
#pragma unroll
                            for (int j = 0; j < KPL; j++) {
                                const int32_t v = __shfl(xk[j], L, 64);
                                if (act && v == yk) pos = L * KPL + j;
                            }
                        }
                        if (pos >= 0) {
                            X yv = X();
                            if (rv) {
                                xm = xvx[xs + pos];
                                yv = yvx[ys + f0 + lane];
                            }
                            const Z z = dt_mult<SR, X, Z, SWAP>(sr, xm, yv, g, yk, o);
                            acc = found ? sr.add(acc, z) : z;
                            found = true;
                        }
                    }
                    if (__ballot(found)) {
                        dt_wave_fold(sr, found, acc);
                        if (lane == 0) {
                            const int64_t p = pb + t;
                            const int64_t q = s.perm ? s.perm[p] : p;
                            tval[q] = acc;
                            tflag[q] = 1;
                        }
                    }
                }
            }
        }
    }
}

// ---------------------------------------------------------------- task groups
// A workgroup per task (a run of <= DT_MAXE entries of one group g with
// 256 < |X(g,:)| <= DT_CAP); the entries' other index, Y bounds and output slot
// come precomputed in task order (k_dt_compact).
//  1. X(g,:)'s keys go to LDS as they are (sorted) plus a hashed membership filter
//     (2^18 bits, <= 6.25 % set): one LDS read rejects most Y keys.
//  2. The entries' Y lists form one flat element space (prefix e_pre), cut into
//     units of DT_PIECE elements that waves take from an LDS counter -- a unit may
//     hold many short entries, so every wave keeps DT_U * 64 loads in flight
//     whatever the entries' lengths.  A lane finds its element's entry from a
//     bitmap of entry starts over the flat space (one 64-bit word per 64 elements,
//     a popcount), loads the Y key (coalesced), filters it, and packs the keys that
//     pass (~hits + 6 %) densely into a per-wave LDS stage; the stage is binary-
//     searched in X's keys with every lane busy.  Hits fold in registers per lane
//     (a lane's staged elements come in entry order) and meet per entry in LDS
//     slots (atomic fold of an exact monoid, one per lane run -- one per wave when
//     the wave's hits share an entry), written to T at the end of the task.
constexpr int DT_TB = 1024;      // task workgroup: 16 waves, two workgroups per CU (74.8 KB LDS, <= 64 VGPRs)
constexpr int DT_U = 4;          // 64-element windows per step (loads in flight per lane)
constexpr int DT_PIECE = 1024;   // elements per unit (a multiple of 64 * DT_U)
constexpr int DT_SMAX = DT_WIN + DT_CAP;  // flat elements per task bound
constexpr int DT_FLOG = 17;      // filter bits (log2)

__device__ __forceinline__ uint32_t dt_hash(int32_t k) { return ((uint32_t)k * 0x9E3779B1u) >> (32 - DT_FLOG); }

// X's keys sit in LDS in Eytzinger (breadth-first) order of a perfect search tree of h levels,
// 1-based, padded with INT32_MAX (round 6): a lower-bound search is h steps of `j = 2 j + (keys[j] <
// key)` -- one LDS read, a compare and a shift-add, against ~10 VALU per step for the round-5
// sorted array with bank-skewed slots (index arithmetic, bounds test, select) -- and its first
// levels are the same few words for every lane (broadcast reads).  Sorted index i of a tree of h
// levels sits at node 2^d + ((i + 1) >> (t + 1)), t = ctz(i + 1), d = h - 1 - t; node k holds
// sorted index ((2 (k - 2^d) + 1) << (h - 1 - d)) - 1, d = floor(log2 k).
constexpr int DT_KSLOTS = 8192;  // nodes 1 .. 2^13 - 1
__device__ __forceinline__ int dt_eytz(int i, int h) {
    const int t = __builtin_ctz(i + 1);
    return (1 << (h - 1 - t)) + ((i + 1) >> (t + 1));
}
__device__ __forceinline__ int dt_inorder(int k, int h) {
    const int d = 31 - __builtin_clz(k);
    return ((2 * (k - (1 << d)) + 1) << (h - 1 - d)) - 1;
}

// fold z into T's 4- or 8-byte output slot (pieces of one entry meet here; exact monoids)
template <class SR, class Z>
__device__ __forceinline__ void dt_global_fold(const SR &sr, bool any_store, Z *slot, Z z) {
    if (any_store) {
        *slot = z;
    } else if constexpr (std::is_same<SR, gb_sr_min_plus<int64_t>>::value) {
        atomicMin((long long *)slot, (long long)z);
    } else if constexpr (sizeof(Z) == 8) {
        unsigned long long *w = (unsigned long long *)slot;
        unsigned long long old = *(volatile unsigned long long *)w;
        while (true) {
            Z cur;
            __builtin_memcpy(&cur, &old, 8);
            const Z nv = sr.add(cur, z);
            unsigned long long nb;
            __builtin_memcpy(&nb, &nv, 8);
            if (nb == old) return;
            const unsigned long long prev = atomicCAS(w, old, nb);
            if (prev == old) return;
            old = prev;
        }
    } else if constexpr (sizeof(Z) == 4) {
        unsigned int *w = (unsigned int *)slot;
        unsigned int old = *(volatile unsigned int *)w;
        while (true) {
            Z cur;
            __builtin_memcpy(&cur, &old, 4);
            const Z nv = sr.add(cur, z);
            unsigned int nb;
            __builtin_memcpy(&nb, &nv, 4);
            if (nb == old) return;
            const unsigned int prev = atomicCAS(w, old, nb);
            if (prev == old) return;
            old = prev;
        }
    }
}


template <class SR, class X, class Z, bool SWAP>
// 8 waves per SIMD: two workgroups per CU (round 3: one workgroup of 149.6 KB LDS and 78 VGPRs
// per CU left the latency-bound stream at 4 waves per SIMD; s22 128 -> 117 ms, s20 27.2 -> 23.5)
__global__ __launch_bounds__(DT_TB, 8) void k_dot_task(
    SR sr, int mon, dt_side s, dt_vals<X> xvx, dt_vals<X> yvx, int64_t ntask, const dt_task *__restrict__ tdesc, const int32_t *__restrict__ eG,
    const int64_t *__restrict__ eYS, const int32_t *__restrict__ eO, const int32_t *__restrict__ eB,
    const int64_t *__restrict__ eQ, Z *__restrict__ tval, uint8_t *__restrict__ tflag, int dbg,
    const uint16_t *__restrict__ ePc, int pcap, unsigned long long *__restrict__ tctr, int chunk, int fratio) {
    __shared__ int32_t keys[DT_KSLOTS];  // X's keys, Eytzinger order (dt_eytz)
    __shared__ uint32_t filt[1 << (DT_FLOG - 5)];
    __shared__ uint64_t estart[DT_SMAX / 64 + 1];     // bit f: an entry starts at flat element f
    // X's values when they are one-byte narrow copies (round 6): a hit reads its X value from LDS
    // instead of global memory (the round-4 staged-survivor diagnostics path held this LDS)
    __shared__ uint8_t xv8[DT_KSLOTS];
    __shared__ int64_t e_off[DT_MAXE];  // entry e's flat element f sits at Y position e_off[e] + f
    __shared__ int32_t e_pre[DT_MAXE + 1];
    __shared__ unsigned long long e_acc[DT_MAXE];
    __shared__ uint32_t e_fnd[DT_MAXE / 32];  // bit e: entry e found a match (the output slot and
                                              // other index stay in global memory: LDS holds 512 entries)
    __shared__ int w_sum[DT_TB / 64];
    __shared__ int next_unit;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const bool rv = SR::reads_values && xvx.v && yvx.v;
    // one-byte narrow X values go to LDS with the keys (knob dot_xlds = 1: off, A/B)
    bool xl8 = false;
    if constexpr (std::is_integral<X>::value && !std::is_same<X, bool>::value && sizeof(X) > 1)
        xl8 = rv && !xvx.iso && xvx.nv && (xvx.nk == 1 || xvx.nk == -1) && !(dbg & 4096);
    // one-byte narrow Y values streamed with the keys, packed in the key's top byte when the keys
    // are below 2^24 (knob dot_ypack = 1: off), so a hit loads nothing from global memory
    bool yp8 = false;
    if constexpr (std::is_integral<X>::value && !std::is_same<X, bool>::value && sizeof(X) > 1)
        yp8 = rv && !yvx.iso && yvx.nv && (yvx.nk == 1 || yvx.nk == -1) && (dbg & 8192);
    // ANY (any_pair, or LOR over pair's 1s): the entry's value is any term -- store it;
    // every other monoid folds into its identity
    const bool ANY = std::is_same<SR, gb_sr_any_pair<Z>>::value || mon == GBAMD_MON_ANY;
    const Z ident = ANY ? Z() : gb_monoid_identity<Z>(mon);
    const unsigned long long ltmask = (1ULL << lane) - 1;
    // tasks are handed out in chunks of `chunk` consecutive tasks from a grid-wide counter
    // (dynamic: the workgroups stay balanced); consecutive tasks of one group share X(g,:),
    // whose keys and filter then stay in LDS
    __shared__ int64_t s_chunk;
    int64_t prev_g = -1;
    int prev_pc = -1;
    bool fdirty = true;  // the filter holds bits (of the current X when a task reuses it)
    for (;;) {
    if (tid == 0) s_chunk = (int64_t)atomicAdd(tctr, (unsigned long long)chunk);
    __syncthreads();
    const int64_t c0 = s_chunk;
    __syncthreads();  // every thread has read the chunk before it is rewritten
    if (c0 >= ntask) break;
    const int64_t c1 = c0 + chunk < ntask ? c0 + chunk : ntask;
    for (int64_t t = c0; t < c1; t++) {
        // the thread index made opaque per task: otherwise the compiler hoists the per-thread
        // Eytzinger slot arithmetic of every X key out of the task loop and spills it to scratch
        // (38 VGPRs: reloaded from scratch in every task's setup)
        int tv = tid;
        asm volatile("" : "+v"(tv));
        const dt_task td = tdesc[t];  // one load (uniform)
        const int64_t e0 = td.e0;
        const int ne = __builtin_amdgcn_readfirstlane(td.ne);
        const int64_t g = td.g;
        const int piece = td.piece;  // a piece of a list longer than the cap
        const bool reuse = g == prev_g && piece == prev_pc && !(dbg & 64);  // dbg 64: reload X every task (A/B)
        prev_g = g;
        prev_pc = piece;
        const int64_t xs = td.xs;
        const int a = __builtin_amdgcn_readfirstlane(td.a);
        // X loads (stat dot_task_xloads), counted only under the statistics knob and a cache line
        // away from the chunk counter the workgroups claim tasks from
        if ((dbg & 1024) && !reuse && tv == 0) atomicAdd(tctr + 16, 1ULL);
        // the entries' and X's loads issued together, before any LDS work (one round trip)
        int b = 0;
        int64_t ysv = 0;
        if (tv < ne) {
            b = eB[e0 + tv];
            ysv = eYS[e0 + tv];
        }
        constexpr int XPT = (DT_CAP + DT_TB - 1) / DT_TB;  // X keys per thread
        int32_t xk[XPT];
        if (!reuse) {
#pragma unroll
            for (int j = 0; j < XPT; j++) xk[j] = tv + j * DT_TB < a ? s.xci[xs + tv + j * DT_TB] : 0;
            if (xl8) {
                const uint8_t *nv = (const uint8_t *)xvx.nv;
#pragma unroll
                for (int j = 0; j < XPT; j++)
                    if (tv + j * DT_TB < a) xv8[tv + j * DT_TB] = nv[xs + tv + j * DT_TB];
            }
        }
        if (!reuse && fdirty) {  // a filter of another X: cleared (the first task: LDS garbage)
            for (int i = tv; i < (1 << (DT_FLOG - 5)); i += DT_TB) filt[i] = 0;
            fdirty = false;
        }
        for (int i = tv; i < DT_SMAX / 64 + 1; i += DT_TB) estart[i] = 0;
        for (int i = tv; i < DT_MAXE / 32; i += DT_TB) e_fnd[i] = 0;
        if (tv < ne) {
            unsigned long long iv = 0;
            __builtin_memcpy(&iv, &ident, sizeof(Z));
            e_acc[tv] = iv;
        }
        int inc = b;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const int y = __shfl_up(inc, off, 64);
            if (lane >= off) inc += y;
        }
        if (lane == 63) w_sum[wid] = inc;
        if (tv == 0) next_unit = 0;
        __syncthreads();  // filter and start bits cleared, wave sums visible
        int ksteps = 0;  // tree levels: the least h with 2^h - 1 >= a
        while ((1 << ksteps) - 1 < a) ksteps++;
        int base = 0, S = 0;
        for (int w = 0; w < DT_TB / 64; w++) {
            if (w < wid) base += w_sum[w];
            S += w_sum[w];
        }
        S = __builtin_amdgcn_readfirstlane(S);
        // the hashed filter pays when the task streams enough keys past it (round 6, knob
        // dot_filt_ratio: built only when S >= ratio * |X|; 0 = always); kept across tasks of one X
        const bool usef = fratio <= 0 || S >= fratio * a;
        const bool fbuild = usef && !fdirty;
        if (!reuse || fbuild) {
#pragma unroll
            for (int j = 0; j < XPT; j++) {
                const int i = tv + j * DT_TB;
                if (!reuse && i < (1 << ksteps) - 1) keys[dt_eytz(i, ksteps)] = i < a ? xk[j] : INT32_MAX;
                if (fbuild && i < a) {
                    const int32_t kx = reuse ? keys[dt_eytz(i, ksteps)] : xk[j];
                    const uint32_t h = dt_hash(kx);
                    atomicOr(&filt[h >> 5], 1u << (h & 31));
                }
            }
        }
        fdirty = fdirty || fbuild;
        if (tv < ne) {
            const int f = base + inc - b;
            e_pre[tv] = f;
            e_off[tv] = ysv - f;
            if (b > 0) atomicOr((unsigned long long *)&estart[f >> 6], 1ULL << (f & 63));
        }
        if (tv == 0) e_pre[ne] = S;
        __syncthreads();
        int esteps = 0;
        while ((1 << esteps) < ne) esteps++;
        const int NU = (S + DT_PIECE - 1) / DT_PIECE;
        // units (wave-uniform bookkeeping in scalar registers; no `continue` in the
        // loop: its body holds cross-lane operations)
        int unit = 0;
        if (lane == 0) unit = atomicAdd(&next_unit, 1);
        unit = __builtin_amdgcn_readlane(unit, 0);
        while (unit < NU) {
            const int fu0 = unit * DT_PIECE, fu1 = min(S, fu0 + DT_PIECE);
            // entry holding fu0 (last e with e_pre[e] <= fu0; empty entries resolve
            // to the last of equal starts, which the bitmap walk also does)
            int ew = 0;
            for (int st = esteps - 1; st >= 0; st--) {
                const int c = ew + (1 << st);
                if (c < ne && e_pre[c] <= fu0) ew = c;
            }
            ew = __builtin_amdgcn_readfirstlane(ew);
            int cur_e = -1;
            bool found = false;
            Z acc = Z();
            // one step's key loads (DT_U windows of 64 flat elements from fb): the entries
            // starting in each window (all windows' words read at once; the entry before each
            // window follows from the previous words' popcounts, so no window waits on another's
            // cross-lane step), the lanes' entries, then the loads back to back.  Measured
            // neutral against the round-4 per-window chain, and so was issuing the next step's
            // loads before this step's search (software pipelining): 118.5 vs 118.8 ms at s22
            auto issue = [&](int fb, int (&ee_o)[DT_U], int32_t (&k_o)[DT_U]) {
                uint64_t sb[DT_U];
#pragma unroll
                for (int u = 0; u < DT_U; u++) sb[u] = estart[(fb >> 6) + u];
#pragma unroll
                for (int u = 0; u < DT_U; u++) {
                    // a start at the window's first element is counted by the popcount
                    // (ew holds the entry of the element before it)
                    const int ustart = (fb + u * 64 == fu0 && (sb[u] & 1ULL)) ? 1 : 0;  // unit start: ew is it
                    ee_o[u] = ew + __popcll(sb[u] & ((ltmask << 1) | 1ULL)) - ustart;
                    ew = __builtin_amdgcn_readfirstlane(ew + __popcll(sb[u]) - ustart);  // lane 63's entry
                }
                int64_t py[DT_U];
#pragma unroll
                for (int u = 0; u < DT_U; u++) {
                    const int f = fb + u * 64 + lane;
                    const int eL = ee_o[u] < ne ? ee_o[u] : ne - 1;
                    py[u] = f < fu1 ? e_off[eL] + f : 0;  // past the unit: a harmless load
                }
#pragma unroll
                for (int u = 0; u < DT_U; u++) k_o[u] = s.yci[py[u]];
                if (yp8) {  // one-byte Y values ride in the key's top byte (keys < 2^24)
                    const uint8_t *nv = (const uint8_t *)yvx.nv;
                    uint32_t v8[DT_U];
#pragma unroll
                    for (int u = 0; u < DT_U; u++) v8[u] = nv[py[u]];
#pragma unroll
                    for (int u = 0; u < DT_U; u++) k_o[u] = (int32_t)((uint32_t)k_o[u] | (v8[u] << 24));
                }
            };
            // one surviving element (its key passed the filter): binary search in X's keys; a hit
            // loads the two values and folds into the lane's run (a lane's survivors come in
            // element order, hence in entry order)
            auto survivor = [&](bool act, int32_t kp, int f, int e) {
                const int32_t kk = yp8 ? (kp & 0xffffff) : kp;
                int jn = 1;  // Eytzinger descent; the lower bound is the last node where it went left
                for (int st = 0; st < ksteps; st++) jn = 2 * jn + (keys[jn] < kk ? 1 : 0);
                const int kn = jn >> __builtin_ffs(~jn);  // 0: every key is < kk
                if (act && !(dbg & 1) && kn && keys[kn] == kk) {
                    const int l = dt_inorder(kn, ksteps);  // X's position of the key
                    X xv = X(), yv = X();
                    if (rv) {
                        if (xl8) xv = xvx.nk == 1 ? (X)xv8[l] : (X)(int8_t)xv8[l];
                        else xv = xvx[xs + l];
                        if (yp8) yv = yvx.nk == 1 ? (X)((uint32_t)kp >> 24) : (X)(int8_t)((uint32_t)kp >> 24);
                        else yv = yvx[e_off[e] + f];
                    }
                    const Z z = dt_mult<SR, X, Z, SWAP>(sr, xv, yv, g, kk, eO[e0 + e]);
                    if (e != cur_e) {
                        if (found) {
                            dt_slot_fold(sr, ANY, &e_acc[cur_e], acc);
                            atomicOr(&e_fnd[cur_e >> 5], 1u << (cur_e & 31));
                        }
                        cur_e = e;
                        found = false;
                    }
                    acc = found ? sr.add(acc, z) : z;
                    found = true;
                }
            };
            {
                // Survivors are compacted in registers: each window's passing keys and their
                // (element | entry << 17) words are forward-permuted (ds_permute, no LDS storage)
                // into lanes [pc, pc + n) of a 64-lane batch -- the other lanes' values go to the
                // complement, a permutation -- and a batch is searched only when full or at the
                // unit's end.  Round 4 staged them in LDS and loaded each key again from global
                // memory before its search, one partly filled round per step.  The step's filter
                // words are read together (all DT_U reads in flight).
                int32_t pk = -1;  // the batch: key and element|entry word per lane
                int pm = 0, pc = 0;
                for (int f0 = fu0; f0 < ((dbg & 8) ? fu0 : fu1); f0 += 64 * DT_U) {
                    int32_t k[DT_U];
                    int ee[DT_U];
                    issue(f0, ee, k);
                    uint32_t hh[DT_U], fw[DT_U];
#pragma unroll
                    for (int u = 0; u < DT_U; u++)
                        hh[u] = dt_hash((dbg & 4) ? f0 + u * 64 + lane : (yp8 ? (k[u] & 0xffffff) : k[u]));
#pragma unroll
                    for (int u = 0; u < DT_U; u++) fw[u] = usef ? filt[hh[u] >> 5] : ~0u;
#pragma unroll
                    for (int u = 0; u < DT_U; u++) {
                        const int f = f0 + u * 64 + lane;
                        const bool c = !(dbg & 2) && f < fu1 && ((fw[u] >> (hh[u] & 31)) & 1u);
                        const unsigned long long m = __ballot(c);
                        const int n = __popcll(m);
                        if (n) {
                            if (pc + n > 64) {  // batch full: search it first
                                survivor(lane < pc, pk, pm & 0x1ffff, pm >> 17);
                                pc = 0;
                            }
                            const int sr_ = __popcll(m & ltmask);
                            const int dst = c ? pc + sr_ : (pc + n + (lane - sr_)) & 63;
                            const int nk = __builtin_amdgcn_ds_permute(dst << 2, k[u]);
                            const int nm = __builtin_amdgcn_ds_permute(dst << 2, f | (ee[u] << 17));
                            if (lane >= pc && lane < pc + n) {
                                pk = nk;
                                pm = nm;
                            }
                            pc += n;
                        }
                    }
                }
                if (pc) survivor(lane < pc, pk, pm & 0x1ffff, pm >> 17);
            }
            // end of the unit: one fold per wave when every lane's run is one entry
            const unsigned long long fb = __ballot(found);
            if (fb) {
                const int e_first = __builtin_amdgcn_readlane(cur_e, __builtin_ctzll(fb));
                if (!__ballot(found && cur_e != e_first)) {
                    dt_wave_fold(sr, found, acc);
                    if (lane == 0) {
                        dt_slot_fold(sr, ANY, &e_acc[e_first], acc);
                        atomicOr(&e_fnd[e_first >> 5], 1u << (e_first & 31));
                    }
                } else if (found) {
                    dt_slot_fold(sr, ANY, &e_acc[cur_e], acc);
                    atomicOr(&e_fnd[cur_e >> 5], 1u << (cur_e & 31));
                }
            }
            int nxt = 0;
            if (lane == 0) nxt = atomicAdd(&next_unit, 1);
            unit = __builtin_amdgcn_readlane(nxt, 0);
        }
        __syncthreads();
        if (tv < ne && ((e_fnd[tv >> 5] >> (tv & 31)) & 1u)) {
            const int64_t q = eQ[e0 + tv];
            Z v;
            const unsigned long long raw = e_acc[tv];
            __builtin_memcpy(&v, &raw, sizeof(Z));
            if (piece >= 0) dt_global_fold(sr, ANY, &tval[q], v);
            else tval[q] = v;
            tflag[q] = 1;
        }
        __syncthreads();
    }
    }
}

}  // namespace

// C-ABI-free internal entry (gb_mxm.hip): the two phases over one mask; tval / tflag
// are indexed by the mask's CSR positions (tflag pre-zeroed by the caller).  Returns
// the CSR positions of the entries left to the per-entry kernel (longer list >
// DT_CAP) in *huge (device, caller frees) and their count.
int64_t gb_dot_two_sided(const gb_csr_view &A, const gb_csr_view &BT, gb_mmask &mask, const gb_sr_info &info,
                         const void *av, const void *btv, void *tval, uint8_t *tflag, int64_t **huge) {
    const int64_t nm = mask.nvals;
    *huge = nullptr;
    if (nm == 0) return 0;
    const int64_t nkey = std::max(A.ncols, BT.ncols);  // the inner dimension: the lists' keys are below it
    gb_scratch s;
    // the mask's CSC with each entry's CSR position: cached on the mask matrix, or built
    const int64_t *mtrp, *mperm;
    const int32_t *mtci;
    int64_t *own_rp = nullptr, *own_perm = nullptr;
    int32_t *own_ci = nullptr;
    void *own_vx = nullptr;
    if (mask.obj) {
        gb_csr_view mt;
        gb_get_csc(mt, mask.obj);
        mtrp = mt.rowptr;
        mtci = mt.colidx;
        mperm = gb_csc_perm(mask.obj);
    } else {
        gb_transpose_csr(A.nrows, BT.nrows, nm, mask.rowptr, mask.colidx, nullptr, 1, false, &own_rp, &own_ci, &own_vx,
                         &own_perm);
        mtrp = own_rp;
        mtci = own_ci;
        mperm = own_perm;
    }
    // knobs dot_cap / dot_win (tests) shrink the LDS list cap and the task window
    int cap = DT_CAP;
    int64_t win = DT_WIN;
    if (gb_knob("dot_cap") > DT_MID && gb_knob("dot_cap") < DT_CAP) cap = (int)gb_knob("dot_cap");
    // per-entry cost of the task cut (knob dot_ovh, >= DT_OVH_MIN): at most win / ovh entries per task
    // tools/spgemm_probe.py (R-MAT, one box each): ovh 256 -> 128 (up to 256 entries per task, so
    // fewer tasks, X loads and filter builds): s22 118.7 -> 111.3 ms, s20 24.1 -> 23.2 ms; with the
    // entry arrays trimmed to fit 512 entries, 128 / 96 / 64: s22 106.2 / 104.2 / 101.7 ms,
    // s20 21.7 / 21.2 / 20.7 ms
    int64_t ovh = DT_OVH;
    if (gb_knob("dot_ovh") >= DT_OVH_MIN) ovh = gb_knob("dot_ovh");
    if (gb_knob("dot_win") >= ovh && gb_knob("dot_win") < DT_WIN) win = gb_knob("dot_win");
    uint8_t *hflag = s.get<uint8_t>(nm);
    gb_memset(hflag, 0, nm);
    uint8_t *tf = s.get<uint8_t>(nm);
    uint8_t *hg = s.get<uint8_t>(nm);
    int64_t *pos = s.get<int64_t>(nm + 1);
    gb_dispatch_sr(info, [&](auto srf, auto x, auto z) {
        using SRT = decltype(srf);
        using X = decltype(x);
        using Z = decltype(z);
        auto phase = [&](auto swapc) {
            constexpr bool SWAP = decltype(swapc)::value;
            dt_side sd;
            if (!SWAP) {
                sd = dt_side{mask.rowptr, mask.colidx, nullptr, A.nrows, A.rowptr, A.colidx, BT.rowptr, BT.colidx};
            } else {
                sd = dt_side{mtrp, mtci, mperm, BT.nrows, BT.rowptr, BT.colidx, A.rowptr, A.colidx};
            }
            // narrow copies apply when the kernels read the matrices' own values (no cast copy)
            const dt_vals<X> va{(const X *)av, av == A.vals ? A.nvx : nullptr, av == A.vals ? A.nvk : 0, A.iso};
            const dt_vals<X> vb{(const X *)btv, btv == BT.vals ? BT.nvx : nullptr, btv == BT.vals ? BT.nvk : 0,
                                BT.iso};
            const dt_vals<X> xv = SWAP ? vb : va, yv = SWAP ? va : vb;
            if (!SWAP && SRT::reads_values && (va.nk || vb.nk)) gb_stat_add("dot_narrow_calls", 1);
            const unsigned gw = dt_grid(sd.ng * 64, DT_BLOCK, 1 << 15);
            // 1: one entry at a time (the round-5 loop, A/B)
            const int sseq = gb_knob("dot_small_seq") == 1 ? 1 : 0;
            hipLaunchKernelGGL((k_dot_small<SRT, X, Z, SWAP, 1>), dim3(gw), dim3(DT_BLOCK), 0, gb_stream(), srf,
                               info.mon, sd, xv, yv, (Z *)tval, tflag, sseq);
            const int64_t skip = gb_knob("dot_skip");  // diagnostics: 1 skips the mid kernel, 2 the task kernel
            if (!(skip & 1))
                hipLaunchKernelGGL((k_dot_small<SRT, X, Z, SWAP, DT_MID / 64>), dim3(gw), dim3(DT_BLOCK), 0,
                                   gb_stream(), srf, info.mon, sd, xv, yv, (Z *)tval, tflag, sseq);
            // lists longer than the cap run as pieces of cap keys (4- and 8-byte results:
            // the pieces of an entry fold into its output slot with atomics)
            const bool pieces = (sizeof(Z) == 4 || sizeof(Z) == 8) && gb_knob("dot_pieces") != 1;
            gb_memset(tf, 0, nm);
            if (pieces) gb_memset(hg, 0, nm);
            // hub groups in chunks (knob dot_hubchunk = 1: a wave per hub group, as in round 4)
            const bool hubc = gb_knob("dot_hubchunk") != 1;
            hipLaunchKernelGGL((k_dt_classify<SWAP>), dim3(gw), dim3(DT_BLOCK), 0, gb_stream(), sd, cap, tf, hflag,
                               pieces ? hg : nullptr, hubc);
            GB_LAUNCH_CHECK();
            gb_scratch hcs;
            int64_t *hcp = nullptr, nhch = 0;
            unsigned long long *amax = hcs.get<unsigned long long>(1);
            gb_memset(amax, 0, sizeof(unsigned long long));
            if (hubc) {
                int32_t *nch = hcs.get<int32_t>(sd.ng);
                hcp = hcs.get<int64_t>(sd.ng + 1);
                hipLaunchKernelGGL(k_dt_hub_count, dim3(dt_grid(sd.ng)), dim3(DT_BLOCK), 0, gb_stream(), sd, cap, nch,
                                   amax);
                GB_LAUNCH_CHECK();
                gb_exclusive_scan_i32(nch, 0, hcp, sd.ng);
                nhch = gb_read_i64(hcp + sd.ng);
                gb_stat_add(SWAP ? "dot_hub_chunks_C" : "dot_hub_chunks_R", nhch);
                if (nhch)
                    hipLaunchKernelGGL((k_dt_hub_classify<SWAP>), dim3((unsigned)std::min<int64_t>(nhch, 1 << 16)),
                                       dim3(DT_BLOCK), 0, gb_stream(), sd, hcp, nhch, hflag, pieces ? hg : nullptr);
                GB_LAUNCH_CHECK();
            }
            // tasks over (eG, eYS, eO, eB, eQ) in task order: cut at group changes and windows
            auto run_tasks = [&](int64_t ne, int32_t *eG, int64_t *eYS, int32_t *eO, int32_t *eB, int64_t *eQ,
                                 const uint16_t *ePc) {
                gb_scratch ts;
                const int64_t K = gb_knob("dot_yblk");
                if (K > 1 && K <= 4096 && ne > 1) {
                    int bits = 0;
                    while ((1LL << bits) < K) bits++;
                    int32_t *key = ts.get<int32_t>(ne);
                    int64_t *idx = ts.get<int64_t>(ne);
                    const int64_t ytot = gb_read_i64(sd.yrp + (SWAP ? A.nrows : BT.nrows));
                    hipLaunchKernelGGL(k_dt_ykey, dim3(dt_grid(ne)), dim3(DT_BLOCK), 0, gb_stream(), ne, (int)K, ytot,
                                       eYS, key, idx);
                    GB_LAUNCH_CHECK();
                    gb_sort_pairs_i32(key, idx, ne, bits);  // stable: G order inside a block
                    auto perm = [&](auto *arr) {
                        using T = std::remove_pointer_t<decltype(arr)>;
                        T *tmp = gb_malloc_n<T>(ne);
                        hipLaunchKernelGGL(k_dt_gather<T>, dim3(dt_grid(ne)), dim3(DT_BLOCK), 0, gb_stream(), ne, idx,
                                           (const T *)arr, tmp);
                        GB_LAUNCH_CHECK();
                        gb_copy_d2d(arr, tmp, ne * sizeof(T));
                        gb_free(tmp);
                    };
                    perm(eG);
                    perm(eYS);
                    perm(eO);
                    perm(eB);
                    perm(eQ);
                    if (ePc) perm(const_cast<uint16_t *>(ePc));
                }
                int64_t *cum = ts.get<int64_t>(ne + 1);
                gb_exclusive_scan_i32(eB, (int)ovh, cum, ne);
                uint8_t *tsf = ts.get<uint8_t>(ne);
                hipLaunchKernelGGL(k_dt_task_flags, dim3(dt_grid(ne)), dim3(DT_BLOCK), 0, gb_stream(), ne, win, eG,
                                   ePc, cum, tsf);
                int64_t *tpos = ts.get<int64_t>(ne + 1);
                gb_exclusive_scan_u8(tsf, tpos, ne);
                const int64_t nt = gb_read_i64(tpos + ne);
                int64_t *tstart = ts.get<int64_t>(nt + 1);
                hipLaunchKernelGGL(k_dt_task_fill, dim3(dt_grid(ne)), dim3(DT_BLOCK), 0, gb_stream(), ne, tsf, tpos,
                                   tstart);
                GB_LAUNCH_CHECK();
                dt_task *tdesc = ts.get<dt_task>(nt);
                hipLaunchKernelGGL(k_dt_task_desc, dim3(dt_grid(nt)), dim3(DT_BLOCK), 0, gb_stream(), nt, tstart, eG,
                                   ePc, sd.xrp, cap, tdesc);
                GB_LAUNCH_CHECK();
                // persistent workgroups (two per CU) taking chunks of consecutive tasks
                const unsigned gt = (unsigned)std::min<int64_t>(nt, 1024);
                unsigned long long *tctr = ts.get<unsigned long long>(17);  // [0] chunk counter, [16] X loads
                gb_memset(tctr, 0, 17 * sizeof(unsigned long long));
                const bool dstat = gb_knob("dot_stats") == 1;
                // tools/spgemm_probe.py (R-MAT, one box): chunk 1/4/8/16/32 -> s20 24.7/24.1/25.3/27.7/33.0 ms,
                // s22 (1/8/32) 128.6/121.5/136.3 ms
                int64_t chunk = gb_knob("dot_chunk");
                if (chunk <= 0) chunk = 4;
                if (!(skip & 2))
                    hipLaunchKernelGGL((k_dot_task<SRT, X, Z, SWAP>), dim3(gt), dim3(DT_TB), 0, gb_stream(), srf,
                                       info.mon, sd, xv, yv, nt, tdesc, eG, eYS, eO, eB, eQ, (Z *)tval,
                                       tflag,
                                       (int)gb_knob("dot_dbg") | (gb_knob("dot_xlds") == 1 ? 4096 : 0) | (dstat ? 1024 : 0) |
                                           ((gb_knob("dot_ypack") != 1 && nkey <= (1LL << 24)) ? 8192 : 0),
                                       ePc,
                                       cap, tctr, (int)chunk,
                                       (int)gb_knob("dot_filt_ratio"));
                GB_LAUNCH_CHECK();
                if (dstat) {  // diagnostics: a host read per launch
                    gb_stat_add(ePc ? "dot_piece_tasks" : "dot_tasks", nt);
                    gb_stat_add("dot_task_xloads", gb_read_i64((const int64_t *)tctr + 16));
                }
            };
            gb_exclusive_scan_u8(tf, pos, nm);
            const int64_t ne = gb_read_i64(pos + nm);
            gb_stat_add(SWAP ? "dot_task_entries_C" : "dot_task_entries_R", ne);
            if (ne) {
                gb_scratch es;
                int32_t *eG = es.get<int32_t>(ne);
                int64_t *eYS = es.get<int64_t>(ne);
                int32_t *eO = es.get<int32_t>(ne);
                int32_t *eB = es.get<int32_t>(ne);
                int64_t *eQ = es.get<int64_t>(ne);
                hipLaunchKernelGGL((k_dt_compact<SWAP>), dim3(gw), dim3(DT_BLOCK), 0, gb_stream(), sd, cap, tf, pos,
                                   eG, eYS, eO, eB, eQ, false, nullptr);
                GB_LAUNCH_CHECK();
                run_tasks(ne, eG, eYS, eO, eB, eQ, nullptr);
            }
            if (!pieces) return;
            gb_exclusive_scan_u8(hg, pos, nm);
            const int64_t nh = gb_read_i64(pos + nm);
            if (nh == 0) return;
            // few huge entries: the per-entry kernel costs less than the piece passes' fixed
            // work (R-MAT s20: 40k entries per phase, 1.5 ms slower as pieces; s22: 937k,
            // 15 ms faster); knob dot_pmin overrides
            int64_t pmin = gb_knob("dot_pmin");
            if (pmin <= 0) pmin = 131072;
            if (gb_knob("dot_dbg") & 16) fprintf(stderr, "dot phase %d: %lld huge entries\n", (int)SWAP, (long long)nh);
            if (nh < pmin) {
                hipLaunchKernelGGL(k_dt_huge_to_csr, dim3(dt_grid(nm)), dim3(DT_BLOCK), 0, gb_stream(), nm, hg, sd.perm,
                                   hflag);
                GB_LAUNCH_CHECK();
                return;
            }
            gb_scratch hs;
            int32_t *hG = hs.get<int32_t>(nh);
            int64_t *hYS = hs.get<int64_t>(nh);
            int32_t *hO = hs.get<int32_t>(nh);
            int32_t *hB = hs.get<int32_t>(nh);
            int64_t *hQ = hs.get<int64_t>(nh);
            if (hubc) {
                hipLaunchKernelGGL((k_dt_hub_compact<SWAP>), dim3((unsigned)std::min<int64_t>(nhch, 1 << 16)),
                                   dim3(DT_BLOCK), 0, gb_stream(), sd, hcp, nhch, hg, pos, hG, hYS, hO, hB, hQ);
            } else {
                hipLaunchKernelGGL((k_dt_compact<SWAP>), dim3(gw), dim3(DT_BLOCK), 0, gb_stream(), sd, cap, hg, pos,
                                   hG, hYS, hO, hB, hQ, true, amax);
            }
            Z ident = Z();
            if (!(std::is_same<SRT, gb_sr_any_pair<Z>>::value || info.mon == GBAMD_MON_ANY))
                ident = gb_monoid_identity<Z>(info.mon);
            hipLaunchKernelGGL((k_dt_ident<Z>), dim3(dt_grid(nh)), dim3(DT_BLOCK), 0, gb_stream(), nh, hQ, (Z *)tval,
                               ident);
            GB_LAUNCH_CHECK();
            const int64_t amx = gb_read_i64((const int64_t *)amax);
            const int64_t np = (amx + cap - 1) / cap;
            if (np > 65535) {  // the piece index travels as 16 bits (ePc): such lists (> 2^29 keys)
                               // go to the per-entry kernel
                hipLaunchKernelGGL(k_dt_huge_to_csr, dim3(dt_grid(nm)), dim3(DT_BLOCK), 0, gb_stream(), nm, hg,
                                   sd.perm, hflag);
                GB_LAUNCH_CHECK();
                return;
            }
            // every piece's runs at once: one scan, one compaction, one task launch (round 4: one
            // pass per piece, each ending on a host read of its size); scratch in proportion to the
            // pieces the entries have (pairs numbered group by group, see dt_group_span)
            int64_t *P = hs.get<int64_t>(nh + 1);
            {
                int64_t *npc = hs.get<int64_t>(nh);
                hipLaunchKernelGGL(k_dt_piece_count, dim3(dt_grid(nh)), dim3(DT_BLOCK), 0, gb_stream(), sd, nh, cap,
                                   hG, npc);
                GB_LAUNCH_CHECK();
                gb_exclusive_scan_i64(npc, P, nh);
            }
            const int64_t npairs = gb_read_i64(P + nh);
            int32_t *pc = hs.get<int32_t>(npairs);
            int64_t *ppos = hs.get<int64_t>(npairs + 1);
            int64_t *pys = hs.get<int64_t>(npairs);
            int32_t *pb = hs.get<int32_t>(npairs);
            hipLaunchKernelGGL(k_dt_piece_flags, dim3(dt_grid(nh)), dim3(DT_BLOCK), 0, gb_stream(), sd, nh, cap, hG,
                               hYS, hB, P, pos, pc, pys, pb);
            GB_LAUNCH_CHECK();
            gb_exclusive_scan_i32(pc, 0, ppos, npairs);
            const int64_t npe = gb_read_i64(ppos + npairs);
            gb_stat_add(SWAP ? "dot_piece_entries_C" : "dot_piece_entries_R", npe);
            if (npe == 0) return;
            gb_scratch ps;
            int32_t *eG = ps.get<int32_t>(npe);
            int64_t *eYS = ps.get<int64_t>(npe);
            int32_t *eO = ps.get<int32_t>(npe);
            int32_t *eB = ps.get<int32_t>(npe);
            int64_t *eQ = ps.get<int64_t>(npe);
            uint16_t *ePc = ps.get<uint16_t>(npe);
            hipLaunchKernelGGL(k_dt_piece_compact, dim3(dt_grid(nh)), dim3(DT_BLOCK), 0, gb_stream(), sd, nh, cap, hG,
                               hO, hQ, P, pos, pc, ppos, pys, pb, eG, eYS, eO, eB, eQ, ePc);
            GB_LAUNCH_CHECK();
            run_tasks(npe, eG, eYS, eO, eB, eQ, ePc);
        };
        phase(std::false_type{});
        phase(std::true_type{});
    });
    // entries left to the per-entry kernel
    gb_exclusive_scan_u8(hflag, pos, nm);
    const int64_t nh = gb_read_i64(pos + nm);
    gb_stat_add("dot_calls", 1);
    gb_stat_add("dot_huge_entries", nh);
    if (nh) {
        int64_t *hq = gb_malloc_n<int64_t>(nh);
        hipLaunchKernelGGL(k_dt_positions, dim3(dt_grid(nm)), dim3(DT_BLOCK), 0, gb_stream(), nm, hflag, pos, hq);
        GB_LAUNCH_CHECK();
        *huge = hq;
    }
    gb_free(own_rp);
    gb_free(own_ci);
    gb_free(own_vx);
    gb_free(own_perm);
    return nh;
}
