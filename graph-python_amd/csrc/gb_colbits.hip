// gb_colbits.hip -- batched frontiers: GrB_mxm with a left operand of at most 64
// rows over a boolean (LOR / ANY) semiring, and the masked scalar assign that
// stamps levels, on a column-word bitmap format.
//
// Why: a multi-source BFS in GraphBLAS (k roots at once, LAGraph style) is
//     V<Q.V> = d;  Q<!V.S, replace> = Q lor.land A      (Q, V: k x n)
// i.e. the north-star's masked GrB_mxm (reference core/matrix.py:2241, dispatched
// by core/base.py:483) with Q and V as the k-row operands.  Held as CSR, every
// level would rewrite V's whole row structure (k x n entries at the end) and Q's;
// SuiteSparse switches such matrices to its bitmap format.  Here a matrix of
// k <= 64 rows switches to column words: cw[j] holds the k presence bits of
// column j (bit r = entry (r, j)), values column-major (cw_vals[j * k + r]).
// Then one level is one pass over the graph for all k sources:
//   pull (rows of B^T = in-edges of output column j):  out[j] = OR_i F[i] & need(j),
//        need(j) = the mask's complement in column j; a wave owns 64 consecutive
//        columns and walks their in-edges as one flat list (cb_pull_chunk), columns
//        longer than 512 edges run as pieces from the cached hub table (a wave per
//        piece, early exit once every needed bit is found);
//   push (rows of B = out-edges of frontier column i):  atomicOr(out[j], F[i] & need(j))
//        with a pre-check, newly set bits counted from the atomic's old value.
// Direction is chosen on the device (Beamer): push iff the frontier's out-edges x
// alpha < nnz(B); each level's kernel leaves the next level's edge count
// (cw_stat[1]) and the count (cw_stat[0]), both published to the host mailbox.
// Result values: a boolean LOR/ANY fold of iso operands is iso, its value
// mult(a, b) computed on the device, so structure is all the kernel produces.
// Traffic per pull level: 4 B per scanned edge (coalesced) plus one random 8-byte
// access per scanned edge (the summary bit, or the frontier word F[i]: n x 8 B =
// 32 MB at s22), each costing a cache line -- that random-line rate, not HBM
// streaming, bounds the kernel.  Level stamps are pending layers
// applied when V's values are read.
//
// Every other API entry point sees CSR: gb_obj_check converts back (gb_cw_to_csr:
// per-column popcounts, scan, CSC fill, transpose).
#include <algorithm>
#include <mutex>
#include <unordered_map>
#include <vector>

#include "gb_dispatch.cuh"
#include "gb_internal.h"

namespace {

constexpr int CB_BLOCK = 256;
constexpr int CB_CAP = 32;  // edges a lane walks alone before the wave takes its column over (push)
constexpr int CB_U = 4;     // 64-edge windows a pull wave has in flight
constexpr int CB_MAX_LAYERS = 16;  // pending level stamps per matrix (LDS: 32 KB per block to apply)

GB_DEV uint64_t cb_shfl(uint64_t v, int src) {
    const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)v, src, 64);
    const uint32_t hi = (uint32_t)__shfl((int)(uint32_t)(v >> 32), src, 64);
    return ((uint64_t)hi << 32) | lo;
}
GB_DEV int64_t cb_shfl_i64(int64_t v, int src) { return (int64_t)cb_shfl((uint64_t)v, src); }
GB_DEV uint64_t cb_wave_or(uint64_t v) {
    for (int off = 32; off > 0; off >>= 1) v |= cb_shfl(v, (int)(threadIdx.x & 63) ^ off);
    return v;
}
GB_DEV void cb_copy(void *dst, const void *src, int size) {
    switch (size) {
        case 1: *(uint8_t *)dst = *(const uint8_t *)src; break;
        case 2: *(uint16_t *)dst = *(const uint16_t *)src; break;
        case 4: *(uint32_t *)dst = *(const uint32_t *)src; break;
        default: *(uint64_t *)dst = *(const uint64_t *)src; break;
    }
}
GB_DEV void cb_publish(gb_host_slot *pub, long long seq, long long value, long long hint) {
    if (!pub) return;
    __hip_atomic_store(&pub->value, value, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(&pub->pad[0], hint, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __threadfence_system();
    __hip_atomic_store(&pub->seq, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

struct cb_step_args {
    int64_t nout, nin, nnz;
    const uint64_t *F;                      // input column words [nin]
    const int64_t *prp;                     // pull CSR: rows = output columns, entries = input columns
    const int32_t *pci;
    const int64_t *srp;                     // push CSR: rows = input columns (nullptr: pull only)
    const int32_t *sci;
    const uint64_t *M;                      // mask words [nout] (nullptr: no mask)
    const void *m_iso;                      // value mask of an iso matrix: its value (nullptr: structure)
    int m_iso_code;                         // its type (mask truth: -0.0 is false, NaN true)
    bool comp;
    uint64_t full;                          // the k row bits
    uint64_t *out;                          // [nout], zeroed
    const int64_t *stat_in;                 // F's [count, out-edges]
    int64_t alpha;
    int dir;                                // 0 auto, 1 pull, 2 push
    int64_t *stat_out;
    unsigned long long *gst, *gst2;
    gb_host_slot *pub;
    long long seq;
    const uint8_t *a_val, *b_val;           // iso values of the operands (nullptr: not iso)
    int mul;
    uint8_t *out_val;
    const uint64_t *S_in;                   // F's summary: bit i = (F[i] != 0), valid when stat_in[2] == 1
    uint64_t *S_out;                        // out's summary (zeroed)
    const int32_t *p_tab, *s_tab;           // hub pieces (row, piece) of the pull / push orientation
    int64_t p_nhub, s_nhub, H;
    const uint64_t *Fhot;                   // pci relabelled (gb_view_hot): F of the hot sources, rank order
    bool serial;                            // knob colbits_serial: the round-4 gather order (A/B)
};

// the level pushes (same rule as k_cw_step)
GB_DEV bool cb_pushes(const cb_step_args &a) {
    return a.srp && (a.dir == 2 || (a.dir == 0 && a.stat_in[1] * a.alpha < a.nnz));
}

// F word of in-edge source i of the pull list: i < 0 names a hot source (relabelled pci),
// whose word was packed into Fhot before the step; a sparse frontier tests the summary bit
// (L2-resident) before gathering a cold word
GB_DEV uint64_t cb_gather(const cb_step_args &a, int64_t i, bool use_sum) {
    if (i < 0) return a.Fhot[i & 0x7fffffffLL];
    if (use_sum && !((a.S_in[i >> 6] >> (i & 63)) & 1ULL)) return 0ULL;
    return a.F[i];
}

GB_DEV uint64_t cb_need(const cb_step_args &a, int64_t j, bool m_on) {
    if (!a.M) return a.full;
    const uint64_t m = m_on ? a.M[j] : 0ULL;
    return a.comp ? (~m & a.full) : (m & a.full);
}

GB_DEV bool cb_mult_value(int mul, bool x, bool y) {
    switch (mul) {
        case GBAMD_OP_FIRST: return x;
        case GBAMD_OP_SECOND: return y;
        case GBAMD_OP_PAIR: return true;
        case GBAMD_OP_LOR:
        case GBAMD_OP_MAX: return x || y;
        default: return x && y;  // LAND, TIMES, MIN
    }
}

// Pull of one wave's 64 output columns j = base + lane: their (non-hub) in-edges
// are walked as one flat list -- list position t belongs to the column found by a
// shuffle binary search over the columns' list offsets -- CB_U windows of 64 gathers
// in flight, OR-folded by a segmented wave scan; the segment ends fold into the
// columns' LDS slots acc_w[0..63].  Columns whose need is empty contribute no edges.
// rp/ci: the pull rows (int64 or int32 row pointers, entries relative to ci).
template <class RP>
GB_DEV void cb_pull_chunk(const cb_step_args &a, int64_t j, bool m_on, bool use_sum, const RP *__restrict__ rp,
                          const int32_t *__restrict__ ci, bool hubs, int64_t H, uint64_t *acc_w, uint64_t &need,
                          bool &hub) {
    const int lane = threadIdx.x & 63;
    int64_t s0 = 0;
    int len = 0;
    if (j < a.nout) {
        need = cb_need(a, j, m_on);
        if (need) {
            s0 = rp[j];
            const int64_t dl = (int64_t)rp[j + 1] - s0;
            hub = hubs && dl > H;
            len = hub ? 0 : (int)dl;
        }
    }
    // exclusive scan of the lengths
    int v = len;
    for (int off = 1; off < 64; off <<= 1) {
        const int g = __shfl_up(v, off, 64);
        if (lane >= off) v += g;
    }
    const int T = __shfl(v, 63, 64);
    v -= len;
    const int64_t eb = s0 - v;  // edge index = t + eb of the owning column
    acc_w[lane] = 0;
    for (int tb = 0; tb < T; tb += 64 * CB_U) {
        // CB_U windows of 64 list positions: searches, then all loads, then the folds
        int c[CB_U];
        uint64_t f[CB_U];
#pragma unroll
        for (int u = 0; u < CB_U; u++) {
            const int t = tb + 64 * u + lane;
            // every lane runs the search (uniform shuffles); lanes past the list get c = 64
            const int tt = t < T ? t : T - 1;
            int lo = 0;
#pragma unroll
            for (int step = 32; step > 0; step >>= 1)
                if (__shfl(v, lo + step, 64) <= tt) lo += step;
            c[u] = t < T ? lo : 64;
            f[u] = 0;
        }
        int32_t src[CB_U];
#pragma unroll
        for (int u = 0; u < CB_U; u++) {
            const int t = tb + 64 * u + lane;
            const int64_t q = (int64_t)t + cb_shfl_i64(eb, c[u] < 64 ? c[u] : 0);
            src[u] = t < T ? ci[q] : 0;
        }
        if (a.serial || !use_sum) {
#pragma unroll
            for (int u = 0; u < CB_U; u++)
                if (c[u] < 64) f[u] = cb_gather(a, src[u], use_sum);
        } else {
            // a sparse frontier: every window's summary word first, then the frontier words of
            // the sources it marks, each round with all loads in flight (cb_gather's test orders
            // each window's summary read behind the previous window's word)
            uint64_t sw[CB_U];
#pragma unroll
            for (int u = 0; u < CB_U; u++) {
                sw[u] = 0;
                if (c[u] < 64 && src[u] >= 0) sw[u] = a.S_in[src[u] >> 6];
            }
#pragma unroll
            for (int u = 0; u < CB_U; u++) {
                if (c[u] < 64) {
                    if (src[u] < 0) f[u] = a.Fhot[src[u] & 0x7fffffff];
                    else if ((sw[u] >> (src[u] & 63)) & 1ULL) f[u] = a.F[src[u]];
                }
            }
        }
#pragma unroll
        for (int u = 0; u < CB_U; u++) {
            uint64_t x = f[u];
            const int cu = c[u];
            for (int off = 1; off < 64; off <<= 1) {
                const uint32_t glo = (uint32_t)__shfl_up((int)(uint32_t)x, off, 64);
                const uint32_t ghi = (uint32_t)__shfl_up((int)(uint32_t)(x >> 32), off, 64);
                const int cc = __shfl_up(cu, off, 64);
                if (lane >= off && cc == cu) x |= ((uint64_t)ghi << 32) | glo;
            }
            const int cn = __shfl_down(cu, 1, 64);
            if (cu < 64 && (lane == 63 || cn != cu)) acc_w[cu] |= x;
        }
    }
}

GB_DEV void cb_finish(const cb_step_args &a, long long cnt, long long hint);

// One level of C<M> = F lor.land B (or any.pair ...): pull or push, chosen from
// stat_in on the device.  Rows longer than H of the chosen orientation run as
// H-edge pieces from the cached hub table (a wave per piece, results OR'ed in
// with atomics) so an R-MAT hub does not serialise one wave; the rest run a lane
// per row.  All blocks call the grid sums once.
__global__ __launch_bounds__(CB_BLOCK) void k_cw_step(cb_step_args a) {
    const int lane = threadIdx.x & 63;
    const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
    const bool m_on = !a.m_iso || gb_dyn_nonzero(a.m_iso, a.m_iso_code);
    const bool push = cb_pushes(a);
    // sparse frontier: test the summary bit (L2-resident) before gathering a word
    const bool use_sum = a.S_in && a.stat_in[2] == 1 && a.stat_in[0] * 4 < a.nin;
    const int64_t H = a.H;
    long long cnt = 0, hint = 0;
    // OR bits into out[j] (out is zeroed): count the new bits, the column's edges when it
    // turns non-empty, and its summary bit
    auto put = [&](int64_t j, uint64_t nb) {
        const uint64_t old = atomicOr((unsigned long long *)&a.out[j], (unsigned long long)nb);
        const uint64_t add = nb & ~old;
        cnt += __popcll(add);
        if (old == 0 && add) {
            atomicOr((unsigned long long *)&a.S_out[j >> 6], 1ULL << (j & 63));
            if (a.srp && j < a.nin) hint += a.srp[j + 1] - a.srp[j];
        }
    };
    if (!push) {
        // hub pieces: rows of the pull orientation longer than H
        for (int64_t t = wave; t < a.p_nhub; t += nwaves) {
            const int64_t j = a.p_tab[2 * t], piece = a.p_tab[2 * t + 1];
            const uint64_t need = cb_need(a, j, m_on);
            if (!need) continue;
            const int64_t beg = a.prp[j] + piece * H, rend = a.prp[j + 1];
            const int64_t end = beg + H < rend ? beg + H : rend;
            uint64_t acc = 0;
            for (int64_t qb = beg; qb < end; qb += 256) {
                uint64_t f = 0;
#pragma unroll
                for (int u = 0; u < 4; u++) {
                    const int64_t q = qb + lane + 64 * u;
                    if (q < end) f |= cb_gather(a, a.pci[q], use_sum);
                }
                acc |= cb_wave_or(f);
                if ((acc & need) == need) break;
            }
            if (lane == 0 && (acc & need)) put(j, acc & need);
        }
        // a wave owns 64 consecutive output columns and walks their (non-hub) in-edges as
        // one flat list: edge t of the list belongs to the column found by a shuffle binary
        // search over the columns' list offsets; gathers are OR-folded by a segmented wave
        // scan and the segment ends fold into the column's LDS slot.  Columns whose need is
        // empty (visited by every source) contribute no edges.
        __shared__ uint64_t lacc[CB_BLOCK / 64][64];
        uint64_t *acc_w = lacc[threadIdx.x >> 6];
        for (int64_t base = wave * 64; base < a.nout; base += nwaves * 64) {
            const int64_t j = base + lane;
            uint64_t need = 0;
            bool hub = false;
            cb_pull_chunk(a, j, m_on, use_sum, a.prp, a.pci, a.p_tab != nullptr, H, acc_w, need, hub);
            const uint64_t w = (j < a.nout && !hub) ? (acc_w[lane] & need) : 0ULL;
            if (w) {
                a.out[j] = w;  // hub columns are OR'ed in by their pieces
                cnt += __popcll(w);
                if (a.srp && j < a.nin) hint += a.srp[j + 1] - a.srp[j];
            }
            const uint64_t sb = __ballot(w != 0);
            if (lane == 0 && sb) atomicOr((unsigned long long *)&a.S_out[base >> 6], (unsigned long long)sb);
        }
    } else {
        auto push_one = [&](int64_t j, uint64_t f) {
            const uint64_t nb = f & cb_need(a, j, m_on);
            if (!nb) return;
            const uint64_t cur = __hip_atomic_load(&a.out[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if ((cur & nb) == nb) return;
            put(j, nb);
        };
        for (int64_t t = wave; t < a.s_nhub; t += nwaves) {
            const int64_t i = a.s_tab[2 * t], piece = a.s_tab[2 * t + 1];
            const uint64_t f = a.F[i];
            if (!f) continue;
            const int64_t beg = a.srp[i] + piece * H, rend = a.srp[i + 1];
            const int64_t end = beg + H < rend ? beg + H : rend;
            for (int64_t q = beg + lane; q < end; q += 64) push_one(a.sci[q], f);
        }
        for (int64_t base = wave * 64; base < a.nin; base += nwaves * 64) {
            const int64_t i = base + lane;
            const uint64_t f = i < a.nin ? a.F[i] : 0ULL;
            int64_t p = 0, e = 0;
            if (f) {
                p = a.srp[i];
                e = a.srp[i + 1];
                if (a.s_tab && e - p > H) p = e;  // a hub: its pieces above
            }
            const int64_t lim = e < p + CB_CAP ? e : p + CB_CAP;
            for (; p < lim; p++) push_one(a.sci[p], f);
            uint64_t longs = __ballot(p < e);
            while (longs) {
                const int L = __ffsll((unsigned long long)longs) - 1;
                longs &= longs - 1;
                const int64_t pL = cb_shfl_i64(p, L), eL = cb_shfl_i64(e, L);
                const uint64_t fL = cb_shfl(f, L);
                for (int64_t q = pL + lane; q < eL; q += 64) push_one(a.sci[q], fL);
            }
        }
    }
    cb_finish(a, cnt, hint);
}

// the hot sources' frontier words, packed in rank order for a pulling step (no-op when it pushes)
__global__ __launch_bounds__(CB_BLOCK) void k_cw_hot_gather(cb_step_args a, const int32_t *__restrict__ hot,
                                                             int64_t nh, uint64_t *__restrict__ Fhot) {
    if (cb_pushes(a)) return;
    for (int64_t h = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; h < nh; h += (int64_t)gridDim.x * blockDim.x)
        Fhot[h] = a.F[hot[h]];
}

// count and edge-hint grid sums; whichever block finishes the second one publishes
// both to the host mailbox (the hint lets the host pick the next call's direction)
GB_DEV void cb_finish(const cb_step_args &a, long long cnt, long long hint) {
    long long tot;
    int nf = 0;
    if (gb_grid_sum(cnt, a.gst, &tot)) {
        __hip_atomic_store(&a.stat_out[0], (int64_t)tot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        nf++;
    }
    if (gb_grid_sum(hint, a.gst2, &tot)) {
        __hip_atomic_store(&a.stat_out[1], (int64_t)tot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        nf++;
    }
    if (nf) {
        __threadfence();
        unsigned long long *flag = a.gst + (size_t)GB_GRID_SHARDS * GB_GRID_STRIDE + 8;
        const unsigned long long old = atomicAdd(flag, (unsigned long long)nf);
        if (old + nf == 2) {
            atomicExch(flag, 0ULL);
            __threadfence();
            const long long c = __hip_atomic_load(&a.stat_out[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const long long h = __hip_atomic_load(&a.stat_out[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            cb_publish(a.pub, a.seq, c, h);
        }
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        a.stat_out[2] = 1;  // summary words valid
        *a.out_val = cb_mult_value(a.mul, a.a_val ? *a.a_val != 0 : true, a.b_val ? *a.b_val != 0 : true);
    }
}

// stat[1] = out-edges (rows of srp) of the non-empty columns of F
__global__ __launch_bounds__(CB_BLOCK) void k_cw_hint(const uint64_t *__restrict__ F, int64_t n,
                                                       const int64_t *__restrict__ srp, int64_t *__restrict__ stat,
                                                       unsigned long long *gst) {
    long long h = 0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        if (F[i]) h += srp[i + 1] - srp[i];
    long long tot;
    if (gb_grid_sum(h, gst, &tot)) stat[1] = tot;
}

// CSR (k rows) -> column words; stat = [nvals, out-edges of the entries' columns in srp]
__global__ __launch_bounds__(CB_BLOCK) void k_csr_to_cw(int k, int64_t nvals, const int64_t *__restrict__ rowptr,
                                                         const int32_t *__restrict__ colidx, const uint8_t *vals,
                                                         int vsize, uint64_t *__restrict__ cw, uint64_t *__restrict__ S,
                                                         uint8_t *cwv,
                                                         const int64_t *__restrict__ srp, int64_t nsrp,
                                                         int64_t *__restrict__ stat, unsigned long long *gst) {
    long long h = 0;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < nvals;
         e += (int64_t)gridDim.x * blockDim.x) {
        int lo = 0, hi = k;  // row r: rowptr[r] <= e < rowptr[r + 1]
        while (hi - lo > 1) {
            const int mid = (lo + hi) >> 1;
            if (rowptr[mid] <= e) lo = mid;
            else hi = mid;
        }
        const int64_t j = colidx[e];
        atomicOr((unsigned long long *)&cw[j], 1ULL << lo);
        atomicOr((unsigned long long *)&S[j >> 6], 1ULL << (j & 63));
        if (cwv) cb_copy(cwv + (j * k + lo) * vsize, vals + e * vsize, vsize);
        if (srp && j < nsrp) h += srp[j + 1] - srp[j];
    }
    long long tot;
    if (gb_grid_sum(h, gst, &tot)) {
        stat[0] = nvals;
        stat[1] = tot;
        stat[2] = 1;
    }
}

__global__ void k_cw_pop(const uint64_t *__restrict__ cw, int64_t n, int64_t *__restrict__ pop) {
    for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n; j += (int64_t)gridDim.x * blockDim.x)
        pop[j] = __popcll(cw[j]);
}

// CSC of a column-word matrix: column j's rows in ascending order (+ values)
__global__ void k_cw_fill(const uint64_t *__restrict__ cw, int64_t n, int k, const int64_t *__restrict__ cptr,
                          int32_t *__restrict__ ridx, const uint8_t *cwv, uint8_t *tv, int vsize) {
    for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n; j += (int64_t)gridDim.x * blockDim.x) {
        uint64_t w = cw[j];
        int64_t o = cptr[j];
        while (w) {
            const int r = __ffsll((unsigned long long)w) - 1;
            w &= w - 1;
            ridx[o] = r;
            if (tv) cb_copy(tv + o * vsize, cwv + (j * k + r) * vsize, vsize);
            o++;
        }
    }
}

// C<M> = x (all indices, no accum): bits OR'ed in, x stored at the mask's entries,
// count delta added to stat[0].  A wave owns 64 columns; the value stores of each
// column with new bits go out as one wave-wide store (lane r -> row r), so a
// column's values are written as one coalesced segment.
__global__ __launch_bounds__(CB_BLOCK) void k_cw_assign(int64_t n, int k, const uint64_t *__restrict__ M,
                                                         const void *m_iso, int m_code, const uint8_t *m_vals,
                                                         int m_vsize, uint64_t *__restrict__ C, uint8_t *cv,
                                                         unsigned long long x, int vsize, int64_t *stat,
                                                         unsigned long long *gst) {
    const int lane = threadIdx.x & 63;
    const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
    const bool m_on = !m_iso || gb_dyn_nonzero(m_iso, m_code);
    long long delta = 0;
    for (int64_t base = wave * 64; base < n; base += nwaves * 64) {
        const int64_t j = base + lane;
        uint64_t m = (m_on && j < n) ? M[j] : 0ULL;
        if (m && m_vals) {  // value mask: keep the bits whose value is nonzero
            uint64_t t = m, keep = 0;
            while (t) {
                const int r = __ffsll((unsigned long long)t) - 1;
                t &= t - 1;
                if (gb_dyn_nonzero(m_vals + (j * k + r) * m_vsize, m_code)) keep |= 1ULL << r;
            }
            m = keep;
        }
        if (m) {
            const uint64_t old = C[j];
            C[j] = old | m;
            delta += __popcll(m & ~old);
        }
        uint64_t cols = __ballot(m != 0);
        while (cols) {
            const int c = __ffsll((unsigned long long)cols) - 1;
            cols &= cols - 1;
            const uint64_t mc = cb_shfl(m, c);
            if (lane < k && ((mc >> lane) & 1ULL)) cb_copy(cv + ((base + c) * k + lane) * vsize, &x, vsize);
        }
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) stat[2] = 0;  // the summary words no longer match
    gb_grid_add(delta, (unsigned long long *)stat, gst);
}

// count + summary of rewritten words; publish the count
__global__ __launch_bounds__(CB_BLOCK) void k_cw_recount(const uint64_t *__restrict__ W, int64_t n,
                                                          uint64_t *__restrict__ S, int64_t *stat,
                                                          unsigned long long *gst, gb_host_slot *pub, long long seq) {
    const int lane = threadIdx.x & 63;
    const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
    long long cnt = 0;
    for (int64_t base = wave * 64; base < n; base += nwaves * 64) {
        const int64_t j = base + lane;
        const uint64_t w = j < n ? W[j] : 0ULL;
        cnt += __popcll(w);
        const uint64_t sb = __ballot(w != 0);
        if (lane == 0) S[base >> 6] = sb;
    }
    long long tot;
    if (gb_grid_sum(cnt, gst, &tot)) {
        stat[0] = tot;
        stat[1] = 0;
        stat[2] = 1;
        cb_publish(pub, seq, tot, 0);
    }
}

// Pending level stamps.  C<M> = x over all indices with a structural (or iso-valued)
// mask only ORs M's words into C and records them as a layer (words, x); the values are
// written when something reads them (gb_cw_materialize: conversion, GrB_Matrix_wait,
// a value mask), in one pass that applies the layers in order -- GraphBLAS
// nonblocking pending work.  One pass over all entries replaces one scattered store
// per level (measured: 0.20-0.24 ms per dense level of the 64-root s22 BFS).
__global__ __launch_bounds__(CB_BLOCK) void k_cw_assign_layer(int64_t n, const uint64_t *__restrict__ M,
                                                               const void *m_iso, int m_code,
                                                               uint64_t *__restrict__ C, uint64_t *__restrict__ L,
                                                               int64_t *stat, unsigned long long *gst) {
    const bool m_on = !m_iso || gb_dyn_nonzero(m_iso, m_code);
    long long delta = 0;
    for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n; j += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t m = m_on ? M[j] : 0ULL;
        L[j] = m;
        if (m) {
            const uint64_t old = C[j];
            if ((old | m) != old) C[j] = old | m;
            delta += __popcll(m & ~old);
        }
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) stat[2] = 0;  // the summary words no longer match
    gb_grid_add(delta, (unsigned long long *)stat, gst);
}

struct cb_layers_dev {
    const uint64_t *bits[CB_MAX_LAYERS];
    unsigned long long x[CB_MAX_LAYERS];
};

// apply the layers in order: a wave owns 64 columns; their layer words are staged in
// LDS ([layer][column], coalesced loads), then each column with stamps is written as one
// wave-wide store (lane r -> row r, value of the last layer holding bit r)
__global__ __launch_bounds__(CB_BLOCK) void k_cw_apply_layers(int64_t n, int k, int nl, cb_layers_dev Ls,
                                                               uint8_t *cv, int vsize, bool full) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
    __shared__ uint64_t lw[CB_BLOCK / 64][CB_MAX_LAYERS][64];
    for (int64_t base = wave * 64; base < n; base += nwaves * 64) {
        const int64_t j = base + lane;
        uint64_t any = 0;
#pragma unroll
        for (int l = 0; l < CB_MAX_LAYERS; l++) {
            if (l < nl) {
                const uint64_t w = j < n ? Ls.bits[l][j] : 0ULL;
                lw[wid][l][lane] = w;
                any |= w;
            }
        }
        __builtin_amdgcn_wave_barrier();
        uint64_t cols = __ballot(any != 0);
        while (cols) {
            const int c = __ffsll((unsigned long long)cols) - 1;
            cols &= cols - 1;
            bool have = false;
            unsigned long long x = 0;
#pragma unroll
            for (int l = 0; l < CB_MAX_LAYERS; l++) {
                if (l < nl) {
                    const uint64_t w = lw[wid][l][c];
                    if ((w >> lane) & 1ULL) {
                        have = true;
                        x = Ls.x[l];
                    }
                }
            }
            // full: the matrix had no entries before its first layer, so every value of a
            // stamped column is a layer's or unused -- write the whole k-value segment
            // (full cache lines, no partial-line merges)
            if ((have || full) && lane < k) cb_copy(cv + ((base + c) * k + lane) * vsize, &x, vsize);
        }
        __builtin_amdgcn_wave_barrier();
    }
}

// whole-segment variant for 4-byte values, k % 4 == 0 and a target that was empty
// before its first layer (the level stamps of a BFS): a lane per column writes its
// k values as k/4 16-byte stores (a column's segment is contiguous, so the lane's
// stores fill whole lines; a wave store instruction touches 64 lines instead of the
// LDS-staged variant's 4 for 4x fewer instructions per value)
__global__ __launch_bounds__(CB_BLOCK) void k_cw_apply_layers_w4(int64_t n, int k, int nl, cb_layers_dev Ls,
                                                                  uint32_t *cv) {
    for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n; j += (int64_t)gridDim.x * blockDim.x) {
        uint64_t w[CB_MAX_LAYERS];
        uint64_t any = 0;
#pragma unroll
        for (int l = 0; l < CB_MAX_LAYERS; l++) {
            w[l] = l < nl ? Ls.bits[l][j] : 0ULL;
            any |= w[l];
        }
        if (!any) continue;
        uint4 *dst = (uint4 *)(cv + j * k);
        for (int rb = 0; rb < k; rb += 4) {
            uint32_t v[4] = {0, 0, 0, 0};
#pragma unroll
            for (int l = 0; l < CB_MAX_LAYERS; l++) {
                if (l < nl) {
                    const uint32_t x = (uint32_t)Ls.x[l];
#pragma unroll
                    for (int t = 0; t < 4; t++)
                        if ((w[l] >> (rb + t)) & 1ULL) v[t] = x;
                }
            }
            dst[rb >> 2] = make_uint4(v[0], v[1], v[2], v[3]);
        }
    }
}

// dense fill of an iso value (expanding an iso column-word matrix)
__global__ void k_cw_fill_iso(uint8_t *v, int64_t count, const uint8_t *one, int vsize) {
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < count; e += (int64_t)gridDim.x * blockDim.x)
        cb_copy(v + e * vsize, one, vsize);
}

unsigned cb_grid(int64_t items, unsigned cap) {
    int64_t g = (items + CB_BLOCK - 1) / CB_BLOCK;
    if (g < 1) g = 1;
    if (g > cap) g = cap;
    return (unsigned)g;
}

unsigned long long *grid_state(int which) {
    unsigned long long *st = gb_device_state();
    return which == 0 ? st : st + GB_GRID2_OFFSET;
}

// A (CSR, 1 <= k <= 64 rows) -> column words in place.  srp (optional): push rows
// keyed by hint_key for the out-edge hint.
void to_cw(GB_Obj *A, const int64_t *srp, int64_t nsrp, const void *hint_key) {
    const int k = (int)A->nrows;
    const int64_t n = A->ncols, nv = A->nvals;
    const int vs = (int)A->type->size;
    const int64_t nw = n + gb_words(n) + 1;  // words, then the summary bitmap
    uint64_t *cw = gb_malloc_n<uint64_t>(nw);
    gb_memset(cw, 0, nw * sizeof(uint64_t));
    int64_t *stat = gb_malloc_n<int64_t>(4);
    gb_memset(stat, 0, 4 * sizeof(int64_t));
    const bool iso = A->iso && nv > 0;
    void *cwv;
    if (iso) {
        cwv = gb_malloc(vs);
        gb_copy_d2d(cwv, A->vals, vs);
    } else {
        cwv = gb_malloc((size_t)vs * (size_t)k * (size_t)(n > 0 ? n : 1));
    }
    if (nv > 0) {
        hipLaunchKernelGGL(k_csr_to_cw, dim3(cb_grid(nv, 2048)), dim3(CB_BLOCK), 0, gb_stream(), k, nv, A->rowptr,
                           A->colidx, (const uint8_t *)A->vals, vs, cw, cw + n, iso ? nullptr : (uint8_t *)cwv, srp, nsrp,
                           stat, grid_state(0));
        GB_LAUNCH_CHECK();
    }
    gb_drop_transpose(A);
    gb_free(A->rowptr);
    gb_free(A->colidx);
    gb_free(A->vals);
    A->rowptr = nullptr;
    A->colidx = nullptr;
    A->vals = nullptr;
    A->cw = cw;
    A->cw_vals = cwv;
    A->cw_stat = stat;
    A->iso = iso;
    A->nvals = nv;
    A->nvals_valid = true;
    A->pub_seq = 0;
    A->hint_valid = srp != nullptr;  // stat[1]: the kernel's sum (or 0 when empty)
    A->hint_key = hint_key;
}

// make a column-word matrix's values per-entry (C of an assign)
void cw_expand(GB_Obj *A) {
    if (!A->iso) return;
    const int vs = (int)A->type->size;
    const int64_t count = A->nrows * A->ncols;
    uint8_t *v = (uint8_t *)gb_malloc((size_t)vs * (size_t)(count > 0 ? count : 1));
    if (count > 0) {
        hipLaunchKernelGGL(k_cw_fill_iso, dim3(cb_grid(count, 4096)), dim3(CB_BLOCK), 0, gb_stream(), v, count,
                           (const uint8_t *)A->cw_vals, vs);
        GB_LAUNCH_CHECK();
    }
    gb_free(A->cw_vals);
    A->cw_vals = v;
    A->iso = false;
}

bool small_rows(const GB_Obj *A) { return A->kind == GB_KIND_MATRIX && A->nrows >= 1 && A->nrows <= 64; }

struct cb_layer {
    uint64_t *bits;
    unsigned long long x;
};
std::mutex g_layers_mu;
std::unordered_map<const GB_Obj *, std::vector<cb_layer>> g_layers;

void drop_layers(const GB_Obj *A) {
    std::lock_guard<std::mutex> lk(g_layers_mu);
    auto it = g_layers.find(A);
    if (it == g_layers.end()) return;
    for (auto &l : it->second) gb_free(l.bits);
    g_layers.erase(it);
}

}  // namespace

void gb_cw_materialize(GB_Obj *A) {
    if (!A || !A->cw) return;
    std::vector<cb_layer> ls;
    {
        std::lock_guard<std::mutex> lk(g_layers_mu);
        auto it = g_layers.find(A);
        if (it == g_layers.end()) return;
        ls.swap(it->second);
        g_layers.erase(it);
    }
    // a leading {nullptr} entry marks "no entries before the first layer"
    const bool full = !ls.empty() && ls[0].bits == nullptr;
    if (full) ls.erase(ls.begin());
    if (ls.empty()) return;
    cb_layers_dev d{};
    for (size_t l = 0; l < ls.size(); l++) {
        d.bits[l] = ls[l].bits;
        d.x[l] = ls[l].x;
    }
    if (full && A->type->size == 4 && A->nrows % 4 == 0 && gb_knob("colbits_apply") != 2)
        hipLaunchKernelGGL(k_cw_apply_layers_w4, dim3(cb_grid(A->ncols, 8192)), dim3(CB_BLOCK), 0, gb_stream(),
                           A->ncols, (int)A->nrows, (int)ls.size(), d, (uint32_t *)A->cw_vals);
    else
        hipLaunchKernelGGL(k_cw_apply_layers, dim3(cb_grid(A->ncols, 2048)), dim3(CB_BLOCK), 0, gb_stream(), A->ncols,
                           (int)A->nrows, (int)ls.size(), d, (uint8_t *)A->cw_vals, (int)A->type->size, full);
    GB_LAUNCH_CHECK();
    for (auto &l : ls) gb_free(l.bits);
}

// ================================================================== storage
void gb_cw_release(GB_Obj *A) {
    if (!A->cw) return;
    drop_layers(A);
    gb_free(A->cw);
    gb_free(A->cw_vals);
    gb_free(A->cw_stat);
    A->cw = nullptr;
    A->cw_vals = nullptr;
    A->cw_stat = nullptr;
    A->pub_seq = 0;
    A->hint_valid = false;
}

void gb_cw_to_csr(GB_Obj *A) {
    if (!A->cw) return;
    gb_cw_materialize(A);
    const int k = (int)A->nrows;
    const int64_t n = A->ncols;
    const int vs = (int)A->type->size;
    const int64_t nv = gb_nvals(A);
    const bool iso = A->iso && nv > 0;
    int64_t *rp = nullptr;
    int32_t *ci = nullptr;
    void *vv = nullptr;
    if (nv == 0) {
        rp = gb_malloc_n<int64_t>(k + 1);
        gb_memset(rp, 0, (k + 1) * sizeof(int64_t));
    } else {
        gb_scratch s;
        int64_t *pop = s.get<int64_t>(n);
        int64_t *cptr = s.get<int64_t>(n + 1);
        int32_t *ridx = s.get<int32_t>(nv);
        uint8_t *tv = iso ? nullptr : s.get<uint8_t>((size_t)nv * vs);
        hipLaunchKernelGGL(k_cw_pop, dim3(cb_grid(n, 4096)), dim3(CB_BLOCK), 0, gb_stream(), A->cw, n, pop);
        GB_LAUNCH_CHECK();
        gb_exclusive_scan_i64(pop, cptr, n);
        hipLaunchKernelGGL(k_cw_fill, dim3(cb_grid(n, 4096)), dim3(CB_BLOCK), 0, gb_stream(), A->cw, n, k, cptr, ridx,
                           (const uint8_t *)A->cw_vals, tv, vs);
        GB_LAUNCH_CHECK();
        // (n x k) CSR of A^T -> CSR of A
        gb_transpose_csr(n, k, nv, cptr, ridx, iso ? A->cw_vals : (const void *)tv, vs, iso, &rp, &ci, &vv);
    }
    gb_cw_release(A);
    A->rowptr = rp;
    A->colidx = ci;
    A->vals = vv;
    A->nvals = nv;
    A->iso = iso;
    A->nvals_valid = true;
}

// ================================================================== C<M> = A (+).(x) B, A of <= 64 rows
bool gb_colbits_mxm(GB_Obj *C, GB_Obj *M, GrB_BinaryOp accum, GrB_Semiring sr, GB_Obj *A, GB_Obj *B,
                    const gb_desc &d) {
    const int64_t knob = gb_knob("colbits");  // 0 auto, 1 always when legal, 2 never
    if (knob == 2 || accum || !sr || sr->magic != GB_MAGIC) return false;
    if (!small_rows(A) || !small_rows(C) || B->kind != GB_KIND_MATRIX || d.tran0) return false;
    if (B->cw) return false;  // B is the graph; a column-word B takes the general path (converted)
    const int mon = sr->add->mcode, mul = sr->mul->opcode;
    if (sr->add->type->code != GBAMD_T_BOOL || (mon != GBAMD_MON_LOR && mon != GBAMD_MON_ANY)) return false;
    if (!sr->mul->xtype || sr->mul->xtype->code != GBAMD_T_BOOL || sr->mul->ztype->code != GBAMD_T_BOOL) return false;
    if (A->type->code != GBAMD_T_BOOL || B->type->code != GBAMD_T_BOOL || C->type->code != GBAMD_T_BOOL) return false;
    const bool uses_a = mul != GBAMD_OP_SECOND && mul != GBAMD_OP_PAIR;
    const bool uses_b = mul != GBAMD_OP_FIRST && mul != GBAMD_OP_PAIR;
    switch (mul) {
        case GBAMD_OP_FIRST: case GBAMD_OP_SECOND: case GBAMD_OP_PAIR: case GBAMD_OP_LAND:
        case GBAMD_OP_LOR: case GBAMD_OP_TIMES: case GBAMD_OP_MIN: case GBAMD_OP_MAX: break;
        default: return false;
    }
    const int64_t k = A->nrows;
    const int64_t inner = A->ncols, br = d.tran1 ? B->ncols : B->nrows, bc = d.tran1 ? B->nrows : B->ncols;
    if (inner != br || C->nrows != k || C->ncols != bc) return false;  // the general path reports it
    // result values: every product's value is mult(a, b) of the iso operand values
    if ((uses_a && !(A->iso || (!A->cw && A->nvals == 0))) || (uses_b && !(B->iso || B->nvals == 0))) return false;
    // ~NULL selects nothing (C kept, or cleared under replace): the general path's rule
    // (gb_writeback.hip, gb_make_mmask) -- not a shape of this kernel
    if (!M && d.comp) return false;
    if (M) {
        if (!small_rows(M) || M->nrows != k || M->ncols != bc) return false;
        if (!d.structure && !M->iso && !(M->cw == nullptr && M->nvals == 0)) return false;
        // C<M> without replace keeps C's entries outside the mask: only when C is empty
        if (!d.replace && (C->cw || C->nvals != 0)) return false;
        if (M == B) return false;  // converting M would free the CSR the kernel reads
    }
    if (A == B) return false;
    if (knob == 0 && !A->cw && inner < 4096) return false;  // small problems keep the CSR kernels

    // operand views: pull rows = output columns (B^T), push rows = inner index (B)
    gb_csr_view pv, sv;
    if (d.tran1) {
        gb_get_csr(pv, B);
        gb_get_csc(sv, B);
    } else {
        gb_get_csc(pv, B);
        gb_get_csr(sv, B);
    }
    const bool square = bc == inner;
    const int64_t dir = gb_knob("colbits_direction");  // 0 auto, 1 pull, 2 push
    if (!A->cw) to_cw(A, sv.rowptr, inner, sv.rowptr);
    if (M && !M->cw) to_cw(M, nullptr, 0, nullptr);
    if (!A->hint_valid || A->hint_key != (const void *)sv.rowptr) {
        hipLaunchKernelGGL(k_cw_hint, dim3(cb_grid(inner, 1024)), dim3(CB_BLOCK), 0, gb_stream(), A->cw, inner,
                           sv.rowptr, A->cw_stat, grid_state(0));
        GB_LAUNCH_CHECK();
        A->hint_valid = true;
        A->hint_key = sv.rowptr;
    }
    const int64_t onw = bc + gb_words(bc) + 1;  // words, then the summary bitmap
    uint64_t *out = gb_malloc_n<uint64_t>(onw);
    int64_t *stat = gb_malloc_n<int64_t>(4);
    uint8_t *oval = (uint8_t *)gb_malloc(1);
    GB_HIP(hipMemsetAsync(out, 0, onw * sizeof(uint64_t), gb_stream()));
    int64_t H = gb_knob("colbits_hub");
    if (H <= 0) H = 512;
    gb_view_hubs(pv, B, d.tran1 ? 0 : 1, H);
    if (dir != 1) gb_view_hubs(sv, B, d.tran1 ? 1 : 0, H);
    if (!C->pub) C->pub = gb_host_slot_alloc();
    const uint64_t seq = gb_next_pub_seq(C->pub);

    cb_step_args a{};
    a.nout = bc;
    a.nin = inner;
    a.nnz = sv.nvals;
    a.F = A->cw;
    a.prp = pv.rowptr;
    a.pci = pv.colidx;
    a.srp = dir == 1 ? nullptr : sv.rowptr;
    a.sci = dir == 1 ? nullptr : sv.colidx;
    a.M = M ? M->cw : nullptr;
    a.m_iso = (M && !d.structure && M->iso) ? M->cw_vals : nullptr;
    a.m_iso_code = M ? M->type->code : GBAMD_T_BOOL;
    a.comp = d.comp;
    a.full = k == 64 ? ~0ULL : ((1ULL << k) - 1);
    a.out = out;
    a.stat_in = A->cw_stat;
    int64_t alpha = gb_knob("colbits_alpha");
    a.alpha = alpha > 0 ? alpha : 8;
    a.dir = (int)dir;
    a.serial = gb_knob("colbits_serial") == 1;
    a.stat_out = stat;
    a.gst = grid_state(0);
    a.gst2 = grid_state(1);
    a.pub = gb_host_slot_device(C->pub);
    a.seq = (long long)seq;
    a.a_val = (uses_a && A->iso) ? (const uint8_t *)A->cw_vals : nullptr;
    a.b_val = (uses_b && B->iso) ? (const uint8_t *)B->vals : nullptr;
    a.mul = mul;
    a.out_val = oval;
    a.S_in = A->cw + inner;
    a.S_out = out + bc;
    a.p_tab = pv.hubs;
    a.p_nhub = pv.hubs ? pv.nhubs : 0;
    a.s_tab = (dir != 1) ? sv.hubs : nullptr;
    a.s_nhub = (dir != 1 && sv.hubs) ? sv.nhubs : 0;
    a.H = H;
    // pulls on a large graph read the in-edge sources' words through the hot-column relabel
    // (gb_view_hot): the most frequent sources' words are packed first, L2-resident
    uint64_t *Fhot = nullptr;
    if (dir != 2 && gb_knob("colbits_hot") != 1) {
        gb_view_hot(pv, B, d.tran1 ? 0 : 1);
        if (pv.hcolidx) {
            Fhot = gb_malloc_n<uint64_t>(pv.nhot);
            hipLaunchKernelGGL(k_cw_hot_gather, dim3(cb_grid(pv.nhot, 1024)), dim3(CB_BLOCK), 0, gb_stream(), a,
                               pv.hcols, pv.nhot, Fhot);
            GB_LAUNCH_CHECK();
            a.pci = pv.hcolidx;
            a.Fhot = Fhot;
        }
    }
    // enough waves to cover the output in a few chunks each; every block joins the grid sums
    const int64_t gcap = gb_knob("colbits_grid");
    hipLaunchKernelGGL(k_cw_step, dim3(cb_grid((bc > inner ? bc : inner), gcap > 0 ? (unsigned)gcap : 2048)),
                       dim3(CB_BLOCK), 0, gb_stream(), a);
    GB_LAUNCH_CHECK();
    gb_free(Fhot);  // stream-ordered

    // install into C (stream-ordered frees: the kernel has read A/M before they go)
    if (C->kind == GB_KIND_MATRIX && !C->cw) {
        gb_drop_transpose(C);
        gb_free(C->rowptr);
        gb_free(C->colidx);
        gb_free(C->vals);
        C->rowptr = nullptr;
        C->colidx = nullptr;
        C->vals = nullptr;
    } else {
        drop_layers(C);
        gb_free(C->cw);
        gb_free(C->cw_vals);
        gb_free(C->cw_stat);
    }
    C->cw = out;
    C->cw_vals = oval;
    C->cw_stat = stat;
    C->iso = true;
    C->nvals_valid = false;
    C->hint_valid = square && a.srp != nullptr;
    C->hint_key = sv.rowptr;
    C->pub_seq = seq;
    C->pub_epoch = gb_epoch();
    return true;
}

// ================================================================== C<M> = x, C of <= 64 rows
bool gb_colbits_assign_scalar(GB_Obj *C, GB_Obj *M, GrB_BinaryOp accum, const void *x, int xcode,
                              const GrB_Index *I, const GrB_Index *J, const gb_desc &d) {
    const int64_t knob = gb_knob("colbits");
    if (knob == 2 || accum || I != GrB_ALL || J != GrB_ALL || !M || d.comp || d.replace) return false;
    if (!small_rows(C) || !small_rows(M) || M->nrows != C->nrows || M->ncols != C->ncols) return false;
    if (C->type->code >= GBAMD_T_COUNT || M->type->code >= GBAMD_T_COUNT) return false;
    // auto: when either side already is column words, or the matrix is wide (the general
    // path materialises every index pair of a whole-matrix assign)
    if (knob == 0 && !C->cw && !M->cw && C->ncols < 4096) return false;
    const int64_t k = C->nrows, n = C->ncols;
    const int vs = (int)C->type->size;
    if ((double)k * (double)n * vs > 64e9) return false;
    unsigned long long xv = 0;
    gb_with_type(C->type->code, [&](auto z) {
        using D = decltype(z);
        gb_with_type(xcode, [&](auto y) {
            using S = decltype(y);
            S s;
            memcpy(&s, x, sizeof(S));
            D dv = gb_cast<D, S>(s);
            memcpy(&xv, &dv, sizeof(D));
        });
    });
    if (!M->cw) to_cw(M, nullptr, 0, nullptr);
    if (!C->cw) to_cw(C, nullptr, 0, nullptr);
    cw_expand(C);
    const bool value_mask = !d.structure;
    const void *m_iso = (value_mask && M->iso) ? M->cw_vals : nullptr;
    if (value_mask && !M->iso) {
        // a value mask with per-entry values: read them, stamp eagerly
        gb_cw_materialize(M);
        gb_cw_materialize(C);
        hipLaunchKernelGGL(k_cw_assign, dim3(cb_grid(n, 2048)), dim3(CB_BLOCK), 0, gb_stream(), n, (int)k, M->cw,
                           nullptr, M->type->code, (const uint8_t *)M->cw_vals, (int)M->type->size, C->cw,
                           (uint8_t *)C->cw_vals, xv, vs, C->cw_stat, grid_state(0));
        GB_LAUNCH_CHECK();
    } else {
        // structural or iso-valued mask: OR the words in, record (mask words, x) as a layer
        size_t nl;
        {
            std::lock_guard<std::mutex> lk(g_layers_mu);
            nl = g_layers[C].size();
        }
        if (nl >= (size_t)CB_MAX_LAYERS || gb_knob("colbits_eager") == 1) {
            gb_cw_materialize(C);
            nl = 0;
        }
        const bool base_empty = nl == 0 && C->nvals_valid && C->nvals == 0;
        uint64_t *L = gb_malloc_n<uint64_t>(n > 0 ? n : 1);
        hipLaunchKernelGGL(k_cw_assign_layer, dim3(cb_grid(n, 2048)), dim3(CB_BLOCK), 0, gb_stream(), n, M->cw, m_iso,
                           M->type->code, C->cw, L, C->cw_stat, grid_state(0));
        GB_LAUNCH_CHECK();
        {
            std::lock_guard<std::mutex> lk(g_layers_mu);
            if (base_empty) g_layers[C].push_back({nullptr, 0});
            g_layers[C].push_back({L, xv});
        }
        if (gb_knob("colbits_eager") == 1) gb_cw_materialize(C);
    }
    C->nvals_valid = false;
    C->pub_seq = 0;
    C->hint_valid = false;
    return true;
}

// ================================================================== device access (frontier exchange)
extern "C" {

GrB_Info GxB_Matrix_colwords_view(uint64_t **words, GrB_Index *nwords, GrB_Matrix A) {
    if (!words || !nwords) return GrB_NULL_POINTER;
    return gb_api(OBJ(A), [&] {
        GB_Obj *o = gb_obj_check_raw(A);
        GB_REQUIRE(small_rows(o), GrB_INVALID_VALUE, "column words need a matrix of 1 to 64 rows");
        if (!o->cw) to_cw(o, nullptr, 0, nullptr);
        *words = o->cw;
        *nwords = (GrB_Index)o->ncols;
    });
}

GrB_Info GxB_Matrix_colwords_touch(GrB_Matrix A) {
    return gb_api(OBJ(A), [&] {
        GB_Obj *o = gb_obj_check_raw(A);
        GB_REQUIRE(o->cw, GrB_INVALID_OBJECT, "matrix is not in column-word format");
        gb_cw_materialize(o);  // (pending stamps are replaced below when the matrix is not iso)
        if (!o->iso) {  // every entry written through the view carries the value 1
            const int vs = (int)o->type->size;
            char one[16] = {0};
            gb_with_type(o->type->code, [&](auto z) {
                using T = decltype(z);
                T v = gb_cast<T, bool>(true);
                memcpy(one, &v, sizeof(T));
            });
            void *nv = gb_malloc(vs);
            gb_copy_h2d(nv, one, vs);
            gb_free(o->cw_vals);
            o->cw_vals = nv;
            o->iso = true;
        }
        if (!o->pub) o->pub = gb_host_slot_alloc();
        const uint64_t seq = gb_next_pub_seq(o->pub);
        const int64_t n = o->ncols;
        hipLaunchKernelGGL(k_cw_recount, dim3(cb_grid(n, 2048)), dim3(CB_BLOCK), 0, gb_stream(), o->cw, n, o->cw + n,
                           o->cw_stat, grid_state(0), gb_host_slot_device(o->pub), (long long)seq);
        GB_LAUNCH_CHECK();
        o->nvals_valid = false;
        o->hint_valid = false;
        o->pub_seq = seq;
        o->pub_epoch = gb_epoch();
    });
}

}  // extern "C"
