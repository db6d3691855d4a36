// gb_spgemm_hash.hip -- Gustavson SpGEMM with hash accumulation, the default
// kernel behind unmasked / complement-masked GrB_mxm (replaces SuiteSparse's
// GB_AxB_saxpy3 hash method reached from reference core/matrix.py:2241).
//
// C(i,:) = sum_k A(i,k) * B(k,:) is accumulated per output row in a hash table
// keyed by column:
//   1. flops(i) = sum over A(i,:) of |B(k,:)|                  (k_row_flops)
//   2. symbolic: distinct columns per row -> C's row pointers   (keys only)
//   3. numeric: keys + values, occupied slots written at rowptr[i] unsorted
//   4. segmented sort of every row by column                    (hipcub)
// Rows are binned by their table need so every table lives in the fastest
// memory that holds it: one wave per row with a private LDS table (small
// rows), one workgroup per row with an LDS table (medium rows), or one
// workgroup per row with a table in HBM sized 2x the row (large rows; the
// table of a row being worked on stays hot in the XCD's L2).
// Products are streamed as one flat list per row: the lanes of a wave (or the
// threads of a workgroup) take 64 (256) consecutive products, locating their
// B row by a search over the prefix sum of the row lengths, so a row of A with
// a few hub neighbours keeps every lane busy (coalesced colidx / value reads).
// Values are accumulated with atomics over monoid-identity-initialised slots
// (native LDS/HBM atomics for plus / min / max on 32/64-bit, CAS otherwise; ANY
// keeps the value of whichever product claimed the key), so integer / boolean
// semirings are bit-exact and floating plus / times are exact up to summation
// order (the fp64 tolerance of BASELINE.json's north_star).  The
// expand-sort-compress path of gb_mxm.hip folds in ascending k instead and is
// kept as the deterministic alternative (knob spgemm_method = 1).
#include <algorithm>
#include <type_traits>
#include <vector>

#include <hipcub/hipcub.hpp>

#include "gb_dispatch.cuh"
#include "gb_internal.h"

namespace {

constexpr int HB = 256;                 // workgroup of the wave-bin and block-bin kernels
constexpr int HG = 1024;                // workgroup of the large-table kernels
constexpr int TW_SYM = 1024, TW_NUM = 512;        // per-wave LDS table slots
constexpr int TB_SYM = 8192, TB_NUM = 4096;       // per-workgroup (HB) LDS table slots
constexpr int TL_SYM = 16384, TL_NUM = 8192;      // per-workgroup (HG) LDS table slots
constexpr uint32_t HMUL = 0x9E3779B1u;

template <class Z>
using slot_of = typename std::conditional<sizeof(Z) == 8, unsigned long long, unsigned int>::type;

template <class Z, class S>
__device__ __forceinline__ S to_slot(Z z) {
    S s = 0;
    __builtin_memcpy(&s, &z, sizeof(Z));
    return s;
}
template <class Z, class S>
__device__ __forceinline__ Z from_slot(S s) {
    Z z;
    __builtin_memcpy(&z, &s, sizeof(Z));
    return z;
}

// identity of the monoid in Z; false for ANY (no identity: the claiming product's value is kept).
// fp PLUS uses -0.0 (exact identity of IEEE addition), fp MIN/MAX use NaN (identity of the
// NaN-ignoring fmin/fmax the monoids are defined with).
template <class Z>
__device__ __forceinline__ bool mon_identity(int mon, Z &id) {
    constexpr bool fl = std::is_floating_point<Z>::value;
    switch (mon) {
    case GBAMD_MON_PLUS: id = fl ? (Z)(-0.0) : (Z)0; return true;
    case GBAMD_MON_TIMES: id = (Z)1; return true;
    case GBAMD_MON_MIN:
        if constexpr (fl) id = (Z)__builtin_nan("");
        else id = gb_tmax<Z>();
        return true;
    case GBAMD_MON_MAX:
        if constexpr (fl) id = (Z)__builtin_nan("");
        else id = gb_tmin<Z>();
        return true;
    case GBAMD_MON_LOR: case GBAMD_MON_LXOR: id = (Z)0; return true;
    case GBAMD_MON_LAND: case GBAMD_MON_LXNOR: id = (Z)1; return true;
    case GBAMD_MON_BOR: case GBAMD_MON_BXOR:
        id = (Z)0;
        return true;
    case GBAMD_MON_BAND: case GBAMD_MON_BXNOR:
        if constexpr (gb_traits<Z>::is_int) id = (Z)~(Z)0;
        else id = (Z)0;
        return true;
    default: return false;  // ANY
    }
}

// slot <- slot (+) z, atomically (LDS or global memory)
template <class SR, class Z, class S>
__device__ __forceinline__ void slot_accum(const SR &sr, int mon, S *slot, Z z) {
    if constexpr (std::is_same<Z, double>::value || std::is_same<Z, float>::value) {
        if (mon == GBAMD_MON_PLUS) {
            atomicAdd((Z *)slot, z);
            return;
        }
    } else if constexpr (sizeof(Z) >= 4 && gb_traits<Z>::is_int) {
        if (mon == GBAMD_MON_PLUS) {  // two's complement wrap == unsigned add
            atomicAdd((S *)slot, (S)z);
            return;
        }
        if (mon == GBAMD_MON_MIN || mon == GBAMD_MON_MAX) {
            using I = typename std::conditional<sizeof(Z) == 8,
                                                typename std::conditional<std::is_signed<Z>::value, long long,
                                                                          unsigned long long>::type,
                                                typename std::conditional<std::is_signed<Z>::value, int,
                                                                          unsigned int>::type>::type;
            if (mon == GBAMD_MON_MIN) atomicMin((I *)slot, (I)z);
            else atomicMax((I *)slot, (I)z);
            return;
        }
    }
    S old = *(volatile S *)slot;
    while (true) {
        const Z cur = from_slot<Z, S>(old);
        if (sr.terminal(cur)) return;
        const S nv = to_slot<Z, S>(sr.add(cur, z));
        if (nv == old) return;
        const S prev = atomicCAS(slot, old, nv);
        if (prev == old) return;
        old = prev;
    }
}

// insert column j; returns the slot, `claimed` = this call created the key
__device__ __forceinline__ uint32_t h_insert(int32_t *keys, int32_t j, int shift, uint32_t mask, bool &claimed) {
    uint32_t h = ((uint32_t)j * HMUL) >> shift;
    while (true) {
        int32_t cur = *(volatile int32_t *)(keys + h);
        if (cur == j) {
            claimed = false;
            return h;
        }
        if (cur == -1) {
            cur = atomicCAS(keys + h, -1, j);
            if (cur == -1) {
                claimed = true;
                return h;
            }
            if (cur == j) {
                claimed = false;
                return h;
            }
        }
        h = (h + 1) & mask;
    }
}

template <class T>
__device__ __forceinline__ T shfl_idx(T v, int src) {
    if constexpr (sizeof(T) == 8) {
        long long x;
        __builtin_memcpy(&x, &v, 8);
        x = __shfl(x, src, 64);
        T r;
        __builtin_memcpy(&r, &x, 8);
        return r;
    } else {
        int x = 0;
        __builtin_memcpy(&x, &v, sizeof(T));
        x = __shfl(x, src, 64);
        T r;
        __builtin_memcpy(&r, &x, sizeof(T));
        return r;
    }
}

__device__ __forceinline__ int log2i(uint32_t t) { return 31 - __builtin_clz(t); }

// one product: key insert, then (numeric) the value update
template <bool SYM, bool VALS, class SR, class X, class Z, class S>
__device__ __forceinline__ void h_product(const SR &sr, int mon, int32_t *keys, S *vals, int shift, uint32_t mask,
                                          int64_t i, int32_t k, int32_t j, X av, const X *__restrict__ bvx,
                                          bool b_iso, bool rv, int64_t pb, int &nclaim) {
    bool claimed;
    const uint32_t h = h_insert(keys, j, shift, mask, claimed);
    if constexpr (SYM) {
        nclaim += claimed ? 1 : 0;
    } else if constexpr (VALS) {
        X bv = X();
        if (rv) bv = bvx[b_iso ? 0 : pb];
        const Z z = sr.mult(av, bv, i, k, j);
        if (mon == GBAMD_MON_ANY) {
            if (claimed) vals[h] = to_slot<Z, S>(z);
        } else {
            slot_accum<SR, Z, S>(sr, mon, vals + h, z);
        }
    }
}

// ------------------------------------------------------------------ wave per row (LDS)
template <bool SYM, bool VALS, class SR, class X, class Z, int TW>
__global__ __launch_bounds__(HB) void k_hash_wave(
    SR sr, int mon, const int32_t *__restrict__ rows, int64_t nr, const int64_t *__restrict__ arp,
    const int32_t *__restrict__ aci, const X *__restrict__ avx, bool a_iso, const int64_t *__restrict__ brp,
    const int32_t *__restrict__ bci, const X *__restrict__ bvx, bool b_iso, int64_t *__restrict__ cnt,
    const int64_t *__restrict__ crp, int32_t *__restrict__ cci, Z *__restrict__ cvx) {
    using S = slot_of<Z>;
    constexpr bool NV = !SYM && VALS;
    __shared__ int32_t skeys[HB / 64][TW];
    __shared__ S svals[NV ? HB / 64 : 1][NV ? TW : 1];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    int32_t *keys = skeys[w];
    S *vals = svals[NV ? w : 0];
    constexpr int shift = 32 - __builtin_ctz(TW);
    const bool rv = SR::reads_values && avx && bvx;
    Z idv = Z();
    const bool has_id = NV ? mon_identity<Z>(mon, idv) : false;
    const S ids = to_slot<Z, S>(idv);
    for (int64_t r = (int64_t)blockIdx.x * (HB / 64) + w; r < nr; r += (int64_t)gridDim.x * (HB / 64)) {
        const int64_t i = rows[r];
        for (int s = lane; s < TW; s += 64) {
            keys[s] = -1;
            if (NV && has_id) vals[s] = ids;
        }
        int nclaim = 0;
        const int64_t a0 = arp[i], a1 = arp[i + 1];
        for (int64_t g = a0; g < a1; g += 64) {
            const int64_t p = g + lane;
            const bool v = p < a1;
            const int32_t k = v ? aci[p] : 0;
            const int64_t b0 = v ? brp[k] : 0;
            const int64_t len = v ? brp[k + 1] - b0 : 0;
            X av = X();
            if (rv && v) av = avx[a_iso ? 0 : p];
            int64_t inc = len;
#pragma unroll
            for (int off = 1; off < 64; off <<= 1) {
                const int64_t t = __shfl_up(inc, off, 64);
                if (lane >= off) inc += t;
            }
            const int64_t excl = inc - len;
            const int64_t G = __shfl(inc, 63, 64);
            for (int64_t t0 = 0; t0 < G; t0 += 64) {
                const int64_t t = t0 + lane;
                int s = 0;
#pragma unroll
                for (int st = 32; st > 0; st >>= 1)
                    if (__shfl(excl, s + st, 64) <= t) s += st;
                const int64_t es = __shfl(excl, s, 64), bs = __shfl(b0, s, 64);
                const int32_t ks = __shfl(k, s, 64);
                const X as = shfl_idx(av, s);
                if (t < G) {
                    const int64_t pb = bs + (t - es);
                    h_product<SYM, VALS, SR, X, Z, S>(sr, mon, keys, vals, shift, TW - 1, i, ks, bci[pb], as, bvx,
                                                      b_iso, rv, pb, nclaim);
                }
            }
        }
        if constexpr (SYM) {
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) nclaim += __shfl_xor(nclaim, off, 64);
            if (lane == 0) cnt[i] = nclaim;
        } else {
            int64_t pos = crp[i];
            for (int s0 = 0; s0 < TW; s0 += 64) {
                const int32_t kj = keys[s0 + lane];
                const bool occ = kj >= 0;
                const uint64_t bal = __ballot(occ);
                if (occ) {
                    const int64_t o = pos + __popcll(bal & ((1ULL << lane) - 1));
                    cci[o] = kj;
                    if (NV) cvx[o] = from_slot<Z, S>(vals[s0 + lane]);
                }
                pos += __popcll(bal);
            }
        }
    }
}

// ------------------------------------------------------------------ workgroup per row (LDS table)
// Table in dynamic LDS: 2^logT int32 keys, then (numeric) 2^logT value slots.
template <bool SYM, bool VALS, class SR, class X, class Z, int BS>
__global__ __launch_bounds__(BS) void k_hash_block(
    SR sr, int mon, const int32_t *__restrict__ rows, int64_t nr, int logT, const int64_t *__restrict__ arp, const int32_t *__restrict__ aci, const X *__restrict__ avx, bool a_iso,
    const int64_t *__restrict__ brp, const int32_t *__restrict__ bci, const X *__restrict__ bvx, bool b_iso,
    int64_t *__restrict__ cnt, const int64_t *__restrict__ crp, int32_t *__restrict__ cci, Z *__restrict__ cvx) {
    using S = slot_of<Z>;
    constexpr bool NV = !SYM && VALS;
    constexpr int NW = BS / 64;
    extern __shared__ __align__(16) char smem[];
    __shared__ int64_t s_excl[BS + 1];
    __shared__ int64_t s_b0[BS];
    __shared__ int32_t s_k[BS];
    __shared__ X s_av[BS];
    __shared__ int64_t s_wsum[NW];
    __shared__ int64_t s_pos;
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
    const bool rv = SR::reads_values && avx && bvx;
    Z idv = Z();
    const bool has_id = NV ? mon_identity<Z>(mon, idv) : false;
    const S ids = to_slot<Z, S>(idv);
    for (int64_t r = blockIdx.x; r < nr; r += gridDim.x) {
        const int64_t i = rows[r];
        const int lT = logT;
        int32_t *keys = (int32_t *)smem;
        S *vals = (S *)(smem + ((size_t)4 << lT));
        const int64_t T = 1LL << lT;
        const int shift = 32 - lT;
        for (int64_t s = tid; s < T; s += BS) {
            keys[s] = -1;
            if (NV && has_id) vals[s] = ids;
        }
        if (tid == 0) s_pos = crp ? crp[i] : 0;
        __syncthreads();
        int nclaim = 0;
        const int64_t a0 = arp[i], a1 = arp[i + 1];
        for (int64_t g = a0; g < a1; g += BS) {
            const int64_t p = g + tid;
            const bool v = p < a1;
            const int32_t k = v ? aci[p] : 0;
            const int64_t b0 = v ? brp[k] : 0;
            const int64_t len = v ? brp[k + 1] - b0 : 0;
            X av = X();
            if (rv && v) av = avx[a_iso ? 0 : p];
            int64_t inc = len;
#pragma unroll
            for (int off = 1; off < 64; off <<= 1) {
                const int64_t t = __shfl_up(inc, off, 64);
                if (lane >= off) inc += t;
            }
            if (lane == 63) s_wsum[w] = inc;
            __syncthreads();
            int64_t wbase = 0;
            for (int q = 0; q < w; q++) wbase += s_wsum[q];
            s_excl[tid] = wbase + inc - len;
            s_b0[tid] = b0;
            s_k[tid] = k;
            s_av[tid] = av;
            if (tid == BS - 1) s_excl[BS] = wbase + inc;
            __syncthreads();
            const int64_t G = s_excl[BS];
            for (int64_t t0 = 0; t0 < G; t0 += BS) {
                const int64_t t = t0 + tid;
                if (t < G) {
                    int s = 0;
#pragma unroll
                    for (int st = BS / 2; st > 0; st >>= 1)
                        if (s_excl[s + st] <= t) s += st;
                    const int64_t pb = s_b0[s] + (t - s_excl[s]);
                    h_product<SYM, VALS, SR, X, Z, S>(sr, mon, keys, vals, shift, (uint32_t)(T - 1), i, s_k[s],
                                                      bci[pb], s_av[s], bvx, b_iso, rv, pb, nclaim);
                }
            }
            __syncthreads();
        }
        if constexpr (SYM) {
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) nclaim += __shfl_xor(nclaim, off, 64);
            if (lane == 0) s_wsum[w] = nclaim;
            __syncthreads();
            if (tid == 0) {
                int64_t c = 0;
                for (int q = 0; q < NW; q++) c += s_wsum[q];
                cnt[i] = c;
            }
        } else {
            __syncthreads();
            for (int64_t s0 = 0; s0 < T; s0 += BS) {
                const int64_t s = s0 + tid;
                const int32_t kj = s < T ? keys[s] : -1;
                const bool occ = kj >= 0;
                const uint64_t bal = __ballot(occ);
                int64_t base = 0;
                if (lane == 0 && bal) base = atomicAdd((unsigned long long *)&s_pos, (unsigned long long)__popcll(bal));
                base = __shfl(base, 0, 64);
                if (occ) {
                    const int64_t o = base + __popcll(bal & ((1ULL << lane) - 1));
                    cci[o] = kj;
                    if (NV) cvx[o] = from_slot<Z, S>(vals[s]);
                }
            }
        }
        __syncthreads();
    }
}

// ------------------------------------------------------------------ workgroup per row (column windows)
// Rows too large for an LDS hash table.  The row is swept in column windows
// [c0, c0 + W): a presence bitmap of the window in LDS is set by every
// product whose column falls in it (each B row's part of the window is a
// contiguous range, found by galloping from a per-entry cursor), then
//  * symbolic: the window's distinct columns are counted (popcount);
//  * numeric: the set bits are written out in column order (C's colidx comes
//    out sorted), and every product adds into the value at its column's rank
//    in the window (prefix popcounts): in LDS when the window holds <= vcap
//    entries, else with HBM atomics straight into C's values.
// Empty stretches of columns are skipped: the next window starts at the
// smallest column any cursor points at.
__device__ __forceinline__ int64_t gallop_lb(const int32_t *__restrict__ ci, int64_t lo, int64_t hi, int32_t key) {
    // first position in [lo, hi) with ci[pos] >= key
    if (lo >= hi || ci[lo] >= key) return lo;
    int64_t a = lo, step = 1;  // ci[a] < key
    while (a + step < hi && ci[a + step] < key) {
        a += step;
        step <<= 1;
    }
    int64_t b = a + step < hi ? a + step : hi;  // ci[b] >= key or b == hi
    while (b - a > 1) {
        const int64_t m = (a + b) >> 1;
        if (ci[m] < key) a = m;
        else b = m;
    }
    return b;
}

template <bool SYM, bool VALS, class SR, class X, class Z>
__global__ __launch_bounds__(HG) void k_row_window(
    SR sr, int mon, const int32_t *__restrict__ rows, int64_t nr, int logW, int vcap, int in_c_groups,
    int64_t *__restrict__ cur,
    const int64_t *__restrict__ arp, const int32_t *__restrict__ aci, const X *__restrict__ avx, bool a_iso,
    const int64_t *__restrict__ brp, const int32_t *__restrict__ bci, const X *__restrict__ bvx, bool b_iso,
    int64_t ncols, int64_t *__restrict__ cnt, const int64_t *__restrict__ crp, int32_t *__restrict__ cci,
    Z *__restrict__ cvx) {
    using S = slot_of<Z>;
    constexpr bool NV = !SYM && VALS;
    constexpr int NW = HG / 64;
    extern __shared__ __align__(16) char smem[];
    const int W = 1 << logW;        // columns per window (multiple of 256)
    const int NWD = W >> 5;         // bitmap words
    uint32_t *bm = (uint32_t *)smem;
    int32_t *prew = (int32_t *)(smem + (size_t)NWD * 4);  // numeric: exclusive popcount prefix per word
    S *vals = (S *)(smem + (size_t)NWD * 8);              // numeric with values: [vcap] (32-B aligned)
    __shared__ int64_t s_excl[HG + 1];
    __shared__ int64_t s_lo[HG];
    __shared__ int32_t s_k[HG];
    __shared__ X s_av[HG];
    __shared__ int64_t s_wsum[NW];
    __shared__ int32_t s_wmin[NW];
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
    const bool rv = SR::reads_values && avx && bvx;
    Z idv = Z();
    const bool has_id = NV ? mon_identity<Z>(mon, idv) : false;
    const S ids = to_slot<Z, S>(idv);

    auto block_min = [&](int32_t v) -> int32_t {
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
            const int32_t o = __shfl_xor(v, off, 64);
            v = o < v ? o : v;
        }
        __syncthreads();
        if (lane == 0) s_wmin[w] = v;
        __syncthreads();
        int32_t m = s_wmin[0];
        for (int q = 1; q < NW; q++) m = s_wmin[q] < m ? s_wmin[q] : m;
        return m;
    };
    auto block_sum = [&](int64_t v) -> int64_t {
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
        __syncthreads();
        if (lane == 0) s_wsum[w] = v;
        __syncthreads();
        int64_t m = 0;
        for (int q = 0; q < NW; q++) m += s_wsum[q];
        return m;
    };

    for (int64_t r = blockIdx.x; r < nr; r += gridDim.x) {
        const int64_t i = rows[r];
        const int64_t a0 = arp[i], a1 = arp[i + 1];
        int32_t nmin = 0x7fffffff;
        for (int64_t p = a0 + tid; p < a1; p += HG) {
            const int32_t k = aci[p];
            const int64_t b0 = brp[k];
            cur[p] = b0;
            if (b0 < brp[k + 1]) nmin = bci[b0] < nmin ? bci[b0] : nmin;
        }
        int32_t c0 = block_min(nmin);
        int64_t count = 0;
        int64_t outpos = SYM ? 0 : crp[i];
        while (c0 < ncols) {
            const int64_t c1 = (int64_t)c0 + W;
            for (int q = tid; q < NWD; q += HG) bm[q] = 0u;
            __syncthreads();
            // products with columns in [cursor, cend), group by group of A entries; f(t-th product)
            // for each; advance: move the cursors to cend and return the smallest column left
            auto sweep = [&](auto &&f, int64_t cend, bool advance) {
                int32_t mn = 0x7fffffff;
                for (int64_t g = a0; g < a1; g += HG) {
                    const int64_t p = g + tid;
                    const bool v = p < a1;
                    int32_t k = 0;
                    int64_t lo = 0, hi = 0;
                    X av = X();
                    if (v) {
                        k = aci[p];
                        lo = cur[p];
                        const int64_t end = brp[k + 1];
                        hi = gallop_lb(bci, lo, end, cend > 0x7fffffff ? 0x7fffffff : (int32_t)cend);
                        if (cend > 0x7fffffff) hi = end;
                        if (advance) {
                            cur[p] = hi;
                            if (hi < end) mn = bci[hi] < mn ? bci[hi] : mn;
                        }
                        if (rv) av = avx[a_iso ? 0 : p];
                    }
                    const int64_t len = hi - lo;
                    int64_t inc = len;
#pragma unroll
                    for (int off = 1; off < 64; off <<= 1) {
                        const int64_t t = __shfl_up(inc, off, 64);
                        if (lane >= off) inc += t;
                    }
                    if (lane == 63) s_wsum[w] = inc;
                    __syncthreads();
                    int64_t wbase = 0;
                    for (int q = 0; q < w; q++) wbase += s_wsum[q];
                    s_excl[tid] = wbase + inc - len;
                    s_lo[tid] = lo;
                    s_k[tid] = k;
                    s_av[tid] = av;
                    if (tid == HG - 1) s_excl[HG] = wbase + inc;
                    __syncthreads();
                    const int64_t G = s_excl[HG];
                    for (int64_t t0 = 0; t0 < G; t0 += HG) {
                        const int64_t t = t0 + tid;
                        if (t < G) {
                            int s = 0;
#pragma unroll
                            for (int st = HG / 2; st > 0; st >>= 1)
                                if (s_excl[s + st] <= t) s += st;
                            const int64_t pb = s_lo[s] + (t - s_excl[s]);
                            f(pb, s_k[s], s_av[s]);
                        }
                    }
                    __syncthreads();
                }
                return mn;
            };
            // ---- presence bits
            int32_t mn = sweep(
                [&](int64_t pb, int32_t, X) {
                    const int32_t c = bci[pb] - c0;
                    atomicOr(bm + (c >> 5), 1u << (c & 31));
                },
                c1, SYM || !VALS);
            __syncthreads();
            if constexpr (SYM) {
                int64_t mine = 0;
                for (int q = tid; q < NWD; q += HG) mine += __popc(bm[q]);
                count += block_sum(mine);
            } else {
                // ---- exclusive popcount prefix per word (each thread a run of `per` words)
                const int per = (NWD + HG - 1) / HG;
                const int q0 = tid * per < NWD ? tid * per : NWD;
                const int q1 = q0 + per < NWD ? q0 + per : NWD;
                int32_t s = 0;
                for (int q = q0; q < q1; q++) s += __popc(bm[q]);
                int32_t inc = s;
#pragma unroll
                for (int off = 1; off < 64; off <<= 1) {
                    const int32_t t = __shfl_up(inc, off, 64);
                    if (lane >= off) inc += t;
                }
                if (lane == 63) s_wsum[w] = inc;
                __syncthreads();
                int32_t run = inc - s;
                int64_t m = 0;
                for (int q = 0; q < NW; q++) {
                    if (q < w) run += (int32_t)s_wsum[q];
                    m += s_wsum[q];
                }
                for (int q = q0; q < q1; q++) {
                    prew[q] = run;
                    run += __popc(bm[q]);
                }
                __syncthreads();
                // sorted columns of the window: a wave per 64-column stretch, ballot + prefix
                for (int q = w * 2; q < NWD; q += NW * 2) {
                    const uint64_t bits = (uint64_t)bm[q] | ((uint64_t)bm[q + 1] << 32);
                    if ((bits >> lane) & 1ULL)
                        cci[outpos + prew[q] + __popcll(bits & ((1ULL << lane) - 1))] = c0 + q * 32 + lane;
                }
                if constexpr (VALS) {
                    // value groups of < vcap entries (see the kernel comment)
                    const int NB = W >> 8;
                    const int64_t G = vcap - 256;
                    auto chunk_pre = [&](int b) -> int64_t { return b < NB ? (int64_t)prew[b * 8] : m; };
                    auto first_chunk = [&](int64_t key) {  // first b in [0, NB) with chunk_pre(b) >= key, else NB
                        int lo = 0, hi = NB;
                        while (lo < hi) {
                            const int mid = (lo + hi) >> 1;
                            if (chunk_pre(mid) >= key) hi = mid;
                            else lo = mid + 1;
                        }
                        return lo;
                    };
                    // more than in_c_groups groups of LDS value slots and a slot as wide as a
                    // value: one sweep accumulating straight into C's values (this row's output
                    // range, L2-resident) instead of one sweep per group; 1-2-byte values use
                    // 4-byte slots and keep the grouped path
                    constexpr bool IN_C = sizeof(S) == sizeof(Z);
                    const int ngg = (int)(chunk_pre(NB - 1) / G) + 1;
                    const bool in_c = IN_C && ngg > in_c_groups;
                    const int ng = in_c ? 0 : ngg;
                    if (in_c) {
                        S *dst = (S *)(cvx + outpos);
                        if (has_id)
                            for (int64_t q = tid; q < m; q += HG) dst[q] = ids;
                        __syncthreads();
                        mn = sweep(
                            [&](int64_t pb, int32_t k, X av) {
                                const int32_t j = bci[pb];
                                X bv = X();
                                if (rv) bv = bvx[b_iso ? 0 : pb];
                                const Z z = sr.mult(av, bv, i, k, j);
                                const int32_t c = j - c0;
                                const int32_t rk = prew[c >> 5] + __popc(bm[c >> 5] & ((1u << (c & 31)) - 1u));
                                if (mon == GBAMD_MON_ANY) dst[rk] = to_slot<Z, S>(z);
                                else slot_accum<SR, Z, S>(sr, mon, dst + rk, z);
                            },
                            c1, true);
                        __syncthreads();
                    }
                    for (int g = 0; g < ng; g++) {
                        const int bs = first_chunk((int64_t)g * G), be = first_chunk((int64_t)(g + 1) * G);
                        const int64_t rbase = chunk_pre(bs), rcnt = chunk_pre(be) - rbase;
                        if (has_id)
                            for (int64_t q = tid; q < rcnt; q += HG) vals[q] = ids;
                        __syncthreads();
                        mn = sweep(
                            [&](int64_t pb, int32_t k, X av) {
                                const int32_t j = bci[pb];
                                X bv = X();
                                if (rv) bv = bvx[b_iso ? 0 : pb];
                                const Z z = sr.mult(av, bv, i, k, j);
                                const int32_t c = j - c0;
                                const int32_t rk =
                                    prew[c >> 5] + __popc(bm[c >> 5] & ((1u << (c & 31)) - 1u)) - (int32_t)rbase;
                                if (mon == GBAMD_MON_ANY) vals[rk] = to_slot<Z, S>(z);
                                else slot_accum<SR, Z, S>(sr, mon, vals + rk, z);
                            },
                            c0 + (int64_t)be * 256, true);
                        for (int64_t q = tid; q < rcnt; q += HG) cvx[outpos + rbase + q] = from_slot<Z, S>(vals[q]);
                        __syncthreads();
                    }
                }
                outpos += m;
            }
            c0 = block_min(mn);
        }
        if constexpr (SYM) {
            if (tid == 0) cnt[i] = count;
        }
        __syncthreads();
    }
}

// ------------------------------------------------------------------ binning
// bins: 0 empty, 1 wave (<= lim1), 2 workgroup HB (<= lim2), 3 workgroup HG (<= lim3), 4 HBM table
__global__ void k_bin_rows(const int64_t *__restrict__ size, int64_t n, int64_t lim1, int64_t lim2, int64_t lim3,
                           int64_t cap, int pass, unsigned long long *__restrict__ fill,
                           const int64_t *__restrict__ start, int32_t *__restrict__ rows) {
    const int lane = threadIdx.x & 63;
    for (int64_t i0 = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) - lane; i0 < n;
         i0 += (int64_t)gridDim.x * blockDim.x) {
        const int64_t i = i0 + lane;
        int b = -1;
        if (i < n) {
            int64_t sz = size[i];
            if (sz > cap) sz = cap;
            b = sz == 0 ? 0 : sz <= lim1 ? 1 : sz <= lim2 ? 2 : sz <= lim3 ? 3 : 4;
        }
        for (int q = 0; q < 5; q++) {
            const uint64_t m = __ballot(b == q);
            if (!m) continue;
            unsigned long long base = 0;
            const int leader = __builtin_ctzll(m);
            if (lane == leader) base = atomicAdd(&fill[q], (unsigned long long)__popcll(m));
            base = __shfl(base, leader, 64);
            if (pass == 1 && b == q) rows[start[q] + base + __popcll(m & ((1ULL << lane) - 1))] = (int32_t)i;
        }
    }
}

__global__ void k_zero_rows_cnt(const int32_t *__restrict__ rows, int64_t nr, int64_t *__restrict__ cnt) {
    for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < nr; r += (int64_t)gridDim.x * blockDim.x)
        cnt[rows[r]] = 0;
}

__global__ void k_sub_base(const int64_t *__restrict__ in, int64_t n, int64_t base, int64_t *__restrict__ out) {
    for (int64_t q = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; q < n; q += (int64_t)gridDim.x * blockDim.x)
        out[q] = in[q] - base;
}

template <class K>
void set_lds(K kernel, size_t bytes) {
    static size_t done = 0;  // per instantiation
    if (bytes > done) {
        GB_HIP(hipFuncSetAttribute((const void *)kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes));
        done = bytes;
    }
}

inline unsigned hgrid(int64_t work, int64_t per_block, int64_t cap = 65535) {
    int64_t g = (work + per_block - 1) / per_block;
    if (g < 1) g = 1;
    if (g > cap) g = cap;
    return (unsigned)g;
}

__global__ void k_seg_ends(const int64_t *__restrict__ rp, int64_t n, int64_t *__restrict__ ends) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        ends[i] = rp[i + 1];
}
__global__ void k_seg_skip(const int32_t *__restrict__ rows, int64_t nr, const int64_t *__restrict__ rp,
                           int64_t *__restrict__ ends) {
    for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < nr; r += (int64_t)gridDim.x * blockDim.x)
        ends[rows[r]] = rp[rows[r]];
}

}  // namespace

// C = A * B (no mask applied here): T gets sorted CSR rows.
void gb_spgemm_hash(gb_mat_result &T, gb_csr_view &A, gb_csr_view &B, GrB_Semiring sring, bool iso,
                    const void *av, const void *bv, const int64_t *flops) {
    gb_sr_info info = gb_sr_describe(sring);
    const int64_t nrows = A.nrows, ncols = B.ncols;
    const size_t zs = gb_type_size(info.zcode);
    const bool vals_needed = !iso;
    gb_scratch s;
    int64_t *cnt = s.get<int64_t>(nrows + 1);
    int32_t *rows = s.get<int32_t>(nrows);
    unsigned long long *fill = s.get<unsigned long long>(5);
    int64_t *start = s.get<int64_t>(5);
    int64_t *cur = nullptr;  // per-A-entry cursors of the window kernel
    T.rowptr = gb_malloc_n<int64_t>(nrows + 1);

    struct bins_t {
        int64_t c[5], st[5];
    };
    auto make_bins = [&](const int64_t *size, int64_t lim1, int64_t lim2, int64_t lim3) {
        bins_t b;
        const int64_t cap = ncols;  // a row never has more distinct columns than B
        if (gb_knob("hash_window") == 1) lim1 = lim2 = lim3 = 0;  // every row to the window kernel (tests)
        const unsigned g = hgrid(nrows, 256, 4096);
        gb_memset(fill, 0, 5 * sizeof(unsigned long long));
        hipLaunchKernelGGL(k_bin_rows, dim3(g), dim3(256), 0, gb_stream(), size, nrows, lim1, lim2, lim3, cap, 0,
                           fill, (const int64_t *)nullptr, (int32_t *)nullptr);
        GB_LAUNCH_CHECK();
        unsigned long long hc[5];
        gb_copy_d2h(hc, fill, sizeof(hc));
        int64_t acc = 0;
        for (int q = 0; q < 5; q++) {
            b.c[q] = (int64_t)hc[q];
            b.st[q] = acc;
            acc += b.c[q];
        }
        gb_copy_h2d(start, b.st, sizeof(b.st));
        gb_memset(fill, 0, 5 * sizeof(unsigned long long));
        hipLaunchKernelGGL(k_bin_rows, dim3(g), dim3(256), 0, gb_stream(), size, nrows, lim1, lim2, lim3, cap, 1,
                           fill, (const int64_t *)start, rows);
        GB_LAUNCH_CHECK();
        if (b.c[4] && !cur) cur = s.get<int64_t>(A.nvals + 1);
        return b;
    };
    // window width: a power of two >= 256 columns, no wider than needed for B
    auto win_log = [&](int maxlog) {
        int l = 8;
        while (l < maxlog && (1LL << l) < ncols) l++;
        return l;
    };

    gb_dispatch_sr(info, [&](auto srf, auto x, auto z) {
        using SRT = decltype(srf);
        using X = decltype(x);
        using Z = decltype(z);
        using S = slot_of<Z>;
        const X *ax = (const X *)av, *bx = (const X *)bv;
        const int mon = info.mon;

        // one phase over the bins; SYM counts into cnt, else writes rows: hash bins into (hci, hvx),
        // window rows (already in column order) into (wci, wvx)
        auto phase = [&](auto symc, auto valsc, const bins_t &b, int32_t *hci, Z *hvx, int32_t *wci, Z *wvx) {
            constexpr bool SYM = decltype(symc)::value;
            constexpr bool VALS = decltype(valsc)::value;
            constexpr int TW = SYM ? TW_SYM : TW_NUM;
            constexpr int TB = SYM ? TB_SYM : TB_NUM;
            constexpr int TL = SYM ? TL_SYM : TL_NUM;
            constexpr size_t slot_b = 4 + ((!SYM && VALS) ? sizeof(S) : 0);
            const int64_t *crp = SYM ? nullptr : T.rowptr;
            if (b.c[0] && SYM)
                hipLaunchKernelGGL(k_zero_rows_cnt, dim3(hgrid(b.c[0], 256, 4096)), dim3(256), 0, gb_stream(),
                                   rows + b.st[0], b.c[0], cnt);
            if (b.c[1])
                hipLaunchKernelGGL((k_hash_wave<SYM, VALS, SRT, X, Z, TW>), dim3(hgrid(b.c[1], HB / 64)), dim3(HB), 0,
                                   gb_stream(), srf, mon, rows + b.st[1], b.c[1], A.rowptr, A.colidx, ax, A.iso,
                                   B.rowptr, B.colidx, bx, B.iso, cnt, crp, hci, hvx);
            if (b.c[2]) {
                const size_t sh = slot_b * TB;
                set_lds(k_hash_block<SYM, VALS, SRT, X, Z, HB>, sh);
                hipLaunchKernelGGL((k_hash_block<SYM, VALS, SRT, X, Z, HB>), dim3(hgrid(b.c[2], 1)), dim3(HB), sh,
                                   gb_stream(), srf, mon, rows + b.st[2], b.c[2], __builtin_ctz(TB), A.rowptr,
                                   A.colidx, ax, A.iso, B.rowptr, B.colidx, bx, B.iso, cnt, crp, hci, hvx);
            }
            if (b.c[3]) {
                const size_t sh = slot_b * TL;
                set_lds(k_hash_block<SYM, VALS, SRT, X, Z, HG>, sh);
                hipLaunchKernelGGL((k_hash_block<SYM, VALS, SRT, X, Z, HG>), dim3(hgrid(b.c[3], 1)), dim3(HG), sh,
                                   gb_stream(), srf, mon, rows + b.st[3], b.c[3], __builtin_ctz(TL), A.rowptr,
                                   A.colidx, ax, A.iso, B.rowptr, B.colidx, bx, B.iso, cnt, crp, hci, hvx);
            }
            if (b.c[4]) {
                // symbolic: 2^19-column bitmap windows (64 KB); numeric: 2^17 columns (bitmap + word
                // prefixes 32 KB) with values in LDS in groups of < 8192 entries (64 KB for 8-byte
                // values; one-to-two-byte values: a group can hold the whole window)
                // narrow values: at least 512 columns, so a value group (vcap - 256 entries,
                // one 256-column chunk of headroom) is never empty
                const int lw = SYM ? win_log(19) : (sizeof(Z) < 4 ? std::max(9, win_log(13)) : win_log(17));
                int vcap = (SYM || !VALS) ? 0 : (sizeof(Z) < 4 ? (1 << lw) : 8192);
                // tests: a small LDS value capacity sends windows to the C-resident accumulation
                const int64_t kv = gb_knob("window_vcap");
                if (vcap && kv > 256 && kv < vcap) vcap = (int)kv;
                // grouped sweeps (one per vcap entries) up to this many, then C-resident accumulation
                const int64_t kg = gb_knob("window_in_c_groups");
                const int in_c_groups = kg > 0 ? (int)kg : 8;  // tools/sweep_in_c.sh: 2 226 ms, 4 208, 8 204, never 206 (config 5)
                const size_t sh = SYM ? (size_t)(1 << lw) / 8 : (size_t)(1 << lw) / 4 + (size_t)vcap * sizeof(S);
                set_lds(k_row_window<SYM, VALS, SRT, X, Z>, sh);
                hipLaunchKernelGGL((k_row_window<SYM, VALS, SRT, X, Z>), dim3(hgrid(b.c[4], 1, 2048)), dim3(HG), sh,
                                   gb_stream(), srf, mon, rows + b.st[4], b.c[4], lw, vcap, in_c_groups, cur, A.rowptr, A.colidx,
                                   ax, A.iso, B.rowptr, B.colidx, bx, B.iso, ncols, cnt, crp, wci, wvx);
            }
            GB_LAUNCH_CHECK();
        };

        // ---- symbolic: bin by min(flops, ncols) against the key-only table capacities
        bins_t bs = make_bins(flops, TW_SYM / 2, TB_SYM / 2, TL_SYM / 2);
        phase(std::true_type{}, std::false_type{}, bs, (int32_t *)nullptr, (Z *)nullptr, (int32_t *)nullptr,
              (Z *)nullptr);
        gb_exclusive_scan_i64(cnt, T.rowptr, nrows);
        const int64_t nz = gb_read_i64(T.rowptr + nrows);
        T.colidx = gb_malloc_n<int32_t>(nz ? nz : 1);
        T.vals = gb_malloc((vals_needed ? (nz ? nz : 1) : 1) * zs);
        T.nvals = nz;
        if (nz == 0) return;
        // ---- numeric: bin by the exact row counts against the key+value capacities
        bins_t bn = make_bins(cnt, TW_NUM / 2, TB_NUM / 2, TL_NUM / 2);
        const int64_t nhash = bn.c[1] + bn.c[2] + bn.c[3];
        gb_scratch us;  // unsorted rows of the hash bins
        int32_t *hci = nhash ? us.get<int32_t>(nz) : nullptr;
        Z *hvx = (nhash && vals_needed) ? us.get<Z>(nz) : nullptr;
        Z *fvx = vals_needed ? (Z *)T.vals : nullptr;
        if (vals_needed) phase(std::false_type{}, std::true_type{}, bn, hci, hvx, T.colidx, fvx);
        else phase(std::false_type{}, std::false_type{}, bn, hci, hvx, T.colidx, fvx);
        if (!nhash) return;

        // ---- sort the hash-bin rows by column into T (window rows are empty segments: left as written)
        int endbit = 1;
        while (endbit < 31 && (1LL << endbit) < ncols) endbit++;
        int64_t *ends = us.get<int64_t>(nrows);
        hipLaunchKernelGGL(k_seg_ends, dim3(hgrid(nrows, 256, 4096)), dim3(256), 0, gb_stream(), T.rowptr, nrows, ends);
        if (bn.c[4])
            hipLaunchKernelGGL(k_seg_skip, dim3(hgrid(bn.c[4], 256, 4096)), dim3(256), 0, gb_stream(),
                               rows + bn.st[4], bn.c[4], T.rowptr, ends);
        if (bn.c[0])
            hipLaunchKernelGGL(k_seg_skip, dim3(hgrid(bn.c[0], 256, 4096)), dim3(256), 0, gb_stream(),
                               rows + bn.st[0], bn.c[0], T.rowptr, ends);
        GB_LAUNCH_CHECK();
        // hipcub takes int counts: sort in row ranges of < 2^31 entries
        std::vector<int64_t> hrp;
        std::vector<int64_t> cuts{0};
        if (nz >= (1LL << 31) - 1) {
            hrp.resize(nrows + 1);
            gb_copy_d2h(hrp.data(), T.rowptr, (nrows + 1) * sizeof(int64_t));
            int64_t r = 0;
            while (r < nrows) {
                int64_t e = std::upper_bound(hrp.begin() + r + 1, hrp.end(), hrp[r] + ((1LL << 31) - 2)) - hrp.begin() - 1;
                if (e <= r) e = r + 1;
                cuts.push_back(e);
                r = e;
            }
        } else {
            cuts.push_back(nrows);
        }
        for (size_t c = 0; c + 1 < cuts.size(); c++) {
            const int64_t r0 = cuts[c], r1 = cuts[c + 1];
            const int64_t e0 = cuts.size() > 2 ? hrp[r0] : 0, e1 = cuts.size() > 2 ? hrp[r1] : nz;
            if (e1 <= e0) continue;
            gb_scratch ss;
            const int64_t *ob = T.rowptr + r0, *oe = ends + r0;
            if (e0 != 0) {
                int64_t *rb = ss.get<int64_t>(r1 - r0), *re = ss.get<int64_t>(r1 - r0);
                hipLaunchKernelGGL(k_sub_base, dim3(hgrid(r1 - r0, 256, 4096)), dim3(256), 0, gb_stream(),
                                   T.rowptr + r0, r1 - r0, e0, rb);
                hipLaunchKernelGGL(k_sub_base, dim3(hgrid(r1 - r0, 256, 4096)), dim3(256), 0, gb_stream(), ends + r0,
                                   r1 - r0, e0, re);
                GB_LAUNCH_CHECK();
                ob = rb;
                oe = re;
            }
            size_t tmp = 0;
            if (vals_needed) {
                GB_HIP(hipcub::DeviceSegmentedSort::SortPairs(nullptr, tmp, hci + e0, T.colidx + e0, hvx + e0,
                                                              fvx + e0, (int)(e1 - e0), (int)(r1 - r0), ob, oe,
                                                              gb_stream()));
                void *tb = ss.get<char>(tmp);
                GB_HIP(hipcub::DeviceSegmentedSort::SortPairs(tb, tmp, hci + e0, T.colidx + e0, hvx + e0, fvx + e0,
                                                              (int)(e1 - e0), (int)(r1 - r0), ob, oe, gb_stream()));
            } else {
                GB_HIP(hipcub::DeviceSegmentedSort::SortKeys(nullptr, tmp, hci + e0, T.colidx + e0, (int)(e1 - e0),
                                                             (int)(r1 - r0), ob, oe, gb_stream()));
                void *tb = ss.get<char>(tmp);
                GB_HIP(hipcub::DeviceSegmentedSort::SortKeys(tb, tmp, hci + e0, T.colidx + e0, (int)(e1 - e0),
                                                             (int)(r1 - r0), ob, oe, gb_stream()));
            }
        }
    });
}
