// gb_spgemm_hash.cuh -- Gustavson SpGEMM with hash accumulation, the default
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
// semirings are bit-exact whatever the order.
// Floating plus / times (order-dependent) take the deterministic ("DET") kernels
// by default (knob spgemm_det = 2 turns them off): in the workgroup-table and
// column-window bins every value slot has one owning wave, which applies its
// products in the flat product order (A entries ascending, then B positions);
// the wave-per-row bin is deterministic by construction (one wave owns the whole
// table).  What DET guarantees is run-to-run identical bits for identical inputs
// on one device -- ties inside a single LDS/HBM atomic instruction resolve in the
// hardware's fixed lane order, which tests/test_spgemm_det.py pins by repetition,
// not by proof -- and agreement with the ascending-k oracle within the fp64
// tolerance of BASELINE.json's north_star (rtol 1e-12 in the tests), not bit
// equality with it.  The expand-sort-compress path of gb_mxm.hip folds in
// ascending k and is bit-identical to the oracle (knob spgemm_method = 1).
#pragma once
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

// ------------------------------------------------------------------ deterministic accumulation
// Floating plus / times are order-dependent, and slots shared by the waves of a
// workgroup would take their products in whatever order the waves happen to
// run.  The deterministic kernels give every value slot ONE owning wave (a
// contiguous slice of the slots): each tile of products is split by owner
// (ballot ranks, so every owner's products keep the flat product order -- A
// entries ascending, then B positions), staged in LDS, and the owners apply
// their own products in that order.  Ties inside one apply instruction are
// resolved by the hardware's fixed lane order, so the same inputs always give
// the same bits (tests/test_spgemm_det.py).
template <int NW>
struct lg2c {
    static constexpr int v = NW >= 16 ? 4 : NW >= 8 ? 3 : NW >= 4 ? 2 : NW >= 2 ? 1 : 0;
};

// ow[u]: owner of this thread's u-th product (NW = none).  Returns the staging position of
// each product, ordered by (owner, u, wave, lane) -- the flat product order inside an owner --
// and this wave's own range [beg, end) of the staging array.  All threads of the workgroup call.
template <int NW, int P>
__device__ __forceinline__ void msplit(const int (&ow)[P], int (&pos)[P], int32_t (*cnt)[NW][NW], int &beg,
                                       int &end) {
    static_assert(P * NW <= 64, "one lane per (step, owner)");
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const unsigned long long lt = (1ULL << lane) - 1;
    int rk[P];
#pragma unroll
    for (int u = 0; u < P; u++) {
        // the lanes sharing this lane's owner, from one ballot per bit of the owner number
        // (lg2(NW) + 1 ballots; round 4 took one ballot per owner, NW of them)
        unsigned long long same = ~0ULL;
#pragma unroll
        for (int b = 0; b <= lg2c<NW>::v; b++) {
            const bool bit = (ow[u] >> b) & 1;
            const unsigned long long bb = __ballot(bit);
            same &= bit ? bb : ~bb;
        }
        rk[u] = __popcll(same & lt);
        if (lane < NW) cnt[u][w][lane] = 0;
        if (ow[u] < NW && rk[u] == 0) cnt[u][w][ow[u]] = __popcll(same);  // after the zeros (same wave)
    }
    __syncthreads();
    const int uu = lane / NW, oo = lane % NW;
    int tot = 0, pre = 0;
    if (lane < P * NW) {
#pragma unroll
        for (int q = 0; q < NW; q++) {
            const int c = cnt[uu][q][oo];
            tot += c;
            pre += q < w ? c : 0;
        }
    }
    int incl = tot;  // over the steps u of one owner (lanes oo, oo + NW, ...)
#pragma unroll
    for (int st = 1; st < P; st <<= 1) {
        const int v = __shfl_up(incl, st * NW, 64);
        if (uu >= st) incl += v;
    }
    const int T = __shfl(incl, (P - 1) * NW + oo, 64);  // owner total
    int y = T;
#pragma unroll
    for (int st = 1; st < NW; st <<= 1) {
        const int v = __shfl_up(y, st, 64);
        if (oo >= st) y += v;
    }
    const int base = y - T;
    const int off = base + (incl - tot) + pre;
#pragma unroll
    for (int u = 0; u < P; u++) {
        const int o = __shfl(off, u * NW + (ow[u] < NW ? ow[u] : 0), 64);
        pos[u] = ow[u] < NW ? o + rk[u] : -1;
    }
    beg = __shfl(base, w, 64);
    end = beg + __shfl(T, w, 64);
}

template <class SR, class Z, class S>
__device__ __forceinline__ void slot_apply(const SR &sr, int mon, S *slot, Z z) {
    if (mon == GBAMD_MON_ANY) *slot = to_slot<Z, S>(z);
    else slot_accum<SR, Z, S>(sr, mon, slot, z);
}

// ------------------------------------------------------------------ workgroup per row (LDS table)
// Table in dynamic LDS: 2^logT int32 keys, then (numeric) 2^logT value slots, then (DET) the
// staging of one tile (TILE values, TILE slot offsets).  P products per thread per tile: their
// loads are issued together (latency), and DET splits each tile by slot owner.
template <bool SYM, bool VALS, bool DET, class SR, class X, class Z, int BS, int P>
__global__ __launch_bounds__(BS) void k_hash_block(
    SR sr, int mon, const int32_t *__restrict__ rows, int64_t nr, int logT, const int64_t *__restrict__ arp,
    const int32_t *__restrict__ aci, const X *__restrict__ avx, bool a_iso, const int64_t *__restrict__ brp,
    const int32_t *__restrict__ bci, const X *__restrict__ bvx, bool b_iso, int64_t *__restrict__ cnt,
    const int64_t *__restrict__ crp, int32_t *__restrict__ cci, Z *__restrict__ cvx) {
    using S = slot_of<Z>;
    constexpr bool NV = !SYM && VALS;
    constexpr int NW = BS / 64, TILE = BS * P, LNW = lg2c<NW>::v;
    static_assert(!DET || NV, "deterministic accumulation is for numeric values");
    extern __shared__ __align__(16) char smem[];
    __shared__ int64_t s_excl[BS + 1];
    __shared__ int64_t s_b0[BS];
    __shared__ int32_t s_k[BS];
    __shared__ X s_av[BS];
    __shared__ int64_t s_wsum[NW];
    __shared__ int64_t s_pos;
    __shared__ int32_t s_cnt[DET ? P : 1][NW][NW];
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
    const bool rv = SR::reads_values && avx && bvx;
    Z idv = Z();
    const bool has_id = NV ? mon_identity<Z>(mon, idv) : false;
    const S ids = to_slot<Z, S>(idv);
    const int lT = logT;
    const int64_t T = 1LL << lT;
    const int shift = 32 - lT;
    int32_t *keys = (int32_t *)smem;
    S *vals = (S *)(smem + ((size_t)4 << lT));
    S *stz = vals + (DET ? T : 0);
    uint16_t *sto = (uint16_t *)(stz + (DET ? TILE : 0));
    const int osh = lT - LNW;
    for (int64_t r = blockIdx.x; r < nr; r += gridDim.x) {
        const int64_t i = rows[r];
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
            const int ne = a1 - g < BS ? (int)(a1 - g) : BS;  // entries of this group
            int top = 1;
            while (top < ne) top <<= 1;
            for (int64_t t0 = 0; t0 < G; t0 += TILE) {
                int sx[P];
                int64_t pb[P];
                bool ok[P];
#pragma unroll
                for (int u = 0; u < P; u++) {
                    const int64_t t = t0 + tid + (int64_t)BS * u;
                    ok[u] = t < G;
                    int s = 0;
                    if (ok[u]) {
                        for (int st = top >> 1; st > 0; st >>= 1)
                            if (s + st < ne && s_excl[s + st] <= t) s += st;
                    }
                    sx[u] = s;
                    pb[u] = ok[u] ? s_b0[s] + (t - s_excl[s]) : 0;
                }
                int32_t j[P];
#pragma unroll
                for (int u = 0; u < P; u++) j[u] = ok[u] ? bci[pb[u]] : 0;
                if constexpr (!NV) {
#pragma unroll
                    for (int u = 0; u < P; u++) {
                        if (!ok[u]) continue;
                        bool claimed;
                        h_insert(keys, j[u], shift, (uint32_t)(T - 1), claimed);
                        nclaim += claimed ? 1 : 0;
                    }
                } else {
                    X bv[P];
#pragma unroll
                    for (int u = 0; u < P; u++) {
                        bv[u] = X();
                        if (rv && ok[u]) bv[u] = bvx[b_iso ? 0 : pb[u]];
                    }
                    uint32_t h[P];
                    Z z[P];
                    bool cl[P];
#pragma unroll
                    for (int u = 0; u < P; u++) {
                        h[u] = 0;
                        cl[u] = false;
                        z[u] = Z();
                        if (ok[u]) {
                            h[u] = h_insert(keys, j[u], shift, (uint32_t)(T - 1), cl[u]);
                            z[u] = sr.mult(s_av[sx[u]], bv[u], i, s_k[sx[u]], j[u]);
                        }
                    }
                    if constexpr (DET) {
                        int ow[P], pos[P], beg, end;
#pragma unroll
                        for (int u = 0; u < P; u++) ow[u] = ok[u] ? (int)(h[u] >> osh) : NW;
                        msplit<NW, P>(ow, pos, s_cnt, beg, end);
#pragma unroll
                        for (int u = 0; u < P; u++)
                            if (ok[u]) {
                                stz[pos[u]] = to_slot<Z, S>(z[u]);
                                sto[pos[u]] = (uint16_t)(h[u] & ((1u << osh) - 1u));
                            }
                        __syncthreads();
                        S *od = vals + ((int64_t)w << osh);
                        for (int q = beg + lane; q < end; q += 64)
                            slot_accum<SR, Z, S>(sr, mon, od + sto[q], from_slot<Z, S>(stz[q]));
                    } else {
#pragma unroll
                        for (int u = 0; u < P; u++) {
                            if (!ok[u]) continue;
                            if (mon == GBAMD_MON_ANY) {
                                if (cl[u]) vals[h[u]] = to_slot<Z, S>(z[u]);
                            } else {
                                slot_accum<SR, Z, S>(sr, mon, vals + h[u], z[u]);
                            }
                        }
                    }
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

constexpr int WEG = 512;  // A entries per sweep group of the window kernels
constexpr int WP = 2;     // products per thread per tile of the window kernels

// The products of row i with columns in [cursor, cend) are enumerated WEG A entries at a
// time: win_entries finds every entry's end of range, win_tiles hands WP products per thread
// per tile to f (their loads issued together), win_advance moves the cursors to the end of
// range and returns the smallest column left.  All threads of the workgroup call.
struct win_sweep_lds {
    int32_t excl[WEG + 1];  // exclusive prefix of the products per entry
    int64_t lo[WEG];        // cursor
    int32_t rem[WEG];       // entries left in the B row
    int32_t len[WEG];       // products in [cursor, cend)
    int32_t k[WEG];
    int64_t wsum[HG / 64];
};

// Window index of the long B rows (numeric pass, round 5): for each B row longer than
// WIX_MIN entries, the positions where its columns cross the multiples of the window width
// 2^lw (pos[slot * (nw + 1) + t] = first position with column >= t * 2^lw, t = 0..nw).  A
// window end then costs one load (the row's index line, L2-resident across the row's sweeps)
// instead of a cooperative search over the rest of the B row -- round 4's numeric pass moved
// 12x the symbolic pass's bytes (profiles/r04_config5_s20_pmc.json), most of it those probes,
// repeated for every (A entry, window, value group) of a row; a value group's end inside a
// window is searched within the window's slice of the row only.
constexpr int WIX_MIN = 64;
struct win_index {
    const int32_t *slot = nullptr;  // [B rows] slot of the row's index, -1: short row (searched)
    const int64_t *pos = nullptr;
    int lw = 0, nw = 0;
};

// Entries [g, g + ne): the end of range, lb(cend) in B(k,:), by a cooperative search --
// 2^lg lanes per entry (as many as HG / ne allows, at most a wave) probe evenly spaced
// positions, so a row of few entries with long (hub) B rows takes log_{2^lg}(length)
// dependent loads instead of a per-thread gallop's ~2 log2(distance).
__device__ __forceinline__ void win_entries(win_sweep_lds &L, int64_t g, int ne, int64_t cend,
                                            const int64_t *__restrict__ cur, const int32_t *__restrict__ aci,
                                            const int64_t *__restrict__ brp, const int32_t *__restrict__ bci,
                                            const win_index &wx = win_index{}) {
    constexpr int NEW = WEG / 64;
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
    if (tid < ne) {
        const int64_t p = g + tid;
        const int32_t k = aci[p];
        const int64_t lo = cur[p];
        L.k[tid] = k;
        L.lo[tid] = lo;
        L.rem[tid] = (int32_t)(brp[k + 1] - lo);
    }
    __syncthreads();
    int lg = 6;
    while (lg > 1 && (ne << lg) > HG) lg--;
    const int Lw = 1 << lg;
    const int e = tid >> lg, q = tid & (Lw - 1);
    const bool act = e < ne;
    const uint64_t gmask = Lw == 64 ? ~0ULL : ((1ULL << Lw) - 1);
    const int gsh = lane & ~(Lw - 1);
    const int32_t ce = cend > 0x7fffffff ? 0x7fffffff : (int32_t)cend;
    int64_t a = 0, b = 0;
    if (act) {
        a = L.lo[e];
        b = a + L.rem[e];
        if (cend > 0x7fffffff) {
            a = b;  // the whole rest of the row
        } else if (wx.slot && q == 0) {
            const int32_t sl = wx.slot[L.k[e]];
            if (sl >= 0) {  // narrow [a, b) to the window slice holding cend (exact at a window end)
                const int64_t W = 1LL << wx.lw;
                const int64_t t = (cend + W - 1) >> wx.lw;
                const int64_t *ip = wx.pos + (int64_t)sl * (wx.nw + 1);
                const int64_t hi = ip[t < wx.nw ? t : wx.nw];
                b = hi < b ? hi : b;
                if ((cend & (W - 1)) == 0) a = b > a ? b : a;
                else if (t >= 1 && ip[t - 1] > a) a = ip[t - 1] < b ? ip[t - 1] : b;
            }
        }
    }
    if (wx.slot) {  // the group's other lanes take lane q == 0's narrowed bracket
        a = __shfl(a, gsh, 64);
        b = __shfl(b, gsh, 64);
    }
    while (__ballot(a < b)) {
        const bool open = a < b;
        const int64_t step = open ? (b - a + Lw - 1) >> lg : 1;  // Lw = 2^lg: a shift, not a 64-bit division
        const int64_t pos = a + q * step;
        const bool pr = open && pos < b && bci[pos] < ce;
        const int t = __popcll((__ballot(pr) >> gsh) & gmask);
        if (open) {
            if (t == 0) {
                b = a;
            } else {
                const int64_t nb = a + t * step < b ? a + t * step : b;
                a = a + (t - 1) * step + 1;
                b = nb;
            }
        }
    }
    if (act && q == 0) L.len[e] = (int32_t)(a - L.lo[e]);
    __syncthreads();
    const int32_t len = tid < ne ? L.len[tid] : 0;
    int32_t inc = len;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const int32_t t = __shfl_up(inc, off, 64);
        if (lane >= off) inc += t;
    }
    if (lane == 63 && w < NEW) L.wsum[w] = inc;
    __syncthreads();
    if (tid < WEG) {
        int32_t wbase = 0;
        for (int qq = 0; qq < w; qq++) wbase += (int32_t)L.wsum[qq];
        L.excl[tid] = wbase + inc - len;
        if (tid == WEG - 1) L.excl[WEG] = wbase + inc;
    }
    __syncthreads();
}

// cursors of entries [g, g + ne) to the end of range; this thread's smallest column left
__device__ __forceinline__ int32_t win_advance(const win_sweep_lds &L, int64_t g, int ne, int64_t *__restrict__ cur,
                                               const int32_t *__restrict__ bci) {
    const int tid = threadIdx.x;
    int32_t mn = 0x7fffffff;
    if (tid < ne) {
        const int64_t hi = L.lo[tid] + L.len[tid];
        cur[g + tid] = hi;
        if (L.len[tid] < L.rem[tid]) mn = bci[hi];
    }
    return mn;
}

template <class F>
__device__ __forceinline__ void win_tiles(const win_sweep_lds &L, int64_t g, int ne, int32_t c0,
                                          const int32_t *__restrict__ bci, F &&f) {
    constexpr int TILE = HG * WP;
    const int tid = threadIdx.x;
    const int32_t G = L.excl[WEG];
    int top = 1;  // the search covers entries [0, ne): the last entry with excl <= t is below ne
    while (top < ne) top <<= 1;
    for (int32_t t0 = 0; t0 < G; t0 += TILE) {
        int sx[WP];
        int64_t pb[WP];
        bool ok[WP];
        // a thread's WP products are consecutive in the flat order (round 5; round 4 strided them
        // by HG): one binary search for the first, the next entry found by stepping forward
        // (loads stay coalesced: a wave covers 64 * WP consecutive products)
        int s = 0;
#pragma unroll
        for (int u = 0; u < WP; u++) {
            const int32_t t = t0 + tid * WP + u;
            ok[u] = t < G;
            if (ok[u]) {
                if (u == 0) {
#pragma unroll
                    for (int st = top >> 1; st > 0; st >>= 1)
                        if (s + st < ne && L.excl[s + st] <= t) s += st;
                } else {
                    while (s + 1 < ne && L.excl[s + 1] <= t) s++;
                }
            }
            sx[u] = s;
            pb[u] = ok[u] ? L.lo[s] + (t - L.excl[s]) : 0;
        }
        int32_t c[WP];
#pragma unroll
        for (int u = 0; u < WP; u++) c[u] = ok[u] ? bci[pb[u]] - c0 : 0;
        f(ok, c, pb, sx, g);
    }
}

// all entry groups of the row: entries, (advance), tiles
template <class F>
__device__ __forceinline__ int32_t win_sweep(win_sweep_lds &L, int64_t a0, int64_t a1, int32_t c0, int64_t cend,
                                             bool advance, int64_t *__restrict__ cur,
                                             const int32_t *__restrict__ aci, const int64_t *__restrict__ brp,
                                             const int32_t *__restrict__ bci, F &&f,
                                             const win_index &wx = win_index{}) {
    int32_t mn = 0x7fffffff;
    for (int64_t g = a0; g < a1; g += WEG) {
        const int ne = a1 - g < WEG ? (int)(a1 - g) : WEG;
        win_entries(L, g, ne, cend, cur, aci, brp, bci, wx);
        if (advance) {
            const int32_t m = win_advance(L, g, ne, cur, bci);
            mn = m < mn ? m : mn;
        }
        win_tiles(L, g, ne, c0, bci, f);
        __syncthreads();
    }
    return mn;
}

// Symbolic (SYM: distinct columns per row) and key-only numeric (the window's set bits
// written out in column order: C's colidx comes out sorted).
template <bool SYM, class SR, class X, class Z>
__global__ __launch_bounds__(HG, 8) void k_row_window(
    SR sr, const int32_t *__restrict__ rows, int64_t nr, int logW, int64_t *__restrict__ cur,
    const int64_t *__restrict__ arp, const int32_t *__restrict__ aci, const int64_t *__restrict__ brp,
    const int32_t *__restrict__ bci, int64_t ncols, int64_t *__restrict__ cnt, const int64_t *__restrict__ crp,
    int32_t *__restrict__ cci, uint32_t *__restrict__ rowbits, int64_t nwrow, int32_t *__restrict__ bslot) {
    constexpr int NW = HG / 64;
    extern __shared__ __align__(16) char smem[];
    const int W = 1 << logW;        // columns per window (multiple of 256)
    const int NWD = W >> 5;         // bitmap words
    uint32_t *bm = (uint32_t *)smem;
    int32_t *prew = (int32_t *)(smem + (size_t)NWD * 4);  // numeric: exclusive popcount prefix per word
    __shared__ win_sweep_lds L;
    __shared__ int64_t s_wsum[NW];
    __shared__ int32_t s_wmin[NW];
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;

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
        // windows start at multiples of 32 columns (bitmap words line up with the stored row bitmap)
        int32_t c0 = block_min(nmin) & ~31;
        int64_t count = 0;
        int64_t outpos = SYM ? 0 : crp[i];
        uint32_t *rb = (SYM && rowbits) ? rowbits + r * nwrow : nullptr;  // this row's stored bitmap (zeroed)
        if (rb && tid == 0) bslot[i] = (int32_t)r;
        while (c0 < ncols) {
            const int64_t c1 = (int64_t)c0 + W;
            for (int q = tid; q < NWD; q += HG) bm[q] = 0u;
            __syncthreads();
            const int32_t mn = win_sweep(L, a0, a1, c0, c1, true, cur, aci, brp, bci,
                                         [&](const bool(&ok)[WP], const int32_t(&c)[WP], const int64_t(&)[WP],
                                             const int(&)[WP], int64_t) {
#pragma unroll
                                             for (int u = 0; u < WP; u++)
                                                 if (ok[u]) atomicOr(bm + (c[u] >> 5), 1u << (c[u] & 31));
                                         });
            __syncthreads();
            // exclusive popcount prefix per word (each thread a run of `per` words)
            const int per = (NWD + HG - 1) / HG;
            const int q0 = tid * per < NWD ? tid * per : NWD;
            const int q1 = q0 + per < NWD ? q0 + per : NWD;
            int32_t sm = 0;
            for (int q = q0; q < q1; q++) sm += __popc(bm[q]);
            int32_t inc = sm;
#pragma unroll
            for (int off = 1; off < 64; off <<= 1) {
                const int32_t t = __shfl_up(inc, off, 64);
                if (lane >= off) inc += t;
            }
            if (lane == 63) s_wsum[w] = inc;
            __syncthreads();
            int32_t run = inc - sm;
            int64_t m = 0;
            for (int q = 0; q < NW; q++) {
                if (q < w) run += (int32_t)s_wsum[q];
                m += s_wsum[q];
            }
            if constexpr (SYM) {
                count += m;
                if (rb) {  // the window's presence bits, for the numeric pass (k_window_num)
                    const int64_t w0 = c0 >> 5;
                    for (int q = tid; q < NWD && w0 + q < nwrow; q += HG) rb[w0 + q] = bm[q];
                }
            } else {
                for (int q = q0; q < q1; q++) {
                    uint32_t bits = bm[q];
                    while (bits) {
                        cci[outpos + run++] = c0 + q * 32 + __builtin_ctz(bits);
                        bits &= bits - 1u;
                    }
                }
                outpos += m;
            }
            c0 = block_min(mn) & ~31;
        }
        if constexpr (SYM) {
            if (tid == 0) cnt[i] = count;
        }
        __syncthreads();
    }
}

// ------------------------------------------------------------------ numeric column windows
// The numeric counterpart of k_row_window with values: per window, a presence sweep sets the
// bitmap; the window's sorted columns are written; then the values are accumulated group by
// group (LDS slots of < vcap entries, one sweep each) or, past in_c_groups groups, in one
// sweep straight into C's values.  DET: the slots are owned by waves (msplit above).
template <bool DET, class SR, class X, class Z>
__global__ __launch_bounds__(HG, 8) void k_window_num(
    SR sr, int mon, const int32_t *__restrict__ rows, int64_t nr, int logW, int vcap, int in_c_groups,
    int64_t *__restrict__ cur, const int64_t *__restrict__ arp, const int32_t *__restrict__ aci,
    const X *__restrict__ avx, bool a_iso, const int64_t *__restrict__ brp, const int32_t *__restrict__ bci,
    const X *__restrict__ bvx, bool b_iso, int64_t ncols, const int64_t *__restrict__ crp,
    int32_t *__restrict__ cci, Z *__restrict__ cvx, const uint32_t *__restrict__ rowbits, int64_t nwrow,
    const int32_t *__restrict__ bslot, win_index wx) {
    using S = slot_of<Z>;
    constexpr int NW = HG / 64, TILE = HG * WP;
    extern __shared__ __align__(16) char smem[];
    const int W = 1 << logW;
    const int NWD = W >> 5;
    uint32_t *bm = (uint32_t *)smem;
    // exclusive popcount prefix per 64-bit word pair, 16 bits relative to its 2^16-column half
    // (s_hb): W/32 bytes instead of round 4's 32-bit prefix per word (W/8), so 2^17-column
    // windows still fit two workgroups per CU
    uint16_t *pre16 = (uint16_t *)(smem + (size_t)NWD * 4);
    S *vals = (S *)(smem + (size_t)NWD * 4 + (size_t)NWD);
    S *stz = vals + vcap;                                  // DET: staged values
    uint16_t *sto = (uint16_t *)(stz + (DET ? TILE : 0));  // DET: staged slot offsets in the owner's slice
    __shared__ win_sweep_lds L;
    __shared__ int32_t s_cnt[DET ? WP : 1][NW][NW];
    __shared__ int64_t s_wsum[NW];
    __shared__ int32_t s_wmin[NW];
    __shared__ int32_t s_hb[8];  // window prefix at each 2^16-column half (W <= 2^19)
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
    const bool rv = SR::reads_values && avx && bvx;
    // the window's exclusive prefix at word q (q even: a pair boundary); pre16 holds the prefix's
    // low 16 bits, and inside one 2^16-column half it grows by less than 2^16 from s_hb
    auto wpre = [&](int q) -> int32_t {
        const int32_t hb = s_hb[q >> 11];
        return hb + (int32_t)(((uint32_t)pre16[q >> 1] - (uint32_t)hb) & 0xffffu);
    };
    Z idv = Z();
    const bool has_id = mon_identity<Z>(mon, idv);
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
    auto ceil_log2 = [](int64_t x) -> int {  // smallest e with 2^e >= x
        int e = 0;
        while ((1LL << e) < x) e++;
        return e;
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
        // with the window index, windows start at multiples of W (their ends are index entries)
        const int32_t calign = wx.slot ? ~(W - 1) : ~31;
        int32_t c0 = block_min(nmin) & calign;
        int64_t outpos = crp[i];
        // the row's presence bits from the symbolic pass (k_row_window), when it stored them
        const int32_t slot = rowbits ? bslot[i] : -1;
        const uint32_t *rb = slot >= 0 ? rowbits + (int64_t)slot * nwrow : nullptr;
        while (c0 < ncols) {
            const int64_t c1 = (int64_t)c0 + W;
            if (rb) {
                const int64_t w0 = c0 >> 5;
                for (int q = tid; q < NWD; q += HG) bm[q] = w0 + q < nwrow ? rb[w0 + q] : 0u;
            } else {
                for (int q = tid; q < NWD; q += HG) bm[q] = 0u;
            }
            __syncthreads();
            auto presence = [&](const bool(&ok)[WP], const int32_t(&c)[WP], const int64_t(&)[WP], const int(&)[WP],
                                int64_t) {
#pragma unroll
                for (int u = 0; u < WP; u++)
                    if (ok[u]) atomicOr(bm + (c[u] >> 5), 1u << (c[u] & 31));
            };
            // a row of one entry group keeps its entry tables in LDS from the presence sweep to a
            // value sweep over the whole window (one group, or C-resident)
            const bool one = !rb && a1 - a0 <= WEG;
            if (one) {
                win_entries(L, a0, (int)(a1 - a0), c1, cur, aci, brp, bci, wx);
                win_tiles(L, a0, (int)(a1 - a0), c0, bci, presence);
            } else if (!rb) {
                win_sweep(L, a0, a1, c0, c1, false, cur, aci, brp, bci, presence, wx);
            }
            __syncthreads();
            // exclusive popcount prefix per word (each thread a run of `per` words)
            const int per = (NWD + HG - 1) / HG;
            const int q0 = tid * per < NWD ? tid * per : NWD;
            const int q1 = q0 + per < NWD ? q0 + per : NWD;
            int32_t sm = 0;
            for (int q = q0; q < q1; q++) sm += __popc(bm[q]);
            int32_t inc = sm;
#pragma unroll
            for (int off = 1; off < 64; off <<= 1) {
                const int32_t t = __shfl_up(inc, off, 64);
                if (lane >= off) inc += t;
            }
            if (lane == 63) s_wsum[w] = inc;
            __syncthreads();
            int32_t run = inc - sm;
            int64_t m = 0;
            for (int q = 0; q < NW; q++) {
                if (q < w) run += (int32_t)s_wsum[q];
                m += s_wsum[q];
            }
            // sorted columns of the window: each thread writes the set bits of its own words
            for (int q = q0; q < q1; q++) {
                if ((q & 2047) == 0) s_hb[q >> 11] = run;
                if (!(q & 1)) pre16[q >> 1] = (uint16_t)run;
                uint32_t bits = bm[q];
                while (bits) {
                    cci[outpos + run++] = c0 + q * 32 + __builtin_ctz(bits);
                    bits &= bits - 1u;
                }
            }
            __syncthreads();
            // values of the products in [cursor, cend) into dst[rank - rbase], owner slices of
            // 2^osh slots; the cursors advance to cend
            // whole: the sweep covers the window from its start (one group, or C-resident)
            auto values = [&](int64_t cend, S *dst, int32_t rbase, int osh, bool whole) -> int32_t {
                auto f = [&](const bool(&ok)[WP], const int32_t(&c)[WP], const int64_t(&pb)[WP], const int(&sx)[WP],
                             int64_t g) {
                        X bv[WP], av[WP];
#pragma unroll
                        for (int u = 0; u < WP; u++) {
                            bv[u] = X();
                            av[u] = X();
                            if (rv && ok[u]) {
                                bv[u] = bvx[b_iso ? 0 : pb[u]];
                                av[u] = avx[a_iso ? 0 : g + sx[u]];
                            }
                        }
                        Z z[WP];
                        int32_t rk[WP];
#pragma unroll
                        for (int u = 0; u < WP; u++) {
                            z[u] = Z();
                            rk[u] = 0;
                            if (ok[u]) {
                                z[u] = sr.mult(av[u], bv[u], i, L.k[sx[u]], c[u] + c0);
                                const int q = c[u] >> 5;
                                const int qe = q & ~1;
                                rk[u] = wpre(qe) + ((q & 1) ? __popc(bm[qe]) : 0) +
                                        __popc(bm[q] & ((1u << (c[u] & 31)) - 1u)) - rbase;
                            }
                        }
                        if constexpr (DET) {
                            int ow[WP], pos[WP], beg, end;
#pragma unroll
                            for (int u = 0; u < WP; u++) ow[u] = ok[u] ? (rk[u] >> osh) : NW;
                            msplit<NW, WP>(ow, pos, s_cnt, beg, end);
#pragma unroll
                            for (int u = 0; u < WP; u++)
                                if (ok[u]) {
                                    stz[pos[u]] = to_slot<Z, S>(z[u]);
                                    sto[pos[u]] = (uint16_t)(rk[u] & ((1 << osh) - 1));
                                }
                            __syncthreads();
                            S *od = dst + ((int64_t)w << osh);
                            for (int q = beg + lane; q < end; q += 64)
                                slot_apply<SR, Z, S>(sr, mon, od + sto[q], from_slot<Z, S>(stz[q]));
                        } else {
#pragma unroll
                            for (int u = 0; u < WP; u++)
                                if (ok[u]) slot_apply<SR, Z, S>(sr, mon, dst + rk[u], z[u]);
                        }
                };
                if (one && whole) {  // entry tables still in LDS from the presence sweep
                    win_tiles(L, a0, (int)(a1 - a0), c0, bci, f);
                    __syncthreads();
                    return win_advance(L, a0, (int)(a1 - a0), cur, bci);
                }
                return win_sweep(L, a0, a1, c0, cend, true, cur, aci, brp, bci, f, wx);
            };
            // value groups of < vcap entries, each a run of 256-column chunks
            const int NB = W >> 8;
            const int64_t GV = vcap - 256;
            auto chunk_pre = [&](int b) -> int64_t { return b < NB ? (int64_t)wpre(b * 8) : m; };
            auto first_chunk = [&](int64_t key) {  // first b in [0, NB) with chunk_pre(b) >= key, else NB
                int lo = 0, hi = NB;
                while (lo < hi) {
                    const int mid = (lo + hi) >> 1;
                    if (chunk_pre(mid) >= key) hi = mid;
                    else lo = mid + 1;
                }
                return lo;
            };
            // many groups and a slot as wide as a value: one sweep accumulating straight into C's
            // values (this row's output range, L2-resident) instead of one sweep per group
            constexpr bool IN_C = sizeof(S) == sizeof(Z);
            const int ngg = (int)(chunk_pre(NB - 1) / GV) + 1;
            int32_t mn = 0x7fffffff;
            if (IN_C && ngg > in_c_groups) {
                S *dst = (S *)(cvx + outpos);
                if (has_id)
                    for (int64_t q = tid; q < m; q += HG) dst[q] = ids;
                __syncthreads();
                mn = values(c1, dst, 0, ceil_log2((m + NW - 1) / NW), true);
                __syncthreads();
            } else {
                for (int g = 0; g < ngg; g++) {
                    const int bs = first_chunk((int64_t)g * GV), be = first_chunk((int64_t)(g + 1) * GV);
                    const int64_t rbase = chunk_pre(bs), rcnt = chunk_pre(be) - rbase;
                    if (has_id)
                        for (int64_t q = tid; q < rcnt; q += HG) vals[q] = ids;
                    __syncthreads();
                    mn = values(c0 + (int64_t)be * 256, vals, (int32_t)rbase, ceil_log2((rcnt + NW - 1) / NW),
                                ngg == 1);
                    for (int64_t q = tid; q < rcnt; q += HG) cvx[outpos + rbase + q] = from_slot<Z, S>(vals[q]);
                    __syncthreads();
                }
            }
            outpos += m;
            c0 = block_min(mn) & calign;
        }
        __syncthreads();
    }
}

// window index (win_index above): flag the long rows, then per long row a wave fills its
// nw + 1 crossing positions by binary searches
__global__ void k_wix_flag(const int64_t *__restrict__ brp, int64_t n, uint8_t *__restrict__ flag) {
    for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < n; k += (int64_t)gridDim.x * blockDim.x)
        flag[k] = brp[k + 1] - brp[k] > WIX_MIN ? 1 : 0;
}

__global__ void k_wix_fill(const int64_t *__restrict__ brp, const int32_t *__restrict__ bci, int64_t n, int lw, int nw,
                           const uint8_t *__restrict__ flag, const int64_t *__restrict__ pos,
                           int32_t *__restrict__ slot, int64_t *__restrict__ ix) {
    const int lane = threadIdx.x & 63;
    for (int64_t k = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6; k < n;
         k += ((int64_t)gridDim.x * blockDim.x) >> 6) {
        if (!flag[k]) {
            if (lane == 0) slot[k] = -1;
            continue;
        }
        const int64_t sl = pos[k], rs = brp[k], re = brp[k + 1];
        if (lane == 0) slot[k] = (int32_t)sl;
        for (int t = lane; t <= nw; t += 64) {
            const int64_t key = (int64_t)t << lw;
            int64_t lo = rs, hi = re;
            while (lo < hi) {
                const int64_t m = (lo + hi) >> 1;
                if ((int64_t)bci[m] < key) lo = m + 1;
                else hi = m;
            }
            ix[sl * (nw + 1) + t] = lo;
        }
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

__global__ void k_row_keys(const int32_t *__restrict__ rows, int64_t nr, const int64_t *__restrict__ size,
                           uint32_t *__restrict__ keys) {
    for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < nr; r += (int64_t)gridDim.x * blockDim.x) {
        const int64_t v = size[rows[r]];
        keys[r] = v > 0xffffffffLL ? 0xffffffffu : (uint32_t)v;
    }
}

// entries of row i kept in the hash bins' scratch (0 for window / empty rows)
__global__ void k_hash_sizes(const int64_t *__restrict__ cnt, int64_t n, int64_t ncols, int64_t lim3,
                             int64_t *__restrict__ out) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t c = cnt[i], sz = c < ncols ? c : ncols;
        out[i] = (sz > 0 && sz <= lim3) ? c : 0;
    }
}

// sorted hash-bin rows from the compact scratch (offsets hoff) to C (offsets crp): a wave per row
template <class Z>
__global__ void k_place_rows(const int32_t *__restrict__ rows, int64_t nr, const int64_t *__restrict__ hoff,
                             const int64_t *__restrict__ crp, const int32_t *__restrict__ sci,
                             const Z *__restrict__ svx, int32_t *__restrict__ cci, Z *__restrict__ cvx) {
    const int lane = threadIdx.x & 63;
    for (int64_t r = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6; r < nr;
         r += ((int64_t)gridDim.x * blockDim.x) >> 6) {
        const int64_t i = rows[r], h0 = hoff[i], len = hoff[i + 1] - h0, c0 = crp[i];
        for (int64_t q = lane; q < len; q += 64) {
            cci[c0 + q] = sci[h0 + q];
            if (svx) cvx[c0 + q] = svx[h0 + q];
        }
    }
}

}  // namespace

namespace gbh {

// C = A * B (no mask applied here) for one semiring instantiation: T gets sorted CSR rows.
// Instantiated per semiring in gb_spgemm_hash_p*.hip (compiled in parallel).
template <class SRT, class X, class Z>
void spgemm_hash_run(gb_mat_result &T, gb_csr_view &A, gb_csr_view &B, const gb_sr_info &info, SRT srf,
                     bool vals_needed, const void *av, const void *bv, const int64_t *flops) {

    const int64_t nrows = A.nrows, ncols = B.ncols;
    const size_t zs = gb_type_size(info.zcode);
    gb_scratch s;
    int64_t *cnt = s.get<int64_t>(nrows + 1);
    int32_t *rows = s.get<int32_t>(nrows);
    unsigned long long *fill = s.get<unsigned long long>(5);
    int64_t *start = s.get<int64_t>(5);
    int64_t *cur = nullptr;  // per-A-entry cursors of the window kernel
    T.rowptr = gb_malloc_n<int64_t>(nrows + 1);

    struct bins_t {
        int64_t c[5], st[5];
        int64_t lim3;  // largest row size of the hash bins
    };
    auto make_bins = [&](const int64_t *size, int64_t lim1, int64_t lim2, int64_t lim3) {
        bins_t b;
        const int64_t cap = ncols;  // a row never has more distinct columns than B
        if (gb_knob("hash_window") == 1) lim1 = lim2 = lim3 = 0;  // every row to the window kernel (tests)
        b.lim3 = lim3;
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
        if (b.c[4] > 1 && gb_knob("window_order") != 1) {
            // the window bin's rows largest first, so the longest rows do not start last
            const int64_t nw = b.c[4];
            gb_scratch ks;
            uint32_t *k0 = ks.get<uint32_t>(nw), *k1 = ks.get<uint32_t>(nw);
            int32_t *r1 = ks.get<int32_t>(nw);
            hipLaunchKernelGGL(k_row_keys, dim3(hgrid(nw, 256, 4096)), dim3(256), 0, gb_stream(), rows + b.st[4], nw,
                               size, k0);
            GB_LAUNCH_CHECK();
            size_t tmp = 0;
            GB_HIP(hipcub::DeviceRadixSort::SortPairsDescending(nullptr, tmp, k0, k1, rows + b.st[4], r1, (int)nw, 0, 32,
                                                                gb_stream()));
            void *tb = ks.get<char>(tmp);
            GB_HIP(hipcub::DeviceRadixSort::SortPairsDescending(tb, tmp, k0, k1, rows + b.st[4], r1, (int)nw, 0, 32,
                                                                gb_stream()));
            gb_copy_d2d(rows + b.st[4], r1, nw * sizeof(int32_t));
        }
        return b;
    };
    // window width: a power of two >= 256 columns, no wider than needed for B
    auto win_log = [&](int maxlog) {
        int l = 8;
        while (l < maxlog && (1LL << l) < ncols) l++;
        return l;
    };

    using S = slot_of<Z>;
    const X *ax = (const X *)av, *bx = (const X *)bv;
    const int mon = info.mon;

    // one phase over the bins; SYM counts into cnt, else writes rows: hash bins into (hci, hvx),
    // window rows (already in column order) into (wci, wvx)
    const int64_t *hrow = nullptr;  // row offsets of the hash bins' scratch (numeric)
    uint32_t *rowbits = nullptr;    // window rows' presence bitmaps (symbolic -> numeric)
    int32_t *bslot = nullptr;       // per row: its bitmap's slot, -1 none
    int64_t nwrow = 0;              // words per row bitmap
    auto phase = [&](auto symc, auto valsc, const bins_t &b, int32_t *hci, Z *hvx, int32_t *wci, Z *wvx) {
        constexpr bool SYM = decltype(symc)::value;
        constexpr bool VALS = decltype(valsc)::value;
        constexpr int TW = SYM ? TW_SYM : TW_NUM;
        constexpr int TB = SYM ? TB_SYM : TB_NUM;
        constexpr int TL = SYM ? TL_SYM : TL_NUM;
        constexpr size_t slot_b = 4 + ((!SYM && VALS) ? sizeof(S) : 0);
        const int64_t *crp = SYM ? nullptr : T.rowptr;     // window rows: C's row offsets
        const int64_t *hcrp = SYM ? nullptr : hrow;         // hash rows: the scratch's
        if (b.c[0] && SYM)
            hipLaunchKernelGGL(k_zero_rows_cnt, dim3(hgrid(b.c[0], 256, 4096)), dim3(256), 0, gb_stream(),
                               rows + b.st[0], b.c[0], cnt);
        if (b.c[1])
            hipLaunchKernelGGL((k_hash_wave<SYM, VALS, SRT, X, Z, TW>), dim3(hgrid(b.c[1], HB / 64)), dim3(HB), 0,
                               gb_stream(), srf, mon, rows + b.st[1], b.c[1], A.rowptr, A.colidx, ax, A.iso,
                               B.rowptr, B.colidx, bx, B.iso, cnt, hcrp, hci, hvx);
        // deterministic accumulation where the order matters: floating plus / times
        constexpr bool FP = std::is_floating_point<Z>::value && !SYM && VALS;
        const bool det = FP && (mon == GBAMD_MON_PLUS || mon == GBAMD_MON_TIMES) && gb_knob("spgemm_det") != 2;
        auto block = [&](auto detc, auto bsc, auto pc, int64_t nb, int64_t st, int lt) {
            constexpr bool D = decltype(detc)::value;
            constexpr int BS = decltype(bsc)::value, P = decltype(pc)::value;
            const size_t sh = slot_b * ((size_t)1 << lt) + (D ? (size_t)BS * P * (sizeof(S) + 2) : 0);
            set_lds(k_hash_block<SYM, VALS, D, SRT, X, Z, BS, P>, sh);
            hipLaunchKernelGGL((k_hash_block<SYM, VALS, D, SRT, X, Z, BS, P>), dim3(hgrid(nb, 1)), dim3(BS), sh,
                               gb_stream(), srf, mon, rows + st, nb, lt, A.rowptr, A.colidx, ax, A.iso, B.rowptr,
                               B.colidx, bx, B.iso, cnt, hcrp, hci, hvx);
        };
        using I4 = std::integral_constant<int, 4>;
        using I2 = std::integral_constant<int, 2>;
        using IHB = std::integral_constant<int, HB>;
        using IHG = std::integral_constant<int, HG>;
        if (b.c[2]) {
            if constexpr (FP) {
                if (det) block(std::true_type{}, IHB{}, I4{}, b.c[2], b.st[2], __builtin_ctz(TB));
                else block(std::false_type{}, IHB{}, I4{}, b.c[2], b.st[2], __builtin_ctz(TB));
            } else {
                block(std::false_type{}, IHB{}, I4{}, b.c[2], b.st[2], __builtin_ctz(TB));
            }
        }
        if (b.c[3]) {
            if constexpr (FP) {
                if (det) block(std::true_type{}, IHG{}, I2{}, b.c[3], b.st[3], __builtin_ctz(TL));
                else block(std::false_type{}, IHG{}, I2{}, b.c[3], b.st[3], __builtin_ctz(TL));
            } else {
                block(std::false_type{}, IHG{}, I2{}, b.c[3], b.st[3], __builtin_ctz(TL));
            }
        }
        if (b.c[4]) {
            // symbolic: 2^19-column bitmap windows (64 KB); numeric: 2^17 columns (bitmap + word
            // prefixes 32 KB) with values in LDS in groups of < 8192 entries (64 KB for 8-byte
            // values; one-to-two-byte values: a group can hold the whole window)
            // narrow values: at least 512 columns, so a value group (vcap - 256 entries,
            // one 256-column chunk of headroom) is never empty
            // numeric windows sized for two 1024-thread workgroups per CU (round 3: 2^17 columns,
            // 8192 LDS values and 4 products per thread held one workgroup of 153 KB LDS per
            // CU at 4 waves per SIMD; config 5 s19 219 -> 204 ms at 2^16 / 3072 / 2, <= 64 VGPRs)
            int lw = SYM ? win_log(19) : (sizeof(Z) < 4 ? std::max(9, win_log(13)) : win_log(16));
            // knob window_lw (numeric, 4-8-byte values): wider windows, fewer windows per row but
            // more value groups per window (round 5: 2^17 slower at s19 and s20 even at two
            // workgroups per CU)
            const int64_t klw = gb_knob("window_lw");
            if (!SYM && sizeof(Z) >= 4 && klw >= 10 && klw <= 18) lw = win_log((int)klw);
            // round 5: the window prefix takes W/32 bytes instead of W/8, and the LDS it frees
            // holds more values per group (fewer value groups, hence fewer sweeps of the row's A
            // entries): 4480 slots keep two workgroups per CU (tools/spgemm_time.py, one box:
            // 3072 / 3584 / 4096 / 4480 -> s20 510 / 484 / 488 / 480 ms, s19 168.5 / - / 157.0 /
            // 154.6 ms; 6144 / 8192 drop to one workgroup per CU: s20 668 / 650 ms)
            int vcap = (SYM || !VALS) ? 0 : (sizeof(Z) < 4 ? (1 << lw) : 4480);
            // tests: a small LDS value capacity sends windows to the C-resident accumulation (and
            // A/B sweeps: up to 8192 for 4-8-byte values)
            const int64_t kv = gb_knob("window_vcap");
            if (vcap && kv > 256 && (kv < vcap || (sizeof(Z) >= 4 && kv <= 8192))) vcap = (int)kv;
            // grouped sweeps (one per vcap entries) up to this many, then C-resident accumulation
            const int64_t kg = gb_knob("window_in_c_groups");
            // round 3 (3072-value groups, s19): 2 226 ms, 4 208, 8 204, never 206; round 5 (4480-value
            // groups, tools/spgemm_time.py): 4 / 5 / 6 / 7 / 8 -> s20 513 / 480 / 465 / 470 / 477 ms,
            // s19 - / 157.1 / 153.4 / 153.0 / 154.1 ms
            const int in_c_groups = kg > 0 ? (int)kg : 6;
            if constexpr (!SYM && VALS) {
                // the long B rows' window index (knob window_index = 1: none; at most 1024 windows)
                win_index wx;
                gb_scratch xs;
                const int64_t nwx = (ncols + (1LL << lw) - 1) >> lw;
                if (gb_knob("window_index") != 1 && nwx <= 1024 && B.nrows > 0) {
                    uint8_t *fl = xs.get<uint8_t>(B.nrows);
                    int64_t *pos = xs.get<int64_t>(B.nrows + 1);
                    int32_t *slot = xs.get<int32_t>(B.nrows);
                    hipLaunchKernelGGL(k_wix_flag, dim3(hgrid(B.nrows, 256, 4096)), dim3(256), 0, gb_stream(),
                                       B.rowptr, B.nrows, fl);
                    GB_LAUNCH_CHECK();
                    gb_exclusive_scan_u8(fl, pos, B.nrows);
                    const int64_t nlong = gb_read_i64(pos + B.nrows);
                    // an optional speed-up: its index (8 B per long row and window) is capped at twice
                    // B's column indices (or 64 MB), so a wide matrix whose windows would make it
                    // outgrow B runs without it (wx.slot == nullptr: the kernel searches instead)
                    const int64_t ixbytes = nlong * (nwx + 1) * (int64_t)sizeof(int64_t);
                    const int64_t budget = std::max<int64_t>((int64_t)64 << 20, 8 * B.nvals);
                    if (ixbytes <= budget) {
                        int64_t *ix = xs.get<int64_t>(std::max<int64_t>(1, nlong * (nwx + 1)));
                        hipLaunchKernelGGL(k_wix_fill, dim3(hgrid(B.nrows * 64, 256, 8192)), dim3(256), 0,
                                           gb_stream(), B.rowptr, B.colidx, B.nrows, lw, (int)nwx, fl, pos, slot, ix);
                        GB_LAUNCH_CHECK();
                        wx.slot = slot;
                        wx.pos = ix;
                        wx.lw = lw;
                        wx.nw = (int)nwx;
                    }
                }
                auto win = [&](auto detc) {
                    constexpr bool D = decltype(detc)::value;
                    const size_t sh = (size_t)(1 << lw) / 8 + (size_t)(1 << lw) / 32 + (size_t)vcap * sizeof(S) +
                                      (D ? (size_t)HG * WP * (sizeof(S) + 2) : 0);
                    set_lds(k_window_num<D, SRT, X, Z>, sh);
                    hipLaunchKernelGGL((k_window_num<D, SRT, X, Z>), dim3(hgrid(b.c[4], 1, 2048)), dim3(HG), sh,
                                       gb_stream(), srf, mon, rows + b.st[4], b.c[4], lw, vcap, in_c_groups, cur,
                                       A.rowptr, A.colidx, ax, A.iso, B.rowptr, B.colidx, bx, B.iso, ncols, crp,
                                       wci, wvx, (const uint32_t *)rowbits, nwrow, (const int32_t *)bslot, wx);
                };
                if constexpr (FP) {
                    if (det) win(std::true_type{});
                    else win(std::false_type{});
                } else {
                    win(std::false_type{});
                }
            } else {
                const size_t sh = SYM ? (size_t)(1 << lw) / 8 : (size_t)(1 << lw) / 4;
                set_lds(k_row_window<SYM, SRT, X, Z>, sh);
                hipLaunchKernelGGL((k_row_window<SYM, SRT, X, Z>), dim3(hgrid(b.c[4], 1, 2048)), dim3(HG), sh,
                                   gb_stream(), srf, rows + b.st[4], b.c[4], lw, cur, A.rowptr, A.colidx,
                                   B.rowptr, B.colidx, ncols, cnt, crp, wci, SYM ? rowbits : nullptr, nwrow,
                                   SYM ? bslot : nullptr);
            }
        }
        GB_LAUNCH_CHECK();
    };

    // ---- symbolic: bin by min(flops, ncols) against the key-only table capacities
    bins_t bs = make_bins(flops, TW_SYM / 2, TB_SYM / 2, TL_SYM / 2);
    // the window rows' presence bitmaps (n bits each) are kept from the symbolic pass for the
    // numeric one, which then skips its presence sweep -- when they take at most a quarter of
    // the free device memory (knob window_bits=1: never)
    gb_scratch rbs;
    if (bs.c[4] && gb_knob("window_bits") != 1) {
        const int64_t nw = (ncols + 31) / 32;
        const size_t bytes = (size_t)bs.c[4] * (size_t)nw * 4;
        size_t fr = 0, tot = 0;
        if (hipMemGetInfo(&fr, &tot) == hipSuccess && bytes <= fr / 4) {
            rowbits = rbs.get<uint32_t>((size_t)bs.c[4] * (size_t)nw);
            bslot = rbs.get<int32_t>(nrows);
            nwrow = nw;
            gb_memset(rowbits, 0, bytes);
            gb_memset(bslot, 0xff, (size_t)nrows * sizeof(int32_t));
        }
    }
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
    Z *fvx = vals_needed ? (Z *)T.vals : nullptr;
    if (!nhash) {  // window rows only: written sorted, in place
        if (vals_needed) phase(std::false_type{}, std::true_type{}, bn, nullptr, nullptr, T.colidx, fvx);
        else phase(std::false_type{}, std::false_type{}, bn, nullptr, nullptr, T.colidx, fvx);
        return;
    }
    // the hash bins write their rows unsorted into a compact scratch (row offsets hoff, only
    // the hash rows' entries: the window rows, most of C at scale, go straight to C)
    gb_scratch us;
    int64_t *hsz = us.get<int64_t>(nrows), *hoff = us.get<int64_t>(nrows + 1);
    hipLaunchKernelGGL(k_hash_sizes, dim3(hgrid(nrows, 256, 4096)), dim3(256), 0, gb_stream(), cnt, nrows, ncols,
                       bn.lim3, hsz);
    GB_LAUNCH_CHECK();
    gb_exclusive_scan_i64(hsz, hoff, nrows);
    const int64_t nzh = gb_read_i64(hoff + nrows);
    int32_t *hci = us.get<int32_t>(nzh), *sci = us.get<int32_t>(nzh);
    Z *hvx = vals_needed ? us.get<Z>(nzh) : nullptr, *svx = vals_needed ? us.get<Z>(nzh) : nullptr;
    hrow = hoff;
    if (vals_needed) phase(std::false_type{}, std::true_type{}, bn, hci, hvx, T.colidx, fvx);
    else phase(std::false_type{}, std::false_type{}, bn, hci, hvx, T.colidx, fvx);
    hrow = nullptr;

    // ---- sort the hash rows by column (segments [hoff[i], hoff[i+1]); other rows are empty)
    // hipcub takes int counts: sort in row ranges of < 2^31 entries
    std::vector<int64_t> hrp;
    std::vector<int64_t> cuts{0};
    if (nzh >= (1LL << 31) - 1) {
        hrp.resize(nrows + 1);
        gb_copy_d2h(hrp.data(), hoff, (nrows + 1) * sizeof(int64_t));
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
        const int64_t e0 = cuts.size() > 2 ? hrp[r0] : 0, e1 = cuts.size() > 2 ? hrp[r1] : nzh;
        if (e1 <= e0) continue;
        gb_scratch ss;
        const int64_t *ob = hoff + r0, *oe = hoff + r0 + 1;
        if (e0 != 0) {
            int64_t *rb = ss.get<int64_t>(r1 - r0 + 1);
            hipLaunchKernelGGL(k_sub_base, dim3(hgrid(r1 - r0 + 1, 256, 4096)), dim3(256), 0, gb_stream(),
                               hoff + r0, r1 - r0 + 1, e0, rb);
            GB_LAUNCH_CHECK();
            ob = rb;
            oe = rb + 1;
        }
        size_t tmp = 0;
        if (vals_needed) {
            GB_HIP(hipcub::DeviceSegmentedSort::SortPairs(nullptr, tmp, hci + e0, sci + e0, hvx + e0, svx + e0,
                                                          (int)(e1 - e0), (int)(r1 - r0), ob, oe, gb_stream()));
            void *tb = ss.get<char>(tmp);
            GB_HIP(hipcub::DeviceSegmentedSort::SortPairs(tb, tmp, hci + e0, sci + e0, hvx + e0, svx + e0,
                                                          (int)(e1 - e0), (int)(r1 - r0), ob, oe, gb_stream()));
        } else {
            GB_HIP(hipcub::DeviceSegmentedSort::SortKeys(nullptr, tmp, hci + e0, sci + e0, (int)(e1 - e0),
                                                         (int)(r1 - r0), ob, oe, gb_stream()));
            void *tb = ss.get<char>(tmp);
            GB_HIP(hipcub::DeviceSegmentedSort::SortKeys(tb, tmp, hci + e0, sci + e0, (int)(e1 - e0),
                                                         (int)(r1 - r0), ob, oe, gb_stream()));
        }
    }
    // ---- the sorted hash rows into C
    hipLaunchKernelGGL(k_place_rows<Z>, dim3(hgrid(nhash, 4, 8192)), dim3(256), 0, gb_stream(), rows + bn.st[1],
                       nhash, (const int64_t *)hoff, (const int64_t *)T.rowptr, (const int32_t *)sci,
                       (const Z *)svx, T.colidx, fvx);
    GB_LAUNCH_CHECK();
}

}  // namespace gbh

#define GB_SPGEMM_HASH_INST(SRT, X, Z)                                                                    \
    template void gbh::spgemm_hash_run<SRT, X, Z>(gb_mat_result &, gb_csr_view &, gb_csr_view &,           \
                                                  const gb_sr_info &, SRT, bool, const void *, const void *, \
                                                  const int64_t *);
