// gb_prim.hip -- device primitives shared by the kernels: scans, radix sorts
// (rocPRIM through hipCUB, used only on ingest / format conversion paths),
// typecasts, bitmap <-> CSR conversion, CSR transpose.
#include <hipcub/hipcub.hpp>

#include <climits>

#include "gb_device.cuh"
#include "gb_dispatch.cuh"
#include "gb_internal.h"

#define GB_BLOCK 256

static inline unsigned gb_grid(int64_t n, int per_block = GB_BLOCK) {
    int64_t g = (n + per_block - 1) / per_block;
    if (g < 1) g = 1;
    if (g > (1LL << 30)) g = 1LL << 30;
    return (unsigned)g;
}

// ------------------------------------------------------------------ scans / sorts
// out[0..len) += *carry (the previous chunk's last prefix, already final on the stream)
__global__ void k_add_carry(int64_t *__restrict__ out, int64_t len, const int64_t *__restrict__ carry) {
    const int64_t c = *carry;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < len; i += (int64_t)gridDim.x * blockDim.x)
        out[i] += c;
}

struct gb_u8_to_i64 {
    __host__ __device__ int64_t operator()(uint8_t x) const { return (int64_t)x; }
};

// Inclusive sums into out[1..n] in chunks of < 2^31 items (hipCUB's item count is an
// int); chunk c > 0 then adds out[start_c], the previous chunk's total.
template <class It>
static void scan_chunked(It in, int64_t *out, int64_t n) {
    gb_memset(out, 0, sizeof(int64_t));
    if (n == 0) return;
    const int64_t CH = (int64_t)1 << 30;
    size_t tmp = 0;
    GB_HIP(hipcub::DeviceScan::InclusiveSum(nullptr, tmp, in, out + 1, (int)std::min(n, CH), gb_stream()));
    void *t = gb_malloc(tmp);
    for (int64_t off = 0; off < n; off += CH) {
        const int64_t len = std::min(n - off, CH);
        size_t tb = tmp;
        GB_HIP(hipcub::DeviceScan::InclusiveSum(t, tb, in + off, out + 1 + off, (int)len, gb_stream()));
        if (off) {
            hipLaunchKernelGGL(k_add_carry, dim3(gb_grid(len, GB_BLOCK * 8)), dim3(GB_BLOCK), 0, gb_stream(),
                               out + 1 + off, len, out + off);
            GB_LAUNCH_CHECK();
        }
    }
    gb_free(t);
}


struct gb_i32_plus {
    int64_t add;
    __host__ __device__ int64_t operator()(int32_t x) const { return (int64_t)x + add; }
};

// wave-tile scan of 4- or 8-byte integers (each + add_each), as the byte-flag scan below:
// four consecutive items per lane per round, SCW_ROUNDS rounds per wave tile
constexpr int SCW_ROUNDS = 8;
constexpr int64_t SCW_TILE = 64 * 4 * SCW_ROUNDS;

template <class T>
__device__ __forceinline__ void scw_load4(const T *__restrict__ in, int64_t i, int64_t n, int64_t add, int64_t (&v)[4]) {
    if (i + 4 <= n) {
        if constexpr (sizeof(T) == 4) {
            const int4 q = *reinterpret_cast<const int4 *>(in + i);
            v[0] = (int64_t)q.x + add;
            v[1] = (int64_t)q.y + add;
            v[2] = (int64_t)q.z + add;
            v[3] = (int64_t)q.w + add;
        } else {
            const longlong2 a = reinterpret_cast<const longlong2 *>(in + i)[0];
            const longlong2 b = reinterpret_cast<const longlong2 *>(in + i)[1];
            v[0] = a.x + add;
            v[1] = a.y + add;
            v[2] = b.x + add;
            v[3] = b.y + add;
        }
    } else {
        for (int b = 0; b < 4; b++) v[b] = i + b < n ? (int64_t)in[i + b] + add : 0;
    }
}

template <class T>
__global__ __launch_bounds__(256) void k_scanw_sums(const T *__restrict__ in, int64_t add, int64_t n, int64_t ntiles,
                                                    int64_t *__restrict__ tsum) {
    const int lane = threadIdx.x & 63;
    const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
    for (int64_t t = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6; t < ntiles; t += nw) {
        const int64_t base = t * SCW_TILE;
        int64_t s = 0;
#pragma unroll
        for (int r = 0; r < SCW_ROUNDS; r++) {
            const int64_t i = base + (int64_t)r * 256 + 4 * lane;
            int64_t v[4];
            scw_load4(in, i, n, add, v);
            s += v[0] + v[1] + v[2] + v[3];
        }
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
        if (lane == 0) tsum[t] = s;
    }
}

template <class T>
__global__ __launch_bounds__(256) void k_scanw_tiles(const T *__restrict__ in, int64_t add, int64_t n, int64_t ntiles,
                                                     const int64_t *__restrict__ toff, int64_t *__restrict__ out) {
    const int lane = threadIdx.x & 63;
    const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
    for (int64_t t = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6; t < ntiles; t += nw) {
        const int64_t base = t * SCW_TILE;
        int64_t run = toff[t];
#pragma unroll
        for (int r = 0; r < SCW_ROUNDS; r++) {
            const int64_t i = base + (int64_t)r * 256 + 4 * lane;
            int64_t v[4];
            scw_load4(in, i, n, add, v);
            const int64_t sm = v[0] + v[1] + v[2] + v[3];
            int64_t inc = sm;
#pragma unroll
            for (int off = 1; off < 64; off <<= 1) {
                const int64_t y = __shfl_up(inc, off, 64);
                if (lane >= off) inc += y;
            }
            const int64_t e = run + (inc - sm);
            if (i + 4 <= n) {
                longlong2 *o = reinterpret_cast<longlong2 *>(out + i);
                o[0] = make_longlong2(e, e + v[0]);
                o[1] = make_longlong2(e + v[0] + v[1], e + v[0] + v[1] + v[2]);
            } else {
                const int64_t v4[4] = {e, e + v[0], e + v[0] + v[1], e + v[0] + v[1] + v[2]};
                for (int b = 0; b < 4; b++)
                    if (i + b < n) out[i + b] = v4[b];
            }
            run += __shfl(inc, 63, 64);
        }
        if (t == ntiles - 1 && lane == 0) out[n] = run;
    }
}

// the wave-tile path for n items from SCW_TILE * 64 up, with 16-byte aligned input and output
template <class T>
static bool scanw(const T *in, int64_t add, int64_t *out, int64_t n) {
    if (n < SCW_TILE * 64 || ((uintptr_t)in & 15) || ((uintptr_t)out & 15) || gb_knob("scan_u8") == 1) return false;
    const int64_t nt = (n + SCW_TILE - 1) / SCW_TILE;
    int64_t *ts = gb_malloc_n<int64_t>(nt);
    int64_t *to = gb_malloc_n<int64_t>(nt + 1);
    const unsigned g = (unsigned)std::min<int64_t>((nt + 3) / 4, 8192);
    hipLaunchKernelGGL(k_scanw_sums<T>, dim3(g), dim3(256), 0, gb_stream(), in, add, n, nt, ts);
    GB_LAUNCH_CHECK();
    scan_chunked(ts, to, nt);
    hipLaunchKernelGGL(k_scanw_tiles<T>, dim3(g), dim3(256), 0, gb_stream(), in, add, n, nt, to, out);
    GB_LAUNCH_CHECK();
    gb_free(ts);
    gb_free(to);
    return true;
}

void gb_exclusive_scan_i64(const int64_t *in, int64_t *out, int64_t n) {
    // out has n+1 slots: out[0] = 0, out[i+1] = in[0] + ... + in[i]; any n (chunked)
    if (scanw(in, (int64_t)0, out, n)) return;
    scan_chunked(in, out, n);
}

void gb_exclusive_scan_i32(const int32_t *in, int64_t add_each, int64_t *out, int64_t n) {
    if (scanw(in, add_each, out, n)) return;
    scan_chunked(hipcub::TransformInputIterator<int64_t, gb_i32_plus, const int32_t *>(in, gb_i32_plus{add_each}), out,
                 n);
}

// Byte-flag scan (the compactions' positions, e.g. 65 M mask entries per masked-dot phase at
// R-MAT s22): a wave per tile of SC_TILE flags, no block barriers.  Pass 1 sums each tile;
// the tile sums are scanned (hipCUB, n / 4096 items); pass 2 rescans each tile four flags per
// lane per round (one 4-byte load, a 64-lane shuffle scan, two 16-byte stores of the four
// exclusive prefixes).  Reads the flags twice and writes the prefixes once: round 5 measured
// hipCUB's transform-iterator scan at 386 us for 65 M flags (~1.5 TB/s).
constexpr int SC_ROUNDS = 16;
constexpr int64_t SC_TILE = 64 * 4 * SC_ROUNDS;  // flags per wave tile

__device__ __forceinline__ int sc_bytesum(uint32_t w) {
    const uint32_t x = (w & 0x00ff00ffu) + ((w >> 8) & 0x00ff00ffu);
    return (int)((x & 0xffffu) + (x >> 16));
}
__device__ __forceinline__ uint32_t sc_word(const uint8_t *__restrict__ in, int64_t i, int64_t n) {
    if (i + 4 <= n) return *reinterpret_cast<const uint32_t *>(in + i);
    uint32_t w = 0;
    for (int b = 0; b < 4; b++)
        if (i + b < n) w |= (uint32_t)in[i + b] << (8 * b);
    return w;
}

__global__ __launch_bounds__(256) void k_scan_u8_sums(const uint8_t *__restrict__ in, int64_t n, int64_t ntiles,
                                                      int64_t *__restrict__ tsum) {
    const int lane = threadIdx.x & 63;
    const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
    for (int64_t t = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6; t < ntiles; t += nw) {
        const int64_t base = t * SC_TILE;
        int64_t s = 0;
        if (base + SC_TILE <= n) {
            const uint4 *v = reinterpret_cast<const uint4 *>(in + base);
            uint4 q[4];
#pragma unroll
            for (int r = 0; r < 4; r++) q[r] = v[r * 64 + lane];
#pragma unroll
            for (int r = 0; r < 4; r++) s += sc_bytesum(q[r].x) + sc_bytesum(q[r].y) + sc_bytesum(q[r].z) + sc_bytesum(q[r].w);
        } else {
            for (int64_t i = base + 4 * lane; i < n && i < base + SC_TILE; i += 256) s += sc_bytesum(sc_word(in, i, n));
        }
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
        if (lane == 0) tsum[t] = s;
    }
}

__global__ __launch_bounds__(256) void k_scan_u8_tiles(const uint8_t *__restrict__ in, int64_t n, int64_t ntiles,
                                                       const int64_t *__restrict__ toff, int64_t *__restrict__ out) {
    const int lane = threadIdx.x & 63;
    const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
    for (int64_t t = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6; t < ntiles; t += nw) {
        const int64_t base = t * SC_TILE;
        int64_t run = toff[t];
        const bool full = base + SC_TILE <= n;
        uint32_t w[SC_ROUNDS];
#pragma unroll
        for (int r = 0; r < SC_ROUNDS; r++) {
            const int64_t i = base + (int64_t)r * 256 + 4 * lane;
            w[r] = full ? *reinterpret_cast<const uint32_t *>(in + i) : (i < n ? sc_word(in, i, n) : 0u);
        }
#pragma unroll
        for (int r = 0; r < SC_ROUNDS; r++) {
            const int64_t i = base + (int64_t)r * 256 + 4 * lane;
            const int f0 = (int)(w[r] & 0xffu), f1 = (int)((w[r] >> 8) & 0xffu), f2 = (int)((w[r] >> 16) & 0xffu);
            const int sm = sc_bytesum(w[r]);
            int inc = sm;
#pragma unroll
            for (int off = 1; off < 64; off <<= 1) {
                const int y = __shfl_up(inc, off, 64);
                if (lane >= off) inc += y;
            }
            const int64_t e = run + (inc - sm);
            if (full || i + 4 <= n) {
                longlong2 *o = reinterpret_cast<longlong2 *>(out + i);
                o[0] = make_longlong2(e, e + f0);
                o[1] = make_longlong2(e + f0 + f1, e + f0 + f1 + f2);
            } else {
                const int64_t v4[4] = {e, e + f0, e + f0 + f1, e + f0 + f1 + f2};
                for (int b = 0; b < 4; b++)
                    if (i + b < n) out[i + b] = v4[b];
            }
            run += __shfl(inc, 63, 64);
        }
        if (t == ntiles - 1 && lane == 0) out[n] = run;
    }
}

void gb_exclusive_scan_u8(const uint8_t *in, int64_t *out, int64_t n) {
    // as gb_exclusive_scan_i64 over byte flags (any byte values), summed in int64
    if (n < SC_TILE * 64 || ((uintptr_t)in & 15) || ((uintptr_t)out & 15) || gb_knob("scan_u8") == 1) {
        scan_chunked(hipcub::TransformInputIterator<int64_t, gb_u8_to_i64, const uint8_t *>(in, gb_u8_to_i64()), out,
                     n);
        return;
    }
    const int64_t nt = (n + SC_TILE - 1) / SC_TILE;
    int64_t *ts = gb_malloc_n<int64_t>(nt);
    int64_t *to = gb_malloc_n<int64_t>(nt + 1);
    const unsigned g = (unsigned)std::min<int64_t>((nt + 3) / 4, 8192);
    hipLaunchKernelGGL(k_scan_u8_sums, dim3(g), dim3(256), 0, gb_stream(), in, n, nt, ts);
    GB_LAUNCH_CHECK();
    gb_exclusive_scan_i64(ts, to, nt);
    hipLaunchKernelGGL(k_scan_u8_tiles, dim3(g), dim3(256), 0, gb_stream(), in, n, nt, to, out);
    GB_LAUNCH_CHECK();
    gb_free(ts);
    gb_free(to);
}

__global__ void k_iota(int64_t *x, int64_t n) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x)
        x[i] = i;
}

__global__ void k_copy_i64(int64_t *dst, const int64_t *src) { *dst = *src; }

void gb_sort_pairs_u64(uint64_t *keys, int64_t *vals, int64_t n, int end_bit) {
    if (n <= 1) return;
    GB_REQUIRE(n < (1LL << 31), GrB_NOT_IMPLEMENTED, "sort of more than 2^31 items");
    uint64_t *k2 = gb_malloc_n<uint64_t>(n);
    int64_t *v2 = gb_malloc_n<int64_t>(n);
    hipcub::DoubleBuffer<uint64_t> kb(keys, k2);
    hipcub::DoubleBuffer<int64_t> vb(vals, v2);
    size_t tmp = 0;
    GB_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, tmp, kb, vb, (int)n, 0, end_bit, gb_stream()));
    void *t = gb_malloc(tmp);
    GB_HIP(hipcub::DeviceRadixSort::SortPairs(t, tmp, kb, vb, (int)n, 0, end_bit, gb_stream()));
    if (kb.Current() != keys) gb_copy_d2d(keys, kb.Current(), n * sizeof(uint64_t));
    if (vb.Current() != vals) gb_copy_d2d(vals, vb.Current(), n * sizeof(int64_t));
    gb_free(t);
    gb_free(k2);
    gb_free(v2);
}

void gb_sort_pairs_i32(int32_t *keys, int64_t *vals, int64_t n, int end_bit) {
    if (n <= 1) return;
    GB_REQUIRE(n < (1LL << 31), GrB_NOT_IMPLEMENTED, "sort of more than 2^31 items");
    int32_t *k2 = gb_malloc_n<int32_t>(n);
    int64_t *v2 = gb_malloc_n<int64_t>(n);
    hipcub::DoubleBuffer<int32_t> kb(keys, k2);
    hipcub::DoubleBuffer<int64_t> vb(vals, v2);
    size_t tmp = 0;
    GB_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, tmp, kb, vb, (int)n, 0, end_bit, gb_stream()));
    void *t = gb_malloc(tmp);
    GB_HIP(hipcub::DeviceRadixSort::SortPairs(t, tmp, kb, vb, (int)n, 0, end_bit, gb_stream()));
    if (kb.Current() != keys) gb_copy_d2d(keys, kb.Current(), n * sizeof(int32_t));
    if (vb.Current() != vals) gb_copy_d2d(vals, vb.Current(), n * sizeof(int64_t));
    gb_free(t);
    gb_free(k2);
    gb_free(v2);
}

// ------------------------------------------------------------------ casts
template <class D, class S>
__global__ void k_cast(D *__restrict__ dst, const S *__restrict__ src, int64_t n) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x)
        dst[i] = gb_cast<D, S>(src[i]);
}

template <class D>
static void cast_from(void *dst, const void *src, int src_code, int64_t n) {
    unsigned g = gb_grid(n);
    if (g > 4096) g = 4096;
#define GB_CASE(code, S)                                                                        \
    case code:                                                                                  \
        hipLaunchKernelGGL((k_cast<D, S>), dim3(g), dim3(GB_BLOCK), 0, gb_stream(), (D *)dst, \
                           (const S *)src, n);                                                  \
        break;
    switch (src_code) {
        GB_CASE(GBAMD_T_BOOL, bool)
        GB_CASE(GBAMD_T_INT8, int8_t)
        GB_CASE(GBAMD_T_UINT8, uint8_t)
        GB_CASE(GBAMD_T_INT16, int16_t)
        GB_CASE(GBAMD_T_UINT16, uint16_t)
        GB_CASE(GBAMD_T_INT32, int32_t)
        GB_CASE(GBAMD_T_UINT32, uint32_t)
        GB_CASE(GBAMD_T_INT64, int64_t)
        GB_CASE(GBAMD_T_UINT64, uint64_t)
        GB_CASE(GBAMD_T_FP32, float)
        GB_CASE(GBAMD_T_FP64, double)
    }
#undef GB_CASE
    GB_LAUNCH_CHECK();
}

void gb_cast_array(void *dst, int dst_code, const void *src, int src_code, int64_t n) {
    if (n <= 0) return;
    if (dst_code == src_code) {
        gb_copy_d2d(dst, src, n * gb_type_size(dst_code));
        return;
    }
    switch (dst_code) {
    case GBAMD_T_BOOL: cast_from<bool>(dst, src, src_code, n); break;
    case GBAMD_T_INT8: cast_from<int8_t>(dst, src, src_code, n); break;
    case GBAMD_T_UINT8: cast_from<uint8_t>(dst, src, src_code, n); break;
    case GBAMD_T_INT16: cast_from<int16_t>(dst, src, src_code, n); break;
    case GBAMD_T_UINT16: cast_from<uint16_t>(dst, src, src_code, n); break;
    case GBAMD_T_INT32: cast_from<int32_t>(dst, src, src_code, n); break;
    case GBAMD_T_UINT32: cast_from<uint32_t>(dst, src, src_code, n); break;
    case GBAMD_T_INT64: cast_from<int64_t>(dst, src, src_code, n); break;
    case GBAMD_T_UINT64: cast_from<uint64_t>(dst, src, src_code, n); break;
    case GBAMD_T_FP32: cast_from<float>(dst, src, src_code, n); break;
    case GBAMD_T_FP64: cast_from<double>(dst, src, src_code, n); break;
    }
}

// ------------------------------------------------------------------ iso expansion
template <class W>
__global__ void k_fill(W *__restrict__ dst, const W *__restrict__ one, int64_t n) {
    W v = *one;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x)
        dst[i] = v;
}

void *gb_expand_iso(const void *one_value, size_t tsize, int64_t n) {
    void *out = gb_malloc(n * tsize);
    if (n == 0) return out;
    unsigned g = gb_grid(n);
    if (g > 4096) g = 4096;
    switch (tsize) {
    case 1: hipLaunchKernelGGL(k_fill<uint8_t>, dim3(g), dim3(GB_BLOCK), 0, gb_stream(), (uint8_t *)out, (const uint8_t *)one_value, n); break;
    case 2: hipLaunchKernelGGL(k_fill<uint16_t>, dim3(g), dim3(GB_BLOCK), 0, gb_stream(), (uint16_t *)out, (const uint16_t *)one_value, n); break;
    case 4: hipLaunchKernelGGL(k_fill<uint32_t>, dim3(g), dim3(GB_BLOCK), 0, gb_stream(), (uint32_t *)out, (const uint32_t *)one_value, n); break;
    default: hipLaunchKernelGGL(k_fill<uint64_t>, dim3(g), dim3(GB_BLOCK), 0, gb_stream(), (uint64_t *)out, (const uint64_t *)one_value, n); break;
    }
    GB_LAUNCH_CHECK();
    return out;
}

// ------------------------------------------------------------------ bitmap helpers
// one 64-bit word per lane; wave-level popcount reduction, one atomic per block
__global__ void k_bitmap_count(const uint64_t *__restrict__ bits, int64_t nwords,
                               unsigned long long *__restrict__ count) {
    __shared__ unsigned long long part;
    if (threadIdx.x == 0) part = 0;
    __syncthreads();
    unsigned long long c = 0;
    for (int64_t w = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; w < nwords;
         w += (int64_t)gridDim.x * blockDim.x)
        c += __popcll(bits[w]);
    for (int off = 32; off > 0; off >>= 1) c += __shfl_xor(c, off, 64);
    if ((threadIdx.x & 63) == 0) atomicAdd(&part, c);
    __syncthreads();
    if (threadIdx.x == 0 && part) atomicAdd(count, part);
}

// one launch: grid-wide popcount, the finishing block stores the count (no prior
// zeroing) and, when given a host mailbox, publishes it there too
__global__ void k_bitmap_count_store(const uint64_t *__restrict__ bits, int64_t nwords, int64_t *__restrict__ count,
                                     unsigned long long *__restrict__ gst, gb_host_slot *pub, long long seq) {
    long long c = 0;
    for (int64_t w = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; w < nwords;
         w += (int64_t)gridDim.x * blockDim.x)
        c += __popcll(bits[w]);
    long long tot;
    if (gb_grid_sum(c, gst, &tot)) {
        *count = tot;
        if (pub) {
            __hip_atomic_store(&pub->value, tot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __threadfence_system();
            __hip_atomic_store(&pub->seq, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}

void gb_bitmap_count_pub(const uint64_t *bits, int64_t n, int64_t *d_count, gb_host_slot *pub_host, uint64_t seq) {
    const int64_t nw = gb_words(n);
    unsigned g = gb_grid(nw);
    if (g > 512) g = 512;
    hipLaunchKernelGGL(k_bitmap_count_store, dim3(g), dim3(GB_BLOCK), 0, gb_stream(), bits, nw, d_count,
                       gb_device_state(), pub_host ? gb_host_slot_device(pub_host) : nullptr, (long long)seq);
    GB_LAUNCH_CHECK();
}

__global__ void k_zero_bitmap(uint64_t *__restrict__ bits, int64_t nw, int64_t *__restrict__ count) {
    const int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    for (int64_t w = t; w < nw; w += (int64_t)gridDim.x * blockDim.x) bits[w] = 0;
    if (t == 0 && count) *count = 0;
}

void gb_zero_bitmap(uint64_t *bits, int64_t nw, int64_t *d_count) {
    unsigned g = gb_grid(nw);
    if (g > 1024) g = 1024;
    hipLaunchKernelGGL(k_zero_bitmap, dim3(g), dim3(GB_BLOCK), 0, gb_stream(), bits, nw, d_count);
    GB_LAUNCH_CHECK();
}

void gb_bitmap_count(const uint64_t *bits, int64_t n, int64_t *d_count) {
    gb_bitmap_count_pub(bits, n, d_count, nullptr, 0);
}

// per-word popcount -> exclusive scan -> positions
__global__ void k_word_pop(const uint64_t *__restrict__ bits, int64_t nwords, int64_t *__restrict__ pop) {
    for (int64_t w = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; w < nwords;
         w += (int64_t)gridDim.x * blockDim.x)
        pop[w] = __popcll(bits[w]);
}

template <class W>
__global__ void k_bitmap_scatter(const uint64_t *__restrict__ bits, const W *__restrict__ dense,
                                 bool iso, int64_t n, const int64_t *__restrict__ woff,
                                 int64_t *__restrict__ rowptr_n1, int32_t *__restrict__ colidx,
                                 W *__restrict__ vals) {
    // n x 1 CSR: row i has one entry (col 0) iff bit i set.  rowptr[i] = rank(i).
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        uint64_t w = bits[i >> 6];
        int b = i & 63;
        int64_t rank = woff[i >> 6] + __popcll(w & ((b == 0) ? 0ULL : (~0ULL >> (64 - b))));
        rowptr_n1[i] = rank;
        if ((w >> b) & 1ULL) {
            colidx[rank] = 0;
            if (vals) vals[rank] = iso ? dense[0] : dense[i];
        }
    }
}

void gb_bitmap_to_csr(const uint64_t *bits, const void *dense, bool iso, int64_t n, size_t tsize,
                      int64_t **rowptr, int32_t **colidx, void **vals, int64_t *nvals) {
    int64_t nw = gb_words(n);
    int64_t *pop = gb_malloc_n<int64_t>(nw + 1);
    int64_t *woff = gb_malloc_n<int64_t>(nw + 1);
    if (nw) {
        unsigned g = gb_grid(nw);
        hipLaunchKernelGGL(k_word_pop, dim3(g), dim3(GB_BLOCK), 0, gb_stream(), bits, nw, pop);
        GB_LAUNCH_CHECK();
    }
    gb_exclusive_scan_i64(pop, woff, nw);
    int64_t nz = gb_read_i64(woff + nw);
    int64_t *rp = gb_malloc_n<int64_t>(n + 1);
    int32_t *ci = gb_malloc_n<int32_t>(nz);
    void *vx = iso ? gb_malloc(tsize) : gb_malloc(nz * tsize);
    if (iso) gb_copy_d2d(vx, dense, tsize);
    if (n) {
        unsigned g = gb_grid(n);
        if (g > 8192) g = 8192;
        void *vout = iso ? nullptr : vx;
        switch (tsize) {
        case 1: hipLaunchKernelGGL(k_bitmap_scatter<uint8_t>, dim3(g), dim3(GB_BLOCK), 0, gb_stream(), bits, (const uint8_t *)dense, false, n, woff, rp, ci, (uint8_t *)vout); break;
        case 2: hipLaunchKernelGGL(k_bitmap_scatter<uint16_t>, dim3(g), dim3(GB_BLOCK), 0, gb_stream(), bits, (const uint16_t *)dense, false, n, woff, rp, ci, (uint16_t *)vout); break;
        case 4: hipLaunchKernelGGL(k_bitmap_scatter<uint32_t>, dim3(g), dim3(GB_BLOCK), 0, gb_stream(), bits, (const uint32_t *)dense, false, n, woff, rp, ci, (uint32_t *)vout); break;
        default: hipLaunchKernelGGL(k_bitmap_scatter<uint64_t>, dim3(g), dim3(GB_BLOCK), 0, gb_stream(), bits, (const uint64_t *)dense, false, n, woff, rp, ci, (uint64_t *)vout); break;
        }
        GB_LAUNCH_CHECK();
    }
    hipLaunchKernelGGL(k_copy_i64, dim3(1), dim3(1), 0, gb_stream(), rp + n, woff + nw);
    GB_LAUNCH_CHECK();
    gb_free(pop);
    gb_free(woff);
    *rowptr = rp;
    *colidx = ci;
    *vals = vx;
    *nvals = nz;
}

// n x m CSR with m == 1 (or any CSR: entry (i, 0) only) -> bitmap
template <class W>
__global__ void k_csr_col_to_bitmap(const int64_t *__restrict__ rowptr, const W *__restrict__ vals,
                                    bool iso, int64_t n, uint64_t *__restrict__ bits,
                                    W *__restrict__ dense) {
    int64_t w = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    int64_t nw = (n + 63) >> 6;
    if (w >= nw) return;
    uint64_t word = 0;
    for (int b = 0; b < 64; b++) {
        int64_t i = (w << 6) + b;
        if (i >= n) break;
        int64_t p = rowptr[i];
        if (rowptr[i + 1] > p) {
            word |= 1ULL << b;
            if (dense) dense[i] = iso ? vals[0] : vals[p];
        }
    }
    bits[w] = word;
}

void gb_csr_col_to_bitmap(const gb_csr_view &v, size_t tsize, uint64_t **bits, void **dense,
                          int64_t **d_nvals) {
    int64_t n = v.nrows;
    int64_t nw = gb_words(n);
    uint64_t *b = gb_malloc_n<uint64_t>(nw);
    void *d = v.iso ? gb_malloc(tsize) : gb_malloc(n * tsize);
    if (v.iso) gb_copy_d2d(d, v.vals, tsize);
    if (nw) {
        unsigned g = gb_grid(nw);
        void *dout = v.iso ? nullptr : d;
        switch (tsize) {
        case 1: hipLaunchKernelGGL(k_csr_col_to_bitmap<uint8_t>, dim3(g), dim3(GB_BLOCK), 0, gb_stream(), v.rowptr, (const uint8_t *)v.vals, false, n, b, (uint8_t *)dout); break;
        case 2: hipLaunchKernelGGL(k_csr_col_to_bitmap<uint16_t>, dim3(g), dim3(GB_BLOCK), 0, gb_stream(), v.rowptr, (const uint16_t *)v.vals, false, n, b, (uint16_t *)dout); break;
        case 4: hipLaunchKernelGGL(k_csr_col_to_bitmap<uint32_t>, dim3(g), dim3(GB_BLOCK), 0, gb_stream(), v.rowptr, (const uint32_t *)v.vals, false, n, b, (uint32_t *)dout); break;
        default: hipLaunchKernelGGL(k_csr_col_to_bitmap<uint64_t>, dim3(g), dim3(GB_BLOCK), 0, gb_stream(), v.rowptr, (const uint64_t *)v.vals, false, n, b, (uint64_t *)dout); break;
        }
        GB_LAUNCH_CHECK();
    }
    int64_t *cnt = gb_malloc_n<int64_t>(1);
    gb_bitmap_count(b, n, cnt);
    *bits = b;
    *dense = d;
    *d_nvals = cnt;
}

// ------------------------------------------------------------------ transpose
__global__ void k_expand_rows(const int64_t *__restrict__ rowptr, int64_t nrows,
                              int64_t *__restrict__ rowof) {
    // one wave per row
    int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
    int lane = threadIdx.x & 63;
    int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
    for (int64_t i = wave; i < nrows; i += nw)
        for (int64_t p = rowptr[i] + lane; p < rowptr[i + 1]; p += 64) rowof[p] = i;
}

__global__ void k_count_cols(const int32_t *__restrict__ colidx, int64_t nvals,
                             unsigned long long *__restrict__ cnt) {
    for (int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; p < nvals;
         p += (int64_t)gridDim.x * blockDim.x)
        atomicAdd(&cnt[colidx[p]], 1ULL);
}

template <class W>
__global__ void k_transpose_fill(const int64_t *__restrict__ perm, const int64_t *__restrict__ rowof,
                                 const W *__restrict__ vals, int64_t nvals,
                                 int32_t *__restrict__ tcol, W *__restrict__ tvals) {
    for (int64_t q = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; q < nvals;
         q += (int64_t)gridDim.x * blockDim.x) {
        int64_t p = perm[q];
        tcol[q] = (int32_t)rowof[p];
        if (tvals) tvals[q] = vals[p];
    }
}

void gb_transpose_csr(int64_t nrows, int64_t ncols, int64_t nvals, const int64_t *rowptr,
                      const int32_t *colidx, const void *vals, size_t tsize, bool iso,
                      int64_t **trowptr, int32_t **tcolidx, void **tvals, int64_t **tperm) {
    int64_t *trp = gb_malloc_n<int64_t>(ncols + 1);
    int32_t *tci = gb_malloc_n<int32_t>(nvals);
    void *tvx = vals ? (iso ? gb_malloc(tsize) : gb_malloc(nvals * tsize)) : nullptr;
    if (vals && iso) gb_copy_d2d(tvx, vals, tsize);
    // column counts -> row pointers of the transpose
    int64_t *cnt = gb_malloc_n<int64_t>(ncols + 1);
    gb_memset(cnt, 0, (ncols + 1) * sizeof(int64_t));
    if (nvals) {
        unsigned g = gb_grid(nvals);
        if (g > 8192) g = 8192;
        hipLaunchKernelGGL(k_count_cols, dim3(g), dim3(GB_BLOCK), 0, gb_stream(), colidx, nvals,
                           (unsigned long long *)cnt);
        GB_LAUNCH_CHECK();
    }
    gb_exclusive_scan_i64(cnt, trp, ncols);
    gb_free(cnt);
    if (nvals) {
        // stable sort of positions by column (rows come out ascending within a column)
        int32_t *keys = gb_malloc_n<int32_t>(nvals);
        int64_t *perm = gb_malloc_n<int64_t>(nvals);
        int64_t *rowof = gb_malloc_n<int64_t>(nvals);
        gb_copy_d2d(keys, colidx, nvals * sizeof(int32_t));
        hipLaunchKernelGGL(k_expand_rows, dim3(gb_grid(nrows * 64 > (1LL << 24) ? (1LL << 24) : nrows * 64)),
                           dim3(GB_BLOCK), 0, gb_stream(), rowptr, nrows, rowof);
        GB_LAUNCH_CHECK();
        // perm = 0..nvals-1 : reuse rowof-type iota via thrust-free kernel
        int64_t *iota = perm;
        {
            unsigned g = gb_grid(nvals);
            if (g > 8192) g = 8192;
            hipLaunchKernelGGL(k_iota, dim3(g), dim3(GB_BLOCK), 0, gb_stream(), iota, nvals);
            GB_LAUNCH_CHECK();
        }
        int bits = 1;
        while (bits < 31 && (1LL << bits) < ncols) bits++;
        gb_sort_pairs_i32(keys, perm, nvals, bits);
        unsigned g = gb_grid(nvals);
        if (g > 8192) g = 8192;
        void *vout = (vals && !iso) ? tvx : nullptr;
        switch (tsize) {
        case 1: hipLaunchKernelGGL(k_transpose_fill<uint8_t>, dim3(g), dim3(GB_BLOCK), 0, gb_stream(), perm, rowof, (const uint8_t *)vals, nvals, tci, (uint8_t *)vout); break;
        case 2: hipLaunchKernelGGL(k_transpose_fill<uint16_t>, dim3(g), dim3(GB_BLOCK), 0, gb_stream(), perm, rowof, (const uint16_t *)vals, nvals, tci, (uint16_t *)vout); break;
        case 4: hipLaunchKernelGGL(k_transpose_fill<uint32_t>, dim3(g), dim3(GB_BLOCK), 0, gb_stream(), perm, rowof, (const uint32_t *)vals, nvals, tci, (uint32_t *)vout); break;
        default: hipLaunchKernelGGL(k_transpose_fill<uint64_t>, dim3(g), dim3(GB_BLOCK), 0, gb_stream(), perm, rowof, (const uint64_t *)vals, nvals, tci, (uint64_t *)vout); break;
        }
        GB_LAUNCH_CHECK();
        gb_free(keys);
        if (tperm) {
            *tperm = perm;
            perm = nullptr;
        }
        gb_free(perm);
        gb_free(rowof);
    } else if (tperm) {
        *tperm = gb_malloc_n<int64_t>(1);
    }
    *trowptr = trp;
    *tcolidx = tci;
    *tvals = tvx;
}

// ---------------------------------------------------------------- hot-column relabel
// A dense-input SpMV gathers x[k] for every entry; on a power-law matrix most entries name a
// few columns (R-MAT s22: the 2^19 most frequent of 4.2M columns carry 93% of the entries), but
// their x values are scattered over all of x, one 8-byte value per 128-byte line, so the
// gathers miss in L2.  The relabel packs the hot columns' values into a contiguous array
// (gathered once per call, 2 MB for 2^18 fp64: 85% of the s22 entries) that stays L2-resident: entries of hot columns
// carry INT32_MIN | rank instead of the column, the rest keep their column.  Built once per
// matrix version and orientation (freed with the other cached views).
__global__ void k_hot_count(const int32_t *__restrict__ colidx, int64_t nvals, uint32_t *__restrict__ cnt) {
    for (int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; p < nvals; p += (int64_t)gridDim.x * blockDim.x)
        atomicAdd(&cnt[colidx[p]], 1u);
}

__global__ void k_iota_i32(int32_t *__restrict__ out, int64_t n) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        out[i] = (int32_t)i;
}

__global__ void k_hot_rank(const int32_t *__restrict__ hot, int64_t nh, int32_t *__restrict__ rank) {
    for (int64_t h = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; h < nh; h += (int64_t)gridDim.x * blockDim.x)
        rank[hot[h]] = (int32_t)h;
}

__global__ void k_hot_remap(const int32_t *__restrict__ colidx, int64_t nvals, const int32_t *__restrict__ rank,
                            int32_t *__restrict__ out) {
    for (int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; p < nvals;
         p += (int64_t)gridDim.x * blockDim.x) {
        const int32_t c = colidx[p], r = rank[c];
        out[p] = r >= 0 ? (int32_t)((uint32_t)r | 0x80000000u) : c;
    }
}

void gb_view_hot(gb_csr_view &v, GB_Obj *A, int orient) {
    if (A->kind != GB_KIND_MATRIX || !v.colidx) return;
    const int64_t knob = gb_knob("xhot");  // 0 auto, 1 never, 2 always (tests)
    if (knob == 1) return;
    int64_t H = gb_knob("xhot_cols");
    if (H <= 0) H = 1LL << 18;  // 2 MB of fp64 x (tools/xhot_probe.py, s22: 2^16 684 us, 2^18 662, 2^19 667, 2^20 677)
    if (H > v.ncols) H = v.ncols;
    if (!A->hot_ci[orient]) {
        // worth it only when x does not fit the L2 anyway and there is enough to gather
        if (knob != 2 && (v.nvals < (1LL << 22) || v.ncols <= 2 * H)) return;
        if (H <= 0 || v.nvals == 0) return;
        const int64_t nc = v.ncols;
        gb_scratch s;
        uint32_t *cnt = s.get<uint32_t>(nc), *cnt2 = s.get<uint32_t>(nc);
        int32_t *ids = s.get<int32_t>(nc), *ids2 = s.get<int32_t>(nc);
        gb_memset(cnt, 0, nc * sizeof(uint32_t));
        unsigned g = gb_grid(v.nvals);
        if (g > 8192) g = 8192;
        hipLaunchKernelGGL(k_hot_count, dim3(g), dim3(GB_BLOCK), 0, gb_stream(), v.colidx, v.nvals, cnt);
        GB_LAUNCH_CHECK();
        unsigned gc = gb_grid(nc);
        if (gc > 8192) gc = 8192;
        hipLaunchKernelGGL(k_iota_i32, dim3(gc), dim3(GB_BLOCK), 0, gb_stream(), ids, nc);
        GB_LAUNCH_CHECK();
        size_t tmp = 0;
        GB_HIP(hipcub::DeviceRadixSort::SortPairsDescending(nullptr, tmp, cnt, cnt2, ids, ids2, (int)nc, 0, 32,
                                                            gb_stream()));
        void *tb = s.get<char>(tmp);
        GB_HIP(hipcub::DeviceRadixSort::SortPairsDescending(tb, tmp, cnt, cnt2, ids, ids2, (int)nc, 0, 32,
                                                            gb_stream()));
        int32_t *hot = gb_malloc_n<int32_t>(H);
        gb_copy_d2d(hot, ids2, H * sizeof(int32_t));
        int32_t *rank = ids;  // reuse: -1 everywhere, then the hot ranks
        gb_memset(rank, 0xff, nc * sizeof(int32_t));
        hipLaunchKernelGGL(k_hot_rank, dim3(std::max(1u, std::min(gb_grid(H), 8192u))), dim3(GB_BLOCK), 0,
                           gb_stream(), hot, H, rank);
        GB_LAUNCH_CHECK();
        int32_t *hci = gb_malloc_n<int32_t>(v.nvals);
        hipLaunchKernelGGL(k_hot_remap, dim3(g), dim3(GB_BLOCK), 0, gb_stream(), v.colidx, v.nvals, rank, hci);
        GB_LAUNCH_CHECK();
        A->hot_ci[orient] = hci;
        A->hot_cols[orient] = hot;
        A->hot_n[orient] = H;
    }
    v.hcolidx = A->hot_ci[orient];
    v.hcols = A->hot_cols[orient];
    v.nhot = A->hot_n[orient];
}

// ------------------------------------------------------------------ narrow values
// Integer values that all fit fewer bytes are kept a second time in that width (exact: the
// kernels widen on load), so a kernel whose value reads are scattered -- the masked dot's hits
// read one value per matching key -- touches 2-8x fewer cache lines.  R-MAT's INT64 weights
// (1..255) take one byte.  Built once per matrix version and orientation (dropped with the
// transpose cache).
template <class T>
__global__ void k_minmax(const T *__restrict__ x, int64_t n, long long *__restrict__ mn,
                         unsigned long long *__restrict__ mx_u, long long *__restrict__ mx_s) {
    long long lmn = LLONG_MAX, lmx = LLONG_MIN;
    unsigned long long umx = 0;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const T v = x[i];
        if constexpr (std::is_signed<T>::value) {
            lmn = (long long)v < lmn ? (long long)v : lmn;
            lmx = (long long)v > lmx ? (long long)v : lmx;
        } else {
            umx = (unsigned long long)v > umx ? (unsigned long long)v : umx;
        }
    }
    for (int off = 32; off > 0; off >>= 1) {
        const long long a = __shfl_xor(lmn, off, 64), b = __shfl_xor(lmx, off, 64);
        const unsigned long long c = __shfl_xor(umx, off, 64);
        lmn = a < lmn ? a : lmn;
        lmx = b > lmx ? b : lmx;
        umx = c > umx ? c : umx;
    }
    if ((threadIdx.x & 63) == 0) {
        if constexpr (std::is_signed<T>::value) {
            atomicMin(mn, lmn);
            atomicMax(mx_s, lmx);
        } else {
            atomicMax(mx_u, umx);
        }
    }
}

template <class D, class T>
__global__ void k_narrow(const T *__restrict__ x, int64_t n, D *__restrict__ y) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        y[i] = (D)x[i];
}

void gb_view_narrow(gb_csr_view &v, GB_Obj *A, int orient) {
    v.nvx = nullptr;
    v.nvk = 0;
    if (A->kind != GB_KIND_MATRIX || v.iso || !v.vals || v.nvals == 0 || gb_knob("narrow") == 1) return;
    const int code = v.tcode;
    const bool sgn = code == GBAMD_T_INT16 || code == GBAMD_T_INT32 || code == GBAMD_T_INT64;
    const bool uns = code == GBAMD_T_UINT16 || code == GBAMD_T_UINT32 || code == GBAMD_T_UINT64;
    if (!sgn && !uns) return;
    if (!A->nar_done[orient]) {
        const size_t ts = gb_type_size(code);
        gb_scratch s;
        long long *st = s.get<long long>(3);
        const long long init[3] = {LLONG_MAX, LLONG_MIN, 0};
        gb_copy_h2d(st, init, sizeof(init));
        unsigned g = gb_grid(v.nvals);
        if (g > 4096) g = 4096;
        gb_with_type(code, [&](auto z) {
            using T = decltype(z);
            if constexpr (std::is_integral<T>::value && sizeof(T) >= 2)
                hipLaunchKernelGGL(k_minmax<T>, dim3(g), dim3(GB_BLOCK), 0, gb_stream(), (const T *)v.vals, v.nvals,
                                   st, (unsigned long long *)(st + 2), st + 1);
        });
        GB_LAUNCH_CHECK();
        long long h[3];
        gb_copy_d2h(h, st, sizeof(h));
        int k = 0;
        auto fits = [&](int kk) -> bool {
            if ((size_t)(kk < 0 ? -kk : kk) >= ts) return false;
            if (uns) {
                const unsigned long long mx = (unsigned long long)h[2];
                return kk > 0 && mx <= (kk == 1 ? 0xffULL : kk == 2 ? 0xffffULL : 0xffffffffULL);
            }
            const long long mn = h[0], mx = h[1];
            if (kk == 1) return mn >= 0 && mx <= 0xff;
            if (kk == -1) return mn >= -128 && mx <= 127;
            if (kk == 2) return mn >= 0 && mx <= 0xffff;
            if (kk == -2) return mn >= -32768 && mx <= 32767;
            if (kk == 4) return mn >= 0 && mx <= 0xffffffffLL;
            return mn >= INT32_MIN && mx <= INT32_MAX;
        };
        for (int kk : {1, -1, 2, -2, 4, -4})
            if (fits(kk)) {
                k = kk;
                break;
            }
        void *nv = nullptr;
        if (k) {
            const int nb = k < 0 ? -k : k;
            nv = gb_malloc((size_t)v.nvals * nb);
            gb_with_type(code, [&](auto z) {
                using T = decltype(z);
                if constexpr (std::is_integral<T>::value && sizeof(T) >= 2) {
                    auto go = [&](auto d) {
                        using D = decltype(d);
                        hipLaunchKernelGGL((k_narrow<D, T>), dim3(g), dim3(GB_BLOCK), 0, gb_stream(),
                                           (const T *)v.vals, v.nvals, (D *)nv);
                    };
                    switch (k) {
                    case 1: go(uint8_t()); break;
                    case -1: go(int8_t()); break;
                    case 2: go(uint16_t()); break;
                    case -2: go(int16_t()); break;
                    case 4: go(uint32_t()); break;
                    default: go(int32_t()); break;
                    }
                }
            });
            GB_LAUNCH_CHECK();
        }
        A->nar_vx[orient] = nv;
        A->nar_k[orient] = k;
        A->nar_done[orient] = true;
    }
    v.nvx = A->nar_vx[orient];
    v.nvk = A->nar_vx[orient] ? A->nar_k[orient] : 0;
}
