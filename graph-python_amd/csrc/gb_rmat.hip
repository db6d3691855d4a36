// gb_rmat.hip -- on-device Graph500-style R-MAT generator (GxB_Matrix_rmat).
//
// Same counter-based construction as the oracle (oracle/gb_oracle.c or_rmat):
// edge e, level l draws h = splitmix64(splitmix64(seed) ^ (64 e + l)) >> 11 and
// picks the quadrant by integer thresholds of (a, b, c, d) = (.57, .19, .19, .05);
// vertex labels pass through a seeded bijection; self-loops are dropped and
// duplicates removed.  CPU and GPU therefore build bit-identical graphs, and a
// row shard [row_begin, row_end) is exactly that block of the full graph's rows.
#include <hipcub/hipcub.hpp>

#include "gb_device.cuh"
#include "gb_internal.h"

#define RM_A 5134103575202365ULL
#define RM_B 6845471433603153ULL
#define RM_C 8556839292003942ULL

GB_HD uint64_t rm_smix(uint64_t x) {
    x += 0x9E3779B97F4A7C15ULL;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ULL;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBULL;
    return x ^ (x >> 31);
}

GB_HD uint64_t rm_scramble(uint64_t v, int scale, uint64_t k1, uint64_t k2) {
    uint64_t mask = (scale >= 64) ? ~0ULL : ((1ULL << scale) - 1);
    for (int r = 0; r < 3; r++) {
        v = (v * k1) & mask;
        v ^= (v >> ((scale + 1) / 2));
        v = (v + k2) & mask;
    }
    return v;
}

__global__ void k_rmat_edges(int64_t ne, int scale, uint64_t s0, uint64_t k1, uint64_t k2, uint64_t rb,
                             uint64_t re, bool transpose, uint64_t *__restrict__ keys,
                             unsigned long long *__restrict__ count) {
    for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < ne; e += (int64_t)gridDim.x * blockDim.x) {
        uint64_t r = 0, c = 0;
        for (int l = 0; l < scale; l++) {
            uint64_t h = rm_smix(s0 ^ ((uint64_t)e * 64 + (uint64_t)l)) >> 11;
            uint64_t rbit = (h >= RM_B), cbit = (h >= RM_A && h < RM_B) || (h >= RM_C);
            r |= rbit << l;
            c |= cbit << l;
        }
        r = rm_scramble(r, scale, k1, k2);
        c = rm_scramble(c, scale, k1, k2);
        if (transpose) {  // generate rows of A^T: swap the endpoints
            uint64_t t = r;
            r = c;
            c = t;
        }
        bool keep = (r != c) && r >= rb && r < re;
        // keys outside the shard / self-loops sort to the end and are dropped
        keys[e] = keep ? (((r - rb) << 32) | c) : ~0ULL;
        if (keep) atomicAdd(count, 1ULL);
    }
}

__global__ void k_rmat_heads(const uint64_t *__restrict__ k, int64_t n, int64_t *__restrict__ head) {
    for (int64_t q = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; q < n; q += (int64_t)gridDim.x * blockDim.x)
        head[q] = (q == 0 || k[q] != k[q - 1]) ? 1 : 0;
}

__global__ void k_rmat_emit(const uint64_t *__restrict__ k, const int64_t *__restrict__ pos, int64_t n,
                            unsigned long long *__restrict__ rowcnt, int32_t *__restrict__ colidx) {
    for (int64_t q = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; q < n; q += (int64_t)gridDim.x * blockDim.x) {
        if (q != 0 && k[q] == k[q - 1]) continue;
        colidx[pos[q]] = (int32_t)(k[q] & 0xffffffffULL);
        atomicAdd(&rowcnt[k[q] >> 32], 1ULL);
    }
}

__global__ void k_rmat_values(const int64_t *__restrict__ rowptr, const int32_t *__restrict__ colidx, int64_t nrows,
                              int64_t rb, uint64_t s0, int kind, bool transpose, void *__restrict__ vals) {
    int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
    int lane = threadIdx.x & 63;
    int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
    for (int64_t i = wave; i < nrows; i += nw)
        for (int64_t p = rowptr[i] + lane; p < rowptr[i + 1]; p += 64) {
            uint64_t gi = (uint64_t)(i + rb), gj = (uint64_t)(uint32_t)colidx[p];
            if (transpose) {
                uint64_t t = gi;
                gi = gj;
                gj = t;
            }
            uint64_t h = rm_smix(s0 ^ ((gi << 32) | gj));
            if (kind == 1) ((int64_t *)vals)[p] = 1 + (int64_t)(h % 255);
            else ((double *)vals)[p] = (double)(h >> 11) * 0x1.0p-53;
        }
}

extern "C" GrB_Info GxB_Matrix_rmat(GrB_Matrix *A, int scale, int edge_factor, uint64_t seed, int values,
                                    uint64_t value_seed, GrB_Index row_begin, GrB_Index row_end) {
    if (!A) return GrB_NULL_POINTER;
    return gb_api(nullptr, [&] {
        GB_REQUIRE(scale >= 1 && scale <= 30, GrB_INVALID_VALUE, "scale must be in [1, 30]");
        const int64_t n = 1LL << scale;
        const int64_t ne = (int64_t)edge_factor << scale;
        if (row_end == 0 || (int64_t)row_end > n) row_end = n;
        GB_REQUIRE(row_begin < row_end, GrB_INVALID_VALUE, "empty row range");
        const int64_t nr = (int64_t)(row_end - row_begin);
        const bool transpose = (values & 0x100) != 0;
        values &= 0xff;
        GrB_Type t = values == 1 ? GrB_INT64 : values == 2 ? GrB_FP64 : GrB_BOOL;
        GB_Obj *o = gb_new_object(GB_KIND_MATRIX, t, nr, n);
        try {
            gb_scratch s;
            uint64_t *keys = s.get<uint64_t>(ne);
            unsigned long long *cnt = s.get<unsigned long long>(1);
            gb_memset(cnt, 0, 8);
            const uint64_t s0 = rm_smix(seed);
            const uint64_t k1 = rm_smix(seed ^ 0x5851F42D4C957F2DULL) | 1ULL, k2 = rm_smix(seed ^ 0x14057B7EF767814FULL);
            hipLaunchKernelGGL(k_rmat_edges, dim3(8192), dim3(256), 0, gb_stream(), ne, scale, s0, k1, k2,
                               (uint64_t)row_begin, (uint64_t)row_end, transpose, keys, cnt);
            GB_LAUNCH_CHECK();
            // sort all keys (dropped ones are ~0 and land at the end)
            {
                uint64_t *k2b = s.get<uint64_t>(ne);
                hipcub::DoubleBuffer<uint64_t> kb(keys, k2b);
                size_t tmp = 0;
                GB_REQUIRE(ne < (1LL << 31), GrB_NOT_IMPLEMENTED, "too many edges");
                GB_HIP(hipcub::DeviceRadixSort::SortKeys(nullptr, tmp, kb, (int)ne, 0, 64, gb_stream()));
                void *tb = s.get<char>(tmp);
                GB_HIP(hipcub::DeviceRadixSort::SortKeys(tb, tmp, kb, (int)ne, 0, 64, gb_stream()));
                keys = kb.Current();
            }
            unsigned long long hc = 0;
            gb_copy_d2h(&hc, cnt, 8);
            const int64_t m = (int64_t)hc;
            int64_t *head = s.get<int64_t>(m + 1), *pos = s.get<int64_t>(m + 1);
            unsigned grid = (unsigned)std::min<int64_t>(8192, (m + 255) / 256 + 1);
            hipLaunchKernelGGL(k_rmat_heads, dim3(grid), dim3(256), 0, gb_stream(), keys, m, head);
            GB_LAUNCH_CHECK();
            gb_exclusive_scan_i64(head, pos, m);
            const int64_t nz = gb_read_i64(pos + m);
            int32_t *colidx = gb_malloc_n<int32_t>(nz);
            unsigned long long *rowcnt = s.get<unsigned long long>(nr + 1);
            gb_memset(rowcnt, 0, (nr + 1) * 8);
            hipLaunchKernelGGL(k_rmat_emit, dim3(grid), dim3(256), 0, gb_stream(), keys, pos, m, rowcnt, colidx);
            GB_LAUNCH_CHECK();
            int64_t *rowptr = gb_malloc_n<int64_t>(nr + 1);
            gb_exclusive_scan_i64((const int64_t *)rowcnt, rowptr, nr);
            void *vals;
            bool iso = values == 0;
            if (iso) {
                vals = gb_malloc(1);
                gb_memset(vals, 1, 1);
            } else {
                vals = gb_malloc(nz * 8);
                const uint64_t vs0 = rm_smix(value_seed ^ 0xA0761D6478BD642FULL);
                hipLaunchKernelGGL(k_rmat_values, dim3(4096), dim3(256), 0, gb_stream(), rowptr, colidx, nr,
                                   (int64_t)row_begin, vs0, values, transpose, vals);
                GB_LAUNCH_CHECK();
            }
            gb_install_csr(o, nr, n, nz, rowptr, colidx, vals, iso);
        } catch (...) {
            GrB_Matrix m = (GrB_Matrix)o;
            GrB_Matrix_free(&m);
            throw;
        }
        *A = (GrB_Matrix)o;
    });
}
