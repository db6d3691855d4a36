// gb_io.cpp -- Matrix Market coordinate reader (host side of ingest).
//
// The reference reads .mtx files through scipy / fast_matrix_market and then
// builds with Matrix.from_coo (reference graphblas/io/_matrixmarket.py:6-61);
// SuiteSparse-Collection inputs such as com-Orkut (234M entries, SURVEY §8d
// config 2) make that the dominant ingest cost.  This reader memory-maps the
// file and parses the entry lines on all host threads into COO arrays that the
// caller hands to GrB_Matrix_build_* (device sort + fold).  Symmetric and
// skew-symmetric files are expanded (the mirrored entry of every off-diagonal
// one), pattern files give iso-true BOOL, integer INT64, real FP64.
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cctype>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "gb_internal.h"

namespace {
enum Field { F_PATTERN, F_INTEGER, F_REAL };
enum Sym { S_GENERAL, S_SYMMETRIC, S_SKEW };

struct Parsed {
    std::vector<uint64_t> I, J;
    std::vector<int64_t> Xi;
    std::vector<double> Xd;
};

inline const char *skip_ws(const char *p, const char *e) {
    while (p < e && (*p == ' ' || *p == '\t' || *p == '\r')) p++;
    return p;
}

inline const char *parse_u64(const char *p, const char *e, uint64_t *v, bool *ok) {
    p = skip_ws(p, e);
    uint64_t x = 0;
    const char *s = p;
    while (p < e && *p >= '0' && *p <= '9') x = x * 10 + (uint64_t)(*p++ - '0');
    *ok = p > s;
    *v = x;
    return p;
}

inline const char *parse_i64(const char *p, const char *e, int64_t *v, bool *ok) {
    p = skip_ws(p, e);
    bool neg = false;
    if (p < e && (*p == '-' || *p == '+')) neg = (*p++ == '-');
    uint64_t x = 0;
    p = parse_u64(p, e, &x, ok);
    *v = neg ? -(int64_t)x : (int64_t)x;
    return p;
}

inline const char *parse_f64(const char *p, const char *e, double *v, bool *ok) {
    p = skip_ws(p, e);
    char buf[64];
    size_t n = 0;
    while (p < e && n < sizeof(buf) - 1 && !isspace((unsigned char)*p)) buf[n++] = *p++;
    buf[n] = 0;
    char *end = nullptr;
    *v = strtod(buf, &end);
    *ok = n > 0 && end == buf + n;
    return p;
}

// parse the entry lines in [b, e) (whole lines)
void parse_chunk(const char *b, const char *e, Field f, Sym sym, Parsed &out, bool *bad) {
    const char *p = b;
    while (p < e) {
        const char *nl = (const char *)memchr(p, '\n', e - p);
        const char *le = nl ? nl : e;
        const char *q = skip_ws(p, le);
        if (q < le && *q != '%') {
            uint64_t i, j;
            bool ok1, ok2, ok3 = true;
            q = parse_u64(q, le, &i, &ok1);
            q = parse_u64(q, le, &j, &ok2);
            int64_t xi = 1;
            double xd = 1.0;
            if (f == F_INTEGER) q = parse_i64(q, le, &xi, &ok3);
            if (f == F_REAL) q = parse_f64(q, le, &xd, &ok3);
            if (!ok1 || !ok2 || !ok3 || i == 0 || j == 0) {
                *bad = true;
                return;
            }
            out.I.push_back(i - 1);
            out.J.push_back(j - 1);
            if (f == F_INTEGER) out.Xi.push_back(xi);
            if (f == F_REAL) out.Xd.push_back(xd);
            if (sym != S_GENERAL && i != j) {
                out.I.push_back(j - 1);
                out.J.push_back(i - 1);
                if (f == F_INTEGER) out.Xi.push_back(sym == S_SKEW ? -xi : xi);
                if (f == F_REAL) out.Xd.push_back(sym == S_SKEW ? -xd : xd);
            }
        }
        p = nl ? nl + 1 : e;
    }
}

std::string lower(std::string s) {
    for (auto &c : s) c = (char)tolower((unsigned char)c);
    return s;
}
}  // namespace

extern "C" GrB_Info GxB_MatrixMarket_read_coo(const char *path, GrB_Index *nrows, GrB_Index *ncols,
                                              GrB_Index *nvals, int *type_code, GrB_Index **I, GrB_Index **J,
                                              void **X) {
    if (!path || !nrows || !ncols || !nvals || !type_code || !I || !J || !X) return GrB_NULL_POINTER;
    int fd = open(path, O_RDONLY);
    if (fd < 0) return GrB_INVALID_VALUE;
    struct stat st;
    if (fstat(fd, &st) != 0 || st.st_size == 0) {
        close(fd);
        return GrB_INVALID_VALUE;
    }
    const size_t size = (size_t)st.st_size;
    const char *base = (const char *)mmap(nullptr, size, PROT_READ, MAP_PRIVATE, fd, 0);
    close(fd);
    if (base == MAP_FAILED) return GrB_INVALID_VALUE;
    const char *end = base + size;
    auto fail = [&](GrB_Info info) {
        munmap((void *)base, size);
        return info;
    };
    // header: %%MatrixMarket matrix coordinate <field> <symmetry>
    const char *nl = (const char *)memchr(base, '\n', size);
    if (!nl) return fail(GrB_INVALID_VALUE);
    std::string hdr(base, nl - base), w[5];
    {
        size_t k = 0, pos = 0;
        while (k < 5 && pos < hdr.size()) {
            while (pos < hdr.size() && isspace((unsigned char)hdr[pos])) pos++;
            size_t s0 = pos;
            while (pos < hdr.size() && !isspace((unsigned char)hdr[pos])) pos++;
            if (pos > s0) w[k++] = lower(hdr.substr(s0, pos - s0));
        }
    }
    if (w[0] != "%%matrixmarket" || w[1] != "matrix" || w[2] != "coordinate") return fail(GrB_NOT_IMPLEMENTED);
    Field f;
    if (w[3] == "pattern") f = F_PATTERN;
    else if (w[3] == "integer") f = F_INTEGER;
    else if (w[3] == "real" || w[3] == "double") f = F_REAL;
    else return fail(GrB_NOT_IMPLEMENTED);  // complex: no complex types on this backend
    Sym sym;
    if (w[4] == "general") sym = S_GENERAL;
    else if (w[4] == "symmetric" || w[4] == "hermitian") sym = S_SYMMETRIC;
    else if (w[4] == "skew-symmetric") sym = S_SKEW;
    else return fail(GrB_INVALID_VALUE);
    // comments, then the size line
    const char *p = nl + 1;
    uint64_t nr = 0, nc = 0, nz = 0;
    for (;;) {
        if (p >= end) return fail(GrB_INVALID_VALUE);
        const char *le = (const char *)memchr(p, '\n', end - p);
        if (!le) le = end;
        const char *q = skip_ws(p, le);
        if (q < le && *q != '%') {
            bool a, b, c;
            q = parse_u64(q, le, &nr, &a);
            q = parse_u64(q, le, &nc, &b);
            q = parse_u64(q, le, &nz, &c);
            if (!a || !b || !c) return fail(GrB_INVALID_VALUE);
            p = le < end ? le + 1 : end;
            break;
        }
        p = le < end ? le + 1 : end;
    }
    // entry lines, split at line boundaries over the host threads
    unsigned nt = std::max(1u, std::min(64u, std::thread::hardware_concurrency()));
    if ((size_t)(end - p) < (1u << 20)) nt = 1;
    std::vector<const char *> cut(nt + 1);
    cut[0] = p;
    cut[nt] = end;
    for (unsigned t = 1; t < nt; t++) {
        const char *c = p + (size_t)(end - p) * t / nt;
        if (c < cut[t - 1]) c = cut[t - 1];
        const char *q = (const char *)memchr(c, '\n', end - c);
        cut[t] = q ? q + 1 : end;
    }
    std::vector<Parsed> parts(nt);
    std::vector<char> bad(nt, 0);
    std::vector<std::thread> th;
    for (unsigned t = 0; t < nt; t++)
        th.emplace_back([&, t] {
            bool b = false;
            parse_chunk(cut[t], cut[t + 1], f, sym, parts[t], &b);
            bad[t] = b;
        });
    for (auto &x : th) x.join();
    munmap((void *)base, size);
    for (unsigned t = 0; t < nt; t++)
        if (bad[t]) return GrB_INVALID_VALUE;
    size_t total = 0;
    for (auto &pt : parts) total += pt.I.size();
    const size_t expect_max = sym == S_GENERAL ? nz : 2 * nz;
    if ((sym == S_GENERAL && total != nz) || total > expect_max) return GrB_INVALID_VALUE;
    const size_t vs = f == F_PATTERN ? 1 : 8;
    GrB_Index *oi = (GrB_Index *)malloc(std::max<size_t>(total, 1) * sizeof(GrB_Index));
    GrB_Index *oj = (GrB_Index *)malloc(std::max<size_t>(total, 1) * sizeof(GrB_Index));
    void *ox = malloc(std::max<size_t>(total, 1) * vs);
    if (!oi || !oj || !ox) {
        free(oi);
        free(oj);
        free(ox);
        return GrB_OUT_OF_MEMORY;
    }
    size_t off = 0;
    for (auto &pt : parts) {
        const size_t m = pt.I.size();
        for (size_t k = 0; k < m; k++) {
            if (pt.I[k] >= nr || pt.J[k] >= nc) {
                free(oi);
                free(oj);
                free(ox);
                return GrB_INDEX_OUT_OF_BOUNDS;
            }
        }
        memcpy(oi + off, pt.I.data(), m * sizeof(GrB_Index));
        memcpy(oj + off, pt.J.data(), m * sizeof(GrB_Index));
        if (f == F_INTEGER) memcpy((int64_t *)ox + off, pt.Xi.data(), m * 8);
        if (f == F_REAL) memcpy((double *)ox + off, pt.Xd.data(), m * 8);
        if (f == F_PATTERN) memset((char *)ox + off, 1, m);
        off += m;
    }
    *nrows = nr;
    *ncols = nc;
    *nvals = total;
    *type_code = f == F_PATTERN ? GBAMD_T_BOOL : (f == F_INTEGER ? GBAMD_T_INT64 : GBAMD_T_FP64);
    *I = oi;
    *J = oj;
    *X = ox;
    return GrB_SUCCESS;
}

extern "C" GrB_Info GxB_MatrixMarket_free(void *p) {
    free(p);
    return GrB_SUCCESS;
}
