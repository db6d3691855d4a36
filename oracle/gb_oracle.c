/*
 * gb_oracle.c -- TEST INFRASTRUCTURE ONLY (see gb_oracle.h).
 *
 * Restatement of the GraphBLAS C API 2.0 mxm semantics that python-graphblas
 * relies on (reference core/base.py:23-54 -> SuiteSparse GrB_mxm; SURVEY.md
 * §8(a) rules 1-6), with SuiteSparse:GraphBLAS 7.4.x's published builtin-op
 * definitions for typecasting, integer division and boolean operator renaming.
 *
 * Determinism: every output entry is folded in ascending k order, so
 * floating-point plus_times is reproducible; integer ops wrap (two's
 * complement), as pinned by reference tests/test_matrix.py:4367 (test_power
 * overflows int64) and tests/test_ssjit.py:40 (-fwrapv).
 * The ANY monoid keeps the first (smallest-k) term.
 */
#include "gb_oracle.h"
#include <math.h>
#include <stdlib.h>
#include <string.h>

typedef union {
    int64_t i;
    uint64_t u;
    double f;
} gval;

enum { CL_BOOL, CL_SINT, CL_UINT, CL_FP32, CL_FP64 };

static int tclass(int t) {
    switch (t) {
    case GBAMD_T_BOOL: return CL_BOOL;
    case GBAMD_T_INT8: case GBAMD_T_INT16: case GBAMD_T_INT32: case GBAMD_T_INT64: return CL_SINT;
    case GBAMD_T_FP32: return CL_FP32;
    case GBAMD_T_FP64: return CL_FP64;
    default: return CL_UINT;
    }
}

static int tbits(int t) {
    switch (t) {
    case GBAMD_T_BOOL: return 1;
    case GBAMD_T_INT8: case GBAMD_T_UINT8: return 8;
    case GBAMD_T_INT16: case GBAMD_T_UINT16: return 16;
    case GBAMD_T_INT32: case GBAMD_T_UINT32: case GBAMD_T_FP32: return 32;
    default: return 64;
    }
}

int or_type_size(int t) {
    int b = tbits(t);
    return b == 1 ? 1 : b / 8;
}

/* wrap an integer to the width of type t (signed: sign-extend; unsigned: zero-extend) */
static gval wrap(int t, uint64_t r) {
    gval v;
    int b = tbits(t);
    if (tclass(t) == CL_SINT) {
        if (b == 64) v.i = (int64_t)r;
        else {
            uint64_t m = (1ULL << b) - 1, s = 1ULL << (b - 1);
            r &= m;
            v.i = (int64_t)((r ^ s) - s);
        }
    } else if (tclass(t) == CL_BOOL) {
        v.u = r != 0;
    } else {
        v.u = (b == 64) ? r : (r & ((1ULL << b) - 1));
    }
    return v;
}

static gval load(int t, const void *x, int64_t p) {
    gval v;
    switch (t) {
    case GBAMD_T_BOOL: v.u = ((const uint8_t *)x)[p] != 0; break;
    case GBAMD_T_INT8: v.i = ((const int8_t *)x)[p]; break;
    case GBAMD_T_UINT8: v.u = ((const uint8_t *)x)[p]; break;
    case GBAMD_T_INT16: v.i = ((const int16_t *)x)[p]; break;
    case GBAMD_T_UINT16: v.u = ((const uint16_t *)x)[p]; break;
    case GBAMD_T_INT32: v.i = ((const int32_t *)x)[p]; break;
    case GBAMD_T_UINT32: v.u = ((const uint32_t *)x)[p]; break;
    case GBAMD_T_INT64: v.i = ((const int64_t *)x)[p]; break;
    case GBAMD_T_UINT64: v.u = ((const uint64_t *)x)[p]; break;
    case GBAMD_T_FP32: v.f = ((const float *)x)[p]; break;
    default: v.f = ((const double *)x)[p]; break;
    }
    return v;
}

static void store(int t, void *x, int64_t p, gval v) {
    switch (t) {
    case GBAMD_T_BOOL: ((uint8_t *)x)[p] = (uint8_t)(v.u != 0); break;
    case GBAMD_T_INT8: ((int8_t *)x)[p] = (int8_t)v.i; break;
    case GBAMD_T_UINT8: ((uint8_t *)x)[p] = (uint8_t)v.u; break;
    case GBAMD_T_INT16: ((int16_t *)x)[p] = (int16_t)v.i; break;
    case GBAMD_T_UINT16: ((uint16_t *)x)[p] = (uint16_t)v.u; break;
    case GBAMD_T_INT32: ((int32_t *)x)[p] = (int32_t)v.i; break;
    case GBAMD_T_UINT32: ((uint32_t *)x)[p] = (uint32_t)v.u; break;
    case GBAMD_T_INT64: ((int64_t *)x)[p] = v.i; break;
    case GBAMD_T_UINT64: ((uint64_t *)x)[p] = v.u; break;
    case GBAMD_T_FP32: ((float *)x)[p] = (float)v.f; break;
    default: ((double *)x)[p] = v.f; break;
    }
}

/* SuiteSparse GB_cast_to_int*: NaN -> 0, saturate at the type's range, else truncate */
static gval f2int(int t, double d) {
    gval v;
    int b = tbits(t);
    if (tclass(t) == CL_SINT) {
        double lo = -ldexp(1.0, b - 1), hi = ldexp(1.0, b - 1);
        if (isnan(d)) v.i = 0;
        else if (d <= lo) v.i = (b == 64) ? INT64_MIN : -(int64_t)(1LL << (b - 1));
        else if (d >= hi) v.i = (b == 64) ? INT64_MAX : (int64_t)((1LL << (b - 1)) - 1);
        else v.i = (int64_t)d;
    } else {
        double hi = ldexp(1.0, b);
        if (isnan(d) || d <= 0) v.u = 0;
        else if (d >= hi) v.u = (b == 64) ? UINT64_MAX : ((1ULL << b) - 1);
        else v.u = (uint64_t)d;
    }
    return v;
}

static double as_double(int t, gval v) {
    switch (tclass(t)) {
    case CL_SINT: return (double)v.i;
    case CL_FP32: case CL_FP64: return v.f;
    default: return (double)v.u;
    }
}

static gval cast(int from, int to, gval v) {
    if (from == to) return v;
    int cf = tclass(from), ct = tclass(to);
    gval r;
    if (ct == CL_BOOL) {
        if (cf == CL_FP32 || cf == CL_FP64) r.u = (v.f != 0);
        else r.u = (v.u != 0);
        return r;
    }
    if (cf == CL_FP32 || cf == CL_FP64) {
        if (ct == CL_FP32) { r.f = (float)v.f; return r; }
        if (ct == CL_FP64) { r.f = v.f; return r; }
        return f2int(to, v.f);
    }
    /* from integer / bool */
    if (ct == CL_FP32) { r.f = (cf == CL_SINT) ? (double)(float)v.i : (double)(float)v.u; return r; }
    if (ct == CL_FP64) { r.f = (cf == CL_SINT) ? (double)v.i : (double)v.u; return r; }
    return wrap(to, v.u);
}

static gval mkbool(int b) { gval v; v.u = b ? 1 : 0; return v; }

/* value of "1" / "0" in type t */
static gval one(int t) {
    gval v;
    if (tclass(t) == CL_FP32 || tclass(t) == CL_FP64) v.f = 1.0;
    else v.u = 1;
    return v;
}
static gval zero(int t) {
    gval v;
    if (tclass(t) == CL_FP32 || tclass(t) == CL_FP64) v.f = 0.0;
    else v.u = 0;
    return v;
}

static int nz(int t, gval v) {
    int c = tclass(t);
    return (c == CL_FP32 || c == CL_FP64) ? (v.f != 0) : (v.u != 0);
}

/* comparisons within type t: returns -1, 0, 1, or 2 for unordered (NaN) */
static int cmp(int t, gval x, gval y) {
    switch (tclass(t)) {
    case CL_SINT: return (x.i < y.i) ? -1 : (x.i > y.i);
    case CL_FP32: case CL_FP64:
        if (isnan(x.f) || isnan(y.f)) return 2;
        return (x.f < y.f) ? -1 : (x.f > y.f);
    default: return (x.u < y.u) ? -1 : (x.u > y.u);
    }
}

/* SuiteSparse GB_IDIV_SIGNED / GB_IDIV_UNSIGNED */
static gval idiv(int t, gval x, gval y) {
    if (tclass(t) == CL_SINT) {
        int b = tbits(t);
        int64_t mx = (b == 64) ? INT64_MAX : (int64_t)((1LL << (b - 1)) - 1);
        int64_t mn = (b == 64) ? INT64_MIN : -(int64_t)(1LL << (b - 1));
        gval r;
        if (y.i == -1) return wrap(t, (uint64_t)0 - x.u);
        if (y.i == 0) { r.i = (x.i == 0) ? 0 : (x.i < 0 ? mn : mx); return r; }
        r.i = x.i / y.i;
        return r;
    } else {
        int b = tbits(t);
        gval r;
        if (y.u == 0) { r.u = (x.u == 0) ? 0 : ((b == 64) ? UINT64_MAX : ((1ULL << b) - 1)); return r; }
        r.u = x.u / y.u;
        return r;
    }
}

static int is_float(int t) { int c = tclass(t); return c == CL_FP32 || c == CL_FP64; }

static gval fround(int t, double d) {
    gval v;
    v.f = (t == GBAMD_T_FP32) ? (double)(float)d : d;
    return v;
}

/* boolean operator renaming (SuiteSparse GB_boolean_rename) */
static int bool_rename(int op) {
    switch (op) {
    case GBAMD_OP_PLUS: case GBAMD_OP_MAX: return GBAMD_OP_LOR;
    case GBAMD_OP_TIMES: case GBAMD_OP_MIN: return GBAMD_OP_LAND;
    case GBAMD_OP_MINUS: case GBAMD_OP_RMINUS: case GBAMD_OP_ISNE: case GBAMD_OP_NE: return GBAMD_OP_LXOR;
    case GBAMD_OP_DIV: return GBAMD_OP_FIRST;
    case GBAMD_OP_RDIV: return GBAMD_OP_SECOND;
    case GBAMD_OP_ISEQ: case GBAMD_OP_EQ: return GBAMD_OP_LXNOR;
    case GBAMD_OP_ISGT: return GBAMD_OP_GT;
    case GBAMD_OP_ISLT: return GBAMD_OP_LT;
    case GBAMD_OP_ISGE: return GBAMD_OP_GE;
    case GBAMD_OP_ISLE: return GBAMD_OP_LE;
    default: return op;
    }
}

/* z = op(x, y) with x, y in type t.  Positional ops use (i, k, j). */
static gval binop(int op, int t, gval x, gval y, int64_t i, int64_t k, int64_t j, int zt) {
    gval r;
    switch (op) {
    case GBAMD_OP_FIRSTI: return wrap(zt, (uint64_t)i);
    case GBAMD_OP_FIRSTI1: return wrap(zt, (uint64_t)(i + 1));
    case GBAMD_OP_FIRSTJ: return wrap(zt, (uint64_t)k);
    case GBAMD_OP_FIRSTJ1: return wrap(zt, (uint64_t)(k + 1));
    case GBAMD_OP_SECONDI: return wrap(zt, (uint64_t)k);
    case GBAMD_OP_SECONDI1: return wrap(zt, (uint64_t)(k + 1));
    case GBAMD_OP_SECONDJ: return wrap(zt, (uint64_t)j);
    case GBAMD_OP_SECONDJ1: return wrap(zt, (uint64_t)(j + 1));
    default: break;
    }
    if (t == GBAMD_T_BOOL) op = bool_rename(op);
    int c;
    switch (op) {
    case GBAMD_OP_FIRST: return x;
    case GBAMD_OP_SECOND: case GBAMD_OP_ANY: return y;
    case GBAMD_OP_PAIR: return one(t);
    case GBAMD_OP_LOR: return nz(t, x) || nz(t, y) ? one(t) : zero(t);
    case GBAMD_OP_LAND: return nz(t, x) && nz(t, y) ? one(t) : zero(t);
    case GBAMD_OP_LXOR: return (nz(t, x) != nz(t, y)) ? one(t) : zero(t);
    case GBAMD_OP_LXNOR: return (nz(t, x) == nz(t, y)) ? one(t) : zero(t);
    case GBAMD_OP_EQ: c = cmp(t, x, y); return mkbool(c == 0);
    case GBAMD_OP_NE: c = cmp(t, x, y); return mkbool(c != 0);
    case GBAMD_OP_GT: c = cmp(t, x, y); return mkbool(c == 1);
    case GBAMD_OP_LT: c = cmp(t, x, y); return mkbool(c == -1);
    case GBAMD_OP_GE: c = cmp(t, x, y); return mkbool(c == 1 || c == 0);
    case GBAMD_OP_LE: c = cmp(t, x, y); return mkbool(c == -1 || c == 0);
    case GBAMD_OP_ISEQ: c = cmp(t, x, y); return (c == 0) ? one(t) : zero(t);
    case GBAMD_OP_ISNE: c = cmp(t, x, y); return (c != 0) ? one(t) : zero(t);
    case GBAMD_OP_ISGT: c = cmp(t, x, y); return (c == 1) ? one(t) : zero(t);
    case GBAMD_OP_ISLT: c = cmp(t, x, y); return (c == -1) ? one(t) : zero(t);
    case GBAMD_OP_ISGE: c = cmp(t, x, y); return (c == 1 || c == 0) ? one(t) : zero(t);
    case GBAMD_OP_ISLE: c = cmp(t, x, y); return (c == -1 || c == 0) ? one(t) : zero(t);
    default: break;
    }
    if (is_float(t)) {
        double a = x.f, b = y.f;
        if (t == GBAMD_T_FP32) {
            float fa = (float)a, fb = (float)b;
            switch (op) {
            case GBAMD_OP_MIN: r.f = fminf(fa, fb); return r;
            case GBAMD_OP_MAX: r.f = fmaxf(fa, fb); return r;
            case GBAMD_OP_PLUS: r.f = fa + fb; return r;
            case GBAMD_OP_MINUS: r.f = fa - fb; return r;
            case GBAMD_OP_RMINUS: r.f = fb - fa; return r;
            case GBAMD_OP_TIMES: r.f = fa * fb; return r;
            case GBAMD_OP_DIV: r.f = fa / fb; return r;
            case GBAMD_OP_RDIV: r.f = fb / fa; return r;
            case GBAMD_OP_POW: r.f = powf(fa, fb); return r;
            default: break;
            }
        } else {
            switch (op) {
            case GBAMD_OP_MIN: r.f = fmin(a, b); return r;
            case GBAMD_OP_MAX: r.f = fmax(a, b); return r;
            case GBAMD_OP_PLUS: r.f = a + b; return r;
            case GBAMD_OP_MINUS: r.f = a - b; return r;
            case GBAMD_OP_RMINUS: r.f = b - a; return r;
            case GBAMD_OP_TIMES: r.f = a * b; return r;
            case GBAMD_OP_DIV: r.f = a / b; return r;
            case GBAMD_OP_RDIV: r.f = b / a; return r;
            case GBAMD_OP_POW: r.f = pow(a, b); return r;
            default: break;
            }
        }
        return fround(t, 0.0);
    }
    /* integers (bool has been renamed to logical ops above) */
    int sgn = tclass(t) == CL_SINT;
    switch (op) {
    case GBAMD_OP_MIN: return (sgn ? (x.i < y.i) : (x.u < y.u)) ? x : y;
    case GBAMD_OP_MAX: return (sgn ? (x.i > y.i) : (x.u > y.u)) ? x : y;
    case GBAMD_OP_PLUS: return wrap(t, x.u + y.u);
    case GBAMD_OP_MINUS: return wrap(t, x.u - y.u);
    case GBAMD_OP_RMINUS: return wrap(t, y.u - x.u);
    case GBAMD_OP_TIMES: return wrap(t, x.u * y.u);
    case GBAMD_OP_DIV: return idiv(t, x, y);
    case GBAMD_OP_RDIV: return idiv(t, y, x);
    case GBAMD_OP_POW: return f2int(t, pow(as_double(t, x), as_double(t, y)));
    case GBAMD_OP_BOR: return wrap(t, x.u | y.u);
    case GBAMD_OP_BAND: return wrap(t, x.u & y.u);
    case GBAMD_OP_BXOR: return wrap(t, x.u ^ y.u);
    case GBAMD_OP_BXNOR: return wrap(t, ~(x.u ^ y.u));
    default: break;
    }
    return zero(t);
}

/* monoid fold: acc (+) z, both in type t.  ANY keeps the first term. */
static gval monoid(int mon, int t, gval acc, gval z) {
    switch (mon) {
    case GBAMD_MON_ANY: return acc;
    case GBAMD_MON_PLUS: return binop(GBAMD_OP_PLUS, t, acc, z, 0, 0, 0, t);
    case GBAMD_MON_TIMES: return binop(GBAMD_OP_TIMES, t, acc, z, 0, 0, 0, t);
    case GBAMD_MON_MIN: return binop(GBAMD_OP_MIN, t, acc, z, 0, 0, 0, t);
    case GBAMD_MON_MAX: return binop(GBAMD_OP_MAX, t, acc, z, 0, 0, 0, t);
    case GBAMD_MON_LOR: return binop(GBAMD_OP_LOR, t, acc, z, 0, 0, 0, t);
    case GBAMD_MON_LAND: return binop(GBAMD_OP_LAND, t, acc, z, 0, 0, 0, t);
    case GBAMD_MON_LXOR: return binop(GBAMD_OP_LXOR, t, acc, z, 0, 0, 0, t);
    case GBAMD_MON_LXNOR: return binop(GBAMD_OP_LXNOR, t, acc, z, 0, 0, 0, t);
    case GBAMD_MON_BOR: return binop(GBAMD_OP_BOR, t, acc, z, 0, 0, 0, t);
    case GBAMD_MON_BAND: return binop(GBAMD_OP_BAND, t, acc, z, 0, 0, 0, t);
    case GBAMD_MON_BXOR: return binop(GBAMD_OP_BXOR, t, acc, z, 0, 0, 0, t);
    case GBAMD_MON_BXNOR: return binop(GBAMD_OP_BXNOR, t, acc, z, 0, 0, 0, t);
    default: return acc;
    }
}

void or_csr_free(or_csr *m) {
    if (!m) return;
    free(m->p); free(m->j); free(m->x);
    m->p = NULL; m->j = NULL; m->x = NULL;
}

static void *xmalloc(size_t n) { return malloc(n ? n : 1); }

int or_transpose(or_csr *out, const or_csr *a) {
    int64_t tnz = a->p[a->nrows];
    int sz = or_type_size(a->type);
    out->nrows = a->ncols; out->ncols = a->nrows; out->type = a->type;
    out->p = (int64_t *)calloc((size_t)out->nrows + 1, sizeof(int64_t));
    out->j = (int64_t *)xmalloc((size_t)tnz * sizeof(int64_t));
    out->x = a->x ? xmalloc((size_t)tnz * sz) : NULL;
    for (int64_t q = 0; q < tnz; q++) out->p[a->j[q] + 1]++;
    for (int64_t r = 0; r < out->nrows; r++) out->p[r + 1] += out->p[r];
    int64_t *w = (int64_t *)xmalloc((size_t)(out->nrows + 1) * sizeof(int64_t));
    memcpy(w, out->p, (size_t)(out->nrows + 1) * sizeof(int64_t));
    for (int64_t i = 0; i < a->nrows; i++)
        for (int64_t q = a->p[i]; q < a->p[i + 1]; q++) {
            int64_t d = w[a->j[q]]++;
            out->j[d] = i;
            if (a->x) memcpy((char *)out->x + d * sz, (const char *)a->x + q * sz, sz);
        }
    free(w);
    return 0;
}

/* growable output builder */
typedef struct { int64_t n, cap; int64_t *j; gval *v; } obuf;
static void ob_push(obuf *b, int64_t j, gval v) {
    if (b->n == b->cap) {
        b->cap = b->cap ? 2 * b->cap : 1024;
        b->j = (int64_t *)realloc(b->j, (size_t)b->cap * sizeof(int64_t));
        b->v = (gval *)realloc(b->v, (size_t)b->cap * sizeof(gval));
    }
    b->j[b->n] = j; b->v[b->n] = v; b->n++;
}

static int cmp_i64(const void *a, const void *b) {
    int64_t x = *(const int64_t *)a, y = *(const int64_t *)b;
    return (x > y) - (x < y);
}

/* T = A (+).(x) B   (A, B already transposed as requested; values loaded as
 * type ta / tb then cast to the multiplier input type).  T rows into
 * tp (nrows+1) / tbuf (values in ztype). */
static void compute_T(const or_csr *A, const or_csr *B, const or_csr *BT,
                      const or_csr *Mf, /* structural filtered mask or NULL (dot method) */
                      int add_mon, int mul_op, int xt, int zt,
                      int64_t *tp, obuf *tb) {
    int64_t n = A->nrows, m = B->ncols;
    int positional = xt < 0;
    if (Mf) {
        /* masked dot product ("dot3"): T(i,j) for (i,j) in M only, folded in ascending k */
        for (int64_t i = 0; i < n; i++) {
            tp[i] = tb->n;
            for (int64_t q = Mf->p[i]; q < Mf->p[i + 1]; q++) {
                int64_t j = Mf->j[q];
                int64_t pa = A->p[i], ea = A->p[i + 1], pb = BT->p[j], eb = BT->p[j + 1];
                int found = 0;
                gval acc; acc.u = 0;
                while (pa < ea && pb < eb) {
                    int64_t ka = A->j[pa], kb = BT->j[pb];
                    if (ka < kb) pa++;
                    else if (kb < ka) pb++;
                    else {
                        gval x, y, z;
                        x.u = 0; y.u = 0;
                        if (!positional) {
                            x = cast(A->type, xt, load(A->type, A->x, pa));
                            y = cast(BT->type, xt, load(BT->type, BT->x, pb));
                        }
                        z = binop(mul_op, positional ? zt : xt, x, y, i, ka, j, zt);
                        acc = found ? monoid(add_mon, zt, acc, z) : z;
                        found = 1;
                        pa++; pb++;
                    }
                }
                if (found) ob_push(tb, j, acc);
            }
        }
        tp[n] = tb->n;
        return;
    }
    /* Gustavson, row by row, k ascending => each T(i,j) folded in ascending k */
    int64_t *mark = (int64_t *)xmalloc((size_t)(m ? m : 1) * sizeof(int64_t));
    gval *spa = (gval *)xmalloc((size_t)(m ? m : 1) * sizeof(gval));
    int64_t *list = (int64_t *)xmalloc((size_t)(m ? m : 1) * sizeof(int64_t));
    for (int64_t j = 0; j < m; j++) mark[j] = -1;
    for (int64_t i = 0; i < n; i++) {
        int64_t cnt = 0;
        tp[i] = tb->n;
        for (int64_t pa = A->p[i]; pa < A->p[i + 1]; pa++) {
            int64_t k = A->j[pa];
            gval x; x.u = 0;
            if (!positional) x = cast(A->type, xt, load(A->type, A->x, pa));
            for (int64_t pb = B->p[k]; pb < B->p[k + 1]; pb++) {
                int64_t j = B->j[pb];
                gval y, z;
                y.u = 0;
                if (!positional) y = cast(B->type, xt, load(B->type, B->x, pb));
                z = binop(mul_op, positional ? zt : xt, x, y, i, k, j, zt);
                if (mark[j] != i) { mark[j] = i; spa[j] = z; list[cnt++] = j; }
                else spa[j] = monoid(add_mon, zt, spa[j], z);
            }
        }
        qsort(list, (size_t)cnt, sizeof(int64_t), cmp_i64);
        for (int64_t c = 0; c < cnt; c++) ob_push(tb, list[c], spa[list[c]]);
    }
    tp[n] = tb->n;
    free(mark); free(spa); free(list);
}

/* structural copy of M keeping entries whose mask value is true (value mask) */
static void mask_filter(or_csr *out, const or_csr *M, int structural) {
    int64_t n = M->nrows, mnz = M->p[n];
    out->nrows = M->nrows; out->ncols = M->ncols; out->type = GBAMD_T_BOOL; out->x = NULL;
    out->p = (int64_t *)xmalloc((size_t)(n + 1) * sizeof(int64_t));
    out->j = (int64_t *)xmalloc((size_t)mnz * sizeof(int64_t));
    int64_t c = 0;
    for (int64_t i = 0; i < n; i++) {
        out->p[i] = c;
        for (int64_t q = M->p[i]; q < M->p[i + 1]; q++) {
            if (structural || !M->x || nz(M->type, load(M->type, M->x, q))) out->j[c++] = M->j[q];
        }
    }
    out->p[n] = c;
}

int or_mxm(or_csr *C, const or_csr *M, int mask_comp, int mask_struct, int replace,
           int accum_op, int accum_type, int accum_ztype,
           int add_mon, int mul_op, int sr_xtype, int sr_ztype,
           const or_csr *A0, int tran0, const or_csr *B0, int tran1) {
    or_csr At = {0}, Bt = {0}, BT = {0}, Mf = {0};
    const or_csr *A = A0, *B = B0;
    if (tran0) { or_transpose(&At, A0); A = &At; }
    if (tran1) { or_transpose(&Bt, B0); B = &Bt; }
    if (A->ncols != B->nrows || C->nrows != A->nrows || C->ncols != B->ncols ||
        (M && (M->nrows != C->nrows || M->ncols != C->ncols))) {
        or_csr_free(&At); or_csr_free(&Bt);
        return -6;
    }
    int64_t n = C->nrows, m = C->ncols;
    if (M) mask_filter(&Mf, M, mask_struct);
    int use_dot = (M && !mask_comp);
    if (use_dot) or_transpose(&BT, B);

    /* 1. T */
    int64_t *tp = (int64_t *)xmalloc((size_t)(n + 1) * sizeof(int64_t));
    obuf tb = {0, 0, NULL, NULL};
    compute_T(A, B, &BT, use_dot ? &Mf : NULL, add_mon, mul_op, sr_xtype, sr_ztype, tp, &tb);

    /* 2-4. Z = C (accum) T; mask; replace; write back (SURVEY §8(a) rules 2-4) */
    int ct = C->type, zt = sr_ztype;
    int csz = or_type_size(ct);
    int64_t cap = C->p[n] + tb.n;
    int64_t *np = (int64_t *)xmalloc((size_t)(n + 1) * sizeof(int64_t));
    int64_t *nj = (int64_t *)xmalloc((size_t)(cap ? cap : 1) * sizeof(int64_t));
    char *nx = (char *)xmalloc((size_t)(cap ? cap : 1) * csz);
    char *mrow = (char *)calloc((size_t)(m ? m : 1), 1);
    int64_t c = 0;
    for (int64_t i = 0; i < n; i++) {
        np[i] = c;
        if (M) for (int64_t q = Mf.p[i]; q < Mf.p[i + 1]; q++) mrow[Mf.j[q]] = 1;
        int64_t pc = C->p[i], ec = C->p[i + 1], pt = tp[i], et = tp[i + 1];
        while (pc < ec || pt < et) {
            int64_t jc = pc < ec ? C->j[pc] : INT64_MAX;
            int64_t jt = pt < et ? tb.j[pt] : INT64_MAX;
            int64_t j = jc < jt ? jc : jt;
            int inC = (jc == j), inT = (jt == j);
            int mk = M ? mrow[j] : 1;
            if (mask_comp) mk = !mk;
            int have = 0;
            gval out; out.u = 0;
            if (mk) {
                if (accum_op >= 0 && inC && inT) {
                    gval cx = cast(ct, accum_type, load(ct, C->x, pc));
                    gval tx = cast(zt, accum_type, tb.v[pt]);
                    gval z = binop(accum_op, accum_type, cx, tx, 0, 0, 0, accum_ztype);
                    out = cast(accum_ztype, ct, z);
                    have = 1;
                } else if (inT) {
                    out = cast(zt, ct, tb.v[pt]);
                    have = 1;
                } else if (accum_op >= 0 && inC) {
                    out = load(ct, C->x, pc);
                    have = 1;
                }
            } else if (!replace && inC) {
                out = load(ct, C->x, pc);
                have = 1;
            }
            if (have) { nj[c] = j; store(ct, nx, c, out); c++; }
            if (inC) pc++;
            if (inT) pt++;
        }
        if (M) for (int64_t q = Mf.p[i]; q < Mf.p[i + 1]; q++) mrow[Mf.j[q]] = 0;
    }
    np[n] = c;
    free(mrow); free(tp); free(tb.j); free(tb.v);
    or_csr_free(&At); or_csr_free(&Bt); or_csr_free(&BT); or_csr_free(&Mf);
    /* the caller owns C's previous arrays; the new ones are malloc'ed here */
    C->p = np; C->j = nj; C->x = nx;
    return 0;
}

/* ---------------------------------------------------------------- R-MAT */
static uint64_t smix(uint64_t x) {
    x += 0x9E3779B97F4A7C15ULL;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ULL;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBULL;
    return x ^ (x >> 31);
}

/* bijective scramble of a scale-bit vertex label */
static uint64_t scramble(uint64_t v, int scale, uint64_t seed) {
    uint64_t mask = (scale >= 64) ? ~0ULL : ((1ULL << scale) - 1);
    uint64_t k1 = smix(seed ^ 0x5851F42D4C957F2DULL) | 1ULL, k2 = smix(seed ^ 0x14057B7EF767814FULL);
    for (int r = 0; r < 3; r++) {
        v = (v * k1) & mask;
        v ^= (v >> ((scale + 1) / 2));
        v = (v + k2) & mask;
    }
    return v;
}

/* thresholds of the quadrant probabilities in units of 2^-53 */
#define RM_A 5134103575202365ULL  /* floor(0.57 * 2^53) */
#define RM_B 6845471433603153ULL  /* floor(0.76 * 2^53) */
#define RM_C 8556839292003942ULL  /* floor(0.95 * 2^53) */

int or_rmat(or_csr *out, int scale, int edge_factor, uint64_t seed) {
    int64_t n = 1LL << scale, ne = (int64_t)edge_factor << scale;
    uint64_t *k = (uint64_t *)xmalloc((size_t)ne * sizeof(uint64_t));
    uint64_t *t = (uint64_t *)xmalloc((size_t)ne * sizeof(uint64_t));
    uint64_t s0 = smix(seed);
    int64_t m = 0;
    for (int64_t e = 0; e < ne; e++) {
        uint64_t r = 0, c = 0;
        for (int l = 0; l < scale; l++) {
            uint64_t h = smix(s0 ^ ((uint64_t)e * 64 + (uint64_t)l)) >> 11;
            uint64_t rb = (h >= RM_B), cb = (h >= RM_A && h < RM_B) || (h >= RM_C);
            r |= rb << l; c |= cb << l;
        }
        r = scramble(r, scale, seed);
        c = scramble(c, scale, seed);
        if (r != c) k[m++] = (r << 32) | c;
    }
    int passes = 0;
    uint64_t *a = k, *b = t;
    int64_t cnt[65536];
    for (int shift = 0; shift < 2 * 32 && shift < 32 + scale; shift += 16) {
        if (shift >= scale && shift < 32) continue;  /* column bits above scale are zero */
        memset(cnt, 0, sizeof(cnt));
        for (int64_t q = 0; q < m; q++) cnt[(a[q] >> shift) & 0xFFFF]++;
        int64_t s = 0;
        for (int d = 0; d < 65536; d++) { int64_t x = cnt[d]; cnt[d] = s; s += x; }
        for (int64_t q = 0; q < m; q++) b[cnt[(a[q] >> shift) & 0xFFFF]++] = a[q];
        uint64_t *x = a; a = b; b = x; passes++;
    }
    out->nrows = n; out->ncols = n; out->type = GBAMD_T_BOOL; out->x = NULL;
    out->p = (int64_t *)calloc((size_t)n + 1, sizeof(int64_t));
    out->j = (int64_t *)xmalloc((size_t)m * sizeof(int64_t));
    int64_t u = 0;
    for (int64_t q = 0; q < m; q++) {
        if (q > 0 && a[q] == a[q - 1]) continue;
        out->j[u++] = (int64_t)(a[q] & 0xFFFFFFFFULL);
        out->p[(a[q] >> 32) + 1]++;
    }
    for (int64_t i = 0; i < n; i++) out->p[i + 1] += out->p[i];
    free(k); free(t);
    return 0;
}

int or_rmat_values(or_csr *mtx, int kind, uint64_t seed) {
    int64_t n = mtx->nrows, vnz = mtx->p[n];
    uint64_t s0 = smix(seed ^ 0xA0761D6478BD642FULL);
    if (kind == 0) {
        int64_t *x = (int64_t *)xmalloc((size_t)vnz * sizeof(int64_t));
        for (int64_t i = 0; i < n; i++)
            for (int64_t q = mtx->p[i]; q < mtx->p[i + 1]; q++)
                x[q] = 1 + (int64_t)(smix(s0 ^ (((uint64_t)i << 32) | (uint64_t)mtx->j[q])) % 255);
        free(mtx->x); mtx->x = x; mtx->type = GBAMD_T_INT64;
    } else {
        double *x = (double *)xmalloc((size_t)vnz * sizeof(double));
        for (int64_t i = 0; i < n; i++)
            for (int64_t q = mtx->p[i]; q < mtx->p[i + 1]; q++)
                x[q] = (double)(smix(s0 ^ (((uint64_t)i << 32) | (uint64_t)mtx->j[q])) >> 11) * 0x1.0p-53;
        free(mtx->x); mtx->x = x; mtx->type = GBAMD_T_FP64;
    }
    return 0;
}

int or_bfs_levels(const or_csr *A, int64_t src, int32_t *levels, int64_t *edges) {
    int64_t n = A->nrows;
    int64_t *q = (int64_t *)xmalloc((size_t)n * sizeof(int64_t));
    int64_t *nq = (int64_t *)xmalloc((size_t)n * sizeof(int64_t));
    memset(levels, 0, (size_t)n * sizeof(int32_t));
    int64_t qn = 1, e = 0;
    int lev = 1;
    q[0] = src; levels[src] = 1;
    while (qn > 0) {
        int64_t nn = 0;
        for (int64_t a = 0; a < qn; a++) {
            int64_t v = q[a];
            e += A->p[v + 1] - A->p[v];
            for (int64_t p = A->p[v]; p < A->p[v + 1]; p++) {
                int64_t w = A->j[p];
                if (!levels[w]) { levels[w] = lev + 1; nq[nn++] = w; }
            }
        }
        int64_t *t = q; q = nq; nq = t; qn = nn;
        if (qn) lev++;
    }
    free(q); free(nq);
    if (edges) *edges = e;
    return lev;
}

/* The same level BFS as or_bfs_levels -- per level q(~v.S, replace) = q lor.land A,
 * the masked vxm of the reference notebook loop (Example B.1 cell 8) -- run on
 * `nthreads` host threads the way a CPU GraphBLAS library runs a masked vxm with
 * a bitmap frontier: push (saxpy over the frontier's rows of A) or pull (dot over
 * the unvisited rows of A^T, stopping at the first frontier hit), chosen per level
 * by Beamer's rule (frontier edges x 14 > unvisited edges -> pull).  CPU BASELINE
 * ONLY (bench.py cpu_baseline); same levels as or_bfs_levels. */
int or_bfs_levels_par(const or_csr *A, const or_csr *AT, int64_t src, int32_t *levels, int64_t *edges,
                      int nthreads) {
    const int64_t n = A->nrows, nw = (n + 63) / 64, nnz = A->p[n];
    if (nthreads < 1) nthreads = 1;
    int64_t *q = (int64_t *)xmalloc((size_t)(n ? n : 1) * sizeof(int64_t));
    int64_t *nq = (int64_t *)xmalloc((size_t)(n ? n : 1) * sizeof(int64_t));
    uint64_t *fb = (uint64_t *)calloc((size_t)(nw ? nw : 1), sizeof(uint64_t));
    memset(levels, 0, (size_t)n * sizeof(int32_t));
    int64_t qn = 1, e = 0, open_edges = nnz;
    int lev = 1;
    q[0] = src; levels[src] = 1;
    while (qn > 0) {
        int64_t mf = 0;
#pragma omp parallel for num_threads(nthreads) reduction(+ : mf) schedule(static)
        for (int64_t a = 0; a < qn; a++) mf += A->p[q[a] + 1] - A->p[q[a]];
        e += mf;
        open_edges -= mf;
        const int pull = AT && mf * 14 > open_edges;
        int64_t nn = 0;
        if (pull) {
#pragma omp parallel for num_threads(nthreads) schedule(static)
            for (int64_t a = 0; a < qn; a++)
                __atomic_fetch_or(&fb[q[a] >> 6], 1ULL << (q[a] & 63), __ATOMIC_RELAXED);
#pragma omp parallel num_threads(nthreads)
            {
                int64_t cap = 4096, cnt = 0;
                int64_t *buf = (int64_t *)xmalloc((size_t)cap * sizeof(int64_t));
#pragma omp for schedule(dynamic, 4096) nowait
                for (int64_t w = 0; w < n; w++) {
                    if (levels[w]) continue;
                    for (int64_t p = AT->p[w]; p < AT->p[w + 1]; p++) {
                        const int64_t k = AT->j[p];
                        if ((fb[k >> 6] >> (k & 63)) & 1) {
                            if (cnt == cap) buf = (int64_t *)realloc(buf, (size_t)(cap *= 2) * sizeof(int64_t));
                            buf[cnt++] = w;
                            break;
                        }
                    }
                }
                const int64_t at = __atomic_fetch_add(&nn, cnt, __ATOMIC_RELAXED);
                memcpy(nq + at, buf, (size_t)cnt * sizeof(int64_t));
                free(buf);
            }
#pragma omp parallel for num_threads(nthreads) schedule(static)
            for (int64_t a = 0; a < qn; a++) fb[q[a] >> 6] = 0;
#pragma omp parallel for num_threads(nthreads) schedule(static)
            for (int64_t a = 0; a < nn; a++) levels[nq[a]] = lev + 1;
        } else {
#pragma omp parallel num_threads(nthreads)
            {
                int64_t cap = 4096, cnt = 0;
                int64_t *buf = (int64_t *)xmalloc((size_t)cap * sizeof(int64_t));
#pragma omp for schedule(dynamic, 16) nowait
                for (int64_t a = 0; a < qn; a++) {
                    const int64_t v = q[a];
                    for (int64_t p = A->p[v]; p < A->p[v + 1]; p++) {
                        const int64_t w = A->j[p];
                        int32_t zero = 0;
                        if (!__atomic_load_n(&levels[w], __ATOMIC_RELAXED) &&
                            __atomic_compare_exchange_n(&levels[w], &zero, lev + 1, 0, __ATOMIC_RELAXED,
                                                        __ATOMIC_RELAXED)) {
                            if (cnt == cap) buf = (int64_t *)realloc(buf, (size_t)(cap *= 2) * sizeof(int64_t));
                            buf[cnt++] = w;
                        }
                    }
                }
                const int64_t at = __atomic_fetch_add(&nn, cnt, __ATOMIC_RELAXED);
                memcpy(nq + at, buf, (size_t)cnt * sizeof(int64_t));
                free(buf);
            }
        }
        int64_t *t = q; q = nq; nq = t; qn = nn;
        if (qn) lev++;
    }
    free(q); free(nq); free(fb);
    if (edges) *edges = e;
    return lev;
}

/* Level BFS exactly as the reference notebook loop (Example B.1 cell 8), every
 * step through or_mxm:  v[:](mask=q.V) << d ; q(~v.S, replace) << q.vxm(A, lor_land).
 * This is the CPU baseline "port" of the GraphBLAS formulation. */
int or_bfs_graphblas(const or_csr *A, int64_t src, int32_t *levels, int64_t *edges) {
    int64_t n = A->nrows;
    memset(levels, 0, (size_t)n * sizeof(int32_t));
    /* q: 1 x n BOOL row */
    or_csr q = {1, n, GBAMD_T_BOOL, NULL, NULL, NULL};
    q.p = (int64_t *)xmalloc(2 * sizeof(int64_t));
    q.j = (int64_t *)xmalloc(sizeof(int64_t));
    q.x = xmalloc(1);
    q.p[0] = 0; q.p[1] = 1; q.j[0] = src; ((uint8_t *)q.x)[0] = 1;
    /* v: visited structure as a 1 x n row (values unused: structural mask) */
    or_csr v = {1, n, GBAMD_T_INT32, NULL, NULL, NULL};
    v.p = (int64_t *)calloc(2, sizeof(int64_t));
    v.j = (int64_t *)xmalloc((size_t)n * sizeof(int64_t));
    v.x = NULL;
    int d = 0;
    int64_t e = 0;
    for (;;) {
        d++;
        /* v<q.V> = d : merge q's true entries into the sorted visited list */
        int64_t nv = v.p[1], nq = q.p[1], a = 0, b = 0, o = 0;
        int64_t *nj = (int64_t *)xmalloc((size_t)(nv + nq + 1) * sizeof(int64_t));
        while (a < nv || b < nq) {
            int64_t ja = a < nv ? v.j[a] : INT64_MAX;
            int64_t jb = INT64_MAX;
            while (b < nq && !((uint8_t *)q.x)[b]) b++;
            if (b < nq) jb = q.j[b];
            if (ja == INT64_MAX && jb == INT64_MAX) break;
            if (jb < ja) { nj[o++] = jb; levels[jb] = d; e += A->p[jb + 1] - A->p[jb]; b++; }
            else if (ja < jb) { nj[o++] = ja; a++; }
            else { nj[o++] = ja; a++; b++; }
        }
        free(v.j); v.j = nj; v.p[1] = o;
        /* q(~v.S, replace) << q.vxm(A, lor_land) */
        or_csr q0 = q;
        or_mxm(&q, &v, 1, 1, 1, -1, 0, 0, GBAMD_MON_LOR, GBAMD_OP_LAND, GBAMD_T_BOOL, GBAMD_T_BOOL,
               &q0, 0, A, 0);
        or_csr_free(&q0);
        int any = 0;
        for (int64_t t = 0; t < q.p[1]; t++) if (((uint8_t *)q.x)[t]) { any = 1; break; }
        if (!any) break;
    }
    or_csr_free(&q); or_csr_free(&v);
    if (edges) *edges = e;
    return d;
}

/* ================================================================== CPU baselines
 * (bench.py cpu_baseline legs of SURVEY §8(d) configs 2 and 4; not a parity oracle:
 * tests/test_cpu_baseline.py checks them against or_mxm and scipy) */

/* y = x plus.times A (GrB_vxm with a dense FP64 x), pulled over AT = A^T (rows of AT are
 * the output positions); each output folds its column in ascending row order, nthreads
 * host threads.  present[j] = 1 iff column j of A holds an entry. */
void or_spmv_plus_times_fp64_par(const or_csr *AT, const double *x, double *y, uint8_t *present, int nthreads) {
    const int64_t n = AT->nrows;
    const double *ax = (const double *)AT->x;
    if (nthreads < 1) nthreads = 1;
#pragma omp parallel for num_threads(nthreads) schedule(dynamic, 1024)
    for (int64_t j = 0; j < n; j++) {
        double s = 0.0;
        const int64_t p0 = AT->p[j], p1 = AT->p[j + 1];
        for (int64_t p = p0; p < p1; p++) s += ax[p] * x[AT->j[p]];
        y[j] = s;
        present[j] = p1 > p0;
    }
}

/* first position in j[lo, hi) with j[pos] >= key (galloping from lo, then binary search) */
static int64_t gallop(const int64_t *j, int64_t lo, int64_t hi, int64_t key) {
    int64_t step = 1, a = lo, b = lo;
    while (b < hi && j[b] < key) {
        a = b + 1;
        b = lo + step;
        step <<= 1;
    }
    if (b > hi) b = hi;
    while (a < b) {
        const int64_t m = (a + b) >> 1;
        if (j[m] < key) a = m + 1;
        else b = m;
    }
    return a;
}

/* C<A.S> = A min.+ A (INT64) over the mask rows [row0, row1): for each mask entry (i, j) the
 * intersection of A(i,:) with A(:,j) = AT(j,:) by a sorted merge, galloping through the longer
 * list when the lengths differ by 8x or more -- the dot form a CPU GraphBLAS library runs for
 * a masked mxm whose mask is sparse (SuiteSparse dot3).  Integer wrap as GB_ADD.  cvals /
 * present are indexed by the mask entry's position minus A->p[row0].  Returns the number of
 * entries of C in those rows; *work = sum over the mask entries of deg_out(i) + deg_in(j)
 * (the GTEPS numerator of SURVEY §8(d) config 4). */
int64_t or_masked_dot_min_plus_int64_par(const or_csr *A, const or_csr *AT, int64_t row0, int64_t row1,
                                         int64_t *cvals, uint8_t *present, int64_t *work, int nthreads) {
    const int64_t *ax = (const int64_t *)A->x, *tx = (const int64_t *)AT->x;
    const int64_t base = A->p[row0];
    int64_t nc = 0, wk = 0;
    if (nthreads < 1) nthreads = 1;
#pragma omp parallel for num_threads(nthreads) schedule(dynamic, 64) reduction(+ : nc, wk)
    for (int64_t i = row0; i < row1; i++) {
        const int64_t a0 = A->p[i], a1 = A->p[i + 1];
        for (int64_t e = a0; e < a1; e++) {
            const int64_t jcol = A->j[e];
            int64_t p = a0, q = AT->p[jcol];
            const int64_t pe = a1, qe = AT->p[jcol + 1];
            wk += (pe - p) + (qe - q);
            int have = 0;
            int64_t best = INT64_MAX;
            const int64_t la = pe - p, lb = qe - q;
            while (p < pe && q < qe) {
                const int64_t ka = A->j[p], kb = AT->j[q];
                if (ka == kb) {
                    const int64_t z = (int64_t)((uint64_t)ax[p] + (uint64_t)tx[q]);
                    if (!have || z < best) best = z;
                    have = 1;
                    p++;
                    q++;
                } else if (ka < kb) {
                    p = la >= 8 * lb ? gallop(A->j, p + 1, pe, kb) : p + 1;
                } else {
                    q = lb >= 8 * la ? gallop(AT->j, q + 1, qe, ka) : q + 1;
                }
            }
            present[e - base] = (uint8_t)have;
            if (have) {
                cvals[e - base] = best;
                nc++;
            }
        }
    }
    if (work) *work = wk;
    return nc;
}

static int cmp_i64_asc(const void *a, const void *b) {
    const int64_t x = *(const int64_t *)a, y = *(const int64_t *)b;
    return (x > y) - (x < y);
}

/* C = A plus.times B (FP64, unmasked) over the rows [row0, row1) of A: Gustavson's row-wise
 * saxpy with a dense accumulator per thread (values + a row stamp + the list of touched
 * columns, sorted when the row is done) -- the method a CPU GraphBLAS library uses for an
 * unmasked A*B (SuiteSparse saxpy3's Gustavson variant), nthreads host threads, rows handed
 * out dynamically.  Each output value folds its products in ascending k (A's row order), like
 * or_mxm.  C (rows row1 - row0, B->ncols columns) is allocated here; *products = sum over the
 * rows' entries A(i,k) of |B(k,:)|.  Returns nnz(C). */
int64_t or_spgemm_plus_times_fp64_par(const or_csr *A, const or_csr *B, int64_t row0, int64_t row1, or_csr *C,
                                      int64_t *products, int nthreads) {
    const int64_t nr = row1 - row0, n = B->ncols;
    const double *ax = (const double *)A->x, *bx = (const double *)B->x;
    if (nthreads < 1) nthreads = 1;
    int64_t *rlen = (int64_t *)calloc((size_t)nr + 1, sizeof(int64_t));
    int64_t **rcol = (int64_t **)calloc((size_t)nr + 1, sizeof(int64_t *));
    double **rval = (double **)calloc((size_t)nr + 1, sizeof(double *));
    int64_t prods = 0;
#pragma omp parallel num_threads(nthreads) reduction(+ : prods)
    {
        double *acc = (double *)malloc((size_t)n * sizeof(double));
        int64_t *stamp = (int64_t *)malloc((size_t)n * sizeof(int64_t));
        int64_t *cols = (int64_t *)malloc((size_t)n * sizeof(int64_t));
        for (int64_t c = 0; c < n; c++) stamp[c] = -1;
#pragma omp for schedule(dynamic, 16)
        for (int64_t i = row0; i < row1; i++) {
            int64_t m = 0;
            for (int64_t e = A->p[i]; e < A->p[i + 1]; e++) {
                const int64_t k = A->j[e];
                const double a = ax[e];
                prods += B->p[k + 1] - B->p[k];
                for (int64_t q = B->p[k]; q < B->p[k + 1]; q++) {
                    const int64_t c = B->j[q];
                    if (stamp[c] != i) {
                        stamp[c] = i;
                        acc[c] = a * bx[q];
                        cols[m++] = c;
                    } else {
                        acc[c] += a * bx[q];
                    }
                }
            }
            qsort(cols, (size_t)m, sizeof(int64_t), cmp_i64_asc);
            int64_t *rc = (int64_t *)xmalloc((size_t)m * sizeof(int64_t));
            double *rv = (double *)xmalloc((size_t)m * sizeof(double));
            for (int64_t t = 0; t < m; t++) {
                rc[t] = cols[t];
                rv[t] = acc[cols[t]];
            }
            rlen[i - row0] = m;
            rcol[i - row0] = rc;
            rval[i - row0] = rv;
        }
        free(acc);
        free(stamp);
        free(cols);
    }
    C->nrows = nr;
    C->ncols = n;
    C->type = GBAMD_T_FP64;
    C->p = (int64_t *)xmalloc(((size_t)nr + 1) * sizeof(int64_t));
    C->p[0] = 0;
    for (int64_t r = 0; r < nr; r++) C->p[r + 1] = C->p[r] + rlen[r];
    const int64_t nz = C->p[nr];
    C->j = (int64_t *)xmalloc((size_t)nz * sizeof(int64_t));
    C->x = xmalloc((size_t)nz * sizeof(double));
#pragma omp parallel for num_threads(nthreads) schedule(dynamic, 64)
    for (int64_t r = 0; r < nr; r++) {
        memcpy(C->j + C->p[r], rcol[r], (size_t)rlen[r] * sizeof(int64_t));
        memcpy((double *)C->x + C->p[r], rval[r], (size_t)rlen[r] * sizeof(double));
        free(rcol[r]);
        free(rval[r]);
    }
    free(rlen);
    free(rcol);
    free(rval);
    if (products) *products = prods;
    return nz;
}
