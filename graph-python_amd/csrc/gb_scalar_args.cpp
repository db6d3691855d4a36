// gb_scalar_args.cpp -- the C API 2.0 entry points that take a GrB_Scalar where the typed
// variants take a C value.  python-graphblas calls them whenever a value is a GrB_Scalar
// (Scalar.from_value's default, is_cscalar=False):
//   GrB_{Vector,Matrix}_extractElement_Scalar  reference core/vector.py:1769, core/matrix.py:2837
//   GrB_{Vector,Matrix}_setElement_Scalar      reference core/vector.py:1808, core/matrix.py:2902
//   GrB_{Vector,Matrix}_assign_Scalar          reference core/vector.py:1918,1939,
//                                              core/matrix.py:3279,3305
//   GrB_{Vector,Matrix}_apply_BinaryOp{1st,2nd}_Scalar
//                                              reference core/vector.py:1406,1449,
//                                              core/matrix.py:2392,2435
// Each reads the scalar's value (its own type) on the host and forwards to the typed entry
// point of that type, which casts it as the typed call would.  An empty GrB_Scalar means
// "no value" (C API 2.0): setElement deletes the entry; extractElement of a missing entry
// clears the scalar and succeeds; assign acts as the assignment of an empty object (the
// selected part of the region is deleted, or left alone under accum); apply fails with
// GrB_EMPTY_OBJECT.  Host work only (a one-element read); the hot path never calls these.
#include <cstring>

#include "gb_internal.h"

namespace {

struct sval {
    int code = -1;
    bool present = false;
    alignas(8) unsigned char bytes[16] = {};
};

// s's value in its own type; the error (uninitialised handle, ...) is returned
GrB_Info read_scalar(sval &v, const GrB_Scalar s) {
    if (!s) return GrB_NULL_POINTER;
    GB_Obj *S = OBJ(s);
    if (S->magic != GB_MAGIC) return GrB_UNINITIALIZED_OBJECT;
    v.code = S->type->code;
    GrB_Info r = GrB_NO_VALUE;
    switch (v.code) {
#define GB_READ(T, ctype)                                                          \
    case GBAMD_T_##T: {                                                            \
        ctype x;                                                                   \
        r = GrB_Scalar_extractElement_##T(&x, s);                                  \
        if (r == GrB_SUCCESS) std::memcpy(v.bytes, &x, sizeof(ctype));             \
        break;                                                                     \
    }
        GB_FOR_EACH_TYPE(GB_READ)
#undef GB_READ
    default: return GrB_DOMAIN_MISMATCH;
    }
    if (r == GrB_NO_VALUE) return GrB_SUCCESS;
    v.present = r == GrB_SUCCESS;
    return r;
}

// an error raised here (not by a forwarded call) is attached to the output object
GrB_Info fail_on(const void *out, GrB_Info info, const char *msg) {
    return gb_api(OBJ(out), [&] { gb_throw(info, msg); });
}

// the mask flags of desc, without replace or transposes (nullptr when there are none)
struct mask_desc {
    GrB_Descriptor d = nullptr;
    explicit mask_desc(const gb_desc &src, bool replace) {
        const int m = (src.comp ? GrB_COMP : 0) | (src.structure ? GrB_STRUCTURE : 0);
        if (!m && !replace) return;
        if (GrB_Descriptor_new(&d) != GrB_SUCCESS) {
            d = nullptr;
            throw std::bad_alloc();
        }
        if (m) GrB_Descriptor_set(d, GrB_MASK, (GrB_Desc_Value)m);
        if (replace) GrB_Descriptor_set(d, GrB_OUTP, GrB_REPLACE);
    }
    ~mask_desc() {
        if (d) GrB_Descriptor_free(&d);
    }
};

// w<mask>(I) = (empty vector of the list's length) [accum]: GrB_Vector_assign deletes the
// selected part of the region when there is no accum and leaves it under accum
GrB_Info vector_assign_empty(GrB_Vector w, const GrB_Vector mask, const GrB_BinaryOp accum, const GrB_Index *I,
                             GrB_Index ni, const GrB_Descriptor desc) {
    GB_Obj *W = OBJ(w);
    if (!w) return GrB_NULL_POINTER;
    if (W->magic != GB_MAGIC) return GrB_UNINITIALIZED_OBJECT;
    int64_t len = 0;
    GrB_Info e = gb_api(W, [&] {
        gb_index_list L;
        gb_expand_indices(L, I, ni, W->nrows);
        len = L.n;
    });
    if (e != GrB_SUCCESS) return e;
    GrB_Vector u = nullptr;
    e = GrB_Vector_new(&u, W->type, (GrB_Index)len);
    if (e != GrB_SUCCESS) return e;
    e = GrB_Vector_assign(w, mask, accum, u, I, ni, desc);
    GrB_Vector_free(&u);
    return e;
}

// C<Mask>(I, J) = (empty) [accum].  No accum: R = the region I x J where the mask selects
// (a scalar assign of `true` into an empty bool matrix with the same mask flags), then
// C<!R.S, replace> = C deletes it.  Either way a replace descriptor then applies the mask to
// all of C (C<Mask, replace> = C).
GrB_Info matrix_assign_empty(GrB_Matrix C, const GrB_Matrix Mask, const GrB_BinaryOp accum, const GrB_Index *I,
                             GrB_Index ni, const GrB_Index *J, GrB_Index nj, const GrB_Descriptor desc) {
    if (!C) return GrB_NULL_POINTER;
    GB_Obj *Co = OBJ(C);
    if (Co->magic != GB_MAGIC) return GrB_UNINITIALIZED_OBJECT;
    if (Co->kind != GB_KIND_MATRIX) return vector_assign_empty((GrB_Vector)C, (GrB_Vector)Mask, accum, I, ni, desc);
    gb_desc d;
    GrB_Info e = gb_api(Co, [&] { d = gb_read_desc(desc); });
    if (e != GrB_SUCCESS) return e;
    const GrB_Index nr = (GrB_Index)Co->nrows, nc = (GrB_Index)Co->ncols;
    if (!accum) {
        GrB_Matrix R = nullptr;
        e = GrB_Matrix_new(&R, GrB_BOOL, nr, nc);
        if (e != GrB_SUCCESS) return e;
        try {
            mask_desc md(d, false);
            e = GrB_Matrix_assign_BOOL(R, Mask, nullptr, true, I, ni, J, nj, md.d);
            if (e == GrB_SUCCESS) e = GrB_Matrix_assign(C, R, nullptr, C, GrB_ALL, nr, GrB_ALL, nc, GrB_DESC_RSC);
        } catch (const std::bad_alloc &) {
            e = GrB_OUT_OF_MEMORY;
        }
        if (e != GrB_SUCCESS && e != GrB_NO_VALUE) {
            // the region's error (bad index, dimension) belongs to the output
            const char *msg = nullptr;
            GrB_Matrix_error(&msg, R);
            std::string m = msg ? msg : "assign of an empty scalar failed";
            GrB_Matrix_free(&R);
            return fail_on(C, e, m.c_str());
        }
        GrB_Matrix_free(&R);
    }
    if (d.replace && Mask) {
        try {
            mask_desc md(d, true);
            e = GrB_Matrix_assign(C, Mask, nullptr, C, GrB_ALL, nr, GrB_ALL, nc, md.d);
        } catch (const std::bad_alloc &) {
            e = GrB_OUT_OF_MEMORY;
        }
    }
    return e;
}

// first = 1: op(s, u(i)); first = 0: op(u(i), s)
template <class OUT, class IN>
GrB_Info apply_scalar(bool vec, bool first, OUT w, const OUT mask, const GrB_BinaryOp accum,
                             const GrB_BinaryOp op, const GrB_Scalar s, const IN u, const GrB_Descriptor desc) {
    sval v;
    GrB_Info e = read_scalar(v, s);
    if (e != GrB_SUCCESS) return e;
    if (!v.present) return fail_on(w, GrB_EMPTY_OBJECT, "apply: the bound GrB_Scalar holds no value");
    switch (v.code) {
#define GB_APPLY(T, ctype)                                                                                       \
    case GBAMD_T_##T: {                                                                                          \
        ctype c;                                                                                                 \
        std::memcpy(&c, v.bytes, sizeof(ctype));                                                                 \
        if (vec)                                                                                                 \
            return first ? GrB_Vector_apply_BinaryOp1st_##T((GrB_Vector)w, (GrB_Vector)mask, accum, op, c,      \
                                                            (GrB_Vector)u, desc)                                 \
                         : GrB_Vector_apply_BinaryOp2nd_##T((GrB_Vector)w, (GrB_Vector)mask, accum, op,         \
                                                            (GrB_Vector)u, c, desc);                             \
        return first ? GrB_Matrix_apply_BinaryOp1st_##T((GrB_Matrix)w, (GrB_Matrix)mask, accum, op, c,          \
                                                        (GrB_Matrix)u, desc)                                     \
                     : GrB_Matrix_apply_BinaryOp2nd_##T((GrB_Matrix)w, (GrB_Matrix)mask, accum, op, (GrB_Matrix)u, \
                                                        c, desc);                                                \
    }
        GB_FOR_EACH_TYPE(GB_APPLY)
#undef GB_APPLY
    }
    return GrB_DOMAIN_MISMATCH;
}
}  // namespace

extern "C" {

GrB_Info GrB_Vector_setElement_Scalar(GrB_Vector w, const GrB_Scalar x, GrB_Index i) {
    sval v;
    GrB_Info e = read_scalar(v, x);
    if (e != GrB_SUCCESS) return e;
    if (!v.present) return GrB_Vector_removeElement(w, i);
    switch (v.code) {
#define GB_SET(T, ctype)                                          \
    case GBAMD_T_##T: {                                           \
        ctype c;                                                  \
        std::memcpy(&c, v.bytes, sizeof(ctype));                  \
        return GrB_Vector_setElement_##T(w, c, i);                \
    }
        GB_FOR_EACH_TYPE(GB_SET)
#undef GB_SET
    }
    return GrB_DOMAIN_MISMATCH;
}

GrB_Info GrB_Matrix_setElement_Scalar(GrB_Matrix C, const GrB_Scalar x, GrB_Index i, GrB_Index j) {
    sval v;
    GrB_Info e = read_scalar(v, x);
    if (e != GrB_SUCCESS) return e;
    if (!v.present) return GrB_Matrix_removeElement(C, i, j);
    switch (v.code) {
#define GB_SET(T, ctype)                                          \
    case GBAMD_T_##T: {                                           \
        ctype c;                                                  \
        std::memcpy(&c, v.bytes, sizeof(ctype));                  \
        return GrB_Matrix_setElement_##T(C, c, i, j);             \
    }
        GB_FOR_EACH_TYPE(GB_SET)
#undef GB_SET
    }
    return GrB_DOMAIN_MISMATCH;
}

// s = A(i, j) cast to s's type; a missing entry leaves s empty and returns GrB_SUCCESS
GrB_Info GrB_Matrix_extractElement_Scalar(GrB_Scalar s, const GrB_Matrix A, GrB_Index i, GrB_Index j) {
    if (!s || !A) return GrB_NULL_POINTER;
    if (OBJ(s)->magic != GB_MAGIC || OBJ(A)->magic != GB_MAGIC) return GrB_UNINITIALIZED_OBJECT;
    switch (OBJ(A)->type->code) {
#define GB_GET(T, ctype)                                                  \
    case GBAMD_T_##T: {                                                   \
        ctype c;                                                          \
        GrB_Info r = GrB_Matrix_extractElement_##T(&c, A, i, j);          \
        if (r == GrB_NO_VALUE) return GrB_Scalar_clear(s);                \
        if (r != GrB_SUCCESS) return r;                                   \
        return GrB_Scalar_setElement_##T(s, c);                           \
    }
        GB_FOR_EACH_TYPE(GB_GET)
#undef GB_GET
    }
    return GrB_DOMAIN_MISMATCH;
}

GrB_Info GrB_Vector_extractElement_Scalar(GrB_Scalar s, const GrB_Vector v, GrB_Index i) {
    return GrB_Matrix_extractElement_Scalar(s, (GrB_Matrix)v, i, 0);
}

GrB_Info GrB_Vector_assign_Scalar(GrB_Vector w, const GrB_Vector mask, const GrB_BinaryOp accum,
                                  const GrB_Scalar x, const GrB_Index *I, GrB_Index ni, const GrB_Descriptor desc) {
    sval v;
    GrB_Info e = read_scalar(v, x);
    if (e != GrB_SUCCESS) return e;
    if (!v.present) return vector_assign_empty(w, mask, accum, I, ni, desc);
    switch (v.code) {
#define GB_ASG(T, ctype)                                          \
    case GBAMD_T_##T: {                                           \
        ctype c;                                                  \
        std::memcpy(&c, v.bytes, sizeof(ctype));                  \
        return GrB_Vector_assign_##T(w, mask, accum, c, I, ni, desc); \
    }
        GB_FOR_EACH_TYPE(GB_ASG)
#undef GB_ASG
    }
    return GrB_DOMAIN_MISMATCH;
}

GrB_Info GrB_Matrix_assign_Scalar(GrB_Matrix C, const GrB_Matrix Mask, const GrB_BinaryOp accum,
                                  const GrB_Scalar x, const GrB_Index *I, GrB_Index ni, const GrB_Index *J,
                                  GrB_Index nj, const GrB_Descriptor desc) {
    sval v;
    GrB_Info e = read_scalar(v, x);
    if (e != GrB_SUCCESS) return e;
    if (!v.present) return matrix_assign_empty(C, Mask, accum, I, ni, J, nj, desc);
    switch (v.code) {
#define GB_ASG(T, ctype)                                          \
    case GBAMD_T_##T: {                                           \
        ctype c;                                                  \
        std::memcpy(&c, v.bytes, sizeof(ctype));                  \
        return GrB_Matrix_assign_##T(C, Mask, accum, c, I, ni, J, nj, desc); \
    }
        GB_FOR_EACH_TYPE(GB_ASG)
#undef GB_ASG
    }
    return GrB_DOMAIN_MISMATCH;
}


GrB_Info GrB_Vector_apply_BinaryOp1st_Scalar(GrB_Vector w, const GrB_Vector mask, const GrB_BinaryOp accum,
                                             const GrB_BinaryOp op, const GrB_Scalar x, const GrB_Vector u,
                                             const GrB_Descriptor desc) {
    return apply_scalar(true, true, w, mask, accum, op, x, u, desc);
}
GrB_Info GrB_Vector_apply_BinaryOp2nd_Scalar(GrB_Vector w, const GrB_Vector mask, const GrB_BinaryOp accum,
                                             const GrB_BinaryOp op, const GrB_Vector u, const GrB_Scalar y,
                                             const GrB_Descriptor desc) {
    return apply_scalar(true, false, w, mask, accum, op, y, u, desc);
}
GrB_Info GrB_Matrix_apply_BinaryOp1st_Scalar(GrB_Matrix C, const GrB_Matrix Mask, const GrB_BinaryOp accum,
                                             const GrB_BinaryOp op, const GrB_Scalar x, const GrB_Matrix A,
                                             const GrB_Descriptor desc) {
    return apply_scalar(false, true, C, Mask, accum, op, x, A, desc);
}
GrB_Info GrB_Matrix_apply_BinaryOp2nd_Scalar(GrB_Matrix C, const GrB_Matrix Mask, const GrB_BinaryOp accum,
                                             const GrB_BinaryOp op, const GrB_Matrix A, const GrB_Scalar y,
                                             const GrB_Descriptor desc) {
    return apply_scalar(false, false, C, Mask, accum, op, y, A, desc);
}

}  // extern "C"
