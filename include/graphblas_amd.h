/*
 * graphblas_amd.h -- C ABI of libgraphblas_amd.so, the MI355X-native GraphBLAS
 * semiring backend.
 *
 * This is the drop-in boundary.  python-graphblas reaches its C library only
 * through `graphblas.core.base.call(cfunc_name, args)` (reference
 * graphblas/core/base.py:23-54), which looks the *name* up on the injected
 * `lib` object (core/utils.py:9-21, graphblas/__init__.py:193-197) and passes
 * opaque handles (`x._carg`, e.g. core/matrix.py:1902-1903) plus plain C
 * scalars / numpy buffers.  Every entry point below is declared with the
 * GraphBLAS C API 2.0 name and signature that `call` would bind, so the
 * library can stand where SuiteSparse:GraphBLAS 7.4.x stood (reference
 * pyproject.toml:65).  No torch types appear in any signature.
 *
 * Replacement map (reference call sites -> entry point):
 *   core/matrix.py:2241 (cfunc "GrB_mxm"), core/vector.py:1686 (outer)  -> GrB_mxm
 *   core/matrix.py:2196 (cfunc "GrB_mxv")                              -> GrB_mxv
 *   core/vector.py:1298 (vxm), core/vector.py:1643 (inner)             -> GrB_vxm
 *   core/descriptor.py:51-89 (GrB_DESC_* globals), :138-155             -> GrB_Descriptor_*
 *   core/operator/{semiring,monoid,binary}.py regex discovery            -> builtin globals
 *   core/exceptions.py:93-155 (GrB_Info codes, GrB_<T>_error)           -> GrB_Info, *_error
 *   core/matrix.py:178-213, 643-697, 543-611, 1057-1133, 1658-1702      -> Matrix lifecycle,
 *       build, extractTuples, import, export
 *   core/vector.py:152-184, 538, 482                                    -> Vector lifecycle
 *   core/matrix.py:391-398 (isequal: eWiseMult + reduce)               -> eWiseMult, reduce
 *   notebooks Example B.1 (BFS: Vector assign / reduce)                 -> assign, reduce
 *
 * Storage (device resident, HBM): matrices CSR (int64 row pointers, int32
 * column indices, typed values or one iso value) with a lazily built CSC
 * (transpose) cache; vectors a 64-bit-word presence bitmap plus a dense value
 * array (or one iso value).  All work is enqueued on one HIP stream
 * (GxB_Context_set_stream); results a host read needs (nvals, extract,
 * export, reduce-to-C-scalar) synchronise that stream, i.e. GrB_NONBLOCKING
 * semantics with GrB_wait as the explicit completion point.
 */
#ifndef GRAPHBLAS_AMD_H
#define GRAPHBLAS_AMD_H

#include <stdbool.h>
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
#define GB_EXTERN extern "C"
extern "C" {
#else
#define GB_EXTERN extern
#endif

#define GxB_IMPLEMENTATION_NAME "graphblas_amd (MI355X / gfx950)"
#define GRB_VERSION 2
#define GRB_SUBVERSION 0

typedef uint64_t GrB_Index;
/* index constants as SuiteSparse:GraphBLAS 7.4 defines them (python-graphblas reads them
 * from lib: GxB_RANGE/GxB_STRIDE/GxB_BACKWARDS in core/slice.py:10-49, and its vanilla
 * backend deletes GxB_BACKWARDS/GxB_STRIDE from lib, graphblas/__init__.py:185-186) */
#define GrB_INDEX_MAX ((GrB_Index)(1ULL << 60) - 1)
#define GxB_INDEX_MAX ((GrB_Index)(1ULL << 60))
/* special values of ni in assign/extract: I = [begin, end] (RANGE), [begin, end, inc]
 * (STRIDE), [begin, end, dec] (BACKWARDS), bounds inclusive */
#define GxB_RANGE (INT64_MAX)
#define GxB_STRIDE (INT64_MAX - 1)
#define GxB_BACKWARDS (INT64_MAX - 2)
#define GxB_BEGIN 0
#define GxB_END 1
#define GxB_INC 2
#define GxB_MAX_NAME_LEN 128

typedef enum {
    GrB_SUCCESS = 0,
    GrB_NO_VALUE = 1,
    GrB_UNINITIALIZED_OBJECT = -1,
    GrB_NULL_POINTER = -2,
    GrB_INVALID_VALUE = -3,
    GrB_INVALID_INDEX = -4,
    GrB_DOMAIN_MISMATCH = -5,
    GrB_DIMENSION_MISMATCH = -6,
    GrB_OUTPUT_NOT_EMPTY = -7,
    GrB_NOT_IMPLEMENTED = -8,
    GrB_PANIC = -101,
    GrB_OUT_OF_MEMORY = -102,
    GrB_INSUFFICIENT_SPACE = -103,
    GrB_INVALID_OBJECT = -104,
    GrB_INDEX_OUT_OF_BOUNDS = -105,
    GrB_EMPTY_OBJECT = -106
} GrB_Info;

typedef enum { GrB_NONBLOCKING = 0, GrB_BLOCKING = 1 } GrB_Mode;
typedef enum { GrB_COMPLETE = 0, GrB_MATERIALIZE = 1 } GrB_WaitMode;
typedef enum { GrB_OUTP = 0, GrB_MASK = 1, GrB_INP0 = 2, GrB_INP1 = 3 } GrB_Desc_Field;
typedef enum {
    GxB_DEFAULT = 0,
    GrB_REPLACE = 1,
    GrB_COMP = 2,
    GrB_STRUCTURE = 4,
    GrB_COMP_STRUCTURE = 6,
    GrB_TRAN = 3
} GrB_Desc_Value;
typedef enum { GrB_CSR_FORMAT = 0, GrB_CSC_FORMAT = 1, GrB_COO_FORMAT = 2 } GrB_Format;
/* global option fields (GxB_Global_Option_get_INT32; python-graphblas reads GxB_MODE when the
 * library was initialised before it, graphblas/__init__.py:156-166) */
typedef enum { GxB_MODE = 2 } GxB_Option_Field;

typedef struct GB_Type_opaque *GrB_Type;
typedef struct GB_BinaryOp_opaque *GrB_BinaryOp;
typedef struct GB_UnaryOp_opaque *GrB_UnaryOp;
typedef struct GB_Monoid_opaque *GrB_Monoid;
typedef struct GB_Semiring_opaque *GrB_Semiring;
typedef struct GB_Descriptor_opaque *GrB_Descriptor;
typedef struct GB_Matrix_opaque *GrB_Matrix;
typedef struct GB_Vector_opaque *GrB_Vector;
typedef struct GB_Scalar_opaque *GrB_Scalar;

/* GrB_ALL: the "all indices" sentinel for assign */
GB_EXTERN const GrB_Index *GrB_ALL;

#include "graphblas_amd_builtins.h"

/* ---------------------------------------------------------------- context */
GrB_Info GrB_init(GrB_Mode mode);
GrB_Info GrB_finalize(void);
GrB_Info GrB_getVersion(unsigned int *version, unsigned int *subversion);
/* Extension: run all library work on this HIP stream (hipStream_t as void*;
 * NULL = the library's own stream).  Lets torch.distributed / RCCL collectives
 * on the caller's stream order against GraphBLAS kernels without host syncs. */
GrB_Info GxB_Context_set_stream(void *hip_stream);
GrB_Info GxB_Context_get_stream(void **hip_stream);
/* Extension: which HIP device the library uses (call before GrB_init). */
GrB_Info GxB_Context_set_device(int device);
/* Extension: look up a builtin object by its exported name (kind: 0 type,
 * 1 binop, 2 monoid, 3 semiring, 4 descriptor).  For FFIs that cannot read
 * data symbols directly. */
GrB_Info GxB_builtin_lookup(void **handle, int *kind, const char *name);
/* Extension: object names for diagnostics / recorder strings. */
GrB_Info GxB_name(const char **name, const void *builtin_object);

/* ---------------------------------------------------------------- types/ops */
GrB_Info GrB_Type_free(GrB_Type *type);
GrB_Info GrB_BinaryOp_free(GrB_BinaryOp *op);
GrB_Info GrB_Monoid_free(GrB_Monoid *monoid);
GrB_Info GrB_Semiring_free(GrB_Semiring *semiring);
GrB_Info GrB_UnaryOp_free(GrB_UnaryOp *op);
/* semiring from a builtin monoid and a builtin binary operator whose output type is the
 * monoid's (python-graphblas registers e.g. plus_pow this way for agg.sum_of_squares,
 * reference core/operator/agg.py:271-276) */
GrB_Info GrB_Semiring_new(GrB_Semiring *semiring, GrB_Monoid add, GrB_BinaryOp multiply);
GrB_Info GxB_Semiring_add(GrB_Monoid *add, GrB_Semiring semiring);
GrB_Info GxB_Semiring_multiply(GrB_BinaryOp *multiply, GrB_Semiring semiring);

/* ---------------------------------------------------------------- descriptor */
GrB_Info GrB_Descriptor_new(GrB_Descriptor *desc);
GrB_Info GrB_Descriptor_set(GrB_Descriptor desc, GrB_Desc_Field field, GrB_Desc_Value val);
GrB_Info GrB_Descriptor_free(GrB_Descriptor *desc);

/* ---------------------------------------------------------------- Matrix */
GrB_Info GrB_Matrix_new(GrB_Matrix *A, GrB_Type type, GrB_Index nrows, GrB_Index ncols);
GrB_Info GrB_Matrix_dup(GrB_Matrix *C, const GrB_Matrix A);
GrB_Info GrB_Matrix_clear(GrB_Matrix A);
GrB_Info GrB_Matrix_nrows(GrB_Index *nrows, const GrB_Matrix A);
GrB_Info GrB_Matrix_ncols(GrB_Index *ncols, const GrB_Matrix A);
GrB_Info GrB_Matrix_nvals(GrB_Index *nvals, const GrB_Matrix A);
GrB_Info GrB_Matrix_resize(GrB_Matrix C, GrB_Index nrows, GrB_Index ncols);
GrB_Info GrB_Matrix_free(GrB_Matrix *A);
GrB_Info GrB_Matrix_wait(GrB_Matrix A, GrB_WaitMode mode);
GrB_Info GrB_Matrix_error(const char **error, const GrB_Matrix A);
GrB_Info GxB_Matrix_type(GrB_Type *type, const GrB_Matrix A);
GrB_Info GrB_Matrix_removeElement(GrB_Matrix C, GrB_Index row, GrB_Index col);
GrB_Info GrB_Matrix_exportSize(GrB_Index *Ap_len, GrB_Index *Ai_len, GrB_Index *Ax_len,
                               GrB_Format format, GrB_Matrix A);
GrB_Info GrB_Matrix_exportHint(GrB_Format *format, GrB_Matrix A);

#define GB_DECLARE_TYPED_MATRIX(T, ctype)                                                          \
    GrB_Info GrB_Matrix_build_##T(GrB_Matrix C, const GrB_Index *I, const GrB_Index *J,          \
                                  const ctype *X, GrB_Index nvals, const GrB_BinaryOp dup);     \
    GrB_Info GrB_Matrix_setElement_##T(GrB_Matrix C, ctype x, GrB_Index i, GrB_Index j);         \
    GrB_Info GrB_Matrix_extractElement_##T(ctype *x, const GrB_Matrix A, GrB_Index i,           \
                                           GrB_Index j);                                        \
    GrB_Info GrB_Matrix_extractTuples_##T(GrB_Index *I, GrB_Index *J, ctype *X,                 \
                                          GrB_Index *nvals, const GrB_Matrix A);                \
    GrB_Info GrB_Matrix_import_##T(GrB_Matrix *A, GrB_Type type, GrB_Index nrows,               \
                                   GrB_Index ncols, const GrB_Index *Ap, const GrB_Index *Ai,   \
                                   const ctype *Ax, GrB_Index Ap_len, GrB_Index Ai_len,         \
                                   GrB_Index Ax_len, GrB_Format format);                        \
    GrB_Info GrB_Matrix_export_##T(GrB_Index *Ap, GrB_Index *Ai, ctype *Ax, GrB_Index *Ap_len,  \
                                   GrB_Index *Ai_len, GrB_Index *Ax_len, GrB_Format format,     \
                                   GrB_Matrix A);                                               \
    GrB_Info GrB_Matrix_assign_##T(GrB_Matrix C, const GrB_Matrix Mask, const GrB_BinaryOp accum, \
                                   ctype x, const GrB_Index *I, GrB_Index ni,                   \
                                   const GrB_Index *J, GrB_Index nj, const GrB_Descriptor desc); \
    GrB_Info GrB_Matrix_reduce_##T(ctype *c, const GrB_BinaryOp accum, const GrB_Monoid monoid, \
                                   const GrB_Matrix A, const GrB_Descriptor desc);              \
    GrB_Info GxB_Matrix_build_Scalar_##T(GrB_Matrix C, const GrB_Index *I, const GrB_Index *J,  \
                                         ctype x, GrB_Index nvals);                              \
    GrB_Info GrB_Matrix_apply_BinaryOp1st_##T(GrB_Matrix C, const GrB_Matrix Mask,              \
                                              const GrB_BinaryOp accum, const GrB_BinaryOp op,  \
                                              ctype x, const GrB_Matrix A,                      \
                                              const GrB_Descriptor desc);                       \
    GrB_Info GrB_Matrix_apply_BinaryOp2nd_##T(GrB_Matrix C, const GrB_Matrix Mask,              \
                                              const GrB_BinaryOp accum, const GrB_BinaryOp op,  \
                                              const GrB_Matrix A, ctype y,                      \
                                              const GrB_Descriptor desc);

#define GB_DECLARE_TYPED_VECTOR(T, ctype)                                                          \
    GrB_Info GrB_Vector_build_##T(GrB_Vector w, const GrB_Index *I, const ctype *X,             \
                                  GrB_Index nvals, const GrB_BinaryOp dup);                     \
    GrB_Info GrB_Vector_setElement_##T(GrB_Vector w, ctype x, GrB_Index i);                     \
    GrB_Info GrB_Vector_extractElement_##T(ctype *x, const GrB_Vector v, GrB_Index i);          \
    GrB_Info GrB_Vector_extractTuples_##T(GrB_Index *I, ctype *X, GrB_Index *nvals,             \
                                          const GrB_Vector v);                                  \
    GrB_Info GrB_Vector_assign_##T(GrB_Vector w, const GrB_Vector mask,                         \
                                   const GrB_BinaryOp accum, ctype x, const GrB_Index *I,       \
                                   GrB_Index ni, const GrB_Descriptor desc);                    \
    GrB_Info GrB_Vector_reduce_##T(ctype *c, const GrB_BinaryOp accum, const GrB_Monoid monoid, \
                                   const GrB_Vector u, const GrB_Descriptor desc);              \
    GrB_Info GrB_Scalar_setElement_##T(GrB_Scalar s, ctype x);                                   \
    GrB_Info GrB_Scalar_extractElement_##T(ctype *x, const GrB_Scalar s);                        \
    GrB_Info GxB_Vector_build_Scalar_##T(GrB_Vector w, const GrB_Index *I, ctype x,             \
                                         GrB_Index nvals);                                      \
    GrB_Info GrB_Vector_apply_BinaryOp1st_##T(GrB_Vector w, const GrB_Vector mask,              \
                                              const GrB_BinaryOp accum, const GrB_BinaryOp op,  \
                                              ctype x, const GrB_Vector u,                      \
                                              const GrB_Descriptor desc);                       \
    GrB_Info GrB_Vector_apply_BinaryOp2nd_##T(GrB_Vector w, const GrB_Vector mask,              \
                                              const GrB_BinaryOp accum, const GrB_BinaryOp op,  \
                                              const GrB_Vector u, ctype y,                      \
                                              const GrB_Descriptor desc);

#define GB_FOR_EACH_TYPE(X)                                                                        \
    X(BOOL, bool)                                                                                  \
    X(INT8, int8_t)                                                                                \
    X(UINT8, uint8_t)                                                                              \
    X(INT16, int16_t)                                                                              \
    X(UINT16, uint16_t)                                                                            \
    X(INT32, int32_t)                                                                              \
    X(UINT32, uint32_t)                                                                            \
    X(INT64, int64_t)                                                                              \
    X(UINT64, uint64_t)                                                                            \
    X(FP32, float)                                                                                 \
    X(FP64, double)

GB_FOR_EACH_TYPE(GB_DECLARE_TYPED_MATRIX)
GB_FOR_EACH_TYPE(GB_DECLARE_TYPED_VECTOR)

/* ---------------------------------------------------------------- Vector */
GrB_Info GrB_Vector_new(GrB_Vector *v, GrB_Type type, GrB_Index n);
GrB_Info GrB_Vector_dup(GrB_Vector *w, const GrB_Vector u);
GrB_Info GrB_Vector_clear(GrB_Vector v);
GrB_Info GrB_Vector_size(GrB_Index *n, const GrB_Vector v);
GrB_Info GrB_Vector_nvals(GrB_Index *nvals, const GrB_Vector v);
GrB_Info GrB_Vector_resize(GrB_Vector w, GrB_Index n);
GrB_Info GrB_Vector_free(GrB_Vector *v);
GrB_Info GrB_Vector_wait(GrB_Vector v, GrB_WaitMode mode);
GrB_Info GrB_Vector_error(const char **error, const GrB_Vector v);
GrB_Info GxB_Vector_type(GrB_Type *type, const GrB_Vector v);
GrB_Info GrB_Vector_removeElement(GrB_Vector v, GrB_Index i);

/* ---------------------------------------------------------------- Scalar */
GrB_Info GrB_Scalar_new(GrB_Scalar *s, GrB_Type type);
GrB_Info GrB_Scalar_dup(GrB_Scalar *s, const GrB_Scalar t);
GrB_Info GrB_Scalar_clear(GrB_Scalar s);
GrB_Info GrB_Scalar_nvals(GrB_Index *nvals, const GrB_Scalar s);
GrB_Info GrB_Scalar_free(GrB_Scalar *s);
GrB_Info GrB_Scalar_wait(GrB_Scalar s, GrB_WaitMode mode);
GrB_Info GrB_Scalar_error(const char **error, const GrB_Scalar s);

/* GrB_Scalar-argument variants (C API 2.0; python-graphblas calls them for non-C scalars):
 * extractElement: reference core/vector.py:1769, core/matrix.py:2837 -- a missing entry leaves
 *   s empty and returns GrB_SUCCESS;
 * setElement: core/vector.py:1808, core/matrix.py:2902 -- an empty x deletes the entry;
 * assign: core/vector.py:1918,1939, core/matrix.py:3279,3305 -- an empty x assigns "no value"
 *   (the selected part of the region is deleted; left alone under accum);
 * apply_BinaryOp1st/2nd: core/vector.py:1406,1449, core/matrix.py:2392,2435 -- an empty x is
 *   GrB_EMPTY_OBJECT. */
GrB_Info GrB_Vector_extractElement_Scalar(GrB_Scalar s, const GrB_Vector v, GrB_Index i);
GrB_Info GrB_Matrix_extractElement_Scalar(GrB_Scalar s, const GrB_Matrix A, GrB_Index i, GrB_Index j);
GrB_Info GrB_Vector_setElement_Scalar(GrB_Vector w, const GrB_Scalar x, GrB_Index i);
GrB_Info GrB_Matrix_setElement_Scalar(GrB_Matrix C, const GrB_Scalar x, GrB_Index i, GrB_Index j);
GrB_Info GrB_Vector_assign_Scalar(GrB_Vector w, const GrB_Vector mask, const GrB_BinaryOp accum,
                                  const GrB_Scalar x, const GrB_Index *I, GrB_Index ni,
                                  const GrB_Descriptor desc);
GrB_Info GrB_Matrix_assign_Scalar(GrB_Matrix C, const GrB_Matrix Mask, const GrB_BinaryOp accum,
                                  const GrB_Scalar x, const GrB_Index *I, GrB_Index ni,
                                  const GrB_Index *J, GrB_Index nj, const GrB_Descriptor desc);
GrB_Info GrB_Vector_apply_BinaryOp1st_Scalar(GrB_Vector w, const GrB_Vector mask,
                                             const GrB_BinaryOp accum, const GrB_BinaryOp op,
                                             const GrB_Scalar x, const GrB_Vector u,
                                             const GrB_Descriptor desc);
GrB_Info GrB_Vector_apply_BinaryOp2nd_Scalar(GrB_Vector w, const GrB_Vector mask,
                                             const GrB_BinaryOp accum, const GrB_BinaryOp op,
                                             const GrB_Vector u, const GrB_Scalar y,
                                             const GrB_Descriptor desc);
GrB_Info GrB_Matrix_apply_BinaryOp1st_Scalar(GrB_Matrix C, const GrB_Matrix Mask,
                                             const GrB_BinaryOp accum, const GrB_BinaryOp op,
                                             const GrB_Scalar x, const GrB_Matrix A,
                                             const GrB_Descriptor desc);
GrB_Info GrB_Matrix_apply_BinaryOp2nd_Scalar(GrB_Matrix C, const GrB_Matrix Mask,
                                             const GrB_BinaryOp accum, const GrB_BinaryOp op,
                                             const GrB_Matrix A, const GrB_Scalar y,
                                             const GrB_Descriptor desc);

/* ---------------------------------------------------------------- the hot path */
/* C<Mask> = C accum (A' (+).(x) B')      replaces SuiteSparse GrB_mxm */
GrB_Info GrB_mxm(GrB_Matrix C, const GrB_Matrix Mask, const GrB_BinaryOp accum,
                 const GrB_Semiring op, const GrB_Matrix A, const GrB_Matrix B,
                 const GrB_Descriptor desc);
/* w<mask> = w accum (A' (+).(x) u)       replaces SuiteSparse GrB_mxv */
GrB_Info GrB_mxv(GrB_Vector w, const GrB_Vector mask, const GrB_BinaryOp accum,
                 const GrB_Semiring op, const GrB_Matrix A, const GrB_Vector u,
                 const GrB_Descriptor desc);
/* w<mask> = w accum (u' (+).(x) A')      replaces SuiteSparse GrB_vxm */
GrB_Info GrB_vxm(GrB_Vector w, const GrB_Vector mask, const GrB_BinaryOp accum,
                 const GrB_Semiring op, const GrB_Vector u, const GrB_Matrix A,
                 const GrB_Descriptor desc);

/* ---------------------------------------------------------------- loop companions */
GrB_Info GrB_Matrix_eWiseMult_BinaryOp(GrB_Matrix C, const GrB_Matrix Mask,
                                       const GrB_BinaryOp accum, const GrB_BinaryOp op,
                                       const GrB_Matrix A, const GrB_Matrix B,
                                       const GrB_Descriptor desc);
GrB_Info GrB_Vector_eWiseMult_BinaryOp(GrB_Vector w, const GrB_Vector mask,
                                       const GrB_BinaryOp accum, const GrB_BinaryOp op,
                                       const GrB_Vector u, const GrB_Vector v,
                                       const GrB_Descriptor desc);
GrB_Info GrB_Matrix_eWiseAdd_BinaryOp(GrB_Matrix C, const GrB_Matrix Mask,
                                      const GrB_BinaryOp accum, const GrB_BinaryOp op,
                                      const GrB_Matrix A, const GrB_Matrix B,
                                      const GrB_Descriptor desc);
GrB_Info GrB_Vector_eWiseAdd_BinaryOp(GrB_Vector w, const GrB_Vector mask,
                                      const GrB_BinaryOp accum, const GrB_BinaryOp op,
                                      const GrB_Vector u, const GrB_Vector v,
                                      const GrB_Descriptor desc);
GrB_Info GrB_Vector_assign(GrB_Vector w, const GrB_Vector mask, const GrB_BinaryOp accum,
                           const GrB_Vector u, const GrB_Index *I, GrB_Index ni,
                           const GrB_Descriptor desc);
GrB_Info GrB_Matrix_assign(GrB_Matrix C, const GrB_Matrix Mask, const GrB_BinaryOp accum,
                           const GrB_Matrix A, const GrB_Index *I, GrB_Index ni,
                           const GrB_Index *J, GrB_Index nj, const GrB_Descriptor desc);
GrB_Info GrB_Matrix_reduce_Monoid_Scalar(GrB_Scalar s, const GrB_BinaryOp accum,
                                         const GrB_Monoid monoid, const GrB_Matrix A,
                                         const GrB_Descriptor desc);
GrB_Info GrB_Vector_reduce_Monoid_Scalar(GrB_Scalar s, const GrB_BinaryOp accum,
                                         const GrB_Monoid monoid, const GrB_Vector u,
                                         const GrB_Descriptor desc);
/* w<mask> = accum(w, reduce each row of A' with the monoid): lowered to a semiring SpMV
 * (monoid, FIRST) against an iso-full vector, the reference's own lowering of reductions
 * (core/operator/agg.py:207-279); A' = A^T (desc INP0 = TRAN) reduces columns
 * (core/matrix.py:2583,2620). */
GrB_Info GrB_Matrix_reduce_Monoid(GrB_Vector w, const GrB_Vector mask, const GrB_BinaryOp accum,
                                  const GrB_Monoid monoid, const GrB_Matrix A,
                                  const GrB_Descriptor desc);
GrB_Info GrB_Matrix_reduce_BinaryOp(GrB_Vector w, const GrB_Vector mask, const GrB_BinaryOp accum,
                                    const GrB_BinaryOp op, const GrB_Matrix A,
                                    const GrB_Descriptor desc);
/* apply (reference core/vector.py:1370,1404,1447; core/matrix.py:2356,2390,2433): values map,
 * structure kept; iso inputs stay iso (one value computed). */
GrB_Info GrB_Vector_apply(GrB_Vector w, const GrB_Vector mask, const GrB_BinaryOp accum,
                          const GrB_UnaryOp op, const GrB_Vector u, const GrB_Descriptor desc);
GrB_Info GrB_Matrix_apply(GrB_Matrix C, const GrB_Matrix Mask, const GrB_BinaryOp accum,
                          const GrB_UnaryOp op, const GrB_Matrix A, const GrB_Descriptor desc);
GrB_Info GrB_transpose(GrB_Matrix C, const GrB_Matrix Mask, const GrB_BinaryOp accum,
                       const GrB_Matrix A, const GrB_Descriptor desc);

/* extract (reference core/matrix.py:2868 "GrB_Matrix_extract", :2903/2917 "GrB_Col_extract",
 * core/vector.py:1026 "GrB_Vector_extract"): C<M> = accum(C, A'(I, J)); w<m> = accum(w, A'(I, j));
 * w<m> = accum(w, u(I)).  I, J: GrB_ALL, an explicit list, or the GxB_RANGE / GxB_STRIDE /
 * GxB_BACKWARDS encodings above. */
GrB_Info GrB_Matrix_extract(GrB_Matrix C, const GrB_Matrix Mask, const GrB_BinaryOp accum,
                            const GrB_Matrix A, const GrB_Index *I, GrB_Index ni,
                            const GrB_Index *J, GrB_Index nj, const GrB_Descriptor desc);
GrB_Info GrB_Col_extract(GrB_Vector w, const GrB_Vector mask, const GrB_BinaryOp accum,
                         const GrB_Matrix A, const GrB_Index *I, GrB_Index ni, GrB_Index j,
                         const GrB_Descriptor desc);
GrB_Info GrB_Vector_extract(GrB_Vector w, const GrB_Vector mask, const GrB_BinaryOp accum,
                            const GrB_Vector u, const GrB_Index *I, GrB_Index ni,
                            const GrB_Descriptor desc);
/* GrB_MODE of the running library (GrB_BLOCKING / GrB_NONBLOCKING) for field GxB_MODE */
GrB_Info GxB_Global_Option_get_INT32(GxB_Option_Field field, int32_t *value);

/* ---------------------------------------------------------------- device extensions */
/* Zero-copy views of device storage, for RCCL / torch.distributed exchange of
 * row-shard panels and frontier bitmaps (1-D row sharding). */
typedef struct {
    int format;          /* 0 = CSR matrix, 1 = bitmap vector */
    int type_code;       /* gbamd_type_code */
    int iso;             /* all values equal to the single stored value */
    int64_t nrows, ncols, nvals;
    void *rowptr;        /* int64[nrows+1] (CSR) */
    void *colidx;        /* int32[nvals]   (CSR) */
    void *values;        /* typed values (CSR: nvals or 1; bitmap: n or 1) */
    void *bitmap;        /* uint64[ceil(n/64)] (bitmap) */
} GxB_DeviceView;
GrB_Info GxB_Matrix_device_view(GxB_DeviceView *view, const GrB_Matrix A);
GrB_Info GxB_Vector_device_view(GxB_DeviceView *view, const GrB_Vector v);
/* Build a CSR matrix from device buffers (copied on the library stream):
 * rowptr int64[nrows+1] (rowptr[0] = 0), colidx int32[nvals] sorted and unique per
 * row, values typed [nvals] or [1] when iso.  Receives all-gathered row panels
 * (1-D row-sharded GrB_mxm); the device-side counterpart of
 * GxB_Matrix_import_CSR (reference core/ss/matrix.py:1282-1352). */
GrB_Info GxB_Matrix_import_device(GrB_Matrix *A, GrB_Type type, GrB_Index nrows, GrB_Index ncols,
                                  const void *rowptr, const void *colidx, const void *values,
                                  GrB_Index nvals, bool iso);
/* Mark that the vector's bitmap/values were rewritten through a device view
 * (nvals recomputed on device, on the library stream). */
GrB_Info GxB_Vector_device_touch(GrB_Vector v);
/* The ticket of the vector's last device publish of its count (0: none; device_touch,
 * bitmap_import and the SpMV kernels publish), and a wait on it: *nvals = the count the
 * vector had at that publish, read from the pinned host mailbox without synchronising the
 * stream -- valid although later work that does not write the vector was enqueued since
 * (GrB_Vector_nvals trusts a mailbox only while nothing was).  GrB_INVALID_VALUE if a later
 * publish of the same vector superseded it; if the stream drained without the publish (a
 * failed or skipped launch) the count is read synchronously when the vector is unchanged since,
 * GrB_PANIC otherwise.  The pipelined sharded level loop
 * (graphblas_amd/dist.py: pipelined_levels) enqueues level d + 1 before it waits for level
 * d's frontier count.  Replaces the nvals read of reference notebooks/Example B.1 cell 8
 * (`q.nvals`, core/vector.py: Vector.nvals -> GrB_Vector_nvals). */
GrB_Info GxB_Vector_publish_ticket(uint64_t *ticket, GrB_Vector v);
GrB_Info GxB_Vector_wait_ticket(GrB_Index *nvals, GrB_Vector v, uint64_t ticket);
/* Copy the first nwords 64-bit words of a vector's presence bitmap to /
 * from device memory on the library stream (frontier exchange over RCCL).
 * Import makes the vector iso-valued 1 (true) on every set bit. */
GrB_Info GxB_Vector_bitmap_export(GrB_Vector v, void *dst_device, GrB_Index nwords);
/* Column-word format of a matrix of at most 64 rows (batched frontiers,
 * gb_colbits.hip): converts A to it if needed and returns the device address of
 * its ncols 64-bit words (bit r of word j = entry (r, j)).  The words may be
 * rewritten in place on the library stream (a frontier all-gather over RCCL),
 * followed by GxB_Matrix_colwords_touch. */
GrB_Info GxB_Matrix_colwords_view(uint64_t **words, GrB_Index *nwords, GrB_Matrix A);
/* Recount a column-word matrix (count + summary, published to the host mailbox)
 * after its words were rewritten; a non-iso matrix becomes iso-valued 1 (true),
 * like GxB_Vector_bitmap_import. */
GrB_Info GxB_Matrix_colwords_touch(GrB_Matrix A);
GrB_Info GxB_Vector_bitmap_import(GrB_Vector v, const void *src_device, GrB_Index nwords);
/* Device-initiated frontier exchange of the 1-D row-sharded level BFS (gb_peer.hip, DESIGN.md
 * §6): replaces the host-issued all-gather of the frontier slices (GxB_Vector_bitmap_export +
 * RCCL all-gather + GxB_Vector_device_touch) that follows each shard's GrB_mxv in the
 * sharded form of reference notebooks/Example B.1 cell 8 (core/matrix.py:2163-2204).
 * Each rank owns a window (frontier bitmap x 2, per-rank counts and arrival flags) mapped into
 * every peer: _handle exports it (GxB_PEER_HANDLE_BYTES opaque bytes, hipIpcGetMemHandle), a
 * peer maps it with _open (hipIpcOpenMemHandle, over xGMI), and several shards driven from one
 * process link their windows with _attach.  bounds: nranks + 1 offsets in 64-row bitmap words
 * (NULL: equal slots).  _put(w, qloc) writes the rank's slice qloc (rows [64 bounds[rank],
 * 64 bounds[rank+1]) of the frontier) into every window and raises the rank's flag there;
 * _wait(q, w) waits on the device for every rank's flag, assembles the whole frontier in q
 * (iso true) and publishes its count to q's host mailbox (GxB_Vector_publish_ticket /
 * wait_ticket, GrB_Vector_nvals) -- no host round trip and no collective per level.  Calls
 * pair up in order (put, wait, put, wait ...) on every rank.  A peer that never arrives ends
 * the wait after ~5 s with an empty q; _error then reports 1 (it synchronises the stream). */
#define GxB_PEER_HANDLE_BYTES 64
typedef struct GB_PeerWindow_opaque *GxB_PeerWindow;
GrB_Info GxB_PeerWindow_new(GxB_PeerWindow *w, GrB_Index n, int nranks, int rank, const GrB_Index *bounds);
GrB_Info GxB_PeerWindow_handle(void *handle, GxB_PeerWindow w);
GrB_Info GxB_PeerWindow_open(GxB_PeerWindow w, int peer, const void *handle);
GrB_Info GxB_PeerWindow_attach(GxB_PeerWindow w, int peer, GxB_PeerWindow other);
GrB_Info GxB_PeerWindow_put(GxB_PeerWindow w, const GrB_Vector qloc);
GrB_Info GxB_PeerWindow_wait(GrB_Vector q, GxB_PeerWindow w);
GrB_Info GxB_PeerWindow_error(int64_t *code, GxB_PeerWindow w);
GrB_Info GxB_PeerWindow_free(GxB_PeerWindow *w);
/* Build a pattern R-MAT graph on the device (same generator as the oracle):
 * scale, edge factor, seed; values: 0 = BOOL iso true, 1 = INT64 [1,255],
 * 2 = FP64 [0,1); | 0x100 = generate A^T.  Rows [row_begin, row_end) only (row shard),
 * all columns; row_end = 0 means all rows. */
GrB_Info GxB_Matrix_rmat(GrB_Matrix *A, int scale, int edge_factor, uint64_t seed,
                         int values, uint64_t value_seed, GrB_Index row_begin,
                         GrB_Index row_end);
/* Force the cached CSC (transpose) of A to be built now (outside timed regions), with the
 * narrow value copies of both orientations when A's integer values fit 1-4 bytes (otherwise the
 * first masked GrB_mxm reading them builds them: a min/max pass, one blocking read, and up to
 * 4 B per entry and orientation kept until the transpose is dropped). */
GrB_Info GxB_Matrix_prepare_transpose(GrB_Matrix A);
/* Matrix Market coordinate reader (host, multithreaded; replaces the scipy /
 * fast_matrix_market parse behind reference graphblas/io/_matrixmarket.py:6-61).
 * Returns 0-based COO arrays allocated with malloc (free each with
 * GxB_MatrixMarket_free) for GrB_Matrix_build_*: pattern -> BOOL (X all 1),
 * integer -> INT64, real -> FP64 (*type_code: gbamd_type_code); symmetric and
 * skew-symmetric files come back expanded. */
GrB_Info GxB_MatrixMarket_read_coo(const char *path, GrB_Index *nrows, GrB_Index *ncols, GrB_Index *nvals,
                                   int *type_code, GrB_Index **I, GrB_Index **J, void **X);
GrB_Info GxB_MatrixMarket_free(void *p);
/* Backend selection knobs for benchmarking ablations: 0 = automatic.  get_int also reads
 * the read-only counters "stat_bfs_spec_adopted" / "stat_bfs_spec_rollbacks" (BFS level
 * speculation) and "stat_nvals_copy" (vector counts read by a device copy
 * instead of the producing kernel's host mailbox). */
GrB_Info GxB_Global_set_int(const char *key, int64_t value);
GrB_Info GxB_Global_get_int(const char *key, int64_t *value);

#ifdef __cplusplus
}
#endif
#endif
