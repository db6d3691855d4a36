"""Matrix collection and its delayed expressions (mirrors the hot-path parts of
reference core/matrix.py: new/free :178-213, build :643-697, from_coo
:885-960, to_coo :543-611, _from_csx :1057-1133, _to_csx :1658-1702,
isequal :357-398, mxv :2163-2204, mxm :2206-2251, power :2754-2806,
MatrixExpression :3371-3412, TransposedMatrix :3614-3778)."""
import ctypes

import numpy as np

from . import operator as _op
from ._lib import lib
from .base import (BaseExpression, BaseType, ComplementedStructuralMask, StructuralMask, ValueMask,
                   _autoname, _check_mask, _Pointer, call, descriptor_lookup)
from .dtypes import BOOL, FP64, INT64, UINT64, lookup_dtype, unify
from .exceptions import DimensionMismatch, NoValue, check_status_carg


class _CArray:
    __slots__ = "array", "name"

    def __init__(self, array, name="array"):
        self.array = np.ascontiguousarray(array)
        self.name = name

    @property
    def _carg(self):
        return ctypes.c_void_p(self.array.ctypes.data)


def _values_dtype(values, dtype):
    if dtype is not None:
        return lookup_dtype(dtype)
    a = np.asarray(values)
    if a.dtype == object:  # reference core/utils.py values_to_numpy_buffer
        raise ValueError("object dtype for values is not allowed")
    if a.dtype == np.bool_:
        return lookup_dtype(BOOL)
    if np.issubdtype(a.dtype, np.integer) or np.issubdtype(a.dtype, np.floating):
        return lookup_dtype(a.dtype)
    raise TypeError(f"Cannot infer a GraphBLAS dtype from {a.dtype}")


def _index_array(x, name):
    a = np.asarray(x)
    if a.size and not (np.issubdtype(a.dtype, np.integer) or a.dtype == np.bool_):
        raise ValueError(f"{name} must be integers, not {a.dtype.name}")
    if a.size and a.min() < 0:
        raise ValueError(f"{name} must be non-negative")
    return np.ascontiguousarray(a, np.uint64)


class Matrix(BaseType):
    ndim = 2

    def __init__(self, dtype=FP64, nrows=0, ncols=0, *, name=None):
        self.dtype = lookup_dtype(dtype)
        self.name = _autoname("M") if name is None else name
        self._h = ctypes.c_void_p()
        self._nrows = int(nrows)
        self._ncols = int(ncols)
        call("GrB_Matrix_new", [_Pointer(self), self.dtype, self._nrows, self._ncols])

    def __del__(self):
        h = getattr(self, "_h", None)
        if getattr(self, "_parent", None) is not None:
            return  # a cast view (Vector._as_matrix) does not own the handle
        if h is not None and h.value:
            try:
                lib.GrB_Matrix_free(ctypes.byref(h))
            except Exception:
                pass

    # ---------------------------------------------------------------- properties
    @property
    def nrows(self):
        return self._nrows

    @property
    def ncols(self):
        return self._ncols

    @property
    def shape(self):
        return (self._nrows, self._ncols)

    @property
    def nvals(self):
        n = ctypes.c_uint64()
        check_status_carg(lib.GrB_Matrix_nvals(ctypes.byref(n), self._h), "Matrix", self._h)
        return n.value

    _nvals = nvals

    @property
    def T(self):
        return TransposedMatrix(self)

    @property
    def ss(self):
        from .ss import MatrixSS

        return MatrixSS(self)

    @property
    def S(self):
        return StructuralMask(self)

    @property
    def V(self):
        return ValueMask(self)

    def __repr__(self):
        return f"<Matrix {self.name}: {self._nrows}x{self._ncols}, nvals={self.nvals}, {self.dtype}>"

    # ---------------------------------------------------------------- construction
    @classmethod
    def from_coo(cls, rows, columns, values=1.0, dtype=None, *, nrows=None, ncols=None, dup_op=None,
                 name=None):
        rows = _index_array(rows, "row indices")
        columns = _index_array(columns, "column indices")
        if nrows is None:
            nrows = int(rows.max()) + 1 if rows.size else 0
        if ncols is None:
            ncols = int(columns.max()) + 1 if columns.size else 0
        if np.ndim(values) == 0 and not isinstance(values, np.ndarray):
            dt = _values_dtype(values, dtype)
            C = cls(dt, nrows, ncols, name=name)
            n = rows.size
            if rows.size != columns.size:
                raise ValueError("`rows` and `columns` lengths must match")
            if n:
                x = np.asarray(values, dt.np_type).item()
                call(f"GxB_Matrix_build_Scalar_{dt.name}",
                     [C, _CArray(rows, "rows"), _CArray(columns, "cols"), x, n])
            return C
        vals = np.asarray(values)
        dt = _values_dtype(vals, dtype)
        C = cls(dt, nrows, ncols, name=name)
        C.build(rows, columns, vals, dup_op=dup_op)
        return C

    def build(self, rows, columns, values, *, dup_op=None, clear=False, nrows=None, ncols=None):
        rows = _index_array(rows, "row indices")
        columns = _index_array(columns, "column indices")
        values = np.ascontiguousarray(np.broadcast_to(np.asarray(values, self.dtype.np_type), rows.shape))
        n = values.shape[0]
        if rows.size != n or columns.size != n:
            raise ValueError("`rows` and `columns` and `values` lengths must match: "
                             f"{rows.size}, {columns.size}, {values.size}")
        if clear:
            self.clear()
        if nrows is not None or ncols is not None:
            self.resize(self._nrows if nrows is None else nrows, self._ncols if ncols is None else ncols)
        if n == 0:
            return
        dup = None if dup_op is None else _binary_for(dup_op, self.dtype)
        call(f"GrB_Matrix_build_{self.dtype.name}",
             [self, _CArray(rows, "rows"), _CArray(columns, "cols"), _CArray(values, "values"), n, dup])
        if dup_op is None and self.nvals < n:
            raise ValueError("Duplicate indices found, must provide `dup_op` BinaryOp")

    @classmethod
    def from_csr(cls, indptr, col_indices, values=1.0, dtype=None, *, ncols=None, name=None):
        indptr = np.ascontiguousarray(indptr, np.uint64)
        col_indices = np.ascontiguousarray(col_indices, np.uint64)
        nrows = indptr.size - 1
        if ncols is None:
            ncols = int(col_indices.max()) + 1 if col_indices.size else 0
        vals = np.asarray(values)
        dt = _values_dtype(vals, dtype)
        vals = np.ascontiguousarray(np.broadcast_to(np.asarray(vals, dt.np_type), col_indices.shape))
        C = cls.__new__(cls)
        C.dtype = dt
        C.name = _autoname("M") if name is None else name
        C._h = ctypes.c_void_p()
        C._nrows, C._ncols = int(nrows), int(ncols)
        call(f"GrB_Matrix_import_{dt.name}",
             [_Pointer(C), dt, nrows, ncols, _CArray(indptr, "indptr"), _CArray(col_indices, "col"),
              _CArray(vals, "values"), indptr.size, col_indices.size, vals.size, lib.GrB_CSR_FORMAT])
        return C

    def to_csr(self, dtype=None):
        dt = self.dtype if dtype is None else lookup_dtype(dtype)
        n = self.nvals
        ap = np.empty(self._nrows + 1, np.uint64)
        ai = np.empty(n, np.uint64)
        ax = np.empty(n, dt.np_type)
        lens = [ctypes.c_uint64(ap.size), ctypes.c_uint64(ai.size), ctypes.c_uint64(ax.size)]
        rc = getattr(lib, f"GrB_Matrix_export_{dt.name}")(
            ctypes.c_void_p(ap.ctypes.data), ctypes.c_void_p(ai.ctypes.data),
            ctypes.c_void_p(ax.ctypes.data), *[ctypes.byref(x) for x in lens], lib.GrB_CSR_FORMAT, self._h)
        check_status_carg(rc, "Matrix", self._h)
        return ap.astype(np.int64), ai.astype(np.int64), ax

    def to_coo(self, dtype=None, *, rows=True, columns=True, values=True, sort=True):
        dt = self.dtype if dtype is None else lookup_dtype(dtype)
        n = self.nvals
        r = np.empty(n, np.uint64)
        c = np.empty(n, np.uint64)
        v = np.empty(n, dt.np_type)
        nv = ctypes.c_uint64(n)
        rc = getattr(lib, f"GrB_Matrix_extractTuples_{dt.name}")(
            ctypes.c_void_p(r.ctypes.data), ctypes.c_void_p(c.ctypes.data), ctypes.c_void_p(v.ctypes.data),
            ctypes.byref(nv), self._h)
        check_status_carg(rc, "Matrix", self._h)
        return (r if rows else None, c if columns else None, v if values else None)

    def to_dict(self):
        r, c, v = self.to_coo()
        return {(int(a), int(b)): x.item() for a, b, x in zip(r, c, v)}

    def dup(self, dtype=None, *, clear=False, mask=None, name=None):
        if dtype is None and not clear and mask is None:
            C = Matrix.__new__(Matrix)
            C.dtype = self.dtype
            C.name = _autoname("M") if name is None else name
            C._h = ctypes.c_void_p()
            C._nrows, C._ncols = self._nrows, self._ncols
            call("GrB_Matrix_dup", [_Pointer(C), self])
            return C
        C = Matrix(self.dtype if dtype is None else dtype, self._nrows, self._ncols, name=name)
        if not clear:
            if mask is None:
                C << self
            else:
                C(mask=mask) << self
        return C

    def clear(self):
        call("GrB_Matrix_clear", [self])

    def resize(self, nrows, ncols):
        call("GrB_Matrix_resize", [self, nrows, ncols])
        self._nrows, self._ncols = int(nrows), int(ncols)

    def wait(self):
        call("GrB_Matrix_wait", [self, lib.GrB_MATERIALIZE])

    # ---------------------------------------------------------------- elements
    def __getitem__(self, keys):
        """A[i, j] element; A[I, J] -> GrB_Matrix_extract; A[I, j] / A[i, J] -> GrB_Col_extract
        (the row form with INP0 transposed), reference core/matrix.py:2860-2920."""
        if not isinstance(keys, tuple) or len(keys) != 2:
            raise TypeError("Matrix indexing requires a (rows, columns) pair")
        rk, rc, rn = _axis_index(keys[0], self._nrows)
        ck, cc, cn = _axis_index(keys[1], self._ncols)
        if rk == "scalar" and ck == "scalar":
            return _MatrixElement(self, rc, cc)
        from .vector import VectorExpression

        if rk == "scalar":
            return VectorExpression("extract", "GrB_Col_extract", [self, cc, cn, rc], at=True, dtype=self.dtype,
                                    size=cn)
        if ck == "scalar":
            return VectorExpression("extract", "GrB_Col_extract", [self, rc, rn, cc], dtype=self.dtype, size=rn)
        return MatrixExpression("extract", "GrB_Matrix_extract", [self, rc, rn, cc, cn], dtype=self.dtype,
                                nrows=rn, ncols=cn)

    def __setitem__(self, keys, value):
        if keys is Ellipsis or (isinstance(keys, tuple) and all(k == slice(None) for k in keys)):
            self._assign(Ellipsis, value, None, None, False)
            return
        i, j = _scalar_keys(keys, 2)
        from .scalar import Scalar

        if isinstance(value, Scalar):
            value = value.value
            if value is None:
                del self[i, j]
                return
        call(f"GrB_Matrix_setElement_{self.dtype.name}", [self, value, i, j])

    def __delitem__(self, keys):
        i, j = _scalar_keys(keys, 2)
        call("GrB_Matrix_removeElement", [self, i, j])

    def _assign(self, keys, value, mask, accum, replace):
        from .scalar import Scalar

        if keys not in (Ellipsis,) and not (isinstance(keys, tuple) and all(k == slice(None) for k in keys)) \
                and keys != slice(None):
            raise NotImplementedError("Matrix assign supports whole-matrix (A[:, :]) targets")
        desc = descriptor_lookup(mask_complement=mask.complement if mask is not None else False,
                                 mask_structure=mask.structure if mask is not None else False,
                                 output_replace=replace)
        if isinstance(value, TransposedMatrix):
            desc = descriptor_lookup(mask_complement=mask.complement if mask is not None else False,
                                     mask_structure=mask.structure if mask is not None else False,
                                     output_replace=replace, transpose_first=True)
            value = value._matrix
        if isinstance(value, Matrix):
            call("GrB_Matrix_assign", [self, mask, accum, value, lib.GrB_ALL, self._nrows, lib.GrB_ALL,
                                       self._ncols, desc])
            return
        if isinstance(value, Scalar):
            value = value.value
        call(f"GrB_Matrix_assign_{self.dtype.name}",
             [self, mask, accum, value, lib.GrB_ALL, self._nrows, lib.GrB_ALL, self._ncols, desc])

    # ---------------------------------------------------------------- operations
    def mxm(self, other, op=None):
        return _mxm(self, other, op)

    def mxv(self, other, op=None):
        return _mxv(self, other, op)

    def ewise_mult(self, other, op=None):
        return _ewise(self, other, op if op is not None else _op.binary.times, "mult")

    def ewise_add(self, other, op=None):
        return _ewise(self, other, op if op is not None else _op.monoid.plus, "add")

    def reduce_scalar(self, op=None, *, allow_empty=True):
        return _reduce_scalar(self, op, allow_empty)

    def reduce_rowwise(self, op=None):
        return _reduce_rows(self, op, columnwise=False)

    def reduce_columnwise(self, op=None):
        return _reduce_rows(self, op, columnwise=True)

    def apply(self, op, right=None, *, left=None):
        return _apply_expr(self, op, right, left)

    def isequal(self, other, *, check_dtype=False):
        """reference core/matrix.py:357-398"""
        if isinstance(other, TransposedMatrix):
            other = other.new()
        if not isinstance(other, Matrix):
            raise TypeError(f"Expected Matrix, got {type(other)}")
        if check_dtype and self.dtype != other.dtype:
            return False
        if self.shape != other.shape or self.nvals != other.nvals:
            return False
        opr = _op.binary.eq[self.dtype] if check_dtype else _op.get_typed_op(_op.binary.eq, self.dtype,
                                                                             other.dtype)
        matches = Matrix(BOOL, self._nrows, self._ncols, name="M_isequal")
        matches << self.ewise_mult(other, opr)
        if matches.nvals != self.nvals:
            return False
        return matches.reduce_scalar(_op.monoid.land, allow_empty=False).new().value

    def isclose(self, other, *, rel_tol=1e-7, abs_tol=0.0, check_dtype=False):
        if isinstance(other, TransposedMatrix):
            other = other.new()
        if check_dtype and self.dtype != other.dtype:
            return False
        if self.shape != other.shape or self.nvals != other.nvals:
            return False
        r1, c1, v1 = self.to_coo()
        r2, c2, v2 = other.to_coo()
        if not (np.array_equal(r1, r2) and np.array_equal(c1, c2)):
            return False
        return bool(np.all(np.isclose(v1, v2, rtol=rel_tol, atol=abs_tol, equal_nan=True)))

    def power(self, n, op=None):
        """A^n by repeated squaring with GrB_mxm (reference core/matrix.py:95-154, 2754-2806)."""
        if isinstance(n, bool) or not isinstance(n, (int, np.integer)):
            raise TypeError(f"n must be a positive integer; got bad type: {type(n)}")
        if n <= 0:
            raise ValueError(f"n must be a positive integer; got: {n}")
        if self._nrows != self._ncols:
            raise DimensionMismatch(f"power only works for square Matrix; shape is {self.shape}")
        op = _op.get_typed_op(op if op is not None else _op.semiring.plus_times, self.dtype,
                              kind="semiring")
        return MatrixExpression("power", None, [self, _power, (self, n, op)], op=op, nrows=self._nrows,
                                ncols=self._ncols, dtype=op.return_type)


def _power(updater, A, n, op):
    result = None
    base = A
    while True:
        if n & 1:
            result = base if result is None else result.mxm(base, op).new()
        n >>= 1
        if not n:
            break
        base = base.mxm(base, op).new()
    updater << result


def _axis_index(key, size):
    """One axis of an index: ("scalar", i, 1), or ("list", GrB_ALL | _CArray, length).  Slices
    other than ':' become explicit index arrays (the reference's non-SuiteSparse path,
    core/slice.py:26-33)."""
    if isinstance(key, (int, np.integer)) and not isinstance(key, bool):
        i = int(key)
        if i < 0:
            i += size
        if not 0 <= i < size:
            raise IndexError(f"index {int(key)} out of range for size {size}")
        return "scalar", i, 1
    if isinstance(key, slice):
        start, stop, step = key.indices(size)
        n = len(range(start, stop, step))
        if n == size and step == 1:
            return "list", lib.GrB_ALL, size
        return "list", _CArray(np.arange(start, stop, step, dtype=np.uint64), "I"), n
    arr = np.asarray(key)
    if arr.dtype == np.bool_:
        raise TypeError("boolean index arrays are not supported")
    arr = np.where(arr < 0, arr + size, arr) if arr.size else arr
    arr = _index_array(np.atleast_1d(arr), "indices")
    if arr.size and int(arr.max()) >= size:
        raise IndexError(f"index {int(arr.max())} out of range for size {size}")
    return "list", _CArray(arr, "I"), int(arr.size)


def _scalar_keys(keys, nd):
    if not isinstance(keys, tuple) or len(keys) != nd:
        raise TypeError(f"Expected {nd} integer indices")
    out = []
    for k in keys:
        if isinstance(k, (int, np.integer)) and not isinstance(k, bool):
            out.append(int(k))
        else:
            raise NotImplementedError("only scalar element indexing is supported")
    return out


class _MatrixElement:
    __slots__ = "parent", "i", "j"

    def __init__(self, parent, i, j):
        self.parent, self.i, self.j = parent, i, j

    def new(self, dtype=None, *, name=None):
        from .scalar import Scalar

        s = Scalar(self.parent.dtype if dtype is None else dtype, name=name)
        s.value = self.value
        return s

    @property
    def value(self):
        A = self.parent
        out = np.empty(1, A.dtype.np_type)
        rc = getattr(lib, f"GrB_Matrix_extractElement_{A.dtype.name}")(
            ctypes.c_void_p(out.ctypes.data), A._h, self.i, self.j)
        if check_status_carg(rc, "Matrix", A._h) is NoValue:
            return None
        return out[0].item()

    def __lshift__(self, value):
        self.parent[self.i, self.j] = value

    def __eq__(self, other):
        return self.value == other


class TransposedMatrix:
    ndim = 2
    _is_transposed = True
    _is_scalar = False

    def __init__(self, matrix):
        self._matrix = matrix

    @property
    def _carg(self):
        return self._matrix._carg

    @property
    def name(self):
        return self._matrix.name

    @property
    def dtype(self):
        return self._matrix.dtype

    @property
    def nrows(self):
        return self._matrix._ncols

    @property
    def ncols(self):
        return self._matrix._nrows

    _nrows = property(lambda self: self._matrix._ncols)
    _ncols = property(lambda self: self._matrix._nrows)

    @property
    def shape(self):
        return (self.nrows, self.ncols)

    @property
    def nvals(self):
        return self._matrix.nvals

    @property
    def T(self):
        return self._matrix

    def new(self, dtype=None, *, mask=None, name=None):
        C = Matrix(self.dtype if dtype is None else dtype, self.nrows, self.ncols, name=name)
        expr = MatrixExpression("transpose", "GrB_transpose", [self._matrix], dtype=self.dtype,
                                nrows=self.nrows, ncols=self.ncols)
        if mask is None:
            C << expr
        else:
            C(mask=_check_mask(mask)) << expr
        return C

    def mxm(self, other, op=None):
        return _mxm(self, other, op)

    def mxv(self, other, op=None):
        return _mxv(self, other, op)

    def ewise_mult(self, other, op=None):
        return _ewise(self, other, op if op is not None else _op.binary.times, "mult")

    def ewise_add(self, other, op=None):
        return _ewise(self, other, op if op is not None else _op.monoid.plus, "add")

    def power(self, n, op=None):
        return self.new().power(n, op)

    def reduce_rowwise(self, op=None):
        return _reduce_rows(self, op, columnwise=False)

    def reduce_columnwise(self, op=None):
        return _reduce_rows(self, op, columnwise=True)

    def reduce_scalar(self, op=None, *, allow_empty=True):
        return self._matrix.reduce_scalar(op, allow_empty=allow_empty)

    def apply(self, op, right=None, *, left=None):
        return _apply_expr(self, op, right, left)

    def to_coo(self, *args, **kw):
        r, c, v = self._matrix.to_coo(*args, **kw)
        o = np.lexsort((r, c))
        return c[o], r[o], v[o]

    def isequal(self, other, **kw):
        return self.new().isequal(other, **kw)

    def __matmul__(self, other):
        from .infix import _matmul_infix_expr

        return _matmul_infix_expr(self, other)

    def __rmatmul__(self, other):
        from .infix import _matmul_infix_expr

        return _matmul_infix_expr(other, self)


def _is_agg(op):
    return getattr(op, "opclass", None) == "Aggregator"


def _reduce_rows(A, op, *, columnwise):
    """A.reduce_rowwise / reduce_columnwise (reference core/matrix.py:2556-2623): a monoid (or a
    BinaryOp that is one) -> GrB_Matrix_reduce_Monoid (desc INP0=TRAN for columns of A, rows of
    A.T); an Aggregator -> its semiring lowering (agg.py)."""
    from .vector import VectorExpression

    if op is None:
        op = _op.monoid.plus
    size = A.ncols if columnwise else A.nrows
    if _is_agg(op):
        from .agg import reduce_rowwise_recipe

        typed = op[A.dtype] if op.opclass == "Aggregator" and not hasattr(op, "parent") else op
        return VectorExpression("reduce_columnwise" if columnwise else "reduce_rowwise", None,
                                [A, reduce_rowwise_recipe, (A, typed, columnwise)],
                                dtype=typed.return_type, size=size)
    t = _op.get_typed_op(op, A.dtype, kind="monoid")
    if t.opclass == "BinaryOp":
        mon = getattr(_op.monoid, t.parent.name, None)
        if mon is None or t.type not in mon._typed:
            raise TypeError(f"{op!r} is not a monoid; reduce needs a Monoid")
        t = mon[t.type]
    if t.opclass != "Monoid":
        raise TypeError(f"Expected a Monoid or Aggregator, got {t.opclass}")
    a, at = _unwrap(A)
    return VectorExpression("reduce_columnwise" if columnwise else "reduce_rowwise", "GrB_Matrix_reduce_Monoid",
                            [a], op=t, at=(at != columnwise), size=size)


def _reduce_scalar(x, op, allow_empty):
    """Vector.reduce / Matrix.reduce_scalar: monoids -> GrB_*_reduce_Monoid_Scalar; Aggregators ->
    the two-SpMV lowering of reference core/operator/agg.py:229-276."""
    from .scalar import ScalarExpression

    if op is None:
        op = _op.monoid.plus
    if _is_agg(op):
        from .agg import matrix_scalar_forbidden, reduce_scalar_recipe

        typed = op[x.dtype] if not hasattr(op, "parent") else op
        bad = matrix_scalar_forbidden(typed.parent) if x.ndim == 2 else None
        if bad:
            raise ValueError(f"Aggregator {bad} may not be used with Matrix.reduce_scalar.")
        if not allow_empty:
            if typed.parent._monoid is None:
                raise ValueError("allow_empty=False not allowed when using Aggregators")
            return _reduce_scalar(x, typed.parent._monoid[typed.type], allow_empty)
        return ScalarExpression("reduce", None, [x, reduce_scalar_recipe, (x, typed)],
                                dtype=typed.return_type)
    op = _op.get_typed_op(op, x.dtype, kind="monoid")
    if op.opclass == "BinaryOp":
        op = getattr(_op.monoid, op.parent.name)[op.type]
    kind = "Matrix" if x.ndim == 2 else "Vector"
    return ScalarExpression("reduce_scalar" if kind == "Matrix" else "reduce",
                            f"GrB_{kind}_reduce_Monoid_Scalar", [x], op=op, allow_empty=allow_empty)


def _apply_expr(x, op, right, left):
    """x.apply(op[, right= | left=]) (reference core/vector.py:1311-1460, core/matrix.py:2297-2447):
    a UnaryOp -> GrB_*_apply; a BinaryOp with a bound scalar -> GrB_*_apply_BinaryOp{1st,2nd}_<T>."""
    from .scalar import Scalar
    from .vector import VectorExpression

    kind = "Vector" if x.ndim == 1 else "Matrix"
    src, at = _unwrap(x) if kind == "Matrix" else (x, False)

    def mk(cf, args, t):
        if kind == "Vector":
            return VectorExpression("apply", cf, args, op=t, size=x.size)
        return MatrixExpression("apply", cf, args, op=t, at=at, nrows=x.nrows, ncols=x.ncols)

    if left is None and right is None:
        t = _op.get_typed_op(op, x.dtype, kind="unary")
        if t.opclass != "UnaryOp":
            raise TypeError(f"Bad type for argument `op`: expected UnaryOp, got {t.opclass}")
        return mk(f"GrB_{kind}_apply", [src], t)
    if left is not None and right is not None:
        raise TypeError("Cannot provide both `left` and `right` to apply")
    val = left if right is None else right
    sc = val if isinstance(val, Scalar) else Scalar.from_value(val)
    if right is None:
        t = _op.get_typed_op(op, sc.dtype, x.dtype, kind="binary", is_left_scalar=True)
    else:
        t = _op.get_typed_op(op, x.dtype, sc.dtype, kind="binary", is_right_scalar=True)
    if t.opclass == "Monoid":
        t = getattr(_op.binary, t.parent.name)[t.type]
    elif t.opclass != "BinaryOp":
        raise TypeError(f"Bad type for argument `op`: expected BinaryOp, got {t.opclass}")
    if t.is_positional:
        raise NotImplementedError("positional operators in apply")
    cv = sc.value
    if right is None:
        return mk(f"GrB_{kind}_apply_BinaryOp1st_{sc.dtype.name}", [cv, src], t)
    return mk(f"GrB_{kind}_apply_BinaryOp2nd_{sc.dtype.name}", [src, cv], t)


def _unwrap(x):
    if isinstance(x, TransposedMatrix):
        return x._matrix, True
    return x, False


def _binary_for(opobj, dtype):
    t = _op.get_typed_op(opobj, dtype, kind="binary")
    if t.opclass == "Monoid":
        t = getattr(_op.binary, t.parent.name)[t.type]
    return t


def _mxm(left, right, op):
    from .vector import Vector

    if isinstance(right, Vector):
        raise TypeError("mxm requires a Matrix on the right; use mxv for vectors")
    if op is None:
        op = _op.semiring.plus_times
    op = _op.get_typed_op(op, left.dtype, right.dtype, kind="semiring")
    if op.opclass != "Semiring":
        raise TypeError(f"Expected a Semiring, got {op.opclass}")
    a, at = _unwrap(left)
    b, bt = _unwrap(right)
    if left.ncols != right.nrows:
        raise DimensionMismatch(f"Dimensions not compatible for mxm: {left.shape} and {right.shape}")
    return MatrixExpression("mxm", "GrB_mxm", [a, b], op=op, at=at, bt=bt, nrows=left.nrows,
                            ncols=right.ncols)


def _mxv(left, v, op):
    from .vector import Vector, VectorExpression

    if not isinstance(v, Vector):
        raise TypeError(f"mxv requires a Vector, got {type(v)}")
    if op is None:
        op = _op.semiring.plus_times
    op = _op.get_typed_op(op, left.dtype, v.dtype, kind="semiring")
    if op.opclass != "Semiring":
        raise TypeError(f"Expected a Semiring, got {op.opclass}")
    a, at = _unwrap(left)
    if left.ncols != v.size:
        raise DimensionMismatch(f"Dimensions not compatible for mxv: {left.shape} and {v.size}")
    return VectorExpression("mxv", "GrB_mxv", [a, v], op=op, at=at, size=left.nrows)


def _ewise(left, right, opobj, kind):
    a, at = _unwrap(left)
    b, bt = _unwrap(right)
    op = _op.get_typed_op(opobj, left.dtype, right.dtype, kind="binary")
    if op.opclass == "Monoid":
        op = getattr(_op.binary, op.parent.name if op.parent.name != "eq" else "lxnor")[op.type]
    if left.shape != right.shape:
        raise DimensionMismatch(f"Dimensions do not match: {left.shape} and {right.shape}")
    cf = "GrB_Matrix_eWiseMult_BinaryOp" if kind == "mult" else "GrB_Matrix_eWiseAdd_BinaryOp"
    return MatrixExpression(f"ewise_{kind}", cf, [a, b], op=op, at=at, bt=bt, nrows=left.nrows,
                            ncols=left.ncols)


class MatrixExpression(BaseExpression):
    output_type = Matrix
    ndim = 2

    def __init__(self, method_name, cfunc_name, args, *, at=False, bt=False, op=None, dtype=None,
                 nrows=None, ncols=None, expr_repr=None):
        super().__init__(method_name, cfunc_name, args, at=at, bt=bt, op=op, dtype=dtype,
                         expr_repr=expr_repr)
        self._nrows = nrows
        self._ncols = ncols

    @property
    def nrows(self):
        return self._nrows

    @property
    def ncols(self):
        return self._ncols

    @property
    def shape(self):
        return (self._nrows, self._ncols)

    def construct_output(self, dtype=None, *, name=None):
        return Matrix(self.dtype if dtype is None else dtype, self._nrows, self._ncols, name=name)

    def __repr__(self):
        return f"<MatrixExpression {self.method_name} {self._nrows}x{self._ncols} {self.dtype}>"
