"""Vector collection and its delayed expressions (mirrors the hot-path parts of
reference core/vector.py: new :152-184, build :538, from_coo :731,
to_coo :482, isequal :329, reduce :1561, vxm :1259-1307, inner :1609-1651,
outer :1653-1693)."""
import ctypes

import numpy as np

from . import operator as _op
from ._lib import lib
from .base import (BaseExpression, BaseType, StructuralMask, ValueMask, _autoname, _Cast, _Pointer, call,
                   descriptor_lookup)
from .dtypes import BOOL, FP64, lookup_dtype
from .exceptions import DimensionMismatch, NoValue, check_status_carg
from .matrix import Matrix, MatrixExpression, TransposedMatrix, _apply_expr, _axis_index, _binary_for, \
    _CArray, _index_array, _reduce_scalar, _values_dtype


class Vector(BaseType):
    ndim = 1

    def __init__(self, dtype=FP64, size=0, *, name=None):
        self.dtype = lookup_dtype(dtype)
        self.name = _autoname("v") if name is None else name
        self._h = ctypes.c_void_p()
        self._size = int(size)
        call("GrB_Vector_new", [_Pointer(self), self.dtype, self._size])

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            try:
                lib.GrB_Vector_free(ctypes.byref(h))
            except Exception:
                pass

    @property
    def size(self):
        return self._size

    @property
    def shape(self):
        return (self._size,)

    @property
    def nvals(self):
        n = ctypes.c_uint64()
        check_status_carg(lib.GrB_Vector_nvals(ctypes.byref(n), self._h), "Vector", self._h)
        return n.value

    _nvals = nvals

    @property
    def ss(self):
        from .ss import VectorSS

        return VectorSS(self)

    @property
    def S(self):
        return StructuralMask(self)

    @property
    def V(self):
        return ValueMask(self)

    def __repr__(self):
        return f"<Vector {self.name}: size={self._size}, nvals={self.nvals}, {self.dtype}>"

    # ---------------------------------------------------------------- construction
    @classmethod
    def from_coo(cls, indices, values=1.0, dtype=None, *, size=None, dup_op=None, name=None):
        indices = _index_array(indices, "indices")
        if size is None:
            size = int(indices.max()) + 1 if indices.size else 0
        if np.ndim(values) == 0 and not isinstance(values, np.ndarray):
            dt = _values_dtype(values, dtype)
            v = cls(dt, size, name=name)
            if indices.size:
                x = np.asarray(values, dt.np_type).item()
                call(f"GxB_Vector_build_Scalar_{dt.name}", [v, _CArray(indices, "indices"), x, indices.size])
            return v
        vals = np.asarray(values)
        dt = _values_dtype(vals, dtype)
        v = cls(dt, size, name=name)
        v.build(indices, vals, dup_op=dup_op)
        return v

    def build(self, indices, values, *, dup_op=None, clear=False, size=None):
        indices = _index_array(indices, "indices")
        values = np.ascontiguousarray(np.broadcast_to(np.asarray(values, self.dtype.np_type), indices.shape))
        n = values.shape[0]
        if indices.size != n:
            raise ValueError(f"`indices` and `values` lengths must match: {indices.size}, {values.size}")
        if clear:
            self.clear()
        if size is not None:
            self.resize(size)
        if n == 0:
            return
        dup = None if dup_op is None else _binary_for(dup_op, self.dtype)
        call(f"GrB_Vector_build_{self.dtype.name}", [self, _CArray(indices, "indices"),
                                                    _CArray(values, "values"), n, dup])
        if dup_op is None and self.nvals < n:
            raise ValueError("Duplicate indices found, must provide `dup_op` BinaryOp")

    def to_coo(self, dtype=None, *, indices=True, values=True, sort=True):
        dt = self.dtype if dtype is None else lookup_dtype(dtype)
        n = self.nvals
        idx = np.empty(n, np.uint64)
        vals = np.empty(n, dt.np_type)
        nv = ctypes.c_uint64(n)
        rc = getattr(lib, f"GrB_Vector_extractTuples_{dt.name}")(
            ctypes.c_void_p(idx.ctypes.data), ctypes.c_void_p(vals.ctypes.data), ctypes.byref(nv), self._h)
        check_status_carg(rc, "Vector", self._h)
        return (idx if indices else None, vals if values else None)

    def to_dict(self):
        i, v = self.to_coo()
        return {int(a): x.item() for a, x in zip(i, v)}

    def to_dense(self, fill_value=None, dtype=None):
        i, v = self.to_coo(dtype)
        dt = v.dtype
        if fill_value is None:
            if i.size != self._size:
                raise TypeError("fill_value must be given when the Vector is not full")
            fill_value = 0
        out = np.full(self._size, fill_value, dt)
        out[i.astype(np.int64)] = v
        return out

    def dup(self, dtype=None, *, clear=False, mask=None, name=None):
        if dtype is None and not clear and mask is None:
            w = Vector.__new__(Vector)
            w.dtype = self.dtype
            w.name = _autoname("v") if name is None else name
            w._h = ctypes.c_void_p()
            w._size = self._size
            call("GrB_Vector_dup", [_Pointer(w), self])
            return w
        w = Vector(self.dtype if dtype is None else dtype, self._size, name=name)
        if not clear:
            if mask is None:
                w << self
            else:
                w(mask=mask) << self
        return w

    def clear(self):
        call("GrB_Vector_clear", [self])

    def resize(self, size):
        call("GrB_Vector_resize", [self, size])
        self._size = int(size)

    def wait(self):
        call("GrB_Vector_wait", [self, lib.GrB_MATERIALIZE])

    # ---------------------------------------------------------------- elements / assign
    def __getitem__(self, key):
        """v[i] element; v[I] -> GrB_Vector_extract (reference core/vector.py:1010-1030)."""
        kind, idx, n = _axis_index(key, self._size)
        if kind == "scalar":
            return _VectorElement(self, idx)
        return VectorExpression("extract", "GrB_Vector_extract", [self, idx, n], dtype=self.dtype, size=n)

    def _as_matrix(self):
        """The same object as an n x 1 Matrix (reference core/vector.py:186-205: a
        `(GrB_Matrix)` cast of the handle; the library accepts either kind)."""
        A = Matrix.__new__(Matrix)
        A.dtype = self.dtype
        A.name = f"(GrB_Matrix){self.name}"
        A._h = ctypes.c_void_p(self._h.value)
        A._nrows, A._ncols = self._size, 1
        A._parent = self
        return A

    def __setitem__(self, key, value):
        if isinstance(key, (int, np.integer)) and not isinstance(key, bool):
            from .scalar import Scalar

            if isinstance(value, Scalar):
                value = value.value
                if value is None:
                    del self[key]
                    return
            call(f"GrB_Vector_setElement_{self.dtype.name}", [self, value, int(key)])
            return
        self._assign(key, value, None, None, False)

    def __delitem__(self, key):
        call("GrB_Vector_removeElement", [self, int(key)])

    def _assign(self, keys, value, mask, accum, replace):
        """w(mask, accum, replace)[I] = value  (GrB_Vector_assign[_T], GrB_ALL for ':')."""
        from .scalar import Scalar

        if keys is Ellipsis or keys == slice(None):
            idx, ni = lib.GrB_ALL, self._size
            idx_obj = None
        else:
            if isinstance(keys, slice):
                keys = np.arange(self._size)[keys]
            arr = _index_array(np.atleast_1d(keys), "indices")
            idx_obj = _CArray(arr, "I")
            idx, ni = idx_obj, arr.size
        desc = descriptor_lookup(mask_complement=mask.complement if mask is not None else False,
                                 mask_structure=mask.structure if mask is not None else False, output_replace=replace)
        if isinstance(value, Vector):
            call("GrB_Vector_assign", [self, mask, accum, value, idx, ni, desc])
            return
        if isinstance(value, Scalar):
            value = value.value
        call(f"GrB_Vector_assign_{self.dtype.name}", [self, mask, accum, value, idx, ni, desc])

    # ---------------------------------------------------------------- operations
    def vxm(self, other, op=None):
        if not isinstance(other, (Matrix, TransposedMatrix)):
            raise TypeError(f"vxm requires a Matrix, got {type(other)}")
        if op is None:
            op = _op.semiring.plus_times
        op = _op.get_typed_op(op, self.dtype, other.dtype, kind="semiring")
        if op.opclass != "Semiring":
            raise TypeError(f"Expected a Semiring, got {op.opclass}")
        if self._size != other.nrows:
            raise DimensionMismatch(f"Dimensions not compatible for vxm: {self._size} and {other.shape}")
        bt = isinstance(other, TransposedMatrix)
        A = other._matrix if bt else other
        return VectorExpression("vxm", "GrB_vxm", [self, A], op=op, bt=bt, size=other.ncols)

    def inner(self, other, op=None):
        """s = u' v  through GrB_vxm with v cast to an n x 1 matrix (reference core/vector.py:1609-1651)."""
        from .scalar import ScalarExpression

        if op is None:
            op = _op.semiring.plus_times
        op = _op.get_typed_op(op, self.dtype, other.dtype, kind="semiring")
        if self._size != other._size:
            raise DimensionMismatch(f"Size mismatch for inner: {self._size} and {other._size}")
        return ScalarExpression("inner", "GrB_vxm", [self, _Cast(other, "GrB_Matrix")], op=op,
                                scalar_as_vector=True)

    def outer(self, other, op=None):
        """C = u v' through GrB_mxm with any_<op> (reference core/vector.py:1653-1693)."""
        opobj = _op.binary.times if op is None else op
        bop = _op.get_typed_op(opobj, self.dtype, other.dtype, kind="binary")
        if bop.opclass == "Monoid":
            bop = getattr(_op.binary, bop.parent.name)[bop.type]
        sr = getattr(_op.semiring, f"any_{bop.parent.name}")[bop.type]
        return MatrixExpression("outer", "GrB_mxm", [_Cast(self, "GrB_Matrix"), _Cast(other, "GrB_Matrix")],
                                op=sr, bt=True, nrows=self._size, ncols=other._size)

    def ewise_mult(self, other, op=None):
        return self._ewise(other, op if op is not None else _op.binary.times, "mult")

    def ewise_add(self, other, op=None):
        return self._ewise(other, op if op is not None else _op.monoid.plus, "add")

    def _ewise(self, other, opobj, kind):
        op = _op.get_typed_op(opobj, self.dtype, other.dtype, kind="binary")
        if op.opclass == "Monoid":
            op = getattr(_op.binary, op.parent.name if op.parent.name != "eq" else "lxnor")[op.type]
        if self._size != other._size:
            raise DimensionMismatch(f"Size mismatch: {self._size} and {other._size}")
        cf = "GrB_Vector_eWiseMult_BinaryOp" if kind == "mult" else "GrB_Vector_eWiseAdd_BinaryOp"
        return VectorExpression(f"ewise_{kind}", cf, [self, other], op=op, size=self._size)

    def reduce(self, op=None, *, allow_empty=True):
        return _reduce_scalar(self, op, allow_empty)

    def apply(self, op, right=None, *, left=None):
        return _apply_expr(self, op, right, left)

    def isequal(self, other, *, check_dtype=False):
        if not isinstance(other, Vector):
            raise TypeError(f"Expected Vector, got {type(other)}")
        if check_dtype and self.dtype != other.dtype:
            return False
        if self._size != other._size or self.nvals != other.nvals:
            return False
        opr = _op.binary.eq[self.dtype] if check_dtype else _op.get_typed_op(_op.binary.eq, self.dtype,
                                                                             other.dtype)
        matches = Vector(BOOL, self._size, name="v_isequal")
        matches << self.ewise_mult(other, opr)
        if matches.nvals != self.nvals:
            return False
        return matches.reduce(_op.monoid.land, allow_empty=False).new().value

    def isclose(self, other, *, rel_tol=1e-7, abs_tol=0.0, check_dtype=False):
        if check_dtype and self.dtype != other.dtype:
            return False
        if self._size != other._size or self.nvals != other.nvals:
            return False
        i1, v1 = self.to_coo()
        i2, v2 = other.to_coo()
        if not np.array_equal(i1, i2):
            return False
        return bool(np.all(np.isclose(v1, v2, rtol=rel_tol, atol=abs_tol, equal_nan=True)))


class _VectorElement:
    __slots__ = "parent", "i"

    def __init__(self, parent, i):
        self.parent, self.i = parent, i

    def new(self, dtype=None, *, name=None):
        from .scalar import Scalar

        s = Scalar(self.parent.dtype if dtype is None else dtype, name=name)
        s.value = self.value
        return s

    @property
    def value(self):
        v = self.parent
        out = np.empty(1, v.dtype.np_type)
        rc = getattr(lib, f"GrB_Vector_extractElement_{v.dtype.name}")(
            ctypes.c_void_p(out.ctypes.data), v._h, self.i)
        if check_status_carg(rc, "Vector", v._h) is NoValue:
            return None
        return out[0].item()

    def __lshift__(self, value):
        self.parent[self.i] = value

    def __eq__(self, other):
        return self.value == other


class VectorExpression(BaseExpression):
    output_type = Vector
    ndim = 1

    def __init__(self, method_name, cfunc_name, args, *, at=False, bt=False, op=None, dtype=None, size=None,
                 expr_repr=None):
        super().__init__(method_name, cfunc_name, args, at=at, bt=bt, op=op, dtype=dtype, expr_repr=expr_repr)
        self._size = size

    @property
    def size(self):
        return self._size

    @property
    def shape(self):
        return (self._size,)

    def construct_output(self, dtype=None, *, name=None):
        return Vector(self.dtype if dtype is None else dtype, self._size, name=name)

    def __repr__(self):
        return f"<VectorExpression {self.method_name} size={self._size} {self.dtype}>"
