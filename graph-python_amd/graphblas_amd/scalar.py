"""Scalar collection (a GrB_Scalar, i.e. a one-element vector in this backend)
and scalar-valued expressions (reference core/scalar.py:555-594, 884-895)."""
import ctypes

import numpy as np

from ._lib import lib
from .base import BaseExpression, BaseType, _autoname, _Pointer, call
from .dtypes import FP64, lookup_dtype
from .exceptions import EmptyObject, NoValue, check_status_carg


class _CPtr:
    """Pointer to a host C scalar output (recorded as &s_temp)."""

    __slots__ = "array"
    name = "&s_temp"

    def __init__(self, array):
        self.array = array

    @property
    def _carg(self):
        return ctypes.c_void_p(self.array.ctypes.data)


class Scalar(BaseType):
    _is_scalar = True
    ndim = 0

    def __init__(self, dtype=FP64, *, name=None):
        self.dtype = lookup_dtype(dtype)
        self.name = _autoname("s") if name is None else name
        self._h = ctypes.c_void_p()
        call("GrB_Scalar_new", [_Pointer(self), self.dtype])

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            try:
                lib.GrB_Scalar_free(ctypes.byref(h))
            except Exception:
                pass

    @classmethod
    def from_value(cls, value, dtype=None, *, name=None, **_):
        if isinstance(value, Scalar):
            dtype = value.dtype if dtype is None else dtype
            value = value.value
        if dtype is None:
            a = np.asarray(value)
            dtype = a.dtype if a.dtype != object else FP64
        s = cls(dtype, name=name)
        s.value = value
        return s

    @property
    def nvals(self):
        n = ctypes.c_uint64()
        check_status_carg(lib.GrB_Scalar_nvals(ctypes.byref(n), self._h), "Scalar", self._h)
        return n.value

    @property
    def is_empty(self):
        return self.nvals == 0

    @property
    def value(self):
        out = np.empty(1, self.dtype.np_type)
        rc = getattr(lib, f"GrB_Scalar_extractElement_{self.dtype.name}")(
            ctypes.c_void_p(out.ctypes.data), self._h)
        if check_status_carg(rc, "Scalar", self._h) is NoValue:
            return None
        return out[0].item()

    @value.setter
    def value(self, val):
        if isinstance(val, Scalar):
            val = val.value
        if val is None:
            call("GrB_Scalar_clear", [self])
            return
        call(f"GrB_Scalar_setElement_{self.dtype.name}", [self, np.asarray(val, self.dtype.np_type).item()])

    def clear(self):
        call("GrB_Scalar_clear", [self])

    def dup(self, dtype=None, *, name=None):
        s = Scalar(self.dtype if dtype is None else dtype, name=name)
        s.value = self.value
        return s

    def isequal(self, other, *, check_dtype=False):
        if not isinstance(other, Scalar):
            other = Scalar.from_value(other)
        if check_dtype and self.dtype != other.dtype:
            return False
        return self.value == other.value

    def __eq__(self, other):
        if isinstance(other, Scalar):
            other = other.value
        return self.value == other

    def __hash__(self):
        return id(self)

    def __bool__(self):
        return bool(self.value)

    def __int__(self):
        return int(self.value)

    def __float__(self):
        return float(self.value)

    def __repr__(self):
        return f"<Scalar {self.name}: {self.value!r}, {self.dtype}>"

    def _assign(self, keys, value, mask, accum, replace):
        self.value = value


class ScalarExpression(BaseExpression):
    """Scalar-valued expression: reduce (GrB_*_reduce_Monoid_Scalar) or inner (GrB_vxm with the
    output scalar cast to a 1-element vector, reference core/base.py:456-474)."""

    output_type = Scalar
    _is_scalar = True

    def __init__(self, method_name, cfunc_name, args, *, op=None, dtype=None, scalar_as_vector=False,
                 allow_empty=True, **_):
        super().__init__(method_name, cfunc_name, args, op=op, dtype=dtype)
        self._scalar_as_vector = scalar_as_vector
        self._allow_empty = allow_empty

    def construct_output(self, dtype=None, *, name=None):
        return Scalar(self.dtype if dtype is None else dtype, name=name)

    def new(self, dtype=None, *, mask=None, name=None, **opts):
        if mask is not None:
            raise TypeError("Mask not allowed for Scalars")
        s = self.construct_output(dtype, name=name)
        if not self._allow_empty and self.cfunc_name and self.cfunc_name.endswith("reduce_Monoid_Scalar"):
            # allow_empty=False: C-scalar reduce, an empty input yields the monoid identity
            # (reference core/vector.py:1561 reduce -> GrB_Vector_reduce_<T>)
            A = self.args[0]
            kind = "Matrix" if A.ndim == 2 else "Vector"
            dt = self.op.type
            out = np.zeros(1, dt.np_type)
            call(f"GrB_{kind}_reduce_{dt.name}", [_CPtr(out), None, self.op, A, None])
            s.value = out[0].item()
            return s
        s._update(self, opts=opts)
        return s

    @property
    def value(self):
        return self.new().value

    def __eq__(self, other):
        return self.new() == other

    def __bool__(self):
        return bool(self.new())
