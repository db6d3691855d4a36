"""`A @ B` delayed matmul expressions (reference core/infix.py:251-259, 388-397,
444-497; default semiring resolution core/expr.py:504-508)."""
from . import operator as _op


class InfixExpr:
    def __init__(self, left, right, method):
        self.left = left
        self.right = right
        self.method = method

    def _with_op(self, op):
        return getattr(self.left, self.method)(self.right, op)

    def _to_expr(self):
        default = {"ewise_mult": _op.binary.times, "ewise_add": _op.monoid.plus}.get(self.method,
                                                                                   _op.semiring.plus_times)
        return self._with_op(default)

    def new(self, dtype=None, *, mask=None, name=None, **opts):
        return self._to_expr().new(dtype, mask=mask, name=name, **opts)

    @property
    def dtype(self):
        return self._to_expr().dtype

    @property
    def size(self):
        return self._to_expr().size

    @property
    def nrows(self):
        return self._to_expr().nrows

    @property
    def ncols(self):
        return self._to_expr().ncols

    @property
    def shape(self):
        return self._to_expr().shape


def _matmul_infix_expr(left, right):
    from .matrix import Matrix, TransposedMatrix
    from .vector import Vector

    lm = isinstance(left, (Matrix, TransposedMatrix))
    rm = isinstance(right, (Matrix, TransposedMatrix))
    if lm and rm:
        method = "mxm"
    elif lm and isinstance(right, Vector):
        method = "mxv"
    elif isinstance(left, Vector) and rm:
        method = "vxm"
    elif isinstance(left, Vector) and isinstance(right, Vector):
        method = "inner"
    else:
        return NotImplemented
    expr = InfixExpr(left, right, method)
    expr._to_expr()  # shape check now (reference core/infix.py:492)
    return expr


def _ewise_infix_expr(left, right, method):
    """`x & y` (eWiseMult) / `x | y` (eWiseAdd) (reference core/infix.py:251-259, 388-397)."""
    from .base import Mask

    if isinstance(right, Mask):  # v | mask, v & mask (reference core/infix.py:420-423)
        return right.__ror__(left) if method == "ewise_add" else right.__rand__(left)
    if getattr(left, "ndim", None) is None or getattr(right, "ndim", None) is None:
        return NotImplemented
    return InfixExpr(left, right, method)
