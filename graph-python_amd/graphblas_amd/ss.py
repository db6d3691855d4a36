"""``Vector.ss`` / ``Matrix.ss`` extension namespaces: the prefix scan.

``prefix_scan`` restates reference core/ss/prefix_scan.py:12-172: a
Blelloch up-sweep / down-sweep expressed entirely as masked, accumulated
``mxm`` / ``vxm`` calls with the semiring ``<monoid>_first`` against small
iso selection matrices (one per level, log2(N) levels), on the entries of
each row compacted to positions 0..deg-1.  Every level is one library call,
so the scan runs on the device kernels of the hot path (masked SpGEMM /
SpMV + accumulate write-back).  Compaction / de-compaction of the index
space goes through to_coo / from_coo (the reference uses the ss export /
import of the same arrays).
"""
from math import ceil, log2

import numpy as np

from . import operator as _op
from .dtypes import INT8


def _scan_monoid(x, op):
    t = _op.get_typed_op(op, x.dtype, kind="monoid")
    if t.opclass == "BinaryOp":
        mon = getattr(_op.monoid, t.parent.name, None)
        if mon is None or t.type not in mon._typed:
            raise TypeError(f"Bad type for argument `op` in scan: {op!r} is a BinaryOp with no Monoid")
        t = mon[t.type]
    if t.opclass != "Monoid":
        raise TypeError(f"Bad type for argument `op` in scan: expected Monoid, got {t.opclass}")
    return t


def _iso_pattern(rows, cols, nrows, ncols, name):
    from .matrix import Matrix

    return Matrix.from_coo(np.asarray(rows, np.uint64), np.asarray(cols, np.uint64), 1, dtype=INT8,
                           nrows=nrows, ncols=ncols, name=name)


def prefix_scan(A, op, *, name=None):
    from .matrix import Matrix, TransposedMatrix
    from .vector import Vector

    mon = _scan_monoid(A, op)
    mname = mon.parent.name
    semiring = getattr(_op.semiring, f"{'lxnor' if mname == 'eq' else mname}_first")[mon.type]
    accum = getattr(_op.binary, "lxnor" if mname == "eq" else mname)[mon.type]
    is_vector = A.ndim == 1
    is_transposed = isinstance(A, TransposedMatrix)
    if A.shape[-1] < 2:
        return A.T.dup(name=name) if is_transposed else A.dup(name=name)

    # compact every row to positions 0..deg-1 (reference prefix_scan.py:36-63)
    if is_vector:
        idx, vals = A.to_coo()
        n_cols = len(idx)
        Ac = Vector.from_coo(np.arange(n_cols, dtype=np.uint64), vals, dtype=A.dtype, size=n_cols)
    else:
        rows, cols, vals = A.to_coo()
        nr = A.nrows
        rows64 = rows.astype(np.int64)
        deg = np.bincount(rows64, minlength=nr)
        start = np.zeros(nr + 1, np.int64)
        np.cumsum(deg, out=start[1:])
        pos = np.arange(len(rows64), dtype=np.int64) - start[rows64]
        n_cols = int(deg.max()) if len(deg) else 0
        Ac = Matrix.from_coo(rows, pos.astype(np.uint64), vals, dtype=A.dtype, nrows=nr, ncols=max(n_cols, 1))
    if n_cols < 2:
        return A.T.dup(name=name) if is_transposed else A.dup(name=name)
    n_half = n_cols // 2

    def mul(X, S):
        return X.vxm(S, semiring) if is_vector else X.mxm(S, semiring)

    # first iteration: pairwise sums (reference :75-92)
    j = np.arange(n_half)
    S = _iso_pattern(np.stack([2 * j, 2 * j + 1], 1).ravel(), np.repeat(j, 2), n_cols, n_half, "Up_0")
    B = mul(Ac, S).new(name="B")
    mask = None if is_vector else B.S

    # up-sweep (reference :94-116)
    stride, stride2 = 1, 2
    while stride2 <= n_half:
        c = np.arange(stride2 - 1, n_half, stride2)
        S = _iso_pattern(c - stride, c, n_half, n_half, "Up")
        B(accum, mask=mask) << mul(B, S)
        stride, stride2 = stride2, stride2 * 2

    # down-sweep (reference :118-146)
    if n_half > 2:
        stride2 = max(2, 2 ** ceil(log2(n_half // 2)))
        stride = stride2 // 2
        while stride > 0:
            c = np.arange(stride2 + stride - 1, n_half, stride2)
            if c.size == 0:
                stride2 = stride
                stride //= 2
                continue
            S = _iso_pattern(c - stride, c, n_half, n_half, "Down")
            B(accum, mask=mask) << mul(B, S)
            stride2 = stride
            stride //= 2

    # last iteration: spread to odd positions, then add the even originals (reference :148-170)
    indptr = np.arange(0, 2 * n_half + 2, 2)
    indptr[-1] = n_cols - 1
    lr = np.repeat(np.arange(n_half), np.diff(indptr))
    S = _iso_pattern(lr, np.arange(1, n_cols), n_half, n_cols, "Down_last")
    RV = mul(B, S).new(mask=Ac.S, name="RV")
    ev = np.arange(0, n_cols, 2)
    D = _iso_pattern(ev, ev, n_cols, n_cols, "D")
    RV(accum) << mul(Ac, D)

    # de-compact into the input's index space
    if is_vector:
        _, rv = RV.to_coo()
        return Vector.from_coo(idx, rv, dtype=RV.dtype, size=A.size, name=name)
    _, _, rv = RV.to_coo()
    if is_transposed:
        M = A.T
        return Matrix.from_coo(cols, rows, rv, dtype=RV.dtype, nrows=M.nrows, ncols=M.ncols, name=name)
    return Matrix.from_coo(rows, cols, rv, dtype=RV.dtype, nrows=A.nrows, ncols=A.ncols, name=name)


_ORDERS = {"rowwise": "rowwise", "row": "rowwise", "rows": "rowwise", "c": "rowwise",
           "columnwise": "columnwise", "col": "columnwise", "cols": "columnwise", "column": "columnwise",
           "columns": "columnwise", "f": "columnwise"}


class VectorSS:
    def __init__(self, parent):
        self._parent = parent

    def scan(self, op=None, *, name=None):
        """Prefix scan with a monoid (reference core/ss/vector.py:1365-1375)."""
        return prefix_scan(self._parent, _op.monoid.plus if op is None else op, name=name)


class MatrixSS:
    def __init__(self, parent):
        self._parent = parent

    def scan(self, op=None, order="rowwise", *, name=None):
        """Prefix scan along rows (default) or columns (reference core/ss/matrix.py:3701-3715)."""
        key = order.lower() if isinstance(order, str) else order
        if key not in _ORDERS:
            raise ValueError(f"Bad value for order: {order!r}")
        parent = self._parent
        if _ORDERS[key] == "columnwise":
            parent = parent.T
        return prefix_scan(parent, _op.monoid.plus if op is None else op, name=name)
