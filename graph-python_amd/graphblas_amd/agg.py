"""Aggregators and their lowering onto the library's semiring kernels.

Restates reference core/operator/agg.py: the ``Aggregator`` / ``TypedAggregator``
pair (:31-160) and ``TypedAggregator._new`` (:162-279), which turns every
reduction into GraphBLAS calls:

* monoid aggregators (sum, prod, min, max, any, all, any_value, bitwise_*) ->
  GrB_Matrix_reduce_Monoid / GrB_*_reduce_Monoid_Scalar;
* semiring aggregators (count, count_nonzero, count_zero, exists,
  sum_of_squares, sum_of_inverses, hypot, logaddexp, logaddexp2, L1norm,
  Linfnorm) -> ``A @ init`` SpMV with an iso-full init vector (the reference's
  "O(1) dense vector", :220-227), then GrB_*_apply for the finalizer;
* composite aggregators (mean, ptp, varp, vars, stdp, stds, geometric_mean,
  harmonic_mean, root_mean_square) -> their parts, combined with eWiseMult /
  apply (:286-353).

Row/column reductions thus run on the general SpMV kernel (gb_mxv.hip
k_spmv_words) with no host round trip.  The positional aggregators
(``agg.ss.first/last/first_index/last_index/argmin/argmax``, reference :478-696)
run on the positional semirings (min/max_secondi, min_firstj), any_eq mxm and
a masked any_first mxm, as the reference lowers them; the diagonal matrices
the reference takes with ``diag()`` are built from the step vector's COO.
"""
from functools import partial

import numpy as np

from . import operator as _op
from .dtypes import FP64, INT64, lookup_dtype


def _chain_types(ops, initdtype):
    """Input dtype -> result dtype through a chain of ops (reference agg.py:12-28)."""
    first = ops[0]
    if initdtype is None:
        prev = dict(first.types)
    else:
        prev = {}
        for key in first.types:
            try:
                prev[key] = _op.get_typed_op(first, key, initdtype).return_type
            except KeyError:
                pass
    for o in ops[1:]:
        prev = {k: o.types[v] for k, v in prev.items() if v in o.types}
    return prev


class Aggregator:
    opclass = "Aggregator"

    def __init__(self, name, *, initval=None, monoid=None, semiring=None, switch=False, semiring2=None,
                 applybegin=None, finalize=None, composite=None, custom=None, types=None, any_dtype=None):
        self.name = name
        self._custom = custom
        self._initval_orig = initval
        self._initval = False if initval is None else initval
        self._initdtype = lookup_dtype(np.asarray(self._initval).dtype)
        self._monoid = monoid
        self._semiring = semiring
        self._semiring2 = semiring2
        self._switch = switch
        self._applybegin = applybegin
        self._finalize = finalize
        self._composite = composite
        if types is None and composite is not None:
            raise TypeError("types must be provided for composite aggregators")
        if types is None:
            if monoid is not None:
                types = [monoid]
            else:
                types = [semiring, semiring2] + ([finalize] if finalize is not None else [])
        self._types_orig = types
        self._types = None
        self._typed = {}
        self._any_dtype = any_dtype

    @property
    def types(self):
        if self._types is None:
            init = None if self._initval_orig is None else self._initdtype
            self._types = _chain_types(self._types_orig, init)
        return self._types

    def __getitem__(self, dtype):
        dtype = lookup_dtype(dtype)
        if not self._any_dtype and dtype not in self.types:
            raise KeyError(f"{self.name} does not work with {dtype}")
        if dtype not in self._typed:
            self._typed[dtype] = TypedAggregator(self, dtype)
        return self._typed[dtype]

    def __contains__(self, dtype):
        dtype = lookup_dtype(dtype)
        return self._any_dtype or dtype in self.types

    def __repr__(self):
        return f"agg.ss.{self.name}" if self._custom is not None else f"agg.{self.name}"

    def __call__(self, val, *, rowwise=False, columnwise=False):
        """agg(v) / agg(A, rowwise=True) sugar for the reduce methods (reference agg.py:111-138)."""
        if getattr(val, "ndim", None) == 1:
            if rowwise or columnwise:
                raise ValueError("rowwise and columnwise arguments should not be used with Vector input")
            return val.reduce(self)
        if getattr(val, "ndim", None) == 2:
            if rowwise:
                if columnwise:
                    raise ValueError("rowwise and columnwise arguments cannot both be True")
                return val.reduce_rowwise(self)
            if columnwise:
                return val.reduce_columnwise(self)
            return val.reduce_scalar(self)
        raise TypeError(f"Bad type when calling {self!r}: {type(val)}")


class TypedAggregator:
    opclass = "Aggregator"

    def __init__(self, agg, dtype):
        self.name = agg.name
        self.parent = agg
        self.type = dtype
        if dtype in agg.types:
            self.return_type = agg.types[dtype]
        elif agg._any_dtype is True:
            self.return_type = dtype
        else:
            self.return_type = agg._any_dtype

    def __repr__(self):
        return f"agg.{self.name}[{self.type}]"

    __call__ = Aggregator.__call__


# ---------------------------------------------------------------- lowering
def _materialize(x):
    """A finalizer may return a collection or a (delayed / infix) expression."""
    return x if getattr(x, "_h", None) is not None and hasattr(x, "nvals") else x.new()


def _iso_vector(dtype, size, value):
    from .vector import Vector

    v = Vector(dtype, size, name="agg_init")
    v[:] = value  # one assign launch: iso-full bitmap vector
    return v


def _semiring_for(agg, dtype):
    return _op.get_typed_op(agg._semiring, dtype, agg._initdtype, kind="semiring")


def _finalize(agg, v):
    """Apply the finalizer to a Vector, returning a new Vector."""
    fin = _op.get_typed_op(agg._finalize, v.dtype, kind="unary")
    return v.apply(fin).new(fin.return_type)


def _rows(A, agg, dtype, opts):
    """Vector of per-row aggregates of A (A may be a TransposedMatrix)."""
    if agg._custom is not None:
        return agg._custom(agg, "rows", A, opts)
    if agg._monoid is not None:
        mon = _op.get_typed_op(agg._monoid, dtype, kind="monoid")
        return A.reduce_rowwise(mon).new(**opts)
    if agg._composite is not None:
        parts = [_rows(A, sub, dtype, opts) for sub in agg._composite]
        return _materialize(agg._finalize(*parts, opts))
    if agg._applybegin is not None:
        A = A.apply(agg._applybegin).new()
    sr = _semiring_for(agg, A.dtype)
    init = _iso_vector(agg._initdtype, A.ncols, agg._initval)
    if agg._switch:
        w = init.vxm(A.T, sr).new(**opts)
    else:
        w = A.mxv(init, sr).new(**opts)
    if agg._finalize is not None:
        w = _finalize(agg, w)
    return w


def _to_scalar(w, agg, opts):
    """Scalar aggregate of a Vector (reference agg.py:229-248), as a 1-element Vector."""
    from .matrix import Matrix

    if agg._custom is not None:
        return agg._custom(agg, "vector", w, opts)
    if agg._monoid is not None:
        mon = _op.get_typed_op(agg._monoid, w.dtype, kind="monoid")
        from .vector import Vector

        out = Vector(mon.return_type, 1)
        s = w.reduce(mon).new()
        if s.value is not None:
            out[0] = s.value
        return out
    if agg._composite is not None:
        parts = [_to_scalar(w, sub, opts) for sub in agg._composite]
        return _materialize(agg._finalize(*parts, opts))
    if agg._applybegin is not None:
        w = w.apply(agg._applybegin).new()
    sr = _semiring_for(agg, w.dtype)
    init = Matrix(agg._initdtype, w.size, 1, name="agg_init")
    init[:, :] = agg._initval
    if agg._switch:
        step1 = init.T.mxv(w, sr).new(**opts)
    else:
        step1 = w.vxm(init, sr).new(**opts)
    if agg._finalize is not None:
        step1 = _finalize(agg, step1)
    return step1


def _matrix_to_scalar(A, agg, opts):
    """Matrix -> Vector -> Scalar in two SpMVs (reference agg.py:249-276)."""
    from .vector import Vector

    if agg._custom is not None:
        return agg._custom(agg, "matrix", A, opts)
    if agg._monoid is not None:
        mon = _op.get_typed_op(agg._monoid, A.dtype, kind="monoid")
        out = Vector(mon.return_type, 1)
        s = A.reduce_scalar(mon).new()
        if s.value is not None:
            out[0] = s.value
        return out
    if agg._composite is not None:
        parts = [_matrix_to_scalar(A, sub, opts) for sub in agg._composite]
        return _materialize(agg._finalize(*parts, opts))
    if agg._applybegin is not None:
        A = A.apply(agg._applybegin).new()
    sr = _semiring_for(agg, A.dtype)
    init1 = _iso_vector(agg._initdtype, A.ncols, agg._initval)
    if agg._switch:
        step1 = init1.vxm(A.T, sr).new(**opts)
    else:
        step1 = A.mxv(init1, sr).new(**opts)
    sr2 = _op.get_typed_op(agg._semiring2, step1.dtype, kind="semiring")
    from .matrix import Matrix

    init2 = Matrix(agg._initdtype, A.nrows, 1, name="agg_init2")
    init2[:, :] = agg._initval
    step2 = step1.vxm(init2, sr2).new(**opts)
    if agg._finalize is not None:
        step2 = _finalize(agg, step2)
    return step2


# ---------------------------------------------------------------- positional aggregators
def _false_vector(n):
    from .dtypes import BOOL

    return _iso_vector(BOOL, n, False)


def _false_column(n):
    """n x 1 iso-False matrix (the reference's "O(1) dense column vector", agg.py:520)."""
    from .dtypes import BOOL
    from .matrix import Matrix

    m = Matrix(BOOL, n, 1, name="agg_init")
    m[:, :] = False
    return m


def _one_vector(dtype, value):
    from .vector import Vector

    out = Vector(dtype, 1)
    if value is not None:
        out[0] = value
    return out


def _diag_of(w, n):
    """diag(w) as an n x n Matrix (reference uses Vector.diag(), agg.py:494)."""
    from .matrix import Matrix

    idx, vals = w.to_coo()
    return Matrix.from_coo(idx, idx, vals, dtype=w.dtype, nrows=n, ncols=n)


def matrix_scalar_forbidden(agg):
    """Name of the (sub-)aggregator of `agg` that has no Matrix.reduce_scalar form, or None
    (reference agg.py:564-565, 664-665: argmin/argmax/first_index/last_index)."""
    if getattr(agg, "_no_matrix_scalar", False):
        return agg.name
    for sub in agg._composite or ():
        bad = matrix_scalar_forbidden(sub)
        if bad:
            return bad
    return None


def _argminmax(agg, kind, x, opts, *, monoid):
    """argmin/argmax (reference agg.py:478-566): the row extremum, any_eq against it through a
    diagonal, the true entries kept (value mask), then the least column index by min_firstj."""
    from .dtypes import INT64

    S = _op.semiring
    if kind == "rows":
        mon = _op.get_typed_op(monoid, x.dtype, kind="monoid")
        step1 = x.reduce_rowwise(mon).new(**opts)
        D = _diag_of(step1, x.nrows)
        masked = D.mxm(x, S.any_eq).new(**opts)
        masked(mask=masked.V, replace=True, **opts) << masked
        return masked.mxv(_false_vector(x.ncols), S.min_firstj).new(**opts)
    if kind == "vector":
        mon = _op.get_typed_op(monoid, x.dtype, kind="monoid")
        s = x.reduce(mon).new()
        if s.value is None:
            return _one_vector(INT64, None)
        masked = x.apply(_op.binary.eq, right=s.value).new(**opts)
        masked(mask=masked.V, replace=True, **opts) << masked
        return masked.vxm(_false_column(x.size), S.min_secondi).new(**opts)
    raise ValueError(f"Aggregator {agg.name} may not be used with Matrix.reduce_scalar.")


def _first_last(agg, kind, x, opts, *, semiring_):
    """first/last (reference agg.py:582-628): the position of each row's first (last) entry by
    min_secondi (max_secondi), then its value through a masked any_first product with the
    permutation-like matrix P[j_i, i] (the diagonal keeps only row i's pick)."""
    from .dtypes import BOOL
    from .matrix import Matrix

    S = _op.semiring
    if kind == "rows":
        pos = x.mxv(_false_vector(x.ncols), semiring_).new(**opts)
        I, J = pos.to_coo()
        P = Matrix.from_coo(J, I, True, dtype=BOOL, nrows=x.ncols, ncols=x.nrows)
        D = Matrix.from_coo(I, I, True, dtype=BOOL, nrows=x.nrows, ncols=x.nrows)
        C = Matrix(x.dtype, x.nrows, x.nrows, name="agg_pick")
        C(mask=D.S, **opts) << x.mxm(P, S.any_first)
        return C.reduce_rowwise(_op.monoid.any).new(**opts)
    if kind == "vector":
        pos = x.vxm(_false_column(x.size), semiring_).new(**opts)
        i = pos[0].value if pos.nvals else None
        return _one_vector(x.dtype, None if i is None else x[int(i)].value)
    # Matrix.reduce_scalar: the first (last) row holding entries, then its first (last) column
    step1 = x.mxm(_false_column(x.ncols), semiring_).new(**opts)
    step2 = step1.T.mxv(_false_vector(x.nrows), semiring_).new(**opts)
    i = step2[0].value if step2.nvals else None
    if i is None:
        return _one_vector(x.dtype, None)
    j = step1[int(i), 0].value
    M, (r, c) = (x._matrix, (int(j), int(i))) if hasattr(x, "_matrix") else (x, (int(i), int(j)))
    return _one_vector(x.dtype, M[r, c].value)


def _first_last_index(agg, kind, x, opts, *, semiring_):
    """first_index/last_index (reference agg.py:645-667): min_secondi / max_secondi against an
    iso-False vector gives each row's first / last column index directly."""
    if kind == "rows":
        return x.mxv(_false_vector(x.ncols), semiring_).new(**opts)
    if kind == "vector":
        return x.vxm(_false_column(x.size), semiring_).new(**opts)
    raise ValueError(f"Aggregator {agg.name} may not be used with Matrix.reduce_scalar.")


def reduce_rowwise_recipe(updater, A, typed, columnwise):
    src = A.T if columnwise else A
    agg = typed.parent
    if agg._monoid is not None:
        mon = _op.get_typed_op(agg._monoid, typed.type, kind="monoid")
        updater << src.reduce_rowwise(mon)
        return
    w = _rows(src, agg, typed.type, {})
    updater << w  # (masked / accumulated) assign of the finished vector


def reduce_scalar_recipe(updater, x, typed):
    agg = typed.parent
    w = _to_scalar(x, agg, {}) if x.ndim == 1 else _matrix_to_scalar(x, agg, {})
    val = w[0].value if w.nvals else None
    if val is None:
        updater.parent.clear()
        return
    updater << val


# ---------------------------------------------------------------- composite finalizers
def _truediv(x, c):
    """x / c elementwise in floating point (binary.truediv, reference agg.py:286-287)."""
    dt = FP64 if x.dtype.name not in ("FP32",) else x.dtype
    xf = x if x.dtype == dt else x.dup(dt)
    cf = c if c.dtype == dt else c.dup(dt)
    return xf.ewise_mult(cf, _op.binary.div[dt]).new()


def _mean(c, x, opts):
    return _truediv(x, c)


def _ptp(mx, mn, opts):
    return mx.ewise_mult(mn, _op.binary.minus).new()


def _varp(c, x, x2, opts=None):
    left = _truediv(x2, c)
    right = _truediv(x, c)
    right = right.apply(_op.binary.pow, right=2).new()
    return left.ewise_mult(right, _op.binary.minus).new()


def _vars(c, x, x2, opts=None):
    xsq = x.apply(_op.binary.pow, right=2).new()
    right = _truediv(xsq, c)
    c1 = c.apply(_op.binary.minus, right=1).new()
    right = _truediv(right, c1)
    left = _truediv(x2, c1)
    return left.ewise_mult(right, _op.binary.minus).new()


def _stdp(c, x, x2, opts):
    return _varp(c, x, x2).apply(_op.unary.sqrt).new()


def _stds(c, x, x2, opts):
    return _vars(c, x, x2).apply(_op.unary.sqrt).new()


def _geometric_mean(c, x, opts):
    cf = c if c.dtype == FP64 else c.dup(FP64)
    inv = cf.apply(_op.unary.minv[FP64]).new()
    xf = x if x.dtype == FP64 else x.dup(FP64)
    return xf.ewise_mult(inv, _op.binary.pow[FP64]).new()


def _harmonic_mean(c, x, opts):
    return _truediv(c, x)


def _root_mean_square(c, x2, opts):
    return _truediv(x2, c).apply(_op.unary.sqrt).new()


class _TrueDivTypes:
    """Result types of binary.truediv (floats keep their type, the rest -> FP64)."""

    @property
    def types(self):
        from .dtypes import _ALL

        return {dt: (dt if dt.name == "FP32" else FP64) for dt in _ALL}


_truediv_types = _TrueDivTypes()


# ---------------------------------------------------------------- the agg namespace
class _AggNamespace:
    def __repr__(self):
        return "agg"


agg = _AggNamespace()
_s = _op.semiring
_m = _op.monoid
agg.sum = Aggregator("sum", monoid=_m.plus)
agg.prod = Aggregator("prod", monoid=_m.times)
agg.all = Aggregator("all", monoid=_m.land)
agg.any = Aggregator("any", monoid=_m.lor)
agg.min = Aggregator("min", monoid=_m.min)
agg.max = Aggregator("max", monoid=_m.max)
agg.any_value = Aggregator("any_value", monoid=_m.any, any_dtype=True)
agg.bitwise_all = Aggregator("bitwise_all", monoid=_m.band)
agg.bitwise_any = Aggregator("bitwise_any", monoid=_m.bor)
agg.count = Aggregator("count", semiring=_s.plus_pair, semiring2=_s.plus_first, any_dtype=INT64)
agg.count_nonzero = Aggregator("count_nonzero", semiring=_s.plus_isne, semiring2=_s.plus_first)
agg.count_zero = Aggregator("count_zero", semiring=_s.plus_iseq, semiring2=_s.plus_first)
agg.sum_of_squares = Aggregator("sum_of_squares", initval=2, semiring=_s.plus_pow, semiring2=_s.plus_first)
agg.sum_of_inverses = Aggregator("sum_of_inverses", initval=-1.0, semiring=_s.plus_pow,
                                 semiring2=_s.plus_first)
agg.exists = Aggregator("exists", semiring=_s.any_pair, semiring2=_s.any_pair, any_dtype=INT64)
agg.hypot = Aggregator("hypot", initval=2, semiring=_s.plus_pow, semiring2=_s.plus_first,
                       finalize=_op.unary.sqrt)
agg.logaddexp = Aggregator("logaddexp", initval=np.e, semiring=_s.plus_pow, switch=True,
                           semiring2=_s.plus_first, finalize=_op.unary.log)
agg.logaddexp2 = Aggregator("logaddexp2", initval=2, semiring=_s.plus_pow, switch=True,
                            semiring2=_s.plus_first, finalize=_op.unary.log2)
agg.L0norm = agg.count_nonzero
agg.L2norm = agg.hypot
agg.L1norm = Aggregator("L1norm", applybegin=_op.unary.abs, semiring=_s.plus_first, semiring2=_s.plus_first)
agg.Linfnorm = Aggregator("Linfnorm", applybegin=_op.unary.abs, semiring=_s.max_first,
                          semiring2=_s.max_first)

agg.mean = Aggregator("mean", composite=[agg.count, agg.sum], finalize=_mean, types=[_truediv_types])
agg.peak_to_peak = Aggregator("peak_to_peak", composite=[agg.max, agg.min], finalize=_ptp, types=[_m.min])
agg.ptp = agg.peak_to_peak
_C3 = [agg.count, agg.sum, agg.sum_of_squares]
agg.varp = Aggregator("varp", composite=_C3, finalize=_varp, types=[_truediv_types])
agg.vars = Aggregator("vars", composite=_C3, finalize=_vars, types=[_truediv_types])
agg.stdp = Aggregator("stdp", composite=_C3, finalize=_stdp, types=[_truediv_types])
agg.stds = Aggregator("stds", composite=_C3, finalize=_stds, types=[_truediv_types])
agg.geometric_mean = Aggregator("geometric_mean", composite=[agg.count, agg.prod], finalize=_geometric_mean,
                                types=[_truediv_types])
agg.harmonic_mean = Aggregator("harmonic_mean", composite=[agg.count, agg.sum_of_inverses],
                               finalize=_harmonic_mean, types=[_truediv_types])
agg.root_mean_square = Aggregator("root_mean_square", composite=[agg.count, agg.sum_of_squares],
                                  finalize=_root_mean_square, types=[_truediv_types])

# positional aggregators (reference agg.py:569-696; SuiteSparse-only there, so under agg.ss)
_sr = _op.semiring
_argmin = Aggregator("argmin", custom=partial(_argminmax, monoid=_m.min), types=[_sr.min_firsti])
_argmax = Aggregator("argmax", custom=partial(_argminmax, monoid=_m.max), types=[_sr.min_firsti])
_first = Aggregator("first", custom=partial(_first_last, semiring_=_sr.min_secondi), types=[_op.binary.first],
                    any_dtype=True)
_last = Aggregator("last", custom=partial(_first_last, semiring_=_sr.max_secondi), types=[_op.binary.second],
                   any_dtype=True)
_first_index = Aggregator("first_index", custom=partial(_first_last_index, semiring_=_sr.min_secondi),
                          types=[_sr.min_secondi], any_dtype=INT64)
_last_index = Aggregator("last_index", custom=partial(_first_last_index, semiring_=_sr.max_secondi),
                         types=[_sr.min_secondi], any_dtype=INT64)
for _a in (_argmin, _argmax, _first_index, _last_index):
    _a._no_matrix_scalar = True


class _AggSS:
    def __repr__(self):
        return "agg.ss"


agg.ss = _AggSS()
for _a in (_argmin, _argmax, _first, _last, _first_index, _last_index):
    setattr(agg.ss, _a.name, _a)
agg._deprecated = {a.name: a for a in (_argmin, _argmax, _first, _last, _first_index, _last_index)}

agg.Aggregator = Aggregator
agg.TypedAggregator = TypedAggregator
