"""The C API 2.0 GrB_Scalar-argument entry points (csrc/gb_scalar_args.cpp), called through the
ctypes C ABI exactly as python-graphblas calls them for non-C scalars:
GrB_{Vector,Matrix}_{extractElement,setElement,assign}_Scalar (reference core/vector.py:1769,
1808, 1918, 1939; core/matrix.py:2837, 2902, 3279, 3305) and
GrB_{Vector,Matrix}_apply_BinaryOp{1st,2nd}_Scalar (core/vector.py:1406, 1449;
core/matrix.py:2392, 2435).  An empty GrB_Scalar means "no value": setElement deletes,
extractElement of a missing entry empties the scalar (GrB_SUCCESS), assign deletes the selected
part of the region (nothing under accum), apply is GrB_EMPTY_OBJECT.  Expectations are numpy
restatements of those rules on small seeded inputs (index/value work: exact)."""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

U64 = ctypes.c_uint64


@pytest.fixture(scope="module")
def gb():
    import graphblas_amd

    return graphblas_amd


def _scalar(lib, tname, value=None):
    s = ctypes.c_void_p()
    assert lib.GrB_Scalar_new(ctypes.byref(s), getattr(lib, f"GrB_{tname}")) == 0
    if value is not None:
        assert getattr(lib, f"GrB_Scalar_setElement_{tname}")(s, value) == 0
    return s


def _scalar_value(lib, s, tname, ct):
    nv = U64()
    assert lib.GrB_Scalar_nvals(ctypes.byref(nv), s) == 0
    if nv.value == 0:
        return None
    x = ct()
    assert getattr(lib, f"GrB_Scalar_extractElement_{tname}")(ctypes.byref(x), s) == 0
    return x.value


def _vdict(v):
    i, x = v.to_coo()
    return dict(zip(i.tolist(), x.tolist()))


def _mdict(A):
    r, c, x = A.to_coo()
    return {(a, b): y for a, b, y in zip(r.tolist(), c.tolist(), x.tolist())}


def _idx(lst):
    a = np.asarray(lst, np.uint64)
    return a, ctypes.c_void_p(a.ctypes.data), len(a)


def test_set_element_scalar(gb):
    lib = gb.lib
    w = gb.Vector.from_coo([1, 4], [1.5, 2.5], dtype="FP64", size=8)
    s = _scalar(lib, "INT64", 7)
    assert lib.GrB_Vector_setElement_Scalar(w._carg, s, 3) == 0  # cast INT64 -> FP64
    assert _vdict(w) == {1: 1.5, 3: 7.0, 4: 2.5}
    e = _scalar(lib, "INT64")
    assert lib.GrB_Vector_setElement_Scalar(w._carg, e, 4) == 0  # empty: deletes
    assert _vdict(w) == {1: 1.5, 3: 7.0}
    assert lib.GrB_Vector_setElement_Scalar(w._carg, e, 5) == 0  # deleting a missing entry is fine
    assert lib.GrB_Vector_setElement_Scalar(w._carg, s, 8) == lib.GrB_INVALID_INDEX
    A = gb.Matrix.from_coo([0, 2], [1, 3], [10, 20], dtype="INT32", nrows=3, ncols=4)
    f = _scalar(lib, "FP64", 3.75)
    assert lib.GrB_Matrix_setElement_Scalar(A._carg, f, 1, 1) == 0  # FP64 -> INT32 truncates
    assert _mdict(A) == {(0, 1): 10, (1, 1): 3, (2, 3): 20}
    assert lib.GrB_Matrix_setElement_Scalar(A._carg, e, 2, 3) == 0
    assert _mdict(A) == {(0, 1): 10, (1, 1): 3}
    for h in (s, e, f):
        lib.GrB_Scalar_free(ctypes.byref(h))


def test_extract_element_scalar(gb):
    lib = gb.lib
    v = gb.Vector.from_coo([2, 5], [2.5, -1.25], dtype="FP64", size=6)
    s = _scalar(lib, "FP64", 99.0)
    assert lib.GrB_Vector_extractElement_Scalar(s, v._carg, 5) == 0
    assert _scalar_value(lib, s, "FP64", ctypes.c_double) == -1.25
    # a missing entry: GrB_SUCCESS and an empty scalar (not GrB_NO_VALUE)
    assert lib.GrB_Vector_extractElement_Scalar(s, v._carg, 3) == 0
    assert _scalar_value(lib, s, "FP64", ctypes.c_double) is None
    i32 = _scalar(lib, "INT32")
    assert lib.GrB_Vector_extractElement_Scalar(i32, v._carg, 2) == 0  # cast to the scalar's type
    assert _scalar_value(lib, i32, "INT32", ctypes.c_int32) == 2
    assert lib.GrB_Vector_extractElement_Scalar(i32, v._carg, 6) == lib.GrB_INVALID_INDEX
    A = gb.Matrix.from_coo([0, 1], [2, 0], [True, False], dtype="BOOL", nrows=2, ncols=3)
    b = _scalar(lib, "INT64")
    assert lib.GrB_Matrix_extractElement_Scalar(b, A._carg, 0, 2) == 0
    assert _scalar_value(lib, b, "INT64", ctypes.c_int64) == 1
    assert lib.GrB_Matrix_extractElement_Scalar(b, A._carg, 1, 0) == 0  # a stored False is a value
    assert _scalar_value(lib, b, "INT64", ctypes.c_int64) == 0
    assert lib.GrB_Matrix_extractElement_Scalar(b, A._carg, 1, 1) == 0
    assert _scalar_value(lib, b, "INT64", ctypes.c_int64) is None
    for h in (s, i32, b):
        lib.GrB_Scalar_free(ctypes.byref(h))


def test_vector_assign_scalar(gb):
    lib = gb.lib
    n = 10
    base = {k: 100 + k for k in range(0, n, 2)}  # entries at the even positions
    mk = lambda: gb.Vector.from_coo(list(base), list(base.values()), dtype="INT64", size=n)
    I, Ip, ni = _idx([0, 1, 2, 3, 4, 5])
    m = gb.Vector.from_coo([1, 2, 3, 8], True, size=n)
    s = _scalar(lib, "INT32", -5)
    e = _scalar(lib, "INT32")
    # w<m.S>(I) = -5
    w = mk()
    assert lib.GrB_Vector_assign_Scalar(w._carg, m._carg, None, s, Ip, ni, lib.GrB_DESC_S) == 0
    exp = dict(base)
    exp.update({1: -5, 2: -5, 3: -5})
    assert _vdict(w) == exp
    # w<m.S>(I) = empty: the selected part of the region {1, 2, 3} is deleted (2 was present)
    w = mk()
    assert lib.GrB_Vector_assign_Scalar(w._carg, m._carg, None, e, Ip, ni, lib.GrB_DESC_S) == 0
    assert _vdict(w) == {k: x for k, x in base.items() if k != 2}
    # w(I) = empty with no mask: every entry of the region goes
    w = mk()
    assert lib.GrB_Vector_assign_Scalar(w._carg, None, None, e, Ip, ni, None) == 0
    assert _vdict(w) == {k: x for k, x in base.items() if k > 5}
    # with accum the empty scalar changes nothing
    w = mk()
    assert lib.GrB_Vector_assign_Scalar(w._carg, None, lib.GrB_PLUS_INT64, e, Ip, ni, None) == 0
    assert _vdict(w) == base
    # GrB_ALL, complemented structural mask, replace: outside the mask everything is deleted,
    # inside (positions not in m) the entries are deleted by the empty assign
    w = mk()
    assert lib.GrB_Vector_assign_Scalar(w._carg, m._carg, None, e, lib.GrB_ALL, n, lib.GrB_DESC_RSC) == 0
    assert _vdict(w) == {}
    # present scalar, GrB_ALL, complemented mask: every position outside m becomes -5
    w = mk()
    assert lib.GrB_Vector_assign_Scalar(w._carg, m._carg, None, s, lib.GrB_ALL, n, lib.GrB_DESC_SC) == 0
    exp = {k: -5 for k in range(n) if k not in (1, 2, 3, 8)}
    exp[2] = base[2]
    exp[8] = base[8]
    assert _vdict(w) == exp
    for h in (s, e):
        lib.GrB_Scalar_free(ctypes.byref(h))


def test_matrix_assign_scalar(gb):
    lib = gb.lib
    rng = np.random.default_rng(5)
    nr, nc = 7, 9
    have = rng.random((nr, nc)) < 0.5
    vals = rng.integers(1, 50, (nr, nc))
    r, c = np.nonzero(have)
    mk = lambda: gb.Matrix.from_coo(r, c, vals[r, c], dtype="INT64", nrows=nr, ncols=nc)
    mhave = rng.random((nr, nc)) < 0.5
    mr, mc = np.nonzero(mhave)
    M = gb.Matrix.from_coo(mr, mc, True, nrows=nr, ncols=nc)
    Il, Jl = [1, 3, 4, 6], [0, 2, 5, 7, 8]
    I, Ip, ni = _idx(Il)
    J, Jp, nj = _idx(Jl)
    region = np.zeros((nr, nc), bool)
    region[np.ix_(Il, Jl)] = True
    s = _scalar(lib, "INT64", 77)
    e = _scalar(lib, "INT64")

    def as_dict(h, v):
        rr, cc = np.nonzero(h)
        return {(a, b): int(v[a, b]) for a, b in zip(rr.tolist(), cc.tolist())}

    # C<M.S>(I, J) = 77
    C = mk()
    assert lib.GrB_Matrix_assign_Scalar(C._carg, M._carg, None, s, Ip, ni, Jp, nj, lib.GrB_DESC_S) == 0
    sel = region & mhave
    hv, vv = have | sel, np.where(sel, 77, vals)
    assert _mdict(C) == as_dict(hv, vv)
    # C<M.S>(I, J) = empty: the selected part of the region is deleted
    C = mk()
    assert lib.GrB_Matrix_assign_Scalar(C._carg, M._carg, None, e, Ip, ni, Jp, nj, lib.GrB_DESC_S) == 0
    assert _mdict(C) == as_dict(have & ~sel, vals)
    # C<!M.S, replace>(I, J) = empty: region & !M deleted, and everything under M deleted (replace)
    C = mk()
    assert lib.GrB_Matrix_assign_Scalar(C._carg, M._carg, None, e, Ip, ni, Jp, nj, lib.GrB_DESC_RSC) == 0
    assert _mdict(C) == as_dict(have & ~(region & ~mhave) & ~mhave, vals)
    # accum with an empty scalar: unchanged
    C = mk()
    assert lib.GrB_Matrix_assign_Scalar(C._carg, None, lib.GrB_PLUS_INT64, e, Ip, ni, Jp, nj, None) == 0
    assert _mdict(C) == as_dict(have, vals)
    # GrB_ALL, no mask, empty: C is emptied
    C = mk()
    assert lib.GrB_Matrix_assign_Scalar(C._carg, None, None, e, lib.GrB_ALL, nr, lib.GrB_ALL, nc, None) == 0
    assert _mdict(C) == {}
    for h in (s, e):
        lib.GrB_Scalar_free(ctypes.byref(h))


def test_apply_binaryop_scalar(gb):
    lib = gb.lib
    u = gb.Vector.from_coo([0, 3, 4], [4, 9, -2], dtype="INT64", size=6)
    w = gb.Vector(gb.INT64, 6)
    s = _scalar(lib, "INT64", 10)
    assert lib.GrB_Vector_apply_BinaryOp1st_Scalar(w._carg, None, None, lib.GrB_MINUS_INT64, s, u._carg,
                                                   None) == 0
    assert _vdict(w) == {0: 6, 3: 1, 4: 12}  # 10 - u
    assert lib.GrB_Vector_apply_BinaryOp2nd_Scalar(w._carg, None, None, lib.GrB_MINUS_INT64, u._carg, s,
                                                   None) == 0
    assert _vdict(w) == {0: -6, 3: -1, 4: -12}  # u - 10
    A = gb.Matrix.from_coo([0, 1], [1, 2], [2.0, 8.0], dtype="FP64", nrows=2, ncols=3)
    C = gb.Matrix(gb.FP64, 2, 3)
    f = _scalar(lib, "FP64", 4.0)
    assert lib.GrB_Matrix_apply_BinaryOp1st_Scalar(C._carg, None, None, lib.GrB_DIV_FP64, f, A._carg, None) == 0
    assert _mdict(C) == {(0, 1): 2.0, (1, 2): 0.5}
    assert lib.GrB_Matrix_apply_BinaryOp2nd_Scalar(C._carg, None, None, lib.GrB_DIV_FP64, A._carg, f, None) == 0
    assert _mdict(C) == {(0, 1): 0.5, (1, 2): 2.0}
    # an empty bound scalar is GrB_EMPTY_OBJECT, reported on the output
    e = _scalar(lib, "INT64")
    rc = lib.GrB_Vector_apply_BinaryOp2nd_Scalar(w._carg, None, None, lib.GrB_MINUS_INT64, u._carg, e, None)
    assert rc == lib.GrB_EMPTY_OBJECT
    msg = ctypes.c_char_p()
    assert lib.GrB_Vector_error(ctypes.byref(msg), w._carg) == 0
    assert b"no value" in msg.value
    for h in (s, f, e):
        lib.GrB_Scalar_free(ctypes.byref(h))


@pytest.mark.parametrize("src,dst", [("INT8", "INT64"), ("INT16", "INT32"), ("INT32", "INT64"), ("INT8", "UINT64"),
                                     ("INT64", "INT8"), ("UINT32", "INT64"), ("INT32", "UINT16")])
def test_integer_casts_follow_c(gb, src, dst):
    """C's integer conversions (SuiteSparse GB_cast for integer types): widening sign-extends a
    signed source, narrowing keeps the value modulo 2^bits -- numpy's astype gives the same --
    through a typed setElement, a GrB_Scalar setElement, an assign of a whole vector, and apply"""
    lib = gb.lib
    vals = np.array([-5, -1, 0, 7, -128, 127], dtype=np.int64)
    sv = vals.astype(getattr(np, src.lower()))
    exp = sv.astype(getattr(np, dst.lower()))
    n = len(vals)
    ct = {"INT8": ctypes.c_int8, "INT16": ctypes.c_int16, "INT32": ctypes.c_int32, "INT64": ctypes.c_int64,
          "UINT32": ctypes.c_uint32}[src]
    w = gb.Vector(getattr(gb, dst), n)
    for i, x in enumerate(sv.tolist()):
        assert getattr(lib, f"GrB_Vector_setElement_{src}")(w._carg, ct(x), i) == 0
    i, got = w.to_coo()
    assert np.array_equal(got, exp)
    w2 = gb.Vector(getattr(gb, dst), n)
    for k, x in enumerate(sv.tolist()):
        s = _scalar(lib, src, x)
        assert lib.GrB_Vector_setElement_Scalar(w2._carg, s, k) == 0
        lib.GrB_Scalar_free(ctypes.byref(s))
    assert np.array_equal(w2.to_coo()[1], exp)
    u = gb.Vector.from_coo(np.arange(n), sv, dtype=src, size=n)
    w3 = gb.Vector(getattr(gb, dst), n)
    assert lib.GrB_Vector_assign(w3._carg, None, None, u._carg, lib.GrB_ALL, n, None) == 0
    assert np.array_equal(w3.to_coo()[1], exp)
    w4 = gb.Vector(getattr(gb, dst), n)
    assert lib.GrB_Vector_apply(w4._carg, None, None, getattr(lib, f"GrB_IDENTITY_{src}"), u._carg, None) == 0
    assert np.array_equal(w4.to_coo()[1], exp)
