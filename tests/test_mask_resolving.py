"""Mask algebra and output-binding resolution, restated from the reference's
graphblas/tests/test_mask.py:9-126 and graphblas/tests/test_resolving.py, run through
the MI355X front end (every mask combination is a masked assign on the device).

Expected values come from tests/golden/mask_golden.json (tests/golden/make_mask_golden.py:
the tests' own assign recipes restated as set algebra over the two vectors the reference
builds) and tests/golden/reference_golden.json["cases"]["test_resolving"] (the literal
from_coo data of test_resolving.py, tests/golden/make_golden.py)."""
import itertools
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
MASKG = json.load(open(os.path.join(HERE, "golden", "mask_golden.json")))


@pytest.fixture(scope="module")
def gb():
    import graphblas_amd

    return graphblas_amd


def _vectors(gb, mask_dtype, as_matrix):
    out = []
    for name in ("v1", "v2"):
        v = gb.Vector(mask_dtype, size=MASKG["size"])
        for start, stop, step, value in MASKG["vectors"][name]["assigns"]:
            v[slice(start, stop, step)] = value  # index-list GrB_Vector_assign_<T>
        out.append(v._as_matrix() if as_matrix else v)
    return out


def _masks(v1, v2):
    return [v1.S, v1.V, ~v1.S, ~v1.V, v2.S, v2.V, ~v2.S, ~v2.V]


def _check(gb, x, expected_idx, dtype, as_matrix):
    dt = gb.BOOL if dtype is None else gb.lookup_dtype(dtype)
    assert x.dtype == dt
    if as_matrix:
        assert isinstance(x, gb.Matrix) and x.shape == (MASKG["size"], 1)
        r, c, v = x.to_coo()
        assert np.all(c == 0)
        idx = r
    else:
        assert isinstance(x, gb.Vector) and x.size == MASKG["size"]
        idx, v = x.to_coo()
    assert sorted(idx.tolist()) == expected_idx
    assert np.all(v == 1)  # True, cast to the result dtype


@pytest.mark.parametrize("as_matrix", [False, True])
@pytest.mark.parametrize("mask_dtype", ["BOOL", "INT64"])
def test_mask_new(gb, as_matrix, mask_dtype):
    """test_mask.py:9-56"""
    cases = MASKG["cases"][mask_dtype]
    v1, v2 = _vectors(gb, mask_dtype, as_matrix)
    masks = _masks(v1, v2)
    names = MASKG["masks"]
    for dtype in MASKG["result_dtypes"]:
        for (n1, m1), (n2, m2) in itertools.product(zip(names, masks), repeat=2):
            exp = cases["pairs"][f"{n1}|{n2}"]
            r = m1.new(dtype, mask=m2, name="howdy")
            assert r.name == "howdy"
            _check(gb, r, exp["new"], dtype, as_matrix)
            r = m1.new(dtype, mask=m2, complement=True, name="howdy")
            _check(gb, r, exp["new_complement"], dtype, as_matrix)
        for n, m in zip(names, masks):
            _check(gb, m.new(dtype, name="howdy"), cases["single"][n]["new"], dtype, as_matrix)
            _check(gb, m.new(dtype, complement=True), cases["single"][n]["new_complement"], dtype, as_matrix)
    m = masks[-1]
    with pytest.raises(TypeError, match="Invalid mask"):
        m.new(mask=object())
    if mask_dtype == "BOOL":
        m.new(mask=v1)  # a bool collection is taken as its value mask
    else:
        with pytest.raises(TypeError, match="Mask must be"):
            m.new(mask=v1)


@pytest.mark.parametrize("op", ["or", "and"])
@pytest.mark.parametrize("as_matrix", [False, True])
@pytest.mark.parametrize("mask_dtype", ["BOOL", "INT64"])
def test_mask_or_and(gb, op, as_matrix, mask_dtype):
    """test_mask.py:59-126"""
    from graphblas_amd.base import Mask

    cases = MASKG["cases"][mask_dtype]
    v1, v2 = _vectors(gb, mask_dtype, as_matrix)
    masks = _masks(v1, v2)
    names = MASKG["masks"]
    for (n1, m1), (n2, m2) in itertools.product(zip(names, masks), repeat=2):
        combined = (m1 | m2) if op == "or" else (m1 & m2)
        assert isinstance(combined, Mask)
        _check(gb, combined.new(), cases["pairs"][f"{n1}|{n2}"][op], None, as_matrix)
    m1 = masks[0]
    f = (lambda a, b: a | b) if op == "or" else (lambda a, b: a & b)
    with pytest.raises(TypeError, match="Invalid mask"):
        f(m1, object())
    with pytest.raises(TypeError, match="Invalid mask"):
        f(object(), m1)
    if mask_dtype == "BOOL":
        assert isinstance(f(m1, v1), Mask)
        assert isinstance(f(v1, m1), Mask)
    else:
        with pytest.raises(TypeError, match="Mask must be"):
            f(m1, v1)
        with pytest.raises(TypeError, match="Mask must be"):
            f(v1, m1)


# ------------------------------------------------------------------ test_resolving.py
@pytest.fixture(scope="module")
def res(golden):
    return golden["cases"]["test_resolving"]["cases"]


def _dtype(gb, d):
    if d is None:
        return None
    d = d.replace("dtypes.", "")
    return {"float": float, "int": int, "bool": bool}.get(d, d)


def _mk(gb, d):
    if d["kind"] == "Vector":
        return gb.Vector.from_coo(d["indices"], d["values"], dtype=_dtype(gb, d["dtype"]), size=d.get("size"))
    return gb.Matrix.from_coo(d["rows"], d["cols"], d["values"], dtype=_dtype(gb, d["dtype"]),
                              nrows=d.get("nrows"), ncols=d.get("ncols"))


def test_from_coo_dtype_resolving(gb, res):
    """test_resolving.py:13-21"""
    got = [_mk(gb, d).dtype for d in res["test_from_coo_dtype_resolving"]]
    assert got == [gb.INT32, gb.INT32, gb.UINT8, gb.FP64]


def test_from_coo_invalid_dtype(gb, res):
    """test_resolving.py:24-30"""
    A, expected = [_mk(gb, d) for d in res["test_from_coo_invalid_dtype"]]
    assert A.isequal(expected)
    with pytest.raises(ValueError, match="object dtype for values is not allowed"):
        gb.Matrix.from_coo([0, 1, 2], [2, 0, 1], [0, 2, object()])


def test_resolve_ops_using_common_dtype(gb, res):
    """test_resolving.py:33-40: PLUS runs in FP64 (unify(INT64, FP64)), the result is cast to FP32"""
    u, v, result = [_mk(gb, d) for d in res["test_resolve_ops_using_common_dtype"]]
    w = gb.Vector("FP32", u.size)
    w << u.ewise_mult(v, gb.binary.plus)
    assert w.isclose(result, check_dtype=True)


def test_order_of_updater_params_does_not_matter(gb, res):
    """test_resolving.py:43-71"""
    d = res["test_order_of_updater_params_does_not_matter"]
    u, mask, result = _mk(gb, d[0]), _mk(gb, d[1]), _mk(gb, d[2])
    accum = gb.binary.plus
    forms = [
        lambda v: v(mask.V, accum, replace=True),
        lambda v: v(accum, mask.V, replace=True),
        lambda v: v(accum, mask=mask.V, replace=True),
        lambda v: v(mask.V, accum=accum, replace=True),
        lambda v: v(replace=True, mask=mask.V, accum=accum),
        lambda v: v(gb.replace, mask=mask.V, accum=accum),
    ]
    for form, dv in zip(forms, d[3:]):
        v = _mk(gb, dv)
        form(v) << u.ewise_mult(u, gb.binary.times)
        assert v.isequal(result)


def test_updater_replace_no_mask(gb):
    """test_resolving.py:74-83"""
    u = gb.Vector.from_coo([0, 1, 2], [1, 2, 3])
    with pytest.raises(TypeError, match="'replace' argument may only be True if a mask is provided"):
        u(replace=True)
    with pytest.raises(TypeError, match="'replace' argument may only be True if a mask is provided"):
        u(gb.replace)
    assert repr(gb.replace) == "replace" and str(gb.replace) == "replace"  # :86-88


def test_updater_repeat_argument_types(gb):
    """test_resolving.py:91-102"""
    mask = gb.Vector.from_coo([0, 3], [True, True])
    accum = gb.binary.plus
    v = gb.Vector.from_coo([0, 1, 2, 3], [4, 3, 2, 1])
    for call in (lambda: v(mask.S, mask.S), lambda: v(mask.S, mask=mask.S), lambda: v(accum, accum),
                 lambda: v(accum, accum=accum)):
        with pytest.raises(TypeError, match="multiple"):
            call()


def test_updater_bad_types(gb):
    """test_resolving.py:105-117"""
    v = gb.Vector.from_coo([0, 1, 2, 3], [4, 3, 2, 1])
    M = gb.Matrix.from_coo([0, 1, 2], [2, 0, 1], [0, 2, 3], dtype="UINT8")
    with pytest.raises(TypeError, match="Invalid mask"):
        v(mask=object())
    with pytest.raises(TypeError, match="Invalid mask"):
        v[[1, 2]].new(mask=object())
    with pytest.raises(TypeError, match="Mask object must be type Vector"):
        v.ewise_mult(v).new(mask=M.S)
    with pytest.raises(TypeError, match="Invalid"):
        v(object())
    with pytest.raises(TypeError, match="Expected type: BinaryOp"):
        v(gb.unary.one)


def test_already_resolved_ops_allowed_in_updater(gb, res):
    """test_resolving.py:120-125"""
    u, result = [_mk(gb, d) for d in res["test_already_resolved_ops_allowed_in_updater"]]
    u(gb.binary.plus["INT64"]) << u.ewise_mult(u, gb.binary.times["INT64"])
    assert u.isequal(result)


def test_updater_returns_updater(gb, res):
    """test_resolving.py:128-136"""
    from graphblas_amd.base import Updater

    u, final = [_mk(gb, d) for d in res["test_updater_returns_updater"]]
    y = u(accum=gb.binary.times)
    assert isinstance(y, Updater)
    z = y << u.apply(gb.unary.ainv)
    assert z is None
    assert isinstance(y, Updater)
    assert u.isequal(final)


def test_py_indices_extract(gb, res):
    """test_resolving.py:194-280, the non-SuiteSparse branch: the extracted vectors"""
    v = gb.Vector.from_coo(np.arange(5), np.arange(5))
    ref = np.arange(5)
    for key in [slice(None), [0, 2], slice(0, 0), slice(2, 0), slice(None, None, -1), slice(4, -3, -1),
                slice(1, None, 2), slice(0, 2), slice(1, 5), slice(1, 3, 1), slice(0, 5, 1)]:
        w = v[key].new()
        exp = ref[key]
        assert w.size == len(exp)
        i, x = w.to_coo()
        assert i.tolist() == list(range(len(exp))) and x.tolist() == list(exp)
    assert v[3].new().value == 3
    (d,) = res["test_py_indices"]
    A = _mk(gb, d)
    dense = np.zeros((10, 10), np.int64)
    have = np.zeros((10, 10), bool)
    dense[d["rows"], d["cols"]] = d["values"]
    have[d["rows"], d["cols"]] = True
    B = A[1:6, 8:-8:-2].new()
    rows, cols = list(range(10))[1:6], list(range(10))[8:-8:-2]
    assert B.shape == (len(rows), len(cols))
    r, c, x = B.to_coo()
    sub_have = have[np.ix_(rows, cols)]
    er, ec = np.nonzero(sub_have)
    assert r.tolist() == er.tolist() and c.tolist() == ec.tolist()
    assert x.tolist() == dense[np.ix_(rows, cols)][sub_have].tolist()
