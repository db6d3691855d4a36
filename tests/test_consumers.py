"""In-library consumers of the semiring kernels: aggregator
lowering (reference core/operator/agg.py:207-279), apply, Matrix.reduce_rowwise /
reduce_columnwise, and the prefix scan (reference core/ss/prefix_scan.py).

Expected values are the reference's own: graphblas/tests/test_matrix.py
test_reduce_row :1355, test_reduce_agg :1364, test_reduce_agg_empty :1612,
test_reduce_column :1648; graphblas/tests/test_vector.py test_reduce_agg :908,
test_reduce_agg_empty :1000; graphblas/tests/test_prefix_scan.py :11-80 (numpy
cumsum / cumprod as the expected output).  Larger seeded cases compare with
numpy on the same inputs (exact for integers; fp64 within 1e-12 relative).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gb():
    import graphblas_amd

    return graphblas_amd


@pytest.fixture
def A(gb, golden):
    g = golden["A"]
    return gb.Matrix.from_coo(g["rows"], g["cols"], g["values"])


@pytest.fixture
def v(gb, golden):
    g = golden["v"]
    return gb.Vector.from_coo(g["indices"], g["values"])


def V(gb, idx, vals, dtype=None):
    return gb.Vector.from_coo(idx, vals, dtype=dtype)


# ------------------------------------------------------------------ reduce_rowwise / columnwise
def test_reduce_row(gb, A):
    result = V(gb, range(7), [5, 12, 1, 6, 7, 1, 15])
    assert A.reduce_rowwise(gb.monoid.plus).new().isequal(result)
    assert A.reduce_rowwise(gb.binary.plus).new().isequal(result)


def test_reduce_column(gb, A):
    result = V(gb, range(7), [3, 2, 9, 10, 11, 8, 4])
    assert A.reduce_columnwise(gb.monoid.plus).new().isequal(result)
    assert A.reduce_columnwise(gb.binary.plus).new().isequal(result)
    assert A.T.reduce_rowwise(gb.monoid.plus).new().isequal(result)


def test_reduce_rowwise_masked_accum(gb, A):
    w = V(gb, [0, 6], [100, 100])
    m = V(gb, [0, 1, 6], [True, True, True])
    w(m.S, gb.binary.plus) << A.reduce_rowwise(gb.monoid.max)
    # row maxima: 0:3 1:8 6:7
    assert w.isequal(V(gb, [0, 1, 6], [103, 8, 107]))


# ------------------------------------------------------------------ aggregators
def test_reduce_agg(gb, A):
    agg = gb.agg
    result = V(gb, range(7), [5, 12, 1, 6, 7, 1, 15])
    assert A.reduce_rowwise(agg.sum).new().isequal(result)
    assert A.T.reduce_columnwise(agg.sum).new().isequal(result)

    counts = A.dup(dtype=bool).reduce_rowwise(gb.monoid.plus[int]).new()
    assert A.reduce_rowwise(agg.count).new().isequal(counts)
    assert A.T.reduce_columnwise(agg.count).new().isequal(counts)

    Asquared = gb.monoid.times(A & A).new()
    squared = Asquared.reduce_rowwise(gb.monoid.plus).new()
    expected = gb.unary.sqrt[float](squared).new()
    w5 = A.reduce_rowwise(agg.hypot).new()
    assert w5.isclose(expected)
    w7 = gb.Vector(w5.dtype, size=w5.size)
    w7 << A.reduce_rowwise(agg.hypot)
    assert w7.isclose(expected)

    result = V(gb, range(7), [3, 2, 9, 10, 11, 8, 4])
    assert A.reduce_columnwise(agg.sum).new().isequal(result)
    assert A.T.reduce_rowwise(agg.sum).new().isequal(result)
    counts = A.dup(dtype=bool).reduce_columnwise(gb.monoid.plus[int]).new()
    assert A.reduce_columnwise(agg.count).new().isequal(counts)
    assert A.T.reduce_rowwise(agg.count).new().isequal(counts)

    assert A.reduce_rowwise(agg.mean).new().isequal(V(gb, range(7), [2.5, 6, 1, 3, 7, 1, 5]))
    assert A.reduce_columnwise(agg.mean).new().isequal(V(gb, range(7), [3, 2, 3, 5, 5.5, 4, 4]))
    ones = V(gb, range(7), [1] * 7)
    assert A.reduce_rowwise(agg.exists).new().isequal(ones)
    assert A.reduce_columnwise(agg.exists).new().isequal(ones)

    assert A.reduce_scalar(agg.sum).new() == 47
    assert A.reduce_scalar(agg.prod).new() == 1270080
    assert A.reduce_scalar(agg.count).new() == 12
    assert A.reduce_scalar(agg.count_nonzero).new() == 12
    assert A.reduce_scalar(agg.count_zero).new() == 0
    assert A.reduce_scalar(agg.sum_of_squares).new() == 245
    assert np.isclose(A.reduce_scalar(agg.hypot).new().value, 245**0.5)
    assert np.isclose(A.reduce_scalar(agg.logaddexp).new().value, 8.6071076)
    assert np.isclose(A.reduce_scalar(agg.logaddexp2).new().value, 9.2288187)
    assert np.isclose(A.reduce_scalar(agg.mean).new().value, 47 / 12)
    assert A.reduce_scalar(agg.exists).new() == 1

    silly = agg.Aggregator("silly", composite=[agg.varp, agg.stdp],
                           finalize=lambda x, y, opts: gb.binary.times(x & y), types=[agg.varp])
    v1 = A.reduce_rowwise(agg.varp).new()
    v2 = A.reduce_rowwise(agg.stdp).new()
    assert v1.isclose(gb.binary.times(v2 & v2).new())
    v3 = A.reduce_rowwise(silly).new()
    assert v3.isclose(gb.binary.times(v1 & v2).new())
    s1 = A.reduce_scalar(agg.varp).new()
    s2 = A.reduce_scalar(agg.stdp).new()
    assert np.isclose(s1.value, s2.value * s2.value)
    s3 = A.reduce_scalar(silly).new()
    assert np.isclose(s3.value, s1.value * s2.value)

    B = gb.Matrix(int, nrows=4, ncols=5)
    assert B.reduce_scalar(agg.sum, allow_empty=True).new().is_empty
    assert B.reduce_scalar(agg.sum, allow_empty=False).new() == 0
    assert B.reduce_scalar(agg.vars, allow_empty=True).new().is_empty
    with pytest.raises(ValueError, match="allow_empty=False not allowed when using Aggregators"):
        B.reduce_scalar(agg.vars, allow_empty=False)


def test_reduce_agg_vector(gb, v):
    agg = gb.agg
    s = v.reduce(agg.sum).new()
    assert s.dtype == "INT64" and s == 4
    s = v.reduce(agg.sum[float]).new()
    assert s.dtype == "FP64" and s == 4
    assert v.reduce(agg.prod).new() == 0
    assert v.reduce(agg.count).new() == 4
    assert v.reduce(agg.count_nonzero).new() == 3
    assert v.reduce(agg.count_zero).new() == 1
    assert v.reduce(agg.sum_of_squares).new() == 6
    assert np.isclose(v.reduce(agg.hypot).new().value, 6**0.5)
    assert np.isclose(v.reduce(agg.logaddexp).new().value, np.log(1 + 2 * np.e + np.e**2))
    assert np.isclose(v.reduce(agg.logaddexp2).new().value, np.log2(9))
    assert v.reduce(agg.mean).new() == 1
    assert v.reduce(agg.peak_to_peak).new() == 2
    assert np.isclose(v.reduce(agg.varp).new().value, 0.5)
    assert np.isclose(v.reduce(agg.vars).new().value, 2 / 3)
    assert np.isclose(v.reduce(agg.stdp).new().value, 0.5**0.5)
    assert np.isclose(v.reduce(agg.stds).new().value, (2 / 3) ** 0.5)
    assert v.reduce(agg.L0norm).new() == 3
    assert v.reduce(agg.L1norm).new() == 4
    assert np.isclose(v.reduce(agg.L2norm).new().value, 6**0.5)
    assert v.reduce(agg.Linfnorm).new() == 2
    assert v.reduce(agg.exists).new() == 1
    w = gb.binary.plus(v, 1).new()
    assert np.isclose(w.reduce(agg.geometric_mean).new().value, 12**0.25)
    assert np.isclose(w.reduce(agg.harmonic_mean).new().value, 12 / 7)
    silly = agg.Aggregator("silly", composite=[agg.varp, agg.stdp],
                           finalize=lambda x, y, opts: gb.binary.times(x & y), types=[agg.varp])
    assert np.isclose(v.reduce(silly).new().value, 0.5**1.5)
    assert gb.Vector(int, size=5).reduce(silly).new().is_empty
    empty = gb.Vector(int, size=3)
    assert empty.reduce(agg.sum, allow_empty=False).new() == 0
    assert empty.reduce(agg.mean, allow_empty=True).new().is_empty
    with pytest.raises(ValueError, match="allow_empty=False not allowed when using Aggregators"):
        empty.reduce(agg.mean, allow_empty=False)


def _aggregators(gb):
    return [(k, a) for k, a in vars(gb.agg).items() if isinstance(a, gb.agg.Aggregator)]


def test_reduce_agg_empty(gb):
    A = gb.Matrix("UINT8", nrows=3, ncols=4)
    for B in [A, A.T]:
        ve = gb.Vector(bool, size=B.nrows)
        we = gb.Vector(bool, size=B.ncols)
        for attr, aggr in _aggregators(gb):
            assert ve.isequal(B.reduce_rowwise(aggr).new()), attr
            assert we.isequal(B.reduce_columnwise(aggr).new()), attr
            assert B.reduce_scalar(aggr).new().value is None, attr
    v = gb.Vector("UINT8", size=3)
    for attr, aggr in _aggregators(gb):
        assert v.reduce(aggr).new().value is None, attr


def test_agg_rowwise_random_vs_numpy(gb):
    """count / sum / min / max / mean / sum_of_squares per row and column of a seeded
    sparse fp64 matrix, against numpy on the dense form."""
    rng = np.random.default_rng(11)
    n, m, nnz = 600, 450, 9000
    r = rng.integers(0, n, nnz)
    c = rng.integers(0, m, nnz)
    key = np.unique(r * m + c)
    r, c = key // m, key % m
    vals = rng.random(len(r)) * 4 - 1
    A = gb.Matrix.from_coo(r, c, vals, nrows=n, ncols=m)
    D = np.full((n, m), np.nan)
    D[r, c] = vals
    P = ~np.isnan(D)
    for axis, red in [(1, "reduce_rowwise"), (0, "reduce_columnwise")]:
        cnt = P.sum(axis)
        has = cnt > 0
        got = {}
        for name in ["count", "sum", "min", "max", "mean", "sum_of_squares", "hypot"]:
            w = getattr(A, red)(getattr(gb.agg, name)).new()
            idx, wv = w.to_coo()
            assert np.array_equal(idx.astype(np.int64), np.nonzero(has)[0]), name
            got[name] = wv
        with np.errstate(all="ignore"):
            ref = {"count": cnt[has], "sum": np.nansum(D, axis)[has], "min": np.nanmin(D, axis)[has],
                   "max": np.nanmax(D, axis)[has], "mean": (np.nansum(D, axis) / cnt)[has],
                   "sum_of_squares": np.nansum(D * D, axis)[has],
                   "hypot": np.sqrt(np.nansum(D * D, axis))[has]}
        for name, e in ref.items():
            assert np.allclose(got[name], e, rtol=1e-12, atol=1e-12), (red, name)
        assert np.array_equal(got["min"], ref["min"]) and np.array_equal(got["max"], ref["max"])


# ------------------------------------------------------------------ apply
def test_apply_unary_and_bound(gb, A, v):
    r, c, vals = A.to_coo()
    B = A.apply(gb.unary.ainv).new()
    assert np.array_equal(B.to_coo()[2], -vals)
    B = gb.unary.abs(B).new()
    assert B.isequal(A)
    C = A.apply(gb.binary.minus, right=1).new()
    assert np.array_equal(C.to_coo()[2], vals - 1)
    C = A.apply(gb.binary.minus, left=10).new()
    assert np.array_equal(C.to_coo()[2], 10 - vals)
    C = A.T.apply(gb.binary.times, right=2).new()
    rt, ct, vt = C.to_coo()
    o = np.lexsort((r, c))
    assert np.array_equal(rt, c[o]) and np.array_equal(ct, r[o]) and np.array_equal(vt, 2 * vals[o])
    s = v.apply(gb.unary.sqrt).new()
    assert s.dtype == "FP64"
    assert np.allclose(s.to_coo()[1], np.sqrt([1, 1, 2, 0]))
    g = v.apply(gb.binary.gt, right=0).new()
    assert g.dtype == "BOOL" and np.array_equal(g.to_coo()[1], [True, True, True, False])
    # masked + accumulated apply
    w = v.dup()
    w(gb.binary.plus, mask=v.S) << v.apply(gb.binary.pow, right=2)
    assert np.array_equal(w.to_coo()[1], [2, 2, 6, 0])
    # iso input stays iso, value mapped once
    iso = gb.Vector.from_coo([0, 5, 9], 3.0, size=10)
    e = iso.apply(gb.unary.exp).new()
    assert np.allclose(e.to_coo()[1], np.exp(3.0))


# ------------------------------------------------------------------ prefix scan
@pytest.mark.parametrize("method", ["scan_rowwise", "scan_columnwise"])
@pytest.mark.parametrize("length", list(range(34)))
@pytest.mark.parametrize("do_random", [False, True])
def test_scan_matrix(gb, method, length, do_random):
    if do_random:
        rng = np.random.default_rng(length)
        a = rng.integers(10, size=2 * length).reshape((2, length))
        mask = (a % 2).astype(bool)
        a[~mask] = 0
        rr, cc = np.nonzero(mask)
        M = gb.Matrix.from_coo(rr, cc, a[rr, cc], nrows=2, ncols=length, dtype="INT64")
        expected = a.cumsum(axis=1)
        expected[~mask] = 0
    else:
        a = np.arange(2 * length).reshape((2, length))
        rr, cc = np.nonzero(np.ones_like(a, bool))
        M = gb.Matrix.from_coo(rr, cc, a[rr, cc], nrows=2, ncols=length, dtype="INT64")
        expected = a.cumsum(axis=1)
    if method == "scan_rowwise":
        R = M.ss.scan()
    else:
        M = M.T.new()
        R = M.ss.scan(gb.binary.plus, order="col").T.new()
    got = np.zeros((2, length), np.int64)
    r, c, vals = R.to_coo()
    got[r.astype(np.int64), c.astype(np.int64)] = vals
    np.testing.assert_array_equal(got, expected)


@pytest.mark.parametrize("length", list(range(34)))
@pytest.mark.parametrize("do_random", [False, True])
def test_scan_vector(gb, length, do_random):
    if do_random:
        rng = np.random.default_rng(100 + length)
        a = rng.integers(10, size=length)
        mask = (a % 2).astype(bool)
        a[~mask] = 0
        idx = np.nonzero(mask)[0]
        vec = gb.Vector.from_coo(idx, a[idx], size=length, dtype="INT64")
        expected = a.cumsum()
        expected[~mask] = 0
    else:
        a = np.arange(length)
        vec = gb.Vector.from_coo(np.arange(length), a, size=length, dtype="INT64")
        expected = a.cumsum()
    r = vec.ss.scan()
    got = np.zeros(length, np.int64)
    i, vals = r.to_coo()
    got[i.astype(np.int64)] = vals
    np.testing.assert_array_equal(got, expected)


def test_cumprod(gb):
    v = gb.Vector.from_coo([1, 3, 4, 6], [2, 3, 4, 5])
    expected = gb.Vector.from_coo([1, 3, 4, 6], [2, 6, 24, 120])
    assert v.ss.scan(gb.monoid.times).isequal(expected)


def test_bad_scan(gb):
    v = gb.Vector.from_coo(range(10), range(10))
    with pytest.raises(TypeError, match="Bad type for argument `op`"):
        v.ss.scan(op=gb.binary.first)


def test_scan_matrix_random_vs_numpy(gb):
    """Row scans of a ragged seeded matrix (rows of 0..300 entries), plus and max."""
    rng = np.random.default_rng(5)
    n, m = 200, 1000
    deg = rng.integers(0, 300, n)
    rows = np.repeat(np.arange(n), deg)
    cols = np.concatenate([np.sort(rng.choice(m, d, replace=False)) for d in deg])
    vals = rng.integers(-50, 50, len(rows))
    A = gb.Matrix.from_coo(rows, cols, vals, nrows=n, ncols=m, dtype="INT64")
    starts = np.concatenate([[0], np.cumsum(deg)])
    for mon, fn in [(gb.monoid.plus, np.cumsum), (gb.monoid.max, np.maximum.accumulate)]:
        R = A.ss.scan(mon)
        r, c, rv = R.to_coo()
        assert np.array_equal(r.astype(np.int64), rows) and np.array_equal(c.astype(np.int64), cols)
        exp = np.concatenate([fn(vals[starts[i]:starts[i + 1]]) for i in range(n) if deg[i]])
        assert np.array_equal(rv, exp)


# ------------------------------------------------------------------ positional aggregators
# Expected values: reference graphblas/tests/test_matrix.py test_reduce_agg_argminmax :1458,
# test_reduce_agg_firstlast :1510, test_reduce_agg_firstlast_index :1566;
# graphblas/tests/test_vector.py :952-997.
def test_reduce_agg_argminmax_matrix(gb, A):
    agg = gb.agg
    for op, exp in [(agg.ss.argmin, [1, 6, 5, 0, 5, 2, 4]), (agg.ss.argmax, [3, 4, 5, 0, 5, 2, 3])]:
        assert A.reduce_rowwise(op).new().isequal(V(gb, range(7), exp))
        assert A.T.reduce_columnwise(op).new().isequal(V(gb, range(7), exp))
    for op, exp in [(agg.ss.argmin, [3, 0, 5, 0, 6, 2, 1]), (agg.ss.argmax, [3, 0, 6, 6, 1, 4, 1])]:
        assert A.reduce_columnwise(op).new().isequal(V(gb, range(7), exp))
        assert A.T.reduce_rowwise(op).new().isequal(V(gb, range(7), exp))
    with pytest.raises(ValueError, match="Aggregator argmin may not be used with Matrix.reduce_scalar"):
        A.reduce_scalar(agg.ss.argmin)
    silly = agg.Aggregator("silly", composite=[agg.ss.argmin, agg.ss.argmax],
                           finalize=lambda x, y, opts: gb.binary.plus(x & y), types=[agg.ss.argmin])
    for method in ("reduce_rowwise", "reduce_columnwise"):
        v1 = getattr(A, method)(agg.ss.argmin).new()
        v2 = getattr(A, method)(agg.ss.argmax).new()
        v3 = getattr(A, method)(silly).new()
        assert v3.isequal(gb.binary.plus(v1 & v2).new())
    with pytest.raises(ValueError, match="Aggregator"):
        A.reduce_scalar(silly).new()


def test_reduce_agg_firstlast_matrix(gb, A):
    agg = gb.agg
    cases = [("reduce_rowwise", agg.ss.first, [2, 8, 1, 3, 7, 1, 5]),
             ("reduce_rowwise", agg.ss.last, [3, 4, 1, 3, 7, 1, 3]),
             ("reduce_columnwise", agg.ss.first, [3, 2, 3, 3, 8, 1, 4]),
             ("reduce_columnwise", agg.ss.last, [3, 2, 5, 7, 3, 7, 4])]
    other = {"reduce_rowwise": "reduce_columnwise", "reduce_columnwise": "reduce_rowwise"}
    for method, op, exp in cases:
        assert getattr(A, method)(op).new().isequal(V(gb, range(7), exp))
        assert getattr(A.T, other[method])(op).new().isequal(V(gb, range(7), exp))
    assert A.reduce_scalar(agg.ss.first).new() == 2
    assert A.reduce_scalar(agg.ss.last).new() == 3
    B = gb.Matrix(float, nrows=2, ncols=3)
    assert B.reduce_scalar(agg.ss.first).new().is_empty
    assert B.reduce_scalar(agg.ss.last).new().is_empty
    assert B.reduce_rowwise(agg.ss.first).new().isequal(gb.Vector(float, size=B.nrows))
    assert B.reduce_columnwise(agg.ss.last).new().isequal(gb.Vector(float, size=B.ncols))
    silly = agg.Aggregator("silly", composite=[agg.ss.first, agg.ss.last],
                           finalize=lambda x, y, opts: gb.binary.plus(x & y), types=[agg.ss.first])
    v1 = A.reduce_rowwise(agg.ss.first).new()
    v2 = A.reduce_rowwise(agg.ss.last).new()
    assert A.reduce_rowwise(silly).new().isequal(gb.binary.plus(v1 & v2).new())
    s1 = A.reduce_scalar(agg.ss.first).new()
    s2 = A.reduce_scalar(agg.ss.last).new()
    assert A.reduce_scalar(silly).new().isequal(s1.value + s2.value)


def test_reduce_agg_firstlast_index_matrix(gb, A):
    agg = gb.agg
    cases = [("reduce_rowwise", agg.ss.first_index, [1, 4, 5, 0, 5, 2, 2]),
             ("reduce_rowwise", agg.ss.last_index, [3, 6, 5, 2, 5, 2, 4]),
             ("reduce_columnwise", agg.ss.first_index, [3, 0, 3, 0, 1, 2, 1]),
             ("reduce_columnwise", agg.ss.last_index, [3, 0, 6, 6, 6, 4, 1])]
    other = {"reduce_rowwise": "reduce_columnwise", "reduce_columnwise": "reduce_rowwise"}
    for method, op, exp in cases:
        assert getattr(A, method)(op).new().isequal(V(gb, range(7), exp))
        assert getattr(A.T, other[method])(op).new().isequal(V(gb, range(7), exp))
    with pytest.raises(ValueError, match="Aggregator first_index may not"):
        A.reduce_scalar(agg.ss.first_index).new()
    with pytest.raises(ValueError, match="Aggregator last_index may not"):
        A.reduce_scalar(agg.ss.last_index).new()
    silly = agg.Aggregator("silly", composite=[agg.ss.first_index, agg.ss.last_index],
                           finalize=lambda x, y, opts: gb.binary.plus(x & y), types=[agg.ss.first_index])
    v1 = A.reduce_rowwise(agg.ss.first_index).new()
    v2 = A.reduce_rowwise(agg.ss.last_index).new()
    assert A.reduce_rowwise(silly).new().isequal(gb.binary.plus(v1 & v2).new())
    with pytest.raises(ValueError, match="Aggregator"):
        A.reduce_scalar(silly).new()


def test_reduce_agg_positional_vector(gb, v):
    agg = gb.agg
    assert v.reduce(agg.ss.argmin).new() == 6
    assert v.reduce(agg.ss.argmax).new() == 4
    empty = gb.Vector(int, size=4)
    assert empty.reduce(agg.ss.first).new().is_empty
    assert empty.reduce(agg.ss.last).new().is_empty
    assert v.reduce(agg.ss.first).new() == 1
    assert v.reduce(agg.ss.last).new() == 0
    assert v.reduce(agg.ss.first_index).new() == 1
    assert v.reduce(agg.ss.last_index).new() == 6
    for parts, expect in [((agg.ss.argmin, agg.ss.argmax), 10), ((agg.ss.first, agg.ss.last), 1),
                          ((agg.ss.first_index, agg.ss.last_index), 7)]:
        silly = agg.Aggregator("silly", composite=list(parts),
                               finalize=lambda x, y, opts: gb.binary.plus(x & y), types=[parts[0]])
        assert v.reduce(silly).new() == expect
    assert repr(agg.ss.first) == "agg.ss.first"


def test_reduce_agg_positional_random_vs_numpy(gb):
    """Seeded 40 x 50 int64 matrix: row argmin/argmax/first/last vs numpy on the same entries."""
    rng = np.random.default_rng(11)
    dense = rng.integers(-5, 6, size=(40, 50))
    keep = rng.random((40, 50)) < 0.2
    r, c = np.nonzero(keep)
    M = gb.Matrix.from_coo(r, c, dense[r, c], nrows=40, ncols=50)
    got = {k: dict(zip(*getattr(M.reduce_rowwise(getattr(gb.agg.ss, k)).new(), "to_coo")()))
           for k in ("argmin", "argmax", "first", "last", "first_index", "last_index")}
    for i in range(40):
        cols = np.nonzero(keep[i])[0]
        if cols.size == 0:
            assert all(i not in g for g in got.values())
            continue
        vals = dense[i, cols]
        assert got["argmin"][i] == cols[np.argmin(vals)]
        assert got["argmax"][i] == cols[np.argmax(vals)]
        assert got["first"][i] == vals[0] and got["last"][i] == vals[-1]
        assert got["first_index"][i] == cols[0] and got["last_index"][i] == cols[-1]
