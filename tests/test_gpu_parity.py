"""GPU parity: the reference's own hot-path tests, restated through the
MI355X backend (graphblas_amd over libgraphblas_amd.so), plus seeded random
parity against the CPU oracle.  Integer / bool semirings must match bit for
bit; fp64 plus_times within 1e-6 relative (BASELINE.json north_star).

Reference tests restated here: graphblas/tests/test_matrix.py test_mxm :307,
test_mxm_transpose :317, test_mxm_nonsquare :335, test_mxm_mask :348,
test_mxm_accum :377, test_mxv :389, test_power :4367;
graphblas/tests/test_vector.py test_vxm :297, test_vxm_transpose :303,
test_vxm_nonsquare :309, test_vxm_mask :323, test_vxm_accum :348,
test_inner :1479, test_outer :1521; graphblas/tests/test_infix.py :80;
graphblas/tests/test_recorder.py :15; docs/user_guide/operations.rst:24-148.
"""
import contextlib
import zlib

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

import oracle as O  # noqa: E402


@pytest.fixture(scope="module")
def gb():
    import graphblas_amd

    return graphblas_amd


def Mat(gb, d, dtype=None):
    return gb.Matrix.from_coo(d["rows"], d["cols"], d["values"], dtype=dtype, nrows=d.get("nrows"),
                              ncols=d.get("ncols"))


def Vec(gb, d, dtype=None):
    return gb.Vector.from_coo(d["indices"], d["values"], dtype=dtype, size=d.get("size"))


@pytest.fixture
def A(gb, golden):
    g = golden["A"]
    return gb.Matrix.from_coo(g["rows"], g["cols"], g["values"])


@pytest.fixture
def v(gb, golden):
    g = golden["v"]
    return gb.Vector.from_coo(g["indices"], g["values"])


# ------------------------------------------------------------------ reference tests, restated
def test_mxm(gb, golden, A):
    C = A.mxm(A, gb.semiring.plus_times).new()
    assert C.isequal(Mat(gb, golden["cases"]["test_mxm"]["expected"]))


def test_mxm_transpose(gb, golden, A):
    C = A.dup()
    C << A.mxm(A.T, gb.semiring.plus_times)
    assert C.isequal(Mat(gb, golden["cases"]["test_mxm_transpose_AAT"]["expected"]))
    C << A.T.mxm(A, gb.semiring.plus_times)
    assert C.isequal(Mat(gb, golden["cases"]["test_mxm_transpose_ATA"]["expected"]))


def test_mxm_nonsquare(gb, golden):
    c = golden["cases"]["test_mxm_nonsquare"]
    A1, B1 = Mat(gb, c["A"]), Mat(gb, c["B"])
    C = gb.Matrix(A1.dtype, nrows=1, ncols=1)
    C << A1.mxm(B1, gb.semiring.max_plus)
    assert C[0, 0].new() == c["expected_scalar"]
    C1 = A1.mxm(B1, gb.semiring.max_plus).new()
    assert C1.isequal(C)
    C2 = A1.T.mxm(B1.T, gb.semiring.max_plus).new()
    assert C2.nrows == 5 and C2.ncols == 5


def test_mxm_mask(gb, golden, A):
    c = golden["cases"]["test_mxm_mask"]
    val_mask = Mat(gb, c["val_mask"])
    struct_mask = Mat(gb, c["struct_mask"])
    C = A.dup()
    C(val_mask.V) << A.mxm(A, gb.semiring.plus_times)
    assert C.isequal(Mat(gb, c["expected_value"]))
    C = A.dup()
    C(~val_mask.V) << A.mxm(A, gb.semiring.plus_times)
    assert C.isequal(Mat(gb, c["expected_comp"]))
    C = A.dup()
    C(struct_mask.S, replace=True).update(A.mxm(A, gb.semiring.plus_times))
    result3 = Mat(gb, c["expected_struct_replace"])
    assert C.isequal(result3)
    C2 = A.mxm(A, gb.semiring.plus_times).new(mask=struct_mask.S)
    assert C2.isequal(result3)
    with pytest.raises(TypeError, match="Mask must be"):
        A.mxm(A).new(mask=struct_mask)


def test_mxm_accum(gb, golden, A):
    A(gb.binary.plus) << A.mxm(A, gb.semiring.plus_times)
    assert A.isequal(Mat(gb, golden["cases"]["test_mxm_accum"]["expected"]))


def test_mxv(gb, golden, A, v):
    w = A.mxv(v, gb.semiring.plus_times).new()
    assert w.isequal(Vec(gb, golden["cases"]["test_mxv"]["expected"]))


def test_vxm(gb, golden, A, v):
    w = v.vxm(A, gb.semiring.plus_times).new()
    assert w.isequal(Vec(gb, golden["cases"]["test_vxm"]["expected"]))
    w = v.vxm(A.T, gb.semiring.plus_times).new()
    assert w.isequal(Vec(gb, golden["cases"]["test_vxm_transpose"]["expected"]))


def test_vxm_nonsquare(gb, golden, v):
    c = golden["cases"]["test_vxm_nonsquare"]
    A72 = Mat(gb, c["A"])
    u = gb.Vector(v.dtype, size=2)
    u().update(v.vxm(A72, gb.semiring.min_plus))
    assert u.isequal(Vec(gb, c["expected"]))
    w1 = v.vxm(A72, gb.semiring.min_plus).new()
    assert w1.isequal(u)
    v2 = gb.Vector.from_coo([0, 1], [1, 2])
    w2 = v2.vxm(A72.T, gb.semiring.min_plus).new()
    assert w2.size == 7


def test_vxm_mask(gb, golden, A, v):
    c = golden["cases"]["test_vxm_mask"]
    val_mask = Vec(gb, c["val_mask"])
    struct_mask = Vec(gb, c["struct_mask"])
    u = v.dup()
    u(struct_mask.S) << v.vxm(A, gb.semiring.plus_times)
    result = Vec(gb, c["expected_struct"])
    assert u.isequal(result)
    u = v.dup()
    u(~~struct_mask.S) << v.vxm(A, gb.semiring.plus_times)
    assert u.isequal(result)
    u = v.dup()
    u(~struct_mask.S) << v.vxm(A, gb.semiring.plus_times)
    assert u.isequal(Vec(gb, c["expected_comp"]))
    u = v.dup()
    u(replace=True, mask=val_mask.V) << v.vxm(A, gb.semiring.plus_times)
    result3 = Vec(gb, c["expected_value_replace"])
    assert u.isequal(result3)
    w = v.vxm(A, gb.semiring.plus_times).new(mask=val_mask.V)
    assert w.isequal(result3)


def test_vxm_accum(gb, golden, A, v):
    result = Vec(gb, golden["cases"]["test_vxm_accum"]["expected"])
    w1 = v.dup()
    w1(gb.binary.plus) << v.vxm(A, gb.semiring.plus_times)
    assert w1.isequal(result)
    w2 = v.dup()
    w2(gb.monoid.plus) << v.vxm(A, gb.semiring.plus_times)
    assert w2.isequal(result)
    w4 = v.dup()
    w4("+") << v.vxm(A, gb.semiring.plus_times)
    assert w4.isequal(result)


def test_inner_outer(gb, golden, v):
    c = golden["cases"]["test_inner"]
    s = gb.Scalar(v.dtype)
    s << v.inner(v)
    assert s == c["expected_scalar"]
    s(gb.binary.plus) << v.inner(v)
    assert s == c["expected_accum"]
    assert (v @ v).new() == c["expected_scalar"]
    R = gb.Matrix(v.dtype, nrows=1, ncols=v.size)
    Cc = gb.Matrix(v.dtype, nrows=v.size, ncols=1)
    idx, vals = v.to_coo()
    R.build(np.zeros_like(idx), idx, vals)
    Cc.build(idx, np.zeros_like(idx), vals)
    expected = Cc.mxm(R).new()
    assert v.outer(v).new().isequal(expected)
    assert v.outer(v, gb.monoid.times).new().isequal(expected)


def test_infix_fp64(gb, golden):
    fx = golden["cases"]["test_infix_matmul"]["fixtures"]
    v1, v2 = Vec(gb, fx["v1"], gb.FP64), Vec(gb, fx["v2"], gb.FP64)
    A1 = gb.Matrix.from_coo(fx["A1"]["rows"], fx["A1"]["cols"], fx["A1"]["values"], ncols=3)
    A2 = Mat(gb, fx["A2"], gb.FP64)
    for method, left, right in [("vxm", v2, A2), ("vxm", v2, A1.T), ("mxv", A1, v1), ("mxv", A2.T, v1),
                                ("mxm", A1, A2), ("mxm", A1.T, A2.T), ("mxm", A1, A1.T), ("mxm", A2.T, A2),
                                ("inner", v1, v2), ("inner", v1, v1)]:
        expected = getattr(left, method)(right, gb.op.plus_times).new()
        assert expected.isequal(gb.op.plus_times(left @ right).new())
        assert expected.isequal(gb.op.plus_times[float](left @ right).new())
        assert expected.isequal((left @ right).new())


def test_docs_tables(gb, golden):
    c = golden["cases"]
    d = c["docs_mxm_min_plus"]
    Am, Bm = Mat(gb, d["A"], gb.FP64), Mat(gb, d["B"], gb.FP64)
    C = gb.Matrix(float, Am.nrows, Bm.ncols)
    C << Am.mxm(Bm, op="min_plus")
    got = C.to_dict()
    exp = Mat(gb, d["expected"], gb.FP64).to_dict()
    # see tests/test_oracle_golden.py: the docs table's C[2,1] = 5.0 contradicts its inputs (5.5)
    assert got.pop((2, 1)) == 5.5 and exp.pop((2, 1)) == 5.0
    assert got == exp
    C2 = gb.Matrix(float, Am.nrows, Bm.ncols)
    C2 << gb.semiring.min_plus(Am @ Bm)
    assert C2.isequal(C)
    d = c["docs_mxv_plus_times"]
    w = Mat(gb, d["A"], gb.FP64).mxv(Vec(gb, d["v"], gb.FP64), op="plus_times").new()
    assert w.to_dict() == Vec(gb, d["expected"], gb.FP64).to_dict()
    d = c["docs_vxm_plus_plus"]
    u = Vec(gb, d["v"], gb.FP64).vxm(Mat(gb, d["B"], gb.FP64), op="plus_plus").new()
    assert u.to_dict() == Vec(gb, d["expected"], gb.FP64).to_dict()


def test_recorder_strings(gb, golden):
    A = gb.Matrix.from_coo([0, 1], [1, 1], [1, 2], name="A")
    B = gb.Matrix.from_coo([0, 1], [0, 1], [3, 4], name="B")
    with gb.Recorder() as rec:
        C = A.mxm(B).new(name="C")
    with rec:
        D = A.mxm(B.T, gb.semiring.min_plus).new(name="D")
        C(D.S) << A.T.ewise_mult(B)
    assert list(rec) == golden["cases"]["test_recorder"]["expected"]


def test_power(gb, A):
    expected = A.dup()
    for i in range(1, 50):
        result = A.power(i).new()
        assert result.isequal(expected)
        expected << A @ expected
    expected = A.T.new()
    for i in range(1, 10):
        result = A.T.power(i).new()
        assert result.isequal(expected)
        expected << A.T @ expected
    expected = A.dup()
    for i in range(1, 10):
        result = A.power(i, gb.semiring.min_plus).new()
        assert result.isequal(expected)
        expected << gb.semiring.min_plus(A @ expected)
    with pytest.raises(TypeError, match="must be a positive integer"):
        A.power(1.5)
    with pytest.raises(ValueError, match="must be a positive integer"):
        A.power(0)


def test_notebook_sssp_and_bfs(gb, golden):
    c = golden["cases"]["notebook_sssp"]
    g = c["graph"]
    m = gb.Matrix.from_coo(g["rows"], g["cols"], g["values"])
    v = gb.Vector(m.dtype, m.nrows)
    v[c["source"]] << 0
    w = v.dup()
    while True:
        w_old = w.dup()
        w(gb.binary.min) << w.vxm(m, gb.semiring.min_plus)
        if w.isequal(w_old):
            break
    assert w.to_dict() == {int(k): x for k, x in c["expected"].items()}
    # Level BFS (Example B.1 cell 8)
    lev = golden["cases"]["notebook_level_bfs"]
    Ab = gb.Matrix.from_coo(g["rows"], g["cols"], [True] * len(g["rows"]))
    vv = gb.Vector(gb.INT32, Ab.nrows)
    q = gb.Vector(bool, Ab.nrows)
    q[lev["source"]] << True
    d = 0
    while True:
        d += 1
        vv(mask=q.V)[:] = d
        q(~vv.S, replace=True) << q.vxm(Ab, gb.semiring.lor_land)
        if not q.reduce(gb.monoid.lor, allow_empty=False).new():
            break
    assert vv.to_dict() == {int(k): x for k, x in lev["expected"].items()}


def test_parent_bfs_min_first(gb, golden):
    """Example B.3 (Parent BFS) -- min_first over UINT64 with a complemented structural mask."""
    g = golden["cases"]["notebook_sssp"]["graph"]
    A = gb.Matrix.from_coo(g["rows"], g["cols"], True)
    N = A.nrows
    index_ramp = gb.Vector(gb.UINT64, N)
    index_ramp.build(range(N), range(N))
    parents = gb.Vector(gb.UINT64, N)
    parents[1] << 1
    wavefront = gb.Vector(gb.UINT64, N)
    wavefront[1] << 1
    while wavefront.nvals > 0:
        wavefront << index_ramp.ewise_mult(wavefront, gb.binary.first)
        wavefront(~parents.S, replace=True) << wavefront.vxm(A, gb.semiring.min_first)
        parents(gb.binary.plus) << wavefront
    # every non-root parent must be an in-neighbour already on a shallower level
    lev = golden["cases"]["notebook_level_bfs"]["expected"]
    got = parents.to_dict()
    edges = set(zip(g["rows"], g["cols"]))
    assert set(got) == {int(k) for k in lev}
    for child, par in got.items():
        if child != 1:
            assert (par, child) in edges and lev[str(par)] == lev[str(child)] - 1


# ------------------------------------------------------------------ random parity vs the oracle
def _rand_csr(rng, n, m, density, dtype):
    nnz = int(n * m * density)
    r = rng.integers(0, n, nnz)
    c = rng.integers(0, m, nnz)
    key = np.unique(r * m + c)
    r, c = key // m, key % m
    if dtype == "BOOL":
        vals = rng.random(key.size) < 0.8
    elif dtype in ("FP32", "FP64"):
        vals = rng.standard_normal(key.size).astype(O.NP[dtype])
    else:
        info = np.iinfo(O.NP[dtype])
        lo, hi = max(info.min, -50), min(info.max, 50)
        vals = rng.integers(lo, hi, key.size).astype(O.NP[dtype])
    return O.Csr.from_coo(r, c, vals, nrows=n, ncols=m, dtype=dtype)


@contextlib.contextmanager
def _knobs(gb, **kv):
    for k, v in kv.items():
        gb.set_knob(k, v)
    try:
        yield
    finally:
        for k in kv:
            gb.set_knob(k, 0)


def _to_gb(gb, M):
    r, c, v = M.to_coo()
    return gb.Matrix.from_coo(r, c, v, dtype=M.dtype, nrows=M.nrows, ncols=M.ncols)


def _check_mat(got, ref, fp=False):
    r, c, v = got.to_coo()
    er, ec, ev = ref.to_coo()
    assert np.array_equal(r.astype(np.int64), er) and np.array_equal(c.astype(np.int64), ec)
    if fp:
        np.testing.assert_allclose(v, ev, rtol=1e-6, atol=1e-9)
    else:
        assert np.array_equal(v, ev)


SEMIRINGS = [
    ("plus_times", "PLUS", "TIMES", "INT64"),
    ("min_plus", "MIN", "PLUS", "INT64"),
    ("max_plus", "MAX", "PLUS", "INT32"),
    ("plus_times", "PLUS", "TIMES", "FP64"),
    ("min_plus", "MIN", "PLUS", "FP64"),
    ("plus_pair", "PLUS", "PAIR", "INT64"),
    ("any_pair", "ANY", "PAIR", "INT64"),
    ("lor_land", "LOR", "LAND", "BOOL"),
    ("min_first", "MIN", "FIRST", "UINT64"),
    ("max_second", "MAX", "SECOND", "INT16"),
    ("plus_min", "PLUS", "MIN", "UINT8"),
    ("min_secondi", "MIN", "SECONDI", "INT64"),
    ("plus_times", "PLUS", "TIMES", "FP32"),
]


@pytest.mark.parametrize("name,mon,mul,dt", SEMIRINGS)
@pytest.mark.parametrize("masked", ["none", "struct", "comp_replace", "value", "struct_accum", "value_keep",
                                    "comp_accum"])
def test_random_mxm_vs_oracle(gb, name, mon, mul, dt, masked):
    rng = np.random.default_rng(zlib.crc32(repr((name, dt, masked)).encode()))
    n, k, m = 37, 53, 41
    Ao = _rand_csr(rng, n, k, 0.15, dt)
    Bo = _rand_csr(rng, k, m, 0.15, dt)
    Mo = _rand_csr(rng, n, m, 0.3, "BOOL")
    nonempty = masked in ("comp_replace", "struct_accum", "value_keep", "comp_accum")
    Co = _rand_csr(rng, n, m, 0.25, dt) if nonempty else O.Csr.empty(n, m, dt)
    sr = getattr(gb.semiring, name)[dt]
    Ag, Bg, Mg = _to_gb(gb, Ao), _to_gb(gb, Bo), _to_gb(gb, Mo)
    Cg = _to_gb(gb, Co)
    kw = {}
    if masked == "none":
        Cg << Ag.mxm(Bg, sr)
    elif masked == "struct":
        Cg(Mg.S) << Ag.mxm(Bg, sr)
        kw = dict(mask=Mo, mask_struct=True)
    elif masked == "comp_replace":
        Cg(~Mg.S, replace=True) << Ag.mxm(Bg, sr)
        kw = dict(mask=Mo, mask_struct=True, mask_comp=True, replace=True)
    elif masked == "struct_accum":
        # merge into a non-empty C: entries outside the mask kept, accum where both exist
        Cg(Mg.S, gb.binary.max) << Ag.mxm(Bg, sr)
        kw = dict(mask=Mo, mask_struct=True, accum=("MAX", dt))
    elif masked == "value_keep":
        Cg(Mg.V) << Ag.mxm(Bg, sr)
        kw = dict(mask=Mo)
    elif masked == "comp_accum":
        Cg(~Mg.S, gb.binary.plus) << Ag.mxm(Bg, sr)
        kw = dict(mask=Mo, mask_struct=True, mask_comp=True, accum=("PLUS", dt))
    else:
        Cg(Mg.V) << Ag.mxm(Bg, sr)
        kw = dict(mask=Mo)
    ref = O.mxm(Co, Ao, Bo, (mon, mul, dt), **kw)
    if mon == "ANY":
        r, c, _ = Cg.to_coo()
        er, ec, _ = ref.to_coo()
        assert np.array_equal(r.astype(np.int64), er) and np.array_equal(c.astype(np.int64), ec)
    else:
        _check_mat(Cg, ref, fp=dt in ("FP32", "FP64") and mon in ("PLUS", "TIMES"))


@pytest.mark.parametrize("name,mon,mul,dt", SEMIRINGS)
@pytest.mark.parametrize("kind", ["mxv", "vxm", "mxv_T", "vxm_T"])
def test_random_spmv_vs_oracle(gb, name, mon, mul, dt, kind):
    rng = np.random.default_rng(zlib.crc32(repr((name, dt, kind)).encode()))
    n = 301
    Ao = _rand_csr(rng, n, n, 0.03, dt)
    uo = _rand_csr(rng, n, 1, 0.4, dt)
    mo = _rand_csr(rng, n, 1, 0.5, "BOOL")
    wo = _rand_csr(rng, n, 1, 0.2, dt)
    Ag = _to_gb(gb, Ao)
    u = O.Vec.from_col(uo)
    m = O.Vec.from_col(mo)
    w0 = O.Vec.from_col(wo)
    ug = gb.Vector.from_coo(u.indices, u.values, dtype=dt, size=n)
    mg = gb.Vector.from_coo(m.indices, m.values, dtype="BOOL", size=n)
    wg = gb.Vector.from_coo(w0.indices, w0.values, dtype=dt, size=n)
    sr = getattr(gb.semiring, name)[dt]
    tran = kind.endswith("_T")
    AgT = Ag.T if tran else Ag
    if kind.startswith("mxv"):
        wg(mg.V, gb.binary.first) << AgT.mxv(ug, sr)
        ref = O.mxv(w0, Ao, u, (mon, mul, dt), mask=m, tran0=tran, accum=("FIRST", dt))
    else:
        wg(~mg.S, replace=True) << ug.vxm(AgT, sr)
        ref = O.vxm(w0, u, Ao, (mon, mul, dt), mask=m, mask_comp=True, mask_struct=True,
                    replace=True, tran1=tran)
    gi, gv = wg.to_coo()
    assert np.array_equal(gi.astype(np.int64), ref.indices)
    if mon == "ANY":
        return
    if dt in ("FP32", "FP64") and mon in ("PLUS", "TIMES"):
        # the SpMV kernels fold a row by a segmented scan across lanes (long rows: per-chunk
        # lane folds, then chunk order), not strictly in ascending k as the oracle does: fp
        # sums may differ by a few ulps of the terms (|terms| ~ 1 here)
        np.testing.assert_allclose(gv, ref.values, rtol=1e-5 if dt == "FP32" else 1e-12,
                                   atol=1e-6 if dt == "FP32" else 1e-12)
    else:
        assert np.array_equal(gv, ref.values)


def _skewed_csr(rng, n, dtype):
    """rows of very different lengths: empty, short, and longer than the SpMV's
    long-row threshold (128) and chunk (1024), so every kernel path runs."""
    lens = rng.integers(0, 12, n)
    lens[::17] = rng.integers(129, 3000, lens[::17].size)
    lens[5] = n  # a full row
    lens = np.minimum(lens, n)
    r = np.repeat(np.arange(n), lens)
    c = np.concatenate([rng.choice(n, size=min(L, n), replace=False) for L in lens])
    if dtype in ("FP32", "FP64"):
        v = rng.standard_normal(r.size).astype(O.NP[dtype])
    elif dtype == "BOOL":
        v = rng.random(r.size) < 0.8
    else:
        v = rng.integers(-40, 40, r.size).astype(O.NP[dtype])
    return O.Csr.from_coo(r, c, v, nrows=n, ncols=n, dtype=dtype)


@pytest.mark.parametrize("name,mon,mul,dt", [s for s in SEMIRINGS if s[0] not in ("any_pair", "lor_land")])
@pytest.mark.parametrize("udense", [True, False])
def test_spmv_long_rows_vs_oracle(gb, name, mon, mul, dt, udense):
    rng = np.random.default_rng(zlib.crc32(repr((name, dt, udense, "long")).encode()))
    n = 3000
    Ao = _skewed_csr(rng, n, dt)
    if udense:
        u = O.Vec.from_col(_rand_csr(rng, n, 1, 0.3, dt))
        u = O.Vec(n, dt, np.arange(n), np.resize(u.values, n) if u.values.size else np.zeros(n, O.NP[dt]))
    else:
        u = O.Vec.from_col(_rand_csr(rng, n, 1, 0.3, dt))
    mo = _rand_csr(rng, n, 1, 0.6, "BOOL")
    Ag = _to_gb(gb, Ao)
    m = O.Vec.from_col(mo)
    ug = gb.Vector.from_coo(u.indices, u.values, dtype=dt, size=n)
    mg = gb.Vector.from_coo(m.indices, m.values, dtype="BOOL", size=n)
    sr = getattr(gb.semiring, name)[dt]
    for masked in (False, True):
        wg = gb.Vector(dt, n)
        if masked:
            wg(mg.S) << Ag.mxv(ug, sr)
            ref = O.mxv(O.Vec(n, dt, [], []), Ao, u, (mon, mul, dt), mask=m, mask_struct=True)
        else:
            wg << ug.vxm(Ag, sr)
            ref = O.vxm(O.Vec(n, dt, [], []), u, Ao, (mon, mul, dt))
        gi, gv = wg.to_coo()
        assert np.array_equal(gi.astype(np.int64), ref.indices)
        if dt in ("FP32", "FP64") and mon in ("PLUS", "TIMES"):
            # long rows are folded per chunk then in chunk order; |row sums| up to ~sqrt(3000)
            np.testing.assert_allclose(gv, ref.values, rtol=1e-5 if dt == "FP32" else 1e-12,
                                       atol=1e-3 if dt == "FP32" else 1e-10)
        else:
            assert np.array_equal(gv, ref.values)


@pytest.mark.parametrize("name,mon,mul,dt", [("min_plus", "MIN", "PLUS", "INT64"),
                                             ("plus_times", "PLUS", "TIMES", "INT64"),
                                             ("max_second", "MAX", "SECOND", "INT16"),
                                             ("plus_times", "PLUS", "TIMES", "FP64"),
                                             ("min_secondi", "MIN", "SECONDI", "INT64"),
                                             ("any_pair", "ANY", "PAIR", "INT64")])
@pytest.mark.parametrize("group", [0, 1, 8])  # dot kernel: auto (wave per entry), thread per entry, 8 lanes
def test_masked_spgemm_long_lists_vs_oracle(gb, name, mon, mul, dt, group):
    """C<A.S> = A (+).(x) A on a matrix with rows up to 3000 entries: the masked dot's
    sampled-bucket search (lists >= 256) and the galloping merge both run."""
    rng = np.random.default_rng(zlib.crc32(repr((name, dt, "spgemm-long")).encode()))
    n = 2000
    Ao = _skewed_csr(rng, n, dt)
    Ag = _to_gb(gb, Ao)
    sr = getattr(gb.semiring, name)[dt]
    gb.set_knob("dot_group", group)
    try:
        Cg = Ag.mxm(Ag, sr).new(mask=Ag.S)
    finally:
        gb.set_knob("dot_group", 0)
    ref = O.mxm(O.Csr.empty(n, n, dt), Ao, Ao, (mon, mul, dt), mask=Ao, mask_struct=True)
    if mon == "ANY":
        r, c, _ = Cg.to_coo()
        er, ec, _ = ref.to_coo()
        assert np.array_equal(r.astype(np.int64), er) and np.array_equal(c.astype(np.int64), ec)
    else:
        _check_mat(Cg, ref, fp=dt in ("FP32", "FP64"))


@pytest.mark.parametrize("scale", [10, 12, 14])
def test_rmat_device_matches_oracle(gb, scale):
    G = O.rmat(scale, 16, 42, values="INT64", value_seed=2)
    import ctypes

    h = ctypes.c_void_p()
    assert gb.lib.GxB_Matrix_rmat(ctypes.byref(h), scale, 16, 42, 1, 2, 0, 0) == 0
    D = gb.Matrix.__new__(gb.Matrix)
    D._h, D.dtype, D.name = h, gb.INT64, "rmat"
    D._nrows = D._ncols = 1 << scale
    _check_mat(D, G)
    # a row shard equals the same rows of the full graph
    lo, hi = (1 << scale) // 4, (1 << scale) // 2
    h2 = ctypes.c_void_p()
    assert gb.lib.GxB_Matrix_rmat(ctypes.byref(h2), scale, 16, 42, 1, 2, lo, hi) == 0
    S = gb.Matrix.__new__(gb.Matrix)
    S._h, S.dtype, S.name = h2, gb.INT64, "shard"
    S._nrows, S._ncols = hi - lo, 1 << scale
    sr, sc, sv = S.to_coo()
    p0, p1 = G.indptr[lo], G.indptr[hi]
    assert np.array_equal(sc.astype(np.int64), G.indices[p0:p1])
    assert np.array_equal(sv, G.values[p0:p1])


@pytest.mark.parametrize("scale", [10, 14, 16])
@pytest.mark.parametrize("direction", [0, 1, 2])  # auto (device-chosen), pull only, push only
@pytest.mark.parametrize("heavy", [0, 8])  # push: default hub threshold, or hubs = rows > 8 edges
# lor_land: the notebook's semiring; any_pair: BASELINE.json configs[2]'s (semiring.py:174-203 binds
# any_pair[BOOL] to GxB_ANY_PAIR_BOOL)
@pytest.mark.parametrize("semiring", ["lor_land", "any_pair"])
def test_bfs_rmat_vs_oracle(gb, scale, direction, heavy, semiring):
    if heavy and direction == 1:
        pytest.skip("pull does not use the hub split")
    G = O.rmat(scale, 16, 42)
    r, c, _ = G.to_coo()
    A = gb.Matrix.from_coo(r, c, True, nrows=G.nrows, ncols=G.ncols)
    gb.set_knob("spmv_direction", direction)
    gb.set_knob("push_heavy", heavy)
    try:
        _bfs_check(gb, G, A, semiring)
    finally:
        gb.set_knob("spmv_direction", 0)
        gb.set_knob("push_heavy", 0)


def _bfs_check(gb, G, A, semiring="lor_land"):
    sr = getattr(gb.semiring, semiring)
    if semiring == "any_pair":
        assert sr[bool].gb_name == "GxB_ANY_PAIR_BOOL"
    for src in [int(np.argmax(np.diff(G.indptr))), 0, G.nrows // 3]:
        lev_ref, _, _ = O.bfs_levels(G, src)
        vv = gb.Vector(gb.INT32, G.nrows)
        q = gb.Vector(bool, G.nrows)
        q[src] = True
        d = 0
        while True:
            d += 1
            vv(mask=q.V)[:] = d
            q(~vv.S, replace=True) << q.vxm(A, sr)
            if q.nvals == 0:
                break
        got = np.zeros(G.nrows, np.int32)
        i, x = vv.to_coo()
        got[i.astype(np.int64)] = x
        assert np.array_equal(got, lev_ref)


@pytest.mark.parametrize("scale", [10, 13])
def test_masked_spgemm_rmat_vs_oracle(gb, scale):
    G = O.rmat(scale, 16, 42, values="INT64", value_seed=2)
    A = _to_gb(gb, G)
    C = A.mxm(A, gb.semiring.min_plus).new(mask=A.S)
    ref = O.mxm(O.Csr.empty(G.nrows, G.ncols, "INT64"), G, G, ("MIN", "PLUS", "INT64"), mask=G, mask_struct=True)
    _check_mat(C, ref)


@pytest.mark.parametrize("method", ["hash", "hash_window", "esc"])
@pytest.mark.parametrize("scale", [9, 11])
def test_unmasked_spgemm_fp64_rmat_vs_oracle(gb, scale, method):
    G = O.rmat(scale, 8, 42, values="FP64", value_seed=2)
    A = _to_gb(gb, G)
    with _knobs(gb, spgemm_method=1 if method == "esc" else 0, hash_window=int(method == "hash_window")):
        C = A.mxm(A, gb.semiring.plus_times).new()
    ref = O.mxm(O.Csr.empty(G.nrows, G.ncols, "FP64"), G, G, ("PLUS", "TIMES", "FP64"))
    _check_mat(C, ref, fp=True)
    if method == "esc":
        # the expand-sort-compress path folds in ascending k: bit-identical to the oracle
        r, c, vv = C.to_coo()
        assert np.array_equal(vv, ref.values)


UNMASKED_SR = [s for s in SEMIRINGS if s[1] != "ANY"] + [("any_pair", "ANY", "PAIR", "BOOL")]


@pytest.mark.parametrize("name,mon,mul,dt", UNMASKED_SR)
@pytest.mark.parametrize("method", ["hash", "hash_window", "hash_window_c", "hash_window_lw10"])
def test_hash_spgemm_rmat_vs_oracle(gb, name, mon, mul, dt, method):
    """Hash Gustavson on R-MAT s12 (rows in every bin: wave / workgroup LDS tables and, for
    the hub rows or with hash_window, the column-window kernel; hash_window_c shrinks the window's
    LDS value capacity so windows accumulate in C's values) against the oracle: bit-exact for exact
    monoids, rtol 1e-6 for floating plus / times (summation order)."""
    G = O.rmat(12, 16, 7, values="INT64" if dt != "BOOL" else None, value_seed=5)
    if dt != "BOOL":
        vals = (G.values % 13 + 1).astype(O.NP[dt]) if dt not in ("FP32", "FP64") else \
            (G.values.astype(np.float64) / 7.0).astype(O.NP[dt])
    else:
        vals = np.ones(G.nvals, bool)
    G = O.Csr(G.nrows, G.ncols, dt, G.indptr, G.indices, vals)
    A = _to_gb(gb, G)
    sr = getattr(gb.semiring, name)[dt]
    with _knobs(gb, hash_window=int(method != "hash"), window_vcap=512 if method == "hash_window_c" else 0,
                window_in_c_groups=1 if method == "hash_window_c" else 0,
                window_lw=10 if method == "hash_window_lw10" else 0):
        C = A.mxm(A, sr).new()
    ref = O.mxm(O.Csr.empty(G.nrows, G.ncols, dt), G, G, (mon, mul, dt))
    if mon == "ANY":
        r, c, _ = C.to_coo()
        er, ec, _ = ref.to_coo()
        assert np.array_equal(r.astype(np.int64), er) and np.array_equal(c.astype(np.int64), ec)
    else:
        _check_mat(C, ref, fp=dt in ("FP32", "FP64") and mon in ("PLUS", "TIMES"))


def test_spmv_fp64_rmat_vs_scipy(gb):
    import scipy.sparse as sp

    G = O.rmat(14, 16, 42, values="FP64", value_seed=2)
    A = _to_gb(gb, G)
    rng = np.random.default_rng(1)
    x = rng.random(G.nrows)
    xg = gb.Vector.from_coo(np.arange(G.nrows), x)
    y = xg.vxm(A, gb.semiring.plus_times).new()
    S = sp.csr_matrix((G.values, G.indices, G.indptr), shape=(G.nrows, G.ncols))
    ref = S.T @ x
    i, yv = y.to_coo()
    dense = np.zeros(G.nrows)
    dense[i.astype(np.int64)] = yv
    np.testing.assert_allclose(dense, ref, rtol=1e-6, atol=1e-12)


def test_edge_cases(gb):
    # empty operands, empty mask, dimension errors, aliasing, ~NULL-like behaviour
    A = gb.Matrix(gb.INT64, 5, 7)
    B = gb.Matrix(gb.INT64, 7, 3)
    C = A.mxm(B, gb.semiring.plus_times).new()
    assert C.nvals == 0 and C.shape == (5, 3)
    v = gb.Vector(gb.INT64, 7)
    w = A.mxv(v).new()
    assert w.nvals == 0 and w.size == 5
    with pytest.raises(gb.DimensionMismatch):
        A.mxm(A)
    # explicit zeros are kept (structural semantics)
    Z = gb.Matrix.from_coo([0, 1], [1, 0], [0, 0])
    P = Z.mxm(Z, gb.semiring.plus_times).new()
    assert P.to_dict() == {(0, 0): 0, (1, 1): 0}
    # build errors
    with pytest.raises(ValueError, match="Duplicate indices found"):
        gb.Matrix.from_coo([0, 0], [1, 1], [1, 2])
    with pytest.raises(gb.IndexOutOfBound):
        M = gb.Matrix(int, 2, 2)
        M.build([0, 11], [0, 0], [1, 1])
    M = gb.Matrix.from_coo([0, 6], [0, 1], [1, 2])
    with pytest.raises(gb.OutputNotEmpty):
        M.build([1, 5], [0, 1], [3, 4])
    # element access
    assert M[0, 0].new() == 1
    assert M[1, 1].new().value is None
    M[3, 1] = 9
    del M[0, 0]
    assert M.to_dict() == {(3, 1): 9, (6, 1): 2}


@pytest.mark.parametrize("fuse", [0, 1])
@pytest.mark.parametrize("direction", [0, 1, 2])
def test_bfs_fused_level_stamp(gb, fuse, direction):
    """The level stamp v<q> = d is deferred and carried out inside the next vxm's kernel
    (knob fuse_assign 0); with fuse_assign 1 it runs as its own launch.  Both must give
    the oracle's levels."""
    G = O.rmat(12, 16, 7)
    r, c, _ = G.to_coo()
    A = gb.Matrix.from_coo(r, c, True, nrows=G.nrows, ncols=G.ncols)
    gb.set_knob("fuse_assign", fuse)
    gb.set_knob("spmv_direction", direction)
    try:
        _bfs_check(gb, G, A)
    finally:
        gb.set_knob("fuse_assign", 0)
        gb.set_knob("spmv_direction", 0)


def _deferred_sequences(gb, seed):
    """Sequences around a deferrable assign v<q>(:) = x whose results must not depend on
    whether the assign is deferred / fused; returns the observable state."""
    rng = np.random.default_rng(seed)
    n = 700
    G = O.rmat(9, 8, seed)
    r, c, _ = G.to_coo()
    P = gb.Matrix.from_coo(r, c, True, nrows=G.nrows, ncols=G.ncols)
    n = G.nrows
    out = []
    for variant in ["fused", "read_v_between", "other_u", "struct_mask", "false_iso", "value_mask_noniso",
                    "v_as_output", "twice"]:
        v = gb.Vector(gb.INT32, n)
        pre = rng.choice(n, 20, replace=False)
        v.build(pre, np.arange(20, dtype=np.int32) + 100)
        qi = rng.choice(n, 15, replace=False)
        q = gb.Vector.from_coo(qi, False if variant == "false_iso" else True, dtype=bool, size=n)
        if variant == "value_mask_noniso":
            q = gb.Vector.from_coo(qi, (np.arange(15) % 2).astype(bool), dtype=bool, size=n)
        mask = q.S if variant == "struct_mask" else q.V
        v(mask=mask)[:] = 5
        if variant == "read_v_between":
            out.append(v.nvals)
        if variant == "other_u":
            u2 = gb.Vector.from_coo(rng.choice(n, 10, replace=False), True, dtype=bool, size=n)
            q2 = u2.vxm(P, gb.semiring.lor_land).new(mask=~v.S)
            out.append(q2.to_coo()[0])
        elif variant == "v_as_output":
            v(~v.S) << q.vxm(P, gb.semiring.plus_pair[gb.INT32])
        elif variant == "twice":
            v(mask=mask)[:] = 6
            q(~v.S, replace=True) << q.vxm(P, gb.semiring.lor_land)
        else:
            q(~v.S, replace=True) << q.vxm(P, gb.semiring.lor_land)
        out.append(q.to_coo()[0])
        out.append(v.to_coo())
        out.append(v.nvals)
    return out


def test_deferred_assign_is_unobservable(gb):
    results = []
    for fuse in (1, 0):
        gb.set_knob("fuse_assign", fuse)
        try:
            results.append(_deferred_sequences(gb, 3))
        finally:
            gb.set_knob("fuse_assign", 0)
    a, b = results
    assert len(a) == len(b)
    for x, y in zip(a, b):
        if isinstance(x, tuple):
            assert np.array_equal(x[0], y[0]) and np.array_equal(x[1], y[1])
        else:
            assert np.array_equal(np.asarray(x), np.asarray(y))


def test_deferred_assign_failure_is_recorded_on_its_vector(gb):
    """a failing deferred assign (injected) is an execution error of the
    deferred vector -- the unrelated call that triggers the flush succeeds, and the
    vector reports GrB_INVALID_OBJECT from then on."""
    from graphblas_amd import exceptions as ex

    n = 300
    v = gb.Vector(gb.INT32, n)
    q = gb.Vector.from_coo([1, 5, 9], True, dtype=bool, size=n)
    other = gb.Vector.from_coo([2, 3], [1, 2], dtype=gb.INT64, size=n)
    v(mask=q.V)[:] = 5  # deferred
    gb.set_knob("inject_flush_fail", 1)
    try:
        assert other.nvals == 2  # triggers the flush; the failure is not this call's
    finally:
        gb.set_knob("inject_flush_fail", 0)
    with pytest.raises(ex.InvalidObject):
        v.nvals
    assert q.nvals == 3 and other.nvals == 2


def _skewed_both(rng, n, dtype):
    """long rows AND long columns (the union of a row-skewed matrix and the transpose of
    another), so both phases of the two-sided masked dot get task-sized groups."""
    R, T = _skewed_csr(rng, n, dtype), _skewed_csr(rng, n, dtype)
    r1, c1, v1 = R.to_coo()
    r2, c2, v2 = T.to_coo()
    r, c, v = np.concatenate([r1, c2]), np.concatenate([c1, r2]), np.concatenate([v1, v2])
    key, idx = np.unique(r * n + c, return_index=True)
    return O.Csr.from_coo(key // n, key % n, v[idx], nrows=n, ncols=n, dtype=dtype)


TWO_SIDED = [
    ("min_plus", "MIN", "PLUS", "INT64"),
    ("plus_times", "PLUS", "TIMES", "INT64"),
    ("max_plus", "MAX", "PLUS", "INT32"),
    ("plus_pair", "PLUS", "PAIR", "INT64"),
    ("any_pair", "ANY", "PAIR", "INT64"),
    ("any_pair", "ANY", "PAIR", "BOOL"),
    ("lor_land", "LOR", "LAND", "BOOL"),
    ("min_first", "MIN", "FIRST", "UINT64"),
    ("max_second", "MAX", "SECOND", "INT16"),
    ("min_secondi", "MIN", "SECONDI", "INT64"),
    ("plus_min", "PLUS", "MIN", "UINT8"),
    ("times_plus", "TIMES", "PLUS", "INT32"),
]


@pytest.mark.parametrize("name,mon,mul,dt", TWO_SIDED)
# (dot_cap, dot_win, dot_pieces, dot_yblk): defaults; short task windows; a cap of 300 keys, so
# the hub lists run as pieces (default) or on the per-entry kernel (dot_pieces = 1); tasks in
# Y-blocked order (8 / 3 blocks)
@pytest.mark.parametrize("knobs", [(0, 0, 0, 0), (128, 256, 0, 0), (300, 256, 0, 0), (300, 256, 1, 0),
                                   (300, 256, 0, 8), (0, 0, 0, 3)])
@pytest.mark.parametrize("form", ["AA_struct", "AAT_struct", "ATA_value", "AB_rect"])
def test_masked_spgemm_two_sided_vs_oracle(gb, name, mon, mul, dt, knobs, form):
    """The two-sided LDS masked dot (gb_dot.hip): entries grouped by the side owning the
    longer list -- mask rows (CSR) or mask columns (the mask's CSC + position map, cached
    on a structural mask matrix, built per call for a value mask) -- in the small-group,
    task and per-entry kernels; shrunken cap/window knobs send hub lists to the per-entry
    kernel and cut groups into many tasks.  Bit-exact vs the oracle."""
    rng = np.random.default_rng(zlib.crc32(repr((name, dt, form, knobs)).encode()))  # same inputs every run
    n = 1500
    Ao = _skewed_both(rng, n, dt)
    sr = getattr(gb.semiring, name)[dt]
    Ag = _to_gb(gb, Ao)
    cap, win, pieces, yblk = knobs
    gb.set_knob("dot_yblk", yblk)
    gb.set_knob("dot_cap", cap)
    gb.set_knob("dot_win", win)
    gb.set_knob("dot_pieces", pieces)
    gb.set_knob("dot_pmin", 1)  # pieces for any number of huge entries
    try:
        if form == "AA_struct":
            Cg = Ag.mxm(Ag, sr).new(mask=Ag.S)
            ref = O.mxm(O.Csr.empty(n, n, dt), Ao, Ao, (mon, mul, dt), mask=Ao, mask_struct=True)
        elif form == "AAT_struct":
            Mo = _skewed_both(rng, n, "BOOL")
            Mg = _to_gb(gb, Mo)
            Cg = Ag.mxm(Ag.T, sr).new(mask=Mg.S)
            ref = O.mxm(O.Csr.empty(n, n, dt), Ao, Ao, (mon, mul, dt), mask=Mo, mask_struct=True, tran1=True)
        elif form == "ATA_value":
            Mo = _skewed_both(rng, n, "BOOL")
            Mg = _to_gb(gb, Mo)
            Cg = Ag.T.mxm(Ag, sr).new(mask=Mg.V)
            ref = O.mxm(O.Csr.empty(n, n, dt), Ao, Ao, (mon, mul, dt), mask=Mo, tran0=True)
        else:
            k, m = 900, 1100
            Bo = _skewed_both(rng, 1200, dt)
            r, c, v = Bo.to_coo()
            keep = (r < k) & (c < m)
            Bo = O.Csr.from_coo(r[keep], c[keep], v[keep], nrows=k, ncols=m, dtype=dt)
            r, c, v = Ao.to_coo()
            keep = c < k
            A2 = O.Csr.from_coo(r[keep], c[keep], v[keep], nrows=n, ncols=k, dtype=dt)
            Mo = _rand_csr(rng, n, m, 0.05, "BOOL")
            Cg = _to_gb(gb, A2).mxm(_to_gb(gb, Bo), sr).new(mask=_to_gb(gb, Mo).S)
            ref = O.mxm(O.Csr.empty(n, m, dt), A2, Bo, (mon, mul, dt), mask=Mo, mask_struct=True)
    finally:
        gb.set_knob("dot_cap", 0)
        gb.set_knob("dot_win", 0)
        gb.set_knob("dot_pieces", 0)
        gb.set_knob("dot_pmin", 0)
        gb.set_knob("dot_yblk", 0)
    if mon == "ANY":
        r, c, _ = Cg.to_coo()
        er, ec, _ = ref.to_coo()
        assert np.array_equal(r.astype(np.int64), er) and np.array_equal(c.astype(np.int64), ec)
    else:
        _check_mat(Cg, ref)


@pytest.mark.parametrize("name,mon,mul,dt", [("plus_times", "PLUS", "TIMES", "FP64"),
                                             ("plus_times", "PLUS", "TIMES", "FP32"),
                                             ("min_plus", "MIN", "PLUS", "INT64"),
                                             ("max_times", "MAX", "TIMES", "INT32"),
                                             ("min_first", "MIN", "FIRST", "UINT64"),
                                             ("plus_secondi", "PLUS", "SECONDI", "INT64")])
@pytest.mark.parametrize("hot", [64, 1000, 3000])
def test_spmv_hot_columns_vs_oracle(gb, name, mon, mul, dt, hot):
    """Dense-u SpMV on the hot-column relabel (gb_prim.hip gb_view_hot; knob xhot=2 builds it at
    any size, xhot_cols sets how many columns are hot): entries of the hot columns read the
    packed copy of their x values.  mxv, vxm (the CSC's relabel), masked and complemented;
    positional multipliers keep the true column.  Bit-exact for exact monoids."""
    rng = np.random.default_rng(zlib.crc32(repr((name, dt, hot, "xhot")).encode()))
    n = 3000
    Ao = _skewed_csr(rng, n, dt)
    uvals = (rng.standard_normal(n) if dt in ("FP32", "FP64") else rng.integers(0, 30, n)).astype(O.NP[dt])
    u = O.Vec(n, dt, np.arange(n), uvals)
    mo = _rand_csr(rng, n, 1, 0.5, "BOOL")
    m = O.Vec.from_col(mo)
    sr = getattr(gb.semiring, name)[dt]
    w0 = O.Vec(n, dt, np.zeros(0, np.int64), np.zeros(0, O.NP[dt]))
    with _knobs(gb, xhot=2, xhot_cols=hot):
        Ag = _to_gb(gb, Ao)
        ug = gb.Vector.from_coo(np.arange(n), uvals, dtype=dt, size=n)
        mg = gb.Vector.from_coo(m.indices, m.values, dtype="BOOL", size=n)
        for kind in ("mxv", "vxm", "mxv_mask", "vxm_comp"):
            wg = gb.Vector(dt, n)
            if kind == "mxv":
                wg << Ag.mxv(ug, sr)
                ref = O.mxv(w0, Ao, u, (mon, mul, dt))
            elif kind == "vxm":
                wg << ug.vxm(Ag, sr)
                ref = O.vxm(w0, u, Ao, (mon, mul, dt))
            elif kind == "mxv_mask":
                wg(mg.V) << Ag.mxv(ug, sr)
                ref = O.mxv(w0, Ao, u, (mon, mul, dt), mask=m)
            else:
                wg(~mg.S, replace=True) << ug.vxm(Ag, sr)
                ref = O.vxm(w0, u, Ao, (mon, mul, dt), mask=m, mask_comp=True, mask_struct=True, replace=True)
            gi, gv = wg.to_coo()
            assert np.array_equal(gi.astype(np.int64), ref.indices), kind
            if dt in ("FP32", "FP64") and mon == "PLUS":
                np.testing.assert_allclose(gv, ref.values, rtol=1e-5 if dt == "FP32" else 1e-12,
                                           atol=1e-3 if dt == "FP32" else 1e-10)
            else:
                assert np.array_equal(gv, ref.values), kind


@pytest.mark.parametrize("lo,hi,dt", [(1, 256, "INT64"), (-128, 128, "INT64"), (0, 65536, "INT64"),
                                      (-32768, 32768, "INT32"), (0, 1 << 32, "UINT64"), (-(1 << 31), 1 << 31, "INT64"),
                                      (0, 1 << 40, "INT64"), (0, 60000, "UINT32")])
def test_masked_dot_narrow_values(gb, lo, hi, dt):
    """The masked dot reads hit values from a cached narrow copy when every integer value fits
    1 / 2 / 4 bytes (gb_prim.hip gb_view_narrow; unsigned and signed kinds, and a range that fits
    none).  C<A.S> = A min.+ A and plus.times, bit-exact vs the oracle and vs knob narrow = 1."""
    rng = np.random.default_rng(abs(lo) + hi % 1000 + len(dt))
    n = 1500
    S = _skewed_both(rng, n, "BOOL")
    r, c, _ = S.to_coo()
    v = rng.integers(lo, hi, r.size, dtype=np.int64).astype(O.NP[dt])
    Ao = O.Csr.from_coo(r, c, v, nrows=n, ncols=n, dtype=dt)
    for name, mon, mul in (("min_plus", "MIN", "PLUS"), ("plus_times", "PLUS", "TIMES")):
        sr = getattr(gb.semiring, name)[dt]
        ref = O.mxm(O.Csr.empty(n, n, dt), Ao, Ao, (mon, mul, dt), mask=Ao, mask_struct=True)
        got = []
        for narrow in (0, 1):
            gb.set_knob("narrow", narrow)
            try:
                Ag = _to_gb(gb, Ao)  # a fresh matrix: no narrow copy cached yet
                got.append(Ag.mxm(Ag, sr).new(mask=Ag.S))
            finally:
                gb.set_knob("narrow", 0)
        for Cg in got:
            _check_mat(Cg, ref)


@pytest.mark.parametrize("knobs", [{}, {"dot_ypack": 1}, {"dot_xlds": 1}, {"dot_ypack": 1, "dot_xlds": 1},
                                   {"dot_small_seq": 1}])
@pytest.mark.parametrize("lo,hi", [(1, 256), (-128, 128), (0, 1 << 20)])
def test_masked_dot_round6_value_paths(gb, knobs, lo, hi):
    """Round 6's dot paths (gb_dot.hip): one-byte X values staged in LDS (knob dot_xlds = 1: off),
    one-byte Y values packed into the streamed keys' top byte (dot_ypack = 1: off), the flat
    small groups with LDS-slot folds (dot_small_seq = 1: the one-entry-at-a-time loop); unsigned,
    signed and wider-than-a-byte values (the byte paths must stand aside), min.plus, plus.times
    and max.plus, bit-exact vs the oracle under every knob setting."""
    rng = np.random.default_rng(abs(lo) + hi % 977)
    n = 1500
    S = _skewed_both(rng, n, "BOOL")
    r, c, _ = S.to_coo()
    v = rng.integers(lo, hi, r.size, dtype=np.int64)
    Ao = O.Csr.from_coo(r, c, v, nrows=n, ncols=n, dtype="INT64")
    import ctypes

    def stat(nm):
        c = ctypes.c_int64()
        assert gb.lib.GxB_Global_get_int(f"stat_{nm}".encode(), ctypes.byref(c)) == 0
        return c.value

    t0 = stat("dot_task_entries_R") + stat("dot_task_entries_C")
    with _knobs(gb, **knobs):
        Ag = _to_gb(gb, Ao)  # a fresh matrix: its narrow copies are built under these knobs
        for name, mon, mul in (("min_plus", "MIN", "PLUS"), ("plus_times", "PLUS", "TIMES"),
                               ("max_plus", "MAX", "PLUS")):
            sr = getattr(gb.semiring, name)["INT64"]
            ref = O.mxm(O.Csr.empty(n, n, "INT64"), Ao, Ao, (mon, mul, "INT64"), mask=Ao, mask_struct=True)
            _check_mat(Ag.mxm(Ag, sr).new(mask=Ag.S), ref)
    assert stat("dot_task_entries_R") + stat("dot_task_entries_C") > t0  # the task kernel ran
