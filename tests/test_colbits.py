"""GPU parity of the batched-frontier path (csrc/gb_colbits.hip): GrB_mxm with a
left operand of at most 64 rows over a boolean LOR/ANY semiring, and the masked
scalar assign, on the column-word bitmap format.

The workload is the multi-source level BFS written with the reference's own
operations -- `V(Q.V)[:, :] = d; Q(~V.S, replace=True) << Q.mxm(A, lor_land)`
(the north-star's masked mxm, reference core/matrix.py:2206-2251 / core/base.py:483,
with the level stamp of notebooks/Example B.1 -- Level BFS.ipynb cell 8 applied
to k roots at once).  Row r of V must equal the oracle's single-source BFS levels
from root r bit for bit; single calls are checked against the oracle's GrB_mxm
restatement (oracle/gb_oracle.c) for every mask kind the fast path accepts, and
the shapes it declines must still give the general path's results.
"""
import zlib

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

import oracle as O  # noqa: E402


@pytest.fixture(scope="module")
def gb():
    import graphblas_amd

    return graphblas_amd


def _knobs(gb, **kv):
    class K:
        def __enter__(self):
            for k, v in kv.items():
                gb.set_knob(k, v)

        def __exit__(self, *a):
            for k in kv:
                gb.set_knob(k, 0)

    return K()


def _msbfs(gb, A, roots, n, semiring="lor_land"):
    sr = getattr(gb.semiring, semiring)
    k = len(roots)
    Q = gb.Matrix.from_coo(np.arange(k), roots, True, nrows=k, ncols=n)
    V = gb.Matrix(gb.INT32, k, n)
    d = 0
    while True:
        d += 1
        V(mask=Q.V)[:, :] = d
        Q(~V.S, replace=True) << Q.mxm(A, sr)
        if Q.nvals == 0:
            break
    r, c, x = V.to_coo()
    got = np.zeros((k, n), np.int32)
    got[r.astype(np.int64), c.astype(np.int64)] = x
    return got, d


@pytest.mark.parametrize("scale", [10, 13])
@pytest.mark.parametrize("k", [1, 7, 64])
@pytest.mark.parametrize("direction", [0, 1, 2])  # auto (device-chosen), pull only, push only
@pytest.mark.parametrize("hub", [0, 8])  # hub pieces of the default 512 edges, or of 8 (most rows)
@pytest.mark.parametrize("eager", [0, 1])  # level stamps as pending layers (default) or written at once
@pytest.mark.parametrize("hot", [0, 2])  # pull sources through the hot-column relabel: auto (off here) / forced
def test_msbfs_rmat_vs_oracle(gb, scale, k, direction, hub, eager, hot):
    G = O.rmat(scale, 16, 42)
    n = G.nrows
    r, c, _ = G.to_coo()
    A = gb.Matrix.from_coo(r, c, True, nrows=n, ncols=n)
    rng = np.random.default_rng(scale * 100 + k)
    deg = np.diff(G.indptr)
    roots = rng.choice(np.flatnonzero(deg > 0), k, replace=False)
    roots[0] = int(np.argmax(deg))  # the hub: long columns go to the wave path
    with _knobs(gb, colbits=1, colbits_direction=direction, colbits_hub=hub, colbits_eager=eager,
                xhot=hot, xhot_cols=300):
        got, _ = _msbfs(gb, A, roots, n)
    for i, src in enumerate(roots):
        lev, _, _ = O.bfs_levels(G, int(src))
        assert np.array_equal(got[i], lev), f"root {src} (row {i})"


@pytest.mark.parametrize("scale", [10, 13])
@pytest.mark.parametrize("k", [1, 7, 64])
@pytest.mark.parametrize("direction", [0, 1, 2])
@pytest.mark.parametrize("hub", [0, 8])
def test_msbfs_any_pair_vs_oracle(gb, scale, k, direction, hub):
    """BASELINE.json configs[2] names any_pair BOOL: the batched BFS with GxB_ANY_PAIR_BOOL, every
    direction mode (the ANY monoid + PAIR multiplier take the column-word path, gb_colbits.hip)"""
    G = O.rmat(scale, 16, 42)
    n = G.nrows
    r, c, _ = G.to_coo()
    A = gb.Matrix.from_coo(r, c, True, nrows=n, ncols=n)
    rng = np.random.default_rng(scale * 1000 + k)
    deg = np.diff(G.indptr)
    roots = rng.choice(np.flatnonzero(deg > 0), k, replace=False)
    roots[0] = int(np.argmax(deg))
    with _knobs(gb, colbits=1, colbits_direction=direction, colbits_hub=hub):
        got, _ = _msbfs(gb, A, roots, n, "any_pair")
    for i, src in enumerate(roots):
        lev, _, _ = O.bfs_levels(G, int(src))
        assert np.array_equal(got[i], lev), f"root {src} (row {i})"


def test_msbfs_duplicate_and_isolated_roots(gb):
    G = O.rmat(11, 16, 42)
    n = G.nrows
    r, c, _ = G.to_coo()
    A = gb.Matrix.from_coo(r, c, True, nrows=n, ncols=n)
    deg = np.diff(G.indptr)
    iso = int(np.flatnonzero(deg == 0)[0])
    hub = int(np.argmax(deg))
    roots = np.array([hub, hub, iso, 5, iso])
    with _knobs(gb, colbits=1):
        got, _ = _msbfs(gb, A, roots, n)
    for i, src in enumerate(roots):
        lev, _, _ = O.bfs_levels(G, int(src))
        assert np.array_equal(got[i], lev)


def _rand(rng, n, m, density, dtype="BOOL", iso=False):
    nnz = int(n * m * density)
    key = np.unique(rng.integers(0, n, nnz) * m + rng.integers(0, m, nnz))
    r, c = key // m, key % m
    if dtype == "BOOL":
        v = np.ones(key.size, bool) if iso else rng.random(key.size) < 0.7
    else:
        v = rng.integers(-3, 4, key.size).astype(O.NP[dtype])
    return O.Csr.from_coo(r, c, v, nrows=n, ncols=m, dtype=dtype)


def _gbm(gb, M, iso=False):
    r, c, v = M.to_coo()
    if iso:
        return gb.Matrix.from_coo(r, c, True, nrows=M.nrows, ncols=M.ncols)
    return gb.Matrix.from_coo(r, c, v, dtype=M.dtype, nrows=M.nrows, ncols=M.ncols)


def _same(got, ref):
    r, c, v = got.to_coo()
    er, ec, ev = ref.to_coo()
    assert np.array_equal(r.astype(np.int64), er) and np.array_equal(c.astype(np.int64), ec)
    assert np.array_equal(v, ev)


SR = [("lor_land", "LOR", "LAND"), ("any_pair", "ANY", "PAIR"), ("lor_first", "LOR", "FIRST"),
      ("lor_second", "LOR", "SECOND"), ("land_lor", "LAND", "LOR")]


@pytest.mark.parametrize("name,mon,mul", SR)
@pytest.mark.parametrize("masked", ["none", "struct", "comp_replace", "value_iso", "value_replace", "keep",
                                    "nullcomp", "nullcomp_replace"])
@pytest.mark.parametrize("tran1", [False, True])
@pytest.mark.parametrize("iso_a", [True, False])
def test_colbits_mxm_vs_oracle(gb, name, mon, mul, masked, tran1, iso_a):
    """single calls (forced onto the fast path where legal) against the oracle's GrB_mxm"""
    rng = np.random.default_rng(zlib.crc32(repr((name, masked, tran1, iso_a)).encode()))
    k, n, m = 13, 300, 300
    Ao = _rand(rng, k, n, 0.05, iso=iso_a)
    Bo = _rand(rng, m if tran1 else n, n if tran1 else m, 0.02, iso=True)
    Mo = _rand(rng, k, m, 0.3, iso=masked == "value_iso")
    Co = _rand(rng, k, m, 0.1, iso=True) if masked in ("keep", "nullcomp", "nullcomp_replace") \
        else O.Csr.empty(k, m, "BOOL")
    sr = getattr(gb.semiring, name)["BOOL"]
    Ag, Bg, Mg, Cg = _gbm(gb, Ao, iso_a), _gbm(gb, Bo, True), _gbm(gb, Mo, masked == "value_iso"), _gbm(gb, Co, True)
    Bx = Bg.T if tran1 else Bg
    kw = {}
    with _knobs(gb, colbits=1):
        if masked == "none":
            Cg << Ag.mxm(Bx, sr)
        elif masked == "struct":
            Cg(Mg.S) << Ag.mxm(Bx, sr)
            kw = dict(mask=Mo, mask_struct=True)
        elif masked == "comp_replace":
            Cg(~Mg.S, replace=True) << Ag.mxm(Bx, sr)
            kw = dict(mask=Mo, mask_struct=True, mask_comp=True, replace=True)
        elif masked == "value_iso":
            Cg(Mg.V) << Ag.mxm(Bx, sr)
            kw = dict(mask=Mo)
        elif masked == "value_replace":  # non-iso value mask: the general path
            Cg(Mg.V, replace=True) << Ag.mxm(Bx, sr)
            kw = dict(mask=Mo, replace=True)
        elif masked in ("nullcomp", "nullcomp_replace"):
            # ~NULL mask (C API: selects nothing), only reachable through the C ABI
            rep = masked == "nullcomp_replace"
            lib = gb.lib
            desc = {(False, False): lib.GrB_DESC_C, (False, True): lib.GrB_DESC_CT1,
                    (True, False): lib.GrB_DESC_RC, (True, True): lib.GrB_DESC_RCT1}[(rep, tran1)]
            assert lib.GrB_mxm(Cg._h, None, None, sr._carg, Ag._h, Bg._h, desc) == 0
            kw = dict(mask=None, mask_comp=True, replace=rep)
        else:  # mask without replace into a non-empty C: the general path
            Cg(Mg.S) << Ag.mxm(Bx, sr)
            kw = dict(mask=Mo, mask_struct=True)
        # a second product from the column-word result (format kept between calls)
        Dg = Cg.mxm(Bx, sr).new()
    ref = O.mxm(Co, Ao, Bo, (mon, mul, "BOOL"), tran1=tran1, **kw)
    _same(Cg, ref)
    _same(Dg, O.mxm(O.Csr.empty(k, m, "BOOL"), ref, Bo, (mon, mul, "BOOL"), tran1=tran1))


@pytest.mark.parametrize("structure", [True, False])
@pytest.mark.parametrize("dtype", ["INT32", "FP64", "UINT8"])
def test_colbits_assign_vs_numpy(gb, structure, dtype):
    rng = np.random.default_rng(7 + structure)
    k, n = 9, 500
    Mo = _rand(rng, k, n, 0.2)  # bool values, some false
    M = _gbm(gb, Mo)
    C = gb.Matrix(dtype, k, n)
    C[0, 3] = 11
    exp = np.zeros((k, n))
    have = np.zeros((k, n), bool)
    exp[0, 3], have[0, 3] = 11, True
    r, c, v = Mo.to_coo()
    with _knobs(gb, colbits=1):
        for step, x in enumerate([5, 2]):
            if structure:
                C(M.S)[:, :] = x
                sel = np.ones(r.size, bool)
            else:
                C(M.V)[:, :] = x
                sel = v.astype(bool)
            exp[r[sel], c[sel]] = x
            have[r[sel], c[sel]] = True
            assert C.nvals == int(have.sum())
    gr, gc, gv = C.to_coo()
    er, ec = np.nonzero(have)
    assert np.array_equal(gr.astype(np.int64), er) and np.array_equal(gc.astype(np.int64), ec)
    assert np.array_equal(gv, exp[er, ec].astype(gv.dtype))


def test_colbits_roundtrip_and_general_ops(gb):
    """a column-word result converts back for every other operation"""
    G = O.rmat(12, 8, 3)
    n = G.nrows
    r, c, _ = G.to_coo()
    A = gb.Matrix.from_coo(r, c, True, nrows=n, ncols=n)
    roots = np.array([1, 17, 200])
    Q = gb.Matrix.from_coo(np.arange(3), roots, True, nrows=3, ncols=n)
    with _knobs(gb, colbits=1):
        Q << Q.mxm(A, gb.semiring.any_pair)
    assert Q.nvals == sum(int(np.diff(G.indptr)[s]) for s in roots)
    D = Q.dup()
    E = Q.ewise_add(D, gb.binary.lor).new()
    for i, s in enumerate(roots):
        cols = G.indices[G.indptr[s]:G.indptr[s + 1]]
        rr, cc, _ = E.to_coo()
        assert np.array_equal(np.sort(cc[rr == i].astype(np.int64)), np.sort(cols))
    Q.clear()
    assert Q.nvals == 0


def test_colwords_view_touch(gb):
    """the frontier exchange's device access: words copied from one column-word matrix
    into another through GxB_Matrix_colwords_view, then GxB_Matrix_colwords_touch.
    (The copy goes through the HIP runtime the library uses: torch's bundled runtime
    cannot initialise after it in the same process.)"""
    import ctypes

    from graphblas_amd import device as gdev

    hip = ctypes.CDLL("libamdhip64.so")
    n = 5000
    rng = np.random.default_rng(3)
    r = rng.integers(0, 5, 900)
    c = rng.integers(0, n, 900)
    key = np.unique(r * n + c)
    Q = gb.Matrix.from_coo(key // n, key % n, True, nrows=5, ncols=n)
    D = gb.Matrix(bool, 5, n)
    p1, n1 = gdev.colwords_view(Q._h)
    p2, n2 = gdev.colwords_view(D._h)
    assert n1 == n2 == n
    assert hip.hipDeviceSynchronize() == 0
    assert hip.hipMemcpy(ctypes.c_void_p(p2), ctypes.c_void_p(p1), ctypes.c_size_t(8 * n), 3) == 0
    assert hip.hipDeviceSynchronize() == 0
    assert gb.lib.GxB_Matrix_colwords_touch(D._h) == 0
    assert D.nvals == key.size
    rr, cc, vv = D.to_coo()
    assert np.array_equal(rr.astype(np.int64) * n + cc.astype(np.int64), key) and vv.all()
    with pytest.raises(Exception):
        gdev.colwords_view(gb.Matrix(bool, 65, 10)._h)


def test_pending_stamps_wait_and_overwrite(gb):
    """layers applied in order (a later stamp overwrites an earlier one), across an explicit
    wait, with more stamps than the layer cap, and through dup / extract"""
    k, n = 6, 4200
    rng = np.random.default_rng(11)
    C = gb.Matrix(gb.INT64, k, n)
    exp = np.zeros((k, n), np.int64)
    have = np.zeros((k, n), bool)
    for step in range(40):  # > CB_MAX_LAYERS (16): materialised on the way
        r = rng.integers(0, k, 300)
        c = rng.integers(0, n, 300)
        key = np.unique(r * n + c)
        M = gb.Matrix.from_coo(key // n, key % n, True, nrows=k, ncols=n)
        C(M.S)[:, :] = step + 1
        exp[key // n, key % n] = step + 1
        have[key // n, key % n] = True
        if step == 10:
            C.wait()
        if step == 20:
            D = C.dup()
            dr, dc, dv = D.to_coo()
            er, ec = np.nonzero(have)
            assert np.array_equal(dv, exp[er, ec])
    assert C.nvals == int(have.sum())
    gr, gc, gv = C.to_coo()
    er, ec = np.nonzero(have)
    assert np.array_equal(gr.astype(np.int64), er) and np.array_equal(gc.astype(np.int64), ec)
    assert np.array_equal(gv, exp[er, ec])


def test_colbits_fp_value_mask_negative_zero(gb):
    """value masks follow the mask truth of their type: -0.0 is false, NaN true"""
    k, n = 3, 5000
    vals = np.array([-0.0, 0.0, np.nan, 2.5, -1.0])
    rows = np.array([0, 0, 1, 2, 2])
    cols = np.array([10, 11, 12, 4999, 7])
    M = gb.Matrix.from_coo(rows, cols, vals, dtype="FP64", nrows=k, ncols=n)
    C = gb.Matrix(gb.INT32, k, n)
    C(M.V)[:, :] = 9
    r, c, v = C.to_coo()
    got = sorted(zip(r.astype(int).tolist(), c.astype(int).tolist()))
    assert got == [(1, 12), (2, 7), (2, 4999)] and (v == 9).all()
