"""Parity at benchmark scale with the library's default knobs (-m gpu).

Several paths switch on only at the bench's sizes -- the hot-column relabel (matrices with at
least 2^22 entries), the BFS pull heads and the packed one-round finish, the dot kernels' task
and huge-list classes, the hash SpGEMM's column-window bins -- so the bench's own workloads are
checked here, through the C ABI exactly as bench.py drives them, against the CPU oracle
(oracle/gb_oracle.c via oracle.py: test infrastructure only):

* config 3: the notebook's level BFS (`v<q.V> = d; q<!v.S,replace> = q any.pair A`, reference
  notebooks/Example B.1 -- Level BFS.ipynb cell 8) on R-MAT s22 from the bench's 16 roots, with
  any_pair and lor_land, levels bit-exact vs O.bfs_levels; the 64-root batched form (masked
  GrB_mxm on column words): every root's levels;
* config 4: C<A.S> = A min.+ A (reference core/matrix.py:2241 via core/base.py:483), INT64,
  the whole C at s18 and 1024 sampled rows at s20, bit-exact vs O.mxm, and the whole C at s20 vs
  the parallel oracle; north_star's own form C(M.V, accum=plus) << A.mxm(A, min_plus) with a
  stored-false value mask and a pre-filled C, the whole C at s18 and 1024 rows at s20, every dot
  class asserted by the library's stat counters;
* config 2: y = x plus.times A (GrB_vxm, dense fp64 x) at s20 and s22, ef 16 and 60, rtol 1e-6 vs
  scipy (BASELINE.json north_star's fp64 tolerance);
* config 5: C = A plus.times A (unmasked hash Gustavson) at s19, 512 sampled rows (the 32
  longest rows first: the column-window bins) vs a numpy fold, rtol 1e-6.
The graphs are generated on the device (GxB_Matrix_rmat, the bench's generator) and exported
for the oracle, so both sides see the same matrix."""
import ctypes

import numpy as np
import pytest

import oracle as O

pytestmark = pytest.mark.gpu

U64 = ctypes.c_uint64
NP_OF = {"BOOL": np.bool_, "INT64": np.int64, "FP64": np.float64}
KIND = {"BOOL": 0, "INT64": 1, "FP64": 2}


@pytest.fixture(scope="module")
def gb():
    import graphblas_amd

    return graphblas_amd


def ok(rc, what):
    assert rc == 0, f"{what}: GrB_Info {rc}"


def rmat(lib, scale, tname, ef=16, seed=42):
    h = ctypes.c_void_p()
    ok(lib.GxB_Matrix_rmat(ctypes.byref(h), scale, ef, seed, KIND[tname], 2, 0, 0), "rmat")
    ok(lib.GxB_Matrix_prepare_transpose(h), "transpose")
    return h


def export(lib, h, nrows, tname, ncols=None):
    nv = U64()
    ok(lib.GrB_Matrix_nvals(ctypes.byref(nv), h), "nvals")
    nz = nv.value
    ap = np.empty(nrows + 1, np.uint64)
    ai = np.empty(nz, np.uint64)
    ax = np.empty(max(nz, 1), NP_OF[tname])
    lens = [U64(nrows + 1), U64(nz), U64(nz)]
    ok(getattr(lib, f"GrB_Matrix_export_{tname}")(ctypes.c_void_p(ap.ctypes.data), ctypes.c_void_p(ai.ctypes.data),
                                                  ctypes.c_void_p(ax.ctypes.data), *[ctypes.byref(x) for x in lens],
                                                  0, h), "export")
    return O.Csr(nrows, nrows if ncols is None else ncols, tname, ap.astype(np.int64), ai.astype(np.int64), ax[:nz])


def free(lib, *hs):
    for h in hs:
        lib.GrB_Matrix_free(ctypes.byref(h))


def bench_roots(deg, seed=42, k=16):
    """bench.py's roots: 16 seeded vertices with out-edges (Graph500)"""
    return np.random.default_rng(seed).choice(np.flatnonzero(deg > 0), k, replace=False)


@pytest.fixture(scope="module")
def s22(gb):
    lib = gb.lib
    A = rmat(lib, 22, "BOOL")
    G = export(lib, A, 1 << 22, "BOOL")
    yield A, G
    free(lib, A)


@pytest.mark.parametrize("semiring", ["any_pair", "lor_land"])
def test_level_bfs_s22_bench_roots(gb, s22, semiring):
    lib = gb.lib
    A, G = s22
    n = G.nrows
    sr = lib.GxB_ANY_PAIR_BOOL if semiring == "any_pair" else lib.GrB_LOR_LAND_SEMIRING_BOOL
    q, v = ctypes.c_void_p(), ctypes.c_void_p()
    ok(lib.GrB_Vector_new(ctypes.byref(q), lib.GrB_BOOL, n), "q")
    ok(lib.GrB_Vector_new(ctypes.byref(v), lib.GrB_INT32, n), "v")
    nv = U64()
    try:
        for src in bench_roots(np.diff(G.indptr)):
            ok(lib.GrB_Vector_clear(q), "clear q")
            ok(lib.GrB_Vector_clear(v), "clear v")
            ok(lib.GrB_Vector_setElement_BOOL(q, True, int(src)), "q[src]")
            d = 0
            while True:
                d += 1
                ok(lib.GrB_Vector_assign_INT32(v, q, None, d, lib.GrB_ALL, n, None), "v<q> = d")
                ok(lib.GrB_vxm(q, v, None, sr, q, A, lib.GrB_DESC_RSC), "q<!v.S> = q sr A")
                ok(lib.GrB_Vector_nvals(ctypes.byref(nv), q), "nvals")
                if nv.value == 0:
                    break
            ok(lib.GrB_Vector_nvals(ctypes.byref(nv), v), "nvals v")
            idx = np.empty(nv.value, np.uint64)
            lv = np.empty(nv.value, np.int32)
            ok(lib.GrB_Vector_extractTuples_INT32(ctypes.c_void_p(idx.ctypes.data), ctypes.c_void_p(lv.ctypes.data),
                                                  ctypes.byref(nv), v), "extract v")
            got = np.zeros(n, np.int32)
            got[idx.astype(np.int64)] = lv
            ref, _, _ = O.bfs_levels(G, int(src))
            assert np.array_equal(got, ref), f"root {src}: levels differ from the oracle"
    finally:
        lib.GrB_Vector_free(ctypes.byref(q))
        lib.GrB_Vector_free(ctypes.byref(v))


def test_msbfs_s22_64_roots(gb, s22):
    """bench.py config3_msbfs: the 16 bench roots + 48 more, every root's levels vs the oracle"""
    lib = gb.lib
    A, G = s22
    n = G.nrows
    K = 64
    deg = np.diff(G.indptr)
    roots16 = bench_roots(deg)
    pool = np.setdiff1d(np.flatnonzero(deg > 0), roots16)
    roots = np.concatenate([roots16, np.random.default_rng(43).choice(pool, K - 16, replace=False)]).astype(np.uint64)
    Q, V = ctypes.c_void_p(), ctypes.c_void_p()
    ok(lib.GrB_Matrix_new(ctypes.byref(Q), lib.GrB_BOOL, K, n), "Q")
    ok(lib.GrB_Matrix_new(ctypes.byref(V), lib.GrB_INT32, K, n), "V")
    qi = np.arange(K, dtype=np.uint64)
    nv = U64()
    try:
        ok(lib.GxB_Matrix_build_Scalar_BOOL(Q, ctypes.c_void_p(qi.ctypes.data), ctypes.c_void_p(roots.ctypes.data),
                                            True, K), "build Q")
        d = 0
        while True:
            d += 1
            ok(lib.GrB_Matrix_assign_INT32(V, Q, None, d, lib.GrB_ALL, K, lib.GrB_ALL, n, None), "V<Q> = d")
            ok(lib.GrB_mxm(Q, V, None, lib.GxB_ANY_PAIR_BOOL, Q, A, lib.GrB_DESC_RSC), "Q<!V.S> = Q any.pair A")
            ok(lib.GrB_Matrix_nvals(ctypes.byref(nv), Q), "nvals Q")
            if nv.value == 0:
                break
        ok(lib.GrB_Matrix_nvals(ctypes.byref(nv), V), "nvals V")
        m = nv.value
        vi, vj, vx = np.empty(m, np.uint64), np.empty(m, np.uint64), np.empty(m, np.int32)
        ok(lib.GrB_Matrix_extractTuples_INT32(ctypes.c_void_p(vi.ctypes.data), ctypes.c_void_p(vj.ctypes.data),
                                              ctypes.c_void_p(vx.ctypes.data), ctypes.byref(nv), V), "extract V")
        vi, vj = vi.astype(np.int64), vj.astype(np.int64)
        starts = np.searchsorted(vi, np.arange(K + 1))
        for r in range(K):
            got = np.zeros(n, np.int32)
            got[vj[starts[r]:starts[r + 1]]] = vx[starts[r]:starts[r + 1]]
            ref, _, _ = O.bfs_levels(G, int(roots[r]))
            assert np.array_equal(got, ref), f"root #{r} ({roots[r]}): levels differ from the oracle"
    finally:
        free(lib, Q, V)


def _rows_csr(G, rows):
    """the CSR of the given rows of G (same columns)"""
    lens = np.diff(G.indptr)[rows]
    p = np.concatenate([[0], np.cumsum(lens)])
    sel = np.concatenate([np.arange(G.indptr[r], G.indptr[r + 1]) for r in rows]) if len(rows) else np.zeros(0, int)
    return O.Csr(len(rows), G.ncols, G.dtype, p, G.indices[sel], G.values[sel])


@pytest.mark.parametrize("scale,rows", [(18, None), (20, 1024)])
def test_masked_min_plus_spgemm_bench_scale(gb, scale, rows):
    """config 4: C<A.S> = A min.+ A, INT64 weights in [1,255]; the whole C at s18, sampled rows
    at s20 (bit-exact)"""
    lib = gb.lib
    n = 1 << scale
    B = rmat(lib, scale, "INT64")
    C = ctypes.c_void_p()
    ok(lib.GrB_Matrix_new(ctypes.byref(C), lib.GrB_INT64, n, n), "C")
    try:
        ok(lib.GrB_mxm(C, B, None, lib.GrB_MIN_PLUS_SEMIRING_INT64, B, B, lib.GrB_DESC_S), "mxm")
        G = export(lib, B, n, "INT64")
        Cg = export(lib, C, n, "INT64")
    finally:
        free(lib, B, C)
    sr = ("MIN", "PLUS", "INT64")
    if rows is None:
        ref = O.mxm(O.Csr.empty(n, n, "INT64"), G, G, sr, mask=G, mask_struct=True)
        assert np.array_equal(Cg.indptr, ref.indptr)
        assert np.array_equal(Cg.indices, ref.indices)
        assert np.array_equal(Cg.values, ref.values)
        return
    # sampled rows: the 64 longest rows (the dot's long-list classes) + random ones
    deg = np.diff(G.indptr)
    pick = np.concatenate([np.argsort(deg)[-64:], np.random.default_rng(7).choice(n, rows - 64, replace=False)])
    pick = np.unique(pick)
    Gs = _rows_csr(G, pick)
    ref = O.mxm(O.Csr.empty(len(pick), n, "INT64"), Gs, G, sr, mask=Gs, mask_struct=True)
    Cs = _rows_csr(Cg, pick)
    assert np.array_equal(Cs.indptr, ref.indptr)
    assert np.array_equal(Cs.indices, ref.indices)
    assert np.array_equal(Cs.values, ref.values)


def _threads():
    import os
    return max(1, min(16, int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)))


def _import_csr(lib, M, tname):
    """a host Csr into a new GrB_Matrix (GrB_Matrix_import, CSR format)"""
    h = ctypes.c_void_p()
    ap = M.indptr.astype(np.uint64)
    ai = M.indices.astype(np.uint64)
    ax = np.ascontiguousarray(M.values, NP_OF[tname]) if M.nvals else np.zeros(1, NP_OF[tname])
    ok(getattr(lib, f"GrB_Matrix_import_{tname}")(ctypes.byref(h), getattr(lib, f"GrB_{tname}"), M.nrows, M.ncols,
                                                  ctypes.c_void_p(ap.ctypes.data), ctypes.c_void_p(ai.ctypes.data),
                                                  ctypes.c_void_p(ax.ctypes.data), len(ap), len(ai), len(ax), 0),
       "import")
    return h


def _stats(lib, names):
    v = ctypes.c_int64()
    out = {}
    for nm in names:
        ok(lib.GxB_Global_get_int(f"stat_{nm}".encode(), ctypes.byref(v)), nm)
        out[nm] = v.value
    return out


DOT_STATS = ["dot_calls", "dot_task_entries_R", "dot_task_entries_C", "dot_piece_entries_R", "dot_piece_entries_C",
             "dot_hub_chunks_R", "dot_hub_chunks_C", "dot_huge_entries", "dot_narrow_calls"]


def test_masked_min_plus_spgemm_whole_c_s20(gb):
    """config 4 at BASELINE's own scale (configs[3]: R-MAT s20): the WHOLE C of C<A.S> = A min.+ A,
    bit-exact against the parallel oracle (or_masked_dot_min_plus_int64_par: per mask entry a
    sorted merge / galloping dot over A(i,:) and A^T(j,:), every mask row)"""
    import scipy.sparse as sp

    lib = gb.lib
    scale = 20
    n = 1 << scale
    B = rmat(lib, scale, "INT64")
    C = ctypes.c_void_p()
    ok(lib.GrB_Matrix_new(ctypes.byref(C), lib.GrB_INT64, n, n), "C")
    try:
        ok(lib.GrB_mxm(C, B, None, lib.GrB_MIN_PLUS_SEMIRING_INT64, B, B, lib.GrB_DESC_S), "mxm")
        G = export(lib, B, n, "INT64")
        Cg = export(lib, C, n, "INT64")
    finally:
        free(lib, B, C)
    T = sp.csr_matrix((G.values, G.indices, G.indptr), shape=(n, n)).T.tocsr()
    T.sort_indices()
    GT = O.Csr(n, n, "INT64", T.indptr, T.indices, T.data)
    vals, present, nc, _ = O.masked_dot_min_plus_int64_par(G, GT, 0, n, _threads())
    rows = np.repeat(np.arange(n), np.diff(G.indptr))
    ref_p = np.concatenate([[0], np.cumsum(np.bincount(rows[present], minlength=n))])
    assert nc == int(present.sum()) == Cg.nvals
    assert np.array_equal(Cg.indptr, ref_p)
    assert np.array_equal(Cg.indices, G.indices[present])
    assert np.array_equal(Cg.values, vals[present])


def _north_star_operands(G, seed):
    """M: A's structure as a BOOL value mask with ~30 % stored falses; C0: a pre-filled INT64 C holding
    half of A's entries plus as many entries outside A's structure (so the accum merge, the kept entries
    under false / absent mask entries and the new entries all occur)"""
    rng = np.random.default_rng(seed)
    n = G.nrows
    M = O.Csr(n, n, "BOOL", G.indptr, G.indices, rng.random(G.nvals) >= 0.3)
    rows = np.repeat(np.arange(n), np.diff(G.indptr))
    keep = rng.random(G.nvals) < 0.5
    extra = G.nvals // 2
    er, ec = rng.integers(0, n, extra), rng.integers(0, n, extra)
    r = np.concatenate([rows[keep], er])
    c = np.concatenate([G.indices[keep], ec])
    lin = np.unique(r * n + c)
    r, c = lin // n, lin % n
    C0 = O.Csr(n, n, "INT64", np.concatenate([[0], np.cumsum(np.bincount(r, minlength=n))]), c,
               rng.integers(-1000, 1000, len(lin)))
    return M, C0


@pytest.mark.parametrize("scale,rows", [(18, None), (20, 1024)])
@pytest.mark.parametrize("pieces", ["default", "forced"])
def test_north_star_value_mask_accum_bench_scale(gb, scale, rows, pieces):
    """BASELINE north_star's expression at bench scale: C(M.V, accum=binary.plus) << A.mxm(A, min_plus)
    (reference core/base.py:318-483 -> GrB_mxm(C, M, GrB_PLUS_INT64, min_plus, A, A, NULL); small cases
    pinned at graphblas/tests/test_matrix.py:348-386) with M a value mask holding stored falses and C
    pre-filled: the whole C at s18, the 64 longest + random rows at s20, bit-exact vs O.mxm.  The dot's
    classes must all fire (stat counters): task entries in both phases, hub chunks, narrow values,
    and -- with pieces="forced" (knob dot_pmin = 1) -- the hub-piece tasks; by default s20's few hub
    entries go to the per-entry kernel instead (dot_huge_entries)."""
    lib = gb.lib
    n = 1 << scale
    A = rmat(lib, scale, "INT64")
    G = export(lib, A, n, "INT64")
    Mh_, Ch_ = ctypes.c_void_p(), ctypes.c_void_p()
    Mc, C0 = _north_star_operands(G, 5 + scale)
    try:
        Mh_ = _import_csr(lib, Mc, "BOOL")
        Ch_ = _import_csr(lib, C0, "INT64")
        if pieces == "forced":
            ok(lib.GxB_Global_set_int(b"dot_pmin", 1), "knob")
        before = _stats(lib, DOT_STATS)
        ok(lib.GrB_mxm(Ch_, Mh_, lib.GrB_PLUS_INT64, lib.GrB_MIN_PLUS_SEMIRING_INT64, A, A, None), "mxm")
        after = _stats(lib, DOT_STATS)
        Cg = export(lib, Ch_, n, "INT64")
    finally:
        lib.GxB_Global_set_int(b"dot_pmin", 0)
        free(lib, A, Mh_, Ch_)
    d = {k: after[k] - before[k] for k in DOT_STATS}
    assert d["dot_calls"] == 1, d
    for k in ("dot_task_entries_R", "dot_task_entries_C", "dot_hub_chunks_R", "dot_hub_chunks_C", "dot_narrow_calls"):
        assert d[k] > 0, (k, d)
    if pieces == "forced":
        assert d["dot_piece_entries_R"] > 0 and d["dot_piece_entries_C"] > 0, d
    else:
        assert d["dot_piece_entries_R"] + d["dot_piece_entries_C"] + d["dot_huge_entries"] > 0, d
    sr = ("MIN", "PLUS", "INT64")
    if rows is None:
        ref = O.mxm(C0, G, G, sr, mask=Mc, accum=("PLUS", "INT64"))
        assert np.array_equal(Cg.indptr, ref.indptr)
        assert np.array_equal(Cg.indices, ref.indices)
        assert np.array_equal(Cg.values, ref.values)
        return
    deg = np.diff(G.indptr)
    pick = np.unique(np.concatenate([np.argsort(deg)[-64:],
                                     np.random.default_rng(9).choice(n, rows - 64, replace=False)]))
    Gs, Ms, C0s = _rows_csr(G, pick), _rows_csr(Mc, pick), _rows_csr(C0, pick)
    ref = O.mxm(C0s, Gs, G, sr, mask=Ms, accum=("PLUS", "INT64"))
    Cs = _rows_csr(Cg, pick)
    assert np.array_equal(Cs.indptr, ref.indptr)
    assert np.array_equal(Cs.indices, ref.indices)
    assert np.array_equal(Cs.values, ref.values)


@pytest.mark.parametrize("scale,ef", [(20, 16), (22, 16), (22, 60)])
def test_spmv_plus_times_fp64_bench_scale(gb, scale, ef):
    """config 2's kernel: y = x plus.times A, dense fp64 x (hot-column relabel on by default); ef 60
    is the com-Orkut entry count the bench's second config 2 line stands in for (235 M entries)"""
    import scipy.sparse as sp

    lib = gb.lib
    n = 1 << scale
    A = rmat(lib, scale, "FP64", ef=ef)
    x, y = ctypes.c_void_p(), ctypes.c_void_p()
    xv = np.random.default_rng(1).random(n)
    idx = np.arange(n, dtype=np.uint64)
    try:
        ok(lib.GrB_Vector_new(ctypes.byref(x), lib.GrB_FP64, n), "x")
        ok(lib.GrB_Vector_build_FP64(x, ctypes.c_void_p(idx.ctypes.data), ctypes.c_void_p(xv.ctypes.data), n, None),
           "build x")
        ok(lib.GrB_Vector_new(ctypes.byref(y), lib.GrB_FP64, n), "y")
        for _ in range(2):  # the second call runs on the cached relabel
            ok(lib.GrB_vxm(y, None, None, lib.GrB_PLUS_TIMES_SEMIRING_FP64, x, A, None), "vxm")
        nv = U64()
        ok(lib.GrB_Vector_nvals(ctypes.byref(nv), y), "nvals y")
        yi, yv = np.empty(nv.value, np.uint64), np.empty(nv.value, np.float64)
        ok(lib.GrB_Vector_extractTuples_FP64(ctypes.c_void_p(yi.ctypes.data), ctypes.c_void_p(yv.ctypes.data),
                                             ctypes.byref(nv), y), "extract y")
        G = export(lib, A, n, "FP64")
    finally:
        free(lib, A)
        lib.GrB_Vector_free(ctypes.byref(x))
        lib.GrB_Vector_free(ctypes.byref(y))
    S = sp.csr_matrix((G.values, G.indices, G.indptr), shape=(n, n))
    ref = S.T @ xv
    present = np.diff(S.tocsc().indptr) > 0
    assert np.array_equal(np.sort(yi.astype(np.int64)), np.flatnonzero(present))
    got = np.zeros(n)
    got[yi.astype(np.int64)] = yv
    np.testing.assert_allclose(got, ref, rtol=1e-6, atol=0)


def test_unmasked_spgemm_plus_times_s19_sampled(gb):
    """config 5: C = A plus.times A, fp64, unmasked, R-MAT s19 (the bench's N = 1 line); 512 rows
    (the 32 longest first) vs a numpy fold of the same rows, structure exact, values rtol 1e-6"""
    lib = gb.lib
    scale = 19
    n = 1 << scale
    A = rmat(lib, scale, "FP64")
    C = ctypes.c_void_p()
    Cs = ctypes.c_void_p()
    try:
        G = export(lib, A, n, "FP64")
        deg = np.diff(G.indptr)
        pick = np.unique(np.concatenate([np.argsort(deg)[-32:],
                                         np.random.default_rng(11).choice(n, 480, replace=False)])).astype(np.uint64)
        ok(lib.GrB_Matrix_new(ctypes.byref(C), lib.GrB_FP64, n, n), "C")
        ok(lib.GrB_mxm(C, None, None, lib.GrB_PLUS_TIMES_SEMIRING_FP64, A, A, None), "mxm")
        ok(lib.GrB_Matrix_new(ctypes.byref(Cs), lib.GrB_FP64, len(pick), n), "Cs")
        ok(lib.GrB_Matrix_extract(Cs, None, None, C, ctypes.c_void_p(pick.ctypes.data), len(pick), lib.GrB_ALL, n,
                                  None), "extract rows")
        free(lib, C)
        C = ctypes.c_void_p()
        Cg = export(lib, Cs, len(pick), "FP64", ncols=n)
    finally:
        free(lib, A, C, Cs)
    for k, r in enumerate(pick.astype(np.int64)):
        acc = np.zeros(n)
        present = np.zeros(n, bool)
        for p in range(G.indptr[r], G.indptr[r + 1]):
            kk = G.indices[p]
            s, e = G.indptr[kk], G.indptr[kk + 1]
            acc[G.indices[s:e]] += G.values[p] * G.values[s:e]
            present[G.indices[s:e]] = True
        cols = np.flatnonzero(present)
        gc = Cg.indices[Cg.indptr[k]:Cg.indptr[k + 1]]
        gv = Cg.values[Cg.indptr[k]:Cg.indptr[k + 1]]
        assert np.array_equal(gc, cols), f"row {r}: structure"
        np.testing.assert_allclose(gv, acc[cols], rtol=1e-6, atol=0, err_msg=f"row {r}")
