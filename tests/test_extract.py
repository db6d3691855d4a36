"""GrB_Matrix_extract / GrB_Col_extract / GrB_Vector_extract (gb_extract.hip) and the
SuiteSparse index-list encodings python-graphblas passes for slices (GxB_RANGE,
GxB_STRIDE, GxB_BACKWARDS; reference core/slice.py:10-49), against numpy on seeded
random inputs -- index/byte work, so exact.  Also the index-list assign w(I) = u without
accumulator, which replaces the region (entries of w at I that u lacks are deleted)."""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

RANGE, STRIDE, BACKWARDS = 2**63 - 1, 2**63 - 2, 2**63 - 3


@pytest.fixture(scope="module")
def gb():
    import graphblas_amd

    return graphblas_amd


def _rand_matrix(gb, rng, m, n, density, dtype="INT64"):
    have = rng.random((m, n)) < density
    vals = rng.integers(-50, 50, (m, n))
    r, c = np.nonzero(have)
    A = gb.Matrix.from_coo(r, c, vals[r, c], dtype=dtype, nrows=m, ncols=n)
    return A, have, vals


def _dense(x, shape):
    have = np.zeros(shape, bool)
    vals = np.zeros(shape, np.int64)
    if len(shape) == 2:
        r, c, v = x.to_coo()
        have[r.astype(np.int64), c.astype(np.int64)] = True
        vals[r.astype(np.int64), c.astype(np.int64)] = v
    else:
        i, v = x.to_coo()
        have[i.astype(np.int64)] = True
        vals[i.astype(np.int64)] = v
    return have, vals


@pytest.mark.parametrize("seed", range(6))
@pytest.mark.parametrize("transpose", [False, True])
def test_matrix_extract_vs_numpy(gb, seed, transpose):
    rng = np.random.default_rng(seed)
    m, n = 37, 53
    A, have, vals = _rand_matrix(gb, rng, m, n, 0.2)
    if transpose:
        have, vals = have.T, vals.T
    M_, N_ = have.shape
    # index lists with duplicates and any order, a strided slice, and all
    I = rng.integers(0, M_, 23)
    J = [rng.integers(0, N_, 31), np.arange(N_)[3:40:3], slice(None)][seed % 3]
    src = A.T.new() if transpose else A  # GrB_transpose, then extract
    if isinstance(J, slice):
        C = src[I, :].new()
        Jl = np.arange(N_)
    else:
        C = src[I, J].new()
        Jl = J
    exp_have, exp_vals = have[np.ix_(I, Jl)], vals[np.ix_(I, Jl)]
    gh, gv = _dense(C, exp_have.shape)
    assert np.array_equal(gh, exp_have)
    assert np.array_equal(gv[gh], exp_vals[exp_have])


def test_matrix_extract_transposed_desc_mask_accum(gb):
    """C<M> += A'(I, J) through the C ABI with GrB_DESC_T0 / GrB_DESC_RT0 (mask + accum)"""
    rng = np.random.default_rng(11)
    A, have, vals = _rand_matrix(gb, rng, 40, 30, 0.3)
    I = rng.integers(0, 30, 12).astype(np.uint64)
    J = rng.permutation(40)[:17].astype(np.uint64)
    Ch, Cv = rng.random((12, 17)) < 0.4, rng.integers(1, 9, (12, 17))
    Mh = rng.random((12, 17)) < 0.5
    cr, cc = np.nonzero(Ch)
    C = gb.Matrix.from_coo(cr, cc, Cv[cr, cc], dtype="INT64", nrows=12, ncols=17)
    mr, mc = np.nonzero(Mh)
    M = gb.Matrix.from_coo(mr, mc, True, nrows=12, ncols=17)
    lib = gb.lib
    rc = lib.GrB_Matrix_extract(C._h, M._h, gb.binary.plus["INT64"]._carg, A._h, ctypes.c_void_p(I.ctypes.data),
                                I.size, ctypes.c_void_p(J.ctypes.data), J.size, lib.GrB_DESC_RT0)
    assert rc == 0
    Th, Tv = have.T[np.ix_(I, J)], vals.T[np.ix_(I, J)]
    # Z = C plus T on the union; C<M, replace> = Z
    Zh = Ch | Th
    Zv = np.where(Ch & Th, Cv + Tv, np.where(Th, Tv, Cv))
    exp_h = Zh & Mh
    gh, gv = _dense(C, (12, 17))
    assert np.array_equal(gh, exp_h)
    assert np.array_equal(gv[gh], Zv[exp_h])


@pytest.mark.parametrize("row", [False, True])
def test_col_extract_vs_numpy(gb, row):
    rng = np.random.default_rng(5 + row)
    A, have, vals = _rand_matrix(gb, rng, 45, 45, 0.25)
    for j in (0, 7, 44):
        I = rng.integers(0, 45, 19)
        w = (A[j, I] if row else A[I, j]).new()
        eh = have[j, I] if row else have[I, j]
        ev = vals[j, I] if row else vals[I, j]
        gh, gv = _dense(w, (19,))
        assert np.array_equal(gh, eh) and np.array_equal(gv[gh], ev[eh])
        w = (A[j, :] if row else A[:, j]).new()
        eh = have[j, :] if row else have[:, j]
        gh, gv = _dense(w, (45,))
        assert np.array_equal(gh, eh) and np.array_equal(gv[gh], (vals[j, :] if row else vals[:, j])[eh])


def test_vector_extract_vs_numpy(gb):
    rng = np.random.default_rng(3)
    n = 300
    h = rng.random(n) < 0.3
    x = rng.integers(-9, 9, n)
    v = gb.Vector.from_coo(np.flatnonzero(h), x[h], dtype="INT64", size=n)
    for I in (rng.integers(0, n, 77), np.arange(n)[::-7], np.arange(n)[250:10:-3]):
        w = v[I].new()
        gh, gv = _dense(w, (len(I),))
        assert np.array_equal(gh, h[I]) and np.array_equal(gv[gh], x[I][h[I]])
    iso = gb.Vector.from_coo(np.flatnonzero(h), True, size=n)  # iso values stay iso
    w = iso[np.arange(0, n, 2)].new()
    gh, gv = _dense(w, (n // 2,))
    assert np.array_equal(gh, h[::2]) and np.all(gv[gh] == 1)


def test_index_encodings_through_abi(gb):
    """GxB_RANGE [b, e], GxB_STRIDE [b, e, inc], GxB_BACKWARDS [b, e, dec] (bounds inclusive) in
    GrB_Vector_extract and GrB_Vector_assign_INT64, as SuiteSparse 7.4 defines them"""
    lib = gb.lib
    n = 50
    v = gb.Vector.from_coo(np.arange(n), np.arange(n) * 10, dtype="INT64", size=n)
    cases = [(RANGE, [5, 12], list(range(5, 13))), (STRIDE, [3, 40, 7], list(range(3, 41, 7))),
             (BACKWARDS, [45, 20, 6], list(range(45, 19, -6))), (RANGE, [9, 8], [])]
    for ni, spec, expect in cases:
        I = np.array(spec, np.uint64)
        w = gb.Vector("INT64", len(expect))
        assert lib.GrB_Vector_extract(w._h, None, None, v._h, ctypes.c_void_p(I.ctypes.data), ni, None) == 0
        i, x = w.to_coo()
        assert i.tolist() == list(range(len(expect))) and x.tolist() == [10 * e for e in expect]
        u = gb.Vector("INT64", n)
        assert lib.GrB_Vector_assign_INT64(u._h, None, None, 7, ctypes.c_void_p(I.ctypes.data), ni, None) == 0
        i, x = u.to_coo()
        assert i.tolist() == sorted(expect) and np.all(x == 7)
    # out of range: an error, not a fault
    I = np.array([40, 60], np.uint64)
    w = gb.Vector("INT64", 21)
    assert lib.GrB_Vector_extract(w._h, None, None, v._h, ctypes.c_void_p(I.ctypes.data), RANGE, None) == \
        -105  # GrB_INDEX_OUT_OF_BOUNDS


def test_vector_index_assign_replaces_region(gb):
    """w(I) = u with no accum: inside I, w becomes u (entries u lacks are deleted); outside I, w is
    kept (C API 2.0 GrB_assign); with a mask only the selected part of the region changes"""
    n = 12
    w = gb.Vector.from_coo(np.arange(n), np.arange(n) + 100, dtype="INT64", size=n)
    u = gb.Vector.from_coo([0, 2], [-1, -3], dtype="INT64", size=4)
    w[[1, 3, 5, 7]] = u  # region {1, 3, 5, 7}: 1 <- -1, 5 <- -3, 3 and 7 deleted
    i, x = w.to_coo()
    exp = {k: k + 100 for k in range(n) if k not in (3, 7)}
    exp.update({1: -1, 5: -3})
    assert dict(zip(i.tolist(), x.tolist())) == exp
    w2 = gb.Vector.from_coo(np.arange(n), np.arange(n) + 100, dtype="INT64", size=n)
    m = gb.Vector.from_coo([3, 5], True, size=n)
    w2(m.S)[[1, 3, 5, 7]] = u  # only 3 (deleted) and 5 (set) are selected
    i, x = w2.to_coo()
    exp = {k: k + 100 for k in range(n) if k != 3}
    exp[5] = -3
    assert dict(zip(i.tolist(), x.tolist())) == exp
    w3 = gb.Vector.from_coo(np.arange(n), np.arange(n) + 100, dtype="INT64", size=n)
    w3(gb.binary.plus)[[1, 3, 5, 7]] = u  # accum: nothing deleted
    i, x = w3.to_coo()
    exp = {k: k + 100 for k in range(n)}
    exp[1] += -1
    exp[5] += -3
    assert dict(zip(i.tolist(), x.tolist())) == exp
    # the mask aliases the output: the mask is w as it was before the call (the region clear must
    # not remove the selected positions from it before u is written back)
    keep = [k for k in range(n) if k != 5]
    w4 = gb.Vector.from_coo(keep, np.array(keep) + 100, dtype="INT64", size=n)
    w4(w4.S)[[1, 3, 5, 7]] = u  # selected: 1 (<- -1), 3, 7 (deleted); 5 is outside the mask
    i, x = w4.to_coo()
    exp = {k: k + 100 for k in keep if k not in (3, 7)}
    exp[1] = -1
    assert dict(zip(i.tolist(), x.tolist())) == exp
    vals = np.arange(n) + 100
    vals[1] = 0
    w5 = gb.Vector.from_coo(np.arange(n), vals, dtype="INT64", size=n)
    w5(w5.V)[[1, 3, 5, 7]] = u  # value mask: 1 holds 0, so it is not selected and keeps its 0
    i, x = w5.to_coo()
    exp = {k: int(vals[k]) for k in range(n) if k not in (3, 7)}
    exp[5] = -3
    assert dict(zip(i.tolist(), x.tolist())) == exp
