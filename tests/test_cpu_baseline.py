"""The multi-threaded CPU baseline BFS (oracle or_bfs_levels_par, bench.py's
cpu_baseline) gives the same levels and edge counts as the sequential oracle loop."""
import numpy as np
import scipy.sparse as sp

import oracle as O


def _transpose(A):
    S = sp.csr_matrix((np.ones(A.indices.size, np.bool_), A.indices, A.indptr), shape=(A.nrows, A.ncols))
    T = S.T.tocsr()
    T.sort_indices()
    return O.Csr(A.ncols, A.nrows, "BOOL", T.indptr, T.indices, np.ones(T.indices.size, np.bool_))


def test_par_bfs_matches_sequential_rmat():
    A = O.rmat(14, 16, 42)
    AT = _transpose(A)
    deg = np.diff(A.indptr)
    for src in np.flatnonzero(deg > 0)[:: max(1, int((deg > 0).sum()) // 6)][:6]:
        ref, nl, e = O.bfs_levels(A, int(src))
        for nt in (1, 4):
            got, nl2, e2 = O.bfs_levels_par(A, AT, int(src), nt)
            assert np.array_equal(got, ref) and nl2 == nl and e2 == e


def test_par_bfs_push_only_and_isolated_root():
    rng = np.random.default_rng(3)
    n = 300
    S = sp.random(n, n, density=0.01, random_state=rng, format="csr")
    S.sort_indices()
    A = O.Csr(n, n, "BOOL", S.indptr, S.indices, np.ones(S.indices.size, np.bool_))
    for src in (0, 17, 299):
        ref, nl, e = O.bfs_levels(A, src)
        got, nl2, e2 = O.bfs_levels_par(A, None, src, 3)  # no A^T: push every level
        assert np.array_equal(got, ref) and nl2 == nl and e2 == e


def _transpose_vals(A):
    S = sp.csr_matrix((A.values, A.indices, A.indptr), shape=(A.nrows, A.ncols))
    T = S.T.tocsr()
    T.sort_indices()
    return O.Csr(A.ncols, A.nrows, A.dtype, T.indptr, T.indices, T.data)


def test_masked_dot_cpu_baseline_matches_oracle():
    """bench.py config-4 cpu_baseline: or_masked_dot_min_plus_int64_par == or_mxm (bit-exact)"""
    A = O.rmat(11, 16, 42, values="INT64", value_seed=2)
    AT = _transpose_vals(A)
    ref = O.mxm(O.Csr.empty(A.nrows, A.ncols, "INT64"), A, A, ("MIN", "PLUS", "INT64"), mask=A, mask_struct=True)
    for r0, r1, nt in ((0, A.nrows, 4), (100, 900, 1)):
        vals, present, nc, work = O.masked_dot_min_plus_int64_par(A, AT, r0, r1, nt)
        rows = np.repeat(np.arange(A.nrows), np.diff(A.indptr))[A.indptr[r0]:A.indptr[r1]]
        cols = A.indices[A.indptr[r0]:A.indptr[r1]]
        rr = np.repeat(np.arange(A.nrows), np.diff(ref.indptr))
        sel = (rr >= r0) & (rr < r1)
        key_ref = rr[sel] * A.ncols + ref.indices[sel]
        key_got = rows[present] * A.ncols + cols[present]
        assert nc == int(present.sum()) and np.array_equal(key_got, key_ref)
        assert np.array_equal(vals[present], ref.values[sel])
        dout, din = np.diff(A.indptr), np.diff(AT.indptr)
        assert work == int((dout[rows] + din[cols]).sum())


def test_spmv_cpu_baseline_matches_scipy():
    """bench.py config-2 cpu_baseline: or_spmv_plus_times_fp64_par == scipy A^T x"""
    A = O.rmat(12, 16, 42, values="FP64", value_seed=2)
    AT = _transpose_vals(A)
    x = np.random.default_rng(1).random(A.nrows)
    y, present = O.spmv_plus_times_fp64_par(AT, x, 4)
    S = sp.csr_matrix((A.values, A.indices, A.indptr), shape=(A.nrows, A.ncols))
    assert np.array_equal(present, np.diff(AT.indptr) > 0)
    assert np.allclose(y, S.T @ x, rtol=1e-12, atol=0)


def test_spgemm_cpu_baseline_matches_oracle():
    """bench.py config-5 cpu_baseline: or_spgemm_plus_times_fp64_par == or_mxm (same ascending-k
    fold: bit-identical), on the whole matrix and on a row range"""
    A = O.rmat(10, 8, 42, values="FP64", value_seed=2)
    ref = O.mxm(O.Csr.empty(A.nrows, A.ncols, "FP64"), A, A, ("PLUS", "TIMES", "FP64"))
    deg = np.diff(A.indptr)
    for r0, r1, nt in ((0, A.nrows, 4), (200, 700, 1), (5, 5, 2)):
        C, prods = O.spgemm_plus_times_fp64_par(A, A, r0, r1, nt)
        p0, p1 = ref.indptr[r0], ref.indptr[r1]
        assert np.array_equal(C.indptr, ref.indptr[r0:r1 + 1] - p0)
        assert np.array_equal(C.indices, ref.indices[p0:p1])
        assert np.array_equal(C.values, ref.values[p0:p1])
        assert prods == int(deg[A.indices[A.indptr[r0]:A.indptr[r1]]].sum())
