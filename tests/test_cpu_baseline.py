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
