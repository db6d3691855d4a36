"""Matrix Market ingest (reference graphblas/io/_matrixmarket.py:6-61).
CPU: the native reader (host code, no GPU call) against scipy.io.mmread on the
field/symmetry combinations; GPU: mmread -> device matrix -> to_coo, and an
mmwrite/mmread round trip."""
import numpy as np
import pytest
import scipy.io
import scipy.sparse as sp

from graphblas_amd import io as gio

CASES = {
    "general_real": """%%MatrixMarket matrix coordinate real general
% a comment
4 5 6
1 1 1.5
2 3 -2.25e3
4 5 7
3 1 0.0
1 5 3.125
4 2 1e-3
""",
    "symmetric_integer": """%%MatrixMarket matrix coordinate integer symmetric
3 3 4
1 1 5
2 1 -7
3 2 11
3 3 2
""",
    "skew_real": """%%MatrixMarket matrix coordinate real skew-symmetric
3 3 2
2 1 1.5
3 1 -4
""",
    "pattern_general": """%%MatrixMarket matrix coordinate pattern general
%%
5 5 4
1 2
2 3

5 1
4 4
""",
    "empty": """%%MatrixMarket matrix coordinate real general
3 4 0
""",
}


def _scipy_coo(path):
    m = scipy.io.mmread(path)
    m = sp.coo_matrix(m)
    o = np.lexsort((m.col, m.row))
    return m.shape, m.row[o], m.col[o], m.data[o]


@pytest.mark.parametrize("case", sorted(CASES))
def test_native_reader_matches_scipy(tmp_path, case):
    path = tmp_path / f"{case}.mtx"
    path.write_text(CASES[case])
    nr, nc, r, c, v, dt = gio.read_coo(str(path))
    shape, er, ec, ev = _scipy_coo(str(path))
    assert (nr, nc) == shape
    o = np.lexsort((c, r))
    assert np.array_equal(r[o].astype(np.int64), er) and np.array_equal(c[o].astype(np.int64), ec)
    if dt == "BOOL":
        assert v.all()
    else:
        assert np.array_equal(v[o], ev.astype(v.dtype))


def test_native_reader_large_multithreaded(tmp_path):
    rng = np.random.default_rng(3)
    n, nnz = 5000, 300000
    r = rng.integers(0, n, nnz)
    c = rng.integers(0, n, nnz)
    v = rng.integers(-1000, 1000, nnz)
    path = tmp_path / "big.mtx"
    with open(path, "w") as f:
        f.write(f"%%MatrixMarket matrix coordinate integer general\n{n} {n} {nnz}\n")
        np.savetxt(f, np.column_stack([r + 1, c + 1, v]), fmt="%d %d %d")
    nr, nc, gr, gc, gv, dt = gio.read_coo(str(path))
    assert (nr, nc, dt) == (n, n, "INT64")
    assert np.array_equal(gr.astype(np.int64), r) and np.array_equal(gc.astype(np.int64), c)
    assert np.array_equal(gv, v)


def test_native_reader_rejects_bad(tmp_path):
    path = tmp_path / "bad.mtx"
    path.write_text("%%MatrixMarket matrix coordinate real general\n2 2 1\n3 1 1.0\n")
    with pytest.raises(ValueError):
        gio.read_coo(str(path))
    path.write_text("%%MatrixMarket matrix array real general\n2 2\n1\n2\n3\n4\n")
    with pytest.raises(ValueError):
        gio.read_coo(str(path))


@pytest.mark.gpu
@pytest.mark.parametrize("case", sorted(CASES))
def test_mmread_to_device(tmp_path, case):
    path = tmp_path / f"{case}.mtx"
    path.write_text(CASES[case])
    A = gio.mmread(str(path))
    shape, er, ec, ev = _scipy_coo(str(path))
    r, c, v = A.to_coo()
    assert (A.nrows, A.ncols) == shape
    assert np.array_equal(r.astype(np.int64), er) and np.array_equal(c.astype(np.int64), ec)
    if case.startswith("pattern"):
        assert v.all()
    else:
        assert np.array_equal(v, ev.astype(v.dtype))
    out = tmp_path / "rt.mtx"
    gio.mmwrite(str(out), A)
    B = gio.mmread(str(out))
    assert B.isequal(A)
