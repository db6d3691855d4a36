"""Deterministic floating-point accumulation of the hash Gustavson SpGEMM (gb_spgemm_hash.hip):
C = A plus.times A repeated on the same inputs must give the same bits every time, through every
kernel the rows can land in -- the wave table, the workgroup LDS tables (wave-owned slots,
msplit), the column-window kernel with LDS value groups and with C-resident accumulation
(window_vcap / window_in_c_groups).  Values are also checked against the oracle (fold in
ascending k, oracle/gb_oracle.c) at rtol 1e-6, the floating-point tolerance of BASELINE.json's
north_star; how many differ in the last bits is reported, not asserted (ties inside one apply
instruction follow the hardware's lane order)."""
import contextlib
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
import oracle as O  # noqa: E402

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gb():
    import graphblas_amd

    return graphblas_amd


@contextlib.contextmanager
def _knobs(gb, **kv):
    for k, v in kv.items():
        gb.set_knob(k, v)
    try:
        yield
    finally:
        for k in kv:
            gb.set_knob(k, 0)


METHODS = {
    "bins": {},  # wave / workgroup tables for most rows, windows for the hubs
    "window": {"hash_window": 1},  # every row through the column windows (LDS value groups)
    "window_sweep": {"hash_window": 1, "window_bits": 1},  # presence by a product sweep, not stored bitmaps
    "window_in_c": {"hash_window": 1, "window_vcap": 512, "window_in_c_groups": 1},
    # 4 windows of 1024 columns: window ends from the long B rows' window index (round 5), value
    # groups inside a window searched in the row's window slice; and the same without the index
    "window_lw10": {"hash_window": 1, "window_lw": 10},
    "window_lw10_groups": {"hash_window": 1, "window_lw": 10, "window_vcap": 300},
    "window_lw10_noindex": {"hash_window": 1, "window_lw": 10, "window_index": 1},
}


@pytest.mark.parametrize("dt", ["FP64", "FP32"])
@pytest.mark.parametrize("method", list(METHODS))
def test_spgemm_fp_deterministic(gb, method, dt):
    G = O.rmat(12, 16, 3, values="FP64", value_seed=9)
    vals = (G.values * 3.0 - 1.0).astype(O.NP[dt])  # mixed signs: order matters
    G = O.Csr(G.nrows, G.ncols, dt, G.indptr, G.indices, vals)
    r, c, v = G.to_coo()
    A = gb.Matrix.from_coo(r, c, v, dtype=dt, nrows=G.nrows, ncols=G.ncols)
    runs = []
    with _knobs(gb, **METHODS[method]):
        for _ in range(3):
            C = A.mxm(A, gb.semiring.plus_times[dt]).new()
            runs.append(C.to_coo())
    for rr, cc, vv in runs[1:]:
        assert np.array_equal(rr, runs[0][0]) and np.array_equal(cc, runs[0][1])
        assert vv.tobytes() == runs[0][2].tobytes(), "run-to-run bits differ"
    ref = O.mxm(O.Csr.empty(G.nrows, G.ncols, dt), G, G, ("PLUS", "TIMES", dt))
    er, ec, ev = ref.to_coo()
    rr, cc, vv = runs[0]
    assert np.array_equal(rr.astype(np.int64), er) and np.array_equal(cc.astype(np.int64), ec)
    tol = 1e-6 if dt == "FP64" else 1e-3
    np.testing.assert_allclose(vv, ev, rtol=tol, atol=tol * 1e-2 * np.abs(ev).max())
    print(f"{method} {dt}: {int(np.count_nonzero(vv != ev))} of {vv.size} values differ from the "
          f"ascending-k fold in the last bits")
