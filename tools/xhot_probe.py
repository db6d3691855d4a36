"""Config-2 SpMV (y = x plus.times A, dense fp64 x, R-MAT) with and without the hot-column
relabel (gb_view_hot) and with several hot-set sizes; event-timed on the library stream.
usage: python3 tools/xhot_probe.py SCALE EF [HOT_COLS ...].  Diagnostic, GPU box."""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "graph-python_amd"))
import graphblas_amd as gb  # noqa: E402

scale = int(sys.argv[1]) if len(sys.argv) > 1 else 22
ef = int(sys.argv[2]) if len(sys.argv) > 2 else 16
hots = [int(a) for a in sys.argv[3:]] or [1 << 18, 1 << 19, 1 << 20]
lib = gb.lib
stream = torch.cuda.Stream()
gb.set_stream(stream)
n = 1 << scale
A0 = ctypes.c_void_p()
assert lib.GxB_Matrix_rmat(ctypes.byref(A0), scale, ef, 42, 2, 2, 0, 0) == 0
assert lib.GxB_Matrix_prepare_transpose(A0) == 0
nv = ctypes.c_uint64()
lib.GrB_Matrix_nvals(ctypes.byref(nv), A0)
nnz = nv.value
x = gb.Vector.from_coo(np.arange(n), np.random.default_rng(1).random(n), dtype=gb.FP64, size=n)
sr = lib.GrB_PLUS_TIMES_SEMIRING_FP64


def timed(A, reps=20):
    y = ctypes.c_void_p()
    lib.GrB_Vector_new(ctypes.byref(y), lib.GrB_FP64, n)
    for _ in range(3):
        lib.GrB_vxm(y, None, None, sr, x._h, A, None)
    torch.cuda.synchronize()
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    with torch.cuda.stream(stream):
        torch.cuda._sleep(200000)
    e0.record(stream)
    for _ in range(reps):
        lib.GrB_vxm(y, None, None, sr, x._h, A, None)
    e1.record(stream)
    torch.cuda.synchronize()
    t = e0.elapsed_time(e1) / 1e3 / reps
    vals = np.empty(n, np.float64)
    idx = np.empty(n, np.uint64)
    cnt = ctypes.c_uint64(n)
    lib.GrB_Vector_extractTuples_FP64(ctypes.c_void_p(idx.ctypes.data), ctypes.c_void_p(vals.ctypes.data),
                                      ctypes.byref(cnt), y)
    lib.GrB_Vector_free(ctypes.byref(y))
    return t, idx[:cnt.value].copy(), vals[:cnt.value].copy()


by = 12 * nnz + 8 * (n + 1) + 16 * n
gb.set_knob("xhot", 1)
t0, i0, v0 = timed(A0)
print(f"s{scale} ef{ef} nnz {nnz}: plain colidx {t0*1e6:8.1f} us  {by/t0/1e9:6.0f} GB/s", flush=True)
gb.set_knob("xhot", 0)
for h in hots:
    gb.set_knob("xhot_cols", h)
    A = ctypes.c_void_p()
    assert lib.GrB_Matrix_dup(ctypes.byref(A), A0) == 0
    assert lib.GxB_Matrix_prepare_transpose(A) == 0
    t, i1, v1 = timed(A)
    same = np.array_equal(i0, i1) and np.allclose(v0, v1, rtol=1e-12, atol=1e-12)
    print(f"  hot {h:8d}: {t*1e6:8.1f} us  {by/t/1e9:6.0f} GB/s  x{t0/t:4.2f}  match {same}", flush=True)
    lib.GrB_Matrix_free(ctypes.byref(A))
