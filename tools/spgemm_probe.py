"""Masked min_plus SpGEMM C<A.S> = A min.+ A on R-MAT: time
and GTEPS = sum over mask entries (i,j) of (deg_out(i) + deg_in(j)) / t.  Diagnostic."""
import ctypes
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "graph-python_amd"))
import graphblas_amd as gb  # noqa: E402

scale = int(sys.argv[1]) if len(sys.argv) > 1 else 20
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
for kv in sys.argv[3:]:  # library knobs k=v
    k_, v_ = kv.split("=")
    gb.set_knob(k_, int(v_))
lib = gb.lib
stream = torch.cuda.Stream()
gb.set_stream(stream)
n = 1 << scale
A = ctypes.c_void_p()
assert lib.GxB_Matrix_rmat(ctypes.byref(A), scale, 16, 42, 1, 2, 0, 0) == 0
assert lib.GxB_Matrix_prepare_transpose(A) == 0
nv = ctypes.c_uint64()
lib.GrB_Matrix_nvals(ctypes.byref(nv), A)
nnz = nv.value
ap = np.empty(n + 1, np.uint64)
ai = np.empty(nnz, np.uint64)
ax = np.empty(nnz, np.int64)
lens = [ctypes.c_uint64(n + 1), ctypes.c_uint64(nnz), ctypes.c_uint64(nnz)]
lib.GrB_Matrix_export_INT64(ctypes.c_void_p(ap.ctypes.data), ctypes.c_void_p(ai.ctypes.data),
                            ctypes.c_void_p(ax.ctypes.data), *[ctypes.byref(x) for x in lens], 0, A)
ap = ap.astype(np.int64)
ai = ai.astype(np.int64)
dout = np.diff(ap)
din = np.bincount(ai, minlength=n)
rows = np.repeat(np.arange(n), dout)
work = int((dout[rows] + din[ai]).sum())
sr = lib.GrB_MIN_PLUS_SEMIRING_INT64


def run():
    C = ctypes.c_void_p()  # C = A.mxm(A).new(mask=A.S): a fresh output each call
    lib.GrB_Matrix_new(ctypes.byref(C), lib.GrB_INT64, n, n)
    lib.GrB_mxm(C, A, None, sr, A, A, lib.GrB_DESC_S)
    lib.GrB_Matrix_nvals(ctypes.byref(nv), C)
    lib.GrB_Matrix_free(ctypes.byref(C))
    return nv.value


for g in sys.argv[3:] or ["0"]:
    # "k=v" sets a knob for this measurement, a bare number sets dot_group
    if "=" in g:
        kk, vv = g.split("=")
        gb.set_knob(kk, int(vv))
    else:
        gb.set_knob("dot_group", int(g))
    run()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        nc = run()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    t = min(ts)
    print(f"s{scale} {g}: nnz(A) {nnz} nnz(C) {nc} work {work:.3e} time {t*1e3:.2f} ms "
          f"GTEPS {work / t / 1e9:.2f}  (all: {' '.join(f'{x * 1e3:.2f}' for x in ts)})", flush=True)
