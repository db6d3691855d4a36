"""plus_times FP64 SpMV y = x plus.times A (vxm, dense x) on R-MAT (SURVEY §8d config 2's
kernel on a synthetic graph): time, GTEPS = nnz/t, HBM GB/s of 12*nnz + 8(n+1) + 16n bytes."""
import ctypes
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "graph-python_amd"))
import graphblas_amd as gb  # noqa: E402

scale = int(sys.argv[1]) if len(sys.argv) > 1 else 22
ef = int(sys.argv[2]) if len(sys.argv) > 2 else 16
lib = gb.lib
stream = torch.cuda.Stream()
gb.set_stream(stream)
if os.environ.get("SPMV_NO_X_GATHER"):  # timing experiment: x treated as iso (wrong values)
    gb.set_knob("spmv_timing_no_x_gather", 1)
if os.environ.get("SPMV_WORDS"):  # 1: segmented-scan words kernel instead of merge path
    gb.set_knob("spmv_words", int(os.environ["SPMV_WORDS"]))
n = 1 << scale
A = ctypes.c_void_p()
assert lib.GxB_Matrix_rmat(ctypes.byref(A), scale, ef, 42, 2, 2, 0, 0) == 0
assert lib.GxB_Matrix_prepare_transpose(A) == 0
nv = ctypes.c_uint64()
lib.GrB_Matrix_nvals(ctypes.byref(nv), A)
nnz = nv.value
x = gb.Vector.from_coo(np.arange(n), np.random.default_rng(1).random(n), dtype=gb.FP64, size=n)
y = ctypes.c_void_p()
lib.GrB_Vector_new(ctypes.byref(y), lib.GrB_FP64, n)
sr = lib.GrB_PLUS_TIMES_SEMIRING_FP64
for lgk in [0] + [int(a) for a in sys.argv[3:]]:
    gb.set_knob("spmv_lg", lgk)
    for _ in range(2):
        lib.GrB_vxm(y, None, None, sr, x._h, A, None)
    torch.cuda.synchronize()
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    reps = 20
    with torch.cuda.stream(stream):
        torch.cuda._sleep(200000)
    e0.record(stream)
    for _ in range(reps):
        lib.GrB_vxm(y, None, None, sr, x._h, A, None)
    e1.record(stream)
    torch.cuda.synchronize()
    t = e0.elapsed_time(e1) / 1e3 / reps
    by = 12 * nnz + 8 * (n + 1) + 16 * n
    print(f"s{scale} ef{ef} spmv_lg={lgk}: nnz {nnz} time {t*1e6:.1f} us GTEPS {nnz/t/1e9:.1f} "
          f"HBM {by/t/1e9:.0f} GB/s", flush=True)
