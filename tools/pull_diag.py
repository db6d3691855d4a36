"""Time one BFS level's GrB_vxm (pull forced) under diagnostic knobs, input restored
each repetition.  usage: pull_diag.py LEVEL [root_idx] [k=v,k=v ...]  (each argument
after root_idx is one variant; knobs in it are set for that variant only).  Diagnostic."""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "graph-python_amd"))
import graphblas_amd as gb  # noqa: E402

level = int(sys.argv[1]) if len(sys.argv) > 1 else 3
root_idx = int(sys.argv[2]) if len(sys.argv) > 2 else 7
variants = sys.argv[3:] or ["iso_dbg=0"]
lib = gb.lib
stream = torch.cuda.Stream()
gb.set_stream(stream)
scale = 22
n = 1 << scale
A = ctypes.c_void_p()
assert lib.GxB_Matrix_rmat(ctypes.byref(A), scale, 16, 42, 0, 0, 0, 0) == 0
assert lib.GxB_Matrix_prepare_transpose(A) == 0
nv = ctypes.c_uint64()
lib.GrB_Matrix_nvals(ctypes.byref(nv), A)
ap = np.empty(n + 1, np.uint64)
ai = np.empty(nv.value, np.uint64)
ax = np.empty(nv.value, np.bool_)
lens = [ctypes.c_uint64(n + 1), ctypes.c_uint64(nv.value), ctypes.c_uint64(nv.value)]
lib.GrB_Matrix_export_BOOL(ctypes.c_void_p(ap.ctypes.data), ctypes.c_void_p(ai.ctypes.data),
                           ctypes.c_void_p(ax.ctypes.data), *[ctypes.byref(x) for x in lens], 0, A)
deg = np.diff(ap.astype(np.int64))
rng = np.random.default_rng(42)
roots = rng.choice(np.flatnonzero(deg > 0), 16, replace=False)
src = int(roots[root_idx])
q = ctypes.c_void_p()
v = ctypes.c_void_p()
lib.GrB_Vector_new(ctypes.byref(q), lib.GrB_BOOL, n)
lib.GrB_Vector_new(ctypes.byref(v), lib.GrB_INT32, n)
lib.GrB_Vector_setElement_BOOL(q, True, src)
for d in range(1, level + 1):
    lib.GrB_Vector_assign_INT32(v, q, None, d, lib.GrB_ALL, n, None)
    if d < level:
        lib.GrB_vxm(q, v, None, lib.GrB_LOR_LAND_SEMIRING_BOOL, q, A, lib.GrB_DESC_RSC)
lib.GrB_Vector_nvals(ctypes.byref(nv), q)
print(f"level {level}: frontier {nv.value}")
gb.set_knob("spmv_direction", 1)
for var in variants:
    kv = [x.split("=") for x in var.split(",")]
    for k_, v_ in kv:
        gb.set_knob(k_, int(v_))
    ts = []
    for rep in range(12):
        qi = ctypes.c_void_p()
        lib.GrB_Vector_dup(ctypes.byref(qi), q)
        lib.GrB_Vector_nvals(ctypes.byref(nv), qi)
        torch.cuda.synchronize()
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        lib.GrB_vxm(qi, v, None, lib.GrB_LOR_LAND_SEMIRING_BOOL, qi, A, lib.GrB_DESC_RSC)
        e1.record(stream)
        lib.GrB_Vector_nvals(ctypes.byref(nv), qi)
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3)
        lib.GrB_Vector_free(ctypes.byref(qi))
    for k_, v_ in kv:
        gb.set_knob(k_, 0)
    print(f"{var:32s} median {np.median(ts[2:]):8.1f} us  min {min(ts[2:]):8.1f}  next {nv.value}", flush=True)
