"""Per-level timing of the BFS SpMV (GrB_vxm) on R-MAT s22 for one root under each
direction setting (0 auto, 1 pull only, 2 push only).  Diagnostic, run on the GPU box."""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "graph-python_amd"))
import graphblas_amd as gb  # noqa: E402

scale = int(sys.argv[1]) if len(sys.argv) > 1 else 22
root_idx = int(sys.argv[2]) if len(sys.argv) > 2 else 7
for kv in sys.argv[3:]:  # library knobs k=v
    k_, v_ = kv.split("=")
    gb.set_knob(k_, int(v_))
lib = gb.lib
stream = torch.cuda.Stream()
gb.set_stream(stream)
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


def run(direction):
    gb.set_knob("spmv_direction", direction)
    lib.GrB_Vector_clear(q)
    lib.GrB_Vector_clear(v)
    lib.GrB_Vector_setElement_BOOL(q, True, src)
    out = []
    d = 0
    while True:
        d += 1
        lib.GrB_Vector_assign_INT32(v, q, None, d, lib.GrB_ALL, n, None)
        lib.GrB_Vector_nvals(ctypes.byref(nv), q)
        fsz = nv.value
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        lib.GrB_vxm(q, v, None, lib.GrB_LOR_LAND_SEMIRING_BOOL, q, A, lib.GrB_DESC_RSC)
        e1.record(stream)
        lib.GrB_Vector_nvals(ctypes.byref(nv), q)
        torch.cuda.synchronize()
        out.append((d, fsz, e0.elapsed_time(e1) * 1e3, nv.value))
        if nv.value == 0:
            break
    gb.set_knob("spmv_direction", 0)
    return out


for rep in range(2):
    res = {k: run(k) for k in (0, 1, 2)}
print(f"root {src} (index {root_idx}), out-degree {deg[src]}")
print(" lvl  frontier     auto_us     pull_us     push_us   next")
for i in range(len(res[0])):
    d, f, ta, nx = res[0][i]
    tp = res[1][i][2] if i < len(res[1]) else float("nan")  # diagnostic knobs may change the levels
    tu = res[2][i][2] if i < len(res[2]) else float("nan")
    print(f"{d:4d} {f:9d} {ta:11.1f} {tp:11.1f} {tu:11.1f} {nx:7d}")
