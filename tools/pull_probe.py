"""Run BFS levels of one root with a fixed direction (for counter collection on k_iso_work).
usage: pull_probe.py <direction 1=pull 2=push 0=auto> [root index] [reps]"""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "graph-python_amd"))
import graphblas_amd as gb  # noqa: E402

direction = int(sys.argv[1]) if len(sys.argv) > 1 else 1
ridx = int(sys.argv[2]) if len(sys.argv) > 2 else 7
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 1
lib = gb.lib
stream = torch.cuda.Stream()
gb.set_stream(stream)
scale = 22
n = 1 << scale
A = ctypes.c_void_p()
assert lib.GxB_Matrix_rmat(ctypes.byref(A), scale, 16, 42, 0, 0, 0, 0) == 0
assert lib.GxB_Matrix_prepare_transpose(A) == 0
roots = [1840495, 3192592]
src = roots[1] if ridx == 7 else roots[0]
q = ctypes.c_void_p()
v = ctypes.c_void_p()
lib.GrB_Vector_new(ctypes.byref(q), lib.GrB_BOOL, n)
lib.GrB_Vector_new(ctypes.byref(v), lib.GrB_INT32, n)
nv = ctypes.c_uint64()
gb.set_knob("spmv_direction", direction)
for _ in range(reps):
    lib.GrB_Vector_clear(q)
    lib.GrB_Vector_clear(v)
    lib.GrB_Vector_setElement_BOOL(q, True, src)
    d = 0
    while True:
        d += 1
        lib.GrB_Vector_assign_INT32(v, q, None, d, lib.GrB_ALL, n, None)
        lib.GrB_vxm(q, v, None, lib.GrB_LOR_LAND_SEMIRING_BOOL, q, A, lib.GrB_DESC_RSC)
        lib.GrB_Vector_nvals(ctypes.byref(nv), q)
        if nv.value == 0:
            break
torch.cuda.synchronize()
print("levels", d)
