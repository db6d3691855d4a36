"""Sweep launch-grid knobs of the BFS path on R-MAT s22; prints ms per BFS for each setting.  Diagnostic."""
import ctypes
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "graph-python_amd"))
import graphblas_amd as gb  # noqa: E402

lib = gb.lib
stream = torch.cuda.Stream()
gb.set_stream(stream)
scale = 22
n = 1 << scale
A = ctypes.c_void_p()
assert lib.GxB_Matrix_rmat(ctypes.byref(A), scale, 16, 42, 0, 0, 0, 0) == 0
assert lib.GxB_Matrix_prepare_transpose(A) == 0
q = ctypes.c_void_p()
v = ctypes.c_void_p()
lib.GrB_Vector_new(ctypes.byref(q), lib.GrB_BOOL, n)
lib.GrB_Vector_new(ctypes.byref(v), lib.GrB_INT32, n)
nv = ctypes.c_uint64()
roots = [1840495, 3192592, 12345, 777777, 2000001, 99]


def bfs(src):
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
            return


def timeit():
    for r in roots:
        bfs(r)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(3):
        for r in roots:
            bfs(r)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / (3 * len(roots)) * 1e3


for knob in sys.argv[1:]:
    name, vals = knob.split("=")
    for val in vals.split(","):
        gb.set_knob(name, int(val))
        print(f"{name}={val}: {timeit():.3f} ms/BFS", flush=True)
    gb.set_knob(name, 0)
