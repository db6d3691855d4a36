"""Fixed cost of one BFS SpMV call: q<!v.S,replace> = q lor.land A with a one-vertex
frontier, R-MAT scales from argv; the kernel time comes from rocprofv3 (run under it)."""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "graph-python_amd"))
import graphblas_amd as gb  # noqa: E402

lib = gb.lib
stream = torch.cuda.Stream()
gb.set_stream(stream)
knobs = [a for a in sys.argv[1:] if "=" in a]
scales = [int(a) for a in sys.argv[1:] if "=" not in a] or [22]
for kv in knobs:
    k, v_ = kv.split("=")
    gb.set_knob(k, int(v_))
for scale in scales:
    n = 1 << scale
    A = ctypes.c_void_p()
    assert lib.GxB_Matrix_rmat(ctypes.byref(A), scale, 16, 42, 0, 0, 0, 0) == 0
    assert lib.GxB_Matrix_prepare_transpose(A) == 0
    q = ctypes.c_void_p()
    v = ctypes.c_void_p()
    lib.GrB_Vector_new(ctypes.byref(q), lib.GrB_BOOL, n)
    lib.GrB_Vector_new(ctypes.byref(v), lib.GrB_INT32, n)
    nv = ctypes.c_uint64()
    for rep in range(50):
        lib.GrB_Vector_clear(q)
        lib.GrB_Vector_clear(v)
        lib.GrB_Vector_setElement_BOOL(q, True, 5)
        lib.GrB_Vector_assign_INT32(v, q, None, 1, lib.GrB_ALL, n, None)
        lib.GrB_vxm(q, v, None, lib.GrB_LOR_LAND_SEMIRING_BOOL, q, A, lib.GrB_DESC_RSC)
        lib.GrB_Vector_nvals(ctypes.byref(nv), q)
    torch.cuda.synchronize()
    print("scale", scale, "next frontier", nv.value, flush=True)
    for h in (A, q, v):
        lib.GrB_Matrix_free(ctypes.byref(h))
