"""Fixed cost of one BFS-step SpMV (GrB_vxm, any_pair, R-MAT s22, RSC mask) on a tiny frontier:
GPU time per call (HIP events, GPU kept busy ahead) under library-knob settings, e.g. the
k_iso_work diagnostics iso_dbg = 1 (count by copy), 4 (no direction phase), 8 (empty kernel).
usage: python3 tools/iso_probe.py SCALE "k=v,k=v" ...  Diagnostic, GPU box."""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "graph-python_amd"))
import graphblas_amd as gb  # noqa: E402

scale = int(sys.argv[1])
settings = sys.argv[2:] or [""]
lib = gb.lib
stream = torch.cuda.Stream()
gb.set_stream(stream)
n = 1 << scale
A = ctypes.c_void_p()
assert lib.GxB_Matrix_rmat(ctypes.byref(A), scale, 16, 42, 0, 0, 0, 0) == 0
assert lib.GxB_Matrix_prepare_transpose(A) == 0
q, v, w = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_void_p()
lib.GrB_Vector_new(ctypes.byref(q), lib.GrB_BOOL, n)
lib.GrB_Vector_new(ctypes.byref(v), lib.GrB_INT32, n)
lib.GrB_Vector_new(ctypes.byref(w), lib.GrB_BOOL, n)
src = 12345
lib.GrB_Vector_setElement_BOOL(q, True, src)
lib.GrB_Vector_setElement_INT32(v, 1, src)
sr = lib.GxB_ANY_PAIR_BOOL
nv = ctypes.c_uint64()


def knobs(s, on):
    for kv in [x for x in s.split(",") if x]:
        k, val = kv.split("=")
        gb.set_knob(k, int(val) if on else 0)


for s in settings:
    knobs(s, True)
    ts = []
    for rep in range(40):
        with torch.cuda.stream(stream):
            torch.cuda._sleep(100000)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        lib.GrB_vxm(w, v, None, sr, q, A, lib.GrB_DESC_RSC)
        e1.record(stream)
        lib.GrB_Vector_nvals(ctypes.byref(nv), w)
        torch.cuda.synchronize()
        if rep >= 5:
            ts.append(e0.elapsed_time(e1) * 1e3)
    knobs(s, False)
    print(f"[{s or 'defaults'}] us median {np.median(ts):.1f} min {np.min(ts):.1f}  nvals {nv.value}", flush=True)
