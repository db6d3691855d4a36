"""Unmasked plus_times fp64 SpGEMM C = A plus.times A on R-MAT (SURVEY §8d config 5 kernel,
one GPU): time, flops, nnz(C), GFLOP-rate.  Diagnostic; knobs as key=value args."""
import ctypes
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "graph-python_amd"))
import graphblas_amd as gb  # noqa: E402

scales = [int(s) for s in sys.argv[1].split(",")] if len(sys.argv) > 1 else [16]
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
for kv in sys.argv[3:]:
    k, v = kv.split("=")
    gb.set_knob(k, int(v))
lib = gb.lib
stream = torch.cuda.Stream()
gb.set_stream(stream)
nv = ctypes.c_uint64()
sr = lib.GrB_PLUS_TIMES_SEMIRING_FP64
for scale in scales:
    n = 1 << scale
    A = ctypes.c_void_p()
    assert lib.GxB_Matrix_rmat(ctypes.byref(A), scale, 16, 42, 2, 2, 0, 0) == 0
    torch.cuda.synchronize()  # the generator ran on the library stream
    lib.GrB_Matrix_nvals(ctypes.byref(nv), A)
    nnz = nv.value
    from graphblas_amd import device as gdev
    v = gdev.matrix_view(A)
    rp = gdev.device_tensor(torch, v.rowptr, n + 1)
    ci = gdev.device_tensor(torch, v.colidx, nnz, "<i4")
    deg = rp[1:] - rp[:-1]
    flops = int(deg[ci.long()].sum().item())

    def run():
        C = ctypes.c_void_p()
        lib.GrB_Matrix_new(ctypes.byref(C), lib.GrB_FP64, n, n)
        assert lib.GrB_mxm(C, None, None, sr, A, A, None) == 0
        lib.GrB_Matrix_nvals(ctypes.byref(nv), C)
        lib.GrB_Matrix_free(ctypes.byref(C))
        return nv.value

    run()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        nc = run()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    t = min(ts)
    print(f"s{scale}: nnz(A) {nnz} flops {flops:.3e} nnz(C) {nc} ({nc / max(flops, 1):.3f} of flops) "
          f"time {t * 1e3:.2f} ms  {flops / t / 1e9:.2f} GFLOP/s(products)", flush=True)
    lib.GrB_Matrix_free(ctypes.byref(A))
