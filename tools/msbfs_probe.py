"""Per-level anatomy of the multi-source BFS (masked GrB_mxm on column words).

usage (GPU box): python tools/msbfs_probe.py [--scale 22] [--k 64] [--knob name=value ...]
Prints, per level, the frontier count and the event-bracketed time of the assign and
of the mxm (a GPU spin is queued first so the events time kernels, not host enqueue),
then the wall time of whole batches.
"""
import argparse
import ctypes
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "graph-python_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=int, default=22)
    ap.add_argument("--k", type=int, default=64)
    ap.add_argument("--knob", action="append", default=[])
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    import torch

    import graphblas_amd as gb

    lib = gb.lib
    for kv in a.knob:
        k, v = kv.split("=")
        gb.set_knob(k, int(v))
    stream = torch.cuda.Stream()
    gb.set_stream(stream)
    A = ctypes.c_void_p()
    assert lib.GxB_Matrix_rmat(ctypes.byref(A), a.scale, 16, 42, 0, 0, 0, 0) == 0
    assert lib.GxB_Matrix_prepare_transpose(A) == 0
    n = 1 << a.scale
    rng = np.random.default_rng(7)
    roots = rng.choice(n, a.k, replace=False).astype(np.uint64)
    qi = np.arange(a.k, dtype=np.uint64)
    Q, V = ctypes.c_void_p(), ctypes.c_void_p()
    assert lib.GrB_Matrix_new(ctypes.byref(Q), lib.GrB_BOOL, a.k, n) == 0
    assert lib.GrB_Matrix_new(ctypes.byref(V), lib.GrB_INT32, a.k, n) == 0
    nv = ctypes.c_uint64()
    sr, desc, ALL = lib.GrB_LOR_LAND_SEMIRING_BOOL, lib.GrB_DESC_RSC, lib.GrB_ALL

    def batch(probe):
        lib.GrB_Matrix_clear(Q)
        lib.GrB_Matrix_clear(V)
        assert lib.GxB_Matrix_build_Scalar_BOOL(Q, ctypes.c_void_p(qi.ctypes.data),
                                                ctypes.c_void_p(roots.ctypes.data), True, a.k) == 0
        d = 0
        rows = []
        while True:
            d += 1
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
            if probe:
                with torch.cuda.stream(stream):
                    torch.cuda._sleep(2_000_000)
                ev[0].record(stream)
            assert lib.GrB_Matrix_assign_INT32(V, Q, None, d, ALL, a.k, ALL, n, None) == 0
            if probe:
                ev[1].record(stream)
            assert lib.GrB_mxm(Q, V, None, sr, Q, A, desc) == 0
            if probe:
                ev[2].record(stream)
            assert lib.GrB_Matrix_nvals(ctypes.byref(nv), Q) == 0
            if probe:
                torch.cuda.synchronize()
                rows.append((d, nv.value, ev[0].elapsed_time(ev[1]) * 1e3, ev[1].elapsed_time(ev[2]) * 1e3))
            if nv.value == 0:
                return rows

    batch(False)
    for d, cnt, ta, tm in batch(True):
        print(f"level {d:2d}  next frontier {cnt:>10d}  assign {ta:8.1f} us  mxm {tm:8.1f} us", flush=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.reps):
        batch(False)
    torch.cuda.synchronize()
    print(f"batch wall {(time.perf_counter() - t0) / a.reps * 1e3:.3f} ms ({a.k} roots, s{a.scale})", flush=True)


if __name__ == "__main__":
    main()
