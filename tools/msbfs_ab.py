"""A/B of the 64-root batched BFS (V<Q.V> = d; Q<!V.S,replace> = Q lor.land A, R-MAT s22) under
library knob settings, interleaved over rounds in one process.
usage: python3 tools/msbfs_ab.py ROUNDS "k=v,k=v" "k=v" ...  ("" = defaults).  Diagnostic."""
import ctypes
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "graph-python_amd"))
import graphblas_amd as gb  # noqa: E402

rounds = int(sys.argv[1])
settings = sys.argv[2:] or [""]
scale, k = 22, 64
lib = gb.lib
stream = torch.cuda.Stream()
gb.set_stream(stream)
A = ctypes.c_void_p()
assert lib.GxB_Matrix_rmat(ctypes.byref(A), scale, 16, 42, 0, 0, 0, 0) == 0
assert lib.GxB_Matrix_prepare_transpose(A) == 0
n = 1 << scale
roots = np.random.default_rng(7).choice(n, k, replace=False).astype(np.uint64)
qi = np.arange(k, dtype=np.uint64)
Q, V = ctypes.c_void_p(), ctypes.c_void_p()
assert lib.GrB_Matrix_new(ctypes.byref(Q), lib.GrB_BOOL, k, n) == 0
assert lib.GrB_Matrix_new(ctypes.byref(V), lib.GrB_INT32, k, n) == 0
nv = ctypes.c_uint64()
sr, desc, ALL = lib.GrB_LOR_LAND_SEMIRING_BOOL, lib.GrB_DESC_RSC, lib.GrB_ALL


def batch():
    lib.GrB_Matrix_clear(Q)
    lib.GrB_Matrix_clear(V)
    assert lib.GxB_Matrix_build_Scalar_BOOL(Q, ctypes.c_void_p(qi.ctypes.data), ctypes.c_void_p(roots.ctypes.data),
                                            True, k) == 0
    d = 0
    while True:
        d += 1
        assert lib.GrB_Matrix_assign_INT32(V, Q, None, d, ALL, k, ALL, n, None) == 0
        assert lib.GrB_mxm(Q, V, None, sr, Q, A, desc) == 0
        assert lib.GrB_Matrix_nvals(ctypes.byref(nv), Q) == 0
        if nv.value == 0:
            break
    assert lib.GrB_Matrix_wait(V, lib.GrB_MATERIALIZE) == 0
    assert lib.GrB_Matrix_nvals(ctypes.byref(nv), V) == 0
    return nv.value


def knobs(setting, on):
    for kv in [s for s in setting.split(",") if s]:
        kk, v = kv.split("=")
        gb.set_knob(kk, int(v) if on else 0)


times = {s: [] for s in settings}
ref = None
for r in range(rounds):
    for st in settings:
        knobs(st, True)
        got = batch()
        ref = got if ref is None else ref
        assert got == ref, (st, got, ref)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(3):
            batch()
        torch.cuda.synchronize()
        times[st].append((time.perf_counter() - t0) / 3 * 1e3)
        knobs(st, False)
for st in settings:
    t = sorted(times[st])
    print(f"[{st or 'defaults'}] 64-root s22 batch: median {t[len(t) // 2]:.3f} ms min {t[0]:.3f}", flush=True)
