"""A/B of config 2's SpMV (y = x plus.times A, dense fp64 x, R-MAT SCALE ef EF) under library
knob settings, interleaved over rounds in one process; checks every setting's y against the
first's.  usage: python3 tools/spmv_ab.py SCALE EF ROUNDS "k=v,k=v" "k=v" ...  Diagnostic."""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "graph-python_amd"))
import graphblas_amd as gb  # noqa: E402

scale, ef, rounds = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
settings = sys.argv[4:] or [""]
lib = gb.lib
stream = torch.cuda.Stream()
gb.set_stream(stream)
n = 1 << scale
A = ctypes.c_void_p()
assert lib.GxB_Matrix_rmat(ctypes.byref(A), scale, ef, 42, 2, 2, 0, 0) == 0
assert lib.GxB_Matrix_prepare_transpose(A) == 0
x = gb.Vector.from_coo(np.arange(n), np.random.default_rng(1).random(n), dtype=gb.FP64, size=n)
sr = lib.GrB_PLUS_TIMES_SEMIRING_FP64
y = ctypes.c_void_p()
lib.GrB_Vector_new(ctypes.byref(y), lib.GrB_FP64, n)


def knobs(setting, on):
    for kv in [s for s in setting.split(",") if s]:
        k, v = kv.split("=")
        gb.set_knob(k, int(v) if on else 0)


def result():
    vals = np.empty(n, np.float64)
    idx = np.empty(n, np.uint64)
    cnt = ctypes.c_uint64(n)
    lib.GrB_Vector_extractTuples_FP64(ctypes.c_void_p(idx.ctypes.data), ctypes.c_void_p(vals.ctypes.data),
                                      ctypes.byref(cnt), y)
    return idx[:cnt.value].copy(), vals[:cnt.value].copy()


times = {s: [] for s in settings}
ref = None
for r in range(rounds):
    for st in settings:
        knobs(st, True)
        for _ in range(2):
            lib.GrB_vxm(y, None, None, sr, x._h, A, None)
        torch.cuda.synchronize()
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        with torch.cuda.stream(stream):
            torch.cuda._sleep(200000)
        e0.record(stream)
        for _ in range(10):
            lib.GrB_vxm(y, None, None, sr, x._h, A, None)
        e1.record(stream)
        torch.cuda.synchronize()
        times[st].append(e0.elapsed_time(e1) / 10 * 1e3)
        if r == 0:
            got = result()
            if ref is None:
                ref = got
            else:
                assert np.array_equal(ref[0], got[0]) and np.allclose(ref[1], got[1], rtol=1e-12, atol=1e-12), st
        knobs(st, False)
for st in settings:
    t = sorted(times[st])
    print(f"[{st or 'defaults'}] s{scale} ef{ef}: median {t[len(t) // 2]:.1f} us min {t[0]:.1f}", flush=True)
