"""A/B timing of the headline BFS loop (bench.py's notebook loop, any_pair, R-MAT s22, 16
roots) under several library-knob settings, interleaved in one process so box-to-box and
drift noise cancel.  usage: python3 tools/ab_bfs.py SCALE ROUNDS "k=v,k=v" "k=v" ...
("" = defaults).  Prints per setting: median and min ms per BFS over the rounds, and the
per-level minimum event-bracketed SpMV time of root 7.  Diagnostic, GPU box."""
import ctypes
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "graph-python_amd"))
import graphblas_amd as gb  # noqa: E402

scale = int(sys.argv[1])
rounds = int(sys.argv[2])
settings = sys.argv[3:] or [""]
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
roots = np.random.default_rng(42).choice(np.flatnonzero(deg > 0), 16, replace=False)
q, v = ctypes.c_void_p(), ctypes.c_void_p()
lib.GrB_Vector_new(ctypes.byref(q), lib.GrB_BOOL, n)
lib.GrB_Vector_new(ctypes.byref(v), lib.GrB_INT32, n)
sr = lib.GxB_ANY_PAIR_BOOL


def apply(setting):
    for kv in [s for s in setting.split(",") if s]:
        k, val = kv.split("=")
        gb.set_knob(k, int(val))


def reset(setting):
    for kv in [s for s in setting.split(",") if s]:
        gb.set_knob(kv.split("=")[0], 0)


def bfs(src, ev=None):
    lib.GrB_Vector_clear(q)
    lib.GrB_Vector_clear(v)
    lib.GrB_Vector_setElement_BOOL(q, True, int(src))
    d = 0
    while True:
        d += 1
        lib.GrB_Vector_assign_INT32(v, q, None, d, lib.GrB_ALL, n, None)
        if ev is not None:
            with torch.cuda.stream(stream):
                torch.cuda._sleep(100000)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
        lib.GrB_vxm(q, v, None, sr, q, A, lib.GrB_DESC_RSC)
        if ev is not None:
            e1.record(stream)
            ev.append((e0, e1))
        lib.GrB_Vector_nvals(ctypes.byref(nv), q)
        if nv.value == 0:
            return d


res = {s: [] for s in settings}
lev = {s: [] for s in settings}
for s in settings:  # warm-up (builds the caches of each setting)
    apply(s)
    for r in roots[:4]:
        bfs(r)
    reset(s)
torch.cuda.synchronize()
for rnd in range(rounds):
    for s in settings:
        apply(s)
        t0 = time.perf_counter()
        for r in roots:
            bfs(r)
        res[s].append((time.perf_counter() - t0) / len(roots) * 1e3)
        ev = []
        bfs(roots[7], ev)
        torch.cuda.synchronize()
        lev[s].append([a.elapsed_time(b) * 1e3 for a, b in ev])
        reset(s)
for s in settings:
    t = np.array(res[s])
    per = np.array(lev[s]).min(axis=0)
    print(f"[{s or 'defaults'}] ms/BFS median {np.median(t):.4f} min {t.min():.4f} | root7 levels us "
          + " ".join(f"{x:.1f}" for x in per), flush=True)
