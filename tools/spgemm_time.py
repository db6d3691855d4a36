"""Config-5 SpGEMM (C = A plus.times A, FP64, unmasked, R-MAT) timing under library-knob
settings, interleaved in one process, plus a run-to-run determinism check of C's values.
usage: python3 tools/spgemm_time.py SCALE REPS "k=v,k=v" "k=v" ...   ("" = defaults).
Diagnostic, GPU box."""
import ctypes
import hashlib
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "graph-python_amd"))
import graphblas_amd as gb  # noqa: E402
from graphblas_amd import device as gdev  # noqa: E402

scale, reps = int(sys.argv[1]), int(sys.argv[2])
settings = sys.argv[3:] or [""]
lib = gb.lib
stream = torch.cuda.Stream()
gb.set_stream(stream)
n = 1 << scale
A = ctypes.c_void_p()
assert lib.GxB_Matrix_rmat(ctypes.byref(A), scale, 16, 42, 2, 2, 0, n) == 0
sr = lib.GrB_PLUS_TIMES_SEMIRING_FP64
nv = ctypes.c_uint64()


def knobs(setting, on):
    for kv in [x for x in setting.split(",") if x]:
        k, v = kv.split("=")
        gb.set_knob(k, int(v) if on else 0)


def run(keep=False):
    C = ctypes.c_void_p()
    assert lib.GrB_Matrix_new(ctypes.byref(C), lib.GrB_FP64, n, n) == 0
    assert lib.GrB_mxm(C, None, None, sr, A, A, None) == 0
    assert lib.GrB_Matrix_nvals(ctypes.byref(nv), C) == 0
    if keep:
        return C
    lib.GrB_Matrix_free(ctypes.byref(C))
    return None


def digest(C):
    """order-sensitive checksum of C's arrays, computed on the device in chunks"""
    v = gdev.matrix_view(C)
    acc = []
    for ptr, cnt, ty in ((v.rowptr, n + 1, "<i8"), (v.colidx, v.nvals, "<i4"), (v.values, v.nvals, "<i8")):
        t = gdev.device_tensor(torch, ptr, cnt, ty)
        s1 = torch.zeros((), dtype=torch.int64, device="cuda")
        s2 = torch.zeros((), dtype=torch.int64, device="cuda")
        step = 1 << 27
        for a in range(0, cnt, step):
            x = t[a:a + step].to(torch.int64)
            pos = torch.arange(a, a + x.numel(), device="cuda", dtype=torch.int64)
            s1 += x.sum()
            s2 += ((x ^ (x >> 29)) * (pos * 2 + 1)).sum()
        acc += [int(s1.item()), int(s2.item())]
    return hashlib.sha1(str(acc).encode()).hexdigest()[:16]


res = {s: [] for s in settings}
dig = {s: set() for s in settings}
for s in settings:
    knobs(s, True)
    t0 = time.perf_counter()
    run()
    torch.cuda.synchronize()
    print(f"  [{s or 'defaults'}] first run {(time.perf_counter() - t0) * 1e3:.1f} ms", flush=True)
    knobs(s, False)
torch.cuda.synchronize()
for rnd in range(reps):
    for s in settings:
        knobs(s, True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        run()
        torch.cuda.synchronize()
        res[s].append((time.perf_counter() - t0) * 1e3)
        print(f"  [{s or 'defaults'}] round {rnd}: {res[s][-1]:.1f} ms", flush=True)
        if rnd < 3:
            C = run(keep=True)
            torch.cuda.synchronize()
            dig[s].add(digest(C))
            lib.GrB_Matrix_free(ctypes.byref(C))
        knobs(s, False)
for s in settings:
    t = np.array(res[s])
    print(f"[{s or 'defaults'}] s{scale} nnzC {nv.value} ms median {np.median(t):.1f} min {t.min():.1f} "
          f"| distinct digests over 3 runs: {len(dig[s])} {sorted(dig[s])}", flush=True)
