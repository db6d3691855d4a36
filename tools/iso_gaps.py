"""Kernel gaps of the bench's level BFS without a profiler: the library stamps each k_iso_work
launch's start and end on the device wall clock (s_memrealtime, 100 MHz) when
GRAPHBLAS_AMD_ISO_TS names a dump file (csrc/gb_mxv.hip iso_ts_mark).  Runs bench.py's timed
loop shape (16 seeded roots on R-MAT s22, any_pair, warm-up first) and prints, per BFS, the
launches, the summed launch durations and the summed idle gaps between them, then the
averages.  Diagnostic only (tools/)."""
import ctypes
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "graph-python_amd"))
path = os.path.join(ROOT, "gpurun_out", "iso_ts.bin")
os.makedirs(os.path.dirname(path), exist_ok=True)
os.environ["GRAPHBLAS_AMD_ISO_TS"] = path
import torch  # noqa: E402,F401

import graphblas_amd as gb  # noqa: E402

scale = int(sys.argv[1]) if len(sys.argv) > 1 else 22
for kv in sys.argv[2:]:
    k_, v_ = kv.split("=")
    gb.set_knob(k_, int(v_))
lib = gb.lib
stream = torch.cuda.Stream()
gb.set_stream(stream)
n = 1 << scale
A = ctypes.c_void_p()
assert lib.GxB_Matrix_rmat(ctypes.byref(A), scale, 16, 42, 0, 0, 0, 0) == 0
assert lib.GxB_Matrix_prepare_transpose(A) == 0
ap = np.empty(n + 1, np.uint64)
nv = ctypes.c_uint64()
lib.GrB_Matrix_nvals(ctypes.byref(nv), A)
ai = np.empty(nv.value, np.uint64)
ax = np.empty(nv.value, np.bool_)
lens = [ctypes.c_uint64(n + 1), ctypes.c_uint64(nv.value), ctypes.c_uint64(nv.value)]
assert lib.GrB_Matrix_export_BOOL(ctypes.c_void_p(ap.ctypes.data), ctypes.c_void_p(ai.ctypes.data),
                                  ctypes.c_void_p(ax.ctypes.data), *[ctypes.byref(x) for x in lens], 0, A) == 0
deg = np.diff(ap.astype(np.int64))
roots = np.random.default_rng(42).choice(np.flatnonzero(deg > 0), 16, replace=False)
q, v = ctypes.c_void_p(), ctypes.c_void_p()
lib.GrB_Vector_new(ctypes.byref(q), lib.GrB_BOOL, n)
lib.GrB_Vector_new(ctypes.byref(v), lib.GrB_INT32, n)
sr, desc, ALL = lib.GxB_ANY_PAIR_BOOL, lib.GrB_DESC_RSC, lib.GrB_ALL


def bfs(src):
    lib.GrB_Vector_clear(q)
    lib.GrB_Vector_clear(v)
    lib.GrB_Vector_setElement_BOOL(q, True, int(src))
    d = 0
    while True:
        d += 1
        lib.GrB_Vector_assign_INT32(v, q, None, d, ALL, n, None)
        lib.GrB_vxm(q, v, None, sr, q, A, desc)
        lib.GrB_Vector_nvals(ctypes.byref(nv), q)
        if nv.value == 0:
            return d


for s in range(3):
    bfs(roots[s % 16])
torch.cuda.synchronize()
c = ctypes.c_int64()
lib.GxB_Global_get_int(b"iso_ts_dump", ctypes.byref(c))
n_warm = c.value
t0 = time.perf_counter()
levels = [bfs(roots[s]) for s in range(16)]
torch.cuda.synchronize()
wall = (time.perf_counter() - t0) / 16
lib.GxB_Global_get_int(b"iso_ts_dump", ctypes.byref(c))
raw = np.fromfile(path, np.uint64)
k = c.value
st = raw[2::2][:k].astype(np.int64)
en = raw[3::2][:k].astype(np.int64)
st, en = st[n_warm:], en[n_warm:]
dur = (en - st) / 100.0  # us
gap = (st[1:] - en[:-1]) / 100.0
print(f"wall per BFS {wall * 1e6:.1f} us over 16 roots; {len(st)} launches ({len(st) / 16:.2f} per BFS)")
print(f"launch durations (start of block 0 -> publish) per BFS {dur.sum() / 16:.1f} us; gaps per BFS "
      f"{gap.sum() / 16:.1f} us (incl. the other kernels, e.g. k_vec_set, and launch latency)")
# per-BFS listing: the speculation adds one launch per BFS (levels + 1)
i = 0
for b, L in enumerate(levels[:4]):
    m = L + 1
    seg_d = dur[i:i + m]
    seg_g = gap[i:i + m] if i + m <= len(gap) else gap[i:]
    print(f"BFS {b}: " + " ".join(f"[{dg:5.1f}|{dd:5.1f}]" for dd, dg in zip(seg_d, np.concatenate([[0.0], seg_g])[:m])))
    i += m
