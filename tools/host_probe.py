"""Host-side cost of each C-ABI call in the BFS loop (R-MAT s22): time spent
inside GrB_Vector_assign_INT32 / GrB_vxm / GrB_Vector_nvals per level.  Diagnostic."""
import ctypes
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "graph-python_amd"))
import graphblas_amd as gb  # noqa: E402

scale = int(sys.argv[1]) if len(sys.argv) > 1 else 22
lib = gb.lib
anypair = "anypair" in sys.argv[2:]  # the bench's semiring (default lor_land)
for kv in sys.argv[2:]:  # library knobs k=v
    if "=" not in kv:
        continue
    k_, v_ = kv.split("=")
    gb.set_knob(k_, int(v_))


def stat(key):
    x = ctypes.c_int64()
    lib.GxB_Global_get_int(key.encode(), ctypes.byref(x))
    return x.value


stream = torch.cuda.Stream()
gb.set_stream(stream)
n = 1 << scale
A = ctypes.c_void_p()
assert lib.GxB_Matrix_rmat(ctypes.byref(A), scale, 16, 42, 0, 0, 0, 0) == 0
assert lib.GxB_Matrix_prepare_transpose(A) == 0
q = ctypes.c_void_p()
v = ctypes.c_void_p()
lib.GrB_Vector_new(ctypes.byref(q), lib.GrB_BOOL, n)
lib.GrB_Vector_new(ctypes.byref(v), lib.GrB_INT32, n)
nv = ctypes.c_uint64()
sr = lib.GxB_ANY_PAIR_BOOL if anypair else lib.GrB_LOR_LAND_SEMIRING_BOOL
desc, ALL = lib.GrB_DESC_RSC, lib.GrB_ALL
f_assign, f_vxm, f_nvals = lib.GrB_Vector_assign_INT32, lib.GrB_vxm, lib.GrB_Vector_nvals
tot = {"assign": [], "vxm": [], "nvals": [], "loop": [], "start_clear_q": [], "start_clear_v": [],
       "start_setElement": []}
last = []
sync_start = "nosync" not in sys.argv[2:]  # nosync: BFS after BFS as the bench runs them
for rep in range(20):
    s0 = time.perf_counter()
    lib.GrB_Vector_clear(q)
    s1 = time.perf_counter()
    lib.GrB_Vector_clear(v)
    s2 = time.perf_counter()
    lib.GrB_Vector_setElement_BOOL(q, True, 12345 + rep)
    s3 = time.perf_counter()
    if rep >= 5:
        tot["start_clear_q"].append(s1 - s0)
        tot["start_clear_v"].append(s2 - s1)
        tot["start_setElement"].append(s3 - s2)
    if sync_start:
        torch.cuda.synchronize()
    d = 0
    while True:
        d += 1
        t0 = time.perf_counter()
        f_assign(v, q, None, d, ALL, n, None)
        t1 = time.perf_counter()
        f_vxm(q, v, None, sr, q, A, desc)
        t2 = time.perf_counter()
        f_nvals(ctypes.byref(nv), q)
        t3 = time.perf_counter()
        copies = stat("stat_nvals_copy")
        adopted = stat("stat_bfs_spec_adopted")
        if rep >= 5:
            tot["assign"].append(t1 - t0)
            tot["vxm"].append(t2 - t1)
            tot["nvals"].append(t3 - t2)
        if rep == 19:
            last.append((d, t1 - t0, t2 - t1, t3 - t2, nv.value, copies, adopted))
        if nv.value == 0:
            break
for k, xs in tot.items():
    if xs:
        a = np.array(xs) * 1e6
        print(f"{k:7s} median {np.median(a):7.1f} us  p10 {np.percentile(a, 10):7.1f}  p90 {np.percentile(a, 90):7.1f}  n={a.size}")
print("last BFS per level (us): level assign vxm nvals | frontier  nvals-copies adopted (cumulative)")
for d_, a_, b_, c_, f_, cp_, ad_ in last:
    print(f"  {d_:2d} {a_ * 1e6:7.1f} {b_ * 1e6:7.1f} {c_ * 1e6:7.1f} | {f_:8d} {cp_:6d} {ad_:6d}")
# empty C call for ctypes overhead
t0 = time.perf_counter()
for _ in range(10000):
    lib.GxB_Global_get_int(b"spmv_direction", ctypes.byref(ctypes.c_int64()))
print(f"ctypes round trip: {(time.perf_counter() - t0) / 10000 * 1e6:.2f} us")
