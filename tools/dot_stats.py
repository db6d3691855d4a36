"""Masked min_plus SpGEMM C<A.S> = A min.+ A on R-MAT: one call with the dot-task statistics on
(knob dot_stats: tasks, piece tasks, X loads per launch) and the entry classes.  Diagnostic."""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "graph-python_amd"))
import graphblas_amd as gb  # noqa: E402

scale = int(sys.argv[1]) if len(sys.argv) > 1 else 20
gb.set_knob("dot_stats", 1)
for kv in sys.argv[2:]:
    k_, v_ = kv.split("=")
    gb.set_knob(k_, int(v_))
lib = gb.lib
A = ctypes.c_void_p()
assert lib.GxB_Matrix_rmat(ctypes.byref(A), scale, 16, 42, 1, 2, 0, 0) == 0
assert lib.GxB_Matrix_prepare_transpose(A) == 0
C = ctypes.c_void_p()
lib.GrB_Matrix_new(ctypes.byref(C), lib.GrB_INT64, 1 << scale, 1 << scale)
names = ["dot_tasks", "dot_piece_tasks", "dot_task_xloads", "dot_task_entries_R", "dot_task_entries_C",
         "dot_piece_entries_R", "dot_piece_entries_C", "dot_hub_chunks_R", "dot_hub_chunks_C", "dot_huge_entries"]


def stats():
    out = {}
    for nm in names:
        c = ctypes.c_int64()
        lib.GxB_Global_get_int(("stat_" + nm).encode(), ctypes.byref(c))
        out[nm] = c.value
    return out


s0 = stats()
assert lib.GrB_mxm(C, A, None, lib.GrB_MIN_PLUS_SEMIRING_INT64, A, A, lib.GrB_DESC_S) == 0
nv = ctypes.c_uint64()
lib.GrB_Matrix_nvals(ctypes.byref(nv), C)
torch.cuda.synchronize()
s1 = stats()
print(f"s{scale}", " ".join(f"{k}={s1[k] - s0[k]}" for k in names))
