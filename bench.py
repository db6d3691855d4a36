#!/usr/bin/env python3
"""Benchmark: masked GrB_vxm level-BFS on R-MAT scale 22 (BASELINE.json configs[2];
the metric "GTEPS + achieved HBM GB/s, masked mxm/mxv on R-MAT s22").

One step = one full level-synchronous BFS from one of 16 seeded roots, exactly
the reference notebook loop (notebooks/Example B.1 -- Level BFS.ipynb cell 8):
    v<q.V>[:] = d ;  q<!v.S, replace> = q lor.land A ;  stop when q is empty
issued through the C ABI of libgraphblas_amd.so (GrB_Vector_assign_INT32,
GrB_vxm with GrB_DESC_RSC, GrB_Vector_nvals).  The graph is generated on the
device (GxB_Matrix_rmat) and its CSC cache is built before timing (ingest).

value  = GTEPS = sum over BFS of edges in the reached component / time (all ranks).
roofline: dominant kernel = the masked pull SpMV (k_spmv_pull), timed with HIP
events on the library's stream; algorithmic bytes per BFS = SURVEY §8(d):
4*nnz + 8*(n+1) + L*3*ceil(n/8).
cpu_baseline: the oracle's GraphBLAS-loop BFS (oracle/gb_oracle.c or_bfs_graphblas)
on a bounded sample of roots, single host thread.

Multi-GPU (torchrun): the vertex set is split into 64-aligned blocks, rank r owns
rows [lo,hi) of A^T (generated directly, GxB_Matrix_rmat transposed shard) and
computes its slice of the next frontier with GrB_mxv; the frontier bitmap is
all-gathered over RCCL each level (the path's only exchange step).
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "graph-python_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

PEAK_HBM_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=16)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--scale", type=int, default=22)
    p.add_argument("--edge-factor", type=int, default=16)
    p.add_argument("--seed", type=int, default=42)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-seconds", type=float, default=15.0)
    p.add_argument("--traffic-file", default=os.path.join(ROOT, "profiles", "traffic_r01.json"))
    return p.parse_args()


class Lib:
    def __init__(self):
        import graphblas_amd as gb

        self.gb = gb
        self.lib = gb.lib
        self.h = {}

    def __getattr__(self, name):
        return getattr(self.lib, name)

    def ok(self, rc, what):
        if rc != 0:
            raise RuntimeError(f"{what} failed with GrB_Info {rc}")


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    import torch

    dist = None
    if world > 1:
        import torch.distributed as dist

        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
    else:
        torch.cuda.set_device(0)
    os.environ["GRAPHBLAS_AMD_DEVICE"] = str(local_rank)
    L = Lib()
    gb = L.gb
    stream = torch.cuda.Stream()
    L.ok(L.GxB_Context_set_device(local_rank), "set_device")
    gb.set_stream(stream)

    scale, n = args.scale, 1 << args.scale
    # 64-aligned vertex blocks per rank
    words = (n + 63) // 64
    lo_w = words * rank // world
    hi_w = words * (rank + 1) // world
    lo, hi = lo_w * 64, min(n, hi_w * 64)

    # ---------------- graph (ingest, untimed)
    A = ctypes.c_void_p()
    t0 = time.time()
    if world == 1:
        L.ok(L.GxB_Matrix_rmat(ctypes.byref(A), scale, args.edge_factor, args.seed, 0, 0, 0, 0), "rmat")
        L.ok(L.GxB_Matrix_prepare_transpose(A), "transpose")
    else:
        # rows [lo,hi) of A^T (values flag 0x100 = generate the transpose)
        L.ok(L.GxB_Matrix_rmat(ctypes.byref(A), scale, args.edge_factor, args.seed, 0x100, 0, lo, hi),
             "rmat shard")
    torch.cuda.synchronize()
    nnz_local = ctypes.c_uint64()
    L.ok(L.GrB_Matrix_nvals(ctypes.byref(nnz_local), A), "nvals")
    ingest_s = time.time() - t0

    # out-degrees for the TEPS edge count (host, untimed): export the CSR row pointers
    if world == 1:
        view = gb._lib.ctypes.c_void_p
    # degree array of the full graph: each rank computes the degrees of its rows of A (not A^T)
    deg = None
    if world == 1:
        nr = ctypes.c_uint64(n + 1)
        ni = ctypes.c_uint64(nnz_local.value)
        nx = ctypes.c_uint64(nnz_local.value)
        ap = np.empty(n + 1, np.uint64)
        ai = np.empty(nnz_local.value, np.uint64)
        ax = np.empty(nnz_local.value, np.bool_)
        L.ok(L.GrB_Matrix_export_BOOL(ctypes.c_void_p(ap.ctypes.data), ctypes.c_void_p(ai.ctypes.data),
                                      ctypes.c_void_p(ax.ctypes.data), ctypes.byref(nr), ctypes.byref(ni),
                                      ctypes.byref(nx), 0, A), "export")
        deg = np.diff(ap.astype(np.int64))
        host_csr = (ap.astype(np.int64), ai.astype(np.int64))
        del ax
    rng = np.random.default_rng(args.seed)
    # 16 roots with out-degree > 0 (Graph500 convention); same on every rank
    if world == 1:
        cand = np.flatnonzero(deg > 0)
        roots = rng.choice(cand, 16, replace=False)
    else:
        roots = rng.integers(0, n, 64)

    sr = L.GrB_LOR_LAND_SEMIRING_BOOL
    desc = L.GrB_DESC_RSC
    grb_all = L.GrB_ALL

    # ---------------- single-GPU BFS through the C ABI
    q = ctypes.c_void_p()
    v = ctypes.c_void_p()
    nloc = hi - lo
    L.ok(L.GrB_Vector_new(ctypes.byref(q), L.GrB_BOOL, n), "q")
    L.ok(L.GrB_Vector_new(ctypes.byref(v), L.GrB_INT32, nloc), "v")
    qloc = ctypes.c_void_p()
    if world > 1:
        L.ok(L.GrB_Vector_new(ctypes.byref(qloc), L.GrB_BOOL, nloc), "qloc")
        gath = torch.empty(words if world == 1 else (hi_w - lo_w) * world, dtype=torch.int64, device="cuda")
    nv = ctypes.c_uint64()
    ev_pairs = []
    level_counts = []

    def bfs(src, timing):
        L.ok(L.GrB_Vector_clear(q), "clear q")
        L.ok(L.GrB_Vector_clear(v), "clear v")
        L.ok(L.GrB_Vector_setElement_BOOL(q, True, int(src)), "q[src]")
        d = 0
        while True:
            d += 1
            if world == 1:
                L.ok(L.GrB_Vector_assign_INT32(v, q, None, d, grb_all, n, None), "assign")
                if timing:
                    e0 = torch.cuda.Event(enable_timing=True)
                    e1 = torch.cuda.Event(enable_timing=True)
                    e0.record(stream)
                L.ok(L.GrB_vxm(q, v, None, sr, q, A, desc), "vxm")
                if timing:
                    e1.record(stream)
                    ev_pairs.append((e0, e1))
                L.ok(L.GrB_Vector_nvals(ctypes.byref(nv), q), "nvals")
                if nv.value == 0:
                    break
            else:
                L.ok(L.GxB_Vector_slice_assign_INT32(v, q, d, lo), "assign shard")
                if timing:
                    e0 = torch.cuda.Event(enable_timing=True)
                    e1 = torch.cuda.Event(enable_timing=True)
                    e0.record(stream)
                L.ok(L.GrB_mxv(qloc, v, None, sr, A, q, desc), "mxv")
                if timing:
                    e1.record(stream)
                    ev_pairs.append((e0, e1))
                # all-gather the frontier bitmap (the path's only exchange)
                part = gath.narrow(0, rank * (hi_w - lo_w), hi_w - lo_w)
                L.ok(L.GxB_Vector_bitmap_export(qloc, ctypes.c_void_p(part.data_ptr()), hi_w - lo_w), "bm out")
                with torch.cuda.stream(stream):
                    dist.all_gather_into_tensor(gath, part.clone())
                L.ok(L.GxB_Vector_bitmap_import(q, ctypes.c_void_p(gath.data_ptr()), words), "bm in")
                L.ok(L.GrB_Vector_nvals(ctypes.byref(nv), q), "nvals")
                if nv.value == 0:
                    break
        level_counts.append(d)
        return d

    # verification + edge counts (untimed): GPU levels == oracle levels on root 0
    edges = []
    import oracle as O

    if world == 1:
        for src in roots:
            bfs(src, False)
            nvl = ctypes.c_uint64()
            L.ok(L.GrB_Vector_nvals(ctypes.byref(nvl), v), "nvals v")
            idx = np.empty(nvl.value, np.uint64)
            lv = np.empty(nvl.value, np.int32)
            L.ok(L.GrB_Vector_extractTuples_INT32(ctypes.c_void_p(idx.ctypes.data), ctypes.c_void_p(lv.ctypes.data),
                                                  ctypes.byref(nvl), v), "extract")
            edges.append(int(deg[idx.astype(np.int64)].sum()))
            if src == roots[0]:
                G = O.Csr(n, n, "BOOL", host_csr[0], host_csr[1], np.ones(host_csr[1].size, np.bool_))
                lev_ref, _, _ = O.bfs_levels(G, int(src))
                got = np.zeros(n, np.int32)
                got[idx.astype(np.int64)] = lv
                parity = bool(np.array_equal(got, lev_ref))
                if not parity:
                    raise SystemExit("BFS parity failure vs oracle")
    level_counts.clear()

    for w in range(args.warmup):
        bfs(roots[w % len(roots)], False)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    ev_pairs.clear()
    level_counts.clear()
    t0 = time.perf_counter()
    for s in range(args.steps):
        bfs(roots[s % len(roots)], True)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if dist:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    kern_ms = sum(a.elapsed_time(b) for a, b in ev_pairs)
    launches = len(ev_pairs)

    if rank != 0:
        dist.destroy_process_group()
        return
    total_edges = sum(edges[s % len(roots)] for s in range(args.steps)) if edges else None
    gteps = total_edges / elapsed / 1e9 if total_edges else None
    nnz = nnz_local.value
    levels_total = sum(level_counts)
    alg_bytes = args.steps * (4 * nnz + 8 * (n + 1)) + levels_total * 3 * ((n + 7) // 8)
    achieved = alg_bytes / (kern_ms / 1e3) / 1e9 if kern_ms > 0 else None
    traffic = None
    if os.path.exists(args.traffic_file):
        try:
            traffic = json.load(open(args.traffic_file)).get("bytes_per_launch")
        except Exception:
            traffic = None

    cpu = None
    if not args.no_cpu_baseline and world == 1:
        G = O.Csr(n, n, "BOOL", host_csr[0], host_csr[1], np.ones(host_csr[1].size, np.bool_))
        lev = np.zeros(n, np.int32)
        e = ctypes.c_int64()
        done_edges, t_cpu, runs = 0, 0.0, 0
        for src in roots:
            t1 = time.perf_counter()
            O.lib().or_bfs_graphblas(ctypes.byref(G._c()), ctypes.c_int64(int(src)),
                                     lev.ctypes.data_as(ctypes.c_void_p), ctypes.byref(e))
            t_cpu += time.perf_counter() - t1
            done_edges += e.value
            runs += 1
            if t_cpu > args.cpu_seconds:
                break
        cpu = {"value": done_edges / t_cpu / 1e9, "unit": "GTEPS", "cores": 1, "kind": "port",
               "sample": f"{runs} full BFS runs (notebook GraphBLAS loop via or_mxm) on the same "
                         f"R-MAT s{scale} graph, {t_cpu:.1f} s, single host thread"}

    out = {
        "metric": "GTEPS (masked mxv level-BFS, R-MAT s22)",
        "value": gteps,
        "unit": "GTEPS",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "bool",
        "data": "synthetic (Graph500 R-MAT, a,b,c,d=.57,.19,.19,.05, generated on device, seed 42)",
        "config": {"workload": f"level-BFS q<!v.S,replace> = q lor.land A on R-MAT scale {scale}, "
                               f"edge factor {args.edge_factor}, 16 roots",
                   "n": n, "nnz": nnz, "parallelism": f"row-sharded x{world}" if world > 1 else "single GPU"},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                     "frac": achieved / PEAK_HBM_GBS if achieved else None, "traffic": traffic,
                     "kernel": "k_spmv_pull (GrB_vxm)", "kernel_ms_total": kern_ms, "launches": launches,
                     "alg_bytes": alg_bytes},
        "cpu_baseline": cpu,
        "ingest_s": ingest_s,
    }
    print(json.dumps(out))
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
