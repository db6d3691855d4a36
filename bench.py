#!/usr/bin/env python3
"""Benchmark: masked GrB_vxm / GrB_mxv level-BFS on R-MAT scale 22 (BASELINE.json
configs[2]; the metric "GTEPS + achieved HBM GB/s, masked mxm/mxv on R-MAT s22").

One step = one full level-synchronous BFS from one of 16 seeded roots, exactly
the reference notebook loop (notebooks/Example B.1 -- Level BFS.ipynb cell 8):
    v<q.V>[:] = d ;  q<!v.S, replace> = q any.pair A ;  stop when q is empty
with BASELINE.json configs[2]'s semiring any_pair[BOOL] = GxB_ANY_PAIR_BOOL (the notebook
writes lor_land; `--semiring lor_land` swaps them, and the other one is reported as a
secondary line), issued through the C ABI of libgraphblas_amd.so (GrB_Vector_assign_INT32,
GrB_vxm with GrB_DESC_RSC, GrB_Vector_nvals).  The graph is generated on the
device (GxB_Matrix_rmat) and its CSC cache is built before timing (ingest).

value  = GTEPS = edges of the reached component, summed over the K timed BFS,
         / wall time of the K BFS (max over ranks).
value is total edges / wall time; gteps_harmonic_mean is Graph500's per-root
harmonic mean.  roofline: the dominant op is the masked SpMV (GrB_vxm: the
k_dir_prep + k_iso_work launches), timed with HIP events on the library's
stream in a separate pass after the timed region (one BFS per root);
algorithmic bytes per BFS = SURVEY §8(d) config 3: 4*nnz + 8*(n+1) +
L*3*ceil(n/8), divided evenly over the BFS's L launches.
cpu_baseline: the oracle's GraphBLAS-loop BFS (oracle/gb_oracle.c
or_bfs_graphblas) on a bounded sample of the same roots, one host thread.

Multi-GPU (torchrun): vertices split into 64-aligned blocks; rank r owns rows
[lo,hi) of A^T (generated directly as a transposed shard) and computes its slice
of the next frontier with GrB_mxv (q_r<!v_r.S,replace> = A^T_r lor.land q);
the frontier bitmap (n/8 bytes) is all-gathered over RCCL each level -- the
path's only exchange step.  Total work is fixed (strong scaling).
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np
import scipy.sparse as sp

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "graph-python_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

PEAK_HBM_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level table)
SLEEP_CYCLES = 100000  # ~40 us GPU spin ahead of each timed SpMV in the roofline pass


def _profile_rounds():
    """the rounds with a committed headline traffic file (profiles/traffic_rNN.json), newest first"""
    import glob
    import re

    rs = set()
    for f in glob.glob(os.path.join(ROOT, "profiles", "traffic_r*.json")):
        m = re.match(r"traffic_(r\d+)\.json$", os.path.basename(f))
        if m:
            rs.add(m.group(1))
    return sorted(rs, key=lambda r: int(r[1:]), reverse=True)


ROUNDS = _profile_rounds()
CUR_ROUND = ROUNDS[0] if ROUNDS else "r00"


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=16)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--scale", type=int, default=22)
    p.add_argument("--edge-factor", type=int, default=16)
    p.add_argument("--seed", type=int, default=42)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-secondary", action="store_true", help="skip the config 2 / config 4 lines")
    p.add_argument("--no-msbfs", action="store_true", help="skip the multi-source (masked mxm) BFS line")
    p.add_argument("--no-msbfs-sharded", action="store_true",
                   help="N > 1: skip the row-sharded 64-root BFS line (one exchange per level for 64 roots)")
    p.add_argument("--cpu-seconds", type=float, default=15.0)
    p.add_argument("--traffic-file", default=os.path.join(ROOT, "profiles", f"traffic_{CUR_ROUND}.json"))
    # rehearsal of the N>1 path on one GPU: all ranks on one device, gloo transport
    p.add_argument("--dist-backend", default="nccl")
    p.add_argument("--no-pipeline", action="store_true",
                   help="N > 1: wait for each level's count before enqueuing the next (round-4 loop)")
    p.add_argument("--exchange", default="peer", choices=["allgather", "peer"],
                   help="N > 1 BFS frontier exchange: host-issued all-gather (RCCL / gloo), or device-initiated "
                        "writes into IPC-mapped peer windows (GxB_PeerWindow_*, no collective per level)")
    p.add_argument("--partition", default="balanced", choices=["balanced", "equal"],
                   help="N > 1 BFS: vertex ranges balanced by the shards' entries, or equal word slots")
    p.add_argument("--device", type=int, default=None, help="override LOCAL_RANK's device")
    p.add_argument("--knob", action="append", default=[], help="library knob key=value (ablations)")
    p.add_argument("--semiring", default="any_pair", choices=["any_pair", "lor_land"],
                   help="BFS semiring: any_pair (BASELINE.json configs[2]) or lor_land (the notebook's)")
    p.add_argument("--cpu-secondary-seconds", type=float, default=8.0,
                   help="bound of each secondary line's CPU-baseline sample")
    p.add_argument("--spgemm-scale", type=int, default=19, help="config 5 (unmasked fp64 SpGEMM) R-MAT scale")
    p.add_argument("--spgemm-steps", type=int, default=2)
    p.add_argument("--spgemm-warmup", type=int, default=1)
    p.add_argument("--no-spgemm", action="store_true", help="skip the config 5 line")
    p.add_argument("--spgemm-scale-big", type=int, default=20,
                   help="a second config 5 line at this scale (the largest that fits one GPU); 0 skips")
    p.add_argument("--spgemm-extra", default="21:2,22:4",
                   help="more config 5 lines, scale:min_gpus comma-separated (BASELINE.md:35: s21/s22)")
    p.add_argument("--spgemm-partition", default="products", choices=["products", "equal"],
                   help="N > 1 config 5: row ranges balanced by Gustavson products, or equal word slots")
    return p.parse_args()


def ok(rc, what):
    if rc != 0:
        raise RuntimeError(f"{what} failed with GrB_Info {rc}")


def export_csr(lib, A, nrows):
    nv = ctypes.c_uint64()
    ok(lib.GrB_Matrix_nvals(ctypes.byref(nv), A), "nvals")
    nz = nv.value
    ap = np.empty(nrows + 1, np.uint64)
    ai = np.empty(nz, np.uint64)
    ax = np.empty(nz, np.bool_)
    lens = [ctypes.c_uint64(nrows + 1), ctypes.c_uint64(nz), ctypes.c_uint64(nz)]
    ok(lib.GrB_Matrix_export_BOOL(ctypes.c_void_p(ap.ctypes.data), ctypes.c_void_p(ai.ctypes.data),
                                  ctypes.c_void_p(ax.ctypes.data), *[ctypes.byref(x) for x in lens], 0, A),
       "export")
    return ap.astype(np.int64), ai.astype(np.int64)


def vector_indices(lib, v):
    nv = ctypes.c_uint64()
    ok(lib.GrB_Vector_nvals(ctypes.byref(nv), v), "nvals")
    idx = np.empty(nv.value, np.uint64)
    lv = np.empty(nv.value, np.int32)
    ok(lib.GrB_Vector_extractTuples_INT32(ctypes.c_void_p(idx.ctypes.data), ctypes.c_void_p(lv.ctypes.data),
                                          ctypes.byref(nv), v), "extract")
    return idx.astype(np.int64), lv

def _time_calls(torch, stream, fn, reps):
    """GPU time per call of fn (HIP events on the library stream, GPU kept busy ahead)."""
    fn()
    torch.cuda.synchronize()
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    with torch.cuda.stream(stream):
        torch.cuda._sleep(SLEEP_CYCLES)
    e0.record(stream)
    for _ in range(reps):
        fn()
    e1.record(stream)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / 1e3 / reps


def _bfs_semiring(lib, args):
    """any_pair[BOOL] -> GxB_ANY_PAIR_BOOL (BASELINE.json configs[2]; reference semiring.py:174-203),
    lor_land[BOOL] -> GrB_LOR_LAND_SEMIRING_BOOL (the notebook's, Example B.1 cell 8)"""
    return lib.GxB_ANY_PAIR_BOOL if args.semiring == "any_pair" else lib.GrB_LOR_LAND_SEMIRING_BOOL


def _threads():
    """all of this box's host cores given to the job (OMP_NUM_THREADS; the machine's count otherwise)"""
    return int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)


def _profile_traffic(*stems):
    """HBM bytes per call of the newest round's committed per-workload profile
    profiles/rNN_<stem> (tools/pmc_passes.sh + tools/pmc_table.py + tools/pmc_percall.py:
    2 x FETCH_SIZE + WRITE_SIZE summed over the call's kernels); the stems are tried in order
    within a round, and older rounds only when the newest has none of them."""
    for name in [f"{r}_{st}" for r in ROUNDS for st in stems]:
        path = os.path.join(ROOT, "profiles", name)
        try:
            return json.load(open(path))["hbm_bytes_per_call"], f"profiles/{name}"
        except Exception:
            continue
    return None, None


def _roofline(alg_bytes, seconds, traffic=None, source=None, kernel=None):
    ach = alg_bytes / seconds / 1e9
    r = {"bound": "hbm", "achieved": ach, "peak": PEAK_HBM_GBS, "unit": "GB/s", "frac": ach / PEAK_HBM_GBS,
         "traffic": traffic, "alg_bytes": alg_bytes}
    if source:
        r["traffic_source"] = source
    if kernel:
        r["kernel"] = kernel
    return r


def _sym_transpose(O, n, indptr, indices, values, dtype):
    S = sp.csr_matrix((values, indices, indptr), shape=(n, n))
    T = S.T.tocsr()
    T.sort_indices()
    return O.Csr(n, n, dtype, T.indptr, T.indices, T.data)


def secondary_workloads(lib, torch, stream, O, args):
    """SURVEY 8(d) configs 2 and 4 on one GPU, reported beside the headline BFS line:
    * config 2's kernel: y = x plus.times A, fp64, dense x (vxm) -- on R-MAT s22 (com-Orkut is
      not available here); parity vs scipy (fp64, rtol 1e-6);
    * config 4: C<A.S> = A min.plus A, INT64 weights in [1,255], R-MAT s20; parity vs the oracle
      on a sample of 256 rows (bit-exact)."""
    import scipy.sparse as sp

    out = {}
    # ---- config 2 kernel: plus_times fp64 SpMV, R-MAT s22 at edge factor 16 (the BFS graph)
    # and at edge factor 60 (nnz 235M: com-Orkut's nnz, 234M, whose file is not available)
    out["config2_spmv_plus_times_fp64"] = config2_spmv(lib, torch, stream, args, args.scale, args.edge_factor, O,
                                                       cpu=True)
    out["config2_spmv_plus_times_fp64_orkut_nnz"] = config2_spmv(lib, torch, stream, args, args.scale, 60)
    # ---- config 4: masked min_plus SpGEMM, R-MAT s20 (configs[3]) and s22 (north_star's target)
    for s4 in (20, 22):
        out[f"config4_masked_spgemm_min_plus_int64_s{s4}"] = config4_masked_spgemm(lib, torch, stream, O, args, s4,
                                                                                   cpu=True)
    return out


def config3_msbfs(lib, torch, stream, O, args, A, n, ap, ai, deg, roots16):
    """Config 3's workload as a masked GrB_mxm: K level BFSs at once (LAGraph's multi-source
    form of the reference notebook loop), Q and V K x n:
        V<Q.V> = d;  Q<!V.S, replace> = Q lor.land A;  until Q.nvals == 0
    K = 64 roots (the 16 headline roots first), R-MAT s22, timed from a fresh Q to the last
    nvals.  GTEPS = sum over the K roots of the edges incident to each root's reached set
    (the headline's convention) / time.  Parity: rows of V vs the oracle's level BFS."""
    K = 64
    rng = np.random.default_rng(args.seed + 1)
    pool = np.setdiff1d(np.flatnonzero(deg > 0), roots16)
    roots = np.concatenate([roots16, rng.choice(pool, K - len(roots16), replace=False)]).astype(np.uint64)
    Q, V = ctypes.c_void_p(), ctypes.c_void_p()
    ok(lib.GrB_Matrix_new(ctypes.byref(Q), lib.GrB_BOOL, K, n), "Q")
    ok(lib.GrB_Matrix_new(ctypes.byref(V), lib.GrB_INT32, K, n), "V")
    qi = np.arange(K, dtype=np.uint64)
    nv = ctypes.c_uint64()
    sr, desc, grb_all = _bfs_semiring(lib, args), lib.GrB_DESC_RSC, lib.GrB_ALL

    def batch():
        ok(lib.GrB_Matrix_clear(Q), "clear Q")
        ok(lib.GrB_Matrix_clear(V), "clear V")
        # iso build (one scalar for every entry), as from_coo(rows, cols, True) issues it
        ok(lib.GxB_Matrix_build_Scalar_BOOL(Q, ctypes.c_void_p(qi.ctypes.data), ctypes.c_void_p(roots.ctypes.data),
                                            True, K), "build Q")
        d = 0
        while True:
            d += 1
            ok(lib.GrB_Matrix_assign_INT32(V, Q, None, d, grb_all, K, grb_all, n, None), "V<Q> = d")
            ok(lib.GrB_mxm(Q, V, None, sr, Q, A, desc), "Q<!V.S> = Q lor.land A")
            ok(lib.GrB_Matrix_nvals(ctypes.byref(nv), Q), "nvals")
            if nv.value == 0:
                # the level stamps are pending work on V's column words: materialise its
                # values inside the timed batch
                ok(lib.GrB_Matrix_wait(V, lib.GrB_MATERIALIZE), "wait V")
                return d

    levels = batch()
    # parity + edge counts (untimed): extract V
    ok(lib.GrB_Matrix_nvals(ctypes.byref(nv), V), "nvals V")
    m = nv.value
    vi = np.empty(m, np.uint64)
    vj = np.empty(m, np.uint64)
    vx = np.empty(m, np.int32)
    cnt = ctypes.c_uint64(m)
    ok(lib.GrB_Matrix_extractTuples_INT32(ctypes.c_void_p(vi.ctypes.data), ctypes.c_void_p(vj.ctypes.data),
                                          ctypes.c_void_p(vx.ctypes.data), ctypes.byref(cnt), V), "extract V")
    vi, vj = vi.astype(np.int64), vj.astype(np.int64)
    edges = int(np.bincount(vi, weights=deg[vj], minlength=K).sum())
    G = O.Csr(n, n, "BOOL", ap, ai, np.ones(ai.size, np.bool_))
    parity = True
    for r in (0, K - 1):
        lev, _, _ = O.bfs_levels(G, int(roots[r]))
        got = np.zeros(n, np.int32)
        sel = vi == r
        got[vj[sel]] = vx[sel]
        parity = parity and bool(np.array_equal(got, lev))
    if not parity:
        raise SystemExit("multi-source BFS parity failure vs oracle")
    del vi, vj, vx
    for _ in range(2):
        batch()
    torch.cuda.synchronize()
    reps = 5
    t0 = time.perf_counter()
    for _ in range(reps):
        batch()
    torch.cuda.synchronize()
    el = (time.perf_counter() - t0) / reps
    ok(lib.GrB_Matrix_free(ctypes.byref(Q)), "free Q")
    ok(lib.GrB_Matrix_free(ctypes.byref(V)), "free V")
    return {"workload": f"multi-source level BFS, {K} roots at once: V<Q.V> = d; Q<!V.S,replace> = Q "
                        f"{args.semiring.replace('_', '.')} A "
                        f"(GrB_Matrix_assign + masked GrB_mxm, Q/V {K} x n), R-MAT s{args.scale}",
            "roots": K, "levels": levels, "ms_per_batch": el * 1e3, "gteps": edges / el / 1e9,
            "edges": edges, "parity_vs_oracle_2_roots": parity}


def config3_msbfs_sharded(lib, torch, stream, O, args, dist, world, rank, AT, part, deg, roots16):
    """The 64-root batched BFS 1-D row-sharded (north_star's mxm sharding): rank r holds
    rows [lo, hi) of A^T and per level computes its slice of every root's next frontier,
        Vloc<Qloc.V> = d;  Qloc<!Vloc.S, replace> = Q lor.land (A^T shard)^T   (GrB_DESC_RSCT1)
    then the slices' column words (8 B per vertex: all 64 roots' bits) are all-gathered
    straight into Q's words (GxB_Matrix_colwords_view / _touch) -- one collective per level
    for all 64 roots.  On by default at N > 1 (--no-msbfs-sharded skips it): it is the form of the
    headline workload whose exchange amortises over 64 roots."""
    from graphblas_amd import device as gdev
    from graphblas_amd import dist as gdist

    K = 64
    n = 1 << args.scale
    lo, hi = part["lo"], part["hi"]
    nloc = hi - lo
    rng = np.random.default_rng(args.seed + 1)
    pool = np.setdiff1d(np.flatnonzero(deg > 0), roots16)
    roots = np.concatenate([roots16, rng.choice(pool, K - len(roots16), replace=False)]).astype(np.uint64)
    mine = (roots >= lo) & (roots < hi)
    li, lj = np.flatnonzero(mine).astype(np.uint64), (roots[mine] - lo).astype(np.uint64)
    Q, Ql, Vl = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_void_p()
    ok(lib.GrB_Matrix_new(ctypes.byref(Q), lib.GrB_BOOL, K, n), "Q")
    ok(lib.GrB_Matrix_new(ctypes.byref(Ql), lib.GrB_BOOL, K, nloc), "Qloc")
    ok(lib.GrB_Matrix_new(ctypes.byref(Vl), lib.GrB_INT32, K, nloc), "Vloc")
    qi = np.arange(K, dtype=np.uint64)
    vslot = part["slot"] * 64  # vertices per rank slot (column words exchanged per rank)
    # the ranks' vertex ranges in column-word units (one word per vertex): with unequal (balanced)
    # ranges the gather packs them into place (BitmapAllGather's index gather)
    vb = None if part.get("bounds") is None else [min(n, b * 64) for b in part["bounds"]]
    ex = gdist.BitmapAllGather(dist, {"slot": vslot, "bounds": vb}, world, "cuda")
    packed = ex._pack is not None
    zero_copy = packed or (vslot * world == n and args.dist_backend == "nccl")
    nv = ctypes.c_uint64()
    sr, desc, ALL = _bfs_semiring(lib, args), lib.GrB_DESC_RSCT1, lib.GrB_ALL

    def exchange():
        ptr, cnt = gdev.colwords_view(Ql)
        with torch.cuda.stream(stream):
            ex.send[:cnt].copy_(gdev.device_tensor(torch, ptr, cnt))
            qptr, qn = gdev.colwords_view(Q)
            qw = gdev.device_tensor(torch, qptr, qn)
            if zero_copy:
                ex.run(qw)
            else:
                g = ex.run()
                qw.copy_(g[:qn])
        ok(lib.GxB_Matrix_colwords_touch(Q), "touch Q")

    def batch():
        ok(lib.GrB_Matrix_clear(Q), "clear Q")
        ok(lib.GrB_Matrix_clear(Ql), "clear Qloc")
        ok(lib.GrB_Matrix_clear(Vl), "clear Vloc")
        ok(lib.GxB_Matrix_build_Scalar_BOOL(Q, ctypes.c_void_p(qi.ctypes.data), ctypes.c_void_p(roots.ctypes.data),
                                            True, K), "build Q")
        if li.size:
            ok(lib.GxB_Matrix_build_Scalar_BOOL(Ql, ctypes.c_void_p(li.ctypes.data), ctypes.c_void_p(lj.ctypes.data),
                                                True, li.size), "build Qloc")
        d = 0
        while True:
            d += 1
            ok(lib.GrB_Matrix_assign_INT32(Vl, Ql, None, d, ALL, K, ALL, nloc, None), "Vloc<Qloc> = d")
            ok(lib.GrB_mxm(Ql, Vl, None, sr, Q, AT, desc), "Qloc<!Vloc.S> = Q lor.land AT'")
            exchange()
            ok(lib.GrB_Matrix_nvals(ctypes.byref(nv), Q), "nvals")
            if nv.value == 0:
                ok(lib.GrB_Matrix_wait(Vl, lib.GrB_MATERIALIZE), "wait Vloc")
                return d

    levels = batch()
    # parity (row 0 = the first headline root) and reached edges, gathered over ranks
    ok(lib.GrB_Matrix_nvals(ctypes.byref(nv), Vl), "nvals Vloc")
    m = nv.value
    vi, vj, vx = np.empty(m, np.uint64), np.empty(m, np.uint64), np.empty(m, np.int32)
    cnt = ctypes.c_uint64(m)
    ok(lib.GrB_Matrix_extractTuples_INT32(ctypes.c_void_p(vi.ctypes.data), ctypes.c_void_p(vj.ctypes.data),
                                          ctypes.c_void_p(vx.ctypes.data), ctypes.byref(cnt), Vl), "extract Vloc")
    vi, vj = vi.astype(np.int64), vj.astype(np.int64) + lo
    dev = "cuda" if args.dist_backend == "nccl" else "cpu"
    e_t = torch.tensor([int(deg[vj].sum())], dtype=torch.int64, device=dev)
    dist.all_reduce(e_t)
    edges = int(e_t.item())
    row0 = torch.zeros(vslot, dtype=torch.int32)
    sel = vi == 0
    row0[torch.from_numpy(vj[sel] - lo)] = torch.from_numpy(vx[sel])
    allv = [torch.zeros_like(row0).to(dev) for _ in range(world)]
    dist.all_gather(allv, row0.to(dev))
    parity = None
    if rank == 0:
        # rank k's slice belongs at its range [lo_k, hi_k)
        b = vb if vb is not None else [min(n, k * vslot) for k in range(world + 1)]
        got = np.concatenate([allv[k].cpu().numpy()[:b[k + 1] - b[k]] for k in range(world)])
        lev, _, _ = O.bfs_levels(O.rmat(args.scale, args.edge_factor, args.seed), int(roots[0]))
        parity = bool(np.array_equal(got, lev))
    for _ in range(2):
        batch()
    torch.cuda.synchronize()
    dist.barrier()
    reps = 5
    t0 = time.perf_counter()
    for _ in range(reps):
        batch()
    torch.cuda.synchronize()
    dist.barrier()
    el = (time.perf_counter() - t0) / reps
    t = torch.tensor([el], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    el = float(t.item())
    for h in (Q, Ql, Vl):
        ok(lib.GrB_Matrix_free(ctypes.byref(h)), "free")
    return {"workload": f"multi-source level BFS, {K} roots at once, 1-D row shards x{world}: Vloc<Qloc.V> = d; "
                        f"Qloc<!Vloc.S,replace> = Q {args.semiring.replace('_', '.')} (A^T shard)^T, column words "
                        f"all-gathered per level",
            "roots": K, "levels": levels, "ms_per_batch": el * 1e3, "gteps": edges / el / 1e9, "edges": edges,
            "parity_vs_oracle_root0": parity, "zero_copy": zero_copy}


def config2_spmv(lib, torch, stream, args, scale, ef, O=None, cpu=False):
    """y = x plus.times A, dense fp64 x, on R-MAT (scale, ef)."""
    sc = scale
    n = 1 << sc
    A = ctypes.c_void_p()
    ok(lib.GxB_Matrix_rmat(ctypes.byref(A), sc, ef, args.seed, 2, 2, 0, 0), "rmat fp64")
    ok(lib.GxB_Matrix_prepare_transpose(A), "transpose")
    nv = ctypes.c_uint64()
    ok(lib.GrB_Matrix_nvals(ctypes.byref(nv), A), "nvals")
    nnz = nv.value
    xv = np.random.default_rng(1).random(n)
    x = ctypes.c_void_p()
    ok(lib.GrB_Vector_new(ctypes.byref(x), lib.GrB_FP64, n), "x")
    idx = np.arange(n, dtype=np.uint64)
    ok(lib.GrB_Vector_build_FP64(x, ctypes.c_void_p(idx.ctypes.data), ctypes.c_void_p(xv.ctypes.data), n, None),
       "x build")
    y = ctypes.c_void_p()
    ok(lib.GrB_Vector_new(ctypes.byref(y), lib.GrB_FP64, n), "y")
    sr = lib.GrB_PLUS_TIMES_SEMIRING_FP64
    t = _time_calls(torch, stream, lambda: ok(lib.GrB_vxm(y, None, None, sr, x, A, None), "vxm"), 20)
    ap = np.empty(n + 1, np.uint64)
    ai = np.empty(nnz, np.uint64)
    ax = np.empty(nnz, np.float64)
    lens = [ctypes.c_uint64(n + 1), ctypes.c_uint64(nnz), ctypes.c_uint64(nnz)]
    ok(lib.GrB_Matrix_export_FP64(ctypes.c_void_p(ap.ctypes.data), ctypes.c_void_p(ai.ctypes.data),
                                  ctypes.c_void_p(ax.ctypes.data), *[ctypes.byref(v) for v in lens], 0, A), "export")
    S = sp.csr_matrix((ax, ai.astype(np.int64), ap.astype(np.int64)), shape=(n, n))
    ref = S.T @ xv
    ny = ctypes.c_uint64()
    ok(lib.GrB_Vector_nvals(ctypes.byref(ny), y), "nvals y")
    yi = np.empty(ny.value, np.uint64)
    yv = np.empty(ny.value, np.float64)
    ok(lib.GrB_Vector_extractTuples_FP64(ctypes.c_void_p(yi.ctypes.data), ctypes.c_void_p(yv.ctypes.data),
                                         ctypes.byref(ny), y), "extract y")
    got = np.zeros(n)
    got[yi.astype(np.int64)] = yv
    present = np.zeros(n, bool)
    present[yi.astype(np.int64)] = True
    parity2 = bool(np.array_equal(present, np.diff(S.tocsc().indptr) > 0) and
                   np.allclose(got, ref, rtol=1e-6, atol=1e-9))
    by = 12 * nnz + 8 * (n + 1) + 16 * n
    traffic, src = _profile_traffic(f"config2_s{sc}_pmc.json" if ef == 16 else f"config2_s{sc}_ef{ef}_pmc.json")
    res = {
        "workload": f"y = x plus.times A (GrB_vxm, dense fp64 x) on R-MAT s{sc} ef {ef} fp64 U[0,1) "
                    f"(com-Orkut stand-in)",
        "nnz": nnz, "ms": t * 1e3, "gteps": nnz / t / 1e9, "alg_bytes": by, "hbm_GBs": by / t / 1e9,
        "parity_vs_scipy": parity2,
        "roofline": _roofline(by, t, traffic, src, "k_spmv_words + k_spmv_fold (one call)")}
    if cpu and not args.no_cpu_baseline:
        # the same SpMV on all host cores (oracle or_spmv_plus_times_fp64_par: pull over A^T), repeated
        # for about --cpu-secondary-seconds
        th = _threads()
        AT = _sym_transpose(O, n, ap.astype(np.int64), ai.astype(np.int64), ax, "FP64")
        yc, pc = O.spmv_plus_times_fp64_par(AT, xv, th)
        cpu_ok = bool(np.array_equal(pc, present) and np.allclose(yc, ref, rtol=1e-9, atol=0))
        reps, tc = 0, 0.0
        while tc < args.cpu_secondary_seconds and reps < 1000:
            t1 = time.perf_counter()
            O.spmv_plus_times_fp64_par(AT, xv, th)
            tc += time.perf_counter() - t1
            reps += 1
        res["cpu_baseline"] = {"value": nnz * reps / tc / 1e9, "unit": "GTEPS", "cores": th, "kind": "port",
                               "ms": tc / reps * 1e3, "hbm_GBs": by * reps / tc / 1e9, "matches_scipy": cpu_ok,
                               "sample": f"{reps} full SpMVs of the same matrix and x, {tc:.1f} s: pull over A^T "
                                         f"on {th} host threads (oracle or_spmv_plus_times_fp64_par, OpenMP; "
                                         f"not SuiteSparse)"}
        del AT
    for h in (A, x, y):
        lib.GrB_Matrix_free(ctypes.byref(h))
    return res


def config4_masked_spgemm(lib, torch, stream, O, args, s4, cpu=False):
    """C<A.S> = A min.plus A (GrB_mxm, GrB_DESC_S), INT64 weights in
    [1,255] on R-MAT scale s4; parity vs the oracle on 256 sampled rows (bit-exact)."""
    n4 = 1 << s4
    nv = ctypes.c_uint64()
    B = ctypes.c_void_p()
    ok(lib.GxB_Matrix_rmat(ctypes.byref(B), s4, args.edge_factor, args.seed, 1, 2, 0, 0), "rmat int64")
    ok(lib.GxB_Matrix_prepare_transpose(B), "transpose")
    ok(lib.GrB_Matrix_nvals(ctypes.byref(nv), B), "nvals")
    nnz4 = nv.value
    sr4 = lib.GrB_MIN_PLUS_SEMIRING_INT64
    # each call writes a NEW C, as the reference's `semiring.min_plus(A @ A).new(mask=A.S)` does
    # (SURVEY 3.4); the previous call's C is freed.  Round 4 re-used one C, so each timed call was
    # the update C<M> = T over the previous result, which also merges C's existing entries.
    cbox = [None]

    def call4():
        cn = ctypes.c_void_p()
        ok(lib.GrB_Matrix_new(ctypes.byref(cn), lib.GrB_INT64, n4, n4), "C")
        ok(lib.GrB_mxm(cn, B, None, sr4, B, B, lib.GrB_DESC_S), "mxm")
        if cbox[0] is not None:
            lib.GrB_Matrix_free(ctypes.byref(cbox[0]))
        cbox[0] = cn

    t4 = _time_calls(torch, stream, call4, 3)
    C = cbox[0]
    bp = np.empty(n4 + 1, np.uint64)
    bi = np.empty(nnz4, np.uint64)
    bx = np.empty(nnz4, np.int64)
    lens = [ctypes.c_uint64(n4 + 1), ctypes.c_uint64(nnz4), ctypes.c_uint64(nnz4)]
    ok(lib.GrB_Matrix_export_INT64(ctypes.c_void_p(bp.ctypes.data), ctypes.c_void_p(bi.ctypes.data),
                                   ctypes.c_void_p(bx.ctypes.data), *[ctypes.byref(v) for v in lens], 0, B),
       "export B")
    bp, bi = bp.astype(np.int64), bi.astype(np.int64)
    ok(lib.GrB_Matrix_nvals(ctypes.byref(nv), C), "nvals C")
    nnzc = nv.value
    cp = np.empty(n4 + 1, np.uint64)
    ci = np.empty(nnzc, np.uint64)
    cx = np.empty(nnzc, np.int64)
    lens = [ctypes.c_uint64(n4 + 1), ctypes.c_uint64(nnzc), ctypes.c_uint64(nnzc)]
    ok(lib.GrB_Matrix_export_INT64(ctypes.c_void_p(cp.ctypes.data), ctypes.c_void_p(ci.ctypes.data),
                                   ctypes.c_void_p(cx.ctypes.data), *[ctypes.byref(v) for v in lens], 0, C),
       "export C")
    cp = cp.astype(np.int64)
    dout = np.diff(bp)
    din = np.bincount(bi, minlength=n4)
    rows_of = np.repeat(np.arange(n4), dout)
    work = int((dout[rows_of] + din[bi]).sum())
    inter = int(np.minimum(dout[rows_of], din[bi]).sum())
    del rows_of
    # oracle on 256 sampled rows: C[rows] <A[rows].S> = A[rows] min.+ A
    rows = np.sort(np.random.default_rng(7).choice(n4, 256, replace=False))
    sub_p = np.concatenate([[0], np.cumsum(dout[rows])])
    sub_i = np.concatenate([bi[bp[r]:bp[r + 1]] for r in rows])
    sub_x = np.concatenate([bx[bp[r]:bp[r + 1]] for r in rows])
    Asub = O.Csr(len(rows), n4, "INT64", sub_p, sub_i, sub_x)
    Afull = O.Csr(n4, n4, "INT64", bp, bi, bx)
    ref4 = O.mxm(O.Csr.empty(len(rows), n4, "INT64"), Asub, Afull, ("MIN", "PLUS", "INT64"), mask=Asub,
                 mask_struct=True)
    gsub_p = np.concatenate([[0], np.cumsum(np.diff(cp)[rows])])
    gsub_i = np.concatenate([ci[cp[r]:cp[r + 1]] for r in rows]).astype(np.int64)
    gsub_x = np.concatenate([cx[cp[r]:cp[r + 1]] for r in rows])
    parity4 = bool(np.array_equal(gsub_p, ref4.indptr) and np.array_equal(gsub_i, ref4.indices) and
                   np.array_equal(gsub_x, ref4.values))
    by4 = 2 * (12 * nnz4 + 8 * (n4 + 1)) + 4 * nnz4 + 8 * (n4 + 1) + 12 * nnzc + 8 * (n4 + 1)
    for h in (B, C):
        lib.GrB_Matrix_free(ctypes.byref(h))
    traffic, src = _profile_traffic(f"config4_s{s4}_pmc.json")
    res = {
        "workload": f"C<A.S> = A min.plus A (GrB_mxm, GrB_DESC_S), R-MAT s{s4}, INT64 weights in [1,255]",
        "nnz_A": nnz4, "nnz_C": nnzc, "ms": t4 * 1e3, "gteps": work / t4 / 1e9,
        "gteps_def": "sum over mask entries (i,j) of deg_out(i) + deg_in(j), per second",
        "intersection_keys_per_s": inter / t4,
        "intersection_def": "sum over mask entries of min(deg_out(i), deg_in(j)): the keys the dot streams",
        "alg_bytes": by4, "hbm_GBs": by4 / t4 / 1e9, "parity_vs_oracle_256_rows": parity4,
        "roofline": _roofline(by4, t4, traffic, src, "masked dot kernels (k_dot_task, k_dot_small, ...; one call)"),
        # the dot form's own floor: every mask entry streams its shorter list once (4-byte keys;
        # SURVEY 8(d)'s compulsory bytes beside it) -- the bytes the method cannot avoid
        "roofline_dot_floor": dict(_roofline(by4 + 4 * inter, t4, traffic, src, "the same call"),
                                   alg_bytes_def="SURVEY 8(d) config 4 bytes + 4 B x sum over mask entries of "
                                                 "min(deg_out(i), deg_in(j)) (each shorter list streamed once)")}
    if cpu and not args.no_cpu_baseline:
        # the masked dot on all host cores (oracle or_masked_dot_min_plus_int64_par: per mask entry a
        # sorted merge / galloping of A(i,:) with A(:,j)) over the mask rows [0, r1) -- labels are
        # scrambled, so a leading block of rows is a random sample -- doubling r1 until the sample takes
        # --cpu-secondary-seconds; GTEPS by the same definition as the GPU line
        th = _threads()
        Ac = O.Csr(n4, n4, "INT64", bp, bi, bx)
        AT = _sym_transpose(O, n4, bp, bi, bx, "INT64")
        r1 = max(64, n4 >> 12)
        while True:
            t1 = time.perf_counter()
            vals_c, pres_c, nc_c, work_c = O.masked_dot_min_plus_int64_par(Ac, AT, 0, r1, th)
            tc = time.perf_counter() - t1
            if tc >= args.cpu_secondary_seconds / 2 or r1 >= n4:
                break
            r1 = min(n4, r1 * 2)
        # the CPU sample's entries equal the GPU's C on those rows (bit-exact)
        e1 = int(bp[r1])
        cpu_ok = bool(int(cp[r1]) == int(pres_c.sum()) and
                      np.array_equal(ci[:int(cp[r1])].astype(np.int64), bi[:e1][pres_c]) and
                      np.array_equal(cx[:int(cp[r1])], vals_c[pres_c]))
        res["cpu_baseline"] = {"value": work_c / tc / 1e9, "unit": "GTEPS", "cores": th, "kind": "port",
                               "matches_gpu": cpu_ok,
                               "sample": f"mask rows [0, {r1}) of {n4} ({e1} mask entries, {work_c:.3e} list "
                                         f"elements), {tc:.1f} s on {th} host threads: per mask entry a sorted "
                                         f"merge / galloping dot (oracle or_masked_dot_min_plus_int64_par, OpenMP; "
                                         f"not SuiteSparse)"}
        del Ac, AT
    return res


def config5_spgemm(lib, torch, stream, O, dist, world, rank, args, sc, cpu=False):
    """SURVEY 8(d) config 5 / 8(e) mxm row: C = A plus.times A, FP64, unmasked, on R-MAT scale sc
    (s23 does not fit 8 x 288 GB; BASELINE.md:35 asks for s21/s22), 1-D row shards.
    Rank r holds rows [lo, hi) of A (generated as a row shard), which is also its panel of B; with
    N > 1 the row ranges are balanced by Gustavson products (dist.product_balanced_bounds: SpGEMM
    work on R-MAT is far more skewed than entry counts).  One step = the all-gatherv of B's CSR row
    panels over RCCL (dist.RowPanelAllGather, on the library stream) + GxB_Matrix_import_device +
    the local GrB_mxm(C_r, A_r, B).  Total work is fixed as N grows (strong scaling).
    GTEPS = products (sum over A's entries (i,k) of |B(k,:)|) / max-over-ranks time.
    Parity: 16 sampled rows of each rank's C_r (its longest rows first) against a numpy fold of the
    same rows (fp64, rtol 1e-6; structure exact).
    roofline: SURVEY 8(d)'s compulsory bytes per GPU (A_r and B read once, C_r written once, the
    panels received) / the step time; `stream` beside it prices Gustavson's B-row reads (12 B per
    product) instead of one read of B.  traffic: HBM bytes per call from the committed PMC table
    (N = 1).  cpu_baseline (cpu=True, N = 1): oracle or_spgemm_plus_times_fp64_par (OpenMP
    Gustavson, all host threads) on the leading rows (labels are scrambled: a random sample),
    its rows checked against the GPU's."""
    from graphblas_amd import device as gdev
    from graphblas_amd import dist as gdist

    n = 1 << sc
    xdev = "cuda" if args.dist_backend == "nccl" else "cpu"
    part = gdist.partition(n, world, rank)
    lo, hi = part["lo"], part["hi"]
    A = ctypes.c_void_p()
    ok(lib.GxB_Matrix_rmat(ctypes.byref(A), sc, args.edge_factor, args.seed, 2, 2, lo, hi), "rmat fp64 row panel")
    torch.cuda.synchronize()
    balance = None
    if world > 1 and args.spgemm_partition == "products":
        va = gdev.matrix_view(A)
        rp = gdev.device_tensor(torch, va.rowptr, va.nrows + 1)
        ci = gdev.device_tensor(torch, va.colidx, va.nvals, "<i4")
        bounds, wp = gdist.product_balanced_bounds(dist, torch, n, world, rank, rp, ci, xdev)
        del rp, ci
        eq = [gdist.partition(n, world, k) for k in range(world)]
        cw = np.concatenate([[0], np.cumsum(wp)])
        part = gdist.partition(n, world, rank, bounds)
        balance = {"partition": "rows balanced by products",
                   "products_per_rank_equal_slots": [int(cw[p["hi_w"]] - cw[p["lo_w"]]) for p in eq],
                   "products_per_rank": [int(cw[bounds[k + 1]] - cw[bounds[k]]) for k in range(world)]}
        if (part["lo"], part["hi"]) != (lo, hi):
            lo, hi = part["lo"], part["hi"]
            ok(lib.GrB_Matrix_free(ctypes.byref(A)), "free shard")
            A = ctypes.c_void_p()
            ok(lib.GxB_Matrix_rmat(ctypes.byref(A), sc, args.edge_factor, args.seed, 2, 2, lo, hi),
               "rmat fp64 balanced row panel")
            torch.cuda.synchronize()
    va = gdev.matrix_view(A)
    nr, nnz_a = va.nrows, va.nvals
    gath = gdist.RowPanelAllGather(dist, world, rank) if world > 1 else None
    sr = lib.GrB_PLUS_TIMES_SEMIRING_FP64
    nv = ctypes.c_uint64()
    keep = {}

    def gather():
        with torch.cuda.stream(stream):
            B, _ = gdist.gather_row_panels(lib, torch, gath, A, n)
        return B

    def step(keep_c=False):
        B = gather() if world > 1 else A
        C = ctypes.c_void_p()
        ok(lib.GrB_Matrix_new(ctypes.byref(C), lib.GrB_FP64, nr, n), "C")
        rc = lib.GrB_mxm(C, None, None, sr, A, B, None)
        if rc == 0:
            ok(lib.GrB_Matrix_nvals(ctypes.byref(nv), C), "nvals C")
        if keep_c and rc == 0:
            keep["C"], keep["B"] = C, B
        else:
            ok(lib.GrB_Matrix_free(ctypes.byref(C)), "free C")
            if world > 1:
                ok(lib.GrB_Matrix_free(ctypes.byref(B)), "free B")
        if rc != 0:
            return -rc  # GrB_Info codes are negative
        return nv.value

    def agree(flag):
        """every rank's flag, max-reduced (a failed rank makes all ranks skip together)"""
        if not dist:
            return flag
        t = torch.tensor([flag], dtype=torch.int64, device=xdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return int(t.item())

    # untimed: one step kept for the product count and the parity sample
    r0 = step(keep_c=True)
    failed = agree(1 if "C" not in keep else 0)
    if failed:
        ok(lib.GrB_Matrix_free(ctypes.byref(A)), "free A")
        for h in ("C", "B"):
            if h in keep:
                lib.GrB_Matrix_free(ctypes.byref(keep[h]))
        return {"workload": f"C = A plus.times A, R-MAT s{sc}, 1-D row shards x{world}",
                "skipped": f"GrB_mxm failed on at least one rank (this rank's GrB_Info: "
                           f"{-r0 if 'C' not in keep else 0}; -102 = out of device memory)"}
    nnz_c = r0
    B = keep["B"]
    vb = gdev.matrix_view(B)
    brp = gdev.device_tensor(torch, vb.rowptr, n + 1)
    deg = brp[1:] - brp[:-1]
    aci = gdev.device_tensor(torch, va.colidx, nnz_a, "<i4").long()
    arp_t = gdev.device_tensor(torch, va.rowptr, nr + 1)
    rprod = gdist.row_products(torch, arp_t, aci, deg)
    prods = int(rprod.sum().item())
    # parity sample (host): rows of C_r vs a numpy fold over A_r and B
    C = keep["C"]
    vc = gdev.matrix_view(C)
    crp = gdev.device_tensor(torch, vc.rowptr, nr + 1).cpu().numpy()
    arp = arp_t.cpu().numpy()
    ax = gdev.device_tensor(torch, va.values, nnz_a, "<f8").cpu().numpy()
    ai = aci.cpu().numpy()
    bp = brp.cpu().numpy()
    bi = gdev.device_tensor(torch, vb.colidx, vb.nvals, "<i4").cpu().numpy()
    bx = gdev.device_tensor(torch, vb.values, vb.nvals, "<f8").cpu().numpy()
    cit = gdev.device_tensor(torch, vc.colidx, vc.nvals, "<i4")
    cvt = gdev.device_tensor(torch, vc.values, vc.nvals, "<f8")
    rows = []
    if nr:
        heavy = torch.argsort(rprod, descending=True)[:3].cpu().numpy()  # the column-window bins
        rnd = np.random.default_rng(11 + rank).choice(nr, min(12, nr), replace=False)
        rows = np.unique(np.concatenate([heavy, rnd]))
    parity = True
    for r in rows:
        acc = np.zeros(n)
        present = np.zeros(n, bool)
        for p in range(arp[r], arp[r + 1]):
            k = ai[p]
            s, e = bp[k], bp[k + 1]
            acc[bi[s:e]] += ax[p] * bx[s:e]
            present[bi[s:e]] = True
        cols = np.flatnonzero(present)
        gc = cit[crp[r]:crp[r + 1]].cpu().numpy()
        gv = cvt[crp[r]:crp[r + 1]].cpu().numpy()
        parity &= bool(np.array_equal(gc, cols) and np.allclose(gv, acc[cols], rtol=1e-6, atol=0))
    cpu_res = None
    if cpu and world == 1 and not args.no_cpu_baseline:
        # the same product on all host threads over the leading rows [0, r1), doubling r1 until the
        # sample takes about --cpu-secondary-seconds / 2 or its C would pass 1.5e8 entries (host
        # memory of the check); checked against the GPU's rows
        th = _threads()
        Ah = O.Csr(n, n, "FP64", arp, ai, ax)
        r1 = max(64, n >> 12)
        cap = 150_000_000
        while True:
            t1 = time.perf_counter()
            Cc, prods_c = O.spgemm_plus_times_fp64_par(Ah, Ah, 0, r1, th)
            tc = time.perf_counter() - t1
            if tc >= args.cpu_secondary_seconds / 2 or r1 >= n or int(crp[min(n, 2 * r1)]) > cap:
                break
            r1 = min(n, r1 * 2)
        e1 = int(crp[r1])
        gci = cit[:e1].cpu().numpy().astype(np.int64)
        gcv = cvt[:e1].cpu().numpy()
        cpu_ok = bool(np.array_equal(Cc.indptr, crp[:r1 + 1]) and np.array_equal(Cc.indices, gci) and
                      np.allclose(Cc.values, gcv, rtol=1e-6, atol=0))
        cpu_res = {"value": prods_c / tc / 1e9, "unit": "GTEPS", "cores": th, "kind": "port", "matches_gpu": cpu_ok,
                   "gteps_def": "products per second (the GPU line's definition)",
                   "sample": f"rows [0, {r1}) of {n} ({prods_c:.3e} products, {Cc.nvals} entries of C), {tc:.1f} s "
                             f"on {th} host threads: Gustavson with a dense per-thread accumulator (oracle "
                             f"or_spgemm_plus_times_fp64_par, OpenMP; not SuiteSparse)"}
        del Ah, Cc
    del cit, cvt, aci, arp_t, rprod, brp, deg
    ok(lib.GrB_Matrix_free(ctypes.byref(C)), "free C")
    if world > 1:
        ok(lib.GrB_Matrix_free(ctypes.byref(B)), "free B")
    # the exchange alone (untimed pass): panel all-gather + import, bytes received per rank
    xg = None
    if world > 1:
        torch.cuda.synchronize()
        dist.barrier()
        t1 = time.perf_counter()
        reps = 3
        for _ in range(reps):
            Bx = gather()
            torch.cuda.synchronize()
            ok(lib.GrB_Matrix_free(ctypes.byref(Bx)), "free B")
        tx = (time.perf_counter() - t1) / reps
        t = torch.tensor([tx], dtype=torch.float64, device=xdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        tx = float(t.item())
    for _ in range(args.spgemm_warmup):
        step()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.spgemm_steps):
        step()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    el = (time.perf_counter() - t0) / args.spgemm_steps
    # per-rank compulsory bytes: A_r read, B read, C_r written (+ the other ranks' panels received)
    panel_rx = (12 * (vb.nvals - nnz_a) + 8 * (n - nr)) if world > 1 else 0
    by_r = (12 * nnz_a + 8 * (nr + 1)) + (12 * vb.nvals + 8 * (n + 1)) + (12 * nnz_c + 8 * (nr + 1)) + panel_rx
    st_r = (12 * nnz_a + 8 * (nr + 1)) + 12 * prods + (12 * nnz_c + 8 * (nr + 1)) + panel_rx
    tot = [prods, nnz_c, nnz_a, 1 - int(parity), by_r, st_r, panel_rx]
    if dist:
        t = torch.tensor([el], dtype=torch.float64, device=xdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
        tt = torch.tensor(tot, dtype=torch.int64, device=xdev)
        dist.all_reduce(tt)
        tot = [int(x) for x in tt.tolist()]
    prods_all, nnzc_all, nnza_all, nfail, by_all, st_all, rx_all = tot
    ok(lib.GrB_Matrix_free(ctypes.byref(A)), "free A")
    traffic, src = _profile_traffic(f"config5_s{sc}_pmc.json") \
        if world == 1 else (None, None)
    roof = _roofline(by_all / world, el, traffic, src, "one GrB_mxm call per GPU (k_row_flops, hash bins, "
                                                       "k_row_window, k_window_num, segmented sort)")
    roof["alg_bytes_def"] = ("SURVEY 8(d) config 5, per GPU: 12 nnz(A_r) + 12 nnz(B) + 12 nnz(C_r) + row pointers "
                             "+ the panels received")
    res = {
        "workload": f"C = A plus.times A (GrB_mxm, unmasked, FP64 U[0,1)), R-MAT s{sc} ef {args.edge_factor}, "
                    f"1-D row shards x{world}, B row panels all-gathered over "
                    f"{'RCCL' if world > 1 else '(none: one GPU)'}",
        "n": n, "nnz_A": nnza_all, "nnz_C": nnzc_all, "products": prods_all, "ms": el * 1e3,
        "gteps": prods_all / el / 1e9, "gteps_def": "products (sum over A(i,k) of |B(k,:)|) per second",
        "alg_bytes": by_all, "hbm_GBs_per_gpu": by_all / world / el / 1e9, "parity_sampled_rows": nfail == 0,
        "roofline": roof,
        "roofline_stream": _roofline(st_all / world, el, None, None, "the same call, B rows priced per product "
                                                                    "(12 B each): Gustavson's streamed bytes"),
        "steps": args.spgemm_steps, "warmup": args.spgemm_warmup, "scaling": "strong"}
    if balance:
        res["balance"] = balance
    if world > 1:
        res["allgather"] = {"bytes_received_per_rank_avg": rx_all / world, "ms": tx * 1e3,
                            "GBs_per_rank": rx_all / world / tx / 1e9,
                            "what": "B's row panels all-gathered (RowPanelAllGather: sizes, then one group of "
                                    "send/recv pairs at the panels' true sizes) + GxB_Matrix_import_device, "
                                    "max over ranks"}
    if cpu_res:
        res["cpu_baseline"] = cpu_res
    return res


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.device is not None:
        local_rank = args.device
    import torch

    dist = None
    torch.cuda.set_device(local_rank)
    if world > 1:
        import torch.distributed as dist

        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
        else:
            dist.init_process_group(args.dist_backend)
    os.environ["GRAPHBLAS_AMD_DEVICE"] = str(local_rank)
    import graphblas_amd as gb
    import oracle as O

    lib = gb.lib
    for kv in args.knob:
        k, v = kv.split("=")
        gb.set_knob(k, int(v))
    ok(lib.GxB_Context_set_device(local_rank), "set_device")
    stream = torch.cuda.Stream()
    gb.set_stream(stream)

    from graphblas_amd import dist as gdist

    scale, n = args.scale, 1 << args.scale
    part = gdist.partition(n, world, rank)  # equal 64-aligned bitmap-word slots per rank
    words, lo_w, hi_w, lo, hi = part["words"], part["lo_w"], part["hi_w"], part["lo"], part["hi"]
    nloc = hi - lo

    # ---------------- graph (ingest, untimed)
    A = ctypes.c_void_p()
    t0 = time.time()
    if world == 1:
        ok(lib.GxB_Matrix_rmat(ctypes.byref(A), scale, args.edge_factor, args.seed, 0, 0, 0, 0), "rmat")
        ok(lib.GxB_Matrix_prepare_transpose(A), "transpose")
    else:
        ok(lib.GxB_Matrix_rmat(ctypes.byref(A), scale, args.edge_factor, args.seed, 0x100, 0, lo, hi),
           "rmat shard (rows of A^T)")
        if args.partition == "balanced":
            # 1-D row blocks balanced by entries: the shards' per-word entry
            # counts are all-gathered, cut into equal-entry word ranges, and each rank
            # regenerates its shard for its range when it moved
            ap0, _ = export_csr(lib, A, nloc)
            wl = np.zeros(part["slot"] * 64, np.int64)
            wl[:nloc] = np.diff(ap0)
            xdev = "cuda" if args.dist_backend == "nccl" else "cpu"  # gloo: host tensors
            wsum = torch.from_numpy(wl.reshape(-1, 64).sum(1)).to(xdev)
            got = torch.zeros(part["slot"] * world, dtype=torch.int64, device=xdev)
            dist.all_gather(list(got.chunk(world)), wsum)
            gw = got.cpu().numpy()
            word_nnz = np.concatenate([gw[k * part["slot"]:k * part["slot"] + (
                gdist.partition(n, world, k)["hi_w"] - gdist.partition(n, world, k)["lo_w"])] for k in range(world)])
            part = gdist.partition(n, world, rank, gdist.balanced_bounds(word_nnz, world))
            if (part["lo"], part["hi"]) != (lo, hi):
                lo_w, hi_w, lo, hi = part["lo_w"], part["hi_w"], part["lo"], part["hi"]
                nloc = hi - lo
                ok(lib.GrB_Matrix_free(ctypes.byref(A)), "free shard")
                A = ctypes.c_void_p()
                ok(lib.GxB_Matrix_rmat(ctypes.byref(A), scale, args.edge_factor, args.seed, 0x100, 0, lo, hi),
                   "rmat balanced shard (rows of A^T)")
    torch.cuda.synchronize()
    ingest_s = time.time() - t0
    nnz_local = ctypes.c_uint64()
    ok(lib.GrB_Matrix_nvals(ctypes.byref(nnz_local), A), "nvals")

    # out-degrees (for the TEPS edge count) -- untimed
    ap, ai = export_csr(lib, A, nloc if world > 1 else n)
    if world == 1:
        deg = np.diff(ap)
        nnz = int(ap[-1])
    else:
        deg_t = torch.from_numpy(np.bincount(ai, minlength=n).astype(np.int64)).cuda()
        dist.all_reduce(deg_t)
        deg = deg_t.cpu().numpy()
        nnz_t = torch.tensor([int(ap[-1])], dtype=torch.int64, device="cuda")
        dist.all_reduce(nnz_t)
        nnz = int(nnz_t.item())
    rng = np.random.default_rng(args.seed)
    roots = rng.choice(np.flatnonzero(deg > 0), 16, replace=False)  # Graph500: roots with out-edges

    sr_box = [_bfs_semiring(lib, args)]  # the BFS semiring (swapped for the other-semiring line)
    desc = lib.GrB_DESC_RSC
    grb_all = lib.GrB_ALL
    q = ctypes.c_void_p()
    v = ctypes.c_void_p()
    qloc = ctypes.c_void_p()
    ok(lib.GrB_Vector_new(ctypes.byref(q), lib.GrB_BOOL, n), "q")
    ok(lib.GrB_Vector_new(ctypes.byref(v), lib.GrB_INT32, nloc), "v")
    q2 = ctypes.c_void_p()  # the second frontier buffer of the pipelined sharded loop
    if world > 1:
        ok(lib.GrB_Vector_new(ctypes.byref(qloc), lib.GrB_BOOL, nloc), "qloc")
        ok(lib.GrB_Vector_new(ctypes.byref(q2), lib.GrB_BOOL, n), "q2")
        exchange = gdist.BitmapAllGather(dist, part, world, "cuda")
    peerx = None
    exchange_note = None
    if world > 1 and args.exchange == "peer":
        # one collective at setup (the windows' IPC handles); none per level.  A setup failure on any
        # rank, or a self-test exchange that does not assemble the known pattern, falls back to the
        # all-gather on every rank (the verdict is all-reduced)
        xdev = "cuda" if args.dist_backend == "nccl" else "cpu"
        try:
            peerx = gdist.PeerFrontierExchange(lib, dist, n, world, rank, part, device=xdev)
            ok_setup = 1
        except Exception as e:  # noqa: BLE001
            exchange_note = f"peer window setup failed on rank {rank}: {e}"
            ok_setup = 0
        f = torch.tensor([ok_setup], dtype=torch.int64, device=xdev)
        dist.all_reduce(f, op=dist.ReduceOp.MIN)
        if f.item() and not peerx.self_test(dist, qloc, q, lo, hi, n, xdev):
            exchange_note = "peer window self-test failed: all-gather used"
            f.zero_()
        if not f.item():
            if peerx is not None:
                peerx.free()
            peerx = None
            exchange_note = exchange_note or "peer window setup failed on another rank: all-gather used"
    nv = ctypes.c_uint64()
    ev_pairs, level_counts = [], []

    # the gathered bitmap lands in q's own device bitmap when it comes out contiguous: equal
    # slots that tile the words exactly, or packed ranges (balanced bounds)
    zero_copy = world > 1 and (part.get("bounds") is not None or part["slot"] * world == words)

    def exchange_frontier(into_q_bits, qv=None):
        """all-gather the ranks' frontier slices (RCCL, on the library stream) into qv (q)"""
        qv = q if qv is None else qv
        if peerx is not None:  # device-initiated: put the slice into every window, wait for all
            peerx.run(qloc, qv)
            return
        ok(lib.GxB_Vector_bitmap_export(qloc, ctypes.c_void_p(exchange.send.data_ptr()), hi_w - lo_w), "bm out")
        with torch.cuda.stream(stream):
            gath = exchange.run(into_q_bits)  # into_q_bits: straight into q's device bitmap
        if into_q_bits is not None:
            ok(lib.GxB_Vector_device_touch(qv), "touch q")
        else:
            ok(lib.GxB_Vector_bitmap_import(qv, ctypes.c_void_p(gath.data_ptr()), words), "bm in")

    def sharded_levels_pipelined(timing):
        """N > 1, default: the level loop with the host one level behind the device
        (gdist.pipelined_levels) -- level d + 1's stamp, shard SpMV, all-gather
        and recount are enqueued before the host waits for level d's count (publish ticket)"""
        bufs = [q, q2]
        views = [None, None]
        if zero_copy:
            from graphblas_amd import device as gdev

            views = [gdev.device_tensor(torch, gdev.vector_view(b).bitmap, words) for b in bufs]
        first = {1: True}  # q2's first exchange of a BFS goes through bitmap_import (iso true)

        def enqueue(d):
            ok(lib.GrB_Vector_assign_INT32(v, qloc, None, d, grb_all, nloc, None), "assign")
            if timing:
                e0 = torch.cuda.Event(enable_timing=True)
                e1 = torch.cuda.Event(enable_timing=True)
                e0.record(stream)
            ok(lib.GrB_mxv(qloc, v, None, sr_box[0], A, bufs[(d - 1) % 2], desc), "mxv")
            if timing:
                e1.record(stream)
                ev_pairs.append((e0, e1))
            tgt = d % 2
            exchange_frontier(None if first.pop(tgt, False) else views[tgt], bufs[tgt])
            t = ctypes.c_uint64()
            ok(lib.GxB_Vector_publish_ticket(ctypes.byref(t), bufs[tgt]), "ticket")
            return bufs[tgt], t.value

        def count_of(tok):
            c = ctypes.c_uint64()
            ok(lib.GxB_Vector_wait_ticket(ctypes.byref(c), tok[0], ctypes.c_uint64(tok[1])), "wait ticket")
            return c.value

        return gdist.pipelined_levels(enqueue, count_of, max_levels=n + 2)

    def bfs(src, timing):
        ok(lib.GrB_Vector_clear(q), "clear q")
        ok(lib.GrB_Vector_clear(v), "clear v")
        q_bits = None
        if world == 1:
            ok(lib.GrB_Vector_setElement_BOOL(q, True, int(src)), "q[src]")
        else:
            ok(lib.GrB_Vector_clear(qloc), "clear qloc")
            if lo <= src < hi:
                ok(lib.GrB_Vector_setElement_BOOL(qloc, True, int(src) - lo), "qloc[src]")
            exchange_frontier(None)  # q = root, iso true
            if not args.no_pipeline:
                d = sharded_levels_pipelined(timing)
                level_counts.append(d)
                return d
            if peerx is not None:
                raise SystemExit("--exchange peer runs the pipelined loop only (drop --no-pipeline)")
            if zero_copy:
                from graphblas_amd import device as gdev

                q_bits = gdev.device_tensor(torch, gdev.vector_view(q).bitmap, words)
        d = 0
        while True:
            d += 1
            if timing:
                e0 = torch.cuda.Event(enable_timing=True)
                e1 = torch.cuda.Event(enable_timing=True)
            if world == 1:
                ok(lib.GrB_Vector_assign_INT32(v, q, None, d, grb_all, n, None), "assign")
                if timing:
                    # keep the GPU busy while the host enqueues e0 + the SpMV launch + e1, so
                    # the events bracket the kernel itself, not the host's launch latency
                    with torch.cuda.stream(stream):
                        torch.cuda._sleep(SLEEP_CYCLES)
                    e0.record(stream)
                ok(lib.GrB_vxm(q, v, None, sr_box[0], q, A, desc), "vxm")
                if timing:
                    e1.record(stream)
                    ev_pairs.append((e0, e1))
            else:
                ok(lib.GrB_Vector_assign_INT32(v, qloc, None, d, grb_all, nloc, None), "assign")
                if timing:
                    with torch.cuda.stream(stream):
                        torch.cuda._sleep(SLEEP_CYCLES)
                    e0.record(stream)
                ok(lib.GrB_mxv(qloc, v, None, sr_box[0], A, q, desc), "mxv")
                if timing:
                    e1.record(stream)
                    ev_pairs.append((e0, e1))
                # exchange: all-gather the frontier bitmap over RCCL (stream-ordered)
                exchange_frontier(q_bits)
            ok(lib.GrB_Vector_nvals(ctypes.byref(nv), q), "nvals")
            if nv.value == 0:
                break
        level_counts.append(d)
        return d

    def reached_edges():
        idx, lv = vector_indices(lib, v)
        e = int(deg[idx + lo].sum())
        if world > 1:
            t = torch.tensor([e], dtype=torch.int64, device="cuda")
            dist.all_reduce(t)
            e = int(t.item())
        return e, idx, lv

    # verification (untimed): GPU levels == oracle levels for root 0; edge counts per root
    edges = []
    parity = None
    for k, src in enumerate(roots):
        bfs(src, False)
        e, idx, lv = reached_edges()
        edges.append(e)
        if k == 0 and world == 1:
            G = O.Csr(n, n, "BOOL", ap, ai, np.ones(ai.size, np.bool_))
            lev_ref, _, _ = O.bfs_levels(G, int(src))
            got = np.zeros(n, np.int32)
            got[idx] = lv
            parity = bool(np.array_equal(got, lev_ref))
            if not parity:
                raise SystemExit("BFS parity failure vs oracle")
        elif k == 0:
            # sharded run: gather every rank's level slice, rank 0 checks against the oracle
            dev = "cuda" if args.dist_backend == "nccl" else "cpu"
            mine = torch.zeros(part["slot"] * 64, dtype=torch.int32)
            mine[torch.from_numpy(idx.astype(np.int64))] = torch.from_numpy(lv)
            allv = [torch.zeros_like(mine).to(dev) for _ in range(world)]
            dist.all_gather(allv, mine.to(dev))
            if rank == 0:
                got = torch.cat([t.cpu() for t in allv]).numpy()[:n]
                lev_ref, _, _ = O.bfs_levels(O.rmat(scale, args.edge_factor, args.seed), int(src))
                parity = bool(np.array_equal(got, lev_ref))
                if not parity:
                    raise SystemExit("sharded BFS parity failure vs oracle")
    level_counts.clear()

    for w in range(args.warmup):
        bfs(roots[w % len(roots)], False)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    level_counts.clear()
    per_bfs = []
    t0 = time.perf_counter()
    for s in range(args.steps):
        tb = time.perf_counter()
        bfs(roots[s % len(roots)], False)  # ends on the host-side nvals read: the BFS is complete
        per_bfs.append(time.perf_counter() - tb)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if dist:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    total_edges = sum(edges[s % len(roots)] for s in range(args.steps))
    gteps = total_edges / elapsed / 1e9
    # Graph500 convention: harmonic mean of the per-root TEPS (rank 0's clock)
    hm = len(per_bfs) / sum(t / edges[s % len(roots)] for s, t in enumerate(per_bfs)) / 1e9

    # roofline pass (after the timed region): HIP events on the library stream around
    # every GrB_vxm / GrB_mxv (k_dir_prep + k_iso_work), one BFS per root
    ev_pairs.clear()
    level_counts.clear()
    # the events bracket each level's own launch: the library's speculative enqueue of the next
    # level is switched off for this pass, or a bracket would hold two levels
    spec_knob = gb.get_knob("bfs_spec")
    gb.set_knob("bfs_spec", 1)
    for src in roots:
        bfs(src, True)
    torch.cuda.synchronize()
    gb.set_knob("bfs_spec", spec_knob)
    kern_ms = sum(a.elapsed_time(b) for a, b in ev_pairs)
    launches = len(ev_pairs)
    levels_total = sum(level_counts)
    # per-rank algorithmic bytes of the SpMV calls (each rank streams its shard)
    alg_bytes = len(roots) * (4 * int(ap[-1]) + 8 * (nloc + 1)) + levels_total * 3 * ((n + 7) // 8)
    achieved = alg_bytes / (kern_ms / 1e3) / 1e9 if kern_ms > 0 else None
    traffic = None
    trace_us = None
    # the committed PMC traffic is per launch of the single-GPU kernel (whole matrix): N = 1 only;
    # the same file's kernel trace (speculation off, one launch per level) gives the launch's
    # average duration without the event pair's kernel boundary
    if world == 1 and os.path.exists(args.traffic_file):
        try:
            tj = json.load(open(args.traffic_file))
            traffic = tj.get("bytes_per_launch")
            trace_us = tj.get("per_kernel", {}).get("k_iso_work", {}).get("avg_us")
        except Exception:
            traffic = None
    # measured stream-copy ceiling (device-to-device copy of 2 GiB: read + write bytes)
    copy_gbs = None
    if rank == 0:
        xs = torch.empty(1 << 31, dtype=torch.uint8, device="cuda")
        ys = torch.empty_like(xs)
        ys.copy_(xs)
        torch.cuda.synchronize()
        c0 = time.perf_counter()
        for _ in range(5):
            ys.copy_(xs)
        torch.cuda.synchronize()
        copy_gbs = 5 * 2 * xs.numel() / (time.perf_counter() - c0) / 1e9
        del xs, ys

    secondary = {}
    # the same timed loop with the other boolean semiring (BASELINE.json names any_pair, the notebook
    # lor_land): both take the iso-result SpMV; parity of root 0's levels vs the oracle
    other = "lor_land" if args.semiring == "any_pair" else "any_pair"
    sr_box[0] = lib.GrB_LOR_LAND_SEMIRING_BOOL if other == "lor_land" else lib.GxB_ANY_PAIR_BOOL
    bfs(roots[0], False)
    e0_, idx0, lv0 = reached_edges()
    par_other = None
    if world == 1:
        got = np.zeros(n, np.int32)
        got[idx0] = lv0
        par_other = bool(np.array_equal(got, lev_ref))
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    t0 = time.perf_counter()
    for s in range(len(roots)):
        bfs(roots[s], False)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    el_o = time.perf_counter() - t0
    if dist:
        tt = torch.tensor([el_o], dtype=torch.float64, device="cuda")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        el_o = float(tt.item())
    sr_box[0] = _bfs_semiring(lib, args)
    secondary[f"config3_level_bfs_{other}"] = {
        "workload": f"the headline loop with {other}[BOOL] "
                    f"({'GrB_LOR_LAND_SEMIRING_BOOL' if other == 'lor_land' else 'GxB_ANY_PAIR_BOOL'}), "
                    f"the {len(roots)} roots once each", "gteps": sum(edges) / el_o / 1e9,
        "ms_per_bfs": el_o / len(roots) * 1e3, "parity_vs_oracle_root0": par_other}
    if world > 1 and not args.no_msbfs_sharded:
        secondary["config3_msbfs_64_roots_sharded"] = config3_msbfs_sharded(
            lib, torch, stream, O, args, dist, world, rank, A, part, deg, roots)
    if rank == 0 and world == 1 and not args.no_msbfs:
        secondary["config3_msbfs_64_roots"] = config3_msbfs(lib, torch, stream, O, args, A, n, ap, ai, deg, roots)
    if rank == 0 and world == 1 and not args.no_secondary:
        secondary.update(secondary_workloads(lib, torch, stream, O, args))
    if not args.no_spgemm:
        # config 5 lines: s19 (every N), s20 (every N: pairs the N = 1 line, the largest scale one GPU
        # holds), and from --spgemm-extra the scales BASELINE.md:35 names for larger N (s21 at N >= 2,
        # s22 at N >= 4); a scale whose C does not fit is reported as skipped, not failed
        scales = [(args.spgemm_scale, 1)]
        if args.spgemm_scale_big > args.spgemm_scale:
            scales.append((args.spgemm_scale_big, 1))
        for kv in [x for x in args.spgemm_extra.split(",") if x]:
            s_, w_ = (int(v) for v in kv.split(":"))
            scales.append((s_, w_))
        for s5, wmin in scales:
            if world < wmin:
                continue
            key = "config5_spgemm_plus_times_fp64" + ("" if s5 == args.spgemm_scale else f"_s{s5}")
            # a bounded CPU sample on both single-GPU lines (s19 and s20)
            secondary[key] = config5_spgemm(lib, torch, stream, O, dist, world, rank, args, s5,
                                            cpu=s5 in (args.spgemm_scale, args.spgemm_scale_big))

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        G = O.Csr(n, n, "BOOL", ap, ai, np.ones(ai.size, np.bool_))
        S = sp.csr_matrix((np.ones(ai.size, np.bool_), ai.astype(np.int64), ap.astype(np.int64)), shape=(n, n))
        ST = S.T.tocsr()
        ST.sort_indices()
        GT = O.Csr(n, n, "BOOL", ST.indptr, ST.indices, np.ones(ST.indices.size, np.bool_))
        del S, ST
        # all of this box's host cores given to the job (OMP_NUM_THREADS; the machine's count otherwise)
        threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)
        done_edges, t_cpu, runs = 0, 0.0, 0
        while t_cpu < args.cpu_seconds and runs < 16 * 100:
            src = roots[runs % len(roots)]
            t1 = time.perf_counter()
            _, _, e_cpu = O.bfs_levels_par(G, GT, int(src), threads)
            t_cpu += time.perf_counter() - t1
            done_edges += e_cpu
            runs += 1
        cpu = {"value": done_edges / t_cpu / 1e9, "unit": "GTEPS", "cores": threads, "kind": "port",
               "sample": f"{runs} BFS over the same 16 roots (cycled), R-MAT s{scale}, {t_cpu:.1f} s: the "
                         f"notebook's level loop with each masked vxm run push/pull per level on {threads} "
                         f"host threads (oracle or_bfs_levels_par, OpenMP; not SuiteSparse)"}
        # the oracle's sequential GraphBLAS loop (or_mxm per level), one thread, a shorter sample
        lev = np.zeros(n, np.int32)
        e = ctypes.c_int64()
        done1, t1_cpu, runs1 = 0, 0.0, 0
        cG = G._c()
        for src in roots:
            t1 = time.perf_counter()
            O.lib().or_bfs_graphblas(ctypes.byref(cG), ctypes.c_int64(int(src)),
                                     lev.ctypes.data_as(ctypes.c_void_p), ctypes.byref(e))
            t1_cpu += time.perf_counter() - t1
            done1 += e.value
            runs1 += 1
            if t1_cpu > args.cpu_seconds / 3:
                break
        cpu["graphblas_loop_1thread"] = {"value": done1 / t1_cpu / 1e9, "unit": "GTEPS", "cores": 1,
                                         "sample": f"{runs1} roots, {t1_cpu:.1f} s"}

    if peerx is not None:
        peerx.check()  # raises if a wait timed out (a peer never arrived): no line is printed then
    if rank == 0:
        out = {
            "metric": "GTEPS (masked mxv/vxm level-BFS, R-MAT s22)",
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
            "data": "synthetic (Graph500-style R-MAT .57/.19/.19/.05, generated on device, seed 42)",
            "config": {"workload": f"level-BFS q<!v.S,replace> = q {args.semiring.replace('_', '.')} A "
                                   f"({'GxB_ANY_PAIR_BOOL' if args.semiring == 'any_pair' else 'GrB_LOR_LAND_SEMIRING_BOOL'}"
                                   f"; GrB_vxm, GrB_mxv on A^T "
                                   f"shards for N>1), R-MAT scale {scale}, edge factor {args.edge_factor}, "
                                   f"16 roots", "n": n, "nnz": nnz,
                       "parallelism": (f"1-D row shards x{world}, frontier exchange: "
                                       f"{'device-initiated peer windows' if peerx else 'all-gather'}"
                                       + (f" ({exchange_note})" if exchange_note else ""))
                       if world > 1 else "single GPU"},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                         "frac": (achieved / PEAK_HBM_GBS) if achieved else None, "traffic": traffic,
                         "traffic_source": os.path.relpath(args.traffic_file, ROOT) if traffic else None,
                         "kernel": "k_iso_work (+ k_dir_prep on a BFS's first level)",
                         "rocprof_note": "timed with the level speculation off (one launch per level); under "
                                         "rocprofv3 the speculating loop shows one more, empty k_iso_work per BFS "
                                         f"(the level after the last) -- profiles/{CUR_ROUND}_bfs_nospec_kernel_stats.csv "
                                         "is the BFS with bfs_spec=1, whose average is this one's",
                         "avg_launch_us": kern_ms * 1e3 / launches,
                         # the same bytes over the committed kernel trace's average k_iso_work duration
                         "avg_launch_us_trace": trace_us,
                         "frac_trace": (alg_bytes / launches / (trace_us * 1e-6) / 1e9 / PEAK_HBM_GBS)
                         if trace_us else None,
                         "launches": launches, "alg_bytes_per_launch": alg_bytes / launches,
                         "stream_copy_GBs": copy_gbs},
            "gteps_harmonic_mean": hm,
            "cpu_baseline": cpu,
            "parity_vs_oracle": parity,
            "ingest_s": ingest_s,
            "secondary": secondary,
        }
        print(json.dumps(out), flush=True)
    if peerx is not None:
        peerx.free()
    if dist:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
