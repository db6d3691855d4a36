"""Row-sharded SpGEMM exchange at world_size 2 and 3 on CPU (gloo): each rank holds a
consecutive block of rows of A (= its panel of B, since C = A*A); the CSR row panels
are all-gathered (graphblas_amd.dist.RowPanelAllGather: sizes, then one group of send/recv
pairs moving every packed panel at its true size) and the local product C_r = A_r plus.times B
(here the oracle; GrB_mxm on the GPU, bench.py config 5) stacked over the ranks must
equal the oracle's A plus.times A.  SURVEY §8(e) mxm row; DESIGN.md §6."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle as O
from graphblas_amd import dist as gdist


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, scale, ef, out_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    G = O.rmat(scale, ef, 42, values="FP64", value_seed=2)
    n = G.nrows
    part = gdist.partition(n, world, rank)
    lo, hi = part["lo"], part["hi"]
    p0, p1 = int(G.indptr[lo]), int(G.indptr[hi])
    rp = torch.from_numpy(G.indptr[lo:hi + 1] - p0)
    ci = torch.from_numpy(G.indices[p0:p1].astype(np.int32))
    vx = torch.from_numpy(G.values[p0:p1].copy())
    brp, bci, bvx, biso = gdist.RowPanelAllGather(dist, world, rank).run(rp, ci, vx)
    assert not biso
    B = O.Csr(n, n, "FP64", brp.numpy(), bci.numpy(), bvx.numpy())
    Ar = O.Csr(hi - lo, n, "FP64", rp.numpy(), ci.numpy(), vx.numpy())
    C = O.mxm(O.Csr.empty(hi - lo, n, "FP64"), Ar, B, ("PLUS", "TIMES", "FP64"))
    out_q.put((rank, lo, hi, brp.numpy(), bci.numpy(), bvx.numpy(), C.indptr, C.indices, C.values))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,scale,ef", [(2, 8, 8), (3, 9, 8), (2, 6, 4)])
def test_row_panel_spgemm_matches_oracle(world, scale, ef):
    G = O.rmat(scale, ef, 42, values="FP64", value_seed=2)
    ref = O.mxm(O.Csr.empty(G.nrows, G.ncols, "FP64"), G, G, ("PLUS", "TIMES", "FP64"))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, scale, ef, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in range(world)], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # every rank assembled exactly A (scale 6 with 2 ranks: rank 1 holds an empty panel)
    for _, lo, hi, brp, bci, bvx, _, _, _ in res:
        assert np.array_equal(brp, G.indptr) and np.array_equal(bci.astype(np.int64), G.indices)
        assert np.array_equal(bvx, G.values)
    # the stacked row panels of C are the oracle's C (the same fold order: bit-exact)
    cp = [np.zeros(1, np.int64)]
    ci, cv = [], []
    base = 0
    for _, lo, hi, _, _, _, rp, idx, val in res:
        cp.append(rp[1:] + base)
        base += int(rp[-1])
        ci.append(idx)
        cv.append(val)
    assert np.array_equal(np.concatenate(cp), ref.indptr)
    assert np.array_equal(np.concatenate(ci), ref.indices)
    assert np.array_equal(np.concatenate(cv), ref.values)


def test_row_panel_world1_and_iso():
    """world 1 (no collective issued): the panel comes back as is; iso panels keep one value."""

    class _One:
        def all_gather(self, out, t):
            out[0].copy_(t)

        def broadcast(self, t, src):
            raise AssertionError("no broadcast at world 1")

        def get_backend(self):
            raise AssertionError("no panel collective at world 1")

    G = O.rmat(7, 8, 42, values="FP64", value_seed=2)
    rp = torch.from_numpy(G.indptr.copy())
    ci = torch.from_numpy(G.indices.astype(np.int32))
    vx = torch.from_numpy(G.values.copy())
    brp, bci, bvx, biso = gdist.RowPanelAllGather(_One(), 1, 0).run(rp, ci, vx)
    assert not biso
    assert np.array_equal(brp.numpy(), G.indptr) and np.array_equal(bci.numpy(), ci.numpy())
    assert np.array_equal(bvx.numpy(), G.values)
    one = torch.ones(1, dtype=torch.float64)
    _, _, ivx, iiso = gdist.RowPanelAllGather(_One(), 1, 0).run(rp, ci, one, iso=True)
    assert iiso and ivx.numel() == 1 and float(ivx[0]) == 1.0


def _iso_worker(rank, world, port, kinds, out_q):
    """rank r's panel: rows [lo, hi) of a fixed R-MAT pattern with values per kinds[r]:
    ("iso", v) -> one value v, ("full", None) -> its own values."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    G = O.rmat(7, 8, 42, values="FP64", value_seed=2)
    part = gdist.partition(G.nrows, world, rank)
    lo, hi = part["lo"], part["hi"]
    p0, p1 = int(G.indptr[lo]), int(G.indptr[hi])
    rp = torch.from_numpy(G.indptr[lo:hi + 1] - p0)
    ci = torch.from_numpy(G.indices[p0:p1].astype(np.int32))
    kind, val = kinds[rank]
    if kind == "iso":
        vx, iso = torch.tensor([val], dtype=torch.float64), True
    else:
        vx, iso = torch.from_numpy(G.values[p0:p1].copy()), False
    brp, bci, bvx, biso = gdist.RowPanelAllGather(dist, world, rank).run(rp, ci, vx, iso=iso)
    out_q.put((rank, brp.numpy(), bci.numpy(), bvx.numpy(), biso))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("kinds", [
    [("iso", 3.0), ("full", None)],       # mixed: iso panel expanded, no collective mismatch
    [("iso", 3.0), ("iso", 5.0)],         # all iso, different values: expanded per panel
    [("iso", 2.5), ("iso", 2.5)],         # all iso, same value: iso result
])
def test_row_panel_mixed_iso(kinds):
    """every rank must issue the same collective sequence and the assembled
    values must be each panel's own (iso panels expanded unless all agree)."""
    world = len(kinds)
    G = O.rmat(7, 8, 42, values="FP64", value_seed=2)
    expect = np.empty(G.nvals)
    for r, (kind, val) in enumerate(kinds):
        part = gdist.partition(G.nrows, world, r)
        p0, p1 = int(G.indptr[part["lo"]]), int(G.indptr[part["hi"]])
        expect[p0:p1] = val if kind == "iso" else G.values[p0:p1]
    all_same_iso = all(k == "iso" for k, _ in kinds) and len({v for _, v in kinds}) == 1
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_iso_worker, args=(r, world, port, kinds, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for _, brp, bci, bvx, biso in res:
        assert np.array_equal(brp, G.indptr) and np.array_equal(bci.astype(np.int64), G.indices)
        assert biso == all_same_iso
        if biso:
            assert bvx.size == 1 and bvx[0] == kinds[0][1]
        else:
            assert np.array_equal(bvx, expect)


def _degree_sorted_fp64(G):
    """G relabelled so ids fall with out-degree (hubs first): equal row slots give rank 0 most of
    the Gustavson work"""
    order = np.argsort(-np.diff(G.indptr), kind="stable")
    new = np.empty_like(order)
    new[order] = np.arange(order.size)
    rows = new[np.repeat(np.arange(G.nrows), np.diff(G.indptr))]
    return O.Csr.from_coo(rows, new[G.indices], G.values, nrows=G.nrows, ncols=G.ncols, dtype="FP64")


def _balanced_worker(rank, world, port, scale, out_q, mode=None):
    """bench.py config 5 at N > 1: equal-slot shards -> product-balanced bounds -> re-cut shards ->
    panel all-gather -> local product"""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    G = _degree_sorted_fp64(O.rmat(scale, 8, 42, values="FP64", value_seed=2))
    n = G.nrows
    eq = gdist.partition(n, world, rank)
    p0, p1 = int(G.indptr[eq["lo"]]), int(G.indptr[eq["hi"]])
    rp = torch.from_numpy(G.indptr[eq["lo"]:eq["hi"] + 1] - p0)
    ci = torch.from_numpy(G.indices[p0:p1].astype(np.int32))
    bounds, wp = gdist.product_balanced_bounds(dist, torch, n, world, rank, rp, ci, "cpu")
    part = gdist.partition(n, world, rank, bounds)
    lo, hi = part["lo"], part["hi"]
    p0, p1 = int(G.indptr[lo]), int(G.indptr[hi])
    rp = torch.from_numpy(G.indptr[lo:hi + 1] - p0)
    ci = torch.from_numpy(G.indices[p0:p1].astype(np.int32))
    vx = torch.from_numpy(G.values[p0:p1].copy())
    g = gdist.RowPanelAllGather(dist, world, rank, mode=mode)
    brp, bci, bvx, _ = g.run(rp, ci, vx)
    # the panels travel at their true sizes (no padding to the largest panel)
    true_rx = 0
    for k in range(world):
        pk = gdist.partition(n, world, k, bounds)
        if k != rank:
            true_rx += g._layout(pk["hi"] - pk["lo"], int(G.indptr[pk["hi"]] - G.indptr[pk["lo"]]), 8, True)[2]
    assert g.last_rx_bytes == true_rx, (g.last_rx_bytes, true_rx)
    B = O.Csr(n, n, "FP64", brp.numpy(), bci.numpy(), bvx.numpy())
    Ar = O.Csr(hi - lo, n, "FP64", rp.numpy(), ci.numpy(), vx.numpy())
    C = O.mxm(O.Csr.empty(hi - lo, n, "FP64"), Ar, B, ("PLUS", "TIMES", "FP64"))
    out_q.put((rank, bounds, wp, lo, hi, C.indptr, C.indices, C.values))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,mode", [(2, None), (3, None), (3, "bcast")])
def test_product_balanced_bounds(world, mode):
    """dist.product_balanced_bounds (bench.py config 5, N > 1): every rank derives the same row
    ranges (mode "bcast": the panels move as the per-owner broadcasts RCCL uses; None: gloo's
    send/recv pairs); the per-word products equal a direct count; each range carries at most total/world plus
    one word's products; on a hubs-first graph it evens out what equal slots leave on rank 0; and the
    stacked local products over the re-cut ranges are the oracle's C (bit-exact)"""
    scale = 9
    G = _degree_sorted_fp64(O.rmat(scale, 8, 42, values="FP64", value_seed=2))
    n = G.nrows
    deg = np.diff(G.indptr)
    row_prod = np.add.reduceat(np.concatenate([deg[G.indices], [0]]), G.indptr[:-1])
    row_prod[deg == 0] = 0
    words = (n + 63) // 64
    wp_ref = np.zeros(words * 64, np.int64)
    wp_ref[:n] = row_prod
    wp_ref = wp_ref.reshape(words, 64).sum(1)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_balanced_worker, args=(r, world, port, scale, q, mode)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in range(world)], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    bounds = res[0][1]
    for r in res:
        assert r[1] == bounds and np.array_equal(r[2], wp_ref)
    cw = np.concatenate([[0], np.cumsum(wp_ref)])
    tot = int(cw[-1])
    per = [int(cw[bounds[k + 1]] - cw[bounds[k]]) for k in range(world)]
    assert sum(per) == tot and max(per) <= tot / world + int(wp_ref.max())
    eq = [int(cw[gdist.partition(n, world, k)["hi_w"]] - cw[gdist.partition(n, world, k)["lo_w"]])
          for k in range(world)]
    assert max(per) < max(eq)
    ref = O.mxm(O.Csr.empty(n, n, "FP64"), G, G, ("PLUS", "TIMES", "FP64"))
    cp, cidx, cval, base = [np.zeros(1, np.int64)], [], [], 0
    for _, _, _, lo, hi, rp, idx, val in res:
        cp.append(rp[1:] + base)
        base += int(rp[-1])
        cidx.append(idx)
        cval.append(val)
    assert np.array_equal(np.concatenate(cp), ref.indptr)
    assert np.array_equal(np.concatenate(cidx), ref.indices)
    assert np.array_equal(np.concatenate(cval), ref.values)
