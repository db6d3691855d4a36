"""Sharded BFS exchange logic at world_size 2 on CPU (gloo): the partition and
bitmap all-gather of graphblas_amd.dist, with a numpy local step over each
rank's row shard of A^T, must reproduce the oracle's BFS levels.
The GPU run uses the same partition and exchange with GrB_mxv as the local step
and RCCL as the transport (bench.py)."""
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


class _Csr:
    def __init__(self, indptr, indices):
        self.indptr, self.indices = indptr, indices


def _transpose(G):
    rows = np.repeat(np.arange(G.nrows), np.diff(G.indptr))
    order = np.lexsort((rows, G.indices))
    indptr = np.zeros(G.ncols + 1, np.int64)
    np.cumsum(np.bincount(G.indices, minlength=G.ncols), out=indptr[1:])
    return _Csr(indptr, rows[order])


def _degree_sorted(G):
    """G relabelled so vertex ids fall with out-degree: hubs first, the unscrambled layout of
    real graphs for which equal vertex slots are badly unbalanced."""
    order = np.argsort(-np.diff(G.indptr), kind="stable")
    new = np.empty_like(order)
    new[order] = np.arange(order.size)
    rows = new[np.repeat(np.arange(G.nrows), np.diff(G.indptr))]
    return O.Csr.from_coo(rows, new[G.indices], np.ones(rows.size, bool), nrows=G.nrows, ncols=G.ncols,
                          dtype="BOOL")


def _graph(scale, skewed):
    G = O.rmat(scale, 16, 42)
    return _degree_sorted(G) if skewed else G


def _worker(rank, world, port, scale, src, out_q, balanced=False):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    G = _graph(scale, balanced)
    n = G.nrows
    AT = _transpose(G)  # rows of A^T = in-edges: pull mxv, as in bench.py
    bounds = None
    if balanced:  # 1-D row blocks balanced by the shard's entries
        words = (n + 63) // 64
        deg = np.zeros(words * 64, np.int64)
        deg[:n] = np.diff(AT.indptr)
        bounds = gdist.balanced_bounds(deg.reshape(words, 64).sum(1), world)
    part = gdist.partition(n, world, rank, bounds)
    lo, hi = part["lo"], part["hi"]
    ex = gdist.BitmapAllGather(dist, part, world, "cpu")
    frontier = np.zeros(n, bool)
    frontier[src] = True
    visited = np.zeros(hi - lo, bool)
    level = np.zeros(hi - lo, np.int32)
    d = 0
    while True:
        d += 1
        loc = frontier[lo:hi]
        level[loc & ~visited] = d
        visited |= loc
        # q_r<!v_r.S, replace> = A^T_r lor.land q  (pull over the shard's rows)
        nxt = np.zeros(hi - lo, bool)
        for r in range(lo, hi):
            if visited[r - lo]:
                continue
            cols = AT.indices[AT.indptr[r]:AT.indptr[r + 1]]
            nxt[r - lo] = bool(frontier[cols].any())
        ex.send.copy_(torch.from_numpy(gdist.pack_bits(nxt, part["slot"])))
        full = ex.run().numpy()
        if bounds is not None:  # ranges packed together: the whole bitmap
            frontier = gdist.unpack_bits(full[:part["words"]], n)
        else:  # words are slot-aligned per rank: rank k's slice starts at word k*slot
            frontier = np.zeros(n, bool)
            for k in range(world):
                pk = gdist.partition(n, world, k)
                sl = full[k * part["slot"]:k * part["slot"] + (pk["hi_w"] - pk["lo_w"])]
                frontier[pk["lo"]:pk["hi"]] = gdist.unpack_bits(sl, pk["hi"] - pk["lo"])
        if not frontier.any():
            break
    out_q.put((rank, lo, hi, level))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("scale,world,balanced", [(8, 2, False), (10, 2, False), (10, 2, True), (9, 3, True)])
def test_sharded_bfs_world2_matches_oracle(scale, world, balanced):
    G = _graph(scale, balanced)
    src = int(np.argmax(np.diff(G.indptr)))
    ref, _, _ = O.bfs_levels(G, src)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, scale, src, q, balanced))
             for r in range(world)]
    for p in procs:
        p.start()
    got = np.zeros(G.nrows, np.int32)
    for _ in range(world):
        rank, lo, hi, level = q.get(timeout=120)
        got[lo:hi] = level
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert np.array_equal(got, ref)


def test_partition_covers_vertices():
    for n in [1, 63, 64, 65, 1000, 4096 + 7]:
        for world in [1, 2, 3, 8]:
            parts = [gdist.partition(n, world, r) for r in range(world)]
            covered = np.zeros(n, int)
            for p in parts:
                covered[p["lo"]:p["hi"]] += 1
                assert p["lo"] % 64 == 0 and p["hi_w"] - p["lo_w"] <= p["slot"]
            assert (covered == 1).all()


def test_balanced_bounds_even_out_a_skewed_graph():
    """On a degree-sorted graph equal vertex slots put most entries on rank 0; nnz-balanced
    word ranges keep every rank within a few words' entries of the mean."""
    G = _degree_sorted(O.rmat(12, 16, 42))
    n = G.nrows
    words = (n + 63) // 64
    deg = np.zeros(words * 64, np.int64)
    deg[:n] = np.diff(G.indptr)
    wn = deg.reshape(words, 64).sum(1)
    for world in (2, 3, 8):
        b = gdist.balanced_bounds(wn, world)
        assert b[0] == 0 and b[-1] == words and all(b[k] <= b[k + 1] for k in range(world))
        per = [int(wn[b[k]:b[k + 1]].sum()) for k in range(world)]
        eq = [int(wn[gdist.partition(n, world, k)["lo_w"]:gdist.partition(n, world, k)["hi_w"]].sum())
              for k in range(world)]
        mean = wn.sum() / world
        assert max(per) <= mean + wn.max()
        assert max(eq) > 1.5 * mean  # what the equal slots would have done
        parts = [gdist.partition(n, world, k, b) for k in range(world)]
        covered = np.zeros(n, int)
        for p in parts:
            covered[p["lo"]:p["hi"]] += 1
            assert p["hi_w"] - p["lo_w"] <= p["slot"]
        assert (covered == 1).all()


def _worker_pipelined(rank, world, port, scale, src, out_q, balanced):
    """The sharded loop with the host one level behind (gdist.pipelined_levels): level d + 1 is
    enqueued -- stamp, local pull step, all-gather into the other frontier buffer -- before the
    count of level d's frontier is read.  Same numpy local step as _worker."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    G = _graph(scale, balanced)
    n = G.nrows
    AT = _transpose(G)
    bounds = None
    if balanced:
        words = (n + 63) // 64
        deg = np.zeros(words * 64, np.int64)
        deg[:n] = np.diff(AT.indptr)
        bounds = gdist.balanced_bounds(deg.reshape(words, 64).sum(1), world)
    part = gdist.partition(n, world, rank, bounds)
    lo, hi = part["lo"], part["hi"]
    ex = gdist.BitmapAllGather(dist, part, world, "cpu")
    bufs = [np.zeros(n, bool), np.zeros(n, bool)]  # the two frontier buffers (q_a, q_b)
    bufs[0][src] = True
    qloc = bufs[0][lo:hi].copy()  # this rank's slice of the current frontier (the stamp's mask)
    visited = np.zeros(hi - lo, bool)
    level = np.zeros(hi - lo, np.int32)
    issued = []

    def enqueue(d):
        nonlocal qloc
        issued.append(d)
        cur, nxt_buf = bufs[(d - 1) % 2], bufs[d % 2]
        level[qloc & ~visited] = d  # v<qloc> = d
        visited[:] |= qloc
        nxt = np.zeros(hi - lo, bool)  # qloc<!v.S, replace> = A^T_r lor.land q
        for r in range(lo, hi):
            if not visited[r - lo]:
                cols = AT.indices[AT.indptr[r]:AT.indptr[r + 1]]
                nxt[r - lo] = bool(cur[cols].any())
        qloc = nxt
        ex.send.copy_(torch.from_numpy(gdist.pack_bits(nxt, part["slot"])))
        full = ex.run().numpy()
        if bounds is not None:
            nxt_buf[:] = gdist.unpack_bits(full[:part["words"]], n)
        else:
            nxt_buf[:] = False
            for k in range(world):
                pk = gdist.partition(n, world, k)
                sl = full[k * part["slot"]:k * part["slot"] + (pk["hi_w"] - pk["lo_w"])]
                nxt_buf[pk["lo"]:pk["hi"]] = gdist.unpack_bits(sl, pk["hi"] - pk["lo"])
        return int(nxt_buf.sum())  # the token: the device-published count

    nlev = gdist.pipelined_levels(enqueue, lambda tok: tok, max_levels=n + 2)
    out_q.put((rank, lo, hi, level, nlev, issued))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("scale,world,balanced", [(9, 2, False), (10, 2, True), (9, 3, True)])
def test_pipelined_sharded_bfs_matches_oracle(scale, world, balanced):
    """the sharded level loop with the host one level behind the device gives the
    oracle's levels; it issues exactly one level past the last (over an empty frontier, a no-op)."""
    G = _graph(scale, balanced)
    src = int(np.argmax(np.diff(G.indptr)))
    ref, nref, _ = O.bfs_levels(G, src)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_pipelined, args=(r, world, port, scale, src, q, balanced))
             for r in range(world)]
    for p in procs:
        p.start()
    got = np.zeros(G.nrows, np.int32)
    for _ in range(world):
        rank, lo, hi, level, nlev, issued = q.get(timeout=120)
        got[lo:hi] = level
        assert issued == list(range(1, nlev + 2))
        assert nlev == int(ref.max())
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert np.array_equal(got, ref)


def test_pipelined_levels_order():
    """the driver alone: level d + 1 is enqueued before level d's count is read"""
    log = []
    counts = {1: 3, 2: 5, 3: 0}

    def enqueue(d):
        log.append(("enqueue", d))
        return d

    def count_of(d):
        log.append(("count", d))
        return counts.get(d, 0)

    assert gdist.pipelined_levels(enqueue, count_of) == 3
    assert log == [("enqueue", 1), ("enqueue", 2), ("count", 1), ("enqueue", 3), ("count", 2),
                   ("enqueue", 4), ("count", 3)]
