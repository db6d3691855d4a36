"""The device-initiated frontier exchange's protocol (csrc/gb_peer.hip) at world
size 2 and 3 on CPU: graphblas_amd.dist.HostPeerWindow restates it over shared memory (two
parity buffers, per-rank counts, per-rank arrival flags carrying the exchange number).  Each
rank runs the pipelined sharded level loop (dist.pipelined_levels) with a "device" thread that
executes its enqueued levels in order -- stamp, local pull step, put, wait -- like the library
stream, and sleeps at random points, so fast and slow ranks overlap as they would on the GPUs.
The levels must equal the oracle's (reference notebooks/Example B.1 cell 8 via O.bfs_levels).
gloo carries only the setup (barriers); the levels' data moves through the windows alone."""
import os
import queue
import socket
import threading
import time
import uuid

import numpy as np
import pytest
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


def _transpose(G):
    rows = np.repeat(np.arange(G.nrows), np.diff(G.indptr))
    order = np.lexsort((rows, G.indices))
    indptr = np.zeros(G.ncols + 1, np.int64)
    np.cumsum(np.bincount(G.indices, minlength=G.ncols), out=indptr[1:])
    return indptr, rows[order]


def _worker(rank, world, port, tag, scale, srcs, balanced, seed, out_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    G = O.rmat(scale, 16, 42)
    n = G.nrows
    tp, ti = _transpose(G)
    bounds = None
    if balanced:
        words = (n + 63) // 64
        deg = np.zeros(words * 64, np.int64)
        deg[:n] = np.diff(tp)
        bounds = gdist.balanced_bounds(deg.reshape(words, 64).sum(1), world)
    part = gdist.partition(n, world, rank, bounds)
    lo, hi = part["lo"], part["hi"]
    win = gdist.HostPeerWindow(dist, tag, n, world, rank, bounds)
    rng = np.random.default_rng(seed + 101 * rank)

    def jitter():
        if rng.random() < 0.5:
            time.sleep(float(rng.random()) * 2e-3)

    # the "stream": a device thread executing the enqueued levels in order
    ops = queue.Queue()

    def device():
        while True:
            f = ops.get()
            if f is None:
                return
            f()

    th = threading.Thread(target=device, daemon=True)
    th.start()
    results = []
    for src in srcs:
        bufs = [np.zeros(n, bool), np.zeros(n, bool)]  # the rank's two frontier buffers
        st = {"qloc": np.zeros(hi - lo, bool), "visited": np.zeros(hi - lo, bool),
              "level": np.zeros(hi - lo, np.int32)}
        if lo <= src < hi:
            st["qloc"][src - lo] = True
        first = queue.Queue()

        def exchange(into, done):
            q = st["qloc"]
            jitter()
            win.put(gdist.pack_bits(q, max(1, part["hi_w"] - part["lo_w"])), int(q.sum()))
            jitter()
            words, total = win.wait()
            into[:] = gdist.unpack_bits(words, n)
            assert int(into.sum()) == total
            done.put(total)

        ops.put(lambda: exchange(bufs[0], first))
        first.get()

        def enqueue(d):
            done = queue.Queue()

            def level():
                cur, nxt = bufs[(d - 1) % 2], bufs[d % 2]
                st["level"][st["qloc"] & ~st["visited"]] = d  # v<qloc> = d
                st["visited"] |= st["qloc"]
                new = np.zeros(hi - lo, bool)  # qloc<!v.S, replace> = A^T_r lor.land q
                for r in range(lo, hi):
                    if not st["visited"][r - lo]:
                        new[r - lo] = bool(cur[ti[tp[r]:tp[r + 1]]].any())
                st["qloc"] = new
                exchange(nxt, done)

            ops.put(level)
            return done

        nlev = gdist.pipelined_levels(enqueue, lambda done: done.get(), max_levels=n + 2)
        drained = threading.Event()  # the level enqueued past the last has run (stream sync)
        ops.put(drained.set)
        drained.wait()
        results.append((src, nlev, st["level"].copy()))
    ops.put(None)
    th.join()
    win.close(dist)
    out_q.put((rank, lo, hi, results))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("scale,world,balanced,seed", [(9, 2, False, 1), (10, 2, True, 2), (9, 3, True, 3),
                                                        (8, 3, False, 4)])
def test_peer_window_protocol_pipelined_bfs(scale, world, balanced, seed):
    G = O.rmat(scale, 16, 42)
    deg = np.diff(G.indptr)
    srcs = [int(np.argmax(deg)), int(np.random.default_rng(seed).choice(np.flatnonzero(deg > 0)))]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    tag = f"gbpw{uuid.uuid4().hex[:10]}"
    procs = [ctx.Process(target=_worker, args=(r, world, port, tag, scale, srcs, balanced, seed, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for i, src in enumerate(srcs):
        ref, nref, _ = O.bfs_levels(G, src)
        got = np.zeros(G.nrows, np.int32)
        for rank, lo, hi, results in res:
            s, nlev, lev = results[i]
            assert s == src and nlev == int(ref.max())
            got[lo:hi] = lev
        assert np.array_equal(got, ref), f"source {src}"
