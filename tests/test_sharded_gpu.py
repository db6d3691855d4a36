"""The 1-D row-sharded product paths of DESIGN.md §6, run through the HIP
library on one GPU from one process: every shard of a world of W = 2 (and 3) is driven
here in turn, and the exchange step is the same device-memory operation the RCCL
collective performs -- the shards' slices are written into the full frontier / B panel
through the zero-copy views (GxB_Vector_device_view / GxB_Matrix_colwords_view /
GxB_Vector_bitmap_export+import / GxB_Matrix_import_device) on the library stream, then
GxB_Vector_device_touch / GxB_Matrix_colwords_touch recount.  The collective itself is
covered on CPU by tests/test_dist.py and tests/test_dist_spgemm.py (gloo, world size 2).

Parity (bit-exact for the BFS levels, structure-exact and rtol 1e-9 for fp64 plus_times)
against the oracle: O.bfs_levels, O.mxm.  Reference call shapes: core/matrix.py:2163-2251
(mxv / mxm builders), notebooks/Example B.1 cell 8 (level BFS)."""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

import oracle as O  # noqa: E402


@pytest.fixture(scope="module")
def env():
    import torch

    import graphblas_amd as gb

    stream = torch.cuda.Stream()
    gb.set_stream(stream)
    yield gb, torch, stream
    torch.cuda.synchronize()
    gb.set_stream(None)


def ok(rc, what):
    assert rc == 0, f"{what}: GrB_Info {rc}"


def _extract_int32(lib, v):
    nv = ctypes.c_uint64()
    ok(lib.GrB_Vector_nvals(ctypes.byref(nv), v), "nvals")
    idx = np.empty(nv.value, np.uint64)
    x = np.empty(nv.value, np.int32)
    ok(lib.GrB_Vector_extractTuples_INT32(ctypes.c_void_p(idx.ctypes.data), ctypes.c_void_p(x.ctypes.data),
                                          ctypes.byref(nv), v), "extract")
    return idx.astype(np.int64), x


@pytest.mark.parametrize("scale", [10, 12, 14])
@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("exchange", ["view", "bitmap"])
@pytest.mark.parametrize("semiring", ["GrB_LOR_LAND_SEMIRING_BOOL", "GxB_ANY_PAIR_BOOL"])
def test_sharded_bfs_mxv_vs_oracle(env, scale, world, exchange, semiring):
    """bench.py's N > 1 loop: rank r holds rows [lo, hi) of A^T and runs
    v_r<qloc_r> = d;  qloc_r<!v_r.S, replace> = A^T_r lor.land q  (GrB_mxv, GrB_DESC_RSC)
    then the frontier slices are gathered into q's bitmap (in place through the device view, or
    GxB_Vector_bitmap_export/_import), as the RCCL all-gather does."""
    gb, torch, stream = env
    from graphblas_amd import device as gdev
    from graphblas_amd import dist as gdist

    lib = gb.lib
    n = 1 << scale
    G = O.rmat(scale, 16, 42)
    deg = np.diff(G.indptr)
    parts = [gdist.partition(n, world, r) for r in range(world)]
    words, slot = parts[0]["words"], parts[0]["slot"]
    AT, v, ql = [], [], []
    for p in parts:
        nloc = p["hi"] - p["lo"]
        h = ctypes.c_void_p()
        ok(lib.GxB_Matrix_rmat(ctypes.byref(h), scale, 16, 42, 0x100, 0, p["lo"], p["hi"]), "rmat shard")
        AT.append(h)
        for lst, t in ((v, lib.GrB_INT32), (ql, lib.GrB_BOOL)):
            x = ctypes.c_void_p()
            ok(lib.GrB_Vector_new(ctypes.byref(x), t, nloc), "new")
            lst.append(x)
    q = ctypes.c_void_p()
    ok(lib.GrB_Vector_new(ctypes.byref(q), lib.GrB_BOOL, n), "q")
    gathered = torch.zeros(slot * world, dtype=torch.int64, device="cuda")
    sr = getattr(lib, semiring)
    nv = ctypes.c_uint64()

    def exchange_frontier(first=False):
        # the first exchange of a BFS goes through GxB_Vector_bitmap_import, which makes q iso
        # true (bench.py does the same); later ones rewrite q's words in place
        if exchange == "view" and not first:
            with torch.cuda.stream(stream):
                qb = gdev.device_tensor(torch, gdev.vector_view(q).bitmap, words)
                for r, p in enumerate(parts):
                    cnt = p["hi_w"] - p["lo_w"]
                    if cnt:
                        qb[p["lo_w"]:p["hi_w"]].copy_(gdev.device_tensor(torch, gdev.vector_view(ql[r]).bitmap, cnt))
            ok(lib.GxB_Vector_device_touch(q), "touch")
        else:
            for r, p in enumerate(parts):
                cnt = p["hi_w"] - p["lo_w"]
                if cnt:
                    ok(lib.GxB_Vector_bitmap_export(ql[r], ctypes.c_void_p(gathered.data_ptr() + 8 * r * slot), cnt),
                       "export")
            ok(lib.GxB_Vector_bitmap_import(q, ctypes.c_void_p(gathered.data_ptr()), words), "import")

    rng = np.random.default_rng(scale + world)
    for src in [int(np.argmax(deg)), int(rng.choice(np.flatnonzero(deg > 0)))]:
        for x in v + ql:
            ok(lib.GrB_Vector_clear(x), "clear")
        for r, p in enumerate(parts):
            if p["lo"] <= src < p["hi"]:
                ok(lib.GrB_Vector_setElement_BOOL(ql[r], True, src - p["lo"]), "root")
        exchange_frontier(first=True)
        d = 0
        while True:
            d += 1
            for r, p in enumerate(parts):
                ok(lib.GrB_Vector_assign_INT32(v[r], ql[r], None, d, lib.GrB_ALL, p["hi"] - p["lo"], None), "assign")
            for r in range(world):
                ok(lib.GrB_mxv(ql[r], v[r], None, sr, AT[r], q, lib.GrB_DESC_RSC), "mxv")
            exchange_frontier()
            ok(lib.GrB_Vector_nvals(ctypes.byref(nv), q), "nvals")
            if nv.value == 0:
                break
        got = np.zeros(n, np.int32)
        for r, p in enumerate(parts):
            idx, lv = _extract_int32(lib, v[r])
            got[idx + p["lo"]] = lv
        lev, _, _ = O.bfs_levels(G, src)
        assert np.array_equal(got, lev), f"source {src}"
    for h in AT:
        ok(lib.GrB_Matrix_free(ctypes.byref(h)), "free")
    for h in v + ql + [q]:
        ok(lib.GrB_Vector_free(ctypes.byref(h)), "free")


@pytest.mark.parametrize("scale", [10, 14])
@pytest.mark.parametrize("world", [2, 3])
def test_sharded_bfs_pipelined_vs_oracle(env, scale, world):
    """bench.py's N > 1 loop as it runs by default: two frontier buffers, the
    host one level behind the device (graphblas_amd.dist.pipelined_levels) -- level d + 1's
    stamps, shard SpMVs, exchange and recount are enqueued before the host waits for level d's
    count through its publish ticket (GxB_Vector_publish_ticket / GxB_Vector_wait_ticket), which
    stays readable although level d + 1 was enqueued behind it.  Levels bit-exact vs the
    oracle; exactly one level is issued past the last."""
    gb, torch, stream = env
    from graphblas_amd import device as gdev
    from graphblas_amd import dist as gdist

    lib = gb.lib
    n = 1 << scale
    G = O.rmat(scale, 16, 42)
    deg = np.diff(G.indptr)
    parts = [gdist.partition(n, world, r) for r in range(world)]
    words, slot = parts[0]["words"], parts[0]["slot"]
    AT, v, ql = [], [], []
    for p in parts:
        nloc = p["hi"] - p["lo"]
        h = ctypes.c_void_p()
        ok(lib.GxB_Matrix_rmat(ctypes.byref(h), scale, 16, 42, 0x100, 0, p["lo"], p["hi"]), "rmat shard")
        AT.append(h)
        for lst, t in ((v, lib.GrB_INT32), (ql, lib.GrB_BOOL)):
            x = ctypes.c_void_p()
            ok(lib.GrB_Vector_new(ctypes.byref(x), t, nloc), "new")
            lst.append(x)
    bufs = []
    for _ in range(2):
        x = ctypes.c_void_p()
        ok(lib.GrB_Vector_new(ctypes.byref(x), lib.GrB_BOOL, n), "q")
        bufs.append(x)
    staged = torch.zeros(slot * world, dtype=torch.int64, device="cuda")
    sr = lib.GxB_ANY_PAIR_BOOL
    nv = ctypes.c_uint64()

    def gather_into(q, via_import):
        if via_import:  # the buffer's first exchange of a BFS makes it iso true
            for r, p in enumerate(parts):
                cnt = p["hi_w"] - p["lo_w"]
                if cnt:
                    ok(lib.GxB_Vector_bitmap_export(ql[r], ctypes.c_void_p(staged.data_ptr() + 8 * r * slot), cnt),
                       "export")
            ok(lib.GxB_Vector_bitmap_import(q, ctypes.c_void_p(staged.data_ptr()), words), "import")
        else:
            with torch.cuda.stream(stream):
                qb = gdev.device_tensor(torch, gdev.vector_view(q).bitmap, words)
                for r, p in enumerate(parts):
                    cnt = p["hi_w"] - p["lo_w"]
                    if cnt:
                        qb[p["lo_w"]:p["hi_w"]].copy_(gdev.device_tensor(torch, gdev.vector_view(ql[r]).bitmap, cnt))
            ok(lib.GxB_Vector_device_touch(q), "touch")
        t = ctypes.c_uint64()
        ok(lib.GxB_Vector_publish_ticket(ctypes.byref(t), q), "ticket")
        assert t.value > 0
        return q, t.value

    rng = np.random.default_rng(scale + 10 * world)
    for src in [int(np.argmax(deg)), int(rng.choice(np.flatnonzero(deg > 0)))]:
        for x in v + ql:
            ok(lib.GrB_Vector_clear(x), "clear")
        for r, p in enumerate(parts):
            if p["lo"] <= src < p["hi"]:
                ok(lib.GrB_Vector_setElement_BOOL(ql[r], True, src - p["lo"]), "root")
        gather_into(bufs[0], True)
        first = {1: True}
        issued = []

        def enqueue(d):
            issued.append(d)
            for r, p in enumerate(parts):
                ok(lib.GrB_Vector_assign_INT32(v[r], ql[r], None, d, lib.GrB_ALL, p["hi"] - p["lo"], None), "assign")
            for r in range(world):
                ok(lib.GrB_mxv(ql[r], v[r], None, sr, AT[r], bufs[(d - 1) % 2], lib.GrB_DESC_RSC), "mxv")
            return gather_into(bufs[d % 2], first.pop(d % 2, False))

        def count_of(tok):
            c = ctypes.c_uint64()
            ok(lib.GxB_Vector_wait_ticket(ctypes.byref(c), tok[0], ctypes.c_uint64(tok[1])), "wait ticket")
            return c.value

        nlev = gdist.pipelined_levels(enqueue, count_of, max_levels=n + 2)
        got = np.zeros(n, np.int32)
        for r, p in enumerate(parts):
            idx, lv = _extract_int32(lib, v[r])
            got[idx + p["lo"]] = lv
        lev, _, _ = O.bfs_levels(G, src)
        assert np.array_equal(got, lev), f"source {src}"
        assert nlev == int(lev.max()) and issued == list(range(1, nlev + 2))
        ok(lib.GrB_Vector_nvals(ctypes.byref(nv), bufs[nlev % 2]), "nvals")
        assert nv.value == 0
    # a ticket superseded by a later publish of the same vector is refused, never misread
    t_old = gather_into(bufs[0], False)[1]
    gather_into(bufs[0], False)
    torch.cuda.synchronize()
    c = ctypes.c_uint64()
    assert lib.GxB_Vector_wait_ticket(ctypes.byref(c), bufs[0], ctypes.c_uint64(t_old)) == -3
    for h in AT:
        ok(lib.GrB_Matrix_free(ctypes.byref(h)), "free")
    for h in v + ql + bufs:
        ok(lib.GrB_Vector_free(ctypes.byref(h)), "free")


@pytest.mark.parametrize("scale", [10, 14])
@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("balanced", [False, True])
def test_sharded_bfs_peer_windows_vs_oracle(env, scale, world, balanced):
    """the sharded loop's exchange without a host-issued collective
    (GxB_PeerWindow_*, csrc/gb_peer.hip).  Every shard owns a window and its own two frontier
    buffers; the windows are linked with GxB_PeerWindow_attach (the same mapping an IPC-opened
    peer window gives, here inside one process and one GPU); per level every shard's GrB_mxv is
    followed by GxB_PeerWindow_put of its slice into every window, then GxB_PeerWindow_wait
    assembles each shard's full frontier on the device and publishes its count -- read through
    a publish ticket one level behind (dist.pipelined_levels).  Levels bit-exact vs the oracle,
    every shard's frontier equal, and no wait timed out."""
    gb, torch, stream = env
    from graphblas_amd import dist as gdist

    lib = gb.lib
    n = 1 << scale
    G = O.rmat(scale, 16, 42)
    deg = np.diff(G.indptr)
    bounds = None
    if balanced:  # 1-D row blocks balanced by the A^T shards' entries (in-degrees)
        words = (n + 63) // 64
        din = np.zeros(words * 64, np.int64)
        din[:n] = np.bincount(G.indices, minlength=n)
        bounds = gdist.balanced_bounds(din.reshape(words, 64).sum(1), world)
    parts = [gdist.partition(n, world, r, bounds) for r in range(world)]
    bvec = [p["lo_w"] for p in parts] + [parts[0]["words"]]
    AT, v, ql, win = [], [], [], []
    qb = [[], []]
    for r, p in enumerate(parts):
        nloc = p["hi"] - p["lo"]
        h = ctypes.c_void_p()
        ok(lib.GxB_Matrix_rmat(ctypes.byref(h), scale, 16, 42, 0x100, 0, p["lo"], p["hi"]), "rmat shard")
        AT.append(h)
        for lst, t, sz in ((v, lib.GrB_INT32, nloc), (ql, lib.GrB_BOOL, nloc), (qb[0], lib.GrB_BOOL, n),
                           (qb[1], lib.GrB_BOOL, n)):
            x = ctypes.c_void_p()
            ok(lib.GrB_Vector_new(ctypes.byref(x), t, sz), "new")
            lst.append(x)
        w = ctypes.c_void_p()
        ok(lib.GxB_PeerWindow_new(ctypes.byref(w), n, world, r, (ctypes.c_uint64 * (world + 1))(*bvec)), "window")
        win.append(w)
    for r in range(world):
        for k in range(world):
            if k != r:
                ok(lib.GxB_PeerWindow_attach(win[r], k, win[k]), "attach")
    sr = lib.GxB_ANY_PAIR_BOOL

    def exchange(tgt):
        for r in range(world):
            ok(lib.GxB_PeerWindow_put(win[r], ql[r]), "put")
        for r in range(world):
            ok(lib.GxB_PeerWindow_wait(qb[tgt][r], win[r]), "wait")
        t = ctypes.c_uint64()
        ok(lib.GxB_Vector_publish_ticket(ctypes.byref(t), qb[tgt][0]), "ticket")
        return qb[tgt][0], t.value

    rng = np.random.default_rng(scale + 10 * world)
    for src in [int(np.argmax(deg)), int(rng.choice(np.flatnonzero(deg > 0)))]:
        for x in v + ql:
            ok(lib.GrB_Vector_clear(x), "clear")
        for r, p in enumerate(parts):
            if p["lo"] <= src < p["hi"]:
                ok(lib.GrB_Vector_setElement_BOOL(ql[r], True, src - p["lo"]), "root")
        exchange(0)
        issued = []

        def enqueue(d):
            issued.append(d)
            for r, p in enumerate(parts):
                ok(lib.GrB_Vector_assign_INT32(v[r], ql[r], None, d, lib.GrB_ALL, p["hi"] - p["lo"], None), "assign")
            for r in range(world):
                ok(lib.GrB_mxv(ql[r], v[r], None, sr, AT[r], qb[(d - 1) % 2][r], lib.GrB_DESC_RSC), "mxv")
            return exchange(d % 2)

        def count_of(tok):
            c = ctypes.c_uint64()
            ok(lib.GxB_Vector_wait_ticket(ctypes.byref(c), tok[0], ctypes.c_uint64(tok[1])), "wait ticket")
            return c.value

        nlev = gdist.pipelined_levels(enqueue, count_of, max_levels=n + 2)
        got = np.zeros(n, np.int32)
        for r, p in enumerate(parts):
            idx, lv = _extract_int32(lib, v[r])
            got[idx + p["lo"]] = lv
        lev, _, _ = O.bfs_levels(G, src)
        assert np.array_equal(got, lev), f"source {src}"
        assert nlev == int(lev.max()) and issued == list(range(1, nlev + 2))
        # every shard assembled the same (empty) last frontier
        for r in range(world):
            nv = ctypes.c_uint64()
            ok(lib.GrB_Vector_nvals(ctypes.byref(nv), qb[nlev % 2][r]), "nvals")
            assert nv.value == 0
    # a mid-BFS frontier is the same on every shard (the bitmaps, word for word)
    from graphblas_amd import device as gdev
    ok(lib.GrB_Vector_clear(ql[0]), "clear")
    for r in range(1, world):
        ok(lib.GrB_Vector_clear(ql[r]), "clear")
    p0 = parts[0]
    for i in range(0, p0["hi"] - p0["lo"], 3):
        ok(lib.GrB_Vector_setElement_BOOL(ql[0], True, i), "set")
    exchange(1)
    torch.cuda.synchronize()
    ref = gdev.device_tensor(torch, gdev.vector_view(qb[1][0]).bitmap, parts[0]["words"]).cpu()
    for r in range(1, world):
        assert torch.equal(gdev.device_tensor(torch, gdev.vector_view(qb[1][r]).bitmap, parts[0]["words"]).cpu(), ref)
    for r in range(world):
        e = ctypes.c_int64()
        ok(lib.GxB_PeerWindow_error(ctypes.byref(e), win[r]), "error")
        assert e.value == 0
        ok(lib.GxB_PeerWindow_free(ctypes.byref(win[r])), "free window")
    for h in AT:
        ok(lib.GrB_Matrix_free(ctypes.byref(h)), "free")
    for h in v + ql + qb[0] + qb[1]:
        ok(lib.GrB_Vector_free(ctypes.byref(h)), "free")


def test_peer_window_wait_times_out_instead_of_hanging(env):
    """a wait whose peer never puts ends after the timeout (knob peer_timeout_ms) with an empty
    frontier and the window's error word raised -- the kernel does not spin forever"""
    gb, torch, stream = env
    lib = gb.lib
    n = 1 << 10
    w = [ctypes.c_void_p(), ctypes.c_void_p()]
    for r in range(2):
        ok(lib.GxB_PeerWindow_new(ctypes.byref(w[r]), n, 2, r, None), "window")
    ok(lib.GxB_PeerWindow_attach(w[0], 1, w[1]), "attach")
    ok(lib.GxB_PeerWindow_attach(w[1], 0, w[0]), "attach")
    ql, q = ctypes.c_void_p(), ctypes.c_void_p()
    ok(lib.GrB_Vector_new(ctypes.byref(ql), lib.GrB_BOOL, n // 2), "ql")
    ok(lib.GrB_Vector_new(ctypes.byref(q), lib.GrB_BOOL, n), "q")
    ok(lib.GrB_Vector_setElement_BOOL(ql, True, 3), "set")
    try:
        ok(lib.GxB_Global_set_int(b"peer_timeout_ms", 50), "knob")
        ok(lib.GxB_PeerWindow_put(w[0], ql), "put")  # rank 1 never puts
        ok(lib.GxB_PeerWindow_wait(q, w[0]), "wait")
        nv = ctypes.c_uint64()
        ok(lib.GrB_Vector_nvals(ctypes.byref(nv), q), "nvals")
        assert nv.value == 0
        e = ctypes.c_int64()
        ok(lib.GxB_PeerWindow_error(ctypes.byref(e), w[0]), "error")
        assert e.value == 1
        # misuse is refused on the host: a wait without its put, a slice of the wrong size
        assert lib.GxB_PeerWindow_wait(q, w[1]) == lib.GrB_INVALID_VALUE
        assert lib.GxB_PeerWindow_put(w[1], q) == lib.GrB_DIMENSION_MISMATCH
    finally:
        lib.GxB_Global_set_int(b"peer_timeout_ms", 0)
        for r in range(2):
            lib.GxB_PeerWindow_free(ctypes.byref(w[r]))
        lib.GrB_Vector_free(ctypes.byref(ql))
        lib.GrB_Vector_free(ctypes.byref(q))


@pytest.mark.parametrize("scale", [10, 13])
@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("k", [7, 64])
@pytest.mark.parametrize("semiring", ["GrB_LOR_LAND_SEMIRING_BOOL", "GxB_ANY_PAIR_BOOL"])
def test_sharded_msbfs_mxm_vs_oracle(env, scale, world, k, semiring):
    """bench.py config3_msbfs_sharded: per level
    Vloc_r<Qloc_r.V> = d;  Qloc_r<!Vloc_r.S, replace> = Q lor.land (A^T_r)^T   (GrB_DESC_RSCT1)
    then each shard's column words (k bits per vertex) are written into Q's words through
    GxB_Matrix_colwords_view, and GxB_Matrix_colwords_touch recounts Q."""
    gb, torch, stream = env
    from graphblas_amd import device as gdev
    from graphblas_amd import dist as gdist

    lib = gb.lib
    n = 1 << scale
    G = O.rmat(scale, 16, 42)
    deg = np.diff(G.indptr)
    rng = np.random.default_rng(scale * 10 + k)
    roots = rng.choice(np.flatnonzero(deg > 0), k, replace=False).astype(np.uint64)
    roots[0] = int(np.argmax(deg))
    parts = [gdist.partition(n, world, r) for r in range(world)]
    AT, Ql, Vl = [], [], []
    for p in parts:
        nloc = p["hi"] - p["lo"]
        h = ctypes.c_void_p()
        ok(lib.GxB_Matrix_rmat(ctypes.byref(h), scale, 16, 42, 0x100, 0, p["lo"], p["hi"]), "rmat shard")
        AT.append(h)
        for lst, t in ((Ql, lib.GrB_BOOL), (Vl, lib.GrB_INT32)):
            x = ctypes.c_void_p()
            ok(lib.GrB_Matrix_new(ctypes.byref(x), t, k, nloc), "new")
            lst.append(x)
    Q = ctypes.c_void_p()
    ok(lib.GrB_Matrix_new(ctypes.byref(Q), lib.GrB_BOOL, k, n), "Q")
    qi = np.arange(k, dtype=np.uint64)
    ok(lib.GxB_Matrix_build_Scalar_BOOL(Q, ctypes.c_void_p(qi.ctypes.data), ctypes.c_void_p(roots.ctypes.data), True,
                                        k), "build Q")
    keep = []
    for r, p in enumerate(parts):
        mine = (roots >= p["lo"]) & (roots < p["hi"])
        li = np.flatnonzero(mine).astype(np.uint64)
        lj = (roots[mine] - p["lo"]).astype(np.uint64)
        keep += [li, lj]
        if li.size:
            ok(lib.GxB_Matrix_build_Scalar_BOOL(Ql[r], ctypes.c_void_p(li.ctypes.data), ctypes.c_void_p(lj.ctypes.data),
                                                True, li.size), "build Qloc")
    sr = getattr(lib, semiring)
    nv = ctypes.c_uint64()
    d = 0
    while True:
        d += 1
        for r, p in enumerate(parts):
            nloc = p["hi"] - p["lo"]
            ok(lib.GrB_Matrix_assign_INT32(Vl[r], Ql[r], None, d, lib.GrB_ALL, k, lib.GrB_ALL, nloc, None), "stamp")
        for r in range(world):
            ok(lib.GrB_mxm(Ql[r], Vl[r], None, sr, Q, AT[r], lib.GrB_DESC_RSCT1), "mxm")
        with torch.cuda.stream(stream):
            qptr, qn = gdev.colwords_view(Q)
            qw = gdev.device_tensor(torch, qptr, qn)
            for r, p in enumerate(parts):
                ptr, cnt = gdev.colwords_view(Ql[r])
                qw[p["lo"]:p["lo"] + cnt].copy_(gdev.device_tensor(torch, ptr, cnt))
        ok(lib.GxB_Matrix_colwords_touch(Q), "touch")
        ok(lib.GrB_Matrix_nvals(ctypes.byref(nv), Q), "nvals")
        if nv.value == 0:
            break
    got = np.zeros((k, n), np.int32)
    for r, p in enumerate(parts):
        ok(lib.GrB_Matrix_nvals(ctypes.byref(nv), Vl[r]), "nvals V")
        m = nv.value
        vi, vj, vx = np.empty(m, np.uint64), np.empty(m, np.uint64), np.empty(m, np.int32)
        cnt = ctypes.c_uint64(m)
        ok(lib.GrB_Matrix_extractTuples_INT32(ctypes.c_void_p(vi.ctypes.data), ctypes.c_void_p(vj.ctypes.data),
                                              ctypes.c_void_p(vx.ctypes.data), ctypes.byref(cnt), Vl[r]), "extract")
        got[vi.astype(np.int64), vj.astype(np.int64) + p["lo"]] = vx
    for i, s in enumerate(roots):
        lev, _, _ = O.bfs_levels(G, int(s))
        assert np.array_equal(got[i], lev), f"root {s} (row {i})"
    for h in AT + Ql + Vl + [Q]:
        ok(lib.GrB_Matrix_free(ctypes.byref(h)), "free")


@pytest.mark.parametrize("scale", [9, 11])
@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("method", [0, 1])  # spgemm_method: 0 hash Gustavson (default), 1 ESC
def test_sharded_spgemm_plus_times_vs_oracle(env, scale, world, method):
    """bench.py config5_spgemm at N > 1: rank r holds rows [lo, hi) of A (FP64 U[0,1)), which is
    also its panel of B; B is assembled from the row panels (dist.concat_row_panels, the assembly
    RowPanelAllGather.run performs after its broadcasts) and imported with
    GxB_Matrix_import_device; each rank then runs C_r = A_r plus.times B (GrB_mxm)."""
    gb, torch, stream = env
    from graphblas_amd import device as gdev
    from graphblas_amd import dist as gdist

    lib = gb.lib
    n = 1 << scale
    G = O.rmat(scale, 16, 42, values="FP64", value_seed=2)
    parts = [gdist.partition(n, world, r) for r in range(world)]
    A, panels = [], []
    for p in parts:
        h = ctypes.c_void_p()
        ok(lib.GxB_Matrix_rmat(ctypes.byref(h), scale, 16, 42, 2, 2, p["lo"], p["hi"]), "rmat fp64 panel")
        A.append(h)
        va = gdev.matrix_view(h)
        panels.append((gdev.device_tensor(torch, va.rowptr, va.nrows + 1),
                       gdev.device_tensor(torch, va.colidx, va.nvals, "<i4"),
                       gdev.device_tensor(torch, va.values, 1 if va.iso else va.nvals, "<f8"), bool(va.iso)))
    with torch.cuda.stream(stream):
        brp, bci, bvx, biso = gdist.concat_row_panels(torch, panels)
    B = ctypes.c_void_p()
    ok(lib.GxB_Matrix_import_device(ctypes.byref(B), lib.GrB_FP64, n, n, ctypes.c_void_p(brp.data_ptr()),
                                    ctypes.c_void_p(bci.data_ptr()), ctypes.c_void_p(bvx.data_ptr()), bci.numel(),
                                    bool(biso)), "import B")
    gb.set_knob("spgemm_method", method)
    try:
        for r, p in enumerate(parts):
            nloc = p["hi"] - p["lo"]
            C = ctypes.c_void_p()
            ok(lib.GrB_Matrix_new(ctypes.byref(C), lib.GrB_FP64, nloc, n), "C")
            ok(lib.GrB_mxm(C, None, None, lib.GrB_PLUS_TIMES_SEMIRING_FP64, A[r], B, None), "mxm")
            vc = gdev.matrix_view(C)
            stream.synchronize()  # the views are read on torch's stream: wait for the library's
            crp = gdev.device_tensor(torch, vc.rowptr, nloc + 1).cpu().numpy()
            cci = gdev.device_tensor(torch, vc.colidx, vc.nvals, "<i4").cpu().numpy().astype(np.int64)
            cvx = gdev.device_tensor(torch, vc.values, vc.nvals, "<f8").cpu().numpy()
            lo, hi = p["lo"], p["hi"]
            sub = O.Csr(nloc, n, "FP64", G.indptr[lo:hi + 1] - G.indptr[lo], G.indices[G.indptr[lo]:G.indptr[hi]],
                        G.values[G.indptr[lo]:G.indptr[hi]])
            ref = O.mxm(O.Csr.empty(nloc, n, "FP64"), sub, G, ("PLUS", "TIMES", "FP64"))
            assert np.array_equal(crp, ref.indptr) and np.array_equal(cci, ref.indices), f"shard {r} structure"
            if method == 1:  # ESC folds in ascending k like the oracle: bit-identical
                assert np.array_equal(cvx, ref.values), f"shard {r} values"
            else:
                assert np.allclose(cvx, ref.values, rtol=1e-9, atol=0), f"shard {r} values"
            ok(lib.GrB_Matrix_free(ctypes.byref(C)), "free C")
    finally:
        gb.set_knob("spgemm_method", 0)
    for h in A + [B]:
        ok(lib.GrB_Matrix_free(ctypes.byref(h)), "free")
