"""BFS level speculation (csrc/gb_ops.hip, knob bfs_spec): after a level of the notebook loop
(reference notebooks/Example B.1 -- Level BFS.ipynb cell 8: `v<q.V> = d; q<!v.S,replace> = q
(+).(x) A`) the library enqueues the next level behind it and installs that result when the host
issues exactly the predicted stamp and SpMV; anything else rolls it back first.  These tests drive
the loop through the C ABI with speculation on (the default) and check that

* the levels equal the oracle's and the speculation was actually adopted (GxB_Global_get_int
  "stat_bfs_spec_adopted"), for any_pair and lor_land, vxm and mxv, value and structural stamps;
* every interleaving a caller might do observes no speculative state: reading v mid-loop (nvals,
  extractTuples), a stamp value other than d + 1, a level without the stamp, a different semiring
  or descriptor, touching another object;
and the same with speculation off (knob bfs_spec = 1) gives identical results.

The expected results come from a direct numpy restatement of the loop (any stamp sequence), which
the oracle's level BFS pins for the plain d = 1, 2, ... loop."""
import ctypes

import numpy as np
import pytest

import oracle as O

pytestmark = pytest.mark.gpu
U64 = ctypes.c_uint64


@pytest.fixture(scope="module")
def gb():
    import graphblas_amd

    return graphblas_amd


@pytest.fixture(scope="module")
def graph(gb):
    G = O.rmat(13, 16, 42)
    r, c, _ = G.to_coo()
    A = gb.Matrix.from_coo(r, c, True, nrows=G.nrows, ncols=G.ncols)
    return G, A


def stat(gb, key):
    v = ctypes.c_int64()
    assert gb.lib.GxB_Global_get_int(key.encode(), ctypes.byref(v)) == 0
    return v.value


def ok(rc, what=""):
    assert rc == 0, f"{what}: GrB_Info {rc}"


def read_vec(lib, v, n):
    nv = U64()
    ok(lib.GrB_Vector_nvals(ctypes.byref(nv), v), "nvals")
    idx = np.empty(nv.value, np.uint64)
    x = np.empty(nv.value, np.int32)
    ok(lib.GrB_Vector_extractTuples_INT32(ctypes.c_void_p(idx.ctypes.data), ctypes.c_void_p(x.ctypes.data),
                                          ctypes.byref(nv), v), "extract")
    out = np.zeros(n, np.int32)
    out[idx.astype(np.int64)] = x
    return out, nv.value


def ref_loop(G, src, stamps, mxv=False, stop=True):
    """numpy restatement: for level k the stamp value stamps[k] (None: no stamp that level);
    v<q> = s; q<!v.S, replace> = q (any.pair) A  (vxm: successors; mxv on A: predecessors)"""
    n = G.nrows
    rows = np.repeat(np.arange(n), np.diff(G.indptr))
    v = np.zeros(n, np.int32)
    have = np.zeros(n, bool)
    q = np.zeros(n, bool)
    q[src] = True
    for s in stamps:
        if s is not None:
            v[q] = s
            have |= q
        nxt = np.zeros(n, bool)
        if mxv:  # w(i) = OR_k A(i,k) q(k)
            nxt[rows[q[G.indices]]] = True
        else:    # w(j) = OR_i q(i) A(i,j)
            nxt[G.indices[q[rows]]] = True
        q = nxt & ~have
        if stop and not q.any():
            break
    return v, q


def run_loop(gb, A, n, src, stamps, sr_name="any_pair", mxv=False, stamp_desc=None, hooks=None, stop=True,
             counts=None):
    """the loop through the C ABI; hooks[k](q, v) runs after level k's nvals; stop=False keeps
    going after an empty frontier; counts collects each level's nvals(q)"""
    lib = gb.lib
    sr = lib.GxB_ANY_PAIR_BOOL if sr_name == "any_pair" else lib.GrB_LOR_LAND_SEMIRING_BOOL
    q, v = ctypes.c_void_p(), ctypes.c_void_p()
    ok(lib.GrB_Vector_new(ctypes.byref(q), lib.GrB_BOOL, n))
    ok(lib.GrB_Vector_new(ctypes.byref(v), lib.GrB_INT32, n))
    ok(lib.GrB_Vector_setElement_BOOL(q, True, int(src)))
    nv = U64()
    for k, s in enumerate(stamps):
        if s is not None:
            ok(lib.GrB_Vector_assign_INT32(v, q, None, s, lib.GrB_ALL, n, stamp_desc), "stamp")
        if mxv:
            ok(lib.GrB_mxv(q, v, None, sr, A._carg, q, lib.GrB_DESC_RSC), "mxv")
        else:
            ok(lib.GrB_vxm(q, v, None, sr, q, A._carg, lib.GrB_DESC_RSC), "vxm")
        ok(lib.GrB_Vector_nvals(ctypes.byref(nv), q), "nvals q")
        if counts is not None:
            counts.append(nv.value)
        if hooks and k in hooks:
            hooks[k](q, v)
        if stop and nv.value == 0:
            break
    got, cnt = read_vec(lib, v, n)
    qb, _ = read_vec_bool(lib, q, n)
    lib.GrB_Vector_free(ctypes.byref(q))
    lib.GrB_Vector_free(ctypes.byref(v))
    return got, qb


def read_vec_bool(lib, q, n):
    nv = U64()
    ok(lib.GrB_Vector_nvals(ctypes.byref(nv), q))
    idx = np.empty(nv.value, np.uint64)
    x = np.empty(nv.value, np.bool_)
    ok(lib.GrB_Vector_extractTuples_BOOL(ctypes.c_void_p(idx.ctypes.data), ctypes.c_void_p(x.ctypes.data),
                                         ctypes.byref(nv), q))
    out = np.zeros(n, bool)
    out[idx.astype(np.int64)] = True
    return out, nv.value


def roots(G, k=3):
    deg = np.diff(G.indptr)
    return [int(np.argmax(deg)), int(np.flatnonzero(deg > 0)[7]), int(np.flatnonzero(deg > 0)[-3])][:k]


@pytest.mark.parametrize("sr_name", ["any_pair", "lor_land"])
@pytest.mark.parametrize("mxv", [False, True])
@pytest.mark.parametrize("structural", [False, True])
def test_spec_levels_match_oracle(gb, graph, sr_name, mxv, structural):
    G, A = graph
    n = G.nrows
    a0 = stat(gb, "stat_bfs_spec_adopted")
    for src in roots(G):
        got, q = run_loop(gb, A, n, src, list(range(1, 64)), sr_name, mxv,
                          gb.lib.GrB_DESC_S if structural else None)
        if not mxv:
            ref, _, _ = O.bfs_levels(G, src)
            assert np.array_equal(got, ref)
        exp, _ = ref_loop(G, src, list(range(1, 64)), mxv)
        assert np.array_equal(got, exp) and not q.any()
    assert stat(gb, "stat_bfs_spec_adopted") > a0, "the speculation was never adopted"


def test_spec_off_gives_the_same(gb, graph):
    G, A = graph
    src = roots(G)[0]
    on, _ = run_loop(gb, A, G.nrows, src, list(range(1, 64)))
    gb.set_knob("bfs_spec", 1)
    try:
        a0 = stat(gb, "stat_bfs_spec_adopted")
        off, _ = run_loop(gb, A, G.nrows, src, list(range(1, 64)))
        assert stat(gb, "stat_bfs_spec_adopted") == a0
    finally:
        gb.set_knob("bfs_spec", 0)
    assert np.array_equal(on, off)


def test_spec_past_the_empty_level(gb, graph):
    """levels issued after the frontier emptied: the speculated level on an empty q ends its
    launch early (a zero count, an empty result, no stamp); adopting it must look like a full
    level -- v unchanged, q empty, every count 0 -- and a loop that then stamps v again agrees"""
    G, A = graph
    n = G.nrows
    src = roots(G)[0]
    ref, _ = ref_loop(G, src, list(range(1, 64)))
    depth = int(ref.max())
    stamps = list(range(1, depth + 5))
    a0 = stat(gb, "stat_bfs_spec_adopted")
    counts = []
    got, q = run_loop(gb, A, n, src, stamps, stop=False, counts=counts)
    exp, eq = ref_loop(G, src, stamps, stop=False)
    assert np.array_equal(got, exp) and np.array_equal(q, eq) and not q.any()
    assert counts[depth - 1:] == [0] * (len(stamps) - depth + 1), counts
    assert stat(gb, "stat_bfs_spec_adopted") >= a0 + len(stamps) - 2
    gb.set_knob("spec_empty_exit", 1)  # the same loop with full launches on the empty levels
    try:
        counts_full = []
        full, _ = run_loop(gb, A, n, src, stamps, stop=False, counts=counts_full)
    finally:
        gb.set_knob("spec_empty_exit", 0)
    assert np.array_equal(full, got) and counts_full == counts


def test_spec_unexpected_stamps(gb, graph):
    """stamp values other than d + 1 (a repeated value, a jump, a skipped stamp): each breaks
    the prediction and must roll the speculated level back"""
    G, A = graph
    n = G.nrows
    src = roots(G)[0]
    for stamps in ([1, 2, 2, 3, 4, 5, 6, 7, 8, 9], [1, 2, 3, 7, 8, 9, 10, 11, 12], [1, 2, None, 3, 4, 5, 6, 7, 8],
                   [5, 4, 3, 2, 1, 0, -1, -2, -3]):
        r0 = stat(gb, "stat_bfs_spec_rollbacks")
        got, q = run_loop(gb, A, n, src, stamps)
        exp, eq = ref_loop(G, src, stamps)
        assert np.array_equal(got, exp), stamps
        assert np.array_equal(q, eq), stamps
        assert stat(gb, "stat_bfs_spec_rollbacks") > r0


def test_spec_reads_and_writes_mid_loop(gb, graph):
    """nvals / extractTuples of v between levels (v carries the speculative stamp until the
    rollback), a read of an unrelated object (no rollback needed) and an assign to it"""
    G, A = graph
    n = G.nrows
    lib = gb.lib
    src = roots(G)[0]
    ref, _, _ = O.bfs_levels(G, src)
    seen = {}

    def read_v(q, v):
        got, cnt = read_vec(lib, v, n)
        seen[len(seen)] = (got.copy(), cnt)

    other = ctypes.c_void_p()
    ok(lib.GrB_Vector_new(ctypes.byref(other), lib.GrB_INT64, n))

    def touch_other(q, v):
        nv = U64()
        ok(lib.GrB_Vector_nvals(ctypes.byref(nv), other))
        ok(lib.GrB_Vector_assign_INT64(other, None, None, 7, lib.GrB_ALL, n, None))

    hooks = {1: read_v, 2: touch_other, 3: read_v}
    got, _ = run_loop(gb, A, n, src, list(range(1, 64)), hooks=hooks)
    assert np.array_equal(got, ref)
    # what v held after levels 2 and 4 (hooks 1 and 3): the stamps up to that level only
    for (lv, cnt), lvl in zip(seen.values(), (2, 4)):
        exp = np.where((ref > 0) & (ref <= lvl), ref, 0)
        assert np.array_equal(lv, exp) and cnt == int((exp > 0).sum())
    lib.GrB_Vector_free(ctypes.byref(other))


def test_spec_other_call_between_stamp_and_spmv(gb, graph):
    """the predicted stamp is issued (absorbed), then another call reads v before the SpMV: the
    rollback re-issues the absorbed stamp, so v holds it"""
    G, A = graph
    n = G.nrows
    lib = gb.lib
    src = roots(G)[0]
    sr = lib.GxB_ANY_PAIR_BOOL
    q, v = ctypes.c_void_p(), ctypes.c_void_p()
    ok(lib.GrB_Vector_new(ctypes.byref(q), lib.GrB_BOOL, n))
    ok(lib.GrB_Vector_new(ctypes.byref(v), lib.GrB_INT32, n))
    ok(lib.GrB_Vector_setElement_BOOL(q, True, src))
    nv = U64()
    ref, _, _ = O.bfs_levels(G, src)
    d = 0
    while True:
        d += 1
        ok(lib.GrB_Vector_assign_INT32(v, q, None, d, lib.GrB_ALL, n, None))
        if d == 3:
            got, cnt = read_vec(lib, v, n)  # v after the level-3 stamp, before the SpMV
            exp = np.where((ref > 0) & (ref <= 3), ref, 0)
            assert np.array_equal(got, exp) and cnt == int((exp > 0).sum())
        ok(lib.GrB_vxm(q, v, None, sr, q, A._carg, lib.GrB_DESC_RSC))
        ok(lib.GrB_Vector_nvals(ctypes.byref(nv), q))
        if nv.value == 0:
            break
    got, _ = read_vec(lib, v, n)
    assert np.array_equal(got, ref)
    lib.GrB_Vector_free(ctypes.byref(q))
    lib.GrB_Vector_free(ctypes.byref(v))


def test_spec_changed_call_shape(gb, graph):
    """the predicted stamp, then an SpMV that differs from the prediction (another semiring, a
    non-replace descriptor): rolled back, the absorbed stamp re-issued, results as without
    speculation"""
    G, A = graph
    n = G.nrows
    lib = gb.lib
    src = roots(G)[0]
    for variant in ("semiring", "descriptor"):
        results = []
        for spec in (0, 1):
            gb.set_knob("bfs_spec", spec)
            q, v = ctypes.c_void_p(), ctypes.c_void_p()
            ok(lib.GrB_Vector_new(ctypes.byref(q), lib.GrB_BOOL, n))
            ok(lib.GrB_Vector_new(ctypes.byref(v), lib.GrB_INT32, n))
            ok(lib.GrB_Vector_setElement_BOOL(q, True, src))
            nv = U64()
            for d in range(1, 7):
                ok(lib.GrB_Vector_assign_INT32(v, q, None, d, lib.GrB_ALL, n, None))
                sr, desc = lib.GxB_ANY_PAIR_BOOL, lib.GrB_DESC_RSC
                if d == 3:
                    if variant == "semiring":
                        sr = lib.GrB_LOR_LAND_SEMIRING_BOOL
                    else:
                        desc = lib.GrB_DESC_SC
                ok(lib.GrB_vxm(q, v, None, sr, q, A._carg, desc))
                ok(lib.GrB_Vector_nvals(ctypes.byref(nv), q))
                if nv.value == 0:
                    break
            results.append((read_vec(lib, v, n)[0], read_vec_bool(lib, q, n)[0]))
            lib.GrB_Vector_free(ctypes.byref(q))
            lib.GrB_Vector_free(ctypes.byref(v))
        gb.set_knob("bfs_spec", 0)
        assert np.array_equal(results[0][0], results[1][0]) and np.array_equal(results[0][1], results[1][1])


def test_spec_rollback_failure_is_recorded_on_v(gb, graph):
    """the predicted stamp is absorbed, then an SpMV of another shape rolls the
    speculation back; re-issuing the absorbed stamp fails (injected).  The failure is an
    execution error of v -- recorded on v (GrB_INVALID_OBJECT from then on), never raised
    across the C boundary -- and q stays usable."""
    G, A = graph
    n = G.nrows
    lib = gb.lib
    src = roots(G)[0]
    q, v = ctypes.c_void_p(), ctypes.c_void_p()
    ok(lib.GrB_Vector_new(ctypes.byref(q), lib.GrB_BOOL, n))
    ok(lib.GrB_Vector_new(ctypes.byref(v), lib.GrB_INT32, n))
    ok(lib.GrB_Vector_setElement_BOOL(q, True, src))
    nv = U64()
    r0 = stat(gb, "stat_bfs_spec_rollbacks")
    try:
        for d in range(1, 4):
            ok(lib.GrB_Vector_assign_INT32(v, q, None, d, lib.GrB_ALL, n, None), "stamp")
            sr = lib.GxB_ANY_PAIR_BOOL
            if d == 3:
                gb.set_knob("inject_spec_fail", 1)
                sr = lib.GrB_LOR_LAND_SEMIRING_BOOL  # not the predicted SpMV: rollback
            lib.GrB_vxm(q, v, None, sr, q, A._carg, lib.GrB_DESC_RSC)
            gb.set_knob("inject_spec_fail", 0)
            ok(lib.GrB_Vector_nvals(ctypes.byref(nv), q), "nvals q")
    finally:
        gb.set_knob("inject_spec_fail", 0)
    assert stat(gb, "stat_bfs_spec_rollbacks") > r0
    assert lib.GrB_Vector_nvals(ctypes.byref(nv), v) == -104  # GrB_INVALID_OBJECT
    ok(lib.GrB_Vector_nvals(ctypes.byref(nv), q), "q stays valid")
    lib.GrB_Vector_free(ctypes.byref(q))
    lib.GrB_Vector_free(ctypes.byref(v))


def test_spec_absorb_needs_valid_call(gb, graph):
    """a stamp the normal path would treat differently (ni != n with GrB_ALL) is not
    absorbed: the speculation rolls back and the normal path runs -- same levels as the oracle"""
    G, A = graph
    n = G.nrows
    lib = gb.lib
    src = roots(G)[0]
    ref, _, _ = O.bfs_levels(G, src)
    q, v = ctypes.c_void_p(), ctypes.c_void_p()
    ok(lib.GrB_Vector_new(ctypes.byref(q), lib.GrB_BOOL, n))
    ok(lib.GrB_Vector_new(ctypes.byref(v), lib.GrB_INT32, n))
    ok(lib.GrB_Vector_setElement_BOOL(q, True, src))
    nv = U64()
    r0 = stat(gb, "stat_bfs_spec_rollbacks")
    d = 0
    while True:
        d += 1
        ok(lib.GrB_Vector_assign_INT32(v, q, None, d, lib.GrB_ALL, n + 1 if d == 3 else n, None), "stamp")
        ok(lib.GrB_vxm(q, v, None, lib.GxB_ANY_PAIR_BOOL, q, A._carg, lib.GrB_DESC_RSC), "vxm")
        ok(lib.GrB_Vector_nvals(ctypes.byref(nv), q))
        if nv.value == 0:
            break
    got, _ = read_vec(lib, v, n)
    assert np.array_equal(got, ref)
    assert stat(gb, "stat_bfs_spec_rollbacks") > r0
    lib.GrB_Vector_free(ctypes.byref(q))
    lib.GrB_Vector_free(ctypes.byref(v))


def test_value_mask_false_entries_no_host_push(gb, graph):
    """the host proves push only from a lower bound on the open rows.  A value mask
    whose stored entries are all false opens no row, so its stored count must not be read as open
    rows (no host-decided push); the BFS's first level (v just cleared, structural stamp) is the
    positive control: there the host does decide push."""
    G, A = graph
    n = G.nrows
    lib = gb.lib
    src = roots(G)[0]
    h0 = stat(gb, "stat_spmv_host_push")
    run_loop(gb, A, n, src, list(range(1, 64)))
    assert stat(gb, "stat_spmv_host_push") > h0, "positive control: first BFS level decided on the host"
    u, m, w = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_void_p()
    ok(lib.GrB_Vector_new(ctypes.byref(u), lib.GrB_BOOL, n))
    ok(lib.GrB_Vector_new(ctypes.byref(m), lib.GrB_BOOL, n))
    ok(lib.GrB_Vector_new(ctypes.byref(w), lib.GrB_BOOL, n))
    ok(lib.GrB_Vector_setElement_BOOL(u, True, src))
    ok(lib.GrB_Vector_assign_BOOL(m, None, None, False, lib.GrB_ALL, n, None))  # n stored falses
    nv = U64()
    ok(lib.GrB_Vector_nvals(ctypes.byref(nv), m))
    assert nv.value == n
    for _ in range(2):  # the second call finds the zeroed output bitmap the first one left
        h1 = stat(gb, "stat_spmv_host_push")
        ok(lib.GrB_vxm(w, m, None, lib.GxB_ANY_PAIR_BOOL, u, A._carg, lib.GrB_DESC_R), "vxm")
        ok(lib.GrB_Vector_nvals(ctypes.byref(nv), w))
        assert nv.value == 0
        assert stat(gb, "stat_spmv_host_push") == h1
    for x in (u, m, w):
        lib.GrB_Vector_free(ctypes.byref(x))


def test_pending_root_is_unobservable(gb, graph):
    """`GrB_Vector_setElement_BOOL(q, true, src)` on an empty BOOL vector stays
    pending (no launch) and the first level's kernel pushes from src (gb_push_root; counter
    stat_bfs_root_push).  Every other use of q sees the entry: its count and tuples, q as a mask,
    q as the input of an SpMV of another shape, an assign into q, a second setElement -- each
    against the same calls with the deferral off (knob root_defer = 1) and the numpy loop."""
    G, A = graph
    n = G.nrows
    lib = gb.lib
    src = int(roots(G)[1])
    sr = lib.GxB_ANY_PAIR_BOOL
    nv = U64()

    def fresh(t=lib.GrB_BOOL):
        x = ctypes.c_void_p()
        ok(lib.GrB_Vector_new(ctypes.byref(x), t, n))
        return x

    def bits(x):
        ok(lib.GrB_Vector_nvals(ctypes.byref(nv), x))
        idx = np.empty(nv.value, np.uint64)
        val = np.empty(nv.value, np.bool_)
        ok(lib.GrB_Vector_extractTuples_BOOL(ctypes.c_void_p(idx.ctypes.data), ctypes.c_void_p(val.ctypes.data),
                                             ctypes.byref(nv), x))
        return sorted(idx.astype(np.int64).tolist()), val.tolist()

    succ = sorted(set(G.indices[G.indptr[src]:G.indptr[src + 1]].tolist()))
    results = []
    for knob in (0, 1):
        gb.set_knob("root_defer", knob)
        try:
            out = {}
            q = fresh()
            ok(lib.GrB_Vector_setElement_BOOL(q, True, src))
            out["tuples"] = bits(q)
            q2 = fresh()
            ok(lib.GrB_Vector_setElement_BOOL(q2, True, src))
            w = fresh()  # another shape: w = q2 any.pair A, no mask, w != q2
            ok(lib.GrB_vxm(w, None, None, sr, q2, A._carg, None), "vxm other shape")
            out["vxm_other"] = bits(w)[0]
            q3 = fresh()
            m = fresh()
            ok(lib.GrB_Vector_setElement_BOOL(q3, True, src))
            ok(lib.GrB_Vector_assign_BOOL(m, q3, None, True, lib.GrB_ALL, n, None), "q3 as a mask")
            out["as_mask"] = bits(m)[0]
            q4 = fresh()
            ok(lib.GrB_Vector_setElement_BOOL(q4, True, src))
            ok(lib.GrB_Vector_setElement_BOOL(q4, True, (src + 1) % n), "a second entry")
            out["two"] = bits(q4)[0]
            q5 = fresh()
            v5 = fresh(lib.GrB_INT32)
            ok(lib.GrB_Vector_setElement_BOOL(q5, True, src))
            ok(lib.GrB_Vector_assign_INT32(v5, q5, None, 1, lib.GrB_ALL, n, None), "stamp")
            ok(lib.GrB_Vector_nvals(ctypes.byref(nv), v5), "read v between the stamp and the SpMV")
            out["v_count"] = nv.value
            r0 = stat(gb, "stat_bfs_root_push")
            ok(lib.GrB_vxm(q5, v5, None, sr, q5, A._carg, lib.GrB_DESC_RSC), "level 1")
            out["level1"] = bits(q5)[0]
            q6, v6 = fresh(), fresh(lib.GrB_INT32)
            ok(lib.GrB_Vector_setElement_BOOL(q6, True, src))
            ok(lib.GrB_Vector_assign_INT32(v6, q6, None, 1, lib.GrB_ALL, n, None), "stamp")
            ok(lib.GrB_vxm(q6, v6, None, sr, q6, A._carg, lib.GrB_DESC_RSC), "level 1 (root consumed)")
            out["level1_consumed"] = bits(q6)[0]
            out["v6"] = read_vec(lib, v6, n)[0][src]
            out["root_pushes"] = stat(gb, "stat_bfs_root_push") - r0
            for x in (q, q2, w, q3, m, q4, q5, v5, q6, v6):
                lib.GrB_Vector_free(ctypes.byref(x))
            results.append(out)
        finally:
            gb.set_knob("root_defer", 0)
    on, off = results
    assert on["tuples"] == off["tuples"] == ([src], [True])
    assert on["vxm_other"] == off["vxm_other"] == succ
    assert on["as_mask"] == off["as_mask"] == [src]
    assert on["two"] == off["two"] == sorted({src, (src + 1) % n})
    assert on["v_count"] == off["v_count"] == 1
    expect = [j for j in succ if j != src]
    assert on["level1"] == off["level1"] == expect
    assert on["level1_consumed"] == off["level1_consumed"] == expect
    assert on["v6"] == off["v6"] == 1
    assert on["root_pushes"] >= 1 and off["root_pushes"] == 0
