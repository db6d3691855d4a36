#!/usr/bin/env python3
"""Generate tests/golden/reference_golden.json from the reference's own tests and docs.

Runs only in the build container (the reference tree does not exist on the GPU box).
The reference is read as TEXT: `ast` pulls the literal arguments of the
`Matrix.from_coo` / `Vector.from_coo` calls and the literal right-hand sides of
scalar asserts out of the named test functions; the docs' csv-tables are parsed
from the .rst.  Nothing from the reference is imported or executed.  Each case
records the file:line it came from.  The *operation* applied in each case is
restated here in words (it is the test's own statement, e.g.
``C(val_mask.V) << A.mxm(A, semiring.plus_times)``).

Also writes two survey-derived notebook results (SSSP distances / BFS levels
on the Intro-notebook 7x7 graph) computed independently with plain Python
Dijkstra / BFS, so the oracle is not checked against itself.
"""
import ast
import heapq
import json
import os
import re
import sys

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))


def _literal(node):
    return ast.literal_eval(node)


def from_coo_calls(relpath, funcname):
    """All X.from_coo(...) calls inside function `funcname`, in source order."""
    path = os.path.join(REF, relpath)
    tree = ast.parse(open(path).read())
    fn = None
    for node in ast.walk(tree):
        if isinstance(node, ast.FunctionDef) and node.name == funcname:
            fn = node
            break
    if fn is None:
        raise KeyError(f"{relpath}::{funcname}")
    calls = []
    for node in ast.walk(fn):
        if (
            isinstance(node, ast.Call)
            and isinstance(node.func, ast.Attribute)
            and node.func.attr == "from_coo"
            and isinstance(node.func.value, ast.Name)
        ):
            kind = node.func.value.id
            try:
                args = [_literal(a) for a in node.args]
                kw = {k.arg: _literal(k.value) for k in node.keywords}
            except ValueError:  # data in a variable (fixture style): resolve later
                args, kw = None, None
            calls.append(
                {"kind": kind, "args": args, "kw": kw, "line": node.lineno,
                 "src": f"graphblas/tests/{os.path.basename(relpath)}:{node.lineno}"
                 if "tests" in relpath else f"{relpath}:{node.lineno}"}
            )
    calls.sort(key=lambda c: c["line"])
    return calls, fn


def fixture_data(relpath, funcname, varname="data"):
    path = os.path.join(REF, relpath)
    tree = ast.parse(open(path).read())
    for node in ast.walk(tree):
        if isinstance(node, ast.FunctionDef) and node.name == funcname:
            for sub in ast.walk(node):
                if isinstance(sub, ast.Assign) and any(
                    isinstance(t, ast.Name) and t.id == varname for t in sub.targets
                ):
                    return _literal(sub.value), f"{relpath}:{sub.lineno}"
    raise KeyError(funcname)


def scalar_asserts(fn):
    """Literal constants compared in `assert X == <const>` statements, in order."""
    out = []
    for node in ast.walk(fn):
        if isinstance(node, ast.Assert) and isinstance(node.test, ast.Compare):
            cmp = node.test
            if len(cmp.ops) == 1 and isinstance(cmp.ops[0], ast.Eq):
                try:
                    out.append((_literal(cmp.comparators[0]), node.lineno))
                except ValueError:
                    pass
    out.sort(key=lambda t: t[1])
    return out


def coo(call):
    a, kw = call["args"], call["kw"]
    d = {"src": call["src"]}
    if call["kind"] == "Matrix":
        d.update(rows=list(a[0]), cols=list(a[1]), values=a[2] if len(a) > 2 else kw.get("values"))
        if "nrows" in kw:
            d["nrows"] = kw["nrows"]
        if "ncols" in kw:
            d["ncols"] = kw["ncols"]
    else:
        d.update(indices=list(a[0]), values=a[1] if len(a) > 1 else kw.get("values"))
        if "size" in kw:
            d["size"] = kw["size"]
    return d


def rst_tables(relpath):
    """Parse docs csv-tables into {title: {'header': [...], 'rows': {label: [cells]}}}."""
    text = open(os.path.join(REF, relpath)).read().splitlines()
    tables = []
    i = 0
    while i < len(text):
        line = text[i]
        m = re.match(r"\.\. csv-table:: (.*)", line)
        if m:
            title = m.group(1).strip()
            start = i + 1
            header = None
            rows = []
            i += 1
            while i < len(text) and (text[i].startswith("    ") or not text[i].strip()):
                s = text[i].strip()
                if s.startswith(":header:"):
                    header = [h.strip() for h in s[len(":header:"):].split(",")]
                elif s and not s.startswith(":"):
                    rows.append([c.strip() for c in s.split(",")])
                if not text[i].strip() and rows:
                    break
                i += 1
            tables.append({"title": title, "header": header, "rows": rows,
                           "src": f"{relpath}:{start}"})
            continue
        i += 1
    return tables


def table_to_matrix(t):
    hdr = t["header"]
    cols = [int(h) for h in hdr[1:]]
    rows, cs, vals = [], [], []
    for r in t["rows"]:
        label = int(r[0].strip("*"))
        for c, cell in zip(cols, r[1:]):
            if cell:
                rows.append(label); cs.append(c); vals.append(float(cell))
    return {"rows": rows, "cols": cs, "values": vals, "nrows": len(t["rows"]),
            "ncols": len(cols), "src": t["src"]}


def table_to_vector(t):
    hdr = t["header"]
    cells = t["rows"][0]
    idx, vals = [], []
    for h, cell in zip(hdr, cells):
        if cell:
            idx.append(int(h)); vals.append(float(cell))
    return {"indices": idx, "values": vals, "size": len(hdr), "src": t["src"]}


def rst_from_coo(relpath):
    """Literal Matrix/Vector.from_coo(...) calls inside code blocks of an .rst, in order."""
    text = open(os.path.join(REF, relpath)).read()
    out = []
    for m in re.finditer(r"gb\.(Matrix|Vector)\.from_coo\(", text):
        # find matching paren
        depth, j = 0, m.end() - 1
        while True:
            ch = text[j]
            if ch == "(":
                depth += 1
            elif ch == ")":
                depth -= 1
                if depth == 0:
                    break
            j += 1
        src = text[m.start() + 3 : j + 1]
        call = ast.parse(src, mode="eval").body
        args = [_literal(a) for a in call.args]
        kw = {k.arg: _literal(k.value) for k in call.keywords}
        line = text[: m.start()].count("\n") + 1
        out.append({"kind": m.group(1), "args": args, "kw": kw, "src": f"{relpath}:{line}",
                    "line": line})
    return out


def notebook_graph():
    import json as _j
    nb = _j.load(open(os.path.join(REF, "notebooks", "Intro to GraphBLAS + SSSP example.ipynb")))
    src = "".join(nb["cells"][2]["source"])
    data = ast.literal_eval(src.split("=", 1)[1].strip())
    return data


def dijkstra(n, rows, cols, w, src):
    adj = [[] for _ in range(n)]
    for r, c, x in zip(rows, cols, w):
        adj[r].append((c, x))
    dist = {src: 0}
    h = [(0, src)]
    while h:
        d, u = heapq.heappop(h)
        if d > dist.get(u, float("inf")):
            continue
        for v, x in adj[u]:
            if d + x < dist.get(v, float("inf")):
                dist[v] = d + x
                heapq.heappush(h, (d + x, v))
    return dist


def bfs_levels(n, rows, cols, src):
    adj = [[] for _ in range(n)]
    for r, c in zip(rows, cols):
        adj[r].append(c)
    lev = {src: 1}
    fr = [src]
    d = 1
    while fr:
        d += 1
        nxt = []
        for u in fr:
            for v in adj[u]:
                if v not in lev:
                    lev[v] = d
                    nxt.append(v)
        fr = nxt
    return lev


def main():
    if not os.path.isdir(REF):
        sys.exit("reference tree not present; fixtures are committed")
    G = {"generator": "tests/golden/make_golden.py", "cases": {}}
    A_data, A_src = fixture_data("graphblas/tests/test_matrix.py", "A")
    v_data, v_src = fixture_data("graphblas/tests/test_matrix.py", "v")
    G["A"] = {"rows": A_data[0], "cols": A_data[1], "values": A_data[2], "src": A_src}
    G["v"] = {"indices": v_data[0], "values": v_data[1], "src": v_src}
    c = G["cases"]
    tm = "graphblas/tests/test_matrix.py"
    tv = "graphblas/tests/test_vector.py"

    calls, _ = from_coo_calls(tm, "test_mxm")
    c["test_mxm"] = {"stmt": "C = A.mxm(A, semiring.plus_times).new()",
                     "expected": coo(calls[0])}
    calls, _ = from_coo_calls(tm, "test_mxm_transpose")
    c["test_mxm_transpose_AAT"] = {"stmt": "C << A.mxm(A.T, semiring.plus_times)",
                                   "expected": coo(calls[0])}
    c["test_mxm_transpose_ATA"] = {"stmt": "C << A.T.mxm(A, semiring.plus_times)",
                                   "expected": coo(calls[1])}
    calls, fn = from_coo_calls(tm, "test_mxm_nonsquare")
    sc = scalar_asserts(fn)
    c["test_mxm_nonsquare"] = {"stmt": "C << A.mxm(B, semiring.max_plus); C[0,0] == 33",
                               "A": coo(calls[0]), "B": coo(calls[1]),
                               "expected_scalar": sc[0][0],
                               "expected_src": f"{tm}:{sc[0][1]}"}
    calls, _ = from_coo_calls(tm, "test_mxm_mask")
    c["test_mxm_mask"] = {
        "val_mask": coo(calls[0]), "struct_mask": coo(calls[1]),
        "stmt_value": "C = A.dup(); C(val_mask.V) << A.mxm(A, semiring.plus_times)",
        "expected_value": coo(calls[2]),
        "stmt_comp": "C = A.dup(); C(~val_mask.V) << A.mxm(A, semiring.plus_times)",
        "expected_comp": coo(calls[3]),
        "stmt_struct_replace": "C = A.dup(); C(struct_mask.S, replace=True) << A.mxm(A, plus_times)",
        "expected_struct_replace": coo(calls[4]),
    }
    calls, _ = from_coo_calls(tm, "test_mxm_accum")
    c["test_mxm_accum"] = {"stmt": "A(binary.plus) << A.mxm(A, semiring.plus_times)",
                           "expected": coo(calls[0])}
    calls, _ = from_coo_calls(tm, "test_mxv")
    c["test_mxv"] = {"stmt": "w = A.mxv(v, semiring.plus_times).new()", "expected": coo(calls[0])}

    calls, _ = from_coo_calls(tv, "test_vxm")
    c["test_vxm"] = {"stmt": "w = v.vxm(A, semiring.plus_times).new()", "expected": coo(calls[0])}
    calls, _ = from_coo_calls(tv, "test_vxm_transpose")
    c["test_vxm_transpose"] = {"stmt": "w = v.vxm(A.T, semiring.plus_times).new()",
                               "expected": coo(calls[0])}
    calls, _ = from_coo_calls(tv, "test_vxm_nonsquare")
    c["test_vxm_nonsquare"] = {"stmt": "u(size 2) << v.vxm(A7x2, semiring.min_plus)",
                               "A": coo(calls[0]), "expected": coo(calls[1])}
    calls, _ = from_coo_calls(tv, "test_vxm_mask")
    c["test_vxm_mask"] = {
        "val_mask": coo(calls[0]), "struct_mask": coo(calls[1]),
        "stmt_struct": "u = v.dup(); u(struct_mask.S) << v.vxm(A, semiring.plus_times)",
        "expected_struct": coo(calls[2]),
        "stmt_comp": "u = v.dup(); u(~struct_mask.S) << v.vxm(A, semiring.plus_times)",
        "expected_comp": coo(calls[3]),
        "stmt_value_replace": "u = v.dup(); u(replace=True, mask=val_mask.V) << v.vxm(A, plus_times)",
        "expected_value_replace": coo(calls[4]),
    }
    calls, _ = from_coo_calls(tv, "test_vxm_accum")
    c["test_vxm_accum"] = {"stmt": "w1 = v.dup(); w1(binary.plus) << v.vxm(A, semiring.plus_times)",
                           "expected": coo(calls[0])}
    _, fn = from_coo_calls(tv, "test_inner")
    sc = scalar_asserts(fn)
    c["test_inner"] = {"stmt": "s << v.inner(v)  (plus_times); then s(binary.plus) << v.inner(v)",
                       "expected_scalar": sc[0][0], "expected_accum": sc[1][0],
                       "expected_src": f"{tv}:{sc[0][1]}"}

    # infix fixtures (fp64; the test is a self-consistency test: expected computed here)
    ti = "graphblas/tests/test_infix.py"
    fx = {}
    for name in ["v1", "v2", "A1", "A2"]:
        calls, _ = from_coo_calls(ti, name)
        fx[name] = coo(calls[0])
        if calls[0]["kw"] and "ncols" in calls[0]["kw"]:
            fx[name]["ncols"] = calls[0]["kw"]["ncols"]
    c["test_infix_matmul"] = {"fixtures": fx,
                              "pairs": [["vxm", "v2", "A2", 0, 0], ["vxm", "v2", "A1", 0, 1],
                                        ["mxv", "A1", "v1", 0, 0], ["mxv", "A2", "v1", 1, 0],
                                        ["mxm", "A1", "A2", 0, 0], ["mxm", "A1", "A2", 1, 1],
                                        ["mxm", "A1", "A1", 0, 1], ["mxm", "A2", "A2", 1, 0]],
                              "src": f"{ti}:80"}

    # docs tables (fp64)
    doc = "docs/user_guide/operations.rst"
    dc = rst_from_coo(doc)
    tabs = rst_tables(doc)
    bytitle = {}
    for t in tabs:
        bytitle.setdefault(t["title"], t)
    c["docs_mxm_min_plus"] = {"stmt": "C << A.mxm(B, op='min_plus')",
                              "A": coo(dc[0]), "B": coo(dc[1]),
                              "expected": table_to_matrix(bytitle["C << min_plus(A @ B)"])}
    c["docs_mxv_plus_times"] = {"stmt": "w << A.mxv(v, op='plus_times')",
                                "A": coo(dc[2]), "v": coo(dc[3]),
                                "expected": table_to_vector(bytitle["w << plus_times(A @ v)"])}
    c["docs_vxm_plus_plus"] = {"stmt": "u << v.vxm(B, op='plus_plus')",
                               "v": coo(dc[4]), "B": coo(dc[5]),
                               "expected": table_to_vector(bytitle["u << plus_plus(v @ B)"])}

    # recorder strings pinned by the reference (boundary call sequence)
    tr = "graphblas/tests/test_recorder.py"
    tree = ast.parse(open(os.path.join(REF, tr)).read())
    for node in ast.walk(tree):
        if isinstance(node, ast.FunctionDef) and node.name == "test_recorder":
            for sub in ast.walk(node):
                if isinstance(sub, ast.Compare) and isinstance(sub.comparators[0], ast.List):
                    c["test_recorder"] = {"expected": _literal(sub.comparators[0]),
                                          "src": f"{tr}:{sub.lineno}"}

    # test_resolving.py: the literal inputs / expected results of the output-binding tests
    # (dtype resolution, Updater argument order, accumulators, extraction by index lists);
    # dtype keywords given as names (dtypes.INT32, float) are kept as their source text
    tres = "graphblas/tests/test_resolving.py"
    tree = ast.parse(open(os.path.join(REF, tres)).read())
    fns = {n.name: n for n in ast.walk(tree) if isinstance(n, ast.FunctionDef)}
    res = {}
    for fname in ["test_from_coo_dtype_resolving", "test_from_coo_invalid_dtype",
                  "test_resolve_ops_using_common_dtype", "test_order_of_updater_params_does_not_matter",
                  "test_already_resolved_ops_allowed_in_updater", "test_updater_returns_updater",
                  "test_py_indices"]:
        lst = []
        for n in ast.walk(fns[fname]):
            if not (isinstance(n, ast.Call) and isinstance(n.func, ast.Attribute) and n.func.attr == "from_coo"
                    and isinstance(n.func.value, ast.Name)):
                continue
            try:
                args = [_literal(a) for a in n.args]
            except ValueError:
                continue  # data built in the test (np.arange ...): restated in the test itself
            kw = {}
            for k in n.keywords:
                try:
                    kw[k.arg] = _literal(k.value)
                except ValueError:
                    kw[k.arg] = ast.unparse(k.value)
            d = coo({"kind": n.func.value.id, "args": args, "kw": kw, "src": f"{tres}:{n.lineno}"})
            d.update(kind=n.func.value.id, dtype=kw.get("dtype"), line=n.lineno)
            lst.append(d)
        lst.sort(key=lambda d: d["line"])
        res[fname] = lst
    c["test_resolving"] = {"src": tres, "cases": res}

    # notebooks (survey-derived expected values, computed independently here)
    data = notebook_graph()
    rows, cols, w = data
    dist = dijkstra(7, rows, cols, w, 1)
    lev = bfs_levels(7, rows, cols, 1)
    c["notebook_sssp"] = {"graph": {"rows": rows, "cols": cols, "values": w,
                                    "src": "notebooks/Intro to GraphBLAS + SSSP example.ipynb cell 2"},
                          "source": 1, "expected": {str(k): v for k, v in sorted(dist.items())},
                          "stmt": "w(binary.min) << w.vxm(m, semiring.min_plus) until fixpoint (cell 21)"}
    c["notebook_level_bfs"] = {"source": 1, "expected": {str(k): v for k, v in sorted(lev.items())},
                               "stmt": "q(~v.S, replace=True) << q.vxm(A, semiring.lor_land) "
                                       "(Example B.1 -- Level BFS.ipynb cell 8)"}
    with open(os.path.join(HERE, "reference_golden.json"), "w") as f:
        json.dump(G, f, indent=1)
    print("wrote", len(c), "cases")


if __name__ == "__main__":
    main()
