#!/usr/bin/env python3
"""Generate tests/golden/mask_golden.json: the mask-algebra expectations of the
reference's tests/test_mask.py:9-126 (test_mask_new, test_mask_or, test_mask_and).

Runs only in the build container (the reference tree does not exist on the GPU box).
The reference is read as TEXT: `ast` pulls the two input vectors' construction out of
test_mask_new -- `Vector(mask_dtype, size=10)` and the slice assigns `v1[3:6] = 0`,
`v1[:3] = 10`, `v2[1::3] = 0`, `v2[::3] = 10` -- and checks that test_mask_or and
test_mask_and build the same vectors.  Nothing from the reference is imported or run.

The expected results are restated here in plain Python set algebra, following the
tests' own assign-based recipes:
  * the set a mask selects: structural -> stored indices; value -> stored indices whose
    value is nonzero (for a bool mask vector the stored value 10 is True, 0 is False);
    complemented -> the other indices;
  * test_mask_new:  m1.new(mask=m2) == expected.dup(mask=m1).dup(mask=m2)  -> S1 & S2,
    complement=True -> expected(~expected.S, replace=True) << True  -> ~(S1 & S2);
    m.new() -> S, m.new(complement=True) -> ~S    (test_mask.py:23-49);
  * test_mask_or:   expected(m1) << True; expected(m2) << True        -> S1 | S2 (:72-79);
  * test_mask_and:  expected.dup(mask=m1).dup(mask=m2)                -> S1 & S2 (:107-114).
"""
import ast
import json
import os

REF = "/root/reference"
SRC = "graphblas/tests/test_mask.py"
HERE = os.path.dirname(os.path.abspath(__file__))


def vector_setup(fn):
    """{name: (size, [(start, stop, step, value), ...], line)} from a test function body."""
    out = {}
    for node in ast.walk(fn):
        if not isinstance(node, ast.Assign) or len(node.targets) != 1:
            continue
        tgt = node.targets[0]
        if isinstance(tgt, ast.Name) and isinstance(node.value, ast.Call) and \
                getattr(node.value.func, "id", None) == "Vector":
            size = [ast.literal_eval(k.value) for k in node.value.keywords if k.arg == "size"][0]
            out.setdefault(tgt.id, {"size": size, "assigns": [], "line": node.lineno})
        elif isinstance(tgt, ast.Subscript) and isinstance(tgt.value, ast.Name) and isinstance(tgt.slice, ast.Slice):
            s = tgt.slice
            lit = [ast.literal_eval(x) if x is not None else None for x in (s.lower, s.upper, s.step)]
            out[tgt.value.id]["assigns"].append(lit + [ast.literal_eval(node.value)])
    return out


def entries(setup):
    size = setup["size"]
    vals = {}
    for start, stop, step, value in setup["assigns"]:
        for i in range(size)[slice(start, stop, step)]:
            vals[i] = value
    return vals


def main():
    tree = ast.parse(open(os.path.join(REF, SRC)).read())
    fns = {n.name: n for n in ast.walk(tree) if isinstance(n, ast.FunctionDef)}
    setups = {name: vector_setup(fns[name]) for name in ("test_mask_new", "test_mask_or", "test_mask_and")}
    base = setups["test_mask_new"]
    for name, s in setups.items():
        assert {k: (v["size"], v["assigns"]) for k, v in s.items()} == \
               {k: (v["size"], v["assigns"]) for k, v in base.items()}, name
    size = base["v1"]["size"]
    universe = set(range(size))
    cases = {}
    for mask_dtype in ("BOOL", "INT64"):
        sel = {}
        for vname in ("v1", "v2"):
            e = entries(base[vname])
            stored = set(e)
            nonzero = {i for i, x in e.items() if x != 0}  # 10 -> True, 0 -> False for a bool vector
            sel[f"{vname}.S"] = stored
            sel[f"{vname}.V"] = nonzero
            sel[f"~{vname}.S"] = universe - stored
            sel[f"~{vname}.V"] = universe - nonzero
        order = ["v1.S", "v1.V", "~v1.S", "~v1.V", "v2.S", "v2.V", "~v2.S", "~v2.V"]
        pairs = {}
        for a in order:
            for b in order:
                pairs[f"{a}|{b}"] = {
                    "new": sorted(sel[a] & sel[b]),
                    "new_complement": sorted(universe - (sel[a] & sel[b])),
                    "and": sorted(sel[a] & sel[b]),
                    "or": sorted(sel[a] | sel[b]),
                }
        single = {m: {"new": sorted(sel[m]), "new_complement": sorted(universe - sel[m])} for m in order}
        cases[mask_dtype] = {"pairs": pairs, "single": single}
    out = {
        "source": f"{SRC}:9-126 (test_mask_new, test_mask_or, test_mask_and)",
        "size": size,
        "vectors": {k: {"assigns": base[k]["assigns"], "src": f"{SRC}:{base[k]['line']}"} for k in ("v1", "v2")},
        "masks": ["v1.S", "v1.V", "~v1.S", "~v1.V", "v2.S", "v2.V", "~v2.S", "~v2.V"],
        "mask_dtypes": {"BOOL": "bool", "INT64": "int"},
        "result_dtypes": [None, "BOOL", "INT64"],
        "cases": cases,
    }
    json.dump(out, open(os.path.join(HERE, "mask_golden.json"), "w"), indent=0, sort_keys=True)
    print("mask cases:", sum(len(c["pairs"]) for c in cases.values()))


if __name__ == "__main__":
    main()
