#!/usr/bin/env python3
"""Generate the builtin GraphBLAS object tables for the MI355X backend.

The reference discovers builtin operators by regex over the names the C library
exports (reference: graphblas/core/operator/base.py:397-486, the per-class
``_parse_config`` tables at core/operator/semiring.py:170-204,
core/operator/monoid.py:179-195, core/operator/binary.py:332-369, and the
dtype bindings at core/dtypes.py:154-245).  So the drop-in library must export
GraphBLAS-conformant *names*.  This script writes, from one table:

  include/gbamd_codes.h                      type / operator / monoid codes
  include/graphblas_amd_builtins.h           extern declarations of every object
  graph-python_amd/csrc/gb_builtins.cpp      the object definitions
  graph-python_amd/graphblas_amd/_builtins.py  name -> metadata for the front end

Run:  python tools/gen_builtins.py   (outputs are committed; build() re-runs it)
"""
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

TYPES = [  # name, C type, size
    ("BOOL", "bool", 1),
    ("INT8", "int8_t", 1),
    ("UINT8", "uint8_t", 1),
    ("INT16", "int16_t", 2),
    ("UINT16", "uint16_t", 2),
    ("INT32", "int32_t", 4),
    ("UINT32", "uint32_t", 4),
    ("INT64", "int64_t", 8),
    ("UINT64", "uint64_t", 8),
    ("FP32", "float", 4),
    ("FP64", "double", 8),
]
TCODE = {t[0]: i for i, t in enumerate(TYPES)}
NUMERIC = [t[0] for t in TYPES[1:]]
INTS = ["INT8", "UINT8", "INT16", "UINT16", "INT32", "UINT32", "INT64", "UINT64"]
UINTS = ["UINT8", "UINT16", "UINT32", "UINT64"]

BINOPS = [
    "FIRST", "SECOND", "ANY", "PAIR", "MIN", "MAX", "PLUS", "MINUS", "RMINUS",
    "TIMES", "DIV", "RDIV", "POW",
    "ISEQ", "ISNE", "ISGT", "ISLT", "ISGE", "ISLE",
    "LOR", "LAND", "LXOR", "LXNOR",
    "EQ", "NE", "GT", "LT", "GE", "LE",
    "BOR", "BAND", "BXOR", "BXNOR",
    "FIRSTI", "FIRSTI1", "FIRSTJ", "FIRSTJ1",
    "SECONDI", "SECONDI1", "SECONDJ", "SECONDJ1",
    "ATAN2", "HYPOT", "FMOD", "REMAINDER", "LDEXP", "COPYSIGN",
]
OPCODE = {n: i for i, n in enumerate(BINOPS)}
BOOL_OUT = {"EQ", "NE", "GT", "LT", "GE", "LE"}
POSITIONAL = {"FIRSTI", "FIRSTI1", "FIRSTJ", "FIRSTJ1", "SECONDI", "SECONDI1", "SECONDJ", "SECONDJ1"}

# unary operators (reference core/operator/unary.py:289-340 name patterns)
UNOPS = ["IDENTITY", "AINV", "MINV", "ABS", "LNOT", "ONE", "BNOT",
         "SQRT", "LOG", "LOG2", "LOG10", "EXP", "EXP2", "FLOOR", "CEIL", "ROUND", "TRUNC",
         "SIN", "COS", "TAN"]
UCODE = {n: i for i, n in enumerate(UNOPS)}

MONOIDS = ["PLUS", "TIMES", "MIN", "MAX", "ANY", "LOR", "LAND", "LXOR", "LXNOR",
           "BOR", "BAND", "BXOR", "BXNOR"]
MCODE = {n: i for i, n in enumerate(MONOIDS)}
# the binary op that backs each monoid (EQ_BOOL monoid == LXNOR)
MONOID_BINOP = {m: m for m in MONOIDS}

DESCS = {
    # OUTP(replace), MSK_COMP, MSK_STRUCT, TRANS0, TRANS1 (reference core/descriptor.py:51-89)
    (False, False, False, False, True): "GrB_DESC_T1",
    (False, False, False, True, False): "GrB_DESC_T0",
    (False, False, False, True, True): "GrB_DESC_T0T1",
    (False, True, False, False, False): "GrB_DESC_C",
    (False, False, True, False, False): "GrB_DESC_S",
    (False, True, False, False, True): "GrB_DESC_CT1",
    (False, False, True, False, True): "GrB_DESC_ST1",
    (False, True, False, True, False): "GrB_DESC_CT0",
    (False, False, True, True, False): "GrB_DESC_ST0",
    (False, True, False, True, True): "GrB_DESC_CT0T1",
    (False, False, True, True, True): "GrB_DESC_ST0T1",
    (False, True, True, False, False): "GrB_DESC_SC",
    (False, True, True, False, True): "GrB_DESC_SCT1",
    (False, True, True, True, False): "GrB_DESC_SCT0",
    (False, True, True, True, True): "GrB_DESC_SCT0T1",
    (True, False, False, False, False): "GrB_DESC_R",
    (True, False, False, False, True): "GrB_DESC_RT1",
    (True, False, False, True, False): "GrB_DESC_RT0",
    (True, False, False, True, True): "GrB_DESC_RT0T1",
    (True, True, False, False, False): "GrB_DESC_RC",
    (True, False, True, False, False): "GrB_DESC_RS",
    (True, True, False, False, True): "GrB_DESC_RCT1",
    (True, False, True, False, True): "GrB_DESC_RST1",
    (True, True, False, True, False): "GrB_DESC_RCT0",
    (True, False, True, True, False): "GrB_DESC_RST0",
    (True, True, False, True, True): "GrB_DESC_RCT0T1",
    (True, False, True, True, True): "GrB_DESC_RST0T1",
    (True, True, True, False, False): "GrB_DESC_RSC",
    (True, True, True, False, True): "GrB_DESC_RSCT1",
    (True, True, True, True, False): "GrB_DESC_RSCT0",
    (True, True, True, True, True): "GrB_DESC_RSCT0T1",
}



def _write_if_changed(path, text):
    """Leave an unchanged file alone so make does not rebuild everything that includes it."""
    try:
        with open(path) as f:
            if f.read() == text:
                return
    except FileNotFoundError:
        pass
    with open(path, "w") as f:
        f.write(text)

def binop_table():
    """-> list of (name, opcode name, xtype, ztype); xtype None = positional."""
    out = []
    seen = set()

    def add(name, op, x, z):
        if name in seen:
            return
        seen.add(name)
        out.append((name, op, x, z))

    for op in ["FIRST", "SECOND", "PLUS", "MINUS", "TIMES", "DIV", "MIN", "MAX"]:
        for t in TYPES:
            add(f"GrB_{op}_{t[0]}", op, t[0], t[0])
    for op in ["POW", "RMINUS", "RDIV", "PAIR", "ANY", "ISEQ", "ISNE", "ISGT", "ISLT",
               "ISGE", "ISLE", "LOR", "LAND", "LXOR", "LXNOR"]:
        for t in TYPES:
            add(f"GxB_{op}_{t[0]}", op, t[0], t[0])
    for op in ["LOR", "LAND", "LXOR", "LXNOR"]:
        add(f"GrB_{op}", op, "BOOL", "BOOL")
    for op in ["EQ", "NE", "GT", "LT", "GE", "LE"]:
        for t in TYPES:
            add(f"GrB_{op}_{t[0]}", op, t[0], "BOOL")
    for op in ["BOR", "BAND", "BXOR", "BXNOR"]:
        for t in INTS:
            add(f"GrB_{op}_{t}", op, t, t)
    for op in sorted(POSITIONAL):
        for t in ["INT32", "INT64"]:
            add(f"GxB_{op}_{t}", op, None, t)
    # floating-point only (reference binary.py:348; python-graphblas's BinaryOp._initialize
    # coerces integer inputs onto them, binary.py:818-822, and deletes ldexp[FP32/FP64], :867)
    for op in ["ATAN2", "HYPOT", "FMOD", "REMAINDER", "LDEXP", "COPYSIGN"]:
        for t in ["FP32", "FP64"]:
            add(f"GxB_{op}_{t}", op, t, t)
    return out


def unop_table():
    """-> list of (name, opcode name, type)."""
    out = []
    for op in ["IDENTITY", "AINV", "MINV", "ABS"]:
        for t in TYPES:
            out.append((f"GrB_{op}_{t[0]}", op, t[0]))
    out.append(("GrB_LNOT", "LNOT", "BOOL"))
    for t in TYPES[1:]:
        out.append((f"GxB_LNOT_{t[0]}", "LNOT", t[0]))
    for t in TYPES:
        out.append((f"GxB_ONE_{t[0]}", "ONE", t[0]))
    for t in INTS:
        out.append((f"GrB_BNOT_{t}", "BNOT", t))
    for op in ["SQRT", "LOG", "LOG2", "LOG10", "EXP", "EXP2", "FLOOR", "CEIL", "ROUND", "TRUNC",
               "SIN", "COS", "TAN"]:
        for t in ["FP32", "FP64"]:
            out.append((f"GxB_{op}_{t}", op, t))
    return out


def monoid_table():
    """-> list of (name, monoid code name, type, binop name)."""
    out = []
    for m in ["MIN", "MAX", "PLUS", "TIMES"]:
        for t in NUMERIC:
            out.append((f"GrB_{m}_MONOID_{t}", m, t, f"GrB_{m}_{t}"))
    for m in ["LOR", "LAND", "LXOR", "LXNOR"]:
        out.append((f"GrB_{m}_MONOID_BOOL", m, "BOOL", f"GrB_{m}"))
    for t in NUMERIC:
        out.append((f"GxB_ANY_{t}_MONOID", "ANY", t, f"GxB_ANY_{t}"))
    out.append(("GxB_ANY_BOOL_MONOID", "ANY", "BOOL", "GxB_ANY_BOOL"))
    out.append(("GxB_EQ_BOOL_MONOID", "LXNOR", "BOOL", "GrB_LXNOR"))
    for m in ["BOR", "BAND", "BXOR", "BXNOR"]:
        for t in UINTS:
            out.append((f"GxB_{m}_{t}_MONOID", m, t, f"GrB_{m}_{t}"))
    return out


def semiring_table(binops, monoids):
    """-> list of (name, monoid object name, binop object name, aliases)."""
    bop = {b[0]: b for b in binops}
    mon = {(m[1], m[2]): m[0] for m in monoids}
    # monoid (code, type) lookup that also maps EQ monoid on bool
    out = []

    def binop_name(op, t):
        for pre in ("GrB", "GxB"):
            n = f"{pre}_{op}_{t}"
            if n in bop:
                return n
        if t == "BOOL" and f"GrB_{op}" in bop:
            return f"GrB_{op}"
        raise KeyError((op, t))

    grb_sr = {  # C API 2.0 predefined semirings (numeric)
        ("PLUS", "TIMES"), ("PLUS", "MIN"), ("MIN", "PLUS"), ("MIN", "TIMES"), ("MIN", "FIRST"),
        ("MIN", "SECOND"), ("MIN", "MAX"), ("MAX", "PLUS"), ("MAX", "TIMES"), ("MAX", "SECOND"),
        ("MAX", "MIN"),
    }
    mulops = ["FIRST", "SECOND", "PAIR", "MIN", "MAX", "PLUS", "MINUS", "RMINUS", "TIMES",
              "DIV", "RDIV", "ISEQ", "ISNE", "ISGT", "ISLT", "ISGE", "ISLE", "LOR", "LAND",
              "LXOR"]
    for m in ["MIN", "MAX", "PLUS", "TIMES", "ANY"]:
        for op in mulops:
            for t in NUMERIC:
                aliases = []
                if (m, op) in grb_sr:
                    aliases.append(f"GrB_{m}_{op}_SEMIRING_{t}")
                out.append((f"GxB_{m}_{op}_{t}", mon[(m, t)], binop_name(op, t), aliases))
        for op in sorted(POSITIONAL):
            for t in ["INT32", "INT64"]:
                out.append((f"GxB_{m}_{op}_{t}", mon[(m, t)], f"GxB_{op}_{t}", []))
    # bool-valued
    for m, op in [("LOR", "LAND"), ("LAND", "LOR"), ("LXOR", "LAND"), ("LXNOR", "LOR")]:
        out.append((f"GxB_{m}_{op}_BOOL" if m != "LXNOR" else "GxB_EQ_LOR_BOOL",
                    mon[(m, "BOOL")], f"GrB_{op}", [f"GrB_{m}_{op}_SEMIRING_BOOL"]))
    for m in ["LOR", "LAND", "LXOR", "EQ", "ANY"]:
        mk = "LXNOR" if m == "EQ" else m
        for op in ["EQ", "NE", "GT", "LT", "GE", "LE"]:
            for t in NUMERIC:
                out.append((f"GxB_{m}_{op}_{t}", mon[(mk, "BOOL")], f"GrB_{op}_{t}", []))
        for op in ["FIRST", "SECOND", "PAIR", "LOR", "LAND", "LXOR", "EQ", "GT", "LT", "GE", "LE"]:
            name = f"GxB_{m}_{op}_BOOL"
            if any(s[0] == name for s in out):
                continue
            out.append((name, mon[(mk, "BOOL")], binop_name(op, "BOOL"), []))
    for m in ["BOR", "BAND", "BXOR", "BXNOR"]:
        for op in ["BOR", "BAND", "BXOR", "BXNOR"]:
            for t in UINTS:
                out.append((f"GxB_{m}_{op}_{t}", mon[(m, t)], f"GrB_{op}_{t}", []))
    return out


HEADER_NOTE = "/* GENERATED by tools/gen_builtins.py -- do not edit. */\n"


def main():
    binops = binop_table()
    unops = unop_table()
    monoids = monoid_table()
    semirings = semiring_table(binops, monoids)
    bmap = {b[0]: b for b in binops}

    # ---------------- codes header
    lines = [HEADER_NOTE, "#ifndef GBAMD_CODES_H\n#define GBAMD_CODES_H\n"]
    lines.append("/* type codes */\nenum gbamd_type_code {\n")
    for i, t in enumerate(TYPES):
        lines.append(f"    GBAMD_T_{t[0]} = {i},\n")
    lines.append(f"    GBAMD_T_COUNT = {len(TYPES)}\n}};\n")
    lines.append("/* binary operator codes */\nenum gbamd_binop_code {\n")
    for i, n in enumerate(BINOPS):
        lines.append(f"    GBAMD_OP_{n} = {i},\n")
    lines.append(f"    GBAMD_OP_COUNT = {len(BINOPS)}\n}};\n")
    lines.append("/* unary operator codes */\nenum gbamd_unop_code {\n")
    for i, n in enumerate(UNOPS):
        lines.append(f"    GBAMD_UOP_{n} = {i},\n")
    lines.append(f"    GBAMD_UOP_COUNT = {len(UNOPS)}\n}};\n")
    lines.append("/* monoid codes */\nenum gbamd_monoid_code {\n")
    for i, n in enumerate(MONOIDS):
        lines.append(f"    GBAMD_MON_{n} = {i},\n")
    lines.append(f"    GBAMD_MON_COUNT = {len(MONOIDS)}\n}};\n")
    lines.append("#endif\n")
    _write_if_changed(os.path.join(ROOT, "include", "gbamd_codes.h"), "".join(lines))

    # ---------------- extern declarations
    d = [HEADER_NOTE, "#ifndef GRAPHBLAS_AMD_BUILTINS_H\n#define GRAPHBLAS_AMD_BUILTINS_H\n"]
    d.append("/* builtin types (reference core/dtypes.py:154-245) */\n")
    for t in TYPES:
        d.append(f"GB_EXTERN GrB_Type GrB_{t[0]};\n")
    d.append("/* builtin binary operators (reference core/operator/binary.py:332-369) */\n")
    for b in binops:
        d.append(f"GB_EXTERN GrB_BinaryOp {b[0]};\n")
    d.append("/* builtin unary operators (reference core/operator/unary.py) */\n")
    for u in unops:
        d.append(f"GB_EXTERN GrB_UnaryOp {u[0]};\n")
    d.append("/* builtin monoids (reference core/operator/monoid.py:179-195) */\n")
    for m in monoids:
        d.append(f"GB_EXTERN GrB_Monoid {m[0]};\n")
    d.append("/* builtin semirings (reference core/operator/semiring.py:170-204) */\n")
    for s in semirings:
        d.append(f"GB_EXTERN GrB_Semiring {s[0]};\n")
        for a in s[3]:
            d.append(f"GB_EXTERN GrB_Semiring {a};\n")
    d.append("/* predefined descriptors (reference core/descriptor.py:51-89) */\n")
    for name in DESCS.values():
        d.append(f"GB_EXTERN GrB_Descriptor {name};\n")
    d.append("#endif\n")
    _write_if_changed(os.path.join(ROOT, "include", "graphblas_amd_builtins.h"), "".join(d))

    # ---------------- definitions
    c = [HEADER_NOTE, '#include "gb_internal.h"\n\n']
    c.append("namespace {\n")
    for i, t in enumerate(TYPES):
        c.append(f"GB_Type_opaque T_{t[0]} = {{GB_MAGIC, {i}, {t[2]}, \"GrB_{t[0]}\"}};\n")
    for b in binops:
        x = f"&T_{b[2]}" if b[2] else "nullptr"
        c.append(f"GB_BinaryOp_opaque B_{b[0]} = {{GB_MAGIC, GBAMD_OP_{b[1]}, {x}, {x}, &T_{b[3]}, \"{b[0]}\"}};\n")
    for u in unops:
        c.append(f"GB_UnaryOp_opaque U_{u[0]} = {{GB_MAGIC, GBAMD_UOP_{u[1]}, &T_{u[2]}, &T_{u[2]}, \"{u[0]}\"}};\n")
    for m in monoids:
        c.append(f"GB_Monoid_opaque M_{m[0]} = {{GB_MAGIC, GBAMD_MON_{m[1]}, &T_{m[2]}, &B_{m[3]}, \"{m[0]}\"}};\n")
    for s in semirings:
        nm = s[3][0] if s[3] else s[0]
        c.append(f"GB_Semiring_opaque S_{s[0]} = {{GB_MAGIC, &M_{s[1]}, &B_{s[2]}, \"{nm}\"}};\n")
    for key, name in DESCS.items():
        r, comp, st, t0, t1 = key
        mask = (2 if comp else 0) | (4 if st else 0)
        c.append(f"GB_Descriptor_opaque D_{name} = {{GB_MAGIC, {1 if r else 0}, {mask}, {3 if t0 else 0}, {3 if t1 else 0}, true, \"{name}\"}};\n")
    c.append("}  // namespace\n\nextern \"C\" {\n")
    for t in TYPES:
        c.append(f"GrB_Type GrB_{t[0]} = &T_{t[0]};\n")
    for b in binops:
        c.append(f"GrB_BinaryOp {b[0]} = &B_{b[0]};\n")
    for u in unops:
        c.append(f"GrB_UnaryOp {u[0]} = &U_{u[0]};\n")
    for m in monoids:
        c.append(f"GrB_Monoid {m[0]} = &M_{m[0]};\n")
    for s in semirings:
        c.append(f"GrB_Semiring {s[0]} = &S_{s[0]};\n")
        for a in s[3]:
            c.append(f"GrB_Semiring {a} = &S_{s[0]};\n")
    for name in DESCS.values():
        c.append(f"GrB_Descriptor {name} = &D_{name};\n")
    c.append("}  // extern \"C\"\n\n")
    # registry used by GxB_builtin_lookup (name -> handle) for ctypes-free introspection
    c.append("const GB_builtin_entry GB_builtin_registry[] = {\n")
    for t in TYPES:
        c.append(f"    {{\"GrB_{t[0]}\", 0, (void*)&T_{t[0]}}},\n")
    for b in binops:
        c.append(f"    {{\"{b[0]}\", 1, (void*)&B_{b[0]}}},\n")
    for m in monoids:
        c.append(f"    {{\"{m[0]}\", 2, (void*)&M_{m[0]}}},\n")
    for s in semirings:
        c.append(f"    {{\"{s[0]}\", 3, (void*)&S_{s[0]}}},\n")
        for a in s[3]:
            c.append(f"    {{\"{a}\", 3, (void*)&S_{s[0]}}},\n")
    for name in DESCS.values():
        c.append(f"    {{\"{name}\", 4, (void*)&D_{name}}},\n")
    for u in unops:
        c.append(f"    {{\"{u[0]}\", 5, (void*)&U_{u[0]}}},\n")
    c.append("    {nullptr, -1, nullptr}\n};\n")
    _write_if_changed(os.path.join(ROOT, "graph-python_amd", "csrc", "gb_builtins.cpp"), "".join(c))

    # ---------------- python table
    p = ['"""GENERATED by tools/gen_builtins.py -- do not edit.\n\n'
         'Name tables for the builtin objects exported by libgraphblas_amd.so.\n"""\n\n']
    p.append("TYPES = " + repr([(t[0], t[2]) for t in TYPES]) + "\n\n")
    p.append("BINOP_CODES = " + repr(BINOPS) + "\n\n")
    p.append("MONOID_CODES = " + repr(MONOIDS) + "\n\n")
    p.append("UNOP_CODES = " + repr(UNOPS) + "\n\n")
    p.append("# name: (opcode name, xtype or None for positional, ztype)\nBINOPS = {\n")
    for b in binops:
        p.append(f"    {b[0]!r}: ({b[1]!r}, {b[2]!r}, {b[3]!r}),\n")
    p.append("}\n\n# name: (opcode name, type)\nUNOPS = {\n")
    for u in unops:
        p.append(f"    {u[0]!r}: ({u[1]!r}, {u[2]!r}),\n")
    p.append("}\n\n# name: (monoid code name, type, binop name)\nMONOIDS = {\n")
    for m in monoids:
        p.append(f"    {m[0]!r}: ({m[1]!r}, {m[2]!r}, {m[3]!r}),\n")
    p.append("}\n\n# name: (monoid name, binop name, [aliases])\nSEMIRINGS = {\n")
    for s in semirings:
        p.append(f"    {s[0]!r}: ({s[1]!r}, {s[2]!r}, {s[3]!r}),\n")
    p.append("}\n\n# (replace, complement, structure, tran0, tran1): name\nDESCRIPTORS = {\n")
    for k, v in DESCS.items():
        p.append(f"    {k!r}: {v!r},\n")
    p.append("}\n")
    _write_if_changed(os.path.join(ROOT, "graph-python_amd", "graphblas_amd", "_builtins.py"), "".join(p))
    print(f"types={len(TYPES)} binops={len(binops)} unops={len(unops)} monoids={len(monoids)} "
          f"semirings={len(semirings)} (+{sum(len(s[3]) for s in semirings)} aliases) "
          f"descriptors={len(DESCS)}")


if __name__ == "__main__":
    main()
