"""The suitesparse_graphblas-shaped cffi adapter binds every
declared entry point and the names python-graphblas's discovery regexes look for
(reference graphblas/core/operator/semiring.py:174-203, monoid.py:184-193,
binary.py:336-367, dtypes.py:154-245, descriptor.py:51-89).  Needs cffi, which
the default interpreter lacks; uses /opt/conda/bin/python3.9 (cffi 1.14.6) when
present.  No GPU calls.

test_reference_init_replay transcribes, step by step, what python-graphblas does
with the module between `from suitesparse_graphblas import ...` and its first
mxm dispatch (the reference cannot be imported here: `donfig` is missing, SURVEY
§8c), and runs those steps over the adapter's `lib`:
  1. graphblas/__init__.py:156-186 -- is_initialized / initialize, then the
     "suitesparse-vanilla" strip: drop callable GxB_* and FC32/FC64 names, then
     `delattr(lib, "GxB_BACKWARDS")` and `delattr(lib, "GxB_STRIDE")`;
  2. core/dtypes.py:13, 154-282 -- the builtin types bound to lib.GrB_<T>;
  3. core/operator/base.py:291, 397-486 -- OpBase._initialize: the regex pass over
     dir(lib) for binary ops, monoids and semirings with the parse configs of
     binary.py:332-369, monoid.py:179-195, semiring.py:170-204;
  4. the post-passes that index typed ops by name and must find them:
     binary.py:754-868 (cdiv/truediv, positional and lxnor coercions, del ldexp),
     monoid.py:400-435, semiring.py:351-510 (cdiv, plus_pow via GrB_Semiring_new,
     *_ne <- *_lxor, positional / boolean coercions, max_* -> lor_* remaps);
  5. core/slice.py:10-49 -- the index constants the suitesparse backend reads.
"""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PY39 = "/opt/conda/bin/python3.9"

SNIPPET = r"""
import re, sys
sys.path.insert(0, %r)
import suitesparse_graphblas_amd as ss
from suitesparse_graphblas_amd import ffi, lib, initialize, is_initialized
names = set(vars(lib))
for f in ["GrB_mxm", "GrB_mxv", "GrB_vxm", "GrB_Matrix_new", "GrB_Vector_assign_INT32",
          "GrB_Matrix_build_FP64", "GrB_Vector_extractTuples_BOOL", "GrB_Matrix_eWiseMult_BinaryOp",
          "GrB_Vector_reduce_Monoid_Scalar", "GrB_Descriptor_new", "GrB_Matrix_error",
          "GrB_Matrix_extract", "GrB_Col_extract", "GrB_Vector_extract",
          # GrB_Scalar-argument variants (reference core/vector.py:1406,1449,1769,1808,1918,1939;
          # core/matrix.py:2392,2435,2837,2902,3279,3305)
          "GrB_Vector_extractElement_Scalar", "GrB_Matrix_extractElement_Scalar",
          "GrB_Vector_setElement_Scalar", "GrB_Matrix_setElement_Scalar",
          "GrB_Vector_assign_Scalar", "GrB_Matrix_assign_Scalar",
          "GrB_Vector_apply_BinaryOp1st_Scalar", "GrB_Vector_apply_BinaryOp2nd_Scalar",
          "GrB_Matrix_apply_BinaryOp1st_Scalar", "GrB_Matrix_apply_BinaryOp2nd_Scalar"]:
    assert callable(getattr(lib, f)), f
assert lib.GrB_SUCCESS == 0 and lib.GrB_NO_VALUE == 1
sr = [n for n in names if re.match(r"GrB_(PLUS|MIN|MAX)_(PLUS|TIMES|MIN|MAX|FIRST|SECOND)_SEMIRING_", n)]
gx = [n for n in names if re.match(r"GxB_(ANY|LOR|MIN|PLUS)_(PAIR|LAND|FIRST|PLUS)_", n)]
assert len(sr) > 50 and len(gx) > 50, (len(sr), len(gx))
assert lib.GrB_LOR_LAND_SEMIRING_BOOL != ffi.NULL
assert lib.GxB_ANY_PAIR_BOOL != ffi.NULL and lib.GrB_MIN_PLUS_SEMIRING_INT64 != ffi.NULL
descs = [n for n in names if n.startswith("GrB_DESC_")]
assert len(descs) == 31, len(descs)
assert lib.GrB_BOOL != ffi.NULL and lib.GrB_FP64 != ffi.NULL
assert not is_initialized()
print("ok", len(names))
"""

# Steps 1-5 of the module docstring, transcribed from the reference (file:line per block).
REPLAY = r"""
import itertools, re, sys
sys.path.insert(0, %r)
import suitesparse_graphblas_amd
sys.modules["suitesparse_graphblas"] = suitesparse_graphblas_amd
from suitesparse_graphblas import ffi, initialize, is_initialized, lib   # __init__.py:141

# ---- 1. __init__.py:156-186 (initialize needs a GPU: GrB_init is not called here)
assert is_initialized() is False
orig_lib = lib
class Lib:
    pass
lib = Lib()
for key, val in vars(orig_lib).items():
    if callable(val) and key.startswith("GxB") or "FC32" in key or "FC64" in key:
        continue
    setattr(lib, key, getattr(orig_lib, key))
for key in ["GxB_BACKWARDS", "GxB_STRIDE"]:
    delattr(lib, key)
NULL = ffi.NULL

# ---- 2. dtypes.py:13, 154-282
supports_complex = hasattr(lib, "GrB_FC64") or hasattr(lib, "GxB_FC64")
assert not supports_complex  # the vanilla strip removed nothing else complex-typed
TYPES = ["BOOL", "INT8", "UINT8", "INT16", "UINT16", "INT32", "UINT32", "INT64", "UINT64", "FP32", "FP64"]
for t in TYPES:
    assert getattr(lib, "GrB_" + t) != NULL, t

# ---- 3. operator/base.py:291 and :397-486 with each class's _parse_config
VARNAMES = tuple(x for x in dir(lib) if x[0] != "_")
INT = "(INT8|UINT8|INT16|UINT16|INT32|UINT32|INT64|UINT64|FP32|FP64)"
BINARY = {  # binary.py:332-369
    "trim_from_front": 4, "num_underscores": 1,
    "re_exprs": [
        re.compile("^GrB_(FIRST|SECOND|PLUS|MINUS|TIMES|DIV|MIN|MAX)"
                   "_(BOOL|INT8|UINT8|INT16|UINT16|INT32|UINT32|INT64|UINT64|FP32|FP64|FC32|FC64)$"),
        re.compile("GrB_(BOR|BAND|BXOR|BXNOR)_(INT8|INT16|INT32|INT64|UINT8|UINT16|UINT32|UINT64)$"),
        re.compile("^GxB_(POW|RMINUS|RDIV|PAIR|ANY|ISEQ|ISNE|ISGT|ISLT|ISGE|ISLE|LOR|LAND|LXOR)"
                   "_(BOOL|INT8|UINT8|INT16|UINT16|INT32|UINT32|INT64|UINT64|FP32|FP64|FC32|FC64)$"),
        re.compile("^GxB_(FIRST|SECOND|PLUS|MINUS|TIMES|DIV)_(FC32|FC64)$"),
        re.compile("^GxB_(ATAN2|HYPOT|FMOD|REMAINDER|LDEXP|COPYSIGN)_(FP32|FP64)$"),
        re.compile("GxB_(BGET|BSET|BCLR|BSHIFT|FIRSTI1|FIRSTI|FIRSTJ1|FIRSTJ"
                   "|SECONDI1|SECONDI|SECONDJ1|SECONDJ)_(INT8|INT16|INT32|INT64|UINT8|UINT16|UINT32|UINT64)$"),
        re.compile("^GxB_(LOR|LAND|LXOR|LXNOR)_(BOOL|INT8|UINT8|INT16|UINT16|INT32|UINT32|INT64|UINT64|FP32|FP64)$"),
    ],
    "re_exprs_return_bool": [
        re.compile("^GrB_(LOR|LAND|LXOR|LXNOR)$"),
        re.compile("^GrB_(EQ|NE|GT|LT|GE|LE)_(BOOL|INT8|UINT8|INT16|UINT16|INT32|UINT32|INT64|UINT64|FP32|FP64)$"),
        re.compile("^GxB_(EQ|NE)_(FC32|FC64)$"),
    ],
}
MONOID = {  # monoid.py:179-195
    "trim_from_front": 4, "delete_exact": "MONOID", "num_underscores": 1,
    "re_exprs": [
        re.compile("^GrB_(MIN|MAX|PLUS|TIMES|LOR|LAND|LXOR|LXNOR)_MONOID"
                   "_(BOOL|INT8|UINT8|INT16|UINT16|INT32|UINT32|INT64|UINT64|FP32|FP64)$"),
        re.compile("^GxB_(ANY)_" + INT + "_MONOID$"),
        re.compile("^GxB_(PLUS|TIMES|ANY)_(FC32|FC64)_MONOID$"),
        re.compile("^GxB_(EQ|ANY)_BOOL_MONOID$"),
        re.compile("^GxB_(BOR|BAND|BXOR|BXNOR)_(UINT8|UINT16|UINT32|UINT64)_MONOID$"),
    ],
}
SEMIRING = {  # semiring.py:170-204
    "trim_from_front": 4, "delete_exact": "SEMIRING", "num_underscores": 2,
    "re_exprs": [
        re.compile("^GrB_(PLUS|MIN|MAX)_(PLUS|TIMES|FIRST|SECOND|MIN|MAX)_SEMIRING_" + INT + "$"),
        re.compile("^GxB_(MIN|MAX|PLUS|TIMES|ANY)"
                   "_(FIRST|SECOND|PAIR|MIN|MAX|PLUS|MINUS|RMINUS|TIMES"
                   "|DIV|RDIV|ISEQ|ISNE|ISGT|ISLT|ISGE|ISLE|LOR|LAND|LXOR"
                   "|FIRSTI1|FIRSTI|FIRSTJ1|FIRSTJ|SECONDI1|SECONDI|SECONDJ1|SECONDJ)_" + INT + "$"),
        re.compile("^GxB_(PLUS|TIMES|ANY)_(FIRST|SECOND|PAIR|PLUS|MINUS|TIMES|DIV|RDIV|RMINUS)_(FC32|FC64)$"),
        re.compile("^GxB_(BOR|BAND|BXOR|BXNOR)_(BOR|BAND|BXOR|BXNOR)_(UINT8|UINT16|UINT32|UINT64)$"),
    ],
    "re_exprs_return_bool": [
        re.compile("^GrB_(LOR|LAND|LXOR|LXNOR)_(LOR|LAND)_SEMIRING_BOOL$"),
        re.compile("^GxB_(LOR|LAND|LXOR|EQ|ANY)_(EQ|NE|GT|LT|GE|LE)_" + INT + "$"),
        re.compile("^GxB_(LOR|LAND|LXOR|EQ|ANY)_(FIRST|SECOND|PAIR|LOR|LAND|LXOR|EQ|GT|LT|GE|LE)_BOOL$"),
    ],
}


def initialize_ops(cfg):
    # name -> {input type: (return type, lib object, varname)}
    ops = {}
    trim, delete_exact, nu = cfg.get("trim_from_front", 0), cfg.get("delete_exact"), cfg["num_underscores"]
    for re_str, return_prefix in [("re_exprs", None), ("re_exprs_return_bool", "BOOL"),
                                  ("re_exprs_return_float", "FP"), ("re_exprs_return_complex", "FC")]:
        if re_str not in cfg:
            continue
        if "complex" in re_str and not supports_complex:
            continue
        for r in reversed(cfg[re_str]):
            for varname in VARNAMES:
                m = r.match(varname)
                if not m:
                    continue
                splitname = m.string[trim:].split("_")
                if delete_exact and delete_exact in splitname:
                    splitname.remove(delete_exact)
                if len(splitname) == nu + 1:
                    *splitname, type_ = splitname
                else:
                    type_ = None
                name = "_".join(splitname).lower()
                gb_obj = getattr(lib, varname)
                if return_prefix == "BOOL":
                    return_type = "BOOL"
                    if type_ is None:
                        type_ = "BOOL"
                else:
                    assert type_ is not None, varname
                    return_type = type_ if return_prefix is None else return_prefix + type_[-2:]
                assert type_ in TYPES, (varname, type_)  # lookup_dtype must succeed
                ops.setdefault(name, {})[type_] = (return_type, gb_obj, varname)
    return ops


binary, monoid, semiring = initialize_ops(BINARY), initialize_ops(MONOID), initialize_ops(SEMIRING)

# ---- 4a. binary.py:754-868
binary["cdiv"] = dict(binary.pop("div"))
for new, builtin in [("truediv", "cdiv"), ("rtruediv", "rdiv")]:
    for dtype in binary[builtin]:
        binary.setdefault(new, {})[dtype] = binary[builtin]["FP32" if dtype == "FP32" else "FP64"]
position = ["BOOL", "FP32", "FP64", "INT8", "INT16", "UINT8", "UINT16", "UINT32", "UINT64"]
notbool = ["FP32", "FP64", "INT8", "INT16", "INT32", "INT64", "UINT8", "UINT16", "UINT32", "UINT64"]
name_types = [
    (("atan2", "copysign", "fmod", "hypot", "ldexp", "remainder"),
     (("BOOL", "INT8", "INT16", "UINT8", "UINT16"), "FP32"), (("INT32", "INT64", "UINT32", "UINT64"), "FP64")),
    (("firsti", "firsti1", "firstj", "firstj1", "secondi", "secondi1", "secondj", "secondj1"), (position, "INT64")),
    (["lxnor"], (notbool, "BOOL")),
]
for names, *types in name_types:
    for name in names:
        for input_types, target in types:
            typed = binary[name][target]  # KeyError = python-graphblas's init would fail
            for dtype in input_types:
                binary[name].setdefault(dtype, typed)
del binary["ldexp"]["FP32"]
del binary["ldexp"]["FP64"]
for name in ["first", "second", "pair", "any", "eq", "ne"]:
    assert name in binary, name

# ---- 4b. monoid.py:400-435
lor, land = monoid["lor"]["BOOL"], monoid["land"]["BOOL"]
for name, typed in [("max", lor), ("min", land), ("times", land)]:
    monoid[name].setdefault("BOOL", typed)
for name in ["lor", "land", "lxnor", "lxor"]:
    assert "BOOL" in monoid[name], name
for name in ["any", "band", "bor", "land", "lor", "max", "min"]:
    assert name in monoid, name

# ---- 4c. semiring.py:351-510
for orig_name in [k for k in semiring if k.endswith("_div")]:
    semiring[orig_name[:-3] + "cdiv"] = semiring.pop(orig_name)
made = 0
for dtype, (ret, pow_obj, _) in binary["pow"].items():   # register_new("plus_pow", ...), semiring.py:217-243
    if ret not in monoid["plus"]:
        continue
    cell = ffi.new("GrB_Semiring*")
    assert orig_lib.GrB_Semiring_new(cell, monoid["plus"][ret][1], pow_obj) == 0, dtype
    assert orig_lib.GrB_Semiring_free(cell) == 0
    made += 1
assert made >= 10, made
for lname in ["any", "eq", "land", "lor", "lxnor", "lxor"]:
    if lname + "_ne" in semiring and "BOOL" not in semiring[lname + "_ne"]:
        semiring[lname + "_ne"]["BOOL"] = semiring[lname + "_lxor"]["BOOL"]
for lnames, rnames, *types in [
        (("any", "max", "min", "plus", "times"),
         ("firsti", "firsti1", "firstj", "firstj1", "secondi", "secondi1", "secondj", "secondj1"),
         (position, "INT64")),
        (("eq", "land", "lor", "lxnor", "lxor"), ("first", "pair", "second"), (notbool, "BOOL")),
        (("band", "bor", "bxnor", "bxor"), ("band", "bor", "bxnor", "bxor"),
         (["INT8"], "UINT16"), (["INT16"], "UINT32"), (["INT32"], "UINT64"), (["INT64"], "UINT64")),
        (("any", "eq", "land", "lor", "lxnor", "lxor"), ("eq", "land", "lor", "lxnor", "lxor", "ne"),
         (notbool, "BOOL"))]:
    for left, right in itertools.product(lnames, rnames):
        name = left + "_" + right
        if name not in semiring:
            continue
        for input_types, target in types:
            typed = semiring[name][target]
            for dtype in input_types:
                semiring[name].setdefault(dtype, typed)
for opname, target in [("max_first", "lor_first"), ("max_second", "lor_second"), ("max_land", "lor_land"),
                       ("max_lor", "lor_lor"), ("max_lxor", "lor_lxor"), ("min_first", "land_first"),
                       ("min_second", "land_second"), ("min_land", "land_land"), ("min_lor", "land_lor"),
                       ("min_lxor", "land_lxor")]:
    assert "BOOL" in semiring[target], target
    semiring[opname].setdefault("BOOL", semiring[target]["BOOL"])

# the north-star's operators resolve to the exported objects
assert semiring["min_plus"]["INT64"][2] == "GrB_MIN_PLUS_SEMIRING_INT64"
assert semiring["min_plus"]["INT64"][1] == orig_lib.GrB_MIN_PLUS_SEMIRING_INT64
assert semiring["any_pair"]["BOOL"][2] == "GxB_ANY_PAIR_BOOL"
assert semiring["any_pair"]["BOOL"][1] == orig_lib.GxB_ANY_PAIR_BOOL
assert semiring["lor_land"]["BOOL"][2] == "GrB_LOR_LAND_SEMIRING_BOOL"
assert semiring["plus_times"]["FP64"][2] == "GrB_PLUS_TIMES_SEMIRING_FP64"
assert semiring["max_land"]["BOOL"][2] == "GrB_LOR_LAND_SEMIRING_BOOL"
# the C API name wins over the GxB alias (the GrB regex is scanned last, base.py:420)
assert semiring["min_first"]["UINT64"][2] == "GrB_MIN_FIRST_SEMIRING_UINT64"
assert semiring["min_first"]["UINT64"][1] == orig_lib.GxB_MIN_FIRST_UINT64
assert monoid["plus"]["INT64"][2] == "GrB_PLUS_MONOID_INT64"
assert binary["plus"]["FP64"][2] == "GrB_PLUS_FP64"

# ---- 5. slice.py:10-16 (suitesparse backend) and the vanilla strip's survivors
assert orig_lib.GxB_RANGE == 2**63 - 1 and orig_lib.GxB_STRIDE == 2**63 - 2 and orig_lib.GxB_BACKWARDS == 2**63 - 3
assert (orig_lib.GxB_BEGIN, orig_lib.GxB_END, orig_lib.GxB_INC) == (0, 1, 2)
assert lib.GxB_RANGE == 2**63 - 1 and not hasattr(lib, "GxB_STRIDE") and not hasattr(lib, "GxB_BACKWARDS")
assert lib.GrB_INDEX_MAX == 2**60 - 1
assert callable(lib.GrB_Matrix_extract) and callable(lib.GrB_Col_extract) and callable(lib.GrB_Vector_extract)
assert not hasattr(lib, "GxB_Matrix_rmat")  # a callable GxB_* name: stripped
assert callable(orig_lib.GxB_Global_Option_get_INT32) and orig_lib.GxB_MODE == 2
print("replay ok", len(semiring), len(monoid), len(binary))
"""


@pytest.mark.skipif(not os.path.exists(PY39), reason="no cffi-capable interpreter")
def test_cffi_adapter_binds_the_surface():
    r = subprocess.run([PY39, "-c", SNIPPET % os.path.join(ROOT, "graph-python_amd")], capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    assert r.stdout.startswith("ok")


@pytest.mark.skipif(not os.path.exists(PY39), reason="no cffi-capable interpreter")
def test_reference_init_replay():
    r = subprocess.run([PY39, "-c", REPLAY % os.path.join(ROOT, "graph-python_amd")], capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-3000:]
    assert r.stdout.startswith("replay ok"), r.stdout
