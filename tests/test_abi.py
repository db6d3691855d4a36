"""CPU checks of the drop-in boundary: libgraphblas_amd.so loads, exports every
entry point and builtin object include/*.h declares, and the front end binds
the names python-graphblas's regex discovery expects (reference
core/operator/base.py:397-486; tests/test_op.py:82-91 name contract).  No
compute calls (no GPU here)."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "include", "graphblas_amd.h")
BHDR = os.path.join(ROOT, "include", "graphblas_amd_builtins.h")
TYPES = ["BOOL", "INT8", "UINT8", "INT16", "UINT16", "INT32", "UINT32", "INT64", "UINT64", "FP32", "FP64"]


def declared_functions():
    text = open(HDR).read()
    names = set(re.findall(r"^GrB_Info\s+(\w+)\s*\(", text, re.M))
    names |= set(re.findall(r"^GB_EXTERN\s+GrB_Info\s+(\w+)\s*\(", text, re.M))
    # typed families declared through the GB_DECLARE_TYPED_* macros
    for fam in re.findall(r"GrB_Info\s+(\w+)_##T\(", text):
        for t in TYPES:
            names.add(f"{fam}_{t}")
    return names


def declared_objects():
    return re.findall(r"^GB_EXTERN\s+\w+\s+(\w+);", open(BHDR).read(), re.M) + ["GrB_ALL"]


@pytest.fixture(scope="module")
def dll():
    import graphblas_amd

    return ctypes.CDLL(graphblas_amd.LIB_PATH)


def test_every_declared_function_is_exported(dll):
    names = declared_functions()
    assert len(names) > 250
    missing = [n for n in sorted(names) if not hasattr(dll, n)]
    assert not missing, missing[:20]


def test_every_declared_object_is_exported(dll):
    objs = declared_objects()
    assert len(objs) > 1900
    missing = []
    for n in objs:
        try:
            v = ctypes.c_void_p.in_dll(dll, n).value
            assert v
        except ValueError:
            missing.append(n)
    assert not missing, missing[:20]


def test_hot_path_signatures_match_c_api():
    text = open(HDR).read()
    for name, args in [
        ("GrB_mxm", "GrB_Matrix C, const GrB_Matrix Mask, const GrB_BinaryOp accum,\n"
                    "                 const GrB_Semiring op, const GrB_Matrix A, const GrB_Matrix B,\n"
                    "                 const GrB_Descriptor desc"),
    ]:
        assert f"GrB_Info {name}({args});" in text
    for name in ("GrB_mxv", "GrB_vxm"):
        assert re.search(rf"GrB_Info {name}\(GrB_Vector w, const GrB_Vector mask, const GrB_BinaryOp accum,", text)


def test_name_contract_and_aliases(dll):
    import graphblas_amd as gb

    # reference tests/test_op.py:87-91
    assert gb.semiring.min_plus["INT32"].gb_obj.value == ctypes.c_void_p.in_dll(
        dll, "GrB_MIN_PLUS_SEMIRING_INT32").value
    # GrB_ and GxB_ names of one semiring are one object (identity compare)
    assert ctypes.c_void_p.in_dll(dll, "GxB_MIN_PLUS_INT64").value == ctypes.c_void_p.in_dll(
        dll, "GrB_MIN_PLUS_SEMIRING_INT64").value
    assert gb.semiring.lor_land[bool].gb_name == "GrB_LOR_LAND_SEMIRING_BOOL"
    assert gb.semiring.any_pair[bool].gb_name == "GxB_ANY_PAIR_BOOL"
    assert gb.semiring.min_first["UINT64"].gb_name == "GrB_MIN_FIRST_SEMIRING_UINT64"
    assert gb.semiring.plus_times[float].gb_name == "GrB_PLUS_TIMES_SEMIRING_FP64"
    # bool coercions (reference core/operator/semiring.py:491-510)
    assert gb.semiring.max_land[bool] is gb.semiring.lor_land[bool]
    # positional semirings coerce to INT64
    assert gb.semiring.min_secondi[gb.FP64].gb_name == "GxB_MIN_SECONDI_INT64"


def test_builtin_lookup_extension(dll):
    h = ctypes.c_void_p()
    kind = ctypes.c_int()
    f = dll.GxB_builtin_lookup
    f.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_char_p]
    assert f(ctypes.byref(h), ctypes.byref(kind), b"GrB_LOR_LAND_SEMIRING_BOOL") == 0
    assert kind.value == 3 and h.value == ctypes.c_void_p.in_dll(dll, "GrB_LOR_LAND_SEMIRING_BOOL").value
    assert f(ctypes.byref(h), ctypes.byref(kind), b"nope") == -3


def test_descriptor_table_matches_reference():
    import graphblas_amd.base as B

    # 31 predefined descriptors + NULL (reference core/descriptor.py:51-89)
    assert len([k for k, d in B._desc_map.items() if d is not None]) == 31
    assert B.descriptor_lookup() is None
    assert B.descriptor_lookup(output_replace=True, mask_complement=True, mask_structure=True).name == "GrB_DESC_RSC"
    assert B.descriptor_lookup(transpose_second=True).name == "GrB_DESC_T1"
    assert B.descriptor_lookup(mask_structure=True, transpose_first=True).name == "GrB_DESC_ST0"


def test_descriptor_set_on_cpu(dll):
    # descriptor objects live on the host: exercise new/set/free without a GPU
    d = ctypes.c_void_p()
    dll.GrB_Descriptor_new.argtypes = [ctypes.c_void_p]
    dll.GrB_Descriptor_set.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
    dll.GrB_Descriptor_free.argtypes = [ctypes.c_void_p]
    assert dll.GrB_Descriptor_new(ctypes.byref(d)) == 0
    assert dll.GrB_Descriptor_set(d, 1, 2) == 0  # GrB_MASK, GrB_COMP
    assert dll.GrB_Descriptor_set(d, 1, 4) == 0  # | GrB_STRUCTURE
    assert dll.GrB_Descriptor_set(d, 2, 3) == 0  # INP0 TRAN
    assert dll.GrB_Descriptor_set(d, 0, 99) == -3
    pre = ctypes.c_void_p.in_dll(dll, "GrB_DESC_T0")
    assert dll.GrB_Descriptor_set(pre, 2, 0) == -3  # predefined descriptors are read-only
    assert dll.GrB_Descriptor_free(ctypes.byref(d)) == 0


def test_product_fails_loudly_without_gpu():
    import torch

    if torch.cuda.is_available():
        pytest.skip("GPU present")
    import graphblas_amd as gb

    with pytest.raises(gb.GraphblasException):
        gb.Matrix(gb.INT64, 3, 3)
