"""The suitesparse_graphblas-shaped cffi adapter binds every
declared entry point and the names python-graphblas's discovery regexes look for
(reference graphblas/core/operator/semiring.py:174-203, monoid.py:184-193,
binary.py:336-367, dtypes.py:154-245, descriptor.py:51-89).  Needs cffi, which
the default interpreter lacks; uses /opt/conda/bin/python3.9 (cffi 1.14.6) when
present.  No GPU calls."""
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
          "GrB_Vector_reduce_Monoid_Scalar", "GrB_Descriptor_new", "GrB_Matrix_error"]:
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


@pytest.mark.skipif(not os.path.exists(PY39), reason="no cffi-capable interpreter")
def test_cffi_adapter_binds_the_surface():
    r = subprocess.run([PY39, "-c", SNIPPET % os.path.join(ROOT, "graph-python_amd")], capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    assert r.stdout.startswith("ok")
