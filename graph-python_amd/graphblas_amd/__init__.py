"""graphblas_amd -- MI355X-native GraphBLAS semiring backend (front end).

A python-graphblas-shaped API over libgraphblas_amd.so: the same delayed
expressions (`A.mxm(B, semiring.min_plus)`, `v.vxm(A, ...)`, `A @ v`), the
same output binding (`C(mask.V, accum=binary.plus, replace=True) << expr`),
the same descriptor selection and recorder strings, executed by hand-written
HIP kernels for gfx950 instead of SuiteSparse:GraphBLAS.

    >>> import graphblas_amd as gb
    >>> A = gb.Matrix.from_coo([0, 1], [1, 0], [2, 3])
    >>> C = A.mxm(A, gb.semiring.min_plus).new()
"""
import ctypes

from . import _builtins  # noqa: F401
from ._lib import LIB_PATH, NULL, lib
from .base import Recorder, _reset_name_counters, replace
from .dtypes import (BOOL, FP32, FP64, INT8, INT16, INT32, INT64, UINT8, UINT16, UINT32, UINT64,
                     DataType, lookup_dtype)
from .exceptions import (DimensionMismatch, DomainMismatch, EmptyObject, GraphblasException,
                         IndexOutOfBound, InsufficientSpace, InvalidIndex, InvalidObject, InvalidValue,
                         NotImplementedException, NoValue, NullPointer, OutOfMemory, OutputNotEmpty,
                         Panic, UninitializedObject)
from .matrix import Matrix, MatrixExpression, TransposedMatrix
from .operator import binary, monoid, op, semiring, unary
from .scalar import Scalar, ScalarExpression
from .vector import Vector, VectorExpression

backend = "graphblas_amd"
__version__ = "0.1.0"

_initialized = False


def init(blocking=False, device=None):
    """Initialise the library (optional: first use initialises it lazily)."""
    global _initialized
    if device is not None:
        lib.GxB_Context_set_device(int(device))
    rc = lib.GrB_init(lib.GrB_BLOCKING if blocking else lib.GrB_NONBLOCKING)
    if rc not in (0, -3):  # -3: already initialised
        raise Panic(f"GrB_init failed: {rc}")
    _initialized = True


def set_stream(stream):
    """Run library work on a HIP stream (an int handle, a torch.cuda.Stream, or None)."""
    handle = getattr(stream, "cuda_stream", stream)
    rc = lib.GxB_Context_set_stream(ctypes.c_void_p(handle) if handle else None)
    if rc != 0:
        raise Panic(f"GxB_Context_set_stream failed: {rc}")


def set_knob(key, value):
    lib.GxB_Global_set_int(key.encode(), int(value))


def get_knob(key):
    """A library knob's value (GxB_Global_get_int; 0 when unset), or a read-only statistic
    ("stat_bfs_spec_adopted", "stat_bfs_spec_rollbacks")."""
    v = ctypes.c_int64()
    lib.GxB_Global_get_int(key.encode(), ctypes.byref(v))
    return v.value


def wait():
    """Block until all queued device work is complete."""
    s = Scalar(BOOL)
    s.wait()


__all__ = ["Matrix", "Vector", "Scalar", "TransposedMatrix", "Recorder", "binary", "monoid", "semiring",
           "op", "unary", "agg", "dtypes", "init", "replace", "backend", "lib"]

from . import dtypes  # noqa: E402
from . import io  # noqa: E402,F401
from .agg import agg  # noqa: E402
