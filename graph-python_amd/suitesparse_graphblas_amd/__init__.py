"""A `suitesparse_graphblas`-shaped binding of libgraphblas_amd.so.

python-graphblas reaches its C library only through the module it imports at
graphblas/__init__.py:141 (`from suitesparse_graphblas import ffi, initialize,
is_initialized, lib`) and then injects as `graphblas.core.ffi/lib/NULL`
(:195-197).  This module provides those names over libgraphblas_amd.so with cffi
in ABI mode (no compiler needed): `ffi` parses include/graphblas_amd_cdef.h
(generated from the C ABI header by tools/gen_cdef.py) and `lib` is a plain
namespace holding every declared function, enum constant and builtin object, so
both `getattr(lib, name)` (core/utils.py:9-21) and `vars(lib)` (the
"suitesparse-vanilla" backend, graphblas/__init__.py:173-183) work.

Scope: the vanilla C API 2.0 surface of the masked mxm/mxv/vxm path (SURVEY.md
§8b).  SuiteSparse-only GxB pack/unpack (which needs `utils.claim_buffer`) is
not provided.  See INTEGRATION.md.
"""
import os

import cffi

__version__ = "7.4.0.0+mi355x"  # API level of the replaced suitesparse-graphblas pin (pyproject.toml:65)

_HERE = os.path.dirname(os.path.abspath(__file__))
_REPO = os.path.dirname(os.path.dirname(_HERE))
_CDEF = os.path.join(_REPO, "include", "graphblas_amd_cdef.h")
_SO = os.environ.get("GRAPHBLAS_AMD_LIB", os.path.join(_REPO, "graph-python_amd", "graphblas_amd",
                                                        "libgraphblas_amd.so"))

ffi = cffi.FFI()
with open(_CDEF) as _f:
    ffi.cdef(_f.read())
if not os.path.exists(_SO):
    raise ImportError(f"libgraphblas_amd.so not found at {_SO} (build it: python -c "
                      "'import __graft_entry__; __graft_entry__.build()')")
_dl = ffi.dlopen(_SO)

class _GlobalVar:
    """What `vars(lib)` holds for a C global variable (builtin types, operators, semirings,
    descriptors, GrB_ALL), as in the compiled cffi module python-graphblas normally gets:
    not the value and not callable, so the "suitesparse-vanilla" strip
    (`callable(val) and key.startswith("GxB")`, reference graphblas/__init__.py:180-184)
    keeps GxB_* objects and drops only GxB_* functions; `getattr(lib, name)` returns the
    value (the strip copies with getattr, :184)."""

    __slots__ = ("name",)

    def __init__(self, name):
        self.name = name

    def __repr__(self):
        return f"<global variable {self.name}>"


def _make_lib():
    """`lib`: every declared function, integer constant and global variable, resolved once
    (vars(lib) lists them all; reference core/operator/base.py:291 scans dir(lib))."""
    props, inst = {}, {}
    for name in dir(_dl):
        val = getattr(_dl, name)
        if isinstance(val, ffi.CData) and ffi.typeof(val).kind != "function":
            props[name] = property(lambda self, _v=val: _v)  # data descriptor: wins over vars()
            inst[name] = _GlobalVar(name)
        else:
            inst[name] = val
    cls = type("lib", (), props)
    obj = cls()
    obj.__dict__.update(inst)
    return obj


lib = _make_lib()

_initialized = False


def is_initialized():
    return _initialized


def initialize(*, blocking=False, memory_manager="numpy"):
    """GrB_init in the requested mode.  Export buffers are always caller-allocated
    (numpy) on this backend, so `memory_manager` is accepted for compatibility."""
    global _initialized
    if _initialized:
        raise RuntimeError("GraphBLAS is already initialized")
    info = lib.GrB_init(lib.GrB_BLOCKING if blocking else lib.GrB_NONBLOCKING)
    if info != lib.GrB_SUCCESS:
        raise RuntimeError(f"GrB_init failed with GrB_Info {info}")
    _initialized = True


class utils:  # noqa: N801  (mirrors suitesparse_graphblas.utils)
    @staticmethod
    def claim_buffer(*args, **kwargs):
        raise NotImplementedError("GxB pack/unpack buffers are not part of this backend's surface")

    @staticmethod
    def unclaim_buffer(*args, **kwargs):
        raise NotImplementedError("GxB pack/unpack buffers are not part of this backend's surface")
