"""ctypes binding of libgraphblas_amd.so, shaped like the cffi ``lib`` that
python-graphblas injects as ``graphblas.core.lib`` (reference
graphblas/__init__.py:193-197) and calls through ``core.base.call``
(reference core/base.py:23-54).

``lib.<name>`` returns a callable with its C signature for functions, and the
handle value for exported data symbols (builtin types, operators, monoids,
semirings, descriptors).  The shared library is required: importing this
module on a machine without the built ``.so`` raises ImportError -- there is
no CPU fallback.
"""
import ctypes
import os

from . import _builtins

# One HIP runtime per process: torch ships its own libamdhip64 / libhsa-runtime64.  When this
# library is loaded first, its DT_NEEDED pulls /opt/rocm's runtime in and torch's later CUDA
# init finds "no ROCm-capable device"; importing torch first makes the dynamic loader resolve
# our libamdhip64.so.7 to the runtime torch already loaded (bench.py, the device views and the
# RCCL exchange all share torch's stream / device with the library).  torch's bundled runtime
# (ROCm 7.0 wheel, soname libamdhip64.so.7) is ABI-compatible with the ROCm 7.2 the library is
# built against; a process that never uses torch can skip the import (and its seconds of start-up)
# with GRAPHBLAS_AMD_TORCH=0, after which it must not import torch's GPU side either.
if os.environ.get("GRAPHBLAS_AMD_TORCH", "1") != "0":
    try:  # torch is optional (plumbing only)
        import torch  # noqa: F401
    except Exception:
        pass

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("GRAPHBLAS_AMD_LIB", os.path.join(_HERE, "libgraphblas_amd.so"))

TYPE_NAMES = [t[0] for t in _builtins.TYPES]
_CTYPES = {
    "BOOL": ctypes.c_bool, "INT8": ctypes.c_int8, "UINT8": ctypes.c_uint8,
    "INT16": ctypes.c_int16, "UINT16": ctypes.c_uint16, "INT32": ctypes.c_int32,
    "UINT32": ctypes.c_uint32, "INT64": ctypes.c_int64, "UINT64": ctypes.c_uint64,
    "FP32": ctypes.c_float, "FP64": ctypes.c_double,
}
P, I, E, L, U = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int, ctypes.c_int64, ctypes.c_uint64

# ---------------------------------------------------------------- signatures (include/graphblas_amd.h)
_SIGS = {
    "GrB_init": [E], "GrB_finalize": [], "GrB_getVersion": [P, P],
    "GxB_Context_set_stream": [P], "GxB_Context_get_stream": [P], "GxB_Context_set_device": [E],
    "GxB_builtin_lookup": [P, P, ctypes.c_char_p], "GxB_name": [P, P],
    "GxB_Global_set_int": [ctypes.c_char_p, L], "GxB_Global_get_int": [ctypes.c_char_p, P],
    "GxB_MatrixMarket_read_coo": [ctypes.c_char_p, P, P, P, P, P, P, P], "GxB_MatrixMarket_free": [P],
    "GrB_Descriptor_new": [P], "GrB_Descriptor_set": [P, E, E], "GrB_Descriptor_free": [P],
    "GrB_Matrix_new": [P, P, I, I], "GrB_Matrix_dup": [P, P], "GrB_Matrix_clear": [P],
    "GrB_Matrix_nrows": [P, P], "GrB_Matrix_ncols": [P, P], "GrB_Matrix_nvals": [P, P],
    "GrB_Matrix_resize": [P, I, I], "GrB_Matrix_free": [P], "GrB_Matrix_wait": [P, E],
    "GrB_Matrix_error": [P, P], "GxB_Matrix_type": [P, P], "GrB_Matrix_removeElement": [P, I, I],
    "GrB_Matrix_exportSize": [P, P, P, E, P], "GrB_Matrix_exportHint": [P, P],
    "GrB_Vector_new": [P, P, I], "GrB_Vector_dup": [P, P], "GrB_Vector_clear": [P],
    "GrB_Vector_size": [P, P], "GrB_Vector_nvals": [P, P], "GrB_Vector_resize": [P, I],
    "GrB_Vector_free": [P], "GrB_Vector_wait": [P, E], "GrB_Vector_error": [P, P],
    "GxB_Vector_type": [P, P], "GrB_Vector_removeElement": [P, I],
    "GrB_Scalar_new": [P, P], "GrB_Scalar_dup": [P, P], "GrB_Scalar_clear": [P],
    "GrB_Scalar_nvals": [P, P], "GrB_Scalar_free": [P], "GrB_Scalar_wait": [P, E],
    "GrB_Scalar_error": [P, P],
    "GrB_mxm": [P] * 7, "GrB_mxv": [P] * 7, "GrB_vxm": [P] * 7,
    "GrB_Matrix_eWiseMult_BinaryOp": [P] * 7, "GrB_Vector_eWiseMult_BinaryOp": [P] * 7,
    "GrB_Matrix_eWiseAdd_BinaryOp": [P] * 7, "GrB_Vector_eWiseAdd_BinaryOp": [P] * 7,
    "GrB_Vector_assign": [P, P, P, P, P, I, P], "GrB_Matrix_assign": [P, P, P, P, P, I, P, I, P],
    "GrB_Matrix_reduce_Monoid_Scalar": [P] * 5, "GrB_Vector_reduce_Monoid_Scalar": [P] * 5,
    "GrB_transpose": [P] * 5,
    "GrB_Matrix_reduce_Monoid": [P] * 6, "GrB_Matrix_reduce_BinaryOp": [P] * 6,
    "GrB_Vector_apply": [P] * 6, "GrB_Matrix_apply": [P] * 6,
    "GrB_Semiring_new": [P, P, P], "GrB_UnaryOp_free": [P],
    "GrB_Matrix_extract": [P, P, P, P, P, I, P, I, P], "GrB_Col_extract": [P, P, P, P, P, I, I, P],
    "GrB_Vector_extract": [P, P, P, P, P, I, P], "GxB_Global_Option_get_INT32": [E, P],
    "GxB_Matrix_device_view": [P, P], "GxB_Vector_device_view": [P, P],
    "GxB_Vector_device_touch": [P], "GxB_Matrix_prepare_transpose": [P],
    "GxB_Vector_publish_ticket": [P, P], "GxB_Vector_wait_ticket": [P, P, U],
    "GxB_Matrix_rmat": [P, E, E, U, E, U, I, I],
    "GxB_Vector_bitmap_export": [P, P, I], "GxB_Vector_bitmap_import": [P, P, I],
    "GxB_Matrix_import_device": [P, P, I, I, P, P, P, I, ctypes.c_bool],
    "GxB_Matrix_colwords_view": [P, P, P], "GxB_Matrix_colwords_touch": [P],
    # device-initiated frontier exchange (gb_peer.hip)
    "GxB_PeerWindow_new": [P, I, E, E, P], "GxB_PeerWindow_handle": [P, P], "GxB_PeerWindow_open": [P, E, P],
    "GxB_PeerWindow_attach": [P, E, P], "GxB_PeerWindow_put": [P, P], "GxB_PeerWindow_wait": [P, P],
    "GxB_PeerWindow_error": [P, P], "GxB_PeerWindow_free": [P],
    # GrB_Scalar-argument variants (gb_scalar_args.cpp)
    "GrB_Vector_extractElement_Scalar": [P, P, I], "GrB_Matrix_extractElement_Scalar": [P, P, I, I],
    "GrB_Vector_setElement_Scalar": [P, P, I], "GrB_Matrix_setElement_Scalar": [P, P, I, I],
    "GrB_Vector_assign_Scalar": [P, P, P, P, P, I, P], "GrB_Matrix_assign_Scalar": [P, P, P, P, P, I, P, I, P],
    "GrB_Vector_apply_BinaryOp1st_Scalar": [P] * 7, "GrB_Vector_apply_BinaryOp2nd_Scalar": [P] * 7,
    "GrB_Matrix_apply_BinaryOp1st_Scalar": [P] * 7, "GrB_Matrix_apply_BinaryOp2nd_Scalar": [P] * 7,
}
for _t in TYPE_NAMES:
    _T = _CTYPES[_t]
    _SIGS.update({
        f"GrB_Matrix_build_{_t}": [P, P, P, P, I, P],
        f"GxB_Matrix_build_Scalar_{_t}": [P, P, P, _T, I],
        f"GrB_Matrix_setElement_{_t}": [P, _T, I, I],
        f"GrB_Matrix_extractElement_{_t}": [P, P, I, I],
        f"GrB_Matrix_extractTuples_{_t}": [P, P, P, P, P],
        f"GrB_Matrix_import_{_t}": [P, P, I, I, P, P, P, I, I, I, E],
        f"GrB_Matrix_export_{_t}": [P, P, P, P, P, P, E, P],
        f"GrB_Matrix_assign_{_t}": [P, P, P, _T, P, I, P, I, P],
        f"GrB_Matrix_reduce_{_t}": [P, P, P, P, P],
        f"GrB_Vector_build_{_t}": [P, P, P, I, P],
        f"GxB_Vector_build_Scalar_{_t}": [P, P, _T, I],
        f"GrB_Vector_setElement_{_t}": [P, _T, I],
        f"GrB_Vector_extractElement_{_t}": [P, P, I],
        f"GrB_Vector_extractTuples_{_t}": [P, P, P, P],
        f"GrB_Vector_assign_{_t}": [P, P, P, _T, P, I, P],
        f"GrB_Vector_reduce_{_t}": [P, P, P, P, P],
        f"GrB_Scalar_setElement_{_t}": [P, _T],
        f"GrB_Scalar_extractElement_{_t}": [P, P],
        f"GrB_Vector_apply_BinaryOp1st_{_t}": [P, P, P, P, _T, P, P],
        f"GrB_Vector_apply_BinaryOp2nd_{_t}": [P, P, P, P, P, _T, P],
        f"GrB_Matrix_apply_BinaryOp1st_{_t}": [P, P, P, P, _T, P, P],
        f"GrB_Matrix_apply_BinaryOp2nd_{_t}": [P, P, P, P, P, _T, P],
    })

# GrB_Info codes (C API 2.0; include/graphblas_amd.h)
INFO = {
    "GrB_SUCCESS": 0, "GrB_NO_VALUE": 1, "GrB_UNINITIALIZED_OBJECT": -1,
    "GrB_NULL_POINTER": -2, "GrB_INVALID_VALUE": -3, "GrB_INVALID_INDEX": -4,
    "GrB_DOMAIN_MISMATCH": -5, "GrB_DIMENSION_MISMATCH": -6, "GrB_OUTPUT_NOT_EMPTY": -7,
    "GrB_NOT_IMPLEMENTED": -8, "GrB_PANIC": -101, "GrB_OUT_OF_MEMORY": -102,
    "GrB_INSUFFICIENT_SPACE": -103, "GrB_INVALID_OBJECT": -104,
    "GrB_INDEX_OUT_OF_BOUNDS": -105, "GrB_EMPTY_OBJECT": -106,
}
ENUMS = {
    "GrB_NONBLOCKING": 0, "GrB_BLOCKING": 1, "GrB_COMPLETE": 0, "GrB_MATERIALIZE": 1,
    "GrB_OUTP": 0, "GrB_MASK": 1, "GrB_INP0": 2, "GrB_INP1": 3, "GxB_DEFAULT": 0,
    "GrB_REPLACE": 1, "GrB_COMP": 2, "GrB_STRUCTURE": 4, "GrB_COMP_STRUCTURE": 6, "GrB_TRAN": 3,
    "GrB_CSR_FORMAT": 0, "GrB_CSC_FORMAT": 1, "GrB_COO_FORMAT": 2,
}


class _Lib:
    """Attribute-style access to the C ABI (functions, handles, constants)."""

    def __init__(self, path):
        if not os.path.exists(path):
            raise ImportError(
                f"libgraphblas_amd.so not found at {path}; build it with "
                "`python -c 'import __graft_entry__ as g; g.build()'` (no CPU fallback exists)")
        self._dll = ctypes.CDLL(path)
        self._cache = {}
        self.path = path

    def __getattr__(self, name):
        cache = self.__dict__.get("_cache")
        if cache is not None and name in cache:
            return cache[name]
        if name in INFO:
            return INFO[name]
        if name in ENUMS:
            return ENUMS[name]
        if name == "GrB_ALL":
            v = ctypes.c_void_p.in_dll(self._dll, "GrB_ALL").value
            self._cache[name] = ctypes.c_void_p(v)
            return self._cache[name]
        if name in _SIGS:
            f = getattr(self._dll, name)
            f.argtypes = _SIGS[name]
            f.restype = ctypes.c_int
            self._cache[name] = f
            return f
        try:
            v = ctypes.c_void_p.in_dll(self._dll, name).value
        except ValueError:
            raise AttributeError(name) from None
        h = ctypes.c_void_p(v)
        self._cache[name] = h
        return h

    def __dir__(self):
        names = list(_SIGS) + list(INFO) + list(ENUMS)
        names += [f"GrB_{t}" for t in TYPE_NAMES]
        names += list(_builtins.BINOPS) + list(_builtins.UNOPS) + list(_builtins.MONOIDS) + list(_builtins.DESCRIPTORS.values())
        for k, v in _builtins.SEMIRINGS.items():
            names.append(k)
            names.extend(v[2])
        return names


lib = _Lib(LIB_PATH)
NULL = None
