"""Zero-copy access to device storage (GxB_Matrix_device_view / GxB_Vector_device_view):
lets torch.distributed (RCCL) read or write a vector's bitmap in place.
After writing through a view, call GxB_Vector_device_touch so the library recounts."""
import ctypes

from ._lib import lib


class DeviceView(ctypes.Structure):  # include/graphblas_amd.h GxB_DeviceView
    _fields_ = [("format", ctypes.c_int), ("type_code", ctypes.c_int), ("iso", ctypes.c_int),
                ("nrows", ctypes.c_int64), ("ncols", ctypes.c_int64), ("nvals", ctypes.c_int64),
                ("rowptr", ctypes.c_void_p), ("colidx", ctypes.c_void_p), ("values", ctypes.c_void_p),
                ("bitmap", ctypes.c_void_p)]


def vector_view(handle):
    v = DeviceView()
    rc = lib.GxB_Vector_device_view(ctypes.byref(v), handle)
    if rc != 0:
        raise RuntimeError(f"GxB_Vector_device_view failed: {rc}")
    return v


class _CudaArray:
    def __init__(self, ptr, n, typestr):
        self.__cuda_array_interface__ = {"shape": (int(n),), "typestr": typestr, "data": (int(ptr), False),
                                         "version": 2}


def device_tensor(torch, ptr, n, typestr="<i8"):
    """A torch tensor aliasing n elements of library device memory (no copy)."""
    return torch.as_tensor(_CudaArray(ptr, n, typestr), device="cuda")


def matrix_view(handle):
    v = DeviceView()
    rc = lib.GxB_Matrix_device_view(ctypes.byref(v), handle)
    if rc != 0:
        raise RuntimeError(f"GxB_Matrix_device_view failed: {rc}")
    return v


def colwords_view(handle):
    """(device address, count) of a <=64-row matrix's column words (GxB_Matrix_colwords_view);
    rewrite them in place on the library stream, then GxB_Matrix_colwords_touch."""
    ptr = ctypes.c_void_p()
    n = ctypes.c_uint64()
    rc = lib.GxB_Matrix_colwords_view(ctypes.byref(ptr), ctypes.byref(n), handle)
    if rc != 0:
        raise RuntimeError(f"GxB_Matrix_colwords_view failed: {rc}")
    return ptr.value, n.value
