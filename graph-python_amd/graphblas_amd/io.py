"""Matrix Market I/O (reference graphblas/io/_matrixmarket.py:6-61 mmread / mmwrite).

`mmread` parses coordinate files with the library's multithreaded host reader
(GxB_MatrixMarket_read_coo) and builds the matrix on the device
(GrB_Matrix_build_*, like Matrix.from_coo); engine="scipy" (also used for
file objects and compressed files) goes through scipy.io.mmread as the
reference does.  `mmwrite` writes a coordinate file from to_coo()."""
import ctypes
import os

import numpy as np

from ._lib import lib
from .matrix import Matrix

_CODE_DTYPE = {0: "BOOL", 7: "INT64", 10: "FP64"}


def read_coo(path):
    """(nrows, ncols, rows, cols, values, dtype_name) from a .mtx file, via the native reader."""
    nr, nc, nv = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
    code = ctypes.c_int()
    pi, pj, px = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_void_p()
    rc = lib.GxB_MatrixMarket_read_coo(os.fsencode(path), ctypes.byref(nr), ctypes.byref(nc), ctypes.byref(nv),
                                       ctypes.byref(code), ctypes.byref(pi), ctypes.byref(pj), ctypes.byref(px))
    if rc != 0:
        raise ValueError(f"cannot read Matrix Market file {path!r} (GrB_Info {rc})")
    n = nv.value
    dt = _CODE_DTYPE[code.value]
    npdt = {"BOOL": np.bool_, "INT64": np.int64, "FP64": np.float64}[dt]
    try:
        if n:
            rows = np.ctypeslib.as_array((ctypes.c_uint64 * n).from_address(pi.value)).copy()
            cols = np.ctypeslib.as_array((ctypes.c_uint64 * n).from_address(pj.value)).copy()
            vals = np.frombuffer((ctypes.c_char * (n * np.dtype(npdt).itemsize)).from_address(px.value),
                                 dtype=npdt).copy()
        else:
            rows = cols = np.empty(0, np.uint64)
            vals = np.empty(0, npdt)
    finally:
        for p in (pi, pj, px):
            lib.GxB_MatrixMarket_free(p)
    return nr.value, nc.value, rows, cols, vals, dt


def mmread(source, engine="auto", *, dup_op=None, name=None, **kwargs):
    engine = engine.lower()
    if engine not in {"auto", "native", "scipy", "fmm", "fast_matrix_market"}:
        raise ValueError(f'Bad engine value: {engine!r}. Must be "auto", "native" or "scipy"')
    is_path = isinstance(source, (str, os.PathLike))
    if engine in {"auto", "native"} and is_path and not os.fspath(source).endswith((".gz", ".bz2")):
        try:
            nr, nc, r, c, v, dt = read_coo(source)
        except ValueError:
            if engine == "native":
                raise
        else:
            vals = True if dt == "BOOL" else v  # pattern: iso true, as from_coo with a scalar
            return Matrix.from_coo(r, c, vals, dtype=dt, nrows=nr, ncols=nc, dup_op=dup_op, name=name)
    from scipy.io import mmread as sp_mmread

    array = sp_mmread(source, **kwargs)
    if getattr(array, "format", None) == "coo":
        nrows, ncols = array.shape
        return Matrix.from_coo(array.row, array.col, array.data, nrows=nrows, ncols=ncols, dup_op=dup_op,
                               name=name)
    arr = np.asarray(array)
    rows, cols = np.nonzero(np.ones_like(arr, dtype=bool))
    return Matrix.from_coo(rows, cols, arr[rows, cols], nrows=arr.shape[0], ncols=arr.shape[1], name=name)


def mmwrite(target, matrix, engine="auto", *, comment="", field=None, precision=None, symmetry=None, **kwargs):
    if symmetry not in (None, "general"):
        raise NotImplementedError("only general symmetry is written")
    rows, cols, vals = matrix.to_coo()
    dt = matrix.dtype.name if hasattr(matrix.dtype, "name") else str(matrix.dtype)
    if field is None:
        field = "pattern" if dt == "BOOL" else ("real" if dt.startswith("FP") else "integer")
    lines = [f"%%MatrixMarket matrix coordinate {field} general"]
    if comment:
        lines += ["%" + ln for ln in comment.split("\n")]
    lines.append(f"{matrix.nrows} {matrix.ncols} {len(rows)}")
    r1 = np.asarray(rows, np.int64) + 1
    c1 = np.asarray(cols, np.int64) + 1
    if field == "pattern":
        body = np.column_stack([r1, c1])
        fmt = "%d %d"
    elif field == "real":
        body = np.column_stack([r1, c1, np.asarray(vals, np.float64)])
        fmt = "%d %d %." + str(precision or 17) + "g"
    else:
        body = np.column_stack([r1, c1, np.asarray(vals, np.int64)])
        fmt = "%d %d %d"
    with open(target, "w") as f:
        f.write("\n".join(lines) + "\n")
        if len(rows):
            np.savetxt(f, body, fmt=fmt)
