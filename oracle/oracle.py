"""CPU oracle for GrB_mxm / GrB_mxv / GrB_vxm -- TEST INFRASTRUCTURE ONLY.

ctypes + numpy front for the C restatement in gb_oracle.c (see its header for
what it restates and how it is pinned).  Only tests/, __graft_entry__.smoke()
and bench.py's cpu_baseline leg may import this module; the product package
(graph-python_amd/graphblas_amd) never does.

Objects are plain numpy CSR triples.  Vectors are (size, indices, values) and
are lifted to n x 1 (mxv) or 1 x n (vxm) matrices exactly as the C API defines
GrB_mxv / GrB_vxm (reference docs/user_guide/operations.rst:17-22).
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "_build", "libgb_oracle.so")

TYPES = ["BOOL", "INT8", "UINT8", "INT16", "UINT16", "INT32", "UINT32", "INT64", "UINT64",
         "FP32", "FP64"]
TCODE = {t: i for i, t in enumerate(TYPES)}
NP = {"BOOL": np.bool_, "INT8": np.int8, "UINT8": np.uint8, "INT16": np.int16,
      "UINT16": np.uint16, "INT32": np.int32, "UINT32": np.uint32, "INT64": np.int64,
      "UINT64": np.uint64, "FP32": np.float32, "FP64": np.float64}

BINOPS = ["FIRST", "SECOND", "ANY", "PAIR", "MIN", "MAX", "PLUS", "MINUS", "RMINUS",
          "TIMES", "DIV", "RDIV", "POW", "ISEQ", "ISNE", "ISGT", "ISLT", "ISGE", "ISLE",
          "LOR", "LAND", "LXOR", "LXNOR", "EQ", "NE", "GT", "LT", "GE", "LE",
          "BOR", "BAND", "BXOR", "BXNOR", "FIRSTI", "FIRSTI1", "FIRSTJ", "FIRSTJ1",
          "SECONDI", "SECONDI1", "SECONDJ", "SECONDJ1"]
OPCODE = {n: i for i, n in enumerate(BINOPS)}
MONOIDS = ["PLUS", "TIMES", "MIN", "MAX", "ANY", "LOR", "LAND", "LXOR", "LXNOR",
           "BOR", "BAND", "BXOR", "BXNOR"]
MCODE = {n: i for i, n in enumerate(MONOIDS)}
MCODE["EQ"] = MCODE["LXNOR"]
BOOL_OUT = {"EQ", "NE", "GT", "LT", "GE", "LE"}
POSITIONAL = {"FIRSTI", "FIRSTI1", "FIRSTJ", "FIRSTJ1", "SECONDI", "SECONDI1", "SECONDJ",
              "SECONDJ1"}


class _Csr(ctypes.Structure):
    _fields_ = [("nrows", ctypes.c_int64), ("ncols", ctypes.c_int64), ("type", ctypes.c_int),
                ("p", ctypes.c_void_p), ("j", ctypes.c_void_p), ("x", ctypes.c_void_p)]


_lib = None


def build():
    """Compile the oracle (gcc) into oracle/_build/."""
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        _lib = ctypes.CDLL(LIB)
        _lib.or_mxm.restype = ctypes.c_int
        _lib.or_rmat.restype = ctypes.c_int
    return _lib


class Csr:
    """Host CSR: indptr int64[nrows+1], indices int64 (sorted per row), values numpy."""

    def __init__(self, nrows, ncols, dtype, indptr, indices, values):
        self.nrows, self.ncols, self.dtype = int(nrows), int(ncols), dtype
        self.indptr = np.ascontiguousarray(indptr, np.int64)
        self.indices = np.ascontiguousarray(indices, np.int64)
        self.values = np.ascontiguousarray(values, NP[dtype])

    @property
    def nvals(self):
        return int(self.indptr[-1])

    @classmethod
    def from_coo(cls, rows, cols, values, nrows=None, ncols=None, dtype=None):
        rows = np.asarray(rows, np.int64)
        cols = np.asarray(cols, np.int64)
        if dtype is None:
            dtype = dtype_of(values)
        vals = np.broadcast_to(np.asarray(values, NP[dtype]), rows.shape).copy()
        nrows = int(rows.max() + 1) if nrows is None else nrows
        ncols = int(cols.max() + 1) if ncols is None else ncols
        order = np.lexsort((cols, rows))
        rows, cols, vals = rows[order], cols[order], vals[order]
        if len(rows) > 1:
            dup = (rows[1:] == rows[:-1]) & (cols[1:] == cols[:-1])
            if dup.any():
                raise ValueError("duplicate indices")
        indptr = np.zeros(nrows + 1, np.int64)
        np.add.at(indptr, rows + 1, 1)
        return cls(nrows, ncols, dtype, np.cumsum(indptr), cols, vals)

    @classmethod
    def empty(cls, nrows, ncols, dtype):
        return cls(nrows, ncols, dtype, np.zeros(nrows + 1, np.int64), np.zeros(0, np.int64),
                   np.zeros(0, NP[dtype]))

    def to_coo(self):
        rows = np.repeat(np.arange(self.nrows, dtype=np.int64), np.diff(self.indptr))
        return rows, self.indices.copy(), self.values.copy()

    def to_dict(self):
        r, c, v = self.to_coo()
        return {(int(a), int(b)): v[i].item() for i, (a, b) in enumerate(zip(r, c))}

    def copy(self):
        return Csr(self.nrows, self.ncols, self.dtype, self.indptr.copy(), self.indices.copy(),
                   self.values.copy())

    def _c(self):
        s = _Csr(self.nrows, self.ncols, TCODE[self.dtype], self.indptr.ctypes.data,
                 self.indices.ctypes.data, self.values.ctypes.data if self.values.size else None)
        return s

    @staticmethod
    def _from_c(s, dtype):
        n = s.nrows
        p = np.ctypeslib.as_array(ctypes.cast(s.p, ctypes.POINTER(ctypes.c_int64)), (n + 1,)).copy()
        nz = int(p[-1])
        j = (np.ctypeslib.as_array(ctypes.cast(s.j, ctypes.POINTER(ctypes.c_int64)), (nz,)).copy()
             if nz else np.zeros(0, np.int64))
        if nz and s.x:
            raw = ctypes.string_at(s.x, nz * np.dtype(NP[dtype]).itemsize)
            x = np.frombuffer(raw, NP[dtype]).copy()
        else:
            x = np.zeros(nz, NP[dtype])
        return Csr(s.nrows, s.ncols, dtype, p, j, x)


def dtype_of(values):
    a = np.asarray(values)
    if a.dtype == np.bool_:
        return "BOOL"
    if np.issubdtype(a.dtype, np.floating):
        return "FP32" if a.dtype == np.float32 else "FP64"
    if np.issubdtype(a.dtype, np.unsignedinteger):
        return {1: "UINT8", 2: "UINT16", 4: "UINT32", 8: "UINT64"}[a.dtype.itemsize]
    if np.issubdtype(a.dtype, np.integer):
        return {1: "INT8", 2: "INT16", 4: "INT32", 8: "INT64"}[a.dtype.itemsize]
    raise TypeError(a.dtype)


def semiring_types(monoid, mulop, xtype):
    """(xtype or None, ztype) of a builtin semiring named monoid_mulop over xtype."""
    mulop = mulop.upper()
    if mulop in POSITIONAL:
        return None, xtype
    if mulop in BOOL_OUT:
        return xtype, "BOOL"
    return xtype, xtype


def mxm(C, A, B, semiring, *, mask=None, mask_comp=False, mask_struct=False, replace=False,
        accum=None, tran0=False, tran1=False):
    """C<mask> = C accum (A' (+).(x) B') -> new Csr.

    semiring = (monoid name, mulop name, xtype); accum = (binop name, type) or None.
    """
    mon, mul, xt = semiring
    xt_, zt = semiring_types(mon, mul, xt)
    out = C._c()
    keep = [C, A, B, mask]
    if accum is not None:
        aop, at = accum
        azt = "BOOL" if aop.upper() in BOOL_OUT else at
        acode, atc, aztc = OPCODE[aop.upper()], TCODE[at], TCODE[azt]
    else:
        acode, atc, aztc = -1, 0, 0
    rc = lib().or_mxm(
        ctypes.byref(out), ctypes.byref(mask._c()) if mask is not None else None,
        int(mask_comp), int(mask_struct), int(replace), acode, atc, aztc,
        MCODE[mon.upper()], OPCODE[mul.upper()], TCODE[xt_] if xt_ else -1, TCODE[zt],
        ctypes.byref(A._c()), int(tran0), ctypes.byref(B._c()), int(tran1))
    del keep
    if rc != 0:
        raise ValueError(f"oracle or_mxm failed: {rc}")
    res = Csr._from_c(out, C.dtype)
    libc = ctypes.CDLL(None)
    libc.free.argtypes = [ctypes.c_void_p]
    for ptr in (out.p, out.j, out.x):
        if ptr:
            libc.free(ptr)
    return res


# ---- vectors as (size, indices, values)
class Vec:
    def __init__(self, size, dtype, indices, values):
        self.size, self.dtype = int(size), dtype
        self.indices = np.asarray(indices, np.int64)
        self.values = np.asarray(values, NP[dtype])

    @classmethod
    def from_coo(cls, indices, values, size=None, dtype=None):
        indices = np.asarray(indices, np.int64)
        dtype = dtype or dtype_of(values)
        vals = np.broadcast_to(np.asarray(values, NP[dtype]), indices.shape).copy()
        size = int(indices.max() + 1) if size is None else size
        o = np.argsort(indices, kind="stable")
        return cls(size, dtype, indices[o], vals[o])

    def col(self):  # n x 1
        p = np.zeros(self.size + 1, np.int64)
        p[self.indices + 1] = 1
        return Csr(self.size, 1, self.dtype, np.cumsum(p), np.zeros(len(self.indices), np.int64),
                   self.values)

    def row(self):  # 1 x n
        return Csr(1, self.size, self.dtype, np.array([0, len(self.indices)], np.int64),
                   self.indices, self.values)

    @classmethod
    def from_col(cls, m):
        rows = np.repeat(np.arange(m.nrows), np.diff(m.indptr))
        return cls(m.nrows, m.dtype, rows, m.values)

    @classmethod
    def from_row(cls, m):
        return cls(m.ncols, m.dtype, m.indices, m.values)

    def to_dict(self):
        return {int(i): v.item() for i, v in zip(self.indices, self.values)}

    def copy(self):
        return Vec(self.size, self.dtype, self.indices.copy(), self.values.copy())


def mxv(w, A, u, semiring, *, mask=None, tran0=False, **kw):
    """w<mask> = w accum (A' (+).(x) u), u treated as n x 1."""
    C = mxm(w.col(), A, u.col(), semiring, mask=mask.col() if mask is not None else None,
            tran0=tran0, **kw)
    return Vec.from_col(C)


def vxm(w, u, A, semiring, *, mask=None, tran1=False, **kw):
    """w<mask> = w accum (u' (+).(x) A'), u treated as 1 x n."""
    C = mxm(w.row(), u.row(), A, semiring, mask=mask.row() if mask is not None else None,
            tran1=tran1, **kw)
    return Vec.from_row(C)


# ---- R-MAT (same generator as the device; gb_oracle.c or_rmat)
def rmat(scale, edge_factor=16, seed=42, values=None, value_seed=2):
    s = _Csr()
    lib().or_rmat(ctypes.byref(s), int(scale), int(edge_factor), ctypes.c_uint64(seed))
    if values == "INT64":
        lib().or_rmat_values(ctypes.byref(s), 0, ctypes.c_uint64(value_seed))
        dtype = "INT64"
    elif values == "FP64":
        lib().or_rmat_values(ctypes.byref(s), 1, ctypes.c_uint64(value_seed))
        dtype = "FP64"
    else:
        dtype = "BOOL"
    m = Csr._from_c(s, dtype)
    if dtype == "BOOL":
        m.values = np.ones(m.nvals, np.bool_)
    libc = ctypes.CDLL(None)
    libc.free.argtypes = [ctypes.c_void_p]
    for ptr in (s.p, s.j, s.x):
        if ptr:
            libc.free(ptr)
    return m


def bfs_levels(A, src):
    """Direct-loop level BFS (levels: src = 1, unreached = 0); returns (levels, nlevels, edges)."""
    lev = np.zeros(A.nrows, np.int32)
    edges = ctypes.c_int64(0)
    nl = lib().or_bfs_levels(ctypes.byref(A._c()), ctypes.c_int64(src),
                             lev.ctypes.data_as(ctypes.c_void_p), ctypes.byref(edges))
    return lev, nl, edges.value


def bfs_levels_par(A, AT, src, nthreads):
    """or_bfs_levels on nthreads host threads (push/pull per level); AT = A^T or None."""
    lev = np.zeros(A.nrows, np.int32)
    edges = ctypes.c_int64(0)
    cat = AT._c() if AT is not None else None
    nl = lib().or_bfs_levels_par(ctypes.byref(A._c()), ctypes.byref(cat) if cat is not None else None,
                                 ctypes.c_int64(src), lev.ctypes.data_as(ctypes.c_void_p), ctypes.byref(edges),
                                 ctypes.c_int(nthreads))
    return lev, nl, edges.value


def spmv_plus_times_fp64_par(AT, x, nthreads):
    """CPU baseline (config 2): y = x plus.times A over AT = A^T (FP64 Csr); -> (y, present)."""
    y = np.empty(AT.nrows, np.float64)
    present = np.empty(AT.nrows, np.uint8)
    x = np.ascontiguousarray(x, np.float64)
    lib().or_spmv_plus_times_fp64_par(ctypes.byref(AT._c()), x.ctypes.data_as(ctypes.c_void_p),
                                      y.ctypes.data_as(ctypes.c_void_p), present.ctypes.data_as(ctypes.c_void_p),
                                      ctypes.c_int(nthreads))
    return y, present.astype(bool)


def masked_dot_min_plus_int64_par(A, AT, row0, row1, nthreads):
    """CPU baseline (config 4): C<A.S> = A min.+ A over mask rows [row0, row1) (INT64 Csr A and
    AT = A^T); -> (values per mask entry, present per mask entry, nnz(C) rows, work)."""
    m = int(A.indptr[row1] - A.indptr[row0])
    vals = np.zeros(max(m, 1), np.int64)
    present = np.zeros(max(m, 1), np.uint8)
    work = ctypes.c_int64(0)
    f = lib().or_masked_dot_min_plus_int64_par
    f.restype = ctypes.c_int64
    nc = f(ctypes.byref(A._c()), ctypes.byref(AT._c()), ctypes.c_int64(row0), ctypes.c_int64(row1),
           vals.ctypes.data_as(ctypes.c_void_p), present.ctypes.data_as(ctypes.c_void_p), ctypes.byref(work),
           ctypes.c_int(nthreads))
    return vals[:m], present[:m].astype(bool), int(nc), work.value


def spgemm_plus_times_fp64_par(A, B, row0, row1, nthreads):
    """CPU baseline (config 5): C = A plus.times B (FP64 Csr, unmasked) over the rows [row0, row1)
    of A, Gustavson on nthreads host threads; -> (C rows as a Csr, products)."""
    out = _Csr()
    prods = ctypes.c_int64(0)
    f = lib().or_spgemm_plus_times_fp64_par
    f.restype = ctypes.c_int64
    f(ctypes.byref(A._c()), ctypes.byref(B._c()), ctypes.c_int64(row0), ctypes.c_int64(row1), ctypes.byref(out),
      ctypes.byref(prods), ctypes.c_int(nthreads))
    C = Csr._from_c(out, "FP64")
    lib().or_csr_free(ctypes.byref(out))
    return C, prods.value


def bfs_graphblas(A, src):
    """The Level-BFS loop of the reference notebook (Example B.1 cell 8) through or_mxm:
       v[:](mask=q.V) << d ; q(~v.S, replace) << q.vxm(A, lor_land) ; stop when q empty."""
    n = A.nrows
    v_lev = np.zeros(n, np.int32)
    visited = np.zeros(n, np.bool_)
    q = Vec(n, "BOOL", [src], [True])
    d = 0
    while True:
        d += 1
        sel = q.indices[q.values]
        v_lev[sel] = d
        visited[sel] = True
        vmask = Vec(n, "INT32", np.flatnonzero(visited), v_lev[visited])
        q = vxm(q, q, A, ("LOR", "LAND", "BOOL"), mask=vmask, mask_comp=True, mask_struct=True,
                replace=True)
        if not q.values.any():
            break
    return v_lev
