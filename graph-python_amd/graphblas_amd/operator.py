"""Operator registry: BinaryOp / Monoid / Semiring objects discovered from the
names the C library exports, exactly as python-graphblas discovers them from
``dir(lib)`` (reference core/operator/base.py:397-486, semiring.py:170-204,
monoid.py:179-195, binary.py:332-369), plus the typed-op selection rules of
``get_typed_op`` (reference core/operator/utils.py:38-132) and the boolean /
positional coercions of ``Semiring._initialize`` (semiring.py:346-511).
"""
import types

from . import _builtins
from ._lib import lib
from .dtypes import BOOL, INT64, DataType, lookup_dtype, unify


class TypedOp:
    __slots__ = ("parent", "name", "type", "return_type", "gb_obj", "gb_name", "opclass",
                 "_monoid", "_binaryop")

    def __init__(self, parent, name, dtype, ret, gb_name, opclass):
        self.parent = parent
        self.name = name
        self.type = dtype
        self.return_type = ret
        self.gb_name = gb_name
        self.gb_obj = getattr(lib, gb_name)
        self.opclass = opclass
        self._monoid = None
        self._binaryop = None

    @property
    def _carg(self):
        return self.gb_obj

    @property
    def monoid(self):
        return self._monoid

    @property
    def binaryop(self):
        return self._binaryop

    @property
    def is_positional(self):
        return self.parent.is_positional

    def __repr__(self):
        return f"{self.opclass.lower()}.{self.name}[{self.type}]"

    def __call__(self, expr, right=None):
        return _call_op(self, expr, right)


class OpBase:
    opclass = None

    def __init__(self, name):
        self.name = name
        self._typed = {}  # DataType -> TypedOp
        self.types = {}  # DataType -> return DataType
        self.coercions = {}
        self.is_positional = False

    def _add(self, typed):
        self._typed[typed.type] = typed
        self.types[typed.type] = typed.return_type

    def __getitem__(self, dtype):
        dtype = lookup_dtype(dtype)
        if dtype in self._typed:
            return self._typed[dtype]
        raise KeyError(f"{self.opclass.lower()}.{self.name} does not work with {dtype}")

    def __contains__(self, dtype):
        try:
            return lookup_dtype(dtype) in self._typed
        except ValueError:
            return False

    def __repr__(self):
        return f"{self.opclass.lower()}.{self.name}"

    def __call__(self, expr, right=None):
        return _call_op(self, expr, right)


class BinaryOp(OpBase):
    opclass = "BinaryOp"


class UnaryOp(OpBase):
    opclass = "UnaryOp"


class Monoid(OpBase):
    opclass = "Monoid"

    @property
    def binaryop(self):
        return getattr(binary, self.name)


class Semiring(OpBase):
    opclass = "Semiring"


class _Namespace(types.SimpleNamespace):
    def __getitem__(self, name):
        return getattr(self, name)


binary = _Namespace()
unary = _Namespace()
monoid = _Namespace()
semiring = _Namespace()


def _get(ns, cls, name):
    obj = getattr(ns, name, None)
    if obj is None:
        obj = cls(name)
        setattr(ns, name, obj)
    return obj


# ---------------------------------------------------------------- discovery
for _gb, (_op, _x, _z) in _builtins.BINOPS.items():
    _tname = _gb.split("_")[-1] if _gb.count("_") >= 2 else "BOOL"
    _pyname = _op.lower()
    _o = _get(binary, BinaryOp, _pyname)
    _o.is_positional = _x is None
    _dt = lookup_dtype(_tname)
    # GrB_LOR (no suffix) is the BOOL version; keep the GrB_ name when both exist
    if _dt in _o._typed and _o._typed[_dt].gb_name.startswith("GrB_"):
        continue
    _o._add(TypedOp(_o, _pyname, _dt, lookup_dtype(_z), _gb, "BinaryOp"))

for _gb, (_op, _t) in _builtins.UNOPS.items():
    _pyname = _op.lower()
    _o = _get(unary, UnaryOp, _pyname)
    _dt = lookup_dtype(_t)
    if _dt in _o._typed and _o._typed[_dt].gb_name.startswith("GrB_"):
        continue
    _o._add(TypedOp(_o, _pyname, _dt, _dt, _gb, "UnaryOp"))

for _gb, (_m, _t, _bop) in _builtins.MONOIDS.items():
    _pyname = "eq" if _gb == "GxB_EQ_BOOL_MONOID" else _m.lower()
    _o = _get(monoid, Monoid, _pyname)
    _dt = lookup_dtype(_t)
    if _dt in _o._typed:
        continue
    _to = TypedOp(_o, _pyname, _dt, _dt, _gb, "Monoid")
    _to._binaryop = binary.__dict__.get(_bop.split("_")[1].lower() if _bop.count("_") else _bop)
    _o._add(_to)

for _gb, (_mon, _bop, _aliases) in _builtins.SEMIRINGS.items():
    _src = _aliases[0] if _aliases else _gb
    _body = _src[4:].replace("_SEMIRING", "")
    _parts = _body.split("_")
    _tname = _parts[-1]
    _pyname = "_".join(_parts[:-1]).lower()
    _o = _get(semiring, Semiring, _pyname)
    _xt, _zt = _builtins.BINOPS[_bop][1], _builtins.BINOPS[_bop][2]
    _o.is_positional = _xt is None
    _dt = lookup_dtype(_tname)
    _to = TypedOp(_o, _pyname, _dt, lookup_dtype(_builtins.MONOIDS[_mon][1]), _src, "Semiring")
    _to._monoid = monoid.__dict__.get(_pyname.split("_")[0])
    _to._binaryop = binary.__dict__.get("_".join(_pyname.split("_")[1:]))
    _o._add(_to)

# ---- coercions (reference core/operator/semiring.py:383-510)
_NOTBOOL = [lookup_dtype(t) for t in
            ["FP32", "FP64", "INT8", "INT16", "INT32", "INT64", "UINT8", "UINT16", "UINT32", "UINT64"]]
_POSDT = [lookup_dtype(t) for t in ["BOOL", "FP32", "FP64", "INT8", "INT16", "UINT8", "UINT16",
                                    "UINT32", "UINT64"]]


def _coerce(op, dtypes, target):
    if target not in op._typed:
        return
    for dt in dtypes:
        if dt not in op._typed:
            op._typed[dt] = op._typed[target]
            op.types[dt] = op.types[target]
            op.coercions[dt] = target


for _l in ["any", "max", "min", "plus", "times"]:
    for _r in ["firsti", "firsti1", "firstj", "firstj1", "secondi", "secondi1", "secondj", "secondj1"]:
        if hasattr(semiring, f"{_l}_{_r}"):
            _coerce(getattr(semiring, f"{_l}_{_r}"), _POSDT, INT64)
for _l in ["eq", "land", "lor", "lxnor", "lxor"]:
    for _r in ["first", "pair", "second"]:
        if hasattr(semiring, f"{_l}_{_r}"):
            _coerce(getattr(semiring, f"{_l}_{_r}"), _NOTBOOL, BOOL)
for _l in ["any", "eq", "land", "lor", "lxnor", "lxor"]:
    for _r in ["eq", "land", "lor", "lxnor", "lxor", "ne"]:
        if hasattr(semiring, f"{_l}_{_r}"):
            _coerce(getattr(semiring, f"{_l}_{_r}"), _NOTBOOL, BOOL)
for _opname, _target in [("max_first", "lor_first"), ("max_second", "lor_second"),
                         ("max_land", "lor_land"), ("max_lor", "lor_lor"), ("max_lxor", "lor_lxor"),
                         ("min_first", "land_first"), ("min_second", "land_second"),
                         ("min_land", "land_land"), ("min_lor", "land_lor"),
                         ("min_lxor", "land_lxor")]:
    _a, _b = getattr(semiring, _opname, None), getattr(semiring, _target, None)
    if _a is not None and _b is not None and BOOL not in _a._typed and BOOL in _b._typed:
        _a._typed[BOOL] = _b._typed[BOOL]
        _a.types[BOOL] = _b.types[BOOL]
        _a.coercions[BOOL] = BOOL
# positional binary ops on non-integer inputs use the INT64 version
for _r in ["firsti", "firsti1", "firstj", "firstj1", "secondi", "secondi1", "secondj", "secondj1"]:
    _coerce(getattr(binary, _r), _POSDT, INT64)

# monoid coercions (reference core/operator/monoid.py:396-431): bool max/min/times are lor/land/land;
# the logical monoids on numeric inputs use the BOOL monoid (values cast to bool)
for _name, _target in [("max", "lor"), ("min", "land"), ("times", "land")]:
    _a, _b = getattr(monoid, _name), getattr(monoid, _target)
    if BOOL not in _a._typed:
        _a._typed[BOOL] = _b._typed[BOOL]
        _a.types[BOOL] = BOOL
        _a.coercions[BOOL] = BOOL
for _name in ["lor", "land", "lxnor", "lxor"]:
    _a = getattr(monoid, _name)
    for _dt in _NOTBOOL:
        if _dt not in _a._typed:
            _a._typed[_dt] = _a._typed[BOOL]
            _a.types[_dt] = BOOL
            _a.coercions[_dt] = BOOL

# float-only unary ops on integer / bool inputs (reference core/operator/unary.py:381-428)
_F32_FROM = [lookup_dtype(t) for t in ["BOOL", "INT8", "INT16", "UINT8", "UINT16"]]
_F64_FROM = [lookup_dtype(t) for t in ["INT32", "INT64", "UINT32", "UINT64"]]
for _u in unary.__dict__.values():
    if lookup_dtype("FP64") in _u._typed and lookup_dtype("INT64") not in _u._typed:
        _coerce(_u, _F32_FROM, lookup_dtype("FP32"))
        _coerce(_u, _F64_FROM, lookup_dtype("FP64"))


# ---- semirings python-graphblas builds from a monoid and a binary op when the library has no
# builtin of that name (e.g. plus_pow for agg.sum_of_squares, reference core/operator/agg.py:266-276):
# GrB_Semiring_new on the builtin pieces
class _UserTypedSemiring(TypedOp):
    __slots__ = ("_cell",)

    def __init__(self, parent, name, dtype, ret, mon, bop):
        import ctypes

        self.parent, self.name, self.type, self.return_type = parent, name, dtype, ret
        self.gb_name, self.opclass = name, "Semiring"
        self._cell = ctypes.c_void_p()
        rc = lib.GrB_Semiring_new(ctypes.byref(self._cell), mon.gb_obj, bop.gb_obj)
        if rc != 0:
            raise ValueError(f"GrB_Semiring_new({mon.gb_name}, {bop.gb_name}) failed ({rc})")
        self.gb_obj = self._cell
        self._monoid = mon.parent
        self._binaryop = bop.parent


def _user_semiring(mon_name, bop_name):
    name = f"{mon_name}_{bop_name}"
    if hasattr(semiring, name):
        return getattr(semiring, name)
    mon, bop = getattr(monoid, mon_name), getattr(binary, bop_name)
    o = Semiring(name)
    for dt, bt in bop._typed.items():
        if dt in bop.coercions or bt.return_type not in mon._typed:
            continue
        mt = mon._typed[bt.return_type]
        o._add(_UserTypedSemiring(o, name, dt, bt.return_type, mt, bt))
    setattr(semiring, name, o)
    return o


_user_semiring("plus", "pow")

op = _Namespace(**{**binary.__dict__, **unary.__dict__, **monoid.__dict__, **semiring.__dict__})

_BINARY_STRINGS = {"+": "plus", "-": "minus", "*": "times", "/": "truediv", "==": "eq", "!=": "ne",
                   ">": "gt", "<": "lt", ">=": "ge", "<=": "le", "|": "lor", "&": "land",
                   "^": "lxor", "min": "min", "max": "max"}


def _from_string(s, kind):
    name = s.strip()
    dt = None
    if name.endswith("]") and "[" in name:
        name, dt = name[:-1].split("[", 1)
    name = _BINARY_STRINGS.get(name, name).lower()
    ns = {"binary": binary, "monoid": monoid, "semiring": semiring, "unary": unary}[kind]
    if not hasattr(ns, name):
        raise ValueError(f"Unknown {kind} string: {s!r}")
    obj = getattr(ns, name)
    return obj[dt] if dt else obj


def get_typed_op(opobj, dtype, dtype2=None, *, kind=None, is_left_scalar=False, is_right_scalar=False):
    """Select the typed builtin for the given input dtypes (reference core/operator/utils.py:38-60)."""
    if isinstance(opobj, TypedOp):
        return opobj
    if isinstance(opobj, str):
        opobj = _from_string(opobj, kind)
        if isinstance(opobj, TypedOp):
            return opobj
    if not isinstance(opobj, OpBase):
        raise TypeError(f"Unable to get typed operator from object with type {type(opobj)}")
    dt = dtype if dtype2 is None else unify(dtype, dtype2, is_left_scalar=is_left_scalar,
                                            is_right_scalar=is_right_scalar)
    if opobj.is_positional and dt not in opobj._typed:
        dt = INT64
    return opobj[dt]


def find_opclass(obj):
    if isinstance(obj, (TypedOp, OpBase)):
        return obj, obj.opclass
    return obj, "Unknown"


def _call_op(opobj, expr, right=None):
    """semiring(A @ B) / binary.plus(x | y) / binary.plus(x, 1) / unary.abs(x) style
    (reference core/operator/base.py:110-161, binary.py:175-230)."""
    from .infix import InfixExpr

    if isinstance(expr, InfixExpr):
        return expr._with_op(opobj)
    if right is not None:
        lcol, rcol = getattr(expr, "ndim", None) is not None, getattr(right, "ndim", None) is not None
        if lcol and rcol:
            return expr.ewise_add(right, opobj)
        if lcol:
            return expr.apply(opobj, right=right)
        if rcol:
            return right.apply(opobj, left=expr)
        raise TypeError(f"Bad types when calling {opobj!r}")
    if opobj.opclass == "UnaryOp" and hasattr(expr, "apply"):
        return expr.apply(opobj)
    raise TypeError(f"Bad type when calling {opobj!r}: {type(expr)}")
