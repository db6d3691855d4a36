"""The C-call trampoline, recorder, descriptors, masks and the output-binding
layer (mirrors reference core/base.py:23-54, 169-495, 563-596;
core/recorder.py:34-178; core/descriptor.py:51-156; core/mask.py:9-200;
core/expr.py:402-478).  Every GraphBLAS operation funnels through `call()`,
which issues exactly one C-ABI call into libgraphblas_amd.so."""
import ctypes
import itertools
from contextvars import ContextVar

from . import _builtins
from ._lib import lib
from .dtypes import BOOL, DataType
from .exceptions import check_status
from .operator import Monoid, OpBase, TypedOp, _from_string, binary, get_typed_op

_recorder = ContextVar("recorder", default=None)


# ---------------------------------------------------------------- names
_counters = {"M": itertools.count(), "v": itertools.count(), "s": itertools.count()}


def _autoname(prefix):
    return f"{prefix}_{next(_counters[prefix])}"


def _reset_name_counters():
    for k in _counters:
        _counters[k] = itertools.count()


# ---------------------------------------------------------------- recorder
class _Pointer:
    __slots__ = "val"

    def __init__(self, val):
        self.val = val

    @property
    def _carg(self):
        return ctypes.byref(self.val._h)

    @property
    def name(self):
        return f"&{self.val.name}"


class _Cast:
    """`(GrB_Matrix)v` -- the same handle passed where another object type is expected."""

    __slots__ = "obj", "ctype"

    def __init__(self, obj, ctype):
        self.obj = obj
        self.ctype = ctype

    @property
    def _carg(self):
        return self.obj._carg

    @property
    def name(self):
        return f"({self.ctype}){self.obj.name}"


def gbstr(arg):
    if arg is None:
        return "NULL"
    if isinstance(arg, TypedOp):
        return arg.gb_name
    if isinstance(arg, Mask):
        return arg.parent.name
    if isinstance(arg, DataType):
        return arg.gb_name
    if isinstance(arg, Descriptor):
        return arg.name
    if isinstance(arg, bool):
        return "true" if arg else "false"
    if isinstance(arg, (int, float)):
        return repr(arg)
    name = getattr(arg, "name", None)
    if name is None:
        return repr(arg)
    return name


class Recorder:
    """Record every C call as C source text (reference core/recorder.py:34-178)."""

    def __init__(self, *, start=True, max_rows=20):
        self.data = []
        self._token = None
        self.max_rows = max_rows
        if start:
            self.start()

    def record(self, cfunc_name, args, *, exc=None):
        val = f'{cfunc_name}({", ".join(gbstr(x) for x in args)});'
        if exc is not None:
            val += f" /* ERROR: {type(exc).__name__} */"
        self.data.append(val)

    def start(self):
        if self._token is None:
            self._token = _recorder.set(self)

    def stop(self):
        if self._token is not None:
            _recorder.reset(self._token)
            self._token = None

    def clear(self):
        self.data.clear()

    def __enter__(self):
        self.start()
        return self

    def __exit__(self, *exc):
        self.stop()

    def __iter__(self):
        return iter(self.data)

    def __len__(self):
        return len(self.data)

    @property
    def is_recording(self):
        return self._token is not None and _recorder.get() is self

    def __repr__(self):
        lines = [f'gb.Recorder ({"" if self.is_recording else "not "}recording)']
        lines.append("-" * len(lines[0]))
        lines.extend(f"  {line}" for line in self.data)
        return "\n".join(lines)


def call(cfunc_name, args):
    """One C-ABI call (reference core/base.py:23-54)."""
    cargs = [getattr(x, "_carg", x) if x is not None else None for x in args]
    fn = getattr(lib, cfunc_name)
    rc = fn(*cargs)
    try:
        rv = check_status(rc, args)
    except Exception as exc:
        rec = _recorder.get()
        if rec is not None:
            rec.record(cfunc_name, args, exc=exc)
        raise
    rec = _recorder.get()
    if rec is not None:
        rec.record(cfunc_name, args)
    return rv


# ---------------------------------------------------------------- descriptors
class Descriptor:
    __slots__ = "gb_obj", "name", "key"

    def __init__(self, gb_obj, name, key):
        self.gb_obj = gb_obj
        self.name = name
        self.key = key

    @property
    def _carg(self):
        return self.gb_obj


_desc_map = {}
for _key, _name in _builtins.DESCRIPTORS.items():
    _desc_map[_key] = Descriptor(getattr(lib, _name), _name, _key)
_desc_map[(False, False, False, False, False)] = None


def descriptor_lookup(*, output_replace=False, mask_complement=False, mask_structure=False,
                      transpose_first=False, transpose_second=False, **opts):
    """5 flags -> predefined GrB_DESC_* (reference core/descriptor.py:51-156)."""
    if opts:
        raise ValueError(f"Extra descriptor options not supported; got {', '.join(map(str, opts))}")
    return _desc_map[(bool(output_replace), bool(mask_complement), bool(mask_structure),
                      bool(transpose_first), bool(transpose_second))]


# ---------------------------------------------------------------- masks
class Mask:
    complement = False
    structure = False
    __slots__ = "parent", "__weakref__"

    def __init__(self, mask):
        self.parent = mask

    @property
    def _carg(self):
        return self.parent._carg

    def __repr__(self):
        return f"{'~' if self.complement else ''}{self.parent.name}.{'S' if self.structure else 'V'}"

    @property
    def name(self):
        return self.parent.name

    def __eq__(self, other):
        raise TypeError(f"__eq__ not defined for objects of type {type(self)}.")

    def __bool__(self):
        raise TypeError(f"__bool__ not defined for objects of type {type(self)}.")

    __hash__ = object.__hash__

    # ---- mask algebra (reference core/mask.py:34-128).  The reference picks one of 16
    # recipes per (mask kind, mask kind) pair; each recipe computes the set its docstring
    # defines, and that definition is what is issued here -- masked assigns on the device:
    #   new(mask=m2)                 val(m1) << True; val(m2, replace=True) << val   (:51-56)
    #   new(mask=m2, complement=True) val(~m1) << True; val(~m2) << True             (:58-63)
    #   m1 & m2                      the set of new(mask=m2) as a structural mask    (:86-91)
    #   m1 | m2                      val(m1) << True; val(m2) << True; val.S          (:114-118)
    def new(self, dtype=None, *, complement=False, mask=None, name=None, **opts):
        if dtype is None:
            dtype = BOOL
        val = type(self.parent)(dtype, *self.parent.shape, name=name)
        if mask is None:
            val(~self if complement else self, **opts) << True
            return val
        mask = _check_mask(mask)
        if complement:
            val(~self, **opts) << True
            val(~mask, **opts) << True
        else:
            val(self, **opts) << True
            val(mask, replace=True, **opts) << val
        return val

    def __and__(self, other, **opts):
        other = _check_mask(other)
        complement = self.complement or other.complement
        val = self.new(BOOL, mask=other, complement=complement, **opts)
        # with a complemented operand the complement of the intersection is the smaller object
        return ComplementedStructuralMask(val) if complement else StructuralMask(val)

    __rand__ = __and__

    def __or__(self, other, **opts):
        other = _check_mask(other)
        val = type(self.parent)(BOOL, *self.parent.shape)
        val(self, **opts) << True
        val(other, **opts) << True
        return StructuralMask(val)

    __ror__ = __or__


class StructuralMask(Mask):
    complement, structure = False, True

    def __invert__(self):
        return ComplementedStructuralMask(self.parent)


class ValueMask(Mask):
    complement, structure = False, False

    def __invert__(self):
        return ComplementedValueMask(self.parent)


class ComplementedStructuralMask(Mask):
    complement, structure = True, True

    def __invert__(self):
        return StructuralMask(self.parent)


class ComplementedValueMask(Mask):
    complement, structure = True, False

    def __invert__(self):
        return ValueMask(self.parent)


def _check_mask(mask, output=None):
    """reference core/base.py:169-183"""
    if not isinstance(mask, Mask):
        if type(mask).__name__ in {"Vector", "Matrix"}:
            if mask.dtype != BOOL:
                raise TypeError(f"Mask must be boolean objects (got {mask.dtype}) "
                                "or indicate values (M.V) or structure (M.S)")
            mask = mask.V
        else:
            raise TypeError(f"Invalid mask: {type(mask)}")
    if output is not None and output.ndim == 1 and mask.parent.ndim != 1:
        raise TypeError(f"Mask object must be type Vector; got {type(mask.parent)}")
    return mask


class _ReplaceSentinel:
    def __repr__(self):
        return "replace"


replace = _ReplaceSentinel()
_REPLACE = replace  # BaseType.__call__'s `replace` parameter shadows the module name


def _normalize_accum(accum, dtype):
    if isinstance(accum, str):
        accum = _from_string(accum, "binary")
    accum = get_typed_op(accum, dtype, kind="binary")
    if accum.opclass == "Monoid":
        accum = getattr(binary, accum.parent.name if accum.parent.name != "eq" else "lxnor")[accum.type]
    elif accum.opclass != "BinaryOp":
        # reference core/base.py:256 -> _expect_op: "Expected type: BinaryOp, Monoid ..."
        raise TypeError(f"Expected type: BinaryOp, Monoid for accum; got {accum.opclass}")
    return accum


# ---------------------------------------------------------------- output binding
class Updater:
    """C(mask, accum, replace) -- holds the output parameters (reference core/expr.py:402-478)."""

    __slots__ = "parent", "mask", "accum", "replace", "opts"

    def __init__(self, parent, mask=None, accum=None, replace=False, opts=None):
        self.parent = parent
        self.mask = mask
        self.accum = accum
        self.replace = replace
        self.opts = opts or {}

    def __lshift__(self, expr):
        self.parent._update(expr, self.mask, self.accum, self.replace, opts=self.opts)

    def update(self, expr):
        self.parent._update(expr, self.mask, self.accum, self.replace, opts=self.opts)

    def __setitem__(self, keys, value):
        self.parent._assign(keys, value, self.mask, self.accum, self.replace)

    def __getitem__(self, keys):
        return _UpdaterItem(self, keys)


class _UpdaterItem:
    __slots__ = "updater", "keys"

    def __init__(self, updater, keys):
        self.updater = updater
        self.keys = keys

    def __lshift__(self, value):
        self.updater[self.keys] = value

    def update(self, value):
        self.updater[self.keys] = value


class BaseType:
    _is_scalar = False
    ndim = None

    @property
    def _carg(self):
        return self._h

    def __call__(self, *optional_mask_accum_replace, mask=None, accum=None, replace=False, **opts):
        """reference core/base.py:192-263"""
        mask_arg = accum_arg = None
        for arg in optional_mask_accum_replace:
            if arg is _REPLACE:
                replace = True
            elif isinstance(arg, (BaseType, Mask)):
                if self._is_scalar:
                    raise TypeError("Mask not allowed for Scalars")
                if mask_arg is not None:
                    raise TypeError("Got multiple values for argument 'mask'")
                mask_arg = arg
            elif isinstance(arg, (TypedOp, OpBase, str)):
                if accum_arg is not None:
                    raise TypeError("Got multiple values for argument 'accum'")
                accum_arg = arg
            else:
                raise TypeError(f"Invalid item found in output params: {type(arg)}")
        if mask_arg is not None and mask is not None:
            raise TypeError("Got multiple values for argument 'mask'")
        if mask_arg is not None:
            mask = mask_arg
        if mask is None:
            if replace:
                raise TypeError("'replace' argument may only be True if a mask is provided")
        elif self._is_scalar:
            raise TypeError("Mask not allowed for Scalars")
        else:
            mask = _check_mask(mask)
        if accum_arg is not None:
            if accum is not None:
                raise TypeError("Got multiple values for argument 'accum'")
            accum = accum_arg
        if accum is not None:
            accum = _normalize_accum(accum, self.dtype)
        return Updater(self, mask=mask, accum=accum, replace=replace, opts=opts)

    def __lshift__(self, expr):
        return self._update(expr, opts={})

    def update(self, expr, **opts):
        return self._update(expr, opts=opts)

    def __matmul__(self, other):
        from .infix import _matmul_infix_expr

        return _matmul_infix_expr(self, other)

    def __rmatmul__(self, other):
        from .infix import _matmul_infix_expr

        return _matmul_infix_expr(other, self)

    def __and__(self, other):
        from .infix import _ewise_infix_expr

        return _ewise_infix_expr(self, other, "ewise_mult")

    def __or__(self, other):
        from .infix import _ewise_infix_expr

        return _ewise_infix_expr(self, other, "ewise_add")

    def __imatmul__(self, other):
        self << self @ other
        return self

    def __bool__(self):
        raise TypeError(f"__bool__ not defined for objects of type {type(self)}.  "
                        "Perhaps use .nvals attribute instead.")

    def _update(self, expr, mask=None, accum=None, replace=False, *, opts):
        """reference core/base.py:318-495"""
        from .infix import InfixExpr

        if isinstance(expr, InfixExpr):
            expr = expr._to_expr()
        if not isinstance(expr, BaseExpression):
            if type(expr) is type(self) and not self._is_scalar:
                # w << v : assign over everything
                self._assign(Ellipsis, expr, mask, accum, replace)
                return
            if type(expr).__name__ == "TransposedMatrix" and type(self).__name__ == "Matrix":
                from .matrix import MatrixExpression

                expr = MatrixExpression("transpose", "GrB_transpose", [expr._matrix], at=True,
                                        dtype=expr.dtype, nrows=expr.nrows, ncols=expr.ncols)
            elif self._is_scalar:
                if accum is not None:
                    from .scalar import Scalar

                    other = expr if isinstance(expr, Scalar) else Scalar.from_value(expr, self.dtype)
                    cur = self.value
                    if cur is None:
                        self.value = other.value
                    else:
                        self.value = _apply_binop_host(accum, cur, other.value)
                    return
                self.value = expr
                return
            else:
                self._assign(Ellipsis, expr, mask, accum, replace)
                return
        if expr.output_type is not type(self):
            if expr.output_type.__name__ == "Scalar" and not self._is_scalar:
                # autocompute a scalar result then assign it everywhere
                s = expr.new()
                self._assign(Ellipsis, s, mask, accum, replace)
                return
            if not (self._is_scalar and expr.output_type.__name__ == "Scalar"):
                raise TypeError(f"Bad type for update: {type(self).__name__} << "
                                f"{expr.output_type.__name__}Expression")
        if expr.cfunc_name is None:  # custom recipe
            expr.args[-2](self(mask=mask, accum=accum, replace=replace), *expr.args[-1])
            return
        if mask is None:
            complement = structure = False
        else:
            mask = _check_mask(mask, self)
            complement, structure = mask.complement, mask.structure
        desc = descriptor_lookup(transpose_first=expr.at, transpose_second=expr.bt,
                                 mask_complement=complement, mask_structure=structure,
                                 output_replace=replace, **opts)
        if self._is_scalar and not getattr(expr, "_scalar_as_vector", False):
            args = [self, accum]  # GrB_*_reduce_Monoid_Scalar(s, accum, monoid, A, desc)
        else:
            out = self
            if self._is_scalar:
                out = _Cast(self, "GrB_Vector")
            args = [out, mask, accum]
        if expr.op is not None:
            args.append(expr.op)
        args.extend(expr.args)
        args.append(desc)
        call(expr.cfunc_name, args)


def _apply_binop_host(accum, x, y):
    import numpy as np

    name = accum.parent.name
    fns = {"plus": np.add, "minus": np.subtract, "times": np.multiply, "min": np.minimum,
           "max": np.maximum, "first": lambda a, b: a, "second": lambda a, b: b,
           "lor": np.logical_or, "land": np.logical_and}
    return fns[name](np.asarray(x, accum.type.np_type), np.asarray(y, accum.type.np_type)).item()


class BaseExpression:
    """A delayed operation: no compute until bound to an output (reference core/base.py:498-596)."""

    output_type = None
    _is_scalar = False

    def __init__(self, method_name, cfunc_name, args, *, at=False, bt=False, op=None, dtype=None,
                 expr_repr=None):
        self.method_name = method_name
        self.cfunc_name = cfunc_name
        self.args = args
        self.at = at
        self.bt = bt
        self.op = op
        self.dtype = op.return_type if dtype is None else dtype
        self.expr_repr = expr_repr

    def new(self, dtype=None, *, mask=None, name=None, **opts):
        output = self.construct_output(dtype, name=name)
        if mask is None:
            output.update(self, **opts)
        else:
            mask = _check_mask(mask, output)
            output(mask=mask, **opts).update(self)
        return output

    def _new_scalar(self):
        return self.new()
