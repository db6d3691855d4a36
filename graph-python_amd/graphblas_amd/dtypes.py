"""Builtin GraphBLAS data types bound to the library's ``GrB_<T>`` handles
(mirrors reference core/dtypes.py:16-73, 154-282, 352-394)."""
import numpy as np

from ._lib import lib


class DataType:
    __slots__ = "name", "gb_obj", "gb_name", "np_type", "c_type", "_is_udt"

    def __init__(self, name, np_type, c_type):
        self.name = name
        self.gb_name = f"GrB_{name}"
        self.gb_obj = getattr(lib, self.gb_name)
        self.np_type = np.dtype(np_type)
        self.c_type = c_type
        self._is_udt = False

    def __repr__(self):
        return self.name

    def __reduce__(self):
        return self.name

    def __eq__(self, other):
        if isinstance(other, DataType):
            return self is other
        try:
            return self is lookup_dtype(other)
        except (ValueError, TypeError):
            return False

    def __hash__(self):
        return hash(self.name)

    def __lt__(self, other):
        return self.name < other.name

    @property
    def _carg(self):
        return self.gb_obj


BOOL = DataType("BOOL", np.bool_, "bool")
INT8 = DataType("INT8", np.int8, "int8_t")
UINT8 = DataType("UINT8", np.uint8, "uint8_t")
INT16 = DataType("INT16", np.int16, "int16_t")
UINT16 = DataType("UINT16", np.uint16, "uint16_t")
INT32 = DataType("INT32", np.int32, "int32_t")
UINT32 = DataType("UINT32", np.uint32, "uint32_t")
INT64 = DataType("INT64", np.int64, "int64_t")
UINT64 = DataType("UINT64", np.uint64, "uint64_t")
FP32 = DataType("FP32", np.float32, "float")
FP64 = DataType("FP64", np.float64, "double")

_ALL = [BOOL, INT8, UINT8, INT16, UINT16, INT32, UINT32, INT64, UINT64, FP32, FP64]
_registry = {}
for _dt in _ALL:
    _registry[_dt.name] = _dt
    _registry[_dt.name.lower()] = _dt
    _registry[_dt.np_type] = _dt
    _registry[_dt.np_type.type] = _dt
    _registry[_dt.np_type.name] = _dt
    _registry[_dt.gb_name] = _dt
_registry[bool] = BOOL
_registry[int] = INT64
_registry[float] = FP64
_registry["bool"] = BOOL
_registry["int"] = INT64
_registry["float"] = FP64
_registry["double"] = FP64
_registry["float32"] = FP32
_registry["float64"] = FP64
_registry["FP32"] = FP32


def lookup_dtype(key):
    if isinstance(key, DataType):
        return key
    try:
        return _registry[key]
    except (KeyError, TypeError):
        pass
    try:
        return _registry[np.dtype(key)]
    except (KeyError, TypeError):
        pass
    raise ValueError(f"Unknown dtype: {key} of type {type(key)}")


def unify(type1, type2, *, is_left_scalar=False, is_right_scalar=False):
    """A type that can hold both (numpy promotion, reference core/dtypes.py:377-394)."""
    if type1 is type2:
        return type1
    if is_left_scalar:
        if not is_right_scalar:
            return lookup_dtype(np.result_type(np.array(0, type1.np_type), type2.np_type))
    elif is_right_scalar:
        return lookup_dtype(np.result_type(type1.np_type, np.array(0, type2.np_type)))
    return lookup_dtype(np.promote_types(type1.np_type, type2.np_type))


def from_values(values):
    a = np.asarray(values)
    if a.dtype == object:
        a = np.asarray(values.tolist() if hasattr(values, "tolist") else list(values))
    return lookup_dtype(a.dtype)
