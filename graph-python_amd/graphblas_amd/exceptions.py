"""GrB_Info -> exception mapping (mirrors reference graphblas/exceptions.py:8-155).

``GrB_NO_VALUE`` is returned (as the ``NoValue`` class), not raised; every other
negative code raises the class below with the text of ``GrB_<Type>_error`` on
the call's output object.
"""
import ctypes


class GraphblasException(Exception):
    pass


class NoValue(GraphblasException):
    pass


class UninitializedObject(GraphblasException):
    pass


class InvalidObject(GraphblasException):
    pass


class NullPointer(GraphblasException):
    pass


class InvalidValue(GraphblasException):
    pass


class InvalidIndex(GraphblasException):
    pass


class DomainMismatch(GraphblasException):
    pass


class DimensionMismatch(GraphblasException):
    pass


class OutputNotEmpty(GraphblasException):
    pass


class OutOfMemory(GraphblasException):
    pass


class InsufficientSpace(GraphblasException):
    pass


class IndexOutOfBound(GraphblasException):
    pass


class Panic(GraphblasException):
    pass


class EmptyObject(GraphblasException):
    pass


class NotImplementedException(GraphblasException):
    pass


_error_code_lookup = {
    1: NoValue,
    -1: UninitializedObject,
    -104: InvalidObject,
    -2: NullPointer,
    -3: InvalidValue,
    -4: InvalidIndex,
    -5: DomainMismatch,
    -6: DimensionMismatch,
    -7: OutputNotEmpty,
    -102: OutOfMemory,
    -103: InsufficientSpace,
    -105: IndexOutOfBound,
    -101: Panic,
    -106: EmptyObject,
    -8: NotImplementedException,
}


def check_status_carg(code, type_name, carg):
    if code == 0:
        return None
    if code == 1:
        return NoValue
    from ._lib import lib

    text = ""
    try:
        fn = getattr(lib, f"GrB_{type_name}_error")
        s = ctypes.c_char_p()
        fn(ctypes.byref(s), carg)
        text = (s.value or b"").decode()
    except AttributeError:
        pass
    raise _error_code_lookup.get(code, Panic)(text or f"GrB_Info {code}")


def check_status(code, args):
    if code == 0:
        return None
    if code == 1:
        return NoValue
    arg = args[0] if isinstance(args, list) else args
    arg = getattr(arg, "_exc_arg", arg)
    type_name = {"Matrix": "Matrix", "Vector": "Vector", "Scalar": "Scalar",
                 "TransposedMatrix": "Matrix"}.get(type(arg).__name__, "Matrix")
    return check_status_carg(code, type_name, getattr(arg, "_carg", None))
