// gb_device.cuh -- device-side value semantics for the GraphBLAS builtins.
//
// Typecasts, binary operators and monoids evaluated on gfx950.  The semantics
// are the GraphBLAS C API 2.0 ones with SuiteSparse:GraphBLAS 7.4.x's builtin
// definitions (integer ops wrap; x/0 saturates; float->int casts saturate and
// map NaN to 0; bool PLUS/TIMES/MIN/MAX/MINUS are LOR/LAND/LAND/LOR/LXOR).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <type_traits>

#include "../../include/gbamd_codes.h"
#include "gb_state.h"

#define GB_DEV __device__ __forceinline__
#define GB_HD __host__ __device__ __forceinline__

template <class T>
struct gb_traits {
    static constexpr bool is_bool = std::is_same<T, bool>::value;
    static constexpr bool is_float = std::is_floating_point<T>::value;
    static constexpr bool is_signed = std::is_signed<T>::value && !is_float;
    static constexpr bool is_int = std::is_integral<T>::value && !is_bool;
};

template <class T>
GB_HD T gb_tmax() {
    if constexpr (std::is_same<T, bool>::value) return true;
    else if constexpr (std::is_same<T, float>::value) return __builtin_inff();
    else if constexpr (std::is_same<T, double>::value) return __builtin_inf();
    else if constexpr (std::is_signed<T>::value) {
        using U = typename std::make_unsigned<T>::type;
        return (T)(U)((U)~U(0) >> 1);  // cast before the shift: narrow types promote to int
    }
    else return (T)~(T)0;
}
template <class T>
GB_HD T gb_tmin() {
    if constexpr (std::is_same<T, bool>::value) return false;
    else if constexpr (std::is_same<T, float>::value) return -__builtin_inff();
    else if constexpr (std::is_same<T, double>::value) return -__builtin_inf();
    else if constexpr (std::is_signed<T>::value) return (T)(-gb_tmax<T>() - 1);
    else return (T)0;
}

// ------------------------------------------------------------------ casts
template <class D, class S>
GB_HD D gb_cast(S x) {
    if constexpr (std::is_same<D, S>::value) {
        return x;
    } else if constexpr (std::is_same<D, bool>::value) {
        return x != (S)0;
    } else if constexpr (std::is_floating_point<S>::value && std::is_integral<D>::value) {
        // SuiteSparse GB_cast_to_int*: NaN -> 0, saturate, else truncate
        if (x != x) return (D)0;
        if (x <= (S)gb_tmin<D>()) return gb_tmin<D>();
        if (x >= (S)gb_tmax<D>()) return gb_tmax<D>();
        return (D)x;
    } else if constexpr (std::is_same<S, bool>::value) {
        return (D)(x ? 1 : 0);
    } else if constexpr (std::is_integral<S>::value && std::is_integral<D>::value) {
        // C's integer conversion: the value modulo 2^bits(D) (signed sources sign-extend when
        // widening -- converting to S's unsigned type first would zero-extend: int32 -5 -> int64
        // 4294967291)
        using UD = typename std::make_unsigned<D>::type;
        return (D)(UD)x;
    } else {
        return (D)x;
    }
}

// ------------------------------------------------------------------ ops
GB_HD bool gb_op_is_positional(int op) { return op >= GBAMD_OP_FIRSTI; }
GB_HD bool gb_op_is_cmp(int op) { return op >= GBAMD_OP_EQ && op <= GBAMD_OP_LE; }

GB_HD int gb_bool_rename(int op) {
    switch (op) {
    case GBAMD_OP_PLUS: case GBAMD_OP_MAX: return GBAMD_OP_LOR;
    case GBAMD_OP_TIMES: case GBAMD_OP_MIN: return GBAMD_OP_LAND;
    case GBAMD_OP_MINUS: case GBAMD_OP_RMINUS: case GBAMD_OP_ISNE: case GBAMD_OP_NE: return GBAMD_OP_LXOR;
    case GBAMD_OP_DIV: return GBAMD_OP_FIRST;
    case GBAMD_OP_RDIV: return GBAMD_OP_SECOND;
    case GBAMD_OP_ISEQ: case GBAMD_OP_EQ: return GBAMD_OP_LXNOR;
    case GBAMD_OP_ISGT: return GBAMD_OP_GT;
    case GBAMD_OP_ISLT: return GBAMD_OP_LT;
    case GBAMD_OP_ISGE: return GBAMD_OP_GE;
    case GBAMD_OP_ISLE: return GBAMD_OP_LE;
    default: return op;
    }
}

template <class T>
GB_HD T gb_idiv(T x, T y) {
    if constexpr (std::is_signed<T>::value) {
        if (y == (T)-1) return (T)((typename std::make_unsigned<T>::type)0 - (typename std::make_unsigned<T>::type)x);
        if (y == 0) return x == 0 ? (T)0 : (x < 0 ? gb_tmin<T>() : gb_tmax<T>());
        return (T)(x / y);
    } else {
        if (y == 0) return x == 0 ? (T)0 : gb_tmax<T>();
        return (T)(x / y);
    }
}

template <class T>
GB_HD bool gb_cmp(int op, T x, T y) {
    switch (op) {
    case GBAMD_OP_EQ: return x == y;
    case GBAMD_OP_NE: return x != y;
    case GBAMD_OP_GT: return x > y;
    case GBAMD_OP_LT: return x < y;
    case GBAMD_OP_GE: return x >= y;
    case GBAMD_OP_LE: return x <= y;
    default: return false;
    }
}

template <class T>
GB_HD T gb_wrap_add(T x, T y) {
    if constexpr (gb_traits<T>::is_int) {
        using U = typename std::make_unsigned<T>::type;
        return (T)(U)((U)x + (U)y);
    } else return x + y;
}
template <class T>
GB_HD T gb_wrap_sub(T x, T y) {
    if constexpr (gb_traits<T>::is_int) {
        using U = typename std::make_unsigned<T>::type;
        return (T)(U)((U)x - (U)y);
    } else return x - y;
}
template <class T>
GB_HD T gb_wrap_mul(T x, T y) {
    if constexpr (gb_traits<T>::is_int) {
        using U = typename std::make_unsigned<T>::type;
        // promote narrow unsigned to 64-bit to avoid int promotion UB
        return (T)(U)((uint64_t)(U)x * (uint64_t)(U)y);
    } else return x * y;
}
template <class T>
GB_HD T gb_min(T x, T y) {
    if constexpr (std::is_floating_point<T>::value) return fmin(x, y);
    else return x < y ? x : y;
}
template <class T>
GB_HD T gb_max(T x, T y) {
    if constexpr (std::is_floating_point<T>::value) return fmax(x, y);
    else return x > y ? x : y;
}

// z = op(x, y), x, y, z all of type T (non-positional, non-comparison ops;
// comparison ops return 1/0 of type T here, which callers cast).
template <class T>
GB_HD T gb_binop(int op, T x, T y) {
    if constexpr (std::is_same<T, bool>::value) {
        op = gb_bool_rename(op);
        switch (op) {
        case GBAMD_OP_FIRST: return x;
        case GBAMD_OP_SECOND: case GBAMD_OP_ANY: return y;
        case GBAMD_OP_PAIR: return true;
        case GBAMD_OP_LOR: return x || y;
        case GBAMD_OP_LAND: return x && y;
        case GBAMD_OP_LXOR: return x != y;
        case GBAMD_OP_LXNOR: return x == y;
        case GBAMD_OP_GT: return x && !y;
        case GBAMD_OP_LT: return !x && y;
        case GBAMD_OP_GE: return x || !y;
        case GBAMD_OP_LE: return !x || y;
        case GBAMD_OP_POW: return x || !y;
        case GBAMD_OP_BOR: return x || y;
        case GBAMD_OP_BAND: return x && y;
        case GBAMD_OP_BXOR: return x != y;
        case GBAMD_OP_BXNOR: return x == y;
        default: return false;
        }
    } else {
        const T one = (T)1, zero = (T)0;
        switch (op) {
        case GBAMD_OP_FIRST: return x;
        case GBAMD_OP_SECOND: case GBAMD_OP_ANY: return y;
        case GBAMD_OP_PAIR: return one;
        case GBAMD_OP_MIN: return gb_min(x, y);
        case GBAMD_OP_MAX: return gb_max(x, y);
        case GBAMD_OP_PLUS: return gb_wrap_add(x, y);
        case GBAMD_OP_MINUS: return gb_wrap_sub(x, y);
        case GBAMD_OP_RMINUS: return gb_wrap_sub(y, x);
        case GBAMD_OP_TIMES: return gb_wrap_mul(x, y);
        case GBAMD_OP_DIV:
            if constexpr (gb_traits<T>::is_int) return gb_idiv(x, y);
            else return x / y;
        case GBAMD_OP_RDIV:
            if constexpr (gb_traits<T>::is_int) return gb_idiv(y, x);
            else return y / x;
        case GBAMD_OP_POW:
            if constexpr (std::is_same<T, float>::value) return powf(x, y);
            else if constexpr (std::is_same<T, double>::value) return pow(x, y);
            else return gb_cast<T, double>(pow((double)x, (double)y));
        case GBAMD_OP_ISEQ: return x == y ? one : zero;
        case GBAMD_OP_ISNE: return x != y ? one : zero;
        case GBAMD_OP_ISGT: return x > y ? one : zero;
        case GBAMD_OP_ISLT: return x < y ? one : zero;
        case GBAMD_OP_ISGE: return x >= y ? one : zero;
        case GBAMD_OP_ISLE: return x <= y ? one : zero;
        case GBAMD_OP_LOR: return (x != zero || y != zero) ? one : zero;
        case GBAMD_OP_LAND: return (x != zero && y != zero) ? one : zero;
        case GBAMD_OP_LXOR: return ((x != zero) != (y != zero)) ? one : zero;
        case GBAMD_OP_LXNOR: return ((x != zero) == (y != zero)) ? one : zero;
        case GBAMD_OP_EQ: return x == y ? one : zero;
        case GBAMD_OP_NE: return x != y ? one : zero;
        case GBAMD_OP_GT: return x > y ? one : zero;
        case GBAMD_OP_LT: return x < y ? one : zero;
        case GBAMD_OP_GE: return x >= y ? one : zero;
        case GBAMD_OP_LE: return x <= y ? one : zero;
        default: break;
        }
        if constexpr (gb_traits<T>::is_int) {
            using U = typename std::make_unsigned<T>::type;
            switch (op) {
            case GBAMD_OP_BOR: return (T)((U)x | (U)y);
            case GBAMD_OP_BAND: return (T)((U)x & (U)y);
            case GBAMD_OP_BXOR: return (T)((U)x ^ (U)y);
            case GBAMD_OP_BXNOR: return (T)(U)~((U)x ^ (U)y);
            default: break;
            }
        } else {
            switch (op) {
            case GBAMD_OP_ATAN2: return (T)atan2((double)x, (double)y);
            case GBAMD_OP_HYPOT: return (T)hypot((double)x, (double)y);
            case GBAMD_OP_FMOD: return (T)fmod((double)x, (double)y);
            case GBAMD_OP_REMAINDER: return (T)remainder((double)x, (double)y);
            case GBAMD_OP_LDEXP: return (T)ldexp((double)x, (int)y);
            case GBAMD_OP_COPYSIGN: return (T)copysign((double)x, (double)y);
            default: break;
            }
        }
        return zero;
    }
}

// z = op(x) for the builtin unary operators (x, z of type T)
template <class T>
GB_HD T gb_unop(int op, T x) {
    if constexpr (std::is_same<T, bool>::value) {
        switch (op) {
        case GBAMD_UOP_LNOT: case GBAMD_UOP_BNOT: return !x;
        case GBAMD_UOP_ONE: return true;
        case GBAMD_UOP_MINV: return true;  // SuiteSparse: MINV_BOOL(x) = true
        default: return x;                 // IDENTITY, AINV, ABS
        }
    } else {
        switch (op) {
        case GBAMD_UOP_IDENTITY: return x;
        case GBAMD_UOP_AINV: return gb_wrap_sub((T)0, x);
        case GBAMD_UOP_MINV:
            if constexpr (gb_traits<T>::is_int) return gb_idiv((T)1, x);
            else return (T)1 / x;
        case GBAMD_UOP_ABS:
            if constexpr (std::is_unsigned<T>::value) return x;
            else if constexpr (std::is_floating_point<T>::value) return (T)fabs(x);
            else return x < 0 ? gb_wrap_sub((T)0, x) : x;
        case GBAMD_UOP_LNOT: return x == (T)0 ? (T)1 : (T)0;
        case GBAMD_UOP_ONE: return (T)1;
        default: break;
        }
        if constexpr (gb_traits<T>::is_int) {
            using U = typename std::make_unsigned<T>::type;
            if (op == GBAMD_UOP_BNOT) return (T)(U)~(U)x;
            return x;
        } else {
            switch (op) {
            case GBAMD_UOP_SQRT: return (T)sqrt((double)x);
            case GBAMD_UOP_LOG: return (T)log((double)x);
            case GBAMD_UOP_LOG2: return (T)log2((double)x);
            case GBAMD_UOP_LOG10: return (T)log10((double)x);
            case GBAMD_UOP_EXP: return (T)exp((double)x);
            case GBAMD_UOP_EXP2: return (T)exp2((double)x);
            case GBAMD_UOP_FLOOR: return (T)floor((double)x);
            case GBAMD_UOP_CEIL: return (T)ceil((double)x);
            case GBAMD_UOP_ROUND: return (T)round((double)x);
            case GBAMD_UOP_TRUNC: return (T)trunc((double)x);
            case GBAMD_UOP_SIN: return (T)sin((double)x);
            case GBAMD_UOP_COS: return (T)cos((double)x);
            case GBAMD_UOP_TAN: return (T)tan((double)x);
            default: return x;
            }
        }
    }
}

GB_HD int64_t gb_posop(int op, int64_t i, int64_t k, int64_t j) {
    switch (op) {
    case GBAMD_OP_FIRSTI: return i;
    case GBAMD_OP_FIRSTI1: return i + 1;
    case GBAMD_OP_FIRSTJ: return k;
    case GBAMD_OP_FIRSTJ1: return k + 1;
    case GBAMD_OP_SECONDI: return k;
    case GBAMD_OP_SECONDI1: return k + 1;
    case GBAMD_OP_SECONDJ: return j;
    case GBAMD_OP_SECONDJ1: return j + 1;
    default: return 0;
    }
}

// general binary op with output type Z (comparison ops produce bool)
template <class X, class Z>
GB_HD Z gb_binop_z(int op, X x, X y, int64_t i, int64_t k, int64_t j) {
    if (gb_op_is_positional(op)) return gb_cast<Z, int64_t>(gb_posop(op, i, k, j));
    if (gb_op_is_cmp(op)) {
        if constexpr (std::is_same<X, bool>::value) return gb_cast<Z, bool>(gb_binop<bool>(op, x, y));
        else return gb_cast<Z, bool>(gb_cmp<X>(op, x, y));
    }
    return gb_cast<Z, X>(gb_binop<X>(op, x, y));
}

// ------------------------------------------------------------------ monoids
template <class T>
GB_HD T gb_monoid(int m, T x, T y) {
    switch (m) {
    case GBAMD_MON_PLUS: return gb_binop<T>(GBAMD_OP_PLUS, x, y);
    case GBAMD_MON_TIMES: return gb_binop<T>(GBAMD_OP_TIMES, x, y);
    case GBAMD_MON_MIN: return gb_binop<T>(GBAMD_OP_MIN, x, y);
    case GBAMD_MON_MAX: return gb_binop<T>(GBAMD_OP_MAX, x, y);
    case GBAMD_MON_ANY: return x;
    case GBAMD_MON_LOR: return gb_binop<T>(GBAMD_OP_LOR, x, y);
    case GBAMD_MON_LAND: return gb_binop<T>(GBAMD_OP_LAND, x, y);
    case GBAMD_MON_LXOR: return gb_binop<T>(GBAMD_OP_LXOR, x, y);
    case GBAMD_MON_LXNOR: return gb_binop<T>(GBAMD_OP_LXNOR, x, y);
    case GBAMD_MON_BOR: return gb_binop<T>(GBAMD_OP_BOR, x, y);
    case GBAMD_MON_BAND: return gb_binop<T>(GBAMD_OP_BAND, x, y);
    case GBAMD_MON_BXOR: return gb_binop<T>(GBAMD_OP_BXOR, x, y);
    case GBAMD_MON_BXNOR: return gb_binop<T>(GBAMD_OP_BXNOR, x, y);
    default: return x;
    }
}

// identity of a monoid on T (ANY has none: callers store its first value instead)
template <class T>
GB_HD T gb_monoid_identity(int m) {
    switch (m) {
    case GBAMD_MON_TIMES: return (T)1;
    case GBAMD_MON_MIN: return gb_tmax<T>();
    case GBAMD_MON_MAX: return gb_tmin<T>();
    case GBAMD_MON_LAND: return (T)1;
    case GBAMD_MON_LXNOR: return (T)1;
    case GBAMD_MON_BAND:
    case GBAMD_MON_BXNOR:
        if constexpr (gb_traits<T>::is_int) return (T)~(T)0;
        else return (T)1;
    default: return (T)0;  // PLUS, LOR, LXOR, BOR, BXOR
    }
}

// terminal value of a monoid: once reached, further terms cannot change it
template <class T>
GB_HD bool gb_monoid_terminal(int m, T z) {
    switch (m) {
    case GBAMD_MON_ANY: return true;
    case GBAMD_MON_LOR: return z != (T)0;
    case GBAMD_MON_LAND: return z == (T)0;
    case GBAMD_MON_MIN:
        if constexpr (std::is_floating_point<T>::value) return false;  // NaN-ignoring fmin
        else return z == gb_tmin<T>();
    case GBAMD_MON_MAX:
        if constexpr (std::is_floating_point<T>::value) return false;
        else return z == gb_tmax<T>();
    case GBAMD_MON_TIMES:
        if constexpr (gb_traits<T>::is_int) return z == (T)0;
        else return false;
    case GBAMD_MON_BOR:
        if constexpr (gb_traits<T>::is_int) return z == (T)~(T)0;
        else return false;
    case GBAMD_MON_BAND:
        if constexpr (gb_traits<T>::is_int) return z == (T)0;
        else return false;
    default: return false;
    }
}

// ------------------------------------------------------------------ semirings
// Runtime-op semiring (generic path): every builtin (monoid, multiply) pair.
template <class X, class Z>
struct gb_sr_dyn {
    int mon, mul;
    GB_DEV Z mult(X a, X b, int64_t i, int64_t k, int64_t j) const {
        return gb_binop_z<X, Z>(mul, a, b, i, k, j);
    }
    GB_DEV Z add(Z x, Z y) const { return gb_monoid<Z>(mon, x, y); }
    GB_DEV bool terminal(Z z) const { return gb_monoid_terminal<Z>(mon, z); }
    static constexpr bool reads_values = true;
};

// Compile-time semirings for the configured hot paths.
template <class T>
struct gb_sr_plus_times {
    GB_DEV T mult(T a, T b, int64_t, int64_t, int64_t) const { return gb_wrap_mul(a, b); }
    GB_DEV T add(T x, T y) const { return gb_wrap_add(x, y); }
    GB_DEV bool terminal(T) const { return false; }
    static constexpr bool reads_values = true;
};
template <class T>
struct gb_sr_min_plus {
    GB_DEV T mult(T a, T b, int64_t, int64_t, int64_t) const { return gb_wrap_add(a, b); }
    GB_DEV T add(T x, T y) const { return gb_min(x, y); }
    GB_DEV bool terminal(T z) const {
        if constexpr (std::is_floating_point<T>::value) return false;
        else return z == gb_tmin<T>();
    }
    static constexpr bool reads_values = true;
};
template <class T>
struct gb_sr_any_pair {
    GB_DEV T mult(T, T, int64_t, int64_t, int64_t) const { return (T)1; }
    GB_DEV T add(T x, T) const { return x; }
    GB_DEV bool terminal(T) const { return true; }
    static constexpr bool reads_values = false;
};
struct gb_sr_lor_land {
    GB_DEV bool mult(bool a, bool b, int64_t, int64_t, int64_t) const { return a && b; }
    GB_DEV bool add(bool x, bool y) const { return x || y; }
    GB_DEV bool terminal(bool z) const { return z; }
    static constexpr bool reads_values = true;
};

// ------------------------------------------------------------------ wave helpers
GB_DEV int gb_lane() { return __lane_id(); }

// LDS written by some lanes of a wave, read by others: order the wave's accesses
GB_DEV void gb_wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <class T>
GB_DEV T gb_shfl_xor(T v, int mask, int width) {
    if constexpr (sizeof(T) == 8) {
        int64_t x;
        __builtin_memcpy(&x, &v, 8);
        int lo = __shfl_xor((int)(x & 0xffffffff), mask, width);
        int hi = __shfl_xor((int)(x >> 32), mask, width);
        int64_t y = ((int64_t)(uint32_t)lo) | ((int64_t)hi << 32);
        T r;
        __builtin_memcpy(&r, &y, 8);
        return r;
    } else if constexpr (sizeof(T) == 4) {
        int x;
        __builtin_memcpy(&x, &v, 4);
        x = __shfl_xor(x, mask, width);
        T r;
        __builtin_memcpy(&r, &x, 4);
        return r;
    } else {
        int x = 0;
        __builtin_memcpy(&x, &v, sizeof(T));
        x = __shfl_xor(x, mask, width);
        T r;
        __builtin_memcpy(&r, &x, sizeof(T));
        return r;
    }
}

// read v from lane src (any lane pattern: ds_bpermute), any type up to 8 bytes
template <class T>
GB_DEV T gb_shfl(T v, int src, int width = 64) {
    if constexpr (sizeof(T) == 8) {
        int64_t x;
        __builtin_memcpy(&x, &v, 8);
        int lo = __shfl((int)(x & 0xffffffff), src, width);
        int hi = __shfl((int)(x >> 32), src, width);
        int64_t y = ((int64_t)(uint32_t)lo) | ((int64_t)hi << 32);
        T r;
        __builtin_memcpy(&r, &y, 8);
        return r;
    } else {
        int x = 0;
        __builtin_memcpy(&x, &v, sizeof(T));
        x = __shfl(x, src, width);
        T r;
        __builtin_memcpy(&r, &x, sizeof(T));
        return r;
    }
}

template <class T>
GB_DEV T gb_shfl_up(T v, int delta, int width) {
    if constexpr (sizeof(T) == 8) {
        int64_t x;
        __builtin_memcpy(&x, &v, 8);
        int lo = __shfl_up((int)(x & 0xffffffff), delta, width);
        int hi = __shfl_up((int)(x >> 32), delta, width);
        int64_t y = ((int64_t)(uint32_t)lo) | ((int64_t)hi << 32);
        T r;
        __builtin_memcpy(&r, &y, 8);
        return r;
    } else {
        int x = 0;
        __builtin_memcpy(&x, &v, sizeof(T));
        x = __shfl_up(x, delta, width);
        T r;
        __builtin_memcpy(&r, &x, sizeof(T));
        return r;
    }
}

template <class T>
GB_DEV T gb_shfl_down(T v, int delta, int width) {
    if constexpr (sizeof(T) == 8) {
        int64_t x;
        __builtin_memcpy(&x, &v, 8);
        int lo = __shfl_down((int)(x & 0xffffffff), delta, width);
        int hi = __shfl_down((int)(x >> 32), delta, width);
        int64_t y = ((int64_t)(uint32_t)lo) | ((int64_t)hi << 32);
        T r;
        __builtin_memcpy(&r, &y, 8);
        return r;
    } else {
        int x = 0;
        __builtin_memcpy(&x, &v, sizeof(T));
        x = __shfl_down(x, delta, width);
        T r;
        __builtin_memcpy(&r, &x, sizeof(T));
        return r;
    }
}

GB_DEV bool gb_bit(const uint64_t *bits, int64_t i) { return (bits[i >> 6] >> (i & 63)) & 1ULL; }

// (bool) of one value of runtime type `code` (mask semantics: -0.0 is false, NaN true)
GB_DEV bool gb_dyn_nonzero(const void *p, int code) {
    switch (code) {
        case GBAMD_T_BOOL:
        case GBAMD_T_INT8:
        case GBAMD_T_UINT8: return *(const uint8_t *)p != 0;
        case GBAMD_T_INT16:
        case GBAMD_T_UINT16: return *(const uint16_t *)p != 0;
        case GBAMD_T_INT32:
        case GBAMD_T_UINT32: return *(const uint32_t *)p != 0;
        case GBAMD_T_INT64:
        case GBAMD_T_UINT64: return *(const uint64_t *)p != 0;
        case GBAMD_T_FP32: return *(const float *)p != 0.0f;
        case GBAMD_T_FP64: return *(const double *)p != 0.0;
        default: return true;
    }
}

// Add v (per thread) into *global with ONE atomic per block: wave shuffle
// reduction, then the block's waves through LDS.  Every thread of the block
// must call it (it contains a barrier).  Same-address atomics from every wave
// of a large grid serialise at the memory side (tens of microseconds per
// 10^4 adds), so counters are always reduced per block first.
// Sum over the block, result in thread 0.  All threads must call.
GB_DEV long long gb_block_sum(long long v) {
    __shared__ long long part[16];
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    const int wid = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
    if ((threadIdx.x & 63) == 0) part[wid] = v;
    __syncthreads();
    long long s = 0;
    if (threadIdx.x == 0)
        for (int w = 0; w < nw; w++) s += part[w];
    __syncthreads();
    return s;
}

// Grid-wide sum without a same-address pile-up.  Adds to one device-scope
// counter serialise at the memory side (about 12 ns each), so each block adds
// (sum << 20 | 1) to one of GB_GRID_SHARDS counters 256 B apart; the last
// arrival of a shard forwards the shard's sum to a root counter, and the last
// arrival there receives the grand total.  Every block of the grid must call it
// exactly once; it leaves the counters zeroed.  Returns true in thread 0 of
// exactly one block, with *total set.  Needs |sum| < 2^43, grid < 2^25 blocks.
GB_DEV bool gb_grid_sum(long long v, unsigned long long *st, long long *total) {
    v = gb_block_sum(v);
    if (threadIdx.x != 0) return false;
    const unsigned nb = gridDim.x;
    const unsigned s = blockIdx.x % GB_GRID_SHARDS;
    const unsigned in_shard = (nb - s + GB_GRID_SHARDS - 1) / GB_GRID_SHARDS;
    unsigned long long *cs = st + (size_t)s * GB_GRID_STRIDE;
    const long long old = (long long)atomicAdd(cs, ((unsigned long long)v << 20) + 1ULL);
    if ((unsigned)(old & 0xFFFFF) + 1 != in_shard) return false;
    atomicExch(cs, 0ULL);
    const long long shard_sum = (old >> 20) + v;
    const unsigned nshards = nb < GB_GRID_SHARDS ? nb : GB_GRID_SHARDS;
    unsigned long long *root = st + (size_t)GB_GRID_SHARDS * GB_GRID_STRIDE;
    const long long o2 = (long long)atomicAdd(root, ((unsigned long long)shard_sum << 20) + 1ULL);
    if ((unsigned)(o2 & 0xFFFFF) + 1 != nshards) return false;
    atomicExch(root, 0ULL);
    *total = (o2 >> 20) + shard_sum;
    return true;
}

// *global += grid-wide sum of v (one add on *global).  All threads of every block must call.
GB_DEV void gb_grid_add(long long v, unsigned long long *global, unsigned long long *st) {
    long long t;
    if (gb_grid_sum(v, st, &t) && t) atomicAdd(global, (unsigned long long)t);
}

GB_DEV void gb_block_add(unsigned long long v, unsigned long long *global) {
    __shared__ unsigned long long part[16];
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    const int wid = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
    if ((threadIdx.x & 63) == 0) part[wid] = v;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long s = 0;
        for (int w = 0; w < nw; w++) s += part[w];
        if (s) atomicAdd(global, s);
    }
    __syncthreads();
}
