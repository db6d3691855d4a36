// gb_dispatch.cuh -- map a (semiring, input type, output type) triple to a
// kernel instantiation: compile-time semirings for the configured hot paths,
// the runtime-op semiring for every other builtin.
#pragma once
#include "gb_device.cuh"
#include "gb_internal.h"

template <class F>
static void gb_with_type(int code, F &&f) {
    switch (code) {
    case GBAMD_T_BOOL: f((bool)0); break;
    case GBAMD_T_INT8: f((int8_t)0); break;
    case GBAMD_T_UINT8: f((uint8_t)0); break;
    case GBAMD_T_INT16: f((int16_t)0); break;
    case GBAMD_T_UINT16: f((uint16_t)0); break;
    case GBAMD_T_INT32: f((int32_t)0); break;
    case GBAMD_T_UINT32: f((uint32_t)0); break;
    case GBAMD_T_INT64: f((int64_t)0); break;
    case GBAMD_T_UINT64: f((uint64_t)0); break;
    case GBAMD_T_FP32: f((float)0); break;
    default: f((double)0); break;
    }
}

struct gb_sr_info {
    int mon, mul;
    int xcode;        // multiplier input type (== zcode for positional ops)
    int zcode;        // monoid / output type
    bool positional;
    bool reads_values;
};

inline gb_sr_info gb_sr_describe(GrB_Semiring sr) {
    gb_sr_info s;
    s.mon = sr->add->mcode;
    s.mul = sr->mul->opcode;
    s.zcode = sr->add->type->code;
    s.positional = sr->mul->xtype == nullptr;
    s.xcode = s.positional ? s.zcode : sr->mul->xtype->code;
    s.reads_values = !(s.positional || s.mul == GBAMD_OP_PAIR);
    return s;
}

// f(sr_functor, X{}, Z{})
template <class F>
static void gb_dispatch_sr(const gb_sr_info &s, F &&f) {
    // ---- compile-time fast paths (benchmarked configurations)
    if (s.mon == GBAMD_MON_PLUS && s.mul == GBAMD_OP_TIMES && s.xcode == s.zcode) {
        switch (s.zcode) {
        case GBAMD_T_FP64: f(gb_sr_plus_times<double>{}, double{}, double{}); return;
        case GBAMD_T_FP32: f(gb_sr_plus_times<float>{}, float{}, float{}); return;
        case GBAMD_T_INT64: f(gb_sr_plus_times<int64_t>{}, int64_t{}, int64_t{}); return;
        default: break;
        }
    }
    if (s.mon == GBAMD_MON_MIN && s.mul == GBAMD_OP_PLUS && s.xcode == s.zcode) {
        switch (s.zcode) {
        case GBAMD_T_INT64: f(gb_sr_min_plus<int64_t>{}, int64_t{}, int64_t{}); return;
        case GBAMD_T_INT32: f(gb_sr_min_plus<int32_t>{}, int32_t{}, int32_t{}); return;
        case GBAMD_T_FP64: f(gb_sr_min_plus<double>{}, double{}, double{}); return;
        default: break;
        }
    }
    if (s.mul == GBAMD_OP_PAIR && (s.mon == GBAMD_MON_ANY || s.mon == GBAMD_MON_LOR)) {
        switch (s.zcode) {
        case GBAMD_T_BOOL: f(gb_sr_any_pair<bool>{}, bool{}, bool{}); return;
        case GBAMD_T_INT64: f(gb_sr_any_pair<int64_t>{}, int64_t{}, int64_t{}); return;
        case GBAMD_T_INT32: f(gb_sr_any_pair<int32_t>{}, int32_t{}, int32_t{}); return;
        default: break;
        }
    }
    if (s.mon == GBAMD_MON_LOR && s.mul == GBAMD_OP_LAND && s.xcode == GBAMD_T_BOOL && s.zcode == GBAMD_T_BOOL) {
        f(gb_sr_lor_land{}, bool{}, bool{});
        return;
    }
    // ---- generic: runtime operator codes, typed loads/stores
    if (s.zcode == s.xcode) {
        gb_with_type(s.zcode, [&](auto z) {
            using T = decltype(z);
            f(gb_sr_dyn<T, T>{s.mon, s.mul}, T{}, T{});
        });
        return;
    }
    if (s.zcode == GBAMD_T_BOOL) {
        gb_with_type(s.xcode, [&](auto x) {
            using X = decltype(x);
            f(gb_sr_dyn<X, bool>{s.mon, s.mul}, X{}, bool{});
        });
        return;
    }
    gb_throw(GrB_NOT_IMPLEMENTED, "semiring type combination not supported");
}
