// mx_dispatch.hpp -- the (op, type-slot) -> (element type, functor) map,
// shared by the op kernels (mx_reduce.hip) and the collective fold kernels
// (mx_coll.hip).  It restates the non-NULL pattern of the reference tables
// ompi_op_base_functions / ompi_op_base_3buff_functions
// (ompi/mca/op/base/op_base_functions.c:1485-1655): C integers x
// {MAX MIN SUM PROD LAND LOR LXOR BAND BOR BXOR}; Fortran integers x
// {MAX MIN SUM PROD BAND BOR BXOR}; float/double/long double (+ Fortran
// reals) x {MAX MIN SUM PROD}; LOGICAL and bool x {LAND LOR LXOR}; complex x
// {SUM PROD}; BYTE x {BAND BOR BXOR}; pair types x {MAXLOC MINLOC}.
//
// A visitor V provides `template <class T, class OP2, class OP3> R go()` and
// `R none()`; OP2 is the 2-buffer functor (x = target/out, y = source/in),
// OP3 the 3-buffer one (x = in1, y = in2).
#pragma once
#include "mx_ops.hpp"
#include "mx_x87.hpp"
#include "../../include/mx_kernels.h"

namespace mx {

using f32c = cplx<float>;
using f64c = cplx<double>;
using p_float_int = pair_t<float, int>;
using p_double_int = pair_t<double, int>;
using p_long_int = pair_t<long, int>;
using p_2int = pair_t<int, int>;
using p_short_int = pair_t<short, int>;
using p_2real = pair_t<float, float>;
using p_2double = pair_t<double, double>;

// Types whose storage has bytes outside the value fields: the struct pair
// types (gaps that MPI never transfers -- their datatypes have size <
// extent) and x87 long double (10 value bytes in 16).  Results are stored
// field by field so those bytes keep the destination's content, as the
// reference's field assignments (LOC_FUNC, op_base_functions.c:88-104) and
// gap-skipping copies (opal_datatype_copy.h) leave them.
template <class T> struct has_pad { static constexpr bool value = false; };
template <> struct has_pad<pair_t<short, int>> { static constexpr bool value = true; };
template <> struct has_pad<pair_t<double, int>> { static constexpr bool value = true; };
template <> struct has_pad<pair_t<long, int>> { static constexpr bool value = true; };
template <> struct has_pad<x87> { static constexpr bool value = true; };
template <> struct has_pad<x87c> { static constexpr bool value = true; };
template <> struct has_pad<x87_pair> { static constexpr bool value = true; };

template <class T> __device__ __forceinline__ void store_fields(T *p, const T &r) { *p = r; }
template <class V, class K> __device__ __forceinline__ void store_fields(pair_t<V, K> *p, const pair_t<V, K> &r) {
  p->v = r.v;
  p->k = r.k;
}
__device__ __forceinline__ void store_fields(x87 *p, const x87 &r) { p->m = r.m; p->se = r.se; }
__device__ __forceinline__ void store_fields(x87c *p, const x87c &r) {
  store_fields(&p->re, r.re);
  store_fields(&p->im, r.im);
}
__device__ __forceinline__ void store_fields(x87_pair *p, const x87_pair &r) {
  store_fields(&p->v, r.v);
  p->k = r.k;
}

static_assert(sizeof(p_float_int) == 8 && sizeof(p_double_int) == 16 && sizeof(p_long_int) == 16 &&
              sizeof(p_2int) == 8 && sizeof(p_short_int) == 8 && sizeof(p_2real) == 8 &&
              sizeof(p_2double) == 16 && sizeof(x87_pair) == 32 && sizeof(f32c) == 8 &&
              sizeof(f64c) == 16 && sizeof(x87) == 16 && sizeof(x87c) == 32,
              "pair/complex layouts must match the host ABI");

template <class T, class V> static auto d_int(int op, V &v) {
  switch (op) {
    case MX_OP_MAX: return v.template go<T, OpMax, OpMax>();
    case MX_OP_MIN: return v.template go<T, OpMin, OpMin>();
    case MX_OP_SUM: return v.template go<T, OpSum, OpSum>();
    case MX_OP_PROD: return v.template go<T, OpProd, OpProd>();
    case MX_OP_LAND: return v.template go<T, OpLand, OpLand>();
    case MX_OP_LOR: return v.template go<T, OpLor, OpLor>();
    case MX_OP_LXOR: return v.template go<T, OpLxor, OpLxor>();
    case MX_OP_BAND: return v.template go<T, OpBand, OpBand>();
    case MX_OP_BOR: return v.template go<T, OpBor, OpBor>();
    case MX_OP_BXOR: return v.template go<T, OpBxor, OpBxor>();
    default: return v.none();
  }
}
// Fortran integers: no logical ops
template <class T, class V> static auto d_fint(int op, V &v) {
  if (op == MX_OP_LAND || op == MX_OP_LOR || op == MX_OP_LXOR) return v.none();
  return d_int<T>(op, v);
}
template <class T, class V> static auto d_flt(int op, V &v) {
  switch (op) {
    case MX_OP_MAX: return v.template go<T, OpMax, OpMax>();
    case MX_OP_MIN: return v.template go<T, OpMin, OpMin>();
    case MX_OP_SUM: return v.template go<T, OpSum, OpSum>();
    case MX_OP_PROD: return v.template go<T, OpProd, OpProd>();
    default: return v.none();
  }
}
template <class V> static auto d_x87(int op, V &v) {
  switch (op) {
    case MX_OP_MAX: return v.template go<x87, OpX87Max, OpX87Max>();
    case MX_OP_MIN: return v.template go<x87, OpX87Min, OpX87Min>();
    case MX_OP_SUM: return v.template go<x87, OpX87Sum, OpX87Sum>();
    case MX_OP_PROD: return v.template go<x87, OpX87Prod, OpX87Prod>();
    default: return v.none();
  }
}
template <class T, class V> static auto d_cplx(int op, V &v) {
  switch (op) {
    case MX_OP_SUM: return v.template go<T, OpCsum, OpCsum>();
    case MX_OP_PROD: return v.template go<T, OpCprod, OpCprod>();
    default: return v.none();
  }
}
template <class V> static auto d_x87c(int op, V &v) {
  switch (op) {
    case MX_OP_SUM: return v.template go<x87c, OpX87Csum, OpX87Csum>();
    case MX_OP_PROD: return v.template go<x87c, OpX87Cprod, OpX87Cprod>();
    default: return v.none();
  }
}
template <class P, class V> static auto d_loc(int op, V &v) {
  switch (op) {
    case MX_OP_MAXLOC: return v.template go<P, OpLoc2<true>, OpLoc3<true>>();
    case MX_OP_MINLOC: return v.template go<P, OpLoc2<false>, OpLoc3<false>>();
    default: return v.none();
  }
}
template <class T, class V> static auto d_logic(int op, V &v) {  // LOGICAL, bool
  switch (op) {
    case MX_OP_LAND: return v.template go<T, OpLand, OpLand>();
    case MX_OP_LOR: return v.template go<T, OpLor, OpLor>();
    case MX_OP_LXOR: return v.template go<T, OpLxor, OpLxor>();
    default: return v.none();
  }
}
template <class V> static auto d_byte(int op, V &v) {  // MPI_BYTE slot
  switch (op) {
    case MX_OP_BAND: return v.template go<uint8_t, OpBand, OpBand>();
    case MX_OP_BOR: return v.template go<uint8_t, OpBor, OpBor>();
    case MX_OP_BXOR: return v.template go<uint8_t, OpBxor, OpBxor>();
    default: return v.none();
  }
}

template <class V> static auto dispatch(int op, int type, V &v) {
  switch (type) {
    case MX_TYPE_INT8_T: return d_int<int8_t>(op, v);
    case MX_TYPE_UINT8_T: return d_int<uint8_t>(op, v);
    case MX_TYPE_INT16_T: return d_int<int16_t>(op, v);
    case MX_TYPE_UINT16_T: return d_int<uint16_t>(op, v);
    case MX_TYPE_INT32_T: return d_int<int32_t>(op, v);
    case MX_TYPE_UINT32_T: return d_int<uint32_t>(op, v);
    case MX_TYPE_INT64_T: return d_int<int64_t>(op, v);
    case MX_TYPE_UINT64_T: return d_int<uint64_t>(op, v);
    case MX_TYPE_INTEGER: case MX_TYPE_INTEGER4: return d_fint<int32_t>(op, v);
    case MX_TYPE_INTEGER1: return d_fint<int8_t>(op, v);
    case MX_TYPE_INTEGER2: return d_fint<int16_t>(op, v);
    case MX_TYPE_INTEGER8: return d_fint<int64_t>(op, v);
    case MX_TYPE_FLOAT: case MX_TYPE_REAL: case MX_TYPE_REAL4: return d_flt<float>(op, v);
    case MX_TYPE_DOUBLE: case MX_TYPE_REAL8: case MX_TYPE_DOUBLE_PRECISION: return d_flt<double>(op, v);
    case MX_TYPE_LONG_DOUBLE: return d_x87(op, v);
    case MX_TYPE_LOGICAL: return d_logic<int32_t>(op, v);
    case MX_TYPE_BOOL: return d_logic<uint8_t>(op, v);
    case MX_TYPE_C_FLOAT_COMPLEX: return d_cplx<f32c>(op, v);
    case MX_TYPE_C_DOUBLE_COMPLEX: return d_cplx<f64c>(op, v);
    case MX_TYPE_C_LONG_DOUBLE_COMPLEX: return d_x87c(op, v);
    case MX_TYPE_BYTE: return d_byte(op, v);
    case MX_TYPE_2REAL: return d_loc<p_2real>(op, v);
    case MX_TYPE_2DOUBLE_PRECISION: return d_loc<p_2double>(op, v);
    case MX_TYPE_2INTEGER: return d_loc<p_2int>(op, v);
    case MX_TYPE_FLOAT_INT: return d_loc<p_float_int>(op, v);
    case MX_TYPE_DOUBLE_INT: return d_loc<p_double_int>(op, v);
    case MX_TYPE_LONG_INT: return d_loc<p_long_int>(op, v);
    case MX_TYPE_2INT: return d_loc<p_2int>(op, v);
    case MX_TYPE_SHORT_INT: return d_loc<p_short_int>(op, v);
    case MX_TYPE_LONG_DOUBLE_INT: return d_loc<x87_pair>(op, v);
    default: return v.none();
  }
}

}  // namespace mx
