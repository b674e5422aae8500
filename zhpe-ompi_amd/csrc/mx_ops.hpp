// mx_ops.hpp -- device-side element operators for the predefined MPI_Ops.
//
// Each functor computes r = f(x, y) where x is the reference's FIRST operand
// and y the SECOND:
//   2-buffer  (op_base_functions.c:40-104)   x = inout (out), y = in
//   3-buffer  (op_base_functions.c:654-775)  x = in1,         y = in2
// i.e. exactly the operand roles of the reference's `current_func(*(b),*(a))`
// and `*(b) op= *(a)`, which matters for MAX/MIN with NaN or +-0 and for
// MAXLOC/MINLOC ties.
//
// Bit-exactness rules (hard parts):
//  * MAX/MIN are `x > y ? x : y` / `x < y ? x : y` -- never v_max/v_min
//    (those differ on NaN and -0); the file is compiled without fast-math.
//  * integer SUM/PROD wrap: computed in the unsigned type of at least 32
//    bits, then truncated (== C promotion + truncation on the host).
//  * LAND/LOR/LXOR normalise to 0/1 (:417, :439, :461).
//  * complex PROD is the unfused (ac-bd, ad+bc) of GCC's inline expansion,
//    with libgcc __mulsc3/__muldc3's Annex-G recovery when both parts are
//    NaN; the library is compiled with -ffp-contract=off.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mx {

template <class T> struct utype { using type = T; };
template <> struct utype<int8_t> { using type = uint32_t; };
template <> struct utype<uint8_t> { using type = uint32_t; };
template <> struct utype<int16_t> { using type = uint32_t; };
template <> struct utype<uint16_t> { using type = uint32_t; };
template <> struct utype<int32_t> { using type = uint32_t; };
template <> struct utype<uint32_t> { using type = uint32_t; };
template <> struct utype<int64_t> { using type = uint64_t; };
template <> struct utype<uint64_t> { using type = uint64_t; };
template <> struct utype<char> { using type = uint32_t; };
template <> struct utype<bool> { using type = uint32_t; };

// ---- scalar operators ---------------------------------------------------
struct OpMax {
  template <class T> __device__ __forceinline__ T operator()(T x, T y) const { return x > y ? x : y; }
};
struct OpMin {
  template <class T> __device__ __forceinline__ T operator()(T x, T y) const { return x < y ? x : y; }
};
struct OpSum {
  template <class T> __device__ __forceinline__ T operator()(T x, T y) const {
    using U = typename utype<T>::type;
    return (T)((U)x + (U)y);
  }
  __device__ __forceinline__ float operator()(float x, float y) const { return __fadd_rn(x, y); }
  __device__ __forceinline__ double operator()(double x, double y) const { return __dadd_rn(x, y); }
};
struct OpProd {
  template <class T> __device__ __forceinline__ T operator()(T x, T y) const {
    using U = typename utype<T>::type;
    return (T)((U)x * (U)y);
  }
  __device__ __forceinline__ float operator()(float x, float y) const { return __fmul_rn(x, y); }
  __device__ __forceinline__ double operator()(double x, double y) const { return __dmul_rn(x, y); }
};
struct OpLand {
  template <class T> __device__ __forceinline__ T operator()(T x, T y) const { return (T)((x != 0) & (y != 0)); }
};
struct OpLor {
  template <class T> __device__ __forceinline__ T operator()(T x, T y) const { return (T)((x != 0) | (y != 0)); }
};
struct OpLxor {
  template <class T> __device__ __forceinline__ T operator()(T x, T y) const { return (T)((x != 0) ^ (y != 0)); }
};
struct OpBand {
  template <class T> __device__ __forceinline__ T operator()(T x, T y) const { return (T)(x & y); }
};
struct OpBor {
  template <class T> __device__ __forceinline__ T operator()(T x, T y) const { return (T)(x | y); }
};
struct OpBxor {
  template <class T> __device__ __forceinline__ T operator()(T x, T y) const { return (T)(x ^ y); }
};

// ---- complex (interleaved re, im; C _Complex layout) -------------------
template <class F> struct alignas(2 * sizeof(F)) cplx { F re, im; };

template <class F> __device__ __forceinline__ F fmul_(F a, F b);
template <> __device__ __forceinline__ float fmul_(float a, float b) { return __fmul_rn(a, b); }
template <> __device__ __forceinline__ double fmul_(double a, double b) { return __dmul_rn(a, b); }
template <class F> __device__ __forceinline__ F fadd_(F a, F b);
template <> __device__ __forceinline__ float fadd_(float a, float b) { return __fadd_rn(a, b); }
template <> __device__ __forceinline__ double fadd_(double a, double b) { return __dadd_rn(a, b); }
template <class F> __device__ __forceinline__ F fsub_(F a, F b);
template <> __device__ __forceinline__ float fsub_(float a, float b) { return __fsub_rn(a, b); }
template <> __device__ __forceinline__ double fsub_(double a, double b) { return __dsub_rn(a, b); }

template <class F> __device__ __forceinline__ F box_(bool inf, F sign_of) {
  return copysign(inf ? (F)1 : (F)0, sign_of);
}

// (a + ib) * (c + id) with the semantics of GCC's inline complex multiply:
// x = ac - bd, y = ad + bc, and -- only if both are NaN -- the C99 Annex G
// recovery of libgcc's __mulsc3/__muldc3 (boxing infinities, zeroing NaNs).
template <class F>
__device__ __noinline__ void cmul_recover(F a, F b, F c, F d, F ac, F bd, F ad, F bc, F &x, F &y) {
  bool recalc = false;
  if (isinf(a) || isinf(b)) {
    a = box_(isinf(a), a);
    b = box_(isinf(b), b);
    if (isnan(c)) c = copysign((F)0, c);
    if (isnan(d)) d = copysign((F)0, d);
    recalc = true;
  }
  if (isinf(c) || isinf(d)) {
    c = box_(isinf(c), c);
    d = box_(isinf(d), d);
    if (isnan(a)) a = copysign((F)0, a);
    if (isnan(b)) b = copysign((F)0, b);
    recalc = true;
  }
  if (!recalc && (isinf(ac) || isinf(bd) || isinf(ad) || isinf(bc))) {
    if (isnan(a)) a = copysign((F)0, a);
    if (isnan(b)) b = copysign((F)0, b);
    if (isnan(c)) c = copysign((F)0, c);
    if (isnan(d)) d = copysign((F)0, d);
    recalc = true;
  }
  if (recalc) {
    const F inf = (F)INFINITY;
    x = fmul_(inf, fsub_(fmul_(a, c), fmul_(b, d)));
    y = fmul_(inf, fadd_(fmul_(a, d), fmul_(b, c)));
  }
}

template <class F>
__device__ __forceinline__ cplx<F> cmul(cplx<F> p, cplx<F> q) {
  const F a = p.re, b = p.im, c = q.re, d = q.im;
  const F ac = fmul_(a, c), bd = fmul_(b, d), ad = fmul_(a, d), bc = fmul_(b, c);
  F x = fsub_(ac, bd), y = fadd_(ad, bc);
  if (__builtin_expect(isnan(x) && isnan(y), 0)) cmul_recover<F>(a, b, c, d, ac, bd, ad, bc, x, y);
  return cplx<F>{x, y};
}

struct OpCsum {
  template <class F> __device__ __forceinline__ cplx<F> operator()(cplx<F> x, cplx<F> y) const {
    return cplx<F>{fadd_(x.re, y.re), fadd_(x.im, y.im)};
  }
};
struct OpCprod {
  template <class F> __device__ __forceinline__ cplx<F> operator()(cplx<F> x, cplx<F> y) const {
    return cmul<F>(x, y);
  }
};

// ---- MAXLOC / MINLOC pairs (value, index), host struct layout ----------
template <class V, class K> struct pair_t { V v; K k; };

// Value-field assignment of a pair; overloaded for x87 so that only the 10
// value bytes move (the host's `b->v = a->v` is an fldt/fstpt pair).
template <class V> __device__ __forceinline__ void loc_assign(V &a, const V &b) { a = b; }

// 2-buffer LOC_FUNC (:88-104): x = out, y = in.
//   if (in.v OP out.v) out = in; else if (in.v == out.v) out.k = min(out.k, in.k)
// Only the v and k fields are written, so padding keeps the out bytes.
template <bool IS_MAX>
struct OpLoc2 {
  template <class P> __device__ __forceinline__ P operator()(P x, P y) const {
    const bool take = IS_MAX ? (y.v > x.v) : (y.v < x.v);
    if (take) { loc_assign(x.v, y.v); x.k = y.k; }
    else if (y.v == x.v) { x.k = x.k < y.k ? x.k : y.k; }
    return x;
  }
};
// 3-buffer LOC_FUNC_3BUF (:709-731): x = in1, y = in2.
template <bool IS_MAX>
struct OpLoc3 {
  template <class P> __device__ __forceinline__ P operator()(P x, P y) const {
    const bool take = IS_MAX ? (x.v > y.v) : (x.v < y.v);
    if (take) return x;
    if (x.v == y.v) { x.k = y.k < x.k ? y.k : x.k; return x; }
    return y;
  }
};

}  // namespace mx
