// mx_x87.hpp -- device emulation of the host's `long double` (x87 80-bit
// extended precision stored in 16 bytes) for the 8 reference kernels that
// use it: MAX/MIN/SUM/PROD long double, SUM/PROD complex long double and
// MAXLOC/MINLOC long_double_int (op_base_functions.c:189,252,316,385,341,
// 410,620,640).  The GPU has no 80-bit type, so values are unpacked to
// (sign, exponent, 64-bit significand), operated on with 128-bit integer
// arithmetic and rounded to nearest-even at 64 significand bits, with the
// x87 rules the host reference follows (precision control = extended):
//   * gradual underflow (denormals), overflow to +-inf;
//   * NaN propagation per Intel SDM vol.1 table 4-7: one NaN -> it, quieted;
//     SNaN vs QNaN -> the QNaN; two of a kind -> larger significand,
//     ties -> positive sign (probed on the host x87);
//   * invalid operations (inf-inf, 0*inf) -> the "real indefinite" QNaN
//     (sign 1, exponent 0x7fff, significand 0xC000000000000000);
//   * comparisons are IEEE ordered compares (fucomi): NaN -> false,
//     +0 == -0.
// Only the 10 value bytes are written; the 6 padding bytes of each element
// are passed through from the destination operand.
#pragma once
#ifdef MX_X87_HOST_TEST  // host build for tests/native/x87_check.cpp
#define __device__
#define __forceinline__ inline
#define __noinline__ __attribute__((noinline))
#else
#include <hip/hip_runtime.h>
#endif
#include <stdint.h>

namespace mx {

struct alignas(16) x87 {
  uint64_t m;    // significand, explicit integer bit 63
  uint16_t se;   // sign bit 15, biased exponent bits 0..14
  uint16_t pad[3];
};
struct alignas(16) x87c { x87 re, im; };
struct alignas(16) x87_pair { x87 v; int k; int pad[3]; };

typedef unsigned __int128 u128;

__device__ __forceinline__ void loc_assign(x87 &a, const x87 &b) { a.m = b.m; a.se = b.se; }

__device__ __forceinline__ int x87_exp(const x87 &a) { return a.se & 0x7fff; }
__device__ __forceinline__ int x87_sign(const x87 &a) { return a.se >> 15; }
// Unsupported encodings (a nonzero exponent with the explicit integer bit
// clear: unnormals, pseudo-NaNs, pseudo-infinities) are invalid operands
// since the 387: arithmetic returns the indefinite QNaN whatever the other
// operand, comparisons are unordered -- so for every test they are NaNs.
__device__ __forceinline__ bool x87_unsupported(const x87 &a) {
  return x87_exp(a) != 0 && (a.m >> 63) == 0;
}
__device__ __forceinline__ bool x87_isnan(const x87 &a) {
  return (x87_exp(a) == 0x7fff && (a.m << 1) != 0) || x87_unsupported(a);
}
__device__ __forceinline__ bool x87_isinf(const x87 &a) {
  return x87_exp(a) == 0x7fff && a.m == (1ull << 63);
}
__device__ __forceinline__ bool x87_iszero(const x87 &a) { return x87_exp(a) == 0 && a.m == 0; }

__device__ __forceinline__ x87 x87_make(const x87 &like, int s, int e, uint64_t m) {
  x87 r = like;  // keep padding of the destination operand
  r.m = m;
  r.se = (uint16_t)((s << 15) | (e & 0x7fff));
  return r;
}

__device__ __forceinline__ int clz128(u128 v) {
  const uint64_t hi = (uint64_t)(v >> 64), lo = (uint64_t)v;
  return hi ? __builtin_clzll(hi) : 64 + __builtin_clzll(lo);
}

// Magnitude key comparable lexicographically: (max(e,1), m).
__device__ __forceinline__ int x87_cmp_mag(const x87 &a, const x87 &b) {
  int ea = x87_exp(a), eb = x87_exp(b);
  if (ea == 0) ea = 1;
  if (eb == 0) eb = 1;
  if (ea != eb) return ea < eb ? -1 : 1;
  if (a.m != b.m) return a.m < b.m ? -1 : 1;
  return 0;
}

// Ordered compare: returns -1, 0, 1, or 2 for unordered.
__device__ __forceinline__ int x87_cmp(const x87 &a, const x87 &b) {
  if (x87_isnan(a) || x87_isnan(b)) return 2;
  const bool za = (a.m == 0 && x87_exp(a) == 0), zb = (b.m == 0 && x87_exp(b) == 0);
  if (za && zb) return 0;
  const int sa = x87_sign(a), sb = x87_sign(b);
  if (sa != sb) return sa ? -1 : 1;
  const int c = x87_cmp_mag(a, b);
  return sa ? -c : c;
}
__device__ __forceinline__ bool operator>(const x87 &a, const x87 &b) { return x87_cmp(a, b) == 1; }
__device__ __forceinline__ bool operator<(const x87 &a, const x87 &b) { return x87_cmp(a, b) == -1; }
__device__ __forceinline__ bool operator==(const x87 &a, const x87 &b) { return x87_cmp(a, b) == 0; }

__device__ __forceinline__ x87 x87_indefinite(const x87 &like) {
  return x87_make(like, 1, 0x7fff, 0xC000000000000000ull);
}

// NaN result for an operation with at least one NaN operand.  Inlined: a
// call taking its operands by reference puts them in scratch on the hot path
// (the reference escapes), which cost complex PROD a 304-byte frame.
__device__ __forceinline__ x87 x87_nan_result(const x87 &like, const x87 &a, const x87 &b) {
  const bool na = x87_isnan(a), nb = x87_isnan(b);
  const uint64_t q = 1ull << 62;
  // the operand chosen is selected by value (a select between references
  // would force both operands into scratch)
  bool take_a = na;
  if (na && nb) {
    const bool qa = (a.m & q) != 0, qb = (b.m & q) != 0;
    if (qa != qb) take_a = qa;
    else if (a.m != b.m) take_a = a.m > b.m;
    else take_a = !x87_sign(a);   // tie: positive sign
  }
  const uint64_t wm = take_a ? a.m : b.m;
  const int ws = take_a ? x87_sign(a) : x87_sign(b);
  return x87_make(like, ws, 0x7fff, wm | q);
}

// value = S * 2^X with S normalised (bit 127 set): round to nearest even at
// 64 bits, handle gradual underflow and overflow.  The arithmetic fast paths
// are inlined (a call per element spills the 128-bit temporaries to
// scratch); only the NaN / complex-recovery paths stay out of line.
__device__ __forceinline__ x87 x87_round_norm(const x87 &like, int s, u128 S, int X) {
  int e = X + 64 + 16446;  // biased: value = m * 2^(e - 16446)
  if (__builtin_expect(e < 1, 0)) {
    const int sh = 1 - e;
    if (sh >= 128) {
      S = 1;  // pure sticky
    } else {
      const u128 lost = S & ((((u128)1) << sh) - 1);
      S >>= sh;
      if (lost) S |= 1;
    }
    e = 0;
  }
  uint64_t m = (uint64_t)(S >> 64);
  const uint64_t lo = (uint64_t)S;
  const bool rbit = (lo >> 63) != 0, sticky = (lo << 1) != 0;
  if (rbit && (sticky || (m & 1))) {
    m++;
    if (m == 0) { m = 1ull << 63; e++; }
  }
  if (e == 0 && (m >> 63)) e = 1;     // rounded up out of the denormal range
  if (e >= 0x7fff) return x87_make(like, s, 0x7fff, 1ull << 63);  // overflow -> inf
  return x87_make(like, s, e, m);
}

// value = S * 2^X, S != 0, any normalisation
__device__ __forceinline__ x87 x87_round_pack(const x87 &like, int s, u128 S, int X) {
  const int z = clz128(S);
  return x87_round_norm(like, s, S << z, X - z);
}

// unpack finite nonzero to normalised (m with bit 63 set, value m*2^E)
__device__ __forceinline__ void x87_unpack(const x87 &a, uint64_t &m, int &E) {
  int e = x87_exp(a);
  m = a.m;
  E = (e ? e : 1) - 16446;
  const int lz = __builtin_clzll(m);
  m <<= lz;
  E -= lz;
}

// both operands normal finite (exponent 1..0x7ffe, integer bit set): the
// common case, taken with one test instead of the special-case ladder
__device__ __forceinline__ bool x87_both_normal(const x87 &a, const x87 &b) {
  return (unsigned)(x87_exp(a) - 1) < 0x7ffeu && (unsigned)(x87_exp(b) - 1) < 0x7ffeu && (int64_t)(a.m & b.m) < 0;
}

// sum of two normal finite values (x87_add's general case without unpacking)
__device__ __forceinline__ x87 x87_add_normal(const x87 &like, const x87 &a, const x87 &b) {
  const int sa = x87_sign(a), sb = x87_sign(b);
  uint64_t ma = a.m, mb = b.m;
  int ea = x87_exp(a), eb = x87_exp(b);
  int s = sa;
  if (ea < eb || (ea == eb && ma < mb)) {  // |a| >= |b|
    const uint64_t tm = ma; ma = mb; mb = tm;
    const int te = ea; ea = eb; eb = te;
    s = sb;
  }
  const int d = ea - eb;
  const u128 A = ((u128)ma) << 62;
  u128 B = ((u128)mb) << 62;
  if (d >= 128) {
    B = 1;
  } else if (d > 0) {
    const u128 lost = B & ((((u128)1) << d) - 1);
    B >>= d;
    if (lost) B |= 1;
  }
  const u128 S = (sa == sb) ? A + B : A - B;
  if (S == 0) return x87_make(like, 0, 0, 0);  // exact cancellation: +0 under RNE
  return x87_round_pack(like, s, S, ea - 16446 - 62);
}

__device__ __forceinline__ x87 x87_add(const x87 &like, const x87 &a, const x87 &b) {
  if (__builtin_expect(x87_both_normal(a, b), 1)) return x87_add_normal(like, a, b);
  if (x87_unsupported(a) || x87_unsupported(b)) return x87_indefinite(like);
  if (x87_isnan(a) || x87_isnan(b)) return x87_nan_result(like, a, b);
  const int sa = x87_sign(a), sb = x87_sign(b);
  if (x87_isinf(a) || x87_isinf(b)) {
    if (x87_isinf(a) && x87_isinf(b) && sa != sb) return x87_indefinite(like);
    return x87_make(like, x87_isinf(a) ? sa : sb, 0x7fff, 1ull << 63);
  }
  const bool za = x87_iszero(a), zb = x87_iszero(b);
  if (za && zb) return x87_make(like, sa & sb, 0, 0);
  // x + 0: the other operand, with a pseudo-denormal (e = 0, integer bit
  // set) re-encoded as the equal-valued normal, as the x87 does
  if (za) return x87_make(like, sb, (x87_exp(b) == 0 && (b.m >> 63)) ? 1 : x87_exp(b), b.m);
  if (zb) return x87_make(like, sa, (x87_exp(a) == 0 && (a.m >> 63)) ? 1 : x87_exp(a), a.m);
  uint64_t ma, mb;
  int Ea, Eb;
  x87_unpack(a, ma, Ea);
  x87_unpack(b, mb, Eb);
  int s = sa;
  if (Ea < Eb || (Ea == Eb && ma < mb)) {  // |a| >= |b|
    uint64_t tm = ma; ma = mb; mb = tm;
    int te = Ea; Ea = Eb; Eb = te;
    s = sb;
  }
  const int d = Ea - Eb;
  const u128 A = ((u128)ma) << 62;
  u128 B = ((u128)mb) << 62;
  if (d >= 128) {
    B = 1;
  } else if (d > 0) {
    const u128 lost = B & ((((u128)1) << d) - 1);
    B >>= d;
    if (lost) B |= 1;
  }
  // one path for effective addition and subtraction: a branch on the signs
  // would diverge on mixed-sign data
  const u128 S = (sa == sb) ? A + B : A - B;
  if (S == 0) return x87_make(like, 0, 0, 0);  // exact cancellation: +0 under RNE
  return x87_round_pack(like, s, S, Ea - 62);
}

__device__ __forceinline__ x87 x87_neg(const x87 &a) {
  x87 r = a;
  r.se ^= 0x8000;
  return r;
}
// fsub does not negate a NaN operand: NaNs propagate with their own sign
__device__ __forceinline__ x87 x87_sub(const x87 &like, const x87 &a, const x87 &b) {
  if (x87_isnan(b)) return x87_add(like, a, b);
  return x87_add(like, a, x87_neg(b));
}

__device__ __forceinline__ x87 x87_mul(const x87 &like, const x87 &a, const x87 &b) {
  if (__builtin_expect(x87_both_normal(a, b), 1)) {   // no unpacking: both integer bits set
    u128 P = (u128)a.m * (u128)b.m;
    int X = x87_exp(a) + x87_exp(b) - 2 * 16446;
    if (!(uint64_t)(P >> 127)) { P <<= 1; X--; }
    return x87_round_norm(like, x87_sign(a) ^ x87_sign(b), P, X);
  }
  if (x87_unsupported(a) || x87_unsupported(b)) return x87_indefinite(like);
  if (x87_isnan(a) || x87_isnan(b)) return x87_nan_result(like, a, b);
  const int s = x87_sign(a) ^ x87_sign(b);
  const bool ia = x87_isinf(a), ib = x87_isinf(b), za = x87_iszero(a), zb = x87_iszero(b);
  if (ia || ib) {
    if (za || zb) return x87_indefinite(like);
    return x87_make(like, s, 0x7fff, 1ull << 63);
  }
  if (za || zb) return x87_make(like, s, 0, 0);
  uint64_t ma, mb;
  int Ea, Eb;
  x87_unpack(a, ma, Ea);
  x87_unpack(b, mb, Eb);
  u128 P = (u128)ma * (u128)mb;  // normalised inputs: bit 127 or 126 set
  int X = Ea + Eb;
  if (!(uint64_t)(P >> 127)) { P <<= 1; X--; }
  return x87_round_norm(like, s, P, X);
}

// ---- operator functors (x = first operand, y = second) -----------------
struct OpX87Max {
  __device__ __forceinline__ x87 operator()(x87 x, x87 y) const { return x > y ? x : y; }
};
struct OpX87Min {
  __device__ __forceinline__ x87 operator()(x87 x, x87 y) const { return x < y ? x : y; }
};
// 2-buffer and 3-buffer write the destination's padding: x is the operand
// whose padding survives (2-buffer: out; 3-buffer: in1, out is fresh).
struct OpX87Sum {
  __device__ __forceinline__ x87 operator()(x87 x, x87 y) const { return x87_add(x, x, y); }
};
struct OpX87Prod {
  __device__ __forceinline__ x87 operator()(x87 x, x87 y) const { return x87_mul(x, x, y); }
};

// complex long double: gcc expands `*=` inline (x87) and calls __mulxc3 on
// NaN+iNaN; the same recovery as mx_ops.hpp's cmul_recover.
__device__ __forceinline__ x87 x87_copysign01(const x87 &like, bool one, const x87 &sign_of) {
  return one ? x87_make(like, x87_sign(sign_of), 16383, 1ull << 63) : x87_make(like, x87_sign(sign_of), 0, 0);
}

// Annex-G recovery of an x87 complex product whose both parts came out NaN
// (rare: out of line).  The operands travel as scalars and the partial
// products are recomputed here: a call taking references would keep the
// operands in scratch on the hot path.
struct x87c_bits { uint64_t xm, ym; uint32_t xse, yse; };
__device__ __noinline__ x87c_bits x87c_mul_recover(uint64_t am, uint32_t ase, uint64_t bm, uint32_t bse, uint64_t cm,
                                                   uint32_t cse, uint64_t dm, uint32_t dse) {
  x87 a{}, b{}, c{}, d{};
  a.m = am; a.se = (uint16_t)ase;
  b.m = bm; b.se = (uint16_t)bse;
  c.m = cm; c.se = (uint16_t)cse;
  d.m = dm; d.se = (uint16_t)dse;
  const x87 L = a;
  const x87 ac = x87_mul(L, a, c), bd = x87_mul(L, b, d), ad = x87_mul(L, a, d), bc = x87_mul(L, b, c);
  x87 x = x87_sub(L, ac, bd), y = x87_add(L, ad, bc);
  {
    bool recalc = false;
    if (x87_isinf(a) || x87_isinf(b)) {
      a = x87_copysign01(L, x87_isinf(a), a);
      b = x87_copysign01(L, x87_isinf(b), b);
      if (x87_isnan(c)) c = x87_copysign01(L, false, c);
      if (x87_isnan(d)) d = x87_copysign01(L, false, d);
      recalc = true;
    }
    if (x87_isinf(c) || x87_isinf(d)) {
      c = x87_copysign01(L, x87_isinf(c), c);
      d = x87_copysign01(L, x87_isinf(d), d);
      if (x87_isnan(a)) a = x87_copysign01(L, false, a);
      if (x87_isnan(b)) b = x87_copysign01(L, false, b);
      recalc = true;
    }
    if (!recalc && (x87_isinf(ac) || x87_isinf(bd) || x87_isinf(ad) || x87_isinf(bc))) {
      if (x87_isnan(a)) a = x87_copysign01(L, false, a);
      if (x87_isnan(b)) b = x87_copysign01(L, false, b);
      if (x87_isnan(c)) c = x87_copysign01(L, false, c);
      if (x87_isnan(d)) d = x87_copysign01(L, false, d);
      recalc = true;
    }
    if (recalc) {
      const x87 inf = x87_make(L, 0, 0x7fff, 1ull << 63);
      x = x87_mul(L, inf, x87_sub(L, x87_mul(L, a, c), x87_mul(L, b, d)));
      y = x87_mul(L, inf, x87_add(L, x87_mul(L, a, d), x87_mul(L, b, c)));
    }
  }
  return x87c_bits{x.m, y.m, x.se, y.se};
}

__device__ __forceinline__ x87c x87c_mul(const x87c &p, const x87c &q) {
  const x87 &a = p.re, &b = p.im, &c = q.re, &d = q.im;
  const x87 &L = p.re;
  const x87 ac = x87_mul(L, a, c), bd = x87_mul(L, b, d), ad = x87_mul(L, a, d), bc = x87_mul(L, b, c);
  x87 x = x87_sub(p.re, ac, bd), y = x87_add(p.im, ad, bc);
  if (__builtin_expect(x87_isnan(x) && x87_isnan(y), 0)) {
    const x87c_bits r = x87c_mul_recover(a.m, a.se, b.m, b.se, c.m, c.se, d.m, d.se);
    x.m = r.xm; x.se = (uint16_t)r.xse;
    y.m = r.ym; y.se = (uint16_t)r.yse;
  }
  return x87c{x, y};
}

struct OpX87Csum {
  __device__ __forceinline__ x87c operator()(x87c x, x87c y) const {
    return x87c{x87_add(x.re, x.re, y.re), x87_add(x.im, x.im, y.im)};
  }
};
struct OpX87Cprod {
  __device__ __forceinline__ x87c operator()(x87c x, x87c y) const { return x87c_mul(x, y); }
};

}  // namespace mx
