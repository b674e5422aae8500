// mx_reduce.hip -- K1..K4: the predefined MPI_Op element kernels on gfx950.
//
// Replaces the host loops of ompi/mca/op/base/op_base_functions.c
// (OP_FUNC :40-51, FUNC_FUNC :60-73, LOC_FUNC :88-104, 3-buffer :654-775)
// with HBM-streaming kernels:
//  * one 16-byte vector per lane per access (global_load/store_dwordx4),
//    UNROLL independent vectors in flight per lane, grid-stride over a grid
//    sized to fill the 256 CUs (no reuse => no LDS, no MFMA: the op is
//    <= 1 flop per element, arithmetic intensity ~0.08 flop/B -> HBM bound);
//  * head/tail elements that do not fill a 16-byte vector are handled by
//    the first lanes of the grid (ragged counts, unaligned sub-blocks of a
//    ring step);
//  * buffers whose misalignment differs mod 16 fall back to an
//    element-per-lane kernel (still coalesced).
// Algorithmic bytes per launch: 2-buffer 3*n*size (read in, read inout,
// write inout), 3-buffer 3*n*size.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stddef.h>

#include "mx_ops.hpp"
#include "mx_internal.h"
#include "mx_x87.hpp"

namespace mx {

constexpr int kBlock = 256;
constexpr int kUnroll = 4;

template <class T>
struct alignas(16) vec16 {
  static constexpr int N = 16 / sizeof(T);
  T e[N];
};

// Scalar per-element application, inout-form (x = b, y = a) or 3-buffer.
template <class T, class OP>
__device__ __forceinline__ void red2_elem(const T *__restrict__ a, T *__restrict__ b, size_t i) {
  b[i] = OP()(b[i], a[i]);
}

// 2-buffer, vector body: elements [head, head + nvec*N) as 16-B vectors.
template <class T, class OP>
__global__ void __launch_bounds__(kBlock)
k_reduce2(const T *__restrict__ a, T *__restrict__ b, size_t n, size_t head, size_t nvec) {
  using V = vec16<T>;
  constexpr int N = V::N;
  const size_t tid = (size_t)blockIdx.x * kBlock + threadIdx.x;
  const size_t stride = (size_t)gridDim.x * kBlock;
  const V *__restrict__ av = reinterpret_cast<const V *>(a + head);
  V *__restrict__ bv = reinterpret_cast<V *>(b + head);
  OP op;
  size_t i = tid;
  for (; i + (kUnroll - 1) * stride < nvec; i += kUnroll * stride) {
    V x[kUnroll], y[kUnroll];
#pragma unroll
    for (int u = 0; u < kUnroll; u++) { x[u] = bv[i + u * stride]; y[u] = av[i + u * stride]; }
#pragma unroll
    for (int u = 0; u < kUnroll; u++) {
#pragma unroll
      for (int j = 0; j < N; j++) x[u].e[j] = op(x[u].e[j], y[u].e[j]);
      bv[i + u * stride] = x[u];
    }
  }
  for (; i < nvec; i += stride) {
    V x = bv[i], y = av[i];
#pragma unroll
    for (int j = 0; j < N; j++) x.e[j] = op(x.e[j], y.e[j]);
    bv[i] = x;
  }
  // ragged head and tail
  const size_t tail0 = head + nvec * N;
  if (tid < head) red2_elem<T, OP>(a, b, tid);
  if (tid < n - tail0) red2_elem<T, OP>(a, b, tail0 + tid);
}

// 2-buffer, one element per lane (mismatched alignment, or element > 16 B).
template <class T, class OP>
__global__ void __launch_bounds__(kBlock)
k_reduce2_elem(const T *__restrict__ a, T *__restrict__ b, size_t n) {
  const size_t stride = (size_t)gridDim.x * kBlock;
  for (size_t i = (size_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride)
    red2_elem<T, OP>(a, b, i);
}

template <class T, class OP>
__global__ void __launch_bounds__(kBlock)
k_reduce3(const T *__restrict__ a1, const T *__restrict__ a2, T *__restrict__ o, size_t n,
          size_t head, size_t nvec) {
  using V = vec16<T>;
  constexpr int N = V::N;
  const size_t tid = (size_t)blockIdx.x * kBlock + threadIdx.x;
  const size_t stride = (size_t)gridDim.x * kBlock;
  const V *__restrict__ p = reinterpret_cast<const V *>(a1 + head);
  const V *__restrict__ q = reinterpret_cast<const V *>(a2 + head);
  V *__restrict__ ov = reinterpret_cast<V *>(o + head);
  OP op;
  size_t i = tid;
  for (; i + (kUnroll - 1) * stride < nvec; i += kUnroll * stride) {
    V x[kUnroll], y[kUnroll];
#pragma unroll
    for (int u = 0; u < kUnroll; u++) { x[u] = p[i + u * stride]; y[u] = q[i + u * stride]; }
#pragma unroll
    for (int u = 0; u < kUnroll; u++) {
#pragma unroll
      for (int j = 0; j < N; j++) x[u].e[j] = op(x[u].e[j], y[u].e[j]);
      ov[i + u * stride] = x[u];
    }
  }
  for (; i < nvec; i += stride) {
    V x = p[i], y = q[i];
#pragma unroll
    for (int j = 0; j < N; j++) x.e[j] = op(x.e[j], y.e[j]);
    ov[i] = x;
  }
  const size_t tail0 = head + nvec * N;
  if (tid < head) o[tid] = op(a1[tid], a2[tid]);
  if (tid < n - tail0) o[tail0 + tid] = op(a1[tail0 + tid], a2[tail0 + tid]);
}

template <class T, class OP>
__global__ void __launch_bounds__(kBlock)
k_reduce3_elem(const T *__restrict__ a1, const T *__restrict__ a2, T *__restrict__ o, size_t n) {
  const size_t stride = (size_t)gridDim.x * kBlock;
  OP op;
  for (size_t i = (size_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride)
    o[i] = op(a1[i], a2[i]);
}

static inline unsigned grid_for(size_t work_items) {
  // memory-bound: up to 8 blocks of 256 per CU, grid-stride beyond that
  size_t g = (work_items + kBlock - 1) / kBlock;
  const size_t cap = (size_t)g_num_cus * 8;
  if (g > cap) g = cap;
  if (g < 1) g = 1;
  return (unsigned)g;
}

template <class T, class OP>
static int launch2(const void *in, void *inout, size_t n, hipStream_t s) {
  const T *a = static_cast<const T *>(in);
  T *b = static_cast<T *>(inout);
  if (n == 0) return MX_SUCCESS;
  constexpr size_t N = (sizeof(T) <= 16 && 16 % sizeof(T) == 0) ? 16 / sizeof(T) : 0;
  const uintptr_t ma = (uintptr_t)a & 15, mb = (uintptr_t)b & 15;
  if (N == 0 || ma != mb || (ma % sizeof(T)) != 0) {
    hipLaunchKernelGGL((k_reduce2_elem<T, OP>), dim3(grid_for(n)), dim3(kBlock), 0, s, a, b, n);
    return mx_check_launch();
  }
  size_t head = ma ? (16 - ma) / sizeof(T) : 0;
  if (head > n) head = n;
  const size_t nvec = N ? (n - head) / N : 0;
  size_t work = nvec / kUnroll + 1;
  if (work < head + N) work = head + N;  // enough lanes for head + tail
  hipLaunchKernelGGL((k_reduce2<T, OP>), dim3(grid_for(work)), dim3(kBlock), 0, s, a, b, n, head, nvec);
  return mx_check_launch();
}

template <class T, class OP>
static int launch3(const void *in1, const void *in2, void *out, size_t n, hipStream_t s) {
  const T *a1 = static_cast<const T *>(in1);
  const T *a2 = static_cast<const T *>(in2);
  T *o = static_cast<T *>(out);
  if (n == 0) return MX_SUCCESS;
  constexpr size_t N = (sizeof(T) <= 16 && 16 % sizeof(T) == 0) ? 16 / sizeof(T) : 0;
  const uintptr_t m1 = (uintptr_t)a1 & 15, m2 = (uintptr_t)a2 & 15, mo = (uintptr_t)o & 15;
  if (N == 0 || m1 != m2 || m1 != mo || (m1 % sizeof(T)) != 0) {
    hipLaunchKernelGGL((k_reduce3_elem<T, OP>), dim3(grid_for(n)), dim3(kBlock), 0, s, a1, a2, o, n);
    return mx_check_launch();
  }
  size_t head = m1 ? (16 - m1) / sizeof(T) : 0;
  if (head > n) head = n;
  const size_t nvec = N ? (n - head) / N : 0;
  size_t work = nvec / kUnroll + 1;
  if (work < head + N) work = head + N;
  hipLaunchKernelGGL((k_reduce3<T, OP>), dim3(grid_for(work)), dim3(kBlock), 0, s, a1, a2, o, n, head, nvec);
  return mx_check_launch();
}

// ---- type-slot dispatch ---------------------------------------------------
typedef int (*launch2_fn)(const void *, void *, size_t, hipStream_t);
typedef int (*launch3_fn)(const void *, const void *, void *, size_t, hipStream_t);

struct entry { launch2_fn f2; launch3_fn f3; };

template <class T, class OP2, class OP3 = OP2>
constexpr entry E() { return entry{&launch2<T, OP2>, &launch3<T, OP3>}; }

using f32c = cplx<float>;
using f64c = cplx<double>;
using p_float_int = pair_t<float, int>;
using p_double_int = pair_t<double, int>;
using p_long_int = pair_t<long, int>;
using p_2int = pair_t<int, int>;
using p_short_int = pair_t<short, int>;
using p_2real = pair_t<float, float>;
using p_2double = pair_t<double, double>;
using p_ldouble_int = x87_pair;

static_assert(sizeof(p_float_int) == 8 && sizeof(p_double_int) == 16 && sizeof(p_long_int) == 16 &&
              sizeof(p_2int) == 8 && sizeof(p_short_int) == 8 && sizeof(p_2real) == 8 &&
              sizeof(p_2double) == 16 && sizeof(p_ldouble_int) == 32 && sizeof(f32c) == 8 &&
              sizeof(f64c) == 16 && sizeof(x87) == 16 && sizeof(x87c) == 32,
              "pair/complex layouts must match the host ABI");

// Integer-like op row for element type T (C integers and the Fortran
// integers that alias them).
template <class T>
static entry int_entry(int op) {
  switch (op) {
    case MX_OP_MAX: return E<T, OpMax>();
    case MX_OP_MIN: return E<T, OpMin>();
    case MX_OP_SUM: return E<T, OpSum>();
    case MX_OP_PROD: return E<T, OpProd>();
    case MX_OP_LAND: return E<T, OpLand>();
    case MX_OP_LOR: return E<T, OpLor>();
    case MX_OP_LXOR: return E<T, OpLxor>();
    case MX_OP_BAND: return E<T, OpBand>();
    case MX_OP_BOR: return E<T, OpBor>();
    case MX_OP_BXOR: return E<T, OpBxor>();
    default: return entry{nullptr, nullptr};
  }
}
template <class T>
static entry flt_entry(int op) {
  switch (op) {
    case MX_OP_MAX: return E<T, OpMax>();
    case MX_OP_MIN: return E<T, OpMin>();
    case MX_OP_SUM: return E<T, OpSum>();
    case MX_OP_PROD: return E<T, OpProd>();
    default: return entry{nullptr, nullptr};
  }
}
template <class T>
static entry cplx_entry(int op) {
  switch (op) {
    case MX_OP_SUM: return E<T, OpCsum>();
    case MX_OP_PROD: return E<T, OpCprod>();
    default: return entry{nullptr, nullptr};
  }
}
template <class P>
static entry loc_entry(int op) {
  switch (op) {
    case MX_OP_MAXLOC: return E<P, OpLoc2<true>, OpLoc3<true>>();
    case MX_OP_MINLOC: return E<P, OpLoc2<false>, OpLoc3<false>>();
    default: return entry{nullptr, nullptr};
  }
}
static entry logic_entry_i32(int op) {  // Fortran LOGICAL: LAND/LOR/LXOR only
  switch (op) {
    case MX_OP_LAND: return E<int32_t, OpLand>();
    case MX_OP_LOR: return E<int32_t, OpLor>();
    case MX_OP_LXOR: return E<int32_t, OpLxor>();
    default: return entry{nullptr, nullptr};
  }
}
static entry bool_entry(int op) {
  switch (op) {
    case MX_OP_LAND: return E<uint8_t, OpLand>();
    case MX_OP_LOR: return E<uint8_t, OpLor>();
    case MX_OP_LXOR: return E<uint8_t, OpLxor>();
    default: return entry{nullptr, nullptr};
  }
}
static entry bit_entry_u8(int op) {  // MPI_BYTE slot: BAND/BOR/BXOR only
  switch (op) {
    case MX_OP_BAND: return E<uint8_t, OpBand>();
    case MX_OP_BOR: return E<uint8_t, OpBor>();
    case MX_OP_BXOR: return E<uint8_t, OpBxor>();
    default: return entry{nullptr, nullptr};
  }
}
// Fortran integers: MAX MIN SUM PROD BAND BOR BXOR (no logical ops)
template <class T>
static entry fint_entry(int op) {
  if (op == MX_OP_LAND || op == MX_OP_LOR || op == MX_OP_LXOR) return entry{nullptr, nullptr};
  return int_entry<T>(op);
}

static entry x87_entry(int op) {  // long double: MAX MIN SUM PROD
  switch (op) {
    case MX_OP_MAX: return E<x87, OpX87Max>();
    case MX_OP_MIN: return E<x87, OpX87Min>();
    case MX_OP_SUM: return E<x87, OpX87Sum>();
    case MX_OP_PROD: return E<x87, OpX87Prod>();
    default: return entry{nullptr, nullptr};
  }
}
static entry x87c_entry(int op) {  // complex long double: SUM PROD
  switch (op) {
    case MX_OP_SUM: return E<x87c, OpX87Csum>();
    case MX_OP_PROD: return E<x87c, OpX87Cprod>();
    default: return entry{nullptr, nullptr};
  }
}
static entry x87_loc_entry(int op) { return loc_entry<x87_pair>(op); }

static entry lookup(int op, int type) {
  switch (type) {
    case MX_TYPE_INT8_T: return int_entry<int8_t>(op);
    case MX_TYPE_UINT8_T: return int_entry<uint8_t>(op);
    case MX_TYPE_INT16_T: return int_entry<int16_t>(op);
    case MX_TYPE_UINT16_T: return int_entry<uint16_t>(op);
    case MX_TYPE_INT32_T: return int_entry<int32_t>(op);
    case MX_TYPE_UINT32_T: return int_entry<uint32_t>(op);
    case MX_TYPE_INT64_T: return int_entry<int64_t>(op);
    case MX_TYPE_UINT64_T: return int_entry<uint64_t>(op);
    case MX_TYPE_INTEGER: case MX_TYPE_INTEGER4: return fint_entry<int32_t>(op);
    case MX_TYPE_INTEGER1: return fint_entry<int8_t>(op);
    case MX_TYPE_INTEGER2: return fint_entry<int16_t>(op);
    case MX_TYPE_INTEGER8: return fint_entry<int64_t>(op);
    case MX_TYPE_FLOAT: case MX_TYPE_REAL: case MX_TYPE_REAL4: return flt_entry<float>(op);
    case MX_TYPE_DOUBLE: case MX_TYPE_REAL8: case MX_TYPE_DOUBLE_PRECISION: return flt_entry<double>(op);
    case MX_TYPE_LONG_DOUBLE: return x87_entry(op);
    case MX_TYPE_LOGICAL: return logic_entry_i32(op);
    case MX_TYPE_BOOL: return bool_entry(op);
    case MX_TYPE_C_FLOAT_COMPLEX: return cplx_entry<f32c>(op);
    case MX_TYPE_C_DOUBLE_COMPLEX: return cplx_entry<f64c>(op);
    case MX_TYPE_C_LONG_DOUBLE_COMPLEX: return x87c_entry(op);
    case MX_TYPE_BYTE: return bit_entry_u8(op);
    case MX_TYPE_2REAL: return loc_entry<p_2real>(op);
    case MX_TYPE_2DOUBLE_PRECISION: return loc_entry<p_2double>(op);
    case MX_TYPE_2INTEGER: return loc_entry<p_2int>(op);
    case MX_TYPE_FLOAT_INT: return loc_entry<p_float_int>(op);
    case MX_TYPE_DOUBLE_INT: return loc_entry<p_double_int>(op);
    case MX_TYPE_LONG_INT: return loc_entry<p_long_int>(op);
    case MX_TYPE_2INT: return loc_entry<p_2int>(op);
    case MX_TYPE_SHORT_INT: return loc_entry<p_short_int>(op);
    case MX_TYPE_LONG_DOUBLE_INT: return x87_loc_entry(op);
    default: return entry{nullptr, nullptr};
  }
}

}  // namespace mx

using namespace mx;

static bool is_fortran_slot(int t) {
  switch (t) {
    case MX_TYPE_INTEGER: case MX_TYPE_INTEGER1: case MX_TYPE_INTEGER2: case MX_TYPE_INTEGER4:
    case MX_TYPE_INTEGER8: case MX_TYPE_REAL: case MX_TYPE_REAL4: case MX_TYPE_REAL8:
    case MX_TYPE_DOUBLE_PRECISION: case MX_TYPE_LOGICAL: case MX_TYPE_2REAL:
    case MX_TYPE_2DOUBLE_PRECISION: case MX_TYPE_2INTEGER:
      return true;
    default:
      return false;
  }
}

extern "C" int mx_op_supported(int op, int type, int table_variant) {
  if (op < 0 || op >= MX_OP_COUNT || type < 0 || type >= MX_TYPE_COUNT) return 0;
  if (table_variant == MX_TABLE_C_ONLY && is_fortran_slot(type)) return 0;
  return lookup(op, type).f2 != nullptr;
}

extern "C" size_t mx_type_size(int t) {
  switch (t) {
    case MX_TYPE_INT8_T: case MX_TYPE_UINT8_T: case MX_TYPE_INTEGER1: case MX_TYPE_BOOL: case MX_TYPE_BYTE:
      return 1;
    case MX_TYPE_INT16_T: case MX_TYPE_UINT16_T: case MX_TYPE_INTEGER2:
      return 2;
    case MX_TYPE_INT32_T: case MX_TYPE_UINT32_T: case MX_TYPE_INTEGER: case MX_TYPE_INTEGER4:
    case MX_TYPE_FLOAT: case MX_TYPE_REAL: case MX_TYPE_REAL4: case MX_TYPE_LOGICAL:
      return 4;
    case MX_TYPE_INT64_T: case MX_TYPE_UINT64_T: case MX_TYPE_INTEGER8: case MX_TYPE_DOUBLE:
    case MX_TYPE_REAL8: case MX_TYPE_DOUBLE_PRECISION: case MX_TYPE_C_FLOAT_COMPLEX:
    case MX_TYPE_FLOAT_INT: case MX_TYPE_2INT: case MX_TYPE_SHORT_INT: case MX_TYPE_2REAL:
    case MX_TYPE_2INTEGER:
      return 8;
    case MX_TYPE_LONG_DOUBLE: case MX_TYPE_C_DOUBLE_COMPLEX: case MX_TYPE_DOUBLE_INT:
    case MX_TYPE_LONG_INT: case MX_TYPE_2DOUBLE_PRECISION:
      return 16;
    case MX_TYPE_C_LONG_DOUBLE_COMPLEX: case MX_TYPE_LONG_DOUBLE_INT:
      return 32;
    default:
      return 0;
  }
}

extern "C" int mx_reduce2(int op, int type, const void *in, void *inout, size_t count, void *stream) {
  if (op < 0 || op >= MX_OP_COUNT || type < 0 || type >= MX_TYPE_COUNT) return MX_ERR_ARG;
  entry e = lookup(op, type);
  if (!e.f2) return MX_ERR_UNSUPPORTED;
  if (count == 0) return MX_SUCCESS;
  if (!in || !inout) return MX_ERR_ARG;
  int rc = mx_ensure_init();
  if (rc) return rc;
  return e.f2(in, inout, count, (hipStream_t)stream);
}

extern "C" int mx_reduce3(int op, int type, const void *in1, const void *in2, void *out, size_t count,
                          void *stream) {
  if (op < 0 || op >= MX_OP_COUNT || type < 0 || type >= MX_TYPE_COUNT) return MX_ERR_ARG;
  entry e = lookup(op, type);
  if (!e.f3) return MX_ERR_UNSUPPORTED;
  if (count == 0) return MX_SUCCESS;
  if (!in1 || !in2 || !out) return MX_ERR_ARG;
  int rc = mx_ensure_init();
  if (rc) return rc;
  return e.f3(in1, in2, out, count, (hipStream_t)stream);
}
