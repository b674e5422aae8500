// mx_mem.hpp -- 16-byte global accesses with an explicit cache policy.
//
// Streaming kernels (K1 op kernels, collective copies) touch every byte once.
// Measured on MI355X (tools/bw_probe3.hip, profiles/r01/bw_probe3_policy.txt):
// the dense one-vector-per-lane 2-buffer SUM streams 1 GiB buffers at
// 5.65-5.86 TB/s with default loads/stores, 6.30-6.46 TB/s when BOTH the
// loads and the store are non-temporal (`global_load/store_dwordx4 ... nt`),
// and no better with only one side nt.  Below the Infinity-Cache capacity a
// re-used working set is served on-die, which nt would forfeit, so the
// policy is chosen per launch from the bytes all its streams touch
// (mx_nt_for(bytes), threshold MX_NT_MIN_BYTES, default 384 MiB).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace mx {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// The global-address-space view of a pointer.  Through a generic pointer the
// compiler emits flat instructions, which count on lgkmcnt as well as vmcnt,
// so in a kernel that also uses LDS every LDS wait then waits for the
// outstanding global stores too (round 6: found in the service's tagged-word
// loop and the LDS-staged convertor kernels).  Use it on every global access
// of a kernel that mixes them with LDS.
template <class T>
__device__ __forceinline__ __attribute__((address_space(1))) T *gp(T *p) {
  return (__attribute__((address_space(1))) T *)p;
}

// Both policies move the 16 bytes as one u32x4 copied straight into the
// destination object, so bytes outside a struct's fields (padding of the
// pair types) travel unchanged.  (Returning the struct by value would let
// the compiler treat those bytes as undefined.)
// (global memory only: the accesses are global_*, never flat -- see gp)
template <bool NT, class V>
__device__ __forceinline__ void ld16(V &out, const V *p) {
  if constexpr (sizeof(V) == 16) {   // other sizes: never on a vector path
    const __attribute__((address_space(1))) u32x4 *q = gp(reinterpret_cast<const u32x4 *>(p));
    u32x4 r;
    if constexpr (NT) r = __builtin_nontemporal_load(q);
    else r = *q;
    __builtin_memcpy(&out, &r, 16);
  } else {
    out = *p;
  }
}

template <bool NT, class V>
__device__ __forceinline__ void st16(V *p, const V &v) {
  if constexpr (sizeof(V) == 16) {
    u32x4 r;
    __builtin_memcpy(&r, &v, 16);
    __attribute__((address_space(1))) u32x4 *q = gp(reinterpret_cast<u32x4 *>(p));
    if constexpr (NT) __builtin_nontemporal_store(r, q);
    else *q = r;
  } else {
    *p = v;
  }
}

// true if a launch whose streams together touch `bytes` should use nt accesses
bool mx_nt_for(size_t bytes);

}  // namespace mx
