// mx_fold.hpp -- device side of the collective fold: the kernels that read
// the n contributions of a range of elements and evaluate, per element, the
// reduction tree of a reference algorithm (see mx_coll.hip for the host
// side).  Three evaluators:
//   k_fold     CHAIN / BUTTERFLY programs in registers (allreduce and
//              reduce_scatter: the ring / recursive-doubling / Rabenseifner /
//              recursive-halving trees);
//   k_oneshot  the same programs fused with the all-peer exchange for small
//              allreduce messages;
//   k_vm       an LDS-register VM for arbitrary trees and multi-output DAGs:
//              rooted reduce (binomial / binary / pipeline / chain /
//              in-order binary trees of coll_base_topo.c), scan / exscan
//              (linear and recursive doubling) and reduce_scatter_block.
// The per-type instantiations are split over mx_fold_f*.hip by element-type
// family (build time); fold_fns() finds the launchers of an (op, type) pair.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include "mx_dispatch.hpp"
#include "mx_internal.h"
#include "mx_mem.hpp"
#include "../../include/mx_coll.h"

namespace mx {

constexpr int MAXR = MX_MAX_RANKS;
constexpr int kFB = 256;  // fold / copy block size

// one-shot small-message allreduce: flag layout shared with mx_coll.hip
// READY carries (generation << 1) | info bit: the info bit is the root's
// MPI_IN_PLACE choice in a rooted reduce (the operand roles of the root's
// own combination depend on it, and the element parts are folded by other
// ranks); PUSHED and DONE carry the plain generation.
enum { FLAG_READY = 0, FLAG_PUSHED = 1, FLAG_DONE = 2, NFLAGS = 3 };
constexpr int OSWG = 64;
constexpr int OS_MAXSEG = 16;


// Poisoned communicator (mx_comm::poison): a peer wait of an earlier kernel
// timed out.  The word is device memory written at agent scope; kernels of
// the same stream that run later see it (kernel boundaries order it).
__device__ __forceinline__ bool poisoned(const int *poison) {
  return poison && __hip_atomic_load(gp(poison), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
}
__device__ __forceinline__ void raise_timeout(int *err, int *poison) {
  __hip_atomic_store(err, MX_ERR_TIMEOUT, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  if (poison) __hip_atomic_store(poison, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ---------------------------------------------------------------------------
// fold programs
// ---------------------------------------------------------------------------
enum { PROG_CHAIN = 0, PROG_BFLY = 1 };

struct FoldProg {
  int kind;
  int n;           // chain: number of operands; butterfly: p' leaves
  int D;           // butterfly depth (p' = 1 << D)
  int acc_first;   // chain: accumulator is the target (first operand)
  uint32_t pref;   // butterfly: bit s set -> upper half is the target at level s
  int8_t ord[MAXR];  // chain: source index per step
  int8_t la[MAXR];   // butterfly leaf slot i: first operand source
  int8_t lb[MAXR];   //   second operand source, -1 = plain leaf
};

struct FoldArgs {
  const char *src[MAXR];
  char *dst[MAXR];
  int ndst;
  size_t n, head, nvec;  // elements; scalar head; 16-B vectors after head
  const int *poison;     // communicator poison word (null: local)
  int nt_force;          // non-temporal accesses whatever the footprint (operands read once over xGMI)
  FoldProg p;
};

template <class T> struct alignas(16) fvec {
  static constexpr int N = 16 / sizeof(T);
  T e[N];
};

template <class OP, class T>
__device__ __forceinline__ T comb(const T &x, const T &y) { return OP()(x, y); }
template <class OP, class T>
__device__ __forceinline__ fvec<T> comb(const fvec<T> &x, const fvec<T> &y) {
  fvec<T> r;
#pragma unroll
  for (int j = 0; j < fvec<T>::N; j++) r.e[j] = OP()(x.e[j], y.e[j]);
  return r;
}

// Evaluates the program; LD(j) returns operand j at this lane's position.
// NM bounds the program's operand count (p.n <= NM): the loops unroll to
// NM steps, so a small program costs a few instructions, not MAXR guarded
// steps (eval_prog_small picks NM from p.n).
template <int NM, class OP, class V, class L>
__device__ __forceinline__ V eval_prog_nm(const FoldProg &p, L LD) {
  if (p.kind == PROG_CHAIN) {
    V acc = LD(p.ord[0]);
#pragma unroll
    for (int j = 1; j < NM; j++) {
      if (j < p.n) {
        const V v = LD(p.ord[j]);
        acc = p.acc_first ? comb<OP>(acc, v) : comb<OP>(v, acc);
      }
    }
    return acc;
  }
  V R[NM];
#pragma unroll
  for (int i = 0; i < NM; i++) {
    if (i < p.n) {
      V a = LD(p.la[i]);
      if (p.lb[i] >= 0) a = comb<OP>(a, LD(p.lb[i]));
      R[i] = a;
    }
  }
#pragma unroll
  for (int s = 0; (1 << s) < NM; s++) {
    if (s < p.D) {
      const int h = 1 << s;
      const bool hi_first = (p.pref >> s) & 1;
#pragma unroll
      for (int u = 0; u + h < NM; u += 2 << s) {
        if (u < p.n) R[u] = hi_first ? comb<OP>(R[u + h], R[u]) : comb<OP>(R[u], R[u + h]);
      }
    }
  }
  return R[0];
}
template <class OP, class V, class L>
__device__ __forceinline__ V eval_prog(const FoldProg &p, L LD) {
  return eval_prog_nm<MAXR, OP, V>(p, LD);
}
// the same with the bound picked from the program (uniform branch): the
// latency-bound small-message folds (one-shot, tagged words)
template <class OP, class V, class L>
__device__ __forceinline__ V eval_prog_small(const FoldProg &p, L LD) {
  if (p.n <= 2) return eval_prog_nm<2, OP, V>(p, LD);
  if (p.n <= 4) return eval_prog_nm<4, OP, V>(p, LD);
  if (p.n <= 8) return eval_prog_nm<8, OP, V>(p, LD);
  return eval_prog_nm<MAXR, OP, V>(p, LD);
}

template <class T, class OP, bool NT>
__global__ void __launch_bounds__(kFB) k_fold(FoldArgs a) {
  if (poisoned(a.poison)) return;
  using V = fvec<T>;
  constexpr int N = V::N;
  const size_t tid = (size_t)blockIdx.x * kFB + threadIdx.x;
  if (N > 0 && tid < a.nvec) {
    const size_t off = a.head * sizeof(T) + tid * 16;
    const V r = eval_prog<OP, V>(a.p, [&](int j) {
      V v;
      ld16<NT>(v, reinterpret_cast<const V *>(a.src[j] + off));
      return v;
    });
#pragma unroll
    for (int d = 0; d < MAXR; d++)
      if (d < a.ndst) st16<NT>(reinterpret_cast<V *>(a.dst[d] + off), r);
  }
  // scalar elements: the head, the tail, or everything (element path)
  const size_t tail0 = a.head + a.nvec * N;
  size_t e = (size_t)-1;
  if (tid < a.head) e = tid;
  else if (tid - a.head < a.n - tail0 && tid >= a.head) e = tail0 + (tid - a.head);
  if (e < a.n) {
    const size_t off = e * sizeof(T);
    const T r = eval_prog<OP, T>(a.p, [&](int j) { return *reinterpret_cast<const T *>(a.src[j] + off); });
#pragma unroll
    for (int d = 0; d < MAXR; d++)
      if (d < a.ndst) store_fields(reinterpret_cast<T *>(a.dst[d] + off), r);
  }
}

typedef int (*fold_launch_fn)(FoldArgs &, hipStream_t);

template <class T, class OP>
int fold_launch(FoldArgs &a, hipStream_t s) {
  constexpr size_t N = (sizeof(T) <= 16 && 16 % sizeof(T) == 0) ? 16 / sizeof(T) : 0;
  bool vec = N > 0 && !has_pad<T>::value;   // padded types: field stores, element path
  uintptr_t m = (uintptr_t)a.src[0] & 15;
  for (int j = 0; j < MAXR; j++)
    if (a.src[j] && ((uintptr_t)a.src[j] & 15) != m) vec = false;
  for (int d = 0; d < a.ndst; d++)
    if (((uintptr_t)a.dst[d] & 15) != m) vec = false;
  if (vec && (m % sizeof(T)) != 0) vec = false;
  if (vec) {
    size_t head = m ? (16 - m) / sizeof(T) : 0;
    if (head > a.n) head = a.n;
    a.head = head;
    a.nvec = (a.n - head) / (N ? N : 1);
  } else {
    a.head = a.n;  // everything scalar (element per lane)
    a.nvec = 0;
  }
  size_t work = a.nvec + a.head + (N ? N : 1);
  if (!vec) work = a.n;
  const size_t g = (work + kFB - 1) / kFB;
  int nsrc = 0;
  for (int j = 0; j < MAXR; j++) nsrc += a.src[j] != nullptr;
  if (vec && (a.nt_force || mx_nt_for((size_t)(nsrc + a.ndst) * a.n * sizeof(T))))
    hipLaunchKernelGGL((k_fold<T, OP, true>), dim3((unsigned)(g ? g : 1)), dim3(kFB), 0, s, a);
  else
    hipLaunchKernelGGL((k_fold<T, OP, false>), dim3((unsigned)(g ? g : 1)), dim3(kFB), 0, s, a);
  return mx_check_launch();
}



// ---------------------------------------------------------------------------
// one-shot allreduce for small messages: ONE launch per call.  Workgroup w
// owns element slice w: it pushes that slice of my contribution into every
// peer's one-shot slot (double-buffered by generation parity), raises READY
// (source=me, slice=w) at each peer, waits for every peer's READY for slice
// w, and folds the slice for the WHOLE vector from the n copies (every rank
// evaluates the same fold program per element, so all ranks agree bit for
// bit).  Reuse of a parity buffer needs the peer to have finished gen-2,
// i.e. DONE >= gen-2; the last workgroup to finish raises DONE(gen).
// ---------------------------------------------------------------------------
struct OsSeg { size_t lo, hi; FoldProg p; };
struct OneShotArgs {
  const char *sb;
  char *rb;
  char *peer_slot[MAXR];        // peer p's buffer (this parity) at my slot; null for me
  const char *src[MAXR];        // operand j: my buffer (this parity) slot j; src[rank] = sb
  uint64_t *peer_ready[MAXR];   // peer p's OS READY row for source = me
  uint64_t *peer_done[MAXR];    // peer p's DONE flag for source = me
  const uint64_t *my_ready;     // my OS READY rows [src][wg]
  const uint64_t *my_done;      // my DONE flags [src]
  uint64_t *counter;
  uint64_t counter_last, gen, timeout_ticks;
  int *err;
  int *poison;
  int n, rank, nseg;
  size_t count, es, slice;
  uint64_t *mflags;             // the blocking call's completion flags (Mark.flags), or null
  uint64_t mv;                  // their sequence number
  int ll;                       // the tagged-word protocol (os_ll): peer_slot / src[p] point at the LL areas
  OsSeg seg[OS_MAXSEG];
};

constexpr int kOSB = 256;

__device__ __forceinline__ void os_spin(const uint64_t *f, uint64_t v, uint64_t ticks, int *err, int *poison) {
  const uint64_t t0 = wall_clock64();
  while (__hip_atomic_load(gp(f), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < v) {
    __builtin_amdgcn_s_sleep(1);
    if (wall_clock64() - t0 > ticks) {
      raise_timeout(err, poison);
      break;
    }
  }
}

// ---------------------------------------------------------------------------
// The tagged-word (LL) variant for one-workgroup calls (4- and 8-byte element
// types, at most OS_LL_MAX bytes per rank): every 4-byte word of my
// contribution travels to each peer as one 8-byte store {gen, word} into the
// LL area of my slot there, so the data is its own READY -- no release fence
// between data and flag, no READY row, no acquire before the fold.  A peer's
// word is taken when its tag reads this generation (stale words carry gen-2
// or older; the LL area is never written by the raw path, so raw bytes can
// never pass for a tag).  Each lane gathers its elements' words from every
// peer into its own LDS column and evaluates the call's fold program there
// (the same program as the raw path: the results are bit for bit the raw
// path's).  DONE(gen) follows once every lane's gathers have returned.  The
// loads and stores are system-scope (L2 bypassed), so the resident service
// (SYS: its operand and result words too) runs with no cache maintenance at
// all.  Returns false when the call failed (poisoned, or a peer timed out).
// ---------------------------------------------------------------------------
constexpr size_t OS_LL_MAX = 4096;         // bytes per rank and workgroup (one slice)
constexpr size_t OS_LL_CAP = 64 << 10;     // bytes per rank of the launched tagged-word class

__device__ __forceinline__ uint64_t ll_ld(const uint64_t *p) {
  return __hip_atomic_load(gp(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// tk (the service's phase trace, or null): thread 0 stamps [0] the gen-2
// check, [1] the push issued, [2] the gather, [3] the fold
// dchk = false: the caller knows every peer is past gen-2 -- it gathered
// every peer's gen-1 words, and a peer starts a call only after its previous
// one (reads of that parity's LL area included) has finished
template <class T, class OP, bool SYS>
__device__ bool os_ll(const OneShotArgs &a, uint64_t *tk = nullptr, bool dchk = true) {
  constexpr int W = (int)(sizeof(T) / 4);
  static_assert(sizeof(T) == 4 || sizeof(T) == 8, "LL carries 4- and 8-byte elements");
  // Roles by wave: waves 0-1 (kG lanes) gather and fold, waves 2-3 push.
  // gfx950 has one vmcnt for loads and stores, so a wave that has pushed
  // must wait for its pushes' acknowledgements before it can use any load
  // issued after them; with the roles split the gathering waves' waits see
  // only their own loads.
  constexpr int kG = kOSB / 2, kP = kOSB - kG;
  constexpr int MW = (int)(OS_LL_MAX / 4 / kP);   // words per pushing lane
  constexpr int ME = (int)(OS_LL_MAX / 4 / kG);   // words per peer and gathering lane
  // gathering lane t's words, [f * kG + t]: at most (MAXR - 1) peers x ME
  __shared__ uint32_t col[(MAXR - 1) * ME * kG];
  __shared__ uint32_t mine[OS_LL_MAX / 4];   // my words, for the fold
  __shared__ int s_bad;
  const int t = threadIdx.x, n = a.n, r = a.rank;
  const uint32_t g = (uint32_t)a.gen;
  const uint64_t tag = (uint64_t)g << 32;
  if (t == 0) s_bad = poisoned(a.poison);
  __syncthreads();
  if (s_bad) return false;
  // this workgroup's slice of the elements, [lo, hi) (the launch: one per
  // OS_LL_MAX bytes; the service: one workgroup, the whole call)
  const size_t lo = (size_t)blockIdx.x * a.slice;
  const size_t hi = lo + a.slice < a.count ? lo + a.slice : a.count;
  const size_t cnt = hi > lo ? hi - lo : 0;
  const int E = (int)((cnt + kG - 1) / kG);   // elements per gathering lane
  const size_t w0 = lo * W, nw = cnt * W;     // this slice's words: [w0, w0 + nw)
  // (2a) the pushing lanes' own words (MW per lane, all loads in flight at
  // once) are loaded before the gen-2 check below, which they overlap
  uint32_t mv[MW];
  if (t >= kG) {
    const int q = t - kG;
    const bool al = ((uintptr_t)a.sb & 3) == 0;
    const uint32_t *sw = reinterpret_cast<const uint32_t *>(a.sb);
#pragma unroll
    for (int u = 0; u < MW; u++) {
      const size_t i = (size_t)q + (size_t)u * kP;
      if (i < nw) {
        if (SYS) mv[u] = __hip_atomic_load(gp(sw + w0 + i), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        else if (al) mv[u] = sw[w0 + i];
        else __builtin_memcpy(&mv[u], a.sb + 4 * (w0 + i), 4);
      }
    }
  }
  // (1) every peer is past gen-2: its reads of this parity's LL area are over
  if (dchk && t < n && t != r && a.gen > 2) os_spin(a.my_done + t, a.gen - 2, a.timeout_ticks, a.err, a.poison);
  __syncthreads();
  if (t == 0) {
    s_bad = poisoned(a.poison);
    if (tk) tk[0] = wall_clock64();
  }
  __syncthreads();
  if (s_bad) return false;
  bool bad = false;
  if (t >= kG) {
    // (2b) my words into LDS for my own operand of the fold, then, tagged,
    // into every peer's LL area
    const int q = t - kG;
#pragma unroll
    for (int u = 0; u < MW; u++) {
      const size_t i = (size_t)q + (size_t)u * kP;
      if (i < nw) mine[i] = mv[u];
    }
    for (int p = 0; p < n; p++) {
      if (p == r) continue;
      uint64_t *d = reinterpret_cast<uint64_t *>(a.peer_slot[p]) + w0;
#pragma unroll
      for (int u = 0; u < MW; u++) {
        const size_t i = (size_t)q + (size_t)u * kP;
        if (i < nw) __hip_atomic_store(gp(d + i), tag | mv[u], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
    }
    if (tk && t == kG) tk[1] = wall_clock64();
  } else {
    // (3) gather: lane t's words of every peer -- E elements (t, t + kG, ...)
    // of W words each -- flattened as f = (peer * E + i) * W + k and loaded
    // eight at a time (all eight in flight), into LDS column t
    const int Lw = (n - 1) * E * W;
    const uint64_t t0 = wall_clock64();
    for (int f0 = 0; f0 < Lw && !bad; f0 += 8) {
      uint64_t v[8];
      const uint64_t *ad[8];
#pragma unroll
      for (int u = 0; u < 8; u++) {
        const int f = f0 + u;
        ad[u] = nullptr;
        if (f < Lw) {
          const int k = f % W, ii = (f / W) % E, jj = f / (W * E);
          const size_t e = lo + (size_t)t + (size_t)ii * kG;
          if (e < hi) {
            ad[u] = reinterpret_cast<const uint64_t *>(a.src[jj < r ? jj : jj + 1]) + e * W + k;
            v[u] = ll_ld(ad[u]);
          }
        }
      }
      // words not yet of this generation are loaded again, all together
      for (;;) {
        bool all = true;
#pragma unroll
        for (int u = 0; u < 8; u++)
          if (ad[u] && (uint32_t)(v[u] >> 32) != g) all = false;
        if (all) break;
        __builtin_amdgcn_s_sleep(1);
        if (wall_clock64() - t0 > a.timeout_ticks) {
          raise_timeout(a.err, a.poison);
          bad = true;
          break;
        }
#pragma unroll
        for (int u = 0; u < 8; u++)
          if (ad[u] && (uint32_t)(v[u] >> 32) != g) v[u] = ll_ld(ad[u]);
      }
#pragma unroll
      for (int u = 0; u < 8; u++)
        if (ad[u]) col[(f0 + u) * kG + t] = (uint32_t)v[u];
    }
  }
  if (bad) s_bad = 1;
  __syncthreads();
  if (s_bad) return false;   // a peer's words never came: no DONE
  if (tk && t == 0) tk[2] = wall_clock64();
  // (4) every lane folds elements t, t + kOSB, ... from the gathering
  // lanes' columns (element e was gathered by lane e % kG, as its e / kG-th)
  {
    int sidx = 0;
    // (SYS: the segment's program copied out of the LDS argument block once
    // per segment -- evaluated from LDS, every step re-read its operand
    // indices, a dependent LDS load per step of every element)
    // (the result pointer, the segment count and bound likewise: loop
    // invariants the compiler would otherwise reload from LDS per element)
    FoldProg P;
    if constexpr (SYS) P = a.seg[0].p;
    const int nseg = a.nseg;
    size_t seg_hi = a.seg[0].hi;
    char *const rbase = a.rb;
    for (size_t e = lo + t; e < hi; e += kOSB) {
      const int gl = (int)((e - lo) % kG), gi = (int)((e - lo) / kG);
      if (sidx + 1 < nseg && e >= seg_hi) {
        while (sidx + 1 < nseg && e >= a.seg[sidx].hi) sidx++;
        seg_hi = a.seg[sidx].hi;
        if constexpr (SYS) P = a.seg[sidx].p;
      }
      const size_t off = e * sizeof(T);
      auto LDo = [&](int j) {
        T x;
        uint32_t u[W];
        if (j != r) {
          const int jj = j < r ? j : j - 1;
#pragma unroll
          for (int k = 0; k < W; k++) u[k] = col[((jj * E + gi) * W + k) * kG + gl];
        } else {
#pragma unroll
          for (int k = 0; k < W; k++) u[k] = mine[(e - lo) * W + k];
        }
        __builtin_memcpy(&x, u, sizeof(T));
        return x;
      };
      // (the bounded evaluation only where the arguments live in LDS: with
      // the launch's by-value arguments its copies would spill them)
      T v;
      if constexpr (SYS) v = eval_prog_small<OP, T>(P, LDo);
      else v = eval_prog<OP, T>(a.seg[sidx].p, LDo);
      if (SYS) {
        uint32_t u[W];
        __builtin_memcpy(u, &v, sizeof(T));
#pragma unroll
        for (int k = 0; k < W; k++)
          __hip_atomic_store(gp(reinterpret_cast<uint32_t *>(rbase) + e * W + k), u[k], __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_SYSTEM);
      } else {
        store_fields(reinterpret_cast<T *>(rbase + off), v);
      }
    }
  }
  if (tk && t == 0) tk[3] = wall_clock64();
  // (5) every gathering lane's loads returned before the barrier above:
  // DONE(gen) at every peer -- with several workgroups, by the last one out
  if (t == 0) {
    bool last = gridDim.x == 1;
    if (!last) last = __hip_atomic_fetch_add(gp(a.counter), (uint64_t)1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
                      a.counter_last;
    if (last)
      for (int p = 0; p < n; p++)
        if (p != r) __hip_atomic_store(gp(a.peer_done[p]), a.gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  return true;
}

// the raw protocol, steps (1)-(6) of k_oneshot; false when the call failed
template <class T, class OP>
__device__ bool os_raw(const OneShotArgs &a) {
  const int w = blockIdx.x, t = threadIdx.x;
  const size_t lo = (size_t)w * a.slice, hi = lo + a.slice < a.count ? lo + a.slice : a.count;
  // poison checks are taken by thread 0 and shared, so the whole workgroup
  // leaves together (no thread may skip a barrier the others reach)
  __shared__ int s_bad;
  if (t == 0) s_bad = poisoned(a.poison);
  __syncthreads();
  if (s_bad) return false;
  // (1) every peer is past gen-2: its reads of this parity buffer are over
  if (t < a.n && t != a.rank && a.gen > 2) os_spin(a.my_done + t, a.gen - 2, a.timeout_ticks, a.err, a.poison);
  __syncthreads();
  if (t == 0) s_bad = poisoned(a.poison);
  __syncthreads();
  if (s_bad) return false;   // a peer never freed its buffer: push nothing
  // (2) push my slice (bytes [lo*es, hi*es)) to every peer
  if (lo < hi) {
    const size_t b0 = lo * a.es, b1 = hi * a.es;
    const bool vec = (((uintptr_t)a.sb | b0 | b1) & 15) == 0;
    for (int p = 0; p < a.n; p++) {
      if (p == a.rank) continue;
      char *d = a.peer_slot[p];
      if (vec) {
        for (size_t i = b0 / 16 + t; i < b1 / 16; i += kOSB)
          reinterpret_cast<uint4 *>(d)[i] = reinterpret_cast<const uint4 *>(a.sb)[i];
      } else {
        for (size_t i = b0 + t; i < b1; i += kOSB) d[i] = a.sb[i];
      }
    }
  }
  __threadfence_system();
  __syncthreads();
  // (3) READY(me, w) at every peer; (4) wait READY(p, w) from every peer
  if (t < a.n && t != a.rank) {   // (the system fence above is the release)
    __hip_atomic_store(a.peer_ready[t] + w, a.gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    os_spin(a.my_ready + (size_t)t * OSWG + w, a.gen, a.timeout_ticks, a.err, a.poison);
  }
  __syncthreads();
  if (t == 0) s_bad = poisoned(a.poison);
  __syncthreads();
  __atomic_thread_fence(__ATOMIC_ACQUIRE);
  if (s_bad) return false;   // stale slots: no fold, and DONE is never raised
  // (5) fold the slice
  int sidx = 0;
  for (size_t e = lo + t; e < hi; e += kOSB) {
    while (sidx + 1 < a.nseg && e >= a.seg[sidx].hi) sidx++;
    const size_t off = e * sizeof(T);
    const T r = eval_prog<OP, T>(a.seg[sidx].p, [&](int j) { return *reinterpret_cast<const T *>(a.src[j] + off); });
    store_fields(reinterpret_cast<T *>(a.rb + off), r);
  }
  // (6) the last workgroup out raises DONE(gen) at every peer
  __syncthreads();
  if (t == 0) {
    __threadfence();
    const uint64_t old = __hip_atomic_fetch_add(a.counter, (uint64_t)1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if (old == a.counter_last) {
      __threadfence_system();
      for (int p = 0; p < a.n; p++)
        if (p != a.rank) __hip_atomic_store(a.peer_done[p], a.gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
  return true;
}

template <class T, class OP>
__global__ void __launch_bounds__(kOSB) k_oneshot(OneShotArgs a) {
  const int w = blockIdx.x, t = threadIdx.x;
  bool ok;
  if constexpr (sizeof(T) == 4 || sizeof(T) == 8)
    ok = a.ll ? os_ll<T, OP, false>(a) : os_raw<T, OP>(a);
  else
    ok = os_raw<T, OP>(a);
  if (!ok) return;
  // (7) a blocking call: every workgroup, once its stores of rb have landed,
  // releases them at system scope and raises its own completion flag (the
  // host waits for the grid's flags instead of a marker kernel, mark_wait)
  if (a.mflags) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (t == 0 && w < (int)kMarkFlags) {
      __threadfence_system();
      __hip_atomic_store(a.mflags + w, (a.mv << 12) | (uint64_t)(gridDim.x - 1), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

typedef int (*oneshot_launch_fn)(OneShotArgs &, int nwg, hipStream_t);

template <class T, class OP>
int oneshot_launch(OneShotArgs &a, int nwg, hipStream_t s) {
  hipLaunchKernelGGL((k_oneshot<T, OP>), dim3(nwg), dim3(kOSB), 0, s, a);
  return mx_check_launch();
}

// ---------------------------------------------------------------------------
// fold VM: arbitrary reduction trees / DAGs with LDS-resident registers.
// Registers 0..nsrc-1 hold the n contributions of this lane's element(s);
// COMB r[d] = OP(r[a], r[b]) (a = target/first operand, b = source); EMIT
// stores r[a] to destination d.  Register j of lane t lives at LDS
// (j * kVB + t) * SLOT, so each lane only touches its own column (no
// barriers) and the uniform register index costs one address add -- where a
// VGPR array indexed by a run-time register number would be spilled to
// scratch or expanded into selects.
// ---------------------------------------------------------------------------
constexpr int kVB = 128;         // VM block size
constexpr int VM_MAXI = 192;     // instructions per program
constexpr int VM_MAXREG = 40;    // registers (contributions + temporaries)
constexpr size_t kVmLdsMax = 160 * 1024;   // LDS per CU, all of it available to one workgroup
// op: VM_COMB / VM_EMIT, optionally guarded by the call's info bit (the
// root's MPI_IN_PLACE in a rooted reduce): executed only if set / clear
enum { VM_COMB = 0, VM_EMIT = 1, VM_IF_SET = 4, VM_IF_CLEAR = 8 };
struct VmIns { int8_t op, d, a, b; };
struct VmProg {
  int nsrc, nregs, nins;
  VmIns ins[VM_MAXI];
};
struct VmArgs {
  const char *src[MAXR];
  char *dst[MAXR];
  size_t n, head, nvec;
  const int *poison;      // communicator poison word (null: local)
  const uint64_t *info;   // READY word carrying the info bit (bit 0), or null
  int info_host;          // info bit when `info` is null
  VmProg p;
};

template <class T> constexpr int vm_slot() { return sizeof(T) > 16 ? (int)sizeof(T) : 16; }

template <class OP, bool NT, bool VEC, class E, int SLOT>
__device__ __forceinline__ void vm_run(const VmArgs &a, char *my, size_t off, int info) {
  auto R = [&](int j) { return reinterpret_cast<E *>(my + (size_t)j * kVB * SLOT); };
  for (int j = 0; j < a.p.nsrc; j++) {
    E v;
    if constexpr (VEC) ld16<NT>(v, reinterpret_cast<const E *>(a.src[j] + off));
    else v = *reinterpret_cast<const E *>(a.src[j] + off);
    *R(j) = v;
  }
  const int skip = info ? VM_IF_CLEAR : VM_IF_SET;
  for (int i = 0; i < a.p.nins; i++) {
    const VmIns in = a.p.ins[i];
    if (in.op & skip) continue;
    if ((in.op & 3) == VM_COMB) {
      const E x = *R(in.a), y = *R(in.b);
      *R(in.d) = comb<OP>(x, y);
    } else {
      const E v = *R(in.a);
      if constexpr (VEC) st16<NT>(reinterpret_cast<E *>(a.dst[in.d] + off), v);
      else store_fields(reinterpret_cast<E *>(a.dst[in.d] + off), v);
    }
  }
}

template <class T, class OP, bool NT>
__global__ void __launch_bounds__(kVB) k_vm(VmArgs a) {
  using V = fvec<T>;
  constexpr int N = V::N;
  constexpr int SLOT = vm_slot<T>();
  extern __shared__ __align__(16) char vm_lds[];
  if (poisoned(a.poison)) return;
  char *const my = vm_lds + (size_t)threadIdx.x * SLOT;
  const size_t tid = (size_t)blockIdx.x * kVB + threadIdx.x;
  const int info = a.info ? (int)(__hip_atomic_load(a.info, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) & 1)
                          : a.info_host;
  if constexpr (N > 0) {
    if (tid < a.nvec) vm_run<OP, NT, true, V, SLOT>(a, my, a.head * sizeof(T) + tid * 16, info);
  }
  const size_t tail0 = a.head + a.nvec * N;
  size_t e = (size_t)-1;
  if (tid < a.head) e = tid;
  else if (tid >= a.head && tid - a.head < a.n - tail0) e = tail0 + (tid - a.head);
  if (e < a.n) vm_run<OP, false, false, T, SLOT>(a, my, e * sizeof(T), info);
}

typedef int (*vm_launch_fn)(VmArgs &, hipStream_t);

template <class T, class OP>
int vm_launch(VmArgs &a, hipStream_t s) {
  constexpr size_t N = (sizeof(T) <= 16 && 16 % sizeof(T) == 0) ? 16 / sizeof(T) : 0;
  // a gfx950 workgroup may take the whole 160 KiB of its CU's LDS; above the
  // 64 KiB default the kernel has to opt in (x87 pair types at 16 ranks:
  // ~20 registers x 128 lanes x 32 B)
  const size_t lds = (size_t)a.p.nregs * kVB * vm_slot<T>();
  if (lds > kVmLdsMax || a.p.nregs > VM_MAXREG || a.p.nins > VM_MAXI) return MX_ERR_UNSUPPORTED;
  if (lds > 64 * 1024) {
    static const bool opted = [] {
      return hipFuncSetAttribute(reinterpret_cast<const void *>(&k_vm<T, OP, true>),
                                 hipFuncAttributeMaxDynamicSharedMemorySize, (int)kVmLdsMax) == hipSuccess &&
             hipFuncSetAttribute(reinterpret_cast<const void *>(&k_vm<T, OP, false>),
                                 hipFuncAttributeMaxDynamicSharedMemorySize, (int)kVmLdsMax) == hipSuccess;
    }();
    if (!opted) return MX_ERR_UNSUPPORTED;
  }
  bool vec = N > 0 && !has_pad<T>::value;
  const uintptr_t m = (uintptr_t)a.src[0] & 15;
  for (int j = 0; j < a.p.nsrc; j++)
    if (((uintptr_t)a.src[j] & 15) != m) vec = false;
  for (int i = 0; i < a.p.nins; i++)
    if ((a.p.ins[i].op & 3) == VM_EMIT && ((uintptr_t)a.dst[a.p.ins[i].d] & 15) != m) vec = false;
  if (vec && (m % sizeof(T)) != 0) vec = false;
  if (vec) {
    size_t head = m ? (16 - m) / sizeof(T) : 0;
    if (head > a.n) head = a.n;
    a.head = head;
    a.nvec = (a.n - head) / (N ? N : 1);
  } else {
    a.head = a.n;
    a.nvec = 0;
  }
  const size_t work = vec ? a.nvec + a.head + N : a.n;
  const size_t g = (work + kVB - 1) / kVB;
  int nemit = 0;
  for (int i = 0; i < a.p.nins; i++) nemit += (a.p.ins[i].op & 3) == VM_EMIT;
  if (vec && mx_nt_for((size_t)(a.p.nsrc + nemit) * a.n * sizeof(T)))
    hipLaunchKernelGGL((k_vm<T, OP, true>), dim3((unsigned)(g ? g : 1)), dim3(kVB), lds, s, a);
  else
    hipLaunchKernelGGL((k_vm<T, OP, false>), dim3((unsigned)(g ? g : 1)), dim3(kVB), lds, s, a);
  return mx_check_launch();
}

// ---------------------------------------------------------------------------
// per-(op, type) launchers, instantiated by element-type family
// ---------------------------------------------------------------------------
struct FoldFns {
  fold_launch_fn fold;
  oneshot_launch_fn oneshot;
  vm_launch_fn vm;
};

// family of an element type: 0 8/16-bit integers, 1 32/64-bit integers,
// 2 float / double / complex, 3 x87 long double (+ complex), 4 pair types
template <class T> struct fam { static constexpr int value = sizeof(T) <= 2 ? 0 : 1; };
template <> struct fam<float> { static constexpr int value = 2; };
template <> struct fam<double> { static constexpr int value = 2; };
template <> struct fam<cplx<float>> { static constexpr int value = 2; };
template <> struct fam<cplx<double>> { static constexpr int value = 2; };
template <> struct fam<x87> { static constexpr int value = 3; };
template <> struct fam<x87c> { static constexpr int value = 3; };
template <class V, class K> struct fam<pair_t<V, K>> { static constexpr int value = 4; };
template <> struct fam<x87_pair> { static constexpr int value = 4; };
constexpr int NFAM = 5;

template <int F>
struct FamVisitor {
  template <class T, class OP2, class OP3> FoldFns go() {
    if constexpr (fam<T>::value == F)
      return FoldFns{&fold_launch<T, OP2>, &oneshot_launch<T, OP2>, &vm_launch<T, OP2>};
    else
      return FoldFns{nullptr, nullptr, nullptr};
  }
  FoldFns none() { return FoldFns{nullptr, nullptr, nullptr}; }
};

// defined in mx_fold_f<F>.hip
FoldFns fold_fns_fam0(int op, int type);
FoldFns fold_fns_fam1(int op, int type);
FoldFns fold_fns_fam2(int op, int type);
FoldFns fold_fns_fam3(int op, int type);
FoldFns fold_fns_fam4(int op, int type);

inline FoldFns fold_fns(int op, int type) {
  FoldFns (*const f[NFAM])(int, int) = {fold_fns_fam0, fold_fns_fam1, fold_fns_fam2, fold_fns_fam3,
                                         fold_fns_fam4};
  for (int i = 0; i < NFAM; i++) {
    const FoldFns r = f[i](op, type);
    if (r.fold) return r;
  }
  return FoldFns{nullptr, nullptr, nullptr};
}

}  // namespace mx
