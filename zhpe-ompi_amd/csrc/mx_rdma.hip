// mx_rdma.hip -- one-sided device copies between processes of a node
// (include/mx_rdma.h): the data mover behind the BTL's get / put slots
// (mca/btl_mi355x.c), the role btl/smcuda's CUDA IPC get plays in the
// reference (btl_smcuda.c:1077-1180).
//
// Registration exports the IPC handle of the allocation that holds a range
// (once per allocation; the runtime buffer id tells a live allocation from
// one re-made at the same address).  A peer maps the allocation once and
// keeps the mapping in a process-wide cache; a copy is one streaming copy
// kernel (copy_async, 16-byte non-temporal accesses at large sizes).  A get
// reads memory another GPU wrote, so an acquire kernel runs first: one
// workgroup per XCD slot takes a system-scope acquire, dropping lines of an
// earlier get from every XCD's L2 (the rule of the zero-copy collectives,
// DESIGN 7.1 rule 3).  Mappings are closed through the deferred release
// (release_later): hipIpcCloseMemHandle waits for every stream of the device.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>
#include <unistd.h>

#include <mutex>
#include <vector>

#include "mx_internal.h"
#include "../../include/mx_rdma.h"

using namespace mx;

struct mx_rdma_op {
  hipEvent_t ev;
};

namespace {

constexpr int kAcqBlocks = 16;        // two per XCD (workgroups are dealt round-robin over the 8 XCDs)
constexpr size_t kMaxImports = 64;

__global__ void k_rdma_acquire() {
  if (threadIdx.x == 0) __atomic_thread_fence(__ATOMIC_ACQUIRE);   // system scope: buffer_inv sc0 sc1
}

struct Import {
  int32_t pid;
  uint64_t base, size, id;
  char *ptr;
  uint64_t used;
};

std::mutex g_mu;
std::vector<Import> g_imp;
std::vector<IpcGone> g_gone;          // the imports closed (ipc_open_checked)
uint64_t g_tick;
hipStream_t g_stream;
std::vector<hipEvent_t> g_ev_free;

struct Export { uint64_t base, size, id; hipIpcMemHandle_t h; };
std::vector<Export> g_exp;            // most recent last, at most 16

// a blocking stream: implicitly after the work already queued on the legacy
// default stream (a receive buffer the application just zeroed or wrote
// there is written by the get only after that), with no event per call
hipStream_t rdma_stream() {
  if (!g_stream && hipStreamCreateWithFlags(&g_stream, hipStreamDefault) != hipSuccess) {
    (void)hipGetLastError();
    g_stream = nullptr;
  }
  return g_stream;
}

// the peer allocation described by h, mapped here (caller holds g_mu)
int import_locked(const mx_rdma_handle_t &h, char **out) {
  if (h.pid == (int32_t)getpid()) {   // this process's own allocation
    *out = (char *)(uintptr_t)h.base;
    return MX_SUCCESS;
  }
  for (Import &m : g_imp)
    if (m.pid == h.pid && m.base == h.base && m.size == h.size && m.id == h.id) {
      m.used = ++g_tick;
      *out = m.ptr;
      return MX_SUCCESS;
    }
  for (size_t i = 0; i < g_imp.size();) {
    Import &m = g_imp[i];
    if (m.pid == h.pid && m.base < h.base + h.size && h.base < m.base + m.size) {
      // the owner freed that allocation and made another in its place: the
      // stale import must be closed before the new handle is opened; while
      // the device is not quiet it stays cached and the call is retried
      ipc_gone_add(g_gone, m.pid, m.base, m.size, m.ptr);
      if (!release_now_or_keep(m.ptr, REL_IPC)) return MX_ERR_STATE;
      g_imp.erase(g_imp.begin() + (long)i);
      continue;
    }
    i++;
  }
  if (g_imp.size() >= kMaxImports) {
    size_t lru = 0;
    for (size_t i = 1; i < g_imp.size(); i++)
      if (g_imp[i].used < g_imp[lru].used) lru = i;
    ipc_gone_add(g_gone, g_imp[lru].pid, g_imp[lru].base, g_imp[lru].size, g_imp[lru].ptr);
    release_later(g_imp[lru].ptr, REL_IPC);
    g_imp.erase(g_imp.begin() + (long)lru);
  }
  // checked against the imports closed at that range: the runtime may hand
  // one back (then MX_ERR_STATE: the caller's fallback, as a busy device)
  char *p = nullptr;
  uint64_t oid = 0;
  const int oc = ipc_open_checked(h.ipc, g_gone, h.pid, h.base, h.size, &p, &oid);
  if (oc < 0) return oc;
  if (oc == 0) return MX_ERR_STATE;
  g_imp.push_back(Import{h.pid, h.base, h.size, h.id, p, ++g_tick});
  *out = p;
  return MX_SUCCESS;
}

int op_new(hipStream_t s, mx_rdma_op_t **op) {
  mx_rdma_op_t *o = new (std::nothrow) mx_rdma_op_t;
  if (!o) return MX_ERR_NOMEM;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    if (!g_ev_free.empty()) {
      o->ev = g_ev_free.back();
      g_ev_free.pop_back();
    } else if (hipEventCreateWithFlags(&o->ev, hipEventDisableTiming) != hipSuccess) {
      delete o;
      return MX_ERR_HIP;
    }
  }
  if (hipEventRecord(o->ev, s) != hipSuccess) {
    mx_rdma_op_free(o);
    return MX_ERR_HIP;
  }
  *op = o;
  return MX_SUCCESS;
}

int rdma_copy(void *dst_local, const void *src_local, const mx_rdma_handle_t *remote, uint64_t remote_addr,
              size_t bytes, void *stream, mx_rdma_op_t **op, bool get) {
  if (!remote || (!dst_local && get) || (!src_local && !get)) return MX_ERR_ARG;
  if (remote_addr < remote->base || remote_addr + bytes > remote->base + remote->size) return MX_ERR_ARG;
  if (int rc = mx_ensure_init()) return rc;
  if (op) *op = nullptr;
  char *map = nullptr;
  hipStream_t s = (hipStream_t)stream;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    if (int rc = import_locked(*remote, &map)) return rc;
    if (!s && !(s = rdma_stream())) return MX_ERR_HIP;
  }
  char *rp = map + (remote_addr - remote->base);
  if (bytes) {
    if (get) {
      hipLaunchKernelGGL(k_rdma_acquire, dim3(kAcqBlocks), dim3(64), 0, s);
      if (int rc = mx_check_launch()) return rc;
      if (int rc = copy_async(dst_local, rp, bytes, s)) return rc;
    } else if (int rc = copy_async(rp, src_local, bytes, s)) {
      return rc;
    }
  }
  return op ? op_new(s, op) : MX_SUCCESS;
}

}  // namespace

// the pull of a single-copy rendezvous receive (mx_p2p.hip): a get with no
// completion event (the caller's next kernel on `stream` follows it)
int mx::rdma_pull(void *local, const mx_rdma_handle_t *remote, uint64_t remote_addr, size_t bytes, hipStream_t s) {
  return rdma_copy(local, nullptr, remote, remote_addr, bytes, s, nullptr, true);
}

extern "C" int mx_rdma_register(const void *ptr, size_t bytes, mx_rdma_handle_t *h) {
  if (!ptr || !h) return MX_ERR_ARG;
  if (int rc = mx_ensure_init()) return rc;
  void *base = nullptr;
  size_t size = 0;
  unsigned long long id = 0;
  if (hipMemGetAddressRange(&base, &size, const_cast<void *>(ptr)) != hipSuccess || !base ||
      (const char *)ptr + bytes > (const char *)base + size ||
      hipPointerGetAttribute(&id, HIP_POINTER_ATTRIBUTE_BUFFER_ID, (hipDeviceptr_t)base) != hipSuccess) {
    (void)hipGetLastError();
    return MX_ERR_ARG;                 // not one device allocation
  }
  memset(h, 0, sizeof *h);
  std::lock_guard<std::mutex> lk(g_mu);
  bool hit = false;
  for (const Export &e : g_exp)
    if (e.base == (uint64_t)(uintptr_t)base && e.size == size && e.id == id) {
      memcpy(h->ipc, &e.h, sizeof e.h);
      hit = true;
      break;
    }
  if (!hit) {
    if (export_remade((uint64_t)(uintptr_t)base, size, id)) return MX_ERR_UNSUPPORTED;   // 
    hipIpcMemHandle_t ih;
    if (hipIpcGetMemHandle(&ih, base) != hipSuccess) {
      (void)hipGetLastError();
      return MX_ERR_HIP;
    }
    if (g_exp.size() >= 16) g_exp.erase(g_exp.begin());
    g_exp.push_back(Export{(uint64_t)(uintptr_t)base, size, id, ih});
    memcpy(h->ipc, &ih, sizeof ih);
  }
  h->base = (uint64_t)(uintptr_t)base;
  h->size = size;
  h->id = id;
  h->pid = (int32_t)getpid();
  h->device = g_device;
  return MX_SUCCESS;
}

extern "C" int mx_rdma_get(void *local, const mx_rdma_handle_t *remote, uint64_t remote_addr, size_t bytes,
                           void *stream, mx_rdma_op_t **op) {
  if (!op) return MX_ERR_ARG;
  return rdma_copy(local, nullptr, remote, remote_addr, bytes, stream, op, true);
}

extern "C" int mx_rdma_put(const void *local, const mx_rdma_handle_t *remote, uint64_t remote_addr, size_t bytes,
                           void *stream, mx_rdma_op_t **op) {
  if (!op) return MX_ERR_ARG;
  return rdma_copy(nullptr, local, remote, remote_addr, bytes, stream, op, false);
}

extern "C" int mx_rdma_test(mx_rdma_op_t *op) {
  if (!op) return MX_ERR_ARG;
  const hipError_t e = hipEventQuery(op->ev);
  if (e == hipSuccess) return 1;
  (void)hipGetLastError();
  return e == hipErrorNotReady ? 0 : MX_ERR_HIP;
}

extern "C" int mx_rdma_wait(mx_rdma_op_t *op) {
  if (!op) return MX_ERR_ARG;
  return mx_hip_rc(hipEventSynchronize(op->ev));
}

extern "C" int mx_rdma_op_free(mx_rdma_op_t *op) {
  if (!op) return MX_SUCCESS;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    g_ev_free.push_back(op->ev);
  }
  delete op;
  return MX_SUCCESS;
}

extern "C" int mx_rdma_mapped(void) {
  std::lock_guard<std::mutex> lk(g_mu);
  return (int)g_imp.size();
}
