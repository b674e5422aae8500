// ipc_realloc_probe -- does an allocation freed and re-made at the same
// address get a different IPC handle / runtime buffer id?  (The zero-copy
// import cache keys on them)  Then, in a child process: open the
// first handle, read it, close; open the second one and read again -- does
// the import show the new allocation's contents?
// build: hipcc --offload-arch=gfx950 -O2 -o /tmp/ipc_realloc_probe tools/ipc_realloc_probe.cpp
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <string.h>
#include <sys/wait.h>
#include <unistd.h>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      printf("%s:%d %s -> %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      return 1;                                                                \
    }                                                                          \
  } while (0)

struct Rec { hipIpcMemHandle_t h; unsigned long long id; void *va; unsigned v; };

static int export_one(size_t bytes, unsigned v, Rec *r, void **keep) {
  void *p = nullptr;
  CK(hipMalloc(&p, bytes));
  CK(hipMemset(p, (int)v, bytes));
  CK(hipDeviceSynchronize());
  CK(hipIpcGetMemHandle(&r->h, p));
  CK(hipPointerGetAttribute(&r->id, HIP_POINTER_ATTRIBUTE_BUFFER_ID, (hipDeviceptr_t)p));
  r->va = p;
  r->v = v;
  *keep = p;
  return 0;
}

int main() {
  const size_t bytes = 256u << 20;
  int pipefd[2], back[2];
  if (pipe(pipefd) || pipe(back)) return 1;
  const pid_t pid = fork();   // before any HIP call in the parent
  if (pid == 0) {
    // importer: receives the two records and reports the byte each mapping reads;
    // the first mapping stays open while the second handle is opened (what
    // a handle-keyed cache would do), then both are read and closed
    CK(hipSetDevice(0));
    void *m[2] = {nullptr, nullptr};
    hipError_t e[2];
    for (int k = 0; k < 2; k++) {
      Rec r;
      if (read(pipefd[0], &r, sizeof r) != (ssize_t)sizeof r) return 1;
      e[k] = hipIpcOpenMemHandle(&m[k], r.h, hipIpcMemLazyEnablePeerAccess);
      for (int j = 0; j <= k; j++) {
        unsigned char b = 0;
        if (e[j] == hipSuccess) CK(hipMemcpy(&b, m[j], 1, hipMemcpyDeviceToHost));
        printf("after import %d: mapping %d (open=%s, %p) reads 0x%02x; exporter's current value 0x%02x\n", k, j,
               hipGetErrorString(e[j]), m[j], b, r.v & 0xff);
      }
      fflush(stdout);
      const char ok = 1;
      if (write(back[1], &ok, 1) != 1) return 1;
    }
    for (int k = 0; k < 2; k++)
      if (e[k] == hipSuccess) (void)hipIpcCloseMemHandle(m[k]);
    return 0;
  }
  CK(hipSetDevice(0));
  Rec a, b;
  void *pa = nullptr, *pb = nullptr;
  if (export_one(bytes, 0x11, &a, &pa)) return 1;
  if (write(pipefd[1], &a, sizeof a) != (ssize_t)sizeof a) return 1;
  char ok;
  if (read(back[0], &ok, 1) != 1) return 1;
  CK(hipFree(pa));
  if (export_one(bytes, 0x22, &b, &pb)) return 1;
  printf("first  va=%p id=%llu\nsecond va=%p id=%llu\nsame va: %d, same handle bytes: %d, same id: %d\n", a.va, a.id,
         b.va, b.id, a.va == b.va, !memcmp(&a.h, &b.h, sizeof a.h), a.id == b.id);
  fflush(stdout);
  if (write(pipefd[1], &b, sizeof b) != (ssize_t)sizeof b) return 1;
  if (read(back[0], &ok, 1) != 1) return 1;
  int st = 0;
  waitpid(pid, &st, 0);
  CK(hipFree(pb));
  return WIFEXITED(st) ? WEXITSTATUS(st) : 1;
}
