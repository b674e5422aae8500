// ipc_alias_probe.cpp -- diagnostic (not product): can hipIpcOpenMemHandle
// hand a process its OWN buffer when a peer's exported buffer sits at the
// same virtual address as one of the importer's live allocations?
//
// Round-1 finding: with 3-4 processes on one GPU, a heap
// exported after the processes had imported each other's staging sometimes
// opened as the importer's own heap.  The ranks are replicas running the
// same allocation sequence, so their buffers usually share virtual
// addresses, and the handle carries the exporter's virtual address
// (profiles/r02/ipc_handle_probe.txt).  This probe replays the sequence with
// N processes (forked before any HIP call) and reports, for every import,
// whose signature the mapping shows and whether the importer had a live
// allocation at the exporter's address:
//   step 1  every rank allocates S (4 MiB uncached), exports, imports all peers' S
//   step 2  every rank allocates H (8 MiB uncached), exports, imports all peers' H
//   step 3  every rank frees H, allocates H2 (same size: VA reuse), exports,
//           imports all peers' H2 (their earlier H imports closed first)
#include <hip/hip_runtime.h>
#include <sys/stat.h>
#include <sys/wait.h>
#include <unistd.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

static const char *kDir = "gpurun_out/ipcalias";
constexpr int N = 3;

static void put_file(const std::string &name, const void *data, size_t n) {
  std::string tmp = std::string(kDir) + "/" + name + ".tmp", fin = std::string(kDir) + "/" + name;
  FILE *f = fopen(tmp.c_str(), "wb");
  fwrite(data, 1, n, f);
  fclose(f);
  rename(tmp.c_str(), fin.c_str());
}
static void get_file(const std::string &name, void *data, size_t n) {
  std::string fin = std::string(kDir) + "/" + name;
  for (int i = 0; i < 60000; i++) {
    FILE *f = fopen(fin.c_str(), "rb");
    if (f) {
      size_t got = fread(data, 1, n, f);
      fclose(f);
      if (got == n) return;
    }
    usleep(1000);
  }
  fprintf(stderr, "timeout waiting for %s\n", fin.c_str());
  _exit(2);
}

static uint64_t sig(int step, int rank) { return 0x5EED000000ull + (uint64_t)step * 0x100 + (uint64_t)rank; }

// one exchange step: allocate (unless `buf` given), sign, export, import every peer's
static void step(int rank, int s, size_t bytes, char **buf, void **imp) {
  if (!*buf) hipExtMallocWithFlags((void **)buf, bytes, hipDeviceMallocUncached);
  const uint64_t v = sig(s, rank);
  hipMemcpy(*buf, &v, 8, hipMemcpyHostToDevice);
  hipDeviceSynchronize();
  hipIpcMemHandle_t h;
  hipIpcGetMemHandle(&h, *buf);
  put_file("s" + std::to_string(s) + "_r" + std::to_string(rank), &h, sizeof h);
  for (int p = 0; p < N; p++) {
    if (p == rank) continue;
    hipIpcMemHandle_t hp;
    get_file("s" + std::to_string(s) + "_r" + std::to_string(p), &hp, sizeof hp);
    const void *peer_va = *reinterpret_cast<void *const *>(&hp);   // first handle word: exporter VA
    hipPointerAttribute_t at;
    const bool mine = hipPointerGetAttributes(&at, peer_va) == hipSuccess && at.type == hipMemoryTypeDevice;
    (void)hipGetLastError();
    void *m = nullptr;
    const hipError_t e = hipIpcOpenMemHandle(&m, hp, hipIpcMemLazyEnablePeerAccess);
    uint64_t got = 0;
    if (e == hipSuccess) hipMemcpy(&got, m, 8, hipMemcpyDeviceToHost);
    const char *verdict = got == sig(s, p) ? "peer's" : got == v ? "OWN (aliased)" : "other";
    printf("step %d rank %d <- %d: my buf %p, peer VA %p (%s at that VA here), map %p rc %d reads %llx = %s\n", s,
           rank, p, (void *)*buf, peer_va, mine ? "live allocation" : "nothing", m, (int)e,
           (unsigned long long)got, verdict);
    fflush(stdout);
    imp[p] = m;
  }
  int one = 1;
  put_file("done" + std::to_string(s) + "_r" + std::to_string(rank), &one, sizeof one);
  for (int p = 0; p < N; p++) get_file("done" + std::to_string(s) + "_r" + std::to_string(p), &one, sizeof one);
}

static int run(int rank) {
  hipSetDevice(0);
  char *S = nullptr, *H = nullptr, *H2 = nullptr;
  void *impS[N] = {}, *impH[N] = {}, *impH2[N] = {};
  step(rank, 1, 4 << 20, &S, impS);
  step(rank, 2, 8 << 20, &H, impH);
  for (int p = 0; p < N; p++)
    if (impH[p]) hipIpcCloseMemHandle(impH[p]);
  hipFree(H);
  step(rank, 3, 8 << 20, &H2, impH2);
  for (int p = 0; p < N; p++) {
    if (impS[p]) hipIpcCloseMemHandle(impS[p]);
    if (impH2[p]) hipIpcCloseMemHandle(impH2[p]);
  }
  hipFree(S);
  hipFree(H2);
  return 0;
}

int main() {
  mkdir("gpurun_out", 0755);
  mkdir(kDir, 0755);
  pid_t kids[N];
  for (int r = 1; r < N; r++) {
    kids[r] = fork();
    if (kids[r] == 0) _exit(run(r));
  }
  run(0);
  int bad = 0;
  for (int r = 1; r < N; r++) {
    int st = 0;
    waitpid(kids[r], &st, 0);
    if (!WIFEXITED(st) || WEXITSTATUS(st)) bad = 1;
  }
  printf("children %s\n", bad ? "FAILED" : "ok");
  return bad;
}
