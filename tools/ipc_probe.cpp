// ipc_probe.cpp -- diagnostic (not product): does a HIP IPC export made
// AFTER a process imported peers' buffers map correctly in the importers?
// N processes (fork before any HIP call) on device 0 exchange handles through
// files under gpurun_out/ipcprobe and read each exporter's signature back
// through every mapping.  Phases: A = uncached 1 MiB (exported before any
// import, like mx_comm_create's staging), B = uncached 64 MiB and
// C = plain hipMalloc 64 MiB (both exported after phase A's imports).
#include <hip/hip_runtime.h>
#include <sys/stat.h>
#include <sys/wait.h>
#include <unistd.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

static const char *kDir = "gpurun_out/ipcprobe";

static void put_file(const std::string &name, const void *data, size_t n) {
  std::string tmp = std::string(kDir) + "/" + name + ".tmp", fin = std::string(kDir) + "/" + name;
  FILE *f = fopen(tmp.c_str(), "wb");
  fwrite(data, 1, n, f);
  fclose(f);
  rename(tmp.c_str(), fin.c_str());
}
static void get_file(const std::string &name, void *data, size_t n) {
  std::string fin = std::string(kDir) + "/" + name;
  for (int i = 0; i < 200000; i++) {
    FILE *f = fopen(fin.c_str(), "rb");
    if (f) {
      size_t got = fread(data, 1, n, f);
      fclose(f);
      if (got == n) return;
    }
    usleep(1000);
  }
  fprintf(stderr, "timeout waiting for %s\n", fin.c_str());
  exit(2);
}

static void *g_maps[64];
static int g_nmaps;
static char *g_own;

static int phase(int rank, int n, const char *tag, size_t bytes, bool uncached, bool keep = true) {
  char *buf = nullptr;
  hipError_t e = uncached ? hipExtMallocWithFlags((void **)&buf, bytes, hipDeviceMallocUncached)
                          : hipMalloc((void **)&buf, bytes);
  if (e != hipSuccess) { printf("rank %d %s alloc failed\n", rank, tag); return 1; }
  unsigned long long sig = 0x5EED0000ull + (unsigned long long)rank;
  hipMemcpy(buf, &sig, 8, hipMemcpyHostToDevice);
  hipDeviceSynchronize();
  hipIpcMemHandle_t h;
  if (hipIpcGetMemHandle(&h, buf) != hipSuccess) { printf("rank %d %s export failed\n", rank, tag); return 1; }
  put_file(std::string(tag) + "_" + std::to_string(rank), &h, sizeof h);
  int bad = 0;
  for (int p = 0; p < n; p++) {
    if (p == rank) continue;
    hipIpcMemHandle_t ph;
    get_file(std::string(tag) + "_" + std::to_string(p), &ph, sizeof ph);
    void *m = nullptr;
    if (hipIpcOpenMemHandle(&m, ph, hipIpcMemLazyEnablePeerAccess) != hipSuccess) {
      printf("rank %d %s: open of PE %d failed\n", rank, tag, p);
      bad++;
      continue;
    }
    unsigned long long v = 0;
    hipMemcpy(&v, m, 8, hipMemcpyDeviceToHost);
    if (!keep) g_maps[g_nmaps++] = m;
    printf("rank %d %s: PE %d -> %p reads %llx %s\n", rank, tag, p, m, v, v == 0x5EED0000ull + p ? "ok" : "WRONG");
    bad += v != 0x5EED0000ull + p;
  }
  fflush(stdout);
  int done = 1;
  put_file(std::string(tag) + "_done_" + std::to_string(rank), &done, sizeof done);
  for (int p = 0; p < n; p++) get_file(std::string(tag) + "_done_" + std::to_string(p), &done, sizeof done);
  if (!keep) {   // like mx_heap_destroy: close the imports, free my buffer
    for (int i = 0; i < g_nmaps; i++) hipIpcCloseMemHandle(g_maps[i]);
    g_nmaps = 0;
    hipFree(buf);
  }
  return bad;
}

int main(int argc, char **argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 3;
  mkdir("gpurun_out", 0755);
  mkdir(kDir, 0755);
  for (int r = 0; r < n; r++) {
    if (fork() == 0) {
      hipSetDevice(0);
      int bad = phase(r, n, "A", 1 << 20, true);
      bad += phase(r, n, "A2", 4096, true);            // mx_comm_create: staging + flag words
      // churn like a torch process: allocations of assorted sizes, some freed
      void *keepers[64];
      for (int i = 0; i < 64; i++) {
        void *q = nullptr;
        hipMalloc(&q, (size_t)((i * 7919) % 97 + 1) << 16);
        keepers[i] = q;
        if (i % 3 == 0) { hipFree(q); keepers[i] = nullptr; }
      }
      bad += phase(r, n, "B", (64 << 20) + 4096, true, false);   // heap 1 (unaligned size), destroyed
      bad += phase(r, n, "B2", (64 << 20) + 4096, true, false);  // heap 2
      bad += phase(r, n, "B3", (8 << 20) + 4096, true, false);
      bad += phase(r, n, "C", 64 << 20, false);
      bad += phase(r, n, "D", 1 << 20, true);
      for (int i = 0; i < 64; i++) if (keepers[i]) hipFree(keepers[i]);
      printf("rank %d: %d wrong mappings\n", r, bad);
      fflush(stdout);
      _exit(bad ? 1 : 0);
    }
  }
  int fails = 0, st = 0;
  for (int r = 0; r < n; r++) {
    wait(&st);
    fails += !(WIFEXITED(st) && WEXITSTATUS(st) == 0);
  }
  printf("%d of %d processes saw wrong mappings\n", fails, n);
  return 0;
}
