// ipc_handle_probe.cpp -- diagnostic (not product): what does a HIP IPC
// handle carry in the dmabuf IPC mode (HSA_ENABLE_IPC_MODE_LEGACY=0), and
// which file descriptors does exporting / importing create and keep?
// Two processes (forked before any HIP call) on device 0:
//   A: allocates two uncached buffers, exports each (twice for the first),
//      dumps the handle words and its fd table after every step;
//   B: imports both handles, reads the signatures, dumps its fd table,
//      closes the imports, dumps again;
//   A: frees buffer 1, allocates buffer 3, exports it, dumps fds + handle.
// Question under test: the handle names an exporter fd; if that
// fd number could be closed and reused (e.g. by an import of a peer's
// buffer) before every importer attached, an importer would map whatever now
// sits behind the number -- possibly its own buffer.
#include <dirent.h>
#include <hip/hip_runtime.h>
#include <sys/stat.h>
#include <sys/wait.h>
#include <unistd.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

static const char *kDir = "gpurun_out/ipchandle";

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

static void dump_fds(const char *who, const char *when) {
  printf("[%s] fds %s:", who, when);
  DIR *d = opendir("/proc/self/fd");
  if (!d) { printf(" (no /proc)\n"); return; }
  while (dirent *e = readdir(d)) {
    if (e->d_name[0] == '.') continue;
    char path[64], target[256];
    snprintf(path, sizeof path, "/proc/self/fd/%s", e->d_name);
    ssize_t k = readlink(path, target, sizeof target - 1);
    if (k < 0) continue;
    target[k] = 0;
    if (strstr(target, "dmabuf") || strstr(target, "kfd") || strstr(target, "dri") || strstr(target, "anon_inode"))
      printf(" %s->%s", e->d_name, target);
  }
  closedir(d);
  printf("\n");
  fflush(stdout);
}

static void dump_handle(const char *who, const char *what, const hipIpcMemHandle_t &h) {
  const uint32_t *w = reinterpret_cast<const uint32_t *>(&h);
  printf("[%s] handle %s (pid %d):", who, what, (int)getpid());
  for (size_t i = 0; i < sizeof h / 4; i++) printf(" %08x", w[i]);
  printf("\n");
  fflush(stdout);
}

int main() {
  mkdir("gpurun_out", 0755);
  mkdir(kDir, 0755);
  const pid_t pb = fork();
  if (pb == 0) {   // B: importer
    hipSetDevice(0);
    dump_fds("B", "after init");
    hipIpcMemHandle_t h1, h2;
    get_file("h1", &h1, sizeof h1);
    get_file("h2", &h2, sizeof h2);
    void *m1 = nullptr, *m2 = nullptr;
    const hipError_t e1 = hipIpcOpenMemHandle(&m1, h1, hipIpcMemLazyEnablePeerAccess);
    const hipError_t e2 = hipIpcOpenMemHandle(&m2, h2, hipIpcMemLazyEnablePeerAccess);
    unsigned long long v1 = 0, v2 = 0;
    if (e1 == hipSuccess) hipMemcpy(&v1, m1, 8, hipMemcpyDeviceToHost);
    if (e2 == hipSuccess) hipMemcpy(&v2, m2, 8, hipMemcpyDeviceToHost);
    printf("[B] open h1 -> %p rc %d reads %llx; open h2 -> %p rc %d reads %llx\n", m1, (int)e1, v1, m2, (int)e2, v2);
    dump_fds("B", "after two imports");
    if (m1) hipIpcCloseMemHandle(m1);
    if (m2) hipIpcCloseMemHandle(m2);
    dump_fds("B", "after closing both");
    int done = 1;
    put_file("b_done", &done, sizeof done);
    hipIpcMemHandle_t h3;
    get_file("h3", &h3, sizeof h3);
    void *m3 = nullptr;
    const hipError_t e3 = hipIpcOpenMemHandle(&m3, h3, hipIpcMemLazyEnablePeerAccess);
    unsigned long long v3 = 0;
    if (e3 == hipSuccess) hipMemcpy(&v3, m3, 8, hipMemcpyDeviceToHost);
    printf("[B] open h3 -> %p rc %d reads %llx\n", m3, (int)e3, v3);
    dump_fds("B", "after import 3");
    if (m3) hipIpcCloseMemHandle(m3);
    put_file("b_done3", &done, sizeof done);
    fflush(stdout);
    _exit(0);
  }
  // A: exporter
  hipSetDevice(0);
  dump_fds("A", "after init");
  char *b1 = nullptr, *b2 = nullptr, *b3 = nullptr;
  hipExtMallocWithFlags((void **)&b1, 4 << 20, hipDeviceMallocUncached);
  hipExtMallocWithFlags((void **)&b2, 4 << 20, hipDeviceMallocUncached);
  const unsigned long long s1 = 0x5EED0001ull, s2 = 0x5EED0002ull, s3 = 0x5EED0003ull;
  hipMemcpy(b1, &s1, 8, hipMemcpyHostToDevice);
  hipMemcpy(b2, &s2, 8, hipMemcpyHostToDevice);
  hipDeviceSynchronize();
  printf("[A] b1 %p b2 %p\n", (void *)b1, (void *)b2);
  dump_fds("A", "after allocs");
  hipIpcMemHandle_t h1, h1b, h2;
  hipIpcGetMemHandle(&h1, b1);
  dump_handle("A", "b1", h1);
  dump_fds("A", "after export b1");
  hipIpcGetMemHandle(&h1b, b1);
  dump_handle("A", "b1 again", h1b);
  dump_fds("A", "after export b1 again");
  hipIpcGetMemHandle(&h2, b2);
  dump_handle("A", "b2", h2);
  dump_fds("A", "after export b2");
  put_file("h1", &h1, sizeof h1);
  put_file("h2", &h2, sizeof h2);
  int done = 0;
  get_file("b_done", &done, sizeof done);
  dump_fds("A", "after B imported and closed");
  hipFree(b1);
  dump_fds("A", "after freeing b1");
  hipExtMallocWithFlags((void **)&b3, 4 << 20, hipDeviceMallocUncached);
  hipMemcpy(b3, &s3, 8, hipMemcpyHostToDevice);
  hipDeviceSynchronize();
  hipIpcMemHandle_t h3;
  hipIpcGetMemHandle(&h3, b3);
  printf("[A] b3 %p\n", (void *)b3);
  dump_handle("A", "b3", h3);
  dump_fds("A", "after export b3");
  put_file("h3", &h3, sizeof h3);
  get_file("b_done3", &done, sizeof done);
  int st = 0;
  waitpid(pb, &st, 0);
  printf("[A] B exited %d\n", WIFEXITED(st) ? WEXITSTATUS(st) : -1);
  hipFree(b2);
  hipFree(b3);
  return 0;
}
