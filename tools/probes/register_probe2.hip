// Probe 2: cost of pinning (hipHostRegister) pages of a POSIX shm file that another mapping
// populated -- the situation of h2d="direct", where the main process pins broker log pages the
// producer wrote -- with 4 KiB pages and with transparent huge pages (MADV_HUGEPAGE), if the
// kernel allows THP on shmem.
#include <hip/hip_runtime.h>
#include <fcntl.h>
#include <sys/mman.h>
#include <unistd.h>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <string>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)
static double now_us() { return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

static int run(bool huge, size_t chunk) {
  const size_t total = size_t(1) << 30;
  std::string name = "/tk_reg2_" + std::to_string(getpid()) + (huge ? "h" : "s");
  int fd = shm_open(name.c_str(), O_RDWR | O_CREAT, 0600);
  if (fd < 0 || ftruncate(fd, total) != 0) { perror("shm"); return 1; }
  uint8_t* w = (uint8_t*)mmap(nullptr, total, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  int adv = huge ? madvise(w, total, MADV_HUGEPAGE) : 0;
  memset(w, 1, total);  // the "producer" mapping writes the log
  uint8_t* r = (uint8_t*)mmap(nullptr, total, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);  // the driver's own mapping
  if (huge) madvise(r, total, MADV_HUGEPAGE);
  double t0 = now_us();
  size_t n = 0;
  for (size_t off = 0; off + chunk <= total; off += chunk, ++n) CK(hipHostRegister(r + off, chunk, hipHostRegisterMapped));
  double t1 = now_us();
  for (size_t off = 0; off + chunk <= total; off += chunk) CK(hipHostUnregister(r + off));
  // populate the page tables first, then register
  munmap(r, total);
  r = (uint8_t*)mmap(nullptr, total, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  if (huge) madvise(r, total, MADV_HUGEPAGE);
  double t2 = now_us();
  int pop = madvise(r, total, MADV_POPULATE_READ);
  double t3 = now_us();
  for (size_t off = 0; off + chunk <= total; off += chunk) CK(hipHostRegister(r + off, chunk, hipHostRegisterMapped));
  double t4 = now_us();
  for (size_t off = 0; off + chunk <= total; off += chunk) CK(hipHostUnregister(r + off));
  printf("{\"probe\":\"register_fresh_mapping\",\"huge\":%d,\"madvise_rc\":%d,\"chunk_MiB\":%zu,\"register_GBps\":%.1f,"
         "\"populate_GBps\":%.1f,\"populate_rc\":%d,\"register_after_populate_GBps\":%.1f}\n",
         huge, adv, chunk >> 20, total / (t1 - t0) / 1e3, total / (t3 - t2) / 1e3, pop, total / (t4 - t3) / 1e3);
  munmap(w, total);
  munmap(r, total);
  shm_unlink(name.c_str());
  close(fd);
  return 0;
}

int main() {
  FILE* f = fopen("/sys/kernel/mm/transparent_hugepage/shmem_enabled", "r");
  char buf[256] = {0};
  if (f) { fgets(buf, sizeof buf, f); fclose(f); }
  buf[strcspn(buf, "\n")] = 0;
  printf("{\"probe\":\"thp_shmem_enabled\",\"value\":\"%s\"}\n", buf);
  f = fopen("/sys/kernel/mm/transparent_hugepage/enabled", "r");
  memset(buf, 0, sizeof buf);
  if (f) { fgets(buf, sizeof buf, f); fclose(f); }
  buf[strcspn(buf, "\n")] = 0;
  printf("{\"probe\":\"thp_enabled\",\"value\":\"%s\"}\n", buf);
  CK(hipSetDevice(0));
  for (size_t chunk : {size_t(64) << 20, size_t(256) << 20})
    for (bool huge : {false, true})
      if (run(huge, chunk)) return 1;
  return 0;
}
