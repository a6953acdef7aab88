// Probe: does the GPU read pinned host memory slower when every read lands on pages it has not
// touched before (a streaming Kafka log) than when it re-reads a small window (a reused ring)?
// Zero-copy kernel reads and SDMA copies of 2 MiB chunks, from a window cycling over 32 MiB and
// from fresh chunks of a 3 GiB region; shm (4 KiB pages, as the broker log) and hipHostMalloc.
#include <hip/hip_runtime.h>
#include <fcntl.h>
#include <sys/mman.h>
#include <unistd.h>

#include <cstdio>
#include <cstring>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

__global__ void read_kernel(const uint4* __restrict__ src, uint4* __restrict__ dst, size_t n16) {
  uint4 acc = {0, 0, 0, 0};
  for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n16; i += size_t(gridDim.x) * blockDim.x) {
    const uint4 v = src[i];
    acc.x ^= v.x; acc.y ^= v.y; acc.z ^= v.z; acc.w ^= v.w;
  }
  if ((acc.x | acc.y | acc.z | acc.w) == 0x12345678u) dst[0] = acc;
}

static int run(const char* what, uint8_t* dp, size_t total, uint4* dst, void* dbuf) {
  const size_t chunk = size_t(2) << 20, window = size_t(32) << 20;
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int fresh = 0; fresh < 2; ++fresh) {
    for (int blocks : {32, 128, 512}) {
      const int iters = int((total / chunk) / 3);  // a third of the region per pass: fresh pages each pass
      const size_t span = fresh ? total : window;
      static size_t base = 0;
      CK(hipEventRecord(a));
      for (int i = 0; i < iters; ++i) {
        const size_t off = fresh ? (base + size_t(i) * chunk) % span : (size_t(i) * chunk) % span;
        read_kernel<<<blocks, 256>>>((const uint4*)(dp + off), dst, chunk / 16);
      }
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      base += size_t(iters) * chunk;
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      printf("{\"probe\":\"zerocopy\",\"mem\":\"%s\",\"fresh_pages\":%d,\"blocks\":%d,\"GBps\":%.1f}\n", what, fresh,
             blocks, double(chunk) * iters / (ms * 1e-3) / 1e9);
    }
    const int iters = int((total / chunk) / 3);
    static size_t dbase = 0;
    CK(hipEventRecord(a));
    for (int i = 0; i < iters; ++i) {
      const size_t off = fresh ? (dbase + size_t(i) * chunk) % total : (size_t(i) * chunk) % window;
      CK(hipMemcpyAsync(dbuf, dp + off, chunk, hipMemcpyHostToDevice, 0));
    }
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    dbase += size_t(iters) * chunk;
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    printf("{\"probe\":\"sdma\",\"mem\":\"%s\",\"fresh_pages\":%d,\"GBps\":%.1f}\n", what, fresh,
           double(chunk) * iters / (ms * 1e-3) / 1e9);
  }
  return 0;
}

int main() {
  const size_t total = size_t(3) << 30;
  uint4* dst;
  void* dbuf;
  CK(hipMalloc(&dst, 64));
  CK(hipMalloc(&dbuf, size_t(2) << 20));
  {
    const char* name = "/tk_tlb_probe";
    int fd = shm_open(name, O_RDWR | O_CREAT, 0600);
    if (fd < 0 || ftruncate(fd, off_t(total)) != 0) { perror("shm"); return 1; }
    uint8_t* p = (uint8_t*)mmap(nullptr, total, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    shm_unlink(name);
    memset(p, 1, total);
    CK(hipHostRegister(p, total, hipHostRegisterMapped));
    void* dp;
    CK(hipHostGetDevicePointer(&dp, p, 0));
    if (run("shm_registered", (uint8_t*)dp, total, dst, dbuf)) return 1;
    CK(hipHostUnregister(p));
    munmap(p, total);
    close(fd);
  }
  {
    void* h;
    CK(hipHostMalloc(&h, total, hipHostMallocMapped));
    memset(h, 1, total);
    void* dp;
    CK(hipHostGetDevicePointer(&dp, h, 0));
    if (run("hipHostMalloc", (uint8_t*)dp, total, dst, dbuf)) return 1;
    CK(hipHostFree(h));
  }
  return 0;
}
