// Probe: hipHostRegister cost on POSIX shm pages and zero-copy PCIe read bandwidth
// from registered host memory, as a function of grid size.  Informs whether the
// loader can let the GPU read records straight out of the broker log.
#include <hip/hip_runtime.h>
#include <fcntl.h>
#include <sys/mman.h>
#include <unistd.h>
#include <chrono>
#include <cstdio>
#include <cstring>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)
static double now_us() { return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

__global__ void read_kernel(const uint4* __restrict__ src, uint4* __restrict__ dst, size_t n16) {
  uint4 acc = {0, 0, 0, 0};
  for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n16; i += size_t(gridDim.x) * blockDim.x) {
    uint4 v = src[i];
    acc.x ^= v.x; acc.y ^= v.y; acc.z ^= v.z; acc.w ^= v.w;
  }
  if ((acc.x | acc.y | acc.z | acc.w) == 0x12345678u) dst[0] = acc;
}

int main() {
  const size_t total = size_t(1) << 30;
  const char* name = "/tk_register_probe";
  int fd = shm_open(name, O_RDWR | O_CREAT, 0600);
  if (fd < 0 || ftruncate(fd, total) != 0) { perror("shm"); return 1; }
  uint8_t* p = (uint8_t*)mmap(nullptr, total, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  memset(p, 1, total);
  shm_unlink(name);
  uint4* dst;
  CK(hipMalloc(&dst, 64));
  // registration cost vs chunk size
  for (size_t chunk : {size_t(4) << 20, size_t(64) << 20, size_t(256) << 20}) {
    double t0 = now_us();
    size_t n = 0;
    for (size_t off = 0; off + chunk <= total; off += chunk, ++n) CK(hipHostRegister(p + off, chunk, hipHostRegisterMapped));
    double t1 = now_us();
    for (size_t off = 0; off + chunk <= total; off += chunk) CK(hipHostUnregister(p + off));
    double t2 = now_us();
    printf("{\"probe\":\"register\",\"chunk_MiB\":%zu,\"register_GBps\":%.1f,\"us_per_chunk\":%.1f,\"unregister_us_per_chunk\":%.1f}\n",
           chunk >> 20, total / (t1 - t0) / 1e3, (t1 - t0) / n, (t2 - t1) / n);
  }
  CK(hipHostRegister(p, total, hipHostRegisterMapped));
  void* dp;
  CK(hipHostGetDevicePointer(&dp, p, 0));
  printf("{\"probe\":\"devptr_equals_hostptr\",\"value\":%d}\n", dp == (void*)p);
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  for (size_t bytes : {size_t(256) << 10, size_t(1) << 20, size_t(8) << 20, size_t(64) << 20}) {
    for (int blocks : {32, 64, 128, 256, 512, 1024, 2048}) {
      size_t n16 = bytes / 16;
      const int iters = 20;
      for (int w = 0; w < 3; ++w) read_kernel<<<blocks, 256>>>((const uint4*)dp, dst, n16);
      CK(hipEventRecord(a));
      for (int i = 0; i < iters; ++i) read_kernel<<<blocks, 256>>>((const uint4*)((uint8_t*)dp + (i % 4) * bytes), dst, n16);
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      printf("{\"probe\":\"zerocopy_read\",\"bytes\":%zu,\"blocks\":%d,\"us\":%.2f,\"GBps\":%.1f}\n", bytes, blocks,
             ms * 1e3 / iters, bytes * iters / (ms * 1e-3) / 1e9);
    }
  }
  // DMA H2D for comparison
  void* d;
  CK(hipMalloc(&d, size_t(64) << 20));
  for (size_t bytes : {size_t(256) << 10, size_t(1) << 20, size_t(8) << 20, size_t(64) << 20}) {
    const int iters = 20;
    CK(hipMemcpyAsync(d, p, bytes, hipMemcpyHostToDevice, 0));
    CK(hipEventRecord(a));
    for (int i = 0; i < iters; ++i) CK(hipMemcpyAsync(d, p + (i % 4) * bytes, bytes, hipMemcpyHostToDevice, 0));
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    printf("{\"probe\":\"dma_h2d\",\"bytes\":%zu,\"us\":%.2f,\"GBps\":%.1f}\n", bytes, ms * 1e3 / iters,
           bytes * iters / (ms * 1e-3) / 1e9);
  }
  CK(hipHostUnregister(p));
  return 0;
}
