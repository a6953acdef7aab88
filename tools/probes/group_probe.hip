// Probe: zero-copy f32->bf16 conversion of k ring slots (256 KiB each) per kernel, reading pinned
// host memory over PCIe: time per kernel vs (slots per kernel, blocks per slot, loads in flight
// per thread).  Decides the grid shape of fixed_group_kernel.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

struct alignas(16) F8 { float v[8]; };
struct alignas(16) B8 { __bf16 v[8]; };

template <int U>
__global__ __launch_bounds__(256) void conv(const F8* __restrict__ const* src, B8* __restrict__ const* dst, int64_t groups, int bps) {
  const int k = blockIdx.x / bps, b = blockIdx.x % bps;
  const F8* s = src[k];
  B8* d = dst[k];
  const int64_t tile = int64_t(256) * U;
  for (int64_t base = int64_t(b) * tile + threadIdx.x; base < groups; base += int64_t(bps) * tile) {
    F8 in[U];
#pragma unroll
    for (int u = 0; u < U; ++u) if (base + u * 256 < groups) in[u] = s[base + u * 256];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (base + u * 256 >= groups) break;
      B8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) o.v[j] = __bf16(in[u].v[j]);
      d[base + u * 256] = o;
    }
  }
}

int main() {
  const int kMax = 8;
  const size_t slot = 256 << 10;
  void* h;
  CK(hipHostMalloc(&h, slot * kMax * 4, hipHostMallocDefault));
  for (size_t i = 0; i < slot * kMax; i += 4) reinterpret_cast<float*>(h)[i / 4] = float(i % 1000);
  void* d;
  CK(hipMalloc(&d, slot * kMax));
  const F8** srcs;
  B8** dsts;
  CK(hipHostMalloc(&srcs, sizeof(void*) * kMax * 4, hipHostMallocDefault));
  CK(hipMalloc(&dsts, sizeof(void*) * kMax));
  B8* hd[kMax];
  for (int k = 0; k < kMax; ++k) hd[k] = reinterpret_cast<B8*>(static_cast<char*>(d) + k * slot / 2);
  CK(hipMemcpy(dsts, hd, sizeof(hd), hipMemcpyHostToDevice));
  const F8** dsrc;
  CK(hipMalloc(&dsrc, sizeof(void*) * kMax * 4));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const int64_t groups = slot / 32;
  for (int nslots : {1, 2, 4, 8}) {
    for (int bps : {4, 8, 16, 32}) {
      for (int U : {1, 2, 4}) {
        const int iters = 40;
        // rotate through 4 sets of source slots so no kernel re-reads the previous one's lines
        const F8* hs[kMax * 4];
        for (int r = 0; r < 4; ++r)
          for (int k = 0; k < kMax; ++k)
            hs[r * kMax + k] = reinterpret_cast<const F8*>(static_cast<char*>(h) + ((r * kMax + k) % (kMax * 4)) * slot);
        CK(hipMemcpy(dsrc, hs, sizeof(hs), hipMemcpyHostToDevice));
        auto launch = [&](int r) {
          const dim3 g(nslots * bps);
          if (U == 1) hipLaunchKernelGGL(conv<1>, g, dim3(256), 0, 0, dsrc + r * kMax, dsts, groups, bps);
          if (U == 2) hipLaunchKernelGGL(conv<2>, g, dim3(256), 0, 0, dsrc + r * kMax, dsts, groups, bps);
          if (U == 4) hipLaunchKernelGGL(conv<4>, g, dim3(256), 0, 0, dsrc + r * kMax, dsts, groups, bps);
        };
        for (int w = 0; w < 4; ++w) launch(w % 4);
        CK(hipEventRecord(a));
        for (int i = 0; i < iters; ++i) launch(i % 4);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        const double us = ms * 1e3 / iters;
        printf("{\"probe\":\"group\",\"slots\":%d,\"blocks_per_slot\":%d,\"U\":%d,\"us\":%.2f,\"us_per_slot\":%.2f,\"GBps\":%.1f}\n",
               nslots, bps, U, us, us / nslots, nslots * slot / us / 1e3);
      }
    }
  }
  return 0;
}
