// Can a kernel read STALE cache lines of HBM that an SDMA copy rewrote after an earlier kernel read
// them, when the second kernel is launched with no stream dependency on the copy (the HBM log
// mirror's no-wait policy: the host learned from the copy stream's event that the copy completed)?
//
// Per round: kernel A reads region R (every XCD: a grid of 64 workgroups, each reading all of R),
// the host waits for A; the copy stream copies generation g + 1 of R's pattern from registered host
// memory; the host polls the copy's event until it completed; kernel B (same decode stream, no
// dependency) checks R against generation g + 1.  variant 0: as above; 1: B's stream first waits
// on the (already complete) copy event; 2: B starts with a system-scope acquire fence.
//
// Why: session 21 -- the four-rank dma block fails its device CRC check only in the mirror's no-wait
// mode (the wait mode's stream waits passed), and mirror_stress (long reuse distance) saw nothing.
//
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/probes/reread_stress.hip -o tools/probes/bin/reread_stress
// Run: reread_stress [rounds] [region_kib] [variant]
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                              \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) {                                                                \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(3);                                                                        \
    }                                                                                      \
  } while (0)

__host__ __device__ inline uint32_t pat(uint64_t i, uint32_t g) {
  uint64_t x = (i + (uint64_t(g) << 40)) * 0x9E3779B97F4A7C15ull + 0x632BE59BD9B4E019ull;
  x ^= x >> 29;
  x *= 0xBF58476D1CE4E5B9ull;
  return uint32_t(x >> 32);
}

// every workgroup reads the whole region (so every XCD's L2 holds it); sums into a sink
__global__ void touch_kernel(const uint32_t* __restrict__ r, uint32_t n, uint32_t* sink) {
  uint32_t s = 0;
  for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) s += r[i];
  if (s == 0x12345678u) sink[0] = s;
}

template <bool FENCE>
__global__ void check_kernel(const uint32_t* __restrict__ r, uint32_t n, uint32_t g, unsigned long long* bad) {
  if (FENCE) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  uint32_t miss = 0;
  for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) miss += r[i] != pat(i, g);
  if (miss) atomicAdd(bad, (unsigned long long)miss);
}

int main(int argc, char** argv) {
  const int rounds = argc > 1 ? std::atoi(argv[1]) : 2000;
  const uint32_t kib = uint32_t(argc > 2 ? std::atoi(argv[2]) : 64);
  const int variant = argc > 3 ? std::atoi(argv[3]) : 0;
  if (rounds < 1 || rounds > 100000 || kib < 4 || kib > 4096 || variant < 0 || variant > 2) {
    std::fprintf(stderr, "bad arguments\n");
    return 2;
  }
  const uint32_t n = kib * 256;  // words
  const int gens = 8;
  std::vector<uint32_t*> host(gens);
  for (int g = 0; g < gens; ++g) {
    host[size_t(g)] = static_cast<uint32_t*>(std::aligned_alloc(4096, size_t(n) * 4));
    for (uint32_t i = 0; i < n; ++i) host[size_t(g)][i] = pat(i, uint32_t(g));
    CK(hipHostRegister(host[size_t(g)], size_t(n) * 4, hipHostRegisterMapped));
  }
  uint32_t *r = nullptr, *sink = nullptr;
  unsigned long long* bad = nullptr;
  CK(hipMalloc(reinterpret_cast<void**>(&r), size_t(n) * 4));
  CK(hipMalloc(reinterpret_cast<void**>(&sink), 64));
  CK(hipMalloc(reinterpret_cast<void**>(&bad), 8));
  CK(hipMemset(bad, 0, 8));
  CK(hipMemcpy(r, host[0], size_t(n) * 4, hipMemcpyHostToDevice));
  hipStream_t cs, ds;
  CK(hipStreamCreateWithFlags(&cs, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&ds, hipStreamNonBlocking));
  hipEvent_t copied, touched;
  CK(hipEventCreateWithFlags(&copied, hipEventDisableTiming));
  CK(hipEventCreateWithFlags(&touched, hipEventDisableTiming));
  uint64_t polls = 0, bad_rounds = 0;
  unsigned long long last = 0;
  for (int k = 0; k < rounds; ++k) {
    const uint32_t g = uint32_t(k % gens), g1 = uint32_t((k + 1) % gens);
    hipLaunchKernelGGL(touch_kernel, dim3(64), dim3(256), 0, ds, r, n, sink);
    CK(hipEventRecord(touched, ds));
    CK(hipEventSynchronize(touched));
    (void)g;
    CK(hipMemcpyAsync(r, host[g1], size_t(n) * 4, hipMemcpyHostToDevice, cs));
    CK(hipEventRecord(copied, cs));
    while (hipEventQuery(copied) != hipSuccess) ++polls;
    if (variant == 1) CK(hipStreamWaitEvent(ds, copied, 0));
    if (variant == 2)
      hipLaunchKernelGGL(check_kernel<true>, dim3(64), dim3(256), 0, ds, r, n, g1, bad);
    else
      hipLaunchKernelGGL(check_kernel<false>, dim3(64), dim3(256), 0, ds, r, n, g1, bad);
    CK(hipGetLastError());
    if ((k & 63) == 63 || k == rounds - 1) {
      CK(hipStreamSynchronize(ds));
      unsigned long long h = 0;
      CK(hipMemcpy(&h, bad, 8, hipMemcpyDeviceToHost));
      if (h != last) ++bad_rounds;
      last = h;
    }
  }
  CK(hipDeviceSynchronize());
  std::printf("{\"rounds\": %d, \"region_kib\": %u, \"variant\": %d, \"polls\": %llu, \"bad_words\": %llu, "
              "\"windows_with_bad\": %llu}\n",
              rounds, kib, variant, (unsigned long long)polls, last, (unsigned long long)bad_rounds);
  return last ? 1 : 0;
}
