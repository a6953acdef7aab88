// Kernel-argument size probe: does a by-value struct of N bytes reach the kernel intact on gfx950?
// Build: hipcc --offload-arch=gfx950 -O2 tools/probes/kernarg_probe.hip -o /tmp/kernarg_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>

template <int N>
struct Args {
  uint32_t v[N];
};

template <int N>
__global__ void sum_kernel(Args<N> a, uint64_t* out) {
  if (threadIdx.x != 0) return;
  uint64_t s = 0;
  for (int i = 0; i < N; ++i) s += uint64_t(a.v[i]) * uint64_t(i + 1);
  out[0] = s;
}

template <int N>
bool probe(uint64_t* dout) {
  Args<N> a;
  uint64_t want = 0;
  for (int i = 0; i < N; ++i) {
    a.v[i] = uint32_t(i * 2654435761u);
    want += uint64_t(a.v[i]) * uint64_t(i + 1);
  }
  hipLaunchKernelGGL(sum_kernel<N>, dim3(1), dim3(64), 0, 0, a, dout);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    std::printf("%6zu bytes: launch error %s\n", sizeof(a), hipGetErrorString(e));
    return false;
  }
  uint64_t got = 0;
  if (hipMemcpy(&got, dout, 8, hipMemcpyDeviceToHost) != hipSuccess) {
    std::printf("%6zu bytes: copy failed\n", sizeof(a));
    return false;
  }
  std::printf("%6zu bytes: %s\n", sizeof(a), got == want ? "ok" : "WRONG");
  return got == want;
}

int main() {
  uint64_t* dout = nullptr;
  if (hipMalloc(&dout, 8) != hipSuccess) return 2;
  bool ok = probe<512>(dout) && probe<1000>(dout) && probe<1024>(dout) && probe<1536>(dout) && probe<2048>(dout);
  hipFree(dout);
  return ok ? 0 : 1;
}
