// Host cost of one kernel launch on gfx950, by launch API, for a kernel taking a ~2.8 KiB by-value
// argument (the size of the decode kernels' launch structs): hipLaunchKernelGGL (triple-chevron
// path, a function lookup per launch) against hipModuleLaunchKernel on a hipFunction_t fetched
// once with hipGetFuncBySymbol, and hipEventRecord for comparison.
// Build: hipcc --offload-arch=gfx950 -O2 tools/probes/launch_cost_probe.hip -o tools/probes/launch_cost_probe
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdint>

struct Args {
  uint32_t v[704];  // 2816 bytes
};

__global__ void tiny_kernel(Args a, uint32_t* out) {
  if (threadIdx.x == 0 && blockIdx.x == 0) out[0] = a.v[0] + a.v[703];
}

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main() {
  uint32_t* out = nullptr;
  if (hipMalloc(&out, 64) != hipSuccess) return 2;
  hipStream_t s;
  if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return 2;
  hipEvent_t ev;
  if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) return 2;
  Args a{};
  for (int i = 0; i < 704; ++i) a.v[i] = uint32_t(i);
  const int N = 1000;  // below the hardware queue depth: measures the host side, not the GPU
  for (int rep = 0; rep < 5; ++rep) {
    // triple-chevron path
    double t0 = now_us();
    for (int i = 0; i < N; ++i) hipLaunchKernelGGL(tiny_kernel, dim3(16), dim3(256), 0, s, a, out);
    double t1 = now_us();
    if (hipStreamSynchronize(s) != hipSuccess) return 3;
    // module path with a cached function handle
    hipFunction_t f = nullptr;
    if (hipGetFuncBySymbol(&f, reinterpret_cast<const void*>(&tiny_kernel)) != hipSuccess) {
      std::printf("hipGetFuncBySymbol failed\n");
      return 4;
    }
    struct {
      Args a;
      uint32_t* out;
    } packed{a, out};
    size_t sz = sizeof(packed);
    void* extra[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, &packed, HIP_LAUNCH_PARAM_BUFFER_SIZE, &sz, HIP_LAUNCH_PARAM_END};
    double t2 = now_us();
    for (int i = 0; i < N; ++i)
      if (hipModuleLaunchKernel(f, 16, 1, 1, 256, 1, 1, 0, s, nullptr, extra) != hipSuccess) return 5;
    double t3 = now_us();
    if (hipStreamSynchronize(s) != hipSuccess) return 3;
    double t4 = now_us();
    for (int i = 0; i < N; ++i) hipEventRecord(ev, s);
    double t5 = now_us();
    if (hipStreamSynchronize(s) != hipSuccess) return 3;
    uint32_t h = 0;
    hipMemcpy(&h, out, 4, hipMemcpyDeviceToHost);
    std::printf("rep %d: hipLaunchKernelGGL %.2f us, hipModuleLaunchKernel(cached) %.2f us, hipEventRecord %.2f us"
                " per call (result %u, want %u)\n",
                rep, (t1 - t0) / N, (t3 - t2) / N, (t5 - t4) / N, h, 0u + 703u);
  }
  return 0;
}
