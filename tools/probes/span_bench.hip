// Standalone timing of the fixed-width span decode kernel (csrc/hip/span_decode.hip) on one MI355X:
// what a decode group costs the GPU with nothing else running ("a lone 2 MiB group
// finishes in <= 45 us over PCIe and <= 10 us from HBM") and how many CU-microseconds it holds.
//
// A synthetic log of RecordBatch-shaped segments: each segment is `seg_kib` KiB whose CRC32C over
// bytes [21, len) is stored as its header CRC (so the kernel's verdict must come out clean), with
// f32[dim] values every (4 dim + 32) bytes from byte 61 -- config 2's record shape.  One group =
// `segs` segments (16 x 128 KiB = 2 MiB by default) decoded to bf16, one launch.  The log lives in
// pinned host memory (zero-copy over PCIe, the loader's default) or in HBM (the loader's mirror).
//
//   lone:  launch, synchronize, repeat -- event time of one group alone (median, p90);
//   busy:  `streams` streams launching back to back -- groups per second (throughput);
// and checks the verdict is clean and the values decoded bit-exactly.
//
// Build (CPU container): hipcc -O3 -std=c++17 --offload-arch=gfx950 -Itorchkafka_amd/csrc/core
//   -Itorchkafka_amd/csrc/hip tools/probes/span_bench.hip torchkafka_amd/csrc/hip/span_decode.hip
//   torchkafka_amd/csrc/core/crc32c.cpp -o tools/probes/bin/span_bench
// Run: tools/probes/bin/span_bench [segs] [seg_kib] [reps]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "crc32c.h"
#include "dtypes.h"
#include "span_decode.h"

#define CK(x)                                                                              \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) {                                                                \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(1);                                                                        \
    }                                                                                      \
  } while (0)

__global__ void empty_kernel() {}

static uint16_t bf16_rne(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  if ((u & 0x7FFFFFFFu) > 0x7F800000u) return uint16_t((u >> 16) | 0x40);
  return uint16_t((u + 0x7FFFu + ((u >> 16) & 1u)) >> 16);
}

int main(int argc, char** argv) {
  const int segs = argc > 1 ? std::atoi(argv[1]) : 16;
  const uint32_t seg_len = uint32_t(argc > 2 ? std::atoi(argv[2]) : 128) << 10;
  const int reps = argc > 3 ? std::atoi(argv[3]) : 200;
  const int parts = argc > 4 ? std::atoi(argv[4]) : 1;  // workgroups per segment (SpanLaunch::parts)
  const int dim = 256, rec = 4 * dim + 32;
  if (segs < 1 || segs > tkh::kMaxLaunchSegs || seg_len > tk::kSpanSegMax) {
    std::fprintf(stderr, "bad shape\n");
    return 2;
  }
  const size_t log_bytes = size_t(segs) * seg_len + 64;
  // host log: random bytes, f32 values at the row positions, per-segment header CRC
  std::vector<uint8_t> host(log_bytes);
  uint64_t x = 88172645463325252ull;
  for (auto& b : host) {
    x ^= x << 13, x ^= x >> 7, x ^= x << 17;
    b = uint8_t(x);
  }
  std::vector<uint64_t> row_pos;
  std::vector<tkh::SpanDevSeg> ds(static_cast<size_t>(segs));
  std::vector<uint32_t> seg_row0;
  for (int s = 0; s < segs; ++s) {
    const uint64_t base = uint64_t(s) * seg_len + 7;  // an unaligned segment start, like a log
    seg_row0.push_back(uint32_t(row_pos.size()));
    for (uint64_t p = base + 61; p + uint64_t(4 * dim) <= base + seg_len; p += uint64_t(rec)) {
      for (int e = 0; e < dim; ++e) {
        const float f = float(row_pos.size()) * 0.5f + float(e) * 0.25f - 17.0f;
        std::memcpy(&host[p + 4 * uint64_t(e)], &f, 4);
      }
      row_pos.push_back(p);
    }
  }
  seg_row0.push_back(uint32_t(row_pos.size()));
  for (int s = 0; s < segs; ++s) {
    const uint64_t base = uint64_t(s) * seg_len + 7;
    tkh::SpanDevSeg& d = ds[size_t(s)];
    d = tkh::SpanDevSeg{};
    d.log_pos = base;
    d.len = seg_len;
    d.flags = tk::kSegCrc | tk::kSegCrcFirst | tk::kSegCrcLast;
    d.crc = tk::crc32c(&host[base + 21], seg_len - 21);
    d.row_begin = seg_row0[size_t(s)];
    d.row_end = seg_row0[size_t(s) + 1];
    d.batch = 0;
    d.seg = uint16_t(s);
  }
  const int64_t rows = int64_t(row_pos.size());
  // device buffers
  uint8_t *hlog = nullptr, *hlog_dev = nullptr, *dlog = nullptr;
  CK(hipHostMalloc(reinterpret_cast<void**>(&hlog), log_bytes, hipHostMallocMapped));
  std::memcpy(hlog, host.data(), log_bytes);
  CK(hipHostGetDevicePointer(reinterpret_cast<void**>(&hlog_dev), hlog, 0));
  CK(hipMalloc(reinterpret_cast<void**>(&dlog), log_bytes));
  CK(hipMemcpy(dlog, host.data(), log_bytes, hipMemcpyHostToDevice));
  uint64_t* rp = nullptr;
  CK(hipMalloc(reinterpret_cast<void**>(&rp), row_pos.size() * 8));
  CK(hipMemcpy(rp, row_pos.data(), row_pos.size() * 8, hipMemcpyHostToDevice));
  std::vector<uint32_t> tabs(tk::kSpanTabWords);
  tk::crc32c_span_tables(tabs.data());
  uint32_t* dtabs = nullptr;
  CK(hipMalloc(reinterpret_cast<void**>(&dtabs), tabs.size() * 4));
  CK(hipMemcpy(dtabs, tabs.data(), tabs.size() * 4, hipMemcpyHostToDevice));
  uint16_t* out = nullptr;
  CK(hipMalloc(reinterpret_cast<void**>(&out), size_t(rows) * dim * 2));
  int32_t* err = nullptr;
  uint32_t* partials = nullptr;
  CK(hipHostMalloc(reinterpret_cast<void**>(&err), 64, hipHostMallocMapped));
  CK(hipHostMalloc(reinterpret_cast<void**>(&partials), 4 * 64, hipHostMallocMapped));
  int32_t* err_dev = nullptr;
  uint32_t* part_dev = nullptr;
  CK(hipHostGetDevicePointer(reinterpret_cast<void**>(&err_dev), err, 0));
  CK(hipHostGetDevicePointer(reinterpret_cast<void**>(&part_dev), partials, 0));

  const int nstreams = 3;
  uint32_t* acc[nstreams];
  for (auto& p : acc) {
    CK(hipMalloc(reinterpret_cast<void**>(&p), tkh::kMaxLaunchSegs * 2 * sizeof(uint32_t)));
    CK(hipMemset(p, 0, tkh::kMaxLaunchSegs * 2 * sizeof(uint32_t)));
  }
  auto make = [&](const uint8_t* logp, int si) {
    tkh::SpanLaunch a{};
    a.parts = parts;
    a.part_acc = acc[si];
    a.n_seg = segs;
    a.vec_store = 1;
    a.row_elems = dim;
    a.tabs = dtabs;
    a.b[0].out = out;
    a.b[0].row_pos = rp;
    a.b[0].err = err_dev;
    a.b[0].partials = part_dev;
    for (int s = 0; s < segs; ++s) {
      a.s[s] = ds[size_t(s)];
      a.s[s].src = logp + ds[size_t(s)].log_pos;
    }
    return a;
  };
  hipStream_t st[nstreams];
  for (auto& s : st) CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::printf("{\"segments\": %d, \"segment_bytes\": %u, \"group_bytes\": %zu, \"rows\": %lld, \"parts\": %d", segs,
              seg_len, size_t(segs) * seg_len, static_cast<long long>(rows), parts);
  for (int mode = 0; mode < 2; ++mode) {
    const char* name = mode == 0 ? "pcie_zero_copy" : "hbm";
    const tkh::SpanLaunch a = make(mode == 0 ? hlog_dev : dlog, 0);
    const tkh::SpanLaunch a1 = make(mode == 0 ? hlog_dev : dlog, 1), a2 = make(mode == 0 ? hlog_dev : dlog, 2);
    const tkh::SpanLaunch* per_stream[nstreams] = {&a, &a1, &a2};
    *err = -1;
    CK(hipMemset(out, 0, size_t(rows) * dim * 2));
    tkh::launch_span_decode(a, tkh::kF32, tkh::kBF16, nullptr, nullptr, st[0]);
    CK(hipStreamSynchronize(st[0]));
    // verdict and values
    std::vector<uint16_t> got(size_t(rows) * dim);
    CK(hipMemcpy(got.data(), out, got.size() * 2, hipMemcpyDeviceToHost));
    int64_t bad = 0;
    for (int64_t r = 0; r < rows; ++r)
      for (int e = 0; e < dim; ++e) {
        float f;
        std::memcpy(&f, &host[row_pos[size_t(r)] + 4 * uint64_t(e)], 4);
        bad += got[size_t(r) * dim + size_t(e)] != bf16_rne(f);
      }
    // lone groups
    std::vector<float> ms;
    for (int i = 0; i < reps; ++i) {
      CK(hipEventRecord(e0, st[0]));
      tkh::launch_span_decode(a, tkh::kF32, tkh::kBF16, nullptr, nullptr, st[0]);
      CK(hipEventRecord(e1, st[0]));
      CK(hipEventSynchronize(e1));
      float t = 0;
      CK(hipEventElapsedTime(&t, e0, e1));
      ms.push_back(t);
    }
    std::sort(ms.begin(), ms.end());
    // back to back on 3 streams
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0, st[0]));
    for (int i = 0; i < reps; ++i)
      tkh::launch_span_decode(*per_stream[i % nstreams], tkh::kF32, tkh::kBF16, nullptr, nullptr, st[i % nstreams]);
    for (int s = 1; s < nstreams; ++s) {
      hipEvent_t ej;
      CK(hipEventCreateWithFlags(&ej, hipEventDisableTiming));
      CK(hipEventRecord(ej, st[s]));
      CK(hipStreamWaitEvent(st[0], ej, 0));
    }
    CK(hipEventRecord(e1, st[0]));
    CK(hipEventSynchronize(e1));
    float tb = 0;
    CK(hipEventElapsedTime(&tb, e0, e1));
    const double gb = double(size_t(segs) * seg_len) * reps / (tb * 1e-3) / 1e9;
    std::printf(", \"%s\": {\"verdict\": %d, \"value_mismatches\": %lld, \"lone_us_p50\": %.1f, \"lone_us_p10\": %.1f, "
                "\"lone_us_p90\": %.1f, \"lone_gb_per_s\": %.1f, \"busy_gb_per_s\": %.1f, \"busy_us_per_group\": %.2f, "
                "\"cu_us_per_mib_upper\": %.1f}",
                name, *err, static_cast<long long>(bad), ms[ms.size() / 2] * 1e3, ms[ms.size() / 10] * 1e3,
                ms[ms.size() * 9 / 10] * 1e3, double(size_t(segs) * seg_len) / (ms[ms.size() / 2] * 1e-3) / 1e9, gb,
                tb * 1e3 / reps, ms[ms.size() / 2] * 1e3 * segs / (double(size_t(segs) * seg_len) / (1 << 20)));
  }
  // partial CRCs of RecordBatches cut into several segments (flags First-only / Last-only /
  // neither, short and long segments), the same accumulator words for two launches in a row on one
  // stream: every partial must equal the host emulation's
  {
    tkh::SpanLaunch pa = make(dlog, 0);
    std::vector<uint32_t> want(static_cast<size_t>(segs));
    for (int s = 0; s < segs; ++s) {
      tkh::SpanDevSeg& d = pa.s[s];
      const int kind = s % 3;  // 0: first part of a batch, 1: a middle part, 2: the last part
      d.flags = tk::kSegCrc | (kind == 0 ? tk::kSegCrcFirst : kind == 2 ? tk::kSegCrcLast : 0u);
      d.len = kind == 2 ? 3600u + 977u * uint32_t(s % 5) : seg_len - 1000u * uint32_t(s % 4);
      d.row_begin = d.row_end = 0;
      const uint32_t c0 = kind == 0 ? 21u : 0u;
      want[size_t(s)] = tk::crc32c_span_emulate(&host[d.log_pos], c0, d.len, kind == 0, 1);
    }
    int64_t bad_partials = 0;
    for (int rep = 0; rep < 2; ++rep) {
      for (int s = 0; s < segs; ++s) partials[s] = 0xDEADBEEFu;
      *err = -1;
      tkh::launch_span_decode(pa, tkh::kF32, tkh::kBF16, nullptr, nullptr, st[0]);
      tkh::launch_span_decode(pa, tkh::kF32, tkh::kBF16, nullptr, nullptr, st[0]);
      CK(hipStreamSynchronize(st[0]));
      for (int s = 0; s < segs; ++s) bad_partials += partials[s] != want[size_t(s)];
    }
    std::printf(", \"partials\": {\"segments\": %d, \"mismatches\": %lld, \"verdict\": %d}", segs,
                static_cast<long long>(bad_partials), *err);
  }
  // where a lone group's time goes: an empty kernel's lone time (launch + completion), and the
  // HBM group with no CRC (values only: no lane merge, no part accumulation, no verdict)
  auto lone = [&](auto&& launch) {
    std::vector<float> v;
    for (int i = 0; i < reps; ++i) {
      CK(hipEventRecord(e0, st[0]));
      launch();
      CK(hipEventRecord(e1, st[0]));
      CK(hipEventSynchronize(e1));
      float t = 0;
      CK(hipEventElapsedTime(&t, e0, e1));
      v.push_back(t);
    }
    std::sort(v.begin(), v.end());
    return v[v.size() / 2] * 1e3;
  };
  const double empty_us = lone([&] { hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, st[0]); });
  const double empty_wide_us =
      lone([&] { hipLaunchKernelGGL(empty_kernel, dim3(segs * parts), dim3(576), 0, st[0]); });
  tkh::SpanLaunch nc = make(dlog, 0);
  for (int s = 0; s < segs; ++s) nc.s[s].flags = 0;
  const double nocrc_us = lone([&] { tkh::launch_span_decode(nc, tkh::kF32, tkh::kBF16, nullptr, nullptr, st[0]); });
  std::printf(", \"empty_lone_us_p50\": %.1f, \"empty_grid_lone_us_p50\": %.1f, \"hbm_nocrc_lone_us_p50\": %.1f}\n",
              empty_us, empty_wide_us, nocrc_us);
  return 0;
}
