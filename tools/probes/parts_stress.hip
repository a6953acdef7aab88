// Stress of the span decode kernel's split segments (SpanLaunch::parts > 1, the HBM-mirror path):
// the parts of a segment merge their CRC partials in an accumulator word (span_device.h
// crc_finish), handed out per launch in rotation over `sets` sets per stream, as Engine::part_acc
// does.  Every launch gets a verdict word of its own, so a launch whose merge went wrong shows
// as a CRC verdict on a log whose CRCs are all correct.
//
// Why: the driver's four-rank rehearsal on one GPU (profiles/r06_s18) failed one device CRC
// check in the h2d='dma' block (the only path that splits segments), once in two runs.
//
// Build (CPU container): hipcc -O3 -std=c++17 --offload-arch=gfx950 -Itorchkafka_amd/csrc/core
//   -Itorchkafka_amd/csrc/hip tools/probes/parts_stress.hip torchkafka_amd/csrc/hip/span_decode.hip
//   torchkafka_amd/csrc/core/crc32c.cpp -o tools/probes/bin/parts_stress
// Run: parts_stress [launches_per_stream] [streams] [parts] [sets] [segs] [seg_kib]
#include <hip/hip_runtime.h>

#include <chrono>
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

int main(int argc, char** argv) {
  const int launches = argc > 1 ? std::atoi(argv[1]) : 5000;
  const int nstreams = argc > 2 ? std::atoi(argv[2]) : 4;
  const int parts = argc > 3 ? std::atoi(argv[3]) : 8;
  const int sets = argc > 4 ? std::atoi(argv[4]) : 16;
  const int segs = argc > 5 ? std::atoi(argv[5]) : 12;
  const uint32_t seg_len = uint32_t(argc > 6 ? std::atoi(argv[6]) : 128) << 10;
  const int dim = 256, rec = 4 * dim + 32;
  if (launches < 1 || launches > 200000 || nstreams < 1 || nstreams > 16 || sets < 1 || sets > 4096 ||
      segs < 1 || segs > tkh::kMaxLaunchSegs || seg_len > tk::kSpanSegMax ||
      !(parts == 1 || parts == 2 || parts == 4 || parts == tk::kSpanMaxParts)) {
    std::fprintf(stderr, "bad shape\n");
    return 2;
  }
  const size_t log_bytes = size_t(segs) * seg_len + 64;
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
    const uint64_t base = uint64_t(s) * seg_len + 7;
    seg_row0.push_back(uint32_t(row_pos.size()));
    for (uint64_t p = base + 61; p + uint64_t(4 * dim) <= base + seg_len; p += uint64_t(rec)) row_pos.push_back(p);
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
  uint8_t* dlog = nullptr;
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
  // one verdict word per launch (host-mapped, as the loader's), one output and partials buffer per stream
  const size_t total = size_t(launches) * size_t(nstreams);
  int32_t* err = nullptr;
  CK(hipHostMalloc(reinterpret_cast<void**>(&err), total * sizeof(int32_t), hipHostMallocMapped));
  for (size_t i = 0; i < total; ++i) err[i] = -1;
  int32_t* err_dev = nullptr;
  CK(hipHostGetDevicePointer(reinterpret_cast<void**>(&err_dev), err, 0));
  const size_t set_words = size_t(tkh::kMaxLaunchSegs) * 2;
  std::vector<uint32_t*> acc(static_cast<size_t>(nstreams)), part(static_cast<size_t>(nstreams));
  std::vector<uint16_t*> out(static_cast<size_t>(nstreams));
  std::vector<hipStream_t> st(static_cast<size_t>(nstreams));
  for (int s = 0; s < nstreams; ++s) {
    CK(hipMalloc(reinterpret_cast<void**>(&acc[size_t(s)]), set_words * size_t(sets) * sizeof(uint32_t)));
    CK(hipMemset(acc[size_t(s)], 0, set_words * size_t(sets) * sizeof(uint32_t)));
    CK(hipMalloc(reinterpret_cast<void**>(&part[size_t(s)]), 64 * sizeof(uint32_t)));
    CK(hipMalloc(reinterpret_cast<void**>(&out[size_t(s)]), size_t(rows) * dim * 2));
    CK(hipStreamCreateWithFlags(&st[size_t(s)], hipStreamNonBlocking));
  }
  tkh::SpanLaunch a{};
  a.parts = parts;
  a.n_seg = segs;
  a.vec_store = 1;
  a.row_elems = dim;
  a.tabs = dtabs;
  a.b[0].row_pos = rp;
  for (int s = 0; s < segs; ++s) {
    a.s[s] = ds[size_t(s)];
    a.s[s].src = dlog + ds[size_t(s)].log_pos;
  }
  CK(hipDeviceSynchronize());
  const auto t0 = std::chrono::steady_clock::now();
  for (int i = 0; i < launches; ++i)
    for (int s = 0; s < nstreams; ++s) {
      a.b[0].out = out[size_t(s)];
      a.b[0].err = err_dev + size_t(i) * size_t(nstreams) + size_t(s);
      a.b[0].partials = part[size_t(s)];
      a.part_acc = acc[size_t(s)] + size_t(i % sets) * set_words;
      tkh::launch_span_decode(a, tkh::kF32, tkh::kBF16, nullptr, nullptr, st[size_t(s)]);
    }
  CK(hipDeviceSynchronize());
  const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  size_t bad = 0, first_bad = total;
  for (size_t i = 0; i < total; ++i)
    if (err[i] != -1) {
      ++bad;
      if (first_bad == total) first_bad = i;
    }
  // every accumulator word must be back at zero
  size_t dirty = 0;
  for (int s = 0; s < nstreams; ++s) {
    std::vector<uint32_t> h(set_words * size_t(sets));
    CK(hipMemcpy(h.data(), acc[size_t(s)], h.size() * 4, hipMemcpyDeviceToHost));
    for (uint32_t w : h) dirty += w != 0;
  }
  std::printf("{\"launches\": %zu, \"streams\": %d, \"parts\": %d, \"sets\": %d, \"segs\": %d, \"seg_kib\": %u, "
              "\"bad_launches\": %zu, \"first_bad\": %lld, \"dirty_acc_words\": %zu, \"s\": %.3f, \"gb_per_s\": %.1f}\n",
              total, nstreams, parts, sets, segs, seg_len >> 10, bad,
              first_bad == total ? -1LL : static_cast<long long>(first_bad), dirty, el,
              double(total) * double(segs) * seg_len / el / 1e9);
  return bad || dirty ? 1 : 0;
}
