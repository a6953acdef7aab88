// Stress of the HBM log mirror's ordering (csrc/hip/log_mirror.h) outside the loader: SDMA copies of
// a registered host log into K rotating HBM buffers on a copy stream, their completion learned the
// mirror's way (one event per copy stream, re-recorded at its tail once the previous record
// completed; a buffer is read only once its copy's sequence number is known complete), readers on
// several decode streams, and a buffer refilled only after the copy stream waited for its readers'
// events.  Every reader kernel checks its chunk word by word against the host pattern and counts
// mismatches; the host copy is rewritten nowhere.
//
// Why: session 20's four-rank rehearsal on one GPU failed the device CRC check of the h2d='dma'
// block again with the parts-merge fix in (parts_stress found no bad merge), so the mirror's data
// is the suspect.  mode 0: the no-wait policy (default); mode 1: TORCHKAFKA_MIRROR_WAIT's
// hipStreamWaitEvent of the reader on the copy event; mode 2: a reader launched right after the
// copy is issued with a stream wait (the pure HIP ordering, no host bookkeeping).
//
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/probes/mirror_stress.hip -o tools/probes/bin/mirror_stress
// Run: mirror_stress [log_mib] [chunk_mib] [K] [passes] [mode] [decode_streams]
#include <hip/hip_runtime.h>
#include <sys/mman.h>

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

__host__ __device__ inline uint32_t pat(uint64_t i) {
  uint64_t x = i * 0x9E3779B97F4A7C15ull + 0x632BE59BD9B4E019ull;
  x ^= x >> 29;
  x *= 0xBF58476D1CE4E5B9ull;
  return uint32_t(x >> 32);
}

// one workgroup per 64 KiB: every word of the chunk against the pattern of its log position
__global__ void check_kernel(const uint32_t* __restrict__ buf, uint64_t first_word, uint64_t n_words,
                             unsigned long long* __restrict__ bad) {
  const uint64_t base = uint64_t(blockIdx.x) * 16384;
  uint32_t miss = 0;
  for (uint64_t i = base + threadIdx.x; i < base + 16384 && i < n_words; i += blockDim.x)
    miss += buf[i] != pat(first_word + i);
  if (miss) atomicAdd(bad, (unsigned long long)miss);
}

int main(int argc, char** argv) {
  const uint64_t log_mib = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 1024;
  const uint64_t chunk_mib = argc > 2 ? std::strtoull(argv[2], nullptr, 10) : 8;
  const int K = argc > 3 ? std::atoi(argv[3]) : 4;
  const int passes = argc > 4 ? std::atoi(argv[4]) : 4;
  const int mode = argc > 5 ? std::atoi(argv[5]) : 0;
  const int nd = argc > 6 ? std::atoi(argv[6]) : 4;
  if (log_mib < 64 || log_mib > 8192 || log_mib % 64 || chunk_mib < 1 || chunk_mib > 64 || 64 % chunk_mib || K < 3 ||
      K > 16 || passes < 1 || passes > 64 || mode < 0 || mode > 2 || nd < 1 || nd > 8) {
    std::fprintf(stderr, "bad arguments\n");
    return 2;
  }
  const uint64_t log_bytes = log_mib << 20, chunk = chunk_mib << 20, reg = uint64_t(64) << 20;
  uint8_t* log = static_cast<uint8_t*>(mmap(nullptr, log_bytes, PROT_READ | PROT_WRITE, MAP_SHARED | MAP_ANONYMOUS, -1, 0));
  if (log == MAP_FAILED) return 3;
  uint32_t* w = reinterpret_cast<uint32_t*>(log);
  for (uint64_t i = 0; i < log_bytes / 4; ++i) w[i] = pat(i);
  for (uint64_t a = 0; a < log_bytes; a += reg) CK(hipHostRegister(log + a, reg, hipHostRegisterMapped));
  uint8_t* dev = nullptr;
  CK(hipMalloc(reinterpret_cast<void**>(&dev), chunk * size_t(K)));
  unsigned long long* bad = nullptr;
  CK(hipMalloc(reinterpret_cast<void**>(&bad), 8));
  CK(hipMemset(bad, 0, 8));
  hipStream_t cs;
  CK(hipStreamCreateWithFlags(&cs, hipStreamNonBlocking));
  std::vector<hipStream_t> ds(static_cast<size_t>(nd));
  for (auto& s : ds) CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipEvent_t copied;
  CK(hipEventCreateWithFlags(&copied, hipEventDisableTiming));
  std::vector<hipEvent_t> reader(static_cast<size_t>(K));  // the last reader of each buffer
  std::vector<bool> has_reader(static_cast<size_t>(K), false);
  for (auto& e : reader) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  const int64_t n_chunks = int64_t(log_bytes / chunk);
  std::vector<uint64_t> copy_seq(static_cast<size_t>(K), 0);
  std::vector<int64_t> holds(static_cast<size_t>(K), -1);
  uint64_t seq = 0, recorded = 0, done = 0, reads = 0, waits = 0, polls = 0;
  auto fill = [&](int64_t c) {  // copy chunk c into its buffer after the buffer's last reader
    const int j = int(c % K);
    if (has_reader[size_t(j)]) CK(hipStreamWaitEvent(cs, reader[size_t(j)], 0));
    CK(hipMemcpyAsync(dev + size_t(j) * chunk, log + uint64_t(c) * chunk, chunk, hipMemcpyHostToDevice, cs));
    holds[size_t(j)] = c;
    copy_seq[size_t(j)] = ++seq;
  };
  auto learn = [&] {
    if (recorded > done && hipEventQuery(copied) == hipSuccess) done = recorded;
    if (seq > recorded && recorded == done) {
      CK(hipEventRecord(copied, cs));
      recorded = seq;
    }
  };
  const int ahead = K - 2;
  for (int p = 0; p < passes; ++p) {
    for (int64_t c = 0; c < n_chunks; ++c) {
      const int j = int(c % K);
      if (c == 0)
        for (int64_t k = 0; k <= ahead && k < n_chunks; ++k) fill(k);
      const int64_t next = c + ahead;  // the prefetch behind this read (the mirror's K - 2 ahead)
      hipStream_t d = ds[size_t(c % nd)];
      if (mode == 2) {
        CK(hipEventRecord(copied, cs));
        CK(hipStreamWaitEvent(d, copied, 0));
      } else if (mode == 1) {
        if (copy_seq[size_t(j)] > done) {
          CK(hipEventRecord(copied, cs));
          recorded = seq;
          CK(hipStreamWaitEvent(d, copied, 0));
          ++waits;
        }
      } else {
        learn();
        while (copy_seq[size_t(j)] > done) {  // the loader reads the pinned log meanwhile; here: poll
          ++polls;
          learn();
        }
      }
      if (holds[size_t(j)] != c) {
        std::fprintf(stderr, "bookkeeping: buffer %d holds %lld, want %lld\n", j, (long long)holds[size_t(j)],
                     (long long)c);
        return 3;
      }
      const uint64_t nw = chunk / 4;
      hipLaunchKernelGGL(check_kernel, dim3(unsigned((nw + 16383) / 16384)), dim3(256), 0, d,
                         reinterpret_cast<const uint32_t*>(dev + size_t(j) * chunk), uint64_t(c) * nw, nw, bad);
      CK(hipGetLastError());
      CK(hipEventRecord(reader[size_t(j)], d));
      has_reader[size_t(j)] = true;
      ++reads;
      if (next + 1 < n_chunks) fill(next + 1);
    }
    CK(hipDeviceSynchronize());
    recorded = done = seq;
  }
  unsigned long long h = 0;
  CK(hipMemcpy(&h, bad, 8, hipMemcpyDeviceToHost));
  std::printf("{\"log_mib\": %llu, \"chunk_mib\": %llu, \"K\": %d, \"passes\": %d, \"mode\": %d, \"decode_streams\": %d, "
              "\"reads\": %llu, \"host_polls\": %llu, \"stream_waits\": %llu, \"bad_words\": %llu}\n",
              (unsigned long long)log_mib, (unsigned long long)chunk_mib, K, passes, mode, nd,
              (unsigned long long)reads, (unsigned long long)polls, (unsigned long long)waits, h);
  return h ? 1 : 0;
}
