// Shared helpers for the torchkafka_amd native core (host C++ only, no HIP).
//
// The native core is everything on the host side of the record path:
//   Kafka RecordBatch v2 codec + CRC32C, the shared-memory synthetic broker,
//   the consumer fetch/decode loop, the batch packers and the pinned slot ring.
// It deliberately contains no HIP calls: it is imported inside forked
// DataLoader-style worker processes, which must never touch the GPU.
#pragma once

#include <atomic>
#include <cerrno>
#include <cstddef>
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#include <pthread.h>
#include <time.h>

namespace tk {

// ---------------------------------------------------------------- errors
// Error classes surfaced to Python with distinct exception types.
struct KafkaError : std::runtime_error {
  using std::runtime_error::runtime_error;
};
struct CommitFailed : KafkaError {
  using KafkaError::KafkaError;
};
struct CorruptRecord : KafkaError {
  using KafkaError::KafkaError;
};
struct OffsetOutOfRange : KafkaError {
  using KafkaError::KafkaError;
};
struct InjectedFetchError : KafkaError {
  using KafkaError::KafkaError;
};

[[noreturn]] inline void throw_errno(const std::string& what) {
  throw std::runtime_error(what + ": " + std::strerror(errno));
}

// ---------------------------------------------------------------- time
inline int64_t now_ns() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return int64_t(ts.tv_sec) * 1000000000LL + ts.tv_nsec;
}
inline int64_t wall_ms() {
  timespec ts;
  clock_gettime(CLOCK_REALTIME, &ts);
  return int64_t(ts.tv_sec) * 1000LL + ts.tv_nsec / 1000000;
}

// Names the calling thread (<= 15 characters) so a per-thread CPU census (/proc/<pid>/task/*/comm,
// bench.py TK_BENCH_CPU=1) tells the native threads apart.
inline void name_thread(const char* name) { pthread_setname_np(pthread_self(), name); }

inline void cpu_relax() {
#if defined(__x86_64__)
  __builtin_ia32_pause();
#else
  std::atomic_signal_fence(std::memory_order_seq_cst);
#endif
}

// ---------------------------------------------------------------- big-endian IO
inline void put_be16(uint8_t* p, uint16_t v) { v = __builtin_bswap16(v); std::memcpy(p, &v, 2); }
inline void put_be32(uint8_t* p, uint32_t v) { v = __builtin_bswap32(v); std::memcpy(p, &v, 4); }
inline void put_be64(uint8_t* p, uint64_t v) { v = __builtin_bswap64(v); std::memcpy(p, &v, 8); }
inline uint16_t get_be16(const uint8_t* p) { uint16_t v; std::memcpy(&v, p, 2); return __builtin_bswap16(v); }
inline uint32_t get_be32(const uint8_t* p) { uint32_t v; std::memcpy(&v, p, 4); return __builtin_bswap32(v); }
inline uint64_t get_be64(const uint8_t* p) { uint64_t v; std::memcpy(&v, p, 8); return __builtin_bswap64(v); }

inline size_t align_up(size_t v, size_t a) { return (v + a - 1) / a * a; }

// ---------------------------------------------------------------- slot layouts
// kPackJsonText rows (device JSON parse): one descriptor per row at the start of the
// slot payload; `off` is relative to the slot's values area.  tlen >= 0: `tlen` bytes
// of raw JSON text at `off` (32-byte aligned) holding `count` numbers; tlen == -1: the
// row was parsed on the host, `n_out` float32 at `off`.  n_out = count after max_len
// truncation -- the row's output length.
struct alignas(16) JsonRowDesc {
  uint32_t off;
  int32_t tlen;
  int32_t count;
  int32_t n_out;
};
static_assert(sizeof(JsonRowDesc) == 16, "JsonRowDesc is read with one 16-byte load");

}  // namespace tk
