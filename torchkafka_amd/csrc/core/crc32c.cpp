// CRC32C (Castagnoli, reflected polynomial 0x82F63B78).
//
// Kafka's RecordBatch v2 protects attributes..end with CRC32C; kafka-python
// verifies it on every fetched batch when `check_crcs=True` (its default), so
// our consumer does the same.  On x86 the SSE4.2 `crc32` instruction has a
// 3-cycle latency and 1/cycle throughput: a single dependency chain reaches
// ~1/3 of the unit's rate, so long buffers are split into three independent
// streams whose raw states are merged with a GF(2) "shift by L zero bytes".
#include "crc32c.h"

#include <cstdlib>
#include <cstring>

#if defined(__x86_64__)
#include <nmmintrin.h>
#include <xmmintrin.h>
#endif

namespace tk {
namespace {

constexpr uint32_t kPoly = 0x82F63B78u;

// ---- table (slicing-by-8) fallback -------------------------------------
struct Tables {
  uint32_t t[8][256];
  // x^(2^k) mod P in zlib's reflected representation (x^0 == 1<<31).
  uint32_t x2n[32];
  Tables() {
    for (uint32_t i = 0; i < 256; ++i) {
      uint32_t c = i;
      for (int k = 0; k < 8; ++k) c = (c & 1) ? (c >> 1) ^ kPoly : c >> 1;
      t[0][i] = c;
    }
    for (uint32_t i = 0; i < 256; ++i) {
      uint32_t c = t[0][i];
      for (int s = 1; s < 8; ++s) {
        c = t[0][c & 0xFF] ^ (c >> 8);
        t[s][i] = c;
      }
    }
    uint32_t p = 1u << 30;  // x^1
    x2n[0] = p;
    for (int n = 1; n < 32; ++n) x2n[n] = p = multmodp(p, p);
  }
  static uint32_t multmodp(uint32_t a, uint32_t b) {
    uint32_t m = 1u << 31, p = 0;
    for (;;) {
      if (a & m) {
        p ^= b;
        if ((a & (m - 1)) == 0) break;
      }
      m >>= 1;
      b = (b & 1) ? (b >> 1) ^ kPoly : b >> 1;
    }
    return p;
  }
  // x^(n * 2^k) mod P
  uint32_t x2nmodp(uint64_t n, unsigned k) const {
    uint32_t p = 1u << 31;
    while (n) {
      if (n & 1) p = multmodp(x2n[k & 31], p);
      n >>= 1;
      ++k;
    }
    return p;
  }
};

const Tables& tables() {
  static const Tables t;
  return t;
}

uint32_t raw_sw(uint32_t s, const uint8_t* p, size_t n) {
  const auto& T = tables().t;
  while (n && (reinterpret_cast<uintptr_t>(p) & 7)) {
    s = T[0][(s ^ *p++) & 0xFF] ^ (s >> 8);
    --n;
  }
  while (n >= 8) {
    uint64_t w;
    std::memcpy(&w, p, 8);
    w ^= s;
    s = T[7][w & 0xFF] ^ T[6][(w >> 8) & 0xFF] ^ T[5][(w >> 16) & 0xFF] ^ T[4][(w >> 24) & 0xFF] ^
        T[3][(w >> 32) & 0xFF] ^ T[2][(w >> 40) & 0xFF] ^ T[1][(w >> 48) & 0xFF] ^ T[0][w >> 56];
    p += 8;
    n -= 8;
  }
  while (n--) s = T[0][(s ^ *p++) & 0xFF] ^ (s >> 8);
  return s;
}

#if defined(__x86_64__)
// Block lengths for the 3-stream interleave and their shift constants.
constexpr size_t kBlocks[] = {8192, 1024, 128};
// Software prefetch distance (bytes) inside each stream (0 disables; TORCHKAFKA_CRC_PREFETCH).
const size_t kPrefetch = [] {
  const char* e = std::getenv("TORCHKAFKA_CRC_PREFETCH");
  return e ? size_t(std::strtoul(e, nullptr, 10)) : size_t(1024);
}();

struct ShiftConsts {
  uint32_t k[3];
  ShiftConsts() {
    for (int i = 0; i < 3; ++i) k[i] = tables().x2nmodp(kBlocks[i], 3);
  }
};
const ShiftConsts& shift_consts() {
  static const ShiftConsts c;
  return c;
}

__attribute__((target("sse4.2"))) inline uint32_t stream_hw(uint32_t s, const uint8_t* p, size_t n) {
  uint64_t c = s;
  while (n >= 8) {
    uint64_t w;
    std::memcpy(&w, p, 8);
    c = _mm_crc32_u64(c, w);
    p += 8;
    n -= 8;
  }
  uint32_t c32 = uint32_t(c);
  while (n--) c32 = _mm_crc32_u8(c32, *p++);
  return c32;
}

__attribute__((target("sse4.2"))) uint32_t raw_hw(uint32_t s, const uint8_t* p, size_t n) {
  const auto& K = shift_consts();
  for (int bi = 0; bi < 3; ++bi) {
    const size_t L = kBlocks[bi];
    while (n >= 3 * L) {
      uint64_t a = s, b = 0, c = 0;
      const uint8_t* pa = p;
      const uint8_t* pb = p + L;
      const uint8_t* pc = p + 2 * L;
      for (size_t i = 0; i < L; i += 8) {
        if ((i & 63) == 0 && kPrefetch) {
          // the log is read cold from DRAM; the L2 streamer stops at 4 KiB page boundaries, so
          // keep each of the three streams' next lines requested ahead explicitly
          _mm_prefetch(reinterpret_cast<const char*>(pa + i + kPrefetch), _MM_HINT_T0);
          _mm_prefetch(reinterpret_cast<const char*>(pb + i + kPrefetch), _MM_HINT_T0);
          _mm_prefetch(reinterpret_cast<const char*>(pc + i + kPrefetch), _MM_HINT_T0);
        }
        uint64_t wa, wb, wc;
        std::memcpy(&wa, pa + i, 8);
        std::memcpy(&wb, pb + i, 8);
        std::memcpy(&wc, pc + i, 8);
        a = _mm_crc32_u64(a, wa);
        b = _mm_crc32_u64(b, wb);
        c = _mm_crc32_u64(c, wc);
      }
      // state(A||B||C) = shift(shift(a, L) ^ b, L) ^ c
      uint32_t ab = Tables::multmodp(K.k[bi], uint32_t(a)) ^ uint32_t(b);
      s = Tables::multmodp(K.k[bi], ab) ^ uint32_t(c);
      p += 3 * L;
      n -= 3 * L;
    }
  }
  return stream_hw(s, p, n);
}

bool detect_hw() { return __builtin_cpu_supports("sse4.2"); }
#else
bool detect_hw() { return false; }
uint32_t raw_hw(uint32_t s, const uint8_t* p, size_t n) { return raw_sw(s, p, n); }
#endif

const bool g_hw = detect_hw();

}  // namespace

bool crc32c_hw() { return g_hw; }

uint32_t crc32c_extend(uint32_t crc, const void* data, size_t n) {
  const auto* p = static_cast<const uint8_t*>(data);
  uint32_t s = ~crc;
  s = g_hw ? raw_hw(s, p, n) : raw_sw(s, p, n);
  return ~s;
}

uint32_t crc32c(const void* data, size_t n) { return crc32c_extend(0, data, n); }

}  // namespace tk
