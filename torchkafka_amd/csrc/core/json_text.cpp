// Host JSON numeric arrays (JsonArray records): the parser the workers run on the host path
// (parse_json_f32, bit-exact with json.loads + float32), and the pre-scan that frames a row for
// the device parse (json_scan_*: element count and the "simple row" check, AVX-512 when present).
// Declared in consumer.h; the device side is csrc/hip/json_parse.hip and json_span.hip.
#include "consumer.h"

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <limits>

#if defined(__x86_64__)
#include <immintrin.h>
#endif

namespace tk {

#if defined(__x86_64__)
namespace {
// the copying pre-scan streams its output (non-temporal stores), like the slot packers'
// copy_to_slot in consumer.cpp; TORCHKAFKA_NT_COPY=0 turns both off
const bool g_avx2 = [] {
  const char* e = std::getenv("TORCHKAFKA_NT_COPY");
  return __builtin_cpu_supports("avx2") && !(e && e[0] == '0');
}();
}  // namespace
#endif

// ------------------------------------------------------------ JSON
namespace {

inline bool is_ws(char c) { return c == ' ' || c == '\n' || c == '\t' || c == '\r'; }
inline bool is_digit(char c) { return c >= '0' && c <= '9'; }

const double kPow10[] = {1e0,  1e1,  1e2,  1e3,  1e4,  1e5,  1e6,  1e7,  1e8,  1e9,  1e10, 1e11,
                         1e12, 1e13, 1e14, 1e15, 1e16, 1e17, 1e18, 1e19, 1e20, 1e21, 1e22};

// Parses one JSON number (or NaN/Infinity/-Infinity, which Python's json accepts).
// Returns the end pointer or nullptr.
const char* parse_number(const char* p, const char* e, double* out) {
  const char* start = p;
  bool neg = false;
  if (p < e && *p == '-') { neg = true; ++p; }
  if (p < e && (*p == 'N' || *p == 'I')) {
    if (e - p >= 3 && std::memcmp(p, "NaN", 3) == 0 && !neg) { *out = std::numeric_limits<double>::quiet_NaN(); return p + 3; }
    if (e - p >= 8 && std::memcmp(p, "Infinity", 8) == 0) {
      *out = neg ? -std::numeric_limits<double>::infinity() : std::numeric_limits<double>::infinity();
      return p + 8;
    }
    return nullptr;
  }
  uint64_t mant = 0;
  int nd = 0, exp10 = 0;
  bool any = false, truncated = false;
  while (p < e && is_digit(*p)) {
    const int d = *p++ - '0';
    any = true;
    if (mant == 0 && d == 0) continue;
    if (nd < 19) { mant = mant * 10 + uint64_t(d); ++nd; } else { ++exp10; truncated = true; }
  }
  const bool is_int_so_far = !(p < e && (*p == '.' || *p == 'e' || *p == 'E'));
  if (p < e && *p == '.') {
    ++p;
    bool frac = false;
    while (p < e && is_digit(*p)) {
      const int d = *p++ - '0';
      frac = true;
      if (mant == 0 && d == 0) { --exp10; continue; }
      if (nd < 19) { mant = mant * 10 + uint64_t(d); ++nd; --exp10; } else { truncated = true; }
    }
    if (!frac) return nullptr;
    any = true;
  }
  if (!any) return nullptr;
  if (p < e && (*p == 'e' || *p == 'E')) {
    ++p;
    bool eneg = false;
    if (p < e && (*p == '+' || *p == '-')) eneg = *p++ == '-';
    if (p >= e || !is_digit(*p)) return nullptr;
    int ev = 0;
    while (p < e && is_digit(*p)) { if (ev < 100000) ev = ev * 10 + (*p - '0'); ++p; }
    exp10 += eneg ? -ev : ev;
  }
  // "-0" is the JSON integer 0 for Python (json.loads gives int 0, float() +0.0); "-0.0" stays -0.0
  if (neg && mant == 0 && is_int_so_far) neg = false;
  double v;
  if (!truncated && mant <= (1ull << 53) && exp10 >= -22 && exp10 <= 22) {
    // Clinger's fast path: both operands exact, one correctly rounded op.
    v = exp10 < 0 ? double(mant) / kPow10[-exp10] : double(mant) * kPow10[exp10];
    if (neg) v = -v;
  } else {
    char buf[128];
    const size_t len = std::min<size_t>(size_t(p - start), sizeof(buf) - 1);
    std::memcpy(buf, start, len);
    buf[len] = 0;
    v = std::strtod(buf, nullptr);
  }
  *out = v;
  return p;
}

}  // namespace

int64_t parse_json_f32(const char* s, size_t n, float* out, int64_t cap) {
  const char* p = s;
  const char* e = s + n;
  while (p < e && is_ws(*p)) ++p;
  if (p >= e || *p != '[') return -1;
  ++p;
  while (p < e && is_ws(*p)) ++p;
  int64_t k = 0;
  if (p < e && *p == ']') {
    ++p;
  } else {
    for (;;) {
      while (p < e && is_ws(*p)) ++p;
      double v;
      p = parse_number(p, e, &v);
      if (!p) return -1;
      if (k >= cap) return -2;
      out[k++] = float(v);
      while (p < e && is_ws(*p)) ++p;
      if (p >= e) return -1;
      if (*p == ',') { ++p; continue; }
      if (*p == ']') { ++p; break; }
      return -1;
    }
  }
  while (p < e && is_ws(*p)) ++p;
  return p == e ? k : -1;
}

int64_t json_array_len(const char* s, size_t n) {
  const char* p = s;
  const char* e = s + n;
  while (p < e && is_ws(*p)) ++p;
  if (p >= e || *p != '[') return -1;
  ++p;
  int64_t k = 0;
  bool in_tok = false;
  for (; p < e; ++p) {
    if (*p == ']') return in_tok ? k + 1 : k;
    if (*p == ',') { if (!in_tok) return -1; ++k; in_tok = false; }
    else if (!is_ws(*p)) in_tok = true;
  }
  return -1;
}

// ------------------------------------------------------------ JSON pre-scan (device parse)
// A row is "simple" -- parsed on the GPU (json_parse.hip) -- when, after trimming
// whitespace, it is '[' ... ']' whose interior holds only digits, '.', '-', ',' and
// whitespace, and no run of number characters is longer than 16.  Such numbers have at
// most 16 digits and no exponent, so Clinger's fast path (or an exact u64 -> f64
// conversion for integers) gives Python's float() on the device too.  Returns the
// element count (commas + 1, or 0 for an empty array), or -1 when the row is not simple
// (the host parser then decides: a valid row is parsed, a malformed one is bad()).
namespace {

constexpr int kMaxSimpleToken = 16;

inline bool scan_tok(uint8_t c) { return uint8_t(c - '0') <= 9 || c == '.' || c == '-'; }
inline bool scan_ws(uint8_t c) { return c == ' ' || c == '\t' || c == '\n' || c == '\r'; }

// interior scan state carried across blocks
struct ScanState {
  int64_t commas = 0;
  int run = 0;       // length of the token-character run ending at the previous byte
  bool any_tok = false;
};

bool scan_interior_scalar(const uint8_t* p, size_t n, ScanState& st) {
  for (size_t i = 0; i < n; ++i) {
    const uint8_t c = p[i];
    if (scan_tok(c)) {
      st.any_tok = true;
      if (++st.run > kMaxSimpleToken) return false;
    } else {
      st.run = 0;
      if (c == ',') ++st.commas;
      else if (!scan_ws(c)) return false;
    }
  }
  return true;
}

#if defined(__x86_64__)
// 64 bytes per iteration, branch-free: the character-class and long-run verdicts are
// OR-ed into `bad` and checked once.  A run of > 16 token characters ending in this block
// either lies inside the 80 bits (previous block's top 16 + this block's 64) or was already
// caught in the previous block, so one 128-bit AND-of-shifts per block finds every run.
// 32 bytes -> token-character and comma masks; returns the mask of bytes outside the row alphabet
__attribute__((target("avx2"), always_inline)) inline uint32_t scan_classify32(const uint8_t* q, uint32_t* tokm,
                                                                               uint32_t* comm) {
  const __m256i v = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(q));
  const __m256i c9 = _mm256_set1_epi8(9);
  const __m256i dv = _mm256_sub_epi8(v, _mm256_set1_epi8('0'));
  const __m256i dig = _mm256_cmpeq_epi8(_mm256_min_epu8(dv, c9), dv);
  const __m256i tok = _mm256_or_si256(dig, _mm256_or_si256(_mm256_cmpeq_epi8(v, _mm256_set1_epi8('.')),
                                                            _mm256_cmpeq_epi8(v, _mm256_set1_epi8('-'))));
  const __m256i com = _mm256_cmpeq_epi8(v, _mm256_set1_epi8(','));
  const __m256i ws = _mm256_or_si256(
      _mm256_or_si256(_mm256_cmpeq_epi8(v, _mm256_set1_epi8(' ')), _mm256_cmpeq_epi8(v, _mm256_set1_epi8('\t'))),
      _mm256_or_si256(_mm256_cmpeq_epi8(v, _mm256_set1_epi8('\n')), _mm256_cmpeq_epi8(v, _mm256_set1_epi8('\r'))));
  *tokm = uint32_t(_mm256_movemask_epi8(tok));
  *comm = uint32_t(_mm256_movemask_epi8(com));
  return ~uint32_t(_mm256_movemask_epi8(_mm256_or_si256(tok, _mm256_or_si256(com, ws))));
}

__attribute__((target("avx2,bmi,popcnt"))) bool scan_interior_avx2(const uint8_t* p, size_t n, ScanState& st) {
  // carry the previous run as the top bits of a virtual previous mask
  uint64_t prev = st.run >= 16 ? ~uint64_t(0) : (st.run ? ~uint64_t(0) << (64 - st.run) : 0);
  uint64_t bad = st.run > kMaxSimpleToken ? 1 : 0, anyt = 0;
  int64_t commas = 0;
  size_t i = 0;
  for (; i + 64 <= n; i += 64) {
    uint32_t t0, t1, c0m, c1m;
    bad |= scan_classify32(p + i, &t0, &c0m);
    bad |= scan_classify32(p + i + 32, &t1, &c1m);
    const uint64_t m = uint64_t(t0) | (uint64_t(t1) << 32);
    commas += __builtin_popcountll(uint64_t(c0m) | (uint64_t(c1m) << 32));
    anyt |= m;
    const unsigned __int128 y = (static_cast<unsigned __int128>(m) << 16) | (prev >> 48);
    unsigned __int128 r = y & (y >> 1);  // runs >= 2
    r &= r >> 2;                          // >= 4
    r &= r >> 4;                          // >= 8
    r &= r >> 8;                          // >= 16
    r &= y >> 16;                         // >= 17
    bad |= uint64_t(r) | uint64_t(r >> 64);
    prev = m;
  }
  if (bad) return false;
  st.commas += commas;
  st.any_tok = st.any_tok || anyt != 0;
  if (i) st.run = prev == ~uint64_t(0) ? std::max(st.run, 0) + 64 : __builtin_clzll(~prev);
  if (i && prev == ~uint64_t(0)) return false;  // a 64-character token
  return scan_interior_scalar(p + i, n - i, st);
}
const bool g_scan_avx2 = __builtin_cpu_supports("avx2") && __builtin_cpu_supports("bmi") &&
                         __builtin_cpu_supports("popcnt");
#endif

int64_t json_scan_impl(const char* s, size_t n, bool simd) {
  const uint8_t* p = reinterpret_cast<const uint8_t*>(s);
  size_t a = 0, b = n;
  while (a < b && scan_ws(p[a])) ++a;
  while (b > a && scan_ws(p[b - 1])) --b;
  if (b - a < 2 || p[a] != '[' || p[b - 1] != ']') return -1;
  ScanState st;
  bool ok;
#if defined(__x86_64__)
  if (simd && g_scan_avx2)
    ok = scan_interior_avx2(p + a + 1, b - a - 2, st);
  else
#endif
    ok = scan_interior_scalar(p + a + 1, b - a - 2, st);
  (void)simd;
  if (!ok) return -1;
  if (!st.any_tok) return st.commas == 0 ? 0 : -1;
  return st.commas + 1;
}

}  // namespace

int64_t json_scan_simple(const char* s, size_t n, bool simd) { return json_scan_impl(s, n, simd); }

// Fused pre-scan + copy for the worker's hot path: every 32-byte chunk of the row is loaded
// once, classified (json_scan_simple's rules) and streamed to the slot.  Bytes outside the
// array's interior -- leading/trailing whitespace, the brackets, the read-ahead past `n` --
// are masked out of the verdicts.  Needs: dst 32-byte aligned, src readable and dst writable
// up to align_up(n, 32).  Returns what json_scan_simple returns; the text is copied either way.
#if defined(__x86_64__)
__attribute__((target("avx2,bmi,popcnt"))) int64_t json_scan_copy_avx2(const uint8_t* src, size_t n, uint8_t* dst) {
  size_t a = 0, b = n;
  while (a < b && scan_ws(src[a])) ++a;
  while (b > a && scan_ws(src[b - 1])) --b;
  const bool framed = b - a >= 2 && src[a] == '[' && src[b - 1] == ']';
  const size_t lo = a + 1, hi = framed ? b - 1 : lo;  // interior [lo, hi)
  uint64_t bad = 0, anyt = 0, prev = 0;
  int64_t commas = 0;
  const size_t nr = (n + 31) & ~size_t(31);
  for (size_t i = 0; i < nr; i += 32) {
    const __m256i v = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(src + i));
    _mm256_stream_si256(reinterpret_cast<__m256i*>(dst + i), v);
    uint32_t tokm, comm;
    uint32_t badm = scan_classify32(src + i, &tokm, &comm);
    // interior bits of this chunk
    uint32_t in = 0xFFFFFFFFu;
    if (i < lo) in = lo - i >= 32 ? 0u : in << (lo - i);
    if (i + 32 > hi) in &= hi <= i ? 0u : (0xFFFFFFFFu >> (32 - (hi - i)));
    tokm &= in;
    bad |= badm & in;
    commas += __builtin_popcount(comm & in);
    anyt |= tokm;
    // runs of > 16 number characters: this chunk plus the previous chunk's top 16 bits
    const uint64_t y = (uint64_t(tokm) << 16) | (prev >> 16);
    uint64_t q = y & (y >> 1);
    q &= q >> 2;
    q &= q >> 4;
    q &= q >> 8;
    q &= y >> 16;
    bad |= q;
    prev = tokm;
  }
  if (!framed || bad) return -1;
  if (!anyt) return commas == 0 ? 0 : -1;
  return commas + 1;
}
#endif

// In-place pre-scan for the device parse from the log (kPackJsonSpan): json_scan_simple's verdict
// without a per-row scalar tail -- whole 64-byte blocks, bytes outside the array interior masked
// out of the verdicts (AVX-512BW: one compare per character class per 64 bytes).  Needs the text
// readable up to align_up(n, 64) bytes from s.
#if defined(__x86_64__)
__attribute__((target("avx512f,avx512bw,bmi,popcnt"))) int64_t json_scan_inplace_avx512(const uint8_t* src,
                                                                                         size_t n) {
  size_t a = 0, b = n;
  while (a < b && scan_ws(src[a])) ++a;
  while (b > a && scan_ws(src[b - 1])) --b;
  if (b - a < 2 || src[a] != '[' || src[b - 1] != ']') return -1;
  const size_t lo = a + 1, hi = b - 1;  // interior [lo, hi)
  const __m512i c0 = _mm512_set1_epi8('0'), c9 = _mm512_set1_epi8(9), dot = _mm512_set1_epi8('.'),
                mi = _mm512_set1_epi8('-'), co = _mm512_set1_epi8(','), sp = _mm512_set1_epi8(' '),
                tb = _mm512_set1_epi8('\t'), nl = _mm512_set1_epi8('\n'), cr = _mm512_set1_epi8('\r');
  uint64_t bad = 0, anyt = 0, prev = 0;
  int64_t commas = 0;
  for (size_t i = lo & ~size_t(63); i < hi; i += 64) {
    const __m512i v = _mm512_loadu_si512(reinterpret_cast<const void*>(src + i));
    uint64_t in = ~uint64_t(0);
    if (i < lo) in <<= (lo - i);
    if (i + 64 > hi) in &= ~uint64_t(0) >> (64 - (hi - i));
    const uint64_t tok = (_mm512_cmple_epu8_mask(_mm512_sub_epi8(v, c0), c9) | _mm512_cmpeq_epi8_mask(v, dot) |
                          _mm512_cmpeq_epi8_mask(v, mi)) & in;
    const uint64_t com = _mm512_cmpeq_epi8_mask(v, co) & in;
    const uint64_t ws = _mm512_cmpeq_epi8_mask(v, sp) | _mm512_cmpeq_epi8_mask(v, tb) |
                        _mm512_cmpeq_epi8_mask(v, nl) | _mm512_cmpeq_epi8_mask(v, cr);
    bad |= in & ~(tok | com | ws);
    commas += __builtin_popcountll(com);
    anyt |= tok;
    // runs of > 16 number characters ending in this block: this block plus the previous one's top 16 bits
    const unsigned __int128 y = (static_cast<unsigned __int128>(tok) << 16) | (prev >> 48);
    unsigned __int128 r = y & (y >> 1);
    r &= r >> 2;
    r &= r >> 4;
    r &= r >> 8;
    r &= y >> 16;
    bad |= uint64_t(r) | uint64_t(r >> 64);
    prev = tok;
  }
  if (bad) return -1;
  if (!anyt) return commas == 0 ? 0 : -1;
  return commas + 1;
}
const bool g_scan_avx512 = __builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512bw") &&
                           __builtin_cpu_supports("bmi") && __builtin_cpu_supports("popcnt");

// The same scan with one byte-class lookup per 64 bytes (AVX-512 VBMI vpermt2b over a 128-entry
// table: bit 0 number character [0-9.-], bit 1 ',', bit 2 JSON whitespace) instead of nine
// compares, and the long-run check in plain 64-bit words: runs of >= 17 inside the block by
// shift-and, runs across the block boundary from the previous block's top run + this one's bottom
// run.  ~3x the compare version on the worker's hot path.
constexpr uint8_t scan_class(int c) {
  return uint8_t(((c >= '0' && c <= '9') || c == '.' || c == '-') ? 1
                 : c == ','                                        ? 2
                 : (c == ' ' || c == '\t' || c == '\n' || c == '\r') ? 4
                                                                   : 0);
}
struct ScanTable {
  alignas(64) uint8_t t[128];
  constexpr ScanTable() : t{} {
    for (int i = 0; i < 128; ++i) t[i] = scan_class(i);
  }
};
constexpr ScanTable kScanTable{};

__attribute__((target("avx512f,avx512bw,avx512vbmi,bmi,lzcnt,popcnt"))) int64_t json_scan_inplace_vbmi(
    const uint8_t* src, size_t n) {
  size_t a = 0, b = n;
  while (a < b && scan_ws(src[a])) ++a;
  while (b > a && scan_ws(src[b - 1])) --b;
  if (b - a < 2 || src[a] != '[' || src[b - 1] != ']') return -1;
  const size_t lo = a + 1, hi = b - 1;  // interior [lo, hi)
  const __m512i tlo = _mm512_load_si512(reinterpret_cast<const void*>(kScanTable.t));
  const __m512i thi = _mm512_load_si512(reinterpret_cast<const void*>(kScanTable.t + 64));
  const __m512i b_tok = _mm512_set1_epi8(1), b_com = _mm512_set1_epi8(2), b_any = _mm512_set1_epi8(7);
  uint64_t bad = 0, anyt = 0;
  int64_t commas = 0;
  int prev_run = 0;  // number characters ending at the previous block's top
  for (size_t i = lo & ~size_t(63); i < hi; i += 64) {
    const __m512i v = _mm512_loadu_si512(reinterpret_cast<const void*>(src + i));
    uint64_t in = ~uint64_t(0);
    if (i < lo) in <<= (lo - i);
    if (i + 64 > hi) in &= ~uint64_t(0) >> (64 - (hi - i));
    const __m512i cls = _mm512_permutex2var_epi8(tlo, v, thi);  // index: the low 7 bits
    const uint64_t tok = _mm512_test_epi8_mask(cls, b_tok) & in;
    const uint64_t com = _mm512_test_epi8_mask(cls, b_com) & in;
    const uint64_t ok = _mm512_test_epi8_mask(cls, b_any) & ~_mm512_movepi8_mask(v);  // ASCII, in the alphabet
    bad |= in & ~ok;
    commas += __builtin_popcountll(com);
    anyt |= tok;
    uint64_t r = tok & (tok >> 1);
    r &= r >> 2;
    r &= r >> 4;
    r &= r >> 8;
    r &= tok >> 16;  // bit j: 17 number characters at j .. j + 16
    bad |= r;
    const int lead = tok == ~uint64_t(0) ? 64 : int(__builtin_ctzll(~tok));
    bad |= uint64_t(prev_run + lead > kMaxSimpleToken);
    prev_run = tok == ~uint64_t(0) ? prev_run + 64 : int(__builtin_clzll(~tok));
  }
  if (bad) return -1;
  if (!anyt) return commas == 0 ? 0 : -1;
  return commas + 1;
}
const bool g_scan_vbmi = g_scan_avx512 && __builtin_cpu_supports("avx512vbmi") && __builtin_cpu_supports("lzcnt");
#endif

int64_t json_scan_inplace(const char* s, size_t n, size_t readable, int variant) {
#if defined(__x86_64__)
  if (readable >= ((n + 63) & ~size_t(63)) + 64) {
    if (g_scan_vbmi && variant <= 0) return json_scan_inplace_vbmi(reinterpret_cast<const uint8_t*>(s), n);
    if (g_scan_avx512 && variant <= 1) return json_scan_inplace_avx512(reinterpret_cast<const uint8_t*>(s), n);
  }
#endif
  (void)readable;
  (void)variant;
  return json_scan_impl(s, n, variant <= 2);
}

int64_t json_scan_copy(const char* s, size_t n, uint8_t* dst) {
#if defined(__x86_64__)
  if (g_scan_avx2 && g_avx2 && (reinterpret_cast<uintptr_t>(dst) & 31) == 0)
    return json_scan_copy_avx2(reinterpret_cast<const uint8_t*>(s), n, dst);
#endif
  std::memcpy(dst, s, n);
  return json_scan_impl(s, n, false);
}

}  // namespace tk
