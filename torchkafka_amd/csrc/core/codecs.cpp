// Kafka record-set compression: see codecs.h.
//
// Every decoder writes into a caller-given buffer (decompress_into): the replica ingest inflates a
// batch straight into the partition log, so an inflated byte is written once.  Each decoder throws
// NoRoom when the output would not fit, which decompress_into turns into kNoRoom (the caller then
// retries with more room, or refetches once consumers freed ring space).
#include "codecs.h"

#include <dlfcn.h>
#include <zlib.h>

#include <algorithm>
#include <climits>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <new>
#include <stdexcept>
#include <string>

#include "common.h"

namespace tk {

const char* codec_name(int codec) {
  switch (codec) {
    case kCodecNone: return "none";
    case kCodecGzip: return "gzip";
    case kCodecSnappy: return "snappy";
    case kCodecLz4: return "lz4";
    case kCodecZstd: return "zstd";
    default: return "unknown";
  }
}

namespace {

struct NoRoom {};

[[noreturn]] void bad(const char* what) { throw CorruptRecord(std::string("corrupt compressed record set: ") + what); }
[[noreturn]] void bad(const std::string& what) { bad(what.c_str()); }

uint32_t be32(const uint8_t* p) { return (uint32_t(p[0]) << 24) | (uint32_t(p[1]) << 16) | (uint32_t(p[2]) << 8) | p[3]; }
uint32_t le32(const uint8_t* p) { return uint32_t(p[0]) | (uint32_t(p[1]) << 8) | (uint32_t(p[2]) << 16) | (uint32_t(p[3]) << 24); }
void put_le32(std::vector<uint8_t>& v, uint32_t x) {
  for (int i = 0; i < 4; ++i) v.push_back(uint8_t(x >> (8 * i)));
}

// dst[0, len) = dst[-off, -off + len) with LZ77 semantics (off < len repeats a pattern).  `slack`:
// writable bytes past len (16-byte chunks may then run over the end).
inline void match_copy(uint8_t* d, size_t off, size_t len, size_t slack) {
  const uint8_t* m = d - off;
  if (off >= 16 && slack >= 16) {
    for (size_t i = 0; i < len; i += 16) std::memcpy(d + i, m + i, 16);  // each chunk's source is written
    return;
  }
  if (off >= len) {
    std::memcpy(d, m, len);
    return;
  }
  // overlapping: copy the pattern, which doubles with each copy
  size_t left = len;
  while (left) {
    const size_t k = std::min(left, size_t(d - m));
    std::memcpy(d, m, k);
    d += k;
    left -= k;
  }
}

// ------------------------------------------------------------------ LZ4
// One LZ4 block into dst[o, cap); matches may reach back to dst[lo].  Returns the new o.
size_t lz4_block_raw(const uint8_t* src, size_t n, uint8_t* dst, size_t o, size_t cap, size_t lo) {
  const uint8_t* ip = src;
  const uint8_t* const iend = src + n;
  while (ip < iend) {
    const unsigned token = *ip++;
    size_t lit = token >> 4;
    if (lit == 15) {
      unsigned b;
      do {
        if (ip >= iend) bad("lz4 literal length");
        b = *ip++;
        lit += b;
      } while (b == 255);
    }
    if (size_t(iend - ip) < lit) bad("lz4 literals");
    if (cap - o < lit) throw NoRoom{};
    if (lit <= 16 && size_t(iend - ip) >= 16 && cap - o >= 16) std::memcpy(dst + o, ip, 16);
    else std::memcpy(dst + o, ip, lit);
    o += lit;
    ip += lit;
    if (ip == iend) break;  // the last sequence has literals only
    if (iend - ip < 2) bad("lz4 offset");
    const size_t off = size_t(ip[0]) | (size_t(ip[1]) << 8);
    ip += 2;
    size_t len = token & 15;
    if (len == 15) {
      unsigned b;
      do {
        if (ip >= iend) bad("lz4 match length");
        b = *ip++;
        len += b;
      } while (b == 255);
    }
    len += 4;
    if (off == 0 || off > o - lo) bad("match offset");
    if (cap - o < len) throw NoRoom{};
    match_copy(dst + o, off, len, cap - o - len);
    o += len;
  }
  return o;
}

// The system liblz4 (the image ships liblz4.so.1 but no header): its block codec's stable ABI.
struct Lz4Api {
  int (*dec)(const char*, char*, int, int) = nullptr;
  int (*dec_dict)(const char*, char*, int, int, const char*, int) = nullptr;
  int (*enc)(const char*, char*, int, int, int) = nullptr;
  int (*enc_hc)(const char*, char*, int, int, int) = nullptr;
  int (*bound)(int) = nullptr;
  bool ok = false;      // decodes blocks (TORCHKAFKA_LZ4_LIB=0: the decoder here does)
  bool enc_ok = false;  // compress()
};

const Lz4Api& lz4_api() {
  static Lz4Api api;
  static std::once_flag once;
  std::call_once(once, [] {
    void* h = dlopen("liblz4.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) return;
    api.dec = reinterpret_cast<int (*)(const char*, char*, int, int)>(dlsym(h, "LZ4_decompress_safe"));
    api.dec_dict = reinterpret_cast<int (*)(const char*, char*, int, int, const char*, int)>(
        dlsym(h, "LZ4_decompress_safe_usingDict"));
    api.enc = reinterpret_cast<int (*)(const char*, char*, int, int, int)>(dlsym(h, "LZ4_compress_fast"));
    api.enc_hc = reinterpret_cast<int (*)(const char*, char*, int, int, int)>(dlsym(h, "LZ4_compress_HC"));
    api.bound = reinterpret_cast<int (*)(int)>(dlsym(h, "LZ4_compressBound"));
    api.enc_ok = api.enc && api.bound;
    const char* env = std::getenv("TORCHKAFKA_LZ4_LIB");
    api.ok = api.dec && api.dec_dict && !(env && std::strcmp(env, "0") == 0);
  });
  return api;
}

// xxHash32 of a short input (< 16 bytes): the LZ4 frame descriptor's header checksum.
uint32_t xxh32_short(const uint8_t* p, size_t n) {
  constexpr uint32_t P1 = 2654435761u, P2 = 2246822519u, P3 = 3266489917u, P4 = 668265263u, P5 = 374761393u;
  auto rotl = [](uint32_t x, int r) { return (x << r) | (x >> (32 - r)); };
  uint32_t h = P5 + uint32_t(n);
  size_t i = 0;
  for (; i + 4 <= n; i += 4) h = rotl(h + le32(p + i) * P3, 17) * P4;
  for (; i < n; ++i) h = rotl(h + p[i] * P5, 11) * P1;
  h ^= h >> 15;
  h *= P2;
  h ^= h >> 13;
  h *= P3;
  h ^= h >> 16;
  return h;
}

size_t unlz4_frame(const uint8_t* src, size_t n, uint8_t* dst, size_t cap) {
  if (n < 7 || le32(src) != 0x184D2204u) bad("lz4 frame magic");
  const uint8_t flg = src[4];
  if ((flg >> 6) != 1) bad("lz4 frame version");
  const int bsid = (src[5] >> 4) & 7;
  if (bsid < 4) bad("lz4 block size id");
  const size_t block_max = size_t(1) << (8 + 2 * bsid);  // 64 KiB .. 4 MiB
  const bool independent = flg & 0x20;
  size_t o = 6;                     // magic, FLG, BD
  if (flg & 0x08) o += 8;           // content size
  if (flg & 0x01) o += 4;           // dictionary id
  o += 1;                           // header checksum
  if (o > n) bad("lz4 frame header");  // invariant from here on: o <= n, so n - o never wraps
  const bool block_sum = flg & 0x10;
  const Lz4Api& lib = lz4_api();
  size_t out = 0;
  while (true) {
    if (n - o < 4) bad("lz4 block size");
    const uint32_t word = le32(src + o);
    o += 4;
    if (word == 0) break;           // end mark (a content checksum may follow)
    const uint32_t len = word & 0x7fffffffu;
    if (n - o < len) bad("lz4 block");
    if (word & 0x80000000u) {       // stored uncompressed
      if (cap - out < len) throw NoRoom{};
      std::memcpy(dst + out, src + o, len);
      out += len;
    } else if (lib.ok && cap - out >= block_max) {
      // a whole block always fits: any failure of the library's decoder is corrupt input
      const int room = int(block_max);
      int r;
      if (independent || out == 0) {
        r = lib.dec(reinterpret_cast<const char*>(src + o), reinterpret_cast<char*>(dst + out), int(len), room);
      } else {                      // linked blocks: the previous 64 KiB of output is the dictionary
        const size_t d = std::min<size_t>(out, 64 << 10);
        r = lib.dec_dict(reinterpret_cast<const char*>(src + o), reinterpret_cast<char*>(dst + out), int(len), room,
                         reinterpret_cast<const char*>(dst + out - d), int(d));
      }
      if (r < 0) bad("lz4 block");
      out += size_t(r);
    } else {
      out = lz4_block_raw(src + o, len, dst, out, cap, independent ? out : 0);
    }
    o += len;
    if (block_sum) {
      if (n - o < 4) bad("lz4 block checksum");
      o += 4;
    }
  }
  return out;
}

// ------------------------------------------------------------------ snappy
size_t snappy_raw_into(const uint8_t* src, size_t n, uint8_t* dst, size_t o, size_t cap) {
  const uint8_t* p = src;
  const uint8_t* end = src + n;
  uint64_t want = 0;
  for (int shift = 0;; shift += 7) {
    if (p >= end || shift > 35) bad("snappy length");
    const uint8_t b = *p++;
    want |= uint64_t(b & 0x7f) << shift;
    if (!(b & 0x80)) break;
  }
  if (want > cap - o) throw NoRoom{};  // the declared size is checked before anything is written
  const size_t base = o, stop = o + want;
  while (p < end) {
    const uint8_t tag = *p++;
    const int type = tag & 3;
    if (type == 0) {  // literal
      size_t len = tag >> 2;
      if (len >= 60) {
        const int nb = int(len) - 59;
        if (end - p < nb) bad("snappy literal length");
        len = 0;
        for (int i = 0; i < nb; ++i) len |= size_t(p[i]) << (8 * i);
        p += nb;
      }
      len += 1;
      if (size_t(end - p) < len) bad("snappy literal");
      if (stop - o < len) bad("snappy size");
      std::memcpy(dst + o, p, len);
      o += len;
      p += len;
    } else {
      size_t len, off;
      if (type == 1) {
        if (p >= end) bad("snappy copy1");
        len = 4 + ((tag >> 2) & 7);
        off = (size_t(tag >> 5) << 8) | *p++;
      } else if (type == 2) {
        if (end - p < 2) bad("snappy copy2");
        len = 1 + (tag >> 2);
        off = size_t(p[0]) | (size_t(p[1]) << 8);
        p += 2;
      } else {
        if (end - p < 4) bad("snappy copy4");
        len = 1 + (tag >> 2);
        off = le32(p);
        p += 4;
      }
      if (off == 0 || off > o - base) bad("match offset");
      if (stop - o < len) bad("snappy size");
      match_copy(dst + o, off, len, 0);
      o += len;
    }
  }
  if (o != stop) bad("snappy size");
  return o;
}

size_t unsnappy(const uint8_t* src, size_t n, uint8_t* dst, size_t cap) {
  static const uint8_t kXerial[8] = {0x82, 'S', 'N', 'A', 'P', 'P', 'Y', 0};
  if (n >= 16 && std::memcmp(src, kXerial, 8) == 0) {  // xerial framing: header, then [BE len][block]...
    size_t o = 16, out = 0;
    while (o < n) {
      if (n - o < 4) bad("xerial block header");
      const uint32_t len = be32(src + o);
      o += 4;
      if (n - o < len) bad("xerial block");
      out = snappy_raw_into(src + o, len, dst, out, cap);
      o += len;
    }
    return out;
  }
  return snappy_raw_into(src, n, dst, 0, cap);
}

// ------------------------------------------------------------------ gzip
size_t gunzip_into(const uint8_t* src, size_t n, uint8_t* dst, size_t cap) {
  z_stream z{};
  if (inflateInit2(&z, 16 + MAX_WBITS) != Z_OK) bad("zlib init");
  z.next_in = const_cast<Bytef*>(src);
  z.avail_in = uInt(n);
  z.next_out = dst;
  z.avail_out = uInt(std::min<size_t>(cap, UINT_MAX));
  while (true) {
    const int rc = inflate(&z, Z_NO_FLUSH);
    if (rc == Z_STREAM_END) {
      // concatenated gzip members (some producers flush per message set)
      if (z.avail_in == 0 || inflateReset(&z) != Z_OK) break;
      continue;
    }
    if (rc == Z_OK) continue;
    const bool full = z.avail_out == 0;
    inflateEnd(&z);
    if (rc == Z_BUF_ERROR && full) throw NoRoom{};
    bad(rc == Z_BUF_ERROR ? "gzip stream truncated" : "gzip stream");
  }
  const size_t got = size_t(z.next_out - dst);
  inflateEnd(&z);
  return got;
}

// ------------------------------------------------------------------ zstd
// The image ships the system's libzstd.so.1 but no header, so the streaming decoder's stable ABI
// (zstd.h, v1.3+) is declared here and resolved once with dlopen.  Streaming, because producers
// (librdkafka, the Java client's ZstdOutputStream) may leave the frame content size out.
struct ZstdIn { const void* src; size_t size; size_t pos; };
struct ZstdOut { void* dst; size_t size; size_t pos; };
struct ZstdApi {
  void* (*create)() = nullptr;
  size_t (*free_ds)(void*) = nullptr;
  size_t (*init)(void*) = nullptr;
  size_t (*stream)(void*, ZstdOut*, ZstdIn*) = nullptr;
  unsigned (*is_error)(size_t) = nullptr;
  const char* (*error_name)(size_t) = nullptr;
  size_t (*compress)(void*, size_t, const void*, size_t, int) = nullptr;
  size_t (*bound)(size_t) = nullptr;
  bool ok = false;
};

const ZstdApi& zstd_api() {
  static ZstdApi api;
  static std::once_flag once;
  std::call_once(once, [] {
    void* h = dlopen("libzstd.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) return;
    api.create = reinterpret_cast<void* (*)()>(dlsym(h, "ZSTD_createDStream"));
    api.free_ds = reinterpret_cast<size_t (*)(void*)>(dlsym(h, "ZSTD_freeDStream"));
    api.init = reinterpret_cast<size_t (*)(void*)>(dlsym(h, "ZSTD_initDStream"));
    api.stream = reinterpret_cast<size_t (*)(void*, ZstdOut*, ZstdIn*)>(dlsym(h, "ZSTD_decompressStream"));
    api.is_error = reinterpret_cast<unsigned (*)(size_t)>(dlsym(h, "ZSTD_isError"));
    api.error_name = reinterpret_cast<const char* (*)(size_t)>(dlsym(h, "ZSTD_getErrorName"));
    api.compress = reinterpret_cast<size_t (*)(void*, size_t, const void*, size_t, int)>(dlsym(h, "ZSTD_compress"));
    api.bound = reinterpret_cast<size_t (*)(size_t)>(dlsym(h, "ZSTD_compressBound"));
    api.ok = api.create && api.free_ds && api.init && api.stream && api.is_error && api.error_name;
  });
  return api;
}

// One decoder context per thread (each fetch thread inflates its own responses), reset per call.
struct ZstdStream {
  void* ds = nullptr;
  ~ZstdStream() {
    if (ds) zstd_api().free_ds(ds);
  }
};

size_t unzstd(const uint8_t* src, size_t n, uint8_t* dst, size_t cap) {
  const ZstdApi& z = zstd_api();
  if (!z.ok) throw KafkaError("UnsupportedCodecError: zstd record batches need libzstd.so.1, which is not loadable");
  thread_local ZstdStream st;
  if (!st.ds) st.ds = z.create();
  if (!st.ds || z.is_error(z.init(st.ds))) bad("zstd init");
  ZstdIn in{src, n, 0};
  ZstdOut o{dst, cap, 0};
  size_t rc = 1;
  while (in.pos < in.size || rc != 0) {
    const size_t ip0 = in.pos, op0 = o.pos;
    rc = z.stream(st.ds, &o, &in);
    if (z.is_error(rc)) bad(std::string("zstd: ") + z.error_name(rc));
    if (in.pos == ip0 && o.pos == op0) {
      if (o.pos == o.size) throw NoRoom{};
      bad("zstd frame truncated");  // input exhausted mid-frame
    }
  }
  return o.pos;
}

// Runs a raw decoder into `out` (appending), growing the room up to max_out.
template <typename Fn>
void grow_into(std::vector<uint8_t>& out, size_t n, size_t max_out, Fn&& fn) {
  const size_t base = out.size();
  if (base > max_out) bad("inflated size exceeds the bound");
  size_t room = std::min(max_out - base, std::max<size_t>(n * 4, 64 << 10));
  while (true) {
    out.resize(base + room);
    try {
      const size_t got = fn(out.data() + base, room);
      out.resize(base + got);
      return;
    } catch (const NoRoom&) {
      if (room == max_out - base) {
        out.resize(base);
        bad("inflated size exceeds the bound");
      }
      room = std::min(max_out - base, room * 4);
    } catch (...) {
      out.resize(base);
      throw;
    }
  }
}

}  // namespace

bool zstd_available() { return zstd_api().ok; }
bool lz4_library_available() { return lz4_api().ok; }

size_t decompress_into(int codec, const uint8_t* src, size_t n, uint8_t* dst, size_t cap) {
  try {
    switch (codec) {
      case kCodecGzip: return gunzip_into(src, n, dst, cap);
      case kCodecSnappy: return unsnappy(src, n, dst, cap);
      case kCodecLz4: return unlz4_frame(src, n, dst, cap);
      case kCodecZstd: return unzstd(src, n, dst, cap);
      default:
        throw KafkaError(std::string("UnsupportedCodecError: ") + codec_name(codec) +
                         " record batches cannot be decoded (gzip, snappy, lz4 and zstd can)");
    }
  } catch (const NoRoom&) {
    return kNoRoom;
  } catch (const std::bad_alloc&) {
    bad("out of memory while inflating");
  }
}

void decompress(int codec, const uint8_t* src, size_t n, std::vector<uint8_t>& out, size_t max_out) {
  try {
    grow_into(out, n, max_out, [&](uint8_t* d, size_t cap) {
      const size_t got = decompress_into(codec, src, n, d, cap);
      if (got == kNoRoom) throw NoRoom{};
      return got;
    });
  } catch (const std::bad_alloc&) {
    bad("out of memory while inflating");
  } catch (const std::length_error&) {
    bad("inflated size exceeds the bound");
  }
}

void snappy_raw_decompress(const uint8_t* src, size_t n, std::vector<uint8_t>& out, size_t max_out) {
  grow_into(out, n, max_out, [&](uint8_t* d, size_t cap) { return snappy_raw_into(src, n, d, 0, cap); });
}

void lz4_block_decompress(const uint8_t* src, size_t n, std::vector<uint8_t>& out, size_t max_out) {
  grow_into(out, n, max_out, [&](uint8_t* d, size_t cap) { return lz4_block_raw(src, n, d, 0, cap, 0); });
}

void compress(int codec, const uint8_t* src, size_t n, std::vector<uint8_t>& out, int level) {
  switch (codec) {
    case kCodecGzip: {
      z_stream z{};
      if (deflateInit2(&z, level ? level : Z_DEFAULT_COMPRESSION, Z_DEFLATED, 16 + MAX_WBITS, 8,
                       Z_DEFAULT_STRATEGY) != Z_OK)
        throw KafkaError("gzip: deflateInit2 failed");
      const size_t base = out.size();
      out.resize(base + deflateBound(&z, uLong(n)));
      z.next_in = const_cast<Bytef*>(src);
      z.avail_in = uInt(n);
      z.next_out = out.data() + base;
      z.avail_out = uInt(out.size() - base);
      const int rc = deflate(&z, Z_FINISH);
      out.resize(base + z.total_out);
      deflateEnd(&z);
      if (rc != Z_STREAM_END) throw KafkaError("gzip: deflate failed");
      return;
    }
    case kCodecLz4: {
      const Lz4Api& lib = lz4_api();
      if (!lib.enc_ok) throw KafkaError("UnsupportedCodecError: lz4 compression needs liblz4.so.1, which is not loadable");
      // frame: independent 64 KiB blocks, no checksums (what the Java client's KafkaLZ4BlockOutputStream writes)
      const uint8_t desc[2] = {0x60, 0x40};
      put_le32(out, 0x184D2204u);
      out.push_back(desc[0]);
      out.push_back(desc[1]);
      out.push_back(uint8_t(xxh32_short(desc, 2) >> 8));
      constexpr size_t kBlock = 64 << 10;
      for (size_t a = 0; a < n; a += kBlock) {
        const int k = int(std::min(kBlock, n - a));
        const size_t at = out.size();
        const int bound = lib.bound(k);
        out.resize(at + 4 + size_t(bound));
        char* d = reinterpret_cast<char*>(out.data() + at + 4);
        const char* s = reinterpret_cast<const char*>(src + a);
        const int r = level >= 3 && lib.enc_hc ? lib.enc_hc(s, d, k, bound, level) : lib.enc(s, d, k, bound, 1);
        uint32_t word;
        if (r <= 0 || r >= k) {  // incompressible: stored
          std::memcpy(d, s, size_t(k));
          word = uint32_t(k) | 0x80000000u;
          out.resize(at + 4 + size_t(k));
        } else {
          word = uint32_t(r);
          out.resize(at + 4 + size_t(r));
        }
        for (int i = 0; i < 4; ++i) out[at + size_t(i)] = uint8_t(word >> (8 * i));
      }
      put_le32(out, 0);  // end mark
      return;
    }
    case kCodecZstd: {
      const ZstdApi& z = zstd_api();
      if (!z.ok || !z.compress || !z.bound)
        throw KafkaError("UnsupportedCodecError: zstd compression needs libzstd.so.1, which is not loadable");
      const size_t base = out.size();
      out.resize(base + z.bound(n));
      const size_t r = z.compress(out.data() + base, out.size() - base, src, n, level ? level : 3);
      if (z.is_error(r)) throw KafkaError(std::string("zstd: ") + z.error_name(r));
      out.resize(base + r);
      return;
    }
    default:
      throw KafkaError(std::string("UnsupportedCodecError: cannot compress ") + codec_name(codec) +
                       " record sets (gzip, lz4 and zstd can)");
  }
}

}  // namespace tk
