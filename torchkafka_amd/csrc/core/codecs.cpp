// Kafka record-set decompression: see codecs.h.
#include "codecs.h"

#include <dlfcn.h>
#include <zlib.h>

#include <cstring>
#include <memory>
#include <new>
#include <stdexcept>
#include <mutex>
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

[[noreturn]] void bad(const char* what) { throw CorruptRecord(std::string("corrupt compressed record set: ") + what); }

uint32_t be32(const uint8_t* p) { return (uint32_t(p[0]) << 24) | (uint32_t(p[1]) << 16) | (uint32_t(p[2]) << 8) | p[3]; }
uint32_t le32(const uint8_t* p) { return uint32_t(p[0]) | (uint32_t(p[1]) << 8) | (uint32_t(p[2]) << 16) | (uint32_t(p[3]) << 24); }

// Output would exceed the caller's bound.
void room(const std::vector<uint8_t>& out, size_t add, size_t max_out) {
  if (add > max_out || out.size() > max_out - add) bad("inflated size exceeds the bound");
}

// Back-reference copy; may overlap its own output (offset < length repeats a pattern).
void copy_match(std::vector<uint8_t>& out, size_t base, size_t offset, size_t len, size_t max_out) {
  if (offset == 0 || offset > out.size() - base) bad("match offset");
  room(out, len, max_out);
  size_t from = out.size() - offset;
  out.reserve(out.size() + len);
  for (size_t i = 0; i < len; ++i) out.push_back(out[from + i]);
}

void gunzip(const uint8_t* src, size_t n, std::vector<uint8_t>& out, size_t max_out) {
  z_stream z{};
  if (inflateInit2(&z, 16 + MAX_WBITS) != Z_OK) bad("zlib init");
  z.next_in = const_cast<Bytef*>(src);
  z.avail_in = uInt(n);
  int rc = Z_OK;
  while (rc != Z_STREAM_END) {
    const size_t old = out.size();
    if (old >= max_out) {
      inflateEnd(&z);
      bad("inflated size exceeds the bound");
    }
    out.resize(old + std::min<size_t>(std::max<size_t>(n * 2, 64 << 10), max_out - old));
    z.next_out = out.data() + old;
    z.avail_out = uInt(out.size() - old);
    rc = inflate(&z, Z_NO_FLUSH);
    out.resize(out.size() - z.avail_out);
    if (rc == Z_STREAM_END) {
      // concatenated gzip members (some producers flush per message set)
      if (z.avail_in == 0) break;
      if (inflateReset(&z) != Z_OK) break;
      rc = Z_OK;
      continue;
    }
    if (rc != Z_OK && !(rc == Z_BUF_ERROR && z.avail_in)) {
      inflateEnd(&z);
      bad("gzip stream");
    }
  }
  inflateEnd(&z);
}

}  // namespace

void snappy_raw_decompress(const uint8_t* src, size_t n, std::vector<uint8_t>& out, size_t max_out) {
  const uint8_t* p = src;
  const uint8_t* end = src + n;
  uint64_t want = 0;
  for (int shift = 0;; shift += 7) {
    if (p >= end || shift > 35) bad("snappy length");
    const uint8_t b = *p++;
    want |= uint64_t(b & 0x7f) << shift;
    if (!(b & 0x80)) break;
  }
  const size_t base = out.size();
  room(out, want, max_out);  // the declared size is checked before anything is reserved for it
  out.reserve(base + want);
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
      room(out, len, max_out);
      out.insert(out.end(), p, p + len);
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
      copy_match(out, base, off, len, max_out);
    }
  }
  if (out.size() - base != want) bad("snappy size");
}

void lz4_block_decompress(const uint8_t* src, size_t n, std::vector<uint8_t>& out, size_t max_out) {
  const uint8_t* p = src;
  const uint8_t* end = src + n;
  const size_t base = out.size();
  while (p < end) {
    const uint8_t token = *p++;
    size_t lit = token >> 4;
    if (lit == 15) {
      uint8_t b;
      do {
        if (p >= end) bad("lz4 literal length");
        b = *p++;
        lit += b;
      } while (b == 255);
    }
    if (size_t(end - p) < lit) bad("lz4 literals");
    room(out, lit, max_out);
    out.insert(out.end(), p, p + lit);
    p += lit;
    if (p == end) break;  // the last sequence has literals only
    if (end - p < 2) bad("lz4 offset");
    const size_t off = size_t(p[0]) | (size_t(p[1]) << 8);
    p += 2;
    size_t len = token & 15;
    if (len == 15) {
      uint8_t b;
      do {
        if (p >= end) bad("lz4 match length");
        b = *p++;
        len += b;
      } while (b == 255);
    }
    copy_match(out, base, off, len + 4, max_out);
  }
}

namespace {

void unsnappy(const uint8_t* src, size_t n, std::vector<uint8_t>& out, size_t max_out) {
  static const uint8_t kXerial[8] = {0x82, 'S', 'N', 'A', 'P', 'P', 'Y', 0};
  if (n >= 16 && std::memcmp(src, kXerial, 8) == 0) {  // xerial framing: header, then [BE len][block]...
    size_t o = 16;
    while (o < n) {
      if (n - o < 4) bad("xerial block header");
      const uint32_t len = be32(src + o);
      o += 4;
      if (n - o < len) bad("xerial block");
      snappy_raw_decompress(src + o, len, out, max_out);
      o += len;
    }
    return;
  }
  snappy_raw_decompress(src, n, out, max_out);
}

void unlz4_frame(const uint8_t* src, size_t n, std::vector<uint8_t>& out, size_t max_out) {
  if (n < 7 || le32(src) != 0x184D2204u) bad("lz4 frame magic");
  const uint8_t flg = src[4];
  if ((flg >> 6) != 1) bad("lz4 frame version");
  size_t o = 6;                     // magic, FLG, BD
  if (flg & 0x08) o += 8;           // content size
  if (flg & 0x01) o += 4;           // dictionary id
  o += 1;                           // header checksum
  if (o > n) bad("lz4 frame header");  // invariant from here on: o <= n, so n - o never wraps
  const bool block_sum = flg & 0x10;
  while (true) {
    if (n - o < 4) bad("lz4 block size");
    const uint32_t word = le32(src + o);
    o += 4;
    if (word == 0) break;           // end mark
    const uint32_t len = word & 0x7fffffffu;
    if (n - o < len) bad("lz4 block");
    if (word & 0x80000000u) {       // stored uncompressed
      room(out, len, max_out);
      out.insert(out.end(), src + o, src + o + len);
    } else {
      lz4_block_decompress(src + o, len, out, max_out);
    }
    o += len;
    if (block_sum) {
      if (n - o < 4) bad("lz4 block checksum");
      o += 4;
    }
  }
}

// zstd: the image ships the system's libzstd.so.1 but no header, so the streaming decoder's stable
// ABI (zstd.h, v1.3+) is declared here and resolved once with dlopen.  Streaming, because producers
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
    api.ok = api.create && api.free_ds && api.init && api.stream && api.is_error && api.error_name;
  });
  return api;
}

void unzstd(const uint8_t* src, size_t n, std::vector<uint8_t>& out, size_t max_out) {
  const ZstdApi& z = zstd_api();
  if (!z.ok) throw KafkaError("UnsupportedCodecError: zstd record batches need libzstd.so.1, which is not loadable");
  std::unique_ptr<void, size_t (*)(void*)> ds(z.create(), z.free_ds);
  if (!ds || z.is_error(z.init(ds.get()))) bad("zstd init");
  ZstdIn in{src, n, 0};
  size_t rc = 1;
  while (in.pos < in.size || rc != 0) {
    const size_t old = out.size();
    if (old >= max_out) bad("inflated size exceeds the bound");
    out.resize(old + std::min<size_t>(std::max<size_t>(n * 4, 128 << 10), max_out - old));
    ZstdOut o{out.data() + old, out.size() - old, 0};
    const size_t in_before = in.pos;
    rc = z.stream(ds.get(), &o, &in);
    out.resize(old + o.pos);
    if (z.is_error(rc)) bad((std::string("zstd: ") + z.error_name(rc)).c_str());
    // input exhausted mid-frame with no progress: the frame is truncated
    if (rc != 0 && in.pos == in.size && o.pos == 0 && in.pos == in_before) bad("zstd frame truncated");
  }
}

}  // namespace

bool zstd_available() { return zstd_api().ok; }

void decompress(int codec, const uint8_t* src, size_t n, std::vector<uint8_t>& out, size_t max_out) {
  try {
    switch (codec) {
      case kCodecGzip: gunzip(src, n, out, max_out); return;
      case kCodecSnappy: unsnappy(src, n, out, max_out); return;
      case kCodecLz4: unlz4_frame(src, n, out, max_out); return;
      case kCodecZstd: unzstd(src, n, out, max_out); return;
      default:
        throw KafkaError(std::string("UnsupportedCodecError: ") + codec_name(codec) +
                         " record batches cannot be decoded (gzip, snappy, lz4 and zstd can)");
    }
  } catch (const std::bad_alloc&) {
    bad("out of memory while inflating");
  } catch (const std::length_error&) {
    bad("inflated size exceeds the bound");
  }
}

}  // namespace tk
