// Host-sanitizer fuzz test of the RecordBatch v2 codec, CRC32C and the JSON parser
// (built with -fsanitize=address,undefined by tools/sanitize.sh).  Every decode of a randomly
// corrupted batch must either throw CorruptRecord or stay inside the buffer; ASan turns an
// out-of-bounds read into a failure.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "codecs.h"
#include "consumer.h"
#include "crc32c.h"
#include "record_batch.h"

using namespace tk;

#define CHECK(c)                                                                  \
  do {                                                                            \
    if (!(c)) {                                                                   \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c);   \
      std::abort();                                                               \
    }                                                                             \
  } while (0)

int main(int argc, char** argv) {
  const int iters = argc > 1 ? std::atoi(argv[1]) : 3000;
  std::mt19937_64 rng(12345);
  uint64_t decoded = 0, rejected = 0;
  for (int it = 0; it < iters; ++it) {
    const int n = 1 + int(rng() % 20);
    std::vector<std::vector<uint8_t>> keys(n), vals(n), hk(n), hv(n);
    std::vector<HeaderView> hdrs(n);
    std::vector<RecordIn> recs(n);
    for (int i = 0; i < n; ++i) {
      keys[i].resize(rng() % 9);
      vals[i].resize(rng() % 300);
      for (auto& c : vals[i]) c = uint8_t(rng());
      hk[i].assign(rng() % 5, 'h');
      hv[i].assign(rng() % 5, 'v');
      hdrs[i] = HeaderView{hk[i].data(), int32_t(hk[i].size()), hv[i].data(), int32_t(hv[i].size())};
      const bool null_key = rng() % 3 == 0, null_val = rng() % 5 == 0;
      recs[i] = RecordIn{int64_t(1000 + i), null_key ? nullptr : keys[i].data(), null_key ? -1 : int32_t(keys[i].size()),
                         null_val ? nullptr : vals[i].data(), null_val ? -1 : int32_t(vals[i].size()),
                         rng() % 2 ? &hdrs[i] : nullptr, 0};
      recs[i].header_count = recs[i].headers ? 1 : 0;
    }
    const size_t sz = batch_encoded_size(recs.data(), n, 1000);
    std::vector<uint8_t> buf(sz);
    CHECK(encode_batch(buf.data(), int64_t(it) * 100, recs.data(), n) == sz);
    // clean decode round trip
    BatchHeader h = parse_batch_header(buf.data(), buf.size());
    CHECK(verify_batch_crc(buf.data(), h));
    RecordIter ri(buf.data(), h);
    RecordView rv;
    int k = 0;
    while (ri.next(&rv)) {
      CHECK(rv.value_len == recs[k].value_len);
      if (rv.value_len > 0) CHECK(std::memcmp(rv.value, recs[k].value, size_t(rv.value_len)) == 0);
      ++k;
    }
    CHECK(k == n);
    // corrupt 1-4 bytes (header or body) and decode from an exact-size heap copy
    std::vector<uint8_t> bad(buf);
    const int flips = 1 + int(rng() % 4);
    for (int f = 0; f < flips; ++f) bad[rng() % bad.size()] ^= uint8_t(1 + rng() % 255);
    uint8_t* p = static_cast<uint8_t*>(std::malloc(bad.size()));
    std::memcpy(p, bad.data(), bad.size());
    try {
      BatchHeader hb = parse_batch_header(p, bad.size());
      if (hb.total_size() <= bad.size()) {
        (void)verify_batch_crc(p, hb);
        RecordIter rb(p, hb);
        RecordView r2;
        while (rb.next(&r2)) {
          if (r2.value_len > 0) CHECK(r2.value >= p && r2.value + r2.value_len <= p + bad.size());
          if (r2.header_count > 0) (void)parse_headers(r2);
        }
      }
      ++decoded;
    } catch (const CorruptRecord&) {
      ++rejected;
    } catch (const std::exception&) {
      ++rejected;
    }
    std::free(p);
    // CRC32C: extend() over splits equals one pass
    const size_t cut = bad.size() ? rng() % bad.size() : 0;
    CHECK(crc32c_extend(crc32c(bad.data(), cut), bad.data() + cut, bad.size() - cut) == crc32c(bad.data(), bad.size()));
  }
  // JSON parser on random printable strings and on mutated arrays
  std::vector<float> out(512);
  const char alphabet[] = "[],.-+eE0123456789 NaInfity";
  for (int it = 0; it < iters * 4; ++it) {
    const size_t len = rng() % 64;
    char* s = static_cast<char*>(std::malloc(len ? len : 1));
    for (size_t i = 0; i < len; ++i) s[i] = alphabet[rng() % (sizeof(alphabet) - 1)];
    const int64_t got = parse_json_f32(s, len, out.data(), int64_t(out.size()));
    CHECK(got >= -2 && got <= int64_t(out.size()));
    const int64_t n2 = json_array_len(s, len);
    CHECK(n2 >= -1);
    std::free(s);
  }
  // decompressors (replica ingest of compressed record sets): random and mutated inputs must
  // either decode or throw CorruptRecord, never read or write outside their buffers
  uint64_t inflated = 0, refused = 0;
  for (int it = 0; it < iters * 4; ++it) {
    std::vector<uint8_t> in(rng() % 512);
    for (auto& c : in) c = uint8_t(rng() % 4 == 0 ? rng() : (rng() % 8));
    if (it % 3 == 1 && in.size() >= 7) {  // an LZ4 frame header in front
      const uint8_t hdr[7] = {0x04, 0x22, 0x4D, 0x18, 0x60, 0x40, 0x82};
      std::memcpy(in.data(), hdr, 7);
    }
    const int codec = it % 3 == 0 ? kCodecSnappy : it % 3 == 1 ? kCodecLz4 : -1;
    std::vector<uint8_t> out;
    try {
      if (codec < 0) snappy_raw_decompress(in.data(), in.size(), out);
      else decompress(codec, in.data(), in.size(), out);
      ++inflated;
    } catch (const CorruptRecord&) {
      ++refused;
    }
    std::vector<uint8_t> out2;
    try {
      lz4_block_decompress(in.data(), in.size(), out2);
      ++inflated;
    } catch (const CorruptRecord&) {
      ++refused;
    }
  }
  // LZ4 frames whose FLG announces a content size (0x08) and/or a dictionary id (0x01) or block
  // checksums (0x10), cut short anywhere in the header: the parser must refuse them, never read
  // past the (exact-size, heap) input
  const uint8_t flgs[] = {0x68, 0x61, 0x69, 0x70, 0x78, 0x79};
  for (uint8_t flg : flgs) {
    for (size_t n = 7; n <= 32; ++n) {
      uint8_t* in = static_cast<uint8_t*>(std::malloc(n));
      const uint8_t hdr[6] = {0x04, 0x22, 0x4D, 0x18, flg, 0x40};
      std::memcpy(in, hdr, 6);
      for (size_t i = 6; i < n; ++i) in[i] = uint8_t(rng() % 3 == 0 ? 0 : rng());
      std::vector<uint8_t> out;
      try {
        decompress(kCodecLz4, in, n, out);
        ++inflated;
      } catch (const CorruptRecord&) {
        ++refused;
      }
      std::free(in);
    }
  }
  // output bounds: a snappy stream declaring 2^40 bytes, and real output past a small bound,
  // are CorruptRecord -- not bad_alloc / length_error, which the replica would retry forever
  {
    const uint8_t huge[] = {0x80, 0x80, 0x80, 0x80, 0x80, 0x20, 0x00};
    std::vector<uint8_t> out;
    bool threw = false;
    try {
      decompress(kCodecSnappy, huge, sizeof(huge), out);
    } catch (const CorruptRecord&) {
      threw = true;
    }
    CHECK(threw);
    // literal run of 200 bytes then a 4 KiB repeat: over a 1 KiB bound
    std::vector<uint8_t> blk;
    blk.push_back(uint8_t(0xFF));  // 15 literals (+ext), match length 15 (+ext)
    blk.push_back(uint8_t(200 - 15));
    for (int i = 0; i < 200; ++i) blk.push_back(uint8_t(i));
    blk.push_back(1);
    blk.push_back(0);                      // offset 1
    for (int i = 0; i < 16; ++i) blk.push_back(255);
    blk.push_back(0);
    blk.push_back(0x00);                   // final sequence: no literals
    std::vector<uint8_t> o2;
    threw = false;
    try {
      lz4_block_decompress(blk.data(), blk.size(), o2, 1024);
    } catch (const CorruptRecord&) {
      threw = true;
    }
    CHECK(threw && o2.size() <= 1024);
  }
  // round trips through compress() (gzip, lz4 frame, zstd) into exact-size heap buffers: the
  // exact size decodes, one byte less is kNoRoom, never a write past the buffer (ASan); mutated
  // compressed bytes decode, refuse or report kNoRoom within the buffer
  uint64_t trips = 0;
  for (int it = 0; it < iters / 4 + 3; ++it) {
    const size_t n = 1 + size_t(rng() % (it % 7 == 0 ? 300000 : 5000));
    std::vector<uint8_t> plain(n);
    const int alpha = 1 + int(rng() % 40);
    for (size_t i = 0; i < n; ++i)
      plain[i] = i > 20 && rng() % 3 ? plain[i - 1 - rng() % 20] : uint8_t(rng() % alpha);
    for (int codec : {kCodecGzip, kCodecLz4, kCodecZstd}) {
      if (codec == kCodecZstd && !zstd_available()) continue;
      std::vector<uint8_t> z;
      try {
        compress(codec, plain.data(), n, z, it % 5 == 0 ? 9 : 0);
      } catch (const KafkaError&) {
        continue;  // the system library is not loadable
      }
      for (size_t cap : {n, n - 1, size_t(rng() % n)}) {
        uint8_t* d = static_cast<uint8_t*>(std::malloc(cap ? cap : 1));
        const size_t got = decompress_into(codec, z.data(), z.size(), d, cap);
        if (cap >= n) CHECK(got == n && std::memcmp(d, plain.data(), n) == 0);
        else CHECK(got == kNoRoom);
        std::free(d);
      }
      std::vector<uint8_t> zb(z);
      zb[rng() % zb.size()] ^= uint8_t(1 + rng() % 255);
      uint8_t* zi = static_cast<uint8_t*>(std::malloc(zb.size()));
      std::memcpy(zi, zb.data(), zb.size());
      const size_t cap = size_t(rng() % (2 * n + 1));
      uint8_t* d = static_cast<uint8_t*>(std::malloc(cap ? cap : 1));
      try {
        const size_t got = decompress_into(codec, zi, zb.size(), d, cap);
        CHECK(got == kNoRoom || got <= cap);
      } catch (const CorruptRecord&) {
        ++refused;
      }
      std::free(d);
      std::free(zi);
      ++trips;
    }
  }
  std::printf("codec round trips: %llu (liblz4 decoder %s)\n", (unsigned long long)trips,
              lz4_library_available() ? "on" : "off");
  std::printf("codec fuzz: %d batches, %llu corrupted decodes survived, %llu rejected; JSON fuzz ok; "
              "decompressors: %llu decoded, %llu refused\n", iters,
              (unsigned long long)decoded, (unsigned long long)rejected, (unsigned long long)inflated,
              (unsigned long long)refused);
  return 0;
}
