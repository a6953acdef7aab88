// Kafka RecordBatch v2 (magic = 2) wire format: encoder + zero-copy decoder.
//
// This is the on-log / on-wire format the synthetic broker stores and serves,
// exactly as a real broker stores producer batches and returns them in Fetch
// responses.  Uncompressed batches only (attributes bits 0-2 = 0).
//
//   baseOffset int64 | batchLength int32 | partitionLeaderEpoch int32 |
//   magic int8 | crc uint32 (CRC32C of attributes..end) | attributes int16 |
//   lastOffsetDelta int32 | baseTimestamp int64 | maxTimestamp int64 |
//   producerId int64 | producerEpoch int16 | baseSequence int32 |
//   recordCount int32 | records...
//   record: length varint | attributes int8 | timestampDelta varlong |
//           offsetDelta varint | keyLen varint | key | valueLen varint |
//           value | headerCount varint | (hKeyLen varint, hKey, hValLen varint, hVal)*
#pragma once
#include <cstddef>
#include <cstdint>
#include <vector>

#include "common.h"

namespace tk {

constexpr size_t kBatchHeaderBytes = 61;
constexpr size_t kBatchLengthOffset = 8;   // batchLength field
constexpr size_t kBatchCrcOffset = 17;     // crc field
constexpr size_t kBatchAttrOffset = 21;    // CRC covers [21, end)

// ------------------------------------------------------------ varints
inline size_t varint_size_u(uint64_t v) {
  size_t n = 1;
  while (v >= 0x80) { v >>= 7; ++n; }
  return n;
}
inline uint64_t zigzag(int64_t v) { return (uint64_t(v) << 1) ^ uint64_t(v >> 63); }
inline int64_t unzigzag(uint64_t v) { return int64_t(v >> 1) ^ -int64_t(v & 1); }
inline size_t varint_size(int64_t v) { return varint_size_u(zigzag(v)); }

inline uint8_t* put_varint(uint8_t* p, int64_t sv) {
  uint64_t v = zigzag(sv);
  while (v >= 0x80) { *p++ = uint8_t(v | 0x80); v >>= 7; }
  *p++ = uint8_t(v);
  return p;
}
// Returns nullptr on truncation / overlong encoding.
inline const uint8_t* get_varint(const uint8_t* p, const uint8_t* end, int64_t* out) {
  uint64_t v = 0;
  for (int shift = 0; shift < 70; shift += 7) {
    if (p >= end) return nullptr;
    uint8_t b = *p++;
    v |= uint64_t(b & 0x7F) << shift;
    if (!(b & 0x80)) { *out = unzigzag(v); return p; }
  }
  return nullptr;
}

// ------------------------------------------------------------ headers
struct BatchHeader {
  int64_t base_offset;
  int32_t batch_length;     // bytes after the batchLength field
  int32_t leader_epoch;
  int8_t magic;
  uint32_t crc;
  int16_t attributes;
  int32_t last_offset_delta;
  int64_t base_timestamp;
  int64_t max_timestamp;
  int64_t producer_id;
  int16_t producer_epoch;
  int32_t base_sequence;
  int32_t record_count;
  size_t total_size() const { return size_t(batch_length) + 12; }
  int64_t next_offset() const { return base_offset + last_offset_delta + 1; }
  int timestamp_type() const { return (attributes >> 3) & 1; }
};

// Parses the fixed 61-byte header.  Throws CorruptRecord when malformed (or compressed, unless
// `allow_compressed`: the replica ingest inflates those, codecs.h).
BatchHeader parse_batch_header(const uint8_t* p, size_t avail, bool allow_compressed = false);
// Verifies the CRC of a complete batch starting at p.
bool verify_batch_crc(const uint8_t* p, const BatchHeader& h);

struct RecordView {
  int64_t offset;
  int64_t timestamp;
  const uint8_t* key;      // nullptr when null
  int32_t key_len;         // -1 when null
  const uint8_t* value;
  int32_t value_len;
  const uint8_t* headers;  // start of the first header (raw)
  int32_t header_count;
  int32_t header_bytes;    // sum of header key + value lengths (kafka-python's serialized_header_size), -1 if none
};

// Iterates the records of one batch in order.  `next` returns false at the end.
class RecordIter {
 public:
  static constexpr int kPrefetchAhead = 8;
  RecordIter(const uint8_t* batch, const BatchHeader& h);
  bool next(RecordView* out);
  int remaining() const { return remaining_; }

 private:
  const uint8_t* p_;
  const uint8_t* end_;
  int64_t base_offset_, base_ts_;
  int remaining_;
};

// Parse header tuples of a record into (key, key_len, value, value_len) quads.
struct HeaderView {
  const uint8_t* key;
  int32_t key_len;
  const uint8_t* value;
  int32_t value_len;  // -1 for null
};
std::vector<HeaderView> parse_headers(const RecordView& r);

// ------------------------------------------------------------ encoder
struct RecordIn {
  int64_t timestamp;
  const uint8_t* key;
  int32_t key_len;  // -1 null
  const uint8_t* value;
  int32_t value_len;  // -1 null
  const HeaderView* headers;
  int32_t header_count;
};

// Exact encoded size of one record's body (excluding its own length varint).
size_t record_body_size(const RecordIn& r, int64_t ts_delta, int32_t off_delta);
// Size of a whole batch holding `recs`.
size_t batch_encoded_size(const RecordIn* recs, size_t n, int64_t base_ts);
// Encodes a batch at `out` (capacity must be >= batch_encoded_size).  Returns bytes written.
size_t encode_batch(uint8_t* out, int64_t base_offset, const RecordIn* recs, size_t n, bool log_append_time = false);

}  // namespace tk
