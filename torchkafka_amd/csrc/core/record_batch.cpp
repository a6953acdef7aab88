#include "record_batch.h"

#include "crc32c.h"

namespace tk {

BatchHeader parse_batch_header(const uint8_t* p, size_t avail, bool allow_compressed) {
  if (avail < kBatchHeaderBytes) throw CorruptRecord("truncated record batch header");
  BatchHeader h;
  h.base_offset = int64_t(get_be64(p));
  h.batch_length = int32_t(get_be32(p + 8));
  h.leader_epoch = int32_t(get_be32(p + 12));
  h.magic = int8_t(p[16]);
  h.crc = get_be32(p + 17);
  h.attributes = int16_t(get_be16(p + 21));
  h.last_offset_delta = int32_t(get_be32(p + 23));
  h.base_timestamp = int64_t(get_be64(p + 27));
  h.max_timestamp = int64_t(get_be64(p + 35));
  h.producer_id = int64_t(get_be64(p + 43));
  h.producer_epoch = int16_t(get_be16(p + 51));
  h.base_sequence = int32_t(get_be32(p + 53));
  h.record_count = int32_t(get_be32(p + 57));
  if (h.magic != 2) throw CorruptRecord("unsupported record batch magic " + std::to_string(int(h.magic)));
  if (h.batch_length < int32_t(kBatchHeaderBytes - 12) || h.total_size() > avail)
    throw CorruptRecord("record batch length out of range");
  if ((h.attributes & 0x7) && !allow_compressed)
    throw CorruptRecord("compressed record batches are not supported (a KafkaBridge replica stores them inflated)");
  if (h.record_count < 0) throw CorruptRecord("negative record count");
  return h;
}

bool verify_batch_crc(const uint8_t* p, const BatchHeader& h) {
  return crc32c(p + kBatchAttrOffset, h.total_size() - kBatchAttrOffset) == h.crc;
}

RecordIter::RecordIter(const uint8_t* batch, const BatchHeader& h)
    : p_(batch + kBatchHeaderBytes),
      end_(batch + h.total_size()),
      base_offset_(h.base_offset),
      base_ts_(h.base_timestamp),
      remaining_(h.record_count) {}

bool RecordIter::next(RecordView* r) {
  if (remaining_ <= 0) return false;
  int64_t len;
  const uint8_t* p = get_varint(p_, end_, &len);
  if (!p || len < 0 || p + len > end_) throw CorruptRecord("bad record length");
  const uint8_t* rend = p + len;
  p += 1;  // attributes
  int64_t ts_delta, off_delta, klen, vlen, hcount;
  if (!(p = get_varint(p, rend, &ts_delta))) throw CorruptRecord("bad timestamp delta");
  if (!(p = get_varint(p, rend, &off_delta))) throw CorruptRecord("bad offset delta");
  if (!(p = get_varint(p, rend, &klen))) throw CorruptRecord("bad key length");
  if (klen >= 0) {
    if (p + klen > rend) throw CorruptRecord("key overruns record");
    r->key = p;
    r->key_len = int32_t(klen);
    p += klen;
  } else {
    r->key = nullptr;
    r->key_len = -1;
  }
  if (!(p = get_varint(p, rend, &vlen))) throw CorruptRecord("bad value length");
  if (vlen >= 0) {
    if (p + vlen > rend) throw CorruptRecord("value overruns record");
    r->value = p;
    r->value_len = int32_t(vlen);
    p += vlen;
  } else {
    r->value = nullptr;
    r->value_len = -1;
  }
  if (!(p = get_varint(p, rend, &hcount))) throw CorruptRecord("bad header count");
  r->headers = p;
  r->header_count = int32_t(hcount);
  if (hcount > 0) {
    int64_t bytes = 0;
    const uint8_t* q = p;
    for (int64_t i = 0; i < hcount; ++i) {
      int64_t hk, hv;
      if (!(q = get_varint(q, rend, &hk)) || hk < 0 || q + hk > rend) throw CorruptRecord("bad header key");
      q += hk;
      bytes += hk;
      if (!(q = get_varint(q, rend, &hv)) || q + (hv > 0 ? hv : 0) > rend) throw CorruptRecord("bad header value");
      if (hv > 0) { q += hv; bytes += hv; }
    }
    r->header_bytes = int32_t(bytes);
  } else {
    r->header_bytes = -1;
  }
  r->offset = base_offset_ + off_delta;
  r->timestamp = base_ts_ + ts_delta;
  // The walk is a chain of dependent loads (each record's length varint locates the next).  A
  // consumer that skips the values (the device-decode walk) would pay one DRAM miss per
  // record; records of one batch usually have the same size, so prefetch where the record
  // kPrefetchAhead positions further down would start if they all had this one's size.
  {
    const ptrdiff_t step = rend - p_;
    const uint8_t* ahead = rend + kPrefetchAhead * step;
    if (ahead < end_) __builtin_prefetch(ahead);
  }
  p_ = rend;
  --remaining_;
  return true;
}

std::vector<HeaderView> parse_headers(const RecordView& r) {
  std::vector<HeaderView> out;
  const uint8_t* q = r.headers;
  const uint8_t* end = q + (1u << 30);  // bounds were validated by RecordIter
  for (int i = 0; i < r.header_count; ++i) {
    int64_t hk, hv;
    q = get_varint(q, end, &hk);
    HeaderView h;
    h.key = q;
    h.key_len = int32_t(hk);
    q += hk;
    q = get_varint(q, end, &hv);
    h.value = hv >= 0 ? q : nullptr;
    h.value_len = int32_t(hv);
    if (hv > 0) q += hv;
    out.push_back(h);
  }
  return out;
}

size_t record_body_size(const RecordIn& r, int64_t ts_delta, int32_t off_delta) {
  size_t n = 1;  // attributes
  n += varint_size(ts_delta) + varint_size(off_delta);
  n += varint_size(r.key_len) + (r.key_len > 0 ? size_t(r.key_len) : 0);
  n += varint_size(r.value_len) + (r.value_len > 0 ? size_t(r.value_len) : 0);
  n += varint_size(r.header_count);
  for (int32_t i = 0; i < r.header_count; ++i) {
    const HeaderView& h = r.headers[i];
    n += varint_size(h.key_len) + size_t(h.key_len);
    n += varint_size(h.value_len) + (h.value_len > 0 ? size_t(h.value_len) : 0);
  }
  return n;
}

size_t batch_encoded_size(const RecordIn* recs, size_t n, int64_t base_ts) {
  size_t total = kBatchHeaderBytes;
  for (size_t i = 0; i < n; ++i) {
    size_t body = record_body_size(recs[i], recs[i].timestamp - base_ts, int32_t(i));
    total += varint_size(int64_t(body)) + body;
  }
  return total;
}

size_t encode_batch(uint8_t* out, int64_t base_offset, const RecordIn* recs, size_t n, bool log_append_time) {
  if (n == 0) throw std::invalid_argument("empty record batch");
  int64_t base_ts = recs[0].timestamp, max_ts = recs[0].timestamp;
  for (size_t i = 1; i < n; ++i) {
    if (recs[i].timestamp < base_ts) base_ts = recs[i].timestamp;
    if (recs[i].timestamp > max_ts) max_ts = recs[i].timestamp;
  }
  uint8_t* p = out + kBatchHeaderBytes;
  for (size_t i = 0; i < n; ++i) {
    const RecordIn& r = recs[i];
    const int64_t ts_delta = r.timestamp - base_ts;
    const size_t body = record_body_size(r, ts_delta, int32_t(i));
    p = put_varint(p, int64_t(body));
    *p++ = 0;  // record attributes (unused)
    p = put_varint(p, ts_delta);
    p = put_varint(p, int64_t(i));
    p = put_varint(p, r.key_len);
    if (r.key_len > 0) { std::memcpy(p, r.key, size_t(r.key_len)); p += r.key_len; }
    p = put_varint(p, r.value_len);
    if (r.value_len > 0) { std::memcpy(p, r.value, size_t(r.value_len)); p += r.value_len; }
    p = put_varint(p, r.header_count);
    for (int32_t h = 0; h < r.header_count; ++h) {
      const HeaderView& hv = r.headers[h];
      p = put_varint(p, hv.key_len);
      if (hv.key_len > 0) std::memcpy(p, hv.key, size_t(hv.key_len));  // empty key: pointer may be null
      p += hv.key_len;
      p = put_varint(p, hv.value_len);
      if (hv.value_len > 0) { std::memcpy(p, hv.value, size_t(hv.value_len)); p += hv.value_len; }
    }
  }
  const size_t total = size_t(p - out);
  put_be64(out, uint64_t(base_offset));
  put_be32(out + 8, uint32_t(total - 12));
  put_be32(out + 12, 0);       // partitionLeaderEpoch
  out[16] = 2;                 // magic
  const int16_t attrs = log_append_time ? int16_t(1 << 3) : int16_t(0);
  put_be16(out + 21, uint16_t(attrs));
  put_be32(out + 23, uint32_t(n - 1));
  put_be64(out + 27, uint64_t(base_ts));
  put_be64(out + 35, uint64_t(max_ts));
  put_be64(out + 43, uint64_t(int64_t(-1)));  // producerId (non-idempotent)
  put_be16(out + 51, uint16_t(int16_t(-1)));
  put_be32(out + 53, uint32_t(int32_t(-1)));
  put_be32(out + 57, uint32_t(n));
  put_be32(out + 17, crc32c(out + kBatchAttrOffset, total - kBatchAttrOffset));
  return total;
}

}  // namespace tk
