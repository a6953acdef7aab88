#include "consumer.h"

#include <sys/mman.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <cstdlib>
#include <limits>

#if defined(__x86_64__)
#include <immintrin.h>
#endif

namespace tk {

void Fetcher::assign(const std::vector<uint32_t>& pidxs, const std::vector<int64_t>& positions) {
  if (pidxs.size() != positions.size()) throw std::invalid_argument("assign: size mismatch");
  std::vector<FetchPart> np;
  for (size_t i = 0; i < pidxs.size(); ++i) {
    b_->part(pidxs[i]);  // validates
    FetchPart fp;
    fp.pidx = pidxs[i];
    fp.position = positions[i];
    // keep decode caches of partitions that stay assigned at the same position
    for (const auto& old : parts_) {
      if (old.pidx == fp.pidx) fp.populated_end = old.populated_end;
      if (old.pidx == fp.pidx && old.position == fp.position) {
        fp.batch_hint = old.batch_hint;
        fp.verified_base = old.verified_base;
        fp.paused = old.paused;
      }
    }
    np.push_back(fp);
  }
  parts_ = std::move(np);
}

size_t Fetcher::find(uint32_t pidx) const {
  for (size_t i = 0; i < parts_.size(); ++i)
    if (parts_[i].pidx == pidx) return i;
  return size_t(-1);
}

bool Fetcher::has_data(const FetchPart& fp) {
  const PartitionEntry& P = b_->part(fp.pidx);
  const int64_t hw = P.high_watermark.load(std::memory_order_acquire);
  if (fp.position > hw || fp.position < P.log_start_offset.load(std::memory_order_acquire))
    throw OffsetOutOfRange("OffsetOutOfRangeError: position " + std::to_string(fp.position) +
                           " outside [" + std::to_string(P.log_start_offset.load()) + ", " + std::to_string(hw) +
                           "] of partition index " + std::to_string(fp.pidx));
  return fp.position < hw;
}

void Fetcher::prefault(FetchPart& fp, const uint8_t* log, uint64_t pos, uint64_t log_end, uint64_t ring) {
  static const long page = sysconf(_SC_PAGESIZE);
  const uint64_t pg = uint64_t(page > 0 ? page : 4096);
  const uint64_t lo = std::max<uint64_t>(pos, fp.populated_end) & ~(pg - 1);
  const uint64_t hi = ring ? (ring + pg - 1) & ~(pg - 1)  // the whole ring (its pages exist: populate_ring)
                           : std::min<uint64_t>(pos + kPrefaultBytes, (log_end + pg - 1) & ~(pg - 1));
  if (hi > lo && prefault_ok_) {
#ifdef MADV_POPULATE_READ
    if (madvise(const_cast<uint8_t*>(log) + lo, hi - lo, MADV_POPULATE_READ) != 0 && errno == EINVAL)
      prefault_ok_ = false;  // kernel < 5.14: fall back to faulting pages on first touch
#else
    prefault_ok_ = false;
#endif
  }
  fp.populated_end = std::max<uint64_t>(hi, pos + 1);
}

// ------------------------------------------------------------ streaming copy
namespace {

// Copies record values into a ring slot.  The slot is never read again by
// this CPU -- the GPU's DMA engine reads it -- so 32-byte-aligned
// destinations use non-temporal stores: no read-for-ownership of the
// destination lines and no eviction of the log data being decoded.  Ordering:
// Ring::worker_publish issues an sfence before the slot's release store.
#if defined(__x86_64__)
__attribute__((target("avx2"))) void copy_nt_avx2(uint8_t* dst, const uint8_t* src, size_t n) {
  size_t i = 0;
  for (; i + 128 <= n; i += 128) {
    const __m256i a = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(src + i));
    const __m256i b = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(src + i + 32));
    const __m256i c = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(src + i + 64));
    const __m256i d = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(src + i + 96));
    _mm256_stream_si256(reinterpret_cast<__m256i*>(dst + i), a);
    _mm256_stream_si256(reinterpret_cast<__m256i*>(dst + i + 32), b);
    _mm256_stream_si256(reinterpret_cast<__m256i*>(dst + i + 64), c);
    _mm256_stream_si256(reinterpret_cast<__m256i*>(dst + i + 96), d);
  }
  for (; i + 32 <= n; i += 32)
    _mm256_stream_si256(reinterpret_cast<__m256i*>(dst + i),
                        _mm256_loadu_si256(reinterpret_cast<const __m256i*>(src + i)));
  if (i < n) std::memcpy(dst + i, src + i, n - i);
}
bool nt_enabled() {
  const char* e = std::getenv("TORCHKAFKA_NT_COPY");
  return __builtin_cpu_supports("avx2") && !(e && e[0] == '0');
}
const bool g_avx2 = nt_enabled();
#endif

inline void copy_to_slot(uint8_t* dst, const uint8_t* src, size_t n) {
#if defined(__x86_64__)
  if (n >= 256 && g_avx2 && (reinterpret_cast<uintptr_t>(dst) & 31) == 0) {
    copy_nt_avx2(dst, src, n);
    return;
  }
#endif
  std::memcpy(dst, src, n);
}

}  // namespace

// ------------------------------------------------------------ device-decode segments (span.h)
namespace {

// A RecordBatch a span fill walked into, and the slot rows [row_first, row_last) taken from it.
struct SpanRB {
  uint32_t pidx;
  uint32_t size;
  uint64_t pos;
  uint32_t crc;
  bool verify;  // first visit with check_crcs: the device verifies its CRC
  int64_t row_first, row_last;
};

// Cuts the log ranges the device must read into SpanSeg entries (<= kSpanSegMax bytes and
// <= kSpanMaxSegRows rows each, cuts never inside an element).  Returns the count.
uint32_t build_span_segments(const SpanRB* rbs, size_t n_rbs, const uint64_t* row_pos, uint64_t row_bytes,
                             uint32_t esz, SpanSeg* out, uint64_t cap) {
  uint32_t n = 0;
  for (size_t i = 0; i < n_rbs; ++i) {
    const SpanRB& rb = rbs[i];
    uint64_t lo, hi;
    if (rb.verify) {
      lo = rb.pos;  // the whole batch: its CRC covers [pos + 21, pos + size)
      hi = rb.pos + rb.size;
    } else if (rb.row_last > rb.row_first) {
      lo = row_pos[rb.row_first];  // CRC already checked: only the values taken from it
      hi = row_pos[rb.row_last - 1] + row_bytes;
    } else {
      continue;  // nothing taken and nothing to verify (skipped records only)
    }
    int64_t r = rb.row_first;  // first row that may intersect [cur, ...)
    uint64_t cur = lo;
    bool first = true;
    while (cur < hi) {
      while (r < rb.row_last && row_pos[r] + row_bytes <= cur) ++r;
      uint64_t cut = std::min<uint64_t>(cur + kSpanSegMax, hi);
      // at most kSpanMaxSegRows rows: end before the value of row r + kSpanMaxSegRows
      if (rb.row_last - r > int64_t(kSpanMaxSegRows) && row_pos[r + kSpanMaxSegRows] < cut)
        cut = std::max<uint64_t>(row_pos[r + kSpanMaxSegRows], cur + 1);
      if (cut < hi) {
        // never split an element: move the cut back to an element boundary of the row it hits
        int64_t q = r;
        while (q < rb.row_last && row_pos[q] + row_bytes <= cut) ++q;
        if (q < rb.row_last && row_pos[q] < cut) {
          const uint64_t in = (cut - row_pos[q]) / esz * esz;
          cut = row_pos[q] + in;
          if (cut <= cur) cut = row_pos[q] + esz;  // cur sits inside this element's row start
        }
      }
      int64_t re = r;
      while (re < rb.row_last && row_pos[re] < cut) ++re;
      if (n >= cap) throw std::runtime_error("ring slot too small for the batch's device-decode segments");
      SpanSeg& sg = out[n++];
      sg.log_pos = cur;
      sg.len = uint32_t(cut - cur);
      sg.pidx = rb.pidx;
      sg.flags = rb.verify ? (kSegCrc | (first ? kSegCrcFirst : 0u) | (cut == hi ? kSegCrcLast : 0u)) : 0u;
      sg.crc = rb.crc;
      sg.row_begin = uint32_t(r);
      sg.row_end = uint32_t(re);
      first = false;
      cur = cut;
    }
  }
  return n;
}

// kPackJsonSpan: the same log ranges, but cut only between row texts (a row's text lies whole in
// one segment, so one wave parses it from LDS), at most kJsonSpanMaxSegRows rows per segment;
// then kSegHostRows pseudo-segments over the rows the worker parsed itself.
uint32_t build_json_segments(const SpanRB* rbs, size_t n_rbs, const JsonSpanRow* rows, int64_t n_rows, SpanSeg* out,
                             uint64_t cap) {
  uint32_t n = 0;
  auto emit = [&](uint64_t pos, uint32_t len, uint32_t pidx, uint32_t flags, uint32_t crc, int64_t r0, int64_t r1) {
    if (n >= cap) throw std::runtime_error("ring slot too small for the batch's device-parse segments");
    SpanSeg& sg = out[n++];
    sg.log_pos = pos;
    sg.len = len;
    sg.pidx = pidx;
    sg.flags = flags;
    sg.crc = crc;
    sg.row_begin = uint32_t(r0);
    sg.row_end = uint32_t(r1);
  };
  for (size_t i = 0; i < n_rbs; ++i) {
    const SpanRB& rb = rbs[i];
    uint64_t lo = UINT64_MAX, hi = 0;
    for (int64_t r = rb.row_first; r < rb.row_last; ++r) {
      if (rows[r].tlen < 0) continue;
      lo = std::min<uint64_t>(lo, rows[r].pos);
      hi = std::max<uint64_t>(hi, rows[r].pos + uint64_t(rows[r].tlen));
    }
    if (rb.verify) {
      lo = rb.pos;  // the whole batch: its CRC covers [pos + 21, pos + size)
      hi = rb.pos + rb.size;
    } else if (lo >= hi) {
      continue;  // nothing for the device: skipped records or worker-parsed rows only
    }
    int64_t r = rb.row_first;
    uint64_t cur = lo;
    bool first = true;
    while (cur < hi) {
      while (r < rb.row_last && (rows[r].tlen < 0 || rows[r].pos < cur)) ++r;  // rows of earlier segments
      uint64_t cut = std::min<uint64_t>(cur + kSpanSegMax, hi);
      int64_t re = r;
      for (; re < rb.row_last && re - r < int64_t(kJsonSpanMaxSegRows); ++re) {
        if (rows[re].tlen < 0) continue;
        if (rows[re].pos >= cut) break;
        if (rows[re].pos + uint64_t(rows[re].tlen) > cut) {  // the text would straddle the cut: cut before it
          cut = rows[re].pos;
          break;
        }
      }
      if (re - r == int64_t(kJsonSpanMaxSegRows)) {
        // row limit: end the segment at the next device row's text
        int64_t q = re;
        while (q < rb.row_last && rows[q].tlen < 0) ++q;
        if (q < rb.row_last && rows[q].pos < cut) cut = rows[q].pos;
      }
      if (cut <= cur) throw std::logic_error("json span: empty segment");
      emit(cur, uint32_t(cut - cur), rb.pidx,
           rb.verify ? (kSegCrc | (first ? kSegCrcFirst : 0u) | (cut == hi ? kSegCrcLast : 0u)) : 0u, rb.crc, r, re);
      first = false;
      cur = cut;
    }
  }
  int64_t h0 = -1;
  for (int64_t r = 0; r <= n_rows; ++r) {
    const bool host = r < n_rows && rows[r].tlen < 0;
    if (h0 >= 0 && (!host || r - h0 == int64_t(kJsonSpanMaxSegRows))) {
      emit(0, 0, UINT32_MAX, kSegHostRows, 0, h0, r);
      h0 = -1;
    }
    if (host && h0 < 0) h0 = r;
  }
  return n;
}

}  // namespace

int64_t key_int64(const uint8_t* key, int32_t len, int enc, int64_t dflt) {
  if (!key || len < 0) return dflt;
  if (enc == kKeyAscii) {
    int32_t i = 0;
    bool neg = false;
    if (i < len && (key[i] == '-' || key[i] == '+')) neg = key[i++] == '-';
    if (i == len || len - i > 19) return dflt;
    // accumulate unsigned and bound before each step: 19 digits reach 9999999999999999999, past
    // INT64_MAX; the most a key may hold is INT64_MAX, or INT64_MAX + 1 when negative
    const uint64_t lim = neg ? uint64_t(INT64_MAX) + 1 : uint64_t(INT64_MAX);
    uint64_t v = 0;
    for (; i < len; ++i) {
      if (key[i] < '0' || key[i] > '9') return dflt;
      const uint64_t d = uint64_t(key[i] - '0');
      if (v > (lim - d) / 10) return dflt;  // v * 10 + d would exceed lim
      v = v * 10 + d;
    }
    return neg ? int64_t(0 - v) : int64_t(v);
  }
  if (len != 8) return dflt;
  uint64_t v;
  std::memcpy(&v, key, 8);
  if (enc == kKeyBigEndian) v = __builtin_bswap64(v);
  return int64_t(v);
}

// ------------------------------------------------------------ fill
FillOutcome fill_slot(Fetcher& f, Ring& ring, uint32_t g, const PackSpec& spec, int64_t B, int64_t timeout_ms,
                      size_t* rr) {
  SlotHeader* h = ring.slot(g);
  uint8_t* pay = ring.payload(g);
  const uint64_t cap = ring.payload_capacity();
  auto& parts = f.parts();
  FillOutcome out;
  const bool gather = spec.kind == kPackFixed && spec.gather;
  const bool span = spec.kind == kPackFixed && spec.span && !gather;
  const bool jspan = spec.kind == kPackJsonText && spec.span;  // JSON text parsed on the device from the logs
  // ... and counted there: the walk reads headers only (span.h kJsonCountOnDevice)
  const bool jcount = jspan && spec.span == kSpanJsonDevCount;
  if (jcount && (spec.min_len > 0 || (spec.max_len >= 0 && !spec.truncate) || spec.skip_bad))
    throw std::invalid_argument("device element counting cannot drop rows (min_len, max_len without truncate, "
                                "skip_bad): the worker must count them");
  const bool vspan = spec.kind == kPackVarlen && spec.span;    // var-len values decoded on the device from the logs
  const bool rspan = jspan || vspan;                           // rows + segments slot layout (span.h)
  h->n_rows = 0;
  h->n_parts = 0;
  h->n_segs = 0;
  h->flags = 0;
  h->kind = uint32_t(gather ? kPackGatherFixed : span ? kPackRecordSpan : jspan ? kPackJsonSpan
                    : vspan ? kPackVarSpan : spec.kind);
  h->trunc_len = -1;
  h->err_len = 0;
  h->max_row_len = 0;
  h->total_elems = 0;
  h->n_scanned = 0;
  h->src_dtype = -1;
  h->ndim = 0;
  h->extras_offset = 0;
  h->extras_n = 0;
  h->t_fill_start_ns = now_ns();
  if (B <= 0) throw std::invalid_argument("batch size must be positive");

  const bool fixed = spec.kind == kPackFixed;
  const bool json_text = spec.kind == kPackJsonText;
  f.set_sparse_touch(span && uint64_t(spec.row_elems) * uint64_t(spec.elem_size) >= (16u << 10));
  JsonRowDesc* jrows = nullptr;
  JsonSpanRow* srows = nullptr;
  const uint64_t row_bytes = fixed ? uint64_t(spec.row_elems) * uint64_t(spec.elem_size) : 0;
  uint64_t values_off = 0;
  int32_t* offs = nullptr;
  uint64_t* gat = nullptr;
  std::vector<const uint8_t*> log_of;
  std::vector<uint64_t> log_cap;
  if (gather || span) {
    // gather: one (pidx << 44 | log offset) per row; span: one log position per row (span.h)
    if (uint64_t(B) * 8 > cap) throw std::invalid_argument("ring slot too small for the batch's row table");
    gat = reinterpret_cast<uint64_t*>(pay);
    log_of.reserve(parts.size());
    for (const auto& fp : parts) log_of.push_back(f.broker().log_base(fp.pidx));
  } else if (fixed) {
    if (uint64_t(B) * row_bytes > cap) throw std::invalid_argument("ring slot too small for the batch");
  } else if (rspan) {
    for (const auto& fp : parts) {
      log_of.push_back(f.broker().log_base(fp.pidx));
      log_cap.push_back(f.broker().part(fp.pidx).log_capacity);
    }
    values_off = align_up(uint64_t(B) * sizeof(JsonSpanRow), 256);  // worker-parsed rows' f32 values follow
    if (values_off >= cap) throw std::invalid_argument("ring slot too small for the batch's row table");
    srows = reinterpret_cast<JsonSpanRow*>(pay);
  } else if (json_text) {
    for (const auto& fp : parts) {
      log_of.push_back(f.broker().log_base(fp.pidx));
      log_cap.push_back(f.broker().part(fp.pidx).log_capacity);
    }
    values_off = align_up(uint64_t(B) * sizeof(JsonRowDesc), 256);
    if (values_off >= cap) throw std::invalid_argument("ring slot too small for the batch's row table");
    jrows = reinterpret_cast<JsonRowDesc*>(pay);
  } else {
    values_off = align_up(uint64_t(B + 1) * 4, 256);
    if (values_off >= cap) throw std::invalid_argument("ring slot too small for the batch offsets");
    offs = reinterpret_cast<int32_t*>(pay);
    offs[0] = 0;
  }
  uint8_t* vals = pay + values_off;
  const uint64_t vcap = cap - values_off;
  uint64_t vused = 0;
  int64_t rows = 0, elems = 0, max_len = 0, scanned = 0;
  std::vector<int> wm_of(parts.size(), -1);
  size_t cur_part = 0;
  bool slot_full = false;

  auto touch = [&](const RecordView& r) {
    int k = wm_of[cur_part];
    if (k < 0) {
      if (h->n_parts >= uint32_t(kMaxSlotParts)) throw std::runtime_error("too many partitions in one slot");
      k = int(h->n_parts++);
      wm_of[cur_part] = k;
      h->wm[k].pidx = parts[cur_part].pidx;
      h->wm[k].count = 0;
      h->wm[k].first_offset = parts[cur_part].position;
      h->log_end[k] = 0;
    }
    h->wm[k].count++;
    h->wm[k].next_offset = r.offset + 1;
    ++scanned;
  };
  auto bad = [&](const RecordView& r, const char* why) -> int {
    if (!spec.skip_bad)
      throw CorruptRecord(std::string("record at offset ") + std::to_string(r.offset) + ": " + why);
    touch(r);
    return kTake;
  };

  // var-len device decode: the software prefetch stream ahead of the header walk
  constexpr uint64_t kWalkAhead = 2048, kWalkStreamMax = 16u << 10;
  const uint8_t* pf_frontier = nullptr;

  // span: the RecordBatches the walk entered, in slot order (segments are cut from them below)
  thread_local std::vector<SpanRB> rbs;
  rbs.clear();
  auto on_batch = [&](const IndexEntry& e, const BatchHeader& bh, bool unverified) -> bool {
    if (!span && !rspan) return true;
    const uint32_t pidx = parts[cur_part].pidx;
    if (rbs.empty() || rbs.back().pidx != pidx || rbs.back().pos != e.pos)
      rbs.push_back(SpanRB{pidx, e.size, e.pos, bh.crc, unverified, rows, rows});
    return false;  // no host CRC pass: the walk never reads the values
  };

  auto visit = [&](const RecordView& r) -> int {
    if (r.value == nullptr) { touch(r); return kTake; }  // null value == `_process` returned None
    if (fixed) {
      if (uint64_t(r.value_len) != row_bytes) return bad(r, "value size does not match the fixed-width schema");
      if (span) {
        gat[rows] = uint64_t(r.value - log_of[cur_part]);
        touch(r);
        rbs.back().row_last = ++rows;
        return rows == B ? kTakeStop : kTake;
      }
      if (gather) {
        const uint64_t off = uint64_t(r.value - log_of[cur_part]);
        gat[rows] = (uint64_t(parts[cur_part].pidx) << kGatherShift) | off;
        touch(r);
        uint64_t& e = h->log_end[wm_of[cur_part]];
        e = std::max<uint64_t>(e, off + row_bytes);
        ++rows;
        return rows == B ? kTakeStop : kTake;
      }
      copy_to_slot(vals + uint64_t(rows) * row_bytes, r.value, row_bytes);
      touch(r);
      ++rows;
      return rows == B ? kTakeStop : kTake;
    }
    int64_t len;
    uint64_t nbytes;
    if (vspan) {
      // device decode from the log: the header gave the value's length; nothing else is read.  A
      // value too long for one segment is copied into the slot here (rare).  Variable-length
      // records defeat the hardware prefetcher (the next header sits a data-dependent distance
      // ahead): a software stream kAhead bytes in front of the walk turns the chain of dependent
      // misses into sequential reads (~160 -> ~60 ns per 1 KiB record).
      if (uint64_t(r.value_len) < kWalkStreamMax) {
        const uint8_t* want = r.value + r.value_len + kWalkAhead;
        if (pf_frontier < r.value || pf_frontier > want + kWalkAhead) pf_frontier = r.value;  // a jump: restart
        for (; pf_frontier < want; pf_frontier += 64) __builtin_prefetch(pf_frontier);
      }
      if (r.value_len % spec.elem_size) return bad(r, "value size is not a multiple of the element size");
      const int64_t cnt = r.value_len / spec.elem_size;
      if (cnt < spec.min_len) { touch(r); return kTake; }
      len = cnt;
      if (spec.max_len >= 0 && len > spec.max_len) {
        if (!spec.truncate) { touch(r); return kTake; }
        len = spec.max_len;
      }
      if (cnt > INT32_MAX) throw std::runtime_error("var-len row too large for the device decode");
      JsonSpanRow d;
      d.count = int32_t(cnt);
      if (uint64_t(r.value_len) <= kVarSpanRowMax) {
        d.pos = uint64_t(r.value - log_of[cur_part]);
        d.tlen = int32_t(r.value_len);
      } else {
        nbytes = uint64_t(len) * uint64_t(spec.elem_size);
        const uint64_t at = align_up(vused, 16);
        if (at + nbytes > vcap) {
          if (rows == 0) throw std::runtime_error("a single record exceeds the ring slot capacity");
          slot_full = true;
          return kStopBefore;
        }
        copy_to_slot(vals + at, r.value, nbytes);
        d.pos = values_off + at;
        d.tlen = -1;
        vused = at + nbytes;
      }
      srows[rows] = d;
      elems += len;
      max_len = std::max(max_len, len);
      touch(r);
      rbs.back().row_last = ++rows;
      return rows == B ? kTakeStop : kTake;
    }
    if (jspan) {
      // device parse from the log: count + simple check of the text where it lies (no copy, no
      // CRC pass); rows that are not simple are parsed here, their float32 values ride in the slot
      const char* txt = reinterpret_cast<const char*>(r.value);
      const size_t tn = size_t(r.value_len);
      JsonSpanRow d;
      const uint64_t at_log = uint64_t(r.value - log_of[cur_part]);
      if (jcount && tn <= kJsonSpanRowMax) {
        // the header gave the text's place and length; the device counts its elements
        if (uint64_t(r.value_len) < kWalkStreamMax) {  // the var-len walk's software prefetch stream
          const uint8_t* want = r.value + r.value_len + kWalkAhead;
          if (pf_frontier < r.value || pf_frontier > want + kWalkAhead) pf_frontier = r.value;
          for (; pf_frontier < want; pf_frontier += 64) __builtin_prefetch(pf_frontier);
        }
        d.pos = at_log;
        d.tlen = int32_t(tn);
        d.count = kJsonCountOnDevice;
        srows[rows] = d;
        int64_t bound = json_count_bound(tn);
        if (spec.max_len >= 0 && bound > spec.max_len) bound = spec.max_len;
        elems += bound;
        max_len = std::max(max_len, bound);
        touch(r);
        rbs.back().row_last = ++rows;
        return rows == B ? kTakeStop : kTake;
      }
      int64_t cnt = tn <= kJsonSpanRowMax ? json_scan_inplace(txt, tn, size_t(log_cap[cur_part] - at_log)) : -1;
      uint64_t at = vused;
      if (cnt >= 0) {
        d.pos = at_log;
        d.tlen = int32_t(tn);
        nbytes = 0;
      } else {
        at = align_up(vused, 16);
        const int64_t room = at < vcap ? int64_t((vcap - at) / 4) : 0;
        cnt = parse_json_f32(txt, tn, reinterpret_cast<float*>(vals + at), room);
        if (cnt == -2) {
          if (rows == 0) throw std::runtime_error("a single record exceeds the ring slot capacity");
          slot_full = true;
          return kStopBefore;
        }
        if (cnt < 0) return bad(r, "value is not a flat numeric JSON array");
        d.pos = values_off + at;
        d.tlen = -1;
        nbytes = 0;
      }
      if (cnt < spec.min_len) { touch(r); return kTake; }
      len = cnt;
      if (spec.max_len >= 0 && len > spec.max_len) {
        if (!spec.truncate) { touch(r); return kTake; }
        len = spec.max_len;
      }
      if (d.tlen < 0) nbytes = uint64_t(len) * 4;
      if (cnt > INT32_MAX) throw std::runtime_error("JSON row too large for the device parser");
      d.count = int32_t(cnt);
      srows[rows] = d;
      if (d.tlen < 0) vused = at + nbytes;
      elems += len;
      max_len = std::max(max_len, len);
      touch(r);
      rbs.back().row_last = ++rows;
      return rows == B ? kTakeStop : kTake;
    }
    if (json_text) {
      // device parse: frame the row (count + simple check), copy its text; rows that are not
      // simple are parsed here and travel as float32 (JsonRowDesc::tlen == -1)
      const char* txt = reinterpret_cast<const char*>(r.value);
      const size_t tn = size_t(r.value_len);
      const uint64_t at = align_up(vused, 32);
      JsonRowDesc dsc;
      if (at + tn + 32 > vcap) {
        if (rows == 0) throw std::runtime_error("a single record exceeds the ring slot capacity");
        slot_full = true;
        return kStopBefore;
      }
      // one pass: classify + stream the text into the slot (the 32-byte read-ahead must stay
      // inside the partition log's mapping); else scan, and copy below
      const bool fused = uint64_t(r.value - log_of[cur_part]) + tn + 32 <= log_cap[cur_part];
      int64_t cnt = fused ? json_scan_copy(txt, tn, vals + at) : json_scan_simple(txt, tn);
      if (cnt >= 0) {
        dsc.tlen = int32_t(tn);
        nbytes = tn;
      } else {
        const int64_t room = at + 32 < vcap ? int64_t((vcap - at - 32) / 4) : 0;
        cnt = parse_json_f32(txt, tn, reinterpret_cast<float*>(vals + at), room);
        if (cnt == -2) {
          if (rows == 0) throw std::runtime_error("a single record exceeds the ring slot capacity");
          slot_full = true;
          return kStopBefore;
        }
        if (cnt < 0) return bad(r, "value is not a flat numeric JSON array");
        dsc.tlen = -1;
        nbytes = 0;
      }
      if (cnt < spec.min_len) { touch(r); return kTake; }
      len = cnt;
      if (spec.max_len >= 0 && len > spec.max_len) {
        if (!spec.truncate) { touch(r); return kTake; }
        len = spec.max_len;
      }
      if (dsc.tlen < 0)
        nbytes = uint64_t(len) * 4;
      else if (!fused)
        copy_to_slot(vals + at, r.value, tn);
      if (cnt > INT32_MAX || at > UINT32_MAX) throw std::runtime_error("JSON row too large for the device parser");
      dsc.off = uint32_t(at);
      dsc.count = int32_t(cnt);
      dsc.n_out = int32_t(len);
      jrows[rows] = dsc;
      vused = at + nbytes;
      elems += len;
      max_len = std::max(max_len, len);
      touch(r);
      ++rows;
      return rows == B ? kTakeStop : kTake;
    }
    if (spec.kind == kPackVarlen) {
      if (r.value_len % spec.elem_size) return bad(r, "value size is not a multiple of the element size");
      len = r.value_len / spec.elem_size;
      if (len < spec.min_len) { touch(r); return kTake; }
      if (spec.max_len >= 0 && len > spec.max_len) {
        if (!spec.truncate) { touch(r); return kTake; }
        len = spec.max_len;
      }
      nbytes = uint64_t(len) * uint64_t(spec.elem_size);
      if (vused + nbytes > vcap) {
        if (rows == 0) throw std::runtime_error("a single record exceeds the ring slot capacity");
        slot_full = true;
        return kStopBefore;
      }
      copy_to_slot(vals + vused, r.value, nbytes);
    } else {  // JSON -> f32
      float* dst = reinterpret_cast<float*>(vals + vused);
      const int64_t room = int64_t((vcap - vused) / 4);
      len = parse_json_f32(reinterpret_cast<const char*>(r.value), size_t(r.value_len), dst, room);
      if (len == -2) {
        if (rows == 0) throw std::runtime_error("a single record exceeds the ring slot capacity");
        slot_full = true;
        return kStopBefore;
      }
      if (len < 0) return bad(r, "value is not a flat numeric JSON array");
      if (len < spec.min_len) { touch(r); return kTake; }
      if (spec.max_len >= 0 && len > spec.max_len) {
        if (!spec.truncate) { touch(r); return kTake; }
        len = spec.max_len;
      }
      nbytes = uint64_t(len) * 4;
    }
    vused += nbytes;
    elems += len;
    if (elems > INT32_MAX) throw std::runtime_error("slot exceeds int32 element offsets");
    max_len = std::max(max_len, len);
    offs[rows + 1] = int32_t(elems);
    touch(r);
    ++rows;
    return rows == B ? kTakeStop : kTake;
  };

  // record fields beside the value: captured for every row the visit takes, stored after the layout
  const int n_extras = ((spec.extras & kExtraKey) ? 1 : 0) + ((spec.extras & kExtraTimestamp) ? 1 : 0);
  thread_local std::vector<int64_t> xkey, xts;
  xkey.clear();
  xts.clear();
  auto visit_x = [&](const RecordView& r) -> int {
    const int64_t before = rows;
    const int res = visit(r);
    if (rows > before) {
      if (spec.extras & kExtraKey) xkey.push_back(key_int64(r.key, r.key_len, spec.key_enc, spec.key_default));
      if (spec.extras & kExtraTimestamp) xts.push_back(r.timestamp);
    }
    return res;
  };
  auto put_extras = [&]() {
    if (!n_extras) return;
    const uint64_t off = align_up(h->payload_bytes, 256);
    const uint64_t need = uint64_t(rows) * 8u * uint64_t(n_extras);
    if (off + need > cap) throw std::invalid_argument("ring slot too small for the batch's record fields");
    int64_t* dst = reinterpret_cast<int64_t*>(pay + off);
    if (spec.extras & kExtraKey) {
      std::memcpy(dst, xkey.data(), size_t(rows) * 8);
      dst += rows;
    }
    if (spec.extras & kExtraTimestamp) std::memcpy(dst, xts.data(), size_t(rows) * 8);
    h->extras_offset = off;
    h->extras_n = uint32_t(n_extras);
    h->payload_bytes = off + need;
  };

  const int64_t idle_ns = timeout_ms < 0 ? INT64_MAX : timeout_ms * 1000000LL;
  int64_t last_progress = now_ns();
  int64_t backoff_ns = 20000;
  bool stop = false;
  while (rows < B && !stop && (!parts.empty() || f.watching())) {
    bool progress = false;
    for (size_t k = 0; k < parts.size() && rows < B; ++k) {
      cur_part = (*rr + k) % parts.size();
      FetchPart& fp = parts[cur_part];
      if (fp.paused) continue;
      size_t n;
      try {
        n = n_extras ? f.scan(fp, 1u << 20, visit_x, on_batch) : f.scan(fp, 1u << 20, visit, on_batch);
      } catch (const OffsetOutOfRange&) {
        if (rows == 0 && scanned == 0) throw;  // nothing packed yet: let the caller reset positions
        stop = true;                           // keep what is packed; the reset happens on the next fill
        break;
      }
      if (n) progress = true;
      if (slot_full) {  // the next record does not fit: close the batch early
        stop = true;
        break;
      }
    }
    *rr = (*rr + 1) % std::max<size_t>(parts.size(), 1);  // (no partitions: a group member waits for some)
    if (rows >= B || stop) break;
    if (progress) {
      last_progress = now_ns();
      backoff_ns = 20000;
      continue;
    }
    if (ring.header()->shutdown.load(std::memory_order_acquire)) { out.shutdown = true; break; }
    if (f.watching() && f.watch_changed()) { out.reassigned = true; break; }
    const int64_t now = now_ns();
    if (now - last_progress >= idle_ns) { out.timed_out = true; break; }
    const int64_t sl = std::min<int64_t>(backoff_ns, idle_ns - (now - last_progress));
    timespec ts{time_t(sl / 1000000000LL), long(sl % 1000000000LL)};
    nanosleep(&ts, nullptr);
    backoff_ns = std::min<int64_t>(backoff_ns * 2, 1000000);
  }
  h->n_rows = uint32_t(rows);
  h->row_bytes = uint32_t(row_bytes);
  if (span) {
    values_off = align_up(uint64_t(B) * 8, 256);
    const uint32_t n = build_span_segments(rbs.data(), rbs.size(), gat, row_bytes, uint32_t(spec.elem_size),
                                           reinterpret_cast<SpanSeg*>(pay + values_off),
                                           cap > values_off ? (cap - values_off) / sizeof(SpanSeg) : 0);
    h->n_segs = n;
    h->values_offset = values_off;
    h->values_bytes = uint64_t(n) * sizeof(SpanSeg);
    h->payload_bytes = values_off + h->values_bytes;
    h->max_row_len = spec.row_elems;
    h->total_elems = rows * spec.row_elems;
    h->n_scanned = scanned;
    put_extras();
    out.rows = rows;
    out.scanned = scanned;
    return out;
  }
  if (rspan) {
    const uint64_t seg_off = align_up(values_off + vused, 256);
    const uint32_t n = build_json_segments(rbs.data(), rbs.size(), srows, rows,
                                           reinterpret_cast<SpanSeg*>(pay + seg_off),
                                           cap > seg_off ? (cap - seg_off) / sizeof(SpanSeg) : 0);
    h->n_segs = n;
    h->values_offset = seg_off;
    h->values_bytes = uint64_t(n) * sizeof(SpanSeg);
    h->payload_bytes = seg_off + h->values_bytes;
    h->max_row_len = max_len;
    h->total_elems = elems;
    h->trunc_len = spec.max_len >= 0 && spec.max_len < INT32_MAX ? int32_t(spec.max_len) : -1;
    if (jcount) h->flags |= kSlotDevCount;
    h->n_scanned = scanned;
    put_extras();
    out.rows = rows;
    out.scanned = scanned;
    return out;
  }
  h->values_offset = values_off;
  h->values_bytes = gather ? uint64_t(rows) * 8 : (fixed ? uint64_t(rows) * row_bytes : vused);
  if (json_text) h->values_bytes = align_up(vused, 16);  // the kernel reads whole 16-byte chunks
  h->payload_bytes = values_off + h->values_bytes;
  h->max_row_len = fixed ? spec.row_elems : max_len;
  h->total_elems = fixed ? rows * spec.row_elems : elems;
  h->n_scanned = scanned;
  put_extras();
  out.rows = rows;
  out.scanned = scanned;
  return out;
}

}  // namespace tk
