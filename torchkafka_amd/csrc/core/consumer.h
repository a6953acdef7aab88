// Consumer-side native core: partition fetch/decode and the batch packers.
//
// The reference's hot loop is kafka-python's per-record iterator feeding a
// Python `_process` (kafka_dataset.py:156-162), then torch.stack in the
// DataLoader.  Here the same work for schema-declared records is
// one native call per batch: walk RecordBatches straight out of the broker's
// mapped log (CRC-checked once per batch), apply the None-skip filter, and
// pack values into a pinned ring slot as either a dense [rows, D] block or a
// CSR (int32 row offsets + values) for variable-length rows.
#pragma once
#include <atomic>
#include <memory>
#include <vector>

#include "broker.h"
#include "record_batch.h"
#include "ring.h"
#include "span.h"

namespace tk {

struct FetchPart {
  uint32_t pidx;
  int64_t position;
  int64_t batch_hint = -1;
  int64_t verified_base = INT64_MIN;
  uint64_t populated_end = 0;  // log bytes [.., populated_end) already mapped into this process
  bool paused = false;
};

// What the visitor returns for each record.
enum VisitAction : int { kTake = 0, kTakeStop = 1, kStopBefore = 2 };

class Fetcher {
 public:
  Fetcher(std::shared_ptr<Broker> b, bool check_crcs) : b_(std::move(b)), check_crcs_(check_crcs) {}
  Broker& broker() { return *b_; }
  std::vector<FetchPart>& parts() { return parts_; }
  void assign(const std::vector<uint32_t>& pidxs, const std::vector<int64_t>& positions);
  size_t find(uint32_t pidx) const;  // index into parts(), or npos
  bool check_crcs() const { return check_crcs_; }

  // Visits up to `max_records` records of one partition at/after its position
  // without blocking.  Applies fetch fault injection.  Returns records taken.
  template <class F>
  size_t scan(FetchPart& fp, size_t max_records, F&& visit) {
    return scan(fp, max_records, visit, [](const IndexEntry&, const BatchHeader&, bool) { return true; });
  }
  // The same, calling on_batch(index entry, header, unverified) when the walk enters a
  // RecordBatch; `unverified`: CRC checks are on and this batch's CRC was not checked yet.
  // on_batch returns whether the host checks it now (false: the device will, kPackRecordSpan).
  template <class F, class G>
  size_t scan(FetchPart& fp, size_t max_records, F&& visit, G&& on_batch);

  // Throws OffsetOutOfRange when position is outside [log_start, hw].
  bool has_data(const FetchPart& fp);

  // Maps the log bytes ahead of `pos` into this process's page tables in one
  // madvise(MADV_POPULATE_READ) per kPrefaultBytes.  A worker maps the broker's
  // log files itself, so every first read of a page is a minor fault (the kernel
  // maps 16 pages per fault): ~6 faults per 256 KiB batch, about a quarter of a
  // worker's fill time.  One syscall per 4 MiB replaces them.  A ring log (KafkaBridge replica;
  // `ring` its bytes) is mapped whole at its first read: its writer keeps only just ahead of the
  // reader when it inflates compressed batches, so per-read prefaults shrank to a batch each and
  // the first lap's faults stayed on the workers' path (worker fill 47-50 us per batch against
  // 22 us uncompressed, profiles/r06_s28, r06_s34).
  static constexpr uint64_t kPrefaultBytes = 4u << 20;
  void prefault(FetchPart& fp, const uint8_t* log, uint64_t pos, uint64_t log_end, uint64_t ring = 0);

  // Group-managed consumers: the assignment epochs of the replicas whose group assigns this
  // fetcher's partitions (replicator.h).  While a fill waits for data it returns early
  // (FillOutcome::reassigned) once their sum leaves `base`, so the caller can take the new
  // assignment instead of waiting on partitions that moved to another member.
  void set_watch(std::vector<const std::atomic<uint64_t>*> epochs) { watch_ = std::move(epochs); }
  void set_watch_base(uint64_t base) { watch_base_ = base; }
  bool watching() const { return !watch_.empty(); }
  bool watch_changed() const {
    uint64_t sum = 0;
    for (auto* e : watch_) sum += e->load(std::memory_order_acquire);
    return sum != watch_base_;
  }

 private:
  std::shared_ptr<Broker> b_;
  bool check_crcs_;
  bool prefault_ok_ = true;
 public:
  // Device decode of large fixed-width values: the walk touches one record header per value, so
  // populating every page of the log ahead (most of them value bytes nobody on the host reads)
  // costs more than the few faults it saves (config 5: ~270 us per 8 MiB batch).
  void set_sparse_touch(bool on) { sparse_touch_ = on; }
 private:
  bool sparse_touch_ = false;
  std::vector<FetchPart> parts_;
  std::vector<const std::atomic<uint64_t>*> watch_;
  uint64_t watch_base_ = 0;
};

// ------------------------------------------------------------ packers
enum PackKind : int {
  kPackFixed = 0,
  kPackVarlen = 1,
  kPackJsonF32 = 2,
  kPackGatherFixed = 3,
  kPackJsonText = 4,
  kPackRecordSpan = 5,  // fixed-width rows decoded on the device from the pinned logs (span.h)
  kPackJsonSpan = 6,    // JsonArray rows parsed on the device straight from the pinned logs (span.h)
  kPackVarSpan = 7,     // VarLen rows padded/cast on the device straight from the pinned logs (span.h)
  kPackTree = 8,        // structured `_process` samples (tuple / list / dict of tensors): a descriptor
                        // plus one stacked region per leaf; copied to the device as one block
};

// kPackJsonText: JsonArray rows for the device parser (json_parse.hip).  The payload starts
// with one JsonRowDesc per row (common.h); the values area (at values_offset) holds each
// simple row's raw text, or the host-parsed float32 values of a row that is not simple.

// kPackGatherFixed: the slot holds no values, only one uint64 per row locating the row's value
// inside the broker log it was fetched from, (pidx << kGatherShift) | byte offset.  The main
// process pins the logs in place and the collate kernel gathers rows straight out of them
// (DeviceLoader h2d="direct"): the worker never copies the payload.
constexpr int kGatherShift = 44;
constexpr uint64_t kGatherOffsetMask = (uint64_t(1) << kGatherShift) - 1;

struct PackSpec {
  int kind = kPackFixed;
  int elem_size = 4;        // bytes per stored element (fixed/var-len); JSON emits f32
  int64_t row_elems = 0;    // fixed-width: elements per row
  int64_t min_len = 0;      // var-len/JSON: shorter rows are skipped (the reference's `_process -> None`)
  int64_t max_len = -1;     // var-len/JSON: longer rows truncated (truncate) or skipped
  int truncate = 1;
  int skip_bad = 0;         // malformed rows: 1 = skip, 0 = raise
  int gather = 0;           // fixed-width: emit log locations (kPackGatherFixed) instead of values
  int span = 0;             // fixed-width / JSON text: emit log ranges + row positions (kPackRecordSpan /
                            // kPackJsonSpan) instead of values; CRC and decode on the device;
                            // kSpanJsonDevCount: JSON elements counted on the device too (span.h)
  // Record fields delivered beside the value, one int64 per row each (SlotHeader::extras_*):
  // kExtraKey = the record key as an integer (key_enc), kExtraTimestamp = its timestamp (ms).
  int extras = 0;
  int key_enc = 0;           // kKeyBigEndian (Kafka's LongSerializer) | kKeyLittleEndian | kKeyAscii
  int64_t key_default = -1;  // a null key, or one the encoding cannot read
};

enum ExtraField : int { kExtraKey = 1, kExtraTimestamp = 2 };
enum KeyEncoding : int { kKeyBigEndian = 0, kKeyLittleEndian = 1, kKeyAscii = 2 };
// The integer of a record key (KeyEncoding); `dflt` when null or unreadable.
int64_t key_int64(const uint8_t* key, int32_t len, int enc, int64_t dflt);

struct FillOutcome {
  int64_t rows = 0;
  int64_t scanned = 0;
  bool timed_out = false;
  bool shutdown = false;
  bool reassigned = false;  // a watched group assignment changed while waiting (Fetcher::set_watch)
};

// Fills one ring slot with up to `batch_rows` rows, blocking until the batch
// is full, `timeout_ms` passes without new data (-1 = forever) or shutdown.
// Writes header fields (rows, watermarks, layout) but does not publish.
FillOutcome fill_slot(Fetcher& f, Ring& ring, uint32_t gslot, const PackSpec& spec, int64_t batch_rows,
                      int64_t timeout_ms, size_t* rr_cursor);

// Numeric JSON array -> float32 (correctly rounded as Python float()+float32 cast).
// Returns elements parsed, or -1 when the text is not a flat numeric array.
int64_t parse_json_f32(const char* s, size_t n, float* out, int64_t cap);

// Device-parse pre-scan: element count of a "simple" JSON number array (digits, '.', '-'
// only, tokens <= 16 characters), or -1 if the row must be parsed on the host.
// simd=false forces the scalar reference implementation (tests compare the two).
int64_t json_scan_simple(const char* s, size_t n, bool simd = true);
// The same verdict, scanning whole 64-byte blocks in place (`readable`: bytes readable from s).
// variant (tests/benchmarks): 0 best available, 1 AVX-512BW compares, 2 AVX2 rows, 3 scalar.
int64_t json_scan_inplace(const char* s, size_t n, size_t readable, int variant = 0);
// The same verdict, fused with a streaming copy of the text to `dst` (32-byte aligned; src
// readable and dst writable up to align_up(n, 32)).
int64_t json_scan_copy(const char* s, size_t n, uint8_t* dst);
// Element count of a flat numeric JSON array without converting (-1 if malformed).
int64_t json_array_len(const char* s, size_t n);

// ------------------------------------------------------------ template impl
template <class F, class G>
size_t Fetcher::scan(FetchPart& fp, size_t max_records, F&& visit, G&& on_batch) {
  Broker& b = *b_;
  PartitionEntry& P = b.part(fp.pidx);
  const int64_t delay = P.fetch_delay_ns.load(std::memory_order_relaxed);
  if (delay > 0) {
    timespec ts{time_t(delay / 1000000000LL), long(delay % 1000000000LL)};
    nanosleep(&ts, nullptr);
  }
  int32_t errs = P.fetch_errors.load(std::memory_order_relaxed);
  while (errs > 0) {
    if (P.fetch_errors.compare_exchange_weak(errs, errs - 1))
      throw InjectedFetchError("KafkaError: injected fetch failure on partition " + std::to_string(fp.pidx));
  }
  P.fetch_calls.fetch_add(1, std::memory_order_relaxed);
  if (!has_data(fp)) return 0;
  const int64_t hw = P.high_watermark.load(std::memory_order_acquire);
  const uint8_t* log = b.log_base(fp.pidx);
  const IndexEntry* idx = b.index_base(fp.pidx);
  size_t taken = 0;
  uint64_t bytes = 0;
  while (taken < max_records && fp.position < hw) {
    const int64_t bi = b.find_batch(fp.pidx, fp.position, fp.batch_hint);
    fp.batch_hint = bi;
    const IndexEntry e = idx[uint64_t(bi) % P.index_capacity];  // ring-indexed (replica ring logs)
    if (!sparse_touch_ && e.pos + e.size > fp.populated_end)
      prefault(fp, log, e.pos, P.log_end_pos.load(std::memory_order_acquire),
               P.ring_bytes.load(std::memory_order_relaxed));
    const uint8_t* bp = log + e.pos;
    const BatchHeader h = parse_batch_header(bp, e.size);
    if ((h.attributes >> 5) & 1) {  // control batch (a transaction marker): never delivered, as in Kafka clients
      if (fp.position < h.next_offset()) fp.position = h.next_offset();
      continue;
    }
    const bool unverified = check_crcs_ && fp.verified_base != h.base_offset;
    if (on_batch(e, h, unverified) && unverified) {
      if (!verify_batch_crc(bp, h))
        throw CorruptRecord("Record batch at offset " + std::to_string(h.base_offset) + " failed CRC check");
    }
    if (unverified) fp.verified_base = h.base_offset;  // checked here, or by the device before any commit
    bytes += e.size;
    RecordIter it(bp, h);
    RecordView r;
    while (it.next(&r)) {
      if (r.offset < fp.position) continue;
      const int act = visit(r);
      if (act == kStopBefore) {
        P.bytes_fetched.fetch_add(bytes, std::memory_order_relaxed);
        return taken;
      }
      fp.position = r.offset + 1;
      ++taken;
      if (act == kTakeStop || taken >= max_records) {
        P.bytes_fetched.fetch_add(bytes, std::memory_order_relaxed);
        return taken;
      }
    }
    if (fp.position < h.next_offset()) fp.position = h.next_offset();
  }
  P.bytes_fetched.fetch_add(bytes, std::memory_order_relaxed);
  return taken;
}

}  // namespace tk
