// Device-decode slots (kPackRecordSpan): what a worker hands the GPU instead of packed values.
//
// The reference's hot loop is kafka-python's per-record iterator: CRC-check every fetched
// RecordBatch (check_crcs), decode each record, call `_process` (kafka_dataset.py:156-162).
// On the device path of this framework the worker only WALKS the record headers of the
// batches it consumes (a chain of small reads, one or two cache lines per record: it never
// touches the values) to fix the exact batch boundary -- which records are taken, which are
// skipped (null values, the schema's `_process -> None`) -- and writes:
//   * SpanSeg[n_segs] at payload offset 0: byte ranges of the partition logs to read.  A
//     RecordBatch the worker has not seen before is covered whole, so the GPU can verify its
//     CRC32C; one it already had verified (a batch boundary falls inside it) only over the
//     values taken from it.  Ranges longer than kSpanSegMax are split at element boundaries.
//   * uint64 row_pos[n_rows] at values_offset: log byte position of every taken value.
// The gfx950 kernel (csrc/hip/span_decode.hip) then reads the ranges straight out of the
// pinned broker logs (zero-copy over PCIe, one workgroup per segment staged in LDS),
// verifies the CRC32C of every whole RecordBatch, extracts + casts the values into the
// batch tensor and reports a bad CRC through an error word that blocks the batch's commit.
// Host DRAM sees each payload byte once (the GPU's read) instead of three times (worker
// read, worker slot write, GPU read).
#pragma once
#include <cstdint>

namespace tk {

// Largest log range one workgroup stages in LDS (plus 32 bytes of 16-byte alignment slack),
// and most rows whose values may intersect one range (their positions are staged in LDS too).
constexpr uint32_t kSpanSegMax = 128u << 10;
constexpr uint32_t kSpanMaxSegRows = 2048;

// A segment holds a whole RecordBatch of up to 128 KiB, so producer batches of the usual sizes
// (Kafka's batch.size default is 16 KiB; config 2's 64 x 1 KiB records are 66 KB) are verified
// on the device alone; longer ones are split and their partial CRCs chained by the driver.
//
// CRC32C on the device: a segment's CRC range [c0, c1) is cut into kSpanLanes chunks of L bytes
// ENDING at c1 (the first chunk is front-padded with zeros, which leave a zero-initialised CRC
// unchanged).  Each lane folds its chunk -- one slice-by-4 step for its first 4 bytes, then
// slice-by-8 steps -- and a log2(kSpanLanes)-level tree merges neighbours with "shift by 2^j
// chunks" operators.  L is 260 bytes (65 dwords) for ranges up to 66,560 bytes, so a config-2
// RecordBatch (64 x 1 KiB records, 66 KB) keeps all 256 lanes busy, else 516 (129 dwords): an
// odd dword count puts the 32 lanes of a ds_read_b32 group on 32 different LDS banks.
constexpr uint32_t kSpanLaneSmall = 260;
constexpr uint32_t kSpanLaneLarge = 516;
constexpr uint32_t kSpanLanes = 256;
constexpr uint32_t kSpanLevels = 8;
static_assert(kSpanLaneLarge * kSpanLanes >= kSpanSegMax, "lanes must cover a whole segment");
inline constexpr uint32_t span_lane_bytes(uint32_t crc_len) {
  return crc_len <= kSpanLaneSmall * kSpanLanes ? kSpanLaneSmall : kSpanLaneLarge;
}

// A segment decoded by `parts` workgroups (span_decode.hip step 0; parts = 1, 2 or 4).  Part j runs
// CRC lanes [j n, (j+1) n) (n = kSpanLanes / parts) of the whole segment's lane layout, owns the
// bytes those lanes cover (the first part also the bytes before the CRC range, the last part up to
// the end) -- a value's 16-byte group belongs to the part owning its first byte in the segment --
// and stages its bytes with 16 before and 32 after (a group starting at the end of its range, and
// the lanes' dword reads).  Offsets from the segment's first byte, `len` its length, `crc_first`:
// the segment holds its RecordBatch's start (CRC from byte 21).  Tested by
// tests/native/span_split_test.cpp.
struct SpanPart {
  int32_t own_lo, own_hi;      // the bytes this part checks and decodes
  int32_t stage_lo, stage_hi;  // the bytes it stages
};
inline constexpr int32_t span_part_cut(uint32_t len, bool crc_first, int parts, int q) {
  const int32_t n = int32_t(len), c0 = crc_first ? 21 : 0;
  const int32_t L = int32_t(span_lane_bytes(uint32_t(n - c0)));
  const int32_t x = n - (int32_t(kSpanLanes) - q * (int32_t(kSpanLanes) / parts)) * L;
  return x < 0 ? 0 : x;
}
inline constexpr SpanPart span_part(uint32_t len, bool crc_first, int parts, int part) {
  const int32_t n = int32_t(len);
  if (parts <= 1) return SpanPart{0, n, 0, n};
  const int32_t lo = part > 0 ? span_part_cut(len, crc_first, parts, part) : 0;
  const int32_t hi = part < parts - 1 ? span_part_cut(len, crc_first, parts, part + 1) : n;
  return SpanPart{lo, hi, lo - 16 > 0 ? lo - 16 : 0, hi + 32 < n ? hi + 32 : n};
}
// Device table layout (uint32 words): slice-by-8 byte tables T0..T7, then for each lane size
// (small, large), level j and byte k of the value: shift-by-(L << j)-bytes of (b << 8k), then the
// nibble split of T0..T7 the kernels keep in LDS: row 2k + h holds T_k[n << 4h] for n < 16.  A
// byte table is linear over GF(2), so T_k[b] = row(2k)[b & 15] ^ row(2k + 1)[b >> 4]; a 16-entry
// row spans 16 LDS banks, so a ds_read_b32 of one row by any 32 lanes is conflict-free (distinct
// nibbles hit distinct banks, equal ones broadcast), where a data-dependent 256-entry lookup put
// ~3 lanes on a bank.
constexpr uint32_t kSpanTabSlice = 0;
constexpr uint32_t kSpanTabShift = 8 * 256;
constexpr uint32_t kSpanTabShiftSet = kSpanLevels * 4 * 256;
constexpr uint32_t kSpanTabNib = kSpanTabShift + 2 * kSpanTabShiftSet;
constexpr uint32_t kSpanTabNibWords = 16 * 16;
constexpr uint32_t kSpanTabWords = kSpanTabNib + kSpanTabNibWords;

enum SpanSegFlags : uint32_t {
  kSegCrcFirst = 1,   // the segment holds the first CRC'd byte of its RecordBatch (offset 21)
  kSegCrcLast = 2,    // ... and/or the last byte of its RecordBatch
  kSegCrc = 4,        // the segment is part of a RecordBatch whose CRC is verified
  kSegHostRows = 8,   // kPackJsonSpan: no log bytes; rows [row_begin, row_end) parsed by the worker
};

// ---- kPackJsonSpan: JsonArray rows parsed on the device from the pinned logs.
// The reference decodes each record with json.loads in `_process` (README.md:54,74).  Here the
// worker walks the record headers and pre-scans each value's text once (element count and the
// "simple row" check of json_scan_simple, no copy, no CRC); the slot then holds
//   * JsonSpanRow[n_rows] at payload offset 0;
//   * the float32 values of the rare rows that are not simple (exponents, NaN, long tokens),
//     parsed by the worker, right after the row table;
//   * SpanSeg[n_segs] at values_offset: log ranges as for kPackRecordSpan, cut only between row
//     texts (a row's text always lies whole in one segment), plus kSegHostRows pseudo-segments
//     for the worker-parsed rows.
// The gfx950 kernel (csrc/hip/json_span.hip) stages each segment in LDS, verifies the
// RecordBatch CRC32C like span_decode.hip, and parses every row with one wave.
struct JsonSpanRow {
  uint64_t pos;    // tlen >= 0: log byte position of the row's text; tlen < 0: payload offset of its f32 values
  int32_t tlen;    // bytes of text (parsed on the device), or -1 (parsed by the worker)
  int32_t count;   // elements of the row (the device checks its own token count against it)
};
static_assert(sizeof(JsonSpanRow) == 16, "JsonSpanRow layout");
// Rows whose values one JSON segment may hold (their tables are staged in LDS next to the text),
// and the longest text parsed on the device (a longer row is parsed by the worker).
constexpr uint32_t kJsonSpanMaxSegRows = 1024;
constexpr uint32_t kJsonSpanRowMax = 64u << 10;
// Device counting (PackSpec::span == kSpanJsonDevCount, the slot flagged kSlotDevCount): the worker
// reads only the record headers -- no byte of text -- and leaves JsonSpanRow::count at
// kJsonCountOnDevice.  json_span.hip then runs json_scan_simple's rules on the staged text (trim,
// '[' ... ']' framing, interior alphabet, token runs <= 16, element count), the batch's padded width
// comes from a device max over its rows (json_parse.hip), and a row that is not simple is parsed on
// the host when its batch is delivered (MainDriver::json_host_rows).  Until then the slot's
// max_row_len is only a bound: json_count_bound(text bytes) elements per row.
constexpr int32_t kJsonCountOnDevice = -2;
constexpr int kSpanJsonDevCount = 2;
inline constexpr int64_t json_count_bound(uint64_t text_bytes) { return int64_t(text_bytes / 2); }

// ---- kPackVarSpan: VarLen rows (raw little-endian elements, e.g. int32 token ids) decoded on the
// device from the logs.  The same slot layout as kPackJsonSpan, with JsonSpanRow::tlen the value's
// bytes and ::count its elements (no scan: the worker reads only the record headers); a value of
// more than kVarSpanRowMax bytes is copied into the slot by the worker (tlen = -1).  The kernel
// (span_decode.hip varlen_span_kernel) pads, casts, and writes lengths/mask straight into the batch.
constexpr uint32_t kVarSpanRowMax = kSpanSegMax - 1024;

struct SpanSeg {
  uint64_t log_pos;    // byte position of the range in partition `pidx`'s log
  uint32_t len;        // bytes (<= kSpanSegMax)
  uint32_t pidx;
  uint32_t flags;      // SpanSegFlags
  uint32_t crc;        // kSegCrc: the header CRC of the RecordBatch (every piece of it carries it)
  uint32_t row_begin;  // rows of the slot whose values intersect this range: [row_begin, row_end)
  uint32_t row_end;
};
static_assert(sizeof(SpanSeg) == 32, "SpanSeg layout");

// Parse-error words of the device JSON parse carry this bit over the slot row index (a CRC
// failure stores the segment index, below it).
constexpr int32_t kSpanParseErrBit = 1 << 30;

}  // namespace tk
