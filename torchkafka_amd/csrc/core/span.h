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

// Largest log range one workgroup decodes, and most rows whose values may intersect one range
// (their positions are staged in LDS).
constexpr uint32_t kSpanSegMax = 128u << 10;
constexpr uint32_t kSpanMaxSegRows = 2048;

// A segment holds a whole RecordBatch of up to 128 KiB, so producer batches of the usual sizes
// (Kafka's batch.size default is 16 KiB; config 2's 64 x 1 KiB records are 66 KB) are verified
// on the device alone; longer ones are split and their partial CRCs chained by the driver.
//
// The kernels never hold a whole segment: they stream it through a ring of 2-3 LDS windows of
// kSpanWin bytes (span_device.h) -- a loader wave keeps the next windows in flight while eight
// compute waves check and decode the current one -- so a workgroup needs 39-47 KiB of LDS.
//
// CRC32C on the device: a segment's CRC range [c0, c1) is cut into windows of kSpanWin bytes
// ENDING at c1 (the first window reaches below the segment; bytes below c0 count as zeros, which
// leave a zero CRC state unchanged).  In every window lane t folds its kSpanPiece bytes
// [w + t P, w + (t+1) P) into a running state -- one slice-by-4 step for the piece's first 4 bytes,
// then slice-by-8 steps -- and between windows the state crosses the other lanes' bytes with one
// "shift by kSpanWin - kSpanPiece zero bytes" operator (kSpanTabGap).  After the last window lane t
// holds the CRC of its bytes followed by zeros up to the end of its last piece; it is moved to the
// end of the last window (and, for a segment part, on to the segment's end) by ONE multiplication
// with a per-lane constant (kSpanTabLaneMul), and the lanes' products are xored.  kSpanPiece is
// 20 bytes (5 dwords): an odd dword count puts the 32 lanes of a ds_read_b32 group on 32 different
// LDS banks; 4 + 2 x 8 bytes per lane per window, 512 lanes (8 compute waves, two per SIMD: one
// hides the other's LDS latency).  Host mirror: crc32c_span_emulate (csrc/core/crc32c.cpp).
constexpr uint32_t kSpanPiece = 20;
constexpr uint32_t kSpanLanes = 512;
constexpr uint32_t kSpanWin = kSpanPiece * kSpanLanes;  // 10,240 bytes
constexpr uint32_t kSpanMaxWins = (kSpanSegMax + kSpanWin - 1) / kSpanWin;
static_assert(kSpanMaxWins <= 32, "window tables hold 32 entries");
// Windows of a segment of `len` bytes (>= 1).
inline constexpr uint32_t span_windows(uint32_t len) { return len == 0 ? 1u : (len + kSpanWin - 1) / kSpanWin; }

// Window geometry of one segment (span_device.h), in the kernels' image coordinates: segment byte
// i is image byte 16 + (address & 15) + i, so image byte 16 is the segment's first byte rounded
// down to 16 bytes and [lo, hi) are its bytes.  Window k owns [own_lo(k), own_hi(k)) -- a partition
// of [lo, hi): a value group, a text piece or a CRC byte belongs to the window owning its first
// byte -- and stages [stage_lo(k), stage_hi(k)), 16-byte aligned, from 16 bytes before its bytes to
// 48 after them (a 16-byte group starting in the window is whole in LDS).  Tested on the host by
// tests/native/span_window_test.cpp.
struct SpanWindows {
  int32_t lo, hi, w0;
  int32_t nw;
  constexpr SpanWindows(int32_t lo_b, int32_t hi_b)
      : lo(lo_b), hi(hi_b), w0(hi_b - int32_t(span_windows(uint32_t(hi_b - lo_b)) * kSpanWin)),
        nw(int32_t(span_windows(uint32_t(hi_b - lo_b)))) {}
  constexpr int32_t own_lo(int32_t k) const { return k == 0 ? lo : w0 + k * int32_t(kSpanWin); }
  constexpr int32_t own_hi(int32_t k) const { return k == nw - 1 ? hi : w0 + (k + 1) * int32_t(kSpanWin); }
  constexpr int32_t stage_lo(int32_t k) const {
    const int32_t a = (own_lo(k) - 16) & ~15;
    return a > 16 ? a : 16;
  }
  constexpr int32_t stage_hi(int32_t k) const {
    const int32_t e = (hi + 15) & ~15, b = (own_hi(k) + 48 + 15) & ~15;
    return e < b ? e : b;
  }
  // the window owning image byte x (clamped into the segment's windows)
  constexpr int32_t win_of(int32_t x) const {
    const int32_t k = (x - w0) / int32_t(kSpanWin);
    return k < 0 ? 0 : k >= nw ? nw - 1 : k;
  }
};
// LDS bytes of one window buffer: 16 before the staged bytes (reads start at most 10 below them),
// the loader wave's kSpanWinLoads KiB-wide LDS-DMA instructions (at most kSpanWin + 96 bytes of them
// staged; the lanes past the end repeat the last chunk into their own slot: every window costs the
// same instruction count, so the loader can wait with a counted vmcnt), 32 after (a 16-byte read
// of the slot past the last one).
constexpr int32_t kSpanWinPad = 16;
constexpr int32_t kSpanWinLoads = (int32_t(kSpanWin) + 96 + 1023) / 1024;
constexpr int32_t kSpanWinBytes = kSpanWinPad + 1024 * kSpanWinLoads + 32;

// Device table layout (uint32 words): slice-by-8 byte tables T0..T7; the nibble split of T0..T7 the kernels keep
// in LDS: row 2k + h holds T_k[n << 4h] for n < 16 (a byte table is linear over GF(2), so
// T_k[b] = row(2k)[b & 15] ^ row(2k + 1)[b >> 4]; a 16-entry row spans 16 LDS banks, so a
// ds_read_b32 of one row by any 32 lanes is conflict-free); and the window gap operator, nibble
// split too: row i holds shift-by-(kSpanWin - kSpanPiece)-bytes of (n << 4i); then the lane
// constants: entry m * kSpanLanes + t is x^(8 (kSpanPiece (kSpanLanes - 1 - t) + kSpanWin m)) mod P
// in zlib's reflected representation -- multiplying a raw CRC state by x^(8n) advances it over n zero
// bytes -- i.e. lane t's state moved past the later lanes' pieces of its last window and m whole
// windows more (the windows after a segment part's last one, SpanLaunch::parts).
constexpr uint32_t kSpanTabSlice = 0;
constexpr uint32_t kSpanTabNib = 8 * 256;
constexpr uint32_t kSpanTabNibWords = 16 * 16;
constexpr uint32_t kSpanTabGap = kSpanTabNib + kSpanTabNibWords;
constexpr uint32_t kSpanTabGapWords = 8 * 16;
constexpr uint32_t kSpanTabLaneMul = kSpanTabGap + kSpanTabGapWords;
constexpr uint32_t kSpanTabWords = kSpanTabLaneMul + 32 * kSpanLanes;
// Workgroups one segment may be split over (SpanLaunch::parts: 1, 2, 4 or 8).
constexpr int kSpanMaxParts = 8;
// Windows [k0, k1) of part q of P over a segment of nw windows.
inline constexpr int32_t span_part_k0(int32_t q, int32_t P, int32_t nw) { return q * nw / P; }

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
