// Host-side launchers of the gfx950 collate kernels (collate.hip).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "common.h"

namespace tkh {

// Dense [rows, row] -> [rows, row] cast with optional fused (x - shift) * scale.
void launch_fixed(const void* src, int src_dt, void* dst, int dst_dt, int64_t rows, int64_t row, const float* shift,
                  const float* scale, hipStream_t stream);

// CSR (int32 offsets[rows+1] in elements, values 16B-aligned) -> padded
// [rows, L] with `pad`; optional int64 lengths[rows] and uint8 mask[rows, L].
void launch_varlen(const int32_t* offs, const void* vals, int src_dt, void* out, int dst_dt, int64_t rows, int64_t L,
                   double pad, int64_t* lengths, uint8_t* mask, hipStream_t stream);

// Up to kMaxGroup dense casts (consecutive batches, same dtypes and row width) in one launch.
// 8: JSON groups of 16 were tried (config 4: 35-36.6 M rec/s against 38.6-39.1 M for 8, even with
// a 32-deep ring: the first batch of a group waits longer for its parse kernel; profiles/r04_s6).
constexpr int kMaxGroup = 8;
// host_src: the sources are pinned host memory read over PCIe (zero-copy), which sizes the grid.
void launch_fixed_group(const void* const* srcs, int src_dt, void* const* dsts, int dst_dt, const int64_t* rows, int n,
                        int64_t row, const float* shift, const float* scale, hipStream_t stream, bool host_src);

// Fixed-width rows gathered from pinned broker logs: ents[k][i] = (pidx << 44) | byte offset,
// bases[pidx] = device address of partition pidx's log.  Rows of `row_bytes` at any alignment.
void launch_gather_group(const uint64_t* const* ents, int src_dt, void* const* dsts, int dst_dt, const int64_t* rows,
                         int n, const uint64_t* bases, int64_t row_bytes, const float* shift, const float* scale,
                         hipStream_t stream);

// JSON text rows (tk::JsonRowDesc[n_rows] + values area, kPackJsonText) parsed on the
// device -> padded [n_rows, L] float dtype; a row with a grammar error stores its index
// into *err (host-mapped, may be null) and gets NaN for the bad numbers.
using tk::JsonRowDesc;
void launch_json_rows(const JsonRowDesc* rows, const void* vals, void* out, int dst_dt, int64_t n_rows, int64_t L,
                      double pad, int64_t* lengths, uint8_t* mask, int32_t* err, hipStream_t stream);

// Up to kMaxGroup JSON batches in one launch; row_base[k] = first global row of batch k,
// row_base[n] = total rows.  Entries k >= n are ignored.
struct JsonGroupArgs {
  int n;
  float pad;
  int64_t row_base[kMaxGroup + 1];
  const JsonRowDesc* rows[kMaxGroup];
  const uint8_t* vals[kMaxGroup];
  void* out[kMaxGroup];
  int64_t L[kMaxGroup];
  int64_t* lengths[kMaxGroup];
  uint8_t* mask[kMaxGroup];
  int32_t* err[kMaxGroup];
  // kPackJsonSpan: bytes of each batch's staging area (a descriptor reaching beyond it is a bad
  // row, never read), and the tag OR-ed into a parse error's row index (tk::kSpanParseErrBit); a
  // parse error then never overwrites an earlier verdict (the stage kernel's CRC failure).
  uint64_t vals_cap[kMaxGroup];
  int32_t err_tag;
  // Device-counted batches (kSlotDevCount): L[k] is only the capacity of out/mask; the width is
  // min(L[k], the stage kernel's count rounded up to `mult`) (mult 0: L[k], a fixed pad_to width),
  // and the batch's first block stores {width, rows left to the host (0/1), 1} into the
  // host-mapped info[k] (MainDriver::json_width).  ctr[k]: the tagged count words
  // (JsonStageBatch::ctr), valid where their high half equals ctr_tag[k]; nullptr: L[k].
  const unsigned long long* ctr[kMaxGroup];
  uint32_t ctr_tag[kMaxGroup];
  int32_t trunc[kMaxGroup];  // json_count_kernel: rows keep at most this many elements (-1: all)
  int32_t* info[kMaxGroup];
  int32_t mult;
  // 1 (mult 0 only): no json_count_kernel ran -- each parse block counts its own device-counted
  // row and raises info[k][1] when it leaves the row to the host; json_report_kernel, launched
  // behind the parse on the same stream, stores the width and the done flag
  int32_t fused_count;
};
void launch_json_group(JsonGroupArgs& a, int dst_dt, hipStream_t stream);
// Device counting of a staged group (json_span.hip): before launch_json_group on the same stream.
void launch_json_count(const JsonGroupArgs& a, hipStream_t stream);

std::vector<std::pair<std::string, double>> api_bench(int device, int iters);

}  // namespace tkh
