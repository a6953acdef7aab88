// Device decode of Kafka RecordBatches (kPackRecordSpan): launch interface of span_decode.hip.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "collate.h"
#include "span.h"

namespace tkh {

// Segments one launch can carry in its kernel arguments (one workgroup each).
constexpr int kMaxLaunchSegs = 48;

struct SpanDevSeg {
  const uint8_t* src;   // device address of log byte `log_pos` (pinned broker log, zero-copy)
  uint64_t log_pos;
  uint32_t len;
  uint32_t flags;       // tk::SpanSegFlags
  uint32_t crc;         // the RecordBatch's header CRC (kSegCrc)
  uint32_t row_begin;   // rows of the batch intersecting the range
  uint32_t row_end;
  uint16_t batch;       // index into SpanLaunch::b
  uint16_t seg;         // index of the segment in its slot (partials[seg], *err = seg)
};

struct SpanBatchOut {
  void* out;                 // [rows, row_elems] output of the batch
  const uint64_t* row_pos;   // device view of the slot's row table (log positions of the values)
  int32_t* err;              // host-mapped status word: -1 clean, else the first bad segment
  uint32_t* partials;        // host-mapped raw CRC per segment (RecordBatches spanning segments)
};

struct SpanLaunch {
  int n_seg;
  int vec_store;             // every batch's rows start 16-byte aligned for vector stores
  int burst;                 // > 0: each wave waits for its loads after every `burst` of them
  int64_t row_elems;
  const uint32_t* tabs;      // device CRC tables (tk::kSpanTabWords)
  SpanBatchOut b[kMaxGroup];
  SpanDevSeg s[kMaxLaunchSegs];
};

// Queries the attributes of the span kernel instantiations (loads their code object), so the
// first real launch does not pay for it.
void prewarm_span_kernels(int device);

void launch_span_decode(const SpanLaunch& a, int src_dt, int dst_dt, const float* shift, const float* scale,
                        hipStream_t stream);

}  // namespace tkh
