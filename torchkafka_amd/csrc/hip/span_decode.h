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
  uint32_t stage_off;   // kPackJsonSpan: the segment's region in its batch's HBM staging area
  uint32_t reserved;
};

struct SpanBatchOut {
  void* out;                 // [rows, row_elems] output of the batch
  const uint64_t* row_pos;   // device view of the slot's row table (log positions of the values)
  int32_t* err;              // host-mapped status word: -1 clean, else the first bad segment
  uint32_t* partials;        // host-mapped raw CRC per segment (RecordBatches spanning segments)
  // Record fields beside the values (key / timestamp, one int64 per row each): the workgroup of
  // the batch's first segment copies ext_words of them from the slot (ext_src; the driver gives
  // the payload offset in ext_off, the engine turns it into the slot's device address) to ext_out.
  int64_t* ext_out;
  const int64_t* ext_src;
  uint64_t ext_off;
  uint32_t ext_words;
  uint32_t ext_pad;
};

struct SpanLaunch {
  int n_seg;
  int vec_store;             // every batch's rows start 16-byte aligned for vector stores
  int64_t row_elems;
  const uint32_t* tabs;      // device CRC tables (tk::kSpanTabWords)
  int parts;                 // workgroups per segment (1, 2, 4, 8; span_device.h Part): grid n_seg * parts
  uint32_t* part_acc;        // parts > 1: [kMaxLaunchSegs][2] zeroed device words of this launch's stream
  SpanBatchOut b[kMaxGroup];
  SpanDevSeg s[kMaxLaunchSegs];
};

// kPackJsonSpan (json_span.hip): JSON text parsed straight from the pinned logs, in two kernels on
// one stream: json_stage_kernel (a workgroup per segment: LDS-DMA stage, RecordBatch CRC, each row's
// text copied 16-byte aligned into an HBM staging area + its JsonRowDesc) and json_parse.hip's
// json_rows_kernel over those descriptors (a 256-thread block per row: the whole GPU parses).
struct JsonStageBatch {
  const tk::JsonSpanRow* rows;  // device view of the slot's row table
  const uint8_t* slot;          // device view of the slot payload (the worker-parsed rows' float32 values)
  JsonRowDesc* desc;            // [rows] descriptors for json_rows_kernel (HBM)
  uint8_t* stage;               // the batch's staging area (HBM): texts / float32 values at desc[r].off
  int32_t* err;                 // host-mapped status word: -1 clean, else the first bad segment (CRC)
  uint32_t* partials;           // host-mapped raw CRC per segment (RecordBatches spanning segments)
  int32_t trunc_len;            // rows with more elements keep this many (-1: no limit)
  uint32_t ctr_tag;             // this launch's tag of the ctr words
  // kSlotDevCount batches: device words tagged with ctr_tag in their high 32 bits (never zeroed:
  // a launch's tag is higher than any earlier tag of the same words, BatchVerdicts::ctr_tag) --
  // [0] atomicMax of the elements kept by a row, [1] set when a row is left to the host (not
  // simple); the kernel counts rows whose JsonSpanRow::count is kJsonCountOnDevice.  nullptr:
  // every count came from the worker.
  unsigned long long* ctr;
};

struct JsonStageLaunch {
  int n_seg;
  const uint32_t* tabs;         // device CRC tables (tk::kSpanTabWords)
  int parts;                    // workgroups per segment (as SpanLaunch)
  uint32_t* part_acc;
  JsonStageBatch b[kMaxGroup];
  SpanDevSeg s[kMaxLaunchSegs];
};

void launch_json_stage(const JsonStageLaunch& a, hipStream_t stream);

// kPackVarSpan (span_decode.hip varlen_span_kernel): VarLen rows padded + cast straight from the
// logs into the batch (one kernel: stage, CRC, a wave per row).
struct VarSpanBatch {
  void* out;                    // [rows, L] padded output
  const tk::JsonSpanRow* rows;  // device view of the slot's row table
  const uint8_t* slot;          // device view of the slot payload (rows the worker copied)
  int64_t* lengths;             // [rows] elements per row (may be null)
  uint8_t* mask;                // [rows, L] (may be null)
  int32_t* err;                 // host-mapped status word (-1 clean, else the first bad segment)
  uint32_t* partials;           // host-mapped raw CRC per segment
  int64_t L;
  int32_t trunc_len;            // rows with more elements keep this many (-1: no limit)
  int32_t reserved;             // 1: every row starts 16-byte aligned (vector stores of 16 source bytes)
};

struct VarSpanLaunch {
  int n_seg;
  const uint32_t* tabs;
  int parts;                    // workgroups per segment (as SpanLaunch)
  uint32_t* part_acc;
  VarSpanBatch b[kMaxGroup];
  SpanDevSeg s[kMaxLaunchSegs];
};

void launch_var_span(const VarSpanLaunch& a, int src_dt, int dst_dt, double pad, hipStream_t stream);
void prewarm_json_span_kernels();

// Queries the attributes of the span kernel instantiations (loads their code object), so the
// first real launch does not pay for it.
void prewarm_span_kernels(int device);

void launch_span_decode(const SpanLaunch& a, int src_dt, int dst_dt, const float* shift, const float* scale,
                        hipStream_t stream);

// Validates SpanLaunch::parts (1, 2, 4, 8; accumulator words needed past 1); returns it (0 -> 1).
int check_parts(int parts, const uint32_t* acc, const char* what);

}  // namespace tkh
