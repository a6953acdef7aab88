// gfx950 JSON-array parse straight out of the pinned broker logs (kPackJsonSpan, csrc/core/span.h).
//
// The reference decodes each record with `json.loads(record.value)` in `_process` and stacks the
// samples (README.md:54,74; kafka_dataset.py:156-162), after kafka-python's CRC check of every
// fetched RecordBatch (check_crcs).  Here the worker only walks the record headers and pre-scans
// each text in place (element count + "simple row" check); it neither copies the text nor CRCs
// the batch.  Two kernels on one decode stream:
//   json_stage_kernel, one 256-thread workgroup per log segment (<= 128 KiB, a row's text never
//     cut): stage the segment in LDS by LDS-DMA and verify the RecordBatch CRC32C (span_device.h)
//     -- PCIe-bound, like span_decode.hip -- then copy each row's text 16-byte aligned into the
//     batch's HBM staging area (a block-wide scan of the rounded lengths places them) and write
//     its JsonRowDesc;
//   json_parse.hip's json_rows_kernel over those descriptors: a 256-thread block per row, one
//     token per thread (bit-exact with json.loads).  Parsing is ~100x the work of the copy, so it
//     gets the whole GPU (a block per row) instead of the few workgroups the segments give.
// Rows the worker parsed itself (not simple) arrive as float32 in the slot: the block of their
// kSegHostRows pseudo-segment copies them into the staging area too.
#include <hip/hip_runtime.h>

#include <stdexcept>
#include <string>

#include "dtypes.h"
#include "span_decode.h"
#include "span_device.h"

namespace tkh {

namespace {

using span::kBufBytes;
using span::kFront;
using span::kThreads;
constexpr int kWaves = kThreads / 64;
constexpr int kMaxRows = int(tk::kJsonSpanMaxSegRows);
constexpr int kRowsPerThread = kMaxRows / kThreads;

__device__ __forceinline__ uint32_t align16(uint32_t x) { return (x + 15u) & ~15u; }

__global__ __launch_bounds__(kThreads) void json_stage_kernel(JsonStageLaunch a) {
  __shared__ __attribute__((aligned(16))) uint8_t buf[kBufBytes];
  __shared__ int32_t rel[kMaxRows];
  __shared__ int32_t tln[kMaxRows];
  __shared__ int32_t cnt[kMaxRows];
  __shared__ uint32_t dst[kMaxRows];
  __shared__ __attribute__((aligned(256))) uint32_t tab[span::kNibLdsWords];
  __shared__ uint32_t wcrc[kWaves];
  __shared__ uint32_t wsum[kWaves];

  const int t = int(threadIdx.x), lane = t & 63, wv = t >> 6;
  const SpanDevSeg& sg = a.s[blockIdx.x];
  const JsonStageBatch& bo = a.b[sg.batch];
  const uint32_t row_begin = sg.row_begin;
  const uint32_t nrows = sg.row_end - row_begin;
  const uint32_t flags = sg.flags;
  const int32_t trunc = bo.trunc_len;

  if (flags & tk::kSegHostRows) {
    // rows the worker parsed (rare): one wave copies their float32 values, row after row
    if (wv != 0) return;
    uint32_t off = sg.stage_off;
    for (uint32_t rr = 0; rr < nrows; ++rr) {
      const int64_t row = int64_t(row_begin + rr);
      const tk::JsonSpanRow d = bo.rows[row];
      if (d.tlen >= 0) continue;
      const int32_t n_out = trunc >= 0 && d.count > trunc ? trunc : d.count;
      const float* __restrict__ src = reinterpret_cast<const float*>(bo.slot + d.pos);
      float* __restrict__ o = reinterpret_cast<float*>(bo.stage + off);
      for (int32_t k = lane; k < n_out; k += 64) o[k] = src[k];
      if (lane == 0) bo.desc[row] = JsonRowDesc{off, -1, d.count, n_out};
      off += align16(uint32_t(n_out) * 4u);
    }
    return;
  }

  const uint32_t len = sg.len;
  const int32_t head = int32_t(reinterpret_cast<uintptr_t>(sg.src) & 15u);
  const bool do_crc = (flags & tk::kSegCrc) != 0;

  // ---- 1. stage the segment; the row table and CRC tables load behind its first chunk
  span::stage(sg.src, len, buf, a.burst, [&] {
    const int64_t base = int64_t(sg.log_pos) - int64_t(head) - kFront;  // log position of LDS byte 0
    for (uint32_t r = uint32_t(t); r < nrows; r += kThreads) {
      const tk::JsonSpanRow d = bo.rows[row_begin + r];
      rel[r] = d.tlen >= 0 ? int32_t(int64_t(d.pos) - base) : 0;
      tln[r] = d.tlen;
      cnt[r] = d.count;
    }
    if (do_crc)
      span::load_nib_rows(tab, a.tabs);
  });
  __syncthreads();
  const uint32_t* b32 = reinterpret_cast<const uint32_t*>(buf);
  const int32_t lo_b = kFront + head, hi_b = kFront + head + int32_t(len);

  // ---- 2. CRC32C lanes (the verdict comes last)
  const uint32_t* shift_set = nullptr;
  if (do_crc) shift_set = span::crc_lanes(b32, tab, a.tabs, lo_b, hi_b, flags, wcrc);

  // ---- 3. place the rows: exclusive scan of the 16-byte-rounded text lengths (thread t holds
  // rows t * kRowsPerThread ..)
  {
    uint32_t sz[kRowsPerThread], local = 0;
#pragma unroll
    for (int i = 0; i < kRowsPerThread; ++i) {
      const uint32_t r = uint32_t(t * kRowsPerThread + i);
      sz[i] = r < nrows && tln[r] >= 0 ? align16(uint32_t(tln[r])) : 0u;
      local += sz[i];
    }
    uint32_t incl = local;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t u = __shfl_up(incl, o, 64);
      if (lane >= o) incl += u;
    }
    if (lane == 63) wsum[wv] = incl;
    __syncthreads();
    uint32_t off = sg.stage_off + incl - local;
    for (int w = 0; w < wv; ++w) off += wsum[w];
#pragma unroll
    for (int i = 0; i < kRowsPerThread; ++i) {
      const uint32_t r = uint32_t(t * kRowsPerThread + i);
      if (r < nrows) dst[r] = off;
      off += sz[i];
    }
  }
  __syncthreads();

  // ---- 4. copy: a wave per row, 16 bytes per lane (any LDS alignment: 5-dword window +
  // v_alignbyte), aligned 16-byte stores into HBM; then the row's descriptor
  bool off_seg = false;
  for (uint32_t rr = uint32_t(wv); rr < nrows; rr += kWaves) {
    const int32_t T = tln[rr];
    if (T < 0) continue;  // parsed by the worker (its kSegHostRows block writes it)
    const int32_t r0 = rel[rr];
    if (r0 < lo_b || r0 + T > hi_b) {  // the row table disagrees with the segment: read nothing
      off_seg = true;
      if (lane == 0) bo.desc[row_begin + rr] = JsonRowDesc{dst[rr], 0, 0, 0};
      continue;
    }
    uint8_t* __restrict__ o = bo.stage + dst[rr];
    for (int32_t c = 16 * lane; c < T; c += 64 * 16) {
      const int32_t b0 = r0 + c, w = b0 >> 2, sh = b0 & 3;
      const uint32_t x0 = b32[w], x1 = b32[w + 1], x2 = b32[w + 2], x3 = b32[w + 3], x4 = b32[w + 4];
      uint4 v;
      v.x = __builtin_amdgcn_alignbyte(x1, x0, sh);
      v.y = __builtin_amdgcn_alignbyte(x2, x1, sh);
      v.z = __builtin_amdgcn_alignbyte(x3, x2, sh);
      v.w = __builtin_amdgcn_alignbyte(x4, x3, sh);
      *reinterpret_cast<uint4*>(o + c) = v;
    }
    if (lane == 0) {
      const int32_t count = cnt[rr];
      bo.desc[row_begin + rr] = JsonRowDesc{dst[rr], T, count, trunc >= 0 && count > trunc ? trunc : count};
    }
  }
  if (off_seg && lane == 0) *bo.err = int32_t(sg.seg);  // never committed (reported as this segment)

  // ---- 5. CRC verdict
  if (do_crc) {
    __syncthreads();
    if (t == 0) span::crc_verdict(shift_set, wcrc, flags, sg.crc, sg.seg, bo.err, bo.partials);
  }
}

}  // namespace

void launch_json_stage(const JsonStageLaunch& a, hipStream_t stream) {
  if (a.n_seg < 0 || a.n_seg > kMaxLaunchSegs) throw std::invalid_argument("json stage: bad segment count");
  if (a.n_seg == 0) return;
  for (int i = 0; i < a.n_seg; ++i) {
    // the kernel stages a segment whole in LDS and its row table next to it
    const SpanDevSeg& s = a.s[i];
    const bool host = (s.flags & tk::kSegHostRows) != 0;
    if ((!host && (s.len == 0 || s.len > tk::kSpanSegMax || s.src == nullptr)) || s.row_end < s.row_begin ||
        s.row_end - s.row_begin > tk::kJsonSpanMaxSegRows || s.batch >= kMaxGroup || a.b[s.batch].stage == nullptr ||
        a.b[s.batch].desc == nullptr || (s.stage_off & 15u) != 0)
      throw std::invalid_argument("json stage: malformed segment");
  }
  hipLaunchKernelGGL(json_stage_kernel, dim3(unsigned(a.n_seg)), dim3(kThreads), 0, stream, a);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw std::runtime_error(std::string("json stage launch: ") + hipGetErrorString(e));
}

void prewarm_json_span_kernels() {
  hipFuncAttributes attr;
  (void)hipFuncGetAttributes(&attr, reinterpret_cast<const void*>(&json_stage_kernel));
}

}  // namespace tkh
