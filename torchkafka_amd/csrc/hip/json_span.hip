// gfx950 JSON-array parse straight out of the pinned broker logs (kPackJsonSpan, csrc/core/span.h).
//
// The reference decodes each record with `json.loads(record.value)` in `_process` and stacks the
// samples (README.md:54,74; kafka_dataset.py:156-162), after kafka-python's CRC check of every
// fetched RecordBatch (check_crcs).  Here the worker only walks the record headers and pre-scans
// each text in place (element count + "simple row" check); it neither copies the text nor CRCs
// the batch.  Two kernels on one decode stream:
//   json_stage_kernel, one 256-thread workgroup per log segment (<= 128 KiB, a row's text never
//     cut): a block-wide scan of the rounded text lengths places each row in the batch's HBM
//     staging area and writes its JsonRowDesc, then the segment streams through two 15 KiB LDS
//     windows (span_device.h: LDS-DMA staging of window k+1 behind the work on window k) -- each
//     window verifies its share of the RecordBatch CRC32C and copies the 16-byte text pieces that
//     start in it to their 16-byte aligned place;
//   json_count_kernel (device counting, kSlotDevCount): a wave per row scans the staged text --
//     json_scan_simple's rules -- and completes the row's descriptor and the batch's width word;
//   json_parse.hip's json_rows_kernel over those descriptors: a 256-thread block per row, one
//     token per thread (bit-exact with json.loads).  Parsing is ~100x the work of the copy, so it
//     gets the whole GPU (a block per row) instead of the few workgroups the segments give.
// Rows the worker parsed itself (not simple) arrive as float32 in the slot: the block of their
// kSegHostRows pseudo-segment copies them into the staging area too.
#include <hip/hip_runtime.h>

#include <stdexcept>
#include <string>

#include "dtypes.h"
#include "json_scan_dev.h"
#include "span_decode.h"
#include "span_device.h"

namespace tkh {

namespace {

using span::kBlock;
using span::kFront;
using span::kThreads;
using span::kWinBytes;
constexpr int kBufs = 2;  // LDS windows per workgroup (1 in flight; the row tables take the rest)
constexpr int kWaves = kThreads / 64;
constexpr int kMaxRows = int(tk::kJsonSpanMaxSegRows);
constexpr int kRowsPerThread = kMaxRows / kThreads;

__device__ __forceinline__ uint32_t align16(uint32_t x) { return (x + 15u) & ~15u; }

__global__ __launch_bounds__(kBlock) void json_stage_kernel(JsonStageLaunch a) {
  __shared__ __attribute__((aligned(16))) uint8_t bufs[kBufs][kWinBytes];
  __shared__ int32_t rel[kMaxRows];
  __shared__ int32_t tln[kMaxRows];
  __shared__ uint32_t dst[kMaxRows];
  __shared__ __attribute__((aligned(256))) uint32_t tab[span::kNibLdsWords];
  __shared__ span::RowWins rw;
  __shared__ uint32_t wcrc[kWaves];
  __shared__ uint32_t wsum[kWaves];
  __shared__ int32_t bad;

  const int t = int(threadIdx.x), lane = t & 63, wv = t >> 6;
  const int P = a.parts;
  const SpanDevSeg& sg = a.s[int(blockIdx.x) / P];
  const JsonStageBatch& bo = a.b[sg.batch];
  const uint32_t row_begin = sg.row_begin;
  const int32_t nrows = int32_t(sg.row_end - row_begin);
  const uint32_t flags = sg.flags;
  const int32_t trunc = bo.trunc_len;

  if (flags & tk::kSegHostRows) {
    // rows the worker parsed (rare): one wave of part 0 copies their float32 values, row after row
    if (wv != 0 || int(blockIdx.x) % P != 0) return;
    uint32_t off = sg.stage_off;
    for (int32_t rr = 0; rr < nrows; ++rr) {
      const int64_t row = int64_t(row_begin) + rr;
      const tk::JsonSpanRow d = bo.rows[row];
      if (d.tlen >= 0) continue;
      const int32_t n_out = trunc >= 0 && d.count > trunc ? trunc : d.count;
      const float* __restrict__ src = reinterpret_cast<const float*>(bo.slot + d.pos);
      float* __restrict__ o = reinterpret_cast<float*>(bo.stage + off);
      for (int32_t k = lane; k < n_out; k += 64) o[k] = src[k];
      if (lane == 0) {
        bo.desc[row] = JsonRowDesc{off, -1, d.count, n_out};
        if (bo.ctr) atomicMax(bo.ctr, (static_cast<unsigned long long>(bo.ctr_tag) << 32) | uint32_t(max(n_out, 0)));
      }
      off += align16(uint32_t(n_out) * 4u);
    }
    return;
  }

  const uint32_t len = sg.len;
  const int32_t head = int32_t(reinterpret_cast<uintptr_t>(sg.src) & 15u);
  const bool do_crc = (flags & tk::kSegCrc) != 0;
  const int32_t lo_b = kFront + head, hi_b = lo_b + int32_t(len);
  const span::Windows W(lo_b, hi_b);
  const span::Part pt = span::part_of(P, W.nw);

  const uint32_t crc = span::pipeline<kBufs>(
      sg.src, W, pt.k0, pt.k1, bufs, tab, a.tabs, lo_b + ((flags & tk::kSegCrcFirst) ? 21 : 0), do_crc,
      (flags & tk::kSegCrcFirst) != 0,
      [&] {  // setup: the row table (image bytes, text lengths; -2: the row disagrees with the segment)
        const int64_t base = int64_t(sg.log_pos) - int64_t(head) - kFront;  // log position of image byte 0
        for (int32_t r = t; r < nrows; r += kThreads) {
          const tk::JsonSpanRow d = bo.rows[row_begin + uint32_t(r)];
          const int32_t r0 = d.tlen >= 0 ? int32_t(int64_t(d.pos) - base) : 0;
          rel[r] = r0;
          tln[r] = d.tlen < 0 ? -1 : (r0 < lo_b || r0 + d.tlen > hi_b) ? -2 : d.tlen;
        }
        span::row_wins_init(rw, W.nw);
        if (t == 0) bad = 0;
      },
      [&] {  // prepare: place the rows (exclusive scan of the 16-byte-rounded text lengths, thread t
             // holding rows t * kRowsPerThread ..), write their descriptors, find their windows.  The
             // loader wave's threads only meet the barrier.
        const bool cw = t < kThreads;
        uint32_t sz[kRowsPerThread], local = 0;
#pragma unroll
        for (int i = 0; i < kRowsPerThread; ++i) {
          const int32_t r = t * kRowsPerThread + i;
          sz[i] = cw && r < nrows && tln[r] >= 0 ? align16(uint32_t(tln[r])) : 0u;
          local += sz[i];
        }
        uint32_t incl = local;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
          const uint32_t u = __shfl_up(incl, o, 64);
          if (lane >= o) incl += u;
        }
        if (cw && lane == 63) wsum[wv] = incl;
        __syncthreads();
        if (!cw) return;
        uint32_t off = sg.stage_off + incl - local;
        for (int w = 0; w < wv; ++w) off += wsum[w];
#pragma unroll
        for (int i = 0; i < kRowsPerThread; ++i) {
          const int32_t r = t * kRowsPerThread + i;
          if (r < nrows) {
            dst[r] = off;
            const int32_t T = tln[r];
            if (pt.q != 0) {
              // the descriptors and the verdict on the row table are part 0's
            } else if (T == -2) {  // the row table disagrees with the segment: read nothing, never commit
              bo.desc[row_begin + uint32_t(r)] = JsonRowDesc{off, 0, 0, 0};
              bad = 1;
            } else if (T >= 0) {
              // a device-counted row (count kJsonCountOnDevice) keeps that count here: json_count_kernel
              // scans its staged text and completes the descriptor before json_rows_kernel reads it
              const int32_t c = bo.rows[row_begin + uint32_t(r)].count;
              const int32_t n_out = c < 0 ? 0 : trunc >= 0 && c > trunc ? trunc : c;
              bo.desc[row_begin + uint32_t(r)] = JsonRowDesc{off, T, c, n_out};
            }
          }
          off += sz[i];
        }
        for (int32_t r0w = 0; r0w < nrows; r0w += kThreads) {
          const int32_t r = r0w + t;
          const int32_t T = r < nrows ? tln[r] : -1;
          const int32_t r0 = r < nrows ? rel[r] : 0;
          span::row_wins_add(rw, W.nw, r0w + (t & ~63), T > 0, W.win_of(r0), W.win_of(r0 + ((T - 1) & ~15)));
        }
      },
      [&](int k, const uint8_t* buf, int32_t off) {  // body: copy the 16-byte pieces window k owns
        const int32_t ra = rw.lo[k], rb = rw.hi[k];
        if (ra >= rb) return;
        const int32_t own_lo = W.own_lo(k), own_hi = W.own_hi(k);
        span::for_rows(
            ra, rb, false,
            [&](int32_t rr, int32_t* ulo, int32_t* uhi) {
              const int32_t T = tln[rr], r0 = rel[rr];
              *ulo = span::unit_from(r0, own_lo);
              *uhi = min(T > 0 ? (T + 15) >> 4 : 0, span::unit_from(r0, own_hi));
            },
            [&](int32_t rr, int32_t u) {
              *reinterpret_cast<uint4*>(bo.stage + dst[rr] + 16u * uint32_t(u)) =
                  span::lds16_row(reinterpret_cast<const uint4*>(buf), rel[rr] + 16 * u + off);
            });
      });

  if (do_crc) {
    if (t < kThreads) span::crc_merge(crc, wcrc);
    __syncthreads();
    if (t == 0)
      span::crc_finish(wcrc, flags, sg.crc, sg.seg, bo.err, bo.partials, P, pt.q,
                       a.part_acc + 2 * pt.seg);
  }
  if (t == 0 && bad) *bo.err = int32_t(sg.seg);  // never committed (reported as this segment)
}

// Device counting, between the stage and the parse: a wave per device-counted row (a block of four
// rows; blocks [row_base[k] / 4 ..) of batch k) scans the row's staged, 16-byte aligned HBM text,
// completes its descriptor and raises the batch's tagged width word.  Kept out of the stage kernel,
// whose few workgroups (one per segment) are busy with PCIe loads: here every row gets a wave.
__global__ __launch_bounds__(256) void json_count_kernel(JsonGroupArgs a) {
  const int lane = int(threadIdx.x) & 63;
  const int64_t g = int64_t(blockIdx.x) * 4 + int64_t(threadIdx.x >> 6);  // this wave's global row
  if (g >= a.row_base[a.n]) return;
  int bk = 0;
#pragma unroll
  for (int k = 1; k < kMaxGroup; ++k) bk += (k < a.n && g >= a.row_base[k]) ? 1 : 0;
  if (!a.ctr[bk]) return;
  const int64_t r = g - a.row_base[bk];
  JsonRowDesc* desc = const_cast<JsonRowDesc*>(a.rows[bk]) + r;
  const JsonRowDesc d = *desc;
  if (d.count != tk::kJsonCountOnDevice || d.tlen < 0) return;
  const int32_t T = d.tlen;
  if (uint64_t(d.off) + ((uint64_t(T) + 15u) & ~uint64_t(15)) > a.vals_cap[bk]) return;  // json_rows_kernel flags it
  const uint8_t* __restrict__ text = a.vals[bk] + d.off;
  int32_t guess = 0;
  const int32_t count = json_scan_row([&](int32_t c) { return *reinterpret_cast<const uint4*>(text + c); },
                                      [&](int32_t i) { return uint32_t(text[i]); }, T, lane, &guess);
  if (lane == 0) {
    // a row that is not simple: the host parses it when the batch is delivered (tlen
    // kJsonCountOnDevice: json_rows_kernel writes its padding, lengths and mask only)
    const bool host = count < 0;
    const int32_t c = host ? guess : count;
    const int32_t trunc = a.trunc[bk];
    const int32_t n_out = trunc >= 0 && c > trunc ? trunc : c;
    *desc = JsonRowDesc{d.off, host ? tk::kJsonCountOnDevice : T, c, n_out};
    const unsigned long long tag = static_cast<unsigned long long>(a.ctr_tag[bk]) << 32;
    atomicMax(const_cast<unsigned long long*>(a.ctr[bk]), tag | uint32_t(max(n_out, 0)));
    if (host) atomicMax(const_cast<unsigned long long*>(a.ctr[bk]) + 1, tag | 1u);
  }
}

}  // namespace

void launch_json_count(const JsonGroupArgs& a, hipStream_t stream) {
  if (a.n < 1 || a.n > kMaxGroup) throw std::invalid_argument("json count: group size out of range");
  const int64_t total = a.row_base[a.n];
  if (total <= 0) return;
  if (total > INT32_MAX) throw std::invalid_argument("json count: too many rows");
  for (int k = 0; k < a.n; ++k) {
    // the kernel reads each row's staged text as 16-byte vectors from its 16-byte aligned region
    if (a.ctr[k] && (reinterpret_cast<uintptr_t>(a.vals[k]) % 16 || reinterpret_cast<uintptr_t>(a.rows[k]) % 16 ||
                     a.row_base[k + 1] < a.row_base[k]))
      throw std::invalid_argument("json count: malformed group");
  }
  hipLaunchKernelGGL(json_count_kernel, dim3(unsigned((total + 3) / 4)), dim3(256), 0, stream, a);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw std::runtime_error(std::string("json count launch: ") + hipGetErrorString(e));
}

void launch_json_stage(const JsonStageLaunch& a0, hipStream_t stream) {
  JsonStageLaunch a = a0;
  a.parts = check_parts(a.parts, a.part_acc, "json stage");
  if (a.n_seg < 0 || a.n_seg > kMaxLaunchSegs) throw std::invalid_argument("json stage: bad segment count");
  if (a.n_seg == 0) return;
  for (int i = 0; i < a.n_seg; ++i) {
    // the kernel streams a segment of <= kSpanSegMax bytes and keeps its row table in LDS
    const SpanDevSeg& s = a.s[i];
    const bool host = (s.flags & tk::kSegHostRows) != 0;
    if ((!host && (s.len == 0 || s.len > tk::kSpanSegMax || s.src == nullptr)) || s.row_end < s.row_begin ||
        s.row_end - s.row_begin > tk::kJsonSpanMaxSegRows || s.batch >= kMaxGroup || a.b[s.batch].stage == nullptr ||
        a.b[s.batch].desc == nullptr || (s.stage_off & 15u) != 0)
      throw std::invalid_argument("json stage: malformed segment");
  }
  hipLaunchKernelGGL(json_stage_kernel, dim3(unsigned(a.n_seg * a.parts)), dim3(kBlock), 0, stream, a);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw std::runtime_error(std::string("json stage launch: ") + hipGetErrorString(e));
}

void prewarm_json_span_kernels() {
  hipFuncAttributes attr;
  (void)hipFuncGetAttributes(&attr, reinterpret_cast<const void*>(&json_stage_kernel));
  (void)hipFuncGetAttributes(&attr, reinterpret_cast<const void*>(&json_count_kernel));
}

}  // namespace tkh
