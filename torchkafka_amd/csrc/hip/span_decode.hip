// gfx950 decode of Kafka RecordBatches straight out of the pinned broker logs (kPackRecordSpan,
// csrc/core/span.h) or their HBM mirror.
//
// Replaces, for schema-declared fixed-width records, the work the reference does per record on
// the CPU -- kafka-python's CRC check of every fetched batch (check_crcs) and value decode,
// then `_process` and torch.stack (kafka_dataset.py:156-162) -- and, in this
// framework's host path, the worker's CRC pass and value copy into the ring slot.
//
// One workgroup per segment -- 8 compute waves and a loader wave -- streamed through a ring of 3
// LDS windows of 10 KiB (span_device.h: the loader wave keeps 2 windows in flight while the compute
// waves check and decode one; 46 KiB of LDS).  In each window
//   values: the 16-byte groups that START in the window's bytes -- a wave per row, its lanes over
//   the row's groups (all waves on rows of > 128 groups), or (row, group) pairs strided over
//   the block for rows of < 32 groups; each group is read as two aligned 16-byte LDS reads cut to
//   the group's bytes (span::lds16_row: values sit at arbitrary byte offsets behind their varint
//   headers), converted (dtypes.h: bit-exact with Tensor.to), stored 8-16 B per lane;
//   CRC32C: every lane folds its 20-byte piece into its running state (span::crc_piece).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <stdexcept>
#include <string>

#include "convert.h"
#include "span_decode.h"
#include "span_device.h"

namespace tkh {

namespace {

using span::kBlock;
using span::kFront;
using span::kThreads;
using span::kWinBytes;
constexpr int kBufs = 3;  // LDS windows per workgroup (2 in flight)

template <typename S>
__device__ __forceinline__ S lds_elem(const uint32_t* b32, int32_t b) {
  // one element at LDS byte b (any alignment)
  const int32_t w = b >> 2, sh = b & 3;
  if constexpr (sizeof(S) <= 4) {
    const uint32_t x = __builtin_amdgcn_alignbyte(b32[w + 1], b32[w], sh);
    S v;
    __builtin_memcpy(&v, &x, sizeof(S));
    return v;
  } else {
    const uint32_t x0 = b32[w], x1 = b32[w + 1], x2 = b32[w + 2];
    const uint32_t o[2] = {__builtin_amdgcn_alignbyte(x1, x0, sh), __builtin_amdgcn_alignbyte(x2, x1, sh)};
    S v;
    __builtin_memcpy(&v, o, sizeof(S));
    return v;
  }
}

template <typename S, typename D, bool AFFINE>
__global__ __launch_bounds__(kBlock) void span_decode_kernel(SpanLaunch a, const float* __restrict__ shift,
                                                               const float* __restrict__ scale) {
  using C = Conv<S, D, IsIntDst<D>::value>;
  constexpr int kPer = 16 / int(sizeof(S));  // source elements per 16-byte group
  __shared__ __attribute__((aligned(16))) uint8_t bufs[kBufs][kWinBytes];
  __shared__ int32_t rel[tk::kSpanMaxSegRows];
  __shared__ __attribute__((aligned(256))) uint32_t tab[span::kNibLdsWords];
  __shared__ span::RowWins rw;
  __shared__ uint32_t wcrc[kThreads / 64];

  const int t = int(threadIdx.x);
  const int P = a.parts;
  const SpanDevSeg& sg = a.s[int(blockIdx.x) / P];
  const SpanBatchOut& bo = a.b[sg.batch];
  const uint32_t len = sg.len, flags = sg.flags;
  const int32_t head = int32_t(reinterpret_cast<uintptr_t>(sg.src) & 15u);
  const uint32_t row_begin = sg.row_begin;
  const int32_t nrows = int32_t(sg.row_end - row_begin);
  const bool do_crc = (flags & tk::kSegCrc) != 0;
  const int32_t lo_b = kFront + head, hi_b = lo_b + int32_t(len);  // the segment's image bytes
  const span::Windows W(lo_b, hi_b);
  const span::Part pt = span::part_of(P, W.nw);
  const int64_t RE = a.row_elems;
  const int32_t G = int32_t((RE + kPer - 1) / kPer);  // 16-byte groups per row
  const int32_t row_bytes = int32_t(RE * int64_t(sizeof(S)));
  D* __restrict__ out = static_cast<D*>(bo.out);

  // group gi of row rr, when its key (first byte in the segment) lies in [own_lo, own_hi)
  // row_wave: every lane of the wave is on row rr (lds16_row's uniform alignment)
  auto group = [&](const uint8_t* buf, int32_t off, int32_t own_lo, int32_t own_hi, int32_t rr, int32_t gi,
                   bool row_wave) {
    const uint32_t* b32 = reinterpret_cast<const uint32_t*>(buf);
    const int32_t e0 = gi * kPer;
    const int32_t b0 = rel[rr] + e0 * int32_t(sizeof(S));
    const int64_t rem = RE - e0;
    const int nel = rem < kPer ? int(rem) : kPer;
    if (b0 + nel * int32_t(sizeof(S)) <= lo_b || b0 >= hi_b) return;  // held by another segment
    const int32_t key = b0 > lo_b ? b0 : lo_b;
    if (key < own_lo || key >= own_hi) return;  // another window's
    D* __restrict__ orow = out + int64_t(row_begin + uint32_t(rr)) * RE;
    if (nel == kPer && b0 >= lo_b && b0 + 16 <= hi_b) {
      const uint4 o = row_wave ? span::lds16_row(reinterpret_cast<const uint4*>(buf), b0 + off)
                               : span::lds16(reinterpret_cast<const uint4*>(buf), b0 + off);
      S sv[kPer];
      __builtin_memcpy(sv, &o, 16);
      Vec<D, kPer> ov;
#pragma unroll
      for (int k = 0; k < kPer; ++k) {
        if constexpr (AFFINE)
          ov.v[k] = C::apply(sv[k], shift[e0 + k], scale[e0 + k], true);
        else
          ov.v[k] = C::apply(sv[k], 0.f, 1.f, false);
      }
      if (a.vec_store) {
        *reinterpret_cast<Vec<D, kPer>*>(orow + e0) = ov;
      } else {
#pragma unroll
        for (int k = 0; k < kPer; ++k) orow[e0 + k] = ov.v[k];
      }
    } else {
      // a group cut by the segment's edge (large rows) or a short row tail
      for (int k = 0; k < nel; ++k) {
        const int32_t be = b0 + k * int32_t(sizeof(S));
        if (be < lo_b || be + int32_t(sizeof(S)) > hi_b) continue;
        const S sv = lds_elem<S>(b32, be + off);
        if constexpr (AFFINE)
          orow[e0 + k] = C::apply(sv, shift[e0 + k], scale[e0 + k], true);
        else
          orow[e0 + k] = C::apply(sv, 0.f, 1.f, false);
      }
    }
  };

  const uint32_t crc = span::pipeline<kBufs>(
      sg.src, W, pt.k0, pt.k1, bufs, tab, a.tabs, lo_b + ((flags & tk::kSegCrcFirst) ? 21 : 0), do_crc,
      (flags & tk::kSegCrcFirst) != 0,
      [&] {  // setup: row positions (image bytes) and the window table, behind the first windows' loads
        const int64_t base = int64_t(sg.log_pos) - int64_t(head) - kFront;  // log position of image byte 0
        for (int32_t r = t; r < nrows; r += kThreads) rel[r] = int32_t(int64_t(bo.row_pos[row_begin + uint32_t(r)]) - base);
        span::row_wins_init(rw, W.nw);
      },
      [&] {  // prepare: the windows each row's groups start in; the record fields beside the values
        if (t >= kThreads) return;
        for (int32_t r0w = 0; r0w < nrows; r0w += kThreads) {
          const int32_t r = r0w + t;
          const int32_t r0 = r < nrows ? rel[r] : 0;
          const bool in = r < nrows && r0 + row_bytes > lo_b && r0 < hi_b;
          const int32_t kf = r0 > lo_b ? r0 : lo_b, kl = min(r0 + (G - 1) * 16, hi_b - 1);
          span::row_wins_add(rw, W.nw, r0w + (t & ~63), in, W.win_of(kf), W.win_of(kl));
        }
        if (sg.seg == 0 && pt.q == 0 && bo.ext_words)
          for (uint32_t i = uint32_t(t); i < bo.ext_words; i += kThreads) bo.ext_out[i] = bo.ext_src[i];
      },
      [&](int k, const uint8_t* buf, int32_t off) {  // body: the groups window k owns
        const int32_t ra = rw.lo[k], rb = rw.hi[k];
        if (ra >= rb) return;
        const int32_t own_lo = W.own_lo(k), own_hi = W.own_hi(k);
        if (G >= 32) {
          span::for_rows(
              ra, rb, G > 128,
              [&](int32_t rr, int32_t* ulo, int32_t* uhi) {
                const int32_t r0 = rel[rr];
                // k == 0 also owns the group cut by the segment's start (its key is lo_b)
                *ulo = k == 0 ? (r0 >= lo_b ? 0 : (lo_b - r0) >> 4) : span::unit_from(r0, own_lo);
                *uhi = min(G, span::unit_from(r0, own_hi));
              },
              [&](int32_t rr, int32_t gi) { group(buf, off, own_lo, own_hi, rr, gi, true); });
        } else {
          const int32_t total = (rb - ra) * G;
          for (int32_t p = t; p < total; p += kThreads) {
            const int32_t q = p / G;
            group(buf, off, own_lo, own_hi, ra + q, p - q * G, false);
          }
        }
      });

  // ---- verdict: merge the lanes; thread 0 compares (or leaves the partial for the driver)
  if (do_crc) {
    if (t < kThreads) span::crc_merge(crc, wcrc);
    __syncthreads();
    if (t == 0)
      span::crc_finish(wcrc, flags, sg.crc, sg.seg, bo.err, bo.partials, P, pt.q,
                       a.part_acc + 2 * pt.seg);
  }
}

// VarLen rows (kPackVarSpan): staged and checked as above; each row's elements (any byte alignment)
// converted in 16-byte units by the window its unit starts in; padding, mask and lengths written
// before the windows (they need only the row table).
template <typename S, typename D>
__global__ __launch_bounds__(kBlock) void varlen_span_kernel(VarSpanLaunch a, D pad) {
  using C = Conv<S, D, IsIntDst<D>::value>;
  constexpr int kWaves = kThreads / 64;
  constexpr int kPer = 16 / int(sizeof(S));
  __shared__ __attribute__((aligned(16))) uint8_t bufs[kBufs][kWinBytes];
  __shared__ int32_t rel[tk::kJsonSpanMaxSegRows];
  __shared__ int32_t nout[tk::kJsonSpanMaxSegRows];  // elements to convert (-1: a worker-copied row)
  __shared__ __attribute__((aligned(256))) uint32_t tab[span::kNibLdsWords];
  __shared__ span::RowWins rw;
  __shared__ uint32_t wcrc[kWaves];
  __shared__ int32_t bad;

  const int t = int(threadIdx.x), lane = t & 63, wv = t >> 6;
  const int P = a.parts;
  const SpanDevSeg& sg = a.s[int(blockIdx.x) / P];
  const VarSpanBatch& bo = a.b[sg.batch];
  const uint32_t row_begin = sg.row_begin;
  const int32_t nrows = int32_t(sg.row_end - row_begin);
  const uint32_t flags = sg.flags;
  const int64_t L = bo.L;
  const int32_t trunc = bo.trunc_len;
  D* __restrict__ out = static_cast<D*>(bo.out);
  auto finish = [&](D* orow, int64_t row, int64_t n_out) {
    for (int64_t k = n_out + lane; k < L; k += 64) orow[k] = pad;
    if (bo.mask) {
      uint8_t* mrow = bo.mask + row * L;
      for (int64_t k = lane; k < L; k += 64) mrow[k] = uint8_t(k < n_out);
    }
    if (bo.lengths && lane == 0) bo.lengths[row] = n_out;
  };

  if (flags & tk::kSegHostRows) {
    // rows the worker copied into the slot (longer than one segment): a wave per row, part 0's
    if (wv >= kWaves || int(blockIdx.x) % P != 0) return;  // the loader wave has nothing to stage here
    for (int32_t rr = wv; rr < nrows; rr += kWaves) {
      const int64_t row = int64_t(row_begin) + rr;
      const tk::JsonSpanRow d = bo.rows[row];
      if (d.tlen >= 0) continue;
      int64_t n_out = trunc >= 0 && d.count > trunc ? trunc : d.count;
      n_out = n_out < L ? n_out : L;
      const S* __restrict__ v = reinterpret_cast<const S*>(bo.slot + d.pos);
      D* orow = out + row * L;
      for (int64_t k = lane; k < n_out; k += 64) orow[k] = C::apply(v[k], 0.f, 1.f, false);
      finish(orow, row, n_out);
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
      [&] {  // setup: the row table (image bytes, elements to convert)
        const int64_t base = int64_t(sg.log_pos) - int64_t(head) - kFront;  // log position of image byte 0
        for (int32_t r = t; r < nrows; r += kThreads) {
          const tk::JsonSpanRow d = bo.rows[row_begin + uint32_t(r)];
          rel[r] = d.tlen >= 0 ? int32_t(int64_t(d.pos) - base) : 0;
          int32_t n = -1;
          if (d.tlen >= 0) {
            int64_t n_out = trunc >= 0 && d.count > trunc ? trunc : d.count;
            n_out = n_out < L ? n_out : L;
            // the row table must agree with the segment: else read nothing and never commit
            const bool ok = rel[r] >= lo_b && rel[r] + d.tlen <= hi_b && int64_t(d.count) * int64_t(sizeof(S)) == d.tlen;
            n = ok ? int32_t(n_out) : -2;
          }
          nout[r] = n;
        }
        span::row_wins_init(rw, W.nw);
        if (t == 0) bad = 0;
      },
      [&] {  // prepare: padding, mask and lengths of every row (part 0); the windows its units start in
        if (t >= kThreads) return;
        for (int32_t rr = wv; rr < nrows; rr += kWaves) {
          const int32_t n = nout[rr];
          if (n == -1) continue;  // copied by the worker (its kSegHostRows block writes it)
          if (n == -2 && lane == 0) bad = 1;
          const int64_t row = int64_t(row_begin) + rr;
          if (pt.q == 0) finish(out + row * L, row, n < 0 ? 0 : n);
        }
        for (int32_t r0w = 0; r0w < nrows; r0w += kThreads) {
          const int32_t r = r0w + t;
          const int32_t n = r < nrows ? nout[r] : 0;
          const int32_t r0 = r < nrows ? rel[r] : 0;
          const int32_t units = n > 0 ? (n + kPer - 1) / kPer : 0;
          span::row_wins_add(rw, W.nw, r0w + (t & ~63), units > 0, W.win_of(r0), W.win_of(r0 + 16 * (units - 1)));
        }
      },
      [&](int k, const uint8_t* buf, int32_t off) {  // body: the 16-byte units window k owns
        const int32_t ra = rw.lo[k], rb = rw.hi[k];
        if (ra >= rb) return;
        const int32_t own_lo = W.own_lo(k), own_hi = W.own_hi(k);
        const uint32_t* b32 = reinterpret_cast<const uint32_t*>(buf);
        span::for_rows(
            ra, rb, false,
            [&](int32_t rr, int32_t* ulo, int32_t* uhi) {
              const int32_t n = nout[rr], r0 = rel[rr];
              const int32_t units = n > 0 ? (n + kPer - 1) / kPer : 0;
              *ulo = span::unit_from(r0, own_lo);
              *uhi = min(units, span::unit_from(r0, own_hi));
            },
            [&](int32_t rr, int32_t u) {
              const int32_t n = nout[rr], r0 = rel[rr];
              D* orow = out + (int64_t(row_begin) + rr) * L;
              const int32_t e0 = u * kPer, b0 = r0 + 16 * u + off;
              if (bo.reserved && e0 + kPer <= n) {
                // 16 source bytes (span::lds16: values sit at any byte offset behind their headers),
                // a vector store (the row starts 16-byte aligned)
                const uint4 o = span::lds16_row(reinterpret_cast<const uint4*>(buf), b0);
                S sv[kPer];
                __builtin_memcpy(sv, &o, 16);
                Vec<D, kPer> ov;
#pragma unroll
                for (int q = 0; q < kPer; ++q) ov.v[q] = C::apply(sv[q], 0.f, 1.f, false);
                *reinterpret_cast<Vec<D, kPer>*>(orow + e0) = ov;
              } else {
                for (int q = 0; q < kPer && e0 + q < n; ++q)
                  orow[e0 + q] = C::apply(lds_elem<S>(b32, b0 + q * int32_t(sizeof(S))), 0.f, 1.f, false);
              }
            });
      });

  if (do_crc) {
    if (t < kThreads) span::crc_merge(crc, wcrc);
    __syncthreads();
    if (t == 0)
      span::crc_finish(wcrc, flags, sg.crc, sg.seg, bo.err, bo.partials, P, pt.q,
                       a.part_acc + 2 * pt.seg);
  }
  if (t == 0 && bad) *bo.err = int32_t(sg.seg);
}

template <typename S, typename D>
void launch_var_span_t(const VarSpanLaunch& a, double pad, hipStream_t stream) {
  D padv;
  if constexpr (IsIntDst<D>::value) padv = D(int64_t(pad)); else padv = Store<D>::cvt(float(pad));
  hipLaunchKernelGGL((varlen_span_kernel<S, D>), dim3(unsigned(a.n_seg * a.parts)), dim3(kBlock), 0, stream, a, padv);
}

template <typename S, typename D>
void launch_span_t(const SpanLaunch& a, const float* shift, const float* scale, hipStream_t stream) {
  if (a.n_seg <= 0) return;
  const dim3 grid(unsigned(a.n_seg * a.parts));
  if (shift)
    hipLaunchKernelGGL((span_decode_kernel<S, D, true>), grid, dim3(kBlock), 0, stream, a, shift, scale);
  else
    hipLaunchKernelGGL((span_decode_kernel<S, D, false>), grid, dim3(kBlock), 0, stream, a, shift, scale);
}

}  // namespace

int check_parts(int parts, const uint32_t* acc, const char* what) {
  if (parts <= 1) return 1;
  if ((parts != 2 && parts != 4 && parts != tk::kSpanMaxParts) || acc == nullptr)
    throw std::invalid_argument(std::string(what) + ": parts must be 1, 2, 4 or 8 (with accumulator words)");
  return parts;
}

void prewarm_span_kernels(int device) {
  (void)device;
  hipFuncAttributes attr;
  // the common instantiations (f32 records -> bf16 / f32 / f16 / fp8, no normalisation)
  (void)hipFuncGetAttributes(&attr, reinterpret_cast<const void*>(&span_decode_kernel<float, __bf16, false>));
  (void)hipFuncGetAttributes(&attr, reinterpret_cast<const void*>(&span_decode_kernel<float, float, false>));
  (void)hipFuncGetAttributes(&attr, reinterpret_cast<const void*>(&span_decode_kernel<float, _Float16, false>));
  (void)hipFuncGetAttributes(&attr, reinterpret_cast<const void*>(&span_decode_kernel<float, fp8e4m3, false>));
}

void launch_var_span(const VarSpanLaunch& a0, int src_dt, int dst_dt, double pad, hipStream_t stream) {
  VarSpanLaunch a = a0;
  a.parts = check_parts(a.parts, a.part_acc, "var span");
  if (a.n_seg < 0 || a.n_seg > kMaxLaunchSegs) throw std::invalid_argument("var span: bad segment count");
  if (a.n_seg == 0) return;
  if (!is_float_dt(dst_dt) && is_float_dt(src_dt))
    throw std::invalid_argument("collate: float records cannot be cast to an integer dtype");
  for (int i = 0; i < a.n_seg; ++i) {
    const SpanDevSeg& s = a.s[i];
    const bool host = (s.flags & tk::kSegHostRows) != 0;
    if ((!host && (s.len == 0 || s.len > tk::kSpanSegMax || s.src == nullptr)) || s.row_end < s.row_begin ||
        s.row_end - s.row_begin > tk::kJsonSpanMaxSegRows || s.batch >= kMaxGroup ||
        (a.b[s.batch].L > 0 && a.b[s.batch].out == nullptr))
      throw std::invalid_argument("var span: malformed segment");
  }
  TK_DISPATCH_SRC(launch_var_span_t, a, pad, stream)
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw std::runtime_error(std::string("var span launch: ") + hipGetErrorString(e));
}

void launch_span_decode(const SpanLaunch& a0, int src_dt, int dst_dt, const float* shift, const float* scale,
                        hipStream_t stream) {
  SpanLaunch a = a0;
  a.parts = check_parts(a.parts, a.part_acc, "span decode");
  if (a.n_seg < 0 || a.n_seg > kMaxLaunchSegs) throw std::invalid_argument("span decode: bad segment count");
  if (!is_float_dt(dst_dt) && is_float_dt(src_dt))
    throw std::invalid_argument("collate: float records cannot be cast to an integer dtype");
  if (shift && !is_float_dt(dst_dt)) throw std::invalid_argument("collate: normalisation needs a float dtype");
  for (int i = 0; i < a.n_seg; ++i) {
    // the kernel streams a segment of <= kSpanSegMax bytes and keeps its row positions in LDS
    if (a.s[i].len == 0 || a.s[i].len > tk::kSpanSegMax || a.s[i].row_end < a.s[i].row_begin ||
        a.s[i].row_end - a.s[i].row_begin > tk::kSpanMaxSegRows || a.s[i].batch >= kMaxGroup)
      throw std::invalid_argument("span decode: malformed segment");
  }
  TK_DISPATCH_SRC(launch_span_t, a, shift, scale, stream)
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw std::runtime_error(std::string("span decode launch: ") + hipGetErrorString(e));
}

}  // namespace tkh
