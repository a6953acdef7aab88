// gfx950 decode of Kafka RecordBatches straight out of the pinned broker logs
// (kPackRecordSpan, csrc/core/span.h).
//
// Replaces, for schema-declared fixed-width records, the work the reference does per record on
// the CPU -- kafka-python's CRC check of every fetched batch (check_crcs) and value decode,
// then `_process` and torch.stack (kafka_dataset.py:156-162) -- and, in this
// framework's host path, the worker's CRC pass and value copy into the ring slot.
//
// One 256-thread workgroup per segment (or `split` of them, each with a share of its CRC lanes and
// bytes -- opt-in, slower over PCIe: profiles/r04_s21_window): stage it in LDS and verify its
// RecordBatch CRC32C (span_device.h), then
//   values: a wave per row for rows of >= 32 16-byte groups (lanes over the row's groups
//   held by this segment), else (row, group) pairs strided over the block; each group is
//   read as two aligned 16-byte LDS reads cut to the group's bytes (span::lds16: values sit
//   at arbitrary byte offsets behind their varint headers), converted (dtypes.h: bit-exact
//   with Tensor.to), stored 8-16 B per lane.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <stdexcept>
#include <string>

#include "convert.h"
#include "span_decode.h"
#include "span_device.h"

namespace tkh {

namespace {

using span::kBufBytes;
using span::kFront;
using span::kThreads;

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
__global__ __launch_bounds__(kThreads) void span_decode_kernel(SpanLaunch a, const float* __restrict__ shift,
                                                               const float* __restrict__ scale) {
  using C = Conv<S, D, IsIntDst<D>::value>;
  constexpr int kPer = 16 / int(sizeof(S));  // source elements per 16-byte group
  __shared__ __attribute__((aligned(16))) uint8_t buf[kBufBytes];
  __shared__ int32_t rel[tk::kSpanMaxSegRows];
  __shared__ __attribute__((aligned(256))) uint32_t tab[span::kNibLdsWords];
  __shared__ uint32_t wcrc[kThreads / 64];

  const int t = int(threadIdx.x);
  const int P = a.split, part = int(blockIdx.x) % P;
  const int nl = int(tk::kSpanLanes) / P;  // CRC lanes of the whole segment's layout per part
  const SpanDevSeg& sg = a.s[blockIdx.x / P];
  const SpanBatchOut& bo = a.b[sg.batch];
  const uint32_t len = sg.len, flags = sg.flags;
  const int32_t head = int32_t(reinterpret_cast<uintptr_t>(sg.src) & 15u);
  const uint32_t row_begin = sg.row_begin;
  const uint32_t nrows = sg.row_end - row_begin;
  const bool do_crc = (flags & tk::kSegCrc) != 0;

  // ---- 0. split: P workgroups share the segment.  Part j runs CRC lanes [j nl, (j+1) nl) of the
  // whole segment's layout (chunks of L bytes ending at its last byte), owns the values whose
  // 16-byte group starts in those lanes' bytes, and stages them with a margin.  Coordinates below
  // are LDS bytes of this part's image: the whole-segment image's shifted down by `sh` (a multiple
  // of 16, so 16-byte slots stay aligned).
  const int32_t w_lo = kFront + head, w_hi = w_lo + int32_t(len);  // the segment, whole image
  int32_t o_lo = w_lo, o_hi = w_hi, sh = 0;
  const uint8_t* src = sg.src;
  uint32_t slen = len;
  if (P > 1) {
    const tk::SpanPart pr = tk::span_part(len, (flags & tk::kSegCrcFirst) != 0, P, part);  // span.h
    o_lo = w_lo + pr.own_lo;
    o_hi = w_lo + pr.own_hi;
    src = sg.src + pr.stage_lo;
    slen = uint32_t(pr.stage_hi - pr.stage_lo);
    sh = head + pr.stage_lo - int32_t(reinterpret_cast<uintptr_t>(src) & 15u);
  }
  const int32_t lo_b = w_lo - sh, hi_b = w_hi - sh;  // the segment's bytes (valid where staged)
  const int32_t own_lo = o_lo - sh, own_hi = o_hi - sh;

  // ---- 1. stage the segment (span_device.h); the row positions and CRC tables load behind it
  span::stage(src, slen, buf, a.burst, [&] {
    const int64_t base = int64_t(sg.log_pos) - int64_t(head) - kFront + sh;  // log position of LDS byte 0
    for (uint32_t r = uint32_t(t); r < nrows; r += kThreads)
      rel[r] = int32_t(int64_t(bo.row_pos[row_begin + r]) - base);
    if (do_crc)
      span::load_nib_rows(tab, a.tabs);
  });
  __syncthreads();
  const uint32_t* b32 = reinterpret_cast<const uint32_t*>(buf);
  const uint4* b128 = reinterpret_cast<const uint4*>(buf);  // 16-byte slots (span::lds16)

  // ---- 2. CRC32C lanes (a part: its lanes on its first nl threads, whole waves)
  const uint32_t* shift_set = nullptr;
  if (do_crc && t < nl) shift_set = span::crc_lanes(b32, tab, a.tabs, lo_b, hi_b, flags, wcrc, part * nl);

  // ---- 3. values -> out[row, :]
  {
    const int64_t RE = a.row_elems;
    const uint32_t G = uint32_t((RE + kPer - 1) / kPer);  // 16-byte groups per row
    D* __restrict__ out = static_cast<D*>(bo.out);
    auto group = [&](uint32_t rr, uint32_t gi) {
      const int32_t e0 = int32_t(gi) * kPer;
      const int32_t b0 = rel[rr] + e0 * int32_t(sizeof(S));
      const int64_t rem = RE - e0;
      const int nel = rem < kPer ? int(rem) : kPer;
      if (b0 + nel * int32_t(sizeof(S)) <= lo_b || b0 >= hi_b) return;  // group held by another segment
      const int32_t key = b0 > lo_b ? b0 : lo_b;
      if (key < own_lo || key >= own_hi) return;  // held by another part of this segment
      D* __restrict__ orow = out + int64_t(row_begin + rr) * RE;
      if (nel == kPer && b0 >= lo_b && b0 + 16 <= hi_b) {
        const uint4 o = span::lds16(b128, b0);
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
          const S sv = lds_elem<S>(b32, be);
          if constexpr (AFFINE)
            orow[e0 + k] = C::apply(sv, shift[e0 + k], scale[e0 + k], true);
          else
            orow[e0 + k] = C::apply(sv, 0.f, 1.f, false);
        }
      }
    };
    if (G >= 32) {
      // wide rows: a wave per row, its lanes over the groups of the row held by this segment
      const int lane = t & 63;
      for (uint32_t rr = uint32_t(t >> 6); rr < nrows; rr += kThreads / 64) {
        const int32_t r0 = rel[rr];
        const int32_t glo = r0 >= lo_b ? 0 : (lo_b - r0) / 16;
        const int64_t ghi64 = (int64_t(hi_b) - r0 + 15) / 16;
        const uint32_t ghi = uint32_t(ghi64 < 0 ? 0 : ghi64 < int64_t(G) ? ghi64 : int64_t(G));
        for (uint32_t gi = uint32_t(glo) + uint32_t(lane); gi < ghi; gi += 64) group(rr, gi);
      }
    } else {
      const uint32_t total = nrows * G;
      for (uint32_t p = uint32_t(t); p < total; p += kThreads) {
        const uint32_t rr = p / G;
        group(rr, p - rr * G);
      }
    }
  }

  // ---- 4. record fields beside the values (key / timestamp): the batch's first segment copies them
  if (sg.seg == 0 && part == 0 && bo.ext_words)
    for (uint32_t i = uint32_t(t); i < bo.ext_words; i += kThreads) bo.ext_out[i] = bo.ext_src[i];

  // ---- 5. verdict; split: each part leaves its wave CRCs in part_crc and the last to arrive
  // (agent-scope acq_rel count) combines all four, then zeroes the count for the stream's next launch
  if (do_crc) {
    __syncthreads();
    if (t == 0) {
      if (P == 1) {
        span::crc_verdict(shift_set, wcrc, flags, sg.crc, sg.seg, bo.err, bo.partials);
      } else {
        uint32_t* pc = a.part_crc + (blockIdx.x / P) * kPartCrcWords;
        const int nw = nl / 64;
        for (int w = part * nw; w < (part + 1) * nw; ++w)
          __hip_atomic_store(pc + w, wcrc[w], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint32_t prev = __hip_atomic_fetch_add(pc + 4, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
        if (prev == uint32_t(P - 1)) {
          uint32_t all[4];
          for (int w = 0; w < 4; ++w) all[w] = __hip_atomic_load(pc + w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(pc + 4, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          span::crc_verdict(shift_set, all, flags, sg.crc, sg.seg, bo.err, bo.partials);
        }
      }
    }
  }
}

// VarLen rows (kPackVarSpan): stage + CRC as above, then a wave per row converts its elements
// (any byte alignment: two dwords + v_alignbyte per element) and pads the row to L.
template <typename S, typename D>
__global__ __launch_bounds__(kThreads) void varlen_span_kernel(VarSpanLaunch a, D pad) {
  using C = Conv<S, D, IsIntDst<D>::value>;
  constexpr int kWaves = kThreads / 64;
  __shared__ __attribute__((aligned(16))) uint8_t buf[kBufBytes];
  __shared__ int32_t rel[tk::kJsonSpanMaxSegRows];
  __shared__ int32_t tln[tk::kJsonSpanMaxSegRows];
  __shared__ int32_t cnt[tk::kJsonSpanMaxSegRows];
  __shared__ __attribute__((aligned(256))) uint32_t tab[span::kNibLdsWords];
  __shared__ uint32_t wcrc[kWaves];

  const int t = int(threadIdx.x), lane = t & 63, wv = t >> 6;
  const SpanDevSeg& sg = a.s[blockIdx.x];
  const VarSpanBatch& bo = a.b[sg.batch];
  const uint32_t row_begin = sg.row_begin;
  const uint32_t nrows = sg.row_end - row_begin;
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
    // rows the worker copied into the slot (longer than one segment): a wave per row
    for (uint32_t rr = uint32_t(wv); rr < nrows; rr += kWaves) {
      const int64_t row = int64_t(row_begin + rr);
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
  const uint4* b128 = reinterpret_cast<const uint4*>(buf);  // 16-byte slots (span::lds16)
  const int32_t lo_b = kFront + head, hi_b = kFront + head + int32_t(len);
  const uint32_t* shift_set = nullptr;
  if (do_crc) shift_set = span::crc_lanes(b32, tab, a.tabs, lo_b, hi_b, flags, wcrc);

  bool off_seg = false;
  for (uint32_t rr = uint32_t(wv); rr < nrows; rr += kWaves) {
    const int32_t T = tln[rr];
    if (T < 0) continue;  // copied by the worker (its kSegHostRows block writes it)
    const int32_t r0 = rel[rr];
    const int64_t row = int64_t(row_begin + rr);
    D* orow = out + row * L;
    const int32_t count = cnt[rr];
    int64_t n_out = trunc >= 0 && count > trunc ? trunc : count;
    n_out = n_out < L ? n_out : L;
    if (r0 < lo_b || r0 + T > hi_b || int64_t(count) * int64_t(sizeof(S)) != T) {
      off_seg = true;  // the row table disagrees with the segment: read nothing, never commit
      n_out = 0;
    }
    // 16 source bytes per lane per step (span::lds16: values sit at any byte offset behind their
    // headers), vector stores when the row is aligned; then the tail
    constexpr int kPer = 16 / int(sizeof(S));
    const int64_t full = bo.reserved ? n_out / kPer * kPer : 0;
    for (int64_t e0 = int64_t(lane) * kPer; e0 < full; e0 += 64 * kPer) {
      const uint4 o = span::lds16(b128, r0 + int32_t(e0) * int32_t(sizeof(S)));
      S sv[kPer];
      __builtin_memcpy(sv, &o, 16);
      Vec<D, kPer> ov;
#pragma unroll
      for (int k = 0; k < kPer; ++k) ov.v[k] = C::apply(sv[k], 0.f, 1.f, false);
      *reinterpret_cast<Vec<D, kPer>*>(orow + e0) = ov;
    }
    for (int64_t k = full + lane; k < n_out; k += 64)
      orow[k] = C::apply(lds_elem<S>(b32, r0 + int32_t(k) * int32_t(sizeof(S))), 0.f, 1.f, false);
    finish(orow, row, n_out);
  }
  if (off_seg && lane == 0) *bo.err = int32_t(sg.seg);

  if (do_crc) {
    __syncthreads();
    if (t == 0) span::crc_verdict(shift_set, wcrc, flags, sg.crc, sg.seg, bo.err, bo.partials);
  }
}

template <typename S, typename D>
void launch_var_span_t(const VarSpanLaunch& a, double pad, hipStream_t stream) {
  D padv;
  if constexpr (IsIntDst<D>::value) padv = D(int64_t(pad)); else padv = Store<D>::cvt(float(pad));
  hipLaunchKernelGGL((varlen_span_kernel<S, D>), dim3(unsigned(a.n_seg)), dim3(kThreads), 0, stream, a, padv);
}

template <typename S, typename D>
void launch_span_t(const SpanLaunch& a, const float* shift, const float* scale, hipStream_t stream) {
  if (a.n_seg <= 0) return;
  const dim3 grid(unsigned(a.n_seg * a.split));
  if (shift)
    hipLaunchKernelGGL((span_decode_kernel<S, D, true>), grid, dim3(kThreads), 0, stream, a, shift, scale);
  else
    hipLaunchKernelGGL((span_decode_kernel<S, D, false>), grid, dim3(kThreads), 0, stream, a, shift, scale);
}

}  // namespace

void prewarm_span_kernels(int device) {
  (void)device;
  hipFuncAttributes attr;
  // the common instantiations (f32 records -> bf16 / f32 / f16 / fp8, no normalisation)
  (void)hipFuncGetAttributes(&attr, reinterpret_cast<const void*>(&span_decode_kernel<float, __bf16, false>));
  (void)hipFuncGetAttributes(&attr, reinterpret_cast<const void*>(&span_decode_kernel<float, float, false>));
  (void)hipFuncGetAttributes(&attr, reinterpret_cast<const void*>(&span_decode_kernel<float, _Float16, false>));
  (void)hipFuncGetAttributes(&attr, reinterpret_cast<const void*>(&span_decode_kernel<float, fp8e4m3, false>));
}

void launch_var_span(const VarSpanLaunch& a, int src_dt, int dst_dt, double pad, hipStream_t stream) {
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

void launch_span_decode(const SpanLaunch& a, int src_dt, int dst_dt, const float* shift, const float* scale,
                        hipStream_t stream) {
  if (a.n_seg < 0 || a.n_seg > kMaxLaunchSegs) throw std::invalid_argument("span decode: bad segment count");
  if ((a.split != 1 && a.split != 2 && a.split != 4) || (a.split > 1 && a.part_crc == nullptr))
    throw std::invalid_argument("span decode: bad split");
  if (!is_float_dt(dst_dt) && is_float_dt(src_dt))
    throw std::invalid_argument("collate: float records cannot be cast to an integer dtype");
  if (shift && !is_float_dt(dst_dt)) throw std::invalid_argument("collate: normalisation needs a float dtype");
  for (int i = 0; i < a.n_seg; ++i) {
    // the kernel stages a segment whole in LDS and its row positions next to it
    if (a.s[i].len == 0 || a.s[i].len > tk::kSpanSegMax || a.s[i].row_end < a.s[i].row_begin ||
        a.s[i].row_end - a.s[i].row_begin > tk::kSpanMaxSegRows || a.s[i].batch >= kMaxGroup)
      throw std::invalid_argument("span decode: malformed segment");
  }
  TK_DISPATCH_SRC(launch_span_t, a, shift, scale, stream)
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw std::runtime_error(std::string("span decode launch: ") + hipGetErrorString(e));
}

}  // namespace tkh
