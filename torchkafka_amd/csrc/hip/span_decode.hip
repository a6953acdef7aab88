// gfx950 decode of Kafka RecordBatches straight out of the pinned broker logs
// (kPackRecordSpan, csrc/core/span.h).
//
// Replaces, for schema-declared fixed-width records, the work the reference does per record on
// the CPU -- kafka-python's CRC check of every fetched batch (check_crcs) and value decode,
// then `_process` and torch.stack (kafka_dataset.py:156-162) -- and, in this
// framework's host path, the worker's CRC pass and value copy into the ring slot.
//
// One 256-thread workgroup per segment (<= 128 KiB of one partition log; 1 workgroup per CU):
//   1. the segment is copied into a contiguous LDS image (16-byte front offset) by LDS-DMA,
//      global_load_lds_dwordx4, one 1 KiB load in flight per wave (fewer outstanding PCIe reads
//      move more bytes; the launches of two or three decode streams keep the link busy), plus
//      the slot's row positions and the CRC slice tables;
//   2. CRC32C of a RecordBatch's bytes [21, end): 256 lanes x 260- or 516-byte chunks ending at
//      the range end (an odd dword count per chunk: the 32 lanes of a ds_read_b32 group hit 32
//      different banks), slice-by-8 tables in LDS fed by a sliding dword window (two
//      ds_read_b32 + two v_alignbyte per 8 bytes), then 6 shuffle levels and 2 LDS levels of
//      "shift by 2^j chunks" (4 table lookups each, csrc/core/crc32c.cpp crc32c_span_tables);
//   3. values: a wave per row for rows of >= 32 16-byte groups (lanes over the row's groups
//      held by this segment), else (row, group) pairs strided over the block; each group is
//      read as a 5-dword window + v_alignbyte (values sit at arbitrary byte offsets behind
//      their varint headers), converted (dtypes.h: bit-exact with Tensor.to), stored 8-16 B
//      per lane;
//   4. lane 0: a RecordBatch held whole by the segment is compared with its header CRC; a
//      mismatch stores the segment index into the batch's host-mapped error word (the driver
//      reads it when the slot is released and never commits the batch); a RecordBatch cut
//      into several segments stores the raw partial CRC for the driver to chain.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <stdexcept>
#include <string>

#include "convert.h"
#include "span_decode.h"

namespace tkh {

namespace {

constexpr int kThreads = 256;
constexpr int kFront = 16;  // LDS image offset: boundary reads may start up to 3 bytes before it
constexpr int kLoads = int((tk::kSpanSegMax + 32) / 16 / kThreads) + 1;
constexpr int kBufBytes = kFront + int(tk::kSpanSegMax) + 64;

__device__ __forceinline__ uint32_t keep_from(int32_t a, int32_t c) {
  // bytes of the dword at address a whose address is >= c
  const int32_t d = c - a;
  return d <= 0 ? 0xFFFFFFFFu : d >= 4 ? 0u : (0xFFFFFFFFu << (8 * d));
}

__device__ __forceinline__ uint32_t shift_op(const uint32_t* __restrict__ set, uint32_t level, uint32_t c) {
  const uint32_t* S = set + level * 1024u;
  return S[c & 255u] ^ S[256u + ((c >> 8) & 255u)] ^ S[512u + ((c >> 16) & 255u)] ^ S[768u + (c >> 24)];
}

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
  __shared__ uint32_t tab[2048];
  __shared__ uint32_t wcrc[kThreads / 64];

  const int t = int(threadIdx.x);
  const SpanDevSeg& sg = a.s[blockIdx.x];
  const SpanBatchOut& bo = a.b[sg.batch];
  const uint32_t len = sg.len, flags = sg.flags;
  const uintptr_t su = reinterpret_cast<uintptr_t>(sg.src);
  const int32_t head = int32_t(su & 15u);
  const uint32_t nchunk = (uint32_t(head) + len + 15u) >> 4;
  const uint32_t row_begin = sg.row_begin;
  const uint32_t nrows = sg.row_end - row_begin;
  const bool do_crc = (flags & tk::kSegCrc) != 0;

  // ---- 1. stage: LDS-DMA (global_load_lds_dwordx4).  Wave w's i-th load writes chunks
  // [i * 256 + 64 w, +64) -- one contiguous KiB of the image, exactly the instruction's
  // wave-uniform-base + 16 * lane layout -- with no VGPR staging.  Each wave keeps ONE load in
  // flight: zero-copy PCIe reads lose bandwidth with many outstanding requests (tools/probes/
  // tlb_probe.hip: 53 GB/s at 32 reading blocks, 40 at 512), and with two or three decode
  // kernels running at once the link stays full (config 2: 53 M rec/s with one load in flight
  // per wave, 41-44 M with 2-8, 46 M with all 17 issued up front).
  {
    const uint8_t* gsrc = reinterpret_cast<const uint8_t*>(su - uint32_t(head));
    const int wv = t >> 6;
    auto dma = [&](int i) {
      const uint32_t c = uint32_t(t + i * kThreads);
      if (c < nchunk)
        __builtin_amdgcn_global_load_lds(
            gsrc + 16u * c,
            (__attribute__((address_space(3))) void*)(buf + kFront + 16 * (i * kThreads + wv * 64)), 16, 0, 0);
    };
    const int burst = a.burst;  // 0: all in flight; k > 0: wait after every k (default 1)
    dma(0);
    // the row positions and CRC tables load behind the first chunk (waiting for them waits for it)
    const int64_t base = int64_t(sg.log_pos) - int64_t(head) - kFront;  // log position of LDS byte 0
    for (uint32_t r = uint32_t(t); r < nrows; r += kThreads)
      rel[r] = int32_t(int64_t(bo.row_pos[row_begin + r]) - base);
    if (do_crc)
      for (int i = t; i < 2048; i += kThreads) tab[i] = a.tabs[tk::kSpanTabSlice + i];
#pragma unroll
    for (int i = 1; i < kLoads; ++i) {
      if (16u * uint32_t(i * kThreads) >= 16u * nchunk) break;  // block-uniform: no wave has chunk i
      dma(i);
      if (burst > 0 && (i % burst) == burst - 1) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  }
  __syncthreads();
  const uint32_t* b32 = reinterpret_cast<const uint32_t*>(buf);
  const int32_t lo_b = kFront + head, hi_b = kFront + head + int32_t(len);  // valid LDS bytes

  // ---- 2. CRC32C lanes (span.h: end-aligned chunks of L bytes: one slice-by-4 step, then
  // slice-by-8 steps over a sliding dword window)
  uint32_t crc = 0;
  const uint32_t* shift_set = a.tabs + tk::kSpanTabShift;
  if (do_crc) {
    const bool first = (flags & tk::kSegCrcFirst) != 0;
    const int32_t c0 = lo_b + (first ? 21 : 0), c1 = hi_b;
    const int32_t L = int32_t(tk::span_lane_bytes(uint32_t(c1 - c0)));
    if (L != int32_t(tk::kSpanLaneSmall)) shift_set += tk::kSpanTabShiftSet;
    const int32_t start = c1 - (int32_t(tk::kSpanLanes) - t) * L;
    const int32_t nsteps = (L - 4) >> 3;
    if (start + 4 > c0) {  // the chunk's first 4 bytes (>= kFront - 3 whenever start + 4 > c0)
      const int32_t w = start >> 2, sh = start & 3;
      uint32_t x = __builtin_amdgcn_alignbyte(b32[w + 1], b32[w], sh);
      if (start < c0 + 4) {
        const uint32_t keep = keep_from(start, c0);
        x &= keep;
        if (first) x ^= keep & ~keep_from(start, c0 + 4);  // the 0xFFFFFFFF initial value
      }
      crc = tab[768 + (x & 255u)] ^ tab[512 + ((x >> 8) & 255u)] ^ tab[256 + ((x >> 16) & 255u)] ^ tab[x >> 24];
    }
    const int32_t a1 = start + 4;
    const int32_t j0 = a1 >= c0 ? 0 : (c0 - a1) >> 3;  // 8-byte groups wholly below c0 are skipped
    if (j0 < nsteps) {
      int32_t ad = a1 + 8 * j0;
      int32_t w = ad >> 2;
      const int32_t sh = ad & 3;
      uint32_t lo = b32[w];
      for (int32_t j = j0; j < nsteps; ++j, ad += 8) {
        const uint32_t m1 = b32[w + 1], m2 = b32[w + 2];
        w += 2;
        uint32_t x = __builtin_amdgcn_alignbyte(m1, lo, sh), y = __builtin_amdgcn_alignbyte(m2, m1, sh);
        lo = m2;
        if (ad < c0 + 4) {
          const uint32_t kx = keep_from(ad, c0), ky = keep_from(ad + 4, c0);
          x &= kx;
          y &= ky;
          if (first) {
            x ^= kx & ~keep_from(ad, c0 + 4);
            y ^= ky & ~keep_from(ad + 4, c0 + 4);
          }
        }
        x ^= crc;
        crc = tab[1792 + (x & 255u)] ^ tab[1536 + ((x >> 8) & 255u)] ^ tab[1280 + ((x >> 16) & 255u)] ^
              tab[1024 + (x >> 24)] ^ tab[768 + (y & 255u)] ^ tab[512 + ((y >> 8) & 255u)] ^
              tab[256 + ((y >> 16) & 255u)] ^ tab[y >> 24];
      }
    }
    const int lane = t & 63;
#pragma unroll
    for (uint32_t j = 0; j < 6; ++j) {
      const uint32_t other = __shfl_down(crc, 1u << j, 64);
      if ((lane & ((2 << j) - 1)) == 0) crc = shift_op(shift_set, j, crc) ^ other;
    }
    if (lane == 0) wcrc[t >> 6] = crc;
  }

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
      D* __restrict__ orow = out + int64_t(row_begin + rr) * RE;
      if (nel == kPer && b0 >= lo_b && b0 + 16 <= hi_b) {
        const int32_t w = b0 >> 2, sh = b0 & 3;
        const uint32_t x0 = b32[w], x1 = b32[w + 1], x2 = b32[w + 2], x3 = b32[w + 3], x4 = b32[w + 4];
        const uint32_t o[4] = {__builtin_amdgcn_alignbyte(x1, x0, sh), __builtin_amdgcn_alignbyte(x2, x1, sh),
                               __builtin_amdgcn_alignbyte(x3, x2, sh), __builtin_amdgcn_alignbyte(x4, x3, sh)};
        S sv[kPer];
        __builtin_memcpy(sv, o, 16);
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

  // ---- 4. verdict
  if (do_crc) {
    __syncthreads();
    if (t == 0) {
      uint32_t c = shift_op(shift_set, 6, wcrc[0]) ^ wcrc[1];
      c = shift_op(shift_set, 7, c) ^ (shift_op(shift_set, 6, wcrc[2]) ^ wcrc[3]);
      constexpr uint32_t kWhole = tk::kSegCrcFirst | tk::kSegCrcLast;
      if ((flags & kWhole) == kWhole) {
        if ((c ^ 0xFFFFFFFFu) != sg.crc) *bo.err = int32_t(sg.seg);
      } else {
        bo.partials[sg.seg] = c;
      }
    }
  }
}

template <typename S, typename D>
void launch_span_t(const SpanLaunch& a, const float* shift, const float* scale, hipStream_t stream) {
  if (a.n_seg <= 0) return;
  if (shift)
    hipLaunchKernelGGL((span_decode_kernel<S, D, true>), dim3(unsigned(a.n_seg)), dim3(kThreads), 0, stream, a, shift,
                       scale);
  else
    hipLaunchKernelGGL((span_decode_kernel<S, D, false>), dim3(unsigned(a.n_seg)), dim3(kThreads), 0, stream, a,
                       shift, scale);
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

void launch_span_decode(const SpanLaunch& a, int src_dt, int dst_dt, const float* shift, const float* scale,
                        hipStream_t stream) {
  if (a.n_seg < 0 || a.n_seg > kMaxLaunchSegs) throw std::invalid_argument("span decode: bad segment count");
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
