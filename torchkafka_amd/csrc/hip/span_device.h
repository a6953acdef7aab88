// Device code shared by the span kernels (span_decode.hip: fixed-width values, json_span.hip: JSON
// text): one 256-thread workgroup per log segment (<= 128 KiB of one pinned partition log, so one
// workgroup per CU),
//   1. stage: the segment is copied into a contiguous LDS image (16-byte front offset) by LDS-DMA,
//      global_load_lds_dwordx4, one 1 KiB load in flight per wave (fewer outstanding PCIe reads
//      move more bytes; the launches of two or three decode streams keep the link busy);
//   2. crc_lanes: CRC32C of a RecordBatch's bytes [21, end): 256 lanes x 260- or 516-byte chunks
//      ending at the range end (an odd dword count per chunk: the 32 lanes of a ds_read_b32
//      group hit 32 different banks), slice-by-8 fed by a sliding dword window (two ds_read_b32 +
//      two v_alignbyte per 8 bytes) and looked up per NIBBLE in 16-entry LDS rows (span.h
//      kSpanTabNib: 16 conflict-free reads per 8 bytes instead of 8 byte-table reads at ~3-way
//      conflicts), then 6 shuffle levels of "shift by 2^j chunks" (4 table lookups each,
//      csrc/core/crc32c.cpp crc32c_span_tables);
//   3. crc_verdict (thread 0, after a barrier): 2 LDS levels merge the 4 wave CRCs; a RecordBatch
//      held whole by the segment is compared with its header CRC -- a mismatch stores the segment
//      index into the batch's host-mapped error word (the driver reads it when the slot is
//      released and never commits the batch) -- and a RecordBatch cut into several segments
//      stores the raw partial CRC for the driver to chain.
// Replaces kafka-python's check_crcs pass over every fetched RecordBatch.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "span.h"

namespace tkh {
namespace span {

constexpr int kThreads = 256;
constexpr int kFront = 16;  // LDS image offset: boundary reads may start up to 3 bytes before it
constexpr int kLoads = int((tk::kSpanSegMax + 32) / 16 / kThreads) + 1;
constexpr int kBufBytes = kFront + int(tk::kSpanSegMax) + 64;

// 16 bytes at LDS byte b0 of a 16-byte aligned image (any alignment of b0), for loops whose
// lanes read consecutive 16-byte pieces: two 16-byte-aligned ds_read_b128 per lane -- consecutive
// slots across the wave, conflict-free -- and the unaligned 16 bytes cut out of those 32 in
// registers.  Five ds_read_b32 at a 16-byte lane stride (the 5-dword window used before) cost a
// 4-way bank conflict each: banks (a/4) mod 32 in 32-lane groups (MI355X_MICROARCH.md §LDS).
// Reads up to the 16-byte boundary at or below b0 + 31: the image keeps 64 spare bytes at its end.
// `img` is the image as 16-byte slots.  The reads are nontemporal loads (a no-op hint for LDS)
// because the compiler otherwise narrows them to the dwords the selects below can pick --
// ds_read2_b32 pairs at a 16-byte lane stride, the conflicting pattern this replaces.
typedef uint32_t lds_v4u __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 lds16(const uint4* img16, int32_t b0) {
  const lds_v4u* img = reinterpret_cast<const lds_v4u*>(img16);
  const int32_t q = (b0 >> 2) & 3, sh = b0 & 3;
  const lds_v4u lv = __builtin_nontemporal_load(img + (b0 >> 4));
  const lds_v4u hv = __builtin_nontemporal_load(img + (b0 >> 4) + 1);
  const uint4 lo = make_uint4(lv.x, lv.y, lv.z, lv.w), hi = make_uint4(hv.x, hv.y, hv.z, hv.w);
  // dwords q .. q + 4 of lo:hi
  const uint32_t d0 = q == 0 ? lo.x : q == 1 ? lo.y : q == 2 ? lo.z : lo.w;
  const uint32_t d1 = q == 0 ? lo.y : q == 1 ? lo.z : q == 2 ? lo.w : hi.x;
  const uint32_t d2 = q == 0 ? lo.z : q == 1 ? lo.w : q == 2 ? hi.x : hi.y;
  const uint32_t d3 = q == 0 ? lo.w : q == 1 ? hi.x : q == 2 ? hi.y : hi.z;
  const uint32_t d4 = q == 0 ? hi.x : q == 1 ? hi.y : q == 2 ? hi.z : hi.w;
  uint4 v;
  v.x = __builtin_amdgcn_alignbyte(d1, d0, sh);
  v.y = __builtin_amdgcn_alignbyte(d2, d1, sh);
  v.z = __builtin_amdgcn_alignbyte(d3, d2, sh);
  v.w = __builtin_amdgcn_alignbyte(d4, d3, sh);
  return v;
}

__device__ __forceinline__ uint32_t keep_from(int32_t a, int32_t c) {
  // bytes of the dword at address a whose address is >= c
  const int32_t d = c - a;
  return d <= 0 ? 0xFFFFFFFFu : d >= 4 ? 0u : (0xFFFFFFFFu << (8 * d));
}

__device__ __forceinline__ uint32_t shift_op(const uint32_t* __restrict__ set, uint32_t level, uint32_t c) {
  const uint32_t* S = set + level * 1024u;
  return S[c & 255u] ^ S[256u + ((c >> 8) & 255u)] ^ S[512u + ((c >> 16) & 255u)] ^ S[768u + (c >> 24)];
}

// Stage 1.  Wave w's i-th load writes chunks [i * 256 + 64 w, +64) -- one contiguous KiB of the
// image, exactly the instruction's wave-uniform-base + 16 * lane layout -- with no VGPR staging.
// Each wave keeps `burst` loads in flight (0: all): zero-copy PCIe reads lose bandwidth with many
// outstanding requests (tools/probes/tlb_probe.hip: 53 GB/s at 32 reading blocks, 40 at 512), and
// with two or three decode kernels running at once the link stays full (config 2: 53 M rec/s with
// one load in flight per wave, 41-44 M with 2-8, 46 M with all 17 issued up front).
// `behind_first()` runs once the first load is issued (the row tables and CRC tables load behind
// it: waiting for them waits for it).  The caller's __syncthreads() completes the image.
template <class F>
__device__ __forceinline__ void stage(const uint8_t* src, uint32_t len, uint8_t* buf, int burst, F&& behind_first) {
  const int t = int(threadIdx.x);
  const uintptr_t su = reinterpret_cast<uintptr_t>(src);
  const uint32_t head = uint32_t(su & 15u);
  const uint32_t nchunk = (head + len + 15u) >> 4;
  const uint8_t* gsrc = reinterpret_cast<const uint8_t*>(su - head);
  const int wv = t >> 6;
  auto dma = [&](int i) {
    const uint32_t c = uint32_t(t + i * kThreads);
    if (c < nchunk)
      __builtin_amdgcn_global_load_lds(
          gsrc + 16u * c, (__attribute__((address_space(3))) void*)(buf + kFront + 16 * (i * kThreads + wv * 64)), 16,
          0, 0);
  };
  dma(0);
  behind_first();
#pragma unroll
  for (int i = 1; i < kLoads; ++i) {
    if (16u * uint32_t(i * kThreads) >= 16u * nchunk) break;  // block-uniform: no wave has chunk i
    dma(i);
    if (burst > 0 && (i % burst) == burst - 1) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
}

// The nibble rows in LDS: row r (16 words) at byte r * 256 of a 256-byte aligned 4 KiB array, so a
// lookup's LDS address is (row base) | (nibble * 4) with the nibble in the address's low byte.
constexpr int kNibRowWords = 64;
constexpr int kNibLdsWords = 16 * kNibRowWords;
using lds_u32 = __attribute__((address_space(3))) const uint32_t;

__device__ __forceinline__ void load_nib_rows(uint32_t* tab, const uint32_t* __restrict__ tabs) {
  for (int i = int(threadIdx.x); i < int(tk::kSpanTabNibWords); i += kThreads)
    tab[(i >> 4) * kNibRowWords + (i & 15)] = tabs[tk::kSpanTabNib + i];
}

// Slice-by-4 of one dword through the nibble rows: byte i of w goes through byte table B - i,
// i.e. rows 2 (B - i) (low nibble) and 2 (B - i) + 1 (high nibble).  The nibbles of all four
// bytes are pre-scaled to byte offsets (x4) at once; each lookup is then ONE v_perm_b32 (byte i of
// the scaled nibbles into the address's low byte, the row base's upper bytes above it) and a
// ds_read_b32.
template <int B>
__device__ __forceinline__ uint32_t nib_dword(uint32_t nbase, uint32_t w) {
  const uint32_t lo = (w << 2) & 0x3C3C3C3Cu, hi = (w >> 2) & 0x3C3C3C3Cu;
  uint32_t r = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const uint32_t sel = 0x07060500u | uint32_t(i);  // byte 0 <- byte i of src1, bytes 1-3 <- src0
    const uint32_t a0 = __builtin_amdgcn_perm(nbase + uint32_t(2 * (B - i)) * 256u, lo, sel);
    const uint32_t a1 = __builtin_amdgcn_perm(nbase + uint32_t(2 * (B - i) + 1) * 256u, hi, sel);
    r ^= *(lds_u32*)uintptr_t(a0) ^ *(lds_u32*)uintptr_t(a1);
  }
  return r;
}

// Stage 2 (every thread, after the barrier that completed the image).  The CRC range is
// [c0, c1) in LDS bytes: [lo_b + 21, hi_b) for the segment holding a RecordBatch's start, else
// [lo_b, hi_b); `tab` is the LDS copy of the nibble rows (load_nib_rows).  Each wave's lane 0 leaves the wave's CRC in wcrc[wave]; returns the shift-table
// set of the lane size used (for crc_verdict).
// `lane_base`: a workgroup that holds only part of the range (span_decode_kernel's split) runs
// lanes lane_base.. of the whole range's layout on its first threads (whole waves).
__device__ __forceinline__ const uint32_t* crc_lanes(const uint32_t* __restrict__ b32, const uint32_t* __restrict__ tab,
                                                     const uint32_t* __restrict__ tabs, int32_t lo_b, int32_t hi_b,
                                                     uint32_t flags, uint32_t* wcrc, int lane_base = 0) {
  const int t = int(threadIdx.x) + lane_base;
  const uint32_t* shift_set = tabs + tk::kSpanTabShift;
  uint32_t crc = 0;
  const uint32_t nbase = uint32_t(uintptr_t((lds_u32*)tab));  // the LDS byte address
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
    crc = nib_dword<3>(nbase, x);
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
      crc = nib_dword<7>(nbase, x) ^ nib_dword<3>(nbase, y);
    }
  }
  const int lane = t & 63;
#pragma unroll
  for (uint32_t j = 0; j < 6; ++j) {
    const uint32_t other = __shfl_down(crc, 1u << j, 64);
    if ((lane & ((2 << j) - 1)) == 0) crc = shift_op(shift_set, j, crc) ^ other;
  }
  if (lane == 0) wcrc[t >> 6] = crc;
  return shift_set;
}

// Stage 3 (thread 0 only, after a barrier that follows crc_lanes).
__device__ __forceinline__ void crc_verdict(const uint32_t* __restrict__ shift_set, const uint32_t* wcrc,
                                            uint32_t flags, uint32_t want, uint32_t seg, int32_t* err,
                                            uint32_t* partials) {
  uint32_t c = shift_op(shift_set, 6, wcrc[0]) ^ wcrc[1];
  c = shift_op(shift_set, 7, c) ^ (shift_op(shift_set, 6, wcrc[2]) ^ wcrc[3]);
  constexpr uint32_t kWhole = tk::kSegCrcFirst | tk::kSegCrcLast;
  if ((flags & kWhole) == kWhole) {
    if ((c ^ 0xFFFFFFFFu) != want) *err = int32_t(seg);
  } else {
    partials[seg] = c;
  }
}

}  // namespace span
}  // namespace tkh
