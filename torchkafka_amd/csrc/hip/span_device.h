// Device code shared by the span kernels (span_decode.hip: fixed-width and var-len values,
// json_span.hip: JSON text): one workgroup per log segment (<= 128 KiB of one partition log, pinned
// host memory or its HBM mirror), streamed through a ring of NB LDS windows of 10 KiB:
//
//   window k = segment bytes [w0 + k W, w0 + (k+1) W), W = kSpanWin (10,240), the windows ending at
//   the segment's end (span.h SpanWindows).  The workgroup is 8 compute waves (512 threads: the CRC
//   lanes; two waves per SIMD, so one hides the other's LDS latency) and ONE loader wave.  The loader wave only issues LDS-DMA loads (global_load_lds_dwordx4, a
//   contiguous KiB per instruction, kSpanWinLoads of them per window) and keeps NB - 1 windows in
//   flight; since nothing else is on its vector-memory counter it waits for the oldest window with a
//   counted s_waitcnt vmcnt (the compute waves' stores would make a count meaningless, and a
//   vmcnt(0) would drain the windows behind it).  One raw s_barrier per window hands window k to the
//   compute waves and hands them window k-1's buffer back.  The compute waves, per window:
//     * the values / texts whose 16-byte group (or piece) STARTS in the window's bytes (staged with
//       16 bytes before and 48 after, so a group reaching past the window is whole in LDS): a wave
//       per row, its lanes over the row's groups (a row's groups share one alignment, so the 16
//       bytes of a group are cut out of two aligned ds_read_b128 with wave-uniform selects);
//     * CRC32C: lane t folds its 20-byte piece of the window into a running state (slice-by-8 fed by
//       a sliding dword window, looked up per NIBBLE in 16-entry LDS rows: conflict-free), the state
//       crossing the other lanes' bytes with one gap operator between windows; after the last
//       window each lane's state is multiplied by its lane constant (span.h kSpanTabLaneMul: the
//       shift over the later lanes' bytes, loaded before the first window) and the products are
//       xored over the wave and the 8 waves (span.h, host mirror crc32c.cpp crc32c_span_emulate).
//   A workgroup needs 39-47 KiB of LDS (round 4: the whole 143 KiB segment) and its loads are always
//   NB - 1 windows ahead of its compute, so it holds a CU for a fraction of the time it used to.
//
// A RecordBatch held whole by the segment is compared with its header CRC -- a mismatch stores the
// segment index into the batch's host-mapped error word (the driver reads it when the slot is
// released and never commits the batch) -- and one cut into several segments stores the raw
// partial CRC for the driver to chain.
// Replaces kafka-python's check_crcs pass over every fetched RecordBatch.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "span.h"

namespace tkh {
namespace span {

constexpr int kThreads = int(tk::kSpanLanes);  // compute threads: 8 waves, one CRC lane each
constexpr int kBlock = kThreads + 64;      // + the loader wave
constexpr int kFront = 16;     // image coordinates: segment byte i is image byte kFront + (src & 15) + i
constexpr int32_t kWin = int32_t(tk::kSpanWin);
constexpr int kPad = tk::kSpanWinPad;          // LDS bytes before a window's first staged byte
constexpr int kWinBytes = tk::kSpanWinBytes;    // one window buffer (span.h)
constexpr int kWinLoads = tk::kSpanWinLoads;    // the loader wave's LDS-DMA instructions per window
static_assert(kWinBytes % 16 == 0, "window buffers stay 16-byte aligned");
static_assert(kWinLoads <= 21, "counted waits: at most 3 windows of loads in flight (vmcnt <= 63)");
static_assert(kThreads == 512, "crc_merge / crc_finish: 8 compute waves, one lane constant per thread");

__device__ __forceinline__ bool loader_wave() { return threadIdx.x >= kThreads; }

// 16 bytes at LDS byte b0 of a 16-byte aligned image (any alignment of b0), for loops whose
// lanes read consecutive 16-byte pieces: two 16-byte-aligned ds_read_b128 per lane -- consecutive
// slots across the wave, conflict-free -- and the unaligned 16 bytes cut out of those 32 in
// registers.  Five ds_read_b32 at a 16-byte lane stride cost a 4-way bank conflict each: banks
// (a/4) mod 32 in 32-lane groups (MI355X_MICROARCH.md §LDS).  Reads up to the 16-byte boundary at
// or below b0 + 31.  The reads are nontemporal loads (a no-op hint for LDS) because the compiler
// otherwise narrows them to the dwords the selects below can pick -- ds_read2_b32 pairs at a
// 16-byte lane stride, the conflicting pattern this replaces.
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

// span::lds16 for a whole wave reading the same row: the lanes' groups share one alignment
// (b0 mod 16), so the dword selects are one wave-uniform branch instead of 15 v_cndmask per lane.
__device__ __forceinline__ uint4 lds16_row(const uint4* img16, int32_t b0) {
  const lds_v4u* img = reinterpret_cast<const lds_v4u*>(img16);
  const int32_t a = __builtin_amdgcn_readfirstlane(b0 & 15), q = a >> 2, sh = a & 3;
  const lds_v4u lv = __builtin_nontemporal_load(img + (b0 >> 4));
  const lds_v4u hv = __builtin_nontemporal_load(img + (b0 >> 4) + 1);
  uint32_t d[5];
  if (q == 0) {
    d[0] = lv.x, d[1] = lv.y, d[2] = lv.z, d[3] = lv.w, d[4] = hv.x;
  } else if (q == 1) {
    d[0] = lv.y, d[1] = lv.z, d[2] = lv.w, d[3] = hv.x, d[4] = hv.y;
  } else if (q == 2) {
    d[0] = lv.z, d[1] = lv.w, d[2] = hv.x, d[3] = hv.y, d[4] = hv.z;
  } else {
    d[0] = lv.w, d[1] = hv.x, d[2] = hv.y, d[3] = hv.z, d[4] = hv.w;
  }
  uint4 v;
  v.x = __builtin_amdgcn_alignbyte(d[1], d[0], sh);
  v.y = __builtin_amdgcn_alignbyte(d[2], d[1], sh);
  v.z = __builtin_amdgcn_alignbyte(d[3], d[2], sh);
  v.w = __builtin_amdgcn_alignbyte(d[4], d[3], sh);
  return v;
}

__device__ __forceinline__ uint32_t keep_from(int32_t a, int32_t c) {
  // bytes of the dword at address a whose address is >= c
  const int32_t d = c - a;
  return d <= 0 ? 0xFFFFFFFFu : d >= 4 ? 0u : (0xFFFFFFFFu << (8 * d));
}

// c times the constant k modulo the CRC32C polynomial, both in zlib's reflected representation
// (crc32c.cpp Tables::multmodp), branch-free: 32 steps of a bit-field extract, a masked xor and a
// multiply-by-x -- about 220 VALU instructions and no memory access, where the shift-table tree it
// replaces waited for 9 dependent global table reads after the last window (profiles/r05_s29).
__device__ __forceinline__ uint32_t gf_mul(uint32_t k, uint32_t c) {
  uint32_t p = 0;
#pragma unroll
  for (int i = 31; i >= 0; --i) {
    p ^= c & uint32_t(int32_t(k << (31 - i)) >> 31);
    c = (c >> 1) ^ (0x82F63B78u & uint32_t(int32_t(c << 31) >> 31));
  }
  return p;
}

using Windows = tk::SpanWindows;  // span.h

// The loader wave issues window k's LDS-DMA loads into `buf` (kWinBytes); `gbase` is the global
// address of image byte kFront (the segment's first byte rounded down to 16).  LDS byte of image
// byte x: kPad + x - stage_lo(k).  Instruction r writes chunks [64 r, 64 r + 64) -- one contiguous
// KiB, the instruction's wave-uniform-base + 16 * lane layout -- with no VGPR staging; lanes past
// the window's chunks reload its last chunk into their own slot (past the staged bytes), so every
// window is exactly kWinLoads instructions.
__device__ __forceinline__ void issue_window(const uint8_t* gbase, const Windows& W, int k, uint8_t* buf) {
  const int lane = int(threadIdx.x) & 63;
  const int32_t a = W.stage_lo(k);
  const int32_t last = ((W.stage_hi(k) - a) >> 4) - 1;
  const uint8_t* g = gbase + (a - kFront);
#pragma unroll
  for (int r = 0; r < kWinLoads; ++r) {
    const int32_t c = min(r * 64 + lane, last);
    __builtin_amdgcn_global_load_lds(g + 16 * c, (__attribute__((address_space(3))) void*)(buf + kPad + 1024 * r), 16,
                                     0, 0);
  }
}

// The loader wave: every load older than the youngest `n` windows it issued has landed.
__device__ __forceinline__ void loader_wait(int n) {
  if (n <= 0)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  else if (n == 1)
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(kWinLoads) : "memory");
  else
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * kWinLoads) : "memory");
}

// A workgroup barrier that leaves the loader wave's loads in flight (a __syncthreads() fence waits
// for every vector-memory operation): LDS operations completed, then s_barrier.
__device__ __forceinline__ void window_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// Row ranges per window: rows [lo[k], hi[k]) hold every group a window owns (rows in any order;
// a row outside the range owns nothing there).  Each thread reports its row's first and last
// owned key window (kf > kl: the row owns nothing); wave ballots keep one LDS atomic per window.
struct RowWins {
  int32_t lo[32], hi[32];
};
__device__ __forceinline__ void row_wins_init(RowWins& rw, int nw) {
  const int t = int(threadIdx.x);
  if (t < nw) {
    rw.lo[t] = 0x7FFFFFFF;
    rw.hi[t] = 0;
  }
}
__device__ __forceinline__ void row_wins_add(RowWins& rw, int nw, int32_t row_base, bool valid, int kf, int kl) {
  const int lane = int(threadIdx.x) & 63;
  for (int k = 0; k < nw; ++k) {
    const unsigned long long m = __ballot(valid && kf <= k && k <= kl);
    if (m && lane == 0) {
      atomicMin(&rw.lo[k], row_base + int32_t(__builtin_ctzll(m)));
      atomicMax(&rw.hi[k], row_base + 64 - int32_t(__builtin_clzll(m)));
    }
  }
}

// The 16-byte units a window owns, spread over the compute waves: rows [ra, rb), each row's owned
// units [ulo, uhi) (range(rr, &ulo, &uhi)) in chunks of 64 lanes.  A wave per row (rows strided
// over the compute waves), or with `wide` all of them on every row (its chunks strided over them) --
// for rows so long that a window holds only a few of them.  fn(rr, u, row_key0) runs with every lane
// of the wave on the same row.
template <class Range, class Fn>
__device__ __forceinline__ void for_rows(int32_t ra, int32_t rb, bool wide, Range&& range, Fn&& fn) {
  const int t = int(threadIdx.x), lane = t & 63, wv = t >> 6;
  const int32_t r_step = wide ? 1 : kThreads / 64, c_off = wide ? 64 * wv : 0, c_step = wide ? kThreads : 64;
  for (int32_t rr = ra + (wide ? 0 : wv); rr < rb; rr += r_step) {
    int32_t ulo = 0, uhi = 0;
    range(rr, &ulo, &uhi);
    for (int32_t u = ulo + c_off + lane; u < uhi; u += c_step) fn(rr, u);
  }
}
// First unit of a row whose key (key0 + 16 u) is >= x.
__device__ __forceinline__ int32_t unit_from(int32_t key0, int32_t x) { return key0 >= x ? 0 : (x - key0 + 15) >> 4; }

// The nibble rows in LDS: row r (16 words) at byte r * 256 of a 256-byte aligned 4 KiB array, so a
// lookup's LDS address is (row base) | (nibble * 4) with the nibble in the address's low byte; the
// gap operator's row i sits in words 16..31 of row i.
constexpr int kNibRowWords = 64;
constexpr int kNibLdsWords = 16 * kNibRowWords;
using lds_u32 = __attribute__((address_space(3))) const uint32_t;

__device__ __forceinline__ void load_nib_rows(uint32_t* tab, const uint32_t* __restrict__ tabs) {  // compute threads
  for (int i = int(threadIdx.x); i < int(tk::kSpanTabNibWords); i += kThreads)
    tab[(i >> 4) * kNibRowWords + (i & 15)] = tabs[tk::kSpanTabNib + i];
  for (int i = int(threadIdx.x); i < int(tk::kSpanTabGapWords); i += kThreads)
    tab[(i >> 4) * kNibRowWords + 16 + (i & 15)] = tabs[tk::kSpanTabGap + i];
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

// The window gap: the state after kSpanWin - kSpanPiece zero bytes (8 nibble lookups).
__device__ __forceinline__ uint32_t gap_op(uint32_t nbase, uint32_t c) {
  uint32_t r = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) r ^= *(lds_u32*)uintptr_t(nbase + uint32_t(i) * 256u + 64u + ((c >> (4 * i)) & 15u) * 4u);
  return r;
}

// One lane's piece of window k folded into its running state `crc` (every compute thread, every
// window).  b32: the window's LDS bytes as dwords; `off` = LDS byte of image byte 0 (kPad -
// stage_lo(k)); c0: image byte of the first CRC'd byte ([lo + 21, hi) for the segment holding a
// RecordBatch's start, else [lo, hi)); `first`: inject the 0xFFFFFFFF initial value into its first
// 4 bytes.  A piece wholly past c0 + 4 takes the straight-line path (no masks); the few around c0
// take the masked loop.
__device__ __forceinline__ uint32_t crc_piece(const uint32_t* __restrict__ b32, uint32_t nbase, const Windows& W,
                                              int k, int32_t off, int32_t c0, bool first, uint32_t crc) {
  const int t = int(threadIdx.x);
  constexpr int32_t P = int32_t(tk::kSpanPiece);
  constexpr int32_t nsteps = (P - 4) >> 3;
  if (k > 0) crc = gap_op(nbase, crc);  // still zero before the first CRC'd byte
  const int32_t start = W.w0 + k * kWin + t * P + off;  // LDS byte of the piece
  const int32_t cl = c0 + off;                          // LDS byte of c0
  const int32_t sh = start & 3;                         // the same for every lane and window
  int32_t w = start >> 2;
  if (start >= cl + 4) {
    uint32_t lo = b32[w + 1];
    crc = nib_dword<3>(nbase, __builtin_amdgcn_alignbyte(lo, b32[w], sh) ^ crc);
#pragma unroll
    for (int32_t j = 0; j < nsteps; ++j) {
      const uint32_t m1 = b32[w + 2 + 2 * j], m2 = b32[w + 3 + 2 * j];
      const uint32_t x = __builtin_amdgcn_alignbyte(m1, lo, sh) ^ crc, y = __builtin_amdgcn_alignbyte(m2, m1, sh);
      lo = m2;
      crc = nib_dword<7>(nbase, x) ^ nib_dword<3>(nbase, y);
    }
    return crc;
  }
  if (start + 4 > cl) {
    uint32_t x = __builtin_amdgcn_alignbyte(b32[w + 1], b32[w], sh);
    const uint32_t keep = keep_from(start, cl);
    x &= keep;
    if (first) x ^= keep & ~keep_from(start, cl + 4);  // the 0xFFFFFFFF initial value
    crc = nib_dword<3>(nbase, x ^ crc);
  }
  const int32_t a1 = start + 4;
  const int32_t j0 = a1 >= cl ? 0 : (cl - a1) >> 3;  // 8-byte groups wholly below c0 are skipped
  if (j0 < nsteps) {
    int32_t ad = a1 + 8 * j0;
    w = ad >> 2;
    uint32_t lo = b32[w];
    for (int32_t j = j0; j < nsteps; ++j, ad += 8) {
      const uint32_t m1 = b32[w + 1], m2 = b32[w + 2];
      w += 2;
      uint32_t x = __builtin_amdgcn_alignbyte(m1, lo, sh), y = __builtin_amdgcn_alignbyte(m2, m1, sh);
      lo = m2;
      if (ad < cl + 4) {
        const uint32_t kx = keep_from(ad, cl), ky = keep_from(ad + 4, cl);
        x &= kx;
        y &= ky;
        if (first) {
          x ^= kx & ~keep_from(ad, cl + 4);
          y ^= ky & ~keep_from(ad + 4, cl + 4);
        }
      }
      x ^= crc;
      crc = nib_dword<7>(nbase, x) ^ nib_dword<3>(nbase, y);
    }
  }
  return crc;
}

// After the last window (compute threads, `crc` as pipeline() returns it: already moved to the
// segment part's end): the xor of the wave's 64 lane states; lane 0 leaves it in wcrc[wave].
__device__ __forceinline__ void crc_merge(uint32_t crc, uint32_t* wcrc) {
  const int t = int(threadIdx.x), lane = t & 63;
#pragma unroll
  for (int j = 32; j >= 1; j >>= 1) crc ^= uint32_t(__shfl_xor(int(crc), j, 64));
  if (lane == 0) wcrc[t >> 6] = crc;
}

// Segment parts (SpanLaunch::parts = P > 1): P workgroups share one segment, part q taking windows
// [span_part_k0(q), span_part_k0(q + 1)) -- P times the loads in flight for a lone segment.  Each
// part folds its windows' CRC pieces from a zero state (the gap operator of a zero state is zero),
// its lane constants also carry the whole windows after its last one (so its merged CRC sits at the
// segment's end), and it xors that CRC and its own bit into the segment's 64-bit accumulator with
// ONE returning agent-scope atomic: the part whose returned bits complete the set takes the sum,
// gives the verdict and zeroes the word for the next launch on its stream.  Host mirror:
// crc32c_span_emulate.
struct Part {
  int32_t seg, q, k0, k1;
};
__device__ __forceinline__ Part part_of(int parts, int32_t nw) {
  const int32_t b = int32_t(blockIdx.x), seg = b / parts, q = b - seg * parts;
  return Part{seg, q, tk::span_part_k0(q, parts, nw), tk::span_part_k0(q + 1, parts, nw)};
}

// Thread 0 only, after a barrier that follows crc_merge: the xor of the 8 wave CRCs; with parts,
// the accumulation above (`acc`: the segment's two words, 8-byte aligned); then the verdict (a
// RecordBatch held whole) or the raw partial.
__device__ __forceinline__ void crc_finish(const uint32_t* wcrc, uint32_t flags, uint32_t want, uint32_t seg,
                                           int32_t* err, uint32_t* partials, int parts, int q, uint32_t* acc) {
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < kThreads / 64; ++i) c ^= wcrc[i];
  if (parts > 1) {
    auto* word = reinterpret_cast<unsigned long long*>(acc);
    const uint32_t bit = 1u << q;
    const unsigned long long old = __hip_atomic_fetch_xor(word, (static_cast<unsigned long long>(bit) << 32) | c,
                                                          __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if ((uint32_t(old >> 32) | bit) != (1u << parts) - 1u) return;  // another part gives the verdict
    c ^= uint32_t(old);
    // every part of this launch has arrived: zero for the launch that reuses the set.  An atomic,
    // like the parts' xors: the parts run on all 8 XCDs (blocks b .. b + 7), and a plain store
    // stays in this XCD's L2, not coherent with the atomics of the next user of the word
    // (MI355X_MICROARCH.md, inter-workgroup visibility: 8-B agent atomics on both sides)
    __hip_atomic_exchange(word, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  constexpr uint32_t kWhole = tk::kSegCrcFirst | tk::kSegCrcLast;
  if ((flags & kWhole) == kWhole) {
    if ((c ^ 0xFFFFFFFFu) != want) *err = int32_t(seg);
  } else {
    partials[seg] = c;
  }
}

// The pipeline every span kernel runs (all kBlock threads call it) over windows [k0, k1) of the
// segment (all of them, or one part's).  The loader wave issues the
// first NB - 1 windows; the compute threads meanwhile run `setup` (row tables into LDS); after a
// barrier every thread runs `prepare` (per-row work that needs the tables: row window ranges,
// scans, descriptors -- it may contain __syncthreads(); the loader wave's threads must do no work
// in it), then for every window k:
//   loader: wait until window k landed (counted vmcnt) -- barrier -- issue window k + NB - 1 into
//           the buffer window k - 1 used;
//   compute: barrier -- `body(k, buf, off)` (the window's values; off = LDS byte of image byte 0) --
//           its CRC pieces.
// Returns the lane's CRC state moved to the segment's end (lane constant, span.h kSpanTabLaneMul: its
// load is issued before the windows), or 0 when the segment carries no CRC, and on the loader wave.
template <int NB, class Setup, class Prepare, class Body>
__device__ __forceinline__ uint32_t pipeline(const uint8_t* src, const Windows& W, int32_t k0, int32_t k1,
                                             uint8_t (*bufs)[kWinBytes], uint32_t* tab,
                                             const uint32_t* __restrict__ tabs, int32_t c0, bool do_crc, bool first,
                                             Setup&& setup, Prepare&& prepare, Body&& body) {
  static_assert(NB >= 2 && NB <= 4, "2..4 window buffers");
  const uint8_t* gbase = reinterpret_cast<const uint8_t*>(reinterpret_cast<uintptr_t>(src) & ~uintptr_t(15));
  const bool loader = loader_wave();
  if (loader) {
    for (int j = 0; j < NB - 1 && k0 + j < k1; ++j) issue_window(gbase, W, k0 + j, bufs[j]);
  } else {
    if (do_crc) load_nib_rows(tab, tabs);
    setup();
  }
  window_barrier();  // the row tables (the compute waves' LDS writes)
  prepare();
  __syncthreads();  // (drains the loader's first windows: they were needed first anyway)
  const uint32_t nbase = uint32_t(uintptr_t((lds_u32*)tab));  // the LDS byte address
  const uint32_t lane_k =
      do_crc && !loader ? tabs[tk::kSpanTabLaneMul + uint32_t(W.nw - k1) * tk::kSpanLanes + threadIdx.x] : 0u;
  uint32_t crc = 0;
  for (int k = k0; k < k1; ++k) {
    const int j = k - k0;
    if (loader) {
      // windows issued so far: up to min(k + NB - 2, k1 - 1); all but those after k must have landed
      loader_wait(min(k + NB - 2, k1 - 1) - k);
      window_barrier();
      if (k + NB - 1 < k1) issue_window(gbase, W, k + NB - 1, bufs[(j + NB - 1) % NB]);
    } else {
      window_barrier();  // window k landed; every compute wave is done with window k - 1's buffer
      uint8_t* buf = bufs[j % NB];
      const int32_t off = kPad - W.stage_lo(k);
#ifndef TKH_SPAN_PROBE_NO_BODY  // tools/probes/span_bench.hip builds variants without one stage
      body(k, buf, off);  // stores first: they drain while the CRC runs
#endif
#ifndef TKH_SPAN_PROBE_NO_CRC
      if (do_crc) crc = crc_piece(reinterpret_cast<const uint32_t*>(buf), nbase, W, k, off, c0, first, crc);
#endif
    }
  }
  return do_crc && !loader ? gf_mul(lane_k, crc) : 0u;
}

}  // namespace span
}  // namespace tkh
