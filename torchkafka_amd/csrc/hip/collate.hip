// CDNA4 (gfx950) collate kernels: the device half of the batch collate that
// the reference leaves to torch's CPU `default_collate`.
//
// Both kernels are HBM/L2-bandwidth-bound element-wise work; the design
// follows the memory-bound playbook of cdna_hip_programming.md:
//   * 64-wide waves, 256-thread blocks, 16-byte-per-lane global accesses
//     (Guideline 13) and grid-stride loops capped at ~2048 blocks (Guideline 11);
//   * conversions bit-exact with torch (dtypes.h), optional per-feature affine
//     normalisation fused into the same pass (no second read of the batch);
//   * variable-length pad, 4/8-byte sources: each lane loads its 8 elements
//     with dword-aligned global_load_dwordx4 (full width on gfx950 wherever a
//     CSR row starts), no LDS and no barrier;
//   * variable-length pad, 1/2-byte sources (row starts not dword-aligned):
//     the row chunk is staged through LDS with aligned 16-byte global loads
//     and read back through a padded layout (one dword after every lane's
//     8-element chunk): lane t reads dword (2*sizeof(S)+1)*t + c, an odd
//     stride, so each 32-lane read group hits 32 distinct banks
//     (MI355X_MICROARCH.md §LDS: ds_read_b32/u16/u8 bank = (a/4) mod 32).
#include <hip/hip_runtime.h>

#include "collate.h"

#include <algorithm>
#include <chrono>
#include <string>
#include <vector>
#include "convert.h"
#include "dtypes.h"

namespace tkh {

namespace {

constexpr int kThreads = 256;
constexpr int kEPT = 8;                   // elements per thread
constexpr int kChunk = kThreads * kEPT;   // var-len: output elements per block

// ---------------------------------------------------------------- fixed width
// dst[i] = conv(src[i]) over a dense [rows, D] block; vector path needs
// D % 8 == 0 and both pointers 16-byte aligned (checked on the host).
// Each thread owns U groups of kEPT elements per iteration, spaced kThreads groups
// apart so every wave access stays one contiguous 64-lane span; all U loads are
// issued before the first convert, so a wave keeps U x 16-32 B per lane in flight
// (a large stream needs that memory-level parallelism to approach HBM rate; small
// batches use U = 1 so they still spread over many CUs).
template <typename S, typename D, bool AFFINE, int U>
__global__ __launch_bounds__(kThreads) void fixed_vec_kernel(const S* __restrict__ src, D* __restrict__ dst,
                                                             int64_t n_groups, int64_t row, const float* __restrict__ shift,
                                                             const float* __restrict__ scale) {
  using C = Conv<S, D, IsIntDst<D>::value>;
  const int64_t tile = int64_t(kThreads) * U;
  const int64_t stride = int64_t(gridDim.x) * tile;
  for (int64_t base = int64_t(blockIdx.x) * tile + threadIdx.x; base < n_groups; base += stride) {
    Vec<S, kEPT> in[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t g = base + int64_t(u) * kThreads;
      if (g < n_groups) in[u] = *reinterpret_cast<const Vec<S, kEPT>*>(src + g * kEPT);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t g = base + int64_t(u) * kThreads;
      if (g >= n_groups) break;
      const int64_t e = g * kEPT;
      Vec<D, kEPT> out;
      if constexpr (AFFINE) {
        const int64_t d = e % row;
        const Vec<float, kEPT> sh = *reinterpret_cast<const Vec<float, kEPT>*>(shift + d);
        const Vec<float, kEPT> sc = *reinterpret_cast<const Vec<float, kEPT>*>(scale + d);
#pragma unroll
        for (int k = 0; k < kEPT; ++k) out.v[k] = C::apply(in[u].v[k], sh.v[k], sc.v[k], true);
      } else {
#pragma unroll
        for (int k = 0; k < kEPT; ++k) out.v[k] = C::apply(in[u].v[k], 0.f, 1.f, false);
      }
      *reinterpret_cast<Vec<D, kEPT>*>(dst + e) = out;
    }
  }
}

template <typename S, typename D, bool AFFINE>
__global__ __launch_bounds__(kThreads) void fixed_scalar_kernel(const S* __restrict__ src, D* __restrict__ dst,
                                                                int64_t n, int64_t row, const float* __restrict__ shift,
                                                                const float* __restrict__ scale) {
  using C = Conv<S, D, IsIntDst<D>::value>;
  const int64_t stride = int64_t(gridDim.x) * kThreads;
  for (int64_t i = int64_t(blockIdx.x) * kThreads + threadIdx.x; i < n; i += stride) {
    if constexpr (AFFINE) {
      const int64_t d = i % row;
      dst[i] = C::apply(src[i], shift[d], scale[d], true);
    } else {
      dst[i] = C::apply(src[i], 0.f, 1.f, false);
    }
  }
}

// ---------------------------------------------------------------- var-len pad
// Padded LDS byte address: one dword of padding after every lane chunk (kEPT elements,
// 8 * sizeof(S) bytes), so lane t's k-th ds_read lands on dword (2 * sizeof(S) + 1) * t + c:
// an odd stride, hence a different bank for each of the 32 lanes of a read group.
template <typename S>
__device__ __forceinline__ uint32_t lds_pad(uint32_t b) {
  constexpr uint32_t kLaneBytes = kEPT * sizeof(S);
  return b + (b / kLaneBytes) * 4;
}

template <typename S, typename D>
__global__ __launch_bounds__(kThreads) void varlen_pad_kernel(const int32_t* __restrict__ offs,
                                                              const uint8_t* __restrict__ vals, D* __restrict__ out,
                                                              int64_t L, D pad, int64_t* __restrict__ lengths,
                                                              uint8_t* __restrict__ mask, int vec_store_ok) {
  using C = Conv<S, D, IsIntDst<D>::value>;
  constexpr uint32_t kStageBytes = kChunk * sizeof(S) + 32;
  __shared__ __attribute__((aligned(16))) uint8_t lds[kStageBytes + (kStageBytes / (kEPT * sizeof(S)) + 1) * 4 + 16];

  const int64_t r = blockIdx.y;
  const int64_t c0 = int64_t(blockIdx.x) * kChunk;
  const int32_t beg = offs[r];
  const int64_t len = int64_t(offs[r + 1]) - beg;
  const int64_t nreal = len - c0 < 0 ? 0 : (len - c0 > kChunk ? kChunk : len - c0);

  uint32_t shift_b = 0;
  if (nreal > 0) {
    const uint64_t sb = (uint64_t(beg) + uint64_t(c0)) * sizeof(S);
    const uint64_t ab = sb & ~uint64_t(15);
    const uint64_t eb = (sb + uint64_t(nreal) * sizeof(S) + 15) & ~uint64_t(15);
    shift_b = uint32_t(sb - ab);
    const uint32_t nv = uint32_t((eb - ab) >> 4);
    for (uint32_t i = threadIdx.x; i < nv; i += kThreads) {
      const uint4 v = *reinterpret_cast<const uint4*>(vals + ab + (uint64_t(i) << 4));
      // the padded addresses are only 4-byte aligned and, for 1-byte sources, a pad
      // falls inside the 16 bytes: store each dword at its own padded address
      const uint32_t b = i << 4;
      *reinterpret_cast<uint32_t*>(lds + lds_pad<S>(b)) = v.x;
      *reinterpret_cast<uint32_t*>(lds + lds_pad<S>(b + 4)) = v.y;
      *reinterpret_cast<uint32_t*>(lds + lds_pad<S>(b + 8)) = v.z;
      *reinterpret_cast<uint32_t*>(lds + lds_pad<S>(b + 12)) = v.w;
    }
  }
  __syncthreads();

  const int64_t j0 = c0 + int64_t(threadIdx.x) * kEPT;
  if (j0 >= L) return;
  Vec<D, kEPT> o;
#pragma unroll
  for (int k = 0; k < kEPT; ++k) {
    const int64_t local = int64_t(threadIdx.x) * kEPT + k;
    if (local < nreal) {
      const S s = *reinterpret_cast<const S*>(lds + lds_pad<S>(shift_b + uint32_t(local) * sizeof(S)));
      o.v[k] = C::apply(s, 0.f, 1.f, false);
    } else {
      o.v[k] = pad;
    }
  }
  D* orow = out + r * L;
  if (vec_store_ok && j0 + kEPT <= L) {
    *reinterpret_cast<Vec<D, kEPT>*>(orow + j0) = o;
  } else {
#pragma unroll
    for (int k = 0; k < kEPT; ++k)
      if (j0 + k < L) orow[j0 + k] = o.v[k];
  }
  if (mask) {
    uint8_t* mrow = mask + r * L;
#pragma unroll
    for (int k = 0; k < kEPT; ++k)
      if (j0 + k < L) mrow[j0 + k] = uint8_t((j0 + k) < len);  // j < L already bounds len
  }
  if (lengths && blockIdx.x == 0 && threadIdx.x == 0) lengths[r] = len < L ? len : L;
}

int grid_for(int64_t work_items) {
  int64_t g = (work_items + kThreads - 1) / kThreads;
  if (g < 1) g = 1;
  if (g > 2048) g = 2048;
  return int(g);
}

template <typename S, typename D>
void launch_fixed_t(const void* src, void* dst, int64_t rows, int64_t row, const float* shift, const float* scale,
                    hipStream_t stream) {
  const int64_t n = rows * row;
  if (n == 0) return;
  const bool affine = shift != nullptr;
  const bool vec = (row % kEPT == 0) && (reinterpret_cast<uintptr_t>(src) % 16 == 0) &&
                   (reinterpret_cast<uintptr_t>(dst) % 16 == 0) &&
                   (!affine || (reinterpret_cast<uintptr_t>(shift) % 16 == 0 && reinterpret_cast<uintptr_t>(scale) % 16 == 0));
  if (vec) {
    const int64_t groups = n / kEPT;
    // U = 4 once there is at least one full 4-deep tile per CU (256 CUs); below that U = 1
    constexpr int64_t kBigGroups = int64_t(256) * kThreads * 4;
    const bool big = groups >= kBigGroups;
    const int grid = big ? grid_for((groups + 3) / 4) : grid_for(groups);
    const S* s = static_cast<const S*>(src);
    D* d = static_cast<D*>(dst);
    if (affine) {
      if (big)
        hipLaunchKernelGGL((fixed_vec_kernel<S, D, true, 4>), dim3(grid), dim3(kThreads), 0, stream, s, d, groups, row,
                           shift, scale);
      else
        hipLaunchKernelGGL((fixed_vec_kernel<S, D, true, 1>), dim3(grid), dim3(kThreads), 0, stream, s, d, groups, row,
                           shift, scale);
    } else {
      if (big)
        hipLaunchKernelGGL((fixed_vec_kernel<S, D, false, 4>), dim3(grid), dim3(kThreads), 0, stream, s, d, groups,
                           row, shift, scale);
      else
        hipLaunchKernelGGL((fixed_vec_kernel<S, D, false, 1>), dim3(grid), dim3(kThreads), 0, stream, s, d, groups,
                           row, shift, scale);
    }
  } else {
    const int grid = grid_for(n);
    if (affine)
      hipLaunchKernelGGL((fixed_scalar_kernel<S, D, true>), dim3(grid), dim3(kThreads), 0, stream,
                         static_cast<const S*>(src), static_cast<D*>(dst), n, row, shift, scale);
    else
      hipLaunchKernelGGL((fixed_scalar_kernel<S, D, false>), dim3(grid), dim3(kThreads), 0, stream,
                         static_cast<const S*>(src), static_cast<D*>(dst), n, row, shift, scale);
  }
}

// Coalesced launch: up to kMaxGroup ring slots (consecutive batches) collated by one
// kernel, block range [k * bps, (k + 1) * bps) serving slot k.  One launch replaces k
// (host: ~3-4 us of hipLaunchKernel + bookkeeping per batch), and in zero-copy mode
// k x 256 KiB of PCIe reads are in flight at once instead of 256 KiB: a 256 KiB
// zero-copy read is latency-bound at ~37 GB/s, 1 MiB reaches ~50 GB/s (measured,
// profiles/r01_s3_baseline/register_probe.log).
struct FixedGroupArgs {
  const void* src[kMaxGroup];
  void* dst[kMaxGroup];
  int64_t groups[kMaxGroup];  // kEPT-element groups of slot k
  int n;
  int bps;                    // blocks per slot
};

template <typename S, typename D, bool AFFINE>
__global__ __launch_bounds__(kThreads) void fixed_group_kernel(FixedGroupArgs a, int64_t row,
                                                               const float* __restrict__ shift,
                                                               const float* __restrict__ scale) {
  using C = Conv<S, D, IsIntDst<D>::value>;
  const int k = int(blockIdx.x) / a.bps;
  const int b = int(blockIdx.x) - k * a.bps;
  const S* __restrict__ src = static_cast<const S*>(a.src[k]);
  D* __restrict__ dst = static_cast<D*>(a.dst[k]);
  const int64_t n_groups = a.groups[k];
  const int64_t stride = int64_t(a.bps) * kThreads;
  for (int64_t g = int64_t(b) * kThreads + threadIdx.x; g < n_groups; g += stride) {
    const Vec<S, kEPT> in = *reinterpret_cast<const Vec<S, kEPT>*>(src + g * kEPT);
    const int64_t e = g * kEPT;
    Vec<D, kEPT> out;
    if constexpr (AFFINE) {
      const int64_t d = e % row;
      const Vec<float, kEPT> sh = *reinterpret_cast<const Vec<float, kEPT>*>(shift + d);
      const Vec<float, kEPT> sc = *reinterpret_cast<const Vec<float, kEPT>*>(scale + d);
#pragma unroll
      for (int j = 0; j < kEPT; ++j) out.v[j] = C::apply(in.v[j], sh.v[j], sc.v[j], true);
    } else {
#pragma unroll
      for (int j = 0; j < kEPT; ++j) out.v[j] = C::apply(in.v[j], 0.f, 1.f, false);
    }
    *reinterpret_cast<Vec<D, kEPT>*>(dst + e) = out;
  }
}

template <typename S, typename D>
void launch_fixed_group_t(const void* const* srcs, void* const* dsts, const int64_t* rows, int n, int64_t row,
                          const float* shift, const float* scale, hipStream_t stream, bool host_src) {
  const bool affine = shift != nullptr;
  bool vec = (row % kEPT == 0) &&
             (!affine || (reinterpret_cast<uintptr_t>(shift) % 16 == 0 && reinterpret_cast<uintptr_t>(scale) % 16 == 0));
  int64_t max_groups = 0;
  for (int k = 0; k < n && vec; ++k) {
    vec = reinterpret_cast<uintptr_t>(srcs[k]) % 16 == 0 && reinterpret_cast<uintptr_t>(dsts[k]) % 16 == 0;
    max_groups = std::max<int64_t>(max_groups, rows[k] * row / kEPT);
  }
  if (!vec || max_groups == 0) {  // unaligned or odd rows: one ordinary launch per slot
    for (int k = 0; k < n; ++k) launch_fixed_t<S, D>(srcs[k], dsts[k], rows[k], row, shift, scale, stream);
    (void)host_src;
    return;
  }
  FixedGroupArgs a{};
  a.n = n;
  for (int k = 0; k < n; ++k) {
    a.src[k] = srcs[k];
    a.dst[k] = dsts[k];
    a.groups[k] = rows[k] * row / kEPT;
  }
  // A zero-copy read is PCIe-latency-bound: ~16 blocks in total keep enough bytes in flight per
  // wave, more blocks only add request overhead (probe over k x 256 KiB slots, group_probe.log:
  // 4 slots 20.9 us at 4 blocks/slot vs 24.7 us at 32; 8 slots 39.4 vs 50.2 us).  HBM sources
  // (DMA staging) are not latency-bound and get one block per 256 groups.
  const int64_t full = std::max<int64_t>(1, std::min<int64_t>((max_groups + kThreads - 1) / kThreads, 2048 / n));
  a.bps = int(host_src ? std::min<int64_t>(full, std::max(4, 16 / n)) : full);
  const dim3 grid(unsigned(a.bps * n));
  if (affine)
    hipLaunchKernelGGL((fixed_group_kernel<S, D, true>), grid, dim3(kThreads), 0, stream, a, row, shift, scale);
  else
    hipLaunchKernelGGL((fixed_group_kernel<S, D, false>), grid, dim3(kThreads), 0, stream, a, row, shift, scale);
}

// ---------------------------------------------------------------- log gather (h2d="direct")
// Rows are gathered straight out of the broker's partition logs, pinned in place by the main
// process: the worker only wrote one uint64 per row, (pidx << 44) | byte offset of the value in
// that partition's log (consumer.h kPackGatherFixed).  Record values sit at arbitrary byte
// offsets (RecordBatch v2 varint headers precede them), so one wave per row:
//   * lane l loads the 16-byte-aligned chunk l of the row's span (one contiguous 1 KiB+ wave
//     access, coalesced into full PCIe reads), lane 63 also loads the chunk after it;
//   * the next lane's chunk comes over a lane shuffle (no second PCIe read of any byte);
//   * the misalignment s = 4q + r is wave-uniform: dword q selects the window, v_alignbyte_b32
//     shifts by r bytes, giving 16 aligned bytes per lane -> 16/sizeof(S) elements, converted
//     and stored (16 B per lane for f32 -> bf16 ... 8 B).
struct GatherGroupArgs {
  const uint64_t* ent[kMaxGroup];  // per slot: gather table (zero-copy view of the ring slot)
  void* dst[kMaxGroup];
  int32_t first[kMaxGroup + 1];    // prefix sum of rows: slot k owns global rows [first[k], first[k+1])
  int n;
};

__device__ __forceinline__ uint32_t shfl_down1(uint32_t v) {
  // lane l receives lane l+1's value (lane 63 gets its own; it loads its successor itself)
  const int lane = int(threadIdx.x & 63);
  const int src = lane == 63 ? lane : lane + 1;
  return uint32_t(__builtin_amdgcn_ds_bpermute(src << 2, int(v)));
}

template <typename S, typename D, bool AFFINE>
__global__ __launch_bounds__(kThreads) void gather_fixed_kernel(GatherGroupArgs a, const uint64_t* __restrict__ bases,
                                                                int64_t row_bytes, const float* __restrict__ shift,
                                                                const float* __restrict__ scale) {
  using C = Conv<S, D, IsIntDst<D>::value>;
  constexpr int kPer = 16 / int(sizeof(S));  // source elements per lane per segment
  const int lane = int(threadIdx.x & 63);
  const int64_t row_elems = row_bytes / int64_t(sizeof(S));
  const int64_t total = a.first[a.n];
  const int64_t waves = int64_t(gridDim.x) * (kThreads / 64);
  const bool vec_store = ((row_elems * int64_t(sizeof(D))) % (kPer * int64_t(sizeof(D)))) == 0;
  for (int64_t gr = int64_t(blockIdx.x) * (kThreads / 64) + (threadIdx.x >> 6); gr < total; gr += waves) {
    int k = 0;
    while (k + 1 < a.n && gr >= a.first[k + 1]) ++k;
    const int64_t r = gr - a.first[k];
    const uint64_t e = a.ent[k][r];
    const uint8_t* src = reinterpret_cast<const uint8_t*>(bases[e >> 44]) + (e & ((uint64_t(1) << 44) - 1));
    const uint32_t s = uint32_t(reinterpret_cast<uintptr_t>(src) & 15);
    const uint4* A = reinterpret_cast<const uint4*>(src - s);
    const uint32_t q = s >> 2, rb = s & 3;
    D* drow = static_cast<D*>(a.dst[k]) + r * row_elems;
    for (int64_t seg = 0; seg < row_bytes; seg += 1024) {
      const int64_t rem = row_bytes - seg;              // row bytes left from this segment on
      const int64_t need = int64_t(s) + rem;            // source bytes needed from A + seg on
      const uint4* Aseg = A + seg / 16;
      uint4 c = {0u, 0u, 0u, 0u};
      if (int64_t(lane) * 16 < need) c = Aseg[lane];
      uint4 nx;
      nx.x = shfl_down1(c.x);
      nx.y = shfl_down1(c.y);
      nx.z = shfl_down1(c.z);
      nx.w = shfl_down1(c.w);
      if (lane == 63) {
        nx = {0u, 0u, 0u, 0u};
        if (int64_t(64) * 16 < need) nx = Aseg[64];
      }
      const int64_t o = int64_t(lane) * 16;             // this lane's output bytes [o, o + 16) of the segment
      if (o >= rem) continue;
      const uint32_t w[8] = {c.x, c.y, c.z, c.w, nx.x, nx.y, nx.z, nx.w};
      uint32_t out4[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        // q is wave-uniform: the selects resolve to one path per row
        const uint32_t lo = q == 0 ? w[j] : q == 1 ? w[j + 1] : q == 2 ? w[j + 2] : w[j + 3];
        const uint32_t hi = q == 0 ? w[j + 1] : q == 1 ? w[j + 2] : q == 2 ? w[j + 3] : w[j + 4];
        out4[j] = __builtin_amdgcn_alignbyte(hi, lo, rb);
      }
      S sv[kPer];
      __builtin_memcpy(sv, out4, 16);
      const int64_t e0 = (seg + o) / int64_t(sizeof(S));  // first element of this lane in the row
      const int nel = rem - o >= 16 ? kPer : int((rem - o) / int64_t(sizeof(S)));
      Vec<D, kPer> ov;
#pragma unroll
      for (int j = 0; j < kPer; ++j) {
        if constexpr (AFFINE)
          ov.v[j] = C::apply(sv[j], j < nel ? shift[e0 + j] : 0.f, j < nel ? scale[e0 + j] : 1.f, true);
        else
          ov.v[j] = C::apply(sv[j], 0.f, 1.f, false);
      }
      if (nel == kPer && vec_store) {
        *reinterpret_cast<Vec<D, kPer>*>(drow + e0) = ov;
      } else {
        for (int j = 0; j < nel; ++j) drow[e0 + j] = ov.v[j];
      }
    }
  }
}

template <typename S, typename D>
void launch_gather_group_t(const uint64_t* const* ents, void* const* dsts, const int64_t* rows, int n,
                           const uint64_t* bases, int64_t row_bytes, const float* shift, const float* scale,
                           hipStream_t stream) {
  GatherGroupArgs a{};
  a.n = n;
  a.first[0] = 0;
  for (int k = 0; k < n; ++k) {
    a.ent[k] = ents[k];
    a.dst[k] = dsts[k];
    a.first[k + 1] = a.first[k] + int32_t(rows[k]);
  }
  const int64_t total = a.first[n];
  if (total == 0) return;
  constexpr int kWavesPerBlock = kThreads / 64;
  const int grid = int(std::min<int64_t>((total + kWavesPerBlock - 1) / kWavesPerBlock, 4096));
  if (shift)
    hipLaunchKernelGGL((gather_fixed_kernel<S, D, true>), dim3(grid), dim3(kThreads), 0, stream, a, bases, row_bytes,
                       shift, scale);
  else
    hipLaunchKernelGGL((gather_fixed_kernel<S, D, false>), dim3(grid), dim3(kThreads), 0, stream, a, bases,
                       row_bytes, shift, scale);
}

// Direct variant for 4- and 8-byte sources (f32 JSON values, i32/i64 token ids): a row's
// elements are dword-aligned wherever the row starts, and gfx950 serves dword-aligned
// global_load_dwordx4 at full width, so each lane loads its 8 elements straight from
// global memory (2-4 x 16 B, one contiguous span per wave) with no LDS round trip or
// barrier.  1- and 2-byte sources keep the LDS-staged kernel above (their row starts
// are not dword-aligned).
template <typename S>
struct alignas(4) LoadVec {  // 8 source elements with only dword alignment
  typedef S type __attribute__((ext_vector_type(8), aligned(4)));
};

template <typename S, typename D>
__global__ __launch_bounds__(kThreads) void varlen_direct_kernel(const int32_t* __restrict__ offs,
                                                                 const S* __restrict__ vals, D* __restrict__ out,
                                                                 int64_t L, D pad, int64_t* __restrict__ lengths,
                                                                 uint8_t* __restrict__ mask, int vec_store_ok) {
  static_assert(sizeof(S) >= 4, "direct var-len loads need dword-sized elements");
  using C = Conv<S, D, IsIntDst<D>::value>;
  const int64_t r = blockIdx.y;
  const int64_t j0 = int64_t(blockIdx.x) * kChunk + int64_t(threadIdx.x) * kEPT;
  const int32_t beg = offs[r];
  const int64_t len = int64_t(offs[r + 1]) - beg;
  if (lengths && blockIdx.x == 0 && threadIdx.x == 0) lengths[r] = len < L ? len : L;
  if (j0 >= L) return;
  const S* row = vals + beg;
  D* orow = out + r * L;
  if (j0 + kEPT <= len && vec_store_ok) {
    // interior of a row (len <= L so j0 + 8 <= L too): load, convert in pairs, one 16 B store
    const typename LoadVec<S>::type v = *reinterpret_cast<const typename LoadVec<S>::type*>(row + j0);
    Vec<D, kEPT> o;
#pragma unroll
    for (int k = 0; k < kEPT; ++k) o.v[k] = C::apply(v[k], 0.f, 1.f, false);
    *reinterpret_cast<Vec<D, kEPT>*>(orow + j0) = o;
  } else if (j0 >= len && vec_store_ok && j0 + kEPT <= L) {
    // all padding (typically half of a batch padded to its longest row): one vector store
    Vec<D, kEPT> o;
#pragma unroll
    for (int k = 0; k < kEPT; ++k) o.v[k] = pad;
    *reinterpret_cast<Vec<D, kEPT>*>(orow + j0) = o;
  } else {
#pragma unroll
    for (int k = 0; k < kEPT; ++k)
      if (j0 + k < L) orow[j0 + k] = (j0 + k < len) ? C::apply(row[j0 + k], 0.f, 1.f, false) : pad;
  }
  if (mask) {
    uint8_t* mrow = mask + r * L;
#pragma unroll
    for (int k = 0; k < kEPT; ++k)
      if (j0 + k < L) mrow[j0 + k] = uint8_t((j0 + k) < len);
  }
}

template <typename S, typename D>
void launch_varlen_t(const int32_t* offs, const void* vals, void* out, int64_t rows, int64_t L, double pad,
                     int64_t* lengths, uint8_t* mask, hipStream_t stream) {
  if (rows == 0 || L == 0) {
    return;
  }
  if (rows > 65535) throw std::runtime_error("varlen collate: more than 65535 rows per batch");
  D padv;
  if constexpr (IsIntDst<D>::value) padv = D(int64_t(pad)); else padv = Store<D>::cvt(float(pad));
  const int vec_ok = (L % kEPT == 0) && (reinterpret_cast<uintptr_t>(out) % 16 == 0);
  dim3 grid(unsigned((L + kChunk - 1) / kChunk), unsigned(rows));
  if constexpr (sizeof(S) >= 4) {
    hipLaunchKernelGGL((varlen_direct_kernel<S, D>), grid, dim3(kThreads), 0, stream, offs,
                       static_cast<const S*>(vals), static_cast<D*>(out), L, padv, lengths, mask, vec_ok);
  } else {
    hipLaunchKernelGGL((varlen_pad_kernel<S, D>), grid, dim3(kThreads), 0, stream, offs,
                       static_cast<const uint8_t*>(vals), static_cast<D*>(out), L, padv, lengths, mask, vec_ok);
  }
}


}  // namespace

void launch_fixed(const void* src, int src_dt, void* dst, int dst_dt, int64_t rows, int64_t row, const float* shift,
                  const float* scale, hipStream_t stream) {
  if (!is_float_dt(dst_dt) && is_float_dt(src_dt))
    throw std::invalid_argument("collate: float records cannot be cast to an integer dtype");
  if (shift && !is_float_dt(dst_dt)) throw std::invalid_argument("collate: normalisation needs a float dtype");
  TK_DISPATCH_SRC(launch_fixed_t, src, dst, rows, row, shift, scale, stream)
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw std::runtime_error(std::string("fixed collate launch: ") + hipGetErrorString(e));
}

void launch_varlen(const int32_t* offs, const void* vals, int src_dt, void* out, int dst_dt, int64_t rows, int64_t L,
                   double pad, int64_t* lengths, uint8_t* mask, hipStream_t stream) {
  if (!is_float_dt(dst_dt) && is_float_dt(src_dt))
    throw std::invalid_argument("collate: float records cannot be cast to an integer dtype");
  if (reinterpret_cast<uintptr_t>(vals) % 16) throw std::invalid_argument("varlen collate: values must be 16B aligned");
  TK_DISPATCH_SRC(launch_varlen_t, offs, vals, out, rows, L, pad, lengths, mask, stream)
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw std::runtime_error(std::string("varlen collate launch: ") + hipGetErrorString(e));
}

void launch_fixed_group(const void* const* srcs, int src_dt, void* const* dsts, int dst_dt, const int64_t* rows, int n,
                        int64_t row, const float* shift, const float* scale, hipStream_t stream, bool host_src) {
  if (n < 1 || n > kMaxGroup) throw std::invalid_argument("collate: group size out of range");
  if (!is_float_dt(dst_dt) && is_float_dt(src_dt))
    throw std::invalid_argument("collate: float records cannot be cast to an integer dtype");
  if (shift && !is_float_dt(dst_dt)) throw std::invalid_argument("collate: normalisation needs a float dtype");
  TK_DISPATCH_SRC(launch_fixed_group_t, srcs, dsts, rows, n, row, shift, scale, stream, host_src)
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw std::runtime_error(std::string("fixed group collate launch: ") + hipGetErrorString(e));
}

void launch_gather_group(const uint64_t* const* ents, int src_dt, void* const* dsts, int dst_dt, const int64_t* rows,
                         int n, const uint64_t* bases, int64_t row_bytes, const float* shift, const float* scale,
                         hipStream_t stream) {
  if (n < 1 || n > kMaxGroup) throw std::invalid_argument("collate: group size out of range");
  if (!is_float_dt(dst_dt) && is_float_dt(src_dt))
    throw std::invalid_argument("collate: float records cannot be cast to an integer dtype");
  if (shift && !is_float_dt(dst_dt)) throw std::invalid_argument("collate: normalisation needs a float dtype");
  int64_t total = 0;
  for (int k = 0; k < n; ++k) total += rows[k];
  if (total > INT32_MAX) throw std::invalid_argument("gather collate: too many rows");
  TK_DISPATCH_SRC(launch_gather_group_t, ents, dsts, rows, n, bases, row_bytes, shift, scale, stream)
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw std::runtime_error(std::string("gather collate launch: ") + hipGetErrorString(e));
}

__global__ void empty_kernel() {}

// Host cost (ns per call, averaged over `iters`) of the HIP calls on the per-batch path.
std::vector<std::pair<std::string, double>> api_bench(int device, int iters) {
  std::vector<std::pair<std::string, double>> out;
  hipSetDevice(device);
  hipStream_t st;
  hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
  hipEvent_t ev;
  hipEventCreateWithFlags(&ev, hipEventDisableTiming);
  void* d = nullptr;
  void* h = nullptr;
  hipMalloc(&d, 1 << 20);
  hipHostMalloc(&h, 1 << 20, hipHostMallocDefault);
  auto now = [] { return std::chrono::steady_clock::now(); };
  auto time_it = [&](const char* name, auto&& fn) {
    hipStreamSynchronize(st);
    auto t0 = now();
    for (int i = 0; i < iters; ++i) fn(i);
    auto t1 = now();
    hipStreamSynchronize(st);
    out.emplace_back(name, std::chrono::duration<double, std::nano>(t1 - t0).count() / iters);
  };
  time_it("hipLaunchKernel(empty)", [&](int) { hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, st); });
  time_it("hipEventRecord", [&](int) { hipEventRecord(ev, st); });
  time_it("hipEventQuery", [&](int) { (void)hipEventQuery(ev); });
  time_it("hipStreamWaitEvent", [&](int) { hipStreamWaitEvent(st, ev, 0); });
  time_it("hipMemcpyAsync(4KiB pinned H2D)", [&](int) { hipMemcpyAsync(d, h, 4096, hipMemcpyHostToDevice, st); });
  time_it("hipMemcpyAsync(256KiB pinned H2D)", [&](int) { hipMemcpyAsync(d, h, 262144, hipMemcpyHostToDevice, st); });
  time_it("hipGetLastError", [&](int) { (void)hipGetLastError(); });
  time_it("launch_fixed(256x256 f32->bf16)", [&](int) {
    launch_fixed(h, kF32, d, kBF16, 256, 256, nullptr, nullptr, st);
  });
  hipStreamSynchronize(st);
  hipFree(d);
  hipHostFree(h);
  hipEventDestroy(ev);
  hipStreamDestroy(st);
  return out;
}

}  // namespace tkh
