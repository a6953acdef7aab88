// gfx950 JSON-array parse + pad/stack + cast: the device half of the JsonArray
// schema's "device parse" mode (the reference's README decodes
// each record with `json.loads(record.value)` in Python, README.md:54,74).
//
// The worker no longer parses numbers.  It only frames each record
// (Fetcher::fill_slot, kPackJsonText): an AVX2 pre-scan counts the elements
// and checks the row is "simple" (numbers made of [0-9.-] only, every token at
// most 16 characters), then copies the raw text into the pinned slot.  Rows
// that are not simple (exponents, NaN/Infinity, long tokens, anything odd) are
// parsed on the host as before and ride in the same slot as float32.
//
// One 256-thread block (4 waves) owns one row.  The row's text goes through
// LDS in 2 KiB windows (one 16-byte load per thread), then:
//   1. token starts: thread t classifies its 8 contiguous bytes in registers
//      -> an 8-bit start mask; a block-wide exclusive scan of the popcounts
//      (wave shuffles + per-wave totals) gives every token its index, and its
//      window-relative start goes to an LDS table;
//   2. parse: thread t parses tokens t, t+256, ... (one per thread for a
//      typical window) from registers loaded off LDS with the host
//      parser's grammar and arithmetic (Clinger's fast path in fp64: both
//      operands exact, one correctly rounded IEEE op; u64 -> f64 for plain
//      integers), then f64 -> f32 -> destination dtype, bit-exact with
//      Python float() + torch's casts; consecutive lanes store consecutive
//      columns (coalesced);
//   3. a token cut by the window end restarts the next window (16-byte
//      aligned at or below its start).
// Grammar errors (e.g. "1..2", "[1,,2]": they pass the worker's character
// scan) write the row index into a host-mapped error word; the step driver
// checks it before the batch is committed and raises CorruptRecordException.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <stdexcept>
#include <string>

#include "collate.h"
#include "dtypes.h"
#include "json_scan_dev.h"
#include "json_token.h"
#include "span.h"

namespace tkh {

namespace {

constexpr int kWave = 64;
constexpr int kThreads = 256;                 // one block (4 waves) per row
constexpr int kWaves = kThreads / kWave;
constexpr int kWin = 2048;                    // bytes of text per window (one 8-byte slice per thread)
constexpr int kLaneBytes = kWin / kThreads;   // 8 contiguous bytes classified per thread
constexpr int kMaxTok = kWin / 2 + 1;         // a token needs >= 1 char and 1 separator
// fused count: the byte classes of a row (json_scan_simple's rules), OR-ed over its windows
constexpr int kClsOther = 1;     // a byte that is not [0-9.-], ',' or whitespace
constexpr int kClsNumber = 2;    // a number character
constexpr int kClsAny = 4;       // anything but whitespace
constexpr int kClsLong = 8;      // a token that does not end within 17 bytes
constexpr int kClsUnframed = 16;  // the text is not '[' ... ']' at its very ends

template <typename D>
__device__ __forceinline__ D pad_value(float p) { return Store<D>::cvt(p); }

// Blocks [row_base[k], row_base[k+1]) parse batch k: one launch serves up to kMaxGroup
// staged batches (the driver's coalesced launches), each with its own slot, output and L.
template <typename D>
__global__ __launch_bounds__(kThreads) void json_rows_kernel(JsonGroupArgs a) {
  __shared__ __attribute__((aligned(16))) uint8_t buf[kWin + 32];  // + the 32-byte token reads
  // one dword per token start: 16-bit entries put two lanes' stores on one dword, which the LDS
  // serialises (46 % of this kernel's LDS cycles were bank conflicts with uint16_t, r04_s10)
  __shared__ uint32_t starts[kMaxTok];
  __shared__ int s_wsum[kWaves];
  __shared__ int s_cut, s_bad;
  __shared__ int32_t s_count, s_guess;
  __shared__ int32_t s_commas, s_cls;  // fused count: the row's commas and byte classes (kCls*)
  __shared__ bool s_host;              // fused count: this block's row is left to the host (thread 0's)

  int bk = 0;
#pragma unroll
  for (int k = 1; k < kMaxGroup; ++k) bk += (k < a.n && int64_t(blockIdx.x) >= a.row_base[k]) ? 1 : 0;
  const int64_t r = int64_t(blockIdx.x) - a.row_base[bk];
  const JsonRowDesc* __restrict__ rows = a.rows[bk];
  const uint8_t* __restrict__ vals = a.vals[bk];
  D* __restrict__ out = static_cast<D*>(a.out[bk]);
  int64_t L = a.L[bk];
  const bool fused = a.ctr[bk] && a.fused_count;
  if (a.ctr[bk] && !fused) {
    // device-counted batch: its width is the longest kept row (rounded up to the pad multiple),
    // within the capacity the host allocated; the first block reports it (and the rows left to
    // the host) through the host-mapped info words
    const unsigned long long c0 = a.ctr[bk][0], c1 = a.ctr[bk][1];
    const uint32_t tag = a.ctr_tag[bk];
    if (a.mult > 0) {  // 0: the allocated width stays (pad_to)
      int64_t w = uint32_t(c0 >> 32) == tag ? int64_t(uint32_t(c0)) : 0;  // no row counted: 0
      if (a.mult > 1) w = (w + a.mult - 1) / a.mult * a.mult;
      if (w < L) L = w;
    }
    if (int64_t(blockIdx.x) == a.row_base[bk] && threadIdx.x == 0 && a.info[bk]) {
      volatile int32_t* info = a.info[bk];
      info[0] = int32_t(L);
      info[1] = uint32_t(c1 >> 32) == tag ? 1 : 0;
      __threadfence_system();
      info[2] = 1;
    }
  }
  const float pad = a.pad;
  int64_t* __restrict__ lengths = a.lengths[bk];
  uint8_t* __restrict__ mask = a.mask[bk];
  int32_t* __restrict__ err = a.err[bk];
  const int tid = threadIdx.x, lane = tid & (kWave - 1), wid = tid / kWave;
  if (tid == 0) s_host = false;
  JsonRowDesc d = rows[r];
  // A fixed width (pad_to) and a device-counted row: this block counts the row while it parses it
  // -- json_count_kernel's work without its launch and its pass over the text.  The windows below
  // classify every byte by json_scan_simple's rules (commas, bytes outside [0-9.-] / ',' /
  // whitespace, '[' and ']' at the text's ends, runs of more than 16 number characters: the parse
  // reports a token that does not end within 17 bytes); values are written up to the width (or
  // the truncation) and the row's count, verdict and length are settled after its last window.
  const int32_t tr = a.trunc[bk];
  const bool intg = fused && d.count == tk::kJsonCountOnDevice && d.tlen >= 0 &&
                    uint64_t(d.off) + ((uint64_t(d.tlen) + 15u) & ~uint64_t(15)) <= a.vals_cap[bk];
  if (intg) {
    const int64_t lim = tr >= 0 && int64_t(tr) < L ? int64_t(tr) : L;
    d = JsonRowDesc{d.off, d.tlen, INT32_MAX, int32_t(lim)};
    if (tid == 0) {
      s_commas = 0;
      s_cls = d.tlen < 2 ? kClsUnframed : 0;
    }
  }
  bool bad = false;  // block-uniform: only read after a barrier
  if (a.vals_cap[bk] > 0) {
    // staged by json_stage_kernel: a descriptor must stay inside the batch's staging area
    const uint64_t need = d.tlen >= 0                     ? uint64_t(d.tlen)
                          : d.tlen == tk::kJsonCountOnDevice ? 0u
                                                             : uint64_t(d.n_out < 0 ? 0 : d.n_out) * 4u;
    if (d.count < 0 || d.n_out < 0 || d.n_out > d.count || uint64_t(d.off) + ((need + 15u) & ~uint64_t(15)) > a.vals_cap[bk]) {
      bad = true;
      d = JsonRowDesc{0, 0, 0, 0};
    }
  }
  int64_t n_out = d.n_out < L ? d.n_out : L;
  D* orow = out + r * L;
  int64_t pad_from = n_out;

  if (d.tlen == tk::kJsonCountOnDevice) {
    pad_from = 0;  // not a simple row: the host writes its values when the batch is delivered
  } else if (d.tlen < 0) {
    // parsed on the host (not a simple row): float32 values
    const float* f = reinterpret_cast<const float*>(vals + d.off);
    for (int64_t k = tid; k < n_out; k += kThreads) orow[k] = Store<D>::cvt(f[k]);
  } else {
    const uint8_t* text = vals + d.off;  // 32-byte aligned (worker)
    const int T = d.tlen;
    int pend = 0;    // tokens starting before pend are done; text[pend-1] is a separator or pend starts a token
    int64_t k0 = 0;  // index of the first token of this window
    int seen = 0;    // intg: bytes before `seen` were classified by an earlier window
    bool long_tok = false;
    if (tid == 0) s_bad = 0;
    while (pend < T) {
      const int base = pend & ~15;
      const int wlen = T - base < kWin ? T - base : kWin;
      const bool last = base + wlen >= T;
      // stage the window: one 16-byte load per thread for the first 128 threads
      if (tid * 16 < wlen)
        *reinterpret_cast<uint4*>(buf + tid * 16) = *reinterpret_cast<const uint4*>(text + base + tid * 16);
      if (tid == 0) s_cut = kMaxTok;
      __syncthreads();
      // 1. token starts in this thread's 8 bytes, classified in registers.  A byte is a number
      // character iff it lies in '-'..'9' (0x2D-0x39); simple rows hold nothing else but
      // separators, and anything odd fails the parse below.
      const int b0 = tid * kLaneBytes;
      const uint2 cw = *reinterpret_cast<const uint2*>(buf + b0);
      uint32_t tokm = 0;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const uint32_t c = ((j < 4 ? cw.x : cw.y) >> ((j & 3) * 8)) & 0xFFu;
        tokm |= uint32_t(c - 0x2Du <= 0x0Cu) << j;
      }
      const int lim = wlen - b0;  // valid bytes of this thread (may be <= 0 or > 8)
      if (lim < 8) tokm &= lim <= 0 ? 0u : ((1u << lim) - 1u);
      if (intg) {  // block-uniform: the wave reductions below need every lane
        // json_scan_simple's classes of the interior bytes this window is the first to see
        uint32_t com = 0, oth = 0, num = 0;
        bool unframed = false;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const uint32_t c = ((j < 4 ? cw.x : cw.y) >> ((j & 3) * 8)) & 0xFFu;
          const int pos = base + b0 + j;
          const bool fresh = j < lim && pos >= seen;
          const bool in = fresh && pos > 0 && pos < T - 1;
          const bool isnum = c - 48u <= 9u || c == 46u || c == 45u;
          com |= uint32_t(in && c == 44u) << j;
          oth |= uint32_t(in && !isnum && c != 44u && !json_is_ws(c)) << j;
          num |= uint32_t(in && isnum) << j;
          unframed = unframed || (fresh && ((pos == 0 && c != '[') || (pos == T - 1 && c != ']')));
        }
        // one LDS atomic per wave (a per-lane atomic on one address serialises: 38 us per group
        // against 17 us, profiles/r06_s12)
        int nc = __popc(com);
#pragma unroll
        for (int o = 32; o; o >>= 1) nc += __shfl_xor(nc, o, kWave);
        const int cls = (__ballot(oth != 0) ? kClsOther : 0) | (__ballot(num != 0) ? kClsNumber : 0) |
                        (__ballot((com | oth | num) != 0) ? kClsAny : 0) | (__ballot(unframed) ? kClsUnframed : 0);
        if (lane == 0) {
          if (nc) atomicAdd(&s_commas, nc);
          if (cls) atomicOr(&s_cls, cls);
        }
      }
      // the byte before this thread's 8: the last byte of the previous lane's (a shuffle, not a
      // byte read at an 8-byte lane stride, which is a 2-way bank conflict); lane 0 reads it
      const uint32_t pw = __shfl_up(cw.y, 1, kWave) >> 24;
      const uint32_t pc = b0 > 0 && b0 <= wlen ? (lane == 0 ? uint32_t(buf[b0 - 1]) : pw) : uint32_t(',');
      const uint32_t prev_tok = uint32_t(pc - 0x2Du <= 0x0Cu);
      uint32_t m = tokm & ~((tokm << 1) | prev_tok);
      // only tokens at or after pend (pend itself starts a token when it is a number character)
      const int rel = pend - base - b0;  // pend relative to this thread's first byte
      if (rel > 0) {
        m &= rel >= 8 ? 0u : ~((1u << rel) - 1u);
        if (rel < 8) m |= tokm & (1u << rel);
      } else if (rel == 0) {
        m |= tokm & 1u;
      }
      // block-wide exclusive scan of the start counts: wave scan + per-wave totals
      const int cnt = __popc(m);
      int incl = cnt;
#pragma unroll
      for (int o = 1; o < kWave; o <<= 1) {
        const int t = __shfl_up(incl, o, kWave);
        if (lane >= o) incl += t;
      }
      if (lane == kWave - 1) s_wsum[wid] = incl;
      __syncthreads();
      int woff = 0, total = 0;
#pragma unroll
      for (int w = 0; w < kWaves; ++w) {
        const int ws = s_wsum[w];
        woff += w < wid ? ws : 0;
        total += ws;
      }
      int idx = woff + incl - cnt;
      while (m) {
        const int j = __ffs(m) - 1;
        m &= m - 1;
        starts[idx++] = uint32_t(b0 + j);
      }
      __syncthreads();
      // 2. parse; only the window's last token can be cut
      bool lbad = false, llong = false;
      for (int t = tid; t < total; t += kThreads) {
        float v;
        const int st0 = starts[t];
        const int rc = parse_token_regs(buf, st0, wlen - st0, last, &v);
        if (rc == 2) {
          s_cut = t;
        } else {
          if (rc != 1) {
            lbad = true;
            llong = llong || rc == 3;
            v = __builtin_nanf("");
          }
          const int64_t k = k0 + t;
          if (k < n_out) orow[k] = Store<D>::cvt(v);
        }
      }
      if (lbad) s_bad = 1;
      if (intg && llong) atomicOr(&s_cls, kClsLong);
      __syncthreads();
      seen = base + wlen;
      const int cut = s_cut;
      if (cut < total) {
        if (base + int(starts[cut]) == pend) {  // one token longer than a window: no progress possible
          bad = !intg;  // intg: a run of > 16 number characters, the host's row
          long_tok = true;
          break;
        }
        k0 += cut;
        pend = base + starts[cut];
      } else {
        k0 += total;
        pend = base + wlen;
      }
      __syncthreads();  // buf/starts/s_wsum are rewritten by the next window
    }
    if (intg) {
      __syncthreads();  // the classes of every window
      const int cls = s_cls;
      const int32_t commas = s_commas;
      bool simple;
      int32_t count, guess;
      if (cls & kClsUnframed) {
        // not '[' ... ']' at the very ends (whitespace around them, or no framing at all): the
        // wave-0 scan of the staged text decides (json_scan_simple's trimming), as json_count_kernel
        if (wid == 0) {
          int32_t g = 0;
          const int32_t c = json_scan_row([&](int32_t o) { return *reinterpret_cast<const uint4*>(text + o); },
                                          [&](int32_t i) { return uint32_t(text[i]); }, T, lane, &g);
          if (lane == 0) {
            s_count = c;
            s_guess = g;
          }
        }
        __syncthreads();
        count = s_count;
        guess = s_guess;
        simple = count >= 0;
      } else {
        simple = !(cls & (kClsOther | kClsLong)) && !long_tok && ((cls & kClsNumber) || commas == 0);
        count = (cls & kClsNumber) ? commas + 1 : 0;
        guess = (cls & kClsAny) ? commas + 1 : 0;
      }
      if (simple) {
        bad = bad || s_bad != 0 || k0 != count;
        n_out = tr >= 0 && count > tr ? tr : count;
      } else {
        // not simple: the host parses the row at delivery; its padding, lengths and mask here
        bad = false;
        n_out = tr >= 0 && guess > tr ? tr : guess;
        pad_from = 0;
        if (tid == 0) s_host = true;
      }
      if (n_out > L) n_out = L;
      if (simple) pad_from = n_out;
    } else {
      bad = bad || s_bad != 0 || k0 != d.count;
    }
  }
  // padding, lengths, mask
  for (int64_t k = pad_from + tid; k < L; k += kThreads) orow[k] = pad_value<D>(pad);
  if (mask) {
    uint8_t* mrow = mask + r * L;
    for (int64_t k = tid; k < L; k += kThreads) mrow[k] = uint8_t(k < n_out);
  }
  if (lengths && tid == 0) lengths[r] = n_out;
  if (err && bad && tid == 0 && (a.err_tag == 0 || *err < 0)) *err = a.err_tag | int32_t(r);
  if (fused && tid == 0 && s_host && a.info[bk]) {
    // a row left to the host: the batch's "rows left to the host" word (host-mapped; rare).  The
    // width and the done flag come from json_report_kernel once every block finished -- a done
    // counter per block was one device-scope atomic on one address per row, serialised at memory:
    // 28.8 us per group against 17.1 us without it (profiles/r06_s12)
    a.info[bk][1] = 1;
    __threadfence_system();
  }
}

template <typename D>
void launch_json_t(const JsonGroupArgs& a, int64_t total_rows, hipStream_t stream) {
  hipLaunchKernelGGL((json_rows_kernel<D>), dim3(unsigned(total_rows)), dim3(kThreads), 0, stream, a);
}

// After a fused-count parse launch, on its stream: each device-counted batch's {width, -, done}
// (the parse blocks raised "rows left to the host" themselves).  One wave, a lane per batch.
__global__ void json_report_kernel(JsonGroupArgs a) {
  const int k = int(threadIdx.x);
  if (k >= a.n || !a.ctr[k] || !a.info[k]) return;
  volatile int32_t* info = a.info[k];
  info[0] = int32_t(a.L[k]);
  __threadfence_system();
  info[2] = 1;
}

void launch_json_args(JsonGroupArgs& a, int dst_dt, hipStream_t stream) {
  if (a.n < 1 || a.n > kMaxGroup) throw std::invalid_argument("json collate: group size out of range");
  const int64_t total = a.row_base[a.n];
  if (total == 0) return;
  if (total > INT32_MAX) throw std::invalid_argument("json collate: too many rows");
  for (int k = 0; k < a.n; ++k)
    if (reinterpret_cast<uintptr_t>(a.vals[k]) % 16 || reinterpret_cast<uintptr_t>(a.rows[k]) % 16)
      throw std::invalid_argument("json collate: slot regions must be 16-byte aligned");
  switch (dst_dt) {
    case kF32: launch_json_t<float>(a, total, stream); break;
    case kF16: launch_json_t<_Float16>(a, total, stream); break;
    case kBF16: launch_json_t<__bf16>(a, total, stream); break;
    case kFP8E4M3: launch_json_t<fp8e4m3>(a, total, stream); break;
    default: throw std::invalid_argument("json collate: destination must be a float dtype");
  }
  if (a.fused_count) hipLaunchKernelGGL(json_report_kernel, dim3(1), dim3(64), 0, stream, a);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) throw std::runtime_error(std::string("json collate launch: ") + hipGetErrorString(e));
}

}  // namespace

void launch_json_rows(const JsonRowDesc* rows, const void* vals, void* out, int dst_dt, int64_t n_rows, int64_t L,
                      double pad, int64_t* lengths, uint8_t* mask, int32_t* err, hipStream_t stream) {
  JsonGroupArgs a{};
  a.n = 1;
  a.row_base[1] = n_rows;
  a.rows[0] = rows;
  a.vals[0] = static_cast<const uint8_t*>(vals);
  a.out[0] = out;
  a.L[0] = L;
  a.lengths[0] = lengths;
  a.mask[0] = mask;
  a.err[0] = err;
  a.pad = float(pad);
  launch_json_args(a, dst_dt, stream);
}

void launch_json_group(JsonGroupArgs& a, int dst_dt, hipStream_t stream) { launch_json_args(a, dst_dt, stream); }

}  // namespace tkh
