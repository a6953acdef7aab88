// H2D engine: pinned-ring registration, side-stream copies, collate launches.
//
// DMA mode (default): when a slot is acquired -- `prefetch` batches before
// the user asks for it -- its payload is copied by hipMemcpyAsync into
// staging[s] on copy stream streams[s % J] and copied[s] is recorded there.
// Slots on different copy streams use different SDMA queues, so copies run
// concurrently (one stream alone measured ~12 us per 256 KiB on MI355X).
// When the batch is handed out, the user's stream waits on copied[s], the
// collate kernel runs on the user's stream (ordered after the user's prior
// work, so a recycled output block is never overwritten early) and done[s]
// is recorded.  The host slot is released once done[s] completed; a staging
// buffer is therefore only rewritten after its previous kernel has run.
//
// Zero-copy mode: no copy; the kernel reads the pinned slot directly through
// its device mapping (hipHostRegisterMapped) over PCIe.
//
// Per batch the host issues memcpyAsync + eventRecord (prefetch) and
// streamWaitEvent + launch + eventRecord (hand-out); zero-copy mode only the
// last two.  No allocation, no synchronisation (Guideline 9).
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <stdexcept>
#include <string>
#include <vector>

#include "collate.h"
#include "crc32c.h"
#include "engine.h"
#include "hip_queue.h"
#include "reaper.h"
#include "span_decode.h"

namespace tkh {

#define TKH_CHECK(expr)                                                                       \
  do {                                                                                        \
    hipError_t _e = (expr);                                                                   \
    if (_e != hipSuccess) throw std::runtime_error(std::string(#expr) + ": " + hipGetErrorString(_e)); \
  } while (0)

Engine::Engine(int device, int n_slots, size_t staging_bytes, int n_streams, int mode)
    : device_(device), n_slots_(n_slots), mode_(mode), q_(std::make_unique<HipQueue>(device)) {
  if (const char* e = std::getenv("TORCHKAFKA_SPAN_PARTS")) {
    const int p = std::atoi(e);
    span_parts_ = p == 2 || p == 4 || p == tk::kSpanMaxParts ? p : 1;
  }
  json_parts_ = std::getenv("TORCHKAFKA_SPAN_PARTS") ? span_parts_ : 1;
  if (n_slots <= 0) throw std::invalid_argument("engine: n_slots must be positive");
  if (mode != kH2DDma && mode != kH2DZeroCopy) throw std::invalid_argument("engine: bad h2d mode");
  if (n_streams < 1) n_streams = 1;
  if (n_streams > n_slots) n_streams = n_slots;
  // Zero-copy mode issues no copies: no copy streams.  Every stream takes one of the process's
  // few hardware queues (GPU_MAX_HW_QUEUES, 4 by default) round-robin, and idle ones would push
  // the decode streams onto a shared queue, serialising the launches they exist to overlap.
  if (mode == kH2DZeroCopy) n_streams = 0;
  TKH_CHECK(hipSetDevice(device_));
  streams_.resize(size_t(n_streams));
  for (auto& st : streams_) TKH_CHECK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  stride_ = (staging_bytes + 256 + 4095) / 4096 * 4096;
  if (mode_ == kH2DDma) TKH_CHECK(hipMalloc(&staging_, stride_ * size_t(n_slots)));
  done_.resize(size_t(n_slots));
  for (auto& e : done_) TKH_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  done_seq_.assign(size_t(n_slots), 0);
  copied_.resize(size_t(n_slots));
  for (auto& e : copied_) TKH_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  host_src_.assign(size_t(n_slots), nullptr);
}

Engine::~Engine() {
  try {
    queue().drain();  // queued calls use the streams and events below
  } catch (...) {
  }
  hipSetDevice(device_);
  for (auto st : streams_) hipStreamSynchronize(st);
  if (host_ptr_) {  // registered by the user, never released: deferred like the rest (reaper.h)
    void* p = host_ptr_;
    Reaper::post(device_, [p] { (void)hipHostUnregister(p); });
  }
  for (auto e : done_) hipEventDestroy(e);
  for (auto e : copied_) hipEventDestroy(e);
  Reaper::free_device(device_, staging_);
  Reaper::free_device(device_, span_tabs_);
  for (auto& pa : part_acc_) Reaper::free_device(device_, pa.words);
  for (auto st : decode_streams_)
    if (st) {
      hipStreamSynchronize(st);
      hipStreamDestroy(st);
    }
  for (auto e : order_events_) hipEventDestroy(e);
  for (auto st : streams_) hipStreamDestroy(st);
}

void Engine::check_slot(int s) const {
  if (s < 0 || s >= n_slots_) throw std::out_of_range("engine: bad slot");
}

void Engine::register_host(void* p, size_t len) {
  if (host_ptr_) throw std::runtime_error("engine: a host region is already registered");
  TKH_CHECK(hipSetDevice(device_));
  TKH_CHECK(hipHostRegister(p, len, hipHostRegisterMapped));
  void* dev = nullptr;
  TKH_CHECK(hipHostGetDevicePointer(&dev, p, 0));
  host_ptr_ = p;
  host_dev_ = static_cast<uint8_t*>(dev);
  host_len_ = len;
}

void Engine::unregister_host() {
  if (!host_ptr_) return;
  synchronize();
  TKH_CHECK(hipHostUnregister(host_ptr_));
  host_ptr_ = nullptr;
  host_dev_ = nullptr;
  host_len_ = 0;
}

void Engine::unregister_host_deferred(std::shared_ptr<void> keep) {
  if (!host_ptr_) return;
  synchronize();  // this engine's streams: the user's are not waited for
  void* p = host_ptr_;
  Reaper::post(device_, [p, keep = std::move(keep)] { (void)hipHostUnregister(p); });
  host_ptr_ = nullptr;
  host_dev_ = nullptr;
  host_len_ = 0;
}

void Engine::h2d(int s, const void* host, size_t nbytes) {
  check_slot(s);
  const auto* h = static_cast<const uint8_t*>(host);
  if (host_ptr_ && (h < static_cast<uint8_t*>(host_ptr_) || h + nbytes > static_cast<uint8_t*>(host_ptr_) + host_len_))
    throw std::invalid_argument("engine: slot payload outside the registered host region");
  host_src_[size_t(s)] = h;
  if (mode_ == kH2DZeroCopy) {
    if (!host_dev_) throw std::runtime_error("engine: zero-copy mode needs a registered host region");
    return;
  }
  if (nbytes + 256 > stride_) throw std::invalid_argument("engine: copy larger than the staging buffer");
  hipStream_t st = stream_of_slot(s);
  if (nbytes) TKH_CHECK(hipMemcpyAsync(staging(s), host, nbytes, hipMemcpyHostToDevice, st));
  TKH_CHECK(hipEventRecord(copied_[size_t(s)], st));
}

const uint8_t* Engine::src_base(int s) const {
  if (mode_ == kH2DDma) return static_cast<const uint8_t*>(staging(s));
  const uint8_t* h = host_src_[size_t(s)];
  if (!h) throw std::runtime_error("engine: slot has no payload (h2d not called)");
  return host_dev_ + (h - static_cast<const uint8_t*>(host_ptr_));
}

void Engine::set_command_queue(bool on) {
  if (!on && cq_) queue().drain();  // calls queued so far stay ahead of the direct ones
  cq_ = on && queue().on();
}

bool Engine::queued(hipStream_t stream) const {
  if (!cq_ || !stream) return false;
  for (auto st : decode_streams_)
    if (st == stream) return true;
  return false;
}

void Engine::run_on(hipStream_t stream, std::function<void()>&& f) {
  if (queued(stream))
    queue().submit(std::move(f));
  else
    f();
}

bool Engine::slot_done(int s) {
  check_slot(s);
  if (!queue().ran(done_seq_[size_t(s)])) return false;  // its record has not even run yet
  hipError_t e = hipEventQuery(done_[size_t(s)]);
  if (e == hipSuccess) return true;
  if (e == hipErrorNotReady) return false;
  throw std::runtime_error(std::string("engine: slot event: ") + hipGetErrorString(e));
}

void Engine::wait_slot(int s) {
  check_slot(s);
  queue().wait(done_seq_[size_t(s)]);
  TKH_CHECK(hipEventSynchronize(done_[size_t(s)]));
}

void Engine::wait_copy(int s) {
  check_slot(s);
  if (mode_ == kH2DDma) TKH_CHECK(hipEventSynchronize(copied_[size_t(s)]));
}

void Engine::begin(int s, hipStream_t user) {
  if (mode_ == kH2DDma) TKH_CHECK(hipStreamWaitEvent(user, copied_[size_t(s)], 0));
}

void Engine::finish(int s, hipStream_t user) {
  hipEvent_t e = done_[size_t(s)];
  if (queued(user)) {
    done_seq_[size_t(s)] = queue().submit([e, user] { TKH_CHECK(hipEventRecord(e, user)); });
  } else {
    TKH_CHECK(hipEventRecord(e, user));
    done_seq_[size_t(s)] = 0;
  }
}

void Engine::collate_fixed(int s, hipStream_t user, size_t values_offset, int src_dt, void* dst, int dst_dt,
                           int64_t rows, int64_t row, const float* shift, const float* scale, bool record) {
  if (queued(user)) queue().drain();  // a direct launch on a queued stream: after the queue
  check_slot(s);
  begin(s, user);
  launch_fixed(src_base(s) + values_offset, src_dt, dst, dst_dt, rows, row, shift, scale, user);
  if (record) finish(s, user);
}

void Engine::collate_fixed_group(const int* slots, int n, hipStream_t user, const size_t* values_offsets, int src_dt,
                                 void* const* dsts, int dst_dt, const int64_t* rows, int64_t row, const float* shift,
                                 const float* scale) {
  if (queued(user)) queue().drain();  // a direct launch on a queued stream: after the queue
  if (n < 1 || n > kMaxGroup) throw std::invalid_argument("engine: bad group size");
  const void* srcs[kMaxGroup];
  for (int k = 0; k < n; ++k) {
    check_slot(slots[k]);
    begin(slots[k], user);
    srcs[k] = src_base(slots[k]) + values_offsets[k];
  }
  launch_fixed_group(srcs, src_dt, dsts, dst_dt, rows, n, row, shift, scale, user, mode_ == kH2DZeroCopy);
  finish(slots[n - 1], user);
}

void Engine::collate_gather_group(const int* slots, int n, hipStream_t user, int src_dt, void* const* dsts, int dst_dt,
                                  const int64_t* rows, int64_t row_bytes, const uint64_t* bases, const float* shift,
                                  const float* scale, bool record) {
  if (queued(user)) queue().drain();  // a direct launch on a queued stream: after the queue
  if (n < 1 || n > kMaxGroup) throw std::invalid_argument("engine: bad group size");
  const uint64_t* ents[kMaxGroup];
  for (int k = 0; k < n; ++k) {
    check_slot(slots[k]);
    begin(slots[k], user);
    ents[k] = reinterpret_cast<const uint64_t*>(src_base(slots[k]));
  }
  launch_gather_group(ents, src_dt, dsts, dst_dt, rows, n, bases, row_bytes, shift, scale, user);
  if (record) finish(slots[n - 1], user);
}

void Engine::stream_wait_done(int s, hipStream_t user) {
  check_slot(s);
  hipEvent_t e = done_[size_t(s)];
  if (queued(user)) {
    queue().submit([e, user] { TKH_CHECK(hipStreamWaitEvent(user, e, 0)); });
  } else {
    queue().wait(done_seq_[size_t(s)]);  // the record the wait refers to has run
    TKH_CHECK(hipStreamWaitEvent(user, e, 0));
  }
}

void Engine::collate_varlen(int s, hipStream_t user, size_t values_offset, int src_dt, void* out, int dst_dt,
                            int64_t rows, int64_t L, double pad, int64_t* lengths, uint8_t* mask, bool record) {
  if (queued(user)) queue().drain();  // a direct launch on a queued stream: after the queue
  check_slot(s);
  const uint8_t* base = src_base(s);
  begin(s, user);
  launch_varlen(reinterpret_cast<const int32_t*>(base), base + values_offset, src_dt, out, dst_dt, rows, L, pad,
                lengths, mask, user);
  if (record) finish(s, user);
}

void Engine::collate_json(int s, hipStream_t user, size_t values_offset, void* out, int dst_dt, int64_t rows,
                          int64_t L, double pad, int64_t* lengths, uint8_t* mask, int32_t* err, bool record) {
  if (queued(user)) queue().drain();  // a direct launch on a queued stream: after the queue
  check_slot(s);
  const uint8_t* base = src_base(s);
  begin(s, user);
  launch_json_rows(reinterpret_cast<const JsonRowDesc*>(base), base + values_offset, out, dst_dt, rows, L, pad,
                   lengths, mask, err, user);
  if (record) finish(s, user);
}

void Engine::collate_json_group(const int* slots, int n, hipStream_t user, const size_t* values_offsets,
                                const int64_t* rows, void* const* outs, const int64_t* Ls, int64_t* const* lengths,
                                uint8_t* const* masks, int32_t* const* errs, double pad, int dst_dt) {
  if (queued(user)) queue().drain();  // a direct launch on a queued stream: after the queue
  if (n < 1 || n > kMaxGroup) throw std::invalid_argument("engine: bad group size");
  JsonGroupArgs a{};
  a.n = n;
  a.pad = float(pad);
  a.row_base[0] = 0;
  for (int k = 0; k < n; ++k) {
    check_slot(slots[k]);
    begin(slots[k], user);
    const uint8_t* base = src_base(slots[k]);
    a.rows[k] = reinterpret_cast<const JsonRowDesc*>(base);
    a.vals[k] = base + values_offsets[k];
    a.out[k] = outs[k];
    a.L[k] = Ls[k];
    a.lengths[k] = lengths[k];
    a.mask[k] = masks[k];
    a.err[k] = errs[k];
    a.row_base[k + 1] = a.row_base[k] + rows[k];
  }
  launch_json_group(a, dst_dt, user);
  finish(slots[n - 1], user);
}

uint32_t* Engine::part_acc(hipStream_t stream) {
  constexpr size_t kSetWords = size_t(kMaxLaunchSegs) * 2;
  for (auto& pa : part_acc_)
    if (pa.stream == stream) return pa.words + (pa.next++ % kPartAccSets) * kSetWords;
  uint32_t* p = nullptr;
  const size_t bytes = kSetWords * kPartAccSets * sizeof(uint32_t);
  TKH_CHECK(hipSetDevice(device_));
  TKH_CHECK(hipMalloc(reinterpret_cast<void**>(&p), bytes));
  TKH_CHECK(hipMemset(p, 0, bytes));
  part_acc_.push_back(PartAcc{stream, p, 1});
  return p;
}

const uint32_t* Engine::span_tables() {
  if (!span_tabs_) {
    std::vector<uint32_t> t(tk::kSpanTabWords);
    tk::crc32c_span_tables(t.data());
    TKH_CHECK(hipSetDevice(device_));
    TKH_CHECK(hipMalloc(reinterpret_cast<void**>(&span_tabs_), t.size() * sizeof(uint32_t)));
    TKH_CHECK(hipMemcpy(span_tabs_, t.data(), t.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
  }
  return span_tabs_;
}

int Engine::default_decode_streams() {
  // three decode streams + the user's stream fill the 4 hardware queues HIP gives a process by
  // default (config 2: 2 streams 52.9 M rec/s, 3 streams 54.0 M, 4 streams 45.0 M -- the fourth
  // shares a queue).  TORCHKAFKA_DECODE_STREAMS / Tuning.decode_streams override it.
  const char* e = std::getenv("TORCHKAFKA_DECODE_STREAMS");
  const int v = e ? std::atoi(e) : 3;
  return v < 1 ? 1 : v > 4 ? 4 : v;
}

void Engine::set_decode_streams(int n) {
  for (auto st : decode_streams_)
    if (st != nullptr) throw std::runtime_error("set_decode_streams: decode streams already created");
  n_decode_ = n < 1 ? 1 : n > 4 ? 4 : n;
}

__global__ void decode_warm_kernel() {}

void Engine::prepare_decode() {
  queue().drain();
  span_tables();
  for (int k = 0; k < decode_streams(); ++k) {
    hipStream_t st = decode_stream(k);
    hipLaunchKernelGGL(decode_warm_kernel, dim3(1), dim3(64), 0, st);
    TKH_CHECK(hipGetLastError());
    TKH_CHECK(hipStreamSynchronize(st));
  }
  prewarm_span_kernels(device_);
  prewarm_json_span_kernels();
}

hipStream_t Engine::decode_stream(int k) {
  hipStream_t& st = decode_streams_[k % decode_streams()];
  if (!st) {
    TKH_CHECK(hipSetDevice(device_));
    const int prio = decode_priority();
    if (prio == 0) {
      TKH_CHECK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    } else {
      int least = 0, greatest = 0;
      TKH_CHECK(hipDeviceGetStreamPriorityRange(&least, &greatest));
      TKH_CHECK(hipStreamCreateWithPriority(&st, hipStreamNonBlocking, prio > 0 ? greatest : least));
    }
  }
  return st;
}

int Engine::decode_priority() {
  // the HSA queue priority of the decode streams: "high" lets the dispatcher hand freed CUs to the
  // decode workgroups before a co-running training job's next tiles (benchmarks/compute_overlap.py);
  // "normal" is HIP's default, "low" the opposite.  TORCHKAFKA_DECODE_PRIORITY overrides.
  const char* e = std::getenv("TORCHKAFKA_DECODE_PRIORITY");
  if (!e) return kDefaultDecodePriority;
  const std::string v(e);
  return v == "high" ? 1 : v == "low" ? -1 : 0;
}

void Engine::stream_after(hipStream_t later, hipStream_t earlier) {
  if (later == earlier) return;
  if (queued(later) || queued(earlier)) queue().drain();  // rare: keep both in order
  if (order_events_.empty()) {
    order_events_.resize(16);
    for (auto& e : order_events_) TKH_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  }
  // an event may be re-recorded once the wait that used it was enqueued (the wait captured it)
  hipEvent_t e = order_events_[order_next_++ % order_events_.size()];
  TKH_CHECK(hipEventRecord(e, earlier));
  TKH_CHECK(hipStreamWaitEvent(later, e, 0));
}

void Engine::collate_span(const int* slots, int n, hipStream_t user, SpanLaunch& a, int src_dt, int dst_dt,
                          const float* shift, const float* scale, bool record) {
  if (n < 1 || n > kMaxGroup) throw std::invalid_argument("engine: bad group size");
  for (int k = 0; k < n; ++k) {
    check_slot(slots[k]);
    begin(slots[k], user);  // DMA mode: the row table was copied with the slot payload
    a.b[k].row_pos = reinterpret_cast<const uint64_t*>(src_base(slots[k]));
    if (a.b[k].ext_words) a.b[k].ext_src = reinterpret_cast<const int64_t*>(src_base(slots[k]) + a.b[k].ext_off);
  }
  a.tabs = span_tables();
  a.part_acc = a.parts > 1 ? part_acc(user) : nullptr;  // the caller chose the parts
  if (queued(user)) {
    queue().submit([a, src_dt, dst_dt, shift, scale, user] {
      launch_span_decode(a, src_dt, dst_dt, shift, scale, user);
    });
  } else {
    launch_span_decode(a, src_dt, dst_dt, shift, scale, user);
  }
  if (record) finish(slots[n - 1], user);
}

void Engine::collate_json_stage(const int* slots, int n, hipStream_t user, JsonStageLaunch& a) {
  if (n < 1 || n > kMaxGroup) throw std::invalid_argument("engine: bad group size");
  for (int k = 0; k < n; ++k) {
    check_slot(slots[k]);
    begin(slots[k], user);  // DMA mode: the row table and host-parsed values were copied with the slot
    a.b[k].slot = src_base(slots[k]);
    a.b[k].rows = reinterpret_cast<const tk::JsonSpanRow*>(a.b[k].slot);
  }
  a.tabs = span_tables();
  a.part_acc = a.parts > 1 ? part_acc(user) : nullptr;  // the caller chose the parts
  if (queued(user))
    queue().submit([a, user] { launch_json_stage(a, user); });
  else
    launch_json_stage(a, user);
}

void Engine::copy_bytes(int s, hipStream_t user, size_t offset, void* dst, size_t nbytes) {
  if (queued(user)) queue().drain();  // a direct launch on a queued stream: after the queue
  check_slot(s);
  begin(s, user);
  if (nbytes) TKH_CHECK(hipMemcpyAsync(dst, src_base(s) + offset, nbytes, hipMemcpyDefault, user));
}

void Engine::copy_raw(int s, hipStream_t user, size_t offset, void* dst, size_t nbytes) {
  if (queued(user)) queue().drain();  // a direct launch on a queued stream: after the queue
  check_slot(s);
  begin(s, user);
  if (nbytes) TKH_CHECK(hipMemcpyAsync(dst, src_base(s) + offset, nbytes, hipMemcpyDefault, user));
  finish(s, user);
}

void Engine::synchronize() {
  queue().drain();
  for (auto st : streams_) TKH_CHECK(hipStreamSynchronize(st));
  for (auto st : decode_streams_)
    if (st) TKH_CHECK(hipStreamSynchronize(st));
}

}  // namespace tkh
