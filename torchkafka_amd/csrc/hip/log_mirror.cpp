#include "log_mirror.h"

#include "reaper.h"

#include <algorithm>
#include <cstdlib>
#include <stdexcept>
#include <string>

#include "hip_queue.h"
#include "span.h"

namespace tkh {

#define TKM_CHECK(expr)                                                                                \
  do {                                                                                                 \
    hipError_t _e = (expr);                                                                            \
    if (_e != hipSuccess) throw std::runtime_error(std::string("log mirror: ") + #expr + ": " + hipGetErrorString(_e)); \
  } while (0)

LogMirror::LogMirror(int device, HipQueue* queue, uint64_t chunk_bytes, int chunks_per_partition, int copy_streams,
                     int wait)
    : device_(device), chunk_(chunk_bytes), K_(chunks_per_partition), q_(queue) {
  if (!q_) throw std::invalid_argument("log mirror: no command queue");
  if (chunk_ < (uint64_t(1) << 20) || chunk_ % 4096 != 0) throw std::invalid_argument("log mirror: chunk must be >= 1 MiB, 4 KiB aligned");
  if (K_ < 2) throw std::invalid_argument("log mirror: at least 2 chunks per partition");
  prefetch_ = K_ > 3 ? K_ - 2 : 1;
  stride_ = (chunk_ + tk::kSpanSegMax + 256 + 4095) / 4096 * 4096;
  TKM_CHECK(hipSetDevice(device_));
  const char* w = std::getenv("TORCHKAFKA_MIRROR_WAIT");
  wait_ = w && (w[0] == '0' || w[0] == '1') ? w[0] == '1' : wait == 1;  // the variable wins (A/B runs)
  const char* e = std::getenv("TORCHKAFKA_MIRROR_COPY_STREAMS");
  const int n = e ? std::atoi(e) : copy_streams > 0 ? copy_streams : 2;  // the variable wins (A/B runs)
  cs_.resize(size_t(n < 1 ? 1 : n > 4 ? 4 : n));
  for (auto& c : cs_) {
    TKM_CHECK(hipStreamCreateWithFlags(&c.stream, hipStreamNonBlocking));
    TKM_CHECK(hipEventCreateWithFlags(&c.copied, hipEventDisableTiming));
  }
  pool_.resize(256);
  for (auto& e : pool_) TKM_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  pool_seq_.assign(pool_.size(), 0);
  pool_rec_q_.assign(pool_.size(), 0);
  pool_refs_.assign(pool_.size(), 0);
}

LogMirror::~LogMirror() {
  try {
    q_->drain();  // queued copies and records use the streams and events below
  } catch (...) {
  }
  hipSetDevice(device_);
  for (auto& c : cs_)
    if (c.stream) hipStreamSynchronize(c.stream);
  // no decode kernel still reads a buffer: the owner (LogPins) synchronized the decode streams
  for (auto& P : parts_) Reaper::free_device(device_, P.dev);  // hipFree waits for the whole device
  for (auto e : pool_) hipEventDestroy(e);
  for (auto& c : cs_) {
    if (c.copied) hipEventDestroy(c.copied);
    if (c.stream) hipStreamDestroy(c.stream);
  }
}

void LogMirror::set_command_queue(bool on) {
  if (!on && cq_) q_->drain();
  cq_ = on && q_->on();
}

uint64_t LogMirror::issue(std::function<void()>&& f) {
  if (cq_) return q_->submit(std::move(f));
  f();
  return 0;
}

LogMirror::Part& LogMirror::part(uint32_t pidx) {
  if (pidx >= parts_.size()) parts_.resize(size_t(pidx) + 1);
  Part& P = parts_[pidx];
  if (!P.dev) {
    TKM_CHECK(hipSetDevice(device_));
    TKM_CHECK(hipMalloc(reinterpret_cast<void**>(&P.dev), stride_ * size_t(K_)));
    P.bufs.assign(size_t(K_), Buf{});
    for (auto& b : P.bufs) b.s = int(pidx % cs_.size());
    dev_bytes_ += stride_ * size_t(K_);
  }
  return P;
}

void LogMirror::retarget(Buf& b, int64_t c) {
  // the copy stream overwrites the buffer only after every reader of its previous chunk
  hipStream_t copy = cs_[size_t(b.s)].stream;
  for (auto& r : b.readers) {
    if (r.ev >= 0 && pool_seq_[size_t(r.ev)] == r.seq) {
      hipEvent_t ev = pool_[size_t(r.ev)];
      issue([copy, ev] { TKM_CHECK(hipStreamWaitEvent(copy, ev, 0)); });
      --pool_refs_[size_t(r.ev)];
    }
    r = Reader{};
  }
  b.chunk = c;
  b.end = uint64_t(c) * chunk_;
  b.copy_seq = 0;
}

LogMirror::Buf* LogMirror::ensure(Part& P, uint32_t pidx, int64_t c, uint64_t want_end, const uint8_t* log,
                                  uint64_t pinned, bool prefetch) {
  (void)pidx;
  const size_t j = size_t(c % K_);
  Buf& b = P.bufs[j];
  if (b.chunk != c) {
    if (b.pending) return nullptr;  // read by the launch being formed
    retarget(b, c);
  }
  const uint64_t lo_c = uint64_t(c) * chunk_;
  const uint64_t target = std::min<uint64_t>(pinned, lo_c + chunk_ + tk::kSpanSegMax);
  if (want_end > b.end) {
    if (target < want_end) return nullptr;  // not pinned/written that far (the caller pins first)
  } else if (!prefetch || target <= b.end || (target - b.end < chunk_ / 4 && target < lo_c + chunk_ + tk::kSpanSegMax)) {
    return &b;  // resident (a prefetch tops up only in sizeable pieces)
  }
  if (target > b.end) {
    // one copy per pinned registration: a DMA source must lie inside one registered range, and the
    // driver pins the logs in kRegAlign pieces (so that consumed pieces can be unpinned)
    for (uint64_t a = b.end; a < target;) {
      const uint64_t e = std::min<uint64_t>(target, (a / kRegAlign + 1) * kRegAlign);
      uint8_t* dst = P.dev + j * stride_ + (a - lo_c);
      const uint8_t* src = log + a;
      const size_t n = size_t(e - a);
      hipStream_t st = cs_[size_t(b.s)].stream;
      issue([dst, src, n, st] { TKM_CHECK(hipMemcpyAsync(dst, src, n, hipMemcpyHostToDevice, st)); });
      ++copies_;
      a = e;
    }
    bytes_ += target - b.end;
    b.end = target;
    b.copy_seq = ++cs_[size_t(b.s)].seq;
  }
  return &b;
}

const uint8_t* LogMirror::map(uint32_t pidx, uint64_t pos, uint32_t len, const uint8_t* log, uint64_t pinned) {
  if (len > tk::kSpanSegMax) throw std::invalid_argument("log mirror: segment longer than kSpanSegMax");
  if (backoff_left_ > 0) {  // copies fell behind the decode (header): the pinned log, no copy
    --backoff_left_;
    ++fallbacks_;
    return nullptr;
  }
  if (!wait_ && ++eval_maps_ == kEvalMaps) {
    if (eval_pending_ * 2 > kEvalMaps) {
      backoff_left_ = kBackoffMaps;
      ++backoffs_;
    }
    eval_maps_ = eval_pending_ = 0;
  }
  Part& P = part(pidx);
  const int64_t c = int64_t(pos / chunk_);
  Buf* b = ensure(P, pidx, c, pos + len, log, pinned, false);
  if (!b) {
    ++fallbacks_;
    return nullptr;
  }
  if (!wait_ && b->copy_seq > cs_[size_t(b->s)].done) {
    CopyStream& cs = cs_[size_t(b->s)];
    if (!cs.queried) learn(cs);
    if (b->copy_seq > cs.done) {
      // its copy is still in flight: read the pinned log this time (the prefetches keep going)
      ++fallbacks_;
      ++pending_fallbacks_;
      ++eval_pending_;
      deferred_.push_back(Deferred{pidx, c, log, pinned});
      return nullptr;
    }
  }
  if (!b->pending) {
    b->pending = true;
    pending_.emplace_back(pidx, int(c % K_));
  }
  // the next chunks stream in behind this one while the decode catches up with it: K - 2 ahead (one
  // buffer for the chunk being read, one for the chunk its readers may still finish).  Queued after
  // before() has recorded this launch's copy event, so the launch never waits for its prefetches.
  deferred_.push_back(Deferred{pidx, c, log, pinned});
  return P.dev + size_t(c % K_) * stride_ + (pos - uint64_t(c) * chunk_);
}

void LogMirror::issue_prefetches() {
  for (const auto& d : deferred_) {
    Part& P = parts_[d.pidx];
    for (int64_t k = 1; k <= prefetch_ && d.pinned > uint64_t(d.chunk + k) * chunk_; ++k)
      if (!ensure(P, d.pidx, d.chunk + k, 0, d.log, d.pinned, true)) break;
  }
  deferred_.clear();
}

// The copy stream's event is recorded through the HIP command queue when it is on: until that
// record has run, the copies it covers count as in flight (no HIP call).
bool LogMirror::copied_done(CopyStream& c) {
  return q_->ran(c.rec_q) && hipEventQuery(c.copied) == hipSuccess;
}

void LogMirror::record_copied(CopyStream& c) {
  hipEvent_t ev = c.copied;
  hipStream_t st = c.stream;
  c.rec_q = issue([ev, st] { TKM_CHECK(hipEventRecord(ev, st)); });
  c.recorded = c.seq;
}

void LogMirror::learn(CopyStream& c) {
  c.queried = true;
  if (c.recorded > c.done && copied_done(c)) c.done = c.recorded;
  if (c.seq > c.recorded && c.recorded == c.done) record_copied(c);
}

void LogMirror::before(hipStream_t stream) {
  if (!wait_) {
    // every buffer this launch maps was found complete: nothing to wait for; queue the
    // prefetches, then mark the copy streams' tails so their completion can be learned
    issue_prefetches();
    for (auto& c : cs_) {
      if (c.seq > c.recorded && c.recorded == c.done) record_copied(c);
      c.queried = false;
    }
    return;
  }
  uint64_t need[4] = {0, 0, 0, 0};
  for (const auto& pb : pending_) {
    const Buf& b = parts_[pb.first].bufs[size_t(pb.second)];
    need[b.s] = std::max(need[b.s], b.copy_seq);
  }
  for (size_t s = 0; s < cs_.size(); ++s) {
    CopyStream& c = cs_[s];
    if (need[s] == 0 || need[s] <= c.done) continue;
    // One event per copy stream, recorded only when a launch needs a copy not known complete: it
    // also covers the prefetches queued behind that copy (a longer wait), but events between SDMA
    // copies cost more than they save (measured, config 2 --h2d dma: 46.5 M rec/s this way,
    // 32-34 M with an event after every copy).
    if (c.recorded < need[s]) record_copied(c);
    if (copied_done(c)) {  // found complete: no wait, and remembered
      c.done = c.recorded;
    } else {
      hipEvent_t ev = c.copied;
      issue([stream, ev] { TKM_CHECK(hipStreamWaitEvent(stream, ev, 0)); });
    }
  }
  issue_prefetches();
}

int LogMirror::next_event() {
  const int e = int(pool_next_++ % pool_.size());
  if (pool_refs_[size_t(e)] > 0) {
    // still named by a buffer: that reader is 256 launches old; make sure it completed, then
    // every reference to its old recording counts as completed (the sequence moves on)
    q_->wait(pool_rec_q_[size_t(e)]);
    TKM_CHECK(hipEventSynchronize(pool_[size_t(e)]));
    pool_refs_[size_t(e)] = 0;
  }
  ++pool_seq_[size_t(e)];
  return e;
}

void LogMirror::after(hipStream_t stream) {
  if (pending_.empty()) return;
  const int e = next_event();
  {
    hipEvent_t ev = pool_[size_t(e)];
    pool_rec_q_[size_t(e)] = issue([ev, stream] { TKM_CHECK(hipEventRecord(ev, stream)); });
  }
  for (const auto& pb : pending_) {
    Buf& b = parts_[pb.first].bufs[size_t(pb.second)];
    b.pending = false;
    Reader* slot = nullptr;
    for (auto& r : b.readers) {
      if (r.ev >= 0 && pool_seq_[size_t(r.ev)] != r.seq) r = Reader{};  // completed long ago
      if (r.ev >= 0 && r.stream == stream) {
        --pool_refs_[size_t(r.ev)];  // superseded: the new event follows it on the same stream
        r = Reader{};
      }
      if (r.ev < 0 && !slot) slot = &r;
    }
    if (!slot) {
      // more reader streams than remembered: retire the first one on the host
      slot = &b.readers[0];
      q_->wait(pool_rec_q_[size_t(slot->ev)]);
      TKM_CHECK(hipEventSynchronize(pool_[size_t(slot->ev)]));
      --pool_refs_[size_t(slot->ev)];
    }
    *slot = Reader{stream, e, pool_seq_[size_t(e)]};
    ++pool_refs_[size_t(e)];
  }
  pending_.clear();
}

}  // namespace tkh
