#include "driver.h"

#include "dtypes.h"
#include "hip_queue.h"
#include "reaper.h"

#include <unistd.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>

namespace {
const bool g_trace = [] {
  const char* e = std::getenv("TORCHKAFKA_DRIVER_TRACE");
  return e && e[0] == '1';
}();
}  // namespace
#define DTRACE(...)                                       \
  do {                                                    \
    if (g_trace) {                                        \
      std::fprintf(stderr, "[driver %d] ", int(getpid())); \
      std::fprintf(stderr, __VA_ARGS__);                  \
      std::fputc('\n', stderr);                           \
    }                                                     \
  } while (0)

namespace tkh {

MainDriver::MainDriver(Engine* engine, const std::string& ring_name, const std::string& broker_url,
                       const std::string& group, int prefetch, bool in_order, int default_src_dt)
    : eng_(engine), prefetch_(std::max(0, prefetch)) {
  std::shared_ptr<tk::Ring> ring = tk::Ring::open(ring_name);
  ring_keep_ = ring;
  if (int(ring->n_slots()) > eng_->n_slots()) throw std::invalid_argument("driver: engine has fewer slots than ring");
  // Pin THIS mapping of the ring: it is the one whose addresses the copies use
  // (another mapping of the same shm object has different virtual addresses).
  if (!eng_->host_registered()) {
    eng_->register_host(ring->base(), ring->total_bytes());
    registered_ = true;
  }
  uint32_t gidx = 0;
  if (!broker_url.empty() && !group.empty()) {
    broker_ = std::make_shared<tk::Broker>(broker_url, false, tk::BrokerConfig{});
    gidx = broker_->group_index(group, true);
  }
  ledger_ = std::make_unique<CommitLedger>(broker_, gidx);
  pins_ = std::make_unique<LogPins>(eng_, broker_);
  verdicts_ = std::make_unique<BatchVerdicts>(ring.get(), broker_.get(), &eng_->queue());
  poller_ = std::make_unique<RingPoller>(std::move(ring), eng_, pins_.get(), ledger_.get(), broker_.get(), in_order,
                                         default_src_dt);
}

MainDriver::~MainDriver() {
  // Quiesce this loader only -- never the device: the user's stream may hold a training step's
  // work for milliseconds, and a device-wide synchronize here would block the host on it.
  quiesce();
  // Memory and registrations go to the deferred-release thread (reaper.h): hipFree and
  // hipHostUnregister wait for the whole device, and this runs on the training thread.
  pins_.reset();  // pinned log ranges: every kernel that read them completed (quiesce)
  Reaper::free_device(eng_->device(), stage_dev_);
  stage_dev_ = nullptr;
  if (registered_) {
    try {
      eng_->unregister_host_deferred(ring_keep_);  // the release keeps the ring's mapping alive
    } catch (...) {
    }
  }
  for (auto& f : fenced_)
    if (std::get<0>(f)) hipEventDestroy(std::get<0>(f));
  verdicts_.reset();  // no kernel still writes a status word (quiesce)
  for (auto e : event_pool_) hipEventDestroy(e);
}

void MainDriver::quiesce() noexcept {
  try {
    eng_->queue().drain();  // queued launches read the slots, logs and staging freed by the caller
  } catch (...) {
  }
  // every slot handed out: its completion event follows its kernel, on whichever stream (a decode
  // stream, or the user's for the host-decode collates) -- not the user's later work
  for (const Handed& h : handed_) {
    if (!h.ev) continue;
    try {
      eng_->wait_slot(int(h.g));
    } catch (...) {
    }
  }
  try {
    eng_->synchronize();  // the decode and copy streams (ahead groups nobody was handed yet)
  } catch (...) {
  }
}

// ---------------------------------------------------------------------------------------------
// Launched slots: completion events and release

// Host slots whose collate kernel ran are handed back to their worker.  Kernels
// run in hand-out order on the user's stream, so the scan stops at the first
// incomplete one (one event query per batch in steady state).
// With batched events only some slots carry one; a completed event also completes
// every slot launched before it on that stream (note_handed keeps one stream per run).
void MainDriver::release_completed() {
  const int64_t t0 = tk::now_ns();
  // hipEventQuery costs ~0.5-1 us of host time; a group's kernel runs for tens of us, so an
  // event found pending is not asked again for kReleaseRequeryNs (a step calls this 2-3 times)
  if (t0 - pending_query_ns_ < kReleaseRequeryNs) return;
  release_completed_impl();
  rel_ns_ += tk::now_ns() - t0;
}

void MainDriver::release_completed_impl() {
  tk::Ring& ring = poller_->ring();
  size_t k = 0;
  while (k < handed_.size()) {
    size_t e = k;
    while (e < handed_.size() && !handed_[e].ev) ++e;  // next slot with an event
    if (e == handed_.size()) break;
    if (!eng_->slot_done(int(handed_[e].g))) {
      pending_query_ns_ = tk::now_ns();
      break;
    }
    for (; k <= e; ++k, ++released_) {
      const Handed& h = handed_[k];
      if (h.perr >= 0) verdicts_->on_release(h.g, h.perr, h.span);  // reads the slot: before its release
      if (h.stage_end) stage_tail_ = h.stage_end;  // its group's kernels completed
      ring.main_release(uint32_t(h.g));
    }
  }
  if (k) handed_.erase(handed_.begin(), handed_.begin() + long(k));
}

void MainDriver::cover_handed() {
  if (unevented_ == 0 || handed_.empty()) return;
  // the newest handed slot has no event: one recorded now on its stream covers it and
  // every unevented slot before it (they all ran on last_stream_)
  Handed& h = handed_.back();
  eng_->record_done(int(h.g), last_stream_);
  h.ev = true;
  unevented_ = 0;
  ++events_;
}

void MainDriver::switch_stream(hipStream_t stream) {
  if (stream == last_stream_) return;
  cover_handed();  // earlier unevented slots ran on the previous stream
  last_stream_ = stream;
}

void MainDriver::note_handed(int64_t g, hipStream_t stream, bool* record) {
  switch_stream(stream);
  *record = (unevented_ + 1 >= event_every_);
  if (*record) {
    unevented_ = 0;
    ++events_;
  } else {
    ++unevented_;
  }
  handed_.push_back(Handed{g, *record});
}

void MainDriver::force_event() {
  if (handed_.back().ev) return;
  handed_.back().ev = true;
  unevented_ = 0;
  ++events_;
}

int64_t MainDriver::group_handed(const int* slots, int n, hipStream_t stream, const int64_t* perrs, bool span,
                                 std::vector<std::shared_ptr<void>>&& handles, size_t first) {
  const int64_t gid = ++group_seq_;
  for (int k = 0; k < n; ++k) handed_.push_back(Handed{slots[k], k == n - 1, perrs ? perrs[k] : -1, span});
  handed_.back().stage_end = stage_last_end_;  // 0 unless a JSON group just took a staging region
  stage_last_end_ = 0;
  last_ev_slot_ = slots[n - 1];
  unevented_ = 0;
  ++events_;
  if (n > 1) ++groups_;
  auto& staged = poller_->staged();
  for (size_t k = first; k < size_t(n); ++k) {
    SlotView& v = staged[group_idx_[k - first]];
    if (perrs) v.perr = perrs[k];
    v.pre = true;
    v.pre_stream = stream;
    v.pre_event_slot = slots[n - 1];
    v.pre_group = gid;
    v.pre_out = std::move(handles[k - first]);
  }
  return gid;
}

void MainDriver::wait_launch(int64_t slot, int64_t group, hipStream_t stream) {
  if (waited_group_ == group && waited_stream_ == stream) return;  // one wait per group
  eng_->stream_wait_done(int(slot), stream);
  waited_group_ = group;
  waited_stream_ = stream;
}

// True while the latest launch that recorded a completion event has not finished on the GPU.
bool MainDriver::gpu_busy() {
  if (last_ev_slot_ < 0) return false;
  const int64_t now = tk::now_ns();
  if (now - busy_query_ns_ < kReleaseRequeryNs) return true;  // found busy a moment ago
  if (eng_->slot_done(int(last_ev_slot_))) {
    last_ev_slot_ = -1;
    return false;
  }
  busy_query_ns_ = now;
  return true;
}

int MainDriver::poll_blocking(int64_t timeout_ms) {
  // Workers may be waiting for slots the GPU still reads: cover them with an event and keep
  // releasing while waiting, so a full ring drains without a round trip through the caller.
  // While slots are in flight on the GPU this must not sleep on the ring futex: the next READY
  // slot may depend on a release only this thread can do (worker waits for a FREE slot, the
  // slot waits for its kernel, nobody would wake us before the futex timeout).  So: poll the
  // ring and the completion events together, spinning first (a kernel or a worker is usually
  // microseconds away), then in short sleeps; block on the futex only with nothing in flight.
  cover_handed();
  const int64_t start = tk::now_ns();
  const int64_t deadline = timeout_ms < 0 ? INT64_MAX : start + timeout_ms * 1000000LL;
  for (;;) {
    const int r = poller_->poll(false, 0);
    if (r != -1) return r;
    const int64_t now = tk::now_ns();
    if (now >= deadline) return -1;
    if (handed_.empty()) {
      const int64_t left_ms = deadline == INT64_MAX ? 20 : std::max<int64_t>(0, (deadline - now) / 1000000LL);
      const int r2 = poller_->poll(true, std::min<int64_t>(left_ms, 20));
      if (r2 != -1) return r2;
      continue;
    }
    release_completed();
    if (now - start < 200000) {
      for (int k = 0; k < 32; ++k) tk::cpu_relax();
    } else {
      timespec ts{0, 20000};
      nanosleep(&ts, nullptr);
    }
  }
}

// ---------------------------------------------------------------------------------------------
// Taking batches: lockstep or free-running

// The rank's data path as the lockstep protocol sees it (csrc/core/lockstep.h).
class MainDriver::Source : public tk::LockstepSource {
 public:
  explicit Source(MainDriver& d) : d_(d) {}
  int64_t staged() override { return d_.poller_->data_staged(); }
  bool all_done() override { return d_.poller_->all_done(); }
  int wait_data(int64_t timeout_ms) override {
    const int64_t t0 = tk::now_ns();
    const int r = d_.poll_blocking(timeout_ms);
    d_.blocked_ns_ += tk::now_ns() - t0;
    ++d_.blocked_calls_;
    return r == -3 ? -3 : r == 1 ? 1 : 0;
  }

 private:
  MainDriver& d_;
};

void MainDriver::enable_lockstep(LockstepTransport* ls, int depth, int commit_every) {
  ls_ = std::make_unique<tk::CreditLockstep>(ls, depth);
  ls_->set_commit_every(commit_every);
  ls_->set_on_committable([this](std::vector<tk::Watermark>&& wms) { ledger_->batch_committable(wms); });
  ls_->set_sync(sync_commit_);
  delivered_index_ = -1;
}

int MainDriver::next_slot_lockstep(int64_t timeout_ms, SlotView* out) {
  if (ls_->stopped()) return -2;
  // stage everything already published (non-blocking): these are the credits this rank can offer
  for (;;) {
    int r = poller_->poll(false, 0);
    if (r == -3) return -3;
    if (r <= 0) break;
  }
  Source src(*this);
  const int r = ls_->next(src, timeout_ms);
  DTRACE("lockstep next=%d step %ld granted %ld staged %d", r, long(ls_->step()), long(ls_->granted()),
         poller_->data_staged());
  if (r != 1) return r;
  if (!poller_->pop(out)) throw std::logic_error("lockstep: granted a batch that is not staged");
  delivered_index_ = ls_->delivered();
  return 1;
}

void MainDriver::finish_lockstep() {
  drain_fenced(true);
  if (ls_) ls_->finish();
}

int MainDriver::next_slot(int64_t timeout_ms, SlotView* out) {
  release_completed();
  // sync commits under a lockstep: the previous batch enters the protocol's finished queue (its
  // verdict landed) before the agreement that makes it committable on every rank is issued
  if (!fenced_.empty()) drain_fenced(ls_ && sync_commit_);
  if (!parse_error_.empty()) return -4;
  if (ls_) return next_slot_lockstep(timeout_ms, out);
  auto& staged = poller_->staged();
  for (;;) {
    // keep `prefetch` batches beyond the one handed out in flight to the device
    while (int(staged.size()) < prefetch_ + 1) {
      int r = poller_->poll(false, 0);
      if (r == -3) return -3;
      if (r <= 0) break;
    }
    if (staged.empty()) {
      const int64_t t0 = tk::now_ns();
      int r = poll_blocking(timeout_ms);
      blocked_ns_ += tk::now_ns() - t0;
      ++blocked_calls_;
      if (r < 0) return r;
      if (r == 0) return -1;
    }
    if (poller_->pop(out)) return 1;  // else only watermarks were staged: they ride on the next batch
  }
}

void MainDriver::stage_ready(int extra) {
  if (ls_) return;
  while (int(poller_->staged().size()) < prefetch_ + extra) {
    const int r = poller_->poll(false, 0);
    if (r <= 0) break;  // -3 is reported by next_slot
  }
}

// ---------------------------------------------------------------------------------------------
// Delivery, fencing and commits

void MainDriver::deliver(const SlotView& v) { set_delivered(v); }

void MainDriver::set_delivered(const SlotView& v) {
  delivered_ = v.wms;
  for (const tk::Watermark& w : v.wms) {
    if (w.pidx >= delivered_pos_.size()) delivered_pos_.resize(size_t(w.pidx) + 1, -1);
    if (w.next_offset > delivered_pos_[w.pidx]) delivered_pos_[w.pidx] = w.next_offset;
  }
  ++delivered_batches_;
  const bool checked = v.kind == tk::kPackJsonText || v.kind == tk::kPackRecordSpan || row_span_kind(v.kind);
  delivered_perr_ = checked ? (v.perr >= 0 ? v.perr : last_perr_) : -1;
}

void MainDriver::discard(const SlotView& v) {
  if (v.g < 0) return;
  eng_->wait_copy(int(v.g));
  poller_->ring().main_release(uint32_t(v.g));
}

void MainDriver::stage_finished(int64_t index, std::vector<tk::Watermark>&& wms) {
  if (ls_)
    ls_->finished(index, std::move(wms));
  else
    ledger_->batch_committable(wms);
}

void MainDriver::finish_delivered(hipStream_t fence) {
  if (delivered_.empty()) return;
  ledger_->batch_finished();
  const int64_t perr = delivered_perr_;
  delivered_perr_ = -1;
  if (perr >= 0 && !commit_on_device_) {
    // a device-checked batch commits only once its kernel ran clean (read at slot release)
    fenced_.emplace_back(nullptr, delivered_index_, std::move(delivered_), perr);
  } else if (commit_on_device_) {
    hipEvent_t ev;
    if (event_pool_.empty()) {
      if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess)
        throw std::runtime_error("driver: hipEventCreate failed");
    } else {
      ev = event_pool_.back();
      event_pool_.pop_back();
    }
    if (hipEventRecord(ev, fence) != hipSuccess) throw std::runtime_error("driver: hipEventRecord failed");
    fenced_.emplace_back(ev, delivered_index_, std::move(delivered_), perr);
  } else {
    stage_finished(delivered_index_, std::move(delivered_));
  }
  delivered_.clear();
}

// Waits (wait=true) until every launched device-checked kernel completed and its slot was
// released, so each pending status word has been read.
void MainDriver::settle_parse_errors(bool wait) {
  if (!wait) {
    release_completed();
    return;
  }
  cover_handed();
  while (!handed_.empty()) {
    for (const auto& h : handed_)
      if (h.ev) eng_->wait_slot(int(h.g));
    pending_query_ns_ = 0;
    release_completed();
  }
}

void MainDriver::drain_fenced(bool wait) {
  bool settled = false;
  while (!fenced_.empty() && parse_error_.empty()) {
    auto& f = fenced_.front();
    hipEvent_t ev = std::get<0>(f);
    const int64_t pe = std::get<3>(f);
    if (ev) {
      if (wait) {
        if (hipEventSynchronize(ev) != hipSuccess) throw std::runtime_error("driver: hipEventSynchronize failed");
      } else if (hipEventQuery(ev) != hipSuccess) {
        break;  // in order: a later batch is never committed before an earlier one
      }
    }
    if (pe >= 0 && verdicts_->state(pe) == 0) {
      if (!settled) {
        settle_parse_errors(wait);
        settled = true;
      }
      if (verdicts_->state(pe) == 0) break;  // its kernel has not completed yet
    }
    if (pe >= 0 && verdicts_->state(pe) == 2) {
      parse_error_ = verdicts_->failure(pe, std::get<2>(f));
      break;  // never committed
    }
    stage_finished(std::get<1>(f), std::move(std::get<2>(f)));
    if (ev) event_pool_.push_back(ev);
    fenced_.pop_front();
  }
}

bool MainDriver::delivered_verdict_known() {
  const int64_t pe = delivered_perr_;
  if (pe < 0 || !parse_error_.empty() || verdicts_->state(pe) != 0) return true;
  cover_handed();
  pending_query_ns_ = 0;
  release_completed_impl();
  return verdicts_->state(pe) != 0;
}

int MainDriver::verify_delivered() {
  const int64_t pe = delivered_perr_;
  if (!parse_error_.empty()) return -4;
  if (pe < 0) return 0;  // not device-checked: the worker verified it before publishing
  if (verdicts_->state(pe) == 0) {
    const int64_t t0 = tk::now_ns();
    cover_handed();
    for (;;) {
      size_t i = 0;
      while (i < handed_.size() && handed_[i].perr != pe) ++i;
      if (i == handed_.size()) break;  // released: its verdict was read
      size_t e = i;
      while (e < handed_.size() && !handed_[e].ev) ++e;
      if (e == handed_.size()) throw std::logic_error("driver: a delivered batch has no completion event");
      // release is in hand-out order: every earlier launch (other decode streams too) must be done
      for (size_t k = 0; k <= e; ++k)
        if (handed_[k].ev) eng_->wait_slot(int(handed_[k].g));
      pending_query_ns_ = 0;
      release_completed_impl();
    }
    verify_wait_ns_ += tk::now_ns() - t0;
  }
  if (verdicts_->state(pe) == 2) {
    drain_fenced(true);  // batches finished before this one stay committable (the reference commits
                         // batch k-1 before the fetch of batch k fails its CRC check)
    if (parse_error_.empty()) parse_error_ = verdicts_->failure(pe, delivered_);
    delivered_.clear();  // never finished, never committed
    delivered_perr_ = -1;
    return -4;
  }
  return 0;
}

int MainDriver::commit_pending() {
  drain_fenced(false);
  const int status = ledger_->commit();
  if (status == 1 && !ledger_->worker_sink()) pins_->committed(ledger_->committed_map());
  if (!parse_error_.empty()) return -2;  // the batches before the bad one were committed
  return status;
}

void MainDriver::reset_stats() {
  ledger_->reset_stats();
  pins_->reset_stats();
  poller_->reset_stats();
  blocked_ns_ = blocked_calls_ = 0;
  ph_commit_ns_ = ph_next_ns_ = ph_launch_ns_ = ph_steps_ = events_ = groups_ = 0;
  rel_ns_ = released_ = cwait_ns_ = 0;
  occ_handed_ = occ_staged_ = occ_samples_ = 0;
  ahead_groups_ = ahead_ns_ = split_launches_ = 0;
  verdicts_->width_wait_ns = 0;
  fast_batches_ = fast_records_ = fast_ns_ = 0;
  verify_wait_ns_ = 0;
  if (ls_) ls_->reset_stats();
}

}  // namespace tkh
