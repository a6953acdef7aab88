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

void MainDriver::enable_lockstep(LockstepTransport* ls, int depth) {
  ls_ = std::make_unique<tk::CreditLockstep>(ls, depth);
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
// Kernel launches

void MainDriver::launch_group(const int* slots, const int64_t* rows, const size_t* voffs, int n, const SlotView& v,
                              hipStream_t stream, int dst_dt, void* const* dsts, int64_t row, const float* shift,
                              const float* scale) {
  if (v.kind == uint32_t(tk::kPackGatherFixed))
    eng_->collate_gather_group(slots, n, stream, v.src_dtype, dsts, dst_dt, rows, int64_t(v.row_bytes),
                               pins_->bases_dev(), shift, scale);
  else
    eng_->collate_fixed_group(slots, n, stream, voffs, v.src_dtype, dsts, dst_dt, rows, row, shift, scale);
}

void MainDriver::copy_extras(const int* slots, const SlotView* const* views, int n, hipStream_t stream) {
  for (int k = 0; k < n && k < ext_n_; ++k) {
    const SlotView& v = *views[k];
    if (v.extras_n && ext_dsts_[k])
      eng_->copy_bytes(slots[k], stream, size_t(v.extras_offset), ext_dsts_[k], size_t(v.n_rows) * v.extras_n * 8u);
  }
  ext_n_ = 0;
}

void MainDriver::collate_fixed(const SlotView& v, hipStream_t stream, int dst_dt, void* dst, int64_t row,
                               const float* shift, const float* scale) {
  const int slot = int(v.g);
  const SlotView* vs[1] = {&v};
  if (v.kind != uint32_t(tk::kPackRecordSpan) && ext_n_) copy_extras(&slot, vs, 1, stream);  // its event covers the copy
  bool record;
  note_handed(v.g, stream, &record);
  if (!record && coalesce_wait_ns_ > 0 && coalesce_ > 1) {
    // adaptive coalescing decides from the latest launch's completion: give this one its event
    force_event();
    record = true;
  }
  if (record) last_ev_slot_ = v.g;
  if (v.kind == uint32_t(tk::kPackRecordSpan)) {
    void* d = dst;
    int64_t pe;
    launch_span(&slot, vs, 1, stream, dst_dt, &d, shift, scale, record, &pe);
    handed_.back().perr = pe;
    handed_.back().span = true;
    last_perr_ = pe;
    return;
  }
  if (v.kind == uint32_t(tk::kPackGatherFixed)) {
    const int64_t rows = v.n_rows;
    void* d = dst;
    eng_->collate_gather_group(&slot, 1, stream, v.src_dtype, &d, dst_dt, &rows, int64_t(v.row_bytes),
                               pins_->bases_dev(), shift, scale, record);
    return;
  }
  eng_->collate_fixed(slot, stream, v.values_offset, v.src_dtype, dst, dst_dt, v.n_rows, row, shift, scale, record);
}

void MainDriver::collate_varlen(const SlotView& v, hipStream_t stream, int dst_dt, void* out, int64_t L, double pad,
                                int64_t* lengths, uint8_t* mask) {
  bool record;
  if (row_span_kind(v.kind)) {
    // decoded from the logs on the user's stream, its own completion event
    switch_stream(stream);
    const int slot = int(v.g);
    const SlotView* vs[1] = {&v};
    void* outs[1] = {out};
    const int64_t Ls[1] = {L};
    int64_t* lens[1] = {lengths};
    uint8_t* masks[1] = {mask};
    int64_t pe;
    launch_row_span(&slot, vs, 1, stream, dst_dt, pad, outs, Ls, lens, masks, true, &pe);
    group_handed(&slot, 1, stream, &pe, true, {}, 1);
    last_perr_ = pe;
    return;
  }
  if (v.kind == tk::kPackJsonText) {
    const int64_t idx = verdicts_->next_word();
    note_handed(v.g, stream, &record);
    handed_.back().perr = idx;
    eng_->collate_json(int(v.g), stream, v.values_offset, out, dst_dt, v.n_rows, L, pad, lengths, mask,
                       verdicts_->err_dev(idx), record);
    last_perr_ = idx;
    return;
  }
  note_handed(v.g, stream, &record);
  eng_->collate_varlen(int(v.g), stream, v.values_offset, v.src_dtype, out, dst_dt, v.n_rows, L, pad, lengths, mask,
                       record);
}

void MainDriver::copy_payload(const SlotView& v, hipStream_t stream, void* dst) {
  bool record;
  note_handed(v.g, stream, &record);
  force_event();  // copy_raw always records the slot's completion event
  eng_->copy_raw(int(v.g), stream, 0, dst, size_t(v.payload_bytes));
}

void MainDriver::check_seg_count(const tk::SpanSeg& sg, uint32_t i) const {
  constexpr uint32_t kWhole = tk::kSegCrcFirst | tk::kSegCrcLast;
  if ((sg.flags & tk::kSegCrc) && (sg.flags & kWhole) != kWhole && i >= uint32_t(BatchVerdicts::kPartials))
    throw std::runtime_error("driver: a batch splits RecordBatches into more than 512 device segments");
}

void MainDriver::fill_seg(SpanDevSeg& d, const tk::SpanSeg& sg, const uint8_t* src, int k, uint32_t i) {
  d = SpanDevSeg{};
  d.src = src;
  d.log_pos = sg.log_pos;
  d.len = sg.len;
  d.flags = sg.flags;
  d.crc = sg.crc;
  d.row_begin = sg.row_begin;
  d.row_end = sg.row_end;
  d.batch = uint16_t(k);
  d.seg = uint16_t(i);
}

void MainDriver::launch_span(const int* slots, const SlotView* const* views, int n, hipStream_t stream, int dst_dt,
                             void* const* dsts, const float* shift, const float* scale, bool record_last,
                             int64_t* perrs) {
  if (!broker_) throw std::runtime_error("driver: device decode needs the synthetic broker");
  verdicts_->ensure_partials();
  LogMirror* mirror = pins_->mirror();
  const SlotView& v0 = *views[0];
  SpanLaunch a{};
  a.row_elems = v0.max_row_len;
  const int ssz = dtype_size(v0.src_dtype), dsz = dtype_size(dst_dt);
  const int per = ssz > 0 ? 16 / ssz : 1;
  bool vec = ssz > 0 && a.row_elems % per == 0 && (a.row_elems * dsz) % 16 == 0;
  for (int k = 0; k < n; ++k) {
    vec = vec && reinterpret_cast<uintptr_t>(dsts[k]) % 16 == 0;
    perrs[k] = verdicts_->next_word();
    a.b[k].out = dsts[k];
    a.b[k].err = verdicts_->err_dev(perrs[k]);
    a.b[k].partials = verdicts_->partials_dev(perrs[k]);
    const SlotView& v = *views[k];
    if (v.extras_n && k < ext_n_ && ext_dsts_[k]) {  // key / timestamp columns ride in the same kernel
      a.b[k].ext_out = ext_dsts_[k];
      a.b[k].ext_off = v.extras_offset;
      a.b[k].ext_words = v.n_rows * v.extras_n;
    }
  }
  ext_n_ = 0;
  a.vec_store = vec ? 1 : 0;
  bool pcie = false;  // a segment of this launch is read over PCIe (not from the HBM mirror)
  auto flush = [&](bool record) {
    // segments split over parts only when every one is read from HBM: parts multiply the loads in
    // flight of a lone group from the mirror (2 MiB: 30.6 -> 12.6 us with 8), while over PCIe the
    // link is the limit and more workgroups only add their fixed costs (profiles/r05_s30_lane_merge)
    a.parts = pcie ? 1 : eng_->span_parts();
    split_launches_ += a.parts > 1;
    pcie = false;
    if (mirror) mirror->before(stream);
    eng_->collate_span(slots, n, stream, a, v0.src_dtype, dst_dt, shift, scale, record);
    if (mirror) mirror->after(stream);
  };
  for (int k = 0; k < n; ++k) {
    const tk::SpanSeg* sg = segs(*views[k]);
    for (uint32_t i = 0; i < views[k]->n_segs; ++i) {
      check_seg_count(sg[i], i);
      if (a.n_seg == kMaxLaunchSegs) {
        flush(false);
        a.n_seg = 0;
      }
      fill_seg(a.s[a.n_seg++], sg[i], seg_src(sg[i], &pcie), k, i);
    }
  }
  flush(record_last);
}

uint64_t MainDriver::stage_alloc(uint64_t bytes) {
  bytes = (bytes + 255) & ~uint64_t(255);
  if (bytes > kStageBytes) throw std::runtime_error("driver: a device JSON group exceeds the staging ring");
  if (!stage_dev_ && hipMalloc(reinterpret_cast<void**>(&stage_dev_), kStageBytes) != hipSuccess)
    throw std::runtime_error("driver: hipMalloc of the JSON staging ring failed");
  uint64_t pos = stage_head_;
  const uint64_t in = pos % kStageBytes;
  if (in + bytes > kStageBytes) pos += kStageBytes - in;  // never split a region: restart at the front
  while (pos + bytes - stage_tail_ > kStageBytes) {
    // the oldest groups still read their regions: wait for the first one with an event
    cover_handed();
    bool waited = false;
    for (const auto& h : handed_) {
      if (!h.ev) continue;
      eng_->wait_slot(int(h.g));
      waited = true;
      break;
    }
    if (!waited) throw std::logic_error("driver: JSON staging ring full with nothing in flight");
    pending_query_ns_ = 0;
    release_completed_impl();
  }
  stage_head_ = pos + bytes;
  stage_last_end_ = stage_head_;
  return pos % kStageBytes;
}

void MainDriver::launch_json_span(const int* slots, const SlotView* const* views, int n, hipStream_t stream,
                                  int dst_dt, double pad, void* const* outs, const int64_t* Ls,
                                  int64_t* const* lengths, uint8_t* const* masks, bool record_last, int64_t* perrs) {
  if (!broker_) throw std::runtime_error("driver: device JSON parse needs the synthetic broker");
  verdicts_->ensure_partials();
  LogMirror* mirror = pins_->mirror();
  tk::Ring& ring = poller_->ring();
  // staging per batch: the row descriptors, then one region per segment (row texts rounded up to
  // 16 bytes, or the float32 values of the rows the worker parsed)
  constexpr uint64_t kA = 256;
  auto up = [](uint64_t x, uint64_t a) { return (x + a - 1) / a * a; };
  // bytes of segment i's region in its batch's staging area
  auto seg_bytes = [&](const SlotView& v, const tk::SpanSeg& sg) {
    if (!(sg.flags & tk::kSegHostRows)) return up(up(sg.len, 16) + 16 * uint64_t(sg.row_end - sg.row_begin), kA);
    const auto* rows = reinterpret_cast<const tk::JsonSpanRow*>(ring.payload(uint32_t(v.g)));
    uint64_t b = 0;
    for (uint32_t r = sg.row_begin; r < sg.row_end; ++r) {
      int64_t c = rows[r].count;
      if (v.trunc_len >= 0 && c > v.trunc_len) c = v.trunc_len;
      b += up(uint64_t(c < 0 ? 0 : c) * 4, 16);
    }
    return up(b, kA);
  };
  uint64_t batch_bytes[kMaxGroup], total = 0;
  for (int k = 0; k < n; ++k) {
    const SlotView& v = *views[k];
    const tk::SpanSeg* sg = segs(v);
    uint64_t b = up(uint64_t(v.n_rows) * sizeof(JsonRowDesc), kA);
    for (uint32_t i = 0; i < v.n_segs; ++i) b += seg_bytes(v, sg[i]);
    batch_bytes[k] = b;
    total += b;
  }
  const uint64_t base = stage_alloc(total);
  JsonStageLaunch a{};
  bool pcie = false;
  JsonGroupArgs ga{};
  ga.n = n;
  ga.pad = float(pad);
  ga.err_tag = tk::kSpanParseErrBit;
  ga.mult = json_mult_;
  uint64_t off = base;
  for (int k = 0; k < n; ++k) {
    const SlotView& v = *views[k];
    perrs[k] = verdicts_->next_word();
    JsonStageBatch& b = a.b[k];
    if (v.flags & tk::kSlotDevCount) {  // tagged count words: nothing to zero per launch
      b.ctr = verdicts_->json_ctr_dev(perrs[k]);
      b.ctr_tag = verdicts_->ctr_tag(perrs[k]);
      ga.ctr[k] = b.ctr;
      ga.ctr_tag[k] = b.ctr_tag;
      ga.info[k] = verdicts_->json_info_dev(perrs[k]);
    }
    b.desc = reinterpret_cast<JsonRowDesc*>(stage_dev_ + off);
    const uint64_t dbytes = up(uint64_t(v.n_rows) * sizeof(JsonRowDesc), kA);
    b.stage = stage_dev_ + off + dbytes;
    b.err = verdicts_->err_dev(perrs[k]);
    b.partials = verdicts_->partials_dev(perrs[k]);
    b.trunc_len = v.trunc_len;
    ga.rows[k] = b.desc;
    ga.vals[k] = b.stage;
    ga.vals_cap[k] = batch_bytes[k] - dbytes;
    ga.out[k] = outs[k];
    ga.L[k] = Ls[k];
    ga.lengths[k] = lengths[k];
    ga.mask[k] = masks[k];
    ga.err[k] = b.err;
    ga.row_base[k + 1] = ga.row_base[k] + int64_t(v.n_rows);
    ga.trunc[k] = v.trunc_len;
    off += batch_bytes[k];
  }
  auto flush = [&]() {
    a.parts = pcie ? 1 : eng_->json_span_parts();  // parts only for segments all read from HBM (launch_span)
    split_launches_ += a.parts > 1;
    pcie = false;
    if (mirror) mirror->before(stream);
    eng_->collate_json_stage(slots, n, stream, a);
    if (mirror) mirror->after(stream);
  };
  for (int k = 0; k < n; ++k) {
    const SlotView& v = *views[k];
    const tk::SpanSeg* sg = segs(v);
    uint64_t soff = 0;  // offset in the batch's staging area (after its descriptors)
    for (uint32_t i = 0; i < v.n_segs; ++i) {
      check_seg_count(sg[i], i);
      if (a.n_seg == kMaxLaunchSegs) {
        flush();
        a.n_seg = 0;
      }
      SpanDevSeg& d = a.s[a.n_seg++];
      fill_seg(d, sg[i], (sg[i].flags & tk::kSegHostRows) ? nullptr : seg_src(sg[i], &pcie), k, i);
      d.stage_off = uint32_t(soff);
      soff += seg_bytes(v, sg[i]);
    }
  }
  flush();
  bool devc = false;
  for (int k = 0; k < n; ++k) devc = devc || ga.ctr[k] != nullptr;
  // a wave per row: counts, simple check, the width words.  Not fused into json_stage_kernel: its
  // few workgroups (one per segment) took 149 us per group doing it instead of 71 us, and config 4
  // fell from 40.5 M to 35.5 M rec/s (profiles/r04_s4)
  if (devc) eng_->run_on(stream, [ga, stream] { launch_json_count(ga, stream); });
  // the parse: a block per row over the staged texts, on the same stream
  eng_->run_on(stream, [ga, dst_dt, stream]() mutable { launch_json_group(ga, dst_dt, stream); });
  if (record_last) eng_->record_done(slots[n - 1], stream);
}

void MainDriver::launch_var_span(const int* slots, const SlotView* const* views, int n, hipStream_t stream,
                                 int dst_dt, double pad, void* const* outs, const int64_t* Ls,
                                 int64_t* const* lengths, uint8_t* const* masks, bool record_last, int64_t* perrs) {
  if (!broker_) throw std::runtime_error("driver: device decode needs the synthetic broker");
  verdicts_->ensure_partials();
  LogMirror* mirror = pins_->mirror();
  VarSpanLaunch a{};
  bool pcie = false;
  const int src_dt = views[0]->src_dtype;
  for (int k = 0; k < n; ++k) {
    perrs[k] = verdicts_->next_word();
    VarSpanBatch& b = a.b[k];
    b.out = outs[k];
    b.L = Ls[k];
    b.lengths = lengths[k];
    b.mask = masks[k];
    b.err = verdicts_->err_dev(perrs[k]);
    b.partials = verdicts_->partials_dev(perrs[k]);
    b.trunc_len = views[k]->trunc_len;
    // vector stores of a 16-byte source group (16 / ssz elements of dsz bytes): rows and groups aligned
    const int ssz = dtype_size(src_dt), dsz = dtype_size(dst_dt);
    const int64_t gbytes = ssz > 0 ? int64_t(16 / ssz) * dsz : 0;
    b.reserved = (gbytes >= 16 && gbytes % 16 == 0 && reinterpret_cast<uintptr_t>(outs[k]) % 16 == 0 &&
                  (Ls[k] * dsz) % 16 == 0) ? 1 : 0;
  }
  auto flush = [&](bool record) {
    for (int k = 0; k < n; ++k) {
      a.b[k].slot = eng_->slot_src(slots[k], stream);  // DMA mode: after the slot's copy
      a.b[k].rows = reinterpret_cast<const tk::JsonSpanRow*>(a.b[k].slot);
    }
    a.tabs = eng_->span_tables();
    a.parts = pcie ? 1 : eng_->span_parts();  // parts only for segments all read from HBM (launch_span)
    a.part_acc = a.parts > 1 ? eng_->part_acc(stream) : nullptr;
    split_launches_ += a.parts > 1;
    pcie = false;
    if (mirror) mirror->before(stream);
    eng_->run_on(stream, [a, src_dt, dst_dt, pad, stream] { tkh::launch_var_span(a, src_dt, dst_dt, pad, stream); });
    if (mirror) mirror->after(stream);
    if (record) eng_->record_done(slots[n - 1], stream);
  };
  for (int k = 0; k < n; ++k) {
    const SlotView& v = *views[k];
    if (v.src_dtype != src_dt) throw std::invalid_argument("driver: a var-len group mixes element dtypes");
    const tk::SpanSeg* sg = segs(v);
    for (uint32_t i = 0; i < v.n_segs; ++i) {
      check_seg_count(sg[i], i);
      if (a.n_seg == kMaxLaunchSegs) {
        flush(false);
        a.n_seg = 0;
      }
      fill_seg(a.s[a.n_seg++], sg[i], (sg[i].flags & tk::kSegHostRows) ? nullptr : seg_src(sg[i], &pcie), k, i);
    }
  }
  flush(record_last);
}

// ---------------------------------------------------------------------------------------------
// Group formation and the coalesced steps

size_t MainDriver::json_group_extend() {
  group_idx_.clear();
  if (coalesce_ <= 1 || (last.kind != uint32_t(tk::kPackJsonText) && !row_span_kind(last.kind))) return 0;
  const auto& staged = poller_->staged();
  uint64_t bytes = last.span_bytes;
  for (size_t i = 0; i < staged.size() && int(1 + group_idx_.size()) < coalesce_; ++i) {
    const SlotView& v = staged[i];
    if (v.g < 0) continue;  // watermark-only slot: rides on the next delivered batch
    if (v.pre || v.kind != last.kind || v.n_rows == 0 || group_full(bytes, v)) break;
    bytes += v.span_bytes;
    group_idx_.push_back(i);
  }
  return group_idx_.size();
}

void MainDriver::json_group_launch(hipStream_t stream, int dst_dt, double pad, void* const* outs, const int64_t* Ls,
                                   int64_t* const* lengths, uint8_t* const* masks,
                                   std::vector<std::shared_ptr<void>>&& handles) {
  const int n = 1 + int(group_idx_.size());
  if (int(handles.size()) != n - 1) throw std::invalid_argument("driver: group handles do not match the group");
  auto& staged = poller_->staged();
  int slots[kMaxGroup];
  const SlotView* vs[kMaxGroup];
  for (int k = 0; k < n; ++k) {
    vs[k] = k == 0 ? &last : &staged[group_idx_[size_t(k - 1)]];
    slots[k] = int(vs[k]->g);
  }
  int64_t perrs[kMaxGroup];
  if (row_span_kind(last.kind)) {
    // decoded on the next decode stream (outputs allocated there, torch_step.cpp); the user's
    // stream waits for the group's completion
    cover_handed();
    hipStream_t ks = next_decode_stream();
    ++span_launches_;
    last_stream_ = ks;
    launch_row_span(slots, vs, n, ks, dst_dt, pad, outs, Ls, lengths, masks, true, perrs);
    last.perr = perrs[0];
    const int64_t gid = group_handed(slots, n, ks, perrs, true, std::move(handles), 1);
    wait_launch(slots[n - 1], gid, stream);
    group_idx_.clear();
    return;
  }
  size_t voffs[kMaxGroup];
  int64_t rows[kMaxGroup];
  int32_t* errs[kMaxGroup];
  for (int k = 0; k < n; ++k) {
    voffs[k] = vs[k]->values_offset;
    rows[k] = vs[k]->n_rows;
    perrs[k] = verdicts_->next_word();
    errs[k] = verdicts_->err_dev(perrs[k]);
  }
  last.perr = perrs[0];
  switch_stream(stream);
  eng_->collate_json_group(slots, n, stream, voffs, rows, outs, Ls, lengths, masks, errs, pad, dst_dt);
  group_handed(slots, n, stream, perrs, false, std::move(handles), 1);
  group_idx_.clear();
}

int64_t MainDriver::step_fixed(hipStream_t stream, int dst_dt, void* dst, int64_t row, const float* shift,
                               const float* scale, bool auto_commit, int64_t timeout_ms, int* commit_status,
                               SlotView* out) {
  *commit_status = 0;
  const int64_t t0 = tk::now_ns();
  finish_delivered(stream);  // asking for the next batch finishes the previous one
  if (auto_commit) *commit_status = commit_pending();
  const int64_t t1 = tk::now_ns();
  int r = next_slot(timeout_ms, out);
  const int64_t t2 = tk::now_ns();
  ph_commit_ns_ += t1 - t0;
  ph_next_ns_ += t2 - t1;
  if (r < 0) return r;
  collate_fixed(*out, stream, dst_dt, dst, row, shift, scale);
  set_delivered(*out);
  poller_->prefetch_ready();
  ph_launch_ns_ += tk::now_ns() - t2;
  ++ph_steps_;
  return out->n_rows;
}

int64_t MainDriver::step_group_begin(hipStream_t stream, bool auto_commit, int64_t timeout_ms, int* commit_status,
                                     std::vector<int64_t>* group_rows, std::shared_ptr<void>* pre_out) {
  *commit_status = 0;
  group_rows->clear();
  group_idx_.clear();
  const int64_t t0 = tk::now_ns();
  finish_delivered(stream);  // asking for the next batch finishes the previous one
  if (auto_commit) *commit_status = commit_pending();
  const int64_t t1 = tk::now_ns();
  auto& staged = poller_->staged();
  if (!ls_ && coalesce_ > 1) {
    // stage what the workers already published, so a group can form (never blocks)
    while (int(staged.size()) < prefetch_ + coalesce_) {
      const int r = poller_->poll(false, 0);
      if (r == -3) return -3;
      if (r <= 0) break;
    }
  }
  occ_handed_ += int64_t(handed_.size());
  occ_staged_ += int64_t(staged.size());
  ++occ_samples_;
  const int r = next_slot(timeout_ms, &last);
  const int64_t t2 = tk::now_ns();
  ph_commit_ns_ += t1 - t0;
  ph_next_ns_ += t2 - t1;
  if (r < 0) return r;
  if (last.pre) {
    // collated by an earlier group launch; a consumer on another stream waits for that kernel
    if (last.pre_stream != stream) wait_launch(last.pre_event_slot, last.pre_group, stream);
    *pre_out = std::move(last.pre_out);
    set_delivered(last);
    poller_->prefetch_ready();
    ++ph_steps_;
    return last.n_rows;
  }
  group_rows->push_back(last.n_rows);
  if (last.kind == uint32_t(tk::kPackFixed) || last.kind == uint32_t(tk::kPackGatherFixed) ||
      last.kind == uint32_t(tk::kPackRecordSpan)) {
    group_capped_ = false;
    extend_group();
    if (coalesce_wait_ns_ > 0 && int(1 + group_idx_.size()) < coalesce_ && !group_capped_) {
      const int64_t cw0 = tk::now_ns();
      const int64_t until = cw0 + coalesce_wait_ns_;
      while (int(1 + group_idx_.size()) < coalesce_ && !group_capped_ && gpu_busy() && tk::now_ns() < until) {
        const int r2 = poller_->poll(false, 0);
        if (r2 == -3) break;  // reported by the next call
        if (r2 == 1) {
          extend_group();
          continue;
        }
        release_completed();
        for (int k = 0; k < 16; ++k) tk::cpu_relax();
      }
      cwait_ns_ += tk::now_ns() - cw0;
    }
    for (size_t i : group_idx_) group_rows->push_back(staged[i].n_rows);
  }
  return last.n_rows;
}

// Appends to group_idx_ the staged batches right behind `last` that one kernel can collate with it.
void MainDriver::extend_group() {
  const auto& staged = poller_->staged();
  size_t i = group_idx_.empty() ? 0 : group_idx_.back() + 1;
  uint64_t bytes = last.span_bytes;
  for (size_t k : group_idx_) bytes += staged[k].span_bytes;
  for (; i < staged.size() && int(1 + group_idx_.size()) < coalesce_; ++i) {
    const SlotView& v = staged[i];
    if (v.g < 0) continue;  // watermark-only slot: rides on the next delivered batch
    if (group_full(bytes, v)) group_capped_ = true;
    if (v.pre || v.kind != last.kind || v.src_dtype != last.src_dtype || v.max_row_len != last.max_row_len ||
        v.row_bytes != last.row_bytes || v.shape != last.shape || v.n_rows == 0 || group_capped_)
      return;
    bytes += v.span_bytes;
    group_idx_.push_back(i);
  }
}

void MainDriver::step_group_launch(hipStream_t stream, int dst_dt, void* const* dsts, int64_t row,
                                   const float* shift, const float* scale,
                                   std::vector<std::shared_ptr<void>>&& handles) {
  const int64_t t0 = tk::now_ns();
  const int n = 1 + int(group_idx_.size());
  if (int(handles.size()) != n - 1) throw std::invalid_argument("driver: group handles do not match the group");
  auto& staged = poller_->staged();
  int slots[kMaxGroup];
  size_t voffs[kMaxGroup];
  int64_t rows[kMaxGroup];
  const SlotView* vs[kMaxGroup];
  for (int k = 0; k < n; ++k) {
    vs[k] = k == 0 ? &last : &staged[group_idx_[size_t(k - 1)]];
    slots[k] = int(vs[k]->g);
    voffs[k] = vs[k]->values_offset;
    rows[k] = vs[k]->n_rows;
  }
  if (last.kind == uint32_t(tk::kPackRecordSpan)) {
    // Device decode rotates over the decode streams: a group's kernel is PCIe-bound while it
    // loads and compute-bound in its CRC/extract tail, so the next group's loads overlap that
    // tail.  The outputs were allocated on the decode stream (torch_step.cpp: the caching
    // allocator orders their reuse against it, and knows the user's stream uses them); the
    // user's stream waits for the group's completion before it touches a batch of it.
    cover_handed();
    hipStream_t ks = next_decode_stream();
    ++span_launches_;
    last_stream_ = ks;
    int64_t perrs[kMaxGroup];
    launch_span(slots, vs, n, ks, dst_dt, dsts, shift, scale, true, perrs);
    last.perr = perrs[0];
    const int64_t gid = group_handed(slots, n, ks, perrs, true, std::move(handles), 1);
    wait_launch(slots[n - 1], gid, stream);
  } else if (n == 1) {
    collate_fixed(last, stream, dst_dt, dsts[0], row, shift, scale);
  } else {
    switch_stream(stream);
    if (ext_n_) copy_extras(slots, vs, n, stream);
    launch_group(slots, rows, voffs, n, last, stream, dst_dt, dsts, row, shift, scale);
    group_handed(slots, n, stream, nullptr, false, std::move(handles), 1);
  }
  group_idx_.clear();
  set_delivered(last);
  poller_->prefetch_ready();
  ph_launch_ns_ += tk::now_ns() - t0;
  ++ph_steps_;
}

void MainDriver::ahead_begin(std::vector<int64_t>* rows) {
  rows->clear();
  group_idx_.clear();
  if (ahead_depth_ <= 0 || coalesce_ <= 1) return;
  const auto& staged = poller_->staged();
  const size_t want = size_t(prefetch_ + (ahead_depth_ + 1) * coalesce_);
  while (staged.size() < want) {
    if (poller_->poll(false, 0) <= 0) break;  // nothing ready (an error is reported by next_slot)
  }
  int pre = 0;
  size_t i0 = staged.size();
  for (size_t i = 0; i < staged.size(); ++i) {
    const SlotView& v = staged[i];
    if (v.g < 0) continue;
    if (v.pre)
      ++pre;
    else if (i0 == staged.size())
      i0 = i;
  }
  if (pre >= ahead_depth_ * coalesce_ || i0 == staged.size()) return;
  const SlotView& f = staged[i0];
  const bool json = row_span_kind(f.kind);  // outputs sized per batch: no shape match needed
  if ((f.kind != uint32_t(tk::kPackRecordSpan) && !json) || f.n_rows == 0) return;
  uint64_t bytes = 0;
  bool capped = false;
  for (size_t i = i0; i < staged.size() && int(group_idx_.size()) < coalesce_; ++i) {
    const SlotView& v = staged[i];
    if (v.g < 0) continue;  // watermark-only slot: rides on the next delivered batch
    if (v.pre || v.kind != f.kind || v.n_rows == 0) break;
    if (group_full(bytes, v)) {
      capped = true;  // a full group by bytes
      break;
    }
    bytes += v.span_bytes;
    if (!json && (v.src_dtype != f.src_dtype || v.max_row_len != f.max_row_len || v.row_bytes != f.row_bytes ||
                  v.shape != f.shape))
      break;
    group_idx_.push_back(i);
  }
  // a group that could not take one more batch of its last one's size is full without waiting to
  // see that batch: config 5 (8 MiB batches, 16 MiB groups, a 4-slot ring) never has a third
  // batch staged while two are in flight, so its groups would otherwise never go ahead
  if (!capped && !group_idx_.empty() && bytes + staged[group_idx_.back()].span_bytes > group_bytes_max_)
    capped = true;
  if (int(group_idx_.size()) < coalesce_ && !capped) {  // only full groups go ahead; the rest waits for the user
    group_idx_.clear();
    return;
  }
  for (size_t i : group_idx_) rows->push_back(staged[i].n_rows);
}

void MainDriver::ahead_launch(int dst_dt, void* const* dsts, const float* shift, const float* scale,
                              std::vector<std::shared_ptr<void>>&& handles) {
  const int n = int(group_idx_.size());
  if (n < 1 || int(handles.size()) != n) throw std::invalid_argument("driver: ahead group does not match");
  const int64_t t0 = tk::now_ns();
  auto& staged = poller_->staged();
  int slots[kMaxGroup];
  const SlotView* vs[kMaxGroup];
  for (int k = 0; k < n; ++k) {
    vs[k] = &staged[group_idx_[size_t(k)]];
    slots[k] = int(vs[k]->g);
  }
  cover_handed();
  hipStream_t ks = next_decode_stream();
  ++span_launches_;
  last_stream_ = ks;
  int64_t perrs[kMaxGroup];
  launch_span(slots, vs, n, ks, dst_dt, dsts, shift, scale, true, perrs);
  group_handed(slots, n, ks, perrs, true, std::move(handles), 0);
  group_idx_.clear();
  ++ahead_groups_;
  ph_launch_ns_ += tk::now_ns() - t0;
}

void MainDriver::ahead_launch_json(int dst_dt, double pad, void* const* outs, const int64_t* Ls,
                                   int64_t* const* lengths, uint8_t* const* masks,
                                   std::vector<std::shared_ptr<void>>&& handles) {
  const int n = int(group_idx_.size());
  if (n < 1 || int(handles.size()) != n) throw std::invalid_argument("driver: ahead group does not match");
  const int64_t t0 = tk::now_ns();
  auto& staged = poller_->staged();
  int slots[kMaxGroup];
  const SlotView* vs[kMaxGroup];
  for (int k = 0; k < n; ++k) {
    vs[k] = &staged[group_idx_[size_t(k)]];
    slots[k] = int(vs[k]->g);
  }
  cover_handed();
  hipStream_t ks = next_decode_stream();
  ++span_launches_;
  last_stream_ = ks;
  int64_t perrs[kMaxGroup];
  launch_row_span(slots, vs, n, ks, dst_dt, pad, outs, Ls, lengths, masks, true, perrs);
  group_handed(slots, n, ks, perrs, true, std::move(handles), 0);
  group_idx_.clear();
  ++ahead_groups_;
  ph_launch_ns_ += tk::now_ns() - t0;
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
