#include "driver.h"

#include "consumer.h"
#include "crc32c.h"
#include "dtypes.h"

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
    : eng_(engine), prefetch_(std::max(0, prefetch)), in_order_(in_order), default_src_dt_(default_src_dt) {
  ring_ = tk::Ring::open(ring_name);
  if (int(ring_->n_slots()) > eng_->n_slots()) throw std::invalid_argument("driver: engine has fewer slots than ring");
  // Pin THIS mapping of the ring: it is the one whose addresses the copies use
  // (another mapping of the same shm object has different virtual addresses).
  if (!eng_->host_registered()) {
    eng_->register_host(ring_->base(), ring_->total_bytes());
    registered_ = true;
  }
  cursor_.assign(ring_->n_workers(), 0);
  done_.assign(ring_->n_workers(), 0);
  if (!broker_url.empty() && !group.empty()) {
    broker_ = std::make_shared<tk::Broker>(broker_url, false, tk::BrokerConfig{});
    group_ = broker_->group_index(group, true);
    reg_end_.assign(broker_->meta().max_partitions, 0);  // log ranges pinned for direct / span reads
    reg_ranges_.resize(broker_->meta().max_partitions);
    release_consumed_ = (broker_->flags() & tk::kReleaseConsumed) != 0;
  }
  commit_ns_.reserve(1 << 16);
}

MainDriver::~MainDriver() {
  mirror_.reset();  // its copies read the pinned logs: before they are unregistered
  // pinned log ranges first: the kernels that read them completed (slots drained by the caller)
  bool any = false;
  for (auto& q : reg_ranges_) any = any || !q.empty();
  if (any) hipDeviceSynchronize();
  for (size_t pidx = 0; pidx < reg_ranges_.size(); ++pidx) {
    auto& q = reg_ranges_[pidx];
    for (auto& r : q) hipHostUnregister(r.first);
    if (!q.empty() && broker_) broker_->part(uint32_t(pidx)).pinned.fetch_sub(1, std::memory_order_acq_rel);
  }
  if (bases_dev_) hipFree(bases_dev_);
  if (stage_dev_) {
    hipDeviceSynchronize();
    hipFree(stage_dev_);
  }
  if (registered_) {
    try {
      eng_->unregister_host();  // before ring_'s mapping goes away
    } catch (...) {
    }
  }
  for (auto& f : fenced_)
    if (std::get<0>(f)) hipEventDestroy(std::get<0>(f));
  if (perr_host_ || part_host_) hipDeviceSynchronize();  // no kernel may still write a status word
  if (perr_host_) hipHostFree(perr_host_);
  if (jinfo_host_) hipHostFree(jinfo_host_);
  if (patch_dev_) hipFree(patch_dev_);
  if (part_host_) hipHostFree(part_host_);
  for (auto e : event_pool_) hipEventDestroy(e);
}

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
      const int64_t pe = handed_[k].perr;
      if (pe >= 0) {
        // a device-counted JSON batch with rows left to the host: parse them while the slot (their
        // row table) is still held, in case the batch is delivered after this release
        if (handed_[k].span && __atomic_load_n(jinfo_host_ + pe * 4 + 1, __ATOMIC_ACQUIRE) > 0)
          json_parse_host_rows(handed_[k].g, pe);
        if (handed_[k].span) check_span(handed_[k].g, pe);  // reads the slot: before its release
        perr_state_[size_t(pe)] = __atomic_load_n(perr_host_ + pe, __ATOMIC_ACQUIRE) < 0 ? 1 : 2;
      }
      if (handed_[k].stage_end) stage_tail_ = handed_[k].stage_end;  // its group's kernels completed
      ring_->main_release(uint32_t(handed_[k].g));
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

void MainDriver::note_handed(int64_t g, hipStream_t stream, bool* record) {
  if (stream != last_stream_) {
    cover_handed();  // earlier unevented slots ran on the previous stream
    last_stream_ = stream;
  }
  *record = (unevented_ + 1 >= event_every_);
  if (*record) {
    unevented_ = 0;
    ++events_;
  } else {
    ++unevented_;
  }
  handed_.push_back(Handed{g, *record});
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
    const int r = poll_one(false, 0);
    if (r != -1) return r;
    const int64_t now = tk::now_ns();
    if (now >= deadline) return -1;
    if (handed_.empty()) {
      const int64_t left_ms = deadline == INT64_MAX ? 20 : std::max<int64_t>(0, (deadline - now) / 1000000LL);
      const int r2 = poll_one(true, std::min<int64_t>(left_ms, 20));
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

int MainDriver::poll_one(bool block, int64_t timeout_ms) {
  const int64_t t0 = block ? 0 : tk::now_ns();
  const int r = poll_one_impl(block, timeout_ms);
  if (!block) poll_ns_ += tk::now_ns() - t0;
  if (r == 1) ++polled_;
  return r;
}

int MainDriver::poll_one_impl(bool block, int64_t timeout_ms) {
  for (;;) {
    const int64_t g = ring_->main_acquire(cursor_.data(), &rr_, done_.data(), in_order_, block ? timeout_ms : 0);
    if (g == -2) return -2;
    if (g < 0) return -1;
    tk::SlotHeader* h = ring_->slot(uint32_t(g));
    if (h->flags & tk::kSlotError) {
      error_.assign(h->err, h->err_len);
      ring_->main_release(uint32_t(g));
      return -3;
    }
    if (h->flags & tk::kSlotEOS) {
      done_.at(h->worker) = 1;
      DTRACE("EOS from worker %u (rows %u)", h->worker, h->n_rows);
    }
    fill_ns_ += h->t_ready_ns - h->t_fill_start_ns;
    ready_age_ns_ += tk::now_ns() - h->t_ready_ns;
    {
      // worker idle: from its previous publish to the start of this fill (waiting for a FREE
      // slot, plus its per-batch Python work)
      if (last_ready_.size() <= h->worker) last_ready_.resize(h->worker + 1, 0);
      int64_t& lr = last_ready_[h->worker];
      if (lr > 0 && h->t_fill_start_ns > lr) worker_idle_ns_ += h->t_fill_start_ns - lr;
      worker_slot_wait_ns_ += h->t_acquire_wait_ns;
      lr = h->t_ready_ns;
    }
    ++fills_;
    SlotView v;
    v.g = g;
    v.n_rows = h->n_rows;
    v.flags = h->flags;
    v.kind = h->kind;
    v.worker = h->worker;
    v.payload_bytes = h->payload_bytes;
    v.values_offset = h->values_offset;
    v.extras_offset = h->extras_offset;
    v.extras_n = h->extras_n;
    v.row_bytes = h->row_bytes;
    v.max_row_len = h->max_row_len;
    v.total_elems = h->total_elems;
    v.n_scanned = h->n_scanned;
    v.src_dtype = h->src_dtype >= 0 ? h->src_dtype : default_src_dt_;
    if (h->src_dtype >= 0) v.shape.assign(h->shape, h->shape + h->ndim);
    v.wms.assign(h->wm, h->wm + h->n_parts);
    if (sink_table_)
      for (uint32_t k = 0; k < h->n_parts; ++k) pidx_worker_[h->wm[k].pidx] = h->worker;
    if (v.n_rows == 0) {
      // empty (end-of-stream) slot: keep its watermarks in delivery order
      ring_->main_release(uint32_t(g));
      if (!v.wms.empty()) {
        v.g = -1;
        staged_.push_back(std::move(v));
        return 1;
      }
      if (!block) return 0;
      continue;
    }
    if (v.kind == uint32_t(tk::kPackRecordSpan) || row_span_kind(v.kind)) {
      if (!broker_) {
        error_ = "DeviceLoader: device decode needs the synthetic broker (group_id + bootstrap_servers)";
        return -3;
      }
      // pin every log range the segments cover (plus the 16-byte tail the kernel's aligned loads
      // may touch) before any kernel may read them
      v.n_segs = h->n_segs;
      v.trunc_len = h->trunc_len;
      const auto* sg = reinterpret_cast<const tk::SpanSeg*>(ring_->payload(uint32_t(g)) + h->values_offset);
      for (uint32_t i = 0; i < h->n_segs; ++i) {
        if (sg[i].flags & tk::kSegHostRows) continue;  // worker-parsed rows: no log bytes
        v.span_bytes += sg[i].len;
        const uint64_t cap = broker_->part(sg[i].pidx).log_capacity;
        ensure_log(sg[i].pidx, std::min<uint64_t>(sg[i].log_pos + sg[i].len + 16, cap));
      }
    }
    if (v.kind == uint32_t(tk::kPackGatherFixed)) {
      if (!direct_) {
        error_ = "DeviceLoader: a worker produced a log-gather slot but direct mode is off";
        return -3;
      }
      // pin every log range this slot's rows live in before any kernel may read them
      for (uint32_t k = 0; k < h->n_parts; ++k) ensure_log(h->wm[k].pidx, h->log_end[k]);
    }
    eng_->h2d(int(g), ring_->payload(uint32_t(g)), v.payload_bytes);
    staged_.push_back(std::move(v));
    return 1;
  }
}

// Pull the headers of the slots the next acquisition will look at into this core's
// cache while the caller runs Python: they were written by worker processes on other
// cores, and reading them cold costs several cross-core transfers per batch.  Only
// READY slots are touched, so a worker still filling a slot never loses its lines.
void MainDriver::prefetch_ready() const {
  const uint32_t nw = ring_->n_workers(), spw = ring_->slots_per_worker();
  for (uint32_t w = 0; w < nw; ++w) {
    if (done_[w]) continue;
    const tk::SlotHeader* h = ring_->slot(w * spw + cursor_[w]);
    if (h->state.load(std::memory_order_relaxed) != tk::kSlotReady) continue;
    const char* p = reinterpret_cast<const char*>(h);
    __builtin_prefetch(p + 64);
    __builtin_prefetch(p + 128);
    __builtin_prefetch(reinterpret_cast<const char*>(&h->wm[0]));
  }
}

int MainDriver::data_staged() const {
  int n = 0;
  for (const auto& v : staged_) n += v.g >= 0 ? 1 : 0;
  return n;
}

bool MainDriver::all_done() const {
  for (auto d : done_)
    if (!d) return false;
  return true;
}

bool MainDriver::pop_data(SlotView* out) {
  while (!staged_.empty()) {
    SlotView v = std::move(staged_.front());
    staged_.pop_front();
    if (v.g < 0) {
      carry_.insert(carry_.end(), v.wms.begin(), v.wms.end());
      continue;
    }
    if (!carry_.empty()) {
      v.wms.insert(v.wms.begin(), carry_.begin(), carry_.end());
      carry_.clear();
    }
    *out = std::move(v);
    return true;
  }
  return false;
}

// The rank's data path as the lockstep protocol sees it (csrc/core/lockstep.h).
class MainDriver::Source : public tk::LockstepSource {
 public:
  explicit Source(MainDriver& d) : d_(d) {}
  int64_t staged() override { return d_.data_staged(); }
  bool all_done() override { return d_.all_done(); }
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
  ls_->set_on_committable([this](std::vector<tk::Watermark>&& wms) { batch_committable(wms); });
  delivered_index_ = -1;
}

int MainDriver::next_slot_lockstep(int64_t timeout_ms, SlotView* out) {
  if (ls_->stopped()) return -2;
  // stage everything already published (non-blocking): these are the credits this rank can offer
  for (;;) {
    int r = poll_one(false, 0);
    if (r == -3) return -3;
    if (r <= 0) break;
  }
  Source src(*this);
  const int r = ls_->next(src, timeout_ms);
  DTRACE("lockstep next=%d step %ld granted %ld staged %d", r, long(ls_->step()), long(ls_->granted()),
         data_staged());
  if (r != 1) return r;
  if (!pop_data(out)) throw std::logic_error("lockstep: granted a batch that is not staged");
  delivered_index_ = ls_->delivered();
  return 1;
}

void MainDriver::finish_lockstep() {
  drain_fenced(true);
  if (ls_) ls_->finish();
}

int MainDriver::next_slot(int64_t timeout_ms, SlotView* out) {
  release_completed();
  if (!fenced_.empty()) drain_fenced(false);
  if (!parse_error_.empty()) return -4;
  if (ls_) return next_slot_lockstep(timeout_ms, out);
  for (;;) {
    // keep `prefetch` batches beyond the one handed out in flight to the device
    while (int(staged_.size()) < prefetch_ + 1) {
      int r = poll_one(false, 0);
      if (r == -3) return -3;
      if (r <= 0) break;
    }
    if (staged_.empty()) {
      const int64_t t0 = tk::now_ns();
      int r = poll_blocking(timeout_ms);
      blocked_ns_ += tk::now_ns() - t0;
      ++blocked_calls_;
      if (r < 0) return r;
      if (r == 0) return -1;
    }
    SlotView v = std::move(staged_.front());
    staged_.pop_front();
    if (v.g < 0) {  // empty slot: its watermarks ride on the next delivered batch
      carry_.insert(carry_.end(), v.wms.begin(), v.wms.end());
      continue;
    }
    if (!carry_.empty()) {
      v.wms.insert(v.wms.begin(), carry_.begin(), carry_.end());
      carry_.clear();
    }
    *out = std::move(v);
    return 1;
  }
}

void MainDriver::enable_direct() {
  if (!broker_) throw std::runtime_error("DeviceLoader h2d='direct' needs the synthetic broker (group_id + URL)");
  if (direct_) return;
  const uint32_t np = broker_->meta().max_partitions;
  reg_end_.assign(np, 0);
  if (hipMalloc(reinterpret_cast<void**>(&bases_dev_), size_t(np) * sizeof(uint64_t)) != hipSuccess)
    throw std::runtime_error("driver: hipMalloc(log base table) failed");
  if (hipMemset(bases_dev_, 0, size_t(np) * sizeof(uint64_t)) != hipSuccess)
    throw std::runtime_error("driver: hipMemset failed");
  direct_ = true;
}

void MainDriver::pin_logs(const std::vector<uint32_t>& pidxs) {
  if (!broker_) return;
  eng_->prepare_decode();
  for (uint32_t p : pidxs) {
    if (p >= reg_end_.size()) continue;
    const uint64_t written = broker_->part(p).log_end_pos.load(std::memory_order_acquire);
    if (written) ensure_log(p, written);
  }
}

static_assert(MainDriver::kLogChunk == LogMirror::kRegAlign, "mirror copies split at the pin pieces");

void MainDriver::ensure_log(uint32_t pidx, uint64_t end) {
  if (pidx >= reg_end_.size()) throw std::out_of_range("driver: partition index beyond the broker's table");
  if (end <= reg_end_[pidx]) return;
  const int64_t t0 = tk::now_ns();
  const uint8_t* base = broker_->log_base(pidx);
  const uint64_t cap = broker_->part(pidx).log_capacity;
  if (end > cap) throw std::runtime_error("driver: slot references bytes beyond the partition log");
  // Everything already written (a retained backlog is pinned once, at its first use), then whole
  // chunks, so a growing log pays one registration per 64 MiB.  Pinning costs ~13 GB/s of fresh
  // shm pages on the MI355X host (profiles/*/register_probe2.log): it is what bounds this mode
  // on a log that grows faster than that.
  const uint64_t written = broker_->part(pidx).log_end_pos.load(std::memory_order_acquire);
  uint64_t hi = (std::max(end, written) + kLogChunk - 1) / kLogChunk * kLogChunk;
  if (hi > cap) hi = cap;
  const uint64_t lo = reg_end_[pidx];
  if (reg_ranges_.size() <= pidx) reg_ranges_.resize(size_t(pidx) + 1);
  auto& part = broker_->part(pidx);
  if (reg_ranges_[pidx].empty()) {  // announce the pin before it exists (the replicator reads these)
    part.pin_floor.store(lo, std::memory_order_release);
    part.pinned.fetch_add(1, std::memory_order_acq_rel);
  }
  // kLogChunk pieces, so that consumed ranges can be unpinned piecewise (release_consumed)
  for (uint64_t a = lo; a < hi; a += kLogChunk) {
    const uint64_t b = std::min(hi, a + kLogChunk);
    void* p = const_cast<uint8_t*>(base) + a;
    if (hipHostRegister(p, b - a, hipHostRegisterMapped) != hipSuccess)
      throw std::runtime_error("driver: hipHostRegister of a partition log failed");
    reg_ranges_[pidx].emplace_back(p, b);
    void* dp = nullptr;
    if (hipHostGetDevicePointer(&dp, p, 0) != hipSuccess || dp != p)
      throw std::runtime_error("driver: h2d='direct' needs device addresses of pinned host memory to equal host "
                               "addresses (unified addressing)");
  }
  if (lo == 0 && bases_dev_) {
    const uint64_t b = reinterpret_cast<uint64_t>(base);
    if (hipMemcpy(bases_dev_ + pidx, &b, sizeof(b), hipMemcpyHostToDevice) != hipSuccess)
      throw std::runtime_error("driver: log base table update failed");
  }
  reg_end_[pidx] = hi;
  reg_total_ += hi - lo;
  reg_ns_ += tk::now_ns() - t0;
  DTRACE("pinned log of partition %u: [%lu, %lu)", pidx, (unsigned long)lo, (unsigned long)hi);
}

void MainDriver::launch_group(const int* slots, const int64_t* rows, const size_t* voffs, int n, const SlotView& v,
                              hipStream_t stream, int dst_dt, void* const* dsts, int64_t row, const float* shift,
                              const float* scale) {
  if (v.kind == uint32_t(tk::kPackGatherFixed))
    eng_->collate_gather_group(slots, n, stream, v.src_dtype, dsts, dst_dt, rows, int64_t(v.row_bytes), bases_dev_,
                               shift, scale);
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
  if (v.kind != uint32_t(tk::kPackRecordSpan) && ext_n_) {  // before the collate: its event covers the copy
    const int slot = int(v.g);
    const SlotView* vs[1] = {&v};
    copy_extras(&slot, vs, 1, stream);
  }
  bool record;
  note_handed(v.g, stream, &record);
  if (!record && coalesce_wait_ns_ > 0 && coalesce_ > 1) {
    // adaptive coalescing decides from the latest launch's completion: give this one its event
    handed_.back().ev = true;
    unevented_ = 0;
    ++events_;
    record = true;
  }
  if (record) last_ev_slot_ = v.g;
  if (v.kind == uint32_t(tk::kPackRecordSpan)) {
    const int slot = int(v.g);
    const SlotView* vs[1] = {&v};
    void* d = dst;
    int64_t pe;
    launch_span(&slot, vs, 1, stream, dst_dt, &d, shift, scale, record, &pe);
    handed_.back().perr = pe;
    handed_.back().span = true;
    last_perr_ = pe;
    return;
  }
  if (v.kind == uint32_t(tk::kPackGatherFixed)) {
    const int slot = int(v.g);
    const int64_t rows = v.n_rows;
    void* d = dst;
    eng_->collate_gather_group(&slot, 1, stream, v.src_dtype, &d, dst_dt, &rows, int64_t(v.row_bytes), bases_dev_,
                               shift, scale, record);
    return;
  }
  eng_->collate_fixed(int(v.g), stream, v.values_offset, v.src_dtype, dst, dst_dt, v.n_rows, row, shift, scale,
                      record);
}

void MainDriver::collate_varlen(const SlotView& v, hipStream_t stream, int dst_dt, void* out, int64_t L, double pad,
                                int64_t* lengths, uint8_t* mask) {
  bool record;
  if (row_span_kind(v.kind)) {
    // decoded from the logs on the user's stream, its own completion event
    if (stream != last_stream_) {
      cover_handed();
      last_stream_ = stream;
    }
    const int slot = int(v.g);
    const SlotView* vs[1] = {&v};
    void* outs[1] = {out};
    const int64_t Ls[1] = {L};
    int64_t* lens[1] = {lengths};
    uint8_t* masks[1] = {mask};
    int64_t pe;
    launch_row_span(&slot, vs, 1, stream, dst_dt, pad, outs, Ls, lens, masks, true, &pe);
    span_group_handed(&slot, 1, stream, &pe, {}, 1);
    last_perr_ = pe;
    return;
  }
  if (v.kind == tk::kPackJsonText) {
    const int64_t idx = next_err_word();
    note_handed(v.g, stream, &record);
    handed_.back().perr = idx;
    eng_->collate_json(int(v.g), stream, v.values_offset, out, dst_dt, v.n_rows, L, pad, lengths, mask,
                       perr_dev_ + idx, record);
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
  if (!record) {  // copy_raw always records the slot's completion event
    handed_.back().ev = true;
    unevented_ = 0;
    ++events_;
  }
  eng_->copy_raw(int(v.g), stream, 0, dst, size_t(v.payload_bytes));
}

void MainDriver::deliver(const SlotView& v) { set_delivered(v); }

void MainDriver::set_delivered(const SlotView& v) {
  delivered_ = v.wms;
  const bool checked = v.kind == tk::kPackJsonText || v.kind == tk::kPackRecordSpan || row_span_kind(v.kind);
  delivered_perr_ = checked ? (v.perr >= 0 ? v.perr : last_perr_) : -1;
}

void MainDriver::ensure_status() {
  if (perr_host_) return;
  void* h = nullptr;
  if (hipHostMalloc(&h, kErrWords * sizeof(int32_t), hipHostMallocMapped) != hipSuccess)
    throw std::runtime_error("driver: hipHostMalloc of the status words failed");
  perr_host_ = static_cast<int32_t*>(h);
  void* d = nullptr;
  if (hipHostGetDevicePointer(&d, h, 0) != hipSuccess) throw std::runtime_error("driver: hipHostGetDevicePointer failed");
  perr_dev_ = static_cast<int32_t*>(d);
  if (perr_state_.empty()) perr_state_.assign(size_t(kErrWords), 1);
  if (hipHostMalloc(&h, kErrWords * 4 * sizeof(int32_t), hipHostMallocMapped) != hipSuccess)
    throw std::runtime_error("driver: hipHostMalloc of the JSON width words failed");
  jinfo_host_ = static_cast<int32_t*>(h);
  std::memset(jinfo_host_, 0, kErrWords * 4 * sizeof(int32_t));
  if (hipHostGetDevicePointer(&d, h, 0) != hipSuccess) throw std::runtime_error("driver: hipHostGetDevicePointer failed");
  jinfo_dev_ = static_cast<int32_t*>(d);
  jrows_.assign(size_t(kErrWords), {});
  jparsed_.assign(size_t(kErrWords), 0);
}

int64_t MainDriver::next_err_word() {
  ensure_status();
  // an error word is reused after kErrWords launches; its batch was checked long before
  // (fenced batches are checked in order and the ring holds far fewer slots)
  const int64_t idx = int64_t(perr_seq_++ % uint64_t(kErrWords));
  if (perr_state_[size_t(idx)] == 0)
    throw std::runtime_error("driver: more than 4096 device-checked batches awaiting their kernels");
  perr_host_[idx] = -1;
  jinfo_host_[idx * 4 + 1] = 0;
  __atomic_store_n(jinfo_host_ + idx * 4 + 2, 0, __ATOMIC_RELEASE);
  jrows_[size_t(idx)].clear();
  jparsed_[size_t(idx)] = 0;
  perr_state_[size_t(idx)] = 0;
  if (!perr_msg_.empty()) perr_msg_[size_t(idx)].clear();
  return idx;
}

void MainDriver::ensure_partials() {
  if (part_host_) return;
  void* h = nullptr;
  if (hipHostMalloc(&h, size_t(kErrWords * kPartials) * sizeof(uint32_t), hipHostMallocMapped) != hipSuccess)
    throw std::runtime_error("driver: hipHostMalloc of the partial CRC words failed");
  part_host_ = static_cast<uint32_t*>(h);
  void* d = nullptr;
  if (hipHostGetDevicePointer(&d, h, 0) != hipSuccess) throw std::runtime_error("driver: hipHostGetDevicePointer failed");
  part_dev_ = static_cast<uint32_t*>(d);
  perr_msg_.assign(size_t(kErrWords), std::string());
}

void MainDriver::launch_span(const int* slots, const SlotView* const* views, int n, hipStream_t stream, int dst_dt,
                             void* const* dsts, const float* shift, const float* scale, bool record_last,
                             int64_t* perrs) {
  if (!broker_) throw std::runtime_error("driver: device decode needs the synthetic broker");
  ensure_partials();
  const SlotView& v0 = *views[0];
  SpanLaunch a{};
  a.row_elems = v0.max_row_len;
  const int ssz = dtype_size(v0.src_dtype), dsz = dtype_size(dst_dt);
  const int per = ssz > 0 ? 16 / ssz : 1;
  bool vec = ssz > 0 && a.row_elems % per == 0 && (a.row_elems * dsz) % 16 == 0;
  for (int k = 0; k < n; ++k) {
    vec = vec && reinterpret_cast<uintptr_t>(dsts[k]) % 16 == 0;
    perrs[k] = next_err_word();
    a.b[k].out = dsts[k];
    a.b[k].err = perr_dev_ + perrs[k];
    a.b[k].partials = part_dev_ + perrs[k] * kPartials;
    const SlotView& v = *views[k];
    if (v.extras_n && k < ext_n_ && ext_dsts_[k]) {  // key / timestamp columns ride in the same kernel
      a.b[k].ext_out = ext_dsts_[k];
      a.b[k].ext_off = v.extras_offset;
      a.b[k].ext_words = v.n_rows * v.extras_n;
    }
  }
  ext_n_ = 0;
  a.vec_store = vec ? 1 : 0;
  a.burst = span_burst_;  // loads a wave keeps in flight (span_decode.hip stage 1)
  int launches = 0;
  for (int k = 0; k < n; ++k) {
    const SlotView& v = *views[k];
    const auto* sg = reinterpret_cast<const tk::SpanSeg*>(ring_->payload(uint32_t(v.g)) + v.values_offset);
    for (uint32_t i = 0; i < v.n_segs; ++i) {
      constexpr uint32_t kWhole = tk::kSegCrcFirst | tk::kSegCrcLast;
      if ((sg[i].flags & tk::kSegCrc) && (sg[i].flags & kWhole) != kWhole && i >= uint32_t(kPartials))
        throw std::runtime_error("driver: a batch splits RecordBatches into more than 512 device segments");
      if (a.n_seg == kMaxLaunchSegs) {
        if (mirror_) mirror_->before(stream);
        eng_->collate_span(slots, n, stream, a, v0.src_dtype, dst_dt, shift, scale, false);
        if (mirror_) mirror_->after(stream);
        ++launches;
        a.n_seg = 0;
      }
      SpanDevSeg& d = a.s[a.n_seg++];
      d.src = seg_src(sg[i]);
      d.log_pos = sg[i].log_pos;
      d.len = sg[i].len;
      d.flags = sg[i].flags;
      d.crc = sg[i].crc;
      d.row_begin = sg[i].row_begin;
      d.row_end = sg[i].row_end;
      d.batch = uint16_t(k);
      d.seg = uint16_t(i);
    }
  }
  if (mirror_) mirror_->before(stream);
  eng_->collate_span(slots, n, stream, a, v0.src_dtype, dst_dt, shift, scale, record_last);
  if (mirror_) mirror_->after(stream);
  (void)launches;
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
  ensure_partials();
  // staging per batch: the row descriptors, then one region per segment (row texts rounded up to
  // 16 bytes, or the float32 values of the rows the worker parsed)
  constexpr uint64_t kA = 256;
  auto up = [](uint64_t x, uint64_t a) { return (x + a - 1) / a * a; };
  uint64_t batch_bytes[kMaxGroup], total = 0;
  for (int k = 0; k < n; ++k) {
    const SlotView& v = *views[k];
    const uint8_t* pay = ring_->payload(uint32_t(v.g));
    const auto* sg = reinterpret_cast<const tk::SpanSeg*>(pay + v.values_offset);
    const auto* rows = reinterpret_cast<const tk::JsonSpanRow*>(pay);
    uint64_t b = up(uint64_t(v.n_rows) * sizeof(JsonRowDesc), kA);
    for (uint32_t i = 0; i < v.n_segs; ++i) {
      const uint64_t nr = sg[i].row_end - sg[i].row_begin;
      if (sg[i].flags & tk::kSegHostRows) {
        for (uint32_t r = sg[i].row_begin; r < sg[i].row_end; ++r) {
          int64_t c = rows[r].count;
          if (v.trunc_len >= 0 && c > v.trunc_len) c = v.trunc_len;
          b += up(uint64_t(c < 0 ? 0 : c) * 4, 16);
        }
        b = up(b, kA);
      } else {
        b += up(up(sg[i].len, 16) + 16 * nr, kA);
      }
    }
    batch_bytes[k] = b;
    total += b;
  }
  // device-counted batches: two zeroed counter words each at the front of the group's region
  bool devc = false;
  for (int k = 0; k < n; ++k) devc = devc || (views[k]->flags & tk::kSlotDevCount) != 0;
  const uint64_t ctr_bytes = devc ? kA : 0;
  const uint64_t base = stage_alloc(total + ctr_bytes);
  if (devc && hipMemsetAsync(stage_dev_ + base, 0, ctr_bytes, stream) != hipSuccess)
    throw std::runtime_error("driver: hipMemsetAsync of the JSON counters failed");
  JsonStageLaunch a{};
  a.burst = span_burst_;
  JsonGroupArgs ga{};
  ga.n = n;
  ga.pad = float(pad);
  ga.err_tag = tk::kSpanParseErrBit;
  ga.mult = json_mult_;
  uint64_t off = base + ctr_bytes;
  for (int k = 0; k < n; ++k) {
    const SlotView& v = *views[k];
    perrs[k] = next_err_word();
    JsonStageBatch& b = a.b[k];
    if (v.flags & tk::kSlotDevCount) {
      b.ctr = reinterpret_cast<int32_t*>(stage_dev_ + base) + 4 * k;
      ga.ctr[k] = b.ctr;
      ga.info[k] = jinfo_dev_ + perrs[k] * 4;
    }
    b.desc = reinterpret_cast<JsonRowDesc*>(stage_dev_ + off);
    const uint64_t dbytes = up(uint64_t(v.n_rows) * sizeof(JsonRowDesc), kA);
    b.stage = stage_dev_ + off + dbytes;
    b.err = perr_dev_ + perrs[k];
    b.partials = part_dev_ + perrs[k] * kPartials;
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
    off += batch_bytes[k];
  }
  for (int k = 0; k < n; ++k) {
    const SlotView& v = *views[k];
    const uint8_t* pay = ring_->payload(uint32_t(v.g));
    const auto* sg = reinterpret_cast<const tk::SpanSeg*>(pay + v.values_offset);
    const auto* rows = reinterpret_cast<const tk::JsonSpanRow*>(pay);
    uint64_t soff = 0;  // offset in the batch's staging area (after its descriptors)
    for (uint32_t i = 0; i < v.n_segs; ++i) {
      constexpr uint32_t kWhole = tk::kSegCrcFirst | tk::kSegCrcLast;
      if ((sg[i].flags & tk::kSegCrc) && (sg[i].flags & kWhole) != kWhole && i >= uint32_t(kPartials))
        throw std::runtime_error("driver: a batch splits RecordBatches into more than 512 device segments");
      if (a.n_seg == kMaxLaunchSegs) {
        if (mirror_) mirror_->before(stream);
        eng_->collate_json_stage(slots, n, stream, a);
        if (mirror_) mirror_->after(stream);
        a.n_seg = 0;
      }
      SpanDevSeg& d = a.s[a.n_seg++];
      const bool host = (sg[i].flags & tk::kSegHostRows) != 0;
      d.src = host ? nullptr : seg_src(sg[i]);
      d.log_pos = sg[i].log_pos;
      d.len = sg[i].len;
      d.flags = sg[i].flags;
      d.crc = sg[i].crc;
      d.row_begin = sg[i].row_begin;
      d.row_end = sg[i].row_end;
      d.batch = uint16_t(k);
      d.seg = uint16_t(i);
      d.stage_off = uint32_t(soff);
      const uint64_t nr = sg[i].row_end - sg[i].row_begin;
      if (host) {
        for (uint32_t r = sg[i].row_begin; r < sg[i].row_end; ++r) {
          int64_t c = rows[r].count;
          if (v.trunc_len >= 0 && c > v.trunc_len) c = v.trunc_len;
          soff += up(uint64_t(c < 0 ? 0 : c) * 4, 16);
        }
        soff = up(soff, kA);
      } else {
        soff += up(up(sg[i].len, 16) + 16 * nr, kA);
      }
    }
  }
  if (mirror_) mirror_->before(stream);
  eng_->collate_json_stage(slots, n, stream, a);
  if (mirror_) mirror_->after(stream);
  // the parse: a block per row over the staged texts, on the same stream
  launch_json_group(ga, dst_dt, stream);
  if (record_last) eng_->record_done(slots[n - 1], stream);
}

void MainDriver::launch_var_span(const int* slots, const SlotView* const* views, int n, hipStream_t stream,
                                 int dst_dt, double pad, void* const* outs, const int64_t* Ls,
                                 int64_t* const* lengths, uint8_t* const* masks, bool record_last, int64_t* perrs) {
  if (!broker_) throw std::runtime_error("driver: device decode needs the synthetic broker");
  ensure_partials();
  VarSpanLaunch a{};
  a.burst = span_burst_;
  for (int k = 0; k < n; ++k) {
    perrs[k] = next_err_word();
    VarSpanBatch& b = a.b[k];
    b.out = outs[k];
    b.L = Ls[k];
    b.lengths = lengths[k];
    b.mask = masks[k];
    b.err = perr_dev_ + perrs[k];
    b.partials = part_dev_ + perrs[k] * kPartials;
    b.trunc_len = views[k]->trunc_len;
    // vector stores of a 16-byte source group (16 / ssz elements of dsz bytes): rows and groups aligned
    const int ssz = dtype_size(views[0]->src_dtype), dsz = dtype_size(dst_dt);
    const int64_t gbytes = ssz > 0 ? int64_t(16 / ssz) * dsz : 0;
    b.reserved = (gbytes >= 16 && gbytes % 16 == 0 && reinterpret_cast<uintptr_t>(outs[k]) % 16 == 0 &&
                  (Ls[k] * dsz) % 16 == 0) ? 1 : 0;
  }
  const int src_dt = views[0]->src_dtype;
  auto flush = [&](bool record) {
    for (int k = 0; k < n; ++k) {
      a.b[k].slot = eng_->slot_src(slots[k], stream);  // DMA mode: after the slot's copy
      a.b[k].rows = reinterpret_cast<const tk::JsonSpanRow*>(a.b[k].slot);
    }
    a.tabs = eng_->span_tables();
    if (mirror_) mirror_->before(stream);
    tkh::launch_var_span(a, src_dt, dst_dt, pad, stream);
    if (mirror_) mirror_->after(stream);
    if (record) eng_->record_done(slots[n - 1], stream);
  };
  for (int k = 0; k < n; ++k) {
    const SlotView& v = *views[k];
    if (v.src_dtype != src_dt) throw std::invalid_argument("driver: a var-len group mixes element dtypes");
    const auto* sg = reinterpret_cast<const tk::SpanSeg*>(ring_->payload(uint32_t(v.g)) + v.values_offset);
    for (uint32_t i = 0; i < v.n_segs; ++i) {
      constexpr uint32_t kWhole = tk::kSegCrcFirst | tk::kSegCrcLast;
      if ((sg[i].flags & tk::kSegCrc) && (sg[i].flags & kWhole) != kWhole && i >= uint32_t(kPartials))
        throw std::runtime_error("driver: a batch splits RecordBatches into more than 512 device segments");
      if (a.n_seg == kMaxLaunchSegs) {
        flush(false);
        a.n_seg = 0;
      }
      SpanDevSeg& d = a.s[a.n_seg++];
      d = SpanDevSeg{};
      d.src = (sg[i].flags & tk::kSegHostRows) ? nullptr : seg_src(sg[i]);
      d.log_pos = sg[i].log_pos;
      d.len = sg[i].len;
      d.flags = sg[i].flags;
      d.crc = sg[i].crc;
      d.row_begin = sg[i].row_begin;
      d.row_end = sg[i].row_end;
      d.batch = uint16_t(k);
      d.seg = uint16_t(i);
    }
  }
  flush(record_last);
}

const uint8_t* MainDriver::seg_src(const tk::SpanSeg& sg) {
  const uint8_t* log = broker_->log_base(sg.pidx);  // pinned: device address == host address
  // a ring log (KafkaBridge replica) writes over its chunks: an HBM mirror of them would go stale,
  // so its segments are read zero-copy
  if (mirror_ && broker_->part(sg.pidx).ring_bytes.load(std::memory_order_relaxed) == 0) {
    // pin ahead of the segment so the mirror can copy (and prefetch) whole chunks
    const auto& part = broker_->part(sg.pidx);
    ensure_log(sg.pidx, std::min<uint64_t>(part.log_capacity, sg.log_pos + mirror_->span_bytes()));
    const uint64_t written = part.log_end_pos.load(std::memory_order_acquire);
    const uint8_t* m = mirror_->map(sg.pidx, sg.log_pos, sg.len, log, std::min<uint64_t>(reg_end_[sg.pidx], written));
    if (m) return m;
  }
  return log + sg.log_pos;
}

void MainDriver::enable_mirror(uint64_t chunk_bytes, int chunks_per_partition) {
  if (!broker_) throw std::runtime_error("DeviceLoader h2d='dma' device decode needs the synthetic broker");
  mirror_ = std::make_unique<LogMirror>(eng_->device(), chunk_bytes, chunks_per_partition);
}

int64_t MainDriver::json_width(const SlotView& v, int64_t* n_host) {
  *n_host = 0;
  if (v.perr < 0 || !jinfo_host_) throw std::logic_error("driver: json_width of a batch without a parse launch");
  const int32_t* info = jinfo_host_ + v.perr * 4;
  // the parse kernel's first block of the batch reports the width: usually long done (the batch was
  // parsed ahead), else within one kernel's latency
  const int64_t t0 = tk::now_ns();
  for (int spin = 0; __atomic_load_n(info + 2, __ATOMIC_ACQUIRE) == 0; ++spin) {
    if (spin < 4096) {
      tk::cpu_relax();
      continue;
    }
    if (tk::now_ns() - t0 > 60'000'000'000LL)
      throw std::runtime_error("driver: the JSON parse kernel did not report a batch width within 60 s");
    timespec ts{0, 20000};
    nanosleep(&ts, nullptr);
  }
  *n_host = __atomic_load_n(info + 1, __ATOMIC_ACQUIRE);
  return __atomic_load_n(info, __ATOMIC_ACQUIRE);
}

void MainDriver::json_parse_host_rows(int64_t g, int64_t pe) {
  if (jparsed_[size_t(pe)]) return;
  jparsed_[size_t(pe)] = 1;
  // the rows the device found not simple are the device-counted rows json_scan_simple rejects;
  // parse them as the worker would have (parse_json_f32: Python's float() of each number)
  const tk::SlotHeader* h = ring_->slot(uint32_t(g));
  const uint8_t* pay = ring_->payload(uint32_t(g));
  const auto* rows = reinterpret_cast<const tk::JsonSpanRow*>(pay);
  const auto* sg = reinterpret_cast<const tk::SpanSeg*>(pay + h->values_offset);
  auto& out = jrows_[size_t(pe)];
  for (uint32_t i = 0; i < h->n_segs; ++i) {
    if (sg[i].flags & tk::kSegHostRows) continue;
    const uint8_t* log = broker_->log_base(sg[i].pidx);
    for (uint32_t r = sg[i].row_begin; r < sg[i].row_end && r < h->n_rows; ++r) {
      const tk::JsonSpanRow& d = rows[r];
      if (d.count != tk::kJsonCountOnDevice || d.tlen < 0) continue;
      const char* txt = reinterpret_cast<const char*>(log + d.pos);
      if (tk::json_scan_simple(txt, size_t(d.tlen)) >= 0) continue;  // parsed on the device
      HostRow hr;
      hr.row = int64_t(r);
      hr.vals.resize(size_t(tk::json_count_bound(uint64_t(d.tlen))) + 1);
      const int64_t c = tk::parse_json_f32(txt, size_t(d.tlen), hr.vals.data(), int64_t(hr.vals.size()));
      if (c < 0) {
        // not a flat numeric JSON array: the batch is never committed (as a device parse error)
        int32_t expect = -1;
        __atomic_compare_exchange_n(perr_host_ + pe, &expect, tk::kSpanParseErrBit | int32_t(r), false,
                                    __ATOMIC_ACQ_REL, __ATOMIC_ACQUIRE);
        if (perr_state_[size_t(pe)] == 1) perr_state_[size_t(pe)] = 2;
        if (pe < int64_t(perr_msg_.size()) && perr_msg_[size_t(pe)].empty())
          perr_msg_[size_t(pe)] = "batch row " + std::to_string(r) + " is not a flat numeric JSON array";
        continue;
      }
      hr.count = int32_t(c);
      hr.vals.resize(size_t(c));
      out.push_back(std::move(hr));
    }
  }
}

void MainDriver::json_host_rows(const SlotView& v, void* out, int64_t L, int dst_dt, double pad, int64_t* lengths,
                                uint8_t* mask, hipStream_t stream) {
  if (v.perr < 0) return;
  if (!jparsed_[size_t(v.perr)]) json_parse_host_rows(v.g, v.perr);  // the slot is still held
  const int dsz = dtype_size(dst_dt);
  constexpr size_t kVals = 256;  // the values start 256 bytes after the row descriptor
  for (const HostRow& hr : jrows_[size_t(v.perr)]) {
    int64_t n_out = hr.count;
    if (v.trunc_len >= 0 && n_out > v.trunc_len) n_out = v.trunc_len;
    if (n_out > L) {
      // wider than the device count made the batch: cannot happen for a flat numeric array
      int32_t expect = -1;
      __atomic_compare_exchange_n(perr_host_ + v.perr, &expect, tk::kSpanParseErrBit | int32_t(hr.row), false,
                                  __ATOMIC_ACQ_REL, __ATOMIC_ACQUIRE);
      if (perr_state_[size_t(v.perr)] == 1) perr_state_[size_t(v.perr)] = 2;
      continue;
    }
    const size_t need = kVals + hr.vals.size() * sizeof(float) + 16;
    if (need > patch_cap_) {
      if (patch_dev_ && hipFree(patch_dev_) != hipSuccess) throw std::runtime_error("driver: hipFree failed");
      patch_dev_ = nullptr;
      patch_cap_ = std::max<size_t>(need, size_t(1) << 20);
      if (hipMalloc(&patch_dev_, patch_cap_) != hipSuccess) throw std::runtime_error("driver: hipMalloc failed");
    }
    const tk::JsonRowDesc d{0, -1, hr.count, int32_t(n_out)};
    if (hipMemcpyAsync(patch_dev_, &d, sizeof(d), hipMemcpyHostToDevice, stream) != hipSuccess ||
        (!hr.vals.empty() && hipMemcpyAsync(patch_dev_ + kVals, hr.vals.data(), hr.vals.size() * sizeof(float),
                                            hipMemcpyHostToDevice, stream) != hipSuccess))
      throw std::runtime_error("driver: hipMemcpyAsync of a host-parsed JSON row failed");
    launch_json_rows(reinterpret_cast<const tk::JsonRowDesc*>(patch_dev_), patch_dev_ + kVals,
                     static_cast<uint8_t*>(out) + hr.row * L * dsz, dst_dt, 1, L, pad, lengths ? lengths + hr.row : nullptr,
                     mask ? mask + hr.row * L : nullptr, nullptr, stream);
    // the descriptor and values are read before the next row's copies overwrite them
    if (hipStreamSynchronize(stream) != hipSuccess) throw std::runtime_error("driver: hipStreamSynchronize failed");
  }
}

void MainDriver::span_group_handed(const int* slots, int n, hipStream_t ks, const int64_t* perrs,
                                   std::vector<std::shared_ptr<void>>&& handles, size_t first) {
  for (int k = 0; k < n; ++k) handed_.push_back(Handed{slots[k], k == n - 1, perrs[k], true});
  handed_.back().stage_end = stage_last_end_;  // 0 unless a JSON group just took a staging region
  stage_last_end_ = 0;
  last_ev_slot_ = slots[n - 1];
  unevented_ = 0;
  ++events_;
  if (n > 1) ++groups_;
  for (size_t k = first; k < size_t(n); ++k) {
    SlotView& v = staged_[group_idx_[k - first]];
    v.perr = perrs[k];
    v.pre = true;
    v.pre_stream = ks;
    v.pre_event_slot = slots[n - 1];
    v.pre_out = std::move(handles[k - first]);
  }
}

void MainDriver::check_span(int64_t g, int64_t pe) {
  const tk::SlotHeader* h = ring_->slot(uint32_t(g));
  const auto* sg = reinterpret_cast<const tk::SpanSeg*>(ring_->payload(uint32_t(g)) + h->values_offset);
  // a whole RecordBatch failed its CRC on the device (segment index), or a JSON row its parse
  const int32_t dev = __atomic_load_n(perr_host_ + pe, __ATOMIC_ACQUIRE);
  int32_t bad = dev >= tk::kSpanParseErrBit ? -1 : dev;
  const uint32_t* part = part_host_ + pe * kPartials;
  uint32_t acc = 0;
  for (uint32_t i = 0; i < h->n_segs && bad < 0; ++i) {
    const uint32_t f = sg[i].flags;
    constexpr uint32_t kWhole = tk::kSegCrcFirst | tk::kSegCrcLast;
    if (!(f & tk::kSegCrc) || (f & kWhole) == kWhole) continue;
    const uint32_t crc_len = sg[i].len - ((f & tk::kSegCrcFirst) ? 21u : 0u);
    if (f & tk::kSegCrcFirst) acc = 0;
    acc = tk::crc32c_shift_raw(acc, crc_len) ^ __atomic_load_n(part + i, __ATOMIC_ACQUIRE);
    if ((f & tk::kSegCrcLast) && (acc ^ 0xFFFFFFFFu) != sg[i].crc) bad = int32_t(i);
  }
  if (bad < 0) {
    if (dev >= tk::kSpanParseErrBit)
      perr_msg_[size_t(pe)] = "batch row " + std::to_string(dev & ~tk::kSpanParseErrBit) +
                              " is not a flat numeric JSON array (device parse from the log)";
    return;
  }
  // the RecordBatch of segment `bad`: walk back to its first segment for its base offset
  uint32_t i = uint32_t(bad);
  while (i > 0 && !(sg[i].flags & tk::kSegCrcFirst)) --i;
  const uint8_t* rb = broker_->log_base(sg[i].pidx) + sg[i].log_pos;
  int64_t base = 0;
  for (int b = 0; b < 8; ++b) base = (base << 8) | int64_t(rb[b]);
  perr_msg_[size_t(pe)] = "Record batch at offset " + std::to_string(base) + " of partition index " +
                          std::to_string(sg[i].pidx) + " failed CRC check (verified on the device)";
  __atomic_store_n(perr_host_ + pe, bad, __ATOMIC_RELEASE);
}

void MainDriver::stage_ready(int extra) {
  if (ls_) return;
  while (int(staged_.size()) < prefetch_ + extra) {
    const int r = poll_one(false, 0);
    if (r <= 0) break;  // -3 is reported by next_slot
  }
}

size_t MainDriver::json_group_extend() {
  group_idx_.clear();
  if (coalesce_ <= 1 || (last.kind != uint32_t(tk::kPackJsonText) && !row_span_kind(last.kind)))
    return 0;
  uint64_t bytes = last.span_bytes;
  for (size_t i = 0; i < staged_.size() && int(1 + group_idx_.size()) < coalesce_; ++i) {
    const SlotView& v = staged_[i];
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
  if (row_span_kind(last.kind)) {
    // decoded on the next decode stream (outputs allocated there, torch_step.cpp); the user's
    // stream waits for the group's completion
    int slots[kMaxGroup];
    const SlotView* vs[kMaxGroup];
    for (int k = 0; k < n; ++k) {
      vs[k] = k == 0 ? &last : &staged_[group_idx_[size_t(k - 1)]];
      slots[k] = int(vs[k]->g);
    }
    cover_handed();
    hipStream_t ks = next_decode_stream();
    ++span_launches_;
    last_stream_ = ks;
    int64_t perrs[kMaxGroup];
    launch_row_span(slots, vs, n, ks, dst_dt, pad, outs, Ls, lengths, masks, true, perrs);
    last.perr = perrs[0];
    span_group_handed(slots, n, ks, perrs, std::move(handles), 1);
    eng_->stream_wait_done(slots[n - 1], stream);
    waited_ev_slot_ = slots[n - 1];
    waited_stream_ = stream;
    group_idx_.clear();
    return;
  }
  int slots[kMaxGroup];
  size_t voffs[kMaxGroup];
  int64_t rows[kMaxGroup], perr[kMaxGroup];
  int32_t* errs[kMaxGroup];
  for (int k = 0; k < n; ++k) {
    SlotView& v = k == 0 ? last : staged_[group_idx_[size_t(k - 1)]];
    slots[k] = int(v.g);
    voffs[k] = v.values_offset;
    rows[k] = v.n_rows;
    const int64_t idx = next_err_word();
    perr[k] = idx;
    errs[k] = perr_dev_ + idx;
    v.perr = idx;
  }
  if (stream != last_stream_) {
    cover_handed();
    last_stream_ = stream;
  }
  eng_->collate_json_group(slots, n, stream, voffs, rows, outs, Ls, lengths, masks, errs, pad, dst_dt);
  // one completion event (after the group kernel, on the last slot) releases every slot of the group
  for (int k = 0; k < n; ++k) handed_.push_back(Handed{slots[k], k == n - 1, perr[k]});
  last_ev_slot_ = slots[n - 1];
  unevented_ = 0;
  ++events_;
  if (n > 1) ++groups_;
  for (int k = 1; k < n; ++k) {
    SlotView& v = staged_[group_idx_[size_t(k - 1)]];
    v.pre = true;
    v.pre_stream = stream;
    v.pre_event_slot = slots[n - 1];
    v.pre_out = std::move(handles[size_t(k - 1)]);
  }
  group_idx_.clear();
}


void MainDriver::discard(const SlotView& v) {
  if (v.g < 0) return;
  eng_->wait_copy(int(v.g));
  ring_->main_release(uint32_t(v.g));
}

void MainDriver::add_finished(const std::vector<tk::Watermark>& wms) {
  for (const auto& w : wms) {
    auto it = pending_.find(w.pidx);
    if (it == pending_.end() || w.next_offset > it->second) pending_[w.pidx] = w.next_offset;
  }
}

void MainDriver::stage_finished(int64_t index, std::vector<tk::Watermark>&& wms) {
  if (ls_)
    ls_->finished(index, std::move(wms));
  else
    batch_committable(wms);
}

void MainDriver::batch_committable(const std::vector<tk::Watermark>& wms) {
  add_finished(wms);
  ++committable_batches_;
}

// Batches become committable in delivery order, so the first committable_batches_ finish times
// belong to the batches whose offsets the commit that just ran stored (durable) or dropped.
void MainDriver::settle_commit_latency(bool durable) {
  const int64_t now = tk::now_ns();
  for (; committable_batches_ > 0 && !finish_t_.empty(); --committable_batches_) {
    if (durable && commit_lat_ns_.size() < (1u << 20)) commit_lat_ns_.push_back(now - finish_t_.front());
    finish_t_.pop_front();
  }
  committable_batches_ = 0;
}

void MainDriver::finish_delivered(hipStream_t fence) {
  if (delivered_.empty()) return;
  finish_t_.push_back(tk::now_ns());
  if (finish_t_.size() > (1u << 20)) {  // manual mode that never commits: keep the queue bounded
    finish_t_.pop_front();
    if (committable_batches_ > 0) --committable_batches_;
  }
  const int64_t perr = delivered_perr_;
  delivered_perr_ = -1;
  if (perr >= 0 && !commit_on_device_) {
    // a device-parsed batch commits only once its kernel ran clean (read at slot release)
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

// Waits (wait=true) until every launched device-parse kernel completed and its slot was
// released, so each pending error word has been read.
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
    if (pe >= 0 && perr_state_[size_t(pe)] == 0) {
      if (!settled) {
        settle_parse_errors(wait);
        settled = true;
      }
      if (perr_state_[size_t(pe)] == 0) break;  // its kernel has not completed yet
    }
    if (pe >= 0 && perr_state_[size_t(pe)] == 2) {
      const int32_t row = __atomic_load_n(perr_host_ + pe, __ATOMIC_ACQUIRE);
      std::string where;
      for (const auto& w : std::get<2>(f))
        where += (where.empty() ? "" : ", ") + std::string("partition index ") + std::to_string(w.pidx) +
                 " offsets [" + std::to_string(w.first_offset) + ", " + std::to_string(w.next_offset) + ")";
      if (pe < int64_t(perr_msg_.size()) && !perr_msg_[size_t(pe)].empty())
        parse_error_ = perr_msg_[size_t(pe)] + " (batch: " + where + ")";
      else
        parse_error_ = "batch row " + std::to_string(row) +
                       " is not a flat numeric JSON array (device parse; batch: " + where + ")";
      break;  // never committed
    }
    stage_finished(std::get<1>(f), std::move(std::get<2>(f)));
    if (ev) event_pool_.push_back(ev);
    fenced_.pop_front();
  }
}

void MainDriver::set_worker_sink(uintptr_t table, int n_workers, int capacity) {
  if (!table || n_workers < 1 || capacity < 1) throw std::invalid_argument("driver: bad worker commit table");
  sink_table_ = reinterpret_cast<int64_t*>(table);
  sink_workers_ = n_workers;
  sink_cap_ = capacity;
  sink_index_.assign(size_t(n_workers), {});
}

void MainDriver::publish_to_workers() {
  std::vector<uint8_t> touched(size_t(sink_workers_), 0);
  const int64_t block = 1 + 2 * int64_t(sink_cap_);
  for (const auto& kv : pending_) {
    auto it = pidx_worker_.find(kv.first);
    if (it == pidx_worker_.end()) throw std::logic_error("driver: finished offsets of a partition no worker delivered");
    const uint32_t w = it->second;
    if (int(w) >= sink_workers_) throw std::logic_error("driver: worker index beyond the commit table");
    int64_t* b = sink_table_ + 2 * int64_t(sink_workers_) + int64_t(w) * block;
    auto& idx = sink_index_[w];
    auto e = idx.find(kv.first);
    if (e == idx.end()) {
      const int64_t k = __atomic_load_n(b, __ATOMIC_RELAXED);
      if (k >= sink_cap_) throw std::runtime_error("driver: worker commit table full");
      __atomic_store_n(b + 1 + 2 * k, int64_t(kv.first), __ATOMIC_RELAXED);
      __atomic_store_n(b + 2 + 2 * k, kv.second, __ATOMIC_RELAXED);
      __atomic_store_n(b, k + 1, __ATOMIC_RELEASE);  // the entry is complete before n covers it
      idx.emplace(kv.first, int(k));
    } else if (kv.second > __atomic_load_n(b + 2 + 2 * e->second, __ATOMIC_RELAXED)) {
      __atomic_store_n(b + 2 + 2 * e->second, kv.second, __ATOMIC_RELAXED);
    }
    touched[w] = 1;
  }
  for (int w = 0; w < sink_workers_; ++w)
    if (touched[size_t(w)]) __atomic_fetch_add(sink_table_ + 2 * w, int64_t(1), __ATOMIC_RELEASE);
}

// A replica's log bytes below the committed position are never read again (one group consumes
// it; the replicator punches them out of the files): unpin whole registered ranges below it, so
// the pages are freed and a long stream holds only its in-flight window pinned.  Every kernel that
// read them completed: a batch is committed only after its decode verdict.
void MainDriver::release_consumed() {
  commits_since_release_ = 0;
  for (const auto& kv : committed_) {
    const uint32_t pidx = kv.first;
    if (pidx >= reg_ranges_.size() || reg_ranges_[pidx].size() < 2) continue;  // keep the range being read
    auto& q = reg_ranges_[pidx];
    const uint64_t pos = broker_->position_of(pidx, kv.second);
    const uint8_t* base = broker_->log_base(pidx);
    bool moved = false;
    while (q.size() > 1 && q.front().second <= pos) {
      if (hipHostUnregister(q.front().first) != hipSuccess)
        throw std::runtime_error("driver: hipHostUnregister of a consumed log range failed");
      unpinned_bytes_ += q.front().second - uint64_t(static_cast<const uint8_t*>(q.front().first) - base);
      q.pop_front();
      moved = true;
    }
    if (moved)  // the replicator may now punch the bytes below the first range still pinned
      broker_->part(pidx).pin_floor.store(uint64_t(static_cast<const uint8_t*>(q.front().first) - base),
                                          std::memory_order_release);
  }
}

int MainDriver::commit_pending() {
  drain_fenced(false);
  if (pending_.empty()) return parse_error_.empty() ? 0 : -2;
  if (sink_table_) {
    // the workers' consumers commit (and log, and swallow CommitFailedError) asynchronously
    const int64_t t0 = tk::now_ns();
    publish_to_workers();
    for (const auto& kv : pending_) committed_[kv.first] = kv.second;
    pending_.clear();
    ++commits_;
    if (commit_ns_.size() < (1u << 20)) commit_ns_.push_back(tk::now_ns() - t0);
    settle_commit_latency(true);
    return parse_error_.empty() ? 1 : -2;
  }
  if (!broker_) throw std::runtime_error("DeviceLoader cannot commit: no group_id / broker");
  const int64_t t0 = tk::now_ns();
  entries_.clear();
  for (const auto& kv : pending_) entries_.push_back(tk::CommitEntry{kv.first, kv.second, std::string()});
  int status = 1;
  try {
    broker_->commit(group_, -1, 0, 0, entries_);
    for (const auto& kv : pending_) committed_[kv.first] = kv.second;
    ++commits_;
    if (release_consumed_ && ++commits_since_release_ >= 32) release_consumed();
  } catch (const tk::CommitFailed&) {
    ++commit_failures_;
    status = -1;
  }
  pending_.clear();
  if (commit_ns_.size() < (1u << 20)) commit_ns_.push_back(tk::now_ns() - t0);
  settle_commit_latency(status == 1);
  if (!parse_error_.empty()) return -2;  // the batches before the bad one were committed
  return status;
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
  prefetch_ready();
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
  if (!ls_ && coalesce_ > 1) {
    // stage what the workers already published, so a group can form (never blocks)
    while (int(staged_.size()) < prefetch_ + coalesce_) {
      const int r = poll_one(false, 0);
      if (r == -3) return -3;
      if (r <= 0) break;
    }
  }
  occ_handed_ += int64_t(handed_.size());
  occ_staged_ += int64_t(staged_.size());
  ++occ_samples_;
  const int r = next_slot(timeout_ms, &last);
  const int64_t t2 = tk::now_ns();
  ph_commit_ns_ += t1 - t0;
  ph_next_ns_ += t2 - t1;
  if (r < 0) return r;
  if (last.pre) {
    // collated by an earlier group launch; a consumer on another stream waits for that kernel
    if (last.pre_stream != stream && !(waited_ev_slot_ == last.pre_event_slot && waited_stream_ == stream)) {
      eng_->stream_wait_done(int(last.pre_event_slot), stream);
      waited_ev_slot_ = last.pre_event_slot;
      waited_stream_ = stream;
    }
    *pre_out = std::move(last.pre_out);
    set_delivered(last);
    prefetch_ready();
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
        const int r2 = poll_one(false, 0);
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
    for (size_t i : group_idx_) group_rows->push_back(staged_[i].n_rows);
  }
  return last.n_rows;
}

void MainDriver::ahead_begin(std::vector<int64_t>* rows) {
  rows->clear();
  group_idx_.clear();
  if (ahead_depth_ <= 0 || coalesce_ <= 1) return;
  const size_t want = size_t(prefetch_ + (ahead_depth_ + 1) * coalesce_);
  while (staged_.size() < want) {
    if (poll_one(false, 0) <= 0) break;  // nothing ready (an error is reported by next_slot)
  }
  int pre = 0;
  size_t i0 = staged_.size();
  for (size_t i = 0; i < staged_.size(); ++i) {
    const SlotView& v = staged_[i];
    if (v.g < 0) continue;
    if (v.pre)
      ++pre;
    else if (i0 == staged_.size())
      i0 = i;
  }
  if (pre >= ahead_depth_ * coalesce_ || i0 == staged_.size()) return;
  const SlotView& f = staged_[i0];
  const bool json = row_span_kind(f.kind);  // outputs sized per batch: no shape match needed
  if ((f.kind != uint32_t(tk::kPackRecordSpan) && !json) || f.n_rows == 0) return;
  uint64_t bytes = 0;
  bool capped = false;
  for (size_t i = i0; i < staged_.size() && int(group_idx_.size()) < coalesce_; ++i) {
    const SlotView& v = staged_[i];
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
  if (int(group_idx_.size()) < coalesce_ && !capped) {  // only full groups go ahead; the rest waits for the user
    group_idx_.clear();
    return;
  }
  for (size_t i : group_idx_) rows->push_back(staged_[i].n_rows);
}

void MainDriver::ahead_launch(int dst_dt, void* const* dsts, const float* shift, const float* scale,
                              std::vector<std::shared_ptr<void>>&& handles) {
  const int n = int(group_idx_.size());
  if (n < 1 || int(handles.size()) != n) throw std::invalid_argument("driver: ahead group does not match");
  const int64_t t0 = tk::now_ns();
  int slots[kMaxGroup];
  const SlotView* vs[kMaxGroup];
  for (int k = 0; k < n; ++k) {
    const SlotView& v = staged_[group_idx_[size_t(k)]];
    slots[k] = int(v.g);
    vs[k] = &v;
  }
  cover_handed();
  hipStream_t ks = next_decode_stream();
  ++span_launches_;
  last_stream_ = ks;
  int64_t perrs[kMaxGroup];
  launch_span(slots, vs, n, ks, dst_dt, dsts, shift, scale, true, perrs);
  for (int k = 0; k < n; ++k) handed_.push_back(Handed{slots[k], k == n - 1, perrs[k], true});
  last_ev_slot_ = slots[n - 1];
  unevented_ = 0;
  ++events_;
  ++groups_;
  ++ahead_groups_;
  for (int k = 0; k < n; ++k) {
    SlotView& v = staged_[group_idx_[size_t(k)]];
    v.perr = perrs[k];
    v.pre = true;
    v.pre_stream = ks;
    v.pre_event_slot = slots[n - 1];
    v.pre_out = std::move(handles[size_t(k)]);
  }
  group_idx_.clear();
  ph_launch_ns_ += tk::now_ns() - t0;
}

void MainDriver::ahead_launch_json(int dst_dt, double pad, void* const* outs, const int64_t* Ls,
                                   int64_t* const* lengths, uint8_t* const* masks,
                                   std::vector<std::shared_ptr<void>>&& handles) {
  const int n = int(group_idx_.size());
  if (n < 1 || int(handles.size()) != n) throw std::invalid_argument("driver: ahead group does not match");
  const int64_t t0 = tk::now_ns();
  int slots[kMaxGroup];
  const SlotView* vs[kMaxGroup];
  for (int k = 0; k < n; ++k) {
    vs[k] = &staged_[group_idx_[size_t(k)]];
    slots[k] = int(vs[k]->g);
  }
  cover_handed();
  hipStream_t ks = next_decode_stream();
  ++span_launches_;
  last_stream_ = ks;
  int64_t perrs[kMaxGroup];
  launch_row_span(slots, vs, n, ks, dst_dt, pad, outs, Ls, lengths, masks, true, perrs);
  span_group_handed(slots, n, ks, perrs, std::move(handles), 0);
  ++ahead_groups_;
  group_idx_.clear();
  ph_launch_ns_ += tk::now_ns() - t0;
}

// Appends to group_idx_ the staged batches right behind `last` that one kernel can collate with it.
void MainDriver::extend_group() {
  size_t i = group_idx_.empty() ? 0 : group_idx_.back() + 1;
  uint64_t bytes = last.span_bytes;
  for (size_t k : group_idx_) bytes += staged_[k].span_bytes;
  for (; i < staged_.size() && int(1 + group_idx_.size()) < coalesce_; ++i) {
    const SlotView& v = staged_[i];
    if (v.g < 0) continue;  // watermark-only slot: rides on the next delivered batch
    if (group_full(bytes, v)) group_capped_ = true;
    if (v.pre || v.kind != last.kind || v.src_dtype != last.src_dtype || v.max_row_len != last.max_row_len ||
        v.row_bytes != last.row_bytes || v.shape != last.shape || v.n_rows == 0 || group_capped_)
      return;
    bytes += v.span_bytes;
    group_idx_.push_back(i);
  }
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

void MainDriver::step_group_launch(hipStream_t stream, int dst_dt, void* const* dsts, int64_t row,
                                   const float* shift, const float* scale,
                                   std::vector<std::shared_ptr<void>>&& handles) {
  const int64_t t0 = tk::now_ns();
  const int n = 1 + int(group_idx_.size());
  if (int(handles.size()) != n - 1) throw std::invalid_argument("driver: group handles do not match the group");
  int slots[kMaxGroup];
  size_t voffs[kMaxGroup];
  int64_t rows[kMaxGroup];
  slots[0] = int(last.g);
  voffs[0] = last.values_offset;
  rows[0] = last.n_rows;
  for (int k = 1; k < n; ++k) {
    const SlotView& v = staged_[group_idx_[size_t(k - 1)]];
    slots[k] = int(v.g);
    voffs[k] = v.values_offset;
    rows[k] = v.n_rows;
  }
  if (last.kind == uint32_t(tk::kPackRecordSpan)) {
    // Device decode runs on two decode streams in turn: a group's kernel is PCIe-bound while it
    // loads and compute-bound in its CRC/extract tail, so the next group's loads overlap that
    // tail.  The outputs were allocated on the decode stream (torch_step.cpp: the caching
    // allocator orders their reuse against it, and knows the user's stream uses them); the
    // user's stream waits for the group's completion before it touches a batch of it.
    cover_handed();
    hipStream_t ks = next_decode_stream();
    ++span_launches_;
    last_stream_ = ks;
    int64_t perrs[kMaxGroup];
    const SlotView* vs[kMaxGroup];
    vs[0] = &last;
    for (int k = 1; k < n; ++k) vs[k] = &staged_[group_idx_[size_t(k - 1)]];
    launch_span(slots, vs, n, ks, dst_dt, dsts, shift, scale, true, perrs);
    last.perr = perrs[0];
    for (int k = 0; k < n; ++k) handed_.push_back(Handed{slots[k], k == n - 1, perrs[k], true});
    last_ev_slot_ = slots[n - 1];
    unevented_ = 0;
    ++events_;
    if (n > 1) ++groups_;
    for (int k = 1; k < n; ++k) {
      SlotView& v = staged_[group_idx_[size_t(k - 1)]];
      v.perr = perrs[k];
      v.pre = true;
      v.pre_stream = ks;
      v.pre_event_slot = slots[n - 1];
      v.pre_out = std::move(handles[size_t(k - 1)]);
    }
    eng_->stream_wait_done(slots[n - 1], stream);
    waited_ev_slot_ = slots[n - 1];
    waited_stream_ = stream;
  } else if (n == 1) {
    collate_fixed(last, stream, dst_dt, dsts[0], row, shift, scale);
  } else {
    if (stream != last_stream_) {
      cover_handed();
      last_stream_ = stream;
    }
    if (ext_n_) {
      const SlotView* vs[kMaxGroup];
      vs[0] = &last;
      for (int k = 1; k < n; ++k) vs[k] = &staged_[group_idx_[size_t(k - 1)]];
      copy_extras(slots, vs, n, stream);
    }
    launch_group(slots, rows, voffs, n, last, stream, dst_dt, dsts, row, shift, scale);
    // one completion event (after the group kernel, on the last slot) releases every slot of the group
    for (int k = 0; k < n; ++k) handed_.push_back(Handed{slots[k], k == n - 1});
    last_ev_slot_ = slots[n - 1];
    unevented_ = 0;
    ++events_;
    ++groups_;
    for (int k = 1; k < n; ++k) {
      SlotView& v = staged_[group_idx_[size_t(k - 1)]];
      v.pre = true;
      v.pre_stream = stream;
      v.pre_event_slot = slots[n - 1];
      v.pre_out = std::move(handles[size_t(k - 1)]);
    }
  }
  group_idx_.clear();
  set_delivered(last);
  prefetch_ready();
  ph_launch_ns_ += tk::now_ns() - t0;
  ++ph_steps_;
}

std::vector<std::pair<uint32_t, int64_t>> MainDriver::committed() const {
  std::vector<std::pair<uint32_t, int64_t>> v(committed_.begin(), committed_.end());
  std::sort(v.begin(), v.end());
  return v;
}

std::vector<std::pair<uint32_t, int64_t>> MainDriver::take_pending() {
  std::vector<std::pair<uint32_t, int64_t>> v(pending_.begin(), pending_.end());
  pending_.clear();
  settle_commit_latency(false);  // handed to Python (manual commit): not timed here
  return v;
}

void MainDriver::reset_stats() {
  commits_ = commit_failures_ = 0;
  fill_ns_ = fills_ = blocked_ns_ = blocked_calls_ = ready_age_ns_ = worker_idle_ns_ = worker_slot_wait_ns_ = 0;
  ph_commit_ns_ = ph_next_ns_ = ph_launch_ns_ = ph_steps_ = events_ = groups_ = 0;
  reg_ns_ = 0;
  reg_total_ = 0;
  rel_ns_ = released_ = polled_ = poll_ns_ = cwait_ns_ = 0;
  occ_handed_ = occ_staged_ = occ_samples_ = 0;
  ahead_groups_ = 0;
  fast_batches_ = fast_records_ = fast_ns_ = 0;
  commit_ns_.clear();
  commit_lat_ns_.clear();
  if (ls_) ls_->reset_stats();
}

}  // namespace tkh
