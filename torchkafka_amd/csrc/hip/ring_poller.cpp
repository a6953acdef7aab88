#include "ring_poller.h"

#include <algorithm>

namespace tkh {

RingPoller::RingPoller(std::shared_ptr<tk::Ring> ring, Engine* engine, LogPins* pins, CommitLedger* ledger,
                       tk::Broker* broker, bool in_order, int default_src_dt)
    : ring_(std::move(ring)),
      eng_(engine),
      pins_(pins),
      ledger_(ledger),
      broker_(broker),
      in_order_(in_order),
      default_src_dt_(default_src_dt) {
  cursor_.assign(ring_->n_workers(), 0);
  done_.assign(ring_->n_workers(), 0);
}

int RingPoller::poll(bool block, int64_t timeout_ms) {
  const int64_t t0 = block ? 0 : tk::now_ns();
  const int r = acquire(block, timeout_ms);
  if (!block) stats.poll_ns += tk::now_ns() - t0;
  if (r == 1) ++stats.polled;
  return r;
}

int RingPoller::acquire(bool block, int64_t timeout_ms) {
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
    if (h->flags & tk::kSlotEOS) done_.at(h->worker) = 1;
    stats.fill_ns += h->t_ready_ns - h->t_fill_start_ns;
    stats.ready_age_ns += tk::now_ns() - h->t_ready_ns;
    {
      // worker idle: from its previous publish to the start of this fill (waiting for a FREE
      // slot, plus its per-batch Python work)
      if (last_ready_.size() <= h->worker) last_ready_.resize(h->worker + 1, 0);
      int64_t& lr = last_ready_[h->worker];
      if (lr > 0 && h->t_fill_start_ns > lr) stats.worker_idle_ns += h->t_fill_start_ns - lr;
      stats.worker_slot_wait_ns += h->t_acquire_wait_ns;
      lr = h->t_ready_ns;
    }
    ++stats.fills;
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
    if (ledger_->worker_sink())
      for (uint32_t k = 0; k < h->n_parts; ++k) ledger_->note_worker(h->wm[k].pidx, h->worker);
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
        pins_->ensure(sg[i].pidx, std::min<uint64_t>(sg[i].log_pos + sg[i].len + 16, cap));
      }
    }
    if (v.kind == uint32_t(tk::kPackGatherFixed)) {
      if (!pins_->direct()) {
        error_ = "DeviceLoader: a worker produced a log-gather slot but direct mode is off";
        return -3;
      }
      // pin every log range this slot's rows live in before any kernel may read them
      for (uint32_t k = 0; k < h->n_parts; ++k) pins_->ensure(h->wm[k].pidx, h->log_end[k]);
    }
    eng_->h2d(int(g), ring_->payload(uint32_t(g)), v.payload_bytes);
    staged_.push_back(std::move(v));
    return 1;
  }
}

// Pull the headers of the slots the next acquisition will look at into this core's cache while
// the caller runs Python: they were written by worker processes on other cores, and reading them
// cold costs several cross-core transfers per batch.  Only READY slots are touched, so a worker
// still filling a slot never loses its lines.
void RingPoller::prefetch_ready() const {
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

int RingPoller::data_staged() const {
  int n = 0;
  for (const auto& v : staged_) n += v.g >= 0 ? 1 : 0;
  return n;
}

bool RingPoller::all_done() const {
  for (auto d : done_)
    if (!d) return false;
  return true;
}

bool RingPoller::pop(SlotView* out) {
  while (!staged_.empty()) {
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
    return true;
  }
  return false;
}

}  // namespace tkh
