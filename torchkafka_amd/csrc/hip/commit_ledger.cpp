#include "commit_ledger.h"

#include <algorithm>
#include <stdexcept>

namespace tkh {

CommitLedger::CommitLedger(std::shared_ptr<tk::Broker> broker, uint32_t group)
    : broker_(std::move(broker)), group_(group) {
  commit_ns_.reserve(1 << 16);
}

void CommitLedger::set_worker_sink(uintptr_t table, int n_workers, int capacity) {
  if (!table || n_workers < 1 || capacity < 1) throw std::invalid_argument("driver: bad worker commit table");
  sink_table_ = reinterpret_cast<int64_t*>(table);
  sink_workers_ = n_workers;
  sink_cap_ = capacity;
  sink_index_.assign(size_t(n_workers), {});
}

void CommitLedger::batch_finished() {
  finish_t_.push_back(tk::now_ns());
  if (finish_t_.size() > (1u << 20)) {  // manual mode that never commits: keep the queue bounded
    finish_t_.pop_front();
    if (committable_batches_ > 0) --committable_batches_;
  }
}

void CommitLedger::add_finished(const std::vector<tk::Watermark>& wms) {
  for (const auto& w : wms) {
    auto it = pending_.find(w.pidx);
    if (it == pending_.end() || w.next_offset > it->second) pending_[w.pidx] = w.next_offset;
  }
}

// Batches become committable in delivery order, so the first committable_batches_ finish times
// belong to the batches whose offsets the commit that just ran stored (durable) or dropped.
void CommitLedger::settle_latency(bool durable) {
  const int64_t now = tk::now_ns();
  for (; committable_batches_ > 0 && !finish_t_.empty(); --committable_batches_) {
    if (durable && commit_lat_ns_.size() < (1u << 20)) commit_lat_ns_.push_back(now - finish_t_.front());
    finish_t_.pop_front();
  }
  committable_batches_ = 0;
}

void CommitLedger::publish_to_workers() {
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

int CommitLedger::commit() {
  if (pending_.empty()) return 0;
  const int64_t t0 = tk::now_ns();
  int status = 1;
  if (sink_table_) {
    // the workers' consumers commit (and log, and swallow CommitFailedError) asynchronously
    publish_to_workers();
    for (const auto& kv : pending_) committed_[kv.first] = kv.second;
    ++commits_;
  } else {
    if (!broker_) throw std::runtime_error("DeviceLoader cannot commit: no group_id / broker");
    entries_.clear();
    for (const auto& kv : pending_) entries_.push_back(tk::CommitEntry{kv.first, kv.second, std::string()});
    try {
      broker_->commit(group_, -1, 0, 0, entries_);
      for (const auto& kv : pending_) committed_[kv.first] = kv.second;
      ++commits_;
    } catch (const tk::CommitFailed&) {
      ++commit_failures_;
      status = -1;
    }
  }
  pending_.clear();
  if (commit_ns_.size() < (1u << 20)) commit_ns_.push_back(tk::now_ns() - t0);
  settle_latency(status == 1);
  return status;
}

std::vector<std::pair<uint32_t, int64_t>> CommitLedger::take_pending() {
  std::vector<std::pair<uint32_t, int64_t>> v(pending_.begin(), pending_.end());
  pending_.clear();
  settle_latency(false);
  return v;
}

std::vector<std::pair<uint32_t, int64_t>> CommitLedger::committed() const {
  std::vector<std::pair<uint32_t, int64_t>> v(committed_.begin(), committed_.end());
  std::sort(v.begin(), v.end());
  return v;
}

void CommitLedger::reset_stats() {
  commits_ = commit_failures_ = 0;
  commit_ns_.clear();
  commit_lat_ns_.clear();
}

}  // namespace tkh
