// Commit ledger of the main-process step driver: finished offsets -> durable commits.
//
// The reference commits a batch's offsets once the training loop asked for the next one
// (/root/reference/src/auto_commit.py:55-58 -> kafka_dataset.py:128-130).  Here the driver
// decides WHEN a batch is finished (its decode verdict landed, the user's GPU work fenced, the
// ranks agreed); the ledger keeps WHAT is finished and stores it: highest next-offset per
// partition, merged until the next commit, then written into the synthetic broker's offset table
// (or published to the workers' consumers through the shared-memory WatermarkTable).  It also
// times each batch from the request that finished it to its offsets being durable.
#pragma once

#include <cstdint>
#include <deque>
#include <memory>
#include <string>
#include <unordered_map>
#include <utility>
#include <vector>

#include "broker.h"
#include "ring.h"

namespace tkh {

class CommitLedger {
 public:
  // broker may be null (no group_id: nothing to commit into unless a worker sink is set)
  CommitLedger(std::shared_ptr<tk::Broker> broker, uint32_t group);

  bool can_commit() const { return broker_ != nullptr || sink_table_ != nullptr; }
  // commit_sink='worker' (loader/commit_channel.py WatermarkTable): offsets go to the worker that
  // delivered each partition; its own consumer commits them as a group member.
  void set_worker_sink(uintptr_t table, int n_workers, int capacity);
  bool worker_sink() const { return sink_table_ != nullptr; }
  // partition -> the worker that delivers it (worker sink only)
  void note_worker(uint32_t pidx, uint32_t worker) { pidx_worker_[pidx] = worker; }

  // The user finished a batch (its commit latency starts now).
  void batch_finished();
  // Offsets of a finished batch, merged into the pending set (highest next-offset per partition).
  void add_finished(const std::vector<tk::Watermark>& wms);
  // A finished batch that passed every check: its offsets are pending and its latency is timed.
  void batch_committable(const std::vector<tk::Watermark>& wms) {
    add_finished(wms);
    ++committable_batches_;
  }
  bool has_pending() const { return !pending_.empty(); }

  // Stores every pending offset.  0 nothing to do, 1 committed, -1 CommitFailedError (dropped).
  int commit();
  // Manual mode: the pending offsets handed to Python (not timed here).
  std::vector<std::pair<uint32_t, int64_t>> take_pending();

  const std::unordered_map<uint32_t, int64_t>& committed_map() const { return committed_; }
  std::vector<std::pair<uint32_t, int64_t>> committed() const;
  uint64_t commits() const { return commits_; }
  uint64_t commit_failures() const { return commit_failures_; }
  const std::vector<int64_t>& commit_ns() const { return commit_ns_; }
  const std::vector<int64_t>& commit_latency_ns() const { return commit_lat_ns_; }
  void reset_stats();

 private:
  void settle_latency(bool durable);
  void publish_to_workers();

  std::shared_ptr<tk::Broker> broker_;
  uint32_t group_;
  std::unordered_map<uint32_t, int64_t> pending_;
  std::unordered_map<uint32_t, int64_t> committed_;
  std::vector<tk::CommitEntry> entries_;
  int64_t* sink_table_ = nullptr;  // WatermarkTable layout, see set_worker_sink
  int sink_workers_ = 0, sink_cap_ = 0;
  std::vector<std::unordered_map<uint32_t, int>> sink_index_;  // per worker: pidx -> entry
  std::unordered_map<uint32_t, uint32_t> pidx_worker_;
  uint64_t commits_ = 0, commit_failures_ = 0;
  std::vector<int64_t> commit_ns_;
  std::vector<int64_t> commit_lat_ns_;
  std::deque<int64_t> finish_t_;     // finish time of each finished batch not yet committed
  int64_t committable_batches_ = 0;  // of those, batches whose offsets are in pending_
};

}  // namespace tkh
