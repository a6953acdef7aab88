// Device residency of the partition logs the decode kernels read.
//
// Device decode and h2d='direct' read record bytes straight out of the synthetic broker's
// shared-memory logs, so every byte range a slot references must be pinned and device-mapped
// (hipHostRegister, whole kChunk pieces) before its kernel is launched.  With h2d='dma' the
// kernels read an HBM mirror that the copy engines fill from those pinned pieces instead
// (log_mirror.h).  A replica log (KafkaBridge, tk::kReleaseConsumed) is unpinned piecewise below
// the committed position, so a long stream keeps only its in-flight window pinned.
//
// Registration runs ~13 GB/s of fresh shm pages on the MI355X host (register_probe2.log), i.e.
// ~5 ms per 64 MiB piece.  The retained backlog is pinned once, up front (pin_written); a log that
// keeps growing is pinned by a background thread that follows each partition's written end chunk
// by chunk, so the thread that launches kernels only waits when it outruns that thread.
#pragma once

#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <unordered_set>
#include <utility>
#include <vector>

#include "broker.h"
#include "engine.h"
#include "log_mirror.h"
#include "span.h"

namespace tkh {

class LogPins {
 public:
  static constexpr uint64_t kChunk = uint64_t(64) << 20;

  LogPins(Engine* engine, std::shared_ptr<tk::Broker> broker);  // broker may be null: nothing to pin
  ~LogPins();
  LogPins(const LogPins&) = delete;
  LogPins& operator=(const LogPins&) = delete;

  // Pins partition pidx's log up to `end` (and whatever is already written, in kChunk pieces): at
  // once when nothing is pinned yet, else by waiting for the pin thread, which is asked for it.
  void ensure(uint32_t pidx, uint64_t end);
  // The retained backlog of these partitions, pinned now instead of by the first batches.
  void pin_written(const std::vector<uint32_t>& pidxs);

  // h2d='direct': a device table of the logs' base addresses for the gather kernel.
  void enable_direct();
  bool direct() const { return bases_dev_ != nullptr; }
  const uint64_t* bases_dev() const { return bases_dev_; }
  // h2d='dma' with device decode: segments are read from an HBM mirror.
  void enable_mirror(uint64_t chunk_bytes, int chunks_per_partition, int copy_streams = 0, int wait = -1);
  LogMirror* mirror() { return mirror_.get(); }
  const LogMirror* mirror() const { return mirror_.get(); }
  // The address a decode kernel reads a segment from (mirror, else the pinned log); *hbm tells which.
  const uint8_t* seg_src(const tk::SpanSeg& sg, bool* hbm);

  // A commit stored these offsets: every 32 commits, unpin replica ranges wholly below them.
  void committed(const std::unordered_map<uint32_t, int64_t>& committed);

  // pinned end of partition pidx's log (device-mapped bytes [0, end))
  uint64_t pinned_end(uint32_t pidx) const {
    return pidx < n_parts_ ? reg_end_[pidx].load(std::memory_order_acquire) : 0;
  }

  uint64_t bytes_registered() const { return reg_total_.load(); }
  uint64_t bytes_unpinned() const { return unpinned_bytes_; }
  int64_t register_ns() const { return reg_ns_.load(); }       // registration time, any thread
  int64_t register_wait_ns() const { return wait_ns_.load(); }  // the launch thread waiting for it
  // registrations that first found their pages still registered by a pending deferred release
  uint64_t register_retries() const { return register_retries_.load(); }
  void reset_stats() {
    reg_total_ = 0;
    reg_ns_ = 0;
    wait_ns_ = 0;
    if (mirror_) mirror_->reset_stats();
  }

 private:
  void release_consumed(const std::unordered_map<uint32_t, int64_t>& committed);
  // registers [reg_end, roundup(max(end, written))) in kChunk pieces; false: nothing to do
  bool pin_some(uint32_t pidx, uint64_t end, bool one_piece);
  void pin_loop();

  Engine* eng_;
  std::shared_ptr<tk::Broker> broker_;
  uint64_t* bases_dev_ = nullptr;
  std::unique_ptr<LogMirror> mirror_;
  uint32_t n_parts_ = 0;
  // per pidx: bytes of its log pinned (and device-mapped); written by whoever registers
  std::unique_ptr<std::atomic<uint64_t>[]> reg_end_;
  // per pidx: pinned ranges (address, end position), unpinned once committed past or at teardown
  std::vector<std::deque<std::pair<void*, uint64_t>>> reg_ranges_;
  std::mutex reg_m_;  // reg_ranges_ and registration itself (one registration at a time)
  // the pin thread: follows the written end of every partition pinned so far, and serves demands
  std::thread pin_thread_;
  std::mutex pm_;
  std::condition_variable pcv_, done_cv_;
  std::unordered_set<uint32_t> tracked_;
  std::unordered_map<uint32_t, uint64_t> demand_;
  bool stop_ = false;
  std::string err_;
  bool release_consumed_ = false;
  uint64_t commits_since_release_ = 0;
  uint64_t unpinned_bytes_ = 0;
  std::atomic<uint64_t> reg_total_{0};
  std::atomic<int64_t> reg_ns_{0}, wait_ns_{0};
  std::atomic<uint64_t> register_retries_{0};
};

}  // namespace tkh
