// Device residency of the partition logs the decode kernels read.
//
// Device decode and h2d='direct' read record bytes straight out of the synthetic broker's
// shared-memory logs, so every byte range a slot references must be pinned and device-mapped
// (hipHostRegister, whole kChunk pieces) before its kernel is launched.  With h2d='dma' the
// kernels read an HBM mirror that the copy engines fill from those pinned pieces instead
// (log_mirror.h).  A replica log (KafkaBridge, tk::kReleaseConsumed) is unpinned piecewise below
// the committed position, so a long stream keeps only its in-flight window pinned.
#pragma once

#include <cstdint>
#include <deque>
#include <memory>
#include <unordered_map>
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

  // Pins partition pidx's log up to `end` (and whatever is already written, in kChunk pieces).
  void ensure(uint32_t pidx, uint64_t end);
  // The retained backlog of these partitions, pinned now instead of by the first batches.
  void pin_written(const std::vector<uint32_t>& pidxs);

  // h2d='direct': a device table of the logs' base addresses for the gather kernel.
  void enable_direct();
  bool direct() const { return bases_dev_ != nullptr; }
  const uint64_t* bases_dev() const { return bases_dev_; }
  // h2d='dma' with device decode: segments are read from an HBM mirror.
  void enable_mirror(uint64_t chunk_bytes, int chunks_per_partition, int copy_streams = 0);
  LogMirror* mirror() { return mirror_.get(); }
  const LogMirror* mirror() const { return mirror_.get(); }
  // The address a decode kernel reads a segment from (mirror, else the pinned log); *hbm tells which.
  const uint8_t* seg_src(const tk::SpanSeg& sg, bool* hbm);

  // A commit stored these offsets: every 32 commits, unpin replica ranges wholly below them.
  void committed(const std::unordered_map<uint32_t, int64_t>& committed);

  uint64_t bytes_registered() const { return reg_total_; }
  uint64_t bytes_unpinned() const { return unpinned_bytes_; }
  int64_t register_ns() const { return reg_ns_; }
  void reset_stats() {
    reg_total_ = 0;
    reg_ns_ = 0;
  }

 private:
  void release_consumed(const std::unordered_map<uint32_t, int64_t>& committed);

  Engine* eng_;
  std::shared_ptr<tk::Broker> broker_;
  uint64_t* bases_dev_ = nullptr;
  std::unique_ptr<LogMirror> mirror_;
  std::vector<uint64_t> reg_end_;  // per pidx: bytes of its log pinned (and device-mapped)
  // per pidx: pinned ranges (address, end position), unpinned once committed past or at teardown
  std::vector<std::deque<std::pair<void*, uint64_t>>> reg_ranges_;
  bool release_consumed_ = false;
  uint64_t commits_since_release_ = 0;
  uint64_t unpinned_bytes_ = 0;
  uint64_t reg_total_ = 0;
  int64_t reg_ns_ = 0;
};

}  // namespace tkh
