#include "log_pins.h"

#include <algorithm>
#include <stdexcept>

namespace tkh {

static_assert(LogPins::kChunk == LogMirror::kRegAlign, "mirror copies split at the pin pieces");

LogPins::LogPins(Engine* engine, std::shared_ptr<tk::Broker> broker) : eng_(engine), broker_(std::move(broker)) {
  if (broker_) {
    reg_end_.assign(broker_->meta().max_partitions, 0);
    reg_ranges_.resize(broker_->meta().max_partitions);
    release_consumed_ = (broker_->flags() & tk::kReleaseConsumed) != 0;
  }
}

LogPins::~LogPins() {
  mirror_.reset();  // its copies read the pinned logs: before they are unregistered
  // the kernels that read the ranges completed (slots drained by the caller)
  bool any = false;
  for (auto& q : reg_ranges_) any = any || !q.empty();
  if (any) hipDeviceSynchronize();
  for (size_t pidx = 0; pidx < reg_ranges_.size(); ++pidx) {
    auto& q = reg_ranges_[pidx];
    for (auto& r : q) hipHostUnregister(r.first);
    if (!q.empty() && broker_) broker_->part(uint32_t(pidx)).pinned.fetch_sub(1, std::memory_order_acq_rel);
  }
  if (bases_dev_) hipFree(bases_dev_);
}

void LogPins::enable_direct() {
  if (!broker_) throw std::runtime_error("DeviceLoader h2d='direct' needs the synthetic broker (group_id + URL)");
  if (bases_dev_) return;
  const uint32_t np = broker_->meta().max_partitions;
  reg_end_.assign(np, 0);
  if (hipMalloc(reinterpret_cast<void**>(&bases_dev_), size_t(np) * sizeof(uint64_t)) != hipSuccess)
    throw std::runtime_error("driver: hipMalloc(log base table) failed");
  if (hipMemset(bases_dev_, 0, size_t(np) * sizeof(uint64_t)) != hipSuccess)
    throw std::runtime_error("driver: hipMemset failed");
}

void LogPins::enable_mirror(uint64_t chunk_bytes, int chunks_per_partition, int copy_streams) {
  if (!broker_) throw std::runtime_error("DeviceLoader h2d='dma' device decode needs the synthetic broker");
  mirror_ = std::make_unique<LogMirror>(eng_->device(), chunk_bytes, chunks_per_partition, copy_streams);
}

void LogPins::pin_written(const std::vector<uint32_t>& pidxs) {
  if (!broker_) return;
  eng_->prepare_decode();
  for (uint32_t p : pidxs) {
    if (p >= reg_end_.size()) continue;
    const uint64_t written = broker_->part(p).log_end_pos.load(std::memory_order_acquire);
    if (written) ensure(p, written);
  }
}

void LogPins::ensure(uint32_t pidx, uint64_t end) {
  if (pidx >= reg_end_.size()) throw std::out_of_range("driver: partition index beyond the broker's table");
  if (end <= reg_end_[pidx]) return;
  const int64_t t0 = tk::now_ns();
  const uint8_t* base = broker_->log_base(pidx);
  auto& part = broker_->part(pidx);
  const uint64_t cap = part.log_capacity;
  if (end > cap) throw std::runtime_error("driver: slot references bytes beyond the partition log");
  // Everything already written (a retained backlog is pinned once, at its first use), then whole
  // chunks, so a growing log pays one registration per 64 MiB.  Pinning costs ~13 GB/s of fresh
  // shm pages on the MI355X host (profiles/*/register_probe2.log): it is what bounds this mode
  // on a log that grows faster than that.
  const uint64_t written = part.log_end_pos.load(std::memory_order_acquire);
  uint64_t hi = (std::max(end, written) + kChunk - 1) / kChunk * kChunk;
  if (hi > cap) hi = cap;
  const uint64_t lo = reg_end_[pidx];
  if (reg_ranges_.size() <= pidx) reg_ranges_.resize(size_t(pidx) + 1);
  if (reg_ranges_[pidx].empty()) {  // announce the pin before it exists (the replicator reads these)
    part.pin_floor.store(lo, std::memory_order_release);
    part.pinned.fetch_add(1, std::memory_order_acq_rel);
  }
  // kChunk pieces, so that consumed ranges can be unpinned piecewise (release_consumed)
  for (uint64_t a = lo; a < hi; a += kChunk) {
    const uint64_t b = std::min(hi, a + kChunk);
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
}

const uint8_t* LogPins::seg_src(const tk::SpanSeg& sg, bool* hbm) {
  *hbm = false;
  const uint8_t* log = broker_->log_base(sg.pidx);  // pinned: device address == host address
  // a ring log (KafkaBridge replica) writes over its chunks: an HBM mirror of them would go stale,
  // so its segments are read zero-copy
  if (mirror_ && broker_->part(sg.pidx).ring_bytes.load(std::memory_order_relaxed) == 0) {
    // pin ahead of the segment so the mirror can copy (and prefetch) whole chunks -- of what is
    // written only: the mirror never copies past it, and registering fresh pages of the log beyond
    // it stalled this thread for 20-28 ms (128 MiB) in the only two config-4 runs that collapsed
    // (profiles/r03_final/c4_auto_mirror_trial/c4_6.log, profiles/r03_s3/mirror_stability/)
    const auto& part = broker_->part(sg.pidx);
    const uint64_t written = part.log_end_pos.load(std::memory_order_acquire);
    ensure(sg.pidx, std::min<uint64_t>(std::max<uint64_t>(written, sg.log_pos + sg.len),
                                       sg.log_pos + mirror_->span_bytes()));
    const uint8_t* m = mirror_->map(sg.pidx, sg.log_pos, sg.len, log, std::min<uint64_t>(reg_end_[sg.pidx], written));
    if (m) {
      *hbm = true;
      return m;
    }
  }
  return log + sg.log_pos;
}

void LogPins::committed(const std::unordered_map<uint32_t, int64_t>& committed) {
  if (release_consumed_ && ++commits_since_release_ >= 32) release_consumed(committed);
}

// A replica's log bytes below the committed position are never read again (one group consumes
// it; the replicator punches them out of the files): unpin whole registered ranges below it, so
// the pages are freed.  Every kernel that read them completed: a batch is committed only after
// its decode verdict.
void LogPins::release_consumed(const std::unordered_map<uint32_t, int64_t>& committed) {
  commits_since_release_ = 0;
  for (const auto& kv : committed) {
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

}  // namespace tkh
