#include "log_pins.h"

#include "reaper.h"

#include <algorithm>
#include <chrono>
#include <stdexcept>

namespace tkh {

static_assert(LogPins::kChunk == LogMirror::kRegAlign, "mirror copies split at the pin pieces");

LogPins::LogPins(Engine* engine, std::shared_ptr<tk::Broker> broker) : eng_(engine), broker_(std::move(broker)) {
  if (broker_) {
    n_parts_ = broker_->meta().max_partitions;
    reg_end_ = std::make_unique<std::atomic<uint64_t>[]>(n_parts_);
    for (uint32_t i = 0; i < n_parts_; ++i) reg_end_[i].store(0, std::memory_order_relaxed);
    reg_ranges_.resize(n_parts_);
    release_consumed_ = (broker_->flags() & tk::kReleaseConsumed) != 0;
  }
}

LogPins::~LogPins() {
  {
    std::lock_guard<std::mutex> l(pm_);
    stop_ = true;
  }
  pcv_.notify_all();
  if (pin_thread_.joinable()) pin_thread_.join();
  try {
    eng_->synchronize();  // the decode streams that read the mirror and the ranges (the driver quiesced)
  } catch (...) {
  }
  mirror_.reset();  // its copies read the pinned logs: before they are unregistered
  // the registrations go to the deferred-release thread (reaper.h), which holds the broker's
  // mapping until they are gone and only then tells the replicator the logs are unpinned
  std::vector<std::pair<uint32_t, std::vector<void*>>> regs;
  for (size_t pidx = 0; pidx < reg_ranges_.size(); ++pidx) {
    auto& q = reg_ranges_[pidx];
    if (q.empty()) continue;
    std::vector<void*> ps;
    for (auto& r : q) ps.push_back(r.first);
    regs.emplace_back(uint32_t(pidx), std::move(ps));
  }
  if (!regs.empty())
    Reaper::post(eng_->device(), [regs = std::move(regs), broker = broker_] {
      for (auto& [pidx, ps] : regs) {
        for (void* p : ps) (void)hipHostUnregister(p);
        if (broker) broker->part(pidx).pinned.fetch_sub(1, std::memory_order_acq_rel);
      }
    });
  Reaper::free_device(eng_->device(), bases_dev_);
}

void LogPins::enable_direct() {
  if (!broker_) throw std::runtime_error("DeviceLoader h2d='dma' direct needs the synthetic broker (group_id + URL)");
  if (bases_dev_) return;
  const uint32_t np = n_parts_;
  if (hipMalloc(reinterpret_cast<void**>(&bases_dev_), size_t(np) * sizeof(uint64_t)) != hipSuccess)
    throw std::runtime_error("driver: hipMalloc(log base table) failed");
  if (hipMemset(bases_dev_, 0, size_t(np) * sizeof(uint64_t)) != hipSuccess)
    throw std::runtime_error("driver: hipMemset failed");
}

void LogPins::enable_mirror(uint64_t chunk_bytes, int chunks_per_partition, int copy_streams, int wait) {
  if (!broker_) throw std::runtime_error("DeviceLoader h2d='dma' device decode needs the synthetic broker");
  mirror_ = std::make_unique<LogMirror>(eng_->device(), &eng_->queue(), chunk_bytes, chunks_per_partition, copy_streams,
                                        wait);
}

void LogPins::pin_written(const std::vector<uint32_t>& pidxs) {
  if (!broker_) return;
  eng_->prepare_decode();
  for (uint32_t p : pidxs) {
    if (p >= n_parts_) continue;
    // a ring log (KafkaBridge replica) whole: its pages are written over lap after lap and stay
    // pinned, and its first lap otherwise ran at the pin thread's registration rate (~12 GB/s, one
    // 64 MiB piece per ~5 ms: the compressed bridge blocks, whose timed steps all fell in the first
    // lap, profiles/r06_s27)
    const auto& part = broker_->part(p);
    const uint64_t ring = part.ring_bytes.load(std::memory_order_relaxed);
    const uint64_t want = ring ? ring : part.log_end_pos.load(std::memory_order_acquire);
    if (want) ensure(p, want);
  }
}

bool LogPins::pin_some(uint32_t pidx, uint64_t end, bool one_piece) {
  std::lock_guard<std::mutex> l(reg_m_);
  const uint64_t lo = reg_end_[pidx].load(std::memory_order_relaxed);
  auto& part = broker_->part(pidx);
  const uint64_t cap = part.log_capacity;
  if (end > cap) throw std::runtime_error("driver: slot references bytes beyond the partition log");
  // Everything already written, then whole chunks, so a growing log pays one registration per
  // 64 MiB (and a mirror never copies across two registrations).  What is pinned past the written
  // end is at most the rest of the chunk the end falls in -- fresh pages of the sparse file.
  const uint64_t written = part.log_end_pos.load(std::memory_order_acquire);
  uint64_t hi = (std::max(end, written) + kChunk - 1) / kChunk * kChunk;
  if (hi > cap) hi = cap;
  if (one_piece) hi = std::min(hi, lo + kChunk);
  if (hi <= lo) return false;
  const int64_t t0 = tk::now_ns();
  const uint8_t* base = broker_->log_base(pidx);
  if (reg_ranges_[pidx].empty()) {  // announce the pin before it exists (the replicator reads these)
    part.pin_floor.store(lo, std::memory_order_release);
    part.pinned.fetch_add(1, std::memory_order_acq_rel);
  }
  // kChunk pieces, so that consumed ranges can be unpinned piecewise (release_consumed)
  for (uint64_t a = lo; a < hi; a += kChunk) {
    const uint64_t b = std::min(hi, a + kChunk);
    void* p = const_cast<uint8_t*>(base) + a;
    hipError_t e = hipHostRegister(p, b - a, hipHostRegisterMapped);
    if (e == hipErrorHostMemoryAlreadyRegistered) {
      // the previous iteration (or a closed loader) over this same broker mapping handed its
      // registration of these pages to the deferred-release thread, which has not run it yet
      // (it waits for the device, e.g. behind the user's queued kernels): wait for it, once
      (void)hipGetLastError();
      Reaper::drain(60000);
      ++register_retries_;
      e = hipHostRegister(p, b - a, hipHostRegisterMapped);
    }
    if (e != hipSuccess)
      throw std::runtime_error(std::string("driver: hipHostRegister of a partition log failed: ") +
                               hipGetErrorString(e) +
                               (e == hipErrorHostMemoryAlreadyRegistered
                                    ? " (another live loader of this process pins the same broker mapping)"
                                    : ""));
    reg_ranges_[pidx].emplace_back(p, b);
    void* dp = nullptr;
    if (hipHostGetDevicePointer(&dp, p, 0) != hipSuccess || dp != p)
      throw std::runtime_error("driver: device decode needs device addresses of pinned host memory to equal host "
                               "addresses (unified addressing)");
  }
  if (lo == 0 && bases_dev_) {
    const uint64_t b = reinterpret_cast<uint64_t>(base);
    if (hipMemcpy(bases_dev_ + pidx, &b, sizeof(b), hipMemcpyHostToDevice) != hipSuccess)
      throw std::runtime_error("driver: log base table update failed");
  }
  reg_end_[pidx].store(hi, std::memory_order_release);
  reg_total_ += hi - lo;
  reg_ns_ += tk::now_ns() - t0;
  return true;
}

void LogPins::ensure(uint32_t pidx, uint64_t end) {
  if (pidx >= n_parts_) throw std::out_of_range("driver: partition index beyond the broker's table");
  if (end <= reg_end_[pidx].load(std::memory_order_acquire)) return;
  if (end > broker_->part(pidx).log_capacity)
    throw std::runtime_error("driver: slot references bytes beyond the partition log");
  if (bases_dev_ || reg_end_[pidx].load(std::memory_order_acquire) == 0) {
    // the first pin of a log (its retained backlog, before any batch of it) and h2d='direct'
    // (experimental) register here; afterwards the pin thread follows the log as it grows
    pin_some(pidx, end, false);
    if (!bases_dev_) {
      std::lock_guard<std::mutex> l(pm_);
      tracked_.insert(pidx);
      if (!pin_thread_.joinable()) pin_thread_ = std::thread([this] { pin_loop(); });
    }
    return;
  }
  const int64_t t0 = tk::now_ns();
  std::unique_lock<std::mutex> l(pm_);
  uint64_t& d = demand_[pidx];
  d = std::max(d, end);
  pcv_.notify_one();
  done_cv_.wait(l, [&] { return reg_end_[pidx].load(std::memory_order_acquire) >= end || !err_.empty(); });
  wait_ns_ += tk::now_ns() - t0;
  if (reg_end_[pidx].load(std::memory_order_acquire) < end) throw std::runtime_error(err_);
}

// The pin thread: demands first (the launch thread is waiting), then one chunk for any tracked
// partition whose written end has passed its pinned end; otherwise a 1 ms nap.
void LogPins::pin_loop() {
  tk::name_thread("tk-log-pins");
  std::unique_lock<std::mutex> l(pm_);
  while (!stop_) {
    uint32_t pidx = UINT32_MAX;
    uint64_t want = 0;
    for (auto it = demand_.begin(); it != demand_.end();) {
      if (reg_end_[it->first].load(std::memory_order_acquire) >= it->second) {
        it = demand_.erase(it);
      } else {
        pidx = it->first;
        want = it->second;
        break;
      }
    }
    if (pidx == UINT32_MAX) {
      for (uint32_t p : tracked_) {
        const uint64_t w = broker_->part(p).log_end_pos.load(std::memory_order_acquire);
        if (w > reg_end_[p].load(std::memory_order_acquire)) {
          pidx = p;
          want = w;
          break;
        }
      }
    }
    if (pidx == UINT32_MAX) {
      pcv_.wait_for(l, std::chrono::milliseconds(1));
      continue;
    }
    l.unlock();
    std::string err;
    try {
      pin_some(pidx, want, true);
    } catch (const std::exception& e) {
      err = e.what();
    }
    l.lock();
    if (!err.empty()) {
      err_ = err;
      done_cv_.notify_all();
      return;
    }
    done_cv_.notify_all();
  }
}

const uint8_t* LogPins::seg_src(const tk::SpanSeg& sg, bool* hbm) {
  *hbm = false;
  const uint8_t* log = broker_->log_base(sg.pidx);  // pinned: device address == host address
  // a ring log (KafkaBridge replica) writes over its chunks: an HBM mirror of them would go stale,
  // so its segments are read zero-copy
  if (mirror_ && broker_->part(sg.pidx).ring_bytes.load(std::memory_order_relaxed) == 0) {
    // pin ahead of the segment so the mirror can copy (and prefetch) whole chunks.  No look-ahead
    // past the written end: the mirror never copies past it.  (A growing log still gets whole
    // chunks registered -- up to the next 64 MiB boundary -- but by the pin thread, not here.)
    // The look-ahead this replaced registered up to 128 MiB of unwritten log on the launch thread.
    // It was not what made round 3's config-4 mirror runs collapse: round 4's slow runs registered
    // nothing in their timed windows (profiles/r04_s1/c4); their launches waited for the copy
    // stream's whole queue, which LogMirror's no-wait policy removed (profiles/r04_s2, r04_s3).
    const auto& part = broker_->part(sg.pidx);
    const uint64_t written = part.log_end_pos.load(std::memory_order_acquire);
    ensure(sg.pidx, std::min<uint64_t>(std::max<uint64_t>(written, sg.log_pos + sg.len),
                                       sg.log_pos + mirror_->span_bytes()));
    const uint8_t* m = mirror_->map(sg.pidx, sg.log_pos, sg.len, log, std::min<uint64_t>(pinned_end(sg.pidx), written));
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
  std::lock_guard<std::mutex> l(reg_m_);
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
