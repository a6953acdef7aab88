#include "batch_verdicts.h"

#include "reaper.h"

#include <algorithm>
#include <cstring>
#include <ctime>
#include <stdexcept>

#include "collate.h"
#include "consumer.h"
#include "crc32c.h"
#include "dtypes.h"
#include "hip_queue.h"
#include "span.h"

namespace tkh {

namespace {
template <typename T>
void host_mapped(size_t n, T** host, T** dev, const char* what) {
  void* h = nullptr;
  if (hipHostMalloc(&h, n * sizeof(T), hipHostMallocMapped) != hipSuccess)
    throw std::runtime_error(std::string("driver: hipHostMalloc of the ") + what + " failed");
  void* d = nullptr;
  if (hipHostGetDevicePointer(&d, h, 0) != hipSuccess) throw std::runtime_error("driver: hipHostGetDevicePointer failed");
  *host = static_cast<T*>(h);
  *dev = static_cast<T*>(d);
}
}  // namespace

BatchVerdicts::~BatchVerdicts() {
  // no kernel still writes a status word: the driver waited for every handed slot (quiesce)
  // hipFree / hipHostFree wait for the whole device: the deferred-release thread runs them (reaper.h)
  const int dev = q_ ? q_->device() : 0;
  Reaper::free_host(dev, perr_host_);
  Reaper::free_host(dev, jinfo_host_);
  Reaper::free_device(dev, patch_dev_);
  Reaper::free_host(dev, part_host_);
  Reaper::free_device(dev, ctr_dev_);
}

void BatchVerdicts::ensure_status() {
  if (perr_host_) return;
  host_mapped(size_t(kWords), &perr_host_, &perr_dev_, "status words");
  state_.assign(size_t(kWords), 1);
  host_mapped(size_t(kWords) * 4, &jinfo_host_, &jinfo_dev_, "JSON width words");
  std::memset(jinfo_host_, 0, size_t(kWords) * 4 * sizeof(int32_t));
  jrows_.assign(size_t(kWords), {});
  jparsed_.assign(size_t(kWords), 0);
  if (hipMalloc(reinterpret_cast<void**>(&ctr_dev_), size_t(kWords) * kCtrWords * sizeof(unsigned long long)) != hipSuccess ||
      hipMemset(ctr_dev_, 0, size_t(kWords) * kCtrWords * sizeof(unsigned long long)) != hipSuccess)
    throw std::runtime_error("driver: allocating the JSON count words failed");
  tag_.assign(size_t(kWords), 0);
}

void BatchVerdicts::ensure_partials() {
  if (part_host_) return;
  host_mapped(size_t(kWords * kPartials), &part_host_, &part_dev_, "partial CRC words");
  msg_.assign(size_t(kWords), std::string());
}

int64_t BatchVerdicts::next_word() {
  ensure_status();
  const int64_t w = int64_t(seq_ % uint64_t(kWords));
  tag_[size_t(w)] = uint32_t(seq_ / uint64_t(kWords)) + 1;  // 0 is the zeroed words' tag
  ++seq_;
  if (state_[size_t(w)] == 0) throw std::runtime_error("driver: more than 4096 device-checked batches awaiting their kernels");
  perr_host_[w] = -1;
  jinfo_host_[w * 4 + 1] = 0;
  __atomic_store_n(jinfo_host_ + w * 4 + 2, 0, __ATOMIC_RELEASE);
  jrows_[size_t(w)].clear();
  jparsed_[size_t(w)] = 0;
  state_[size_t(w)] = 0;
  if (!msg_.empty()) msg_[size_t(w)].clear();
  return w;
}

void BatchVerdicts::on_release(int64_t g, int64_t w, bool span) {
  if (span && __atomic_load_n(jinfo_host_ + w * 4 + 1, __ATOMIC_ACQUIRE) > 0) parse_host_rows(g, w);
  if (span) check_span(g, w);  // reads the slot: before its release
  state_[size_t(w)] = __atomic_load_n(perr_host_ + w, __ATOMIC_ACQUIRE) < 0 ? 1 : 2;
}

void BatchVerdicts::mark_bad(int64_t w, int64_t row) {
  int32_t expect = -1;
  __atomic_compare_exchange_n(perr_host_ + w, &expect, tk::kSpanParseErrBit | int32_t(row), false, __ATOMIC_ACQ_REL,
                              __ATOMIC_ACQUIRE);
  if (state_[size_t(w)] == 1) state_[size_t(w)] = 2;
}

void BatchVerdicts::check_span(int64_t g, int64_t w) {
  const tk::SlotHeader* h = ring_->slot(uint32_t(g));
  const auto* sg = reinterpret_cast<const tk::SpanSeg*>(ring_->payload(uint32_t(g)) + h->values_offset);
  // a whole RecordBatch failed its CRC on the device (segment index), or a JSON row its parse
  const int32_t dev = __atomic_load_n(perr_host_ + w, __ATOMIC_ACQUIRE);
  int32_t bad = dev >= tk::kSpanParseErrBit ? -1 : dev;
  const uint32_t* part = part_host_ + w * kPartials;
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
      msg_[size_t(w)] = "batch row " + std::to_string(dev & ~tk::kSpanParseErrBit) +
                        " is not a flat numeric JSON array (device parse from the log)";
    return;
  }
  // the RecordBatch of segment `bad`: walk back to its first segment for its base offset
  uint32_t i = uint32_t(bad);
  while (i > 0 && !(sg[i].flags & tk::kSegCrcFirst)) --i;
  const uint8_t* rb = broker_->log_base(sg[i].pidx) + sg[i].log_pos;
  int64_t base = 0;
  for (int b = 0; b < 8; ++b) base = (base << 8) | int64_t(rb[b]);
  msg_[size_t(w)] = "Record batch at offset " + std::to_string(base) + " of partition index " +
                    std::to_string(sg[i].pidx) + " failed CRC check (verified on the device)";
  __atomic_store_n(perr_host_ + w, bad, __ATOMIC_RELEASE);
}

std::string BatchVerdicts::failure(int64_t w, const std::vector<tk::Watermark>& wms) const {
  std::string where;
  for (const auto& m : wms)
    where += (where.empty() ? "" : ", ") + std::string("partition index ") + std::to_string(m.pidx) + " offsets [" +
             std::to_string(m.first_offset) + ", " + std::to_string(m.next_offset) + ")";
  if (w < int64_t(msg_.size()) && !msg_[size_t(w)].empty()) return msg_[size_t(w)] + " (batch: " + where + ")";
  const int32_t row = __atomic_load_n(perr_host_ + w, __ATOMIC_ACQUIRE);
  return "batch row " + std::to_string(row) + " is not a flat numeric JSON array (device parse; batch: " + where + ")";
}

int64_t BatchVerdicts::json_width(int64_t w, int64_t* n_host) {
  *n_host = 0;
  if (w < 0 || !jinfo_host_) throw std::logic_error("driver: json_width of a batch without a parse launch");
  const int32_t* info = jinfo_host_ + w * 4;
  // the parse kernel's first block of the batch reports the width: usually long done (the batch was
  // parsed ahead), else within one kernel's latency
  const int64_t t0 = tk::now_ns();
  for (int spin = 0; __atomic_load_n(info + 2, __ATOMIC_ACQUIRE) == 0; ++spin) {
    if (spin < 4096) {
      tk::cpu_relax();
      continue;
    }
    q_->check();  // a failed queue never ran the parse: report its failure, not a timeout
    if (tk::now_ns() - t0 > 60'000'000'000LL)
      throw std::runtime_error("driver: the JSON parse kernel did not report a batch width within 60 s");
    timespec ts{0, 20000};
    nanosleep(&ts, nullptr);
  }
  width_wait_ns += tk::now_ns() - t0;
  *n_host = __atomic_load_n(info + 1, __ATOMIC_ACQUIRE);
  return __atomic_load_n(info, __ATOMIC_ACQUIRE);
}

void BatchVerdicts::parse_host_rows(int64_t g, int64_t w) {
  if (jparsed_[size_t(w)]) return;
  jparsed_[size_t(w)] = 1;
  // the rows the device found not simple are the device-counted rows json_scan_simple rejects;
  // parse them as the worker would have (parse_json_f32: Python's float() of each number)
  const tk::SlotHeader* h = ring_->slot(uint32_t(g));
  const uint8_t* pay = ring_->payload(uint32_t(g));
  const auto* rows = reinterpret_cast<const tk::JsonSpanRow*>(pay);
  const auto* sg = reinterpret_cast<const tk::SpanSeg*>(pay + h->values_offset);
  auto& out = jrows_[size_t(w)];
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
        mark_bad(w, r);
        if (w < int64_t(msg_.size()) && msg_[size_t(w)].empty())
          msg_[size_t(w)] = "batch row " + std::to_string(r) + " is not a flat numeric JSON array";
        continue;
      }
      hr.count = int32_t(c);
      hr.vals.resize(size_t(c));
      out.push_back(std::move(hr));
    }
  }
}

void BatchVerdicts::json_host_rows(int64_t g, int64_t w, int32_t trunc_len, void* out, int64_t L, int dst_dt,
                                   double pad, int64_t* lengths, uint8_t* mask, hipStream_t stream) {
  if (w < 0) return;
  q_->drain();  // the copies below go on `stream` after its queued parse kernel
  if (!jparsed_[size_t(w)]) parse_host_rows(g, w);  // the slot is still held
  const int dsz = dtype_size(dst_dt);
  constexpr size_t kVals = 256;  // the values start 256 bytes after the row descriptor
  for (const HostRow& hr : jrows_[size_t(w)]) {
    int64_t n_out = hr.count;
    if (trunc_len >= 0 && n_out > trunc_len) n_out = trunc_len;
    if (n_out > L) {  // wider than the device count made the batch: cannot happen for a flat numeric array
      mark_bad(w, hr.row);
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

}  // namespace tkh
