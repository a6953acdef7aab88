// Ring poller of the main-process step driver: READY slots -> staged batches.
//
// The workers publish collated (or log-located) batches into the shared-memory ring (ring.h);
// the poller takes them in the ring's fair order, reads each header once into a SlotView, pins
// the log ranges a device-decode slot references (LogPins), issues the slot's H2D copy (Engine)
// and queues it as staged.  Empty end-of-stream slots keep their watermarks in delivery order:
// pop() folds them into the next delivered batch.  No GPU work is launched here -- the driver
// (the launcher) decides what staged batches are collated together and when.
#pragma once

#include <cstdint>
#include <deque>
#include <memory>
#include <string>
#include <vector>

#include "broker.h"
#include "commit_ledger.h"
#include "consumer.h"
#include "engine.h"
#include "log_pins.h"
#include "ring.h"
#include "span.h"

namespace tkh {

// Slots whose rows are decoded on the device from the logs into a padded batch (span.h).
inline bool row_span_kind(uint32_t k) { return k == uint32_t(tk::kPackJsonSpan) || k == uint32_t(tk::kPackVarSpan); }

struct SlotView {
  int64_t g = -1;
  uint32_t n_rows = 0, flags = 0, kind = 0, worker = 0;
  uint64_t payload_bytes = 0, values_offset = 0;
  uint32_t row_bytes = 0;
  int64_t max_row_len = 0, total_elems = 0, n_scanned = 0;
  int32_t src_dtype = -1;
  uint32_t n_segs = 0;                // kPackRecordSpan / kPackJsonSpan: SpanSeg entries at values_offset
  int32_t trunc_len = -1;             // kPackJsonSpan: rows keep at most this many elements (-1: all)
  uint64_t span_bytes = 0;            // device decode: log bytes its segments read
  uint64_t extras_offset = 0;         // record fields beside the values (SlotHeader::extras_*)
  uint32_t extras_n = 0;
  std::vector<int64_t> shape;
  std::vector<tk::Watermark> wms;
  // coalesced fast path: collated ahead of delivery by a group launch
  bool pre = false;
  hipStream_t pre_stream = nullptr;
  int64_t pre_event_slot = -1;        // slot whose completion event follows the group kernel
  int64_t pre_group = -1;             // that group launch's sequence number (slot numbers recur)
  std::shared_ptr<void> pre_out;      // the output tensor (opaque here: libtorch stays in torch_step.cpp)
  int64_t perr = -1;                  // device-checked batch: its status word (set at launch)
};

class RingPoller {
 public:
  RingPoller(std::shared_ptr<tk::Ring> ring, Engine* engine, LogPins* pins, CommitLedger* ledger,
             tk::Broker* broker, bool in_order, int default_src_dt);

  // One ring acquisition: 1 a batch was staged, 0 an empty slot without watermarks was consumed
  // (non-blocking only), -1 nothing ready (timeout), -2 every worker ended, -3 a worker failed (error()).
  int poll(bool block, int64_t timeout_ms);
  // The next staged batch, carrying the watermarks of the empty slots staged before it.
  bool pop(SlotView* out);

  std::deque<SlotView>& staged() { return staged_; }
  const std::deque<SlotView>& staged() const { return staged_; }
  int data_staged() const;  // staged batches with rows (not watermark-only entries)
  bool all_done() const;
  bool worker_done(uint32_t w) const { return done_.at(w) != 0; }
  // Pulls the headers of the slots the next acquisition looks at into this core's cache.
  void prefetch_ready() const;
  const std::string& error() const { return error_; }
  tk::Ring& ring() { return *ring_; }

  struct Stats {
    // worker fill time of staged slots, their age when taken, worker idle (previous publish ->
    // next fill start) and FREE-slot waits, slots staged and host time in non-blocking polls
    int64_t fill_ns = 0, fills = 0, ready_age_ns = 0, worker_idle_ns = 0, worker_slot_wait_ns = 0, polled = 0,
            poll_ns = 0;
  } stats;
  void reset_stats() { stats = Stats{}; }

 private:
  int acquire(bool block, int64_t timeout_ms);

  std::shared_ptr<tk::Ring> ring_;
  Engine* eng_;
  LogPins* pins_;
  CommitLedger* ledger_;
  tk::Broker* broker_;
  bool in_order_;
  int default_src_dt_;
  std::vector<uint32_t> cursor_;
  std::vector<uint8_t> done_;
  uint32_t rr_ = 0;
  std::deque<SlotView> staged_;
  std::vector<tk::Watermark> carry_;
  std::vector<int64_t> last_ready_;
  std::string error_;
};

}  // namespace tkh
