// Main-process step driver: the per-batch host path of DeviceLoader in one native call.
//
// Python-level per-batch work (ring polling, summary/watermark reads, H2D issue, event
// bookkeeping, commit) cost ~20 us per batch; at 256 x 1 KiB records per batch that capped one
// MI355X at ~11 M records/s.  The driver keeps all of it native.  It is the LAUNCHER: it forms
// groups of staged batches, launches their collate / decode kernels on the user's or the decode
// streams, tracks the launched slots' completion events and releases the slots, and decides when
// a delivered batch is finished and committable.  The parts around it are their own classes:
//   RingPoller    (ring_poller.h)    READY ring slots -> staged batches (H2D issued)
//   LogPins       (log_pins.h)       partition logs pinned / mirrored for device decode
//   BatchVerdicts (batch_verdicts.h) device CRC / parse status words of launched batches
//   CommitLedger  (commit_ledger.h)  finished offsets -> durable commits, commit latency
//   CreditLockstep (core/lockstep.h) cross-rank agreement on the step count (DDP)
#pragma once

#include <hip/hip_runtime.h>

#include <cstdlib>
#include <deque>
#include <memory>
#include <string>
#include <tuple>
#include <vector>

#include "batch_verdicts.h"
#include "broker.h"
#include "collate.h"
#include "commit_ledger.h"
#include "consumer.h"
#include "engine.h"
#include "lockstep.h"
#include "log_mirror.h"
#include "log_pins.h"
#include "rccl_lockstep.h"
#include "ring.h"
#include "ring_poller.h"
#include "span_decode.h"

namespace tkh {

class MainDriver {
 public:
  MainDriver(Engine* engine, const std::string& ring_name, const std::string& broker_url, const std::string& group,
             int prefetch, bool in_order, int default_src_dt);
  ~MainDriver();

  // Next batch slot (H2D issued).  Returns 1 (out filled), -1 timeout, -2 end of stream, -3 worker error,
  // -4 an earlier device-parsed batch was malformed (parse_error()).
  int next_slot(int64_t timeout_ms, SlotView* out);
  const std::string& error() const { return poller_->error(); }

  void collate_fixed(const SlotView& v, hipStream_t stream, int dst_dt, void* dst, int64_t row, const float* shift,
                     const float* scale);
  // Record fields beside the values (SlotView::extras_*): the next fixed-width launch (single,
  // group or ahead) writes batch k's [extras_n, rows] int64 columns to dsts[k].  Consumed by that
  // launch; torch_step.cpp allocates them with the value tensors.
  void set_extra_outputs(int64_t* const* dsts, int n) {
    ext_n_ = n;
    for (int k = 0; k < n && k < kMaxGroup; ++k) ext_dsts_[k] = dsts[k];
  }
  // The slot's whole payload copied to `dst` (device memory) on `stream` (kPackTree slots: the
  // fields are views of that block); the slot is released once the copy completed.
  void copy_payload(const SlotView& v, hipStream_t stream, void* dst);
  void collate_varlen(const SlotView& v, hipStream_t stream, int dst_dt, void* out, int64_t L, double pad,
                      int64_t* lengths, uint8_t* mask);

  // Device JSON parse / span decode: a batch's status word is checked once its GPU work completed,
  // before the batch can be committed; a bad batch stops the commits (commit_pending() returns -2,
  // next_slot() -4) and parse_error() describes it.
  const std::string& parse_error() const { return parse_error_; }

  void deliver(const SlotView& v);   // batch handed to the user
  void set_delivered(const SlotView& v);
  void discard(const SlotView& v);   // consumed but not handed out (drop_last): free its slot
  // The user is done with every delivered batch.  With commit-on-device, `fence`
  // (the user's stream) gets an event and the batch only becomes committable
  // once the GPU has executed everything the user queued for it.
  void finish_delivered(hipStream_t fence = nullptr);
  void set_commit_on_device(bool on) { commit_on_device_ = on; }
  // Moves fenced batches whose GPU work completed to the committable stage.
  void drain_fenced(bool wait);
  void add_finished(const std::vector<tk::Watermark>& wms) { ledger_->add_finished(wms); }
  // Commits every finished batch.  Returns 0 nothing to do, 1 committed, -1 CommitFailedError,
  // -2 a device-checked batch failed (the batches before it were committed).
  int commit_pending();
  bool can_commit() const { return ledger_->can_commit(); }
  void set_worker_sink(uintptr_t table, int n_workers, int capacity) {
    ledger_->set_worker_sink(table, n_workers, capacity);
  }

  // Fused fast path: [finish+commit previous] -> next slot -> fixed-width collate into dst.
  // Returns n_rows (>0), or -1 timeout, -2 end, -3 error; *commit_status as commit_pending().
  int64_t step_fixed(hipStream_t stream, int dst_dt, void* dst, int64_t row, const float* shift, const float* scale,
                     bool auto_commit, int64_t timeout_ms, int* commit_status, SlotView* out);

  // Coalesced fast path, two phases around the caller's output allocation:
  //   begin:  finish+commit the previous batch, take the next one.  If it was collated by an
  //           earlier group launch, *pre_out receives its tensor and nothing is launched.
  //           Otherwise *group_rows lists the rows of the batches to collate now: the one being
  //           returned, then up to coalesce-1 already-staged fixed-width batches behind it.
  //   launch: one kernel collates the group into dsts[k]; handles[k-1] (k >= 1) ride with the
  //           staged batches until they are delivered.
  // Returns n_rows (>0), or -1 timeout, -2 end, -3 error.
  int64_t step_group_begin(hipStream_t stream, bool auto_commit, int64_t timeout_ms, int* commit_status,
                           std::vector<int64_t>* group_rows, std::shared_ptr<void>* pre_out);
  void step_group_launch(hipStream_t stream, int dst_dt, void* const* dsts, int64_t row, const float* shift,
                         const float* scale, std::vector<std::shared_ptr<void>>&& handles);
  // Coalesced device JSON parse (kPackJsonText), two phases around the caller's allocations:
  //   json_group_extend: after next_slot() returned a JSON batch in `last`, lists the staged
  //                      JSON batches right behind it that one launch can parse too (<= coalesce-1);
  //   json_group_launch: one kernel for last + those; outs/Ls/... hold 1 + n entries, handles
  //                      (the staged batches' outputs) ride with them until they are delivered.
  size_t json_group_extend();
  // Stages READY slots until `extra` beyond prefetch are staged (never blocks).
  void stage_ready(int extra);
  // A batch parsed by a group launch on another stream: `stream` waits for that kernel.
  void wait_group(const SlotView& v, hipStream_t stream) { wait_launch(v.pre_event_slot, v.pre_group, stream); }
  const SlotView& group_member(size_t k) const { return poller_->staged()[group_idx_[k]]; }
  void json_group_launch(hipStream_t stream, int dst_dt, double pad, void* const* outs, const int64_t* Ls,
                         int64_t* const* lengths, uint8_t* const* masks,
                         std::vector<std::shared_ptr<void>>&& handles);
  // Device decode AHEAD of delivery: once the user has taken a batch, the driver forms the next
  // group from staged batches nobody has asked for yet and launches it at once, so its kernel
  // (tens of us: PCIe-bound, sharing the link with the groups before it) runs while the user
  // works through the batches already decoded.  ahead_begin stages what the workers published
  // (never blocks) and lists the rows of a full group of not-yet-decoded device-decode batches
  // (empty: nothing to launch, or ahead_depth groups are already decoded ahead); ahead_launch
  // decodes them into dsts[k] (handles[k] keep each output alive until its batch is delivered).
  void ahead_begin(std::vector<int64_t>* rows);
  void ahead_launch(int dst_dt, void* const* dsts, const float* shift, const float* scale,
                    std::vector<std::shared_ptr<void>>&& handles);
  // The batches of the group ahead_begin formed (JSON: their row counts and max row lengths size
  // the outputs), and the JSON-span variant of ahead_launch (outputs as json_group_launch).
  const SlotView& ahead_member(size_t k) const { return poller_->staged()[group_idx_[k]]; }
  void ahead_launch_json(int dst_dt, double pad, void* const* outs, const int64_t* Ls, int64_t* const* lengths,
                         uint8_t* const* masks, std::vector<std::shared_ptr<void>>&& handles);
  void set_ahead_depth(int n) { ahead_depth_ = n < 0 ? 0 : n; }
  int ahead_depth() const { return ahead_depth_; }
  // (stream, bytes) of the output blocks already cached on a decode stream (torch_step.cpp
  // warm_group_blocks)
  std::vector<std::pair<hipStream_t, int64_t>> warm_blocks_;
  // Device-counted JSON batches (kSlotDevCount, span.h kJsonCountOnDevice).  Their outputs are
  // allocated at the worker's bound (max_row_len); the parse kernel picks the real width from the
  // device count of the longest row, rounded up to `mult` (0: the allocated width stays, pad_to).
  void set_json_mult(int64_t mult) { json_mult_ = mult < 0 ? 0 : int32_t(mult); }
  // json_width: the width of delivered batch v (waits for its parse kernel to report it) and, in
  // *n_host, the rows that were not simple.  json_host_rows: parses those rows on the host (from the
  // pinned logs, when the batch is delivered or its slot released, whichever comes first) and
  // writes them into the batch's outputs on `stream`, which it then synchronizes.
  int64_t json_width(const SlotView& v, int64_t* n_host) { return verdicts_->json_width(v.perr, n_host); }
  void json_host_rows(const SlotView& v, void* out, int64_t L, int dst_dt, double pad, int64_t* lengths,
                      uint8_t* mask, hipStream_t stream) {
    verdicts_->json_host_rows(v.g, v.perr, v.trunc_len, out, L, dst_dt, pad, lengths, mask, stream);
  }
  hipStream_t last_stream() const { return last_stream_; }
  int64_t last_perr() const { return last_perr_; }
  // The stream the next device-decode group launch runs on (its outputs are allocated there).
  hipStream_t next_decode_stream() { return eng_->decode_stream(int(span_launches_ % 4096)); }
  void set_coalesce(int n) { coalesce_ = n < 1 ? 1 : (n > kMaxGroup ? kMaxGroup : n); }
  // Device-decode groups stop growing at this many log bytes: a group's batches become committable
  // together when its kernel completes, so 8 x 8 MiB batches (config 5) would hold every commit for
  // a 64 MiB transfer (~1.3 ms); small batches still group 8 at a time.
  void set_group_bytes(uint64_t b) { group_bytes_max_ = b < (1u << 20) ? (1u << 20) : b; }
  // Adaptive coalescing: while the GPU is still running an earlier launch, wait up to `us` for
  // more staged batches so the next launch carries a full group (0 disables).  Waiting costs no
  // GPU time -- the GPU is busy anyway -- and a zero-copy batch costs 7.1 us alone but 5.2 us
  // in a group of 4 (PCIe latency amortised).
  void set_coalesce_wait_us(int64_t us) { coalesce_wait_ns_ = us < 0 ? 0 : us * 1000; }

  // h2d="direct": the workers' slots hold log locations (kPackGatherFixed); the logs are pinned in
  // place just ahead of what a slot references, with a device table of their addresses.
  static constexpr uint64_t kLogChunk = LogPins::kChunk;
  void enable_direct() { pins_->enable_direct(); }
  // Device decode / direct: pin the logs of these partitions as far as they are written now (the
  // retained backlog), so their registration (~13 GB/s of fresh pages on the MI355X host) is paid
  // when the iteration starts instead of by the first batches that reach each partition.
  void pin_logs(const std::vector<uint32_t>& pidxs) { pins_->pin_written(pidxs); }
  bool direct() const { return pins_->direct(); }
  // h2d='dma' with device decode: the decode kernels read the logs from an HBM mirror that the copy
  // engines fill chunk by chunk (log_mirror.h) instead of over PCIe from the pinned logs.
  int mirror_copy_streams() const { return pins_->mirror() ? pins_->mirror()->copy_streams() : 0; }
  bool mirror_waits() const { return pins_->mirror() && pins_->mirror()->waits(); }
  // wait: 1 the mirror's launches wait for copies in flight (fixed-width decode: segments may be
  // split over workgroups), 0 they read those segments from the pinned log, -1 the default (0);
  // TORCHKAFKA_MIRROR_WAIT overrides either (log_mirror.h)
  void enable_mirror(uint64_t chunk_bytes, int chunks_per_partition, int copy_streams = 0, int wait = -1) {
    pins_->enable_mirror(chunk_bytes, chunks_per_partition, copy_streams, wait);
  }
  const LogMirror* mirror() const { return pins_->mirror(); }
  // The decode-stream and mirror HIP calls of this driver go through the HIP command queue
  // (hip_queue.h): DeviceLoader turns it on for var-len / JSON device decode.
  void set_command_queue(bool on) {
    eng_->set_command_queue(on);
    if (pins_->mirror()) pins_->mirror()->set_command_queue(on);
  }
  uint64_t log_bytes_registered() const { return pins_->bytes_registered(); }
  uint64_t log_bytes_unpinned() const { return pins_->bytes_unpinned(); }
  int64_t log_register_ns() const { return pins_->register_ns(); }
  int64_t log_register_wait_ns() const { return pins_->register_wait_ns(); }
  uint64_t log_register_retries() const { return pins_->register_retries(); }
  int coalesce() const { return coalesce_; }
  int64_t groups() const { return groups_; }

  const std::vector<tk::Watermark>& delivered() const { return delivered_; }
  // Every partition's position after the batches handed out so far (-1: none from it), and how
  // many batches that is: DeviceLoader.state_dict(global_step=True) -- the end of a global step
  // on every rank, ahead of the commits (which under the async lockstep land at agreements).
  std::vector<std::pair<uint32_t, int64_t>> delivered_positions() const {
    std::vector<std::pair<uint32_t, int64_t>> out;
    for (size_t p = 0; p < delivered_pos_.size(); ++p)
      if (delivered_pos_[p] >= 0) out.emplace_back(uint32_t(p), delivered_pos_[p]);
    return out;
  }
  uint64_t delivered_batches() const { return delivered_batches_; }
  std::vector<std::pair<uint32_t, int64_t>> committed() const { return ledger_->committed(); }
  std::vector<std::pair<uint32_t, int64_t>> take_pending() { return ledger_->take_pending(); }
  bool worker_done(uint32_t w) const { return poller_->worker_done(w); }
  uint64_t commits() const { return ledger_->commits(); }
  uint64_t commit_failures() const { return ledger_->commit_failures(); }
  const std::vector<int64_t>& commit_ns() const { return ledger_->commit_ns(); }
  // Commit latency per batch: from the request that finished batch k (the user asking for k+1)
  // to k's offsets being stored -- including the wait for its decode kernel's CRC verdict, the
  // user's GPU work (commit_on='device') and the cross-rank lockstep agreement.  With the worker
  // commit sink it ends when the offsets are handed to the workers.
  const std::vector<int64_t>& commit_latency_ns() const { return ledger_->commit_latency_ns(); }
  const RingPoller::Stats& poll_stats() const { return poller_->stats; }
  int64_t json_width_wait_ns() const { return verdicts_->width_wait_ns; }
  void reset_stats();

  // Cross-rank lockstep over RCCL, pipelined `depth` steps ahead (ls is owned by the caller).
  // Async mode: an agreement grants at most commit_every batches (0: no cap), see lockstep.h.
  void enable_lockstep(LockstepTransport* ls, int depth, int commit_every = 0);
  // commit='sync': batch k+1 is taken only after batch k's verdict landed and (under a lockstep)
  // an agreement at step k+1 made k committable on every rank (CreditLockstep sync mode).
  void set_sync_commit(bool s) {
    sync_commit_ = s;
    if (ls_) ls_->set_sync(s);
  }
  // Sync mode under a lockstep: this rank's commit status for the next agreement (lockstep.h).
  void set_commit_status(int64_t s) {
    if (ls_) ls_->set_commit_status(s);
  }
  uint64_t group_commit_failures() const { return ls_ ? ls_->group_commit_failures() : 0; }
  // verify='deliver': waits for the device verdict (CRC32C / JSON grammar) of the batch just
  // delivered.  0 clean or not device-checked; -4 corrupt (parse_error() says why: the batches
  // finished before it were made committable first, it and what follows never are).
  int verify_delivered();
  // The non-blocking half of verify_delivered: true once the delivered batch's verdict is known
  // (its kernel completed and its slot was released) or it carries none.  The fast paths poll it
  // while launching the groups the workers finish meanwhile (torch_step.cpp verify_ahead), so the
  // GPU is not left idle between the verdict and the next request.
  bool delivered_verdict_known();
  int64_t verify_wait_ns_ = 0;  // host time verify_delivered() spent waiting for kernels
  // End of a lock-stepped iteration: barrier, then every finished batch becomes committable.
  void finish_lockstep();
  bool lockstep_enabled() const { return bool(ls_); }
  uint64_t lockstep_agreements() const { return ls_ ? ls_->agreements_since_reset() : 0; }
  int64_t lockstep_wait_ns() const { return ls_ ? ls_->wait_ns() : 0; }
  int64_t lockstep_issue_ns() const { return ls_ ? ls_->issue_ns() : 0; }
  int64_t lockstep_step_wait_max_ns() const { return ls_ ? ls_->step_wait_max_ns() : 0; }

  SlotView last;  // the slot most recently returned by next_slot / step_fixed

  // Completion events are recorded for one handed-out slot in `n` (>= 1); the others are
  // released when a later event on the same stream completes.  An event is always recorded
  // before the driver blocks and when the user's stream changes.
  void set_event_every(int n) { event_every_ = n < 1 ? 1 : n; }
  int event_every() const { return event_every_; }

  // profiling counters (ns): main time blocked on the ring
  int64_t blocked_ns_ = 0, blocked_calls_ = 0;
  // step_fixed phases (ns): finish+commit of the previous batch, slot acquisition/release, collate launch
  int64_t ph_commit_ns_ = 0, ph_next_ns_ = 0, ph_launch_ns_ = 0, ph_steps_ = 0, events_ = 0;
  // inside the next phase: slot releases (event queries + ring hand-back)
  int64_t rel_ns_ = 0, released_ = 0;
  int64_t cwait_ns_ = 0;  // time spent waiting for a full group while the GPU was busy
  int64_t ahead_groups_ = 0;  // device-decode groups launched ahead of delivery
  int64_t ahead_ns_ = 0;      // host time forming, allocating and launching them (torch_step.cpp)
  int64_t split_launches_ = 0;  // decode launches with each segment split over workgroups (parts > 1)
  // Segments are split over workgroups only under a mirror that waits for its copies: with the
  // no-wait policy (segments whose copy is in flight read from the pinned log) split launches failed
  // the device CRC check at four ranks on one GPU in 4 of 5 runs, while either one workgroup per
  // segment or the waiting mirror passed 6 of 6 each (profiles/r06_s21, r06_s23; the parts merge,
  // the copy-event protocol and SDMA-rewritten lines probed clean alone: tools/probes/*_stress.hip)
  static bool mirror_splits(const LogMirror* m) { return m && m->waits(); }
  int64_t occ_handed_ = 0, occ_staged_ = 0, occ_samples_ = 0;  // slots launched / staged, summed per step

  // Per-iteration constants of the fixed-width fast path (set once by torch_step.cpp's
  // configure_fast; fast_next() then takes no arguments) and its own counters.
  struct FastConfig {
    int device = 0;
    std::vector<int64_t> shape;
    int dst_dt = 0;
    int64_t row = 0;
    const float* shift = nullptr;
    const float* scale = nullptr;
    bool auto_commit = true;
    int64_t timeout_ms = 100;
    bool grouped = true;
    int extras = 0;  // record-field columns per batch (key / timestamp), 0: values only
    bool verify = false;  // verify='deliver': the step returns once the batch's verdict is known
  } fast;
  // The var-len / JSON fast path's constants (torch_step.cpp varlen_fast_next).
  struct VarlenConfig {
    int device = 0;
    int dst_dt = 0;
    int64_t pad_to = -1;  // -1: each batch's longest row (rounded up to pad_multiple)
    int64_t pad_multiple = 1;
    double pad = 0.0;
    bool want_mask = false;
    bool auto_commit = true;
    int64_t timeout_ms = 100;
    bool verify = false;
  } varlen;
  int64_t fast_batches_ = 0, fast_records_ = 0, fast_ns_ = 0;

 private:
  // --- launched slots and their completion events
  struct Handed {
    int64_t g;
    bool ev;            // its own completion event was recorded
    int64_t perr = -1;  // device-checked batch: its status word, read at slot release
    bool span = false;  // decoded from the logs: chain split RecordBatch CRCs at release
    uint64_t stage_end = 0;  // kPackJsonSpan group: staging ring position freed when this slot is released
  };
  void release_completed();
  void release_completed_impl();
  // Teardown: waits for this loader's own work (queued calls, handed slots' events, its decode and
  // copy streams) -- never the device.
  void quiesce() noexcept;
  static constexpr int64_t kReleaseRequeryNs = 3000;
  int64_t pending_query_ns_ = 0;  // when an event was last found pending (release_completed)
  int64_t busy_query_ns_ = 0;     // when gpu_busy() last found the latest launch running
  void note_handed(int64_t g, hipStream_t stream, bool* record);  // decides whether slot g records its event
  void force_event();   // the slot just handed records its event after all
  void cover_handed();  // records an event for the newest handed slot without one
  void switch_stream(hipStream_t stream);  // later launches run on `stream`
  // One group launch on `stream` handed out slots[0..n): the last slot's event (after the kernel)
  // releases them all.  Members from slots[first] on are staged batches (group_idx_) that are now
  // collated ahead of delivery; handles keep their outputs alive.  perrs: status words or null.
  // Returns the launch's sequence number.
  int64_t group_handed(const int* slots, int n, hipStream_t stream, const int64_t* perrs, bool span,
                       std::vector<std::shared_ptr<void>>&& handles, size_t first);
  // `stream` waits for group launch `group` (its last slot's completion event), once per stream.
  void wait_launch(int64_t slot, int64_t group, hipStream_t stream);
  int poll_blocking(int64_t timeout_ms);  // blocks for a slot, releasing completed ones meanwhile
  bool gpu_busy();
  std::deque<Handed> handed_;  // slots whose collate was launched, in launch order
  hipStream_t last_stream_ = nullptr;
  int event_every_ = 1, unevented_ = 0;
  int64_t last_ev_slot_ = -1;  // slot whose completion event was recorded by the latest launch
  int64_t group_seq_ = 0;                // group launches so far
  int64_t waited_group_ = -1;            // the user's stream already waits for this launch ...
  hipStream_t waited_stream_ = nullptr;  // ... (skips repeated waits for one group's batches)

  // --- group formation
  void extend_group();
  bool group_full(uint64_t bytes, const SlotView& next) const {
    return next.span_bytes > 0 && bytes > 0 && bytes + next.span_bytes > group_bytes_max_;
  }
  std::vector<size_t> group_idx_;  // staged indices of the batches behind `last` in the pending group
  int coalesce_ = 1;
  int64_t coalesce_wait_ns_ = 0;
  uint64_t group_bytes_max_ = uint64_t(16) << 20;
  bool group_capped_ = false;  // extend_group stopped at group_bytes_max_
  int ahead_depth_ = 4;  // config 2: depth 0 52.2 M, 3-6 52.3-52.7 M steady, and 54 M over 2000 steps
  int64_t groups_ = 0;
  uint64_t span_launches_ = 0;  // device-decode group launches (they rotate over the decode streams)

  // --- kernel launches
  void copy_extras(const int* slots, const SlotView* const* views, int n, hipStream_t stream);
  void launch_group(const int* slots, const int64_t* rows, const size_t* voffs, int n, const SlotView& v,
                    hipStream_t stream, int dst_dt, void* const* dsts, int64_t row, const float* shift,
                    const float* scale);
  void launch_span(const int* slots, const SlotView* const* views, int n, hipStream_t stream, int dst_dt,
                   void* const* dsts, const float* shift, const float* scale, bool record_last, int64_t* perrs);
  void launch_json_span(const int* slots, const SlotView* const* views, int n, hipStream_t stream, int dst_dt,
                        double pad, void* const* outs, const int64_t* Ls, int64_t* const* lengths,
                        uint8_t* const* masks, bool record_last, int64_t* perrs);
  void launch_var_span(const int* slots, const SlotView* const* views, int n, hipStream_t stream, int dst_dt,
                       double pad, void* const* outs, const int64_t* Ls, int64_t* const* lengths,
                       uint8_t* const* masks, bool record_last, int64_t* perrs);
  // kPackJsonSpan or kPackVarSpan by the views' kind
  void launch_row_span(const int* slots, const SlotView* const* views, int n, hipStream_t stream, int dst_dt,
                       double pad, void* const* outs, const int64_t* Ls, int64_t* const* lengths,
                       uint8_t* const* masks, bool record_last, int64_t* perrs) {
    if (views[0]->kind == uint32_t(tk::kPackVarSpan))
      launch_var_span(slots, views, n, stream, dst_dt, pad, outs, Ls, lengths, masks, record_last, perrs);
    else
      launch_json_span(slots, views, n, stream, dst_dt, pad, outs, Ls, lengths, masks, record_last, perrs);
  }
  const tk::SpanSeg* segs(const SlotView& v) {
    return reinterpret_cast<const tk::SpanSeg*>(poller_->ring().payload(uint32_t(v.g)) + v.values_offset);
  }
  void check_seg_count(const tk::SpanSeg& sg, uint32_t i) const;
  static void fill_seg(SpanDevSeg& d, const tk::SpanSeg& sg, const uint8_t* src, int k, uint32_t i);
  int ext_n_ = 0;  // set_extra_outputs(): destinations of the next launch
  int64_t* ext_dsts_[kMaxGroup] = {};
  // the segment source of a decode launch; *pcie is set when it is not the HBM mirror
  const uint8_t* seg_src(const tk::SpanSeg& sg, bool* pcie) {
    bool hbm = false;
    const uint8_t* s = pins_->seg_src(sg, &hbm);
    *pcie = *pcie || !hbm;
    return s;
  }
  int32_t json_mult_ = 1;
  // a fixed JSON width (json_mult_ 0): the parse kernel counts each row itself, no json_count_kernel
  // launch (TORCHKAFKA_JSON_FUSED_COUNT: 1 on, 0 the separate count kernel)
  bool json_fused_count_ = [] {
    const char* e = std::getenv("TORCHKAFKA_JSON_FUSED_COUNT");
    return e && e[0] == '1';
  }();
  // HBM staging ring of the device JSON parse (row texts between the two kernels, json_span.hip):
  // positions are monotonic, regions are freed in launch order as their groups' slots are released.
  static constexpr uint64_t kStageBytes = uint64_t(128) << 20;
  uint8_t* stage_dev_ = nullptr;
  uint64_t stage_head_ = 0, stage_tail_ = 0, stage_last_end_ = 0;
  uint64_t stage_alloc(uint64_t bytes);

  // --- delivery, fencing and the commit decision
  void stage_finished(int64_t index, std::vector<tk::Watermark>&& wms);
  void settle_parse_errors(bool wait);
  int next_slot_lockstep(int64_t timeout_ms, SlotView* out);
  bool commit_on_device_ = false;
  // (event or null, batch index, watermarks, status word or -1).  A device-checked batch needs no
  // event of its own: it becomes committable once its slot was released (its kernel completed)
  // and its status word read clean.
  std::deque<std::tuple<hipEvent_t, int64_t, std::vector<tk::Watermark>, int64_t>> fenced_;
  std::vector<hipEvent_t> event_pool_;
  std::vector<tk::Watermark> delivered_;
  std::vector<int64_t> delivered_pos_;  // per partition index: position after the batches handed out
  uint64_t delivered_batches_ = 0;
  int64_t delivered_index_ = -1;
  int64_t last_perr_ = -1, delivered_perr_ = -1;
  std::string parse_error_;

  // Cross-rank lockstep: the credit protocol (csrc/core/lockstep.h) over the caller's transport.
  class Source;
  std::unique_ptr<tk::CreditLockstep> ls_;
  bool sync_commit_ = false;

  Engine* eng_;
  bool registered_ = false;
  std::shared_ptr<tk::Ring> ring_keep_;  // the mapping the engine registered: kept until the unregistration ran
  int prefetch_;
  std::shared_ptr<tk::Broker> broker_;
  std::unique_ptr<CommitLedger> ledger_;
  std::unique_ptr<LogPins> pins_;
  std::unique_ptr<RingPoller> poller_;  // owns the ring mapping: destroyed after the members above use it
  std::unique_ptr<BatchVerdicts> verdicts_;
};

}  // namespace tkh
