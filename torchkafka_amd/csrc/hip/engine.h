#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>
#include <functional>
#include <memory>
#include <vector>

#include "hip_queue.h"

namespace tkh {

struct SpanLaunch;      // span_decode.h
struct JsonStageLaunch;

// How a ring slot's bytes reach the collate kernel.
enum H2DMode : int {
  kH2DDma = 0,       // hipMemcpyAsync (SDMA engine) into a device staging buffer, then the kernel
  kH2DZeroCopy = 1,  // the kernel reads the pinned slot straight over PCIe (no copy, no staging)
};

class Engine {
 public:
  Engine(int device, int n_slots, size_t staging_bytes, int n_streams = 4, int mode = kH2DDma);
  ~Engine();
  Engine(const Engine&) = delete;
  Engine& operator=(const Engine&) = delete;

  int device() const { return device_; }
  int n_slots() const { return n_slots_; }
  int mode() const { return mode_; }
  size_t staging_stride() const { return stride_; }
  void* staging(int s) const { return static_cast<uint8_t*>(staging_) + stride_ * size_t(s); }
  hipStream_t stream_of_slot(int s) const { return streams_[size_t(s) % streams_.size()]; }

  void register_host(void* p, size_t len);
  void unregister_host();
  // Hands the unregistration to the deferred-release thread (reaper.h) after this engine's own
  // streams drained; `keep` holds the registered mapping until it ran.
  void unregister_host_deferred(std::shared_ptr<void> keep);
  bool host_registered() const { return host_ptr_ != nullptr; }

  // DMA mode: start the slot's copy (its stream runs the slot's kernel after it).
  // Zero-copy mode: no-op.  `host` must lie in the registered region.
  void h2d(int s, const void* host, size_t nbytes);
  // True once the slot's kernel completed: the host slot and its staging buffer are reusable.
  bool slot_done(int s);
  void wait_slot(int s);
  void wait_copy(int s);  // DMA mode: the slot's copy has finished reading host memory
  // Launch the collate of slot `s` on the user's stream (after the slot's copy in DMA mode).
  // `record` = false skips the slot's completion event: a later slot's event on the same
  // stream (record_done) then stands for it (the driver batches events this way).
  void collate_fixed(int s, hipStream_t user, size_t values_offset, int src_dt, void* dst, int dst_dt, int64_t rows,
                     int64_t row, const float* shift, const float* scale, bool record = true);
  void collate_varlen(int s, hipStream_t user, size_t values_offset, int src_dt, void* out, int dst_dt, int64_t rows,
                      int64_t L, double pad, int64_t* lengths, uint8_t* mask, bool record = true);
  // kPackJsonText slot: rows parsed from JSON text on the device (json_parse.hip); a grammar
  // error stores the row index into *err (host-mapped).
  void collate_json(int s, hipStream_t user, size_t values_offset, void* out, int dst_dt, int64_t rows, int64_t L,
                    double pad, int64_t* lengths, uint8_t* mask, int32_t* err, bool record = true);
  // Up to kMaxGroup kPackJsonText slots parsed by one kernel; the completion event of the last
  // slot is recorded (it stands for all of them).
  void collate_json_group(const int* slots, int n, hipStream_t user, const size_t* values_offsets, const int64_t* rows,
                          void* const* outs, const int64_t* Ls, int64_t* const* lengths, uint8_t* const* masks,
                          int32_t* const* errs, double pad, int dst_dt);
  // Consecutive fixed-width slots collated by one kernel (collate.h launch_fixed_group);
  // the completion event of the last slot is recorded (it stands for all of them).
  void collate_fixed_group(const int* slots, int n, hipStream_t user, const size_t* values_offsets, int src_dt,
                           void* const* dsts, int dst_dt, const int64_t* rows, int64_t row, const float* shift,
                           const float* scale);
  // Log-gather slots (h2d="direct"): each slot's payload is its gather table; rows are read from
  // the pinned broker logs through `bases` (device table, one address per partition index).
  void collate_gather_group(const int* slots, int n, hipStream_t user, int src_dt, void* const* dsts, int dst_dt,
                            const int64_t* rows, int64_t row_bytes, const uint64_t* bases, const float* shift,
                            const float* scale, bool record = true);
  // Device decode (kPackRecordSpan, span_decode.hip): `a` lists the segments of up to kMaxGroup
  // slots (a.b[k].row_pos is filled in here from slots[k]); records the completion event of
  // slots[n - 1] when `record`.  The log bytes are read from the pinned broker logs.
  void collate_span(const int* slots, int n, hipStream_t user, SpanLaunch& a, int src_dt, int dst_dt,
                    const float* shift, const float* scale, bool record = true);
  // Device JSON parse from the logs (kPackJsonSpan, json_span.hip), first kernel: stage + CRC +
  // row texts into HBM (a.b[k].rows / .slot are filled in here from slots[k]); the driver then
  // launches json_rows_kernel over the descriptors and records the completion event.
  void collate_json_stage(const int* slots, int n, hipStream_t user, JsonStageLaunch& a);
  // Where a kernel launched on `user` reads slot s's payload (DMA mode: after its copy; the
  // stream waits for it).
  const uint8_t* slot_src(int s, hipStream_t user) {
    check_slot(s);
    begin(s, user);
    return src_base(s);
  }
  // Device copy of the CRC tables of the span kernel (uploaded on first use).
  const uint32_t* span_tables();
  // Workgroups per span segment (TORCHKAFKA_SPAN_PARTS: 1, 2, 4 or 8; span_device.h Part) and the
  // accumulator words the parts of the next launch on `stream` meet in: zeroed once, left zero by
  // every launch, and handed out in rotation over kPartAccSets sets per stream -- the dispatches of
  // one stream may overlap (a launch's first workgroups start before the previous launch's last
  // ones finished), so consecutive launches must not share words.  64 sets (24 KiB per stream): a
  // set comes back only after 63 later launches on its stream were handed theirs.
  static constexpr int kPartAccSets = 64;
  int span_parts() const { return span_parts_; }
  // The JSON stage kernel keeps one workgroup per segment unless TORCHKAFKA_SPAN_PARTS is set: its
  // parts each redo the segment's row scan (config 4 through the mirror: 47-50 M with 4 parts
  // against 51-52 M with 1, profiles/r05_s23).
  int json_span_parts() const { return json_parts_; }
  uint32_t* part_acc(hipStream_t stream);
  // The streams device-decode groups rotate over (created on first use; kDecodeStreams).
  hipStream_t decode_stream(int k);
  int decode_streams() const { return n_decode_; }
  int copy_streams() const { return int(streams_.size()); }  // 0 in zero-copy mode
  // number of decode streams (1..4); only before the first decode stream is created
  void set_decode_streams(int n);
  // Creates the decode streams, uploads the CRC tables and runs an empty kernel on every decode
  // stream (the runtime binds a stream to a hardware queue at its first launch), so none of that
  // lands on the first batches of an iteration.
  void prepare_decode();
  // `later` runs after everything queued on `earlier` so far (an event on `earlier`).
  void stream_after(hipStream_t later, hipStream_t earlier);
  // `user` waits for slot s's completion event (a batch collated on another stream).
  void stream_wait_done(int s, hipStream_t user);
  void record_done(int s, hipStream_t user) { finish(s, user); }
  // Runs f -- HIP calls on `stream` -- now, or through the HIP command queue when `stream` is a
  // decode stream and the queue is on (hip_queue.h).
  void run_on(hipStream_t stream, std::function<void()>&& f);
  bool queued(hipStream_t stream) const;  // calls on `stream` go through the command queue
  // Whether this engine's decode-stream calls use the command queue (set per loader: var-len and
  // JSON device decode; fixed-width decode keeps its calls on the stepping thread).
  void set_command_queue(bool on);
  // This engine's (this loader's) HIP command queue (hip_queue.h).
  HipQueue& queue() { return *q_; }
  void copy_raw(int s, hipStream_t user, size_t offset, void* dst, size_t nbytes);
  // The same without the slot's completion event: a kernel queued after it on `user` records it.
  void copy_bytes(int s, hipStream_t user, size_t offset, void* dst, size_t nbytes);
  void synchronize();

  // legacy names used by tests
  bool h2d_complete(int s) { return slot_done(s); }
  void wait_h2d(int s) { wait_slot(s); }
  hipStream_t copy_stream() const { return streams_.empty() ? nullptr : streams_[0]; }

 private:
  void check_slot(int s) const;
  const uint8_t* src_base(int s) const;  // where slot s's payload is read from by kernels
  void begin(int s, hipStream_t user);
  void finish(int s, hipStream_t user);

  int device_;
  int n_slots_;
  int mode_;
  size_t stride_ = 0;
  void* staging_ = nullptr;
  std::vector<hipStream_t> streams_;
  std::vector<hipEvent_t> done_, copied_;
  std::vector<uint64_t> done_seq_;  // command-queue number of each done_ record (0: recorded directly)
  bool cq_ = false;                 // set_command_queue
  std::unique_ptr<HipQueue> q_;     // made with the engine; its thread starts at the first queued call
  std::vector<const uint8_t*> host_src_;  // per slot: host payload pointer given at h2d()
  void* host_ptr_ = nullptr;
  uint8_t* host_dev_ = nullptr;           // device view of the registered host region (zero-copy)
  size_t host_len_ = 0;
  uint32_t* span_tabs_ = nullptr;
  int span_parts_ = 8;  // HBM-sourced fixed-width / var-len launches (profiles/r05_s30_lane_merge)
  int json_parts_ = 1;
  struct PartAcc {
    hipStream_t stream;
    uint32_t* words;
    uint64_t next;
  };
  std::vector<PartAcc> part_acc_;
  hipStream_t decode_streams_[4] = {nullptr, nullptr, nullptr, nullptr};
  int n_decode_ = default_decode_streams();
  static int default_decode_streams();

 public:
  // 1: decode streams at the device's greatest stream priority, 0: HIP's default, -1: the least
  static int decode_priority();
  static constexpr int kDefaultDecodePriority = 0;

 private:
  std::vector<hipEvent_t> order_events_;  // stream_after: a small pool used round-robin
  size_t order_next_ = 0;
};

}  // namespace tkh
