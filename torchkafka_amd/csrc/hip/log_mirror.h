// HBM mirror of the pinned partition logs for the device-decode kernels (DeviceLoader h2d='dma'
// with decode='device'; BASELINE config 2's "pinned hipMemcpyAsync H2D overlap").
//
// Zero-copy decode (the default) reads each segment over PCIe from inside the kernel: the
// workgroup holds its CU for the whole transfer.  With the mirror, the copy engines (SDMA) move
// the log bytes into HBM in large chunks ahead of use, on a copy stream of their own, and the
// decode kernels read HBM: the CUs are busy only for the CRC and the decode, which leaves them to
// the model that trains on the batches.  A partition log is mirrored chunk by chunk: chunk c holds
// log bytes [c * C, (c + 1) * C + kSpanSegMax) -- the overlap keeps every segment (<= kSpanSegMax)
// that starts in chunk c whole in one buffer -- in one of K buffers per partition (c % K), copied
// as one hipMemcpyAsync of what is written (plus the next K - 2 chunks as a prefetch, so the copy
// engine always has work queued), topped up when the log grows.  Ordering is all on the GPU: a
// decode stream waits for the copy stream's event before its kernel, and a buffer is
// overwritten only after the copy stream waited for the events of every decode stream that read
// its previous chunk.  A segment whose buffer is still in use by the
// group being formed is served from the pinned log instead (map() returns nullptr).
//
// A launch never waits for a copy (the no-wait policy; JSON / var-len decode): a
// segment is served from HBM only once its chunk's copy is known complete, else from the pinned
// log over PCIe while the copy engines catch up.  A copy stream's completion is learned from one
// event at a time, re-recorded at its tail once the previous one completed.  Waiting instead made
// a launch that caught up with the copies wait for the copy stream's whole queue -- the needed
// chunk and every prefetch queued behind it (up to (K - 2) chunks per partition of that stream):
// config-4 mirror runs then ranged 38-50 M rec/s on one box (profiles/r04_s1/c4_dma_*.log).
//
// Back-off: when the copy engines fall behind the decode (more than half of a window of kEvalMaps
// segments found their copy in flight), every byte crosses PCIe twice -- once copied, once read by
// the kernel that could not wait for it -- and the loader ran at half the zero-copy rate (27 M
// against 50 M rec/s, fixed-width under the RCCL lockstep with one copy stream: 188 000 of 188 000
// segments fell back, profiles/r05_s35).  The mirror then stops copying for kBackoffMaps segments
// (served from the pinned log, as zero-copy), the copy queue drains, and it starts again ahead of
// the read position.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <functional>
#include <vector>

#include "hip_queue.h"
#include "span.h"

namespace tkh {

inline constexpr uint64_t tk_seg_max() { return tk::kSpanSegMax; }

class LogMirror {
 public:
  // The driver registers (pins) partition logs in pieces of this many bytes, at multiples of it
  // (MainDriver::kLogChunk): one copy never spans two registrations.
  static constexpr uint64_t kRegAlign = uint64_t(64) << 20;
  // copy_streams: SDMA copy streams (partitions split p % n); TORCHKAFKA_MIRROR_COPY_STREAMS when
  // set, else copy_streams when > 0, else 2.  Each takes one of the process's hardware queues.
  // `queue`: the loader's HIP command queue (Engine::queue), used once set_command_queue(true)
  // wait: 1 a launch waits for a copy in flight (the stream waits on the copy stream's event), 0
  // the no-wait policy below, -1 the default (0); TORCHKAFKA_MIRROR_WAIT=0/1 overrides either.
  LogMirror(int device, HipQueue* queue, uint64_t chunk_bytes, int chunks_per_partition, int copy_streams = 0,
            int wait = -1);
  bool waits() const { return wait_; }
  ~LogMirror();
  // The mirror's HIP calls go through the HIP command queue (hip_queue.h) when on.
  void set_command_queue(bool on);
  int copy_streams() const { return int(cs_.size()); }
  LogMirror(const LogMirror&) = delete;
  LogMirror& operator=(const LogMirror&) = delete;

  // Device address of log bytes [pos, pos + len) of partition `pidx` (`log`: its pinned host base;
  // bytes [0, pinned) are pinned and written), copying their chunk first when needed.  nullptr:
  // not mirrored for this launch -- read the pinned log.
  const uint8_t* map(uint32_t pidx, uint64_t pos, uint32_t len, const uint8_t* log, uint64_t pinned);
  // Before the launch that reads what map() returned on `stream`: `stream` waits for the copies.
  void before(hipStream_t stream);
  // After that launch: the buffers it reads are released once `stream` passes this point.
  void after(hipStream_t stream);

  uint64_t chunk_bytes() const { return chunk_; }
  // log bytes from a mapped position that the mirror may copy (the chunk and its prefetches)
  uint64_t span_bytes() const { return chunk_ * uint64_t(prefetch_ + 1) + tk_seg_max(); }
  uint64_t bytes_copied() const { return bytes_; }
  uint64_t copies() const { return copies_; }
  uint64_t fallbacks() const { return fallbacks_; }
  uint64_t pending_fallbacks() const { return pending_fallbacks_; }  // served from the log: copy in flight
  uint64_t backoffs() const { return backoffs_; }  // times the mirror stopped copying (header)
  void reset_stats() { bytes_ = copies_ = fallbacks_ = pending_fallbacks_ = backoffs_ = 0; }
  uint64_t device_bytes() const { return dev_bytes_; }

 private:
  static constexpr int kStreams = 8;  // distinct reader streams remembered per buffer
  struct Reader {
    hipStream_t stream = nullptr;
    int ev = -1;        // pool index
    uint64_t seq = 0;   // pool_seq_[ev] when recorded; a newer value means it completed
  };
  struct Buf {
    int64_t chunk = -1;
    int s = 0;               // the copy stream that fills it (its partition's)
    uint64_t end = 0;        // log position up to which the buffer holds the chunk's bytes
    uint64_t copy_seq = 0;   // copy that brought in its latest bytes
    bool pending = false;    // mapped for the launch being formed
    Reader readers[kStreams];
  };
  struct Part {
    uint8_t* dev = nullptr;
    std::vector<Buf> bufs;
  };
  Part& part(uint32_t pidx);
  Buf* ensure(Part& P, uint32_t pidx, int64_t c, uint64_t want_end, const uint8_t* log, uint64_t pinned,
              bool prefetch);
  void retarget(Buf& b, int64_t c);
  int next_event();
  void issue_prefetches();
  struct Deferred {
    uint32_t pidx;
    int64_t chunk;
    const uint8_t* log;
    uint64_t pinned;
  };
  std::vector<Deferred> deferred_;  // prefetches of the launch being formed, queued after its copy event

  int device_;
  uint64_t chunk_, stride_;
  int K_;
  int prefetch_ = 1;  // chunks copied ahead of the one being read
  // Copy streams: partition p is copied on stream p % S.  A buffer is refilled only after the
  // copy stream waited for the readers of its previous chunk; with one stream that wait holds up
  // every partition's copies behind it, with S it holds up only its own partitions'.
  // TORCHKAFKA_MIRROR_COPY_STREAMS (1..4, default 2).
  struct CopyStream {
    hipStream_t stream = nullptr;
    hipEvent_t copied = nullptr;  // recorded after the latest copy (when a launch needs it)
    uint64_t seq = 0, recorded = 0, done = 0;
    bool queried = false;  // its event was queried for the launch being formed
    uint64_t rec_q = 0;    // HIP command-queue number of the latest record of `copied` (hip_queue.h)
  };
  // no-wait mode: what the copy stream has completed (one query per launch), and a fresh event
  // at its tail once the last one completed
  void learn(CopyStream& c);
  bool copied_done(CopyStream& c);   // its latest record ran and completed
  // f (HIP calls on the copy or decode streams) through the command queue when set_command_queue
  // turned it on, else now; returns its queue number (0: ran now)
  uint64_t issue(std::function<void()>&& f);
  bool cq_ = false;
  HipQueue* q_ = nullptr;  // the loader's command queue
  void record_copied(CopyStream& c);  // records `copied` at the stream's tail (queued when the queue is on)
  bool wait_ = false;
  uint64_t pending_fallbacks_ = 0;
  // back-off (header): segments mapped / found in flight in the current window, segments left to
  // serve from the pinned log
  static constexpr uint32_t kEvalMaps = 512, kBackoffMaps = 8192;
  uint32_t eval_maps_ = 0, eval_pending_ = 0, backoff_left_ = 0;
  uint64_t backoffs_ = 0;
  std::vector<CopyStream> cs_;
  CopyStream& cs_of(uint32_t pidx) { return cs_[pidx % cs_.size()]; }
  std::vector<Part> parts_;
  std::vector<std::pair<uint32_t, int>> pending_;
  std::vector<hipEvent_t> pool_;
  std::vector<uint64_t> pool_seq_;
  std::vector<uint64_t> pool_rec_q_;  // HIP command-queue number of each pool event's latest record
  std::vector<int> pool_refs_;
  size_t pool_next_ = 0;
  uint64_t bytes_ = 0, copies_ = 0, fallbacks_ = 0, dev_bytes_ = 0;
};

}  // namespace tkh
