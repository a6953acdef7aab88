// Shared-memory slot ring between loader workers and the main process.
//
// Replaces the reference's per-batch path through torch's DataLoader
// (pickled index messages + a freshly allocated shared-memory storage per
// batch + an optional pin-memory thread copy) with one
// fixed POSIX shm segment:
//   * created by the main process BEFORE it forks workers (workers inherit the
//     mapping and never touch HIP; spawn workers re-open it by name);
//   * hipHostRegister()ed once by the main process, so every slot payload is
//     DMA-able pinned memory: workers pack straight into what the GPU copies;
//   * per worker, a FIFO sub-ring of slots cycling FREE -> FILLING -> READY ->
//     INFLIGHT -> FREE; every slot carries the exact per-partition offset
//     watermarks of the records in it (exact commits, fixes reference D3/D5);
//   * futex wake-ups in both directions, no signals (fixes D4/D7).
#pragma once
#include <atomic>
#include <memory>
#include <string>

#include "common.h"

namespace tk {

constexpr uint64_t kRingMagic = 0x31474E49524B54ULL;  // "TKRING1"
constexpr int kMaxWorkers = 64;
constexpr int kMaxSlotParts = 256;
constexpr size_t kSlotHeaderBytes = 16384;

enum SlotState : uint32_t { kSlotFree = 0, kSlotFilling = 1, kSlotReady = 2, kSlotInflight = 3 };
// kSlotDevCount (kPackJsonSpan): the worker walked only the headers; the device counts the elements
// of the rows whose JsonSpanRow::count is kJsonCountOnDevice, and max_row_len is an upper bound.
enum SlotFlags : uint32_t { kSlotEOS = 1, kSlotError = 2, kSlotDevCount = 4 };

struct Watermark {
  uint32_t pidx;
  uint32_t count;        // records consumed from this partition into the slot (incl. skipped)
  int64_t first_offset;  // position before the slot
  int64_t next_offset;   // position after the slot (what a commit stores)
};

struct alignas(64) SlotHeader {
  std::atomic<uint32_t> state;
  uint32_t worker;
  uint64_t seq;
  uint32_t n_rows;
  uint32_t n_parts;
  uint32_t flags;
  uint32_t kind;
  uint64_t payload_bytes;  // bytes to copy host->device, from payload start
  uint64_t values_offset;  // byte offset of the values region in the payload
  uint64_t values_bytes;
  int64_t max_row_len;     // var-len: max elements in a row
  int64_t total_elems;
  int64_t n_scanned;       // records consumed incl. skipped ones
  int64_t t_fill_start_ns;
  int64_t t_ready_ns;
  int64_t t_acquire_wait_ns;  // how long the worker waited for this slot to come back FREE
  uint32_t err_len;
  uint32_t row_bytes;      // fixed-width: bytes per row
  int32_t src_dtype;       // element dtype code of the payload (-1: decided by the loader's schema)
  int32_t ndim;            // sample rank for fixed-width payloads written by the generic path
  uint32_t n_segs;         // kPackRecordSpan / kPackJsonSpan: SpanSeg entries at values_offset
  int32_t trunc_len;       // kPackJsonSpan: rows longer than this are truncated to it (-1: no limit)
  int64_t shape[8];
  char err[2048];
  Watermark wm[kMaxSlotParts];
  // direct (log-gather) slots: bytes of wm[k]'s partition log referenced by this slot, [0, log_end[k])
  uint64_t log_end[kMaxSlotParts];
  // Per-row record fields a schema asked for beside the value (PackSpec::extras): extras_n int64
  // columns of n_rows each (key, then timestamp), at extras_offset in the payload (inside
  // payload_bytes); 0 columns: none.
  uint64_t extras_offset;
  uint32_t extras_n;
  uint32_t extras_pad;
};
static_assert(sizeof(SlotHeader) <= kSlotHeaderBytes, "slot header too large");

struct alignas(64) RingHeader {
  uint64_t magic;
  uint32_t n_workers, slots_per_worker;
  uint64_t slot_stride, payload_capacity, total_bytes;
  std::atomic<uint32_t> shutdown;
  std::atomic<uint32_t> ready_seq;  // futex: bumped on every publish
  std::atomic<uint32_t> ready_waiters;  // main blocked in futex_wait on ready_seq (0/1)
  alignas(64) std::atomic<uint32_t> free_seq[kMaxWorkers];  // futex per worker: bumped on release
  alignas(64) std::atomic<uint32_t> free_waiters[kMaxWorkers];  // worker blocked on free_seq[w]
  alignas(64) std::atomic<int64_t> worker_pid[kMaxWorkers];
};

class Ring {
 public:
  static std::unique_ptr<Ring> create(const std::string& name, uint32_t n_workers, uint32_t slots_per_worker,
                                      uint64_t payload_capacity);
  static std::unique_ptr<Ring> open(const std::string& name);
  ~Ring();

  const std::string& name() const { return name_; }
  RingHeader* header() const { return hdr_; }
  uint8_t* base() const { return base_; }
  size_t total_bytes() const { return len_; }
  uint32_t n_workers() const { return hdr_->n_workers; }
  uint32_t slots_per_worker() const { return hdr_->slots_per_worker; }
  uint32_t n_slots() const { return hdr_->n_workers * hdr_->slots_per_worker; }
  uint64_t payload_capacity() const { return hdr_->payload_capacity; }
  SlotHeader* slot(uint32_t gslot) const;
  uint8_t* payload(uint32_t gslot) const { return reinterpret_cast<uint8_t*>(slot(gslot)) + kSlotHeaderBytes; }
  uint32_t gslot(uint32_t worker, uint32_t i) const { return worker * hdr_->slots_per_worker + i; }

  // ---- worker side: waits until sub-ring slot `i` of `worker` is FREE, marks it FILLING.
  // Returns false on timeout or shutdown.
  bool worker_acquire(uint32_t worker, uint32_t i, int64_t timeout_ms);
  void worker_publish(uint32_t gslot);  // FILLING -> READY (+wake main)

  // ---- main side
  // Waits for the next READY slot.  `cursor` holds the per-worker next index
  // (n_workers entries) and the round-robin position; workers with done[w]
  // set are skipped.  Returns the global slot id, or -1 on timeout.
  int64_t main_acquire(uint32_t* cursor, uint32_t* rr, const uint8_t* done, bool in_order, int64_t timeout_ms);
  void main_release(uint32_t gslot);    // INFLIGHT/READY -> FREE (+wake worker)
  void shutdown();
  void unlink();
  // Worker side: how long worker_acquire spins on a full sub-ring before sleeping (ns).
  void set_worker_spin_ns(int64_t ns) { spin_ns_ = ns < 0 ? 0 : ns; }

 private:
  Ring() = default;
  int64_t spin_ns_ = 200000;
  std::string name_;
  int fd_ = -1;
  uint8_t* base_ = nullptr;
  size_t len_ = 0;
  RingHeader* hdr_ = nullptr;
  bool owner_ = false;
};

// futex helpers on a shared mapping (non-private futexes).
void futex_wait(std::atomic<uint32_t>* addr, uint32_t expected, int64_t timeout_ns);
void futex_wake_all(std::atomic<uint32_t>* addr);

// Bumps `seq` and wakes its waiters, skipping the syscall when nobody sleeps on it.
// Pairs with wait_seq(): both sides use seq_cst, so either the waker sees the
// waiter's registration or the waiter sees the new sequence value (no lost wakeup).
void bump_and_wake(std::atomic<uint32_t>* seq, std::atomic<uint32_t>* waiters);
void wait_seq(std::atomic<uint32_t>* seq, std::atomic<uint32_t>* waiters, uint32_t seen, int64_t timeout_ns);

}  // namespace tk
