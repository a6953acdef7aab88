// Ordered HIP command queue executed by a thread of its own, one per loader (Engine::queue();
// TORCHKAFKA_HIP_QUEUE=0 turns them off).
//
// On the device-decode paths the stepping thread spends about a third of each step in HIP calls
// for groups it will hand out later (config 4: three kernel launches and two or three events per
// group of 8 batches, 12-15 us; tools/probes/launch_cost_probe.hip: 3.0-4.8 us per launch).  With
// the queue on, every HIP call the loader makes on the streams only it uses -- the decode streams
// and the HBM mirror's copy streams -- is queued as a closure and run, in submission order, by
// this thread.  The stepping thread keeps everything else: the decisions, the allocations and the
// calls on the user's stream.
//
// Each queued call gets a sequence number.  An event whose record is queued carries the number of
// that record (Engine::done_seq_, LogMirror tags); until the thread has run it, the event counts
// as not complete (no HIP call), and a blocking wait first waits for it to run.  Before the user's
// stream is made to wait for a decoded batch, the batch's record has run -- groups decoded ahead
// were queued long before, so that wait is nearly always free.  Used per loader
// (Engine::set_command_queue): var-len and JSON device decode -- config 4 45.3-50.3 M rec/s against
// 42.7-44.9 M without it on one box, VarLen tokens 43.2 against 41.8 M; fixed-width decode does not
// use it -- its 20-step headline fell 12 % with it (the window's ahead groups are handed to the
// thread and drained after it), its steady state did not move (profiles/r04_s14, r04_s16).
//
// Failures: a call that throws marks the queue failed; the calls queued after it are skipped, and
// every later submit / wait / ran() of THIS queue rethrows the failure -- so a slot whose decode
// launch never ran is never released as done (Engine::slot_done), and a verdict is never read from
// it.  The failure stays with its loader: another loader has a queue of its own.
#pragma once

#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace tkh {

class HipQueue {
 public:
  // A queue whose calls run on `device` (started lazily, at the first queued call).
  explicit HipQueue(int device);
  ~HipQueue();  // runs what was queued, stops the thread (bounded: see shutdown)
  HipQueue(const HipQueue&) = delete;
  HipQueue& operator=(const HipQueue&) = delete;

  // TORCHKAFKA_HIP_QUEUE (on unless "0"), read once per process
  static bool enabled();
  bool on() const { return on_ && !child(); }
  // Queues f (on) or runs it now (off, or a forked child: returns 0).  Returns f's sequence number.
  // Rethrows an earlier failure of this queue.
  uint64_t submit(std::function<void()>&& f);
  // Every call up to `seq` ran (0: nothing to wait for).  Rethrows the failure of this queue.
  void wait(uint64_t seq);
  void drain() { wait(submitted_.load(std::memory_order_acquire)); }
  // Call `seq` ran (a failed queue throws instead of answering: the calls after the failure were
  // skipped, so "ran" would lie about them).
  bool ran(uint64_t seq) const {
    check();
    return seq <= done_.load(std::memory_order_acquire);
  }
  void check() const;  // throws the thread's failure, if any
  int device() const { return device_; }
  uint64_t calls() const { return done_.load(std::memory_order_relaxed); }
  // Runs everything queued, then stops the thread; gives up waiting after `timeout_ms` (logged).
  // Also run for every live queue at process exit (atexit, registered when the first thread
  // starts) -- before the HIP runtime's own teardown, registered earlier.
  void shutdown(int timeout_ms = 10000);

 private:
  void start();
  void run();
  bool child() const;  // this process is a fork of the one that made the queue

  static constexpr uint64_t kCap = 8192;
  bool on_ = false;
  bool started_ = false;
  int device_ = 0;
  uint64_t fork_gen_ = 0;  // the process's fork generation when the queue was made
  std::vector<std::function<void()>> ring_;
  std::mutex push_m_;                      // producers (the stepping thread; the pin thread never queues)
  std::atomic<uint64_t> submitted_{0};     // last sequence number handed out (and published)
  std::atomic<uint64_t> done_{0};          // last sequence number that ran (or was skipped after a failure)
  std::atomic<bool> failed_{false};
  std::atomic<bool> stop_{false}, exited_{false};
  std::atomic<bool> sleeping_{false};
  std::mutex sleep_m_;
  std::condition_variable wake_;
  std::mutex exit_m_;
  std::condition_variable exit_cv_;
  std::string error_;
  std::thread th_;
};

}  // namespace tkh
