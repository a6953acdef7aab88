#include "hip_queue.h"

#include <hip/hip_runtime_api.h>

#include <chrono>
#include <cstdlib>
#include <ctime>
#include <stdexcept>

#include <pthread.h>

#include "common.h"

namespace tkh {

HipQueue& HipQueue::get() {
  static HipQueue* q = new HipQueue();  // leaked on purpose: no teardown race with the HIP runtime
  return *q;
}

HipQueue::HipQueue() {
  const char* e = std::getenv("TORCHKAFKA_HIP_QUEUE");  // on unless "0"
  on_ = !(e && e[0] == '0');
  if (on_) ring_.resize(kCap);
  // DataLoader workers are forked from the loader's process: the thread does not survive a fork,
  // so in the child every call runs inline (the workers make no HIP calls; this is a guard)
  pthread_atfork(nullptr, nullptr, [] {
    HipQueue& q = get();
    q.on_ = false;
    q.child_ = true;
  });
}

void HipQueue::start() {
  if (hipGetDevice(&device_) != hipSuccess) device_ = 0;
  th_ = std::thread([this] { run(); });
  th_.detach();
  started_ = true;
  std::atexit([] { get().shutdown(); });
}

void HipQueue::shutdown() {
  if (child_ || !started_) return;
  try {
    drain();
  } catch (...) {
  }
  stop_.store(true, std::memory_order_seq_cst);
  {
    std::lock_guard<std::mutex> g(sleep_m_);
    wake_.notify_one();
  }
  for (int i = 0; i < 100000 && !exited_.load(std::memory_order_acquire); ++i) std::this_thread::yield();
}

uint64_t HipQueue::submit(std::function<void()>&& f) {
  if (!on_) {
    f();
    return 0;
  }
  check();
  uint64_t seq;
  {
    std::lock_guard<std::mutex> g(push_m_);
    if (!started_) start();
    const uint64_t last = submitted_.load(std::memory_order_relaxed);
    if (sleeping_.load(std::memory_order_seq_cst) && done_.load(std::memory_order_acquire) == last) {
      // the thread is asleep with nothing queued (a pause between iterations, a synchronize): run
      // f here -- waiting for the thread to wake would delay it by tens of microseconds -- and wake
      // the thread for the calls that follow
      f();
      std::lock_guard<std::mutex> w(sleep_m_);
      wake_.notify_one();
      return 0;
    }
    seq = last + 1;
    while (seq - done_.load(std::memory_order_acquire) > kCap) tk::cpu_relax();  // full: the thread catches up
    ring_[seq % kCap] = std::move(f);
    submitted_.store(seq, std::memory_order_seq_cst);
  }
  // seq_cst on both sides (here and in run()): the thread either sees this submission before it
  // sleeps or is seen asleep here and woken
  if (sleeping_.load(std::memory_order_seq_cst)) {
    std::lock_guard<std::mutex> g(sleep_m_);
    wake_.notify_one();
  }
  return seq;
}

void HipQueue::check() const {
  if (failed_.load(std::memory_order_acquire)) throw std::runtime_error("HIP command queue: " + error_);
}

void HipQueue::wait(uint64_t seq) {
  if (seq == 0) return;
  for (int i = 0; done_.load(std::memory_order_acquire) < seq; ++i) {
    check();
    if (i < 20000)
      tk::cpu_relax();
    else
      std::this_thread::yield();
  }
  check();
}

void HipQueue::run() {
  (void)hipSetDevice(device_);  // a failure shows in the first queued call
  uint64_t next = 1;
  int idle = 0;
  while (!stop_.load(std::memory_order_acquire)) {
    if (submitted_.load(std::memory_order_acquire) >= next) {
      std::function<void()> f = std::move(ring_[next % kCap]);
      ring_[next % kCap] = nullptr;
      if (!failed_.load(std::memory_order_relaxed)) {
        try {
          f();
        } catch (const std::exception& ex) {
          error_ = ex.what();
          failed_.store(true, std::memory_order_release);
        }
      }
      done_.store(next, std::memory_order_release);
      ++next;
      idle = 0;
      continue;
    }
    if (++idle < 4000) {  // a few hundred microseconds of spinning: steps come every few microseconds
      tk::cpu_relax();
      continue;
    }
    std::unique_lock<std::mutex> lk(sleep_m_);
    sleeping_.store(true, std::memory_order_seq_cst);
    // the timeout is a safety net only (the seq_cst hand-off above loses no wake-up); it is taken
    // against the system clock -- pthread_cond_timedwait, which ThreadSanitizer follows (the
    // steady-clock wait_for calls pthread_cond_clockwait, which GCC 11's TSan does not intercept:
    // it then reports the sleeping thread as still holding sleep_m_)
    if (submitted_.load(std::memory_order_seq_cst) < next)
      wake_.wait_until(lk, std::chrono::system_clock::now() + std::chrono::milliseconds(5));
    sleeping_.store(false, std::memory_order_release);
    idle = 0;
  }
  exited_.store(true, std::memory_order_release);
}

}  // namespace tkh
