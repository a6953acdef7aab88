#include "hip_queue.h"

#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <ctime>
#include <stdexcept>

#include <pthread.h>

#include "common.h"

namespace tkh {

namespace {

// Forks seen by this process image: a queue made before a fork belongs to the parent (its thread
// did not survive into the child).  DataLoader workers are forked from the loader's process; they
// make no HIP calls, so in a child every call runs inline and waits return at once (a guard).
std::atomic<uint64_t> g_fork_gen{0};

// Live queues, shut down at process exit before the HIP runtime tears down.
std::mutex g_live_m;
std::vector<HipQueue*>* g_live = nullptr;  // leaked on purpose: atexit may run after static teardown
bool g_atexit = false;

void register_live(HipQueue* q) {
  std::lock_guard<std::mutex> g(g_live_m);
  if (!g_live) g_live = new std::vector<HipQueue*>();
  g_live->push_back(q);
  if (!g_atexit) {
    g_atexit = true;
    std::atexit([] {
      std::vector<HipQueue*> qs;
      {
        std::lock_guard<std::mutex> g(g_live_m);
        if (g_live) qs = *g_live;
      }
      for (HipQueue* q : qs) q->shutdown();
    });
  }
}

void unregister_live(HipQueue* q) {
  std::lock_guard<std::mutex> g(g_live_m);
  if (g_live) g_live->erase(std::remove(g_live->begin(), g_live->end(), q), g_live->end());
}

}  // namespace

bool HipQueue::enabled() {
  static const bool on = [] {
    const char* e = std::getenv("TORCHKAFKA_HIP_QUEUE");  // on unless "0"
    pthread_atfork(nullptr, nullptr, [] { g_fork_gen.fetch_add(1, std::memory_order_relaxed); });
    return !(e && e[0] == '0');
  }();
  return on;
}

HipQueue::HipQueue(int device) : on_(enabled()), device_(device), fork_gen_(g_fork_gen.load()) {
  if (on_) ring_.resize(kCap);
}

HipQueue::~HipQueue() {
  if (started_ && !child()) {
    shutdown();
    unregister_live(this);
  }
}

bool HipQueue::child() const { return g_fork_gen.load(std::memory_order_relaxed) != fork_gen_; }

void HipQueue::start() {
  th_ = std::thread([this] { run(); });
  started_ = true;
  register_live(this);
}

void HipQueue::shutdown(int timeout_ms) {
  if (child() || !started_ || !th_.joinable()) return;
  try {
    drain();
  } catch (...) {
  }
  stop_.store(true, std::memory_order_seq_cst);
  {
    std::lock_guard<std::mutex> g(sleep_m_);
    wake_.notify_one();
  }
  std::unique_lock<std::mutex> lk(exit_m_);
  // system clock: pthread_cond_timedwait, which ThreadSanitizer follows (see run())
  const bool stopped = exit_cv_.wait_until(lk, std::chrono::system_clock::now() + std::chrono::milliseconds(timeout_ms),
                                           [this] { return exited_.load(std::memory_order_acquire); });
  lk.unlock();
  if (stopped) {
    th_.join();
  } else {
    // still inside a HIP call: leave it running rather than hang the process
    std::fprintf(stderr, "[torchkafka] HIP command queue thread did not stop within %d ms; detached\n", timeout_ms);
    th_.detach();
  }
}

uint64_t HipQueue::submit(std::function<void()>&& f) {
  if (!on_ || child()) {
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
  if (seq == 0 || child()) return;
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
  tk::name_thread("tk-hip-queue");
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
    if (submitted_.load(std::memory_order_seq_cst) < next && !stop_.load(std::memory_order_acquire))
      wake_.wait_until(lk, std::chrono::system_clock::now() + std::chrono::milliseconds(5));
    sleeping_.store(false, std::memory_order_release);
    idle = 0;
  }
  {
    std::lock_guard<std::mutex> g(exit_m_);
    exited_.store(true, std::memory_order_release);
  }
  exit_cv_.notify_all();
}

}  // namespace tkh
