#include "reaper.h"

#include <hip/hip_runtime_api.h>
#include <unistd.h>

#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <deque>
#include <mutex>
#include <thread>
#include <utility>

namespace tkh {

namespace {

struct Item {
  int device;
  std::function<void()> fn;
};

struct State {
  std::mutex m;
  std::condition_variable cv, done_cv;
  std::deque<Item> q;
  uint64_t posted = 0, released = 0;
  bool started = false, stop = false;
  pid_t owner = 0;  // the process whose thread this is (a forked child has none)
  std::thread th;
};

State& state() {
  static State* s = new State();  // leaked on purpose: atexit may run after static teardown
  return *s;
}

void run() {
  State& s = state();
  std::unique_lock<std::mutex> lk(s.m);
  while (true) {
    s.cv.wait(lk, [&] { return s.stop || !s.q.empty(); });
    if (s.q.empty()) break;  // stop, and nothing left
    Item it = std::move(s.q.front());
    s.q.pop_front();
    lk.unlock();
    (void)hipSetDevice(it.device);
    try {
      it.fn();
    } catch (...) {  // a release that fails leaks; nothing can be done about it at teardown
    }
    it.fn = nullptr;  // drop what the closure kept alive outside the lock
    lk.lock();
    ++s.released;
    s.done_cv.notify_all();
  }
}

void shutdown_at_exit() {
  State& s = state();
  {
    std::lock_guard<std::mutex> g(s.m);
    if (!s.started || s.owner != getpid()) return;
  }
  Reaper::drain(10000);
  {
    std::lock_guard<std::mutex> g(s.m);
    s.stop = true;
  }
  s.cv.notify_all();
  std::unique_lock<std::mutex> lk(s.m);
  const bool idle = s.done_cv.wait_for(lk, std::chrono::seconds(5), [&] { return s.q.empty(); });
  lk.unlock();
  if (idle && s.th.joinable()) {
    s.th.join();
  } else if (s.th.joinable()) {
    std::fprintf(stderr, "[torchkafka] deferred-release thread still busy at exit; detached\n");
    s.th.detach();
  }
}

}  // namespace

bool Reaper::enabled() {
  static const bool on = [] {
    const char* e = std::getenv("TORCHKAFKA_DEFERRED_FREE");
    return !(e && e[0] == '0');
  }();
  return on;
}

void Reaper::post(int device, std::function<void()> fn) {
  State& s = state();
  const pid_t me = getpid();
  {
    std::lock_guard<std::mutex> g(s.m);
    if (s.started && s.owner != me) return;  // a forked child: the parent's HIP state is not ours
    if (enabled() && !s.stop) {
      if (!s.started) {
        s.started = true;
        s.owner = me;
        s.th = std::thread(run);
        std::atexit(shutdown_at_exit);
      }
      ++s.posted;
      s.q.push_back(Item{device, std::move(fn)});
      s.cv.notify_one();
      return;
    }
  }
  (void)hipSetDevice(device);
  try {
    fn();
  } catch (...) {
  }
}

bool Reaper::drain(int timeout_ms) {
  State& s = state();
  std::unique_lock<std::mutex> lk(s.m);
  if (!s.started || s.owner != getpid()) return true;
  const uint64_t want = s.posted;
  return s.done_cv.wait_for(lk, std::chrono::milliseconds(timeout_ms), [&] { return s.released >= want; });
}

uint64_t Reaper::posted() {
  std::lock_guard<std::mutex> g(state().m);
  return state().posted;
}

uint64_t Reaper::released() {
  std::lock_guard<std::mutex> g(state().m);
  return state().released;
}

void Reaper::free_device(int device, void* p) {
  if (p) post(device, [p] { (void)hipFree(p); });
}

void Reaper::free_host(int device, void* p) {
  if (p) post(device, [p] { (void)hipHostFree(p); });
}

}  // namespace tkh
