// Host test of the HIP command queue (torchkafka_amd/csrc/hip/hip_queue.h), run under
// ThreadSanitizer and AddressSanitizer by tools/sanitize.sh.  The two device calls the queue's
// thread makes are stubbed below, so no GPU is needed.  Checks: calls run in submission order;
// wait(seq) returns once call seq ran; a call made while the thread sleeps with nothing queued runs
// inline on the caller, and the calls after it run on the thread again; a failing call is reported
// to the caller -- and every later ran() / wait() / submit() of that queue throws (a slot whose
// launch was skipped is never reported done), while another loader's queue keeps working; a
// queue's destructor stops its thread.
#include <hip/hip_runtime_api.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <stdexcept>
#include <string>
#include <thread>

#include "hip_queue.h"

extern "C" hipError_t hipGetDevice(int* d) {
  *d = 0;
  return hipSuccess;
}
extern "C" hipError_t hipSetDevice(int) { return hipSuccess; }

#define CHECK(c)                                                                  \
  do {                                                                            \
    if (!(c)) {                                                                   \
      std::fprintf(stderr, "hip_queue_test FAILED %s:%d: %s\n", __FILE__, __LINE__, #c); \
      return 1;                                                                   \
    }                                                                             \
  } while (0)

int main(int argc, char** argv) {
  const int n = argc > 1 ? std::atoi(argv[1]) : 200000;
  tkh::HipQueue q(0);
  CHECK(q.on());

  // 1. order: every call sees exactly its predecessors' effects; waits at random points
  std::atomic<int> next{0};
  std::atomic<bool> order_ok{true};
  for (int i = 0; i < n; ++i) {
    const uint64_t s = q.submit([i, &next, &order_ok] {
      if (next.load(std::memory_order_relaxed) != i) order_ok.store(false, std::memory_order_relaxed);
      next.store(i + 1, std::memory_order_relaxed);
    });
    if (i % 997 == 0) {
      q.wait(s);
      CHECK(next.load(std::memory_order_relaxed) >= i + 1);
    }
  }
  q.drain();
  CHECK(next.load() == n);
  CHECK(order_ok.load());

  // 2. a call submitted while the thread sleeps with nothing queued runs inline on the caller
  bool inline_seen = false;
  for (int tries = 0; tries < 200 && !inline_seen; ++tries) {
    std::this_thread::sleep_for(std::chrono::milliseconds(20));  // the thread spins briefly, then sleeps
    std::thread::id ran_on;
    const uint64_t s = q.submit([&ran_on] { ran_on = std::this_thread::get_id(); });
    q.wait(s);
    if (s == 0) {
      CHECK(ran_on == std::this_thread::get_id());
      inline_seen = true;
    }
  }
  CHECK(inline_seen);
  // ... and the thread, woken by it, takes the calls that follow
  std::atomic<int> after{0};
  for (int i = 0; i < 1000; ++i) q.submit([&after] { after.fetch_add(1, std::memory_order_relaxed); });
  q.drain();
  CHECK(after.load() == 1000);

  // 3. a failing call is reported to the caller (from submit when it ran inline, else from wait)
  bool reported = false;
  try {
    const uint64_t s = q.submit([] { throw std::runtime_error("boom"); });
    q.wait(s);
  } catch (const std::runtime_error& e) {
    reported = std::string(e.what()).find("boom") != std::string::npos;
  }
  CHECK(reported);

  // 4. after the failure the queue answers nothing: a later call was skipped, and ran() of it (or of
  // any number) throws instead of reporting it done; so do wait() and submit()
  tkh::HipQueue f(0);
  std::atomic<bool> skipped_ran{false};
  uint64_t s_bad = 0, s_after = 0;
  for (int tries = 0; tries < 100 && s_bad == 0; ++tries) {
    // queue behind a slow call, so the failing call and the one after it run on the thread
    f.submit([] { std::this_thread::sleep_for(std::chrono::milliseconds(5)); });
    s_bad = f.submit([] { throw std::runtime_error("launch failed"); });
  }
  CHECK(s_bad != 0);
  s_after = f.submit([&skipped_ran] { skipped_ran.store(true); });
  auto throws = [](auto&& fn) {
    try {
      fn();
    } catch (const std::runtime_error& e) {
      return std::string(e.what()).find("launch failed") != std::string::npos;
    }
    return false;
  };
  CHECK(throws([&] { f.wait(s_after); }));
  CHECK(!skipped_ran.load());
  CHECK(throws([&] { (void)f.ran(s_after); }));
  CHECK(throws([&] { (void)f.ran(1); }));
  CHECK(throws([&] { f.submit([] {}); }));
  CHECK(throws([&] { f.drain(); }));

  // 5. another loader's queue is not affected, and a destroyed queue stops its thread
  {
    tkh::HipQueue g(0);
    std::atomic<int> ok{0};
    for (int i = 0; i < 100; ++i) g.submit([&ok] { ok.fetch_add(1); });
    g.drain();
    CHECK(ok.load() == 100);
    CHECK(g.ran(1));
  }
  std::printf("hip_queue_test: ok (%d ordered calls, inline path, failure report, failed-queue answers, "
              "per-loader queues)\n", n);
  return 0;
}
