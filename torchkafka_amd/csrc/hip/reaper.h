// Deferred release of device and pinned-host memory (VERDICT r4 "do this" 9).
//
// hipFree, hipHostFree and hipHostUnregister wait for the whole device -- every stream of every
// user -- before they return (profiles/r05_s8_span_kernels/sync_probe.json: ~170 ms behind a
// 200 ms kernel on another stream).  A loader closed while the training job's stream holds a step
// of work would block the training thread on that step.  So a loader's teardown waits for its own
// streams only (MainDriver::quiesce) and hands its allocations and registrations here; one
// process-wide thread releases them, in order.  What a release needs alive (the broker mapping a
// log registration covers, the ring mapping the engine registered) is captured by the closure.
//
// TORCHKAFKA_DEFERRED_FREE=0 releases inline (the old behaviour; the GPU test compares both).
// At process exit the pending releases run (bounded wait) before the HIP runtime tears down.
#pragma once
#include <cstdint>
#include <functional>

namespace tkh {

class Reaper {
 public:
  static bool enabled();
  // Runs `fn` (HIP release calls for `device`) on the reaper thread -- inline when disabled, or
  // in a forked child (which never owns the parent's HIP state: it runs nothing).
  static void post(int device, std::function<void()> fn);
  // Waits until everything posted so far ran (tests, shutdown); false on timeout.
  static bool drain(int timeout_ms = 60000);
  static uint64_t posted();
  static uint64_t released();
  // Convenience wrappers
  static void free_device(int device, void* p);
  static void free_host(int device, void* p);
};

}  // namespace tkh
