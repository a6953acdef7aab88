// Native RCCL lockstep collective for multi-GPU streaming.
//
// One tiny all-reduce(MIN) of int64 [have_batch, step, -step] per loader step
// decides, for every rank at once, whether all ranks have a batch for that
// step (so they continue or stop together) and proves they are on the same
// step.  Issued from C++ on a private HIP stream -- never behind the user's
// queued compute -- and pipelined `depth` steps ahead, so the host never
// waits on the ~10-30 us xGMI round trip: the result for step k was issued
// at step k - depth and is normally complete when it is read.
//
// RCCL is resolved with dlopen() against the librccl that torch already
// loaded (same library instance as torch.distributed's "nccl" backend); the
// communicator is our own, bootstrapped from a unique id the caller
// broadcasts through torch.distributed.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>
#include <vector>

#include "lockstep.h"

namespace tkh {

struct RcclApi;

// The transport interface lives in the HIP-free core (csrc/core/lockstep.h), next to the credit
// protocol that drives it.
using LockstepTransport = tk::LockstepTransport;

class RcclLockstep : public LockstepTransport {
 public:
  // Generates a unique id (rank 0) -- 128 opaque bytes.
  static std::string unique_id(const std::string& lib_path);
  RcclLockstep(const std::string& lib_path, const std::string& id, int rank, int world, int device, int slots);
  ~RcclLockstep();
  RcclLockstep(const RcclLockstep&) = delete;
  RcclLockstep& operator=(const RcclLockstep&) = delete;

  // Enqueues all-reduce(MIN) of {a, b, c}; returns a ticket.
  int issue(int64_t a, int64_t b, int64_t c) override;
  // Waits for a ticket's result.
  void wait(int ticket, int64_t out[3]) override;
  bool ready(int ticket);
  // Failure detection: a round trip not complete after `ms` (a peer rank died or hung) aborts
  // the communicator and raises instead of blocking forever; <= 0 waits indefinitely.
  void set_timeout_ms(int64_t ms) { timeout_ms_ = ms; }
  int64_t timeout_ms() const { return timeout_ms_; }
  bool aborted() const { return aborted_; }
  int world() const { return world_; }
  int rank() const { return rank_; }
  uint64_t issued() const { return issued_; }
  // What RCCL itself reports for the communicator: its size (ncclCommCount) -- the proof that
  // the lockstep spans `world` ranks -- and a blocking all-reduce(SUM) for start-up checks
  // (sum of rank ids == world * (world - 1) / 2).
  int comm_count() const;
  int64_t allreduce_sum(int64_t v);

 private:
  RcclApi* api_ = nullptr;
  void* comm_ = nullptr;
  int rank_, world_, device_, slots_;
  hipStream_t stream_ = nullptr;
  int64_t* d_ = nullptr;       // device [slots][2][3]: in, out
  int64_t* h_in_ = nullptr;    // pinned [slots][3]
  int64_t* h_out_ = nullptr;   // pinned [slots][3]
  std::vector<hipEvent_t> ev_;
  uint64_t issued_ = 0;
  int64_t timeout_ms_ = 600000;  // like torch.distributed's default NCCL timeout
  bool aborted_ = false;
  void wait_event(int t, const char* what);  // bounded wait with async-error checks
};

}  // namespace tkh
