// Native RCCL lockstep collective for multi-GPU streaming.
//
// One tiny all-reduce(MIN) of int64 [credit, step, -step, commit status] per
// agreement decides, for every rank at once, how far all ranks may go (so they
// continue or stop together), proves they are on the same step and, under
// commit='sync', tells every rank whether every rank's commit went through.
//
// The words never take a hipMemcpyAsync (two 32-byte copies per
// agreement, three queue operations): by default a one-wave kernel reads them
// from pinned host memory into the device buffer RCCL reduces, and another
// writes the result back to pinned host memory (TORCHKAFKA_RCCL_WORDS=kernel);
// `host` hands RCCL the host-mapped buffers themselves (one queue operation);
// `copy` keeps the two hipMemcpyAsync (A/B only).  Issued from C++ on a private HIP stream -- never behind the user's
// queued compute -- and pipelined `depth` steps ahead, so the host never
// waits on the ~10-30 us xGMI round trip: the result for step k was issued
// at step k - depth and is normally complete when it is read.
//
// RCCL is resolved with dlopen() against the librccl that torch already
// loaded (same library instance as torch.distributed's "nccl" backend); the
// communicator is our own, bootstrapped from a unique id the caller
// broadcasts through torch.distributed.
#pragma once
#include <hip/hip_runtime_api.h>

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

  // Enqueues all-reduce(MIN) of the agreement's words; returns a ticket.
  int issue(const int64_t in[tk::kLockstepWords]) override;
  // Waits for a ticket's result.
  void wait(int ticket, int64_t out[tk::kLockstepWords]) override;
  const char* words_mode() const {
    return mode_ == 0 ? (graph_fallback_ ? "kernel (graph capture failed)" : "kernel")
                      : mode_ == 1 ? "host" : mode_ == 2 ? "copy" : "graph";
  }
  bool high_priority() const { return high_prio_; }
  bool ready(int ticket) override;
  // a poll is a hipEventQuery of the agreement's event: every poll_every_ steps
  // (TORCHKAFKA_RCCL_POLL_EVERY, default 8; 0: never -- agreements are read where their grant
  // is needed, as before round 6)
  int ready_poll_every() const override { return poll_every_ > 0 ? poll_every_ : (1 << 30); }
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
  // TORCHKAFKA_LOCKSTEP_TRACE=1: host timestamps (steady clock, ns) of every agreement -- issue
  // begin / end, wait begin / end (tools/probes: where an agreement's round trip goes).
  struct TraceRec {
    int64_t issue0, issue1, wait0, wait1;
  };
  std::vector<TraceRec> take_trace() {
    std::vector<TraceRec> t;
    t.swap(trace_);
    return t;
  }

 private:
  RcclApi* api_ = nullptr;
  void* comm_ = nullptr;
  int rank_, world_, device_, slots_;
  hipStream_t stream_ = nullptr;
  int64_t* d_ = nullptr;       // device [slots][2][kLockstepWords]: in, out
  int64_t* h_in_ = nullptr;    // pinned, device-mapped [slots][kLockstepWords]
  int64_t* h_out_ = nullptr;   // pinned, device-mapped [slots][kLockstepWords]
  int64_t* h_in_dev_ = nullptr;   // their device addresses
  int64_t* h_out_dev_ = nullptr;
  int mode_ = 0;               // 0 kernel, 1 host, 2 copy, 3 graph (TORCHKAFKA_RCCL_WORDS)
  int poll_every_ = 8;
  bool graph_fallback_ = false;
  std::vector<void*> graphs_;  // mode 3: a hipGraphExec_t per slot (rccl_issue.hip)
  void capture_graphs();
  void release_graphs();
  bool high_prio_ = false;     // stream_ at the greatest priority (its own hardware-queue pool)
  std::vector<hipEvent_t> ev_;
  uint64_t issued_ = 0;
  int64_t timeout_ms_ = 600000;  // like torch.distributed's default NCCL timeout
  bool aborted_ = false;
  bool tracing_ = false;
  std::vector<TraceRec> trace_;
  std::vector<int64_t> slot_rec_;  // per slot: its agreement's record in trace_ (-1: none)
  void wait_event(int t, const char* what);  // bounded wait with async-error checks
};

}  // namespace tkh
