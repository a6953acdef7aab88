// Node-local lockstep transport: the all-reduce(MIN) of an agreement's words through a shared-memory
// segment the ranks of one host map.
//
// Why not RCCL for this: an agreement is 4 int64 words of HOST state (credit, step, commit status)
// that the host must read back before it may hand out the next batch.  Over RCCL that is a round
// trip host -> device -> collective -> device -> host per agreement: on MI355X three dependent
// dispatches spanning 19 us at the median on the device (profiles/r06_s1: words-in kernel, RCCL's
// copy, words-out kernel, 5.8 us gaps between them) plus the issue and the completion poll -- a
// per-step barrier (commit='sync') could not run faster than ~9 M rec/s (BENCH_r05 steady_rccl_sync).
// The ranks of one node share host memory: each writes its words into its own cache line of the
// agreement's slot and reads the others' lines -- well under a microsecond when the ranks arrive
// together.  RCCL keeps carrying what is device data (the model's gradients); jobs that span hosts
// use the RCCL transport (rccl_lockstep.h) for the lockstep.
//
// Protocol.  Ticket t uses slot t % slots.  issue(): wait until every rank has acknowledged ticket
// t - slots (read its result, so the slot is free), write the words, then publish seq = t + 1 with
// release.  wait(): spin until every rank's seq in that slot is t + 1 (acquire), take the MIN, then
// acknowledge t.  Every rank issues and waits the same tickets in the same order (lockstep.h), so
// a rank is at most `slots` tickets ahead of the slowest.  Failure detection while waiting: a peer
// that left the lockstep (its transport destroyed before the agreement) or whose process is gone
// (kill(pid, 0) == ESRCH) fails the wait at once; otherwise the timeout does.
#pragma once
#include <atomic>
#include <cstdint>
#include <string>

#include "lockstep.h"

namespace tk {

class ShmLockstep : public LockstepTransport {
 public:
  static constexpr int kMaxRanks = 256;
  // Rank 0: creates a segment for `world` ranks and `slots` tickets in flight; returns its name.
  static std::string create(int world, int slots);
  // Every rank (rank 0 included): maps the segment and registers as `rank`.
  ShmLockstep(const std::string& name, int rank, int world);
  ~ShmLockstep() override;
  ShmLockstep(const ShmLockstep&) = delete;
  ShmLockstep& operator=(const ShmLockstep&) = delete;

  int issue(const int64_t in[kLockstepWords]) override;
  void wait(int ticket, int64_t out[kLockstepWords]) override;
  bool ready(int ticket) override;  // (ticket = the slot issue() returned)

  // Removes the segment's name (after every rank attached): the mapping lives on, nothing is left
  // in /dev/shm when a rank crashes.
  void unlink();
  int attached() const;  // ranks that mapped the segment so far
  void set_timeout_ms(int64_t ms) { timeout_ms_ = ms; }
  int64_t timeout_ms() const { return timeout_ms_; }
  // The whole exchange once (issue + wait) with one word summed instead of MIN'd: a start-up check
  // that every rank of the process group reached the same segment.
  int64_t allreduce_sum(int64_t v);
  int rank() const { return rank_; }
  int world() const { return world_; }
  int slots() const { return slots_; }
  uint64_t issued() const { return issued_; }
  int64_t spin_ns() const { return spin_ns_; }  // time spent waiting for peers

 private:
  struct Layout;
  void check_peers(int64_t ticket, const char* what, bool acks);
  void wait_acks(int64_t ticket_done);
  void reduce(int slot, int64_t ticket, int64_t out[kLockstepWords], bool sum_first);

  std::string name_;
  int rank_, world_, slots_ = 0;
  int fd_ = -1;
  void* base_ = nullptr;
  size_t bytes_ = 0;
  Layout* L_ = nullptr;
  uint64_t issued_ = 0;
  int64_t acked_ = 0;  // tickets this rank has read the results of
  int64_t timeout_ms_ = 300000;
  int64_t spin_ns_ = 0;
  int64_t slot_ticket_[1024];
};

}  // namespace tk
