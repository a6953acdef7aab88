// Cross-rank lockstep of the loader as a credit protocol -- HIP-free, so the
// exact protocol the device driver runs is also driven by CPU tests over gloo at world 2..8.
//
// The reference has no notion of ranks: under torchrun every rank's consumers would run at their
// own pace, so one rank running dry leaves the others hanging in the next gradient all-reduce,
// and offsets committed by a fast rank describe steps the job never finished.
//
// Ranks deliver batch indices in the same order; `granted` is the index below which every rank
// is known to hold a batch.  An agreement carries each rank's CREDIT -- how many batches it holds
// beyond `granted` (what is staged now: never a wait on data a worker cannot publish while its
// ring slots are all staged here), or -1 once its stream ended and it holds none -- as an
// all-reduce(MIN); the minimum extends `granted` for every rank, -1 means no credit will ever
// come again, so all ranks stop at the same index.  A new agreement is issued while `depth`
// credits remain, so its round trip overlaps the delivery of those batches.  Every decision
// depends only on (step, granted) and agreement results, identical on all ranks, so the
// collective sequences stay aligned.  Completion of an agreement issued at step s proves every
// rank reached s: batches < s are finished everywhere and become committable.  Two more words
// ride along as a consistency check: step and -step (MIN of both = min and -max).
//
// Sync mode (commit='sync', the reference's per-batch commit contract, auto_commit.py:55-58 /
// kafka_dataset.py:130, made a cross-rank barrier): a finished batch is committable at once on
// its own rank; the caller commits it (its store, the coordinator's answer through a bridge) and
// reports how that went (set_commit_status); then, before batch k+1 may be handed out, an
// agreement issued at step k+1 must complete.  So when any rank hands out k+1, EVERY rank has
// committed k.  The agreement's fourth word is the MIN of the ranks' commit statuses: a rank whose
// commit failed fatally makes every rank raise at the same step (kCommitFatal), a swallowed
// CommitFailedError (the reference logs it and continues, kafka_dataset.py:131-135) lets every rank
// continue (kCommitFailed is counted).  One collective per step: the issue-ahead pipelining is
// off, the agreement's credit still grants the following batches.
#pragma once
#include <chrono>
#include <cstdint>
#include <deque>
#include <functional>
#include <stdexcept>
#include <utility>
#include <vector>

#include "ring.h"

namespace tk {

// The words of one agreement, all-reduced with MIN: [credit, step, -step, commit status].
constexpr int kLockstepWords = 4;
// Commit status word (sync mode): every batch committed so far was stored / a CommitFailedError
// was swallowed on some rank / a commit raised on some rank.
constexpr int64_t kCommitOk = 2, kCommitFailed = 1, kCommitFatal = 0;

// A pipelined all-reduce(MIN) of kLockstepWords int64: issue() returns a ticket, wait() its result.
// Implemented over RCCL (csrc/hip/rccl_lockstep.*) and over any Python all-reduce (gloo).
class LockstepTransport {
 public:
  virtual ~LockstepTransport() = default;
  virtual int issue(const int64_t in[kLockstepWords]) = 0;
  virtual void wait(int ticket, int64_t out[kLockstepWords]) = 0;
  // wait(ticket) would return at once (a transport that computes the result in issue(): always)
  virtual bool ready(int ticket) { return true; }
  // Steps between two ready() polls of an agreement in flight: a poll that costs a runtime call
  // (hipEventQuery, ~1-2 us) is not made every step.
  virtual int ready_poll_every() const { return 1; }
};

class LockstepError : public std::runtime_error {
 public:
  using std::runtime_error::runtime_error;
};

// What the protocol needs from the rank's data path.
class LockstepSource {
 public:
  virtual ~LockstepSource() = default;
  virtual int64_t staged() = 0;   // data batches held now and not yet delivered
  virtual bool all_done() = 0;    // every producer of this rank has ended its stream
  // Blocks up to timeout_ms for more data: 1 got some, 0/-1 nothing, -3 producer error.
  virtual int wait_data(int64_t timeout_ms) = 0;
};

class CreditLockstep {
 public:
  CreditLockstep(LockstepTransport* t, int depth) : t_(t), depth_(depth < 0 ? 0 : depth) {
    if (!t_) throw std::invalid_argument("lockstep: no transport");
  }
  // May the next batch be delivered?  1: yes (the caller delivers its oldest staged batch, then
  // calls delivered()), -1: starved for now (let the caller check worker health, call again),
  // -2: every rank stops here, -3: the source reported a producer error.
  int next(LockstepSource& src, int64_t timeout_ms);
  // The batch next() allowed was handed out; returns its index.
  int64_t delivered() { return step_++; }
  // A delivered batch is finished (the user asked for the next one): it becomes committable
  // once an agreement proves every rank got past it (settle) -- in sync mode at once (the
  // agreement after its commit is the barrier).
  void finished(int64_t index, std::vector<Watermark>&& wms) {
    if (sync_)
      emit(std::move(wms));
    else
      finished_q_.emplace_back(index, std::move(wms));
  }
  // Sync mode: how this rank's commits since the last agreement went (kCommitOk / kCommitFailed /
  // kCommitFatal); carried by the next agreement, then reset to kCommitOk.
  void set_commit_status(int64_t s) { commit_status_ = s < commit_status_ ? s : commit_status_; }
  // The MIN commit status of the last settled agreement, and agreements that carried a failure.
  int64_t group_commit_status() const { return group_status_; }
  uint64_t group_commit_failures() const { return group_failures_; }
  // End of the iteration: settle every agreement in flight, then one more round (a barrier:
  // every rank stopped at the same step); everything finished becomes committable.
  void finish();
  // Committable batches are handed to this callback (settle / finish order = delivery order).
  void set_on_committable(std::function<void(std::vector<Watermark>&&)> f) { on_commit_ = std::move(f); }
  // Sync mode (see above).  Every rank must use the same mode: it decides which collectives run.
  void set_sync(bool s) { sync_ = s; }
  // Async mode: an agreement is issued every `n` steps and grants at most up to step + 2n (0: one
  // agreement at a time, granting whatever every rank holds), so finished batches become
  // committable about every n steps.  Every rank must use the same value.
  void set_commit_every(int n) { commit_every_ = n < 0 ? 0 : n; }
  int commit_every() const { return commit_every_; }
  bool sync() const { return sync_; }

  int64_t step() const { return step_; }
  int64_t granted() const { return granted_; }
  bool stopped() const { return stopped_; }
  uint64_t agreements() const { return agreements_; }
  int depth() const { return depth_; }
  // Host time spent waiting for agreement results: in total, and the most one delivered step
  // (one next() call) waited -- what the collective's round trip cost the critical path.
  int64_t wait_ns() const { return wait_ns_; }
  int64_t issue_ns() const { return issue_ns_; }  // host time spent issuing agreements
  int64_t step_wait_max_ns() const { return step_wait_max_ns_; }
  uint64_t agreements_since_reset() const { return agreements_ - agreements_at_reset_; }
  void reset_stats() {
    wait_ns_ = step_wait_max_ns_ = issue_ns_ = 0;
    agreements_at_reset_ = agreements_;
  }

 private:
  struct Ticket {
    int64_t step;  // step at which it was issued
    int64_t base;  // granted at issue time
    int ticket;
    bool observed = false;  // its result was read (committable batches emitted), grant not applied
    int64_t res[kLockstepWords] = {0, 0, 0, 0};
  };
  int next_impl(LockstepSource& src, int64_t timeout_ms);
  int64_t credit(LockstepSource& src) const;
  void issue(LockstepSource& src);
  void settle();
  // Reads the front ticket's result (blocking unless the transport says it is ready) and emits the
  // batches it made committable.  The grant is applied by settle() only, at a step every rank
  // reaches with the same state -- observing early is local and never changes what is issued.
  void observe(Ticket& t);
  void emit(std::vector<Watermark>&& wms) {
    if (on_commit_) on_commit_(std::move(wms));
  }

  LockstepTransport* t_;
  int depth_;
  int64_t step_ = 0, granted_ = 0;
  bool stopped_ = false, no_more_credit_ = false, sync_ = false;
  int commit_every_ = 0;
  int64_t last_issue_step_ = -1;
  int64_t last_poll_step_ = -1;
  static constexpr int kMaxInflight = 3;  // agreements in flight under commit_every (transport slots >= 4)
  int64_t settled_step_ = -1;  // highest step an agreement was issued at and has completed
  int64_t commit_status_ = kCommitOk, group_status_ = kCommitOk;
  uint64_t group_failures_ = 0;
  uint64_t agreements_ = 0, agreements_at_reset_ = 0;
  int64_t wait_ns_ = 0, step_wait_max_ns_ = 0, step_wait_ns_ = 0, issue_ns_ = 0;
  std::deque<Ticket> tickets_;
  std::deque<std::pair<int64_t, std::vector<Watermark>>> finished_q_;
  std::function<void(std::vector<Watermark>&&)> on_commit_;
};

}  // namespace tk
