#include "lockstep.h"

#include <algorithm>
#include <string>

namespace tk {

int64_t CreditLockstep::credit(LockstepSource& src) const {
  const int64_t beyond = src.staged() - (granted_ - step_);
  if (beyond > 0) return beyond;
  return src.all_done() ? -1 : 0;
}

void CreditLockstep::issue(LockstepSource& src) {
  int64_t c = credit(src);
  // commit_every: never grant past step + 2 x commit_every (granted_ is this ticket's base): the next
  // agreement, issued commit_every steps on, has another commit_every steps to come back
  if (commit_every_ > 0 && !sync_ && c > step_ + 2 * commit_every_ - granted_)
    c = std::max<int64_t>(0, step_ + 2 * commit_every_ - granted_);
  last_issue_step_ = step_;
  const int64_t w[kLockstepWords] = {c, step_, -step_, commit_status_};
  commit_status_ = kCommitOk;
  const auto t0 = std::chrono::steady_clock::now();
  tickets_.push_back(Ticket{step_, granted_, t_->issue(w)});
  issue_ns_ += std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count();
  ++agreements_;
}

void CreditLockstep::observe(Ticket& t) {
  if (t.observed) return;
  const auto w0 = std::chrono::steady_clock::now();
  t_->wait(t.ticket, t.res);
  const int64_t waited =
      std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - w0).count();
  wait_ns_ += waited;
  step_wait_ns_ += waited;
  t.observed = true;
  const int64_t* res = t.res;
  if (res[1] != -res[2])
    throw LockstepError("lockstep: ranks are out of step (min " + std::to_string(res[1]) + ", max " +
                        std::to_string(-res[2]) + ")");
  group_status_ = res[3];
  if (res[3] == kCommitFailed) ++group_failures_;
  if (res[3] <= kCommitFatal)
    throw LockstepError("lockstep: a rank's commit before step " + std::to_string(t.step) +
                        " failed; every rank stops at this step");
  // completion proves every rank reached t.step: the batches before it are finished everywhere
  while (!finished_q_.empty() && finished_q_.front().first < t.step) {
    emit(std::move(finished_q_.front().second));
    finished_q_.pop_front();
  }
}

void CreditLockstep::settle() {
  observe(tickets_.front());
  const Ticket t = tickets_.front();
  tickets_.pop_front();
  const int64_t* res = t.res;
  if (t.step > settled_step_) settled_step_ = t.step;
  if (res[0] < 0)
    no_more_credit_ = true;
  else if (t.base + res[0] > granted_)
    granted_ = t.base + res[0];
}

int CreditLockstep::next(LockstepSource& src, int64_t timeout_ms) {
  if (stopped_) return -2;
  step_wait_ns_ = 0;
  const int r = next_impl(src, timeout_ms);
  if (step_wait_ns_ > step_wait_max_ns_) step_wait_max_ns_ = step_wait_ns_;
  return r;
}

int CreditLockstep::next_impl(LockstepSource& src, int64_t timeout_ms) {
  if (sync_) {
    // every rank is at this step with the same tickets in flight (none, in sync mode): one
    // agreement at step_ proves batches < step_ finished everywhere and settles them now
    while (!tickets_.empty()) settle();
    if (settled_step_ < step_) {
      issue(src);
      settle();
    }
  } else {
    // agreements already back: their batches become committable now, in issue order (local: the
    // grants are applied where every rank applies them, below)
    if (!tickets_.empty() && step_ - last_poll_step_ >= t_->ready_poll_every()) {
      last_poll_step_ = step_;
      for (auto& t : tickets_) {
        if (t.observed) continue;
        if (!t_->ready(t.ticket)) break;
        observe(t);
      }
    }
    const bool low = tickets_.empty() && granted_ - step_ <= depth_;
    // commit_every: a fresh agreement every commit_every steps, a few in flight, so batches become
    // committable at that cadence without the host ever waiting for one round trip.  Every input
    // to this decision (step, applied grant, tickets issued) is the same on every rank.
    const bool cadence = commit_every_ > 0 && int(tickets_.size()) < kMaxInflight &&
                         step_ - last_issue_step_ >= commit_every_;
    if (!no_more_credit_ && step_ < granted_ && (low || cadence)) {
      // issue ahead while credits remain, so the round trip overlaps the delivery of granted batches
      issue(src);
    }
  }
  while (step_ >= granted_) {
    if (no_more_credit_) {
      stopped_ = true;
      return -2;
    }
    bool starved = false;
    if (tickets_.empty()) {
      if (src.staged() == 0 && !src.all_done()) {
        // nothing to offer yet: give the producers a moment before spending a collective round
        const int r = src.wait_data(timeout_ms);
        if (r == -3) return -3;
        starved = r <= 0;
      }
      issue(src);  // credit 0 when still starved: the other ranks wait with us, nobody hangs
    }
    settle();
    if (starved && step_ >= granted_) return -1;
  }
  return 1;
}

void CreditLockstep::finish() {
  while (!tickets_.empty()) settle();  // every rank issued the same agreements
  const int64_t w[kLockstepWords] = {0, 0, 0, commit_status_};
  commit_status_ = kCommitOk;
  int64_t res[kLockstepWords];
  t_->wait(t_->issue(w), res);   // every rank has stopped at the same step
  ++agreements_;
  group_status_ = res[3];
  if (res[3] <= kCommitFatal) {
    stopped_ = true;
    throw LockstepError("lockstep: a rank's last commit failed");
  }
  for (auto& f : finished_q_) emit(std::move(f.second));
  finished_q_.clear();
  stopped_ = true;
}

}  // namespace tk
