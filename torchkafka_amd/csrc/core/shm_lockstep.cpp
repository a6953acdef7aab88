// Node-local lockstep transport: see shm_lockstep.h.
#include "shm_lockstep.h"

#include <fcntl.h>
#include <sched.h>
#include <signal.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cerrno>
#include <chrono>
#include <cstring>
#include <random>
#include <stdexcept>
#include <thread>

#if defined(__x86_64__)
#include <immintrin.h>
#endif

namespace tk {

namespace {

constexpr uint64_t kMagic = 0x746b2d6c6f636b31ULL;  // "tk-lock1"

inline void ls_relax() {
#if defined(__x86_64__)
  _mm_pause();
#endif
}

int64_t mono_ns() {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

[[noreturn]] void shm_errno(const std::string& what) {
  throw std::runtime_error("lockstep shm: " + what + ": " + std::strerror(errno));
}

}  // namespace

// One rank's words of one ticket: a cache line of its own, written by that rank only.
struct alignas(64) LsCell {
  std::atomic<int64_t> seq;  // ticket + 1 once the words are published
  int64_t w[kLockstepWords];
};

// One rank's state: tickets it read the results of (frees their slots), its pid, attached / left.
struct alignas(64) LsRank {
  std::atomic<int64_t> acked;
  std::atomic<int32_t> pid;
  std::atomic<int32_t> state;  // 0 not yet attached, 1 attached, 2 left (transport destroyed)
};

struct alignas(64) LsHeader {
  uint64_t magic;
  int32_t world, slots;
  std::atomic<int32_t> attached;
};

struct ShmLockstep::Layout {
  LsHeader h;
  LsRank* ranks() { return reinterpret_cast<LsRank*>(reinterpret_cast<char*>(this) + sizeof(LsHeader)); }
  LsCell* cell(int slot, int rank) {
    auto* c = reinterpret_cast<LsCell*>(reinterpret_cast<char*>(this) + sizeof(LsHeader) +
                                        sizeof(LsRank) * size_t(h.world));
    return c + size_t(slot) * size_t(h.world) + size_t(rank);
  }
  static size_t bytes(int world, int slots) {
    return sizeof(LsHeader) + sizeof(LsRank) * size_t(world) + sizeof(LsCell) * size_t(world) * size_t(slots);
  }
};

std::string ShmLockstep::create(int world, int slots) {
  if (world < 1 || world > kMaxRanks) throw std::invalid_argument("lockstep shm: 1 <= world <= 256");
  if (slots < 2 || slots > 1024) throw std::invalid_argument("lockstep shm: 2 <= slots <= 1024");
  std::random_device rd;
  const std::string name = "/tk-ls-" + std::to_string(::getpid()) + "-" + std::to_string(rd() & 0xffffff);
  const int fd = shm_open(name.c_str(), O_RDWR | O_CREAT | O_EXCL, 0600);
  if (fd < 0) shm_errno("shm_open " + name);
  const size_t bytes = Layout::bytes(world, slots);
  if (ftruncate(fd, off_t(bytes)) != 0) {
    close(fd);
    shm_unlink(name.c_str());
    shm_errno("ftruncate");
  }
  void* p = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  if (p == MAP_FAILED) {
    shm_unlink(name.c_str());
    shm_errno("mmap");
  }
  auto* L = static_cast<Layout*>(p);  // fresh pages are zero: every seq / acked / state starts at 0
  L->h.world = world;
  L->h.slots = slots;
  L->h.attached.store(0, std::memory_order_relaxed);
  std::atomic_thread_fence(std::memory_order_release);
  reinterpret_cast<std::atomic<uint64_t>*>(&L->h.magic)->store(kMagic, std::memory_order_release);
  munmap(p, bytes);
  return name;
}

ShmLockstep::ShmLockstep(const std::string& name, int rank, int world) : name_(name), rank_(rank), world_(world) {
  if (rank < 0 || rank >= world) throw std::invalid_argument("lockstep shm: rank out of range");
  fd_ = shm_open(name.c_str(), O_RDWR, 0600);
  if (fd_ < 0) shm_errno("shm_open " + name);
  struct stat st;
  if (fstat(fd_, &st) != 0) shm_errno("fstat");
  bytes_ = size_t(st.st_size);
  base_ = mmap(nullptr, bytes_, PROT_READ | PROT_WRITE, MAP_SHARED, fd_, 0);
  if (base_ == MAP_FAILED) {
    base_ = nullptr;
    shm_errno("mmap");
  }
  L_ = static_cast<Layout*>(base_);
  if (reinterpret_cast<std::atomic<uint64_t>*>(&L_->h.magic)->load(std::memory_order_acquire) != kMagic)
    throw std::runtime_error("lockstep shm: " + name + " is not a lockstep segment");
  if (L_->h.world != world)
    throw std::runtime_error("lockstep shm: segment made for " + std::to_string(L_->h.world) + " ranks, not " +
                             std::to_string(world));
  slots_ = L_->h.slots;
  if (bytes_ < Layout::bytes(world, slots_)) throw std::runtime_error("lockstep shm: segment too small");
  LsRank& me = L_->ranks()[rank_];
  int32_t expect = 0;
  if (!me.state.compare_exchange_strong(expect, 1))
    throw std::runtime_error("lockstep shm: rank " + std::to_string(rank_) + " attached twice");
  me.pid.store(int32_t(::getpid()), std::memory_order_relaxed);
  me.acked.store(0, std::memory_order_release);
  L_->h.attached.fetch_add(1, std::memory_order_acq_rel);
  for (auto& s : slot_ticket_) s = -1;
}

ShmLockstep::~ShmLockstep() {
  if (L_) L_->ranks()[rank_].state.store(2, std::memory_order_release);  // peers waiting on us fail fast
  if (base_) munmap(base_, bytes_);
  if (fd_ >= 0) close(fd_);
}

void ShmLockstep::unlink() { shm_unlink(name_.c_str()); }

int ShmLockstep::attached() const { return L_->h.attached.load(std::memory_order_acquire); }

// A wait that found some peer missing for a while: is that peer still part of the job?  Only the
// peers the wait still needs are asked (a rank that finished and left has published everything).
void ShmLockstep::check_peers(int64_t ticket, const char* what, bool acks) {
  LsRank* R = L_->ranks();
  for (int r = 0; r < world_; ++r) {
    if (r == rank_) continue;
    const bool missing = acks ? R[r].acked.load(std::memory_order_acquire) <= ticket
                              : L_->cell(int(ticket % slots_), r)->seq.load(std::memory_order_acquire) != ticket + 1;
    if (!missing) continue;
    const int32_t state = R[r].state.load(std::memory_order_acquire);
    const int32_t pid = R[r].pid.load(std::memory_order_relaxed);
    if (state == 2)
      throw LockstepError(std::string("lockstep: rank ") + std::to_string(r) + " left the lockstep (" + what +
                          ", agreement " + std::to_string(ticket) + "): every rank stops");
    if (state == 1 && pid > 0 && ::kill(pid, 0) != 0 && errno == ESRCH)
      throw LockstepError(std::string("lockstep: rank ") + std::to_string(r) + " (pid " + std::to_string(pid) +
                          ") died (" + what + ", agreement " + std::to_string(ticket) + "): every rank stops");
  }
}

// Spins until every rank acknowledged tickets below `ticket_done` + 1 (their slots are free).
void ShmLockstep::wait_acks(int64_t ticket_done) {
  LsRank* R = L_->ranks();
  const int64_t t0 = mono_ns();
  int64_t next_check = 0;
  for (uint64_t spins = 0;; ++spins) {
    bool all = true;
    for (int r = 0; r < world_ && all; ++r) all = R[r].acked.load(std::memory_order_acquire) > ticket_done;
    if (all) break;
    if ((spins & 255) == 255) {
      const int64_t el = mono_ns() - t0;
      if (el > next_check) {
        check_peers(ticket_done, "slot reuse", true);
        next_check = el + 1000000;
      }
      if (timeout_ms_ > 0 && el > timeout_ms_ * 1000000)
        throw LockstepError("lockstep: no answer from the other ranks within " + std::to_string(timeout_ms_) +
                            " ms (a peer rank hung)");
      if (el > 1000000) std::this_thread::sleep_for(std::chrono::microseconds(20));
      else if (el > 20000) sched_yield();
    }
    ls_relax();
  }
  spin_ns_ += mono_ns() - t0;
}

int ShmLockstep::issue(const int64_t in[kLockstepWords]) {
  const int64_t t = int64_t(issued_);
  const int s = int(t % slots_);
  if (t >= slots_) wait_acks(t - slots_);
  LsCell* c = L_->cell(s, rank_);
  for (int k = 0; k < kLockstepWords; ++k) c->w[k] = in[k];
  c->seq.store(t + 1, std::memory_order_release);
  slot_ticket_[s] = t;
  ++issued_;
  return s;
}

bool ShmLockstep::ready(int slot) {
  const int64_t want = slot_ticket_[slot] + 1;
  for (int r = 0; r < world_; ++r)
    if (L_->cell(slot, r)->seq.load(std::memory_order_acquire) != want) return false;
  return true;
}

void ShmLockstep::reduce(int slot, int64_t ticket, int64_t out[kLockstepWords], bool sum_first) {
  const int64_t want = ticket + 1;
  const int64_t t0 = mono_ns();
  int64_t next_check = 0;
  int from = 0;  // ranks below `from` have published this ticket
  for (uint64_t spins = 0; from < world_; ++spins) {
    while (from < world_ && L_->cell(slot, from)->seq.load(std::memory_order_acquire) == want) ++from;
    if (from == world_) break;
    if ((spins & 255) == 255) {
      const int64_t el = mono_ns() - t0;
      if (el > next_check) {
        check_peers(ticket, "agreement", false);
        next_check = el + 1000000;
      }
      if (timeout_ms_ > 0 && el > timeout_ms_ * 1000000)
        throw LockstepError("lockstep: no answer from the other ranks within " + std::to_string(timeout_ms_) +
                            " ms (a peer rank died or hung)");
      if (el > 1000000) std::this_thread::sleep_for(std::chrono::microseconds(20));
      else if (el > 20000) sched_yield();
    }
    ls_relax();
  }
  spin_ns_ += mono_ns() - t0;
  for (int k = 0; k < kLockstepWords; ++k) out[k] = L_->cell(slot, 0)->w[k];
  for (int r = 1; r < world_; ++r) {
    const LsCell* c = L_->cell(slot, r);
    for (int k = 0; k < kLockstepWords; ++k) {
      if (k == 0 && sum_first)
        out[0] += c->w[0];
      else if (c->w[k] < out[k])
        out[k] = c->w[k];
    }
  }
  // read: the slot may be reused by every rank once all of them acknowledged this ticket
  L_->ranks()[rank_].acked.store(ticket + 1, std::memory_order_release);
  acked_ = ticket + 1;
}

void ShmLockstep::wait(int slot, int64_t out[kLockstepWords]) {
  if (slot < 0 || slot >= slots_ || slot_ticket_[slot] < 0) throw std::invalid_argument("lockstep shm: bad ticket");
  reduce(slot, slot_ticket_[slot], out, false);
}

int64_t ShmLockstep::allreduce_sum(int64_t v) {
  const int64_t in[kLockstepWords] = {v, 0, 0, 0};
  const int s = issue(in);  // every rank of the start-up check calls allreduce_sum: word 0 is summed
  int64_t out[kLockstepWords];
  reduce(s, slot_ticket_[s], out, true);
  return out[0];
}

}  // namespace tk
