#include "ring.h"

#include <fcntl.h>
#include <linux/futex.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <climits>

namespace tk {

void futex_wait(std::atomic<uint32_t>* addr, uint32_t expected, int64_t timeout_ns) {
  timespec ts{time_t(timeout_ns / 1000000000LL), long(timeout_ns % 1000000000LL)};
  syscall(SYS_futex, reinterpret_cast<uint32_t*>(addr), FUTEX_WAIT, expected, timeout_ns >= 0 ? &ts : nullptr,
          nullptr, 0);
}

void futex_wake_all(std::atomic<uint32_t>* addr) {
  syscall(SYS_futex, reinterpret_cast<uint32_t*>(addr), FUTEX_WAKE, INT_MAX, nullptr, nullptr, 0);
}

void bump_and_wake(std::atomic<uint32_t>* seq, std::atomic<uint32_t>* waiters) {
  seq->fetch_add(1, std::memory_order_seq_cst);
  if (waiters->load(std::memory_order_seq_cst) != 0) futex_wake_all(seq);
}

void wait_seq(std::atomic<uint32_t>* seq, std::atomic<uint32_t>* waiters, uint32_t seen, int64_t timeout_ns) {
  waiters->fetch_add(1, std::memory_order_seq_cst);
  if (seq->load(std::memory_order_seq_cst) == seen) futex_wait(seq, seen, timeout_ns);
  waiters->fetch_sub(1, std::memory_order_seq_cst);
}

std::unique_ptr<Ring> Ring::create(const std::string& name, uint32_t n_workers, uint32_t slots_per_worker,
                                   uint64_t payload_capacity) {
  if (n_workers == 0 || n_workers > kMaxWorkers) throw std::invalid_argument("ring: bad worker count");
  if (slots_per_worker == 0) throw std::invalid_argument("ring: need at least one slot per worker");
  payload_capacity = align_up(payload_capacity ? payload_capacity : 4096, 4096);
  const uint64_t stride = kSlotHeaderBytes + payload_capacity;
  const uint64_t hdr_bytes = align_up(sizeof(RingHeader), 65536);
  const uint64_t total = hdr_bytes + stride * n_workers * slots_per_worker;
  std::unique_ptr<Ring> r(new Ring());
  r->name_ = name;
  r->fd_ = shm_open(name.c_str(), O_RDWR | O_CREAT | O_EXCL, 0600);
  if (r->fd_ < 0) throw_errno("shm_open " + name);
  r->owner_ = true;
  if (ftruncate(r->fd_, off_t(total)) != 0) throw_errno("ftruncate ring");
  void* p = mmap(nullptr, total, PROT_READ | PROT_WRITE, MAP_SHARED, r->fd_, 0);
  if (p == MAP_FAILED) throw_errno("mmap ring");
  r->base_ = static_cast<uint8_t*>(p);
  r->len_ = total;
  r->hdr_ = reinterpret_cast<RingHeader*>(p);
  RingHeader* h = r->hdr_;
  h->n_workers = n_workers;
  h->slots_per_worker = slots_per_worker;
  h->slot_stride = stride;
  h->payload_capacity = payload_capacity;
  h->total_bytes = total;
  h->shutdown.store(0);
  h->ready_seq.store(0);
  h->ready_waiters.store(0);
  for (int w = 0; w < kMaxWorkers; ++w) {
    h->free_seq[w].store(0);
    h->free_waiters[w].store(0);
    h->worker_pid[w].store(0);
  }
  for (uint32_t s = 0; s < n_workers * slots_per_worker; ++s) {
    SlotHeader* sh = r->slot(s);
    sh->state.store(kSlotFree);
    sh->worker = s / slots_per_worker;
    sh->seq = 0;
  }
  std::atomic_thread_fence(std::memory_order_release);
  h->magic = kRingMagic;
  return r;
}

std::unique_ptr<Ring> Ring::open(const std::string& name) {
  std::unique_ptr<Ring> r(new Ring());
  r->name_ = name;
  r->fd_ = shm_open(name.c_str(), O_RDWR, 0600);
  if (r->fd_ < 0) throw_errno("shm_open " + name);
  struct stat st;
  if (fstat(r->fd_, &st) != 0) throw_errno("fstat ring");
  void* p = mmap(nullptr, size_t(st.st_size), PROT_READ | PROT_WRITE, MAP_SHARED, r->fd_, 0);
  if (p == MAP_FAILED) throw_errno("mmap ring");
  r->base_ = static_cast<uint8_t*>(p);
  r->len_ = size_t(st.st_size);
  r->hdr_ = reinterpret_cast<RingHeader*>(p);
  if (r->hdr_->magic != kRingMagic) throw std::runtime_error("ring '" + name + "' is not initialised");
  return r;
}

Ring::~Ring() {
  if (base_) munmap(base_, len_);
  if (fd_ >= 0) close(fd_);
}

void Ring::unlink() { shm_unlink(name_.c_str()); }

SlotHeader* Ring::slot(uint32_t g) const {
  if (g >= n_slots()) throw std::out_of_range("ring: bad slot");
  const uint64_t hdr_bytes = align_up(sizeof(RingHeader), 65536);
  return reinterpret_cast<SlotHeader*>(base_ + hdr_bytes + uint64_t(g) * hdr_->slot_stride);
}

// A worker whose sub-ring is full spins for up to spin_ns_ (200 µs) before sleeping on the futex.
// With workers ahead of the consumer (the common case), a slot comes back every few µs; if
// the worker slept instead, every main_release would pay a futex_wake syscall (~1-2 µs) on the
// main thread's per-batch path, plus the worker's wake-up latency.  Workers run on their own
// cores (one per worker), so the spin costs no one else's time.
bool Ring::worker_acquire(uint32_t worker, uint32_t i, int64_t timeout_ms) {
  SlotHeader* s = slot(gslot(worker, i));
  const int64_t start = now_ns();
  const int64_t deadline = timeout_ms < 0 ? INT64_MAX : start + timeout_ms * 1000000LL;
  const int64_t spin_until = std::min(deadline, start + spin_ns_);
  for (;;) {
    if (hdr_->shutdown.load(std::memory_order_acquire)) return false;
    const uint32_t seq = hdr_->free_seq[worker].load(std::memory_order_acquire);
    uint32_t st = s->state.load(std::memory_order_acquire);
    if (st == kSlotFree) {
      s->state.store(kSlotFilling, std::memory_order_relaxed);
      s->t_acquire_wait_ns = now_ns() - start;
      return true;
    }
    const int64_t now = now_ns();
    if (now >= deadline) return false;
    if (now < spin_until) {
      for (int k = 0; k < 64; ++k) cpu_relax();
      continue;
    }
    wait_seq(&hdr_->free_seq[worker], &hdr_->free_waiters[worker], seq, std::min<int64_t>(deadline - now, 100000000LL));
  }
}

void Ring::worker_publish(uint32_t g) {
  SlotHeader* s = slot(g);
#if defined(__x86_64__)
  __builtin_ia32_sfence();  // order the packer's non-temporal stores before the release below
#endif
  s->t_ready_ns = now_ns();
  s->state.store(kSlotReady, std::memory_order_release);
  bump_and_wake(&hdr_->ready_seq, &hdr_->ready_waiters);
}

int64_t Ring::main_acquire(uint32_t* cursor, uint32_t* rr, const uint8_t* done, bool in_order, int64_t timeout_ms) {
  const uint32_t nw = hdr_->n_workers, spw = hdr_->slots_per_worker;
  const int64_t deadline = timeout_ms < 0 ? INT64_MAX : now_ns() + timeout_ms * 1000000LL;
  int spins = 0;
  for (;;) {
    const uint32_t seq = hdr_->ready_seq.load(std::memory_order_acquire);
    bool any_live = false;
    for (uint32_t k = 0; k < nw; ++k) {
      const uint32_t w = (*rr + k) % nw;
      if (done[w]) continue;
      any_live = true;
      const uint32_t g = w * spw + cursor[w];
      SlotHeader* s = slot(g);
      if (s->state.load(std::memory_order_acquire) == kSlotReady) {
        s->state.store(kSlotInflight, std::memory_order_relaxed);
        cursor[w] = (cursor[w] + 1) % spw;
        *rr = (w + 1) % nw;
        return int64_t(g);
      }
      if (in_order) break;  // strict round robin: wait for this worker
    }
    if (!any_live) return -2;
    const int64_t now = now_ns();
    if (now >= deadline) return -1;
    if (++spins < 2000) {
      cpu_relax();
      continue;
    }
    wait_seq(&hdr_->ready_seq, &hdr_->ready_waiters, seq, std::min<int64_t>(deadline - now, 20000000LL));
  }
}

void Ring::main_release(uint32_t g) {
  SlotHeader* s = slot(g);
  const uint32_t w = s->worker;
  s->state.store(kSlotFree, std::memory_order_release);
  bump_and_wake(&hdr_->free_seq[w], &hdr_->free_waiters[w]);
}

void Ring::shutdown() {
  hdr_->shutdown.store(1, std::memory_order_release);
  for (uint32_t w = 0; w < hdr_->n_workers; ++w) {
    hdr_->free_seq[w].fetch_add(1);
    futex_wake_all(&hdr_->free_seq[w]);
  }
  hdr_->ready_seq.fetch_add(1);
  futex_wake_all(&hdr_->ready_seq);
}

}  // namespace tk
