// Host-sanitizer stress test of the slot ring and the fetch/pack path (no GPU, no Python).
//
// Built twice by tools/sanitize.sh: with -fsanitize=thread (data races in the FREE -> FILLING
// -> READY -> INFLIGHT protocol, the futex hand-offs, the broker's per-partition locks) and with
// -fsanitize=address,undefined (bounds of the packers and the RecordBatch decoder).  Threads
// stand in for the loader's worker processes: the ring and broker code is the same, and TSan
// only sees races between threads of one process.
//
//   ring_stress [n_workers] [slots_per_worker] [batches_per_worker]
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <unistd.h>
#include <vector>

#include "broker.h"
#include "consumer.h"
#include "ring.h"

using namespace tk;

#define CHECK(c)                                                                  \
  do {                                                                            \
    if (!(c)) {                                                                   \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c);   \
      std::abort();                                                               \
    }                                                                             \
  } while (0)

// Part 1: ring protocol with synthetic payloads (each slot carries worker id + sequence).
static void ring_protocol(uint32_t nw, uint32_t spw, uint32_t per_worker) {
  const std::string name = "/tk_ring_stress_" + std::to_string(getpid());
  auto ring = Ring::create(name, nw, spw, 4096);
  std::vector<std::thread> ws;
  for (uint32_t w = 0; w < nw; ++w) {
    ws.emplace_back([&, w] {
      for (uint32_t i = 0; i < per_worker; ++i) {
        const uint32_t slot_i = i % spw;
        CHECK(ring->worker_acquire(w, slot_i, 60000));
        const uint32_t g = ring->gslot(w, slot_i);
        SlotHeader* h = ring->slot(g);
        uint32_t* pay = reinterpret_cast<uint32_t*>(ring->payload(g));
        for (int k = 0; k < 1024; ++k) pay[k] = w * 1000003u + i + uint32_t(k);
        h->n_rows = i;
        h->n_parts = 1;
        h->wm[0].pidx = w;
        h->wm[0].next_offset = int64_t(i) + 1;
        h->flags = (i + 1 == per_worker) ? kSlotEOS : 0;
        ring->worker_publish(g);
      }
    });
  }
  std::vector<uint32_t> cursor(nw, 0), next(nw, 0);
  std::vector<uint8_t> done(nw, 0);
  uint32_t rr = 0;
  uint64_t got = 0;
  for (;;) {
    const int64_t g = ring->main_acquire(cursor.data(), &rr, done.data(), false, 60000);
    if (g == -2) break;
    CHECK(g >= 0);
    SlotHeader* h = ring->slot(uint32_t(g));
    const uint32_t w = h->worker;
    CHECK(h->wm[0].pidx == w);
    CHECK(h->n_rows == next[w]);  // per-worker FIFO order
    const uint32_t* pay = reinterpret_cast<const uint32_t*>(ring->payload(uint32_t(g)));
    for (int k = 0; k < 1024; ++k) CHECK(pay[k] == w * 1000003u + h->n_rows + uint32_t(k));
    ++next[w];
    if (h->flags & kSlotEOS) done[w] = 1;
    ring->main_release(uint32_t(g));
    ++got;
  }
  for (auto& t : ws) t.join();
  CHECK(got == uint64_t(nw) * per_worker);
  ring->shutdown();
  ring->unlink();
  std::printf("ring protocol: %u workers x %u slots, %llu batches ok\n", nw, spw, (unsigned long long)got);
}

// Part 2: broker + fetcher + packer: producer threads append while packer threads fill ring
// slots from the same partitions and a committer commits watermarks.
static void broker_pipeline(uint32_t nw, uint32_t per_part) {
  const std::string url = "shm://tk_broker_stress_" + std::to_string(getpid());
  BrokerConfig cfg;
  cfg.default_log_capacity = 64ull << 20;
  cfg.default_index_capacity = 1 << 16;
  auto b = std::make_shared<Broker>(url, true, cfg);
  const uint32_t np = 2 * nw;
  TopicInfo t = b->create_topic("s", np);
  const std::string rname = "/tk_ring_stress2_" + std::to_string(getpid());
  auto ring = Ring::create(rname, nw, 3, 64 * 256);
  std::atomic<bool> stop{false};
  // producers: one thread per partition pair, 16-float records in batches of 7
  std::vector<std::thread> prod;
  for (uint32_t w = 0; w < nw; ++w) {
    prod.emplace_back([&, w] {
      std::vector<float> v(16);
      std::vector<RecordIn> recs(7);
      for (uint32_t n = 0; n < per_part; n += 7) {
        for (uint32_t pp = 0; pp < 2; ++pp) {
          const uint32_t pidx = t.first_pidx + w * 2 + pp;
          const uint32_t k = std::min<uint32_t>(7, per_part - n);
          for (uint32_t i = 0; i < k; ++i) {
            for (int j = 0; j < 16; ++j) v[j] = float(n + i);
            v[1] = float(pidx);
            recs[i] = RecordIn{0, nullptr, -1, reinterpret_cast<const uint8_t*>(v.data()), 64, nullptr, 0};
            b->append(pidx, recs.data(), 1);
          }
        }
      }
    });
  }
  // packers: worker w owns partitions {2w, 2w+1}
  std::vector<std::thread> packers;
  for (uint32_t w = 0; w < nw; ++w) {
    packers.emplace_back([&, w] {
      Fetcher f(b, true);
      f.assign({t.first_pidx + 2 * w, t.first_pidx + 2 * w + 1}, {0, 0});
      PackSpec spec;
      spec.kind = kPackFixed;
      spec.elem_size = 4;
      spec.row_elems = 16;
      size_t rr = 0;
      uint32_t i = 0;
      uint64_t rows = 0;
      while (rows < 2ull * per_part) {
        CHECK(ring->worker_acquire(w, i % 3, 60000));
        const uint32_t g = ring->gslot(w, i % 3);
        FillOutcome o = fill_slot(f, *ring, g, spec, 64, 50, &rr);
        rows += uint64_t(o.rows);
        if (rows >= 2ull * per_part) ring->slot(g)->flags |= kSlotEOS;
        ring->worker_publish(g);
        ++i;
      }
    });
  }
  std::vector<uint32_t> cursor(nw, 0);
  std::vector<uint8_t> done(nw, 0);
  uint32_t rr = 0;
  uint64_t rows = 0;
  const uint32_t grp = b->group_index("stress", true);
  std::vector<int64_t> expect(np, 0);
  for (;;) {
    const int64_t g = ring->main_acquire(cursor.data(), &rr, done.data(), false, 60000);
    if (g == -2) break;
    CHECK(g >= 0);
    SlotHeader* h = ring->slot(uint32_t(g));
    const float* vals = reinterpret_cast<const float*>(ring->payload(uint32_t(g)));
    std::vector<CommitEntry> ce;
    // rows of different partitions may interleave (a packer revisits a partition that grew
    // while it read another); per partition they are contiguous offsets from first_offset
    std::vector<int64_t> next_row(np, -1);
    uint32_t total = 0;
    for (uint32_t k = 0; k < h->n_parts; ++k) {
      const Watermark& wm = h->wm[k];
      CHECK(wm.first_offset == expect[wm.pidx - t.first_pidx]);  // contiguous, exact offsets
      next_row[wm.pidx - t.first_pidx] = wm.first_offset;
      total += wm.count;
    }
    CHECK(total == h->n_rows);
    for (uint32_t r = 0; r < h->n_rows; ++r) {
      const uint32_t p = uint32_t(vals[r * 16 + 1]) - t.first_pidx;
      CHECK(p < np && next_row[p] >= 0);
      CHECK(vals[r * 16] == float(next_row[p]));
      ++next_row[p];
    }
    for (uint32_t k = 0; k < h->n_parts; ++k) {
      const Watermark& wm = h->wm[k];
      CHECK(next_row[wm.pidx - t.first_pidx] == wm.next_offset);
      expect[wm.pidx - t.first_pidx] = wm.next_offset;
      ce.push_back(CommitEntry{wm.pidx, wm.next_offset, std::string()});
    }
    rows += h->n_rows;
    b->commit(grp, -1, 0, 0, ce);
    if (h->flags & kSlotEOS) done[h->worker] = 1;
    ring->main_release(uint32_t(g));
  }
  stop = true;
  for (auto& th : prod) th.join();
  for (auto& th : packers) th.join();
  CHECK(rows == uint64_t(np) * per_part);
  for (uint32_t p = 0; p < np; ++p) CHECK(b->committed(grp, t.first_pidx + p) == int64_t(per_part));
  ring->shutdown();
  ring->unlink();
  std::string dir = b->dir();
  b.reset();
  if (std::system(("rm -rf '" + dir + "'").c_str()) != 0) std::fprintf(stderr, "could not remove %s\n", dir.c_str());
  std::printf("broker pipeline: %u packers, %llu rows, exact commits ok\n", nw, (unsigned long long)rows);
}

int main(int argc, char** argv) {
  const uint32_t nw = argc > 1 ? uint32_t(std::atoi(argv[1])) : 4;
  const uint32_t spw = argc > 2 ? uint32_t(std::atoi(argv[2])) : 3;
  const uint32_t n = argc > 3 ? uint32_t(std::atoi(argv[3])) : 3000;
  ring_protocol(nw, spw, n);
  broker_pipeline(nw, n / 2);
  return 0;
}
