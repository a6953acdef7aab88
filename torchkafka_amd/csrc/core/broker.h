// Synthetic Kafka broker living in shared memory (or a persistent directory).
//
// Role: stands in for the Kafka cluster the reference talks to through
// kafka-python (reference kafka_dataset.py:21-22,206).  It keeps
// the exact semantics the reference's commit protocol depends on:
//   * partitioned append-only logs of RecordBatch v2 bytes (zero-copy fetch);
//   * per-(group, partition) committed offsets that survive process restarts
//     when the broker directory is on disk (the "checkpoint");
//   * consumer groups with range assignment, generations and rebalances, so
//     a stale member's commit fails with CommitFailedError (B14);
//   * fault injection: commit failures, slow and failing fetches (D3/D4/D8 tests).
//
// Layout of a broker directory:
//   lock          flock()ed while the meta file is created
//   meta          MetaHeader | TopicEntry[] | PartitionEntry[] | GroupEntry[] |
//                 owners int16[groups][partitions] | OffsetEntry[groups][partitions]
//   pNNNNN.log    RecordBatch bytes of global partition NNNNN (sparse, mmap'ed)
//   pNNNNN.idx    IndexEntry per batch (base offset -> file position)
// Every process maps the files MAP_SHARED; cross-process synchronisation uses
// atomics in the mapping plus robust process-shared pthread mutexes.
#pragma once
#include <pthread.h>

#include <atomic>
#include <utility>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "common.h"
#include "record_batch.h"

namespace tk {

constexpr uint64_t kBrokerMagic = 0x31304B4F5242544BULL;  // "TKBROK01"
constexpr uint32_t kBrokerVersion = 1;
constexpr int kMaxMembers = 64;
constexpr int kMaxSubscribedTopics = 16;
constexpr int kNameLen = 160;

struct BrokerConfig {
  uint32_t max_topics = 256;
  uint32_t max_partitions = 4096;
  uint32_t max_groups = 64;
  uint64_t default_log_capacity = 256ull << 20;   // bytes per partition (sparse)
  uint64_t default_index_capacity = 1u << 20;     // batches per partition
  uint32_t group_initial_rebalance_delay_ms = 100;
};

enum BrokerFlags : uint32_t {
  // Log bytes below a partition's committed position may be released (a replica: KafkaBridge owns
  // the broker and one group consumes it).  The replicator punches them out of the log files, the
  // device driver unpins them; the log start offset moves up to the committed offset.
  kReleaseConsumed = 1,
};

struct alignas(64) MetaHeader {
  uint64_t magic;
  uint32_t version;
  std::atomic<uint32_t> ready;
  uint32_t max_topics, max_partitions, max_groups, group_initial_rebalance_delay_ms;
  uint64_t default_log_capacity, default_index_capacity;
  std::atomic<uint32_t> n_topics, n_partitions, n_groups, flags;  // flags: BrokerFlags
  pthread_mutex_t lock;  // topic/group creation, membership changes
};

struct alignas(64) TopicEntry {
  char name[kNameLen];
  uint32_t n_partitions;
  uint32_t first_pidx;
  uint64_t log_capacity;
  uint64_t index_capacity;
};

struct IndexEntry {
  int64_t base_offset;
  uint64_t pos;
  uint32_t size;
  int32_t last_offset_delta;
  int64_t max_timestamp;
};
static_assert(sizeof(IndexEntry) == 32, "index entry layout");

struct alignas(64) PartitionEntry {
  pthread_mutex_t lock;                   // producer append lock
  std::atomic<int64_t> high_watermark;    // next offset to be produced
  std::atomic<int64_t> log_start_offset;  // first retained offset
  std::atomic<uint64_t> log_end_pos;      // bytes used in the .log file
  std::atomic<uint64_t> n_batches;        // published index entries
  uint64_t log_capacity, index_capacity;
  uint32_t topic_index, partition;
  // fault injection & metrics
  std::atomic<int64_t> fetch_delay_ns;
  std::atomic<int32_t> fetch_errors;
  // Device readers (MainDriver) that pinned this log with hipHostRegister, and the lowest log byte
  // they still hold pinned.  Released (punched) bytes must stay below pin_floor: invalidating the
  // CPU mapping of a pinned range makes the GPU driver evict and re-pin it (a ~100 ms stall).
  std::atomic<uint32_t> pinned;
  std::atomic<uint64_t> fetch_calls, bytes_fetched, records_produced;
  std::atomic<uint64_t> pin_floor;  // in the struct's former tail padding: the layout is unchanged
  // Ring logs (KafkaBridge replicas): the log is a ring of ring_bytes whose pages are written over
  // once their batches are committed -- the pages stay allocated and pinned, so a long stream
  // needs no page freeing, unpinning or re-pinning.  Index entries are a ring too: logical batch
  // i lives in slot i % index_capacity; [first_batch, n_batches) are live.  Linear logs: 0, 0.
  std::atomic<uint64_t> ring_bytes;
  std::atomic<uint64_t> first_batch;
};
static_assert(sizeof(PartitionEntry) == 192, "partition entry layout (shared with existing broker files)");

struct alignas(64) MemberEntry {
  std::atomic<uint32_t> active;
  int32_t pid;
  std::atomic<int64_t> last_poll_ns;
  int64_t session_timeout_ns;
  int64_t max_poll_interval_ns;
  uint64_t member_id;
  uint32_t n_topics;
  uint32_t topics[kMaxSubscribedTopics];
  // a rebalance round of a group that had members (GroupEntry::awaiting): this member rejoined
  // (committed what it finished and gave its partitions up) -- in the struct's tail padding
  std::atomic<uint32_t> rejoined;
};

enum GroupState : uint32_t { kGroupEmpty = 0, kGroupPreparing = 1, kGroupStable = 2 };

struct alignas(64) GroupEntry {
  char name[kNameLen];
  std::atomic<uint32_t> generation;
  std::atomic<uint32_t> state;
  int64_t prepare_deadline_ns;
  uint64_t next_member_id;
  std::atomic<int32_t> inject_commit_failures;
  // Preparing because the membership of a group with members changed: every member must rejoin
  // (Kafka's PreparingRebalance; commits of the current generation are still accepted) before the
  // partitions are reassigned, or be dropped at prepare_deadline_ns (the rebalance timeout).
  // 0: Preparing is the initial delay of an empty group.
  std::atomic<int32_t> awaiting;
  std::atomic<uint64_t> n_commits;
  std::atomic<int64_t> last_expiry_check_ns;
  MemberEntry members[kMaxMembers];
};

struct alignas(64) OffsetEntry {
  std::atomic<int64_t> offset;  // -1 = nothing committed
  std::atomic<uint64_t> seq;
  std::atomic<int64_t> commit_wall_ms;
  int32_t meta_len;
  char metadata[36];
};

struct TopicInfo {
  uint32_t index, n_partitions, first_pidx;
  std::string name;
};

struct CommitEntry {
  uint32_t pidx;
  int64_t offset;
  std::string metadata;
};

struct GroupView {
  uint32_t generation;
  uint32_t state;
  bool member_active;       // false: this member was evicted / left
  std::vector<uint32_t> assignment;  // global partition indices (sorted)
};

class Broker {
 public:
  // url: "shm://name" -> /dev/shm/torchkafka/name ; "file:///abs/dir" or a plain path.
  static std::string url_to_dir(const std::string& url);
  Broker(const std::string& url, bool create, const BrokerConfig& cfg);
  ~Broker();
  Broker(const Broker&) = delete;
  Broker& operator=(const Broker&) = delete;

  const std::string& dir() const { return dir_; }
  const MetaHeader& meta() const { return *meta_; }

  // ---- topics
  TopicInfo create_topic(const std::string& name, uint32_t n_partitions, uint64_t log_capacity = 0,
                         uint64_t index_capacity = 0);
  bool find_topic(const std::string& name, TopicInfo* out) const;
  std::vector<TopicInfo> topics() const;
  PartitionEntry& part(uint32_t pidx);
  const PartitionEntry& part(uint32_t pidx) const;

  // ---- log access (zero-copy)
  const uint8_t* log_base(uint32_t pidx);
  const IndexEntry* index_base(uint32_t pidx);
  // Index of the batch containing `offset` (requires log_start <= offset < hw), hint = last result.
  int64_t find_batch(uint32_t pidx, int64_t offset, int64_t hint) ;
  // ListOffsets-by-timestamp: earliest retained record with timestamp >= ts, as {offset, timestamp};
  // {-1, -1} when none.  Skips whole batches by the index's max_timestamp.
  std::pair<int64_t, int64_t> offset_for_time(uint32_t pidx, int64_t ts);

  // ---- produce: appends one batch, returns its base offset.
  int64_t append(uint32_t pidx, const RecordIn* recs, size_t n);
  // Synthetic generator (see SyntheticSpec in broker.cpp): fills n records per partition.
  // keyed: every record carries an 8-byte big-endian key, its offset % 1000 (a label).
  void fill_synthetic(const std::vector<uint32_t>& pidxs, int64_t n_records, int kind, int64_t size_a,
                      int64_t size_b, uint32_t records_per_batch, uint64_t seed, int n_threads, bool keyed = false);
  void delete_records(uint32_t pidx, int64_t before_offset);

  // ---- replica ingest (replicator.h: a Kafka cluster mirrored into this broker's logs)
  // Writable tail of a partition log: bytes [log_end_pos, capacity) -- a Fetch response's record
  // set is received straight into it, then ingest() indexes the whole batches it holds.
  uint8_t* log_tail(uint32_t pidx, uint64_t* avail);
  // An empty partition starts at `offset` (log start = high watermark = offset).
  void reset_empty(uint32_t pidx, int64_t offset);
  // Drops everything a replica partition holds and restarts it, empty, at `offset` (the log is
  // rewritten from byte 0; a ring stays a ring).  For a partition a group rebalance gives back to
  // this replica: its cluster-committed offset may lie outside what the local log still holds.
  // Nobody may be reading the partition (the replica's consumers dropped it when it was revoked).
  void reset_partition(uint32_t pidx, int64_t offset);
  struct Ingested {
    uint64_t consumed = 0;     // bytes of whole batches walked (kept or dropped)
    uint64_t kept_bytes = 0;
    uint32_t kept = 0, control = 0, inflated = 0;  // inflated: compressed batches stored decompressed
    uint64_t inflated_bytes = 0;  // bytes of those batches as stored
    uint64_t inflated_from = 0;   // ... and as received (compressed)
    uint64_t inflate_ns = 0;      // time spent inflating them (+ their fresh CRC)
    bool full = false;         // stopped at a batch the space left could not hold
    int64_t next_offset = -1;  // next offset to fetch (-1: no whole batch in the data)
  };
  // Walks the RecordBatches received at log_tail(): keeps (indexes, publishes) whole data
  // batches at or beyond `from_offset`, drops control batches (transaction markers) and
  // batches already held, compacting in place; a trailing partial batch is left for the next
  // fetch to overwrite.  Compressed batches (gzip/snappy/lz4/zstd, codecs.h) are CRC-checked and
  // inflated straight into the log, as plain RecordBatch v2 with a fresh CRC: the device path
  // decodes raw records.  Runs on the calling (fetch) thread.
  // keep_control: store control batches too (a broker's own log, e.g. the wire server's tests).
  // `limit`: bytes from the write position the batches may occupy (0: up to the capacity); a batch
  // that does not fit ends the walk (Ingested::full) and is fetched again later.
  // `src`: the record set lies in a buffer of the caller's instead of at log_tail() (a fetch
  // thread handing compressed record sets to an inflater, replicator.cpp).
  Ingested ingest(uint32_t pidx, uint64_t len, int64_t from_offset, bool keep_control = false, uint64_t limit = 0,
                  const uint8_t* src = nullptr);
  // Log byte position of the first batch holding an offset >= `offset` (log end if none).
  uint64_t position_of(uint32_t pidx, int64_t offset);
  // Index entry of logical batch i (ring-indexed: slot i % index_capacity).
  IndexEntry entry(uint32_t pidx, int64_t i) { return mapped(pidx).idx[uint64_t(i) % part(pidx).index_capacity]; }
  // Turns an empty partition into a ring log of `bytes` (<= its capacity).
  void make_ring(uint32_t pidx, uint64_t bytes);
  // Faults in the pages of partition pidx's ring (a replica's first pass through it then pays none).
  void populate_ring(uint32_t pidx);
  // Ring logs: retires live batches that end at or below `keep_offset` (log start moves up), then
  // returns the write position with up to `want` contiguous bytes that overwrite no live batch
  // (wrapping to the ring's start when the tail is too short); *avail = those bytes (may be < want).
  uint8_t* ring_reserve(uint32_t pidx, uint64_t want, int64_t keep_offset, uint64_t* avail);
  uint32_t flags() const { return meta_->flags.load(std::memory_order_acquire); }
  void set_flags(uint32_t f) { meta_->flags.fetch_or(f, std::memory_order_acq_rel); }
  // Frees log bytes [from, to) (page-aligned inwards) of a partition: FALLOC_FL_PUNCH_HOLE on its
  // log file, so every process's mapping of them drops to the zero page.  Returns bytes released.
  uint64_t release_log(uint32_t pidx, uint64_t from, uint64_t to);

  // ---- groups / offsets
  uint32_t group_index(const std::string& group, bool create = true);
  std::string group_name(uint32_t g) const;
  // Joins (subscribe mode).  Returns member slot.
  int join_group(uint32_t g, const std::vector<uint32_t>& topic_indices, int64_t session_timeout_ms,
                 int64_t max_poll_interval_ms);
  void leave_group(uint32_t g, int member_slot, uint64_t member_id);
  // During a rejoin round (poll_group reports Preparing): this member committed what it finished
  // and gave its partitions up.  No-op outside a round.
  void rejoin_group(uint32_t g, int member_slot, uint64_t member_id);
  uint64_t member_id(uint32_t g, int slot) const;
  GroupView poll_group(uint32_t g, int member_slot, uint64_t member_id);
  // member_slot < 0: manual-assignment ("simple") consumer.
  void commit(uint32_t g, int member_slot, uint64_t member_id, uint32_t generation,
              const std::vector<CommitEntry>& entries);
  int64_t committed(uint32_t g, uint32_t pidx, std::string* metadata = nullptr) const;
  uint64_t commit_count(uint32_t g) const;
  void inject_commit_failures(uint32_t g, int32_t n);
  void reset_group_offsets(uint32_t g);

  // ---- fault injection
  void set_fetch_delay(uint32_t pidx, int64_t delay_ns) { part(pidx).fetch_delay_ns.store(delay_ns); }
  void inject_fetch_errors(uint32_t pidx, int32_t n) { part(pidx).fetch_errors.store(n); }

 private:
  struct Mapped {
    uint8_t* log = nullptr;
    IndexEntry* idx = nullptr;
    size_t log_len = 0, idx_len = 0;
  };
  void map_meta(bool create, const BrokerConfig& cfg);
  Mapped& mapped(uint32_t pidx);
  GroupEntry& group(uint32_t g) const;
  int16_t* owners(uint32_t g) const;
  OffsetEntry& offset_entry(uint32_t g, uint32_t pidx) const;
  void rebalance_locked(GroupEntry& G, uint32_t g, int64_t now, bool immediate);
  // The membership of a group with members changed: start a rejoin round (or, with nobody left
  // to wait for, reassign now).
  void membership_changed_locked(GroupEntry& G, uint32_t g, int64_t now);
  // A rejoin round ends once every active member rejoined, or at its deadline (absentees dropped).
  void try_complete_round_locked(GroupEntry& G, uint32_t g, int64_t now);
  void assign_locked(GroupEntry& G, uint32_t g);
  bool expire_members_locked(GroupEntry& G, int64_t now);

  std::string dir_;
  int meta_fd_ = -1;
  uint8_t* meta_map_ = nullptr;
  size_t meta_len_ = 0;
  MetaHeader* meta_ = nullptr;
  TopicEntry* topics_ = nullptr;
  PartitionEntry* parts_ = nullptr;
  GroupEntry* groups_ = nullptr;
  int16_t* owners_ = nullptr;
  OffsetEntry* offsets_ = nullptr;
  std::vector<Mapped> maps_;
  std::mutex maps_mu_;
};

// Locks a robust process-shared mutex, recovering it if its owner died.
class RobustLock {
 public:
  explicit RobustLock(pthread_mutex_t* m);
  ~RobustLock();

 private:
  pthread_mutex_t* m_;
};
void init_robust_mutex(pthread_mutex_t* m);

}  // namespace tk
