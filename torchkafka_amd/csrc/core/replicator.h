// Kafka cluster -> local partition logs: the native bridge between a real cluster and the
// device path.
//
// The reference consumes through kafka-python (kafka_dataset.py:21-22, 206-210): every worker
// owns a KafkaConsumer whose fetcher parses each response in Python and CRC-checks every batch
// on the CPU before `_process` sees a record.  Here one native replicator per rank (threads,
// no GIL) fetches the rank's partitions over the Kafka protocol (kafka_wire.h) and receives
// each response's record set directly into the tail of a local partition log -- the same
// mapped RecordBatch v2 logs the synthetic broker serves.  Everything downstream is unchanged:
// workers walk record headers in those logs, the main process pins them, and the gfx950
// kernels verify CRC32C and decode values from them (span_decode.hip / json_span.hip).
// Offsets are preserved, so what the loader commits into the local offset table is exactly the
// cluster's offset; a committer thread forwards those commits to the group coordinator
// (OffsetCommit), and close() flushes the last one.
//
// Flow control: a partition is not fetched while its replicated-but-uncommitted bytes exceed
// `max_lag_bytes` (the loader commits every batch, so this bounds host memory per partition).
#pragma once
#include <atomic>
#include <condition_variable>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "broker.h"
#include "kafka_wire.h"

namespace tk {

struct ReplicaConfig {
  std::string bootstrap;               // "host:port[,host:port]" (kafka:// accepted)
  std::string topic;
  std::string group;                   // committed offsets: read at start, forwarded on commit
  std::string client_id = "torchkafka-replicator";
  wire::Security security;             // TLS / SASL (kafka-python's security_protocol, ssl_*, sasl_*)
  std::vector<int32_t> partitions;     // empty: every partition of the topic
  // Subscribe mode: join `group` (JoinGroup/SyncGroup, range or round-robin assignor) and mirror
  // the partitions the coordinator assigns, as kafka-python's subscribe() does.  Rebalances are
  // followed in process: heartbeats (on the commit thread) notice a rebalance, the replica forwards
  // what was consumed, rejoins, stops fetching revoked partitions and starts the newly assigned
  // ones at the group's committed offset.  assignment_epoch() / partition_epoch() tell consumers
  // of the local replica which partitions (re)started, so they drop what they buffered of them.
  bool subscribe = false;
  std::vector<std::string> assignors{"range"};  // partition_assignment_strategy, in preference order
  int32_t session_timeout_ms = 10000;
  int32_t heartbeat_interval_ms = 3000;
  int32_t rebalance_timeout_ms = 0;    // JoinGroup v1+ (kafka-python: max_poll_interval_ms); 0: session timeout
  std::string auto_offset_reset = "earliest";  // without a committed offset: earliest | latest
  int32_t max_wait_ms = 100;
  int32_t min_bytes = 1;
  int32_t max_bytes = 64 << 20;        // per Fetch response
  int32_t partition_max_bytes = 8 << 20;
  int32_t timeout_ms = 30000;
  int64_t max_lag_bytes = int64_t(1) << 30;
  int32_t commit_interval_ms = 5;
  int32_t fetchers = 0;                // fetch threads (0: one per partition, at most 8; at least one per leader)
  bool release_consumed = true;        // free committed log bytes (punch holes; kReleaseConsumed)
  uint64_t release_bytes = 256u << 20; // ... keeping this many consumed bytes per partition resident
  uint64_t release_step = 1u << 30;    // ... in bursts, once a partition has this many releasable bytes
  // Ring replica (the default for device loaders): each partition log is a ring of this many bytes
  // whose committed batches are written over -- pages allocated and pinned once, no release.
  // 0: a linear log (grows; committed bytes released per release_consumed).
  uint64_t ring_bytes = 0;
  uint64_t log_capacity = 0;           // local topic creation (0: the broker default)
  uint64_t index_capacity = 0;
};

struct ReplicaPartStats {
  int32_t partition;
  uint32_t pidx;
  int64_t start_offset;
  int64_t fetch_offset;
  int64_t remote_hw;
  int64_t forwarded;        // last offset committed to the cluster (-1 none)
  uint64_t bytes;
  uint64_t batches;
  uint64_t control_batches;
  uint64_t fetches;
  uint64_t throttled;       // fetch rounds skipped by flow control
  uint64_t released;        // log bytes released below the committed position
  bool owned;               // subscribe mode: assigned to this member now
  // where a fetch thread's time goes, per partition: the record sets as received (compressed),
  // the time reading them off the socket into the log, the whole ingest walk, and the part of it
  // spent inflating compressed batches (decode + fresh CRC), which yielded inflated_bytes
  uint64_t wire_bytes;
  uint64_t recv_ns;
  uint64_t ingest_ns;
  uint64_t inflate_ns;
  uint64_t inflated_batches;
  uint64_t inflated_bytes;
};

class Replicator {
 public:
  Replicator(std::shared_ptr<Broker> local, ReplicaConfig cfg);
  ~Replicator();
  Replicator(const Replicator&) = delete;
  Replicator& operator=(const Replicator&) = delete;

  // Metadata, local topic, start positions (committed offset, else auto_offset_reset), threads.
  void start();
  // Stops fetching; forwards the latest local commits first when `flush`.
  void stop(bool flush = true);
  // SASL/OAUTHBEARER: the token (and extensions) the connections made from now on present
  // (KafkaBridge refreshes it from the sasl_oauth_token_provider).
  void set_oauth_token(const std::string& token, const std::string& extensions);
  // Forwards every changed local commit to the coordinator now; returns partitions committed.
  int flush_commits();
  // Synchronous commit (DeviceLoader commit="sync"): wakes the commit thread, which forwards every
  // changed local commit on its coordinator connection; returns once that OffsetCommit was answered
  // -- true when every partition committed cleanly, false on an error or after timeout_ms.
  bool commit_sync(int timeout_ms);
  // Durations of the OffsetCommit round trips the commit thread made since the last call.
  std::vector<int64_t> take_forward_ns();
  bool running() const { return running_.load(); }
  std::string last_error();
  int64_t errors() const { return errors_.load(); }
  std::vector<ReplicaPartStats> stats();
  uint32_t first_pidx() const { return first_pidx_; }
  int32_t n_partitions() const { return n_remote_parts_; }
  // subscribe mode: this member's id / generation / assigned partitions (snapshots: the commit
  // thread rewrites them during a rebalance)
  std::string member_id() const;
  int32_t generation() const;
  std::vector<int32_t> assignment() const;
  // Bumped whenever the assignment changes; partition_epoch(p) is the epoch at which partition p
  // was last (re)assigned to this replica -- a consumer holding older state of p must drop it.
  uint64_t assignment_epoch() const { return epoch_.load(std::memory_order_acquire); }
  const std::atomic<uint64_t>* epoch_ptr() const { return &epoch_; }
  std::vector<std::pair<int32_t, uint64_t>> assignment_epochs() const;
  uint64_t rebalances() const { return rebalances_.load(); }
  // record sets dropped because they did not start at the log's end (then refetched)
  uint64_t out_of_order() const { return out_of_order_.load(); }
  // Never set any more (rebalances are followed in process); kept for API compatibility.
  bool fenced() const { return false; }
  int fetch_threads() const { return n_fetch_threads_; }
  // Summed over the fetch threads: time from a Fetch request sent to its response's first bytes.
  uint64_t fetch_wait_ns() const { return fetch_wait_ns_.load(std::memory_order_relaxed); }
  // Inflater threads started (one per fetch thread that met a compressed partition).
  int inflate_threads() const { return n_inflaters_.load(std::memory_order_relaxed); }
  // Blocks until every replicated partition has fetched up to the cluster's high watermark as
  // seen at call time (tests, tools); false on timeout.
  bool wait_caught_up(int timeout_ms);

 private:
  struct Part {
    int32_t partition;
    uint32_t pidx;
    int64_t start_offset = 0;
    std::atomic<int64_t> fetch_offset{0};
    std::atomic<int64_t> remote_hw{-1};
    std::atomic<int64_t> forwarded{-1};
    std::atomic<uint64_t> bytes{0}, batches{0}, control{0}, fetches{0}, throttled{0};
    std::atomic<uint64_t> released{0};  // log bytes [0, released) freed (committed past)
    std::atomic<uint64_t> wire_bytes{0}, recv_ns{0}, ingest_ns{0}, inflate_ns{0}, inflated{0}, inflated_bytes{0};
    // inflation of the compressed batches last received, x16 (16: uncompressed): a ring replica
    // reserves that much more room and asks for that much less per Fetch, so what it fetches fits
    std::atomic<uint32_t> ratio16{16};
    // compressed partitions (ratio16 > 16): record sets handed to the fetch thread's inflater and
    // not yet stored, the offset to ask for next while any are, and the assignment epoch at which
    // the inflater failed on this partition (~0: never)
    std::atomic<int> inflight{0};
    std::atomic<int64_t> ask_offset{0};
    std::atomic<uint64_t> failed_since{~uint64_t(0)};
    // pipeline generation: bumped whenever fetch_offset jumps (OffsetOutOfRange reset, a restart by
    // a rebalance, an out-of-order set): record sets asked for under an older generation are dropped
    std::atomic<uint64_t> gen{0};
    std::atomic<bool> owned{true};       // subscribe mode: assigned to this member now
    std::atomic<uint64_t> since{0};      // assignment epoch at which it was (re)assigned
    std::mutex mu;                       // a fetch's write into the log vs. a restart of the partition
  };
  // A compressed partition's record set, received by a fetch thread into a buffer of its own and
  // inflated into the log by that thread's inflater (one per fetch thread), so the wait for the
  // next Fetch response overlaps this one's inflation.  At most max_inflight_ per partition
  // (TORCHKAFKA_BRIDGE_INFLIGHT, default 2).
  int max_inflight_ = 2;
  struct Pending {
    Part* p;
    uint64_t since;
    uint64_t gen;    // Part::gen when the set was asked for
    int64_t asked;   // the offset it was asked from: stored only where the log ends (contiguity)
    std::vector<uint8_t> data;
  };
  struct Inflater {
    std::mutex m;
    std::condition_variable cv, done_cv;
    std::deque<Pending> q;
    std::vector<std::vector<uint8_t>> spare;
    bool stop = false;
  };
  void inflate_loop(Inflater* inf);
  void inflate_one(Pending& pd);
  void release_loop();
  void fetch_loop(std::vector<Part*> mine);
  void commit_loop();
  bool throttled(Part& p);
  int64_t keep_offset(Part& p);
  uint8_t* room(Part& p, uint64_t* avail);
  void reset_offset(wire::Client& c, Part& p);
  void resync(Part& p, const char* where);
  void grow_reserve(Part& p);
  void set_error(const std::string& e);
  int forward(wire::Client& c);

  std::shared_ptr<Broker> local_;
  ReplicaConfig cfg_;
  uint32_t group_ = 0;
  uint32_t first_pidx_ = 0;
  int32_t n_remote_parts_ = 0;
  std::vector<std::unique_ptr<Part>> parts_;
  std::vector<std::thread> threads_;
  std::atomic<bool> running_{false};
  std::atomic<bool> stop_{false};
  std::atomic<int64_t> errors_{0};
  std::mutex err_mu_;
  std::string last_error_;
  std::mutex commit_mu_;  // serialises forward() between the committer thread and flush_commits()
  std::mutex sync_mu_;    // commit_sync() requests / the commit thread's answers
  std::condition_variable sync_cv_;
  uint64_t sync_req_ = 0, sync_done_ = 0;
  bool sync_ok_ = true;
  std::mutex stats_mu_;
  std::vector<int64_t> forward_ns_;
  std::unique_ptr<wire::Client> commit_client_;
  std::vector<int32_t> join_group(wire::Client& c);  // sets member_id_ / generation_
  void heartbeat(wire::Client& c);
  // Starts owned partitions at the group's committed offset (else auto_offset_reset).
  void start_parts(wire::Client& c, const std::vector<Part*>& ps, bool fresh);
  void apply_assignment(wire::Client& c, const std::vector<int32_t>& mine);
  mutable std::mutex assign_mu_;  // member_id_ / generation_ / assigned_ snapshots for readers
  std::string member_id_;
  int32_t generation_ = -1;
  std::vector<int32_t> assigned_;
  std::atomic<uint64_t> epoch_{0}, rebalances_{0}, out_of_order_{0};
  int64_t last_heartbeat_ms_ = 0;
  int n_fetch_threads_ = 0;
  std::atomic<uint64_t> fetch_wait_ns_{0};
  std::atomic<int> n_inflaters_{0};
};

}  // namespace tk
