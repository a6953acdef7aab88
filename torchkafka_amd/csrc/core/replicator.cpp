// Kafka cluster -> local partition logs: see replicator.h.
#include "replicator.h"

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <set>

namespace tk {

namespace {
void sleep_ms(int ms) { std::this_thread::sleep_for(std::chrono::milliseconds(ms)); }
int64_t now_ms() {
  return std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
}  // namespace

Replicator::Replicator(std::shared_ptr<Broker> local, ReplicaConfig cfg) : local_(std::move(local)), cfg_(std::move(cfg)) {
  if (const char* e = std::getenv("TORCHKAFKA_BRIDGE_INFLIGHT")) max_inflight_ = std::max(1, std::min(16, std::atoi(e)));
  if (cfg_.topic.empty()) throw std::invalid_argument("replicator: a topic is required");
  if (cfg_.auto_offset_reset != "earliest" && cfg_.auto_offset_reset != "latest" &&
      cfg_.auto_offset_reset != "smallest" && cfg_.auto_offset_reset != "largest")
    throw std::invalid_argument("replicator: auto_offset_reset must be 'earliest' or 'latest'");
  if (cfg_.partition_max_bytes < 4096 || cfg_.max_bytes < cfg_.partition_max_bytes)
    throw std::invalid_argument("replicator: need 4096 <= partition_max_bytes <= max_bytes");
}

Replicator::~Replicator() {
  try {
    stop(false);
  } catch (...) {
  }
}

void Replicator::set_error(const std::string& e) {
  errors_.fetch_add(1);
  std::lock_guard<std::mutex> g(err_mu_);
  last_error_ = e;
}

std::string Replicator::last_error() {
  std::lock_guard<std::mutex> g(err_mu_);
  return last_error_;
}

void Replicator::start() {
  if (running_.load()) return;
  wire::Client c(cfg_.bootstrap, cfg_.client_id, cfg_.timeout_ms, cfg_.security);
  wire::TopicMeta t = c.metadata(cfg_.topic);
  if (t.error != wire::kNone || t.partitions.empty())
    throw wire::WireError(t.error ? t.error : int16_t(wire::kUnknownTopicOrPartition),
                          std::string(wire::error_name(t.error)) + ": topic '" + cfg_.topic + "'");
  n_remote_parts_ = int32_t(t.partitions.size());
  TopicInfo ti;
  if (!local_->find_topic(cfg_.topic, &ti)) ti = local_->create_topic(cfg_.topic, uint32_t(n_remote_parts_),
                                                                     cfg_.log_capacity, cfg_.index_capacity);
  if (int32_t(ti.n_partitions) != n_remote_parts_)
    throw KafkaError("replicator: local topic '" + cfg_.topic + "' has " + std::to_string(ti.n_partitions) +
                     " partitions, the cluster " + std::to_string(n_remote_parts_));
  first_pidx_ = ti.first_pidx;
  if (cfg_.ring_bytes && cfg_.ring_bytes < (uint64_t(cfg_.partition_max_bytes) * 4))
    throw std::invalid_argument("replicator: ring_bytes must hold at least 4 x partition_max_bytes");
  if (cfg_.ring_bytes) cfg_.release_consumed = false;  // a ring reuses its pages: nothing to free
  if (cfg_.release_consumed && !cfg_.group.empty()) local_->set_flags(kReleaseConsumed);
  std::vector<int32_t> mine;
  if (cfg_.subscribe) {
    if (cfg_.group.empty()) throw std::invalid_argument("replicator: subscribe mode needs a group");
    mine = join_group(c);
  }
  // subscribe mode keeps a Part for every partition of the topic (the assignment moves between
  // them); static mode only for the partitions it mirrors
  std::vector<int32_t> ids = cfg_.subscribe ? std::vector<int32_t>() : cfg_.partitions;
  if (ids.empty())
    for (auto& p : t.partitions) ids.push_back(p.partition);
  std::sort(ids.begin(), ids.end());
  ids.erase(std::unique(ids.begin(), ids.end()), ids.end());
  for (int32_t id : ids)
    if (id < 0 || id >= n_remote_parts_)
      throw KafkaError("UnknownTopicOrPartitionError: " + cfg_.topic + "-" + std::to_string(id));
  if (!cfg_.group.empty()) group_ = local_->group_index(cfg_.group, true);

  parts_.clear();
  std::vector<Part*> owned;
  const std::set<int32_t> assigned(mine.begin(), mine.end());
  for (int32_t id : ids) {
    auto p = std::make_unique<Part>();
    p->partition = id;
    p->pidx = first_pidx_ + uint32_t(id);
    p->owned = !cfg_.subscribe || assigned.count(id) > 0;
    p->fetch_offset = -1;
    if (p->owned) owned.push_back(p.get());
    parts_.push_back(std::move(p));
  }
  start_parts(c, owned, true);
  {
    std::lock_guard<std::mutex> g(assign_mu_);
    for (Part* p : owned) p->since = 1;
    assigned_ = mine;
    epoch_.store(1, std::memory_order_release);
  }

  // fetch threads: partitions grouped by leader, leaders spread over the threads
  std::map<int32_t, std::vector<Part*>> by_leader;
  for (auto& p : parts_) by_leader[c.leader(cfg_.topic, p->partition)].push_back(p.get());
  // default: one thread per partition, at most 8 (and at least one per leader): a thread inflates
  // the compressed batches it receives, so compressed topics spread that work over the threads
  int n_threads = cfg_.fetchers > 0 ? cfg_.fetchers
                                    : std::max<int>(int(by_leader.size()), std::min<int>(8, int(parts_.size())));
  n_threads = std::max(1, std::min<int>(n_threads, int(parts_.size())));
  std::vector<std::vector<Part*>> per(static_cast<size_t>(n_threads));
  size_t k = 0;
  for (auto& [leader, ps] : by_leader)
    for (Part* p : ps) per[(k++) % per.size()].push_back(p);
  stop_ = false;
  running_ = true;
  n_fetch_threads_ = 0;
  for (auto& v : per)
    if (!v.empty()) {
      threads_.emplace_back([this, v]() { fetch_loop(v); });
      ++n_fetch_threads_;
    }
  if (!cfg_.group.empty()) {
    commit_client_ = std::make_unique<wire::Client>(cfg_.bootstrap, cfg_.client_id + "-commit", cfg_.timeout_ms, cfg_.security);
    threads_.emplace_back([this]() { commit_loop(); });
    if (cfg_.release_consumed) threads_.emplace_back([this]() { release_loop(); });
  }
}

// Positions of partitions this replica starts owning: the group's committed offset, else
// auto_offset_reset.  `fresh` (start()): a persistent replica's log that can serve that offset is
// resumed; otherwise -- and always for a partition a rebalance handed over -- the local partition
// restarts, empty, at that offset (the log may hold a stale or overwritten range of it).
void Replicator::start_parts(wire::Client& c, const std::vector<Part*>& ps, bool fresh) {
  if (ps.empty()) return;
  std::vector<uint32_t> fresh_rings;
  std::vector<int32_t> ids;
  for (Part* p : ps) ids.push_back(p->partition);
  std::map<int32_t, int64_t> committed;
  if (!cfg_.group.empty()) committed = c.offset_fetch(cfg_.group, cfg_.topic, ids);
  std::vector<int32_t> need_reset;
  for (int32_t id : ids) {
    auto it = committed.find(id);
    if (it == committed.end() || it->second < 0) need_reset.push_back(id);
  }
  const bool latest = cfg_.auto_offset_reset == "latest" || cfg_.auto_offset_reset == "largest";
  std::map<int32_t, int64_t> reset;
  if (!need_reset.empty()) reset = c.list_offsets(cfg_.topic, need_reset, latest ? -1 : -2);
  for (Part* p : ps) {
    auto ci = committed.find(p->partition);
    const int64_t remote_committed = ci != committed.end() ? ci->second : -1;
    const int64_t start = remote_committed >= 0 ? remote_committed : reset.at(p->partition);
    std::lock_guard<std::mutex> pg(p->mu);
    PartitionEntry& P = local_->part(p->pidx);
    const bool resume = fresh && P.n_batches.load() != 0 && P.ring_bytes.load() == 0 &&
                        start >= P.log_start_offset.load() && start <= P.high_watermark.load();
    if (resume) {
      p->fetch_offset = P.high_watermark.load();  // a persistent (file://) replica resumes its log
    } else {
      if (P.n_batches.load() != 0 || P.high_watermark.load() != start) local_->reset_partition(p->pidx, start);
      if (cfg_.ring_bytes && P.ring_bytes.load() == 0) {
        local_->make_ring(p->pidx, std::min<uint64_t>(cfg_.ring_bytes, P.log_capacity));
        fresh_rings.push_back(p->pidx);
      }
      p->fetch_offset = start;
      p->released = 0;
    }
    p->start_offset = start;
    p->forwarded = remote_committed;
    // sets still in flight for the old position are dropped (the fetch thread reads gen first)
    p->ask_offset.store(p->fetch_offset.load(), std::memory_order_relaxed);
    p->gen.fetch_add(1, std::memory_order_release);
    if (!cfg_.group.empty() && (!fresh || (remote_committed >= 0 && local_->committed(group_, p->pidx) < remote_committed))) {
      // the local table is where the replica's consumers resume: the group's offset (a partition
      // handed over by a rebalance starts where its last owner committed, not where we left it)
      try {
        local_->commit(group_, -1, 0, 0, {CommitEntry{p->pidx, start, std::string()}});
      } catch (const KafkaError& e) {
        set_error(std::string("replicator: seeding the local committed offset failed: ") + e.what());
      }
    }
  }
  // the new rings' pages, faulted in in parallel before the first fetch writes into them
  std::vector<std::thread> th;
  for (uint32_t pidx : fresh_rings) th.emplace_back([this, pidx] { local_->populate_ring(pidx); });
  for (auto& t : th) t.join();
}

std::vector<int32_t> Replicator::join_group(wire::Client& c) {
  const std::string sub = wire::encode_subscription({cfg_.topic});
  std::string mid;
  {
    std::lock_guard<std::mutex> g(assign_mu_);
    mid = member_id_;
  }
  for (int attempt = 0; attempt < 8; ++attempt) {
    wire::JoinResult j = c.join_group(cfg_.group, cfg_.session_timeout_ms, mid, sub, cfg_.assignors,
                                      cfg_.rebalance_timeout_ms);
    if (j.error == wire::kMemberIdRequired) {  // JoinGroup v4+: join again with the id the coordinator chose
      mid = j.member_id;
      --attempt;
      continue;
    }
    if (j.error == wire::kUnknownMemberId) {
      mid.clear();
      continue;
    }
    if (j.error == wire::kRebalanceInProgress || wire::needs_metadata(j.error)) {
      sleep_ms(20 << std::min(attempt, 5));
      continue;
    }
    if (j.error != wire::kNone)
      throw wire::WireError(j.error, std::string(wire::error_name(j.error)) + ": JoinGroup '" + cfg_.group + "'");
    mid = j.member_id;
    std::map<std::string, std::string> plan;
    if (j.leader == j.member_id) {  // the leader assigns every member's subscription
      std::map<std::string, int32_t> counts;
      for (auto& [m, meta] : j.members)
        for (auto& topic : wire::decode_subscription(meta))
          if (!counts.count(topic)) {
            wire::TopicMeta tm = c.metadata(topic);
            counts[topic] = tm.error ? 0 : int32_t(tm.partitions.size());
          }
      auto plan_of = j.protocol == "roundrobin" ? wire::roundrobin_assign(j.members, counts)
                                                : wire::range_assign(j.members, counts);
      for (auto& [m, a] : plan_of) plan[m] = wire::encode_assignment(a);
    }
    auto [e, bytes] = c.sync_group(cfg_.group, j.generation, mid, plan);
    if (e == wire::kRebalanceInProgress || e == wire::kIllegalGeneration || wire::needs_metadata(e)) {
      sleep_ms(20 << std::min(attempt, 5));
      continue;
    }
    if (e == wire::kUnknownMemberId) {
      mid.clear();
      continue;
    }
    if (e != wire::kNone)
      throw wire::WireError(e, std::string(wire::error_name(e)) + ": SyncGroup '" + cfg_.group + "'");
    {
      std::lock_guard<std::mutex> g(assign_mu_);
      member_id_ = mid;
      generation_ = j.generation;
    }
    last_heartbeat_ms_ = now_ms();
    std::vector<int32_t> mine = wire::decode_assignment(bytes)[cfg_.topic];
    std::sort(mine.begin(), mine.end());
    return mine;
  }
  throw KafkaError("replicator: group '" + cfg_.group + "' did not settle (JoinGroup/SyncGroup kept rebalancing)");
}

// A new assignment, in process: revoked partitions stop (fetching, forwarding) at once, newly
// assigned ones start at the group's committed offset; consumers of the local replica learn both
// from assignment_epoch().  Runs on the commit thread under commit_mu_.
void Replicator::apply_assignment(wire::Client& c, const std::vector<int32_t>& mine) {
  const std::set<int32_t> now(mine.begin(), mine.end());
  std::vector<Part*> added;
  bool revoked = false;
  {
    std::lock_guard<std::mutex> g(assign_mu_);
    for (auto& p : parts_) {
      const bool want = now.count(p->partition) > 0;
      if (p->owned.load() && !want) {
        p->owned = false;
        revoked = true;
      } else if (!p->owned.load() && want) {
        added.push_back(p.get());
      }
    }
    if (revoked) epoch_.fetch_add(1, std::memory_order_acq_rel);
  }
  start_parts(c, added, false);  // network: outside the lock
  std::lock_guard<std::mutex> g(assign_mu_);
  const uint64_t e = epoch_.load() + (added.empty() ? 0 : 1);
  for (Part* p : added) {
    p->since = e;
    p->owned = true;
  }
  assigned_ = mine;
  epoch_.store(e, std::memory_order_release);
}

void Replicator::heartbeat(wire::Client& c) {
  if (!cfg_.subscribe || now_ms() - last_heartbeat_ms_ < cfg_.heartbeat_interval_ms) return;
  last_heartbeat_ms_ = now_ms();
  const int16_t e = c.heartbeat(cfg_.group, generation(), member_id());
  if (e == wire::kRebalanceInProgress || e == wire::kIllegalGeneration || e == wire::kUnknownMemberId) {
    try {
      forward(c);  // the current generation may still commit what was consumed
    } catch (const KafkaError&) {
    }
    std::lock_guard<std::mutex> g(commit_mu_);  // forward() reads generation_ / member_id_
    if (e == wire::kUnknownMemberId) {
      std::lock_guard<std::mutex> a(assign_mu_);
      member_id_.clear();
    }
    const std::vector<int32_t> mine = join_group(c);
    rebalances_.fetch_add(1);
    apply_assignment(c, mine);
  } else if (e != wire::kNone) {
    throw wire::WireError(e, std::string(wire::error_name(e)) + ": Heartbeat");
  }
}

std::string Replicator::member_id() const {
  std::lock_guard<std::mutex> g(assign_mu_);
  return member_id_;
}

int32_t Replicator::generation() const {
  std::lock_guard<std::mutex> g(assign_mu_);
  return generation_;
}

std::vector<int32_t> Replicator::assignment() const {
  std::lock_guard<std::mutex> g(assign_mu_);
  return assigned_;
}

std::vector<std::pair<int32_t, uint64_t>> Replicator::assignment_epochs() const {
  std::lock_guard<std::mutex> g(assign_mu_);
  std::vector<std::pair<int32_t, uint64_t>> v;
  for (auto& p : parts_)
    if (p->owned.load()) v.emplace_back(p->partition, p->since.load());
  return v;
}

void Replicator::set_oauth_token(const std::string& token, const std::string& extensions) {
  if (!cfg_.security.oauth) throw std::invalid_argument("replicator: not configured for SASL/OAUTHBEARER");
  std::lock_guard<std::mutex> l(cfg_.security.oauth->m);
  cfg_.security.oauth->token = token;
  cfg_.security.oauth->extensions = extensions;
}

void Replicator::stop(bool flush) {
  if (!running_.load() && threads_.empty()) return;
  {
    std::lock_guard<std::mutex> l(sync_mu_);
    stop_ = true;
  }
  sync_cv_.notify_all();
  for (auto& t : threads_)
    if (t.joinable()) t.join();
  threads_.clear();
  running_ = false;
  if (flush && !cfg_.group.empty()) {
    commit_client_.reset();  // its connections may carry the stop flag: flush on fresh ones
    const int flush_timeout = std::min(cfg_.timeout_ms, 5000);  // close() must not hang on a dead cluster
    for (int attempt = 0; attempt < 3; ++attempt) {
      try {
        if (!commit_client_)
          commit_client_ = std::make_unique<wire::Client>(cfg_.bootstrap, cfg_.client_id + "-commit", flush_timeout, cfg_.security);
        forward(*commit_client_);
        const std::string mid = member_id();
        if (cfg_.subscribe && !mid.empty()) commit_client_->leave_group(cfg_.group, mid);
        break;
      } catch (const KafkaError& e) {
        set_error(std::string("replicator: final commit: ") + e.what());
        commit_client_.reset();
        sleep_ms(50 << attempt);
      }
    }
  }
}

int64_t Replicator::keep_offset(Part& p) {
  int64_t c = cfg_.group.empty() ? -1 : local_->committed(group_, p.pidx);
  return c < 0 ? p.start_offset : c;
}

// Write room for the next record set: a ring log reuses the bytes of committed batches, a linear
// log has its tail up to the capacity.
uint8_t* Replicator::room(Part& p, uint64_t* avail) {
  if (cfg_.ring_bytes) {
    // a compressed topic inflates: reserve room for what a full Fetch inflates to (<= ring / 4)
    const uint64_t want = std::min<uint64_t>(uint64_t(cfg_.partition_max_bytes) * p.ratio16.load() / 16,
                                             std::max<uint64_t>(cfg_.ring_bytes / 4, uint64_t(cfg_.partition_max_bytes)));
    return local_->ring_reserve(p.pidx, want, keep_offset(p), avail);
  }
  return local_->log_tail(p.pidx, avail);
}

bool Replicator::throttled(Part& p) {
  if (cfg_.ring_bytes) {  // a ring is full while the consumers hold it: flow control by itself
    uint64_t avail = 0;
    local_->ring_reserve(p.pidx, uint64_t(cfg_.partition_max_bytes), keep_offset(p), &avail);
    return avail < std::min<uint64_t>(uint64_t(cfg_.partition_max_bytes), 256u << 10);
  }
  const PartitionEntry& P = local_->part(p.pidx);
  const uint64_t end = P.log_end_pos.load(std::memory_order_acquire);
  if (end == 0) return false;
  int64_t c = cfg_.group.empty() ? -1 : local_->committed(group_, p.pidx);
  if (c < 0) c = p.start_offset;
  const uint64_t pos = local_->position_of(p.pidx, c);
  return end > pos && int64_t(end - pos) > cfg_.max_lag_bytes;
}

void Replicator::reset_offset(wire::Client& c, Part& p) {
  const bool latest = cfg_.auto_offset_reset == "latest" || cfg_.auto_offset_reset == "largest";
  auto r = c.list_offsets(cfg_.topic, {p.partition}, latest ? -1 : -2);
  {
    std::lock_guard<std::mutex> pg(p.mu);  // vs. the inflater storing a queued set
    p.fetch_offset = r.at(p.partition);
    p.ask_offset.store(p.fetch_offset.load(), std::memory_order_relaxed);
    p.gen.fetch_add(1, std::memory_order_release);  // queued sets of the old position are dropped
  }
  set_error("OffsetOutOfRangeError: " + cfg_.topic + "-" + std::to_string(p.partition) + " reset to offset " +
            std::to_string(p.fetch_offset.load()));
}

void Replicator::fetch_loop(std::vector<Part*> mine) {
  name_thread("tk-bridge-fetch");
  std::unique_ptr<wire::Client> c;
  std::map<Part*, uint64_t> failed;  // -> assignment epoch at the failure
  int backoff_ms = 0;
  // this thread's inflater: started once one of its partitions turns out compressed
  Inflater inf;
  std::thread inf_th;
  struct StopInflater {
    Inflater& inf;
    std::thread& th;
    ~StopInflater() {
      {
        std::lock_guard<std::mutex> g(inf.m);
        inf.stop = true;
      }
      inf.cv.notify_all();
      if (th.joinable()) th.join();
    }
  } stop_inflater{inf, inf_th};
  while (!stop_.load()) {
    // subscribe mode: a thread whose partitions are all assigned elsewhere holds no connection
    if (cfg_.subscribe && std::none_of(mine.begin(), mine.end(), [](Part* p) { return p->owned.load(); })) {
      c.reset();
      sleep_ms(5);
      continue;
    }
    try {
      if (!c) {
        c = std::make_unique<wire::Client>(cfg_.bootstrap, cfg_.client_id, cfg_.timeout_ms, cfg_.security);
        c->set_cancel(&stop_);
        c->metadata(cfg_.topic);
      }
      std::map<int32_t, std::vector<Part*>> by;
      bool unknown_leader = false;
      for (Part* p : mine) {
        if (!p->owned.load(std::memory_order_acquire)) continue;
        if (p->failed_since.load(std::memory_order_acquire) == p->since.load()) failed[p] = p->since.load();
        auto f = failed.find(p);
        if (f != failed.end()) {
          if (f->second == p->since.load()) continue;
          failed.erase(f);  // restarted by a rebalance since it failed
        }
        if (p->inflight.load(std::memory_order_acquire) >= max_inflight_) continue;  // its inflater is behind
        if (throttled(*p)) {
          p->throttled.fetch_add(1, std::memory_order_relaxed);
          continue;
        }
        const int32_t node = c->leader(cfg_.topic, p->partition);
        if (node < 0) unknown_leader = true; else by[node].push_back(p);
      }
      if (unknown_leader) c->metadata(cfg_.topic);
      if (by.empty()) {
        if (inf_th.joinable() && !unknown_leader) {  // woken early when an inflater finishes a set
          std::unique_lock<std::mutex> lk(inf.m);
          inf.done_cv.wait_for(lk, std::chrono::milliseconds(1));
        } else {
          sleep_ms(unknown_leader ? 50 : 1);
        }
        continue;
      }
      const int32_t wait = by.size() > 1 ? std::min<int32_t>(cfg_.max_wait_ms, 10) : cfg_.max_wait_ms;
      bool refresh = false;
      for (auto& [node, ps] : by) {
        std::vector<wire::FetchPartReq> req;
        std::map<int32_t, Part*> lookup;
        std::map<Part*, uint64_t> since;  // a partition restarted while its fetch was in flight drops the data
        std::map<Part*, uint64_t> gens;   // ... and so does one whose position jumped (Part::gen)
        std::map<Part*, int64_t> asked;   // the offset each partition was asked from
        for (Part* p : ps) {
          uint64_t avail = 0;
          room(*p, &avail);
          if (avail < 4096 && cfg_.ring_bytes) continue;  // waits for the consumers to commit
          if (avail < 4096) {
            if (!failed.count(p))
              set_error("replicator: local log of " + cfg_.topic + "-" + std::to_string(p->partition) +
                        " is full (raise log_capacity)");
            failed[p] = p->since.load();
            continue;
          }
          // compressed data inflates by ratio16 / 16 in the log: ask for what will fit
          const uint64_t fit = std::max<uint64_t>(avail * 16 / p->ratio16.load(), 4096);
          // the generation first: offsets read after it are at least as new (stored before its bump)
          const uint64_t g = p->gen.load(std::memory_order_acquire);
          const bool piped = p->inflight.load(std::memory_order_acquire) > 0;
          const int64_t from = piped ? p->ask_offset.load() : p->fetch_offset.load();
          req.push_back({p->partition, from,
                         int32_t(std::min<uint64_t>({uint64_t(cfg_.partition_max_bytes), piped ? fit : avail, fit}))});
          lookup[p->partition] = p;
          since[p] = p->since.load();
          gens[p] = g;
          asked[p] = from;
        }
        if (req.empty()) continue;
        wire::Conn& k = c->conn(node);
        const int16_t fv = k.version(wire::kFetch);
        k.send(wire::kFetch, fv, c->client_id(),
               wire::fetch_request(fv, cfg_.topic, req, wait, cfg_.min_bytes, cfg_.max_bytes));
        const auto t_sent = std::chrono::steady_clock::now();
        k.begin_response(cfg_.timeout_ms + wait);
        fetch_wait_ns_.fetch_add(uint64_t(std::chrono::duration_cast<std::chrono::nanoseconds>(
                                              std::chrono::steady_clock::now() - t_sent).count()),
                                 std::memory_order_relaxed);
        wire::fetch_response_header(k, fv);
        std::vector<Part*> out_of_range;  // reset once the response is read: ListOffsets reuses the connection
        const int32_t nt = k.r32();
        for (int32_t i = 0; i < nt; ++i) {
          k.rstr();
          const int32_t np = k.r32();
          for (int32_t j = 0; j < np; ++j) {
            const wire::FetchPartHeader ph = wire::fetch_partition_header(k, fv);
            const int32_t pid = ph.partition, len = ph.records_len;
            const int16_t err = ph.error;
            auto it = lookup.find(pid);
            Part* p = it == lookup.end() ? nullptr : it->second;
            if (!p || err != wire::kNone) {
              if (len > 0) k.skip(size_t(len));
              if (!p) continue;
              if (err == wire::kOffsetOutOfRange) {
                out_of_range.push_back(p);
              } else {
                set_error(std::string(wire::error_name(err)) + ": fetch " + cfg_.topic + "-" + std::to_string(pid));
                if (wire::needs_metadata(err)) refresh = true;
              }
              continue;
            }
            std::unique_lock<std::mutex> pg(p->mu);
            if (!p->owned.load() || p->since.load() != since[p] || p->gen.load() != gens[p]) {
              pg.unlock();  // revoked / restarted / repositioned meanwhile
              if (len > 0) k.skip(size_t(len));
              continue;
            }
            p->remote_hw.store(ph.high_watermark, std::memory_order_relaxed);
            p->fetches.fetch_add(1, std::memory_order_relaxed);
            if (len <= 0) continue;
            if (p->ratio16.load(std::memory_order_relaxed) > 16 || p->inflight.load(std::memory_order_acquire) > 0) {
              // a compressed partition: receive into a buffer, hand it to this thread's inflater,
              // and ask for the next record set while it inflates.  While any set is queued every
              // later one queues behind it (even if the last ratio fell to 1): the inflater stores
              // them in the order they were asked for
              pg.unlock();
              std::vector<uint8_t> buf;
              {
                std::lock_guard<std::mutex> g(inf.m);
                if (!inf.spare.empty()) {
                  buf = std::move(inf.spare.back());
                  inf.spare.pop_back();
                }
              }
              buf.resize(size_t(len));
              const auto t_recv = std::chrono::steady_clock::now();
              k.read(buf.data(), size_t(len));
              p->wire_bytes.fetch_add(uint64_t(len), std::memory_order_relaxed);
              p->recv_ns.fetch_add(uint64_t(std::chrono::duration_cast<std::chrono::nanoseconds>(
                                                std::chrono::steady_clock::now() - t_recv).count()),
                                   std::memory_order_relaxed);
              // the next offset to ask for: past the last whole batch received
              const int64_t from = asked[p];
              int64_t next = from;
              for (size_t r = 0; size_t(len) - r >= 61;) {
                const uint8_t* b = buf.data() + r;
                const uint64_t total = uint64_t((uint32_t(b[8]) << 24) | (uint32_t(b[9]) << 16) |
                                                (uint32_t(b[10]) << 8) | uint32_t(b[11])) + 12;
                if (total < 61 || total > size_t(len) - r) break;
                int64_t base = 0;
                for (int q = 0; q < 8; ++q) base = (base << 8) | int64_t(b[q]);
                const int32_t lod = int32_t((uint32_t(b[23]) << 24) | (uint32_t(b[24]) << 16) |
                                            (uint32_t(b[25]) << 8) | uint32_t(b[26]));
                next = std::max(next, base + int64_t(lod) + 1);
                r += size_t(total);
              }
              if (next <= from) {  // no whole batch: ask again from the same offset
                std::lock_guard<std::mutex> g(inf.m);
                inf.spare.push_back(std::move(buf));
                continue;
              }
              p->ask_offset.store(next, std::memory_order_release);
              p->inflight.fetch_add(1, std::memory_order_acq_rel);
              if (!inf_th.joinable()) {
                inf_th = std::thread([this, &inf] { inflate_loop(&inf); });
                n_inflaters_.fetch_add(1, std::memory_order_relaxed);
              }
              {
                std::lock_guard<std::mutex> g(inf.m);
                inf.q.push_back(Pending{p, since[p], gens[p], from, std::move(buf)});
              }
              inf.cv.notify_one();
              continue;
            }
            if (asked[p] > p->fetch_offset.load()) {  // would leave a gap in the log: ask again
              pg.unlock();
              k.skip(size_t(len));
              resync(*p, "fetch");
              continue;
            }
            uint64_t avail = 0;
            uint8_t* tail = room(*p, &avail);
            if (uint64_t(len) > avail) {  // an oversized first batch (KIP-74) the log cannot hold now
              pg.unlock();
              k.skip(size_t(len));
              if (cfg_.ring_bytes && uint64_t(len) < cfg_.ring_bytes / 2) continue;  // refetched when room frees
              set_error("replicator: local log of " + cfg_.topic + "-" + std::to_string(pid) + " is full");
              failed[p] = since[p];
              continue;
            }
            const auto t_recv = std::chrono::steady_clock::now();
            k.read(tail, size_t(len));  // the record set lands in the log tail: no second copy
            const auto t_ingest = std::chrono::steady_clock::now();
            p->wire_bytes.fetch_add(uint64_t(len), std::memory_order_relaxed);
            p->recv_ns.fetch_add(uint64_t(std::chrono::duration_cast<std::chrono::nanoseconds>(t_ingest - t_recv).count()),
                                 std::memory_order_relaxed);
            try {
              const Broker::Ingested in = local_->ingest(p->pidx, uint64_t(len), p->fetch_offset.load(), false,
                                                         cfg_.ring_bytes ? avail : 0);
              p->ingest_ns.fetch_add(uint64_t(std::chrono::duration_cast<std::chrono::nanoseconds>(
                                                  std::chrono::steady_clock::now() - t_ingest).count()),
                                     std::memory_order_relaxed);
              p->inflate_ns.fetch_add(in.inflate_ns, std::memory_order_relaxed);
              p->inflated.fetch_add(in.inflated, std::memory_order_relaxed);
              p->inflated_bytes.fetch_add(in.inflated_bytes, std::memory_order_relaxed);
              if (in.inflated_from)
                p->ratio16.store(uint32_t(std::clamp<uint64_t>(in.inflated_bytes * 16 / in.inflated_from, 16, 16 * 64)),
                                 std::memory_order_relaxed);
              if (in.next_offset > p->fetch_offset.load()) p->fetch_offset.store(in.next_offset);
              if (in.full && in.kept == 0) grow_reserve(*p);
              p->bytes.fetch_add(in.kept_bytes, std::memory_order_relaxed);
              p->batches.fetch_add(in.kept, std::memory_order_relaxed);
              p->control.fetch_add(in.control, std::memory_order_relaxed);
            } catch (const KafkaError& e) {  // compressed / corrupt / old-format data: this partition stops
              set_error(std::string("replicator: ") + cfg_.topic + "-" + std::to_string(pid) + ": " + e.what());
              failed[p] = since[p];
            }
          }
        }
        k.finish();
        for (Part* p : out_of_range) reset_offset(*c, *p);
      }
      if (refresh) {
        c->metadata(cfg_.topic);
        sleep_ms(10);
      }
      backoff_ms = 0;
    } catch (const std::exception& e) {
      if (stop_.load()) break;  // a wait cancelled by stop(): not an error
      set_error(std::string("replicator: ") + e.what());
      c.reset();  // reconnect + fresh metadata
      backoff_ms = std::min(1000, std::max(10, backoff_ms * 2));
      for (int s = 0; s < backoff_ms && !stop_.load(); s += 10) sleep_ms(10);
    }
  }
}

void Replicator::inflate_loop(Inflater* inf) {
  name_thread("tk-inflate");
  std::unique_lock<std::mutex> lk(inf->m);
  while (true) {
    inf->cv.wait(lk, [&] { return inf->stop || !inf->q.empty(); });
    if (inf->stop) break;  // what is still queued is refetched by the next replicator start
    Pending pd = std::move(inf->q.front());
    inf->q.pop_front();
    lk.unlock();
    inflate_one(pd);
    pd.p->inflight.fetch_sub(1, std::memory_order_acq_rel);
    lk.lock();
    pd.data.clear();
    if (inf->spare.size() < size_t(max_inflight_)) inf->spare.push_back(std::move(pd.data));
    inf->done_cv.notify_all();
  }
  inf->q.clear();
}

// Stores one received record set of a compressed partition: inflated into the log as room allows
// (a full ring waits for the consumers' commits), in order, never dropped -- the fetch thread has
// already asked for what follows it.
void Replicator::inflate_one(Pending& pd) {
  Part* p = pd.p;
  size_t off = 0;
  // fault injection for tests: an inflater this much slower keeps sets queued behind each other
  const char* delay = std::getenv("TORCHKAFKA_TEST_INFLATE_DELAY_US");
  const int delay_us = delay ? std::atoi(delay) : 0;
  if (delay_us > 0) std::this_thread::sleep_for(std::chrono::microseconds(delay_us));
  while (!stop_.load() && off < pd.data.size()) {
    std::unique_lock<std::mutex> pg(p->mu);
    // revoked / restarted / repositioned: dropped; so are the sets queued behind one that failed
    // (storing them would publish the batches after the failure with the failed ones missing)
    if (!p->owned.load() || p->since.load() != pd.since || p->gen.load() != pd.gen ||
        p->failed_since.load(std::memory_order_acquire) == pd.since)
      return;
    if (off == 0 && pd.asked > p->fetch_offset.load()) {  // does not follow the log's end: a gap
      pg.unlock();
      resync(*p, "inflater");
      return;
    }
    uint64_t avail = 0;
    room(*p, &avail);
    if (avail < 4096) {
      pg.unlock();
      if (!cfg_.ring_bytes) {
        set_error("replicator: local log of " + cfg_.topic + "-" + std::to_string(p->partition) +
                  " is full (raise log_capacity)");
        p->failed_since.store(pd.since, std::memory_order_release);
        return;
      }
      sleep_ms(1);  // a ring frees room as the consumers commit
      continue;
    }
    const auto t0 = std::chrono::steady_clock::now();
    Broker::Ingested in;
    try {
      in = local_->ingest(p->pidx, uint64_t(pd.data.size() - off), p->fetch_offset.load(), false,
                          cfg_.ring_bytes ? avail : 0, pd.data.data() + off);
    } catch (const KafkaError& e) {
      set_error(std::string("replicator: ") + cfg_.topic + "-" + std::to_string(p->partition) + ": " + e.what());
      p->failed_since.store(pd.since, std::memory_order_release);
      return;
    }
    p->ingest_ns.fetch_add(uint64_t(std::chrono::duration_cast<std::chrono::nanoseconds>(
                                        std::chrono::steady_clock::now() - t0).count()),
                           std::memory_order_relaxed);
    p->inflate_ns.fetch_add(in.inflate_ns, std::memory_order_relaxed);
    p->inflated.fetch_add(in.inflated, std::memory_order_relaxed);
    p->inflated_bytes.fetch_add(in.inflated_bytes, std::memory_order_relaxed);
    if (in.inflated_from)
      p->ratio16.store(uint32_t(std::clamp<uint64_t>(in.inflated_bytes * 16 / in.inflated_from, 16, 16 * 64)),
                       std::memory_order_relaxed);
    if (in.next_offset > p->fetch_offset.load()) p->fetch_offset.store(in.next_offset);
    p->bytes.fetch_add(in.kept_bytes, std::memory_order_relaxed);
    p->batches.fetch_add(in.kept, std::memory_order_relaxed);
    p->control.fetch_add(in.control, std::memory_order_relaxed);
    off += size_t(in.consumed);
    if (!in.full) return;  // stored (a trailing partial batch is asked for again by the fetch thread)
    if (in.kept == 0) grow_reserve(*p);
    pg.unlock();
    sleep_ms(1);
  }
}

// A ring replica reserves room for what a set inflates to by the ratio learnt from the last
// inflated batches; before any (or when a batch inflates more than those did) the first batch may
// not fit the reservation at all, and nothing would ever be stored: double the ratio assumed.
void Replicator::grow_reserve(Part& p) {
  if (!cfg_.ring_bytes) return;  // a linear log offers its whole tail
  const uint32_t r = p.ratio16.load(std::memory_order_relaxed);
  p.ratio16.store(std::min<uint32_t>(r * 2, 16 * 64), std::memory_order_relaxed);
}

// A record set that does not start where the partition's log ends would leave a silent gap: it
// is dropped, and so is everything asked for after it; the fetch thread asks again from the end.
void Replicator::resync(Part& p, const char* where) {
  std::lock_guard<std::mutex> pg(p.mu);
  out_of_order_.fetch_add(1, std::memory_order_relaxed);
  p.ask_offset.store(p.fetch_offset.load(), std::memory_order_relaxed);
  p.gen.fetch_add(1, std::memory_order_release);
  set_error(std::string("replicator: ") + where + ": a record set of " + cfg_.topic + "-" + std::to_string(p.partition) +
            " did not follow the log end (offset " + std::to_string(p.fetch_offset.load()) + "): refetched");
}

int Replicator::forward(wire::Client& c) {
  std::lock_guard<std::mutex> g(commit_mu_);
  std::map<int32_t, int64_t> offs;
  std::map<int32_t, Part*> by;
  for (auto& p : parts_) {
    if (!p->owned.load()) continue;  // revoked: another member's commits now
    const int64_t off = local_->committed(group_, p->pidx);
    // subscribe mode: an offset below where this ownership started (the group's committed offset
    // then) comes from a batch consumed in an earlier ownership -- never move the group back
    if (cfg_.subscribe && off < p->start_offset) continue;
    if (off >= 0 && off != p->forwarded.load()) {
      offs[p->partition] = off;
      by[p->partition] = p.get();
    }
  }
  if (offs.empty()) return 0;
  int n = 0;
  std::string mid;
  int32_t gen;
  {
    std::lock_guard<std::mutex> a(assign_mu_);
    mid = member_id_;
    gen = generation_;
  }
  auto errs = c.offset_commit(cfg_.group, cfg_.topic, offs, "", gen, mid);
  for (auto& [pid, e] : errs) {
    auto it = by.find(pid);
    if (it == by.end()) continue;
    if (e == wire::kNone) {
      it->second->forwarded.store(offs[pid]);
      ++n;
    } else {
      set_error(std::string("CommitFailedError: ") + wire::error_name(e) + " committing " + cfg_.topic + "-" +
                std::to_string(pid));
    }
  }
  return n;
}

int Replicator::flush_commits() {
  if (cfg_.group.empty()) return 0;
  wire::Client c(cfg_.bootstrap, cfg_.client_id + "-flush", cfg_.timeout_ms, cfg_.security);
  return forward(c);
}

void Replicator::commit_loop() {
  name_thread("tk-bridge-cmt");
  int backoff_ms = cfg_.commit_interval_ms;
  while (!stop_.load()) {
    uint64_t serving;
    {
      // every commit_interval_ms, or at once when commit_sync() asks
      std::unique_lock<std::mutex> l(sync_mu_);
      sync_cv_.wait_for(l, std::chrono::milliseconds(backoff_ms),
                        [&] { return stop_.load() || sync_req_ > sync_done_; });
      serving = sync_req_;
    }
    if (stop_.load()) break;
    bool ok = false;
    try {
      if (!commit_client_) {
        commit_client_ = std::make_unique<wire::Client>(cfg_.bootstrap, cfg_.client_id + "-commit", cfg_.timeout_ms, cfg_.security);
        commit_client_->set_cancel(&stop_);
      }
      const int64_t errs0 = errors_.load();
      const int64_t t0 = now_ns();
      const int n = forward(*commit_client_);
      if (n > 0) {
        std::lock_guard<std::mutex> g(stats_mu_);
        if (forward_ns_.size() < (1u << 16)) forward_ns_.push_back(now_ns() - t0);
      }
      ok = errors_.load() == errs0;
      heartbeat(*commit_client_);
      backoff_ms = cfg_.commit_interval_ms;
    } catch (const std::exception& e) {
      if (stop_.load()) break;
      set_error(std::string("replicator: commit: ") + e.what());
      commit_client_.reset();
      backoff_ms = std::min(1000, std::max(10, backoff_ms * 2));
    }
    {
      std::lock_guard<std::mutex> l(sync_mu_);
      if (serving > sync_done_) {
        sync_done_ = serving;
        sync_ok_ = ok;
      }
    }
    sync_cv_.notify_all();
  }
  sync_cv_.notify_all();
}

bool Replicator::commit_sync(int timeout_ms) {
  if (cfg_.group.empty() || !running_.load()) return false;
  std::unique_lock<std::mutex> l(sync_mu_);
  const uint64_t want = ++sync_req_;
  sync_cv_.notify_all();
  const bool done = sync_cv_.wait_for(l, std::chrono::milliseconds(timeout_ms),
                                      [&] { return sync_done_ >= want || stop_.load(); });
  return done && sync_done_ >= want && sync_ok_;
}

std::vector<int64_t> Replicator::take_forward_ns() {
  std::lock_guard<std::mutex> g(stats_mu_);
  std::vector<int64_t> v;
  v.swap(forward_ns_);
  return v;
}

// Committed log bytes are never read again (the bridge's broker has one consuming group): move
// the log start up to the committed offset, then punch the bytes below it out of the log file, so
// host memory holds the uncommitted window (max_lag_bytes) plus up to release_bytes + release_step
// of consumed log per partition, not the whole stream.  Bytes a device loader still holds pinned
// are never punched (pin_floor).  Punching a range that was pinned once (even after
// hipHostUnregister) stalls the GPU of the loader's process for ~20-30 ms per punch, about
// independent of its size (tools/probes/punch_probe.py, profiles/r02_s5_bridge/punch_probe.log),
// so releases come in rare bursts: once some partition has release_step (1 GiB) releasable bytes,
// every partition releases what it can in one punch each, back to back.
void Replicator::release_loop() {
  name_thread("tk-bridge-rel");
  constexpr uint64_t kAlign = 2u << 20;
  while (!stop_.load()) {
    sleep_ms(10);
    std::vector<std::pair<Part*, uint64_t>> todo;
    uint64_t most = 0;
    for (auto& p : parts_) {
      if (!p->owned.load()) continue;
      const int64_t c = local_->committed(group_, p->pidx);
      if (c < 0) continue;
      uint64_t pos = local_->position_of(p->pidx, c);
      const PartitionEntry& P = local_->part(p->pidx);
      if (P.pinned.load(std::memory_order_acquire)) pos = std::min<uint64_t>(pos, P.pin_floor.load());
      if (pos <= cfg_.release_bytes) continue;
      const uint64_t target = (pos - cfg_.release_bytes) / kAlign * kAlign;
      const uint64_t from = p->released.load();
      if (target <= from) continue;
      todo.emplace_back(p.get(), target);
      most = std::max(most, target - from);
    }
    if (most < cfg_.release_step) continue;
    for (auto& [p, target] : todo) {
      const uint64_t from = p->released.load();
      if (target - from < std::min<uint64_t>(64u << 20, cfg_.release_step)) continue;
      local_->delete_records(p->pidx, local_->committed(group_, p->pidx));  // readers below see OffsetOutOfRange
      local_->release_log(p->pidx, from, target);
      p->released.store(target);
    }
  }
}

std::vector<ReplicaPartStats> Replicator::stats() {
  std::vector<ReplicaPartStats> v;
  for (auto& p : parts_)
    v.push_back(ReplicaPartStats{p->partition, p->pidx, p->start_offset, p->fetch_offset.load(), p->remote_hw.load(),
                                 p->forwarded.load(), p->bytes.load(), p->batches.load(), p->control.load(),
                                 p->fetches.load(), p->throttled.load(), p->released.load(), p->owned.load(),
                                 p->wire_bytes.load(), p->recv_ns.load(), p->ingest_ns.load(), p->inflate_ns.load(),
                                 p->inflated.load(), p->inflated_bytes.load()});
  return v;
}

bool Replicator::wait_caught_up(int timeout_ms) {
  std::vector<int32_t> ids;
  for (auto& p : parts_)
    if (p->owned.load()) ids.push_back(p->partition);
  if (ids.empty()) return true;
  wire::Client c(cfg_.bootstrap, cfg_.client_id + "-lag", cfg_.timeout_ms, cfg_.security);
  auto hw = c.list_offsets(cfg_.topic, ids, -1);
  const auto deadline = std::chrono::steady_clock::now() + std::chrono::milliseconds(timeout_ms);
  while (std::chrono::steady_clock::now() < deadline) {
    bool all = true;
    for (auto& p : parts_)
      if (p->owned.load() && p->fetch_offset.load() < hw[p->partition]) all = false;
    if (all) return true;
    sleep_ms(2);
  }
  return false;
}

}  // namespace tk
