// Broker consumer groups (broker.h): membership with session timeouts and generations, the
// range assignment of a group's subscribed partitions over its members, committed offsets with
// metadata, and the commit-failure injection the tests use (the coordinator
// side kafka-python's KafkaConsumer talks to, /root/reference/src/kafka_dataset.py:124-143).
// All state lives in the broker's shared metadata file under its robust mutex.  Split from
// broker.cpp.
#include "broker.h"

#include <signal.h>

#include <algorithm>
#include <cerrno>

namespace tk {

namespace {

bool pid_alive(int32_t pid) {  // a member process that no longer exists
  if (pid <= 0) return false;
  if (kill(pid, 0) == 0) return true;
  return errno == EPERM;
}

}  // namespace

// ------------------------------------------------------------ groups
GroupEntry& Broker::group(uint32_t g) const {
  if (g >= meta_->n_groups.load(std::memory_order_acquire)) throw std::out_of_range("bad group index");
  return groups_[g];
}
int16_t* Broker::owners(uint32_t g) const { return owners_ + size_t(g) * meta_->max_partitions; }
OffsetEntry& Broker::offset_entry(uint32_t g, uint32_t pidx) const {
  if (pidx >= meta_->max_partitions) throw std::out_of_range("bad partition index");
  return offsets_[size_t(g) * meta_->max_partitions + pidx];
}

uint32_t Broker::group_index(const std::string& name, bool create) {
  if (name.empty() || name.size() >= kNameLen) throw std::invalid_argument("bad group id");
  auto scan = [&]() -> int64_t {
    const uint32_t n = meta_->n_groups.load(std::memory_order_acquire);
    for (uint32_t i = 0; i < n; ++i)
      if (name == groups_[i].name) return i;
    return -1;
  };
  int64_t g = scan();
  if (g >= 0 || !create) {
    if (g < 0) throw KafkaError("unknown group '" + name + "'");
    return uint32_t(g);
  }
  RobustLock l(&meta_->lock);
  g = scan();
  if (g >= 0) return uint32_t(g);
  const uint32_t n = meta_->n_groups.load();
  if (n >= meta_->max_groups) throw KafkaError("broker group table full");
  GroupEntry& G = groups_[n];
  std::memset(G.name, 0, kNameLen);
  std::memcpy(G.name, name.data(), name.size());
  G.generation.store(0);
  G.state.store(kGroupEmpty);
  G.next_member_id = 0;
  G.awaiting.store(0);
  for (auto& m : G.members) m.active.store(0);
  meta_->n_groups.store(n + 1, std::memory_order_release);
  return n;
}

std::string Broker::group_name(uint32_t g) const { return group(g).name; }

uint64_t Broker::member_id(uint32_t g, int slot) const { return group(g).members[slot].member_id; }

bool Broker::expire_members_locked(GroupEntry& G, int64_t now) {
  bool changed = false;
  for (auto& M : G.members) {
    if (!M.active.load()) continue;
    const bool dead = !pid_alive(M.pid);
    const bool stale = now - M.last_poll_ns.load() > M.max_poll_interval_ns;
    if (dead || stale) {
      M.active.store(0);
      changed = true;
    }
  }
  G.last_expiry_check_ns.store(now);
  return changed;
}

void Broker::assign_locked(GroupEntry& G, uint32_t g) {
  // Range assignor (kafka-python's default): per topic, members subscribed to
  // it sorted by member id; partition count split into contiguous ranges.
  int16_t* own = owners(g);
  std::fill(own, own + meta_->max_partitions, int16_t(-1));
  const uint32_t nt = meta_->n_topics.load();
  for (uint32_t t = 0; t < nt; ++t) {
    std::vector<std::pair<uint64_t, int>> subs;
    for (int s = 0; s < kMaxMembers; ++s) {
      const MemberEntry& M = G.members[s];
      if (!M.active.load()) continue;
      for (uint32_t i = 0; i < M.n_topics; ++i)
        if (M.topics[i] == t) { subs.emplace_back(M.member_id, s); break; }
    }
    if (subs.empty()) continue;
    std::sort(subs.begin(), subs.end());
    const uint32_t np = topics_[t].n_partitions, first = topics_[t].first_pidx;
    const uint32_t m = uint32_t(subs.size()), per = np / m, extra = np % m;
    uint32_t p = 0;
    for (uint32_t k = 0; k < m; ++k) {
      const uint32_t cnt = per + (k < extra ? 1 : 0);
      for (uint32_t c = 0; c < cnt; ++c) own[first + p++] = int16_t(subs[k].second);
    }
  }
}

void Broker::rebalance_locked(GroupEntry& G, uint32_t g, int64_t now, bool immediate) {
  int active = 0;
  for (auto& M : G.members) active += M.active.load() ? 1 : 0;
  if (active == 0) {
    int16_t* own = owners(g);
    std::fill(own, own + meta_->max_partitions, int16_t(-1));
    G.generation.fetch_add(1);
    G.state.store(kGroupEmpty);
    G.awaiting.store(0);
    return;
  }
  const uint32_t st = G.state.load();
  if (st == kGroupEmpty && !immediate && meta_->group_initial_rebalance_delay_ms > 0) {
    G.prepare_deadline_ns = now + int64_t(meta_->group_initial_rebalance_delay_ms) * 1000000LL;
    G.state.store(kGroupPreparing);
    return;
  }
  if (st == kGroupPreparing && !immediate && now < G.prepare_deadline_ns) return;
  assign_locked(G, g);
  G.awaiting.store(0);
  G.generation.fetch_add(1);
  G.state.store(kGroupStable, std::memory_order_release);
}

void Broker::membership_changed_locked(GroupEntry& G, uint32_t g, int64_t now) {
  int active = 0;
  int64_t timeout = 0;
  for (auto& M : G.members)
    if (M.active.load()) {
      ++active;
      timeout = std::max(timeout, M.max_poll_interval_ns);
    }
  const uint32_t st = G.state.load();
  if (active == 0 || st == kGroupEmpty || (st == kGroupPreparing && !G.awaiting.load())) {
    // nobody left, or a group forming: the initial rebalance delay lets its first members join
    // one round together (group.initial.rebalance.delay.ms)
    rebalance_locked(G, g, now, active == 0);
    return;
  }
  if (st == kGroupStable) {
    // Kafka's PreparingRebalance: the members keep their partitions (and may commit them) until
    // they rejoin; the rebalance timeout is the members' largest max.poll.interval.ms
    for (auto& M : G.members) M.rejoined.store(0);
    G.prepare_deadline_ns = now + timeout;
    G.awaiting.store(1);
    G.state.store(kGroupPreparing, std::memory_order_release);
  }
  try_complete_round_locked(G, g, now);
}

void Broker::try_complete_round_locked(GroupEntry& G, uint32_t g, int64_t now) {
  if (G.state.load() != kGroupPreparing || !G.awaiting.load()) return;
  bool all = true;
  for (auto& M : G.members)
    if (M.active.load() && !M.rejoined.load()) all = false;
  if (!all) {
    if (now < G.prepare_deadline_ns) return;
    for (auto& M : G.members)  // the absentees are dropped from the group, as Kafka does
      if (M.active.load() && !M.rejoined.load()) M.active.store(0);
  }
  rebalance_locked(G, g, now, true);
}

void Broker::rejoin_group(uint32_t g, int slot, uint64_t mid) {
  GroupEntry& G = group(g);
  RobustLock l(&meta_->lock);
  MemberEntry& M = G.members[slot];
  if (!M.active.load() || M.member_id != mid) return;
  const int64_t now = now_ns();
  M.last_poll_ns.store(now);
  if (G.state.load() != kGroupPreparing || !G.awaiting.load()) return;
  M.rejoined.store(1);
  try_complete_round_locked(G, g, now);
}

int Broker::join_group(uint32_t g, const std::vector<uint32_t>& topic_indices, int64_t session_timeout_ms,
                       int64_t max_poll_interval_ms) {
  if (topic_indices.size() > size_t(kMaxSubscribedTopics)) throw std::invalid_argument("too many topics");
  GroupEntry& G = group(g);
  RobustLock l(&meta_->lock);
  const int64_t now = now_ns();
  expire_members_locked(G, now);
  int slot = -1;
  for (int s = 0; s < kMaxMembers; ++s)
    if (!G.members[s].active.load()) { slot = s; break; }
  if (slot < 0) throw KafkaError("consumer group '" + std::string(G.name) + "' is full");
  MemberEntry& M = G.members[slot];
  M.pid = int32_t(getpid());
  M.last_poll_ns.store(now);
  M.session_timeout_ns = session_timeout_ms * 1000000LL;
  M.max_poll_interval_ns = max_poll_interval_ms * 1000000LL;
  M.member_id = ++G.next_member_id;
  M.n_topics = uint32_t(topic_indices.size());
  for (size_t i = 0; i < topic_indices.size(); ++i) M.topics[i] = topic_indices[i];
  M.active.store(1, std::memory_order_release);
  membership_changed_locked(G, g, now);
  M.rejoined.store(1);  // a new member is part of the round its join started
  try_complete_round_locked(G, g, now);
  return slot;
}

void Broker::leave_group(uint32_t g, int slot, uint64_t mid) {
  GroupEntry& G = group(g);
  RobustLock l(&meta_->lock);
  MemberEntry& M = G.members[slot];
  if (!M.active.load() || M.member_id != mid) return;
  M.active.store(0);
  membership_changed_locked(G, g, now_ns());
}

GroupView Broker::poll_group(uint32_t g, int slot, uint64_t mid) {
  GroupEntry& G = group(g);
  GroupView v{};
  MemberEntry& M = G.members[slot];
  const int64_t now = now_ns();
  if (M.active.load() && M.member_id == mid) M.last_poll_ns.store(now);
  RobustLock l(&meta_->lock);
  if (now - G.last_expiry_check_ns.load() > 50000000LL && expire_members_locked(G, now))
    membership_changed_locked(G, g, now);
  if (G.state.load() == kGroupPreparing && now >= G.prepare_deadline_ns) {
    if (G.awaiting.load())
      try_complete_round_locked(G, g, now);
    else
      rebalance_locked(G, g, now, false);
  }
  v.member_active = M.active.load() && M.member_id == mid;
  v.generation = G.generation.load();
  v.state = G.state.load();
  if (v.member_active && v.state == kGroupStable) {
    const int16_t* own = owners(g);
    const uint32_t np = meta_->n_partitions.load();
    for (uint32_t p = 0; p < np; ++p)
      if (own[p] == slot) v.assignment.push_back(p);
  }
  return v;
}

void Broker::commit(uint32_t g, int slot, uint64_t mid, uint32_t generation, const std::vector<CommitEntry>& entries) {
  GroupEntry& G = group(g);
  int32_t inj = G.inject_commit_failures.load();
  while (inj > 0) {
    if (G.inject_commit_failures.compare_exchange_weak(inj, inj - 1))
      throw CommitFailed("CommitFailedError: injected commit failure");
  }
  if (slot >= 0) {
    RobustLock l(&meta_->lock);
    MemberEntry& M = G.members[slot];
    if (!M.active.load() || M.member_id != mid)
      throw CommitFailed("CommitFailedError: member is no longer part of the group (rebalanced)");
    const int64_t now = now_ns();
    if (now - M.last_poll_ns.load() > M.max_poll_interval_ns) {
      M.active.store(0);
      membership_changed_locked(G, g, now);
      throw CommitFailed("CommitFailedError: time between polls exceeded max_poll_interval_ms");
    }
    // Kafka accepts a current-generation commit during PreparingRebalance (a member commits what
    // it finished before it rejoins -- kafka-python's _on_join_prepare), not once reassigned
    const uint32_t st = G.state.load();
    const bool open = st == kGroupStable || (st == kGroupPreparing && G.awaiting.load());
    if (!open || G.generation.load() != generation)
      throw CommitFailed("CommitFailedError: the group has rebalanced (generation " +
                         std::to_string(G.generation.load()) + ", member had " + std::to_string(generation) + ")");
  } else if (G.state.load(std::memory_order_acquire) != kGroupEmpty) {
    throw CommitFailed("CommitFailedError: group has active members; commit from a non-member rejected");
  }
  const int64_t wall = wall_ms();
  for (const auto& e : entries) {
    OffsetEntry& O = offset_entry(g, e.pidx);
    const size_t ml = std::min(e.metadata.size(), sizeof(O.metadata));
    std::memcpy(O.metadata, e.metadata.data(), ml);
    O.meta_len = int32_t(ml);
    O.commit_wall_ms.store(wall, std::memory_order_relaxed);
    O.offset.store(e.offset, std::memory_order_release);
    O.seq.fetch_add(1, std::memory_order_release);
  }
  G.n_commits.fetch_add(1, std::memory_order_relaxed);
}

int64_t Broker::committed(uint32_t g, uint32_t pidx, std::string* metadata) const {
  const OffsetEntry& O = offset_entry(g, pidx);
  const int64_t off = O.offset.load(std::memory_order_acquire);
  if (metadata && off >= 0) metadata->assign(O.metadata, size_t(O.meta_len));
  return off;
}

uint64_t Broker::commit_count(uint32_t g) const { return group(g).n_commits.load(); }

void Broker::inject_commit_failures(uint32_t g, int32_t n) { group(g).inject_commit_failures.store(n); }

void Broker::reset_group_offsets(uint32_t g) {
  group(g);
  for (uint32_t p = 0; p < meta_->max_partitions; ++p) offset_entry(g, p).offset.store(-1);
}

}  // namespace tk
