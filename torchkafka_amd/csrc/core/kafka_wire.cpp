// Native Kafka wire-protocol client: see kafka_wire.h.
#include "kafka_wire.h"

#include <arpa/inet.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/socket.h>
#include <openssl/err.h>
#include <openssl/evp.h>
#include <openssl/hmac.h>
#include <openssl/rand.h>
#include <openssl/ssl.h>
#include <openssl/x509v3.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <cstring>

namespace tk::wire {

const char* error_name(int16_t code) {
  switch (code) {
    case kNone: return "NoError";
    case kOffsetOutOfRange: return "OffsetOutOfRangeError";
    case kCorruptMessage: return "CorruptRecordException";
    case kUnknownTopicOrPartition: return "UnknownTopicOrPartitionError";
    case kLeaderNotAvailable: return "LeaderNotAvailableError";
    case kNotLeaderForPartition: return "NotLeaderForPartitionError";
    case kRequestTimedOut: return "RequestTimedOutError";
    case kCoordinatorLoadInProgress: return "CoordinatorLoadInProgressError";
    case kCoordinatorNotAvailable: return "CoordinatorNotAvailableError";
    case kNotCoordinator: return "NotCoordinatorError";
    case kIllegalGeneration: return "IllegalGenerationError";
    case kUnknownMemberId: return "UnknownMemberIdError";
    case kRebalanceInProgress: return "RebalanceInProgressError";
    case kUnsupportedVersion: return "UnsupportedVersionError";
    case kMemberIdRequired: return "MemberIdRequiredError";
    case kUnsupportedSaslMechanism: return "UnsupportedSaslMechanismError";
    case kSaslAuthenticationFailed: return "SaslAuthenticationFailedError";
    default: return "KafkaError";
  }
}

const std::map<int16_t, ApiRange>& client_versions() {
  static const std::map<int16_t, ApiRange> v = {
      {kFetch, {4, 11}},         {kListOffsets, {1, 5}},     {kMetadata, {1, 8}},
      {kOffsetCommit, {2, 7}},   {kOffsetFetch, {1, 5}},     {kFindCoordinator, {0, 2}},
      {kJoinGroup, {0, 5}},      {kHeartbeat, {0, 3}},       {kLeaveGroup, {0, 2}},
      {kSyncGroup, {0, 3}},      {kSaslHandshake, {1, 1}},   {kApiVersions, {0, 0}},
      {kSaslAuthenticate, {0, 1}},
  };
  return v;
}

int16_t legacy_version(int16_t api_key) {
  switch (api_key) {
    case kFetch: return 4;
    case kListOffsets: return 1;
    case kMetadata: return 1;
    case kOffsetCommit: return 2;
    case kOffsetFetch: return 1;
    case kSaslHandshake: return 1;
    default: return 0;
  }
}

// ------------------------------------------------------------ Writer / Reader
void Writer::i16(int16_t v) {
  const uint16_t b = htons(uint16_t(v));
  buf_.append(reinterpret_cast<const char*>(&b), 2);
}
void Writer::i32(int32_t v) {
  const uint32_t b = htonl(uint32_t(v));
  buf_.append(reinterpret_cast<const char*>(&b), 4);
}
void Writer::i64(int64_t v) {
  i32(int32_t(uint64_t(v) >> 32));
  i32(int32_t(uint64_t(v) & 0xffffffffu));
}
void Writer::str(const std::string& s) {
  if (s.size() > 32767) throw KafkaError("wire: string too long");
  i16(int16_t(s.size()));
  buf_.append(s);
}

void Reader::need(size_t n) const {
  if (size_t(end_ - p_) < n) throw KafkaError("wire: truncated response");
}
int8_t Reader::i8() { need(1); return int8_t(*p_++); }
int16_t Reader::i16() {
  need(2);
  uint16_t v;
  std::memcpy(&v, p_, 2);
  p_ += 2;
  return int16_t(ntohs(v));
}
int32_t Reader::i32() {
  need(4);
  uint32_t v;
  std::memcpy(&v, p_, 4);
  p_ += 4;
  return int32_t(ntohl(v));
}
int64_t Reader::i64() {
  const uint64_t hi = uint32_t(i32());
  const uint64_t lo = uint32_t(i32());
  return int64_t((hi << 32) | lo);
}
std::string Reader::str() {
  const int16_t n = i16();
  if (n < 0) return std::string();
  need(size_t(n));
  std::string s(reinterpret_cast<const char*>(p_), size_t(n));
  p_ += n;
  return s;
}
const uint8_t* Reader::bytes(int32_t* len) {
  const int32_t n = i32();
  *len = n;
  if (n < 0) return nullptr;
  need(size_t(n));
  const uint8_t* p = p_;
  p_ += n;
  return p;
}

// ------------------------------------------------------------ Client
std::vector<std::pair<std::string, int>> Client::parse_bootstrap(const std::string& s0) {
  std::vector<std::pair<std::string, int>> out;
  std::string s = s0;
  size_t start = 0;
  while (start <= s.size()) {
    size_t comma = s.find(',', start);
    std::string item = s.substr(start, comma == std::string::npos ? std::string::npos : comma - start);
    start = comma == std::string::npos ? s.size() + 1 : comma + 1;
    item.erase(0, item.find_first_not_of(" \t"));
    item.erase(item.find_last_not_of(" \t") + 1);
    if (item.rfind("kafka://", 0) == 0) item = item.substr(8);
    if (item.empty()) continue;
    int port = 9092;
    std::string host = item;
    const size_t close_br = item.find(']');
    const size_t colon = item.rfind(':');
    if (colon != std::string::npos && (close_br == std::string::npos ? item.find(':') == colon : colon > close_br)) {
      host = item.substr(0, colon);
      port = std::stoi(item.substr(colon + 1));
    }
    if (!host.empty() && host.front() == '[' && host.back() == ']') host = host.substr(1, host.size() - 2);
    out.emplace_back(host, port);
  }
  if (out.empty()) throw KafkaError("NoBrokersAvailable: empty bootstrap_servers");
  return out;
}

Client::Client(const std::string& bootstrap, const std::string& client_id, int timeout_ms, const Security& security)
    : bootstrap_(parse_bootstrap(bootstrap)), client_id_(client_id), timeout_ms_(timeout_ms), sec_(security) {
  if (sec_.protocol != "PLAINTEXT" && sec_.protocol != "SSL" && sec_.protocol != "SASL_PLAINTEXT" &&
      sec_.protocol != "SASL_SSL")
    throw std::invalid_argument("security_protocol must be PLAINTEXT, SSL, SASL_PLAINTEXT or SASL_SSL");
  if (!sec_.tls()) return;
  ctx_ = SSL_CTX_new(TLS_client_method());
  if (!ctx_) throw KafkaError(ssl_error("wire: SSL_CTX_new"));
  SSL_CTX_set_min_proto_version(ctx_, TLS1_2_VERSION);
  SSL_CTX_set_verify(ctx_, SSL_VERIFY_PEER, nullptr);
  const bool ok = sec_.cafile.empty() ? SSL_CTX_set_default_verify_paths(ctx_) == 1
                                      : SSL_CTX_load_verify_locations(ctx_, sec_.cafile.c_str(), nullptr) == 1;
  if (!ok) {
    SSL_CTX_free(ctx_);
    ctx_ = nullptr;
    throw KafkaError(ssl_error("wire: loading ssl_cafile"));
  }
  if (!sec_.certfile.empty()) {  // client certificate (mutual TLS)
    if (SSL_CTX_use_certificate_chain_file(ctx_, sec_.certfile.c_str()) != 1 ||
        SSL_CTX_use_PrivateKey_file(ctx_, (sec_.keyfile.empty() ? sec_.certfile : sec_.keyfile).c_str(),
                                    SSL_FILETYPE_PEM) != 1) {
      SSL_CTX_free(ctx_);
      ctx_ = nullptr;
      throw KafkaError(ssl_error("wire: loading ssl_certfile/ssl_keyfile"));
    }
  }
}

Client::~Client() {
  conns_.clear();  // TLS sessions before their context
  if (ctx_) SSL_CTX_free(ctx_);
}

Conn& Client::bootstrap_conn() {
  auto it = conns_.find(-1);
  if (it != conns_.end() && it->second->ok()) return *it->second;
  std::string why;
  for (auto& [h, p] : bootstrap_) {
    try {
      conns_[-1] = std::make_unique<Conn>(h, p, timeout_ms_, &sec_, ctx_);
      conns_[-1]->set_cancel(cancel_);
      return *conns_[-1];
    } catch (const KafkaError& e) {
      why = e.what();
    }
  }
  throw KafkaError("NoBrokersAvailable: " + why);
}

Conn& Client::conn(int32_t node_id) {
  if (node_id < 0) return bootstrap_conn();
  auto it = conns_.find(node_id);
  if (it != conns_.end() && it->second->ok()) return *it->second;
  auto nd = nodes_.find(node_id);
  if (nd == nodes_.end()) throw WireError(kLeaderNotAvailable, "wire: unknown broker node " + std::to_string(node_id));
  conns_[node_id] = std::make_unique<Conn>(nd->second.host, nd->second.port, timeout_ms_, &sec_, ctx_);
  conns_[node_id]->set_cancel(cancel_);
  return *conns_[node_id];
}

void Client::drop(int32_t node_id) { conns_.erase(node_id); }

std::vector<BrokerAddr> Client::brokers() {
  std::vector<BrokerAddr> v;
  for (auto& [id, b] : nodes_) v.push_back(b);
  return v;
}

TopicMeta Client::metadata(const std::string& topic) {
  std::vector<uint8_t> resp;
  int16_t v = 1;
  auto ask = [&]() {
    Conn& k = bootstrap_conn();
    v = k.version(kMetadata);
    Writer w;
    w.array(1);
    w.str(topic);
    if (v >= 4) w.i8(0);  // allow_auto_topic_creation: false (a consumer never creates topics)
    if (v >= 8) {
      w.i8(0);  // include_cluster_authorized_operations
      w.i8(0);  // include_topic_authorized_operations
    }
    resp = k.roundtrip(kMetadata, v, client_id_, w.data(), timeout_ms_);
  };
  try {
    ask();
  } catch (const WireError&) {
    throw;
  } catch (const KafkaError&) {
    drop(-1);
    ask();
  }
  Reader r(resp.data(), resp.size());
  if (v >= 3) r.i32();  // throttle_time_ms
  const int32_t nb = r.i32();
  for (int32_t i = 0; i < nb; ++i) {
    BrokerAddr b;
    b.node_id = r.i32();
    b.host = r.str();
    b.port = r.i32();
    if (v >= 1) r.str();  // rack
    auto old = nodes_.find(b.node_id);
    if (old != nodes_.end() && (old->second.host != b.host || old->second.port != b.port)) drop(b.node_id);
    nodes_[b.node_id] = b;
  }
  if (v >= 2) r.str();  // cluster id
  r.i32();              // controller
  const int32_t nt = r.i32();
  TopicMeta out;
  out.name = topic;
  out.error = kUnknownTopicOrPartition;
  for (int32_t i = 0; i < nt; ++i) {
    TopicMeta t;
    t.error = r.i16();
    t.name = r.str();
    r.i8();  // is_internal
    const int32_t np = r.i32();
    for (int32_t j = 0; j < np; ++j) {
      PartitionMeta p;
      p.error = r.i16();
      p.partition = r.i32();
      p.leader = r.i32();
      if (v >= 7) r.i32();  // leader epoch
      const int32_t nrep = r.i32();
      for (int32_t k = 0; k < nrep; ++k) r.i32();
      const int32_t nisr = r.i32();
      for (int32_t k = 0; k < nisr; ++k) r.i32();
      if (v >= 5) {
        const int32_t noff = r.i32();  // offline replicas
        for (int32_t k = 0; k < noff; ++k) r.i32();
      }
      t.partitions.push_back(p);
    }
    if (v >= 8) r.i32();  // topic authorized operations
    std::sort(t.partitions.begin(), t.partitions.end(),
              [](const PartitionMeta& a, const PartitionMeta& b) { return a.partition < b.partition; });
    if (t.name == topic) out = t;
    topics_[t.name] = t;
  }
  return out;
}

int32_t Client::leader(const std::string& topic, int32_t partition) {
  auto it = topics_.find(topic);
  if (it == topics_.end()) return -1;
  for (auto& p : it->second.partitions)
    if (p.partition == partition) return p.error == kNone || p.error == kLeaderNotAvailable ? p.leader : -1;
  return -1;
}

std::map<int32_t, int64_t> Client::list_offsets(const std::string& topic, const std::vector<int32_t>& parts,
                                                int64_t timestamp) {
  if (topics_.find(topic) == topics_.end()) metadata(topic);
  std::map<int32_t, std::vector<int32_t>> by_leader;
  for (int32_t p : parts) by_leader[leader(topic, p)].push_back(p);
  std::map<int32_t, int64_t> out;
  for (auto& [node, ps] : by_leader) {
    if (node < 0) throw WireError(kLeaderNotAvailable, "LeaderNotAvailableError: " + topic);
    Conn& k = conn(node);
    const int16_t v = k.version(kListOffsets);
    Writer w;
    w.i32(-1);           // replica id
    if (v >= 2) w.i8(0);  // isolation level: read_uncommitted
    w.array(1);
    w.str(topic);
    w.array(int32_t(ps.size()));
    for (int32_t p : ps) {
      w.i32(p);
      if (v >= 4) w.i32(-1);  // current leader epoch: unknown
      w.i64(timestamp);
    }
    auto resp = k.roundtrip(kListOffsets, v, client_id_, w.data(), timeout_ms_);
    Reader r(resp.data(), resp.size());
    if (v >= 2) r.i32();  // throttle
    const int32_t nt = r.i32();
    for (int32_t i = 0; i < nt; ++i) {
      r.str();
      const int32_t np = r.i32();
      for (int32_t j = 0; j < np; ++j) {
        const int32_t p = r.i32();
        const int16_t e = r.i16();
        r.i64();  // timestamp
        const int64_t off = r.i64();
        if (v >= 4) r.i32();  // leader epoch
        if (e != kNone)
          throw WireError(e, std::string(error_name(e)) + ": ListOffsets " + topic + "-" + std::to_string(p));
        out[p] = off;
      }
    }
  }
  return out;
}

int32_t Client::coordinator(const std::string& group) {
  if (coordinator_ >= 0 && coordinator_group_ == group) return coordinator_;
  Conn& k = bootstrap_conn();
  const int16_t v = k.version(kFindCoordinator);
  Writer w;
  w.str(group);
  if (v >= 1) w.i8(0);  // key type: group
  auto resp = k.roundtrip(kFindCoordinator, v, client_id_, w.data(), timeout_ms_);
  Reader r(resp.data(), resp.size());
  if (v >= 1) r.i32();  // throttle
  const int16_t e = r.i16();
  std::string msg;
  if (v >= 1) msg = r.str();
  BrokerAddr b;
  b.node_id = r.i32();
  b.host = r.str();
  b.port = r.i32();
  if (e != kNone)
    throw WireError(e, std::string(error_name(e)) + ": FindCoordinator " + group + (msg.empty() ? "" : " (" + msg + ")"));
  auto old = nodes_.find(b.node_id);
  if (old != nodes_.end() && (old->second.host != b.host || old->second.port != b.port)) drop(b.node_id);
  nodes_[b.node_id] = b;
  coordinator_ = b.node_id;
  coordinator_group_ = group;
  return coordinator_;
}

std::map<int32_t, int64_t> Client::offset_fetch(const std::string& group, const std::string& topic,
                                                const std::vector<int32_t>& parts) {
  Writer w;
  w.str(group);
  w.array(1);
  w.str(topic);
  w.array(int32_t(parts.size()));
  for (int32_t p : parts) w.i32(p);
  int16_t v = 1;
  auto resp = coordinator_roundtrip(group, kOffsetFetch, -1, w.data(), timeout_ms_, &v);
  Reader r(resp.data(), resp.size());
  if (v >= 3) r.i32();  // throttle
  std::map<int32_t, int64_t> out;
  const int32_t nt = r.i32();
  int16_t first_err = kNone;
  int32_t err_part = -1;
  for (int32_t i = 0; i < nt; ++i) {
    r.str();
    const int32_t np = r.i32();
    for (int32_t j = 0; j < np; ++j) {
      const int32_t p = r.i32();
      const int64_t off = r.i64();
      if (v >= 5) r.i32();  // committed leader epoch
      r.str();              // metadata
      const int16_t e = r.i16();
      if (e != kNone && first_err == kNone) {
        first_err = e;
        err_part = p;
      }
      out[p] = off;
    }
  }
  const int16_t top = v >= 2 ? r.i16() : int16_t(kNone);
  const int16_t e = top != kNone ? top : first_err;
  if (e != kNone) {
    if (needs_metadata(e)) invalidate_coordinator();
    throw WireError(e, std::string(error_name(e)) + ": OffsetFetch " + topic +
                           (top == kNone ? "-" + std::to_string(err_part) : std::string()));
  }
  return out;
}

std::vector<uint8_t> Client::coordinator_roundtrip(const std::string& group, int16_t key, int16_t version,
                                                  const std::string& body, int timeout_ms, int16_t* used) {
  const int32_t node = coordinator(group);
  try {
    Conn& k = conn(node);
    const int16_t v = version >= 0 ? version : k.version(key);
    if (used) *used = v;
    return k.roundtrip(key, v, client_id_, body, timeout_ms);
  } catch (const WireError& e) {
    if (e.code != kUnsupportedVersion) {
      drop(node);
      invalidate_coordinator();
    }
    throw;
  } catch (const KafkaError&) {
    drop(node);
    invalidate_coordinator();
    throw;
  }
}

int16_t Client::coordinator_version(const std::string& group, int16_t key) {
  return conn(coordinator(group)).version(key);
}

JoinResult Client::join_group(const std::string& group, int32_t session_timeout_ms, const std::string& member_id,
                              const std::string& subscription, const std::vector<std::string>& protocols,
                              int32_t rebalance_timeout_ms) {
  const int16_t v = coordinator_version(group, kJoinGroup);
  const int32_t rebalance = rebalance_timeout_ms > 0 ? rebalance_timeout_ms : session_timeout_ms;
  Writer w;
  w.str(group);
  w.i32(session_timeout_ms);
  if (v >= 1) w.i32(rebalance);
  w.str(member_id);
  if (v >= 5) w.nullable_str_null();  // group instance id: dynamic membership
  w.str("consumer");
  w.array(int32_t(protocols.size()));
  for (auto& name : protocols) {
    w.str(name);
    w.i32(int32_t(subscription.size()));
    w.data() += subscription;
  }
  // the coordinator holds the request until the join round ends
  auto resp = coordinator_roundtrip(group, kJoinGroup, v, w.data(),
                                    timeout_ms_ + std::max(session_timeout_ms, v >= 1 ? rebalance : 0));
  Reader r(resp.data(), resp.size());
  JoinResult j;
  if (v >= 2) r.i32();  // throttle
  j.error = r.i16();
  j.generation = r.i32();
  j.protocol = r.str();
  j.leader = r.str();
  j.member_id = r.str();
  const int32_t n = r.i32();
  for (int32_t i = 0; i < n; ++i) {
    std::string m = r.str();
    if (v >= 5) r.str();  // group instance id
    int32_t len = 0;
    const uint8_t* p = r.bytes(&len);
    j.members.emplace_back(std::move(m), len > 0 ? std::string(reinterpret_cast<const char*>(p), size_t(len)) : "");
  }
  if (needs_metadata(j.error)) invalidate_coordinator();
  return j;
}

std::pair<int16_t, std::string> Client::sync_group(const std::string& group, int32_t generation,
                                                   const std::string& member_id,
                                                   const std::map<std::string, std::string>& assignments) {
  const int16_t v = coordinator_version(group, kSyncGroup);
  Writer w;
  w.str(group);
  w.i32(generation);
  w.str(member_id);
  if (v >= 3) w.nullable_str_null();  // group instance id
  w.array(int32_t(assignments.size()));
  for (auto& [m, a] : assignments) {
    w.str(m);
    w.i32(int32_t(a.size()));
    w.data() += a;
  }
  auto resp = coordinator_roundtrip(group, kSyncGroup, v, w.data(), timeout_ms_ * 2);
  Reader r(resp.data(), resp.size());
  if (v >= 1) r.i32();  // throttle
  const int16_t e = r.i16();
  int32_t len = 0;
  const uint8_t* p = r.bytes(&len);
  if (needs_metadata(e)) invalidate_coordinator();
  return {e, len > 0 ? std::string(reinterpret_cast<const char*>(p), size_t(len)) : std::string()};
}

int16_t Client::heartbeat(const std::string& group, int32_t generation, const std::string& member_id) {
  const int16_t v = coordinator_version(group, kHeartbeat);
  Writer w;
  w.str(group);
  w.i32(generation);
  w.str(member_id);
  if (v >= 3) w.nullable_str_null();  // group instance id
  auto resp = coordinator_roundtrip(group, kHeartbeat, v, w.data(), timeout_ms_);
  Reader r(resp.data(), resp.size());
  if (v >= 1) r.i32();  // throttle
  const int16_t e = r.i16();
  if (needs_metadata(e)) invalidate_coordinator();
  return e;
}

int16_t Client::leave_group(const std::string& group, const std::string& member_id) {
  const int16_t v = coordinator_version(group, kLeaveGroup);
  Writer w;
  w.str(group);
  w.str(member_id);
  auto resp = coordinator_roundtrip(group, kLeaveGroup, v, w.data(), timeout_ms_);
  Reader r(resp.data(), resp.size());
  if (v >= 1) r.i32();  // throttle
  return r.i16();
}

std::string encode_subscription(const std::vector<std::string>& topics) {
  Writer w;
  w.i16(0);  // version
  w.array(int32_t(topics.size()));
  for (auto& t : topics) w.str(t);
  w.i32(-1);  // user data: null
  return w.data();
}

std::vector<std::string> decode_subscription(const std::string& metadata) {
  Reader r(reinterpret_cast<const uint8_t*>(metadata.data()), metadata.size());
  r.i16();
  std::vector<std::string> out(size_t(std::max(0, r.i32())));
  for (auto& t : out) t = r.str();
  return out;
}

std::string encode_assignment(const Assignment& a) {
  Writer w;
  w.i16(0);
  w.array(int32_t(a.size()));
  for (auto& [t, ps] : a) {
    w.str(t);
    w.array(int32_t(ps.size()));
    for (int32_t p : ps) w.i32(p);
  }
  w.i32(-1);
  return w.data();
}

Assignment decode_assignment(const std::string& bytes) {
  Assignment a;
  if (bytes.size() < 2) return a;  // an empty assignment
  Reader r(reinterpret_cast<const uint8_t*>(bytes.data()), bytes.size());
  r.i16();
  const int32_t nt = r.i32();
  for (int32_t i = 0; i < nt; ++i) {
    std::string t = r.str();
    auto& ps = a[t];
    const int32_t np = r.i32();
    for (int32_t j = 0; j < np; ++j) ps.push_back(r.i32());
  }
  return a;
}

std::map<std::string, Assignment> range_assign(const std::vector<std::pair<std::string, std::string>>& members,
                                               const std::map<std::string, int32_t>& partitions_per_topic) {
  std::map<std::string, Assignment> out;
  std::map<std::string, std::vector<std::string>> subscribers;  // topic -> member ids (sorted: std::map order)
  std::map<std::string, std::vector<std::string>> subs;
  for (auto& [m, meta] : members) {
    out[m];
    subs[m] = decode_subscription(meta);
  }
  for (auto& [m, topics] : subs)
    for (auto& t : topics) subscribers[t].push_back(m);
  for (auto& [t, ms] : subscribers) {
    auto it = partitions_per_topic.find(t);
    if (it == partitions_per_topic.end() || ms.empty()) continue;
    const int32_t P = it->second, C = int32_t(ms.size()), per = P / C, extra = P % C;
    for (int32_t i = 0; i < C; ++i) {
      const int32_t start = per * i + std::min(i, extra), len = per + (i < extra ? 1 : 0);
      auto& ps = out[ms[size_t(i)]][t];
      for (int32_t p = start; p < start + len; ++p) ps.push_back(p);
    }
  }
  return out;
}

std::map<std::string, Assignment> roundrobin_assign(const std::vector<std::pair<std::string, std::string>>& members,
                                                    const std::map<std::string, int32_t>& partitions_per_topic) {
  std::map<std::string, Assignment> out;
  std::map<std::string, std::vector<std::string>> subs;  // member -> topics (sorted by member id)
  for (auto& [m, meta] : members) {
    out[m];
    subs[m] = decode_subscription(meta);
  }
  std::vector<std::string> ids;
  for (auto& [m, t] : subs) ids.push_back(m);
  size_t next = 0;
  for (auto& [topic, n] : partitions_per_topic)
    for (int32_t p = 0; p < n && !ids.empty(); ++p)
      for (size_t k = 0; k < ids.size(); ++k) {  // next member (cyclically) subscribed to `topic`
        const std::string& m = ids[(next + k) % ids.size()];
        const auto& ts = subs[m];
        if (std::find(ts.begin(), ts.end(), topic) == ts.end()) continue;
        out[m][topic].push_back(p);
        next = (next + k + 1) % ids.size();
        break;
      }
  return out;
}

std::map<int32_t, int16_t> Client::offset_commit(const std::string& group, const std::string& topic,
                                                 const std::map<int32_t, int64_t>& offsets,
                                                 const std::string& metadata, int32_t generation,
                                                 const std::string& member_id) {
  const int16_t v = coordinator_version(group, kOffsetCommit);
  Writer w;
  w.str(group);
  w.i32(generation);  // -1 with an empty member id: a manually assigned ("simple") consumer
  w.str(member_id);
  if (v >= 7) w.nullable_str_null();  // group instance id
  if (v <= 4) w.i64(-1);              // retention: the broker's default (dropped in v5)
  w.array(1);
  w.str(topic);
  w.array(int32_t(offsets.size()));
  for (auto& [p, o] : offsets) {
    w.i32(p);
    w.i64(o);
    if (v >= 6) w.i32(-1);  // committed leader epoch: unknown
    w.str(metadata);
  }
  auto resp = coordinator_roundtrip(group, kOffsetCommit, v, w.data(), timeout_ms_);
  Reader r(resp.data(), resp.size());
  if (v >= 3) r.i32();  // throttle
  std::map<int32_t, int16_t> out;
  const int32_t nt = r.i32();
  for (int32_t i = 0; i < nt; ++i) {
    r.str();
    const int32_t np = r.i32();
    for (int32_t j = 0; j < np; ++j) {
      const int32_t p = r.i32();
      const int16_t e = r.i16();
      if (needs_metadata(e)) invalidate_coordinator();
      out[p] = e;
    }
  }
  return out;
}

std::string fetch_request(int16_t v, const std::string& topic, const std::vector<FetchPartReq>& parts,
                          int32_t max_wait_ms, int32_t min_bytes, int32_t max_bytes) {
  Writer w;
  w.i32(-1);  // replica id: a consumer
  w.i32(max_wait_ms);
  w.i32(min_bytes);
  w.i32(max_bytes);
  w.i8(0);    // isolation level: read_uncommitted (kafka-python's default)
  if (v >= 7) {
    w.i32(0);   // session id 0 + epoch -1: a sessionless (full) fetch (KIP-227)
    w.i32(-1);
  }
  w.array(1);
  w.str(topic);
  w.array(int32_t(parts.size()));
  for (auto& p : parts) {
    w.i32(p.partition);
    if (v >= 9) w.i32(-1);  // current leader epoch: unknown
    w.i64(p.offset);
    if (v >= 5) w.i64(-1);  // log start offset: a consumer sends -1
    w.i32(p.max_bytes);
  }
  if (v >= 7) w.array(0);  // forgotten topics
  if (v >= 11) w.str("");  // rack id
  return std::move(w.data());
}

void fetch_response_header(Conn& k, int16_t v) {
  k.r32();  // throttle_time_ms
  if (v >= 7) {
    const int16_t e = k.r16();
    k.r32();  // session id
    if (e != kNone) throw WireError(e, std::string(error_name(e)) + ": Fetch");
  }
}

FetchPartHeader fetch_partition_header(Conn& k, int16_t v) {
  FetchPartHeader h;
  h.partition = k.r32();
  h.error = k.r16();
  h.high_watermark = k.r64();
  k.r64();              // last stable offset
  if (v >= 5) k.r64();  // log start offset
  const int32_t n_aborted = k.r32();
  if (n_aborted > 0) k.skip(size_t(n_aborted) * 16);
  if (v >= 11) k.r32();  // preferred read replica
  h.records_len = k.r32();
  return h;
}

}  // namespace tk::wire
