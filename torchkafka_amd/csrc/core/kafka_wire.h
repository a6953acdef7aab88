// Native Kafka wire-protocol client (the part of a consumer this framework needs).
//
// The reference reaches its cluster through kafka-python's KafkaConsumer
// (kafka_dataset.py:21-22, 206): a Python client that parses every Fetch response, checks
// every RecordBatch CRC on the CPU and hands out Python records one by one.  Here the
// cluster is read by a native replicator (replicator.h) that speaks the protocol directly:
// Fetch responses are received straight into the local partition logs (the same mapped
// RecordBatch v2 logs the synthetic broker keeps), so workers walk headers and the gfx950
// decode kernels verify CRCs and decode values from those bytes exactly as they do for the
// synthetic broker -- no Python, no per-record objects, no second host copy.
//
// Protocol subset: the non-flexible request versions, negotiated per connection.  Every new
// connection first sends ApiVersions v0 and each request then goes out at the highest version
// both sides implement (client ranges in client_versions(); the broker's from its answer), as
// kafka-python and the Java client do.  A broker that predates ApiVersions (it closes the
// connection) gets the fixed pre-negotiation set: Metadata v1, ListOffsets v1, Fetch v4,
// FindCoordinator v0, OffsetCommit v2, OffsetFetch v1, JoinGroup / SyncGroup / Heartbeat /
// LeaveGroup v0.  Client ranges: Metadata 1-8, ListOffsets 1-5, Fetch 4-11 (sessionless),
// FindCoordinator 0-2, OffsetCommit 2-7, OffsetFetch 1-5, JoinGroup 0-5 (v4+: the
// MEMBER_ID_REQUIRED round trip), SyncGroup 0-3, Heartbeat 0-3, LeaveGroup 0-2 -- which covers
// brokers from 0.11 through Kafka 4.x, whose KIP-896 dropped the pre-2.1 versions (e.g. JoinGroup
// v0-1, Fetch v0-3).  Group membership uses the "consumer" protocol with Kafka's range and
// round-robin assignors.
// By default partitions are assigned statically by (rank, worker) as in the rest of the
// framework, and offsets are committed like kafka-python's manually-assigned consumer with a
// group_id (generation -1, empty member id).
#pragma once
#include <sys/types.h>

#include <atomic>
#include <cstdint>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <utility>
#include <vector>

#include "common.h"

typedef struct ssl_st SSL;
typedef struct ssl_ctx_st SSL_CTX;

namespace tk::wire {

// Connection security, named as kafka-python's configuration: security_protocol PLAINTEXT | SSL |
// SASL_PLAINTEXT | SASL_SSL; TLS through OpenSSL (server verified against ssl_cafile, or the
// system store); SASL mechanisms PLAIN, SCRAM-SHA-256 and SCRAM-SHA-512 (SaslHandshake v1 +
// SaslAuthenticate v0).
// SASL/OAUTHBEARER (RFC 7628): the bearer token (and "key=value" extensions joined by 0x01) a
// connection authenticates with.  Shared by every copy of the Security it belongs to, so a token
// refreshed through one handle (Replicator::set_oauth_token) reaches the connections made later.
struct OAuthToken {
  std::mutex m;
  std::string token, extensions;
};

struct Security {
  std::string protocol = "PLAINTEXT";
  std::string cafile, certfile, keyfile;
  bool check_hostname = true;
  std::string sasl_mechanism = "PLAIN";
  std::string username, password;
  std::shared_ptr<OAuthToken> oauth;  // sasl_mechanism OAUTHBEARER
  bool tls() const { return protocol == "SSL" || protocol == "SASL_SSL"; }
  bool sasl() const { return protocol == "SASL_PLAINTEXT" || protocol == "SASL_SSL"; }
};

enum ApiKey : int16_t {
  kFetch = 1, kListOffsets = 2, kMetadata = 3, kOffsetCommit = 8, kOffsetFetch = 9,
  kFindCoordinator = 10, kJoinGroup = 11, kHeartbeat = 12, kLeaveGroup = 13, kSyncGroup = 14, kSaslHandshake = 17, kApiVersions = 18, kSaslAuthenticate = 36,
};

// Kafka error codes the client acts on.
enum ErrorCode : int16_t {
  kNone = 0, kOffsetOutOfRange = 1, kCorruptMessage = 2, kUnknownTopicOrPartition = 3,
  kLeaderNotAvailable = 5, kNotLeaderForPartition = 6, kRequestTimedOut = 7,
  kCoordinatorLoadInProgress = 14, kCoordinatorNotAvailable = 15, kNotCoordinator = 16,
  kIllegalGeneration = 22, kUnknownMemberId = 25, kRebalanceInProgress = 27,
  kUnsupportedSaslMechanism = 33, kIllegalSaslState = 34, kUnsupportedVersion = 35,
  kSaslAuthenticationFailed = 58, kMemberIdRequired = 79,
};

// Version range of one API.
struct ApiRange {
  int16_t min, max;
};
// What this client implements, per API key.
const std::map<int16_t, ApiRange>& client_versions();
// What it sends to a broker that does not answer ApiVersions.
int16_t legacy_version(int16_t api_key);
const char* error_name(int16_t code);
// OpenSSL's latest error appended to `what` (kafka_wire_conn.cpp)
std::string ssl_error(const std::string& what);
// Errors after which the partition's leader (or the group's coordinator) must be looked up again.
inline bool needs_metadata(int16_t e) {
  return e == kUnknownTopicOrPartition || e == kLeaderNotAvailable || e == kNotLeaderForPartition ||
         e == kCoordinatorNotAvailable || e == kNotCoordinator || e == kCoordinatorLoadInProgress ||
         e == kRequestTimedOut;
}

struct WireError : KafkaError {
  int16_t code;
  WireError(int16_t c, const std::string& what) : KafkaError(what), code(c) {}
};

// ------------------------------------------------------------ encoding (big-endian)
class Writer {
 public:
  void i8(int8_t v) { buf_.push_back(char(v)); }
  void i16(int16_t v);
  void i32(int32_t v);
  void i64(int64_t v);
  void str(const std::string& s);   // int16 length + bytes
  void nullable_str_null() { i16(-1); }
  void array(int32_t n) { i32(n); }
  std::string& data() { return buf_; }

 private:
  std::string buf_;
};

class Reader {
 public:
  Reader(const uint8_t* p, size_t n) : p_(p), end_(p + n) {}
  int8_t i8();
  int16_t i16();
  int32_t i32();
  int64_t i64();
  std::string str();          // nullable: null -> ""
  const uint8_t* bytes(int32_t* len);  // nullable bytes (int32 length; null -> len -1)
  size_t left() const { return size_t(end_ - p_); }

 private:
  void need(size_t n) const;
  const uint8_t* p_;
  const uint8_t* end_;
};

// ------------------------------------------------------------ one TCP connection
class Conn {
 public:
  // sec/ctx: TLS handshake and SASL authentication right after the TCP connect (nullptr: plaintext).
  Conn(const std::string& host, int port, int timeout_ms, const Security* sec = nullptr, SSL_CTX* ctx = nullptr);
  ~Conn();
  Conn(const Conn&) = delete;
  Conn& operator=(const Conn&) = delete;
  const std::string& host() const { return host_; }
  int port() const { return port_; }
  bool ok() const { return fd_ >= 0; }

  // The version to send `api_key` at on this connection: the highest one both this client and the
  // broker implement (WireError UNSUPPORTED_VERSION when the ranges do not meet).
  int16_t version(int16_t api_key) const;
  // The broker's ApiVersions answer (empty: it predates ApiVersions, legacy_version() is used).
  const std::map<int16_t, ApiRange>& broker_versions() const { return broker_; }

  // Request/response with the whole response body in memory (small responses).
  std::vector<uint8_t> roundtrip(int16_t api_key, int16_t api_version, const std::string& client_id,
                                 const std::string& body, int timeout_ms);

  // Streaming responses (Fetch): send, then read the body field by field; record sets are
  // received straight into the caller's memory.
  void send(int16_t api_key, int16_t api_version, const std::string& client_id, const std::string& body);
  size_t begin_response(int timeout_ms);  // reads size + correlation id; returns body bytes
  void read(void* dst, size_t n);
  int8_t r8();
  int16_t r16();
  int32_t r32();
  int64_t r64();
  std::string rstr();
  void skip(size_t n);
  void finish();  // drains the rest of the current response
  size_t remaining() const { return remaining_; }
  void close();
  // Waits for the socket end early (KafkaError "cancelled") once *flag is true: a stopping
  // replicator does not sit out a request timeout on an unresponsive broker.
  void set_cancel(const std::atomic<bool>* flag) { cancel_ = flag; }

 private:
  void send_all(const std::string& frame);
  void fill(size_t want);  // at least min(want, remaining) bytes buffered
  ssize_t io_recv(void* dst, size_t n);
  bool wait_readable(int ms);
  void open_socket(const Security* sec, SSL_CTX* ctx);  // TCP connect (+ TLS handshake)
  void negotiate(const Security* sec, SSL_CTX* ctx);    // ApiVersions
  std::map<int16_t, ApiRange> broker_;
  void authenticate(const Security& sec);
  void scram(const Security& sec);
  void oauthbearer(const Security& sec);
  std::string sasl_round(const std::string& token);
  SSL* ssl_ = nullptr;
  std::string host_;
  int port_;
  int fd_ = -1;
  int timeout_ms_;
  int64_t deadline_ms_ = 0;
  int32_t corr_ = 0;
  int32_t expect_corr_ = -1;
  size_t remaining_ = 0;
  std::vector<uint8_t> buf_;
  size_t b0_ = 0, b1_ = 0;
  const std::atomic<bool>* cancel_ = nullptr;
  void check_cancel();
};

// ------------------------------------------------------------ cluster view
struct BrokerAddr {
  int32_t node_id;
  std::string host;
  int32_t port;
};
struct PartitionMeta {
  int32_t partition;
  int32_t leader;  // -1 when none
  int16_t error;
};
struct TopicMeta {
  std::string name;
  int16_t error = 0;
  std::vector<PartitionMeta> partitions;  // sorted by partition id
};

// JoinGroup response; `members` (member id, subscription metadata) is filled for the leader only.
struct JoinResult {
  int16_t error = 0;
  int32_t generation = -1;
  std::string protocol, leader, member_id;
  std::vector<std::pair<std::string, std::string>> members;
};
using Assignment = std::map<std::string, std::vector<int32_t>>;  // topic -> partitions

// Consumer protocol v0 (ConsumerProtocolSubscription / ConsumerProtocolAssignment).
std::string encode_subscription(const std::vector<std::string>& topics);
std::vector<std::string> decode_subscription(const std::string& metadata);
std::string encode_assignment(const Assignment& a);
Assignment decode_assignment(const std::string& bytes);
// Kafka's RangeAssignor: per topic, the subscribed members sorted by id take contiguous ranges,
// the first (P % members) one partition more.  members: (id, subscription metadata).
std::map<std::string, Assignment> range_assign(const std::vector<std::pair<std::string, std::string>>& members,
                                               const std::map<std::string, int32_t>& partitions_per_topic);
// Kafka's RoundRobinAssignor: every (topic, partition) in order, dealt to the members sorted by id
// (skipping members not subscribed to that topic).
std::map<std::string, Assignment> roundrobin_assign(const std::vector<std::pair<std::string, std::string>>& members,
                                                    const std::map<std::string, int32_t>& partitions_per_topic);

struct FetchPartReq {
  int32_t partition;
  int64_t offset;
  int32_t max_bytes;
};

class Client {
 public:
  // bootstrap: "host:port[,host:port...]" (an optional "kafka://" prefix is accepted).
  Client(const std::string& bootstrap, const std::string& client_id, int timeout_ms,
         const Security& security = Security());
  ~Client();
  static std::vector<std::pair<std::string, int>> parse_bootstrap(const std::string& s);

  TopicMeta metadata(const std::string& topic);          // refreshes the broker table too
  std::vector<BrokerAddr> brokers();
  // ListOffsets: timestamp -2 = earliest, -1 = latest, else first offset with ts >= timestamp.
  std::map<int32_t, int64_t> list_offsets(const std::string& topic, const std::vector<int32_t>& parts,
                                          int64_t timestamp);
  std::map<int32_t, int64_t> offset_fetch(const std::string& group, const std::string& topic,
                                          const std::vector<int32_t>& parts);
  // Returns per-partition error codes (0 = committed).
  std::map<int32_t, int16_t> offset_commit(const std::string& group, const std::string& topic,
                                           const std::map<int32_t, int64_t>& offsets,
                                           const std::string& metadata = "", int32_t generation = -1,
                                           const std::string& member_id = "");
  // Group membership against the group's coordinator.  join_group blocks at the coordinator
  // until the join round ends (up to the session timeout).
  // protocols: assignor names in preference order ("range", "roundrobin")
  // rebalance_timeout_ms (JoinGroup v1+): how long the coordinator waits for every member to
  // rejoin during a rebalance (kafka-python: max_poll_interval_ms); <= 0: the session timeout.
  JoinResult join_group(const std::string& group, int32_t session_timeout_ms, const std::string& member_id,
                        const std::string& subscription,
                        const std::vector<std::string>& protocols = std::vector<std::string>{"range"},
                        int32_t rebalance_timeout_ms = -1);
  std::pair<int16_t, std::string> sync_group(const std::string& group, int32_t generation,
                                             const std::string& member_id,
                                             const std::map<std::string, std::string>& assignments);
  int16_t heartbeat(const std::string& group, int32_t generation, const std::string& member_id);
  int16_t leave_group(const std::string& group, const std::string& member_id);
  void invalidate_coordinator() { coordinator_ = -1; }
  void set_cancel(const std::atomic<bool>* flag) { cancel_ = flag; }  // every connection of this client

  // Connection to a node (-1: any bootstrap server).  Owned by the client; one per node.
  Conn& conn(int32_t node_id);
  void drop(int32_t node_id);
  const std::string& client_id() const { return client_id_; }
  int timeout_ms() const { return timeout_ms_; }
  int32_t leader(const std::string& topic, int32_t partition);  // cached, -1 unknown

 private:
  Conn& bootstrap_conn();
  int32_t coordinator(const std::string& group);
  // version < 0: negotiated on the coordinator's connection (reported through *used)
  std::vector<uint8_t> coordinator_roundtrip(const std::string& group, int16_t key, int16_t version,
                                             const std::string& body, int timeout_ms, int16_t* used = nullptr);
  int16_t coordinator_version(const std::string& group, int16_t key);
  std::vector<std::pair<std::string, int>> bootstrap_;
  std::string client_id_;
  int timeout_ms_;
  std::map<int32_t, BrokerAddr> nodes_;
  std::map<int32_t, std::unique_ptr<Conn>> conns_;  // node -> connection (-1: bootstrap)
  std::map<std::string, TopicMeta> topics_;
  int32_t coordinator_ = -1;
  std::string coordinator_group_;
  const std::atomic<bool>* cancel_ = nullptr;
  Security sec_;
  SSL_CTX* ctx_ = nullptr;
};

// Encodes a sessionless Fetch request body of `version` (4..11).
std::string fetch_request(int16_t version, const std::string& topic, const std::vector<FetchPartReq>& parts,
                          int32_t max_wait_ms, int32_t min_bytes, int32_t max_bytes);
// Streaming Fetch response parts that vary with the version (the replicator reads the rest).
void fetch_response_header(Conn& k, int16_t version);  // throttle / error / session, up to the topic array
struct FetchPartHeader {
  int32_t partition;
  int16_t error;
  int64_t high_watermark;
  int32_t records_len;  // -1: null
};
FetchPartHeader fetch_partition_header(Conn& k, int16_t version);  // up to (and including) the records length

}  // namespace tk::wire
