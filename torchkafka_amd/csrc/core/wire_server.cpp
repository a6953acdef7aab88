// Native Kafka-protocol front end for the shared-memory broker: see wire_server.h.
#include "wire_server.h"

#include <arpa/inet.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/socket.h>
#include <sys/uio.h>
#include <unistd.h>

#include <chrono>
#include <climits>
#include <cstring>

#include "kafka_wire.h"

namespace tk {

namespace {

bool recv_exact(int fd, void* dst, size_t n, const std::atomic<bool>& stop) {
  auto* d = static_cast<uint8_t*>(dst);
  size_t got = 0;
  while (got < n) {
    pollfd p{fd, POLLIN, 0};
    const int r = ::poll(&p, 1, 100);
    if (stop.load()) return false;
    if (r <= 0) continue;
    const ssize_t k = ::recv(fd, d + got, n - got, 0);
    if (k <= 0) return false;
    got += size_t(k);
  }
  return true;
}

bool send_iov(int fd, std::vector<iovec>& iov) {
  size_t i = 0;
  while (i < iov.size()) {
    const int cnt = int(std::min<size_t>(iov.size() - i, IOV_MAX));
    msghdr m{};
    m.msg_iov = &iov[i];
    m.msg_iovlen = size_t(cnt);
    ssize_t k = ::sendmsg(fd, &m, MSG_NOSIGNAL);
    if (k < 0) {
      if (errno == EINTR) continue;
      return false;
    }
    while (k > 0 && i < iov.size()) {  // advance over what was sent
      if (size_t(k) >= iov[i].iov_len) {
        k -= ssize_t(iov[i].iov_len);
        ++i;
      } else {
        iov[i].iov_base = static_cast<uint8_t*>(iov[i].iov_base) + k;
        iov[i].iov_len -= size_t(k);
        k = 0;
      }
    }
  }
  return true;
}

// A response assembled from small encoded pieces and zero-copy slices of the partition logs.
struct Response {
  std::vector<std::string> pieces;
  std::vector<std::pair<int, std::pair<const uint8_t*, size_t>>> order;  // (piece index or -1, slice)
  wire::Writer w;
  void cut() {
    pieces.push_back(std::move(w.data()));
    w = wire::Writer();
    order.push_back({int(pieces.size()) - 1, {nullptr, 0}});
  }
  void slice(const uint8_t* p, size_t n) {
    cut();
    order.push_back({-1, {p, n}});
  }
  bool send(int fd, int32_t corr, std::atomic<uint64_t>* bytes) {
    cut();
    size_t total = 4;
    for (auto& o : order) total += o.first >= 0 ? pieces[size_t(o.first)].size() : o.second.second;
    wire::Writer h;
    h.i32(int32_t(total));
    h.i32(corr);
    std::vector<iovec> iov;
    iov.push_back({h.data().data(), h.data().size()});
    for (auto& o : order) {
      if (o.first >= 0) {
        auto& s = pieces[size_t(o.first)];
        if (!s.empty()) iov.push_back({s.data(), s.size()});
      } else if (o.second.second) {
        iov.push_back({const_cast<uint8_t*>(o.second.first), o.second.second});
      }
    }
    bytes->fetch_add(total + 4, std::memory_order_relaxed);
    return send_iov(fd, iov);
  }
};

}  // namespace

WireServer::WireServer(std::shared_ptr<Broker> broker, const std::string& host, int port, int32_t node_id,
                       std::vector<WireNode> cluster, const std::string& profile)
    : b_(std::move(broker)), host_(host), port_(port), node_(node_id), cluster_(std::move(cluster)) {
  // the Python server's PROFILES (broker/wire_server.py) for the APIs served here
  if (profile == "legacy" || profile == "ancient") {
    versions_ = {{1, 4, 4}, {2, 0, 1}, {3, 0, 1}, {8, 2, 2}, {9, 1, 1}, {10, 0, 0}, {18, 0, 0}};
    api_versions_ = profile == "legacy";
  } else if (profile == "kafka4") {
    versions_ = {{1, 4, 11}, {2, 1, 5}, {3, 4, 8}, {8, 2, 7}, {9, 1, 5}, {10, 0, 2}, {18, 0, 2}};
  } else {
    throw std::invalid_argument("wire server profile '" + profile + "': legacy | kafka4 | ancient");
  }
  listen_fd_ = ::socket(AF_INET, SOCK_STREAM | SOCK_CLOEXEC, 0);
  if (listen_fd_ < 0) throw_errno("wire server socket");
  int one = 1;
  ::setsockopt(listen_fd_, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_port = htons(uint16_t(port));
  if (inet_pton(AF_INET, host.c_str(), &a.sin_addr) != 1) throw std::invalid_argument("wire server: IPv4 host");
  if (::bind(listen_fd_, reinterpret_cast<sockaddr*>(&a), sizeof(a)) != 0 || ::listen(listen_fd_, 128) != 0) {
    ::close(listen_fd_);
    throw_errno("wire server bind/listen");
  }
  socklen_t len = sizeof(a);
  ::getsockname(listen_fd_, reinterpret_cast<sockaddr*>(&a), &len);
  port_ = ntohs(a.sin_port);
  if (cluster_.empty()) cluster_.push_back(WireNode{node_, host_, port_});
}

WireServer::~WireServer() { stop(); }

void WireServer::start() {
  if (acceptor_.joinable()) return;
  acceptor_ = std::thread([this]() { accept_loop(); });
}

void WireServer::stop() {
  if (stop_.exchange(true)) return;
  if (listen_fd_ >= 0) {
    ::shutdown(listen_fd_, SHUT_RDWR);
    ::close(listen_fd_);
  }
  if (acceptor_.joinable()) acceptor_.join();
  {
    std::lock_guard<std::mutex> g(mu_);
    for (int fd : conns_) ::shutdown(fd, SHUT_RDWR);
  }
  for (auto& t : workers_)
    if (t.joinable()) t.join();
}

void WireServer::accept_loop() {
  name_thread("tk-wire-accept");
  while (!stop_.load()) {
    pollfd p{listen_fd_, POLLIN, 0};
    if (::poll(&p, 1, 100) <= 0) continue;
    const int fd = ::accept4(listen_fd_, nullptr, nullptr, SOCK_CLOEXEC);
    if (fd < 0) continue;
    int one = 1;
    ::setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
    int sndbuf = 8 << 20;
    ::setsockopt(fd, SOL_SOCKET, SO_SNDBUF, &sndbuf, sizeof(sndbuf));
    std::lock_guard<std::mutex> g(mu_);
    conns_.insert(fd);
    workers_.emplace_back([this, fd]() { serve(fd); });
  }
}

void WireServer::serve(int fd) {
  name_thread("tk-wire-serve");
  std::vector<uint8_t> req;
  while (!stop_.load()) {
    uint32_t n;
    if (!recv_exact(fd, &n, 4, stop_)) break;
    n = ntohl(n);
    if (n > (64u << 20)) break;
    req.resize(n);
    if (!recv_exact(fd, req.data(), n, stop_)) break;
    try {
      if (!handle(fd, req)) break;
    } catch (const std::exception&) {
      break;  // malformed request: a broker drops the connection
    }
  }
  {
    std::lock_guard<std::mutex> g(mu_);
    conns_.erase(fd);
  }
  ::close(fd);
}

bool WireServer::serves(int16_t key, int16_t ver) const {
  for (auto& v : versions_)
    if (v[0] == key) return ver >= v[1] && ver <= v[2] && (key != wire::kApiVersions || api_versions_);
  return false;
}

int32_t WireServer::leader(int32_t partition) const {
  return cluster_[size_t(partition) % cluster_.size()].node_id;
}

bool WireServer::handle(int fd, const std::vector<uint8_t>& req) {
  wire::Reader r(req.data(), req.size());
  const int16_t key = r.i16();
  const int16_t ver = r.i16();
  const int32_t corr = r.i32();
  r.str();  // client id
  requests_.fetch_add(1, std::memory_order_relaxed);
  Response out;
  wire::Writer& w = out.w;
  if (key == wire::kApiVersions) {
    if (!api_versions_) return false;  // predates ApiVersions: close
    const bool ok = serves(key, ver);
    w.i16(ok ? int16_t(0) : int16_t(wire::kUnsupportedVersion));  // v0 layout on a version error
    w.array(int32_t(versions_.size()));
    for (auto& a : versions_) {
      w.i16(a[0]);
      w.i16(a[1]);
      w.i16(a[2]);
    }
    if (ok && ver >= 1) w.i32(0);  // throttle
    return out.send(fd, corr, &bytes_);
  }
  if (!serves(key, ver)) return false;  // an unsupported version / API closes the connection, as Kafka does
  switch (key) {
    case wire::kMetadata: {
      std::vector<std::string> names;
      const int32_t nt = r.i32();
      if (nt < 0 || (nt == 0 && ver == 0)) {
        for (auto& t : b_->topics()) names.push_back(t.name);
      } else {
        for (int32_t i = 0; i < nt; ++i) names.push_back(r.str());
      }
      if (ver >= 3) w.i32(0);  // throttle
      w.array(int32_t(cluster_.size()));
      for (auto& n : cluster_) {
        w.i32(n.node_id);
        w.str(n.host);
        w.i32(n.port);
        if (ver >= 1) w.nullable_str_null();
      }
      if (ver >= 2) w.str("torchkafka-synthetic");  // cluster id
      if (ver >= 1) w.i32(cluster_[0].node_id);
      w.array(int32_t(names.size()));
      for (auto& name : names) {
        TopicInfo t;
        const bool ok = b_->find_topic(name, &t);
        w.i16(ok ? 0 : int16_t(wire::kUnknownTopicOrPartition));
        w.str(name);
        if (ver >= 1) w.i8(0);
        w.array(ok ? int32_t(t.n_partitions) : 0);
        for (uint32_t p = 0; ok && p < t.n_partitions; ++p) {
          const int32_t l = leader(int32_t(p));
          w.i16(0);
          w.i32(int32_t(p));
          w.i32(l);
          if (ver >= 7) w.i32(0);  // leader epoch
          w.array(1);
          w.i32(l);
          w.array(1);
          w.i32(l);
          if (ver >= 5) w.array(0);  // offline replicas
        }
        if (ver >= 8) w.i32(INT32_MIN);  // topic authorized operations: not requested
      }
      if (ver >= 8) w.i32(INT32_MIN);
      break;
    }
    case wire::kListOffsets: {
      r.i32();  // replica
      if (ver >= 2) {
        r.i8();    // isolation level
        w.i32(0);  // throttle
      }
      const int32_t nt = r.i32();
      w.array(nt);
      for (int32_t i = 0; i < nt; ++i) {
        const std::string name = r.str();
        TopicInfo t;
        const bool ok = b_->find_topic(name, &t);
        const int32_t np = r.i32();
        w.str(name);
        w.array(np);
        for (int32_t j = 0; j < np; ++j) {
          const int32_t p = r.i32();
          if (ver >= 4) r.i32();  // current leader epoch
          const int64_t ts = r.i64();
          if (ver == 0) r.i32();
          int16_t err = 0;
          int64_t off = -1;
          if (!ok || p < 0 || uint32_t(p) >= t.n_partitions) {
            err = wire::kUnknownTopicOrPartition;
          } else {
            const uint32_t pidx = t.first_pidx + uint32_t(p);
            if (ts == -1) off = b_->part(pidx).high_watermark.load();
            else if (ts == -2) off = b_->part(pidx).log_start_offset.load();
            else off = b_->offset_for_time(pidx, ts).first;
          }
          w.i32(p);
          w.i16(err);
          if (ver == 0) {
            w.array(off >= 0 ? 1 : 0);
            if (off >= 0) w.i64(off);
          } else {
            w.i64(-1);
            w.i64(off);
            if (ver >= 4) w.i32(0);  // leader epoch
          }
        }
      }
      break;
    }
    case wire::kFetch: {
      r.i32();  // replica
      const int32_t max_wait = r.i32();
      const int32_t min_bytes = r.i32();
      const int32_t max_bytes = r.i32();
      r.i8();   // isolation level
      if (ver >= 7) {
        r.i32();  // session id / epoch: every fetch is answered in full
        r.i32();
      }
      struct Req { std::string topic; TopicInfo t; bool ok; std::vector<std::tuple<int32_t, int64_t, int32_t>> parts; };
      std::vector<Req> reqs(size_t(std::max(0, r.i32())));
      for (auto& q : reqs) {
        q.topic = r.str();
        q.ok = b_->find_topic(q.topic, &q.t);
        const int32_t np = r.i32();
        for (int32_t j = 0; j < np; ++j) {
          const int32_t p = r.i32();
          if (ver >= 9) r.i32();  // current leader epoch
          const int64_t off = r.i64();
          if (ver >= 5) r.i64();  // log start offset (a follower's)
          const int32_t pmax = r.i32();
          q.parts.emplace_back(p, off, pmax);
        }
      }
      // long poll: wait (bounded) until some requested partition has data past its offset
      const auto deadline = std::chrono::steady_clock::now() + std::chrono::milliseconds(std::max(0, max_wait));
      while (min_bytes > 0 && !stop_.load()) {
        bool any = false;
        for (auto& q : reqs)
          for (auto& [p, off, pmax] : q.parts)
            if (q.ok && p >= 0 && uint32_t(p) < q.t.n_partitions && leader(p) == node_ &&
                b_->part(q.t.first_pidx + uint32_t(p)).high_watermark.load() != off)
              any = true;
        if (any || std::chrono::steady_clock::now() >= deadline) break;
        std::this_thread::sleep_for(std::chrono::microseconds(500));
      }
      w.i32(0);  // throttle
      if (ver >= 7) {
        w.i16(0);  // error
        w.i32(0);  // session id: none
      }
      w.array(int32_t(reqs.size()));
      int64_t budget = max_bytes;
      auto part_tail = [&](int64_t log_start) {  // the fields between last_stable_offset and the records
        if (ver >= 5) w.i64(log_start);
        w.i32(-1);                 // aborted transactions: null
        if (ver >= 11) w.i32(-1);  // preferred read replica
      };
      for (auto& q : reqs) {
        w.str(q.topic);
        w.array(int32_t(q.parts.size()));
        for (auto& [p, off, pmax] : q.parts) {
          w.i32(p);
          if (!q.ok || p < 0 || uint32_t(p) >= q.t.n_partitions || leader(p) != node_) {
            w.i16(q.ok && p >= 0 && uint32_t(p) < q.t.n_partitions ? int16_t(wire::kNotLeaderForPartition)
                                                                    : int16_t(wire::kUnknownTopicOrPartition));
            w.i64(-1);
            w.i64(-1);
            part_tail(-1);
            w.i32(-1);
            continue;
          }
          const uint32_t pidx = q.t.first_pidx + uint32_t(p);
          PartitionEntry& P = b_->part(pidx);
          const int64_t hw = P.high_watermark.load(std::memory_order_acquire);
          const int64_t start = P.log_start_offset.load(std::memory_order_acquire);
          if (off < start || off > hw) {
            w.i16(wire::kOffsetOutOfRange);
            w.i64(hw);
            w.i64(hw);
            part_tail(start);
            w.i32(-1);
            continue;
          }
          const uint8_t* data = nullptr;
          size_t n = 0;
          if (off < hw && budget > 0) {
            const IndexEntry* idx = b_->index_base(pidx);
            const uint64_t nb = P.n_batches.load(std::memory_order_acquire);
            const int64_t i = b_->find_batch(pidx, off, -1);
            const uint64_t icap = P.index_capacity;
            const uint64_t pos0 = idx[uint64_t(i) % icap].pos;
            const uint64_t cap = uint64_t(std::max<int64_t>(1, std::min<int64_t>(pmax, budget)));
            uint64_t end = pos0 + idx[uint64_t(i) % icap].size;  // at least one batch (KIP-74)
            for (uint64_t k = uint64_t(i) + 1; k < nb && idx[k % icap].pos + idx[k % icap].size - pos0 <= cap; ++k)
              end = idx[k % icap].pos + idx[k % icap].size;
            data = b_->log_base(pidx) + pos0;
            n = size_t(end - pos0);
            budget -= int64_t(n);
          }
          w.i16(0);
          w.i64(hw);
          w.i64(hw);
          part_tail(start);
          w.i32(int32_t(n));
          if (n) out.slice(data, n);  // sent from the mapped log
        }
      }
      break;
    }
    case wire::kFindCoordinator: {
      r.str();
      if (ver >= 1) {
        r.i8();    // key type
        w.i32(0);  // throttle
      }
      w.i16(0);
      if (ver >= 1) w.nullable_str_null();  // error message
      w.i32(cluster_[0].node_id);
      w.str(cluster_[0].host);
      w.i32(cluster_[0].port);
      break;
    }
    case wire::kOffsetCommit: {
      const std::string group = r.str();
      r.i32();
      r.str();
      if (ver >= 7) r.str();  // group instance id
      if (ver <= 4) r.i64();  // retention
      if (ver >= 3) w.i32(0);  // throttle
      const uint32_t g = b_->group_index(group, true);
      const int32_t nt = r.i32();
      w.array(nt);
      for (int32_t i = 0; i < nt; ++i) {
        const std::string name = r.str();
        TopicInfo t;
        const bool ok = b_->find_topic(name, &t);
        const int32_t np = r.i32();
        w.str(name);
        w.array(np);
        for (int32_t j = 0; j < np; ++j) {
          const int32_t p = r.i32();
          const int64_t off = r.i64();
          if (ver >= 6) r.i32();  // committed leader epoch
          const std::string meta = r.str();
          int16_t err = 0;
          if (!ok || p < 0 || uint32_t(p) >= t.n_partitions) {
            err = wire::kUnknownTopicOrPartition;
          } else {
            try {
              b_->commit(g, -1, 0, 0, {CommitEntry{t.first_pidx + uint32_t(p), off, meta}});
            } catch (const KafkaError&) {
              err = wire::kIllegalGeneration;  // a group with live members refuses a simple commit
            }
          }
          w.i32(p);
          w.i16(err);
        }
      }
      break;
    }
    case wire::kOffsetFetch: {
      const uint32_t g = b_->group_index(r.str(), true);
      if (ver >= 3) w.i32(0);  // throttle
      const int32_t nt = r.i32();
      std::vector<std::pair<std::string, std::vector<int32_t>>> reqs;
      if (nt < 0) {  // v2+: every topic
        for (auto& t : b_->topics()) {
          std::vector<int32_t> ps;
          for (uint32_t p = 0; p < t.n_partitions; ++p) ps.push_back(int32_t(p));
          reqs.emplace_back(t.name, ps);
        }
      } else {
        for (int32_t i = 0; i < nt; ++i) {
          std::string name = r.str();
          std::vector<int32_t> ps(size_t(std::max(0, r.i32())));
          for (auto& p : ps) p = r.i32();
          reqs.emplace_back(std::move(name), std::move(ps));
        }
      }
      w.array(int32_t(reqs.size()));
      for (auto& [name, ps] : reqs) {
        TopicInfo t;
        const bool ok = b_->find_topic(name, &t);
        w.str(name);
        w.array(int32_t(ps.size()));
        for (int32_t p : ps) {
          std::string meta;
          int64_t off = -1;
          int16_t err = 0;
          if (!ok || p < 0 || uint32_t(p) >= t.n_partitions) err = wire::kUnknownTopicOrPartition;
          else off = b_->committed(g, t.first_pidx + uint32_t(p), &meta);
          w.i32(p);
          w.i64(off);
          if (ver >= 5) w.i32(-1);  // committed leader epoch
          w.str(meta);
          w.i16(err);
        }
      }
      if (ver >= 2) w.i16(0);  // top-level error
      break;
    }
    default:
      return false;  // an API this broker does not serve: close, as Kafka does
  }
  return out.send(fd, corr, &bytes_);
}

}  // namespace tk
