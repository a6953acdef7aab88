// A native Kafka-protocol front end for the shared-memory broker (the fast twin of
// broker/wire_server.py).
//
// It answers the requests the native replicator and other consumers make -- ApiVersions,
// Metadata, ListOffsets, Fetch, FindCoordinator, OffsetCommit, OffsetFetch, at the versions of its
// profile ("legacy": v0/v1-era ranges; "kafka4": Kafka 4.x after KIP-896, up to Metadata v8,
// ListOffsets v5, Fetch v11, FindCoordinator v2, OffsetCommit v7, OffsetFetch v5; "ancient": no
// ApiVersions at all) -- with one thread per connection, and sends every Fetch response's record sets
// straight out of the mapped partition logs (writev from the page cache, no copy), so a cluster of
// these servers can feed the replicator at memory/NIC speed where the Python server is bound by
// its interpreter.  Partition p of a multi-node cluster is led by node p % nodes; a fetch sent to
// another node answers NOT_LEADER.  Reference counterpart: the Kafka cluster kafka-python talks to
// (kafka_dataset.py:21-22, 206).
#pragma once
#include <array>
#include <atomic>
#include <memory>
#include <mutex>
#include <set>
#include <string>
#include <thread>
#include <vector>

#include "broker.h"

namespace tk {

struct WireNode {
  int32_t node_id;
  std::string host;
  int32_t port;
};

class WireServer {
 public:
  // port 0: any free port.  cluster: every node (this one included); empty: a one-node cluster.
  WireServer(std::shared_ptr<Broker> broker, const std::string& host, int port, int32_t node_id,
             std::vector<WireNode> cluster, const std::string& profile = "legacy");
  ~WireServer();
  WireServer(const WireServer&) = delete;
  WireServer& operator=(const WireServer&) = delete;
  void start();
  void stop();
  int port() const { return port_; }
  uint64_t requests() const { return requests_.load(); }
  uint64_t bytes_sent() const { return bytes_.load(); }

 private:
  void accept_loop();
  void serve(int fd);
  bool handle(int fd, const std::vector<uint8_t>& req);
  int32_t leader(int32_t partition) const;
  bool serves(int16_t key, int16_t ver) const;

  std::shared_ptr<Broker> b_;
  std::string host_;
  int port_;
  int32_t node_;
  std::vector<WireNode> cluster_;
  std::vector<std::array<int16_t, 3>> versions_;  // {api key, min, max} served
  bool api_versions_ = true;                      // false: the "ancient" profile
  int listen_fd_ = -1;
  std::atomic<bool> stop_{false};
  std::thread acceptor_;
  std::mutex mu_;
  std::set<int> conns_;
  std::vector<std::thread> workers_;
  std::atomic<uint64_t> requests_{0}, bytes_{0};
};

}  // namespace tk
