// `torchkafka_amd._tkcore` bindings: the Kafka wire-protocol client, test server and replicator (KafkaBridge).
#include "bindings_common.h"

namespace tkbind {

void bind_wire(py::module_& m) {
  // ---- Kafka wire protocol (kafka_wire.h) and the cluster -> local log replicator (replicator.h)
  py::class_<wire::Client>(m, "WireClient")
      .def(py::init([](const std::string& bootstrap, const std::string& client_id, int timeout_ms, py::dict security) {
             return std::make_unique<wire::Client>(bootstrap, client_id, timeout_ms, to_security(security));
           }),
           py::arg("bootstrap"), py::arg("client_id") = "torchkafka", py::arg("timeout_ms") = 30000,
           py::arg("security") = py::dict())
      .def("metadata",
           [](wire::Client& c, const std::string& topic) {
             wire::TopicMeta t;
             {
               py::gil_scoped_release nogil;
               t = c.metadata(topic);
             }
             py::list parts;
             for (auto& p : t.partitions) parts.append(py::make_tuple(p.partition, p.leader, p.error));
             return py::make_tuple(t.error, parts);
           })
      .def("brokers",
           [](wire::Client& c) {
             py::list l;
             for (auto& b : c.brokers()) l.append(py::make_tuple(b.node_id, b.host, b.port));
             return l;
           })
      .def("list_offsets", &wire::Client::list_offsets, py::call_guard<py::gil_scoped_release>())
      .def("offset_fetch", &wire::Client::offset_fetch, py::call_guard<py::gil_scoped_release>())
      .def("offset_commit", &wire::Client::offset_commit, py::arg("group"), py::arg("topic"), py::arg("offsets"),
           py::arg("metadata") = "", py::arg("generation") = -1, py::arg("member_id") = "",
           py::call_guard<py::gil_scoped_release>())
      .def("heartbeat", &wire::Client::heartbeat, py::call_guard<py::gil_scoped_release>())
      .def("leave_group", &wire::Client::leave_group, py::call_guard<py::gil_scoped_release>())
      .def_static("parse_bootstrap", &wire::Client::parse_bootstrap);

  py::class_<WireServer>(m, "WireServer")
      .def(py::init([](std::shared_ptr<Broker> b, const std::string& host, int port, int32_t node_id,
                       std::vector<std::tuple<int32_t, std::string, int32_t>> cluster, const std::string& profile) {
             std::vector<WireNode> nodes;
             for (auto& [id, h, p] : cluster) nodes.push_back(WireNode{id, h, p});
             return std::make_unique<WireServer>(std::move(b), host, port, node_id, std::move(nodes), profile);
           }),
           py::arg("broker"), py::arg("host") = "127.0.0.1", py::arg("port") = 0, py::arg("node_id") = 0,
           py::arg("cluster") = std::vector<std::tuple<int32_t, std::string, int32_t>>(),
           py::arg("profile") = "legacy")
      .def("start", &WireServer::start)
      .def("stop", &WireServer::stop, py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("port", &WireServer::port)
      .def_property_readonly("requests", &WireServer::requests)
      .def_property_readonly("bytes_sent", &WireServer::bytes_sent);

  py::class_<Replicator>(m, "Replicator")
      .def(py::init([](std::shared_ptr<Broker> local, const std::string& bootstrap, const std::string& topic,
                       const std::string& group, std::vector<int32_t> partitions, const std::string& reset,
                       int32_t max_wait_ms, int32_t max_bytes, int32_t partition_max_bytes, int32_t timeout_ms,
                       int64_t max_lag_bytes, int32_t commit_interval_ms, int32_t fetchers, uint64_t log_capacity,
                       uint64_t index_capacity, const std::string& client_id, bool release_consumed,
                       uint64_t release_bytes, uint64_t release_step, uint64_t ring_bytes, py::dict security,
                       bool subscribe, int32_t session_timeout_ms, int32_t heartbeat_interval_ms,
                       std::vector<std::string> assignors, int32_t rebalance_timeout_ms) {
             ReplicaConfig c;
             for (auto& a : assignors)
               if (a != "range" && a != "roundrobin")
                 throw std::invalid_argument("partition_assignment_strategy: '" + a + "' (range | roundrobin)");
             if (!assignors.empty()) c.assignors = std::move(assignors);
             c.subscribe = subscribe;
             c.session_timeout_ms = session_timeout_ms;
             c.heartbeat_interval_ms = heartbeat_interval_ms;
             c.rebalance_timeout_ms = rebalance_timeout_ms;
             c.bootstrap = bootstrap;
             c.topic = topic;
             c.group = group;
             c.partitions = std::move(partitions);
             c.auto_offset_reset = reset;
             c.max_wait_ms = max_wait_ms;
             c.max_bytes = max_bytes;
             c.partition_max_bytes = partition_max_bytes;
             c.timeout_ms = timeout_ms;
             c.max_lag_bytes = max_lag_bytes;
             c.commit_interval_ms = commit_interval_ms;
             c.fetchers = fetchers;
             c.log_capacity = log_capacity;
             c.index_capacity = index_capacity;
             c.client_id = client_id;
             c.release_consumed = release_consumed;
             c.release_bytes = release_bytes;
             c.release_step = release_step;
             c.ring_bytes = ring_bytes;
             c.security = to_security(security);
             return std::make_unique<Replicator>(std::move(local), c);
           }),
           py::arg("local"), py::arg("bootstrap"), py::arg("topic"), py::arg("group") = "",
           py::arg("partitions") = std::vector<int32_t>(), py::arg("auto_offset_reset") = "earliest",
           py::arg("max_wait_ms") = 100, py::arg("max_bytes") = 64 << 20, py::arg("partition_max_bytes") = 8 << 20,
           py::arg("timeout_ms") = 30000, py::arg("max_lag_bytes") = int64_t(1) << 30,
           py::arg("commit_interval_ms") = 5, py::arg("fetchers") = 0, py::arg("log_capacity") = 0,
           py::arg("index_capacity") = 0, py::arg("client_id") = "torchkafka-replicator",
           py::arg("release_consumed") = true, py::arg("release_bytes") = uint64_t(256) << 20,
           py::arg("release_step") = uint64_t(1) << 30, py::arg("ring_bytes") = uint64_t(0),
           py::arg("security") = py::dict(), py::arg("subscribe") = false, py::arg("session_timeout_ms") = 10000,
           py::arg("heartbeat_interval_ms") = 3000, py::arg("assignors") = std::vector<std::string>{"range"},
           py::arg("rebalance_timeout_ms") = 0)
      .def("start", &Replicator::start, py::call_guard<py::gil_scoped_release>())
      .def("stop", &Replicator::stop, py::arg("flush") = true, py::call_guard<py::gil_scoped_release>())
      .def("flush_commits", &Replicator::flush_commits, py::call_guard<py::gil_scoped_release>())
      .def("commit_sync", &Replicator::commit_sync, py::arg("timeout_ms"), py::call_guard<py::gil_scoped_release>())
      .def("set_oauth_token", &Replicator::set_oauth_token, py::arg("token"), py::arg("extensions") = "")
      .def("take_forward_ns", &Replicator::take_forward_ns)
      .def("wait_caught_up", &Replicator::wait_caught_up, py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("running", &Replicator::running)
      .def_property_readonly("errors", &Replicator::errors)
      .def_property_readonly("first_pidx", &Replicator::first_pidx)
      .def_property_readonly("n_partitions", &Replicator::n_partitions)
      .def_property_readonly("member_id", &Replicator::member_id)
      .def_property_readonly("generation", &Replicator::generation)
      .def_property_readonly("assignment", &Replicator::assignment)
      .def_property_readonly("fenced", &Replicator::fenced)
      .def_property_readonly("assignment_epoch", &Replicator::assignment_epoch)
      .def_property_readonly("rebalances", &Replicator::rebalances)
      .def_property_readonly("out_of_order", &Replicator::out_of_order)
      .def("assignment_epochs", &Replicator::assignment_epochs,
           "[(partition, epoch at which it was (re)assigned)] of the partitions owned now")
      .def_property_readonly("fetch_threads", &Replicator::fetch_threads)
      .def_property_readonly("fetch_wait_ns", &Replicator::fetch_wait_ns)
      .def_property_readonly("inflate_threads", &Replicator::inflate_threads)
      .def("last_error", &Replicator::last_error)
      .def("stats", [](Replicator& r) {
        py::list l;
        for (auto& s : r.stats()) {
          py::dict d;
          d["partition"] = s.partition;
          d["pidx"] = s.pidx;
          d["start_offset"] = s.start_offset;
          d["fetch_offset"] = s.fetch_offset;
          d["remote_hw"] = s.remote_hw;
          d["forwarded"] = s.forwarded;
          d["bytes"] = s.bytes;
          d["batches"] = s.batches;
          d["control_batches"] = s.control_batches;
          d["fetches"] = s.fetches;
          d["throttled"] = s.throttled;
          d["released"] = s.released;
          d["owned"] = s.owned;
          d["wire_bytes"] = s.wire_bytes;
          d["recv_ns"] = s.recv_ns;
          d["ingest_ns"] = s.ingest_ns;
          d["inflate_ns"] = s.inflate_ns;
          d["inflated_batches"] = s.inflated_batches;
          d["inflated_bytes"] = s.inflated_bytes;
          l.append(d);
        }
        return l;
      });

}

}  // namespace tkbind
