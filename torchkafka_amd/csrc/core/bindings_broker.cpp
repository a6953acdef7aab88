// `torchkafka_amd._tkcore` bindings: the synthetic broker (topics, logs, groups, committed offsets, faults).
#include "bindings_common.h"

namespace tkbind {

void bind_broker(py::module_& m) {
  // ---- broker
  py::class_<Broker, std::shared_ptr<Broker>>(m, "Broker")
      .def(py::init([](const std::string& url, bool create, uint32_t max_topics, uint32_t max_partitions,
                       uint32_t max_groups, uint64_t log_capacity, uint64_t index_capacity, uint32_t rebalance_delay_ms) {
             BrokerConfig c;
             c.max_topics = max_topics;
             c.max_partitions = max_partitions;
             c.max_groups = max_groups;
             c.default_log_capacity = log_capacity;
             c.default_index_capacity = index_capacity;
             c.group_initial_rebalance_delay_ms = rebalance_delay_ms;
             return std::make_shared<Broker>(url, create, c);
           }),
           py::arg("url"), py::arg("create") = false, py::arg("max_topics") = 256, py::arg("max_partitions") = 4096,
           py::arg("max_groups") = 64, py::arg("log_capacity") = uint64_t(256) << 20,
           py::arg("index_capacity") = uint64_t(1) << 20, py::arg("group_initial_rebalance_delay_ms") = 100)
      .def_static("url_to_dir", &Broker::url_to_dir)
      .def_property_readonly("dir", &Broker::dir)
      .def_property_readonly("group_initial_rebalance_delay_ms",
                             [](Broker& b) { return b.meta().group_initial_rebalance_delay_ms; })
      .def("create_topic",
           [](Broker& b, const std::string& name, uint32_t n, uint64_t cap, uint64_t icap) {
             TopicInfo t = b.create_topic(name, n, cap, icap);
             return py::make_tuple(t.index, t.n_partitions, t.first_pidx);
           },
           py::arg("name"), py::arg("num_partitions"), py::arg("log_capacity") = 0, py::arg("index_capacity") = 0)
      .def("find_topic",
           [](Broker& b, const std::string& name) -> py::object {
             TopicInfo t;
             if (!b.find_topic(name, &t)) return py::none();
             return py::make_tuple(t.index, t.n_partitions, t.first_pidx);
           })
      .def("topics",
           [](Broker& b) {
             py::list l;
             for (auto& t : b.topics()) l.append(py::make_tuple(t.name, t.index, t.n_partitions, t.first_pidx));
             return l;
           })
      .def("partition_of",
           [](Broker& b, uint32_t pidx) {
             auto& P = b.part(pidx);
             return py::make_tuple(P.topic_index, P.partition);
           })
      .def("high_watermark", [](Broker& b, uint32_t p) { return b.part(p).high_watermark.load(); })
      .def("log_start_offset", [](Broker& b, uint32_t p) { return b.part(p).log_start_offset.load(); })
      .def("log_bytes", [](Broker& b, uint32_t p) { return b.part(p).log_end_pos.load(); })
      .def("read_log",
           [](Broker& b, uint32_t p, uint64_t off, uint64_t n) {
             if (off + n > b.part(p).log_end_pos.load()) throw std::out_of_range("read_log beyond the log end");
             return py::bytes(reinterpret_cast<const char*>(b.log_base(p)) + off, n);
           },
           py::arg("pidx"), py::arg("offset"), py::arg("n"), "raw bytes of a partition log (tests, tools)")
      .def("offset_for_time", &Broker::offset_for_time, py::arg("pidx"), py::arg("timestamp"))
      .def("partition_stats",
           [](Broker& b, uint32_t p) {
             auto& P = b.part(p);
             py::dict d;
             d["fetch_calls"] = P.fetch_calls.load();
             d["bytes_fetched"] = P.bytes_fetched.load();
             d["records_produced"] = P.records_produced.load();
             d["batches"] = P.n_batches.load();
             d["log_bytes"] = P.log_end_pos.load();
             return d;
           })
      .def(
          "append",
          [](Broker& b, uint32_t pidx, std::vector<py::object> values, std::vector<py::object> keys,
             std::vector<int64_t> timestamps, std::vector<py::object> headers) {
            std::deque<std::string> keep;
            std::vector<std::vector<HeaderView>> hkeep;
            auto recs = to_records(values, keys, timestamps, headers, keep, hkeep);
            py::gil_scoped_release nogil;
            return b.append(pidx, recs.data(), recs.size());
          },
          py::arg("pidx"), py::arg("values"), py::arg("keys"), py::arg("timestamps"), py::arg("headers"))
      .def(
          "fill_synthetic",
          [](Broker& b, std::vector<uint32_t> pidxs, int64_t n, int kind, int64_t a, int64_t bb, uint32_t rpb,
             uint64_t seed, int threads, bool keyed) {
            py::gil_scoped_release nogil;
            b.fill_synthetic(pidxs, n, kind, a, bb, rpb, seed, threads, keyed);
          },
          py::arg("pidxs"), py::arg("n_records"), py::arg("kind"), py::arg("size_a"), py::arg("size_b") = 0,
          py::arg("records_per_batch") = 64, py::arg("seed") = 0, py::arg("threads") = 1, py::arg("keyed") = false)
      .def("delete_records", &Broker::delete_records)
      .def("read_batches",
           [](Broker& b, uint32_t p, int64_t offset, uint64_t max_bytes) {
             // Whole RecordBatches from the one holding `offset` (or the next after a gap), at most
             // max_bytes but at least one batch (a Kafka Fetch response's record set, KIP-74).
             PartitionEntry& P = b.part(p);
             const int64_t hw = P.high_watermark.load(std::memory_order_acquire);
             const int64_t start = P.log_start_offset.load(std::memory_order_acquire);
             if (offset < start || offset > hw) throw OffsetOutOfRange("offset " + std::to_string(offset) + " out of range");
             if (offset == hw) return py::make_tuple(py::bytes(), hw, start);
             const IndexEntry* idx = b.index_base(p);
             const uint64_t nb = P.n_batches.load(std::memory_order_acquire);
             int64_t i = b.find_batch(p, offset, -1);
             const uint64_t icap = P.index_capacity;
             const uint64_t pos0 = idx[uint64_t(i) % icap].pos;
             uint64_t end = pos0 + idx[uint64_t(i) % icap].size;
             for (uint64_t j = uint64_t(i) + 1; j < nb && idx[j % icap].pos + idx[j % icap].size - pos0 <= max_bytes; ++j)
               end = idx[j % icap].pos + idx[j % icap].size;
             return py::make_tuple(py::bytes(reinterpret_cast<const char*>(b.log_base(p)) + pos0, end - pos0), hw, start);
           },
           py::arg("pidx"), py::arg("offset"), py::arg("max_bytes"))
      .def("batch_range",
           [](Broker& b, uint32_t p, int64_t offset, uint64_t max_bytes) -> py::tuple {
             // read_batches without the copy: (log byte position, bytes, high watermark, log start)
             PartitionEntry& P = b.part(p);
             const int64_t hw = P.high_watermark.load(std::memory_order_acquire);
             const int64_t start = P.log_start_offset.load(std::memory_order_acquire);
             if (offset < start || offset > hw) throw OffsetOutOfRange("offset " + std::to_string(offset) + " out of range");
             if (offset == hw) return py::make_tuple(uint64_t(0), uint64_t(0), hw, start);
             const IndexEntry* idx = b.index_base(p);
             const uint64_t nb = P.n_batches.load(std::memory_order_acquire);
             const int64_t i = b.find_batch(p, offset, -1);
             const uint64_t icap = P.index_capacity;
             const uint64_t pos0 = idx[uint64_t(i) % icap].pos;
             uint64_t end = pos0 + idx[uint64_t(i) % icap].size;
             for (uint64_t j = uint64_t(i) + 1; j < nb && idx[j % icap].pos + idx[j % icap].size - pos0 <= max_bytes; ++j)
               end = idx[j % icap].pos + idx[j % icap].size;
             return py::make_tuple(pos0, end - pos0, hw, start);
           },
           py::arg("pidx"), py::arg("offset"), py::arg("max_bytes"))
      .def("log_view",
           [](Broker& b, uint32_t p) {
             // the whole mapped log of a partition, read-only (the wire server sends from it)
             return py::memoryview::from_memory(reinterpret_cast<const void*>(b.log_base(p)),
                                                py::ssize_t(b.part(p).log_capacity));
           },
           py::keep_alive<0, 1>())
      .def("reset_empty", &Broker::reset_empty)
      .def_property("flags", &Broker::flags, &Broker::set_flags)
      .def("ingest_bytes",
           [](Broker& b, uint32_t p, py::bytes data, int64_t from_offset, bool keep_control) {
             std::string s = data;
             uint64_t avail = 0;
             uint8_t* tail = b.log_tail(p, &avail);
             if (s.size() > avail) throw KafkaError("ingest_bytes: log full");
             std::memcpy(tail, s.data(), s.size());
             Broker::Ingested in = b.ingest(p, s.size(), from_offset, keep_control);
             py::dict d;
             d["consumed"] = in.consumed;
             d["kept"] = in.kept;
             d["kept_bytes"] = in.kept_bytes;
             d["control"] = in.control;
             d["inflated"] = in.inflated;
             d["next_offset"] = in.next_offset;
             return d;
           },
           py::arg("pidx"), py::arg("data"), py::arg("from_offset") = -1, py::arg("keep_control") = false)
      .def("copy_compressed",
           [](Broker& b, std::vector<uint32_t> src, std::vector<uint32_t> dst, int codec, int level,
              int64_t max_records, int threads, int64_t start_record) {
             // Appends the batches of partitions `src` whose records lie in [start_record,
             // max_records) of each (-1: to the end), compressed with `codec` batch by batch as a
             // producer would (attributes, length and CRC rewritten; codec 0: copied as they are),
             // to the partitions `dst`: the benchmarks' compressed topics.
             if (src.size() != dst.size()) throw std::invalid_argument("copy_compressed: src and dst differ in length");
             std::atomic<size_t> next{0};
             std::atomic<uint64_t> raw{0}, packed{0}, batches{0};
             std::mutex err_mu;
             std::exception_ptr err;
             auto work = [&]() {
               std::vector<uint8_t> out;
               try {
                 for (size_t j; (j = next.fetch_add(1)) < src.size();) {
                   PartitionEntry& P = b.part(src[j]);
                   const uint64_t nb = P.n_batches.load(std::memory_order_acquire);
                   const uint64_t icap = P.index_capacity;
                   const IndexEntry* idx = b.index_base(src[j]);
                   const uint8_t* log = b.log_base(src[j]);
                   const int64_t start = P.log_start_offset.load(std::memory_order_acquire);
                   for (uint64_t i = P.first_batch.load(std::memory_order_acquire); i < nb; ++i) {
                     const IndexEntry& e = idx[i % icap];
                     if (max_records >= 0 && e.base_offset >= start + max_records) break;
                     if (e.base_offset < start + start_record) continue;
                     const uint8_t* bt = log + e.pos;
                     if (codec == kCodecNone) {
                       out.assign(bt, bt + e.size);
                     } else {
                       out.assign(bt, bt + kBatchHeaderBytes);
                       compress(codec, bt + kBatchHeaderBytes, e.size - kBatchHeaderBytes, out, level);
                       const uint32_t be_len = __builtin_bswap32(uint32_t(out.size() - 12));
                       std::memcpy(out.data() + kBatchLengthOffset, &be_len, 4);
                       out[kBatchAttrOffset + 1] = uint8_t((out[kBatchAttrOffset + 1] & ~7) | (codec & 7));
                       const uint32_t be_crc =
                           __builtin_bswap32(crc32c(out.data() + kBatchAttrOffset, out.size() - kBatchAttrOffset));
                       std::memcpy(out.data() + kBatchCrcOffset, &be_crc, 4);
                     }
                     uint64_t avail = 0;
                     uint8_t* tail = b.log_tail(dst[j], &avail);
                     if (out.size() > avail) throw KafkaError("copy_compressed: destination log full");
                     std::memcpy(tail, out.data(), out.size());
                     b.ingest(dst[j], out.size(), -1, true);
                     raw += e.size;
                     packed += out.size();
                     ++batches;
                   }
                 }
               } catch (...) {
                 std::lock_guard<std::mutex> g(err_mu);
                 if (!err) err = std::current_exception();
               }
             };
             {
               py::gil_scoped_release nogil;
               std::vector<std::thread> ts;
               for (int t = 0; t < std::max(1, std::min<int>(threads, int(src.size()))); ++t) ts.emplace_back(work);
               for (auto& t : ts) t.join();
             }
             if (err) std::rethrow_exception(err);
             py::dict d;
             d["raw_bytes"] = raw.load();
             d["compressed_bytes"] = packed.load();
             d["batches"] = batches.load();
             return d;
           },
           py::arg("src"), py::arg("dst"), py::arg("codec"), py::arg("level") = 0, py::arg("max_records") = -1,
           py::arg("threads") = 8, py::arg("start_record") = 0)
      .def("position_of", &Broker::position_of)
      .def("ring_bytes", [](Broker& b, uint32_t p) { return b.part(p).ring_bytes.load(); })
      .def("first_batch", [](Broker& b, uint32_t p) { return b.part(p).first_batch.load(); })
      .def("group_index", &Broker::group_index, py::arg("group"), py::arg("create") = true)
      .def("group_name", &Broker::group_name)
      .def("join_group", &Broker::join_group)
      .def("leave_group", &Broker::leave_group)
      .def("rejoin_group", &Broker::rejoin_group)
      .def("member_id", &Broker::member_id)
      .def("poll_group",
           [](Broker& b, uint32_t g, int slot, uint64_t mid) {
             GroupView v = b.poll_group(g, slot, mid);
             return py::make_tuple(v.generation, v.state, v.member_active, v.assignment);
           })
      .def("commit",
           [](Broker& b, uint32_t g, int slot, uint64_t mid, uint32_t gen,
              std::vector<std::tuple<uint32_t, int64_t, std::string>> entries) {
             std::vector<CommitEntry> es;
             es.reserve(entries.size());
             for (auto& e : entries) es.push_back(CommitEntry{std::get<0>(e), std::get<1>(e), std::get<2>(e)});
             b.commit(g, slot, mid, gen, es);
           })
      .def("commit_positions",
           [](Broker& b, uint32_t g, int slot, uint64_t mid, uint32_t gen, py::list assignment, py::dict positions) {
             // The consumer's default commit: every assigned partition at its consumed position
             // (0 when nothing was consumed yet), without building Python entry tuples.
             std::vector<CommitEntry> es;
             es.reserve(py::len(assignment));
             for (py::handle h : assignment) {
               PyObject* v = PyDict_GetItem(positions.ptr(), h.ptr());  // borrowed
               const int64_t off = v ? PyLong_AsLongLong(v) : 0;
               if (off == -1 && PyErr_Occurred()) throw py::error_already_set();
               es.push_back(CommitEntry{h.cast<uint32_t>(), off, std::string()});
             }
             if (es.empty()) return;
             b.commit(g, slot, mid, gen, es);
           })
      .def("committed",
           [](Broker& b, uint32_t g, uint32_t pidx) {
             std::string meta;
             int64_t off = b.committed(g, pidx, &meta);
             return py::make_tuple(off, py::str(meta));
           })
      .def("commit_count", &Broker::commit_count)
      .def("inject_commit_failures", &Broker::inject_commit_failures)
      .def("reset_group_offsets", &Broker::reset_group_offsets)
      .def("set_fetch_delay", &Broker::set_fetch_delay)
      .def("inject_fetch_errors", &Broker::inject_fetch_errors);

}

}  // namespace tkbind
