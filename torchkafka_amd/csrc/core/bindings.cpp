// pybind11 bindings of the host native core: module `torchkafka_amd._tkcore`.
// No HIP here (imported in forked workers); device work lives in `_tkhip`.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <deque>

#include "broker.h"
#include "codecs.h"
#include "consumer.h"
#include "crc32c.h"
#include "lockstep.h"
#include "kafka_wire.h"
#include "record_batch.h"
#include "replicator.h"
#include "ring.h"
#include "wire_server.h"

namespace py = pybind11;
using namespace tk;

namespace {

py::object bytes_or_none(const uint8_t* p, int32_t len) {
  if (!p || len < 0) return py::none();
  return py::bytes(reinterpret_cast<const char*>(p), size_t(len));
}

py::tuple record_tuple(const RecordView& r, int ts_type) {
  py::list headers;
  if (r.header_count > 0) {
    for (const auto& h : parse_headers(r)) {
      headers.append(py::make_tuple(py::str(reinterpret_cast<const char*>(h.key), size_t(h.key_len)),
                                    bytes_or_none(h.value, h.value_len)));
    }
  }
  return py::make_tuple(r.offset, r.timestamp, ts_type, bytes_or_none(r.key, r.key_len),
                        bytes_or_none(r.value, r.value_len), headers, py::none(), r.key_len, r.value_len,
                        r.header_bytes);
}

struct PyFetcher {
  Fetcher f;
  size_t rr = 0;
  bool last_reassigned = false;  // the last fill_slot returned early: the watched assignment changed
  py::list watched;              // the Replicators whose epochs f watches (kept alive here)
  PyFetcher(std::shared_ptr<Broker> b, bool crc) : f(std::move(b), crc) {}
};

struct PyRing {
  std::unique_ptr<Ring> r;
  std::vector<uint32_t> cursor;
  std::vector<uint8_t> done;
  uint32_t rr = 0;
  explicit PyRing(std::unique_ptr<Ring> ring) : r(std::move(ring)) {
    cursor.assign(r->n_workers(), 0);
    done.assign(r->n_workers(), 0);
  }
};

std::vector<RecordIn> to_records(const std::vector<py::object>& values, const std::vector<py::object>& keys,
                                 const std::vector<int64_t>& timestamps, const std::vector<py::object>& headers,
                                 std::deque<std::string>& keep, std::vector<std::vector<HeaderView>>& hkeep) {
  // `keep` is a deque: growing it never moves the strings that RecordIn/HeaderView point into
  // (a vector would, and short strings keep their bytes inline).
  const size_t n = values.size();
  if (keys.size() != n || timestamps.size() != n || headers.size() != n)
    throw std::invalid_argument("values/keys/timestamps/headers length mismatch");
  hkeep.resize(n);
  std::vector<RecordIn> recs(n);
  auto hold = [&](const py::object& o, const uint8_t** p, int32_t* len) {
    if (o.is_none()) { *p = nullptr; *len = -1; return; }
    keep.emplace_back(o.cast<std::string>());
    *p = reinterpret_cast<const uint8_t*>(keep.back().data());
    *len = int32_t(keep.back().size());
  };
  for (size_t i = 0; i < n; ++i) {
    RecordIn& r = recs[i];
    r.timestamp = timestamps[i];
    hold(keys[i], &r.key, &r.key_len);
    hold(values[i], &r.value, &r.value_len);
    r.headers = nullptr;
    r.header_count = 0;
    if (!headers[i].is_none()) {
      for (auto item : headers[i].cast<py::list>()) {
        auto t = item.cast<py::tuple>();
        HeaderView h;
        keep.emplace_back(t[0].cast<std::string>());
        h.key = reinterpret_cast<const uint8_t*>(keep.back().data());
        h.key_len = int32_t(keep.back().size());
        hold(py::reinterpret_borrow<py::object>(t[1]), &h.value, &h.value_len);
        hkeep[i].push_back(h);
      }
      r.headers = hkeep[i].data();
      r.header_count = int32_t(hkeep[i].size());
    }
  }
  return recs;
}

// Lockstep transport over a Python all-reduce(MIN) of three ints (gloo in the CPU tests).
class PyLockstepTransport : public LockstepTransport {
 public:
  explicit PyLockstepTransport(py::function fn) : fn_(std::move(fn)) {}
  int issue(int64_t a, int64_t b, int64_t c) override {
    py::tuple r = fn_(a, b, c);
    const int t = int(next_++ % 64);
    for (int k = 0; k < 3; ++k) res_[t][k] = r[size_t(k)].cast<int64_t>();
    return t;
  }
  void wait(int t, int64_t out[3]) override {
    for (int k = 0; k < 3; ++k) out[k] = res_[t][k];
  }

 private:
  py::function fn_;
  uint64_t next_ = 0;
  int64_t res_[64][3];
};

// A rank's data path scripted in Python: an object with staged(), all_done(), wait_data(ms).
class PyLockstepSource : public LockstepSource {
 public:
  explicit PyLockstepSource(py::object o) : o_(std::move(o)) {}
  int64_t staged() override { return o_.attr("staged")().cast<int64_t>(); }
  bool all_done() override { return o_.attr("all_done")().cast<bool>(); }
  int wait_data(int64_t timeout_ms) override { return o_.attr("wait_data")(timeout_ms).cast<int>(); }

 private:
  py::object o_;
};

// kafka-python-named security settings -> wire::Security
wire::Security to_security(const py::dict& d) {
  wire::Security s;
  auto get = [&](const char* k, std::string* out) {
    if (d.contains(k) && !d[k].is_none()) *out = d[k].cast<std::string>();
  };
  get("security_protocol", &s.protocol);
  get("ssl_cafile", &s.cafile);
  get("ssl_certfile", &s.certfile);
  get("ssl_keyfile", &s.keyfile);
  get("sasl_mechanism", &s.sasl_mechanism);
  get("sasl_plain_username", &s.username);
  get("sasl_plain_password", &s.password);
  if (d.contains("ssl_check_hostname") && !d["ssl_check_hostname"].is_none())
    s.check_hostname = d["ssl_check_hostname"].cast<bool>();
  if (d.contains("sasl_oauth_token") && !d["sasl_oauth_token"].is_none()) {
    // resolved from sasl_oauth_token_provider in Python (broker/bridge.py security_config): no
    // native thread ever calls back into the interpreter
    s.oauth = std::make_shared<wire::OAuthToken>();
    s.oauth->token = d["sasl_oauth_token"].cast<std::string>();
    if (d.contains("sasl_oauth_extensions") && !d["sasl_oauth_extensions"].is_none())
      s.oauth->extensions = d["sasl_oauth_extensions"].cast<std::string>();
  }
  return s;
}

py::list wms_to_list(const std::vector<Watermark>& w) {
  py::list l;
  for (const auto& x : w) l.append(py::make_tuple(x.pidx, x.first_offset, x.next_offset, x.count));
  return l;
}

}  // namespace

#ifndef TK_SOURCES_SHA
#define TK_SOURCES_SHA "unversioned"  // built outside _build.py
#endif
// The sha of the sources this binary was built from (_build.sources_sha): _build.embedded_sha finds it
// in the file, ops.build_info() compares it with the tree.
__attribute__((used)) static const char kSourcesSha[] = "TKSRCSHA:" TK_SOURCES_SHA;

PYBIND11_MODULE(_tkcore, m) {
  m.attr("SOURCES_SHA") = std::string(kSourcesSha + 9);
  m.doc() = "torchkafka_amd host native core: RecordBatch codec, shm broker, fetcher, packers, slot ring";

  static py::exception<KafkaError> kafka_error(m, "KafkaError", PyExc_RuntimeError);
  static py::exception<CommitFailed> commit_failed(m, "CommitFailedError", kafka_error.ptr());
  static py::exception<CorruptRecord> corrupt(m, "CorruptRecordException", kafka_error.ptr());
  static py::exception<OffsetOutOfRange> oor(m, "OffsetOutOfRangeError", kafka_error.ptr());
  static py::exception<InjectedFetchError> fetch_err(m, "InjectedFetchError", kafka_error.ptr());
  py::register_exception_translator([](std::exception_ptr p) {
    try {
      if (p) std::rethrow_exception(p);
    } catch (const CommitFailed& e) {
      py::set_error(commit_failed, e.what());
    } catch (const CorruptRecord& e) {
      py::set_error(corrupt, e.what());
    } catch (const OffsetOutOfRange& e) {
      py::set_error(oor, e.what());
    } catch (const InjectedFetchError& e) {
      py::set_error(fetch_err, e.what());
    } catch (const KafkaError& e) {
      py::set_error(kafka_error, e.what());
    }
  });

  // ---- codec
  m.def("crc32c", [](py::bytes b) {
    std::string s = b;
    return crc32c(s.data(), s.size());
  });
  m.def("crc32c_hw", &crc32c_hw);
  m.def("decompress", [](int codec, py::bytes b) {
    std::string s = b;
    std::vector<uint8_t> out;
    decompress(codec, reinterpret_cast<const uint8_t*>(s.data()), s.size(), out);
    return py::bytes(reinterpret_cast<const char*>(out.data()), out.size());
  });
  m.def("zstd_available", &zstd_available);
  m.def("client_versions", []() {
    std::map<int16_t, std::pair<int16_t, int16_t>> out;
    for (auto& [k, r] : wire::client_versions()) out[k] = {r.min, r.max};
    return out;
  }, "{api key: (min, max)} request versions the native Kafka client implements");
  // Kafka's range assignor over (member id, subscribed topics): {member: {topic: [partitions]}}
  m.def("range_assign", [](const std::vector<std::pair<std::string, std::vector<std::string>>>& members,
                           const std::map<std::string, int32_t>& counts, bool rr) {
    std::vector<std::pair<std::string, std::string>> ms;
    for (auto& [m, topics] : members) ms.emplace_back(m, wire::encode_subscription(topics));
    auto out = rr ? wire::roundrobin_assign(ms, counts) : wire::range_assign(ms, counts);
    std::map<std::string, wire::Assignment> back;
    for (auto& [m, a] : out) back[m] = wire::decode_assignment(wire::encode_assignment(a));
    return back;
  }, py::arg("members"), py::arg("counts"), py::arg("roundrobin") = false);
  m.def("crc32c_fold", &crc32c_fold);
  m.def("crc32c_shift_raw", &crc32c_shift_raw, py::arg("raw"), py::arg("n_bytes"));
  m.def(
      "crc32c_span_emulate",
      [](py::bytes b, uint32_t c0, uint32_t c1, bool first) {
        std::string s = b;
        if (c0 > c1 || c1 > s.size() || c1 - c0 > kSpanLaneLarge * kSpanLanes)
          throw std::invalid_argument("crc32c_span_emulate: bad range");
        return crc32c_span_emulate(reinterpret_cast<const uint8_t*>(s.data()), c0, c1, first);
      },
      py::arg("data"), py::arg("c0"), py::arg("c1"), py::arg("first"));
  m.def("span_tables", []() {
    std::vector<uint32_t> t(kSpanTabWords);
    crc32c_span_tables(t.data());
    return t;
  });
  m.def("crc32c_method", [](int method, py::bytes b) {
    std::string s = b;
    return crc32c_method(method, s.data(), s.size());
  });
  m.def(
      "encode_batch",
      [](int64_t base_offset, std::vector<py::object> values, std::vector<py::object> keys,
         std::vector<int64_t> timestamps, std::vector<py::object> headers) {
        std::deque<std::string> keep;
        std::vector<std::vector<HeaderView>> hkeep;
        auto recs = to_records(values, keys, timestamps, headers, keep, hkeep);
        int64_t min_ts = timestamps.empty() ? 0 : *std::min_element(timestamps.begin(), timestamps.end());
        std::string out(batch_encoded_size(recs.data(), recs.size(), min_ts), '\0');
        size_t n = encode_batch(reinterpret_cast<uint8_t*>(&out[0]), base_offset, recs.data(), recs.size());
        out.resize(n);
        return py::bytes(out);
      },
      py::arg("base_offset"), py::arg("values"), py::arg("keys"), py::arg("timestamps"), py::arg("headers"));
  m.def(
      "decode_batches",
      [](py::bytes data, bool check_crcs) {
        std::string s = data;
        const uint8_t* p = reinterpret_cast<const uint8_t*>(s.data());
        size_t left = s.size();
        py::list out;
        while (left >= kBatchHeaderBytes) {
          BatchHeader h = parse_batch_header(p, left);
          if (check_crcs && !verify_batch_crc(p, h)) throw CorruptRecord("batch failed CRC check");
          RecordIter it(p, h);
          RecordView r;
          while (it.next(&r)) out.append(record_tuple(r, h.timestamp_type()));
          p += h.total_size();
          left -= h.total_size();
        }
        return out;
      },
      py::arg("data"), py::arg("check_crcs") = true);
  m.def("parse_json_f32", [](py::bytes b) {
    std::string s = b;
    std::vector<float> v(s.size() / 2 + 2);
    int64_t n = parse_json_f32(s.data(), s.size(), v.data(), int64_t(v.size()));
    if (n < 0) throw std::invalid_argument("not a flat numeric JSON array");
    v.resize(size_t(n));
    return v;
  });
  m.def(
      "json_scan_simple",
      [](py::bytes b, bool simd) {
        std::string s = b;
        return json_scan_simple(s.data(), s.size(), simd);
      },
      py::arg("data"), py::arg("simd") = true);
  m.def(
      "json_scan_inplace",
      [](py::bytes b, int variant, int iters) {
        std::string s = b;
        std::vector<char> src((s.size() + 63) / 64 * 64 + 128, 'x');  // bytes past the row are garbage on purpose
        std::memcpy(src.data(), s.data(), s.size());
        int64_t r = json_scan_inplace(src.data(), s.size(), src.size(), variant);
        if (iters <= 1) return py::make_tuple(r, 0.0);
        const int64_t t0 = now_ns();
        for (int i = 0; i < iters; ++i) r += json_scan_inplace(src.data(), s.size(), src.size(), variant) - r;
        return py::make_tuple(r, double(now_ns() - t0) / iters);  // (verdict, ns per scan)
      },
      py::arg("data"), py::arg("variant") = 0, py::arg("iters") = 1);
  m.def("json_scan_copy", [](py::bytes b) {
    std::string s = b;
    const size_t nr = (s.size() + 31) / 32 * 32 + 64;
    std::vector<char> src(nr, 'x');  // read-ahead bytes are garbage on purpose
    std::memcpy(src.data(), s.data(), s.size());
    void* dst = nullptr;
    if (posix_memalign(&dst, 64, nr) != 0) throw std::bad_alloc();
    const int64_t cnt = json_scan_copy(src.data(), s.size(), static_cast<uint8_t*>(dst));
    const bool same = std::memcmp(dst, s.data(), s.size()) == 0;
    std::free(dst);
    return py::make_tuple(cnt, same);
  });
  m.def("json_array_len", [](py::bytes b) {
    std::string s = b;
    return json_array_len(s.data(), s.size());
  });

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
      .def("assignment_epochs", &Replicator::assignment_epochs,
           "[(partition, epoch at which it was (re)assigned)] of the partitions owned now")
      .def_property_readonly("fetch_threads", &Replicator::fetch_threads)
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
          l.append(d);
        }
        return l;
      });

  // ---- fetcher
  py::class_<PyFetcher>(m, "Fetcher")
      .def(py::init<std::shared_ptr<Broker>, bool>(), py::arg("broker"), py::arg("check_crcs") = true)
      .def("assign", [](PyFetcher& f, std::vector<uint32_t> p, std::vector<int64_t> pos) { f.f.assign(p, pos); })
      .def(
          "watch",
          [](PyFetcher& f, py::list replicators) {
            std::vector<const std::atomic<uint64_t>*> eps;
            for (auto h : replicators) eps.push_back(h.cast<Replicator&>().epoch_ptr());
            f.watched = replicators;
            f.f.set_watch(std::move(eps));
          },
          py::arg("replicators"),
          "group-managed: fills return early (last_reassigned) when these replicas' assignment changes")
      .def("set_watch_base", [](PyFetcher& f, uint64_t base) { f.f.set_watch_base(base); }, py::arg("epoch_sum"))
      .def_property_readonly("last_reassigned", [](PyFetcher& f) { return f.last_reassigned; })
      .def("assigned", [](PyFetcher& f) {
        py::list l;
        for (auto& p : f.f.parts()) l.append(p.pidx);
        return l;
      })
      .def("positions",
           [](PyFetcher& f) {
             py::dict d;
             for (auto& p : f.f.parts()) d[py::int_(p.pidx)] = p.position;
             return d;
           })
      .def("position", [](PyFetcher& f, uint32_t pidx) -> py::object {
        size_t i = f.f.find(pidx);
        if (i == size_t(-1)) return py::none();
        return py::int_(f.f.parts()[i].position);
      })
      .def("seek", [](PyFetcher& f, uint32_t pidx, int64_t off) {
        size_t i = f.f.find(pidx);
        if (i == size_t(-1)) throw std::invalid_argument("partition is not assigned");
        auto& fp = f.f.parts()[i];
        fp.position = off;
        fp.batch_hint = -1;
      })
      .def("pause", [](PyFetcher& f, uint32_t pidx, bool paused) {
        size_t i = f.f.find(pidx);
        if (i == size_t(-1)) throw std::invalid_argument("partition is not assigned");
        f.f.parts()[i].paused = paused;
      })
      .def("has_data", [](PyFetcher& f) {
        for (auto& p : f.f.parts())
          if (!p.paused && f.f.has_data(p)) return true;
        return false;
      })
      .def(
          "poll_records",
          [](PyFetcher& f, int64_t max_records) {
            // Non-blocking: one round-robin pass, returns [(pidx, [record tuples])].
            py::list out;
            auto& parts = f.f.parts();
            int64_t left = max_records;
            for (size_t k = 0; k < parts.size() && left > 0; ++k) {
              FetchPart& fp = parts[(f.rr + k) % parts.size()];
              if (fp.paused) continue;
              py::list recs;
              Broker& b = f.f.broker();
              (void)b;
              f.f.scan(fp, size_t(left), [&](const RecordView& r) {
                recs.append(record_tuple(r, 0));
                return kTake;
              });
              if (py::len(recs)) {
                left -= int64_t(py::len(recs));
                out.append(py::make_tuple(fp.pidx, recs));
              }
            }
            if (!parts.empty()) f.rr = (f.rr + 1) % parts.size();
            return out;
          },
          py::arg("max_records"))
      .def(
          "poll_consumer_records",
          [](PyFetcher& f, int64_t max_records, py::object record_cls, py::dict tps) {
            // Like poll_records, but builds the kafka-python ConsumerRecord namedtuples here:
            // returns [(pidx, ConsumerRecord)], one flat list, in fetch order.  `tps` maps
            // pidx -> TopicPartition for every assigned partition.
            if (!PyType_Check(record_cls.ptr()) || !PyType_IsSubtype(reinterpret_cast<PyTypeObject*>(record_cls.ptr()),
                                                                     &PyTuple_Type))
              throw std::invalid_argument("record_cls must be a tuple subclass (namedtuple)");
            PyTypeObject* cls = reinterpret_cast<PyTypeObject*>(record_cls.ptr());
            py::list out;
            auto& parts = f.f.parts();
            int64_t left = max_records;
            py::object none = py::none();
            for (size_t k = 0; k < parts.size() && left > 0; ++k) {
              FetchPart& fp = parts[(f.rr + k) % parts.size()];
              if (fp.paused) continue;
              py::object tp = tps[py::int_(fp.pidx)];
              py::object topic = tp.attr("__getitem__")(0), part = tp.attr("__getitem__")(1);
              py::int_ pidx(fp.pidx);
              size_t got = f.f.scan(fp, size_t(left), [&](const RecordView& r) {
                // tuple_subtype_new's layout: allocate the namedtuple directly and fill its items
                PyObject* o = cls->tp_alloc(cls, 12);
                if (!o) throw py::error_already_set();
                py::list headers;
                if (r.header_count > 0) {
                  for (const auto& h : parse_headers(r)) {
                    headers.append(py::make_tuple(py::str(reinterpret_cast<const char*>(h.key), size_t(h.key_len)),
                                                  bytes_or_none(h.value, h.value_len)));
                  }
                }
                PyObject* items[12] = {
                    topic.inc_ref().ptr(),
                    part.inc_ref().ptr(),
                    PyLong_FromLongLong(r.offset),
                    PyLong_FromLongLong(r.timestamp),
                    PyLong_FromLong(0),
                    bytes_or_none(r.key, r.key_len).release().ptr(),
                    bytes_or_none(r.value, r.value_len).release().ptr(),
                    headers.release().ptr(),
                    none.inc_ref().ptr(),
                    PyLong_FromLong(r.key_len),
                    PyLong_FromLong(r.value_len),
                    PyLong_FromLong(r.header_bytes),
                };
                for (int i = 0; i < 12; ++i) PyTuple_SET_ITEM(o, i, items[i]);
                PyObject* pair = PyTuple_New(2);
                PyTuple_SET_ITEM(pair, 0, pidx.inc_ref().ptr());
                PyTuple_SET_ITEM(pair, 1, o);
                out.append(py::reinterpret_steal<py::object>(pair));
                return kTake;
              });
              left -= int64_t(got);
            }
            if (!parts.empty()) f.rr = (f.rr + 1) % parts.size();
            return out;
          },
          py::arg("max_records"), py::arg("record_cls"), py::arg("tps"))
      .def(
          "fill_slot",
          [](PyFetcher& f, py::object ring_obj, uint32_t gslot, int kind, int elem_size, int64_t row_elems,
             int64_t min_len, int64_t max_len, bool truncate, bool skip_bad, int64_t batch_rows, int64_t timeout_ms,
             bool gather, int span, int extras, int key_enc, int64_t key_default) {
            PyRing& ring = ring_obj.cast<PyRing&>();
            PackSpec s;
            s.gather = gather;
            s.span = span;
            s.extras = extras;
            s.key_enc = key_enc;
            s.key_default = key_default;
            s.kind = kind;
            s.elem_size = elem_size;
            s.row_elems = row_elems;
            s.min_len = min_len;
            s.max_len = max_len;
            s.truncate = truncate;
            s.skip_bad = skip_bad;
            FillOutcome o;
            {
              py::gil_scoped_release nogil;
              o = fill_slot(f.f, *ring.r, gslot, s, batch_rows, timeout_ms, &f.rr);
            }
            f.last_reassigned = o.reassigned;
            return py::make_tuple(o.rows, o.scanned, o.timed_out, o.shutdown);
          },
          py::arg("ring"), py::arg("gslot"), py::arg("kind"), py::arg("elem_size"), py::arg("row_elems"),
          py::arg("min_len"), py::arg("max_len"), py::arg("truncate"), py::arg("skip_bad"), py::arg("batch_rows"),
          py::arg("timeout_ms"), py::arg("gather") = false, py::arg("span") = 0, py::arg("extras") = 0,
          py::arg("key_enc") = 0, py::arg("key_default") = -1);
  m.def("key_int64", [](py::object key, int enc, int64_t dflt) {
    if (key.is_none()) return key_int64(nullptr, -1, enc, dflt);
    std::string k = key.cast<py::bytes>();
    return key_int64(reinterpret_cast<const uint8_t*>(k.data()), int32_t(k.size()), enc, dflt);
  }, py::arg("key"), py::arg("encoding"), py::arg("default"),
     "the integer a record key carries (the native packer's rule, for the per-record path)");
  m.attr("EXTRA_KEY") = int(kExtraKey);
  m.attr("EXTRA_TIMESTAMP") = int(kExtraTimestamp);

  // ---- ring
  py::class_<PyRing>(m, "Ring")
      .def_static("create",
                  [](const std::string& name, uint32_t nw, uint32_t spw, uint64_t cap) {
                    return new PyRing(Ring::create(name, nw, spw, cap));
                  })
      .def_static("open", [](const std::string& name) { return new PyRing(Ring::open(name)); })
      .def_property_readonly("name", [](PyRing& r) { return r.r->name(); })
      .def_property_readonly("base_address", [](PyRing& r) { return reinterpret_cast<uintptr_t>(r.r->base()); })
      .def_property_readonly("total_bytes", [](PyRing& r) { return r.r->total_bytes(); })
      .def_property_readonly("n_workers", [](PyRing& r) { return r.r->n_workers(); })
      .def_property_readonly("slots_per_worker", [](PyRing& r) { return r.r->slots_per_worker(); })
      .def_property_readonly("n_slots", [](PyRing& r) { return r.r->n_slots(); })
      .def_property_readonly("payload_capacity", [](PyRing& r) { return r.r->payload_capacity(); })
      .def("gslot", [](PyRing& r, uint32_t w, uint32_t i) { return r.r->gslot(w, i); })
      .def("payload_address", [](PyRing& r, uint32_t g) { return reinterpret_cast<uintptr_t>(r.r->payload(g)); })
      .def("payload_view",
           [](PyRing& r, uint32_t g) {
             return py::memoryview::from_memory(r.r->payload(g), ssize_t(r.r->payload_capacity()), false);
           })
      .def("slot_summary",
           [](PyRing& r, uint32_t g) {
             SlotHeader* h = r.r->slot(g);
             return py::make_tuple(h->n_rows, h->flags, h->payload_bytes, h->values_offset, h->max_row_len,
                                   h->total_elems, h->worker, h->kind, h->src_dtype);
           })
      .def("slot_info",
           [](PyRing& r, uint32_t g) {
             SlotHeader* h = r.r->slot(g);
             py::dict d;
             d["state"] = h->state.load();
             d["worker"] = h->worker;
             d["seq"] = h->seq;
             d["n_rows"] = h->n_rows;
             d["flags"] = h->flags;
             d["kind"] = h->kind;
             d["payload_bytes"] = h->payload_bytes;
             d["values_offset"] = h->values_offset;
             d["values_bytes"] = h->values_bytes;
             d["max_row_len"] = h->max_row_len;
             d["total_elems"] = h->total_elems;
             d["n_scanned"] = h->n_scanned;
             d["row_bytes"] = h->row_bytes;
             d["t_fill_start_ns"] = h->t_fill_start_ns;
             d["t_ready_ns"] = h->t_ready_ns;
             d["error"] = std::string(h->err, h->err_len);
             d["log_end"] = std::vector<uint64_t>(h->log_end, h->log_end + h->n_parts);
             d["n_segs"] = h->n_segs;
             d["trunc_len"] = h->trunc_len;
             return d;
           })
      .def("span_segments",
           [](PyRing& r, uint32_t g) {
             // kPackRecordSpan / kPackJsonSpan slots: [(log_pos, len, pidx, flags, crc, row_begin, row_end)]
             SlotHeader* h = r.r->slot(g);
             py::list l;
             if (h->kind != uint32_t(kPackRecordSpan) && h->kind != uint32_t(kPackJsonSpan) &&
                 h->kind != uint32_t(kPackVarSpan))
               return l;
             const auto* sg = reinterpret_cast<const SpanSeg*>(r.r->payload(g) + h->values_offset);
             for (uint32_t i = 0; i < h->n_segs; ++i)
               l.append(py::make_tuple(sg[i].log_pos, sg[i].len, sg[i].pidx, sg[i].flags, sg[i].crc, sg[i].row_begin,
                                       sg[i].row_end));
             return l;
           })
      .def("watermarks",
           [](PyRing& r, uint32_t g) {
             SlotHeader* h = r.r->slot(g);
             py::list l;
             for (uint32_t i = 0; i < h->n_parts; ++i)
               l.append(py::make_tuple(h->wm[i].pidx, h->wm[i].first_offset, h->wm[i].next_offset, h->wm[i].count));
             return l;
           })
      .def("set_slot",
           [](PyRing& r, uint32_t g, uint32_t n_rows, uint32_t flags, uint32_t kind, uint64_t payload_bytes,
              uint64_t values_offset, int64_t max_row_len, int64_t total_elems, int64_t n_scanned,
              std::vector<std::tuple<uint32_t, int64_t, int64_t, uint32_t>> wms) {
             SlotHeader* h = r.r->slot(g);
             if (wms.size() > size_t(kMaxSlotParts)) throw std::invalid_argument("too many watermarks");
             if (payload_bytes > r.r->payload_capacity()) throw std::invalid_argument("payload exceeds slot");
             h->n_rows = n_rows;
             h->flags = flags;
             h->err_len = 0;
             h->kind = kind;
             h->payload_bytes = payload_bytes;
             h->extras_offset = 0;
             h->extras_n = 0;
             h->values_offset = values_offset;
             h->values_bytes = payload_bytes - values_offset;
             h->max_row_len = max_row_len;
             h->total_elems = total_elems;
             h->n_scanned = n_scanned;
             h->n_parts = uint32_t(wms.size());
             for (size_t i = 0; i < wms.size(); ++i)
               h->wm[i] = Watermark{std::get<0>(wms[i]), std::get<3>(wms[i]), std::get<1>(wms[i]), std::get<2>(wms[i])};
           })
      .def("slot_extras",
           [](PyRing& r, uint32_t g) {
             SlotHeader* h = r.r->slot(g);
             return py::make_tuple(h->extras_offset, h->extras_n);
           }, "(payload offset, int64 columns) of the record fields beside the values")
      .def("set_slot_sample",
           [](PyRing& r, uint32_t g, int32_t dtype, std::vector<int64_t> shape) {
             SlotHeader* h = r.r->slot(g);
             if (shape.size() > 8) throw std::invalid_argument("sample rank > 8");
             h->src_dtype = dtype;
             h->ndim = int32_t(shape.size());
             for (size_t i = 0; i < shape.size(); ++i) h->shape[i] = shape[i];
           })
      .def("slot_sample",
           [](PyRing& r, uint32_t g) {
             SlotHeader* h = r.r->slot(g);
             std::vector<int64_t> shape(h->shape, h->shape + h->ndim);
             return py::make_tuple(h->src_dtype, shape);
           })
      .def("slot_states",
           [](PyRing& r) {
             // FREE / FILLING / READY / INFLIGHT counts: how much of the ring the workers have
             // filled ahead of the consumer (bench.py's prefilled_slots_at_t0)
             std::vector<uint32_t> n(4, 0);
             for (uint32_t g = 0; g < r.r->n_slots(); ++g) {
               const uint32_t s = r.r->slot(g)->state.load(std::memory_order_acquire);
               if (s < 4) ++n[s];
             }
             return n;
           })
      .def("set_flags", [](PyRing& r, uint32_t g, uint32_t flags) { r.r->slot(g)->flags |= flags; })
      .def("set_error",
           [](PyRing& r, uint32_t g, const std::string& msg) {
             SlotHeader* h = r.r->slot(g);
             const size_t n = std::min(msg.size(), sizeof(h->err));
             std::memcpy(h->err, msg.data(), n);
             h->err_len = uint32_t(n);
             h->flags |= kSlotError;
           })
      .def("set_worker_pid", [](PyRing& r, uint32_t w, int64_t pid) { r.r->header()->worker_pid[w].store(pid); })
      .def("set_worker_spin_ns", [](PyRing& r, int64_t ns) { r.r->set_worker_spin_ns(ns); })
      .def("worker_pid", [](PyRing& r, uint32_t w) { return r.r->header()->worker_pid[w].load(); })
      .def("worker_acquire",
           [](PyRing& r, uint32_t w, uint32_t i, int64_t timeout_ms) {
             py::gil_scoped_release nogil;
             return r.r->worker_acquire(w, i, timeout_ms);
           })
      .def("worker_publish", [](PyRing& r, uint32_t g) { r.r->worker_publish(g); })
      .def(
          "main_acquire",
          [](PyRing& r, int64_t timeout_ms, bool in_order) {
            py::gil_scoped_release nogil;
            return r.r->main_acquire(r.cursor.data(), &r.rr, r.done.data(), in_order, timeout_ms);
          },
          py::arg("timeout_ms"), py::arg("in_order") = false)
      .def("mark_done", [](PyRing& r, uint32_t w) { r.done.at(w) = 1; })
      .def("is_done", [](PyRing& r, uint32_t w) { return bool(r.done.at(w)); })
      .def("main_release", [](PyRing& r, uint32_t g) { r.r->main_release(g); })
      .def("shutdown", [](PyRing& r) { r.r->shutdown(); })
      .def("is_shutdown", [](PyRing& r) { return bool(r.r->header()->shutdown.load()); })
      .def("unlink", [](PyRing& r) { r.r->unlink(); });

  // ---- lockstep credit protocol (the device driver's, csrc/core/lockstep.h)
  py::register_exception<LockstepError>(m, "LockstepError", PyExc_RuntimeError);
  py::class_<LockstepTransport>(m, "LockstepTransport", py::module_local());
  py::class_<PyLockstepTransport, LockstepTransport>(m, "PyLockstepTransport", py::module_local())
      .def(py::init<py::function>(), py::arg("allreduce_min"));
  py::class_<CreditLockstep>(m, "CreditLockstep")
      .def(py::init<LockstepTransport*, int>(), py::arg("transport"), py::arg("depth"), py::keep_alive<1, 2>())
      .def(
          "next",
          [](CreditLockstep& l, py::object src, int64_t timeout_ms) {
            PyLockstepSource s(std::move(src));
            return l.next(s, timeout_ms);
          },
          py::arg("source"), py::arg("timeout_ms") = 100,
          "1: deliver the next batch (then call delivered()), -1 starved for now, -2 every rank stops here, "
          "-3 producer error")
      .def("delivered", &CreditLockstep::delivered)
      .def(
          "finished",
          [](CreditLockstep& l, int64_t index, std::vector<std::tuple<uint32_t, int64_t, int64_t, uint32_t>> wms) {
            std::vector<Watermark> w;
            for (auto& t : wms) w.push_back(Watermark{std::get<0>(t), std::get<3>(t), std::get<1>(t), std::get<2>(t)});
            l.finished(index, std::move(w));
          },
          py::arg("index"), py::arg("watermarks"))
      .def("finish", &CreditLockstep::finish)
      .def("set_sync", &CreditLockstep::set_sync, py::arg("sync"))
      .def(
          "set_on_committable",
          [](CreditLockstep& l, py::function f) {
            l.set_on_committable([f](std::vector<Watermark>&& w) { f(wms_to_list(w)); });
          },
          py::arg("callback"))
      .def_property_readonly("step", &CreditLockstep::step)
      .def_property_readonly("granted", &CreditLockstep::granted)
      .def_property_readonly("stopped", &CreditLockstep::stopped)
      .def_property_readonly("agreements", &CreditLockstep::agreements)
      .def_property_readonly("wait_ns", &CreditLockstep::wait_ns)
      .def_property_readonly("step_wait_max_ns", &CreditLockstep::step_wait_max_ns);

  m.attr("SLOT_EOS") = int(kSlotEOS);
  m.attr("SLOT_ERROR") = int(kSlotError);
  m.attr("PACK_FIXED") = int(kPackFixed);
  m.attr("PACK_VARLEN") = int(kPackVarlen);
  m.attr("PACK_JSON_F32") = int(kPackJsonF32);
  m.attr("PACK_GATHER_FIXED") = int(kPackGatherFixed);
  m.attr("PACK_JSON_TEXT") = int(kPackJsonText);
  m.attr("PACK_RECORD_SPAN") = int(kPackRecordSpan);
  m.attr("SPAN_SEG_MAX") = kSpanSegMax;
  m.attr("SPAN_MAX_SEG_ROWS") = kSpanMaxSegRows;
  m.attr("PACK_JSON_SPAN") = int(kPackJsonSpan);
  m.attr("PACK_VAR_SPAN") = int(kPackVarSpan);
  m.attr("PACK_TREE") = int(kPackTree);
  m.attr("VAR_SPAN_ROW_MAX") = kVarSpanRowMax;
  m.attr("JSON_SPAN_MAX_SEG_ROWS") = kJsonSpanMaxSegRows;
  m.attr("JSON_SPAN_ROW_MAX") = kJsonSpanRowMax;
  m.attr("SEG_HOST_ROWS") = int(kSegHostRows);
  m.attr("SPAN_JSON_DEV_COUNT") = kSpanJsonDevCount;
  m.attr("JSON_COUNT_ON_DEVICE") = kJsonCountOnDevice;
  m.attr("SLOT_DEV_COUNT") = int(kSlotDevCount);
  m.attr("SLOT_HEADER_BYTES") = kSlotHeaderBytes;
}
