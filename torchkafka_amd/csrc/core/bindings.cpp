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

#include "bindings_common.h"

using namespace tk;
using namespace tkbind;


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
  m.def("compress", [](int codec, py::bytes b, int level) {
    std::string s = b;
    std::vector<uint8_t> out;
    {
      py::gil_scoped_release nogil;
      compress(codec, reinterpret_cast<const uint8_t*>(s.data()), s.size(), out, level);
    }
    return py::bytes(reinterpret_cast<const char*>(out.data()), out.size());
  }, py::arg("codec"), py::arg("data"), py::arg("level") = 0);
  m.def("zstd_available", &zstd_available);
  m.def("lz4_library_available", &lz4_library_available);
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
      [](py::bytes b, uint32_t c0, uint32_t c1, bool first, int parts) {
        std::string s = b;
        if (c0 > c1 || c1 > s.size() || span_windows(c1) > 32 || parts < 1 || parts > kSpanMaxParts)
          throw std::invalid_argument("crc32c_span_emulate: bad range");
        return crc32c_span_emulate(reinterpret_cast<const uint8_t*>(s.data()), c0, c1, first, parts);
      },
      py::arg("data"), py::arg("c0"), py::arg("c1"), py::arg("first"), py::arg("parts") = 1);
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

  bind_broker(m);
  bind_wire(m);
  bind_fetch(m);
  bind_ring(m);
  bind_lockstep(m);

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
