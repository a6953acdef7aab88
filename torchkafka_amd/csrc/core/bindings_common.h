#pragma once
// Shared pieces of the `torchkafka_amd._tkcore` bindings (bindings*.cpp): the helpers that turn
// native records / watermarks / security settings into Python objects and back, and the
// adapters Python objects are wrapped in.  No HIP here (imported in forked workers).
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

namespace tkbind {
using namespace tk;


inline py::object bytes_or_none(const uint8_t* p, int32_t len) {
  if (!p || len < 0) return py::none();
  return py::bytes(reinterpret_cast<const char*>(p), size_t(len));
}

inline py::tuple record_tuple(const RecordView& r, int ts_type) {
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

inline std::vector<RecordIn> to_records(const std::vector<py::object>& values, const std::vector<py::object>& keys,
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
  int issue(const int64_t in[kLockstepWords]) override {
    py::tuple r = fn_(in[0], in[1], in[2], in[3]);
    const int t = int(next_++ % 64);
    for (int k = 0; k < kLockstepWords; ++k) res_[t][k] = r[size_t(k)].cast<int64_t>();
    return t;
  }
  void wait(int t, int64_t out[kLockstepWords]) override {
    for (int k = 0; k < kLockstepWords; ++k) out[k] = res_[t][k];
  }

 private:
  py::function fn_;
  uint64_t next_ = 0;
  int64_t res_[64][kLockstepWords];
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
inline wire::Security to_security(const py::dict& d) {
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

inline py::list wms_to_list(const std::vector<Watermark>& w) {
  py::list l;
  for (const auto& x : w) l.append(py::make_tuple(x.pidx, x.first_offset, x.next_offset, x.count));
  return l;
}


// one registration function per area (bindings_<area>.cpp), called by PYBIND11_MODULE (bindings.cpp)
void bind_broker(py::module_& m);
void bind_wire(py::module_& m);
void bind_fetch(py::module_& m);
void bind_ring(py::module_& m);
void bind_lockstep(py::module_& m);

}  // namespace tkbind
