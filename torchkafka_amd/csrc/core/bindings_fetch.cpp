// `torchkafka_amd._tkcore` bindings: the consumer fetch core and the worker packers.
#include "bindings_common.h"

namespace tkbind {

void bind_fetch(py::module_& m) {
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

}

}  // namespace tkbind
