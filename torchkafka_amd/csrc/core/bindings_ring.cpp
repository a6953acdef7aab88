// `torchkafka_amd._tkcore` bindings: the worker -> main-process slot ring.
#include "bindings_common.h"

namespace tkbind {

void bind_ring(py::module_& m) {
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

}

}  // namespace tkbind
