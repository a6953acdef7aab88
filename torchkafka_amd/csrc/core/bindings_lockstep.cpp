// `torchkafka_amd._tkcore` bindings: the cross-rank credit lockstep (csrc/core/lockstep.h).
#include "bindings_common.h"
#include "bind_shm_lockstep.h"

namespace tkbind {

void bind_lockstep(py::module_& m) {
  // ---- lockstep credit protocol (the device driver's, csrc/core/lockstep.h)
  py::register_exception<LockstepError>(m, "LockstepError", PyExc_RuntimeError);
  py::class_<LockstepTransport>(m, "LockstepTransport", py::module_local());
  py::class_<PyLockstepTransport, LockstepTransport>(m, "PyLockstepTransport", py::module_local())
      .def(py::init<py::function>(), py::arg("allreduce_min"),
           "allreduce_min(credit, step, -step, commit_status) -> the 4 words' MIN over the ranks");
  tkbind_shm::bind_shm_lockstep<LockstepTransport>(m);
  m.attr("LOCKSTEP_WORDS") = kLockstepWords;
  m.attr("COMMIT_OK") = kCommitOk;
  m.attr("COMMIT_FAILED") = kCommitFailed;
  m.attr("COMMIT_FATAL") = kCommitFatal;
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
      .def("set_commit_every", &CreditLockstep::set_commit_every, py::arg("n"),
           "async mode: an agreement grants at most n batches (0: no cap)")
      .def("set_commit_status", &CreditLockstep::set_commit_status, py::arg("status"),
           "sync mode: 2 committed, 1 CommitFailedError swallowed, 0 the commit raised")
      .def_property_readonly("group_commit_status", &CreditLockstep::group_commit_status)
      .def_property_readonly("group_commit_failures", &CreditLockstep::group_commit_failures)
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

}

}  // namespace tkbind
