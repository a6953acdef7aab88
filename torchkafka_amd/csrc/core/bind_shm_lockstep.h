// Python binding of tk::ShmLockstep, shared by _tkcore (CPU tests, the host lockstep) and _tkhip
// (the device driver's transport): each module registers it module-locally next to its own
// LockstepTransport base.
#pragma once
#include <pybind11/pybind11.h>

#include "shm_lockstep.h"

namespace tkbind_shm {

namespace py = pybind11;

template <class Base>
inline void bind_shm_lockstep(py::module_& m) {
  py::class_<tk::ShmLockstep, Base>(m, "ShmLockstep", py::module_local())
      .def(py::init<const std::string&, int, int>(), py::arg("name"), py::arg("rank"), py::arg("world"),
           py::call_guard<py::gil_scoped_release>())
      .def_static("create", &tk::ShmLockstep::create, py::arg("world"), py::arg("slots"),
                  "rank 0: a fresh segment for `world` ranks and `slots` agreements in flight; returns its name")
      .def("unlink", &tk::ShmLockstep::unlink)
      .def_property_readonly("attached", &tk::ShmLockstep::attached)
      .def("set_timeout_ms", &tk::ShmLockstep::set_timeout_ms, py::arg("ms"))
      .def_property_readonly("timeout_ms", &tk::ShmLockstep::timeout_ms)
      .def("allreduce_sum", &tk::ShmLockstep::allreduce_sum, py::arg("value"),
           py::call_guard<py::gil_scoped_release>())
      .def(
          "allreduce_min",
          [](tk::ShmLockstep& l, int64_t a, int64_t b, int64_t c, int64_t d) {
            const int64_t in[tk::kLockstepWords] = {a, b, c, d};
            int64_t r[tk::kLockstepWords];
            {
              py::gil_scoped_release nogil;
              l.wait(l.issue(in), r);
            }
            return py::make_tuple(r[0], r[1], r[2], r[3]);
          },
          "one agreement (issue + wait): the MIN of the 4 words over the ranks")
      .def_property_readonly("rank", &tk::ShmLockstep::rank)
      .def_property_readonly("world", &tk::ShmLockstep::world)
      .def_property_readonly("slots", &tk::ShmLockstep::slots)
      .def_property_readonly("issued", &tk::ShmLockstep::issued)
      .def_property_readonly("spin_ns", &tk::ShmLockstep::spin_ns);
}

}  // namespace tkbind_shm
