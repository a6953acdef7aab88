// pybind11 bindings of the device half: module `torchkafka_amd._tkhip`.
// Tensors cross the boundary as raw device pointers (Tensor.data_ptr()) and
// streams as hipStream_t handles (torch.cuda.Stream.cuda_stream).  The one
// exception is torch_step.cpp (step_fixed_tensor), which allocates the batch
// through libtorch; the module therefore builds against torch's pybind11.
#include <hip/hip_runtime.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "collate.h"
#include "dtypes.h"
#include "engine.h"
#include "driver.h"
#include "rccl_lockstep.h"
#include "bind_shm_lockstep.h"
#include "reaper.h"

namespace py = pybind11;
using namespace tkh;

namespace tkh {
void register_torch_step(py::module_& m);  // torch_step.cpp
}

namespace {
// Lockstep transport backed by a Python callable (e.g. a gloo all_reduce): lets the
// native driver's pipelined protocol run multi-rank where RCCL cannot (several
// ranks on one GPU, CPU tests).  Each issue() performs the collective at once.
class PyLockstep : public LockstepTransport {
 public:
  explicit PyLockstep(py::function fn) : fn_(std::move(fn)) {}
  int issue(const int64_t in[tk::kLockstepWords]) override {
    py::gil_scoped_acquire gil;
    py::tuple r = fn_(in[0], in[1], in[2], in[3]);
    const int t = int(next_++ % 64);
    for (int k = 0; k < tk::kLockstepWords; ++k) res_[t][k] = r[size_t(k)].cast<int64_t>();
    return t;
  }
  void wait(int t, int64_t out[tk::kLockstepWords]) override {
    for (int k = 0; k < tk::kLockstepWords; ++k) out[k] = res_[t][k];
  }

 private:
  py::function fn_;
  uint64_t next_ = 0;
  int64_t res_[64][tk::kLockstepWords];
};

template <typename T>
T* ptr(uintptr_t p) { return reinterpret_cast<T*>(p); }
hipStream_t stream_of(uintptr_t s) { return reinterpret_cast<hipStream_t>(s); }
}  // namespace

#ifndef TK_SOURCES_SHA
#define TK_SOURCES_SHA "unversioned"  // built outside _build.py
#endif
// The sha of the sources this binary was built from (_build.sources_sha): _build.embedded_sha finds it
// in the file, ops.build_info() compares it with the tree.
__attribute__((used)) static const char kSourcesSha[] = "TKSRCSHA:" TK_SOURCES_SHA;

PYBIND11_MODULE(_tkhip, m) {
  m.attr("SOURCES_SHA") = std::string(kSourcesSha + 9);
  m.doc() = "torchkafka_amd gfx950 device path: H2D engine + collate kernels";

  m.def("device_info", [](int dev) {
    hipDeviceProp_t p;
    hipError_t e = hipGetDeviceProperties(&p, dev);
    if (e != hipSuccess) throw std::runtime_error(hipGetErrorString(e));
    py::dict d;
    d["name"] = std::string(p.name);
    d["gcn_arch"] = std::string(p.gcnArchName);
    d["cus"] = p.multiProcessorCount;
    d["warp_size"] = p.warpSize;
    d["total_mem"] = p.totalGlobalMem;
    d["lds_per_block"] = p.sharedMemPerBlock;
    return d;
  });

  m.def("api_bench", &api_bench, py::arg("device") = 0, py::arg("iters") = 10000);
  m.def("reaper_drain", [](int timeout_ms) {
    py::gil_scoped_release nogil;
    return Reaper::drain(timeout_ms);
  }, py::arg("timeout_ms") = 60000, "waits until every deferred release (loader teardown) ran");
  m.def("reaper_stats", []() {
    py::dict d;
    d["enabled"] = Reaper::enabled();
    d["posted"] = Reaper::posted();
    d["released"] = Reaper::released();
    return d;
  });

  m.def(
      "collate_fixed",
      [](uintptr_t src, int src_dt, uintptr_t dst, int dst_dt, int64_t rows, int64_t row, uintptr_t shift,
         uintptr_t scale, uintptr_t stream) {
        launch_fixed(ptr<const void>(src), src_dt, ptr<void>(dst), dst_dt, rows, row, ptr<const float>(shift),
                     ptr<const float>(scale), stream_of(stream));
      },
      py::arg("src"), py::arg("src_dtype"), py::arg("dst"), py::arg("dst_dtype"), py::arg("rows"), py::arg("row"),
      py::arg("shift") = 0, py::arg("scale") = 0, py::arg("stream") = 0);

  m.def(
      "collate_varlen",
      [](uintptr_t offs, uintptr_t vals, int src_dt, uintptr_t out, int dst_dt, int64_t rows, int64_t L, double pad,
         uintptr_t lengths, uintptr_t mask, uintptr_t stream) {
        launch_varlen(ptr<const int32_t>(offs), ptr<const void>(vals), src_dt, ptr<void>(out), dst_dt, rows, L, pad,
                      ptr<int64_t>(lengths), ptr<uint8_t>(mask), stream_of(stream));
      },
      py::arg("offsets"), py::arg("values"), py::arg("src_dtype"), py::arg("out"), py::arg("dst_dtype"),
      py::arg("rows"), py::arg("L"), py::arg("pad") = 0.0, py::arg("lengths") = 0, py::arg("mask") = 0,
      py::arg("stream") = 0);

  m.def(
      "launch_json_rows",
      [](uintptr_t rows, uintptr_t vals, uintptr_t out, int dst_dt, int64_t n_rows, int64_t L, double pad,
         uintptr_t lengths, uintptr_t mask, uintptr_t err, uintptr_t stream) {
        launch_json_rows(ptr<const JsonRowDesc>(rows), ptr<const void>(vals), ptr<void>(out), dst_dt, n_rows, L, pad,
                         ptr<int64_t>(lengths), ptr<uint8_t>(mask), ptr<int32_t>(err), stream_of(stream));
      },
      py::arg("rows"), py::arg("values"), py::arg("out"), py::arg("dst_dtype"), py::arg("n_rows"), py::arg("L"),
      py::arg("pad") = 0.0, py::arg("lengths") = 0, py::arg("mask") = 0, py::arg("err") = 0, py::arg("stream") = 0);

  py::class_<Engine>(m, "Engine")
      .def(py::init<int, int, size_t, int, int>(), py::arg("device"), py::arg("n_slots"), py::arg("staging_bytes"),
           py::arg("n_streams") = 4, py::arg("mode") = int(kH2DDma))
      .def_property_readonly("mode", &Engine::mode)
      .def("wait_copy",
           [](Engine& e, int s) {
             py::gil_scoped_release nogil;
             e.wait_copy(s);
           })
      .def_property_readonly("device", &Engine::device)
      .def_property_readonly("n_slots", &Engine::n_slots)
      .def_property_readonly("staging_stride", &Engine::staging_stride)
      .def_property_readonly("copy_stream", [](Engine& e) { return reinterpret_cast<uintptr_t>(e.copy_stream()); })
      .def("staging_address", [](Engine& e, int s) { return reinterpret_cast<uintptr_t>(e.staging(s)); })
      .def("register_host", [](Engine& e, uintptr_t p, size_t n) { e.register_host(ptr<void>(p), n); })
      .def("unregister_host", &Engine::unregister_host)
      .def_property_readonly("host_registered", &Engine::host_registered)
      .def("h2d", [](Engine& e, int s, uintptr_t host, size_t n) { e.h2d(s, ptr<const void>(host), n); })
      .def("h2d_complete", &Engine::h2d_complete)
      .def("wait_h2d",
           [](Engine& e, int s) {
             py::gil_scoped_release nogil;
             e.wait_h2d(s);
           })
      .def("collate_fixed",
           [](Engine& e, int s, uintptr_t stream, size_t voff, int src_dt, uintptr_t dst, int dst_dt, int64_t rows,
              int64_t row, uintptr_t shift, uintptr_t scale) {
             e.collate_fixed(s, stream_of(stream), voff, src_dt, ptr<void>(dst), dst_dt, rows, row,
                             ptr<const float>(shift), ptr<const float>(scale));
           })
      .def("collate_varlen",
           [](Engine& e, int s, uintptr_t stream, size_t voff, int src_dt, uintptr_t out, int dst_dt, int64_t rows,
              int64_t L, double pad, uintptr_t lengths, uintptr_t mask) {
             e.collate_varlen(s, stream_of(stream), voff, src_dt, ptr<void>(out), dst_dt, rows, L, pad,
                              ptr<int64_t>(lengths), ptr<uint8_t>(mask));
           })
      .def("copy_raw",
           [](Engine& e, int s, uintptr_t stream, size_t off, uintptr_t dst, size_t n) {
             e.copy_raw(s, stream_of(stream), off, ptr<void>(dst), n);
           })
      .def("set_decode_streams", &Engine::set_decode_streams, py::arg("n"))
      .def("decode_streams", &Engine::decode_streams)
      .def("copy_streams", &Engine::copy_streams)
      .def("synchronize", [](Engine& e) {
        py::gil_scoped_release nogil;
        e.synchronize();
      });

  py::class_<LockstepTransport>(m, "LockstepTransport", py::module_local());
  py::class_<PyLockstep, LockstepTransport>(m, "PyLockstep", py::module_local())
      .def(py::init<py::function>(), py::arg("allreduce_min"));
  tkbind_shm::bind_shm_lockstep<LockstepTransport>(m);
  py::class_<RcclLockstep, LockstepTransport>(m, "RcclLockstep", py::module_local())
      .def(py::init([](const std::string& lib, py::bytes id, int rank, int world, int device, int slots) {
             return new RcclLockstep(lib, std::string(id), rank, world, device, slots);
           }),
           py::arg("lib_path"), py::arg("unique_id"), py::arg("rank"), py::arg("world_size"), py::arg("device"),
           py::arg("slots"))
      .def_static("unique_id", [](const std::string& lib) { return py::bytes(RcclLockstep::unique_id(lib)); })
      .def("allreduce_min",
           [](RcclLockstep& l, int64_t a, int64_t b, int64_t c, int64_t d) {
             const int64_t in[tk::kLockstepWords] = {a, b, c, d};
             int64_t r[tk::kLockstepWords];
             {
               py::gil_scoped_release nogil;
               l.wait(l.issue(in), r);
             }
             return py::make_tuple(r[0], r[1], r[2], r[3]);
           },
           py::arg("a"), py::arg("b"), py::arg("c"), py::arg("d") = tk::kCommitOk)
      .def_property_readonly("high_priority", &RcclLockstep::high_priority,
                             "the lockstep stream is at the device's greatest priority (a hardware queue of its own)")
      .def_property_readonly("words_mode", &RcclLockstep::words_mode,
                             "how the agreement words reach RCCL: kernel (tiny copy kernels), host (RCCL on "
                             "host-mapped memory) or copy (hipMemcpyAsync)")
      .def_property_readonly("issued", &RcclLockstep::issued)
      .def("take_trace",
           [](RcclLockstep& l) {
             py::list out;
             for (const auto& r : l.take_trace()) out.append(py::make_tuple(r.issue0, r.issue1, r.wait0, r.wait1));
             return out;
           },
           "TORCHKAFKA_LOCKSTEP_TRACE=1: [(issue begin, issue end, wait begin, wait end)] host ns per agreement")
      .def_property_readonly("nranks", &RcclLockstep::comm_count,
                             "ranks in the private communicator, as RCCL reports them (ncclCommCount)")
      .def(
          "allreduce_sum",
          [](RcclLockstep& l, int64_t v) {
            py::gil_scoped_release nogil;
            return l.allreduce_sum(v);
          },
          py::arg("value"), "blocking all-reduce(SUM) of one int64 over the private communicator")
      .def("set_timeout_ms", &RcclLockstep::set_timeout_ms, py::arg("ms"))
      .def_property_readonly("timeout_ms", &RcclLockstep::timeout_ms)
      .def_property_readonly("aborted", &RcclLockstep::aborted);

  py::class_<MainDriver>(m, "MainDriver")
      .def(py::init([](Engine* e, const std::string& ring, const std::string& url, const std::string& group,
                       int prefetch, bool in_order, int src_dt) {
             return new MainDriver(e, ring, url, group, prefetch, in_order, src_dt);
           }),
           py::keep_alive<1, 2>(), py::arg("engine"), py::arg("ring_name"), py::arg("broker_url"), py::arg("group"),
           py::arg("prefetch"), py::arg("in_order"), py::arg("default_src_dtype"))
      .def_property_readonly("can_commit", &MainDriver::can_commit)
      .def("step_fixed",
           [](MainDriver& d, uintptr_t stream, int dst_dt, uintptr_t dst, int64_t row, uintptr_t shift,
              uintptr_t scale, bool auto_commit, int64_t timeout_ms) {
             int cs = 0;
             int64_t r;
             {
               py::gil_scoped_release nogil;
               r = d.step_fixed(stream_of(stream), dst_dt, ptr<void>(dst), row, ptr<const float>(shift),
                                ptr<const float>(scale), auto_commit, timeout_ms, &cs, &d.last);
             }
             return py::make_tuple(r, cs);
           })
      .def("next_slot",
           [](MainDriver& d, int64_t timeout_ms) -> py::tuple {
             int r;
             {
               py::gil_scoped_release nogil;
               r = d.next_slot(timeout_ms, &d.last);
             }
             if (r < 0) return py::make_tuple(r);
             const SlotView& v = d.last;
             return py::make_tuple(r, v.n_rows, v.kind, v.max_row_len, v.total_elems, v.src_dtype, v.shape,
                                   v.payload_bytes);
           })
      .def("collate_fixed_last",
           [](MainDriver& d, uintptr_t stream, int dst_dt, uintptr_t dst, int64_t row, uintptr_t shift,
              uintptr_t scale, uintptr_t ext_dst) {
             if (ext_dst) {
               int64_t* e = ptr<int64_t>(ext_dst);
               d.set_extra_outputs(&e, 1);
             }
             d.collate_fixed(d.last, stream_of(stream), dst_dt, ptr<void>(dst), row, ptr<const float>(shift),
                             ptr<const float>(scale));
           },
           py::arg("stream"), py::arg("dst_dt"), py::arg("dst"), py::arg("row"), py::arg("shift"), py::arg("scale"),
           py::arg("ext_dst") = 0)
      .def_property_readonly("last_extras", [](MainDriver& d) { return int(d.last.extras_n); })
      .def("collate_varlen_last",
           [](MainDriver& d, uintptr_t stream, int dst_dt, uintptr_t out, int64_t L, double pad, uintptr_t lengths,
              uintptr_t mask, int64_t mult) -> int64_t {
             // -> the batch's width: L, or for a device-counted JSON batch (kSlotDevCount, L its
             // capacity) the width the parse kernel chose; its first rows * width elements hold the batch
             py::gil_scoped_release nogil;
             d.set_json_mult(mult);
             d.collate_varlen(d.last, stream_of(stream), dst_dt, ptr<void>(out), L, pad, ptr<int64_t>(lengths),
                              ptr<uint8_t>(mask));
             if (!(d.last.flags & tk::kSlotDevCount) || d.last.n_rows == 0) return L;
             SlotView v = d.last;
             v.perr = d.last_perr();
             int64_t n_host = 0;
             const int64_t w = d.json_width(v, &n_host);
             if (n_host > 0)
               d.json_host_rows(v, ptr<void>(out), w, dst_dt, pad, ptr<int64_t>(lengths), ptr<uint8_t>(mask),
                                stream_of(stream));
             return w;
           },
           py::arg("stream"), py::arg("dst_dt"), py::arg("out"), py::arg("L"), py::arg("pad"), py::arg("lengths"),
           py::arg("mask"), py::arg("mult") = 1)
      .def("copy_payload_last",
           [](MainDriver& d, uintptr_t stream, uintptr_t dst) { d.copy_payload(d.last, stream_of(stream), ptr<void>(dst)); })
      .def_property_readonly("last_slot", [](MainDriver& d) { return int64_t(d.last.g); })
      .def("last_watermarks",
           [](MainDriver& d) {
             py::list l;
             for (const auto& w : d.last.wms) l.append(py::make_tuple(w.pidx, w.first_offset, w.next_offset, w.count));
             return l;
           })
      .def("deliver_last", [](MainDriver& d) { d.deliver(d.last); })
      .def("parse_error", [](MainDriver& d) { return d.parse_error(); })
      .def("discard_last",
           [](MainDriver& d) {
             py::gil_scoped_release nogil;
             d.discard(d.last);
           })
      .def("finish_delivered", [](MainDriver& d, uintptr_t fence) { d.finish_delivered(stream_of(fence)); },
           py::arg("fence_stream") = 0)
      .def("set_commit_on_device", &MainDriver::set_commit_on_device)
      .def("drain_fenced",
           [](MainDriver& d, bool wait) {
             py::gil_scoped_release nogil;
             d.drain_fenced(wait);
           })
      .def("add_finished",
           [](MainDriver& d, std::vector<std::tuple<uint32_t, int64_t, int64_t, uint32_t>> wms) {
             std::vector<tk::Watermark> v;
             for (auto& w : wms) v.push_back(tk::Watermark{std::get<0>(w), std::get<3>(w), std::get<1>(w), std::get<2>(w)});
             d.add_finished(v);
           })
      .def("commit_pending", &MainDriver::commit_pending)
      .def("committed", &MainDriver::committed)
      .def("take_pending", &MainDriver::take_pending)
      .def("error", &MainDriver::error)
      .def("worker_done", &MainDriver::worker_done)
      .def("stats",
           [](MainDriver& d) {
             py::dict s;
             s["commits"] = d.commits();
             s["commit_failures"] = d.commit_failures();
             s["commit_ns"] = d.commit_ns();
             s["commit_latency_ns"] = d.commit_latency_ns();
             s["fill_ns"] = d.poll_stats().fill_ns;
             s["fills"] = d.poll_stats().fills;
             s["blocked_ns"] = d.blocked_ns_;
             s["blocked_calls"] = d.blocked_calls_;
             s["ready_age_ns"] = d.poll_stats().ready_age_ns;
             s["worker_idle_ns"] = d.poll_stats().worker_idle_ns;
             s["worker_slot_wait_ns"] = d.poll_stats().worker_slot_wait_ns;
             s["phase_commit_ns"] = d.ph_commit_ns_;
             s["phase_next_ns"] = d.ph_next_ns_;
             s["phase_launch_ns"] = d.ph_launch_ns_;
             s["phase_steps"] = d.ph_steps_;
             s["events"] = d.events_;
             s["groups"] = d.groups();
             s["coalesce_wait_ns"] = d.cwait_ns_;
             s["ahead_groups"] = d.ahead_groups_;
             s["ahead_ns"] = d.ahead_ns_;
             s["split_launches"] = d.split_launches_;
             s["json_width_wait_ns"] = d.json_width_wait_ns();
             s["occ_handed"] = d.occ_handed_;
             s["occ_staged"] = d.occ_staged_;
             s["occ_samples"] = d.occ_samples_;
             s["release_ns"] = d.rel_ns_;
             s["fast_batches"] = d.fast_batches_;
             s["fast_records"] = d.fast_records_;
             s["fast_ns"] = d.fast_ns_;
             s["released"] = d.released_;
             s["polled"] = d.poll_stats().polled;
             s["poll_ns"] = d.poll_stats().poll_ns;
             s["log_bytes_registered"] = d.log_bytes_registered();
             s["log_bytes_unpinned"] = d.log_bytes_unpinned();
             if (const LogMirror* m = d.mirror()) {
               s["mirror_bytes_copied"] = m->bytes_copied();
               s["mirror_copies"] = m->copies();
               s["mirror_fallbacks"] = m->fallbacks();
               s["mirror_pending_fallbacks"] = m->pending_fallbacks();
               s["mirror_backoffs"] = m->backoffs();
               s["mirror_device_bytes"] = m->device_bytes();
             }
             s["log_register_ns"] = d.log_register_ns();
             s["log_register_wait_ns"] = d.log_register_wait_ns();
             s["log_register_retries"] = d.log_register_retries();
             s["lockstep_agreements"] = d.lockstep_agreements();
             s["lockstep_wait_ns"] = d.lockstep_wait_ns();
             s["lockstep_issue_ns"] = d.lockstep_issue_ns();
             s["lockstep_step_wait_max_ns"] = d.lockstep_step_wait_max_ns();
             s["verify_wait_ns"] = d.verify_wait_ns_;
             return s;
           })
      .def("reset_stats", &MainDriver::reset_stats)
      .def("set_event_every", &MainDriver::set_event_every, py::arg("n"))
      .def_property_readonly("event_every", &MainDriver::event_every)
      .def("set_coalesce", &MainDriver::set_coalesce, py::arg("n"))
      .def("set_coalesce_wait_us", &MainDriver::set_coalesce_wait_us, py::arg("us"))
      .def("enable_direct", &MainDriver::enable_direct)
      .def("enable_mirror", &MainDriver::enable_mirror, py::arg("chunk_bytes"), py::arg("chunks_per_partition"),
           py::arg("copy_streams") = 0, py::arg("wait") = -1)
      .def_property_readonly("mirror_waits",
                             [](MainDriver& d) { return d.mirror_waits(); })
      .def_property_readonly("mirror_copy_streams",
                             [](MainDriver& d) { return d.mirror_copy_streams(); })
      .def("set_ahead_depth", &MainDriver::set_ahead_depth)
      .def("set_group_bytes", &MainDriver::set_group_bytes)
      .def("set_worker_sink", &MainDriver::set_worker_sink, py::arg("table"), py::arg("n_workers"),
           py::arg("capacity"))
      .def(
          "pin_logs",
          [](MainDriver& d, std::vector<uint32_t> pidxs) {
            py::gil_scoped_release nogil;
            d.pin_logs(pidxs);
          },
          py::arg("pidxs"), "pin (and device-map) what the partition logs hold now, before the first batch")
      .def_property_readonly("direct", &MainDriver::direct)
      .def_property_readonly("coalesce", &MainDriver::coalesce)
      .def("enable_lockstep", &MainDriver::enable_lockstep, py::arg("transport"), py::arg("depth"),
           py::arg("commit_every") = 0, py::keep_alive<1, 2>())
      .def("set_sync_commit", &MainDriver::set_sync_commit, py::arg("sync"))
      .def("set_commit_status", &MainDriver::set_commit_status, py::arg("status"),
           "sync commits under the lockstep: how this rank's commits of the finished batch went (2 stored, 1 "
           "CommitFailedError swallowed, 0 raised); the next agreement carries it to every rank")
      .def_property_readonly("group_commit_failures", &MainDriver::group_commit_failures)
      .def("delivered_positions", &MainDriver::delivered_positions,
           "[(partition index, position after the batches handed out so far)]")
      .def_property_readonly("delivered_batches", &MainDriver::delivered_batches)
      .def("set_command_queue", &MainDriver::set_command_queue, py::arg("on"))
      .def("verify_delivered",
           [](MainDriver& d) {
             py::gil_scoped_release nogil;
             return d.verify_delivered();
           })
      .def("finish_lockstep",
           [](MainDriver& d) {
             py::gil_scoped_release nogil;
             d.finish_lockstep();
           })
      .def_property_readonly("lockstep_enabled", &MainDriver::lockstep_enabled);

  register_torch_step(m);

  m.attr("H2D_DMA") = int(kH2DDma);
  m.attr("H2D_ZERO_COPY") = int(kH2DZeroCopy);
  m.attr("F32") = int(kF32);
  m.attr("F16") = int(kF16);
  m.attr("BF16") = int(kBF16);
  m.attr("FP8E4M3") = int(kFP8E4M3);
  m.attr("U8") = int(kU8);
  m.attr("I8") = int(kI8);
  m.attr("I32") = int(kI32);
  m.attr("I64") = int(kI64);
}
