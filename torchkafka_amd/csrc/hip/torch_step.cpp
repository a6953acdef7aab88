// The fixed-width fast path with the output tensor allocated here, in C++, from
// PyTorch's HIP caching allocator on the caller's current stream.
//
// Per batch the Python loop used to pay for torch.empty(...) through the Python
// argument parser (~1.7 µs on the MI355X host), plus stream and data_ptr lookups.
// at::empty + THPVariable_Wrap cost a fraction of that, and the batch keeps the
// allocator's ordinary stream semantics (freed tensors are reused on the stream
// they were allocated on).  This is the only translation unit that sees libtorch
// headers.
#include <ATen/ATen.h>
#include <c10/hip/HIPCachingAllocator.h>
#include <c10/hip/HIPGuard.h>
#include <c10/hip/HIPStream.h>
#include <torch/csrc/autograd/python_variable.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <ctime>

#include "consumer.h"
#include "driver.h"
#include "collate.h"
#include "dtypes.h"

namespace py = pybind11;

namespace tkh {

namespace {
at::ScalarType scalar_type_of(int code) {
  switch (code) {
    case kF32: return at::kFloat;
    case kF16: return at::kHalf;
    case kBF16: return at::kBFloat16;
    case kFP8E4M3: return at::kFloat8_e4m3fn;
    case kU8: return at::kByte;
    case kI8: return at::kChar;
    case kI32: return at::kInt;
    case kI64: return at::kLong;
    default: throw std::invalid_argument("step_fixed_tensor: unsupported dtype code");
  }
}
at::Tensor alloc_group(MainDriver& d, const std::vector<int64_t>& shape, const at::TensorOptions& opts,
                       c10::DeviceIndex dev, bool span);

// Outputs of a var-len batch.  A batch of a device-decode group owns a region of the group's blocks
// (vals / lens / masks, one allocation each for the whole group) and gets its tensors -- views of
// that region -- only at delivery (finish_json), so forming a group costs three allocations
// instead of three tensors per batch.
struct VarlenOut {
  at::Tensor out, lengths, mask;  // the delivered tensors
  at::Tensor vals, lens, masks;   // group blocks (device-decode groups)
  int64_t vo = 0, ro = 0;         // this batch's first element / row in them
  int64_t m = 0, L = 0;           // rows, allocated width
  // device-counted JSON batch (kSlotDevCount): L is a capacity; the batch is [m, width] with the
  // width the parse kernel reported, at the start of its region
  bool devc = false;
};

// A group batch at delivery: its views -- for a device-counted JSON batch with the width the parse
// kernel reported (the kernel wrote the rows with that stride), and the rows it left to the host
// parsed and written on `ks`.
void finish_json(MainDriver& d, const SlotView& v, VarlenOut* o, int dst_dt, double pad, hipStream_t ks) {
  if (o->out.defined()) return;
  const int64_t m = o->m;
  int64_t n_host = 0, L = o->devc ? 0 : o->L;
  if (o->devc && m > 0) {
    py::gil_scoped_release nogil;
    L = d.json_width(v, &n_host);
  }
  // (as_strided's offset is absolute in the storage the three blocks share)
  o->out = o->vals.as_strided({m, L}, {L, 1}, o->vals.storage_offset() + o->vo);
  o->lengths = o->lens.as_strided({m}, {1}, o->lens.storage_offset() + o->ro);
  if (o->masks.defined()) o->mask = o->masks.as_strided({m, L}, {L, 1}, o->masks.storage_offset() + o->vo);
  if (n_host > 0) {
    uint8_t* mk = o->mask.defined() ? static_cast<uint8_t*>(o->mask.data_ptr()) : nullptr;
    void* out = o->out.data_ptr();
    int64_t* lens = o->lengths.data_ptr<int64_t>();
    py::gil_scoped_release nogil;
    d.json_host_rows(v, out, L, dst_dt, pad, lens, mk, ks);
  }
}

// Outputs of a fixed-width batch: the values, and -- when the schema asks for record fields --
// its [extras, rows] int64 key / timestamp columns (decoded by the same launch).
struct FixedOut {
  at::Tensor out, ext;
};

std::shared_ptr<void> fixed_handle(at::Tensor out, at::Tensor ext) {
  auto h = std::make_shared<FixedOut>();
  h->out = std::move(out);
  h->ext = std::move(ext);
  return h;
}

// [sum(rows) * extras] int64, viewed [extras, rows_k] per batch, allocated like its values block
// (on the decode stream for a device-decode group) and handed to the driver's next launch.
std::vector<at::Tensor> alloc_extras(MainDriver& d, const std::vector<int64_t>& rows, int extras,
                                     c10::DeviceIndex dev, bool span) {
  std::vector<at::Tensor> out;
  if (extras <= 0) return out;
  int64_t total = 0;
  for (auto x : rows) total += x;
  const auto opts = at::TensorOptions().dtype(at::kLong).device(at::kCUDA, dev);
  at::Tensor all = alloc_group(d, {total * extras}, opts, dev, span);
  int64_t* dsts[kMaxGroup];
  int64_t off = 0;
  for (size_t k = 0; k < rows.size(); ++k) {
    // one column (a Key): the [rows] column itself, so delivery hands it out without a select
    // (the label block runs host-bound at ~5 us per step: every view made per batch shows)
    out.push_back(extras == 1 ? all.narrow(0, off, rows[k]) : all.narrow(0, off, rows[k] * extras).view({extras, rows[k]}));
    dsts[k] = out.back().data_ptr<int64_t>();
    off += rows[k] * extras;
  }
  d.set_extra_outputs(dsts, int(rows.size()));
  return out;
}

// The item a fixed-width step hands out: the values, or (values, column 0, column 1, ...).
py::object fixed_item(const at::Tensor& out, const at::Tensor& ext) {
  if (!ext.defined()) return py::reinterpret_steal<py::object>(THPVariable_Wrap(out));
  if (ext.dim() == 1)  // one column, already [rows] (alloc_extras)
    return py::make_tuple(py::reinterpret_steal<py::object>(THPVariable_Wrap(out)),
                          py::reinterpret_steal<py::object>(THPVariable_Wrap(ext)));
  py::list items;
  items.append(py::reinterpret_steal<py::object>(THPVariable_Wrap(out)));
  for (int64_t i = 0; i < ext.size(0); ++i) items.append(py::reinterpret_steal<py::object>(THPVariable_Wrap(ext[i])));
  return py::tuple(items);
}

// Makes `ks` the current stream of its device for the scope's allocations: the caching allocator
// then takes the blocks from (and orders their reuse against) that stream.  The device is already
// the current one, so unlike HIPStreamGuard this makes no hipGetDevice / hipSetDevice calls.
struct StreamScope {
  c10::hip::HIPStream prev;
  StreamScope(const c10::hip::HIPStream& ks, c10::DeviceIndex dev) : prev(c10::hip::getCurrentHIPStream(dev)) {
    c10::hip::setCurrentHIPStream(ks);
  }
  ~StreamScope() { c10::hip::setCurrentHIPStream(prev); }
};

// The first group of a size on a decode stream: the caching allocator has no block of it there
// yet, so each of the first few launches per stream paid a hipMalloc -- 40-80 us on the stepping
// thread, against 11 us for a warm launch, in the first 20-step window after warm-up
// (bench.py --window-trace; profiles/r04_s25).  Allocating and dropping as many blocks as a stream
// holds at once (the decode-ahead depth, the delivered batch, one spare) caches them on that
// stream up front.  Groups above 64 MiB are left alone (config 5's are 16 MiB).
void warm_group_blocks(MainDriver& d, hipStream_t ks, const std::vector<int64_t>& shape,
                       const at::TensorOptions& opts) {
  int64_t bytes = int64_t(c10::elementSize(c10::typeMetaToScalarType(opts.dtype())));
  for (auto x : shape) bytes *= x;
  if (bytes <= 0 || bytes > (int64_t(64) << 20)) return;
  for (const auto& w : d.warm_blocks_)
    if (w.first == ks && w.second == bytes) return;
  d.warm_blocks_.emplace_back(ks, bytes);
  std::vector<at::Tensor> hold;
  for (int i = 0; i < d.ahead_depth() + 2; ++i) hold.push_back(at::empty(shape, opts));
}

// Output block of a coalesced fixed-width launch.  Device decode runs on the driver's decode
// stream: allocate there, so the caching allocator orders the memory's reuse against that stream
// (no wait on the user's stream, which already waits for the previous group), and record the
// user's stream on it (the batches are used there).
at::Tensor alloc_group(MainDriver& d, const std::vector<int64_t>& shape, const at::TensorOptions& opts,
                       c10::DeviceIndex dev, bool span) {
  if (!span) return at::empty(shape, opts);
  const auto ks = c10::hip::getStreamFromExternal(d.next_decode_stream(), dev);
  at::Tensor all;
  {
    StreamScope scope(ks, dev);
    warm_group_blocks(d, ks.stream(), shape, opts);
    all = at::empty(shape, opts);
  }
  c10::hip::HIPCachingAllocator::recordStream(all.storage().data_ptr(), c10::hip::getCurrentHIPStream(dev));
  return all;
}

// Device decode ahead of delivery (MainDriver::ahead_begin): up to three full groups of staged
// batches are decoded while the user still works on earlier ones.  Pure C++ (ATen allocations,
// driver calls): the step functions release the GIL once around the call.  Returns the groups
// launched.
int launch_ahead(MainDriver& d, const std::vector<int64_t>& row_shape, const at::TensorOptions& opts,
                 c10::DeviceIndex dev, int dst_dt, const float* shift, const float* scale, int extras) {
  std::vector<int64_t> rows;
  int launched = 0;
  for (int q = 0; q < 3; ++q) {
    d.ahead_begin(&rows);
    if (rows.empty()) break;
    int64_t total = 0;
    for (auto x : rows) total += x;
    std::vector<int64_t> all_shape(row_shape);
    all_shape[0] = total;
    at::Tensor all = alloc_group(d, all_shape, opts, dev, true);
    std::vector<at::Tensor> ext = alloc_extras(d, rows, extras, dev, true);
    void* dsts[kMaxGroup];
    std::vector<std::shared_ptr<void>> handles;
    handles.reserve(rows.size());
    int64_t off = 0;
    for (size_t k = 0; k < rows.size(); ++k) {
      at::Tensor t = rows.size() == 1 ? all : all.narrow(0, off, rows[k]);
      dsts[k] = t.data_ptr();
      handles.emplace_back(fixed_handle(std::move(t), ext.empty() ? at::Tensor() : ext[k]));
      off += rows[k];
    }
    d.ahead_launch(dst_dt, dsts, shift, scale, std::move(handles));
    ++launched;
  }
  return launched;
}

// verify='deliver' on a device-decode path: waits for the delivered batch's verdict while
// launching, behind its kernel, the groups the workers finish meanwhile (`ahead`).  Waiting in
// MainDriver::verify_delivered instead leaves them staged until the next request, so with a
// shallow ring (config 5: 4 slots of 8 MiB) the GPU idled between each verdict and the next
// launch.  The caller's verify_delivered() then only reads the known verdict.  Called without
// the GIL.
template <class Ahead>
void verify_ahead(MainDriver& d, Ahead&& ahead) {
  const int64_t t0 = tk::now_ns();
  while (!d.delivered_verdict_known()) {
    ahead();
    if (tk::now_ns() - t0 < 200000) {
      for (int k = 0; k < 64; ++k) tk::cpu_relax();
    } else {
      timespec ts{0, 20000};
      nanosleep(&ts, nullptr);
    }
  }
  d.verify_wait_ns_ += tk::now_ns() - t0;
}

// verify='deliver': true when the delivered batch's device verdict is bad (the batches finished
// before it were made committable; parse_error() says why).
bool verdict_bad(MainDriver& d) {
  py::gil_scoped_release nogil;
  return d.verify_delivered() < 0;
}

// Padded width of a var-len batch: pad_to, else its longest row (rounded up to pad_multiple).
int64_t padded_len(const SlotView& s, int64_t pad_to, int64_t pad_multiple) {
  int64_t L = pad_to >= 0 ? pad_to : s.max_row_len;
  if (pad_to < 0 && pad_multiple > 1) L = (L + pad_multiple - 1) / pad_multiple * pad_multiple;
  return L;
}

// Outputs of a group of device-parsed JSON batches (kPackJsonSpan): ONE allocation holds the values
// of all of them, their lengths and their masks (256-byte aligned sub-blocks viewed with their
// dtypes), made on the decode stream the group runs on and recorded on the user's stream (as
// alloc_group): one allocator round trip and one free-time event per group.
void alloc_json_group(MainDriver& d, const int64_t* ms, const int64_t* Ls, const bool* devc, int n, int dst_dt,
                      bool want_mask, c10::DeviceIndex dev, std::shared_ptr<VarlenOut>* outs) {
  int64_t tot = 0, rows = 0;
  for (int k = 0; k < n; ++k) {
    tot += ms[k] * Ls[k];
    rows += ms[k];
  }
  const auto ks = c10::hip::getStreamFromExternal(d.next_decode_stream(), dev);
  auto up = [](int64_t x) { return (x + 255) / 256 * 256; };
  const at::ScalarType vt = scalar_type_of(dst_dt);
  const int64_t vbytes = up(tot * int64_t(c10::elementSize(vt))), lbytes = up(rows * 8);
  const int64_t mbytes = want_mask ? up(tot) : 0;
  at::Tensor all;
  {
    StreamScope scope(ks, dev);
    all = at::empty({vbytes + lbytes + mbytes}, at::TensorOptions().dtype(at::kByte).device(at::kCUDA, dev));
  }
  if (all.numel() > 0)
    c10::hip::HIPCachingAllocator::recordStream(all.storage().data_ptr(), c10::hip::getCurrentHIPStream(dev));
  const at::Tensor vals = all.narrow(0, 0, tot * int64_t(c10::elementSize(vt))).view(vt);
  const at::Tensor lens = all.narrow(0, vbytes, rows * 8).view(at::kLong);
  const at::Tensor masks = want_mask ? all.narrow(0, vbytes + lbytes, tot).view(at::kBool) : at::Tensor();
  int64_t vo = 0, ro = 0;
  for (int k = 0; k < n; ++k) {
    auto o = std::make_shared<VarlenOut>();
    o->vals = vals;
    o->lens = lens;
    o->masks = masks;
    o->vo = vo;
    o->ro = ro;
    o->m = ms[k];
    o->L = Ls[k];
    o->devc = devc[k];
    vo += ms[k] * Ls[k];
    ro += ms[k];
    outs[k] = std::move(o);
  }
}

// Device pointers of a group batch's region (the launch writes them before any view exists).
void* vals_ptr(const VarlenOut& o) {
  return static_cast<uint8_t*>(o.vals.data_ptr()) + o.vo * int64_t(o.vals.element_size());
}
int64_t* lens_ptr(const VarlenOut& o) { return o.lens.data_ptr<int64_t>() + o.ro; }
uint8_t* mask_ptr(const VarlenOut& o) {
  return o.masks.defined() ? static_cast<uint8_t*>(o.masks.data_ptr()) + o.vo : nullptr;
}

// Device JSON parse ahead of delivery (MainDriver::ahead_begin, as launch_ahead; no GIL).
int launch_ahead_json(MainDriver& d, int dst_dt, double pad, int64_t pad_to, int64_t pad_multiple, bool want_mask,
                      c10::DeviceIndex dev) {
  std::vector<int64_t> rows;
  int launched = 0;
  for (int q = 0; q < 3; ++q) {
    d.ahead_begin(&rows);
    if (rows.empty()) break;
    const int n = int(rows.size());
    int64_t ms[kMaxGroup], Ls[kMaxGroup];
    bool devc[kMaxGroup];
    for (int k = 0; k < n; ++k) {
      ms[k] = rows[size_t(k)];
      Ls[k] = padded_len(d.ahead_member(size_t(k)), pad_to, pad_multiple);
      devc[k] = (d.ahead_member(size_t(k)).flags & tk::kSlotDevCount) != 0;
    }
    std::shared_ptr<VarlenOut> o[kMaxGroup];
    alloc_json_group(d, ms, Ls, devc, n, dst_dt, want_mask, dev, o);
    void* outs[kMaxGroup];
    int64_t* lens[kMaxGroup];
    uint8_t* masks[kMaxGroup];
    std::vector<std::shared_ptr<void>> handles;
    handles.reserve(size_t(n));
    for (int k = 0; k < n; ++k) {
      outs[k] = vals_ptr(*o[k]);
      lens[k] = lens_ptr(*o[k]);
      masks[k] = mask_ptr(*o[k]);
      handles.emplace_back(std::move(o[k]));
    }
    d.ahead_launch_json(dst_dt, pad, outs, Ls, lens, masks, std::move(handles));
    ++launched;
  }
  return launched;
}

// One fixed-width step: finish + commit the previous batch, take the next one, collate it
// (coalesced with staged ones when cfg.grouped) into a tensor on the current stream.
py::tuple step_once(MainDriver& d, const MainDriver::FastConfig& cfg) {
  const auto dev = c10::DeviceIndex(cfg.device);
  hipStream_t stream = c10::hip::getCurrentHIPStream(dev).stream();
  const auto opts = at::TensorOptions().dtype(scalar_type_of(cfg.dst_dt)).device(at::kCUDA, dev);
  int cs = 0;
  int64_t r;
  if (!cfg.grouped) {
    at::Tensor out = at::empty(cfg.shape, opts);
    std::vector<at::Tensor> ext = alloc_extras(d, {cfg.shape[0]}, cfg.extras, dev, false);
    {
      py::gil_scoped_release nogil;
      r = d.step_fixed(stream, cfg.dst_dt, out.data_ptr(), cfg.row, cfg.shift, cfg.scale, cfg.auto_commit,
                       cfg.timeout_ms, &cs, &d.last);
    }
    if (r <= 0) return py::make_tuple(r, cs, py::none());
    if (cfg.verify && verdict_bad(d)) return py::make_tuple(-5, cs, py::none());
    at::Tensor e = ext.empty() ? at::Tensor() : ext[0];
    if (r < cfg.shape[0]) {
      out = out.narrow(0, 0, r);
      // a short batch's columns were written back to back: [extras, r] from the block's start
      if (e.defined())
        e = e.dim() == 1 ? e.narrow(0, 0, r) : e.reshape({-1}).narrow(0, 0, e.size(0) * r).view({e.size(0), r});
    }
    return py::make_tuple(r, cs, fixed_item(out, e));
  }
  std::vector<int64_t> rows;
  std::shared_ptr<void> pre;
  {
    py::gil_scoped_release nogil;
    r = d.step_group_begin(stream, cfg.auto_commit, cfg.timeout_ms, &cs, &rows, &pre);
  }
  if (r <= 0) return py::make_tuple(r, cs, py::none());
  at::Tensor out, ext;
  if (pre) {
    const auto* o = static_cast<FixedOut*>(pre.get());
    out = o->out;
    ext = o->ext;
  } else {
    int64_t total = 0;
    for (auto x : rows) total += x;
    std::vector<int64_t> all_shape(cfg.shape);
    all_shape[0] = total;
    const bool span = d.last.kind == uint32_t(tk::kPackRecordSpan);
    at::Tensor all = alloc_group(d, all_shape, opts, dev, span);
    std::vector<at::Tensor> exts = alloc_extras(d, rows, cfg.extras, dev, span);
    void* dsts[kMaxGroup];
    std::vector<std::shared_ptr<void>> handles;
    handles.reserve(rows.size());
    int64_t off = 0;
    for (size_t k = 0; k < rows.size(); ++k) {
      at::Tensor t = rows.size() == 1 ? all : all.narrow(0, off, rows[k]);
      dsts[k] = t.data_ptr();
      if (k == 0) {
        out = t;
        if (!exts.empty()) ext = exts[0];
      } else {
        handles.emplace_back(fixed_handle(std::move(t), exts.empty() ? at::Tensor() : exts[k]));
      }
      off += rows[k];
    }
    py::gil_scoped_release nogil;
    d.step_group_launch(stream, cfg.dst_dt, dsts, cfg.row, cfg.shift, cfg.scale, std::move(handles));
  }
  if (d.last.kind == uint32_t(tk::kPackRecordSpan)) {
    py::gil_scoped_release nogil;
    const int64_t ta = tk::now_ns();
    launch_ahead(d, cfg.shape, opts, dev, cfg.dst_dt, cfg.shift, cfg.scale, cfg.extras);
    d.ahead_ns_ += tk::now_ns() - ta;
    if (cfg.verify)
      verify_ahead(d, [&] { launch_ahead(d, cfg.shape, opts, dev, cfg.dst_dt, cfg.shift, cfg.scale, cfg.extras); });
  }
  if (cfg.verify && verdict_bad(d)) return py::make_tuple(-5, cs, py::none());
  return py::make_tuple(r, cs, fixed_item(out, ext));
}

// Var-len / JSON fast path: one call per batch -- finish + commit the previous batch, take the
// next slot, allocate [rows, L] + lengths (+ mask) on the current stream, launch the pad/stack (or
// JSON parse) kernel and mark the batch delivered; with verify='deliver' return once its verdict
// is known.  -> (r, commit_status, (out, lengths[, mask]) | None); r as next_slot(), or -5 when
// the batch's device verdict is bad (it is not handed out; parse_error() says why).
py::tuple varlen_step(MainDriver& d, const MainDriver::VarlenConfig& c) {
  const int device = c.device, dst_dt = c.dst_dt;
  const int64_t pad_to = c.pad_to, pad_multiple = c.pad_multiple, timeout_ms = c.timeout_ms;
  const double pad = c.pad;
  const bool want_mask = c.want_mask, auto_commit = c.auto_commit, verify = c.verify;
  const int64_t t0 = tk::now_ns();
  const auto dev = c10::DeviceIndex(device);
  hipStream_t stream = c10::hip::getCurrentHIPStream(dev).stream();
  int cs = 0;
  int r;
  int64_t t1, t2;
  size_t extra = 0;
  d.set_json_mult(pad_to >= 0 ? 0 : std::max<int64_t>(1, pad_multiple));
  {
    py::gil_scoped_release nogil;
    d.finish_delivered(stream);
    if (auto_commit) cs = d.commit_pending();
    t1 = tk::now_ns();
    if (d.coalesce() > 1) d.stage_ready(d.coalesce());  // let a group form (never blocks)
    r = d.next_slot(timeout_ms, &d.last);
    if (r == 1 && !d.last.pre) extra = d.json_group_extend();
    t2 = tk::now_ns();
  }
  d.ph_commit_ns_ += t1 - t0;
  d.ph_next_ns_ += t2 - t1;
  if (r != 1) return py::make_tuple(r, cs, py::none());
  SlotView& v = d.last;
  const int64_t n = int64_t(v.n_rows);
  at::Tensor out, lengths, mask;
  if (v.pre) {
    // parsed by an earlier group launch; a consumer on another stream waits for that kernel
    auto* o = static_cast<VarlenOut*>(v.pre_out.get());
    finish_json(d, v, o, dst_dt, pad, v.pre_stream);
    out = o->out;
    lengths = o->lengths;
    mask = o->mask;
    py::gil_scoped_release nogil;
    if (v.pre_stream != stream) d.wait_group(v, stream);
    d.deliver(v);
  } else if (row_span_kind(v.kind)) {
    // parsed from the logs by one launch with the staged JSON batches behind it
    const int ng = 1 + int(extra);
    int64_t ms[kMaxGroup], Ls[kMaxGroup];
    bool devc[kMaxGroup];
    for (int k = 0; k < ng; ++k) {
      const SlotView& s = k == 0 ? v : d.group_member(size_t(k - 1));
      ms[k] = int64_t(s.n_rows);
      Ls[k] = padded_len(s, pad_to, pad_multiple);
      devc[k] = (s.flags & tk::kSlotDevCount) != 0;
    }
    std::shared_ptr<VarlenOut> o[kMaxGroup];
    alloc_json_group(d, ms, Ls, devc, ng, dst_dt, want_mask, dev, o);
    void* outs[kMaxGroup];
    int64_t* lens[kMaxGroup];
    uint8_t* masks[kMaxGroup];
    std::vector<std::shared_ptr<void>> handles;
    handles.reserve(extra);
    for (int k = 0; k < ng; ++k) {
      outs[k] = vals_ptr(*o[k]);
      lens[k] = lens_ptr(*o[k]);
      masks[k] = mask_ptr(*o[k]);
    }
    for (int k = 1; k < ng; ++k) handles.emplace_back(std::move(o[k]));
    {
      py::gil_scoped_release nogil;
      d.json_group_launch(stream, dst_dt, pad, outs, Ls, lens, masks, std::move(handles));
    }
    finish_json(d, v, o[0].get(), dst_dt, pad, d.last_stream());
    out = o[0]->out;
    lengths = o[0]->lengths;
    mask = o[0]->mask;
    py::gil_scoped_release nogil;
    d.deliver(v);
  } else {
    auto alloc = [&](const SlotView& s, VarlenOut* o, int64_t* Lout) {
      const int64_t L = padded_len(s, pad_to, pad_multiple);
      const int64_t m = int64_t(s.n_rows);
      o->out = at::empty({m, L}, at::TensorOptions().dtype(scalar_type_of(dst_dt)).device(at::kCUDA, dev));
      o->lengths = at::empty({m}, at::TensorOptions().dtype(at::kLong).device(at::kCUDA, dev));
      if (want_mask) o->mask = at::empty({m, L}, at::TensorOptions().dtype(at::kBool).device(at::kCUDA, dev));
      *Lout = L;
    };
    if (extra == 0 || v.kind != uint32_t(tk::kPackJsonText)) {
      VarlenOut o;
      int64_t L;
      alloc(v, &o, &L);
      out = o.out;
      lengths = o.lengths;
      mask = o.mask;
      py::gil_scoped_release nogil;
      d.collate_varlen(v, stream, dst_dt, out.data_ptr(), L, pad, lengths.data_ptr<int64_t>(),
                       want_mask ? static_cast<uint8_t*>(mask.data_ptr()) : nullptr);
      d.deliver(v);
    } else {
      // one launch parses `last` and the staged JSON batches behind it
      void* outs[kMaxGroup];
      int64_t Ls[kMaxGroup];
      int64_t* lens[kMaxGroup];
      uint8_t* masks[kMaxGroup];
      std::vector<std::shared_ptr<void>> handles;
      handles.reserve(extra);
      for (size_t k = 0; k <= extra; ++k) {
        auto o = std::make_shared<VarlenOut>();
        alloc(k == 0 ? v : d.group_member(k - 1), o.get(), &Ls[k]);
        outs[k] = o->out.data_ptr();
        lens[k] = o->lengths.data_ptr<int64_t>();
        masks[k] = want_mask ? static_cast<uint8_t*>(o->mask.data_ptr()) : nullptr;
        if (k == 0) {
          out = o->out;
          lengths = o->lengths;
          mask = o->mask;
        } else {
          handles.emplace_back(std::move(o));
        }
      }
      py::gil_scoped_release nogil;
      d.json_group_launch(stream, dst_dt, pad, outs, Ls, lens, masks, std::move(handles));
      d.deliver(v);
    }
  }
  if (row_span_kind(v.kind)) {
    py::gil_scoped_release nogil;
    const int64_t ta = tk::now_ns();
    launch_ahead_json(d, dst_dt, pad, pad_to, pad_multiple, want_mask, dev);
    d.ahead_ns_ += tk::now_ns() - ta;
    if (verify)
      verify_ahead(d, [&] { launch_ahead_json(d, dst_dt, pad, pad_to, pad_multiple, want_mask, dev); });
  }
  d.ph_launch_ns_ += tk::now_ns() - t2;
  ++d.ph_steps_;
  if (verify && verdict_bad(d)) return py::make_tuple(-5, cs, py::none());
  ++d.fast_batches_;
  d.fast_records_ += n;
  d.fast_ns_ += tk::now_ns() - t0;
  py::object o = py::reinterpret_steal<py::object>(THPVariable_Wrap(std::move(out)));
  py::object l = py::reinterpret_steal<py::object>(THPVariable_Wrap(std::move(lengths)));
  py::tuple item = want_mask ? py::make_tuple(o, l, py::reinterpret_steal<py::object>(THPVariable_Wrap(std::move(mask))))
                             : py::make_tuple(o, l);
  return py::make_tuple(r, cs, item);
}

}  // namespace

void register_torch_step(py::module_& m) {
  // Argument-free fast path: the iteration's constants are set once, and each step is one
  // method call on the driver that also keeps the loader's batch/record/time counters, so the
  // per-batch Python work is a bound-method call and a tuple unpack.
  auto cls = py::reinterpret_borrow<py::class_<MainDriver>>(m.attr("MainDriver"));
  cls.def(
      "configure_fast",
      [](MainDriver& d, int device, std::vector<int64_t> shape, int dst_dt, int64_t row, uintptr_t shift,
         uintptr_t scale, bool auto_commit, int64_t timeout_ms, bool grouped, int extras, bool verify) {
        if (shape.empty()) throw std::invalid_argument("configure_fast: empty shape");
        scalar_type_of(dst_dt);  // validates
        auto& c = d.fast;
        c.device = device;
        c.shape = std::move(shape);
        c.dst_dt = dst_dt;
        c.row = row;
        c.shift = reinterpret_cast<const float*>(shift);
        c.scale = reinterpret_cast<const float*>(scale);
        c.auto_commit = auto_commit;
        c.timeout_ms = timeout_ms;
        c.grouped = grouped;
        c.extras = extras;
        c.verify = verify;
      },
      py::arg("device"), py::arg("shape"), py::arg("dst_dt"), py::arg("row"), py::arg("shift"), py::arg("scale"),
      py::arg("auto_commit"), py::arg("timeout_ms"), py::arg("grouped"), py::arg("extras") = 0,
      py::arg("verify") = false);
  cls.def("fast_next", [](MainDriver& d) -> py::tuple {
    const int64_t t0 = tk::now_ns();
    py::tuple res = step_once(d, d.fast);
    const int64_t r = res[0].cast<int64_t>();
    if (r > 0) {
      ++d.fast_batches_;
      d.fast_records_ += r;
      d.fast_ns_ += tk::now_ns() - t0;
    }
    return res;
  });

  // Var-len / JSON fast path: configured once per iteration, then one argument-free call per batch.
  cls.def(
      "configure_varlen",
      [](MainDriver& d, int device, int dst_dt, int64_t pad_to, int64_t pad_multiple, double pad, bool want_mask,
         bool auto_commit, int64_t timeout_ms, bool verify) {
        scalar_type_of(dst_dt);  // validates
        d.varlen = MainDriver::VarlenConfig{device, dst_dt, pad_to, pad_multiple, pad, want_mask, auto_commit,
                                            timeout_ms, verify};
      },
      py::arg("device"), py::arg("dst_dt"), py::arg("pad_to"), py::arg("pad_multiple"), py::arg("pad"),
      py::arg("want_mask"), py::arg("auto_commit"), py::arg("timeout_ms"), py::arg("verify") = false);
  cls.def("varlen_fast_next", [](MainDriver& d) { return varlen_step(d, d.varlen); });
  m.def(
      "step_fixed_tensor",
      [](MainDriver& d, int device, std::vector<int64_t> shape, int dst_dt, int64_t row, uintptr_t shift,
         uintptr_t scale, bool auto_commit, int64_t timeout_ms) -> py::tuple {
        const auto dev = c10::DeviceIndex(device);
        hipStream_t stream = c10::hip::getCurrentHIPStream(dev).stream();
        at::Tensor out = at::empty(shape, at::TensorOptions().dtype(scalar_type_of(dst_dt)).device(at::kCUDA, dev));
        int cs = 0;
        int64_t r;
        {
          py::gil_scoped_release nogil;
          r = d.step_fixed(stream, dst_dt, out.data_ptr(), row, reinterpret_cast<const float*>(shift),
                           reinterpret_cast<const float*>(scale), auto_commit, timeout_ms, &cs, &d.last);
        }
        if (r <= 0) return py::make_tuple(r, cs, py::none());
        if (r < shape[0]) out = out.narrow(0, 0, r);
        return py::make_tuple(r, cs, py::reinterpret_steal<py::object>(THPVariable_Wrap(std::move(out))));
      },
      py::arg("driver"), py::arg("device"), py::arg("shape"), py::arg("dst_dt"), py::arg("row"), py::arg("shift"),
      py::arg("scale"), py::arg("auto_commit"), py::arg("timeout_ms"),
      "finish+commit the previous batch, take the next slot and collate it into a new tensor "
      "allocated on the current stream -> (rows, commit_status, tensor | None)");

  // Coalesced variant: when several fixed-width batches are already staged, one allocation and
  // one kernel launch serve up to driver.coalesce of them; the following calls return the
  // pre-collated tensors without any HIP call (MainDriver::step_group_begin/launch).
  m.def(
      "step_fixed_group_tensor",
      [](MainDriver& d, int device, std::vector<int64_t> shape, int dst_dt, int64_t row, uintptr_t shift,
         uintptr_t scale, bool auto_commit, int64_t timeout_ms) -> py::tuple {
        const auto dev = c10::DeviceIndex(device);
        hipStream_t stream = c10::hip::getCurrentHIPStream(dev).stream();
        int cs = 0;
        int64_t r;
        std::vector<int64_t> rows;
        std::shared_ptr<void> pre;
        {
          py::gil_scoped_release nogil;
          r = d.step_group_begin(stream, auto_commit, timeout_ms, &cs, &rows, &pre);
        }
        if (r <= 0) return py::make_tuple(r, cs, py::none());
        at::Tensor out;
        if (pre) {
          out = static_cast<FixedOut*>(pre.get())->out;
        } else {
          int64_t total = 0;
          for (auto x : rows) total += x;
          std::vector<int64_t> all_shape(shape);
          all_shape[0] = total;
          at::Tensor all =
              alloc_group(d, all_shape, at::TensorOptions().dtype(scalar_type_of(dst_dt)).device(at::kCUDA, dev), dev,
                          d.last.kind == uint32_t(tk::kPackRecordSpan));
          void* dsts[kMaxGroup];
          std::vector<std::shared_ptr<void>> handles;
          handles.reserve(rows.size());
          int64_t off = 0;
          for (size_t k = 0; k < rows.size(); ++k) {
            at::Tensor t = rows.size() == 1 ? all : all.narrow(0, off, rows[k]);
            dsts[k] = t.data_ptr();
            if (k == 0)
              out = t;
            else
              handles.emplace_back(fixed_handle(std::move(t), at::Tensor()));
            off += rows[k];
          }
          py::gil_scoped_release nogil;
          d.step_group_launch(stream, dst_dt, dsts, row, reinterpret_cast<const float*>(shift),
                              reinterpret_cast<const float*>(scale), std::move(handles));
        }
        return py::make_tuple(r, cs, py::reinterpret_steal<py::object>(THPVariable_Wrap(std::move(out))));
      },
      py::arg("driver"), py::arg("device"), py::arg("shape"), py::arg("dst_dt"), py::arg("row"), py::arg("shift"),
      py::arg("scale"), py::arg("auto_commit"), py::arg("timeout_ms"),
      "coalesced step_fixed_tensor: up to driver.coalesce staged batches collated by one launch");
}

}  // namespace tkh
