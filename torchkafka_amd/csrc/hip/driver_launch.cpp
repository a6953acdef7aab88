// MainDriver's kernel launches (driver.h): the per-batch collates (fixed-width, var-len, raw
// payload), and the device-decode group launches -- fixed-width / var-len / JSON segments cut from
// the pinned broker logs (or their HBM mirror), their row tables and the kernel arguments
// (span_decode.h).  Split from driver.cpp; the slot, lockstep and commit side stays there.
#include "driver.h"

#include "dtypes.h"
#include "hip_queue.h"

#include <algorithm>
#include <cstring>

namespace tkh {

// ---------------------------------------------------------------------------------------------
// Kernel launches

void MainDriver::launch_group(const int* slots, const int64_t* rows, const size_t* voffs, int n, const SlotView& v,
                              hipStream_t stream, int dst_dt, void* const* dsts, int64_t row, const float* shift,
                              const float* scale) {
  if (v.kind == uint32_t(tk::kPackGatherFixed))
    eng_->collate_gather_group(slots, n, stream, v.src_dtype, dsts, dst_dt, rows, int64_t(v.row_bytes),
                               pins_->bases_dev(), shift, scale);
  else
    eng_->collate_fixed_group(slots, n, stream, voffs, v.src_dtype, dsts, dst_dt, rows, row, shift, scale);
}

void MainDriver::copy_extras(const int* slots, const SlotView* const* views, int n, hipStream_t stream) {
  for (int k = 0; k < n && k < ext_n_; ++k) {
    const SlotView& v = *views[k];
    if (v.extras_n && ext_dsts_[k])
      eng_->copy_bytes(slots[k], stream, size_t(v.extras_offset), ext_dsts_[k], size_t(v.n_rows) * v.extras_n * 8u);
  }
  ext_n_ = 0;
}

void MainDriver::collate_fixed(const SlotView& v, hipStream_t stream, int dst_dt, void* dst, int64_t row,
                               const float* shift, const float* scale) {
  const int slot = int(v.g);
  const SlotView* vs[1] = {&v};
  if (v.kind != uint32_t(tk::kPackRecordSpan) && ext_n_) copy_extras(&slot, vs, 1, stream);  // its event covers the copy
  bool record;
  note_handed(v.g, stream, &record);
  if (!record && coalesce_wait_ns_ > 0 && coalesce_ > 1) {
    // adaptive coalescing decides from the latest launch's completion: give this one its event
    force_event();
    record = true;
  }
  if (record) last_ev_slot_ = v.g;
  if (v.kind == uint32_t(tk::kPackRecordSpan)) {
    void* d = dst;
    int64_t pe;
    launch_span(&slot, vs, 1, stream, dst_dt, &d, shift, scale, record, &pe);
    handed_.back().perr = pe;
    handed_.back().span = true;
    last_perr_ = pe;
    return;
  }
  if (v.kind == uint32_t(tk::kPackGatherFixed)) {
    const int64_t rows = v.n_rows;
    void* d = dst;
    eng_->collate_gather_group(&slot, 1, stream, v.src_dtype, &d, dst_dt, &rows, int64_t(v.row_bytes),
                               pins_->bases_dev(), shift, scale, record);
    return;
  }
  eng_->collate_fixed(slot, stream, v.values_offset, v.src_dtype, dst, dst_dt, v.n_rows, row, shift, scale, record);
}

void MainDriver::collate_varlen(const SlotView& v, hipStream_t stream, int dst_dt, void* out, int64_t L, double pad,
                                int64_t* lengths, uint8_t* mask) {
  bool record;
  if (row_span_kind(v.kind)) {
    // decoded from the logs on the user's stream, its own completion event
    switch_stream(stream);
    const int slot = int(v.g);
    const SlotView* vs[1] = {&v};
    void* outs[1] = {out};
    const int64_t Ls[1] = {L};
    int64_t* lens[1] = {lengths};
    uint8_t* masks[1] = {mask};
    int64_t pe;
    launch_row_span(&slot, vs, 1, stream, dst_dt, pad, outs, Ls, lens, masks, true, &pe);
    group_handed(&slot, 1, stream, &pe, true, {}, 1);
    last_perr_ = pe;
    return;
  }
  if (v.kind == tk::kPackJsonText) {
    const int64_t idx = verdicts_->next_word();
    note_handed(v.g, stream, &record);
    handed_.back().perr = idx;
    eng_->collate_json(int(v.g), stream, v.values_offset, out, dst_dt, v.n_rows, L, pad, lengths, mask,
                       verdicts_->err_dev(idx), record);
    last_perr_ = idx;
    return;
  }
  note_handed(v.g, stream, &record);
  eng_->collate_varlen(int(v.g), stream, v.values_offset, v.src_dtype, out, dst_dt, v.n_rows, L, pad, lengths, mask,
                       record);
}

void MainDriver::copy_payload(const SlotView& v, hipStream_t stream, void* dst) {
  bool record;
  note_handed(v.g, stream, &record);
  force_event();  // copy_raw always records the slot's completion event
  eng_->copy_raw(int(v.g), stream, 0, dst, size_t(v.payload_bytes));
}

void MainDriver::check_seg_count(const tk::SpanSeg& sg, uint32_t i) const {
  constexpr uint32_t kWhole = tk::kSegCrcFirst | tk::kSegCrcLast;
  if ((sg.flags & tk::kSegCrc) && (sg.flags & kWhole) != kWhole && i >= uint32_t(BatchVerdicts::kPartials))
    throw std::runtime_error("driver: a batch splits RecordBatches into more than 512 device segments");
}

void MainDriver::fill_seg(SpanDevSeg& d, const tk::SpanSeg& sg, const uint8_t* src, int k, uint32_t i) {
  d = SpanDevSeg{};
  d.src = src;
  d.log_pos = sg.log_pos;
  d.len = sg.len;
  d.flags = sg.flags;
  d.crc = sg.crc;
  d.row_begin = sg.row_begin;
  d.row_end = sg.row_end;
  d.batch = uint16_t(k);
  d.seg = uint16_t(i);
}

void MainDriver::launch_span(const int* slots, const SlotView* const* views, int n, hipStream_t stream, int dst_dt,
                             void* const* dsts, const float* shift, const float* scale, bool record_last,
                             int64_t* perrs) {
  if (!broker_) throw std::runtime_error("driver: device decode needs the synthetic broker");
  verdicts_->ensure_partials();
  LogMirror* mirror = pins_->mirror();
  const SlotView& v0 = *views[0];
  SpanLaunch a{};
  a.row_elems = v0.max_row_len;
  const int ssz = dtype_size(v0.src_dtype), dsz = dtype_size(dst_dt);
  const int per = ssz > 0 ? 16 / ssz : 1;
  bool vec = ssz > 0 && a.row_elems % per == 0 && (a.row_elems * dsz) % 16 == 0;
  for (int k = 0; k < n; ++k) {
    vec = vec && reinterpret_cast<uintptr_t>(dsts[k]) % 16 == 0;
    perrs[k] = verdicts_->next_word();
    a.b[k].out = dsts[k];
    a.b[k].err = verdicts_->err_dev(perrs[k]);
    a.b[k].partials = verdicts_->partials_dev(perrs[k]);
    const SlotView& v = *views[k];
    if (v.extras_n && k < ext_n_ && ext_dsts_[k]) {  // key / timestamp columns ride in the same kernel
      a.b[k].ext_out = ext_dsts_[k];
      a.b[k].ext_off = v.extras_offset;
      a.b[k].ext_words = v.n_rows * v.extras_n;
    }
  }
  ext_n_ = 0;
  a.vec_store = vec ? 1 : 0;
  bool pcie = false;  // a segment of this launch is read over PCIe (not from the HBM mirror)
  auto flush = [&](bool record) {
    // segments split over parts only when every one is read from HBM: parts multiply the loads in
    // flight of a lone group from the mirror (2 MiB: 30.6 -> 12.6 us with 8), while over PCIe the
    // link is the limit and more workgroups only add their fixed costs (profiles/r05_s30_lane_merge)
    // ... and only when the mirror waits for its copies (LogMirror::waits): with the no-wait policy,
    // split segments failed the device CRC check at four ranks on one GPU (profiles/r06_s21, s23)
    a.parts = pcie || !mirror_splits(mirror) ? 1 : eng_->span_parts();
    split_launches_ += a.parts > 1;
    pcie = false;
    if (mirror) mirror->before(stream);
    eng_->collate_span(slots, n, stream, a, v0.src_dtype, dst_dt, shift, scale, record);
    if (mirror) mirror->after(stream);
  };
  for (int k = 0; k < n; ++k) {
    const tk::SpanSeg* sg = segs(*views[k]);
    for (uint32_t i = 0; i < views[k]->n_segs; ++i) {
      check_seg_count(sg[i], i);
      if (a.n_seg == kMaxLaunchSegs) {
        flush(false);
        a.n_seg = 0;
      }
      fill_seg(a.s[a.n_seg++], sg[i], seg_src(sg[i], &pcie), k, i);
    }
  }
  flush(record_last);
}

uint64_t MainDriver::stage_alloc(uint64_t bytes) {
  bytes = (bytes + 255) & ~uint64_t(255);
  if (bytes > kStageBytes) throw std::runtime_error("driver: a device JSON group exceeds the staging ring");
  if (!stage_dev_ && hipMalloc(reinterpret_cast<void**>(&stage_dev_), kStageBytes) != hipSuccess)
    throw std::runtime_error("driver: hipMalloc of the JSON staging ring failed");
  uint64_t pos = stage_head_;
  const uint64_t in = pos % kStageBytes;
  if (in + bytes > kStageBytes) pos += kStageBytes - in;  // never split a region: restart at the front
  while (pos + bytes - stage_tail_ > kStageBytes) {
    // the oldest groups still read their regions: wait for the first one with an event
    cover_handed();
    bool waited = false;
    for (const auto& h : handed_) {
      if (!h.ev) continue;
      eng_->wait_slot(int(h.g));
      waited = true;
      break;
    }
    if (!waited) throw std::logic_error("driver: JSON staging ring full with nothing in flight");
    pending_query_ns_ = 0;
    release_completed_impl();
  }
  stage_head_ = pos + bytes;
  stage_last_end_ = stage_head_;
  return pos % kStageBytes;
}

void MainDriver::launch_json_span(const int* slots, const SlotView* const* views, int n, hipStream_t stream,
                                  int dst_dt, double pad, void* const* outs, const int64_t* Ls,
                                  int64_t* const* lengths, uint8_t* const* masks, bool record_last, int64_t* perrs) {
  if (!broker_) throw std::runtime_error("driver: device JSON parse needs the synthetic broker");
  verdicts_->ensure_partials();
  LogMirror* mirror = pins_->mirror();
  tk::Ring& ring = poller_->ring();
  // staging per batch: the row descriptors, then one region per segment (row texts rounded up to
  // 16 bytes, or the float32 values of the rows the worker parsed)
  constexpr uint64_t kA = 256;
  auto up = [](uint64_t x, uint64_t a) { return (x + a - 1) / a * a; };
  // bytes of segment i's region in its batch's staging area
  auto seg_bytes = [&](const SlotView& v, const tk::SpanSeg& sg) {
    if (!(sg.flags & tk::kSegHostRows)) return up(up(sg.len, 16) + 16 * uint64_t(sg.row_end - sg.row_begin), kA);
    const auto* rows = reinterpret_cast<const tk::JsonSpanRow*>(ring.payload(uint32_t(v.g)));
    uint64_t b = 0;
    for (uint32_t r = sg.row_begin; r < sg.row_end; ++r) {
      int64_t c = rows[r].count;
      if (v.trunc_len >= 0 && c > v.trunc_len) c = v.trunc_len;
      b += up(uint64_t(c < 0 ? 0 : c) * 4, 16);
    }
    return up(b, kA);
  };
  uint64_t batch_bytes[kMaxGroup], total = 0;
  for (int k = 0; k < n; ++k) {
    const SlotView& v = *views[k];
    const tk::SpanSeg* sg = segs(v);
    uint64_t b = up(uint64_t(v.n_rows) * sizeof(JsonRowDesc), kA);
    for (uint32_t i = 0; i < v.n_segs; ++i) b += seg_bytes(v, sg[i]);
    batch_bytes[k] = b;
    total += b;
  }
  const uint64_t base = stage_alloc(total);
  JsonStageLaunch a{};
  bool pcie = false;
  JsonGroupArgs ga{};
  ga.n = n;
  ga.pad = float(pad);
  ga.err_tag = tk::kSpanParseErrBit;
  ga.mult = json_mult_;
  ga.fused_count = json_mult_ == 0 && json_fused_count_ ? 1 : 0;
  uint64_t off = base;
  for (int k = 0; k < n; ++k) {
    const SlotView& v = *views[k];
    perrs[k] = verdicts_->next_word();
    JsonStageBatch& b = a.b[k];
    if (v.flags & tk::kSlotDevCount) {  // tagged count words: nothing to zero per launch
      b.ctr = verdicts_->json_ctr_dev(perrs[k]);
      b.ctr_tag = verdicts_->ctr_tag(perrs[k]);
      ga.ctr[k] = b.ctr;
      ga.ctr_tag[k] = b.ctr_tag;
      ga.info[k] = verdicts_->json_info_dev(perrs[k]);
    }
    b.desc = reinterpret_cast<JsonRowDesc*>(stage_dev_ + off);
    const uint64_t dbytes = up(uint64_t(v.n_rows) * sizeof(JsonRowDesc), kA);
    b.stage = stage_dev_ + off + dbytes;
    b.err = verdicts_->err_dev(perrs[k]);
    b.partials = verdicts_->partials_dev(perrs[k]);
    b.trunc_len = v.trunc_len;
    ga.rows[k] = b.desc;
    ga.vals[k] = b.stage;
    ga.vals_cap[k] = batch_bytes[k] - dbytes;
    ga.out[k] = outs[k];
    ga.L[k] = Ls[k];
    ga.lengths[k] = lengths[k];
    ga.mask[k] = masks[k];
    ga.err[k] = b.err;
    ga.row_base[k + 1] = ga.row_base[k] + int64_t(v.n_rows);
    ga.trunc[k] = v.trunc_len;
    off += batch_bytes[k];
  }
  auto flush = [&]() {
    a.parts = pcie || !mirror_splits(mirror) ? 1 : eng_->json_span_parts();  // as launch_span
    split_launches_ += a.parts > 1;
    pcie = false;
    if (mirror) mirror->before(stream);
    eng_->collate_json_stage(slots, n, stream, a);
    if (mirror) mirror->after(stream);
  };
  for (int k = 0; k < n; ++k) {
    const SlotView& v = *views[k];
    const tk::SpanSeg* sg = segs(v);
    uint64_t soff = 0;  // offset in the batch's staging area (after its descriptors)
    for (uint32_t i = 0; i < v.n_segs; ++i) {
      check_seg_count(sg[i], i);
      if (a.n_seg == kMaxLaunchSegs) {
        flush();
        a.n_seg = 0;
      }
      SpanDevSeg& d = a.s[a.n_seg++];
      fill_seg(d, sg[i], (sg[i].flags & tk::kSegHostRows) ? nullptr : seg_src(sg[i], &pcie), k, i);
      d.stage_off = uint32_t(soff);
      soff += seg_bytes(v, sg[i]);
    }
  }
  flush();
  bool devc = false;
  for (int k = 0; k < n; ++k) devc = devc || ga.ctr[k] != nullptr;
  // a wave per row: counts, simple check, the width words.  Not fused into json_stage_kernel: its
  // few workgroups (one per segment) took 149 us per group doing it instead of 71 us, and config 4
  // fell from 40.5 M to 35.5 M rec/s (profiles/r04_s4).  With a fixed width (pad_to) no row waits
  // for another's count: the parse kernel's block of each row counts it (ga.fused_count).
  if (devc && !ga.fused_count) eng_->run_on(stream, [ga, stream] { launch_json_count(ga, stream); });
  // the parse: a block per row over the staged texts, on the same stream
  eng_->run_on(stream, [ga, dst_dt, stream]() mutable { launch_json_group(ga, dst_dt, stream); });
  if (record_last) eng_->record_done(slots[n - 1], stream);
}

void MainDriver::launch_var_span(const int* slots, const SlotView* const* views, int n, hipStream_t stream,
                                 int dst_dt, double pad, void* const* outs, const int64_t* Ls,
                                 int64_t* const* lengths, uint8_t* const* masks, bool record_last, int64_t* perrs) {
  if (!broker_) throw std::runtime_error("driver: device decode needs the synthetic broker");
  verdicts_->ensure_partials();
  LogMirror* mirror = pins_->mirror();
  VarSpanLaunch a{};
  bool pcie = false;
  const int src_dt = views[0]->src_dtype;
  for (int k = 0; k < n; ++k) {
    perrs[k] = verdicts_->next_word();
    VarSpanBatch& b = a.b[k];
    b.out = outs[k];
    b.L = Ls[k];
    b.lengths = lengths[k];
    b.mask = masks[k];
    b.err = verdicts_->err_dev(perrs[k]);
    b.partials = verdicts_->partials_dev(perrs[k]);
    b.trunc_len = views[k]->trunc_len;
    // vector stores of a 16-byte source group (16 / ssz elements of dsz bytes): rows and groups aligned
    const int ssz = dtype_size(src_dt), dsz = dtype_size(dst_dt);
    const int64_t gbytes = ssz > 0 ? int64_t(16 / ssz) * dsz : 0;
    b.reserved = (gbytes >= 16 && gbytes % 16 == 0 && reinterpret_cast<uintptr_t>(outs[k]) % 16 == 0 &&
                  (Ls[k] * dsz) % 16 == 0) ? 1 : 0;
  }
  auto flush = [&](bool record) {
    for (int k = 0; k < n; ++k) {
      a.b[k].slot = eng_->slot_src(slots[k], stream);  // DMA mode: after the slot's copy
      a.b[k].rows = reinterpret_cast<const tk::JsonSpanRow*>(a.b[k].slot);
    }
    a.tabs = eng_->span_tables();
    a.parts = pcie || !mirror_splits(mirror) ? 1 : eng_->span_parts();  // as launch_span
    a.part_acc = a.parts > 1 ? eng_->part_acc(stream) : nullptr;
    split_launches_ += a.parts > 1;
    pcie = false;
    if (mirror) mirror->before(stream);
    eng_->run_on(stream, [a, src_dt, dst_dt, pad, stream] { tkh::launch_var_span(a, src_dt, dst_dt, pad, stream); });
    if (mirror) mirror->after(stream);
    if (record) eng_->record_done(slots[n - 1], stream);
  };
  for (int k = 0; k < n; ++k) {
    const SlotView& v = *views[k];
    if (v.src_dtype != src_dt) throw std::invalid_argument("driver: a var-len group mixes element dtypes");
    const tk::SpanSeg* sg = segs(v);
    for (uint32_t i = 0; i < v.n_segs; ++i) {
      check_seg_count(sg[i], i);
      if (a.n_seg == kMaxLaunchSegs) {
        flush(false);
        a.n_seg = 0;
      }
      fill_seg(a.s[a.n_seg++], sg[i], (sg[i].flags & tk::kSegHostRows) ? nullptr : seg_src(sg[i], &pcie), k, i);
    }
  }
  flush(record_last);
}

}  // namespace tkh
