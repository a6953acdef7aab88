// MainDriver's coalesced steps (driver.h): forming a group of staged batches one kernel collates,
// launching it, and the groups decoded ahead of delivery (torch_step.cpp drives them).  Split from
// driver.cpp.
#include "driver.h"

#include "dtypes.h"
#include "hip_queue.h"

#include <algorithm>
#include <cstring>

namespace tkh {

// ---------------------------------------------------------------------------------------------
// Group formation and the coalesced steps

size_t MainDriver::json_group_extend() {
  group_idx_.clear();
  if (coalesce_ <= 1 || (last.kind != uint32_t(tk::kPackJsonText) && !row_span_kind(last.kind))) return 0;
  const auto& staged = poller_->staged();
  uint64_t bytes = last.span_bytes;
  for (size_t i = 0; i < staged.size() && int(1 + group_idx_.size()) < coalesce_; ++i) {
    const SlotView& v = staged[i];
    if (v.g < 0) continue;  // watermark-only slot: rides on the next delivered batch
    if (v.pre || v.kind != last.kind || v.n_rows == 0 || group_full(bytes, v)) break;
    bytes += v.span_bytes;
    group_idx_.push_back(i);
  }
  return group_idx_.size();
}

void MainDriver::json_group_launch(hipStream_t stream, int dst_dt, double pad, void* const* outs, const int64_t* Ls,
                                   int64_t* const* lengths, uint8_t* const* masks,
                                   std::vector<std::shared_ptr<void>>&& handles) {
  const int n = 1 + int(group_idx_.size());
  if (int(handles.size()) != n - 1) throw std::invalid_argument("driver: group handles do not match the group");
  auto& staged = poller_->staged();
  int slots[kMaxGroup];
  const SlotView* vs[kMaxGroup];
  for (int k = 0; k < n; ++k) {
    vs[k] = k == 0 ? &last : &staged[group_idx_[size_t(k - 1)]];
    slots[k] = int(vs[k]->g);
  }
  int64_t perrs[kMaxGroup];
  if (row_span_kind(last.kind)) {
    // decoded on the next decode stream (outputs allocated there, torch_step.cpp); the user's
    // stream waits for the group's completion
    cover_handed();
    hipStream_t ks = next_decode_stream();
    ++span_launches_;
    last_stream_ = ks;
    launch_row_span(slots, vs, n, ks, dst_dt, pad, outs, Ls, lengths, masks, true, perrs);
    last.perr = perrs[0];
    const int64_t gid = group_handed(slots, n, ks, perrs, true, std::move(handles), 1);
    wait_launch(slots[n - 1], gid, stream);
    group_idx_.clear();
    return;
  }
  size_t voffs[kMaxGroup];
  int64_t rows[kMaxGroup];
  int32_t* errs[kMaxGroup];
  for (int k = 0; k < n; ++k) {
    voffs[k] = vs[k]->values_offset;
    rows[k] = vs[k]->n_rows;
    perrs[k] = verdicts_->next_word();
    errs[k] = verdicts_->err_dev(perrs[k]);
  }
  last.perr = perrs[0];
  switch_stream(stream);
  eng_->collate_json_group(slots, n, stream, voffs, rows, outs, Ls, lengths, masks, errs, pad, dst_dt);
  group_handed(slots, n, stream, perrs, false, std::move(handles), 1);
  group_idx_.clear();
}

int64_t MainDriver::step_fixed(hipStream_t stream, int dst_dt, void* dst, int64_t row, const float* shift,
                               const float* scale, bool auto_commit, int64_t timeout_ms, int* commit_status,
                               SlotView* out) {
  *commit_status = 0;
  const int64_t t0 = tk::now_ns();
  finish_delivered(stream);  // asking for the next batch finishes the previous one
  if (auto_commit) *commit_status = commit_pending();
  const int64_t t1 = tk::now_ns();
  int r = next_slot(timeout_ms, out);
  const int64_t t2 = tk::now_ns();
  ph_commit_ns_ += t1 - t0;
  ph_next_ns_ += t2 - t1;
  if (r < 0) return r;
  collate_fixed(*out, stream, dst_dt, dst, row, shift, scale);
  set_delivered(*out);
  poller_->prefetch_ready();
  ph_launch_ns_ += tk::now_ns() - t2;
  ++ph_steps_;
  return out->n_rows;
}

int64_t MainDriver::step_group_begin(hipStream_t stream, bool auto_commit, int64_t timeout_ms, int* commit_status,
                                     std::vector<int64_t>* group_rows, std::shared_ptr<void>* pre_out) {
  *commit_status = 0;
  group_rows->clear();
  group_idx_.clear();
  const int64_t t0 = tk::now_ns();
  finish_delivered(stream);  // asking for the next batch finishes the previous one
  if (auto_commit) *commit_status = commit_pending();
  const int64_t t1 = tk::now_ns();
  auto& staged = poller_->staged();
  if (!ls_ && coalesce_ > 1) {
    // stage what the workers already published, so a group can form (never blocks)
    while (int(staged.size()) < prefetch_ + coalesce_) {
      const int r = poller_->poll(false, 0);
      if (r == -3) return -3;
      if (r <= 0) break;
    }
  }
  occ_handed_ += int64_t(handed_.size());
  occ_staged_ += int64_t(staged.size());
  ++occ_samples_;
  const int r = next_slot(timeout_ms, &last);
  const int64_t t2 = tk::now_ns();
  ph_commit_ns_ += t1 - t0;
  ph_next_ns_ += t2 - t1;
  if (r < 0) return r;
  if (last.pre) {
    // collated by an earlier group launch; a consumer on another stream waits for that kernel
    if (last.pre_stream != stream) wait_launch(last.pre_event_slot, last.pre_group, stream);
    *pre_out = std::move(last.pre_out);
    set_delivered(last);
    poller_->prefetch_ready();
    ++ph_steps_;
    return last.n_rows;
  }
  group_rows->push_back(last.n_rows);
  if (last.kind == uint32_t(tk::kPackFixed) || last.kind == uint32_t(tk::kPackGatherFixed) ||
      last.kind == uint32_t(tk::kPackRecordSpan)) {
    group_capped_ = false;
    extend_group();
    if (coalesce_wait_ns_ > 0 && int(1 + group_idx_.size()) < coalesce_ && !group_capped_) {
      const int64_t cw0 = tk::now_ns();
      const int64_t until = cw0 + coalesce_wait_ns_;
      while (int(1 + group_idx_.size()) < coalesce_ && !group_capped_ && gpu_busy() && tk::now_ns() < until) {
        const int r2 = poller_->poll(false, 0);
        if (r2 == -3) break;  // reported by the next call
        if (r2 == 1) {
          extend_group();
          continue;
        }
        release_completed();
        for (int k = 0; k < 16; ++k) tk::cpu_relax();
      }
      cwait_ns_ += tk::now_ns() - cw0;
    }
    for (size_t i : group_idx_) group_rows->push_back(staged[i].n_rows);
  }
  return last.n_rows;
}

// Appends to group_idx_ the staged batches right behind `last` that one kernel can collate with it.
void MainDriver::extend_group() {
  const auto& staged = poller_->staged();
  size_t i = group_idx_.empty() ? 0 : group_idx_.back() + 1;
  uint64_t bytes = last.span_bytes;
  for (size_t k : group_idx_) bytes += staged[k].span_bytes;
  for (; i < staged.size() && int(1 + group_idx_.size()) < coalesce_; ++i) {
    const SlotView& v = staged[i];
    if (v.g < 0) continue;  // watermark-only slot: rides on the next delivered batch
    if (group_full(bytes, v)) group_capped_ = true;
    if (v.pre || v.kind != last.kind || v.src_dtype != last.src_dtype || v.max_row_len != last.max_row_len ||
        v.row_bytes != last.row_bytes || v.shape != last.shape || v.n_rows == 0 || group_capped_)
      return;
    bytes += v.span_bytes;
    group_idx_.push_back(i);
  }
}

void MainDriver::step_group_launch(hipStream_t stream, int dst_dt, void* const* dsts, int64_t row,
                                   const float* shift, const float* scale,
                                   std::vector<std::shared_ptr<void>>&& handles) {
  const int64_t t0 = tk::now_ns();
  const int n = 1 + int(group_idx_.size());
  if (int(handles.size()) != n - 1) throw std::invalid_argument("driver: group handles do not match the group");
  auto& staged = poller_->staged();
  int slots[kMaxGroup];
  size_t voffs[kMaxGroup];
  int64_t rows[kMaxGroup];
  const SlotView* vs[kMaxGroup];
  for (int k = 0; k < n; ++k) {
    vs[k] = k == 0 ? &last : &staged[group_idx_[size_t(k - 1)]];
    slots[k] = int(vs[k]->g);
    voffs[k] = vs[k]->values_offset;
    rows[k] = vs[k]->n_rows;
  }
  if (last.kind == uint32_t(tk::kPackRecordSpan)) {
    // Device decode rotates over the decode streams: a group's kernel is PCIe-bound while it
    // loads and compute-bound in its CRC/extract tail, so the next group's loads overlap that
    // tail.  The outputs were allocated on the decode stream (torch_step.cpp: the caching
    // allocator orders their reuse against it, and knows the user's stream uses them); the
    // user's stream waits for the group's completion before it touches a batch of it.
    cover_handed();
    hipStream_t ks = next_decode_stream();
    ++span_launches_;
    last_stream_ = ks;
    int64_t perrs[kMaxGroup];
    launch_span(slots, vs, n, ks, dst_dt, dsts, shift, scale, true, perrs);
    last.perr = perrs[0];
    const int64_t gid = group_handed(slots, n, ks, perrs, true, std::move(handles), 1);
    wait_launch(slots[n - 1], gid, stream);
  } else if (n == 1) {
    collate_fixed(last, stream, dst_dt, dsts[0], row, shift, scale);
  } else {
    switch_stream(stream);
    if (ext_n_) copy_extras(slots, vs, n, stream);
    launch_group(slots, rows, voffs, n, last, stream, dst_dt, dsts, row, shift, scale);
    group_handed(slots, n, stream, nullptr, false, std::move(handles), 1);
  }
  group_idx_.clear();
  set_delivered(last);
  poller_->prefetch_ready();
  ph_launch_ns_ += tk::now_ns() - t0;
  ++ph_steps_;
}

void MainDriver::ahead_begin(std::vector<int64_t>* rows) {
  rows->clear();
  group_idx_.clear();
  if (ahead_depth_ <= 0 || coalesce_ <= 1) return;
  const auto& staged = poller_->staged();
  const size_t want = size_t(prefetch_ + (ahead_depth_ + 1) * coalesce_);
  while (staged.size() < want) {
    if (poller_->poll(false, 0) <= 0) break;  // nothing ready (an error is reported by next_slot)
  }
  int pre = 0;
  size_t i0 = staged.size();
  for (size_t i = 0; i < staged.size(); ++i) {
    const SlotView& v = staged[i];
    if (v.g < 0) continue;
    if (v.pre)
      ++pre;
    else if (i0 == staged.size())
      i0 = i;
  }
  if (pre >= ahead_depth_ * coalesce_ || i0 == staged.size()) return;
  const SlotView& f = staged[i0];
  const bool json = row_span_kind(f.kind);  // outputs sized per batch: no shape match needed
  if ((f.kind != uint32_t(tk::kPackRecordSpan) && !json) || f.n_rows == 0) return;
  uint64_t bytes = 0;
  bool capped = false;
  for (size_t i = i0; i < staged.size() && int(group_idx_.size()) < coalesce_; ++i) {
    const SlotView& v = staged[i];
    if (v.g < 0) continue;  // watermark-only slot: rides on the next delivered batch
    if (v.pre || v.kind != f.kind || v.n_rows == 0) break;
    if (group_full(bytes, v)) {
      capped = true;  // a full group by bytes
      break;
    }
    bytes += v.span_bytes;
    if (!json && (v.src_dtype != f.src_dtype || v.max_row_len != f.max_row_len || v.row_bytes != f.row_bytes ||
                  v.shape != f.shape))
      break;
    group_idx_.push_back(i);
  }
  // a group that could not take one more batch of its last one's size is full without waiting to
  // see that batch: config 5 (8 MiB batches, 16 MiB groups, a 4-slot ring) never has a third
  // batch staged while two are in flight, so its groups would otherwise never go ahead
  if (!capped && !group_idx_.empty() && bytes + staged[group_idx_.back()].span_bytes > group_bytes_max_)
    capped = true;
  if (int(group_idx_.size()) < coalesce_ && !capped) {  // only full groups go ahead; the rest waits for the user
    group_idx_.clear();
    return;
  }
  for (size_t i : group_idx_) rows->push_back(staged[i].n_rows);
}

void MainDriver::ahead_launch(int dst_dt, void* const* dsts, const float* shift, const float* scale,
                              std::vector<std::shared_ptr<void>>&& handles) {
  const int n = int(group_idx_.size());
  if (n < 1 || int(handles.size()) != n) throw std::invalid_argument("driver: ahead group does not match");
  const int64_t t0 = tk::now_ns();
  auto& staged = poller_->staged();
  int slots[kMaxGroup];
  const SlotView* vs[kMaxGroup];
  for (int k = 0; k < n; ++k) {
    vs[k] = &staged[group_idx_[size_t(k)]];
    slots[k] = int(vs[k]->g);
  }
  cover_handed();
  hipStream_t ks = next_decode_stream();
  ++span_launches_;
  last_stream_ = ks;
  int64_t perrs[kMaxGroup];
  launch_span(slots, vs, n, ks, dst_dt, dsts, shift, scale, true, perrs);
  group_handed(slots, n, ks, perrs, true, std::move(handles), 0);
  group_idx_.clear();
  ++ahead_groups_;
  ph_launch_ns_ += tk::now_ns() - t0;
}

void MainDriver::ahead_launch_json(int dst_dt, double pad, void* const* outs, const int64_t* Ls,
                                   int64_t* const* lengths, uint8_t* const* masks,
                                   std::vector<std::shared_ptr<void>>&& handles) {
  const int n = int(group_idx_.size());
  if (n < 1 || int(handles.size()) != n) throw std::invalid_argument("driver: ahead group does not match");
  const int64_t t0 = tk::now_ns();
  auto& staged = poller_->staged();
  int slots[kMaxGroup];
  const SlotView* vs[kMaxGroup];
  for (int k = 0; k < n; ++k) {
    vs[k] = &staged[group_idx_[size_t(k)]];
    slots[k] = int(vs[k]->g);
  }
  cover_handed();
  hipStream_t ks = next_decode_stream();
  ++span_launches_;
  last_stream_ = ks;
  int64_t perrs[kMaxGroup];
  launch_row_span(slots, vs, n, ks, dst_dt, pad, outs, Ls, lengths, masks, true, perrs);
  group_handed(slots, n, ks, perrs, true, std::move(handles), 0);
  group_idx_.clear();
  ++ahead_groups_;
  ph_launch_ns_ += tk::now_ns() - t0;
}

}  // namespace tkh
