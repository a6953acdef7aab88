// Device verdicts of the batches the driver launched: one status word per device-checked batch.
//
// A batch decoded or parsed on the GPU (span decode: CRC32C of every RecordBatch; JSON: the
// grammar of every row) may only be committed once its kernel reported it clean.  Each launch
// takes a word from a ring of kWords host-mapped int32s (-1 clean, else the failing segment or
// row), plus, for span decode, kPartials raw CRC words of RecordBatches split over segments (the
// host chains them at slot release, crc32c_shift_raw) and, for device-counted JSON, {width, rows
// left to the host, done}.  The driver reads a word when the batch's slot is released (its
// kernel completed) and only then lets the batch become committable.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "broker.h"
#include "engine.h"
#include "ring.h"

namespace tkh {

class BatchVerdicts {
 public:
  static constexpr int64_t kWords = 4096;
  static constexpr int64_t kPartials = 512;  // raw CRC words per status word (segments of one slot)

  // `queue`: the loader's HIP command queue (its parse launches are queued there)
  BatchVerdicts(tk::Ring* ring, tk::Broker* broker, HipQueue* queue) : ring_(ring), broker_(broker), q_(queue) {}
  ~BatchVerdicts();
  BatchVerdicts(const BatchVerdicts&) = delete;
  BatchVerdicts& operator=(const BatchVerdicts&) = delete;

  // A fresh word for the next launch (reused after kWords launches; its batch was settled long
  // before -- fenced batches settle in order and the ring holds far fewer slots).
  int64_t next_word();
  void ensure_partials();  // span decode: the partial-CRC words
  int32_t* err_dev(int64_t w) const { return perr_dev_ + w; }
  uint32_t* partials_dev(int64_t w) const { return part_dev_ + w * kPartials; }
  int32_t* json_info_dev(int64_t w) const { return jinfo_dev_ + w * 4; }
  // Device-counted JSON: word w's count words in HBM (zeroed once: width, rows left to the host,
  // both tagged; two spare) and the tag of its current launch (the number of times w was taken:
  // higher than every earlier tag of these words).
  static constexpr int64_t kCtrWords = 4;
  unsigned long long* json_ctr_dev(int64_t w) const { return ctr_dev_ + w * kCtrWords; }
  uint32_t ctr_tag(int64_t w) const { return tag_[size_t(w)]; }

  // 0 kernel pending, 1 clean, 2 malformed (read when the slot was released)
  uint8_t state(int64_t w) const { return state_[size_t(w)]; }
  // The kernel of slot g (word w) completed: read its verdict.  `span`: a log-decoded batch
  // (chain split RecordBatch CRCs; device-counted JSON rows the device left to the host are
  // parsed now, while the slot's row table is still held).
  void on_release(int64_t g, int64_t w, bool span);
  // Why word w's batch (offsets wms) is never committed.
  std::string failure(int64_t w, const std::vector<tk::Watermark>& wms) const;

  // Device-counted JSON (kSlotDevCount): the width the parse kernel chose for the batch (waits for
  // its first block), rows it left to the host in *n_host, and those rows written on `stream`.
  int64_t json_width(int64_t w, int64_t* n_host);
  int64_t width_wait_ns = 0;  // host time json_width spent waiting for a parse kernel's report
  void json_host_rows(int64_t g, int64_t w, int32_t trunc_len, void* out, int64_t L, int dst_dt, double pad,
                      int64_t* lengths, uint8_t* mask, hipStream_t stream);

 private:
  void ensure_status();
  void check_span(int64_t g, int64_t w);
  void parse_host_rows(int64_t g, int64_t w);
  void mark_bad(int64_t w, int64_t row);

  struct HostRow {
    int64_t row;
    int32_t count;
    std::vector<float> vals;
  };
  tk::Ring* ring_;
  tk::Broker* broker_;
  int32_t* perr_host_ = nullptr;  // hipHostMalloc'ed, device-mapped status words
  int32_t* perr_dev_ = nullptr;
  uint32_t* part_host_ = nullptr;  // partial CRCs, kPartials per word
  uint32_t* part_dev_ = nullptr;
  int32_t* jinfo_host_ = nullptr;  // device-counted JSON: {width, rows left to the host, done} per word
  int32_t* jinfo_dev_ = nullptr;
  unsigned long long* ctr_dev_ = nullptr;  // [kWords][kCtrWords] count words (device memory)
  std::vector<uint32_t> tag_;
  std::vector<uint8_t> state_;
  std::vector<std::string> msg_;  // span decode: the message of a bad batch, by word
  std::vector<std::vector<HostRow>> jrows_;
  std::vector<uint8_t> jparsed_;  // per word: its host rows were parsed (jrows_)
  uint8_t* patch_dev_ = nullptr;  // one host-parsed row at a time
  size_t patch_cap_ = 0;
  uint64_t seq_ = 0;
  HipQueue* q_ = nullptr;  // the loader's command queue
};

}  // namespace tkh
