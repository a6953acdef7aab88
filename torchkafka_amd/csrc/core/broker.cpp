#include "broker.h"

#include "codecs.h"
#include "crc32c.h"

#include <fcntl.h>

#include <array>
#include <linux/falloc.h>
#include <signal.h>
#include <sys/file.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <thread>

namespace tk {

// ------------------------------------------------------------ robust mutex
void init_robust_mutex(pthread_mutex_t* m) {
  pthread_mutexattr_t a;
  pthread_mutexattr_init(&a);
  pthread_mutexattr_setpshared(&a, PTHREAD_PROCESS_SHARED);
  pthread_mutexattr_setrobust(&a, PTHREAD_MUTEX_ROBUST);
  pthread_mutex_init(m, &a);
  pthread_mutexattr_destroy(&a);
}

RobustLock::RobustLock(pthread_mutex_t* m) : m_(m) {
  int rc = pthread_mutex_lock(m_);
  if (rc == EOWNERDEAD) {
    // The previous owner died inside the critical section.  Every critical
    // section below publishes with a final atomic store, so the protected
    // state is consistent up to the last publish; adopt the lock.
    pthread_mutex_consistent(m_);
  } else if (rc != 0) {
    errno = rc;
    throw_errno("pthread_mutex_lock");
  }
}
RobustLock::~RobustLock() { pthread_mutex_unlock(m_); }

// ------------------------------------------------------------ helpers
namespace {

void mkdir_p(const std::string& path) {
  std::string cur;
  for (size_t i = 0; i < path.size(); ++i) {
    cur.push_back(path[i]);
    if ((path[i] == '/' && i > 0) || i + 1 == path.size()) {
      if (mkdir(cur.c_str(), 0777) != 0 && errno != EEXIST) throw_errno("mkdir " + cur);
    }
  }
}

struct Layout {
  size_t topics, parts, groups, owners, offsets, total;
};

Layout layout_for(uint32_t max_topics, uint32_t max_parts, uint32_t max_groups) {
  Layout L;
  size_t off = align_up(sizeof(MetaHeader), 4096);
  L.topics = off;
  off = align_up(off + sizeof(TopicEntry) * max_topics, 4096);
  L.parts = off;
  off = align_up(off + sizeof(PartitionEntry) * max_parts, 4096);
  L.groups = off;
  off = align_up(off + sizeof(GroupEntry) * max_groups, 4096);
  L.owners = off;
  off = align_up(off + sizeof(int16_t) * size_t(max_groups) * max_parts, 4096);
  L.offsets = off;
  off = align_up(off + sizeof(OffsetEntry) * size_t(max_groups) * max_parts, 4096);
  L.total = off;
  return L;
}

void* map_file(const std::string& path, size_t len, bool create_size) {
  int fd = open(path.c_str(), O_RDWR | O_CREAT, 0666);
  if (fd < 0) throw_errno("open " + path);
  if (create_size) {
    struct stat st;
    if (fstat(fd, &st) != 0) { close(fd); throw_errno("fstat " + path); }
    if (size_t(st.st_size) < len && ftruncate(fd, off_t(len)) != 0) {
      close(fd);
      throw_errno("ftruncate " + path);
    }
  }
  void* p = mmap(nullptr, len, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  if (p == MAP_FAILED) throw_errno("mmap " + path);
  return p;
}

std::string part_path(const std::string& dir, uint32_t pidx, const char* ext) {
  char buf[32];
  snprintf(buf, sizeof(buf), "/p%05u.%s", pidx, ext);
  return dir + buf;
}

inline uint64_t mix64(uint64_t x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdULL;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ULL;
  x ^= x >> 33;
  return x;
}

}  // namespace

// ------------------------------------------------------------ construction
std::string Broker::url_to_dir(const std::string& url) {
  const std::string shm = "shm://", file = "file://";
  if (url.rfind(shm, 0) == 0) {
    std::string name = url.substr(shm.size());
    if (name.empty() || name.find('/') != std::string::npos || name == "." || name == "..")
      throw std::invalid_argument("bad shm broker name in '" + url + "'");
    return "/dev/shm/torchkafka/" + name;
  }
  if (url.rfind(file, 0) == 0) return url.substr(file.size());
  return url;
}

Broker::Broker(const std::string& url, bool create, const BrokerConfig& cfg) : dir_(url_to_dir(url)) {
  if (create) mkdir_p(dir_);
  struct stat st;
  if (stat(dir_.c_str(), &st) != 0) throw KafkaError("NoBrokersAvailable: no broker at '" + url + "'");
  map_meta(create, cfg);
  maps_.resize(meta_->max_partitions);
}

Broker::~Broker() {
  for (auto& m : maps_) {
    if (m.log) munmap(m.log, m.log_len);
    if (m.idx) munmap(m.idx, m.idx_len);
  }
  if (meta_map_) munmap(meta_map_, meta_len_);
}

void Broker::map_meta(bool create, const BrokerConfig& cfg) {
  const std::string lock_path = dir_ + "/lock", meta_path = dir_ + "/meta";
  int lfd = open(lock_path.c_str(), O_RDWR | (create ? O_CREAT : 0), 0666);
  if (lfd < 0) throw KafkaError("NoBrokersAvailable: cannot open broker at '" + dir_ + "'");
  if (flock(lfd, LOCK_EX) != 0) { close(lfd); throw_errno("flock"); }
  struct Unlock {
    int fd;
    ~Unlock() { flock(fd, LOCK_UN); close(fd); }
  } unlock{lfd};

  int fd = open(meta_path.c_str(), O_RDWR | (create ? O_CREAT : 0), 0666);
  if (fd < 0) throw KafkaError("NoBrokersAvailable: broker meta missing in '" + dir_ + "'");
  struct stat st;
  fstat(fd, &st);
  if (st.st_size == 0) {
    if (!create) { close(fd); throw KafkaError("NoBrokersAvailable: broker not initialised"); }
    Layout L = layout_for(cfg.max_topics, cfg.max_partitions, cfg.max_groups);
    if (ftruncate(fd, off_t(L.total)) != 0) { close(fd); throw_errno("ftruncate meta"); }
    void* p = mmap(nullptr, L.total, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    if (p == MAP_FAILED) throw_errno("mmap meta");
    meta_map_ = static_cast<uint8_t*>(p);
    meta_len_ = L.total;
    meta_ = reinterpret_cast<MetaHeader*>(meta_map_);
    meta_->magic = kBrokerMagic;
    meta_->version = kBrokerVersion;
    meta_->max_topics = cfg.max_topics;
    meta_->max_partitions = cfg.max_partitions;
    meta_->max_groups = cfg.max_groups;
    meta_->group_initial_rebalance_delay_ms = cfg.group_initial_rebalance_delay_ms;
    meta_->default_log_capacity = cfg.default_log_capacity;
    meta_->default_index_capacity = cfg.default_index_capacity;
    init_robust_mutex(&meta_->lock);
    auto* parts = reinterpret_cast<PartitionEntry*>(meta_map_ + L.parts);
    for (uint32_t i = 0; i < cfg.max_partitions; ++i) init_robust_mutex(&parts[i].lock);
    auto* offs = reinterpret_cast<OffsetEntry*>(meta_map_ + L.offsets);
    for (size_t i = 0; i < size_t(cfg.max_groups) * cfg.max_partitions; ++i) offs[i].offset.store(-1);
    auto* own = reinterpret_cast<int16_t*>(meta_map_ + L.owners);
    std::fill(own, own + size_t(cfg.max_groups) * cfg.max_partitions, int16_t(-1));
    meta_->ready.store(1, std::memory_order_release);
  } else {
    MetaHeader hdr;
    if (pread(fd, &hdr, sizeof(uint64_t) + 8 + 16, 0) < 0) { close(fd); throw_errno("read meta"); }
    if (hdr.magic != kBrokerMagic || hdr.version != kBrokerVersion) {
      close(fd);
      throw KafkaError("broker directory '" + dir_ + "' has an incompatible format");
    }
    Layout L = layout_for(hdr.max_topics, hdr.max_partitions, hdr.max_groups);
    void* p = mmap(nullptr, L.total, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    if (p == MAP_FAILED) throw_errno("mmap meta");
    meta_map_ = static_cast<uint8_t*>(p);
    meta_len_ = L.total;
    meta_ = reinterpret_cast<MetaHeader*>(meta_map_);
  }
  Layout L = layout_for(meta_->max_topics, meta_->max_partitions, meta_->max_groups);
  topics_ = reinterpret_cast<TopicEntry*>(meta_map_ + L.topics);
  parts_ = reinterpret_cast<PartitionEntry*>(meta_map_ + L.parts);
  groups_ = reinterpret_cast<GroupEntry*>(meta_map_ + L.groups);
  owners_ = reinterpret_cast<int16_t*>(meta_map_ + L.owners);
  offsets_ = reinterpret_cast<OffsetEntry*>(meta_map_ + L.offsets);
}

// ------------------------------------------------------------ topics
TopicInfo Broker::create_topic(const std::string& name, uint32_t n_partitions, uint64_t log_capacity,
                               uint64_t index_capacity) {
  if (name.empty() || name.size() >= kNameLen) throw std::invalid_argument("bad topic name");
  if (n_partitions == 0) throw std::invalid_argument("a topic needs at least one partition");
  TopicInfo info;
  {
    RobustLock l(&meta_->lock);
    if (find_topic(name, &info)) return info;
    const uint32_t ti = meta_->n_topics.load();
    const uint32_t first = meta_->n_partitions.load();
    if (ti >= meta_->max_topics) throw KafkaError("broker topic table full");
    if (first + n_partitions > meta_->max_partitions) throw KafkaError("broker partition table full");
    if (!log_capacity) log_capacity = meta_->default_log_capacity;
    if (!index_capacity) index_capacity = meta_->default_index_capacity;
    for (uint32_t i = 0; i < n_partitions; ++i) {
      const uint32_t pidx = first + i;
      PartitionEntry& P = parts_[pidx];
      P.high_watermark.store(0);
      P.log_start_offset.store(0);
      P.log_end_pos.store(0);
      P.n_batches.store(0);
      P.log_capacity = log_capacity;
      P.index_capacity = index_capacity;
      P.topic_index = ti;
      P.partition = i;
      P.fetch_delay_ns.store(0);
      P.fetch_errors.store(0);
      P.ring_bytes.store(0);
      P.first_batch.store(0);
      // Create (sparse) backing files now so readers can map them.
      void* a = map_file(part_path(dir_, pidx, "log"), log_capacity, true);
      munmap(a, log_capacity);
      void* b = map_file(part_path(dir_, pidx, "idx"), index_capacity * sizeof(IndexEntry), true);
      munmap(b, index_capacity * sizeof(IndexEntry));
    }
    TopicEntry& T = topics_[ti];
    std::memset(T.name, 0, kNameLen);
    std::memcpy(T.name, name.data(), name.size());
    T.n_partitions = n_partitions;
    T.first_pidx = first;
    T.log_capacity = log_capacity;
    T.index_capacity = index_capacity;
    meta_->n_partitions.store(first + n_partitions, std::memory_order_release);
    meta_->n_topics.store(ti + 1, std::memory_order_release);
    info.index = ti;
    info.n_partitions = n_partitions;
    info.first_pidx = first;
    info.name = name;
  }
  return info;
}

bool Broker::find_topic(const std::string& name, TopicInfo* out) const {
  const uint32_t n = meta_->n_topics.load(std::memory_order_acquire);
  for (uint32_t i = 0; i < n; ++i) {
    if (name == topics_[i].name) {
      out->index = i;
      out->n_partitions = topics_[i].n_partitions;
      out->first_pidx = topics_[i].first_pidx;
      out->name = name;
      return true;
    }
  }
  return false;
}

std::vector<TopicInfo> Broker::topics() const {
  std::vector<TopicInfo> v;
  const uint32_t n = meta_->n_topics.load(std::memory_order_acquire);
  for (uint32_t i = 0; i < n; ++i)
    v.push_back(TopicInfo{i, topics_[i].n_partitions, topics_[i].first_pidx, topics_[i].name});
  return v;
}

PartitionEntry& Broker::part(uint32_t pidx) {
  if (pidx >= meta_->n_partitions.load(std::memory_order_acquire)) throw std::out_of_range("bad partition index");
  return parts_[pidx];
}
const PartitionEntry& Broker::part(uint32_t pidx) const {
  if (pidx >= meta_->n_partitions.load(std::memory_order_acquire)) throw std::out_of_range("bad partition index");
  return parts_[pidx];
}

Broker::Mapped& Broker::mapped(uint32_t pidx) {
  Mapped& m = maps_.at(pidx);
  if (__atomic_load_n(&m.idx, __ATOMIC_ACQUIRE)) return m;
  std::lock_guard<std::mutex> g(maps_mu_);
  if (!m.idx) {
    const PartitionEntry& P = part(pidx);
    m.log_len = P.log_capacity;
    m.idx_len = P.index_capacity * sizeof(IndexEntry);
    m.log = static_cast<uint8_t*>(map_file(part_path(dir_, pidx, "log"), m.log_len, false));
    auto* idx = static_cast<IndexEntry*>(map_file(part_path(dir_, pidx, "idx"), m.idx_len, false));
    __atomic_store_n(&m.idx, idx, __ATOMIC_RELEASE);
  }
  return m;
}

const uint8_t* Broker::log_base(uint32_t pidx) { return mapped(pidx).log; }
const IndexEntry* Broker::index_base(uint32_t pidx) { return mapped(pidx).idx; }

int64_t Broker::find_batch(uint32_t pidx, int64_t offset, int64_t hint) {
  const PartitionEntry& P = part(pidx);
  const IndexEntry* idx = mapped(pidx).idx;
  const uint64_t icap = P.index_capacity;
  const int64_t nb = int64_t(P.n_batches.load(std::memory_order_acquire));
  const int64_t first = int64_t(P.first_batch.load(std::memory_order_acquire));
  auto at = [&](int64_t i) -> const IndexEntry& { return idx[uint64_t(i) % icap]; };
  auto contains = [&](int64_t i) {
    return i >= first && i < nb && at(i).base_offset <= offset && offset <= at(i).base_offset + at(i).last_offset_delta;
  };
  if (contains(hint)) return hint;
  if (contains(hint + 1)) return hint + 1;
  int64_t lo = first, hi = nb;  // first entry with base_offset > offset
  while (lo < hi) {
    int64_t mid = lo + (hi - lo) / 2;
    if (at(mid).base_offset <= offset) lo = mid + 1; else hi = mid;
  }
  int64_t i = lo - 1;
  if (contains(i)) return i;
  // an offset in a gap (compacted away, or a dropped transaction marker of a replica) reads
  // from the next batch; the record walk skips offsets below the position
  if (lo < nb && offset >= P.log_start_offset.load(std::memory_order_acquire)) return lo;
  throw OffsetOutOfRange("offset " + std::to_string(offset) + " not in log");
}

std::pair<int64_t, int64_t> Broker::offset_for_time(uint32_t pidx, int64_t ts) {
  const PartitionEntry& P = part(pidx);
  const Mapped& m = mapped(pidx);
  const int64_t nb = int64_t(P.n_batches.load(std::memory_order_acquire));
  const int64_t start = P.log_start_offset.load(std::memory_order_acquire);
  for (int64_t i = int64_t(P.first_batch.load(std::memory_order_acquire)); i < nb; ++i) {
    const IndexEntry& e = m.idx[uint64_t(i) % P.index_capacity];
    if (e.base_offset + e.last_offset_delta < start || e.max_timestamp < ts) continue;
    const uint8_t* bp = m.log + e.pos;
    BatchHeader h = parse_batch_header(bp, e.size);
    RecordIter it(bp, h);
    RecordView r;
    while (it.next(&r))
      if (r.offset >= start && r.timestamp >= ts) return {r.offset, r.timestamp};
  }
  return {-1, -1};
}

// ------------------------------------------------------------ produce
int64_t Broker::append(uint32_t pidx, const RecordIn* recs, size_t n) {
  if (n == 0) throw std::invalid_argument("empty batch");
  PartitionEntry& P = part(pidx);
  Mapped& m = mapped(pidx);
  int64_t min_ts = recs[0].timestamp;
  for (size_t i = 1; i < n; ++i) min_ts = std::min(min_ts, recs[i].timestamp);
  const size_t size = batch_encoded_size(recs, n, min_ts);
  RobustLock l(&P.lock);
  const uint64_t pos = P.log_end_pos.load(std::memory_order_relaxed);
  const uint64_t nb = P.n_batches.load(std::memory_order_relaxed);
  if (pos + size > P.log_capacity)
    throw KafkaError("partition log full (capacity " + std::to_string(P.log_capacity) + " bytes)");
  if (nb >= P.index_capacity) throw KafkaError("partition index full");
  const int64_t base = P.high_watermark.load(std::memory_order_relaxed);
  const size_t wrote = encode_batch(m.log + pos, base, recs, n);
  int64_t max_ts = recs[0].timestamp;
  for (size_t i = 1; i < n; ++i) max_ts = std::max(max_ts, recs[i].timestamp);
  m.idx[nb % P.index_capacity] = IndexEntry{base, pos, uint32_t(wrote), int32_t(n - 1), max_ts};
  P.log_end_pos.store(pos + wrote, std::memory_order_release);
  P.n_batches.store(nb + 1, std::memory_order_release);
  P.records_produced.fetch_add(n, std::memory_order_relaxed);
  P.high_watermark.store(base + int64_t(n), std::memory_order_release);
  return base;
}

uint8_t* Broker::log_tail(uint32_t pidx, uint64_t* avail) {
  PartitionEntry& P = part(pidx);
  Mapped& m = mapped(pidx);
  const uint64_t pos = P.log_end_pos.load(std::memory_order_acquire);
  *avail = P.log_capacity - pos;
  return m.log + pos;
}

void Broker::reset_empty(uint32_t pidx, int64_t offset) {
  PartitionEntry& P = part(pidx);
  RobustLock l(&P.lock);
  if (P.n_batches.load() != 0) throw KafkaError("reset_empty: partition already holds batches");
  P.log_start_offset.store(offset, std::memory_order_release);
  P.high_watermark.store(offset, std::memory_order_release);
}

void Broker::reset_partition(uint32_t pidx, int64_t offset) {
  PartitionEntry& P = part(pidx);
  RobustLock l(&P.lock);
  P.n_batches.store(0, std::memory_order_release);
  P.first_batch.store(0, std::memory_order_release);
  P.log_end_pos.store(0, std::memory_order_release);
  P.log_start_offset.store(offset, std::memory_order_release);
  P.high_watermark.store(offset, std::memory_order_release);
}

Broker::Ingested Broker::ingest(uint32_t pidx, uint64_t len, int64_t from_offset, bool keep_control,
                                uint64_t limit, const uint8_t* src) {
  PartitionEntry& P = part(pidx);
  Mapped& m = mapped(pidx);
  RobustLock l(&P.lock);
  const uint64_t pos0 = P.log_end_pos.load(std::memory_order_relaxed);
  if (!src && pos0 + len > P.log_capacity) throw KafkaError("ingest beyond the partition log capacity");
  const uint64_t room = limit ? std::min<uint64_t>(limit, P.log_capacity - pos0) : P.log_capacity - pos0;
  uint8_t* base = m.log + pos0;
  uint64_t nb = P.n_batches.load(std::memory_order_relaxed);
  int64_t hw = P.high_watermark.load(std::memory_order_relaxed);
  Ingested out;
  // Input starts in place (the record set was received into the log tail) and output compacts
  // it towards its start; an inflated batch grows, so from the first compressed batch on the
  // unread input moves to `spill` and the output may run past it.
  const uint8_t* in = src ? src : base;
  uint64_t in_len = len, r = 0, w = 0, consumed_base = 0;
  std::vector<uint8_t> spill, plain;
  const bool ring = P.ring_bytes.load(std::memory_order_relaxed) != 0;
  auto fits = [&](uint64_t total) {
    return w + total <= room && (ring ? nb - P.first_batch.load(std::memory_order_relaxed) < P.index_capacity
                                      : nb < P.index_capacity);
  };
  auto publish = [&](const uint8_t* src, uint64_t total, const BatchHeader& h) {
    if (base + w != src) std::memmove(base + w, src, total);
    m.idx[nb % P.index_capacity] = IndexEntry{h.base_offset, pos0 + w, uint32_t(total), h.last_offset_delta,
                                              h.max_timestamp};
    ++nb;
    w += total;
    hw = h.next_offset();
    ++out.kept;
  };
  std::exception_ptr failure;  // the batches before a bad one are still published
  try {
  while (in_len - r >= kBatchHeaderBytes) {
    int32_t blen;
    std::memcpy(&blen, in + r + kBatchLengthOffset, 4);
    blen = int32_t(__builtin_bswap32(uint32_t(blen)));
    if (blen < int32_t(kBatchHeaderBytes - 12)) throw CorruptRecord("replica: bad RecordBatch length");
    const uint64_t total = uint64_t(blen) + 12;
    if (in_len - r < total) break;  // partial trailing batch: the next fetch brings it whole
    if (in[r + 16] != 2)
      throw CorruptRecord("replica: message format v" + std::to_string(int(in[r + 16])) +
                          " (only RecordBatch v2 is supported; upgrade the topic's message.format.version)");
    const BatchHeader h = parse_batch_header(in + r, total, true);
    if (h.magic != 2)
      throw CorruptRecord("replica: message format v" + std::to_string(h.magic) +
                          " (only RecordBatch v2 is supported; upgrade the topic's message.format.version)");
    const bool control = (h.attributes >> 5) & 1;
    const bool keep = (!control || keep_control) && h.next_offset() > from_offset && h.next_offset() > hw;
    const int codec = h.attributes & 7;
    if (keep && (codec == kCodecNone || keep_control) && !fits(total)) {
      out.full = true;  // refetched once committed batches free space
      break;
    }
    out.consumed = consumed_base + r + total;
    out.next_offset = h.next_offset();
    if (control) ++out.control;
    if (keep) {
      if (codec == kCodecNone || keep_control) {
        publish(in + r, total, h);
      } else {
        // inflate once on arrival: the producer's CRC is checked over the compressed bytes, the
        // stored batch is plain RecordBatch v2 with its own CRC, so the device path verifies it
        if (!verify_batch_crc(in + r, h))
          throw CorruptRecord("Record batch at offset " + std::to_string(h.base_offset) + " failed CRC check");
        if (in == base) {
          spill.assign(in + r, in + in_len);
          consumed_base += r;
          in = spill.data();
          in_len = spill.size();
          r = 0;
        }
        // an inflated batch larger than the log (or its ring) could never be stored
        const uint64_t cap = std::min<uint64_t>(ring ? P.ring_bytes.load(std::memory_order_relaxed) : P.log_capacity,
                                                kMaxInflatedBytes);
        const auto t0 = std::chrono::steady_clock::now();
        // straight into the log, after what this walk kept: the input now lives in `spill`
        uint8_t* dst = base + w;
        const uint64_t space = std::min<uint64_t>(room - w, cap);
        size_t got = kNoRoom;
        if (space > kBatchHeaderBytes && fits(kBatchHeaderBytes))
          got = decompress_into(codec, in + r + kBatchHeaderBytes, total - kBatchHeaderBytes, dst + kBatchHeaderBytes,
                                size_t(space - kBatchHeaderBytes));
        if (got == kNoRoom) {
          // does not fit what is left now: left for a later fetch once consumers freed room.  With
          // plenty of room free, inflate it aside to tell a batch larger than the log could ever
          // hold (corrupt: thrown) from one that only needs more room.
          if (space >= std::min<uint64_t>(cap / 4, uint64_t(32) << 20)) {
            plain.assign(in + r, in + r + kBatchHeaderBytes);
            decompress(codec, in + r + kBatchHeaderBytes, total - kBatchHeaderBytes, plain, size_t(cap));
          }
          out.inflate_ns += uint64_t(std::chrono::duration_cast<std::chrono::nanoseconds>(
                                         std::chrono::steady_clock::now() - t0).count());
          out.consumed = consumed_base + r;
          out.next_offset = h.base_offset;  // not taken: fetched again
          out.full = true;
          break;
        }
        std::memcpy(dst, in + r, kBatchHeaderBytes);
        const uint64_t plain_total = kBatchHeaderBytes + got;
        const uint32_t be_len = __builtin_bswap32(uint32_t(plain_total - 12));
        std::memcpy(dst + kBatchLengthOffset, &be_len, 4);
        dst[kBatchAttrOffset + 1] = uint8_t(dst[kBatchAttrOffset + 1] & ~7);  // attributes: no codec
        const uint32_t be_crc = __builtin_bswap32(crc32c(dst + kBatchAttrOffset, plain_total - kBatchAttrOffset));
        std::memcpy(dst + kBatchCrcOffset, &be_crc, 4);
        out.inflate_ns += uint64_t(std::chrono::duration_cast<std::chrono::nanoseconds>(
                                       std::chrono::steady_clock::now() - t0).count());
        out.inflated_bytes += plain_total;
        out.inflated_from += total;
        publish(dst, plain_total, parse_batch_header(dst, plain_total));
        ++out.inflated;
        // visible at once: a Fetch response inflates to up to ~50 MB, and consumers that saw it only
        // when the whole set was stored waited for it in bursts (bridge lz4 / zstd blocks: worker
        // fill 48-112 us per batch against 22 us uncompressed, fetchers idle in long polls,
        // profiles/r06_s25).  The bytes below pos0 + w are final; the end of the walk stores the same.
        P.log_end_pos.store(pos0 + w, std::memory_order_release);
        P.n_batches.store(nb, std::memory_order_release);
        P.high_watermark.store(hw, std::memory_order_release);
      }
    }
    r += total;
  }
  } catch (...) {
    failure = std::current_exception();
  }
  out.kept_bytes = w;
  if (out.kept) {
    P.log_end_pos.store(pos0 + w, std::memory_order_release);
    P.n_batches.store(nb, std::memory_order_release);
    P.records_produced.fetch_add(uint64_t(out.kept), std::memory_order_relaxed);
    P.high_watermark.store(hw, std::memory_order_release);
  }
  if (failure) std::rethrow_exception(failure);
  return out;
}

uint64_t Broker::position_of(uint32_t pidx, int64_t offset) {
  const PartitionEntry& P = part(pidx);
  const IndexEntry* idx = mapped(pidx).idx;
  const uint64_t icap = P.index_capacity;
  const int64_t nb = int64_t(P.n_batches.load(std::memory_order_acquire));
  int64_t lo = int64_t(P.first_batch.load(std::memory_order_acquire)), hi = nb;  // first batch ending >= offset
  while (lo < hi) {
    const int64_t mid = lo + (hi - lo) / 2;
    const IndexEntry& e = idx[uint64_t(mid) % icap];
    if (e.base_offset + e.last_offset_delta < offset) lo = mid + 1; else hi = mid;
  }
  return lo < nb ? idx[uint64_t(lo) % icap].pos : P.log_end_pos.load(std::memory_order_acquire);
}

void Broker::make_ring(uint32_t pidx, uint64_t bytes) {
  PartitionEntry& P = part(pidx);
  RobustLock l(&P.lock);
  if (P.n_batches.load() != 0) throw KafkaError("make_ring: partition already holds batches");
  if (bytes == 0 || bytes > P.log_capacity) throw std::invalid_argument("make_ring: 0 < bytes <= log capacity");
  P.ring_bytes.store(bytes, std::memory_order_release);
  P.first_batch.store(0, std::memory_order_release);
}

// A ring's pages are faulted in up front: a replica's first pass through a fresh ring otherwise
// pays a page fault (tmpfs allocation + zeroing) per 4 KiB on the fetch path -- the bridge
// block ran 38-46 M rec/s after the other blocks against 50-53 M alone (profiles/r06_s6), and
// the bridge alone mirrored its first 300 k records per partition at 8.3 M (r06_s4).
void Broker::populate_ring(uint32_t pidx) {
  const PartitionEntry& P = part(pidx);
  const uint64_t bytes = P.ring_bytes.load(std::memory_order_acquire);
  if (!bytes) return;
  uint8_t* base = mapped(pidx).log;
  const uintptr_t page = 4096;
  const uintptr_t lo = reinterpret_cast<uintptr_t>(base) & ~(page - 1);
  const uintptr_t hi = (reinterpret_cast<uintptr_t>(base) + bytes + page - 1) & ~(page - 1);
#ifndef MADV_POPULATE_WRITE
#define MADV_POPULATE_WRITE 23
#endif
  if (madvise(reinterpret_cast<void*>(lo), hi - lo, MADV_POPULATE_WRITE) == 0) return;
  // older kernels: touch every page (the ring is empty: nothing is overwritten that matters)
  for (uint64_t o = 0; o < bytes; o += page) reinterpret_cast<volatile uint8_t*>(base)[o] = 0;
}

uint8_t* Broker::ring_reserve(uint32_t pidx, uint64_t want, int64_t keep_offset, uint64_t* avail) {
  PartitionEntry& P = part(pidx);
  Mapped& m = mapped(pidx);
  RobustLock l(&P.lock);
  const uint64_t C = P.ring_bytes.load(std::memory_order_relaxed);
  if (!C) throw KafkaError("ring_reserve on a linear log");
  const uint64_t icap = P.index_capacity;
  const uint64_t nb = P.n_batches.load(std::memory_order_relaxed);
  uint64_t first = P.first_batch.load(std::memory_order_relaxed);
  // retire batches every reader is done with (committed past): their bytes may be written over
  bool moved = false;
  while (first < nb) {
    const IndexEntry& e = m.idx[first % icap];
    if (e.base_offset + e.last_offset_delta >= keep_offset) break;
    ++first;
    moved = true;
  }
  if (moved) {
    const int64_t start = first < nb ? m.idx[first % icap].base_offset : P.high_watermark.load();
    if (start > P.log_start_offset.load()) P.log_start_offset.store(start, std::memory_order_release);
    P.first_batch.store(first, std::memory_order_release);
  }
  uint64_t w = P.log_end_pos.load(std::memory_order_relaxed);
  uint64_t free_bytes;
  if (first == nb) {  // nothing live: anywhere
    if (C - w < want) w = 0;
    free_bytes = C - w;
  } else {
    const uint64_t oldest = m.idx[first % icap].pos;
    if (oldest < w) {  // live bytes lie behind the writer: the tail, or the head before them
      free_bytes = C - w;
      if (free_bytes < want && oldest > free_bytes) {
        w = 0;
        free_bytes = oldest;
      }
    } else {  // the writer wrapped and sits behind the oldest live batch
      free_bytes = oldest - w;
    }
  }
  if (w != P.log_end_pos.load(std::memory_order_relaxed)) P.log_end_pos.store(w, std::memory_order_release);
  *avail = std::min(free_bytes, want);
  return m.log + w;
}

uint64_t Broker::release_log(uint32_t pidx, uint64_t from, uint64_t to) {
  const uint64_t page = 4096;
  from = (from + page - 1) / page * page;
  to = to / page * page;
  if (to <= from) return 0;
  const std::string path = part_path(dir_, pidx, "log");
  const int fd = open(path.c_str(), O_RDWR);
  if (fd < 0) throw_errno("open " + path);
  const int rc = fallocate(fd, FALLOC_FL_PUNCH_HOLE | FALLOC_FL_KEEP_SIZE, off_t(from), off_t(to - from));
  const int err = errno;
  close(fd);
  if (rc != 0) {
    errno = err;
    throw_errno("fallocate(PUNCH_HOLE) " + path);
  }
  return to - from;
}

void Broker::delete_records(uint32_t pidx, int64_t before_offset) {
  PartitionEntry& P = part(pidx);
  RobustLock l(&P.lock);
  const int64_t hw = P.high_watermark.load();
  int64_t v = std::min(before_offset, hw);
  if (v > P.log_start_offset.load()) P.log_start_offset.store(v, std::memory_order_release);
}

// Synthetic record generators.  Values are a deterministic
// function of (partition, offset) so any consumer can verify what it got.
//   kind 0 FIXED_F32   : size_a floats; v[0]=offset, v[1]=partition, v[j]=pattern
//   kind 1 JSON_F32    : JSON array text of L in [size_a, size_b] numbers "%.2f"
//   kind 2 BYTES       : L in [size_a, size_b] bytes of a (p, o) pattern
//   kind 3 TOKENS_I32  : L in [size_a, size_b] int32 token ids
//   kind 4 VARLEN_F32  : L in [size_a, size_b] raw float32
namespace {

inline float synth_f32(uint32_t p, int64_t o, int64_t j) {
  return float(int64_t((uint64_t(o) * 31u + uint64_t(j) * 7u + p * 13u) % 2001u) - 1000) * 0.0625f;
}

inline int64_t synth_len(uint64_t seed, uint32_t p, int64_t o, int64_t lo, int64_t hi) {
  if (hi <= lo) return lo;
  return lo + int64_t(mix64(seed ^ (uint64_t(p) << 40) ^ uint64_t(o)) % uint64_t(hi - lo + 1));
}

size_t gen_value(std::vector<uint8_t>& buf, int kind, uint32_t p, int64_t o, int64_t a, int64_t b,
                 uint64_t seed) {
  switch (kind) {
    case 0: {
      buf.resize(size_t(a) * 4);
      float* v = reinterpret_cast<float*>(buf.data());
      if (a > 0) v[0] = float(o);
      if (a > 1) v[1] = float(p);
      for (int64_t j = 2; j < a; ++j) v[j] = synth_f32(p, o, j);
      return buf.size();
    }
    case 1: {
      const int64_t L = synth_len(seed, p, o, a, b);
      buf.resize(size_t(L) * 12 + 2);
      char* s = reinterpret_cast<char*>(buf.data());
      size_t n = 0;
      s[n++] = '[';
      for (int64_t j = 0; j < L; ++j) {
        if (j) { s[n++] = ','; s[n++] = ' '; }
        // value in [-50.00, 50.99] with two decimals, cheap exact formatting
        int64_t cents = int64_t(mix64(seed + uint64_t(o) * 1315423911u + uint64_t(j) * 2654435761u + p) % 10100) - 5000;
        if (cents < 0) { s[n++] = '-'; cents = -cents; }
        int64_t ip = cents / 100, fp = cents % 100;
        if (ip >= 10) s[n++] = char('0' + ip / 10);
        s[n++] = char('0' + ip % 10);
        s[n++] = '.';
        s[n++] = char('0' + fp / 10);
        s[n++] = char('0' + fp % 10);
      }
      s[n++] = ']';
      buf.resize(n);
      return n;
    }
    case 2: {
      const int64_t L = synth_len(seed, p, o, a, b);
      buf.resize(size_t(L));
      uint64_t pat = mix64((uint64_t(p) << 48) ^ uint64_t(o) ^ seed);
      size_t i = 0;
      for (; i + 8 <= buf.size(); i += 8) std::memcpy(buf.data() + i, &pat, 8);
      for (; i < buf.size(); ++i) buf[i] = uint8_t(pat >> (8 * (i & 7)));
      return buf.size();
    }
    case 3: {
      const int64_t L = synth_len(seed, p, o, a, b);
      buf.resize(size_t(L) * 4);
      int32_t* t = reinterpret_cast<int32_t*>(buf.data());
      for (int64_t j = 0; j < L; ++j) t[j] = int32_t((uint64_t(o) * 977u + uint64_t(j) * 131u + p * 7u) % 50000u);
      return buf.size();
    }
    case 4: {
      const int64_t L = synth_len(seed, p, o, a, b);
      buf.resize(size_t(L) * 4);
      float* v = reinterpret_cast<float*>(buf.data());
      for (int64_t j = 0; j < L; ++j) v[j] = synth_f32(p, o, j);
      return buf.size();
    }
    default:
      throw std::invalid_argument("unknown synthetic record kind");
  }
}

}  // namespace

void Broker::fill_synthetic(const std::vector<uint32_t>& pidxs, int64_t n_records, int kind, int64_t size_a,
                            int64_t size_b, uint32_t records_per_batch, uint64_t seed, int n_threads, bool keyed) {
  if (records_per_batch == 0) records_per_batch = 1;
  for (uint32_t pidx : pidxs) { part(pidx); mapped(pidx); }
  std::atomic<size_t> next{0};
  std::exception_ptr err;
  std::mutex err_mu;
  auto work = [&]() {
    std::vector<std::vector<uint8_t>> vals(records_per_batch);
    std::vector<std::array<uint8_t, 8>> keys(records_per_batch);
    std::vector<RecordIn> recs(records_per_batch);
    try {
      for (;;) {
        const size_t k = next.fetch_add(1);
        if (k >= pidxs.size()) break;
        const uint32_t pidx = pidxs[k];
        const uint32_t p = parts_[pidx].partition;
        int64_t done = 0;
        while (done < n_records) {
          const int64_t base = parts_[pidx].high_watermark.load();
          const size_t n = size_t(std::min<int64_t>(records_per_batch, n_records - done));
          for (size_t i = 0; i < n; ++i) {
            const int64_t o = base + int64_t(i);
            size_t len = gen_value(vals[i], kind, p, o, size_a, size_b, seed);
            recs[i] = RecordIn{1700000000000LL + o, nullptr, -1, vals[i].data(), int32_t(len), nullptr, 0};
            if (keyed) {  // a class label: offset % 1000 as 8 bytes big-endian (Kafka's LongSerializer)
              const uint64_t key = __builtin_bswap64(uint64_t(o % 1000));
              std::memcpy(keys[i].data(), &key, 8);
              recs[i].key = keys[i].data();
              recs[i].key_len = 8;
            }
          }
          append(pidx, recs.data(), n);
          done += int64_t(n);
        }
      }
    } catch (...) {
      std::lock_guard<std::mutex> g(err_mu);
      if (!err) err = std::current_exception();
    }
  };
  n_threads = std::max(1, std::min<int>(n_threads, int(pidxs.size())));
  std::vector<std::thread> ts;
  for (int i = 1; i < n_threads; ++i) ts.emplace_back(work);
  work();
  for (auto& t : ts) t.join();
  if (err) std::rethrow_exception(err);
}

}  // namespace tk
