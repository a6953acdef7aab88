// Kafka record-set decompression (RecordBatch attributes bits 0-2) for the replica bridge.
//
// kafka-python decompresses a compressed RecordBatch in its fetcher (gzip, snappy, lz4, zstd via
// optional Python packages) before `_process` sees a record (kafka_dataset.py:156-162).  The
// device decoders read raw records straight out of the logs, so the replicator
// (replicator.cpp -> Broker::ingest) inflates a compressed batch once, on arrival, into an
// uncompressed RecordBatch v2 with a fresh CRC32C (after checking the producer's CRC over the
// compressed bytes).  gzip goes through zlib; snappy (raw or xerial-framed, as the Java client
// writes it) and LZ4 (frame format) are decoded here; zstd goes through the system libzstd.so.1
// (dlopen'd; UnsupportedCodecError when it cannot be loaded).
#pragma once
#include <cstddef>
#include <cstdint>
#include <vector>

namespace tk {

enum Codec : int { kCodecNone = 0, kCodecGzip = 1, kCodecSnappy = 2, kCodecLz4 = 3, kCodecZstd = 4 };
const char* codec_name(int codec);

// A RecordBatch's length field is an int32: no inflated batch can be larger.
constexpr size_t kMaxInflatedBytes = size_t(0x7fffffff);

// Appends the decompressed bytes of `src` to `out`, which may grow to at most `max_out` bytes in
// total (the caller passes what a batch could ever occupy, e.g. its log's capacity): a small
// compressed record set from the network cannot claim unbounded memory.  Throws CorruptRecord on
// malformed or oversized input (allocation failures included), KafkaError("UnsupportedCodecError
// ...") for codecs this build cannot decode.
void decompress(int codec, const uint8_t* src, size_t n, std::vector<uint8_t>& out,
                size_t max_out = kMaxInflatedBytes);
bool zstd_available();

// The raw block formats (tests encode with their own minimal compressors).
void snappy_raw_decompress(const uint8_t* src, size_t n, std::vector<uint8_t>& out,
                           size_t max_out = kMaxInflatedBytes);
void lz4_block_decompress(const uint8_t* src, size_t n, std::vector<uint8_t>& out,
                          size_t max_out = kMaxInflatedBytes);

}  // namespace tk
