// Kafka record-set compression (RecordBatch attributes bits 0-2) for the replica bridge.
//
// kafka-python decompresses a compressed RecordBatch in its fetcher (gzip, snappy, lz4, zstd via
// optional Python packages) before `_process` sees a record (kafka_dataset.py:156-162).  The
// device decoders read raw records straight out of the logs, so the replicator
// (replicator.cpp -> Broker::ingest) inflates a compressed batch once, on arrival, on the fetch
// thread that received it, straight into the partition log (decompress_into): an uncompressed
// RecordBatch v2 with a fresh CRC32C (after checking the producer's CRC over the compressed bytes).
//
// gzip goes through zlib; snappy (raw or xerial-framed, as the Java client writes it) is decoded
// here; LZ4 (frame format) is parsed here and its blocks decoded by the system liblz4.so.1 when it
// loads (dlopen'd; the decoder here otherwise); zstd goes through the system libzstd.so.1
// (dlopen'd; UnsupportedCodecError when it cannot be loaded).  compress() writes gzip, lz4 and zstd
// record sets (the benchmarks' compressed topics, tests).
#pragma once
#include <cstddef>
#include <cstdint>
#include <vector>

namespace tk {

enum Codec : int { kCodecNone = 0, kCodecGzip = 1, kCodecSnappy = 2, kCodecLz4 = 3, kCodecZstd = 4 };
const char* codec_name(int codec);

// A RecordBatch's length field is an int32: no inflated batch can be larger.
constexpr size_t kMaxInflatedBytes = size_t(0x7fffffff);
// decompress_into(): the inflated bytes do not fit the room given.
constexpr size_t kNoRoom = ~size_t(0);

// Decompresses `src` into dst[0, cap).  Returns the bytes written, or kNoRoom when they would not
// fit in `cap` (dst[0, cap) may then hold a partial result).  Throws CorruptRecord on malformed
// input, KafkaError("UnsupportedCodecError ...") for codecs this build cannot decode.
size_t decompress_into(int codec, const uint8_t* src, size_t n, uint8_t* dst, size_t cap);

// Appends the decompressed bytes of `src` to `out`, which may grow to at most `max_out` bytes in
// total (the caller passes what a batch could ever occupy, e.g. its log's capacity): a small
// compressed record set from the network cannot claim unbounded memory.  Throws CorruptRecord on
// malformed or oversized input (allocation failures included), KafkaError("UnsupportedCodecError
// ...") for codecs this build cannot decode.
void decompress(int codec, const uint8_t* src, size_t n, std::vector<uint8_t>& out,
                size_t max_out = kMaxInflatedBytes);

// Appends `src` compressed with `codec` (gzip, lz4 frame with independent 64 KiB blocks as the
// Java client writes it, zstd) to `out`.  `level`: the codec's level (0: its default).  Throws
// KafkaError("UnsupportedCodecError ...") for snappy and for a library that does not load.
void compress(int codec, const uint8_t* src, size_t n, std::vector<uint8_t>& out, int level = 0);

bool zstd_available();
bool lz4_library_available();  // liblz4.so.1 decodes the blocks (else the decoder here does)

// The raw block formats (tests encode with their own minimal compressors).
void snappy_raw_decompress(const uint8_t* src, size_t n, std::vector<uint8_t>& out,
                           size_t max_out = kMaxInflatedBytes);
void lz4_block_decompress(const uint8_t* src, size_t n, std::vector<uint8_t>& out,
                          size_t max_out = kMaxInflatedBytes);

}  // namespace tk
