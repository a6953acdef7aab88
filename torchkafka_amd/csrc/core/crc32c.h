// CRC32C (Castagnoli) as used by Kafka RecordBatch v2 (the `crc` field covers
// attributes .. end of batch).  Hardware path: SSE4.2 `crc32` with three
// interleaved streams combined by GF(2) shifting; portable slicing-by-8 table
// fallback when the CPU lacks SSE4.2.
#pragma once
#include <cstddef>
#include <cstdint>

namespace tk {

// crc32c(data) with the standard init/final xor (0xFFFFFFFF).
uint32_t crc32c(const void* data, size_t n);
// Continue a running crc (value as returned by crc32c over a prefix).
uint32_t crc32c_extend(uint32_t crc, const void* data, size_t n);
// True if the hardware (SSE4.2) path is in use.
bool crc32c_hw();
// True when the AVX-512 VPCLMULQDQ folding path is used for buffers >= 512 bytes.
bool crc32c_fold();
// One implementation explicitly (tests): 0 table, 1 crc32 instruction (3 streams), 2 folding.
uint32_t crc32c_method(int method, const void* data, size_t n);

// Raw (zero-initialised, no final xor) CRC state `raw` advanced over n_bytes zero bytes:
// raw CRC of (A || B) = crc32c_shift_raw(raw(A), |B|) ^ raw(B).
uint32_t crc32c_shift_raw(uint32_t raw, uint64_t n_bytes);
// Tables of the device CRC stage (span.h: kSpanTabWords uint32).
void crc32c_span_tables(uint32_t* out);
// Host emulation of the device CRC stage over buf[c0, c1): raw CRC, with the RecordBatch's
// initial-value xor applied to its first 4 bytes when `first` (tests compare it with crc32c).
uint32_t crc32c_span_emulate(const uint8_t* buf, uint32_t c0, uint32_t c1, bool first, int parts = 1);

}  // namespace tk
