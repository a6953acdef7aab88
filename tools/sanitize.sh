#!/bin/bash
# Host sanitizer runs of the native core: ThreadSanitizer over the ring protocol,
# the futex hand-offs and the broker/fetcher/packer pipeline; AddressSanitizer + UBSan over the
# same stress test and a codec/CRC/JSON fuzz test.  Host code only -- GPU sanitizers are not
# available on this pool.  Usage: tools/sanitize.sh [outdir]
set -euo pipefail
cd "$(dirname "$0")/.."
OUT=${1:-build/sanitize}
mkdir -p "$OUT"
CORE=torchkafka_amd/csrc/core
SRCS="$CORE/ring.cpp $CORE/broker.cpp $CORE/broker_groups.cpp $CORE/consumer.cpp $CORE/json_text.cpp $CORE/record_batch.cpp $CORE/crc32c.cpp $CORE/codecs.cpp"
CXX=${CXX:-g++}
COMMON="-std=c++17 -O1 -g -fno-omit-frame-pointer -I$CORE -pthread"
$CXX $COMMON -fsanitize=thread tests/native/ring_stress.cpp $SRCS -o "$OUT/ring_stress_tsan" -lrt -lz
$CXX $COMMON -fsanitize=address,undefined -fno-sanitize-recover=undefined tests/native/ring_stress.cpp $SRCS \
    -o "$OUT/ring_stress_asan" -lrt -lz
$CXX $COMMON -fsanitize=address,undefined -fno-sanitize-recover=undefined tests/native/codec_fuzz.cpp $SRCS \
    -o "$OUT/codec_fuzz_asan" -lrt -lz
# the HIP command queue (csrc/hip/hip_queue.*) with its two device calls stubbed (no GPU)
HQ="-D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -Itorchkafka_amd/csrc/hip tests/native/hip_queue_test.cpp torchkafka_amd/csrc/hip/hip_queue.cpp"
$CXX $COMMON -fsanitize=thread $HQ -o "$OUT/hip_queue_tsan"
$CXX $COMMON -fsanitize=address,undefined -fno-sanitize-recover=undefined $HQ -o "$OUT/hip_queue_asan"
$CXX $COMMON -fsanitize=address,undefined -fno-sanitize-recover=undefined -Itorchkafka_amd/csrc/core \
  tests/native/span_window_test.cpp -o "$OUT/span_window_asan"
# the RCCL lockstep transport's failure detection (csrc/hip/rccl_lockstep.cpp) with HIP stubbed and a
# stand-in librccl (tests/native/rccl_stub.cpp) it dlopen()s
RL="-D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -Itorchkafka_amd/csrc/hip -I$CORE"
$CXX $COMMON -fsanitize=address,undefined -fno-sanitize-recover=undefined $RL -shared -fPIC \
  tests/native/rccl_stub.cpp -o "$OUT/librccl_stub.so"
$CXX $COMMON -fsanitize=address,undefined -fno-sanitize-recover=undefined $RL tests/native/rccl_lockstep_test.cpp \
  torchkafka_amd/csrc/hip/rccl_lockstep.cpp -o "$OUT/rccl_lockstep_asan" -ldl
export TSAN_OPTIONS="halt_on_error=1 second_deadlock_stack=1"
export ASAN_OPTIONS="halt_on_error=1 detect_leaks=1"
export UBSAN_OPTIONS="halt_on_error=1 print_stacktrace=1"
echo "== tsan ring_stress"; "$OUT/ring_stress_tsan" 4 3 ${TK_SAN_BATCHES:-2000}
echo "== asan ring_stress"; "$OUT/ring_stress_asan" 4 3 ${TK_SAN_BATCHES:-2000}
echo "== asan codec_fuzz"; "$OUT/codec_fuzz_asan" ${TK_SAN_FUZZ:-3000}
echo "== asan codec_fuzz, built-in LZ4 decoder"; TORCHKAFKA_LZ4_LIB=0 "$OUT/codec_fuzz_asan" ${TK_SAN_FUZZ:-3000}
echo "== tsan hip_queue"; "$OUT/hip_queue_tsan" ${TK_SAN_QUEUE:-50000}
echo "== asan hip_queue"; "$OUT/hip_queue_asan" ${TK_SAN_QUEUE:-50000}
echo "== asan span_window"; "$OUT/span_window_asan"
echo "== asan rccl_lockstep"; "$OUT/rccl_lockstep_asan" "$OUT/librccl_stub.so"
echo "sanitizers: all clean"
