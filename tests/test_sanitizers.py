"""Host sanitizers over the native core: ThreadSanitizer on the slot-ring protocol
and the broker -> fetcher -> packer -> commit pipeline (threads standing in for worker processes),
the HIP command queue (its device calls stubbed), the span kernels' window geometry (span.h SpanWindows),
the RCCL lockstep transport's timeout / abort / asynchronous-error paths (HIP and RCCL stubbed),
AddressSanitizer + UBSan on the same stress test and on a RecordBatch/CRC32C/JSON fuzz test.
The sources are tests/native/*.cpp; tools/sanitize.sh builds and runs them."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which(os.environ.get("CXX", "g++")) is None, reason="no host C++ compiler")
@pytest.mark.timeout(600)
def test_native_core_under_tsan_asan_ubsan(tmp_path):
    env = dict(os.environ, TK_SAN_BATCHES="600", TK_SAN_FUZZ="1500")
    r = subprocess.run([os.path.join(ROOT, "tools", "sanitize.sh"), str(tmp_path)], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=590)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert "sanitizers: all clean" in out
    assert "WARNING: ThreadSanitizer" not in out and "ERROR: AddressSanitizer" not in out
    assert "runtime error" not in out, out[-4000:]
