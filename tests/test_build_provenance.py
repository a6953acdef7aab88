"""Build provenance: each extension carries the sha of the sources it was built from
(`_build.sources_sha`, compiled in), the loader rebuilds when it differs from the tree's, and
`ops.build_info()` / bench.py's `native_build` report it."""
import shutil

from torchkafka_amd import _build
from torchkafka_amd.ops import build_info, core


def test_loaded_core_matches_the_tree():
    core()
    info = build_info()["_tkcore"]
    assert info["built_from"] == info["tree"] == _build.sources_sha("core")
    assert info["matches_tree"] and info["file"].startswith("torchkafka_amd/")
    assert _build.embedded_sha(_build.core_target()) == info["built_from"]


def test_sha_follows_the_sources(tmp_path, monkeypatch):
    # a copy of the source tree: editing one byte of one header changes the sha
    src = tmp_path / "csrc"
    shutil.copytree(_build.CSRC, src)
    monkeypatch.setattr(_build, "CSRC", src)
    before_core, before_hip = _build.sources_sha("core"), _build.sources_sha("hip")
    h = src / "core" / "span.h"
    h.write_bytes(h.read_bytes() + b"\n")
    assert _build.sources_sha("core") != before_core
    assert _build.sources_sha("hip") != before_hip  # the device extension embeds the host core
    p = src / "hip" / "driver.h"
    before = _build.sources_sha("hip")
    p.write_bytes(p.read_bytes() + b"\n")
    assert _build.sources_sha("hip") != before
    assert _build.sources_sha("core") == _build.sources_sha("core")  # deterministic


def test_embedded_sha_of_a_file_without_marker(tmp_path):
    f = tmp_path / "x.so"
    f.write_bytes(b"\0" * 100 + b"TKSRCSHA:unversioned")
    assert _build.embedded_sha(f) is None
    assert _build.embedded_sha(tmp_path / "missing.so") is None
