"""Loading of the two in-tree native extensions.

``core()`` returns ``_tkcore`` (host C++: broker, codec, fetcher, ring) and
``hip()`` returns ``_tkhip`` (gfx950 kernels + H2D engine).  A missing
extension is built in-tree on first use (under a file lock, so concurrent
test processes do not race); a build failure raises -- there is no silent
Python fallback for the device path.
"""
from __future__ import annotations

import fcntl
import importlib
import os
import threading
from pathlib import Path

_PKG = Path(__file__).resolve().parent.parent
_lock = threading.Lock()
_mods: dict[str, object] = {}


def _load(name: str, builder: str):
    mod = _mods.get(name)
    if mod is not None:
        return mod
    with _lock:
        mod = _mods.get(name)
        if mod is not None:
            return mod
        from .. import _build

        target = getattr(_build, f"{builder}_target")()
        stale = not target.exists()
        if not stale and os.environ.get("TORCHKAFKA_NO_REBUILD") != "1":
            # rebuild when the binary was built from other sources than the tree's (its embedded sha)
            stale = not _build.up_to_date(builder)
        if stale:
            lock_path = _PKG.parent / "build" / f".{builder}.lock"
            lock_path.parent.mkdir(parents=True, exist_ok=True)
            with open(lock_path, "w") as lf:
                fcntl.flock(lf, fcntl.LOCK_EX)
                try:
                    getattr(_build, f"build_{builder}")(verbose=False)
                finally:
                    fcntl.flock(lf, fcntl.LOCK_UN)
        mod = importlib.import_module(f"torchkafka_amd.{name}")
        _mods[name] = mod
        return mod


def core():
    """Host native core (``_tkcore``)."""
    return _load("_tkcore", "core")


def hip():
    """gfx950 device extension (``_tkhip``).  Raises if it cannot be built/loaded."""
    try:
        return _load("_tkhip", "hip")
    except Exception as e:  # pragma: no cover - exercised on broken toolchains
        raise RuntimeError(
            "torchkafka_amd: the gfx950 HIP extension (_tkhip) is unavailable; "
            "the device path has no Python fallback. Build it with "
            "`python -m torchkafka_amd._build hip`."
        ) from e


def loaded_extensions() -> list[str]:
    return sorted(_mods)


def build_info() -> dict:
    """Provenance of the loaded extensions: the source sha each binary was built from (compiled
    in), the sha of the sources in this tree, whether they match, and the file it was loaded from."""
    from .. import _build

    out = {}
    for name, builder in (("_tkcore", "core"), ("_tkhip", "hip")):
        mod = _mods.get(name)
        if mod is None:
            continue
        tree = _build.sources_sha(builder)
        built = getattr(mod, "SOURCES_SHA", None)
        out[name] = {"built_from": built, "tree": tree, "matches_tree": built == tree,
                     "file": os.path.relpath(mod.__file__, _PKG.parent)}
    return out
