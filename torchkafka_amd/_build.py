"""In-tree builder for the two native extensions.

* ``_tkcore``  host C++17 (g++): RecordBatch codec, shm broker, fetcher,
  packers, slot ring.  No HIP: it is imported inside forked loader workers.
* ``_tkhip``   HIP for gfx950 (hipcc --offload-arch=gfx950): collate kernels,
  the H2D engine, the step driver and the RCCL lockstep.  Built with hipcc -- no
  hipify step, no CUDA shim -- against the installed PyTorch (torch's pybind11;
  libtorch for the batch allocation in torch_step.cpp).

Both land next to this file so the built ``.so`` travel with the repository
snapshot to the GPU box.  Run ``python -m torchkafka_amd._build`` (or
``python setup.py build_ext``); rebuilds are incremental on source mtimes.
"""
from __future__ import annotations

import concurrent.futures as cf
import hashlib
import os
import re
import shutil
import subprocess
import sys
import sysconfig
from pathlib import Path

PKG = Path(__file__).resolve().parent
CSRC = PKG / "csrc"
BUILD = PKG.parent / "build" / "native"
EXT_SUFFIX = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
ARCH = os.environ.get("TORCHKAFKA_ROCM_ARCH", os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")).split(";")[0]
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")


def _py_includes() -> list[str]:
    import pybind11

    return [f"-I{pybind11.get_include()}", f"-I{sysconfig.get_paths()['include']}"]


def _torch_paths() -> tuple[Path, Path]:
    """(include, lib) of the installed PyTorch: the device module links libtorch for
    step_fixed_tensor and must use torch's bundled pybind11 for every binding."""
    import importlib.util

    spec = importlib.util.find_spec("torch")
    if spec is None or spec.origin is None:
        raise RuntimeError("the gfx950 extension needs PyTorch (ROCm build) installed")
    root = Path(spec.origin).parent
    return root / "include", root / "lib"


def core_target() -> Path:
    return PKG / f"_tkcore{EXT_SUFFIX}"


def hip_target() -> Path:
    return PKG / f"_tkhip{EXT_SUFFIX}"


def sources(builder: str) -> list[Path]:
    """Every file an extension is built from (its sources and the headers they may include)."""
    core_dir, hip_dir = CSRC / "core", CSRC / "hip"
    core = sorted(core_dir.glob("*.cpp")) + sorted(core_dir.glob("*.h"))
    if builder == "core":
        return core
    return sorted(hip_dir.glob("*.hip")) + sorted(hip_dir.glob("*.cpp")) + sorted(hip_dir.glob("*.h")) + core


def sources_sha(builder: str) -> str:
    """sha256 over the relative paths and bytes of sources(builder) (plus the target arch for hip):
    compiled into the extension, so a binary names the exact tree it was built from."""
    h = hashlib.sha256(f"{builder}:{ARCH if builder == 'hip' else 'host'}\n".encode())
    for p in sources(builder):
        h.update(str(p.relative_to(CSRC)).encode() + b"\0")
        h.update(p.read_bytes())
    return h.hexdigest()


_SHA_RE = re.compile(rb"TKSRCSHA:([0-9a-f]{64})")


def embedded_sha(path: Path) -> str | None:
    """The sources_sha a built extension carries (read from the file, nothing is loaded)."""
    try:
        m = _SHA_RE.search(path.read_bytes())
    except OSError:
        return None
    return m.group(1).decode() if m else None


def up_to_date(builder: str) -> bool:
    target = core_target() if builder == "core" else hip_target()
    return target.exists() and embedded_sha(target) == sources_sha(builder)


def _run(cmd: list[str]) -> None:
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"build failed ({r.returncode}): {' '.join(cmd)}\n{r.stdout}")


def _compile_all(jobs: list[list[str]]) -> None:
    workers = max(1, min(len(jobs), int(os.environ.get("MAX_JOBS", os.cpu_count() or 4)), 16))
    with cf.ThreadPoolExecutor(workers) as ex:
        for f in [ex.submit(_run, j) for j in jobs]:
            f.result()


def build_core(force: bool = False, verbose: bool = False) -> Path:
    src_dir = CSRC / "core"
    srcs = sorted(src_dir.glob("*.cpp"))
    out = core_target()
    if not force and up_to_date("core"):
        return out
    obj_dir = BUILD / "core"
    obj_dir.mkdir(parents=True, exist_ok=True)
    cxx = os.environ.get("CXX", "g++")
    flags = ["-O3", "-std=c++17", "-fPIC", "-fvisibility=hidden", "-Wall", "-Wno-unused-function",
             "-DNDEBUG", *_py_includes(), f"-I{src_dir}"]
    flags += os.environ.get("TORCHKAFKA_CXXFLAGS", "").split()
    flags.append(f'-DTK_SOURCES_SHA="{sources_sha("core")}"')
    objs, jobs = [], []
    for s in srcs:
        o = obj_dir / (s.stem + ".o")
        objs.append(o)
        jobs.append([cxx, *flags, "-c", str(s), "-o", str(o)])
    _compile_all(jobs)
    tmp = out.with_suffix(".tmp.so")
    _run([cxx, "-shared", "-o", str(tmp), *map(str, objs), "-lpthread", "-lrt", "-lz", "-lssl", "-lcrypto", "-ldl",
          *os.environ.get("TORCHKAFKA_LDFLAGS", "").split()])
    os.replace(tmp, out)
    if verbose:
        print(f"[torchkafka_amd] built {out.name}")
    return out


def hipcc() -> str:
    p = shutil.which("hipcc") or os.path.join(ROCM, "bin", "hipcc")
    if not os.path.exists(p):
        raise RuntimeError("hipcc not found: the gfx950 extension needs ROCm")
    return p


def build_hip(force: bool = False, verbose: bool = False) -> Path:
    src_dir = CSRC / "hip"
    core_dir = CSRC / "core"
    # the main-process step driver embeds the host core (ring, broker) to commit natively
    core_srcs = [p for p in sorted(core_dir.glob("*.cpp")) if not p.name.startswith("bindings")]
    srcs = sorted(src_dir.glob("*.hip")) + sorted(src_dir.glob("*.cpp")) + core_srcs
    out = hip_target()
    if not force and up_to_date("hip"):
        return out
    obj_dir = BUILD / f"hip-{ARCH}"
    obj_dir.mkdir(parents=True, exist_ok=True)
    cc = hipcc()
    t_inc, t_lib = _torch_paths()
    # torch's include dir first: its bundled pybind11 is the one every binding in this module uses
    flags = ["-O3", "-std=c++17", "-fPIC", "-fvisibility=hidden", f"--offload-arch={ARCH}", "-DNDEBUG",
             "-Wno-unused-result", f"-I{t_inc}", f"-I{sysconfig.get_paths()['include']}", f"-I{src_dir}",
             f"-I{core_dir}", f'-DTK_SOURCES_SHA="{sources_sha("hip")}"']
    torch_flags = [f"-I{t_inc / 'torch' / 'csrc' / 'api' / 'include'}", "-DUSE_ROCM=1", "-D__HIP_PLATFORM_AMD__=1",
                   "-DTORCH_API_INCLUDE_EXTENSION_H", "-D_GLIBCXX_USE_CXX11_ABI=1", "-Wno-deprecated-declarations"]
    objs, jobs = [], []
    for s in srcs:
        o = obj_dir / ((("core_" if s.parent == core_dir else "") + s.stem) + ".o")
        objs.append(o)
        lang = ["-x", "hip"] if s.suffix == ".hip" else []
        extra = torch_flags if s.name == "torch_step.cpp" else []
        jobs.append([cc, *flags, *extra, *lang, "-c", str(s), "-o", str(o)])
    _compile_all(jobs)
    tmp = out.with_suffix(".tmp.so")
    _run([cc, "-shared", f"--offload-arch={ARCH}", "-o", str(tmp), *map(str, objs), f"-L{ROCM}/lib", "-lamdhip64",
          f"-L{t_lib}", "-lc10", "-lc10_hip", "-ltorch_cpu", "-ltorch_hip", "-ltorch", "-ltorch_python",
          f"-Wl,-rpath,{t_lib}", "-lpthread", "-lrt", "-lz", "-lssl", "-lcrypto", "-ldl"])
    os.replace(tmp, out)
    if verbose:
        print(f"[torchkafka_amd] built {out.name} for {ARCH}")
    return out


def build_all(force: bool = False, verbose: bool = True) -> list[Path]:
    return [build_core(force, verbose), build_hip(force, verbose)]


if __name__ == "__main__":
    force = "--force" in sys.argv
    only = [a for a in sys.argv[1:] if not a.startswith("--")]
    if not only or "core" in only:
        build_core(force, True)
    if not only or "hip" in only:
        build_hip(force, True)
