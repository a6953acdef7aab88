"""GPU -> NUMA node placement without initialising HIP.

An MI355X node is two CPU sockets; each GPU hangs off one socket's PCIe root
complex (on the measured box: GPU 0000:f4:00.0 -> NUMA node 1, CPUs
64-127,192-255; gpurun_out probe in profiles/).  Every byte the loader moves
crosses host memory twice before it reaches the GPU: the worker reads the
broker log and writes a pinned ring slot, then the GPU reads that slot over
PCIe.  If the worker runs on the other socket, both the slot write and the
GPU's read cross the inter-socket link, and with 8 ranks per node every rank
competes for it.  Binding each rank (and the workers it forks, which inherit
the mask) to its GPU's socket keeps the ring, the log pages it first-touches
and the PCIe reads socket-local.

This runs before the loader forks and before HIP is initialised (HIP must not
be initialised in forked workers), so the device is resolved from sysfs the
way ROCr enumerates it:
  * KFD topology nodes with SIMDs, in node order (the container only shows
    the GPUs it was granted; render nodes that cannot be opened are skipped,
    as ROCr skips them);
  * then ``ROCR_VISIBLE_DEVICES`` (indices or ``GPU-<uuid>``), then
    ``HIP_VISIBLE_DEVICES`` / ``CUDA_VISIBLE_DEVICES`` (indices).
:func:`check_device` cross-checks the prediction against HIP's PCI bus id once
HIP is up.
"""
from __future__ import annotations

import glob
import logging
import os

log = logging.getLogger(__name__)

#: sysfs / devfs roots (tests point these at a fake tree)
SYSFS = "/sys"
DEVDRI = "/dev/dri"


def _kfd_gpus() -> list[dict]:
    nodes = []
    for d in glob.glob(os.path.join(SYSFS, "class/kfd/kfd/topology/nodes", "*")):
        try:
            nid = int(os.path.basename(d))
            props = {}
            with open(os.path.join(d, "properties")) as f:
                for line in f:
                    k, _, v = line.strip().partition(" ")
                    props[k] = v
        except (OSError, ValueError):
            continue
        if int(props.get("simd_count", "0") or 0) <= 0:
            continue
        props["_node"] = nid
        rm = props.get("drm_render_minor")
        if rm and rm != "0" and not os.access(os.path.join(DEVDRI, f"renderD{rm}"), os.R_OK | os.W_OK):
            continue
        nodes.append(props)
    nodes.sort(key=lambda p: p["_node"])
    return nodes


def _apply_visible(devs: list, spec: str | None, allow_uuid: bool) -> list:
    if spec is None:
        return devs
    spec = spec.strip()
    if spec == "":
        return []
    out = []
    for tok in spec.split(","):
        tok = tok.strip()
        if allow_uuid and tok.upper().startswith("GPU-"):
            want = tok[4:].lower()
            hit = [d for d in devs if format(int(d.get("unique_id", "0") or 0), "x") == want]
            out.extend(hit[:1])
            continue
        try:
            i = int(tok)
        except ValueError:
            return out  # the runtimes stop at the first invalid entry
        if i < 0 or i >= len(devs):
            return out
        out.append(devs[i])
    return out


def visible_gpus() -> list[dict]:
    """KFD properties of the GPUs HIP will number 0..n-1 in this process (best effort)."""
    devs = _kfd_gpus()
    devs = _apply_visible(devs, os.environ.get("ROCR_VISIBLE_DEVICES"), True)
    hip = os.environ.get("HIP_VISIBLE_DEVICES", os.environ.get("CUDA_VISIBLE_DEVICES"))
    return _apply_visible(devs, hip, False)


def count_gpus_without_hip() -> dict:
    """How many GPUs this process could use, found without any HIP call (a launcher must not
    initialise HIP before it starts its rank processes): the KFD topology filtered by the
    visibility variables (:func:`visible_gpus`), cross-checked against amdsmi when torch can reach
    it (``torch.cuda._device_count_amdsmi`` -- it never falls back to ``hipGetDeviceCount``).
    ``{"count": n, "sysfs": n_sysfs, "amdsmi": n_smi or None}``; raises RuntimeError when neither
    source answers (the caller refuses to launch rather than guess)."""
    n_sys = len(visible_gpus())
    n_smi = None
    try:
        import torch

        fn = getattr(torch.cuda, "_device_count_amdsmi", None)
        if fn is not None and torch.version.hip:
            v = int(fn())
            n_smi = v if v >= 0 else None
    except Exception:  # noqa: BLE001 - amdsmi absent or broken: sysfs decides
        n_smi = None
    if n_sys > 0:
        count = n_sys if n_smi is None else min(n_sys, n_smi)
    elif n_smi is not None:
        count = n_smi
    else:
        raise RuntimeError("cannot count GPUs without initialising HIP: no KFD GPU nodes in sysfs and amdsmi "
                           "is unavailable")
    return {"count": count, "sysfs": n_sys, "amdsmi": n_smi}


def hip_touched() -> dict:
    """Whether this process has initialised HIP (torch's lazy init) or holds an open /dev/kfd."""
    kfd = 0
    try:
        for fd in os.listdir("/proc/self/fd"):
            try:
                if os.readlink(f"/proc/self/fd/{fd}") == "/dev/kfd":
                    kfd += 1
            except OSError:
                continue
    except OSError:
        pass
    init = False
    try:
        import torch

        init = bool(torch.cuda.is_initialized())
    except Exception:  # noqa: BLE001
        pass
    return {"torch_cuda_initialized": init, "kfd_fds": kfd}


def _bdf(props: dict) -> str | None:
    try:
        loc, dom = int(props["location_id"]), int(props.get("domain", "0") or 0)
    except (KeyError, ValueError):
        return None
    return f"{dom:04x}:{loc >> 8:02x}:{(loc >> 3) & 0x1f:02x}.{loc & 7}"


def gpu_pci_bus(index: int) -> int | None:
    """PCI bus number of HIP device ``index`` as predicted from sysfs."""
    devs = visible_gpus()
    if not 0 <= index < len(devs):
        return None
    try:
        return int(devs[index]["location_id"]) >> 8
    except (KeyError, ValueError):
        return None


def gpu_numa_node(index: int) -> int | None:
    """NUMA node of HIP device ``index`` (None when unknown or the host is not NUMA)."""
    devs = visible_gpus()
    if not 0 <= index < len(devs):
        return None
    bdf = _bdf(devs[index])
    if bdf is None:
        return None
    try:
        with open(os.path.join(SYSFS, "bus/pci/devices", bdf, "numa_node")) as f:
            n = int(f.read().strip())
    except (OSError, ValueError):
        return None
    return n if n >= 0 else None


def parse_cpulist(s: str) -> set[int]:
    cpus: set[int] = set()
    for part in s.strip().split(","):
        if not part:
            continue
        if "-" in part:
            a, b = part.split("-", 1)
            step = 1
            if ":" in b:
                b, st = b.split(":", 1)
                step = int(st)
            cpus.update(range(int(a), int(b) + 1, step))
        else:
            cpus.add(int(part))
    return cpus


def numa_cpus(node: int) -> set[int]:
    try:
        with open(os.path.join(SYSFS, f"devices/system/node/node{node}/cpulist")) as f:
            return parse_cpulist(f.read())
    except OSError:
        return set()


def numa_node_count() -> int:
    return len(glob.glob(os.path.join(SYSFS, "devices/system/node/node[0-9]*")))


def bind_to_gpu_numa(index: int) -> set[int] | None:
    """Restricts this process (and everything it forks afterwards) to the CPUs of
    the socket HIP device ``index`` is attached to.  No-op (returns None) on a
    single-node host, when the node is unknown, when ``TORCHKAFKA_NUMA=0``, or
    when the current affinity mask has no CPU on that node."""
    if os.environ.get("TORCHKAFKA_NUMA", "1") == "0" or numa_node_count() < 2:
        return None
    node = gpu_numa_node(index)
    if node is None:
        return None
    cur = os.sched_getaffinity(0)
    want = cur & numa_cpus(node)
    if not want:
        return None
    if want != cur:
        os.sched_setaffinity(0, want)
        log.debug("bound pid %d to NUMA node %d (%d CPUs) for GPU %d", os.getpid(), node, len(want), index)
    return want


def check_device(index: int) -> bool:
    """After HIP is initialised: does the sysfs prediction match HIP's PCI bus id?"""
    pred = gpu_pci_bus(index)
    if pred is None:
        return True
    try:
        import torch

        actual = torch.cuda.get_device_properties(index).pci_bus_id
    except Exception:  # noqa: BLE001
        return True
    if actual != pred:
        log.warning("NUMA binding predicted PCI bus %#x for GPU %d but HIP reports %#x; the CPU binding may "
                    "be on the wrong socket (set TORCHKAFKA_NUMA=0 to disable it)", pred, index, actual)
        return False
    return True
