"""GPU -> NUMA resolution from a fake sysfs tree (utils/topology.py)."""
import os

import pytest

from torchkafka_amd.utils import topology


def _node(root, nid, simd, loc=None, render=None, uid=None):
    d = root / "sys/class/kfd/kfd/topology/nodes" / str(nid)
    d.mkdir(parents=True)
    lines = [f"simd_count {simd}"]
    if loc is not None:
        lines += [f"location_id {loc}", "domain 0"]
    if render is not None:
        lines.append(f"drm_render_minor {render}")
        (root / "dev/dri").mkdir(parents=True, exist_ok=True)
        (root / f"dev/dri/renderD{render}").write_text("")
    if uid is not None:
        lines.append(f"unique_id {uid}")
    (d / "properties").write_text("\n".join(lines) + "\n")


@pytest.fixture
def fake(tmp_path, monkeypatch):
    root = tmp_path
    _node(root, 0, 0)                                   # CPU node
    _node(root, 1, 0)                                   # CPU node
    _node(root, 2, 1024, loc=0x0500, render=128, uid=0xabc)   # bus 0x05 -> numa 0
    _node(root, 3, 1024, loc=0xF400, render=136, uid=0xdef)   # bus 0xf4 -> numa 1
    for bdf, n in (("0000:05:00.0", 0), ("0000:f4:00.0", 1)):
        p = root / "sys/bus/pci/devices" / bdf
        p.mkdir(parents=True)
        (p / "numa_node").write_text(f"{n}\n")
    for n, cl in ((0, "0-3,8-11"), (1, "4-7,12-15")):
        p = root / f"sys/devices/system/node/node{n}"
        p.mkdir(parents=True)
        (p / "cpulist").write_text(cl + "\n")
    monkeypatch.setattr(topology, "SYSFS", str(root / "sys"))
    monkeypatch.setattr(topology, "DEVDRI", str(root / "dev/dri"))
    for k in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES", "TORCHKAFKA_NUMA"):
        monkeypatch.delenv(k, raising=False)
    return root


def test_parse_cpulist():
    assert topology.parse_cpulist("0-3,8,10-14:2") == {0, 1, 2, 3, 8, 10, 12, 14}
    assert topology.parse_cpulist("") == set()


def test_gpu_order_and_numa(fake):
    assert [topology.gpu_pci_bus(i) for i in range(2)] == [0x05, 0xF4]
    assert topology.gpu_numa_node(0) == 0
    assert topology.gpu_numa_node(1) == 1
    assert topology.gpu_numa_node(2) is None
    assert topology.numa_cpus(1) == {4, 5, 6, 7, 12, 13, 14, 15}
    assert topology.numa_node_count() == 2


def test_visible_devices_env(fake, monkeypatch):
    monkeypatch.setenv("ROCR_VISIBLE_DEVICES", "1")
    assert topology.gpu_pci_bus(0) == 0xF4 and topology.gpu_pci_bus(1) is None
    monkeypatch.setenv("ROCR_VISIBLE_DEVICES", "GPU-abc,GPU-def")
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "1")
    assert topology.gpu_numa_node(0) == 1
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "")
    assert topology.visible_gpus() == []


def test_unopenable_render_node_is_skipped(fake):
    os.remove(fake / "dev/dri/renderD128")
    assert topology.gpu_pci_bus(0) == 0xF4


def test_bind(fake, monkeypatch):
    calls = []
    monkeypatch.setattr(os, "sched_getaffinity", lambda pid: set(range(16)))
    monkeypatch.setattr(os, "sched_setaffinity", lambda pid, cpus: calls.append(set(cpus)))
    assert topology.bind_to_gpu_numa(1) == {4, 5, 6, 7, 12, 13, 14, 15}
    assert calls == [{4, 5, 6, 7, 12, 13, 14, 15}]
    monkeypatch.setenv("TORCHKAFKA_NUMA", "0")
    assert topology.bind_to_gpu_numa(1) is None
    monkeypatch.delenv("TORCHKAFKA_NUMA")
    monkeypatch.setattr(os, "sched_getaffinity", lambda pid: {0, 1})   # user mask on the other socket
    assert topology.bind_to_gpu_numa(1) is None


@pytest.mark.gpu
def test_sysfs_prediction_matches_hip():
    import torch

    for i in range(torch.cuda.device_count()):
        pred = topology.gpu_pci_bus(i)
        assert pred is not None, "KFD topology not readable on a GPU host"
        assert pred == torch.cuda.get_device_properties(i).pci_bus_id
        assert topology.check_device(i)
