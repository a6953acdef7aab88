"""Shared fixtures.  GPU tests are marked ``@pytest.mark.gpu`` and skipped without a GPU."""
import os
import sys
import uuid

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
os.environ.setdefault("PYTHONPATH", ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an AMD GPU (MI355X / gfx950)")
    config.addinivalue_line("markers", "slow: long-running test")


def pytest_collection_modifyitems(config, items):
    import torch

    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason="no GPU available")
    for item in items:
        if "gpu" in item.keywords:
            item.add_marker(skip)


@pytest.fixture(scope="session", autouse=True)
def _remove_leftover_shm():
    """Removes the shared-memory brokers / replicas this test process created and did not destroy
    (a test that failed half-way, a bridge whose cluster was unreachable)."""
    yield
    import glob
    import re
    import shutil

    pid = re.compile(rf"-{os.getpid()}(-|$)")
    for d in glob.glob("/dev/shm/torchkafka/*"):
        if pid.search(os.path.basename(d)):
            shutil.rmtree(d, ignore_errors=True)


@pytest.fixture
def broker():
    """A fresh shared-memory broker, destroyed after the test."""
    from torchkafka_amd.broker import SyntheticBroker

    url = f"shm://tktest-{os.getpid()}-{uuid.uuid4().hex[:8]}"
    b = SyntheticBroker.create(url, log_capacity=64 << 20, index_capacity=1 << 16,
                               group_initial_rebalance_delay_ms=300)
    try:
        yield b
    finally:
        b.destroy()


def synth_f32(p: int, o: int, j: int) -> float:
    """Python mirror of the native FIXED_F32 generator (broker.cpp synth_f32)."""
    if j == 0:
        return float(o)
    if j == 1:
        return float(p)
    return float(((o * 31 + j * 7 + p * 13) % 2001) - 1000) * 0.0625
