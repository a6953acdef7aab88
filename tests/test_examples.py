"""The examples that run without a GPU run here (CPU path)."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_example_05_kafka_cluster_bridge_on_cpu():
    env = {**os.environ, "CUDA_VISIBLE_DEVICES": "", "HIP_VISIBLE_DEVICES": ""}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "examples", "05_kafka_cluster_bridge.py")],
                       capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "20000 records on cpu" in r.stdout
    assert "{0: 5000, 1: 5000, 2: 5000, 3: 5000}" in r.stdout


def test_example_06_group_subscribe_tls():
    import shutil

    import pytest
    if shutil.which("openssl") is None:
        pytest.skip("openssl CLI not available")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "examples", "06_group_subscribe_tls.py")],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "partitions [0, 1, 2], generation 1, 3000 records" in r.stdout
    assert "partitions [3, 4, 5], generation 1, 3000 records" in r.stdout
    assert "{0: 1000, 1: 1000, 2: 1000, 3: 1000, 4: 1000, 5: 1000}" in r.stdout


def test_example_07_labels_and_sync_commits_on_cpu():
    env = {**os.environ, "CUDA_VISIBLE_DEVICES": "", "HIP_VISIBLE_DEVICES": ""}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "examples", "07_labels_and_sync_commits.py")],
                       capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "4000 labelled records on cpu, 0 label mismatches" in r.stdout
    assert "{0: 2000, 1: 2000}" in r.stdout


def test_example_08_rebalance_listener():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "examples", "08_rebalance_listener.py")],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = r.stdout.splitlines()
    assert "worker 0: revoked []" in lines and "main: assigned [3]" in lines  # the visitor took a partition
    assert lines[-1] == "12000 records delivered; committed {0: 3000, 1: 3000, 2: 3000, 3: 3000}"
