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
