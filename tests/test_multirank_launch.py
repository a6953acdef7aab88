"""Launch-level multi-rank checks with torch.distributed.run (127.0.0.1 rendezvous).

* bench.py at N=2 on the CPU (gloo): the driver's multi-GPU command line, rehearsed without GPUs
  -- one JSON line from rank 0 with the whole-job aggregate and dp2.
* tools/lockstep_check.py at N=2 on ONE GPU (marked gpu): the native step driver's credit
  lockstep (csrc/core/lockstep.h) over the gloo transport, both ranks on cuda:0 (RCCL refuses two
  ranks on one device), at pipeline depths 0/2/5: every rank stops at the same step and commits
  only what every rank finished.
"""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _torchrun(nproc, script, *args, timeout=240, env=None):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), script, *args]
    e = dict(os.environ)
    e.update(env or {})
    e["PYTHONPATH"] = ROOT + os.pathsep + e.get("PYTHONPATH", "")
    return subprocess.run(cmd, cwd=ROOT, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True,
                          timeout=timeout, env=e)


def test_bench_two_ranks_gloo_cpu():
    r = _torchrun(2, "bench.py", "--gpus", "2", "--steps", "30", "--warmup", "5", "--device", "cpu",
                  "--steady-steps", "60", "--workers", "2", "--partitions-per-gpu", "4", "--bridge-steps", "8")
    assert r.returncode == 0, r.stdout[-3000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith('{"metric"')]
    assert len(lines) == 1, r.stdout[-3000:]
    out = lines[0]
    assert out["n_gpus"] == 2 and out["steps"] == 30 and out["config"]["parallelism"] == "dp2"
    assert out["config"]["partitions"] == 8 and out["config"]["global_batch"] == 512
    assert out["value"] > 0 and out["steady_state"]["records_per_s"] > 0


def test_bench_late_block_watchdog_still_prints_the_line():
    """A late (RCCL) block that hangs on every rank: each rank's watchdog gives up after
    TK_BENCH_LATE_TIMEOUT, rank 0 prints the one line with the block marked, and the job exits 0."""
    r = _torchrun(2, "bench.py", "--gpus", "2", "--steps", "20", "--warmup", "5", "--device", "cpu",
                  "--steady-steps", "40", "--extra-blocks", "", "--workers", "1", "--partitions-per-gpu", "2",
                  "--bridge-steps", "0", env={"TK_BENCH_TEST_LATE_HANG": "1", "TK_BENCH_LATE_TIMEOUT": "8"})
    assert r.returncode == 0, r.stdout[-3000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith('{"metric"')]
    assert len(lines) == 1, r.stdout[-3000:]
    out = lines[0]
    assert out["n_gpus"] == 2 and out["value"] > 0
    assert "watchdog" in out["steady_test_hang"]["error"]


def test_bench_failed_block_is_reported_and_the_run_goes_on():
    """One rank's secondary block fails (session r06_s18: a device CRC verdict in the four-rank dma
    block): the others leave the lockstepped block at once, the failure is reported under the
    block's key, and the later blocks and the line still run."""
    r = _torchrun(2, "bench.py", "--gpus", "2", "--steps", "20", "--warmup", "5", "--device", "cpu",
                  "--steady-steps", "40", "--extra-blocks", "label,f32", "--extra-steps", "4000", "--workers", "1",
                  "--partitions-per-gpu", "2", "--bridge-steps", "8", "--bridge-codecs", "",
                  env={"TK_BENCH_TEST_FAIL_BLOCK": "label"})
    assert r.returncode == 0, r.stdout[-3000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith('{"metric"')]
    assert len(lines) == 1, r.stdout[-3000:]
    out = lines[0]
    assert "injected" in out["steady_label"]["error"] or "lockstep" in out["steady_label"]["error"]
    assert out["steady_f32"]["records_per_s"] > 0 and out["bridge"]["async"]["records_per_s"] > 0


def _bench(*args, timeout=240):
    e = dict(os.environ)
    e.pop("WORLD_SIZE", None)
    e["PYTHONPATH"] = ROOT + os.pathsep + e.get("PYTHONPATH", "")
    return subprocess.run([sys.executable, "bench.py", *args], cwd=ROOT, stdout=subprocess.PIPE,
                          stderr=subprocess.PIPE, text=True, timeout=timeout, env=e)


def test_bench_self_launches_n_ranks_without_torchrun():
    """The driver's plain `python bench.py --gpus N` runs N ranks (never one rank silently)."""
    r = _bench("--gpus", "2", "--device", "cpu", "--steps", "30", "--warmup", "5", "--steady-steps", "60",
               "--extra-blocks", "f32", "--extra-steps", "40", "--workers", "2", "--bridge-steps", "8")
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith('{"metric"')]
    assert len(lines) == 1, r.stdout[-3000:]
    out = lines[0]
    assert out["n_gpus"] == 2 and out["config"]["parallelism"] == "dp2" and out["config"]["partitions"] == 16
    assert out["launcher"].startswith("bench.py self-launch")
    assert out["ranks"]["world_size"] == 2 and out["ranks"]["rank_id_sum"] == 1
    assert out["lockstep"]["world_size"] == 2
    assert len(out["per_rank_records_per_s"]) == 2
    ss = out["steady_state"]
    assert len(ss["per_rank_records_per_s"]) == 2 and ss["lockstep_agreements"] >= 60
    assert out["steady_f32"]["dtype"] == "f32" and out["steady_f32"]["steps"] == 40
    br = out["bridge"]
    assert br["async"]["steps"] == 8 and br["sync"]["steps"] == 2 and len(br["sync"]["per_rank_records_per_s"]) == 2
    assert br["async"]["bridge_errors"] == 0 and br["sync"]["sync_commits"] >= 1


def test_bench_refuses_more_ranks_than_visible_gpus():
    import torch

    if torch.cuda.device_count() >= 64:
        pytest.skip("64 GPUs visible")
    r = _bench("--gpus", "64", "--steps", "5", "--warmup", "1", timeout=120)
    assert r.returncode == 2 and "refusing" in r.stderr, (r.returncode, r.stderr[-2000:])
    assert '{"metric"' not in r.stdout


def _rank_lines(out: str) -> list:
    """Every '{"rank": ...}' object the ranks printed (their lines may interleave on one line)."""
    dec = json.JSONDecoder()
    found, i = [], out.find('{"rank"')
    while i >= 0:
        obj, end = dec.raw_decode(out, i)
        found.append(obj)
        i = out.find('{"rank"', end)
    return found


@pytest.mark.gpu
def test_native_lockstep_two_ranks_one_gpu():
    r = _torchrun(2, "tools/lockstep_check.py", timeout=200)
    assert r.returncode == 0, r.stdout[-4000:]
    oks = _rank_lines(r.stdout)
    assert len(oks) == 2 and all(o["ok"] for o in oks), r.stdout[-4000:]


def test_bench_eight_ranks_on_cpu_without_torchrun():
    """The driver's N = 8 command line (`python bench.py --gpus 8`, no torchrun) rehearsed on the CPU
    over gloo: 8 self-launched ranks, 64 partitions, every rank's rate reported, one JSON line."""
    r = _bench("--gpus", "8", "--device", "cpu", "--workers", "1", "--steps", "20", "--warmup", "5",
               "--steady-steps", "200", "--extra-blocks", "", "--bridge-steps", "0", "--config-blocks", "",
               timeout=400)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith('{"metric"')]
    assert len(lines) == 1, r.stdout[-3000:]
    out = lines[0]
    assert out["n_gpus"] == 8 and out["config"]["parallelism"] == "dp8" and out["config"]["partitions"] == 64
    assert out["launcher"].startswith("bench.py self-launch")
    assert out["ranks"]["world_size"] == 8 and out["ranks"]["rank_id_sum"] == 28
    assert len(out["per_rank_records_per_s"]) == 8 and all(v > 0 for v in out["per_rank_records_per_s"])
    assert len(out["steady_state"]["per_rank_records_per_s"]) == 8
    assert out["memory_preflight"]["local_ranks"] == 8 and out["memory_preflight"]["scale"] == 1.0


@pytest.mark.gpu
def test_bench_launcher_parent_never_initialises_hip(tmp_path):
    """The launcher path the driver's N > 1 runs take, exercised at --gpus 1 (--self-launch): the
    parent counts GPUs without a HIP call (KFD sysfs + amdsmi) and starts its rank with Popen
    having neither initialised torch's HIP state nor opened /dev/kfd."""
    rep = tmp_path / "parent.json"
    e = dict(os.environ)
    e.pop("WORLD_SIZE", None)
    e["TK_BENCH_PARENT_REPORT"] = str(rep)
    e["PYTHONPATH"] = ROOT + os.pathsep + e.get("PYTHONPATH", "")
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "1", "--self-launch", "--steps", "20", "--warmup", "5",
                        "--steady-steps", "500", "--extra-blocks", "", "--bridge-steps", "0", "--config-blocks", ""],
                       cwd=ROOT, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=240, env=e)
    assert r.returncode == 0, r.stderr[-3000:]
    parent = json.load(open(rep))
    assert parent["torch_cuda_initialized"] is False and parent["kfd_fds"] == 0, parent
    assert parent["gpus_visible"]["count"] >= 1, parent
    out = [json.loads(x) for x in r.stdout.splitlines() if x.startswith('{"metric"')][0]
    assert out["launcher"].startswith("bench.py self-launch") and out["n_gpus"] == 1
