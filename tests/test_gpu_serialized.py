"""Serialized-launch equivalence of the whole loader (VERDICT r4 weak 8 / "do this" 5).

The loader recycles ring slots by events (a slot returns to its worker once its group's event
completed), decodes groups ahead of the user on three decode streams, copies the partition logs
into an HBM mirror on copy streams (a launch reads a chunk still in flight from the pinned log
instead), and -- for var-len and JSON -- hands its decode- and copy-stream HIP calls to a command
queue thread.  Any missing event or stream dependency in that machinery is a race that a normal
run can hide and a serialized run cannot: with AMD_SERIALIZE_KERNEL=3 AMD_SERIALIZE_COPY=3
HIP_LAUNCH_BLOCKING=1 every kernel and copy waits for the previous one to finish, so the order of
completion is the order of submission.  The same four loaders (fixed-width, var-len, JSON, HBM
mirror) over the same topics must deliver bit-identical tensors, in the same order (in_order
delivery), and commit the same offsets -- normally, serialized with the command queue on, and
serialized with it off.  Each configuration is a process of its own (the variables are read at HIP
start-up): tests/helpers/serialized_child.py.  The reference avoids the race by design: its
batches never leave the CPU (/root/reference/src/kafka_dataset.py:164-165).
"""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

CHILD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "helpers", "serialized_child.py")
SERIAL = {"AMD_SERIALIZE_KERNEL": "3", "AMD_SERIALIZE_COPY": "3", "HIP_LAUNCH_BLOCKING": "1"}


@pytest.mark.timeout(300)
def test_serialized_launches_deliver_and_commit_the_same(broker):
    broker.create_topic("fixed", 4)
    broker.fill("fixed", 400, "fixed_f32", size=64, records_per_batch=24)
    broker.create_topic("tokens", 3)
    broker.fill("tokens", 300, "tokens_i32", size=1, max_size=64)
    broker.create_topic("json", 3)
    broker.fill("json", 300, "json_f32", size=4, max_size=40)
    runs = {}
    for tag, extra in (("plain", {}), ("serial-q1", {**SERIAL, "TORCHKAFKA_HIP_QUEUE": "1"}),
                       ("serial-q0", {**SERIAL, "TORCHKAFKA_HIP_QUEUE": "0"})):
        env = {k: v for k, v in os.environ.items() if k not in SERIAL and k != "TORCHKAFKA_HIP_QUEUE"}
        env.update(extra)
        r = subprocess.run([sys.executable, CHILD, broker.url, tag], env=env, capture_output=True, text=True,
                           timeout=240)
        assert r.returncode == 0, (tag, r.stderr[-3000:])
        runs[tag] = json.loads(r.stdout.strip().splitlines()[-1])
    plain = runs["plain"]
    assert plain["fixed"]["rows"] == 1600 and plain["mirror"]["rows"] == 1600
    assert plain["varlen"]["rows"] == 900 and plain["json"]["rows"] == 900
    assert plain["fixed"]["committed"] == {"0": 400, "1": 400, "2": 400, "3": 400}
    for tag in ("serial-q1", "serial-q0"):
        for name, want in plain.items():
            assert runs[tag][name] == want, (tag, name, runs[tag][name], want)
    # the mirror decodes the same records as zero-copy
    assert plain["mirror"]["digest"] == plain["fixed"]["digest"]
