"""LoaderConfig / Tuning: one validated configuration for DeviceLoader."""
import os

import pytest
import torch

from torchkafka_amd import DeviceLoader, FixedWidth, KafkaDataset, LoaderConfig, Tuning
from torchkafka_amd.config import TUNING_ENV


class Vec4(KafkaDataset):
    schema = FixedWidth(torch.float32, (4,))


def test_defaults_are_valid_and_round_trip():
    c = LoaderConfig()
    assert c.tuning.coalesce is None and c.sharding == "static"  # None: 6 fixed-width device decode, else 8
    d = c.to_dict()
    assert LoaderConfig.from_dict(d) == c
    assert set(d) == LoaderConfig.field_names() | {"tuning"}


@pytest.mark.parametrize("kw,msg", [
    ({"sharding": "random"}, "sharding"),
    ({"h2d": "pcie"}, "h2d"),
    ({"decode": "gpu"}, "decode"),
    ({"commit_on": "never"}, "commit_on"),
    ({"commit_sink": "x"}, "commit_sink"),
    ({"lockstep": "sometimes"}, "lockstep"),
    ({"pad_multiple": 0}, "pad_multiple"),
    ({"rank": 3, "world_size": 2}, "rank"),
    ({"normalize": 1.0}, "normalize"),
])
def test_invalid_behaviour_rejected(kw, msg):
    with pytest.raises(ValueError, match=msg):
        LoaderConfig(**kw)


@pytest.mark.parametrize("kw,msg", [
    ({"coalesce": 9}, "coalesce"), ({"copy_streams": 0}, "copy_streams"), ({"decode_streams": 5}, "decode_streams"),
    ({"slots_per_worker": 1}, "slots_per_worker"), ({"worker_spin_us": -1}, "worker_spin_us"),
    ({"ahead_depth": 99}, "ahead_depth"), ({"coalesce_wait_us": -5}, "coalesce_wait_us"),
])
def test_invalid_tuning_rejected(kw, msg):
    with pytest.raises(ValueError, match=msg):
        Tuning(**kw)


def test_environment_sets_tuning_defaults_explicit_wins(monkeypatch):
    monkeypatch.setenv(TUNING_ENV["ahead_depth"], "2")
    monkeypatch.setenv(TUNING_ENV["decode_streams"], "2")
    monkeypatch.setenv(TUNING_ENV["numa_bind"], "0")
    monkeypatch.setenv(TUNING_ENV["worker_spin_us"], "50")
    t = Tuning()
    assert (t.ahead_depth, t.decode_streams, t.numa_bind, t.worker_spin_us) == (2, 2, False, 50)
    assert Tuning(ahead_depth=6).ahead_depth == 6
    monkeypatch.setenv(TUNING_ENV["ahead_depth"], "lots")
    with pytest.raises(ValueError, match="TORCHKAFKA_AHEAD_DEPTH"):
        Tuning()


def test_build_routes_flat_keywords_and_rejects_unknown():
    base = LoaderConfig(sharding="group", tuning=Tuning(coalesce=2))
    c = LoaderConfig.build(base, coalesce=4, in_order=True, slots_per_worker=6)
    assert (c.sharding, c.in_order, c.tuning.coalesce, c.tuning.slots_per_worker) == ("group", True, 4, 6)
    assert base.tuning.coalesce == 2  # the given config is not mutated
    with pytest.raises(TypeError, match="coalese"):
        LoaderConfig.build(None, coalese=4)


def test_device_loader_takes_config_and_keyword_overrides(broker):
    cfg = LoaderConfig(group_id="g", bootstrap_servers=broker.url, in_order=True, tuning=Tuning(coalesce=3))
    dl = DeviceLoader(Vec4.placeholder(), 8, num_workers=1, device="cpu", config=cfg, prefetch=5)
    assert dl.in_order and dl.coalesce == 3 and dl.prefetch == 5
    assert dl.config.tuning.prefetch == 5 and cfg.tuning.prefetch == 2
    dl2 = DeviceLoader(Vec4.placeholder(), 8, num_workers=1, device="cpu", config=cfg.to_dict())
    assert dl2.config == cfg
    with pytest.raises(TypeError, match="unexpected DeviceLoader option"):
        DeviceLoader(Vec4.placeholder(), 8, device="cpu", not_an_option=1)
    with pytest.raises(ValueError, match="coalesce"):
        DeviceLoader(Vec4.placeholder(), 8, device="cpu", coalesce=0)


def test_config_doc_is_generated_from_the_code():
    """docs/CONFIG.md lists every LoaderConfig / Tuning field with a description (tools/gen_config_doc.py)."""
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(root, "tools", "gen_config_doc.py"), "--check"],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    text = open(os.path.join(root, "docs", "CONFIG.md")).read()
    assert not [ln for ln in text.splitlines() if ln.startswith("| `") and ln.rstrip().endswith("|  |")]
