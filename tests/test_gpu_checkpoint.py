"""The global-step checkpoint on the native (GPU) step driver: ``state_dict(global_step=True)``
reads the driver's delivered positions (csrc/hip/driver.h ``delivered_positions``), so a loader
stopped after step S and a new loader resumed from its state see every record exactly once.
The multi-rank form over gloo is tests/test_ddp_checkpoint.py; the reference's checkpoint is the
group's committed offsets (/root/reference/src/kafka_dataset.py:85-91)."""
import json

import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("stop_at", [0, 5])
def test_native_global_step_checkpoint_resumes_exactly_once(broker, stop_at):
    from torchkafka_amd import DeviceLoader, FixedWidth, KafkaDataset, auto_commit

    class Vec(KafkaDataset):
        schema = FixedWidth(torch.float32, (16,))

    broker.create_topic("t", 4)
    broker.fill("t", 200, "fixed_f32", size=16, records_per_batch=20)

    def loader():
        return DeviceLoader(Vec.placeholder(), 32, num_workers=2, device="cuda:0", dtype=torch.float32,
                            worker_init_fn=Vec.init_worker("t", bootstrap_servers=broker.url, group_id="gck",
                                                           auto_offset_reset="earliest", consumer_timeout_ms=400))

    def rows(x):
        return [(int(p), int(o)) for o, p in x[:, :2].long().cpu().tolist()]

    dl = loader()
    seen1, state = [], None
    for step, x in enumerate(auto_commit(dl)):
        seen1 += rows(x)
        if step == stop_at:
            state = dl.state_dict(global_step=True)
            break
    dl.close()
    assert state["version"] == 2 and state["global_step"] == stop_at + 1 and state["world_size"] == 1
    ck = {int(p): o for p, o in state["offsets"]["t"].items()}
    for p in range(4):
        assert sorted(o for q, o in seen1 if q == p) == list(range(ck.get(p, 0)))
    state = json.loads(json.dumps(state))  # as saved beside a model checkpoint
    dl2 = loader()
    dl2.load_state_dict(state)
    seen2 = []
    for x in auto_commit(dl2):
        seen2 += rows(x)
    end = dl2.state_dict(global_step=True)
    dl2.close()
    both = seen1 + seen2
    assert len(both) == len(set(both)) == 800
    assert end["global_step"] > state["global_step"]  # counts on from the checkpoint
    assert {int(p): o for p, o in end["offsets"]["t"].items()} == {0: 200, 1: 200, 2: 200, 3: 200}
