"""``torchkafka``: the reference's import name (setup.py:25-27), re-exporting torchkafka_amd."""
from torchkafka_amd import *  # noqa: F401,F403
from torchkafka_amd import DeviceLoader, KafkaDataset, __version__, auto_commit  # noqa: F401
