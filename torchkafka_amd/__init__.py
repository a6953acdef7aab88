"""torchkafka_amd: Kafka -> PyTorch streaming for AMD Instinct MI355X (gfx950).

Public API of Bendabir/torch-kafka (``KafkaDataset``, ``auto_commit``; reference
src/__init__.py:17-18) plus the MI355X device path (``DeviceLoader``), the
synthetic broker and a kafka-python compatible client.  ``import torchkafka``
is an alias of this package.
"""
import numpy.random  # noqa: F401  -- import eagerly: a lazy import racing a DataLoader fork deadlocks/crashes workers

from .config import LoaderConfig, Tuning
from .loader import DeviceLoader, KafkaBatch, auto_commit
from .models import FixedWidth, JsonArray, KafkaDataset, Key, Timestamp, VarLen, WithFields

__version__ = "1.2.0+mi355x.7"

__all__ = ["KafkaDataset", "auto_commit", "DeviceLoader", "KafkaBatch", "LoaderConfig", "Tuning", "FixedWidth",
           "VarLen", "JsonArray", "Key", "Timestamp", "WithFields", "SyntheticBroker", "KafkaBridge", "KafkaWireServer",
           "KafkaConsumer", "KafkaProducer", "TopicPartition", "ConsumerRebalanceListener"]


def __getattr__(name):
    if name in ("SyntheticBroker", "KafkaBridge", "KafkaWireServer"):
        from . import broker

        return getattr(broker, name)
    if name == "TopicPartition":
        from .client.records import TopicPartition

        return TopicPartition
    if name in ("KafkaConsumer", "KafkaProducer", "ConsumerRebalanceListener"):
        from . import client

        return getattr(client, name)
    raise AttributeError(name)
