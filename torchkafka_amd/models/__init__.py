"""Dataset classes: the reference's KafkaDataset plus declarative record schemas."""
from .kafka_dataset import KafkaDataset
from .schema import FixedWidth, JsonArray, Key, Timestamp, VarLen, WithFields

__all__ = ["KafkaDataset", "FixedWidth", "VarLen", "JsonArray", "Key", "Timestamp", "WithFields"]
