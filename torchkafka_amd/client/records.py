"""Record / partition value types with kafka-python's field names.

``ConsumerRecord`` is what ``KafkaDataset._process`` receives (the reference's
README reads ``record.value``, README.md:74); field set per SURVEY.md §2.2.
"""
from __future__ import annotations

from collections import namedtuple

ConsumerRecord = namedtuple(
    "ConsumerRecord",
    ["topic", "partition", "offset", "timestamp", "timestamp_type", "key", "value", "headers", "checksum",
     "serialized_key_size", "serialized_value_size", "serialized_header_size"],
)

TopicPartition = namedtuple("TopicPartition", ["topic", "partition"])

OffsetAndMetadata = namedtuple("OffsetAndMetadata", ["offset", "metadata"])
OffsetAndTimestamp = namedtuple("OffsetAndTimestamp", ["offset", "timestamp"])

RecordMetadata = namedtuple(
    "RecordMetadata",
    ["topic", "partition", "topic_partition", "offset", "timestamp", "checksum", "serialized_key_size",
     "serialized_value_size", "serialized_header_size"],
)
