"""kafka-python compatible client over the synthetic broker."""
from .consumer import ConsumerRebalanceListener, KafkaConsumer
from .errors import (
    CommitFailedError, CorruptRecordException, KafkaConfigurationError, KafkaError, NoBrokersAvailable,
    OffsetOutOfRangeError,
)
from .producer import KafkaProducer
from .records import ConsumerRecord, OffsetAndMetadata, OffsetAndTimestamp, RecordMetadata, TopicPartition

__all__ = ["KafkaConsumer", "ConsumerRebalanceListener",
           "KafkaProducer", "ConsumerRecord", "TopicPartition", "OffsetAndMetadata",
           "OffsetAndTimestamp",
           "RecordMetadata", "KafkaError", "CommitFailedError", "CorruptRecordException", "NoBrokersAvailable",
           "OffsetOutOfRangeError", "KafkaConfigurationError"]
