"""Kafka error types (names mirror ``kafka.errors`` of kafka-python 2.0.2).

The reference imports ``kafka.errors.CommitFailedError`` (kafka_dataset.py:22)
and swallows it on commit (kafka_dataset.py:131-135).  The synthetic broker's
native core raises the same-named classes defined in ``_tkcore``; when
kafka-python is importable its classes are added to ``COMMIT_FAILED_ERRORS``
so either client's failures are handled identically.
"""
from __future__ import annotations

from ..ops.native import core

_c = core()

KafkaError = _c.KafkaError
CommitFailedError = _c.CommitFailedError
CorruptRecordException = _c.CorruptRecordException
OffsetOutOfRangeError = _c.OffsetOutOfRangeError
InjectedFetchError = _c.InjectedFetchError


class NoBrokersAvailable(KafkaError):
    """No synthetic broker at the given URL (and kafka-python unavailable)."""


class KafkaConfigurationError(KafkaError):
    """Unrecognized or invalid consumer/producer configuration."""


class NoOffsetForPartitionError(KafkaError):
    """No committed offset and ``auto_offset_reset='none'``."""


class IllegalStateError(KafkaError):
    """Operation not valid in the consumer's current state."""


class KafkaTimeoutError(KafkaError):
    """A bounded operation did not complete in time."""


COMMIT_FAILED_ERRORS: tuple[type[BaseException], ...] = (CommitFailedError,)
try:  # pragma: no cover - kafka-python is not installed in this image
    from kafka.errors import CommitFailedError as _KPCommitFailed  # type: ignore

    COMMIT_FAILED_ERRORS = (CommitFailedError, _KPCommitFailed)
except Exception:  # noqa: BLE001
    pass

__all__ = [
    "KafkaError", "CommitFailedError", "CorruptRecordException", "OffsetOutOfRangeError",
    "InjectedFetchError", "NoBrokersAvailable", "KafkaConfigurationError", "NoOffsetForPartitionError",
    "IllegalStateError", "KafkaTimeoutError", "COMMIT_FAILED_ERRORS",
]
