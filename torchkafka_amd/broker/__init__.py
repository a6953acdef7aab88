"""Synthetic shared-memory Kafka broker (stands in for a cluster; kafka-python is not installed)."""
from .synthetic import SyntheticBroker, is_synthetic_url, open_broker, resolve_url

__all__ = ["SyntheticBroker", "open_broker", "resolve_url", "is_synthetic_url"]
