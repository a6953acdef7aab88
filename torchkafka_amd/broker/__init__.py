"""Brokers: the synthetic shared-memory broker, its Kafka-protocol front end, and the bridge that
mirrors a real Kafka cluster into a local broker for the device path."""
from .bridge import KafkaBridge
from .synthetic import SyntheticBroker, is_synthetic_url, open_broker, resolve_url
from .wire_server import KafkaWireServer, NativeWireServer

__all__ = ["SyntheticBroker", "KafkaBridge", "KafkaWireServer", "NativeWireServer", "open_broker", "resolve_url",
           "is_synthetic_url"]
