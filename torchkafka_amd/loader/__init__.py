"""Loaders: auto_commit (reference API) and the device-resident DeviceLoader."""
from .auto_commit import auto_commit
from .device_loader import DeviceLoader, KafkaBatch, WorkerError

__all__ = ["auto_commit", "DeviceLoader", "KafkaBatch", "WorkerError"]
