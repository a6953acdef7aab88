"""Cross-cutting helpers: metrics/timers, platform probes."""
from .metrics import LoaderStats, StageTimer, percentile

__all__ = ["LoaderStats", "StageTimer", "percentile"]
