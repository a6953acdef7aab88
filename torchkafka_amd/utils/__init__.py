"""Cross-cutting helpers: metrics/timers, platform probes."""
from .metrics import LoaderStats, StageTimer, percentile
from .tracing import mark, trace_range

__all__ = ["LoaderStats", "StageTimer", "percentile", "trace_range", "mark"]
