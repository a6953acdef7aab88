"""Native ops: host core (_tkcore) and gfx950 collate kernels (_tkhip)."""
from .native import build_info, core, hip, loaded_extensions

__all__ = ["build_info", "core", "hip", "loaded_extensions", "collate_fixed", "collate_varlen"]


def __getattr__(name):
    if name in ("collate_fixed", "collate_varlen", "reference_fixed", "reference_varlen"):
        from . import collate

        return getattr(collate, name)
    raise AttributeError(name)
