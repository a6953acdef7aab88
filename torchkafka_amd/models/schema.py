"""Declarative record schemas: the native fast path's contract with a dataset.

The reference has one way to turn a record into a sample: a Python
``_process(record)`` per record (kafka_dataset.py:173-186).  A dataset that
declares ``schema = FixedWidth(...)``, ``VarLen(...)`` or ``JsonArray(...)``
additionally lets :class:`~torchkafka_amd.loader.DeviceLoader` decode whole
batches natively (C++ packer into the pinned ring, gfx950 collate kernel on
device) while keeping the per-record semantics, including the reference's
``None``-skip: a null value, or a row shorter than ``min_len``, is skipped and
still advances (and is committed with) the partition position (B6).

Every schema also provides ``process(record)``: the exact per-record
equivalent used by the torch-DataLoader compat path, so one dataset class
works with both loaders and both produce identical samples.
"""
from __future__ import annotations

import json
import math
from dataclasses import dataclass

import torch

from ..ops.native import core

_DT_CODE = {
    torch.float32: 0, torch.float16: 1, torch.bfloat16: 2, torch.float8_e4m3fn: 3, torch.uint8: 4,
    torch.int8: 5, torch.int32: 6, torch.int64: 7,
}


def dtype_code(dt: torch.dtype) -> int:
    try:
        return _DT_CODE[dt]
    except KeyError:
        raise TypeError(f"unsupported dtype {dt}") from None


@dataclass(frozen=True)
class FixedWidth:
    """Each record value is ``prod(shape)`` raw little-endian elements of ``dtype``."""

    dtype: torch.dtype = torch.float32
    shape: tuple = (256,)
    skip_bad: bool = False

    kind = 0

    @property
    def row_elems(self) -> int:
        return int(math.prod(self.shape))

    @property
    def elem_size(self) -> int:
        return torch.empty((), dtype=self.dtype).element_size()

    @property
    def row_bytes(self) -> int:
        return self.row_elems * self.elem_size

    def process(self, record):
        v = record.value
        if v is None:
            return None
        if len(v) != self.row_bytes:
            if self.skip_bad:
                return None
            raise ValueError(f"record at offset {record.offset}: value size {len(v)} != {self.row_bytes}")
        return torch.frombuffer(bytearray(v), dtype=self.dtype).view(self.shape)

    def native_spec(self) -> tuple:
        return (core().PACK_FIXED, self.elem_size, self.row_elems, 0, -1, True, self.skip_bad)


@dataclass(frozen=True)
class VarLen:
    """Each record value is a variable number of raw ``dtype`` elements (e.g. int32 token ids)."""

    dtype: torch.dtype = torch.int32
    min_len: int = 0
    max_len: int | None = None
    truncate: bool = True
    skip_bad: bool = False

    kind = 1

    @property
    def elem_size(self) -> int:
        return torch.empty((), dtype=self.dtype).element_size()

    def _filter(self, t):
        n = t.numel()
        if n < self.min_len:
            return None
        if self.max_len is not None and n > self.max_len:
            if not self.truncate:
                return None
            t = t[: self.max_len]
        return t

    def process(self, record):
        v = record.value
        if v is None:
            return None
        if len(v) % self.elem_size:
            if self.skip_bad:
                return None
            raise ValueError(f"record at offset {record.offset}: size not a multiple of {self.elem_size}")
        return self._filter(torch.frombuffer(bytearray(v), dtype=self.dtype) if v else
                            torch.empty(0, dtype=self.dtype))

    def native_spec(self) -> tuple:
        return (core().PACK_VARLEN, self.elem_size, 0, self.min_len,
                -1 if self.max_len is None else self.max_len, self.truncate, self.skip_bad)


@dataclass(frozen=True)
class JsonArray(VarLen):
    """Each record value is a flat JSON array of numbers, decoded to float32 (README.md:54,74 pattern)."""

    dtype: torch.dtype = torch.float32

    kind = 2

    @property
    def elem_size(self) -> int:
        return 4

    def process(self, record):
        v = record.value
        if v is None:
            return None
        try:
            vals = json.loads(v)
            if not isinstance(vals, list) or any(isinstance(x, (list, dict, str, bool)) or x is None for x in vals):
                raise ValueError
            t = torch.tensor([float(x) for x in vals], dtype=torch.float32)
        except ValueError:
            if self.skip_bad:
                return None
            raise ValueError(f"record at offset {record.offset}: not a flat numeric JSON array") from None
        return self._filter(t)

    def native_spec(self) -> tuple:
        return (core().PACK_JSON_F32, 4, 0, self.min_len, -1 if self.max_len is None else self.max_len,
                self.truncate, self.skip_bad)
