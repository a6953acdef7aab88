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

    def __add__(self, field):
        return WithFields(self, (field,))

    # record fields beside the value (see WithFields): none
    fields: tuple = ()


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


# ---------------------------------------------------------------- record fields beside the value

_KEY_ENCODINGS = {"be": 0, "le": 1, "ascii": 2}


@dataclass(frozen=True)
class Key:
    """The record key as an int64 label beside the value: ``encoding`` "be" (8 bytes big-endian,
    Kafka's LongSerializer -- the default), "le" (8 bytes little-endian) or "ascii" (decimal
    digits).  A null key, or one the encoding cannot read, gives ``default``."""

    encoding: str = "be"
    default: int = -1

    bit = 1  # csrc/core/consumer.h kExtraKey

    def __post_init__(self):
        if self.encoding not in _KEY_ENCODINGS:
            raise ValueError(f"Key encoding {self.encoding!r}: one of {sorted(_KEY_ENCODINGS)}")

    def value_of(self, record) -> int:
        return int(core().key_int64(record.key, _KEY_ENCODINGS[self.encoding], int(self.default)))


@dataclass(frozen=True)
class Timestamp:
    """The record timestamp (ms, int64) beside the value."""

    bit = 2  # csrc/core/consumer.h kExtraTimestamp

    def value_of(self, record) -> int:
        return int(record.timestamp)


@dataclass(frozen=True)
class WithFields:
    """A fixed-width value plus per-record fields, e.g. ``FixedWidth(torch.float32, (256,)) +
    Key()`` -- a label riding with the features (the reference README's ``(features, label)``
    samples, README.md:40-44).  Batches are ``(values, key, timestamp)`` in the order the fields
    were added, each field an int64 tensor of one element per row.  On the device path the worker
    reads the fields while it walks the record headers and the gfx950 decode kernel copies them
    into the batch beside the values (no extra launch)."""

    value: FixedWidth
    fields: tuple = ()

    def __post_init__(self):
        if not isinstance(self.value, FixedWidth):
            raise TypeError("record fields ride with a FixedWidth value schema")
        bits = [f.bit for f in self.fields]
        if len(set(bits)) != len(bits):
            raise ValueError("each record field can be added once")
        if any(not isinstance(f, (Key, Timestamp)) for f in self.fields):
            raise TypeError("fields: Key() and/or Timestamp()")

    def __add__(self, field):
        return WithFields(self.value, self.fields + (field,))

    # the value schema's interface
    kind = 0

    @property
    def dtype(self):
        return self.value.dtype

    @property
    def shape(self):
        return self.value.shape

    @property
    def skip_bad(self):
        return self.value.skip_bad

    @property
    def row_elems(self) -> int:
        return self.value.row_elems

    @property
    def elem_size(self) -> int:
        return self.value.elem_size

    @property
    def row_bytes(self) -> int:
        return self.value.row_bytes

    def native_spec(self) -> tuple:
        return self.value.native_spec()

    def extras_spec(self) -> tuple:
        """(field bits, key encoding, key default) for the native packer; the columns are stored
        key first, then timestamp -- :meth:`column_order` maps them back to the order added."""
        key = next((f for f in self.fields if isinstance(f, Key)), None)
        bits = 0
        for f in self.fields:
            bits |= f.bit
        return bits, _KEY_ENCODINGS[key.encoding] if key else 0, int(key.default) if key else -1

    def column_order(self) -> list[int]:
        """Index of each added field among the native columns (key, timestamp)."""
        native = sorted(self.fields, key=lambda f: f.bit)
        return [native.index(f) for f in self.fields]

    def process(self, record):
        v = self.value.process(record)
        if v is None:
            return None
        return (v, *(torch.tensor(f.value_of(record), dtype=torch.int64) for f in self.fields))
