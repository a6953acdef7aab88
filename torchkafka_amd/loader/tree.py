"""Structured samples on the DeviceLoader: tuple / list / dict ``_process`` results.

In the reference, ``_process`` may return any object the DataLoader's ``default_collate`` can
stack -- typically ``(features, label)`` or ``{"x": ..., "y": ...}`` -- and the batch has the same
structure with every leaf stacked along a new first dimension
(/root/reference/src/kafka_dataset.py:159-162, README.md:40-44, 72-79; [torch]
_utils/collate.py).  Here a worker flattens the samples of one batch into leaves, writes one
stacked region per leaf into its pinned ring slot behind a small JSON descriptor (the
structure, and each leaf's dtype, shape and offset), and the main process moves the whole slot
to the device with ONE copy; each leaf of the delivered batch is a view of that block.  Leaves
follow ``default_collate``: tensors and numpy arrays are stacked (equal shapes required), Python
``bool`` / ``int`` / ``float`` become ``bool`` / ``int64`` / ``float64`` tensors, strings and
bytes stay host lists, and -- as in ``default_collate`` -- a tuple comes back as a list (a
namedtuple keeps its type).

Slot payload (``PACK_TREE``): ``uint32 n`` | ``n`` bytes of JSON | pad to 256 | leaf regions,
each 256-byte aligned.
"""
from __future__ import annotations

import json
import struct

import numpy as np
import torch

_ALIGN = 256


def _align(n: int) -> int:
    return (n + _ALIGN - 1) // _ALIGN * _ALIGN


def flatten(sample, leaves: list) -> list:
    """Structure of ``sample`` (JSON-able), appending its leaves to ``leaves``."""
    if isinstance(sample, dict):
        return ["d", [[k, flatten(v, leaves)] for k, v in sample.items()]]
    if isinstance(sample, tuple) and hasattr(sample, "_fields"):  # a namedtuple keeps its type
        cls = type(sample)
        return ["nt", f"{cls.__module__}:{cls.__qualname__}", [flatten(v, leaves) for v in sample]]
    if isinstance(sample, tuple):
        return ["t", [flatten(v, leaves) for v in sample]]
    if isinstance(sample, list):
        return ["l", [flatten(v, leaves) for v in sample]]
    if sample is None:
        raise TypeError("DeviceLoader samples cannot hold None leaves (return None for the whole record to skip it)")
    leaves.append(sample)
    return ["x", len(leaves) - 1]


def _column(vals: list):
    """A leaf across the batch -> ('tensor', stacked CPU tensor) or ('host', [str | bytes])."""
    v0 = vals[0]
    if isinstance(v0, (str, bytes)):
        if not all(type(v) is type(v0) for v in vals):
            raise TypeError("a leaf mixes strings/bytes with other types across the batch")
        return "host", list(vals)
    if isinstance(v0, bool):
        return "tensor", torch.tensor(vals, dtype=torch.bool)
    if isinstance(v0, int):
        return "tensor", torch.tensor(vals, dtype=torch.int64)
    if isinstance(v0, float):
        return "tensor", torch.tensor(vals, dtype=torch.float64)
    ts = [torch.as_tensor(v) if isinstance(v, (np.ndarray, np.generic)) else v for v in vals]
    if not all(isinstance(t, torch.Tensor) for t in ts):
        raise TypeError("DeviceLoader sample leaves must be tensors, arrays, numbers or strings, "
                        f"got {type(v0).__name__}")
    t0 = ts[0]
    if any(t.shape != t0.shape or t.dtype != t0.dtype for t in ts):
        raise RuntimeError("each element in list of batch should be of equal size")  # default_collate's message
    return "tensor", ts


def pack(samples: list, view: memoryview, cap: int) -> int:
    """Writes one batch of structured samples into a ring slot payload; returns its bytes."""
    leaves0: list = []
    spec = flatten(samples[0], leaves0)
    cols: list = [[] for _ in leaves0]
    for s in samples:
        lv: list = []
        if flatten(s, lv) != spec:
            raise TypeError("the samples of one batch must share their structure (keys, lengths, nesting)")
        for i, x in enumerate(lv):
            cols[i].append(x)
    fields, regions, rel = [], [], 0
    for c in cols:
        kind, v = _column(c)
        if kind == "host":
            fields.append({"k": "s" if isinstance(v[0], str) else "b",
                           "v": v if isinstance(v[0], str) else [x.hex() for x in v]})
            continue
        if isinstance(v, list):
            t0 = v[0]
            shape, dt, nb = [len(v), *t0.shape], t0.dtype, len(v) * t0.numel() * t0.element_size()
        else:
            shape, dt, nb = list(v.shape), v.dtype, v.numel() * v.element_size()
        fields.append({"k": "t", "dt": str(dt).replace("torch.", ""), "shape": shape, "off": rel, "nb": nb})
        regions.append((rel, v, dt, shape, nb))
        rel = _align(rel + nb)
    desc = json.dumps({"tree": spec, "fields": fields, "n": len(samples)}, separators=(",", ":")).encode()
    data = _align(4 + len(desc))
    total = data + rel
    if total > cap:
        raise RuntimeError(f"batch of {total} bytes exceeds the ring slot ({cap}); raise slot_bytes")
    view[0:4] = struct.pack("<I", len(desc))
    view[4:4 + len(desc)] = desc
    for off, v, dt, shape, nb in regions:
        if not nb:
            continue
        dst = torch.frombuffer(view, dtype=torch.uint8, count=nb, offset=data + off)
        if isinstance(v, list):
            torch.stack(v, out=dst.view(dt).view(shape))
        else:
            dst.copy_(v.contiguous().view(-1).view(torch.uint8))
    return total


def descriptor(view: memoryview) -> tuple[dict, int]:
    """(descriptor, byte offset of the leaf regions) of a packed slot."""
    (n,) = struct.unpack_from("<I", view, 0)
    return json.loads(bytes(view[4:4 + n])), _align(4 + n)


def unpack(desc: dict, data: int, block: torch.Tensor, float_dtype: torch.dtype | None = None):
    """The batch: ``block`` holds the slot's bytes (device or host), leaves are views into it;
    floating leaves are cast to ``float_dtype`` when it is given."""
    leaves = []
    for f in desc["fields"]:
        if f["k"] == "s":
            leaves.append(list(f["v"]))
            continue
        if f["k"] == "b":
            leaves.append([bytes.fromhex(x) for x in f["v"]])
            continue
        dt = getattr(torch, f["dt"])
        start = data + f["off"]
        t = block[start:start + f["nb"]].view(dt).view(f["shape"])
        if float_dtype is not None and t.is_floating_point() and t.dtype != float_dtype:
            t = t.to(float_dtype)
        leaves.append(t)
    return _build(desc["tree"], leaves)


def _namedtuple(name: str):
    import importlib

    mod, _, qual = name.partition(":")
    try:
        obj = importlib.import_module(mod)
        for part in qual.split("."):
            obj = getattr(obj, part)
        return obj
    except (ImportError, AttributeError):
        return None


def _build(spec, leaves):
    tag = spec[0]
    if tag == "x":
        return leaves[spec[1]]
    if tag in ("t", "l"):  # default_collate turns a tuple into a list (collate.py: "Backwards compatibility")
        return [_build(c, leaves) for c in spec[1]]
    if tag == "nt":
        cls = _namedtuple(spec[1])
        vals = [_build(c, leaves) for c in spec[2]]
        return cls(*vals) if cls is not None else vals
    return {k: _build(c, leaves) for k, c in spec[1]}
