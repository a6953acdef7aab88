"""PathPlan: which data path a DeviceLoader takes, decided once from its configuration.

Every choice below depends only on the loader's configuration (device, schema, ``native``,
``decode`` / ``h2d`` / ``json_parse`` knobs, whether ``_process`` is overridden, whether commits
go to the synthetic broker) -- never on what the stream delivers -- so it is computed once, when
the loader is built, and read as plain attributes on the hot path.  The reference has a single
path (kafka-python iterator -> ``_process`` -> DataLoader collate, /root/reference/src/
kafka_dataset.py:147-171); everything here is the device side SURVEY §2.6 adds:

* ``span``      fixed-width records decoded by the gfx950 kernel from the pinned broker logs
                (span_decode.hip: CRC32C of every RecordBatch, extraction, cast);
* ``var_span``  VarLen records padded/stacked by the same kernel family (varlen_span_kernel);
* ``json_span`` JsonArray texts parsed on the GPU straight from the logs (json_span.hip);
* ``json_device`` JsonArray texts framed by the workers and parsed by json_parse.hip;
* ``mirror``    h2d='dma' with device decode (and 'auto' for JSON): log bytes reach HBM on SDMA
                copy streams first;
* ``direct``    h2d='direct': fixed-width rows gathered from the pinned logs (experimental);
* ``fast_path`` / ``varlen_fast``: one argument-free native call per batch (torch_step.cpp).

Invalid combinations raise ``ValueError`` when the plan is built, with the reason.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Any

#: largest slot payload that ``h2d="auto"`` moves with zero-copy reads (above: DMA on side streams)
ZERO_COPY_MAX_BYTES = 1 << 20
#: slot room of a device-parsed JSON batch (decode='device') for the rows its worker parses itself
JSON_SPAN_HOST_VALUES_BYTES = 2 << 20
#: slot room of a device-decoded var-len batch for the values its worker copies (longer than a segment)
VAR_SPAN_HOST_VALUES_BYTES = 4 << 20
#: pinned bytes an automatically sized ring may take (fixed-width / var-len slots)
RING_AUTO_BYTES = 64 << 20
RING_AUTO_BYTES_VARLEN = 512 << 20


@dataclass(frozen=True)
class PathPlan:
    """The loader's data path (see the module docstring); build with :meth:`build`."""

    cuda: bool
    kind: Any                 # schema kind: 0 fixed, 1 var-len, 2 JSON array, None generic
    process_overridden: bool
    span: bool
    var_span: bool
    json_span: bool
    json_device: bool
    json_count: bool
    mirror: bool
    direct: bool
    fast_path: bool
    varlen_fast: bool
    h2d: str                  # as configured ('auto', 'dma', 'zerocopy', 'direct')

    @property
    def device_decode(self) -> bool:
        """Any schema decoded on the device straight from the pinned logs."""
        return self.span or self.json_span or self.var_span

    @classmethod
    def build(cls, *, device_type: str, schema, native: bool, decode: str, h2d: str, json_parse: str,
              synthetic_commits: bool, process_overridden: bool, return_info: bool, drop_last: bool,
              json_count_mode: str = "auto") -> "PathPlan":
        """``synthetic_commits``: the loader commits into the synthetic broker (shm:// or file://
        with a group_id) -- the device decoders read that broker's logs."""
        cuda = device_type == "cuda"
        kind = getattr(schema, "kind", None)
        usable = cuda and native and h2d != "direct" and synthetic_commits and not process_overridden

        span = decode != "host" and usable and kind == 0
        if decode == "device" and not span and kind not in (1, 2):
            raise ValueError("decode='device' needs a CUDA device, a FixedWidth schema, native=True, h2d != 'direct' "
                             "and the synthetic broker (bootstrap_servers shm:// or file://) with a group_id")
        var_span = decode != "host" and usable and kind == 1
        if decode == "device" and not var_span and kind == 1:
            raise ValueError("decode='device' for VarLen needs a CUDA device, native=True, h2d != 'direct' and the "
                             "synthetic broker (bootstrap_servers shm:// or file://) with a group_id")

        # JsonArray rows parsed by the gfx950 kernel instead of the workers: skip_bad=True needs a
        # row dropped from its batch, which only the host parser can do
        json_device = False
        if kind == 2 and json_parse != "host" and not process_overridden:
            ok = cuda and native and not getattr(schema, "skip_bad", False)
            if json_parse == "device" and not ok:
                raise ValueError("json_parse='device' needs a CUDA device, native=True and skip_bad=False")
            json_device = ok
        json_span = False
        if decode != "host" and json_device:
            json_span = h2d != "direct" and synthetic_commits
            if decode == "device" and not json_span:
                raise ValueError("decode='device' needs the synthetic broker (bootstrap_servers shm:// or file://) "
                                 "with a group_id and h2d != 'direct'")
        # device-counted JSON rows: filters that drop rows need the counts before the batch is packed
        json_count = False
        if json_span:
            ok = int(getattr(schema, "min_len", 0)) == 0 and (getattr(schema, "max_len", None) is None
                                                              or bool(schema.truncate))
            if json_count_mode == "device" and not ok:
                raise ValueError("tuning.json_count='device' cannot drop rows: needs min_len=0 and truncate=True")
            json_count = ok and json_count_mode != "host"

        fast_common = schema is not None and native and not return_info and not drop_last and not process_overridden
        fast_path = fast_common and kind == 0
        direct = False
        if h2d == "direct":
            if not cuda or not fast_path:
                raise ValueError("h2d='direct' needs a CUDA device, a FixedWidth schema, native=True, "
                                 "return_info=False and drop_last=False")
            if not synthetic_commits:
                raise ValueError("h2d='direct' needs the synthetic broker (bootstrap_servers shm:// or file://) "
                                 "and a group_id")
            direct = True
        # The HBM mirror: always with h2d='dma'; with h2d='auto' for JSON rows, where it beats
        # zero-copy with and without the RCCL lockstep (config 4: 46-52 M rec/s against 38 M, under
        # the lockstep 46-52 M against 33 M; profiles/r05_s35_mirror_rccl).  Fixed-width and var-len
        # decode stay zero-copy under 'auto': fixed-width runs at the PCIe roof either way (and the
        # mirror loses 40 % under the lockstep), var-len tokens 45-47 M zero-copy against 42-43 M
        # mirrored (under the lockstep 42-47 M against 31-37 M; round 4 had measured the reverse,
        # 43.3 / 46.2 M mirrored against 42.2 / 44.2 M) -- and zero-copy needs no HBM and no copy engine.
        mirror = (span or json_span or var_span) if h2d == "dma" else (h2d == "auto" and json_span)
        return cls(cuda=cuda, kind=kind, process_overridden=process_overridden, span=span, var_span=var_span,
                   json_span=json_span, json_device=json_device, json_count=json_count, mirror=mirror,
                   direct=direct, fast_path=fast_path, varlen_fast=fast_common and kind in (1, 2), h2d=h2d)

    # ------------------------------------------------------------------ H2D and ring sizing
    def resolve_h2d(self, slot_payload_bytes: int) -> str:
        """The H2D mechanism for slots of this size."""
        if self.h2d != "auto":
            return self.h2d
        if self.device_decode:
            # device decode: the slots hold row tables (a few KiB read once by the kernel), the values
            # stay in the pinned logs -- a DMA of the slot would only add a copy and an event per batch
            return "zerocopy"
        if self.json_device:
            # JSON text batches are a few hundred KiB whatever the slot capacity; the parse kernel
            # reads each row once, so zero-copy beats a DMA + HBM re-read (14.3 vs 12.6 M rec/s,
            # BASELINE config 4, profiles/r01_s5)
            return "zerocopy"
        return "zerocopy" if slot_payload_bytes <= ZERO_COPY_MAX_BYTES else "dma"

    def layout_capacity(self, batch_size: int, schema) -> int:
        """Slot bytes of one batch's layout (without record-field columns)."""
        B = batch_size
        if self.span:
            # row table (8 B per row) + SpanSeg entries: one per RecordBatch touched, plus one per
            # 32 KiB of values (kSpanSegMax cuts), with headroom
            segs = 2 * B + 128 + (B * schema.row_bytes) // (32 << 10)
            return (B * 8 + 255) // 256 * 256 + 32 * segs
        if self.json_span or self.var_span:
            # row table (16 B per row) + the values of rows the workers handle themselves (JSON rows
            # that are not "simple": exponents, NaN, long tokens; var-len values longer than a
            # segment; a batch closes early if they do not fit) + the segments (one per RecordBatch
            # touched, one per 128 KiB or 1024 rows, host-row groups)
            host = JSON_SPAN_HOST_VALUES_BYTES if self.json_span else VAR_SPAN_HOST_VALUES_BYTES
            return (B * 16 + 255) // 256 * 256 + host + 32 * (3 * B + 128)
        if self.kind == 0 and not self.process_overridden:
            return B * schema.row_bytes
        return 16 << 20

    def slots_per_worker(self, slot_capacity: int, n_producers: int, deep: bool = False) -> int:
        """Ring depth per worker when not configured.  ``deep``: an RCCL lockstep -- its agreements
        grant the batches staged beyond the last grant, so a deeper ring makes them rarer and gives
        each one more steps to come back in (DeviceLoader._lockstep_depth)."""
        if self.device_decode:
            # device-decode slots hold row positions only (a few KiB): a deep ring costs no pinned
            # memory and lets the workers run ahead while slots wait for their kernels
            return 64 if deep else 16
        budget = RING_AUTO_BYTES
        if self.kind in (1, 2) and self.cuda:
            # var-len / JSON slots are sized for the worst row (16 MiB) but hold a few hundred KiB:
            # 8 per worker keeps the workers off the slot-release wait (config 4: +4 %)
            budget = RING_AUTO_BYTES_VARLEN
        fit = budget // max(1, n_producers * slot_capacity)
        return int(max(4, min(8, fit)))

    def describe(self) -> dict:
        """What the plan chose, for logs and benchmark lines."""
        decode = ("host workers" if not self.device_decode else
                  "device from an HBM mirror filled by SDMA copies" if self.mirror else "device from the pinned logs")
        return {"decode": decode, "span": self.span, "var_span": self.var_span, "json_span": self.json_span,
                "json_device": self.json_device, "json_count": self.json_count, "mirror": self.mirror,
                "direct": self.direct, "fast_path": self.fast_path or self.varlen_fast}
