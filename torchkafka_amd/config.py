"""Validated configuration of :class:`~torchkafka_amd.DeviceLoader`.

The reference has no configuration object: ``KafkaDataset(*topics, **kafka_config)`` forwards
everything to kafka-python (/root/reference/src/kafka_dataset.py:54-77) and the DataLoader takes
its own keyword arguments.  The device path adds behaviour switches and performance knobs; they
live here, in two dataclasses that validate on construction:

* :class:`LoaderConfig` -- what the loader does (sharding, padding, commit policy, lockstep,
  decode/H2D mechanism, ...).  Changing one of these changes results or semantics.
* :class:`Tuning` -- how fast it does it (ring depth, coalescing, streams, ...).  Any value
  gives the same batches and the same commits; defaults are the MI355X-measured ones
  (docs/PERFORMANCE.md), and the ``TORCHKAFKA_*`` environment variables listed in
  :data:`TUNING_ENV` override those defaults (an explicit argument wins over the environment).

``DeviceLoader(ds, 256, config=LoaderConfig(...), coalesce=4)`` mixes both: flat keyword
arguments override the config's fields (tuning fields are routed into ``config.tuning``), so
every keyword the loader accepted before keeps working.  ``docs/CONFIG.md`` is the full table.
"""
from __future__ import annotations

import dataclasses
import os
from dataclasses import dataclass, field, fields
from typing import Any, Optional

#: environment variables that change a :class:`Tuning` default (explicit values win)
TUNING_ENV = {
    "numa_bind": "TORCHKAFKA_NUMA",              # "0" disables the NUMA bind
    "ahead_depth": "TORCHKAFKA_AHEAD_DEPTH",
    "decode_streams": "TORCHKAFKA_DECODE_STREAMS",
    "worker_spin_us": "TORCHKAFKA_WORKER_SPIN_US",
}

#: process-wide switches read once by the native libraries or at import (not per loader)
PROCESS_ENV = {
    "TORCHKAFKA_BROKER": "default synthetic broker URL for KafkaDataset/DeviceLoader consumers",
    "TORCHKAFKA_ROCTX": "1: roctx ranges around every loader step (utils/tracing.py)",
    "TORCHKAFKA_CRC_FOLD": "host CRC32C kernel choice in the workers (csrc/core/crc32c.cpp)",
    "TORCHKAFKA_CRC_PREFETCH": "host CRC32C software-prefetch distance (bytes)",
    "TORCHKAFKA_CRC_FOLD_PREFETCH": "prefetch distance of the folded host CRC32C",
    "TORCHKAFKA_NT_COPY": "0: plain (cached) stores when workers pack slots",
    "TORCHKAFKA_DRIVER_TRACE": "1: step-driver trace lines on stderr (debugging)",
    "TORCHKAFKA_NO_REBUILD": "1: never rebuild stale in-tree extensions at import",
    "TORCHKAFKA_RCCL_WORDS": "kernel (default) / host / copy / graph: how the RCCL lockstep's agreement words reach "
                             "RCCL -- tiny copy kernels, RCCL on host-mapped memory, hipMemcpyAsync, or the "
                             "kernels and the all-reduce captured into one HIP graph per slot "
                             "(csrc/hip/rccl_issue.hip)",
    "TORCHKAFKA_LOCKSTEP_PRIORITY": "normal (default) / high: the RCCL lockstep stream's priority; high gives it a "
                                    "hardware queue of its own, where its agreements came back slower "
                                    "(profiles/r05_s19_rccl_matrix)",
    "TORCHKAFKA_TORCH_NCCL_ACTIVE": "1: DeviceLoader.stream_plan() counts torch's own NCCL streams at world 1 "
                                    "(a world-1 nccl group that ran a collective, as bench.py's N = 8 queue "
                                    "rehearsal does)",
    "TORCHKAFKA_DEFERRED_FREE": "0: a closing loader frees its device / pinned memory inline (hipFree waits for "
                                "the whole device) instead of on the deferred-release thread (csrc/hip/reaper.h)",
    "TORCHKAFKA_LOCKSTEP_TRACE": "1: the RCCL lockstep keeps host timestamps of every agreement "
                                 "(RcclLockstep.take_trace)",
    "TORCHKAFKA_SPAN_PARTS": "1 / 2 / 4 / 8 (default 8): workgroups per log segment in a device-decode launch whose "
                             "segments are all read from the HBM mirror (JSON: 1 unless set)",
    "TORCHKAFKA_LZ4_LIB": "0: decode LZ4 blocks with the built-in decoder instead of the system liblz4.so.1",
    "TORCHKAFKA_DECODE_PRIORITY": "high / normal (default) / low: HIP stream priority of the decode streams "
                                  "(csrc/hip/engine.hip; no measured effect beside a GEMM, profiles/r05_s2)",
    "TORCHKAFKA_MIRROR_COPY_STREAMS": "copy streams of the HBM mirror, partitions split p % n (1..4, default 2)",
    "TORCHKAFKA_HIP_QUEUE": "0: var-len / JSON device decode makes its decode- and mirror-copy-stream HIP calls on "
                            "the stepping thread instead of, in order, on a thread of their own (csrc/hip/hip_queue.h)",
    "TORCHKAFKA_MIRROR_WAIT": "1 / 0: a mirror launch waits for the copy of a chunk still in flight / reads that "
                              "segment from the pinned log (default: waits for fixed-width decode, whose launches "
                              "split segments over workgroups only then; not for JSON / var-len; A/B only)",
    "TORCHKAFKA_JSON_FUSED_COUNT": "1: with a fixed JSON width (pad_to) the parse kernel counts each device-counted "
                                   "row itself instead of json_count_kernel (GPU time per group -12 %, end to end "
                                   "within noise: profiles/r06_s12)",
}


def _env_int(name: str, default):
    v = os.environ.get(name)
    if v is None or v == "":
        return default
    try:
        return int(v)
    except ValueError as e:
        raise ValueError(f"{name}={v!r} is not an integer") from e


def _check(cond: bool, msg: str) -> None:
    if not cond:
        raise ValueError(msg)


@dataclass
class Tuning:
    """Performance knobs (results and commits do not depend on them).

    Attributes:
        slots_per_worker: ring depth per worker; None = auto (16 for device decode, else as deep as
            8 while the ring stays within 64 MiB of pinned memory, at least 4).
        slot_bytes: pinned bytes per ring slot; None = sized from the schema and batch size.
        prefetch: batches whose H2D is issued ahead of the user (DMA mode).
        copy_streams: HIP side streams for DMA copies (1..8).
        event_every: record a completion event every k slots; None = ring slots / 4, at most 4.
        coalesce: staged batches collated per kernel launch (1..8; 1 disables).  None: 6 for fixed-width
            device decode (steady 51.3-51.8 M rec/s against 49.5-50.3 M with 8, 20-step window +2 %), 8
            when those rows also carry Key / Timestamp columns (label 44.2-48.1 M against 37.8-40.2 M
            with 6, profiles/r06_s4) and otherwise (JSON 49.1-49.5 M against 44.7-46.6 M with 6;
            profiles/r05_s45_coalesce).
        coalesce_wait_us: how long to wait for a fuller group while the GPU is busy (0..10000).
        lockstep_depth: steps before its credits run out that the next cross-rank agreement is issued
            (0..64); None = auto: 32 under the RCCL lockstep with device decode (whose ring is then 64
            slots per worker deep, so an agreement's ~60-180 µs round trip is covered by the steps
            its credits still allow: profiles/r05_s24), else 2.
        lockstep_commit_every: async lockstep: a fresh agreement every this many steps (a few in
            flight, each granting at most twice that far ahead), so finished batches become
            committable about that often (0..4096; 0: one agreement at a time grants whatever every
            rank holds).  None = auto: 4 on the node-local shared-memory transport (an agreement costs
            well under a microsecond), 0 under RCCL (32 there: 32.5 batches per commit, p99 commit
            latency 279 us, -21 % at world 1; 0: ~220 batches, -3 %; profiles/r06_s5) and over a
            process group's all-reduce.
        numa_bind: bind the loader (and its workers) to the target GPU's socket.
        ahead_depth: device-decode groups launched ahead of the user's request (0..16); None = 4.
        decode_streams: HIP streams for the device decode kernels (1..4); None = 3.
        worker_spin_us: worker spin on a full sub-ring before sleeping (0..100000 us).
        mirror_chunk_mib: h2d='dma' with device decode: log bytes per hipMemcpyAsync into the HBM
            mirror of a partition log (1..1024 MiB).
        mirror_chunks: HBM mirror buffers per partition (2..64); K - 2 of them are prefetched ahead.
            6 by default.  Each launch's prefetches are queued after its copy event (a launch never
            waits for them): 8 MiB x 6 then runs 48-49 M rec/s steady (13-47 M before, when a launch's
            event also covered its own prefetches); 8 buffers still collapse (8-11 M; avoid).
            tools/sessions/experiments/mirror_probe.sh, mirror_probe2.sh.
        group_mib: device-decode groups stop growing at this many MiB of log bytes (1..1024): a
            group's batches become committable together, so large batches form small groups.
        json_count: JsonArray rows parsed on the device from the logs: who counts their elements.
            'auto' / 'device': the gfx950 stage kernel, while it stages the text (the workers read
            only record headers; the batch width is a device max); 'host': the workers pre-scan
            every text.  Filters that drop rows (min_len > 0, max_len without truncate) need the
            workers to count, so 'auto' leaves those to them.
    """

    slots_per_worker: Optional[int] = None
    slot_bytes: Optional[int] = None
    prefetch: int = 2
    copy_streams: int = 4
    event_every: Optional[int] = None
    coalesce: Optional[int] = None
    coalesce_wait_us: int = 50
    lockstep_depth: Optional[int] = None
    lockstep_commit_every: Optional[int] = None
    numa_bind: Optional[bool] = None
    ahead_depth: Optional[int] = None
    decode_streams: Optional[int] = None
    worker_spin_us: Optional[int] = None
    mirror_chunk_mib: int = 8
    mirror_chunks: int = 6
    group_mib: int = 16
    json_count: str = "auto"

    def __post_init__(self):
        # environment defaults for fields left at None
        if self.numa_bind is None:
            self.numa_bind = os.environ.get(TUNING_ENV["numa_bind"], "1") != "0"
        for name in ("ahead_depth", "decode_streams", "worker_spin_us"):
            if getattr(self, name) is None:
                setattr(self, name, _env_int(TUNING_ENV[name], None))
        if self.worker_spin_us is None:
            self.worker_spin_us = 200

        self.validate()

    def validate(self) -> None:
        _check(self.slots_per_worker is None or 2 <= int(self.slots_per_worker) <= 4096,
               "slots_per_worker must be in [2, 4096] (or None for auto)")
        _check(self.slot_bytes is None or int(self.slot_bytes) >= 256, "slot_bytes must be >= 256 (or None)")
        _check(0 <= int(self.prefetch) <= 64, "prefetch must be in [0, 64]")
        _check(1 <= int(self.copy_streams) <= 8, "copy_streams must be in [1, 8]")
        _check(self.event_every is None or 1 <= int(self.event_every) <= 4096, "event_every must be >= 1 (or None)")
        _check(self.coalesce is None or 1 <= int(self.coalesce) <= 8, "coalesce must be in [1, 8] (or None)")
        _check(0 <= int(self.coalesce_wait_us) <= 10_000, "coalesce_wait_us must be in [0, 10000]")
        _check(self.lockstep_depth is None or 0 <= int(self.lockstep_depth) <= 64, "lockstep_depth must be in [0, 64]")
        _check(self.lockstep_commit_every is None or 0 <= int(self.lockstep_commit_every) <= 4096,
               "lockstep_commit_every must be in [0, 4096]")
        _check(self.ahead_depth is None or 0 <= int(self.ahead_depth) <= 16, "ahead_depth must be in [0, 16]")
        _check(self.decode_streams is None or 1 <= int(self.decode_streams) <= 4, "decode_streams must be in [1, 4]")
        _check(0 <= int(self.worker_spin_us) <= 100_000, "worker_spin_us must be in [0, 100000]")
        _check(1 <= int(self.mirror_chunk_mib) <= 1024, "mirror_chunk_mib must be in [1, 1024]")
        _check(2 <= int(self.mirror_chunks) <= 64, "mirror_chunks must be in [2, 64]")
        _check(1 <= int(self.group_mib) <= 1024, "group_mib must be in [1, 1024]")
        _check(self.json_count in ("auto", "device", "host"), "json_count must be 'auto', 'device' or 'host'")


_CHOICES = {
    "sharding": ("static", "group"),
    "commit_on": ("host", "device"),
    "commit": ("async", "sync"),
    "verify": ("commit", "deliver"),
    "commit_sink": ("auto", "broker", "worker"),
    "h2d": ("auto", "dma", "zerocopy", "direct"),
    "decode": ("auto", "device", "host"),
    "json_parse": ("auto", "device", "host"),
    "multiprocessing_context": ("fork", "spawn", "forkserver"),
}
_CHOICE_HELP = {
    "h2d": "'auto', 'dma' (hipMemcpyAsync on side streams), 'zerocopy' or 'direct'",
    "decode": "'auto', 'device' (gfx950 RecordBatch decode) or 'host' (worker pack)",
    "json_parse": "'auto', 'device' (gfx950 parse kernel) or 'host' (worker parse)",
    "commit_sink": ("'auto', 'broker' (the main process stores offsets into the synthetic broker) or "
                    "'worker' (each worker's consumer commits its partitions)"),
    "verify": ("'commit' (a device-checked batch's CRC32C / parse verdict gates its commit: it is handed out "
               "while its kernel may still run) or 'deliver' (the verdict gates delivery: a corrupt batch raises "
               "CorruptRecordException before it is yielded, as kafka-python's check_crcs iterator does)"),
    "commit": ("'async' (batch k's offsets are stored when batch k+1 is requested; a KafkaBridge forwards "
               "them to the coordinator within commit_interval_ms) or 'sync' (batch k+1 is handed out only "
               "once the coordinator answered batch k's OffsetCommit)"),
}


@dataclass
class LoaderConfig:
    """Behaviour of a DeviceLoader (see DeviceLoader's docstring for each field's meaning)."""

    normalize: Any = None
    sharding: str = "static"
    in_order: bool = False
    drop_last: bool = False
    pad_to: Optional[int] = None
    pad_multiple: int = 8
    pad_value: float = 0
    return_mask: bool = False
    return_info: bool = False
    native: bool = True
    multiprocessing_context: str = "fork"
    commit_on: str = "host"
    commit: str = "async"
    verify: str = "deliver"
    commit_sink: str = "auto"
    lockstep: Any = True
    lockstep_timeout: float = 600.0
    rank: Optional[int] = None
    world_size: Optional[int] = None
    timeout: float = 0
    group_id: Optional[str] = None
    bootstrap_servers: Any = None
    base_seed: Optional[int] = None
    h2d: str = "auto"
    decode: str = "auto"
    json_parse: str = "auto"
    bridge: Any = "auto"
    tuning: Tuning = field(default_factory=Tuning)

    def __post_init__(self):
        if isinstance(self.tuning, dict):
            self.tuning = Tuning(**self.tuning)
        self.validate()

    def validate(self) -> None:
        for name, choices in _CHOICES.items():
            v = getattr(self, name)
            if v not in choices:
                raise ValueError(f"{name} must be {_CHOICE_HELP.get(name, ' or '.join(map(repr, choices)))}")
        _check(self.bridge in ("auto", True, False), "bridge must be 'auto', True or False")
        _check(self.lockstep in (True, False, "host", "rccl", "shm", "always"),
               "lockstep must be True, False, 'host', 'rccl', 'shm' or 'always'")
        _check(self.pad_to is None or int(self.pad_to) >= 1, "pad_to must be >= 1 (or None)")
        _check(int(self.pad_multiple) >= 1, "pad_multiple must be >= 1")
        _check(float(self.timeout) >= 0, "timeout must be >= 0 (0 waits forever)")
        _check(self.rank is None or int(self.rank) >= 0, "rank must be >= 0")
        _check(self.world_size is None or int(self.world_size) >= 1, "world_size must be >= 1")
        _check(self.rank is None or self.world_size is None or int(self.rank) < int(self.world_size),
               "rank must be < world_size")
        if self.normalize is not None:
            _check(isinstance(self.normalize, (tuple, list)) and len(self.normalize) == 2,
                   "normalize must be a (mean, std) pair")
        self.tuning.validate()

    # ---- construction helpers
    @classmethod
    def field_names(cls) -> set:
        return {f.name for f in fields(cls)} - {"tuning"}

    @classmethod
    def build(cls, config: "LoaderConfig | dict | None" = None, **overrides) -> "LoaderConfig":
        """A validated copy of ``config`` with ``overrides`` applied; tuning names are routed into
        ``tuning``.  Unknown names raise ``TypeError`` like an unexpected keyword argument."""
        if config is None:
            config = cls()
        elif isinstance(config, dict):
            config = cls.from_dict(config)
        elif not isinstance(config, cls):
            raise TypeError(f"config must be a LoaderConfig or a dict, got {type(config).__name__}")
        top = {k: v for k, v in overrides.items() if k in cls.field_names()}
        tun = {k: v for k, v in overrides.items() if k in {f.name for f in fields(Tuning)}}
        unknown = set(overrides) - set(top) - set(tun) - {"tuning"}
        if unknown:
            raise TypeError(f"unexpected DeviceLoader option(s): {', '.join(sorted(unknown))}")
        tuning = overrides.get("tuning", config.tuning)
        if isinstance(tuning, dict):
            tuning = Tuning(**tuning)
        tuning = dataclasses.replace(tuning, **tun) if tun else dataclasses.replace(tuning)
        return dataclasses.replace(config, **top, tuning=tuning)

    def to_dict(self) -> dict:
        d = {f.name: getattr(self, f.name) for f in fields(self) if f.name != "tuning"}
        d["tuning"] = dataclasses.asdict(self.tuning)
        return d

    @classmethod
    def from_dict(cls, d: dict) -> "LoaderConfig":
        d = dict(d)
        tuning = d.pop("tuning", None)
        unknown = set(d) - cls.field_names()
        if unknown:
            raise TypeError(f"unknown LoaderConfig field(s): {', '.join(sorted(unknown))}")
        return cls(**d, tuning=Tuning(**tuning) if isinstance(tuning, dict) else (tuning or Tuning()))
