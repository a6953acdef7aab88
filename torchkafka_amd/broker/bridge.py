"""KafkaBridge: a real Kafka cluster feeding the device path.

The reference reads its cluster through kafka-python (``/root/reference/src/kafka_dataset.py:21-22,
206``): every worker's consumer parses Fetch responses and CRC-checks record batches in Python.
Here a native replicator (``csrc/core/replicator.cpp``, the Kafka wire protocol in
``csrc/core/kafka_wire.cpp``) fetches a rank's partitions with C++ threads and receives every
record set straight into the tail of a local partition log in shared memory -- the logs the
synthetic broker keeps.  The loader then runs unchanged on that local broker: workers walk record
headers, the main process pins the logs, gfx950 kernels verify CRC32C and decode the values.
Offsets are the cluster's own; every commit the loader makes into the local offset table is
forwarded to the group coordinator (OffsetCommit) by a committer thread, and ``close()`` flushes
the last one::

    bridge = KafkaBridge("broker1:9092,broker2:9092", "events", group_id="trainer",
                         partitions=shard_partitions(n_parts, rank, world))
    ds_init = Events.init_worker("events", bootstrap_servers=bridge.url, group_id="trainer")
    loader = DeviceLoader(Events.placeholder(), 256, num_workers=4, worker_init_fn=ds_init, ...)
    for batch in auto_commit(loader):
        ...
    bridge.close()          # forwards the final commit

Memory: by default (with a ``group_id``) each replica partition is a **ring** of ``ring_bytes``
(512 MiB): the
replicator writes over batches the group has committed, so the pages are allocated, and pinned by
a device loader, once -- a stream of any length needs no page freeing, unpinning or re-pinning,
and a full ring is the flow control (consumers behind by ``ring_bytes`` hold the fetches).  With
``ring_bytes=0`` the logs are linear and, with a ``group_id``, the committed part is released (the device
loader unpins it, the log start moves up to the committed offset and a background thread punches
the bytes below it out of the shm files in bursts of ``release_step``, keeping the last
``release_bytes`` of consumed log), so a long stream holds about ``max_lag_bytes + release_bytes +
release_step`` per partition in host memory, not the whole stream (each burst costs the GPU of a
device loader a ~25 ms stall: punching once-pinned pages makes the GPU driver revalidate);
``log_capacity`` (sparse) bounds the bytes one replica partition can take in over
its lifetime.

Semantics: at-least-once, like the reference's commit-after-batch.  A commit lands in the local
table synchronously and reaches the cluster within ``commit_interval_ms`` (5 ms); a crash in
between replays at most that window's batches.  Records are fetched read_uncommitted, control
batches (transaction markers) are dropped, compressed batches (gzip, snappy, lz4, zstd) are
CRC-checked and stored inflated (the device decoders read raw records); zstd needs the system's
libzstd.so.1 (without it such a batch stops its partition with an ``UnsupportedCodecError``).
"""
from __future__ import annotations

import logging
import os
import threading
import uuid
from typing import Iterable

from ..ops.native import core
from .synthetic import SyntheticBroker

log = logging.getLogger("torchkafka.bridge")

#: kafka-python configuration keys the native client understands for TLS / SASL
SECURITY_KEYS = ("security_protocol", "ssl_cafile", "ssl_check_hostname", "ssl_certfile", "ssl_keyfile",
                 "sasl_mechanism", "sasl_plain_username", "sasl_plain_password", "sasl_oauth_token_provider")


SASL_MECHANISMS = ("PLAIN", "SCRAM-SHA-256", "SCRAM-SHA-512", "OAUTHBEARER")


def oauth_token(provider) -> tuple[str, str]:
    """kafka-python's ``AbstractTokenProvider``: ``token()`` and, optionally, ``extensions()`` (a
    dict) -> (token, the extensions as RFC 7628 ``key=value`` pairs joined by 0x01)."""
    tok = provider.token()
    if not isinstance(tok, str) or not tok:
        raise ValueError("sasl_oauth_token_provider.token() must return a non-empty str")
    ext = {}
    if hasattr(provider, "extensions"):
        ext = provider.extensions() or {}
    bad = [k for k in ext if k == "auth" or not str(k).isalpha()]
    if bad:
        raise ValueError(f"SASL/OAUTHBEARER extension names must be alphabetic and not 'auth': {bad}")
    return tok, "\x01".join(f"{k}={v}" for k, v in ext.items())


def security_config(**kw) -> dict:
    """The TLS / SASL subset of a kafka-python configuration, for the native wire client
    (security_protocol PLAINTEXT | SSL | SASL_PLAINTEXT | SASL_SSL; SASL mechanism PLAIN,
    SCRAM-SHA-256, SCRAM-SHA-512 or OAUTHBEARER).  OAUTHBEARER's token is taken from
    ``sasl_oauth_token_provider`` here, in Python; a :class:`KafkaBridge` refreshes it."""
    out = {k: v for k, v in kw.items() if k in SECURITY_KEYS and v is not None}
    provider = out.pop("sasl_oauth_token_provider", None)
    mech = out.get("sasl_mechanism", "PLAIN")
    if out.get("security_protocol", "PLAINTEXT").startswith("SASL_"):
        if mech not in SASL_MECHANISMS:
            raise ValueError(f"sasl_mechanism {mech!r}: the native client speaks {', '.join(SASL_MECHANISMS)}")
        if mech == "OAUTHBEARER":
            if provider is None:
                raise ValueError("sasl_mechanism OAUTHBEARER needs sasl_oauth_token_provider (kafka-python's "
                                 "AbstractTokenProvider: token() and optionally extensions())")
            out["sasl_oauth_token"], out["sasl_oauth_extensions"] = oauth_token(provider)
    return out


class KafkaBridge:
    """Mirrors ``topic`` (all or ``partitions``) of a Kafka cluster into a local broker at :attr:`url`."""

    def __init__(self, bootstrap_servers: str | Iterable[str], topic: str, *, group_id: str | None = None,
                 partitions: Iterable[int] | None = None, url: str | None = None,
                 auto_offset_reset: str = "earliest", max_lag_bytes: int = 1 << 30,
                 log_capacity: int = 64 << 30, index_capacity: int = 1 << 22, fetch_max_wait_ms: int = 100,
                 fetch_max_bytes: int = 64 << 20, max_partition_fetch_bytes: int = 8 << 20,
                 request_timeout_ms: int = 30000, commit_interval_ms: int = 5, fetchers: int = 0,
                 client_id: str = "torchkafka-bridge", release_consumed: bool = True,
                 release_bytes: int = 256 << 20, release_step: int = 1 << 30, ring_bytes: int | None = None,
                 security_protocol: str = "PLAINTEXT", ssl_cafile: str | None = None, ssl_check_hostname: bool = True,
                 ssl_certfile: str | None = None, ssl_keyfile: str | None = None, sasl_mechanism: str | None = None,
                 sasl_plain_username: str | None = None, sasl_plain_password: str | None = None,
                 sasl_oauth_token_provider=None, oauth_refresh_s: float = 60.0, subscribe: bool = False,
                 session_timeout_ms: int = 10000, heartbeat_interval_ms: int = 3000,
                 partition_assignment_strategy: Iterable[str] = ("range",), rebalance_timeout_ms: int = 0,
                 start: bool = True):
        """``subscribe=True`` (needs ``group_id``, excludes ``partitions``): join the consumer group
        like kafka-python's ``subscribe()`` -- JoinGroup/SyncGroup with the range or round-robin
        assignor -- and mirror the partitions the coordinator assigns (:attr:`assignment`).
        Rebalances are followed in process, as kafka-python does: the bridge forwards what was
        consumed, rejoins, stops fetching revoked partitions and starts newly assigned ones at the
        group's committed offset; :attr:`assignment_epoch` tells the replica's consumers which
        partitions (re)started.  ``partition_assignment_strategy``: assignor names in preference
        order, "range" and/or "roundrobin" (kafka-python's two).  ``rebalance_timeout_ms``: how
        long the coordinator waits for members to rejoin (JoinGroup v1+; 0: the session timeout).
        Default: the static ``partitions`` (kafka-python's ``assign()``)."""
        if subscribe and not group_id:
            raise ValueError("subscribe=True needs a group_id")
        if subscribe and partitions is not None:
            raise ValueError("subscribe=True assigns partitions through the group: pass no partitions")
        if not isinstance(bootstrap_servers, str):
            bootstrap_servers = ",".join(bootstrap_servers)
        self.bootstrap_servers = bootstrap_servers
        self.topic = topic
        self.group_id = group_id
        self.url = url or f"shm://tkbridge-{os.getpid()}-{uuid.uuid4().hex[:8]}"
        if ring_bytes is None:  # a ring frees space as the group commits: without a group, a linear log
            ring_bytes = min(512 << 20, int(log_capacity)) if group_id else 0
        self._own = url is None
        self._subscribe = bool(subscribe)
        # a fresh local broker (or an existing persistent replica: file:// URLs resume their logs)
        self.local = SyntheticBroker(self.url, create=True, log_capacity=log_capacity,
                                     index_capacity=index_capacity)
        try:
            self._r = core().Replicator(
                self.local.native, bootstrap_servers, topic, group=group_id or "",
                partitions=sorted(int(p) for p in partitions) if partitions is not None else [],
                auto_offset_reset=auto_offset_reset, max_wait_ms=int(fetch_max_wait_ms), max_bytes=int(fetch_max_bytes),
                partition_max_bytes=int(max_partition_fetch_bytes), timeout_ms=int(request_timeout_ms),
                max_lag_bytes=int(max_lag_bytes), commit_interval_ms=int(commit_interval_ms), fetchers=int(fetchers),
                log_capacity=int(log_capacity), index_capacity=int(index_capacity), client_id=client_id,
                release_consumed=bool(release_consumed), release_bytes=int(release_bytes),
                release_step=int(release_step), ring_bytes=int(ring_bytes),
                security=security_config(security_protocol=security_protocol, ssl_cafile=ssl_cafile,
                                         ssl_check_hostname=ssl_check_hostname, ssl_certfile=ssl_certfile,
                                         ssl_keyfile=ssl_keyfile, sasl_mechanism=sasl_mechanism,
                                         sasl_plain_username=sasl_plain_username,
                                         sasl_plain_password=sasl_plain_password,
                                         sasl_oauth_token_provider=sasl_oauth_token_provider),
                subscribe=bool(subscribe), session_timeout_ms=int(session_timeout_ms),
                heartbeat_interval_ms=int(heartbeat_interval_ms),
                assignors=[str(a) for a in partition_assignment_strategy],
                rebalance_timeout_ms=int(rebalance_timeout_ms))
        except BaseException:
            if not self.url.startswith("file://"):  # a fresh shm replica nobody else can use
                self.local.destroy()
            raise
        self._closed = False
        self._lock = threading.Lock()
        self._reported = 0
        self._oauth_stop = threading.Event()
        if sasl_oauth_token_provider is not None and sasl_mechanism == "OAUTHBEARER":
            # connections made later (reconnects, the commit client, rebalance rejoins) present a
            # fresh token: the provider is asked again every oauth_refresh_s, from this Python thread
            threading.Thread(target=self._refresh_oauth, args=(sasl_oauth_token_provider, float(oauth_refresh_s)),
                             name="torchkafka-oauth", daemon=True).start()
        if start:
            self.start()

    def _refresh_oauth(self, provider, every: float) -> None:
        while not self._oauth_stop.wait(every):
            try:
                self._r.set_oauth_token(*oauth_token(provider))
            except Exception:  # noqa: BLE001 - the previous token stays; the next round retries
                log.exception("Bridge %s: sasl_oauth_token_provider failed", self.bootstrap_servers)

    # ------------------------------------------------------------ lifecycle
    def start(self) -> "KafkaBridge":
        self._r.start()
        log.debug("Bridge %s -> %s started (%d partitions).", self.bootstrap_servers, self.url,
                  len(self._r.stats()))
        return self

    def close(self, *, flush: bool = True, destroy: bool | None = None) -> None:
        """Stops fetching and forwards the latest commits (``flush``); removes an owned local broker."""
        with self._lock:
            if self._closed:
                return
            self._closed = True
        self._oauth_stop.set()
        self._r.stop(flush)
        self._report_errors()
        if destroy if destroy is not None else self._own:
            self.local.destroy()

    def __enter__(self) -> "KafkaBridge":
        return self

    def __exit__(self, *exc) -> None:
        self.close()

    def __del__(self):
        try:
            if not self._closed:
                self._r.stop(True)
        except Exception:  # noqa: BLE001 -- interpreter teardown
            pass

    # ------------------------------------------------------------ state
    @property
    def running(self) -> bool:
        return bool(self._r.running)

    def flush(self) -> int:
        """Forwards every changed local commit to the cluster now; returns partitions committed."""
        n = self._r.flush_commits()
        self._report_errors()
        return n

    def commit_sync(self, timeout: float = 30.0) -> bool:
        """Forwards the latest local commits now and waits for the coordinator's answer (the
        reference's synchronous ``consumer.commit()``, kafka_dataset.py:130).  True when every
        partition committed; False on a commit error (CommitFailedError in :meth:`last_error`) or
        timeout."""
        ok = bool(self._r.commit_sync(int(timeout * 1000)))
        if not ok:
            self._report_errors()
        return ok

    def take_forward_ns(self) -> list[int]:
        """OffsetCommit round-trip times (ns) of the forwards made since the last call."""
        return list(self._r.take_forward_ns())

    def wait_caught_up(self, timeout: float = 30.0) -> bool:
        """Blocks until every mirrored partition reached the cluster's current end offset."""
        return bool(self._r.wait_caught_up(int(timeout * 1000)))

    def stats(self) -> list[dict]:
        return list(self._r.stats())

    @property
    def subscribed(self) -> bool:
        """Group-managed (subscribe mode): the assignment follows the group's rebalances."""
        return bool(self._subscribe)

    @property
    def assignment(self) -> list[int]:
        """The partitions this bridge mirrors (subscribe mode: what the coordinator assigned)."""
        if self._subscribe:
            return sorted(self._r.assignment)
        return [s["partition"] for s in self.stats()]

    @property
    def assignment_epoch(self) -> int:
        """Bumped by every assignment change (subscribe mode)."""
        return int(self._r.assignment_epoch)

    def assignment_epochs(self) -> list[tuple[int, int]]:
        """``[(partition, epoch at which it was (re)assigned)]`` of the partitions owned now: a
        consumer that holds state of a partition from an older epoch must drop it (the partition
        was revoked and handed back, and restarted at the group's committed offset)."""
        return [(int(p), int(e)) for p, e in self._r.assignment_epochs()]

    @property
    def rebalances(self) -> int:
        """Rebalances this member went through since it started."""
        return int(self._r.rebalances)

    @property
    def out_of_order(self) -> int:
        """Record sets dropped (and refetched) because they did not start at the replica log's end."""
        return int(self._r.out_of_order)

    @property
    def member_id(self) -> str:
        return str(self._r.member_id)

    @property
    def generation(self) -> int:
        return int(self._r.generation)

    @property
    def fenced(self) -> bool:
        """Always False: rebalances are followed in process (kept for API compatibility)."""
        return False

    @property
    def errors(self) -> int:
        return int(self._r.errors)

    def last_error(self) -> str:
        return str(self._r.last_error())

    def _report_errors(self) -> None:
        n = self.errors
        if n > self._reported:
            log.warning("Bridge %s: %d error(s), last: %s", self.bootstrap_servers, n - self._reported,
                        self.last_error())
            self._reported = n
