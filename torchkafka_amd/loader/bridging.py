"""DeviceLoader's Kafka-cluster side: bridges to a real cluster and the commit target.

When ``init_worker`` points the workers at a Kafka cluster (the reference's usage: every
worker's ``KafkaConsumer(topic, bootstrap_servers=..., group_id=...)``,
/root/reference/src/kafka_dataset.py:206, 219-231), the loader starts one native
:class:`~torchkafka_amd.broker.KafkaBridge` per topic that mirrors this rank's partitions into a
local replica broker; the device path then reads the replica and the commits reach the cluster's
group coordinator (``commit='sync'``: answered before the next batch is handed out).  This module
is the part of :class:`~torchkafka_amd.loader.DeviceLoader` that owns those bridges and resolves
where commits go.
"""
from __future__ import annotations

import logging
import os
import time

from ..client.errors import KafkaError

log = logging.getLogger("torchkafka_amd.loader.device_loader")
_ds_logger = logging.getLogger("torchkafka.kafka_dataset")


class LoaderBridges:
    """Mixin of :class:`~torchkafka_amd.loader.DeviceLoader`: ``_bridges`` (KafkaBridge list),
    ``_bridge_spec``, ``_group_id`` / ``_servers`` (the commit target)."""

    def _bridge_cluster(self, wi, forced: bool):
        """``bridge='auto'``: workers told to read a real Kafka cluster (``init_worker(topic,
        bootstrap_servers='host:9092', ...)``, the reference's usage) read a local replica instead,
        which a native :class:`~torchkafka_amd.broker.KafkaBridge` per topic fills with this rank's
        partitions; the device path (header walk, gfx950 CRC + decode) then runs unchanged and the
        commits reach the cluster's group coordinator.  Static sharding only (the bridge assigns
        partitions by rank; ``sharding='group'`` keeps kafka-python's group membership)."""
        from ..broker.synthetic import is_synthetic_url
        from ..models.kafka_dataset import _WorkerInit

        if not isinstance(wi, _WorkerInit) or self.sharding != "static":
            if forced:
                raise ValueError("bridge=True needs static sharding and a worker_init_fn from init_worker()")
            return wi
        servers = wi.kwargs.get("bootstrap_servers", "localhost:9092")  # kafka-python's default
        if is_synthetic_url(servers) or (not forced and os.environ.get("TORCHKAFKA_BROKER")):
            return wi
        topics = list(wi.args)
        if not topics or not all(isinstance(t, str) for t in topics):
            if forced:
                raise ValueError("bridge=True needs the topics named in init_worker()")
            return wi
        from ..broker.bridge import KafkaBridge
        from ..ops.native import core
        from ..parallel.sharding import shard_partitions

        if not isinstance(servers, str):
            servers = ",".join(servers)
        group = wi.kwargs.get("group_id")
        reset = wi.kwargs.get("auto_offset_reset", "latest")  # kafka-python's default
        from ..broker.bridge import SECURITY_KEYS, security_config

        security = security_config(**{k: v for k, v in wi.kwargs.items() if k in SECURITY_KEYS})
        client = core().WireClient(servers, "torchkafka-bridge", int(wi.kwargs.get("request_timeout_ms", 30000)),
                                   security)
        shares = {}
        for t in topics:
            err, parts = client.metadata(t)
            if err:
                raise KafkaError(f"UnknownTopicOrPartitionError: topic {t!r} on {servers}")
            shares[t] = shard_partitions(len(parts), self.rank, self.world_size)
        self._bridge_spec = (servers, group, reset, shares, security)
        url = self._start_bridges(None)
        log.info("DeviceLoader: %s mirrored into %s by %d KafkaBridge(s) (rank %d/%d).", servers, url,
                  len(self._bridges), self.rank, self.world_size)
        return _WorkerInit(wi.cls, wi.args, {**wi.kwargs, "bootstrap_servers": url})

    def _start_bridges(self, url):
        """One KafkaBridge per topic of ``self._bridge_spec`` into one replica broker (``url``: reuse
        that name); returns the replica's URL."""
        from ..broker.bridge import KafkaBridge

        servers, group, reset, shares, security = self._bridge_spec
        first = True
        try:
            for t, mine in shares.items():
                br = KafkaBridge(servers, t, group_id=group, partitions=mine, url=url, auto_offset_reset=reset,
                                 **security)
                br._own = first  # the first bridge owns the shared replica broker
                first = False
                url = br.url
                self._bridges.append(br)
        except BaseException:
            for br in self._bridges:
                br.close(flush=False)
            self._bridges.clear()
            raise
        return url

    def _resolve_commit_target(self, group_id, servers):
        from ..models.kafka_dataset import _WorkerInit

        if group_id is None or servers is None:
            wi = self.worker_init_fn
            if isinstance(wi, _WorkerInit):
                group_id = group_id if group_id is not None else wi.kwargs.get("group_id")
                servers = servers if servers is not None else wi.kwargs.get("bootstrap_servers")
            cons = getattr(self.dataset, "_consumer", None)
            if cons is not None and hasattr(cons, "config"):
                group_id = group_id if group_id is not None else cons.config.get("group_id")
                servers = servers if servers is not None else cons.config.get("bootstrap_servers")
        return group_id, servers

    def _commit_target_url(self) -> tuple[str, str]:
        if self._group_id is None or self._servers is None:
            return "", ""
        from ..broker.synthetic import resolve_url

        try:
            return resolve_url(self._servers), str(self._group_id)
        except Exception:  # noqa: BLE001 - not a synthetic broker: commits go through Python
            return "", ""

    def _sync_bridges(self, t0: int) -> bool:
        """commit='sync': waits for the coordinator's answer through every bridge this process
        commits into -- the loader's own (bridge='auto') or, single-process, the dataset
        consumer's (``KafkaDataset(topic, bootstrap_servers=cluster)``).  False: a coordinator
        refused a commit (logged, as the reference logs CommitFailedError)."""
        bridges = list(self._bridges)
        if self.num_workers == 0:
            bridges += getattr(getattr(self.dataset, "_consumer", None), "_bridges", None) or []
        ok = True
        for br in bridges:
            if not br._closed:
                ok = br.commit_sync() and ok
        if not ok:
            _ds_logger.error("Commit failed.")
            self.stats.commit_failures += 1
        self.stats.record_sync_commit(time.perf_counter_ns() - t0)
        return ok
