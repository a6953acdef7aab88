"""Main -> worker commit requests through shared memory (replaces signals for auto_commit).

The reference asks a worker to commit with SIGUSR1 (kafka_dataset.py:235-239)
and the worker commits its consumer *position*, which already includes every
prefetched batch (B10/D3); after the stream ends the default action of the
signal kills the worker (D4).  Here the main process publishes, per worker,
the cumulative number of that worker's *batches* the user has finished with
(counted by the main process, so a collate_fn that reshapes batches cannot
skew it); the worker maps batch k to the consumer positions it recorded after
its sample min(k * batch_size, produced) and commits exactly those.  Workers acknowledge, so the
main process can wait for the final commit before tearing workers down.
"""
from __future__ import annotations

import time
from multiprocessing import shared_memory

import numpy as np

_REQ, _ACK, _PID, _HDR = 0, 1, 2, 5
_W = 3  # words per worker: request, acknowledgement, pid
_CLOSING = 2  # header word: the main process will send no further requests
_EPOCH = 3  # header word: the iteration (auto_commit pass over the loader) requests belong to
_ACTIVE = 4  # header word: an auto_commit iteration is running (workers stamp their batches)
# Requests and acknowledgements carry their iteration in the high bits: a persistent worker (one
# DataLoader's workers serve every iteration) never takes a request or an acknowledgement of an
# earlier iteration for one of this iteration.
_EPOCH_SHIFT = 40
_COUNT_MASK = (1 << _EPOCH_SHIFT) - 1


class CommitChannel:
    def __init__(self, num_workers: int, batch_size: int):
        if num_workers < 1 or batch_size < 1:
            raise ValueError("commit channel needs num_workers >= 1 and batch_size >= 1")
        self.num_workers = num_workers
        self.batch_size = batch_size
        self._shm = shared_memory.SharedMemory(create=True, size=8 * (_HDR + _W * num_workers))
        self._owner = True
        self._arr = np.ndarray((_HDR + _W * num_workers,), dtype=np.int64, buffer=self._shm.buf)
        self._arr[:] = 0
        self._arr[0] = num_workers
        self._arr[1] = batch_size
        self._arr[_EPOCH] = 1

    # ---- iterations (persistent workers serve several)
    def epoch(self) -> int:
        return int(self._arr[_EPOCH])

    def begin_epoch(self) -> int:
        """The main process starts another iteration over the same workers: requests restart at 0
        (tagged with the new epoch), the channel is open and batches are stamped again."""
        e = self.epoch() + 1
        for w in range(self.num_workers):
            self._arr[self._i(w, _REQ)] = e << _EPOCH_SHIFT
        self._arr[_CLOSING] = 0
        self._arr[_EPOCH] = e
        return e

    def set_active(self, on: bool) -> None:
        self._arr[_ACTIVE] = 1 if on else 0

    def active(self) -> bool:
        return bool(self._arr[_ACTIVE])

    # pickling (spawn workers): re-attach by name, never unlink from a worker
    def __getstate__(self):
        return {"name": self._shm.name, "num_workers": self.num_workers, "batch_size": self.batch_size}

    def __setstate__(self, st):
        self.num_workers = st["num_workers"]
        self.batch_size = st["batch_size"]
        self._shm = shared_memory.SharedMemory(name=st["name"])
        try:  # the creating process owns the segment's lifetime
            from multiprocessing import resource_tracker

            resource_tracker.unregister(self._shm._name, "shared_memory")  # type: ignore[attr-defined]
        except Exception:  # noqa: BLE001
            pass
        self._owner = False
        self._arr = np.ndarray((_HDR + _W * self.num_workers,), dtype=np.int64, buffer=self._shm.buf)

    def _i(self, w: int, which: int) -> int:
        return _HDR + _W * w + which

    def request(self, worker: int, batches: int) -> None:
        self._arr[self._i(worker, _REQ)] = (self.epoch() << _EPOCH_SHIFT) | batches

    def requested(self, worker: int, epoch: int | None = None) -> int:
        """Batches of ``epoch`` (default: the current one) requested from ``worker``; 0 while the
        slot still holds an older iteration's request."""
        v = int(self._arr[self._i(worker, _REQ)])
        return v & _COUNT_MASK if (v >> _EPOCH_SHIFT) == (self.epoch() if epoch is None else epoch) else 0

    def ack(self, worker: int, batches: int, epoch: int | None = None) -> None:
        self._arr[self._i(worker, _ACK)] = ((self.epoch() if epoch is None else epoch) << _EPOCH_SHIFT) | batches

    def acked(self, worker: int, epoch: int | None = None) -> int:
        v = int(self._arr[self._i(worker, _ACK)])
        return v & _COUNT_MASK if (v >> _EPOCH_SHIFT) == (self.epoch() if epoch is None else epoch) else 0

    def register(self, worker: int, pid: int) -> None:
        """A worker announces its process (liveness is read from here, not from the DataLoader)."""
        self._arr[self._i(worker, _PID)] = pid

    def alive(self, worker: int) -> bool:
        """The worker registered and its process still runs (a zombie -- exited, not yet reaped by
        the DataLoader -- counts as dead)."""
        pid = int(self._arr[self._i(worker, _PID)])
        if pid <= 0:
            return False
        try:
            with open(f"/proc/{pid}/stat") as f:
                state = f.read().rsplit(")", 1)[1].split()[0]
        except (OSError, IndexError):
            return False
        return state not in ("Z", "X")

    def close_requests(self) -> None:
        """No more requests will come (end of iteration or the user broke out of the loop)."""
        self._arr[_CLOSING] = 1

    def closing(self) -> bool:
        return bool(self._arr[_CLOSING])

    def wait_acks(self, timeout: float = 5.0, alive=None) -> bool:
        """Waits until every worker acknowledged its latest request; a dead worker (``alive(w)``,
        by default the channel's own pid registry) is not waited for."""
        if alive is None:
            alive = self.alive
        deadline = time.monotonic() + timeout
        while True:
            pending = [w for w in range(self.num_workers) if self.acked(w) < self.requested(w)
                       and (alive is None or alive(w))]
            if not pending:
                return True
            if time.monotonic() >= deadline:
                return False
            time.sleep(0.001)

    def close(self) -> None:
        try:
            self._arr = None
            self._shm.close()
            if self._owner:
                self._shm.unlink()
        except Exception:  # noqa: BLE001
            pass


class WatermarkTable:
    """Main -> worker commit requests carrying exact offsets (DeviceLoader ``commit_sink='worker'``).

    The device loader knows exactly which records the user finished (slot watermarks), but only
    the consumer that read a partition may commit it as a group member (Kafka rejects a commit
    from a non-member once the group has members; a kafka-python consumer lives in its worker).
    So the main process publishes, per worker, the finished offset of every partition that
    worker delivered, and the worker's consumer commits them (kafka_dataset.py:124-143 messages,
    CommitFailedError logged and swallowed as B14).

    Layout (int64): per worker [seq_req, seq_ack], then per worker a block
    [n, pidx_0, off_0, ..., pidx_{cap-1}, off_{cap-1}].  An entry's pidx is written once, before
    ``n`` covers it; offsets only grow and are single aligned 64-bit stores, so a worker reading
    while the main process writes sees each offset old or new, never torn.  ``seq_req`` is bumped
    after every publish; the worker acknowledges the sequence it committed.  The native step
    driver (csrc/hip/driver.cpp) writes the same layout through :attr:`address`.
    """

    def __init__(self, num_workers: int, capacity: int = 4096):
        if num_workers < 1 or capacity < 1:
            raise ValueError("watermark table needs num_workers >= 1 and capacity >= 1")
        self.num_workers = num_workers
        self.capacity = capacity
        self._block = 1 + 2 * capacity
        n = 2 * num_workers + num_workers * self._block
        self._shm = shared_memory.SharedMemory(create=True, size=8 * n)
        self._owner = True
        self._arr = np.ndarray((n,), dtype=np.int64, buffer=self._shm.buf)
        self._arr[:] = 0
        self._index = [dict() for _ in range(num_workers)]

    def __getstate__(self):
        return {"name": self._shm.name, "num_workers": self.num_workers, "capacity": self.capacity}

    def __setstate__(self, st):
        self.num_workers, self.capacity = st["num_workers"], st["capacity"]
        self._block = 1 + 2 * self.capacity
        self._shm = shared_memory.SharedMemory(name=st["name"])
        try:
            from multiprocessing import resource_tracker

            resource_tracker.unregister(self._shm._name, "shared_memory")  # type: ignore[attr-defined]
        except Exception:  # noqa: BLE001
            pass
        self._owner = False
        n = 2 * self.num_workers + self.num_workers * self._block
        self._arr = np.ndarray((n,), dtype=np.int64, buffer=self._shm.buf)
        self._index = [dict() for _ in range(self.num_workers)]

    @property
    def address(self) -> int:
        """Address of the table in this process (the native driver writes through it)."""
        return self._arr.ctypes.data

    def _base(self, w: int) -> int:
        return 2 * self.num_workers + w * self._block

    # ---- main process
    def publish(self, worker: int, offsets: dict) -> None:
        """Offsets (pidx -> next offset) the user finished on ``worker``'s partitions."""
        b = self._base(worker)
        idx = self._index[worker]
        for pidx, off in offsets.items():
            k = idx.get(pidx)
            if k is None:
                k = int(self._arr[b])
                if k >= self.capacity:
                    raise RuntimeError("watermark table full: more partitions per worker than its capacity")
                self._arr[b + 1 + 2 * k] = pidx
                self._arr[b + 2 + 2 * k] = off
                self._arr[b] = k + 1
                idx[pidx] = k
            elif off > self._arr[b + 2 + 2 * k]:
                self._arr[b + 2 + 2 * k] = off
        self._arr[2 * worker] += 1

    def requested(self, worker: int) -> int:
        return int(self._arr[2 * worker])

    def acked(self, worker: int) -> int:
        return int(self._arr[2 * worker + 1])

    def wait_acks(self, timeout: float = 5.0, alive=None) -> bool:
        deadline = time.monotonic() + timeout
        while True:
            pending = [w for w in range(self.num_workers) if self.acked(w) < self.requested(w)
                       and (alive is None or alive(w))]
            if not pending:
                return True
            if time.monotonic() >= deadline:
                return False
            time.sleep(0.001)

    # ---- worker
    def entries(self, worker: int) -> list:
        b = self._base(worker)
        n = int(self._arr[b])
        return [(int(self._arr[b + 1 + 2 * k]), int(self._arr[b + 2 + 2 * k])) for k in range(n)]

    def ack(self, worker: int, seq: int) -> None:
        self._arr[2 * worker + 1] = seq

    def close(self) -> None:
        try:
            self._arr = None
            self._shm.close()
            if self._owner:
                self._shm.unlink()
        except Exception:  # noqa: BLE001
            pass
