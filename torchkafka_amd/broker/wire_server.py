"""The synthetic broker served over the Kafka wire protocol.

A small Kafka-protocol front end for :class:`SyntheticBroker`: it answers the requests a
consumer makes (ApiVersions, Metadata, ListOffsets, Fetch, FindCoordinator, OffsetCommit,
OffsetFetch -- the non-flexible versions every Kafka client speaks) from the broker's
RecordBatch v2 logs and its committed-offset table.  It is what the native replicator
(:class:`~torchkafka_amd.broker.KafkaBridge`, ``csrc/core/replicator.cpp``) is tested
against here, where no Kafka cluster exists, and it lets any Kafka client (kafka-python,
where installed) read a synthetic topic over TCP.

Fault injection mirrors what a real cluster does to a consumer: NOT_LEADER /
OFFSET_OUT_OF_RANGE / arbitrary error codes on fetches, failed commits, record sets cut
inside a batch (a broker's ``partition_max_bytes`` cut), control batches (transaction
markers) between data batches.

Reference: the reference consumes through kafka-python's KafkaConsumer
(``/root/reference/src/kafka_dataset.py:21-22, 206``); this server plays the cluster.
"""
from __future__ import annotations

import base64
import hashlib
import hmac
import os
import socket
import socketserver
import struct
import threading
import time
import uuid

from .synthetic import SyntheticBroker

API_FETCH, API_LIST_OFFSETS, API_METADATA = 1, 2, 3
API_OFFSET_COMMIT, API_OFFSET_FETCH, API_FIND_COORDINATOR, API_API_VERSIONS = 8, 9, 10, 18
API_JOIN_GROUP, API_HEARTBEAT, API_LEAVE_GROUP, API_SYNC_GROUP = 11, 12, 13, 14
API_SASL_HANDSHAKE, API_SASL_AUTHENTICATE = 17, 36

# Version profiles: api key -> (min, max) served.  Requests outside a range close the connection,
# as a Kafka broker does; ApiVersions above its range answers UNSUPPORTED_VERSION in the v0 format.
#   legacy  -- a pre-2.x broker: exactly the versions the native client used before it negotiated;
#   kafka4  -- Kafka 4.x after KIP-896 dropped the pre-2.1 request versions (modelled strictly: the
#              minimums below are at or above the real broker's), up to what this server implements;
#   ancient -- a broker that predates ApiVersions (0.9): the legacy set, and ApiVersions closes the
#              connection (clients must fall back to fixed versions).
PROFILES = {
    "legacy": {API_FETCH: (4, 4), API_LIST_OFFSETS: (0, 1), API_METADATA: (0, 1), API_OFFSET_COMMIT: (2, 2),
               API_OFFSET_FETCH: (1, 1), API_FIND_COORDINATOR: (0, 0), API_API_VERSIONS: (0, 0),
               API_JOIN_GROUP: (0, 0), API_HEARTBEAT: (0, 0), API_LEAVE_GROUP: (0, 0), API_SYNC_GROUP: (0, 0),
               API_SASL_HANDSHAKE: (0, 1), API_SASL_AUTHENTICATE: (0, 0)},
    "kafka4": {API_FETCH: (4, 11), API_LIST_OFFSETS: (1, 5), API_METADATA: (4, 8), API_OFFSET_COMMIT: (2, 7),
               API_OFFSET_FETCH: (1, 5), API_FIND_COORDINATOR: (0, 2), API_API_VERSIONS: (0, 2),
               API_JOIN_GROUP: (2, 5), API_HEARTBEAT: (0, 3), API_LEAVE_GROUP: (0, 2), API_SYNC_GROUP: (0, 3),
               API_SASL_HANDSHAKE: (1, 1), API_SASL_AUTHENTICATE: (0, 1)},
}
PROFILES["ancient"] = {k: v for k, v in PROFILES["legacy"].items() if k != API_API_VERSIONS}
SUPPORTED = PROFILES["legacy"]  # the default profile

NONE, OFFSET_OUT_OF_RANGE, UNKNOWN_TOPIC, NOT_LEADER, UNSUPPORTED_VERSION = 0, 1, 3, 6, 35
ILLEGAL_GENERATION, UNSUPPORTED_SASL_MECHANISM, SASL_AUTHENTICATION_FAILED = 22, 33, 58
UNKNOWN_MEMBER_ID, REBALANCE_IN_PROGRESS, MEMBER_ID_REQUIRED = 25, 27, 79
SASL_MECHANISMS = ("PLAIN", "SCRAM-SHA-256", "SCRAM-SHA-512", "OAUTHBEARER")


class _R:
    """Big-endian reader over one request body."""

    def __init__(self, b: bytes):
        self.b, self.o = b, 0

    def _u(self, fmt: str, n: int):
        v = struct.unpack_from(fmt, self.b, self.o)[0]
        self.o += n
        return v

    def i8(self):
        return self._u(">b", 1)

    def i16(self):
        return self._u(">h", 2)

    def i32(self):
        return self._u(">i", 4)

    def i64(self):
        return self._u(">q", 8)

    def str(self):
        n = self.i16()
        if n < 0:
            return None
        s = self.b[self.o:self.o + n].decode()
        self.o += n
        return s


class _W:
    def __init__(self):
        self.parts: list[bytes] = []

    def i8(self, v):
        self.parts.append(struct.pack(">b", v))

    def i16(self, v):
        self.parts.append(struct.pack(">h", v))

    def i32(self, v):
        self.parts.append(struct.pack(">i", v))

    def i64(self, v):
        self.parts.append(struct.pack(">q", v))

    def str(self, s):
        if s is None:
            self.i16(-1)
        else:
            b = s.encode()
            self.i16(len(b))
            self.parts.append(b)

    def bytes(self, b):
        if b is None:
            self.i32(-1)
        else:
            self.i32(len(b))
            self.parts.append(b)

    def data(self) -> list:
        """The response as a buffer list: record sets stay views of the mapped logs (no copy)."""
        return self.parts


def control_batch(base_offset: int, timestamp_ms: int = 0, commit: bool = True) -> bytes:
    """A transaction-marker RecordBatch (control bit set), as a transactional producer leaves in a log."""
    from ..ops.native import core

    key = struct.pack(">hh", 0, 1 if commit else 0)  # version, type (COMMIT / ABORT)
    val = struct.pack(">hi", 0, 0)
    body = bytearray()
    rec = bytearray()
    rec += b"\x00"                     # attributes
    rec += _varint(0)                  # timestamp delta
    rec += _varint(0)                  # offset delta
    rec += _varint(len(key)) + key
    rec += _varint(len(val)) + val
    rec += _varint(0)                  # headers
    body += _varint(len(rec)) + rec
    attrs = 0x20 | 0x10                # control + transactional
    after_crc = struct.pack(">hiqqqhii", attrs, 0, timestamp_ms, timestamp_ms, 7, 0, -1, 1) + bytes(body)
    crc = core().crc32c(after_crc)
    blen = 4 + 1 + 4 + len(after_crc)
    return struct.pack(">qiibI", base_offset, blen, 0, 2, crc) + after_crc


def _varint(v: int) -> bytes:
    z = (v << 1) ^ (v >> 63)
    out = bytearray()
    while z >= 0x80:
        out.append((z & 0x7F) | 0x80)
        z >>= 7
    out.append(z)
    return bytes(out)


class _Group:
    """A consumer group's membership as the coordinator sees it."""

    def __init__(self):
        self.state = "empty"   # empty | joining | syncing | stable
        self.generation = 0
        self.members: dict[str, bytes] = {}   # member id -> subscription metadata (this generation)
        self.joining: dict[str, dict] = {}    # the round in progress: member -> {assignor: metadata}
        self.leader = ""
        self.protocol = ""
        self.assignments: dict[str, bytes] = {}
        self.pending: set[str] = set()       # ids handed out with MEMBER_ID_REQUIRED, not joined yet
        self.min_end = self.deadline = 0.0


class KafkaWireServer:
    """Serves a :class:`SyntheticBroker` over the Kafka protocol on ``host:port`` (0: a free port)."""

    def __init__(self, broker: SyntheticBroker, host: str = "127.0.0.1", port: int = 0, node_id: int = 0,
                 cluster: list[tuple[int, str, int]] | None = None, ssl_context=None,
                 sasl_users: dict[str, str] | None = None, profile: "str | dict" = "legacy",
                 sasl_oauth_tokens: dict[str, str] | None = None):
        """``cluster``: every node of a multi-node test cluster as (node_id, host, port), this one
        included; partition p is led by ``cluster[p % len(cluster)]`` and fetches sent to another
        node answer NOT_LEADER.  None: a single-node cluster (this server leads everything).
        ``ssl_context``: a server-side ``ssl.SSLContext`` (listeners SSL / SASL_SSL).  ``sasl_users``:
        {user: password} accepted by SASL/PLAIN; every request but ApiVersions and the SASL exchange
        closes the connection until it authenticated.  ``sasl_oauth_tokens``: {bearer token: principal}
        accepted by SASL/OAUTHBEARER (RFC 7628; every exchange is kept in :attr:`oauth_log` as
        (token, extensions dict, accepted)).  ``profile``: the request versions served
        (:data:`PROFILES`: "legacy", "kafka4", "ancient"; or an ``{api key: (min, max)}`` dict)."""
        if isinstance(profile, dict):
            self.profile, self.versions = "custom", dict(profile)
        elif profile in PROFILES:
            self.profile, self.versions = profile, PROFILES[profile]
        else:
            raise ValueError(f"profile {profile!r}: one of {sorted(PROFILES)} or an {{api: (min, max)}} dict")
        self.ssl_context = ssl_context
        self.sasl_users = sasl_users
        self.sasl_oauth_tokens = sasl_oauth_tokens
        self.oauth_log: list = []
        self.broker = broker
        self.node_id = node_id
        self.cluster = cluster
        self._lock = threading.Lock()
        self._fetch_faults: dict[tuple[str, int], list[int]] = {}
        self._commit_faults: list[int] = []
        self.partial_tail = False          # cut every record set inside its last batch
        self.stall_s = 0.0                 # fault injection: hold every Fetch this long (a hung broker)
        self.requests: dict[int, int] = {}  # api key -> count
        self.request_versions: dict[int, set] = {}  # api key -> versions seen (tests)
        self.commit_log: list = []          # (group, topic, partition, offset) of every accepted commit
        self._views: dict[int, memoryview] = {}
        self._conns: set = set()
        self._groups: dict[str, _Group] = {}
        self._gcond = threading.Condition()
        self.join_delay_s = 0.3            # group.initial.rebalance.delay.ms of a fresh group
        srv = self

        class Handler(socketserver.BaseRequestHandler):
            def handle(self):
                sock = self.request
                sock.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
                if srv.ssl_context is not None:
                    try:
                        sock = srv.ssl_context.wrap_socket(sock, server_side=True)
                    except (OSError, ValueError):
                        return  # failed TLS handshake (untrusted client / plaintext probe)
                with srv._lock:
                    srv._conns.add(sock)
                state = {"authed": srv.sasl_users is None and srv.sasl_oauth_tokens is None}
                try:
                    while True:
                        head = _recv_exact(sock, 4)
                        if head is None:
                            return
                        (n,) = struct.unpack(">i", head)
                        req = _recv_exact(sock, n)
                        if req is None:
                            return
                        parts = srv._dispatch(req, state)
                        if parts is None:
                            return
                        n = sum(len(b) for b in parts)
                        if srv.ssl_context is not None:
                            sock.sendall(struct.pack(">i", n) + b"".join(bytes(b) for b in parts))
                        else:
                            _sendall_vec(sock, [struct.pack(">i", n)] + parts)
                except (ConnectionError, OSError):
                    return
                finally:
                    with srv._lock:
                        srv._conns.discard(sock)

        class Server(socketserver.ThreadingTCPServer):
            daemon_threads = True
            allow_reuse_address = True

        self._srv = Server((host, port), Handler)
        self.host, self.port = self._srv.server_address[:2]
        if self.cluster is None:
            self.cluster = [(node_id, self.host, self.port)]
        self._thread = threading.Thread(target=self._srv.serve_forever, daemon=True, name="kafka-wire-server")

    # ------------------------------------------------------------ lifecycle
    @property
    def address(self) -> str:
        return f"{self.host}:{self.port}"

    def start(self) -> "KafkaWireServer":
        self._thread.start()
        return self

    def close(self) -> None:
        """Stops listening and drops every client connection (a broker going down)."""
        self._srv.shutdown()
        self._srv.server_close()
        with self._lock:
            conns = list(self._conns)
        for c in conns:
            try:
                c.shutdown(socket.SHUT_RDWR)
                c.close()
            except OSError:
                pass

    def __enter__(self):
        return self.start()

    def __exit__(self, *exc):
        self.close()

    # ------------------------------------------------------------ fault injection
    def inject_fetch_errors(self, topic: str, partition: int, code: int = NOT_LEADER, n: int = 1) -> None:
        """The next ``n`` fetches of a partition answer ``code`` (NOT_LEADER by default)."""
        with self._lock:
            self._fetch_faults.setdefault((topic, partition), []).extend([code] * n)

    def inject_commit_errors(self, code: int = ILLEGAL_GENERATION, n: int = 1) -> None:
        with self._lock:
            self._commit_faults.extend([code] * n)

    # ------------------------------------------------------------ protocol
    def _log(self, pidx: int) -> memoryview:
        v = self._views.get(pidx)
        if v is None:
            v = self._views[pidx] = self.broker.native.log_view(pidx)
        return v

    def _dispatch(self, req: bytes, state: dict | None = None) -> list | None:
        r = _R(req)
        key, ver, corr = r.i16(), r.i16(), r.i32()
        r.str()  # client id
        with self._lock:
            self.requests[key] = self.requests.get(key, 0) + 1
            self.request_versions.setdefault(key, set()).add(ver)
        w = _W()
        w.i32(corr)
        state = {"authed": True} if state is None else state
        lo_hi = self.versions.get(key)
        if key == API_API_VERSIONS:
            if lo_hi is None:
                return None  # predates ApiVersions: the connection just closes
            err = NONE if lo_hi[0] <= ver <= lo_hi[1] else UNSUPPORTED_VERSION
            w.i16(err)
            w.i32(len(self.versions))
            for k, (lo, hi) in sorted(self.versions.items()):
                w.i16(k)
                w.i16(lo)
                w.i16(hi)
            if err == NONE and ver >= 1:
                w.i32(0)  # throttle
            return w.data()
        if lo_hi is None or not lo_hi[0] <= ver <= lo_hi[1]:
            return None  # a real broker closes the connection on an unsupported version
        if key == API_SASL_HANDSHAKE:
            mech = r.str()
            ok = (self.sasl_oauth_tokens is not None if mech == "OAUTHBEARER"
                  else self.sasl_users is not None and mech in SASL_MECHANISMS)
            w.i16(NONE if ok else UNSUPPORTED_SASL_MECHANISM)
            w.i32(len(SASL_MECHANISMS))
            for m in SASL_MECHANISMS:
                w.str(m)
            state["mech"] = mech if ok else None
            return w.data()
        if key == API_SASL_AUTHENTICATE:
            n = r.i32()
            token = bytes(r.b[r.o:r.o + n])
            reply, ok = self._sasl_step(state, token)
            w.i16(NONE if ok else SASL_AUTHENTICATION_FAILED)
            w.str(None if ok else "Authentication failed: invalid username or password")
            w.bytes(reply if ok else b"")
            if ver >= 1:
                w.i64(0)  # session lifetime: no re-authentication required
            return w.data()
        if not state["authed"]:
            return None  # a SASL listener drops unauthenticated requests
        getattr(self, f"_api_{key}")(r, ver, w)
        return w.data()

    def _sasl_step(self, state: dict, token: bytes) -> tuple[bytes, bool]:
        """One SaslAuthenticate round of the mechanism the handshake chose: PLAIN in one round,
        SCRAM-SHA-256/512 (RFC 5802) in two -- client-first, then client-final with the proof."""
        mech = state.get("mech")
        if mech == "OAUTHBEARER":
            return self._oauth_step(state, token)
        if mech == "PLAIN":
            parts = token.split(b"\0")
            user, pw = (parts[1].decode(), parts[2].decode()) if len(parts) == 3 else ("", None)
            state["authed"] = ok = self.sasl_users.get(user) == pw
            return b"", ok
        if mech not in ("SCRAM-SHA-256", "SCRAM-SHA-512"):
            return b"", False
        h = hashlib.sha512 if mech.endswith("512") else hashlib.sha256
        msg = token.decode()
        attrs = lambda m: dict(kv.split("=", 1) for kv in m.split(",") if "=" in kv)  # noqa: E731
        if "scram" not in state:  # client-first: "n,,n=user,r=cnonce"
            bare = msg[3:] if msg.startswith("n,,") else ""
            a = attrs(bare)
            user = a.get("n", "").replace("=2C", ",").replace("=3D", "=")
            if user not in self.sasl_users or "r" not in a:
                return b"", False
            salt, iters = os.urandom(16), 4096
            snonce, s64 = base64.b64encode(os.urandom(18)).decode(), base64.b64encode(salt).decode()
            first = f"r={a['r']}{snonce},s={s64},i={iters}"
            salted = hashlib.pbkdf2_hmac(h().name, self.sasl_users[user].encode(), salt, iters)
            state["scram"] = (bare, first, salted)
            return first.encode(), True
        bare, first, salted = state.pop("scram")
        a = attrs(msg)
        without_proof = msg[:msg.rfind(",p=")]
        if a.get("r") != attrs(first)["r"]:
            return b"", False
        auth = f"{bare},{first},{without_proof}".encode()
        client_key = hmac.new(salted, b"Client Key", h).digest()
        signature = hmac.new(h(client_key).digest(), auth, h).digest()
        proof = base64.b64decode(a.get("p", ""))
        if len(proof) != len(signature) or bytes(x ^ y for x, y in zip(proof, signature)) != client_key:
            return b"", False
        state["authed"] = True
        server_sig = hmac.new(hmac.new(salted, b"Server Key", h).digest(), auth, h).digest()
        return ("v=" + base64.b64encode(server_sig).decode()).encode(), True

    def _oauth_step(self, state: dict, token: bytes) -> tuple[bytes, bool]:
        """RFC 7628: the client's first message is "n,[a=authzid],", then 0x01-separated key=value
        pairs -- auth=Bearer <token> and the extensions -- and 0x01 0x01.  A bad token gets an error
        challenge (JSON, error code NONE); the client's lone 0x01 that follows fails the exchange."""
        if state.pop("oauth_failed", False):
            return b"", False  # the client acknowledged the error challenge
        try:
            gs2, rest = token.decode().split(",", 2)[:2], token.decode().split(",", 2)[2]
        except (UnicodeDecodeError, IndexError):
            return b"", False
        if gs2[0] not in ("n", "y") or not rest.startswith("\x01") or not rest.endswith("\x01\x01"):
            return b"", False
        pairs = dict(kv.split("=", 1) for kv in rest.strip("\x01").split("\x01") if "=" in kv)
        auth = pairs.pop("auth", "")
        bearer = auth[7:] if auth.startswith("Bearer ") else None
        ok = bearer is not None and bearer in self.sasl_oauth_tokens
        self.oauth_log.append((bearer, pairs, ok))
        if ok:
            state["authed"] = True
            return b"", True
        state["oauth_failed"] = True
        return b'{"status":"invalid_token"}', True

    def _topic_names(self, r: _R, ver: int):
        n = r.i32()
        if n < 0 or (n == 0 and ver == 0):
            return self.broker.topics()
        return [r.str() for _ in range(n)]

    def _api_3(self, r: _R, ver: int, w: _W) -> None:  # Metadata v0-v8
        names = self._topic_names(r, ver)
        if ver >= 4:
            r.i8()  # allow_auto_topic_creation (topics are never created here)
        if ver >= 8:
            r.i8()
            r.i8()  # include cluster / topic authorized operations
        if ver >= 3:
            w.i32(0)  # throttle
        w.i32(len(self.cluster))
        for nid, host, port in self.cluster:
            w.i32(nid)
            w.str(host)
            w.i32(port)
            if ver >= 1:
                w.str(None)  # rack
        if ver >= 2:
            w.str("torchkafka-synthetic")  # cluster id
        if ver >= 1:
            w.i32(self.cluster[0][0])  # controller
        w.i32(len(names))
        for name in names:
            if not self.broker.has_topic(name):
                w.i16(UNKNOWN_TOPIC)
                w.str(name)
                if ver >= 1:
                    w.i8(0)
                w.i32(0)
                if ver >= 8:
                    w.i32(-2147483648)  # authorized operations: not requested
                continue
            n = self.broker.topic(name)[1]
            w.i16(NONE)
            w.str(name)
            if ver >= 1:
                w.i8(0)
            w.i32(n)
            for p in range(n):
                leader = self.leader(p)
                w.i16(NONE)
                w.i32(p)
                w.i32(leader)
                if ver >= 7:
                    w.i32(0)  # leader epoch
                w.i32(1)
                w.i32(leader)
                w.i32(1)
                w.i32(leader)
                if ver >= 5:
                    w.i32(0)  # offline replicas
            if ver >= 8:
                w.i32(-2147483648)
        if ver >= 8:
            w.i32(-2147483648)

    def leader(self, partition: int) -> int:
        return self.cluster[partition % len(self.cluster)][0]

    def _api_2(self, r: _R, ver: int, w: _W) -> None:  # ListOffsets v0-v5
        r.i32()  # replica
        if ver >= 2:
            r.i8()  # isolation level
            w.i32(0)  # throttle
        nt = r.i32()
        w.i32(nt)
        for _ in range(nt):
            name = r.str()
            np_ = r.i32()
            w.str(name)
            w.i32(np_)
            for _ in range(np_):
                p = r.i32()
                if ver >= 4:
                    r.i32()  # current leader epoch
                ts = r.i64()
                if ver == 0:
                    r.i32()  # max offsets
                err, off = NONE, -1
                try:
                    pidx = self.broker.pidx(name, p)
                    nat = self.broker.native
                    if ts == -1:
                        off = nat.high_watermark(pidx)
                    elif ts == -2:
                        off = nat.log_start_offset(pidx)
                    else:
                        off = nat.offset_for_time(pidx, ts)[0]
                except Exception:  # noqa: BLE001 -- any lookup failure is an unknown partition
                    err = UNKNOWN_TOPIC
                w.i32(p)
                w.i16(err)
                if ver == 0:
                    w.i32(1 if off >= 0 else 0)
                    if off >= 0:
                        w.i64(off)
                else:
                    w.i64(-1)
                    w.i64(off)
                    if ver >= 4:
                        w.i32(0)  # leader epoch

    def _api_1(self, r: _R, ver: int, w: _W) -> None:  # Fetch v4-v11 (sessionless)
        if self.stall_s:
            time.sleep(self.stall_s)
        r.i32()  # replica
        max_wait, min_bytes, max_bytes = r.i32(), r.i32(), r.i32()
        r.i8()  # isolation level
        if ver >= 7:
            r.i32()
            r.i32()  # session id / epoch: every fetch is answered in full (no incremental sessions)
        reqs = []
        for _ in range(r.i32()):
            name = r.str()
            parts = []
            for _ in range(r.i32()):
                p = r.i32()
                if ver >= 9:
                    r.i32()  # current leader epoch
                off = r.i64()
                if ver >= 5:
                    r.i64()  # log start offset (a follower's)
                parts.append((p, off, r.i32()))
            reqs.append((name, parts))
        faults = {}
        with self._lock:  # one injected error per partition per request
            for name, parts in reqs:
                for p, _off, _pmax in parts:
                    q = self._fetch_faults.get((name, p))
                    if q:
                        faults[(name, p)] = q.pop(0)
        deadline = time.monotonic() + max_wait / 1000.0
        while True:
            out, total = self._fetch_once(reqs, max_bytes, faults)
            if total >= max(1, min_bytes) or time.monotonic() >= deadline:
                break
            time.sleep(0.002)
        w.i32(0)  # throttle
        if ver >= 7:
            w.i16(NONE)
            w.i32(0)  # session id: none
        w.i32(len(out))
        nat = self.broker.native
        for name, parts in out:
            w.str(name)
            w.i32(len(parts))
            for p, err, hw, data in parts:
                w.i32(p)
                w.i16(err)
                w.i64(hw)
                w.i64(hw)   # last stable offset
                if ver >= 5:
                    try:
                        w.i64(nat.log_start_offset(self.broker.pidx(name, p)))
                    except Exception:  # noqa: BLE001
                        w.i64(-1)
                w.i32(-1)   # aborted transactions: null
                if ver >= 11:
                    w.i32(-1)  # preferred read replica: none
                w.bytes(data)

    def _fetch_once(self, reqs, max_bytes: int, faults: dict):
        out, total = [], 0
        nat = self.broker.native
        for name, parts in reqs:
            po = []
            for p, off, pmax in parts:
                fault = faults.get((name, p))
                if fault is None and self.leader(p) != self.node_id:
                    fault = NOT_LEADER
                if fault is not None:
                    po.append((p, fault, -1, None))
                    continue
                try:
                    pidx = self.broker.pidx(name, p)
                except Exception:  # noqa: BLE001
                    po.append((p, UNKNOWN_TOPIC, -1, None))
                    continue
                try:
                    budget = max(0, min(pmax, max_bytes - total))
                    pos, nbytes, hw, _start = nat.batch_range(pidx, off, max(budget, 1))
                except Exception:  # noqa: BLE001 -- OffsetOutOfRange
                    po.append((p, OFFSET_OUT_OF_RANGE, nat.high_watermark(pidx), None))
                    continue
                data = self._log(pidx)[pos:pos + nbytes]  # a view: the record set is sent from the log
                if nbytes and self.partial_tail:
                    # add the front half of the next batch, as a broker cutting at partition_max_bytes does
                    data = bytes(data)
                    try:
                        more, _, _ = nat.read_batches(pidx, _next_offset(data), 1)
                        data = data + more[:max(12, len(more) // 2)]
                    except Exception:  # noqa: BLE001 -- nothing after it
                        pass
                total += len(data)
                po.append((p, NONE, hw, data))
            out.append((name, po))
        return out, total

    def _api_10(self, r: _R, ver: int, w: _W) -> None:  # FindCoordinator v0-v2
        r.str()
        if ver >= 1:
            r.i8()  # key type
            w.i32(0)  # throttle
        w.i16(NONE)
        if ver >= 1:
            w.str(None)  # error message
        w.i32(self.node_id)
        w.str(self.host)
        w.i32(self.port)

    # ------------------------------------------------------------ group membership (coordinator)
    # JoinGroup v0-v5 / SyncGroup v0-v3 / Heartbeat v0-v3 / LeaveGroup v0-v2 with Kafka's state
    # machine, reduced to what a test needs: a join round ends once every member of the last
    # generation rejoined (a fresh group waits ``join_delay_s`` for more joiners) or after the
    # rebalance timeout (v1+; the session timeout at v0), which drops the absentees; the first
    # joiner leads and sends the assignment through SyncGroup.  From JoinGroup v4 a member joining
    # without an id gets MEMBER_ID_REQUIRED and an id to join again with (KIP-394).
    def _group(self, name: str) -> "_Group":
        g = self._groups.get(name)
        if g is None:
            g = self._groups[name] = _Group()
        return g

    def _begin_round(self, g: "_Group", timeout_s: float) -> None:
        if g.state != "joining":
            g.state, g.joining = "joining", {}
            now = time.monotonic()
            g.min_end = now + (self.join_delay_s if not g.members else 0.0)
            g.deadline = now + max(timeout_s, self.join_delay_s)

    def _api_11(self, r: _R, ver: int, w: _W) -> None:  # JoinGroup v0-v5 (blocks until the round ends)
        group, session_ms = r.str(), r.i32()
        rebalance_ms = r.i32() if ver >= 1 else session_ms
        member = r.str() or ""
        if ver >= 5:
            r.str()  # group instance id (static membership is not modelled)
        r.str()  # protocol type
        protos: list[tuple[str, bytes]] = []
        for _ in range(r.i32()):
            name = r.str()
            n = r.i32()
            protos.append((name, bytes(r.b[r.o:r.o + n])))
            r.o += n
        with self._gcond:
            g = self._group(group)
            if not member and ver >= 4:
                member = f"member-{uuid.uuid4().hex[:12]}"
                g.pending.add(member)
                self._join_reply(w, ver, MEMBER_ID_REQUIRED, -1, "", "", member, {})
                return
            if member and member not in g.members and member not in g.joining and member not in g.pending:
                self._join_reply(w, ver, UNKNOWN_MEMBER_ID, -1, "", "", member, {})
                return
            g.pending.discard(member)
            member = member or f"member-{uuid.uuid4().hex[:12]}"
            self._begin_round(g, rebalance_ms / 1000.0)
            g.joining[member] = dict(protos)  # assignor name -> subscription metadata
            gen0 = g.generation
            self._gcond.notify_all()
            while g.generation == gen0:
                now = time.monotonic()
                done = set(g.members) <= set(g.joining) and now >= g.min_end
                if done or now >= g.deadline:
                    g.generation += 1
                    g.leader = next(iter(g.joining))
                    common = [n for n in g.joining[g.leader] if all(n in ps for ps in g.joining.values())]
                    g.protocol = common[0] if common else ""
                    g.members = {m: ps.get(g.protocol, b"") for m, ps in g.joining.items()}
                    g.state, g.assignments = "syncing", {}
                    self._gcond.notify_all()
                    break
                self._gcond.wait(0.01)
            if member not in g.members:  # joined after the round closed: rejoin
                self._join_reply(w, ver, REBALANCE_IN_PROGRESS, -1, "", "", member, {})
                return
            self._join_reply(w, ver, NONE, g.generation, g.protocol, g.leader, member,
                             g.members if member == g.leader else {})

    @staticmethod
    def _join_reply(w: _W, ver, err, gen, proto, leader, member, members) -> None:
        if ver >= 2:
            w.i32(0)  # throttle
        w.i16(err)
        w.i32(gen)
        w.str(proto)
        w.str(leader)
        w.str(member)
        w.i32(len(members))
        for m, meta in members.items():
            w.str(m)
            if ver >= 5:
                w.str(None)  # group instance id
            w.bytes(meta)

    def _member_error(self, g: "_Group | None", gen: int, member: str) -> int:
        if g is None or member not in g.members:
            return UNKNOWN_MEMBER_ID
        if gen != g.generation:
            return ILLEGAL_GENERATION
        return NONE

    def _api_14(self, r: _R, ver: int, w: _W) -> None:  # SyncGroup v0-v3
        group, gen, member = r.str(), r.i32(), r.str() or ""
        if ver >= 3:
            r.str()  # group instance id
        assign = {}
        for _ in range(r.i32()):
            m = r.str()
            n = r.i32()
            assign[m] = bytes(r.b[r.o:r.o + n])
            r.o += n
        with self._gcond:
            g = self._groups.get(group)
            err = self._member_error(g, gen, member)
            if err == NONE and member == g.leader:
                g.assignments, g.state = assign, "stable"
                self._gcond.notify_all()
            deadline = time.monotonic() + 30
            while err == NONE and g.state == "syncing" and g.generation == gen and time.monotonic() < deadline:
                self._gcond.wait(0.01)
            if err == NONE and (g.generation != gen or g.state != "stable"):
                err = REBALANCE_IN_PROGRESS
            if ver >= 1:
                w.i32(0)  # throttle
            w.i16(err)
            w.bytes(g.assignments.get(member, b"") if err == NONE else b"")

    def _api_12(self, r: _R, ver: int, w: _W) -> None:  # Heartbeat v0-v3
        group, gen, member = r.str(), r.i32(), r.str() or ""
        if ver >= 3:
            r.str()  # group instance id
        with self._gcond:
            g = self._groups.get(group)
            err = self._member_error(g, gen, member)
            if err == NONE and g.state == "joining":
                err = REBALANCE_IN_PROGRESS
            if ver >= 1:
                w.i32(0)  # throttle
            w.i16(err)

    def _api_13(self, r: _R, ver: int, w: _W) -> None:  # LeaveGroup v0-v2
        group, member = r.str(), r.str() or ""
        if ver >= 1:
            w.i32(0)  # throttle
        with self._gcond:
            g = self._groups.get(group)
            if g is None or member not in g.members:
                w.i16(UNKNOWN_MEMBER_ID)
                return
            del g.members[member]
            if g.members:
                self._begin_round(g, 10.0)  # the others learn it from their next heartbeat
            else:
                g.state = "empty"
            self._gcond.notify_all()
            w.i16(NONE)

    def group_members(self, group: str) -> dict[str, bytes]:
        """{member id: assignment} of a group's current generation (tests)."""
        with self._gcond:
            g = self._groups.get(group)
            return {} if g is None else {m: g.assignments.get(m, b"") for m in g.members}

    def committed(self, group: str, topic: str, partition: int) -> int:
        """The group's committed offset of a partition (-1: none) -- what the cluster holds (tests)."""
        nat = self.broker.native
        return nat.committed(nat.group_index(group, True), self.broker.pidx(topic, partition))[0]

    def _api_8(self, r: _R, ver: int, w: _W) -> None:  # OffsetCommit v2-v7
        group = r.str()
        gen = r.i32()
        member = r.str() or ""
        if ver >= 7:
            r.str()  # group instance id
        if ver <= 4:
            r.i64()   # retention
        with self._gcond:
            fenced = NONE if gen == -1 else self._member_error(self._groups.get(group), gen, member)
        nat = self.broker.native
        g = nat.group_index(group, True)
        if ver >= 3:
            w.i32(0)  # throttle
        nt = r.i32()
        w.i32(nt)
        for _ in range(nt):
            name = r.str()
            np_ = r.i32()
            w.str(name)
            w.i32(np_)
            for _ in range(np_):
                p, off = r.i32(), r.i64()
                if ver >= 6:
                    r.i32()  # committed leader epoch
                meta = r.str() or ""
                with self._lock:
                    err = self._commit_faults.pop(0) if self._commit_faults else fenced
                if err == NONE:
                    try:
                        nat.commit(g, -1, 0, 0, [(self.broker.pidx(name, p), int(off), meta)])
                        with self._lock:
                            self.commit_log.append((group, name, p, int(off)))
                    except Exception:  # noqa: BLE001 -- a group with live members refuses a simple commit
                        err = ILLEGAL_GENERATION
                w.i32(p)
                w.i16(err)

    def _api_9(self, r: _R, ver: int, w: _W) -> None:  # OffsetFetch v1-v5
        group = r.str()
        nat = self.broker.native
        g = nat.group_index(group, True)
        if ver >= 3:
            w.i32(0)  # throttle
        nt = r.i32()
        if nt < 0:  # v2+: every topic of the group
            reqs = [(t, list(range(self.broker.topic(t)[1]))) for t in self.broker.topics()]
        else:
            reqs = []
            for _ in range(nt):
                name = r.str()
                reqs.append((name, [r.i32() for _ in range(r.i32())]))
        w.i32(len(reqs))
        for name, parts in reqs:
            w.str(name)
            w.i32(len(parts))
            for p in parts:
                try:
                    off, meta = nat.committed(g, self.broker.pidx(name, p))
                    err = NONE
                except Exception:  # noqa: BLE001
                    off, meta, err = -1, "", UNKNOWN_TOPIC
                w.i32(p)
                w.i64(off)
                if ver >= 5:
                    w.i32(-1)  # committed leader epoch
                w.str(meta)
                w.i16(err)
        if ver >= 2:
            w.i16(NONE)


def _last_batch_start(data: bytes) -> int:
    o = 0
    while True:
        (blen,) = struct.unpack_from(">i", data, o + 8)
        if o + 12 + blen >= len(data):
            return o
        o += 12 + blen


def _next_offset(data: bytes) -> int:
    o = _last_batch_start(data)
    base = struct.unpack_from(">q", data, o)[0]
    (delta,) = struct.unpack_from(">i", data, o + 23)
    return base + delta + 1


def _sendall_vec(sock, bufs: list) -> None:
    """sendall over a buffer list (scatter-gather; partial sends resumed)."""
    views = [memoryview(b) for b in bufs if len(b)]
    while views:
        sent = sock.sendmsg(views[:512])
        while sent:
            if sent >= len(views[0]):
                sent -= len(views[0])
                views.pop(0)
            else:
                views[0] = views[0][sent:]
                sent = 0


def _recv_exact(sock, n: int) -> bytes | None:
    buf = bytearray()
    while len(buf) < n:
        chunk = sock.recv(n - len(buf))
        if not chunk:
            return None
        buf += chunk
    return bytes(buf)


class NativeWireServer:
    """The same protocol served by C++ threads (``csrc/core/wire_server.cpp``): record sets go out
    of the mapped logs by ``sendmsg`` without a copy, so a cluster of these feeds a replicator at
    memory / NIC speed (the Python server above is bound by its interpreter).  No fault injection.
    ``cluster``: every node as (node_id, host, port); partition p is led by node p % len(cluster)."""

    def __init__(self, broker: SyntheticBroker, host: str = "127.0.0.1", port: int = 0, node_id: int = 0,
                 cluster: list[tuple[int, str, int]] | None = None, profile: str = "legacy"):
        from ..ops.native import core

        self.broker = broker
        self.host = host
        self.profile = profile
        self._s = core().WireServer(broker.native, host, int(port), int(node_id), list(cluster or []), profile)
        self.port = self._s.port

    @property
    def address(self) -> str:
        return f"{self.host}:{self.port}"

    @property
    def requests(self) -> int:
        return int(self._s.requests)

    @property
    def bytes_sent(self) -> int:
        return int(self._s.bytes_sent)

    def start(self) -> "NativeWireServer":
        self._s.start()
        return self

    def close(self) -> None:
        self._s.stop()

    def __enter__(self):
        return self.start()

    def __exit__(self, *exc):
        self.close()

