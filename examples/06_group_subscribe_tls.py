#!/usr/bin/env python3
"""Two consumers sharing a Kafka consumer group over TLS + SASL/PLAIN (kafka-python's subscribe()).

Each `KafkaBridge(subscribe=True)` joins group "trainers" on the cluster: the group leader runs
Kafka's range assignor, so the two bridges mirror disjoint halves of the topic, and each commit
is stamped with its member's generation. The connection settings are kafka-python's
(`security_protocol`, `ssl_cafile`, `sasl_plain_username`, ...).

No cluster is reachable here, so this example starts one: a `KafkaWireServer` with a TLS listener
(a throwaway self-signed certificate made by the `openssl` CLI) and one SASL user.

    python examples/06_group_subscribe_tls.py
"""
import os
import ssl
import subprocess
import sys
import tempfile
import threading

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from torchkafka_amd import KafkaConsumer  # noqa: E402
from torchkafka_amd.broker import KafkaBridge, KafkaWireServer, SyntheticBroker  # noqa: E402
from torchkafka_amd.client.records import TopicPartition  # noqa: E402


def main() -> None:
    tmp = tempfile.mkdtemp()
    cert, key = os.path.join(tmp, "cert.pem"), os.path.join(tmp, "key.pem")
    subprocess.run(["openssl", "req", "-x509", "-newkey", "rsa:2048", "-nodes", "-keyout", key, "-out", cert,
                    "-days", "1", "-subj", "/CN=127.0.0.1", "-addext", "subjectAltName=IP:127.0.0.1"],
                   check=True, capture_output=True)
    ctx = ssl.SSLContext(ssl.PROTOCOL_TLS_SERVER)
    ctx.load_cert_chain(cert, key)

    cluster = SyntheticBroker.create(f"shm://example6-{os.getpid()}")
    cluster.create_topic("events", 6)
    cluster.fill("events", 1000, "fixed_f32", size=16)
    server = KafkaWireServer(cluster, ssl_context=ctx, sasl_users={"trainer": "s3cret"}).start()
    security = dict(security_protocol="SASL_SSL", ssl_cafile=cert, sasl_mechanism="PLAIN",
                    sasl_plain_username="trainer", sasl_plain_password="s3cret")
    bridges = [KafkaBridge(server.address, "events", group_id="trainers", subscribe=True, start=False, **security)
               for _ in range(2)]
    try:
        # both members join the same rebalance round (JoinGroup blocks until the round ends)
        ts = [threading.Thread(target=b.start) for b in bridges]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        for i, b in enumerate(bridges):
            b.wait_caught_up(10)
            c = KafkaConsumer(bootstrap_servers=b.url, group_id="trainers", consumer_timeout_ms=300,
                              enable_auto_commit=False)
            c.assign([TopicPartition("events", p) for p in b.assignment])
            c.seek_to_beginning()
            n = sum(1 for _ in c)
            c.commit()  # local commit; the bridge forwards it to the cluster with its generation
            c.close()
            print(f"member {i}: partitions {sorted(b.assignment)}, generation {b.generation}, {n} records")
        for b in bridges:
            b.close()  # final commit, then LeaveGroup
        print("cluster's committed offsets:", cluster.committed_offsets("trainers", "events"))
    finally:
        server.close()
        cluster.destroy()


if __name__ == "__main__":
    main()
