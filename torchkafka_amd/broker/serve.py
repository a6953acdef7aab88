"""Serve a synthetic broker over the Kafka protocol from the command line."""
import time


def main(argv=None) -> int:
    """``python -m torchkafka_amd.broker.serve shm://name [--port 9092] [--python]``: serve an
    existing synthetic broker over the Kafka protocol until interrupted (test pipelines written for
    a Kafka cluster against synthetic topics)."""
    import argparse

    from .synthetic import open_broker
    from .wire_server import KafkaWireServer, NativeWireServer

    ap = argparse.ArgumentParser(description=main.__doc__)
    ap.add_argument("url", help="synthetic broker URL (shm://name or file:///path)")
    ap.add_argument("--host", default="127.0.0.1")
    ap.add_argument("--port", type=int, default=9092)
    ap.add_argument("--python", action="store_true", help="the Python server (fault injection) instead of C++")
    a = ap.parse_args(argv)
    cls = KafkaWireServer if a.python else NativeWireServer
    srv = cls(open_broker(a.url), host=a.host, port=a.port).start()
    print(f"serving {a.url} as a Kafka cluster on {srv.address}", flush=True)
    try:
        while True:
            time.sleep(3600)
    except KeyboardInterrupt:
        pass
    finally:
        srv.close()
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
