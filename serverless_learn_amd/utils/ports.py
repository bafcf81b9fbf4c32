"""Ports for servers that are started later by another process.

Binding port 0 and closing the socket returns an ephemeral port, and the kernel hands out the
same range to every outgoing connection.  When the port is bound again seconds later, some
other process's connection may already hold it: gloo / c10d links between ranks, or gRPC
clients. The GPU elastic test lost a worker this way ("Address already in use"). So these
ports come from below the kernel's ephemeral range, which outgoing connections never get, and
each one is checked by a test bind.
"""
from __future__ import annotations

import random
import socket

_taken: set[int] = set()


def _ephemeral_low() -> int:
    try:
        with open("/proc/sys/net/ipv4/ip_local_port_range") as f:
            return int(f.read().split()[0])
    except (OSError, ValueError, IndexError):
        return 32768


def reserve_port(host: str = "127.0.0.1") -> int:
    """A port below the ephemeral range that binds now and was not returned before by this
    process (10000 <= port < the ephemeral range's start)."""
    hi = max(10001, _ephemeral_low())
    rng = random.Random()
    for _ in range(512):
        port = rng.randrange(10000, hi)
        if port in _taken:
            continue
        s = socket.socket()
        try:
            s.bind((host, port))
        except OSError:
            continue
        finally:
            s.close()
        _taken.add(port)
        return port
    s = socket.socket()  # fall back to an ephemeral port
    s.bind((host, 0))
    port = s.getsockname()[1]
    s.close()
    return port
