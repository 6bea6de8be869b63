"""Rendezvous port choice for locally launched ranks (tests, ``bench.py --gpus N``).

A port handed out by binding port 0 comes from the kernel's ephemeral range (32768-60999 by
default), the same range outgoing connections draw their source ports from: between our probe
and the TCPStore's bind another connection can take it (EADDRINUSE, seen on a shared GPU box).
Ports are therefore drawn at random below that range and checked by a bind."""
from __future__ import annotations

import random
import socket


def free_port(lo: int = 20000, hi: int = 32000) -> int:
    rnd = random.SystemRandom()
    for _ in range(64):
        p = rnd.randrange(lo, hi)
        with socket.socket() as s:
            try:
                s.bind(("127.0.0.1", p))
            except OSError:
                continue
            return p
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]
