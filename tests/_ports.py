"""A rendezvous port for the multi-process tests.

bind(0) hands out a port from the kernel's ephemeral range, the range every
outgoing connection (gloo opens several per rank pair) also draws its local
port from, so by the time torchrun's store binds it the port can be taken
(EADDRINUSE, seen once on a GPU box). Ports below the ephemeral range are
never handed out that way; one that binds now is free for the store.
"""
import random
import socket


def free_port(lo: int = 20000, hi: int = 32000) -> int:
    rnd = random.Random()
    for _ in range(200):
        p = rnd.randrange(lo, hi)
        s = socket.socket()
        try:
            s.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
            s.bind(("127.0.0.1", p))
            return p
        except OSError:
            continue
        finally:
            s.close()
    raise RuntimeError(f"no free port in [{lo}, {hi})")
