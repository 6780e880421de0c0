"""A rendezvous store for the multi-process tests, with no port race.

A port picked by binding a socket and closing it can be taken again before the
store binds it (EADDRINUSE, seen once on a GPU box). Instead the test process
itself hosts the TCPStore on port 0: the kernel assigns a free port and the
store keeps it bound for the whole test; the spawned ranks connect to it
(worker_store). torchrun-launched tests use `--standalone`, whose agent store
is bound the same way and handed to the workers (TORCHELASTIC_USE_AGENT_STORE).
"""
import torch.distributed as dist


def host_store(world: int):
    """(store, port): a master TCPStore on 127.0.0.1, bound by the caller."""
    store = dist.TCPStore("127.0.0.1", 0, world, is_master=True, wait_for_workers=False)
    return store, store.port


def init_worker(rank: int, world: int, port: int, backend: str = "gloo") -> None:
    """init_process_group of one spawned rank against the parent's store."""
    store = dist.TCPStore("127.0.0.1", port, world, is_master=False)
    dist.init_process_group(backend, store=store, rank=rank, world_size=world)
