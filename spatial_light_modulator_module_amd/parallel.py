"""Batch sharding and the torch-free control plane of one-process-per-GPU runs.

Holograms are independent, so a batch of B targets is split
into contiguous shards, one per rank, with no data-path collective; only the
final phase arrays travel, gathered to rank 0 (RCCL send/recv over xGMI in
libslm_hip, slm_plan_gather_phase). The same shard arithmetic drives bench.py,
the sequence CLI and the CPU tests of the N > 1 path.

The control plane -- handing rank 0's RCCL unique id to the other ranks,
barriers, the max of per-rank times, gathering per-frame error lists -- is a
small TCP star centred on rank 0 (:class:`Group`, stdlib sockets only). Ranks
find it through the launcher's environment (RANK, WORLD_SIZE, MASTER_ADDR,
MASTER_PORT as set by torch.distributed.run or by bench.py's own launcher);
the star listens on $SLM_RDZV_PORT, default MASTER_PORT + 1 (torchrun's agent
keeps MASTER_PORT for its own store).
"""
from __future__ import annotations

import os
import pickle
import socket
import struct
import time


def world() -> tuple[int, int, int]:
    """(rank, world_size, local_rank) from the launcher's environment."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def shard_counts(total: int, nranks: int) -> list[int]:
    """Contiguous shard sizes: the first total % nranks ranks take one more."""
    if nranks < 1 or total < 0:
        raise ValueError("need nranks >= 1 and total >= 0")
    q, r = divmod(total, nranks)
    return [q + (1 if k < r else 0) for k in range(nranks)]


def shard_range(total: int, nranks: int, rank: int) -> range:
    """Indices of the holograms owned by `rank`."""
    counts = shard_counts(total, nranks)
    start = sum(counts[:rank])
    return range(start, start + counts[rank])


def assemble(parts: list, counts: list[int]):
    """Concatenate per-rank results (rank order) into the global batch order;
    the host-side twin of the RCCL gather."""
    import numpy as np

    if len(parts) != len(counts):
        raise ValueError("one part per rank")
    for p, c in zip(parts, counts):
        if len(p) != c:
            raise ValueError(f"part of {len(p)} holograms where {c} were expected")
    return np.concatenate([np.asarray(p) for p in parts if len(p)], axis=0)


def free_port(addr: str = "127.0.0.1") -> int:
    with socket.socket() as s:
        s.bind((addr, 0))
        return s.getsockname()[1]


def _send(sock, obj) -> None:
    data = pickle.dumps(obj, protocol=pickle.HIGHEST_PROTOCOL)
    sock.sendall(struct.pack("!Q", len(data)) + data)


def _recv_exact(sock, n: int) -> bytes:
    buf = bytearray()
    while len(buf) < n:
        chunk = sock.recv(min(1 << 20, n - len(buf)))
        if not chunk:
            raise ConnectionError("control-plane peer closed the connection")
        buf += chunk
    return bytes(buf)


def _recv(sock):
    (n,) = struct.unpack("!Q", _recv_exact(sock, 8))
    return pickle.loads(_recv_exact(sock, n))  # peers are this job's own ranks


class Group:
    """Star-shaped host control plane over TCP (no torch, no MPI).

    Every rank calls the same collectives in the same order. Rank 0 accepts
    WORLD_SIZE - 1 connections; messages are length-prefixed pickles exchanged
    between the ranks of one job only."""

    def __init__(self, rank: int, world_size: int, addr: str = "127.0.0.1", port: int | None = None,
                 timeout: float = 300.0):
        if world_size < 1 or not 0 <= rank < world_size:
            raise ValueError(f"bad rank {rank} of {world_size}")
        self.rank, self.world = rank, world_size
        self.peers: list[socket.socket | None] = []
        self.sock: socket.socket | None = None
        if world_size == 1:
            return
        if port is None:
            raise ValueError("a control-plane port is needed for world_size > 1")
        if rank == 0:
            srv = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
            srv.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
            try:
                srv.bind((addr, port))
            except OSError as e:
                srv.close()
                raise OSError(f"control plane cannot listen on {addr}:{port} ({e}); set SLM_RDZV_PORT") from e
            srv.listen(world_size)
            srv.settimeout(timeout)
            peers: list[socket.socket | None] = [None] * world_size
            try:
                for _ in range(world_size - 1):
                    conn, _ = srv.accept()
                    conn.settimeout(timeout)
                    conn.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
                    r = _recv(conn)
                    if not (isinstance(r, int) and 0 < r < world_size) or peers[r] is not None:
                        raise ConnectionError(f"unexpected control-plane hello {r!r}")
                    peers[r] = conn
            finally:
                srv.close()
            self.peers = peers
        else:
            deadline = time.monotonic() + timeout
            while True:
                try:
                    s = socket.create_connection((addr, port), timeout=5.0)
                    break
                except OSError:
                    if time.monotonic() > deadline:
                        raise
                    time.sleep(0.05)
            s.settimeout(timeout)
            s.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
            _send(s, rank)
            self.sock = s

    @classmethod
    def from_env(cls, timeout: float = 300.0) -> "Group":
        rank, ws, _ = world()
        if ws == 1:
            return cls(0, 1)
        addr = os.environ.get("MASTER_ADDR", "127.0.0.1")
        port = int(os.environ.get("SLM_RDZV_PORT") or int(os.environ["MASTER_PORT"]) + 1)
        return cls(rank, ws, addr, port, timeout)

    # -- collectives -------------------------------------------------------
    def gather(self, obj, root: int = 0):
        """Rank 0 gets [obj of rank 0, obj of rank 1, ...]; the others get None."""
        if root != 0:
            raise ValueError("the star gathers to rank 0")
        if self.world == 1:
            return [obj]
        if self.rank == 0:
            return [obj] + [_recv(self.peers[r]) for r in range(1, self.world)]
        _send(self.sock, obj)
        return None

    def bcast(self, obj=None, root: int = 0):
        if root != 0:
            raise ValueError("the star broadcasts from rank 0")
        if self.world == 1:
            return obj
        if self.rank == 0:
            for r in range(1, self.world):
                _send(self.peers[r], obj)
            return obj
        return _recv(self.sock)

    def all_gather(self, obj) -> list:
        return self.bcast(self.gather(obj))

    def barrier(self) -> None:
        self.all_gather(None)

    def max(self, value: float) -> float:
        return max(self.all_gather(float(value)))

    def close(self) -> None:
        for s in self.peers:
            if s is not None:
                s.close()
        if self.sock is not None:
            self.sock.close()
        self.peers, self.sock = [], None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
