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

import hmac
import os
import pickle
import secrets
import socket
import stat
import struct
import tempfile
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


# Largest control-plane message a rank accepts (error lists, unique ids and
# timings are far smaller); a longer length prefix is refused, never allocated.
MAX_MESSAGE = 64 << 20
_HELLO_MAGIC = b"SLMh"
_MAX_TOKEN = 256


def job_token() -> bytes:
    """Shared secret of one job's ranks from the launcher: $SLM_JOB_TOKEN
    (bench.py's own launcher draws a random one), else torchrun's per-job run
    id -- unless that is empty or the constant 'none' a non-standalone torchrun
    sets, which admits nothing (b"": see local_token_file)."""
    tok = os.environ.get("SLM_JOB_TOKEN") or ""
    if not tok:
        run_id = os.environ.get("TORCHELASTIC_RUN_ID") or ""
        tok = "" if run_id.lower() in ("", "none") else run_id
    return tok.encode()[:_MAX_TOKEN]


def _is_local(addr: str) -> bool:
    return addr in ("127.0.0.1", "localhost", "::1") or addr.startswith("127.")


def local_token_file(port: int) -> str:
    """Where rank 0 of a single-host job whose launcher gave no secret leaves a
    fresh random token for the other ranks: a file only this user can read, in
    a directory only this user can enter (checked, never followed through a
    link). Local ranks of the same job run as the same user; a process of
    another user cannot read it, so it cannot pass the hello."""
    d = os.path.join(tempfile.gettempdir(), f"slm-ctl-{os.getuid()}")
    try:
        os.mkdir(d, 0o700)
    except FileExistsError:
        pass
    st = os.lstat(d)
    if not stat.S_ISDIR(st.st_mode) or st.st_uid != os.getuid() or st.st_mode & 0o077:
        raise PermissionError(f"{d} is not a private directory of this user; set SLM_JOB_TOKEN")
    return os.path.join(d, f"job-{port}.token")


def _write_token_file(path: str) -> bytes:
    tok = secrets.token_hex(16).encode()
    tmp = f"{path}.{os.getpid()}"
    fd = os.open(tmp, os.O_WRONLY | os.O_CREAT | os.O_EXCL, 0o600)
    with os.fdopen(fd, "wb") as f:
        f.write(tok)
    os.replace(tmp, path)
    return tok


def _read_token_file(path: str) -> bytes | None:
    try:
        fd = os.open(path, os.O_RDONLY | getattr(os, "O_NOFOLLOW", 0))
    except FileNotFoundError:
        return None
    with os.fdopen(fd, "rb") as f:
        return f.read(_MAX_TOKEN)


def _send(sock, obj) -> None:
    data = pickle.dumps(obj, protocol=pickle.HIGHEST_PROTOCOL)
    if len(data) > MAX_MESSAGE:
        raise ValueError(f"control-plane message of {len(data)} bytes exceeds {MAX_MESSAGE}")
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
    if n > MAX_MESSAGE:
        raise ConnectionError(f"control-plane message of {n} bytes exceeds {MAX_MESSAGE}")
    return pickle.loads(_recv_exact(sock, n))  # only peers that passed the hello check reach here


_ACK = b"\x06"


def _send_hello(sock, rank: int, token: bytes) -> None:
    sock.sendall(_HELLO_MAGIC + struct.pack("!IH", rank, len(token)) + token)


def _recv_hello(sock, world_size: int, token: bytes) -> int:
    """Raw-bytes hello (no unpickling): magic, rank, the job token."""
    head = _recv_exact(sock, 10)
    if head[:4] != _HELLO_MAGIC:
        raise ConnectionError("control-plane hello has the wrong magic")
    rank, ntok = struct.unpack("!IH", head[4:])
    if ntok > _MAX_TOKEN:
        raise ConnectionError("control-plane hello token too long")
    got = _recv_exact(sock, ntok)
    if not hmac.compare_digest(got, token):
        raise ConnectionError("control-plane hello with a foreign job token")
    if not 0 < rank < world_size:
        raise ConnectionError(f"control-plane hello from rank {rank} of {world_size}")
    return rank


class Group:
    """Star-shaped host control plane over TCP (no torch, no MPI).

    Every rank calls the same collectives in the same order. Rank 0 accepts
    WORLD_SIZE - 1 connections. A connection is admitted only after a raw-bytes
    hello carrying the job token (job_token(); when the launcher provides none
    and the job is on this host, rank 0 draws one into local_token_file) and
    acknowledged with one byte; only then are messages -- length-prefixed
    pickles, at most MAX_MESSAGE bytes -- exchanged. A job spread over
    several hosts must set $SLM_JOB_TOKEN (or run under a torchrun with a run
    id)."""

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
            token = job_token()
            token_path = None
            if not token:
                if not _is_local(addr):
                    srv.close()
                    raise RuntimeError("a multi-host control plane needs a job secret: set SLM_JOB_TOKEN")
                token_path = local_token_file(port)
                token = _write_token_file(token_path)
            deadline = time.monotonic() + timeout
            try:
                while any(p is None for p in peers[1:]):
                    srv.settimeout(max(0.01, deadline - time.monotonic()))
                    conn, _ = srv.accept()
                    conn.settimeout(min(timeout, 30.0))
                    conn.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
                    try:
                        r = _recv_hello(conn, world_size, token)
                        if peers[r] is not None:
                            raise ConnectionError(f"second control-plane hello from rank {r}")
                        conn.sendall(_ACK)
                    except (ConnectionError, OSError):
                        conn.close()  # not one of this job's ranks: drop it, keep listening
                        continue
                    conn.settimeout(timeout)
                    peers[r] = conn
            finally:
                srv.close()
                if token_path is not None:
                    try:
                        os.unlink(token_path)  # every rank has joined (or the job failed)
                    except OSError:
                        pass
            self.peers = peers
        else:
            deadline = time.monotonic() + timeout
            token = job_token()
            token_path = None
            if not token:
                if not _is_local(addr):
                    raise RuntimeError("a multi-host control plane needs a job secret: set SLM_JOB_TOKEN")
                token_path = local_token_file(port)
            while True:
                s = None
                try:
                    if token_path is not None:
                        token = _read_token_file(token_path)  # rank 0's, once it has drawn it
                        if token is None:
                            raise ConnectionError("rank 0 has not published the job token yet")
                    s = socket.create_connection((addr, port), timeout=5.0)
                    s.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
                    _send_hello(s, rank, token)
                    if _recv_exact(s, 1) != _ACK:  # a refused hello (e.g. a stale token file) closes
                        raise ConnectionError("control-plane hello not acknowledged")
                    break
                except OSError:
                    if s is not None:
                        s.close()
                    if time.monotonic() > deadline:
                        raise
                    time.sleep(0.05)
            s.settimeout(timeout)
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
