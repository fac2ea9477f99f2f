"""The N > 1 path on CPU: world_size-2 (and 3) process groups.

Holograms are independent: ranks take contiguous shards
(parallel.shard_range), compute with no data-path collective, and only the
results travel (RCCL send/recv to rank 0 on the GPU box). The host control
plane is parallel.Group (stdlib TCP, no torch); a gloo process group is run
beside it as the cross-check. The HIP compute is replaced by the float64
oracle in these CPU tests - the sharding, gather order, file output and the
reference CLI behaviour are what is tested. Workers are spawned processes;
torch is imported only inside the gloo workers.
"""
import multiprocessing
import os

import numpy as np
import pytest

from oracle import gs_gd_oracle as orc
from spatial_light_modulator_module_amd import parallel

_free_port = parallel.free_port


def _spawn(fn, args, nprocs):
    """torch.multiprocessing.spawn's contract on the stdlib: fn(rank, *args)."""
    ctx = multiprocessing.get_context("spawn")
    procs = [ctx.Process(target=fn, args=(r,) + tuple(args)) for r in range(nprocs)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
    for p in procs:
        if p.is_alive():
            p.kill()
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]


def oracle_run_gs(targets, loops, tol=0.0, ain=None, initial_phase=None):
    """Stand-in with run_gs's return contract, computed by the oracle."""
    phases, es, errs = [], [], []
    for t in targets:
        ph, exp, err = orc.gerchberg_saxton_faithful(t, loops, tol)
        phases.append(ph.astype(np.float32))
        es.append(exp)
        errs.append(list(err))
    b = len(targets)
    return np.stack(phases), np.stack(es), errs, np.ones(b), np.ones(b)


@pytest.mark.parametrize("total,nranks", [(0, 2), (1, 2), (5, 2), (7, 3), (8, 8), (3, 5)])
def test_shards_cover_the_batch(total, nranks):
    seen = []
    for r in range(nranks):
        seen += list(parallel.shard_range(total, nranks, r))
    assert seen == list(range(total))
    counts = parallel.shard_counts(total, nranks)
    assert max(counts) - min(counts) <= 1 and sum(counts) == total


def test_assemble_checks_counts():
    parts = [np.zeros((2, 4, 4)), np.ones((1, 4, 4))]
    out = parallel.assemble(parts, [2, 1])
    assert out.shape == (3, 4, 4) and out[2].min() == 1
    with pytest.raises(ValueError):
        parallel.assemble(parts, [1, 2])


def _setup(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), SLM_RDZV_PORT=str(port + 1))
    return parallel.Group.from_env(timeout=60)


def _batch_worker(rank, world, port, targets, loops, out_path):
    group = _setup(rank, world, port)
    mine = parallel.shard_range(len(targets), world, rank)
    phase, _, _, _, _ = oracle_run_gs(targets[mine.start:mine.stop], loops)
    parts = group.gather(phase)
    if rank == 0:
        full = parallel.assemble(parts, parallel.shard_counts(len(targets), world))
        np.save(out_path, full)
    t = group.max(float(rank))
    assert t == world - 1
    group.barrier()
    group.close()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_batch_equals_single_process(tmp_path, world):
    rng = np.random.default_rng(3)
    targets = rng.integers(0, 256, size=(5, 64, 64)).astype(np.uint8)
    out = str(tmp_path / "phase.npy")
    _spawn(_batch_worker, (world, _free_port(), targets, 4, out), world)
    want, _, _, _, _ = oracle_run_gs(targets, 4)
    np.testing.assert_array_equal(np.load(out), want)


def _control_plane_vs_gloo_worker(rank, world, port, out_dir):
    """The torch-free star and a gloo process group agree on every collective
    bench.py and the sequence CLI use (bcast of the RCCL id, all_gather, max)."""
    group = _setup(rank, world, port)
    import torch
    import torch.distributed as dist

    dist.init_process_group("gloo", rank=rank, world_size=world)
    uid = os.urandom(128) if rank == 0 else None
    got = group.bcast(uid)
    ref = [uid]
    dist.broadcast_object_list(ref, src=0)
    assert got == ref[0] and len(got) == 128
    obj = {rank: [np.float64(rank) * 0.5, rank]}
    mine = group.all_gather(obj)
    theirs = [None] * world
    dist.all_gather_object(theirs, obj)
    assert mine == theirs
    t = torch.tensor([float(rank) + 0.25], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    assert group.max(float(rank) + 0.25) == float(t.item())
    group.barrier()
    dist.barrier()
    np.save(os.path.join(out_dir, f"ok{rank}.npy"), np.array([1]))
    dist.destroy_process_group()
    group.close()


def test_control_plane_matches_gloo(tmp_path):
    _spawn(_control_plane_vs_gloo_worker, (2, _free_port(), str(tmp_path)), 2)
    assert all((tmp_path / f"ok{r}.npy").exists() for r in range(2))


def test_group_single_rank_is_local():
    g = parallel.Group(0, 1)
    assert g.all_gather("x") == ["x"] and g.bcast(3) == 3 and g.max(2.5) == 2.5
    g.barrier()
    g.close()


def _make_sequence(root, n):
    from PIL import Image

    d = os.path.join(root, "images", "moving_traps", "seq")
    os.makedirs(d)
    rng = np.random.default_rng(11)
    for i in range(n):
        img = np.zeros((64, 128), np.uint8)
        y, x = rng.integers(4, 60), rng.integers(4, 124)
        img[y - 2:y + 2, x - 2:x + 2] = 255
        Image.fromarray(img).save(os.path.join(d, f"{i}.png"))


def _sequence_worker(rank, world, port, root):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), SLM_RDZV_PORT=str(port + 1))
    from spatial_light_modulator_module_amd import generate_hologram_sequence as ghs

    os.chdir(root)
    ghs.run_gs = oracle_run_gs  # CPU stand-in for the GPU batch
    errors = ghs.cli(["seq", "-v", "w2", "-ct2pi", "255", "-loops", "3", "-p"], plot=False)
    np.save(os.path.join(root, f"errors_rank{rank}.npy"), np.array([errors[i] for i in sorted(errors)]))


def test_sequence_cli_two_ranks_matches_single(tmp_path, monkeypatch):
    from spatial_light_modulator_module_amd import generate_hologram_sequence as ghs

    n = 5
    two, one = tmp_path / "two", tmp_path / "one"
    for r in (two, one):
        r.mkdir()
        _make_sequence(str(r), n)
    _spawn(_sequence_worker, (2, _free_port(), str(two)), 2)

    monkeypatch.chdir(one)
    monkeypatch.setattr(ghs, "run_gs", oracle_run_gs)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
        monkeypatch.delenv(k, raising=False)
    errors = ghs.cli(["seq", "-v", "w2", "-ct2pi", "255", "-loops", "3", "-p"], plot=False)
    assert sorted(errors) == list(range(n))
    for i in range(n):
        a = np.load(two / "holograms" / "seq_w2_holograms" / f"{i}.npy")
        b = np.load(one / "holograms" / "seq_w2_holograms" / f"{i}.npy")
        assert a.dtype == np.float64 and a.shape == (64, 128)
        np.testing.assert_array_equal(a, b)
        assert (two / "images" / "moving_traps" / "seq_w2_preview" / f"{i}.png").exists()
    # both ranks see the gathered error evolutions of every frame
    for r in (0, 1):
        np.testing.assert_array_equal(np.load(two / f"errors_rank{r}.npy"),
                                      np.array([errors[i] for i in range(n)]))


def test_control_plane_admits_only_this_jobs_ranks(monkeypatch):
    """Rank 0 reads a raw-bytes hello (magic, rank, job token) before it
    unpickles anything: a foreign client -- a pickle payload, a wrong token, an
    oversized length prefix -- is dropped and the real rank 1 still joins."""
    import pickle
    import socket
    import struct
    import threading

    monkeypatch.setenv("SLM_JOB_TOKEN", "job-a")
    port = _free_port()
    box = {}

    def rank0():
        box["g0"] = parallel.Group(0, 2, "127.0.0.1", port, timeout=30)

    th = threading.Thread(target=rank0)
    th.start()
    import time

    deadline = time.monotonic() + 10
    while True:  # rank 0 listening?
        try:
            probe = socket.create_connection(("127.0.0.1", port), timeout=1)
            break
        except OSError:
            assert time.monotonic() < deadline
            time.sleep(0.02)
    evil = pickle.dumps(1)  # a pickle instead of a hello
    probe.sendall(struct.pack("!Q", len(evil)) + evil)
    probe.close()
    wrong = socket.create_connection(("127.0.0.1", port), timeout=5)
    parallel._send_hello(wrong, 1, b"job-b")  # right shape, foreign token
    wrong.close()
    huge = socket.create_connection(("127.0.0.1", port), timeout=5)
    huge.sendall(b"SLMh" + struct.pack("!IH", 1, 65535))  # token length beyond the cap
    huge.close()
    g1 = parallel.Group(1, 2, "127.0.0.1", port, timeout=30)
    th.join(30)
    g0 = box["g0"]
    out = {}
    t2 = threading.Thread(target=lambda: out.setdefault(0, g0.all_gather("zero")))
    t2.start()
    assert g1.all_gather("one") == ["zero", "one"]
    t2.join(10)
    assert out[0] == ["zero", "one"]
    with pytest.raises(ValueError):
        parallel._send(g1.sock, b"x" * (parallel.MAX_MESSAGE + 1))
    g0.close()
    g1.close()


def test_control_plane_without_launcher_secret(monkeypatch):
    """A launcher that gives no secret (no $SLM_JOB_TOKEN; a non-standalone
    torchrun's TORCHELASTIC_RUN_ID is the constant 'none') still admits only
    this job's ranks: rank 0 draws a token into a file only this user can read
    (parallel.local_token_file), a stale file of an earlier job on the same
    port is replaced, an empty or 'none' token is refused."""
    import socket
    import threading
    import time

    monkeypatch.delenv("SLM_JOB_TOKEN", raising=False)
    monkeypatch.setenv("TORCHELASTIC_RUN_ID", "none")
    assert parallel.job_token() == b""
    port = _free_port()
    path = parallel.local_token_file(port)
    with open(path, "wb") as f:
        f.write(b"stale-token-of-an-earlier-job")
    box = {}
    th = threading.Thread(target=lambda: box.setdefault("g0", parallel.Group(0, 2, "127.0.0.1", port, timeout=30)))
    th.start()
    deadline = time.monotonic() + 10
    while True:
        try:
            probe = socket.create_connection(("127.0.0.1", port), timeout=1)
            break
        except OSError:
            assert time.monotonic() < deadline
            time.sleep(0.02)
    for bad in (b"", b"none", b"stale-token-of-an-earlier-job"):
        parallel._send_hello(probe, 1, bad)
        assert probe.recv(1) == b""  # dropped without an acknowledgement
        probe.close()
        probe = socket.create_connection(("127.0.0.1", port), timeout=5)
    probe.close()
    g1 = parallel.Group(1, 2, "127.0.0.1", port, timeout=30)
    th.join(30)
    g0 = box["g0"]
    assert not os.path.exists(path)  # removed once every rank joined
    assert os.stat(os.path.dirname(path)).st_mode & 0o077 == 0
    out = {}
    t2 = threading.Thread(target=lambda: out.setdefault(0, g0.all_gather(0)))
    t2.start()
    assert g1.all_gather(1) == [0, 1]
    t2.join(10)
    g0.close()
    g1.close()
