#!/usr/bin/env python3
"""Rehearse the N > 1 gather path (RCCL send/recv of phases and statistics,
slm_plan_gather_phase / slm_plan_gather_stats): each rank runs its shard of a
GS batch; rank 0 checks the gathered phases and error curves bit for bit
against one process running the whole batch (a batch equals its single runs
bitwise, tests/test_gpu_gs.py).

    python tools/rccl_rehearsal.py [--ranks 2] [--size 1024] [--per-rank 2] [--iters 5] [--share-device]

Without a launcher it starts the ranks itself (as bench.py does), one GPU per
rank; --share-device puts every rank on device 0 (a one-GPU box). RCCL 2.27
refuses that ("Duplicate GPU detected": ncclCommInitRank returns invalid
usage on every rank, profiles/r04/rccl_rehearsal_s10.txt), so on one GPU the
script shows the refusal path: every rank fails fast with SLM_ERR_COMM.
"""
import argparse
import os
import secrets
import subprocess
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from spatial_light_modulator_module_amd import _lib, parallel  # noqa: E402


def targets(first, count, n):
    return np.stack([np.random.default_rng(1234 + b).uniform(0, 255, (n, n)).astype(np.float32)
                     for b in range(first, first + count)])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", type=int, default=2)
    ap.add_argument("--size", type=int, default=1024)
    ap.add_argument("--per-rank", type=int, default=2)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--share-device", action="store_true")
    o = ap.parse_args()
    if "WORLD_SIZE" not in os.environ:
        port = parallel.free_port()
        token = secrets.token_hex(16)
        procs = []
        for r in range(o.ranks):
            env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(o.ranks),
                       LOCAL_WORLD_SIZE=str(o.ranks), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                       SLM_RDZV_PORT=str(port), SLM_JOB_TOKEN=token)
            if o.share_device:
                env["SLM_DEVICE"] = "0"
            procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
        sys.exit(max(abs(p.wait()) for p in procs))

    rank, world, local_rank = parallel.world()
    group = parallel.Group.from_env(timeout=120.0)
    _lib.init(0 if o.share_device else local_rank)
    n, per, iters = o.size, o.per_rank, o.iters
    counts = [per] * world
    uid = _lib.comm_unique_id() if rank == 0 else None
    try:
        _lib.comm_init(world, rank, group.bcast(uid))
    except Exception as e:  # noqa: BLE001 -- report RCCL's refusal and stop every rank
        print(f"rank {rank}: comm_init failed: {e}", flush=True)
        group.close()
        sys.exit(3)
    with _lib.Plan(_lib.ALGO_GS, per, n, n, _lib.TGT_F32, False, iters) as plan:
        plan.set_target(targets(rank * per, per, n))
        plan.run(iters)
        gathered = np.empty((per * world, n, n), np.float32) if rank == 0 else None
        plan.gather_phase(counts, root=0, host_out=gathered)
        stats, _ = plan.gather_stats(counts, root=0, want=rank == 0)
        plan.sync()
    group.barrier()
    ok = True
    if rank == 0:
        with _lib.Plan(_lib.ALGO_GS, per * world, n, n, _lib.TGT_F32, False, iters) as ref:
            ref.set_target(targets(0, per * world, n))
            ref.run(iters)
            ph, _, st, _ = ref.read()
        ok = np.array_equal(gathered, ph)
        ok_stats = stats is not None and np.array_equal(np.asarray(stats)[:, :iters], st[:, :iters])
        print(f"RCCL {world}-rank gather on one device, {per * world} x {n}^2, {iters} iterations: phases "
              f"{'bitwise equal' if ok else 'DIFFER'} to one process; statistics "
              f"{'bitwise equal' if ok_stats else 'DIFFER'}", flush=True)
        ok = ok and ok_stats
    _lib.comm_destroy()
    group.close()
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
