#!/usr/bin/env python3
"""Throughput bench of the GS hologram loop on MI355X (BASELINE.json configs).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--size 1024] [--batch-per-gpu 1] [--iters 200]

One *step* is one full GS run (setup + `iters` iterations + phase extraction)
over this rank's batch of synthetic targets already resident in HBM, followed
by the RCCL gather of the final phase arrays to rank 0. Default workload is
BASELINE.json configs[1]: a single 1024x1024 float32 random-amplitude target,
200 iterations, per GPU (weak scaling: N GPUs process N x batch holograms).

For N > 1 the driver launches one process per GPU with torch.distributed.run;
torch.distributed (gloo, CPU) is only the control plane (barriers, max of the
per-rank times, broadcast of the RCCL unique id). The data path is
libslm_hip.so: its kernels and its RCCL send/recv gather over xGMI.

Rank 0 prints ONE JSON line with the metric, a roofline object for the
dominant kernel (HIP-event timing of every launch of a separately replayed,
identical run) and the CPU baseline (the repo's NumPy oracle, 1 core, on a
bounded sample of the same workload, rank 0 at N=1 only).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# libslm_hip.so (torch is imported ahead of it: one HIP runtime per process)
from spatial_light_modulator_module_amd import _lib  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec
METRIC = json.load(open(os.path.join(ROOT, "BASELINE.json")))["metric"]


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--size", type=int, default=1024)
    ap.add_argument("--batch-per-gpu", type=int, default=1)
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extra", action="store_true", help="skip the 4096^2 / batched secondary measurements")
    ap.add_argument("--cpu-sample-seconds", type=float, default=20.0)
    return ap.parse_args()


class Dist:
    """Control plane: gloo process group when launched with WORLD_SIZE > 1."""

    def __init__(self):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local_rank = int(os.environ.get("LOCAL_RANK", "0"))
        self.pg = None
        if self.world > 1:
            import torch.distributed as dist

            dist.init_process_group("gloo")
            self.dist = dist

    def barrier(self):
        if self.world > 1:
            self.dist.barrier()

    def max(self, v: float) -> float:
        if self.world == 1:
            return v
        import torch

        t = torch.tensor([v], dtype=torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def bcast_bytes(self, b: bytes | None) -> bytes:
        if self.world == 1:
            return b
        obj = [b]
        self.dist.broadcast_object_list(obj, src=0)
        return obj[0]


def targets(first: int, count: int, n: int) -> np.ndarray:
    """T_b = default_rng(1234 + b).uniform(0, 255, (n, n)) float32."""
    return np.stack([np.random.default_rng(1234 + b).uniform(0, 255, (n, n)).astype(np.float32)
                     for b in range(first, first + count)])


def kernel_roofline(plan, iters, white_attention=0.0):
    """Time every launch of one run with HIP events on the plan's stream and
    price the dominant kernel class with its algorithmic bytes."""
    us, cnt = plan.run_timed(iters, white_attention=white_attention)
    rows = {}
    for cls in (_lib.KERNEL_COL_MAIN, _lib.KERNEL_ROW_MAIN, _lib.KERNEL_GD_STATS):
        if cnt[cls] == 0:
            continue
        avg_us = us[cls] / cnt[cls]
        nbytes = plan.kernel_bytes(cls)
        rows[_lib.KERNEL_CLASS_NAMES[cls]] = {
            "avg_us": avg_us, "launches": int(cnt[cls]), "total_us": float(us[cls]), "bytes_per_launch": nbytes,
            "achieved_gbs": nbytes / (avg_us * 1e-6) / 1e9}
    dom = max(rows, key=lambda k: rows[k]["total_us"])
    return dom, rows, us, cnt


def pmc_traffic(config_key: str):
    """HBM bytes per launch from the committed rocprofv3 PMC summary, if one was
    collected for this exact configuration (profiles/pmc_traffic.json)."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            return json.load(f).get(config_key)
    except (OSError, ValueError):
        return None


def cpu_baseline(n: int, iters: int, budget_s: float):
    """The repo's NumPy restatement (faithful float64, scipy.fft single thread,
    1 core) on the same synthetic target, k iterations, extrapolated."""
    from oracle import gs_gd_oracle as orc

    t = targets(0, 1, n)[0]
    t0 = time.perf_counter()
    orc.gerchberg_saxton_faithful(t, 2)
    per_iter = (time.perf_counter() - t0) / 2
    k = int(max(3, min(iters, budget_s / max(per_iter, 1e-6))))
    t0 = time.perf_counter()
    orc.gerchberg_saxton_faithful(t, k)
    dt = time.perf_counter() - t0
    per_iter = dt / k
    holo_s = 1.0 / (per_iter * iters)
    return {"value": holo_s, "unit": "holograms/s", "cores": 1, "kind": "port",
            "sample": f"{k} GS iterations of the NumPy/SciPy float64 restatement (oracle/gs_gd_oracle.py) on one "
                      f"{n}x{n} float32 target in {dt:.1f} s, extrapolated to {iters} iterations per hologram",
            "ms_per_iter": per_iter * 1e3, "host_cpus": os.cpu_count()}


def pcie_inclusive(plan, host_targets, iters, reps=5):
    """The drop-in boundary's host-to-host rate: target upload, the run and the
    phase download per step (never the headline value)."""
    t0 = time.perf_counter()
    for _ in range(reps):
        plan.set_target(host_targets)
        plan.run(iters)
        plan.read(phase=True, expected=False, stats=False, iters=False)
    wall = (time.perf_counter() - t0) / reps
    return {"holograms_per_s": host_targets.shape[0] / wall, "ms_per_step": wall * 1e3,
            "includes": "target upload + relayout, run, phase download (pageable host memory)"}


def secondary(n, batch, iters, algo=_lib.ALGO_GS, precision=None, reps=3):
    """Extra single-GPU measurements: one-run wall time and the per-kernel
    roofline of another configuration (4096^2 HBM stress, batched 1024^2, GD,
    float32 butterflies)."""
    t = targets(0, batch, n)
    with _lib.Plan(algo, batch, n, n, _lib.TGT_F32, False, iters) as plan:
        plan.set_target(t)
        if precision is not None:
            plan.set_precision(precision)
        wa = 0.0
        if algo == _lib.ALGO_GD:  # BASELINE.json configs[2]: lr 0.005, white_attention 1, random guess seed 42
            from spatial_light_modulator_module_amd import algorithms as alg

            plan.set_lr(np.full(iters, 0.005, np.float32))
            plan.set_field(np.stack([alg.make_initial_guess("random", None, t[k], 42) for k in range(batch)]))
            wa = 1.0
        plan.run(iters, white_attention=wa)
        plan.sync()
        t0 = time.perf_counter()
        for _ in range(reps):
            plan.run(iters, white_attention=wa)
        plan.sync()
        wall = (time.perf_counter() - t0) / reps
        dom, rows, _, _ = kernel_roofline(plan, iters, wa)
        info = plan.info()
    iter_ms = wall / iters * 1e3
    name = "gd" if algo == _lib.ALGO_GD else "gs"
    traffic = pmc_traffic(f"{name}_{n}x{n}_b{batch}_it{iters}_{info['precision']}")  # rocprofv3 PMC, profiles/
    for k, row in rows.items():
        row["traffic_bytes_per_launch"] = None if traffic is None else traffic.get(k)
    return {"algo": name, "shape": [batch, n, n], "iters": iters,
            "holograms_per_s": batch / wall, "iter_ms": iter_ms, "iter_ms_per_hologram": iter_ms / batch,
            "kernels": rows, "dominant": dom,
            "dominant_frac_of_hbm_peak": round(rows[dom]["achieved_gbs"] / HBM_PEAK_GBS, 4), "tiling": info}


def main():
    opt = parse()
    d = Dist()
    _lib.init(d.local_rank if d.world > 1 else int(os.environ.get("SLM_DEVICE", "0")))
    n, bper, iters = opt.size, opt.batch_per_gpu, opt.iters
    counts = [bper] * d.world

    if d.world > 1:
        uid = _lib.comm_unique_id() if d.rank == 0 else None
        uid = d.bcast_bytes(uid)
        _lib.comm_init(d.world, d.rank, uid)

    plan = _lib.Plan(_lib.ALGO_GS, bper, n, n, _lib.TGT_F32, False, iters)
    plan.set_target(targets(d.rank * bper, bper, n))

    def step():
        plan.run(iters)
        plan.gather_phase(counts, root=0)  # synchronises the plan stream

    for _ in range(opt.warmup):
        step()
    plan.sync()
    d.barrier()
    t0 = time.perf_counter()
    for _ in range(opt.steps):
        step()
    plan.sync()
    d.barrier()
    elapsed = d.max(time.perf_counter() - t0)

    total_holo = bper * d.world * opt.steps
    value = total_holo / elapsed
    ms_per_step = elapsed / opt.steps * 1e3

    dom, rows, _, _ = kernel_roofline(plan, iters)
    info = plan.info()
    # sanity: the phases are finite and the error curve decreases
    phase, _, stats, _ = plan.read(expected=False, iters=False)
    ok = bool(np.isfinite(phase).all() and stats[0, iters - 1, 3] < stats[0, 0, 3])

    if d.rank != 0:
        plan.close()
        if d.world > 1:
            _lib.comm_destroy()
        return

    prec = info["precision"]  # butterflies / twiddles / exchanges; HBM state is complex64
    key = f"gs_{n}x{n}_b{bper}_it{iters}_{prec}"
    traffic = pmc_traffic(key)
    dr = rows[dom]
    roofline = {"bound": "hbm", "achieved": round(dr["achieved_gbs"], 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(dr["achieved_gbs"] / HBM_PEAK_GBS, 4),
                "traffic": None if traffic is None else traffic.get(dom),
                "kernel": dom, "avg_us": round(dr["avg_us"], 3), "bytes_per_launch": dr["bytes_per_launch"],
                "kernels": {k: {kk: (round(vv, 3) if isinstance(vv, float) else vv) for kk, vv in v.items()}
                            for k, v in rows.items()}}
    out = {
        "metric": METRIC, "value": round(value, 3), "unit": "holograms/s", "n_gpus": d.world,
        "steps": opt.steps, "warmup": opt.warmup, "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": prec,
        "data": "synthetic (uniform[0,255) float32 targets, default_rng(1234+b))",
        "config": {"workload": f"GS {n}x{n}, {iters} iterations, {bper} hologram(s) per GPU, float32 target, "
                               "uniform incoming intensity, tolerance 0 (BASELINE.json configs[1])",
                   "height": n, "width": n, "iters": iters, "batch_per_gpu": bper, "global_batch": bper * d.world,
                   "parallelism": f"dp{d.world} (independent holograms; RCCL gather of phases to rank 0)",
                   "storage": "complex64 field, float32 target/phase", "col_tile": info},
        "gs_iter_ms": round(ms_per_step / iters, 5),
        "roofline": roofline,
        "check": "ok" if ok else "FAILED",
    }
    if d.world == 1 and not opt.no_extra:
        extra = {"pcie_inclusive": pcie_inclusive(plan, targets(0, bper, n), iters)}
        try:
            extra["gs_4096"] = secondary(4096, 1, 20)
            extra["gs_4096_batch8"] = secondary(4096, 8, 20)  # configs[4] per GPU at 8 GPUs
            extra["gs_1024_batch64"] = secondary(1024, 64, 20)  # configs[3] per GPU at 8 GPUs
            extra["gd_1024"] = secondary(1024, 1, 500, algo=_lib.ALGO_GD, reps=2)  # configs[2]
            f64 = _lib.PRECISION_F64  # float64 butterflies (parity margin)
            extra["f64_gs_1024"] = secondary(1024, 1, 200, precision=f64)
            extra["f64_gs_4096"] = secondary(4096, 1, 20, precision=f64)
        except _lib.SlmError as e:  # pragma: no cover - report, do not hide
            extra["error"] = str(e)
        out["extra"] = extra
    if d.world == 1 and not opt.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(n, iters, opt.cpu_sample_seconds)
    print(json.dumps(out), flush=True)
    plan.close()
    if d.world > 1:
        _lib.comm_destroy()


if __name__ == "__main__":
    main()
