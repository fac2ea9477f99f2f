#!/usr/bin/env python3
"""Throughput bench of the GS hologram loop on MI355X (BASELINE.json configs).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--size 1024] [--batch-per-gpu 1] [--iters 200]

One *step* is one full GS run (setup + `iters` iterations + phase extraction)
over this rank's batch of synthetic targets already resident in HBM, followed
by the RCCL gather of the final phase arrays to rank 0. Default workload is
BASELINE.json configs[1]: a single 1024x1024 float32 random-amplitude target,
200 iterations, per GPU (weak scaling: N GPUs process N x batch holograms).

N > 1: one process per GPU. Under torch.distributed.run (the driver's
launcher) the ranks come from its environment; `--gpus N` without one makes
this script its own launcher: it starts N child processes (RANK / LOCAL_RANK /
WORLD_SIZE / MASTER_* set, before any GPU call) and exits with their status.
No torch in the ranks: the control plane (RCCL unique-id hand-off, barriers,
the max of per-rank times) is parallel.Group (stdlib TCP), the data path is
libslm_hip.so -- its kernels and its RCCL send/recv gather over xGMI.

Rank 0 prints ONE JSON line with the metric, a roofline object for the
dominant kernel (HIP-event timing of every launch of a separately replayed,
identical run; SURVEY.md 8d byte model and the fused kernels' physical bytes,
both labelled) and the CPU baseline (the repo's NumPy oracle, 1 core and all
cores of the host share, on a bounded sample of the same workload, rank 0 at
N=1 only).
"""
from __future__ import annotations

import argparse
import json
import os
import secrets
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from spatial_light_modulator_module_amd import _lib, parallel  # noqa: E402

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


def launch_ranks(n: int) -> int:
    """bench.py --gpus N outside a launcher: N child processes, one per GPU."""
    port = parallel.free_port()
    token = secrets.token_hex(16)  # admits this job's ranks to the control plane (parallel.job_token)
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), SLM_RDZV_PORT=str(port), SLM_JOB_TOKEN=token)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rcs = [p.wait() for p in procs]
    return max(abs(rc) for rc in rcs)


def targets(first: int, count: int, n: int, w: int | None = None) -> np.ndarray:
    """T_b = default_rng(1234 + b).uniform(0, 255, (n, w or n)) float32."""
    return np.stack([np.random.default_rng(1234 + b).uniform(0, 255, (n, w or n)).astype(np.float32)
                     for b in range(first, first + count)])


def model_bytes(plan, cls, gd_fused=False):
    """SURVEY.md 8d algorithmic bytes per launch (unfused-pass byte model):
    GS 68 B/px/iteration = column passes 32 + target 4 (col_main) + row passes
    32 (row_main); GD 76 = forward column pass 16 (gd_stats) + inverse column
    pass with the target 20 (col_main) + row passes 16 + gradient epilogue 24
    (row_main). When GD's column side is one launch (gd_fused: no gd_stats
    launches) col_main carries both column passes and the target (36). A uint8
    target counts 1 B, a_in adds 4 B."""
    px = plan.batch * plan.height * plan.width
    tb = 1 if plan.tgt_type == _lib.TGT_U8 else 4
    ab = 4 if plan.has_ain else 0
    gd = plan.algo == _lib.ALGO_GD
    if cls == _lib.KERNEL_COL_MAIN:
        return px * ((16 if gd and not gd_fused else 32) + tb)
    if cls == _lib.KERNEL_ROW_MAIN:
        return px * (32 + ab + (8 if gd else 0))
    if cls == _lib.KERNEL_GD_STATS:
        return px * 16
    return 0


def kernel_roofline(plan, iters, white_attention=0.0):
    """Time every launch of one run with HIP events on the plan's stream and
    price each kernel class with both byte models: SURVEY.md 8d's (the
    roofline numerator, `achieved`) and the bytes the fused kernel physically
    reads and writes (`physical`, slm_plan_kernel_bytes)."""
    us, cnt = plan.run_timed(iters, white_attention=white_attention)
    gd_fused = plan.algo == _lib.ALGO_GD and cnt[_lib.KERNEL_GD_STATS] == 0
    rows = {}
    for cls in (_lib.KERNEL_COL_MAIN, _lib.KERNEL_ROW_MAIN, _lib.KERNEL_GD_STATS):
        if cnt[cls] == 0:
            continue
        avg_us = us[cls] / cnt[cls]
        phys = plan.kernel_bytes(cls)
        model = model_bytes(plan, cls, gd_fused)
        rows[_lib.KERNEL_CLASS_NAMES[cls]] = {
            "avg_us": avg_us, "launches": int(cnt[cls]), "total_us": float(us[cls]),
            "model_bytes_per_launch": model, "physical_bytes_per_launch": phys,
            "achieved_gbs": model / (avg_us * 1e-6) / 1e9, "physical_gbs": phys / (avg_us * 1e-6) / 1e9}
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


def traffic_for_plan(traffic, info):
    """The committed PMC entry only if it was collected on the plan being timed:
    entries stamped by tools/pmc_traffic.py with [row plan, col plan, col tile,
    precision, engines] must match (else None); unstamped (pre-r06) entries are
    used as they are, flagged plan_checked False."""
    if not traffic:
        return traffic
    want = [info.get("row_plan"), info.get("col_plan"), info.get("col_cw"), info.get("precision"),
            list(info.get("engine", ()))]
    got = traffic.get("plan")
    if got is None:
        return dict(traffic, plan_checked=False)
    return dict(traffic, plan_checked=True) if list(got) == want else None


def rocprof_kernels(config_key: str):
    """The committed rocprofv3 kernel-trace summary of this configuration
    (profiles/rocprof_kernels.json, written by tools/frac_check.py from a
    `rocprofv3 --kernel-trace --stats` run of this bench): per kernel class
    the trace's average duration over every launch, over the launches of the
    event-timed run, and the event timing bench.py printed in that same run."""
    path = os.path.join(ROOT, "profiles", "rocprof_kernels.json")
    try:
        with open(path) as f:
            return json.load(f).get(config_key)
    except (OSError, ValueError):
        return None


def rank_diagnostics(plan, counts, rank, local_elapsed, steps, rows):
    """What one rank did in the timed region, for the scaling run to break
    down (rank 0 prints every rank's record): its device, its own wall time,
    its kernels' HIP-event times, and the phase gather timed on its own with
    events (collective: every rank calls this)."""
    gather_ms, gather_bytes = plan.time_gather(counts, root=0, reps=5)
    dev = plan.device
    try:
        bus = _lib.pci_bus_id(dev)
    except _lib.SlmError:
        bus = None
    kern = {k: round(v["avg_us"], 3) for k, v in rows.items()}
    run_us = sum(v["total_us"] for v in rows.values())
    return {"rank": rank, "device": dev, "pci_bus_id": bus, "holograms": int(counts[rank]),
            "gather_stream": ("comm stream behind a staging copy (overlaps the next run)"
                              if os.environ.get("SLM_GATHER_STAGED", "0") not in ("", "0")
                              else "plan stream (default; the staged comm-stream gather measured slower)"),
            "step_ms": round(local_elapsed / steps * 1e3, 4), "kernel_avg_us": kern,
            "iteration_kernels_ms_per_run": round(run_us / 1e3, 4),
            "gather_ms": round(gather_ms, 4), "gather_bytes_to_root": gather_bytes,
            "gather_gbs": round(gather_bytes / (gather_ms * 1e-3) / 1e9, 2) if gather_bytes and gather_ms > 0 else None}


def cpu_baseline(n: int, iters: int, budget_s: float):
    """The repo's NumPy restatement of the reference (faithful float64, scipy.fft
    single thread, 1 core, as the reference runs) on the same synthetic target,
    k iterations, extrapolated to `iters`."""
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
    return {"value": 1.0 / (per_iter * iters), "unit": "holograms/s", "cores": 1, "kind": "port",
            "sample": f"{k} GS iterations of the NumPy/SciPy float64 restatement (oracle/gs_gd_oracle.py, "
                      f"single-threaded like the reference) on one {n}x{n} float32 target in {dt:.1f} s, "
                      f"extrapolated to {iters} iterations per hologram",
            "ms_per_iter": per_iter * 1e3, "host_cpus": os.cpu_count()}


def cpu_baseline_configs0(reps: int = 3):
    """BASELINE.json configs[0]: GS on one 256x256 random target, 50 iterations,
    the NumPy CPU path (the faithful float64 restatement, oracle/gs_gd_oracle.py,
    single-threaded like the reference) -- whole runs timed, not extrapolated."""
    from oracle import gs_gd_oracle as orc

    t = targets(0, 1, 256)[0]
    orc.gerchberg_saxton_faithful(t, 50)  # warm-up (imports, FFT plan caches)
    walls = []
    for _ in range(reps):
        t0 = time.perf_counter()
        orc.gerchberg_saxton_faithful(t, 50)
        walls.append(time.perf_counter() - t0)
    wall = min(walls)
    return {"value": 1.0 / wall, "unit": "holograms/s", "cores": 1, "kind": "port",
            "sample": f"{reps} whole 50-iteration GS runs (best of) of the float64 restatement on one 256x256 "
                      "float32 target (BASELINE.json configs[0])",
            "s_per_hologram": wall, "ms_per_iter": wall / 50 * 1e3, "host_cpus": os.cpu_count()}


def cpu_baseline_all_cores(n: int, iters: int, budget_s: float):
    """The multi-threaded float64 restatement (oracle/fast_f64.py: pocketfft and
    element-wise work over the host share's threads) on the same target."""
    from oracle import fast_f64

    workers = fast_f64.DEFAULT_WORKERS
    t = targets(0, 1, n)[0]
    phi = np.zeros(t.shape, np.float32)
    t0 = time.perf_counter()
    fast_f64.gerchberg_saxton_f64(t, 2, initial_phase=phi, workers=workers)
    per_iter = (time.perf_counter() - t0) / 2
    k = int(max(3, min(iters, budget_s / max(per_iter, 1e-6))))
    t0 = time.perf_counter()
    fast_f64.gerchberg_saxton_f64(t, k, initial_phase=phi, workers=workers)
    dt = time.perf_counter() - t0
    per_iter = dt / k
    return {"value": 1.0 / (per_iter * iters), "unit": "holograms/s", "cores": workers, "kind": "port",
            "sample": f"{k} GS iterations of the threaded float64 restatement (oracle/fast_f64.py, {workers} "
                      f"threads) on one {n}x{n} float32 target in {dt:.1f} s, extrapolated to {iters} iterations",
            "ms_per_iter": per_iter * 1e3}


def pcie_inclusive(plan, host_targets, iters, reps=10, warmup=2):
    """The drop-in boundary's host-to-host rate: target upload, the run and the
    phase download per step (never the headline value). Untimed
    warm-up steps first, as for the device-resident value (the first download
    pays the runtime's one-time staging setup)."""
    def step():
        plan.set_target(host_targets)
        plan.run(iters)
        plan.read(phase=True, expected=False, stats=False, iters=False)

    for _ in range(warmup):
        step()
    t0 = time.perf_counter()
    for _ in range(reps):
        step()
    wall = (time.perf_counter() - t0) / reps
    return {"holograms_per_s": host_targets.shape[0] / wall, "ms_per_step": wall * 1e3,
            "includes": "target upload + relayout, run, phase download (pageable host memory)"}


def _round(v):
    return round(v, 4) if isinstance(v, float) else v


def secondary(n, batch, iters, algo=_lib.ALGO_GS, precision=None, reps=3, width=None, engine=None):
    """Extra single-GPU measurements: one-run wall time and the per-kernel
    roofline of another configuration (4096^2 HBM stress, batched 1024^2, GD,
    float64 butterflies, an n x width SLM panel on the any-size engine).
    engine="float64": the plan is created under $SLM_ENGINE=float64 (complex128
    state and arithmetic: the complex128 radix-plan kernels on these sides)."""
    w = width or n
    t = targets(0, batch, n, w)
    saved = os.environ.get("SLM_ENGINE")
    if engine:
        os.environ["SLM_ENGINE"] = engine
    try:
        plan = _lib.Plan(algo, batch, n, w, _lib.TGT_F32, False, iters)
    finally:
        if engine:
            if saved is None:
                os.environ.pop("SLM_ENGINE", None)
            else:
                os.environ["SLM_ENGINE"] = saved
    with plan:
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
        plan_engine = plan.engine()
    iter_s = wall / iters
    # bytes the launches of one iteration physically move (slm_plan_kernel_bytes)
    phys_iter = sum(r["physical_bytes_per_launch"] for r in rows.values())
    name = "gd" if algo == _lib.ALGO_GD else "gs"
    # rocprofv3 PMC, profiles/ (keyed by engine too: complex128 plans move other bytes)
    eng_tag = "" if plan_engine[0] in ("stockham", "shuffle") else "_" + plan_engine[0]
    traffic = pmc_traffic(f"{name}_{n}x{w}_b{batch}_it{iters}_{info['precision']}{eng_tag}")
    traffic = traffic_for_plan(traffic, info)
    for k, row in rows.items():
        row["traffic_bytes_per_launch"] = None if traffic is None else traffic.get(k)
    per_px = 76 if algo == _lib.ALGO_GD else 68
    # the north-star fraction on bytes moved: the committed rocprofv3 PMC traffic
    # (FETCH_SIZE x 2 + WRITE_SIZE per launch, profiles/pmc_traffic.json) of one
    # iteration's launches (GS: a column and a row launch; GD: the column
    # launches and the row launch) over the measured iteration time
    pmc_frac = None
    if traffic and all(traffic.get(k) for k in rows):  # (plan-checked above)
        pmc_frac = round(sum(traffic[k] for k in rows) / iter_s / 1e9 / HBM_PEAK_GBS, 4)
    return {"algo": name, "shape": [batch, n, w], "iters": iters, "engine": list(plan_engine),
            "iter_frac_of_hbm_peak_pmc": pmc_frac,
            "holograms_per_s": batch / wall, "iter_ms": iter_s * 1e3, "iter_ms_per_hologram": iter_s * 1e3 / batch,
            "iter_frac_of_hbm_peak_model": round(per_px * batch * n * w / iter_s / 1e9 / HBM_PEAK_GBS, 4),
            "iter_frac_of_hbm_peak_physical": round(phys_iter / iter_s / 1e9 / HBM_PEAK_GBS, 4),
            "kernels": {k: {kk: _round(vv) for kk, vv in v.items()} for k, v in rows.items()}, "dominant": dom,
            "dominant_frac_of_hbm_peak_model": round(rows[dom]["achieved_gbs"] / HBM_PEAK_GBS, 4),
            "dominant_frac_of_hbm_peak_physical": round(rows[dom]["physical_gbs"] / HBM_PEAK_GBS, 4),
            "tiling": info}


def summary(out):
    """The bench line's last object: every measured configuration in a few
    numbers (the driver keeps only the tail of a long line). Per line: us per
    hologram-iteration, holograms/s, the iteration's fraction of 8 TB/s on
    PMC-counted bytes (profiles/pmc_traffic.json) and on the bytes the kernels
    move, and the engine."""
    s = {"value": out["value"], "unit": out["unit"], "gs_iter_us": round(out["gs_iter_ms"] * 1e3, 3),
         "roofline_frac": out["roofline"]["frac"], "roofline_frac_physical": out["roofline"]["frac_physical"],
         "dominant": out["roofline"]["kernel"]}
    lines = {}
    for k, v in out.get("extra", {}).items():
        if isinstance(v, dict) and "iter_ms" in v:
            lines[k] = [round(v["iter_ms_per_hologram"] * 1e3, 2), round(v["holograms_per_s"], 2),
                        v.get("iter_frac_of_hbm_peak_pmc"), v.get("iter_frac_of_hbm_peak_physical"),
                        v["engine"][0]]
    if lines:
        s["lines"] = {"columns": ["us_per_hologram_iter", "holograms_per_s", "frac_pmc", "frac_physical", "engine"],
                      **lines}
    pc = out.get("extra", {}).get("pcie_inclusive")
    if pc:
        s["pcie_inclusive_holograms_per_s"] = round(pc["holograms_per_s"], 2)
    for k in ("cpu_baseline", "cpu_baseline_all_cores", "cpu_baseline_configs0"):
        if k in out:
            s[k] = round(out[k]["value"], 4)
    if "parity" in out:
        s["parity"] = out["parity"]
    return s


def headline_parity(n, iters):
    """SURVEY.md 8c warm-start parity of the timed configuration, measured in
    this run: bench target 0 (the first hologram of every step), the float64
    restatement's phase after 30 cold iterations, `iters` more on the bench's
    plan configuration vs `iters` more of the restatement (oracle/fast_f64.py,
    threaded pocketfft; pinned to the reference goldens by the CPU tests).
    North-star bar 1e-5 rms."""
    from oracle import fast_f64
    from oracle import gs_gd_oracle as orc

    t = targets(0, 1, n)[0]
    t0 = time.perf_counter()
    phi30 = fast_f64.gerchberg_saxton_f64(t, 30)[0].astype(np.float32)
    ref = fast_f64.gerchberg_saxton_f64(t, iters, initial_phase=phi30)[0]
    with _lib.Plan(_lib.ALGO_GS, 1, n, n, _lib.TGT_F32, False, iters) as p:
        p.set_target(t[None])
        p.set_phase(phi30[None])
        p.run(iters)
        ph = p.read(expected=False, stats=False, iters=False)[0][0]
    return {"gs_warm30_plus_iters_phase_rms": float(f"{orc.phase_rms(ph, ref):.3e}"), "bar": 1e-5,
            "target": "bench target 0", "oracle_s": round(time.perf_counter() - t0, 1)}


def north_star(extra):
    """BASELINE.json north_star's bar (>= 60 % of the HBM roofline on the fused
    GS loop at 4096 x 4096, evidenced by rocprof HBM bytes): each 4096^2 line's
    iteration fraction on the PMC-counted bytes (profiles/pmc_traffic.json)
    beside the bar, plus the sec-8(d) model and physical fractions."""
    rows = {}
    for key in ("gs_4096", "gs_4096_batch8"):
        v = extra.get(key)
        if isinstance(v, dict) and "iter_ms" in v:
            rows[key] = {"iter_us_per_hologram": round(v["iter_ms_per_hologram"] * 1e3, 2),
                         "iter_frac_of_hbm_peak_pmc": v.get("iter_frac_of_hbm_peak_pmc"),
                         "iter_frac_of_hbm_peak_model": v.get("iter_frac_of_hbm_peak_model"),
                         "iter_frac_of_hbm_peak_physical": v.get("iter_frac_of_hbm_peak_physical")}
    return {"bar": 0.60, "basis": "iter_frac_of_hbm_peak_pmc (rocprofv3 FETCH_SIZE x 2 + WRITE_SIZE per launch "
                                  "/ iteration time / 8 TB/s)", "shapes": rows}


def main():
    opt = parse()
    if opt.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(opt.gpus))
    rank, world, local_rank = parallel.world()
    if world > 1 and opt.gpus not in (1, world):
        print(f"bench.py: --gpus {opt.gpus} but the launcher started {world} ranks; using {world}", file=sys.stderr)
    group = parallel.Group.from_env()
    if world == 1:
        _lib.init(int(os.environ.get("SLM_DEVICE", "0")))
    else:
        # every rank must have its GPU before any waits in ncclCommInitRank for the
        # others (a rank that failed here would leave the rest blocked in RCCL)
        try:
            _lib.init(local_rank)
            err = None
        except Exception as e:  # noqa: BLE001 -- reported by every rank, then all exit
            err = f"rank {rank}: {e}"
        errs = [e for e in group.all_gather(err) if e]
        if errs:
            print("bench.py: device initialisation failed: " + "; ".join(errs), file=sys.stderr)
            group.close()
            sys.exit(1)
    n, bper, iters = opt.size, opt.batch_per_gpu, opt.iters
    counts = [bper] * world

    if world > 1:
        uid = _lib.comm_unique_id() if rank == 0 else None
        _lib.comm_init(world, rank, group.bcast(uid))

    plan = _lib.Plan(_lib.ALGO_GS, bper, n, n, _lib.TGT_F32, False, iters)
    plan.set_target(targets(rank * bper, bper, n))

    def step():
        plan.run(iters)
        plan.gather_phase(counts, root=0)  # device-side gather, stream-ordered (no host sync per step)

    for _ in range(opt.warmup):
        step()
    plan.sync()
    group.barrier()
    plan.mark(0)  # device-side stopwatch of the timed region (plan stream)
    t0 = time.perf_counter()
    for _ in range(opt.steps):
        step()
    plan.mark(1)
    plan.sync()
    local_elapsed = time.perf_counter() - t0
    group.barrier()
    elapsed = group.max(time.perf_counter() - t0)
    device_step_ms = plan.marked_ms() / opt.steps

    total_holo = bper * world * opt.steps
    value = total_holo / elapsed
    ms_per_step = elapsed / opt.steps * 1e3

    dom, rows, ev_us, _ = kernel_roofline(plan, iters)
    info = plan.info()
    diag = rank_diagnostics(plan, counts, rank, local_elapsed, opt.steps, rows)
    # Kernel time inside the timed region: the per-launch events of the separate
    # timed run, scaled by (device time of one step of the timed region, gather
    # excluded) / (their sum over every launch of that run). Replayed back to back
    # in the graph a kernel runs a few % longer than launched on its own with
    # events; the scaled times are what the timed steps spent per launch (and what
    # rocprofv3's kernel trace of the same steps reports, profiles/rocprof_kernels.json).
    scale = max(device_step_ms - diag["gather_ms"], 1e-9) * 1e3 / float(np.sum(ev_us))
    diag["device_step_ms"] = round(device_step_ms, 4)
    diag["in_graph_scale"] = round(scale, 4)
    for r in rows.values():
        r["event_avg_us"] = r["avg_us"]
        r["avg_us"] = r["event_avg_us"] * scale
        r["achieved_gbs"] = r["model_bytes_per_launch"] / (r["avg_us"] * 1e-6) / 1e9
        r["physical_gbs"] = r["physical_bytes_per_launch"] / (r["avg_us"] * 1e-6) / 1e9
    ranks = group.gather(diag)
    # sanity on rank 0 over EVERY hologram of the job: the gathered phases are
    # finite and each gathered error curve (slm_plan_gather_stats, the
    # error_evolution of src/generate_hologram_sequence.py:19-31) decreases
    gathered = np.empty((bper * world, n, n), np.float32) if rank == 0 else None
    plan.gather_phase(counts, root=0, host_out=gathered)
    stats, _ = plan.gather_stats(counts, root=0, want=rank == 0)
    ok = True
    if rank == 0:
        err = stats[:, :iters, 3]
        ok = bool(np.isfinite(gathered).all() and np.isfinite(err).all() and (err[:, -1] < err[:, 0]).all())
    ok = group.bcast(ok)

    if rank != 0:
        plan.close()
        if world > 1:
            _lib.comm_destroy()
        group.close()
        return

    prec = info["precision"]  # butterflies / twiddles / exchanges; HBM state is complex64
    key = f"gs_{n}x{n}_b{bper}_it{iters}_{prec}"
    traffic = traffic_for_plan(pmc_traffic(key), info)
    dr = rows[dom]
    iter_s = ms_per_step / iters / 1e3
    roofline = {"bound": "hbm", "achieved": round(dr["achieved_gbs"], 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(dr["achieved_gbs"] / HBM_PEAK_GBS, 4),
                "frac_physical": round(dr["physical_gbs"] / HBM_PEAK_GBS, 4),
                "traffic": None if traffic is None else traffic.get(dom),
                "kernel": dom, "avg_us": round(dr["avg_us"], 3), "event_avg_us": round(dr["event_avg_us"], 3),
                "in_graph_scale": diag["in_graph_scale"],
                "bytes_model": "SURVEY.md 8d: GS 68 B/px/iteration = col_main 36 (two column passes 16+16, "
                               "target 4) + row_main 32 (two row passes); achieved = those bytes per launch / "
                               "the launch's duration inside the timed graph replays (HIP-event duration of "
                               "each launch of a separately timed run x the timed region's device time per "
                               "step / those events' sum: in_graph_scale)",
                "bytes_per_launch": dr["model_bytes_per_launch"],
                "physical": {"bytes_per_launch": dr["physical_bytes_per_launch"],
                             "achieved": round(dr["physical_gbs"], 1),
                             "frac_physical": round(dr["physical_gbs"] / HBM_PEAK_GBS, 4),
                             "model": "bytes the fused kernel moves: col_main X 8 + T 4 in, Y 8 out = 20 B/px; "
                                      "row_main Y 8 in, X 8 out = 16 B/px"},
                "iteration": {"us": round(iter_s * 1e6, 3),
                              "frac_model": round(68 * bper * n * n / iter_s / 1e9 / HBM_PEAK_GBS, 4),
                              "frac_physical": round(36 * bper * n * n / iter_s / 1e9 / HBM_PEAK_GBS, 4)},
                "kernels": {k: {kk: _round(vv) for kk, vv in v.items()} for k, v in rows.items()}}
    # measured streaming-copy rates: HBM-sized buffers, and buffers
    # the size of this loop's working set (field X + Y + target), which the
    # 256 MiB Infinity Cache holds between launches
    work = (8 + 8 + 4) * bper * n * n
    copy = {"hbm_1gib_gbs": round(_lib.copy_bandwidth(1 << 30, 10), 1),
            "working_set_gbs": round(_lib.copy_bandwidth(work // 2, 50), 1), "working_set_bytes": work}
    copy["dominant_frac_of_copy_hbm"] = round(dr["achieved_gbs"] / copy["hbm_1gib_gbs"], 4)
    copy["dominant_physical_frac_of_copy_working_set"] = round(dr["physical_gbs"] / copy["working_set_gbs"], 4)
    roofline["measured_copy"] = copy
    prof = rocprof_kernels(key)
    if prof and dom in prof.get("kernels", {}):
        pk = prof["kernels"][dom]
        # the same frac from the committed rocprofv3 trace of this bench: the trace's
        # mean over every launch (almost all of them the timed graph replays), and
        # over the launches of the separately event-timed run beside those events
        roofline["rocprof"] = {"source": prof.get("source"), "avg_us_all": pk.get("avg_us_all"),
                               "avg_us_timed_run": pk.get("avg_us_timed_run"),
                               "event_avg_us_same_run": pk.get("event_avg_us_same_run"),
                               "frac_from_profile": round(dr["model_bytes_per_launch"] / (pk["avg_us_all"] * 1e-6)
                                                          / 1e9 / HBM_PEAK_GBS, 4)
                               if pk.get("avg_us_all") else None}
    out = {
        "metric": METRIC, "value": round(value, 3), "unit": "holograms/s", "n_gpus": world,
        "steps": opt.steps, "warmup": opt.warmup, "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": prec,
        "data": "synthetic (uniform[0,255) float32 targets, default_rng(1234+b))",
        "config": {"workload": f"GS {n}x{n}, {iters} iterations, {bper} hologram(s) per GPU, float32 target, "
                               "uniform incoming intensity, tolerance 0 (BASELINE.json configs[1])",
                   "height": n, "width": n, "iters": iters, "batch_per_gpu": bper, "global_batch": bper * world,
                   "parallelism": f"dp{world} (independent holograms; RCCL gather of phases to rank 0)",
                   "storage": "complex64 field, float32 target/phase", "col_tile": info},
        "gs_iter_ms": round(ms_per_step / iters, 5),
        "roofline": roofline,
        "check": "ok" if ok else "FAILED",
        "ranks": ranks,
    }
    if world == 1 and not opt.no_extra:
        extra = {"pcie_inclusive": pcie_inclusive(plan, targets(0, bper, n), iters)}
        try:  # every line at its BASELINE.json config's own iteration count
            extra["gs_256_it50"] = secondary(256, 1, 50, reps=20)  # configs[0]'s workload on the GPU
            # a 1080 x 1920 SLM panel (13-smooth sides): the complex64 mixed-plan radix kernels
            extra["gs_1080x1920"] = secondary(1080, 1, 200, width=1920, reps=2)
            extra["gs_4096"] = secondary(4096, 1, 200)  # north-star shape, one hologram
            extra["gs_4096_batch8"] = secondary(4096, 8, 200)  # configs[4] per GPU at 8 GPUs
            extra["gs_1024_batch64"] = secondary(1024, 64, 200)  # configs[3] per GPU at 8 GPUs
            extra["gd_1024"] = secondary(1024, 1, 500, algo=_lib.ALGO_GD, reps=2)  # configs[2]
            f64 = _lib.PRECISION_F64  # float64 butterflies (parity margin)
            extra["f64_gs_1024"] = secondary(1024, 1, 200, precision=f64)
            extra["f64_gs_4096"] = secondary(4096, 1, 200, precision=f64)
            # complex128 state and arithmetic ($SLM_ENGINE=float64: the reference's own
            # dtypes on the radix-plan kernels), configs[4]'s and configs[2]'s run lengths
            extra["c128_gs_4096"] = secondary(4096, 1, 200, engine="float64", reps=2)
            extra["c128_gd_1024"] = secondary(1024, 1, 500, algo=_lib.ALGO_GD, engine="float64", reps=2)
        except _lib.SlmError as e:  # pragma: no cover - report, do not hide
            extra["error"] = str(e)
        out["extra"] = extra
        out["north_star"] = north_star(extra)
        try:
            out["parity"] = headline_parity(n, iters)
        except _lib.SlmError as e:  # pragma: no cover - report, do not hide
            out["parity"] = {"error": str(e)}
    if world == 1 and not opt.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(n, iters, opt.cpu_sample_seconds)
        out["cpu_baseline_all_cores"] = cpu_baseline_all_cores(n, iters, opt.cpu_sample_seconds / 2)
        out["cpu_baseline_configs0"] = cpu_baseline_configs0()
    out["summary"] = summary(out)  # last: inside the driver's tail of the line
    print(json.dumps(out), flush=True)
    plan.close()
    if world > 1:
        _lib.comm_destroy()
    group.close()


if __name__ == "__main__":
    main()
