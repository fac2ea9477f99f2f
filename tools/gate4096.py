#!/usr/bin/env python3
"""4096^2 warm-start precision survey over several targets and library builds.

    python tools/gate4096.py --targets 0,1,2,3 [--libs default,<variant>...] [--plans default,wide]
                             [--spans 50,100] [--batch8]

For each bench target k (default_rng(1234 + k)) the float64
oracle (oracle/fast_f64.py) runs 30 cold iterations, then `max(spans)` warm
iterations with snapshots at every span; each library build (default = the
in-tree libslm_hip.so, else lib/libslm_hip_<name>.so) and each forced radix
plan (--plans: $SLM_PLAN for the child, `default` = the library's pick) then runs the same warm
starts on the GPU at float32 and float64 butterflies, in a child process per
build, and the wrapped phase rms against the oracle is printed per (target,
build, precision, span). --batch8 also runs the configs[4] per-GPU batch
(8 x 4096^2) once per build and reports holograms 0 and 7 against the single
runs (bitwise) and the oracle. Oracle arrays stay under $TMPDIR.
"""
import argparse
import json
import os
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
N = 4096


def bench_target(k):
    return np.random.default_rng(1234 + k).uniform(0, 255, (N, N)).astype(np.float32)


def oracle(k, spans, tmp):
    from oracle import fast_f64

    t = bench_target(k)
    t0 = time.perf_counter()
    phi30, _, _ = fast_f64.gerchberg_saxton_f64(t, 30)
    phi30 = phi30.astype(np.float32)
    snaps = {s: None for s in spans}
    last, _, err = fast_f64.gerchberg_saxton_f64(t, max(spans), initial_phase=phi30, snapshots=snaps)
    snaps[max(spans)] = last
    np.save(os.path.join(tmp, f"phi30_{k}.npy"), phi30)
    for s, ph in snaps.items():
        np.save(os.path.join(tmp, f"ref_{k}_{s}.npy"), ph)
    np.save(os.path.join(tmp, f"err_{k}.npy"), np.asarray(err))
    print(f"oracle target {k}: {time.perf_counter() - t0:.0f} s", flush=True)


def child(args):
    """GPU side for one build (SLM_LIB_PATH set by the parent)."""
    from oracle import gs_gd_oracle as orc
    from spatial_light_modulator_module_amd import _lib

    _lib.init(0)
    spans = [int(s) for s in args.spans.split(",")]
    res = {}
    for k in [int(v) for v in args.targets.split(",")]:
        t = bench_target(k)
        phi30 = np.load(os.path.join(args.tmp, f"phi30_{k}.npy"))
        err = np.load(os.path.join(args.tmp, f"err_{k}.npy"))
        for prec in ("f32", "f64"):
            for span in spans:
                with _lib.Plan(_lib.ALGO_GS, 1, N, N, _lib.TGT_F32, False, span) as p:
                    p.set_precision(_lib.PRECISION_F32 if prec == "f32" else _lib.PRECISION_F64)
                    p.set_target(t[None])
                    p.set_phase(phi30[None])
                    p.run(span)
                    ph, _, st, _ = p.read(expected=False)
                ref = np.load(os.path.join(args.tmp, f"ref_{k}_{span}.npy"))
                rms = orc.phase_rms(ph[0], ref)
                erel = float(np.max(np.abs(st[0, :span, 3] / err[:span] - 1)))
                res[f"{k}/{prec}/{span}"] = (rms, erel)
                print(f"  target {k} {prec} +{span}: phase rms {rms:.3e}  err rel {erel:.1e}", flush=True)
                if prec == "f32" and span == max(spans):
                    np.save(os.path.join(args.tmp, f"gpu_{args.name}_{k}.npy"), ph[0])
    if args.batch8:
        ks = [int(v) for v in args.targets.split(",")]
        span = max(spans)
        phis = np.stack([np.load(os.path.join(args.tmp, f"phi30_{k}.npy")) if k in ks else
                         np.zeros((N, N), np.float32) for k in range(8)])
        with _lib.Plan(_lib.ALGO_GS, 8, N, N, _lib.TGT_F32, False, span) as p:
            info = p.info()
            p.set_target(np.stack([bench_target(k) for k in range(8)]))
            p.set_phase(phis)
            p.run(span)
            ph, _, st, _ = p.read(expected=False)
        print(f"  batch8 plan {info}", flush=True)
        for k in ks:
            single = np.load(os.path.join(args.tmp, f"gpu_{args.name}_{k}.npy"))
            same = bool(np.array_equal(single, ph[k]))
            ref = np.load(os.path.join(args.tmp, f"ref_{k}_{span}.npy"))
            print(f"  batch8 hologram {k}: bitwise == single {same}, phase rms {orc.phase_rms(ph[k], ref):.3e}",
                  flush=True)
    print("RESULT " + json.dumps({"lib": args.name, "res": res}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--targets", default="0,1,2")
    ap.add_argument("--libs", default="default")
    ap.add_argument("--plans", default="default")
    ap.add_argument("--spans", default="50,100")
    ap.add_argument("--batch8", action="store_true")
    ap.add_argument("--child", action="store_true")
    ap.add_argument("--tmp")
    ap.add_argument("--name", default="default")
    args = ap.parse_args()
    if args.child:
        return child(args)
    tmp = tempfile.mkdtemp(prefix="gate4096_")
    spans = [int(s) for s in args.spans.split(",")]
    for k in [int(v) for v in args.targets.split(",")]:
        oracle(k, spans, tmp)
    rc = 0
    for name in args.libs.split(","):
        lib = os.path.join(ROOT, "spatial_light_modulator_module_amd", "lib",
                           "libslm_hip.so" if name == "default" else f"libslm_hip_{name}.so")
        for plan in args.plans.split(","):
            tag = name if plan == "default" else f"{name}_{plan}"
            print(f"== build {name}, plan {plan}", flush=True)
            cmd = [sys.executable, os.path.abspath(__file__), "--child", "--tmp", tmp, "--name", tag,
                   "--targets", args.targets, "--spans", args.spans] + (["--batch8"] if args.batch8 else [])
            env = dict(os.environ, SLM_LIB_PATH=lib)
            env.pop("SLM_PLAN", None)
            if plan != "default":
                env["SLM_PLAN"] = plan
            rc = max(rc, subprocess.call(cmd, env=env))
    return rc


if __name__ == "__main__":
    sys.exit(main())
