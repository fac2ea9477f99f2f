#!/usr/bin/env python3
"""Compare GS runs with column tile widths (SLM_COL_CW) against the default:
per-run determinism and the first iteration at which the phases diverge.
    python tools/diag_cw.py 16 [loops]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from spatial_light_modulator_module_amd import _lib  # noqa: E402


def run(t, phi, loops, cw=None):
    if cw:
        os.environ["SLM_COL_CW"] = str(cw)
    else:
        os.environ.pop("SLM_COL_CW", None)
    with _lib.Plan(_lib.ALGO_GS, t.shape[0], t.shape[1], t.shape[2], _lib.TGT_F32, False, loops) as p:
        p.set_target(t)
        p.set_phase(phi)
        p.run(loops)
        ph, e, st, _ = p.read()
        return ph, e, p.info()


def main():
    cw = int(sys.argv[1])
    loops = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    _lib.init(0)
    t = np.stack([np.random.default_rng(1234 + b).uniform(0, 255, (1024, 1024)).astype(np.float32) for b in range(4)])
    phi = np.random.default_rng(cw).uniform(-np.pi, np.pi, t.shape).astype(np.float32)
    for n in (1, 2, 3, 5, 10, loops):
        ref, eref, i0 = run(t, phi, n)
        outs = [run(t, phi, n, cw) for _ in range(3)]
        same = [np.array_equal(o[0], ref) for o in outs]
        mutual = [np.array_equal(o[0], outs[0][0]) for o in outs]
        d = np.abs(outs[0][0] - ref)
        print(f"loops {n:3d}: == default {same} mutual {mutual} frac diff {np.mean(d > 0):.2e} max {d.max():.2e} "
              f"e== {np.array_equal(outs[0][1], eref)} info {outs[0][2]['col_cw']}/{outs[0][2]['col_threads']}",
              flush=True)


if __name__ == "__main__":
    main()
