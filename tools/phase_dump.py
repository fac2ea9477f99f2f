#!/usr/bin/env python3
"""Run GS on a fixed synthetic target with the library $SLM_LIB_PATH selects and
save the phases, for bitwise A/B checks between builds that must not change the
arithmetic (layouts, access order, register budgets).

    python tools/phase_dump.py <n> <batch> <iters> <out.sha>
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from spatial_light_modulator_module_amd import _lib  # noqa: E402


def main():
    n, b, iters, out = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
    _lib.init(0)
    t = np.random.default_rng(7).uniform(0, 255, (b, n, n)).astype(np.float32)
    with _lib.Plan(_lib.ALGO_GS, b, n, n, _lib.TGT_F32, False, iters) as p:
        p.set_target(t)
        p.set_phase(None)
        p.run(iters, 0.0, False)
        ph, e, stats, _ = p.read()
        print(f"{os.path.basename(_lib.LIB_PATH)} {n}x{n}x{b}: engine {p.engine()} info {p.info()}")
    # a digest, not the array (a 4096^2 batch is 128 MiB; gpurun_out copies back <= 64 MiB)
    import hashlib
    with open(out, "w") as f:
        f.write(hashlib.sha256(np.ascontiguousarray(ph).tobytes()).hexdigest() + "\n")


if __name__ == "__main__":
    main()
