#!/usr/bin/env python3
"""NumPy model of the mixed-E Stockham passes (csrc/radix_c128.hpp mx_from):
pass p holds E_p elements on T_p = N / E_p threads, slot m of thread t is
element t + T_p m, butterfly b = t + k T_p reads elements b + r N / R, the
output goes to (b / Ns) Ns R + j + r Ns; the inverse runs the passes in
reverse order. Checks every mixed plan of csrc/plans.hpp against numpy.fft.

    python tools/mixed_plan_model.py
"""
import re
import os

import numpy as np


def stockham(x, radices, eps, inv):
    n = len(x)
    sign = 1 if inv else -1
    if inv:
        radices, eps = radices[::-1], eps[::-1]
    a = x.astype(complex)
    ns = 1
    for r_, e in zip(radices, eps):
        t_n, nb = n // e, e // r_
        assert e % r_ == 0 and t_n * e == n
        out = np.zeros(n, complex)
        dft = np.exp(sign * 2j * np.pi * np.outer(np.arange(r_), np.arange(r_)) / r_)
        for t in range(t_n):
            for k in range(nb):
                b = t + k * t_n
                j = b % ns
                u = a[b + np.arange(r_) * (n // r_)]
                if ns > 1:
                    u = u * np.exp(sign * 2j * np.pi * j * np.arange(r_) / (ns * r_))
                u = dft @ u
                o = (b // ns) * ns * r_ + j
                out[o + np.arange(r_) * ns] = u
        a = out
        ns *= r_
    return a


def mixed_plans():
    src = open(os.path.join(os.path.dirname(__file__), "..", "spatial_light_modulator_module_amd", "csrc",
                            "plans.hpp")).read()
    for m in re.finditer(r"\{(\d+), (\d+), (\d+), (\d+), \{([\d, ]+)\}, \{([\d, ]+)\}\}", src):
        n, npass = int(m.group(1)), int(m.group(4))
        r = [int(v) for v in m.group(5).split(",")][:npass]
        ep = [int(v) for v in m.group(6).split(",")][:npass]
        yield n, r, ep


def main():
    rng = np.random.default_rng(0)
    worst = 0.0
    for n, r, ep in mixed_plans():
        x = rng.standard_normal(n) + 1j * rng.standard_normal(n)
        ef = np.abs(stockham(x, r, ep, False) - np.fft.fft(x)).max()
        ei = np.abs(stockham(x, r, ep, True) - np.fft.ifft(x) * n).max()
        worst = max(worst, ef, ei)
        print(f"{n:5d} radices {r} elements {ep}: forward {ef:.1e}, inverse {ei:.1e}")
    assert worst < 1e-10


if __name__ == "__main__":
    main()
