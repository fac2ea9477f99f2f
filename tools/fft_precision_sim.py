#!/usr/bin/env python3
"""CPU emulation of the GPU transforms' rounding, to choose an arithmetic
scheme before writing kernels: a Stockham FFT with a given radix plan where
each piece (butterfly adds, constant twiddles, pass twiddles, projections) runs
in float32 or float64 and the state is rounded to complex64 between passes.
Measures the SURVEY.md 8c warm-start GS parity (phi30 -> +iters vs the float64
oracle) for each scheme.

    python tools/fft_precision_sim.py --n 256 --iters 200 --schemes f64,f32,f32tw
"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import gs_gd_oracle as orc  # noqa: E402

PLANS = {256: (16, 16), 512: (16, 2, 16), 1024: (16, 4, 16), 2048: (16, 8, 16), 4096: (8, 8, 8, 8)}


def c64(z):
    return z.astype(np.complex64)


class Scheme:
    def __init__(self, name):
        self.name = name
        # dft: dtype of butterfly adds and constant twiddles; tw: pass-twiddle product
        self.dft = np.complex128 if name in ("f64",) else np.complex64
        self.tw = {"f64": "exact", "f32": "f32", "f32tw": "exact", "f32twsplit": "split", "f32allexact": "exact"}[name]
        self.const_exact = name == "f32allexact"
        self.proj = np.complex128 if name == "f64" else np.complex64

    def dft_r(self, u, inv):
        """Radix-2 DIT DFT over axis -2 (length R), in self.dft arithmetic."""
        R = u.shape[-2]
        if R == 1:
            return u
        ev = self.dft_r(u[..., 0::2, :], inv)
        od = self.dft_r(u[..., 1::2, :], inv)
        k = np.arange(R // 2)
        w = np.exp((2j if inv else -2j) * np.pi * k / R)[:, None]
        if self.const_exact:
            t = (od.astype(np.complex128) * w).astype(self.dft)
        else:
            t = (od * w.astype(self.dft)).astype(self.dft)
        return np.concatenate([ev + t, ev - t], axis=-2).astype(self.dft)

    def twiddle(self, u, w):
        if self.tw == "f32":
            return (u.astype(np.complex64) * w.astype(np.complex64)).astype(self.dft)
        if self.tw == "exact":
            return (u.astype(np.complex128) * w).astype(self.dft)
        # split: w = hi + lo in float32, product accumulated in float32 with the lo term
        hi = w.astype(np.complex64)
        lo = (w - hi).astype(np.complex64)
        u = u.astype(np.complex64)
        return (u * hi + u * lo).astype(self.dft)


def stockham(x, plan, inv, sch):
    """Transform along the last axis; state rounded to complex64 between passes."""
    N = x.shape[-1]
    ns = 1
    x = c64(x)
    for R in plan:
        nb = N // R
        b = np.arange(nb)
        u = np.stack([x[..., b + r * nb] for r in range(R)], axis=-2).astype(sch.dft)  # (..., R, nb)
        if ns > 1:
            j = b % ns
            r = np.arange(R)[:, None]
            w = np.exp((2j if inv else -2j) * np.pi * r * j[None, :] / (ns * R))
            u = sch.twiddle(u, w)
        u = sch.dft_r(u, inv)
        out = np.empty(x.shape, np.complex128)
        o = (b // ns) * ns * R + (b % ns)
        for r in range(R):
            out[..., o + r * ns] = u[..., r, :]
        x = c64(out)
        ns *= R
    return x


def fft2(x, inv, sch):
    """rows (the row kernel's transforms) with sch.rows, columns with sch.cols"""
    plan = PLANS[x.shape[-1]]
    y = stockham(x, plan, inv, sch.rows)
    y = np.swapaxes(stockham(np.swapaxes(y, -1, -2), PLANS[x.shape[-2]], inv, sch.cols), -1, -2)
    return y


class Hybrid:
    """per-axis schemes: "rowsA+colsB" (e.g. f32+f64: float64 butterflies in the
    column kernel only)"""
    def __init__(self, name):
        r, c = name.split("+") if "+" in name else (name, name)
        self.name = name
        self.rows, self.cols = Scheme(r), Scheme(c)
        self.proj = np.complex128 if (r == "f64" and c == "f64") else np.complex64


def gs(t, phi0, iters, sch):
    aT = np.sqrt(t.astype(np.float64))
    B = c64(np.exp(1j * phi0.astype(np.float64)))
    for _ in range(iters):
        C = fft2(B, False, sch).astype(sch.proj)
        D = c64(aT * C / np.abs(C))
        A = fft2(D, True, sch).astype(sch.proj)
        B = c64(A / np.abs(A))
    return np.angle(A.astype(np.complex128))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=256)
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--warm", type=int, default=30)
    ap.add_argument("--schemes", default="f64,f32,f32tw,f32twsplit")
    ap.add_argument("--u8", action="store_true")
    ap.add_argument("--seed", type=int, default=2024)
    o = ap.parse_args()
    rng = np.random.default_rng(o.seed)
    n = o.n
    t = rng.integers(0, 256, (n, n)).astype(np.uint8) if o.u8 else rng.uniform(0, 255, (n, n)).astype(np.float32)
    phi_w, _, _ = orc.gerchberg_saxton_faithful(t, o.warm)
    ref, _, _ = orc.gerchberg_saxton_faithful(t, o.iters, initial_phase=phi_w)
    tt = t.astype(np.float32)
    if o.u8:  # the reference's float16 amplitude
        tt = (np.sqrt(t).astype(np.float16).astype(np.float64)) ** 2
    for s in o.schemes.split(","):
        ph = gs(tt, phi_w, o.iters, Hybrid(s))
        print(f"n={n} seed={o.seed} {s:>10s}: phase rms {orc.phase_rms(ph, ref):.3e}", flush=True)


if __name__ == "__main__":
    main()
