"""Multi-threaded float64 restatements of the GS / GD loops — TEST INFRASTRUCTURE ONLY.

Same rule as oracle/gs_gd_oracle.py: only tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg may use this module, only as the checker.

The faithful restatements (gs_gd_oracle.*_faithful) repeat the reference's
operations one by one (np.angle, np.exp, the dEdX_complex expression of
src/algorithms.py:179-185) on one core; at 4096^2 that is ~3 s per GS
iteration, too slow to gate 100 iterations in the GPU suite. These versions
keep complex128/float64 throughout but use the algebraically equal forms

    a * exp(1j * angle(z)) == a * z / |z|          (angle(0) = 0 -> a)
    dEdX_complex(g, x)     == (g - x Re(conj(x) g) / |x|^2) / |x|

(the z/|z| restatement reproduces the reference to 4e-15..2e-14
rms), run pocketfft with `workers` threads and split every element-wise step
over row blocks in a thread pool (NumPy releases the GIL inside ufuncs). They
are pinned to the faithful restatements and the reference goldens in
tests/test_oracle_golden.py.

    GS: src/algorithms.py:10-49    GD: src/algorithms.py:60-112
"""
from __future__ import annotations

import os
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import scipy.fft as sfft

# the GPU box gives one process a 16-CPU share (os.cpu_count() shows the whole machine)
DEFAULT_WORKERS = int(os.environ.get("SLM_ORACLE_WORKERS", "0")) or min(16, os.cpu_count() or 1)


class _Pool:
    """Row-block parallel map over equally shaped 2-D arrays."""

    def __init__(self, workers):
        self.workers = max(1, int(workers))
        self.ex = ThreadPoolExecutor(self.workers) if self.workers > 1 else None

    def run(self, fn, rows):
        if self.ex is None or rows < 64:
            return [fn(slice(0, rows))]
        step = -(-rows // self.workers)
        futs = [self.ex.submit(fn, slice(r, min(rows, r + step))) for r in range(0, rows, step)]
        return [f.result() for f in futs]

    def close(self):
        if self.ex is not None:
            self.ex.shutdown()


def _unit_into(out, z, a, s):
    """out[s] = a * z / |z| with 0 -> a (np.angle(0) == 0)."""
    zz = z[s]
    mag = np.abs(zz)
    zero = mag == 0
    np.divide(zz, np.where(zero, 1.0, mag), out=out[s])
    out[s][zero] = 1.0
    out[s] *= a if np.ndim(a) == 0 else a[s]


def gerchberg_saxton_f64(demanded_output, loops, initial_phase=None, incoming_intensity=None, tolerance=0.0,
                         workers=None, snapshots=None):
    """src/algorithms.py:10-49 in complex128 with z/|z| projections.

    ``initial_phase`` continues a run whose returned hologram was
    ``initial_phase`` (the GS loop state is angle(A) only). The incoming
    amplitude is float64 here (a uint8 intensity image makes the reference's
    amplitude float16 and its loop complex64: the faithful restatement). Returns
    (angle(A) float64, expected_outcome float64, error_evolution list).
    ``snapshots``: a dict whose keys are iteration counts < ``loops``; each is
    filled with angle(A) after that many iterations (what a run of that length
    would return), so one oracle run serves several gates."""
    pool = _Pool(workers or DEFAULT_WORKERS)
    try:
        t = np.asarray(demanded_output)
        h, w = t.shape
        a_t = np.sqrt(t)  # float16 for uint8 targets, as the reference
        a_t64 = a_t.astype(np.float64)
        a_in = 1.0 if incoming_intensity is None else np.sqrt(np.asarray(incoming_intensity, np.float64))
        norm = np.amax(t)
        tf = t.astype(np.float64)
        b = np.empty((h, w), np.complex128)
        if initial_phase is None:
            a = sfft.ifft2(a_t, workers=pool.workers)  # complex64 for f16/f32 amplitudes, as the reference
            a = a.astype(np.complex128)
        else:
            ph = np.asarray(initial_phase)  # keep its dtype: exp(1j * phi) of a float32 phase is complex64
            pool.run(lambda s: np.multiply(np.exp(1j * ph[s]), a_in if np.ndim(a_in) == 0 else a_in[s],
                                           out=b[s]), h)
            a = None
        err_evol = []
        expected = np.empty((h, w), np.float64)
        error = tolerance + 1
        i = 0
        while error > tolerance and i < loops:
            if a is not None:
                pool.run(lambda s: _unit_into(b, a, a_in, s), h)
            c = sfft.fft2(b, workers=pool.workers)
            pool.run(lambda s: np.square(np.abs(c[s]), out=expected[s]), h)
            emax = np.float64(max(pool.run(lambda s: float(expected[s].max()), h)))
            scale = norm / emax  # float64, as norm / expected_outcome.max() (np.float64)
            d = b  # B is dead once C exists
            pool.run(lambda s: _unit_into(d, c, a_t64, s), h)
            a = sfft.ifft2(d, workers=pool.workers)

            def err_part(s):
                e = expected[s]
                e *= scale
                return float(np.sum((e - tf[s]) ** 2))

            error = sum(pool.run(err_part, h)) / (h * w)
            err_evol.append(np.float64(error))
            i += 1
            if snapshots is not None and i in snapshots and i < loops:
                snapshots[i] = np.angle(a)
        return np.angle(a), expected, err_evol
    finally:
        pool.close()


def gradient_descent_f64(demanded_output, loops, learning_rates, white_attention=1.0, initial_field=None,
                         incoming_intensity=None, tolerance=0.0, workers=None):
    """src/algorithms.py:60-112 in complex128 with the closed-form projection.

    ``learning_rates``: one value per iteration (the unsettle schedule,
    src/algorithms.py:103-104). Returns (angle(x), output, error_evolution,
    x) so a run can be continued."""
    pool = _Pool(workers or DEFAULT_WORKERS)
    try:
        t = np.asarray(demanded_output)
        h, w = t.shape
        tf = t.astype(np.float64)
        a_in = 1.0 if incoming_intensity is None else np.sqrt(np.asarray(incoming_intensity, np.float64))
        norm = np.amax(t)
        mask = 1 + white_attention * t / 255
        x = np.array(initial_field, dtype=np.complex128)
        u = np.empty_like(x)
        out = np.empty((h, w), np.float64)
        err_evol = []
        error = tolerance + 1
        i = 0
        rates = np.broadcast_to(np.asarray(learning_rates, np.float64), (loops,))
        while error > tolerance and i < loops:
            def fwd_in(s):
                np.divide(x[s], np.abs(x[s]), out=u[s])
                u[s] *= a_in if np.ndim(a_in) == 0 else a_in[s]

            pool.run(fwd_in, h)
            f = sfft.fft2(u, workers=pool.workers)
            pool.run(lambda s: np.square(np.abs(f[s]), out=out[s]), h)
            pmax = np.float64(max(pool.run(lambda s: float(out[s].max()), h)))

            def grad_in(s):
                o = out[s]
                o *= norm / pmax
                f[s] *= mask[s] * (o - tf[s])
                return float(np.sum((o - tf[s]) ** 2))

            error = sum(pool.run(grad_in, h)) / (h * w)
            g = sfft.ifft2(f, workers=pool.workers)
            lr = float(rates[i])

            def update(s):
                gs = g[s] * (a_in if np.ndim(a_in) == 0 else a_in[s])
                xs = x[s]
                ax2 = xs.real * xs.real + xs.imag * xs.imag
                re = xs.real * gs.real + xs.imag * gs.imag
                ax = np.sqrt(ax2)
                xs -= lr * ((gs - xs * (re / ax2)) / ax)

            pool.run(update, h)
            err_evol.append(np.float64(error))
            i += 1
        return np.angle(x), out, err_evol, x
    finally:
        pool.close()
