"""CPU oracle for the GS / GD hot path — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this module, and only as the checker (or the timed CPU baseline). The product
(spatial_light_modulator_module_amd) never calls it: it has no CPU fallback.

Two restatements of pranislav/Spatial_Light_Modulator_Module src/algorithms.py
(snapshot 2024-10-08):

* ``*_faithful``: float64/complex128 NumPy+SciPy, same operations in the same
  order and with the same dtype flow as the reference (uint8 target ->
  float16 amplitude, complex64 first ifft2, ...), so it reproduces the
  reference bit for bit. Pinned against golden vectors produced by importing
  the reference itself (tests/golden/make_goldens.py); see
  tests/test_oracle_golden.py.
* ``*_c64``: the numerical model of the GPU kernels (complex64 state, z/|z|
  projections, unscaled inverse transforms where scale-free), used to check
  the HIP path step by step at sizes where the reference's chaotic cold start
  (hard parts) makes a float64 comparison meaningless.
"""
from __future__ import annotations

import math
import random

import numpy as np
import scipy.fft as sfft


# ---------------------------------------------------------------------------
# shared pieces
# ---------------------------------------------------------------------------
def incoming_amplitude(shape, incoming_intensity=None):
    """src/algorithms.py:14-19 / :65-70 (the image is passed in, not a path)."""
    intensity = np.ones(shape) if incoming_intensity is None else np.asarray(incoming_intensity)
    return np.sqrt(intensity)


def error_f(actual, correct, norm):
    """src/algorithms.py:161-162."""
    return np.sum((actual - correct) ** 2) / norm


def dEdX_complex(dEdF, x):
    """src/algorithms.py:179-185, applied element-wise (the reference maps it
    over rows; the operations are element-wise so the bits are the same)."""
    rE, iE = dEdF.real, dEdF.imag
    rx, ix = x.real, x.imag
    ax = abs(x)
    re_res = rE * (1 / ax - rx**2 / ax**3) + iE * (-(rx * ix) / ax**3)
    im_res = rE * (-(rx * ix) / ax**3) + iE * (1 / ax - ix**2 / ax**3)
    return re_res + 1j * im_res


def random_unit_draws(seed, count):
    """``random.seed(seed); [random.random() for _ in range(count)]`` —
    NumPy's legacy MT19937 seeded with init_by_array([seed]) yields the same
    53-bit doubles (src/algorithms.py:117-124). Checked in the goldens."""
    return np.random.RandomState([seed]).random_sample(count)


def make_initial_guess(initial_guess_type, incomming_amplitude, demanded_output, seed):
    """src/algorithms.py:115-158 (vectorised; same draw order, row-major)."""
    h, w = demanded_output.shape
    s = h * w
    if initial_guess_type == "random":
        u = random_unit_draws(seed, s)
        return np.exp(1j * 2 * np.pi * u).reshape(h, w)
    if initial_guess_type == "old":
        u = random_unit_draws(seed, 2 * s).reshape(s, 2)
        return (np.sqrt(u[:, 0]) + 1j * np.sqrt(u[:, 1])).reshape(h, w)
    if initial_guess_type == "unnormed":
        u = random_unit_draws(seed, 2 * s).reshape(s, 2)
        return ((u[:, 0] + 1j * u[:, 1]).reshape(h, w) - 0.5) * 2
    if initial_guess_type == "zeros":
        u = random_unit_draws(seed, s)
        return (np.exp(1j * 2 * np.pi * u) / 100).reshape(h, w)
    if initial_guess_type == "ones":
        return np.ones(demanded_output.shape) + 1j * np.zeros(demanded_output.shape)
    if initial_guess_type == "fourier":
        return incomming_amplitude * np.exp(1j * np.angle(sfft.ifft2(np.sqrt(demanded_output))))
    raise ValueError("unknown type of initial guess")


def make_initial_guess_python(initial_guess_type, shape, seed):
    """Pure-Python restatement using the stdlib ``random`` stream exactly as the
    reference does (small shapes only; used to pin random_unit_draws)."""
    h, w = shape
    random.seed(seed)
    if initial_guess_type == "random":
        return np.array([[np.exp(1j * 2 * np.pi * random.random()) for _ in range(w)] for _ in range(h)])
    raise ValueError(initial_guess_type)


def unsettle_schedule(lr, max_loops, unsettle, iterations):
    """Learning rate of each executed iteration and the final value left in
    args.learning_rate (src/algorithms.py:103-104)."""
    rates = np.empty(iterations, dtype=np.float64)
    for i in range(iterations):
        rates[i] = lr
        k = i + 1
        if unsettle and k % int(round(max_loops / (unsettle + 1))) == 0:
            lr *= 2
    return rates, lr


# ---------------------------------------------------------------------------
# faithful float64 restatements
# ---------------------------------------------------------------------------
def gerchberg_saxton_faithful(demanded_output, max_loops, tolerance=0.0, incoming_intensity=None,
                              initial_phase=None):
    """src/algorithms.py:10-49. ``initial_phase`` continues a run whose
    returned hologram was ``initial_phase`` (the loop state is angle(A) only)."""
    incomming_amplitude = incoming_amplitude(demanded_output.shape, incoming_intensity)
    w, l = demanded_output.shape
    demanded_output_amplitude = np.sqrt(demanded_output)
    space_norm = w * l
    norm = np.amax(demanded_output)
    error = tolerance + 1
    error_evolution = []
    i = 0
    expected_outcome = None
    phase = None
    if initial_phase is None:
        A = sfft.ifft2(demanded_output_amplitude)
    else:
        phase = np.asarray(initial_phase)  # keep its dtype: the loop may run in complex64
    while error > tolerance and i < max_loops:
        if phase is None:
            phase = np.angle(A)
        B = incomming_amplitude * np.exp(1j * phase)
        C = sfft.fft2(B)
        D = np.abs(demanded_output_amplitude) * np.exp(1j * np.angle(C))
        A = sfft.ifft2(D)
        phase = None
        expected_outcome = np.abs(C) ** 2
        expected_outcome *= norm / expected_outcome.max()
        error = error_f(expected_outcome, demanded_output, space_norm)
        error_evolution.append(error)
        i += 1
    if expected_outcome is None:
        raise UnboundLocalError("local variable 'expected_outcome' referenced before assignment")
    return np.angle(A), expected_outcome, error_evolution


def gradient_descent_faithful(demanded_output, max_loops, learning_rate, white_attention=1.0, unsettle=0,
                              tolerance=0.0, incoming_intensity=None, initial_guess="random", random_seed=42,
                              initial_field=None):
    """src/algorithms.py:60-112. Returns (hologram, output, error_evolution,
    final learning rate)."""
    incomming_amplitude = incoming_amplitude(demanded_output.shape, incoming_intensity)
    w, l = demanded_output.shape
    space_norm = w * l
    error_evolution = []
    norm = np.amax(demanded_output)
    if initial_field is None:
        x = make_initial_guess(initial_guess, incomming_amplitude, demanded_output, random_seed)
    else:
        x = np.array(initial_field, dtype=np.complex128)
    error = tolerance + 1
    i = 0
    mask = 1 + white_attention * demanded_output / 255
    output = None
    lr = learning_rate
    while error > tolerance and i < max_loops:
        med_output = sfft.fft2(x / abs(x) * incomming_amplitude)
        output_unnormed = abs(med_output) ** 2
        output = output_unnormed * norm / np.amax(output_unnormed)
        dEdF = sfft.ifft2(mask * med_output * (output - demanded_output)) * incomming_amplitude
        dEdX = dEdX_complex(dEdF, x)
        x -= lr * dEdX
        error = error_f(output, demanded_output, space_norm)
        error_evolution.append(error)
        i += 1
        if unsettle and i % int(round(max_loops / (unsettle + 1))) == 0:
            lr *= 2
    if output is None:
        raise UnboundLocalError("local variable 'output' referenced before assignment")
    return np.angle(x), output, error_evolution, lr


# ---------------------------------------------------------------------------
# complex64 models of the GPU kernels
# ---------------------------------------------------------------------------
def _unit(z, a):
    mag = np.abs(z)
    out = np.where(mag > 0, z / np.where(mag > 0, mag, 1), 1).astype(np.complex64)
    return (out * a).astype(np.complex64)


def gerchberg_saxton_c64(demanded_output, loops, incoming_intensity=None, initial_phase=None):
    """GS in complex64 with z/|z| projections (the GPU's arithmetic model).
    Returns (phase float32, |C|^2 of the last iteration, per-iteration
    (max E, sum E^2, sum E T))."""
    t = np.asarray(demanded_output)
    a_t = np.sqrt(t).astype(np.float32)
    a_in = np.sqrt(np.ones(t.shape) if incoming_intensity is None else incoming_intensity).astype(np.float32)
    tf = t.astype(np.float64)
    if initial_phase is None:
        b = _unit(sfft.ifft2(a_t.astype(np.complex64)), a_in)
    else:
        b = (a_in * np.exp(1j * np.asarray(initial_phase, np.float32))).astype(np.complex64)
    stats = []
    e = None
    a = None
    for _ in range(loops):
        c = sfft.fft2(b)
        e = (c.real.astype(np.float32) ** 2 + c.imag.astype(np.float32) ** 2).astype(np.float32)
        ed = e.astype(np.float64)
        stats.append((ed.max(), np.sum(ed * ed), np.sum(ed * tf)))
        a = sfft.ifft2(_unit(c, a_t))
        b = _unit(a, a_in)
    return np.angle(a).astype(np.float32), e, np.array(stats)


def error_from_stats(stats, norm, sum_t2, space_norm):
    """error_f of E * norm / max(E) expanded in the accumulated sums, evaluated
    in the same operation order as the device (kernels.hpp reduce_slab)."""
    stats = np.asarray(stats, dtype=np.float64)
    mx, s2, st = stats[..., 0], stats[..., 1], stats[..., 2]
    with np.errstate(divide="ignore", invalid="ignore"):
        s = norm / mx
        a = (s * s) * s2
        c = (2.0 * s) * st
        return ((a - c) + sum_t2) * (1.0 / space_norm)


# ---------------------------------------------------------------------------
# comparison helpers
# ---------------------------------------------------------------------------
def phase_rms(a, b):
    """rms of the wrapped phase difference (SURVEY.md section 8c protocol)."""
    d = np.angle(np.exp(1j * (np.asarray(a, np.float64) - np.asarray(b, np.float64))))
    return float(math.sqrt(np.mean(d * d)))
