"""Drop-in replacement for src/algorithms.py's hot path, running on MI355X.

``gerchberg_saxton(demanded_output, args)`` and
``gradient_descent(demanded_output, args)`` keep the reference signatures
(src/algorithms.py:10, :60), read the same ``args`` attributes, print the same
progress lines, mutate ``args.learning_rate`` the same way, raise the same
exceptions and return the same ``(hologram, expected_outcome,
error_evolution)`` triple (float64 arrays and a list of np.float64). All
iteration arithmetic runs in libslm_hip.so; this module only prepares inputs
(dtype rules, initial guesses) and formats results.

Engines and the cost model (see DESIGN.md sections 1, 3 and 5):

* image sides both in SUPPORTED_LENGTHS (2^k from 64 to 4096, and 768): the
  fused FFT kernels, two launches per iteration, loop state in complex64 in
  HBM; float32 butterflies, twiddles and projections for float32 targets
  (GS 1024^2: ~0.017 ms per iteration), float64 butterflies for uint8 GS
  targets (the CLI's input; ~0.019 ms) -- Plan.set_precision or
  $SLM_PRECISION=f32|f64 overrides. Phases match the float64 reference to
  <= 1e-5 rms under the warm-start protocol of SURVEY.md 8c, not bitwise;
* $SLM_ENGINE=float64 on such sides: the complex128 radix-plan kernels
  (complex128 state, float64 arithmetic, the reference's own dtypes; GS
  4096^2 ~0.5 ms, GD 1024^2 ~0.05 ms per iteration);
* 13-smooth SLM panel sides (600, 800, 1000, 1080, 1152, 1200, 1280, 1536,
  1920, and 2^k / 768 on the other axis): the radix kernels on mixed-E
  Stockham plans -- float32 GS targets in complex64 with the float32 engine's
  numerics (GS 1080 x 1920: ~0.043 ms per iteration), uint8 GS, GD and
  float64 runs in complex128 (GS ~0.061, GD ~0.082 ms);
* any other shape whose sides factor into 2, 3, 5, 7, 11, 13: the float64
  mixed-radix kernels, complex128 state, two launches per iteration (~0.08 ms
  per iteration at 2 Mpixel);
* a side with a larger prime factor (97, 1272 = 8 * 3 * 53, ...): float64
  1-D line transforms along rows and transposed columns, Bluestein's chirp-z
  for that side -- O(N log N), several launches per transform.

A float64 target is carried as float32 on the device, with its max and sum of
squares (the error's constant terms) kept exact in float64.
"""
from __future__ import annotations

import collections
import os
import sys
import warnings

import numpy as np

from . import _lib
from ._lib import ALGO_GD, ALGO_GS, TGT_F32, TGT_U8

# ---------------------------------------------------------------------------
# input preparation (reference dtype rules)
# ---------------------------------------------------------------------------


def _check_shape(t: np.ndarray):
    """Any (h, w), as the reference (src/algorithms.py:20-27): sides in
    SUPPORTED_LENGTHS run the fused FFT kernels, every other shape the
    float64 any-size engine (csrc/generic.hip: mixed-radix kernels for
    13-smooth sides, chirp-z line transforms otherwise)."""
    if t.ndim != 2:
        # the reference unpacks `w, l = demanded_output.shape` (src/algorithms.py:20)
        raise ValueError(f"too many values to unpack (expected 2): target has shape {t.shape}")
    h, w = t.shape
    if h < 1 or w < 1:
        raise ValueError(f"empty target of shape {t.shape}")
    return h, w


def target_for_device(demanded_output) -> tuple[np.ndarray, int]:
    """uint8 targets keep numpy's float16 amplitude rule (sqrt(uint8) -> float16,
    src/algorithms.py:21); everything else is carried as float32."""
    t = np.asarray(demanded_output)
    if t.dtype == np.uint8:
        return np.ascontiguousarray(t), TGT_U8
    return np.ascontiguousarray(t, dtype=np.float32), TGT_F32


def _needs_exact_stats(t) -> bool:
    """True for target dtypes that float32 does not hold exactly (float64, wide integers)."""
    return not (t.dtype in (np.uint8, np.float32, np.float16) or (t.dtype.kind in "iu" and t.dtype.itemsize <= 2))


def _exact_target_stats(plan, t):
    """A target that float32 does not hold exactly (float64, wide integers)
    keeps norm = np.amax(T) (src/algorithms.py:23) and sum T^2 (error_f's
    constant term, :161-162) in float64; the cross term sum E*T uses the
    float32 device copy (relative effect <= 2^-24 per pixel)."""
    if not _needs_exact_stats(t):
        return
    tf = t.astype(np.float64).reshape(plan.batch, -1)
    plan.set_target_stats(tf.max(axis=1), np.einsum("ij,ij->i", tf, tf))


def incoming_amplitude(args, shape) -> np.ndarray | None:
    """sqrt of the incoming intensity (src/algorithms.py:14-19); None = uniform."""
    if args.incomming_intensity == "uniform":
        return None
    from PIL import Image

    intensity = np.array(Image.open(args.incomming_intensity))
    amp = np.sqrt(intensity)
    if amp.shape != tuple(shape):
        raise ValueError(f"operands could not be broadcast together with shapes {amp.shape} {tuple(shape)}")
    return np.ascontiguousarray(amp, dtype=np.float32)


def random_unit_draws(seed, count):
    """The stdlib ``random`` stream of src/algorithms.py:117 (random.seed(seed);
    random.random() ...): NumPy's legacy MT19937 seeded with init_by_array([seed])
    produces the same doubles."""
    return np.random.RandomState([seed]).random_sample(count)


def make_initial_guess(initial_guess_type, incomming_amplitude, demanded_output, seed):
    """Host-side initial guesses of src/algorithms.py:115-158. Returns a complex
    field, or None for "fourier" (computed on the GPU from the target)."""
    h, w = np.asarray(demanded_output).shape
    s = h * w
    if initial_guess_type == "random":
        return np.exp(1j * 2 * np.pi * random_unit_draws(seed, s)).reshape(h, w)
    if initial_guess_type == "old":
        u = random_unit_draws(seed, 2 * s).reshape(s, 2)
        return (np.sqrt(u[:, 0]) + 1j * np.sqrt(u[:, 1])).reshape(h, w)
    if initial_guess_type == "unnormed":
        u = random_unit_draws(seed, 2 * s).reshape(s, 2)
        return ((u[:, 0] + 1j * u[:, 1]).reshape(h, w) - 0.5) * 2
    if initial_guess_type == "zeros":
        return (np.exp(1j * 2 * np.pi * random_unit_draws(seed, s)) / 100).reshape(h, w)
    if initial_guess_type == "ones":
        return np.ones((h, w)) + 1j * np.zeros((h, w))
    if initial_guess_type == "fourier":
        return None
    raise ValueError("unknown type of initial guess")


def learning_rates(lr, max_loops, unsettle):
    """Per-iteration learning rate and the value left in args.learning_rate after
    k iterations (src/algorithms.py:103-104)."""
    rates = np.empty(max(max_loops, 0), dtype=np.float64)
    after = np.empty(max(max_loops, 0) + 1, dtype=np.float64)
    after[0] = lr
    for i in range(max_loops):
        rates[i] = lr
        if unsettle and (i + 1) % int(round(max_loops / (unsettle + 1))) == 0:
            lr *= 2
        after[i + 1] = lr
    return rates, after


# ---------------------------------------------------------------------------
# plan cache
# ---------------------------------------------------------------------------
_PLANS: "collections.OrderedDict[tuple, _lib.Plan]" = collections.OrderedDict()
_MAX_PLANS = int(os.environ.get("SLM_PLAN_CACHE", "4"))


def get_plan(algo, batch, h, w, tgt_type, has_ain, max_loops) -> _lib.Plan:
    key = (algo, batch, h, w, tgt_type, bool(has_ain), max_loops)
    plan = _PLANS.pop(key, None)
    if plan is None:
        while len(_PLANS) >= _MAX_PLANS:
            _PLANS.popitem(last=False)[1].close()
        plan = _lib.Plan(algo, batch, h, w, tgt_type, has_ain, max_loops)
    _PLANS[key] = plan
    return plan


def clear_plans():
    while _PLANS:
        _PLANS.popitem()[1].close()
    _lib.release_caches()  # slm_fft2_c128's per-shape engines (move_traps.update_hologram)


# ---------------------------------------------------------------------------
# batch engine
# ---------------------------------------------------------------------------
def _stop_index(err, tol):
    """first iteration i with not (err_i > tol); None if every test passed."""
    bad = ~(np.asarray(err) > tol)
    return int(np.argmax(bad)) if bad.any() else None


def run_gs(targets, loops, tol=0.0, ain=None, initial_phase=None):
    """GS on a batch [B][H][W] (uint8 or float). Returns phase float32 [B][H][W],
    |C|^2 float32 [B][H][W], errors list per hologram, norm [B], max E used
    for expected_outcome [B]."""
    t = np.asarray(targets)
    tdev, tt = target_for_device(t)
    b, h, w = tdev.shape
    plan = get_plan(ALGO_GS, b, h, w, tt, ain is not None, loops)
    plan.set_target(tdev)
    _exact_target_stats(plan, t)
    if ain is not None:
        plan.set_ain(ain)
    plan.set_phase(initial_phase)
    checked = tol > 0
    plan.run(loops, tol, checked)
    phase, e, stats, iters = plan.read()
    if not checked:
        # speculative unchecked run: recheck "while error > tolerance" on the host;
        # a hologram that should have stopped early is rerun with device checks.
        if any(_stop_index(stats[k, :loops, 3], tol) not in (None, loops - 1) for k in range(b)):
            plan.run(loops, tol, True)
            phase, e, stats, iters = plan.read()
            checked = True
    return _collect(plan, phase, e, stats, iters, loops, checked)


def run_gs_multi(targets, loops, devices, tol=0.0, ain=None):
    """run_gs's contract over several GPUs from this one process
    (slm_gs_multi: contiguous shards, one host thread / plan per device).
    slm_gs_multi takes the error's constant terms from its float32 copy of the
    target, so frames that float32 does not hold exactly (float64, wide
    integers) go through run_gs, which keeps them in float64 (the two paths
    then report the same error_evolution)."""
    t = np.asarray(targets)
    if _needs_exact_stats(t):
        if len(set(int(d) for d in devices)) > 1:
            warnings.warn(f"{t.dtype} targets are not exact in float32: the batch runs on this process's one "
                          f"GPU (run_gs) so the error keeps its float64 terms; `devices` {list(devices)} is "
                          "ignored -- pass uint8 or float32 frames to shard them", RuntimeWarning, stacklevel=2)
        return run_gs(t, loops, tol, ain)
    tdev, _ = target_for_device(t)
    phase, e, stats, iters = _lib.gs_multi(tdev, loops, devices, tol=tol, ain=ain)
    norm = t.reshape(t.shape[0], -1).max(axis=1).astype(np.float64)  # np.amax(demanded_output)
    errs, maxes = [], []
    for k in range(t.shape[0]):
        n = loops if iters[k] < 0 else int(iters[k])
        errs.append([np.float64(v) for v in stats[k, :n, 3]])
        maxes.append(stats[k, n - 1, 0])
    return phase, e, errs, norm, np.array(maxes)


def _collect(plan, phase, e, stats, iters, loops, checked):
    norm, _ = plan.target_stats()
    errs, maxes = [], []
    for k in range(plan.batch):
        n = loops if (not checked or iters[k] < 0) else int(iters[k])
        errs.append([np.float64(v) for v in stats[k, :n, 3]])
        maxes.append(stats[k, n - 1, 0])
    return phase, e, errs, norm, np.array(maxes)


def run_gd(targets, loops, rates, white_attention, tol=0.0, ain=None, initial_field=None, return_field=False):
    t = np.asarray(targets)
    tdev, tt = target_for_device(t)
    b, h, w = tdev.shape
    plan = get_plan(ALGO_GD, b, h, w, tt, ain is not None, loops)
    plan.set_target(tdev)
    _exact_target_stats(plan, t)
    if ain is not None:
        plan.set_ain(ain)
    plan.set_field(initial_field)
    plan.set_lr(np.asarray(rates, np.float32)[:loops])
    checked = tol > 0
    plan.run(loops, tol, checked, white_attention)
    phase, e, stats, iters = plan.read()
    if not checked:
        if any(_stop_index(stats[k, :loops, 3], tol) not in (None, loops - 1) for k in range(b)):
            plan.run(loops, tol, True, white_attention)
            phase, e, stats, iters = plan.read()
            checked = True
    out = _collect(plan, phase, e, stats, iters, loops, checked)
    return out + (plan.read_field(),) if return_field else out


def hologram_from(phase):
    """float32 device phase -> float64 hologram in np.angle's range [-pi, pi]
    (float32(pi) rounds above pi; the clip moves such values by < 1e-7)."""
    return np.clip(phase.astype(np.float64), -np.pi, np.pi)


def expected_from(e, norm, emax):
    """expected_outcome = |C|^2 * norm / max|C|^2 in float64 (src/algorithms.py:36-37)."""
    out = e.astype(np.float64)
    out *= norm / np.float64(emax)
    return out


# ---------------------------------------------------------------------------
# reference-compatible entry points
# ---------------------------------------------------------------------------
def _print_loops(n, max_loops):
    sys.stdout.write("".join(f"\rloop {i}/{max_loops}" for i in range(1, n + 1)))
    print()


def printout(error, loop_num, error_evol, plot_error):
    """src/algorithms.py:165-172."""
    print(f"error: {error}")
    print(f"number of loops: {loop_num}")
    if plot_error:
        import matplotlib.pyplot as plt

        plt.plot(error_evol)
        plt.xlabel("loop number")
        plt.ylabel("error")
        plt.show()


def _iterations_allowed(args):
    # `while error > args.tolerance and i < args.max_loops` with error = tol + 1
    tol = args.tolerance
    return args.max_loops > 0 and (tol + 1) > tol


def _gif_frame(args, kind, phase, expected, i):
    """add_gif_image (src/algorithms.py:52-57) for GS; the GD frame of
    src/algorithms.py:94-101 (complex_to_real_phase of x/|x|, :175-176) when
    `phase` is the GD field."""
    from PIL import Image

    if args.gif_type == "h":
        if kind == "gd":
            ang = np.angle(phase.astype(np.complex128))
        else:
            ang = hologram_from(phase)
        img = Image.fromarray((ang + np.pi) * args.correspond_to2pi / (2 * np.pi)
                              if kind == "gs" else (ang + np.pi) / (2 * np.pi) * args.correspond_to2pi)
    elif args.gif_type == "i":
        img = Image.fromarray(expected)
    else:
        return
    img.convert("L").save(f"{args.gif_source_dir}/{i // args.gif_skip}.png")


def gerchberg_saxton(demanded_output, args):
    """Classical Gerchberg-Saxton (far field) on the GPU; drop-in for
    src/algorithms.py:10-49."""
    t = np.asarray(demanded_output)
    h, w = _check_shape(t)
    ain = incoming_amplitude(args, t.shape)
    tol = args.tolerance
    if not _iterations_allowed(args):
        print()
        if args.print_info:
            print()
            printout(tol + 1, 0, [], args.plot_error)
        raise UnboundLocalError("local variable 'expected_outcome' referenced before assignment")
    if args.gif:
        return _gerchberg_saxton_gif(t, args, ain)
    phase, e, errs, norm, emax = run_gs(t[None], args.max_loops, tol, ain)
    error_evolution = errs[0]
    n = len(error_evolution)
    _print_loops(n, args.max_loops)
    if args.print_info:
        print()
        printout(error_evolution[-1], n, error_evolution, args.plot_error)
    hologram = hologram_from(phase[0])
    expected_outcome = expected_from(e[0], norm[0], emax[0])
    return hologram, expected_outcome, error_evolution


def _gerchberg_saxton_gif(t, args, ain):
    """GIF frames need intermediate states: run in warm-started chunks that end
    on every frame iteration (the GS state is angle(A) only)."""
    loops, tol, skip = args.max_loops, args.tolerance, args.gif_skip
    phase = None
    error_evolution = []
    i = 0
    while i < loops:
        step = 1 if i % skip == 0 else min(skip - i % skip, loops - i)
        ph, e, errs, norm, emax = run_gs(t[None], step, tol, ain, initial_phase=phase)
        error_evolution += errs[0]
        phase = ph
        i += len(errs[0])
        expected = expected_from(e[0], norm[0], emax[0])
        if (i - 1) % skip == 0:
            _gif_frame(args, "gs", ph[0], expected, i - 1)
        if len(errs[0]) < step or not (error_evolution[-1] > tol):
            break
    _print_loops(len(error_evolution), loops)
    if args.print_info:
        print()
        printout(error_evolution[-1], len(error_evolution), error_evolution, args.plot_error)
    return hologram_from(phase[0]), expected, error_evolution


def gradient_descent(demanded_output, args):
    """Gradient descent on the unconstrained complex field (far field) on the
    GPU; drop-in for src/algorithms.py:60-112."""
    t = np.asarray(demanded_output)
    h, w = _check_shape(t)
    ain = incoming_amplitude(args, t.shape)
    amp_host = np.ones(t.shape) if ain is None else ain.astype(np.float64)
    field = make_initial_guess(args.initial_guess, amp_host, t, args.random_seed)
    tol = args.tolerance
    if args.print_info:
        print("computing hologram")
    if not _iterations_allowed(args):
        print()
        if args.print_info:
            print()
            printout(tol + 1, 0, [], args.plot_error)
        raise UnboundLocalError("local variable 'output' referenced before assignment")
    if args.unsettle and int(round(args.max_loops / (args.unsettle + 1))) == 0:
        raise ZeroDivisionError("integer division or modulo by zero")
    rates, after = learning_rates(args.learning_rate, args.max_loops, args.unsettle)
    if args.gif:
        return _gradient_descent_gif(t, args, ain, field, rates, after)
    phase, e, errs, norm, emax = run_gd(t[None], args.max_loops, rates, float(args.white_attention), tol, ain,
                                        None if field is None else field[None])
    error_evolution = errs[0]
    n = len(error_evolution)
    args.learning_rate = float(after[n]) if args.unsettle else args.learning_rate
    _print_loops(n, args.max_loops)
    if args.print_info:
        print()
        printout(error_evolution[-1], n, error_evolution, args.plot_error)
    hologram = hologram_from(phase[0])
    output = expected_from(e[0], norm[0], emax[0])
    return hologram, output, error_evolution


def _gradient_descent_gif(t, args, ain, field, rates, after):
    """GD with GIF frames (src/algorithms.py:94-101): warm-started chunks that
    end on every frame iteration; the GD state is the complex field x, read
    back after each chunk (slm_plan_read_field) and handed to the next with the
    matching slice of the learning-rate schedule."""
    loops, tol, skip = args.max_loops, args.tolerance, args.gif_skip
    error_evolution = []
    i = 0
    x = None if field is None else field[None]
    while i < loops:
        step = 1 if i % skip == 0 else min(skip - i % skip, loops - i)
        ph, e, errs, norm, emax, xf = run_gd(t[None], step, rates[i:i + step], float(args.white_attention), tol,
                                             ain, x, return_field=True)
        x = xf
        error_evolution += errs[0]
        i += len(errs[0])
        output = expected_from(e[0], norm[0], emax[0])
        if (i - 1) % skip == 0:
            _gif_frame(args, "gd", xf[0], output, i - 1)
        if len(errs[0]) < step or not (error_evolution[-1] > tol):
            break
    n = len(error_evolution)
    args.learning_rate = float(after[n]) if args.unsettle else args.learning_rate
    _print_loops(n, loops)
    if args.print_info:
        print()
        printout(error_evolution[-1], n, error_evolution, args.plot_error)
    return hologram_from(ph[0]), output, error_evolution
