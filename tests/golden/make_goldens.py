"""Generate the golden vectors under tests/golden/ by running the reference.

Run in the build container only (the reference is not present on the GPU box):

    MPLBACKEND=Agg python tests/golden/make_goldens.py [/root/reference/src]

It imports pranislav/Spatial_Light_Modulator_Module's src/algorithms.py from the
given directory, runs gerchberg_saxton / gradient_descent / make_initial_guess
on seeded inputs and stores inputs and outputs as .npz data files. Nothing from
the reference's source is copied into the repository: only the numbers.
"""
from __future__ import annotations

import argparse
import contextlib
import importlib
import io
import os
import random
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))


def ns(**kw):
    base = dict(incomming_intensity="uniform", tolerance=0.0, max_loops=10, gif=False, print_info=False,
                plot_error=False, learning_rate=0.005, white_attention=1.0, unsettle=0, initial_guess="random",
                random_seed=42)
    base.update(kw)
    return argparse.Namespace(**base)


def quiet(fn, *a):
    with contextlib.redirect_stdout(io.StringIO()):
        return fn(*a)


def trap_target(n, seed, count=12, radius=2):
    """Sparse 255-valued dots on black, like src/traps_images.py targets."""
    rng = np.random.default_rng(seed)
    t = np.zeros((n, n), np.uint8)
    yy, xx = np.mgrid[0:n, 0:n]
    for _ in range(count):
        cy, cx = rng.integers(radius, n - radius, 2)
        t[(yy - cy) ** 2 + (xx - cx) ** 2 <= radius * radius] = 255
    return t


def gaussian_intensity_png(path, n):
    from PIL import Image

    yy, xx = np.mgrid[0:n, 0:n]
    r2 = ((yy - n / 2) ** 2 + (xx - n / 2) ** 2) / (0.35 * n) ** 2
    img = np.clip(np.round(255 * np.exp(-r2)), 1, 255).astype(np.uint8)
    Image.fromarray(img).save(path)
    return img


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("ref_src", nargs="?", default="/root/reference/src")
    opt = ap.parse_args()
    sys.path.insert(0, opt.ref_src)
    alg = importlib.import_module("algorithms")

    # G1 / G2: GS warm-start protocol: phi30 and phi230 of one run
    for tag, target in (
        ("g1_gs_u8_256", np.random.default_rng(2024).integers(0, 256, (256, 256)).astype(np.uint8)),
        ("g2_gs_f32_256", np.random.default_rng(2025).uniform(0, 255, (256, 256)).astype(np.float32)),
    ):
        phi30, _, err30 = quiet(alg.gerchberg_saxton, target, ns(max_loops=30))
        phi230, exp230, err230 = quiet(alg.gerchberg_saxton, target, ns(max_loops=230))
        np.savez_compressed(os.path.join(HERE, tag + ".npz"), target=target, phi30=phi30, phi230=phi230,
                            expected230=exp230.astype(np.float32), err230=np.array(err230),
                            err30=np.array(err30))
        print(tag, "final error", err230[-1])

    # G3: sparse trap target, cold start, full outputs (faithful-oracle check)
    t3 = trap_target(128, 3)
    phi, exp3, err3 = quiet(alg.gerchberg_saxton, t3, ns(max_loops=20))
    np.savez_compressed(os.path.join(HERE, "g3_gs_traps_128.npz"), target=t3, phi=phi, expected=exp3,
                        err=np.array(err3))

    # G4 / G5: GD float32 256^2, seed 42, lr 0.005, wa 1 (config 3 recipe, smaller)
    t4 = np.random.default_rng(4242).uniform(0, 255, (256, 256)).astype(np.float32)
    a = ns(max_loops=100, initial_guess="random", random_seed=42)
    phi4, out4, err4 = quiet(alg.gradient_descent, t4, a)
    a5 = ns(max_loops=500, initial_guess="random", random_seed=42)
    phi5, _, err5 = quiet(alg.gradient_descent, t4, a5)
    np.savez_compressed(os.path.join(HERE, "g4_gd_f32_256.npz"), target=t4, phi100=phi4,
                        output100=out4.astype(np.float32), err100=np.array(err4), phi500=phi5.astype(np.float32),
                        err500=np.array(err5))

    # G6: dtype probes
    sq = np.sqrt(np.arange(256, dtype=np.uint8))
    random.seed(42)
    py_draws = np.array([random.random() for _ in range(4096)])
    guess = quiet(alg.make_initial_guess, "random", np.ones((16, 16)), np.zeros((16, 16)), 42)
    guesses = {k: quiet(alg.make_initial_guess, k, np.ones((8, 8)), np.zeros((8, 8)), 7)
               for k in ("old", "unnormed", "zeros", "ones")}
    np.savez_compressed(os.path.join(HERE, "g6_probes.npz"), sqrt_u8=sq, sqrt_u8_dtype=str(sq.dtype),
                        py_random_42=py_draws, guess_random_16=guess,
                        **{f"guess_{k}_8": v for k, v in guesses.items()})

    # G7: edge cases of the control flow
    edges = {}
    try:
        quiet(alg.gerchberg_saxton, t3, ns(max_loops=0))
        edges["gs_zero_loops"] = "none"
    except Exception as e:  # noqa: BLE001
        edges["gs_zero_loops"] = type(e).__name__
    try:
        quiet(alg.gradient_descent, t3.astype(np.float32), ns(max_loops=2, initial_guess="bogus"))
        edges["gd_bad_guess"] = "none"
    except Exception as e:  # noqa: BLE001
        edges["gd_bad_guess"] = type(e).__name__
    zeros = np.zeros((64, 64), np.uint8)
    _, _, errz = quiet(alg.gerchberg_saxton, zeros, ns(max_loops=5))
    a7 = ns(max_loops=4, unsettle=1, learning_rate=0.005)
    quiet(alg.gradient_descent, t3.astype(np.float32)[:64, :64], a7)
    a8 = ns(max_loops=60, tolerance=1e9)
    _, _, err_tol = quiet(alg.gerchberg_saxton, t3, a8)
    np.savez_compressed(os.path.join(HERE, "g7_edges.npz"), gs_zero_loops=edges["gs_zero_loops"],
                        gd_bad_guess=edges["gd_bad_guess"], zeros_target_err=np.array(errz),
                        unsettle_lr_after=a7.learning_rate, tol_hit_err=np.array(err_tol))

    # G8: non-uniform incoming intensity read from a PNG path (src/algorithms.py:14-19)
    png = os.path.join(HERE, "g8_incoming_128.png")
    gaussian_intensity_png(png, 128)
    t8 = trap_target(128, 8, count=20)
    a_rel = os.path.relpath(png)
    phi8a, _, _ = quiet(alg.gerchberg_saxton, t8, ns(max_loops=10, incomming_intensity=png))
    phi8b, exp8, err8 = quiet(alg.gerchberg_saxton, t8, ns(max_loops=40, incomming_intensity=png))
    np.savez_compressed(os.path.join(HERE, "g8_gs_ain_128.npz"), target=t8, phi10=phi8a, phi40=phi8b,
                        expected40=exp8.astype(np.float32), err40=np.array(err8), png=a_rel)

    # G9: GD, "fourier" initial guess, white_attention 2, unsettle 1, uint8 target
    t9 = trap_target(128, 9, count=30, radius=3)
    a9 = ns(max_loops=60, initial_guess="fourier", white_attention=2.0, unsettle=1, learning_rate=0.002)
    phi9, out9, err9 = quiet(alg.gradient_descent, t9, a9)
    np.savez_compressed(os.path.join(HERE, "g9_gd_fourier_u8_128.npz"), target=t9, phi=phi9,
                        output=out9.astype(np.float32), err=np.array(err9), lr_after=a9.learning_rate)
    print("done")


if __name__ == "__main__":
    main()
