"""Multi-hologram data paths on one GPU box.

* slm_gs_multi: one process cuts the batch into contiguous
  shards, one plan / host thread / stream per shard; devices may repeat, so
  the shard and slice arithmetic runs here on the box's single GPU. Results
  must equal one slm_gs over the whole batch bit for bit (holograms are
  independent; 256^2 keeps every shard on the same kernels) -- the batch loop
  of src/generate_hologram_sequence.py:19-31 as one call.
* slm_plan_gather_stats: the per-iteration statistics (error_evolution) travel
  with the phases; at N = 1 the gather is the local copy into the root's slab.
"""
import numpy as np
import pytest

from oracle import gs_gd_oracle as orc


def _targets(b, n, u8):
    rng = np.random.default_rng(77 + b)
    if u8:
        return rng.integers(0, 256, (b, n, n)).astype(np.uint8)
    return rng.uniform(0, 255, (b, n, n)).astype(np.float32)


def _whole_batch(lib, t, loops, tol=0.0):
    tt = lib.TGT_U8 if t.dtype == np.uint8 else lib.TGT_F32
    b, h, w = t.shape
    with lib.Plan(lib.ALGO_GS, b, h, w, tt, False, loops) as p:
        p.set_target(t)
        p.run(loops, tol, tol > 0)
        return p.read()


@pytest.mark.gpu
@pytest.mark.parametrize("u8", [False, True])
@pytest.mark.parametrize("shards", [1, 2, 3, 7])
def test_gs_multi_equals_one_batch(gpu, u8, shards):
    lib = gpu
    t = _targets(5, 256, u8)
    loops = 12
    ph, e, st, it = lib.gs_multi(t, loops, [0] * shards)  # 7 shards of a 5-batch: two are empty
    rph, re, rst, rit = _whole_batch(lib, t, loops)
    np.testing.assert_array_equal(ph, rph)
    np.testing.assert_array_equal(e, re)
    np.testing.assert_array_equal(st, rst)
    np.testing.assert_array_equal(it, rit)
    # a cold start is chaotic at rounding level: the oracle gates the first errors only
    ref, _, err = orc.gerchberg_saxton_faithful(t[4], 2)
    np.testing.assert_allclose(st[4, :2, 3], err, rtol=1e-5)


@pytest.mark.gpu
def test_gs_multi_tolerance_and_errors(gpu):
    lib = gpu
    t = _targets(4, 128, False)
    loops = 20
    _, _, st, _ = _whole_batch(lib, t, loops)
    tol = float(np.sqrt(st[2, 6, 3] * st[2, 7, 3]))  # hologram 2 stops after iteration 8
    ph, e, st2, it = lib.gs_multi(t, loops, [0, 0], tol=tol)
    rph, re, rst, rit = _whole_batch(lib, t, loops, tol)
    np.testing.assert_array_equal(it, rit)
    np.testing.assert_array_equal(ph, rph)
    assert it[2] == 8
    with pytest.raises(lib.SlmError, match="device"):
        lib.gs_multi(t, 3, [0, 99])


@pytest.mark.gpu
def test_gather_stats_single_rank(gpu):
    lib = gpu
    t = _targets(3, 256, False)
    loops = 9
    with lib.Plan(lib.ALGO_GS, 3, 256, 256, lib.TGT_F32, False, loops) as p:
        p.set_target(t)
        p.run(loops)
        _, _, st, it = p.read()
        gph = np.empty((3, 256, 256), np.float32)
        p.gather_phase([3], 0, gph)
        gst, git = p.gather_stats([3], 0)
        ph = p.read(expected=False, stats=False, iters=False)[0]
    np.testing.assert_array_equal(gph, ph)
    np.testing.assert_array_equal(gst, st)
    np.testing.assert_array_equal(git, it)
    with pytest.raises(lib.SlmError, match="counts"):
        with lib.Plan(lib.ALGO_GS, 3, 256, 256, lib.TGT_F32, False, loops) as p:
            p.set_target(t)
            p.gather_stats([2], 0)
