"""Host-only checks of bench.py's N > 1 output (no GPU): two ranks over the
stdlib control plane, each with a stubbed libslm_hip binding, run bench.main
and rank 0's JSON line must carry the driver contract's fields plus one
diagnostics record per rank (device, PCI bus id, own step time, kernel
times, the gather timed on its own), so a scaling run's efficiency can be
split into compute and collective per rank (the batch loop sharded is
src/generate_hologram_sequence.py:19-31)."""
import json
import multiprocessing as mp
import os
import socket
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


class _FakePlan:
    def __init__(self, algo, batch, h, w, tt, has_ain, max_loops, rank):
        self.algo, self.batch, self.height, self.width = algo, batch, h, w
        self.tgt_type, self.has_ain, self.max_loops = tt, has_ain, max_loops
        self.rank = rank

    def set_target(self, t):
        assert t.shape == (self.batch, self.height, self.width)

    def run(self, loops, *a, **k):
        pass

    def sync(self):
        pass

    def mark(self, which):
        pass

    def marked_ms(self):
        return 3.0 * 3.4  # 3 steps of ~3.4 ms

    def gather_phase(self, counts, root=0, host_out=None):
        if host_out is not None:
            host_out[:] = 0.5

    def gather_stats(self, counts, root=0, want=True):
        total = int(sum(counts))
        st = np.zeros((total, self.max_loops, 4))
        st[:, :, 3] = np.linspace(2.0, 1.0, self.max_loops)
        return (st, np.full(total, -1, np.int32)) if want else (None, None)

    def run_timed(self, loops, **k):
        us = np.array([8.0 * loops, 7.5 * (loops - 1), 0.0, 30.0])
        cnt = np.array([loops, loops - 1, 0, 7], np.int32)
        return us, cnt

    def kernel_bytes(self, cls):
        px = self.batch * self.height * self.width
        return {0: 20 * px, 1: 16 * px}.get(cls, 0)

    def info(self):
        return {"col_cw": 2, "col_workgroups": 8, "col_threads": 256, "row_threads": 256, "rows_per_workgroup": 2,
                "row_plan": 11, "col_plan": 11, "precision": "f32", "layout": (8, 2), "engine": ("shuffle", "shuffle")}

    @property
    def device(self):
        return self.rank

    def time_gather(self, counts, root=0, reps=5):
        return 0.25, 0 if self.rank == root else self.batch * self.height * self.width * 4

    def close(self):
        pass


def _fake_lib(rank, fail_init=False):
    from spatial_light_modulator_module_amd import _lib as real

    class Fake:
        ALGO_GS, ALGO_GD, TGT_U8, TGT_F32 = real.ALGO_GS, real.ALGO_GD, real.TGT_U8, real.TGT_F32
        PRECISION_F32, PRECISION_F64 = real.PRECISION_F32, real.PRECISION_F64
        KERNEL_COL_MAIN, KERNEL_ROW_MAIN, KERNEL_GD_STATS = 0, 1, 2
        KERNEL_CLASS_NAMES = real.KERNEL_CLASS_NAMES
        SlmError = real.SlmError

        @staticmethod
        def init(device=None):
            if fail_init:
                raise real.SlmError(f"slm_init({device}) failed (-1): device {device} outside [0, 1)")

        @staticmethod
        def Plan(*a):
            return _FakePlan(*a, rank=rank)

        @staticmethod
        def comm_unique_id():
            return b"\x01" * 128

        @staticmethod
        def comm_init(n, r, uid):
            assert len(uid) == 128
            if os.environ.get("BENCH_TEST_NO_COMM"):
                raise AssertionError("comm_init reached after a rank failed its device initialisation")

        @staticmethod
        def comm_destroy():
            pass

        @staticmethod
        def copy_bandwidth(nbytes, reps=20):
            return 5000.0

        @staticmethod
        def pci_bus_id(dev):
            return f"0000:{dev:02x}:00.0"

    return Fake


def _rank(rank, world, port, out, fail_rank=-1):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port), SLM_RDZV_PORT=str(port), SLM_JOB_TOKEN="bench-host-test")
    if fail_rank >= 0:
        os.environ["BENCH_TEST_NO_COMM"] = "1"
    sys.path.insert(0, ROOT)
    import bench

    bench._lib = _fake_lib(rank, fail_init=rank == fail_rank)
    sys.argv = ["bench.py", "--gpus", str(world), "--steps", "3", "--warmup", "1", "--size", "64", "--iters", "10",
                "--batch-per-gpu", "2"]
    with open(out, "w") as f:
        sys.stdout = f
        bench.main()
        sys.stdout.flush()


def test_bench_two_ranks_json_shape(tmp_path):
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    procs = [ctx.Process(target=_rank, args=(r, 2, port, str(tmp_path / f"r{r}.out"))) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    lines = [ln for ln in (tmp_path / "r0.out").read_text().splitlines() if ln.startswith("{")]
    assert len(lines) == 1 and not (tmp_path / "r1.out").read_text().strip()
    out = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "roofline"):
        assert k in out, k
    assert out["n_gpus"] == 2 and out["scaling"] == "weak" and out["config"]["global_batch"] == 4
    assert out["value"] > 0 and out["check"] == "ok"
    assert "cpu_baseline" not in out  # rank 0 at N = 1 only
    r = out["roofline"]
    assert {"frac", "frac_physical", "achieved", "peak", "traffic", "event_avg_us", "in_graph_scale"} <= set(r)
    assert r["avg_us"] > r["event_avg_us"]  # 3.4 ms per step against 3.1 ms of per-launch events
    ranks = out["ranks"]
    assert [d["rank"] for d in ranks] == [0, 1]
    assert [d["device"] for d in ranks] == [0, 1] and ranks[1]["pci_bus_id"] == "0000:01:00.0"
    assert ranks[0]["gather_bytes_to_root"] == 0 and ranks[1]["gather_bytes_to_root"] == 2 * 64 * 64 * 4
    for d in ranks:
        assert d["step_ms"] > 0 and d["gather_ms"] == 0.25 and set(d["kernel_avg_us"]) == {"col_main", "row_main"}
        assert "plan stream" in d["gather_stream"] or "overlaps the next run" in d["gather_stream"]


def test_bench_rank_without_device_stops_every_rank(tmp_path):
    """A rank whose GPU fails to initialise makes every rank exit with an error
    before any of them enters RCCL's communicator set-up (where the others
    would otherwise wait for it indefinitely)."""
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    procs = [ctx.Process(target=_rank, args=(r, 2, port, str(tmp_path / f"r{r}.out"), 1)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 1
    assert not [ln for ln in (tmp_path / "r0.out").read_text().splitlines() if ln.startswith("{")]


def test_cpu_baseline_configs0_times_whole_runs():
    """BASELINE.json configs[0] (GS 256^2, 50 iterations, the NumPy CPU path)
    is timed as whole runs of the float64 restatement, with the host's CPU
    count stated."""
    sys.path.insert(0, ROOT)
    import bench

    cb = bench.cpu_baseline_configs0(reps=1)
    assert cb["unit"] == "holograms/s" and cb["cores"] == 1 and cb["kind"] == "port"
    assert cb["value"] > 0 and abs(cb["value"] * cb["s_per_hologram"] - 1) < 1e-9
    assert cb["host_cpus"] == os.cpu_count() and "configs[0]" in cb["sample"]


def test_north_star_summary_reports_the_pmc_fraction_per_4096_line():
    """The bench line's north_star block carries each 4096^2 extra line's
    PMC-based iteration fraction beside BASELINE.json's 60 % bar."""
    sys.path.insert(0, ROOT)
    import bench

    line = {"iter_ms": 1.17, "iter_ms_per_hologram": 0.1467, "iter_frac_of_hbm_peak_pmc": 0.53,
            "iter_frac_of_hbm_peak_model": 0.97, "iter_frac_of_hbm_peak_physical": 0.51}
    ns = bench.north_star({"gs_4096_batch8": line, "gd_1024": {"iter_ms": 0.02}, "error": "x"})
    assert ns["bar"] == 0.60 and "pmc" in ns["basis"]
    assert list(ns["shapes"]) == ["gs_4096_batch8"]
    assert ns["shapes"]["gs_4096_batch8"] == {"iter_us_per_hologram": 146.7, "iter_frac_of_hbm_peak_pmc": 0.53,
                                              "iter_frac_of_hbm_peak_model": 0.97,
                                              "iter_frac_of_hbm_peak_physical": 0.51}
