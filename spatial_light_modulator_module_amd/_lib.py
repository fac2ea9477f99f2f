"""ctypes binding of libslm_hip.so (C-ABI declared in include/slm_hip.h).

The shared library is the only compute path of this package: there is no CPU
fallback. Loading fails loudly when the library has not been built, and every
compute call raises :class:`SlmError` when no gfx950 device is usable.

No torch: the library links the system ROCm runtime (libamdhip64, librccl).
A process that also imports PyTorch-ROCm (which bundles its own HIP runtime)
should import torch first so that one runtime is mapped.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

# $SLM_LIB_PATH selects an experimental build (A/B variants); default is the in-tree library
LIB_PATH = os.environ.get("SLM_LIB_PATH") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib",
                                                          "libslm_hip.so")

ALGO_GS = 0
ALGO_GD = 1
TGT_U8 = 0
TGT_F32 = 1
PRECISION_F32 = 0
PRECISION_F64 = 1

KERNEL_COL_MAIN = 0
KERNEL_ROW_MAIN = 1
KERNEL_GD_STATS = 2
KERNEL_OTHER = 3
NUM_KERNEL_CLASSES = 4
KERNEL_CLASS_NAMES = ("col_main", "row_main", "gd_stats", "other")

# sides with a radix plan (the fused FFT kernels); any other side runs the
# float64 any-size engine (generic.hip: mixed radix, or chirp-z line transforms)
SUPPORTED_LENGTHS = (64, 128, 256, 512, 768, 1024, 2048, 4096)


class SlmError(RuntimeError):
    """A libslm_hip call failed (message from slm_last_error)."""


_c_int = ctypes.c_int
_c_double = ctypes.c_double
_c_float = ctypes.c_float
_vp = ctypes.c_void_p
_P = ctypes.POINTER

# (name, restype, argtypes) for every symbol of include/slm_hip.h
_SIGNATURES = [
    ("slm_init", _c_int, [_c_int]),
    ("slm_device_count", _c_int, []),
    ("slm_last_error", ctypes.c_char_p, []),
    ("slm_version", ctypes.c_char_p, []),
    ("slm_supported_length", _c_int, [_c_int]),
    ("slm_device_pci_bus_id", _c_int, [_c_int, ctypes.c_char_p, _c_int]),
    ("slm_copy_bandwidth", _c_int, [ctypes.c_longlong, _c_int, _P(_c_double)]),
    ("slm_plan_create", _c_int, [_c_int, _c_int, _c_int, _c_int, _c_int, _c_int, _c_int, _P(_vp)]),
    ("slm_plan_destroy", _c_int, [_vp]),
    ("slm_plan_set_target", _c_int, [_vp, _vp]),
    ("slm_plan_set_precision", _c_int, [_vp, _c_int]),
    ("slm_plan_get_precision", _c_int, [_vp]),
    ("slm_plan_set_ain", _c_int, [_vp, _vp]),
    ("slm_plan_set_phase", _c_int, [_vp, _vp]),
    ("slm_plan_set_field", _c_int, [_vp, _vp]),
    ("slm_plan_set_lr", _c_int, [_vp, _vp]),
    ("slm_plan_run", _c_int, [_vp, _c_int, _c_double, _c_int, _c_float]),
    ("slm_plan_run_timed", _c_int, [_vp, _c_int, _c_double, _c_int, _c_float, _vp, _vp]),
    ("slm_plan_sync", _c_int, [_vp]),
    ("slm_plan_mark", _c_int, [_vp, _c_int]),
    ("slm_plan_marked_ms", _c_int, [_vp, _P(_c_double)]),
    ("slm_plan_gd_recoveries", _c_int, [_vp]),
    ("slm_plan_read", _c_int, [_vp, _vp, _vp, _vp, _vp]),
    ("slm_plan_read_target_stats", _c_int, [_vp, _vp, _vp]),
    ("slm_plan_set_target_stats", _c_int, [_vp, _vp, _vp]),
    ("slm_plan_read_field", _c_int, [_vp, _vp]),
    ("slm_plan_kernel_bytes", ctypes.c_longlong, [_vp, _c_int]),
    ("slm_plan_info", _c_int, [_vp, _vp]),
    ("slm_plan_layout", _c_int, [_vp, _vp, _vp]),
    ("slm_plan_engine", _c_int, [_vp, _vp, _vp]),
    ("slm_plan_device", _c_int, [_vp]),
    ("slm_plan_read_trace", _c_int, [_vp, _c_int, _vp]),
    ("slm_gs", _c_int, [_vp, _c_int, _vp, _c_int, _c_int, _c_int, _c_int, _c_double, _vp, _vp, _vp, _vp, _vp]),
    ("slm_gd", _c_int,
     [_vp, _c_int, _vp, _c_int, _c_int, _c_int, _c_int, _c_double, _vp, _vp, _c_float, _vp, _vp, _vp, _vp]),
    ("slm_fft2", _c_int, [_vp, _vp, _c_int, _c_int, _c_int, _c_int]),
    ("slm_gs_multi", _c_int, [_c_int, _vp, _vp, _c_int, _vp, _c_int, _c_int, _c_int, _c_int, _c_double, _vp, _vp,
                              _vp, _vp, _vp]),
    ("slm_gs_multi_timing", _c_int, [_c_int, _vp, _vp]),
    ("slm_comm_unique_id", _c_int, [_vp]),
    ("slm_comm_init", _c_int, [_c_int, _c_int, _vp]),
    ("slm_comm_destroy", _c_int, []),
    ("slm_plan_gather_phase", _c_int, [_vp, _vp, _c_int, _vp]),
    ("slm_plan_gather_stats", _c_int, [_vp, _vp, _c_int, _vp, _vp]),
    ("slm_plan_time_gather", _c_int, [_vp, _vp, _c_int, _c_int, _P(_c_double), _P(ctypes.c_longlong)]),
    ("slm_gather_layout", _c_int, [_c_int, _vp, ctypes.c_longlong, _vp]),
    ("slm_trap_frames", _c_int,
     [_c_int, _c_int, _c_int, _vp, _vp, _vp, _c_double, _c_int, _vp, _vp]),
    ("slm_quantize", _c_int, [_vp, _c_int, _vp, _c_int, _c_int, _c_int, _c_double, _c_int, _vp]),
    ("slm_transform_hologram", _c_int, [_vp, _c_int, _c_int, _c_int, _vp, _vp]),
    ("slm_fft2_intensity", _c_int, [_vp, _c_int, _c_int, _c_int, _vp]),
    ("slm_fft2_c128", _c_int, [_vp, _vp, _c_int, _c_int, _c_int, _c_int]),
    ("slm_release_caches", _c_int, []),
]

TRANSFORM_DEFLECT = 1
TRANSFORM_LENS = 2

QUANT_ASTYPE = 0
QUANT_PIL = 1
SRC_F64 = 0
SRC_I16 = 1

_lib = None


def load() -> ctypes.CDLL:
    """Load libslm_hip.so once; raise ImportError if it was never built."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
            "(or `make -C spatial_light_modulator_module_amd/csrc`). There is no CPU fallback."
        )
    lib = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
    for name, res, args in _SIGNATURES:
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def last_error() -> str:
    msg = load().slm_last_error()
    return msg.decode() if msg else ""


def check(rc: int, what: str) -> None:
    if rc != 0:
        raise SlmError(f"{what} failed ({rc}): {last_error()}")


def ptr(a: np.ndarray | None) -> int | None:
    if a is None:
        return None
    assert a.flags["C_CONTIGUOUS"], "arrays passed to libslm_hip must be C-contiguous"
    return a.ctypes.data


_initialised_device: int | None = None


def init(device: int | None = None) -> None:
    """Bind this process to one GPU (default: $SLM_DEVICE, $LOCAL_RANK or 0)."""
    global _initialised_device
    if device is None:
        device = int(os.environ.get("SLM_DEVICE", os.environ.get("LOCAL_RANK", "0")))
    if _initialised_device == device:
        return
    check(load().slm_init(device), f"slm_init({device})")
    _initialised_device = device


def device_count() -> int:
    return int(load().slm_device_count())


def pci_bus_id(device: int) -> str:
    """PCI bus id of a HIP device (slm_device_pci_bus_id)."""
    buf = ctypes.create_string_buffer(64)
    check(load().slm_device_pci_bus_id(int(device), buf, 64), "slm_device_pci_bus_id")
    return buf.value.decode()


def gs_multi_timing(max_shards: int = 64):
    """(wall_ms, run_ms) per shard of this process's last gs_multi call."""
    wall = np.zeros(max_shards, np.float64)
    run = np.zeros(max_shards, np.float64)
    n = int(load().slm_gs_multi_timing(int(max_shards), ptr(wall), ptr(run)))
    return wall[:min(n, max_shards)].tolist(), run[:min(n, max_shards)].tolist()


def copy_bandwidth(nbytes: int, reps: int = 20) -> float:
    """Measured streaming-copy rate of two nbytes device buffers, GB/s
    (read + write; slm_copy_bandwidth)."""
    init()
    g = ctypes.c_double()
    check(load().slm_copy_bandwidth(int(nbytes), int(reps), ctypes.byref(g)), "slm_copy_bandwidth")
    return float(g.value)


class Plan:
    """A device-resident batch of holograms (slm_plan_* in include/slm_hip.h)."""

    def __init__(self, algo: int, batch: int, height: int, width: int, tgt_type: int, has_ain: bool,
                 max_loops: int):
        init()
        self._lib = load()
        h = ctypes.c_void_p()
        check(self._lib.slm_plan_create(algo, batch, height, width, tgt_type, int(bool(has_ain)), max_loops,
                                        ctypes.byref(h)), "slm_plan_create")
        self.handle = h
        self.algo, self.batch, self.height, self.width = algo, batch, height, width
        self.tgt_type, self.has_ain, self.max_loops = tgt_type, bool(has_ain), max_loops

    def close(self) -> None:
        if getattr(self, "handle", None):
            self._lib.slm_plan_destroy(self.handle)
            self.handle = None

    def __del__(self):  # pragma: no cover - best effort
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    @property
    def shape(self):
        return (self.batch, self.height, self.width)

    def set_target(self, tgt: np.ndarray) -> None:
        dt = np.uint8 if self.tgt_type == TGT_U8 else np.float32
        a = np.ascontiguousarray(tgt, dtype=dt).reshape(self.shape)
        check(self._lib.slm_plan_set_target(self.handle, ptr(a)), "slm_plan_set_target")

    @property
    def precision(self) -> int:
        return int(self._lib.slm_plan_get_precision(self.handle))

    def set_precision(self, precision: int) -> None:
        check(self._lib.slm_plan_set_precision(self.handle, int(precision)), "slm_plan_set_precision")

    def set_ain(self, ain: np.ndarray) -> None:
        a = np.ascontiguousarray(ain, dtype=np.float32).reshape(self.height, self.width)
        check(self._lib.slm_plan_set_ain(self.handle, ptr(a)), "slm_plan_set_ain")

    def set_phase(self, phase: np.ndarray | None) -> None:
        a = None if phase is None else np.ascontiguousarray(phase, dtype=np.float32).reshape(self.shape)
        check(self._lib.slm_plan_set_phase(self.handle, ptr(a)), "slm_plan_set_phase")

    def set_field(self, field: np.ndarray | None) -> None:
        a = None
        if field is not None:
            a = np.ascontiguousarray(np.asarray(field).astype(np.complex64)).reshape(self.shape)
            a = a.view(np.float32)
        check(self._lib.slm_plan_set_field(self.handle, ptr(a)), "slm_plan_set_field")

    def set_lr(self, lr: np.ndarray) -> None:
        a = np.ascontiguousarray(lr, dtype=np.float32)
        if a.size != self.max_loops:
            raise ValueError(f"need {self.max_loops} learning rates, got {a.size}")
        check(self._lib.slm_plan_set_lr(self.handle, ptr(a)), "slm_plan_set_lr")

    def run(self, loops: int, tol: float = 0.0, checked: bool = False, white_attention: float = 0.0) -> None:
        check(self._lib.slm_plan_run(self.handle, loops, float(tol), int(bool(checked)), float(white_attention)),
              "slm_plan_run")

    def run_timed(self, loops: int, tol: float = 0.0, checked: bool = False, white_attention: float = 0.0):
        us = np.zeros(NUM_KERNEL_CLASSES, dtype=np.float64)
        cnt = np.zeros(NUM_KERNEL_CLASSES, dtype=np.int32)
        check(self._lib.slm_plan_run_timed(self.handle, loops, float(tol), int(bool(checked)),
                                           float(white_attention), ptr(us), ptr(cnt)), "slm_plan_run_timed")
        return us, cnt

    def sync(self) -> None:
        check(self._lib.slm_plan_sync(self.handle), "slm_plan_sync")

    def mark(self, which: int) -> None:
        """Record stopwatch event 0 or 1 on the plan stream (slm_plan_mark)."""
        check(self._lib.slm_plan_mark(self.handle, int(which)), "slm_plan_mark")

    def marked_ms(self) -> float:
        """Device time between marks 0 and 1 (slm_plan_marked_ms)."""
        ms = ctypes.c_double()
        check(self._lib.slm_plan_marked_ms(self.handle, ctypes.byref(ms)), "slm_plan_marked_ms")
        return float(ms.value)

    @property
    def gd_recoveries(self) -> int:
        """GD runs redone on the two-launch column side after the one-launch
        grid wait gave up (slm_plan_gd_recoveries)."""
        return int(self._lib.slm_plan_gd_recoveries(self.handle))

    def read(self, phase=True, expected=True, stats=True, iters=True):
        out_phase = np.empty(self.shape, np.float32) if phase else None
        out_exp = np.empty(self.shape, np.float32) if expected else None
        out_stats = np.empty((self.batch, self.max_loops, 4), np.float64) if stats else None
        out_iters = np.empty(self.batch, np.int32) if iters else None
        check(self._lib.slm_plan_read(self.handle, ptr(out_phase), ptr(out_exp), ptr(out_stats), ptr(out_iters)),
              "slm_plan_read")
        return out_phase, out_exp, out_stats, out_iters

    def target_stats(self):
        norm = np.empty(self.batch, np.float64)
        st2 = np.empty(self.batch, np.float64)
        check(self._lib.slm_plan_read_target_stats(self.handle, ptr(norm), ptr(st2)), "slm_plan_read_target_stats")
        return norm, st2

    def set_target_stats(self, norm, sum_t2) -> None:
        n = np.ascontiguousarray(norm, dtype=np.float64).reshape(self.batch)
        s = np.ascontiguousarray(sum_t2, dtype=np.float64).reshape(self.batch)
        check(self._lib.slm_plan_set_target_stats(self.handle, ptr(n), ptr(s)), "slm_plan_set_target_stats")

    def read_field(self) -> np.ndarray:
        """GD state x [batch][h][w] complex64 after the last run."""
        out = np.empty(self.shape, np.complex64)
        check(self._lib.slm_plan_read_field(self.handle, ptr(out.view(np.float32))), "slm_plan_read_field")
        return out

    def kernel_bytes(self, cls: int) -> int:
        return int(self._lib.slm_plan_kernel_bytes(self.handle, cls))

    def info(self) -> dict:
        a = np.zeros(8, np.int32)
        check(self._lib.slm_plan_info(self.handle, ptr(a)), "slm_plan_info")
        return {"col_cw": int(a[0]), "col_workgroups": int(a[1]), "col_threads": int(a[2]),
                "row_threads": int(a[3]), "rows_per_workgroup": int(a[4]), "row_plan": int(a[5]),
                "col_plan": int(a[6]), "precision": "f64" if a[7] == PRECISION_F64 else "f32",
                "layout": self.layout(), "engine": self.engine()}

    @property
    def device(self) -> int:
        """HIP device of the plan (slm_plan_device)."""
        return int(self._lib.slm_plan_device(self.handle))

    def time_gather(self, counts, root: int = 0, reps: int = 5):
        """(ms per device-side phase gather, bytes this rank sends per gather):
        slm_plan_time_gather, collective."""
        c = np.ascontiguousarray(counts, dtype=np.int32)
        ms = ctypes.c_double()
        nb = ctypes.c_longlong()
        check(self._lib.slm_plan_time_gather(self.handle, ptr(c), int(root), int(reps), ctypes.byref(ms),
                                             ctypes.byref(nb)), "slm_plan_time_gather")
        return float(ms.value), int(nb.value)

    def engine(self) -> tuple[str, str]:
        """(column, row) transform engine of the GS iteration kernels:
        "stockham", "shuffle" (wave-shuffle pair, fft_shuffle.hpp) or, for
        sides without a float32 radix plan, "mixed-radix" (float64 radix
        2..13 kernels, mixed_radix.hpp) or "bluestein" (float64 1-D line
        transforms along rows and transposed columns, Bluestein's chirp-z
        for a side with a larger prime factor, generic.hip), and under
        $SLM_ENGINE=float64 on 2^k / 768 sides, and for uint8 GS / GD /
        float64 runs on 13-smooth SLM panel sides, "radix-c128" (float64
        Stockham kernels with complex128 state, radix_c128.hpp); float32 GS on
        panel sides (e.g. 1080 x 1920) "radix-c64" (the same kernels with
        complex64 state and float32 butterflies)."""
        c, r = ctypes.c_int(), ctypes.c_int()
        check(self._lib.slm_plan_engine(self.handle, ctypes.byref(c), ctypes.byref(r)), "slm_plan_engine")
        names = ("stockham", "shuffle", "bluestein", "mixed-radix", "radix-c128", "radix-c64")
        return names[c.value], names[r.value]

    def layout(self) -> tuple[int, int]:
        """(X, Y) panel widths of the plan's blocked device layouts."""
        x, y = ctypes.c_int(), ctypes.c_int()
        check(self._lib.slm_plan_layout(self.handle, ctypes.byref(x), ctypes.byref(y)), "slm_plan_layout")
        return 1 << x.value, 1 << y.value

    def read_trace(self, cls: int) -> np.ndarray:
        """[batch * workgroups, 8] phase timestamps of the last launch of a
        kernel class (SLM_TRACE builds with SLM_TRACE_BUF=1; diagnostics):
        tile start, loads done, transforms done, stores done, kernel entry,
        HW_ID, XCC_ID (kernels.hpp, trace_point)."""
        b, h, w = self.shape
        info = self.info()
        n = info["col_workgroups"] if cls == KERNEL_COL_MAIN else h // info["rows_per_workgroup"]
        out = np.zeros((b * n, 8), np.uint64)
        check(self._lib.slm_plan_read_trace(self.handle, cls, ptr(out)), "slm_plan_read_trace")
        return out

    def gather_phase(self, counts, root: int = 0, host_out: np.ndarray | None = None) -> None:
        c = np.ascontiguousarray(counts, dtype=np.int32)
        check(self._lib.slm_plan_gather_phase(self.handle, ptr(c), root, ptr(host_out)), "slm_plan_gather_phase")

    def gather_stats(self, counts, root: int = 0, want: bool = True):
        """Every rank's per-iteration statistics [sum(counts)][max_loops][4] and
        iterations executed [sum(counts)] on `root` (None elsewhere, or when
        want=False: the collective still runs, nothing is copied to the host)."""
        c = np.ascontiguousarray(counts, dtype=np.int32)
        total = int(c.sum())
        st = np.empty((total, self.max_loops, 4), np.float64) if want else None
        it = np.empty(total, np.int32) if want else None
        check(self._lib.slm_plan_gather_stats(self.handle, ptr(c), root, ptr(st), ptr(it)), "slm_plan_gather_stats")
        return st, it


def fft2(x: np.ndarray, inverse: bool = False) -> np.ndarray:
    """Unscaled 2-D C2C transform of [..., H, W] on the GPU (test entry)."""
    init()
    a = np.ascontiguousarray(x, dtype=np.complex64)
    shape = a.shape
    h, w = shape[-2:]
    b = int(np.prod(shape[:-2])) if len(shape) > 2 else 1
    out = np.empty_like(a)
    check(load().slm_fft2(ptr(a.view(np.float32)), ptr(out.view(np.float32)), b, h, w, int(bool(inverse))),
          "slm_fft2")
    return out


def fft2_c128(x: np.ndarray, inverse: bool = False) -> np.ndarray:
    """Unscaled 2-D C2C transform of [..., H, W] complex128 in float64 on the
    GPU (slm_fft2_c128: the any-size engine's transforms, any shape)."""
    init()
    a = np.ascontiguousarray(x, dtype=np.complex128)
    shape = a.shape
    h, w = shape[-2:]
    b = int(np.prod(shape[:-2])) if len(shape) > 2 else 1
    out = np.empty_like(a)
    check(load().slm_fft2_c128(ptr(a.view(np.float64)), ptr(out.view(np.float64)), b, h, w, int(bool(inverse))),
          "slm_fft2_c128")
    return out


def release_caches() -> None:
    """Free the float64 engines slm_fft2_c128 keeps per shape (no-op without a library)."""
    if _lib is not None:
        check(_lib.slm_release_caches(), "slm_release_caches")


def transform_hologram(hologram, height, width, deflect_params=None, lens_params=None):
    """deflect / lens post-processing of src/generate_hologram.py:82-87 on the
    GPU (slm_transform_hologram). hologram float64 [h][w] or None (zeros);
    deflect_params = (sin(y u), sin(x u), 2 pi px / wl); lens_params =
    (2 pi f / wl, f, px)."""
    flags = 0
    params = np.zeros(6, np.float64)
    if deflect_params is not None:
        flags |= TRANSFORM_DEFLECT
        params[0:3] = deflect_params
    if lens_params is not None:
        flags |= TRANSFORM_LENS
        params[3:6] = lens_params
    src = None if hologram is None else np.ascontiguousarray(hologram, dtype=np.float64).reshape(height, width)
    out = np.empty((height, width), np.float64)
    init()
    check(load().slm_transform_hologram(ptr(src), height, width, flags, ptr(params), ptr(out)),
          "slm_transform_hologram")
    return out


def fft2_intensity(phase) -> np.ndarray:
    """|fft2(exp(1j phase))|^2 on the GPU (float32), phase [..., H, W]."""
    a = np.ascontiguousarray(phase, dtype=np.float32)
    h, w = a.shape[-2:]
    b = int(np.prod(a.shape[:-2])) if a.ndim > 2 else 1
    out = np.empty(a.shape, np.float32)
    init()
    check(load().slm_fft2_intensity(ptr(a), b, h, w, ptr(out)), "slm_fft2_intensity")
    return out


def gs_multi(targets, loops, devices, tol=0.0, ain=None, initial_phase=None):
    """slm_gs_multi: GS on a batch [B][H][W] sharded over `devices` (device ids,
    may repeat) from one process. Returns (phase, expected, stats, iters)."""
    t = np.asarray(targets)
    tt = TGT_U8 if t.dtype == np.uint8 else TGT_F32
    t = np.ascontiguousarray(t, dtype=np.uint8 if tt == TGT_U8 else np.float32)
    b, h, w = t.shape
    dev = np.ascontiguousarray(devices, dtype=np.int32)
    a = None if ain is None else np.ascontiguousarray(ain, dtype=np.float32).reshape(h, w)
    ph0 = None if initial_phase is None else np.ascontiguousarray(initial_phase, dtype=np.float32).reshape(b, h, w)
    phase = np.empty((b, h, w), np.float32)
    expected = np.empty((b, h, w), np.float32)
    stats = np.empty((b, loops, 4), np.float64)
    iters = np.empty(b, np.int32)
    init()
    check(load().slm_gs_multi(int(dev.size), ptr(dev), ptr(t), tt, ptr(a), b, h, w, int(loops), float(tol), ptr(ph0),
                              ptr(phase), ptr(expected), ptr(stats), ptr(iters)), "slm_gs_multi")
    return phase, expected, stats, iters


def gather_layout(counts, per_item: int) -> np.ndarray:
    """Rank-order element offsets of a gather (slm_gather_layout; host only):
    offsets[r] = per_item * sum(counts[:r]), offsets[-1] = the total."""
    c = np.ascontiguousarray(counts, dtype=np.int32)
    out = np.empty(c.size + 1, np.int64)
    check(load().slm_gather_layout(int(c.size), ptr(c), int(per_item), ptr(out)), "slm_gather_layout")
    return out


def comm_unique_id() -> bytes:
    buf = (ctypes.c_ubyte * 128)()
    check(load().slm_comm_unique_id(buf), "slm_comm_unique_id")
    return bytes(buf)


def comm_init(nranks: int, rank: int, uid: bytes) -> None:
    init()
    buf = (ctypes.c_ubyte * 128).from_buffer_copy(uid)
    check(load().slm_comm_init(nranks, rank, buf), "slm_comm_init")


def comm_destroy() -> None:
    load().slm_comm_destroy()


def trap_frames(shape, ys, xs, mask=None, ct2pi=256.0, rule=QUANT_ASTYPE, phase=True, frame=True):
    """Single-trap holograms (angle of ifft2 of one 255 pixel per trap) and/or
    their quantised SLM frames, one launch (slm_trap_frames)."""
    h, w = shape
    ys = np.ascontiguousarray(ys, dtype=np.int32).reshape(-1)
    xs = np.ascontiguousarray(xs, dtype=np.int32).reshape(-1)
    b = ys.size
    m = None if mask is None else np.ascontiguousarray(mask, dtype=np.float64).reshape(h, w)
    ph = np.empty((b, h, w), np.float64) if phase else None
    fr = np.empty((b, h, w), np.uint8) if frame else None
    init()
    check(load().slm_trap_frames(b, h, w, ptr(ys), ptr(xs), ptr(m), float(ct2pi), int(rule), ptr(ph), ptr(fr)),
          "slm_trap_frames")
    return ph, fr


def quantize(src, mask=None, ct2pi=256.0, rule=QUANT_PIL):
    """8-bit SLM levels of a float64 phase hologram (rule QUANT_ASTYPE / QUANT_PIL)
    or of an int16 hologram image, plus an optional float64 mask (slm_quantize)."""
    src = np.asarray(src)
    src_type = SRC_I16 if src.dtype == np.int16 else SRC_F64
    a = np.ascontiguousarray(src, dtype=np.int16 if src_type == SRC_I16 else np.float64)
    h, w = a.shape[-2:]
    b = int(np.prod(a.shape[:-2])) if a.ndim > 2 else 1
    m = None if mask is None else np.ascontiguousarray(np.broadcast_to(mask, (h, w)), dtype=np.float64)
    out = np.empty(a.shape, np.uint8)
    init()
    check(load().slm_quantize(ptr(a), src_type, ptr(m), b, h, w, float(ct2pi), int(rule), ptr(out)), "slm_quantize")
    return out
