"""Trap-sequence CLI, drop-in for src/generate_hologram_sequence.py.

    python -m spatial_light_modulator_module_amd.generate_hologram_sequence <source_dir> -v V -ct2pi N [-loops 5] [-p]

The reference runs gerchberg_saxton once per frame (src/generate_hologram_sequence.py:10-31);
frames are independent, so here they run as batches of holograms in one plan
(one launch pair per GS iteration for the whole batch), and under a
one-process-per-GPU launcher (torch.distributed.run or any that sets RANK /
WORLD_SIZE / MASTER_ADDR / MASTER_PORT) each rank takes a contiguous shard of
the frames (parallel.shard_range) and writes its own .npy files: no collective
touches the data path; only the per-frame error lists travel, over the
torch-free control plane (parallel.Group). Without a launcher, $SLM_GPUS (a
device count, "all", or a comma-separated device list) runs each batch over
several GPUs from this one process instead (slm_gs_multi).
Output files, names and stdout lines are the reference's.
"""
from __future__ import annotations

import argparse
import os
import sys

import numpy as np

from . import parallel
from . import _lib
from .algorithms import (_check_shape, _print_loops, expected_from, hologram_from, incoming_amplitude, run_gs,
                         run_gs_multi)

SEQ_BATCH = int(os.environ.get("SLM_SEQ_BATCH", "64"))  # frames per GPU launch batch


def _load_frame(source_dir_path, i):
    from PIL import Image

    return np.array(Image.open(f"{source_dir_path}/{i}.png"))


def _batches(indices, frames):
    """Split an index list into runs of equal shape and dtype, at most SEQ_BATCH long."""
    run = []
    for i in indices:
        if run and (len(run) == SEQ_BATCH or frames[i].shape != frames[run[0]].shape
                    or frames[i].dtype != frames[run[0]].dtype):
            yield run
            run = []
        run.append(i)
    if run:
        yield run


def multi_devices(nranks):
    """Devices for one-process multi-GPU batches ($SLM_GPUS), or None."""
    spec = os.environ.get("SLM_GPUS", "").strip()
    if not spec or nranks > 1:
        return None
    if "," in spec:
        devs = [int(d) for d in spec.split(",") if d.strip()]
    else:
        devs = list(range(_lib.device_count() if spec == "all" else int(spec)))
    return devs if len(devs) > 1 else None


def generate_hologram_sequence(args, rank=None, nranks=None):
    """src/generate_hologram_sequence.py:10-31. Returns the per-frame error
    evolutions of the frames this rank computed (dict frame -> list)."""
    from PIL import Image

    if rank is None:
        rank, nranks, _ = parallel.world()
    dest_dir_holograms = f"holograms/{args.source_dir}_{args.version}_holograms"
    dest_dir_preview = f"images/moving_traps/{args.source_dir}_{args.version}_preview"
    for dest_dir in (dest_dir_holograms, dest_dir_preview):
        os.makedirs(dest_dir, exist_ok=True)
    source_dir_path = f"images/moving_traps/{args.source_dir}"
    n_files = len(os.listdir(source_dir_path))
    mine = list(parallel.shard_range(n_files, nranks, rank))
    frames = {i: _load_frame(source_dir_path, i) for i in mine}
    errors = {}
    devices = multi_devices(nranks)
    for idx in _batches(mine, frames):
        stack = np.stack([frames[i] for i in idx])
        _check_shape(stack[0])
        ain = incoming_amplitude(args, stack.shape[1:])
        if not (args.max_loops > 0 and (args.tolerance + 1) > args.tolerance):
            raise UnboundLocalError("local variable 'expected_outcome' referenced before assignment")
        if devices:
            phase, e, errs, norm, emax = run_gs_multi(stack, args.max_loops, devices, args.tolerance, ain)
        else:
            phase, e, errs, norm, emax = run_gs(stack, args.max_loops, args.tolerance, ain)
        for k, i in enumerate(idx):
            sys.stdout.write(f"\rcreating {i}. hologram ")
            _print_loops(len(errs[k]), args.max_loops)
            errors[i] = errs[k]
            np.save(f"{dest_dir_holograms}/{i}.npy", hologram_from(phase[k]))
            if args.preview:
                expected = expected_from(e[k], norm[k], emax[k])
                Image.fromarray(expected).convert("L").save(f"{dest_dir_preview}/{i}.png")
    return errors


def plot_error_evolution(err_evl_list):
    """src/generate_hologram_sequence.py:34-39."""
    import matplotlib.pyplot as plt

    for i, err_evl in enumerate(err_evl_list):
        plt.plot(err_evl, label=i)
    plt.legend()
    plt.show()


def build_parser():
    """Argument set of src/generate_hologram_sequence.py:52-103."""
    p = argparse.ArgumentParser(formatter_class=argparse.ArgumentDefaultsHelpFormatter,
                                description="Transform a sequence of trap images into holograms (GS on MI355X).")
    p.add_argument("source_dir", type=str, help="directory of trap images inside images/moving_traps")
    p.add_argument("-v", "--version", type=str, help="suffix distinguishing versions of the same sequence")
    p.add_argument("-ii", "--incomming_intensity", metavar="PATH", type=str, default="uniform",
                   help="incomming intensity image or 'uniform'")
    p.add_argument("-ct2pi", "--correspond_to2pi", metavar="INT", required=True, type=int,
                   help="value of pixel corresponding to 2pi phase shift")
    p.add_argument("-tol", "--tolerance", metavar="FLOAT", default=0, type=float,
                   help="algorithm stops when error descends under tolerance")
    p.add_argument("-loops", "--max_loops", metavar="INT", default=5, type=int,
                   help="algorithm performs no more than max_loops loops")
    p.add_argument("-p", "--preview", action="store_true", help="also write expected images")
    return p


def cli(argv=None, plot=True):
    args = build_parser().parse_args(argv)
    args.gif = False
    args.plot_error = False
    args.print_info = False
    rank, nranks, _ = parallel.world()
    errors = generate_hologram_sequence(args, rank, nranks)
    if nranks > 1:
        # error lists are host objects; the phases went to disk
        with parallel.Group.from_env() as group:
            gathered = group.all_gather(errors)
        errors = {k: v for part in gathered for k, v in part.items()}
    print()
    if plot and rank == 0:
        plot_error_evolution([errors[i] for i in sorted(errors)])
    return errors


if __name__ == "__main__":
    cli()
