"""Hologram CLI, drop-in for src/generate_hologram.py (same arguments, defaults,
output names and .npy format), with the GS / GD loop on the MI355X.

    python -m spatial_light_modulator_module_amd.generate_hologram <img> [-alg gradient_descent] ...

Target preparation (PIL: grey-scale, invert, pad to square, quarterize,
resize to the 1024x768 SLM) follows src/generate_hologram.py:45-110; the
deflect / lens post-processing (:82-87, :178-203, src/wavefront_correction.py:
440-449) is one element-wise float64 kernel (slm_transform_hologram), bit for
bit the reference's per-pixel loops (including lens()'s uint8 truncation), and
the preview's |fft2(exp(1j h))|^2 (:24-34) runs on the plan kernels
(slm_fft2_intensity). The vectorised NumPy forms below (deflect_2pi, lens)
remain as the host twins the CPU tests pin against the reference loops.
"""
from __future__ import annotations

import argparse
import os

import numpy as np

from . import _lib
from . import constants as c
from .algorithms import gerchberg_saxton, gradient_descent


def main(args):
    """src/generate_hologram.py:13-21."""
    if args.img_name is None:
        hologram = np.zeros((c.slm_height, c.slm_width))
    else:
        hologram = make_hologram(args)
    hologram = transform_hologram(hologram, args)
    if args.preview:
        show_expected_outcome(hologram, args)
    return save_hologram_and_gif(hologram, args)


def expected_outcome_image(hologram, norm):
    """|fft2(exp(1j h))|^2 / max * norm as float64 (src/generate_hologram.py:25-30);
    the transform runs on the GPU in complex64 (a preview image)."""
    intensity = _lib.fft2_intensity(np.asarray(hologram)).astype(np.float64)
    return intensity / np.amax(intensity) * norm


def show_expected_outcome(hologram, args):
    """src/generate_hologram.py:24-34."""
    from PIL import Image

    normed = expected_outcome_image(hologram, find_out_norm(args))
    Image.fromarray(normed).resize((c.slm_height, c.slm_height)).show()


def find_out_norm(args):
    from PIL import Image

    if args.img_name is None:
        return 255
    return np.amax(np.array(Image.open(f"images/{args.img_name}").convert("L")))


def pad_to_square(img):
    """Pad with black to a square, original centred (src/generate_hologram.py:45-67)."""
    from PIL import Image

    width, height = img.size
    if width == height:
        return img
    new_size = max(width, height)
    new_img = Image.new("L", (new_size, new_size), 0)
    new_img.paste(img, ((new_size - width) // 2, (new_size - height) // 2))
    return new_img


def quarter(image):
    """Original scaled by 1/2 into the upper-left corner (src/generate_hologram.py:166-175)."""
    from PIL import Image

    w, h = image.size
    resized = image.resize((w // 2, h // 2))
    ground = Image.new("L", (w, h))
    ground.paste(resized)
    return ground


def prepare_target(img_name, args):
    """uint8 (768, 1024) target (src/generate_hologram.py:102-110)."""
    import PIL.ImageOps
    from PIL import Image

    target_img = Image.open(f"images/{img_name}").convert("L")
    if args.invert:
        target_img = PIL.ImageOps.invert(target_img)
    target_img = pad_to_square(target_img)
    if args.quarterize:
        target_img = quarter(target_img)
    return np.array(target_img.resize((int(c.slm_width), int(c.slm_height))))


def make_hologram(args):
    """src/generate_hologram.py:70-79."""
    algorithm = gerchberg_saxton if args.algorithm == "gerchberg_saxton" else gradient_descent
    target = prepare_target(args.img_name, args)
    if args.gif:
        add_gif_dirs(args)
        remove_files_in_dir(args.gif_source_dir)
    hologram, _, _ = algorithm(target, args)
    return hologram


def deflect_params(angle):
    """The host-side scalars of deflect_2pi (src/wavefront_correction.py:440-447),
    computed exactly as the reference computes them."""
    x_angle, y_angle = angle
    const = 2 * np.pi * c.px_distance / c.wavelength
    return float(np.sin(y_angle * c.u)), float(np.sin(x_angle * c.u)), const


def lens_params(focal_length):
    """The host-side scalars of lens() (src/generate_hologram.py:189-203)."""
    return 2 * np.pi * focal_length / c.wavelength, float(focal_length), c.px_distance


def transform_hologram(hologram, args):
    """src/generate_hologram.py:82-87 as one GPU launch (slm_transform_hologram).
    The reference's deflect ramp has the SLM's size (c.slm_height x c.slm_width),
    so the hologram must have it too when deflecting (as in the reference)."""
    d = deflect_params(args.deflect) if args.deflect is not None else None
    f = lens_params(args.lens) if args.lens else None
    if d is None and f is None:
        return hologram
    h, w = np.asarray(hologram).shape
    if d is not None and (h, w) != (c.slm_height, c.slm_width):
        raise ValueError(f"operands could not be broadcast together with shapes {(h, w)} "
                         f"{(c.slm_height, c.slm_width)}")
    return _lib.transform_hologram(hologram, h, w, d, f)


def add_gif_dirs(args):
    if args.gif_type == "h":
        args.gif_dest_dir = "holograms"
    elif args.gif_type == "i":
        args.gif_dest_dir = "images"
    os.makedirs(args.gif_dest_dir, exist_ok=True)
    args.gif_source_dir = f"{args.gif_dest_dir}/gif_source"
    os.makedirs(args.gif_source_dir, exist_ok=True)


def originalize_name(name: str) -> str:
    """Append _1, _2, ... until the file name is new (src/wavefront_correction.py:325-337)."""
    if not os.path.exists(name):
        return name
    base, ext = os.path.splitext(name)
    i = 1
    while True:
        new_name = f"{base}_{i}{ext}"
        if not os.path.exists(new_name):
            return new_name
        i += 1


def save_hologram_and_gif(hologram, args):
    """src/generate_hologram.py:113-128; returns the .npy path written."""
    img_name = os.path.basename(args.img_name).split(".")[0] if args.img_name else "analytical"
    dest_dir = args.destination_directory
    os.makedirs(dest_dir, exist_ok=True)
    hologram_name = make_hologram_name(args, img_name)
    path = originalize_name(f"{dest_dir}/{hologram_name}.npy")
    np.save(path, hologram)
    if args.gif:
        create_gif(args.gif_source_dir, originalize_name(f"{args.gif_dest_dir}/{hologram_name}.gif"))
    return path


_SEP = " " * 8  # the reference's name f-string continues lines inside the literal (src/generate_hologram.py:149-153)


def make_hologram_name(args, img_name):
    """src/generate_hologram.py:131-153, whitespace included."""
    alg_params = ""
    transforms = ""
    img_transforms = ""
    if args.deflect:
        transforms += f"_deflect_x{args.deflect[0]}_y{args.deflect[1]}"
    if args.lens:
        transforms += f"_lens{args.lens}"
    if args.algorithm == "gradient_descent":
        alg_params += f"_lr{args.learning_rate}_mr{args.white_attention}_unsettle{args.unsettle}"
    if args.quarterize:
        img_transforms += "_quarter"
    if args.invert:
        img_transforms += "_inverted"
    if args.img_name is None:
        return f"{img_name}{transforms}"
    return (f"{img_name}{img_transforms}" + _SEP + f"_{args.algorithm}" + _SEP + f"{alg_params}" + _SEP
            + f"_loops{args.max_loops}" + _SEP + f"{transforms}")


def deflect_2pi(angle):
    """Linear phase ramp deflecting by (x, y) units of c.u (src/wavefront_correction.py:440-449)."""
    x_angle, y_angle = angle
    const = 2 * np.pi * c.px_distance / c.wavelength
    i = np.arange(c.slm_height, dtype=np.float64)[:, None]
    j = np.arange(c.slm_width, dtype=np.float64)[None, :]
    new_phase = const * (np.sin(y_angle * c.u) * i + np.sin(x_angle * c.u) * j)
    return new_phase % (2 * np.pi)


def deflect_hologram(hologram, angle):
    return (hologram + deflect_2pi(angle)) % (2 * np.pi)


def lens(focal_length, shape):
    """Lens phase stored in uint8 as the reference does (truncated to 0..6 rad,
    src/generate_hologram.py:189-203)."""
    h, w = shape
    i = np.arange(h, dtype=np.float64)[:, None]
    j = np.arange(w, dtype=np.float64)[None, :]
    r = c.px_distance * np.sqrt((i - h / 2) ** 2 + (j - w / 2) ** 2)
    phase_shift = 2 * np.pi * focal_length / c.wavelength * (1 - np.sqrt(1 + r**2 / focal_length**2))
    return (phase_shift % (2 * np.pi)).astype(np.uint8)


def add_lens(hologram, focal_len):
    return (hologram + lens(focal_len, hologram.shape)) % (2 * np.pi)


def create_gif(img_dir, outgif_path):
    import imageio  # the reference's dependency; only needed for -gif

    with imageio.get_writer(outgif_path, mode="I") as writer:
        for file in os.listdir(img_dir):
            writer.append_data(imageio.imread(f"{img_dir}/{file}"))


def remove_files_in_dir(dir_name):
    for file in os.listdir(dir_name):
        os.remove(f"{dir_name}/{file}")


def build_parser():
    """The argument set of src/generate_hologram.py:231-369."""
    p = argparse.ArgumentParser(formatter_class=argparse.ArgumentDefaultsHelpFormatter,
                                description="Generate phase hologram for transmissive SLM (GS/GD on MI355X).")
    p.add_argument("img_name", nargs="?", default=None, type=str,
                   help="path to the target image from images directory")
    p.add_argument("-ii", "--incomming_intensity", type=str, default="uniform",
                   help="path to the incomming intensity image or 'uniform'")
    p.add_argument("-ig", "--initial_guess", type=str, default="random", choices=["random", "fourier"],
                   help="initial guess for the gradient_descent algorithm")
    p.add_argument("-dest_dir", "--destination_directory", type=str, default="holograms",
                   help="directory where the hologram will be saved")
    p.add_argument("-q", "--quarterize", action="store_true", help="paste the image into one quadrant")
    p.add_argument("-i", "--invert", action="store_true", help="invert colors of the target image")
    p.add_argument("-alg", "--algorithm", default="gerchberg_saxton",
                   choices=["gerchberg_saxton", "gradient_descent"], help="algorithm")
    p.add_argument("-tol", "--tolerance", default=0, metavar="FLOAT", type=float,
                   help="algorithm stops when error descends under tolerance")
    p.add_argument("-l", "--max_loops", default=42, metavar="INTEGER", type=int,
                   help="algorithm performs no more than max_loops loops")
    p.add_argument("-lr", "--learning_rate", default=0.005, type=float, help="gradient descent learning rate")
    p.add_argument("-wa", "--white_attention", metavar="FLOAT", default=1, type=float,
                   help="attention to white places for gradient_descent")
    p.add_argument("-u", "--unsettle", default=0, metavar="INTEGER", type=int,
                   help="learning rate is unsettle times doubled")
    p.add_argument("-gif", action="store_true", help="create gif from hologram computing evolution")
    p.add_argument("-gif_t", "--gif_type", choices=["h", "i"], default="i", help="type of gif")
    p.add_argument("-gif_skip", default=1, type=int, metavar="INTEGER", help="each gif_skip-th frame")
    p.add_argument("-plot_error", action="store_true", help="plot error evolution")
    p.add_argument("-p", "--preview", action="store_true", help="show expected outcome at the end")
    p.add_argument("-deflect", nargs=2, type=float, metavar=("X_ANGLE", "Y_ANGLE"), default=None,
                   help="add a deflecting phase ramp")
    p.add_argument("-lens", default=None, type=float, metavar="FOCAL_LENGTH", help="add a lens (meters)")
    return p


def cli(argv=None):
    args = build_parser().parse_args(argv)
    args.random_seed = 42
    args.print_info = True
    os.makedirs(args.destination_directory, exist_ok=True)
    return main(args)


if __name__ == "__main__":
    cli()
