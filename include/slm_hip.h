/*
 * slm_hip.h — C-ABI of libslm_hip.so, the MI355X (gfx950) hot path of the
 * Gerchberg–Saxton / gradient-descent hologram loops.
 *
 * Reference interfaces replaced (pranislav/Spatial_Light_Modulator_Module,
 * snapshot 2024-10-08; the reference is pure Python and has no FFI, so these
 * are the entry points a ctypes binding of that path binds — see
 * INTEGRATION.md):
 *   slm_gs / slm_plan_* with SLM_ALGO_GS  -> gerchberg_saxton(demanded_output, args)
 *                                            src/algorithms.py:10-49
 *   slm_gd / slm_plan_* with SLM_ALGO_GD  -> gradient_descent(demanded_output, args)
 *                                            src/algorithms.py:60-112 (+ error_f :161,
 *                                            dEdX_complex :179, make_initial_guess
 *                                            "fourier" :153-156)
 *   slm_fft2                              -> scipy.fft.fft2 / ifft2 as called at
 *                                            src/algorithms.py:27,31,34,84,88 (unscaled)
 *   slm_comm_* / slm_plan_gather_phase    -> no reference counterpart: the batch
 *                                            loop of src/generate_hologram_sequence.py:19-31
 *                                            sharded over GPUs, phases gathered over RCCL.
 *
 * Conventions: plain pointers and sizes, C-contiguous row-major host arrays,
 * complex values interleaved (re, im) float32. The caller owns host buffers;
 * the library owns device buffers. Every function returns 0 on success or a
 * negative code; slm_last_error() describes the last failure of the calling
 * thread. Nothing here falls back to the CPU: without a usable gfx950 device
 * every compute entry point fails.
 */
#ifndef SLM_HIP_H
#define SLM_HIP_H

#ifdef __cplusplus
extern "C" {
#endif

#define SLM_ALGO_GS 0
#define SLM_ALGO_GD 1

#define SLM_TGT_U8 0  /* uint8 target; amplitude = float16(sqrt(T)) as numpy does */
#define SLM_TGT_F32 1 /* float32 target; amplitude = sqrtf(T) */

/* arithmetic precision of the transforms (state is complex64 in HBM either way) */
#define SLM_PRECISION_F32 0 /* float32 butterflies and twiddles (default; $SLM_PRECISION=f64 overrides) */
#define SLM_PRECISION_F64 1 /* float64 butterflies and twiddles */

/* kernel classes for timing / roofline queries */
#define SLM_KERNEL_COL_MAIN 0 /* GS column pass, or GD column pass (fused statistics + gradient, or the gradient launch) */
#define SLM_KERNEL_ROW_MAIN 1 /* GS / GD fused row pass */
#define SLM_KERNEL_GD_STATS 2 /* GD statistics column pass */
#define SLM_KERNEL_OTHER 3    /* setup, phase extraction, reductions */
#define SLM_NUM_KERNEL_CLASSES 4

#define SLM_ERR_ARG (-1)
#define SLM_ERR_HIP (-2)
#define SLM_ERR_UNSUPPORTED (-3)
#define SLM_ERR_STATE (-4)
#define SLM_ERR_COMM (-5)

typedef struct slm_plan slm_plan;

/* ---- library ---------------------------------------------------------- */
int slm_init(int device);            /* select the GPU of this process */
int slm_device_count(void);
const char* slm_last_error(void);
const char* slm_version(void);
int slm_supported_length(int n);    /* 1 if n is a supported row/column length */
/* PCI bus id ("0000:05:00.0") of a HIP device: which GPU a rank ran on */
int slm_device_pci_bus_id(int device, char* buf, int len);
/* Measured streaming-copy rate (read + write bytes / s, in GB/s) of two
 * `bytes`-sized device buffers on the current device, `reps` timed copies
 * (16 B per lane, grid-stride): the practical peak next to the 8 TB/s spec
 * (SURVEY.md 8d asks for a measured copy-kernel peak). */
int slm_copy_bandwidth(long long bytes, int reps, double* gbs);

/* ---- plans: device-resident batches ------------------------------------
 * A plan holds `batch` holograms of height x width on the current device.
 * Upload once, run many times (bench), read results.
 * GD plans run their column side as one launch that waits for the hologram's
 * max |F|^2 across workgroups when the whole column grid is resident at once
 * (float32, unchecked runs), else as two launches; $SLM_GD_MODE=auto|fused|
 * two|lin at plan creation picks one ($SLM_GD_FUSE=0 = two). If the one-launch
 * wait ever gives up (other work on the device broke co-residency),
 * slm_plan_sync / slm_plan_read / slm_plan_run_timed redo that run in-process
 * on the two-launch path and the plan keeps that path: the caller sees
 * results, never the fault (slm_plan_gd_recoveries counts such reruns).    */
int slm_plan_create(int algo, int batch, int height, int width, int tgt_type, int has_ain, int max_loops,
                    slm_plan** out);
int slm_plan_destroy(slm_plan* plan);
/* targets [batch][height][width] of tgt_type; norm = max(T) and sum(T^2) are
 * reduced on the device */
int slm_plan_set_target(slm_plan* plan, const void* tgt);
int slm_plan_set_precision(slm_plan* plan, int precision);       /* SLM_PRECISION_* */
int slm_plan_get_precision(slm_plan* plan);
int slm_plan_set_ain(slm_plan* plan, const float* ain);           /* [height][width] sqrt(incoming intensity) */
int slm_plan_set_phase(slm_plan* plan, const float* phase);       /* GS warm start [batch][h][w]; NULL = cold */
int slm_plan_set_field(slm_plan* plan, const float* field_re_im); /* GD initial x [batch][h][w][2]; NULL = fourier */
int slm_plan_set_lr(slm_plan* plan, const float* lr);             /* GD learning rate per iteration [max_loops] */
/* Enqueue one full run (setup + loops iterations + outputs) on the plan's
 * stream. tol as in `while error > tolerance`; checked != 0 evaluates that
 * test on the device after every iteration (required when tol > 0). */
int slm_plan_run(slm_plan* plan, int loops, double tol, int checked, float white_attention);
/* As slm_plan_run, additionally timing every launch with HIP events on the
 * plan's stream; accumulates microseconds and launch counts per kernel class. */
int slm_plan_run_timed(slm_plan* plan, int loops, double tol, int checked, float white_attention,
                       double* us_per_class, int* launches_per_class);
int slm_plan_sync(slm_plan* plan);
/* Device-side stopwatch on the plan stream: slm_plan_mark(plan, 0) and
 * (plan, 1) record the plan's two HIP events; slm_plan_marked_ms waits for
 * mark 1 and returns the device time between them (what bench.py's timed
 * region took on the GPU, graph replays and gathers included). */
int slm_plan_mark(slm_plan* plan, int which);
int slm_plan_marked_ms(slm_plan* plan, double* ms);
int slm_plan_gd_recoveries(slm_plan* plan); /* GD runs redone after a one-launch wait gave up */
/* phase [batch][h][w] float32 (radians, angle convention of np.angle);
 * expected [batch][h][w] float32 = |C|^2 of the last iteration (scale by
 * norm / stats[..][0] for expected_outcome); stats [batch][max_loops][4] =
 * (max E, sum E^2, sum E T, error); iters [batch] iterations executed.
 * Any pointer may be NULL. */
int slm_plan_read(slm_plan* plan, float* phase, float* expected, double* stats, int* iters);
/* norm [batch] and sum T^2 [batch] as reduced on the device */
int slm_plan_read_target_stats(slm_plan* plan, double* norm, double* sum_t2);
/* Override norm = max(T) and sum T^2 per hologram with values the caller
 * computed in float64 from its own target (np.amax(demanded_output),
 * src/algorithms.py:23, and the constant term of error_f :161-162): a
 * float64 target keeps them exact although the device copy of T is float32.
 * Call after slm_plan_set_target. */
int slm_plan_set_target_stats(slm_plan* plan, const double* norm, const double* sum_t2);
/* GD state x [batch][h][w] complex64 (interleaved re, im) after the last run:
 * the field a chunked run continues from with slm_plan_set_field (GIF frames,
 * src/algorithms.py:94-101). */
int slm_plan_read_field(slm_plan* plan, float* field);
/* algorithmic HBM bytes moved by one launch of a kernel class */
long long slm_plan_kernel_bytes(slm_plan* plan, int kernel_class);
/* info[0] = column tile width, info[1] = column workgroups per hologram,
 * info[2] = column threads, info[3] = row threads, info[4] = rows per workgroup,
 * info[5] / info[6] = radix plan keys of rows / columns, info[7] = precision
 * (info must hold 8 ints) */
int slm_plan_info(slm_plan* plan, int* info);
/* panel widths (log2) of the plan's two blocked device layouts: X (row-pass
 * output, column-pass input, target) and Y (column-pass output, GD field) */
int slm_plan_layout(slm_plan* plan, int* x_log2, int* y_log2);
/* transform engine of the GS iteration kernels: 0 = Stockham pair (LDS
 * exchange before every pass), 1 = wave-shuffle pair (fft_shuffle.hpp: 1024-
 * point lines, float32; v_permlane swaps for four of the six exchanges; the
 * GS and GD iteration kernels), 2 = line transforms (float64 1-D transforms
 * along rows and transposed columns, Bluestein's chirp-z for a side with a
 * prime factor above 13), 3 = mixed radix (float64 in-place radix-2..13
 * kernels: other sides without a float32 radix plan), 4 = complex128 radix
 * plans (float64 Stockham kernels with complex128 state: 2^k / 768 sides
 * under $SLM_ENGINE=float64), 5 = complex64 radix plans (the same kernels at
 * float32: GS on 13-smooth SLM panel sides such as 1080 x 1920, float32
 * precision; slm_plan_set_precision(F64) moves such a plan to engine 3) */
int slm_plan_engine(slm_plan* plan, int* col_engine, int* row_engine);
/* HIP device the plan lives on */
int slm_plan_device(slm_plan* plan);

/* Diagnostics: per-workgroup phase timestamps (s_memrealtime, 100 MHz: tile
 * start, loads complete, transforms done, stores complete, kernel entry) plus
 * the wave's HW_ID and XCC_ID, of the last launch of a kernel class,
 * [batch][workgroups][8]. Needs a library built with
 * -DSLM_TRACE=1 and SLM_TRACE_BUF=1 in the environment at plan creation. */
int slm_plan_read_trace(slm_plan* plan, int kernel_class, unsigned long long* out);

/* ---- one-shot helpers (upload, run, read) ------------------------------ */
int slm_gs(const void* tgt, int tgt_type, const float* ain, int batch, int height, int width, int max_loops,
           double tol, const float* init_phase, float* out_phase, float* out_expected, double* out_stats,
           int* out_iters);
int slm_gd(const void* tgt, int tgt_type, const float* ain, int batch, int height, int width, int max_loops,
           double tol, const float* init_field, const float* lr, float white_attention, float* out_phase,
           float* out_expected, double* out_stats, int* out_iters);

/* One process, several GPUs (SURVEY.md 8b's slm_gs_multi): the batch is cut
 * into n_gpus contiguous shards (the first batch % n_gpus one hologram larger,
 * as parallel.shard_counts), shard r runs on devices[r] (NULL = 0..n_gpus-1;
 * a device may repeat) from its own host thread with its own plan and stream,
 * and lands in its slice of the caller's arrays, each GPU copying over its own
 * link concurrently. Arguments otherwise as slm_gs; results are bitwise those
 * of slm_gs on each shard. The reference counterpart is the frame loop of
 * src/generate_hologram_sequence.py:19-31 run as one batch. */
int slm_gs_multi(int n_gpus, const int* devices, const void* tgt, int tgt_type, const float* ain, int batch,
                 int height, int width, int max_loops, double tol, const float* init_phase, float* out_phase,
                 float* out_expected, double* out_stats, int* out_iters);
/* Per-shard timing of the calling process's last slm_gs_multi: wall_ms[r] =
 * shard r's whole thread (plan, upload, run, read back), run_ms[r] = its run
 * alone (enqueue to stream drained); up to max_shards values each (either
 * pointer may be NULL). Returns the number of shards of that call (0 if none). */
int slm_gs_multi_timing(int max_shards, double* wall_ms, double* run_ms);

/* unscaled 2-D C2C transform of [batch][h][w] complex64 (test entry) */
int slm_fft2(const float* in_re_im, float* out_re_im, int batch, int height, int width, int inverse);
/* unscaled 2-D C2C transform of [batch][h][w] complex128 in float64 arithmetic
 * (any shape: mixed-radix kernels where both sides factor into 2..13, else
 * chirp-z line transforms) -> the float64 scipy.fft.ifft2 of move_traps.update_hologram,
 * src/move_traps.py:66 (times h w) */
int slm_fft2_c128(const double* in_re_im, double* out_re_im, int batch, int height, int width, int inverse);
/* frees the float64 engines slm_fft2_c128 keeps per (device, batch, h, w)
 * (a few shapes; the drop-in's clear_plans calls it) */
int slm_release_caches(void);

/* ---- multi-GPU (one process per GPU, RCCL over xGMI) ------------------- */
int slm_comm_unique_id(unsigned char* id128);
int slm_comm_init(int nranks, int rank, const unsigned char* id128);
int slm_comm_destroy(void);
/* Gather every rank's phase output to `root`: rank r contributes its plan's
 * batch (counts[r] holograms, same h x w everywhere); on root, host_out
 * receives sum(counts) x h x w float32 in rank order (may be NULL to leave
 * the gathered array on the device). Collective; enqueued on the plan stream,
 * which is synchronised before returning only when host_out is given (a
 * device-side gather stays stream-ordered with the plan's later work). */
int slm_plan_gather_phase(slm_plan* plan, const int* counts, int root, float* host_out);
/* The same collective for the per-iteration statistics that become each
 * hologram's error_evolution (src/generate_hologram_sequence.py:19-31 keeps one
 * per frame): on root, stats_out receives sum(counts) x
 * max_loops x 4 doubles (max E, sum E^2, sum E T, error) and iters_out
 * sum(counts) ints (iterations executed, -1 = all), rank order; either may be
 * NULL. */
int slm_plan_gather_stats(slm_plan* plan, const int* counts, int root, double* stats_out, int* iters_out);
/* Diagnostics of the phase gather (collective, every rank calls it): drains
 * the plan stream, then times `reps` device-side slm_plan_gather_phase calls
 * with HIP events on the plan stream; *ms = average per gather on this rank,
 * *bytes_out = bytes this rank sends to root per gather (0 on root, whose own
 * slab is a device-local copy). */
int slm_plan_time_gather(slm_plan* plan, const int* counts, int root, int reps, double* ms, long long* bytes_out);
/* Element offsets of a rank-order gather: offsets[r] = per_item x sum(counts[:r]),
 * offsets[nranks] = the total (offsets holds nranks + 1 values). The arithmetic
 * every gather above uses; host-only, needs no device. */
int slm_gather_layout(int nranks, const int* counts, long long per_item, long long* offsets);

/* ---- SLM frames: trap holograms and 8-bit quantisation ------------------
 * (element-wise, one launch per call, host buffers in/out)
 * slm_trap_frames      -> update_hologram(black_image, coords, which)
 *                         src/move_traps.py:64-68 (phase_out, float64, the
 *                         angle of ifft2 of a single 255 pixel at (ys[b], xs[b]))
 *                         fused with display_hologram's quantisation
 *                         src/move_traps.py:135-139 (frame_out, rule ASTYPE)
 * slm_quantize         -> mask_hologram(path, mask_arr, ct2pi)
 *                         src/display_holograms.py:253-266 (.npy branch: SRC_F64 +
 *                         rule PIL; image branch: SRC_I16) and display_hologram
 *                         (SRC_F64 + rule ASTYPE)
 * mask is [height][width] float64 (broadcast over the batch) or NULL; any
 * output pointer may be NULL.                                              */
#define SLM_QUANT_ASTYPE 0 /* ((h + mask) % 2pi * ct2pi / 2pi).astype(uint8) */
#define SLM_QUANT_PIL 1    /* PIL 'F'->'L' (clip, truncate) of ((h + mask) % 2pi) / 2pi * ct2pi */
#define SLM_SRC_F64 0      /* phase hologram, float64 */
#define SLM_SRC_I16 1      /* 8-bit hologram image widened to int16 (PIL 'L' -> np.int16) */
int slm_trap_frames(int batch, int height, int width, const int* ys, const int* xs, const double* mask,
                    double ct2pi, int rule, double* phase_out, unsigned char* frame_out);
int slm_quantize(const void* src, int src_type, const double* mask, int batch, int height, int width, double ct2pi,
                 int rule, unsigned char* out);

/* ---- CLI post-processing ------------------------------
 * slm_transform_hologram -> transform_hologram(hologram, args)
 *                           src/generate_hologram.py:82-87: deflect_hologram
 *                           (:178-181 with wavefront_correction.deflect_2pi,
 *                           src/wavefront_correction.py:440-449) and add_lens
 *                           (:184-203, lens() stored as uint8). float64,
 *                           reference operation order, bit for bit.
 * holo_in [height][width] float64 or NULL (zeros); params = {sin(y_angle u),
 * sin(x_angle u), 2 pi px_distance / wavelength, 2 pi focal / wavelength,
 * focal, px_distance} as the reference computes them on the host.
 * slm_fft2_intensity     -> show_expected_outcome's |fft2(exp(1j h))|^2
 *                           (src/generate_hologram.py:24-34) on the plan
 *                           kernels (complex64), row-major float32 out.   */
#define SLM_TRANSFORM_DEFLECT 1
#define SLM_TRANSFORM_LENS 2
int slm_transform_hologram(const double* holo_in, int height, int width, int flags, const double* params,
                           double* holo_out);
int slm_fft2_intensity(const float* phase, int batch, int height, int width, float* intensity_out);

#ifdef __cplusplus
}
#endif
#endif /* SLM_HIP_H */
