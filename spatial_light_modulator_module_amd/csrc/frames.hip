// SLM frame kernels: single-trap holograms, the
// quantisation of phase (+ correction mask) to the SLM's 8-bit levels, and the
// CLI's hologram post-processing (deflecting ramp + lens).
//
//   transform_hologram src/generate_hologram.py:82-87, 178-203 and
//                      src/wavefront_correction.py:440-449
//                        deflect: (h + (c (sin(y u) i + sin(x u) j)) % 2pi) % 2pi
//                        lens:    (h + uint8(phase_shift(r) % 2pi)) % 2pi
//                      in float64 with the reference's operation order and no
//                      contraction (this file builds with -ffp-contract=off), so the result is
//                      the reference's bit for bit; the two sin() values and
//                      the constants are computed on the host as the
//                      reference computes them (Python floats).
//
//   update_hologram   src/move_traps.py:64-68      np.angle(ifft2(255 at (y, x)))
//   display_hologram  src/move_traps.py:135-139    ((h + mask) % 2pi * ct2pi / 2pi).astype(uint8)
//   mask_hologram     src/display_holograms.py:253-266
//                       .npy : PIL 'F'->'L' of ((h + mask) % 2pi) / 2pi * ct2pi
//                       image: PIL 'F'->'L' of (int16 img + mask / 2pi * ct2pi) % ct2pi
//
// The inverse DFT of a single nonzero pixel is a pure plane wave, so the trap
// hologram needs no transform: A[k][l] = 255/S exp(2 pi i (k y/H + l x/W)) and
// its angle is 2 pi n / S with n = ((k y mod H) W + (l x mod W) H) mod S, taken
// in exact integer arithmetic and wrapped to (-pi, pi] as np.angle does. Every
// kernel here is element-wise and HBM-bound (<= 8 B read + 9 B written per
// pixel), fused so a key press in the trap-moving loop is one launch.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <mutex>

#include "../../include/slm_hip.h"

namespace {

constexpr double kTwoPi = 6.283185307179586;  // 2 * np.pi as float64

// Python / numpy float remainder: sign of the divisor (`%` on float64).
__device__ __forceinline__ double py_mod(double a, double b) {
    double r = fmod(a, b);
    if (r != 0.0 && ((r < 0.0) != (b < 0.0))) r += b;
    return r;
}

// numpy float64 -> uint8 astype: C truncation of the value (through int64,
// so out-of-range levels wrap as they do on x86).
__device__ __forceinline__ uint8_t astype_u8(double v) { return (uint8_t)(long long)v; }

// PIL Image.fromarray(float64) is mode 'F' (float32); convert('L') clips to
// [0, 255] and truncates (probed on Pillow 12.2, see tests/test_frames.py).
__device__ __forceinline__ uint8_t pil_f_to_l(double v) {
    const float f = (float)v;
    if (!(f > 0.0f)) return 0;
    if (f >= 255.0f) return 255;
    return (uint8_t)(int)f;
}

__device__ __forceinline__ uint8_t quantize(double h, double m, double ct2pi, int rule) {
    if (rule == SLM_QUANT_ASTYPE) return astype_u8(py_mod(h + m, kTwoPi) * ct2pi / kTwoPi);
    return pil_f_to_l(py_mod(h + m, kTwoPi) / kTwoPi * ct2pi);
}

struct TransformParams {
    const double* in;  // [H][W] hologram or nullptr (zeros, the CLI's analytical case)
    double* out;
    int H, W;
    int deflect, lens;
    double sin_y, sin_x, ramp_c;  // np.sin(y_angle * u), np.sin(x_angle * u), 2 pi px / wavelength
    double lens_c, focal, px;     // 2 pi focal / wavelength, focal length, pixel pitch
};

__global__ void __launch_bounds__(256) transform_kernel(TransformParams p) {
    const long long n = (long long)p.H * p.W;
    for (long long k = blockIdx.x * 256LL + threadIdx.x; k < n; k += (long long)gridDim.x * 256) {
        const int i = (int)(k / p.W), j = (int)(k - (long long)i * p.W);
        double h = p.in ? p.in[k] : 0.0;
        if (p.deflect) {
            // deflect_2pi: const * (sin(y u) * i + sin(x u) * j) % 2pi; then (h + ramp) % 2pi
            const double s = __dadd_rn(__dmul_rn(p.sin_y, (double)i), __dmul_rn(p.sin_x, (double)j));
            const double ramp = py_mod(__dmul_rn(p.ramp_c, s), kTwoPi);
            h = py_mod(__dadd_rn(h, ramp), kTwoPi);
        }
        if (p.lens) {
            // lens(): r = px * sqrt((i - h/2)^2 + (j - w/2)^2)
            //         shift = 2 pi f / wl * (1 - sqrt(1 + r^2 / f^2)), stored as uint8
            const double di = __dsub_rn((double)i, (double)p.H / 2.0);
            const double dj = __dsub_rn((double)j, (double)p.W / 2.0);
            const double r = __dmul_rn(p.px, __dsqrt_rn(__dadd_rn(__dmul_rn(di, di), __dmul_rn(dj, dj))));
            const double q = __ddiv_rn(__dmul_rn(r, r), __dmul_rn(p.focal, p.focal));
            const double shift = __dmul_rn(p.lens_c, __dsub_rn(1.0, __dsqrt_rn(__dadd_rn(1.0, q))));
            const uint8_t level = astype_u8(py_mod(shift, kTwoPi));
            h = py_mod(__dadd_rn(h, (double)level), kTwoPi);
        }
        p.out[k] = h;
    }
}

struct TrapParams {
    const int* ys;
    const int* xs;
    const double* mask;  // [H][W] or nullptr
    double* phase;       // [B][H][W] or nullptr
    uint8_t* frame;      // [B][H][W] or nullptr
    long long holo;
    int H, W, B;
    double ct2pi;
    int rule;
};

__global__ void __launch_bounds__(256) trap_frames_kernel(TrapParams p) {
    const long long n = (long long)p.B * p.holo;
    for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
        const int b = (int)(i / p.holo);
        const long long r = i - (long long)b * p.holo;
        const long long k = r / p.W, l = r - k * p.W;
        const long long y = p.ys[b], x = p.xs[b];
        const long long q = ((k * y) % p.H * p.W + (l * x) % p.W * p.H) % p.holo;
        double th = kTwoPi * (double)q / (double)p.holo;
        if (2 * q > p.holo) th -= kTwoPi;
        if (p.phase) p.phase[i] = th;
        if (p.frame) p.frame[i] = quantize(th, p.mask ? p.mask[r] : 0.0, p.ct2pi, p.rule);
    }
}

template <typename T>
__global__ void __launch_bounds__(256) quantize_kernel(const T* src, const double* mask, long long n, long long holo,
                                                       double ct2pi, int rule, uint8_t* out) {
    for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
        const double m = mask ? mask[i % holo] : 0.0;
        if constexpr (sizeof(T) == 2) {  // int16 image branch of mask_hologram
            out[i] = pil_f_to_l(py_mod((double)src[i] + m / kTwoPi * ct2pi, ct2pi));
        } else {
            out[i] = quantize((double)src[i], m, ct2pi, rule);
        }
    }
}

// Device scratch reused across calls (frames are small; the interactive loop
// calls these repeatedly).
struct Scratch {
    void* p = nullptr;
    size_t cap = 0;
    hipError_t need(size_t bytes) {
        if (bytes <= cap) return hipSuccess;
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
        hipError_t e = hipMalloc(&p, bytes);
        if (e == hipSuccess) cap = bytes;
        return e;
    }
};
std::mutex g_frames_mu;
Scratch g_in, g_mask, g_out, g_phase, g_coords;
hipStream_t g_frames_stream = nullptr;

int grid_for(long long n) { return (int)std::min<long long>(8192, (n + 255) / 256); }

}  // namespace

// shared with slm_capi.hip: error text for slm_last_error(), device selection
int slm_set_error(int code, const char* msg);
int slm_current_device_ready();

#define FR_TRY(expr)                                                    \
    do {                                                                \
        hipError_t e_ = (expr);                                         \
        if (e_ != hipSuccess) return slm_set_error(SLM_ERR_HIP, #expr); \
    } while (0)

extern "C" {

int slm_trap_frames(int batch, int height, int width, const int* ys, const int* xs, const double* mask,
                    double ct2pi, int rule, double* phase_out, unsigned char* frame_out) {
    if (batch < 1 || height < 1 || width < 1 || !ys || !xs) return slm_set_error(SLM_ERR_ARG, "bad trap arguments");
    if (rule != SLM_QUANT_ASTYPE && rule != SLM_QUANT_PIL) return slm_set_error(SLM_ERR_ARG, "unknown rule");
    for (int b = 0; b < batch; ++b)
        if (ys[b] < 0 || ys[b] >= height || xs[b] < 0 || xs[b] >= width)
            return slm_set_error(SLM_ERR_ARG, "trap coordinate outside the image");
    if (int rc = slm_current_device_ready()) return rc;
    std::lock_guard<std::mutex> lk(g_frames_mu);
    if (!g_frames_stream) FR_TRY(hipStreamCreateWithFlags(&g_frames_stream, hipStreamNonBlocking));
    const long long holo = (long long)height * width, n = holo * batch;
    FR_TRY(g_coords.need(2 * sizeof(int) * (size_t)batch));
    int* dys = static_cast<int*>(g_coords.p);
    int* dxs = dys + batch;
    FR_TRY(hipMemcpyAsync(dys, ys, sizeof(int) * batch, hipMemcpyHostToDevice, g_frames_stream));
    FR_TRY(hipMemcpyAsync(dxs, xs, sizeof(int) * batch, hipMemcpyHostToDevice, g_frames_stream));
    TrapParams p{};
    p.ys = dys;
    p.xs = dxs;
    if (mask && frame_out) {
        FR_TRY(g_mask.need(sizeof(double) * holo));
        FR_TRY(hipMemcpyAsync(g_mask.p, mask, sizeof(double) * holo, hipMemcpyHostToDevice, g_frames_stream));
        p.mask = static_cast<const double*>(g_mask.p);
    }
    if (phase_out) {
        FR_TRY(g_phase.need(sizeof(double) * n));
        p.phase = static_cast<double*>(g_phase.p);
    }
    if (frame_out) {
        FR_TRY(g_out.need((size_t)n));
        p.frame = static_cast<uint8_t*>(g_out.p);
    }
    p.holo = holo;
    p.H = height;
    p.W = width;
    p.B = batch;
    p.ct2pi = ct2pi;
    p.rule = rule;
    hipLaunchKernelGGL(trap_frames_kernel, dim3(grid_for(n)), dim3(256), 0, g_frames_stream, p);
    FR_TRY(hipGetLastError());
    if (phase_out)
        FR_TRY(hipMemcpyAsync(phase_out, p.phase, sizeof(double) * n, hipMemcpyDeviceToHost, g_frames_stream));
    if (frame_out) FR_TRY(hipMemcpyAsync(frame_out, p.frame, (size_t)n, hipMemcpyDeviceToHost, g_frames_stream));
    FR_TRY(hipStreamSynchronize(g_frames_stream));
    return 0;
}

int slm_quantize(const void* src, int src_type, const double* mask, int batch, int height, int width, double ct2pi,
                 int rule, unsigned char* out) {
    if (!src || !out || batch < 1 || height < 1 || width < 1) return slm_set_error(SLM_ERR_ARG, "bad arguments");
    if (src_type != SLM_SRC_F64 && src_type != SLM_SRC_I16) return slm_set_error(SLM_ERR_ARG, "unknown source");
    if (src_type == SLM_SRC_F64 && rule != SLM_QUANT_ASTYPE && rule != SLM_QUANT_PIL)
        return slm_set_error(SLM_ERR_ARG, "unknown rule");
    if (int rc = slm_current_device_ready()) return rc;
    std::lock_guard<std::mutex> lk(g_frames_mu);
    if (!g_frames_stream) FR_TRY(hipStreamCreateWithFlags(&g_frames_stream, hipStreamNonBlocking));
    const long long holo = (long long)height * width, n = holo * batch;
    const size_t eb = src_type == SLM_SRC_F64 ? 8 : 2;
    FR_TRY(g_in.need(eb * n));
    FR_TRY(hipMemcpyAsync(g_in.p, src, eb * n, hipMemcpyHostToDevice, g_frames_stream));
    const double* dmask = nullptr;
    if (mask) {
        FR_TRY(g_mask.need(sizeof(double) * holo));
        FR_TRY(hipMemcpyAsync(g_mask.p, mask, sizeof(double) * holo, hipMemcpyHostToDevice, g_frames_stream));
        dmask = static_cast<const double*>(g_mask.p);
    }
    FR_TRY(g_out.need((size_t)n));
    uint8_t* dout = static_cast<uint8_t*>(g_out.p);
    if (src_type == SLM_SRC_F64)
        hipLaunchKernelGGL(quantize_kernel<double>, dim3(grid_for(n)), dim3(256), 0, g_frames_stream,
                           static_cast<const double*>(g_in.p), dmask, n, holo, ct2pi, rule, dout);
    else
        hipLaunchKernelGGL(quantize_kernel<int16_t>, dim3(grid_for(n)), dim3(256), 0, g_frames_stream,
                           static_cast<const int16_t*>(g_in.p), dmask, n, holo, ct2pi, rule, dout);
    FR_TRY(hipGetLastError());
    FR_TRY(hipMemcpyAsync(out, dout, (size_t)n, hipMemcpyDeviceToHost, g_frames_stream));
    FR_TRY(hipStreamSynchronize(g_frames_stream));
    return 0;
}

int slm_transform_hologram(const double* holo_in, int height, int width, int flags, const double* params,
                           double* holo_out) {
    if (!holo_out || !params || height < 1 || width < 1) return slm_set_error(SLM_ERR_ARG, "bad arguments");
    if (flags & ~(SLM_TRANSFORM_DEFLECT | SLM_TRANSFORM_LENS)) return slm_set_error(SLM_ERR_ARG, "unknown flags");
    if (int rc = slm_current_device_ready()) return rc;
    std::lock_guard<std::mutex> lk(g_frames_mu);
    if (!g_frames_stream) FR_TRY(hipStreamCreateWithFlags(&g_frames_stream, hipStreamNonBlocking));
    const long long n = (long long)height * width;
    TransformParams p{};
    if (holo_in) {
        FR_TRY(g_in.need(sizeof(double) * n));
        FR_TRY(hipMemcpyAsync(g_in.p, holo_in, sizeof(double) * n, hipMemcpyHostToDevice, g_frames_stream));
        p.in = static_cast<const double*>(g_in.p);
    }
    FR_TRY(g_phase.need(sizeof(double) * n));
    p.out = static_cast<double*>(g_phase.p);
    p.H = height;
    p.W = width;
    p.deflect = (flags & SLM_TRANSFORM_DEFLECT) != 0;
    p.lens = (flags & SLM_TRANSFORM_LENS) != 0;
    p.sin_y = params[0];
    p.sin_x = params[1];
    p.ramp_c = params[2];
    p.lens_c = params[3];
    p.focal = params[4];
    p.px = params[5];
    hipLaunchKernelGGL(transform_kernel, dim3(grid_for(n)), dim3(256), 0, g_frames_stream, p);
    FR_TRY(hipGetLastError());
    FR_TRY(hipMemcpyAsync(holo_out, p.out, sizeof(double) * n, hipMemcpyDeviceToHost, g_frames_stream));
    FR_TRY(hipStreamSynchronize(g_frames_stream));
    return 0;
}

}  // extern "C"
