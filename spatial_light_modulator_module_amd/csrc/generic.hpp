// Any-size engine of the GS / GD loops: image sides that no float32 radix plan
// (plans.hpp) covers. The reference takes any (h, w) (src/algorithms.py:20-27;
// scipy.fft handles every length), so such plans run in complex float64 with
// row-major state: on the complex128 radix-plan kernels (radix_c128.hpp) where
// both sides have a radix plan ($SLM_ENGINE=float64; their complex64 variant
// runs GS on 13-smooth SLM panels such as 1080 x 1920), on hand-written
// mixed-radix transforms (mixed_radix.hpp) where both sides factor into 2, 3,
// 5, 7, 11, 13, otherwise as 1-D line transforms (direct, or Bluestein's
// chirp-z over a mixed-radix length) plus element-wise kernels. slm_capi.hip
// owns the plan's buffers; this engine owns its work buffers and line plans.
#pragma once
#include <hip/hip_runtime.h>

namespace slm {

struct GenericEngine;

// the slm_plan buffers the engine reads and writes (row-major [B][H][W])
struct GenericView {
    int algo = 0, B = 0, H = 0, W = 0, tt = 0, has_ain = 0, max_loops = 0, nwg = 0;
    // requested arithmetic (kernels.hpp Precision): PREC_F32 takes the complex64
    // radix kernels where both sides have one (GS only), else the engine runs
    // in float64; generic_precision reports what it runs
    int prec = 1;
    long long holo = 0;
    hipStream_t stream = nullptr;
    const void* tgt = nullptr;      // target intensity (uint8 or float32)
    const float* ain = nullptr;     // incoming amplitude [H][W] or nullptr
    const float* phase_in = nullptr;  // GS warm start
    const float2* field0 = nullptr;   // GD initial field (complex64)
    const float* lr = nullptr;        // GD learning rate per iteration
    float* phase_out = nullptr;
    float* e_out = nullptr;           // |C|^2 (GS) / |F|^2 (GD) of the last iteration, float32
    double* partials = nullptr;       // [B][max_loops][nwg][4]
    double* stats = nullptr;          // [B][max_loops][4]
    int* stop = nullptr;              // [B]
    const double* norm = nullptr;     // max(T) [B]
    const double* sum_t2 = nullptr;   // sum T^2 [B]
    // optional kernel-class marks around each iteration launch (timed runs):
    // mark(ctx, class, 1) before, mark(ctx, class, 0) after
    int (*mark)(void* ctx, int cls, int begin) = nullptr;
    void* mark_ctx = nullptr;
};

// statistics blocks per hologram (the partials' nwg): column tiles of the
// mixed-radix / radix-plan back ends, element chunks of the line-transform one
int generic_nwg(int B, int H, int W, long long holo, int algo = 0, int prec = 1);
// the precision a plan of this shape, algorithm and requested precision runs at
int generic_precision(int B, int H, int W, int algo, int prec);
// true for a back end whose runs cannot be graph-captured (none since r06,
// when the rocBLAS DFT products gave way to the line transforms)
bool generic_uses_blas(const GenericEngine* g);
// back end: 2 line transforms (chirp-z), 3 mixed radix, 4 complex128 radix plans,
// 5 complex64 radix plans (slm_plan_engine codes)
int generic_kind(const GenericEngine* g);
int generic_create(const GenericView& v, GenericEngine** out);
void generic_destroy(GenericEngine* g);
// one full run (setup, loops iterations, phase and expected output, statistics),
// enqueued on v.stream
int generic_enqueue(GenericEngine* g, const GenericView& v, int loops, double tol, int checked, float wa,
                    bool phase_set, bool field_set);
// the GD field x after the last run, as complex64 [B][H][W] (device)
int generic_field(GenericEngine* g, const GenericView& v, float2* out);
// unscaled 2-D DFT of complex64 [B][H][W] (device in / out; in may equal out)
int generic_fft2(GenericEngine* g, const GenericView& v, const float2* in, float2* out, int inverse);
// unscaled 2-D DFT of complex128 [B][H][W] (device in / out; in may equal out)
int generic_fft2_z(GenericEngine* g, const GenericView& v, const double2* in, double2* out, int inverse);
// |fft2(exp(i phase))|^2, float32 [B][H][W] (device)
int generic_intensity(GenericEngine* g, const GenericView& v, const float* phase, float* out);

}  // namespace slm
