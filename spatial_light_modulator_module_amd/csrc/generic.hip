// Any-size engine (generic.hpp): GS / GD iterations on image sides that no
// float32 radix plan covers, in complex float64 like the reference's loop.
//
// Three transform back ends:
//  * radix plans (radix_c128.hpp; the default where both sides have a radix
//    plan, plans.hpp): the mixed-radix launch structure and contract on
//    compile-time Stockham transforms with the line in registers and LDS
//    exchanges. Complex128 on 2^k and 768 sides (reached through
//    $SLM_ENGINE=float64); complex64 for GS at float32 precision where a side
//    is a 13-smooth SLM panel length (600 .. 1920, plans.hpp variant 3) --
//    e.g. 1080 x 1920 -- the float32 engine's numerics on these shapes;
//  * mixed radix (mixed_radix.hpp, mr_inst.hip; the default wherever both
//    sides factor into 2, 3, 5, 7, 11, 13 and fit a workgroup's LDS): the
//    iteration is two fused launches -- column pass (forward transform,
//    projection and statistics, inverse transform) and row pass (inverse,
//    projection, forward) -- O(N log N), hand-written kernels only;
//  * line transforms (any other side, e.g. one with a large prime factor, or
//    $SLM_GENERIC_ENGINE=bluestein): each 2-D transform is a pass of 1-D
//    transforms along the rows, a tiled transpose, a pass along the (former)
//    columns and a transpose back, with element-wise kernels between the
//    transforms. A side with a mixed-radix plan transforms directly; any other
//    side by Bluestein's chirp-z over a mixed-radix length M >= 2n - 1
//    (mr_line_kernel, mr_inst.hip) -- O(N log N) for every length, hand-written
//    kernels only. (Until r05 these sides were products with dense DFT matrices
//    on rocBLAS ZGEMM, O(N^3).)
//
// Numerics follow the reference's float64 path (src/algorithms.py:10-49,
// 60-112): complex128 state, float64 statistics (E = |C|^2 unrounded),
// amplitudes as numpy forms them (sqrt(uint8) -> float16, sqrt(float32) ->
// float32), the cold start's ifft2 of a float amplitude rounded to complex64.
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <cmath>
#include <vector>

#include "../../include/slm_hip.h"
#include "generic.hpp"
#include "kernels.hpp"
#include "mixed_radix.hpp"
#include "radix_c128.hpp"

int slm_set_error(int code, const char* msg);  // slm_capi.hip

namespace slm {

struct GenericEngine {
    // mixed-radix back end: line plans (twiddles, digit reversal) of both sides
    bool mr = false;
    // complex128 radix-plan back end (mr is set too: same launch structure and
    // buffers; its line plans hold Stockham twiddle tables and the identity order)
    bool rz = false;
    int rkey = -1, ckey = -1;  // plan keys (plans.hpp) of the row / column transforms
    int rz_cw = 0;             // columns per column tile
    int rz_lay = 0;            // state layout between the passes (radix_c128.hpp LAY_RM / LAY_B2)
    int prec = PREC_F64;       // PREC_F32: complex64 radix kernels (the state buffers then hold float2)
    float* tgt_blk = nullptr;  // the target as float in the radix kernels' B2 layout (rebuilt per run)
    bool big = false;        // a radix outside mr::small_radix in either plan (7, 11, 13)
    mr::LinePlan pw, ph;     // row (length W) and column (length H) transforms
    int rpw = 1;             // rows per row tile
    int cw_log2 = 0;         // columns per column tile = 2^cw_log2
    int nwg_col = 0;         // column tiles per hologram
    std::vector<void*> tables;  // device twiddle / reversal tables
    float* ain_rev = nullptr;   // a_in with rows in the row transform's digit-reversed order (has_ain)
    // line-transform back end: the row (length W) and column (length H) transforms
    mr::LineArgs lw, lh;
    bool big_w = false, big_h = false;  // their plans need the odd-radix kernels
    // state (row-major complex128 [B][H][W])
    double2* a = nullptr;    // lines GS: A; GD: the inverse-transformed gradient g. Mixed radix: row-pass output
    double2* b = nullptr;    // lines GS: B, then C in place; GD: u, then F in place. Mixed radix: column-pass output
    double2* d = nullptr;    // lines GS: D; GD: G
    double2* x = nullptr;    // GD: the field x
    double2* tmp = nullptr;  // lines: the row-transformed image
    double2* tmp2 = nullptr; // lines: the transposed image [B][W][H]
};

namespace {

constexpr int kGT = 256;  // threads per block of the element-wise kernels

#define G_HIP(expr)                                                                      \
    do {                                                                                 \
        hipError_t e_ = (expr);                                                          \
        if (e_ != hipSuccess) return slm_set_error(SLM_ERR_HIP, hipGetErrorString(e_));  \
    } while (0)

int grid_of(long long n) { return (int)std::min<long long>(16384, (n + kGT - 1) / kGT); }

// numpy's amplitude of the target: sqrt(uint8) is float16,
// sqrt(float32) float32; then widened (the loop multiplies it with complex128)
__device__ __forceinline__ double g_amp(const void* tgt, int tt, long long i) {
    if (tt == TGT_U8) return (double)TgtLoad<TGT_U8>::amp(TgtLoad<TGT_U8>::load(tgt, i));
    return (double)(float)sqrt((double)static_cast<const float*>(tgt)[i]);
}
__device__ __forceinline__ double g_t(const void* tgt, int tt, long long i) {
    return tt == TGT_U8 ? (double)static_cast<const uint8_t*>(tgt)[i] : (double)static_cast<const float*>(tgt)[i];
}
__device__ __forceinline__ double g_ain(const float* ain, long long i, long long holo) {
    return ain ? (double)ain[i % holo] : 1.0;
}
// a exp(i angle(z)) == a z / |z|, angle(0) = 0 -> a (src/algorithms.py:30,33)
__device__ __forceinline__ double2 g_unit(double2 z, double a) {
    const double n2 = z.x * z.x + z.y * z.y;
    if (n2 == 0.0) return make_double2(a, 0.0);
    const double r = a / sqrt(n2);
    return make_double2(z.x * r, z.y * r);
}

__global__ void __launch_bounds__(kGT) k_unit(const double2* A, double2* B, const float* ain, long long holo,
                                              long long n) {
    for (long long i = blockIdx.x * (long long)kGT + threadIdx.x; i < n; i += (long long)gridDim.x * kGT)
        B[i] = g_unit(A[i], g_ain(ain, i, holo));
}
// warm start: B = a_in exp(1j phi) with exp of a float32 phase in complex64 (numpy)
__global__ void __launch_bounds__(kGT) k_warm(const float* phi, double2* B, const float* ain, long long holo,
                                              long long n) {
    for (long long i = blockIdx.x * (long long)kGT + threadIdx.x; i < n; i += (long long)gridDim.x * kGT) {
        double s, c;
        sincos((double)phi[i], &s, &c);
        const double a = g_ain(ain, i, holo);
        B[i] = make_double2((double)(float)c * a, (double)(float)s * a);
    }
}
// a_T + 0i (the cold start's ifft2(sqrt(T)) and the "fourier" guess)
__global__ void __launch_bounds__(kGT) k_amp(const void* tgt, int tt, double2* D, long long n) {
    for (long long i = blockIdx.x * (long long)kGT + threadIdx.x; i < n; i += (long long)gridDim.x * kGT)
        D[i] = make_double2(g_amp(tgt, tt, i), 0.0);
}
// ifft2 of a float16 / float32 amplitude is complex64 in the reference (src/algorithms.py:27)
__global__ void __launch_bounds__(kGT) k_round_c64(double2* A, long long n) {
    for (long long i = blockIdx.x * (long long)kGT + threadIdx.x; i < n; i += (long long)gridDim.x * kGT)
        A[i] = make_double2((double)(float)A[i].x, (double)(float)A[i].y);
}
// "fourier" guess a_in exp(1j angle(ifft2(sqrt T))): angle of complex64 is float32, exp complex64
// (src/algorithms.py:153-156)
__global__ void __launch_bounds__(kGT) k_fourier(const double2* A, double2* X, const float* ain, long long holo,
                                                 long long n) {
    for (long long i = blockIdx.x * (long long)kGT + threadIdx.x; i < n; i += (long long)gridDim.x * kGT) {
        const float ang = atan2f((float)A[i].y, (float)A[i].x);
        double s, c;
        sincos((double)ang, &s, &c);
        const double a = g_ain(ain, i, holo);
        X[i] = make_double2((double)(float)c * a, (double)(float)s * a);
    }
}
__global__ void __launch_bounds__(kGT) k_c64_to_c128(const float2* in, double2* out, long long n) {
    for (long long i = blockIdx.x * (long long)kGT + threadIdx.x; i < n; i += (long long)gridDim.x * kGT)
        out[i] = make_double2((double)in[i].x, (double)in[i].y);
}
__global__ void __launch_bounds__(kGT) k_c128_to_c64(const double2* in, float2* out, long long n) {
    for (long long i = blockIdx.x * (long long)kGT + threadIdx.x; i < n; i += (long long)gridDim.x * kGT)
        out[i] = make_float2((float)in[i].x, (float)in[i].y);
}
// Mixed-radix GD keeps its field x with every row in the digit-reversed order
// of the row transform (element e of a row holds column rev[e]: the row pass
// reads and writes it in place, coalesced); these read it back row-major.
__global__ void __launch_bounds__(kGT) k_phase_rev(const double2* X, float* phase, const int* rev, int W, long long n) {
    for (long long i = blockIdx.x * (long long)kGT + threadIdx.x; i < n; i += (long long)gridDim.x * kGT) {
        const long long r = i / W;
        const int e = (int)(i - r * W);
        phase[r * W + rev[e]] = (float)atan2(X[i].y, X[i].x);
    }
}
__global__ void __launch_bounds__(kGT) k_c128_to_c64_rev(const double2* X, float2* out, const int* rev, int W,
                                                        long long n) {
    for (long long i = blockIdx.x * (long long)kGT + threadIdx.x; i < n; i += (long long)gridDim.x * kGT) {
        const long long r = i / W;
        const int e = (int)(i - r * W);
        out[r * W + rev[e]] = make_float2((float)X[i].x, (float)X[i].y);
    }
}
// a_in [H][W] with every row in that order (read by the iteration row passes)
__global__ void __launch_bounds__(kGT) k_ain_rev(const float* ain, float* out, const int* rev, int W, long long n) {
    for (long long i = blockIdx.x * (long long)kGT + threadIdx.x; i < n; i += (long long)gridDim.x * kGT) {
        const long long r = i / W;
        out[i] = ain[r * W + rev[(int)(i - r * W)]];
    }
}
// the target (uint8 or float32, row-major) as float in the complex128 radix
// kernels' B2 layout (radix_c128.hpp, b2_index): the column passes' reads of it
// are then contiguous like their field reads
__global__ void __launch_bounds__(kGT) k_tgt_b2(const void* tgt, int tt, float* out, int H, int W, long long n) {
    const long long holo = (long long)H * W;
    for (long long i = blockIdx.x * (long long)kGT + threadIdx.x; i < n; i += (long long)gridDim.x * kGT) {
        const long long b = i / holo, r = i - b * holo;
        const int y = (int)(r / W), x = (int)(r - (long long)y * W);
        const float t = tt == TGT_U8 ? (float)static_cast<const uint8_t*>(tgt)[i] : static_cast<const float*>(tgt)[i];
        out[b * holo + rz::b2_index(y, x, H)] = t;
    }
}
__global__ void __launch_bounds__(kGT) k_phase(const double2* A, float* phase, long long n) {
    for (long long i = blockIdx.x * (long long)kGT + threadIdx.x; i < n; i += (long long)gridDim.x * kGT)
        phase[i] = (float)atan2(A[i].y, A[i].x);
}
__global__ void __launch_bounds__(kGT) k_phase_exp(const float* phase, double2* B, long long n) {
    for (long long i = blockIdx.x * (long long)kGT + threadIdx.x; i < n; i += (long long)gridDim.x * kGT) {
        double s, c;
        sincos((double)phase[i], &s, &c);
        B[i] = make_double2(c, s);
    }
}
__global__ void __launch_bounds__(kGT) k_abs2(const double2* C, float* out, long long n) {
    for (long long i = blockIdx.x * (long long)kGT + threadIdx.x; i < n; i += (long long)gridDim.x * kGT)
        out[i] = (float)(C[i].x * C[i].x + C[i].y * C[i].y);
}
// complex64 engine: exp(1j phase) of a float32 phase is complex64 (numpy), |C|^2 float32
__global__ void __launch_bounds__(kGT) k_phase_exp_c64(const float* phase, float2* B, long long n) {
    for (long long i = blockIdx.x * (long long)kGT + threadIdx.x; i < n; i += (long long)gridDim.x * kGT) {
        double s, c;
        sincos((double)phase[i], &s, &c);
        B[i] = make_float2((float)c, (float)s);
    }
}
__global__ void __launch_bounds__(kGT) k_abs2_c64(const float2* C, float* out, long long n) {
    for (long long i = blockIdx.x * (long long)kGT + threadIdx.x; i < n; i += (long long)gridDim.x * kGT)
        out[i] = C[i].x * C[i].x + C[i].y * C[i].y;
}

// Statistics block `blockIdx.x` of hologram `blockIdx.y`: a contiguous chunk.
struct ChunkOf {
    long long lo, hi;
    __device__ ChunkOf(long long holo, int nwg) {
        const long long chunk = (holo + nwg - 1) / nwg;
        lo = (long long)blockIdx.x * chunk;
        hi = lo + chunk < holo ? lo + chunk : holo;
    }
};
__device__ __forceinline__ void store_partials(double* partials, int b, int iter, int max_loops, int nwg, double mx,
                                               double s2, double st) {
    block_reduce_stats<kGT>(mx, s2, st);
    if (threadIdx.x == 0) {
        double* dst = partials + (((long long)b * max_loops + iter) * nwg + blockIdx.x) * 4;
        dst[0] = mx;
        dst[1] = s2;
        dst[2] = st;
        dst[3] = 0.0;
    }
}

// GS: E = |C|^2 and its statistics, expected output, D = a_T C/|C| (src/algorithms.py:33,36-38).
// A hologram whose checked run has stopped keeps D (and E): its later products repeat.
__global__ void __launch_bounds__(kGT) k_gs_project(const double2* C, const void* tgt, int tt, double2* D,
                                                    float* e_out, double* partials, const int* stop, int iter,
                                                    int checked, int write_e, long long holo, int nwg, int max_loops) {
    const int b = blockIdx.y;
    if (checked && iter > stop[b]) return;
    const ChunkOf ch(holo, nwg);
    double mx = 0.0, s2 = 0.0, st = 0.0;
    for (long long r = ch.lo + threadIdx.x; r < ch.hi; r += kGT) {
        const long long i = (long long)b * holo + r;
        const double2 z = C[i];
        const double e = z.x * z.x + z.y * z.y;
        mx = fmax(mx, e);
        s2 += e * e;
        st += e * g_t(tgt, tt, i);
        if (write_e) e_out[i] = (float)e;
        D[i] = g_unit(z, g_amp(tgt, tt, i));
    }
    store_partials(partials, b, iter, max_loops, nwg, mx, s2, st);
}

// GD: u = x / |x| a_in (src/algorithms.py:84; |x| = 0 gives NaN as there)
__global__ void __launch_bounds__(kGT) k_gd_u(const double2* X, double2* U, const float* ain, long long holo,
                                              long long n) {
    for (long long i = blockIdx.x * (long long)kGT + threadIdx.x; i < n; i += (long long)gridDim.x * kGT) {
        const double2 x = X[i];
        const double r = g_ain(ain, i, holo) / sqrt(x.x * x.x + x.y * x.y);
        U[i] = make_double2(x.x * r, x.y * r);
    }
}
// GD: P = |F|^2 statistics (max for the normalisation, src/algorithms.py:85-86) and output
__global__ void __launch_bounds__(kGT) k_gd_stats(const double2* F, const void* tgt, int tt, float* e_out,
                                                  double* partials, const int* stop, int iter, int checked, int write_e,
                                                  long long holo, int nwg, int max_loops) {
    const int b = blockIdx.y;
    if (checked && iter > stop[b]) return;
    const ChunkOf ch(holo, nwg);
    double mx = 0.0, s2 = 0.0, st = 0.0;
    for (long long r = ch.lo + threadIdx.x; r < ch.hi; r += kGT) {
        const long long i = (long long)b * holo + r;
        const double2 z = F[i];
        const double e = z.x * z.x + z.y * z.y;
        mx = fmax(mx, e);
        s2 += e * e;
        st += e * g_t(tgt, tt, i);
        if (write_e) e_out[i] = (float)e;
    }
    store_partials(partials, b, iter, max_loops, nwg, mx, s2, st);
}
// one (hologram, iteration) slab -> stats, and the tolerance test (src/algorithms.py:29,83,92)
__global__ void __launch_bounds__(256) k_reduce_iter(StatsParams p) {
    const int b = blockIdx.x;
    if (p.iter > p.stop_iter[b]) return;
    __shared__ double o[4];
    reduce_slab(p, b, p.iter, o);
    if (threadIdx.x == 0) {
        for (int k = 0; k < 4; ++k) p.stats[((long long)b * p.max_loops + p.iter) * 4 + k] = o[k];
        if (p.tol >= 0.0 && !(o[3] > p.tol)) p.stop_iter[b] = p.iter;
    }
}
// GD: G = mask F (s P - T), s = norm / max P, mask = 1 + wa T / 255 (src/algorithms.py:80,85-88)
__global__ void __launch_bounds__(kGT) k_gd_grad(const double2* F, const void* tgt, int tt, const double* stats,
                                                 const double* norm, double2* G, float wa, const int* stop, int iter,
                                                 int checked, long long holo, int max_loops, long long n) {
    for (long long i = blockIdx.x * (long long)kGT + threadIdx.x; i < n; i += (long long)gridDim.x * kGT) {
        const int b = (int)(i / holo);
        if (checked && iter > stop[b]) continue;
        const double s = norm[b] / stats[((long long)b * max_loops + iter) * 4];
        const double2 z = F[i];
        const double t = g_t(tgt, tt, i);
        // numpy's mask dtype: float32 for a float32 target (the python float scalars are
        // weak), float64 for uint8 (src/algorithms.py:80)
        const double mask = tt == TGT_U8 ? 1.0 + (double)wa * t / 255.0
                                         : (double)(1.0f + __fdiv_rn(__fmul_rn(wa, (float)t), 255.0f));
        const double w = mask * ((z.x * z.x + z.y * z.y) * s - t);
        G[i] = make_double2(z.x * w, z.y * w);
    }
}
// GD: dEdF = ifft2(G) a_in, dEdX_complex (src/algorithms.py:179-185), x -= lr dEdX (:91)
__global__ void __launch_bounds__(kGT) k_gd_update(double2* X, const double2* g, const float* ain, const float* lr,
                                                   const int* stop, int iter, int checked, double inv_s,
                                                   long long holo, long long n) {
    const double l = (double)lr[iter];
    for (long long i = blockIdx.x * (long long)kGT + threadIdx.x; i < n; i += (long long)gridDim.x * kGT) {
        const int b = (int)(i / holo);
        if (checked && iter > stop[b]) continue;
        const double a = g_ain(ain, i, holo) * inv_s;
        const double gx = g[i].x * a, gy = g[i].y * a;
        double2 x = X[i];
        const double ax2 = x.x * x.x + x.y * x.y;
        const double ax = sqrt(ax2);
        const double re = x.x * gx + x.y * gy;
        x.x -= l * ((gx - x.x * (re / ax2)) / ax);
        x.y -= l * ((gy - x.y * (re / ax2)) / ax);
        X[i] = x;
    }
}

// [B][R][C] -> [B][C][R] complex128 through 32 x 32 LDS tiles (the line
// transforms run along contiguous rows only)
__global__ void __launch_bounds__(256) k_transpose(const double2* in, double2* out, int R, int C) {
    __shared__ double2 tile[32][33];
    const long long hb = (long long)blockIdx.z * R * C;
    const int c0 = blockIdx.x * 32, r0 = blockIdx.y * 32;
    const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
    for (int k = ty; k < 32; k += 8) {
        const int r = r0 + k, c = c0 + tx;
        if (r < R && c < C) tile[k][tx] = in[hb + (long long)r * C + c];
    }
    __syncthreads();
    for (int k = ty; k < 32; k += 8) {
        const int c = c0 + k, r = r0 + tx;
        if (r < R && c < C) out[hb + (long long)c * R + r] = tile[tx][k];
    }
}

// 1-D transforms of `lines` rows of the line plan's length
int line_pass(const GenericEngine* g, const mr::LineArgs& base, bool big, const double2* in, double2* out,
              long long lines, bool inverse, hipStream_t st) {
    if (lines > 0x7fffffffLL) return slm_set_error(SLM_ERR_UNSUPPORTED, "line transforms: too many lines");
    mr::LineArgs a = base;
    a.in = in;
    a.out = out;
    a.inverse = inverse ? 1 : 0;
    if (mr::mr_line_launch(big, a, (int)lines, (size_t)a.pl.n * sizeof(double2), st))
        return slm_set_error(SLM_ERR_HIP, "line transform launch failed");
    return 0;
}

// out = op(in): forward or inverse (unscaled) 2-D transform of [B][H][W]
// complex128 as rows -> transpose -> rows -> transpose; in may equal out
int dft2(GenericEngine* g, const GenericView& v, const double2* in, double2* out, bool inverse) {
    hipStream_t st = v.stream;
    if (int rc = line_pass(g, g->lw, g->big_w, in, g->tmp, (long long)v.B * v.H, inverse, st)) return rc;
    hipLaunchKernelGGL(k_transpose, dim3((v.W + 31) / 32, (v.H + 31) / 32, v.B), dim3(256), 0, st, g->tmp, g->tmp2,
                       v.H, v.W);
    if (int rc = line_pass(g, g->lh, g->big_h, g->tmp2, g->tmp2, (long long)v.B * v.W, inverse, st)) return rc;
    hipLaunchKernelGGL(k_transpose, dim3((v.H + 31) / 32, (v.W + 31) / 32, v.B), dim3(256), 0, st, g->tmp2, out,
                       v.W, v.H);
    G_HIP(hipGetLastError());
    return 0;
}

StatsParams stats_of(const GenericView& v, double tol, int iter) {
    StatsParams s{};
    s.partials = v.partials;
    s.stats = v.stats;
    s.stop_iter = v.stop;
    s.norm = v.norm;
    s.sum_t2 = v.sum_t2;
    s.inv_s = 1.0 / (double)v.holo;
    s.tol = tol;
    s.max_loops = v.max_loops;
    s.nwg = v.nwg;
    s.iter = iter;
    return s;
}

// ------------------------------------------------------------------------
// mixed-radix back end (host side)
// ------------------------------------------------------------------------
// DIF stage radices of a length: 8s (then a 4 or a 2) for the powers of two,
// then 3, 5, 7, 11, 13; false if another prime divides n or n is too long
bool mr_radices(int n, std::vector<int>& rad) {
    rad.clear();
    if (n < 1 || n > mr::kMaxLine) return false;
    int t = n, twos = 0;
    while (t % 2 == 0) {
        t /= 2;
        ++twos;
    }
    while (twos >= 3 && twos != 4) {
        rad.push_back(8);
        twos -= 3;
    }
    if (twos == 4) {
        rad.push_back(4);
        rad.push_back(4);
    } else if (twos == 2) {
        rad.push_back(4);
    } else if (twos == 1) {
        rad.push_back(2);
    }
    for (int p : {3, 5, 7, 11, 13})
        while (t % p == 0) {
            rad.push_back(p);
            t /= p;
        }
    return t == 1 && (int)rad.size() <= mr::kMaxPass;
}

// $SLM_GENERIC_ENGINE=bluestein (alias: gemm, r05's name of that back end)
// sends every side through the line transforms, chirp-z included
bool mr_forced_lines() {
    const char* e = std::getenv("SLM_GENERIC_ENGINE");
    return e && (!std::strcmp(e, "bluestein") || !std::strcmp(e, "gemm"));
}

bool mr_shape_ok(int H, int W) {
    std::vector<int> r;
    return !mr_forced_lines() && mr_radices(H, r) && mr_radices(W, r);
}

bool mr_big(int H, int W) {
    std::vector<int> rh, rw;
    if (!mr_radices(H, rh) || !mr_radices(W, rw)) return false;
    for (const auto* v : {&rh, &rw})
        for (int r : *v)
            if (!mr::small_radix(r)) return true;
    return false;
}

// Tiles of the two launches. A launch of `wgs` workgroups of `e` elements on
// `cus` CUs that hold `occ` of them at once takes about rounds x (workgroups
// per CU in a round) x e: so the rows per row tile / columns per column tile
// minimise ceil(wgs / (cus occ)) * min(occ, ceil(wgs / cus)) * e (a grid one
// workgroup too large for a round doubles the launch: 1080 rows in 540
// two-row tiles on 512 slots did, 62.6 against ~35 us). Column tiles that tie
// go to 2 columns (32-B row segments), then the narrower: 1080 x 1920 columns
// in tiles of 2 measured 48.2 us against 58.0 in tiles of 1 and 55.0 in tiles
// of 4 (profiles/r05/mr_tiles_s13.txt); row tiles that tie go to the wider.
// $SLM_MR_RPW / $SLM_MR_CW override.
struct MrTiling {
    int rpw = 1, cw_log2 = 0;
};
MrTiling mr_tiling(int B, int H, int W) {
    MrTiling t;
    const bool big = mr_big(H, W);
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1)
        cus = 256;
    auto cost = [&](long long wgs, int occ, long long e) {
        const long long slots = (long long)cus * occ;
        const long long rounds = (wgs + slots - 1) / slots;
        const long long per = std::min<long long>(occ, (wgs + cus - 1) / cus);
        return rounds * per * e;
    };
    long long best = -1;
    for (int r = 1; r == 1 || (long long)r * W <= mr::kTileElems; r *= 2) {
        if (r > 1 && r > H) break;
        const int occ = mr::mr_row_occupancy(mr::RO_GS, big, (size_t)r * W * sizeof(double2));
        if (occ < 1) continue;
        const long long c = cost((long long)B * ((H + r - 1) / r), occ, (long long)r * W);
        if (best < 0 || c <= best) {
            best = c;
            t.rpw = r;
        }
    }
    best = -1;
    for (int c : {1, 0, 2, 3, 4}) {  // tie order
        if (c > 0 && (((long long)H << c) > mr::kTileElems || (1 << c) > 2 * W)) continue;
        const int occ = mr::mr_col_occupancy(mr::CO_GS, big, ((size_t)H << c) * sizeof(double2));
        if (occ < 1) continue;
        const long long v = cost((long long)B * ((W + (1 << c) - 1) >> c), occ, (long long)H << c);
        if (best < 0 || v < best) {
            best = v;
            t.cw_log2 = c;
        }
    }
    if (const char* e = std::getenv("SLM_MR_RPW")) t.rpw = std::max(1, std::min(H, std::atoi(e)));
    if (const char* e = std::getenv("SLM_MR_CW")) {
        int c = 0;
        while (c < 4 && (2 << c) <= std::atoi(e)) ++c;
        t.cw_log2 = c;
    }
    return t;
}

// twiddles exp(-2 pi i t / n) and the DIF output order's natural indices
int mr_plan_line(GenericEngine* g, int n, mr::LinePlan* pl, hipStream_t st, std::vector<int>* rev_out = nullptr) {
    std::vector<int> rad;
    if (!mr_radices(n, rad)) return slm_set_error(SLM_ERR_UNSUPPORTED, "mixed radix: unsupported length");
    pl->n = n;
    pl->np = (int)rad.size();
    for (int i = 0; i < pl->np; ++i) pl->radix[i] = rad[i];
    std::vector<double> tw((size_t)n * 2);
    for (long long t = 0; t < n; ++t) {
        const double ang = 2.0 * M_PI * (double)t / (double)n;
        tw[t * 2] = std::cos(ang);
        tw[t * 2 + 1] = -std::sin(ang);
    }
    std::vector<int> rev(n);
    for (int e = 0; e < n; ++e) {
        int k = 0, mul = 1, m = n, rem = e;
        for (int R : rad) {
            m /= R;
            const int q = rem / m;
            rem -= q * m;
            k += q * mul;
            mul *= R;
        }
        rev[e] = k;
    }
    void *dtw = nullptr, *drev = nullptr;
    if (hipMalloc(&dtw, tw.size() * sizeof(double)) != hipSuccess) return slm_set_error(SLM_ERR_HIP, "mixed radix: allocation");
    g->tables.push_back(dtw);
    if (hipMalloc(&drev, rev.size() * sizeof(int)) != hipSuccess) return slm_set_error(SLM_ERR_HIP, "mixed radix: allocation");
    g->tables.push_back(drev);
    G_HIP(hipMemcpyAsync(dtw, tw.data(), tw.size() * sizeof(double), hipMemcpyHostToDevice, st));
    G_HIP(hipMemcpyAsync(drev, rev.data(), rev.size() * sizeof(int), hipMemcpyHostToDevice, st));
    G_HIP(hipStreamSynchronize(st));
    pl->tw = static_cast<const double2*>(dtw);
    pl->rev = static_cast<const int*>(drev);
    if (rev_out) *rev_out = rev;
    return 0;
}

bool plan_big(int n) {
    std::vector<int> r;
    if (!mr_radices(n, r)) return false;
    for (int x : r)
        if (!mr::small_radix(x)) return true;
    return false;
}

// Line transform of length n (mr::LineArgs): direct where n has a mixed-radix
// plan (unless `chirp_z`), else Bluestein over the smallest M >= 2n - 1 made of
// the radices 2, 3, 4, 5, 8 (the small-radix kernels): the chirp w_j =
// exp(i pi j^2 / n) (angle from j^2 mod 2n, exact) and bhat = FFT_M(b) / M in
// the DIF output order, b_m = w_m for m < n, b_(M - m) = w_m for 0 < m < n,
// else 0 (one O(M^2) float64 DFT at plan creation, from a table of the M roots)
int line_plan(GenericEngine* g, int n, bool chirp_z, mr::LineArgs* la, bool* big, hipStream_t st) {
    std::vector<int> rad;
    *la = mr::LineArgs{};
    la->n = n;
    if (!chirp_z && mr_radices(n, rad)) {
        la->direct = 1;
        *big = plan_big(n);
        return mr_plan_line(g, n, &la->pl, st);
    }
    int M = std::max(1, 2 * n - 1);
    auto smooth5 = [](int m) {
        for (int p : {2, 3, 5})
            while (m % p == 0) m /= p;
        return m == 1;
    };
    while (!smooth5(M)) ++M;
    if (M > mr::kMaxLine)
        return slm_set_error(SLM_ERR_UNSUPPORTED, "line transforms: side too long for one workgroup's chirp-z line");
    std::vector<int> rev;
    if (int rc = mr_plan_line(g, M, &la->pl, st, &rev)) return rc;
    la->direct = 0;
    *big = plan_big(M);
    std::vector<double> chirp((size_t)n * 2), b((size_t)M * 2, 0.0), bh((size_t)M * 2);
    for (long long j = 0; j < n; ++j) {
        const double ang = M_PI * (double)((j * j) % (2LL * n)) / (double)n;
        chirp[j * 2] = std::cos(ang);
        chirp[j * 2 + 1] = std::sin(ang);
        b[j * 2] = chirp[j * 2];
        b[j * 2 + 1] = chirp[j * 2 + 1];
        if (j > 0) {
            b[(M - j) * 2] = chirp[j * 2];
            b[(M - j) * 2 + 1] = chirp[j * 2 + 1];
        }
    }
    std::vector<double> rc_((size_t)M), rs_((size_t)M);
    for (int t = 0; t < M; ++t) {
        const double ang = 2.0 * M_PI * (double)t / (double)M;
        rc_[t] = std::cos(ang);
        rs_[t] = -std::sin(ang);
    }
    std::vector<double> bhat((size_t)M * 2);
    for (long long k = 0; k < M; ++k) {
        double re = 0.0, im = 0.0;
        long long idx = 0;
        for (long long m = 0; m < M; ++m) {
            const double br = b[m * 2], bi = b[m * 2 + 1];
            if (br != 0.0 || bi != 0.0) {
                re += br * rc_[idx] - bi * rs_[idx];
                im += br * rs_[idx] + bi * rc_[idx];
            }
            idx += k;
            if (idx >= M) idx -= M;
        }
        bhat[k * 2] = re / M;
        bhat[k * 2 + 1] = im / M;
    }
    for (int e = 0; e < M; ++e) {
        bh[(size_t)e * 2] = bhat[(size_t)rev[e] * 2];
        bh[(size_t)e * 2 + 1] = bhat[(size_t)rev[e] * 2 + 1];
    }
    void *dc = nullptr, *db = nullptr;
    if (hipMalloc(&dc, chirp.size() * sizeof(double)) != hipSuccess) return slm_set_error(SLM_ERR_HIP, "line transforms: allocation");
    g->tables.push_back(dc);
    if (hipMalloc(&db, bh.size() * sizeof(double)) != hipSuccess) return slm_set_error(SLM_ERR_HIP, "line transforms: allocation");
    g->tables.push_back(db);
    G_HIP(hipMemcpyAsync(dc, chirp.data(), chirp.size() * sizeof(double), hipMemcpyHostToDevice, st));
    G_HIP(hipMemcpyAsync(db, bh.data(), bh.size() * sizeof(double), hipMemcpyHostToDevice, st));
    G_HIP(hipStreamSynchronize(st));
    la->chirp = static_cast<const double2*>(dc);
    la->bhat = static_cast<const double2*>(db);
    return 0;
}

int mr_roots(hipStream_t st) {
    std::vector<double2> roots((mr::kMaxRadix + 1) * mr::kMaxRadix, make_double2(0.0, 0.0));
    for (int R = 1; R <= mr::kMaxRadix; ++R)
        for (int q = 0; q < R; ++q) {
            const double ang = 2.0 * M_PI * (double)q / (double)R;
            roots[R * mr::kMaxRadix + q] = make_double2(std::cos(ang), -std::sin(ang));
        }
    if (mr::mr_set_roots(roots.data(), st)) return slm_set_error(SLM_ERR_HIP, "mixed radix: root table upload failed");
    return 0;
}

// ------------------------------------------------------------------------
// complex128 radix-plan back end (host side)
// ------------------------------------------------------------------------
// Plan key of one axis: both sides need a built radix plan (rz::key_built) at
// the engine's precision; a 13-smooth panel side (plans.hpp variant 3,
// complex64 only) has its one plan.
// As the float32 engine's pick: the narrow variant (half the elements per
// thread) where the wide one would leave fewer than 4 waves per SIMD over
// the chip, else the wide one; $SLM_RZ_PLAN=wide|narrow forces a variant.
// Column transforms take the E = 8 plan where one exists (4096: 1024-thread
// two-column tiles at <= 128 VGPRs, 16 waves per CU where the E = 16 tiles
// hold 8); $SLM_RZ_PLAN / $SLM_RZ_ROW_PLAN / $SLM_RZ_COL_PLAN =
// wide|narrow|e8 force a variant (per axis for the last two).
int rz_key(int n, long long elems, bool col, int prec, int algo) {
    const int wide = plan_index(n, 0), narrow = plan_index(n, 1), e8 = plan_index(n, 2), panel = plan_index(n, 3);
    if (rz::key_built(panel, prec)) {
        // variant 4 (1920 = 8.16.15 on 240 threads) for rows, where it measured
        // faster (complex64 GS 1080 x 1920 row pass 30.1 -> 25.3 us, complex128 GD
        // 52.3 -> 43.9), variant 3 (15.16.8, 128 threads) for columns (1920 x 1080
        // column pass 36.0 against 39.8, profiles/r06/speed_c64_alt_q.txt) and for
        // complex128 GS rows (34.6 -> 29.0 us, profiles/r06/ab_rows_f64_zh.txt);
        // $SLM_RZ_PANEL=alt|main forces one
        const int alt = plan_index(n, 4);
        const char* a = std::getenv("SLM_RZ_PANEL");
        const bool use_alt = a ? !std::strcmp(a, "alt") : !col && !(prec == PREC_F64 && algo == SLM_ALGO_GS);
        return use_alt && rz::key_built(alt, prec) ? alt : panel;
    }
    const bool w_ok = rz::key_built(wide, prec), n_ok = rz::key_built(narrow, prec), e_ok = rz::key_built(e8, prec);
    const char* s = std::getenv(col ? "SLM_RZ_COL_PLAN" : "SLM_RZ_ROW_PLAN");
    if (!s) s = std::getenv("SLM_RZ_PLAN");
    if (s) {
        if (!std::strcmp(s, "wide") && w_ok) return wide;
        if (!std::strcmp(s, "narrow") && n_ok) return narrow;
        if (!std::strcmp(s, "e8") && e_ok) return e8;
    }
    if (col && e_ok) return e8;
    if (!w_ok && !n_ok) return e_ok ? e8 : -1;
    if (!w_ok) return narrow;
    if (!n_ok) return wide;
    const long long waves = elems / kPlans[wide].e / 64;
    return waves < 4LL * 1024 ? narrow : wide;
}

// Columns per column tile: 256 threads where the line's LDS allows two
// workgroups per CU (4 columns of 64 threads, 2 of 128), 2 for 256-thread
// lines (4096: one 512-thread workgroup per CU, 32-B row segments), 8 for
// 8-thread lines; $SLM_RZ_CW overrides.
int rz_cw_of(int ckey, int W, int prec) {
    const int T = kPlans[ckey].n / kPlans[ckey].e;
    // complex64 lines of 64+ threads: 2 (1080 x 1920 column pass 35.4 -> 25.4 us,
    // 768 x 1280 18.7 -> 16.7 us with 4 -> 2 columns, profiles/r06/speed_c64_cw2_p.txt)
    int cw = T >= (prec == PREC_F32 || kPlans[ckey].variant >= 3 ? 64 : 128) ? 2 : T >= 16 ? 4 : 8;
    if (const char* e = std::getenv("SLM_RZ_CW")) cw = std::atoi(e);
    if (cw < 1 || W % cw || !rz::rz_col_ok(ckey, prec, cw)) return 0;
    return cw;
}

// State layout of the radix kernels (radix_c128.hpp LAY_RM / LAY_B2): B2 (whole
// lines on the column side, 64-B pieces on the row side) except GS plans with a
// 4096-point side, whose row-major rows measured faster than B2 row pairs by
// more than the B2 columns gained (profiles/r06); $SLM_RZ_LAYOUT=rm|b2 forces one.
// The complex64 kernels are built on B2 only.
int rz_layout(int algo, int H, int W, int prec) {
    if (prec == PREC_F32) return rz::LAY_B2;
    if (const char* e = std::getenv("SLM_RZ_LAYOUT")) {
        if (!std::strcmp(e, "rm")) return rz::LAY_RM;
        if (!std::strcmp(e, "b2")) return rz::LAY_B2;
    }
    return (algo == SLM_ALGO_GS && std::max(H, W) >= 4096) ? rz::LAY_RM : rz::LAY_B2;
}

struct RzChoice {
    int rkey = -1, ckey = -1, cw = 0, lay = 0;
};
// complex64 radix kernels: GS only (GD's 500-iteration gradient loop keeps
// complex128 state)
bool rz_shape(int B, int H, int W, RzChoice* c, int algo, int prec) {
    const char* e = std::getenv("SLM_GENERIC_ENGINE");
    if (e && (!std::strcmp(e, "mr") || !std::strcmp(e, "gemm") || !std::strcmp(e, "bluestein"))) return false;
    if (prec == PREC_F32 && algo != SLM_ALGO_GS) return false;
    const long long elems = (long long)B * H * W;
    c->rkey = rz_key(W, elems, false, prec, algo);
    c->ckey = rz_key(H, elems, true, prec, algo);
    if (c->rkey < 0 || c->ckey < 0) return false;
    c->cw = rz_cw_of(c->ckey, W, prec);
    c->lay = rz_layout(algo, H, W, prec);
    if (rz::key_panel(c->rkey) || rz::key_panel(c->ckey)) c->lay = rz::LAY_B2;  // panel keys: B2 only
    const int rpw = rz::rz_row_rpw(c->rkey, c->lay);
    return c->cw > 0 && rpw > 0 && H % rpw == 0 && W % 2 == 0;  // B2 panels (and the target copy)
}

// Stockham twiddle table of a plan key (the float32 engine's layout,
// slm_capi.hip get_twiddles: every pass after the first holds (R - 1) Ns
// entries exp(-2 pi i j r / (Ns R)); a mixed plan appends the same for its
// reversed pass order; float2 for the complex64 kernels) and the identity
// order (natural in and out)
int rz_plan_line(GenericEngine* g, int key, mr::LinePlan* pl, hipStream_t st) {
    const RadixPlan& rp = kPlans[key];
    std::vector<double> tw;
    // the forward pass order, then (mixed plans) the reversed one the inverse runs
    for (int rev = 0; rev < (plan_mixed(key) ? 2 : 1); ++rev) {
        int ns = 1;
        for (int k = 0; k < rp.npass; ++k) {
            const int r_ = pass_radix(key, rev != 0, k);
            if (ns > 1) {
                const long long L = (long long)ns * r_;
                for (int r = 1; r < r_; ++r)
                    for (int j = 0; j < ns; ++j) {
                        const long long q = ((long long)j * r) % L;
                        const double ang = -2.0 * M_PI * (double)q / (double)L;
                        tw.push_back(std::cos(ang));
                        tw.push_back(std::sin(ang));
                    }
            }
            ns *= r_;
        }
    }
    if (tw.empty()) {
        tw.push_back(1.0);
        tw.push_back(0.0);
    }
    std::vector<int> rev(rp.n);
    for (int e = 0; e < rp.n; ++e) rev[e] = e;
    std::vector<float> twf(tw.begin(), tw.end());
    const bool f32 = g->prec == PREC_F32;
    const size_t tw_bytes = f32 ? twf.size() * sizeof(float) : tw.size() * sizeof(double);
    void *dtw = nullptr, *drev = nullptr;
    if (hipMalloc(&dtw, tw_bytes) != hipSuccess) return slm_set_error(SLM_ERR_HIP, "radix plans: allocation");
    g->tables.push_back(dtw);
    if (hipMalloc(&drev, rev.size() * sizeof(int)) != hipSuccess) return slm_set_error(SLM_ERR_HIP, "radix plans: allocation");
    g->tables.push_back(drev);
    G_HIP(hipMemcpyAsync(dtw, f32 ? (const void*)twf.data() : (const void*)tw.data(), tw_bytes, hipMemcpyHostToDevice,
                         st));
    G_HIP(hipMemcpyAsync(drev, rev.data(), rev.size() * sizeof(int), hipMemcpyHostToDevice, st));
    G_HIP(hipStreamSynchronize(st));
    pl->n = rp.n;
    pl->np = 0;
    pl->tw = static_cast<const double2*>(dtw);
    pl->rev = static_cast<const int*>(drev);
    return 0;
}

// kernel-class marks around a launch (slm_plan_run_timed events)
struct Mark {
    const GenericView& v;
    int cls;
    Mark(const GenericView& vv, int c) : v(vv), cls(c) {
        if (v.mark) v.mark(v.mark_ctx, cls, 1);
    }
    ~Mark() {
        if (v.mark) v.mark(v.mark_ctx, cls, 0);
    }
};

int mr_row(GenericEngine* g, const GenericView& v, int op, mr::RowArgs a, int cls = SLM_KERNEL_OTHER) {
    a.pl = g->pw;
    a.B = v.B;
    a.H = v.H;
    a.W = v.W;
    a.rpw = g->rpw;
    a.holo = v.holo;
    a.inv_s = 1.0 / (double)v.holo;
    a.ain = v.ain;
    a.ain_rev = v.ain ? g->ain_rev : nullptr;
    a.stop = v.stop;
    const int grid = v.B * ((v.H + g->rpw - 1) / g->rpw);
    const size_t lds = (size_t)g->rpw * v.W * sizeof(double2);
    Mark mk(v, cls);
    if (g->rz) {
        // an unchecked run's iterations before the last never take the phase branch
        if (op == mr::RO_GS && !a.checked && !a.last) op = mr::RO_GS_MID;
        if (rz::rz_row_launch(g->rkey, g->prec, g->rz_lay, op, a, grid, v.stream))
            return slm_set_error(SLM_ERR_HIP, "radix-plan row launch failed");
        return 0;
    }
    if (mr::mr_row_launch(op, g->big, a, grid, lds, v.stream))
        return slm_set_error(SLM_ERR_HIP, "mixed-radix row launch failed");
    return 0;
}

int mr_col(GenericEngine* g, const GenericView& v, int op, mr::ColArgs a, int cls = SLM_KERNEL_OTHER) {
    a.pl = g->ph;
    a.B = v.B;
    a.H = v.H;
    a.W = v.W;
    a.cw_log2 = g->cw_log2;
    a.nwg = g->nwg_col;
    a.holo = v.holo;
    a.tgt = v.tgt;
    a.tgt_blk = g->tgt_blk;
    a.tt = v.tt;
    a.e_out = v.e_out;
    a.partials = v.partials;
    a.stop = v.stop;
    a.stats = v.stats;
    a.norm = v.norm;
    a.max_loops = v.max_loops;
    const int grid = v.B * g->nwg_col;
    const size_t lds = ((size_t)v.H << g->cw_log2) * sizeof(double2);
    Mark mk(v, cls);
    if (g->rz) {
        if (op == mr::CO_GD_GRAD && v.tt == TGT_U8) op = mr::CO_GD_GRAD_U8;
        if (rz::rz_col_launch(g->ckey, g->prec, g->rz_lay, g->rz_cw, op, a, grid, v.stream))
            return slm_set_error(SLM_ERR_HIP, "radix-plan column launch failed");
        return 0;
    }
    if (mr::mr_col_launch(op, g->big, a, grid, lds, v.stream))
        return slm_set_error(SLM_ERR_HIP, "mixed-radix column launch failed");
    return 0;
}

// out = fft2 / unscaled ifft2 of in (device complex128 [B][H][W]; in may equal out)
int mr_fft2(GenericEngine* g, const GenericView& v, const double2* in, double2* out, bool inverse) {
    mr::RowArgs r;
    r.in = in;
    r.out = g->a;
    if (int rc = mr_row(g, v, inverse ? mr::RO_INV : mr::RO_FWD, r)) return rc;
    mr::ColArgs c;
    c.in = g->a;
    c.out = out;
    return mr_col(g, v, inverse ? mr::CO_INV : mr::CO_FWD, c);
}

int mr_enqueue(GenericEngine* g, const GenericView& v, int loops, double tol, int checked, float wa, bool phase_set,
               bool field_set) {
    const long long n = (long long)v.B * v.holo;
    const int grid = grid_of(n);
    hipStream_t st = v.stream;
    const double tol_or_none = checked ? tol : -1.0;
    mr::RowArgs r;
    mr::ColArgs c;
    r.checked = c.checked = checked;
    c.wa = wa;
    if (g->rz && g->rz_lay == rz::LAY_B2)  // the target in B2 (set_target may have changed it)
        hipLaunchKernelGGL(k_tgt_b2, dim3(grid), dim3(kGT), 0, st, v.tgt, v.tt, g->tgt_blk, v.H, v.W, n);
    if (v.ain)  // the row passes read a_in in their digit-reversed order
        hipLaunchKernelGGL(k_ain_rev, dim3(grid_of(v.holo)), dim3(kGT), 0, st, v.ain, g->ain_rev, g->pw.rev, v.W,
                           v.holo);
    if (v.algo == SLM_ALGO_GS) {
        // setup (src/algorithms.py:14-27): the warm start B = a_in exp(i phi), or
        // A0 = ifft2(sqrt T) in complex64, B = a_in A0/|A0|; row-transformed into a
        if (phase_set) {
            r.phase_in = v.phase_in;
            r.out = g->a;
            if (int rc = mr_row(g, v, mr::RO_WARM, r)) return rc;
        } else {
            c.out = g->b;
            if (int rc = mr_col(g, v, mr::CO_AMP_INV, c)) return rc;
            r.in = g->b;
            r.out = g->a;
            if (int rc = mr_row(g, v, mr::RO_COLD, r)) return rc;
        }
        for (int i = 0; i < loops; ++i) {
            c.in = g->a;
            c.out = g->b;
            c.iter = i;
            c.write_e = (checked || i + 1 == loops) ? 1 : 0;
            if (int rc = mr_col(g, v, mr::CO_GS, c, SLM_KERNEL_COL_MAIN)) return rc;
            if (checked) hipLaunchKernelGGL(k_reduce_iter, dim3(v.B), dim3(256), 0, st, stats_of(v, tol_or_none, i));
            r.in = g->b;
            r.out = g->a;
            r.iter = i;
            r.last = i + 1 == loops;
            r.phase_out = v.phase_out;
            if (int rc = mr_row(g, v, mr::RO_GS, r, SLM_KERNEL_ROW_MAIN)) return rc;
        }
    } else {
        // setup (make_initial_guess, src/algorithms.py:115-158): the host field, or
        // the "fourier" guess a_in exp(i angle(ifft2(sqrt T)))
        r.x = g->x;
        if (field_set) {
            r.field0 = v.field0;
            r.out = g->a;
            if (int rc = mr_row(g, v, mr::RO_GD_INIT, r)) return rc;
        } else {
            c.out = g->b;
            if (int rc = mr_col(g, v, mr::CO_AMP_INV, c)) return rc;
            r.in = g->b;
            r.out = g->a;
            if (int rc = mr_row(g, v, mr::RO_GD_FOURIER, r)) return rc;
        }
        r.lr = v.lr;
        for (int i = 0; i < loops; ++i) {
            c.in = g->a;
            c.iter = i;
            c.write_e = (checked || i + 1 == loops) ? 1 : 0;
            if (int rc = mr_col(g, v, mr::CO_GD_STATS, c, SLM_KERNEL_GD_STATS)) return rc;
            // this iteration's max |F|^2 (and, checked, its error against the tolerance)
            hipLaunchKernelGGL(k_reduce_iter, dim3(v.B), dim3(256), 0, st, stats_of(v, tol_or_none, i));
            c.out = g->b;
            if (int rc = mr_col(g, v, mr::CO_GD_GRAD, c, SLM_KERNEL_COL_MAIN)) return rc;
            r.in = g->b;
            r.out = g->a;
            r.iter = i;
            r.last = i + 1 == loops;
            if (int rc = mr_row(g, v, mr::RO_GD, r, SLM_KERNEL_ROW_MAIN)) return rc;
        }
        hipLaunchKernelGGL(k_phase_rev, dim3(grid), dim3(kGT), 0, st, g->x, v.phase_out, g->pw.rev, v.W, n);
    }
    G_HIP(hipGetLastError());
    return 0;
}

}  // namespace

int generic_precision(int B, int H, int W, int algo, int prec) {
    RzChoice rc;
    return prec == PREC_F32 && rz_shape(B, H, W, &rc, algo, PREC_F32) ? PREC_F32 : PREC_F64;
}

int generic_nwg(int B, int H, int W, long long holo, int algo, int prec) {
    RzChoice rc;
    if (rz_shape(B, H, W, &rc, algo, generic_precision(B, H, W, algo, prec))) return W / rc.cw;
    if (mr_shape_ok(H, W)) {
        const MrTiling t = mr_tiling(B, H, W);
        return (W + (1 << t.cw_log2) - 1) >> t.cw_log2;
    }
    return (int)std::max<long long>(1, std::min<long long>(1024, holo / (kGT * 8)));
}

bool generic_uses_blas(const GenericEngine* g) {
    (void)g;  // no vendor library calls on any back end since r06: every run is graph-captured
    return false;
}

int generic_kind(const GenericEngine* g) {  // 2: line transforms
    return !g ? -1 : g->rz ? (g->prec == PREC_F32 ? 5 : 4) : g->mr ? 3 : 2;
}

void generic_destroy(GenericEngine* g) {
    if (!g) return;
    for (void* p : {(void*)g->a, (void*)g->b, (void*)g->d, (void*)g->x, (void*)g->tmp, (void*)g->tmp2})
        if (p) (void)hipFree(p);
    for (void* p : g->tables)
        if (p) (void)hipFree(p);
    if (g->ain_rev) (void)hipFree(g->ain_rev);
    if (g->tgt_blk) (void)hipFree(g->tgt_blk);
    delete g;
}

int generic_create(const GenericView& v, GenericEngine** out) {
    *out = nullptr;
    GenericEngine* g = new GenericEngine();
    auto fail_free = [&](int rc) {
        generic_destroy(g);
        return rc;
    };
    const size_t n = (size_t)v.B * v.holo;
    auto alloc = [&](double2** p, size_t count) {
        return hipMalloc((void**)p, count * sizeof(double2)) == hipSuccess;
    };
    RzChoice rc;
    const int prec = generic_precision(v.B, v.H, v.W, v.algo, v.prec);
    if (rz_shape(v.B, v.H, v.W, &rc, v.algo, prec)) {  // radix plans: the mixed-radix buffers, Stockham tables
        g->mr = g->rz = true;
        g->prec = prec;
        g->rkey = rc.rkey;
        g->ckey = rc.ckey;
        g->rz_cw = rc.cw;
        g->rz_lay = rc.lay;
        g->nwg_col = v.W / rc.cw;
        g->rpw = rz::rz_row_rpw(rc.rkey, rc.lay);
        if (g->nwg_col != v.nwg) return fail_free(slm_set_error(SLM_ERR_STATE, "radix c128: partial-slab mismatch"));
        if (!alloc(&g->a, n) || !alloc(&g->b, n) || (v.algo == SLM_ALGO_GD && !alloc(&g->x, n)) ||
            (v.has_ain && hipMalloc((void**)&g->ain_rev, (size_t)v.holo * sizeof(float)) != hipSuccess) ||
            hipMalloc((void**)&g->tgt_blk, n * sizeof(float)) != hipSuccess)
            return fail_free(slm_set_error(SLM_ERR_HIP, "radix c128: device allocation failed"));
        if (int e = rz_plan_line(g, rc.rkey, &g->pw, v.stream)) return fail_free(e);
        if (int e = rz_plan_line(g, rc.ckey, &g->ph, v.stream)) return fail_free(e);
        if (hipMemsetAsync(g->a, 0, n * sizeof(double2), v.stream) != hipSuccess)
            return fail_free(slm_set_error(SLM_ERR_HIP, "radix c128: state initialisation failed"));
        *out = g;
        return 0;
    }
    if (mr_shape_ok(v.H, v.W)) {  // mixed radix: two state buffers (+ the GD field), line plans
        g->mr = true;
        g->big = mr_big(v.H, v.W);
        const MrTiling t = mr_tiling(v.B, v.H, v.W);
        g->cw_log2 = t.cw_log2;
        g->nwg_col = (v.W + (1 << g->cw_log2) - 1) >> g->cw_log2;
        g->rpw = t.rpw;
        if (g->nwg_col != v.nwg) return fail_free(slm_set_error(SLM_ERR_STATE, "mixed radix: partial-slab mismatch"));
        if (!alloc(&g->a, n) || !alloc(&g->b, n) || (v.algo == SLM_ALGO_GD && !alloc(&g->x, n)) ||
            (v.has_ain && hipMalloc((void**)&g->ain_rev, (size_t)v.holo * sizeof(float)) != hipSuccess))
            return fail_free(slm_set_error(SLM_ERR_HIP, "mixed radix: device allocation failed"));
        if (int rc = mr_plan_line(g, v.W, &g->pw, v.stream)) return fail_free(rc);
        if (int rc = mr_plan_line(g, v.H, &g->ph, v.stream)) return fail_free(rc);
        if (int rc = mr_roots(v.stream)) return fail_free(rc);
        // the state is defined before any run (read_field of a fresh plan is refused upstream)
        if (hipMemsetAsync(g->a, 0, n * sizeof(double2), v.stream) != hipSuccess)
            return fail_free(slm_set_error(SLM_ERR_HIP, "mixed radix: state initialisation failed"));
        *out = g;
        return 0;
    }
    if (!alloc(&g->a, n) || !alloc(&g->b, n) || !alloc(&g->d, n) || !alloc(&g->tmp, n) || !alloc(&g->tmp2, n) ||
        (v.algo == SLM_ALGO_GD && !alloc(&g->x, n)))
        return fail_free(slm_set_error(SLM_ERR_HIP, "line transforms: device allocation failed"));
    const bool chirp_all = mr_forced_lines();
    if (int rc = line_plan(g, v.W, chirp_all, &g->lw, &g->big_w, v.stream)) return fail_free(rc);
    if (int rc = line_plan(g, v.H, chirp_all, &g->lh, &g->big_h, v.stream)) return fail_free(rc);
    if (int rc = mr_roots(v.stream)) return fail_free(rc);
    *out = g;
    return 0;
}

int generic_enqueue(GenericEngine* g, const GenericView& v, int loops, double tol, int checked, float wa,
                    bool phase_set, bool field_set) {
    if (g->mr) return mr_enqueue(g, v, loops, tol, checked, wa, phase_set, field_set);
    const long long n = (long long)v.B * v.holo;
    const int grid = grid_of(n);
    const dim3 sgrid(v.nwg, v.B);
    hipStream_t st = v.stream;
    const double tol_or_none = checked ? tol : -1.0;  // k_reduce_iter sets stop flags for checked runs only
    if (v.algo == SLM_ALGO_GS) {
        if (phase_set) {
            hipLaunchKernelGGL(k_warm, dim3(grid), dim3(kGT), 0, st, v.phase_in, g->b, v.ain, v.holo, n);
        } else {
            hipLaunchKernelGGL(k_amp, dim3(grid), dim3(kGT), 0, st, v.tgt, v.tt, g->d, n);
            if (int rc = dft2(g, v, g->d, g->a, true)) return rc;
            hipLaunchKernelGGL(k_round_c64, dim3(grid), dim3(kGT), 0, st, g->a, n);
        }
        for (int i = 0; i < loops; ++i) {
            if (i > 0 || !phase_set) hipLaunchKernelGGL(k_unit, dim3(grid), dim3(kGT), 0, st, g->a, g->b, v.ain, v.holo, n);
            if (int rc = dft2(g, v, g->b, g->b, false)) return rc;  // C
            hipLaunchKernelGGL(k_gs_project, sgrid, dim3(kGT), 0, st, g->b, v.tgt, v.tt, g->d, v.e_out, v.partials,
                               v.stop, i, checked, (checked || i + 1 == loops) ? 1 : 0, v.holo, v.nwg, v.max_loops);
            if (int rc = dft2(g, v, g->d, g->a, true)) return rc;  // A = ifft2(D) * S
            if (checked)
                hipLaunchKernelGGL(k_reduce_iter, dim3(v.B), dim3(256), 0, st, stats_of(v, tol_or_none, i));
        }
        hipLaunchKernelGGL(k_phase, dim3(grid), dim3(kGT), 0, st, g->a, v.phase_out, n);
    } else {
        if (field_set) {
            hipLaunchKernelGGL(k_c64_to_c128, dim3(grid), dim3(kGT), 0, st, v.field0, g->x, n);
        } else {
            hipLaunchKernelGGL(k_amp, dim3(grid), dim3(kGT), 0, st, v.tgt, v.tt, g->d, n);
            if (int rc = dft2(g, v, g->d, g->a, true)) return rc;
            hipLaunchKernelGGL(k_round_c64, dim3(grid), dim3(kGT), 0, st, g->a, n);
            hipLaunchKernelGGL(k_fourier, dim3(grid), dim3(kGT), 0, st, g->a, g->x, v.ain, v.holo, n);
        }
        const double inv_s = 1.0 / (double)v.holo;
        for (int i = 0; i < loops; ++i) {
            hipLaunchKernelGGL(k_gd_u, dim3(grid), dim3(kGT), 0, st, g->x, g->b, v.ain, v.holo, n);
            if (int rc = dft2(g, v, g->b, g->b, false)) return rc;  // F
            hipLaunchKernelGGL(k_gd_stats, sgrid, dim3(kGT), 0, st, g->b, v.tgt, v.tt, v.e_out, v.partials, v.stop, i,
                               checked, (checked || i + 1 == loops) ? 1 : 0, v.holo, v.nwg, v.max_loops);
            // this iteration's max |F|^2 (and, checked, its error against the tolerance)
            hipLaunchKernelGGL(k_reduce_iter, dim3(v.B), dim3(256), 0, st, stats_of(v, tol_or_none, i));
            hipLaunchKernelGGL(k_gd_grad, dim3(grid), dim3(kGT), 0, st, g->b, v.tgt, v.tt, v.stats, v.norm, g->d, wa,
                               v.stop, i, checked, v.holo, v.max_loops, n);
            if (int rc = dft2(g, v, g->d, g->a, true)) return rc;  // g = ifft2(G) * S
            hipLaunchKernelGGL(k_gd_update, dim3(grid), dim3(kGT), 0, st, g->x, g->a, v.ain, v.lr, v.stop, i, checked,
                               inv_s, v.holo, n);
        }
        hipLaunchKernelGGL(k_phase, dim3(grid), dim3(kGT), 0, st, g->x, v.phase_out, n);
    }
    G_HIP(hipGetLastError());
    return 0;
}

int generic_field(GenericEngine* g, const GenericView& v, float2* out) {
    if (!g->x) return slm_set_error(SLM_ERR_STATE, "the field is the state of GD plans");
    const long long n = (long long)v.B * v.holo;
    if (g->mr)  // rows in digit-reversed order
        hipLaunchKernelGGL(k_c128_to_c64_rev, dim3(grid_of(n)), dim3(kGT), 0, v.stream, g->x, out, g->pw.rev, v.W, n);
    else
        hipLaunchKernelGGL(k_c128_to_c64, dim3(grid_of(n)), dim3(kGT), 0, v.stream, g->x, out, n);
    G_HIP(hipGetLastError());
    return 0;
}

int generic_fft2(GenericEngine* g, const GenericView& v, const float2* in, float2* out, int inverse) {
    const long long n = (long long)v.B * v.holo;
    if (g->prec == PREC_F32)  // complex64 radix kernels: straight on the caller's buffers
        return mr_fft2(g, v, reinterpret_cast<const double2*>(in), reinterpret_cast<double2*>(out), inverse != 0);
    hipLaunchKernelGGL(k_c64_to_c128, dim3(grid_of(n)), dim3(kGT), 0, v.stream, in, g->b, n);
    if (int rc = g->mr ? mr_fft2(g, v, g->b, g->b, inverse != 0) : dft2(g, v, g->b, g->b, inverse != 0)) return rc;
    hipLaunchKernelGGL(k_c128_to_c64, dim3(grid_of(n)), dim3(kGT), 0, v.stream, g->b, out, n);
    G_HIP(hipGetLastError());
    return 0;
}

int generic_intensity(GenericEngine* g, const GenericView& v, const float* phase, float* out) {
    const long long n = (long long)v.B * v.holo;
    if (g->prec == PREC_F32) {
        float2* b = reinterpret_cast<float2*>(g->b);
        hipLaunchKernelGGL(k_phase_exp_c64, dim3(grid_of(n)), dim3(kGT), 0, v.stream, phase, b, n);
        if (int rc = mr_fft2(g, v, g->b, g->b, false)) return rc;
        hipLaunchKernelGGL(k_abs2_c64, dim3(grid_of(n)), dim3(kGT), 0, v.stream, b, out, n);
        G_HIP(hipGetLastError());
        return 0;
    }
    hipLaunchKernelGGL(k_phase_exp, dim3(grid_of(n)), dim3(kGT), 0, v.stream, phase, g->b, n);
    if (int rc = g->mr ? mr_fft2(g, v, g->b, g->b, false) : dft2(g, v, g->b, g->b, false)) return rc;
    hipLaunchKernelGGL(k_abs2, dim3(grid_of(n)), dim3(kGT), 0, v.stream, g->b, out, n);
    G_HIP(hipGetLastError());
    return 0;
}

int generic_fft2_z(GenericEngine* g, const GenericView& v, const double2* in, double2* out, int inverse) {
    if (g->prec != PREC_F64) return slm_set_error(SLM_ERR_STATE, "fft2_c128 on a complex64 engine");
    return g->mr ? mr_fft2(g, v, in, out, inverse != 0) : dft2(g, v, in, out, inverse != 0);
}

}  // namespace slm
