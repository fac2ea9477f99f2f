// Mixed-radix float64 transforms for image sides without a float32 radix plan
// (plans.hpp covers 2^k and 768): any side whose prime factors are <= 13 and
// that fits one workgroup's LDS, e.g. the 1080 x 1920 and 1280 x 1024 SLM
// panels. The reference transforms every length in O(N log N) through
// pocketfft (src/algorithms.py:27,31,34; scipy.fft); these kernels do the same
// on the device, in complex128 like the reference's loop, so the any-shape
// engine (generic.hip) no longer multiplies by dense DFT matrices there.
//
// One line = one 1-D transform held in LDS (complex128), transformed in place
// one radix pass at a time, one butterfly in registers at a time (no staging
// of a thread's whole share: registers stay far below the 128 that two
// 512-thread workgroups per CU allow). Stages R_0, R_1, ... of span L (L = n
// first, then L / R_0, ...), m = L / R, block start b0 (a multiple of L), j < m:
//   DIF (natural in, digit-reversed out):
//     y = DFT_R(x[b0 + j + r m], r < R);  x[b0 + j + q m] = y_q w_L^(q j)
//   DIT (digit-reversed in, natural out): the adjoint, stages in reverse order
//     u_q = x[b0 + j + q m] w_L^(q j);  x[b0 + j + r m] = DFT_R(u)_r
// (w conjugated, DFT_R conjugated for the inverse). After a DIF the element at
// position e is frequency rev[e] = q_0 + R_0 q_1 + R_0 R_1 q_2 + ..., where
// e = q_0 (n / R_0) + q_1 (n / (R_0 R_1)) + ... (checked against numpy.fft).
// The GS / GD projections between a launch's two transforms are element-wise,
// so they run on the digit-reversed order (reading the target / a_in and
// writing phases / the expected output at the natural index rev[e]), and the
// pair DIF -> projection -> DIT never permutes. A lone transform (setup,
// fft2 helpers) loads its input gathered in digit-reversed order and runs the
// DIT.
//
// A workgroup holds several lines: consecutive rows of a row tile (element
// stride 1), or the columns of a column tile interleaved ([h][c], element
// stride CW, butterflies enumerated column-fastest so neighbouring lanes touch
// neighbouring LDS words).
//
// The GS / GD iteration is two launches (plus the GD statistics split), as in
// the float32 engine (kernels.hpp): the column launch runs forward transform
// -> projection and statistics -> inverse transform, the row launch inverse ->
// projection -> forward, so each launch reads and writes the field once.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kernels.hpp"

namespace slm {
namespace mr {

constexpr int kThreads = 256;  // threads per workgroup of every mixed-radix kernel
constexpr int kMaxPass = 16;
constexpr int kMaxRadix = 13;
// LDS of one tile: at most this many complex128 elements (72 KiB: two
// workgroups per CU); a single line may take up to kMaxLine (one per CU)
constexpr int kTileElems = 4608;
// the odd radices 7, 11, 13 (generic odd DFTs) cost registers in every pass
// of a kernel that can run them: plans made of 2, 3, 4, 5 and 8 only take
// kernels built for those (60-85 VGPRs, five 4-wave workgroups per CU), plans
// with any other radix the full set (<= 128 VGPRs, four)
__host__ __device__ constexpr bool small_radix(int r) { return r == 2 || r == 3 || r == 4 || r == 5 || r == 8; }
constexpr int kMaxLine = 8192;

// one line length's plan: radices in DIF stage order, the twiddle table
// tw[t] = exp(-2 pi i t / n), t < n (host-computed in double), and the
// digit reversal rev[e] of the DIF output order
struct LinePlan {
    int n = 1;
    int np = 0;
    int radix[kMaxPass] = {};
    const double2* tw = nullptr;
    const int* rev = nullptr;
};

// roots of the small DFTs: kRoots[R][q] = exp(-2 pi i q / R) (copied per device
// and per translation unit by mr_set_roots; wave-uniform indices -> scalar loads)
namespace {
__constant__ double2 kRoots[kMaxRadix + 1][kMaxRadix];
}

__device__ __forceinline__ double2 cadd(double2 a, double2 b) { return make_double2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ double2 csub(double2 a, double2 b) { return make_double2(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ double2 cmul(double2 a, double2 b) {
    return make_double2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}
__device__ __forceinline__ double2 cmulc(double2 a, double2 b) {  // a * conj(b)
    return make_double2(a.x * b.x + a.y * b.y, a.y * b.x - a.x * b.y);
}
// i sigma z, sigma = -1 forward, +1 inverse
template <bool INV>
__device__ __forceinline__ double2 isg(double2 z) {
    return INV ? make_double2(-z.y, z.x) : make_double2(z.y, -z.x);
}

template <int R, bool INV>
struct Dft;
template <bool INV>
struct Dft<2, INV> {
    __device__ __forceinline__ static void run(double2 (&u)[2]) {
        const double2 a = u[0];
        u[0] = cadd(a, u[1]);
        u[1] = csub(a, u[1]);
    }
};
template <bool INV>
struct Dft<4, INV> {
    __device__ __forceinline__ static void run(double2 (&u)[4]) {
        const double2 a = cadd(u[0], u[2]), b = csub(u[0], u[2]);
        const double2 c = cadd(u[1], u[3]), d = isg<INV>(csub(u[1], u[3]));
        u[0] = cadd(a, c);
        u[2] = csub(a, c);
        u[1] = cadd(b, d);
        u[3] = csub(b, d);
    }
};
template <bool INV>
struct Dft<8, INV> {
    __device__ __forceinline__ static void run(double2 (&u)[8]) {
        double2 e[4] = {u[0], u[2], u[4], u[6]}, o[4] = {u[1], u[3], u[5], u[7]};
        Dft<4, INV>::run(e);
        Dft<4, INV>::run(o);
        constexpr double h = 0.70710678118654752440;  // sqrt(1/2)
        constexpr double s = INV ? 1.0 : -1.0;
        // o_q *= w8^q, w8 = exp(sigma 2 pi i / 8)
        o[1] = make_double2(h * (o[1].x - s * o[1].y), h * (o[1].y + s * o[1].x));
        o[2] = isg<INV>(o[2]);
        o[3] = make_double2(h * (-o[3].x - s * o[3].y), h * (-o[3].y + s * o[3].x));
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            u[q] = cadd(e[q], o[q]);
            u[q + 4] = csub(e[q], o[q]);
        }
    }
};
// odd R: y_q = u_0 + sum_s a_s cos(2 pi s q / R) + i sigma sum_s b_s sin(2 pi s q / R),
// a_s = u_s + u_(R-s), b_s = u_s - u_(R-s); y_(R-q) the conjugate combination
template <int R, bool INV>
struct Dft {
    static_assert(R % 2 == 1 && R <= kMaxRadix, "odd radices up to kMaxRadix");
    __device__ __forceinline__ static void run(double2 (&u)[R]) {
        constexpr int H = R / 2;
        double2 a[H], b[H];
        double2 y0 = u[0];
#pragma unroll
        for (int s = 1; s <= H; ++s) {
            a[s - 1] = cadd(u[s], u[R - s]);
            b[s - 1] = csub(u[s], u[R - s]);
            y0 = cadd(y0, a[s - 1]);
        }
#pragma unroll
        for (int q = 1; q <= H; ++q) {
            double2 A = u[0], Bv = make_double2(0.0, 0.0);
#pragma unroll
            for (int s = 1; s <= H; ++s) {
                const double2 w = kRoots[R][(s * q) % R];  // (cos, -sin)
                A.x = fma(a[s - 1].x, w.x, A.x);
                A.y = fma(a[s - 1].y, w.x, A.y);
                Bv.x = fma(b[s - 1].x, -w.y, Bv.x);
                Bv.y = fma(b[s - 1].y, -w.y, Bv.y);
            }
            const double2 j = isg<INV>(Bv);
            u[q] = cadd(A, j);
            u[R - q] = csub(A, j);
        }
        u[0] = y0;
    }
};

// Geometry of the lines in one workgroup's LDS: line l, element e at
// lds[l * ls + e * es]. LINEFAST: butterflies enumerated line-fastest (column
// tiles) instead of element-fastest (row tiles).
struct Lines {
    int count, ls, es;
};

// x / d for 0 <= x, x * d < 2^32 by one multiply-high (d > 1: mul = floor((2^32
// - 1) / d) + 1, exact in that range; checked for every d <= 8192, x < 2^15):
// the butterfly indexing divides by the pass's runtime span and line length
// once per butterfly, which the compiler otherwise expands to a ~15-instruction
// float-reciprocal sequence each
struct FastDiv {
    uint32_t d, mul;
};
__device__ __forceinline__ FastDiv fast_div(int d) {
    return {(uint32_t)d, d > 1 ? 0xFFFFFFFFu / (uint32_t)d + 1u : 0u};
}
__device__ __forceinline__ int divq(int x, const FastDiv& f) {
    return f.d == 1 ? x : (int)__umulhi((uint32_t)x, f.mul);
}

template <bool LINEFAST>
__device__ __forceinline__ int bf_base(const Lines& g, int gi, const FastDiv& fpl, const FastDiv& fm,
                                       const FastDiv& fc, int L, int& j) {
    int line, bf;
    if (LINEFAST) {
        bf = divq(gi, fc);
        line = gi - bf * g.count;
    } else {
        line = divq(gi, fpl);
        bf = gi - line * (int)fpl.d;
    }
    const int blk = divq(bf, fm);
    j = bf - blk * (int)fm.d;
    return line * g.ls + (blk * L + j) * g.es;
}

// twiddles w^q, q < R, of one butterfly from w = w_L^j: one table load, the
// powers by complex products (float64: q ulp-scale errors, ~1e-15, where the
// R - 1 table loads per butterfly were the passes' main vector-memory traffic)
template <int R, bool INV>
__device__ __forceinline__ void twiddle(double2 (&u)[R], double2 w1) {
    double2 w = w1;
#pragma unroll
    for (int q = 1; q < R; ++q) {
        if (q > 1) w = cmul(w, w1);
        u[q] = INV ? cmulc(u[q], w) : cmul(u[q], w);
    }
}

// one in-place pass of radix R and span L over every line of the tile
template <int R, bool INV, bool LINEFAST, bool DIT>
__device__ __forceinline__ void pass(double2* lds, const Lines& g, int n, int L, const double2* __restrict__ tw) {
    const int m = L / R;
    const int per_line = n / R;
    const int nb = g.count * per_line;
    const int tstride = n / L;
    const int step = m * g.es;
    const FastDiv fpl = fast_div(per_line), fm = fast_div(m), fc = fast_div(g.count);
    for (int gi = threadIdx.x; gi < nb; gi += kThreads) {
        int j;
        const int base = bf_base<LINEFAST>(g, gi, fpl, fm, fc, L, j);
        const double2 w1 = tw[j * tstride];
        double2 u[R];
#pragma unroll
        for (int r = 0; r < R; ++r) u[r] = lds[base + r * step];
        if (DIT) twiddle<R, INV>(u, w1);
        Dft<R, INV>::run(u);
        if (!DIT) twiddle<R, INV>(u, w1);
#pragma unroll
        for (int r = 0; r < R; ++r) lds[base + r * step] = u[r];
    }
    __syncthreads();
}

template <bool INV, bool LINEFAST, bool DIT, bool BIG>
__device__ __forceinline__ void pass_r(int R, double2* lds, const Lines& g, int n, int L, const double2* tw) {
    switch (R) {
        case 2: pass<2, INV, LINEFAST, DIT>(lds, g, n, L, tw); break;
        case 3: pass<3, INV, LINEFAST, DIT>(lds, g, n, L, tw); break;
        case 4: pass<4, INV, LINEFAST, DIT>(lds, g, n, L, tw); break;
        case 5: pass<5, INV, LINEFAST, DIT>(lds, g, n, L, tw); break;
        case 8: pass<8, INV, LINEFAST, DIT>(lds, g, n, L, tw); break;
        default:
            if constexpr (BIG) {
                switch (R) {
                    case 7: pass<7, INV, LINEFAST, DIT>(lds, g, n, L, tw); break;
                    case 11: pass<11, INV, LINEFAST, DIT>(lds, g, n, L, tw); break;
                    default: pass<13, INV, LINEFAST, DIT>(lds, g, n, L, tw); break;
                }
            }
            break;
    }
}

// natural order in -> digit-reversed (rev) order out, every line of the tile
template <bool INV, bool LINEFAST, bool BIG>
__device__ __forceinline__ void fft_dif(double2* lds, const Lines& g, const LinePlan& pl) {
    int L = pl.n;
    for (int s = 0; s < pl.np; ++s) {
        const int R = pl.radix[s];
        pass_r<INV, LINEFAST, false, BIG>(R, lds, g, pl.n, L, pl.tw);
        L /= R;
    }
}
// digit-reversed order in -> natural order out
template <bool INV, bool LINEFAST, bool BIG>
__device__ __forceinline__ void fft_dit(double2* lds, const Lines& g, const LinePlan& pl) {
    int L = 1;
    for (int s = pl.np - 1; s >= 0; --s) {
        const int R = pl.radix[s];
        L *= R;
        pass_r<INV, LINEFAST, true, BIG>(R, lds, g, pl.n, L, pl.tw);
    }
}

// element-wise pieces shared by the mixed-radix kernels (mr_inst.hip) and the
// complex128 radix-plan kernels (radix_c128.hpp): numpy's dtype rules of the
// reference's loop
__device__ __forceinline__ double amp_of(const void* tgt, int tt, long long i) {
    if (tt == TGT_U8) return (double)TgtLoad<TGT_U8>::amp(TgtLoad<TGT_U8>::load(tgt, i));
    return (double)(float)sqrt((double)static_cast<const float*>(tgt)[i]);  // numpy: sqrt(float32) is float32
}
__device__ __forceinline__ double t_of(const void* tgt, int tt, long long i) {
    return tt == TGT_U8 ? (double)static_cast<const uint8_t*>(tgt)[i] : (double)static_cast<const float*>(tgt)[i];
}
// a exp(i angle(z)) == a z / |z|, angle(0) = 0 -> a (src/algorithms.py:30,33)
__device__ __forceinline__ double2 unit_of(double2 z, double a) {
    const double n2 = z.x * z.x + z.y * z.y;
    if (n2 == 0.0) return make_double2(a, 0.0);
    const double r = a / sqrt(n2);
    return make_double2(z.x * r, z.y * r);
}
// x / |x| a (src/algorithms.py:84; |x| = 0 gives NaN as there)
__device__ __forceinline__ double2 u_of(double2 x, double a) {
    const double r = a / sqrt(x.x * x.x + x.y * x.y);
    return make_double2(x.x * r, x.y * r);
}
__device__ __forceinline__ double2 round_c64(double2 z) { return make_double2((double)(float)z.x, (double)(float)z.y); }

// ------------------------------------------------------------------------
// kernels
// ------------------------------------------------------------------------
enum RowOp : int {
    RO_FWD = 0,        // in -> fwd -> out
    RO_INV = 1,        // in -> inv -> out
    RO_COLD = 2,       // GS cold start: in (column-inverse of a_T) -> inv -> A0 rounded to complex64
                       //   (src/algorithms.py:27) -> B = a_in A0/|A0| -> fwd -> out
    RO_WARM = 3,       // GS warm start: B = a_in exp(i phi) (complex64 exp, as numpy) -> fwd -> out
    RO_GS = 4,         // GS: in -> inv -> A; last (or stopped): phase = angle(A) (:48), else
                       //   B = a_in A/|A| (:30) -> fwd -> out
    RO_GD_FOURIER = 5, // GD "fourier" guess: in -> inv -> complex64 -> x = a_in exp(i angle) (:153-156)
                       //   -> u = a_in x/|x| (:84) -> fwd -> out
    RO_GD_INIT = 6,    // GD host field: x = field0 (complex64) -> u -> fwd -> out
    RO_GD = 7,         // GD: in (column-inverse of G) -> inv -> g a_in / S; dEdX_complex, x -= lr dEdX
                       //   (:87-91, :179-185) -> u -> fwd -> out
    RO_GS_MID = 8,     // RO_GS of an unchecked run's iterations before the last (no phase branch;
                       //   complex128 radix-plan kernels only: the float64 atan2 path costs registers)
    RO_NUM = 9
};
enum ColOp : int {
    CO_FWD = 0,       // in -> fwd -> out
    CO_INV = 1,       // in -> inv -> out
    CO_AMP_INV = 2,   // a_T = sqrt(T) as numpy forms it -> inv -> out
    CO_GS = 3,        // in -> fwd -> C; E = |C|^2 statistics, expected output, D = a_T C/|C| (:33,36-38)
                      //   -> inv -> out
    CO_GD_STATS = 4,  // in -> fwd -> F; statistics of P = |F|^2 (:85-86), output
    CO_GD_GRAD = 5,   // in -> fwd -> G = mask F (s P - T) (:80,85-88) -> inv -> out
    CO_GD_GRAD_U8 = 6,  // CO_GD_GRAD of a uint8 target (complex128 radix-plan kernels only: the
                        //   float64 mask of numpy's dtype rule compiled apart from the float32 one)
    CO_NUM = 7
};

struct RowArgs {
    const double2* in = nullptr;
    double2* out = nullptr;
    const float* ain = nullptr;        // [H][W] or nullptr (uniform)
    const float* ain_rev = nullptr;    // the same with rows in digit-reversed order (DIF side)
    const float* phase_in = nullptr;   // RO_WARM
    float* phase_out = nullptr;        // RO_GS
    double2* x = nullptr;              // GD state, rows in digit-reversed order (element e = column rev[e])
    const float2* field0 = nullptr;    // RO_GD_INIT
    const float* lr = nullptr;         // RO_GD, per iteration
    const int* stop = nullptr;         // [B]
    int iter = 0, checked = 0, last = 0;
    int B = 0, H = 0, W = 0, rpw = 1;  // rows per workgroup
    long long holo = 0;
    double inv_s = 0.0;
    LinePlan pl;                       // length W
};
struct ColArgs {
    const double2* in = nullptr;
    double2* out = nullptr;
    const void* tgt = nullptr;
    const float* tgt_blk = nullptr;    // complex128 radix plans: the target as float in their B2 layout
    int tt = 0;                        // TGT_U8 / TGT_F32 (row-major, as uploaded)
    float* e_out = nullptr;
    double* partials = nullptr;        // [B][max_loops][nwg][4]
    const int* stop = nullptr;
    const double* stats = nullptr;     // CO_GD_GRAD: this iteration's max |F|^2
    const double* norm = nullptr;
    int iter = 0, checked = 0, write_e = 0, max_loops = 1;
    int nwg = 1, cw_log2 = 0, B = 0, H = 0, W = 0;
    float wa = 0.f;
    long long holo = 0;
    LinePlan pl;                       // length H
};

// One 1-D transform per workgroup over rows of `n` complex128 (any n; the
// any-size engine's transforms for sides with a prime factor above 13, and
// their partner side): out[line] = DFT_n(in[line]), forward or the unscaled
// inverse (computed as conj(DFT(conj x))). direct: n has a mixed-radix plan
// `pl` -- DIF, then the digit reversal on the store. Otherwise Bluestein's
// chirp-z: with w_j = exp(i pi j^2 / n), DFT_n(x)_k = conj(w_k) (a * b)_k for
// a_j = x_j conj(w_j), b_j = w_j (j in (-n, n)), the circular convolution over
// a mixed-radix length M = pl.n >= 2n - 1 as DIF -> times bhat (FFT_M(b) / M
// in DIF output order) -> inverse DIT.
struct LineArgs {
    const double2* in = nullptr;
    double2* out = nullptr;
    int n = 0, direct = 1, inverse = 0;
    LinePlan pl;                     // length n (direct) or M (Bluestein)
    const double2* chirp = nullptr;  // w_j, j < n (Bluestein)
    const double2* bhat = nullptr;   // FFT_M(b) / M, DIF order (Bluestein)
};
int mr_line_launch(bool big, const LineArgs& a, int lines, size_t lds, hipStream_t st);

// host launchers (mr_inst.hip; big: a plan radix that is not small_radix; lds =
// tile elements x 16 B; 0 or -1 on a launch error)
int mr_row_launch(int op, bool big, const RowArgs& a, int grid, size_t lds, hipStream_t st);
int mr_col_launch(int op, bool big, const ColArgs& a, int grid, size_t lds, hipStream_t st);
// workgroups of one kernel a CU holds at once (occupancy query; 0 on error)
int mr_row_occupancy(int op, bool big, size_t lds);
int mr_col_occupancy(int op, bool big, size_t lds);
// small-DFT roots (host table [kMaxRadix + 1][kMaxRadix]) into the current device's copy
int mr_set_roots(const double2* roots, hipStream_t st);

}  // namespace mr
}  // namespace slm
