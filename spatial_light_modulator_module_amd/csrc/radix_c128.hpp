// Complex128 radix-plan kernels: the any-size engine's back end for image
// sides that have a compile-time radix plan (plans.hpp: 2^k and 768).
//
// The reference's loop runs in complex128 after its first ifft2
// (src/algorithms.py:27-38, 83-93). The float32 engine (kernels.hpp) keeps
// complex64 between its passes, which sets a phase-drift floor that the
// 4096^2 configuration (200 iterations) and GD's 500 iterations cross
// (DESIGN.md section 5). The mixed-radix kernels (mixed_radix.hpp) keep
// complex128 but run one butterfly at a time with runtime radices and table
// twiddles from L2 (latency-bound, 0.23 of 8 TB/s). These kernels put the
// float32 engine's structure under complex128 state: the Stockham driver of
// fft_core.hpp with C = V = X = double2 (float64 butterflies and twiddles,
// complex128 registers between passes, complex128 LDS exchanges), a whole
// line per thread group with E elements per thread held in registers, and
// the element-wise projection between a launch's two transforms running on
// the last butterfly group still in registers (fft_pair).
//
// Layout and contract are the mixed-radix back end's (mr::RowArgs /
// mr::ColArgs, generic.hip): row-major complex128 [B][H][W] state, row-major
// target / a_in / phase / expected output, the same element-wise formulas
// and numpy dtype rules (mixed_radix.hpp helpers). The Stockham transforms
// are natural order in and out, so the engine gives these lines the identity
// as their "digit reversal" (the GD field, a_in and the read-back kernels
// then need no permutation).
//
// Tiles. Row tile: RPW whole rows (T = N / E threads per row, RPW T = 256
// threads, or one row of 256 threads); each thread loads element t + T m of
// its row (lane-contiguous 16-B accesses). Column tile: CW adjacent columns,
// all H rows, exchanged through CW interleaved LDS lines; lanes alternate
// columns, so a wave instruction reads CW x 16 B of each of 64 / CW rows.
#pragma once
#include <hip/hip_runtime.h>

#include "mixed_radix.hpp"

namespace slm {
namespace rz {

// plan keys built (plans.hpp): every plan with E <= 16 (E = 24 / 32 double2
// would not fit the register file next to the exchange)
__host__ __device__ constexpr bool key_built(int k) { return k >= 0 && k < kNumPlans && kPlans[k].e <= 16; }

template <int K>
struct RowGeo {
    static constexpr int T = PlanOf<K>::T;
    static constexpr int RPW = T >= 256 ? 1 : 256 / T;
    static constexpr int THREADS = RPW * T;
    static constexpr bool WAVE = T <= 64;  // each row inside one wave: exchanges need no barrier
    static constexpr int LINE = PlanOf<K>::ROWSTRIDE;
};

template <int K, int CW>
struct ColGeo {
    static constexpr int T = PlanOf<K>::T;
    static constexpr int THREADS = CW * T;
    static constexpr bool WAVE = THREADS <= 64;
    static constexpr int SLOTS = lds_line(PlanOf<K>::N) * CW;
    static constexpr bool kValid = THREADS >= 64 && THREADS <= 1024 && SLOTS * 16 <= 160 * 1024;
};

template <int K, int OP>
__global__ void __launch_bounds__((RowGeo<K>::THREADS), 1) rz_row_kernel(mr::RowArgs a) {
    using C = double2;
    using namespace mr;
    constexpr int N = PlanOf<K>::N, E = PlanOf<K>::E, T = PlanOf<K>::T;
    constexpr int RPW = RowGeo<K>::RPW, LINE = RowGeo<K>::LINE;
    constexpr bool WV = RowGeo<K>::WAVE;
    __shared__ double2 smem[RPW * LINE];
    const int t = threadIdx.x % T, lrow = threadIdx.x / T;
    const int tiles = a.H / RPW;
    const int id = xcd_remap(blockIdx.x, gridDim.x);  // neighbouring row groups on one XCD
    const int b = id / tiles;
    const long long pix0 = (long long)((id - b * tiles) * RPW + lrow) * N;  // row start within the hologram
    const long long off = (long long)b * a.holo + pix0;
    if constexpr (OP == RO_GS || OP == RO_GD) {
        if (a.checked && a.iter > a.stop[b]) return;  // stopped earlier: frozen (src/algorithms.py:29,83)
    }
    const LdsLine<double2, 0, WV> lds{smem + lrow * LINE, LINE};
    Twiddles<K, C, TW_DIRECT> tw;
    load_twiddles<K, C>(tw, t, a.pl.tw);
    auto ain = [&](int m) -> double { return a.ain ? (double)a.ain[pix0 + t + T * m] : 1.0; };
    C v[1][E];
#pragma unroll
    for (int m = 0; m < E; ++m) {
        const long long i = off + t + T * m;
        if constexpr (OP == RO_WARM) {
            // numpy: exp(1j * float32 phase) is complex64, then times the float64 a_in
            double s, c;
            sincos((double)a.phase_in[i], &s, &c);
            const double am = ain(m);
            v[0][m] = make_double2((double)(float)c * am, (double)(float)s * am);
        } else if constexpr (OP == RO_GD_INIT) {
            const float2 f = a.field0[i];
            const double2 x = make_double2((double)f.x, (double)f.y);
            a.x[i] = x;
            v[0][m] = u_of(x, ain(m));
        } else {
            v[0][m] = a.in[i];
        }
    }
    if constexpr (OP == RO_FWD || OP == RO_WARM || OP == RO_GD_INIT) {
        fft_line<K, false, C>(v, t, tw, lds);
    } else if constexpr (OP == RO_INV) {
        fft_line<K, true, C>(v, t, tw, lds);
    } else if constexpr (OP == RO_COLD) {
        // A0 = ifft2(sqrt T) is complex64 (src/algorithms.py:27); B = a_in A0/|A0| (:30)
        fft_pair<K, true, false, C>(v, t, tw, lds, [&](int, int m, C& z) { z = unit_of(round_c64(z), ain(m)); });
    } else if constexpr (OP == RO_GS) {
        if (a.last || (a.checked && a.stop[b] == a.iter)) {  // uniform per workgroup
            fft_line_epi<K, true, C>(v, t, tw, lds, [&](int, int m, C& z) {
                a.phase_out[off + t + T * m] = (float)atan2(z.y, z.x);  // hologram = np.angle(A) (:48)
            });
            return;
        }
        fft_pair<K, true, false, C>(v, t, tw, lds, [&](int, int m, C& z) { z = unit_of(z, ain(m)); });
    } else if constexpr (OP == RO_GD_FOURIER) {
        // angle of the complex64 ifft2 is float32, exp of it complex64 (:153-156)
        fft_pair<K, true, false, C>(v, t, tw, lds, [&](int, int m, C& z) {
            const double2 c = round_c64(z);
            const float ang = atan2f((float)c.y, (float)c.x);
            double s, co;
            sincos((double)ang, &s, &co);
            const double am = ain(m);
            const double2 x = make_double2((double)(float)co * am, (double)(float)s * am);
            a.x[off + t + T * m] = x;
            z = u_of(x, am);
        });
    } else if constexpr (OP == RO_GD) {
        // dEdF = ifft2(G) a_in (unscaled transform * 1/S), dEdX_complex, x -= lr dEdX
        // (:87-91, :179-185); next forward input u = a_in x/|x| (:84)
        const double l = (double)a.lr[a.iter];
        auto update = [&](int m, const C& z) -> double2 {
            const double am = ain(m);
            const double s = am * a.inv_s;
            const double gx = z.x * s, gy = z.y * s;
            const long long i = off + t + T * m;
            double2 x = a.x[i];
            const double ax2 = x.x * x.x + x.y * x.y;
            const double ax = sqrt(ax2);
            const double re = x.x * gx + x.y * gy;
            x.x -= l * ((gx - x.x * (re / ax2)) / ax);
            x.y -= l * ((gy - x.y * (re / ax2)) / ax);
            a.x[i] = x;
            return x;
        };
        if (a.last) {  // the run's last update needs no next forward transform
            fft_line_epi<K, true, C>(v, t, tw, lds, [&](int, int m, C& z) { (void)update(m, z); });
            return;
        }
        fft_pair<K, true, false, C>(v, t, tw, lds, [&](int, int m, C& z) { z = u_of(update(m, z), ain(m)); });
    }
#pragma unroll
    for (int m = 0; m < E; ++m) a.out[off + t + T * m] = v[0][m];
}

template <int K, int CW, int OP>
__global__ void __launch_bounds__((ColGeo<K, CW>::THREADS), 1) rz_col_kernel(mr::ColArgs a) {
    using C = double2;
    using namespace mr;
    constexpr int E = PlanOf<K>::E, T = PlanOf<K>::T;
    constexpr int THREADS = ColGeo<K, CW>::THREADS;
    constexpr bool WV = ColGeo<K, CW>::WAVE;
    __shared__ double2 smem[ColGeo<K, CW>::SLOTS];
    const int c = threadIdx.x % CW, t = threadIdx.x / CW;
    const int id = xcd_remap(blockIdx.x, gridDim.x);  // neighbouring tiles (partial lines) on one XCD
    const int b = id / a.nwg;
    const int tile = id - b * a.nwg;
    const long long base = (long long)b * a.holo + (long long)t * a.W + tile * CW + c;  // row t, this column
    const long long rstep = (long long)T * a.W;                                        // slot m: + m rstep
    if constexpr (OP == CO_GS || OP == CO_GD_STATS || OP == CO_GD_GRAD) {
        if (a.checked && a.iter > a.stop[b]) return;  // stopped earlier: frozen
    }
    const LdsTile<CW, double2, 0, WV> lds{smem, c};
    Twiddles<K, C, TW_DIRECT> tw;
    load_twiddles<K, C>(tw, t, a.pl.tw);
    C v[1][E];
#pragma unroll
    for (int m = 0; m < E; ++m) {
        if constexpr (OP == CO_AMP_INV)
            v[0][m] = make_double2(amp_of(a.tgt, a.tt, base + m * rstep), 0.0);
        else
            v[0][m] = a.in[base + m * rstep];
    }
    if constexpr (OP == CO_FWD) {
        fft_line<K, false, C>(v, t, tw, lds);
    } else if constexpr (OP == CO_INV || OP == CO_AMP_INV) {
        fft_line<K, true, C>(v, t, tw, lds);
    } else {
        double mx = 0.0, s2 = 0.0, st = 0.0;
        auto stats = [&](int m, const C& z) -> double {
            const long long i = base + m * rstep;
            const double en = z.x * z.x + z.y * z.y;
            mx = fmax(mx, en);
            s2 += en * en;
            st += en * t_of(a.tgt, a.tt, i);
            if (a.write_e) a.e_out[i] = (float)en;
            return en;
        };
        if constexpr (OP == CO_GS) {
            // E = |C|^2 statistics and expected output, D = a_T C/|C| (:33,36-38)
            fft_pair<K, false, true, C>(v, t, tw, lds, [&](int, int m, C& z) {
                (void)stats(m, z);
                z = unit_of(z, amp_of(a.tgt, a.tt, base + m * rstep));
            });
        } else if constexpr (OP == CO_GD_STATS) {
            fft_line_epi<K, false, C>(v, t, tw, lds, [&](int, int m, C& z) { (void)stats(m, z); });
        } else if constexpr (OP == CO_GD_GRAD) {
            // G = mask F (s P - T), s = norm / max P (:80,85-88); numpy's mask dtype:
            // float32 for a float32 target, float64 for uint8
            const double s = a.norm[b] / a.stats[((long long)b * a.max_loops + a.iter) * 4];
            fft_pair<K, false, true, C>(v, t, tw, lds, [&](int, int m, C& z) {
                const double tv = t_of(a.tgt, a.tt, base + m * rstep);
                const double mask = a.tt == TGT_U8 ? 1.0 + (double)a.wa * tv / 255.0
                                                   : (double)(1.0f + __fdiv_rn(__fmul_rn(a.wa, (float)tv), 255.0f));
                const double w = mask * ((z.x * z.x + z.y * z.y) * s - tv);
                z = make_double2(z.x * w, z.y * w);
            });
        }
        if constexpr (OP == CO_GS || OP == CO_GD_STATS) {
            block_reduce_stats<THREADS>(mx, s2, st);
            if (threadIdx.x == 0) {
                double* dst = a.partials + (((long long)b * a.max_loops + a.iter) * a.nwg + tile) * 4;
                dst[0] = mx;
                dst[1] = s2;
                dst[2] = st;
                dst[3] = 0.0;
            }
        }
        if constexpr (OP == CO_GD_STATS) return;
    }
#pragma unroll
    for (int m = 0; m < E; ++m) a.out[base + m * rstep] = v[0][m];
}

// ------------------------------------------------------------------------
// host side (rz_inst.hip, one object per plan key)
// ------------------------------------------------------------------------
#define SLM_RZ_DECLARE(N)                                                                      \
    int rz_row_launch_##N(int op, const mr::RowArgs& a, int grid, hipStream_t st);             \
    int rz_col_launch_##N(int cw, int op, const mr::ColArgs& a, int grid, hipStream_t st);     \
    int rz_row_rpw_##N();                                                                      \
    int rz_col_ok_##N(int cw);
SLM_RZ_DECLARE(0)
SLM_RZ_DECLARE(1)
SLM_RZ_DECLARE(2)
SLM_RZ_DECLARE(3)
SLM_RZ_DECLARE(5)
SLM_RZ_DECLARE(6)
SLM_RZ_DECLARE(8)
SLM_RZ_DECLARE(9)
SLM_RZ_DECLARE(10)
SLM_RZ_DECLARE(11)
SLM_RZ_DECLARE(12)
SLM_RZ_DECLARE(13)
#undef SLM_RZ_DECLARE
#define SLM_RZ_FOR_EACH_KEY(X) X(0) X(1) X(2) X(3) X(5) X(6) X(8) X(9) X(10) X(11) X(12) X(13)

// launch op on plan key k (0 on success, -1 on a launch error or an unbuilt key)
inline int rz_row_launch(int k, int op, const mr::RowArgs& a, int grid, hipStream_t st) {
#define SLM_CASE(N) \
    case N: return rz_row_launch_##N(op, a, grid, st);
    switch (k) { SLM_RZ_FOR_EACH_KEY(SLM_CASE) default: return -1; }
#undef SLM_CASE
}
inline int rz_col_launch(int k, int cw, int op, const mr::ColArgs& a, int grid, hipStream_t st) {
#define SLM_CASE(N) \
    case N: return rz_col_launch_##N(cw, op, a, grid, st);
    switch (k) { SLM_RZ_FOR_EACH_KEY(SLM_CASE) default: return -1; }
#undef SLM_CASE
}
// rows per row tile of key k (0: not built)
inline int rz_row_rpw(int k) {
#define SLM_CASE(N) \
    case N: return rz_row_rpw_##N();
    switch (k) { SLM_RZ_FOR_EACH_KEY(SLM_CASE) default: return 0; }
#undef SLM_CASE
}
// 1 if key k has column kernels of cw columns
inline int rz_col_ok(int k, int cw) {
#define SLM_CASE(N) \
    case N: return rz_col_ok_##N(cw);
    switch (k) { SLM_RZ_FOR_EACH_KEY(SLM_CASE) default: return 0; }
#undef SLM_CASE
}

}  // namespace rz
}  // namespace slm
