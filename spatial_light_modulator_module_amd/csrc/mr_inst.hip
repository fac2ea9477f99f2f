// Mixed-radix float64 iteration kernels (mixed_radix.hpp).
//
// Row tile: `rpw` consecutive rows of one hologram (one contiguous run of
// rpw * W complex128 in HBM). Column tile: 2^cw_log2 adjacent columns of one
// hologram, all H rows, held [h][c] in LDS (each row's 2^cw_log2 * 16 B piece
// is one contiguous segment in HBM). Element-wise work mirrors the DFT-GEMM
// engine's kernels in generic.hip (same formulas, same numpy dtype rules), so
// the two engines differ only in how the transforms round.
//
// Order inside a launch: the first transform is a DIF (natural in, digit-
// reversed out), the projection works on the digit-reversed order with
// natural indices rev[e], the second transform is a DIT (natural out). Lone
// transforms gather their input in digit-reversed order and run a DIT.
#include <hip/hip_runtime.h>

#include <mutex>
#include <set>
#include <utility>

#include "mixed_radix.hpp"

namespace slm {
namespace mr {
namespace {

// waves per SIMD the register budget must allow: 5 (<= 102 VGPRs: five
// 4-wave workgroups per CU) for kernels with radices up to 8, 4 (<= 128) with
// the odd radices 7, 11, 13
template <bool BIG>
constexpr int kWavesPerSimd = BIG ? 4 : 5;

template <int OP, bool BIG>
__global__ void __launch_bounds__(kThreads, kWavesPerSimd<BIG>) mr_row_kernel(RowArgs a) {
    extern __shared__ double2 lds[];
    const int tiles = (a.H + a.rpw - 1) / a.rpw;
    const int id = xcd_remap(blockIdx.x, gridDim.x);  // neighbouring tiles on one XCD
    const int b = id / tiles;
    const int row0 = (id - b * tiles) * a.rpw;
    const int rows = min(a.rpw, a.H - row0);
    const int W = a.W;
    const int ne = rows * W;
    const long long pix0 = (long long)row0 * W;  // within the hologram
    const long long off = (long long)b * a.holo + pix0;
    const int* __restrict__ rev = a.pl.rev;
    if constexpr (OP == RO_GS || OP == RO_GD) {
        if (a.checked && a.iter > a.stop[b]) return;  // stopped earlier: frozen (src/algorithms.py:29,83)
    }
    // position e of the tile (row e / W, slot e % W) <-> natural pixel of that row
    auto nat = [&](int e) -> int {
        const int r = e / W;
        return r * W + rev[e - r * W];
    };
    auto ain = [&](int px) -> double { return a.ain ? (double)a.ain[pix0 + px] : 1.0; };
    // a_in at tile position e on the digit-reversed side (rows in that order)
    auto ain_e = [&](int e) -> double { return a.ain_rev ? (double)a.ain_rev[pix0 + e] : 1.0; };
    constexpr bool GATHER = OP == RO_FWD || OP == RO_INV || OP == RO_WARM || OP == RO_GD_INIT;
    for (int e = threadIdx.x; e < ne; e += kThreads) {
        double2 v;
        if constexpr (GATHER) {
            const int px = nat(e);
            if constexpr (OP == RO_WARM) {
                // numpy: exp(1j * float32 phase) is complex64, then times the float64 a_in
                double s, c;
                sincos((double)a.phase_in[off + px], &s, &c);
                const double am = ain(px);
                v = make_double2((double)(float)c * am, (double)(float)s * am);
            } else if constexpr (OP == RO_GD_INIT) {
                // x keeps each row in digit-reversed order: the GD row pass reads it in place
                const float2 f = a.field0[off + px];
                const double2 x = make_double2((double)f.x, (double)f.y);
                a.x[off + e] = x;
                v = u_of(x, ain(px));
            } else {
                v = a.in[off + px];
            }
        } else {
            v = a.in[off + e];
        }
        lds[e] = v;
    }
    __syncthreads();
    const Lines g{rows, W, 1};
    if constexpr (GATHER) {
        fft_dit<OP == RO_INV, false, BIG>(lds, g, a.pl);
    } else {
        fft_dif<true, false, BIG>(lds, g, a.pl);  // inverse: A (GS), the gradient (GD), A0 (setup)
        // projection on the digit-reversed order, between the inverse and the forward transform
        const bool phase_only = OP == RO_GS && (a.last || (a.checked && a.stop[b] == a.iter));
        const double l = OP == RO_GD ? (double)a.lr[a.iter] : 0.0;
        for (int e = threadIdx.x; e < ne; e += kThreads) {
            const double2 z = lds[e];
            if constexpr (OP == RO_COLD) {
                lds[e] = unit_of(round_c64(z), ain_e(e));  // A0 = ifft2(sqrt T) is complex64 (:27)
            } else if constexpr (OP == RO_GS) {
                if (phase_only)
                    a.phase_out[off + nat(e)] = (float)atan2(z.y, z.x);  // hologram = np.angle(A) (:48)
                else
                    lds[e] = unit_of(z, ain_e(e));
            } else if constexpr (OP == RO_GD_FOURIER) {
                // angle of the complex64 ifft2 is float32, exp of it complex64 (:153-156)
                const double2 c = round_c64(z);
                const float ang = atan2f((float)c.y, (float)c.x);
                double s, co;
                sincos((double)ang, &s, &co);
                const double am = ain_e(e);
                const double2 x = make_double2((double)(float)co * am, (double)(float)s * am);
                a.x[off + e] = x;
                lds[e] = u_of(x, am);
            } else if constexpr (OP == RO_GD) {
                // dEdF = ifft2(G) a_in (unscaled transform * 1/S), dEdX_complex, x -= lr dEdX
                const double am = ain_e(e);
                const double s = am * a.inv_s;
                const double gx = z.x * s, gy = z.y * s;
                double2 x = a.x[off + e];
                const double ax2 = x.x * x.x + x.y * x.y;
                const double ax = sqrt(ax2);
                const double re = x.x * gx + x.y * gy;
                x.x -= l * ((gx - x.x * (re / ax2)) / ax);
                x.y -= l * ((gy - x.y * (re / ax2)) / ax);
                a.x[off + e] = x;
                lds[e] = u_of(x, am);
            }
        }
        // (uniform per workgroup) the run's last GD update needs no next forward transform
        if (phase_only || (OP == RO_GD && a.last)) return;
        __syncthreads();
        fft_dit<false, false, BIG>(lds, g, a.pl);
    }
    for (int e = threadIdx.x; e < ne; e += kThreads) a.out[off + e] = lds[e];
}

template <int OP, bool BIG>
__global__ void __launch_bounds__(kThreads, kWavesPerSimd<BIG>) mr_col_kernel(ColArgs a) {
    extern __shared__ double2 lds[];
    const int id = xcd_remap(blockIdx.x, gridDim.x);  // neighbouring tiles (partial lines) on one XCD
    const int b = id / a.nwg;
    const int tile = id - b * a.nwg;
    const int cw = 1 << a.cw_log2;
    const int c0 = tile * cw;
    const int ne = a.H * cw;
    const long long hoff = (long long)b * a.holo;
    const int* __restrict__ rev = a.pl.rev;
    if constexpr (OP == CO_GS || OP == CO_GD_STATS || OP == CO_GD_GRAD) {
        if (a.checked && a.iter > a.stop[b]) return;  // stopped earlier: frozen
    }
    // element e of the tile: LDS row h = e >> cw_log2, column c0 + (e & (cw - 1));
    // global index at image row `row`
    auto at = [&](int e, int row, long long& i) -> bool {
        const int x = c0 + (e & (cw - 1));
        i = hoff + (long long)row * a.W + x;
        return x < a.W;
    };
    constexpr bool GATHER = OP == CO_FWD || OP == CO_INV || OP == CO_AMP_INV;
    for (int e = threadIdx.x; e < ne; e += kThreads) {
        const int h = e >> a.cw_log2;
        long long i;
        double2 v = make_double2(0.0, 0.0);
        if (at(e, GATHER ? rev[h] : h, i)) {
            if constexpr (OP == CO_AMP_INV)
                v = make_double2(amp_of(a.tgt, a.tt, i), 0.0);
            else
                v = a.in[i];
        }
        lds[e] = v;
    }
    __syncthreads();
    const Lines g{cw, 1, cw};
    if constexpr (GATHER) {
        fft_dit<OP != CO_FWD, true, BIG>(lds, g, a.pl);
    } else {
        fft_dif<false, true, BIG>(lds, g, a.pl);  // C (GS), F (GD)
        double mx = 0.0, s2 = 0.0, st = 0.0, s = 0.0;
        if constexpr (OP == CO_GD_GRAD) s = a.norm[b] / a.stats[((long long)b * a.max_loops + a.iter) * 4];
        for (int e = threadIdx.x; e < ne; e += kThreads) {
            long long i;
            if (!at(e, rev[e >> a.cw_log2], i)) continue;  // frequency row of this position
            const double2 z = lds[e];
            const double en = z.x * z.x + z.y * z.y;
            const double t = t_of(a.tgt, a.tt, i);
            if constexpr (OP == CO_GS || OP == CO_GD_STATS) {
                mx = fmax(mx, en);
                s2 += en * en;
                st += en * t;
                if (a.write_e) a.e_out[i] = (float)en;
            }
            if constexpr (OP == CO_GS) {
                lds[e] = unit_of(z, amp_of(a.tgt, a.tt, i));  // D = a_T C/|C| (:33)
            } else if constexpr (OP == CO_GD_GRAD) {
                // numpy's mask dtype: float32 for a float32 target, float64 for uint8 (:80)
                const double mask = a.tt == TGT_U8 ? 1.0 + (double)a.wa * t / 255.0
                                                   : (double)(1.0f + __fdiv_rn(__fmul_rn(a.wa, (float)t), 255.0f));
                const double w = mask * (en * s - t);
                lds[e] = make_double2(z.x * w, z.y * w);
            }
        }
        if constexpr (OP == CO_GS || OP == CO_GD_STATS) {
            block_reduce_stats<kThreads>(mx, s2, st);
            if (threadIdx.x == 0) {
                double* dst = a.partials + (((long long)b * a.max_loops + a.iter) * a.nwg + tile) * 4;
                dst[0] = mx;
                dst[1] = s2;
                dst[2] = st;
                dst[3] = 0.0;
            }
        }
        if constexpr (OP == CO_GD_STATS) return;
        __syncthreads();
        fft_dit<true, true, BIG>(lds, g, a.pl);
    }
    for (int e = threadIdx.x; e < ne; e += kThreads) {
        long long i;
        if (at(e, e >> a.cw_log2, i)) a.out[i] = lds[e];
    }
}

// one line per workgroup (LineArgs, mixed_radix.hpp): a direct mixed-radix
// transform, or Bluestein's chirp-z over a mixed-radix length M >= 2n - 1
template <bool BIG>
__global__ void __launch_bounds__(kThreads, kWavesPerSimd<BIG>) mr_line_kernel(LineArgs a) {
    extern __shared__ double2 lds[];
    const long long off = (long long)blockIdx.x * a.n;
    const int M = a.pl.n;
    const Lines g{1, M, 1};
    auto cj = [&](double2 z) { return a.inverse ? make_double2(z.x, -z.y) : z; };  // inverse = conj DFT conj
    if (a.direct) {
        for (int e = threadIdx.x; e < a.n; e += kThreads) lds[e] = cj(a.in[off + e]);
        __syncthreads();
        fft_dif<false, false, BIG>(lds, g, a.pl);
        for (int e = threadIdx.x; e < a.n; e += kThreads) a.out[off + a.pl.rev[e]] = cj(lds[e]);
        return;
    }
    for (int e = threadIdx.x; e < M; e += kThreads)
        lds[e] = e < a.n ? cmulc(cj(a.in[off + e]), a.chirp[e]) : make_double2(0.0, 0.0);  // x_j conj(w_j)
    __syncthreads();
    fft_dif<false, false, BIG>(lds, g, a.pl);
    for (int e = threadIdx.x; e < M; e += kThreads) lds[e] = cmul(lds[e], a.bhat[e]);
    __syncthreads();
    fft_dit<true, false, BIG>(lds, g, a.pl);  // the circular convolution (1/M folded into bhat), natural order
    for (int k = threadIdx.x; k < a.n; k += kThreads) a.out[off + k] = cj(cmulc(lds[k], a.chirp[k]));
}

// dynamic LDS above 64 KiB must be allowed per kernel and per device (the
// attribute is a device's property: slm_gs_multi runs plans on several devices
// from several host threads), once each
template <class F>
bool raise_lds(F fn) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return false;
    static std::mutex mu;
    static std::set<std::pair<const void*, int>> done;
    std::lock_guard<std::mutex> lk(mu);
    const auto key = std::make_pair((const void*)fn, dev);
    if (done.count(key)) return true;
    if (hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize, kMaxLine * 16) != hipSuccess)
        return false;
    done.insert(key);
    return true;
}

template <int OP, bool BIG>
int row_one(const RowArgs& a, int grid, size_t lds, hipStream_t st) {
    if (!raise_lds(mr_row_kernel<OP, BIG>)) return -1;
    hipLaunchKernelGGL((mr_row_kernel<OP, BIG>), dim3(grid), dim3(kThreads), lds, st, a);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
template <int OP, bool BIG>
int col_one(const ColArgs& a, int grid, size_t lds, hipStream_t st) {
    if (!raise_lds(mr_col_kernel<OP, BIG>)) return -1;
    hipLaunchKernelGGL((mr_col_kernel<OP, BIG>), dim3(grid), dim3(kThreads), lds, st, a);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
template <class F>
int occupancy_of(F fn, size_t lds) {
    if (!raise_lds(fn)) return 0;
    int n = 0;
    return hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, (const void*)fn, kThreads, lds) == hipSuccess ? n : 0;
}

template <bool BIG>
int row_launch(int op, const RowArgs& a, int grid, size_t lds, hipStream_t st) {
    switch (op) {
        case RO_FWD: return row_one<RO_FWD, BIG>(a, grid, lds, st);
        case RO_INV: return row_one<RO_INV, BIG>(a, grid, lds, st);
        case RO_COLD: return row_one<RO_COLD, BIG>(a, grid, lds, st);
        case RO_WARM: return row_one<RO_WARM, BIG>(a, grid, lds, st);
        case RO_GS: return row_one<RO_GS, BIG>(a, grid, lds, st);
        case RO_GD_FOURIER: return row_one<RO_GD_FOURIER, BIG>(a, grid, lds, st);
        case RO_GD_INIT: return row_one<RO_GD_INIT, BIG>(a, grid, lds, st);
        case RO_GD: return row_one<RO_GD, BIG>(a, grid, lds, st);
        default: return -1;
    }
}
template <bool BIG>
int col_launch(int op, const ColArgs& a, int grid, size_t lds, hipStream_t st) {
    switch (op) {
        case CO_FWD: return col_one<CO_FWD, BIG>(a, grid, lds, st);
        case CO_INV: return col_one<CO_INV, BIG>(a, grid, lds, st);
        case CO_AMP_INV: return col_one<CO_AMP_INV, BIG>(a, grid, lds, st);
        case CO_GS: return col_one<CO_GS, BIG>(a, grid, lds, st);
        case CO_GD_STATS: return col_one<CO_GD_STATS, BIG>(a, grid, lds, st);
        case CO_GD_GRAD: return col_one<CO_GD_GRAD, BIG>(a, grid, lds, st);
        default: return -1;
    }
}

}  // namespace

int mr_row_launch(int op, bool big, const RowArgs& a, int grid, size_t lds, hipStream_t st) {
    return big ? row_launch<true>(op, a, grid, lds, st) : row_launch<false>(op, a, grid, lds, st);
}
int mr_col_launch(int op, bool big, const ColArgs& a, int grid, size_t lds, hipStream_t st) {
    return big ? col_launch<true>(op, a, grid, lds, st) : col_launch<false>(op, a, grid, lds, st);
}
// the iteration kernels' occupancy (the setup kernels share their shape)
int mr_row_occupancy(int op, bool big, size_t lds) {
    (void)op;
    return big ? occupancy_of(mr_row_kernel<RO_GS, true>, lds) : occupancy_of(mr_row_kernel<RO_GS, false>, lds);
}
int mr_col_occupancy(int op, bool big, size_t lds) {
    (void)op;
    return big ? occupancy_of(mr_col_kernel<CO_GS, true>, lds) : occupancy_of(mr_col_kernel<CO_GS, false>, lds);
}
int mr_line_launch(bool big, const LineArgs& a, int lines, size_t lds, hipStream_t st) {
    auto go = [&](auto fn) {
        if (!raise_lds(fn)) return -1;
        hipLaunchKernelGGL(fn, dim3(lines), dim3(kThreads), lds, st, a);
        return hipGetLastError() == hipSuccess ? 0 : -1;
    };
    return big ? go(mr_line_kernel<true>) : go(mr_line_kernel<false>);
}

int mr_set_roots(const double2* roots, hipStream_t st) {
    if (hipMemcpyToSymbolAsync(HIP_SYMBOL(kRoots), roots, sizeof(kRoots), 0, hipMemcpyHostToDevice, st) != hipSuccess)
        return -1;
    return hipStreamSynchronize(st) == hipSuccess ? 0 : -1;
}

}  // namespace mr
}  // namespace slm
