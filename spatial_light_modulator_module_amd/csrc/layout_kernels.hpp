// Small kernels of the plan runtime (slm_capi.hip is their one translation
// unit): the statistics folds, the GD phase extraction and the layout
// transposes between the user's row-major arrays and the blocked iteration
// layout (kernels.hpp, blk_index).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kernels.hpp"

namespace slm {

__global__ void __launch_bounds__(256) stats_reduce_kernel(StatsParams p) {
    const int i = blockIdx.x, b = blockIdx.y;
    const int last = min(p.stop_iter[b], p.max_loops - 1);
    if (i > last) return;
    __shared__ double o[4];
    reduce_slab(p, b, i, o);
    if (threadIdx.x == 0)
        for (int k = 0; k < 4; ++k) p.stats[((long long)b * p.max_loops + i) * 4 + k] = o[k];
}

// Tolerance check of one iteration (while error > tolerance, src/algorithms.py:29,83).
__global__ void __launch_bounds__(256) stats_finalize_kernel(StatsParams p) {
    const int b = blockIdx.x;
    if (p.iter > p.stop_iter[b]) return;
    __shared__ double o[4];
    reduce_slab(p, b, p.iter, o);
    if (threadIdx.x == 0) {
        if (!(o[3] > p.tol)) p.stop_iter[b] = p.iter;
    }
}

// hologram = np.angle(input) of the GD field (src/algorithms.py:111); the
// field is in the blocked layout, the phase row-major.
template <int PLOG>
__global__ void __launch_bounds__(256) field_phase_kernel(const float2* field, float* phase, long long n, int H,
                                                          int W) {
    const long long holo = (long long)H * W;
    for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
        const long long b = i / holo, r = i - b * holo;
        const int y = (int)(r / W), x = (int)(r - (long long)y * W);
        const float2 f = field[b * holo + blk_index<PLOG>(y, x, H)];
        phase[i] = atan2f(f.y, f.x);
    }
}

// Row-major <-> blocked ([x / P][y][x % P]) transposes of float / complex64
// planes through one 64 x 64 LDS tile per workgroup (grid (W / 64, H / 64,
// B), 256 threads; H and W are multiples of 64 for every radix-plan side):
// 16-B pieces of 256-B (float) / 512-B (complex64) row segments on the
// row-major side, panel runs (64 rows x P elements, contiguous in HBM) on the
// blocked side, 16-B accesses both ways -- where the element-wise relayout
// wrote (read) the blocked side in P-element pieces scattered 4 H elements
// apart (the 8 x 4096^2 float32 target upload took 550 us at 2 TB/s, VALU
// 6 % active, r04). AMP: the upload of a float32 GS target stores its
// amplitude sqrt(T) (TgtLoad<TGT_F32>::amp; TGT_AMP device targets).
//
// LDS: tile rows of 64 WV words, unpadded, with the 16-B chunks of row y
// XOR-swizzled by g(y) = (y * PW / 4) mod 16 (PW / 4 = chunks per panel row;
// (y / (4 / PW)) mod 16 for panel rows under 16 B), so that both the
// row-major side (ds_read_b128 / ds_write_b128 along rows) and the blocked side
// (16-lane groups walking down one panel column) hit distinct banks: the
// bank model of tools/lds_bank_sim.py (MI355X_MICROARCH.md LDS table) gives 0
// extra cycles per LDS instruction for every float / complex64 panel width but
// float P = 16 from the blocked layout (2.0; float P = 2 with the lane order
// of `piece` below, 1.3 / 2.7 without),
// where r04's padded rows (LD = 64 WV + 4) cost 2.0 on the 4096^2 unblock
// (measured SQ_LDS_BANK_CONFLICT / LDS instruction, profiles/r05/sq_4096x8_s7.txt).
template <typename V, int PLOG, bool TO_BLOCKED, bool AMP = false>
__global__ void __launch_bounds__(256) tile_relayout_kernel(const V* in, V* out, int H, int W) {
    static_assert(!AMP || sizeof(V) == 4, "the amplitude applies to float planes");
    constexpr int WV = sizeof(V) / 4;   // 32-bit words per element
    constexpr int P = 1 << PLOG;
    constexpr int RW = 64 * WV;         // words per tile row
    constexpr int PW = P * WV;          // words of one panel row
    constexpr int BV = PW < 4 ? PW : 4; // words per LDS access on the blocked side
    constexpr int ROWS = 4 / BV;        // rows of one panel per 16-B blocked-side access
    __shared__ __attribute__((aligned(16))) float tile[64 * RW];
    auto lds = [](int yy, int w) -> int {
        const int g = PW >= 4 ? (yy * (PW / 4)) & 15 : (yy / (4 / (PW < 4 ? PW : 4))) & 15;
        return yy * RW + ((((w >> 2) ^ g)) << 2) + (w & 3);
    };
    const long long holo = (long long)H * W;
    const int x0 = blockIdx.x * 64, y0 = blockIdx.y * 64;
    const float* src = reinterpret_cast<const float*>(in + blockIdx.z * holo);
    float* dst = reinterpret_cast<float*>(out + blockIdx.z * holo);
    // row-major side: tile row yy, words w .. w + 3
    auto rm_at = [&](int i, int& yy, int& w) {
        yy = i / (RW / 4);
        w = (i - yy * (RW / 4)) * 4;
    };
    // blocked side: 16-B piece i of the tile's panel runs (panel q, first row yy,
    // word w of the panel row; ROWS consecutive rows when a panel row is < 16 B)
    auto bl_at = [&](int i, int& q, int& yy, int& w) {
        const int e = i * 4;                  // word offset in the tile's blocked order
        q = e / (64 * PW);
        const int r = e - q * 64 * PW;
        yy = r / PW;
        w = r - yy * PW;
    };
    // blocked-side piece of loop index i: for 8-B panel rows (PW == 2) the
    // lanes of a wave alternate between the two panels of its 1 KB (lane l
    // takes piece 32 (l & 1) + l / 2), so a 16-lane LDS group writes / reads
    // both 8-B halves of 8 chunks -- 16 distinct bank pairs -- instead of one
    // half of 16 rows' chunks (2 / 4 of 8 bank pairs busy twice). The wave's
    // global access still covers the same contiguous 1 KB.
    auto piece = [](int i) { return PW == 2 ? (i & ~63) | ((i & 1) << 5) | ((i & 63) >> 1) : i; };
    auto gbl = [&](int q, int yy, int w) -> long long {
        return (((long long)(x0 >> PLOG) + q) * H + y0 + yy) * PW + w;
    };
    constexpr int N4 = 64 * RW / 4;  // 16-B pieces per tile
    if constexpr (TO_BLOCKED) {
        for (int i = threadIdx.x; i < N4; i += 256) {
            int yy, w;
            rm_at(i, yy, w);
            float4 v = *reinterpret_cast<const float4*>(src + (long long)(y0 + yy) * W * WV + (long long)x0 * WV + w);
            if constexpr (AMP) {
                v.x = TgtLoad<TGT_F32>::amp(v.x);
                v.y = TgtLoad<TGT_F32>::amp(v.y);
                v.z = TgtLoad<TGT_F32>::amp(v.z);
                v.w = TgtLoad<TGT_F32>::amp(v.w);
            }
            *reinterpret_cast<float4*>(tile + lds(yy, w)) = v;
        }
        __syncthreads();
        for (int i = threadIdx.x; i < N4; i += 256) {
            int q, yy, w;
            bl_at(piece(i), q, yy, w);
            float4 v;
            float* pv = reinterpret_cast<float*>(&v);
#pragma unroll
            for (int r = 0; r < ROWS; ++r) {
                const float* t = tile + lds(yy + r, q * PW + w);
                if constexpr (BV == 4) {
                    v = *reinterpret_cast<const float4*>(t);
                } else if constexpr (BV == 2) {
                    const float2 u = *reinterpret_cast<const float2*>(t);
                    pv[2 * r] = u.x;
                    pv[2 * r + 1] = u.y;
                } else {
                    pv[r] = t[0];
                }
            }
            *reinterpret_cast<float4*>(dst + gbl(q, yy, w)) = v;
        }
    } else {
        for (int i = threadIdx.x; i < N4; i += 256) {
            int q, yy, w;
            bl_at(piece(i), q, yy, w);
            const float4 v = *reinterpret_cast<const float4*>(src + gbl(q, yy, w));
            const float* pv = reinterpret_cast<const float*>(&v);
#pragma unroll
            for (int r = 0; r < ROWS; ++r) {
                float* t = tile + lds(yy + r, q * PW + w);
                if constexpr (BV == 4) {
                    *reinterpret_cast<float4*>(t) = v;
                } else if constexpr (BV == 2) {
                    *reinterpret_cast<float2*>(t) = make_float2(pv[2 * r], pv[2 * r + 1]);
                } else {
                    t[0] = pv[r];
                }
            }
        }
        __syncthreads();
        for (int i = threadIdx.x; i < N4; i += 256) {
            int yy, w;
            rm_at(i, yy, w);
            *reinterpret_cast<float4*>(dst + (long long)(y0 + yy) * W * WV + (long long)x0 * WV + w) =
                *reinterpret_cast<const float4*>(tile + lds(yy, w));
        }
    }
}

// row-major <-> blocked layout of byte planes (uint8 targets), element-wise
template <typename V, bool TO_BLOCKED, int PLOG>
__global__ void __launch_bounds__(256) relayout_kernel(const V* in, V* out, long long n, int H, int W) {
    const long long holo = (long long)H * W;
    for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
        const long long b = i / holo, r = i - b * holo;
        const int y = (int)(r / W), x = (int)(r - (long long)y * W);
        const long long j = b * holo + blk_index<PLOG>(y, x, H);
        if (TO_BLOCKED)
            out[j] = in[i];
        else
            out[i] = in[j];
    }
}

}  // namespace slm
