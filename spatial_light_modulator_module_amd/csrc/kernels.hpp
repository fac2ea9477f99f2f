// Fused GS / GD iteration kernels for gfx950.
//
// One GS iteration of the reference (src/algorithms.py:30-38)
//     B = a_in exp(i angle A); C = fft2(B); D = |a_T| exp(i angle C); A = ifft2(D)
// is split at the separable 2-D transform boundaries so that every HBM round
// trip does useful work on both sides of it:
//     col pass : X --fwd col FFT--> C --stats, D = a_T C/|C|--> --inv col FFT--> Y
//     row pass : Y --inv row FFT--> A --B = a_in A/|A|-->      --fwd row FFT--> X
// X holds the row-transformed B, Y the column-inverse-transformed D. The 1/S of
// ifft2 is dropped (the projections are scale free; only angles leave the
// loop). Per pixel and iteration this moves 8+8 B per pass plus the target:
// 36 B (f32 target) or 33 B (u8 target) instead of 68 B for unfused 2-D FFTs.
//
// GD (src/algorithms.py:83-93) needs the global max of |F|^2 before the
// gradient can be formed: its column side is one launch with a grid
// max-barrier between the forward and the inverse transform where the grid is
// resident at once (COL_GD_FUSED), else two launches (stats, then recompute F
// and build the gradient); its row side fuses the inverse row transform, the
// x/|x| Jacobian-transpose, the update and the next forward row transform.
#pragma once
#include <hip/hip_fp16.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "fft_core.hpp"
#include "fft_shuffle.hpp"

namespace slm {

// ------------------------------------------------------------------------
// launch parameter blocks (one struct per kernel family => uniform signatures)
// ------------------------------------------------------------------------
struct RowParams {
    const float2* in;        // row-pass input (Y, or X for the debug FFT)
    float2* out;             // row-pass output (X)
    const float* ain;        // incoming amplitude [H][W], nullptr = uniform 1
    const float* phase_in;   // warm-start phase [B][H][W]
    float* phase_out;        // output phase [B][H][W]
    float2* field;           // GD state x [B][H][W] (written)
    const float2* field_src; // GD state read by this launch: the initial field (iteration 0 of a host-set
                             // field, which a rerun must find intact) or `field`
    const float* lr;         // GD learning rate per iteration
    const int* stop_iter;    // [B], INT_MAX while running
    int checked;             // tolerance run: honour stop_iter (else it is never read)
    int iter;                // iteration index of this launch
    int wt;                  // write-through field stores (store_field)
    int W;                   // row length (== template W; kept for checks)
    int H;                   // rows per hologram (column stride of the blocked layout)
    long long holo;          // elements per hologram (H * W)
    float inv_s;             // 1 / (H * W)
    const void* tw;          // twiddle table for length W (float2 or double2)
    unsigned long long* trace;  // SLM_TRACE builds: [tile][8] phase timestamps (kTraceSlots)
    int B;                   // holograms
    int ntile;               // row groups per hologram (H / rows per workgroup)
    const float2* in2;       // ROW_GD_LIN: second column-pass output (inverse of mask F T)
    const double* gmax;      // ROW_GD_LIN: [B][max_loops][nwg_col] column-workgroup maxima of |F|^2
    const float* norm;       // ROW_GD_LIN: max(T) per hologram
    int nwg_col;             // ROW_GD_LIN: column workgroups per hologram
    int max_loops;           // ROW_GD_LIN: gmax slab stride
};

struct ColParams {
    const float2* in;        // column-pass input X
    const float2* in_alt;    // GD ping-pong partner (expected-output kernel)
    float2* out;             // column-pass output Y
    const void* tgt;         // target intensity T [B][H][W] (uint8 or float)
    double* partials;        // [B][max_loops][nwg] x 4 doubles: max, sum E^2, sum E T, 0
    float* e_out;            // |C|^2 of the final iteration [B][H][W]
    float* e_blk;            // COL_EXPECTED: |C|^2 in layout Y (relayout to e_out by the host)
    const int* stop_iter;    // [B]
    int checked;             // tolerance run: honour stop_iter (else it is never read)
    const float* norm;       // max(T) per hologram
    int iter;                // iteration index of this launch
    int max_loops;           // partial-slab stride
    int loops;               // iterations of this run
    int wt;                  // write-through field stores (store_field)
    int W;                   // image width (row stride)
    int nwg;                 // column workgroups per hologram (W / CW)
    long long holo;          // elements per hologram
    float wa;                // GD white_attention
    float stat_k;            // GS: power of two ~ 1/holo^2 scaling E^2 in the float32 partial sums (no overflow)
    const void* tw;          // twiddle table for length H (float2 or double2)
    unsigned long long* trace;  // SLM_TRACE builds: [tile][8] phase timestamps (kTraceSlots)
    int B;                   // holograms
    double* gresult;         // COL_GD_FUSED: [B][max_loops] hologram max per iteration (kUnset before)
    double* gslots;          // COL_GD_FUSED: [B][max_loops][nwg] workgroup max per iteration (kUnset before)
    int* fault;              // COL_GD_FUSED: set when a grid wait gave up
    int skip_wg_plus1;       // COL_GD_FUSED test knob: workgroup (value - 1) never publishes (0 = off)
    float2* out2;            // COL_GD_LIN: second output (inverse column transform of mask F T)
    double* gmax;            // COL_GD_LIN: [B][max_loops][nwg] workgroup maxima of |F|^2 (dense)
};

enum RowMode : int {
    ROW_GS_MAIN = 0,      // Y -> inv -> a_in A/|A| -> fwd -> X
    ROW_GS_PHASE = 1,     // Y -> inv -> angle -> phase_out
    ROW_PHASE_FWD = 2,    // phase_in -> a_in e^{i phi} -> fwd -> X (warm start)
    ROW_GD_INIT_Y = 3,    // Y -> inv -> x = a_in A/|A| (fourier guess) -> field, fwd(x/|x| a_in) -> X
    ROW_GD_INIT_FIELD = 4,// field -> fwd(x/|x| a_in) -> X
    ROW_GD_MAIN = 5,      // Y -> inv -> gradient, update field -> fwd -> X
    ROW_FFT_FWD = 6,      // in -> fwd -> out (test entry)
    ROW_FFT_INV = 7,      // in -> inv -> out (test entry)
    ROW_GD_LIN = 8,       // s U - V (s from the column maxima) -> inv -> gradient, update field -> fwd -> X
    ROW_NUM_MODES = 9
};

enum ColMode : int {
    COL_GS_MAIN = 0,      // X -> fwd -> stats, a_T C/|C| -> inv -> Y
    COL_REAL_INV = 1,     // T -> a_T -> inv -> Y (cold start, fourier guess)
    COL_EXPECTED = 2,     // X -> fwd -> |C|^2 -> e_out
    COL_GD_STATS = 3,     // X -> fwd -> stats of P = |F|^2
    COL_GD_GRAD = 4,      // X -> fwd -> mask F (sP - T) -> inv -> Y
    COL_FFT_FWD = 5,      // in -> fwd -> out (test entry)
    COL_FFT_INV = 6,      // in -> inv -> out (test entry)
    COL_GD_FUSED = 7,     // X -> fwd -> stats, grid barrier (global max) -> mask F (sP - T) -> inv -> Y
    COL_GD_LIN = 8,       // X -> fwd -> stats; mask F P -> inv -> Y, mask F T -> inv -> Y2 (no global max needed)
    COL_NUM_MODES = 9
};

// target element types: 0 = uint8 (amplitude rounded to float16 as numpy's
// sqrt(uint8) does), 1 = float32 (amplitude = sqrtf),
// 2 = float32 amplitude a_T = sqrtf(T) already (the device copy of a float32
// target in GS plans: set_target takes the square root once, the iteration
// kernels read a_T and form T = a_T^2 only for the error statistics).
enum TgtType : int { TGT_U8 = 0, TGT_F32 = 1, TGT_AMP = 2, TGT_NUM = 3 };

using RowFn = void (*)(RowParams);
using ColFn = void (*)(ColParams);

// arithmetic precision of the transforms: 0 = float32, 1 = float64 (storage is complex64 in both)
enum Precision : int { PREC_F32 = 0, PREC_F64 = 1, PREC_NUM = 2 };

// ------------------------------------------------------------------------
// geometry
// ------------------------------------------------------------------------
// Workgroups of both passes keep their LDS at <= 80 KiB where the line allows,
// so two of them share a CU and one's loads overlap the other's transforms.
constexpr int kLdsPair = 80 * 1024;

// Lines per thread. A thread may carry L = 2 rows (row kernels) or columns
// (column kernels) of the same tile: both lines share the thread's twiddles
// (cached in registers), its exchange barriers and its address arithmetic, and
// the two columns of a column tile are one 16-B access. Used for the narrow
// column plans of kColLines2MinN and longer: one column per thread in
// 8-wave workgroups could not hold a twiddle cache there (the 4096 column pass
// had fallen back to table reads inside every pass).
constexpr int kColLines2MinN = 4096;  // 4096: col pass 715 -> 626 us for 8 x 4096^2 (twiddles cached again)
// Rows: two adjacent rows per thread of the float32 4096 narrow plan, their
// pieces of each 128-B line loaded and stored back to back (slot-major): the
// 8 x 4096^2 row pass 789-806 -> 688 us, 1 x 4096^2 neutral, phases bitwise
// equal (profiles/r04/ab_rows_l2_s6.txt; 228 VGPRs, two workgroups per CU).
// Float64 rows keep one row per thread (290 VGPRs with two: one wave per SIMD).
constexpr int kRowLines2MinN = 4096;
// Wave-local exchanges: where every thread of a line sits in one wave, a
// Stockham exchange needs no workgroup barrier -- LDS writes, s_waitcnt, LDS
// reads (fft_core.hpp, exchange_sync). That holds with the default lane maps
// for rows of T <= 16 threads and for column tiles of T x CW / L <= 64 threads;
// rows of T = 32 are remapped so each row is one half-wave (T consecutive
// lanes per row). Measured per launch (f32,
// tools/kt.py, gpurun_out/s6): rows 256^2 x 64 15.66 -> 14.33 us, one 256^2
// 4.24 -> 3.98 us, 16 x 512^2 23.45 -> 22.95 us; remapping rows of T = 64
// (1024 wide) was slower (64 x 1024^2 260 -> 276 us), and so was remapping
// columns to one column per wave (64 x 1024^2 265 -> 567 us: a wave then reads
// 8 B per lane at a 32-B stride), so neither is done.
template <int K>
constexpr bool row_wave_remap(int lines_per_thread) {
    return lines_per_thread == 1 && PlanOf<K>::T == 32;
}
template <int K>
constexpr bool row_wave_local(int lines_per_thread) {
    return lines_per_thread == 1 && (PlanOf<K>::T <= 16 || row_wave_remap<K>(lines_per_thread));
}

template <int K, bool COL, int P = PREC_F32>
constexpr int lines_of() {
    return (kPlans[K].variant == 1 && PlanOf<K>::N >= (COL ? kColLines2MinN : kRowLines2MinN) &&
            (COL || P == PREC_F32))
               ? 2
               : 1;
}

template <int K, int P = PREC_F32>  // plan key of the row length, precision
struct RowCfg {
    static constexpr int T = PlanOf<K>::T;
    static constexpr int L = lines_of<K, false, P>();  // rows per thread
    // rows per workgroup: a row quad (whole 128-B lines of the blocked layout),
    // or a row pair when a quad would not leave room for two workgroups per CU
    // and a pair still fills 8 waves (the partner pair, which reads the other
    // half of each 128-B line, is placed on the same XCD: row_kernel remap)
    // Narrow plans (single small images: few workgroups per CU) always use
    // pairs: twice the workgroups, measured 11.6 -> 9.1 us per 1024^2 row pass.
    static constexpr bool kPairs = (4 * PlanOf<K>::ROWSTRIDE * 8 > kLdsPair && T >= 256) ||
                                   kPlans[K].variant == 1;
    // 4096 narrow rows with one row per thread run one row per workgroup: two
    // workgroups of 4 waves per CU instead of one of 8 (8 x 4096^2 row pass
    // 931 -> 755 us with write-back stores)
    static constexpr bool kSingle = kPlans[K].variant == 1 && PlanOf<K>::N >= 4096 && L == 1;
    static constexpr int RPW = (T >= 64) ? (kSingle ? 1 : kPairs ? 2 : 4) : 256 / T;
    static_assert(RPW % L == 0, "rows per workgroup must be a multiple of the rows per thread");
    static constexpr bool kWave = row_wave_local<K>(L);    // each row inside one wave (wave-local exchanges)
    static constexpr bool kRemap = row_wave_remap<K>(L);   // ... by T consecutive lanes per row
    static constexpr int RL = RPW / L;              // row groups across lanes
    static constexpr int QR = RL < 4 ? RL : 4;      // rows interleaved across a wave
    static constexpr int THREADS = RL * T;
};

template <int K, int CW>  // plan key of the column length
struct ColCfg {
    static constexpr int T = PlanOf<K>::T;
    static constexpr int L = (CW % 2 == 0) ? lines_of<K, true>() : 1;  // columns per thread
    static constexpr int THREADS = (CW / L) * T;
    static constexpr bool kWave = T * (CW / L) <= 64;  // each column inside one wave
    static constexpr bool kValid =
        THREADS >= 64 && THREADS <= 1024 && lds_line(PlanOf<K>::N) * CW * 8 <= 160 * 1024;
};

// XCD-aware bijective remap: blocks that share (id % 8) — one XCD under the
// observed round-robin dispatch — get consecutive logical column groups, so
// the partial 128-B lines of narrow column tiles are shared through one L2.
// Speed only; correctness does not depend on placement.
__device__ __forceinline__ int xcd_remap(int id, int n) {
    const int q = n >> 3, r = n & 7;
    const int xcd = id & 7, k = id >> 3;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + k;
}

__device__ __forceinline__ int xcd_remap_fwd(int id, int n) { return xcd_remap(id, n); }

// Phase timeline of one workgroup (SLM_TRACE diagnostic builds only), slots
// [tile][8]: s_memrealtime (100 MHz, chip-wide) at 0 tile start (loads
// issued), 1 loads complete, 2 transforms done, 3 stores complete, 4 kernel
// entry (before the twiddle loads); 5 HW_ID and 6 XCC_ID of the wave.
#ifndef SLM_TRACE
#define SLM_TRACE 0
#endif
constexpr int kTraceSlots = 8;
__device__ __forceinline__ void trace_point(unsigned long long* tr, long long wgid, int i, bool drain) {
#if SLM_TRACE
    if (drain) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (tr && threadIdx.x == 0) tr[wgid * kTraceSlots + i] = __builtin_amdgcn_s_memrealtime();
#else
    (void)tr;
    (void)wgid;
    (void)i;
    (void)drain;
#endif
}
__device__ __forceinline__ void trace_entry(unsigned long long* tr) {
#if SLM_TRACE
    if (tr && threadIdx.x == 0 && blockIdx.x < gridDim.x) {
        const long long wg = xcd_remap_fwd(blockIdx.x, gridDim.x);
        tr[wg * kTraceSlots + 4] = __builtin_amdgcn_s_memrealtime();
        tr[wg * kTraceSlots + 5] = (unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 4);
        tr[wg * kTraceSlots + 6] = (unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 20);
    }
#else
    (void)tr;
#endif
}

// Kernels declare no waves-per-SIMD floor (__launch_bounds__(threads, 1)):
// forcing the register budget to what LDS would allow (e.g. 128 VGPRs for
// four workgroups of the batched 1024 tiles) spilled the float64 transforms
// and was slower everywhere (r02).

// Internal layout of the iteration state (X, Y, GD field, device target):
// 4-column blocks, [x / 4][y][x % 4]. A 4-column panel is one contiguous run
// (column pass), and rows y..y+3 (y % 4 == 0) of a block form one 128-B line
// (row pass on row quads), so both passes move whole lines. User-facing
// arrays (phases, a_in, expected output) stay row-major.
// Two blocked layouts, one per direction of the transpose. X (the row pass's
// output, the column pass's input, and the target) and Y (the column pass's
// output, the row pass's input, and the GD field) are [x / P][y][x % P] with
// their own panel widths P: a column tile reads / writes whole panels of the
// narrower layout, a row tile whole chunks of the wider one. The default pair
// is 4-wide both ways (kPanelLog2); wider X or Y panels at 4096 trade the row
// pass against the column pass.
constexpr int kPanelLog2 = 2;
// Layout pairs, chosen per plan (slm_plan_create): 0 = the default panels;
// 1 = 8-wide X / 2-wide Y for single 1024^2 images on the narrow plan (2-column
// tiles write whole Y panels, row pairs write 128-B X chunks: 1024^2 GS
// col 10.31 -> 10.06 us, row 9.50 -> 8.77 us on one box; the batched and
// 4096 plans measured slower with it: 8 x 4096^2 1317 -> 1405 us).
enum LayoutId : int { LAYOUT_DEFAULT = 0, LAYOUT_NARROW = 1, kNumLayouts = 2 };
template <int LID>
struct LayoutOf {
    static constexpr int X = LID == LAYOUT_NARROW ? 3 : kPanelLog2;
    static constexpr int Y = LID == LAYOUT_NARROW ? 1 : kPanelLog2;
};
__host__ __device__ constexpr int layout_x_log2(int lid) { return lid == LAYOUT_NARROW ? 3 : kPanelLog2; }
__host__ __device__ constexpr int layout_y_log2(int lid) { return lid == LAYOUT_NARROW ? 1 : kPanelLog2; }
// plans instantiated with the narrow layout pair (plan key 11: 1024 = 8.4.4.8)
template <int K>
constexpr bool kHasNarrowLayout = (K == 11);
template <int PLOG>
__host__ __device__ __forceinline__ long long blk_index(long long y, int x, int H) {
    return (((long long)(x >> PLOG) * H + y) << PLOG) + (x & ((1 << PLOG) - 1));
}
template <int PLOG>
constexpr int kPanelOf = 1 << PLOG;  // row y + 1 sits kPanelOf elements after row y

// ------------------------------------------------------------------------
// element-wise pieces
// ------------------------------------------------------------------------
// 1/sqrt(n2) to ~0.5 ulp of the compute type: the hardware float estimate plus
// Newton steps (the projections run every iteration, their rounding accumulates).
__device__ __forceinline__ float rsqrt_nr(float n2) {
    const float r = rsqrtf(n2);
    return fmaf(r * 0.5f, fmaf(-n2 * r, r, 1.0f), r);
}
__device__ __forceinline__ double rsqrt_nr(double n2) {
    // one step from the float estimate: ~1e-14 relative, far below the
    // complex64 rounding of every stored value
    const double r = (double)rsqrtf((float)n2);
    return fma(r * 0.5, fma(-n2 * r, r, 1.0), r);
}
// a * z / |z|, with angle(0) = 0 -> a (np.angle(0) == 0, src/algorithms.py:30,33).
template <class C>
__device__ __forceinline__ C unit_scale(C z, Scalar<C> a) {
    using S = Scalar<C>;
    const S n2 = z.x * z.x + z.y * z.y;
    const bool zero = (n2 == (S)0);  // select, not branch: no divergence in the unrolled loops
    const S r = a * rsqrt_nr(zero ? (S)1 : n2);
    return mk<C>(zero ? a : z.x * r, zero ? (S)0 : z.y * r);
}
// x / |x| * a (src/algorithms.py:84); |x| = 0 gives NaN as in the reference
template <class C>
__device__ __forceinline__ C normalize(C x, Scalar<C> a) {
    const Scalar<C> r = rsqrt_nr(x.x * x.x + x.y * x.y);
    return mk<C>(x.x * r * a, x.y * r * a);
}

// Lane i <- lane i ^ 4 within each 16-lane DPP row (row_ror:4 moves lane i - 4
// into lane i, row_ror:12 lane i + 4; lanes with bit 2 set take the first)
__device__ __forceinline__ float lane_xor4(float x, bool b2) {
    const int v = __builtin_bit_cast(int, x);
    const int dn = __builtin_amdgcn_update_dpp(0, v, 0x124, 0xF, 0xF, false);
    const int up = __builtin_amdgcn_update_dpp(0, v, 0x12C, 0xF, 0xF, false);
    return __builtin_bit_cast(float, b2 ? dn : up);
}
__device__ __forceinline__ float2 lane_xor4(float2 z, bool b2) {
    return make_float2(lane_xor4(z.x, b2), lane_xor4(z.y, b2));
}

// Field stores of the iteration passes. wt = write-through (agent-scope
// relaxed atomic store = global_store sc1): the bytes go to memory as they are
// stored, so the kernel ends with no dirty L2 lines to write back before the
// dependent launch (MI355X_MICROARCH.md: a boundary costs + dirty bytes / 6 TB/s).
__device__ __forceinline__ void store_field(float2* dst, float2 v, int wt) {
    if (wt)
        __hip_atomic_store(reinterpret_cast<unsigned long long*>(dst), __builtin_bit_cast(unsigned long long, v),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else
        *dst = v;
}

// Grid max-barrier of one hologram's column workgroups (COL_GD_FUSED), run by
// one thread per workgroup after it stored its statistics partials. The host
// launches that kernel only when every workgroup of the grid is resident at
// once (occupancy query x CUs >= grid, one tile per workgroup), so every
// waiter is eventually released; the bounded spin (2^21 polls of s_sleep 8,
// about 0.5-1.5 s) is a guard that turns a broken residency assumption into a
// fault flag, never a hang: later waits of the run leave at once, and the host
// redoes the run on the two-launch path (slm_capi.hip, recover_grid_fault).
//
// Device-scope atomics on one address serialise at the memory side: a flat
// 512-workgroup counter, and a two-level counter tree, both measured ~13 us
// from the last arrival to the release (tools/trace_gd.py); (max, generation)
// slots with a flag measured ~4 us (five dependent memory round trips). So:
// no atomics and no flags. Every (hologram, iteration) owns a slab of
// per-workgroup slots and one result word, all preset to the bit pattern
// kUnset (no |F|^2 maximum is a NaN); a workgroup stores its max into its
// slot, workgroup 0 of the hologram polls all slots in parallel (one or two
// per thread), folds them and stores the hologram's max into the result word,
// which the other workgroups poll. Two dependent memory round trips. Values
// move with agent-scope (L2-bypassing) 8-byte stores and loads, which are
// single-copy atomic; no release / acquire fences (those write back and
// invalidate a whole XCD L2 per workgroup). Measured alternatives (GD 1024^2,
// per fused launch): every workgroup polling the whole slab itself (one round
// trip, 512 x 512 polls) 16.6 us against 14.3 us; overlapping the wait with
// the inverse transforms of the split gradient (s U - V, see COL_GD_LIN) did
// not hide it -- the last arrivals trail the first by several microseconds.
constexpr unsigned long long kUnset = ~0ull;

constexpr int kGridSpinMax = 1 << 21;
constexpr int kGridSleep = 8;
__device__ __forceinline__ void store_coherent(double* dst, double v) {
    __hip_atomic_store(reinterpret_cast<unsigned long long*>(dst), __builtin_bit_cast(unsigned long long, v),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double load_coherent(const double* src) {
    return __builtin_bit_cast(double, __hip_atomic_load(reinterpret_cast<const unsigned long long*>(src),
                                                        __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}

template <int P>
using CplxOf = std::conditional_t<P == 0, float2, double2>;

// Exchange type of float64 butterflies: float64 for narrow plans up to
// kNarrowF64XchgMax (more passes, hence more exchange roundings; single small
// images, where LDS is plentiful) while the workgroup's LDS stays <= 80 KiB,
// complex64 otherwise: half the LDS traffic, measured -2.5 % (1024^2) / -9 %
// (768x1024) per iteration for warm-start parity 1.2e-6 instead of 4.3e-7 at
// 1024^2.
constexpr int kNarrowF64XchgMax = 512;
template <int P, long long SLOTS, int K>
using XchgOf = std::conditional_t<((kPlans[K].variant == 1 && kPlans[K].n <= kNarrowF64XchgMax) && P == 1 &&
                                   SLOTS * 16 <= 80 * 1024),
                                  double2, float2>;

// float64 butterflies read their twiddles from the table where used (caching
// them in registers measured neutral at 1024^2).
template <int P, int THREADS, int K, bool COL, int L = 1>
constexpr int tw_mode() {
    if constexpr (P == 1) return TW_DIRECT;
    // float32 (measured per launch):
    //  * column kernels of 2048+ lines read the table where used (4096:
    //    156 -> 127 us, 2048: 109 -> 93 us; registers 208 -> 122, two
    //    workgroups per CU);
    //  * everything else caches every twiddle of the thread. (Row kernels that
    //    form w^2.. from w^1 ran 7-10 % faster at 2048/4096 but took the 4096^2
    //    warm-start parity from 3.1e-6 to 1.3e-5 rms after 100 iterations.)
    //  * two-column threads (L = 2) cache them again: one cache serves both lines
    if constexpr (COL && PlanOf<K>::N >= 2048 && L == 1) return TW_DIRECT;
    return THREADS <= 512 && PlanOf<K>::E <= 16 ? TW_CACHED : TW_DIRECT;
}

template <int TT>
struct TgtLoad;
// Target amplitudes. uint8: numpy's sqrt(uint8) is float16 (SURVEY.md
// appendix); every sqrt of 0..255 lies >= 100 float32 ulps from a float16
// rounding midpoint, so the hardware square root (<= 1 ulp) rounds to the same
// float16. float32: the hardware reciprocal square root plus one Newton
// (Markstein) correction -- 0 mismatches against the correctly rounded sqrtf
// over 2e5 random targets, a third of the instructions of the IEEE expansion;
// zero, denormal, infinite and negative inputs take the hardware sqrt.
template <>
struct TgtLoad<TGT_U8> {
    __device__ __forceinline__ static float load(const void* p, long long i) {
        return (float)static_cast<const uint8_t*>(p)[i];
    }
    __device__ __forceinline__ static float amp(float t) {
        return __half2float(__float2half_rn(__builtin_amdgcn_sqrtf(t)));
    }
    __device__ __forceinline__ static float intensity(float t) { return t; }
};
template <>
struct TgtLoad<TGT_F32> {
    __device__ __forceinline__ static float load(const void* p, long long i) {
        return static_cast<const float*>(p)[i];
    }
    __device__ __forceinline__ static float amp(float t) {
        const float y = __builtin_amdgcn_rsqf(t);
        const float s = t * y;
        const float r = fmaf(-s, s, t);
        const float c = fmaf(r, 0.5f * y, s);
        return (t >= 1.17549435e-38f && t <= 3.40282347e38f) ? c : __builtin_amdgcn_sqrtf(t);
    }
    __device__ __forceinline__ static float intensity(float t) { return t; }
};
// The statistics' T from a_T: a_T^2 is within 2^-23 of T relative (one
// correctly rounded square root, one rounded square), so sum E T moves by
// ~1e-7 / sqrt(pixels) relative: far inside the error curves' 1e-4 gates.
template <>
struct TgtLoad<TGT_AMP> {
    __device__ __forceinline__ static float load(const void* p, long long i) {
        return static_cast<const float*>(p)[i];
    }
    __device__ __forceinline__ static float amp(float a) { return a; }
    __device__ __forceinline__ static float intensity(float a) { return a * a; }
};

// Wave reductions of doubles without the LDS pipe (instead of __shfl_xor
// through ds_bpermute: measured GD 1024^2 fused column pass 13.3 -> 12.4 us, the
// statistics and the barrier fold sit before and inside its grid wait):
// within each 16-lane row a rotation by 4 then by 8 folds each residue class
// mod 4 (whichever way DPP row_ror turns), two quad_perm steps fold the quad;
// v_permlane16_swap / v_permlane32_swap of a value with itself then hand every
// lane both rows / halves. Every lane ends with the wave total (the lanes'
// association orders differ; thread 0's value is the one used).
template <int CTRL>
__device__ __forceinline__ double dpp_f64(double x) {
    const unsigned long long b = __builtin_bit_cast(unsigned long long, x);
    const unsigned lo = (unsigned)__builtin_amdgcn_update_dpp(0, (int)(unsigned)b, CTRL, 0xF, 0xF, false);
    const unsigned hi = (unsigned)__builtin_amdgcn_update_dpp(0, (int)(unsigned)(b >> 32), CTRL, 0xF, 0xF, false);
    return __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lo);
}
template <bool HALVES32>
__device__ __forceinline__ void lane_halves_f64(double x, double& lower, double& upper) {
    const unsigned long long b = __builtin_bit_cast(unsigned long long, x);
    const unsigned lo = (unsigned)b, hi = (unsigned)(b >> 32);
    const auto rl = HALVES32 ? __builtin_amdgcn_permlane32_swap(lo, lo, false, false)
                             : __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
    const auto rh = HALVES32 ? __builtin_amdgcn_permlane32_swap(hi, hi, false, false)
                             : __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
    lower = __builtin_bit_cast(double, ((unsigned long long)rh[0] << 32) | rl[0]);
    upper = __builtin_bit_cast(double, ((unsigned long long)rh[1] << 32) | rl[1]);
}
constexpr int kDppRor4 = 0x124, kDppRor8 = 0x128, kDppQuadXor1 = 0xB1, kDppQuadXor2 = 0x4E;
template <bool MAX>
__device__ __forceinline__ double wave_fold(double x) {
    auto op = [](double a, double b) { return MAX ? fmax(a, b) : a + b; };
    x = op(x, dpp_f64<kDppRor4>(x));
    x = op(x, dpp_f64<kDppRor8>(x));
    x = op(x, dpp_f64<kDppQuadXor1>(x));
    x = op(x, dpp_f64<kDppQuadXor2>(x));
    double a, b;
    lane_halves_f64<false>(x, a, b);
    x = op(a, b);
    lane_halves_f64<true>(x, a, b);
    return op(a, b);
}

// Block-wide reduction of (max, sum, sum); result valid in thread 0.
template <int THREADS>
__device__ __forceinline__ void block_reduce_stats(double& mx, double& s2, double& st) {
    if constexpr (THREADS % 64 != 0) {
        // a partial last wave (the panel plans' column tiles, e.g. 4 x 36 threads):
        // its missing lanes hold no values, so fold inside 16-lane rows (DPP row
        // and quad moves) -- or quads where the block is not whole rows -- and
        // combine those through LDS
        constexpr int G = THREADS % 16 == 0 ? 16 : 4;
        static_assert(THREADS % 4 == 0, "partial waves of whole quads");
        constexpr int NR = THREADS / G;
        __shared__ double red16[NR][3];
        auto fold = [](double x, auto op) {
            if constexpr (G == 16) {
                x = op(x, dpp_f64<kDppRor4>(x));
                x = op(x, dpp_f64<kDppRor8>(x));
            }
            x = op(x, dpp_f64<kDppQuadXor1>(x));
            return op(x, dpp_f64<kDppQuadXor2>(x));
        };
        auto fmx = [](double a, double b) { return fmax(a, b); };
        auto add = [](double a, double b) { return a + b; };
        mx = fold(mx, fmx);
        s2 = fold(s2, add);
        st = fold(st, add);
        if (threadIdx.x % G == 0) {
            red16[threadIdx.x / G][0] = mx;
            red16[threadIdx.x / G][1] = s2;
            red16[threadIdx.x / G][2] = st;
        }
        lds_barrier();
        if (threadIdx.x == 0) {
            for (int r = 1; r < NR; ++r) {
                mx = fmax(mx, red16[r][0]);
                s2 += red16[r][1];
                st += red16[r][2];
            }
        }
        return;
    }
    constexpr int NW = (THREADS + 63) / 64;
    __shared__ double red[NW][3];
    mx = wave_fold<true>(mx);
    s2 = wave_fold<false>(s2);
    st = wave_fold<false>(st);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    if (NW > 1) {
        if (lane == 0) {
            red[wid][0] = mx;
            red[wid][1] = s2;
            red[wid][2] = st;
        }
        lds_barrier();
        if (threadIdx.x == 0) {
            for (int w = 1; w < NW; ++w) {
                mx = fmax(mx, red[w][0]);
                s2 += red[w][1];
                st += red[w][2];
            }
        }
    }
}

// Block-wide max; result valid in thread 0.
template <int THREADS>
__device__ __forceinline__ void block_reduce_max(double& mx) {
    constexpr int NW = (THREADS + 63) / 64;
    __shared__ double redm[NW];
    mx = wave_fold<true>(mx);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    if (NW > 1) {
        if (lane == 0) redm[wid] = mx;
        lds_barrier();
        if (threadIdx.x == 0)
            for (int w = 1; w < NW; ++w) mx = fmax(mx, redm[w]);
    }
}

__device__ __forceinline__ unsigned long long load_coherent_bits(const double* src) {
    return __hip_atomic_load(reinterpret_cast<const unsigned long long*>(src), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
}
// spin until *src is set; returns its value. Gives up (and raises the fault
// flag) after the guard, or as soon as another waiter has raised it: once one
// barrier of the run has failed every later wait returns at once, so a broken
// residency assumption costs one guard interval, not one per iteration.
__device__ __forceinline__ double wait_set(const double* src, int* fault) {
    unsigned long long v;
    int spins = 0;
    while ((v = load_coherent_bits(src)) == kUnset) {
        if ((spins & 63) == 0 && __hip_atomic_load(fault, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return 0.0;
        __builtin_amdgcn_s_sleep(kGridSleep);
        if (++spins > kGridSpinMax) {
            __hip_atomic_store(fault, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            return 0.0;
        }
    }
    return __builtin_bit_cast(double, v);
}

// Global max of one hologram's per-workgroup maxima `mx` (every thread of the
// workgroup calls it; thread 0's `mx` counts). slots: this (hologram,
// iteration)'s nwg slots; result: its result word. Returns the max in every
// thread (0 after a fault: the host then discards the run). skip_wg_plus1 - 1
// is a workgroup that never publishes (fault-path test knob; 0 = none).
template <int THREADS>
__device__ __forceinline__ double grid_max_barrier(double* slots, double* result, double mx, int wg, int nwg,
                                                   int* fault, int skip_wg_plus1) {
    __shared__ double shared_max;
    lds_barrier();  // the statistics reduction's LDS is reused below
    if (wg == 0) {
        double m = threadIdx.x == 0 ? mx : 0.0;
        for (int k = 1 + threadIdx.x; k < nwg; k += THREADS) m = fmax(m, wait_set(slots + k, fault));
        block_reduce_max<THREADS>(m);
        if (threadIdx.x == 0) {
            store_coherent(result, m);
            shared_max = m;
        }
    } else if (threadIdx.x == 0) {
        if (wg + 1 != skip_wg_plus1) store_coherent(slots + wg, mx);
        shared_max = wait_set(result, fault);
    }
    lds_barrier();
    return shared_max;
}

// state type between passes: complex64 when the exchange is complex64 (see
// fft_core.hpp, Stockham driver), else the compute type
template <int P, class X>
using StateOf = std::conditional_t<std::is_same_v<X, float2>, float2, CplxOf<P>>;

// Kernel-argument prologue: the fields a tile's addresses need, pulled into
// SGPRs together (one scalar round trip; left to itself the compiler issues one
// per branch of the tile setup before the first field load can go out).
template <class A>
__device__ __forceinline__ void sgpr_pin1(const A& a) {
    asm volatile("" ::"s"(a));
}
template <class... A>
__device__ __forceinline__ void sgpr_pin(const A&... a) {
    (sgpr_pin1(a), ...);
}

// ------------------------------------------------------------------------
// tile of a workgroup (both passes)
// ------------------------------------------------------------------------
// One tile (column panel or row group of one hologram) per workgroup, grid =
// tiles; the XCD-aware remap gives the workgroups of an XCD neighbouring
// tiles. (A persistent loop prefetching the next tile's inputs into registers
// measured neutral: the transforms, not the loads, bound a tile.)
template <class LoadF, class ProcF, class VA, class TA>
__device__ __forceinline__ void tile_loop(long long total, LoadF&& load, ProcF&& process, VA& v, TA& tv) {
    const long long tile = xcd_remap(blockIdx.x, gridDim.x);
    if (tile >= total) return;
    load(tile, v, tv);
    process(tile, v, tv);
}

// ------------------------------------------------------------------------
// row pass
// ------------------------------------------------------------------------
// Double-buffered LDS exchanges (fft_core.hpp, LdsLine / LdsTile ALT): one
// barrier per exchange instead of two, for twice the exchange LDS. Used where
// the second buffer leaves the workgroups per CU the launch gets unchanged.
// Measured: 1024^2 GS 18.3 -> 17.8 us of kernels per iteration; the 4096 rows
// (2 x 34 KB per one-row workgroup still fits the two workgroups their VGPRs
// allow) gained nothing (8 x 4096^2 row pass 799 -> 795 us, one image
// 100 -> 105 us), and 4096 columns would drop to one workgroup per CU.
template <int K, bool COL>
constexpr bool kLdsDouble = K == 11;

// Wave-shuffle transform pair (fft_shuffle.hpp) for the float32 GS iteration
// on 1024-point narrow lines (plan key 11, the headline 1024^2 image): two of
// the pair's six exchanges go through LDS, four are v_permlane swaps. (A
// 4096-point shuffle pair for the float32 rows measured slower, 862 against
// 788 us per 8 x 4096^2 row pass, and failed the float32 +100 gate at 1.02e-5:
// profiles/r04/ab_shuf4096_s1.txt.)
// Float64 butterflies run the pair too (double values between its passes, the
// LDS exchange in complex64), for the GS iteration kernels.
template <int K, int P>
constexpr bool kShuffle = PlanOf<K>::N == kShufN && PlanOf<K>::E == 8;

template <int K, int MODE, int P, int LID>
__global__ void __launch_bounds__((RowCfg<K, P>::THREADS), 1) row_kernel(RowParams p) {
    constexpr int LAYOUT_X = LayoutOf<LID>::X, LAYOUT_Y = LayoutOf<LID>::Y;
    using C = CplxOf<P>;
    using S = Scalar<C>;
    constexpr int W = PlanOf<K>::N;
    constexpr int E = PlanOf<K>::E;
    constexpr int T = PlanOf<K>::T;
    constexpr int RPW = RowCfg<K, P>::RPW;
    constexpr int L = RowCfg<K, P>::L;
    constexpr int LINE = PlanOf<K>::ROWSTRIDE;
    constexpr int TL = T < 16 ? T : 16;
    using X = XchgOf<P, (long long)RPW * LINE, K>;
    using V = StateOf<P, X>;
    constexpr int ALT = kLdsDouble<K, false> ? RPW * LINE : 0;
    constexpr int SMEM_ROW = (ALT ? 2 : 1) * RPW * LINE;
    __shared__ X smem[SMEM_ROW];

    // lane -> (row group within the quad, transform thread t): TL consecutive
    // t of one row group, then the next group of the quad. One wave instruction
    // touches 16 consecutive x of 4 rows = four whole 128-B lines of the
    // blocked layout, and a 16-lane LDS write group stays inside one row. A
    // thread carries rows lrow * L + l, l < L.
    constexpr int QR = RowCfg<K, P>::QR;
    constexpr bool WV = RowCfg<K, P>::kWave;
    // wave-shuffle pair: lane bit 0 selects the row of the pair, t per fft_shuffle.hpp
    constexpr bool SHUF = kShuffle<K, P> &&
                          (MODE == ROW_GS_MAIN || (P == PREC_F32 && (MODE == ROW_GD_MAIN || MODE == ROW_GD_LIN))) &&
                          RPW == 2 && L == 1;
    // Row pairs in 4-wide panels (the float32 4096 rows): a row pair's piece of
    // a panel is one 64-B sector (4 columns x 2 rows). Lanes t and t ^ 4 swap
    // halves (lane_xor4) so that each load / store instruction moves whole
    // sectors -- lanes with t bit 2 clear the row-r halves of panel t / 4, the
    // others the row-(r+1) halves of the same panel -- instead of every
    // instruction writing half of each sector of one row (r04: 1.145x write and
    // 1.15x read traffic per 8 x 4096^2 row pass in partly merged sectors,
    // TCC_EA0_WRREQ_64B = all write requests, profiles/r05).
    constexpr bool kSector = L == 2 && kPanelOf<LAYOUT_X> == 4 && kPanelOf<LAYOUT_Y> == 4 && !SHUF &&
                             !RowCfg<K, P>::kRemap && RowCfg<K, P>::RL == 1 && T % 8 == 0 && std::is_same_v<V, float2>;
    int t, lrow;
    if constexpr (SHUF) {
        t = shuffle_t(threadIdx.x);
        lrow = threadIdx.x & 1;
    } else if constexpr (RowCfg<K, P>::kRemap) {  // wave-line: T consecutive lanes per row, rows never cross a wave
        t = threadIdx.x % T;
        lrow = threadIdx.x / T;
    } else {
        const int tlo = threadIdx.x % TL;
        const int q4 = (threadIdx.x / TL) % QR;
        const int rest = threadIdx.x / (QR * TL);
        const int qq = rest / (T / TL);
        t = tlo + TL * (rest - qq * (T / TL));
        lrow = (qq * QR + q4) * L;
    }
    const long long bstep = (long long)T * p.H;  // slot m adds m * bstep (blocked layout)
    const LdsLine<X, WV ? 0 : ALT, WV> lds{smem + lrow * LINE, LINE};
    if constexpr (MODE == ROW_GS_MAIN || MODE == ROW_GD_MAIN || MODE == ROW_GD_LIN) trace_entry(p.trace);
    sgpr_pin(p.in, p.out, p.holo, p.H, p.B, p.ntile, p.tw, p.ain, p.wt, gridDim.x);
    Twiddles<K, C, tw_mode<P, RowCfg<K, P>::THREADS, K, false>()> tw;
    static_assert(!SHUF || (std::is_same_v<X, float2> && sizeof(smem) >= 4 * kShufN * sizeof(float2)),
                  "the shuffle pair needs two 2-line complex64 exchange buffers");
    ShuffleTwT<C> stw;
    if constexpr (SHUF)
        load_shuffle_tw(stw, threadIdx.x, static_cast<const C*>(p.tw) + twiddle_count_key(K));
    else
        load_twiddles<K, C>(tw, t, p.tw);

    // tile = (hologram b, row group g); rows g * RPW + lrow + l. Inputs (Y,
    // the GD field) are in layout Y, outputs (X) in layout X; row l + 1 sits
    // kPanelOf<layout> elements after row l.
    constexpr int PY = kPanelOf<LAYOUT_Y>, PX = kPanelOf<LAYOUT_X>;
    auto where = [&](long long tile, int& b, long long& hoff, long long& roff, long long& boff, long long& xoff) {
        b = (int)(tile / p.ntile);
        const int row = (int)(tile - (long long)b * p.ntile) * RPW + lrow;
        hoff = (long long)b * p.holo;
        roff = (long long)row * W;                             // row-major (user arrays)
        boff = hoff + blk_index<LAYOUT_Y>(row, t, p.H);        // blocked input / field
        xoff = hoff + blk_index<LAYOUT_X>(row, t, p.H);        // blocked output
    };
    auto load = [&](long long tile, V (&v)[L][E], float (&)[1]) {
        int b;
        long long hoff, roff, boff, xoff;
        where(tile, b, hoff, roff, boff, xoff);
        auto ain_at = [&](int l, int m) -> S { return p.ain ? (S)p.ain[roff + l * W + t + T * m] : (S)1; };
#pragma unroll
        for (int l = 0; l < L; ++l) {
            if constexpr (MODE == ROW_PHASE_FWD) {
#pragma unroll
                for (int m = 0; m < E; ++m) {
                    S sn, cs;
                    if constexpr (P == 0)
                        sincosf(p.phase_in[hoff + roff + l * W + t + T * m], &sn, &cs);
                    else
                        sincos((double)p.phase_in[hoff + roff + l * W + t + T * m], &sn, &cs);
                    const S a = ain_at(l, m);
                    v[l][m] = cv<V>(mk<C>(a * cs, a * sn));
                }
            } else if constexpr (MODE == ROW_GD_INIT_FIELD) {
#pragma unroll
                for (int m = 0; m < E; ++m)
                    v[l][m] = cv<V>(normalize(from_c64<C>(p.field_src[boff + PY * l + m * bstep]), ain_at(l, m)));
            }
        }
        if constexpr (MODE != ROW_PHASE_FWD && MODE != ROW_GD_INIT_FIELD && kSector) {
            // whole 64-B sectors per instruction: lane bit 2 clear loads (r, t) and
            // (r, t ^ 4), set (r + 1, t ^ 4) and (r + 1, t); one lane_xor4 restores
            const bool b2 = (t >> 2) & 1;
            const long long o1 = b2 ? PY - 4LL * p.H : 0, o2 = b2 ? PY : 4LL * p.H;
#pragma unroll
            for (int m = 0; m < E; ++m) {
                const float2 l1 = p.in[boff + o1 + m * bstep];
                const float2 l2 = p.in[boff + o2 + m * bstep];
                const float2 r = lane_xor4(b2 ? l1 : l2, b2);
                v[0][m] = b2 ? r : l1;
                v[1][m] = b2 ? l2 : r;
            }
        } else if constexpr (MODE != ROW_PHASE_FWD && MODE != ROW_GD_INIT_FIELD) {
#pragma unroll
            for (int m = 0; m < E; ++m)  // slot-major, as the stores
#pragma unroll
                for (int l = 0; l < L; ++l) v[l][m] = cv<V>(p.in[boff + PY * l + m * bstep]);
        }
    };
    auto process = [&](long long tile, V (&v)[L][E], float (&)[1]) {
        int b;
        long long hoff, roff, boff, xoff;
        where(tile, b, hoff, roff, boff, xoff);
        auto ain_at = [&](int l, int m) -> S { return p.ain ? (S)p.ain[roff + l * W + t + T * m] : (S)1; };
        // timeline of the iteration launches only (SLM_TRACE)
        unsigned long long* const trace =
            (MODE == ROW_GS_MAIN || MODE == ROW_GD_MAIN || MODE == ROW_GD_LIN) ? p.trace : nullptr;
        trace_point(trace, tile, 0, false);
        // (unchecked runs never stop early: no dependent load of the flag)
        if constexpr (MODE == ROW_GS_MAIN) {
            if (p.checked && p.iter >= p.stop_iter[b]) return;  // stopped after this iteration's column pass
        } else if constexpr (MODE == ROW_GD_MAIN || MODE == ROW_GD_LIN) {
            if (p.checked && p.iter > p.stop_iter[b]) return;
        }
        trace_point(trace, tile, 1, true);
        if constexpr (MODE == ROW_GS_PHASE) {
            fft_line_epi<K, true, C>(v, t, tw, lds, [&](int l, int m, C& z) {
                p.phase_out[hoff + roff + l * W + t + T * m] = (float)atan2(z.y, z.x);
            });
            return;
        } else if constexpr (MODE == ROW_FFT_INV || MODE == ROW_FFT_FWD) {
            fft_line<K, MODE == ROW_FFT_INV, C>(v, t, tw, lds);
        } else if constexpr (MODE == ROW_PHASE_FWD || MODE == ROW_GD_INIT_FIELD) {
            fft_line<K, false, C>(v, t, tw, lds);
        } else if constexpr (MODE == ROW_GS_MAIN) {
            // A -> B = a_in A/|A| (src/algorithms.py:30)
            auto epi = [&](int l, int m, C& z) { z = unit_scale(z, ain_at(l, m)); };
            if constexpr (SHUF)
                shuffle_pair<true, false>(v[0], threadIdx.x, stw, reinterpret_cast<float2*>(smem), epi);
            else
                fft_pair<K, true, false, C>(v, t, tw, lds, epi);
        } else if constexpr (MODE == ROW_GD_INIT_Y) {
            fft_pair<K, true, false, C>(v, t, tw, lds, [&](int l, int m, C& z) {
                const S a = ain_at(l, m);
                const C x = unit_scale(z, a);  // a_in exp(i angle(ifft2(sqrt T)))
                p.field[boff + PY * l + m * bstep] = to_c64(x);
                z = normalize(x, a);
            });
        } else if constexpr (MODE == ROW_GD_MAIN) {
            // dEdF = ifft2(...) * a_in (src/algorithms.py:87-89); dEdX_complex (:179-185);
            // input -= lr * dEdX (:91); next forward input x/|x| a_in (:84).
            const S lr = (S)p.lr[p.iter];
            const S inv_s = (S)1 / (S)p.holo;
            auto epi = [&](int l, int m, C& z) {
                const S a = ain_at(l, m);
                const C g = mk<C>(z.x * inv_s * a, z.y * inv_s * a);
                const long long idx = boff + PY * l + m * bstep;
                // loaded here: fetching the field with the tile's inputs measured slower
                // (GD 1024^2 row pass 10.40 -> 10.89 us, same box, gpurun_out/s11)
                C x = from_c64<C>(p.field_src[idx]);
                const S ax2 = x.x * x.x + x.y * x.y;
                const S inv = rsqrt_nr(ax2);
                const S inv3 = inv * inv * inv;
                const S re = x.x * g.x + x.y * g.y;
                const S dx = g.x * inv - x.x * re * inv3;
                const S dy = g.y * inv - x.y * re * inv3;
                x.x -= lr * dx;
                x.y -= lr * dy;
                const float2 xs = to_c64(x);  // the field is stored in complex64
                p.field[idx] = xs;
                z = normalize(from_c64<C>(xs), a);
            };
            if constexpr (SHUF)
                shuffle_pair<true, false>(v[0], threadIdx.x, stw, reinterpret_cast<float2*>(smem), epi);
            else
                fft_pair<K, true, false, C>(v, t, tw, lds, epi);
        } else if constexpr (MODE == ROW_GD_LIN) {
            // The column pass left U = ifft_col(mask F P) and V = ifft_col(mask F T);
            // ifft_col(mask F (s P - T)) = s U - V with s = norm / max |F|^2 of this
            // iteration (src/algorithms.py:85-88), reduced here from the column
            // workgroups' maxima -- no grid-wide barrier inside a launch.
            V q[L][E];
            float2 xf[L][E];
#pragma unroll
            for (int l = 0; l < L; ++l)
#pragma unroll
                for (int m = 0; m < E; ++m) {
                    q[l][m] = cv<V>(p.in2[boff + PY * l + m * bstep]);
                    xf[l][m] = p.field_src[boff + PY * l + m * bstep];  // fetched with the inputs, used after the inverse
                }
            __shared__ double smax;
            {
                const double* gm = p.gmax + ((long long)b * p.max_loops + p.iter) * p.nwg_col;
                double mx = 0.0;
                for (int k = threadIdx.x; k < p.nwg_col; k += RowCfg<K, P>::THREADS) mx = fmax(mx, gm[k]);
                block_reduce_max<RowCfg<K, P>::THREADS>(mx);
                if (threadIdx.x == 0) smax = mx;
                lds_barrier();
            }
            const S s = (S)p.norm[b] / (S)smax;
#pragma unroll
            for (int l = 0; l < L; ++l)
#pragma unroll
                for (int m = 0; m < E; ++m) {
                    const C u = cv<C>(v[l][m]), w = cv<C>(q[l][m]);
                    v[l][m] = cv<V>(mk<C>(s * u.x - w.x, s * u.y - w.y));
                }
            const S lr = (S)p.lr[p.iter];
            const S inv_s = (S)1 / (S)p.holo;
            auto epi = [&](int l, int m, C& z) {
                // dEdF = ifft2(...) * a_in (:87-89); dEdX_complex (:179-185); x -= lr dEdX (:91)
                const S a = ain_at(l, m);
                const C g = mk<C>(z.x * inv_s * a, z.y * inv_s * a);
                C x = from_c64<C>(xf[l][m]);
                const S ax2 = x.x * x.x + x.y * x.y;
                const S inv = rsqrt_nr(ax2);
                const S inv3 = inv * inv * inv;
                const S re = x.x * g.x + x.y * g.y;
                const S dx = g.x * inv - x.x * re * inv3;
                const S dy = g.y * inv - x.y * re * inv3;
                x.x -= lr * dx;
                x.y -= lr * dy;
                const float2 xs = to_c64(x);
                p.field[boff + PY * l + m * bstep] = xs;
                z = normalize(from_c64<C>(xs), a);
            };
            if constexpr (SHUF)
                shuffle_pair<true, false>(v[0], threadIdx.x, stw, reinterpret_cast<float2*>(smem), epi);
            else
                fft_pair<K, true, false, C>(v, t, tw, lds, epi);
        }
        trace_point(trace, tile, 2, false);
        // slot-major: the L rows of a thread are adjacent in a panel, so their pieces
        // of one 128-B line leave back to back (tools/row_store_probe.hip, a copy of
        // 8 x 4096^2 in the row pass's shapes: 32-B row pieces 711 us, adjacent row
        // pairs 531 us, whole lines 445 us)
        if constexpr (kSector) {
            // whole 64-B sectors per instruction (the loads' exchange, reversed)
            const bool b2 = (t >> 2) & 1;
            const long long o1 = b2 ? PX - 4LL * p.H : 0, o2 = b2 ? PX : 4LL * p.H;
            auto sectors = [&](auto wtc) {
#pragma unroll
                for (int m = 0; m < E; ++m) {
                    const float2 a = cv<float2>(v[0][m]), c = cv<float2>(v[1][m]);
                    const float2 r = lane_xor4(b2 ? a : c, b2);
                    store_field(p.out + xoff + o1 + m * bstep, b2 ? r : a, decltype(wtc)::value);
                    store_field(p.out + xoff + o2 + m * bstep, b2 ? c : r, decltype(wtc)::value);
                }
            };
            if (p.wt)  // uniform: one branch per tile, not per store
                sectors(std::integral_constant<int, 1>{});
            else
                sectors(std::integral_constant<int, 0>{});
        } else if (p.wt) {  // uniform: one branch per tile, not per store
#pragma unroll
            for (int m = 0; m < E; ++m)
#pragma unroll
                for (int l = 0; l < L; ++l) store_field(p.out + xoff + PX * l + m * bstep, cv<float2>(v[l][m]), 1);
        } else {
#pragma unroll
            for (int m = 0; m < E; ++m)
#pragma unroll
                for (int l = 0; l < L; ++l) p.out[xoff + PX * l + m * bstep] = cv<float2>(v[l][m]);
        }
        trace_point(trace, tile, 3, true);
    };
    V v[L][E];
    float none[1];
    tile_loop(p.ntile * (long long)p.B, load, process, v, none);
}

// ------------------------------------------------------------------------
// column pass
// ------------------------------------------------------------------------
// The two terms of the split GD gradient (src/algorithms.py:80,85-88):
// mask F |F|^2 and mask F T, mask = 1 + wa T / 255, from F in the slots.
template <class C, class V, class TV, int L, int E>
__device__ __forceinline__ void gd_split_terms(const V (&v)[L][E], const TV (&tv)[L][E], Scalar<C> wa, V (&wu)[L][E],
                                               V (&wv)[L][E]) {
    using S = Scalar<C>;
#pragma unroll
    for (int l = 0; l < L; ++l)
#pragma unroll
        for (int m = 0; m < E; ++m) {
            const C z = cv<C>(v[l][m]);
            const float tl = tv[l][m];
            const S e = z.x * z.x + z.y * z.y;
            const S mask = (S)1 + wa * (S)tl / (S)255;
            const S a = mask * e, q = mask * (S)tl;
            wu[l][m] = cv<V>(mk<C>(z.x * a, z.y * a));
            wv[l][m] = cv<V>(mk<C>(z.x * q, z.y * q));
        }
}

// Inverse column transforms of both terms: as 2 L lines through one exchange
// region of 2 CW columns (DUAL: shared twiddles and barriers), else one after
// the other through the kernel's own region.
template <int K, class C, bool DUAL, class V, int L, int E, class Tw, class Lds, class X>
__device__ __forceinline__ void gd_inverse_pair(V (&wu)[L][E], V (&wv)[L][E], int t, const Tw& tw, const Lds& lds,
                                                X* smem, int c) {
    if constexpr (DUAL) {
        V w2[2 * L][E];
#pragma unroll
        for (int l = 0; l < L; ++l)
#pragma unroll
            for (int m = 0; m < E; ++m) {
                w2[l][m] = wu[l][m];
                w2[L + l][m] = wv[l][m];
            }
        // the same buffer alternation continues (kDouble exchanges); a wave-local
        // region hands over to the wider, workgroup-synchronised one at a barrier
        if constexpr (Lds::kWave) lds_barrier();
        const LdsTile<2 * Lds::kCW, X, Lds::kAlt> lds2{smem, 2 * c, lds.cur};
        fft_line<K, true, C>(w2, t, tw, lds2);
#pragma unroll
        for (int l = 0; l < L; ++l)
#pragma unroll
            for (int m = 0; m < E; ++m) {
                wu[l][m] = w2[l][m];
                wv[l][m] = w2[L + l][m];
            }
    } else {
        fft_line<K, true, C>(wu, t, tw, lds);
        fft_line<K, true, C>(wv, t, tw, lds);
    }
}

// COL_GD_LIN runs its two inverse column transforms (mask F P and mask F T)
// as two lines per column of the thread, sharing twiddles and
// exchange barriers, where the doubled exchange region still leaves two
// workgroups per CU; else one after the other through the same region.
// Column tiles whose threads carry every column of the tile (CW == L: the
// 4096 narrow plan, two columns per thread) exchange through line-major
// swizzled regions instead of the [o][c] interleave: an instruction then
// touches one line only, and the interleave's stride-2 slots cost 4 / 2 extra
// cycles per write / read (tools/lds_banks.py).
template <int K, int CW>
constexpr bool kColLineMajor = ColCfg<K, CW>::L == CW;

template <int K, int CW, int P, int MODE>
constexpr bool kColDualInv() {
    using X = XchgOf<P, (long long)PlanOf<K>::LINE * CW, K>;
    return MODE == COL_GD_LIN && !kColLineMajor<K, CW> &&
           (kLdsDouble<K, true> ? 2 : 1) * (long long)PlanOf<K>::LINE * 2 * CW * sizeof(X) <= kLdsPair;
}
template <int K, int CW, int P, int MODE>
constexpr int col_lds_width() {
    return kColDualInv<K, CW, P, MODE>() ? 2 * CW : CW;
}

template <int K, int CW, int MODE, int TT, int P, int LID>
__global__ void __launch_bounds__((ColCfg<K, CW>::THREADS), 1) col_kernel(ColParams p) {
    constexpr int LAYOUT_X = LayoutOf<LID>::X, LAYOUT_Y = LayoutOf<LID>::Y;
    using C = CplxOf<P>;
    using S = Scalar<C>;
    constexpr int H = PlanOf<K>::N;
    constexpr int E = PlanOf<K>::E;
    constexpr int T = PlanOf<K>::T;
    constexpr int L = ColCfg<K, CW>::L;
    constexpr int LINE = PlanOf<K>::LINE;
    constexpr int THREADS = ColCfg<K, CW>::THREADS;
    using X = XchgOf<P, (long long)LINE * CW, K>;
    using V = StateOf<P, X>;
    constexpr int LW = col_lds_width<K, CW, P, MODE>();  // exchange columns (2 CW: COL_GD_LIN's paired inverses)
    constexpr int ALT = kLdsDouble<K, true> ? LINE * LW : 0;
    constexpr bool WV = ColCfg<K, CW>::kWave;
    constexpr int RS = PlanOf<K>::ROWSTRIDE;  // line-major regions (one-group tiles)
    constexpr int SMEM = (ALT ? 2 : 1) * LINE * LW > CW * RS ? (ALT ? 2 : 1) * LINE * LW : CW * RS;
    __shared__ X smem[SMEM];

    // a thread carries columns c .. c + L - 1 of the tile (adjacent in the
    // blocked layout: one 16-B access for L = 2)
    // wave-shuffle pair: lane bit 0 selects the column (as here), t per fft_shuffle.hpp
    // (the GS and GD iteration modes)
    constexpr bool SHUF = kShuffle<K, P> && CW == 2 && L == 1 &&
                          (MODE == COL_GS_MAIN || (P == PREC_F32 && (MODE == COL_GD_STATS || MODE == COL_GD_GRAD ||
                                                                      MODE == COL_GD_FUSED || MODE == COL_GD_LIN)));
    const int c = (threadIdx.x % (CW / L)) * L;
    const int t = SHUF ? shuffle_t(threadIdx.x) : threadIdx.x / (CW / L);
    // inputs (X, target) in layout X, outputs (Y) in layout Y: row y = t + T m
    constexpr long long kStep = (long long)kPanelOf<LAYOUT_X> * T;
    constexpr long long kStepY = (long long)kPanelOf<LAYOUT_Y> * T;
    using LdsT = std::conditional_t<kColLineMajor<K, CW>, LdsLine<X, WV ? 0 : ALT, WV>,
                                    LdsTile<CW, X, WV ? 0 : ALT, WV>>;
    const LdsT lds = [&] {
        if constexpr (kColLineMajor<K, CW>)
            return LdsT{smem, RS};  // c == 0: the thread's lines are its columns
        else
            return LdsT{smem, c};
    }();
    if constexpr (MODE == COL_GS_MAIN || MODE == COL_GD_GRAD || MODE == COL_GD_FUSED || MODE == COL_GD_LIN)
        trace_entry(p.trace);
    sgpr_pin(p.in, p.out, p.tgt, p.holo, p.nwg, p.B, p.tw, p.checked, p.wt, gridDim.x);
    Twiddles<K, C, tw_mode<P, THREADS, K, true, L>()> tw;
    static_assert(!SHUF || (std::is_same_v<X, float2> && sizeof(smem) >= 4 * kShufN * sizeof(float2)),
                  "the shuffle pair needs two 2-line complex64 exchange buffers");
    ShuffleTwT<C> stw;
    if constexpr (SHUF)
        load_shuffle_tw(stw, threadIdx.x, static_cast<const C*>(p.tw) + twiddle_count_key(K));
    else
        load_twiddles<K, C>(tw, t, p.tw);
    constexpr bool kTarget = (MODE == COL_GS_MAIN || MODE == COL_GD_STATS || MODE == COL_GD_GRAD ||
                              MODE == COL_GD_FUSED || MODE == COL_GD_LIN);
    constexpr int NT = kTarget ? E : 1;

    // field / target element (row t + T m, column c + l) of a tile at base
    auto ld_field = [&](const float2* src, long long idx, V (&v)[L][E], int m) {
        if constexpr (L == 2) {
            const float4 q = *reinterpret_cast<const float4*>(src + idx);
            v[0][m] = cv<V>(make_float2(q.x, q.y));
            v[1][m] = cv<V>(make_float2(q.z, q.w));
        } else {
            v[0][m] = cv<V>(src[idx]);
        }
    };
    auto ld_tgt = [&](long long idx, float (&tv)[L][NT], int m) {
        if constexpr (L == 2 && (TT == TGT_F32 || TT == TGT_AMP)) {
            const float2 q = *reinterpret_cast<const float2*>(static_cast<const float*>(p.tgt) + idx);
            tv[0][m] = q.x;
            tv[1][m] = q.y;
        } else {
#pragma unroll
            for (int l = 0; l < L; ++l) tv[l][m] = TgtLoad<TT>::load(p.tgt, idx + l);
        }
    };
    // stores of a whole tile (layout Y); `wt` is uniform, so it branches once per tile
    auto st_tile_to = [&](float2* dst, long long base, const V (&v)[L][E]) {
        if (p.wt) {
#pragma unroll
            for (int m = 0; m < E; ++m)
#pragma unroll
                for (int l = 0; l < L; ++l) store_field(dst + base + m * kStepY + l, cv<float2>(v[l][m]), 1);
        } else {
#pragma unroll
            for (int m = 0; m < E; ++m) {
                if constexpr (L == 2) {
                    const float2 a = cv<float2>(v[0][m]), b = cv<float2>(v[1][m]);
                    *reinterpret_cast<float4*>(dst + base + m * kStepY) = make_float4(a.x, a.y, b.x, b.y);
                } else {
                    dst[base + m * kStepY] = cv<float2>(v[0][m]);
                }
            }
        }
    };
    auto st_tile = [&](long long base, const V (&v)[L][E]) { st_tile_to(p.out, base, v); };

    // tile = (hologram b, column group wg); element (y, x) at blk_index<layout>(y, x, H)
    auto where = [&](long long tile, int& b, int& wg, long long& base) {
        b = (int)(tile / p.nwg);
        wg = (int)(tile - (long long)b * p.nwg);
        base = (long long)b * p.holo + blk_index<LAYOUT_X>(t, wg * CW + c, H);
    };
    auto out_base = [&](int b, int wg) {
        return (long long)b * p.holo + blk_index<LAYOUT_Y>(t, wg * CW + c, H);
    };
    auto load = [&](long long tile, V (&v)[L][E], float (&tv)[L][NT]) {
        int b, wg;
        long long base;
        where(tile, b, wg, base);
        if constexpr (MODE == COL_REAL_INV) {
#pragma unroll
            for (int l = 0; l < L; ++l)
#pragma unroll
                for (int m = 0; m < E; ++m) {
                    const float a = TgtLoad<TT>::amp(TgtLoad<TT>::load(p.tgt, base + l + m * kStep));
                    v[l][m] = cv<V>(mk<C>((S)a, (S)0));
                }
        } else if constexpr (MODE == COL_EXPECTED) {
            // GD keeps X of iteration i in buffer i % 2; GS passes the same buffer twice.
            const int s = p.checked ? min(p.stop_iter[b], p.loops - 1) : p.loops - 1;
            const float2* src = (s & 1) ? p.in_alt : p.in;
#pragma unroll
            for (int m = 0; m < E; ++m) ld_field(src, base + m * kStep, v, m);
        } else {
#pragma unroll
            for (int m = 0; m < E; ++m) ld_field(p.in, base + m * kStep, v, m);
        }
        if constexpr (kTarget) {
            // the target is consumed in the middle of the transforms: fetch it with the field
#pragma unroll
            for (int m = 0; m < E; ++m) ld_tgt(base + m * kStep, tv, m);
        }
    };
    auto process = [&](long long tile, V (&v)[L][E], float (&tv)[L][NT]) {
        int b, wg;
        long long base;
        where(tile, b, wg, base);
        unsigned long long* const trace =
            (MODE == COL_GS_MAIN || MODE == COL_GD_GRAD || MODE == COL_GD_FUSED || MODE == COL_GD_LIN) ? p.trace
                                                                                                       : nullptr;
        trace_point(trace, tile, 0, false);
        if constexpr (kTarget) {
            if (p.checked && p.iter > p.stop_iter[b]) return;
        }
        // GD gradient needs this iteration's global max of |F|^2 (src/algorithms.py:86).
        S maxp = 0;
        if constexpr (MODE == COL_GD_GRAD) {
            __shared__ double smax;
            const double* part = p.partials + ((long long)b * p.max_loops + p.iter) * p.nwg * 4;
            double m = 0.0;
            for (int k = threadIdx.x; k < p.nwg; k += THREADS) m = fmax(m, part[k * 4]);
            block_reduce_max<THREADS>(m);
            if (threadIdx.x == 0) smax = m;
            lds_barrier();
            maxp = (S)smax;
        }
        trace_point(trace, tile, 1, true);
        if constexpr (MODE == COL_REAL_INV || MODE == COL_FFT_INV || MODE == COL_FFT_FWD) {
            fft_line<K, MODE != COL_FFT_FWD, C>(v, t, tw, lds);
            st_tile(out_base(b, wg), v);
            return;
        } else if constexpr (MODE == COL_EXPECTED) {
            // |C|^2 in layout Y (a column tile's stores are whole panel runs, like the
            // field's); the host relayouts it to the row-major e_out afterwards --
            // row-major stores from a column tile were one 4-B segment per lane
            const long long ob = out_base(b, wg);
            fft_line_epi<K, false, C>(v, t, tw, lds, [&](int l, int m, C& z) {
                p.e_blk[ob + m * kStepY + l] = (float)(z.x * z.x + z.y * z.y);
            });
            return;
        } else if constexpr (MODE == COL_GD_LIN) {
            // GD column side with no global max inside the launch (src/algorithms.py:84-88):
            // G = mask F (s |F|^2 - T) = s (mask F |F|^2) - (mask F T), s = norm / max |F|^2.
            // Both terms are inverse-transformed along the columns here (Y, Y2); the row
            // pass forms s U - V once every column workgroup's max is in memory.
            double mx = 0.0, s2 = 0.0, st = 0.0;
            auto stats = [&](int l, int m, C& z) {
                const double ed = (double)(float)(z.x * z.x + z.y * z.y);
                mx = fmax(mx, ed);
                s2 += ed * ed;
                st += ed * (double)tv[l][m];
            };
            if constexpr (SHUF) {
                shuffle_first<false>(v[0], threadIdx.x, stw, reinterpret_cast<float2*>(smem));
                static_for<E>([&](auto mc) { stats(0, decltype(mc)::value, v[0][decltype(mc)::value]); });
            } else {
                fft_line_epi<K, false, C>(v, t, tw, lds, stats);
            }
            trace_point(trace, tile, 2, false);
            V wu[L][E], wv[L][E];
            gd_split_terms<C>(v, tv, (S)p.wa, wu, wv);
            if constexpr (SHUF) {
                // U then V: V's exchange reuses the first transform's buffer, which
                // every wave left before U's barrier
                float2* const buf = reinterpret_cast<float2*>(smem);
                shuffle_second<true>(wu[0], threadIdx.x, stw, buf + 2 * kShufN);
                shuffle_second<true>(wv[0], threadIdx.x, stw, buf);
            } else {
                gd_inverse_pair<K, C, LW == 2 * CW>(wu, wv, t, tw, lds, smem, c);
            }
            const long long ob = out_base(b, wg);
            st_tile_to(p.out, ob, wu);
            st_tile_to(p.out2, ob, wv);
            block_reduce_stats<THREADS>(mx, s2, st);
            if (threadIdx.x == 0) {
                const long long it = (long long)b * p.max_loops + p.iter;
                double* dst = p.partials + (it * p.nwg + wg) * 4;
                dst[0] = mx;
                dst[1] = s2;
                dst[2] = st;
                dst[3] = 0.0;
                p.gmax[it * p.nwg + wg] = mx;
            }
            trace_point(trace, tile, 3, true);
            return;
        } else if constexpr (MODE == COL_GD_FUSED) {
            // GD column side in one launch (src/algorithms.py:84-88): F = fft(X)
            // and its statistics, a grid barrier for the hologram's global max
            // of |F|^2, then G = mask F (s|F|^2 - T) and ifft -- F stays in
            // registers across the barrier instead of being recomputed by a
            // second launch (COL_GD_STATS + COL_GD_GRAD).
            double mx = 0.0, s2 = 0.0, st = 0.0;
            auto stats = [&](int l, int m, C& z) {
                const double ed = (double)(float)(z.x * z.x + z.y * z.y);
                mx = fmax(mx, ed);
                s2 += ed * ed;
                st += ed * (double)tv[l][m];
            };
            if constexpr (SHUF) {
                shuffle_first<false>(v[0], threadIdx.x, stw, reinterpret_cast<float2*>(smem));
                static_for<E>([&](auto mc) { stats(0, decltype(mc)::value, v[0][decltype(mc)::value]); });
            } else {
                fft_line_epi<K, false, C>(v, t, tw, lds, stats);
            }
            trace_point(trace, tile, 2, false);
            block_reduce_stats<THREADS>(mx, s2, st);
            if (threadIdx.x == 0) {  // the statistics partials (folded after the run by stats_reduce_kernel)
                double* dst = p.partials + (((long long)b * p.max_loops + p.iter) * p.nwg + wg) * 4;
                dst[0] = mx;
                dst[1] = s2;
                dst[2] = st;
                dst[3] = 0.0;
            }
            const long long it = (long long)b * p.max_loops + p.iter;
            const double smax = grid_max_barrier<THREADS>(p.gslots + it * p.nwg, p.gresult + it, mx, wg, p.nwg,
                                                          p.fault, p.skip_wg_plus1);
            const S maxp = (S)smax;
            const S norm = (S)p.norm[b];
            trace_point(trace, tile, 3, true);
#pragma unroll
            for (int l = 0; l < L; ++l)
#pragma unroll
                for (int mm = 0; mm < E; ++mm) {
                    const C z = cv<C>(v[l][mm]);
                    const float tl = tv[l][mm];
                    const S e = z.x * z.x + z.y * z.y;
                    const S o = e * norm / maxp;
                    const S w = ((S)1 + (S)p.wa * (S)tl / (S)255) * (o - (S)tl);
                    v[l][mm] = cv<V>(mk<C>(z.x * w, z.y * w));
                }
            if constexpr (SHUF)
                shuffle_second<true>(v[0], threadIdx.x, stw, reinterpret_cast<float2*>(smem) + 2 * kShufN);
            else
                fft_line<K, true, C>(v, t, tw, lds);
            st_tile(out_base(b, wg), v);
            return;
        } else {
            double mx = 0.0, s2 = 0.0, st = 0.0;
            const S norm = (MODE == COL_GD_GRAD) ? (S)p.norm[b] : (S)0;
            // GS: the launch of the run's last iteration (every iteration of a
            // checked run) also stores E = |C|^2, the expected output of
            // src/algorithms.py:36, in layout Y (e_blk; relayouted to row-major
            // after the run) -- no separate forward transform for it
            float* const e_blk = MODE == COL_GS_MAIN ? p.e_blk : nullptr;
            const long long eb = MODE == COL_GS_MAIN ? out_base(b, wg) : 0;
            // GS: the thread's partial sums in float32 (its E elements of one
            // column), folded across the workgroup in float64: a few 1e-7 of a
            // partial, averaging out over the hologram's partials (the error's
            // expansion cancels by ~1e2 late in a run: error curves still
            // agree to ~1e-6 relative, gated at 1e-4)
            // E^2 is summed scaled by stat_k (a power of two ~ 1/holo^2: the same
            // bits, and no float32 overflow for a bright incoming amplitude whose
            // energy sits in a few pixels -- E reaches (holo a_in)^2)
            float mxf = 0.f, s2f = 0.f, stf = 0.f;
            const float stat_k = MODE == COL_GS_MAIN ? p.stat_k : 1.f;
            auto epi = [&](int l, int m, C& z) {
                const S e = z.x * z.x + z.y * z.y;
                const float tl = tv[l][m];
                if constexpr (MODE == COL_GS_MAIN) {
                    const float ef = (float)e;  // |C|^2 as the reference's float64 expected_outcome sees it
                    mxf = fmaxf(mxf, ef);
                    s2f = fmaf(ef * stat_k, ef, s2f);
                    stf = fmaf(ef, TgtLoad<TT>::intensity(tl), stf);
                } else if constexpr (MODE == COL_GD_STATS) {
                    const double ed = (double)(float)e;
                    mx = fmax(mx, ed);
                    s2 += ed * ed;
                    st += ed * (double)tl;
                }
                if constexpr (MODE == COL_GS_MAIN) {
                    if (e_blk) e_blk[eb + m * kStepY + l] = (float)e;
                    z = unit_scale(z, (S)TgtLoad<TT>::amp(tl));  // D = a_T C/|C| (src/algorithms.py:33)
                } else if constexpr (MODE == COL_GD_GRAD) {
                    // mask * F * (output - T), output = |F|^2 norm / max (src/algorithms.py:80,85-88)
                    const S o = e * norm / maxp;
                    const S w = ((S)1 + (S)p.wa * (S)tl / (S)255) * (o - (S)tl);
                    z = mk<C>(z.x * w, z.y * w);
                }
            };
            // GD recomputes F in the gradient pass: storing F from the statistics
            // pass and reading it back measured slower at 1024^2 (8.9 + 9.5 us
            // against 5.7 + 10.9 us per iteration: the extra store tail costs
            // more than the forward transform saves)
            if constexpr (MODE == COL_GD_STATS && SHUF) {
                shuffle_first<false>(v[0], threadIdx.x, stw, reinterpret_cast<float2*>(smem));
                static_for<E>([&](auto mc) { epi(0, decltype(mc)::value, v[0][decltype(mc)::value]); });
            } else if constexpr (MODE == COL_GD_STATS)
                fft_line_epi<K, false, C>(v, t, tw, lds, epi);
            else if constexpr (SHUF)
                shuffle_pair<false, true>(v[0], threadIdx.x, stw, reinterpret_cast<float2*>(smem), epi);
            else
                fft_pair<K, false, true, C>(v, t, tw, lds, epi);
            trace_point(trace, tile, 2, false);
            if constexpr (MODE == COL_GS_MAIN || MODE == COL_GD_GRAD) st_tile(out_base(b, wg), v);
            // the cross-lane statistics reduction (LDS only) runs while the field stores drain
            if constexpr (MODE == COL_GS_MAIN) {
                mx = mxf;
                s2 = (double)s2f / (double)stat_k;  // exact: a power of two
                st = stf;
            }
            if constexpr (MODE == COL_GS_MAIN || MODE == COL_GD_STATS) {
                block_reduce_stats<THREADS>(mx, s2, st);
                if (threadIdx.x == 0) {
                    double* dst = p.partials + (((long long)b * p.max_loops + p.iter) * p.nwg + wg) * 4;
                    dst[0] = mx;
                    dst[1] = s2;
                    dst[2] = st;
                    dst[3] = 0.0;
                }
            }
            trace_point(trace, tile, 3, true);
        }
    };
    V v[L][E];
    float tv[L][NT];
    tile_loop(p.nwg * (long long)p.B, load, process, v, tv);
}

// ------------------------------------------------------------------------
// small kernels (size independent)
// ------------------------------------------------------------------------
struct StatsParams {
    const double* partials;  // [B][max_loops][nwg][4]
    double* stats;           // [B][max_loops][4]: max, sum E^2, sum E T, err
    int* stop_iter;          // [B]
    const double* norm;      // [B] max(T)
    const double* sum_t2;    // [B] sum T^2
    double inv_s;            // 1 / S
    double tol;
    int max_loops;
    int nwg;
    int iter;                // finalize: iteration to check; reduce: unused
};

// Deterministic reduction of one (hologram, iteration) slab; 256 threads.
__device__ __forceinline__ void reduce_slab(const StatsParams& p, int b, int i, double* out4) {
    const double* part = p.partials + ((long long)b * p.max_loops + i) * p.nwg * 4;
    double mx = 0.0, s2 = 0.0, st = 0.0;
    for (int k = threadIdx.x; k < p.nwg; k += 256) {
        mx = fmax(mx, part[k * 4 + 0]);
        s2 += part[k * 4 + 1];
        st += part[k * 4 + 2];
    }
    block_reduce_stats<256>(mx, s2, st);
    if (threadIdx.x == 0) {
        // error_f (src/algorithms.py:161-162) of E * norm / max(E) against T,
        // expanded so that E never has to be stored: (s^2 SE2 - 2 s SET + ST2) / S.
        const double s = __ddiv_rn(p.norm[b], mx);
        double a = __dmul_rn(__dmul_rn(s, s), s2);
        double c = __dmul_rn(__dmul_rn(2.0, s), st);
        const double err = __dmul_rn(__dadd_rn(__dsub_rn(a, c), p.sum_t2[b]), p.inv_s);
        out4[0] = mx;
        out4[1] = s2;
        out4[2] = st;
        out4[3] = err;
    }
}


}  // namespace slm
