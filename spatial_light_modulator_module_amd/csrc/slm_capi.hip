// libslm_hip.so host runtime: plans (device-resident batches), launch
// sequencing of the fused GS / GD iterations, HIP-event timing, and the
// RCCL gather of phases for one-process-per-GPU runs. C-ABI in
// include/slm_hip.h.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <climits>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <tuple>
#include <vector>

#include "../../include/slm_hip.h"
#include "dispatch.hpp"
#include "generic.hpp"
#include "layout_kernels.hpp"
#include "kernels.hpp"

using namespace slm;

namespace {

thread_local std::string g_err;
int g_device = -1;
std::mutex g_mu;
std::map<std::tuple<int, int, int>, void*> g_twiddles;  // (device, plan key, precision) -> table
ncclComm_t g_comm = nullptr;
int g_comm_rank = 0, g_comm_size = 1;

int fail(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

#define HIP_TRY(expr)                                                                              \
    do {                                                                                           \
        hipError_t e_ = (expr);                                                                    \
        if (e_ != hipSuccess)                                                                      \
            return fail(SLM_ERR_HIP, "%s failed: %s (%s:%d)", #expr, hipGetErrorString(e_), __FILE__, \
                        __LINE__);                                                                 \
    } while (0)

#define NCCL_TRY(expr)                                                                                       \
    do {                                                                                                     \
        ncclResult_t r_ = (expr);                                                                            \
        if (r_ != ncclSuccess) return fail(SLM_ERR_COMM, "%s failed: %s", #expr, ncclGetErrorString(r_)); \
    } while (0)

#define RC(x)                 \
    do {                      \
        int rc_ = (x);        \
        if (rc_) return rc_;  \
    } while (0)

// Blocking copies go through an explicit stream, never the legacy null stream:
// slm_gs_multi runs plans from several host threads, and a legacy-stream copy
// in one thread while another thread captures its plan's graph is an error.
int copy_sync(void* dst, const void* src, size_t bytes, hipMemcpyKind kind, hipStream_t st) {
    if (!bytes) return 0;
    HIP_TRY(hipMemcpyAsync(dst, src, bytes, kind, st));
    HIP_TRY(hipStreamSynchronize(st));
    return 0;
}

int ensure_device() {
    if (g_device >= 0) {
        HIP_TRY(hipSetDevice(g_device));
        return 0;
    }
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess || n <= 0)
        return fail(SLM_ERR_HIP, "no HIP device available (%s); libslm_hip has no CPU path",
                    hipGetErrorString(e));
    g_device = 0;
    HIP_TRY(hipSetDevice(0));
    return 0;
}

// Twiddle table of one radix plan, in its pass order: entry
// [(r - 1) * Ns + j] = exp(-2 pi i j r / (Ns R)), computed in double and
// stored as float2 (PREC_F32) or double2 (PREC_F64).
int get_twiddles(int pk, int prec, const void** out) {
    int dev = 0;
    HIP_TRY(hipGetDevice(&dev));  // tables live on the calling thread's current device
    std::lock_guard<std::mutex> lk(g_mu);
    auto key = std::make_tuple(dev, pk, prec);
    auto it = g_twiddles.find(key);
    if (it != g_twiddles.end()) {
        *out = it->second;
        return 0;
    }
    if (pk < 0 || pk >= kNumPlans) return fail(SLM_ERR_UNSUPPORTED, "unknown plan key %d", pk);
    const RadixPlan& pl = kPlans[pk];
    std::vector<double> host;  // interleaved re, im
    int ns = 1;
    for (int k = 0; k < pl.npass; ++k) {
        const int r_ = pl.r[k];
        if (ns > 1) {
            const long long L = (long long)ns * r_;
            for (int r = 1; r < r_; ++r)
                for (int j = 0; j < ns; ++j) {
                    const long long q = ((long long)j * r) % L;
                    const double ang = -2.0 * M_PI * (double)q / (double)L;
                    host.push_back(std::cos(ang));
                    host.push_back(std::sin(ang));
                }
        }
        ns *= r_;
    }
    if (host.empty()) {
        host.push_back(1.0);
        host.push_back(0.0);
    }
    if (pl.n == kShufN && pl.e == 8) {
        // the wave-shuffle pair's table (fft_shuffle.hpp): the N roots
        // exp(-2 pi i e / N), after the Stockham entries (twiddle_count_key)
        for (int e = 0; e < pl.n; ++e) {
            const double ang = -2.0 * M_PI * (double)e / (double)pl.n;
            host.push_back(std::cos(ang));
            host.push_back(std::sin(ang));
        }
    }
    void* d = nullptr;
    if (prec == PREC_F64) {
        HIP_TRY(hipMalloc(&d, host.size() * sizeof(double)));
        RC(copy_sync(d, host.data(), host.size() * sizeof(double), hipMemcpyHostToDevice, hipStreamPerThread));
    } else {
        std::vector<float> f(host.begin(), host.end());
        HIP_TRY(hipMalloc(&d, f.size() * sizeof(float)));
        RC(copy_sync(d, f.data(), f.size() * sizeof(float), hipMemcpyHostToDevice, hipStreamPerThread));
    }
    g_twiddles[key] = d;
    *out = d;
    return 0;
}

// Holds a stream for `ticks` of the 100 MHz s_memrealtime clock (one wave,
// bounded by time alone). slm_plan_run_timed queues it first so the host
// enqueues every launch of the timed run while it waits: the timed kernels then
// run back to back, as in the replayed graph of slm_plan_run, instead of each
// starting on an idle device behind the host's per-launch enqueue cost (which
// measured up to 0.5 us shorter per 1024^2 launch than the same kernel in the
// graph, profiles/r04).
__global__ void __launch_bounds__(64) hold_kernel(unsigned long long ticks) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(127);
}

__global__ void fill_int_kernel(int* p, int n, int v) {
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) p[i] = v;
}

// Streaming copy, 16 B per lane, four non-temporal loads in flight per lane
// before their stores, grid-stride (slm_copy_bandwidth): the practical HBM /
// Infinity-Cache rate the roofline fractions are read against.
typedef float v4f __attribute__((ext_vector_type(4)));
__global__ void __launch_bounds__(256) copy_f4_kernel(const v4f* __restrict__ in, v4f* __restrict__ out,
                                                      long long n) {
    const long long stride = (long long)gridDim.x * 1024;
    for (long long base = blockIdx.x * 1024LL + threadIdx.x; base < n; base += stride) {
        v4f r[4];
#pragma unroll
        for (int k = 0; k < 4; ++k)
            if (base + k * 256 < n) r[k] = __builtin_nontemporal_load(in + base + k * 256);
#pragma unroll
        for (int k = 0; k < 4; ++k)
            if (base + k * 256 < n) __builtin_nontemporal_store(r[k], out + base + k * 256);
    }
}

// max(T) and sum(T^2) per hologram in double (np.amax(demanded_output),
// src/algorithms.py:23; sum(T^2) is the constant term of the error expansion).
// Stage 1: ts_blocks(holo) workgroups per hologram, each thread reducing
// kTsPerThread consecutive elements from 16-B vector loads (64 MB of a 4096^2
// float32 target stream at HBM rate: 4096 workgroups, not 64); stage 2 folds
// a hologram's partials in a fixed order (deterministic).
constexpr int kTsPerThread = 16;
constexpr int kTsThreads = 256;
inline int ts_blocks(long long holo) {
    return (int)std::max<long long>(1, holo / ((long long)kTsThreads * kTsPerThread));
}
template <typename TT>
__global__ void __launch_bounds__(kTsThreads) target_stats_partial_kernel(const TT* tgt, long long holo, double* part) {
    const int b = blockIdx.y;
    const int nblk = gridDim.x;
    const long long chunk = (holo + nblk - 1) / nblk;
    const long long lo = (long long)blockIdx.x * chunk, hi = min(holo, lo + chunk);
    const TT* p = tgt + (long long)b * holo;
    double mx = 0.0, s2 = 0.0, d = 0.0;
    constexpr int VEC = 16 / sizeof(TT);  // elements per 16-B load
    const long long vlo = lo / VEC, vhi = hi / VEC;  // holo and chunk are multiples of VEC for supported shapes
    if ((lo % VEC) == 0 && (hi % VEC) == 0) {
        for (long long i = vlo + threadIdx.x; i < vhi; i += kTsThreads) {
            const uint4 q = reinterpret_cast<const uint4*>(p)[i];
            const TT* e = reinterpret_cast<const TT*>(&q);
#pragma unroll
            for (int k = 0; k < VEC; ++k) {
                const double v = (double)e[k];
                mx = fmax(mx, v);
                s2 += v * v;
            }
        }
    } else {
        for (long long i = lo + threadIdx.x; i < hi; i += kTsThreads) {
            const double v = (double)p[i];
            mx = fmax(mx, v);
            s2 += v * v;
        }
    }
    block_reduce_stats<kTsThreads>(mx, s2, d);
    if (threadIdx.x == 0) {
        double* o = part + ((long long)b * nblk + blockIdx.x) * 2;
        o[0] = mx;
        o[1] = s2;
    }
}
__global__ void __launch_bounds__(kTsThreads) target_stats_final_kernel(const double* part, int nblk, double* norm,
                                                                        float* normf, double* sum_t2) {
    const int b = blockIdx.x;
    double mx = 0.0, s2 = 0.0, d = 0.0;
    for (int k = threadIdx.x; k < nblk; k += kTsThreads) {
        mx = fmax(mx, part[((long long)b * nblk + k) * 2]);
        s2 += part[((long long)b * nblk + k) * 2 + 1];
    }
    block_reduce_stats<kTsThreads>(mx, s2, d);
    if (threadIdx.x == 0) {
        norm[b] = mx;
        normf[b] = (float)mx;
        sum_t2[b] = s2;
    }
}

// plog: panel width log2 of the destination / source blocked layout
// (layout_x_log2(lid): X buffers, the target; layout_y_log2(lid): Y, the GD field)
// float / complex64 planes of 64-multiple sides move through LDS tiles
// (layout_kernels.hpp, tile_relayout_kernel), byte planes element-wise
template <int PLOG, typename V>
void relayout_launch(const V* in, V* out, long long n, int H, int W, bool to_blocked, hipStream_t st) {
    if constexpr (sizeof(V) == 4 || sizeof(V) == 8) {
        if (H % 64 == 0 && W % 64 == 0) {
            const dim3 grid(W / 64, H / 64, (unsigned)(n / ((long long)H * W)));
            if (to_blocked)
                hipLaunchKernelGGL((tile_relayout_kernel<V, PLOG, true>), grid, dim3(256), 0, st, in, out, H, W);
            else
                hipLaunchKernelGGL((tile_relayout_kernel<V, PLOG, false>), grid, dim3(256), 0, st, in, out, H, W);
            return;
        }
    }
    const int grid = (int)std::min<long long>(8192, (n + 255) / 256);
    if (to_blocked)
        hipLaunchKernelGGL((relayout_kernel<V, true, PLOG>), dim3(grid), dim3(256), 0, st, in, out, n, H, W);
    else
        hipLaunchKernelGGL((relayout_kernel<V, false, PLOG>), dim3(grid), dim3(256), 0, st, in, out, n, H, W);
}
template <typename V>
int relayout(int plog, const V* in, V* out, long long n, int H, int W, bool to_blocked, hipStream_t st) {
    switch (plog) {
        case 1: relayout_launch<1>(in, out, n, H, W, to_blocked, st); break;
        case 2: relayout_launch<2>(in, out, n, H, W, to_blocked, st); break;
        case 3: relayout_launch<3>(in, out, n, H, W, to_blocked, st); break;
        case 4: relayout_launch<4>(in, out, n, H, W, to_blocked, st); break;
        default: return fail(SLM_ERR_UNSUPPORTED, "no relayout for panel log2 %d", plog);
    }
    HIP_TRY(hipGetLastError());
    return 0;
}

}  // namespace

// GD iteration structures (slm_plan::gd_mode, $SLM_GD_MODE at plan creation)
enum GdMode : int { GD_AUTO = 0, GD_LIN = 1, GD_FUSED = 2, GD_TWO = 3 };

struct slm_plan {
    int algo = 0, B = 0, H = 0, W = 0, tt = 1, has_ain = 0, max_loops = 0;
    int dev_tt = 1;  // TgtType of the device target buffer: tt, or TGT_AMP for float32 GS targets
    int cw = 4, nwg = 0, col_threads = 0, row_threads = 0, rpw = 0;
    int row_key = -1, col_key = -1;  // radix plans (kPlans) of the row / column transforms
    int lid = -1;                    // blocked layout pair (LayoutId), fixed at the first configure
    int device = 0;
    long long holo = 0;
    hipStream_t stream = nullptr;
    int prec = PREC_F32;  // butterflies/twiddles; parity at both precisions: tests/test_gpu_precision.py
    // row kernels' precision: prec, unless $SLM_ROW_PRECISION (f32 / f64, read at
    // creation) splits the two kernels (A/B of float64 in one pass only)
    int prec_row = PREC_F32, prec_row_force = -1;
    // write-through field stores per pass ($SLM_WT=0/1 forces both). Measured
    // (float32): write-through is faster for single images up to 1024^2 (no
    // dirty L2 at the kernel boundary); columns of 2048+ (2-column tiles:
    // half lines, merged in L2 before write-back) and rows of 4096 or of
    // launches with 32M+ elements are faster written back (4096^2 column pass
    // 129 -> 105 us, 4 x 4096^2 row pass 548 -> 480 us).
    int wt_col = 1, wt_row = 1;
    unsigned long long* trace_col = nullptr;  // SLM_TRACE diagnostics ($SLM_TRACE_BUF=1)
    unsigned long long* trace_row = nullptr;
    const void* tw_row = nullptr;
    const void* tw_col = nullptr;
    float2 *xa = nullptr, *xb = nullptr, *y = nullptr, *field = nullptr;
    void* tgt = nullptr;
    float* ain = nullptr;
    float* phase_in = nullptr;
    float* phase_out = nullptr;
    float* e_out = nullptr;
    double* partials = nullptr;
    // COL_GD_FUSED grid max-barrier: [B][max_loops] results, then [B][max_loops][nwg]
    // workgroup slots (preset to kUnset per run), and a fault flag
    double* gsync = nullptr;
    long long gsync_len = 0;
    int* gfault = nullptr;
    int gd_fuse = 1;       // one-launch column side allowed ($SLM_GD_FUSE=0 at creation; cleared by a grid fault)
    // GD iteration structure ($SLM_GD_MODE=auto|lin|fused|two at plan creation):
    // GD_AUTO (default): GD_FUSED where the column grid is resident at once
    //   (float32, unchecked runs), else GD_TWO;
    // GD_FUSED: one column launch -- forward transform, grid max-barrier,
    //   gradient and inverse transform on F in registers -- plus the row launch;
    // GD_TWO: statistics launch + gradient launch that recomputes F;
    // GD_LIN: column launch stores both inverse-transformed terms (Y, Y2), the
    //   row launch folds the maxima and combines them (no in-launch wait at all).
    int gd_mode = GD_AUTO;
    int skip_wg_plus1 = 0;  // $SLM_GD_FAULT_TEST: fused-path fault injection (tests)
    int gd_recoveries = 0;  // runs redone on the two-launch path after a grid fault
    bool fused_pending = false;  // a one-launch GD run is queued and its fault flag not read yet
    bool ran = false;            // a run was enqueued (the state buffers hold something)
    float2* field0 = nullptr;  // GD: host-set initial field (blocked), never overwritten by a run
    bool field_fresh = false;  // set_field since the last run: the plan's field is field0
    // parameters of the last enqueued run (a grid fault reruns it)
    int last_loops = 0, last_checked = 0;
    double last_tol = 0.0;
    float last_wa = 0.f;
    float2* y2 = nullptr;   // GD_LIN: column-inverse transform of mask F T
    double* gmax = nullptr; // GD_LIN: [B][max_loops][nwg] column-workgroup maxima of |F|^2
    double* stats = nullptr;
    int* stop = nullptr;
    double* norm = nullptr;
    float* normf = nullptr;
    double* sum_t2 = nullptr;
    double* ts_part = nullptr;
    float* lr = nullptr;
    float* gather_buf = nullptr;
    long long gather_elems = 0;
    double* gather_stats = nullptr;  // slm_plan_gather_stats on the root
    long long gather_stats_elems = 0;
    int* gather_stop = nullptr;
    long long gather_stop_elems = 0;
    // gathers run on their own stream behind a staging copy, so a rank's next
    // run (plan stream) overlaps the RCCL transfer of the previous step's slab:
    // two staging buffers, used alternately; the copy into one waits for the
    // send that last read it (gather_done)
    hipStream_t comm_stream = nullptr;
    hipEvent_t gather_ready = nullptr;
    hipEvent_t gather_done[2] = {nullptr, nullptr};
    bool gather_done_set[2] = {false, false};
    int gather_last = -1;            // slot of the last gather (its done event orders marks / timing)
    void* stage[2] = {nullptr, nullptr};
    size_t stage_cap[2] = {0, 0};
    int stage_next = 0;
    bool target_set = false, phase_set = false, field_set = false, lr_set = false;
    // timing state (slm_plan_run_timed)
    bool timing = false;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> ev_pool;
    std::vector<int> ev_class;
    size_t ev_used = 0;
    // replayed run (default; SLM_GRAPH=0 launches kernel by kernel): the whole
    // enqueue_run captured once per (loops, tol, checked, wa, warm-start state)
    // and relaunched as one graph -- 3 % per 1024^2 GS iteration, 6 % at 256^2
    // (gpurun_out/exp17: the inter-kernel gaps of 400 dependent launches)
    hipEvent_t marks[2] = {nullptr, nullptr};  // slm_plan_mark stopwatch
    // sides without a radix plan (or $SLM_ENGINE=float64): the any-size engine
    // (generic.hpp) runs the loop; state and arrays row-major, float64 arithmetic
    GenericEngine* gen = nullptr;
    hipGraphExec_t gexec = nullptr;
    bool generic = false;  // an any-size plan (gen is its engine; null only after a failed rebuild)
    int g_loops = -1, g_checked = -1, g_state = -1;
    double g_tol = 0.0;
    float g_wa = 0.f;
};

namespace {


// Column tile width. With the blocked state layout a 4-column panel is one
// contiguous run, so a 4-column tile moves whole lines (2-column tiles, which
// rely on the partner tile fetching the other half of each line through the
// same XCD's L2, measured slower at 4096). SLM_COL_CW overrides.
int pick_cw(int ck, int W) {
    if (const char* s = std::getenv("SLM_COL_CW")) {
        const int cw = std::atoi(s);
        if (col_fn(ck, cw, COL_GS_MAIN, TGT_AMP, PREC_F32) && W % cw == 0) return cw;
    }
    // narrow plans (a single small image) take 2-column tiles: twice the
    // workgroups per CU, the partner tile reads the other half of each line
    // through the same XCD's L2 (measured 13.0 -> 10.7 us per 1024^2 pass)
    if (kPlans[ck].variant == 1 && W % 2 == 0 && col_fn(ck, 2, COL_GS_MAIN, TGT_AMP, PREC_F32)) return 2;
    // first tile (in this order) whose complex64 LDS leaves room for two
    // workgroups per CU; 2-column tiles only with >= 8 waves (long columns)
    for (int cw : {4, 8, 16, 2}) {
        if (W % cw || !col_fn(ck, cw, COL_GS_MAIN, TGT_AMP, PREC_F32)) continue;
        const long long lds = (long long)lds_line(kPlans[ck].n) * cw * 8;
        const int threads = cw * (kPlans[ck].n / kPlans[ck].e);
        if (lds <= 80 * 1024 && (cw != 2 || threads >= 512)) return cw;
    }
    for (int cw : {4, 8, 16, 2})
        if (W % cw == 0 && col_fn(ck, cw, COL_GS_MAIN, TGT_AMP, PREC_F32)) return cw;
    return 0;
}

// Radix plan of one axis: the narrow variant (half the elements per thread)
// when the wide one would leave fewer than 4 waves per SIMD on the chip
// (e.g. a single 1024^2 hologram), else the wide one. $SLM_PLAN=wide|narrow
// forces a variant where it exists.
// Float32 transforms take the narrow plan where the wide one holds more than
// 16 elements per thread (4096: 32 spill).
int pick_plan(int n, long long elems, int prec, bool row = false) {
    const int wide = plan_index(n, 0), narrow = plan_index(n, 1);
    if (narrow < 0) return wide;
    if (const char* s = std::getenv(row ? "SLM_ROW_PLAN" : "SLM_COL_PLAN")) {
        if (!std::strcmp(s, "wide")) return wide;
        if (!std::strcmp(s, "narrow")) return narrow;
    }
    if (const char* s = std::getenv("SLM_PLAN")) {
        if (!std::strcmp(s, "wide")) return wide;
        if (!std::strcmp(s, "narrow")) return narrow;
    }
    if (prec == PREC_F32 && kPlans[wide].e > 16 && kPlans[narrow].e <= 16) return narrow;
    // 2048-point rows: the 4-pass E = 8 plan beats the 3-pass E = 16 one at
    // every batch (gpurun_out/exp19: 1 image 26.7 -> 21.7 us, 16 images
    // 405 -> 292 us per row launch); columns keep the rule below
    if (row && prec == PREC_F32 && n == 2048) return narrow;
    // float64 4096-point rows: the 3-pass E = 16 plan (one row per workgroup)
    // beats the 4-pass E = 32 one (gpurun_out/s5: 4096^2 row pass 180 -> 142 us,
    // columns keep the wide plan: 200 vs 238 us)
    if (row && prec == PREC_F64 && n == 4096) return narrow;
    const long long waves = elems / kPlans[wide].e / 64;
    return waves < 4LL * 1024 ? narrow : wide;
}

// Radix plans, tiles and twiddle tables of a plan for one arithmetic precision
// (slm_plan_create, slm_plan_set_precision).
int configure(slm_plan* p, int prec) {
    const long long elems = (long long)p->B * p->holo;
    const int prow = p->prec_row_force >= 0 ? p->prec_row_force : prec;
    const int row_key = pick_plan(p->W, elems, prow, true);
    const int col_key = pick_plan(p->H, elems, prec);
    const int cw = pick_cw(col_key, p->W);
    if (!cw) return fail(SLM_ERR_UNSUPPORTED, "no column tiling for %dx%d", p->H, p->W);
    const void *tr = nullptr, *tc = nullptr;
    RC(get_twiddles(row_key, prow, &tr));
    RC(get_twiddles(col_key, prec, &tc));
    if (p->gexec) {  // the captured run bakes in kernels and tables
        HIP_TRY(hipStreamSynchronize(p->stream));  // a queued replay still owns the exec
        HIP_TRY(hipGraphExecDestroy(p->gexec));
        p->gexec = nullptr;
    }
    // layout pair: the narrow one where both transforms have kernels for it
    // ($SLM_LAYOUT=default forces the default pair; GS 1024^2 20.9 -> 19.6 us
    // per iteration at r02). Device buffers are laid out at upload, so a plan
    // keeps the pair it was created with.
    int lid = LAYOUT_DEFAULT;
    // GD takes the narrow pair too since its column side became one launch
    // (GD 1024^2 fused column pass 14.55 -> 13.66 us, 25.97 -> 25.19 us per
    // iteration, bitwise the same phases: gpurun_out/s11; $SLM_GD_LAYOUT=default
    // keeps the default pair for GD only)
    const char* gl = std::getenv("SLM_GD_LAYOUT");
    const bool algo_ok = p->algo == SLM_ALGO_GS || !(gl && !std::strcmp(gl, "default"));
    const bool narrow_ok = algo_ok && row_fn(row_key, ROW_GS_MAIN, prow, LAYOUT_NARROW) &&
                           col_fn(col_key, cw, COL_GS_MAIN, TGT_AMP, prec, LAYOUT_NARROW);
    const char* ls = std::getenv("SLM_LAYOUT");
    if (narrow_ok && !(ls && !std::strcmp(ls, "default"))) lid = LAYOUT_NARROW;
    if (p->lid >= 0 && lid != p->lid) {
        if (p->lid == LAYOUT_NARROW && !narrow_ok)
            return fail(SLM_ERR_UNSUPPORTED, "precision change leaves the plan's layout unsupported");
        lid = p->lid;
    }
    p->lid = lid;
    p->prec = prec;
    p->prec_row = prow;
    p->row_key = row_key;
    p->col_key = col_key;
    p->cw = cw;
    p->nwg = p->W / cw;
    p->col_threads = col_threads(col_key, cw);
    p->row_threads = row_threads(row_key, prow);
    p->rpw = row_rpw(row_key, prow);
    p->tw_row = tr;
    p->tw_col = tc;
    return 0;
}

// Every kernel of a run is launched through here. In a timed run
// (slm_plan_run_timed) each launch carries its own start/stop events
// (hipExtLaunchKernelGGL): the dispatch packet stamps them, so they bracket the
// kernel's execution alone, as rocprofv3's kernel trace does, with no marker
// packets between kernels.
template <typename F, typename... Args>
int launch(slm_plan* p, int cls, F fn, dim3 grid, dim3 block, Args... args) {
    if (p->timing) {
        if (p->ev_used == p->ev_pool.size()) {
            hipEvent_t a, b;
            HIP_TRY(hipEventCreate(&a));
            HIP_TRY(hipEventCreate(&b));
            p->ev_pool.emplace_back(a, b);
            p->ev_class.push_back(cls);
        }
        p->ev_class[p->ev_used] = cls;
        auto& ev = p->ev_pool[p->ev_used++];
        hipExtLaunchKernelGGL(fn, grid, block, 0, p->stream, ev.first, ev.second, 0, args...);
    } else {
        hipLaunchKernelGGL(fn, grid, block, 0, p->stream, args...);
    }
    HIP_TRY(hipGetLastError());
    return 0;
}

RowParams row_params(slm_plan* p) {
    RowParams r{};
    r.ain = p->ain;
    r.phase_in = p->phase_in;
    r.phase_out = p->phase_out;
    r.field = p->field;
    r.field_src = p->field;
    r.lr = p->lr;
    r.stop_iter = p->stop;
    r.W = p->W;
    r.H = p->H;
    r.holo = p->holo;
    r.inv_s = (float)(1.0 / (double)p->holo);
    r.tw = p->tw_row;
    r.wt = p->wt_row;
    r.trace = p->trace_row;
    return r;
}

ColParams col_params(slm_plan* p) {
    ColParams c{};
    c.tgt = p->tgt;
    c.partials = p->partials;
    c.e_out = p->e_out;
    c.stop_iter = p->stop;
    c.norm = p->normf;
    c.max_loops = p->max_loops;
    c.W = p->W;
    c.nwg = p->nwg;
    c.holo = p->holo;
    c.stat_k = std::ldexp(1.0f, -2 * (int)std::ceil(std::log2((double)p->holo)));
    c.tw = p->tw_col;
    c.wt = p->wt_col;
    c.trace = p->trace_col;
    return c;
}


// One workgroup per tile (kernels.hpp, tile_loop).
int tile_grid(long long tiles, int* grid) {
    if (tiles > INT_MAX) return fail(SLM_ERR_ARG, "%lld tiles exceed one launch", tiles);
    *grid = (int)tiles;
    return 0;
}

int launch_row(slm_plan* p, int mode, const RowParams& rp, int cls) {
    RowFn fn = row_fn(p->row_key, mode, p->prec_row, p->lid);
    if (!fn) return fail(SLM_ERR_UNSUPPORTED, "no row kernel for width %d mode %d", p->W, mode);
    RowParams r = rp;
    r.B = p->B;
    r.ntile = p->H / p->rpw;
    int grid = 0;
    RC(tile_grid((long long)r.ntile * p->B, &grid));
    return launch(p, cls, fn, dim3(grid), dim3(p->row_threads), r);
}

int launch_col(slm_plan* p, int mode, const ColParams& cp, int cls) {
    const int tt = (mode == COL_EXPECTED || mode == COL_FFT_FWD || mode == COL_FFT_INV) ? TGT_F32 : p->dev_tt;
    ColFn fn = col_fn(p->col_key, p->cw, mode, tt, p->prec, p->lid);
    if (!fn) return fail(SLM_ERR_UNSUPPORTED, "no column kernel for height %d cw %d mode %d", p->H, p->cw, mode);
    ColParams c = cp;
    c.B = p->B;
    int grid = 0;
    RC(tile_grid((long long)p->nwg * p->B, &grid));
    return launch(p, cls, fn, dim3(grid), dim3(p->col_threads), c);
}

// the expected output E written by the GS column pass in layout Y (e_blk) ->
// the row-major e_out (LDS-tiled transpose; one launch for the batch)
int unblock_expected(slm_plan* p, const float* e_blk) {
    const dim3 grid(p->W / 64, p->H / 64, p->B);
    switch (layout_y_log2(p->lid)) {
        case 1: return launch(p, SLM_KERNEL_OTHER, tile_relayout_kernel<float, 1, false>, grid, dim3(256), e_blk, p->e_out, p->H, p->W);
        case 2: return launch(p, SLM_KERNEL_OTHER, tile_relayout_kernel<float, 2, false>, grid, dim3(256), e_blk, p->e_out, p->H, p->W);
        case 3: return launch(p, SLM_KERNEL_OTHER, tile_relayout_kernel<float, 3, false>, grid, dim3(256), e_blk, p->e_out, p->H, p->W);
        case 4: return launch(p, SLM_KERNEL_OTHER, tile_relayout_kernel<float, 4, false>, grid, dim3(256), e_blk, p->e_out, p->H, p->W);
        default: return fail(SLM_ERR_UNSUPPORTED, "no unblock kernel for panel log2 %d", layout_y_log2(p->lid));
    }
}

// expected output |C|^2 (src/algorithms.py:36) of GD (and the intensity
// helper): a forward column pass writes it in layout Y into the free Y buffer
// (every reader of Y precedes this on the stream), then the tiled unblock
int launch_expected(slm_plan* p, ColParams cp) {
    cp.e_blk = reinterpret_cast<float*>(p->y);
    RC(launch_col(p, COL_EXPECTED, cp, SLM_KERNEL_OTHER));
    return unblock_expected(p, reinterpret_cast<const float*>(p->y));
}

StatsParams stats_params(slm_plan* p, double tol) {
    StatsParams s{};
    s.partials = p->partials;
    s.stats = p->stats;
    s.stop_iter = p->stop;
    s.norm = p->norm;
    s.sum_t2 = p->sum_t2;
    s.inv_s = 1.0 / (double)p->holo;
    s.tol = tol;
    s.max_loops = p->max_loops;
    s.nwg = p->nwg;
    return s;
}

int launch_finalize(slm_plan* p, double tol, int iter) {
    StatsParams s = stats_params(p, tol);
    s.iter = iter;
    return launch(p, SLM_KERNEL_OTHER, stats_finalize_kernel, dim3(p->B), dim3(256), s);
}


int enqueue_gs(slm_plan* p, int loops, double tol, int checked) {
    RowParams rp = row_params(p);
    ColParams cp = col_params(p);
    cp.loops = loops;
    rp.checked = cp.checked = checked;
    // setup: X0 = rowFFT(a_in A0/|A0|), A0 = ifft2(sqrt T) (src/algorithms.py:14-27),
    // or the warm start B = a_in exp(i phi).
    if (p->phase_set) {
        rp.out = p->xa;
        RC(launch_row(p, ROW_PHASE_FWD, rp, SLM_KERNEL_OTHER));
    } else {
        cp.out = p->y;
        RC(launch_col(p, COL_REAL_INV, cp, SLM_KERNEL_OTHER));
        rp.in = p->y;
        rp.out = p->xa;
        rp.iter = -1;
        RC(launch_row(p, ROW_GS_MAIN, rp, SLM_KERNEL_OTHER));
    }
    // expected_outcome = |C|^2 of the last iteration (src/algorithms.py:36): the
    // column pass of the last iteration (of every iteration in a checked run,
    // where the last is not known in advance; a stopped hologram's later passes
    // leave it untouched) stores it in layout Y into phase_out, free until the
    // phase extraction below
    float* const e_blk = p->phase_out;
    for (int i = 0; i < loops; ++i) {
        cp.in = p->xa;
        cp.out = p->y;
        cp.iter = i;
        cp.e_blk = (checked || i + 1 == loops) ? e_blk : nullptr;
        RC(launch_col(p, COL_GS_MAIN, cp, SLM_KERNEL_COL_MAIN));
        if (checked) RC(launch_finalize(p, tol, i));
        if (i + 1 < loops) {
            rp.in = p->y;
            rp.out = p->xa;
            rp.iter = i;
            RC(launch_row(p, ROW_GS_MAIN, rp, SLM_KERNEL_ROW_MAIN));
        }
    }
    RC(unblock_expected(p, e_blk));
    // hologram = np.angle(A) (src/algorithms.py:48)
    rp.in = p->y;
    RC(launch_row(p, ROW_GS_PHASE, rp, SLM_KERNEL_OTHER));
    return 0;
}

// GD column side in one launch (COL_GD_FUSED, a grid barrier for the global
// max of |F|^2) when it is safe and built: unchecked runs (no workgroup leaves
// early), float32 kernels, and a grid whose workgroups are all resident at once
// (occupancy x CUs, one tile per workgroup). Otherwise the statistics pass and
// the gradient pass run as two launches. $SLM_GD_FUSE=0 forces two launches.
ColFn gd_fused_fn(slm_plan* p, int checked) {
    if (!p->gd_fuse || !p->gsync || checked) return nullptr;
    if (p->gd_mode != GD_AUTO && p->gd_mode != GD_FUSED) return nullptr;
    if (2LL * p->B * p->max_loops * (1 + p->nwg) > INT_MAX) return nullptr;  // slot area: two launches instead
    ColFn fn = col_fn(p->col_key, p->cw, COL_GD_FUSED, p->tt, p->prec, p->lid);
    if (!fn) return nullptr;
    int dev = 0, cus = 0, per_cu = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)fn, p->col_threads, 0) != hipSuccess)
        return nullptr;
    return (long long)p->nwg * p->B <= (long long)per_cu * cus ? fn : nullptr;
}

int enqueue_gd(slm_plan* p, int loops, double tol, int checked, float wa) {
    RowParams rp = row_params(p);
    ColParams cp = col_params(p);
    cp.loops = loops;
    rp.checked = cp.checked = checked;
    cp.wa = wa;
    // setup (make_initial_guess, src/algorithms.py:115-158): host-provided field
    // or the "fourier" guess a_in exp(i angle(ifft2(sqrt T))).
    if (p->field_set) {
        rp.out = p->xa;
        rp.field_src = p->field0;
        RC(launch_row(p, ROW_GD_INIT_FIELD, rp, SLM_KERNEL_OTHER));
    } else {
        cp.out = p->y;
        RC(launch_col(p, COL_REAL_INV, cp, SLM_KERNEL_OTHER));
        rp.in = p->y;
        rp.out = p->xa;
        RC(launch_row(p, ROW_GD_INIT_Y, rp, SLM_KERNEL_OTHER));
    }
    const bool lin = p->gd_mode == GD_LIN;
    const bool fused = !lin && gd_fused_fn(p, checked) != nullptr;
    if (fused) {
        cp.gresult = p->gsync;
        cp.gslots = p->gsync + (long long)p->B * p->max_loops;
        cp.fault = p->gfault;
        cp.skip_wg_plus1 = p->skip_wg_plus1;
        // every result and slot word to kUnset (all bits set) before the run
        // (gd_fused_fn keeps the slot area within INT_MAX words)
        const long long words = 2LL * p->B * p->max_loops * (1 + p->nwg);
        RC(launch(p, SLM_KERNEL_OTHER, fill_int_kernel, dim3((int)std::min<long long>(65535, (words + 255) / 256)),
                  dim3(256), (int*)p->gsync, (int)words, -1));
    }
    for (int i = 0; i < loops; ++i) {
        float2* xi = (i & 1) ? p->xb : p->xa;
        float2* xn = (i & 1) ? p->xa : p->xb;
        // iteration 0 reads a host-set field from field0 (kept intact for reruns)
        rp.field_src = (i == 0 && p->field_set) ? p->field0 : p->field;
        cp.in = xi;
        cp.iter = i;
        cp.out = p->y;
        if (lin) {
            cp.out2 = p->y2;
            cp.gmax = p->gmax;
            RC(launch_col(p, COL_GD_LIN, cp, SLM_KERNEL_COL_MAIN));
            if (checked) RC(launch_finalize(p, tol, i));
            rp.in = p->y;
            rp.in2 = p->y2;
            rp.gmax = p->gmax;
            rp.norm = p->normf;
            rp.nwg_col = p->nwg;
            rp.max_loops = p->max_loops;
            rp.out = xn;
            rp.iter = i;
            RC(launch_row(p, ROW_GD_LIN, rp, SLM_KERNEL_ROW_MAIN));
            continue;
        }
        if (fused) {
            RC(launch_col(p, COL_GD_FUSED, cp, SLM_KERNEL_COL_MAIN));
        } else {
            RC(launch_col(p, COL_GD_STATS, cp, SLM_KERNEL_GD_STATS));
            if (checked) RC(launch_finalize(p, tol, i));
            RC(launch_col(p, COL_GD_GRAD, cp, SLM_KERNEL_COL_MAIN));
        }
        rp.in = p->y;
        rp.out = xn;
        rp.iter = i;
        RC(launch_row(p, ROW_GD_MAIN, rp, SLM_KERNEL_ROW_MAIN));
    }
    {
        const long long n = (long long)p->B * p->holo;
        const int grid = (int)std::min<long long>(4096, (n + 255) / 256);
        const int yl = layout_y_log2(p->lid);
        auto fk = yl == 1 ? field_phase_kernel<1>
                  : yl == 3 ? field_phase_kernel<3> : yl == 4 ? field_phase_kernel<4> : field_phase_kernel<2>;
        RC(launch(p, SLM_KERNEL_OTHER, fk, dim3(grid), dim3(256), (const float2*)p->field, p->phase_out, n, p->H,
                  p->W));
    }
    cp.in = p->xa;
    cp.in_alt = p->xb;
    RC(launch_expected(p, cp));
    return 0;
}

// A grid wait of COL_GD_FUSED that gave up (kernels.hpp, wait_set) leaves a
// fault flag: that run's results are invalid. Read it after the stream has
// drained; on a fault the plan gives up its one-launch column side for good
// (its workgroups were not co-resident: other work shares the device) and
// redoes the same run on the two-launch path in-process (the run's inputs --
// target, field0, learning rates -- are untouched by a run). *faulted tells
// the caller that the stream now holds the rerun.
int recover_grid_fault(slm_plan* p, bool* faulted) {
    *faulted = false;
    if (!p->gfault) return 0;
    p->fused_pending = false;  // the caller drained the stream: the flag below covers every queued run
    int f = 0;
    RC(copy_sync(&f, p->gfault, sizeof(int), hipMemcpyDeviceToHost, p->stream));
    if (!f) return 0;
    HIP_TRY(hipMemsetAsync(p->gfault, 0, sizeof(int), p->stream));
    HIP_TRY(hipStreamSynchronize(p->stream));
    *faulted = true;
    p->gd_fuse = 0;
    p->gd_recoveries += 1;
    if (p->gexec) {  // the captured run holds the fused kernel
        HIP_TRY(hipGraphExecDestroy(p->gexec));
        p->gexec = nullptr;
    }
    return 0;
}

// GenericView::mark of timed runs: each marked launch between an event pair on
// the plan stream (the any-size engine launches directly)
int generic_mark(void* ctx, int cls, int begin) {
    slm_plan* p = static_cast<slm_plan*>(ctx);
    if (begin) {
        if (p->ev_used == p->ev_pool.size()) {
            hipEvent_t a, b;
            HIP_TRY(hipEventCreate(&a));
            HIP_TRY(hipEventCreate(&b));
            p->ev_pool.emplace_back(a, b);
            p->ev_class.push_back(cls);
        }
        p->ev_class[p->ev_used] = cls;
        HIP_TRY(hipEventRecord(p->ev_pool[p->ev_used].first, p->stream));
    } else {
        HIP_TRY(hipEventRecord(p->ev_pool[p->ev_used++].second, p->stream));
    }
    return 0;
}

GenericView gview(slm_plan* p) {
    GenericView v;
    v.algo = p->algo;
    v.B = p->B;
    v.H = p->H;
    v.W = p->W;
    v.tt = p->tt;
    v.has_ain = p->has_ain;
    v.max_loops = p->max_loops;
    v.nwg = p->nwg;
    v.prec = p->prec;
    v.holo = p->holo;
    v.stream = p->stream;
    v.tgt = p->tgt;
    v.ain = p->ain;
    v.phase_in = p->phase_in;
    v.field0 = p->field0;
    v.lr = p->lr;
    v.phase_out = p->phase_out;
    v.e_out = p->e_out;
    v.partials = p->partials;
    v.stats = p->stats;
    v.stop = p->stop;
    v.norm = p->norm;
    v.sum_t2 = p->sum_t2;
    if (p->timing) {  // slm_plan_run_timed: one event pair per iteration launch
        v.mark = &generic_mark;
        v.mark_ctx = p;
    }
    return v;
}

int enqueue_run(slm_plan* p, int loops, double tol, int checked, float wa) {
    if (!p) return fail(SLM_ERR_ARG, "null plan");
    if (!p->target_set) return fail(SLM_ERR_STATE, "target not set");
    if (loops < 1 || loops > p->max_loops)
        return fail(SLM_ERR_ARG, "loops %d outside [1, %d]", loops, p->max_loops);
    if (p->algo == SLM_ALGO_GD && !p->lr_set) return fail(SLM_ERR_STATE, "learning rates not set");
    if (p->generic && !p->gen) return fail(SLM_ERR_STATE, "the plan lost its engine (failed slm_plan_set_precision)");
    HIP_TRY(hipSetDevice(p->device));
    p->field_fresh = false;  // the run writes the field
    p->ran = true;
    RC(launch(p, SLM_KERNEL_OTHER, fill_int_kernel, dim3((p->B + 255) / 256), dim3(256), p->stop, p->B,
              (int)INT_MAX));
    if (p->gen)
        RC(generic_enqueue(p->gen, gview(p), loops, tol, checked, wa, p->phase_set, p->field_set));
    else
        RC(p->algo == SLM_ALGO_GS ? enqueue_gs(p, loops, tol, checked) : enqueue_gd(p, loops, tol, checked, wa));
    StatsParams s = stats_params(p, tol);
    RC(launch(p, SLM_KERNEL_OTHER, stats_reduce_kernel, dim3(loops, p->B), dim3(256), s));
    return 0;
}

void free_plan(slm_plan* p) {
    if (!p) return;
    (void)hipSetDevice(p->device);
    // work still queued on the plan stream (an unsynchronised run, a
    // stream-ordered device gather or RCCL send) finishes before its buffers go
    if (p->stream) (void)hipStreamSynchronize(p->stream);
    if (p->comm_stream) (void)hipStreamSynchronize(p->comm_stream);  // gathers still reading / writing
    for (void* ptr : {(void*)p->xa, (void*)p->xb, (void*)p->y, (void*)p->field, p->tgt, (void*)p->ain,
                      (void*)p->phase_in, (void*)p->phase_out, (void*)p->e_out, (void*)p->partials,
                      (void*)p->stats, (void*)p->stop, (void*)p->norm, (void*)p->normf, (void*)p->sum_t2,
                      (void*)p->ts_part, (void*)p->lr, (void*)p->gsync, (void*)p->gfault, (void*)p->gather_buf,
                      (void*)p->gather_stats, (void*)p->gather_stop, (void*)p->y2, (void*)p->gmax,
                      (void*)p->field0, (void*)p->trace_col, (void*)p->trace_row})
        if (ptr) (void)hipFree(ptr);
    for (auto& e : p->ev_pool) {
        (void)hipEventDestroy(e.first);
        (void)hipEventDestroy(e.second);
    }
    for (int k = 0; k < 2; ++k) {
        if (p->stage[k]) (void)hipFree(p->stage[k]);
        if (p->gather_done[k]) (void)hipEventDestroy(p->gather_done[k]);
    }
    if (p->gather_ready) (void)hipEventDestroy(p->gather_ready);
    if (p->comm_stream) (void)hipStreamDestroy(p->comm_stream);
    if (p->gexec) (void)hipGraphExecDestroy(p->gexec);
    generic_destroy(p->gen);
    for (hipEvent_t e : p->marks)
        if (e) (void)hipEventDestroy(e);
    if (p->stream) (void)hipStreamDestroy(p->stream);
    delete p;
}

}  // namespace

// used by frames.hip
int slm_set_error(int code, const char* msg) { return fail(code, "%s", msg); }
int slm_current_device_ready() { return ensure_device(); }

// ==========================================================================
// C-ABI
// ==========================================================================
extern "C" {

int slm_init(int device) {
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess || n <= 0)
        return fail(SLM_ERR_HIP, "no HIP device available (%s); libslm_hip has no CPU path",
                    hipGetErrorString(e));
    if (device < 0 || device >= n) return fail(SLM_ERR_ARG, "device %d outside [0, %d)", device, n);
    HIP_TRY(hipSetDevice(device));
    g_device = device;
    return 0;
}

int slm_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

const char* slm_last_error(void) { return g_err.c_str(); }

int slm_copy_bandwidth(long long bytes, int reps, double* gbs) {
    if (!gbs || bytes < 16 || reps < 1) return fail(SLM_ERR_ARG, "bad copy-bandwidth arguments");
    RC(ensure_device());
    const long long n = bytes / 16;
    v4f *a = nullptr, *b = nullptr;
    hipStream_t st = nullptr;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    int dev = 0, cus = 0, rc = 0;
    auto hip = [&](hipError_t e) {
        if (e != hipSuccess && !rc) rc = fail(SLM_ERR_HIP, "copy bandwidth: %s", hipGetErrorString(e));
        return rc == 0;
    };
    if (hip(hipGetDevice(&dev)) && hip(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev)) &&
        hip(hipMalloc(&a, n * 16)) && hip(hipMalloc(&b, n * 16)) && hip(hipStreamCreate(&st)) &&
        hip(hipEventCreate(&e0)) && hip(hipEventCreate(&e1)) && hip(hipMemsetAsync(a, 1, n * 16, st)) &&
        hip(hipMemsetAsync(b, 0, n * 16, st))) {
        // enough workgroups that a working-set-sized copy still fills the chip
        const int grid = (int)std::max<long long>(1, std::min<long long>((long long)cus * 32, (n + 1023) / 1024));
        hipLaunchKernelGGL(copy_f4_kernel, dim3(grid), dim3(256), 0, st, a, b, n);  // warm-up
        // a failed launch would leave the event pair timing an empty stream
        if (hip(hipGetLastError()) && hip(hipEventRecord(e0, st))) {
            for (int i = 0; i < reps; ++i) hipLaunchKernelGGL(copy_f4_kernel, dim3(grid), dim3(256), 0, st, a, b, n);
            float ms = 0.f;
            if (hip(hipGetLastError()) && hip(hipEventRecord(e1, st)) && hip(hipEventSynchronize(e1)) &&
                hip(hipEventElapsedTime(&ms, e0, e1)))
                *gbs = 2.0 * 16.0 * (double)n * reps / (ms * 1e-3) / 1e9;
        }
    }
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
    if (st) (void)hipStreamDestroy(st);
    if (a) (void)hipFree(a);
    if (b) (void)hipFree(b);
    return rc;
}

const char* slm_version(void) { return "libslm_hip 0.1 (gfx950)"; }

int slm_supported_length(int n) { return plan_index(n) >= 0 ? 1 : 0; }

int slm_device_pci_bus_id(int device, char* buf, int len) {
    if (!buf || len < 13) return fail(SLM_ERR_ARG, "need a buffer of at least 13 bytes");
    HIP_TRY(hipDeviceGetPCIBusId(buf, len, device));
    return 0;
}

}  // extern "C"

namespace {
int plan_create_on(int device, int algo, int batch, int height, int width, int tgt_type, int has_ain,
                   int max_loops, slm_plan** out);
}

extern "C" {

int slm_plan_create(int algo, int batch, int height, int width, int tgt_type, int has_ain, int max_loops,
                    slm_plan** out) {
    RC(ensure_device());
    return plan_create_on(g_device, algo, batch, height, width, tgt_type, has_ain, max_loops, out);
}

}  // extern "C"

namespace {
int plan_create_on(int device, int algo, int batch, int height, int width, int tgt_type, int has_ain,
                   int max_loops, slm_plan** out) {
    if (!out) return fail(SLM_ERR_ARG, "null output pointer");
    *out = nullptr;
    if (algo != SLM_ALGO_GS && algo != SLM_ALGO_GD) return fail(SLM_ERR_ARG, "unknown algorithm %d", algo);
    if (batch < 1 || max_loops < 1) return fail(SLM_ERR_ARG, "batch and max_loops must be >= 1");
    if (tgt_type != SLM_TGT_U8 && tgt_type != SLM_TGT_F32) return fail(SLM_ERR_ARG, "unknown target type");
    if (height < 1 || width < 1) return fail(SLM_ERR_ARG, "image shape %dx%d", height, width);
    // sides without a radix plan (plans.hpp) run the any-size engine (generic.hpp:
    // mixed-radix kernels, chirp-z line transforms for large prime factors).
    // $SLM_ENGINE=float64
    // sends every shape there: complex128 state and float64 arithmetic
    // throughout, the reference's own dtypes -- the radix plans keep complex64
    // between their passes, which sets GD's float64-butterfly floor at ~3e-5
    // rms after configs[2]'s 500 iterations (profiles/r05/gd_precision_s19.txt)
    const char* eng = std::getenv("SLM_ENGINE");
    const bool generic = (eng && !std::strcmp(eng, "float64")) || !slm_supported_length(height) ||
                         !slm_supported_length(width);
    HIP_TRY(hipSetDevice(device));
    slm_plan* p = new slm_plan();
    p->algo = algo;
    p->B = batch;
    p->H = height;
    p->W = width;
    p->tt = tgt_type;
    // GS keeps a float32 target as its amplitude on the device (set_target)
    p->dev_tt = (algo == SLM_ALGO_GS && tgt_type == SLM_TGT_F32) ? TGT_AMP : tgt_type;
    p->has_ain = has_ain ? 1 : 0;
    p->max_loops = max_loops;
    p->device = device;
    p->holo = (long long)height * width;
    p->wt_col = height >= 2048 ? 0 : 1;
    p->wt_row = ((long long)batch * p->holo >= (32LL << 20) || width >= 4096) ? 0 : 1;
    if (const char* e = std::getenv("SLM_WT")) p->wt_col = p->wt_row = std::atoi(e) != 0;
    if (const char* e = std::getenv("SLM_GD_FUSE")) p->gd_fuse = std::atoi(e) != 0;
    if (const char* e = std::getenv("SLM_GD_MODE"))
        p->gd_mode = !std::strcmp(e, "fused") ? GD_FUSED
                     : !std::strcmp(e, "two") ? GD_TWO
                     : !std::strcmp(e, "lin") ? GD_LIN
                                              : GD_AUTO;
    if (!p->gd_fuse && p->gd_mode != GD_LIN) p->gd_mode = GD_TWO;
    if (p->gd_mode == GD_TWO || p->gd_mode == GD_LIN) p->gd_fuse = 0;
    if (const char* e = std::getenv("SLM_GD_FAULT_TEST")) p->skip_wg_plus1 = std::atoi(e);
    // GS on uint8 targets -- the CLI's input (src/generate_hologram.py:102-110) --
    // takes float64 butterflies by default: float32 measured 7.7e-6 (1024^2) and
    // 8.2e-6 (768 x 1024, the CLI's own shape) of the 1e-5 bar at the +200 warm
    // start, float64 rows alone still 8.5e-6 at 768 x 1024, float64 butterflies
    // <= 3.3e-6 on all six targets (profiles/r06/u8_margin.txt), for ~3 us per
    // iteration. Float32 targets (the bench's) keep float32; $SLM_PRECISION
    // (f32 / f64) overrides both.
    if (algo == SLM_ALGO_GS && tgt_type == SLM_TGT_U8) p->prec = PREC_F64;
    if (const char* e = std::getenv("SLM_PRECISION")) p->prec = (std::strcmp(e, "f64") == 0) ? PREC_F64 : PREC_F32;
    if (const char* e = std::getenv("SLM_ROW_PRECISION"))
        p->prec_row_force = (std::strcmp(e, "f64") == 0) ? PREC_F64 : PREC_F32;
    // buffers indexed by column panel / row group hold the finer tiling of both precisions
    int max_nwg = 0, min_rpw = INT_MAX;
    if (generic) {
        p->dev_tt = tgt_type;  // row-major target, amplitude formed where used
        // float32 GS (float32 targets unless $SLM_PRECISION) on the complex64
        // radix kernels where both sides have one (13-smooth panels, e.g.
        // 1080 x 1920), float64 otherwise and always under $SLM_ENGINE=float64
        const bool forced64 = eng && !std::strcmp(eng, "float64");
        p->prec = generic_precision(batch, height, width, algo, forced64 ? PREC_F64 : p->prec);
        p->lid = LAYOUT_DEFAULT;
        p->cw = 0;
        p->nwg = generic_nwg(batch, height, width, p->holo, algo, p->prec);
        // slm_plan_set_precision may switch engines: partials for either tiling
        max_nwg = std::max(generic_nwg(batch, height, width, p->holo, algo, PREC_F32),
                           generic_nwg(batch, height, width, p->holo, algo, PREC_F64));
        p->rpw = min_rpw = 1;
    } else {
        const int want = p->prec;
        for (int prec : {PREC_F32, PREC_F64}) {
            int rc = configure(p, prec);
            if (rc) {
                delete p;
                return rc;
            }
            max_nwg = std::max(max_nwg, p->nwg);
            min_rpw = std::min(min_rpw, p->rpw);
        }
        if (int rc = configure(p, want)) {
            delete p;
            return rc;
        }
    }
    const size_t n = (size_t)batch * p->holo;
    const size_t tb = tgt_type == SLM_TGT_U8 ? 1 : 4;
    auto alloc = [&](void** ptr, size_t bytes) -> int {
        hipError_t e = hipMalloc(ptr, bytes);
        if (e != hipSuccess) {
            free_plan(p);
            return fail(SLM_ERR_HIP, "hipMalloc(%zu) failed: %s", bytes, hipGetErrorString(e));
        }
        return 0;
    };
    hipError_t se = hipStreamCreateWithFlags(&p->stream, hipStreamNonBlocking);
    if (se != hipSuccess) {
        delete p;
        return fail(SLM_ERR_HIP, "stream creation failed: %s", hipGetErrorString(se));
    }
    RC(alloc((void**)&p->xa, n * sizeof(float2)));  // generic plans: complex64 staging (fft2, read_field)
    if (!generic) RC(alloc((void**)&p->y, n * sizeof(float2)));
    if (algo == SLM_ALGO_GD && generic) {
        RC(alloc((void**)&p->field0, n * sizeof(float2)));
        RC(alloc((void**)&p->lr, (size_t)max_loops * sizeof(float)));
    } else if (algo == SLM_ALGO_GD) {
        RC(alloc((void**)&p->xb, n * sizeof(float2)));
        RC(alloc((void**)&p->field, n * sizeof(float2)));
        RC(alloc((void**)&p->field0, n * sizeof(float2)));
        RC(alloc((void**)&p->lr, (size_t)max_loops * sizeof(float)));
        if (p->gd_mode == GD_LIN) {
            RC(alloc((void**)&p->y2, n * sizeof(float2)));
            RC(alloc((void**)&p->gmax, (size_t)batch * max_loops * max_nwg * sizeof(double)));
        }
        // the one-launch column side needs the whole grid resident: never beyond 8192 workgroups
        if ((p->gd_mode == GD_FUSED || p->gd_mode == GD_AUTO) && (long long)batch * max_nwg <= 8192) {
            p->gsync_len = (long long)batch * max_loops * (1 + max_nwg);
            RC(alloc((void**)&p->gsync, (size_t)p->gsync_len * sizeof(double)));
            RC(alloc((void**)&p->gfault, sizeof(int)));
            HIP_TRY(hipMemsetAsync(p->gfault, 0, sizeof(int), p->stream));
    HIP_TRY(hipStreamSynchronize(p->stream));
        }
    }
    RC(alloc(&p->tgt, n * tb));
    if (has_ain) RC(alloc((void**)&p->ain, (size_t)p->holo * sizeof(float)));
    RC(alloc((void**)&p->phase_out, n * sizeof(float)));
    RC(alloc((void**)&p->e_out, n * sizeof(float)));
    RC(alloc((void**)&p->partials, (size_t)batch * max_loops * max_nwg * 4 * sizeof(double)));
    RC(alloc((void**)&p->stats, (size_t)batch * max_loops * 4 * sizeof(double)));
    RC(alloc((void**)&p->stop, (size_t)batch * sizeof(int)));
    RC(alloc((void**)&p->norm, (size_t)batch * sizeof(double)));
    RC(alloc((void**)&p->normf, (size_t)batch * sizeof(float)));
    RC(alloc((void**)&p->sum_t2, (size_t)batch * sizeof(double)));
    RC(alloc((void**)&p->ts_part, (size_t)batch * ts_blocks(p->holo) * 2 * sizeof(double)));
    if (const char* e = std::getenv("SLM_TRACE_BUF"); e && std::atoi(e) && !generic) {
        RC(alloc((void**)&p->trace_col, (size_t)batch * max_nwg * kTraceSlots * sizeof(unsigned long long)));
        RC(alloc((void**)&p->trace_row, (size_t)batch * (height / min_rpw) * kTraceSlots * sizeof(unsigned long long)));
    }
    p->generic = generic;
    if (generic) {
        if (int rc = generic_create(gview(p), &p->gen)) {
            free_plan(p);
            return rc;
        }
    }
    *out = p;
    return 0;
}

}  // namespace

extern "C" {

int slm_plan_read_trace(slm_plan* p, int kernel_class, unsigned long long* out) {
    if (!p || !out) return fail(SLM_ERR_ARG, "null argument");
    unsigned long long* src = kernel_class == SLM_KERNEL_COL_MAIN ? p->trace_col
                              : kernel_class == SLM_KERNEL_ROW_MAIN ? p->trace_row : nullptr;
    if (!src) return fail(SLM_ERR_STATE, "no trace buffer (set SLM_TRACE_BUF=1 before creating the plan)");
    const long long n = (long long)p->B * (kernel_class == SLM_KERNEL_COL_MAIN ? p->nwg : p->H / p->rpw) * kTraceSlots;
    HIP_TRY(hipStreamSynchronize(p->stream));
    RC(copy_sync(out, src, n * sizeof(unsigned long long), hipMemcpyDeviceToHost, p->stream));
    return 0;
}

int slm_plan_destroy(slm_plan* plan) {
    free_plan(plan);
    return 0;
}

int slm_plan_set_target(slm_plan* p, const void* tgt) {
    if (!p || !tgt) return fail(SLM_ERR_ARG, "null argument");
    if (p->generic && !p->gen) return fail(SLM_ERR_STATE, "the plan lost its engine (failed slm_plan_set_precision)");
    HIP_TRY(hipSetDevice(p->device));
    const long long n = (long long)p->B * p->holo;
    const size_t tb = p->tt == SLM_TGT_U8 ? 1 : 4;
    void* stage = p->gen ? p->tgt : p->e_out;  // generic plans keep the row-major target as uploaded
    // host arrays stay pageable: HIP's staged copies run at ~45 GB/s for a 4 MB
    // target here; pinning the caller's buffer or a pinned staging buffer plus a
    // host memcpy measured no faster (tools/xfer_probe.py)
    HIP_TRY(hipMemcpyAsync(stage, tgt, (size_t)n * tb, hipMemcpyHostToDevice, p->stream));
    const int nblk = ts_blocks(p->holo);
    if (p->gen) {
        if (p->tt == SLM_TGT_U8)
            hipLaunchKernelGGL(target_stats_partial_kernel<uint8_t>, dim3(nblk, p->B), dim3(kTsThreads), 0,
                               p->stream, (const uint8_t*)stage, p->holo, p->ts_part);
        else
            hipLaunchKernelGGL(target_stats_partial_kernel<float>, dim3(nblk, p->B), dim3(kTsThreads), 0,
                               p->stream, (const float*)stage, p->holo, p->ts_part);
    } else if (p->tt == SLM_TGT_U8) {
        hipLaunchKernelGGL(target_stats_partial_kernel<uint8_t>, dim3(nblk, p->B), dim3(kTsThreads), 0, p->stream,
                           (const uint8_t*)stage, p->holo, p->ts_part);
        RC(relayout(layout_x_log2(p->lid), (const uint8_t*)stage, (uint8_t*)p->tgt, n, p->H, p->W, true, p->stream));
    } else {
        hipLaunchKernelGGL(target_stats_partial_kernel<float>, dim3(nblk, p->B), dim3(kTsThreads), 0, p->stream,
                           (const float*)stage, p->holo, p->ts_part);
        if (p->dev_tt == TGT_AMP) {  // a_T = sqrt(T) in the blocked layout (H, W multiples of 64)
            const int xl = layout_x_log2(p->lid);
            auto k = xl == 1 ? tile_relayout_kernel<float, 1, true, true>
                     : xl == 3 ? tile_relayout_kernel<float, 3, true, true>
                     : xl == 4 ? tile_relayout_kernel<float, 4, true, true> : tile_relayout_kernel<float, 2, true, true>;
            hipLaunchKernelGGL(k, dim3(p->W / 64, p->H / 64, p->B), dim3(256), 0, p->stream, (const float*)stage,
                               (float*)p->tgt, p->H, p->W);
        } else {
            RC(relayout(layout_x_log2(p->lid), (const float*)stage, (float*)p->tgt, n, p->H, p->W, true, p->stream));
        }
    }
    hipLaunchKernelGGL(target_stats_final_kernel, dim3(p->B), dim3(kTsThreads), 0, p->stream, p->ts_part, nblk,
                       p->norm, p->normf, p->sum_t2);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipStreamSynchronize(p->stream));
    p->target_set = true;
    return 0;
}

int slm_plan_set_precision(slm_plan* p, int precision) {
    if (!p) return fail(SLM_ERR_ARG, "null plan");
    if (precision != SLM_PRECISION_F32 && precision != SLM_PRECISION_F64)
        return fail(SLM_ERR_ARG, "unknown precision %d", precision);
    HIP_TRY(hipSetDevice(p->device));
    if (p->gen) {  // any-size engine: rebuilt when the precision it runs at changes
        const int prec = generic_precision(p->B, p->H, p->W, p->algo, precision);
        if (prec == p->prec) return 0;
        HIP_TRY(hipStreamSynchronize(p->stream));
        if (p->gexec) {  // the captured run holds the old engine's kernels and buffers
            HIP_TRY(hipGraphExecDestroy(p->gexec));
            p->gexec = nullptr;
        }
        const int old_prec = p->prec, old_nwg = p->nwg;
        generic_destroy(p->gen);
        p->gen = nullptr;
        p->prec = prec;
        p->nwg = generic_nwg(p->B, p->H, p->W, p->holo, p->algo, prec);
        const int rc = generic_create(gview(p), &p->gen);
        if (rc) {  // keep a usable plan: the engine it had (its error stays the reported one)
            p->prec = old_prec;
            p->nwg = old_nwg;
            const std::string msg = slm_last_error();
            if (generic_create(gview(p), &p->gen)) p->gen = nullptr;
            return fail(rc, "%s", msg.c_str());
        }
        return 0;
    }
    RC(configure(p, precision));
    return 0;
}

int slm_plan_get_precision(slm_plan* p) { return p ? p->prec : -1; }

int slm_plan_set_ain(slm_plan* p, const float* ain) {
    if (!p || !ain) return fail(SLM_ERR_ARG, "null argument");
    if (!p->has_ain) return fail(SLM_ERR_STATE, "plan was created without an incoming amplitude");
    HIP_TRY(hipSetDevice(p->device));
    // Uploads go on the plan stream: the plan's non-blocking stream is not
    // ordered after null-stream copies, and a pageable hipMemcpy may return
    // before its DMA has landed.
    HIP_TRY(hipMemcpyAsync(p->ain, ain, (size_t)p->holo * sizeof(float), hipMemcpyHostToDevice, p->stream));
    HIP_TRY(hipStreamSynchronize(p->stream));
    return 0;
}

int slm_plan_set_phase(slm_plan* p, const float* phase) {
    if (!p) return fail(SLM_ERR_ARG, "null plan");
    if (p->algo != SLM_ALGO_GS) return fail(SLM_ERR_STATE, "initial phase applies to GS plans");
    HIP_TRY(hipSetDevice(p->device));
    if (!phase) {
        p->phase_set = false;
        return 0;
    }
    const size_t bytes = (size_t)p->B * p->holo * sizeof(float);
    if (!p->phase_in) HIP_TRY(hipMalloc((void**)&p->phase_in, bytes));
    HIP_TRY(hipMemcpyAsync(p->phase_in, phase, bytes, hipMemcpyHostToDevice, p->stream));
    HIP_TRY(hipStreamSynchronize(p->stream));
    p->phase_set = true;
    return 0;
}

int slm_plan_set_field(slm_plan* p, const float* field) {
    if (!p) return fail(SLM_ERR_ARG, "null plan");
    if (p->algo != SLM_ALGO_GD) return fail(SLM_ERR_STATE, "initial field applies to GD plans");
    HIP_TRY(hipSetDevice(p->device));
    if (!field) {
        p->field_set = false;
        return 0;
    }
    const long long n = (long long)p->B * p->holo;
    if (p->gen) {
        HIP_TRY(hipMemcpyAsync(p->field0, field, (size_t)n * sizeof(float2), hipMemcpyHostToDevice, p->stream));
    } else {
        HIP_TRY(hipMemcpyAsync(p->y, field, (size_t)n * sizeof(float2), hipMemcpyHostToDevice, p->stream));
        RC(relayout(layout_y_log2(p->lid), (const float2*)p->y, p->field0, n, p->H, p->W, true, p->stream));
    }
    HIP_TRY(hipStreamSynchronize(p->stream));
    p->field_set = true;
    p->field_fresh = true;
    return 0;
}

int slm_plan_set_lr(slm_plan* p, const float* lr) {
    if (!p || !lr) return fail(SLM_ERR_ARG, "null argument");
    if (p->algo != SLM_ALGO_GD) return fail(SLM_ERR_STATE, "learning rates apply to GD plans");
    HIP_TRY(hipSetDevice(p->device));
    HIP_TRY(hipMemcpyAsync(p->lr, lr, (size_t)p->max_loops * sizeof(float), hipMemcpyHostToDevice, p->stream));
    HIP_TRY(hipStreamSynchronize(p->stream));
    p->lr_set = true;
    return 0;
}

int slm_plan_run(slm_plan* p, int loops, double tol, int checked, float wa) {
    if (p) {
        p->timing = false;
        p->field_fresh = false;  // replays skip enqueue_run
        p->last_loops = loops;
        p->last_tol = tol;
        p->last_checked = checked;
        p->last_wa = wa;
    }
    static const bool use_graph = [] {
        const char* e = std::getenv("SLM_GRAPH");
        return !e || std::atoi(e) != 0;
    }();
    if (!p || !use_graph || generic_uses_blas(p->gen)) {  // rocBLAS calls: not captured
        RC(enqueue_run(p, loops, tol, checked, wa));
        if (p && p->gfault && gd_fused_fn(p, checked)) p->fused_pending = true;
        return 0;
    }
    const int state = (p->phase_set ? 1 : 0) | (p->field_set ? 2 : 0);
    if (!p->gexec || p->g_state != state || p->g_loops != loops || p->g_tol != tol || p->g_checked != checked || p->g_wa != wa) {
        HIP_TRY(hipSetDevice(p->device));
        if (p->gexec) {
            // runs are asynchronous: a replay of this exec may still be queued
            HIP_TRY(hipStreamSynchronize(p->stream));
            HIP_TRY(hipGraphExecDestroy(p->gexec));
            p->gexec = nullptr;
        }
        HIP_TRY(hipStreamBeginCapture(p->stream, hipStreamCaptureModeThreadLocal));
        int rc = enqueue_run(p, loops, tol, checked, wa);
        hipGraph_t g = nullptr;
        hipError_t e = hipStreamEndCapture(p->stream, &g);
        if (rc) {
            if (g) (void)hipGraphDestroy(g);
            return rc;
        }
        HIP_TRY(e);
        e = hipGraphInstantiate(&p->gexec, g, nullptr, nullptr, 0);
        (void)hipGraphDestroy(g);
        HIP_TRY(e);
        p->g_loops = loops;
        p->g_tol = tol;
        p->g_checked = checked;
        p->g_wa = wa;
        p->g_state = state;
    }
    HIP_TRY(hipSetDevice(p->device));
    HIP_TRY(hipGraphLaunch(p->gexec, p->stream));
    if (p->gfault && gd_fused_fn(p, checked)) p->fused_pending = true;
    return 0;
}

int slm_plan_run_timed(slm_plan* p, int loops, double tol, int checked, float wa, double* us, int* counts) {
    if (!p) return fail(SLM_ERR_ARG, "null plan");
    // $SLM_TIMED_HOLD: 100 MHz ticks of hold per launch of the run (0 = no hold)
    static const long long hold = [] {
        const char* e = std::getenv("SLM_TIMED_HOLD");
        return e ? std::atoll(e) : 1000LL;
    }();
    if (hold > 0) {
        // ~10 us of host enqueue per launch of the run, at most 0.2 s
        const long long launches = 2LL * loops + 16;
        const unsigned long long ticks = (unsigned long long)std::min<long long>(launches * hold, 20000000LL);
        HIP_TRY(hipSetDevice(p->device));
        hipLaunchKernelGGL(hold_kernel, dim3(1), dim3(64), 0, p->stream, ticks);
        HIP_TRY(hipGetLastError());
    }
    p->timing = true;
    p->ev_used = 0;
    int rc = enqueue_run(p, loops, tol, checked, wa);
    p->timing = false;
    if (rc) return rc;
    HIP_TRY(hipStreamSynchronize(p->stream));
    bool faulted = false;
    RC(recover_grid_fault(p, &faulted));
    if (faulted) return slm_plan_run_timed(p, loops, tol, checked, wa, us, counts);  // now on two launches
    for (int k = 0; k < SLM_NUM_KERNEL_CLASSES; ++k) {
        if (us) us[k] = 0.0;
        if (counts) counts[k] = 0;
    }
    for (size_t i = 0; i < p->ev_used; ++i) {
        float ms = 0.f;
        HIP_TRY(hipEventElapsedTime(&ms, p->ev_pool[i].first, p->ev_pool[i].second));
        const int c = p->ev_class[i];
        if (us) us[c] += 1000.0 * ms;
        if (counts) counts[c] += 1;
    }
    return 0;
}

int slm_plan_sync(slm_plan* p) {
    if (!p) return fail(SLM_ERR_ARG, "null plan");
    HIP_TRY(hipSetDevice(p->device));
    HIP_TRY(hipStreamSynchronize(p->stream));
    if (p->comm_stream) HIP_TRY(hipStreamSynchronize(p->comm_stream));  // queued gathers
    bool faulted = false;
    RC(recover_grid_fault(p, &faulted));
    if (faulted) {  // the last run again, on the two-launch column side (cannot fault)
        RC(slm_plan_run(p, p->last_loops, p->last_tol, p->last_checked, p->last_wa));
        HIP_TRY(hipStreamSynchronize(p->stream));
    }
    return 0;
}

int slm_plan_gd_recoveries(slm_plan* p) { return p ? p->gd_recoveries : -1; }

int slm_plan_mark(slm_plan* p, int which) {
    if (!p || which < 0 || which > 1) return fail(SLM_ERR_ARG, "bad mark arguments");
    HIP_TRY(hipSetDevice(p->device));
    if (!p->marks[which]) HIP_TRY(hipEventCreate(&p->marks[which]));
    // the stopwatch covers the gathers queued on the comm stream too
    if (p->gather_last >= 0) HIP_TRY(hipStreamWaitEvent(p->stream, p->gather_done[p->gather_last], 0));
    HIP_TRY(hipEventRecord(p->marks[which], p->stream));
    return 0;
}

int slm_plan_marked_ms(slm_plan* p, double* ms) {
    if (!p || !ms) return fail(SLM_ERR_ARG, "null argument");
    if (!p->marks[0] || !p->marks[1]) return fail(SLM_ERR_STATE, "record marks 0 and 1 first");
    HIP_TRY(hipEventSynchronize(p->marks[1]));
    float t = 0.f;
    HIP_TRY(hipEventElapsedTime(&t, p->marks[0], p->marks[1]));
    *ms = t;
    return 0;
}

int slm_plan_read(slm_plan* p, float* phase, float* expected, double* stats, int* iters) {
    if (!p) return fail(SLM_ERR_ARG, "null plan");
    RC(slm_plan_sync(p));
    const size_t n = (size_t)p->B * p->holo;
    if (phase) RC(copy_sync(phase, p->phase_out, n * sizeof(float), hipMemcpyDeviceToHost, p->stream));
    if (expected) RC(copy_sync(expected, p->e_out, n * sizeof(float), hipMemcpyDeviceToHost, p->stream));
    if (stats)
        RC(copy_sync(stats, p->stats, (size_t)p->B * p->max_loops * 4 * sizeof(double),
                          hipMemcpyDeviceToHost, p->stream));
    if (iters) {
        std::vector<int> st(p->B);
        RC(copy_sync(st.data(), p->stop, (size_t)p->B * sizeof(int), hipMemcpyDeviceToHost, p->stream));
        for (int b = 0; b < p->B; ++b) iters[b] = st[b] == INT_MAX ? -1 : st[b] + 1;  // -1: ran all loops
    }
    return 0;
}

int slm_plan_read_target_stats(slm_plan* p, double* norm, double* sum_t2) {
    if (!p) return fail(SLM_ERR_ARG, "null plan");
    HIP_TRY(hipSetDevice(p->device));
    HIP_TRY(hipStreamSynchronize(p->stream));
    if (norm) RC(copy_sync(norm, p->norm, (size_t)p->B * sizeof(double), hipMemcpyDeviceToHost, p->stream));
    if (sum_t2) RC(copy_sync(sum_t2, p->sum_t2, (size_t)p->B * sizeof(double), hipMemcpyDeviceToHost, p->stream));
    return 0;
}

int slm_plan_set_target_stats(slm_plan* p, const double* norm, const double* sum_t2) {
    if (!p || !norm || !sum_t2) return fail(SLM_ERR_ARG, "null argument");
    if (!p->target_set) return fail(SLM_ERR_STATE, "target not set");
    HIP_TRY(hipSetDevice(p->device));
    std::vector<float> nf(p->B);
    for (int b = 0; b < p->B; ++b) nf[b] = (float)norm[b];
    HIP_TRY(hipMemcpyAsync(p->norm, norm, (size_t)p->B * sizeof(double), hipMemcpyHostToDevice, p->stream));
    HIP_TRY(hipMemcpyAsync(p->normf, nf.data(), (size_t)p->B * sizeof(float), hipMemcpyHostToDevice, p->stream));
    HIP_TRY(hipMemcpyAsync(p->sum_t2, sum_t2, (size_t)p->B * sizeof(double), hipMemcpyHostToDevice, p->stream));
    HIP_TRY(hipStreamSynchronize(p->stream));
    return 0;
}

long long slm_plan_kernel_bytes(slm_plan* p, int cls) {
    if (!p) return -1;
    const long long px = (long long)p->B * p->holo;
    const long long tb = p->tt == SLM_TGT_U8 ? 1 : 4;
    const long long ab = p->has_ain ? 4 : 0;
    if (p->gen) {
        if (generic_kind(p->gen) == 2) return 0;  // line transforms: no column / row kernel classes
        // mixed radix / radix plans, complex128 state (complex64: z = 8): column pass
        // in z + T + out z (GD statistics: in + T); row pass in z + out z (+ a_in)
        // (+ GD field read and write 2z)
        const long long z = p->prec == PREC_F32 ? 8 : 16;
        switch (cls) {
            case SLM_KERNEL_COL_MAIN: return px * (2 * z + tb);
            case SLM_KERNEL_ROW_MAIN: return px * (2 * z + ab + (p->algo == SLM_ALGO_GD ? 2 * z : 0));
            case SLM_KERNEL_GD_STATS: return px * (z + tb);
            default: return 0;
        }
    }
    const bool lin = p->algo == SLM_ALGO_GD && p->gd_mode == GD_LIN;  // + Y2 out (column) / in (row)
    switch (cls) {
        case SLM_KERNEL_COL_MAIN: return px * (8 + tb + 8 + (lin ? 8 : 0));  // X (GD: F) in, T in, Y out
        case SLM_KERNEL_ROW_MAIN:                                 // Y in, X out (+ a_in) (+ field r/w for GD)
            return px * (16 + ab + (p->algo == SLM_ALGO_GD ? 16 : 0) + (lin ? 8 : 0));
        case SLM_KERNEL_GD_STATS: return px * (8 + tb);           // X in, T in
        default: return 0;
    }
}

int slm_plan_info(slm_plan* p, int* info) {
    if (!p || !info) return fail(SLM_ERR_ARG, "null argument");
    info[0] = p->cw;
    info[1] = p->nwg;
    info[2] = p->col_threads;
    info[3] = p->row_threads;
    info[4] = p->rpw;
    info[5] = p->row_key;
    info[6] = p->col_key;
    info[7] = p->prec;
    return 0;
}

int slm_plan_engine(slm_plan* p, int* col_engine, int* row_engine) {
    if (!p || !col_engine || !row_engine) return fail(SLM_ERR_ARG, "null argument");
    // mirrors kernels.hpp: kShuffle<K, P> && (CW == 2 | RPW == 2) && one line per thread
    if (p->gen) {
        *col_engine = *row_engine = generic_kind(p->gen);  // line transforms / mixed radix / radix plans (generic.hpp)
        return 0;
    }
    auto shuf = [&](int key, int prec) {
        return (prec == PREC_F32 || p->algo == SLM_ALGO_GS) && key >= 0 && kPlans[key].n == kShufN &&
               kPlans[key].e == 8;
    };
    *col_engine = shuf(p->col_key, p->prec) && p->cw == 2 ? 1 : 0;
    *row_engine = shuf(p->row_key, p->prec_row) && p->rpw == 2 ? 1 : 0;
    return 0;
}

int slm_plan_device(slm_plan* p) { return p ? p->device : -1; }

int slm_plan_layout(slm_plan* p, int* x_log2, int* y_log2) {
    if (!p || !x_log2 || !y_log2) return fail(SLM_ERR_ARG, "null argument");
    if (p->gen) {
        *x_log2 = *y_log2 = 0;  // row-major
        return 0;
    }
    *x_log2 = layout_x_log2(p->lid);
    *y_log2 = layout_y_log2(p->lid);
    return 0;
}

int slm_gs(const void* tgt, int tgt_type, const float* ain, int batch, int height, int width, int max_loops,
           double tol, const float* init_phase, float* out_phase, float* out_expected, double* out_stats,
           int* out_iters) {
    slm_plan* p = nullptr;
    RC(slm_plan_create(SLM_ALGO_GS, batch, height, width, tgt_type, ain != nullptr, max_loops, &p));
    int rc = slm_plan_set_target(p, tgt);
    if (!rc && ain) rc = slm_plan_set_ain(p, ain);
    if (!rc && init_phase) rc = slm_plan_set_phase(p, init_phase);
    if (!rc) rc = slm_plan_run(p, max_loops, tol, tol > 0.0 ? 1 : 0, 0.f);
    if (!rc) rc = slm_plan_read(p, out_phase, out_expected, out_stats, out_iters);
    free_plan(p);
    return rc;
}

int slm_gd(const void* tgt, int tgt_type, const float* ain, int batch, int height, int width, int max_loops,
           double tol, const float* init_field, const float* lr, float wa, float* out_phase, float* out_expected,
           double* out_stats, int* out_iters) {
    slm_plan* p = nullptr;
    RC(slm_plan_create(SLM_ALGO_GD, batch, height, width, tgt_type, ain != nullptr, max_loops, &p));
    int rc = slm_plan_set_target(p, tgt);
    if (!rc && ain) rc = slm_plan_set_ain(p, ain);
    if (!rc && init_field) rc = slm_plan_set_field(p, init_field);
    if (!rc) rc = slm_plan_set_lr(p, lr);
    if (!rc) rc = slm_plan_run(p, max_loops, tol, tol > 0.0 ? 1 : 0, wa);
    if (!rc) rc = slm_plan_read(p, out_phase, out_expected, out_stats, out_iters);
    free_plan(p);
    return rc;
}

namespace {
// per-shard timing of the last slm_gs_multi of this process (slm_gs_multi_timing)
std::mutex g_multi_mu;
std::vector<double> g_multi_wall, g_multi_run;
}  // namespace

int slm_gs_multi_timing(int max_shards, double* wall_ms, double* run_ms) {
    std::lock_guard<std::mutex> lk(g_multi_mu);
    const int n = (int)g_multi_wall.size();
    for (int r = 0; r < n && r < max_shards; ++r) {
        if (wall_ms) wall_ms[r] = g_multi_wall[r];
        if (run_ms) run_ms[r] = g_multi_run[r];
    }
    return n;
}

int slm_gs_multi(int n_gpus, const int* devices, const void* tgt, int tgt_type, const float* ain, int batch,
                 int height, int width, int max_loops, double tol, const float* init_phase, float* out_phase,
                 float* out_expected, double* out_stats, int* out_iters) {
    if (n_gpus < 1) return fail(SLM_ERR_ARG, "n_gpus must be >= 1");
    if (!tgt || batch < 1) return fail(SLM_ERR_ARG, "need a target batch");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0)
        return fail(SLM_ERR_HIP, "no HIP device available; libslm_hip has no CPU path");
    std::vector<int> dev(n_gpus);
    for (int r = 0; r < n_gpus; ++r) {
        dev[r] = devices ? devices[r] : r;
        if (dev[r] < 0 || dev[r] >= ndev) return fail(SLM_ERR_ARG, "shard %d: device %d outside [0, %d)", r, dev[r], ndev);
    }
    // contiguous shards in batch order, the first batch % n_gpus one larger
    // (parallel.shard_counts; the same arithmetic as slm_gather_layout)
    std::vector<int> counts(n_gpus);
    for (int r = 0; r < n_gpus; ++r) counts[r] = batch / n_gpus + (r < batch % n_gpus ? 1 : 0);
    std::vector<long long> off(n_gpus + 1);
    RC(slm_gather_layout(n_gpus, counts.data(), 1, off.data()));
    const long long holo = (long long)height * width;
    const size_t tb = tgt_type == SLM_TGT_U8 ? 1 : 4;
    std::vector<int> rcs(n_gpus, 0);
    std::vector<std::string> errs(n_gpus);
    std::vector<double> wall(n_gpus, 0.0), run(n_gpus, 0.0);
    using clk = std::chrono::steady_clock;
    auto ms_since = [](clk::time_point t0) { return std::chrono::duration<double, std::milli>(clk::now() - t0).count(); };
    auto shard = [&](int r) {
        if (!counts[r]) return;
        const auto t0 = clk::now();
        const long long h0 = off[r];
        slm_plan* p = nullptr;
        int rc = plan_create_on(dev[r], SLM_ALGO_GS, counts[r], height, width, tgt_type, ain != nullptr, max_loops,
                                &p);
        if (!rc) rc = slm_plan_set_target(p, static_cast<const char*>(tgt) + (size_t)h0 * holo * tb);
        if (!rc && ain) rc = slm_plan_set_ain(p, ain);
        if (!rc && init_phase) rc = slm_plan_set_phase(p, init_phase + h0 * holo);
        const auto t1 = clk::now();
        if (!rc) rc = slm_plan_run(p, max_loops, tol, tol > 0.0 ? 1 : 0, 0.f);
        if (!rc) rc = slm_plan_sync(p);
        run[r] = ms_since(t1);
        // each shard lands in its own slice of the caller's arrays over its GPU's own link
        if (!rc)
            rc = slm_plan_read(p, out_phase ? out_phase + h0 * holo : nullptr,
                               out_expected ? out_expected + h0 * holo : nullptr,
                               out_stats ? out_stats + h0 * (long long)max_loops * 4 : nullptr,
                               out_iters ? out_iters + h0 : nullptr);
        if (rc) errs[r] = g_err;  // thread-local message of this shard's thread
        free_plan(p);
        rcs[r] = rc;
        wall[r] = ms_since(t0);
    };
    if (n_gpus == 1) {
        shard(0);
    } else {
        std::vector<std::thread> th;
        for (int r = 0; r < n_gpus; ++r) th.emplace_back(shard, r);
        for (auto& t : th) t.join();
    }
    {
        std::lock_guard<std::mutex> lk(g_multi_mu);
        g_multi_wall = wall;
        g_multi_run = run;
    }
    for (int r = 0; r < n_gpus; ++r)
        if (rcs[r]) return fail(rcs[r], "shard %d (device %d): %s", r, dev[r], errs[r].c_str());
    return 0;
}

int slm_fft2(const float* in, float* out, int batch, int height, int width, int inverse) {
    if (!in || !out) return fail(SLM_ERR_ARG, "null argument");
    slm_plan* p = nullptr;
    RC(slm_plan_create(SLM_ALGO_GS, batch, height, width, SLM_TGT_F32, 0, 1, &p));
    const long long n = (long long)batch * p->holo;
    const size_t bytes = (size_t)n * sizeof(float2);
    int rc = 0;
    if (p->gen) {  // any-size engine: row-major in place through the staging buffer
        hipError_t e = hipMemcpyAsync(p->xa, in, bytes, hipMemcpyHostToDevice, p->stream);
        if (e != hipSuccess) rc = fail(SLM_ERR_HIP, "upload failed: %s", hipGetErrorString(e));
        if (!rc) rc = generic_fft2(p->gen, gview(p), p->xa, p->xa, inverse);
        if (!rc) rc = copy_sync(out, p->xa, bytes, hipMemcpyDeviceToHost, p->stream);
        free_plan(p);
        return rc;
    }
    hipError_t e = hipMemcpyAsync(p->y, in, bytes, hipMemcpyHostToDevice, p->stream);
    if (e != hipSuccess) rc = fail(SLM_ERR_HIP, "upload failed: %s", hipGetErrorString(e));
    if (!rc) rc = relayout(layout_y_log2(p->lid), (const float2*)p->y, p->xa, n, height, width, true, p->stream);  // row-pass input
    if (!rc) {
        RowParams rp = row_params(p);
        rp.in = p->xa;
        rp.out = p->y;
        rc = launch_row(p, inverse ? ROW_FFT_INV : ROW_FFT_FWD, rp, SLM_KERNEL_OTHER);
    }
    if (!rc) {
        ColParams cp = col_params(p);
        cp.in = p->y;
        cp.out = p->xa;
        rc = launch_col(p, inverse ? COL_FFT_INV : COL_FFT_FWD, cp, SLM_KERNEL_OTHER);
    }
    if (!rc) rc = relayout(layout_y_log2(p->lid), (const float2*)p->xa, p->y, n, height, width, false, p->stream);  // col-pass output
    if (!rc) {
        e = hipStreamSynchronize(p->stream);
        if (e == hipSuccess) e = hipMemcpyAsync(out, p->y, bytes, hipMemcpyDeviceToHost, p->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(p->stream);
        if (e != hipSuccess) rc = fail(SLM_ERR_HIP, "fft2 failed: %s", hipGetErrorString(e));
    }
    free_plan(p);
    return rc;
}

}  // extern "C"

namespace {
// slm_fft2_c128's float64 engines, cached per (device, batch, h, w) like the
// drop-in's plans: move_traps.update_hologram calls it for every non-blank
// image of the interactive trap loop, which rebuilt stream, buffers, line
// plans and tables each time before r06. A few shapes are kept (oldest out);
// slm_release_caches frees them (algorithms.clear_plans).
struct C128Entry {
    int device = 0, batch = 0, h = 0, w = 0;
    slm_plan* q = nullptr;  // scratch GS view: its stream and engine only
    double2* buf = nullptr;
};
std::mutex g_c128_mu;
std::vector<C128Entry> g_c128;
constexpr size_t kC128CacheMax = 4;

void c128_free(C128Entry& e) {
    if (e.buf) (void)hipFree(e.buf);
    e.buf = nullptr;
    free_plan(e.q);  // waits for its stream, frees the engine
    e.q = nullptr;
}

int c128_entry(int batch, int height, int width, C128Entry** out) {
    for (auto& e : g_c128)
        if (e.device == g_device && e.batch == batch && e.h == height && e.w == width) {
            *out = &e;
            return 0;
        }
    if (g_c128.size() >= kC128CacheMax) {
        (void)hipSetDevice(g_c128.front().device);
        c128_free(g_c128.front());
        g_c128.erase(g_c128.begin());
        HIP_TRY(hipSetDevice(g_device));
    }
    C128Entry e;
    e.device = g_device;
    e.batch = batch;
    e.h = height;
    e.w = width;
    e.q = new slm_plan();
    slm_plan& q = *e.q;
    q.algo = SLM_ALGO_GS;
    q.B = batch;
    q.H = height;
    q.W = width;
    q.holo = (long long)height * width;
    q.max_loops = 1;
    q.prec = PREC_F64;
    q.nwg = generic_nwg(batch, height, width, q.holo, SLM_ALGO_GS, PREC_F64);
    q.device = g_device;
    int rc = 0;
    if (hipStreamCreateWithFlags(&q.stream, hipStreamNonBlocking) != hipSuccess)
        rc = fail(SLM_ERR_HIP, "fft2_c128: stream creation failed");
    const size_t bytes = (size_t)batch * q.holo * sizeof(double2);
    if (!rc && hipMalloc(&e.buf, bytes) != hipSuccess) rc = fail(SLM_ERR_HIP, "fft2_c128: allocation of %zu bytes", bytes);
    if (!rc) rc = generic_create(gview(&q), &q.gen);
    if (rc) {
        c128_free(e);
        return rc;
    }
    g_c128.push_back(e);
    *out = &g_c128.back();
    return 0;
}
}  // namespace

extern "C" {

int slm_fft2_c128(const double* in, double* out, int batch, int height, int width, int inverse) {
    if (!in || !out) return fail(SLM_ERR_ARG, "null argument");
    if (batch < 1 || height < 1 || width < 1) return fail(SLM_ERR_ARG, "shape %d x %d x %d", batch, height, width);
    RC(ensure_device());
    HIP_TRY(hipSetDevice(g_device));
    // the float64 engine of the any-size plans (radix-plan kernels on 2^k / 768
    // sides, mixed radix where the sides factor, else chirp-z line
    // transforms), whatever the shape, cached per shape
    std::lock_guard<std::mutex> lk(g_c128_mu);
    C128Entry* e = nullptr;
    RC(c128_entry(batch, height, width, &e));
    slm_plan& q = *e->q;
    const size_t bytes = (size_t)batch * q.holo * sizeof(double2);
    if (hipMemcpyAsync(e->buf, in, bytes, hipMemcpyHostToDevice, q.stream) != hipSuccess)
        return fail(SLM_ERR_HIP, "fft2_c128: upload failed");
    RC(generic_fft2_z(q.gen, gview(&q), e->buf, e->buf, inverse));
    return copy_sync(out, e->buf, bytes, hipMemcpyDeviceToHost, q.stream);
}

int slm_release_caches(void) {
    std::lock_guard<std::mutex> lk(g_c128_mu);
    int dev = 0;
    const bool have = hipGetDevice(&dev) == hipSuccess;
    for (auto& e : g_c128) {
        (void)hipSetDevice(e.device);
        c128_free(e);
    }
    g_c128.clear();
    if (have) (void)hipSetDevice(dev);
    return 0;
}

int slm_fft2_intensity(const float* phase, int batch, int height, int width, float* intensity_out) {
    if (!phase || !intensity_out) return fail(SLM_ERR_ARG, "null argument");
    slm_plan* p = nullptr;
    RC(slm_plan_create(SLM_ALGO_GS, batch, height, width, SLM_TGT_F32, 0, 1, &p));
    int rc = slm_plan_set_phase(p, phase);
    if (!rc && p->gen) {
        rc = generic_intensity(p->gen, gview(p), p->phase_in, p->e_out);
    } else if (!rc) {
        // fft2(exp(1j phase)) = column FFT of the row-transformed field; |.|^2 row-major
        RowParams rp = row_params(p);
        rp.out = p->xa;
        rc = launch(p, SLM_KERNEL_OTHER, fill_int_kernel, dim3((p->B + 255) / 256), dim3(256), p->stop, p->B,
                    (int)INT_MAX);
        if (!rc) rc = launch_row(p, ROW_PHASE_FWD, rp, SLM_KERNEL_OTHER);
        ColParams cp = col_params(p);
        cp.loops = 1;
        cp.in = p->xa;
        cp.in_alt = p->xa;
        if (!rc) rc = launch_expected(p, cp);
    }
    if (!rc) rc = slm_plan_read(p, nullptr, intensity_out, nullptr, nullptr);
    free_plan(p);
    return rc;
}

int slm_plan_read_field(slm_plan* p, float* field) {
    if (!p || !field) return fail(SLM_ERR_ARG, "null argument");
    if (p->algo != SLM_ALGO_GD) return fail(SLM_ERR_STATE, "the field is the state of GD plans");
    HIP_TRY(hipSetDevice(p->device));
    if (!p->field_fresh && !p->ran) return fail(SLM_ERR_STATE, "no field yet: neither set_field nor a run");
    const long long n = (long long)p->B * p->holo;
    if (p->gen) {
        const float2* src = p->field0;
        if (!p->field_fresh) {
            RC(generic_field(p->gen, gview(p), p->xa));
            src = p->xa;
        }
        RC(copy_sync(field, src, (size_t)n * sizeof(float2), hipMemcpyDeviceToHost, p->stream));
        return 0;
    }
    // p->y is scratch between runs (every run rewrites it before reading it); a
    // field set since the last run is read back from field0 (runs never write it)
    const float2* src = p->field_fresh ? p->field0 : p->field;
    RC(relayout(layout_y_log2(p->lid), src, p->y, n, p->H, p->W, false, p->stream));
    HIP_TRY(hipStreamSynchronize(p->stream));
    RC(copy_sync(field, p->y, (size_t)n * sizeof(float2), hipMemcpyDeviceToHost, p->stream));
    return 0;
}

int slm_comm_unique_id(unsigned char* id128) {
    if (!id128) return fail(SLM_ERR_ARG, "null argument");
    ncclUniqueId id;
    NCCL_TRY(ncclGetUniqueId(&id));
    std::memcpy(id128, id.internal, NCCL_UNIQUE_ID_BYTES);
    return 0;
}

int slm_comm_init(int nranks, int rank, const unsigned char* id128) {
    if (!id128 || nranks < 1 || rank < 0 || rank >= nranks) return fail(SLM_ERR_ARG, "bad communicator arguments");
    RC(ensure_device());
    if (g_comm) {
        ncclCommDestroy(g_comm);
        g_comm = nullptr;
    }
    ncclUniqueId id;
    std::memcpy(id.internal, id128, NCCL_UNIQUE_ID_BYTES);
    NCCL_TRY(ncclCommInitRank(&g_comm, nranks, id, rank));
    g_comm_rank = rank;
    g_comm_size = nranks;
    return 0;
}

int slm_comm_destroy(void) {
    if (g_comm) {
        // device gathers return without waiting: let queued RCCL work finish first
        (void)hipDeviceSynchronize();
        ncclCommDestroy(g_comm);
        g_comm = nullptr;
    }
    return 0;
}

int slm_gather_layout(int nranks, const int* counts, long long per_item, long long* offsets) {
    if (nranks < 1 || !counts || !offsets || per_item < 0) return fail(SLM_ERR_ARG, "bad gather layout arguments");
    long long off = 0;
    for (int r = 0; r < nranks; ++r) {
        if (counts[r] < 0) return fail(SLM_ERR_ARG, "counts[%d] = %d is negative", r, counts[r]);
        offsets[r] = off;
        off += (long long)counts[r] * per_item;
    }
    offsets[nranks] = off;
    return 0;
}

}  // extern "C"

namespace {

// Gather one per-hologram slab of every rank to `root` (rank order): `src`
// holds this rank's counts[me] x per_item elements of `elem` bytes (RCCL type
// `dt`); on root the concatenation lands in *dev_buf (grown as needed) and,
// if host_out, on the host. Default: grouped ncclSend / ncclRecv (one xGMI
// hop per peer) and the root's own slab as a device copy, on the plan stream.
// Staged ($SLM_GATHER_STAGED=1): the slab is first copied into one of two
// staging buffers on the plan stream (so the next run, queued behind that
// copy, may overwrite `src`), then the comm stream -- behind an event -- moves
// it, overlapping the next run. Stream-ordered either way, no host
// synchronisation unless host_out.
int gather_slab(slm_plan* p, const void* src, long long per_item, size_t elem, ncclDataType_t dt, const int* counts,
                int root, void** dev_buf, long long* dev_cap, void* host_out) {
    if (!p || !counts) return fail(SLM_ERR_ARG, "null argument");
    HIP_TRY(hipSetDevice(p->device));
    const int n = g_comm ? g_comm_size : 1;
    const int me = g_comm ? g_comm_rank : 0;
    if (root < 0 || root >= n) return fail(SLM_ERR_ARG, "root %d outside [0, %d)", root, n);
    if (counts[me] != p->B) return fail(SLM_ERR_ARG, "counts[%d]=%d but the plan holds %d", me, counts[me], p->B);
    // a GD run on the one-launch column side may have faulted (its grid wait gave
    // up): settle it -- redo it on two launches -- before its results leave this
    // rank. Only a fused run queued since the last check can have (no host sync
    // per gather otherwise)
    if (p->fused_pending) RC(slm_plan_sync(p));
    std::vector<long long> off(n + 1);
    RC(slm_gather_layout(n, counts, per_item, off.data()));
    // $SLM_GATHER_STAGED=1: stage the slab and move it on the plan's comm stream
    // (overlaps the next run). Off by default: at 1024^2 the second stream cost
    // 0.28 ms per 200-iteration run on one GPU (272-275 against 295-296
    // holograms/s, profiles/r05/gather_ab_s7.txt), more than rank 0's wait for
    // seven 4 MB receives is expected to cost. Read per call (tests switch it).
    const char* st_env = std::getenv("SLM_GATHER_STAGED");
    const bool staged = st_env && std::atoi(st_env) != 0;
    if (!staged) {
        // a staged gather still queued on the comm stream may write the same buffer
        if (p->gather_last >= 0) HIP_TRY(hipStreamWaitEvent(p->stream, p->gather_done[p->gather_last], 0));
        p->gather_last = -1;
        if (me == root) {
            const long long elems = off[n];
            if (*dev_cap < elems) {
                HIP_TRY(hipStreamSynchronize(p->stream));
                if (*dev_buf) HIP_TRY(hipFree(*dev_buf));
                *dev_buf = nullptr;
                *dev_cap = 0;
                HIP_TRY(hipMalloc(dev_buf, std::max<long long>(elems, 1) * elem));
                *dev_cap = elems;
            }
            char* dst = static_cast<char*>(*dev_buf);
            if (n > 1) NCCL_TRY(ncclGroupStart());
            for (int r = 0; r < n; ++r) {
                const size_t cnt = (size_t)(off[r + 1] - off[r]);
                if (!cnt) continue;
                if (r == me)
                    HIP_TRY(hipMemcpyAsync(dst + off[r] * elem, src, cnt * elem, hipMemcpyDeviceToDevice, p->stream));
                else
                    NCCL_TRY(ncclRecv(dst + off[r] * elem, cnt, dt, r, g_comm, p->stream));
            }
            if (n > 1) NCCL_TRY(ncclGroupEnd());
            if (host_out && elems) {
                HIP_TRY(hipStreamSynchronize(p->stream));
                RC(copy_sync(host_out, dst, (size_t)elems * elem, hipMemcpyDeviceToHost, p->stream));
            }
        } else {
            if (!g_comm) return fail(SLM_ERR_COMM, "no communicator");
            if (p->B) NCCL_TRY(ncclSend(src, (size_t)p->B * per_item, dt, root, g_comm, p->stream));
        }
        return 0;
    }
    if (!p->comm_stream) {
        HIP_TRY(hipStreamCreateWithFlags(&p->comm_stream, hipStreamNonBlocking));
        HIP_TRY(hipEventCreateWithFlags(&p->gather_ready, hipEventDisableTiming));
        for (int k = 0; k < 2; ++k) HIP_TRY(hipEventCreateWithFlags(&p->gather_done[k], hipEventDisableTiming));
    }
    const size_t mine = (size_t)(off[me + 1] - off[me]) * elem;
    const int k = p->stage_next;
    p->stage_next ^= 1;
    if (p->stage_cap[k] < mine) {
        HIP_TRY(hipStreamSynchronize(p->comm_stream));  // nothing may still read the old buffer
        if (p->stage[k]) HIP_TRY(hipFree(p->stage[k]));
        p->stage[k] = nullptr;
        p->stage_cap[k] = 0;
        HIP_TRY(hipMalloc(&p->stage[k], mine));
        p->stage_cap[k] = mine;
    }
    // plan stream: wait for the send that last read this staging buffer, copy the slab
    if (p->gather_done_set[k]) HIP_TRY(hipStreamWaitEvent(p->stream, p->gather_done[k], 0));
    if (mine) HIP_TRY(hipMemcpyAsync(p->stage[k], src, mine, hipMemcpyDeviceToDevice, p->stream));
    HIP_TRY(hipEventRecord(p->gather_ready, p->stream));
    hipStream_t cs = p->comm_stream;
    HIP_TRY(hipStreamWaitEvent(cs, p->gather_ready, 0));
    if (me == root) {
        const long long elems = off[n];
        if (*dev_cap < elems) {
            HIP_TRY(hipStreamSynchronize(cs));  // earlier gathers into the old buffer
            if (*dev_buf) HIP_TRY(hipFree(*dev_buf));
            *dev_buf = nullptr;
            *dev_cap = 0;
            HIP_TRY(hipMalloc(dev_buf, std::max<long long>(elems, 1) * elem));
            *dev_cap = elems;
        }
        char* dst = static_cast<char*>(*dev_buf);
        if (n > 1) NCCL_TRY(ncclGroupStart());
        for (int r = 0; r < n; ++r) {
            const size_t cnt = (size_t)(off[r + 1] - off[r]);
            if (!cnt) continue;
            if (r == me) {
                HIP_TRY(hipMemcpyAsync(dst + off[r] * elem, p->stage[k], cnt * elem, hipMemcpyDeviceToDevice, cs));
            } else {
                NCCL_TRY(ncclRecv(dst + off[r] * elem, cnt, dt, r, g_comm, cs));
            }
        }
        if (n > 1) NCCL_TRY(ncclGroupEnd());
        HIP_TRY(hipEventRecord(p->gather_done[k], cs));
        p->gather_done_set[k] = true;
        p->gather_last = k;
        // a device-side gather stays stream-ordered (slm_plan_sync, a read or the
        // stopwatch wait for it); a host copy waits here
        if (host_out && elems) {
            HIP_TRY(hipStreamSynchronize(cs));
            RC(copy_sync(host_out, dst, (size_t)elems * elem, hipMemcpyDeviceToHost, cs));
        }
    } else {
        if (!g_comm) return fail(SLM_ERR_COMM, "no communicator");
        if (p->B) NCCL_TRY(ncclSend(p->stage[k], (size_t)p->B * per_item, dt, root, g_comm, cs));
        HIP_TRY(hipEventRecord(p->gather_done[k], cs));
        p->gather_done_set[k] = true;
        p->gather_last = k;
    }
    return 0;
}

}  // namespace

extern "C" {

int slm_plan_gather_phase(slm_plan* p, const int* counts, int root, float* host_out) {
    if (!p) return fail(SLM_ERR_ARG, "null plan");
    return gather_slab(p, p->phase_out, p->holo, sizeof(float), ncclFloat32, counts, root, (void**)&p->gather_buf,
                       &p->gather_elems, host_out);
}

int slm_plan_time_gather(slm_plan* p, const int* counts, int root, int reps, double* ms, long long* bytes_out) {
    if (!p || !counts || !ms || reps < 1) return fail(SLM_ERR_ARG, "bad gather-timing arguments");
    RC(slm_plan_sync(p));
    const int me = g_comm ? g_comm_rank : 0;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    HIP_TRY(hipEventCreate(&e0));
    HIP_TRY(hipEventCreate(&e1));
    int rc = 0;
    float t = 0.f;
    if (hipEventRecord(e0, p->stream) != hipSuccess) rc = fail(SLM_ERR_HIP, "event record failed");
    for (int i = 0; i < reps && !rc; ++i) rc = slm_plan_gather_phase(p, counts, root, nullptr);
    // the transfers run on the comm stream: the stop event follows the last one
    if (!rc && p->gather_last >= 0 && hipStreamWaitEvent(p->stream, p->gather_done[p->gather_last], 0) != hipSuccess)
        rc = fail(SLM_ERR_HIP, "gather timing wait failed");
    if (!rc && (hipEventRecord(e1, p->stream) != hipSuccess || hipEventSynchronize(e1) != hipSuccess ||
                hipEventElapsedTime(&t, e0, e1) != hipSuccess))
        rc = fail(SLM_ERR_HIP, "gather timing events failed");
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    if (rc) return rc;
    *ms = (double)t / reps;
    if (bytes_out) *bytes_out = me == root ? 0 : (long long)p->B * p->holo * (long long)sizeof(float);
    return 0;
}

int slm_plan_gather_stats(slm_plan* p, const int* counts, int root, double* stats_out, int* iters_out) {
    if (!p) return fail(SLM_ERR_ARG, "null plan");
    // per hologram: [max_loops][4] doubles (max E, sum E^2, sum E T, error), then the stop index
    RC(gather_slab(p, p->stats, (long long)p->max_loops * 4, sizeof(double), ncclFloat64, counts, root,
                   (void**)&p->gather_stats, &p->gather_stats_elems, stats_out));
    RC(gather_slab(p, p->stop, 1, sizeof(int), ncclInt32, counts, root, (void**)&p->gather_stop,
                   &p->gather_stop_elems, iters_out));
    if (iters_out) {  // the stop index -> iterations executed, as slm_plan_read reports it
        const int n = g_comm ? g_comm_size : 1;
        if ((g_comm ? g_comm_rank : 0) == root) {
            long long total = 0;
            for (int r = 0; r < n; ++r) total += counts[r];
            for (long long k = 0; k < total; ++k) iters_out[k] = iters_out[k] == INT_MAX ? -1 : iters_out[k] + 1;
        }
    }
    return 0;
}

}  // extern "C"
