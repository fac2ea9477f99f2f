// Device-side FFT engine for gfx950 (CDNA4): in-register small DFTs plus a
// Stockham autosort driver whose passes exchange through LDS.
//
// Data model. A line of length N is spread over T = N / E threads; thread t
// holds slot m = element (t + T * m). With that layout
//   * the first pass reads its butterfly inputs straight from the slots, so a
//     line can be loaded from HBM with lane-contiguous (coalesced) accesses;
//   * the last pass leaves its outputs in the same slot layout in natural
//     order, so results are stored coalesced and an element-wise projection can
//     run in registers between an inverse and a forward transform with no LDS
//     round trip (the fused GS/GD iteration relies on this).
// Forward = exp(-2 pi i nk/N), unscaled (scipy.fft.fft2, src/algorithms.py:31);
// inverse = exp(+2 pi i nk/N), unscaled (callers apply 1/N where needed).
//
// Precision. The arithmetic type C is float2 or double2. HBM state and LDS
// exchanges are always complex64; with C = double2 the butterflies and the
// twiddles (table computed in double on the host) run in float64, so a
// transform rounds only where it stores. Simulated on the reference's GS
// warm-start protocol (Precision) this cuts the float32 phase drift
// ~10x; the cost is FP64 VALU work and registers.
#pragma once
#include <hip/hip_runtime.h>
#include <type_traits>
#include <utility>

#include "plans.hpp"


namespace slm {

// ------------------------------------------------------------------------
// compile-time helpers
// ------------------------------------------------------------------------
template <int... Rs>
struct IntList {};

template <int I, int N, class F>
__device__ __forceinline__ void static_for_impl(F&& f) {
    if constexpr (I < N) {
        f(std::integral_constant<int, I>{});
        static_for_impl<I + 1, N>(f);
    }
}
template <int N, class F>
__device__ __forceinline__ void static_for(F&& f) {
    static_for_impl<0, N>(f);
}

// Templates below take a plan key K (index into kPlans, plans.hpp).
template <int K, std::size_t... I>
constexpr auto radices_of(std::index_sequence<I...>) {
    return IntList<kPlans[K].r[I]...>{};
}
template <int K>
using RadicesOf = decltype(radices_of<K>(std::make_index_sequence<kPlans[K].npass>{}));

template <int K>
struct PlanOf {
    static_assert(K >= 0 && K < kNumPlans, "unknown plan key");
    static constexpr int N = kPlans[K].n;
    static constexpr int E = kPlans[K].e;
    static constexpr int T = N / E;
    static constexpr int LINE = lds_line(N);
    // row stride of per-line LDS regions (LdsLine): == 16 (mod 32) complex, so
    // the two rows served by one 32-lane ds_read_b64 group hit disjoint halves
    // of the banks. Lines are XOR-swizzled, not padded (lds_slot), so the
    // region is N long.
    static constexpr int LLEN = N;
    static constexpr int ROWSTRIDE = LLEN + ((16 - LLEN % 32) + 32) % 32;
};

// cos(2 pi q / 48) for the constant twiddles of radix 2, 3, 4, 8, 12, 16.
constexpr double kCos48[13] = {1.0,
                               0.99144486137381041,
                               0.96592582628906829,
                               0.92387953251128674,
                               0.86602540378443865,
                               0.79335334029123517,
                               0.70710678118654752,
                               0.60876142900872063,
                               0.5,
                               0.38268343236508977,
                               0.25881904510252076,
                               0.13052619222005159,
                               0.0};
constexpr double cos48(int q) {
    q = ((q % 48) + 48) % 48;
    if (q <= 12) return kCos48[q];
    if (q <= 24) return -kCos48[24 - q];
    if (q <= 36) return -kCos48[q - 24];
    return kCos48[48 - q];
}
constexpr double sin48(int q) { return cos48(q - 12); }
// cos(2 pi q / 240) (correctly rounded doubles, 60-digit decimal evaluation):
// the constant twiddles of radices with a factor 5 (5, 10, 15, 20, 30, 60) --
// the mixed-radix plans of SLM panel lengths (1080, 1920, 1200, 1280, ...).
// Radices dividing 48 keep the 48ths above (their arithmetic is unchanged).
constexpr double kCos240[61] = {
                                 1.0, 0.9996573249755573, 0.9986295347545738, 0.996917333733128,
                                 0.9945218953682733, 0.9914448613738104, 0.9876883405951378, 0.9832549075639546,
                                 0.9781476007338057, 0.9723699203976766, 0.9659258262890683, 0.958819734868193,
                                 0.9510565162951535, 0.9426414910921784, 0.9335804264972017, 0.9238795325112867,
                                 0.9135454576426009, 0.9025852843498606, 0.8910065241883679, 0.8788171126619654,
                                 0.8660254037844386, 0.8526401643540922, 0.838670567945424, 0.8241261886220157,
                                 0.8090169943749475, 0.7933533402912352, 0.7771459614569709, 0.7604059656000309,
                                 0.7431448254773942, 0.7253743710122876, 0.7071067811865476, 0.688354575693754,
                                 0.6691306063588582, 0.6494480483301837, 0.6293203910498375, 0.6087614290087207,
                                 0.5877852522924731, 0.5664062369248328, 0.5446390350150271, 0.5224985647159489,
                                 0.5, 0.4771587602596084, 0.4539904997395468, 0.43051109680829514,
                                 0.4067366430758002, 0.3826834323650898, 0.35836794954530027, 0.3338068592337709,
                                 0.30901699437494745, 0.2840153447039226, 0.25881904510252074, 0.23344536385590542,
                                 0.20791169081775934, 0.18223552549214744, 0.15643446504023087, 0.1305261922200516,
                                 0.10452846326765347, 0.07845909572784494, 0.052335956242943835, 0.026176948307873153,
                                 0.0};
constexpr double cos240(int q) {
    q = ((q % 240) + 240) % 240;
    if (q <= 60) return kCos240[q];
    if (q <= 120) return -kCos240[120 - q];
    if (q <= 180) return -kCos240[q - 120];
    return kCos240[240 - q];
}
constexpr double sin240(int q) { return cos240(q - 60); }

// ------------------------------------------------------------------------
// complex helpers; C = float2 or double2
// ------------------------------------------------------------------------
template <class C>
using Scalar = std::remove_reference_t<decltype(C{}.x)>;

template <class C>
__device__ __forceinline__ C mk(Scalar<C> x, Scalar<C> y) {
    C r;
    r.x = x;
    r.y = y;
    return r;
}
template <class C>
__device__ __forceinline__ C cadd(C a, C b) { return mk<C>(a.x + b.x, a.y + b.y); }
template <class C>
__device__ __forceinline__ C csub(C a, C b) { return mk<C>(a.x - b.x, a.y - b.y); }
template <class C>
__device__ __forceinline__ C cmul(C a, C b) { return mk<C>(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x); }
// a * conj(b)
template <class C>
__device__ __forceinline__ C cmulc(C a, C b) { return mk<C>(a.x * b.x + a.y * b.y, a.y * b.x - a.x * b.y); }

// complex64 storage <-> compute type
template <class C>
__device__ __forceinline__ C from_c64(float2 v) { return mk<C>((Scalar<C>)v.x, (Scalar<C>)v.y); }
template <class C>
__device__ __forceinline__ float2 to_c64(C v) { return make_float2((float)v.x, (float)v.y); }

// Multiply by the constant twiddle w_R^K (forward: exp(-2 pi i K/R)).
template <int K, int R, bool INV, class C>
__device__ __forceinline__ C twc(C a) {
    using S = Scalar<C>;
    if constexpr (48 % R == 0) {
        constexpr int q = ((48 / R) * K) % 48;
        if constexpr (q == 0) {
            return a;
        } else if constexpr (q == 24) {
            return mk<C>(-a.x, -a.y);
        } else if constexpr (q == 12) {  // forward: * (-i)
            return INV ? mk<C>(-a.y, a.x) : mk<C>(a.y, -a.x);
        } else if constexpr (q == 36) {  // forward: * (+i)
            return INV ? mk<C>(a.y, -a.x) : mk<C>(-a.y, a.x);
        } else {
            constexpr S c = (S)cos48(q);
            constexpr S s = (S)(INV ? sin48(q) : -sin48(q));
            return mk<C>(a.x * c - a.y * s, a.x * s + a.y * c);
        }
    } else {
        static_assert(240 % R == 0, "constant twiddles of radices dividing 48 or 240");
        constexpr int q = ((240 / R) * K) % 240;
        if constexpr (q == 0) {
            return a;
        } else if constexpr (q == 120) {
            return mk<C>(-a.x, -a.y);
        } else if constexpr (q == 60) {
            return INV ? mk<C>(-a.y, a.x) : mk<C>(a.y, -a.x);
        } else if constexpr (q == 180) {
            return INV ? mk<C>(a.y, -a.x) : mk<C>(-a.y, a.x);
        } else {
            constexpr S c = (S)cos240(q);
            constexpr S s = (S)(INV ? sin240(q) : -sin240(q));
            return mk<C>(a.x * c - a.y * s, a.x * s + a.y * c);
        }
    }
}

// ------------------------------------------------------------------------
// in-register DFTs, natural order in and out
// ------------------------------------------------------------------------
template <int R, bool INV, class C>
struct Dft;

template <bool INV, class C>
struct Dft<1, INV, C> {
    __device__ __forceinline__ static void run(C*) {}
};

template <bool INV, class C>
struct Dft<2, INV, C> {
    __device__ __forceinline__ static void run(C* v) {
        const C a = v[0], b = v[1];
        v[0] = cadd(a, b);
        v[1] = csub(a, b);
    }
};

template <bool INV, class C>
struct Dft<3, INV, C> {
    __device__ __forceinline__ static void run(C* v) {
        using S = Scalar<C>;
        constexpr S h = (S)0.86602540378443865;  // sqrt(3)/2
        const C s = cadd(v[1], v[2]);
        const C d = csub(v[1], v[2]);
        const C t = mk<C>(v[0].x - (S)0.5 * s.x, v[0].y - (S)0.5 * s.y);
        // forward: (-i) * h * d ; inverse: (+i) * h * d
        const C m = INV ? mk<C>(-h * d.y, h * d.x) : mk<C>(h * d.y, -h * d.x);
        v[0] = cadd(v[0], s);
        v[1] = cadd(t, m);
        v[2] = csub(t, m);
    }
};

template <bool INV, class C>
struct Dft<4, INV, C> {
    __device__ __forceinline__ static void run(C* v) {
        const C a = cadd(v[0], v[2]);
        const C b = csub(v[0], v[2]);
        const C c = cadd(v[1], v[3]);
        const C d = twc<1, 4, INV>(csub(v[1], v[3]));
        v[0] = cadd(a, c);
        v[2] = csub(a, c);
        v[1] = cadd(b, d);
        v[3] = csub(b, d);
    }
};

// Cooley-Tukey split R = R1 * R2: n = R2 n1 + n2, k = k1 + R1 k2.
template <int R1, int R2, bool INV, class C>
__device__ __forceinline__ void dft_split(C* v) {
    constexpr int R = R1 * R2;
    C z[R];
    static_for<R2>([&](auto n2c) {
        constexpr int n2 = decltype(n2c)::value;
        C col[R1];
        static_for<R1>([&](auto n1c) {
            constexpr int n1 = decltype(n1c)::value;
            col[n1] = v[R2 * n1 + n2];
        });
        Dft<R1, INV, C>::run(col);
        static_for<R1>([&](auto k1c) {
            constexpr int k1 = decltype(k1c)::value;
            z[n2 * R1 + k1] = twc<n2 * k1, R, INV>(col[k1]);
        });
    });
    static_for<R1>([&](auto k1c) {
        constexpr int k1 = decltype(k1c)::value;
        C row[R2];
        static_for<R2>([&](auto n2c) {
            constexpr int n2 = decltype(n2c)::value;
            row[n2] = z[n2 * R1 + k1];
        });
        Dft<R2, INV, C>::run(row);
        static_for<R2>([&](auto k2c) {
            constexpr int k2 = decltype(k2c)::value;
            v[k1 + R1 * k2] = row[k2];
        });
    });
}

template <bool INV, class C>
struct Dft<8, INV, C> {
    __device__ __forceinline__ static void run(C* v) { dft_split<2, 4, INV, C>(v); }
};
// radix 5 (the mixed-radix plans): y_0 = v_0 + s_1 + s_2, s_q = v_q + v_(5-q),
// d_q = v_q - v_(5-q); y_1,4 = a_1 -/+ i b_1, y_2,3 = a_2 -/+ i b_2 (forward) with
// a_1 = v_0 + c_1 s_1 + c_2 s_2, a_2 = v_0 + c_2 s_1 + c_1 s_2,
// b_1 = n_1 d_1 + n_2 d_2, b_2 = n_2 d_1 - n_1 d_2 (c_q = cos, n_q = sin of 2 pi q / 5)
template <bool INV, class C>
struct Dft<5, INV, C> {
    __device__ __forceinline__ static void run(C* v) {
        using S = Scalar<C>;
        constexpr S c1 = (S)cos240(48), c2 = (S)cos240(96), n1 = (S)sin240(48), n2 = (S)sin240(96);
        const C s1 = cadd(v[1], v[4]), d1 = csub(v[1], v[4]);
        const C s2 = cadd(v[2], v[3]), d2 = csub(v[2], v[3]);
        const C a1 = mk<C>(v[0].x + c1 * s1.x + c2 * s2.x, v[0].y + c1 * s1.y + c2 * s2.y);
        const C a2 = mk<C>(v[0].x + c2 * s1.x + c1 * s2.x, v[0].y + c2 * s1.y + c1 * s2.y);
        const C b1 = mk<C>(n1 * d1.x + n2 * d2.x, n1 * d1.y + n2 * d2.y);
        const C b2 = mk<C>(n2 * d1.x - n1 * d2.x, n2 * d1.y - n1 * d2.y);
        // forward: -i b = (b.y, -b.x); inverse: +i b = (-b.y, b.x)
        const C j1 = INV ? mk<C>(-b1.y, b1.x) : mk<C>(b1.y, -b1.x);
        const C j2 = INV ? mk<C>(-b2.y, b2.x) : mk<C>(b2.y, -b2.x);
        v[0] = mk<C>(v[0].x + s1.x + s2.x, v[0].y + s1.y + s2.y);
        v[1] = cadd(a1, j1);
        v[4] = csub(a1, j1);
        v[2] = cadd(a2, j2);
        v[3] = csub(a2, j2);
    }
};
template <bool INV, class C>
struct Dft<6, INV, C> {
    __device__ __forceinline__ static void run(C* v) { dft_split<2, 3, INV, C>(v); }
};
template <bool INV, class C>
struct Dft<10, INV, C> {
    __device__ __forceinline__ static void run(C* v) { dft_split<2, 5, INV, C>(v); }
};
template <bool INV, class C>
struct Dft<15, INV, C> {
    __device__ __forceinline__ static void run(C* v) { dft_split<3, 5, INV, C>(v); }
};
template <bool INV, class C>
struct Dft<20, INV, C> {
    __device__ __forceinline__ static void run(C* v) { dft_split<4, 5, INV, C>(v); }
};
template <bool INV, class C>
struct Dft<24, INV, C> {
    __device__ __forceinline__ static void run(C* v) { dft_split<8, 3, INV, C>(v); }
};
template <bool INV, class C>
struct Dft<30, INV, C> {
    __device__ __forceinline__ static void run(C* v) { dft_split<6, 5, INV, C>(v); }
};
template <bool INV, class C>
struct Dft<12, INV, C> {
    __device__ __forceinline__ static void run(C* v) { dft_split<4, 3, INV, C>(v); }
};
template <bool INV, class C>
struct Dft<16, INV, C> {
    __device__ __forceinline__ static void run(C* v) { dft_split<4, 4, INV, C>(v); }
};

// ------------------------------------------------------------------------
// LDS views (complex64). A pass writes output element o and reads element
// t + T m of a line; padding one slot per 16 keeps the strided first-pass
// writes off a single bank. A thread may carry L lines (argument l), which
// share its twiddles and its exchange barriers.
// ------------------------------------------------------------------------
// X = float2 or double2: the element type of the exchange (float64 exchanges
// avoid two conversions per element and pass where the LDS budget allows).
// ALT > 0: two exchange buffers ALT elements apart, used alternately. An
// exchange then needs one barrier (write -> barrier -> read) instead of two:
// exchange k + 2 rewrites buffer k % 2 only after barrier k + 1, which every
// wave passes after its reads of exchange k completed (lgkmcnt(0)). `cur` is
// flipped in fully unrolled code from a constant start, so it folds into the
// ds_read / ds_write offsets.
// Element slot of a line in a per-line region: XOR-swizzle the low 4 index
// bits with bits 4..7 (a bijection inside each 16-element block): the pass-1
// writes (o = 16 t + r), the strided writes of later passes and the
// lane-contiguous reads (o = t + T m) all hit distinct banks in their
// 16-lane write / 32-lane read groups (tools/lds_banks.py: 4096 rows 2.0 -> 0
// extra cycles per read, 768 rows 2.0 -> 0.67 per write, nothing worse than
// one pad slot per 16, which it replaced).
__device__ __forceinline__ int lds_slot(int o) { return o ^ ((o >> 4) & 15); }

// WAVE: every line of the region is written and read by the threads of one
// wave only (wave-line mappings, kernels.hpp), so an exchange needs no
// workgroup barrier: the wave waits for its own LDS writes (lgkmcnt) and
// reads; the next pass's writes cannot pass this pass's reads (a wave's LDS
// operations execute in order).
template <class X, int ALT = 0, bool WAVE = false>
struct LdsLine {  // per-line LDS regions `stride` apart (row kernels; columns of one-group tiles)
    static constexpr bool kDouble = ALT > 0 && !WAVE;
    static constexpr bool kWave = WAVE;
    X* base;
    int stride = 0;
    mutable int cur = 0;
    __device__ __forceinline__ void flip() const { cur = ALT - cur; }
    template <class C>
    __device__ __forceinline__ void store(int l, int o, C v) const {
        base[cur + l * stride + lds_slot(o)] = mk<X>(v.x, v.y);
    }
    template <class C>
    __device__ __forceinline__ C load(int l, int o) const {
        const X v = base[cur + l * stride + lds_slot(o)];
        return mk<C>(v.x, v.y);
    }
};

template <int CW, class X, int ALT = 0, bool WAVE = false>
struct LdsTile {  // CW interleaved columns (column kernels): [o][c]; the thread's lines are c + l
    static constexpr bool kDouble = ALT > 0 && !WAVE;
    static constexpr bool kWave = WAVE;  // as LdsLine: every line's threads in one wave
    static constexpr int kCW = CW, kAlt = ALT;
    X* base;
    int c;
    mutable int cur = 0;
    __device__ __forceinline__ void flip() const { cur = ALT - cur; }
    template <class C>
    __device__ __forceinline__ void store(int l, int o, C v) const {
        base[cur + (o + (o >> 4)) * CW + c + l] = mk<X>(v.x, v.y);
    }
    template <class C>
    __device__ __forceinline__ C load(int l, int o) const {
        const X v = base[cur + (o + (o >> 4)) * CW + c + l];
        return mk<C>(v.x, v.y);
    }
    // unpadded slots (radix_c128.hpp mixed plans, exchanges whose writes are
    // lane-contiguous): the index is linear in o, so the constant part of a
    // butterfly's R outputs folds into the ds_write / ds_read offset
    template <class C>
    __device__ __forceinline__ void store_lin(int l, int o, C v) const {
        base[cur + o * CW + c + l] = mk<X>(v.x, v.y);
    }
    template <class C>
    __device__ __forceinline__ C load_lin(int l, int o) const {
        const X v = base[cur + o * CW + c + l];
        return mk<C>(v.x, v.y);
    }
};


// ------------------------------------------------------------------------
// Per-thread twiddles. Which twiddles a thread needs depends only on its
// transform-thread index t, so they can be loaded once per kernel (one global
// load each; table computed in double on the host, stored as the compute
// type) and shared by every transform the thread runs (inverse and forward
// use conjugates).
// ------------------------------------------------------------------------
template <int N, int Ns, int... Rs>
struct TwCountImpl;
template <int N, int Ns>
struct TwCountImpl<N, Ns> {
    static constexpr int value = 0;
};
template <int N, int Ns, int R, int... Rest>
struct TwCountImpl<N, Ns, R, Rest...> {
    static constexpr int value = (Ns > 1 ? (PlanOf<N>::E / R) * (R - 1) : 0) + TwCountImpl<N, Ns * R, Rest...>::value;
};
template <int N, class L>
struct TwCountOf;
template <int N, int... Rs>
struct TwCountOf<N, IntList<Rs...>> {
    static constexpr int value = TwCountImpl<N, 1, Rs...>::value;
};

// Twiddle sources (TwMode):
//  TW_CACHED: every twiddle of the thread in registers, one table load each per
//             kernel (float32 arithmetic: exact table values matter there);
//  TW_DIRECT: read from the (L1/L2-resident) table where used, for 1024-thread
//             workgroups whose 128-VGPR budget cannot hold a cache;
//  (Forming w^2.. from w^1 in registers, caching the last pass only, and
//  split radix-16 twiddles w^(4a) w^b were measured: faster variants moved
//  the 4096^2 float32 warm-start parity past the bar, slower ones were slower;
//  DESIGN.md sections 4-5.)
enum TwMode : int { TW_CACHED = 0, TW_DIRECT = 1, TW_DIRECT_LAUNDER = 2 };

template <int N, class C, int MODE>
struct Twiddles;

template <int N, class C>
struct Twiddles<N, C, TW_CACHED> {
    static constexpr bool kAlwaysLaunder = false;
    static constexpr int COUNT = TwCountOf<N, RadicesOf<N>>::value > 0 ? TwCountOf<N, RadicesOf<N>>::value : 1;
    C w[COUNT];
    __device__ __forceinline__ void launder() {}
    template <int TwOff, int RegOff, int PowOff, int R, int Ns, bool INV>
    __device__ __forceinline__ void apply(C* u, int k, int) const {
        static_for<R - 1>([&](auto rc) {
            constexpr int r = decltype(rc)::value + 1;
            const C t = w[RegOff + k * (R - 1) + r - 1];
            u[r] = INV ? cmulc(u[r], t) : cmul(u[r], t);
        });
    }
};
template <int N, class C>
struct Twiddles<N, C, TW_DIRECT> {
    static constexpr bool kAlwaysLaunder = false;
    struct alignas(2 * sizeof(Scalar<C>)) Pod {  // trivially copyable twin of C
        Scalar<C> x, y;
    };
    using GlobalPtr = const __attribute__((address_space(1))) Pod*;  // keeps global_load (not flat)
    GlobalPtr table;
    // The table is read-only, so the compiler may legally reuse the first
    // transform's twiddle loads in the second one and keep them all live in
    // between (dozens of float64 registers -> spills). Passing the pointer
    // through an empty asm before each transform makes the loads distinct.
    __device__ __forceinline__ void launder() {
        unsigned long long q = (unsigned long long)table;
        asm volatile("" : "+s"(q));
        table = (GlobalPtr)q;
    }
    template <int TwOff, int RegOff, int PowOff, int R, int Ns, bool INV>
    __device__ __forceinline__ void apply(C* u, int, int j) const {
        static_for<R - 1>([&](auto rc) {
            constexpr int r = decltype(rc)::value + 1;
            const int i = TwOff + (r - 1) * Ns + j;
            const C t = mk<C>(table[i].x, table[i].y);
            u[r] = INV ? cmulc(u[r], t) : cmul(u[r], t);
        });
    }
    // the same split in two (radix_c128.hpp mixed plans: a pass's twiddles fetched
    // before the previous exchange, applied after it)
    template <int TwOff, int R, int Ns>
    __device__ __forceinline__ void fetch(C* w, int j) const {
        static_for<R - 1>([&](auto rc) {
            constexpr int r = decltype(rc)::value + 1;
            const int i = TwOff + (r - 1) * Ns + j;
            w[r - 1] = mk<C>(table[i].x, table[i].y);
        });
    }
    template <int R, bool INV>
    __device__ __forceinline__ static void apply_fetched(C* u, const C* w) {
        static_for<R - 1>([&](auto rc) {
            constexpr int r = decltype(rc)::value + 1;
            u[r] = INV ? cmulc(u[r], w[r - 1]) : cmul(u[r], w[r - 1]);
        });
    }
};
// TW_DIRECT whose loads are laundered before every transform whatever E (the
// complex128 radix-plan kernels: a fused pair's second transform would
// otherwise keep the first one's float64 twiddle loads live across the
// element-wise epilogue -- 162 against 128 VGPRs for 4096-point E = 8 rows)
template <int N, class C>
struct Twiddles<N, C, TW_DIRECT_LAUNDER> : Twiddles<N, C, TW_DIRECT> {
    static constexpr bool kAlwaysLaunder = true;
};
template <int N, class C, int MODE, int E, int Ns, int TwOff, int RegOff, int PowOff, int R, int... Rest>
__device__ __forceinline__ void load_twiddles_pass(Twiddles<N, C, MODE>& tw, int t, const C* __restrict__ table) {
    constexpr int T = PlanOf<N>::T;  // N is the plan key here
    constexpr int NB = E / R;
    if constexpr (Ns > 1) {
        static_for<NB>([&](auto kc) {
            constexpr int k = decltype(kc)::value;
            const int j = (t + k * T) % Ns;
            static_for<R - 1>([&](auto rc) {
                constexpr int r = decltype(rc)::value;
                tw.w[RegOff + k * (R - 1) + r] = table[TwOff + r * Ns + j];
            });
        });
    }
    if constexpr (sizeof...(Rest) > 0) {
        constexpr int kNextOff = TwOff + (Ns > 1 ? (R - 1) * Ns : 0);
        constexpr int kNextReg = RegOff + (Ns > 1 ? NB * (R - 1) : 0);
        constexpr int kNextPow = PowOff + (Ns > 1 ? NB : 0);
        load_twiddles_pass<N, C, MODE, E, Ns * R, kNextOff, kNextReg, kNextPow, Rest...>(tw, t, table);
    }
}
template <int N, class C, int MODE, int... Rs>
__device__ __forceinline__ void load_twiddles_impl(Twiddles<N, C, MODE>& tw, int t, const C* table, IntList<Rs...>) {
    load_twiddles_pass<N, C, MODE, PlanOf<N>::E, 1, 0, 0, 0, Rs...>(tw, t, table);
}
template <int N, class C, int MODE>
__device__ __forceinline__ void load_twiddles(Twiddles<N, C, MODE>& tw, int t, const void* table) {
    if constexpr (MODE == TW_DIRECT || MODE == TW_DIRECT_LAUNDER)
        tw.table = (typename Twiddles<N, C, MODE>::GlobalPtr)table;
    if constexpr (MODE == TW_CACHED)
        load_twiddles_impl<N, C, MODE>(tw, t, static_cast<const C*>(table), RadicesOf<N>{});
}

// Workgroup barrier for the LDS exchanges. __syncthreads() alone did not stop
// hipcc (ROCm 7.2, 1024-thread workgroups under the 128-VGPR cap) from sinking
// the exchange's ds_reads below the following barrier, so a fast wave's next
// pass overwrote LDS a slow wave had not read yet (a ~1.5 % per-launch race).
// The memory clobbers and sched_barrier pin every LDS access to its side.
// The barrier waits for this wave's LDS operations only (lgkmcnt), never for
// vector memory: __syncthreads()' workgroup fence may drain vmcnt, which would
// stall on loads issued for the next tile (kernels.hpp, tile_loop).
__device__ __forceinline__ void lds_barrier() {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("" ::: "memory");
}
// Wave-local exchange point: this wave's LDS writes have landed; no s_barrier.
__device__ __forceinline__ void wave_lds_sync() {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("" ::: "memory");
}
// between the writes and the reads of one exchange
template <class Lds>
__device__ __forceinline__ void exchange_sync(const Lds&) {
    if constexpr (Lds::kWave)
        wave_lds_sync();
    else
        lds_barrier();
}
// after the reads of one exchange, before the next exchange's writes
template <class Lds>
__device__ __forceinline__ void exchange_done(const Lds& lds) {
    if constexpr (Lds::kWave) {
        asm volatile("" ::: "memory");  // keep the next writes behind these reads in program order
    } else if constexpr (Lds::kDouble) {
        lds.flip();
    } else {
        lds_barrier();
    }
}

// ------------------------------------------------------------------------
// Stockham driver.
//
// State: v[m] holds element t + T m of the line between passes, as V. V is
// complex64 whenever the LDS exchange is complex64 (the exchange rounds there
// anyway), which halves the registers a float64 transform keeps live; each
// butterfly widens its R inputs to the compute type C, and only the R values
// of one butterfly group are ever live in C.
//
// The last pass hands each butterfly group k (slots k + r NB, r < R) to a
// sink while it is still in C. Sinks either write it back to v, or apply an
// element-wise epilogue and — when the next transform's first radix equals
// this transform's last one, so that group k is the next first-pass group —
// run that first pass in registers too (fft_pair): the projection between an
// inverse and a forward transform then never rounds to complex64.
// ------------------------------------------------------------------------

template <class To, class From>
__device__ __forceinline__ To cv(From a) {
    return mk<To>((Scalar<To>)a.x, (Scalar<To>)a.y);
}

template <int N, int E, int L, bool INV, int Ns, int TwOff, int RegOff, int PowOff, class C, class V, class Lds,
          class Tw, class Sink, int R, int... Rest>
__device__ __forceinline__ void stockham_from(V (&v)[L][E], int t, const Tw& tw, const Lds& lds, Sink& sink) {
    constexpr int T = N / E;
    // The LDS slots and twiddle indices of a pass are functions of t alone, so
    // the compiler computes every pass's (and both transforms' of a pair) up
    // front and keeps them live: 386 registers for the 1920-point complex64
    // row pair, 149 with t passed through an empty asm per pass (each pass
    // then recomputes its own). The any-size engine's radix kernels
    // (kAlwaysLaunder twiddle modes) take it; the float32 engine keeps its
    // measured schedule.
    if constexpr (Tw::kAlwaysLaunder) asm volatile("" : "+v"(t));
    constexpr int NB = E / R;
    static_assert(E % R == 0, "radix must divide elements per thread");
    static_for<NB>([&](auto kc) {
        constexpr int k = decltype(kc)::value;
        const int b = t + k * T;
        const int j = (Ns == 1) ? 0 : (b % Ns);
        static_for<L>([&](auto lc) {
            constexpr int l = decltype(lc)::value;
            C u[R];
            static_for<R>([&](auto rc) {
                constexpr int r = decltype(rc)::value;
                u[r] = cv<C>(v[l][k + r * NB]);
            });
            if constexpr (Ns > 1) tw.template apply<TwOff, RegOff, PowOff, R, Ns, INV>(u, k, j);
            Dft<R, INV, C>::run(u);
            if constexpr (sizeof...(Rest) == 0) {
                // last pass: Ns * R == N, so b < Ns and output r belongs in slot k + r NB
                sink(lc, kc, u);
            } else {
                const int o = (b / Ns) * Ns * R + j;
                static_for<R>([&](auto rc) {
                    constexpr int r = decltype(rc)::value;
                    lds.store(l, o + r * Ns, u[r]);
                });
            }
        });
        // keep butterfly groups apart in the schedule: bounds the live registers
        // to about one group's worth (per line) in the compute type
        __builtin_amdgcn_sched_barrier(0);
    });
    if constexpr (sizeof...(Rest) > 0) {
        exchange_sync(lds);
        static_for<L>([&](auto lc) {
            constexpr int l = decltype(lc)::value;
            static_for<E>([&](auto mc) {
                constexpr int m = decltype(mc)::value;
                v[l][m] = lds.template load<V>(l, t + m * T);
            });
        });
        exchange_done(lds);
        constexpr int kNextReg = RegOff + (Ns > 1 ? NB * (R - 1) : 0);
        constexpr int kNextOff = TwOff + (Ns > 1 ? (R - 1) * Ns : 0);
        constexpr int kNextPow = PowOff + (Ns > 1 ? NB : 0);
        stockham_from<N, E, L, INV, Ns * R, kNextOff, kNextReg, kNextPow, C, V, Lds, Tw, Sink, Rest...>(v, t, tw, lds,
                                                                                                      sink);
    }
}

template <int... Rs>
struct FirstOf;
template <int R0, int... Rs>
struct FirstOf<R0, Rs...> {
    static constexpr int value = R0;
};
template <int... Rs>
struct LastOf {
    static constexpr int vals[] = {Rs...};
    static constexpr int value = vals[sizeof...(Rs) - 1];
};

// Re-load twiddles per transform (no reuse across the pair) where a thread
// holds 16+ elements: there the reuse costs more registers than the loads.
template <int K>
constexpr bool kLaunder = PlanOf<K>::E >= 16;

// whole transform, starting at pass 0
template <int K, bool INV, class C, int L, class V, class Lds, class Tw, class Sink, int... Rs>
__device__ __forceinline__ void stockham_all(V (&v)[L][PlanOf<K>::E], int t, const Tw& tw0, const Lds& lds,
                                             Sink& sink, IntList<Rs...>) {
    Tw tw = tw0;
    if constexpr (kLaunder<K> || Tw::kAlwaysLaunder) tw.launder();
    stockham_from<PlanOf<K>::N, PlanOf<K>::E, L, INV, 1, 0, 0, 0, C, V, Lds, Tw, Sink, Rs...>(v, t, tw, lds, sink);
}
// passes 1.. of a transform whose first pass already wrote the LDS line
// (pass 0 has no twiddles, so every twiddle offset is still 0 here)
template <int K, bool INV, class C, int L, class V, class Lds, class Tw, class Sink, int R0, int... Rs>
__device__ __forceinline__ void stockham_after_first(V (&v)[L][PlanOf<K>::E], int t, const Tw& tw0, const Lds& lds,
                                                     Sink& sink, IntList<R0, Rs...>) {
    static_assert(sizeof...(Rs) > 0, "fused transforms need at least two passes");
    Tw tw = tw0;
    if constexpr (kLaunder<K> || Tw::kAlwaysLaunder) tw.launder();
    stockham_from<PlanOf<K>::N, PlanOf<K>::E, L, INV, R0, 0, 0, 0, C, V, Lds, Tw, Sink, Rs...>(v, t, tw, lds, sink);
}

template <int... Rs>
constexpr int first_radix(IntList<Rs...>) { return FirstOf<Rs...>::value; }
template <int... Rs>
constexpr int last_radix(IntList<Rs...>) { return LastOf<Rs...>::value; }

// Writes the last pass back to the slots.
template <int L, int E, class V>
struct WriteBack {
    V (&v)[L][E];
    template <class LC, class KC, class C, int R>
    __device__ __forceinline__ void operator()(LC, KC, C (&u)[R]) const {
        constexpr int l = LC::value, k = KC::value, NB = E / R;
        static_for<R>([&](auto rc) {
            constexpr int r = decltype(rc)::value;
            v[l][k + r * NB] = cv<V>(u[r]);
        });
    }
};

// Transform L lines held in the slot layout. Every thread of the workgroup
// must call these (they contain workgroup barriers).
template <int K, bool INV, class C, int L, class V, class Lds, class Tw>
__device__ __forceinline__ void fft_line(V (&v)[L][PlanOf<K>::E], int t, const Tw& tw, const Lds& lds) {
    WriteBack<L, PlanOf<K>::E, V> wb{v};
    stockham_all<K, INV, C>(v, t, tw, lds, wb, RadicesOf<K>{});
}

// Transform, then epi(line l, slot m, C& z) on every output in the compute
// type, then write back.
template <int K, bool INV, class C, int L, class V, class Lds, class Tw, class Epi>
__device__ __forceinline__ void fft_line_epi(V (&v)[L][PlanOf<K>::E], int t, const Tw& tw, const Lds& lds,
                                             Epi&& epi) {
    constexpr int E = PlanOf<K>::E;
    auto sink = [&](auto lc, auto kc, auto& u) {
        constexpr int l = decltype(lc)::value;
        constexpr int k = decltype(kc)::value;
        constexpr int R = sizeof(u) / sizeof(u[0]);
        constexpr int NB = E / R;
        static_for<R>([&](auto rc) {
            constexpr int r = decltype(rc)::value;
            epi(l, k + r * NB, u[r]);
            v[l][k + r * NB] = cv<V>(u[r]);
        });
    };
    stockham_all<K, INV, C>(v, t, tw, lds, sink, RadicesOf<K>{});
}

// Transform (INV1), epi(line l, slot m, C& z) on every output, transform (INV2).
template <int K, bool INV1, bool INV2, class C, int L, class V, class Lds, class Tw, class Epi>
__device__ __forceinline__ void fft_pair(V (&v)[L][PlanOf<K>::E], int t, const Tw& tw, const Lds& lds, Epi&& epi) {
    constexpr int E = PlanOf<K>::E;
    constexpr int T = PlanOf<K>::T;
    constexpr int R0 = first_radix(RadicesOf<K>{});
    constexpr int RL = last_radix(RadicesOf<K>{});
    if constexpr (R0 == RL && kPlans[K].npass > 1) {
        // group k of the last pass is group k of the next transform's first pass
        auto sink = [&](auto lc, auto kc, auto& u) {
            constexpr int l = decltype(lc)::value;
            constexpr int k = decltype(kc)::value;
            constexpr int NB = E / RL;
            static_for<RL>([&](auto rc) {
                constexpr int r = decltype(rc)::value;
                epi(l, k + r * NB, u[r]);
            });
            Dft<RL, INV2, C>::run(u);  // first pass: Ns = 1, no twiddles
            const int o = (t + k * T) * RL;
            static_for<RL>([&](auto rc) {
                constexpr int r = decltype(rc)::value;
                lds.store(l, o + r, u[r]);
            });
        };
        stockham_all<K, INV1, C>(v, t, tw, lds, sink, RadicesOf<K>{});
        exchange_sync(lds);
        static_for<L>([&](auto lc) {
            constexpr int l = decltype(lc)::value;
            static_for<E>([&](auto mc) {
                constexpr int m = decltype(mc)::value;
                v[l][m] = lds.template load<V>(l, t + m * T);
            });
        });
        exchange_done(lds);
        WriteBack<L, E, V> wb{v};
        stockham_after_first<K, INV2, C>(v, t, tw, lds, wb, RadicesOf<K>{});
    } else {
        fft_line_epi<K, INV1, C>(v, t, tw, lds, epi);
        fft_line<K, INV2, C>(v, t, tw, lds);
    }
}

}  // namespace slm
