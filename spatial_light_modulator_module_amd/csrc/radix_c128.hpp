// Radix-plan kernels of the any-size engine: image sides that have a
// compile-time radix plan (plans.hpp) -- complex128 on 2^k and 768 sides,
// complex64 (template P, below) also on the 13-smooth SLM panel sides.
//
// The reference's loop runs in complex128 after its first ifft2
// (src/algorithms.py:27-38, 83-93). The float32 engine (kernels.hpp) keeps
// complex64 between its passes, which sets a phase-drift floor that the
// 4096^2 configuration (200 iterations) and GD's 500 iterations cross
// (DESIGN.md section 5). The mixed-radix kernels (mixed_radix.hpp) keep
// complex128 but run one butterfly at a time with runtime radices and table
// twiddles from L2 (latency-bound, 0.23 of 8 TB/s). These kernels put the
// float32 engine's structure under complex128 state: compile-time Stockham
// transforms (fft_core.hpp's butterflies, the mixed-plan driver mx_from below)
// with C = V = X = double2 (float64 butterflies and twiddles, complex128
// registers between passes, complex128 LDS exchanges), a whole line per thread
// group with its elements held in registers, and the element-wise projection
// between a launch's two transforms running on the last butterfly group still
// in registers (rz_pair).
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

// Precisions of these kernels (template P): PREC_F64 -- complex128 state,
// float64 arithmetic, complex128 exchanges ($SLM_ENGINE=float64, 2^k / 768
// sides); PREC_F32 -- complex64 state, float32 butterflies and projections,
// complex64 exchanges, the float32 engine's numerics (GS on 13-smooth SLM
// panel sides by default: plans.hpp variant 3, e.g. 1080 x 1920).
// Plan keys built per precision: float64 every plan with at most 16 elements
// per thread in any pass (E = 24 / 32 double2 would not fit the register file
// next to the exchange), the panel plans included (GD and uint8 GS on SLM
// panels); float32 every plan with E <= 30.
__host__ __device__ constexpr int plan_emax(int k) {  // register slots of a line (mixed plans: the largest ep)
    int e = kPlans[k].e;
    if (plan_mixed(k))
        for (int q = 0; q < kPlans[k].npass; ++q) e = kPlans[k].ep[q] > e ? kPlans[k].ep[q] : e;
    return e;
}
__host__ __device__ constexpr bool key_built(int k, int p = PREC_F64) {
    return k >= 0 && k < kNumPlans && (p == PREC_F64 ? plan_emax(k) <= 16 : kPlans[k].e <= 30);
}
// 13-smooth panel keys (plans.hpp variants 3 / 4): built on the B2 layout only
__host__ __device__ constexpr bool key_panel(int k) { return k >= 0 && k < kNumPlans && kPlans[k].variant >= 3; }

// Element-wise float64 pieces of these kernels: the reference's exp(i angle z)
// and z / |z| as z times a refined reciprocal square root (v_rsq_f64 and one
// Newton step: within ~1 ulp of 1 / sqrt, where the mixed-radix kernels pay an
// IEEE square root and division -- each a long float64 sequence, ~1,500 VALU
// per wave of the 4096 column pass, profiles/r06/sq_rz4096_d.txt). A float32
// target's amplitude is numpy's float32 square root, formed in float32 (the
// correctly rounded TgtLoad<TGT_F32>::amp, as the float32 engine).
__device__ __forceinline__ double rsq_nr(double x) {
    const double y = __builtin_amdgcn_rsq(x);
    return fma(y * 0.5, fma(-x * y, y, 1.0), y);
}
// a exp(i angle(z)) = a z / |z|, angle(0) = 0 -> a (src/algorithms.py:30,33)
__device__ __forceinline__ double2 unit_rz(double2 z, double a) {
    const double n2 = z.x * z.x + z.y * z.y;
    const bool zero = n2 == 0.0;
    const double r = a * rsq_nr(zero ? 1.0 : n2);
    return make_double2(zero ? a : z.x * r, zero ? 0.0 : z.y * r);
}
// x / |x| a (src/algorithms.py:84; |x| = 0 gives NaN as there)
__device__ __forceinline__ double2 u_rz(double2 x, double a) {
    const double r = a * rsq_nr(x.x * x.x + x.y * x.y);
    return make_double2(x.x * r, x.y * r);
}
// float32 (PREC_F32) counterparts: the float32 engine's (kernels.hpp unit_scale,
// normalize, rsqrt_nr)
__device__ __forceinline__ float2 unit_rz(float2 z, float a) { return unit_scale(z, a); }
__device__ __forceinline__ float2 u_rz(float2 x, float a) { return normalize(x, a); }
__device__ __forceinline__ float rsq_nr(float x) { return rsqrt_nr(x); }
// the cold start's complex64 rounding of ifft2(sqrt T) (src/algorithms.py:27):
// a no-op on complex64 state
__device__ __forceinline__ float2 round_c64(float2 z) { return z; }
using mr::round_c64;
// target intensity T (as uploaded) and numpy's amplitude sqrt(T): float16 for
// uint8, float32 for float32, both widened
__device__ __forceinline__ float tgt_at(const void* tgt, int tt, long long i) {
    return tt == TGT_U8 ? (float)static_cast<const uint8_t*>(tgt)[i] : static_cast<const float*>(tgt)[i];
}
template <class S = double>
__device__ __forceinline__ S amp_rz(float t, int tt) {
    return tt == TGT_U8 ? (S)TgtLoad<TGT_U8>::amp(t) : (S)TgtLoad<TGT_F32>::amp(t);
}
// twiddle source per precision: float64 powers from one load (TW_POW, below),
// float32 every twiddle from the table (powers in float32 would drift ~1e-6)

// Twiddles of the complex128 kernels: per butterfly one table load, w^1 =
// exp(-2 pi i j / (Ns R)), and its powers w^r by complex products (float64:
// r ulp-scale errors, ~1e-15, where the R - 1 table loads per butterfly were
// most of the kernels' vector-memory instructions -- 42 of 62 per wave of the
// 1024-point column pass, profiles/r06/sq_rz1024_d.txt). Loads laundered
// before every transform (TW_DIRECT_LAUNDER).
constexpr int TW_POW = 3;
// Twiddles of the complex64 kernels: every twiddle from the table where used
// (TW_DIRECT_LAUNDER; float32 powers would drift ~1e-6).

}  // namespace rz

template <int N, class C>
struct Twiddles<N, C, rz::TW_POW> {
    static constexpr bool kAlwaysLaunder = true;
    struct alignas(2 * sizeof(Scalar<C>)) Pod {
        Scalar<C> x, y;
    };
    using GlobalPtr = const __attribute__((address_space(1))) Pod*;
    GlobalPtr table;
    __device__ __forceinline__ void launder() {
        unsigned long long q = (unsigned long long)table;
        asm volatile("" : "+s"(q));
        table = (GlobalPtr)q;
    }
    template <int TwOff, int RegOff, int PowOff, int R, int Ns, bool INV>
    __device__ __forceinline__ void apply(C* u, int, int j) const {
        const C w1 = mk<C>(table[TwOff + j].x, table[TwOff + j].y);  // entry (r - 1) Ns + j at r = 1
        C w = w1;
        static_for<R - 1>([&](auto rc) {
            constexpr int r = decltype(rc)::value + 1;
            if constexpr (r > 1) w = cmul(w, w1);
            u[r] = INV ? cmulc(u[r], w) : cmul(u[r], w);
        });
    }
    template <int TwOff, int R, int Ns>
    __device__ __forceinline__ void fetch(C* w, int j) const {
        w[0] = mk<C>(table[TwOff + j].x, table[TwOff + j].y);
    }
    template <int R, bool INV>
    __device__ __forceinline__ static void apply_fetched(C* u, const C* wf) {
        const C w1 = wf[0];
        C w = w1;
        static_for<R - 1>([&](auto rc) {
            constexpr int r = decltype(rc)::value + 1;
            if constexpr (r > 1) w = cmul(w, w1);
            u[r] = INV ? cmulc(u[r], w) : cmul(u[r], w);
        });
    }
};

namespace rz {

// State layouts between the passes (template parameter LAY of both kernels):
//  LAY_RM -- row-major both ways: the row pass moves whole lines, the column
//    pass 32-B pieces of rows 64 KB apart (a wave-instruction load touches 32
//    lines a quarter each);
//  LAY_B2 -- "B2" both ways: 2-column panels, element (y, x) of a hologram at
//    ((x / 2) H + y) 2 + x % 2. A column tile's panel is one contiguous run (a
//    wave instruction moves 1 KB of consecutive rows, 8 whole lines); rows go
//    in pairs (y, y + 1), y even, lanes 4k .. 4k + 3 holding (y, 2k),
//    (y, 2k + 1), (y + 1, 2k), (y + 1, 2k + 1) of a slot: one 64-B piece of a
//    panel per four lanes.
// Measured per 4096^2 GS iteration (profiles/r06, one hologram): LAY_RM col
// 289 + row 125 us, LAY_B2 col 198 + row 250 us (row pairs: one 512-thread
// workgroup per CU), rows reading row-major and writing B2 col 318 + row 245
// us (writes in pieces cost as much as reads). GD and 1024^2 run faster on
// LAY_B2 (GD 1024^2 45.6 -> 40.3 us), GS 4096^2 on LAY_RM: the engine picks
// per plan (generic.hip, rz_layout). LAY_B2 column passes read the target
// from a float copy in B2 made at each run's start (contiguous, where the
// uploaded row-major target gave 8 B per row; LAY_RM reads the upload, where
// the copy measured slower), and user arrays (phases,
// a_in, the expected output, the GD field, the lone transforms' inputs and
// outputs) stay row-major.
constexpr int LAY_RM = 0, LAY_B2 = 1;
__host__ __device__ __forceinline__ long long b2_index(long long y, int x, int H) {
    return (((long long)(x >> 1) * H + y) << 1) + (x & 1);
}

// Row regions of a LAY_B2 pair's two rows: the second row's slots XOR 4 inside
// each 16-slot block (a bijection), so the pair-interleaved lanes of a
// ds_write_b128 group (8 contiguous lanes, banks (a/4) mod 32) and of a
// ds_read_b128 group (lanes {0-3, 12-15, 20-27}, (a/4) mod 64) take
// complementary bank halves (6 extra LDS cycles per instruction measured with
// a plain row offset; 0 modelled for the E = 16 plans, tools/rz_lds_banks.py).
template <class X, bool WAVE>
struct LdsPairRow : LdsLine<X, 0, WAVE> {
    int x = 0;  // 4 for the pair's second row
    template <class C>
    __device__ __forceinline__ void store(int l, int o, C v) const {
        this->base[this->cur + l * this->stride + (lds_slot(o) ^ x)] = mk<X>(v.x, v.y);
    }
    template <class C>
    __device__ __forceinline__ C load(int l, int o) const {
        const X v = this->base[this->cur + l * this->stride + (lds_slot(o) ^ x)];
        return mk<C>(v.x, v.y);
    }
    // unswizzled slots (mixed plans, LdsTile::store_lin)
    template <class C>
    __device__ __forceinline__ void store_lin(int l, int o, C v) const {
        this->base[this->cur + l * this->stride + o] = mk<X>(v.x, v.y);
    }
    template <class C>
    __device__ __forceinline__ C load_lin(int l, int o) const {
        const X v = this->base[this->cur + l * this->stride + o];
        return mk<C>(v.x, v.y);
    }
};

// complex64: table twiddles where used (TW_DIRECT_LAUNDER, L1/L2-resident); a
// copy of the table into LDS at the kernel's start (both pass orders of a mixed
// plan) measured slower once the mixed plans put 2-4 waves per SIMD on the chip
// (1920 x 1080 42.5 against 54.4 us per GS iteration; profiles/r06/speed_c64_twg_r.txt;
// removed)
template <int P>
constexpr int kTwMode = P == PREC_F64 ? TW_POW : TW_DIRECT_LAUNDER;

// ------------------------------------------------------------------------
// Mixed plans (plans.hpp ep[]): the elements per thread change from pass to
// pass. A single-E Stockham plan needs every radix to divide E, so a
// 1920-point line (2^7 3 5) with E = 30 has one factor 2 per pass: seven
// passes on 64 threads, one wave per SIMD over a 1080 x 1920 panel
// (profiles/r06/sq_c64_1080x1920_n.txt: 8,373 VALU and 906 LDS instructions
// per wave). Here pass p holds E_p elements on T_p = N / E_p threads, slot m
// of thread t being element t + T_p m as in the single-E driver; threads
// t >= T_p sit the pass out. The forward transform runs the radices in plan
// order, the inverse backwards, so the pair inverse -> forward (row kernels)
// and forward -> inverse (column kernels) always meets on one radix and one
// slot layout (fft_pair's fused projection).
// ------------------------------------------------------------------------
template <int K>
constexpr int kTMax = PlanOf<K>::T;  // threads of a line (the smallest E_p)

template <int K, bool INV, int P>
struct MxPass {
    static constexpr int NP = kPlans[K].npass;
    static constexpr bool REV = INV && plan_mixed(K);
    static constexpr int I = REV ? NP - 1 - P : P;
    static constexpr int R = kPlans[K].r[I];
    static constexpr int E = plan_mixed(K) ? kPlans[K].ep[I] : kPlans[K].e;
    static constexpr int T = kPlans[K].n / E;
    static constexpr bool LAST = P == NP - 1;
    static constexpr int ns_at() {
        int ns = 1;
        for (int q = 0; q < P; ++q) ns *= pass_radix(K, REV, q);
        return ns;
    }
    static constexpr int tw_at() {  // table offset of this pass's entries
        int ns = 1, off = REV ? twiddle_count_key(K) : 0;
        for (int q = 0; q < P; ++q) {
            if (ns > 1) off += (pass_radix(K, REV, q) - 1) * ns;
            ns *= pass_radix(K, REV, q);
        }
        return off;
    }
    static constexpr int NS = ns_at();
    static constexpr int TWOFF = tw_at();
    static_assert(E % R == 0 && T * E == kPlans[K].n, "mixed plan: radix must divide the pass's elements");
    static_assert(T <= kTMax<K>, "mixed plan: e must be the smallest ep");
};
// slot layout at a transform's ends: elements per thread and threads per line
template <int K, bool INV, bool FIRST>
using MxEnd = MxPass<K, INV, FIRST ? 0 : kPlans[K].npass - 1>;
// register slots a kernel's line array needs
template <int K>
constexpr int kEMax = plan_emax(K);

// A pass's twiddles, fetched before the exchange that precedes the pass (their
// global / LDS loads then overlap that exchange's writes, barrier and reads
// instead of stalling the pass's first butterfly) and applied in it: the same
// values and products as Twiddles::apply.
template <class C, int NB, int R>
struct MxTw {
    C w[NB][R > 1 ? R - 1 : 1];
};
template <int K, bool INV, int P, class C, class Tw>
__device__ __forceinline__ auto mx_fetch(const Tw& tw, int t) {
    using Ps = MxPass<K, INV, P>;
    constexpr int R = Ps::R, T = Ps::T, Ns = Ps::NS, NB = Ps::E / R;
    MxTw<C, NB, R> f;
    if constexpr (Ns > 1) {
        if (T == kTMax<K> || t < T) {
            static_for<NB>([&](auto kc) {
                constexpr int k = decltype(kc)::value;
                tw.template fetch<Ps::TWOFF, R, Ns>(f.w[k], (t + k * T) % Ns);
            });
        }
    }
    return f;
}

template <int K, bool INV, int P, class C, class V, int EM, class Lds, class Tw, class Sink, class Pre>
__device__ __forceinline__ void mx_from(V (&v)[1][EM], int t, const Tw& tw, const Lds& lds, Sink& sink,
                                        const Pre& pre) {
    using Ps = MxPass<K, INV, P>;
    constexpr int R = Ps::R, E = Ps::E, T = Ps::T, Ns = Ps::NS, NB = E / R;
    asm volatile("" : "+v"(t));  // per-pass address arithmetic (stockham_from)
    if (T == kTMax<K> || t < T) {
        static_for<NB>([&](auto kc) {
            constexpr int k = decltype(kc)::value;
            const int b = t + k * T;
            const int j = (Ns == 1) ? 0 : (b % Ns);
            C u[R];
            static_for<R>([&](auto rc) {
                constexpr int r = decltype(rc)::value;
                u[r] = cv<C>(v[0][k + r * NB]);
            });
            if constexpr (Ns > 1) Tw::template apply_fetched<R, INV>(u, pre.w[k]);
            Dft<R, INV, C>::run(u);
            if constexpr (Ps::LAST) {
                sink(kc, u);
            } else {
                // Only a transform's first pass (Ns = 1) writes at a stride (o = R b + r):
                // its exchange keeps the bank swizzle / padding. Later passes write runs
                // of consecutive j, so their exchanges use plain slots, whose index
                // arithmetic folds into the LDS instruction offsets (the swizzle cost
                // ~5 VALU per element access, a third of the 1920-point row pass's VALU)
                const int o = (b / Ns) * Ns * R + j;
                static_for<R>([&](auto rc) {
                    constexpr int r = decltype(rc)::value;
                    if constexpr (Ns == 1)
                        lds.store(0, o + r * Ns, u[r]);
                    else
                        lds.store_lin(0, o + r * Ns, u[r]);
                });
            }
            __builtin_amdgcn_sched_barrier(0);
        });
    }
    if constexpr (!Ps::LAST) {
        using Pn = MxPass<K, INV, P + 1>;
        const auto nxt = mx_fetch<K, INV, P + 1, C>(tw, t);
        exchange_sync(lds);
        if (Pn::T == kTMax<K> || t < Pn::T) {
            static_for<Pn::E>([&](auto mc) {
                constexpr int m = decltype(mc)::value;
                if constexpr (Ns == 1)
                    v[0][m] = lds.template load<V>(0, t + m * Pn::T);
                else
                    v[0][m] = lds.template load_lin<V>(0, t + m * Pn::T);
            });
        }
        exchange_done(lds);
        mx_from<K, INV, P + 1, C>(v, t, tw, lds, sink, nxt);
    }
}

// Transform wrappers of the radix kernels, on mx_from for every plan (a
// single-E plan is a mixed plan with one E): epi(p, z) sees each output z with
// its element position p along the line. Single-E plans ran fft_core.hpp's
// Stockham driver until r06; mx_from's plain slots after the first pass and
// fetched-ahead twiddles measured faster on every complex128 / complex64 shape
// tried (GD 4096^2 0.665 -> 0.640 ms, GD 1024^2 0.0445 -> 0.0415, GS 2048^2
// 0.094 -> 0.089; profiles/r06/ab_mx_all_zb.txt).
template <int K, bool INV, class C, class V, int EM, class Lds, class Tw>
__device__ __forceinline__ void rz_line(V (&v)[1][EM], int t, const Tw& tw0, const Lds& lds) {
    Tw tw = tw0;
    tw.launder();
    using PL = MxEnd<K, INV, false>;
    auto wb = [&](auto kc, auto& u) {
        constexpr int k = decltype(kc)::value, NB = PL::E / PL::R;
        static_for<PL::R>([&](auto rc) {
            constexpr int r = decltype(rc)::value;
            v[0][k + r * NB] = cv<V>(u[r]);
        });
    };
    mx_from<K, INV, 0, C>(v, t, tw, lds, wb, MxTw<C, 1, 1>{});
}
template <int K, bool INV, class C, class V, int EM, class Lds, class Tw, class Epi>
__device__ __forceinline__ void rz_line_epi(V (&v)[1][EM], int t, const Tw& tw0, const Lds& lds, Epi&& epi) {
    Tw tw = tw0;
    tw.launder();
    using PL = MxEnd<K, INV, false>;
    auto sink = [&](auto kc, auto& u) {
        constexpr int k = decltype(kc)::value, NB = PL::E / PL::R;
        static_for<PL::R>([&](auto rc) {
            constexpr int r = decltype(rc)::value;
            epi(t + PL::T * (k + r * NB), u[r]);
            v[0][k + r * NB] = cv<V>(u[r]);
        });
    };
    mx_from<K, INV, 0, C>(v, t, tw, lds, sink, MxTw<C, 1, 1>{});
}
template <int K, bool INV1, bool INV2, class C, class V, int EM, class Lds, class Tw, class Epi>
__device__ __forceinline__ void rz_pair(V (&v)[1][EM], int t, const Tw& tw0, const Lds& lds, Epi&& epi) {
    {
        static_assert(INV1 != INV2, "a pair runs one transform forwards and the other backwards");
        using PL = MxEnd<K, INV1, false>;  // the first transform's last pass ...
        using PF = MxEnd<K, INV2, true>;   // ... is the second one's first (same radix and slots)
        static_assert(PL::R == PF::R && PL::E == PF::E, "mixed pair: passes do not meet");
        Tw tw = tw0;
        tw.launder();
        auto sink = [&](auto kc, auto& u) {
            constexpr int k = decltype(kc)::value, NB = PL::E / PL::R;
            static_for<PL::R>([&](auto rc) {
                constexpr int r = decltype(rc)::value;
                epi(t + PL::T * (k + r * NB), u[r]);
            });
            Dft<PL::R, INV2, C>::run(u);  // the second transform's first pass: Ns = 1, no twiddles
            const int o = (t + k * PL::T) * PL::R;
            static_for<PL::R>([&](auto rc) {
                constexpr int r = decltype(rc)::value;
                lds.store(0, o + r, u[r]);
            });
        };
        mx_from<K, INV1, 0, C>(v, t, tw, lds, sink, MxTw<C, 1, 1>{});
        using P1 = MxPass<K, INV2, 1>;
        Tw tw2 = tw0;
        tw2.launder();
        const auto nxt = mx_fetch<K, INV2, 1, C>(tw2, t);
        exchange_sync(lds);
        if (P1::T == kTMax<K> || t < P1::T) {
            static_for<P1::E>([&](auto mc) {
                constexpr int m = decltype(mc)::value;
                v[0][m] = lds.template load<V>(0, t + m * P1::T);
            });
        }
        exchange_done(lds);
        using PZ = MxEnd<K, INV2, false>;
        auto wb = [&](auto kc, auto& u) {
            constexpr int k = decltype(kc)::value, NB = PZ::E / PZ::R;
            static_for<PZ::R>([&](auto rc) {
                constexpr int r = decltype(rc)::value;
                v[0][k + r * NB] = cv<V>(u[r]);
            });
        };
        mx_from<K, INV2, 1, C>(v, t, tw2, lds, wb, nxt);
    }
}

// the plan's twiddle table (global; every pass reads its entries where used)
template <class Tw>
__device__ __forceinline__ void tw_setup(Tw& tw, const void* table) {
    tw.table = (typename Tw::GlobalPtr)table;
}

template <int K, int LAY>
struct RowGeo {
    static constexpr int T = PlanOf<K>::T;
    static constexpr bool PAIRS = LAY == LAY_B2;
    // rows per workgroup: ~256 threads, whole pairs on B2 (the panel plans' T =
    // 20 .. 100 need not divide 256; the host checks H % RPW)
    static constexpr int RPW = PAIRS ? (T >= 128 ? 2 : 2 * (128 / T)) : (T >= 256 ? 1 : 256 / T);
    static constexpr int THREADS = RPW * T;
    static constexpr int GROUP = PAIRS ? 2 * T : T;  // lanes of one row (pair)
    static constexpr bool WAVE = GROUP <= 64 && 64 % GROUP == 0;  // each row (pair) inside one wave: no barrier
    static constexpr int LINE = PlanOf<K>::ROWSTRIDE;
    // 512 (row-major) / 1024 (pairs) threads, the 4096 E = 8 rows: a register
    // budget of 16 waves per CU (<= 128 VGPRs)
    static constexpr int MIN_WAVES = THREADS == (PAIRS ? 1024 : 512) ? 4 : 1;
};

template <int K, int CW, int P = PREC_F64>
struct ColGeo {
    static constexpr int T = PlanOf<K>::T;
    static constexpr int THREADS = CW * T;
    static constexpr bool WAVE = THREADS <= 64;
    static constexpr int SLOTS = lds_line(PlanOf<K>::N) * CW;
    static constexpr bool kValid = THREADS >= 64 && THREADS <= 1024 &&
                                   SLOTS * (int)sizeof(CplxOf<P>) <= 160 * 1024;
};

// waves-per-SIMD floor of a row kernel: RowGeo's, and for the complex64 rows of
// the 240-thread 1920 plan (480-thread row-pair tiles, 8 waves) 6 per SIMD --
// three tiles per CU, so a 1080-row panel's 540 tiles run in one round
template <int K, int LAY, int P>
constexpr int row_min_waves() {
    return (P == PREC_F32 && RowGeo<K, LAY>::THREADS == 480) ? 6 : RowGeo<K, LAY>::MIN_WAVES;
}

template <int K, int OP, int LAY, int P>
__global__ void __launch_bounds__((RowGeo<K, LAY>::THREADS), (row_min_waves<K, LAY, P>())) rz_row_kernel(mr::RowArgs a) {
    using C = CplxOf<P>;  // compute and state type
    using S = Scalar<C>;
    using namespace mr;
    const C* in = reinterpret_cast<const C*>(a.in);
    C* out = reinterpret_cast<C*>(a.out);
    C* xf = reinterpret_cast<C*>(a.x);
    constexpr int N = PlanOf<K>::N, T = PlanOf<K>::T;
    constexpr int RPW = RowGeo<K, LAY>::RPW, LINE = RowGeo<K, LAY>::LINE;
    constexpr bool WV = RowGeo<K, LAY>::WAVE;
    // slot layouts where the line is loaded and stored: the first pass of the
    // kernel's first transform and the last pass of its last one (one layout,
    // E elements on T threads, unless the plan is mixed)
    constexpr bool INV_FIRST = !(OP == RO_FWD || OP == RO_WARM || OP == RO_GD_INIT);
    constexpr bool INV_LAST = OP == RO_INV;
    using LD = MxEnd<K, INV_FIRST, true>;
    using ST = MxEnd<K, INV_LAST, false>;
    __shared__ C smem[RPW * LINE];
    // lane -> (row of the tile, t); LAY_B2 pairs: lanes 4k .. 4k + 3 = (r, 2k), (r, 2k + 1),
    // (r + 1, 2k), (r + 1, 2k + 1) -- one 64-B piece of a panel per four lanes and slot
    int t, lrow;
    if constexpr (LAY == LAY_B2) {
        const int q = threadIdx.x % (2 * T);
        t = ((q >> 2) << 1) | (q & 1);
        lrow = 2 * (threadIdx.x / (2 * T)) + ((q >> 1) & 1);
    } else {
        t = threadIdx.x % T;
        lrow = threadIdx.x / T;
    }
    const int tiles = a.H / RPW;
    const int id = xcd_remap(blockIdx.x, gridDim.x);  // neighbouring row groups on one XCD
    const int b = id / tiles;
    const int row = (id - b * tiles) * RPW + lrow;
    const long long pix0 = (long long)row * N;  // row start within the hologram (row-major arrays)
    const long long off = (long long)b * a.holo + pix0;
    const long long hoff = (long long)b * a.holo;
    // the state at element p of the row: B2, or row-major
    auto st_at = [&](int p) { return LAY == LAY_B2 ? hoff + b2_index(row, p, a.H) : off + p; };
    if constexpr (OP == RO_GS || OP == RO_GD || OP == RO_GS_MID) {
        if (a.checked && a.iter > a.stop[b]) return;  // stopped earlier: frozen (src/algorithms.py:29,83)
    }
    LdsPairRow<C, WV> lds;
    lds.base = smem + lrow * LINE;
    lds.stride = LINE;
    lds.x = LAY == LAY_B2 ? (lrow & 1) << 2 : 0;
    Twiddles<K, C, kTwMode<P>> tw;
    auto ain = [&](int p) -> S { return a.ain ? (S)a.ain[pix0 + p] : (S)1; };
    C v[1][kEMax<K>];
    if (LD::T == T || t < LD::T) {
#pragma unroll
        for (int m = 0; m < LD::E; ++m) {
            const int p = t + LD::T * m;
            const long long i = off + p;
            if constexpr (OP == RO_WARM) {
                // numpy: exp(1j * float32 phase) is complex64, then times the float64 a_in
                const S am = ain(p);
                if constexpr (P == PREC_F64) {
                    double s, c;
                    sincos((double)a.phase_in[i], &s, &c);
                    v[0][m] = make_double2((double)(float)c * am, (double)(float)s * am);
                } else {
                    float s, c;
                    sincosf(a.phase_in[i], &s, &c);
                    v[0][m] = make_float2(c * am, s * am);
                }
            } else if constexpr (OP == RO_GD_INIT) {
                const float2 f = a.field0[i];
                const C x = mk<C>((S)f.x, (S)f.y);
                xf[i] = x;
                v[0][m] = u_rz(x, ain(p));
            } else if constexpr (OP == RO_FWD || OP == RO_INV) {
                v[0][m] = in[i];  // lone transforms: row-major input
            } else {
                v[0][m] = in[st_at(p)];
            }
        }
    }
    tw_setup(tw, a.pl.tw);
    if constexpr (OP == RO_FWD || OP == RO_WARM || OP == RO_GD_INIT) {
        rz_line<K, false, C>(v, t, tw, lds);
    } else if constexpr (OP == RO_INV) {
        rz_line<K, true, C>(v, t, tw, lds);
    } else if constexpr (OP == RO_COLD) {
        // A0 = ifft2(sqrt T) is complex64 (src/algorithms.py:27); B = a_in A0/|A0| (:30)
        rz_pair<K, true, false, C>(v, t, tw, lds, [&](int p, C& z) { z = unit_rz(round_c64(z), ain(p)); });
    } else if constexpr (OP == RO_GS) {
        if (a.last || (a.checked && a.stop[b] == a.iter)) {  // uniform per workgroup
            rz_line_epi<K, true, C>(v, t, tw, lds, [&](int p, C& z) {
                a.phase_out[off + p] = (float)atan2(z.y, z.x);  // hologram = np.angle(A) (:48)
            });
            return;
        }
        rz_pair<K, true, false, C>(v, t, tw, lds, [&](int p, C& z) { z = unit_rz(z, ain(p)); });
    } else if constexpr (OP == RO_GS_MID) {
        rz_pair<K, true, false, C>(v, t, tw, lds, [&](int p, C& z) { z = unit_rz(z, ain(p)); });
    } else if constexpr (OP == RO_GD_FOURIER) {
        // angle of the complex64 ifft2 is float32, exp of it complex64 (:153-156)
        rz_pair<K, true, false, C>(v, t, tw, lds, [&](int p, C& z) {
            const C c = round_c64(z);
            const float ang = atan2f((float)c.y, (float)c.x);
            float sn, cs;
            sincosf(ang, &sn, &cs);  // (the float64 engine used sincos of the float32 angle, rounded)
            if constexpr (P == PREC_F64) {
                double s, co;
                sincos((double)ang, &s, &co);
                sn = (float)s;
                cs = (float)co;
            }
            const S am = ain(p);
            const C x = mk<C>((S)cs * am, (S)sn * am);
            xf[off + p] = x;
            z = u_rz(x, am);
        });
    } else if constexpr (OP == RO_GD) {
        // dEdF = ifft2(G) a_in (unscaled transform * 1/S), dEdX_complex, x -= lr dEdX
        // (:87-91, :179-185); next forward input u = a_in x/|x| (:84)
        const S l = (S)a.lr[a.iter];
        auto update = [&](int p, const C& z) -> C {
            const S am = ain(p);
            const S s = am * (S)a.inv_s;
            const S gx = z.x * s, gy = z.y * s;
            const long long i = off + p;
            C x = xf[i];
            // dEdX_complex = (g - x Re(conj(x) g) / |x|^2) / |x| (:179-185)
            const S inv = rsq_nr(x.x * x.x + x.y * x.y);
            const S inv3 = inv * inv * inv;
            const S re = x.x * gx + x.y * gy;
            x.x -= l * (gx * inv - x.x * re * inv3);
            x.y -= l * (gy * inv - x.y * re * inv3);
            xf[i] = x;
            return x;
        };
        if (a.last) {  // the run's last update needs no next forward transform
            rz_line_epi<K, true, C>(v, t, tw, lds, [&](int p, C& z) { (void)update(p, z); });
            return;
        }
        rz_pair<K, true, false, C>(v, t, tw, lds, [&](int p, C& z) { z = u_rz(update(p, z), ain(p)); });
    }
    if (ST::T == T || t < ST::T) {
#pragma unroll
        for (int m = 0; m < ST::E; ++m) out[st_at(t + ST::T * m)] = v[0][m];
    }
}

template <int K, int CW, int OP, int LAY, int P>
__global__ void __launch_bounds__((ColGeo<K, CW, P>::THREADS), 1) rz_col_kernel(mr::ColArgs a) {
    using C = CplxOf<P>;  // compute and state type
    using S = Scalar<C>;
    using namespace mr;
    const C* in = reinterpret_cast<const C*>(a.in);
    C* out = reinterpret_cast<C*>(a.out);
    constexpr int T = PlanOf<K>::T;
    constexpr int THREADS = ColGeo<K, CW, P>::THREADS;
    constexpr bool WV = ColGeo<K, CW, P>::WAVE;
    // load / store slot layouts (rz_row_kernel)
    constexpr bool INV_FIRST = OP == CO_INV || OP == CO_AMP_INV;
    constexpr bool INV_LAST = !(OP == CO_FWD || OP == CO_GD_STATS);
    using LD = MxEnd<K, INV_FIRST, true>;
    using ST = MxEnd<K, INV_LAST, false>;
    __shared__ C smem[ColGeo<K, CW, P>::SLOTS];
    const int c = threadIdx.x % CW, t = threadIdx.x / CW;
    const int id = xcd_remap(blockIdx.x, gridDim.x);  // neighbouring tiles (partial lines) on one XCD
    const int b = id / a.nwg;
    const int tile = id - b * a.nwg;
    const int col = tile * CW + c;
    const long long hoff = (long long)b * a.holo;
    const long long cbase = hoff + col;                  // row-major: element p of this column at + p W
    const long long bbase = hoff + b2_index(0, col, a.H);  // B2 (target copy, LAY_B2 state): + 2 p
    auto rm_at = [&](int p) { return cbase + (long long)p * a.W; };
    auto st_at = [&](int p) { return LAY == LAY_B2 ? bbase + 2LL * p : rm_at(p); };
    // the target: the B2 float copy (LAY_B2), else as uploaded (row-major; on LAY_RM the
    // copy measured slower, 4096^2 column pass 289 -> 325 us, profiles/r06)
    auto tgt_val = [&](int p, int tt) -> float {
        return LAY == LAY_B2 ? a.tgt_blk[bbase + 2LL * p] : tgt_at(a.tgt, tt, rm_at(p));
    };
    if constexpr (OP == CO_GS || OP == CO_GD_STATS || OP == CO_GD_GRAD || OP == CO_GD_GRAD_U8) {
        if (a.checked && a.iter > a.stop[b]) return;  // stopped earlier: frozen
    }
    const LdsTile<CW, C, 0, WV> lds{smem, c};
    Twiddles<K, C, kTwMode<P>> tw;
    C v[1][kEMax<K>];
    if (LD::T == T || t < LD::T) {
#pragma unroll
        for (int m = 0; m < LD::E; ++m) {
            const int p = t + LD::T * m;
            if constexpr (OP == CO_AMP_INV)
                v[0][m] = mk<C>(amp_rz<S>(tgt_val(p, a.tt), a.tt), (S)0);
            else
                v[0][m] = in[st_at(p)];
        }
    }
    tw_setup(tw, a.pl.tw);
    if constexpr (OP == CO_FWD) {
        rz_line<K, false, C>(v, t, tw, lds);
    } else if constexpr (OP == CO_INV || OP == CO_AMP_INV) {
        rz_line<K, true, C>(v, t, tw, lds);
    } else {
        double mx = 0.0, s2 = 0.0, st = 0.0;
        auto stats = [&](int p, const C& z, float tv) -> double {
            const double en = (double)(z.x * z.x + z.y * z.y);
            mx = fmax(mx, en);
            s2 += en * en;
            st += en * (double)tv;
            if (a.write_e) a.e_out[rm_at(p)] = (float)en;
            return en;
        };
        if constexpr (OP == CO_GS) {
            // E = |C|^2 statistics and expected output, D = a_T C/|C| (:33,36-38)
            rz_pair<K, false, true, C>(v, t, tw, lds, [&](int p, C& z) {
                const float tv = tgt_val(p, a.tt);
                (void)stats(p, z, tv);
                z = unit_rz(z, amp_rz<S>(tv, a.tt));
            });
        } else if constexpr (OP == CO_GD_STATS) {
            rz_line_epi<K, false, C>(v, t, tw, lds, [&](int p, C& z) { (void)stats(p, z, tgt_val(p, a.tt)); });
        } else if constexpr (OP == CO_GD_GRAD || OP == CO_GD_GRAD_U8) {
            // G = mask F (s P - T), s = norm / max P (:80,85-88); numpy's mask dtype:
            // float32 for a float32 target, float64 for uint8
            const S s = (S)(a.norm[b] / a.stats[((long long)b * a.max_loops + a.iter) * 4]);
            rz_pair<K, false, true, C>(v, t, tw, lds, [&](int p, C& z) {
                const S tv = (S)tgt_val(p, OP == CO_GD_GRAD_U8 ? TGT_U8 : TGT_F32);
                const S mask = OP == CO_GD_GRAD_U8
                                   ? (S)(1.0 + (double)a.wa * (double)tv / 255.0)
                                   : (S)(1.0f + __fdiv_rn(__fmul_rn(a.wa, (float)tv), 255.0f));
                const S w = mask * ((z.x * z.x + z.y * z.y) * s - tv);
                z = mk<C>(z.x * w, z.y * w);
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
    if (ST::T == T || t < ST::T) {
#pragma unroll
        for (int m = 0; m < ST::E; ++m) {
            const int p = t + ST::T * m;
            if constexpr (OP == CO_FWD || OP == CO_INV)
                out[rm_at(p)] = v[0][m];  // lone transforms: row-major output
            else
                out[st_at(p)] = v[0][m];
        }
    }
}

// ------------------------------------------------------------------------
// host side (rz_inst.hip, one object per plan key)
// ------------------------------------------------------------------------
#define SLM_RZ_DECLARE(N)                                                                                    \
    int rz_row_launch_##N(int prec, int lay, int op, const mr::RowArgs& a, int grid, hipStream_t st);        \
    int rz_col_launch_##N(int prec, int lay, int cw, int op, const mr::ColArgs& a, int grid, hipStream_t st); \
    int rz_row_rpw_##N(int lay);                                                                             \
    int rz_col_ok_##N(int prec, int cw);
SLM_RZ_DECLARE(0)
SLM_RZ_DECLARE(1)
SLM_RZ_DECLARE(2)
SLM_RZ_DECLARE(3)
SLM_RZ_DECLARE(4)
SLM_RZ_DECLARE(5)
SLM_RZ_DECLARE(6)
SLM_RZ_DECLARE(8)
SLM_RZ_DECLARE(9)
SLM_RZ_DECLARE(10)
SLM_RZ_DECLARE(11)
SLM_RZ_DECLARE(12)
SLM_RZ_DECLARE(13)
SLM_RZ_DECLARE(14)
SLM_RZ_DECLARE(15)
SLM_RZ_DECLARE(16)
SLM_RZ_DECLARE(17)
SLM_RZ_DECLARE(18)
SLM_RZ_DECLARE(19)
SLM_RZ_DECLARE(20)
SLM_RZ_DECLARE(21)
SLM_RZ_DECLARE(22)
SLM_RZ_DECLARE(23)
SLM_RZ_DECLARE(24)
#undef SLM_RZ_DECLARE
#define SLM_RZ_FOR_EACH_KEY(X) \
    X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(8) X(9) X(10) X(11) X(12) X(13) X(14) X(15) X(16) X(17) X(18) X(19) X(20) \
    X(21) X(22) X(23) X(24)

// launch op on plan key k (0 on success, -1 on a launch error or an unbuilt key)
inline int rz_row_launch(int k, int prec, int lay, int op, const mr::RowArgs& a, int grid, hipStream_t st) {
#define SLM_CASE(N) \
    case N: return rz_row_launch_##N(prec, lay, op, a, grid, st);
    switch (k) { SLM_RZ_FOR_EACH_KEY(SLM_CASE) default: return -1; }
#undef SLM_CASE
}
inline int rz_col_launch(int k, int prec, int lay, int cw, int op, const mr::ColArgs& a, int grid, hipStream_t st) {
#define SLM_CASE(N) \
    case N: return rz_col_launch_##N(prec, lay, cw, op, a, grid, st);
    switch (k) { SLM_RZ_FOR_EACH_KEY(SLM_CASE) default: return -1; }
#undef SLM_CASE
}
// rows per row tile of key k on layout lay (0: not built)
inline int rz_row_rpw(int k, int lay) {
#define SLM_CASE(N) \
    case N: return rz_row_rpw_##N(lay);
    switch (k) { SLM_RZ_FOR_EACH_KEY(SLM_CASE) default: return 0; }
#undef SLM_CASE
}
// 1 if key k has column kernels of cw columns at precision prec
inline int rz_col_ok(int k, int prec, int cw) {
#define SLM_CASE(N) \
    case N: return rz_col_ok_##N(prec, cw);
    switch (k) { SLM_RZ_FOR_EACH_KEY(SLM_CASE) default: return 0; }
#undef SLM_CASE
}

}  // namespace rz
}  // namespace slm
