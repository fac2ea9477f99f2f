// Wave-shuffle transform pair for 1024-point lines (the headline GS loop).
//
// The GS iteration runs, along each line, a transform, an element-wise
// projection and the opposite transform (src/algorithms.py:29-34: fft2, then
// a_T C/|C|, then ifft2; the row side inverse, a_in A/|A|, forward). The
// Stockham engine (fft_core.hpp) exchanges through LDS with a workgroup barrier
// before every pass. This engine instead runs the first transform decimated in
// frequency (natural order in, digit-reversed out) and the second decimated in
// time (digit-reversed in, natural out), so nothing is ever reordered, and it
// places the index bits so that four of the six exchanges of the pair are
// register <-> lane bit swaps inside a wave:
//
//   v_permlane16_swap   swaps a slot bit with lane bit 4 (16-lane rows)
//   v_permlane32_swap   swaps a slot bit with lane bit 5 (32-lane halves)
//
// one VALU instruction per dword pair, no LDS, no barrier. Only the exchange
// that moves index bits across waves goes through LDS (once per transform).
//
// Geometry: 256-thread workgroups of two lines (lane bit 0 selects the line:
// the two columns of a 2-column tile, or the two rows of a row pair), 8 complex
// values per thread, 4 waves. Index bits of a line (pos 0..9) by state; "l1"
// .. "l5" are lane bits 1..5, "w" the wave, slot m = s0 + 2 s1 + 4 s2:
//
//   A (load/store)   s = pos 7,8,9   l1-3 = pos 0-2  w = pos 3,4  l4,l5 = pos 5,6
//   P1 radix 8 on pos 7-9, twiddle w_1024^(pos[0:7] k1)
//   X1 permlane16 (s1 <-> l4), permlane32 (s2 <-> l5)
//   B                s = pos 7,5,6   l1-3 = pos 0-2  w = pos 3,4  l4,l5 = pos 8,9
//   P2 radix 4 on pos 5,6 (two butterflies, by s0), twiddle w_128^(pos[0:5] k2)
//   X2 LDS (+ barrier)
//   C                s = pos 3,4,2   l1-3 = pos 7-9  w = pos 5,6  l4,l5 = pos 0,1
//   P3 radix 4 on pos 3,4 (by s2), twiddle w_32^(pos[0:3] k3)
//   X3 permlane16 (s0 <-> l4), permlane32 (s1 <-> l5)
//   D                s = pos 0,1,2   l1-3 = pos 7-9  w = pos 5,6  l4,l5 = pos 3,4
//   P4 radix 8 on pos 0-2
//
// In state D slot m of a thread holds frequency k = pos[7:10] + 8 pos[5:7] +
// 32 pos[3:5] + 128 pos[0:3], which is exactly the index t + 128 m the thread
// loaded in state A (t = shuffle_t(tid)): the projection reads its per-element
// data (target, a_in) with the load indices. The second transform runs the
// passes backwards as adjoints (conjugate twiddle before the butterfly).
// tools/shuffle_fft_model.py simulates this schedule lane by lane against
// numpy.fft and checks the X2 LDS slot swizzle is bank-conflict-free (both
// directions, ds_write_b64 16-lane and ds_read_b64 32-lane groups).
//
// Twiddles: 16 per thread (7 + 3 + 2 x 3), read once from a table of the 1024
// roots exp(-2 pi i e / 1024) computed in double on the host (slm_capi.hip,
// get_twiddles) and shared by both transforms (the second uses conjugates).
//
// Arithmetic type C: float2 (float32 butterflies) or double2 (float64
// butterflies and twiddles, the values held in double between the passes and
// moved by the lane swaps as two dword pairs; the one LDS exchange X2 stores
// complex64). The plan's state in HBM is complex64 either way; callers hand in
// complex64 slots and get complex64 back (shuffle_pair converts).
#pragma once
#include "fft_core.hpp"

namespace slm {

constexpr int kShufN = 1024;

// transform-thread index t of workgroup thread tid in state A: element
// t + 128 m is held in slot m
__device__ __forceinline__ int shuffle_t(int tid) {
    const int lam = tid & 63, om = tid >> 6;
    return ((lam >> 1) & 7) | (om << 3) | (((lam >> 4) & 3) << 5);
}

template <class C>
struct ShuffleTwT {
    C p1[7];  // w_1024^(t k1), k1 = 1..7
    C p2[3];  // w_128^((t & 31) k2), k2 = 1..3
    C p3[6];  // w_32^(n k3), n = l4 + 2 l5 + 4 s2, [3 s2 + k3 - 1]
};
using ShuffleTw = ShuffleTwT<float2>;

template <class C>
__device__ __forceinline__ void load_shuffle_tw(ShuffleTwT<C>& tw, int tid, const C* __restrict__ roots) {
    const int t = shuffle_t(tid);
    const int lam = tid & 63;
    static_for<7>([&](auto kc) {
        constexpr int k = decltype(kc)::value + 1;
        tw.p1[k - 1] = roots[t * k];
    });
    static_for<3>([&](auto kc) {
        constexpr int k = decltype(kc)::value + 1;
        tw.p2[k - 1] = roots[8 * (t & 31) * k];
    });
    const int n3 = ((lam >> 4) & 1) | (((lam >> 5) & 1) << 1);
    static_for<2>([&](auto hc) {
        constexpr int hi = decltype(hc)::value;
        static_for<3>([&](auto kc) {
            constexpr int k = decltype(kc)::value + 1;
            tw.p3[3 * hi + k - 1] = roots[32 * (n3 | (hi << 2)) * k];
        });
    });
}

// --- register <-> lane bit swaps (one v_permlane*_swap per dword) ---------
__device__ __forceinline__ unsigned as_u(float x) { return __builtin_bit_cast(unsigned, x); }
__device__ __forceinline__ float as_f(unsigned x) { return __builtin_bit_cast(float, x); }

// a = the slot with the bit clear (vdst), b = the slot with the bit set (src)
__device__ __forceinline__ void swap_l4(float2& a, float2& b) {
    const auto x = __builtin_amdgcn_permlane16_swap(as_u(a.x), as_u(b.x), false, false);
    const auto y = __builtin_amdgcn_permlane16_swap(as_u(a.y), as_u(b.y), false, false);
    a = make_float2(as_f(x[0]), as_f(y[0]));
    b = make_float2(as_f(x[1]), as_f(y[1]));
}
__device__ __forceinline__ void swap_l5(float2& a, float2& b) {
    const auto x = __builtin_amdgcn_permlane32_swap(as_u(a.x), as_u(b.x), false, false);
    const auto y = __builtin_amdgcn_permlane32_swap(as_u(a.y), as_u(b.y), false, false);
    a = make_float2(as_f(x[0]), as_f(y[0]));
    b = make_float2(as_f(x[1]), as_f(y[1]));
}
// float64 values: each half of each component is one dword swap
__device__ __forceinline__ unsigned lo_u(double x) { return (unsigned)__builtin_bit_cast(unsigned long long, x); }
__device__ __forceinline__ unsigned hi_u(double x) { return (unsigned)(__builtin_bit_cast(unsigned long long, x) >> 32); }
__device__ __forceinline__ double as_d(unsigned lo, unsigned hi) {
    return __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lo);
}
template <bool HALVES32>
__device__ __forceinline__ void swap_d(double& a, double& b) {
    const auto l = HALVES32 ? __builtin_amdgcn_permlane32_swap(lo_u(a), lo_u(b), false, false)
                            : __builtin_amdgcn_permlane16_swap(lo_u(a), lo_u(b), false, false);
    const auto h = HALVES32 ? __builtin_amdgcn_permlane32_swap(hi_u(a), hi_u(b), false, false)
                            : __builtin_amdgcn_permlane16_swap(hi_u(a), hi_u(b), false, false);
    a = as_d(l[0], h[0]);
    b = as_d(l[1], h[1]);
}
__device__ __forceinline__ void swap_l4(double2& a, double2& b) {
    swap_d<false>(a.x, b.x);
    swap_d<false>(a.y, b.y);
}
__device__ __forceinline__ void swap_l5(double2& a, double2& b) {
    swap_d<true>(a.x, b.x);
    swap_d<true>(a.y, b.y);
}
// X1: s1 <-> l4, s2 <-> l5 (its own inverse)
template <class C>
__device__ __forceinline__ void shuffle_x1(C (&v)[8]) {
    swap_l4(v[0], v[2]);
    swap_l4(v[1], v[3]);
    swap_l4(v[4], v[6]);
    swap_l4(v[5], v[7]);
    swap_l5(v[0], v[4]);
    swap_l5(v[1], v[5]);
    swap_l5(v[2], v[6]);
    swap_l5(v[3], v[7]);
}
// X3: s0 <-> l4, s1 <-> l5 (its own inverse)
template <class C>
__device__ __forceinline__ void shuffle_x3(C (&v)[8]) {
    swap_l4(v[0], v[1]);
    swap_l4(v[2], v[3]);
    swap_l4(v[4], v[5]);
    swap_l4(v[6], v[7]);
    swap_l5(v[0], v[2]);
    swap_l5(v[1], v[3]);
    swap_l5(v[4], v[6]);
    swap_l5(v[5], v[7]);
}

// --- X2: the cross-wave exchange through LDS ----------------------------------
// positions held in states B and C (see the table above)
__device__ __forceinline__ int shuffle_pos_b(int tid, int m) {
    const int lam = tid & 63, om = tid >> 6;
    return ((lam >> 1) & 7) | (om << 3) | ((m & 1) << 7) | (((m >> 1) & 1) << 5) | (((m >> 2) & 1) << 6) |
           (((lam >> 4) & 1) << 8) | (((lam >> 5) & 1) << 9);
}
__device__ __forceinline__ int shuffle_pos_c(int tid, int m) {
    const int lam = tid & 63, om = tid >> 6;
    return (((lam >> 1) & 7) << 7) | (om << 5) | ((lam >> 4) & 1) | (((lam >> 5) & 1) << 1) | ((m & 1) << 3) |
           (((m >> 1) & 1) << 4) | (((m >> 2) & 1) << 2);
}
// LDS slot of position p of line `line` (two lines of 1024 complex64): the low
// five bits are XORed with H(j = p >> 7, line), which leaves every ds_write_b64
// 16-lane group and ds_read_b64 32-lane group of both X2 directions on
// distinct banks (tools/shuffle_fft_model.py: 0 extra cycles)
__device__ __forceinline__ int shuffle_slot(int p, int line) {
    const int j0 = (p >> 7) & 1, j1 = (p >> 8) & 1, j2 = (p >> 9) & 1;
    const int h = j2 | (j0 << 1) | (j1 << 2) | ((line ^ j2) << 3) | ((j2 ^ j1) << 4);
    return line * kShufN + (p ^ h);
}
template <bool B_TO_C, class C>
__device__ __forceinline__ void shuffle_x2(C (&v)[8], int tid, float2* buf) {
    const int line = tid & 1;
    static_for<8>([&](auto mc) {
        constexpr int m = decltype(mc)::value;
        buf[shuffle_slot(B_TO_C ? shuffle_pos_b(tid, m) : shuffle_pos_c(tid, m), line)] = cv<float2>(v[m]);
    });
    lds_barrier();
    static_for<8>([&](auto mc) {
        constexpr int m = decltype(mc)::value;
        v[m] = cv<C>(buf[shuffle_slot(B_TO_C ? shuffle_pos_c(tid, m) : shuffle_pos_b(tid, m), line)]);
    });
}

// --- passes -------------------------------------------------------------------
// DIF: butterfly, then twiddle; DIT (adjoint): twiddle, then butterfly.
template <bool INV, class C>
__device__ __forceinline__ C tw_mul(C a, C w) {
    return INV ? cmulc(a, w) : cmul(a, w);
}
// radix-4 butterflies over slots {base + stride d}, twiddles w[0..2] after (DIF) or before (DIT)
template <bool INV, bool DIF, int BASE, int STRIDE, class C>
__device__ __forceinline__ void shuffle_r4(C (&v)[8], const C* w) {
    C u[4];
    static_for<4>([&](auto dc) {
        constexpr int d = decltype(dc)::value;
        u[d] = v[BASE + STRIDE * d];
    });
    if constexpr (!DIF) {
        static_for<3>([&](auto rc) {
            constexpr int r = decltype(rc)::value + 1;
            u[r] = tw_mul<INV>(u[r], w[r - 1]);
        });
    }
    Dft<4, INV, C>::run(u);
    if constexpr (DIF) {
        static_for<3>([&](auto rc) {
            constexpr int r = decltype(rc)::value + 1;
            u[r] = tw_mul<INV>(u[r], w[r - 1]);
        });
    }
    static_for<4>([&](auto dc) {
        constexpr int d = decltype(dc)::value;
        v[BASE + STRIDE * d] = u[d];
    });
}
template <bool INV, bool DIF, class C>
__device__ __forceinline__ void shuffle_p1(C (&v)[8], const ShuffleTwT<C>& tw) {
    if constexpr (!DIF) {
        static_for<7>([&](auto rc) {
            constexpr int r = decltype(rc)::value + 1;
            v[r] = tw_mul<INV>(v[r], tw.p1[r - 1]);
        });
    }
    Dft<8, INV, C>::run(v);
    if constexpr (DIF) {
        static_for<7>([&](auto rc) {
            constexpr int r = decltype(rc)::value + 1;
            v[r] = tw_mul<INV>(v[r], tw.p1[r - 1]);
        });
    }
}
template <bool INV, bool DIF, class C>
__device__ __forceinline__ void shuffle_p2(C (&v)[8], const ShuffleTwT<C>& tw) {
    shuffle_r4<INV, DIF, 0, 2>(v, tw.p2);  // s0 = 0: slots 0, 2, 4, 6
    shuffle_r4<INV, DIF, 1, 2>(v, tw.p2);  // s0 = 1
}
template <bool INV, bool DIF, class C>
__device__ __forceinline__ void shuffle_p3(C (&v)[8], const ShuffleTwT<C>& tw) {
    shuffle_r4<INV, DIF, 0, 1>(v, tw.p3);      // s2 = 0: slots 0..3
    shuffle_r4<INV, DIF, 4, 1>(v, tw.p3 + 3);  // s2 = 1: slots 4..7
}

// First transform of a pair (INV, decimated in frequency): state A in, state
// D out -- slot m of the thread then holds element (frequency) t + 128 m.
// Every thread of the workgroup must call it (LDS barrier); lds: 2048 complex64.
template <bool INV, class C>
__device__ __forceinline__ void shuffle_first_scalar(C (&v)[8], int tid, const ShuffleTwT<C>& tw, float2* lds) {
    shuffle_p1<INV, true>(v, tw);
    shuffle_x1(v);
    shuffle_p2<INV, true>(v, tw);
    shuffle_x2<true>(v, tid, lds);
    shuffle_p3<INV, true>(v, tw);
    shuffle_x3(v);
    Dft<8, INV, C>::run(v);
}
// Second transform (INV, decimated in time, the adjoint schedule): state D in,
// state A out. lds: 2048 complex64, not the buffer of the first transform
// (one barrier per exchange then suffices).
template <bool INV, class C>
__device__ __forceinline__ void shuffle_second_scalar(C (&v)[8], int tid, const ShuffleTwT<C>& tw, float2* lds) {
    Dft<8, INV, C>::run(v);
    shuffle_x3(v);
    shuffle_p3<INV, false>(v, tw);
    shuffle_x2<false>(v, tid, lds);
    shuffle_p2<INV, false>(v, tw);
    shuffle_x1(v);
    shuffle_p1<INV, false>(v, tw);
}

// First / second transform on complex64 slots v in the arithmetic type C of
// the twiddles (float32: in place; float64: widened for the transform and
// rounded back to complex64 after it).
template <bool INV, class C>
__device__ __forceinline__ void shuffle_first(float2 (&v)[8], int tid, const ShuffleTwT<C>& tw, float2* lds) {
    if constexpr (std::is_same_v<C, float2>) {
        shuffle_first_scalar<INV>(v, tid, tw, lds);
    } else {
        C u[8];
        static_for<8>([&](auto mc) { u[decltype(mc)::value] = cv<C>(v[decltype(mc)::value]); });
        shuffle_first_scalar<INV>(u, tid, tw, lds);
        static_for<8>([&](auto mc) { v[decltype(mc)::value] = cv<float2>(u[decltype(mc)::value]); });
    }
}
template <bool INV, class C>
__device__ __forceinline__ void shuffle_second(float2 (&v)[8], int tid, const ShuffleTwT<C>& tw, float2* lds) {
    if constexpr (std::is_same_v<C, float2>) {
        shuffle_second_scalar<INV>(v, tid, tw, lds);
    } else {
        C u[8];
        static_for<8>([&](auto mc) { u[decltype(mc)::value] = cv<C>(v[decltype(mc)::value]); });
        shuffle_second_scalar<INV>(u, tid, tw, lds);
        static_for<8>([&](auto mc) { v[decltype(mc)::value] = cv<float2>(u[decltype(mc)::value]); });
    }
}

// Transform (INV1), epi(0, m, z) on every output (slot m = element t + 128 m,
// z in the arithmetic type C), transform (INV2); v in state A in and out
// (complex64). lds: 2 x 2048 complex64.
template <bool INV1, bool INV2, class C, class Epi>
__device__ __forceinline__ void shuffle_pair(float2 (&v)[8], int tid, const ShuffleTwT<C>& tw, float2* lds, Epi&& epi) {
    C u[8];
    static_for<8>([&](auto mc) { u[decltype(mc)::value] = cv<C>(v[decltype(mc)::value]); });
    shuffle_first_scalar<INV1>(u, tid, tw, lds);
    static_for<8>([&](auto mc) {
        constexpr int m = decltype(mc)::value;
        epi(0, m, u[m]);
    });
    shuffle_second_scalar<INV2>(u, tid, tw, lds + 2 * kShufN);
    static_for<8>([&](auto mc) { v[decltype(mc)::value] = cv<float2>(u[decltype(mc)::value]); });
}

}  // namespace slm
