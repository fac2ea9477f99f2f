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

struct ShuffleTw {
    float2 p1[7];  // w_1024^(t k1), k1 = 1..7
    float2 p2[3];  // w_128^((t & 31) k2), k2 = 1..3
    float2 p3[6];  // w_32^(n k3), n = l4 + 2 l5 + 4 s2, [3 s2 + k3 - 1]
};

__device__ __forceinline__ void load_shuffle_tw(ShuffleTw& tw, int tid, const float2* __restrict__ roots) {
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
// X1: s1 <-> l4, s2 <-> l5 (its own inverse)
__device__ __forceinline__ void shuffle_x1(float2 (&v)[8]) {
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
__device__ __forceinline__ void shuffle_x3(float2 (&v)[8]) {
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
template <bool B_TO_C>
__device__ __forceinline__ void shuffle_x2(float2 (&v)[8], int tid, float2* buf) {
    const int line = tid & 1;
    static_for<8>([&](auto mc) {
        constexpr int m = decltype(mc)::value;
        buf[shuffle_slot(B_TO_C ? shuffle_pos_b(tid, m) : shuffle_pos_c(tid, m), line)] = v[m];
    });
    lds_barrier();
    static_for<8>([&](auto mc) {
        constexpr int m = decltype(mc)::value;
        v[m] = buf[shuffle_slot(B_TO_C ? shuffle_pos_c(tid, m) : shuffle_pos_b(tid, m), line)];
    });
}

// --- passes -------------------------------------------------------------------
// DIF: butterfly, then twiddle; DIT (adjoint): twiddle, then butterfly.
template <bool INV>
__device__ __forceinline__ float2 tw_mul(float2 a, float2 w) {
    return INV ? cmulc(a, w) : cmul(a, w);
}
// radix-4 butterflies over slots {base + stride d}, twiddles w[0..2] after (DIF) or before (DIT)
template <bool INV, bool DIF, int BASE, int STRIDE>
__device__ __forceinline__ void shuffle_r4(float2 (&v)[8], const float2* w) {
    float2 u[4];
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
    Dft<4, INV, float2>::run(u);
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
template <bool INV, bool DIF>
__device__ __forceinline__ void shuffle_p1(float2 (&v)[8], const ShuffleTw& tw) {
    if constexpr (!DIF) {
        static_for<7>([&](auto rc) {
            constexpr int r = decltype(rc)::value + 1;
            v[r] = tw_mul<INV>(v[r], tw.p1[r - 1]);
        });
    }
    Dft<8, INV, float2>::run(v);
    if constexpr (DIF) {
        static_for<7>([&](auto rc) {
            constexpr int r = decltype(rc)::value + 1;
            v[r] = tw_mul<INV>(v[r], tw.p1[r - 1]);
        });
    }
}
template <bool INV, bool DIF>
__device__ __forceinline__ void shuffle_p2(float2 (&v)[8], const ShuffleTw& tw) {
    shuffle_r4<INV, DIF, 0, 2>(v, tw.p2);  // s0 = 0: slots 0, 2, 4, 6
    shuffle_r4<INV, DIF, 1, 2>(v, tw.p2);  // s0 = 1
}
template <bool INV, bool DIF>
__device__ __forceinline__ void shuffle_p3(float2 (&v)[8], const ShuffleTw& tw) {
    shuffle_r4<INV, DIF, 0, 1>(v, tw.p3);      // s2 = 0: slots 0..3
    shuffle_r4<INV, DIF, 4, 1>(v, tw.p3 + 3);  // s2 = 1: slots 4..7
}

// First transform of a pair (INV, decimated in frequency): state A in, state
// D out -- slot m of the thread then holds element (frequency) t + 128 m.
// Every thread of the workgroup must call it (LDS barrier); lds: 2048 complex64.
template <bool INV>
__device__ __forceinline__ void shuffle_first_scalar(float2 (&v)[8], int tid, const ShuffleTw& tw, float2* lds) {
    shuffle_p1<INV, true>(v, tw);
    shuffle_x1(v);
    shuffle_p2<INV, true>(v, tw);
    shuffle_x2<true>(v, tid, lds);
    shuffle_p3<INV, true>(v, tw);
    shuffle_x3(v);
    Dft<8, INV, float2>::run(v);
}
// Second transform (INV, decimated in time, the adjoint schedule): state D in,
// state A out. lds: 2048 complex64, not the buffer of the first transform
// (one barrier per exchange then suffices).
template <bool INV>
__device__ __forceinline__ void shuffle_second_scalar(float2 (&v)[8], int tid, const ShuffleTw& tw, float2* lds) {
    Dft<8, INV, float2>::run(v);
    shuffle_x3(v);
    shuffle_p3<INV, false>(v, tw);
    shuffle_x2<false>(v, tid, lds);
    shuffle_p2<INV, false>(v, tw);
    shuffle_x1(v);
    shuffle_p1<INV, false>(v, tw);
}

// --- packed float32 arithmetic ----------------------------------------------
// gfx950 executes v_pk_add_f32 / v_pk_mul_f32 / v_pk_fma_f32 on (re, im) pairs
// at the issue rate of one scalar instruction, with per-half source selects
// (op_sel) and negations, so a complex add is one instruction instead of two
// and a complex product two instead of four. The butterflies below are the
// same DFTs as fft_core.hpp's Dft<4> / Dft<8> (same additions in the same
// order); products round as fma(x, a, -(y b)) / fma(x, b, y a) (scalar
// contraction was the compiler's choice per site). Off by default: measured
// neutral at 1024^2 (column pass 8.62 against 8.57 us, row 7.84 / 7.89 us;
// the pair is bound by its loads and exchanges, not by VALU issue) with a
// smaller float32 margin on the 200-iteration gate (6.54e-6 against 5.75e-6),
// profiles/r04/ab_packed_s5.txt. -DSLM_PACKED=1 builds it (A/B).
#ifndef SLM_PACKED
#define SLM_PACKED 0
#endif
typedef float pk2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ pk2 to_pk(float2 a) {
    pk2 r;
    r.x = a.x;
    r.y = a.y;
    return r;
}
__device__ __forceinline__ float2 from_pk(pk2 a) { return make_float2(a.x, a.y); }
__device__ __forceinline__ pk2 pk_fma(pk2 a, pk2 b, pk2 c) { return __builtin_elementwise_fma(a, b, c); }
// a * w
__device__ __forceinline__ pk2 pk_mul(pk2 a, pk2 w) {
    pk2 t = a.yy * w.yx;  // (y wy, y wx)
    t.x = -t.x;
    return pk_fma(a.xx, w, t);
}
// a * conj(w)
__device__ __forceinline__ pk2 pk_mulc(pk2 a, pk2 w) {
    pk2 t = a.yx * w.yy;  // (y wy, x wy)
    t.y = -t.y;
    return pk_fma(a, w.xx, t);
}
// times the constant exp(-+2 pi i K / R) (fft_core.hpp, twc)
template <int K, int R, bool INV>
__device__ __forceinline__ pk2 pk_twc(pk2 a) {
    constexpr int q = ((48 / R) * K) % 48;
    if constexpr (q == 0) {
        return a;
    } else if constexpr (q == 24) {
        return -a;
    } else if constexpr (q == 12 || q == 36) {  // forward q = 12: * (-i); q = 36: * (+i)
        constexpr bool minus_i = (q == 12) != INV;
        pk2 r = a.yx;
        if constexpr (minus_i)
            r.y = -r.y;  // (y, -x)
        else
            r.x = -r.x;  // (-y, x)
        return r;
    } else {
        constexpr float c = (float)cos48(q);
        constexpr float sn = (float)(INV ? sin48(q) : -sin48(q));
        pk2 cs;
        cs.x = c;
        cs.y = sn;
        pk2 t = a.yy * cs.yx;  // (y s, y c)
        t.x = -t.x;
        return pk_fma(a.xx, cs, t);
    }
}
template <bool INV>
__device__ __forceinline__ void pk_dft4(pk2* v) {
    const pk2 a = v[0] + v[2], b = v[0] - v[2], c = v[1] + v[3];
    const pk2 d = pk_twc<1, 4, INV>(v[1] - v[3]);
    v[0] = a + c;
    v[2] = a - c;
    v[1] = b + d;
    v[3] = b - d;
}
// 8 = 2 x 4 (fft_core.hpp, dft_split<2, 4>)
template <bool INV>
__device__ __forceinline__ void pk_dft8(pk2* v) {
    pk2 z[8];
    static_for<4>([&](auto n2c) {
        constexpr int n2 = decltype(n2c)::value;
        const pk2 a = v[n2], b = v[4 + n2];
        z[n2 * 2 + 0] = a + b;
        z[n2 * 2 + 1] = pk_twc<n2, 8, INV>(a - b);
    });
    static_for<2>([&](auto k1c) {
        constexpr int k1 = decltype(k1c)::value;
        pk2 row[4] = {z[k1], z[2 + k1], z[4 + k1], z[6 + k1]};
        pk_dft4<INV>(row);
        static_for<4>([&](auto k2c) {
            constexpr int k2 = decltype(k2c)::value;
            v[k1 + 2 * k2] = row[k2];
        });
    });
}
template <bool INV>
__device__ __forceinline__ pk2 pk_tw(pk2 a, float2 w) {
    return INV ? pk_mulc(a, to_pk(w)) : pk_mul(a, to_pk(w));
}
__device__ __forceinline__ void pk_swap_l4(pk2& a, pk2& b) {
    const auto x = __builtin_amdgcn_permlane16_swap(as_u(a.x), as_u(b.x), false, false);
    const auto y = __builtin_amdgcn_permlane16_swap(as_u(a.y), as_u(b.y), false, false);
    a.x = as_f(x[0]);
    a.y = as_f(y[0]);
    b.x = as_f(x[1]);
    b.y = as_f(y[1]);
}
__device__ __forceinline__ void pk_swap_l5(pk2& a, pk2& b) {
    const auto x = __builtin_amdgcn_permlane32_swap(as_u(a.x), as_u(b.x), false, false);
    const auto y = __builtin_amdgcn_permlane32_swap(as_u(a.y), as_u(b.y), false, false);
    a.x = as_f(x[0]);
    a.y = as_f(y[0]);
    b.x = as_f(x[1]);
    b.y = as_f(y[1]);
}
__device__ __forceinline__ void pk_x1(pk2 (&v)[8]) {
    pk_swap_l4(v[0], v[2]);
    pk_swap_l4(v[1], v[3]);
    pk_swap_l4(v[4], v[6]);
    pk_swap_l4(v[5], v[7]);
    pk_swap_l5(v[0], v[4]);
    pk_swap_l5(v[1], v[5]);
    pk_swap_l5(v[2], v[6]);
    pk_swap_l5(v[3], v[7]);
}
__device__ __forceinline__ void pk_x3(pk2 (&v)[8]) {
    pk_swap_l4(v[0], v[1]);
    pk_swap_l4(v[2], v[3]);
    pk_swap_l4(v[4], v[5]);
    pk_swap_l4(v[6], v[7]);
    pk_swap_l5(v[0], v[2]);
    pk_swap_l5(v[1], v[3]);
    pk_swap_l5(v[4], v[6]);
    pk_swap_l5(v[5], v[7]);
}
template <bool B_TO_C>
__device__ __forceinline__ void pk_x2(pk2 (&v)[8], int tid, float2* buf) {
    const int line = tid & 1;
    pk2* b = reinterpret_cast<pk2*>(buf);
    static_for<8>([&](auto mc) {
        constexpr int m = decltype(mc)::value;
        b[shuffle_slot(B_TO_C ? shuffle_pos_b(tid, m) : shuffle_pos_c(tid, m), line)] = v[m];
    });
    lds_barrier();
    static_for<8>([&](auto mc) {
        constexpr int m = decltype(mc)::value;
        v[m] = b[shuffle_slot(B_TO_C ? shuffle_pos_c(tid, m) : shuffle_pos_b(tid, m), line)];
    });
}
template <bool INV, bool DIF, int BASE, int STRIDE>
__device__ __forceinline__ void pk_r4(pk2 (&v)[8], const float2* w) {
    pk2 u[4];
    static_for<4>([&](auto dc) {
        constexpr int d = decltype(dc)::value;
        u[d] = v[BASE + STRIDE * d];
    });
    if constexpr (!DIF) {
        static_for<3>([&](auto rc) {
            constexpr int r = decltype(rc)::value + 1;
            u[r] = pk_tw<INV>(u[r], w[r - 1]);
        });
    }
    pk_dft4<INV>(u);
    if constexpr (DIF) {
        static_for<3>([&](auto rc) {
            constexpr int r = decltype(rc)::value + 1;
            u[r] = pk_tw<INV>(u[r], w[r - 1]);
        });
    }
    static_for<4>([&](auto dc) {
        constexpr int d = decltype(dc)::value;
        v[BASE + STRIDE * d] = u[d];
    });
}
template <bool INV, bool DIF>
__device__ __forceinline__ void pk_p1(pk2 (&v)[8], const ShuffleTw& tw) {
    if constexpr (!DIF) {
        static_for<7>([&](auto rc) {
            constexpr int r = decltype(rc)::value + 1;
            v[r] = pk_tw<INV>(v[r], tw.p1[r - 1]);
        });
    }
    pk_dft8<INV>(v);
    if constexpr (DIF) {
        static_for<7>([&](auto rc) {
            constexpr int r = decltype(rc)::value + 1;
            v[r] = pk_tw<INV>(v[r], tw.p1[r - 1]);
        });
    }
}
template <bool INV, bool DIF>
__device__ __forceinline__ void pk_p2(pk2 (&v)[8], const ShuffleTw& tw) {
    pk_r4<INV, DIF, 0, 2>(v, tw.p2);
    pk_r4<INV, DIF, 1, 2>(v, tw.p2);
}
template <bool INV, bool DIF>
__device__ __forceinline__ void pk_p3(pk2 (&v)[8], const ShuffleTw& tw) {
    pk_r4<INV, DIF, 0, 1>(v, tw.p3);
    pk_r4<INV, DIF, 4, 1>(v, tw.p3 + 3);
}
template <bool INV>
__device__ __forceinline__ void pk_first(pk2 (&v)[8], int tid, const ShuffleTw& tw, float2* lds) {
    pk_p1<INV, true>(v, tw);
    pk_x1(v);
    pk_p2<INV, true>(v, tw);
    pk_x2<true>(v, tid, lds);
    pk_p3<INV, true>(v, tw);
    pk_x3(v);
    pk_dft8<INV>(v);
}
template <bool INV>
__device__ __forceinline__ void pk_second(pk2 (&v)[8], int tid, const ShuffleTw& tw, float2* lds) {
    pk_dft8<INV>(v);
    pk_x3(v);
    pk_p3<INV, false>(v, tw);
    pk_x2<false>(v, tid, lds);
    pk_p2<INV, false>(v, tw);
    pk_x1(v);
    pk_p1<INV, false>(v, tw);
}
__device__ __forceinline__ void pk_load(pk2 (&w)[8], const float2 (&v)[8]) {
    static_for<8>([&](auto mc) { w[decltype(mc)::value] = to_pk(v[decltype(mc)::value]); });
}
__device__ __forceinline__ void pk_store(float2 (&v)[8], const pk2 (&w)[8]) {
    static_for<8>([&](auto mc) { v[decltype(mc)::value] = from_pk(w[decltype(mc)::value]); });
}

// Transform (INV1), epi(0, m, z) on every output (slot m = element t + 128 m),
// transform (INV2); v in state A in and out. lds: 2 x 2048 complex64.
template <bool INV>
__device__ __forceinline__ void shuffle_first(float2 (&v)[8], int tid, const ShuffleTw& tw, float2* lds) {
#if SLM_PACKED
    pk2 w[8];
    pk_load(w, v);
    pk_first<INV>(w, tid, tw, lds);
    pk_store(v, w);
#else
    shuffle_first_scalar<INV>(v, tid, tw, lds);
#endif
}
template <bool INV>
__device__ __forceinline__ void shuffle_second(float2 (&v)[8], int tid, const ShuffleTw& tw, float2* lds) {
#if SLM_PACKED
    pk2 w[8];
    pk_load(w, v);
    pk_second<INV>(w, tid, tw, lds);
    pk_store(v, w);
#else
    shuffle_second_scalar<INV>(v, tid, tw, lds);
#endif
}

template <bool INV1, bool INV2, class Epi>
__device__ __forceinline__ void shuffle_pair(float2 (&v)[8], int tid, const ShuffleTw& tw, float2* lds, Epi&& epi) {
    shuffle_first<INV1>(v, tid, tw, lds);
    static_for<8>([&](auto mc) {
        constexpr int m = decltype(mc)::value;
        epi(0, m, v[m]);
    });
    shuffle_second<INV2>(v, tid, tw, lds + 2 * kShufN);
}

// ==========================================================================
// 4096-point rows (one row per 256-thread workgroup, 16 slots per thread,
// radices 16.16.16; tools/shuffle4096_model.py simulates the schedule):
//
//   A (load/store)  slots pos 8-11   lanes 0-5 = pos 0-5          waves = pos 6, 7
//   P1 radix 16, twiddle w_4096^(t k1)
//   X1 LDS (+ barrier)
//   B               slots pos 4-7    lanes 1, 3, 4, 5 = pos 0-3   lanes 0, 2, waves = pos 8-11
//   P2 radix 16, twiddle w_256^(n k2), n = pos 0-3
//   X2 registers:   slot bit 0 <-> lane bit 1 (quad_perm), slot bit 1 <-> lane
//                   bit 3 (row_ror:8 under bank masks), slot bit 2 <-> lane bit 4
//                   (v_permlane16_swap), slot bit 3 <-> lane bit 5 (v_permlane32_swap)
//   C               slots pos 0-3    lanes 1, 3, 4, 5 = pos 4-7
//   P3 radix 16: slot m holds frequency klow(tid) + 256 m.
// ==========================================================================
constexpr int kShuf4N = 4096;

__device__ __forceinline__ int lane_bit(int tid, int b) { return (tid >> b) & 1; }

// frequency index (minus 256 m) of the element in slot m after the first transform
__device__ __forceinline__ int shuffle4096_klow(int tid) {
    const int w = tid >> 6;
    return lane_bit(tid, 0) | (lane_bit(tid, 2) << 1) | ((w & 1) << 2) | (((w >> 1) & 1) << 3) |
           (lane_bit(tid, 1) << 4) | (lane_bit(tid, 3) << 5) | (lane_bit(tid, 4) << 6) | (lane_bit(tid, 5) << 7);
}

struct ShuffleTw4096 {
    float2 p1[15];  // w_4096^(t k1)
    float2 p2[15];  // w_256^(n k2), n = lane bits 1, 3, 4, 5
};

__device__ __forceinline__ void load_shuffle4096_tw(ShuffleTw4096& tw, int tid, const float2* __restrict__ roots) {
    const int n = lane_bit(tid, 1) | (lane_bit(tid, 3) << 1) | (lane_bit(tid, 4) << 2) | (lane_bit(tid, 5) << 3);
    static_for<15>([&](auto kc) {
        constexpr int k = decltype(kc)::value + 1;
        tw.p1[k - 1] = roots[tid * k];
        tw.p2[k - 1] = roots[16 * n * k];
    });
}

__device__ __forceinline__ int shuffle4096_pos_b(int tid, int m) {
    const int w = tid >> 6;
    return lane_bit(tid, 1) | (lane_bit(tid, 3) << 1) | (lane_bit(tid, 4) << 2) | (lane_bit(tid, 5) << 3) | (m << 4) |
           (lane_bit(tid, 0) << 8) | (lane_bit(tid, 2) << 9) | ((w & 1) << 10) | (((w >> 1) & 1) << 11);
}
// X1 slot map: p ^ H(p >> 8), H = j0 -> bit 3, j1 -> bits 2 and 4 (0 extra
// LDS cycles for both directions' 16-lane writes and 32-lane reads)
__device__ __forceinline__ int shuffle4096_slot(int p) {
    const int j0 = (p >> 8) & 1, j1 = (p >> 9) & 1;
    return p ^ ((j0 << 3) | (j1 << 2) | (j1 << 4));
}
template <bool A_TO_B>
__device__ __forceinline__ void shuffle4096_x1(float2 (&v)[16], int tid, float2* buf) {
    static_for<16>([&](auto mc) {
        constexpr int m = decltype(mc)::value;
        buf[shuffle4096_slot(A_TO_B ? (tid | (m << 8)) : shuffle4096_pos_b(tid, m))] = v[m];
    });
    lds_barrier();
    static_for<16>([&](auto mc) {
        constexpr int m = decltype(mc)::value;
        v[m] = buf[shuffle4096_slot(A_TO_B ? shuffle4096_pos_b(tid, m) : (tid | (m << 8)))];
    });
}

template <int CTRL>
__device__ __forceinline__ float dpp_f32(float x) {
    return as_f((unsigned)__builtin_amdgcn_update_dpp(0, (int)as_u(x), CTRL, 0xF, 0xF, false));
}
// slot pair (a: bit clear, c: bit set) <-> lane bit 1: partner lane = lane ^ 2 (quad_perm [2,3,0,1])
__device__ __forceinline__ void swap_l1(float2& a, float2& c, int x) {
    constexpr int kXor2 = 0x4E;
    const float2 pa = make_float2(dpp_f32<kXor2>(a.x), dpp_f32<kXor2>(a.y));
    const float2 pc = make_float2(dpp_f32<kXor2>(c.x), dpp_f32<kXor2>(c.y));
    const float2 na = x ? pc : a;
    const float2 nc = x ? c : pa;
    a = na;
    c = nc;
}
// slot pair <-> lane bit 3: partner lane = lane ^ 8 (row_ror:8); lanes with the
// bit set (banks 2, 3) replace a, lanes with it clear (banks 0, 1) replace c
__device__ __forceinline__ float dpp_ror8_banks(float old, float src, int banks_hi) {
    return banks_hi ? as_f((unsigned)__builtin_amdgcn_update_dpp((int)as_u(old), (int)as_u(src), 0x128, 0xF, 0xC, false))
                    : as_f((unsigned)__builtin_amdgcn_update_dpp((int)as_u(old), (int)as_u(src), 0x128, 0xF, 0x3, false));
}
__device__ __forceinline__ void swap_l3(float2& a, float2& c) {
    const float2 na = make_float2(dpp_ror8_banks(a.x, c.x, 1), dpp_ror8_banks(a.y, c.y, 1));
    const float2 nc = make_float2(dpp_ror8_banks(c.x, a.x, 0), dpp_ror8_banks(c.y, a.y, 0));
    a = na;
    c = nc;
}
// X2 (its own inverse): the four slot bits <-> lane bits 1, 3, 4, 5
__device__ __forceinline__ void shuffle4096_x2(float2 (&v)[16], int tid) {
    const int x1 = lane_bit(tid, 1);
    static_for<8>([&](auto ic) {
        constexpr int i = decltype(ic)::value;
        constexpr int m = 2 * i;  // slot bit 0 clear
        swap_l1(v[m], v[m | 1], x1);
    });
    static_for<8>([&](auto ic) {
        constexpr int i = decltype(ic)::value;
        constexpr int m = (i & 1) | ((i >> 1) << 2);  // slot bit 1 clear
        swap_l3(v[m], v[m | 2]);
    });
    static_for<8>([&](auto ic) {
        constexpr int i = decltype(ic)::value;
        constexpr int m = (i & 3) | ((i >> 2) << 3);  // slot bit 2 clear
        swap_l4(v[m], v[m | 4]);
    });
    static_for<8>([&](auto ic) {
        constexpr int m = decltype(ic)::value;  // slot bit 3 clear
        swap_l5(v[m], v[m | 8]);
    });
}

template <bool INV, bool DIF>
__device__ __forceinline__ void shuffle4096_r16(float2 (&v)[16], const float2* w) {
    if constexpr (!DIF) {
        static_for<15>([&](auto rc) {
            constexpr int r = decltype(rc)::value + 1;
            v[r] = tw_mul<INV>(v[r], w[r - 1]);
        });
    }
    Dft<16, INV, float2>::run(v);
    if constexpr (DIF) {
        static_for<15>([&](auto rc) {
            constexpr int r = decltype(rc)::value + 1;
            v[r] = tw_mul<INV>(v[r], w[r - 1]);
        });
    }
}

// Transform (INV1, DIF), epi(0, m, z) on slot m = element shuffle4096_klow(tid)
// + 256 m, transform (INV2, DIT); v in state A (element tid + 256 m) in and
// out. lds: 2 x 4096 complex64 (one buffer per X1 direction).
template <bool INV1, bool INV2, class Epi>
__device__ __forceinline__ void shuffle4096_pair(float2 (&v)[16], int tid, const ShuffleTw4096& tw, float2* lds,
                                                 Epi&& epi) {
    shuffle4096_r16<INV1, true>(v, tw.p1);
    shuffle4096_x1<true>(v, tid, lds);
    shuffle4096_r16<INV1, true>(v, tw.p2);
    shuffle4096_x2(v, tid);
    Dft<16, INV1, float2>::run(v);
    static_for<16>([&](auto mc) {
        constexpr int m = decltype(mc)::value;
        epi(0, m, v[m]);
    });
    Dft<16, INV2, float2>::run(v);
    shuffle4096_x2(v, tid);
    shuffle4096_r16<INV2, false>(v, tw.p2);
    shuffle4096_x1<false>(v, tid, lds + kShuf4N);
    shuffle4096_r16<INV2, false>(v, tw.p1);
}

}  // namespace slm
