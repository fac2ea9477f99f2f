// Radix plans for the 1-D C2C transforms used along image rows and columns.
//
// Shared by host (twiddle-table construction) and device (kernel templates), so
// the two can never disagree on pass order. A plan for length N keeps E complex
// values per thread (T = N / E threads per line) and runs one Stockham pass per
// radix; every radix divides E so each pass is E / R butterflies per thread.
//
// The reference computes these transforms with scipy.fft.fft2 / ifft2
// (pocketfft, src/algorithms.py:27,31,34,84,88); SURVEY.md section 8a row a12.
#pragma once

namespace slm {

struct RadixPlan {
    int n;        // transform length
    int e;        // complex elements held per thread
    int variant;  // 0 = wide (16-24 elements per thread), 1 = narrow (twice the threads)
    int npass;    // number of Stockham passes
    int r[8];     // radices, first pass first
    // Mixed plans (ep[0] != 0, complex64 radix kernels only, radix_c128.hpp):
    // elements per thread of each pass; pass k runs n / ep[k] threads (the line
    // has n / e of them, e = the smallest ep[k]), each holding whole radix-r[k]
    // butterflies, and the inverse runs the passes in reverse order.
    int ep[8];
};

// Lengths the library supports along either image axis. 768 = 3 * 256 is the
// SLM height of the reference CLI (src/constants.py:5-6).
// Kernel templates are keyed by the index into this table (the "plan key").
// Wide plans minimise passes; narrow plans halve the work per thread so a
// single small image still puts several waves on every SIMD. First and last
// radix are equal wherever the length allows, so the projection between an
// inverse and a forward transform runs inside one butterfly group
// (fft_core.hpp, fft_pair).
// 4096: 32 elements per thread in radix-8 passes (512-thread column tiles,
// no float64 spills)
constexpr RadixPlan kPlans[] = {
    {64, 8, 0, 2, {8, 8, 0, 0}},
    {128, 16, 0, 3, {4, 8, 4, 0}},
    {256, 16, 0, 2, {16, 16, 0, 0}},
    {512, 16, 0, 3, {16, 2, 16, 0}},
    {768, 24, 0, 3, {8, 12, 8, 0}},
    {1024, 16, 0, 3, {16, 4, 16, 0}},
    {2048, 16, 0, 3, {16, 8, 16, 0}},
    {4096, 32, 0, 4, {8, 8, 8, 8}},
    {256, 8, 1, 3, {8, 4, 8, 0}},
    {512, 8, 1, 3, {8, 8, 8, 0}},
    {768, 12, 1, 4, {4, 12, 4, 4}},
    {1024, 8, 1, 4, {8, 4, 4, 8}},
    {2048, 8, 1, 4, {8, 4, 8, 8}},
    {4096, 16, 1, 3, {16, 16, 16, 0}},
    // complex128 radix-plan kernels only (radix_c128.hpp; variant 2 is never
    // picked by the float32 engine): 4096 in radix-8 passes, 512 threads per
    // line -- 8 double2 per thread leave the register file room for 16 waves
    // per CU where the E = 16 plan holds 8
    {4096, 8, 2, 4, {8, 8, 8, 8}},
    // complex64 radix kernels of the any-size engine only (radix_c128.hpp at
    // float32, variant 3): 13-smooth SLM panel sides, as mixed plans (ep[]:
    // with one E for every pass, a side with the factors 3 and 5 needed a
    // multiple of 15 elements per thread -- 1920 ran 2.2.2.30.2.2.2 on 64
    // threads, 1080 6.5.6.6 on 36; profiles/r06/speed_c64_n.txt).
    {600, 6, 3, 3, {10, 6, 10}, {10, 6, 10}},  // 100 threads (60 in the radix-10 passes)
    {800, 8, 3, 3, {10, 8, 10}, {10, 8, 10}},  // 100 threads (80)
    {1000, 10, 3, 3, {10, 10, 10}},
    // 1080 = 12.6.15: 90 threads per line (72 in the radix-15 pass), 3 passes
    // where the single-E plan 6.5.6.6 needed 30 elements on 36 threads
    {1080, 12, 3, 3, {12, 6, 15}, {12, 12, 15}},
    {1152, 8, 3, 3, {12, 8, 12}, {12, 8, 12}},  // 144 threads (96)
    {1200, 10, 3, 3, {10, 12, 10}, {10, 12, 10}},  // 120 threads (100 in the radix-12 pass)
    {1280, 10, 3, 3, {16, 5, 16}, {16, 10, 16}},  // 128 threads (80 in the radix-16 passes)
    {1536, 12, 3, 3, {16, 6, 16}, {16, 12, 16}},  // 128 threads (96)
    // 1920 = 15.16.8: 128 threads per line (120 in the radix-16 / 8 passes), 3
    // passes where the single-E plan 2.2.2.30.2.2.2 ran 7 on 64 threads
    {1920, 15, 3, 3, {15, 16, 8}, {15, 16, 16}},
    // variant 4 (A/B, $SLM_RZ_PANEL=alt): 1920 = 8.16.15 on 240 threads (120 / 128
    // in the radix-16 / 15 passes)
    {1920, 8, 4, 3, {8, 16, 15}, {8, 16, 15}},
};
constexpr int kNumPlans = sizeof(kPlans) / sizeof(kPlans[0]);
// plan keys of the float32 engine (kernels_inst.hip, dispatch.hpp, Makefile LENGTHS)
constexpr int kNumF32Plans = 14;

constexpr int plan_index(int n, int variant = 0) {
    for (int i = 0; i < kNumPlans; ++i)
        if (kPlans[i].n == n && kPlans[i].variant == variant) return i;
    return -1;
}

// Number of twiddle entries of a plan: every pass after the first holds
// (R - 1) * Ns entries, entry [(r - 1) * Ns + j] = exp(-2 pi i j r / (Ns R)).
constexpr int twiddle_count_key(int key) {
    int ns = 1, total = 0;
    for (int k = 0; k < kPlans[key].npass; ++k) {
        if (ns > 1) total += (kPlans[key].r[k] - 1) * ns;
        ns *= kPlans[key].r[k];
    }
    return total;
}
constexpr bool plan_mixed(int key) { return kPlans[key].ep[0] != 0; }
// radix of pass p in transform order (mixed plans: the inverse runs backwards)
constexpr int pass_radix(int key, bool rev, int p) {
    return kPlans[key].r[rev ? kPlans[key].npass - 1 - p : p];
}
// the same table layout for the reversed pass order of a mixed plan, stored
// after the forward order's entries
constexpr int twiddle_count_rev(int key) {
    int ns = 1, total = 0;
    for (int k = 0; k < kPlans[key].npass; ++k) {
        if (ns > 1) total += (pass_radix(key, true, k) - 1) * ns;
        ns *= pass_radix(key, true, k);
    }
    return total;
}
constexpr int twiddle_count_all(int key) {
    return twiddle_count_key(key) + (plan_mixed(key) ? twiddle_count_rev(key) : 0);
}

// Padded LDS footprint of one line (one extra complex slot per 16).
constexpr int lds_line(int n) { return n + n / 16; }

}  // namespace slm
