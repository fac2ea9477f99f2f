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
    int npass;    // number of Stockham passes
    int r[4];     // radices, first pass first
};

// Lengths the library supports along either image axis. 768 = 3 * 256 is the
// SLM height of the reference CLI (src/constants.py:5-6).
constexpr RadixPlan kPlans[] = {
    {64, 8, 2, {8, 8, 0, 0}},
    {128, 16, 2, {16, 8, 0, 0}},
    {256, 16, 2, {16, 16, 0, 0}},
    {512, 16, 3, {16, 16, 2, 0}},
    {768, 24, 3, {12, 8, 8, 0}},
    {1024, 16, 3, {16, 16, 4, 0}},
    {2048, 16, 3, {16, 16, 8, 0}},
    {4096, 16, 3, {16, 16, 16, 0}},
};
constexpr int kNumPlans = sizeof(kPlans) / sizeof(kPlans[0]);

constexpr int plan_index(int n) {
    for (int i = 0; i < kNumPlans; ++i)
        if (kPlans[i].n == n) return i;
    return -1;
}

// Number of twiddle entries of a plan: every pass after the first holds
// (R - 1) * Ns entries, entry [(r - 1) * Ns + j] = exp(-2 pi i j r / (Ns R)).
constexpr int twiddle_count(int n) {
    const int p = plan_index(n);
    if (p < 0) return 0;
    int ns = 1, total = 0;
    for (int k = 0; k < kPlans[p].npass; ++k) {
        if (ns > 1) total += (kPlans[p].r[k] - 1) * ns;
        ns *= kPlans[p].r[k];
    }
    return total;
}

// Padded LDS footprint of one line (one extra complex slot per 16).
constexpr int lds_line(int n) { return n + n / 16; }

}  // namespace slm
