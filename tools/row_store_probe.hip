// Access-shape probe of the 4096^2 row pass (csrc/kernels.hpp row_kernel,
// float32, one row per 256-thread workgroup, 16 elements per thread) on the
// blocked layout [b][x/4][y][x%4] (4-wide panels: a 128-B line = 4 rows x 4 x).
// Each kernel loads 16 complex64 per thread in one pattern and stores them back
// to a second buffer in the same pattern (no arithmetic), so the time is the
// memory pipeline's cost of that shape:
//   x2      lane t, element m at x = t + 256 m, 8-B accesses (the shipped row pass)
//   x4      element pairs (x, x+1), x = 2 t + 512 j, 16-B accesses
//   x8      panel rows (x .. x+3), x = 4 t + 1024 j, two 16-B accesses per row piece
//   quad    four rows per workgroup, 16 lanes per 128-B line (whole lines per
//           instruction; what a 4-row tile would issue)
//   wx4     loads as x2, stores as x4 (an LDS-staged output)
// Build: hipcc --offload-arch=gfx950 -O3 tools/row_store_probe.hip -o build/row_store_probe
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int N = 4096;

__device__ __forceinline__ long long blk(int y, int x) { return (long long)(x >> 2) * N * 4 + y * 4 + (x & 3); }

// csrc/kernels.hpp xcd_remap: consecutive logical rows on one XCD (one L2 merges a line's rows)
__device__ __forceinline__ int xcd_remap(int id, int n) {
    const int q = n >> 3, r = n & 7;
    const int xcd = id & 7, k = id >> 3;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + k;
}

template <int MODE_LD, int MODE_ST>
__global__ void __launch_bounds__(256) row_copy(const float2* __restrict__ in, float2* __restrict__ out) {
    const int id = xcd_remap(blockIdx.x, gridDim.x);
    const long long hoff = (long long)(id / N) * N * N;
    const int y = id % N, t = threadIdx.x;
    float2 v[16];
    if constexpr (MODE_LD == 0) {
#pragma unroll
        for (int m = 0; m < 16; ++m) v[m] = in[hoff + blk(y, t + 256 * m)];
    } else if constexpr (MODE_LD == 1) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const float4 q = *reinterpret_cast<const float4*>(in + hoff + blk(y, 2 * t + 512 * j));
            v[2 * j] = make_float2(q.x, q.y);
            v[2 * j + 1] = make_float2(q.z, q.w);
        }
    } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const float4* p = reinterpret_cast<const float4*>(in + hoff + blk(y, 4 * t + 1024 * j));
            const float4 q0 = p[0], q1 = p[1];
            v[4 * j] = make_float2(q0.x, q0.y);
            v[4 * j + 1] = make_float2(q0.z, q0.w);
            v[4 * j + 2] = make_float2(q1.x, q1.y);
            v[4 * j + 3] = make_float2(q1.z, q1.w);
        }
    }
    // keep the compiler from turning the copy into anything else
    asm volatile("" ::: "memory");
    if constexpr (MODE_ST == 0) {
#pragma unroll
        for (int m = 0; m < 16; ++m) out[hoff + blk(y, t + 256 * m)] = v[m];
    } else if constexpr (MODE_ST == 1) {
#pragma unroll
        for (int j = 0; j < 8; ++j)
            *reinterpret_cast<float4*>(out + hoff + blk(y, 2 * t + 512 * j)) =
                make_float4(v[2 * j].x, v[2 * j].y, v[2 * j + 1].x, v[2 * j + 1].y);
    } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            float4* p = reinterpret_cast<float4*>(out + hoff + blk(y, 4 * t + 1024 * j));
            p[0] = make_float4(v[4 * j].x, v[4 * j].y, v[4 * j + 1].x, v[4 * j + 1].y);
            p[1] = make_float4(v[4 * j + 2].x, v[4 * j + 2].y, v[4 * j + 3].x, v[4 * j + 3].y);
        }
    }
}

// four rows y0..y0+3, x in [xb, xb + 1024): lane l of wave w, element m covers
// row y0 + (l >> 2 & 3), x = xb + (l & 3) + 4 ((l >> 4) + 4 (w + 4 m))
__global__ void __launch_bounds__(256) quad_copy(const float2* __restrict__ in, float2* __restrict__ out) {
    const int per_holo = (N / 4) * 4;
    const int id = xcd_remap(blockIdx.x, gridDim.x);
    const long long hoff = (long long)(id / per_holo) * N * N;
    const int r = id % per_holo;
    const int y0 = (r >> 2) * 4, xb = (r & 3) * 1024;
    const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int y = y0 + ((l >> 2) & 3);
    float2 v[16];
#pragma unroll
    for (int m = 0; m < 16; ++m) v[m] = in[hoff + blk(y, xb + (l & 3) + 4 * ((l >> 4) + 4 * (w + 4 * m)))];
    asm volatile("" ::: "memory");
#pragma unroll
    for (int m = 0; m < 16; ++m) out[hoff + blk(y, xb + (l & 3) + 4 * ((l >> 4) + 4 * (w + 4 * m)))] = v[m];
}


// loads only (x2 or quad shape); the sum keeps them alive
template <bool QUAD>
__global__ void __launch_bounds__(256) read_only(const float2* __restrict__ in, float2* __restrict__ out) {
    const int id = xcd_remap(blockIdx.x, gridDim.x);
    const int l = threadIdx.x & 63, w = threadIdx.x >> 6, t = threadIdx.x;
    float2 acc = make_float2(0.f, 0.f);
    if constexpr (QUAD) {
        const int per_holo = N;
        const long long hoff = (long long)(id / per_holo) * N * N;
        const int r = id % per_holo, y0 = (r >> 2) * 4, xb = (r & 3) * 1024, y = y0 + ((l >> 2) & 3);
#pragma unroll
        for (int m = 0; m < 16; ++m) {
            const float2 v = in[hoff + blk(y, xb + (l & 3) + 4 * ((l >> 4) + 4 * (w + 4 * m)))];
            acc.x += v.x;
            acc.y += v.y;
        }
    } else {
        const long long hoff = (long long)(id / N) * N * N;
        const int y = id % N;
#pragma unroll
        for (int m = 0; m < 16; ++m) {
            const float2 v = in[hoff + blk(y, t + 256 * m)];
            acc.x += v.x;
            acc.y += v.y;
        }
    }
    if (acc.x == 12345.f) out[id] = acc;
}
// stores only
template <bool QUAD>
__global__ void __launch_bounds__(256) write_only(const float2* __restrict__ in, float2* __restrict__ out) {
    const int id = xcd_remap(blockIdx.x, gridDim.x);
    const int l = threadIdx.x & 63, w = threadIdx.x >> 6, t = threadIdx.x;
    const float2 v = make_float2((float)t, (float)id);
    if constexpr (QUAD) {
        const long long hoff = (long long)(id / N) * N * N;
        const int r = id % N, y0 = (r >> 2) * 4, xb = (r & 3) * 1024, y = y0 + ((l >> 2) & 3);
#pragma unroll
        for (int m = 0; m < 16; ++m) out[hoff + blk(y, xb + (l & 3) + 4 * ((l >> 4) + 4 * (w + 4 * m)))] = v;
    } else {
        const long long hoff = (long long)(id / N) * N * N;
        const int y = id % N;
#pragma unroll
        for (int m = 0; m < 16; ++m) out[hoff + blk(y, t + 256 * m)] = v;
    }
}
// two adjacent rows per thread (128 threads per row pair... 256 threads, 2 rows, 16 x each
// per row: x = t + 256 m), row pieces of one panel stored back to back (m-major)
__global__ void __launch_bounds__(256) pair_copy(const float2* __restrict__ in, float2* __restrict__ out) {
    const int id = xcd_remap(blockIdx.x, gridDim.x);
    const int per_holo = N / 2;
    const long long hoff = (long long)(id / per_holo) * N * N;
    const int y = (id % per_holo) * 2, t = threadIdx.x;
    float2 v[2][16];
#pragma unroll
    for (int m = 0; m < 16; ++m)
#pragma unroll
        for (int r = 0; r < 2; ++r) v[r][m] = in[hoff + blk(y + r, t + 256 * m)];
    asm volatile("" ::: "memory");
#pragma unroll
    for (int m = 0; m < 16; ++m)
#pragma unroll
        for (int r = 0; r < 2; ++r) out[hoff + blk(y + r, t + 256 * m)] = v[r][m];
}

// column tiles of the 4096 column pass (csrc/kernels.hpp col_kernel, two columns per
// thread): W columns of one 4-wide panel per workgroup, thread t at y = t + 256 m,
// 8 W bytes per (y, tile) -- W = 2: 16 B of every 32-B panel row (the shipped
// 2-column tile), W = 4: the whole panel row (a contiguous 128-KB stream)
template <int W>
__global__ void __launch_bounds__(256) col_copy(const float2* __restrict__ in, float2* __restrict__ out) {
    constexpr int TPP = 4 / W;  // tiles per panel
    const int id = xcd_remap(blockIdx.x, gridDim.x);
    const int per_holo = (N / 4) * TPP;
    const long long hoff = (long long)(id / per_holo) * N * N;
    const int r = id % per_holo, panel = r / TPP, c0 = (r % TPP) * W, t = threadIdx.x;
    const long long base = hoff + (long long)panel * N * 4 + c0;
    float4 v[16][W / 2];
#pragma unroll
    for (int m = 0; m < 16; ++m)
#pragma unroll
        for (int k = 0; k < W / 2; ++k) v[m][k] = *reinterpret_cast<const float4*>(in + base + (t + 256 * m) * 4 + 2 * k);
    asm volatile("" ::: "memory");
#pragma unroll
    for (int m = 0; m < 16; ++m)
#pragma unroll
        for (int k = 0; k < W / 2; ++k) *reinterpret_cast<float4*>(out + base + (t + 256 * m) * 4 + 2 * k) = v[m][k];
}

int main() {
    for (int B : {1, 8}) {
        const size_t bytes = (size_t)B * N * N * sizeof(float2);
        float2 *a, *b;
        if (hipMalloc(&a, bytes) != hipSuccess || hipMalloc(&b, bytes) != hipSuccess) return 1;
        (void)hipMemset(a, 1, bytes);
        (void)hipMemset(b, 0, bytes);
        hipEvent_t e0, e1;
        (void)hipEventCreate(&e0);
        (void)hipEventCreate(&e1);
        auto run = [&](auto kern, int grid, const char* name) {
            for (int i = 0; i < 3; ++i) hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, a, b);
            (void)hipEventRecord(e0);
            constexpr int reps = 20;
            for (int i = 0; i < reps; ++i) hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, a, b);
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            float ms = 0;
            (void)hipEventElapsedTime(&ms, e0, e1);
            const double us = ms * 1e3 / reps;
            printf("B=%d %-8s %8.1f us per launch  %7.1f GB/s (read+write)\n", B, name, us, 2.0 * bytes / (us * 1e-6) / 1e9);
        };
        const int grid = B * N;
        run(row_copy<0, 0>, grid, "x2");
        run(row_copy<1, 1>, grid, "x4");
        run(row_copy<2, 2>, grid, "x8");
        run(row_copy<0, 1>, grid, "wx4");
        run(row_copy<0, 2>, grid, "wx8");
        run(quad_copy, grid, "quad");
        run(read_only<false>, grid, "rd_x2");
        run(read_only<true>, grid, "rd_quad");
        run(write_only<false>, grid, "wr_x2");
        run(write_only<true>, grid, "wr_quad");
        run(pair_copy, grid / 2, "pair");
        run(col_copy<2>, B * N / 2, "col2");
        run(col_copy<4>, B * N / 4, "col4");
        (void)hipFree(a);
        (void)hipFree(b);
    }
    return 0;
}
