// HBM bandwidth of strided-segment copies on gfx950: every wave instruction
// moves 64 lanes x 8 B; SEG contiguous bytes per segment, segments spread
// over a large buffer (the access shape of column tiles of width SEG / 8).
// Build: hipcc --offload-arch=gfx950 -O3 tools/bw_probe.hip -o build/bw_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

template <int SEG>
__global__ void __launch_bounds__(256) seg_copy(const float2* __restrict__ in, float2* __restrict__ out,
                                                long long rows, long long row_elems) {
    // element e of the copy: segment s = e / (SEG/8), within-segment w = e % (SEG/8)
    // segment s covers row (s % rows) at column group (s / rows): column-panel walk.
    constexpr int SE = SEG / 8;
    const long long total = rows * row_elems;
    for (long long e = blockIdx.x * 256LL + threadIdx.x; e < total; e += (long long)gridDim.x * 256) {
        const long long s = e / SE, w = e % SE;
        const long long r = s % rows, g = s / rows;
        const long long idx = r * row_elems + g * SE + w;
        out[idx] = in[idx];
    }
}

int main() {
    const long long rows = 4096, row_elems = 4096 * 8;  // 1 GiB per buffer
    const size_t bytes = rows * row_elems * sizeof(float2);
    float2 *a, *b;
    if (hipMalloc(&a, bytes) != hipSuccess || hipMalloc(&b, bytes) != hipSuccess) return 1;
    (void)hipMemset(a, 1, bytes);
    (void)hipMemset(b, 0, bytes);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    auto run = [&](auto kern, const char* name) {
        for (int grid : {2048, 8192}) {
            hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, a, b, rows, row_elems);
            (void)hipEventRecord(e0);
            for (int i = 0; i < 5; ++i) hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, a, b, rows, row_elems);
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            float ms = 0;
            (void)hipEventElapsedTime(&ms, e0, e1);
            printf("%-10s grid=%5d  %.1f GB/s (read+write)\n", name, grid, 2.0 * bytes * 5 / (ms * 1e-3) / 1e9);
        }
    };
    run(seg_copy<16>, "seg16B");
    run(seg_copy<32>, "seg32B");
    run(seg_copy<64>, "seg64B");
    run(seg_copy<128>, "seg128B");
    run(seg_copy<256>, "seg256B");
    run(seg_copy<1024 * 8>, "contig");
    return 0;
}
