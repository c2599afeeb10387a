// SpMV schedule micro-benchmark on one MI355X: times CSR kernel variants on
// the BAND-10M matrix (n = 1e6, offsets -5..+4, fp32 values, fp32 x/y, fp64
// row sums) in one process, next to a float4 copy kernel (achievable HBM
// rate). Each variant is checked against the first one.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../include -I../icl-mixed-precision-gmres_amd/csrc \
//         tools/spmv_bench.hip -o spmv_bench
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "csr_tile.hpp"

using namespace mpg;

#define CK(x)                                                                     \
    do {                                                                          \
        hipError_t e_ = (x);                                                      \
        if (e_ != hipSuccess) {                                                   \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            std::exit(1);                                                         \
        }                                                                         \
    } while (0)

__global__ void k_copy4(const float4* __restrict__ a, float4* __restrict__ b, size_t n4) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x)
        b[i] = a[i];
}

// V1: one CSR-adaptive row block per workgroup (the shipped schedule)
__global__ __launch_bounds__(kBlock) void k_tile(const int* blocks, const int* rowptr, const int* col,
                                                 const float* val, int64_t nnz, const float* x, float* y) {
    __shared__ double prod[kNnzCap];
    __shared__ double scratch[kBlock / kWave];
    const int b = blockIdx.x;
    csr_row_block(
        blocks[b], blocks[b + 1], rowptr, col, val, nnz, [&](int c) { return (double)x[c]; },
        [&](int i, double s) { y[i] = (float)s; }, prod, scratch);
}

// V2: L lanes per row, no LDS: strided loads inside the row, shuffle reduction
template <int L>
__global__ __launch_bounds__(256) void k_subwave(int n, const int* __restrict__ rowptr, const int* __restrict__ col,
                                                 const float* __restrict__ val, const float* __restrict__ x,
                                                 float* __restrict__ y) {
    const int gl = threadIdx.x % L;
    const int row = (blockIdx.x * 256 + threadIdx.x) / L;
    double acc = 0.0;
    if (row < n) {
        const int s = rowptr[row], e = rowptr[row + 1];
        for (int j = s + gl; j < e; j += L) acc += (double)val[j] * (double)x[col[j]];
    }
#pragma unroll
    for (int off = L / 2; off > 0; off >>= 1) acc += __shfl_down(acc, off, L);
    if (row < n && gl == 0) y[row] = (float)acc;
}

// V3: one thread per row
__global__ __launch_bounds__(256) void k_scalar(int n, const int* __restrict__ rowptr, const int* __restrict__ col,
                                                const float* __restrict__ val, const float* __restrict__ x,
                                                float* __restrict__ y) {
    const int row = blockIdx.x * 256 + threadIdx.x;
    if (row >= n) return;
    double acc = 0.0;
    for (int j = rowptr[row]; j < rowptr[row + 1]; ++j) acc += (double)val[j] * (double)x[col[j]];
    y[row] = (float)acc;
}

// V4: tile schedule, several row blocks per workgroup, loads of block b+1
// issued before block b is reduced (software pipelining through registers)
__global__ __launch_bounds__(kBlock) void k_tile_pipe(const int* blocks, int nblocks, const int* rowptr,
                                                      const int* col, const float* val, int64_t nnz, const float* x,
                                                      float* y) {
    __shared__ double prod[kNnzCap];
    __shared__ double scratch[kBlock / kWave];
    const int rb0 = (int)((int64_t)blockIdx.x * nblocks / gridDim.x);
    const int rb1 = (int)((int64_t)(blockIdx.x + 1) * nblocks / gridDim.x);
    for (int b = rb0; b < rb1; ++b) {
        if (b + 1 < rb1) {  // touch the next block's index/value lines early
            const int s2 = rowptr[blocks[b + 1]];
            const int idx = (s2 & ~3) + 4 * threadIdx.x;
            if (idx < nnz) __builtin_prefetch(col + idx), __builtin_prefetch(val + idx);
        }
        csr_row_block(
            blocks[b], blocks[b + 1], rowptr, col, val, nnz, [&](int c) { return (double)x[c]; },
            [&](int i, double s) { y[i] = (float)s; }, prod, scratch);
    }
}

int main(int argc, char** argv) {
    const int n = argc > 1 ? std::atoi(argv[1]) : 1000000;
    const int reps = 20;
    // BAND matrix, offsets -5..+4
    std::vector<int> rp(n + 1), ci;
    std::vector<float> va;
    ci.reserve((size_t)n * 10);
    va.reserve((size_t)n * 10);
    uint32_t st = 12345;
    for (int i = 0; i < n; ++i) {
        rp[i] = (int)ci.size();
        for (int d = -5; d <= 4; ++d) {
            int c = i + d;
            if (c < 0 || c >= n) continue;
            st = st * 1664525u + 1013904223u;
            ci.push_back(c);
            va.push_back(d == 0 ? 6.0f : -(float)(st >> 8) / 16777216.0f);
        }
    }
    rp[n] = (int)ci.size();
    const int64_t nnz = (int64_t)ci.size();
    // row blocks as mpg_csr_create builds them
    std::vector<int> blocks;
    for (int r = 0; r < n;) {
        blocks.push_back(r);
        int q = r + 1;
        const int base = rp[r];
        if (rp[q] - base <= kNnzCap)
            while (q < n && q - r < kRowCap && rp[q + 1] - base <= kNnzCap) ++q;
        r = q;
    }
    blocks.push_back(n);
    const int nb = (int)blocks.size() - 1;
    std::vector<float> xh(n);
    for (int i = 0; i < n; ++i) xh[i] = (float)((i * 7919) % 1000) / 1000.0f;

    int *d_rp, *d_ci, *d_bl;
    float *d_va, *d_x, *d_y, *d_y0;
    CK(hipMalloc(&d_rp, (n + 1) * 4));
    CK(hipMalloc(&d_ci, nnz * 4 + 256));
    CK(hipMalloc(&d_bl, (nb + 1) * 4));
    CK(hipMalloc(&d_va, nnz * 4 + 256));
    CK(hipMalloc(&d_x, n * 4 + 256));
    CK(hipMalloc(&d_y, n * 4 + 256));
    CK(hipMalloc(&d_y0, n * 4 + 256));
    CK(hipMemcpy(d_rp, rp.data(), (n + 1) * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_ci, ci.data(), nnz * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_bl, blocks.data(), (nb + 1) * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_va, va.data(), nnz * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_x, xh.data(), n * 4, hipMemcpyHostToDevice));
    const double bytes = nnz * 8.0 + (n + 1) * 4.0 + 2.0 * n * 4;

    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto timeit = [&](const char* name, auto launch, bool check) {
        for (int w = 0; w < 3; ++w) launch();
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0));
        for (int r = 0; r < reps; ++r) launch();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        const double us = 1e3 * ms / reps;
        double maxerr = 0;
        if (check) {
            std::vector<float> a(n), b(n);
            CK(hipMemcpy(a.data(), d_y, n * 4, hipMemcpyDeviceToHost));
            CK(hipMemcpy(b.data(), d_y0, n * 4, hipMemcpyDeviceToHost));
            for (int i = 0; i < n; ++i) maxerr = std::fmax(maxerr, std::fabs((double)a[i] - b[i]));
        }
        std::printf("%-28s %9.2f us  %7.0f GB/s  maxdiff %.2e\n", name, us, bytes / (us * 1e-6) / 1e9, maxerr);
    };

    {  // achievable streaming rate: 512 MB float4 copy
        const size_t n4 = (size_t)64 << 20 >> 1;  // 32M float4 = 512 MB
        float4 *a, *b;
        CK(hipMalloc(&a, n4 * 16));
        CK(hipMalloc(&b, n4 * 16));
        CK(hipMemset(a, 0, n4 * 16));
        for (int w = 0; w < 3; ++w) k_copy4<<<8192, 256>>>(a, b, n4);
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0));
        for (int r = 0; r < 10; ++r) k_copy4<<<8192, 256>>>(a, b, n4);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        std::printf("%-28s %9.2f us  %7.0f GB/s\n", "copy float4 512MB", 1e3 * ms / 10, 2.0 * n4 * 16 * 10 / (ms * 1e-3) / 1e9);
        CK(hipFree(a));
        CK(hipFree(b));
    }
    std::printf("n=%d nnz=%ld row blocks=%d algorithmic bytes=%.1f MB\n", n, (long)nnz, nb, bytes / 1e6);
    timeit("tile (1 block/WG)", [&] { k_tile<<<nb, kBlock>>>(d_bl, d_rp, d_ci, d_va, nnz, d_x, d_y0); }, false);
    timeit("tile (1 block/WG) again", [&] { k_tile<<<nb, kBlock>>>(d_bl, d_rp, d_ci, d_va, nnz, d_x, d_y); }, true);
    for (int G : {512, 1024, 2048}) {
        char nm[64];
        std::snprintf(nm, sizeof nm, "tile pipelined G=%d", G);
        timeit(nm, [&] { k_tile_pipe<<<G, kBlock>>>(d_bl, nb, d_rp, d_ci, d_va, nnz, d_x, d_y); }, true);
    }
    timeit("subwave L=4", [&] { k_subwave<4><<<(n * 4 + 255) / 256, 256>>>(n, d_rp, d_ci, d_va, d_x, d_y); }, true);
    timeit("subwave L=8", [&] { k_subwave<8><<<(n * 8 + 255) / 256, 256>>>(n, d_rp, d_ci, d_va, d_x, d_y); }, true);
    timeit("subwave L=16", [&] { k_subwave<16><<<(n * 16 + 255) / 256, 256>>>(n, d_rp, d_ci, d_va, d_x, d_y); }, true);
    timeit("scalar row/thread", [&] { k_scalar<<<(n + 255) / 256, 256>>>(n, d_rp, d_ci, d_va, d_x, d_y); }, true);
    return 0;
}
