// HBM bandwidth probe (mpg_bw_probe, include/mpgmres/capi.h): the measured
// streaming rate of this GPU, which bench.py reports beside the 8 TB/s spec
// as the achievable peak. Buffers are 1 GiB or more, four times the 256 MB
// Infinity Cache, so every byte comes from HBM; each launch is timed by its
// own hipExtLaunchKernel events (kernel start to end) and the best launch of
// a small grid/unroll sweep is the result.
#include <algorithm>

#include "internal.hpp"

namespace mpg {
namespace {

// read-only: fp64 sum of a float4 stream, one partial per workgroup (kept so
// the loads are not dead)
template <int U>
__global__ __launch_bounds__(kBlock) void k_probe_read(const float4* __restrict__ a, int64_t n4,
                                                       double* __restrict__ part) {
    double acc = 0.0;
    const int64_t stride = (int64_t)gridDim.x * kBlock * U;
    for (int64_t i = (int64_t)blockIdx.x * kBlock * U + threadIdx.x; i < n4; i += stride) {
        float4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t j = i + (int64_t)u * kBlock;
            v[u] = a[j < n4 ? j : n4 - 1];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) acc += (double)v[u].x + (double)v[u].y + (double)v[u].z + (double)v[u].w;
    }
    __shared__ double scratch[kBlock / kWave];
    const double s = block_sum<kBlock>(acc, scratch);
    if (threadIdx.x == 0) part[blockIdx.x] = s;
}

// copy: dst = src, float4 per lane
template <int U>
__global__ __launch_bounds__(kBlock) void k_probe_copy(const float4* __restrict__ a, float4* __restrict__ b,
                                                       int64_t n4) {
    const int64_t stride = (int64_t)gridDim.x * kBlock * U;
    for (int64_t i = (int64_t)blockIdx.x * kBlock * U + threadIdx.x; i < n4; i += stride) {
        float4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t j = i + (int64_t)u * kBlock;
            v[u] = a[j < n4 ? j : n4 - 1];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t j = i + (int64_t)u * kBlock;
            if (j < n4) b[j] = v[u];
        }
    }
}

}  // namespace
}  // namespace mpg

using namespace mpg;

extern "C" int mpg_bw_probe(mpg_ctx_t ctx, int kind, size_t bytes, int reps, double* gbs_out) {
    if (!ctx || !gbs_out || (kind != 0 && kind != 1) || bytes < (1u << 20) || reps < 1) return MPG_ERR_ARG;
    *gbs_out = 0;
    const int64_t n4 = (int64_t)(bytes / 16);
    void *a = nullptr, *b = nullptr, *part = nullptr;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    const int grids[] = {1024, 2048, 4096, 8192};
    int st = MPG_OK;
    double best = 0;
    auto run = [&]() -> int {
        MPG_HIP(ctx, hipMalloc(&a, (size_t)n4 * 16));
        MPG_HIP(ctx, hipMemsetAsync(a, 0, (size_t)n4 * 16, ctx->stream));
        if (kind == 1) {
            MPG_HIP(ctx, hipMalloc(&b, (size_t)n4 * 16));
            MPG_HIP(ctx, hipMemsetAsync(b, 0, (size_t)n4 * 16, ctx->stream));
        }
        MPG_HIP(ctx, hipMalloc(&part, 8192 * sizeof(double)));
        MPG_HIP(ctx, hipEventCreate(&e0));
        MPG_HIP(ctx, hipEventCreate(&e1));
        for (int g : grids) {
            for (int u = 0; u < 2; ++u) {
                for (int r = 0; r < reps; ++r) {
                    const auto* src = static_cast<const float4*>(a);
                    if (kind == 0) {
                        if (u == 0)
                            hipExtLaunchKernelGGL(k_probe_read<2>, dim3(g), dim3(kBlock), 0, ctx->stream, e0, e1, 0,
                                                  src, n4, static_cast<double*>(part));
                        else
                            hipExtLaunchKernelGGL(k_probe_read<4>, dim3(g), dim3(kBlock), 0, ctx->stream, e0, e1, 0,
                                                  src, n4, static_cast<double*>(part));
                    } else {
                        auto* dst = static_cast<float4*>(b);
                        if (u == 0)
                            hipExtLaunchKernelGGL(k_probe_copy<2>, dim3(g), dim3(kBlock), 0, ctx->stream, e0, e1, 0,
                                                  src, dst, n4);
                        else
                            hipExtLaunchKernelGGL(k_probe_copy<4>, dim3(g), dim3(kBlock), 0, ctx->stream, e0, e1, 0,
                                                  src, dst, n4);
                    }
                    MPG_LAUNCH_CHECK(ctx);
                    MPG_HIP(ctx, hipEventSynchronize(e1));
                    float ms = 0;
                    MPG_HIP(ctx, hipEventElapsedTime(&ms, e0, e1));
                    const double moved = (double)n4 * 16 * (kind == 1 ? 2 : 1);
                    if (ms > 0) best = std::max(best, moved / (ms * 1e-3) / 1e9);
                }
            }
        }
        return MPG_OK;
    };
    st = run();
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
    (void)hipStreamSynchronize(ctx->stream);
    if (a) (void)hipFree(a);
    if (b) (void)hipFree(b);
    if (part) (void)hipFree(part);
    *gbs_out = best;
    return st;
}
