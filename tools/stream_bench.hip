// Streaming-read micro-benchmark on one MI355X for the Gram-Schmidt panel
// kernels: what rate a read-only reduction reaches on fp32 columns of 1e6
// rows, by grid size and rows per lane, with the working set rotated over
// 8 copies (512 MB > the 256 MB Infinity Cache) so reads come from HBM.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/stream_bench.hip -o tools/stream_bench
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            std::exit(1);                                                                  \
        }                                                                                  \
    } while (0)

constexpr int kCopies = 8;

// sum of a float4 stream; one fp64 partial per workgroup
template <int BS, int U>
__global__ __launch_bounds__(BS) void k_read(const float4* __restrict__ a, size_t n4, double* __restrict__ part) {
    double acc = 0.0;
    size_t i = blockIdx.x * (size_t)BS * U + threadIdx.x;
    const size_t stride = (size_t)gridDim.x * BS * U;
    for (; i < n4; i += stride) {
        float4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = i + u * BS < n4 ? a[i + u * BS] : make_float4(0, 0, 0, 0);
#pragma unroll
        for (int u = 0; u < U; ++u) acc += (double)v[u].x + (double)v[u].y + (double)v[u].z + (double)v[u].w;
    }
    for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off, 64);
    __shared__ double r[BS / 64];
    if ((threadIdx.x & 63) == 0) r[threadIdx.x / 64] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
        double s = 0;
        for (int w = 0; w < BS / 64; ++w) s += r[w];
        part[blockIdx.x] = s;
    }
}

// panel dots: nc fp32 columns (leading dimension ld) against w, 4 rows per
// lane per iteration, one fp64 accumulator per column
template <int NC>
__global__ __launch_bounds__(256) void k_dots(int n, const float* __restrict__ V, size_t ld, int nc,
                                              const float* __restrict__ w, double* __restrict__ part) {
    double acc[NC];
#pragma unroll
    for (int c = 0; c < NC; ++c) acc[c] = 0.0;
    for (int i = 4 * (blockIdx.x * 256 + threadIdx.x); i < n; i += 4 * gridDim.x * 256) {
        const float4 wv = *reinterpret_cast<const float4*>(w + i);
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            if (c < nc) {
                const float4 v = *reinterpret_cast<const float4*>(V + c * ld + i);
                acc[c] += (double)v.x * wv.x + (double)v.y * wv.y + (double)v.z * wv.z + (double)v.w * wv.w;
            }
        }
    }
    double s = 0;
#pragma unroll
    for (int c = 0; c < NC; ++c) s += acc[c];
    for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
    if ((threadIdx.x & 63) == 0) part[blockIdx.x * 4 + threadIdx.x / 64] = s;
}

// panel dots variant: BS threads, R float4 row groups per lane per iteration
template <int NC, int BS, int R>
__global__ __launch_bounds__(BS) void k_dots2(int n, const float* __restrict__ V, size_t ld, int nc,
                                              const float* __restrict__ w, double* __restrict__ part) {
    double acc[NC];
#pragma unroll
    for (int c = 0; c < NC; ++c) acc[c] = 0.0;
    for (int i = 4 * R * (blockIdx.x * BS) + 4 * threadIdx.x; i < n; i += 4 * R * gridDim.x * BS) {
        float4 wv[R];
#pragma unroll
        for (int r = 0; r < R; ++r) wv[r] = *reinterpret_cast<const float4*>(w + i + 4 * BS * r);
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            if (c < nc) {
                float4 v[R];
#pragma unroll
                for (int r = 0; r < R; ++r) v[r] = *reinterpret_cast<const float4*>(V + c * ld + i + 4 * BS * r);
#pragma unroll
                for (int r = 0; r < R; ++r)
                    acc[c] += (double)v[r].x * wv[r].x + (double)v[r].y * wv[r].y + (double)v[r].z * wv[r].z +
                              (double)v[r].w * wv[r].w;
            }
        }
    }
    double s = 0;
#pragma unroll
    for (int c = 0; c < NC; ++c) s += acc[c];
    for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
    if ((threadIdx.x & 63) == 0) part[blockIdx.x * (BS / 64) + threadIdx.x / 64] = s;
}

// PMC calibration: read `bytes` with W-byte loads per lane (k_calib_4/8/16),
// so FETCH_SIZE per dispatch can be compared with a known byte count
template <class V>
__global__ __launch_bounds__(256) void k_calib(const V* __restrict__ a, size_t n, unsigned* __restrict__ out) {
    unsigned acc = 0;
    for (size_t i = blockIdx.x * (size_t)256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
        const V v = a[i];
#pragma unroll
        for (int q = 0; q < (int)(sizeof(V) / 4); ++q) acc ^= reinterpret_cast<const unsigned*>(&v)[q];
    }
    if (acc == 0x9e3779b9u) out[0] = acc;  // keeps the loads
}

template <class F>
static float time_it(int reps, F&& f) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    f(0);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a));
    for (int r = 0; r < reps; ++r) f(r + 1);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms / reps;
}

int main() {
    const int n = 1000000;
    const size_t ld = 1000448;  // 256-B padded, as the engine's V
    const int cols = 16;
    const size_t bytes = ld * 4 * cols;  // 64 MB
    std::vector<float*> bufs(kCopies);
    std::vector<float*> ws(kCopies);
    for (int c = 0; c < kCopies; ++c) {
        CK(hipMalloc(&bufs[c], bytes));
        CK(hipMemset(bufs[c], 0, bytes));
        CK(hipMalloc(&ws[c], ld * 4));
        CK(hipMemset(ws[c], 0, ld * 4));
    }
    double* part;
    CK(hipMalloc(&part, 1 << 20));
    const int reps = 40;
    const size_t n4 = bytes / 16;
    std::printf("read-only float4 sum of 64 MB, rotating over %d copies\n", kCopies);
    for (int G : {256, 512, 1024, 2048, 4096, 8192}) {
        auto run = [&](auto kern, int BS, const char* tag) {
            float ms = time_it(reps, [&](int r) { kern<<<G, BS>>>((const float4*)bufs[r % kCopies], n4, part); });
            std::printf("  G=%5d %-10s %7.2f us  %7.0f GB/s\n", G, tag, ms * 1e3, bytes / (ms * 1e-3) / 1e9);
        };
        run(k_read<256, 1>, 256, "bs256 u1");
        run(k_read<256, 4>, 256, "bs256 u4");
        run(k_read<512, 2>, 512, "bs512 u2");
        run(k_read<1024, 1>, 1024, "bs1024 u1");
    }
    std::printf("panel dots, 16 fp32 columns x 1e6 rows + w (68 MB)\n");
    for (int G : {256, 512, 1024, 2048}) {
        float ms = time_it(reps, [&](int r) {
            k_dots<32><<<G, 256>>>(n, bufs[r % kCopies], ld, cols, ws[r % kCopies], part);
        });
        std::printf("  G=%5d           %7.2f us  %7.0f GB/s\n", G, ms * 1e3, (bytes + ld * 4) / (ms * 1e-3) / 1e9);
    }
    std::printf("panel dots variants (BS threads, R row groups of 4 per lane)\n");
    auto dv = [&](auto kern, int G, int BS, const char* tag) {
        float ms = time_it(reps, [&](int r) { kern<<<G, BS>>>(n, bufs[r % kCopies], ld, cols, ws[r % kCopies], part); });
        std::printf("  G=%5d %-12s %7.2f us  %7.0f GB/s\n", G, tag, ms * 1e3, (bytes + ld * 4) / (ms * 1e-3) / 1e9);
    };
    dv(k_dots2<32, 1024, 1>, 256, 1024, "bs1024 r1");
    dv(k_dots2<32, 1024, 2>, 128, 1024, "bs1024 r2");
    dv(k_dots2<32, 512, 1>, 512, 512, "bs512 r1");
    dv(k_dots2<32, 512, 2>, 256, 512, "bs512 r2");
    dv(k_dots2<32, 512, 2>, 512, 512, "bs512 r2");
    dv(k_dots2<32, 256, 2>, 512, 256, "bs256 r2");
    dv(k_dots2<32, 256, 2>, 1024, 256, "bs256 r2");
    dv(k_dots2<32, 256, 4>, 512, 256, "bs256 r4");
    std::printf("same, one copy only (MALL-resident after the first pass)\n");
    for (int G : {1024}) {
        float ms = time_it(reps, [&](int) { k_dots<32><<<G, 256>>>(n, bufs[0], ld, cols, ws[0], part); });
        std::printf("  G=%5d           %7.2f us  %7.0f GB/s\n", G, ms * 1e3, (bytes + ld * 4) / (ms * 1e-3) / 1e9);
    }
    // calibration reads: 512 MB (beyond the Infinity Cache) at 4, 8, 16 B per lane
    {
        const size_t cb = (size_t)512 << 20;
        char* big;
        CK(hipMalloc(&big, cb));
        CK(hipMemset(big, 1, cb));
        unsigned* o;
        CK(hipMalloc(&o, 64));
        for (int r = 0; r < 3; ++r) {
            k_calib<unsigned><<<4096, 256>>>((const unsigned*)big, cb / 4, o);
            k_calib<uint2><<<4096, 256>>>((const uint2*)big, cb / 8, o);
            k_calib<uint4><<<4096, 256>>>((const uint4*)big, cb / 16, o);
        }
        CK(hipDeviceSynchronize());
        std::printf("calibration: k_calib<4|8|16 B> each read %zu bytes per dispatch\n", cb);
    }
    return 0;
}
