// FETCH_SIZE calibration for the access widths of the SpMV kernels
// (MI355X_MICROARCH.md §HBM: "FETCH_SIZE reports exactly 1/2 of the bytes of
// a wide coalesced streaming read (16 B/lane) ... other access widths are
// uncalibrated"). Each kernel reads a 512 MiB buffer (past the 256 MiB
// Infinity Cache, rotated over two halves so nothing is resident) exactly
// once with one access shape; rocprofv3 --pmc FETCH_SIZE per kernel divided
// by the bytes printed here gives the shape's tally factor:
//   k_lane<16|8|4|2>  coalesced, 16 / 8 / 4 / 2 B per lane (float4, float2,
//                     float, half) -- SELL values (16 B fp32 W = 4, 8 B fp16
//                     W = 4 / fp32 W = 2, 4 B fp16 W = 2), int16 columns
//   k_seg256          each wave reads one 256-B segment (4 B per lane) at a
//                     scattered segment: a stencil slice's x gather of one
//                     element across 64 consecutive rows
// usage: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/pmc_calib.hip -o tools/pmc_calib
//        rocprofv3 --pmc FETCH_SIZE --output-format csv -d out -o calib -- ./tools/pmc_calib
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            std::exit(1);                                                                  \
        }                                                                                  \
    } while (0)

template <int B> struct Vec;
template <> struct Vec<16> { using T = float4; static __device__ float sum(T v) { return v.x + v.y + v.z + v.w; } };
template <> struct Vec<8> { using T = float2; static __device__ float sum(T v) { return v.x + v.y; } };
template <> struct Vec<4> { using T = float; static __device__ float sum(T v) { return v; } };
template <> struct Vec<2> { using T = unsigned short; static __device__ float sum(T v) { return (float)v; } };

template <int B>
__global__ __launch_bounds__(256) void k_lane(const typename Vec<B>::T* __restrict__ a, size_t n, float* __restrict__ out) {
    float acc = 0.f;
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) acc += Vec<B>::sum(a[i]);
    if (acc == 12345.f) out[0] = acc;  // keeps the loads
}

// one 256-B segment per wave per iteration, segments visited in a scattered
// (multiplicative) order: every segment exactly once
__global__ __launch_bounds__(256) void k_seg256(const float* __restrict__ a, size_t nseg, float* __restrict__ out) {
    float acc = 0.f;
    const int lane = threadIdx.x & 63;
    const size_t wave = blockIdx.x * 4ull + threadIdx.x / 64, waves = (size_t)gridDim.x * 4;
    for (size_t s = wave; s < nseg; s += waves) {
        const size_t seg = (s * 2654435761ull) % nseg;  // nseg a power of two, odd multiplier: a permutation
        acc += a[seg * 64 + lane];
    }
    if (acc == 12345.f) out[0] = acc;
}

int main() {
    const size_t bytes = 512ull << 20;
    char* buf = nullptr;
    float* out = nullptr;
    CK(hipMalloc(&buf, 2 * bytes));
    CK(hipMalloc(&out, 64));
    CK(hipMemset(buf, 0, 2 * bytes));
    const int grid = 256 * 8;
    int half = 0;
    auto next = [&]() { half ^= 1; return buf + (size_t)half * bytes; };
    for (int rep = 0; rep < 2; ++rep) {
        k_lane<16><<<grid, 256>>>((const float4*)next(), bytes / 16, out);
        k_lane<8><<<grid, 256>>>((const float2*)next(), bytes / 8, out);
        k_lane<4><<<grid, 256>>>((const float*)next(), bytes / 4, out);
        k_lane<2><<<grid, 256>>>((const unsigned short*)next(), bytes / 2, out);
        k_seg256<<<grid, 256>>>((const float*)next(), bytes / 256, out);
    }
    CK(hipDeviceSynchronize());
    std::printf("{\"bytes_per_launch\": %zu, \"kernels\": [\"k_lane<16>\", \"k_lane<8>\", \"k_lane<4>\", \"k_lane<2>\", "
                "\"k_seg256\"], \"launches_each\": 2}\n", bytes);
    CK(hipFree(buf));
    CK(hipFree(out));
    return 0;
}
