// SELL-64 SpMV schedule micro-benchmark on one MI355X (BAND-10M: n = 1e6,
// offsets -5..+4, fp32 values, int16 slice-relative columns, W = 2, fp32
// x/y, fp64 row sums). Four copies of the matrix rotate so most reads come
// from HBM. Variants:
//   one    one slice per wave, grid = nslices / 4 (the shipped k_step_sell)
//   two    two slices per wave, loads of both issued before either's gathers
//   pers   persistent grid (8 workgroups per CU), waves loop over slices
//   pipe   persistent + the next slice's (col, val) loaded before this
//          slice's gathers (software pipeline)
// Every variant is checked against `one`.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../icl-mixed-precision-gmres_amd/csrc tools/sell_bench.hip -o tools/sell_bench
#include <hip/hip_runtime.h>

#include <cmath>
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

constexpr int kW = 2, kSteps = 5;  // 10 entries per row in 5 steps of 2
constexpr int kCopies = 4;
typedef short short2v __attribute__((ext_vector_type(2)));
typedef float float2v __attribute__((ext_vector_type(2)));

struct Slice {
    short2v c[kSteps];
    float2v v[kSteps];
};

__device__ __forceinline__ void load_slice(const short* col, const float* val, int s, int lane, Slice& d) {
    const size_t o = (size_t)s * 64 * kW * kSteps + lane * kW;
#pragma unroll
    for (int q = 0; q < kSteps; ++q) {
        d.c[q] = *reinterpret_cast<const short2v*>(col + o + (size_t)q * 64 * kW);
        d.v[q] = *reinterpret_cast<const float2v*>(val + o + (size_t)q * 64 * kW);
    }
}

__device__ __forceinline__ double row_sum(const Slice& d, int s, const float* x) {
    double xv[kSteps][kW];
    const int row0 = s * 64;
#pragma unroll
    for (int q = 0; q < kSteps; ++q)
#pragma unroll
        for (int e = 0; e < kW; ++e) xv[q][e] = d.c[q][e] != -32768 ? (double)x[row0 + d.c[q][e]] : 0.0;
    double acc = 0;
#pragma unroll
    for (int q = 0; q < kSteps; ++q)
#pragma unroll
        for (int e = 0; e < kW; ++e)
            if (d.c[q][e] != -32768) acc += (double)d.v[q][e] * xv[q][e];
    return acc;
}

__global__ __launch_bounds__(256) void k_one(int n, int ns, const short* col, const float* val, const float* x,
                                             float* y) {
    const int lane = threadIdx.x & 63, s = blockIdx.x * 4 + threadIdx.x / 64;
    if (s >= ns) return;
    Slice d;
    load_slice(col, val, s, lane, d);
    const double acc = row_sum(d, s, x);
    const int i = s * 64 + lane;
    if (i < n) y[i] = (float)acc;
}

__global__ __launch_bounds__(256) void k_two(int n, int ns, const short* col, const float* val, const float* x,
                                             float* y) {
    const int lane = threadIdx.x & 63, s0 = (blockIdx.x * 4 + threadIdx.x / 64) * 2;
    if (s0 >= ns) return;
    const bool has1 = s0 + 1 < ns;
    Slice a, b;
    load_slice(col, val, s0, lane, a);
    if (has1) load_slice(col, val, s0 + 1, lane, b);
    const double r0 = row_sum(a, s0, x);
    const double r1 = has1 ? row_sum(b, s0 + 1, x) : 0.0;
    int i = s0 * 64 + lane;
    if (i < n) y[i] = (float)r0;
    i += 64;
    if (has1 && i < n) y[i] = (float)r1;
}

__global__ __launch_bounds__(256) void k_pers(int n, int ns, const short* col, const float* val, const float* x,
                                              float* y) {
    const int lane = threadIdx.x & 63;
    const int nw = gridDim.x * 4;
    for (int s = blockIdx.x * 4 + threadIdx.x / 64; s < ns; s += nw) {
        Slice d;
        load_slice(col, val, s, lane, d);
        const double acc = row_sum(d, s, x);
        const int i = s * 64 + lane;
        if (i < n) y[i] = (float)acc;
    }
}

__global__ __launch_bounds__(256) void k_pipe(int n, int ns, const short* col, const float* val, const float* x,
                                              float* y) {
    const int lane = threadIdx.x & 63;
    const int nw = gridDim.x * 4;
    int s = blockIdx.x * 4 + threadIdx.x / 64;
    if (s >= ns) return;
    Slice cur, nxt;
    load_slice(col, val, s, lane, cur);
    for (;;) {
        const int sn = s + nw;
        if (sn < ns) load_slice(col, val, sn, lane, nxt);
        const double acc = row_sum(cur, s, x);
        const int i = s * 64 + lane;
        if (i < n) y[i] = (float)acc;
        if (sn >= ns) break;
        cur = nxt;
        s = sn;
    }
}

// upper bound without gathers: every entry reads x[row] (coalesced)
__global__ __launch_bounds__(256) void k_nog(int n, int ns, const short* col, const float* val, const float* x,
                                             float* y) {
    const int lane = threadIdx.x & 63, s = blockIdx.x * 4 + threadIdx.x / 64;
    if (s >= ns) return;
    Slice d;
    load_slice(col, val, s, lane, d);
    const int i = s * 64 + lane;
    const double xi = i < n ? (double)x[i] : 0.0;
    double acc = 0;
#pragma unroll
    for (int q = 0; q < kSteps; ++q)
#pragma unroll
        for (int e = 0; e < kW; ++e)
            if (d.c[q][e] != -32768) acc += (double)d.v[q][e] * xi;
    if (i < n) y[i] = (float)acc;
}

// x window of the slice staged in LDS (columns within [row0 - 64, row0 + 128))
__global__ __launch_bounds__(256) void k_lds(int n, int ns, const short* col, const float* val, const float* x,
                                             float* y) {
    __shared__ float win[4][192];
    const int lane = threadIdx.x & 63, wid = threadIdx.x / 64, s = blockIdx.x * 4 + wid;
    if (s >= ns) return;
    Slice d;
    load_slice(col, val, s, lane, d);
    const int row0 = s * 64;
#pragma unroll
    for (int q = 0; q < 3; ++q) {
        const int c = row0 - 64 + q * 64 + lane;
        win[wid][q * 64 + lane] = (c >= 0 && c < n) ? x[c] : 0.0f;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    double acc = 0;
#pragma unroll
    for (int q = 0; q < kSteps; ++q)
#pragma unroll
        for (int e = 0; e < kW; ++e)
            if (d.c[q][e] != -32768) acc += (double)d.v[q][e] * (double)win[wid][64 + d.c[q][e]];
    const int i = row0 + lane;
    if (i < n) y[i] = (float)acc;
}

template <class F>
static float time_it(int reps, F&& f) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int r = 0; r < 4; ++r) f(r);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a));
    for (int r = 0; r < reps; ++r) f(r);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms / reps;
}

int main() {
    const int n = 1000000, ns = (n + 63) / 64;
    const size_t per = (size_t)64 * kW * kSteps, tot = per * ns;
    std::vector<short> hc(tot);
    std::vector<float> hv(tot);
    uint32_t st = 12345;
    for (int s = 0; s < ns; ++s)
        for (int lane = 0; lane < 64; ++lane) {
            const int i = s * 64 + lane;
            int j = 0;
            for (int d = -5; d <= 4; ++d, ++j) {
                const int c = i + d;
                const size_t pos = (size_t)s * per + (size_t)(j / kW) * 64 * kW + lane * kW + j % kW;
                st = st * 1664525u + 1013904223u;
                const bool live = i < n && c >= 0 && c < n;
                hc[pos] = live ? (short)(c - s * 64) : (short)-32768;
                hv[pos] = live ? (d == 0 ? 6.0f : -(float)(st >> 8) / 16777216.0f) : 0.0f;
            }
        }
    std::vector<short*> dc(kCopies);
    std::vector<float*> dv(kCopies), dx(kCopies);
    std::vector<float> hx(n);
    for (int i = 0; i < n; ++i) hx[i] = (float)((i * 7919) % 1000) / 1000.0f;
    for (int c = 0; c < kCopies; ++c) {
        CK(hipMalloc(&dc[c], tot * 2));
        CK(hipMalloc(&dv[c], tot * 4));
        CK(hipMalloc(&dx[c], (size_t)n * 4));
        CK(hipMemcpy(dc[c], hc.data(), tot * 2, hipMemcpyHostToDevice));
        CK(hipMemcpy(dv[c], hv.data(), tot * 4, hipMemcpyHostToDevice));
        CK(hipMemcpy(dx[c], hx.data(), (size_t)n * 4, hipMemcpyHostToDevice));
    }
    float *y, *y0;
    CK(hipMalloc(&y, (size_t)n * 4));
    CK(hipMalloc(&y0, (size_t)n * 4));
    const double bytes = (double)tot * 6 + 2.0 * n * 4;
    const int reps = 40;
    auto report = [&](const char* name, float ms) {
        std::vector<float> a(n), b(n);
        CK(hipMemcpy(a.data(), y, (size_t)n * 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(b.data(), y0, (size_t)n * 4, hipMemcpyDeviceToHost));
        double err = 0;
        for (int i = 0; i < n; ++i) err = std::fmax(err, std::fabs(a[i] - b[i]));
        std::printf("%-6s %7.2f us  %6.0f GB/s (actual bytes %.1f MB)  max|diff| %.2e\n", name, ms * 1e3,
                    bytes / (ms * 1e-3) / 1e9, bytes / 1e6, err);
    };
    float ms = time_it(reps, [&](int r) { k_one<<<(ns + 3) / 4, 256>>>(n, ns, dc[r % kCopies], dv[r % kCopies], dx[r % kCopies], y0); });
    CK(hipMemcpy(y, y0, (size_t)n * 4, hipMemcpyDeviceToDevice));
    report("one", ms);
    ms = time_it(reps, [&](int r) { k_two<<<(ns / 2 + 4) / 4, 256>>>(n, ns, dc[r % kCopies], dv[r % kCopies], dx[r % kCopies], y); });
    report("two", ms);
    for (int g : {1024, 2048, 4096}) {
        ms = time_it(reps, [&](int r) { k_pers<<<g, 256>>>(n, ns, dc[r % kCopies], dv[r % kCopies], dx[r % kCopies], y); });
        std::printf("[grid %d] ", g);
        report("pers", ms);
        ms = time_it(reps, [&](int r) { k_pipe<<<g, 256>>>(n, ns, dc[r % kCopies], dv[r % kCopies], dx[r % kCopies], y); });
        std::printf("[grid %d] ", g);
        report("pipe", ms);
    }
    ms = time_it(reps, [&](int) { k_one<<<(ns + 3) / 4, 256>>>(n, ns, dc[0], dv[0], dx[0], y); });
    report("one/1c", ms);
    ms = time_it(reps, [&](int r) { k_lds<<<(ns + 3) / 4, 256>>>(n, ns, dc[r % kCopies], dv[r % kCopies], dx[r % kCopies], y); });
    report("lds", ms);
    ms = time_it(reps, [&](int r) { k_nog<<<(ns + 3) / 4, 256>>>(n, ns, dc[r % kCopies], dv[r % kCopies], dx[r % kCopies], y); });
    report("nogath", ms);  // (wrong values on purpose: the no-gather bound)  // one copy: MALL-resident after the first pass
    return 0;
}
