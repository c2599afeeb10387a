// Internal helpers shared by the gfx950 kernels of libmpgmres_hip.so.
// Not part of the C-ABI (see include/mpgmres/capi.h).
#pragma once

#include <hip/hip_ext.h>
#include <hip/hip_fp16.h>
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdlib>
#include <string>

#include "mpgmres/capi.h"

struct mpg_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    // Reduction workspace: per-workgroup fp64 partials of the two-stage
    // deterministic reductions (dot, nrm2, gemv^T, Jacobi alpha).
    double* red_ws = nullptr;
    size_t red_ws_elems = 0;
    std::string last_error;
    // measurement hook (mpg_arnoldi_time_next_spmv): the next launch made
    // through launch_timed records its own start/stop on these events
    hipEvent_t time_start = nullptr, time_stop = nullptr;
    // measurement hook (mpg_arnoldi_stamp_next): the next stamped launch
    // (Arnoldi SpMV, k_dots_nc, k_cgs_update_nc) stores each wave's start /
    // end wall clock into these slots
    unsigned long long* stamp_next = nullptr;
    int64_t stamp_cap = 0;  // waves the slots hold
    // pinned host staging of the small device-to-host reads (host-value
    // reductions, scalar reads of the reference driver), kHostWsBytes
    void* host_ws = nullptr;
    void* host_ws_dev = nullptr;  // its device address (stage 2 of host-value reductions stores there)
    unsigned* ticket = nullptr;   // zeroed device word: last-workgroup ticket of one-launch reductions
    unsigned host_seq = 0;        // the last sequence number a host read's kernel was given (host_flag)
};

// Analysed CSR structure (row blocks of the CSR-adaptive schedule).
struct mpg_csr {
    mpg_ctx* ctx = nullptr;
    int32_t rows = 0, cols = 0;
    int64_t nnz = 0;
    const int32_t* rowptr = nullptr;  // device, borrowed
    const int32_t* col = nullptr;     // device, borrowed
    int32_t* blocks = nullptr;        // device, owned: nblocks+1 row starts, then nblocks+1 nnz starts
    int32_t* bnnz = nullptr;          // = blocks + nblocks + 1: rowptr[blocks[b]] (one load, not two dependent)
    int nblocks = 0;
};

namespace mpg {

constexpr int kWave = 64;            // CDNA wavefront width (never 32)
constexpr int kBlock = 256;          // default workgroup: 4 waves
constexpr int kMaxRedBlocks = 1024;  // stage-1 grid cap for reductions
constexpr int kGemvMaxCols = 32;     // columns per panel pass of gemv^T
// context workspace (red_ws, doubles): [0, kMaxRedBlocks * kGemvMaxCols)
// stage-1 partials of the one-call reductions and of nrm2 / dot; 64 scalars
// after them; then the split gemv^T partials (mpg_gemv_t_partials_*), kept
// apart so their consumer can write ||y||^2 partials while it reads them
constexpr size_t kWsGemvSplit = (size_t)kMaxRedBlocks * kGemvMaxCols + 64;
constexpr size_t kWsElems = kWsGemvSplit + (size_t)kMaxRedBlocks * kGemvMaxCols;
// the quad form of the nrm2 stage 1 and of the gemv that can emit its
// partials (4 rows per lane, 1024-lane workgroups, this many at most)
constexpr int kQuadBlock = 1024;
constexpr int kQuadGroups = 256;
inline int quad_groups(int64_t rows) {
    const int64_t g = (rows + 4 * kQuadBlock - 1) / (4 * kQuadBlock);
    return (int)(g < 1 ? 1 : g > kQuadGroups ? kQuadGroups : g);
}

constexpr size_t kHostWsBytes = 4096;

// Wait for the context's stream on a host read of the solver's critical
// path (the reference driver's host-value nrm2 / dot and scalar reads,
// gmres.cpp:160-180 and the per-cycle Scalar::access): poll instead of a
// blocking synchronise, which measured 30-50 us between the stream draining
// and the host's next launch per read (rocprofv3 trace of the operator
// surface, profiles/r06f/); bounded, then the blocking wait.
// The word after the staging block (hipHostMalloc'd kHostWsBytes + 64):
// a host read's kernel stores its sequence number there after its payload
// (host_flag_dev), and the host polls that word instead of the stream
// (host_poll), so the read does not wait for the kernel's end-of-pipe
// release and the runtime's completion signal. MPG_HOST_POLL=0: stream polls.
inline volatile unsigned* host_flag(mpg_ctx* ctx) {
    return reinterpret_cast<volatile unsigned*>(static_cast<char*>(ctx->host_ws) + kHostWsBytes);
}
inline unsigned* host_flag_dev(mpg_ctx* ctx) {
    return reinterpret_cast<unsigned*>(static_cast<char*>(ctx->host_ws_dev) + kHostWsBytes);
}
inline bool host_poll_on() {
    const char* e = std::getenv("MPG_HOST_POLL");
    return !(e && *e == '0');
}
// next sequence number (never 0: the word starts at 0)
inline unsigned host_seq_next(mpg_ctx* ctx) {
    if (++ctx->host_seq == 0) ++ctx->host_seq;
    return ctx->host_seq;
}
// Wait until the flag holds seq. Every 256 polls the stream is queried too:
// a failed launch returns its error, and a stream that completed without
// the flag set is an error (the payload cannot be trusted).
inline hipError_t host_poll(mpg_ctx* ctx, unsigned seq) {
    volatile unsigned* f = host_flag(ctx);
    for (unsigned i = 1;; ++i) {
        if (*f == seq) {
            __atomic_thread_fence(__ATOMIC_ACQUIRE);
            return hipSuccess;
        }
        if ((i & 255) == 0) {
            const hipError_t e = hipStreamQuery(ctx->stream);
            if (e == hipSuccess) {
                if (*f == seq) {
                    __atomic_thread_fence(__ATOMIC_ACQUIRE);
                    return hipSuccess;
                }
                return hipErrorUnknown;
            }
            if (e != hipErrorNotReady) return e;
        }
    }
}

inline hipError_t spin_wait(hipStream_t s) {
    for (int i = 0; i < (1 << 22); ++i) {
        const hipError_t e = hipStreamQuery(s);
        if (e != hipErrorNotReady) return e;
    }
    return hipStreamSynchronize(s);
}

inline int set_hip_error(mpg_ctx* ctx, hipError_t e, const char* what) {
    if (ctx) {
        ctx->last_error = std::string(what) + ": " + hipGetErrorString(e);
    }
    return MPG_ERR_HIP;
}

#define MPG_HIP(ctx, call)                                              \
    do {                                                                \
        hipError_t mpg_e_ = (call);                                     \
        if (mpg_e_ != hipSuccess) return mpg::set_hip_error(ctx, mpg_e_, #call); \
    } while (0)

#define MPG_LAUNCH_CHECK(ctx)                                           \
    do {                                                                \
        hipError_t mpg_e_ = hipGetLastError();                          \
        if (mpg_e_ != hipSuccess) return mpg::set_hip_error(ctx, mpg_e_, "kernel launch"); \
    } while (0)

// A kernel launch on the context's stream; when a timing pair is armed it
// goes through hipExtLaunchKernelGGL, whose events carry the kernel's own
// start and end (no queue or dispatch time around it), and is disarmed.
template <class K, class... A>
inline void launch_timed(mpg_ctx* c, K kern, dim3 grid, dim3 block, A... args) {
    if (c->time_start) {
        hipExtLaunchKernelGGL(kern, grid, block, 0, c->stream, c->time_start, c->time_stop, 0, args...);
        c->time_start = c->time_stop = nullptr;
    } else {
        kern<<<grid, block, 0, c->stream>>>(args...);
    }
}

// XCD-aware workgroup order: the hardware places workgroup b on XCD b % 8
// (round robin), so logical block xcd_block(b, G) gives each XCD one
// contiguous range of the grid (its private L2 then caches the neighbourhood
// of its own rows). A bijection of [0, G).
__device__ __forceinline__ int xcd_block(int b, int G) {
    constexpr int X = 8;
    const int q = G / X, r = G % X;
    const int xcd = b % X, idx = b / X;
    return xcd < r ? xcd * (q + 1) + idx : r * (q + 1) + (xcd - r) * q + idx;
}

inline int grid_for(int64_t n, int per_thread, int cap = 2048) {
    int64_t g = (n + (int64_t)kBlock * per_thread - 1) / ((int64_t)kBlock * per_thread);
    if (g < 1) g = 1;
    if (g > cap) g = cap;
    return (int)g;
}

// The wave's index in its workgroup, as a wave-uniform value: the compiler
// does not know threadIdx.x / 64 is the same in every lane, and everything
// derived from it (slice index, offsets, pattern index) would otherwise sit
// in vector registers, one copy per lane.
__device__ __forceinline__ int wave_id() { return __builtin_amdgcn_readfirstlane((int)(threadIdx.x / kWave)); }

// ---- wave / block reductions (wave64 shuffles, then LDS across waves) ----
template <class T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
    for (int off = kWave / 2; off > 0; off >>= 1) v += __shfl_down(v, off, kWave);
    return v;  // valid in lane 0
}

template <class T>
__device__ __forceinline__ T wave_max(T v) {
#pragma unroll
    for (int off = kWave / 2; off > 0; off >>= 1) {
        T o = __shfl_down(v, off, kWave);
        v = v > o ? v : o;
    }
    return v;
}

// Workgroup barrier that waits for this wave's LDS operations only:
// __syncthreads() also waits for every outstanding global load (its
// workgroup-scope release), which would drain loads issued ahead on purpose.
// The signal fences keep the compiler from moving memory accesses across.
__device__ __forceinline__ void lds_barrier() {
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0); vmcnt and expcnt at their maxima (no wait)
    __builtin_amdgcn_s_barrier();
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
}

// Block-wide sum for blockDim.x == BS (multiple of 64). Result valid in
// thread 0. `scratch` must hold BS/64 elements.
template <int BS, class T>
__device__ __forceinline__ T block_sum(T v, T* scratch) {
    const int lane = threadIdx.x & (kWave - 1);
    const int wid = threadIdx.x / kWave;
    v = wave_sum(v);
    if (lane == 0) scratch[wid] = v;
    __syncthreads();
    T r = 0;
    if (threadIdx.x == 0) {
#pragma unroll
        for (int w = 0; w < BS / kWave; ++w) r += scratch[w];
    }
    __syncthreads();
    return r;
}

template <int BS, class T>
__device__ __forceinline__ T block_max(T v, T* scratch) {
    const int lane = threadIdx.x & (kWave - 1);
    const int wid = threadIdx.x / kWave;
    v = wave_max(v);
    if (lane == 0) scratch[wid] = v;
    __syncthreads();
    T r = scratch[0];
    if (threadIdx.x == 0) {
#pragma unroll
        for (int w = 1; w < BS / kWave; ++w) r = r > scratch[w] ? r : scratch[w];
    }
    __syncthreads();
    return r;
}

template <class T> struct acc_type { using type = double; };

// acc + a * b in the accumulation class of a kernel (arnoldi_kernels.hpp):
// fp64 (one fused multiply-add), or fp32 -- the fp64 product (exact for
// fp32 / fp16 operands) rounded to fp32, then an fp32 add: the same two
// roundings in every storage format (SELL, node blocks, CSR tiles), so the
// formats keep giving one another's bits under either class
// (fp32: contraction off -- for fp32 operands the compiler would otherwise
// narrow the exact fp64 product to an fp32 multiply and fuse it with the add
// into an fp32 FMA on the SELL copy, while the tiles add products staged in
// LDS: measured 87 of 90 steps differing between SELL and CSR)
__device__ __forceinline__ void mac(double& acc, double a, double b) { acc += a * b; }
__device__ __forceinline__ void mac(float& acc, double a, double b) {
#pragma clang fp contract(off)
    const float p = (float)(a * b);
    acc = acc + p;
}
// y = alpha * t + beta * y_old, the epilogue of every SpMV storage form
// (CSR tiles, SELL, node blocks) in one rounding order: the two products
// rounded, then their sum. Left to contraction, the compiler fused one
// product or the other depending on the kernel around it (node vs CSR bits
// differed at alpha = -1.5, beta = 0.75 after an unrelated change to the node
// kernel). The solver's own calls (alpha = +-1, beta in {0, 1}) round once
// either way.
template <class X>
__device__ __forceinline__ X spmv_axpby(X alpha, X t, X beta, X yi) {
#pragma clang fp contract(off)
    return beta == X(0) ? alpha * t : alpha * t + beta * yi;
}
// acc + p, p an exact fp64 product (the tiles' LDS products), in the class
__device__ __forceinline__ void add_prod(double& acc, double p) { acc += p; }
__device__ __forceinline__ void add_prod(float& acc, double p) {
#pragma clang fp contract(off)
    acc = acc + (float)p;
}

__device__ __forceinline__ float to_float(uint16_t h) {
    return __half2float(__ushort_as_half(h));
}

}  // namespace mpg
