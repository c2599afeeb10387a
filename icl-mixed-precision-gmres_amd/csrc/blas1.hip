// BLAS-1 surface of the hot path on gfx950 (kernels.hpp:11-101,
// kernels_mkl.cpp:73-260). Elementwise kernels are grid-stride with
// contiguous lanes; reductions are a deterministic two-stage tree that
// accumulates in fp64 for both fp32 and fp64 inputs (stage 1: one fp64
// partial per workgroup into the context workspace, stage 2: one workgroup
// sums the partials in a fixed order and writes the result on device).
#include "internal.hpp"
#include "mpgmres/arnoldi.h"  // mpg_dtype_t
#include "panel.hpp"
#include "scalar_program.hpp"

#include <algorithm>

using namespace mpg;

namespace {

// ---------------- reductions ----------------
template <class T, bool SQUARE>
__global__ __launch_bounds__(kBlock) void k_reduce_stage1(int64_t n, const T* __restrict__ x,
                                                          const T* __restrict__ y,
                                                          double* __restrict__ partial) {
    __shared__ double scratch[kBlock / kWave];
    double acc = 0.0;
    const int64_t stride = (int64_t)gridDim.x * kBlock;
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride) {
        double a = (double)x[i];
        acc += SQUARE ? a * a : a * (double)y[i];
    }
    double s = block_sum<kBlock>(acc, scratch);
    if (threadIdx.x == 0) partial[blockIdx.x] = s;
}

// nrm2 stage 1 on a 16-B aligned vector: 4 rows per lane of 1024-lane
// workgroups (quad_groups), the lane's rows in order, then the tail rows,
// then block_sum<kQuadBlock> -- the layout and order in which the quad gemv
// (k_gemv_n_quad<..., NORM>, blas2.hip) emits the ||y||^2 partials of the y
// it writes, so both give the same partials for the same vector
template <class T>
__device__ __forceinline__ double nrm2_quad_partial(int64_t n, const T* __restrict__ x, double* scratch) {
    double acc = 0.0;
    const int64_t n4 = n & ~int64_t(3);
    const int64_t step = 4 * (int64_t)gridDim.x * kQuadBlock;
    for (int64_t i = 4 * ((int64_t)blockIdx.x * kQuadBlock + threadIdx.x); i < n4; i += step) {
        double v[4];
        Row4<T>::load(x + i, v);
#pragma unroll
        for (int r = 0; r < 4; ++r) acc += v[r] * v[r];
    }
    for (int64_t i = n4 + (int64_t)blockIdx.x * kQuadBlock + threadIdx.x; i < n; i += (int64_t)gridDim.x * kQuadBlock) {
        const double a = (double)x[i];
        acc += a * a;
    }
    return block_sum<kQuadBlock>(acc, scratch);
}

template <class T>
__global__ __launch_bounds__(kQuadBlock) void k_nrm2_quad(int64_t n, const T* __restrict__ x,
                                                          double* __restrict__ partial) {
    __shared__ double scratch[kQuadBlock / kWave];
    const double s = nrm2_quad_partial(n, x, scratch);
    if (threadIdx.x == 0) partial[blockIdx.x] = s;
}

// A host-value nrm2 on a 16-B aligned vector in ONE launch (the operator
// surface's per-cycle r_norm / beta / ||x|| reads, gmres.cpp:173-196): the
// stage 1 of k_nrm2_quad, then the last workgroup to finish (a device-scope
// ticket, zeroed at context creation and reset by that workgroup) sums the
// partials with k_reduce_stage2's block_sum<1024> over the same 1024 lanes --
// the bits of the two launches -- and stores sqrt into the context's pinned
// host word. The hand-off is the guide's write-through form
// (cdna_hip_programming.md, in-launch split-K reduction): each partial is an
// sc1 (agent-scope relaxed atomic) store, waited for, before a relaxed
// agent-scope ticket add; the last arriver reads the partials with sc1 loads.
// No __threadfence: an agent release writes back the XCD's whole L2, in
// every workgroup (12.4 us per launch with it, profiles/r06n/).
template <class T>
__global__ __launch_bounds__(kQuadBlock) void k_nrm2_quad_host(int64_t n, const T* __restrict__ x,
                                                               double* __restrict__ partial,
                                                               unsigned* __restrict__ ticket,
                                                               T* __restrict__ result_host,
                                                               unsigned* __restrict__ flag_host, unsigned seq) {
    static_assert(kQuadBlock == 1024, "the last workgroup runs stage 2's 1024-lane sum");
    __shared__ double scratch[kQuadBlock / kWave];
    __shared__ unsigned arrived;
    const double s = nrm2_quad_partial(n, x, scratch);
    if (threadIdx.x == 0) {
        __hip_atomic_store(partial + blockIdx.x, s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the partial written through before the ticket
        arrived = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    if (arrived != gridDim.x - 1) return;
    const double v = threadIdx.x < gridDim.x
                         ? __hip_atomic_load(partial + threadIdx.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                         : 0.0;
    const double t = block_sum<1024>(v, scratch);
    if (threadIdx.x == 0) {
        __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(result_host, (T)sqrt(t), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        if (flag_host) {  // the result written through before the host's flag (mpg::host_poll)
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __hip_atomic_store(flag_host, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}

template <class T, bool SQRT>
__global__ __launch_bounds__(1024) void k_reduce_stage2(int nparts, const double* __restrict__ partial,
                                                        T* __restrict__ result) {
    __shared__ double scratch[1024 / kWave];
    double v = threadIdx.x < nparts ? partial[threadIdx.x] : 0.0;
    double s = block_sum<1024>(v, scratch);
    if (threadIdx.x == 0) *result = SQRT ? (T)sqrt(s) : (T)s;
}

// Stage 2 of a host-value reduction, storing straight into the context's
// pinned host word (no copy command behind it): the same sum, stored
// write-through at system scope (no L2 write-back fence), so the host's
// read after the stream completes sees it.
template <class T, bool SQRT>
__global__ __launch_bounds__(1024) void k_reduce_stage2_host(int nparts, const double* __restrict__ partial,
                                                             T* __restrict__ result_host) {
    __shared__ double scratch[1024 / kWave];
    double v = threadIdx.x < nparts ? partial[threadIdx.x] : 0.0;
    double s = block_sum<1024>(v, scratch);
    if (threadIdx.x == 0)
        __hip_atomic_store(result_host, SQRT ? (T)sqrt(s) : (T)s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Stage 2 folded into the consumer of the result (the operator surface's
// nrm2 -> scal_recip of add_vector, dot -> naxpy of the MGS kernel): every
// 1024-thread workgroup sums the stage-1 partials with stage 2's own
// block_sum<1024> (the same bits), workgroup 0 stores the result, and all
// apply it. OP 0: y = (1/r) x with r = T(sqrt(s)); OP 1: y -= T(s) x.
template <class T, int OP>
__global__ __launch_bounds__(1024) void k_consume_partials(int nparts, const double* __restrict__ partial,
                                                           T* __restrict__ result, int64_t n, const T* x, T* y) {
    __shared__ double scratch[1024 / kWave];
    __shared__ T r_s;
    double v = threadIdx.x < nparts ? partial[threadIdx.x] : 0.0;
    const double s = block_sum<1024>(v, scratch);
    if (threadIdx.x == 0) {
        const T r = OP == 0 ? (T)sqrt(s) : (T)s;
        r_s = r;
        if (blockIdx.x == 0) *result = r;
    }
    __syncthreads();
    const T r = r_s;
    const int64_t stride = (int64_t)gridDim.x * 1024;
    if (OP == 0) {
        const T a = T(1) / r;  // k_scal_copy<T, true, true>
        for (int64_t i = (int64_t)blockIdx.x * 1024 + threadIdx.x; i < n; i += stride) y[i] = a * x[i];
    } else {
        for (int64_t i = (int64_t)blockIdx.x * 1024 + threadIdx.x; i < n; i += stride) y[i] -= r * x[i];  // k_axpy NEG
    }
}

template <class T, bool SQUARE>
int reduce_partials(mpg_ctx* ctx, int64_t n, const T* x, const T* y, int32_t* nparts) {
    if (!ctx || n < 0 || !nparts) return MPG_ERR_ARG;
    if (SQUARE && n > 0 && (uintptr_t)x % 16 == 0) {
        const int gq = quad_groups(n);
        k_nrm2_quad<T><<<gq, kQuadBlock, 0, ctx->stream>>>(n, x, ctx->red_ws);
        MPG_LAUNCH_CHECK(ctx);
        *nparts = gq;
        return MPG_OK;
    }
    const int g = grid_for(n, 4, kMaxRedBlocks);
    k_reduce_stage1<T, SQUARE><<<g, kBlock, 0, ctx->stream>>>(n, x, y, ctx->red_ws);
    MPG_LAUNCH_CHECK(ctx);
    *nparts = g;
    return MPG_OK;
}

template <class T, bool SQRT>
int reduce_finish(mpg_ctx* ctx, int32_t nparts, T* result_dev) {
    if (!ctx || nparts < 1 || nparts > kMaxRedBlocks) return MPG_ERR_ARG;
    k_reduce_stage2<T, SQRT><<<1, 1024, 0, ctx->stream>>>(nparts, ctx->red_ws, result_dev);
    MPG_LAUNCH_CHECK(ctx);
    return MPG_OK;
}

template <class T, int OP>
int consume_partials(mpg_ctx* ctx, int32_t nparts, T* result_dev, int64_t n, const T* x, T* y) {
    if (!ctx || nparts < 1 || nparts > kMaxRedBlocks || n < 0) return MPG_ERR_ARG;
    const int g = (int)std::max<int64_t>(1, std::min<int64_t>(256, (n + 4 * 1024 - 1) / (4 * 1024)));
    k_consume_partials<T, OP><<<g, 1024, 0, ctx->stream>>>(nparts, ctx->red_ws, result_dev, n, x, y);
    MPG_LAUNCH_CHECK(ctx);
    return MPG_OK;
}

// Two host-value norms in one launch (the operator surface's restart
// section reads ||w|| and then ||x||, gmres.cpp:173-196; kernels_hip.cpp
// pairs them): each vector's stage 1 and stage 2 exactly as
// k_nrm2_quad_host runs them alone (the same workgroups, lanes and
// block_sum orders), so each result has the bits of its own one-launch
// read; one ticket, one hand-off, one host poll.
template <class T1, class T2>
__global__ __launch_bounds__(kQuadBlock) void k_nrm2_pair_quad_host(int64_t n, const T1* __restrict__ a,
                                                                    const T2* __restrict__ b,
                                                                    double* __restrict__ partial,
                                                                    unsigned* __restrict__ ticket,
                                                                    T1* __restrict__ ra_host, T2* __restrict__ rb_host,
                                                                    unsigned* __restrict__ flag_host, unsigned seq) {
    static_assert(kQuadBlock == 1024, "the last workgroup runs stage 2's 1024-lane sum");
    __shared__ double scratch[kQuadBlock / kWave];
    __shared__ unsigned arrived;
    const double sa = nrm2_quad_partial(n, a, scratch);
    const double sb = nrm2_quad_partial(n, b, scratch);
    if (threadIdx.x == 0) {
        __hip_atomic_store(partial + blockIdx.x, sa, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(partial + kQuadGroups + blockIdx.x, sb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // both partials written through before the ticket
        arrived = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    if (arrived != gridDim.x - 1) return;
    const bool mine = threadIdx.x < gridDim.x;
    const double va =
        mine ? __hip_atomic_load(partial + threadIdx.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0.0;
    const double vb = mine ? __hip_atomic_load(partial + kQuadGroups + threadIdx.x, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT)
                           : 0.0;
    const double ta = block_sum<1024>(va, scratch);
    const double tb = block_sum<1024>(vb, scratch);
    if (threadIdx.x == 0) {
        __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(ra_host, (T1)sqrt(ta), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(rb_host, (T2)sqrt(tb), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        if (flag_host) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __hip_atomic_store(flag_host, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}

template <class T1, class T2>
int nrm2_pair_host(mpg_ctx* ctx, int64_t n, const T1* a, const T2* b, double* ra, double* rb) {
    if ((uintptr_t)a % 16 != 0 || (uintptr_t)b % 16 != 0) return MPG_ERR_UNSUPPORTED;
    const bool poll = mpg::host_poll_on();
    const unsigned seq = poll ? mpg::host_seq_next(ctx) : 0u;
    char* hd = static_cast<char*>(ctx->host_ws_dev);
    k_nrm2_pair_quad_host<T1, T2><<<quad_groups(n), kQuadBlock, 0, ctx->stream>>>(
        n, a, b, ctx->red_ws, ctx->ticket, reinterpret_cast<T1*>(hd), reinterpret_cast<T2*>(hd + 8),
        poll ? mpg::host_flag_dev(ctx) : nullptr, seq);
    MPG_LAUNCH_CHECK(ctx);
    MPG_HIP(ctx, poll ? mpg::host_poll(ctx, seq) : mpg::spin_wait(ctx->stream));
    const char* hw = static_cast<const char*>(ctx->host_ws);
    *ra = (double)*reinterpret_cast<const volatile T1*>(hw);
    *rb = (double)*reinterpret_cast<const volatile T2*>(hw + 8);
    return MPG_OK;
}

template <class T, bool SQUARE>
int reduce(mpg_ctx* ctx, int64_t n, const T* x, const T* y, T* result_dev) {
    int32_t g = 0;
    if (int st = reduce_partials<T, SQUARE>(ctx, n, x, y, &g)) return st;
    return reduce_finish<T, SQUARE>(ctx, g, result_dev);
}

template <class T, bool SQUARE>
int reduce_host(mpg_ctx* ctx, int64_t n, const T* x, const T* y, T* result_host) {
    if (!result_host) return MPG_ERR_ARG;
    if (SQUARE && ctx && ctx->host_ws_dev && ctx->ticket && n > 0 && (uintptr_t)x % 16 == 0) {
        const bool poll = mpg::host_poll_on();
        const unsigned seq = poll ? mpg::host_seq_next(ctx) : 0u;
        k_nrm2_quad_host<T><<<quad_groups(n), kQuadBlock, 0, ctx->stream>>>(
            n, x, ctx->red_ws, ctx->ticket, (T*)ctx->host_ws_dev, poll ? mpg::host_flag_dev(ctx) : nullptr, seq);
        MPG_LAUNCH_CHECK(ctx);
        MPG_HIP(ctx, poll ? mpg::host_poll(ctx, seq) : mpg::spin_wait(ctx->stream));
        *result_host = *static_cast<volatile T*>(ctx->host_ws);
        return MPG_OK;
    }
    if (ctx && ctx->host_ws_dev) {  // stage 2 stores into pinned host memory; a polled wait
        int32_t g = 0;
        if (int st = reduce_partials<T, SQUARE>(ctx, n, x, y, &g)) return st;
        if (g < 1 || g > kMaxRedBlocks) return MPG_ERR_ARG;
        k_reduce_stage2_host<T, SQUARE><<<1, 1024, 0, ctx->stream>>>(g, ctx->red_ws, (T*)ctx->host_ws_dev);
        MPG_LAUNCH_CHECK(ctx);
        MPG_HIP(ctx, mpg::spin_wait(ctx->stream));
        *result_host = *static_cast<volatile T*>(ctx->host_ws);
        return MPG_OK;
    }
    T* tmp = reinterpret_cast<T*>(ctx->red_ws + kMaxRedBlocks * kGemvMaxCols);
    int st = reduce<T, SQUARE>(ctx, n, x, y, tmp);
    if (st) return st;
    return mpg_memcpy_d2h(ctx, result_host, tmp, sizeof(T));  // (pinned staging, polled wait)
}

// ---------------- elementwise ----------------
// mode: 0 y += a x ; 1 y -= a x
template <class T, bool ALPHA_DEV, bool NEG>
__global__ __launch_bounds__(kBlock) void k_axpy(int64_t n, T alpha, const T* __restrict__ alpha_dev,
                                                 const T* __restrict__ x, T* __restrict__ y) {
    const T a = ALPHA_DEV ? *alpha_dev : alpha;
    const int64_t stride = (int64_t)gridDim.x * kBlock;
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride) {
        if (NEG) y[i] -= a * x[i];   // naxpy: y(i) -= alpha()*x(i) (kernels_cuda.cpp:271-274)
        else y[i] += a * x[i];
    }
}

// y = a*x ; RECIP: a = 1/alpha formed on device in T
template <class T, bool ALPHA_DEV, bool RECIP>
__global__ __launch_bounds__(kBlock) void k_scal_copy(int64_t n, T alpha, const T* __restrict__ alpha_dev,
                                                      const T* x, T* y) {
    T a = ALPHA_DEV ? *alpha_dev : alpha;
    if (RECIP) a = T(1) / a;
    const int64_t stride = (int64_t)gridDim.x * kBlock;
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride) y[i] = a * x[i];
}

template <class S, class D>
__global__ __launch_bounds__(kBlock) void k_copy(int64_t n, const S* __restrict__ x, D* __restrict__ y) {
    const int64_t stride = (int64_t)gridDim.x * kBlock;
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride) y[i] = (D)x[i];
}

template <class S>
__global__ __launch_bounds__(kBlock) void k_copy_half(int64_t n, const S* __restrict__ x, uint16_t* __restrict__ y) {
    const int64_t stride = (int64_t)gridDim.x * kBlock;
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride)
        y[i] = __half_as_ushort(__float2half_rn((float)x[i]));
}

template <class E>
__global__ __launch_bounds__(kBlock) void k_gather(int64_t n, const int32_t* __restrict__ idx, const E* __restrict__ x,
                                                   E* __restrict__ y) {
    const int64_t stride = (int64_t)gridDim.x * kBlock;
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride) y[i] = x[idx[i]];
}

template <class E>
int gather_impl(mpg_ctx* ctx, int64_t n, const int32_t* idx, const void* x, void* y) {
    if (!ctx || n < 0) return MPG_ERR_ARG;
    if (n == 0) return MPG_OK;
    k_gather<E><<<grid_for(n, 1), kBlock, 0, ctx->stream>>>(n, idx, static_cast<const E*>(x), static_cast<E*>(y));
    MPG_LAUNCH_CHECK(ctx);
    return MPG_OK;
}

template <class T>
__global__ __launch_bounds__(kBlock) void k_fill(T* x, int64_t rows, int64_t cols, int64_t ld, T v) {
    const int64_t total = rows * cols;
    const int64_t stride = (int64_t)gridDim.x * kBlock;
    for (int64_t t = (int64_t)blockIdx.x * kBlock + threadIdx.x; t < total; t += stride) {
        int64_t c = t / rows, r = t - c * rows;
        x[c * ld + r] = v;
    }
}

template <class T>
__global__ __launch_bounds__(kBlock) void k_gdmv(int64_t n, T alpha, const T* __restrict__ d,
                                                 const T* x, T beta, T* y) {
    const int64_t stride = (int64_t)gridDim.x * kBlock;
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride)
        y[i] = beta * y[i] + alpha * d[i] * x[i];   // kernels.hpp:141-144 (x may alias y)
}

template <class T>
__global__ void k_rotg(T* a, T* b, T* c, T* s) { rotg_dev(a, b, c, s); }

template <class T>
__global__ void k_rot(T* a, T* b, const T* c, const T* s) { rot_pair(a, b, *c, *s); }

template <class T>
__global__ void k_rot_vec(int k, T* a, const T* c, const T* s) {
    for (int j = 0; j < k; ++j) rot_pair(a + j, a + j + 1, c[j], s[j]);
}

constexpr int kRotStage = 256;  // rotations staged in LDS per pass

__global__ __launch_bounds__(kWave) void k_scalar_program(ScalarProgram prog) {
    __shared__ double lds[3 * kRotStage + 1];
    run_scalar_program<kRotStage>(prog, lds);
}

template <class T, bool ALPHA_DEV>
__global__ void k_scal_scalar(T alpha, const T* alpha_dev, const T* x, T* y) {
    y[0] = (ALPHA_DEV ? *alpha_dev : alpha) * x[0];
}

template <class T, bool ALPHA_DEV, bool NEG>
int axpy_impl(mpg_ctx* ctx, int64_t n, T alpha, const T* alpha_dev, const T* x, T* y) {
    if (!ctx || n < 0) return MPG_ERR_ARG;
    if (n == 0) return MPG_OK;
    k_axpy<T, ALPHA_DEV, NEG><<<grid_for(n, 4), kBlock, 0, ctx->stream>>>(n, alpha, alpha_dev, x, y);
    MPG_LAUNCH_CHECK(ctx);
    return MPG_OK;
}

template <class T, bool ALPHA_DEV, bool RECIP>
int scal_copy_impl(mpg_ctx* ctx, int64_t n, T alpha, const T* alpha_dev, const T* x, T* y) {
    if (!ctx || n < 0) return MPG_ERR_ARG;
    if (n == 0) return MPG_OK;
    k_scal_copy<T, ALPHA_DEV, RECIP><<<grid_for(n, 4), kBlock, 0, ctx->stream>>>(n, alpha, alpha_dev, x, y);
    MPG_LAUNCH_CHECK(ctx);
    return MPG_OK;
}

template <class S, class D>
int copy_impl(mpg_ctx* ctx, int64_t n, const S* x, D* y) {
    if (!ctx || n < 0) return MPG_ERR_ARG;
    if (n == 0) return MPG_OK;
    k_copy<S, D><<<grid_for(n, 4), kBlock, 0, ctx->stream>>>(n, x, y);
    MPG_LAUNCH_CHECK(ctx);
    return MPG_OK;
}

template <class T>
int fill_impl(mpg_ctx* ctx, T* x, int64_t rows, int64_t cols, int64_t ld, T v) {
    if (!ctx || rows < 0 || cols < 0 || (cols > 1 && ld < rows)) return MPG_ERR_ARG;
    if (rows == 0 || cols == 0) return MPG_OK;
    k_fill<T><<<grid_for(rows * cols, 4), kBlock, 0, ctx->stream>>>(x, rows, cols, ld, v);
    MPG_LAUNCH_CHECK(ctx);
    return MPG_OK;
}

template <class T>
int gdmv_impl(mpg_ctx* ctx, int64_t n, T alpha, const T* d, const T* x, T beta, T* y) {
    if (!ctx || n < 0) return MPG_ERR_ARG;
    if (n == 0) return MPG_OK;
    k_gdmv<T><<<grid_for(n, 4), kBlock, 0, ctx->stream>>>(n, alpha, d, x, beta, y);
    MPG_LAUNCH_CHECK(ctx);
    return MPG_OK;
}

}  // namespace

extern "C" {

int mpg_dot_f64(mpg_ctx_t c, int64_t n, const double* x, const double* y, double* r) { return reduce<double, false>(c, n, x, y, r); }
int mpg_dot_f32(mpg_ctx_t c, int64_t n, const float* x, const float* y, float* r) { return reduce<float, false>(c, n, x, y, r); }
int mpg_dot_f64_host(mpg_ctx_t c, int64_t n, const double* x, const double* y, double* r) { return reduce_host<double, false>(c, n, x, y, r); }
int mpg_dot_f32_host(mpg_ctx_t c, int64_t n, const float* x, const float* y, float* r) { return reduce_host<float, false>(c, n, x, y, r); }
int mpg_dot_partials_f64(mpg_ctx_t c, int64_t n, const double* x, const double* y, int32_t* np) { return reduce_partials<double, false>(c, n, x, y, np); }
int mpg_dot_partials_f32(mpg_ctx_t c, int64_t n, const float* x, const float* y, int32_t* np) { return reduce_partials<float, false>(c, n, x, y, np); }
int mpg_nrm2_partials_f64(mpg_ctx_t c, int64_t n, const double* x, int32_t* np) { return reduce_partials<double, true>(c, n, x, x, np); }
int mpg_nrm2_partials_f32(mpg_ctx_t c, int64_t n, const float* x, int32_t* np) { return reduce_partials<float, true>(c, n, x, x, np); }
int mpg_dot_finish_f64(mpg_ctx_t c, int32_t np, double* r) { return reduce_finish<double, false>(c, np, r); }
int mpg_dot_finish_f32(mpg_ctx_t c, int32_t np, float* r) { return reduce_finish<float, false>(c, np, r); }
int mpg_nrm2_finish_f64(mpg_ctx_t c, int32_t np, double* r) { return reduce_finish<double, true>(c, np, r); }
int mpg_nrm2_finish_f32(mpg_ctx_t c, int32_t np, float* r) { return reduce_finish<float, true>(c, np, r); }
int mpg_scal_recip_nrm2_f64(mpg_ctx_t c, int32_t np, double* h, int64_t n, const double* x, double* y) { return consume_partials<double, 0>(c, np, h, n, x, y); }
int mpg_scal_recip_nrm2_f32(mpg_ctx_t c, int32_t np, float* h, int64_t n, const float* x, float* y) { return consume_partials<float, 0>(c, np, h, n, x, y); }
int mpg_naxpy_dot_f64(mpg_ctx_t c, int32_t np, double* a, int64_t n, const double* x, double* y) { return consume_partials<double, 1>(c, np, a, n, x, y); }
int mpg_naxpy_dot_f32(mpg_ctx_t c, int32_t np, float* a, int64_t n, const float* x, float* y) { return consume_partials<float, 1>(c, np, a, n, x, y); }
int mpg_nrm2_f64(mpg_ctx_t c, int64_t n, const double* x, double* r) { return reduce<double, true>(c, n, x, x, r); }
int mpg_nrm2_f32(mpg_ctx_t c, int64_t n, const float* x, float* r) { return reduce<float, true>(c, n, x, x, r); }
int mpg_nrm2_f64_host(mpg_ctx_t c, int64_t n, const double* x, double* r) { return reduce_host<double, true>(c, n, x, x, r); }
int mpg_nrm2_f32_host(mpg_ctx_t c, int64_t n, const float* x, float* r) { return reduce_host<float, true>(c, n, x, x, r); }
int mpg_nrm2_pair_host(mpg_ctx_t c, int64_t n, int type_a, const void* a, int type_b, const void* b, double* norm_a,
                       double* norm_b) {
    if (!c || !a || !b || !norm_a || !norm_b || n < 1) return MPG_ERR_ARG;
    if (!c->host_ws_dev || !c->ticket) return MPG_ERR_UNSUPPORTED;
    const bool a64 = type_a == MPG_F64, b64 = type_b == MPG_F64;
    if ((!a64 && type_a != MPG_F32) || (!b64 && type_b != MPG_F32)) return MPG_ERR_ARG;
    if (a64 && b64) return nrm2_pair_host(c, n, (const double*)a, (const double*)b, norm_a, norm_b);
    if (a64) return nrm2_pair_host(c, n, (const double*)a, (const float*)b, norm_a, norm_b);
    if (b64) return nrm2_pair_host(c, n, (const float*)a, (const double*)b, norm_a, norm_b);
    return nrm2_pair_host(c, n, (const float*)a, (const float*)b, norm_a, norm_b);
}
int mpg_dot_acc_f64(mpg_ctx_t c, int64_t n, const double* x, const double* y, double* acc) {
    if (!c || n < 0) return MPG_ERR_ARG;
    int g = grid_for(n, 4, kMaxRedBlocks);
    k_reduce_stage1<double, false><<<g, kBlock, 0, c->stream>>>(n, x, y, c->red_ws);
    MPG_LAUNCH_CHECK(c);
    k_reduce_stage2<double, false><<<1, 1024, 0, c->stream>>>(g, c->red_ws, acc);
    MPG_LAUNCH_CHECK(c);
    return MPG_OK;
}
int mpg_dot_acc_f32(mpg_ctx_t c, int64_t n, const float* x, const float* y, double* acc) {
    if (!c || n < 0) return MPG_ERR_ARG;
    int g = grid_for(n, 4, kMaxRedBlocks);
    k_reduce_stage1<float, false><<<g, kBlock, 0, c->stream>>>(n, x, y, c->red_ws);
    MPG_LAUNCH_CHECK(c);
    k_reduce_stage2<double, false><<<1, 1024, 0, c->stream>>>(g, c->red_ws, acc);
    MPG_LAUNCH_CHECK(c);
    return MPG_OK;
}

int mpg_axpy_f64(mpg_ctx_t c, int64_t n, double a, const double* x, double* y) { return axpy_impl<double, false, false>(c, n, a, nullptr, x, y); }
int mpg_axpy_f32(mpg_ctx_t c, int64_t n, float a, const float* x, float* y) { return axpy_impl<float, false, false>(c, n, a, nullptr, x, y); }
int mpg_axpy_dev_f64(mpg_ctx_t c, int64_t n, const double* a, const double* x, double* y) { return axpy_impl<double, true, false>(c, n, 0.0, a, x, y); }
int mpg_axpy_dev_f32(mpg_ctx_t c, int64_t n, const float* a, const float* x, float* y) { return axpy_impl<float, true, false>(c, n, 0.f, a, x, y); }
int mpg_naxpy_dev_f64(mpg_ctx_t c, int64_t n, const double* a, const double* x, double* y) { return axpy_impl<double, true, true>(c, n, 0.0, a, x, y); }
int mpg_naxpy_dev_f32(mpg_ctx_t c, int64_t n, const float* a, const float* x, float* y) { return axpy_impl<float, true, true>(c, n, 0.f, a, x, y); }

int mpg_scal_f64(mpg_ctx_t c, int64_t n, double a, double* x) { return scal_copy_impl<double, false, false>(c, n, a, nullptr, x, x); }
int mpg_scal_f32(mpg_ctx_t c, int64_t n, float a, float* x) { return scal_copy_impl<float, false, false>(c, n, a, nullptr, x, x); }
int mpg_scal_copy_f64(mpg_ctx_t c, int64_t n, double a, const double* x, double* y) { return scal_copy_impl<double, false, false>(c, n, a, nullptr, x, y); }
int mpg_scal_copy_f32(mpg_ctx_t c, int64_t n, float a, const float* x, float* y) { return scal_copy_impl<float, false, false>(c, n, a, nullptr, x, y); }
int mpg_scal_copy_dev_f64(mpg_ctx_t c, int64_t n, const double* a, const double* x, double* y) { return scal_copy_impl<double, true, false>(c, n, 0.0, a, x, y); }
int mpg_scal_copy_dev_f32(mpg_ctx_t c, int64_t n, const float* a, const float* x, float* y) { return scal_copy_impl<float, true, false>(c, n, 0.f, a, x, y); }
int mpg_scal_recip_copy_dev_f64(mpg_ctx_t c, int64_t n, const double* a, const double* x, double* y) { return scal_copy_impl<double, true, true>(c, n, 0.0, a, x, y); }
int mpg_scal_recip_copy_dev_f32(mpg_ctx_t c, int64_t n, const float* a, const float* x, float* y) { return scal_copy_impl<float, true, true>(c, n, 0.f, a, x, y); }

int mpg_copy_f64f64(mpg_ctx_t c, int64_t n, const double* x, double* y) { return copy_impl(c, n, x, y); }
int mpg_copy_f32f32(mpg_ctx_t c, int64_t n, const float* x, float* y) { return copy_impl(c, n, x, y); }
int mpg_copy_f64f32(mpg_ctx_t c, int64_t n, const double* x, float* y) { return copy_impl(c, n, x, y); }
int mpg_copy_f32f64(mpg_ctx_t c, int64_t n, const float* x, double* y) { return copy_impl(c, n, x, y); }
int mpg_copy_f64f16(mpg_ctx_t c, int64_t n, const double* x, uint16_t* y) {
    if (!c || n < 0) return MPG_ERR_ARG;
    if (n == 0) return MPG_OK;
    k_copy_half<double><<<grid_for(n, 4), kBlock, 0, c->stream>>>(n, x, y);
    MPG_LAUNCH_CHECK(c);
    return MPG_OK;
}
int mpg_copy_f32f16(mpg_ctx_t c, int64_t n, const float* x, uint16_t* y) {
    if (!c || n < 0) return MPG_ERR_ARG;
    if (n == 0) return MPG_OK;
    k_copy_half<float><<<grid_for(n, 4), kBlock, 0, c->stream>>>(n, x, y);
    MPG_LAUNCH_CHECK(c);
    return MPG_OK;
}

int mpg_gather_b32(mpg_ctx_t c, int64_t n, const int32_t* idx, const void* x, void* y) { return gather_impl<uint32_t>(c, n, idx, x, y); }
int mpg_gather_b64(mpg_ctx_t c, int64_t n, const int32_t* idx, const void* x, void* y) { return gather_impl<uint64_t>(c, n, idx, x, y); }
int mpg_fill_f64(mpg_ctx_t c, double* x, int64_t r, int64_t cl, int64_t ld, double v) { return fill_impl(c, x, r, cl, ld, v); }
int mpg_fill_f32(mpg_ctx_t c, float* x, int64_t r, int64_t cl, int64_t ld, float v) { return fill_impl(c, x, r, cl, ld, v); }
int mpg_gdmv_f64(mpg_ctx_t c, int64_t n, double a, const double* d, const double* x, double b, double* y) { return gdmv_impl(c, n, a, d, x, b, y); }
int mpg_gdmv_f32(mpg_ctx_t c, int64_t n, float a, const float* d, const float* x, float b, float* y) { return gdmv_impl(c, n, a, d, x, b, y); }

#define MPG_SINGLE(ctx, launch)             \
    do {                                    \
        if (!(ctx)) return MPG_ERR_ARG;     \
        launch;                             \
        MPG_LAUNCH_CHECK(ctx);              \
        return MPG_OK;                      \
    } while (0)

int mpg_rotg_f64(mpg_ctx_t c, double* a, double* b, double* cs, double* s) { MPG_SINGLE(c, (k_rotg<double><<<1, 1, 0, c->stream>>>(a, b, cs, s))); }
int mpg_rotg_f32(mpg_ctx_t c, float* a, float* b, float* cs, float* s) { MPG_SINGLE(c, (k_rotg<float><<<1, 1, 0, c->stream>>>(a, b, cs, s))); }
int mpg_rot_f64(mpg_ctx_t c, double* a, double* b, const double* cs, const double* s) { MPG_SINGLE(c, (k_rot<double><<<1, 1, 0, c->stream>>>(a, b, cs, s))); }
int mpg_rot_f32(mpg_ctx_t c, float* a, float* b, const float* cs, const float* s) { MPG_SINGLE(c, (k_rot<float><<<1, 1, 0, c->stream>>>(a, b, cs, s))); }
int mpg_rot_vec_f64(mpg_ctx_t c, int k, double* a, const double* cs, const double* s) {
    if (k <= 0) return c ? MPG_OK : MPG_ERR_ARG;
    MPG_SINGLE(c, (k_rot_vec<double><<<1, 1, 0, c->stream>>>(k, a, cs, s)));
}
int mpg_rot_vec_f32(mpg_ctx_t c, int k, float* a, const float* cs, const float* s) {
    if (k <= 0) return c ? MPG_OK : MPG_ERR_ARG;
    MPG_SINGLE(c, (k_rot_vec<float><<<1, 1, 0, c->stream>>>(k, a, cs, s)));
}
int mpg_scalar_program(mpg_ctx_t c, const mpg_scalar_op* ops, int count) {
    ScalarProgram prog;
    if (!c || make_scalar_program(ops, count, prog) != MPG_OK) return MPG_ERR_ARG;
    if (count == 0) return MPG_OK;
    MPG_SINGLE(c, (k_scalar_program<<<1, kWave, 0, c->stream>>>(prog)));
}
int mpg_scal_scalar_f64(mpg_ctx_t c, double a, const double* x, double* y) { MPG_SINGLE(c, (k_scal_scalar<double, false><<<1, 1, 0, c->stream>>>(a, nullptr, x, y))); }
int mpg_scal_scalar_f32(mpg_ctx_t c, float a, const float* x, float* y) { MPG_SINGLE(c, (k_scal_scalar<float, false><<<1, 1, 0, c->stream>>>(a, nullptr, x, y))); }
int mpg_scal_scalar_dev_f64(mpg_ctx_t c, const double* a, const double* x, double* y) { MPG_SINGLE(c, (k_scal_scalar<double, true><<<1, 1, 0, c->stream>>>(0.0, a, x, y))); }
int mpg_scal_scalar_dev_f32(mpg_ctx_t c, const float* a, const float* x, float* y) { MPG_SINGLE(c, (k_scal_scalar<float, true><<<1, 1, 0, c->stream>>>(0.f, a, x, y))); }

}  // extern "C"
