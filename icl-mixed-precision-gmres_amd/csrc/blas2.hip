// BLAS-2 surface (kernels_mkl.cpp:264-321): column-major gemv with explicit
// lda, and small triangular solves.
//
// gemv^T on a tall-skinny panel (the CGS V^T w of Orthogonalization.hpp:
// 83-87) is a two-stage panel reduction: every workgroup streams a slab of
// rows once, keeps one fp64 accumulator per column (<= 32 per pass) in
// registers, reduces each across its 4 waves with wave64 shuffles, and
// writes per-workgroup partials; stage 2 sums the partials of each column in
// a fixed order. gemv (no transpose) is row-per-lane with fp64 accumulation.
//
// Panels whose columns start on 16-B granules (A, lda and the row-indexed
// vector aligned: the padded Krylov basis of MultiVect always is) take the
// quad forms: 1024-thread workgroups, one per CU, each lane 4 consecutive
// rows with 16-B loads of every column issued in compile-time batches (the
// fused cycle's panel kernels, arnoldi.hip k_dots_nc / k_cgs_update_nc).
#include "internal.hpp"
#include "panel.hpp"

#include <algorithm>
#include <cstdlib>

using namespace mpg;

namespace {

template <class T>
__global__ __launch_bounds__(kBlock) void k_gemv_t_stage1(int64_t rows, int ncols, const T* __restrict__ A,
                                                          int64_t lda, const T* __restrict__ x,
                                                          double* __restrict__ partial) {
    __shared__ double scratch[kBlock / kWave][kGemvMaxCols];
    double acc[kGemvMaxCols];
#pragma unroll
    for (int c = 0; c < kGemvMaxCols; ++c) acc[c] = 0.0;
    const int64_t stride = (int64_t)gridDim.x * kBlock;
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < rows; i += stride) {
        const double xi = (double)x[i];
#pragma unroll
        for (int c = 0; c < kGemvMaxCols; ++c)
            if (c < ncols) acc[c] += (double)A[(int64_t)c * lda + i] * xi;
    }
    const int lane = threadIdx.x & (kWave - 1);
    const int wid = threadIdx.x / kWave;
#pragma unroll
    for (int c = 0; c < kGemvMaxCols; ++c) {
        if (c < ncols) {
            double v = wave_sum(acc[c]);
            if (lane == 0) scratch[wid][c] = v;
        }
    }
    __syncthreads();
    if (threadIdx.x < ncols) {
        double s = 0.0;
#pragma unroll
        for (int w = 0; w < kBlock / kWave; ++w) s += scratch[w][threadIdx.x];
        partial[(int64_t)threadIdx.x * gridDim.x + blockIdx.x] = s;
    }
}

// k_gemv_t_stage1 with the column count a compile-time constant (the
// driver's gemv calls have k+1 <= 32 columns): every column index is static,
// so a batch of columns' loads issues back to back instead of one guarded
// load (and one memory latency) per column. One row per lane with scalar
// loads: no alignment assumption on A, lda or x.
template <class T, int NC>
__global__ __launch_bounds__(kBlock) void k_gemv_t_nc(int64_t rows, const T* __restrict__ A, int64_t lda,
                                                      const T* __restrict__ x, double* __restrict__ partial) {
    constexpr int B = 16;
    __shared__ double scratch[kBlock / kWave][NC];
    double acc[NC];
#pragma unroll
    for (int c = 0; c < NC; ++c) acc[c] = 0.0;
    const int64_t stride = (int64_t)gridDim.x * kBlock;
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < rows; i += stride) {
        const T xr = x[i];
#pragma unroll
        for (int c0 = 0; c0 < NC; c0 += B) {
            T v[B];
#pragma unroll
            for (int u = 0; u < B; ++u)
                if (c0 + u < NC) v[u] = A[(int64_t)(c0 + u) * lda + i];
            __builtin_amdgcn_sched_barrier(0);  // the batch's loads back to back
#pragma unroll
            for (int u = 0; u < B; ++u)
                if (c0 + u < NC) acc[c0 + u] += (double)v[u] * (double)xr;
        }
    }
    const int lane = threadIdx.x & (kWave - 1);
    const int wid = threadIdx.x / kWave;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
        const double v = wave_sum(acc[c]);
        if (lane == 0) scratch[wid][c] = v;
    }
    __syncthreads();
    if (threadIdx.x < NC) {
        double s = 0.0;
#pragma unroll
        for (int w = 0; w < kBlock / kWave; ++w) s += scratch[w][threadIdx.x];
        partial[(int64_t)threadIdx.x * gridDim.x + blockIdx.x] = s;
    }
}

// k_gemv_n with a compile-time column count (batched loads, same order)
template <class T, int NC>
__global__ __launch_bounds__(kBlock) void k_gemv_n_nc(int64_t rows, T alpha, const T* __restrict__ A, int64_t lda,
                                                      const T* __restrict__ x, T beta, T* __restrict__ y) {
    constexpr int B = 16;
    const int64_t stride = (int64_t)gridDim.x * kBlock;
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < rows; i += stride) {
        const T yi = beta == T(0) ? T(0) : y[i];
        double acc = 0.0;
#pragma unroll
        for (int c0 = 0; c0 < NC; c0 += B) {
            T v[B];
#pragma unroll
            for (int u = 0; u < B; ++u)
                if (c0 + u < NC) v[u] = A[(int64_t)(c0 + u) * lda + i];
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int u = 0; u < B; ++u)
                if (c0 + u < NC) acc += (double)v[u] * (double)x[c0 + u];
        }
        const T t = (T)acc;
        y[i] = beta == T(0) ? alpha * t : alpha * t + beta * yi;
    }
}

// Stage 2 of gemv^T: one wave per column, lane l summing partials l, l + 64,
// ... in order, then the wave's shuffle tree. The fused gemv (N)
// forms its coefficients with the same function, so both give the same bits.
// The loads go out four at a time (clamped addresses) before the adds, which
// stay the same adds in the same order: a runtime-count loop otherwise waits
// one memory latency per partial (the fused gemv's fixed cost, round 4).
__device__ __forceinline__ double column_sum(const double* __restrict__ partial, int nparts, int c, int lane) {
    const double* __restrict__ p = partial + (int64_t)c * nparts;
    double v = 0.0;
    for (int j = lane; j < nparts; j += 4 * kWave) {
        double q[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int jj = j + u * kWave;
            q[u] = p[jj < nparts ? jj : 0];
        }
#pragma unroll
        for (int u = 0; u < 4; ++u)
            if (j + u * kWave < nparts) v += q[u];
    }
    return wave_sum(v);
}


// partial <A(:,c), x> per workgroup, 4 rows per lane (16-B loads)
template <class T, int NC>
__global__ __launch_bounds__(kQuadBlock) void k_gemv_t_quad(int64_t rows, const T* __restrict__ A, int64_t lda,
                                                            const T* __restrict__ x, double* __restrict__ partial) {
    constexpr int NP = Pow2Ceil<NC>::v;
    constexpr int B = kColBatch<T>;
    double acc[NP];
#pragma unroll
    for (int c = 0; c < NP; ++c) acc[c] = 0.0;
    // 32-bit row indices (rows < kQuadMaxRows, quad_aligned), as the fused
    // engine's panel kernels: the 64-bit loop cost ~0.7 us per launch
    const int n4 = (int)rows & ~3;
    const int step = 4 * (int)gridDim.x * kQuadBlock;
    for (int i = 4 * ((int)blockIdx.x * kQuadBlock + (int)threadIdx.x); i < n4; i += step) {
        double xv[4];
        Row4<T>::load(x + i, xv);
#pragma unroll
        for (int c0 = 0; c0 < NC; c0 += B) {
            Raw4<T> v[B];
#pragma unroll
            for (int u = 0; u < B; ++u)
                if (c0 + u < NC) v[u].load(A + (int64_t)(c0 + u) * lda + i);
            __builtin_amdgcn_sched_barrier(0);  // the batch's loads back to back
#pragma unroll
            for (int u = 0; u < B; ++u)
                if (c0 + u < NC) acc[c0 + u] += v[u][0] * xv[0] + v[u][1] * xv[1] + v[u][2] * xv[2] + v[u][3] * xv[3];
        }
    }
    for (int i = n4 + (int)blockIdx.x * kQuadBlock + (int)threadIdx.x; i < (int)rows; i += (int)gridDim.x * kQuadBlock) {
        const double xi = (double)x[i];
#pragma unroll
        for (int c = 0; c < NC; ++c) acc[c] += (double)A[(int64_t)c * lda + i] * xi;
    }
    store_partials<NP, kQuadBlock>(acc, NC, partial);
}

// y = alpha*T(A x) + beta*y, 4 rows per lane, fp64 sums in column order.
// FROM_PARTS: x is the pending result of a gemv^T whose stage-1 partials are
// in `partial` (x = alpha_t * T(sum), beta_t = 0): every workgroup forms the
// coefficients itself with stage 2's column_sum and workgroup 0 stores them
// to x, saving the stage-2 launch (CGS: h = V^T w, then w -= V h).
// NORM: also the ||y||^2 stage-1 partials of the y it writes, in the quad
// nrm2 stage 1's layout and order (k_nrm2_quad, blas1.hip: the lane's rows
// in order, then block_sum<kQuadBlock>), so an nrm2(y) right after needs no
// launch of its own (CGS: w -= V h, then h_{k+1,k} = ||w||)
// y_out (round 5): the result goes there instead of y (a distinct buffer)
template <class T, int NC, bool FROM_PARTS = false, bool NORM = false>
__global__ __launch_bounds__(kQuadBlock) void k_gemv_n_quad(int64_t rows, T alpha, const T* __restrict__ A,
                                                            int64_t lda, T* __restrict__ x, T beta,
                                                            T* __restrict__ y, const double* __restrict__ partial = nullptr,
                                                            int nparts = 0, T alpha_t = T(1),
                                                            double* __restrict__ norm_part = nullptr,
                                                            T* __restrict__ y_out = nullptr) {
    T* __restrict__ yo = y_out ? y_out : y;
    constexpr int B = kColBatch<T>;
    __shared__ double xs[NC];
    double nacc = 0.0;
    if constexpr (FROM_PARTS) {
        const int lane = threadIdx.x & (kWave - 1), wid = threadIdx.x / kWave;
        for (int c = wid; c < NC; c += kQuadBlock / kWave) {
            const double sc = column_sum(partial, nparts, c, lane);
            if (lane == 0) {
                const T h = alpha_t * (T)sc;
                xs[c] = (double)h;
                if (blockIdx.x == 0) x[c] = h;
            }
        }
    } else {
        if (threadIdx.x < NC) xs[threadIdx.x] = (double)x[threadIdx.x];
    }
    __syncthreads();
    const int n4 = (int)rows & ~3;  // (32-bit row indices, as k_gemv_t_quad)
    const int step = 4 * (int)gridDim.x * kQuadBlock;
    for (int i = 4 * ((int)blockIdx.x * kQuadBlock + (int)threadIdx.x); i < n4; i += step) {
        Raw4<T> yr;
        if (beta != T(0)) yr.load(y + i);
        double t[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int c0 = 0; c0 < NC; c0 += B) {
            Raw4<T> v[B];
#pragma unroll
            for (int u = 0; u < B; ++u)
                if (c0 + u < NC) v[u].load(A + (int64_t)(c0 + u) * lda + i);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int u = 0; u < B; ++u)
                if (c0 + u < NC) {
                    const double xu = xs[c0 + u];
#pragma unroll
                    for (int r = 0; r < 4; ++r) t[r] += v[u][r] * xu;
                }
        }
        T out[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) out[r] = beta == T(0) ? alpha * (T)t[r] : alpha * (T)t[r] + beta * (T)yr[r];
        Row4<T>::store(yo + i, out);
        if constexpr (NORM) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const double a = (double)out[r];
                nacc += a * a;
            }
        }
    }
    for (int i = n4 + (int)blockIdx.x * kQuadBlock + (int)threadIdx.x; i < (int)rows; i += (int)gridDim.x * kQuadBlock) {
        double t = 0.0;
#pragma unroll
        for (int c = 0; c < NC; ++c) t += (double)A[(int64_t)c * lda + i] * xs[c];
        const T tt = (T)t;
        const T yi = beta == T(0) ? alpha * tt : alpha * tt + beta * y[i];
        yo[i] = yi;
        if constexpr (NORM) {
            const double a = (double)yi;
            nacc += a * a;
        }
    }
    if constexpr (NORM) {
        __shared__ double scratch[kQuadBlock / kWave];
        const double s = block_sum<kQuadBlock>(nacc, scratch);
        if (threadIdx.x == 0) norm_part[blockIdx.x] = s;
    }
}

// the quad kernels index rows with 32-bit integers
constexpr int64_t kQuadMaxRows = int64_t(1) << 30;

template <class T>
bool quad_aligned(const T* A, int64_t lda, const T* v, int64_t rows) {
    return ((uintptr_t)A % 16 == 0) && ((uintptr_t)v % 16 == 0) && ((lda * (int64_t)sizeof(T)) % 16 == 0) &&
           rows < kQuadMaxRows;
}

// f(integral_constant<int, nc>) for 1 <= nc <= N
template <int N, class F>
int with_cols(int nc, F&& f) {
    if constexpr (N == 0) {
        return MPG_ERR_ARG;
    } else {
        if (nc == N) return f(std::integral_constant<int, N>());
        return with_cols<N - 1>(nc, f);
    }
}


template <class T>
__global__ __launch_bounds__(1024) void k_gemv_t_stage2(int nparts, int nc, const double* __restrict__ partial,
                                                        T alpha, T beta, T* __restrict__ y) {
    const int lane = threadIdx.x & (kWave - 1), wid = threadIdx.x / kWave;
    for (int c = wid; c < nc; c += 1024 / kWave) {
        const double s = column_sum(partial, nparts, c, lane);
        if (lane == 0) {
            const T t = (T)s;
            y[c] = beta == T(0) ? alpha * t : alpha * t + beta * y[c];
        }
    }
}

template <class T>
__global__ __launch_bounds__(kBlock) void k_gemv_n(int64_t rows, int64_t cols, T alpha, const T* __restrict__ A,
                                                   int64_t lda, const T* __restrict__ x, T beta,
                                                   T* __restrict__ y) {
    const int64_t stride = (int64_t)gridDim.x * kBlock;
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < rows; i += stride) {
        double acc = 0.0;
        for (int64_t c = 0; c < cols; ++c) acc += (double)A[c * lda + i] * (double)x[c];
        T t = (T)acc;
        y[i] = beta == T(0) ? alpha * t : alpha * t + beta * y[i];
    }
}

template <class T>
int gemv_impl(mpg_ctx* ctx, int trans, int64_t rows, int64_t cols, T alpha, const T* A, int64_t lda,
              const T* x, T beta, T* y) {
    if (!ctx || rows < 0 || cols < 0 || (cols > 0 && lda < (rows > 0 ? rows : 1))) return MPG_ERR_ARG;
    if (!trans) {
        if (rows == 0) return MPG_OK;
        if (cols >= 1 && cols <= kGemvMaxCols && quad_aligned(A, lda, y, rows)) {
            const int g = (int)std::min<int64_t>(kQuadGroups, (rows + 4 * kQuadBlock - 1) / (4 * kQuadBlock));
            const int st = with_cols<kGemvMaxCols>((int)cols, [&](auto nc) {
                k_gemv_n_quad<T, decltype(nc)::value><<<g, kQuadBlock, 0, ctx->stream>>>(
                    rows, alpha, A, lda, const_cast<T*>(x), beta, y);
                return (int)MPG_OK;
            });
            if (st) return st;
        } else if (cols >= 1 && cols <= kGemvMaxCols) {
            const int st = with_cols<kGemvMaxCols>((int)cols, [&](auto nc) {
                k_gemv_n_nc<T, decltype(nc)::value><<<grid_for(rows, 1), kBlock, 0, ctx->stream>>>(
                    rows, alpha, A, lda, x, beta, y);
                return (int)MPG_OK;
            });
            if (st) return st;
        } else {
            k_gemv_n<T><<<grid_for(rows, 1), kBlock, 0, ctx->stream>>>(rows, cols, alpha, A, lda, x, beta, y);
        }
        MPG_LAUNCH_CHECK(ctx);
        return MPG_OK;
    }
    if (cols == 0) return MPG_OK;
    const bool quad = quad_aligned(A, lda, x, rows);
    int g = quad ? (int)std::max<int64_t>(1, std::min<int64_t>(kQuadGroups, (rows + 4 * kQuadBlock - 1) / (4 * kQuadBlock)))
                 : grid_for(rows, 4, kMaxRedBlocks);
    for (int64_t c0 = 0; c0 < cols; c0 += kGemvMaxCols) {
        int nc = (int)((cols - c0) < kGemvMaxCols ? (cols - c0) : kGemvMaxCols);
        const int st = with_cols<kGemvMaxCols>(nc, [&](auto ncc) {
            if (quad)
                k_gemv_t_quad<T, decltype(ncc)::value><<<g, kQuadBlock, 0, ctx->stream>>>(rows, A + c0 * lda, lda, x,
                                                                                        ctx->red_ws);
            else
                k_gemv_t_nc<T, decltype(ncc)::value><<<g, kBlock, 0, ctx->stream>>>(rows, A + c0 * lda, lda, x,
                                                                                   ctx->red_ws);
            return (int)MPG_OK;
        });
        if (st) return st;
        MPG_LAUNCH_CHECK(ctx);
        k_gemv_t_stage2<T><<<1, 1024, 0, ctx->stream>>>(g, nc, ctx->red_ws, alpha, beta, y + c0);
        MPG_LAUNCH_CHECK(ctx);
    }
    return MPG_OK;
}

// gemv^T stage 1 alone (<= kGemvMaxCols columns): partials in the context
// workspace, *nparts of them per column, until the next reduction on ctx
template <class T>
int gemv_t_partials(mpg_ctx* ctx, int64_t rows, int64_t cols, const T* A, int64_t lda, const T* x, int32_t* nparts) {
    if (!ctx || !nparts || rows < 0 || cols < 1 || (rows > 0 && lda < rows)) return MPG_ERR_ARG;
    if (cols > kGemvMaxCols) return MPG_ERR_UNSUPPORTED;
    const bool quad = quad_aligned(A, lda, x, rows);
    const int g = quad ? (int)std::max<int64_t>(1, std::min<int64_t>(kQuadGroups, (rows + 4 * kQuadBlock - 1) /
                                                                                    (4 * kQuadBlock)))
                       : grid_for(rows, 4, kMaxRedBlocks);
    const int st = with_cols<kGemvMaxCols>((int)cols, [&](auto ncc) {
        if (quad)
            k_gemv_t_quad<T, decltype(ncc)::value><<<g, kQuadBlock, 0, ctx->stream>>>(rows, A, lda, x,
                                                                                    ctx->red_ws + kWsGemvSplit);
        else
            k_gemv_t_nc<T, decltype(ncc)::value><<<g, kBlock, 0, ctx->stream>>>(rows, A, lda, x,
                                                                               ctx->red_ws + kWsGemvSplit);
        return (int)MPG_OK;
    });
    if (st) return st;
    MPG_LAUNCH_CHECK(ctx);
    *nparts = g;
    return MPG_OK;
}

template <class T>
int gemv_t_finish(mpg_ctx* ctx, int32_t nparts, int64_t cols, T alpha, T beta, T* y) {
    if (!ctx || nparts < 1 || cols < 1 || cols > kGemvMaxCols) return MPG_ERR_ARG;
    k_gemv_t_stage2<T><<<1, 1024, 0, ctx->stream>>>(nparts, (int)cols, ctx->red_ws + kWsGemvSplit, alpha, beta, y);
    MPG_LAUNCH_CHECK(ctx);
    return MPG_OK;
}

// y = alpha*T(A x) + beta*y where x = alpha_t * T(pending gemv^T sums);
// MPG_ERR_UNSUPPORTED unless A, lda and y allow the quad form
template <class T>
int gemv_n_from_t(mpg_ctx* ctx, int64_t rows, int64_t cols, T alpha, const T* A, int64_t lda, int32_t nparts,
                  T alpha_t, T* x, T beta, T* y, int32_t* norm_nparts = nullptr, T* y_out = nullptr) {
    if (!ctx || rows < 0 || cols < 1 || nparts < 1 || (rows > 0 && lda < rows)) return MPG_ERR_ARG;
    if (y_out && (!norm_nparts || (y_out < y + rows && y < y_out + rows))) return MPG_ERR_ARG;
    if (cols > kGemvMaxCols || !quad_aligned(A, lda, y, rows) || (y_out && (uintptr_t)y_out % 16)) return MPG_ERR_UNSUPPORTED;
    if (norm_nparts && rows < 1) return MPG_ERR_UNSUPPORTED;
    const int g = quad_groups(rows);
    const int st = with_cols<kGemvMaxCols>((int)cols, [&](auto nc) {
        // the coefficients' partials sit apart from the ||y||^2 partials (kWsGemvSplit)
        if (norm_nparts)
            k_gemv_n_quad<T, decltype(nc)::value, true, true><<<g, kQuadBlock, 0, ctx->stream>>>(
                rows, alpha, A, lda, x, beta, y, ctx->red_ws + kWsGemvSplit, nparts, alpha_t, ctx->red_ws, y_out);
        else
            k_gemv_n_quad<T, decltype(nc)::value, true><<<g, kQuadBlock, 0, ctx->stream>>>(
                rows, alpha, A, lda, x, beta, y, ctx->red_ws + kWsGemvSplit, nparts, alpha_t);
        return (int)MPG_OK;
    });
    if (st) return st;
    MPG_LAUNCH_CHECK(ctx);
    if (norm_nparts) *norm_nparts = g;
    return MPG_OK;
}

// Triangular solve on one workgroup, x staged in LDS. Column-oriented
// (axpy) forms for the non-transposed solves, row-oriented (dot) forms for
// the transposed ones — the operation order of the reference BLAS xTRSV,
// with rounded products (no FMA contraction).
#pragma clang fp contract(off)
template <class T>
__global__ __launch_bounds__(kBlock) void k_trsv(int upper, int trans, int n, const T* __restrict__ A,
                                                 int64_t lda, T* __restrict__ x) {
    extern __shared__ unsigned char smem_raw[];
    T* xs = reinterpret_cast<T*>(smem_raw);
    for (int i = threadIdx.x; i < n; i += kBlock) xs[i] = x[i];
    __syncthreads();
    if (!trans) {
        for (int step = 0; step < n; ++step) {
            const int j = upper ? n - 1 - step : step;
            __shared__ T temp_s;
            if (threadIdx.x == 0) {
                T xj = xs[j];
                if (xj != T(0)) xj = xj / A[(int64_t)j * lda + j];
                xs[j] = xj;
                temp_s = xj;
            }
            __syncthreads();
            const T temp = temp_s;
            if (temp != T(0)) {
                if (upper) {
                    for (int i = threadIdx.x; i < j; i += kBlock) xs[i] = xs[i] - temp * A[(int64_t)j * lda + i];
                } else {
                    for (int i = j + 1 + threadIdx.x; i < n; i += kBlock) xs[i] = xs[i] - temp * A[(int64_t)j * lda + i];
                }
            }
            __syncthreads();
        }
    } else if (threadIdx.x == 0) {
        if (upper) {  // solve U^T x = b : forward
            for (int j = 0; j < n; ++j) {
                T temp = xs[j];
                for (int i = 0; i < j; ++i) temp = temp - A[(int64_t)j * lda + i] * xs[i];
                xs[j] = temp / A[(int64_t)j * lda + j];
            }
        } else {      // solve L^T x = b : backward
            for (int j = n - 1; j >= 0; --j) {
                T temp = xs[j];
                for (int i = n - 1; i > j; --i) temp = temp - A[(int64_t)j * lda + i] * xs[i];
                xs[j] = temp / A[(int64_t)j * lda + j];
            }
        }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < n; i += kBlock) x[i] = xs[i];
}

// lane j's value in every lane (j wave-uniform): scalar reads, no LDS
__device__ __forceinline__ float wave_bcast(float v, int j) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), j));
}
__device__ __forceinline__ double wave_bcast(double v, int j) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffffLL), j);
    const int hi = __builtin_amdgcn_readlane((int)(b >> 32), j);
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

// n <= 64 (the surface's y = H(0:k,0:k)^-1 s of a restart cycle): one wave,
// the matrix staged into LDS with all its loads in flight at once and lane i
// holding x(i), so a step waits on neither global memory nor a barrier (x(j)
// is broadcast by a shuffle). k_trsv waited for two dependent global loads
// per step: 21.7 us at n = 30 in the surface's restart section
// (profiles/r06_surface/r06o_cycle_timeline.txt). The same operations in the
// same order per element as k_trsv: the same bits (MPG_TRSV_WAVE=0: k_trsv).
template <class T, bool UPPER>
__global__ __launch_bounds__(kWave) void k_trsv_wave(int trans, int n, const T* __restrict__ A,
                                                     int64_t lda, T* __restrict__ x) {
    extern __shared__ unsigned char smem_raw[];
    T* As = reinterpret_cast<T*>(smem_raw);  // A(i, j) at As[j n + i]
    const int lane = threadIdx.x;
    // lane i loads row i of 32 columns at a time, every load of a batch
    // issued before any LDS store (clamped indices, masked stores): one
    // memory round trip per 32 columns
    constexpr int B = 32;
    const int ic = lane < n ? lane : n - 1;
    T xi = x[ic];
    for (int j0 = 0; j0 < n; j0 += B) {
        T r[B];
#pragma unroll
        for (int u = 0; u < B; ++u) r[u] = A[(int64_t)(j0 + u < n ? j0 + u : n - 1) * lda + ic];
#pragma unroll
        for (int u = 0; u < B; ++u)
            if (j0 + u < n && lane < n) As[(j0 + u) * n + lane] = r[u];
    }
    if (lane >= n) xi = T(0);
    __syncthreads();
    if (!trans) {
        // per step the chain is lane j's division, a scalar broadcast and
        // one product-difference; the column's LDS read is issued a step
        // ahead. Every lane divides its own entry by its own diagonal (only
        // lane j's quotient is used), so no step reads LDS for the diagonal.
        const T di = As[ic * n + ic];
        int j = UPPER ? n - 1 : 0;
        T aj = As[j * n + ic];
        for (int step = 0; step < n; ++step, j += UPPER ? -1 : 1) {
            const int jn = step + 1 < n ? (UPPER ? j - 1 : j + 1) : j;
            const T a = aj;
            aj = As[jn * n + ic];
            T q = xi;
            if (q != T(0)) q = q / di;
            const T xj = wave_bcast(q, j);
            if (lane == j) xi = xj;
            const bool mine = UPPER ? lane < j : (lane > j && lane < n);
            if (xj != T(0) && mine) xi = xi - xj * a;
        }
        if (lane < n) x[lane] = xi;
        return;
    }
    // the transposed forms are serial dot products (k_trsv's order), from LDS
    T* xs = As + n * n;
    if (lane < n) xs[lane] = xi;
    __syncthreads();
    if (lane == 0) {
        if (UPPER) {
            for (int j = 0; j < n; ++j) {
                T temp = xs[j];
                for (int i = 0; i < j; ++i) temp = temp - As[j * n + i] * xs[i];
                xs[j] = temp / As[j * n + j];
            }
        } else {
            for (int j = n - 1; j >= 0; --j) {
                T temp = xs[j];
                for (int i = n - 1; i > j; --i) temp = temp - As[j * n + i] * xs[i];
                xs[j] = temp / As[j * n + j];
            }
        }
    }
    __syncthreads();
    if (lane < n) x[lane] = xs[lane];
}
#pragma clang fp contract(on)

inline bool trsv_wave() {
    const char* e = std::getenv("MPG_TRSV_WAVE");
    return !(e && *e == '0');
}

template <class T>
int trsv_impl(mpg_ctx* ctx, int upper, int trans, int64_t n, const T* A, int64_t lda, T* x) {
    if (!ctx || n < 0 || n > 4096 || (n > 0 && lda < n)) return MPG_ERR_ARG;
    if (n == 0) return MPG_OK;
    if (n <= kWave && trsv_wave())
        (upper ? k_trsv_wave<T, true> : k_trsv_wave<T, false>)<<<1, kWave, (n * n + n) * sizeof(T), ctx->stream>>>(
            trans, (int)n, A, lda, x);
    else
        k_trsv<T><<<1, kBlock, n * sizeof(T), ctx->stream>>>(upper, trans, (int)n, A, lda, x);
    MPG_LAUNCH_CHECK(ctx);
    return MPG_OK;
}

}  // namespace

extern "C" {

int mpg_gemv_f64(mpg_ctx_t c, int trans, int64_t rows, int64_t cols, double alpha, const double* A,
                 int64_t lda, const double* x, double beta, double* y) {
    return gemv_impl<double>(c, trans, rows, cols, alpha, A, lda, x, beta, y);
}
int mpg_gemv_f32(mpg_ctx_t c, int trans, int64_t rows, int64_t cols, float alpha, const float* A,
                 int64_t lda, const float* x, float beta, float* y) {
    return gemv_impl<float>(c, trans, rows, cols, alpha, A, lda, x, beta, y);
}
int mpg_gemv_t_partials_f64(mpg_ctx_t c, int64_t rows, int64_t cols, const double* A, int64_t lda, const double* x,
                            int32_t* np) {
    return gemv_t_partials<double>(c, rows, cols, A, lda, x, np);
}
int mpg_gemv_t_partials_f32(mpg_ctx_t c, int64_t rows, int64_t cols, const float* A, int64_t lda, const float* x,
                            int32_t* np) {
    return gemv_t_partials<float>(c, rows, cols, A, lda, x, np);
}
int mpg_gemv_t_finish_f64(mpg_ctx_t c, int32_t np, int64_t cols, double alpha, double beta, double* y) {
    return gemv_t_finish<double>(c, np, cols, alpha, beta, y);
}
int mpg_gemv_t_finish_f32(mpg_ctx_t c, int32_t np, int64_t cols, float alpha, float beta, float* y) {
    return gemv_t_finish<float>(c, np, cols, alpha, beta, y);
}
int mpg_gemv_n_from_t_f64(mpg_ctx_t c, int64_t rows, int64_t cols, double alpha, const double* A, int64_t lda,
                          int32_t np, double alpha_t, double* x, double beta, double* y) {
    return gemv_n_from_t<double>(c, rows, cols, alpha, A, lda, np, alpha_t, x, beta, y);
}
int mpg_gemv_n_from_t_f32(mpg_ctx_t c, int64_t rows, int64_t cols, float alpha, const float* A, int64_t lda,
                          int32_t np, float alpha_t, float* x, float beta, float* y) {
    return gemv_n_from_t<float>(c, rows, cols, alpha, A, lda, np, alpha_t, x, beta, y);
}
int mpg_gemv_n_from_t_nrm2_f64(mpg_ctx_t c, int64_t rows, int64_t cols, double alpha, const double* A, int64_t lda,
                               int32_t np, double alpha_t, double* x, double beta, double* y, int32_t* norm_np) {
    if (!norm_np) return MPG_ERR_ARG;
    return gemv_n_from_t<double>(c, rows, cols, alpha, A, lda, np, alpha_t, x, beta, y, norm_np);
}
int mpg_gemv_n_from_t_nrm2_f32(mpg_ctx_t c, int64_t rows, int64_t cols, float alpha, const float* A, int64_t lda,
                               int32_t np, float alpha_t, float* x, float beta, float* y, int32_t* norm_np) {
    if (!norm_np) return MPG_ERR_ARG;
    return gemv_n_from_t<float>(c, rows, cols, alpha, A, lda, np, alpha_t, x, beta, y, norm_np);
}
int mpg_gemv_n_from_t_nrm2_out_f64(mpg_ctx_t c, int64_t rows, int64_t cols, double alpha, const double* A,
                                   int64_t lda, int32_t np, double alpha_t, double* x, double beta, const double* y,
                                   double* y_out, int32_t* norm_np) {
    if (!norm_np || !y_out) return MPG_ERR_ARG;
    return gemv_n_from_t<double>(c, rows, cols, alpha, A, lda, np, alpha_t, x, beta, const_cast<double*>(y), norm_np,
                                 y_out);
}
int mpg_gemv_n_from_t_nrm2_out_f32(mpg_ctx_t c, int64_t rows, int64_t cols, float alpha, const float* A,
                                   int64_t lda, int32_t np, float alpha_t, float* x, float beta, const float* y,
                                   float* y_out, int32_t* norm_np) {
    if (!norm_np || !y_out) return MPG_ERR_ARG;
    return gemv_n_from_t<float>(c, rows, cols, alpha, A, lda, np, alpha_t, x, beta, const_cast<float*>(y), norm_np,
                                y_out);
}
int mpg_trsv_f64(mpg_ctx_t c, int upper, int trans, int64_t n, const double* A, int64_t lda, double* x) {
    return trsv_impl<double>(c, upper, trans, n, A, lda, x);
}
int mpg_trsv_f32(mpg_ctx_t c, int upper, int trans, int64_t n, const float* A, int64_t lda, float* x) {
    return trsv_impl<float>(c, upper, trans, n, A, lda, x);
}

}  // extern "C"
