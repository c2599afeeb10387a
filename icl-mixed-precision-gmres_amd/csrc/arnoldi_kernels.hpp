// Kernels of the fused Arnoldi cycle (gfx950) and the plan object, shared by
// arnoldi.hip (the C-ABI, fp64 accumulation) and arnoldi_acc32.hip (the
// fp32-accumulation instantiations of the fp32-Arnoldi kernels).
//
//
// One restart cycle of GMRES(m) becomes a fixed program of phase kernels
// with no host round trip: the prologue (true residual + preconditioner +
// norms), per step an SpMV that normalises the previous vector on the fly
// and emits the Gram-Schmidt dot partials, the CGS/MGS update kernels that
// emit the next partials, a one-lane Givens kernel, and the solution update.
// Global sums are two-stage and deterministic (per-workgroup fp64 partials,
// then k_reduce_partials in a fixed order), which is also the seam where a
// multi-GPU caller all-reduces across ranks.
//
// Numerics follow the operator surface exactly where the reference fixes
// an order (reciprocal-then-multiply normalisation, y = alpha*t + beta*y
// forms, Givens on rounded products). Accumulation class (template parameter
// A of the dot/norm/gemv/SpMV kernels): A = double (default) sums fp32
// products in fp64 and rounds once to the working precision — the same
// rounding the stand-alone kernels (blas1/blas2/spmv) apply, so the fused
// engine and the operator-surface driver agree to the last bit in most
// steps; A = float (fp32 Arnoldi only, mpg_arnoldi_set_accum) keeps every
// partial sum in fp32, the class of the reference's cblas_sdot / snrm2 /
// sgemv and mkl_sparse_s_mv (kernels_mkl.cpp:82,94,104,284,348) and of
// cublasSdot / Sgemv / cusparseScsrmv (kernels_cuda.cpp:132,160,530,609).
#pragma once

#include "csr_tile.hpp"
#include "node_tile.hpp"
#include "sell_tile.hpp"
#include "handoff.hpp"
#include "panel.hpp"
#include "internal.hpp"
#include "mpgmres/arnoldi.h"

#include <cstdlib>
#include <new>
#include <algorithm>
#include <vector>

using namespace mpg;

namespace {

constexpr int kNC = 32;        // dot columns carried in registers per pass
constexpr int kGroups = 1024;  // max workgroups of the row-block phase kernels
constexpr int kCombineBlock = 1024;  // threads per workgroup of the combining panel dots
constexpr int kCombineGroups = 256;  // its workgroups: one per CU
constexpr int kOrthMGS = 1, kOrthCGSR = 2;  // mpg_orth_t (include/mpgmres/solve.h)

// Jacobi / identity preconditioner in precision P applied to a T value:
// typesafe_apply (gmres.cpp:12-22) + gdmv(1, d, w, 0, w) (kernels.hpp:141-144).
template <class T, class P>
__device__ __forceinline__ T precond(T w, const P* __restrict__ d, int64_t i) {
    P p = (P)w;
    if (d) p = P(0) * p + P(1) * d[i] * p;
    return (T)p;
}

// This workgroup's contiguous run of row blocks [rb0, rb1) — contiguous so
// that its rows form one range [blocks[rb0], blocks[rb1]) for the dot pass.
__device__ __forceinline__ void my_blocks(int nblocks, int& rb0, int& rb1, bool xcd = false) {
    const int b = xcd ? xcd_block((int)blockIdx.x, (int)gridDim.x) : (int)blockIdx.x;
    rb0 = (int)((int64_t)b * nblocks / gridDim.x);
    rb1 = (int)((int64_t)(b + 1) * nblocks / gridDim.x);
}

// For every row of this workgroup's row blocks: fp64 sum of val * xval(col)
// (csr_tile.hpp), then epi(row, sum) on one lane. NT: non-temporal matrix
// loads (a pass that runs once per restart cycle).
// XCD (round 5): workgroups take their runs of row blocks in XCD order
// (xcd_block), so each XCD's L2 holds the neighbourhood of x that its own
// contiguous eighth of the rows gathers (the SELL kernels' placement).
template <bool NT = false, bool XCD = false, class A = double, class V, class XF, class PF, class EPI>
__device__ __forceinline__ void for_rows(const int32_t* __restrict__ blocks, int nblocks,
                                         const int32_t* __restrict__ rowptr, const int32_t* __restrict__ col,
                                         const V* __restrict__ val, int64_t nnz, XF xval, PF pre, EPI epi,
                                         double* prod, double* scratch) {
    const int32_t* __restrict__ bnnz = blocks + nblocks + 1;  // mpg_csr's nnz starts follow the row starts
    int rb0, rb1;
    my_blocks(nblocks, rb0, rb1, XCD);
    for (int b = rb0; b < rb1; ++b)
        csr_row_block<NT, A>(blocks[b], blocks[b + 1], bnnz[b], bnnz[b + 1], rowptr, col, val, nnz, xval, pre, epi,
                             prod, scratch);
}

// Combine in the last arriver: sums[c] = sum over g of partial[c*G + g] for
// c < ncols <= BS/32; 32 lanes per column, each a strided run in g order,
// then a 32-lane xor tree (fixed order).
template <int BS, class A = double>
__device__ __forceinline__ void combine_columns(const double* __restrict__ partial, int G, int ncols,
                                                double* __restrict__ sums) {
    const int c = threadIdx.x / 32, sub = threadIdx.x % 32;
    A v = A(0);
    if (c < ncols)
        for (int g = sub; g < G; g += 32) v += (A)partial[(size_t)c * G + g];
#pragma unroll
    for (int mask = 16; mask >= 1; mask >>= 1) v += __shfl_xor(v, mask, kWave);
    if (c < ncols && sub == 0) sums[c] = (double)v;
}

// ---------------------------------------------------------------- prologue
// r = b - A x (X), w = M(T(r)); partials: ||T(r)||^2, ||w||^2, ||x||^2
template <class T, class X, class P>
__global__ __launch_bounds__(kBlock) void k_prologue(const int32_t* __restrict__ blocks, int nblocks,
                                                     const int32_t* __restrict__ rowptr,
                                                     const int32_t* __restrict__ col, const X* __restrict__ val,
                                                     int64_t nnz, const X* __restrict__ x, const X* __restrict__ b,
                                                     const P* __restrict__ diag, T* __restrict__ w,
                                                     double* __restrict__ partial) {
    __shared__ double prod[kNnzCap];
    __shared__ double scratch[kBlock / kWave];
    double acc[4] = {0.0, 0.0, 0.0, 0.0};
    struct Ops {
        X b, x;
        P d;
    };
    for_rows<true>(  // once per cycle: keep V and the Arnoldi matrix cached
        blocks, nblocks, rowptr, col, val, nnz, [&](int c) { return (double)x[c]; },
        [&](int i) { return Ops{b[i], x[i], diag ? diag[i] : P(0)}; },
        [&](int i, double sum, const Ops& o) {
            const X bi = o.b, xi = o.x;
            const P di = o.d;
            const X t = (X)sum;
            const X r = bi - t;  // copy(b, w); spmv(-1, A, x, 1, w)
            T wi = (T)r;
            acc[0] += (double)wi * (double)wi;
            P pw = (P)wi;  // = precond<T, P> (typesafe_apply's rounding to P included)
            if (diag) pw = P(0) * pw + P(1) * di * pw;
            wi = (T)pw;
            acc[1] += (double)wi * (double)wi;
            acc[2] += (double)xi * (double)xi;
            w[i] = wi;
        },
        prod, scratch);
    store_partials<4>(acc, 3, partial);
}

// The residual prologue on node blocks (round 6), in two launches whose
// arithmetic is k_prologue's: k_node_rowsums forms every row's fp64 sum of
// A x on the node copy of the outer values (the CSR tile's products in CSR
// storage order, node_tile.hpp), then k_prologue_rows runs k_prologue's
// epilogue on those sums with k_prologue's grid, row blocks and lane-to-row
// map (for_rows / csr_row_block: lane t takes rows r0 + t, r0 + t + 256, ...
// of each of its workgroup's blocks), so every lane's three norm partials
// add the same terms in the same order and the cycle keeps the CSR bits.
// (A single row past kNnzCap, csr_row_block's tree-summed row mode, cannot
// occur: a node row holds at most kNodeCap blocks.) fem27 / C4: 8.9 B per
// nonzero of fp64 records against CSR's 12.
template <class X>
__global__ __launch_bounds__(kBlock) void k_node_rowsums(const int32_t* __restrict__ tiles,
                                                         const int32_t* __restrict__ bptr,
                                                         const char* __restrict__ recs, int ntiles, int64_t nblk,
                                                         int tpw, int xcd, const X* __restrict__ x,
                                                         double* __restrict__ rsum) {
    __shared__ double prod[kNodeProd];
    const int g = xcd ? xcd_block((int)blockIdx.x, (int)gridDim.x) : (int)blockIdx.x;
    const int t0 = g * tpw, t1 = t0 + tpw < ntiles ? t0 + tpw : ntiles;
    node_tiles<X>(
        t0, t1, tiles, tiles + ntiles + 1, bptr, recs, nblk, [&](int c) { return x[c]; },
        [&](X v) { return (double)v; }, [&](int) { return 0; }, [&](int i, double sum, int) { rsum[i] = sum; },
        prod);
}

template <class T, class X, class P>
__global__ __launch_bounds__(kBlock) void k_prologue_rows(const int32_t* __restrict__ blocks, int nblocks,
                                                          const double* __restrict__ rsum,
                                                          const X* __restrict__ x, const X* __restrict__ b,
                                                          const P* __restrict__ diag, T* __restrict__ w,
                                                          double* __restrict__ partial) {
    double acc[4] = {0.0, 0.0, 0.0, 0.0};
    auto epi = [&](int i) {  // k_prologue's epilogue, on the same sum
        const X t = (X)rsum[i];
        const X r = b[i] - t;
        T wi = (T)r;
        acc[0] += (double)wi * (double)wi;
        P pw = (P)wi;
        if (diag) pw = P(0) * pw + P(1) * diag[i] * pw;
        wi = (T)pw;
        acc[1] += (double)wi * (double)wi;
        acc[2] += (double)x[i] * (double)x[i];
        w[i] = wi;
    };
    int rb0, rb1;
    my_blocks(nblocks, rb0, rb1);
    for (int bk = rb0; bk < rb1; ++bk) {
        const int r0 = blocks[bk], r1 = blocks[bk + 1];
        for (int r = threadIdx.x; r < r1 - r0; r += kBlock) epi(r0 + r);
    }
    store_partials<4>(acc, 3, partial);
}

// The same prologue on a SELL-64 copy of the outer-precision values (one
// wave per slice, one lane per row; loads issued in need order as in
// k_step_sell): r = b - A x (X), w = M(T(r)), partials ||T(r)||^2,
// ||w||^2, ||x||^2 per workgroup.
template <class T, class X, class P, class CI, int W, bool WIN, bool UNI = false>
__global__ __launch_bounds__(kBlock) void k_prologue_sell(int n, int n_lo, int n_ext, int nslices, const int64_t* __restrict__ off,
                                                          const CI* __restrict__ col, const X* __restrict__ val,
                                                          const X* __restrict__ x, const X* __restrict__ b,
                                                          const P* __restrict__ diag, T* __restrict__ w,
                                                          double* __restrict__ partial,
                                                          const int32_t* __restrict__ sbase,
                                                          const int32_t* __restrict__ spat, const int64_t* __restrict__ coff, const CI* __restrict__ pat,
                                                          const int32_t* __restrict__ xrp,
                                                          const int32_t* __restrict__ xcol,
                                                          const X* __restrict__ xval, int64_t ustride, int xcd,
                                                          const int32_t* __restrict__ rows) {
    constexpr int NQ = kWinLen / kWave;
    __shared__ X win[WIN ? kBlock / kWave : 1][WIN ? kWinLen : 1];
    const int lane = threadIdx.x & (kWave - 1), wid = wave_id();
    const int s = (xcd ? xcd_block(blockIdx.x, gridDim.x) : (int)blockIdx.x) * (kBlock / kWave) + wid;
    const bool live = s < nslices;  // a dead wave still joins the partials' barrier
    const int row0 = s * kWave;
    // the lane's row (a sorted SELL-C-sigma copy: rows[], padding lanes n)
    const int i = rows ? rows[live ? row0 + lane : 0] : row0 + lane;
    const bool own = live && i < n;
    SellRow<X, CI, W, true> row;  // once per cycle: non-temporal slices
    if constexpr (UNI) row.init_uniform(live ? s : 0, ustride, spat, coff);
    else row.init_load(live ? s : 0, off, spat, coff);
    __builtin_amdgcn_sched_barrier(0);
    X xr[WIN ? NQ : 1];
    if constexpr (WIN) {
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            const int c = row0 - kWinLo + q * kWave + lane;
            xr[q] = x[c >= n_lo && c < n_ext ? c : 0];
        }
    }
    const int ic = own ? i : 0;
    const X bi = b[ic], xi = x[ic];
    const P di = diag ? diag[ic] : P(0);
    __builtin_amdgcn_sched_barrier(0);
    row.init_finish(lane, col, val, sbase, pat);
    row.load(0);
    __builtin_amdgcn_sched_barrier(0);
    double sum = 0.0;
    if (live) {
        if constexpr (WIN) {
#pragma unroll
            for (int q = 0; q < NQ; ++q) {
                const int c = row0 - kWinLo + q * kWave + lane;
                win[wid][q * kWave + lane] = (c >= n_lo && c < n_ext) ? xr[q] : X(0);
            }
            wave_lds_sync();
            auto xv = [&](int c) { return (double)win[wid][c - row0 + kWinLo]; };
            row.sum(0, xv, sum);
            for (int q = row.U; q < row.steps; q += row.U) {
                row.load(q);
                row.sum(q, xv, sum);
            }
        } else {
            auto xv = [&](int c) { return (double)x[c]; };
            if (SellCol<CI>::stepped && row.exc) {
                sum = csr_row_sum(own ? row.xrow : -1, xrp, xcol, xval, xv);
            } else {
                row.sum(0, xv, sum);
                for (int q = row.U; q < row.steps; q += row.U) {
                    row.load(q);
                    row.sum(q, xv, sum);
                }
            }
        }
    }
    double acc[4] = {0.0, 0.0, 0.0, 0.0};
    if (own) {
        const X t = (X)sum;
        const X r = bi - t;  // copy(b, w); spmv(-1, A, x, 1, w)
        T wi = (T)r;
        acc[0] = (double)wi * (double)wi;
        P pw = (P)wi;  // = precond<T, P>
        if (diag) pw = P(0) * pw + P(1) * di * pw;
        wi = (T)pw;
        acc[1] = (double)wi * (double)wi;
        acc[2] = (double)xi * (double)xi;
        w[i] = wi;
    }
    store_partials<4>(acc, 3, partial);
}

template <class T, class X>
__global__ void k_prologue_finish(const double* __restrict__ sums, int m, T* __restrict__ s, T* __restrict__ inv,
                                  double* __restrict__ report) {
    const T r_norm = (T)sqrt(sums[0]);
    const T beta = (T)sqrt(sums[1]);
    const X x_norm = (X)sqrt(sums[2]);
    const T iv = beta != T(0) ? T(1) / beta : T(0);  // first_vector: zero fill when beta == 0
    if (threadIdx.x == 0) {
        report[0] = (double)r_norm;
        report[1] = (double)beta;
        report[2] = (double)x_norm;
        report[3] = (double)iv;
        *inv = iv;
    }
    for (int i = threadIdx.x; i <= m; i += blockDim.x) s[i] = i == 0 ? beta : T(0);
}

// ||w||^2 partials again (column 1 of the prologue's partials, same grid)
// after a preconditioner applied outside the prologue kernel (ILU)
template <class T>
__global__ __launch_bounds__(kBlock) void k_wnorm_partials(int n, const T* __restrict__ w, double* __restrict__ partial) {
    double acc[1] = {0.0};
    for (int i = blockIdx.x * kBlock + threadIdx.x; i < n; i += gridDim.x * kBlock) acc[0] += (double)w[i] * (double)w[i];
    store_partials<1>(acc, 1, partial + gridDim.x);
}

// ---------------------------------------------------------------- reductions
// sum of G partials in a fixed order (identical in every workgroup that
// calls it with the same G); result valid in thread 0. A: the accumulation
// class (fp32: the partials are fp32 values, every add rounds to fp32)
template <int BS, class A = double>
__device__ __forceinline__ A sum_partials(const double* __restrict__ p, int G, A* scratch) {
    A v0 = A(0), v1 = A(0);
    int g = threadIdx.x;
    for (; g + BS < G; g += 2 * BS) {
        v0 += (A)p[g];
        v1 += (A)p[g + BS];
    }
    if (g < G) v0 += (A)p[g];
    return block_sum<BS>(v0 + v1, scratch);
}

template <int BS, class A = double>
__global__ __launch_bounds__(BS) void k_reduce_partials(int G, const double* __restrict__ partial,
                                                        double* __restrict__ sums) {
    __shared__ A scratch[BS / kWave];
    const A s = sum_partials<BS, A>(partial + (size_t)blockIdx.x * G, G, scratch);
    if (threadIdx.x == 0) sums[blockIdx.x] = (double)s;
}

// k_reduce_partials of the prologue's 3 columns + k_prologue_finish in one
// workgroup (one GPU: nothing to all-reduce between them): each column is
// summed by sum_partials<BS>, as its k_reduce_partials workgroup would, so
// the sums and everything formed from them have the same bits
template <class T, class X, int BS>
__global__ __launch_bounds__(BS) void k_prologue_finish_parts(int G, const double* __restrict__ partial,
                                                              double* __restrict__ sums, int m, T* __restrict__ s,
                                                              T* __restrict__ inv, double* __restrict__ report) {
    __shared__ double scratch[BS / kWave];
    __shared__ double sm[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        const double v = sum_partials<BS>(partial + (size_t)c * G, G, scratch);
        if (threadIdx.x == 0) {
            sm[c] = v;
            sums[c] = v;
        }
    }
    __syncthreads();
    const T r_norm = (T)sqrt(sm[0]);
    const T beta = (T)sqrt(sm[1]);
    const X x_norm = (X)sqrt(sm[2]);
    const T iv = beta != T(0) ? T(1) / beta : T(0);  // first_vector: zero fill when beta == 0
    if (threadIdx.x == 0) {
        report[0] = (double)r_norm;
        report[1] = (double)beta;
        report[2] = (double)x_norm;
        report[3] = (double)iv;
        *inv = iv;
    }
    for (int i = threadIdx.x; i <= m; i += blockDim.x) s[i] = i == 0 ? beta : T(0);
}

// ---------------------------------------------------------------- step: Givens
#pragma clang fp contract(off)
template <class T>
__device__ void rot_pair(T& a, T& b, T c, T s) {
    const T a1 = a, a2 = b;
    a = c * a1 + s * a2;
    b = c * a2 - s * a1;
}
template <class T>
__device__ void rotg_ref(T& a, T& b, T& c, T& s) {
    const T av = a, bv = b;
    const T roe = fabs(av) > fabs(bv) ? av : bv;
    const T scale = fabs(av) + fabs(bv);
    T r;
    if (scale == T(0)) {
        c = T(1); s = T(0); r = T(0);
    } else {
        const T as = av / scale, bs = bv / scale;
        r = scale * sqrt(as * as + bs * bs);
        r = roe >= T(0) ? r : -r;
        c = av / r;
        s = bv / r;
    }
    a = r;
    b = T(0);
}

// h_{k+1,k} = ||w||; (CGSR: h(0:k,k) += correction); rotations; |s(k+1)|.
// norm2 = the squared norm: sums[0] (nparts == 0) or, on one GPU, the sum
// of `nparts` workgroup partials reduced here (saves a launch per step).
// Givens step k on one workgroup (gmres.cpp:217-226): col/c_s/s_s are LDS
// arrays of at least k + 2 entries; nrm2sq (= ||w||^2) is read in thread 0.
template <class T>
struct GivensArgs {
    int k, m;
    const T* corr;  // CGSR correction (h += corr) or nullptr
    T *H, *cs, *sn, *s, *inv;
    double* report;
};

template <class T>
__device__ void givens_block(const GivensArgs<T>& g, double nrm2sq, T* col, T* c_s, T* s_s) {
    // stage the column and the previous rotations in LDS with all lanes, so
    // the serial rotation chain runs on LDS instead of global latency
    const int k = g.k;
    T* gcol = g.H + (int64_t)k * (g.m + 1);
    for (int j = threadIdx.x; j <= k; j += blockDim.x) {
        col[j] = g.corr ? gcol[j] + T(1) * g.corr[j] : gcol[j];  // axpy(1.0, weights, h_col)
        c_s[j] = g.cs[j];
        s_s[j] = g.sn[j];
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        const T hn = (T)sqrt(nrm2sq);
        col[k + 1] = hn;
        *g.inv = T(1) / hn;  // scal(1/h_final, w, v_{k+1}) — no breakdown guard, as in the reference
        for (int j = 0; j < k; ++j) rot_pair(col[j], col[j + 1], c_s[j], s_s[j]);
        rotg_ref(col[k], col[k + 1], c_s[k], s_s[k]);
        T sk = g.s[k], sk1 = g.s[k + 1];
        rot_pair(sk, sk1, c_s[k], s_s[k]);
        g.s[k] = sk;
        g.s[k + 1] = sk1;
        g.cs[k] = c_s[k];
        g.sn[k] = s_s[k];
        g.report[4 + k] = (double)fabs(sk1);
    }
    __syncthreads();
    for (int j = threadIdx.x; j <= k + 1; j += blockDim.x) gcol[j] = col[j];
}

// the scale 1/h_{k+1,k} exactly as givens_block forms it
template <class T>
__device__ __forceinline__ T inv_of_norm2(double nrm2sq) {
    return T(1) / (T)sqrt(nrm2sq);
}

// norm2 = the squared norm: sums[0] (nparts == 0) or, on one GPU, the sum
// of `nparts` workgroup partials reduced here (saves a launch per step).
template <class T, class A = double>
__global__ __launch_bounds__(kBlock) void k_givens(GivensArgs<T> g, const double* __restrict__ norm2, int nparts) {
    __shared__ T col[1026], c_s[1026], s_s[1026];
    __shared__ A scratch[kBlock / kWave];
    const double nrm2sq = nparts > 0 ? (double)sum_partials<kBlock, A>(norm2, nparts, scratch) : norm2[0];
    givens_block(g, nrm2sq, col, c_s, s_s);
}

// Givens step k-1 folded into the SpMV launch of step k (restart length
// <= kFoldMaxM): every workgroup sums the ||w||^2 partials in the same
// fixed order and forms 1/h_{k,k-1} itself; workgroup 0 also runs the
// rotation step. Returns the scale for v_k in every thread.
constexpr int kFoldMaxM = 128;  // GMRES(100), the reference's published restart length
template <class T>
struct GivensFold {
    const double* norm2;  // nullptr: not folded (use *inv_p)
    int nparts;
    GivensArgs<T> g;
};

// measurement only (mpg_arnoldi_stamp_next): wave q's lane 0 stores the
// wall clock to stamp[2q + end] (end 0 at the wave's start, 1 at its end); a
// one-dimensional grid. Used by the one-panel dots and CGS update only: in
// the SpMVs, whose occupancy sits on VGPR thresholds, even this uniform
// branch cost up to 20 VGPRs (C4's stepped kernel 71 -> 91, -11 % in time),
// and a branch-free form with a sink word slowed the BAND SpMV; the SpMV is
// timed by duplicate launches instead (time_phase_dup, host/fused_gmres.cpp).
// Round 5: a compile-time choice. The product instantiations
// (STAMP = false) hold no stamp code at all; the launch sites pick the STAMP
// = true instantiation only for a launch that mpg_arnoldi_stamp_next armed.
template <bool STAMP>
__device__ __forceinline__ void stamp_at(unsigned long long* stamp, int end) {
    if constexpr (STAMP) {
        if ((threadIdx.x & (kWave - 1)) == 0)
            stamp[2 * (((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / kWave) + end] = wall_clock64();
    }
}

template <bool FOLD, class T, class A = double>
__device__ __forceinline__ T fold_givens(const GivensFold<T>& f, const T* __restrict__ inv_p) {
    if constexpr (!FOLD) {
        return *inv_p;
    } else {
        __shared__ T col[kFoldMaxM + 2], c_s[kFoldMaxM + 2], s_s[kFoldMaxM + 2];
        __shared__ A scratch[kBlock / kWave];
        __shared__ T inv_s;
        const double nrm2sq = f.nparts > 0 ? (double)sum_partials<kBlock, A>(f.norm2, f.nparts, scratch) : f.norm2[0];
        if (threadIdx.x == 0) inv_s = inv_of_norm2<T>(nrm2sq);
        if (blockIdx.x == 0) givens_block(f.g, nrm2sq, col, c_s, s_s);
        __syncthreads();
        return inv_s;
    }
}
#pragma clang fp contract(on)

// ---------------------------------------------------------------- step: SpMV
// v_k = T(w_prev * inv) (local rows stored to V[:,k]); w = M(A v_k).
// inv = 1/h_{k,k-1} from the previous Givens kernel, or formed here with
// that Givens step folded in (fold.norm2 != nullptr). The Gram-Schmidt dots
// follow in k_panel_dots (measured: dots inside this gather-bound launch
// cost more than the separate pass, 71 us vs 30 + 20 us on BAND-10M).
template <class T, class P, class VI, bool FOLD, int MODE = 0, class A = double>
__global__ __launch_bounds__(kBlock) void k_step_spmv(const int32_t* __restrict__ blocks, int nblocks,
                                                      const int32_t* __restrict__ rowptr,
                                                      const int32_t* __restrict__ col, const VI* __restrict__ val,
                                                      int64_t nnz, const T* __restrict__ wprev,
                                                      const T* __restrict__ inv_p, T* __restrict__ V, int64_t ld,
                                                      int k, const P* __restrict__ diag, T* __restrict__ w,
                                                      GivensFold<T> fold, const int8_t* __restrict__ rexp) {
    __shared__ double prod[kNnzCap];
    __shared__ double scratch[kBlock / kWave];
    const T inv = fold_givens<FOLD, T, A>(fold, inv_p);
    T* __restrict__ Vk = V + (int64_t)k * ld;
    struct Ops {
        T wp;
        P d;
        int e;  // row exponent of a scaled fp16 copy (mpg_csr_half_values)
    };
    // MODE bit 0: non-temporal matrix streams; bit 1: XCD-ordered row blocks;
    // bit 2 (measurement only, wrong results): no gathers, x = 1
    for_rows<(MODE & 1) != 0, (MODE & 2) != 0, A>(
        blocks, nblocks, rowptr, col, val, nnz,
        [&](int c) { return (MODE & 4) ? 1.0 + 0.0 * c : (double)(T)(wprev[c] * inv); },
        [&](int i) { return Ops{wprev[i], diag ? diag[i] : P(0), rexp ? (int)rexp[i] : 0}; },
        [&](int i, double sum, const Ops& o) {
            const T t = (T)ldexp(sum, -o.e);  // spmv(1, A, v, 0, w): y = 1*t (exact unscale)
            P pw = (P)t;         // = precond<T, P> with the diagonal loaded ahead
            if (diag) pw = P(0) * pw + P(1) * o.d * pw;
            w[i] = (T)pw;
            Vk[i] = o.wp * inv;
        },
        prod, scratch);
}

// ---------------------------------------------------------------- step: SpMV (node blocks)
// Same contract as k_step_spmv on the node-block copy (node_tile.hpp): one
// tile of node rows per workgroup, the CSR tile's products and row order.
// WALK: each workgroup walks tpw consecutive tiles, the next tile's records
// in flight during this one's gathers and row sums (node_tiles); else one
// tile per workgroup (node_tile).
template <class T, class P, class VI, bool FOLD, bool WALK = true, class A = double>
__global__ __launch_bounds__(kBlock) void k_step_node(const int32_t* __restrict__ tiles,
                                                      const int32_t* __restrict__ bptr, const char* __restrict__ recs,
                                                      const T* __restrict__ wprev, const T* __restrict__ inv_p,
                                                      T* __restrict__ V, int64_t ld, int k,
                                                      const P* __restrict__ diag, T* __restrict__ w,
                                                      GivensFold<T> fold, const int8_t* __restrict__ rexp,
                                                      int ntiles, int64_t nblk, int tpw, int xcd) {
    __shared__ double prod[kNodeProd];
    const T inv = fold_givens<FOLD, T, A>(fold, inv_p);
    T* __restrict__ Vk = V + (int64_t)k * ld;
    struct Ops {
        T wp;
        P d;
        int e;
    };
    auto xraw = [&](int c) { return wprev[c]; };
    auto xfin = [&](T v) { return (double)(T)(v * inv); };
    auto xval = [&](int c) { return xfin(xraw(c)); };
    auto pre = [&](int i) { return Ops{wprev[i], diag ? diag[i] : P(0), rexp ? (int)rexp[i] : 0}; };
    auto epi = [&](int i, double sum, const Ops& o) {
        const T t = (T)ldexp(sum, -o.e);
        P pw = (P)t;
        if (diag) pw = P(0) * pw + P(1) * o.d * pw;
        w[i] = (T)pw;
        Vk[i] = o.wp * inv;
    };
    // xcd: workgroups take their tiles in XCD order (xcd_block), so each
    // XCD's L2 serves one contiguous eighth of the rows' gathers
    const int g = xcd ? xcd_block((int)blockIdx.x, (int)gridDim.x) : (int)blockIdx.x;
    if constexpr (!WALK) {
        node_tile<VI, A>(g, tiles, bptr, recs, xval, pre, epi, prod);
    } else {
        const int t0 = g * tpw, t1 = t0 + tpw < ntiles ? t0 + tpw : ntiles;
        node_tiles<VI, A>(t0, t1, tiles, tiles + ntiles + 1, bptr, recs, nblk, xraw, xfin, pre, epi, prod);
    }
}

// ---------------------------------------------------------------- step: SpMV (SELL-64)
// Same contract as k_step_spmv on the sliced-ELL copy (sell_tile.hpp): one
// wave per slice, one lane per row; v_k and w are written coalesced.
// WIN (every column of a slice within [row0 - kWinLo, row0 + 64 + kWinHi),
// checked when the copy is built): the slice's window of v_k is formed once
// in LDS with three coalesced loads per lane and the gathers read LDS —
// 10 scattered global loads per row become LDS reads (-20 % on BAND-10M,
// tools/sell_bench.hip). Values are the same T(w_prev * inv) either way.

//
// Load order (vmcnt retires in order, so what is needed first is issued
// first, and nothing is waited for before everything is in flight): the
// slice's offsets, the folded Givens step's partial (one per lane), the
// window of w_prev (raw,
// clamped addresses), the slice's first batch of (col, val); then the
// partial sum behind LDS-only barriers, the scaled window into LDS, the
// gathers. A guarded load would be widened inside its branch and waited
// for right there — the previous form waited for each window load and each
// step's loads in turn.
// DN > 0 (one GPU, CGS, k + 1 <= DN): the panel dots <v_j, w> for j <= k
// are formed here too, from the lane's own w(i) (no re-read of w and no dots
// launch). Each workgroup block-reduces its products (store_partials); the
// last arriver of each group of `gs` workgroups sums the group's partials
// in workgroup order, so the CGS update (FROM_PARTS) sees <= 256 partials
// per column, as from k_dots_nc. Deterministic: fixed order throughout.
struct SellDots {
    int nc;            // columns: k + 1
    int gs, ng;        // workgroups per group, groups (<= kCombineGroups)
    double* wgpart;    // [c * gridDim.x + blockIdx.x]
    unsigned* cnt;     // one ticket per group (zero between launches)
    double* out;       // [c * ng + g]
};

template <class T, class P, class VI, class CI, int W, bool WIN, bool FOLD, int DN = 0, int BS = kBlock,
          bool UNI = false, bool PIPE = false, class A = double>
__global__ __launch_bounds__(BS) void k_step_sell(int n, int n_lo, int n_ext, int nslices, const int64_t* __restrict__ off,
                                                      const CI* __restrict__ col,
                                                      const typename SellStore<VI>::type* __restrict__ val,
                                                      const T* __restrict__ wprev, const T* __restrict__ inv_p,
                                                      T* __restrict__ V, int64_t ld, int k,
                                                      const P* __restrict__ diag, T* __restrict__ w,
                                                      GivensFold<T> fold, SellDots dd,
                                                      const int32_t* __restrict__ sbase,
                                                      const int32_t* __restrict__ spat, const int64_t* __restrict__ coff, const CI* __restrict__ pat,
                                                      const int32_t* __restrict__ xrp,
                                                      const int32_t* __restrict__ xcol,
                                                      const typename SellStore<VI>::type* __restrict__ xval,
                                                      const int8_t* __restrict__ rexp, int64_t ustride, int xcd,
                                                      const int32_t* __restrict__ rows) {
    static_assert(DN == 0 || BS == kBlock, "the fused dots' partials assume kBlock-thread workgroups");
    static_assert(DN == 0 || std::is_same_v<A, double>, "the fused dots accumulate in fp64");
    using S = typename SellStore<VI>::type;
    constexpr int NQ = kWinLen / kWave;
    __shared__ T win[WIN ? BS / kWave : 1][WIN ? kWinLen : 1];
    const int lane = threadIdx.x & (kWave - 1), wid = wave_id();
    const int s = (xcd ? xcd_block(blockIdx.x, gridDim.x) : (int)blockIdx.x) * (BS / kWave) + wid;
    const bool live = s < nslices;  // a dead wave still joins the fold's barriers
    const int row0 = s * kWave;
    // the lane's row: row0 + lane, or a sorted (SELL-C-sigma) copy's rows[],
    // loaded behind the slice's first batch (below); nothing before needs it
    int i = row0 + lane;
    // 0. the slice's offsets (UNI: computed) and pattern index
    SellRow<S, CI, W> row;
    if constexpr (UNI) row.init_uniform(live ? s : 0, ustride, spat, coff);
    else row.init_load(live ? s : 0, off, spat, coff);
    __builtin_amdgcn_sched_barrier(0);
    // 1. the fold's ||w||^2 partial (nparts <= kBlock, checked at launch: one per lane)
    // (a workgroup narrower than kBlock loads kBlock / BS per lane: the
    // partials keep their kBlock-lane positions, so the sums below run in
    // the same order whatever BS is)
    constexpr int NPL = BS < kBlock ? kBlock / BS : 1;
    A part[NPL];
#pragma unroll
    for (int j = 0; j < NPL; ++j) part[j] = A(0);
    if constexpr (FOLD) {
#pragma unroll
        for (int j = 0; j < NPL; ++j) {
            const int t = j * BS + (int)threadIdx.x;
            part[j] = (A)fold.norm2[t < fold.nparts ? t : 0];
            if (t >= fold.nparts) part[j] = A(0);
        }
    }
    __builtin_amdgcn_sched_barrier(0);
    // 2. w_prev window (or this row's own w_prev), raw
    T wr[WIN ? NQ : 1];
    if constexpr (WIN) {
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            const int c = row0 - kWinLo + q * kWave + lane;
            wr[q] = wprev[c >= n_lo && c < n_ext ? c : 0];
        }
    } else {
        if (!rows) wr[0] = wprev[i < n ? i : 0];  // the round-3 order (unsorted copies)
    }
    __builtin_amdgcn_sched_barrier(0);
    // 3. the slice's first batch (UNI: the values before the pattern index
    // is waited for, then the columns)
    if constexpr (UNI) {
        row.init_vals(lane, val);
        row.load_vals(0);
        __builtin_amdgcn_sched_barrier(0);
        row.init_finish(lane, col, val, sbase, pat);
        row.load_cols(0);
    } else {
        row.init_finish(lane, col, val, sbase, pat);
        row.load(0);
    }
    __builtin_amdgcn_sched_barrier(0);
    // 3b. without the window, sorted (SELL-C-sigma) copies: the lane's row and
    // its own w_prev, behind the first batch (needed last)
    if constexpr (!WIN) {
        if (rows) {
            i = rows[live ? row0 + lane : 0];
            wr[0] = wprev[i < n ? i : 0];
        }
    }
    // 4. a scaled fp16 copy's row exponent (needed last, issued last)
    int rex = 0;
    if constexpr (std::is_same_v<VI, half_v>) {
        if (rexp) rex = rexp[live && i < n ? i : 0];
    }
    __builtin_amdgcn_sched_barrier(0);
    // the scale 1/h_{k,k-1}: the folded Givens step, or the Givens kernel's
    T inv;
    // the folded step's ||w||^2; workgroup 0 runs the rotation step with it
    // after its own rows (nothing in this launch reads what the rotation
    // writes, and its serial chain then holds none of the slice's loads live)
    double nrm2sq = 0.0;
    if constexpr (FOLD) {
        constexpr int NG = (BS < kBlock ? kBlock : BS) / kWave;
        __shared__ A scratch[NG];
        __shared__ T inv_s;
        if (fold.nparts > 0) {
#pragma unroll
            for (int j = 0; j < NPL; ++j) {
                const A v = wave_sum(part[j] + A(0));  // the same fixed order in every workgroup
                if (lane == 0) scratch[j * (BS / kWave) + wid] = v;
            }
            lds_barrier();
            A r = A(0);
#pragma unroll
            for (int q = 0; q < NG; ++q) r += scratch[q];
            nrm2sq = (double)r;
        } else {
            nrm2sq = fold.norm2[0];
        }
        if (threadIdx.x == 0) inv_s = inv_of_norm2<T>(nrm2sq);
        lds_barrier();
        inv = inv_s;
    } else {
        inv = *inv_p;
    }
    // with dots, a dead wave joins the partials' barriers; with the fold,
    // workgroup 0's waves all join the rotation step's barriers at the end
    if (DN == 0 && !live && !(FOLD && blockIdx.x == 0)) return;
    A sum = A(0);
    T vk = T(0);  // v_k(i) = T(w_prev(i) * inv)
    if (live) {
        if constexpr (WIN) {
#pragma unroll
            for (int q = 0; q < NQ; ++q) {
                const int c = row0 - kWinLo + q * kWave + lane;
                win[wid][q * kWave + lane] = (c >= n_lo && c < n_ext) ? (T)(wr[q] * inv) : T(0);
            }
            wave_lds_sync();
            auto xv = [&](int c) { return (double)win[wid][c - row0 + kWinLo]; };
            row.sum(0, xv, sum);
            for (int q = row.U; q < row.steps; q += row.U) {
                row.load(q);
                row.sum(q, xv, sum);
            }
            vk = win[wid][lane + kWinLo];
        } else {
            auto xv = [&](int c) { return (double)(T)(wprev[c] * inv); };
            if (SellCol<CI>::stepped && row.exc) {
                sum = csr_row_sum<A>(i < n ? row.xrow : -1, xrp, xcol, xval, xv);
            } else if constexpr (PIPE) {
                // two batch buffers: batch q's gathers are issued, then batch
                // q + U's loads, so the wait for the gathers leaves the next
                // batch's loads in flight under the sums (one HBM round trip
                // per batch instead of a load round trip then a gather round
                // trip). x is gathered raw and scaled at the sum: the same
                // (T)(w_prev * inv) operand, the same bits.
                using Row = SellRow<S, CI, W>;
                Row rb;
                rb.geom_from(row);
                auto xraw = [&](int c) { return wprev[c]; };
                auto xs = [&](T r) { return (double)(T)(r * inv); };
                T x[Row::U][W];
                for (int q = 0;;) {
                    row.gather(xraw, x);
                    __builtin_amdgcn_sched_barrier(0);
                    rb.load(q + Row::U);
                    __builtin_amdgcn_sched_barrier(0);
                    row.sum_gathered(q, x, xs, sum);
                    q += Row::U;
                    if (q >= row.steps) break;
                    rb.gather(xraw, x);
                    __builtin_amdgcn_sched_barrier(0);
                    row.load(q + Row::U);
                    __builtin_amdgcn_sched_barrier(0);
                    rb.sum_gathered(q, x, xs, sum);
                    q += Row::U;
                    if (q >= row.steps) break;
                }
            } else {
                row.sum(0, xv, sum);
                for (int q = row.U; q < row.steps; q += row.U) {
                    row.load(q);
                    row.sum(q, xv, sum);
                }
            }
            vk = (T)(wr[0] * inv);
        }
    }
    T wi = T(0);
    if (live && i < n) {
        if constexpr (std::is_same_v<VI, half_v>) sum = ldexp(sum, -rex);  // exact unscale (0: unchanged)
        const T t = (T)sum;  // spmv(1, A, v, 0, w): y = 1*t
        wi = precond<T, P>(t, diag, i);
        w[i] = wi;
        V[(int64_t)k * ld + i] = vk;
    }
    if constexpr (DN > 0) {
        // the earlier basis columns at this row: clamped, branch-free loads
        // issued together (one latency), then one product per column
        // (n >= 1: spmv_impl refuses the fused dots on an empty block, so row n - 1 exists)
        const bool own_row = live && i < n;
        const int ic = i < n ? i : n - 1;
        const int kc = k > 0 ? k - 1 : 0;
        T vc[DN];
#pragma unroll
        for (int c = 0; c < DN; ++c) vc[c] = V[(int64_t)(c < kc ? c : kc) * ld + ic];
        __builtin_amdgcn_sched_barrier(0);
        const double wd = (double)wi;
        double acc[DN];
        // a lane without a row contributes an exact 0 (not a clamped row's
        // value times 0, which is NaN when that value is Inf or NaN)
#pragma unroll
        for (int c = 0; c < DN; ++c)
            acc[c] = own_row ? (c < k ? (double)vc[c] : c == k ? (double)vk : 0.0) * wd : 0.0;
        store_partials<DN, kBlock, true>(acc, dd.nc, dd.wgpart);
        const int g = blockIdx.x / dd.gs;
        const int m0 = g * dd.gs, m1 = m0 + dd.gs < (int)gridDim.x ? m0 + dd.gs : (int)gridDim.x;
        if (last_arriver_of(dd.cnt + g, (unsigned)(m1 - m0)) && (int)threadIdx.x < dd.nc) {
            const int c = threadIdx.x;
            double v = 0.0;
            for (int m = m0; m < m1; ++m) v += dd.wgpart[(size_t)c * gridDim.x + m];
            dd.out[(size_t)c * dd.ng + g] = v;
        }
    }
    if constexpr (FOLD) {
        __shared__ T col_s[kFoldMaxM + 2], c_s[kFoldMaxM + 2], s_s[kFoldMaxM + 2];
        if (blockIdx.x == 0) givens_block(fold.g, nrm2sq, col_s, c_s, s_s);
    }
}

// k_step_sell with two adjacent slices per wave (lane l owns rows
// 128 s' + l and 128 s' + 64 + l): every load of both slices -- one LDS
// window of 64 + 128 + 64 entries for the pair, both slices' first batches --
// is in flight before the wave waits for any, so each wave carries twice the
// bytes through the same fixed work (the fold's partial sum, the barriers,
// the window). Past the Infinity Cache a slice's loads alone do not keep
// enough bytes in flight per CU (MI355X_MICROARCH.md: ~72 KiB per CU hides
// an HBM miss). Same sums in the same order as k_step_sell: same bits.
template <class T, class P, class VI, int W, bool WIN, bool FOLD, int BE, int BS = kBlock, bool PG = true,
          class A = double>
__global__ __launch_bounds__(BS) void k_step_sell2(int n, int n_lo, int n_ext, int nslices, const int64_t* __restrict__ off,
                                                   const int16_t* __restrict__ col,
                                                   const typename SellStore<VI>::type* __restrict__ val,
                                                   const T* __restrict__ wprev, const T* __restrict__ inv_p,
                                                   T* __restrict__ V, int64_t ld, int k,
                                                   const P* __restrict__ diag, T* __restrict__ w,
                                                   GivensFold<T> fold, SellDots,
                                                   const int32_t* __restrict__ sbase,
                                                   const int32_t* __restrict__ spat, const int64_t* __restrict__ coff, const int16_t* __restrict__ pat,
                                                   const int32_t* __restrict__ xrp,
                                                   const int32_t* __restrict__ xcol,
                                                   const typename SellStore<VI>::type* __restrict__ xval,
                                                   const int8_t* __restrict__ rexp, int64_t ustride, int xcd) {
    using S = typename SellStore<VI>::type;
    using CI = int16_t;
    constexpr bool UNI = true;
    constexpr int SPW = 2;
    constexpr int WL = kWinLen + (SPW - 1) * kWave;  // the pair's window
    constexpr int NQ = WL / kWave;
    __shared__ T win[WIN ? BS / kWave : 1][WIN ? WL : 1];
    const int lane = threadIdx.x & (kWave - 1), wid = wave_id();
    const int s0 = ((xcd ? xcd_block(blockIdx.x, gridDim.x) : (int)blockIdx.x) * (BS / kWave) + wid) * SPW;
    const bool live = s0 < nslices;  // a dead wave still joins the fold's barriers
    bool live_p[SPW];
    const int row0 = s0 * kWave;
    // 0. both slices' offsets (UNI: computed) and pattern indices
    SellRow<S, CI, W, (MPG_SELL_NT != 0), BE> row[SPW];
#pragma unroll
    for (int p = 0; p < SPW; ++p) {
        live_p[p] = s0 + p < nslices;
        const int sp = live_p[p] ? s0 + p : 0;
        if constexpr (UNI) row[p].init_uniform(sp, ustride, spat, coff);
        else row[p].init_load(sp, off, spat, coff);
    }
    __builtin_amdgcn_sched_barrier(0);
    // 1. the fold's ||w||^2 partial (one per lane, as k_step_sell)
    constexpr int NPL = BS < kBlock ? kBlock / BS : 1;
    A part[NPL];
#pragma unroll
    for (int j = 0; j < NPL; ++j) part[j] = A(0);
    if constexpr (FOLD) {
#pragma unroll
        for (int j = 0; j < NPL; ++j) {
            const int t = j * BS + (int)threadIdx.x;
            part[j] = (A)fold.norm2[t < fold.nparts ? t : 0];
            if (t >= fold.nparts) part[j] = A(0);
        }
    }
    __builtin_amdgcn_sched_barrier(0);
    // 2. the pair's w_prev window (or the lane's own rows' w_prev), raw
    T wr[WIN ? NQ : SPW];
    if constexpr (WIN) {
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            const int c = row0 - kWinLo + q * kWave + lane;
            wr[q] = wprev[c >= n_lo && c < n_ext ? c : 0];
        }
    } else {
#pragma unroll
        for (int p = 0; p < SPW; ++p) {
            const int i = row0 + p * kWave + lane;
            wr[p] = wprev[i < n ? i : 0];
        }
    }
    __builtin_amdgcn_sched_barrier(0);
    // 3. both slices' first batches (UNI: values first, then the columns)
    if constexpr (UNI) {
#pragma unroll
        for (int p = 0; p < SPW; ++p) {
            row[p].init_vals(lane, val);
            row[p].load_vals(0);
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int p = 0; p < SPW; ++p) {
            row[p].init_finish(lane, col, val, sbase, pat);
            row[p].load_cols(0);
        }
    } else {
#pragma unroll
        for (int p = 0; p < SPW; ++p) {
            row[p].init_finish(lane, col, val, sbase, pat);
            row[p].load(0);
        }
    }
    // 4. a scaled fp16 copy's row exponents
    int rex[SPW] = {};
    if constexpr (std::is_same_v<VI, half_v>) {
        if (rexp) {
#pragma unroll
            for (int p = 0; p < SPW; ++p) {
                const int i = row0 + p * kWave + lane;
                rex[p] = rexp[live_p[p] && i < n ? i : 0];
            }
        }
    }
    __builtin_amdgcn_sched_barrier(0);
    // 5. PG, no window: the first batch's gathers of w_prev, raw, issued
    // before the scale is known (the fold's sums and barriers), and scaled
    // at the sum: (T)(w_prev * inv), the same operation, the same bits.
    // A dead wave gathers for slice 0 (valid addresses) and returns.
    constexpr bool PRE = PG && !WIN;
    using RowT = SellRow<S, CI, W, (MPG_SELL_NT != 0), BE>;
    T xr[PRE ? SPW : 1][PRE ? RowT::U : 1][PRE ? W : 1];
    if constexpr (PRE) {
#pragma unroll
        for (int p = 0; p < SPW; ++p) row[p].gather([&](int c) { return wprev[c]; }, xr[p]);
    }
    __builtin_amdgcn_sched_barrier(0);
    T inv;
    double nrm2sq = 0.0;
    if constexpr (FOLD) {
        constexpr int NG = (BS < kBlock ? kBlock : BS) / kWave;
        __shared__ A scratch[NG];
        __shared__ T inv_s;
        if (fold.nparts > 0) {
#pragma unroll
            for (int j = 0; j < NPL; ++j) {
                const A v = wave_sum(part[j] + A(0));
                if (lane == 0) scratch[j * (BS / kWave) + wid] = v;
            }
            lds_barrier();
            A r = A(0);
#pragma unroll
            for (int q = 0; q < NG; ++q) r += scratch[q];
            nrm2sq = (double)r;
        } else {
            nrm2sq = fold.norm2[0];
        }
        if (threadIdx.x == 0) inv_s = inv_of_norm2<T>(nrm2sq);
        lds_barrier();
        inv = inv_s;
    } else {
        inv = *inv_p;
    }
    if (!live && !(FOLD && blockIdx.x == 0)) return;
    A sum[SPW] = {};
    T vk[SPW] = {};
    if (live) {
        if constexpr (WIN) {
#pragma unroll
            for (int q = 0; q < NQ; ++q) {
                const int c = row0 - kWinLo + q * kWave + lane;
                win[wid][q * kWave + lane] = (c >= n_lo && c < n_ext) ? (T)(wr[q] * inv) : T(0);
            }
            wave_lds_sync();
            auto xv = [&](int c) { return (double)win[wid][c - row0 + kWinLo]; };
#pragma unroll
            for (int p = 0; p < SPW; ++p) row[p].sum(0, xv, sum[p]);
#pragma unroll
            for (int p = 0; p < SPW; ++p) {
                for (int q = row[p].U; q < row[p].steps; q += row[p].U) {
                    row[p].load(q);
                    row[p].sum(q, xv, sum[p]);
                }
                vk[p] = win[wid][p * kWave + lane + kWinLo];
            }
        } else {
            auto xv = [&](int c) { return (double)(T)(wprev[c] * inv); };
#pragma unroll
            for (int p = 0; p < SPW; ++p) {
                const int i = row0 + p * kWave + lane;
                if (SellCol<CI>::stepped && row[p].exc) {
                    sum[p] = csr_row_sum<A>(live_p[p] && i < n ? row[p].xrow : -1, xrp, xcol, xval, xv);
                } else {
                    if constexpr (PRE) row[p].sum_gathered(0, xr[p], [&](T r) { return (double)(T)(r * inv); }, sum[p]);
                    else row[p].sum(0, xv, sum[p]);
                    for (int q = row[p].U; q < row[p].steps; q += row[p].U) {
                        row[p].load(q);
                        row[p].sum(q, xv, sum[p]);
                    }
                }
                vk[p] = (T)(wr[p] * inv);
            }
        }
    }
#pragma unroll
    for (int p = 0; p < SPW; ++p) {
        const int i = row0 + p * kWave + lane;
        if (live_p[p] && i < n) {
            double sp = sum[p];
            if constexpr (std::is_same_v<VI, half_v>) sp = ldexp(sp, -rex[p]);
            const T t = (T)sp;
            w[i] = precond<T, P>(t, diag, i);
            V[(int64_t)k * ld + i] = vk[p];
        }
    }
    if constexpr (FOLD) {
        __shared__ T col_s[kFoldMaxM + 2], c_s[kFoldMaxM + 2], s_s[kFoldMaxM + 2];
        if (blockIdx.x == 0) givens_block(fold.g, nrm2sq, col_s, c_s, s_s);
    }
}

// Tall-skinny panel reduction: partial <v_j, w> for j in [c0, c0 + nc),
// nc <= kNC, over all local rows. Each lane owns 4 consecutive rows per
// iteration (16-B loads of every column: V's leading dimension is padded to
// 256 B), issues all column loads before its FMAs, and keeps one fp64
// accumulator per column; store_partials does the wave64/LDS combine.
// BS threads per workgroup. COMBINE (one GPU, nc <= kNC, c0 == 0): the
// partials go write-through and the last-arriving workgroup sums them into
// sums[0..nc) itself — no separate reduce launch (BS = 1024, so one
// workgroup per CU keeps the partial count at 256 per column).
template <class T, int BS = kBlock, bool COMBINE = false, class A = double>
__global__ __launch_bounds__(BS) void k_panel_dots(int n, const T* __restrict__ V, int64_t ld, int c0, int nc,
                                                   const T* __restrict__ w, double* __restrict__ partial,
                                                   unsigned* __restrict__ cnt, double* __restrict__ sums) {
    A acc[kNC];
#pragma unroll
    for (int c = 0; c < kNC; ++c) acc[c] = A(0);
    const int n4 = n & ~3;
    const T* __restrict__ Vb = V + (int64_t)c0 * ld;
    for (int i = 4 * (blockIdx.x * BS + threadIdx.x); i < n4; i += 4 * gridDim.x * BS) {
        A wv[4];
        Row4<T>::load(w + i, wv);
#pragma unroll
        for (int c = 0; c < kNC; ++c) {
            if (c < nc) {
                A v[4];
                Row4<T>::load(Vb + (int64_t)c * ld + i, v);
                acc[c] += v[0] * wv[0] + v[1] * wv[1] + v[2] * wv[2] + v[3] * wv[3];
            }
        }
    }
    // tail rows (n not a multiple of 4)
    for (int i = n4 + blockIdx.x * BS + threadIdx.x; i < n; i += gridDim.x * BS) {
        const A wi = (A)w[i];
#pragma unroll
        for (int c = 0; c < kNC; ++c)
            if (c < nc) acc[c] += (A)Vb[(int64_t)c * ld + i] * wi;
    }
    store_partials<kNC, BS, COMBINE>(acc, nc, partial + (size_t)c0 * gridDim.x);
    if constexpr (COMBINE) {
        if (last_arriver(cnt)) combine_columns<BS, A>(partial, gridDim.x, nc, sums);
    }
}

// The one-panel forms of the dots and the CGS update with the column count
// NC a compile-time constant (the captured cycle knows k at every step):
// every column index is static, so the loads of a batch of columns issue
// back to back and the accumulators stay in registers. With a runtime
// count the compiler guarded each column's load with its own branch and
// waited for it before the next (one memory latency per column: t(k) =
// 8.6 + 0.50 k us for the dots on BAND-10M, tools/per_step.py).
template <class T, int BS, int NC, class A = double>
__device__ __forceinline__ void dots_panel(int n, const T* __restrict__ V, int64_t ld, const T* __restrict__ w,
                                           double* __restrict__ partial) {
    static_assert(NC >= 1 && NC <= kNC, "one panel");
    constexpr int NP = Pow2Ceil<NC>::v;
    constexpr int B = kColBatch<T>;
    A acc[NP];
#pragma unroll
    for (int c = 0; c < NP; ++c) acc[c] = A(0);
    const int n4 = n & ~3;
    for (int i = 4 * (blockIdx.x * BS + threadIdx.x); i < n4; i += 4 * gridDim.x * BS) {
        A wv[4];
        Row4<T>::load(w + i, wv);
#pragma unroll
        for (int c0 = 0; c0 < NC; c0 += B) {
            Raw4<T> v[B];
#pragma unroll
            for (int u = 0; u < B; ++u)
                if (c0 + u < NC) v[u].load(V + (int64_t)(c0 + u) * ld + i);
            __builtin_amdgcn_sched_barrier(0);  // keep the batch's loads issued back to back
#pragma unroll
            for (int u = 0; u < B; ++u)
                if (c0 + u < NC)
                    acc[c0 + u] += v[u].template at<A>(0) * wv[0] + v[u].template at<A>(1) * wv[1] +
                                   v[u].template at<A>(2) * wv[2] + v[u].template at<A>(3) * wv[3];
            // the next batch's loads after this batch's adds: without it the
            // fp32 class's NC = 32 form issued all 32 columns' loads first
            // (128 VGPRs, 180 B of scratch per lane)
            asm volatile("" : "+v"(acc[c0]) : : "memory");
        }
    }
    for (int i = n4 + blockIdx.x * BS + threadIdx.x; i < n; i += gridDim.x * BS) {
        const A wi = (A)w[i];
#pragma unroll
        for (int c = 0; c < NC; ++c) acc[c] += (A)V[(int64_t)c * ld + i] * wi;
    }
    store_partials<NP, BS>(acc, NC, partial);
}

template <class T, int BS, int NC, bool STAMP = false, class A = double>
__global__ __launch_bounds__(BS) void k_dots_nc(int n, const T* __restrict__ V, int64_t ld,
                                                const T* __restrict__ w, double* __restrict__ partial,
                                                unsigned long long* stamp) {
    stamp_at<STAMP>(stamp, 0);
    dots_panel<T, BS, NC, A>(n, V, ld, w, partial);
    stamp_at<STAMP>(stamp, 1);
}

// V^T w for nc > kNC columns in ONE launch (GMRES(100): the round-3 form ran
// one runtime-count k_panel_dots launch per 32 columns, each re-reading w and
// waiting for every column in turn): blockIdx.y is the 32-column panel,
// the last one holding NCL columns; blockIdx.x a row group. The grid keeps
// about one workgroup per CU in total (gridDim.x = kCombineGroups / panels),
// so each column gets gridDim.x <= 128 partials, [column][gridDim.x], which
// the wide CGS update sums itself (k_cgs_update_wide).
template <class T, int BS, int NCL, class A = double>
__global__ __launch_bounds__(BS) void k_dots_panels(int n, const T* __restrict__ V, int64_t ld,
                                                    const T* __restrict__ w, double* __restrict__ partial) {
    const int c0 = blockIdx.y * kNC;
    double* __restrict__ part = partial + (size_t)c0 * gridDim.x;
    if (blockIdx.y + 1 < gridDim.y) dots_panel<T, BS, kNC, A>(n, V + (int64_t)c0 * ld, ld, w, part);
    else dots_panel<T, BS, NCL, A>(n, V + (int64_t)c0 * ld, ld, w, part);
}

// coef = T(sums[0..NC)); w = w - T(V coef); partial ||w'||^2 (the last
// CGS pass; same arithmetic and order as k_cgs_update).
// FROM_PARTS (one GPU): the coefficients are summed here from the one-panel
// dots' part_G <= kCombineGroups partials per column (32 lanes per column,
// each summing its 8 strided partials in g order, then a 32-lane xor tree:
// the same fixed order in every workgroup) instead of a reduce launch. The 8
// loads per lane are branch-free so they issue together: one latency.
// NEXT_DOTS (CGSR's first pass): the partials of <v_j, w'> for j < NC
// instead of ||w'||^2, from a second batched pass over the lane's columns.
// PF (with FROM_PARTS): the lane's first row group -- w and the first batch
// of basis columns, raw and unconditional (clamped row) -- is issued right
// behind the partial loads, so its memory latency runs under the coefficient
// sums; the coefficients are published with an LDS-only barrier
// (__syncthreads would drain those loads). Same operands, same order.
template <class T, int BS, int NC, bool FROM_PARTS = false, bool NEXT_DOTS = false, bool PF = false,
          bool STAMP = false, class A = double>
__global__ __launch_bounds__(BS) void k_cgs_update_nc(int n, const T* __restrict__ V, int64_t ld,
                                                      const double* __restrict__ sums, int part_G,
                                                      T* __restrict__ coef_out, T* __restrict__ w,
                                                      double* __restrict__ partial, unsigned long long* stamp) {
    static_assert(NC >= 1 && NC <= kNC, "one panel");
    stamp_at<STAMP>(stamp, 0);
    static_assert(!FROM_PARTS || BS >= 32 * NC, "32 lanes per column");
    static_assert(!PF || (FROM_PARTS && !NEXT_DOTS), "prefetch under the partial sums");
    static_assert(!PF || NC <= kColBatch<T>, "the prefetch form holds one batch of columns (the only form run)");
    constexpr int B = kColBatch<T>;
    constexpr int B0 = NC < B ? NC : B;
    __shared__ A coef[NC];
    const int n4 = n & ~3;
    const int i_first = 4 * (blockIdx.x * BS + threadIdx.x);
    Raw4<T> pw, pv[PF ? B0 : 1];
    if constexpr (FROM_PARTS) {
        const int j = threadIdx.x / 32, sub = threadIdx.x % 32;
        const int jc = j < NC ? j : NC - 1;
        constexpr int Q = kCombineGroups / 32;
        A pp[Q];
#pragma unroll
        for (int q = 0; q < Q; ++q) {
            const int g = sub + 32 * q;
            pp[q] = (A)sums[(size_t)jc * part_G + (g < part_G ? g : 0)];
        }
        if constexpr (PF) {
            __builtin_amdgcn_sched_barrier(0);
            const int ip = i_first < n4 ? i_first : 0;
            pw.load(w + ip);
#pragma unroll
            for (int u = 0; u < B0; ++u) pv[u].load(V + (int64_t)u * ld + ip);
            __builtin_amdgcn_sched_barrier(0);
        }
        A v = A(0);
#pragma unroll
        for (int q = 0; q < Q; ++q)
            if (sub + 32 * q < part_G) v += pp[q];
#pragma unroll
        for (int o = 16; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
        if (j < NC && sub == 0) {
            const T c = (T)v;
            coef[j] = (A)c;
            if (blockIdx.x == 0) coef_out[j] = c;
        }
    } else if (threadIdx.x < NC) {
        const T c = (T)sums[threadIdx.x];
        coef[threadIdx.x] = (A)c;
        if (blockIdx.x == 0) coef_out[threadIdx.x] = c;
    }
    if constexpr (PF) lds_barrier();
    else __syncthreads();
    constexpr int NA = NEXT_DOTS ? Pow2Ceil<NC>::v : 1;
    A acc[NA];
#pragma unroll
    for (int c = 0; c < NA; ++c) acc[c] = A(0);
    bool first = PF;
    for (int i = i_first; i < n4; i += 4 * gridDim.x * BS) {
        Raw4<T> wr;
        if (first) wr = pw;
        else wr.load(w + i);
        A t[4] = {A(0), A(0), A(0), A(0)};
#pragma unroll
        for (int c0 = 0; c0 < NC; c0 += B) {
            Raw4<T> v[B];
#pragma unroll
            for (int u = 0; u < B; ++u)
                if (c0 + u < NC) {
                    if (c0 == 0 && first) v[u] = pv[u < B0 ? u : 0];
                    else v[u].load(V + (int64_t)(c0 + u) * ld + i);
                }
            __builtin_amdgcn_sched_barrier(0);  // keep the batch's loads issued back to back
#pragma unroll
            for (int u = 0; u < B; ++u)
                if (c0 + u < NC) {
                    const A cu = coef[c0 + u];
#pragma unroll
                    for (int r = 0; r < 4; ++r) t[r] += v[u].template at<A>(r) * cu;
                }
        }
        T wo[4];
        A wd[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            wo[r] = T(-1) * (T)t[r] + T(1) * (T)wr[r];
            wd[r] = (A)wo[r];
            if (!NEXT_DOTS) acc[0] += wd[r] * wd[r];
        }
        Row4<T>::store(w + i, wo);
        first = false;
        if constexpr (NEXT_DOTS) {
#pragma unroll
            for (int c0 = 0; c0 < NC; c0 += B) {
                Raw4<T> v[B];
#pragma unroll
                for (int u = 0; u < B; ++u)
                    if (c0 + u < NC) v[u].load(V + (int64_t)(c0 + u) * ld + i);
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int u = 0; u < B; ++u)
                    if (c0 + u < NC)
                        acc[c0 + u] += v[u].template at<A>(0) * wd[0] + v[u].template at<A>(1) * wd[1] +
                                       v[u].template at<A>(2) * wd[2] + v[u].template at<A>(3) * wd[3];
            }
        }
    }
    for (int i = n4 + blockIdx.x * BS + threadIdx.x; i < n; i += gridDim.x * BS) {
        A t = A(0);
#pragma unroll
        for (int j = 0; j < NC; ++j) t += (A)V[(int64_t)j * ld + i] * coef[j];
        const T wi = T(-1) * (T)t + T(1) * w[i];
        w[i] = wi;
        if constexpr (NEXT_DOTS) {
#pragma unroll
            for (int c = 0; c < NC; ++c) acc[c] += (A)V[(int64_t)c * ld + i] * (A)wi;
        } else {
            acc[0] += (A)wi * (A)wi;
        }
    }
    store_partials<NA, BS>(acc, NEXT_DOTS ? NC : 1, partial);
    stamp_at<STAMP>(stamp, 1);
}

// The CGS update for kNC < nc <= kWideMax columns (GMRES(100)): the
// coefficients are summed here from k_dots_panels' part_G <= 128 partials per
// column (8 lanes per column, 16 branch-free loads each in g order, then an
// xor tree: the same fixed order in every workgroup; no reduce launch), then
// w = w - T(V coef) with 4 rows per lane, the columns in compile-time batches
// of B (the last batch clamped to column nc - 1 with coefficient 0: +0 terms,
// so t is the j-ordered sum of the real terms), and the ||w'||^2 partials.
constexpr int kWideMax = 128;
template <class T, int BS, class A = double>
__global__ __launch_bounds__(BS) void k_cgs_update_wide(int n, const T* __restrict__ V, int64_t ld, int nc,
                                                        const double* __restrict__ parts, int part_G,
                                                        T* __restrict__ coef_out, T* __restrict__ w,
                                                        double* __restrict__ partial) {
    constexpr int LPC = BS / kWideMax, Q = 128 / LPC, B = kColBatch<T>;
    static_assert(LPC * kWideMax == BS && Q * LPC == 128, "8 lanes per column, <= 128 partials");
    __shared__ A coef[kWideMax];
    {
        const int j = threadIdx.x / LPC, sub = threadIdx.x % LPC;
        const int jc = j < nc ? j : nc - 1;
        A pp[Q];
#pragma unroll
        for (int q = 0; q < Q; ++q) {
            const int g = sub + LPC * q;
            pp[q] = (A)parts[(size_t)jc * part_G + (g < part_G ? g : 0)];
        }
        A v = A(0);
#pragma unroll
        for (int q = 0; q < Q; ++q)
            if (sub + LPC * q < part_G) v += pp[q];
#pragma unroll
        for (int o = LPC / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
        if (sub == 0) {
            const T c = (T)v;
            coef[j] = j < nc ? (A)c : A(0);
            if (blockIdx.x == 0 && j < nc) coef_out[j] = c;
        }
    }
    __syncthreads();
    A acc[1] = {A(0)};
    const int n4 = n & ~3;
    const int nb = (nc + B - 1) / B;
    for (int i = 4 * (blockIdx.x * BS + threadIdx.x); i < n4; i += 4 * gridDim.x * BS) {
        Raw4<T> wr;
        wr.load(w + i);
        A t[4] = {A(0), A(0), A(0), A(0)};
        for (int bi = 0; bi < nb; ++bi) {
            const int c0 = bi * B;
            Raw4<T> v[B];
#pragma unroll
            for (int u = 0; u < B; ++u) {
                const int c = c0 + u < nc ? c0 + u : nc - 1;
                v[u].load(V + (int64_t)c * ld + i);
            }
            __builtin_amdgcn_sched_barrier(0);  // keep the batch's loads issued back to back
#pragma unroll
            for (int u = 0; u < B; ++u) {
                const A cu = coef[c0 + u < kWideMax ? c0 + u : kWideMax - 1];
                if (c0 + u < nc)
#pragma unroll
                    for (int r = 0; r < 4; ++r) t[r] += v[u].template at<A>(r) * cu;
            }
        }
        T wo[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            wo[r] = T(-1) * (T)t[r] + T(1) * (T)wr[r];
            const A wd = (A)wo[r];
            acc[0] += wd * wd;
        }
        Row4<T>::store(w + i, wo);
    }
    for (int i = n4 + blockIdx.x * BS + threadIdx.x; i < n; i += gridDim.x * BS) {
        A t = A(0);
        for (int j = 0; j < nc; ++j) t += (A)V[(int64_t)j * ld + i] * coef[j];
        const T wi = T(-1) * (T)t + T(1) * w[i];
        w[i] = wi;
        acc[0] += (A)wi * (A)wi;
    }
    store_partials<1, BS>(acc, 1, partial);
}

// f(integral_constant<int, nc>) for 1 <= nc <= N
template <int N, class F>
int with_nc(int nc, F&& f) {
    if constexpr (N == 0) {
        return MPG_ERR_ARG;
    } else {
        if (nc == N) return f(std::integral_constant<int, N>());
        return with_nc<N - 1>(nc, f);
    }
}

// ---------------------------------------------------------------- step: CGS
// coef = T(sums[0..k]); w = w - T(V coef) (gemv(-1, V, h, 1, w));
// NEXT_DOTS: partials <v_j, w'> (j <= k) else partial ||w'||^2.
// Each lane owns 4 consecutive rows (16-B loads of every basis column), and
// issues the loads of 8 columns before their FMAs; the row sum t runs over
// j = 0..k in order in fp64, as the scalar form did.
// GIVENS (one GPU, last pass, m <= kFoldMaxM): the ||w'||^2 partials go
// write-through and the last-arriving workgroup sums them and runs the
// Givens step k (givens_block) — no separate Givens launch.
template <class T, bool NEXT_DOTS, bool GIVENS = false, int BS = kBlock, bool FROM_PARTS = false, class A = double>
__global__ __launch_bounds__(BS) void k_cgs_update(int n, const T* __restrict__ V, int64_t ld, int k,
                                                       const double* __restrict__ sums, T* __restrict__ coef_out,
                                                       T* __restrict__ w, double* __restrict__ partial,
                                                       unsigned* __restrict__ cnt, GivensArgs<T> g, int part_G) {
    static_assert(!(NEXT_DOTS && GIVENS), "the Givens step follows the last pass");
    __shared__ A coef[256];
    const int nc = k + 1;
    const int n4 = n & ~3;
    const int i_first = 4 * (blockIdx.x * BS + threadIdx.x);
    // part_G > 0: this lane's first row group (the first kPre columns and w)
    // is loaded BEFORE the coefficient sums, so the partial loads below
    // travel with it and their latency hides behind the basis stream
    constexpr int kPre = 8;
    const int npre = nc < kPre ? nc : kPre;
    const bool pre = FROM_PARTS && i_first < n4;
    A pv[kPre][4], pw[4];
    if (pre) {
#pragma unroll
        for (int u = 0; u < kPre; ++u)
            if (u < npre) Row4<T>::load(V + (int64_t)u * ld + i_first, pv[u]);
        Row4<T>::load(w + i_first, pw);
    }
    if (FROM_PARTS) {
        // sums straight from the panel-dots partials (nc <= kNC, part_G per
        // column): LPC lanes per column, each summing part_G / LPC partials
        // (all loads issued first) in g order, then an xor tree — the same
        // fixed order in every workgroup
        constexpr int LPC = BS / kNC;
        const int j = threadIdx.x / LPC, sub = threadIdx.x % LPC;
        const int per = (part_G + LPC - 1) / LPC;
        A v = A(0);
        if (j < nc) {
            const double* src = sums + (size_t)j * part_G + sub;
#pragma unroll 8
            for (int q = 0; q < per; ++q)
                if (q * LPC + sub < part_G) v += (A)src[q * LPC];
        }
#pragma unroll
        for (int o = LPC / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
        if (j < nc && sub == 0) {
            const T c = (T)v;
            coef[j] = (A)c;
            if (blockIdx.x == 0) coef_out[j] = c;
        }
    } else {
        for (int j = threadIdx.x; j < nc; j += BS) {
            const T c = (T)sums[j];
            coef[j] = (A)c;
            if (blockIdx.x == 0) coef_out[j] = c;
        }
    }
    __syncthreads();
    constexpr int NA = NEXT_DOTS ? kNC : 1;
    A acc[NA];
#pragma unroll
    for (int c = 0; c < NA; ++c) acc[c] = A(0);
    for (int i = i_first; i < n4; i += 4 * gridDim.x * BS) {
        A t[4] = {A(0), A(0), A(0), A(0)};
        int j = 0;
        const bool use_pre = pre && i == i_first;
        if (use_pre) {
#pragma unroll
            for (int u = 0; u < kPre; ++u)
                if (u < npre)
#pragma unroll
                    for (int r = 0; r < 4; ++r) t[r] += pv[u][r] * coef[u];
            j = npre;
        }
        for (; j + 8 <= nc; j += 8) {
            A v[8][4];
#pragma unroll
            for (int u = 0; u < 8; ++u) Row4<T>::load(V + (int64_t)(j + u) * ld + i, v[u]);
#pragma unroll
            for (int u = 0; u < 8; ++u)
#pragma unroll
                for (int r = 0; r < 4; ++r) t[r] += v[u][r] * coef[j + u];
        }
        for (; j < nc; ++j) {
            A v[4];
            Row4<T>::load(V + (int64_t)j * ld + i, v);
#pragma unroll
            for (int r = 0; r < 4; ++r) t[r] += v[r] * coef[j];
        }
        A wv[4];
        if (use_pre) {
#pragma unroll
            for (int r = 0; r < 4; ++r) wv[r] = pw[r];
        } else {
            Row4<T>::load(w + i, wv);
        }
        T wo[4];
        A wd[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            wo[r] = T(-1) * (T)t[r] + T(1) * (T)wv[r];
            wd[r] = (A)wo[r];
        }
        Row4<T>::store(w + i, wo);
        if (NEXT_DOTS) {
#pragma unroll
            for (int c = 0; c < NA; ++c) {
                if (c < nc) {
                    A v[4];
                    Row4<T>::load(V + (int64_t)c * ld + i, v);
                    acc[c] += v[0] * wd[0] + v[1] * wd[1] + v[2] * wd[2] + v[3] * wd[3];
                }
            }
        } else {
            acc[0] += wd[0] * wd[0] + wd[1] * wd[1] + wd[2] * wd[2] + wd[3] * wd[3];
        }
    }
    // tail rows (n not a multiple of 4)
    for (int i = n4 + blockIdx.x * BS + threadIdx.x; i < n; i += gridDim.x * BS) {
        A t = A(0);
        for (int j = 0; j < nc; ++j) t += (A)V[(int64_t)j * ld + i] * coef[j];
        const T wi = T(-1) * (T)t + T(1) * w[i];
        w[i] = wi;
        if (NEXT_DOTS) {
#pragma unroll
            for (int c = 0; c < NA; ++c)
                if (c < nc) acc[c] += (A)V[(int64_t)c * ld + i] * (A)wi;
        } else {
            acc[0] += (A)wi * (A)wi;
        }
    }
    store_partials<NA, BS, GIVENS>(acc, NEXT_DOTS ? (nc < kNC ? nc : kNC) : 1, partial);
    if constexpr (GIVENS) {
        if (last_arriver(cnt)) {
            __shared__ T col[kFoldMaxM + 2], c_s[kFoldMaxM + 2], s_s[kFoldMaxM + 2];
            __shared__ A scratch[BS / kWave];
            const double nrm2sq = (double)sum_partials<BS, A>(partial, gridDim.x, scratch);
            givens_block(g, nrm2sq, col, c_s, s_s);
        }
    }
}

// ---------------------------------------------------------------- step: MGS
// h_jk = T(sums[0]); w -= h_jk v_j (naxpy); partial <v_{j+1}, w> or ||w||^2.
// src_G > 0: h_jk is summed here from the src_G partials of the previous
// launch (the dots or the previous MGS update, one GPU), in the same fixed
// order in every workgroup — one launch per j instead of reduce + update.
// Each lane owns 4 consecutive rows (16-B loads).
template <class T, int BS, class A = double>
__global__ __launch_bounds__(BS) void k_mgs_update(int n, const T* __restrict__ V, int64_t ld, int j, int k,
                                                   const double* __restrict__ src, int src_G, T* __restrict__ hjk,
                                                   T* __restrict__ w, double* __restrict__ partial) {
    __shared__ A scratch[BS / kWave];
    __shared__ T h_s;
    const T* __restrict__ vj = V + (int64_t)j * ld;
    const T* __restrict__ vn = V + (int64_t)(j + 1) * ld;
    const bool last = j == k;
    const int n4 = n & ~3;
    // this lane's first row group is loaded before h_jk is known, so its
    // latency overlaps the partial sum's instead of following it
    const int i_first = 4 * (blockIdx.x * BS + threadIdx.x);
    const bool pre = i_first < n4;
    // raw and unconditional (a clamped address when this lane has no row
    // group): a guarded load would be widened to fp64 inside its branch,
    // i.e. waited for right here. Column j + 1 <= m exists; unused when last.
    // The partial (src_G <= BS: one per lane) is loaded FIRST: vmcnt retires
    // in order, so waiting for it must not wait for the row group behind it.
    static_assert(BS >= kCombineGroups * 4, "one partial per lane");
    A part = (A)src[threadIdx.x < src_G ? threadIdx.x : 0];
    if (threadIdx.x >= src_G) part = A(0);
    __builtin_amdgcn_sched_barrier(0);
    const int ip = pre ? i_first : 0;
    Raw4<T> pw, pv, pn;
    pw.load(w + ip);
    pv.load(vj + ip);
    pn.load(vn + ip);
    __builtin_amdgcn_sched_barrier(0);
    // LDS-only barriers: the first row group's loads stay in flight. The
    // block sum runs unconditionally so the partial load is not sunk below
    // the row group's loads.
    {
        const A v = wave_sum(part + A(0));  // = sum_partials' order for src_G <= BS
        if ((threadIdx.x & (kWave - 1)) == 0) scratch[threadIdx.x / kWave] = v;
        lds_barrier();
        if (threadIdx.x == 0) {
            A r = A(0);
#pragma unroll
            for (int q = 0; q < BS / kWave; ++q) r += scratch[q];
            h_s = src_G > 0 ? (T)r : (T)src[0];
        }
    }
    lds_barrier();
    const T h = h_s;
    if (blockIdx.x == 0 && threadIdx.x == 0) *hjk = h;
    A acc[1] = {A(0)};
    for (int i = i_first; i < n4; i += 4 * gridDim.x * BS) {
        A wv[4], vv[4], nv[4] = {A(0), A(0), A(0), A(0)};
        if (i == i_first) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                wv[r] = pw.template at<A>(r);
                vv[r] = pv.template at<A>(r);
                nv[r] = last ? A(0) : pn.template at<A>(r);
            }
        } else {
            Row4<T>::load(w + i, wv);
            Row4<T>::load(vj + i, vv);
            if (!last) Row4<T>::load(vn + i, nv);
        }
        T wo[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            T wi = (T)wv[r];
            wi -= h * (T)vv[r];
            wo[r] = wi;
            acc[0] += last ? (A)wi * (A)wi : nv[r] * (A)wi;
        }
        Row4<T>::store(w + i, wo);
    }
    for (int i = n4 + blockIdx.x * BS + threadIdx.x; i < n; i += gridDim.x * BS) {
        T wi = w[i];
        wi -= h * vj[i];
        w[i] = wi;
        acc[0] += last ? (A)wi * (A)wi : (A)vn[i] * (A)wi;
    }
    store_partials<1, BS>(acc, 1, partial);
}

#pragma clang fp contract(off)
// upper-triangular solve y = H(0:k,0:k)^-1 s(0:k), in place on s (one lane per
// row of the axpy sweep; k <= m is small)
template <class T>
__global__ __launch_bounds__(kBlock) void k_trsv_upper(int k, int ldh, const T* __restrict__ H, T* __restrict__ y) {
    __shared__ T ys[1024];
    __shared__ T temp_s;
    for (int i = threadIdx.x; i < k; i += kBlock) ys[i] = y[i];
    __syncthreads();
    for (int j = k - 1; j >= 0; --j) {
        if (threadIdx.x == 0) {
            T yj = ys[j];
            if (yj != T(0)) yj = yj / H[(int64_t)j * ldh + j];
            ys[j] = yj;
            temp_s = yj;
        }
        __syncthreads();
        const T t = temp_s;
        if (t != T(0))
            for (int i = threadIdx.x; i < j; i += kBlock) ys[i] = ys[i] - t * H[(int64_t)j * ldh + i];
        __syncthreads();
    }
    for (int i = threadIdx.x; i < k; i += kBlock) y[i] = ys[i];
}
// The same solve for 64 < k <= 64 * KW by one wave64 (GMRES(100): the
// one-lane-per-step form above took 92.6 us at k = 100, one workgroup barrier
// pair per column). The upper triangle of H(0:k,0:k) is staged in LDS packed
// by columns (column j at j(j+1)/2, dynamic shared memory) with one load
// round; lane l holds y_{l + 64q} in register slot q. The column sweep is
// the netlib order of k_trsv_upper (no contraction): y_j /= H(j,j) (when
// y_j != 0), broadcast by a shuffle, then y_i -= y_j H(i,j) for i < j.
// (kBlock threads stage H, 8 independent loads per lane per round; wave 0 solves)
template <class T, int KW>
__global__ __launch_bounds__(kBlock) void k_trsv_upper_lds(int k, int ldh, const T* __restrict__ H,
                                                           T* __restrict__ y) {
    extern __shared__ char trsv_smem[];
    T* Hp = reinterpret_cast<T*>(trsv_smem);
    const int lane = threadIdx.x;
    const int P = k * (k + 1) / 2;
    constexpr int U = 8;
    for (int base = 0; base < P; base += kBlock * U) {
        T v[U];
        int e[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            e[u] = base + kBlock * u + (int)threadIdx.x;
            const int ec = e[u] < P ? e[u] : P - 1;
            // column j of packed entry ec: j(j+1)/2 <= ec < (j+1)(j+2)/2
            int j = (int)((sqrtf(8.0f * (float)ec + 1.0f) - 1.0f) * 0.5f);
            while (j * (j + 1) / 2 > ec) --j;
            while ((j + 1) * (j + 2) / 2 <= ec) ++j;
            v[u] = H[(int64_t)j * ldh + (ec - j * (j + 1) / 2)];
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (e[u] < P) Hp[e[u]] = v[u];
    }
    __syncthreads();
    if (threadIdx.x >= kWave) return;
    T yr[KW];
#pragma unroll
    for (int q = 0; q < KW; ++q) yr[q] = lane + kWave * q < k ? y[lane + kWave * q] : T(0);
    for (int j = k - 1; j >= 0; --j) {
        const int jq = j / kWave, jl = j % kWave;
        T mine = yr[0];
#pragma unroll
        for (int q = 1; q < KW; ++q)
            if (q == jq) mine = yr[q];
        T yj = __shfl(mine, jl, kWave);
        if (yj != T(0)) yj = yj / Hp[j * (j + 1) / 2 + j];
#pragma unroll
        for (int q = 0; q < KW; ++q) {
            const int i = lane + kWave * q;
            if (q == jq && lane == jl) yr[q] = yj;
            if (yj != T(0) && i < j) yr[q] = yr[q] - yj * Hp[j * (j + 1) / 2 + i];
        }
    }
#pragma unroll
    for (int q = 0; q < KW; ++q)
        if (lane + kWave * q < k) y[lane + kWave * q] = yr[q];
}

// The same upper solve by one wave64 (k <= 64): lane i holds y_i, the
// column sweep's scalar is broadcast with a shuffle, H(0:k,0:k) is in LDS
// (column j at Hs[j * 64]). No barrier inside the sweep.
template <class T>
__device__ __forceinline__ T trsv_upper_wave(int k, const T* Hs, T y, int lane) {
    for (int j = k - 1; j >= 0; --j) {
        T yj = __shfl(y, j, kWave);
        if (yj != T(0)) yj = yj / Hs[j * kWave + j];
        if (lane == j) y = yj;
        if (yj != T(0) && lane < j) y = y - yj * Hs[j * kWave + lane];
    }
    return y;
}
#pragma clang fp contract(on)

// x += X(T(V y)): mixed form gemv(1, V, y, 0, tmp); copy; axpy(1, tmp, x)
// (same-precision form gemv(1, V, y, 1, x) gives the same fl(t + x))
// SOLVE (k <= 64): y = H(0:k,0:k)^-1 s(0:k) is formed first by every
// workgroup (trsv_upper_wave) — one launch per restart instead of two. s is
// not overwritten (the next prologue resets it).
template <class T, class X, bool SOLVE, class A = double>
__global__ __launch_bounds__(kBlock) void k_update_x(int n, const T* __restrict__ V, int64_t ld, int k,
                                                     const T* __restrict__ y, const T* __restrict__ H, int ldh,
                                                     X* __restrict__ x) {
    __shared__ T ys[SOLVE ? kWave : 1024];
    if constexpr (SOLVE) {
        __shared__ T Hs[kWave * kWave];
        for (int e = threadIdx.x; e < k * kWave; e += kBlock) {
            const int j = e / kWave, i = e % kWave;
            Hs[e] = i <= j ? H[(int64_t)j * ldh + i] : T(0);
        }
        __syncthreads();
        if (threadIdx.x < kWave) {
            const int lane = threadIdx.x;
            T yv = lane < k ? y[lane] : T(0);
            yv = trsv_upper_wave(k, Hs, yv, lane);
            ys[lane] = yv;  // (s itself is left as is: every workgroup reads it)
        }
    } else {
        for (int j = threadIdx.x; j < k; j += kBlock) ys[j] = y[j];
    }
    __syncthreads();
    for (int i = blockIdx.x * kBlock + threadIdx.x; i < n; i += gridDim.x * kBlock) {
        A t = A(0);
        for (int j = 0; j < k; ++j) t += (A)V[(int64_t)j * ld + i] * (A)ys[j];
        x[i] = x[i] + (X)(T)t;
    }
}

// k_update_x<T, X, true> with the column count NC = k <= kNC a compile-time
// constant: each lane owns 4 rows and loads the basis in batches (the
// runtime-k form waited for every few columns in turn). Same arithmetic:
// t = sum_j V_ij y_j in fp64 in j order, x_i = x_i + X(T(t)).
template <class T, class X, int NC, class A = double>
__global__ __launch_bounds__(kCombineBlock) void k_update_x_nc(int n, const T* __restrict__ V, int64_t ld,
                                                                const T* __restrict__ y, const T* __restrict__ H,
                                                                int ldh, X* __restrict__ x) {
    static_assert(NC >= 1 && NC <= kNC, "one panel");
    constexpr int BS = kCombineBlock, B = kColBatch<T>;
    __shared__ T Hs[NC * kWave];
    __shared__ A ys[NC];
    for (int e = threadIdx.x; e < NC * kWave; e += BS) {
        const int j = e / kWave, i = e % kWave;
        Hs[e] = i <= j && i < NC ? H[(int64_t)j * ldh + i] : T(0);
    }
    __syncthreads();
    if (threadIdx.x < kWave) {
        const int lane = threadIdx.x;
        T yv = lane < NC ? y[lane] : T(0);
        yv = trsv_upper_wave(NC, Hs, yv, lane);
        if (lane < NC) ys[lane] = (A)yv;
    }
    __syncthreads();
    const int n4 = n & ~3;
    for (int i = 4 * (blockIdx.x * BS + threadIdx.x); i < n4; i += 4 * gridDim.x * BS) {
        Raw4<X> xr;
        xr.load(x + i);
        A t[4] = {A(0), A(0), A(0), A(0)};
#pragma unroll
        for (int c0 = 0; c0 < NC; c0 += B) {
            Raw4<T> v[B];
#pragma unroll
            for (int u = 0; u < B; ++u)
                if (c0 + u < NC) v[u].load(V + (int64_t)(c0 + u) * ld + i);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int u = 0; u < B; ++u)
                if (c0 + u < NC) {
                    const A yu = ys[c0 + u];
#pragma unroll
                    for (int r = 0; r < 4; ++r) t[r] += v[u].template at<A>(r) * yu;
                }
        }
        X xo[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) xo[r] = (X)xr[r] + (X)(T)t[r];
        Row4<X>::store(x + i, xo);
    }
    for (int i = n4 + blockIdx.x * BS + threadIdx.x; i < n; i += gridDim.x * BS) {
        A t = A(0);
#pragma unroll
        for (int j = 0; j < NC; ++j) t += (A)V[(int64_t)j * ld + i] * ys[j];
        x[i] = x[i] + (X)(T)t;
    }
}

}  // namespace

// ---------------------------------------------------------------- plan object
struct mpg_arnoldi {
    mpg_ctx* ctx = nullptr;
    mpg_arnoldi_desc d{};
    int combo = 0;    // type combination (see dispatch below)
    int G = 1;        // workgroups of the row-parallel panel kernels
    int Grb = 1;      // workgroups of the row-block (SpMV) kernels: one per row block
    int last_G = 1;   // partial count per column written by the last producer
    double* last_part = nullptr;  // ... and the buffer it wrote (partial or dpart)
    int64_t ld = 0;   // leading dimension of V (elements)
    size_t tsize = 8;
    void* V = nullptr;
    void* H = nullptr;      // (m+1) x m
    void* small = nullptr;  // cs, sn, s (m+1 each), inv, corr (m+1), coef scratch
    void* w[2] = {nullptr, nullptr};      // row 0 of each w buffer
    void* wbase[2] = {nullptr, nullptr};  // the allocations: `front` entries before row 0
    int front = 0;                        // MPG_FRONT_PAD(d.n_front)
    double* partial = nullptr;  // (kNC + 4) x G
    double* dpart = nullptr;    // kNC x Gd: one-panel dots partials (read by the CGS update that writes `partial`)
    double* sums = nullptr;     // m + 4
    double* report = nullptr;   // 4 + m
    unsigned* counters = nullptr;  // last-arriver tickets: [0] dots, [32] CGS + Givens (zeroed at create)
    int Gd = 1;                    // workgroups (kCombineBlock threads) of the combining panel dots
    SellCopy sell;  // sliced-ELL copy of the Arnoldi matrix (nslices == 0: CSR row blocks)
    SellCopy sell_outer;        // ... of the outer-precision values, for the residual prologue
    NodeCopy node;              // node-block copy of the Arnoldi matrix (nblk > 0: the Arnoldi SpMV uses it)
    // the residual prologue on node blocks (round 6): an fp64 node copy of the
    // outer values (or `node` itself when it holds them) and the fp64 row sums
    // A x it writes for k_prologue_rows; nullptr / empty: the CSR prologue
    NodeCopy node_outer;
    const NodeCopy* node_res = nullptr;
    double* rsum = nullptr;
    bool outer_is_inner = false;  // the prologue runs on `sell` (baseline / single modes)
    // SELL SpMV with the panel dots fused (SellDots): per-workgroup partials,
    // group tickets, group size and count
    double* fd_part = nullptr;
    unsigned* fd_cnt = nullptr;
    int fd_gs = 0, fd_ng = 0;
    // fp32 Arnoldi with fp32 accumulation (mpg_arnoldi_set_accum): the
    // launches go through arnoldi_acc32.hip's A = float instantiations
    bool acc32 = false;

    char* small_at(int slot) const { return static_cast<char*>(small) + (size_t)slot * (d.m + 1) * tsize; }
    void* cs() const { return small_at(0); }
    void* sn() const { return small_at(1); }
    void* s() const { return small_at(2); }
    void* corr() const { return small_at(3); }
    void* inv() const { return small_at(4); }
};

namespace {

// combos: 0 baseline <d,d,d,d>; 1 single-prec <d,d,f,d>; 2 single <f,f,f,f>;
//         3 mixed <f,d,f,f>; 4 mixed-half <f,d,f,h>
int combo_of(const mpg_arnoldi_desc& d) {
    if (d.vec_type == MPG_F64 && d.outer_type == MPG_F64 && d.inner_val == MPG_F64)
        return d.prec_type == MPG_F64 ? 0 : (d.prec_type == MPG_F32 ? 1 : -1);
    if (d.vec_type == MPG_F32 && d.prec_type == MPG_F32) {
        if (d.outer_type == MPG_F32 && d.inner_val == MPG_F32) return 2;
        if (d.outer_type == MPG_F64 && d.inner_val == MPG_F32) return 3;
        if (d.outer_type == MPG_F64 && d.inner_val == MPG_F16) return 4;
    }
    return -1;
}

template <class F>
int dispatch(int combo, F&& f) {
    switch (combo) {
        case 0: return f(double(), double(), double(), double());
        case 1: return f(double(), double(), float(), double());
        case 2: return f(float(), float(), float(), float());
        case 3: return f(float(), double(), float(), float());
        case 4: return f(float(), double(), float(), half_v());
        default: return MPG_ERR_UNSUPPORTED;
    }
}

// MPG_CSR_MODE (the Arnoldi CSR SpMV, k_step_spmv<..., MODE>): bit 0
// non-temporal matrix streams, bit 1 XCD-ordered row blocks
int csr_mode() {
    const char* e = std::getenv("MPG_CSR_MODE");
    return e && *e >= '0' && *e <= '4' ? *e - '0' : 0;
}

// Tiles per workgroup of the node-block SpMV (MPG_NODE_TPW: 1 one tile
// each, N > 1 a pipelined walk of N tiles; default 2; 0: as many as keep
// the grid at kNodeGroups workgroups, so the Givens step folds in).
// Measured (profiles/r05_node_ab.jsonl): fem27 248 / 218 / 215-228 / 223-238
// / 255 us at 1 / 2 / 4 / 8 / 16 (auto, folded: 247), C4's stencil 341 /
// 295-312 / 300 / 306-334 / 345 (auto 355): longer walks leave the grid's
// tail to fewer workgroups, two tiles in flight is the gain.
constexpr int kNodeGroups = 2048;
int node_tpw(const NodeCopy& S) {
    const int v = node_tpw_default();
    if (v >= 1) return v;
    return std::max(2, (S.ntiles + kNodeGroups - 1) / kNodeGroups);
}

int row_grid(const mpg_arnoldi* a) { return a->G; }
int rb_grid(const mpg_arnoldi* a) { return a->Grb; }

template <class T>
GivensArgs<T> givens_args(const mpg_arnoldi* a, int k) {
    return GivensArgs<T>{k,
                         a->d.m,
                         a->d.orth == kOrthCGSR ? static_cast<const T*>(a->corr()) : nullptr,
                         static_cast<T*>(a->H),
                         static_cast<T*>(a->cs()),
                         static_cast<T*>(a->sn()),
                         static_cast<T*>(a->s()),
                         static_cast<T*>(a->inv()),
                         a->report};
}

}  // namespace
