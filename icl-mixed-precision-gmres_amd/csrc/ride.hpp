// What rides in an operator-surface SpMV launch (sell.hip, node.hip): the
// previous Arnoldi step's Givens scalar program in one extra workgroup, and
// add_vector's normalisation (Orthogonalization.hpp:51-60) of the vector the
// SpMV multiplies.
#pragma once

#include "internal.hpp"

namespace mpg {

constexpr int kProgStage = 64;  // rot_vec rotations staged per pass by a riding scalar program

// NORM (round 5): the operator surface's add_vector normalisation riding the
// next Arnoldi SpMV (kernels_hip.cpp). x is w (in a scratch copy: the SpMV
// writes its own w); every workgroup sums the <= 256 ||w||^2 partials the
// fused CGS gemv left in the workspace with block_sum<kBlock> (the bits of
// k_consume_partials' block_sum<1024>: the extra lanes add exact zeros, in
// the same sequential wave order), forms r = T(sqrt(s)) and a = T(1) / r
// (k_consume_partials, blas1.hip), gathers T(a x_c) -- scal_recip's
// product -- stores v = T(a x_i) for its own rows, and workgroup 0 stores
// h = r before any riding scalar program (which reads it) runs.
template <class X>
struct NormArgs {
    const double* part = nullptr;
    int nparts = 0;
    X* h = nullptr;
    X* v = nullptr;
};

// a = T(1) / T(sqrt(sum of the partials)), the same in every lane; workgroup
// 0's thread 0 stores r to *h first. Every thread of the workgroup calls it.
template <class X>
__device__ __forceinline__ X norm_scale(const NormArgs<X>& nm, double pv) {
    __shared__ double scratch[kBlock / kWave];
    __shared__ X a_s;
    const double s = block_sum<kBlock>(pv, scratch);
    if (threadIdx.x == 0) {
        const X r = (X)sqrt(s);
        if (blockIdx.x == 0) {
            *nm.h = r;
            __threadfence();  // the riding program reads h(k+1,k)
        }
        a_s = X(1) / r;
    }
    __syncthreads();
    return a_s;
}

// norm_scale with LDS-only barriers (lds_barrier), for a kernel that has
// issued global loads it does not want drained yet (k_node_spmv: the first
// tile's records and raw x gathers are in flight while the workgroup sums the
// partials; a __syncthreads would wait for them first -- C4's node SpMV ran
// 360 us with the plain form against 290 us without the ride). The same
// block_sum<kBlock> order (wave sums, then thread 0 adds them in wave
// order), the same bits. scratch: kBlock / kWave doubles; a_s: one X.
template <class X>
__device__ __forceinline__ X norm_scale_lds(const NormArgs<X>& nm, double pv, double* scratch, X* a_s) {
    const int lane = threadIdx.x & (kWave - 1), wid = threadIdx.x / kWave;
    const double v = wave_sum(pv);
    if (lane == 0) scratch[wid] = v;
    lds_barrier();
    if (threadIdx.x == 0) {
        double s = 0;
#pragma unroll
        for (int w = 0; w < kBlock / kWave; ++w) s += scratch[w];
        const X r = (X)sqrt(s);
        if (blockIdx.x == 0) {
            *nm.h = r;
            __threadfence();  // the riding program reads h(k+1,k)
        }
        *a_s = X(1) / r;
    }
    lds_barrier();
    return *a_s;
}

}  // namespace mpg
