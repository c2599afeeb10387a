// Building blocks of the tall-skinny panel kernels (V^T w dots, V c
// updates) shared by the fused Arnoldi cycle (arnoldi.hip) and the operator
// surface's gemv (blas2.hip): 16-B row quads, the butterfly block reduction
// to per-workgroup partials, compile-time column batching.
#ifndef MPGMRES_PANEL_HPP
#define MPGMRES_PANEL_HPP

#include "handoff.hpp"
#include "internal.hpp"

namespace mpg {

// One transpose round on the first 2H accumulators: lanes with the MASK bit
// set keep the upper half, the others the lower half; recursion keeps every
// index a compile-time constant (a runtime index sends acc to scratch).
template <int H, int MASK, int N, class A>
__device__ __forceinline__ void butterfly_round(A (&acc)[N], int lane) {
    if constexpr (H >= 1) {
        const bool upper = (lane & MASK) != 0;
#pragma unroll
        for (int i = 0; i < H; ++i) {
            const A keep = upper ? acc[i + H] : acc[i];
            const A send = upper ? acc[i] : acc[i + H];
            acc[i] = keep + __shfl_xor(send, MASK, kWave);
        }
        butterfly_round<H / 2, MASK / 2>(acc, lane);
    }
}

// Block-reduce NCOL accumulators (fp64, or fp32 under the fp32
// accumulation class: every add of the trees below rounds to fp32) and store
// them as partial[c*G + blk] (fp64 storage; write-through when WT: the
// last-arriver combine reads them).
//
// Wave stage = transpose (butterfly) reduction: in round r every lane trades
// half of its remaining columns with the lane 32>>r away and keeps the sum
// of the other half, so after log2(NCOL) rounds lane l holds one column
// (l >> (6 - log2 NCOL)) summed over 2^rounds lanes; plain xor shuffles
// finish the remaining lanes. 32 columns cost 32 shuffles instead of the
// 192 of one 6-level reduction per column. Fixed order: deterministic.
template <int NCOL, int BS = kBlock, bool WT = false, class A>
__device__ __forceinline__ void store_partials(A (&acc)[NCOL], int ncols, double* __restrict__ partial) {
    static_assert((NCOL & (NCOL - 1)) == 0 && NCOL <= 32, "NCOL: power of two <= 32");
    __shared__ A red[BS / kWave][NCOL];
    const int lane = threadIdx.x & (kWave - 1), wid = threadIdx.x / kWave;
    constexpr int rounds = NCOL == 1 ? 0 : NCOL == 2 ? 1 : NCOL == 4 ? 2 : NCOL == 8 ? 3 : NCOL == 16 ? 4 : 5;
    butterfly_round<NCOL / 2, 32>(acc, lane);
    A v = acc[0];
#pragma unroll
    for (int mask = 32 >> rounds; mask >= 1; mask >>= 1) v += __shfl_xor(v, mask, kWave);
    constexpr int shift = 6 - rounds;
    if ((lane & ((1 << shift) - 1)) == 0) red[wid][lane >> shift] = v;
    __syncthreads();
    for (int c = threadIdx.x; c < ncols; c += BS) {
        A s = A(0);
#pragma unroll
        for (int w = 0; w < BS / kWave; ++w) s += red[w][c];
        if (WT) store_wt(partial + (size_t)c * gridDim.x + blockIdx.x, (double)s);
        else partial[(size_t)c * gridDim.x + blockIdx.x] = (double)s;
    }
}

// 4 consecutive entries (i a multiple of 4, 16-B aligned for fp32) widened to
// the accumulation type (fp64, or fp32 for an fp32 basis)
template <class T> struct Row4;
template <> struct Row4<float> {
    template <class A>
    static __device__ __forceinline__ void load(const float* p, A (&o)[4]) {
        const float4 v = *reinterpret_cast<const float4*>(p);
        o[0] = v.x; o[1] = v.y; o[2] = v.z; o[3] = v.w;
    }
    static __device__ __forceinline__ void store(float* p, const float (&o)[4]) {
        *reinterpret_cast<float4*>(p) = make_float4(o[0], o[1], o[2], o[3]);
    }
};
template <> struct Row4<double> {
    static __device__ __forceinline__ void load(const double* p, double (&o)[4]) {
        const double2 a = *reinterpret_cast<const double2*>(p);
        const double2 b = *reinterpret_cast<const double2*>(p + 2);
        o[0] = a.x; o[1] = a.y; o[2] = b.x; o[3] = b.y;
    }
    static __device__ __forceinline__ void store(double* p, const double (&o)[4]) {
        *reinterpret_cast<double2*>(p) = make_double2(o[0], o[1]);
        *reinterpret_cast<double2*>(p + 2) = make_double2(o[2], o[3]);
    }
};

template <int N> struct Pow2Ceil {
    static constexpr int v = N <= 1 ? 1 : N <= 2 ? 2 : N <= 4 ? 4 : N <= 8 ? 8 : N <= 16 ? 16 : 32;
};
// columns per load batch: 32 VGPRs of raw column data per batch
template <class T> constexpr int kColBatch = sizeof(T) == 4 ? 8 : 4;

// 4 consecutive entries kept in their storage type until used (a batch of
// raw loads costs half the registers of widened fp32 values)
template <class T> struct Raw4;
template <> struct Raw4<float> {
    float4 v;
    __device__ __forceinline__ void load(const float* p) { v = *reinterpret_cast<const float4*>(p); }
    __device__ __forceinline__ double operator[](int r) const {
        return (double)(r == 0 ? v.x : r == 1 ? v.y : r == 2 ? v.z : v.w);
    }
    // the entry in the accumulation type (exact either way)
    template <class A> __device__ __forceinline__ A at(int r) const {
        return (A)(r == 0 ? v.x : r == 1 ? v.y : r == 2 ? v.z : v.w);
    }
};
template <> struct Raw4<double> {
    double2 a, b;
    __device__ __forceinline__ void load(const double* p) {
        a = *reinterpret_cast<const double2*>(p);
        b = *reinterpret_cast<const double2*>(p + 2);
    }
    __device__ __forceinline__ double operator[](int r) const { return r == 0 ? a.x : r == 1 ? a.y : r == 2 ? b.x : b.y; }
    template <class A> __device__ __forceinline__ A at(int r) const { return (A)(*this)[r]; }
};

}  // namespace mpg

#endif  // MPGMRES_PANEL_HPP
