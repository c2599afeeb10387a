// CSR-adaptive row-block tile, shared by the stand-alone SpMV (spmv.hip) and
// the fused Arnoldi phases (arnoldi.hip).
//
// A row block is either a run of short rows holding at most kNnzCap
// nonzeros (stream mode) or one row (row mode). Stream mode loads the
// block's (col, val) pairs with 16-byte vector loads — the block start is
// rounded down to a 4-element boundary and the extra lanes are masked — and
// issues every load of a lane before its first use: two int4 column loads,
// the matching value loads, then all eight gathers of x. The fp64 products
// land in LDS, one lane per row then sums its segment in column order.
#pragma once

#include "internal.hpp"

namespace mpg {

constexpr int kNnzCap = 2040;                       // nnz per stream-mode row block
constexpr int kRowCap = 2048;                       // rows per stream-mode row block
constexpr int kTileVec = (kNnzCap + 3) / 4 + 1;     // 16-B index vectors per tile (<= 512)
constexpr int kVecPerLane = (kTileVec + kBlock - 1) / kBlock;  // = 2

struct half_v {
    uint16_t bits;
};

// Cache policy of the matrix streams (col + val): NT loads them
// non-temporally, so a once-per-cycle CSR pass (the fp64 residual of the
// fused engine's prologue) does not displace the Krylov basis and the
// Arnoldi matrix from the Infinity Cache (+2 % GMRES it/s on BAND-10M,
// tools/policy_experiment.sh). MPG_CSR_NT=1 forces it for every CSR tile.
#ifndef MPG_CSR_NT
#define MPG_CSR_NT 0
#endif
typedef int i32x4_t __attribute__((ext_vector_type(4)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));
typedef double f64x2_t __attribute__((ext_vector_type(2)));
typedef unsigned short u16x4_t __attribute__((ext_vector_type(4)));

template <bool NT, class V> __device__ __forceinline__ V ld_policy(const V* p) {
    if constexpr (NT) return __builtin_nontemporal_load(p);
    else return *p;
}
template <bool NT, class V> __device__ __forceinline__ V ld_mat(const V* p) {
    return ld_policy<NT || MPG_CSR_NT != 0>(p);
}

// 4 consecutive values (element index i, a multiple of 4) widened to fp64
template <class V> struct Vec4Load;
template <> struct Vec4Load<float> {
    template <bool NT = false>
    static __device__ __forceinline__ void load(const float* p, int64_t i, double (&o)[4]) {
        const f32x4_t v = ld_mat<NT>(reinterpret_cast<const f32x4_t*>(p + i));
        o[0] = v.x; o[1] = v.y; o[2] = v.z; o[3] = v.w;
    }
};
template <> struct Vec4Load<double> {
    template <bool NT = false>
    static __device__ __forceinline__ void load(const double* p, int64_t i, double (&o)[4]) {
        const f64x2_t a = ld_mat<NT>(reinterpret_cast<const f64x2_t*>(p + i));
        const f64x2_t b = ld_mat<NT>(reinterpret_cast<const f64x2_t*>(p + i + 2));
        o[0] = a.x; o[1] = a.y; o[2] = b.x; o[3] = b.y;
    }
};
template <> struct Vec4Load<half_v> {
    template <bool NT = false>
    static __device__ __forceinline__ void load(const half_v* p, int64_t i, double (&o)[4]) {
        const u16x4_t v = ld_mat<NT>(reinterpret_cast<const u16x4_t*>(p + i));
        o[0] = to_float(v.x); o[1] = to_float(v.y); o[2] = to_float(v.z); o[3] = to_float(v.w);
    }
};
template <> struct Vec4Load<uint16_t> {
    template <bool NT = false>
    static __device__ __forceinline__ void load(const uint16_t* p, int64_t i, double (&o)[4]) {
        const u16x4_t v = ld_mat<NT>(reinterpret_cast<const u16x4_t*>(p + i));
        o[0] = to_float(v.x); o[1] = to_float(v.y); o[2] = to_float(v.z); o[3] = to_float(v.w);
    }
};

template <class V>
__device__ __forceinline__ double scalar_val(const V* p, int64_t i) { return (double)p[i]; }
template <>
__device__ __forceinline__ double scalar_val<half_v>(const half_v* p, int64_t i) { return (double)to_float(p[i].bits); }
template <>
__device__ __forceinline__ double scalar_val<uint16_t>(const uint16_t* p, int64_t i) { return (double)to_float(p[i]); }

// Stage the fp64 products val[i] * xval(col[i]) for i in [s, e) into prod[i - s].
// nnz_total bounds the vector loads at the end of the arrays.
template <bool NT = false, class V, class XF>
__device__ __forceinline__ void stage_products(int s, int e, int64_t nnz_total, const int32_t* __restrict__ col,
                                               const V* __restrict__ val, XF xval, double* __restrict__ prod) {
    const int base = s & ~3;
    int4 c[kVecPerLane];
    double v[kVecPerLane][4];
    bool live[kVecPerLane];
#pragma unroll
    for (int u = 0; u < kVecPerLane; ++u) {
        const int idx = base + 4 * (threadIdx.x + u * kBlock);
        live[u] = idx < e;
        if (live[u]) {
            if (idx + 3 < nnz_total) {
                const i32x4_t cv = ld_mat<NT>(reinterpret_cast<const i32x4_t*>(col + idx));
                c[u] = make_int4(cv.x, cv.y, cv.z, cv.w);
                Vec4Load<V>::template load<NT>(val, idx, v[u]);
            } else {
                int cc[4];
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const bool in = idx + q < nnz_total;
                    cc[q] = in ? col[idx + q] : 0;
                    v[u][q] = in ? scalar_val(val, idx + q) : 0.0;
                }
                c[u] = make_int4(cc[0], cc[1], cc[2], cc[3]);
            }
        }
    }
    double x[kVecPerLane][4];
#pragma unroll
    for (int u = 0; u < kVecPerLane; ++u) {
        const int idx = base + 4 * (threadIdx.x + u * kBlock);
        const int cc[4] = {c[u].x, c[u].y, c[u].z, c[u].w};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int i = idx + q;
            x[u][q] = (live[u] && i >= s && i < e) ? xval(cc[q]) : 0.0;
        }
    }
#pragma unroll
    for (int u = 0; u < kVecPerLane; ++u) {
        const int idx = base + 4 * (threadIdx.x + u * kBlock);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int i = idx + q;
            if (live[u] && i >= s && i < e) prod[i - s] = v[u][q] * x[u][q];
        }
    }
}

// 4 consecutive values kept in their storage type until used (a raw load
// into its final registers is not waited for until a consumer reads it)
template <class V> struct RawVal4;
template <> struct RawVal4<double> {
    f64x2_t a, b;
    template <bool NT> __device__ __forceinline__ void load(const double* p, int64_t i) {
        a = ld_mat<NT>(reinterpret_cast<const f64x2_t*>(p + i));
        b = ld_mat<NT>(reinterpret_cast<const f64x2_t*>(p + i + 2));
    }
    __device__ __forceinline__ double operator[](int q) const { return q == 0 ? a.x : q == 1 ? a.y : q == 2 ? b.x : b.y; }
};
template <> struct RawVal4<float> {
    f32x4_t v;
    template <bool NT> __device__ __forceinline__ void load(const float* p, int64_t i) {
        v = ld_mat<NT>(reinterpret_cast<const f32x4_t*>(p + i));
    }
    __device__ __forceinline__ double operator[](int q) const {
        return (double)(q == 0 ? v.x : q == 1 ? v.y : q == 2 ? v.z : v.w);
    }
};
template <> struct RawVal4<uint16_t> {
    u16x4_t v;
    template <bool NT> __device__ __forceinline__ void load(const uint16_t* p, int64_t i) {
        v = ld_mat<NT>(reinterpret_cast<const u16x4_t*>(p + i));
    }
    __device__ __forceinline__ double operator[](int q) const {
        return (double)to_float(q == 0 ? v.x : q == 1 ? v.y : q == 2 ? v.z : v.w);
    }
};
template <> struct RawVal4<half_v> : RawVal4<uint16_t> {
    template <bool NT> __device__ __forceinline__ void load(const half_v* p, int64_t i) {
        RawVal4<uint16_t>::load<NT>(reinterpret_cast<const uint16_t*>(p), i);
    }
};

// stage_products for a block whose every 16-B vector lies inside the arrays
// (e + 3 < nnz_total): every lane's loads are unconditional, at an address
// clamped to the block's last vector, and every gather uses a loaded column
// (an entry of the matrix, so a valid index); positions outside [s, e) are
// masked at the store. Nothing is waited for until all loads are in flight
// (a guarded load is widened or copied inside its branch, i.e. waited for
// there).
template <bool NT, class V, class XF>
__device__ __forceinline__ void stage_products_interior(int s, int e, const int32_t* __restrict__ col,
                                                        const V* __restrict__ val, XF xval,
                                                        double* __restrict__ prod) {
    const int base = s & ~3;
    const int lastv = (e - 1) & ~3;
    i32x4_t c[kVecPerLane];
    RawVal4<V> v[kVecPerLane];
#pragma unroll
    for (int u = 0; u < kVecPerLane; ++u) {
        const int idx = base + 4 * (threadIdx.x + u * kBlock);
        const int idc = idx < lastv ? idx : lastv;
        c[u] = ld_mat<NT>(reinterpret_cast<const i32x4_t*>(col + idc));
        v[u].template load<NT>(val, idc);
    }
    __builtin_amdgcn_sched_barrier(0);
    double x[kVecPerLane][4];
#pragma unroll
    for (int u = 0; u < kVecPerLane; ++u)
#pragma unroll
        for (int q = 0; q < 4; ++q) x[u][q] = xval(c[u][q]);
#pragma unroll
    for (int u = 0; u < kVecPerLane; ++u) {
        const int idx = base + 4 * (threadIdx.x + u * kBlock);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int i = idx + q;
            if (i >= s && i < e) prod[i - s] = v[u][q] * x[u][q];
        }
    }
}

// Row sums of one row block: epi(row, sum, pre(row)) is called once per
// row (the sum in the accumulation class A: fp64, or fp32 -- mac / add_prod,
// internal.hpp). pre(row) loads the row's epilogue operands; for this lane's
// first row it is issued ahead of the tile, so its latency hides under the
// tile's.
template <bool NT = false, class A = double, class V, class XF, class PF, class EPI>
__device__ __forceinline__ void csr_row_block(int r0, int r1, int s, int e, const int32_t* __restrict__ rowptr,
                                              const int32_t* __restrict__ col, const V* __restrict__ val,
                                              int64_t nnz_total, XF xval, PF pre, EPI epi, double* prod,
                                              double* scratch) {
    // s, e = rowptr[r0], rowptr[r1] (the analysis' nnz starts of the block).
    // Row mode (strided lanes, a tree sum) only for a row the stream mode
    // cannot stage: a short row that mpg_csr_create left alone in its block
    // (the next row is long, or it is the matrix's last) is summed in CSR
    // order like every other short row, so the SELL and node-block copies,
    // which sum every row in that order, keep giving its bits.
    if (r1 - r0 == 1 && e - s > kNnzCap) {
        A acc = A(0);
        for (int i = s + threadIdx.x; i < e; i += kBlock) mac(acc, scalar_val(val, i), xval(col[i]));
        const A sum = block_sum<kBlock>(acc, reinterpret_cast<A*>(scratch));
        if (threadIdx.x == 0) epi(r0, sum, pre(r0));
        __syncthreads();  // the row's outputs are visible to the whole workgroup
        return;
    }
    // this lane's first row: bounds and epilogue operands, loaded ahead of the tile
    const int rf = r0 + (threadIdx.x < r1 - r0 ? threadIdx.x : 0);
    const int ra = rowptr[rf], rz = rowptr[rf + 1];
    const auto pf = pre(rf);
    __builtin_amdgcn_sched_barrier(0);
    if (e > s && (int64_t)e + 3 < nnz_total) stage_products_interior<NT>(s, e, col, val, xval, prod);
    else stage_products<NT>(s, e, nnz_total, col, val, xval, prod);
    __syncthreads();
    for (int r = threadIdx.x; r < r1 - r0; r += kBlock) {
        const bool first = r == threadIdx.x;
        const int a = (first ? ra : rowptr[r0 + r]) - s;
        const int z = (first ? rz : rowptr[r0 + r + 1]) - s;
        A acc = A(0);
        for (int j = a; j < z; ++j) add_prod(acc, prod[j]);
        epi(r0 + r, acc, first ? pf : pre(r0 + r));
    }
    __syncthreads();
}

}  // namespace mpg
