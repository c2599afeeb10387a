// Sliced-ELL (SELL-64) copy of a CSR matrix for the Arnoldi SpMV.
//
// A slice is 64 consecutive rows = one wave64; lane l owns row 64 s + l.
// The slice is padded to its longest row, rounded up to W, and stored as
// steps of W entries per lane, lane-major inside a step:
//
//   element j of row 64 s + l  ->  off[s] + (j / W) * 64 W + l W + (j % W)
//
// so one wave-wide W-vector load per step moves 64 W contiguous entries
// and needs no LDS, no segmented reduction and no row pointers. Columns are
// int32, or int16 deltas against the slice's first row when every entry of
// the matrix is within +-32767 of it (banded/stencil matrices: half the
// index bytes). Padding carries a sentinel column and is skipped, so an
// Inf/NaN in x never meets a padded zero. Within a row the entries keep CSR
// order and the fp64 sum runs in that order.
#pragma once

#include "internal.hpp"
#include "csr_tile.hpp"

#include <type_traits>

namespace mpg {

template <class CI> struct SellCol;
template <> struct SellCol<int32_t> {
    static constexpr int32_t kPad = -1;
    static __device__ __forceinline__ bool live(int32_t c) { return c >= 0; }
    static __device__ __forceinline__ int decode(int32_t c, int /*row0*/) { return c; }
};
template <> struct SellCol<int16_t> {
    static constexpr int16_t kPad = INT16_MIN;
    static __device__ __forceinline__ bool live(int16_t c) { return c != INT16_MIN; }
    static __device__ __forceinline__ int decode(int16_t c, int row0) { return row0 + (int)c; }
};

// raw storage of a value type inside the slices
template <class V> struct SellStore { using type = V; };
template <> struct SellStore<half_v> { using type = uint16_t; };

template <class S> __device__ __forceinline__ double widen(S v) { return (double)v; }
template <> __device__ __forceinline__ double widen<uint16_t>(uint16_t v) { return (double)to_float(v); }

// Cache policy of the slices (MPG_SELL_NT=1: non-temporal loads)
#ifndef MPG_SELL_NT
#define MPG_SELL_NT 0
#endif

// W consecutive elements with one aligned vector load (NT: non-temporal)
template <class S, int W, bool NT = (MPG_SELL_NT != 0)> struct VecW {
    typedef S vtype __attribute__((ext_vector_type(W)));
    static __device__ __forceinline__ void load(const S* p, S (&o)[W]) {
        const vtype v = ld_policy<NT>(reinterpret_cast<const vtype*>(p));
#pragma unroll
        for (int e = 0; e < W; ++e) o[e] = v[e];
    }
};
template <class S, bool NT> struct VecW<S, 1, NT> {
    static __device__ __forceinline__ void load(const S* p, S (&o)[1]) { o[0] = ld_policy<NT>(p); }
};

// entries per lane per batch: every load of a batch is issued before its
// gathers, so a row of up to kSellBatch entries costs one load round trip
#ifndef MPG_SELL_BATCH
#define MPG_SELL_BATCH 16
#endif
constexpr int kSellBatch = MPG_SELL_BATCH;
template <int W> constexpr int sell_unroll() { return W >= kSellBatch ? 1 : kSellBatch / W; }

// fp64 row sum of row 64 s + lane (lane valid or not: all lanes take part).
template <class S, class CI, int W, class XF>
__device__ __forceinline__ double sell_row_sum(int s, int lane, const int64_t* __restrict__ off,
                                               const CI* __restrict__ col, const S* __restrict__ val, XF xval) {
    constexpr int U = sell_unroll<W>();
    const int64_t o = off[s];
    const int steps = (int)((off[s + 1] - o) / (kWave * W));
    const int row0 = s * kWave;
    const CI* __restrict__ cp = col + o + lane * W;
    const S* __restrict__ vp = val + o + lane * W;
    double acc = 0.0;
    for (int q = 0; q < steps; q += U) {
        CI c[U][W];
        S v[U][W];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (q + u < steps) {
                VecW<CI, W>::load(cp + (int64_t)(q + u) * kWave * W, c[u]);
                VecW<S, W>::load(vp + (int64_t)(q + u) * kWave * W, v[u]);
            } else {
#pragma unroll
                for (int e = 0; e < W; ++e) c[u][e] = SellCol<CI>::kPad;
            }
        }
        double x[U][W];
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int e = 0; e < W; ++e)
                x[u][e] = SellCol<CI>::live(c[u][e]) ? xval(SellCol<CI>::decode(c[u][e], row0)) : 0.0;
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int e = 0; e < W; ++e)
                if (SellCol<CI>::live(c[u][e])) acc += widen(v[u][e]) * x[u][e];
    }
    return acc;
}

// The same row sum split into load and sum halves, so a kernel can issue a
// batch of slice loads early (before loads it needs sooner have returned,
// or before a barrier) and consume it later. Loads are unconditional: steps
// past the slice's width re-read its last step (cache hits) and are masked
// by step index at use, so nothing widens or selects a loaded value at load
// time (which would wait for it on the spot). An empty slice points at
// offset 0 of the arrays.
// NT: non-temporal slice loads (a pass that runs once per restart cycle, so
// the slices the Arnoldi steps re-read stay in the Infinity Cache)
template <class S, class CI, int W, bool NT = (MPG_SELL_NT != 0)>
struct SellRow {
    static constexpr int U = sell_unroll<W>();
    CI c[U][W];
    S v[U][W];
    int steps, row0;
    const CI* __restrict__ cp;
    const S* __restrict__ vp;

    int64_t o0, o1;
    // the slice's offsets: issue first (everything else needs them), use later
    __device__ __forceinline__ void init_load(int s, const int64_t* __restrict__ off) {
        o0 = off[s];
        o1 = off[s + 1];
        row0 = s * kWave;
    }
    __device__ __forceinline__ void init_finish(int lane, const CI* __restrict__ col, const S* __restrict__ val) {
        steps = (int)((o1 - o0) / (kWave * W));
        const int64_t base = steps > 0 ? o0 + lane * W : 0;
        cp = col + base;
        vp = val + base;
    }
    __device__ __forceinline__ void init(int s, int lane, const int64_t* __restrict__ off, const CI* __restrict__ col,
                                         const S* __restrict__ val) {
        init_load(s, off);
        init_finish(lane, col, val);
    }
    __device__ __forceinline__ void load(int q) {
        const int last = steps > 0 ? steps - 1 : 0;
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int qq = q + u < last ? q + u : last;
            VecW<CI, W, NT>::load(cp + (int64_t)qq * kWave * W, c[u]);
            VecW<S, W, NT>::load(vp + (int64_t)qq * kWave * W, v[u]);
        }
    }
    // acc += the batch loaded at step q, in CSR order. Every gather is issued
    // (padding and steps past the width read x at row0, a valid index) and
    // masked at the sum, so the gathers of a batch are in flight together.
    template <class XF>
    __device__ __forceinline__ void sum(int q, XF xval, double& acc) const {
        double x[U][W];
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int e = 0; e < W; ++e)
                x[u][e] = xval(SellCol<CI>::live(c[u][e]) ? SellCol<CI>::decode(c[u][e], row0) : row0);
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int e = 0; e < W; ++e)
                if (q + u < steps && SellCol<CI>::live(c[u][e])) acc += widen(v[u][e]) * x[u][e];
    }
};

// LDS window of x for a slice (SELL SpMVs): every column of every slice
// within [row0 - kWinLo, row0 + 64 + kWinHi) lets the gathers read LDS
constexpr int kWinLo = 64, kWinHi = 64, kWinLen = kWinLo + kWave + kWinHi;

// A SELL-64 copy of one CSR value array (device memory owned by the copy).
// nslices == 0: no copy (the CSR storage runs).
struct SellCopy {
    int n = 0, nslices = 0, W = 1;
    int vtype = 0;     // mpg_dtype_t of the stored values (MPG_F64 | MPG_F32 | MPG_F16)
    bool c16 = false;  // int16 slice-relative columns
    bool win = false;  // every slice's columns inside the LDS window
    int64_t padded = 0;
    int64_t* off = nullptr;
    void* col = nullptr;
    void* val = nullptr;
};

// Build the copy from the CSR structure and `val` (vtype; F16 = raw IEEE
// half bits). format: 0 auto (only when padding adds <= 20 % to the stored
// entries), 1 never, 2 always. Synchronises the context's stream.
int sell_build(mpg_ctx* ctx, const mpg_csr* A, int vtype, const void* val, int format, SellCopy& S);
void sell_free(SellCopy& S);

// f(column type, integral_constant<int, W>) for the copy's layout
template <class F>
int sell_dispatch(int W, bool c16, F&& f) {
    auto with_w = [&](auto ci) {
        switch (W) {
            case 1: return f(ci, std::integral_constant<int, 1>());
            case 2: return f(ci, std::integral_constant<int, 2>());
            case 4: return f(ci, std::integral_constant<int, 4>());
            default: return (int)MPG_ERR_UNSUPPORTED;
        }
    };
    return c16 ? with_w(int16_t()) : with_w(int32_t());
}
template <class F>
int sell_dispatch_win(bool win, F&& f) {
    return win ? f(std::true_type()) : f(std::false_type());
}

}  // namespace mpg
