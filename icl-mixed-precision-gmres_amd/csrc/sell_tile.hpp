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
// stored in one of three forms (the first that fits):
//   int16_t   c - row0, when every entry of the matrix is within +-32767 of
//             its slice's first row (banded matrices, 7-point stencils);
//   uint16_t  "stepped": the int16 bits of c - (row0 + lane) - base[s][j][e]
//             for element e of step j, with one int32 base per (slice, step,
//             element) (sbase, at index (off[s] / (64 W) + j) W + e): element
//             e of step j of all 64 rows of a slice is, for a stencil in
//             natural order, one neighbour offset +- a few, so wide stencils
//             (the 27-point 3-dof Queen stand-in: offsets up to +-37,299)
//             still store 2-B columns, plus 4 B per 64 entries. A slice where
//             some (step, element) spreads wider (rows on both sides of a
//             boundary plane) gets spat[s] = -2 - e (e: its ordinal
//             among such slices) and its rows are summed from the copy's
//             own CSR of those rows (xrp/xcol/xval, row 64 e + lane) in the
//             same order (same bits);
//   int32_t   c.
// Implicit slices: a slice whose 64 rows all have the same column offsets
// c - row in the same order (every interior slice of a banded matrix) reads
// its columns from a shared pattern instead: spat[s] >= 0 indexes a W-per-step
// run of lane-relative offsets in `pat` that every lane of the wave loads
// (the same address: one cache line), decoded against the lane's own row.
// Identical patterns are stored once, so BAND-10M's 20 MB of int16 columns
// become one 10-entry pattern. spat[s] = -1: stored columns; <= -2 (stepped
// form): the slice is summed from the copy's sub-CSR (below).
// Padding carries a sentinel column and is skipped, so an Inf/NaN in x never
// meets a padded zero. Within a row the entries keep CSR order and the fp64
// sum runs in that order.
#pragma once

#include "internal.hpp"
#include "csr_tile.hpp"

#include <cstdlib>
#include <type_traits>

namespace mpg {

// decode(c, rbase, lane_base): rbase = the row the stored offset is relative
// to (int16: the slice's first row; int32: 0, i.e. absolute; implicit
// patterns: the lane's own row); lane_base = row0 + lane + base (stepped)
template <class CI> struct SellCol;
template <> struct SellCol<int32_t> {
    static constexpr int32_t kPad = INT32_MIN;
    static constexpr bool stepped = false;
    static __device__ __forceinline__ bool live(int32_t c) { return c != INT32_MIN; }
    static __device__ __forceinline__ int decode(int32_t c, int rbase, int /*lane_base*/) { return rbase + c; }
    static __device__ __forceinline__ int stored_base(int /*row0*/) { return 0; }
};
template <> struct SellCol<int16_t> {
    static constexpr int16_t kPad = INT16_MIN;
    static constexpr bool stepped = false;
    static __device__ __forceinline__ bool live(int16_t c) { return c != INT16_MIN; }
    static __device__ __forceinline__ int decode(int16_t c, int rbase, int /*lane_base*/) { return rbase + (int)c; }
    static __device__ __forceinline__ int stored_base(int row0) { return row0; }
};
template <> struct SellCol<uint16_t> {
    static constexpr uint16_t kPad = 0x8000u;
    static constexpr bool stepped = true;
    static __device__ __forceinline__ bool live(uint16_t c) { return c != 0x8000u; }
    static __device__ __forceinline__ int decode(uint16_t c, int /*rbase*/, int lane_base) {
        return lane_base + (int)(int16_t)c;
    }
    static __device__ __forceinline__ int stored_base(int row0) { return row0; }
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

// The same row sum split into load and sum halves, so a kernel can issue a
// batch of slice loads early (before loads it needs sooner have returned,
// or before a barrier) and consume it later. Loads are unconditional: steps
// past the slice's width re-read its last step (cache hits) and are masked
// by step index at use, so nothing widens or selects a loaded value at load
// time (which would wait for it on the spot). An empty slice points at
// offset 0 of the arrays.
// NT: non-temporal slice loads (a pass that runs once per restart cycle, so
// the slices the Arnoldi steps re-read stay in the Infinity Cache)
template <class S, class CI, int W, bool NT = (MPG_SELL_NT != 0), int BE = kSellBatch>
struct SellRow {
    static constexpr int U = W >= BE ? 1 : BE / W;  // steps per batch (BE entries per lane)
    static constexpr bool kStepped = SellCol<CI>::stepped;
    CI c[U][W];
    S v[U][W];
    int32_t bq[kStepped ? U : 1][kStepped ? W : 1];  // stepped columns: the batch's bases
    int steps, row0, lane_row, rbase;
    int pk = -1;       // spat[s]: >= 0 implicit pattern, -1 stored, -2 - e summed from CSR
    bool exc = false;  // stepped: this slice is summed from CSR
    int xrow = 0;      // exc: this lane's row in the copy's sub-CSR
    const CI* __restrict__ cp;
    int64_t cstride;   // column entries between steps: 64 W stored, W for a pattern
    const S* __restrict__ vp;
    const int32_t* __restrict__ bp;

    int64_t o0, o1;
    int64_t co;  // where the slice's columns start: o0, or its shared block (coff)
    // the slice's offsets and pattern index: issue first (everything else
    // needs them), use later. coff: per-slice column starts when slices
    // with identical column blocks share one (SellCopy::coff), else nullptr
    __device__ __forceinline__ void init_load(int s, const int64_t* __restrict__ off,
                                              const int32_t* __restrict__ spat = nullptr,
                                              const int64_t* __restrict__ coff = nullptr) {
        o0 = off[s];
        o1 = off[s + 1];
        row0 = s * kWave;
        if (spat) pk = spat[s];
        co = coff ? coff[s] : o0;
    }
    // every slice of the copy has the same width (SellCopy::ustride entries):
    // the offsets are computed, so the value loads need no load before them
    __device__ __forceinline__ void init_uniform(int s, int64_t ustride, const int32_t* __restrict__ spat = nullptr,
                                                 const int64_t* __restrict__ coff = nullptr) {
        o0 = (int64_t)s * ustride;
        o1 = o0 + ustride;
        row0 = s * kWave;
        if (spat) pk = spat[s];
        co = coff ? coff[s] : o0;
    }
    // sbase: the stepped form's (slice, step, element) bases; pat: the
    // implicit slices' column patterns (nullptr when the copy has none).
    // Stored and implicit slices differ only in where the same column load
    // reads (a pointer and a stride chosen once per slice), never in a branch.
    __device__ __forceinline__ void init_finish(int lane, const CI* __restrict__ col, const S* __restrict__ val,
                                                const int32_t* __restrict__ sbase = nullptr,
                                                const CI* __restrict__ pat = nullptr) {
        steps = (int)((o1 - o0) / (kWave * W));
        const int64_t base = steps > 0 ? o0 + lane * W : 0;
        lane_row = row0 + lane;
        const bool imp = pk >= 0;
        cp = imp ? pat + pk : col + (steps > 0 ? co + lane * W : 0);
        cstride = imp ? W : (int64_t)kWave * W;
        rbase = imp ? lane_row : SellCol<CI>::stored_base(row0);
        vp = val + base;
        exc = pk <= -2;
        xrow = exc ? (-2 - pk) * kWave + lane : 0;
        if constexpr (kStepped) bp = sbase + (steps > 0 ? o0 / kWave : 0);  // (o0 / (64 W)) W
    }
    // a second batch buffer over the same slice (software-pipelined loops):
    // the slice geometry without the loaded registers (copying those would
    // wait for their loads)
    __device__ __forceinline__ void geom_from(const SellRow& o) {
        steps = o.steps;
        row0 = o.row0;
        lane_row = o.lane_row;
        rbase = o.rbase;
        pk = o.pk;
        exc = o.exc;
        xrow = o.xrow;
        cp = o.cp;
        cstride = o.cstride;
        vp = o.vp;
        if constexpr (kStepped) bp = o.bp;
        o0 = o.o0;
        o1 = o.o1;
        co = o.co;
    }
    __device__ __forceinline__ void init(int s, int lane, const int64_t* __restrict__ off, const CI* __restrict__ col,
                                         const S* __restrict__ val, const int32_t* __restrict__ sbase = nullptr,
                                         const int32_t* __restrict__ spat = nullptr,
                                         const CI* __restrict__ pat = nullptr,
                                         const int64_t* __restrict__ coff = nullptr) {
        init_load(s, off, spat, coff);
        init_finish(lane, col, val, sbase, pat);
    }
    __device__ __forceinline__ void load(int q) {
        const int last = steps > 0 ? steps - 1 : 0;
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int qq = q + u < last ? q + u : last;
            if constexpr (kStepped) VecW<int32_t, W, false>::load(bp + (int64_t)qq * W, bq[u]);
            VecW<CI, W, NT>::load(cp + (int64_t)qq * cstride, c[u]);
            VecW<S, W, NT>::load(vp + (int64_t)qq * kWave * W, v[u]);
        }
    }
    // The first batch in two halves, for computed (uniform) offsets: the
    // values need nothing loaded before them, the columns need the pattern
    // index spat[s], so the values go out first and the columns once the
    // index is back (init_vals, load_vals(0), init_finish, load_cols(0)).
    __device__ __forceinline__ void init_vals(int lane, const S* __restrict__ val) {
        steps = (int)((o1 - o0) / (kWave * W));
        vp = val + (steps > 0 ? o0 + lane * W : 0);
    }
    __device__ __forceinline__ void load_vals(int q) {
        const int last = steps > 0 ? steps - 1 : 0;
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int qq = q + u < last ? q + u : last;
            VecW<S, W, NT>::load(vp + (int64_t)qq * kWave * W, v[u]);
        }
    }
    __device__ __forceinline__ void load_cols(int q) {
        const int last = steps > 0 ? steps - 1 : 0;
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int qq = q + u < last ? q + u : last;
            if constexpr (kStepped) VecW<int32_t, W, false>::load(bp + (int64_t)qq * W, bq[u]);
            VecW<CI, W, NT>::load(cp + (int64_t)qq * cstride, c[u]);
        }
    }
    // The gathers of the loaded batch: every one is issued (padding and
    // steps past the width read x at row0, a valid index) and masked at the
    // sum, so the gathers of a batch are in flight together.
    template <class XF, class X>
    __device__ __forceinline__ void gather(XF xval, X (&x)[U][W]) const {
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int e = 0; e < W; ++e)
                x[u][e] = xval(SellCol<CI>::live(c[u][e])
                                   ? SellCol<CI>::decode(c[u][e], rbase, kStepped ? lane_row + bq[u][e] : 0)
                                   : row0);
    }
    // acc += the batch at step q with its gathered x, in CSR order; xs(x)
    // is the fp64 operand (a kernel that gathers x raw, before the scale it
    // is multiplied by is known, applies the scale here); acc in the
    // accumulation class (mac, internal.hpp)
    template <class X, class XS, class A>
    __device__ __forceinline__ void sum_gathered(int q, const X (&x)[U][W], XS xs, A& acc) const {
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int e = 0; e < W; ++e)
                if (q + u < steps && SellCol<CI>::live(c[u][e])) mac(acc, widen(v[u][e]), xs(x[u][e]));
    }
    // acc += the batch loaded at step q, in CSR order
    template <class XF, class A>
    __device__ __forceinline__ void sum(int q, XF xval, A& acc) const {
        double x[U][W];
        gather(xval, x);
        sum_gathered(q, x, [](double a) { return a; }, acc);
    }
};

// The row sum from a CSR in CSR order with SellRow::sum's arithmetic (a
// stepped copy's flagged slices, from the copy's sub-CSR); i < 0: no row, 0.
template <class A = double, class S, class XF>
__device__ __forceinline__ A csr_row_sum(int i, const int32_t* __restrict__ rowptr,
                                         const int32_t* __restrict__ col, const S* __restrict__ val, XF xval) {
    A acc = A(0);
    if (i < 0) return acc;
    const int j0 = rowptr[i], e = rowptr[i + 1];
    if (j0 >= e) return acc;
    // batches of 8: the batch's (column, value) loads, then its gathers, are
    // each in flight together (clamped to the row's last entry, masked at
    // the sum), so a row costs two round trips per 8 entries, not per entry
    // (16 took C4's pipelined kernel from 71 to 100 VGPRs)
    constexpr int B = 8;
    for (int j = j0; j < e; j += B) {
        int c[B];
        S v[B];
#pragma unroll
        for (int b = 0; b < B; ++b) {
            const int jj = j + b < e ? j + b : e - 1;
            c[b] = col[jj];
            v[b] = val[jj];
        }
        double x[B];
#pragma unroll
        for (int b = 0; b < B; ++b) x[b] = xval(c[b]);
#pragma unroll
        for (int b = 0; b < B; ++b)
            if (j + b < e) mac(acc, widen(v[b]), x[b]);
    }
    return acc;
}

// LDS window of x for a slice (SELL SpMVs): every column of every slice
// within [row0 - kWinLo, row0 + 64 + kWinHi) lets the gathers read LDS
constexpr int kWinLo = 64, kWinHi = 64, kWinLen = kWinLo + kWave + kWinHi;

// A SELL-64 copy of one CSR value array (device memory owned by the copy).
// nslices == 0: no copy (the CSR storage runs).
struct SellCopy {
    int n = 0, nslices = 0, W = 1;
    int vtype = 0;     // mpg_dtype_t of the stored values (MPG_F64 | MPG_F32 | MPG_F16)
    bool c16 = false;  // int16 slice-relative columns
    bool c16s = false; // stepped int16 columns (uint16_t bits + sbase)
    bool win = false;  // every slice's columns inside the LDS window
    int64_t padded = 0;
    int64_t* off = nullptr;
    void* col = nullptr;
    void* val = nullptr;
    int32_t* sbase = nullptr;  // c16s: one base per (slice, step, element)
    int32_t* spat = nullptr;   // per slice: implicit pattern index, -1 stored, -2 CSR (nullptr: all stored)
    void* pat = nullptr;       // the implicit slices' column patterns (CI entries, W per step)
    int64_t nexc = 0;          // c16s: slices summed from CSR
    int32_t* xrp = nullptr;    // their rows as a CSR owned by the copy: 64 nexc + 1 row starts
    int32_t* xcol = nullptr;   //   (row 64 e + lane of flagged slice e; rows past n are empty),
    void* xval = nullptr;      //   columns and values (the stored value type) in CSR order
    int64_t nimp = 0;          // implicit slices
    int64_t imp_slots = 0;     // their slots (their columns are not read)
    int64_t npat = 0;          // pattern entries
    int64_t ustride = 0;       // > 0: every slice holds this many slots (off[s] = s * ustride)
    int64_t* coff = nullptr;   // shared column blocks: per slice, where its columns start in col
                               // (slices with identical int16 column blocks store one; nullptr: off)
    int64_t nshared = 0;       // slices that read another slice's column block
    int64_t col_slots = 0;     // column entries stored (after sharing; implicit slices store none)
    // SELL-C-sigma: the rows of every window of `sigma` rows sorted by length
    // (longest first) before slicing; rows[64 s + l] = the row lane l of slice
    // s holds (n for padding lanes). nullptr / 0: slice s holds rows 64 s..
    int32_t* rows = nullptr;
    int sigma = 0;
    int col_bytes() const { return c16 || c16s ? 2 : 4; }
};

// Build the copy from the CSR structure and `val` (vtype; F16 = raw IEEE
// half bits). format: 0 auto (only when padding adds <= 20 % to the stored
// entries), 1 never, 2 always. Synchronises the context's stream.
int sell_build(mpg_ctx* ctx, const mpg_csr* A, int vtype, const void* val, int format, SellCopy& S);
void sell_free(SellCopy& S);
// matrix bytes one SpMV over the copy reads (mpg_sell_bytes)
int64_t sell_matrix_bytes(const SellCopy& S);

// f(column type, integral_constant<int, W>) for the copy's layout
template <class F>
int sell_dispatch(const SellCopy& S, F&& f) {
    auto with_w = [&](auto ci) {
        switch (S.W) {
            case 1: return f(ci, std::integral_constant<int, 1>());
            case 2: return f(ci, std::integral_constant<int, 2>());
            case 4: return f(ci, std::integral_constant<int, 4>());
            default: return (int)MPG_ERR_UNSUPPORTED;
        }
    };
    return S.c16 ? with_w(int16_t()) : S.c16s ? with_w(uint16_t()) : with_w(int32_t());
}
// XCD-ordered slices (MPG_SELL_XCD=0: off): a copy without the LDS window
// gathers x from global memory, and with the default round-robin placement
// of workgroups over the 8 XCDs every XCD's L2 fetches the whole of x for
// the neighbour planes of its scattered slices; in XCD order each L2 serves
// one contiguous run of rows (xcd_block, internal.hpp)
// computed slice offsets whenever every slice has the same width
// (MPG_SELL_UNIFORM=0: always load them). The offsets' load sits in front of
// every slice's value loads; computing them measured BAND-100M fp16 99.1 ->
// 93.6 us, fp32 108.2 -> 103.7, BAND-10M 13.85 -> 13.61, LAP-1M 14.27 ->
// 13.91 (profiles/r03_spmv_uniform_ab.jsonl)
inline bool sell_uniform(const SellCopy& S) {
    if (S.ustride <= 0) return false;
    const char* e = std::getenv("MPG_SELL_UNIFORM");
    return !(e && *e == '0');
}

// two slices per wave in the Arnoldi SpMV (k_step_sell2): int16 columns,
// uniform widths of at most 12 entries per lane in one batch, W 2 or 4
// (banded matrices, 7-point stencils). Returns the batch size in entries
// (8, 10 (W = 2) or 12: the registers of one batch per slice), or 0 for one slice per
// wave (MPG_SELL_PAIR=0: never). In-cycle, Givens folded
// (profiles/r03_spmv_pair_ab.jsonl, median of 5 interleaved): BAND-100M fp16
// 94.5 -> 72.9 us, fp32 102.8 -> 92.2, BAND-10M 14.2 -> 12.9, LAP-1M fp32
// 14.0 -> 12.8, fp64 22.4 -> 19.7.
inline int sell_pair(const SellCopy& S) {
    const char* e = std::getenv("MPG_SELL_PAIR");
    if ((e && *e == '0') || S.nslices < 2 || !S.c16 || S.ustride <= 0 || (S.W != 2 && S.W != 4)) return 0;
    const int64_t entries = S.ustride / kWave;  // per lane (row) of every slice
    if (entries <= 8) return 8;
    if (entries <= 10 && S.W == 2) return 10;  // BAND's 10 entries: no wasted step, fewer registers
    return entries <= 12 ? 12 : 0;
}

// software-pipelined batches in the one-slice-per-wave SpMV without the LDS
// window (k_step_sell<..., PIPE>): on by default for stepped columns (C4
// stand-in, in-cycle SpMV, interleaved: 314.5 -> 311.5 us, one wave per SIMD
// less for one memory round trip per batch less), off for int32 columns
// (unmeasured). MPG_SELL_PIPE=0/1 forces it off/on.
inline bool sell_pipe(const SellCopy& S) {
    const char* e = std::getenv("MPG_SELL_PIPE");
    if (e && (*e == '0' || *e == '1')) return *e == '1';
    return S.c16s;
}

inline bool sell_xcd_order(const SellCopy& S) {
    const char* e = std::getenv("MPG_SELL_XCD");
    return !S.win && !(e && *e == '0');
}

template <class F>
int sell_dispatch_win(bool win, F&& f) {
    return win ? f(std::true_type()) : f(std::false_type());
}

}  // namespace mpg
