// SELL-64 copies of a CSR matrix (sell_tile.hpp) and the stand-alone SELL
// SpMV behind the operator surface (replaces mkl_sparse_?_mv,
// kernels_mkl.cpp:326-352, like mpg_csr_spmv, on the sliced copy).
//
// The builder is shared with the fused Arnoldi engine (arnoldi.hip), whose
// SpMV phase runs on the same copy. A copy is worth it when padding the
// slices to their longest row adds little (banded and stencil matrices);
// the builder reports "no copy" otherwise and the caller keeps CSR.
//
// The SpMV issues its loads in the order they are needed (vmcnt retires in
// issue order): the slice's offsets, the window of x (raw, clamped), y when
// beta != 0, the first batch of (column, value) steps; nothing is waited for
// before all of them are in flight. Sums are fp64 in CSR order, rounded
// once to the vector type: y = alpha*t (+ beta*y), as spmv.hip.
#include "sell_tile.hpp"
#include "scalar_program.hpp"
#include "ride.hpp"
#include "handoff.hpp"
#include "internal.hpp"
#include "mpgmres/arnoldi.h"
#include "mpgmres/capi.h"

#include <algorithm>
#include <cstring>
#include <map>
#include <cstdlib>
#include <new>
#include <vector>

using namespace mpg;

namespace {

// min and max of (col - first row of its slice) over the matrix: int16
// column eligibility and the LDS window
__global__ void k_sell_span(int n, const int32_t* __restrict__ rowptr, const int32_t* __restrict__ col,
                            int* __restrict__ out) {
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    int lo = INT32_MAX, hi = INT32_MIN;
    if (r < n) {
        const int row0 = r & ~(kWave - 1);
        for (int j = rowptr[r]; j < rowptr[r + 1]; ++j) {
            const int d = col[j] - row0;
            lo = min(lo, d);
            hi = max(hi, d);
        }
    }
    if (r < n && rowptr[r] < rowptr[r + 1]) {
        atomicMin(out, lo);
        atomicMax(out + 1, hi);
    }
}

// Slice classification, one wave per slice. For each step j and element e:
// d = c - (row0 + lane) over the rows that have that entry, its min and max
// across the 64 rows, and how many rows have it. The base of (slice, step,
// element) is the midpoint of [min, max] (kBasePad where no row has the
// entry). Kind: implicit when every (step, element) is either present in all
// 64 rows with one d, or absent from all; else, for the stepped form, CSR
// when some spread exceeds +-32767; else stored.
constexpr uint8_t kSliceStored = 0, kSliceCsr = 1, kSliceImplicit = 2;
constexpr int32_t kBasePad = INT32_MIN;  // an element that is padding in every row of the slice

template <int W>
__global__ __launch_bounds__(kBlock) void k_sell_classify(int n, int nslices, const int32_t* __restrict__ rowptr,
                                                          const int32_t* __restrict__ col,
                                                          const int64_t* __restrict__ off, int32_t* __restrict__ sbase,
                                                          uint8_t* __restrict__ skind, int stepped, int implicit) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int s = (int)(t / kWave), lane = (int)(t % kWave);
    if (s >= nslices) return;  // whole waves: the wave's shuffles below stay converged
    const int r = s * kWave + lane;
    const int64_t o = off[s];
    const int steps = (int)((off[s + 1] - o) / (kWave * W));
    const int b = r < n ? rowptr[r] : 0, len = r < n ? rowptr[r + 1] - b : 0;
    bool bad = false, imp = implicit != 0;
    for (int j = 0; j < steps; ++j) {
        for (int e = 0; e < W; ++e) {
            const int k = j * W + e;
            const bool has = k < len;
            int lo = INT32_MAX, hi = INT32_MIN;
            if (has) {
                const int d = col[b + k] - r;
                lo = d;
                hi = d;
            }
            const int cnt = __popcll(__ballot(has));
            for (int m = kWave / 2; m > 0; m >>= 1) {
                lo = min(lo, __shfl_xor(lo, m, kWave));
                hi = max(hi, __shfl_xor(hi, m, kWave));
            }
            const int base = cnt == 0 ? kBasePad : (int)(((int64_t)lo + (int64_t)hi) >> 1);
            if (cnt > 0 && ((int64_t)hi - base > 32767 || (int64_t)lo - base < -32767)) bad = true;
            if (!(cnt == 0 || (cnt == kWave && lo == hi))) imp = false;
            if (lane == 0) sbase[o / kWave + (int64_t)j * W + e] = base;
        }
    }
    if (lane == 0) skind[s] = imp ? kSliceImplicit : (stepped && bad) ? kSliceCsr : kSliceStored;
}

// scatter the CSR (col, val) of row 64 s + lane into its slice; pads get the
// sentinel column and a zero value (S: stored value type, half as raw bits)
template <class S, class CI, int W>
__global__ void k_sell_fill(int n, int nslices, const int32_t* __restrict__ rowptr, const int32_t* __restrict__ col,
                            const S* __restrict__ val, const int64_t* __restrict__ off, const int32_t* __restrict__ sbase,
                            CI* __restrict__ scol, S* __restrict__ sval, const int32_t* __restrict__ rows) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int s = (int)(t / kWave), lane = (int)(t % kWave);
    if (s >= nslices) return;
    const int r = rows ? rows[s * kWave + lane] : s * kWave + lane;  // (sorted copies: int32 columns only)
    const int64_t o = off[s];
    const int width = (int)((off[s + 1] - o) / kWave);
    const int b = r < n ? rowptr[r] : 0, len = r < n ? rowptr[r + 1] - b : 0;
    for (int j = 0; j < width; ++j) {
        const int64_t pos = o + (int64_t)(j / W) * kWave * W + lane * W + (j % W);
        if (j < len) {
            const int c = col[b + j];
            if constexpr (SellCol<CI>::stepped) scol[pos] = (CI)(uint16_t)(int16_t)(c - r - sbase[o / kWave + j]);
            else scol[pos] = sizeof(CI) == 2 ? (CI)(c - s * kWave) : (CI)c;
            sval[pos] = val[b + j];
        } else {
            scol[pos] = SellCol<CI>::kPad;
            sval[pos] = S(0);
        }
    }
}

// Shared column blocks: slices whose stored column blocks are identical
// (2-byte forms: offsets relative to the slice, so every interior slice of
// a stencil with the same boundary pattern has the same block) keep one copy.
__device__ __forceinline__ uint64_t mix_bits(uint64_t z) {
    z += 0x9e3779b97f4a7c15ULL;
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
    return z ^ (z >> 31);
}

// per slice: XOR over its block of mix(position, value), and the length
template <class CI>
__global__ __launch_bounds__(kBlock) void k_sell_col_hash(int nslices, const int64_t* __restrict__ off,
                                                          const CI* __restrict__ col, uint64_t* __restrict__ out) {
    const int64_t t0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int s = (int)(t0 / kWave), lane = (int)(t0 % kWave);
    if (s >= nslices) return;
    const int64_t o = off[s], len = off[s + 1] - o;
    uint64_t h = 0;
    for (int64_t t = lane; t < len; t += kWave)
        h ^= mix_bits(((uint64_t)t << 20) ^ (uint64_t)(uint16_t)col[o + t] ^ ((uint64_t)(uint32_t)col[o + t] << 40));
    for (int m = kWave / 2; m > 0; m >>= 1) {
        const uint32_t lo = __shfl_xor((uint32_t)h, m, kWave), hi = __shfl_xor((uint32_t)(h >> 32), m, kWave);
        h ^= ((uint64_t)hi << 32) | lo;
    }
    if (lane == 0) out[s] = h ^ mix_bits((uint64_t)len);
}

// bad[s] = 1 where slice s's block differs from that of rep[s] (rep[s] >= 0, != s)
template <class CI>
__global__ __launch_bounds__(kBlock) void k_sell_col_verify(int nslices, const int64_t* __restrict__ off,
                                                            const CI* __restrict__ col, const int32_t* __restrict__ rep,
                                                            int* __restrict__ bad) {
    const int64_t t0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int s = (int)(t0 / kWave), lane = (int)(t0 % kWave);
    if (s >= nslices) return;
    const int r = rep[s];
    if (r < 0 || r == s) return;
    const int64_t o = off[s], orr = off[r], len = off[s + 1] - o;
    bool diff = len != off[r + 1] - orr;
    for (int64_t t = lane; t < len && !diff; t += kWave) diff = col[o + t] != col[orr + t];
    if (diff) bad[s] = 1;
}

// the stored blocks into their compacted places (newoff[s] < 0: not stored)
template <class CI>
__global__ __launch_bounds__(kBlock) void k_sell_col_gather(int nslices, const int64_t* __restrict__ off,
                                                            const CI* __restrict__ col,
                                                            const int64_t* __restrict__ newoff, CI* __restrict__ out) {
    const int64_t t0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int s = (int)(t0 / kWave), lane = (int)(t0 % kWave);
    if (s >= nslices) return;
    const int64_t d = newoff[s];
    if (d < 0) return;
    const int64_t o = off[s], len = off[s + 1] - o;
    for (int64_t t = lane; t < len; t += kWave) out[d + t] = col[o + t];
}

template <class F>
int with_store(int vtype, F&& f) {
    switch (vtype) {
        case MPG_F64: return f(double());
        case MPG_F32: return f(float());
        case MPG_F16: return f(uint16_t());
        default: return MPG_ERR_UNSUPPORTED;
    }
}

// y = alpha * T(A x) (+ beta * y) on the sliced copy; one wave per slice.
// prog.count > 0: workgroup 0 runs that scalar program instead (the
// operator surface's Givens step of the previous Arnoldi step, which nothing
// in this SpMV reads or writes: kernels_hip.cpp checks the operands).
template <class X, class S, class CI, int W, bool WIN, bool UNI = false, bool NORM = false>
__global__ __launch_bounds__(kBlock) void k_sell_spmv(int n, int cols, int nslices, const int64_t* __restrict__ off,
                                                      const CI* __restrict__ col, const S* __restrict__ val,
                                                      const int32_t* __restrict__ sbase,
                                                      const int32_t* __restrict__ spat, const int64_t* __restrict__ coff, const CI* __restrict__ pat,
                                                      const int32_t* __restrict__ xrp,
                                                      const int32_t* __restrict__ xcol, const S* __restrict__ xval,
                                                      const X* __restrict__ x, X alpha, X beta, X* __restrict__ y,
                                                      int64_t ustride, int xcd, ScalarProgram prog,
                                                      const int32_t* __restrict__ rows, NormArgs<X> nm) {
    constexpr int NQ = kWinLen / kWave;
    __shared__ X win[WIN ? kBlock / kWave : 1][WIN ? kWinLen : 1];
    const int lane = threadIdx.x & (kWave - 1), wid = wave_id();
    // NORM: the ||w||^2 partial of this lane, issued before anything else
    double pv = 0.0;
    if constexpr (NORM) pv = (int)threadIdx.x < nm.nparts ? nm.part[threadIdx.x] : 0.0;
    // a scalar program riding in this launch: workgroup 0 (dispatched first,
    // so it runs under the slices instead of after them), its first wave
    int b = (int)blockIdx.x, G = (int)gridDim.x;
    if (prog.count > 0) {
        if (b == 0) {
            __shared__ double plds[3 * kProgStage + 1];
            if constexpr (NORM) (void)norm_scale(nm, pv);  // h(k+1,k) stored before the program reads it
            if (wid == 0) run_scalar_program<kProgStage>(prog, plds);
            return;
        }
        --b;
        --G;
    }
    const int s_raw = (xcd ? xcd_block(b, G) : b) * (kBlock / kWave) + wid;
    const bool dead = s_raw >= nslices;
    // without NORM a dead wave may leave (no workgroup barrier below); with it
    // every wave takes part in the partial sum first (on slice 0's loads)
    if (!NORM && dead) return;
    const int s = dead ? 0 : s_raw;
    const int row0 = s * kWave;
    SellRow<S, CI, W> row;
    if constexpr (UNI) row.init_uniform(s, ustride, spat, coff);
    else row.init_load(s, off, spat, coff);
    __builtin_amdgcn_sched_barrier(0);
    // the lane's row: row0 + lane, or a sorted (SELL-C-sigma) copy's rows[]
    const int i = rows ? rows[row0 + lane] : row0 + lane;
    X xr[WIN ? NQ : 1];
    if constexpr (WIN) {
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            const int c = row0 - kWinLo + q * kWave + lane;
            xr[q] = x[c >= 0 && c < cols ? c : 0];
        }
    }
    const X yi = beta != X(0) ? y[i < n ? i : 0] : X(0);
    X xo = X(0);  // NORM, no window: the lane's own entry of w
    if constexpr (NORM && !WIN) xo = x[i < n ? i : 0];
    __builtin_amdgcn_sched_barrier(0);
    row.init_finish(lane, col, val, sbase, pat);
    row.load(0);
    __builtin_amdgcn_sched_barrier(0);
    X a = X(1);
    if constexpr (NORM) {
        a = norm_scale(nm, pv);
        if (dead) return;
    }
    auto sc = [&](X v) { return NORM ? (X)(a * v) : v; };
    double sum = 0.0;
    if constexpr (WIN) {
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            const int c = row0 - kWinLo + q * kWave + lane;
            win[wid][q * kWave + lane] = (c >= 0 && c < cols) ? sc(xr[q]) : X(0);
        }
        wave_lds_sync();
        auto xv = [&](int c) { return (double)win[wid][c - row0 + kWinLo]; };
        if constexpr (NORM) if (i < n) nm.v[i] = win[wid][i - row0 + kWinLo];
        row.sum(0, xv, sum);
        for (int q = row.U; q < row.steps; q += row.U) {
            row.load(q);
            row.sum(q, xv, sum);
        }
    } else {
        if constexpr (NORM) if (i < n) nm.v[i] = sc(xo);
        auto xv = [&](int c) { return (double)sc(x[c]); };
        if (SellCol<CI>::stepped && row.exc) {
            sum = csr_row_sum(i < n ? row.xrow : -1, xrp, xcol, xval, xv);
        } else {
            row.sum(0, xv, sum);
            for (int q = row.U; q < row.steps; q += row.U) {
                row.load(q);
                row.sum(q, xv, sum);
            }
        }
    }
    if (i < n) {
        const X t = (X)sum;
        y[i] = spmv_axpby(alpha, t, beta, yi);
    }
}

// k_sell_spmv with two 64-row slices per wave (the operator surface's form of
// the fused engine's k_step_sell2): uniform int16 copies of W = 2 or 4 with
// at most 12 entries per row (sell_pair). Lane l owns rows 128 s' + l and
// 128 s' + 64 + l; both slices' values, columns, the window (or the first
// batch's gathers) are issued before the wave waits for any of them, so a
// wave carries twice the bytes through the same fixed work. The row sums are
// k_sell_spmv's (fp64, CSR order), so y has the same bits.
template <class X, class S, int W, bool WIN, int BE, bool NORM = false>
__global__ __launch_bounds__(kBlock) void k_sell_spmv2(int n, int cols, int nslices, const int16_t* __restrict__ col,
                                                       const S* __restrict__ val, const int32_t* __restrict__ sbase,
                                                       const int32_t* __restrict__ spat, const int64_t* __restrict__ coff,
                                                       const int16_t* __restrict__ pat, const X* __restrict__ x, X alpha,
                                                       X beta, X* __restrict__ y, int64_t ustride, int xcd,
                                                       ScalarProgram prog, NormArgs<X> nm) {
    using CI = int16_t;
    constexpr int SPW = 2;
    constexpr int WL = kWinLen + (SPW - 1) * kWave;
    constexpr int NQ = WL / kWave;
    __shared__ X win[WIN ? kBlock / kWave : 1][WIN ? WL : 1];
    const int lane = threadIdx.x & (kWave - 1), wid = wave_id();
    double pv = 0.0;  // NORM: the lane's ||w||^2 partial, issued first
    if constexpr (NORM) pv = (int)threadIdx.x < nm.nparts ? nm.part[threadIdx.x] : 0.0;
    int b = (int)blockIdx.x, G = (int)gridDim.x;
    if (prog.count > 0) {  // the riding scalar program: workgroup 0's first wave
        if (b == 0) {
            __shared__ double plds[3 * kProgStage + 1];
            if constexpr (NORM) (void)norm_scale(nm, pv);  // h(k+1,k) stored before the program reads it
            if (wid == 0) run_scalar_program<kProgStage>(prog, plds);
            return;
        }
        --b;
        --G;
    }
    const int s0_raw = ((xcd ? xcd_block(b, G) : b) * (kBlock / kWave) + wid) * SPW;
    const bool dead = s0_raw >= nslices;
    if (!NORM && dead) return;  // no workgroup barrier below (NORM: after the partial sum)
    const int s0 = dead ? 0 : s0_raw;
    const int row0 = s0 * kWave;
    bool live_p[SPW];
    SellRow<S, CI, W, false, BE> row[SPW];
#pragma unroll
    for (int p = 0; p < SPW; ++p) {
        live_p[p] = !dead && s0 + p < nslices;
        row[p].init_uniform(s0 + p < nslices ? s0 + p : s0, ustride, spat, coff);
    }
    __builtin_amdgcn_sched_barrier(0);
    X xw[WIN ? NQ : 1];
    if constexpr (WIN) {
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            const int c = row0 - kWinLo + q * kWave + lane;
            xw[q] = x[c >= 0 && c < cols ? c : 0];
        }
    }
    X yi[SPW];
    X xo[NORM && !WIN ? SPW : 1];  // NORM, no window: the lanes' own entries of w
#pragma unroll
    for (int p = 0; p < SPW; ++p) {
        const int i = row0 + p * kWave + lane;
        yi[p] = beta != X(0) ? y[live_p[p] && i < n ? i : 0] : X(0);
        if constexpr (NORM && !WIN) xo[p] = x[live_p[p] && i < n ? i : 0];
    }
    __builtin_amdgcn_sched_barrier(0);
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
    __builtin_amdgcn_sched_barrier(0);
    using RowT = SellRow<S, CI, W, false, BE>;
    X xg[WIN ? 1 : SPW][WIN ? 1 : RowT::U][WIN ? 1 : W];
    if constexpr (!WIN) {
#pragma unroll
        for (int p = 0; p < SPW; ++p) row[p].gather([&](int c) { return x[c]; }, xg[p]);
    }
    __builtin_amdgcn_sched_barrier(0);
    X a = X(1);
    if constexpr (NORM) {
        a = norm_scale(nm, pv);  // (its barrier also waits for the loads above)
        if (dead) return;
    }
    auto sc = [&](X v) { return NORM ? (X)(a * v) : v; };
    double sum[SPW] = {};
    if constexpr (WIN) {
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            const int c = row0 - kWinLo + q * kWave + lane;
            win[wid][q * kWave + lane] = (c >= 0 && c < cols) ? sc(xw[q]) : X(0);
        }
        wave_lds_sync();
        auto xv = [&](int c) { return (double)win[wid][c - row0 + kWinLo]; };
        if constexpr (NORM) {
#pragma unroll
            for (int p = 0; p < SPW; ++p) {
                const int i = row0 + p * kWave + lane;
                if (live_p[p] && i < n) nm.v[i] = win[wid][i - row0 + kWinLo];
            }
        }
#pragma unroll
        for (int p = 0; p < SPW; ++p) row[p].sum(0, xv, sum[p]);
#pragma unroll
        for (int p = 0; p < SPW; ++p)
            for (int q = row[p].U; q < row[p].steps; q += row[p].U) {
                row[p].load(q);
                row[p].sum(q, xv, sum[p]);
            }
    } else {
        if constexpr (NORM) {
#pragma unroll
            for (int p = 0; p < SPW; ++p) {
                const int i = row0 + p * kWave + lane;
                if (live_p[p] && i < n) nm.v[i] = sc(xo[p]);
            }
        }
        auto xv = [&](int c) { return (double)sc(x[c]); };
#pragma unroll
        for (int p = 0; p < SPW; ++p) {
            row[p].sum_gathered(0, xg[p], [&](X r) { return (double)sc(r); }, sum[p]);
            for (int q = row[p].U; q < row[p].steps; q += row[p].U) {
                row[p].load(q);
                row[p].sum(q, xv, sum[p]);
            }
        }
    }
#pragma unroll
    for (int p = 0; p < SPW; ++p) {
        const int i = row0 + p * kWave + lane;
        if (live_p[p] && i < n) {
            const X t = (X)sum[p];
            y[i] = spmv_axpby(alpha, t, beta, yi[p]);
        }
    }
}

}  // namespace

namespace mpg {

int sell_share_columns(SellCopy& S, const std::vector<int64_t>& off, const std::vector<int32_t>& spat_h, int grid,
                       hipStream_t stream);

int sell_build(mpg_ctx* ctx, const mpg_csr* A, int vtype, const void* val, int format, SellCopy& S) {
    S = SellCopy{};
    const int n = A->rows;
    if (format == 1 || n == 0 || A->nnz == 0) return MPG_OK;
    hipStream_t stream = ctx->stream;
    std::vector<int32_t> rp((size_t)n + 1);
    if (hipMemcpyAsync(rp.data(), A->rowptr, rp.size() * 4, hipMemcpyDeviceToHost, stream) != hipSuccess ||
        hipStreamSynchronize(stream) != hipSuccess)
        return MPG_ERR_HIP;
    const int ns = (n + kWave - 1) / kWave;
    auto len_of = [&](int r) { return r < n ? rp[r + 1] - rp[r] : 0; };
    std::vector<int> width((size_t)ns, 0);
    for (int r = 0; r < n; ++r) width[r / kWave] = std::max(width[r / kWave], len_of(r));
    const char* fw = std::getenv("MPG_SELL_W");  // 1, 2 or 4: force the vector width (experiments)
    const bool forced = fw && (*fw == '1' || *fw == '2' || *fw == '4') && fw[1] == 0;
    // the widest vector whose padding stays within 15 % of the least padded
    // layout: narrow (2-4 B per lane) index loads cost more than the padding
    auto choose = [&](const std::vector<int>& wd, int& bw, int64_t& bp) {
        int64_t padded[5] = {0, 0, 0, 0, 0};
        for (int W : {4, 2, 1})
            for (int s = 0; s < ns; ++s) padded[W] += (int64_t)kWave * ((wd[s] + W - 1) / W * W);
        const int64_t least = std::min(padded[1], std::min(padded[2], padded[4]));
        bw = 1;
        for (int W : {4, 2, 1})
            if ((double)padded[W] <= 1.15 * (double)least) {
                bw = W;
                break;
            }
        if (forced) bw = *fw - '0';
        bp = padded[bw];
    };
    int best_w = 1;
    int64_t best = 0;
    choose(width, best_w, best);
    // SELL-C-sigma (MPG_SELL_SIGMA: the window in rows when slicing pads more
    // than 20 %; default 0 = off; -1 always, window 1024, for tests). Off by
    // default since measured: on fem27 at 4.1M rows the sorted copy's SpMV
    // took 486 us against 418 us unsorted and 423 us CSR (fem27 permuted:
    // 549 / 463 / 458 us; profiles/r04y_irr.jsonl) -- the sorted lanes'
    // scattered row stores and x gathers cost more than the padding they
    // save. Rows of varying length in one slice pad it to its
    // longest row (the FEM-like fem27 stand-in: 26 % at W = 4). Sorting the
    // rows of each window of sigma rows by length (longest first, stable) and
    // slicing that order brings the padding to ~5 %, at the price of the
    // lanes' row numbers (4 B per row, S.rows) and scattered row stores
    // within the window. Sorted copies keep int32 columns and no LDS window:
    // the 2-byte and implicit forms and the window assume a slice holds
    // consecutive rows.
    std::vector<int32_t> order;
    {
        const char* se = std::getenv("MPG_SELL_SIGMA");
        const int sg = se && *se ? std::atoi(se) : 0;
        const int sigma = sg < 0 ? 1024 : sg / kWave * kWave;
        if (sigma >= kWave && (sg < 0 || (double)best > 1.2 * (double)A->nnz)) {
            std::vector<int32_t> ord((size_t)ns * kWave);
            for (int64_t w0 = 0; w0 < (int64_t)ns * kWave; w0 += sigma) {
                const int64_t w1 = std::min<int64_t>(w0 + sigma, (int64_t)ns * kWave);
                for (int64_t p = w0; p < w1; ++p) ord[(size_t)p] = (int32_t)std::min<int64_t>(p, n);
                std::stable_sort(ord.begin() + w0, ord.begin() + w1,
                                 [&](int32_t a, int32_t b) { return len_of(a) > len_of(b); });
            }
            std::vector<int> wd((size_t)ns, 0);
            for (int s = 0; s < ns; ++s)
                for (int l = 0; l < kWave; ++l) wd[s] = std::max(wd[s], len_of(ord[(size_t)s * kWave + l]));
            int bw = 1;
            int64_t bp = 0;
            choose(wd, bw, bp);
            if (sg < 0 || bp < best) {
                order.swap(ord);
                width.swap(wd);
                best_w = bw;
                best = bp;
                S.sigma = sigma;
            }
        }
    }
    // (no copy on these two paths: S.sigma reports a window only for a built copy)
    if (format == 0 && !forced && (double)best > 1.2 * (double)A->nnz) {
        S.sigma = 0;
        return MPG_OK;
    }
    if (best >= ((int64_t)1 << 31) * 4) {
        S.sigma = 0;
        return format == 2 ? MPG_ERR_UNSUPPORTED : MPG_OK;
    }
    std::vector<int64_t> off((size_t)ns + 1, 0);
    for (int s = 0; s < ns; ++s)
        off[s + 1] = off[s] + (int64_t)kWave * ((width[s] + best_w - 1) / best_w * best_w);

    int* span = nullptr;
    int span_h[2] = {INT32_MAX, INT32_MIN};
    if (hipMalloc((void**)&span, 2 * sizeof(int)) != hipSuccess) return MPG_ERR_ALLOC;
    bool ok = hipMemcpyAsync(span, span_h, 2 * sizeof(int), hipMemcpyHostToDevice, stream) == hipSuccess;
    if (ok) {
        k_sell_span<<<(n + kBlock - 1) / kBlock, kBlock, 0, stream>>>(n, A->rowptr, A->col, span);
        ok = hipMemcpyAsync(span_h, span, 2 * sizeof(int), hipMemcpyDeviceToHost, stream) == hipSuccess &&
             hipStreamSynchronize(stream) == hipSuccess;
    }
    (void)hipFree(span);
    if (!ok) return MPG_ERR_HIP;
    const bool sorted = !order.empty();
    const bool c16 = !sorted && span_h[0] >= -32767 && span_h[1] <= 32767;
    const char* senv = std::getenv("MPG_SELL_STEPPED");  // 0: never the stepped int16 form
    const bool try_c16s = !sorted && !c16 && !(senv && *senv == '0');
    const char* wenv = std::getenv("MPG_SELL_WINDOW");  // 0: always gather from global memory
    const bool win = !sorted && !(wenv && *wenv == '0') && span_h[0] >= -kWinLo && span_h[1] < kWave + kWinHi;
    if (sorted) {
        if (hipMalloc((void**)&S.rows, order.size() * 4) != hipSuccess ||
            hipMemcpyAsync(S.rows, order.data(), order.size() * 4, hipMemcpyHostToDevice, stream) != hipSuccess) {
            sell_free(S);
            return MPG_ERR_ALLOC;
        }
    }
    const size_t vsize = vtype == MPG_F64 ? 8 : vtype == MPG_F32 ? 4 : 2;
    if (hipMalloc((void**)&S.off, off.size() * 8) != hipSuccess) {
        sell_free(S);
        return MPG_ERR_ALLOC;
    }
    if (hipMemcpyAsync(S.off, off.data(), off.size() * 8, hipMemcpyHostToDevice, stream) != hipSuccess) {
        sell_free(S);
        return MPG_ERR_HIP;
    }
    S.n = n;
    S.nslices = ns;
    S.W = best_w;
    S.ustride = off[1];
    for (int s2 = 1; s2 < ns && S.ustride > 0; ++s2)
        if (off[s2 + 1] - off[s2] != S.ustride) S.ustride = 0;
    S.vtype = vtype;
    S.c16 = c16;
    S.win = win;
    S.padded = best;
    const int grid = (int)(((int64_t)ns * kWave + kBlock - 1) / kBlock);
    const char* ienv = std::getenv("MPG_SELL_IMPLICIT");  // 0: always read the stored columns
    const bool try_imp = !sorted && !(ienv && *ienv == '0');
    std::vector<int32_t> spat_h;   // per slice (host), when the copy has implicit or CSR slices
    std::vector<int32_t> pat_h;    // implicit patterns: lane-relative offsets, W per step
    if (try_c16s || try_imp) {
        // bases and kinds (k_sell_classify); the stepped form when at most 1 %
        // of the slices need the CSR fallback; implicit slices wherever they
        // occur, their offset patterns deduplicated
        std::vector<uint8_t> kind((size_t)ns, 0);
        const size_t nb = (size_t)(best / kWave);
        uint8_t* kind_d = nullptr;
        bool okb = hipMalloc((void**)&S.sbase, nb * 4 + 256) == hipSuccess &&
                   hipMalloc((void**)&kind_d, (size_t)ns + 256) == hipSuccess;
        if (okb) {
            auto launch = [&](auto wc) {
                k_sell_classify<decltype(wc)::value><<<grid, kBlock, 0, stream>>>(
                    n, ns, A->rowptr, A->col, S.off, S.sbase, kind_d, try_c16s ? 1 : 0, try_imp ? 1 : 0);
            };
            if (best_w == 4) launch(std::integral_constant<int, 4>());
            else if (best_w == 2) launch(std::integral_constant<int, 2>());
            else launch(std::integral_constant<int, 1>());
            okb = hipMemcpyAsync(kind.data(), kind_d, (size_t)ns, hipMemcpyDeviceToHost, stream) == hipSuccess &&
                  hipStreamSynchronize(stream) == hipSuccess;
        }
        if (kind_d) (void)hipFree(kind_d);
        std::vector<int32_t> bases;
        int64_t nexc = 0, nimp = 0;
        for (uint8_t k : kind) {
            nexc += k == kSliceCsr;
            nimp += k == kSliceImplicit;
        }
        if (okb && nimp) {
            bases.resize(nb);
            okb = hipMemcpyAsync(bases.data(), S.sbase, nb * 4, hipMemcpyDeviceToHost, stream) == hipSuccess &&
                  hipStreamSynchronize(stream) == hipSuccess;
        }
        if (!okb) {
            sell_free(S);
            return MPG_ERR_HIP;
        }
        S.c16s = try_c16s && nexc * 100 <= ns;
        if (!S.c16s) nexc = 0;  // int32 columns: those slices are stored
        if (nimp || nexc) {
            spat_h.assign((size_t)ns, -1);
            std::map<std::vector<int32_t>, int32_t> index;
            int32_t e = 0;
            for (int s2 = 0; s2 < ns; ++s2) {
                if (kind[s2] == kSliceCsr && S.c16s) {
                    spat_h[s2] = -2 - e++;
                } else if (kind[s2] == kSliceImplicit) {
                    const int64_t b0 = off[s2] / kWave, b1 = off[s2 + 1] / kWave;
                    std::vector<int32_t> key(bases.begin() + b0, bases.begin() + b1);
                    bool fits = true;  // int16 slice-relative form: the lane-relative offsets must fit too
                    if (S.c16)
                        for (int32_t d : key) fits = fits && (d == kBasePad || (d >= -32767 && d <= 32767));
                    if (!fits) {
                        --nimp;
                        continue;
                    }
                    auto it = index.find(key);
                    if (it == index.end()) {
                        it = index.emplace(key, (int32_t)pat_h.size()).first;
                        // lane-relative offsets; the stepped form stores them
                        // against its bases, i.e. 0 (an implicit element's d
                        // is its base)
                        for (int32_t d : key) pat_h.push_back(d == kBasePad ? INT32_MIN : (S.c16s ? 0 : d));
                    }
                    spat_h[s2] = it->second;
                    S.imp_slots += off[s2 + 1] - off[s2];
                }
            }
            S.nimp = nimp;
        }
        S.nexc = nexc;
        if (!S.c16s) {  // only the stepped form reads the bases
            (void)hipFree(S.sbase);
            S.sbase = nullptr;
        }
    }
    if (hipMalloc(&S.col, (size_t)best * S.col_bytes() + 256) != hipSuccess ||
        hipMalloc(&S.val, (size_t)best * vsize + 256) != hipSuccess) {
        sell_free(S);
        return MPG_ERR_ALLOC;
    }
    int st = with_store(vtype, [&](auto sv) {
        using St = decltype(sv);
        return sell_dispatch(S, [&](auto ci, auto wc) {
            using CI = decltype(ci);
            k_sell_fill<St, CI, decltype(wc)::value><<<grid, kBlock, 0, stream>>>(
                n, ns, A->rowptr, A->col, static_cast<const St*>(val), S.off, S.sbase, static_cast<CI*>(S.col),
                static_cast<St*>(S.val), S.rows);
            return (int)MPG_OK;
        });
    });
    if (!st && S.nexc > 0) {
        // the flagged slices' rows as a CSR the copy owns (the caller's CSR
        // and values may be freed once the copy exists): row 64 e + lane of
        // the e-th flagged slice, entries copied in CSR order, runs of
        // adjacent flagged slices in one copy each
        std::vector<int32_t> xrp_h((size_t)S.nexc * kWave + 1, 0);
        std::vector<std::pair<int64_t, int64_t>> runs;  // (first entry, entry count) per run of flagged slices
        int64_t e = 0, at = 0;
        for (int s2 = 0; s2 < ns; ++s2) {
            if (spat_h[s2] > -2) continue;
            for (int l = 0; l < kWave; ++l) {
                const int r = s2 * kWave + l;
                const int64_t len = r < n ? (int64_t)rp[r + 1] - rp[r] : 0;
                at += len;
                xrp_h[(size_t)e * kWave + l + 1] = (int32_t)at;
            }
            const int64_t b0 = rp[s2 * kWave], b1 = rp[std::min(n, (s2 + 1) * kWave)];
            if (!runs.empty() && runs.back().first + runs.back().second == b0) runs.back().second += b1 - b0;
            else runs.emplace_back(b0, b1 - b0);
            ++e;
        }
        if (hipMalloc((void**)&S.xrp, xrp_h.size() * 4) != hipSuccess ||
            hipMalloc((void**)&S.xcol, (size_t)at * 4 + 256) != hipSuccess ||
            hipMalloc(&S.xval, (size_t)at * vsize + 256) != hipSuccess) {
            st = MPG_ERR_ALLOC;
        } else if (hipMemcpyAsync(S.xrp, xrp_h.data(), xrp_h.size() * 4, hipMemcpyHostToDevice, stream) != hipSuccess) {
            st = MPG_ERR_HIP;
        } else {
            int64_t dst = 0;
            for (const auto& rn : runs) {
                if (hipMemcpyAsync(S.xcol + dst, A->col + rn.first, (size_t)rn.second * 4, hipMemcpyDeviceToDevice,
                                   stream) != hipSuccess ||
                    hipMemcpyAsync(static_cast<char*>(S.xval) + dst * vsize,
                                   static_cast<const char*>(val) + rn.first * vsize, (size_t)rn.second * vsize,
                                   hipMemcpyDeviceToDevice, stream) != hipSuccess) {
                    st = MPG_ERR_HIP;
                    break;
                }
                dst += rn.second;
            }
        }
    }
    if (!st && !spat_h.empty()) {
        // implicit patterns in the copy's column type (int16 forms: the
        // offsets fit, since every slice's columns do)
        const size_t cb = (size_t)S.col_bytes();
        std::vector<char> pat_bytes(std::max<size_t>(pat_h.size(), 1) * cb + 64, 0);
        for (size_t t = 0; t < pat_h.size(); ++t) {
            const int32_t d = pat_h[t];
            if (cb == 4) {
                std::memcpy(pat_bytes.data() + t * 4, &d, 4);
            } else {
                const int16_t v = d == INT32_MIN ? (int16_t)INT16_MIN : (int16_t)d;
                std::memcpy(pat_bytes.data() + t * 2, &v, 2);
            }
        }
        S.npat = (int64_t)pat_h.size();
        if (hipMalloc((void**)&S.spat, spat_h.size() * 4 + 256) != hipSuccess ||
            hipMalloc(&S.pat, pat_bytes.size()) != hipSuccess)
            st = MPG_ERR_ALLOC;
        else if (hipMemcpyAsync(S.spat, spat_h.data(), spat_h.size() * 4, hipMemcpyHostToDevice, stream) !=
                     hipSuccess ||
                 hipMemcpyAsync(S.pat, pat_bytes.data(), pat_bytes.size(), hipMemcpyHostToDevice, stream) !=
                     hipSuccess)
            st = MPG_ERR_HIP;
    }
    S.col_slots = best - S.imp_slots;
    const char* shenv = std::getenv("MPG_SELL_SHARE");  // 0: every slice keeps its own column block
    if (!st && (S.c16 || S.c16s) && !(shenv && *shenv == '0')) st = sell_share_columns(S, off, spat_h, grid, stream);
    if (!st && hipStreamSynchronize(stream) != hipSuccess) st = MPG_ERR_HIP;
    if (st) sell_free(S);
    return st;
}

// Shared column blocks (after the fill): hash every stored slice's block,
// group equal (length, hash) pairs, verify each member against its group's
// first slice on the device, and keep one block per group in a compacted
// column array; coff[s] says where slice s reads its columns. Implicit
// slices (pattern loads) store none. A slice summed from the sub-CSR keeps
// a block of its own (its clamped loads still read one). Nothing changes
// unless at least 1 % of the stored slices share.
int sell_share_columns(SellCopy& S, const std::vector<int64_t>& off, const std::vector<int32_t>& spat_h, int grid,
                       hipStream_t stream) {
    const int ns = S.nslices;
    uint64_t* hash_d = nullptr;
    int32_t* rep_d = nullptr;
    int* bad_d = nullptr;
    int64_t* newoff_d = nullptr;
    void* col2 = nullptr;
    auto cleanup = [&](int st) {
        for (void* p : {(void*)hash_d, (void*)rep_d, (void*)bad_d, (void*)newoff_d}) (void)(p ? hipFree(p) : hipSuccess);
        if (st && col2) (void)hipFree(col2);
        return st;
    };
    std::vector<uint64_t> hash((size_t)ns);
    if (hipMalloc((void**)&hash_d, (size_t)ns * 8) != hipSuccess) return cleanup(MPG_ERR_ALLOC);
    int st = sell_dispatch(S, [&](auto ci, auto) {
        using CI = decltype(ci);
        k_sell_col_hash<CI><<<grid, kBlock, 0, stream>>>(ns, S.off, static_cast<const CI*>(S.col), hash_d);
        return (int)MPG_OK;
    });
    if (st || hipMemcpyAsync(hash.data(), hash_d, (size_t)ns * 8, hipMemcpyDeviceToHost, stream) != hipSuccess ||
        hipStreamSynchronize(stream) != hipSuccess)
        return cleanup(st ? st : MPG_ERR_HIP);
    std::vector<int32_t> rep((size_t)ns, -1);
    std::map<std::pair<int64_t, uint64_t>, int32_t> first;
    int64_t shared = 0, stored = 0;
    for (int s2 = 0; s2 < ns; ++s2) {
        if (!spat_h.empty() && spat_h[s2] >= 0) continue;  // implicit: no block
        ++stored;
        auto it = first.emplace(std::make_pair(off[s2 + 1] - off[s2], hash[s2]), s2).first;
        rep[s2] = it->second;
        shared += it->second != s2;
    }
    if (shared * 100 < stored || shared == 0) return cleanup(MPG_OK);
    if (hipMalloc((void**)&rep_d, (size_t)ns * 4) != hipSuccess || hipMalloc((void**)&bad_d, (size_t)ns * 4) != hipSuccess)
        return cleanup(MPG_ERR_ALLOC);
    std::vector<int> bad((size_t)ns, 0);
    if (hipMemcpyAsync(rep_d, rep.data(), (size_t)ns * 4, hipMemcpyHostToDevice, stream) != hipSuccess ||
        hipMemsetAsync(bad_d, 0, (size_t)ns * 4, stream) != hipSuccess)
        return cleanup(MPG_ERR_HIP);
    st = sell_dispatch(S, [&](auto ci, auto) {
        using CI = decltype(ci);
        k_sell_col_verify<CI><<<grid, kBlock, 0, stream>>>(ns, S.off, static_cast<const CI*>(S.col), rep_d, bad_d);
        return (int)MPG_OK;
    });
    if (st || hipMemcpyAsync(bad.data(), bad_d, (size_t)ns * 4, hipMemcpyDeviceToHost, stream) != hipSuccess ||
        hipStreamSynchronize(stream) != hipSuccess)
        return cleanup(st ? st : MPG_ERR_HIP);
    for (int s2 = 0; s2 < ns; ++s2)
        if (bad[s2]) rep[s2] = s2;  // a hash collision: its own block
    std::vector<int64_t> newoff((size_t)ns, -1), coff((size_t)ns, 0);
    int64_t total = 0;
    shared = 0;
    for (int s2 = 0; s2 < ns; ++s2)
        if (rep[s2] == s2) {
            newoff[s2] = total;
            total += off[s2 + 1] - off[s2];
        }
    for (int s2 = 0; s2 < ns; ++s2)
        if (rep[s2] >= 0) {
            coff[s2] = newoff[rep[s2]];
            shared += rep[s2] != s2;
        }
    if (shared * 100 < stored) return cleanup(MPG_OK);
    const size_t cb = (size_t)S.col_bytes();
    if (hipMalloc((void**)&newoff_d, (size_t)ns * 8) != hipSuccess || hipMalloc(&col2, (size_t)total * cb + 256) != hipSuccess ||
        hipMalloc((void**)&S.coff, (size_t)ns * 8 + 256) != hipSuccess)
        return cleanup(MPG_ERR_ALLOC);
    if (hipMemcpyAsync(newoff_d, newoff.data(), (size_t)ns * 8, hipMemcpyHostToDevice, stream) != hipSuccess ||
        hipMemcpyAsync(S.coff, coff.data(), (size_t)ns * 8, hipMemcpyHostToDevice, stream) != hipSuccess ||
        hipMemsetAsync(col2, 0, (size_t)total * cb + 256, stream) != hipSuccess)
        return cleanup(MPG_ERR_HIP);
    st = sell_dispatch(S, [&](auto ci, auto) {
        using CI = decltype(ci);
        k_sell_col_gather<CI><<<grid, kBlock, 0, stream>>>(ns, S.off, static_cast<const CI*>(S.col), newoff_d,
                                                          static_cast<CI*>(col2));
        return (int)MPG_OK;
    });
    if (st || hipStreamSynchronize(stream) != hipSuccess) return cleanup(st ? st : MPG_ERR_HIP);
    (void)hipFree(S.col);
    S.col = col2;
    S.nshared = shared;
    S.col_slots = total;
    return cleanup(MPG_OK);
}

int64_t sell_matrix_bytes(const SellCopy& S) {
    if (S.nslices == 0) return 0;
    const int64_t vbytes = S.vtype == MPG_F64 ? 8 : S.vtype == MPG_F32 ? 4 : 2;
    const int64_t steps = S.padded / ((int64_t)kWave * S.W);
    // every slot's value; the columns of slots outside implicit slices (the
    // shared patterns are a few cache lines); int64 slice offsets; the
    // pattern indices; the stepped form's bases; a sorted copy's row numbers
    // (shared column blocks: the distinct blocks once, plus the per-slice
    // column starts)
    return S.padded * vbytes + S.col_slots * S.col_bytes() + S.npat * S.col_bytes() +
           ((int64_t)S.nslices + 1) * 8 + (S.spat ? (int64_t)S.nslices * 4 : 0) + (S.c16s ? steps * S.W * 4 : 0) +
           (S.coff ? (int64_t)S.nslices * 8 : 0) + (S.rows ? (int64_t)S.nslices * kWave * 4 : 0);
}

void sell_free(SellCopy& S) {
    if (S.sbase) (void)hipFree(S.sbase);
    if (S.spat) (void)hipFree(S.spat);
    if (S.pat) (void)hipFree(S.pat);
    if (S.off) (void)hipFree(S.off);
    if (S.col) (void)hipFree(S.col);
    if (S.val) (void)hipFree(S.val);
    if (S.xrp) (void)hipFree(S.xrp);
    if (S.xcol) (void)hipFree(S.xcol);
    if (S.xval) (void)hipFree(S.xval);
    if (S.coff) (void)hipFree(S.coff);
    if (S.rows) (void)hipFree(S.rows);
    S = SellCopy{};
}

}  // namespace mpg

struct mpg_sell {
    mpg_ctx* ctx = nullptr;
    int cols = 0;
    SellCopy S;  // owns all its device memory (the flagged slices' rows included)
};

namespace {

template <class X, class St, bool NORM = false>
int sell_spmv_impl(mpg_ctx* ctx, mpg_sell* A, X alpha, const X* x, X beta, X* y,
                   const ScalarProgram& prog = ScalarProgram{}, const NormArgs<X>& nm = NormArgs<X>{}) {
    if (!ctx || !A) return MPG_ERR_ARG;
    const SellCopy& S = A->S;
    if (S.nslices == 0) {
        if (NORM) return MPG_ERR_ARG;
        return prog.count > 0 ? mpg_scalar_program(ctx, prog.ops, prog.count) : MPG_OK;
    }
    const int grid = (S.nslices + kBlock / kWave - 1) / (kBlock / kWave) + (prog.count > 0 ? 1 : 0);
    const int be = sell_uniform(S) ? sell_pair(S) : 0;
    int st = sell_dispatch(S, [&](auto ci, auto wc) {
        using CI = decltype(ci);
        return sell_dispatch_win(S.win, [&](auto wn) {
            constexpr int Wc = decltype(wc)::value;
            constexpr bool WN = decltype(wn)::value;
            // two slices per wave (MPG_SURFACE_PAIR=0: one)
            const char* pe = std::getenv("MPG_SURFACE_PAIR");
            if constexpr (std::is_same_v<CI, int16_t> && (Wc == 2 || Wc == 4)) if (be && !(pe && *pe == '0')) {
                const int grid2 = (S.nslices + 2 * (kBlock / kWave) - 1) / (2 * (kBlock / kWave)) + (prog.count > 0 ? 1 : 0);
                auto go2 = [&](auto kern) {
                    kern<<<grid2, kBlock, 0, ctx->stream>>>(
                        S.n, A->cols, S.nslices, static_cast<const int16_t*>(S.col), static_cast<const St*>(S.val),
                        S.sbase, S.spat, S.coff, static_cast<const int16_t*>(S.pat), x, alpha, beta, y, S.ustride,
                        sell_xcd_order(S) ? 1 : 0, prog, nm);
                    return (int)MPG_OK;
                };
                if (be == 8) return go2(k_sell_spmv2<X, St, Wc, WN, 8, NORM>);
                if constexpr (Wc == 2) if (be == 10) return go2(k_sell_spmv2<X, St, Wc, WN, 10, NORM>);
                if (be == 12) return go2(k_sell_spmv2<X, St, Wc, WN, 12, NORM>);
            }
            auto go = [&](auto kern) {
                kern<<<grid, kBlock, 0, ctx->stream>>>(
                    S.n, A->cols, S.nslices, S.off, static_cast<const CI*>(S.col), static_cast<const St*>(S.val),
                    S.sbase, S.spat, S.coff, static_cast<const CI*>(S.pat), S.xrp, S.xcol, static_cast<const St*>(S.xval), x,
                    alpha, beta, y, S.ustride, sell_xcd_order(S) ? 1 : 0, prog, S.rows, nm);
                return (int)MPG_OK;
            };
            return sell_uniform(S) ? go(k_sell_spmv<X, St, CI, Wc, WN, true, NORM>)
                                   : go(k_sell_spmv<X, St, CI, Wc, WN, false, NORM>);
        });
    });
    if (st) return st;
    MPG_LAUNCH_CHECK(ctx);
    return MPG_OK;
}

}  // namespace

extern "C" {

int mpg_sell_create(mpg_ctx_t ctx, mpg_csr_t A, int32_t vtype, const void* vals, int32_t format, mpg_sell_t* out) {
    if (!ctx || !A || !out || (A->nnz > 0 && !vals) || format < 0 || format > 2) return MPG_ERR_ARG;
    if (vtype != MPG_F64 && vtype != MPG_F32 && vtype != MPG_F16) return MPG_ERR_UNSUPPORTED;
    *out = nullptr;
    mpg_sell* h = new (std::nothrow) mpg_sell();
    if (!h) return MPG_ERR_ALLOC;
    h->ctx = ctx;
    h->cols = A->cols;
    if (int st = sell_build(ctx, A, vtype, vals, format, h->S)) {
        delete h;
        return st;
    }
    if (h->S.nslices == 0) {  // padding would not pay: keep CSR
        delete h;
        return MPG_OK;
    }
    *out = h;
    return MPG_OK;
}

int mpg_sell_destroy(mpg_sell_t A) {
    if (!A) return MPG_OK;
    if (A->ctx) (void)hipStreamSynchronize(A->ctx->stream);
    sell_free(A->S);
    delete A;
    return MPG_OK;
}

int mpg_sell_layout(mpg_sell_t A, int32_t* vec_width, int32_t* col_bytes, int64_t* stored, int32_t* window) {
    if (!A) return MPG_ERR_ARG;
    if (vec_width) *vec_width = A->S.W;
    if (col_bytes) *col_bytes = A->S.col_bytes();
    if (stored) *stored = A->S.padded;
    if (window) *window = A->S.win ? 1 : 0;
    return MPG_OK;
}

int64_t mpg_sell_shared_slices(mpg_sell_t A) { return A ? A->S.nshared : -1; }

int64_t mpg_sell_bytes(mpg_sell_t A) { return A ? sell_matrix_bytes(A->S) : -1; }

int mpg_sell_columns(mpg_sell_t A, int32_t* form, int64_t* csr_slices, int64_t* implicit_slices) {
    if (!A) return MPG_ERR_ARG;
    if (form) *form = A->S.c16 ? 1 : A->S.c16s ? 2 : 0;
    if (csr_slices) *csr_slices = A->S.nexc;
    if (implicit_slices) *implicit_slices = A->S.nimp;
    return MPG_OK;
}

int mpg_sell_spmv_f64(mpg_ctx_t c, mpg_sell_t A, double alpha, const double* x, double beta, double* y) {
    if (A && A->S.vtype != MPG_F64) return MPG_ERR_ARG;
    return sell_spmv_impl<double, double>(c, A, alpha, x, beta, y);
}
int mpg_sell_spmv_f32(mpg_ctx_t c, mpg_sell_t A, float alpha, const float* x, float beta, float* y) {
    if (A && A->S.vtype != MPG_F32) return MPG_ERR_ARG;
    return sell_spmv_impl<float, float>(c, A, alpha, x, beta, y);
}
int mpg_sell_spmv_f16f32(mpg_ctx_t c, mpg_sell_t A, float alpha, const float* x, float beta, float* y) {
    if (A && A->S.vtype != MPG_F16) return MPG_ERR_ARG;
    return sell_spmv_impl<float, uint16_t>(c, A, alpha, x, beta, y);
}
int mpg_sell_spmv_prog_f64(mpg_ctx_t c, mpg_sell_t A, double alpha, const double* x, double beta, double* y,
                           const mpg_scalar_op* ops, int32_t nops) {
    ScalarProgram prog;
    if ((A && A->S.vtype != MPG_F64) || make_scalar_program(ops, nops, prog) != MPG_OK) return MPG_ERR_ARG;
    return sell_spmv_impl<double, double>(c, A, alpha, x, beta, y, prog);
}
int mpg_sell_spmv_prog_f32(mpg_ctx_t c, mpg_sell_t A, float alpha, const float* x, float beta, float* y,
                           const mpg_scalar_op* ops, int32_t nops) {
    ScalarProgram prog;
    if ((A && A->S.vtype != MPG_F32) || make_scalar_program(ops, nops, prog) != MPG_OK) return MPG_ERR_ARG;
    return sell_spmv_impl<float, float>(c, A, alpha, x, beta, y, prog);
}

}  // extern "C"

namespace {
template <class X, int VT>
int sell_spmv_norm(mpg_ctx* c, mpg_sell* A, int32_t nparts, X* h, const X* w, X* v, X alpha, X* y,
                   const mpg_scalar_op* ops, int32_t nops) {
    ScalarProgram prog;
    if (!c || !A || A->S.vtype != VT || !h || !w || !v || !y || nparts < 1 || nparts > kBlock || A->cols != A->S.n ||
        make_scalar_program(ops, nops, prog) != MPG_OK)
        return MPG_ERR_ARG;
    NormArgs<X> nm;
    nm.part = c->red_ws;
    nm.nparts = nparts;
    nm.h = h;
    nm.v = v;
    return sell_spmv_impl<X, X, true>(c, A, alpha, w, X(0), y, prog, nm);
}
}  // namespace

extern "C" {

int mpg_sell_spmv_norm_f64(mpg_ctx_t c, mpg_sell_t A, int32_t nparts, double* h, const double* w, double* v,
                           double alpha, double* y, const mpg_scalar_op* ops, int32_t nops) {
    return sell_spmv_norm<double, MPG_F64>(c, A, nparts, h, w, v, alpha, y, ops, nops);
}
int mpg_sell_spmv_norm_f32(mpg_ctx_t c, mpg_sell_t A, int32_t nparts, float* h, const float* w, float* v,
                           float alpha, float* y, const mpg_scalar_op* ops, int32_t nops) {
    return sell_spmv_norm<float, MPG_F32>(c, A, nparts, h, w, v, alpha, y, ops, nops);
}

}  // extern "C"
