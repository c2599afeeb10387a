// ILU(0) factorisation, sync-free triangular solves and ILU-Jacobi sweeps
// on gfx950 (include/mpgmres/ilu.h).
//
// Factorisation and solves hand rows out in order through an atomic ticket:
// a wave64 (factorisation) or a lane (solves) takes the next row, waits
// only for the rows that row reads, computes it and stores it write-through;
// the factorisation then raises the row's flag (handoff.hpp), the solves
// let the stored value itself be the flag (k_ilu_trsv_tagged). A row only
// ever waits for rows taken earlier by running waves, so the schedule
// always progresses; every wait is bounded (a fault is recorded instead of
// hanging the GPU).
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <limits>
#include <new>
#include <type_traits>
#include <vector>

#include "handoff.hpp"
#include "internal.hpp"
#include "mpgmres/ilu.h"

using namespace mpg;

namespace {

constexpr int kRowCap = 512;                 // entries of one row staged in LDS
constexpr int kUpCap = 128;                  // pivot rows' upper entries staged per row (else read in place)
constexpr int kWaves = kBlock / kWave;       // 4 rows in flight per workgroup
constexpr int kPersistGroups = 2048;         // 8 workgroups per CU
// level-scheduled solves: few spinning waves. 64 workgroups (one per CU on a
// quarter of the chip, 256 waves) solve LAP-1M's L and U in 3.0 ms; 2048
// workgroups flood the memory system with flag polls (waits past 2 s at
// 90^3 and up), 512: 5.1 ms, 256: 3.6 ms (tools/ilu_debug.py). Loading the
// rows' values with sc1 loads instead of the wave's one agent acquire gained
// 4 %: a hop (drain, flag, poll, loads) is ~5 us either way.
constexpr int kSolveGroups = 64;
constexpr uint64_t kDeadline = 3000000000ull;  // 30 s of the 100 MHz clock: a wave gives up (fault 2)

// sync block layout (ints): [0, n) factorisation flags, then tickets at
// n + 0 / 32 / 64 (factorisation, L solve, U solve: separate 128-B lines),
// the fault word at n + 128
inline size_t sync_ints(int n) { return (size_t)n + 160; }

// ---------------------------------------------------------------- set-up
__global__ void k_find_diag(int n, const int* __restrict__ rowptr, const int* __restrict__ col, int* __restrict__ diag,
                            int* __restrict__ bad) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    int d = -1;
    for (int k = rowptr[i]; k < rowptr[i + 1]; ++k)
        if (col[k] == i) {
            d = k;
            break;
        }
    diag[i] = d;
    if (d < 0) atomicOr(bad, 1);
    if (rowptr[i + 1] - rowptr[i] > kRowCap) atomicOr(bad, 2);
}

// max_i sum_j |a_ij| (rows summed in CSR order, as ilu0_impl's parallel_reduce)
__global__ void k_abs_rowsum_max(int n, const int* __restrict__ rowptr, const double* __restrict__ v,
                                 unsigned long long* __restrict__ out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    double s = 0;
    if (i < n)
        for (int k = rowptr[i]; k < rowptr[i + 1]; ++k) s += fabs(v[k]);
    s = wave_max(s);
    // non-negative doubles order like their bit patterns
    if ((threadIdx.x & (kWave - 1)) == 0) atomicMax(out, (unsigned long long)__double_as_longlong(s));
}

// ---------------------------------------------------------------- factorisation
// ilu0_impl (kernels_mkl.cpp:416-500) row by row, in fp64. The row is staged
// in LDS; its elimination steps run in column order, and step k updates each
// later entry of the row with the matching entry of row k's upper part. The
// sorted merge of the reference pairs equal columns in order, so the e-th
// entry, the r-th of its column in the row's remaining run, meets the r-th
// entry of that column in row k (duplicates handled as the merge does).
// Products and differences are not contracted, as in the reference loop.
// Rows are handed out in the L solve's dependency-level order (a row reads
// exactly the rows its L part names): in row order the rows in flight on a
// natural-order 3-D stencil were one chain of x-line hand-offs wide.
#pragma clang fp contract(off)
__global__ __launch_bounds__(kBlock) void k_ilu0_factor(int n, const int* __restrict__ rowptr,
                                                        const int* __restrict__ col, const int* __restrict__ diag,
                                                        double* lu, double eps,
                                                        const unsigned long long* __restrict__ rowmax, int* done,
                                                        unsigned* ticket, int* err, const int* __restrict__ ord) {
    __shared__ double vs[kWaves][kRowCap];
    __shared__ int cs[kWaves][kRowCap];
    __shared__ double uvs[kWaves][kUpCap];  // staged upper parts of the pivot rows
    __shared__ int ucs[kWaves][kUpCap];
    __shared__ int uos[kWaves][kWave], kds[kWaves][kWave];
    const int lane = threadIdx.x & (kWave - 1), wid = threadIdx.x / kWave;
    double* v = vs[wid];
    int* c = cs[wid];
    double* uv = uvs[wid];
    int* uc = ucs[wid];
    int* uo = uos[wid];
    int* ukd = kds[wid];
    const double alpha = __longlong_as_double((long long)*rowmax) * eps;
    const uint64_t t_start = __builtin_amdgcn_s_memrealtime();
    for (;;) {
        if (__builtin_amdgcn_s_memrealtime() - t_start > kDeadline) {
            if (lane == 0) __hip_atomic_store((gu32*)err, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            break;
        }
        int t = 0;
        if (lane == 0) t = (int)__hip_atomic_fetch_add((gu32*)ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        t = __shfl(t, 0, kWave);
        if (t >= n) break;
        const int row = ord[t];  // rows in dependency-level order
        const int rs = rowptr[row], len = rowptr[row + 1] - rs, dpos = diag[row] - rs;
        for (int e = lane; e < len; e += kWave) {
            c[e] = col[rs + e];
            v[e] = lu[rs + e];  // this row's values: written by nobody else before its flag
        }
        wave_lds_sync();
        if (row > 0) {  // the reference loop starts at row 1 (no elimination, no boost on row 0)
            for (int e = lane; e < dpos; e += kWave) wait_flag(done + c[e], err);
            acquire_agent();
            // Stage the pivot rows' upper parts (columns, values) and pivots
            // with all lanes at once (dpos <= 64, <= kUpCap entries): one load
            // round trip for all of them, so the elimination steps below run
            // from LDS and registers instead of a chain of dependent global
            // loads per step (~8 us a row on a chain). Same values, same
            // search, same arithmetic: identical factors.
            int my_kd = 0, my_cnt = 0;
            double my_piv = 1.0;
            if (dpos <= kWave && lane < dpos) {
                const int k = c[lane];
                my_kd = diag[k];
                my_cnt = rowptr[k + 1] - my_kd - 1;
                my_piv = lu[my_kd];
            }
            int incl = my_cnt;
#pragma unroll
            for (int o = 1; o < kWave; o <<= 1) {
                const int t = __shfl_up(incl, o, kWave);
                if (lane >= o) incl += t;
            }
            const int tot = __shfl(incl, kWave - 1, kWave);
            const int my_off = incl - my_cnt;
            const bool staged = dpos <= kWave && tot <= kUpCap;
            if (staged) {
                uo[lane] = my_off;
                ukd[lane] = my_kd;
                wave_lds_sync();
                for (int f = lane; f < tot; f += kWave) {
                    int lo = 0, hi = dpos;  // the last pivot row whose entries start at or before f
                    while (hi - lo > 1) {
                        const int mid = (lo + hi) >> 1;
                        if (uo[mid] <= f) lo = mid;
                        else hi = mid;
                    }
                    const int src = ukd[lo] + 1 + (f - uo[lo]);
                    uc[f] = col[src];
                    uv[f] = lu[src];
                }
                wave_lds_sync();
            }
            for (int p = 0; p < dpos; ++p) {
                int b0, b1;  // the pivot row's upper entries: [b0, b1) of uc / uv, or of col / lu
                double pivot;
                if (staged) {
                    b0 = __shfl(my_off, p, kWave);
                    b1 = b0 + __shfl(my_cnt, p, kWave);
                    pivot = __shfl(my_piv, p, kWave);
                } else {
                    const int k = c[p];
                    const int kd = diag[k];
                    b0 = kd + 1;
                    b1 = rowptr[k + 1];
                    pivot = lu[kd];
                }
                const int* __restrict__ bc = staged ? uc : col;
                const double* bv = staged ? uv : lu;
                const double factor = v[p] / pivot;
                wave_lds_sync();
                if (lane == 0) v[p] = factor;
                for (int e = p + 1 + lane; e < len; e += kWave) {
                    const int cc = c[e];
                    int f = e;
                    while (f > p + 1 && c[f - 1] == cc) --f;
                    int lo = b0, hi = b1;
                    while (lo < hi) {
                        const int mid = (lo + hi) >> 1;
                        if (bc[mid] < cc) lo = mid + 1;
                        else hi = mid;
                    }
                    const int t = lo + (e - f);
                    if (t < b1 && bc[t] == cc) {
                        const double prod = factor * bv[t];
                        v[e] = v[e] - prod;
                    }
                }
                wave_lds_sync();
            }
            if (lane == 0) {
                double d = v[dpos];
                if (d >= 0) {
                    if (d < alpha) d = alpha;
                } else {
                    if (d > -alpha) d = -alpha;
                }
                v[dpos] = d;
            }
            wave_lds_sync();
        }
        for (int e = lane; e < len; e += kWave) store_wt(lu + rs + e, v[e]);
        drain_stores();
        if (lane == 0) set_flag(done + row);
    }
}
#pragma clang fp contract(on)

template <class T>
__global__ void k_round_factors(int64_t nnz, const double* __restrict__ lu64, T* __restrict__ lu) {
    for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < nnz; k += (int64_t)gridDim.x * blockDim.x)
        lu[k] = (T)lu64[k];
}

// diag(i) = 1/vals(j) on the rounded factors (types.hpp:305-316)
template <class T>
__global__ void k_dinv(int n, const int* __restrict__ diag, const T* __restrict__ lu, T* __restrict__ dinv) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) dinv[i] = 1 / lu[diag[i]];
}

// ---------------------------------------------------------------- triangular solves
// out := L^-1 rhs (unit lower) or U^-1 rhs (upper), level-scheduled and
// sync-free. mpg_ilu0_create sorts the rows by dependency level (a row's
// level is one more than the highest level among the rows its off-diagonal
// entries read) and cuts every level into chunks of <= 64 rows, so the rows
// of a chunk never depend on each other. A wave takes the next chunk from an
// atomic ticket (chunks in level order: a wave only waits for rows of
// earlier chunks, taken by running waves, so the schedule always
// progresses), and each lane solves one row, x_i = T((b_i - sum_j a_ij x_j)
// [/ u_ii]) with the sum in fp64 in CSR order, rounded once.
//
// The VALUE is its own flag: the output vector starts filled with a tag (a
// signalling-NaN bit pattern that no arithmetic produces -- results are
// quiet NaNs at worst, and a result equal to the tag is stored as the
// canonical NaN), a lane polls the values of the rows it reads (relaxed
// agent-scope loads, four dependencies in flight at once) until none is the
// tag, and stores its own value write-through. The lane that reads rhs[row]
// overwrites it with the tag, so after the L solve x is the tagged output
// buffer of the U solve.
//
// History (LAP-1M, mixed CGS GMRES(30) with ILU(0), tools/prec_bench.py):
// one row per wave and a ticket per row, 2048 workgroups: ~40 ms per L + U;
// one row per lane with a done-flag per row (store, drain, flag store, flag
// poll, agent acquire, value loads: ~5 us a level hop): 3.0 ms, 318 it/s;
// the value as flag (store, value poll): 746 it/s, ~2.2 us a hop.
template <class T>
struct TrsvTag;
template <>
struct TrsvTag<double> {
    typedef unsigned long long U;
    typedef gu64 G;
    static constexpr U kBits = 0x7FF5A5A5A5A5A5A5ull;
    static constexpr U kQuiet = 0x7FF8000000000000ull;
    __device__ static double val(U u) { return __longlong_as_double((long long)u); }
    __device__ static U bits(double v) { return (U)__double_as_longlong(v); }
};
template <>
struct TrsvTag<float> {
    typedef unsigned U;
    typedef gu32 G;
    static constexpr U kBits = 0x7FA5A5A5u;
    static constexpr U kQuiet = 0x7FC00000u;
    __device__ static float val(U u) { return __uint_as_float(u); }
    __device__ static U bits(float v) { return __float_as_uint(v); }
};

template <class T>
__device__ __forceinline__ typename TrsvTag<T>::U poll_tagged(const T* p, int* err, uint64_t bound) {
    typedef TrsvTag<T> Tg;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    typename Tg::U v;
    while ((v = __hip_atomic_load((const typename Tg::G*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) == Tg::kBits) {
        __builtin_amdgcn_s_sleep(1);
        if (__builtin_amdgcn_s_memrealtime() - t0 > bound) {  // give up: the tag is a NaN, the row goes on
            __hip_atomic_store((gu32*)err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            break;
        }
    }
    return v;
}

constexpr int kTagBatch = 4;  // dependencies polled together
template <class T, bool UPPER>
__global__ __launch_bounds__(kBlock) void k_ilu_trsv_tagged(int nchunks, const int* __restrict__ chunk,
                                                            const int* __restrict__ ord,
                                                            const int* __restrict__ rowptr,
                                                            const int* __restrict__ col,
                                                            const int* __restrict__ diag, const T* __restrict__ lu,
                                                            T* rhs, T* out, unsigned* ticket, int* err,
                                                            uint64_t wait_bound) {
    typedef TrsvTag<T> Tg;
    typedef typename Tg::U U;
    const int lane = threadIdx.x & (kWave - 1);
    const uint64_t t_start = __builtin_amdgcn_s_memrealtime();
    for (;;) {
        if (__builtin_amdgcn_s_memrealtime() - t_start > kDeadline) {
            if (lane == 0) __hip_atomic_store((gu32*)err, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            break;
        }
        int t = 0;
        if (lane == 0) t = (int)__hip_atomic_fetch_add((gu32*)ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        t = __shfl(t, 0, kWave);
        if (t >= nchunks) break;
        const int c0 = chunk[t], cnt = chunk[t + 1] - c0;
        if (lane < cnt) {
            const int row = ord[c0 + lane], d = diag[row];
            const int j0 = UPPER ? d + 1 : rowptr[row];
            const int j1 = UPPER ? rowptr[row + 1] : d;
            const T b = rhs[row];
            const T piv = UPPER ? lu[d] : T(1);
            rhs[row] = TrsvTag<T>::val(Tg::kBits);
            double s = 0.0;
            for (int j = j0; j < j1; j += kTagBatch) {
                int c[kTagBatch];
                U v[kTagBatch];
                T a[kTagBatch];
#pragma unroll
                for (int q = 0; q < kTagBatch; ++q) c[q] = j + q < j1 ? col[j + q] : -1;
#pragma unroll
                for (int q = 0; q < kTagBatch; ++q) {
                    v[q] = c[q] >= 0 ? __hip_atomic_load((const typename Tg::G*)(out + c[q]), __ATOMIC_RELAXED,
                                                         __HIP_MEMORY_SCOPE_AGENT)
                                     : U(0);
                    a[q] = c[q] >= 0 ? lu[j + q] : T(0);
                }
#pragma unroll
                for (int q = 0; q < kTagBatch; ++q)
                    if (c[q] >= 0 && v[q] == Tg::kBits) v[q] = poll_tagged(out + c[q], err, wait_bound);
#pragma unroll
                for (int q = 0; q < kTagBatch; ++q)
                    if (c[q] >= 0) s += (double)a[q] * (double)Tg::val(v[q]);
            }
            double r = (double)b - s;
            if (UPPER) r = r / (double)piv;
            T res = (T)r;
            if (Tg::bits(res) == Tg::kBits) res = Tg::val(Tg::kQuiet);
            store_wt(out + row, res);
        }
    }
}

// out := tag, and the two solve tickets (32 ints apart) zeroed
template <class T>
__global__ void k_trsv_tag_fill(int n, T* __restrict__ out, unsigned* __restrict__ tickets) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = TrsvTag<T>::val(TrsvTag<T>::kBits);
    if (i < 2) tickets[32 * i] = 0u;
}

// dst := src, src := tag (a serial solve next to a tagged one)
template <class T>
__global__ void k_trsv_tag_move(int n, T* __restrict__ src, T* __restrict__ dst) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    dst[i] = src[i];
    src[i] = TrsvTag<T>::val(TrsvTag<T>::kBits);
}

// The same solve for matrices whose dependency levels hold few rows (banded:
// every level one row, depth n), where the level schedule pays a flag
// hand-off (~2 us) per row: ONE workgroup runs the recurrence serially.
// Lane 0 of wave 0 solves the rows of a stage in processing order from LDS,
// keeping the x values it produced in an LDS ring of kRing rows
// (eligibility: every dependency lies within kRing rows); waves 1-3 stage
// the next stage's operands meanwhile (right-hand sides, pivots, and each
// row's off-diagonal entries as ring slots + values, padded to a multiple of
// kPass with zero products on a zero slot). The chain per row is then one
// LDS round trip (the x reads, issued after the previous row's ring write)
// plus the fp64 arithmetic: the next row's slots, values and right-hand side
// are read while the current row finishes. The arithmetic is the level
// kernel's -- fp64 sum in CSR order, rounded once; a padded term adds an
// exact +0 (the sum never holds -0) -- so both modes give identical results.
// P (<= kPass): entries per pass, the direction's longest row (BAND-100k:
// 5 for L, 4 for U), so rows are padded to what the matrix needs: one lane
// runs every padded term, and the chain is bound by its instruction count.
constexpr int kRing = 2048, kStageRows = 256, kStageEnt = 1536, kPass = 8;
template <class T>
struct SerialStage {
    T rhs[kStageRows + 1];
    T piv[kStageRows + 1];
    int eend[kStageRows + 1];        // end of each row's padded entries
    uint16_t slot[kStageEnt + kPass];  // ring slot of each entry's column (kRing: the zero slot)
    T elu[kStageEnt + kPass];
};

template <class T, bool UPPER, int P>
__global__ __launch_bounds__(kBlock) void k_ilu_trsv_serial(int n, int nstages, const int* __restrict__ stage,
                                                            const int* __restrict__ eoff,
                                                            const int* __restrict__ rowptr,
                                                            const int* __restrict__ col, const int* __restrict__ diag,
                                                            const T* __restrict__ lu, T* __restrict__ x) {
    __shared__ T ring[kRing + 1];
    __shared__ SerialStage<T> buf[2];
    auto row_of = [&](int p) { return UPPER ? n - 1 - p : p; };
    // waves 1-3: the operands of stage t into buf[t & 1]
    auto load = [&](int t) {
        SerialStage<T>& B = buf[t & 1];
        const int p0 = stage[t], p1 = stage[t + 1], e0 = eoff[p0];
        for (int p = p0 + (int)threadIdx.x - kWave; p < p1; p += kBlock - kWave) {
            const int row = row_of(p), d = diag[row];
            const int j0 = UPPER ? d + 1 : rowptr[row], j1 = UPPER ? rowptr[row + 1] : d;
            const int eb = eoff[p] - e0, ee = eoff[p + 1] - e0;
            B.rhs[p - p0] = x[row];
            if (UPPER) B.piv[p - p0] = lu[d];
            B.eend[p - p0] = ee;
            int e = eb;
            for (int j = j0; j < j1; ++j, ++e) {
                B.slot[e] = (uint16_t)(col[j] & (kRing - 1));
                B.elu[e] = lu[j];
            }
            for (; e < ee; ++e) {
                B.slot[e] = (uint16_t)kRing;
                B.elu[e] = T(0);
            }
        }
    };
    if (threadIdx.x == 0) ring[kRing] = T(0);
    if (threadIdx.x >= kWave) load(0);
    __syncthreads();
    for (int t = 0; t < nstages; ++t) {
        if (threadIdx.x >= kWave) {
            if (t + 1 < nstages) load(t + 1);
        } else if (threadIdx.x == 0) {
            const SerialStage<T>& B = buf[t & 1];
            const int p0 = stage[t], p1 = stage[t + 1];
            // row p's operands, read one row ahead
            int eb = 0, ee = B.eend[0];
            T rhs = B.rhs[0], piv = UPPER ? B.piv[0] : T(1);
            int sl[P];
            T a[P];
#pragma unroll
            for (int k = 0; k < P; ++k) {
                sl[k] = B.slot[k];
                a[k] = B.elu[k];
            }
            for (int p = p0; p < p1; ++p) {
                T xv[P];
#pragma unroll
                for (int k = 0; k < P; ++k) xv[k] = ring[sl[k]];
                double s = 0.0;
#pragma unroll
                for (int k = 0; k < P; ++k) s += (double)a[k] * (double)xv[k];
                for (int e = eb + P; e < ee; e += P) {  // rows of more than P entries
#pragma unroll
                    for (int k = 0; k < P; ++k) xv[k] = ring[B.slot[e + k]];
#pragma unroll
                    for (int k = 0; k < P; ++k) s += (double)B.elu[e + k] * (double)xv[k];
                }
                // the next row's operands (past the stage's last row: unused reads within the arrays)
                const int q = p + 1 - p0;
                const int nb = ee, ne = B.eend[q];
                const T nrhs = B.rhs[q], npiv = UPPER ? B.piv[q] : T(1);
#pragma unroll
                for (int k = 0; k < P; ++k) {
                    sl[k] = B.slot[nb + k];
                    a[k] = B.elu[nb + k];
                }
                double r = (double)rhs - s;
                if (UPPER) r = r / (double)piv;
                const int row = row_of(p);
                const T v = (T)r;
                ring[row & (kRing - 1)] = v;
                x[row] = v;
                eb = nb;
                ee = ne;
                rhs = nrhs;
                piv = npiv;
            }
        }
        __syncthreads();
    }
}

// ---------------------------------------------------------------- ILU-Jacobi
// One Jacobi sweep on L (x_new = x + (b - (x + L_s x))) or on U
// (x_new = x + d∘(b - U x)), with the reference's operation order
// (ilu_jacobi_mv + axpy / gdmv, kernels.hpp:171-248); row sums in fp64.
template <class T, bool UPPER>
__global__ void k_ilu_jacobi_sweep(int n, const int* __restrict__ rowptr, const int* __restrict__ col,
                                   const int* __restrict__ diag, const T* __restrict__ lu,
                                   const T* __restrict__ dinv, const T* __restrict__ b, const T* __restrict__ xo,
                                   T* __restrict__ xn) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int d = diag[i];
    if (!UPPER) {
        double s = (double)xo[i];
        for (int j = rowptr[i]; j < d; ++j) s += (double)lu[j] * (double)xo[col[j]];
        const T sum = (T)s;
        const T t = T(1) * b[i] + T(-1) * sum;  // temp = beta*temp + alpha*sum
        xn[i] = T(1) * t + xo[i];               // axpy(1.0, temp, x)
    } else {
        double s = 0.0;
        for (int j = d; j < rowptr[i + 1]; ++j) s += (double)lu[j] * (double)xo[col[j]];
        const T sum = (T)s;
        const T t = T(1.0) * b[i] + T(-1.0) * sum;
        xn[i] = T(1) * xo[i] + T(1) * dinv[i] * t;  // gdmv(1.0, diag, temp, 1.0, x)
    }
}

}  // namespace

struct mpg_ilu {
    mpg_ctx* ctx = nullptr;
    const mpg_csr* A = nullptr;
    int n = 0;
    int64_t nnz = 0;
    int type = 0;                // 0 fp64, 1 fp32
    double* lu64 = nullptr;      // fp64 factors
    float* lu32 = nullptr;       // fp32 factors (type 1)
    int* diag = nullptr;
    void* dinv = nullptr;
    int* sync = nullptr;
    uint64_t wait_bound = kWaitBound;  // per-wait bound of the level-scheduled solves (test hook)
    void* w[2] = {nullptr, nullptr};  // ILU-Jacobi: right-hand side and the second sweep buffer
    void* tagbuf = nullptr;           // tagged solves: L^-1 b between the two directions
    unsigned long long* scratch = nullptr;
    // level schedules of the two triangular solves: rows by level, and
    // chunk starts (<= 64 rows, never across a level) into that order
    int* ord[2] = {nullptr, nullptr};
    int* chunk[2] = {nullptr, nullptr};
    int nchunks[2] = {0, 0};
    int levels[2] = {0, 0};
    // serial mode (few rows per level): stage starts and off-diagonal entry
    // offsets in processing order
    bool serial[2] = {false, false};
    int* stage[2] = {nullptr, nullptr};
    int* eoff[2] = {nullptr, nullptr};
    int nstages[2] = {0, 0};
    int spass[2] = {kPass, kPass};  // entries per pass of each serial solve

    size_t tsize() const { return type == 0 ? 8 : 4; }
    void* values() const { return type == 0 ? (void*)lu64 : (void*)lu32; }
    unsigned* ticket(int which) { return reinterpret_cast<unsigned*>(sync + (size_t)n + 32 * which); }
    int* err() { return sync + (size_t)n + 128; }
};

namespace {

template <class F>
int by_type(int type, F&& f) {
    if (type == 0) return f(double());
    if (type == 1) return f(float());
    return MPG_ERR_UNSUPPORTED;
}

// (the factorisation keeps 8 workgroups per CU: 64 / 256 of them took
// 0.75 / 0.22 s on LAP-1M against 0.071 s; one row per wave spins little)
int persist_grid(int n) { return std::max(1, std::min(kPersistGroups, (n + kWaves - 1) / kWaves)); }

// Serial-mode plan of one triangular solve (k_ilu_trsv_serial), or false
// when the solve is not eligible: a level schedule with >= 16 rows per level
// on average (the level kernel is faster), a dependency farther than kRing
// rows, or a row with more than kStageEnt off-diagonal entries. Entry
// offsets count each row padded to a multiple of kPass (at least kPass).
bool serial_plan(int n, int nlev, const std::vector<int>& rp, const std::vector<int>& ci, const std::vector<int>& dg,
                 bool upper, std::vector<int>& stage, std::vector<int>& eoff, int& P) {
    if (n == 0 || (int64_t)n >= 16 * (int64_t)nlev) return false;
    int longest = 1;
    for (int i = 0; i < n; ++i)
        longest = std::max(longest, upper ? rp[(size_t)i + 1] - dg[i] - 1 : dg[i] - rp[i]);
    P = std::min(kPass, longest);
    eoff.assign((size_t)n + 1, 0);
    for (int p = 0; p < n; ++p) {
        const int i = upper ? n - 1 - p : p;
        const int j0 = upper ? dg[i] + 1 : rp[i], j1 = upper ? rp[i + 1] : dg[i];
        const int padded = std::max(P, (j1 - j0 + P - 1) / P * P);
        if (padded > kStageEnt) return false;
        for (int j = j0; j < j1; ++j)
            if (std::abs(ci[j] - i) >= kRing) return false;
        eoff[(size_t)p + 1] = eoff[p] + padded;
    }
    stage.clear();
    for (int p = 0; p < n;) {
        stage.push_back(p);
        int q = p;
        while (q < n && q - p < kStageRows && eoff[(size_t)q + 1] - eoff[p] <= kStageEnt) ++q;
        p = q;
    }
    stage.push_back(n);
    return true;
}

// Level schedule of one triangular solve from host copies of the structure
// (upper: the rows after the diagonal, solved last row first).
void level_schedule(int n, const std::vector<int>& rp, const std::vector<int>& ci, const std::vector<int>& dg,
                    bool upper, std::vector<int>& ord, std::vector<int>& chunk, int& nlev) {
    std::vector<int> lev((size_t)n, 0);
    nlev = 0;
    for (int t = 0; t < n; ++t) {
        const int i = upper ? n - 1 - t : t;
        const int j0 = upper ? dg[i] + 1 : rp[i], j1 = upper ? rp[i + 1] : dg[i];
        int l = 0;
        for (int j = j0; j < j1; ++j) l = std::max(l, lev[ci[j]] + 1);
        lev[i] = l;
        nlev = std::max(nlev, l + 1);
    }
    std::vector<int> start((size_t)nlev + 1, 0);
    for (int i = 0; i < n; ++i) ++start[(size_t)lev[i] + 1];
    for (int l = 0; l < nlev; ++l) start[(size_t)l + 1] += start[l];
    ord.assign((size_t)n, 0);
    std::vector<int> fill(start.begin(), start.end() - 1);
    for (int t = 0; t < n; ++t) {
        const int i = upper ? n - 1 - t : t;
        ord[(size_t)fill[lev[i]]++] = i;
    }
    chunk.clear();
    for (int l = 0; l < nlev; ++l)
        for (int c = start[l]; c < start[(size_t)l + 1]; c += kWave) chunk.push_back(c);
    chunk.push_back(n);
}

}  // namespace

extern "C" {

int mpg_ilu_row_cap(void) { return kRowCap; }

int mpg_ilu0_create(mpg_ctx_t ctx, mpg_csr_t A, const double* val64, int type, mpg_ilu_t* out) {
    if (!ctx || !A || !out || (type != 0 && type != 1) || A->rows != A->cols || (A->nnz > 0 && !val64))
        return MPG_ERR_ARG;
    *out = nullptr;
    mpg_ilu* L = new (std::nothrow) mpg_ilu();
    if (!L) return MPG_ERR_ALLOC;
    L->ctx = ctx;
    L->A = A;
    L->n = A->rows;
    L->nnz = A->nnz;
    L->type = type;
    const int n = L->n;
    hipStream_t s = ctx->stream;
    auto fail = [&](int st) {
        mpg_ilu_destroy(L);
        return st;
    };
    auto ok = [](hipError_t e) { return e == hipSuccess; };
    const size_t nb = std::max<size_t>(1, (size_t)n), zb = std::max<size_t>(1, (size_t)L->nnz);
    if (!ok(hipMalloc((void**)&L->lu64, zb * 8)) || !ok(hipMalloc((void**)&L->diag, nb * 4)) ||
        !ok(hipMalloc(&L->dinv, nb * L->tsize())) || !ok(hipMalloc((void**)&L->sync, sync_ints(n) * 4)) ||
        !ok(hipMalloc(&L->w[0], nb * L->tsize())) || !ok(hipMalloc(&L->w[1], nb * L->tsize())) ||
        !ok(hipMalloc(&L->tagbuf, nb * L->tsize())) ||
        !ok(hipMalloc((void**)&L->scratch, 64)) || (type == 1 && !ok(hipMalloc((void**)&L->lu32, zb * 4))))
        return fail(MPG_ERR_ALLOC);
    if (!ok(hipMemsetAsync(L->sync, 0, sync_ints(n) * 4, s)) || !ok(hipMemsetAsync(L->scratch, 0, 64, s)))
        return fail(MPG_ERR_HIP);
    if (n == 0) {
        *out = L;
        return MPG_OK;
    }
    if (L->nnz && !ok(hipMemcpyAsync(L->lu64, val64, (size_t)L->nnz * 8, hipMemcpyDeviceToDevice, s)))
        return fail(MPG_ERR_HIP);
    int* bad = reinterpret_cast<int*>(L->scratch) + 4;
    const int g = (n + kBlock - 1) / kBlock;
    k_find_diag<<<g, kBlock, 0, s>>>(n, A->rowptr, A->col, L->diag, bad);
    k_abs_rowsum_max<<<g, kBlock, 0, s>>>(n, A->rowptr, L->lu64, L->scratch);
    int bad_h = 0;
    if (!ok(hipMemcpyAsync(&bad_h, bad, 4, hipMemcpyDeviceToHost, s)) || !ok(hipStreamSynchronize(s)))
        return fail(MPG_ERR_HIP);
    if (bad_h) return fail(MPG_ERR_UNSUPPORTED);  // a row without its diagonal, or longer than kRowCap
    {  // level schedules of the two triangular solves (host, O(nnz), once)
        std::vector<int> rp((size_t)n + 1), ci((size_t)std::max<int64_t>(L->nnz, 1)), dg((size_t)n);
        if (!ok(hipMemcpyAsync(rp.data(), A->rowptr, rp.size() * 4, hipMemcpyDeviceToHost, s)) ||
            (L->nnz && !ok(hipMemcpyAsync(ci.data(), A->col, (size_t)L->nnz * 4, hipMemcpyDeviceToHost, s))) ||
            !ok(hipMemcpyAsync(dg.data(), L->diag, dg.size() * 4, hipMemcpyDeviceToHost, s)) ||
            !ok(hipStreamSynchronize(s)))
            return fail(MPG_ERR_HIP);
        for (int u = 0; u < 2; ++u) {
            std::vector<int> ord, chunk;
            level_schedule(n, rp, ci, dg, u == 1, ord, chunk, L->levels[u]);
            L->nchunks[u] = (int)chunk.size() - 1;
            std::vector<int> stage, eoff;
            const char* senv = std::getenv("MPG_ILU_SERIAL");  // 0: always the level schedule
            if (!(senv && *senv == '0') && serial_plan(n, L->levels[u], rp, ci, dg, u == 1, stage, eoff, L->spass[u])) {
                L->serial[u] = true;
                L->nstages[u] = (int)stage.size() - 1;
                if (!ok(hipMalloc((void**)&L->stage[u], stage.size() * 4)) ||
                    !ok(hipMalloc((void**)&L->eoff[u], eoff.size() * 4)) ||
                    !ok(hipMemcpyAsync(L->stage[u], stage.data(), stage.size() * 4, hipMemcpyHostToDevice, s)) ||
                    !ok(hipMemcpyAsync(L->eoff[u], eoff.data(), eoff.size() * 4, hipMemcpyHostToDevice, s)) ||
                    !ok(hipStreamSynchronize(s)))
                    return fail(MPG_ERR_ALLOC);
            }
            if (!ok(hipMalloc((void**)&L->ord[u], ord.size() * 4)) ||
                !ok(hipMalloc((void**)&L->chunk[u], chunk.size() * 4)) ||
                !ok(hipMemcpyAsync(L->ord[u], ord.data(), ord.size() * 4, hipMemcpyHostToDevice, s)) ||
                !ok(hipMemcpyAsync(L->chunk[u], chunk.data(), chunk.size() * 4, hipMemcpyHostToDevice, s)) ||
                !ok(hipStreamSynchronize(s)))
                return fail(MPG_ERR_ALLOC);
        }
    }
    const double eps = type == 0 ? (double)std::numeric_limits<double>::epsilon()
                                 : (double)std::numeric_limits<float>::epsilon();
    k_ilu0_factor<<<persist_grid(n), kBlock, 0, s>>>(n, A->rowptr, A->col, L->diag, L->lu64, eps, L->scratch,
                                                     L->sync, L->ticket(0), L->err(), L->ord[0]);
    int st = by_type(type, [&](auto t) {
        using T = decltype(t);
        T* lu = static_cast<T*>(L->values());
        if (std::is_same<T, float>::value)
            k_round_factors<T><<<grid_for(L->nnz, 4), kBlock, 0, s>>>(L->nnz, L->lu64, lu);
        k_dinv<T><<<g, kBlock, 0, s>>>(n, L->diag, lu, static_cast<T*>(L->dinv));
        return (int)MPG_OK;
    });
    if (st) return fail(st);
    if (!ok(hipGetLastError())) return fail(MPG_ERR_HIP);
    if (int f = mpg_ilu_fault(L)) {
        if (std::getenv("MPG_ILU_DEBUG")) {
            int32_t st4[4];
            mpg_ilu_debug_state(L, st4);
            std::fprintf(stderr, "mpg_ilu0_create: fault %d, tickets %d %d %d, n %d\n", f, st4[0], st4[1], st4[2], n);
        }
        return fail(MPG_ERR_BREAKDOWN);
    }
    if (const char* e = std::getenv("MPG_ILU_WAIT_TICKS"))  // test hook: bound of the solves' waits
        L->wait_bound = std::strtoull(e, nullptr, 10) ? std::strtoull(e, nullptr, 10) : kWaitBound;
    *out = L;
    return MPG_OK;
}

int mpg_ilu_destroy(mpg_ilu_t L) {
    if (!L) return MPG_OK;
    if (L->ctx) (void)hipStreamSynchronize(L->ctx->stream);
    void* ps[] = {L->lu64,    L->lu32,    L->diag,     L->dinv,     L->sync,     L->w[0],    L->w[1],
                  L->scratch, L->ord[0],  L->ord[1],   L->chunk[0], L->chunk[1], L->stage[0], L->stage[1],
                  L->eoff[0], L->eoff[1], L->tagbuf};
    for (void* p : ps)
        if (p) (void)hipFree(p);
    delete L;
    return MPG_OK;
}

int mpg_ilu_solve(mpg_ctx_t ctx, mpg_ilu_t L, void* x) {
    if (!ctx || !L || (!x && L->n)) return MPG_ERR_ARG;
    if (L->n == 0) return MPG_OK;
    const int n = L->n;
    // one wave per chunk in flight at most: a wave per 64 rows, <= 8 workgroups per CU
    static const int cap = [] {
        const char* e = std::getenv("MPG_ILU_GROUPS");  // experiment: cap on the solve grid
        return e && std::atoi(e) > 0 ? std::atoi(e) : kSolveGroups;
    }();
    auto grid = [&](int u) { return std::max(1, std::min(cap, (L->nchunks[u] + kWaves - 1) / kWaves)); };
    // tagged level solves: L x -> y (x left tagged), U y -> x; a serial
    // direction solves in place in x, moved to / from y next to a tagged one
    const int g = (n + kBlock - 1) / kBlock;
    hipStream_t s = ctx->stream;
    int st = by_type(L->type, [&](auto t) {
        using T = decltype(t);
        const T* lu = static_cast<const T*>(L->values());
        T* xv = static_cast<T*>(x);
        T* yv = static_cast<T*>(L->tagbuf);
        auto serial = [&](int u, auto upper) {  // in place in x, P entries per pass
            constexpr bool UP = decltype(upper)::value;
            auto go = [&](auto pc) {
                k_ilu_trsv_serial<T, UP, decltype(pc)::value><<<1, kBlock, 0, s>>>(
                    n, L->nstages[u], L->stage[u], L->eoff[u], L->A->rowptr, L->A->col, L->diag, lu, xv);
            };
            switch (L->spass[u]) {
                case 1: go(std::integral_constant<int, 1>()); break;
                case 2: go(std::integral_constant<int, 2>()); break;
                case 3: go(std::integral_constant<int, 3>()); break;
                case 4: go(std::integral_constant<int, 4>()); break;
                case 5: go(std::integral_constant<int, 5>()); break;
                case 6: go(std::integral_constant<int, 6>()); break;
                case 7: go(std::integral_constant<int, 7>()); break;
                default: go(std::integral_constant<int, kPass>()); break;
            }
        };
        if (!L->serial[0] || !L->serial[1]) k_trsv_tag_fill<T><<<g, kBlock, 0, s>>>(n, yv, L->ticket(1));
        if (L->serial[0]) {
            serial(0, std::false_type());
            if (!L->serial[1]) k_trsv_tag_move<T><<<g, kBlock, 0, s>>>(n, xv, yv);
        } else {
            k_ilu_trsv_tagged<T, false><<<grid(0), kBlock, 0, s>>>(L->nchunks[0], L->chunk[0], L->ord[0],
                                                                   L->A->rowptr, L->A->col, L->diag, lu, xv,
                                                                   yv, L->ticket(1), L->err(), L->wait_bound);
        }
        if (L->serial[1]) {
            if (!L->serial[0]) k_trsv_tag_move<T><<<g, kBlock, 0, s>>>(n, yv, xv);
            serial(1, std::true_type());
        } else {
            k_ilu_trsv_tagged<T, true><<<grid(1), kBlock, 0, s>>>(L->nchunks[1], L->chunk[1], L->ord[1],
                                                                  L->A->rowptr, L->A->col, L->diag, lu, yv,
                                                                  xv, L->ticket(2), L->err(), L->wait_bound);
        }
        return (int)MPG_OK;
    });
    if (st) return st;
    MPG_LAUNCH_CHECK(ctx);
    return MPG_OK;
}

int mpg_ilu_jacobi_solve(mpg_ctx_t ctx, mpg_ilu_t L, int steps, void* x) {
    if (!ctx || !L || steps < 0 || (!x && L->n)) return MPG_ERR_ARG;
    const int n = L->n;
    if (n == 0) return MPG_OK;
    const int g = (n + kBlock - 1) / kBlock;
    const size_t bytes = (size_t)n * L->tsize();
    hipStream_t s = ctx->stream;
    int st = by_type(L->type, [&](auto t) {
        using T = decltype(t);
        const T* lu = static_cast<const T*>(L->values());
        const T* dinv = static_cast<const T*>(L->dinv);
        T* b = static_cast<T*>(L->w[0]);
        T* cur = static_cast<T*>(x);
        T* nxt = static_cast<T*>(L->w[1]);
        if (hipMemcpyAsync(b, cur, bytes, hipMemcpyDeviceToDevice, s) != hipSuccess) return (int)MPG_ERR_HIP;
        for (int i = 0; i < steps; ++i) {
            k_ilu_jacobi_sweep<T, false><<<g, kBlock, 0, s>>>(n, L->A->rowptr, L->A->col, L->diag, lu, dinv, b, cur,
                                                               nxt);
            std::swap(cur, nxt);
        }
        if (hipMemcpyAsync(b, cur, bytes, hipMemcpyDeviceToDevice, s) != hipSuccess) return (int)MPG_ERR_HIP;
        for (int i = 0; i < steps; ++i) {
            k_ilu_jacobi_sweep<T, true><<<g, kBlock, 0, s>>>(n, L->A->rowptr, L->A->col, L->diag, lu, dinv, b, cur,
                                                              nxt);
            std::swap(cur, nxt);
        }
        if (cur != static_cast<T*>(x) && hipMemcpyAsync(x, cur, bytes, hipMemcpyDeviceToDevice, s) != hipSuccess)
            return (int)MPG_ERR_HIP;
        return (int)MPG_OK;
    });
    if (st) return st;
    MPG_LAUNCH_CHECK(ctx);
    return MPG_OK;
}

const void* mpg_ilu_values_dev(mpg_ilu_t L) { return L ? L->values() : nullptr; }
const int32_t* mpg_ilu_diag_dev(mpg_ilu_t L) { return L ? L->diag : nullptr; }
const void* mpg_ilu_dinv_dev(mpg_ilu_t L) { return L ? L->dinv : nullptr; }

int mpg_ilu_debug_state(mpg_ilu_t L, int32_t* out4) {
    if (!L || !out4 || !L->sync) return MPG_ERR_ARG;
    int v[4] = {0, 0, 0, 0};
    for (int k = 0; k < 3; ++k)
        if (hipMemcpyAsync(v + k, L->ticket(k), 4, hipMemcpyDeviceToHost, L->ctx->stream) != hipSuccess) return MPG_ERR_HIP;
    if (hipMemcpyAsync(v + 3, L->err(), 4, hipMemcpyDeviceToHost, L->ctx->stream) != hipSuccess ||
        hipStreamSynchronize(L->ctx->stream) != hipSuccess)
        return MPG_ERR_HIP;
    for (int k = 0; k < 4; ++k) out4[k] = v[k];
    return MPG_OK;
}

int mpg_ilu_fault(mpg_ilu_t L) {
    if (!L || !L->sync) return 0;
    int e = 0;
    if (hipMemcpyAsync(&e, L->err(), 4, hipMemcpyDeviceToHost, L->ctx->stream) != hipSuccess ||
        hipStreamSynchronize(L->ctx->stream) != hipSuccess)
        return -1;
    return e;
}

int mpg_ilu_clear_fault(mpg_ilu_t L) {
    if (!L || !L->sync) return MPG_ERR_ARG;
    MPG_HIP(L->ctx, hipMemsetAsync(L->err(), 0, sizeof(int), L->ctx->stream));
    return MPG_OK;
}

int mpg_ilu_set_wait_bound(mpg_ilu_t L, uint64_t ticks) {
    if (!L) return MPG_ERR_ARG;
    L->wait_bound = ticks ? ticks : kWaitBound;
    return MPG_OK;
}

int mpg_ilu_solve_mode(mpg_ilu_t L) { return L ? (L->serial[0] ? 1 : 0) | (L->serial[1] ? 2 : 0) : 0; }

}  // extern "C"
