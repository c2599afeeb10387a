// Build of the node-block copy of the Arnoldi matrix (node_tile.hpp).
#include "node_tile.hpp"
#include "ride.hpp"
#include "scalar_program.hpp"

#include <algorithm>
#include <cstdlib>
#include <new>
#include <vector>

using namespace mpg;

namespace {

// blocks of node row r (rows 3r .. 3r + 2), or -1 when its rows are not made
// of the same aligned column triples in the same storage positions. One wave
// per node row, a lane per triple (coalesced column reads).
// far[r]: the node row's blocks whose column lies more than kNodeFar rows
// from the row (scattered gathers: node_build's XCD-order choice).
constexpr int kNodeFar = 1 << 18;
__global__ __launch_bounds__(kBlock) void k_node_check(int nn, const int32_t* __restrict__ rowptr,
                                                       const int32_t* __restrict__ col, int32_t* __restrict__ cnt,
                                                       int32_t* __restrict__ far) {
    const int r = (int)(((int64_t)blockIdx.x * kBlock + threadIdx.x) / kWave);
    const int lane = threadIdx.x & (kWave - 1);
    if (r >= nn) return;  // (wave-uniform)
    const int p0 = rowptr[3 * r], p1 = rowptr[3 * r + 1], p2 = rowptr[3 * r + 2], p3 = rowptr[3 * r + 3];
    const int len = p1 - p0;
    int ok = p2 - p1 == len && p3 - p2 == len && len % 3 == 0;
    int nfar = 0;
    if (ok)
        for (int t = 3 * lane; t < len; t += 3 * kWave) {
            const int c = col[p0 + t];
            for (int j = 0; j < 3; ++j)
                ok &= col[p0 + t + j] == c + j && col[p1 + t + j] == c + j && col[p2 + t + j] == c + j;
            nfar += abs(c - 3 * r) > kNodeFar;
        }
    ok = __all(ok);
    nfar = wave_sum(nfar);
    if (lane == 0) {
        cnt[r] = ok ? len / 3 : -1;
        far[r] = nfar;
    }
}

template <class VI>
__device__ __forceinline__ uint32_t val_bits(const VI* v, int64_t i);
template <> __device__ __forceinline__ uint32_t val_bits<float>(const float* v, int64_t i) {
    return __float_as_uint(v[i]);
}
template <> __device__ __forceinline__ uint32_t val_bits<half_v>(const half_v* v, int64_t i) { return v[i].bits; }

// records of node row r: word 0 the block's first column, then the 9 values
// row-major (fp64: from word 2; fp16: two per word). One wave per node row,
// a lane per block: consecutive lanes write consecutive records.
template <class VI>
__global__ __launch_bounds__(kBlock) void k_node_fill(int nn, const int32_t* __restrict__ rowptr,
                                                      const int32_t* __restrict__ col, const VI* __restrict__ val,
                                                      const int32_t* __restrict__ bptr, uint32_t* __restrict__ recs) {
    constexpr int RW = NodeRec<VI>::R / 4;
    const int r = (int)(((int64_t)blockIdx.x * kBlock + threadIdx.x) / kWave);
    const int lane = threadIdx.x & (kWave - 1);
    if (r >= nn) return;
    const int p[3] = {rowptr[3 * r], rowptr[3 * r + 1], rowptr[3 * r + 2]};
    for (int b = bptr[r] + lane; b < bptr[r + 1]; b += kWave) {
        const int t = 3 * (b - bptr[r]);
        uint32_t w[RW];
#pragma unroll
        for (int q = 0; q < RW; ++q) w[q] = 0;
        w[0] = (uint32_t)col[p[0] + t];
#pragma unroll
        for (int k = 0; k < 3; ++k)
#pragma unroll
            for (int j = 0; j < 3; ++j) {
                const int e = 3 * k + j;
                const int64_t i = (int64_t)p[k] + t + j;
                if constexpr (std::is_same_v<VI, double>) {
                    const double v = val[i];
                    w[2 + 2 * e] = (uint32_t)__double2loint(v);
                    w[3 + 2 * e] = (uint32_t)__double2hiint(v);
                } else if constexpr (std::is_same_v<VI, float>) {
                    w[1 + e] = val_bits(val, i);
                } else {
                    w[1 + e / 2] |= val_bits(val, i) << (e & 1 ? 16 : 0);
                }
            }
        uint32_t* o = recs + (int64_t)b * RW;
#pragma unroll
        for (int q = 0; q < RW; ++q) o[q] = w[q];
    }
}

// Padded node blocks, for node rows whose three rows do not share one
// pattern (a constrained dof's identity row, a dropped entry): the blocks of
// node row r are the sorted union of the node columns q = c / 3 of its rows
// (each row strictly increasing, columns in [0, cols)), a block's missing
// entries stored as zeros. A row's sum then meets its CSR entries in CSR
// (ascending) order with +-0 products in between, which leave an fp64 sum
// that starts at +0 unchanged: the bits of the CSR sum for finite x.
// One thread per node row (a three-way merge); cnt[r] = blocks or -1.
__global__ __launch_bounds__(kBlock) void k_node_count_padded(int nn, int cols, const int32_t* __restrict__ rowptr,
                                                              const int32_t* __restrict__ col,
                                                              int32_t* __restrict__ cnt, int32_t* __restrict__ far) {
    const int r = blockIdx.x * kBlock + threadIdx.x;
    if (r >= nn) return;
    int p[3], e[3];
    bool ok = true;
    for (int k = 0; k < 3; ++k) {
        p[k] = rowptr[3 * r + k];
        e[k] = rowptr[3 * r + k + 1];
        for (int i = p[k]; i < e[k] && ok; ++i)
            ok = col[i] >= 0 && col[i] < cols && (i == p[k] || col[i] > col[i - 1]);
    }
    int count = 0, nfar = 0;
    while (ok) {
        int q = INT32_MAX;
        for (int k = 0; k < 3; ++k)
            if (p[k] < e[k]) q = min(q, col[p[k]] / 3);
        if (q == INT32_MAX) break;
        ++count;
        nfar += abs(3 * q - 3 * r) > kNodeFar;
        for (int k = 0; k < 3; ++k)
            while (p[k] < e[k] && col[p[k]] / 3 == q) ++p[k];
    }
    cnt[r] = ok ? count : -1;
    far[r] = nfar;
}

template <class VI>
__global__ __launch_bounds__(kBlock) void k_node_fill_padded(int nn, const int32_t* __restrict__ rowptr,
                                                             const int32_t* __restrict__ col,
                                                             const VI* __restrict__ val,
                                                             const int32_t* __restrict__ bptr,
                                                             uint32_t* __restrict__ recs) {
    constexpr int RW = NodeRec<VI>::R / 4;
    const int r = blockIdx.x * kBlock + threadIdx.x;
    if (r >= nn) return;
    int p[3], e[3];
    for (int k = 0; k < 3; ++k) {
        p[k] = rowptr[3 * r + k];
        e[k] = rowptr[3 * r + k + 1];
    }
    for (int b = bptr[r]; b < bptr[r + 1]; ++b) {
        int q = INT32_MAX;
        for (int k = 0; k < 3; ++k)
            if (p[k] < e[k]) q = min(q, col[p[k]] / 3);
        uint32_t w[RW];
#pragma unroll
        for (int i = 0; i < RW; ++i) w[i] = 0;
        w[0] = (uint32_t)(3 * q);
        for (int k = 0; k < 3; ++k)
            for (; p[k] < e[k] && col[p[k]] / 3 == q; ++p[k]) {
                const int el = 3 * k + col[p[k]] - 3 * q;
                if constexpr (std::is_same_v<VI, double>) {
                    const double v = val[p[k]];
                    w[2 + 2 * el] = (uint32_t)__double2loint(v);
                    w[3 + 2 * el] = (uint32_t)__double2hiint(v);
                } else if constexpr (std::is_same_v<VI, float>) {
                    w[1 + el] = val_bits(val, p[k]);
                } else {
                    w[1 + el / 2] |= val_bits(val, p[k]) << (el & 1 ? 16 : 0);
                }
            }
        uint32_t* o = recs + (int64_t)b * RW;
        for (int i = 0; i < RW; ++i) o[i] = w[i];
    }
}

// y = alpha * A x + beta * y over the node copy: the CSR tile's epilogue
// (spmv.hip k_csr_adaptive) on node_tiles' row sums.
// Rides (round 6; the SELL copy's since round 5, sell.hip):
// prog.count > 0: workgroup 0 runs that scalar program (the surface's Givens
// step of the previous Arnoldi step, which this SpMV neither reads nor
// writes: kernels_hip.cpp checks the operands) and the tiles take the other
// workgroups. NORM: x is w; every workgroup forms a = T(1) / h from the
// ||w||^2 partials (norm_scale, ride.hpp), multiplies T(a x_c) -- scal_recip's
// product, the vector the separate launches would store and read -- and
// stores v_i = T(a x_i) for its own rows: the bits of mpg_scal_recip_nrm2_*
// followed by the plain node SpMV.
template <class VI, class X, bool NORM = false>
__global__ __launch_bounds__(kBlock) void k_node_spmv(const int32_t* __restrict__ tiles,
                                                      const int32_t* __restrict__ bptr, const char* __restrict__ recs,
                                                      int ntiles, int64_t nblk, int tpw, int xcd,
                                                      const X* __restrict__ x, X alpha, X beta, X* __restrict__ y,
                                                      ScalarProgram prog, NormArgs<X> nm) {
    __shared__ double prod[kNodeProd];
    double pv = 0.0;  // NORM: this lane's ||w||^2 partial, issued first
    if constexpr (NORM) pv = (int)threadIdx.x < nm.nparts ? nm.part[threadIdx.x] : 0.0;
    int b = (int)blockIdx.x, G = (int)gridDim.x;
    if (prog.count > 0) {
        if (b == 0) {
            __shared__ double plds[3 * kProgStage + 1];
            if constexpr (NORM) (void)norm_scale(nm, pv);  // h(k+1,k) stored before the program reads it
            if (threadIdx.x < kWave) run_scalar_program<kProgStage>(prog, plds);
            return;
        }
        --b;
        --G;
    }
    X a = X(1);
    __shared__ double nscratch[NORM ? kBlock / kWave : 1];
    __shared__ X a_s;
    const int g = xcd ? xcd_block(b, G) : b;
    const int t0 = g * tpw, t1 = t0 + tpw < ntiles ? t0 + tpw : ntiles;
    auto sc = [&](X v) { return NORM ? (X)(a * v) : v; };
    node_tiles<VI>(
        t0, t1, tiles, tiles + ntiles + 1, bptr, recs, nblk, [&](int c) { return x[c]; },
        [&](X v) { return (double)sc(v); },
        [&](int i) { return beta == X(0) ? X(0) : y[i]; },
        [&](int i, double sum, X yi) {
            const X t = (X)sum;
            y[i] = spmv_axpby(alpha, t, beta, yi);
            if constexpr (NORM) nm.v[i] = sc(x[i]);
        },
        prod, [&] {
            // the scale, formed while the first tile's gathers are in flight
            if constexpr (NORM) a = norm_scale_lds(nm, pv, nscratch, &a_s);
        });
}

}  // namespace

struct mpg_node {
    mpg_ctx* ctx = nullptr;
    int cols = 0;
    mpg::NodeCopy S;
};

namespace mpg {

int node_xcd(const NodeCopy& S) {
    const char* e = std::getenv("MPG_NODE_XCD");  // 0 / 1 force the order (A/B)
    return e && (*e == '0' || *e == '1') ? *e - '0' : S.xcd ? 1 : 0;
}

int node_tpw_default() {
    const char* e = std::getenv("MPG_NODE_TPW");
    return e && *e ? std::atoi(e) : 2;
}

int node_build(mpg_ctx* ctx, const mpg_csr* A, int vtype, const void* val, bool required, NodeCopy& S,
               int64_t alt_bytes) {
    S = NodeCopy{};
    const int fail = required ? MPG_ERR_UNSUPPORTED : MPG_OK;
    const int n = A->rows;
    if (n == 0 || n % kNodeDof || A->nnz == 0 || !val) return fail;
    if (vtype != MPG_F64 && vtype != MPG_F32 && vtype != MPG_F16) return MPG_ERR_ARG;
    hipStream_t stream = ctx->stream;
    const int nn = n / kNodeDof;
    const int grid = (int)(((int64_t)nn * kWave + kBlock - 1) / kBlock);  // one wave per node row
    int32_t* cnt = nullptr;
    MPG_HIP(ctx, hipMalloc((void**)&cnt, (size_t)nn * 8));
    std::vector<int32_t> ch((size_t)nn * 2);
    k_node_check<<<grid, kBlock, 0, stream>>>(nn, A->rowptr, A->col, cnt, cnt + nn);
    hipError_t e = hipMemcpyAsync(ch.data(), cnt, (size_t)nn * 8, hipMemcpyDeviceToHost, stream);
    if (e == hipSuccess) e = hipStreamSynchronize(stream);
    (void)hipFree(cnt);
    if (e != hipSuccess) return set_hip_error(ctx, e, "node_build check");
    // exact node blocks, or else padded ones (columns in [0, cols), cols a
    // multiple of 3, rows sorted; MPG_NODE_PAD=0: exact only)
    bool padded = false;
    if (std::any_of(ch.begin(), ch.begin() + nn, [](int32_t v) { return v < 0; })) {
        const char* pe = std::getenv("MPG_NODE_PAD");
        if ((pe && *pe == '0') || A->cols % kNodeDof) return fail;
        MPG_HIP(ctx, hipMalloc((void**)&cnt, (size_t)nn * 8));
        k_node_count_padded<<<(nn + kBlock - 1) / kBlock, kBlock, 0, stream>>>(nn, A->cols, A->rowptr, A->col, cnt,
                                                                               cnt + nn);
        e = hipMemcpyAsync(ch.data(), cnt, (size_t)nn * 8, hipMemcpyDeviceToHost, stream);
        if (e == hipSuccess) e = hipStreamSynchronize(stream);
        (void)hipFree(cnt);
        if (e != hipSuccess) return set_hip_error(ctx, e, "node_build padded count");
        padded = true;
    }
    int64_t nfar = 0;
    for (int r = 0; r < nn; ++r) nfar += ch[(size_t)nn + r];
    std::vector<int32_t> bptr((size_t)nn + 1, 0);
    int64_t nb = 0;
    for (int r = 0; r < nn; ++r) {
        if (ch[r] < 0 || ch[r] > kNodeCap) return fail;
        bptr[r] = (int32_t)nb;
        nb += ch[r];
        if (nb >= INT32_MAX / 2) return fail;
    }
    bptr[nn] = (int32_t)nb;
    // tiles: runs of node rows with at most kNodeCap blocks (and node rows)
    std::vector<int32_t> tiles{0};
    for (int r = 0; r < nn;) {
        int z = r;
        while (z < nn && bptr[z + 1] - bptr[r] <= kNodeCap && z - r < kNodeCap) ++z;
        tiles.push_back(z);
        r = z;
    }
    const size_t nt1 = tiles.size();
    tiles.resize(2 * nt1);
    for (size_t t = 0; t < nt1; ++t) tiles[nt1 + t] = bptr[tiles[t]];
    // the copy's bytes before it is built: none when it would lose to alt_bytes
    const int64_t est = nb * node_rec_bytes(vtype) + ((int64_t)nn + 1) * 4 + 2 * (int64_t)nt1 * 4;
    if (alt_bytes >= 0 && !node_wins(est, alt_bytes, (int64_t)A->cols * (vtype == MPG_F64 ? 8 : 4))) return fail;
    S.nn = nn;
    S.nblk = nb;
    // scattered columns (over a quarter of the blocks far from their rows,
    // e.g. a node-block permutation): tiles in XCD order, so the tiles of a
    // node block share one L2 for the neighbour blocks they all gather
    // (fem27p 282 -> 253 us, stencil27p 392 -> 355; natural order loses 3 %:
    // fem27 219 -> 226, C4 313 -> 320; profiles/r05_node_ab.jsonl)
    S.xcd = 4 * nfar > nb;
    S.ntiles = (int)nt1 - 1;
    S.vtype = vtype;
    S.rec = node_rec_bytes(vtype);
    bool ok = hipMalloc((void**)&S.bptr, bptr.size() * 4) == hipSuccess &&
              hipMalloc((void**)&S.tiles, tiles.size() * 4) == hipSuccess &&
              hipMalloc(&S.recs, (size_t)std::max<int64_t>(nb, 1) * S.rec) == hipSuccess &&
              hipMemcpyAsync(S.bptr, bptr.data(), bptr.size() * 4, hipMemcpyHostToDevice, stream) == hipSuccess &&
              hipMemcpyAsync(S.tiles, tiles.data(), tiles.size() * 4, hipMemcpyHostToDevice, stream) == hipSuccess;
    S.padded = padded ? nb * kNodeDof * kNodeDof - A->nnz : 0;
    if (ok && padded) {
        auto* o = static_cast<uint32_t*>(S.recs);
        const int g = (nn + kBlock - 1) / kBlock;
        if (vtype == MPG_F64)
            k_node_fill_padded<double><<<g, kBlock, 0, stream>>>(nn, A->rowptr, A->col,
                                                                 static_cast<const double*>(val), S.bptr, o);
        else if (vtype == MPG_F32)
            k_node_fill_padded<float><<<g, kBlock, 0, stream>>>(nn, A->rowptr, A->col,
                                                                static_cast<const float*>(val), S.bptr, o);
        else
            k_node_fill_padded<half_v><<<g, kBlock, 0, stream>>>(nn, A->rowptr, A->col,
                                                                 static_cast<const half_v*>(val), S.bptr, o);
        ok = hipGetLastError() == hipSuccess && hipStreamSynchronize(stream) == hipSuccess;
    } else if (ok) {
        auto* o = static_cast<uint32_t*>(S.recs);
        if (vtype == MPG_F64)
            k_node_fill<double><<<grid, kBlock, 0, stream>>>(nn, A->rowptr, A->col, static_cast<const double*>(val),
                                                             S.bptr, o);
        else if (vtype == MPG_F32)
            k_node_fill<float><<<grid, kBlock, 0, stream>>>(nn, A->rowptr, A->col, static_cast<const float*>(val),
                                                            S.bptr, o);
        else
            k_node_fill<half_v><<<grid, kBlock, 0, stream>>>(nn, A->rowptr, A->col, static_cast<const half_v*>(val),
                                                             S.bptr, o);
        ok = hipGetLastError() == hipSuccess && hipStreamSynchronize(stream) == hipSuccess;
    }
    if (!ok) {
        node_free(S);
        return MPG_ERR_ALLOC;
    }
    return MPG_OK;
}

void node_free(NodeCopy& S) {
    for (void* p : {(void*)S.bptr, (void*)S.tiles, S.recs})
        if (p) (void)hipFree(p);
    S = NodeCopy{};
}

int64_t node_bytes(const NodeCopy& S) {
    return S.nblk * S.rec + ((int64_t)S.nn + 1) * 4 + 2 * ((int64_t)S.ntiles + 1) * 4;
}

}  // namespace mpg

template <class X, bool NORM = false>
static int node_spmv_impl(mpg_ctx_t ctx, mpg_node_t A, X alpha, const X* x, X beta, X* y,
                          const ScalarProgram& prog = ScalarProgram{}, const NormArgs<X>& nm = NormArgs<X>{}) {
    if (!ctx || !A) return MPG_ERR_ARG;
    if (A->S.vtype != (sizeof(X) == 8 ? MPG_F64 : MPG_F32)) return MPG_ERR_ARG;
    if (A->S.ntiles == 0) {
        if (NORM) return MPG_ERR_ARG;
        return prog.count > 0 ? mpg_scalar_program(ctx, prog.ops, prog.count) : MPG_OK;
    }
    int tpw = node_tpw_default();
    if (tpw < 1) tpw = 2;
    using VI = std::conditional_t<sizeof(X) == 8, double, float>;
    const int grid = (A->S.ntiles + tpw - 1) / tpw + (prog.count > 0 ? 1 : 0);
    k_node_spmv<VI, X, NORM><<<grid, kBlock, 0, ctx->stream>>>(
        A->S.tiles, A->S.bptr, static_cast<const char*>(A->S.recs), A->S.ntiles, A->S.nblk, tpw, node_xcd(A->S), x,
        alpha, beta, y, prog, nm);
    MPG_LAUNCH_CHECK(ctx);
    return MPG_OK;
}

template <class X>
static int node_spmv_norm(mpg_ctx_t c, mpg_node_t A, int32_t nparts, X* h, const X* w, X* v, X alpha, X* y,
                          const mpg_scalar_op* ops, int32_t nops) {
    ScalarProgram prog;
    if (!c || !A || !h || !w || !v || !y || nparts < 1 || nparts > kBlock || A->cols != kNodeDof * A->S.nn ||
        make_scalar_program(ops, nops, prog) != MPG_OK)
        return MPG_ERR_ARG;
    NormArgs<X> nm;
    nm.part = c->red_ws;
    nm.nparts = nparts;
    nm.h = h;
    nm.v = v;
    return node_spmv_impl<X, true>(c, A, alpha, w, X(0), y, prog, nm);
}


extern "C" {

int mpg_node_create(mpg_ctx_t ctx, mpg_csr_t A, int32_t vtype, const void* vals, int64_t alt_bytes,
                    mpg_node_t* out) {
    if (!ctx || !A || !out || (A->nnz > 0 && !vals)) return MPG_ERR_ARG;
    if (vtype != MPG_F64 && vtype != MPG_F32) return MPG_ERR_UNSUPPORTED;
    *out = nullptr;
    mpg_node* h = new (std::nothrow) mpg_node();
    if (!h) return MPG_ERR_ALLOC;
    h->ctx = ctx;
    h->cols = A->cols;
    if (int st = node_build(ctx, A, vtype, vals, false, h->S, alt_bytes)) {
        delete h;
        return st;
    }
    if (h->S.nblk == 0) {
        node_free(h->S);
        delete h;
        return MPG_OK;
    }
    *out = h;
    return MPG_OK;
}

int mpg_node_destroy(mpg_node_t A) {
    if (!A) return MPG_OK;
    if (A->ctx) (void)hipStreamSynchronize(A->ctx->stream);
    node_free(A->S);
    delete A;
    return MPG_OK;
}

int mpg_node_layout(mpg_node_t A, int64_t* blocks, int32_t* tiles, int64_t* bytes, int64_t* padded) {
    if (!A) return MPG_ERR_ARG;
    if (padded) *padded = A->S.padded;
    if (blocks) *blocks = A->S.nblk;
    if (tiles) *tiles = A->S.ntiles;
    if (bytes) *bytes = node_bytes(A->S);
    return MPG_OK;
}

int mpg_node_spmv_f64(mpg_ctx_t ctx, mpg_node_t A, double alpha, const double* x, double beta, double* y) {
    return node_spmv_impl(ctx, A, alpha, x, beta, y);
}
int mpg_node_spmv_f32(mpg_ctx_t ctx, mpg_node_t A, float alpha, const float* x, float beta, float* y) {
    return node_spmv_impl(ctx, A, alpha, x, beta, y);
}
int mpg_node_spmv_prog_f64(mpg_ctx_t ctx, mpg_node_t A, double alpha, const double* x, double beta, double* y,
                           const mpg_scalar_op* ops, int32_t nops) {
    ScalarProgram prog;
    if (make_scalar_program(ops, nops, prog) != MPG_OK) return MPG_ERR_ARG;
    return node_spmv_impl(ctx, A, alpha, x, beta, y, prog);
}
int mpg_node_spmv_prog_f32(mpg_ctx_t ctx, mpg_node_t A, float alpha, const float* x, float beta, float* y,
                           const mpg_scalar_op* ops, int32_t nops) {
    ScalarProgram prog;
    if (make_scalar_program(ops, nops, prog) != MPG_OK) return MPG_ERR_ARG;
    return node_spmv_impl(ctx, A, alpha, x, beta, y, prog);
}
int mpg_node_spmv_norm_f64(mpg_ctx_t c, mpg_node_t A, int32_t nparts, double* h, const double* w, double* v,
                           double alpha, double* y, const mpg_scalar_op* ops, int32_t nops) {
    return node_spmv_norm<double>(c, A, nparts, h, w, v, alpha, y, ops, nops);
}
int mpg_node_spmv_norm_f32(mpg_ctx_t c, mpg_node_t A, int32_t nparts, float* h, const float* w, float* v,
                           float alpha, float* y, const mpg_scalar_op* ops, int32_t nops) {
    return node_spmv_norm<float>(c, A, nparts, h, w, v, alpha, y, ops, nops);
}

}  // extern "C"
