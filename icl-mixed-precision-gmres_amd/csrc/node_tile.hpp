// Node-block copy of the Arnoldi matrix (round 5): the storage of a matrix
// whose unknowns come in nodes of 3 degrees of freedom (the FEM class of
// Queen_4147 and the fem27 / stencil27p stand-ins), where every coupling of
// two nodes is a full 3 x 3 block. CSR stores a column index per nonzero
// (8 B per fp32 nonzero); here one record per block holds the block's first
// column and its 9 values, row-major:
//
//   fp32: int32 col, 9 x fp32            40 B per 9 nonzeros (4.44 B each)
//   fp64: int32 col, pad, 9 x fp64       80 B
//   fp16: int32 col, 9 x fp16, pad       24 B
//
// bptr[r] .. bptr[r + 1] are the blocks of node row r (matrix rows 3r ..
// 3r + 2), in the CSR's own storage order: block t of node row r is CSR
// positions 3t .. 3t + 2 of each of the node's three rows, which must hold
// the columns c, c + 1, c + 2 (the same c in all three rows). A tile is a
// run of node rows with at most kNodeCap blocks: one record per lane, the 9
// fp64 products into LDS, then one lane per matrix row sums its products in
// storage order -- the CSR tile's products and summation order (csr_tile.hpp),
// so the Arnoldi SpMV gives the same bits on either copy.
#pragma once

#include "csr_tile.hpp"  // half_v
#include "internal.hpp"
#include "mpgmres/arnoldi.h"  // mpg_dtype_t

#include <type_traits>

namespace mpg {

constexpr int kNodeDof = 3;
constexpr int kNodeCap = kBlock;  // blocks per tile: one record per lane
constexpr int kNodeProd = kNodeCap * kNodeDof * kNodeDof;
// Row sums read this many blocks' products ahead (node_tiles). Measured
// in-cycle (profiles/r05_node_ab.jsonl, interleaved builds): fem27 220 ->
// 212 us, C4 315 -> 300, fem27p 253 -> 250 at 4 (54 VGPRs); 8 ahead was
// slower (241 / 335 / 264), and one lane summing a node's three rows 26 %
// slower: the sums' LDS latency is on the tile's critical path.
constexpr int kNodeSumAhead = 4;

struct NodeCopy {
    int nn = 0;            // node rows (rows / 3)
    int64_t nblk = 0;      // blocks
    int ntiles = 0;
    int vtype = 0;         // MPG_F64 / MPG_F32 / MPG_F16
    int rec = 0;           // record bytes
    bool xcd = false;      // scattered columns: tiles in XCD order (node_xcd)
    int64_t padded = 0;    // zero slots of padded node blocks (0: exact blocks)
    int32_t* bptr = nullptr;   // nn + 1 block starts
    int32_t* tiles = nullptr;  // ntiles + 1 node-row starts, then ntiles + 1 block starts (tb0)
    void* recs = nullptr;      // nblk records
};

// The node-block copy of (A, val) when A qualifies (rows a multiple of 3,
// every node row's three rows made of aligned column triples, at most
// kNodeCap blocks per node row): S.nblk > 0. A matrix that does not qualify
// leaves S empty and returns MPG_OK (required: MPG_ERR_UNSUPPORTED).
// alt_bytes >= 0: build only when node_wins over a copy streaming alt_bytes.
int node_build(mpg_ctx* ctx, const mpg_csr* A, int vtype, const void* val, bool required, NodeCopy& S,
               int64_t alt_bytes = -1);
void node_free(NodeCopy& S);
// bytes the Arnoldi SpMV streams from the copy: records, block and tile starts
int64_t node_bytes(const NodeCopy& S);

// The node copy over an alternative streaming alt bytes: fewer bytes, or
// at most 10 % more when x (x_bytes) outgrows an XCD's 4 MB L2, where the
// alternative's per-entry gathers cost more than the node records' one per
// block (C4's stencil, x 16 MB: node 1506 MB in 295-312 us against the
// stepped SELL copy's 1438 MB in 324 us; one eighth of it, x 2.2 MB: SELL
// 36 us, node 41 us; profiles/r05_node_ab.jsonl).
inline bool node_wins(int64_t node, int64_t alt, int64_t x_bytes) {
    return node * 10 < alt * (x_bytes > ((int64_t)4 << 20) ? 11 : 10);
}
// tiles per workgroup of the pipelined walk (node_tiles): MPG_NODE_TPW, default 2
int node_tpw_default();
// 1: workgroups take their tiles in XCD order (S.xcd, MPG_NODE_XCD overrides)
int node_xcd(const NodeCopy& S);

inline int node_rec_bytes(int vtype) { return vtype == MPG_F64 ? 80 : vtype == MPG_F32 ? 40 : 24; }

template <class VI> struct NodeRec;
template <> struct NodeRec<float> { static constexpr int R = 40; };
template <> struct NodeRec<double> { static constexpr int R = 80; };
template <> struct NodeRec<half_v> { static constexpr int R = 24; };

typedef uint32_t u32x4a8_t __attribute__((ext_vector_type(4), aligned(8)));
typedef uint32_t u32x2a8_t __attribute__((ext_vector_type(2), aligned(8)));

// One record's raw words, loaded with 16-byte (8-byte aligned) loads and
// kept undecoded until used, so that no load is waited for before all are
// in flight.
template <class VI>
struct NodeWords {
    static constexpr int R = NodeRec<VI>::R;
    static constexpr int N16 = R / 16, N8 = (R % 16) / 8;
    u32x4a8_t q[N16 > 0 ? N16 : 1];
    u32x2a8_t d[N8 > 0 ? N8 : 1];
    __device__ __forceinline__ void load(const char* __restrict__ p) {
#pragma unroll
        for (int i = 0; i < N16; ++i) q[i] = *reinterpret_cast<const u32x4a8_t*>(p + 16 * i);
        if constexpr (N8 > 0) d[0] = *reinterpret_cast<const u32x2a8_t*>(p + 16 * N16);
    }
    __device__ __forceinline__ uint32_t word(int w) const {
        return w < 4 * N16 ? q[w / 4][w % 4] : d[0][w - 4 * N16];
    }
    __device__ __forceinline__ int col() const { return (int)word(0); }
    __device__ __forceinline__ double val(int e) const {
        if constexpr (std::is_same_v<VI, float>) {
            return (double)__uint_as_float(word(1 + e));
        } else if constexpr (std::is_same_v<VI, double>) {
            return __hiloint2double((int)word(3 + 2 * e), (int)word(2 + 2 * e));
        } else {
            const uint32_t w = word(1 + e / 2);
            return (double)to_float((uint16_t)(e & 1 ? w >> 16 : w & 0xffffu));
        }
    }
};

// Row sums of tile t: epi(row, sum, pre(row)) once per matrix row of
// the tile's node rows. pre(row) for this lane's first row is issued ahead
// of the tile's loads.
template <class VI, class A = double, class XF, class PF, class EPI>
__device__ __forceinline__ void node_tile(int t, const int32_t* __restrict__ tiles, const int32_t* __restrict__ bptr,
                                          const char* __restrict__ recs, XF xval, PF pre, EPI epi,
                                          double* __restrict__ prod) {
    constexpr int R = NodeRec<VI>::R;
    const int nr0 = tiles[t], nr1 = tiles[t + 1];
    const int b0 = bptr[nr0], nb = bptr[nr1] - b0;
    const int rows = kNodeDof * (nr1 - nr0);
    // this lane's first row: its node row's blocks and epilogue operands
    const int rf = threadIdx.x < rows ? (int)threadIdx.x : 0;
    const int nf = nr0 + rf / kNodeDof;
    const int fa = bptr[nf] - b0, fz = bptr[nf + 1] - b0;
    const auto pf = pre(kNodeDof * nr0 + rf);
    __builtin_amdgcn_sched_barrier(0);
    if (nb > 0) {
        const int l = threadIdx.x;
        NodeWords<VI> w;
        w.load(recs + (int64_t)(b0 + (l < nb ? l : nb - 1)) * R);
        __builtin_amdgcn_sched_barrier(0);
        const int c = w.col();
        const double x0 = xval(c), x1 = xval(c + 1), x2 = xval(c + 2);
        if (l < nb) {
            double* p = prod + l * (kNodeDof * kNodeDof);
#pragma unroll
            for (int k = 0; k < kNodeDof; ++k) {
                p[3 * k + 0] = w.val(3 * k + 0) * x0;
                p[3 * k + 1] = w.val(3 * k + 1) * x1;
                p[3 * k + 2] = w.val(3 * k + 2) * x2;
            }
        }
    }
    __syncthreads();
    for (int r = threadIdx.x; r < rows; r += kBlock) {
        const bool first = r == (int)threadIdx.x;
        const int nr = nr0 + r / kNodeDof, k = r % kNodeDof;
        const int a = first ? fa : bptr[nr] - b0, z = first ? fz : bptr[nr + 1] - b0;
        A acc = A(0);
        for (int b = a; b < z; ++b) {
            const double* p = prod + b * (kNodeDof * kNodeDof) + kNodeDof * k;
            add_prod(acc, p[0]);
            add_prod(acc, p[1]);
            add_prod(acc, p[2]);
        }
        epi(kNodeDof * nr0 + r, acc, first ? pf : pre(kNodeDof * nr0 + r));
    }
}

// Tiles [t0, t1) in turn on one workgroup, software-pipelined: the next
// tile's records are loaded while this tile's gathers, products and row sums
// run, so each workgroup keeps twice the bytes in flight. tb0[t] = bptr of
// tiles[t] (the record addresses without the dependent bptr load). Barriers
// wait for LDS only (lds_barrier): __syncthreads would also drain the
// prefetched records. (Two tiles ahead measured no better: fem27 227 vs
// 218 us, C4 298 vs 295 us, profiles/r05_node_ab.jsonl.)
// xraw(c) loads x's raw entry c, xfin(raw) turns it into the fp64 factor.
// (Issuing the next tile's gathers before this tile's row sums and
// converting them after was slower: fem27 211 -> 231 us, C4 301 -> 327,
// stencil27p 347 -> 357; profiles/r05_node_ab.jsonl.)
// first(): called by every thread once, after the first tile's raw gathers
// are issued and before xfin is applied to them (k_node_spmv's riding
// normalisation forms its scale there, under the gathers' latency).
struct NoFirst {
    __device__ __forceinline__ void operator()() const {}
};
template <class VI, class A = double, class XR, class XF, class PF, class EPI, class FIRST = NoFirst>
__device__ __forceinline__ void node_tiles(int t0, int t1, const int32_t* __restrict__ tiles,
                                           const int32_t* __restrict__ tb0, const int32_t* __restrict__ bptr,
                                           const char* __restrict__ recs, int64_t nblk, XR xraw, XF xfin, PF pre,
                                           EPI epi, double* __restrict__ prod, FIRST first = FIRST{}) {
    constexpr int R = NodeRec<VI>::R;
    const int l = threadIdx.x;
    auto rec = [&](int t) {
        const int b0 = tb0[t], nb = tb0[t + 1] - b0;
        int64_t b = (int64_t)b0 + (l < nb ? l : nb - 1);
        b = b < 0 ? 0 : b >= nblk ? nblk - 1 : b;
        return recs + b * R;
    };
    NodeWords<VI> cur, nxt;
    cur.load(rec(t0));
    for (int t = t0; t < t1; ++t) {
        const int nr0 = tiles[t], nr1 = tiles[t + 1];
        const int b0 = tb0[t], nb = tb0[t + 1] - b0;
        const int rows = kNodeDof * (nr1 - nr0);
        const int rf = l < rows ? l : 0;
        const int nf = nr0 + rf / kNodeDof;
        const int fa = bptr[nf] - b0, fz = bptr[nf + 1] - b0;
        const auto pf = pre(kNodeDof * nr0 + rf);
        const int c = cur.col();
        const auto r0 = xraw(c), r1 = xraw(c + 1), r2 = xraw(c + 2);
        if (t == t0) first();
        const double x0 = xfin(r0), x1 = xfin(r1), x2 = xfin(r2);
        if (t + 1 < t1) nxt.load(rec(t + 1));
        if (l < nb) {
            double* p = prod + l * (kNodeDof * kNodeDof);
#pragma unroll
            for (int k = 0; k < kNodeDof; ++k) {
                p[3 * k + 0] = cur.val(3 * k + 0) * x0;
                p[3 * k + 1] = cur.val(3 * k + 1) * x1;
                p[3 * k + 2] = cur.val(3 * k + 2) * x2;
            }
        }
        lds_barrier();
        for (int r = l; r < rows; r += kBlock) {
            const bool first = r == l;
            const int nr = nr0 + r / kNodeDof, k = r % kNodeDof;
            const int a = first ? fa : bptr[nr] - b0, z = first ? fz : bptr[nr + 1] - b0;
            A acc = A(0);
            int b = a;
            // kNodeSumAhead blocks' products read before any is added (the
            // same order): one LDS round trip per four blocks, not per block
            for (; b + kNodeSumAhead <= z; b += kNodeSumAhead) {
                double v[3 * kNodeSumAhead];
#pragma unroll
                for (int u = 0; u < kNodeSumAhead; ++u) {
                    const double* p = prod + (b + u) * (kNodeDof * kNodeDof) + kNodeDof * k;
                    v[3 * u] = p[0];
                    v[3 * u + 1] = p[1];
                    v[3 * u + 2] = p[2];
                }
#pragma unroll
                for (int u = 0; u < 3 * kNodeSumAhead; ++u) add_prod(acc, v[u]);
            }
            for (; b < z; ++b) {
                const double* p = prod + b * (kNodeDof * kNodeDof) + kNodeDof * k;
                add_prod(acc, p[0]);
                add_prod(acc, p[1]);
                add_prod(acc, p[2]);
            }
            epi(kNodeDof * nr0 + r, acc, first ? pf : pre(kNodeDof * nr0 + r));
        }
        lds_barrier();
        cur = nxt;
    }
}

}  // namespace mpg
