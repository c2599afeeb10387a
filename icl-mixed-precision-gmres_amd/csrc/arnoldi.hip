// Fused Arnoldi phase kernels for gfx950 (include/mpgmres/arnoldi.h).
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
// The kernels live in arnoldi_kernels.hpp, the launch code (templated on the
// accumulation class) in arnoldi_launch.hpp; this file is the C-ABI and the
// fp64-accumulation build, arnoldi_acc32.hip the fp32-accumulation one.
#include "arnoldi_kernels.hpp"
#include "arnoldi_launch.hpp"

#include <cstdlib>
#include <new>
#include <algorithm>
#include <vector>

using namespace mpg;

namespace {

int64_t sell_copy_bytes(const mpg_arnoldi* a);

// the Arnoldi SpMV's copy of the inner-precision values: SELL-64, node
// blocks or none (CSR row blocks). Auto (format 0) takes the node-block copy
// when the matrix has one and node_wins over what auto would run otherwise
// (the SpMV is HBM-bound; 3-dof FEM: 4.44 B per fp32 nonzero against CSR's
// 8). MPG_NODE=0: never.
// The residual prologue on node blocks when the Arnoldi SpMV runs on them
// (k_node_rowsums + k_prologue_rows: the CSR prologue's bits): the node copy
// itself when it holds the outer values (baseline mode), else an fp64 node
// copy of them when it streams fewer bytes than the fp64 CSR arrays. One GPU
// (no lower halo); optional: a copy that cannot be built leaves the CSR
// prologue. MPG_NODE_PROLOGUE=0: never.
void node_prologue_build(mpg_arnoldi* a) {
    const char* e = std::getenv("MPG_NODE_PROLOGUE");
    if ((e && *e == '0') || a->node.nblk == 0 || a->d.n_front != 0 || a->d.outer_type != MPG_F64) return;
    if (hipMalloc((void**)&a->rsum, (size_t)std::max(a->d.n, 1) * sizeof(double)) != hipSuccess) {
        (void)hipGetLastError();
        return;
    }
    if (a->d.val_outer == a->d.val_inner && a->d.inner_val == MPG_F64) {
        a->node_res = &a->node;
        return;
    }
    const int64_t csr = a->d.A->nnz * 12 + ((int64_t)a->d.n + 1) * 4;
    if (node_build(a->ctx, a->d.A, MPG_F64, a->d.val_outer, false, a->node_outer, csr) != MPG_OK ||
        a->node_outer.nblk == 0) {
        node_free(a->node_outer);
        (void)hipGetLastError();
        (void)hipFree(a->rsum);
        a->rsum = nullptr;
        return;
    }
    a->node_res = &a->node_outer;
}

int arnoldi_sell_build(mpg_arnoldi* a, int format) {
    if (format == 3) {
        if (int st = node_build(a->ctx, a->d.A, a->d.inner_val, a->d.val_inner, true, a->node)) return st;
        node_prologue_build(a);
        return MPG_OK;
    }
    if (int st = sell_build(a->ctx, a->d.A, a->d.inner_val, a->d.val_inner, format, a->sell)) return st;
    const char* ne = std::getenv("MPG_NODE");
    if (format == 0 && !(ne && *ne == '0')) {
        const int64_t vb = a->d.inner_val == MPG_F64 ? 8 : a->d.inner_val == MPG_F32 ? 4 : 2;
        const int64_t now = a->sell.nslices > 0 ? sell_copy_bytes(a) : a->d.A->nnz * (4 + vb) + ((int64_t)a->d.n + 1) * 4;
        NodeCopy nc;
        // (auto's node copy is an optimisation: a copy that cannot be built --
        // its records' allocation failing on a large matrix -- leaves the
        // SELL / CSR storage in place instead of failing the create)
        if (node_build(a->ctx, a->d.A, a->d.inner_val, a->d.val_inner, false, nc, now) != MPG_OK) {
            node_free(nc);
            (void)hipGetLastError();
            return MPG_OK;
        }
        if (nc.nblk > 0) {  // (built only when it wins)
            sell_free(a->sell);
            a->node = nc;
            node_prologue_build(a);
            return MPG_OK;
        }
    }
    if (a->sell.nslices == 0) return MPG_OK;
    // the residual prologue on the same slicing: shared when the residual and
    // Arnoldi matrices are the same array, else a copy of the outer values
    a->outer_is_inner = a->d.val_outer == a->d.val_inner && a->d.outer_type == a->d.inner_val;
    const int grid = (a->sell.nslices + kBlock / kWave - 1) / (kBlock / kWave);
    a->fd_gs = (grid + kCombineGroups - 1) / kCombineGroups;
    a->fd_ng = (grid + a->fd_gs - 1) / a->fd_gs;
    if (hipMalloc((void**)&a->fd_part, (size_t)kNC * grid * sizeof(double)) != hipSuccess ||
        hipMalloc((void**)&a->fd_cnt, (size_t)a->fd_ng * sizeof(unsigned)) != hipSuccess ||
        hipMemsetAsync(a->fd_cnt, 0, (size_t)a->fd_ng * sizeof(unsigned), a->ctx->stream) != hipSuccess)
        return MPG_ERR_ALLOC;
    if (a->outer_is_inner) return MPG_OK;
    return sell_build(a->ctx, a->d.A, a->d.outer_type, a->d.val_outer, 2, a->sell_outer);
}


// fp64 accumulation here; fp32 accumulation (mpg_arnoldi_set_accum, fp32
// Arnoldi only) in arnoldi_acc32.hip
int spmv_impl(mpg_arnoldi_t a, int k, int fold, bool dots = false) {
    return a && a->acc32 ? mpg_acc32::spmv(a, k, fold, dots) : spmv_run<double>(a, k, fold, dots);
}
int dots_impl(mpg_arnoldi_t a, int k, bool combine) {
    return a && a->acc32 ? mpg_acc32::dots(a, k, combine) : dots_run<double>(a, k, combine);
}
int cgs_impl(mpg_arnoldi_t a, int k, int pass, bool givens, bool from_partials = false, bool no_next = false) {
    return a && a->acc32 ? mpg_acc32::cgs(a, k, pass, givens, from_partials, no_next)
                         : cgs_run<double>(a, k, pass, givens, from_partials, no_next);
}
int mgs_impl(mpg_arnoldi_t a, int k, int j, bool from_partials) {
    return a && a->acc32 ? mpg_acc32::mgs(a, k, j, from_partials) : mgs_run<double>(a, k, j, from_partials);
}
int givens_impl(mpg_arnoldi_t a, int k, bool from_partials) {
    return a && a->acc32 ? mpg_acc32::givens(a, k, from_partials) : givens_run<double>(a, k, from_partials);
}

}  // namespace

extern "C" {

int mpg_arnoldi_create(mpg_ctx_t ctx, const mpg_arnoldi_desc* desc, mpg_arnoldi_t* out) {
    if (!ctx || !desc || !out || !desc->A || desc->n < 0 || desc->n_ext < desc->n || desc->m < 1 ||
        desc->m > 1000 || desc->orth < 0 || desc->orth > 2)
        return MPG_ERR_ARG;
    *out = nullptr;
    int combo = combo_of(*desc);
    if (combo < 0) return MPG_ERR_UNSUPPORTED;
    if (desc->A->rows != desc->n || desc->A->cols > desc->n_ext) return MPG_ERR_ARG;
    if (desc->inner_row_exp && desc->inner_val != MPG_F16) return MPG_ERR_ARG;  // only fp16 copies are scaled
    mpg_arnoldi* a = new (std::nothrow) mpg_arnoldi();
    if (!a) return MPG_ERR_ALLOC;
    a->ctx = ctx;
    a->d = *desc;
    a->combo = combo;
    a->tsize = desc->vec_type == MPG_F64 ? 8 : 4;
    a->G = desc->A->nblocks < kGroups ? (desc->A->nblocks > 0 ? desc->A->nblocks : 1) : kGroups;
    a->Grb = desc->A->nblocks > 0 ? desc->A->nblocks : 1;
    a->Gd = (int)std::min<int64_t>(kCombineGroups, std::max<int64_t>(1, ((int64_t)desc->n + 4 * kCombineBlock - 1) /
                                                                          (4 * kCombineBlock)));
    if (desc->n_front < 0) {
        delete a;
        return MPG_ERR_ARG;
    }
    a->front = MPG_FRONT_PAD(desc->n_front);
    const size_t align = 256 / a->tsize;
    a->ld = ((int64_t)desc->n + align - 1) / align * align;
    if (a->ld == 0) a->ld = align;
    const int m = desc->m;
    auto alloc = [&](void** p, size_t bytes) {
        if (hipMalloc(p, bytes ? bytes : 16) != hipSuccess) return false;
        return hipMemsetAsync(*p, 0, bytes ? bytes : 16, ctx->stream) == hipSuccess;
    };
    bool ok = alloc(&a->V, (size_t)a->ld * (m + 1) * a->tsize) && alloc(&a->H, (size_t)(m + 1) * m * a->tsize) &&
              alloc(&a->small, (size_t)6 * (m + 1) * a->tsize) &&
              alloc(&a->wbase[0], (size_t)(a->front + desc->n_ext + 64) * a->tsize) &&
              alloc(&a->wbase[1], (size_t)(a->front + desc->n_ext + 64) * a->tsize) &&
              alloc((void**)&a->partial, std::max<size_t>(std::max<size_t>((size_t)(kNC + 4) * a->Grb,
                                                                           (size_t)(m + 4) * a->G),
                                                          (size_t)kNC * kCombineGroups) *  // uniform groups
                                             sizeof(double)) &&
              alloc((void**)&a->sums, (size_t)(m + 8) * sizeof(double)) &&
              alloc((void**)&a->report, (size_t)(m + 8) * sizeof(double)) &&
              alloc((void**)&a->dpart, (size_t)kNC * kCombineGroups * sizeof(double)) &&
              alloc((void**)&a->counters, 256);
    for (int q = 0; q < 2; ++q)
        a->w[q] = a->wbase[q] ? static_cast<char*>(a->wbase[q]) + (size_t)a->front * a->tsize : nullptr;
    if (!ok) {
        mpg_arnoldi_destroy(a);
        return MPG_ERR_ALLOC;
    }
    a->last_part = a->partial;
    if (desc->spmv_format < 0 || desc->spmv_format > 3) {
        mpg_arnoldi_destroy(a);
        return MPG_ERR_ARG;
    }
    if (int st = arnoldi_sell_build(a, desc->spmv_format)) {
        mpg_arnoldi_destroy(a);
        return st;
    }
    *out = a;
    return MPG_OK;
}

int64_t mpg_arnoldi_sell_matrix_bytes(mpg_arnoldi_t a) {
    if (a && a->node.nblk > 0) return node_bytes(a->node) + (a->d.inner_row_exp ? (int64_t)a->d.n : 0);
    if (!a || a->sell.nslices == 0) return 0;
    return sell_copy_bytes(a);
}

namespace {
int64_t sell_copy_bytes(const mpg_arnoldi* a) {
    return sell_matrix_bytes(a->sell) + (a->d.inner_row_exp ? (int64_t)a->d.n : 0);
}
}  // namespace

int mpg_arnoldi_sell_sigma(mpg_arnoldi_t a) { return a ? a->sell.sigma : -1; }

int64_t mpg_arnoldi_sell_shared_slices(mpg_arnoldi_t a) { return a ? a->sell.nshared : -1; }

int mpg_arnoldi_slices_per_wave(mpg_arnoldi_t a) {
    if (!a || a->sell.nslices == 0) return 0;
    return sell_uniform(a->sell) && sell_pair(a->sell) ? 2 : 1;
}

int mpg_arnoldi_sell_columns(mpg_arnoldi_t a, int32_t* form, int64_t* csr_slices, int64_t* implicit_slices) {
    if (!a) return MPG_ERR_ARG;
    const SellCopy& S = a->sell;
    if (form) *form = S.nslices == 0 ? -1 : S.c16 ? 1 : S.c16s ? 2 : 0;
    if (csr_slices) *csr_slices = S.nexc;
    if (implicit_slices) *implicit_slices = S.nimp;
    return MPG_OK;
}

int mpg_arnoldi_spmv_layout(mpg_arnoldi_t a, int32_t* format, int32_t* vec_width, int32_t* col_bytes,
                            int64_t* stored, int32_t* window) {
    if (!a) return MPG_ERR_ARG;
    const bool sell = a->sell.nslices > 0, node = a->node.nblk > 0;
    if (format) *format = node ? 3 : sell ? 2 : 1;
    if (vec_width) *vec_width = node ? kNodeDof * kNodeDof : sell ? a->sell.W : 4;
    if (col_bytes) *col_bytes = sell ? a->sell.col_bytes() : 4;  // (node blocks: one per 9 values)
    if (stored) *stored = node ? a->node.nblk * kNodeDof * kNodeDof : sell ? a->sell.padded : a->d.A->nnz;
    if (window) *window = sell && a->sell.win ? 1 : 0;
    return MPG_OK;
}

int mpg_arnoldi_destroy(mpg_arnoldi_t a) {
    if (!a) return MPG_OK;
    if (a->ctx) (void)hipStreamSynchronize(a->ctx->stream);
    void* ps[] = {a->V, a->H, a->small, a->wbase[0], a->wbase[1], a->partial, a->dpart, a->sums, a->report,
                  a->counters, a->fd_part, a->fd_cnt};
    for (void* p : ps)
        if (p) (void)hipFree(p);
    sell_free(a->sell);
    sell_free(a->sell_outer);
    node_free(a->node);
    node_free(a->node_outer);
    if (a->rsum) (void)hipFree(a->rsum);
    delete a;
    return MPG_OK;
}

int mpg_arnoldi_prologue(mpg_arnoldi_t a) {
    if (!a) return MPG_ERR_ARG;
    const mpg_csr* A = a->d.A;
    int st = dispatch(a->combo, [&](auto t, auto x, auto p, auto) {
        using T = decltype(t);
        using X = decltype(x);
        using P = decltype(p);
        const P* diag = a->d.jacobi ? static_cast<const P*>(a->d.diag) : nullptr;
        if (a->node_res && a->rsum) {
            const NodeCopy& N = *a->node_res;
            int tpw = node_tpw_default();
            if (tpw < 1) tpw = 2;
            k_node_rowsums<X><<<(N.ntiles + tpw - 1) / tpw, kBlock, 0, a->ctx->stream>>>(
                N.tiles, N.bptr, static_cast<const char*>(N.recs), N.ntiles, N.nblk, tpw, node_xcd(N),
                static_cast<const X*>(a->d.x), a->rsum);
            a->last_G = rb_grid(a);
            k_prologue_rows<T, X, P><<<rb_grid(a), kBlock, 0, a->ctx->stream>>>(
                A->blocks, A->nblocks, a->rsum, static_cast<const X*>(a->d.x), static_cast<const X*>(a->d.b), diag,
                static_cast<T*>(a->w[0]), a->partial);
            return (int)MPG_OK;
        }
        const SellCopy* S = a->outer_is_inner ? &a->sell : &a->sell_outer;
        if (S->nslices > 0 && S->vtype == a->d.outer_type) {
            const int grid = (S->nslices + kBlock / kWave - 1) / (kBlock / kWave);
            a->last_G = grid;
            return sell_dispatch(*S, [&](auto ci, auto wc) {
                using CI = decltype(ci);
                return sell_dispatch_win(S->win, [&](auto wn) {
                    auto go = [&](auto kern) {
                        kern<<<grid, kBlock, 0, a->ctx->stream>>>(
                            a->d.n, -a->front, a->d.n_ext, S->nslices, S->off, static_cast<const CI*>(S->col),
                            static_cast<const X*>(S->val), static_cast<const X*>(a->d.x),
                            static_cast<const X*>(a->d.b), diag, static_cast<T*>(a->w[0]), a->partial, S->sbase,
                            S->spat, S->coff, static_cast<const CI*>(S->pat), S->xrp, S->xcol, static_cast<const X*>(S->xval),
                            S->ustride, sell_xcd_order(*S) ? 1 : 0, S->rows);
                        return (int)MPG_OK;
                    };
                    constexpr int Wc = decltype(wc)::value;
                    constexpr bool WN = decltype(wn)::value;
                    return sell_uniform(*S) ? go(k_prologue_sell<T, X, P, CI, Wc, WN, true>)
                                            : go(k_prologue_sell<T, X, P, CI, Wc, WN, false>);
                });
            });
        }
        a->last_G = rb_grid(a);
        k_prologue<T, X, P><<<rb_grid(a), kBlock, 0, a->ctx->stream>>>(
            A->blocks, A->nblocks, A->rowptr, A->col, static_cast<const X*>(a->d.val_outer), A->nnz,
            static_cast<const X*>(a->d.x), static_cast<const X*>(a->d.b), diag, static_cast<T*>(a->w[0]),
            a->partial);
        return (int)MPG_OK;
    });
    a->last_part = a->partial;
    if (st) return st;
    MPG_LAUNCH_CHECK(a->ctx);
    return MPG_OK;
}

int mpg_arnoldi_prologue_wnorm(mpg_arnoldi_t a) {
    if (!a) return MPG_ERR_ARG;
    int st = dispatch(a->combo, [&](auto t, auto, auto, auto) {
        using T = decltype(t);
        // the prologue's grid (CSR row blocks or SELL slices): column 1 of its partials
        k_wnorm_partials<T><<<a->last_G, kBlock, 0, a->ctx->stream>>>(a->d.n, static_cast<const T*>(a->w[0]),
                                                                     a->partial);
        return (int)MPG_OK;
    });
    if (st) return st;
    MPG_LAUNCH_CHECK(a->ctx);
    return MPG_OK;
}

int mpg_arnoldi_prologue_finish(mpg_arnoldi_t a) {
    if (!a) return MPG_ERR_ARG;
    int st = dispatch(a->combo, [&](auto t, auto x, auto, auto) {
        using T = decltype(t);
        using X = decltype(x);
        k_prologue_finish<T, X><<<1, 64, 0, a->ctx->stream>>>(a->sums, a->d.m, static_cast<T*>(a->s()),
                                                                static_cast<T*>(a->inv()), a->report);
        return MPG_OK;
    });
    if (st) return st;
    MPG_LAUNCH_CHECK(a->ctx);
    return MPG_OK;
}

int mpg_arnoldi_prologue_finish_partials(mpg_arnoldi_t a) {
    if (!a) return MPG_ERR_ARG;
    int st = dispatch(a->combo, [&](auto t, auto x, auto, auto) {
        using T = decltype(t);
        using X = decltype(x);
        if (a->last_G <= 2 * kBlock)
            k_prologue_finish_parts<T, X, kBlock><<<1, kBlock, 0, a->ctx->stream>>>(
                a->last_G, a->last_part, a->sums, a->d.m, static_cast<T*>(a->s()), static_cast<T*>(a->inv()), a->report);
        else
            k_prologue_finish_parts<T, X, 1024><<<1, 1024, 0, a->ctx->stream>>>(
                a->last_G, a->last_part, a->sums, a->d.m, static_cast<T*>(a->s()), static_cast<T*>(a->inv()), a->report);
        return MPG_OK;
    });
    if (st) return st;
    MPG_LAUNCH_CHECK(a->ctx);
    return MPG_OK;
}

int mpg_arnoldi_reduce(mpg_arnoldi_t a, int ncols) {
    return a && a->acc32 ? mpg_acc32::reduce(a, ncols) : reduce_run<double>(a, ncols);
}

int mpg_arnoldi_spmv(mpg_arnoldi_t a, int k) { return spmv_impl(a, k, 0); }
int mpg_arnoldi_spmv_dots(mpg_arnoldi_t a, int k, int fold) {
    if (fold < 0 || fold > 2) return MPG_ERR_ARG;
    return spmv_impl(a, k, fold, true);
}
int mpg_arnoldi_givens_spmv(mpg_arnoldi_t a, int k) { return spmv_impl(a, k, 1); }
int mpg_arnoldi_givens_partials_spmv(mpg_arnoldi_t a, int k) { return spmv_impl(a, k, 2); }
int mpg_arnoldi_fold_max_m(void) { return kFoldMaxM; }
int mpg_arnoldi_partials_max_cols(void) { return kWideMax; }

// The folded Givens step costs every SpMV workgroup the sum of the previous
// launch's partials and two barriers; a separate Givens launch costs ~4.6 us.
// Measured whole solves (tools/bench_configs.py, profiles/r03_fold_ab.jsonl):
// fold 25.3k vs 24.3k it/s on LAP-1M (1,954 paired workgroups), but 1,756 vs
// 1,787 on the C4 stand-in (16,029 workgroups) and 2,874 vs 3,015 on BAND-100M
// fp16 (19,532): the fold pays up to kFoldMaxGroups SpMV workgroups.
// (MPG_FOLD_MAX_GROUPS overrides the limit: tests put it between two ranks'
// workgroup counts to check that the ranks still decide alike)
constexpr int kFoldMaxGroups = 4096;
int mpg_arnoldi_fold_pays(mpg_arnoldi_t a) {
    if (!a) return 0;
    const char* env = std::getenv("MPG_FOLD_MAX_GROUPS");
    const int64_t limit = env && *env ? std::atoll(env) : kFoldMaxGroups;
    if (a->node.nblk > 0) {
        const int tpw = node_tpw(a->node);
        return (a->node.ntiles + tpw - 1) / tpw <= limit ? 1 : 0;
    }
    const SellCopy& S = a->sell;
    if (S.nslices == 0) return a->Grb <= limit ? 1 : 0;
    const int per_group = (kStepSellBlock / kWave) * (sell_uniform(S) && sell_pair(S) ? 2 : 1);
    return (S.nslices + per_group - 1) / per_group <= limit ? 1 : 0;
}

int mpg_arnoldi_dots(mpg_arnoldi_t a, int k) { return dots_impl(a, k, false); }
int mpg_arnoldi_dots_sums(mpg_arnoldi_t a, int k) { return dots_impl(a, k, true); }

int mpg_arnoldi_cgs(mpg_arnoldi_t a, int k, int pass) { return cgs_impl(a, k, pass, false); }
int mpg_arnoldi_cgs_partials(mpg_arnoldi_t a, int k) { return cgs_impl(a, k, 0, false, true); }
int mpg_arnoldi_cgs_givens(mpg_arnoldi_t a, int k, int pass) { return cgs_impl(a, k, pass, true); }
int mpg_arnoldi_cgsr_wide_pass(mpg_arnoldi_t a, int k, int pass) { return cgs_impl(a, k, pass, false, true, true); }

int mpg_arnoldi_mgs(mpg_arnoldi_t a, int k, int j) { return mgs_impl(a, k, j, false); }
int mpg_arnoldi_mgs_partials(mpg_arnoldi_t a, int k, int j) { return mgs_impl(a, k, j, true); }

int mpg_arnoldi_givens(mpg_arnoldi_t a, int k) { return givens_impl(a, k, false); }
int mpg_arnoldi_givens_partials(mpg_arnoldi_t a, int k) { return givens_impl(a, k, true); }

int mpg_arnoldi_update(mpg_arnoldi_t a, int k) {
    return a && a->acc32 ? mpg_acc32::update(a, k) : update_run<double>(a, k);
}

int mpg_arnoldi_set_accum(mpg_arnoldi_t a, int accum) {
    if (!a || (accum != MPG_ACCUM_F64 && accum != MPG_ACCUM_F32)) return MPG_ERR_ARG;
    // an fp64 Arnoldi accumulates in fp64 either way (cblas_d*: the reference's class)
    a->acc32 = accum == MPG_ACCUM_F32 && a->tsize == 4;
    return MPG_OK;
}

int mpg_arnoldi_accum(mpg_arnoldi_t a) { return !a ? MPG_ERR_ARG : a->acc32 ? MPG_ACCUM_F32 : MPG_ACCUM_F64; }

int mpg_arnoldi_prologue_format(mpg_arnoldi_t a) {
    if (!a) return MPG_ERR_ARG;
    if (a->node_res && a->rsum) return 3;
    const SellCopy* S = a->outer_is_inner ? &a->sell : &a->sell_outer;
    return S->nslices > 0 && S->vtype == a->d.outer_type ? 2 : 1;
}

double* mpg_arnoldi_sums_dev(mpg_arnoldi_t a) { return a ? a->sums : nullptr; }
void* mpg_arnoldi_wprev_dev(mpg_arnoldi_t a, int k) { return a ? a->w[k & 1] : nullptr; }
int mpg_arnoldi_vec_bytes(mpg_arnoldi_t a) { return a ? (int)a->tsize : 0; }
const double* mpg_arnoldi_report_dev(mpg_arnoldi_t a) { return a ? a->report : nullptr; }
int mpg_arnoldi_report_len(mpg_arnoldi_t a) { return a ? a->d.m + 4 : 0; }
const void* mpg_arnoldi_basis_dev(mpg_arnoldi_t a, int64_t* ld) {
    if (!a) return nullptr;
    if (ld) *ld = a->ld;
    return a->V;
}
const void* mpg_arnoldi_hessenberg_dev(mpg_arnoldi_t a) { return a ? a->H : nullptr; }
const void* mpg_arnoldi_inv_dev(mpg_arnoldi_t a) { return a ? a->inv() : nullptr; }
int mpg_arnoldi_time_next_spmv(mpg_arnoldi_t a, void* start_event, void* stop_event) {
    if (!a || !start_event || !stop_event) return MPG_ERR_ARG;
    a->ctx->time_start = static_cast<hipEvent_t>(start_event);
    a->ctx->time_stop = static_cast<hipEvent_t>(stop_event);
    return MPG_OK;
}
int mpg_arnoldi_stamp_next(mpg_arnoldi_t a, unsigned long long* slots, int64_t cap_waves) {
    if (!a || (slots && cap_waves < 1)) return MPG_ERR_ARG;
    a->ctx->stamp_next = slots;
    a->ctx->stamp_cap = slots ? cap_waves : 0;
    return MPG_OK;
}
int64_t mpg_arnoldi_stamp_waves(mpg_arnoldi_t a) {
    if (!a) return MPG_ERR_ARG;
    // the most waves a stamped launch has: the one-panel dots / CGS update
    // (Gd 1024-thread workgroups, or row_grid 256-thread ones for CGSR's
    // first pass)
    int64_t w = (int64_t)a->Gd * (kCombineBlock / kWave);
    w = std::max<int64_t>(w, (int64_t)row_grid(a) * (kBlock / kWave));
    return w;
}
int mpg_arnoldi_num_groups(mpg_arnoldi_t a) { return a ? a->G : 0; }
double* mpg_arnoldi_partials_dev(mpg_arnoldi_t a) { return a ? a->last_part : nullptr; }
// the last producer wrote last_G partials per column; the one-column
// producers (CGS/MGS updates, MGS dots) are what a caller all-reduces
int mpg_arnoldi_partials_count(mpg_arnoldi_t a) { return a ? a->last_G : 0; }
int mpg_arnoldi_uniform_groups(mpg_arnoldi_t a) {
    if (!a) return MPG_ERR_ARG;
    a->Gd = kCombineGroups;
    return MPG_OK;
}

}  // extern "C"