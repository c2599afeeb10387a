// Launch code of the fused Arnoldi phases, templated on the accumulation
// class A of the fp32-Arnoldi kernels (arnoldi_kernels.hpp): arnoldi.hip
// instantiates A = double for every type combination, arnoldi_acc32.hip A =
// float for the fp32-Arnoldi combinations only (mpg_arnoldi_set_accum), each
// in its own translation unit so the two builds compile in parallel.
#pragma once

#include "arnoldi_kernels.hpp"

#include <algorithm>
#include <cstdlib>
#include <type_traits>

namespace {

// the type combinations an accumulation class exists for: A = double for all
// of them, A = float for the fp32 Arnoldi (single, mixed, mixed-half) only
template <class A, class F>
int dispatch_acc(int combo, F&& f) {
    if constexpr (std::is_same_v<A, double>) {
        return dispatch(combo, f);
    } else {
        switch (combo) {
            case 2: return f(float(), float(), float(), float());
            case 3: return f(float(), double(), float(), float());
            case 4: return f(float(), double(), float(), half_v());
            default: return MPG_ERR_UNSUPPORTED;
        }
    }
}

template <class A>
int reduce_run(mpg_arnoldi_t a, int ncols) {
    if (!a || ncols < 1 || ncols > a->d.m + 4) return MPG_ERR_ARG;
    // one column per workgroup: 256 threads when the producer left <= 512
    // partials per column (one or two loads per thread), else 1024
    if (a->last_G <= 2 * kBlock) k_reduce_partials<kBlock, A><<<ncols, kBlock, 0, a->ctx->stream>>>(a->last_G, a->last_part, a->sums);
    else k_reduce_partials<1024, A><<<ncols, 1024, 0, a->ctx->stream>>>(a->last_G, a->last_part, a->sums);
    MPG_LAUNCH_CHECK(a->ctx);
    return MPG_OK;
}


// fold: 0 plain; 1 Givens(k-1) folded, ||w||^2 from sums[0]; 2 from the partials.
// dots: the panel dots fused (SellDots; MPG_ERR_UNSUPPORTED where the SELL
// copy, an fp32 basis with fp32 values, int16 columns and the window are
// not all present -- the caller then launches the dots itself).
// workgroup of the SELL step kernel without fused dots (4 slices per 256)
#ifndef MPG_STEP_SELL_BLOCK
#define MPG_STEP_SELL_BLOCK 256
#endif
constexpr int kStepSellBlock = MPG_STEP_SELL_BLOCK;
using kBlockC = std::integral_constant<int, kBlock>;

template <class A>
int spmv_run(mpg_arnoldi_t a, int k, int fold, bool dots) {
    if (!a || k < 0 || k >= a->d.m) return MPG_ERR_ARG;
    if (dots && (!std::is_same_v<A, double> || a->d.n <= 0 || a->sell.nslices == 0 || !a->sell.c16 || !a->sell.win ||
                 (a->combo != 2 && a->combo != 3) || k + 1 > kNC || a->d.orth == kOrthMGS))
        return MPG_ERR_UNSUPPORTED;
    if (fold && (k < 1 || a->d.m > kFoldMaxM)) return MPG_ERR_ARG;
    const mpg_csr* Acsr = a->d.A;
    int st = dispatch_acc<A>(a->combo, [&](auto t, auto, auto p, auto vi) {
        using T = decltype(t);
        using P = decltype(p);
        using VI = decltype(vi);
        const P* diag = a->d.jacobi ? static_cast<const P*>(a->d.diag) : nullptr;
        GivensFold<T> gf{nullptr, 0, {}};
        if (fold)
            gf = GivensFold<T>{fold == 2 ? a->last_part : a->sums, fold == 2 ? a->last_G : 0, givens_args<T>(a, k - 1)};
        if (a->sell.nslices > 0) {
            const auto& S = a->sell;
            if (fold == 2 && a->last_G > kBlock) return (int)MPG_ERR_ARG;  // k_step_sell folds <= kBlock partials
            return sell_dispatch(S, [&](auto ci, auto wc) {
                using CI = decltype(ci);
                constexpr int Wc = decltype(wc)::value;
                auto launch = [&](auto kern, SellDots dd, auto bs) {
                    constexpr int BS = decltype(bs)::value;
                    const int grid = (S.nslices + BS / kWave - 1) / (BS / kWave);
                    launch_timed(a->ctx, kern, dim3(grid), dim3(BS),
                            a->d.n, -a->front, a->d.n_ext, S.nslices, S.off, static_cast<const CI*>(S.col),
                            static_cast<const typename SellStore<VI>::type*>(S.val),
                            static_cast<const T*>(a->w[k & 1]), static_cast<const T*>(a->inv()),
                            static_cast<T*>(a->V), a->ld, k, diag, static_cast<T*>(a->w[(k + 1) & 1]), gf, dd,
                            S.sbase, S.spat, S.coff, static_cast<const CI*>(S.pat), S.xrp, S.xcol,
                            static_cast<const typename SellStore<VI>::type*>(S.xval), a->d.inner_row_exp,
                            S.ustride, sell_xcd_order(S) ? 1 : 0, S.rows);
                    return (int)MPG_OK;
                };
                if constexpr (std::is_same_v<T, float> && std::is_same_v<VI, float> &&
                              std::is_same_v<CI, int16_t> && std::is_same_v<A, double>) {
                    if (dots) {
                        const SellDots dd{k + 1, a->fd_gs, a->fd_ng, a->fd_part, a->fd_cnt, a->dpart};
                        auto pick = [&](auto dn) {
                            constexpr int DN = decltype(dn)::value;
                            return fold ? launch(k_step_sell<T, P, VI, CI, Wc, true, true, DN, kBlock, false, false, A>, dd, kBlockC())
                                        : launch(k_step_sell<T, P, VI, CI, Wc, true, false, DN, kBlock, false, false, A>, dd, kBlockC());
                        };
                        if (k + 1 <= 8) return pick(std::integral_constant<int, 8>());
                        if (k + 1 <= 16) return pick(std::integral_constant<int, 16>());
                        return pick(std::integral_constant<int, 32>());
                    }
                }
                return sell_dispatch_win(S.win, [&](auto wn) {
                    constexpr bool WN = decltype(wn)::value;
                    using BSC = std::integral_constant<int, kStepSellBlock>;
                    const int be = sell_uniform(S) ? sell_pair(S) : 0;
                    if constexpr (std::is_same_v<CI, int16_t> && (Wc == 2 || Wc == 4)) if (be) {
                        auto launch2 = [&](auto kern) {
                            const int grid = (S.nslices + 2 * (kStepSellBlock / kWave) - 1) / (2 * (kStepSellBlock / kWave));
                            launch_timed(a->ctx, kern, dim3(grid), dim3(kStepSellBlock),
                                    a->d.n, -a->front, a->d.n_ext, S.nslices, S.off, static_cast<const CI*>(S.col),
                                    static_cast<const typename SellStore<VI>::type*>(S.val),
                                    static_cast<const T*>(a->w[k & 1]), static_cast<const T*>(a->inv()),
                                    static_cast<T*>(a->V), a->ld, k, diag, static_cast<T*>(a->w[(k + 1) & 1]), gf,
                                    SellDots{}, S.sbase, S.spat, S.coff, static_cast<const CI*>(S.pat), S.xrp, S.xcol,
                                    static_cast<const typename SellStore<VI>::type*>(S.xval), a->d.inner_row_exp,
                                    S.ustride, sell_xcd_order(S) ? 1 : 0);
                            return (int)MPG_OK;
                        };
                        const char* pge = std::getenv("MPG_SELL_PREGATHER");
                        if (!WN && pge && *pge == '0') {
                            if (be == 8)
                                return fold ? launch2(k_step_sell2<T, P, VI, Wc, WN, true, 8, kStepSellBlock, false, A>)
                                            : launch2(k_step_sell2<T, P, VI, Wc, WN, false, 8, kStepSellBlock, false, A>);
                            return fold ? launch2(k_step_sell2<T, P, VI, Wc, WN, true, 12, kStepSellBlock, false, A>)
                                        : launch2(k_step_sell2<T, P, VI, Wc, WN, false, 12, kStepSellBlock, false, A>);
                        }
                        if (be == 8)
                            return fold ? launch2(k_step_sell2<T, P, VI, Wc, WN, true, 8, kStepSellBlock, true, A>)
                                        : launch2(k_step_sell2<T, P, VI, Wc, WN, false, 8, kStepSellBlock, true, A>);
                        if constexpr (Wc == 2) if (be == 10)
                            return fold ? launch2(k_step_sell2<T, P, VI, Wc, WN, true, 10, kStepSellBlock, true, A>)
                                        : launch2(k_step_sell2<T, P, VI, Wc, WN, false, 10, kStepSellBlock, true, A>);
                        if (be != 12) return (int)MPG_ERR_UNSUPPORTED;
                        return fold ? launch2(k_step_sell2<T, P, VI, Wc, WN, true, 12, kStepSellBlock, true, A>)
                                    : launch2(k_step_sell2<T, P, VI, Wc, WN, false, 12, kStepSellBlock, true, A>);
                    }
                    if constexpr (!WN && !std::is_same_v<CI, int16_t>) if (sell_pipe(S)) {
                        if (sell_uniform(S))
                            return fold ? launch(k_step_sell<T, P, VI, CI, Wc, WN, true, 0, kStepSellBlock, true, true, A>,
                                                 SellDots{}, BSC())
                                        : launch(k_step_sell<T, P, VI, CI, Wc, WN, false, 0, kStepSellBlock, true, true, A>,
                                                 SellDots{}, BSC());
                        return fold ? launch(k_step_sell<T, P, VI, CI, Wc, WN, true, 0, kStepSellBlock, false, true, A>,
                                             SellDots{}, BSC())
                                    : launch(k_step_sell<T, P, VI, CI, Wc, WN, false, 0, kStepSellBlock, false, true, A>,
                                             SellDots{}, BSC());
                    }
                    if (sell_uniform(S))
                        return fold ? launch(k_step_sell<T, P, VI, CI, Wc, WN, true, 0, kStepSellBlock, true, false, A>,
                                             SellDots{}, BSC())
                                    : launch(k_step_sell<T, P, VI, CI, Wc, WN, false, 0, kStepSellBlock, true, false, A>,
                                             SellDots{}, BSC());
                    return fold ? launch(k_step_sell<T, P, VI, CI, Wc, WN, true, 0, kStepSellBlock, false, false, A>, SellDots{}, BSC())
                                : launch(k_step_sell<T, P, VI, CI, Wc, WN, false, 0, kStepSellBlock, false, false, A>, SellDots{}, BSC());
                });
            });
        }
        if (a->node.nblk > 0) {
            const NodeCopy& S = a->node;
            const int tpw = node_tpw(S);
            auto go = [&](auto kern) {
                launch_timed(a->ctx, kern, dim3((S.ntiles + tpw - 1) / tpw), dim3(kBlock),
                             static_cast<const int32_t*>(S.tiles), static_cast<const int32_t*>(S.bptr),
                             static_cast<const char*>(S.recs), static_cast<const T*>(a->w[k & 1]),
                             static_cast<const T*>(a->inv()), static_cast<T*>(a->V), a->ld, k, diag,
                             static_cast<T*>(a->w[(k + 1) & 1]), gf, a->d.inner_row_exp, S.ntiles, S.nblk, tpw,
                             node_xcd(S));
                return (int)MPG_OK;
            };
            if (tpw > 1) return fold ? go(k_step_node<T, P, VI, true, true, A>) : go(k_step_node<T, P, VI, false, true, A>);
            return fold ? go(k_step_node<T, P, VI, true, false, A>) : go(k_step_node<T, P, VI, false, false, A>);
        }
        const int mode = csr_mode();
        auto kern = mode == 1   ? (fold ? k_step_spmv<T, P, VI, true, 1, A> : k_step_spmv<T, P, VI, false, 1, A>)
                    : mode == 2 ? (fold ? k_step_spmv<T, P, VI, true, 2, A> : k_step_spmv<T, P, VI, false, 2, A>)
                    : mode == 3 ? (fold ? k_step_spmv<T, P, VI, true, 3, A> : k_step_spmv<T, P, VI, false, 3, A>)
                    : mode == 4 ? (fold ? k_step_spmv<T, P, VI, true, 4, A> : k_step_spmv<T, P, VI, false, 4, A>)
                                : (fold ? k_step_spmv<T, P, VI, true, 0, A> : k_step_spmv<T, P, VI, false, 0, A>);
        launch_timed(a->ctx, kern, dim3(rb_grid(a)), dim3(kBlock),
            Acsr->blocks, Acsr->nblocks, Acsr->rowptr, Acsr->col, static_cast<const VI*>(a->d.val_inner), Acsr->nnz,
            static_cast<const T*>(a->w[k & 1]), static_cast<const T*>(a->inv()), static_cast<T*>(a->V), a->ld, k,
            diag, static_cast<T*>(a->w[(k + 1) & 1]), gf, a->d.inner_row_exp);
        return (int)MPG_OK;
    });
    if (st) return st;
    if (dots) {
        a->last_G = a->fd_ng;
        a->last_part = a->dpart;
    }
    MPG_LAUNCH_CHECK(a->ctx);
    return MPG_OK;
}


// row groups per panel of k_dots_panels: about one workgroup per CU in all
// (the same on every rank: uniform groups set Gd = kCombineGroups), so each
// column has <= kCombineGroups / 2 partials for k_cgs_update_wide
inline int wide_groups(const mpg_arnoldi* a, int ncols) {
    const int np = (ncols + kNC - 1) / kNC;
    return std::max(1, std::min(a->Gd, kCombineGroups / np));
}

// measurement: the armed stamp slots (mpg_arnoldi_stamp_next) for this launch when they hold all of its waves;
// disarmed either way
inline unsigned long long* take_stamp(mpg_arnoldi* a, int64_t waves) {
    unsigned long long* p = a->ctx->stamp_next;
    a->ctx->stamp_next = nullptr;
    return p && waves <= a->ctx->stamp_cap ? p : nullptr;
}

template <class A>
int dots_run(mpg_arnoldi_t a, int k, bool combine) {
    if (!a || k < 0 || k >= a->d.m) return MPG_ERR_ARG;
    const int ndots_all = a->d.orth == kOrthMGS ? 1 : k + 1;
    if (combine && ndots_all > kNC) return MPG_ERR_ARG;
    // an armed stamp belongs to this launch whatever its form (disarmed
    // here); only the one-panel k_dots_nc stores stamps
    unsigned long long* sp = take_stamp(a, (int64_t)a->Gd * (kCombineBlock / kWave));
    int st = dispatch_acc<A>(a->combo, [&](auto t, auto, auto, auto) {
        using T = decltype(t);
        if (combine) {
            k_panel_dots<T, kCombineBlock, true, A><<<a->Gd, kCombineBlock, 0, a->ctx->stream>>>(
                a->d.n, static_cast<const T*>(a->V), a->ld, 0, ndots_all, static_cast<const T*>(a->w[(k + 1) & 1]),
                a->partial, a->counters, a->sums);
            return (int)MPG_OK;
        }
        if (ndots_all <= kNC) {  // one panel: 1024-thread workgroups, one per CU -> Gd partials per column
            return with_nc<kNC>(ndots_all, [&](auto nc) {
                constexpr int NC = decltype(nc)::value;
                const T* Vp = static_cast<const T*>(a->V);
                const T* wp = static_cast<const T*>(a->w[(k + 1) & 1]);
                if (sp)
                    k_dots_nc<T, kCombineBlock, NC, true, A>
                        <<<a->Gd, kCombineBlock, 0, a->ctx->stream>>>(a->d.n, Vp, a->ld, wp, a->dpart, sp);
                else
                    k_dots_nc<T, kCombineBlock, NC, false, A>
                        <<<a->Gd, kCombineBlock, 0, a->ctx->stream>>>(a->d.n, Vp, a->ld, wp, a->dpart, nullptr);
                return (int)MPG_OK;
            });
        }
        if (ndots_all <= kWideMax) {  // every panel in one launch -> wide_groups(a, k) partials per column
            const int np = (ndots_all + kNC - 1) / kNC;
            return with_nc<kNC>(ndots_all - (np - 1) * kNC, [&](auto ncl) {
                k_dots_panels<T, kCombineBlock, decltype(ncl)::value, A>
                    <<<dim3(wide_groups(a, ndots_all), np), kCombineBlock, 0, a->ctx->stream>>>(
                        a->d.n, static_cast<const T*>(a->V), a->ld, static_cast<const T*>(a->w[(k + 1) & 1]),
                        a->dpart);
                return (int)MPG_OK;
            });
        }
        for (int c0 = 0; c0 < ndots_all; c0 += kNC) {
            const int nc = ndots_all - c0 < kNC ? ndots_all - c0 : kNC;
            k_panel_dots<T, kBlock, false, A><<<row_grid(a), kBlock, 0, a->ctx->stream>>>(
                a->d.n, static_cast<const T*>(a->V), a->ld, c0, nc, static_cast<const T*>(a->w[(k + 1) & 1]),
                a->partial, nullptr, nullptr);
        }
        return (int)MPG_OK;
    });
    const bool wide = !combine && ndots_all > kNC && ndots_all <= kWideMax;
    a->last_G = combine || ndots_all <= kNC ? a->Gd : wide ? wide_groups(a, ndots_all) : row_grid(a);
    a->last_part = !combine && ndots_all <= kWideMax ? a->dpart : a->partial;
    if (st) return st;
    MPG_LAUNCH_CHECK(a->ctx);
    return MPG_OK;
}


// The in-launch-sum CGS update issuing its first row group under the
// coefficient sums (k_cgs_update_nc<..., PF>, steps with k + 1 <= one batch
// of columns): on by default in the fp32 accumulation class, where the held
// batch fits its registers (BAND-10M, 8 interleaved bench runs each:
// 26.92k against 26.75k it/s, the update 11.98 against 12.27 us;
// profiles/r06_pf/), off in the fp64 class (round 4: no gain).
// MPG_CGS_PREFETCH=0 / 1 forces it.
template <class A>
inline bool cgs_prefetch() {
    const char* e = std::getenv("MPG_CGS_PREFETCH");
    if (e && (*e == '0' || *e == '1')) return *e == '1';
    return std::is_same_v<A, float>;
}

// no_next (CGSR at 32 < k + 1 <= kWideMax, one GPU): a pass that takes its
// coefficients from the preceding one-launch panel dots and emits no next
// dots (the caller launches k_dots_panels on the updated w instead)
template <class A>
int cgs_run(mpg_arnoldi_t a, int k, int pass, bool givens, bool from_partials, bool no_next) {
    if (!a || k < 0 || k >= a->d.m || pass < 0 || pass > 1 || k + 1 > 256) return MPG_ERR_ARG;
    const bool cgsr = a->d.orth == kOrthCGSR;
    const bool next_dots = cgsr && pass == 0 && !no_next;
    if (givens && (next_dots || a->d.m > kFoldMaxM || from_partials)) return MPG_ERR_ARG;
    if (no_next && (!cgsr || !from_partials || k + 1 <= kNC)) return MPG_ERR_ARG;
    // from_partials: the coefficients are summed from the preceding one-panel
    // dots' partials inside this launch (no reduce launch)
    if (from_partials && ((pass != 0 && !no_next) || k + 1 > kWideMax || a->last_part != a->dpart)) return MPG_ERR_ARG;
    if (from_partials && k + 1 > kNC && (next_dots || a->last_G > kWideMax)) return MPG_ERR_ARG;
    const double* src = from_partials ? a->dpart : a->sums;
    const int part_G = from_partials ? a->last_G : 0;  // Gd (k_dots_nc) or fd_ng (k_step_sell's dots)
    if (part_G > kCombineGroups) return MPG_ERR_ARG;
    // an armed stamp belongs to this launch whatever its form (disarmed here);
    // only the one-panel product form below stores stamps
    unsigned long long* sp = take_stamp(a, (int64_t)a->Gd * (kCombineBlock / kWave));
    int st = dispatch_acc<A>(a->combo, [&](auto t, auto, auto, auto) {
        using T = decltype(t);
        T* coef_out = pass == 0 ? static_cast<T*>(a->H) + (int64_t)k * (a->d.m + 1) : static_cast<T*>(a->corr());
        T* w = static_cast<T*>(a->w[(k + 1) & 1]);
        const GivensArgs<T> g = givens_args<T>(a, k);
        if (next_dots && k + 1 <= kNC && !from_partials) {
            // 256-thread workgroups (the NC fp64 dot accumulators need more
            // than the 128 VGPRs of a 1024-thread one) -> row_grid partials
            return with_nc<kNC>(k + 1, [&](auto nc) {
                k_cgs_update_nc<T, kBlock, decltype(nc)::value, false, true, false, false, A><<<row_grid(a), kBlock, 0, a->ctx->stream>>>(
                    a->d.n, static_cast<const T*>(a->V), a->ld, src, 0, coef_out, w, a->partial, nullptr);
                return (int)MPG_OK;
            });
        } else if (next_dots) {
            if (from_partials)
                k_cgs_update<T, true, false, kBlock, true, A><<<row_grid(a), kBlock, 0, a->ctx->stream>>>(
                    a->d.n, static_cast<const T*>(a->V), a->ld, k, src, coef_out, w, a->partial, nullptr, g, part_G);
            else
                k_cgs_update<T, true, false, kBlock, false, A><<<row_grid(a), kBlock, 0, a->ctx->stream>>>(
                    a->d.n, static_cast<const T*>(a->V), a->ld, k, src, coef_out, w, a->partial, nullptr, g, 0);
            for (int c0 = kNC; c0 < k + 1; c0 += kNC) {
                const int nc = k + 1 - c0 < kNC ? k + 1 - c0 : kNC;
                k_panel_dots<T, kBlock, false, A><<<row_grid(a), kBlock, 0, a->ctx->stream>>>(
                    a->d.n, static_cast<const T*>(a->V), a->ld, c0, nc, w, a->partial, nullptr, nullptr);
            }
        } else if (givens) {
            k_cgs_update<T, false, true, kBlock, false, A><<<row_grid(a), kBlock, 0, a->ctx->stream>>>(
                a->d.n, static_cast<const T*>(a->V), a->ld, k, src, coef_out, w, a->partial, a->counters + 32, g, 0);
        } else if (from_partials && k + 1 > kNC) {  // GMRES(100): sums from k_dots_panels' partials
            k_cgs_update_wide<T, kCombineBlock, A><<<a->Gd, kCombineBlock, 0, a->ctx->stream>>>(
                a->d.n, static_cast<const T*>(a->V), a->ld, k + 1, src, part_G, coef_out, w, a->partial);
        } else if (k + 1 <= kNC) {  // last pass: 1024-thread workgroups, one per CU -> Gd ||w||^2 partials
            // the wave stamps of the product form only (in-launch sums, no
            // prefetch): the one bench.py's phases time
            // (an armed stamp times the stamped product form, so a measured
            // launch never takes the prefetch variant)
            if (!from_partials) sp = nullptr;
            const bool pf = from_partials && !sp && cgs_prefetch<A>();
            return with_nc<kNC>(k + 1, [&](auto nc) {
                constexpr int NC = decltype(nc)::value;
                const T* Vp = static_cast<const T*>(a->V);
                // (the prefetch variant for one batch of columns only: wider
                // panels spilled with the prefetched batch held across the sums
                // in the fp64 class, and in the fp32 class the wider forms
                // (NC 9..28, no spills) aborted the process on the box
                // (round 6, profiles/r06_pf/); they are not built)
                if constexpr (NC <= kColBatch<T>) {
                    if (pf) {
                        k_cgs_update_nc<T, kCombineBlock, NC, true, false, true, false, A>
                            <<<a->Gd, kCombineBlock, 0, a->ctx->stream>>>(a->d.n, Vp, a->ld, src, part_G, coef_out,
                                                                           w, a->partial, nullptr);
                        return (int)MPG_OK;
                    }
                }
                if (from_partials && sp)
                    k_cgs_update_nc<T, kCombineBlock, NC, true, false, false, true, A>
                        <<<a->Gd, kCombineBlock, 0, a->ctx->stream>>>(a->d.n, Vp, a->ld, src, part_G, coef_out, w,
                                                                       a->partial, sp);
                else if (from_partials)
                    k_cgs_update_nc<T, kCombineBlock, NC, true, false, false, false, A><<<a->Gd, kCombineBlock, 0, a->ctx->stream>>>(
                        a->d.n, Vp, a->ld, src, part_G, coef_out, w, a->partial, nullptr);
                else
                    k_cgs_update_nc<T, kCombineBlock, NC, false, false, false, false, A><<<a->Gd, kCombineBlock, 0, a->ctx->stream>>>(
                        a->d.n, Vp, a->ld, src, 0, coef_out, w, a->partial, nullptr);
                return (int)MPG_OK;
            });
        } else {
            k_cgs_update<T, false, false, kCombineBlock, false, A><<<a->Gd, kCombineBlock, 0, a->ctx->stream>>>(
                a->d.n, static_cast<const T*>(a->V), a->ld, k, src, coef_out, w, a->partial, nullptr, g, 0);
        }
        return (int)MPG_OK;
    });
    a->last_G = next_dots || givens ? row_grid(a) : a->Gd;
    a->last_part = a->partial;
    if (st) return st;
    MPG_LAUNCH_CHECK(a->ctx);
    return MPG_OK;
}


template <class A>
int mgs_run(mpg_arnoldi_t a, int k, int j, bool from_partials) {
    if (!a || k < 0 || k >= a->d.m || j < 0 || j > k) return MPG_ERR_ARG;
    // from_partials: h_jk from the previous launch's partials; the update
    // writes into the other partial buffer (the previous one is still read)
    const double* src = from_partials ? a->last_part : a->sums;
    const int src_G = from_partials ? a->last_G : 0;
    double* dst = from_partials && a->last_part == a->partial ? a->dpart : a->partial;
    if (from_partials && src_G > kCombineGroups * 4) return MPG_ERR_ARG;
    int st = dispatch_acc<A>(a->combo, [&](auto t, auto, auto, auto) {
        using T = decltype(t);
        T* hjk = static_cast<T*>(a->H) + (int64_t)k * (a->d.m + 1) + j;
        k_mgs_update<T, kCombineBlock, A><<<a->Gd, kCombineBlock, 0, a->ctx->stream>>>(
            a->d.n, static_cast<const T*>(a->V), a->ld, j, k, src, src_G, hjk, static_cast<T*>(a->w[(k + 1) & 1]),
            dst);
        return (int)MPG_OK;
    });
    a->last_G = a->Gd;
    a->last_part = dst;
    if (st) return st;
    MPG_LAUNCH_CHECK(a->ctx);
    return MPG_OK;
}


template <class A>
int givens_run(mpg_arnoldi_t a, int k, bool from_partials) {
    if (!a || k < 0 || k >= a->d.m) return MPG_ERR_ARG;
    int st = dispatch_acc<A>(a->combo, [&](auto t, auto, auto, auto) {
        using T = decltype(t);
        k_givens<T, A><<<1, kBlock, 0, a->ctx->stream>>>(givens_args<T>(a, k), from_partials ? a->last_part : a->sums,
                                                      from_partials ? a->last_G : 0);
        return MPG_OK;
    });
    if (st) return st;
    MPG_LAUNCH_CHECK(a->ctx);
    return MPG_OK;
}


template <class A>
int update_run(mpg_arnoldi_t a, int k) {
    if (!a || k < 0 || k > a->d.m || k > 1024) return MPG_ERR_ARG;
    if (k == 0) return MPG_OK;
    int st = dispatch_acc<A>(a->combo, [&](auto t, auto x, auto, auto) {
        using T = decltype(t);
        using X = decltype(x);
        if (k <= kNC) {  // x is an aligned allocation: row groups of 4 are 16/32-B aligned
            return with_nc<kNC>(k, [&](auto nc) {
                k_update_x_nc<T, X, decltype(nc)::value, A><<<a->Gd, kCombineBlock, 0, a->ctx->stream>>>(
                    a->d.n, static_cast<const T*>(a->V), a->ld, static_cast<const T*>(a->s()),
                    static_cast<const T*>(a->H), a->d.m + 1, static_cast<X*>(a->d.x));
                return (int)MPG_OK;
            });
        } else if (k <= kWave) {
            k_update_x<T, X, true, A><<<row_grid(a), kBlock, 0, a->ctx->stream>>>(
                a->d.n, static_cast<const T*>(a->V), a->ld, k, static_cast<const T*>(a->s()),
                static_cast<const T*>(a->H), a->d.m + 1, static_cast<X*>(a->d.x));
        } else {
            const size_t packed = (size_t)k * (k + 1) / 2 * sizeof(T);
            if (k <= 2 * kWave && packed <= 65536)
                k_trsv_upper_lds<T, 2><<<1, kBlock, packed, a->ctx->stream>>>(
                    k, a->d.m + 1, static_cast<const T*>(a->H), static_cast<T*>(a->s()));
            else
                k_trsv_upper<T><<<1, kBlock, 0, a->ctx->stream>>>(k, a->d.m + 1, static_cast<const T*>(a->H),
                                                                  static_cast<T*>(a->s()));
            k_update_x<T, X, false, A><<<row_grid(a), kBlock, 0, a->ctx->stream>>>(
                a->d.n, static_cast<const T*>(a->V), a->ld, k, static_cast<const T*>(a->s()), nullptr, 0,
                static_cast<X*>(a->d.x));
        }
        return (int)MPG_OK;
    });
    if (st) return st;
    MPG_LAUNCH_CHECK(a->ctx);
    return MPG_OK;
}


}  // namespace

// The A = float launches, compiled in arnoldi_acc32.hip (fp32 Arnoldi only:
// an fp64 combination returns MPG_ERR_UNSUPPORTED there).
namespace mpg_acc32 {
int reduce(mpg_arnoldi* a, int ncols);
int spmv(mpg_arnoldi* a, int k, int fold, bool dots);
int dots(mpg_arnoldi* a, int k, bool combine);
int cgs(mpg_arnoldi* a, int k, int pass, bool givens, bool from_partials, bool no_next);
int mgs(mpg_arnoldi* a, int k, int j, bool from_partials);
int givens(mpg_arnoldi* a, int k, bool from_partials);
int update(mpg_arnoldi* a, int k);
}  // namespace mpg_acc32
