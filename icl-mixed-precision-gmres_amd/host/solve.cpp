// mpg_solve (include/mpgmres/solve.h): problem set-up, driver dispatch and
// report, following DoBaselineProblem / DoMixedPrecisionProblem / run_tests
// (gmres_perf_test.cpp:53-306) for Device = Hip.
#include "mpgmres/solve.h"

#include <chrono>
#include <cstdio>
#include <cstring>
#include <memory>
#include <stdexcept>
#include <string>

#include "IterUtil.hpp"
#include "Orthogonalization.hpp"
#include "fused_gmres.hpp"
#include "gmres.hpp"
#include "kernels.hpp"
#include "types_hip.hpp"

using namespace Orthogonalization;

namespace mpg {

namespace {

using clk = std::chrono::steady_clock;

double seconds_since(clk::time_point t0) {
    return std::chrono::duration<double>(clk::now() - t0).count();
}

// gmres_perf_test.cpp:185-196
template <class T>
std::unique_ptr<Convergence<T, Hip>> make_convergence(const mpg_solve_args& a) {
    const size_t m = (size_t)a.rlen;
    if (a.rtol == 0) return std::make_unique<Convergence<T, Hip>>(a.tol, m, (size_t)a.max_restarts);
    if (a.repeat_iter)
        return std::make_unique<RepeatIteration_Convergence<T, Hip>>(a.tol, a.rtol, m, (size_t)a.max_restarts);
    if (a.orthloss)
        return std::make_unique<LostOrthogonality_Convergence<T, Hip>>(a.tol, a.rtol, m, (size_t)a.max_restarts);
    return std::make_unique<RelPrecRes_Convergence<T, Hip>>(a.tol, a.rtol, m, (size_t)a.max_restarts);
}

// gmres_perf_test.cpp:69-89, 139-159 (ILU from the fp64 A; Jacobi from A
// converted to the preconditioner precision)
template <class P>
std::unique_ptr<LinearOperator<P, Hip>> make_preconditioner(int prec, const SparseMatrix<double, Hip>& A,
                                                            int jacobi_steps) {
    switch (prec) {
        case MPG_PREC_IDENTITY: return std::make_unique<Identity<P, Hip>>();
        case MPG_PREC_JACOBI: return std::make_unique<Jacobi<P, Hip>>(A);
        case MPG_PREC_ILU: return std::make_unique<ILU<P, Hip>>(ilu0<P, Hip>(A));
        case MPG_PREC_ILU_JACOBI: return std::make_unique<ILU_Jacobi<P, Hip>>(ilu0<P, Hip>(A), jacobi_steps);
        default: throw std::invalid_argument("Unknown prec type");
    }
}

template <class T>
void record(const Recorder<T, Hip>& rec, const Convergence<T, Hip>& conv, mpg_solve_result* r) {
    r->total_iters = (int64_t)conv.total_iterations();
    r->n_cycles = (int64_t)rec.cycles.size();
    for (size_t c = 0; c < rec.cycles.size() && (int64_t)c < r->cycle_cap; ++c) {
        if (r->cyc_r_norm) r->cyc_r_norm[c] = rec.cycles[c].r_norm;
        if (r->cyc_normalization) r->cyc_normalization[c] = rec.cycles[c].normalization;
        if (r->cyc_beta) r->cyc_beta[c] = rec.cycles[c].beta;
    }
    if (!rec.cycles.empty()) r->minvb_norm = rec.cycles[0].minvb_norm;
    r->n_steps = (int64_t)rec.step_residual.size();
    for (size_t s = 0; s < rec.step_residual.size() && (int64_t)s < r->step_cap; ++s) {
        if (r->step_res) r->step_res[s] = rec.step_residual[s];
        if (r->step_cycle) r->step_cycle[s] = rec.step_cycle[s];
    }
    r->nonfinite_steps = rec.breakdown.steps;
    r->nonfinite_cycles = rec.breakdown.cycles;
    r->first_nonfinite_step = rec.breakdown.first_step;
    // status: converged iff the last check_initial said so (or a check did)
    r->restarts = rec.cycles.empty() ? 0 : (int64_t)rec.cycles.size() - 1;
}

template <class T>
void finish_status(Convergence<T, Hip>& conv, mpg_solve_result* r) {
    r->status = conv.total_restarts > conv.max_restarts ? MPG_RESULT_ABORTED : MPG_RESULT_CONVERGED;
}

// resNorm / errNorm report with the original fp64 A (gmres_perf_test.cpp:104-115, 169-178)
void report(const SparseMatrix<double, Hip>& A, Vect<double, Hip> b_used, Vect<double, Hip> x,
            const mpg_solve_args& a, const Vect<double, Hip>& x_true, mpg_solve_result* r, double prec_s,
            double gmres_s) {
    const size_t n = x.n();
    if (r->x_out) Hip::to_host(r->x_out, x.data(), n * sizeof(double));
    Vect<double, Hip> res(n);
    copy(b_used, res);
    spmv(-1.0, A, x, 1.0, res);
    r->res_norm = nrm2(res);
    if (a.x_true) {
        axpy(-1.0, x_true, x);
        r->err_norm = nrm2(x);
    }
    r->setup_seconds = prec_s;
    r->gmres_seconds = gmres_s;
    mpg::out() << "  ilu took " << (float)prec_s << "s; gmres took " << (float)gmres_s << "s" << std::endl;
    mpg::out() << "  resNorm = " << r->res_norm << "; errNorm = " << r->err_norm << std::endl;
}

template <class Orth, class Type, class PrecType>
void do_baseline(const mpg_solve_args& a, const SparseMatrix<double, Hip>& A, Vect<double, Hip> b,
                 Vect<double, Hip> x_true, mpg_solve_result* r) {
    mpg::out() << "Doing Baseline test" << std::endl;
    const size_t n = (size_t)A.nrows();
    auto t0 = clk::now();
    // gmres_perf_test.cpp:66 — the matrix handed to the solver is always the
    // fp32-rounded copy, widened back for Type = double.
    const SparseMatrix<float, Hip> A_f32(A);
    const SparseMatrix<Type, Hip> A_type(A_f32);
    auto M = make_preconditioner<PrecType>(a.prec, A, a.jacobi_steps);
    Hip::fence();
    const double prec_s = seconds_since(t0);

    Vect<Type, Hip> x_type(n);
    Vect<Type, Hip> b_type(n);
    copy(b, b_type);
    auto conv = make_convergence<Type>(a);
    Recorder<Type, Hip> rec(*conv);
    rec.breakdown.stop = a.stop_on_breakdown != 0;

    Hip::fence();
    auto t1 = clk::now();
    gmres_baseline<Orth, Hip, Type, PrecType>(rec, A_type, M.get(), b_type, x_type);
    Hip::fence();
    const double gmres_s = seconds_since(t1);

    record(rec, *conv, r);
    finish_status(*conv, r);
    Vect<double, Hip> x(n), b_used(n);
    copy(x_type, x);
    copy(b_type, b_used);
    report(A, b_used, x, a, x_true, r, prec_s, gmres_s);
}

template <class Orth>
void do_mixed(const mpg_solve_args& a, const SparseMatrix<double, Hip>& A, Vect<double, Hip> b,
              Vect<double, Hip> x_true, mpg_solve_result* r) {
    mpg::out() << "Doing Mixed Precision test" << std::endl;
    const size_t n = (size_t)A.nrows();
    Vect<double, Hip> x(n);
    auto t0 = clk::now();
    const SparseMatrix<float, Hip> A_single(A);
    auto M = make_preconditioner<float>(a.prec, A, a.jacobi_steps);
    Hip::fence();
    const double prec_s = seconds_since(t0);

    auto conv = make_convergence<float>(a);
    Recorder<float, Hip> rec(*conv);
    rec.breakdown.stop = a.stop_on_breakdown != 0;
    Hip::fence();
    auto t1 = clk::now();
    gmres_singleUpdate<Orth, Hip>(rec, A, A_single, M.get(), b, x);
    Hip::fence();
    const double gmres_s = seconds_since(t1);

    record(rec, *conv, r);
    finish_status(*conv, r);
    report(A, b, x, a, x_true, r, prec_s, gmres_s);
}

template <class KD, class KS>
void dispatch_mode(const mpg_solve_args& a, const SparseMatrix<double, Hip>& A, Vect<double, Hip> b,
                   Vect<double, Hip> xt, mpg_solve_result* r) {
    switch (a.mode) {
        case MPG_MODE_MIXED: do_mixed<GS<float, KS, Hip>>(a, A, b, xt, r); break;
        case MPG_MODE_BASELINE: do_baseline<GS<double, KD, Hip>, double, double>(a, A, b, xt, r); break;
        case MPG_MODE_SINGLE_PREC: do_baseline<GS<double, KD, Hip>, double, float>(a, A, b, xt, r); break;
        case MPG_MODE_SINGLE: do_baseline<GS<float, KS, Hip>, float, float>(a, A, b, xt, r); break;
        default: throw std::invalid_argument("mode not supported by the surface engine");
    }
}

}  // namespace

int solve_surface(const mpg_solve_args& a, mpg_solve_result* r) {
    SparseMatrix<double, Hip> A(a.n, a.n, a.rowptr, a.col, a.val);
    const size_t n = (size_t)a.n;
    Vect<double, Hip> b(n), xt(n);
    Hip::to_device(b.data(), a.b, n * sizeof(double));
    if (a.x_true) Hip::to_device(xt.data(), a.x_true, n * sizeof(double));
    switch (a.orth) {
        case MPG_ORTH_CGS: dispatch_mode<CGS_Kernel<double, Hip>, CGS_Kernel<float, Hip>>(a, A, b, xt, r); break;
        case MPG_ORTH_MGS: dispatch_mode<MGS_Kernel<double, Hip>, MGS_Kernel<float, Hip>>(a, A, b, xt, r); break;
        case MPG_ORTH_CGSR:
            dispatch_mode<CGSR_Kernel<double, Hip, 2>, CGSR_Kernel<float, Hip, 2>>(a, A, b, xt, r);
            break;
        default: throw std::invalid_argument("Unknown Orthogonalization");
    }
    return 0;
}

}  // namespace mpg

extern "C" int mpg_solve(const mpg_solve_args* args, mpg_solve_result* result) {
    if (!args || !result) return MPG_ERR_ARG;
    result->status = MPG_RESULT_ERROR;
    result->message[0] = '\0';
    result->n_cycles = result->n_steps = 0;
    result->res_norm = result->err_norm = 0;
    result->nonfinite_steps = result->nonfinite_cycles = 0;
    result->first_nonfinite_step = -1;
    try {
        if (args->n <= 0 || args->rlen <= 0 || !args->rowptr || !args->col || !args->val || !args->b)
            throw std::invalid_argument("invalid solve arguments (n, rlen, CSR arrays and b are required)");
        if (args->accum != 0 && args->accum != 1) throw std::invalid_argument("accum: 0 (f64) or 1 (f32)");
        if (args->accum && args->engine != MPG_ENGINE_FUSED && args->mode != MPG_MODE_BASELINE &&
            args->mode != MPG_MODE_SINGLE_PREC)
            throw mpg::StatusError(MPG_ERR_UNSUPPORTED,
                                   "mpgmres: accum f32 runs on the fused engine only (the operator surface's "
                                   "kernels accumulate in fp64)");
        mpg::set_quiet(!args->verbose);
        mpg_ctx_t ctx = nullptr;
        mpg::check(mpg_ctx_create(args->device, &ctx), "mpg_ctx_create");
        std::unique_ptr<mpg_ctx, int (*)(mpg_ctx_t)> guard(ctx, mpg_ctx_destroy);
        int st;
        {
            mpg::ScopedContext scope(ctx);
            st = args->engine == MPG_ENGINE_FUSED ? mpg::solve_fused(*args, result)
                                                  : mpg::solve_surface(*args, result);
            mpg::check(mpg_ctx_sync(ctx), "final sync", ctx);
        }
        return st;
    } catch (const mpg::StatusError& e) {
        result->status = MPG_RESULT_ERROR;
        std::snprintf(result->message, sizeof result->message, "%s", e.what());
        return e.status;
    } catch (const mpg::BreakdownError& e) {
        result->status = MPG_RESULT_ERROR;
        std::snprintf(result->message, sizeof result->message, "%s", e.what());
        return MPG_ERR_BREAKDOWN;
    } catch (const std::exception& e) {
        result->status = MPG_RESULT_ERROR;
        std::snprintf(result->message, sizeof result->message, "%s", e.what());
        return MPG_ERR_ARG;
    }
}
