// Derived from iamsonderr/icl-mixed-precision-gmres, Copyright (c) 2019-2021,
// University of Tennessee (BSD-3-Clause; the license text is in NOTICE).
// mpg_condest (include/mpgmres/condest.h): the reference's condition-number
// estimator (condest.cpp:36-179) over the kernels.hpp operator surface, for
// Device = Hip. The transposed products use SparseMatrix::set_transpose
// (an explicit A^T CSR on the device, types_hip.hpp).
#include "mpgmres/condest.h"

#include <chrono>
#include <cmath>
#include <cstdio>
#include <iostream>
#include <limits>
#include <memory>
#include <stdexcept>
#include <vector>

#include "kernels.hpp"
#include "mpgmres/problems.h"
#include "types_hip.hpp"

namespace mpg {

namespace {

// condest.cpp:28-31
int klein_lu_bound(double eps, double delta, int n) {
    const double log_2n = std::log(2 * n);
    return int(std::ceil((log_2n * log_2n - std::log(eps * delta * delta)) / eps));
}

// condest.cpp:22-26: rand_vect(n, seed) (float draws, as the GMRES driver)
// copied into a device vector
template <class Device>
void rand_fill(Vect<double, Device> x, uint32_t seed) {
    std::vector<double> h(x.n());
    mpg_rand_vect((int64_t)x.n(), seed, h.data());
    Device::to_device(x.data(), h.data(), h.size() * sizeof(double));
}

// condest.cpp:153-164: x := A x / ||A x||, iter_count times; returns the last norm
template <class Device>
double power_iteration(const SparseMatrix<double, Device>& A, Vect<double, Device> x, int iter_count) {
    Vect<double, Device> y(x.n());
    double lambda = 0;
    for (int i = 0; i < iter_count; i++) {
        spmv(1.0, A, x, 0.0, y);
        lambda = nrm2(y);
        scal(1 / lambda, y, x);
    }
    return lambda;
}

// condest.cpp:34-150
template <class Device>
void condest(SparseMatrix<double, Device> A, int rand_seed, int64_t max_iters, bool verbose, mpg_condest_result* r) {
    const int n = A.nrows();

    const double eps = std::numeric_limits<double>::epsilon();
    double c1 = 8 * eps;
    const double erfinv_c2 = 8.862271574665521045654E-4;
    const double c3 = 1 / (64 * eps);
    const double c4 = std::sqrt(eps);
    const double c1_prime = 4 * eps;
    const int power_iter_tol = klein_lu_bound(0.1, 1e-12, n);

    SparseMatrix<double, Device> A_trans = A;
    A_trans.set_transpose(true);

    Vect<double, Device> v_max(n);
    rand_fill(v_max, (uint32_t)(rand_seed + 5));
    const double sigma_max = power_iteration(A, v_max, power_iter_tol);

    Vect<double, Device> v_min(n);
    copy(v_max, v_min);
    double sigma_min = sigma_max;

    Vect<double, Device> x_exact(n);
    rand_fill(x_exact, (uint32_t)rand_seed);
    const double x_rand_norm = nrm2(x_exact);
    scal(1 / x_rand_norm, x_exact);

    Vect<double, Device> b(n);
    spmv(1.0, A, x_exact, 0.0, b);
    const double b_norm = nrm2(b);
    double beta = b_norm;

    Vect<double, Device> u(n);
    scal(1 / beta, b, u);

    Vect<double, Device> v(n);
    spmv(1.0, A_trans, u, 0.0, v);
    double alpha = nrm2(v);
    scal(1 / alpha, v);

    Vect<double, Device> w(n);
    copy(v, w);
    Vect<double, Device> x(n);
    fill(0.0, x);
    Vect<double, Device> d(n);
    Vect<double, Device> Ad(n);
    double d_norm, Ad_norm;

    double phi_bar = beta, rho_bar = alpha;
    double phi, rho, c, s, theta;

    const double tau = std::sqrt(2) * erfinv_c2 / x_rand_norm;
    int64_t T = max_iters;

    if (verbose) std::cout << "sigma_max = " << sigma_max << std::endl;

    r->stop_reason = 0;
    r->finish_t = 0;
    int64_t t;
    for (t = 1; t <= T; t++) {
        spmv(1.0, A, v, -alpha, u);
        beta = nrm2(u);
        scal(1 / beta, u);

        spmv(1.0, A_trans, u, -beta, v);
        alpha = nrm2(v);
        scal(1 / alpha, v);

        rho = std::sqrt(rho_bar * rho_bar + beta * beta);
        c = rho_bar / rho;
        s = beta / rho;
        theta = s * alpha;
        rho_bar = -c * alpha;
        phi = c * phi_bar;
        phi_bar = s * phi_bar;

        axpy(phi / rho, w, x);
        scal(-theta / rho, w);
        axpy(1.0, v, w);

        copy(x_exact, d);
        axpy(-1.0, x, d);
        d_norm = nrm2(d);
        if (d_norm == 0) {
            r->stop_reason = 1;
            break;
        }

        spmv(1.0, A, d, 0.0, Ad);
        Ad_norm = nrm2(Ad);
        if (Ad_norm < sigma_min * d_norm) {
            sigma_min = Ad_norm / d_norm;
            copy(d, v_min);
        }

        if (std::isnan(Ad_norm)) {
            r->stop_reason = 2;
            break;
        }

        if (sigma_min / sigma_max <= c4) c1 = c1_prime;

        if (T == max_iters) {
            const double x_norm = nrm2(x);
            if (Ad_norm / (sigma_max * x_norm + b_norm) <= c1 || d_norm <= tau || sigma_max / sigma_min >= c3) {
                T = int64_t(std::ceil(t * 1.25));
                r->finish_t = t;
                if (verbose) std::cout << "t = " << t << ": finishing" << std::endl;
            }
            if (verbose && t % 10000 == 0) std::cout << "t = " << t << ": sigma_min = " << sigma_min << std::endl;
        }
    }

    if (verbose) {
        std::cout << t << " iterations total" << std::endl;
        std::cout << "Computed cond(A) = " << sigma_max / sigma_min << " = " << sigma_max << "/" << sigma_min
                  << std::endl;
    }
    r->sigma_max = sigma_max;
    r->sigma_min = sigma_min;
    r->cond = sigma_max / sigma_min;
    r->power_iters = power_iter_tol;
    r->iters = t;
}

}  // namespace

}  // namespace mpg

extern "C" int mpg_condest(const mpg_condest_args* a, mpg_condest_result* r) {
    if (!a || !r) return MPG_ERR_ARG;
    *r = mpg_condest_result{};
    r->status = MPG_ERR_ARG;
    try {
        if (a->n <= 0 || !a->rowptr || !a->col || !a->val || a->max_iters < 0)
            throw std::invalid_argument("invalid condest arguments (n, CSR arrays, max_iters >= 0)");
        if (a->rowptr[a->n] != a->nnz) throw std::invalid_argument("rowptr[n] != nnz");
        mpg_ctx_t ctx = nullptr;
        mpg::check(mpg_ctx_create(a->device, &ctx), "mpg_ctx_create");
        std::unique_ptr<mpg_ctx, int (*)(mpg_ctx_t)> guard(ctx, mpg_ctx_destroy);
        {
            mpg::ScopedContext scope(ctx);
            SparseMatrix<double, Hip> A(a->n, a->n, a->rowptr, a->col, a->val);
            mpg::check(mpg_ctx_sync(ctx), "upload", ctx);
            const auto t0 = std::chrono::steady_clock::now();
            mpg::condest<Hip>(A, a->rand_seed, a->max_iters, a->verbose != 0, r);
            Hip::fence();  // issues any queued scalar operators first
            r->seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        }
        r->status = 0;
        return 0;
    } catch (const std::exception& e) {
        r->status = MPG_ERR_ARG;
        std::snprintf(r->message, sizeof r->message, "%s", e.what());
        return MPG_ERR_ARG;
    }
}
