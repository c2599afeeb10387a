// Derived from iamsonderr/icl-mixed-precision-gmres, Copyright (c) 2019-2021,
// University of Tennessee (BSD-3-Clause; the license text is in NOTICE).
// ORACLE — test infrastructure only. Never linked into the product; only
// tests/ load it.
//
// CPU restatement of the reference's condition-number estimator
// (condest.cpp:11-179): rand_vect with float draws (condest.cpp:11-26),
// klein_lu_bound (28-31), power_iteration (153-164) and the LSQR-based
// sigma_min search with its stopping rule (34-150). The reference runs it
// only through cuSPARSE/cuBLAS (condest.cpp:217-223); here the same
// operations call the MKL runtime (mkl_sparse_d_mv with
// SPARSE_OPERATION_TRANSPOSE for A^T u, cblas_dnrm2/daxpy, copy + dscal for
// the 3-argument scal, kernels_mkl.cpp:73-211) or fp64 loops.
// Parity: unpinned by reference fixtures (the reference ships none for it);
// cross-checked by tests/test_condest.py against numpy/scipy singular values.
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <iostream>
#include <limits>
#include <random>
#include <stdexcept>
#include <vector>

#include "cpu_blas.hpp"
#include "mpgmres/condest.h"

namespace oracle {
namespace {

constexpr int kSparseOpTrans = 11;  // SPARSE_OPERATION_TRANSPOSE

struct Mat {
    int n = 0;
    std::vector<int> rp, ci;
    std::vector<double> v;
    void* h = nullptr;
    ~Mat() {
        if (h && mkl().loaded) mkl().destroy(h);
    }
};

// y = alpha op(A) x + beta y
void mv(bool trans, double alpha, const Mat& A, const double* x, double beta, double* y) {
    if (mkl().loaded) {
        if (mkl().d_mv(trans ? kSparseOpTrans : kSparseOpNoTrans, alpha, A.h, SparseDescr{kSparseTypeGeneral, 0, 0},
                       x, beta, y))
            throw std::runtime_error("mkl_sparse_d_mv failed");
        return;
    }
    const int n = A.n;
    if (!trans) {
        for (int i = 0; i < n; ++i) {
            double s = 0;
            for (int k = A.rp[i]; k < A.rp[i + 1]; ++k) s += A.v[k] * x[A.ci[k]];
            y[i] = beta == 0 ? alpha * s : alpha * s + beta * y[i];
        }
        return;
    }
    std::vector<double> t((size_t)n, 0.0);
    for (int i = 0; i < n; ++i)
        for (int k = A.rp[i]; k < A.rp[i + 1]; ++k) t[A.ci[k]] += A.v[k] * x[i];
    for (int j = 0; j < n; ++j) y[j] = beta == 0 ? alpha * t[j] : alpha * t[j] + beta * y[j];
}

using Vec = std::vector<double>;
double norm(const Vec& x) { return nrm2((int)x.size(), x.data()); }
void scal2(double a, Vec& x) { scal((int)x.size(), a, x.data()); }
void scal3(double a, const Vec& x, Vec& y) {  // copy, then ?scal (kernels_mkl.cpp:165-191)
    y = x;
    scal((int)y.size(), a, y.data());
}
void axpy(double a, const Vec& x, Vec& y) { oracle::axpy((int)x.size(), a, x.data(), y.data()); }

Vec rand_vect(int n, unsigned seed) {
    std::mt19937 engine(seed);
    std::uniform_real_distribution<float> dist;
    Vec x((size_t)n);
    for (int i = 0; i < n; ++i) x[(size_t)i] = dist(engine);
    return x;
}

int klein_lu_bound(double eps, double delta, int n) {
    const double l = std::log(2 * n);
    return int(std::ceil((l * l - std::log(eps * delta * delta)) / eps));
}

double power_iteration(const Mat& A, Vec& x, int iters) {
    Vec y(x.size());
    double lambda = 0;
    for (int i = 0; i < iters; ++i) {
        mv(false, 1.0, A, x.data(), 0.0, y.data());
        lambda = norm(y);
        scal3(1 / lambda, y, x);
    }
    return lambda;
}

void condest(const Mat& A, int seed, int64_t max_iters, bool verbose, mpg_condest_result* r) {
    const int n = A.n;
    const double eps = std::numeric_limits<double>::epsilon();
    double c1 = 8 * eps;
    const double erfinv_c2 = 8.862271574665521045654E-4;
    const double c3 = 1 / (64 * eps), c4 = std::sqrt(eps), c1_prime = 4 * eps;
    const int piters = klein_lu_bound(0.1, 1e-12, n);

    Vec v_max = rand_vect(n, (unsigned)(seed + 5));
    const double sigma_max = power_iteration(A, v_max, piters);
    double sigma_min = sigma_max;

    Vec x_exact = rand_vect(n, (unsigned)seed);
    const double x_rand_norm = norm(x_exact);
    scal2(1 / x_rand_norm, x_exact);
    Vec b((size_t)n);
    mv(false, 1.0, A, x_exact.data(), 0.0, b.data());
    const double b_norm = norm(b);
    double beta = b_norm;
    Vec u;
    scal3(1 / beta, b, u);
    Vec v((size_t)n);
    mv(true, 1.0, A, u.data(), 0.0, v.data());
    double alpha = norm(v);
    scal2(1 / alpha, v);
    Vec w = v, x((size_t)n, 0.0), d((size_t)n), Ad((size_t)n);
    double phi_bar = beta, rho_bar = alpha;
    const double tau = std::sqrt(2) * erfinv_c2 / x_rand_norm;
    int64_t T = max_iters;
    if (verbose) std::cout << "sigma_max = " << sigma_max << std::endl;
    r->stop_reason = 0;
    r->finish_t = 0;
    int64_t t;
    for (t = 1; t <= T; ++t) {
        mv(false, 1.0, A, v.data(), -alpha, u.data());
        beta = norm(u);
        scal2(1 / beta, u);
        mv(true, 1.0, A, u.data(), -beta, v.data());
        alpha = norm(v);
        scal2(1 / alpha, v);

        const double rho = std::sqrt(rho_bar * rho_bar + beta * beta);
        const double c = rho_bar / rho, s = beta / rho, theta = s * alpha;
        rho_bar = -c * alpha;
        const double phi = c * phi_bar;
        phi_bar = s * phi_bar;
        axpy(phi / rho, w, x);
        scal2(-theta / rho, w);
        axpy(1.0, v, w);

        d = x_exact;
        axpy(-1.0, x, d);
        const double d_norm = norm(d);
        if (d_norm == 0) {
            r->stop_reason = 1;
            break;
        }
        mv(false, 1.0, A, d.data(), 0.0, Ad.data());
        const double Ad_norm = norm(Ad);
        if (Ad_norm < sigma_min * d_norm) sigma_min = Ad_norm / d_norm;
        if (std::isnan(Ad_norm)) {
            r->stop_reason = 2;
            break;
        }
        if (sigma_min / sigma_max <= c4) c1 = c1_prime;
        if (T == max_iters) {
            const double x_norm = norm(x);
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
    r->power_iters = piters;
    r->iters = t;
}

}  // namespace
}  // namespace oracle

extern "C" int oracle_condest(const mpg_condest_args* a, mpg_condest_result* r) {
    if (!a || !r) return -1;
    *r = mpg_condest_result{};
    try {
        if (a->n <= 0 || !a->rowptr || !a->col || !a->val) throw std::invalid_argument("invalid condest arguments");
        if (a->threads > 0) oracle::set_threads(a->threads);
        oracle::Mat A;
        A.n = a->n;
        A.rp.assign(a->rowptr, a->rowptr + a->n + 1);
        A.ci.assign(a->col, a->col + a->nnz);
        A.v.assign(a->val, a->val + a->nnz);
        if (oracle::mkl().loaded &&
            oracle::mkl().d_create_csr(&A.h, oracle::kSparseIndexZero, A.n, A.n, A.rp.data(), A.rp.data() + 1,
                                       A.ci.data(), A.v.data()))
            throw std::runtime_error("mkl_sparse_d_create_csr failed");
        const auto t0 = std::chrono::steady_clock::now();
        oracle::condest(A, a->rand_seed, a->max_iters, a->verbose != 0, r);
        r->seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        return 0;
    } catch (const std::exception& e) {
        r->status = -1;
        std::snprintf(r->message, sizeof r->message, "%s", e.what());
        return -1;
    }
}
