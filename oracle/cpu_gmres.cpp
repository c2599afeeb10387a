// Derived from iamsonderr/icl-mixed-precision-gmres, Copyright (c) 2019-2021,
// University of Tennessee (BSD-3-Clause; the license text is in NOTICE).
// ORACLE — test infrastructure only. Never linked into the product; only
// tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg load it.
//
// CPU restatement of the reference's restarted mixed-precision GMRES on its
// MKL backend, written independently of the product's C++ driver:
//   rand_vect / problem set-up / report   gmres_perf_test.cpp:39-182
//   gmres_baseline                        gmres.cpp:24-133
//   gmres_singleUpdate                    gmres.cpp:135-245
//   solution_update (both forms)          gmres.cpp:276-303
//   GS first_vector / add_vector / update Orthogonalization.hpp:36-73
//   CGS / MGS / CGSR(2) kernels           Orthogonalization.hpp:76-136
//   Convergence + adaptive strategies     IterUtil.hpp:17-227
//   Jacobi preconditioner                 types.hpp:381-448
//   MKL kernels (dot, nrm2, axpy, scal via copy+scal, rotg + b:=0, per-pair
//   rot, gemv, trsv, mkl_sparse_?_mv)    kernels_mkl.cpp:17-352
// Parity status: the reference cannot be built here (Kokkos absent) and
// holds no tests or golden vectors for this path, so this oracle is pinned
// only to the third-party arithmetic it calls (the MKL 2021.4 runtime in the
// image) and cross-checked against the independent NumPy restatement in
// oracle/gmres_np.py — "parity unpinned" by reference fixtures.
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <limits>
#include <memory>
#include <stdexcept>
#include <string>
#include <type_traits>
#include <vector>

#include "cpu_blas.hpp"
#include "mpgmres/solve.h"

namespace oracle {
namespace {

bool g_verbose = false;
#define OUT(...)                                  \
    do {                                          \
        if (g_verbose) std::printf(__VA_ARGS__);  \
    } while (0)

// ---- CSR with an MKL handle (types_mkl.hpp:17-107) ----
template <class T>
struct Csr {
    int n = 0;
    std::vector<int> rp, ci;
    std::vector<T> v;
    void* h = nullptr;
    Csr() = default;
    Csr(const Csr&) = delete;
    ~Csr() {
        if (h && mkl().loaded) mkl().destroy(h);
    }
    void make_handle();
};
template <>
void Csr<double>::make_handle() {
    if (mkl().loaded && mkl().d_create_csr(&h, kSparseIndexZero, n, n, rp.data(), rp.data() + 1, ci.data(), v.data()))
        throw std::runtime_error("mkl_sparse_d_create_csr failed");
}
template <>
void Csr<float>::make_handle() {
    if (mkl().loaded && mkl().s_create_csr(&h, kSparseIndexZero, n, n, rp.data(), rp.data() + 1, ci.data(), v.data()))
        throw std::runtime_error("mkl_sparse_s_create_csr failed");
}

template <class T, class S>
std::unique_ptr<Csr<T>> make_csr(int n, const int* rp, const int* ci, const S* v) {
    auto A = std::make_unique<Csr<T>>();
    A->n = n;
    A->rp.assign(rp, rp + n + 1);
    A->ci.assign(ci, ci + rp[n]);
    A->v.resize((size_t)rp[n]);
    for (size_t k = 0; k < A->v.size(); ++k) A->v[k] = (T)v[k];
    A->make_handle();
    return A;
}

// y = alpha*A x + beta*y
void spmv(double alpha, const Csr<double>& A, const double* x, double beta, double* y) {
    if (mkl().loaded) {
        if (mkl().d_mv(kSparseOpNoTrans, alpha, A.h, SparseDescr{kSparseTypeGeneral, 0, 0}, x, beta, y))
            throw std::runtime_error("mkl_sparse_d_mv failed");
        return;
    }
#pragma omp parallel for schedule(static)
    for (int i = 0; i < A.n; ++i) {
        double s = 0;
        for (int k = A.rp[i]; k < A.rp[i + 1]; ++k) s += A.v[k] * x[A.ci[k]];
        y[i] = beta == 0 ? alpha * s : alpha * s + beta * y[i];
    }
}
void spmv(float alpha, const Csr<float>& A, const float* x, float beta, float* y) {
    if (mkl().loaded) {
        if (mkl().s_mv(kSparseOpNoTrans, alpha, A.h, SparseDescr{kSparseTypeGeneral, 0, 0}, x, beta, y))
            throw std::runtime_error("mkl_sparse_s_mv failed");
        return;
    }
    if (loop_sum_mode() != kSumF64) {  // fp32 row sums in CSR order, products rounded to fp32
#pragma omp parallel for schedule(static)
        for (int i = 0; i < A.n; ++i) {
            float t = 0.f;
            for (int k = A.rp[i]; k < A.rp[i + 1]; ++k) t += A.v[k] * x[A.ci[k]];
            y[i] = beta == 0 ? alpha * t : alpha * t + beta * y[i];
        }
        return;
    }
#pragma omp parallel for schedule(static)
    for (int i = 0; i < A.n; ++i) {
        double s = 0;
        for (int k = A.rp[i]; k < A.rp[i + 1]; ++k) s += (double)A.v[k] * x[A.ci[k]];
        const float t = (float)s;
        y[i] = beta == 0 ? alpha * t : alpha * t + beta * y[i];
    }
}

template <class S, class D>
void cast(const std::vector<S>& x, std::vector<D>& y) {
    y.resize(x.size());
    for (size_t i = 0; i < x.size(); ++i) y[i] = (D)x[i];
}

// ---- preconditioners (types.hpp:251-448, kernels.hpp:168-248) ----

// ILU(0) of the fp64 matrix (ilu0_impl, kernels_mkl.cpp:416-500), with the
// one change that makes it an ILU: the reference allocates diag_inds (448)
// but never fills it, so every pivot lookup reads entry 0; here
// diag_inds[i] is the position of a_ii. Everything else is as written there:
// rows 1..n-1 in order (row 0 is neither eliminated nor boosted), the
// sorted merge of row i with the upper part of row k, pivots pushed away
// from zero to +-alpha (sign kept), alpha = max_i sum_j |a_ij| * eps(T).
// (cuSPARSE csrilu02's numeric boost, kernels_cuda.cpp:745-746, replaces a
// small pivot by +alpha in every row; the two agree whenever no pivot is
// smaller than alpha.) Returns the factors in fp64; the caller rounds to T.
template <class T>
void ilu0(int n, const int* rp, const int* ci, const double* v64, std::vector<double>& lu, std::vector<int>& di) {
    double alpha = 0;
    for (int i = 0; i < n; ++i) {
        double sum = 0;
        for (int k = rp[i]; k < rp[i + 1]; ++k) sum += std::fabs(v64[k]);
        if (alpha < sum) alpha = sum;
    }
    alpha *= std::numeric_limits<T>::epsilon();
    lu.assign(v64, v64 + rp[n]);
    di.assign((size_t)n, -1);
    for (int i = 0; i < n; ++i)
        for (int k = rp[i]; k < rp[i + 1]; ++k)
            if (ci[k] == i) {
                di[(size_t)i] = k;
                break;
            }
    for (int i = 0; i < n; ++i)
        if (di[(size_t)i] < 0) throw std::invalid_argument("ILU(0) needs an explicit diagonal entry in every row");
    for (int i = 1; i < n; ++i) {
        const int rowEnd = rp[i + 1];
        for (int k_ind = rp[i]; ci[k_ind] < i; ++k_ind) {
            const int k = ci[k_ind];
            int prev_ind = di[(size_t)k];
            const int prev_end = rp[k + 1];
            const double factor = lu[(size_t)k_ind] / lu[(size_t)prev_ind];
            lu[(size_t)k_ind] = factor;
            prev_ind += 1;
            for (int j_ind = k_ind + 1; j_ind < rowEnd && prev_ind < prev_end;) {
                if (ci[prev_ind] < ci[j_ind]) {
                    ++prev_ind;
                } else if (ci[prev_ind] > ci[j_ind]) {
                    ++j_ind;
                } else {
                    const double p = factor * lu[(size_t)prev_ind];
                    lu[(size_t)j_ind] -= p;
                    ++prev_ind;
                    ++j_ind;
                }
            }
        }
        double& d = lu[(size_t)di[(size_t)i]];
        if (d >= 0) {
            if (d < alpha) d = alpha;
        } else {
            if (d > -alpha) d = -alpha;
        }
    }
}

template <class T>
struct Prec {
    int kind = MPG_PREC_IDENTITY;
    std::vector<T> d;  // Jacobi: inverse boosted diagonal; ILU-Jacobi: 1/u_ii (types.hpp:305-316)
    // ILU(0) factors in one CSR (unit-lower L below the diagonal, U on and
    // above it), precision T, with an MKL handle for the triangular solves
    std::unique_ptr<Csr<T>> lu;
    std::vector<int> di;
    int steps = 1;
    mutable std::vector<T> t1, t2;

    void apply(T* w, int n) const {
        if (kind == MPG_PREC_JACOBI) {
            // gdmv(1.0, diag, w, 0.0, w): y = 0*y + 1*d*x
            for (int i = 0; i < n; ++i) w[i] = T(0) * w[i] + T(1) * d[(size_t)i] * w[i];
        } else if (kind == MPG_PREC_ILU) {
            ilusv(w, n);
        } else if (kind == MPG_PREC_ILU_JACOBI) {
            ilusv_jacobi(w, n);
        }
    }

    // ilusv (kernels_mkl.cpp:355-384): L then U sparse triangular solves
    void ilusv(T* x, int n) const {
        if (mkl().loaded) {
            t1.assign(x, x + n);
            trsv_mkl(SparseDescr{kSparseTypeTriangular, kSparseFillLower, kSparseDiagUnit}, t1.data(), x);
            t1.assign(x, x + n);
            trsv_mkl(SparseDescr{kSparseTypeTriangular, kSparseFillUpper, kSparseDiagNonUnit}, t1.data(), x);
            return;
        }
        const auto& A = *lu;
        for (int i = 0; i < n; ++i) {
            double s = x[i];
            for (int k = A.rp[i]; k < di[(size_t)i]; ++k) s -= (double)A.v[(size_t)k] * (double)x[A.ci[k]];
            x[i] = (T)s;
        }
        for (int i = n - 1; i >= 0; --i) {
            double s = x[i];
            for (int k = di[(size_t)i] + 1; k < A.rp[i + 1]; ++k) s -= (double)A.v[(size_t)k] * (double)x[A.ci[k]];
            x[i] = (T)(s / (double)A.v[(size_t)di[(size_t)i]]);
        }
    }
    void trsv_mkl(SparseDescr dsc, const T* in, T* out) const;

    // ilusv_jacobi (kernels.hpp:219-248) with the generic ilu_jacobi_mv
    // (kernels.hpp:171-210): `steps` Jacobi sweeps on L, then on U
    void ilusv_jacobi(T* x, int n) const {
        const auto& A = *lu;
        t1.assign(x, x + n);  // b
        t2.resize((size_t)n);
        for (int s = 0; s < steps; ++s) {
            for (int i = 0; i < n; ++i) {  // temp = b; temp = 1*temp + (-1)*(x_i + L x)
                T sum = x[i];
                for (int j = A.rp[i]; j < di[(size_t)i]; ++j) sum += A.v[(size_t)j] * x[A.ci[j]];
                t2[(size_t)i] = T(1) * t1[(size_t)i] + T(-1) * sum;
            }
            axpy(n, T(1), t2.data(), x);
        }
        t1.assign(x, x + n);
        for (int s = 0; s < steps; ++s) {
            for (int i = 0; i < n; ++i) {  // temp = b; temp = 1.0*temp + -1.0*(U x)
                T sum = 0;
                for (int j = di[(size_t)i]; j < A.rp[i + 1]; ++j) sum += A.v[(size_t)j] * x[A.ci[j]];
                t2[(size_t)i] = T(1.0) * t1[(size_t)i] + T(-1.0) * sum;
            }
            for (int i = 0; i < n; ++i) x[i] = T(1) * x[i] + T(1) * d[(size_t)i] * t2[(size_t)i];  // gdmv
        }
    }
};
template <>
void Prec<double>::trsv_mkl(SparseDescr dsc, const double* in, double* out) const {
    if (mkl().d_trsv(kSparseOpNoTrans, 1.0, lu->h, dsc, in, out)) throw std::runtime_error("mkl_sparse_d_trsv failed");
}
template <>
void Prec<float>::trsv_mkl(SparseDescr dsc, const float* in, float* out) const {
    if (mkl().s_trsv(kSparseOpNoTrans, 1.0f, lu->h, dsc, in, out)) throw std::runtime_error("mkl_sparse_s_trsv failed");
}

// Jacobi<T>(A) with A converted to T first (the implicit SparseMatrix<T>
// conversion at the call site, gmres_perf_test.cpp:80, 151); ILU / ILU-Jacobi
// from ilu0<T>(A) on the fp64 A (gmres_perf_test.cpp:70-79, 140-149).
template <class T>
Prec<T> make_prec(int kind, int n, const int* rp, const int* ci, const double* v64, int steps = 1) {
    Prec<T> M;
    M.kind = kind;
    if (kind == MPG_PREC_IDENTITY) return M;
    if (kind == MPG_PREC_ILU || kind == MPG_PREC_ILU_JACOBI) {
        std::vector<double> f;
        ilu0<T>(n, rp, ci, v64, f, M.di);
        M.lu = make_csr<T>(n, rp, ci, f.data());
        M.steps = steps;
        if (kind == MPG_PREC_ILU_JACOBI) {
            M.d.resize((size_t)n);
            for (int i = 0; i < n; ++i) M.d[(size_t)i] = 1 / M.lu->v[(size_t)M.di[(size_t)i]];
        }
        return M;
    }
    if (kind != MPG_PREC_JACOBI) throw std::invalid_argument("unknown preconditioner");
    M.d.resize((size_t)n);
    T alpha = 0;
    for (int i = 0; i < n; ++i) {
        T s = 0;
        for (int k = rp[i]; k < rp[i + 1]; ++k) s += std::fabs((T)v64[k]);
        if (alpha < s) alpha = s;
    }
    alpha *= std::numeric_limits<float>::epsilon();
    for (int i = 0; i < n; ++i) {
        int j = rp[i];
        while (j < rp[n] - 1 && ci[j] < i) ++j;
        const T a = (T)v64[j];
        M.d[(size_t)i] = a >= T(0) ? T(1) / (a < alpha ? alpha : a) : T(1) / (a > -alpha ? -alpha : a);
    }
    return M;
}

// ---- convergence strategies (IterUtil.hpp:17-227) ----
enum Action { NEXT, CONVERGED, RESTART, ABORTED };

struct Strategy {
    int kind = 0;  // 0 base, 1 repeat-iteration, 2 rel-prec-res, 3 lost-orthogonality
    double tol = 0, rtol = 0;
    size_t m = 0, max_restarts = 0;
    size_t total_iters = 0, total_restarts = 0;
    // adaptive state
    double restart_tol = 0;
    size_t second_len = 0;
    bool first = true;
    double loss2 = 0;
    // history
    std::vector<double> cyc_r, cyc_norm, cyc_beta, step_res;
    std::vector<int> step_cyc;
    double minvb = 0;

    Action base_initial(double r, double nrm) {
        ++total_restarts;
        if (total_restarts > max_restarts) return ABORTED;
        return r / nrm > tol ? NEXT : CONVERGED;
    }
    Action base_check(size_t k) {
        ++total_iters;
        return k >= m ? RESTART : NEXT;
    }
    Action check_initial(double r, double nrm, double pr, double pb) {
        cyc_r.push_back(r);
        cyc_norm.push_back(nrm);
        cyc_beta.push_back(pr);
        minvb = pb;
        if (kind == 1 && first) restart_tol = pr / pb * rtol;
        if (kind == 2) restart_tol = pr / pb * rtol;
        if (kind == 3) loss2 = 0;
        return base_initial(r, nrm);
    }
    bool needs_residual() const { return kind != 0; }
};

// ---- GMRES (gmres.cpp) ----
template <class T>
struct Workspace {
    int n, m;
    std::vector<T> V;  // n x (m+1), column-major, lda = n
    std::vector<T> H;  // (m+1) x m, lda = m+1
    std::vector<T> cs, sn, s, weights;
    std::vector<T> S, u;  // lost-orthogonality state
    Workspace(int n_, int m_)
        : n(n_), m(m_), V((size_t)n_ * (m_ + 1)), H((size_t)(m_ + 1) * m_), cs(m_ + 1), sn(m_ + 1), s(m_ + 1),
          weights(m_), S((size_t)(m_ + 1) * (m_ + 1)), u(m_ + 1) {}
    T* v(int j) { return V.data() + (size_t)j * n; }
    T& h(int i, int j) { return H[(size_t)j * (m + 1) + i]; }
};

template <class T>
void orthogonalize(int orth, Workspace<T>& ws, int k, T* w) {
    const int n = ws.n;
    T* hk = &ws.h(0, k);
    if (orth == MPG_ORTH_MGS) {
        for (int j = 0; j <= k; ++j) {
            hk[j] = dot(n, w, ws.v(j));
            axpy(n, -hk[j], ws.v(j), w);  // naxpy: y += -alpha x
        }
        return;
    }
    gemv(true, n, k + 1, T(1), ws.V.data(), n, w, T(0), hk);
    gemv(false, n, k + 1, T(-1), ws.V.data(), n, hk, T(1), w);
    if (orth == MPG_ORTH_CGSR) {
        gemv(true, n, k + 1, T(1), ws.V.data(), n, w, T(0), ws.weights.data());
        gemv(false, n, k + 1, T(-1), ws.V.data(), n, ws.weights.data(), T(1), w);
        axpy(k + 1, T(1), ws.weights.data(), hk);
    }
}

// copy(w, v) then scal — kernels_mkl.cpp:165-191
template <class T>
void scal_copy(int n, T a, const T* x, T* y) {
    std::memcpy(y, x, sizeof(T) * (size_t)n);
    scal(n, a, y);
}

template <class T>
void givens(Workspace<T>& ws, int k) {
    T* col = &ws.h(0, k);
    for (int j = 0; j < k; ++j) rot1(col + j, col + j + 1, ws.cs[j], ws.sn[j]);
    rotg(&ws.h(k, k), &ws.h(k + 1, k), &ws.cs[k], &ws.sn[k]);
    ws.h(k + 1, k) = 0;
    rot1(&ws.s[k], &ws.s[k + 1], ws.cs[k], ws.sn[k]);
}

// adaptive-strategy check (IterUtil.hpp:57-227) on the Arnoldi residual
template <class T>
Action strategy_check(Strategy& st, Workspace<T>& ws, size_t k, double res, double bnorm) {
    st.step_res.push_back(res);
    st.step_cyc.push_back((int)st.cyc_r.size() - 1);
    const Action a = st.base_check(k);
    switch (st.kind) {
        case 0: return a;
        case 1:
            if (st.first) {
                if (a != NEXT || res / bnorm <= st.restart_tol) {
                    st.first = false;
                    st.second_len = k;
                    return a != NEXT ? a : RESTART;
                }
                return NEXT;
            }
            if (a != NEXT) return a;
            return st.second_len <= k ? RESTART : NEXT;
        case 2:
            if (a != NEXT) return a;
            return res / bnorm <= st.restart_tol ? RESTART : NEXT;
        default: {
            if (a != NEXT) return a;
            const int n = ws.n, kk = (int)k;
            gemv(true, n, kk + 1, T(1), ws.V.data(), n, ws.v(kk + 1), T(0), ws.u.data());
            const int ld = ws.m + 1;
            T* scol = ws.S.data() + (size_t)(kk + 1) * ld;
            std::memcpy(scol, ws.u.data(), sizeof(T) * (size_t)(kk + 1));
            gemv(false, kk + 1, kk + 1, T(-1), ws.S.data(), ld, ws.u.data(), T(1), scol);
            st.loss2 += dot(kk + 1, scol, scol);
            return st.loss2 >= st.rtol * st.rtol ? RESTART : NEXT;
        }
    }
}

// x += V y (same precision) or x64 += double(V y) (mixed)
template <class T, class X>
void solution_update(Workspace<T>& ws, int k, X* x, T* tmp_low) {
    std::vector<T> y(ws.s.begin(), ws.s.begin() + k);
    trsv_upper(k, ws.H.data(), ws.m + 1, y.data());
    if constexpr (std::is_same<T, X>::value) {
        gemv(false, ws.n, k, T(1), ws.V.data(), ws.n, y.data(), T(1), x);
    } else {
        gemv(false, ws.n, k, T(1), ws.V.data(), ws.n, y.data(), T(0), tmp_low);
        std::vector<double> wide((size_t)ws.n);
        for (int i = 0; i < ws.n; ++i) wide[(size_t)i] = tmp_low[i];
        axpy(ws.n, 1.0, wide.data(), x);
    }
}

struct Outcome {
    int status = MPG_RESULT_ABORTED;
    long i = 0, k = 0;
};

// gmres.cpp:24-133 — Type T everywhere, preconditioner in P
template <class T, class P>
Outcome gmres_baseline(Strategy& st, int orth, const Csr<T>& A, const Prec<P>& M, const std::vector<T>& b,
                       std::vector<T>& x) {
    const int n = A.n, m = (int)st.m;
    Workspace<T> ws(n, m);
    std::vector<T> w((size_t)n);
    std::vector<P> wp((size_t)n);
    auto apply = [&](std::vector<T>& v) {
        if constexpr (std::is_same<T, P>::value) {
            M.apply(v.data(), n);
        } else {
            for (int i = 0; i < n; ++i) wp[(size_t)i] = (P)v[(size_t)i];
            M.apply(wp.data(), n);
            for (int i = 0; i < n; ++i) v[(size_t)i] = (T)wp[(size_t)i];
        }
    };
    st.total_iters = 0;
    const T b_norm = nrm2(n, b.data());
    w = b;
    apply(w);
    const T minvb = nrm2(n, w.data());
    const T a_norm = nrm2((int)A.v.size(), A.v.data());
    Outcome out;
    for (long i = 0;; ++i) {
        w = b;
        spmv(T(-1), A, x.data(), T(1), w.data());
        const T r_norm = nrm2(n, w.data());
        apply(w);
        const T beta = nrm2(n, w.data());
        const T x_norm = nrm2(n, x.data());
        const Action a0 = st.check_initial(r_norm, b_norm + a_norm * x_norm, beta, minvb);
        out.i = i;
        if (a0 == CONVERGED) {
            OUT("Found solution with rel prec res norm = %g when k = 0 and i = %ld\n", (double)T(beta / minvb), i);
            OUT("  total iterations = %zu\n", st.total_iters);
            out.status = MPG_RESULT_CONVERGED;
            return out;
        }
        if (a0 == ABORTED) {
            OUT("Aborting after %zu iterations\n", st.total_iters);
            out.status = MPG_RESULT_ABORTED;
            return out;
        }
        {  // first_vector
            const T bt = nrm2(n, w.data());
            if (bt != T(0)) scal_copy(n, T(1) / bt, w.data(), ws.v(0));
            else std::fill(ws.v(0), ws.v(0) + n, T(0));
        }
        std::fill(ws.s.begin(), ws.s.end(), T(0));
        ws.s[0] = beta;
        int k = 0;
        for (bool more = true; more; ++k) {
            spmv(T(1), A, ws.v(k), T(0), w.data());
            apply(w);
            orthogonalize(orth, ws, k, w.data());
            const T hn = nrm2(n, w.data());
            ws.h(k + 1, k) = hn;
            scal_copy(n, T(1) / hn, w.data(), ws.v(k + 1));
            givens(ws, k);
            const T ares = std::fabs(ws.s[(size_t)k + 1]);
            switch (strategy_check(st, ws, (size_t)k + 1, ares, minvb)) {
                case CONVERGED:
                    solution_update<T, T>(ws, k + 1, x.data(), nullptr);
                    OUT("Found solution with rel prec res norm = %g when k = %d and i = %ld\n", (double)(ares / minvb),
                        k + 1, i);
                    OUT("  total iterations = %zu\n", st.total_iters);
                    out.status = MPG_RESULT_CONVERGED;
                    out.k = k + 1;
                    return out;
                case RESTART: more = false; break;
                case ABORTED:
                    OUT("Aborting after %zu iterations\n", st.total_iters);
                    out.status = MPG_RESULT_ABORTED;
                    return out;
                case NEXT: break;
            }
        }
        solution_update<T, T>(ws, k, x.data(), nullptr);
    }
}

// gmres.cpp:135-245 — fp64 residual and update, fp32 Arnoldi
Outcome gmres_mixed(Strategy& st, int orth, const Csr<double>& A, const Csr<float>& As, const Prec<float>& M,
                    const std::vector<double>& b, std::vector<double>& x) {
    const int n = A.n, m = (int)st.m;
    Workspace<float> ws(n, m);
    std::vector<float> w((size_t)n);
    std::vector<double> r((size_t)n);
    st.total_iters = 0;
    const double b_norm = nrm2(n, b.data());
    for (int i = 0; i < n; ++i) w[(size_t)i] = (float)b[(size_t)i];
    M.apply(w.data(), n);
    const double minvb = nrm2(n, w.data());
    const double a_norm = nrm2((int)As.v.size(), As.v.data());
    Outcome out;
    for (long i = 0;; ++i) {
        r = b;
        spmv(-1.0, A, x.data(), 1.0, r.data());
        for (int j = 0; j < n; ++j) w[(size_t)j] = (float)r[(size_t)j];
        const double r_norm = nrm2(n, w.data());
        M.apply(w.data(), n);
        const float beta = nrm2(n, w.data());
        const double x_norm = nrm2(n, x.data());
        const Action a0 = st.check_initial(r_norm, b_norm + a_norm * x_norm, beta, minvb);
        out.i = i;
        if (a0 == CONVERGED) {
            OUT("Found solution with rel prec res norm = %g when k = 0 and i = %ld\n", (double)(beta / minvb), i);
            OUT("  total iterations = %zu\n", st.total_iters);
            out.status = MPG_RESULT_CONVERGED;
            return out;
        }
        if (a0 == ABORTED) {
            OUT("Aborting after %zu iterations\n", st.total_iters);
            out.status = MPG_RESULT_ABORTED;
            return out;
        }
        {
            const float bt = nrm2(n, w.data());
            if (bt != 0.0f) scal_copy(n, 1.0f / bt, w.data(), ws.v(0));
            else std::fill(ws.v(0), ws.v(0) + n, 0.0f);
        }
        std::fill(ws.s.begin(), ws.s.end(), 0.0f);
        ws.s[0] = beta;
        int k = 0;
        for (bool more = true; more; ++k) {
            spmv(1.0f, As, ws.v(k), 0.0f, w.data());
            M.apply(w.data(), n);
            orthogonalize(orth, ws, k, w.data());
            const float hn = nrm2(n, w.data());
            ws.h(k + 1, k) = hn;
            scal_copy(n, 1.0f / hn, w.data(), ws.v(k + 1));
            givens(ws, k);
            const double ares = std::fabs(ws.s[(size_t)k + 1]);
            switch (strategy_check(st, ws, (size_t)k + 1, ares, minvb)) {
                case CONVERGED:
                    solution_update<float, double>(ws, k + 1, x.data(), w.data());
                    OUT("Found solution with rel prec res norm = %g when k = %d and i = %ld\n", ares / minvb, k + 1, i);
                    OUT("  total iterations = %zu\n", st.total_iters);
                    out.status = MPG_RESULT_CONVERGED;
                    out.k = k + 1;
                    return out;
                case RESTART: more = false; break;
                case ABORTED:
                    OUT("Aborting after %zu iterations\n", st.total_iters);
                    out.status = MPG_RESULT_ABORTED;
                    return out;
                case NEXT: break;
            }
        }
        solution_update<float, double>(ws, k, x.data(), w.data());
    }
}

Strategy make_strategy(const mpg_solve_args& a) {
    Strategy st;
    st.tol = a.tol;
    st.rtol = a.rtol;
    st.m = (size_t)a.rlen;
    st.max_restarts = (size_t)a.max_restarts;
    st.kind = a.rtol == 0 ? 0 : a.repeat_iter ? 1 : a.orthloss ? 3 : 2;
    return st;
}

void fill_result(const Strategy& st, const Outcome& o, mpg_solve_result* r) {
    r->status = o.status;
    r->restarts = o.i;
    r->inner_k = o.k;
    r->total_iters = (int64_t)st.total_iters;
    r->minvb_norm = st.minvb;
    r->n_cycles = (int64_t)st.cyc_r.size();
    for (size_t c = 0; c < st.cyc_r.size() && (int64_t)c < r->cycle_cap; ++c) {
        if (r->cyc_r_norm) r->cyc_r_norm[c] = st.cyc_r[c];
        if (r->cyc_normalization) r->cyc_normalization[c] = st.cyc_norm[c];
        if (r->cyc_beta) r->cyc_beta[c] = st.cyc_beta[c];
    }
    r->n_steps = (int64_t)st.step_res.size();
    for (size_t s = 0; s < st.step_res.size() && (int64_t)s < r->step_cap; ++s) {
        if (r->step_res) r->step_res[s] = st.step_res[s];
        if (r->step_cycle) r->step_cycle[s] = st.step_cyc[s];
    }
    // the product's breakdown report (solve.h), counted the same way: steps
    // with a non-finite |s(k+1)|, restarts with a non-finite r_norm or beta
    r->nonfinite_steps = r->nonfinite_cycles = 0;
    r->first_nonfinite_step = -1;
    for (size_t s = 0; s < st.step_res.size(); ++s)
        if (!std::isfinite(st.step_res[s]) && r->nonfinite_steps++ == 0) r->first_nonfinite_step = (int64_t)s;
    for (size_t c = 0; c < st.cyc_r.size(); ++c)
        if (!std::isfinite(st.cyc_r[c]) || !std::isfinite(st.cyc_beta[c])) ++r->nonfinite_cycles;
}

// final report with the original fp64 A (gmres_perf_test.cpp:104-115, 169-178)
void report(const Csr<double>& A, const std::vector<double>& b_used, std::vector<double>& x, const double* x_true,
            mpg_solve_result* r) {
    const int n = A.n;
    if (r->x_out) std::memcpy(r->x_out, x.data(), sizeof(double) * (size_t)n);
    std::vector<double> res = b_used;
    spmv(-1.0, A, x.data(), 1.0, res.data());
    r->res_norm = nrm2(n, res.data());
    if (x_true) {
        axpy(n, -1.0, x_true, x.data());
        r->err_norm = nrm2(n, x.data());
    }
    OUT("  ilu took %gs; gmres took %gs\n", (double)(float)r->setup_seconds, (double)(float)r->gmres_seconds);
    OUT("  resNorm = %g; errNorm = %g\n", r->res_norm, r->err_norm);
}

using clk = std::chrono::steady_clock;
double since(clk::time_point t) { return std::chrono::duration<double>(clk::now() - t).count(); }

template <class T, class P>
void run_baseline(const mpg_solve_args& a, const Csr<double>& A, mpg_solve_result* r) {
    OUT("Doing Baseline test\n");
    const int n = a.n;
    auto t0 = clk::now();
    // gmres_perf_test.cpp:66: the solver matrix is the fp32-rounded A, widened to T
    std::vector<float> vf;
    cast(A.v, vf);
    auto At = make_csr<T>(n, a.rowptr, a.col, vf.data());
    Prec<P> M = make_prec<P>(a.prec, n, a.rowptr, a.col, a.val, a.jacobi_steps);
    r->setup_seconds = since(t0);
    std::vector<T> xt((size_t)n, T(0)), bt((size_t)n);
    for (int i = 0; i < n; ++i) bt[(size_t)i] = (T)a.b[i];
    Strategy st = make_strategy(a);
    auto t1 = clk::now();
    Outcome o = gmres_baseline<T, P>(st, a.orth, *At, M, bt, xt);
    r->gmres_seconds = since(t1);
    fill_result(st, o, r);
    std::vector<double> x((size_t)n), bu((size_t)n);
    for (int i = 0; i < n; ++i) {
        x[(size_t)i] = (double)xt[(size_t)i];
        bu[(size_t)i] = (double)bt[(size_t)i];
    }
    report(A, bu, x, a.x_true, r);
}

void run_mixed(const mpg_solve_args& a, const Csr<double>& A, mpg_solve_result* r) {
    OUT("Doing Mixed Precision test\n");
    const int n = a.n;
    std::vector<double> x((size_t)n, 0.0), b(a.b, a.b + n);
    auto t0 = clk::now();
    auto As = make_csr<float>(n, a.rowptr, a.col, a.val);
    Prec<float> M = make_prec<float>(a.prec, n, a.rowptr, a.col, a.val, a.jacobi_steps);
    r->setup_seconds = since(t0);
    Strategy st = make_strategy(a);
    auto t1 = clk::now();
    Outcome o = gmres_mixed(st, a.orth, A, *As, M, b, x);
    r->gmres_seconds = since(t1);
    fill_result(st, o, r);
    report(A, b, x, a.x_true, r);
}

}  // namespace
}  // namespace oracle

extern "C" {

const char* oracle_backend() { return oracle::backend_name(); }
int oracle_max_threads() { return oracle::max_threads(); }
int oracle_cbwr_branch() { return oracle::cbwr_branch(); }
void oracle_force_loops(int on) { oracle::force_loops(on != 0); }
// -1 MKL, 0 loops with fp64 sums, 1 loops with sequential fp32 sums, 2 loops
// with pairwise fp32 sums (cpu_blas.hpp)
void oracle_force_loops_mode(int mode) { oracle::force_loops_mode(mode); }

int oracle_solve(const mpg_solve_args* a, mpg_solve_result* r) {
    if (!a || !r) return -2;
    r->status = MPG_RESULT_ERROR;
    r->message[0] = 0;
    try {
        if (a->n <= 0 || a->rlen <= 0) throw std::invalid_argument("n and rlen must be positive");
        oracle::g_verbose = a->verbose != 0;
        oracle::set_threads(a->threads);
        auto A = oracle::make_csr<double>(a->n, a->rowptr, a->col, a->val);
        switch (a->mode) {
            case MPG_MODE_MIXED: oracle::run_mixed(*a, *A, r); break;
            case MPG_MODE_BASELINE: oracle::run_baseline<double, double>(*a, *A, r); break;
            case MPG_MODE_SINGLE_PREC: oracle::run_baseline<double, float>(*a, *A, r); break;
            case MPG_MODE_SINGLE: oracle::run_baseline<float, float>(*a, *A, r); break;
            default: throw std::invalid_argument("mode not covered by the oracle");
        }
        std::fflush(stdout);
        return 0;
    } catch (const std::exception& e) {
        std::snprintf(r->message, sizeof r->message, "%s", e.what());
        return -2;
    }
}

// ---- kernel-level oracles for the per-kernel parity tests ----
int oracle_spmv_f64(int n, const int* rp, const int* ci, const double* v, double alpha, const double* x, double beta,
                    double* y) {
    auto A = oracle::make_csr<double>(n, rp, ci, v);
    oracle::spmv(alpha, *A, x, beta, y);
    return 0;
}
int oracle_spmv_f32(int n, const int* rp, const int* ci, const float* v, float alpha, const float* x, float beta,
                    float* y) {
    auto A = oracle::make_csr<float>(n, rp, ci, v);
    oracle::spmv(alpha, *A, x, beta, y);
    return 0;
}
double oracle_dot_f64(int n, const double* x, const double* y) { return oracle::dot(n, x, y); }
float oracle_dot_f32(int n, const float* x, const float* y) { return oracle::dot(n, x, y); }
double oracle_nrm2_f64(int n, const double* x) { return oracle::nrm2(n, x); }
float oracle_nrm2_f32(int n, const float* x) { return oracle::nrm2(n, x); }
void oracle_gemv_f64(int trans, int rows, int cols, double alpha, const double* A, int lda, const double* x,
                     double beta, double* y) {
    oracle::gemv(trans != 0, rows, cols, alpha, A, lda, x, beta, y);
}
void oracle_gemv_f32(int trans, int rows, int cols, float alpha, const float* A, int lda, const float* x, float beta,
                     float* y) {
    oracle::gemv(trans != 0, rows, cols, alpha, A, lda, x, beta, y);
}
void oracle_trsv_upper_f64(int n, const double* A, int lda, double* x) { oracle::trsv_upper(n, A, lda, x); }
void oracle_trsv_upper_f32(int n, const float* A, int lda, float* x) { oracle::trsv_upper(n, A, lda, x); }
void oracle_rotg_f64(double* a, double* b, double* c, double* s) {
    oracle::rotg(a, b, c, s);
    *b = 0;
}
void oracle_rotg_f32(float* a, float* b, float* c, float* s) {
    oracle::rotg(a, b, c, s);
    *b = 0;
}
void oracle_jacobi_f64(int n, const int* rp, const int* ci, const double* v, double* d) {
    auto M = oracle::make_prec<double>(MPG_PREC_JACOBI, n, rp, ci, v);
    std::memcpy(d, M.d.data(), sizeof(double) * (size_t)n);
}
void oracle_jacobi_f32(int n, const int* rp, const int* ci, const double* v, float* d) {
    auto M = oracle::make_prec<float>(MPG_PREC_JACOBI, n, rp, ci, v);
    std::memcpy(d, M.d.data(), sizeof(float) * (size_t)n);
}

// ILU(0) factors (values in CSR order, rounded to fp64 or fp32) and the
// diagonal positions; then one apply of ILU (exact triangular solves) or of
// ILU-Jacobi with `steps` sweeps, in place on x
int oracle_ilu0_f64(int n, const int* rp, const int* ci, const double* v, double* lu, int* di) {
    try {
        std::vector<double> f;
        std::vector<int> d;
        oracle::ilu0<double>(n, rp, ci, v, f, d);
        std::memcpy(lu, f.data(), sizeof(double) * f.size());
        std::memcpy(di, d.data(), sizeof(int) * d.size());
        return 0;
    } catch (...) {
        return -1;
    }
}
int oracle_ilu0_f32(int n, const int* rp, const int* ci, const double* v, float* lu, int* di) {
    try {
        std::vector<double> f;
        std::vector<int> d;
        oracle::ilu0<float>(n, rp, ci, v, f, d);
        for (size_t k = 0; k < f.size(); ++k) lu[k] = (float)f[k];
        std::memcpy(di, d.data(), sizeof(int) * d.size());
        return 0;
    } catch (...) {
        return -1;
    }
}
int oracle_ilu_apply_f64(int n, const int* rp, const int* ci, const double* v, int kind, int steps, double* x) {
    try {
        auto M = oracle::make_prec<double>(kind, n, rp, ci, v, steps);
        M.apply(x, n);
        return 0;
    } catch (...) {
        return -1;
    }
}
int oracle_ilu_apply_f32(int n, const int* rp, const int* ci, const double* v, int kind, int steps, float* x) {
    try {
        auto M = oracle::make_prec<float>(kind, n, rp, ci, v, steps);
        M.apply(x, n);
        return 0;
    } catch (...) {
        return -1;
    }
}

}  // extern "C"
