// Derived from iamsonderr/icl-mixed-precision-gmres, Copyright (c) 2019-2021,
// University of Tennessee (BSD-3-Clause; the license text is in NOTICE).
// Template bodies of the GMRES drivers declared in gmres.hpp.
//
// Control flow and arithmetic order follow the reference drivers
// (gmres.cpp:24-133 baseline, 135-245 mixed, 276-303 solution updates):
//   * the convergence test happens only at restart boundaries, on the true
//     residual, as a normwise backward error r / (||b|| + ||A||_F ||x||);
//   * mixed mode: r_norm is taken from the fp32 copy of the fp64 residual and
//     ||A||_F from the fp32 values (gmres.cpp:168, 175-176);
//   * the second Krylov basis the reference allocates and never uses
//     (gmres.cpp:44, 156) is not allocated.
// Differences: the initial Givens right-hand side s = [beta, 0, ...] is set
// with two fills instead of a Kokkos lambda, and the per-step host read of
// |s(k+1)| is skipped inside a cycle when the strategy does not look at it
// (Convergence::needs_arnoldi_residual) — the values are then read once per
// cycle, after the rotations, which does not change any decision.
#ifndef MPGMRES_GMRES_IMPL_HPP
#define MPGMRES_GMRES_IMPL_HPP

#include <cmath>
#include <type_traits>
#include <vector>

namespace mpg {

// gmres.cpp:12-22 — apply M in its own precision through a temporary
template <class Type, class Device, class RHSType>
void typesafe_apply(LinearOperator<Type, Device>* op, Vect<RHSType, Device> rhs, Vect<Type, Device> temp) {
    copy(rhs, temp);
    op->apply(temp);
    copy(temp, rhs);
}
template <class Type, class Device>
void typesafe_apply(LinearOperator<Type, Device>* op, Vect<Type, Device> rhs, Vect<Type, Device>) {
    op->apply(rhs);
}

// Givens update of column k of H and of the least-squares rhs s
// (gmres.cpp:104-110 / 217-222).
template <class Type, class Device>
void givens_step(size_t k, MultiVect<Type, Device>& h, Vect<Type, Device>& cs, Vect<Type, Device>& sn,
                 Vect<Type, Device>& s) {
    const auto prev = std::make_pair(size_t(0), k);
    rot(h(std::make_pair(size_t(0), k + 1), k), cs(prev), sn(prev));
    rotg(h(k, k), h(k + 1, k), cs(k), sn(k));
    rot(s(k), s(k + 1), cs(k), sn(k));
}

template <class Type, class Device>
void reset_rhs(Vect<Type, Device>& s, Type beta) {
    fill(0.0, s);
    fill(beta, s(0));
}

// Per-step residual bookkeeping: with a strategy that ignores |s(k+1)|
// inside the cycle, record it on the device side and hand the values to
// the strategy in one read at the end of the cycle.
template <class Type, class Device>
struct ArnoldiResidualLog {
    bool deferred = false;
    Vect<Type, Device> buf;   // |s(k+1)| candidates: s(k+1) after step k
    explicit ArnoldiResidualLog(size_t m, bool defer) : deferred(defer), buf(defer ? m : 0) {}
};

}  // namespace mpg

template <class Orth, class Device, class Type, class PrecType>
void gmres_baseline(Convergence<Type, Device>& convergence, SparseMatrix<Type, Device> A,
                    LinearOperator<PrecType, Device>* M, Vect<Type, Device> b, Vect<Type, Device> x) {
    const size_t n = x.n();
    const size_t m = convergence.max_restart_length();

    Orth orth(n, m);
    Vect<Type, Device> cs(m + 1), sn(m + 1), s(m + 1);
    Vect<Type, Device> w(n);
    MultiVect<Type, Device> h(m + 1, m);
    Vect<PrecType, Device> w_temp(std::is_same<PrecType, Type>::value ? 0 : n);
    const bool defer = !convergence.needs_arnoldi_residual();
    mpg::ArnoldiResidualLog<Type, Device> rlog(m, defer);
    mpg::CycleProgram<Device> cycle;
    // the solution update after a full deferred cycle (k = m): device-only
    // too, so recorded and replayed like the cycle (its launches would
    // otherwise be paced by the host's)
    mpg::CycleProgram<Device> update(false);

    convergence.setup(orth);

    const Type b_norm = nrm2(b);
    copy(b, w);
    mpg::typesafe_apply(M, w, w_temp);
    const Type Minvb_norm = nrm2(w);
    const Type A_norm = nrm2(A.vals_vect());

    for (size_t i = 0;; ++i) {
        // M r = M (b - A x)
        copy(b, w);
        spmv(-1.0, A, x, 1.0, w);
        const Type r_norm = nrm2(w);
        mpg::typesafe_apply(M, w, w_temp);
        const Type beta = nrm2(w);
        const Type x_norm = nrm2(x);

        const iteration_action start = convergence.check_initial(r_norm, b_norm + A_norm * x_norm, beta, Minvb_norm);
        if (start == iteration_converged) {
            mpg::out() << "Found solution with rel prec res norm = " << Type(beta / Minvb_norm)
                       << " when k = 0 and i = " << i << std::endl;
            mpg::out() << "  total iterations = " << convergence.total_iterations() << std::endl;
            return;
        }
        if (start == iteration_aborted) {
            mpg::out() << "Aborting after " << convergence.total_iterations() << " iterations" << std::endl;
            return;
        }

        orth.first_vector(w);
        mpg::reset_rhs(s, beta);

        size_t k = 0;
        if (defer) {
            // base strategy: no decision inside the cycle, so its m steps are
            // device-only and run as one cycle program (recorded once on Hip)
            cycle.run([&] {
                for (size_t j = 0; j < m; ++j) {
                    spmv(1.0, A, orth.previous_krylov_vector(j), 0.0, w);
                    mpg::typesafe_apply(M, w, w_temp);
                    orth.add_vector(j, w, h);
                    mpg::givens_step(j, h, cs, sn, s);
                    copy(s(j + 1), rlog.buf(j));
                }
            });
            // (no fence: to_host is ordered after the cycle on the stream and
            // waits for it; a fence first would leave the read's copy to start
            // on an idle queue after the host saw the cycle end)
            std::vector<Type> res(m);
            Device::to_host(res.data(), rlog.buf.data(), m * sizeof(Type));
            for (size_t j = 0; j < m; ++j) {
                const iteration_action a = convergence.check(j + 1, std::fabs(res[j]), Minvb_norm);
                if (a == iteration_aborted) {
                    mpg::out() << "Aborting after " << convergence.total_iterations() << " iterations" << std::endl;
                    return;
                }
            }
            k = m;
        }
        for (bool more = !defer; more; ++k) {
            spmv(1.0, A, orth.previous_krylov_vector(k), 0.0, w);
            mpg::typesafe_apply(M, w, w_temp);
            orth.add_vector(k, w, h);
            mpg::givens_step(k, h, cs, sn, s);

            Device::fence();
            const Type arnoldi_residual = std::fabs(s.access(k + 1));
            switch (convergence.check(k + 1, arnoldi_residual, Minvb_norm)) {
                case iteration_converged:
                    solution_update(orth, x, k + 1, h, s);
                    mpg::out() << "Found solution with rel prec res norm = " << arnoldi_residual / Minvb_norm
                               << " when k = " << k + 1 << " and i = " << i << std::endl;
                    mpg::out() << "  total iterations = " << convergence.total_iterations() << std::endl;
                    return;
                case iteration_restart:
                    more = false;
                    break;
                case iteration_aborted:
                    mpg::out() << "Aborting after " << convergence.total_iterations() << " iterations" << std::endl;
                    return;
                case iteration_next:
                    break;
            }
        }
        if (defer)
            update.run([&] { solution_update(orth, x, k, h, s); });
        else
            solution_update(orth, x, k, h, s);
    }
}

template <class Orth, class Device>
void gmres_singleUpdate(Convergence<float, Device>& convergence, SparseMatrix<double, Device> A,
                        SparseMatrix<float, Device> A_single, LinearOperator<float, Device>* M,
                        Vect<double, Device> b, Vect<double, Device> x) {
    const size_t n = x.n();
    const size_t m = convergence.max_restart_length();

    Orth orth(n, m);
    Vect<float, Device> cs(m + 1), sn(m + 1), s(m + 1);
    Vect<float, Device> w(n);
    MultiVect<float, Device> h(m + 1, m);
    Vect<double, Device> r_accum(n);  // fp64 residual; also the widening temp of the update
    const bool defer = !convergence.needs_arnoldi_residual();
    mpg::ArnoldiResidualLog<float, Device> rlog(m, defer);
    mpg::CycleProgram<Device> cycle;
    // the solution update after a full deferred cycle (k = m): device-only
    // too, so recorded and replayed like the cycle (its launches would
    // otherwise be paced by the host's)
    mpg::CycleProgram<Device> update(false);

    convergence.setup(orth);

    const double b_norm = nrm2(b);
    copy(b, w);
    M->apply(w);
    const double Minvb_norm = nrm2(w);
    const double A_norm = nrm2(A_single.vals_vect());  // Frobenius norm of the fp32 values

    for (size_t i = 0;; ++i) {
        // r = b - A x in fp64, then handed to the fp32 cycle
        copy(b, r_accum);
        spmv(-1.0, A, x, 1.0, r_accum);
        copy(r_accum, w);
        const double r_norm = nrm2(w);
        M->apply(w);
        const float beta = nrm2(w);
        const double x_norm = nrm2(x);

        const iteration_action start = convergence.check_initial(r_norm, b_norm + A_norm * x_norm, beta, Minvb_norm);
        if (start == iteration_converged) {
            mpg::out() << "Found solution with rel prec res norm = " << double(beta / Minvb_norm)
                       << " when k = 0 and i = " << i << std::endl;
            mpg::out() << "  total iterations = " << convergence.total_iterations() << std::endl;
            return;
        }
        if (start == iteration_aborted) {
            mpg::out() << "Aborting after " << convergence.total_iterations() << " iterations" << std::endl;
            return;
        }

        orth.first_vector(w);
        mpg::reset_rhs(s, beta);

        size_t k = 0;
        if (defer) {
            // base strategy: no decision inside the cycle, so its m steps are
            // device-only and run as one cycle program (recorded once on Hip)
            cycle.run([&] {
                for (size_t j = 0; j < m; ++j) {
                    spmv(1.0, A_single, orth.previous_krylov_vector(j), 0.0, w);
                    M->apply(w);
                    orth.add_vector(j, w, h);
                    mpg::givens_step(j, h, cs, sn, s);
                    copy(s(j + 1), rlog.buf(j));
                }
            });
            std::vector<float> res(m);  // (to_host waits for the cycle: no fence)
            Device::to_host(res.data(), rlog.buf.data(), m * sizeof(float));
            for (size_t j = 0; j < m; ++j) {
                const iteration_action a = convergence.check(j + 1, std::fabs(double(res[j])), Minvb_norm);
                if (a == iteration_aborted) {
                    mpg::out() << "Aborting after " << convergence.total_iterations() << " iterations" << std::endl;
                    return;
                }
            }
            k = m;
        }
        for (bool more = !defer; more; ++k) {
            spmv(1.0, A_single, orth.previous_krylov_vector(k), 0.0, w);
            M->apply(w);
            orth.add_vector(k, w, h);
            // mixed driver rotates h(0:k, k) — same k entries touched (gmres.cpp:219-220)
            mpg::givens_step(k, h, cs, sn, s);

            Device::fence();
            const double arnoldi_residual = std::fabs(s.access(k + 1));
            switch (convergence.check(k + 1, arnoldi_residual, Minvb_norm)) {
                case iteration_converged:
                    solution_update(orth, x, k + 1, h, s, w, r_accum);
                    mpg::out() << "Found solution with rel prec res norm = " << arnoldi_residual / Minvb_norm
                               << " when k = " << k + 1 << " and i = " << i << std::endl;
                    mpg::out() << "  total iterations = " << convergence.total_iterations() << std::endl;
                    return;
                case iteration_restart:
                    more = false;
                    break;
                case iteration_aborted:
                    mpg::out() << "Aborting after " << convergence.total_iterations() << " iterations" << std::endl;
                    return;
                case iteration_next:
                    break;
            }
        }
        if (defer)
            update.run([&] { solution_update(orth, x, k, h, s, w, r_accum); });
        else
            solution_update(orth, x, k, h, s, w, r_accum);
    }
}

template <class Orth, class Device>
void solution_update(Orth& orth, Vect<double, Device>& x, const size_t k, const MultiVect<float, Device> h,
                     const Vect<float, Device> s, Vect<float, Device> x_inc_temp, Vect<double, Device> x_temp) {
    const auto lead = std::make_pair(size_t(0), k);
    Vect<float, Device> y(s, lead);
    MultiVect<float, Device> hk(h, lead, lead);
    trsv("Upper", hk, y);
    orth.update_x(k, y, x, x_inc_temp, x_temp);
}

template <class Orth, class Device, class Type>
void solution_update(Orth& orth, Vect<Type, Device>& x, const size_t k, const MultiVect<Type, Device> h,
                     const Vect<Type, Device> s) {
    const auto lead = std::make_pair(size_t(0), k);
    Vect<Type, Device> y(s, lead);
    MultiVect<Type, Device> hk(h, lead, lead);
    trsv("Upper", hk, y);
    orth.update_x(k, y, x);
}

#endif  // MPGMRES_GMRES_IMPL_HPP
