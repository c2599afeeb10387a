// Derived from iamsonderr/icl-mixed-precision-gmres, Copyright (c) 2019-2021,
// University of Tennessee (BSD-3-Clause; the license text is in NOTICE).
// Restart / convergence control (reference IterUtil.hpp:10-227).
//
// Base Convergence (IterUtil.hpp:17-81): convergence is only ever declared
// by check_initial, from the true (unpreconditioned) residual at a restart
// boundary; check() only counts iterations and restarts at k == m. The three
// adaptive-restart strategies follow IterUtil.hpp:84-227 and need the
// per-step Arnoldi residual |s(k+1)| on the host (needs_arnoldi_residual()).
//
// Recorder is our addition: a pass-through that logs every argument the
// driver hands to the strategy, which is exactly the residual history the
// parity tests compare (per restart: r_norm, normalisation, preconditioned
// beta; per step: |s(k+1)|).
#ifndef MPGMRES_ITERUTIL_HPP
#define MPGMRES_ITERUTIL_HPP

#include <cmath>
#include <cstddef>
#include <cstdint>
#include <stdexcept>
#include <string>
#include <vector>

#include "Orthogonalization.hpp"
#include "kernels.hpp"

enum iteration_action { iteration_next, iteration_converged, iteration_restart, iteration_aborted };

template <class T, class Device>
class Convergence {
public:
    const double tol;
    const size_t restart_length;
    const size_t max_restarts;

    size_t total_iters = 0;
    size_t total_restarts = 0;

    Convergence(double tol, size_t restart_length, size_t max_restarts)
        : tol(tol), restart_length(restart_length), max_restarts(max_restarts) {}
    virtual ~Convergence() {}

    virtual void setup(Orthogonalization::Orth<T, Device>&) { total_iters = 0; }

    // (residual norm, ||b|| + ||A||_F ||x||, preconditioned residual norm,
    //  ||M^-1 b||) at the start of an outer iteration.
    virtual iteration_action check_initial(double residual_norm, double normalization, double, double) {
        ++total_restarts;
        if (total_restarts > max_restarts) return iteration_aborted;
        return residual_norm / normalization > tol ? iteration_next : iteration_converged;
    }

    // (inner index k >= 1, |s(k)|, ||M^-1 b||) after each Arnoldi step.
    virtual iteration_action check(size_t k, double, double) {
        ++total_iters;
        return k >= restart_length ? iteration_restart : iteration_next;
    }

    virtual size_t max_restart_length() const { return restart_length; }
    virtual size_t total_iterations() const { return total_iters; }

    // Whether check() looks at the Arnoldi residual. When false a driver may
    // defer the per-step device->host read of |s(k+1)| to the end of the
    // restart cycle without changing any decision.
    virtual bool needs_arnoldi_residual() const { return false; }
};

// Restart when the preconditioned residual improved by `restart_improvement`
// in the first cycle; later cycles reuse that cycle's length (IterUtil.hpp:84-137).
template <class T, class Device>
class RepeatIteration_Convergence : public Convergence<T, Device> {
    using Base = Convergence<T, Device>;
    const double restart_improvement_;
    double restart_tol_;
    size_t second_restart_length_ = 0;
    bool first_iteration_ = true;

public:
    RepeatIteration_Convergence(double tol, double restart_improvement, size_t restart_length, size_t max_restarts)
        : Base(tol, restart_length, max_restarts),
          restart_improvement_(restart_improvement),
          restart_tol_(restart_improvement) {}

    iteration_action check_initial(double r, double nrm, double prec_r, double prec_b) override {
        if (first_iteration_) restart_tol_ = prec_r / prec_b * restart_improvement_;
        return Base::check_initial(r, nrm, prec_r, prec_b);
    }

    iteration_action check(size_t k, double res, double bnorm) override {
        const iteration_action a = Base::check(k, res, bnorm);
        if (first_iteration_) {
            if (a != iteration_next) {
                first_iteration_ = false;
                second_restart_length_ = k;
                return a;
            }
            if (res / bnorm <= restart_tol_) {
                first_iteration_ = false;
                second_restart_length_ = k;
                return iteration_restart;
            }
            return iteration_next;
        }
        if (a != iteration_next) return a;
        return second_restart_length_ <= k ? iteration_restart : iteration_next;
    }
    bool needs_arnoldi_residual() const override { return true; }
};

// Restart once the preconditioned residual dropped by `restart_improvement`
// relative to the cycle start (IterUtil.hpp:139-169).
template <class T, class Device>
class RelPrecRes_Convergence : public Convergence<T, Device> {
    using Base = Convergence<T, Device>;
    const double restart_improvement_;
    double restart_tol_;

public:
    RelPrecRes_Convergence(double tol, double restart_improvement, size_t restart_length, size_t max_restarts)
        : Base(tol, restart_length, max_restarts),
          restart_improvement_(restart_improvement),
          restart_tol_(restart_improvement) {}

    iteration_action check_initial(double r, double nrm, double prec_r, double prec_b) override {
        restart_tol_ = prec_r / prec_b * restart_improvement_;
        return Base::check_initial(r, nrm, prec_r, prec_b);
    }
    iteration_action check(size_t k, double res, double bnorm) override {
        const iteration_action a = Base::check(k, res, bnorm);
        if (a != iteration_next) return a;
        return res / bnorm <= restart_tol_ ? iteration_restart : iteration_next;
    }
    bool needs_arnoldi_residual() const override { return true; }
};

// Restart when the accumulated loss of orthogonality of the basis exceeds
// restart_tol (IterUtil.hpp:172-227): S is updated with one V^T v_{k+1}
// panel product per step.
template <class T, class Device>
class LostOrthogonality_Convergence : public Convergence<T, Device> {
    using Base = Convergence<T, Device>;
    const double restart_tol_squared_;
    double current_loss_squared_ = 0;
    MultiVect<T, Device> S_;
    Vect<T, Device> u_;
    MultiVect<T, Device> v_;

public:
    LostOrthogonality_Convergence(double tol, double restart_tol, size_t restart_length, size_t max_restarts)
        : Base(tol, restart_length, max_restarts),
          restart_tol_squared_(restart_tol * restart_tol),
          S_(restart_length + 1, restart_length + 1),
          u_(restart_length + 1) {}

    void setup(Orthogonalization::Orth<T, Device>& orth) override {
        v_ = orth.basis();
        fill(0.0, S_);
        Base::setup(orth);
    }
    iteration_action check_initial(double r, double nrm, double prec_r, double prec_b) override {
        current_loss_squared_ = 0;
        return Base::check_initial(r, nrm, prec_r, prec_b);
    }
    iteration_action check(size_t k, double res, double bnorm) override {
        const iteration_action a = Base::check(k, res, bnorm);
        if (a != iteration_next) return a;
        const auto lead = std::make_pair(size_t(0), k + 1);
        Vect<T, Device> u(u_, lead);
        Vect<T, Device> vnew(v_, mpg::ALL, k + 1);
        MultiVect<T, Device> vprev(v_, mpg::ALL, lead);
        gemv(1.0, vprev.transpose_matrix(), vnew, 0.0, u);
        Vect<T, Device> scol(S_, lead, k + 1);
        MultiVect<T, Device> sprev(S_, lead, lead);
        copy(u, scol);
        gemv(-1.0, sprev, u, 1.0, scol);
        current_loss_squared_ += dot(scol, scol);
        return current_loss_squared_ >= restart_tol_squared_ ? iteration_restart : iteration_next;
    }
    bool needs_arnoldi_residual() const override { return true; }
};

namespace mpg {

struct CycleRecord {
    double r_norm = 0, normalization = 0, beta = 0, minvb_norm = 0;
};

// Breakdown report (our addition). The reference divides by
// h_{k+1,k} unguarded (Orthogonalization.hpp:56-59), so a zero or non-finite
// h turns |s(k+1)| and everything after it into NaN/Inf and the restart loop
// runs on until max_restarts. The solve keeps that behaviour; this log
// counts what happened, and with `stop` (--stop-on-breakdown) the driver
// ends the solve at the first non-finite value instead (BreakdownError ->
// MPG_ERR_BREAKDOWN).
struct BreakdownError : std::runtime_error {
    using std::runtime_error::runtime_error;
};
struct BreakdownLog {
    int64_t steps = 0, cycles = 0, first_step = -1;
    bool stop = false;
    // step `index` of the step history had |s(k+1)| = res
    void step(double res, int64_t index, int64_t cycle, size_t k) {
        if (std::isfinite(res)) return;
        if (steps++ == 0) first_step = index;
        if (stop)
            throw BreakdownError("non-finite Arnoldi residual |s(k+1)| at step k = " + std::to_string(k) +
                                 " of restart " + std::to_string(cycle) +
                                 " (h(k+1,k) zero or non-finite: breakdown; --stop-on-breakdown)");
    }
    // restart `cycle`: true residual norm and preconditioned beta
    void cycle(double r_norm, double beta, int64_t cycle) {
        if (std::isfinite(r_norm) && std::isfinite(beta)) return;
        ++cycles;
        if (stop)
            throw BreakdownError("non-finite residual norm at restart " + std::to_string(cycle) +
                                 " (--stop-on-breakdown)");
    }
};

// Pass-through strategy that records the residual history.
template <class T, class Device>
class Recorder : public Convergence<T, Device> {
    Convergence<T, Device>& inner_;

public:
    std::vector<CycleRecord> cycles;
    std::vector<double> step_residual;  // |s(k+1)| per Arnoldi step
    std::vector<int> step_cycle;        // cycle index of each step
    BreakdownLog breakdown;

    explicit Recorder(Convergence<T, Device>& inner)
        : Convergence<T, Device>(inner.tol, inner.restart_length, inner.max_restarts), inner_(inner) {}

    void setup(Orthogonalization::Orth<T, Device>& o) override { inner_.setup(o); }
    iteration_action check_initial(double r, double nrm, double pr, double pb) override {
        cycles.push_back(CycleRecord{r, nrm, pr, pb});
        breakdown.cycle(r, pr, (int64_t)cycles.size() - 1);
        return inner_.check_initial(r, nrm, pr, pb);
    }
    iteration_action check(size_t k, double res, double bnorm) override {
        step_residual.push_back(res);
        step_cycle.push_back((int)cycles.size() - 1);
        breakdown.step(res, (int64_t)step_residual.size() - 1, (int64_t)cycles.size() - 1, k - 1);
        return inner_.check(k, res, bnorm);
    }
    size_t max_restart_length() const override { return inner_.max_restart_length(); }
    size_t total_iterations() const override { return inner_.total_iterations(); }
    bool needs_arnoldi_residual() const override { return inner_.needs_arnoldi_residual(); }
};

}  // namespace mpg

#endif  // MPGMRES_ITERUTIL_HPP
