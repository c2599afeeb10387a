// Fused Arnoldi engine: restarted GMRES(m) on one GPU (or one rank of a
// row-partitioned solve) with one host synchronisation per restart cycle.
//
// Same outer control flow as the drivers in gmres_impl.hpp (and the
// reference gmres.cpp:24-245): check_initial on the true residual at every
// restart, m Arnoldi steps, solution update. The cycle itself is the phase
// program of include/mpgmres/arnoldi.h, captured once into a hipGraph and
// replayed every cycle (steps 0..m-1, the solution update and the next
// residual prologue); the host reads back one small report block per cycle
// (r_norm, beta, ||x||, |s(k+1)| for every step). Strategies that look at
// |s(k+1)| inside a cycle run the same program step by step instead.
#ifndef MPGMRES_FUSED_GMRES_HPP
#define MPGMRES_FUSED_GMRES_HPP

#include <hip/hip_runtime.h>

#include <memory>
#include <string>
#include <vector>

#include "IterUtil.hpp"
#include "mpgmres/arnoldi.h"
#include "mpgmres/capi.h"
#include "mpgmres/solve.h"

namespace mpg {

// Communication seam of the row-partitioned solve: a single-GPU engine has
// no communicator; a multi-GPU rank supplies one (see comm.hpp).
class Comm {
public:
    virtual ~Comm() {}
    virtual int size() const = 0;
    virtual int rank() const = 0;
    // in-place sum / max of `count` doubles across ranks (bit-identical on every rank)
    virtual void allreduce_sum(double* dev, int count, hipStream_t s) = 0;
    virtual void allreduce_max(double* dev, int count, hipStream_t s) = 0;
    // fill the halo entries [-n_front, 0) and [n, n_ext) of a vector of
    // `elem_bytes` elements (passed as a pointer to its row 0)
    virtual void halo(void* dev_vec, int elem_bytes, hipStream_t s) = 0;
    // allreduce_sum and halo together (independent inputs): one RCCL group,
    // i.e. one collective launch per Arnoldi step instead of two
    virtual void allreduce_sum_and_halo(double* dev, int count, void* dev_vec, int elem_bytes, hipStream_t s) {
        allreduce_sum(dev, count, s);
        halo(dev_vec, elem_bytes, s);
    }
    // whether the collectives may be captured into a hipGraph (no host waits)
    virtual bool capturable() const = 0;
    // device-side transport (RCCL) whose collectives can hang or fail
    // asynchronously: the engine then waits with a bounded poll
    // (FusedEngine::wait_event) instead of a blocking synchronise
    virtual bool async() const { return false; }
    // "" or the transport's asynchronous error (ncclCommGetAsyncError)
    virtual std::string async_error() { return {}; }
    // tear the communicator down so that pending collectives return
    // (ncclCommAbort); called on the owning rank's thread only
    virtual void abort() {}
    // another rank failed: from any thread, ask the owning rank to abort
    // (RCCL: a flag its bounded wait polls, then abort() on its own thread)
    virtual void request_abort() { abort(); }
    // ranks the transport itself reports (RCCL: ncclCommCount), -1 when it
    // cannot say; the caller's size() otherwise
    virtual int transport_ranks() { return size(); }
};

// RAII device buffer through the C-ABI allocator
struct DevMem {
    mpg_ctx_t ctx = nullptr;
    void* p = nullptr;
    size_t bytes = 0;
    DevMem() = default;
    DevMem(mpg_ctx_t c, size_t b);
    ~DevMem();
    DevMem(const DevMem&) = delete;
    DevMem& operator=(const DevMem&) = delete;
    DevMem(DevMem&& o) noexcept { *this = std::move(o); }
    DevMem& operator=(DevMem&& o) noexcept;
    template <class T> T* as() const { return static_cast<T*>(p); }
};

class FusedEngine {
public:
    // `rows`/`halo` describe the local row block of a partitioned matrix
    // (global columns already remapped to [0, n_ext)); a single GPU passes the
    // whole matrix and no communicator.
    // n_front: halo rows of lower ranks, local ids [-n_front, 0) (dist.h)
    FusedEngine(mpg_ctx_t ctx, const mpg_solve_args& args, Comm* comm = nullptr, int n_ext = -1, int n_front = 0);
    ~FusedEngine();

    // Advance the solve by up to max_cycles outer iterations; returns the
    // number run. `done` is set on convergence or abort.
    int run(int max_cycles, bool& done);
    void finish_report(mpg_solve_result* r);  // resNorm/errNorm + x with the original fp64 A

    size_t total_iters() const { return conv_->total_iterations(); }
    double time_phase(int which, int reps, bool inplace = false, std::vector<double>* per_launch = nullptr);
    double time_phase_graph(int which, int reps, std::vector<double>* per_launch = nullptr);
    double time_phase_stamps(int which, int reps, std::vector<double>* per_launch = nullptr);
    double time_phase_dup(int which, int reps, int64_t* launches = nullptr);
    double phase_bytes(int which) const;
    mpg_arnoldi_t arnoldi() const;
    // mixed-half: what the fp16 cast of the Arnoldi values did (stats of
    // mpg_csr_half_values, capi.h; zeros in other modes)
    const int64_t* half_stats() const;
    // the Givens step rides the next SpMV (MPG_FOLD_GIVENS, mpg_arnoldi_fold_pays)
    bool givens_folded() const;
    void sync();

    // history (per restart / per step)
    std::vector<CycleRecord> cycles;
    std::vector<double> step_res;
    std::vector<int> step_cycle;
    int status = 0;          // MPG_RESULT_*
    int64_t restarts = 0;
    int64_t inner_k = 0;
    double minvb_norm = 0, b_norm = 0, a_norm = 0;
    double setup_seconds = 0;
    BreakdownLog breakdown;  // non-finite |s(k+1)| / restart residuals (IterUtil.hpp)
    // set by every time_phase*: the measurement launches (duplicated kernels,
    // cycles run without the host's checks) change V, H, w and x, so run()
    // refuses to continue the solve afterwards
    bool measured = false;

private:
    struct Impl;
    std::unique_ptr<Impl> p_;
    std::unique_ptr<Convergence<double, void>> conv_;
    void prologue();
    void step(int k, bool fold);
    void reduce(int nc);
    void allreduce_partials(int ncols);
    void givens(int k);
    template <class F>
    void timed(int phase, F&& launch);
    template <class F>
    void dup(int phase, F&& launch);
    void timed_end(int phase);
    void update(int k);
    void store_next_basis(int k);
    double orth_loss_step(size_t k);
    void read_report(int count);
    void wait_event(hipEvent_t ev, int64_t cycle, const char* what);
    void cycle_program();
    void ensure_graph();
    void record_steps(int64_t i);
    int run_pipelined(int max_cycles, bool& done);
    int run_cycles(int max_cycles, bool& done);
    bool check_start(int64_t i);
};

int solve_fused(const mpg_solve_args& args, mpg_solve_result* result);
// status, counts and the per-cycle / per-step history of an engine into r
void fill_history(const FusedEngine& e, mpg_solve_result* r);

}  // namespace mpg

// handle behind mpg_engine_t (solve.h / dist.h)
struct mpg_engine {
    mpg_ctx_t ctx = nullptr;
    std::unique_ptr<mpg::Comm> comm;          // declared first: destroyed after eng
    std::unique_ptr<mpg::FusedEngine> eng;
    std::string last_error;  // the text of the last failed mpg_engine_run
};

#endif  // MPGMRES_FUSED_GMRES_HPP
