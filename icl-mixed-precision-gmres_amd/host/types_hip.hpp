// The `Hip` backend: device tag + CSR matrix type for MI355X (gfx950).
//
// Drop-in counterpart of types_mkl.hpp:11-107 / types_cuda.hpp:39-152. All
// device work goes through the C-ABI of libmpgmres_hip.so
// (include/mpgmres/capi.h); nothing here includes HIP kernels or Kokkos.
#ifndef MPGMRES_TYPES_HIP_HPP
#define MPGMRES_TYPES_HIP_HPP

#include <cstdlib>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "mpgmres/capi.h"
#include "mpgmres/ilu.h"
#include "kernels.hpp"
#include "types.hpp"

namespace mpg {

// Throws StatusError on a non-zero C-ABI status (the reference ignores cuBLAS
// statuses and asserts MKL ones; we never drop an error). mpg_solve returns
// the carried status.
struct StatusError : std::runtime_error {
    int status;
    StatusError(int st, const std::string& msg) : std::runtime_error(msg), status(st) {}
};
void check(int status, const char* what, mpg_ctx_t ctx = nullptr);
// A scheduling fault of the ILU triangular solves (the results of every
// apply since the last check are invalid): StatusError(MPG_ERR_BREAKDOWN).
void check_ilu_fault(mpg_ilu_t ilu);
// throws StatusError(MPG_ERR_UNSUPPORTED) while the current context records
void no_recording(const char* what);
// the queue of batched scalar operators (kernels_hip.cpp): issue it now /
// drop it (a voided recording re-runs its steps, which queue them again)
void flush_scalar_ops();
void discard_scalar_ops();
// a reduction's pending stage 2 (kernels_hip.cpp): issue it now / drop it
// (dropping also drops a deferred normalisation and w's redirect)
void flush_pending_reduction();
void discard_pending_reduction();
// add_vector's normalisation deferred to ride the next SpMV (kernels_hip.cpp,
// MPG_SURFACE_FUSE bit 16): issue it now as the separate calls would have
void flush_ride();
// device work issued outside an operator call (a cycle program's graph replay):
// ends the host-value nrm2 memo (kernels_hip.cpp)
void note_device_writes();
// false (and the redirect off for the rest of the solve) when a node SpMV's
// grid is too large for the normalisation to ride it (kernels_hip.cpp)
bool node_takes_norm_ride(mpg_node_t nd);
bool defer_norm(mpg_ctx_t c, int32_t nparts, void* h, const void* x, void* y, int64_t n, bool f64);
void* redirect_target(mpg_ctx_t c, void* y, int64_t n, bool f64);
void set_redirect(mpg_ctx_t c, void* w, void* sp, int64_t n, bool f64);
bool take_ride(const void* x, const void* y, int64_t n, bool f64, mpg_scalar_op* ops, int& nops, mpg_ctx_t& c,
               int32_t& nparts, void*& h, const void*& w);

// The calling thread's current HIP context (stream + workspace). Created
// lazily on the device named by MPG_DEVICE (default 0) unless a
// ScopedContext installed one.
mpg_ctx_t current_ctx();

class ScopedContext {
    mpg_ctx_t prev_;
    int prev_fuse_;  // the enclosing scope's MPG_SURFACE_FUSE mask (-1: none)
public:
    explicit ScopedContext(mpg_ctx_t ctx);
    ~ScopedContext();
    ScopedContext(const ScopedContext&) = delete;
    ScopedContext& operator=(const ScopedContext&) = delete;
};

// The SELL-64 copy of one SparseMatrix's values (mpg_sell_create), shared by
// the copies of that matrix (spmv takes A by value) and built on its first
// non-transposed spmv, when the values are final. Absent (h == nullptr) when
// slicing would not pay (format 0: padding > 20 %) or MPG_SURFACE_SELL=0.
// Round 5: the node-block copy (mpg_node_create) is built beside it on
// matrices of 3-dof nodes and replaces it when it streams fewer bytes
// (node_tile.hpp node_wins; MPG_SURFACE_NODE=0: never).
struct SellHolder {
    bool tried = false;
    mpg_sell_t h = nullptr;
    mpg_node_t node = nullptr;
    SellHolder() = default;
    SellHolder(const SellHolder&) = delete;
    SellHolder& operator=(const SellHolder&) = delete;
    ~SellHolder() {
        if (h) mpg_sell_destroy(h);
        if (node) mpg_node_destroy(node);
    }
};
bool surface_sell_enabled();
bool surface_node_enabled();

// Device CSR structure shared by every precision of one matrix.
struct CsrStructure {
    int m = 0, n = 0;
    int64_t nnz = 0;
    std::shared_ptr<void> row_map, inds;  // device int32
    std::shared_ptr<mpg_csr> csr;        // analysed CSR-adaptive schedule
    // A^T as its own CSR (mpg_csr_transpose), built on the first
    // set_transpose(true) of any SparseMatrix sharing this structure
    std::shared_ptr<CsrStructure> transposed;
    std::shared_ptr<void> perm;  // device int32[nnz]: source entry of each A^T entry
};

// Builds s.transposed / s.perm once (synchronises).
void build_transpose(CsrStructure& s);
// out[t] = vals[perm[t]] (the values of A^T in its CSR order)
void gather_entries(const CsrStructure& s, const void* vals, void* out, size_t elem_bytes);

}  // namespace mpg

// Device tag (types_mkl.hpp:11-15, types_cuda.hpp:39-44).
struct Hip {
    static constexpr bool host_accessible = false;
    static void* allocate(size_t bytes);
    static void deallocate(void* p);
    static void to_host(void* dst, const void* src, size_t bytes);
    static void to_device(void* dst, const void* src, size_t bytes);
    static void fence();
    using execution_space = Hip;
    using memory_space = Hip;
};

namespace mpg {

// Hip cycle program: the first cycle runs eagerly (lazy set-up such as the
// SELL copy of the Arnoldi matrix happens there), the second is recorded on
// the context's stream (mpg_ctx_record_begin) and launched, every later one
// is one graph launch. A step that cannot be recorded (one that synchronises,
// e.g. the ILU solve's fault check) voids the recording: nothing recorded has
// run, so the steps run eagerly from then on. MPG_SURFACE_GRAPH=0 disables it.
template <>
class CycleProgram<Hip> {
    mpg_graph_t g_ = nullptr;
    mpg_ctx_t ctx_ = nullptr;
    int cycles_ = 0;
    bool eager_;
    bool counted_;  // in mpg_cycle_program_counts (the Arnoldi cycle; not the solution update)

    static bool enabled();
    static void count(int which);  // 0 recorded, 1 replayed, 2 voided

public:
    // (MPG_SURFACE_UPDATE_PROG=0: the solution update runs eagerly)
    explicit CycleProgram(bool counted = true)
        : eager_(!enabled() || (!counted && std::getenv("MPG_SURFACE_UPDATE_PROG") &&
                                *std::getenv("MPG_SURFACE_UPDATE_PROG") == '0')),
          counted_(counted) {}
    ~CycleProgram() {
        if (g_) mpg_graph_destroy(g_);
    }
    CycleProgram(const CycleProgram&) = delete;
    CycleProgram& operator=(const CycleProgram&) = delete;

    bool recorded() const { return g_ != nullptr; }

    template <class F>
    void run(F&& steps) {
        if (g_) {
            note_device_writes();
            check(mpg_graph_launch(ctx_, g_), "cycle program launch", ctx_);
            if (counted_) count(1);
            return;
        }
        if (eager_ || cycles_++ == 0) {
            steps();
            return;
        }
        ctx_ = current_ctx();
        check(mpg_ctx_record_begin(ctx_), "cycle program record", ctx_);
        bool ok = true;
        try {
            steps();
            flush_scalar_ops();  // (issues a deferred normalisation first)
            flush_pending_reduction();
        } catch (const StatusError&) {
            // a step that cannot be recorded: end the recording and run eagerly
            discard_scalar_ops();
            discard_pending_reduction();
            ok = false;
        } catch (...) {
            // anything else: leave the context out of capture mode (a later
            // call on the stream would otherwise be recorded, not run), drop
            // the partial graph and the queued work, then rethrow
            discard_scalar_ops();
            discard_pending_reduction();
            mpg_graph_t partial = nullptr;
            (void)mpg_ctx_record_end(ctx_, &partial);
            if (partial) mpg_graph_destroy(partial);
            eager_ = true;
            throw;
        }
        mpg_graph_t g = nullptr;
        const int st = mpg_ctx_record_end(ctx_, &g);
        if (!ok || st != MPG_OK || !g) {
            if (g) mpg_graph_destroy(g);
            eager_ = true;
            if (counted_) count(2);
            steps();
            return;
        }
        g_ = g;
        note_device_writes();
        check(mpg_graph_launch(ctx_, g_), "cycle program launch", ctx_);
        if (counted_) count(0);
    }
};

}  // namespace mpg

// CSR on the device: shared int32 structure (row_map, inds, analysed row
// blocks) plus values of precision Type.
template <class Type>
class SparseMatrix<Type, Hip> {
    std::shared_ptr<mpg::CsrStructure> s_;
    Vect<Type, Hip> vals_;

    template <class, class> friend class SparseMatrix;

public:
    SparseMatrix() = default;

    // From host CSR arrays (0-based, int32), the values given in Type.
    SparseMatrix(int m, int n, const int* row_map, const int* inds, const Type* vals) {
        s_ = std::make_shared<mpg::CsrStructure>();
        s_->m = m;
        s_->n = n;
        s_->nnz = row_map[m];
        const size_t ib = sizeof(int) * (size_t)(m + 1), jb = sizeof(int) * (size_t)s_->nnz;
        s_->row_map = mpg::device_alloc<Hip>(ib);
        s_->inds = mpg::device_alloc<Hip>(jb);
        Hip::to_device(s_->row_map.get(), row_map, ib);
        if (jb) Hip::to_device(s_->inds.get(), inds, jb);
        mpg_csr_t csr = nullptr;
        mpg::check(mpg_csr_create(mpg::current_ctx(), m, n, s_->nnz, row_map,
                                  static_cast<const int32_t*>(s_->row_map.get()),
                                  static_cast<const int32_t*>(s_->inds.get()), &csr),
                   "mpg_csr_create");
        s_->csr = std::shared_ptr<mpg_csr>(csr, [](mpg_csr* p) { mpg_csr_destroy(p); });
        vals_ = Vect<Type, Hip>((size_t)s_->nnz);
        if (s_->nnz) Hip::to_device(vals_.data(), vals, sizeof(Type) * (size_t)s_->nnz);
    }

    // Precision-converting copy: shares the structure, casts the values on
    // the device, keeps the transpose flag (types_mkl.hpp:46-62,
    // types_cuda.hpp:82-101). Implicit, as in the reference —
    // DoBaselineProblem relies on it (§0.1-2 of SURVEY).
    template <class OldType>
    SparseMatrix(SparseMatrix<OldType, Hip> old) : s_(old.s_), vals_((size_t)old.s_->nnz) {
        copy(old.vals_, vals_);
        set_transpose(old.trans_);
    }

    // spmv then applies A^T (types_cuda.hpp:145-151; cusparse?csrmv with
    // CUSPARSE_OPERATION_TRANSPOSE, kernels_cuda.cpp:588-596). Copies share
    // the values, as the reference's do (condest.cpp:49-50: A_trans = A),
    // so the values are taken in A^T's order here, once; the structure of
    // A^T is built on first use and shared by every precision.
    void set_transpose(bool t) {
        trans_ = t;
        if (t && tvals_.n() != (size_t)s_->nnz) {
            mpg::build_transpose(*s_);
            tvals_ = Vect<Type, Hip>((size_t)s_->nnz);
            if (s_->nnz) mpg::gather_entries(*s_, vals_.data(), tvals_.data(), sizeof(Type));
        }
    }
    bool is_transposed() const { return trans_; }
    // the CSR and values spmv reads (A's, or A^T's when transposed)
    mpg_csr_t applied_csr() const { return trans_ ? s_->transposed->csr.get() : csr(); }
    Type* applied_vals() const { return trans_ ? tvals_.data() : vals_.data(); }

    const std::shared_ptr<mpg::CsrStructure>& structure() const { return s_; }
    int nrows() const { return s_->m; }
    int ncols() const { return s_->n; }
    int64_t nnz() const { return s_->nnz; }
    const int* row_map_data() const { return static_cast<const int*>(s_->row_map.get()); }
    const int* inds_data() const { return static_cast<const int*>(s_->inds.get()); }
    Type* vals_data() const { return vals_.data(); }
    mpg_csr_t csr() const { return s_->csr.get(); }
    Vect<Type, Hip> vals_vect() const { return vals_; }

    // the sliced copy spmv runs on, or nullptr (node blocks or CSR): A only, not A^T
    mpg_sell_t sell() const {
        build_copies();
        return trans_ || !sell_ ? nullptr : sell_->h;
    }
    // the node-block copy spmv runs on, or nullptr: A only, not A^T
    mpg_node_t node() const {
        build_copies();
        return trans_ || !sell_ ? nullptr : sell_->node;
    }

private:
    // SELL (format 0), then the node copy against the SELL copy's bytes or
    // the CSR arrays' (the one of the two that streams less is kept)
    void build_copies() const {
        if (trans_ || !sell_ || sell_->tried) return;
        sell_->tried = true;
        if (s_->nnz == 0) return;
        const int32_t vt = sizeof(Type) == 8 ? 0 : 1;
        if (mpg::surface_sell_enabled())
            mpg::check(mpg_sell_create(mpg::current_ctx(), csr(), vt, vals_.data(), 0, &sell_->h), "mpg_sell_create");
        if (!mpg::surface_node_enabled()) return;
        const int64_t alt = sell_->h ? mpg_sell_bytes(sell_->h)
                                     : s_->nnz * (int64_t)(sizeof(Type) + 4) + ((int64_t)s_->m + 1) * 4;
        // (an optimisation: a node copy that cannot be allocated leaves the
        // SELL copy or CSR in place)
        if (mpg_node_create(mpg::current_ctx(), csr(), vt, vals_.data(), alt, &sell_->node) != MPG_OK)
            sell_->node = nullptr;
        if (sell_->node && sell_->h) {
            mpg_sell_destroy(sell_->h);
            sell_->h = nullptr;
        }
    }
    std::shared_ptr<mpg::SellHolder> sell_ = std::make_shared<mpg::SellHolder>();
    bool trans_ = false;
    Vect<Type, Hip> tvals_;  // values in A^T's CSR order (set_transpose)
};

// ILU(0) factors on the device (types_mkl.hpp:110-190, types_cuda.hpp:155-240):
// a handle to the factor values in the matrix's CSR pattern, the pivot
// positions and the sync-free solve state (include/mpgmres/ilu.h).
template <class Type>
class ILU<Type, Hip> : public LinearOperator<Type, Hip> {
    std::shared_ptr<mpg_ilu> h_;
    int n_ = 0;
    int64_t nnz_ = 0;

public:
    ILU() = default;
    ILU(std::shared_ptr<mpg_ilu> h, int n, int64_t nnz) : h_(std::move(h)), n_(n), nnz_(nnz) {}
    int n() const { return n_; }
    int64_t nnz() const { return nnz_; }
    mpg_ilu_t handle() const { return h_.get(); }
    const Type* vals_data() const { return static_cast<const Type*>(mpg_ilu_values_dev(h_.get())); }
    void apply(Vect<Type, Hip> rhs) override { ilusv(*this, rhs); }
};

// ILU-Jacobi (types.hpp:251-372): the same factors, `steps` Jacobi sweeps
// per triangular factor instead of the exact solves.
template <class Type>
class ILU_Jacobi<Type, Hip> : public LinearOperator<Type, Hip> {
    ILU<Type, Hip> ilu_;
    int steps_ = 1;

public:
    ILU_Jacobi(ILU<Type, Hip> ilu, int steps) : ilu_(std::move(ilu)), steps_(steps) {}
    int n() const { return ilu_.n(); }
    int steps() const { return steps_; }
    mpg_ilu_t handle() const { return ilu_.handle(); }
    void apply(Vect<Type, Hip> rhs) override { ilusv_jacobi(*this, rhs); }
};

#endif  // MPGMRES_TYPES_HIP_HPP
