// Fused Arnoldi engine (see fused_gmres.hpp) and its C-ABI (mpg_engine_*,
// mpg_solve with engine = MPG_ENGINE_FUSED).
#include "fused_gmres.hpp"

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <functional>
#include <stdexcept>
#include <thread>

#include "gmres.hpp"
#include "types_hip.hpp"

namespace mpg {

// ---------------------------------------------------------------- DevMem
DevMem::DevMem(mpg_ctx_t c, size_t b) : ctx(c), bytes(b) { check(mpg_malloc(c, b, &p), "mpg_malloc", c); }
DevMem::~DevMem() {
    if (p) mpg_free(ctx, p);
}
DevMem& DevMem::operator=(DevMem&& o) noexcept {
    if (this != &o) {
        if (p) mpg_free(ctx, p);
        ctx = o.ctx;
        p = o.p;
        bytes = o.bytes;
        o.p = nullptr;
        o.bytes = 0;
    }
    return *this;
}

namespace {

using clk = std::chrono::steady_clock;

void hipck(hipError_t e, const char* what) {
    if (e != hipSuccess) throw std::runtime_error(std::string("mpgmres: ") + what + ": " + hipGetErrorString(e));
}

// the driver's working types for a mode (gmres_perf_test.cpp:240-305)
struct ModeTypes {
    int T, X, P, VI;  // mpg_dtype_t
    bool single_scalars;  // host scalars in float (mode single)
};
ModeTypes types_for(int mode) {
    switch (mode) {
        case MPG_MODE_MIXED: return {MPG_F32, MPG_F64, MPG_F32, MPG_F32, false};
        case MPG_MODE_MIXED_HALF: return {MPG_F32, MPG_F64, MPG_F32, MPG_F16, false};
        case MPG_MODE_BASELINE: return {MPG_F64, MPG_F64, MPG_F64, MPG_F64, false};
        case MPG_MODE_SINGLE_PREC: return {MPG_F64, MPG_F64, MPG_F32, MPG_F64, false};
        case MPG_MODE_SINGLE: return {MPG_F32, MPG_F32, MPG_F32, MPG_F32, true};
        default: throw std::invalid_argument("unknown mode");
    }
}
size_t dsize(int t) { return t == MPG_F64 ? 8 : t == MPG_F32 ? 4 : 2; }

// LostOrthogonality (IterUtil.hpp:172-227) on the fused engine's basis. The
// base check (count, restart at m) comes first, as in the reference; the
// V^T v / S-column update is the engine's (orth_loss_step), which returns
// dot(s_col, s_col) rounded to the basis precision.
class LostOrthogonalityFused : public Convergence<double, void> {
    using Base = Convergence<double, void>;
    const double restart_tol_squared_;
    double current_loss_squared_ = 0;

public:
    std::function<double(size_t)> step_loss;
    LostOrthogonalityFused(double tol, double restart_tol, size_t m, size_t max_restarts)
        : Base(tol, m, max_restarts), restart_tol_squared_(restart_tol * restart_tol) {}
    iteration_action check_initial(double r, double nrm, double pr, double pb) override {
        current_loss_squared_ = 0;
        return Base::check_initial(r, nrm, pr, pb);
    }
    iteration_action check(size_t k, double res, double bnorm) override {
        const iteration_action a = Base::check(k, res, bnorm);
        if (a != iteration_next) return a;
        current_loss_squared_ += step_loss(k);
        return current_loss_squared_ >= restart_tol_squared_ ? iteration_restart : iteration_next;
    }
    bool needs_arnoldi_residual() const override { return true; }
};

}  // namespace

struct FusedEngine::Impl {
    mpg_ctx_t ctx = nullptr;
    mpg_solve_args args{};
    Comm* comm = nullptr;
    ModeTypes ty{};
    int n = 0, n_ext = 0, m = 0, orth = 0;
    int front = 0;       // MPG_FRONT_PAD(n_front): entries of x / x64 before row 0
    void* xp = nullptr;  // row 0 of x (x.p + front entries)
    int64_t nnz = 0;
    DevMem rowptr, col, val64, val_outer_own, val_inner_own, diag, b, x, tmp_t, tmp_p, scal;
    DevMem row_exp;                 // mixed-half: per-row exponents of the scaled fp16 values
    int64_t half_stats[4] = {0, 0, 0, 0};
    const void* val_outer = nullptr;
    const void* val_inner = nullptr;
    mpg_csr_t csr = nullptr;
    mpg_arnoldi_t arn = nullptr;
    double* rep[2] = {nullptr, nullptr};  // pinned report buffers (two: pipelined cycles)
    double* report_host = nullptr;       // = rep[0] or rep[1]: the report the host works on
    int report_len = 0;
    // pipelined cycles: the next cycle's graph is launched before this
    // cycle's report is read; it starts by saving x, so a cycle launched past
    // a stop decision is undone by restoring x
    bool pipeline = true;
    DevMem x_snap;
    hipEvent_t report_ev[2] = {nullptr, nullptr};
    hipGraph_t graph = nullptr;
    hipGraphExec_t graph_exec = nullptr;
    bool use_graph = true;
    bool fold = false;     // Givens step folded into the next SpMV launch
    bool combine = false;  // last-arriver combines in the dots and CGS launches
    bool cgs_partials = false;  // CGS update sums the dots partials in-launch
    bool fuse_dots = false;     // ... from dots formed in the SpMV launch
    bool fuse_dots_required = false;
    int fuse_dots_k0 = 32;      // ... for the steps with k + 1 <= fuse_dots_k0
    int timed = -1;                  // phase whose launches time_phase brackets with events
    bool timed_inplace = false;      // ... the cycle's own SpMV launch, by its kernel events
    bool timed_graph = false;        // ... external event nodes around it in a captured cycle
    std::vector<hipEvent_t> marks;   // ... begin/end pairs
    unsigned long long* stamps = nullptr;  // time_phase_stamps: wave stamp slots of each timed launch
    int dup_phase = -1;   // time_phase_dup: phase whose site launches its kernel twice
    int64_t dup_count = 0;  // ... extra launches captured
    int64_t dup_with_dots = 0;  // ... of which re-ran the dots ahead of a CGS update
    int64_t stamp_cap = 0, stamp_q = 0, stamp_max = 0;  // waves per launch, launches armed, launch slots
    std::vector<int32_t> rowptr_host;
    mpg_ilu_t ilu = nullptr;  // ILU(0) factors (prec ilu / ilu_jacobi), applied between phase kernels
    bool orthloss = false;    // LostOrthogonality: v_{k+1} stored each step, S / u below
    DevMem loss_S, loss_u;    // (m+1) x (m+1) and m+2 of T, zero-filled (IterUtil.hpp:185-191)

    ~Impl() {
        if (ilu) mpg_ilu_destroy(ilu);
        if (graph_exec) (void)hipGraphExecDestroy(graph_exec);
        if (graph) (void)hipGraphDestroy(graph);
        if (arn) mpg_arnoldi_destroy(arn);
        if (csr) mpg_csr_destroy(csr);
        for (double* r : rep)
            if (r) (void)hipHostFree(r);
        for (hipEvent_t e : report_ev)
            if (e) (void)hipEventDestroy(e);
    }
    hipStream_t stream() const { return static_cast<hipStream_t>(mpg_ctx_stream(ctx)); }

    // cast-copy between device arrays of runtime dtypes
    void cast(const void* src, int st, void* dst, int dt, int64_t count) {
        if (count == 0) return;
        if (st == MPG_F64 && dt == MPG_F64) check(mpg_copy_f64f64(ctx, count, (const double*)src, (double*)dst), "copy", ctx);
        else if (st == MPG_F64 && dt == MPG_F32) check(mpg_copy_f64f32(ctx, count, (const double*)src, (float*)dst), "copy", ctx);
        else if (st == MPG_F32 && dt == MPG_F64) check(mpg_copy_f32f64(ctx, count, (const float*)src, (double*)dst), "copy", ctx);
        else if (st == MPG_F32 && dt == MPG_F32) check(mpg_copy_f32f32(ctx, count, (const float*)src, (float*)dst), "copy", ctx);
        else if (st == MPG_F64 && dt == MPG_F16) check(mpg_copy_f64f16(ctx, count, (const double*)src, (uint16_t*)dst), "copy", ctx);
        else throw std::invalid_argument("unsupported cast");
    }
    // fp64 accumulator of <u, v> over local rows, summed across ranks
    double dot_acc(const void* u, const void* v, int t, int64_t count) {
        double* acc = scal.as<double>();
        if (t == MPG_F64) check(mpg_dot_acc_f64(ctx, count, (const double*)u, (const double*)v, acc), "dot", ctx);
        else check(mpg_dot_acc_f32(ctx, count, (const float*)u, (const float*)v, acc), "dot", ctx);
        if (comm) comm->allreduce_sum(acc, 1, stream());
        double h = 0;
        check(mpg_memcpy_d2h(ctx, &h, acc, sizeof h), "d2h", ctx);
        return h;
    }
    // M^-1 w for the ILU preconditioners, with typesafe_apply's casts when
    // the preconditioner precision differs (gmres.cpp:12-22)
    void apply_ilu(void* w) {
        void* wp = w;
        if (ty.P != ty.T) {
            cast(w, ty.T, tmp_p.p, ty.P, n);
            wp = tmp_p.p;
        }
        solve_ilu(wp);
        if (ty.P != ty.T) cast(tmp_p.p, ty.P, w, ty.T, n);
    }
    void solve_ilu(void* wp) {
        if (args.prec == MPG_PREC_ILU) check(mpg_ilu_solve(ctx, ilu, wp), "ilusv", ctx);
        else check(mpg_ilu_jacobi_solve(ctx, ilu, args.jacobi_steps, wp), "ilusv_jacobi", ctx);
    }
    // nrm2 rounded to the vector's precision
    double nrm2(const void* u, int t, int64_t count) {
        const double s = std::sqrt(dot_acc(u, u, t, count));
        return t == MPG_F64 ? s : (double)(float)s;
    }
};

FusedEngine::FusedEngine(mpg_ctx_t ctx, const mpg_solve_args& a, Comm* comm, int n_ext, int n_front)
    : p_(new Impl) {
    auto t0 = clk::now();
    Impl& I = *p_;
    I.ctx = ctx;
    I.args = a;
    I.comm = comm;
    I.ty = types_for(a.mode);
    I.n = a.n;
    I.n_ext = n_ext < 0 ? a.n : n_ext;
    if (n_front < 0) throw std::invalid_argument("n_front < 0");
    I.front = MPG_FRONT_PAD(n_front);
    I.m = a.rlen;
    I.orth = a.orth;
    I.nnz = a.nnz;
    const bool ilu = a.prec == MPG_PREC_ILU || a.prec == MPG_PREC_ILU_JACOBI;
    if (ilu && comm)
        throw std::invalid_argument("ILU / ILU-Jacobi factor the whole matrix: not available on a row-partitioned solve");
    if (!ilu && a.prec != MPG_PREC_IDENTITY && a.prec != MPG_PREC_JACOBI) throw std::invalid_argument("Unknown prec type");
    I.orthloss = a.orthloss && a.rtol != 0 && !a.repeat_iter;  // alloc_convergence order (gmres_perf_test.cpp:184-195)
    if (I.orthloss && comm)
        throw std::invalid_argument("LostOrthogonality restarts are not available on a row-partitioned solve");
    if (a.rowptr[a.n] != a.nnz) throw std::invalid_argument("rowptr[n] != nnz");

    // structure + analysed schedule
    const size_t n1 = (size_t)I.n + 1, nz = (size_t)I.nnz;
    I.rowptr = DevMem(ctx, n1 * 4);
    I.col = DevMem(ctx, std::max<size_t>(nz, 1) * 4);
    check(mpg_memcpy_h2d(ctx, I.rowptr.p, a.rowptr, n1 * 4), "h2d", ctx);
    if (nz) check(mpg_memcpy_h2d(ctx, I.col.p, a.col, nz * 4), "h2d", ctx);
    check(mpg_csr_create(ctx, I.n, I.n_ext, I.nnz, a.rowptr, I.rowptr.as<int32_t>(), I.col.as<int32_t>(), &I.csr),
          "mpg_csr_create", ctx);

    // values: the original fp64 A, the residual matrix (outer type) and the
    // Arnoldi matrix (inner type) — gmres_perf_test.cpp:66 (baseline solves with
    // double(float(A))) and :136 (mixed: fp64 residual, fp32 Arnoldi)
    I.val64 = DevMem(ctx, std::max<size_t>(nz, 1) * 8);
    if (nz) check(mpg_memcpy_h2d(ctx, I.val64.p, a.val, nz * 8), "h2d", ctx);
    const ModeTypes& ty = I.ty;
    const bool rounded_outer = a.mode != MPG_MODE_MIXED && a.mode != MPG_MODE_MIXED_HALF;
    if (rounded_outer) {
        DevMem f32(ctx, std::max<size_t>(nz, 1) * 4);
        I.cast(I.val64.p, MPG_F64, f32.p, MPG_F32, (int64_t)nz);
        if (ty.X == MPG_F64) {
            I.val_outer_own = DevMem(ctx, std::max<size_t>(nz, 1) * 8);
            I.cast(f32.p, MPG_F32, I.val_outer_own.p, MPG_F64, (int64_t)nz);
        } else {
            I.val_outer_own = std::move(f32);
        }
        I.val_outer = I.val_outer_own.p;
        I.val_inner = I.val_outer;  // the same matrix drives the Arnoldi cycle
    } else {
        I.val_outer = I.val64.p;
        I.val_inner_own = DevMem(ctx, std::max<size_t>(nz, 1) * dsize(ty.VI));
        if (ty.VI == MPG_F16) {
            // fp16 values, scaled per row by powers of two where a row's
            // magnitude falls outside fp16's range (mpg_csr_half_values);
            // with a.half_unscaled such a matrix fails here (MPG_ERR_RANGE)
            const bool scale = a.half_unscaled == 0;
            if (scale) I.row_exp = DevMem(ctx, (size_t)I.n + 64);
            check(mpg_csr_half_values(ctx, I.csr, I.val64.as<double>(), scale ? 1 : 0,
                                      I.val_inner_own.as<uint16_t>(), scale ? I.row_exp.as<int8_t>() : nullptr,
                                      I.half_stats),
                  "fp16 Arnoldi values", ctx);
            // a row whose own range exceeds fp16's (~2^39 below its largest
            // entry) loses its smallest entries to 0 even when scaled: not an
            // error (the plain cast's MPG_ERR_RANGE case), but said
            if (I.half_stats[1] > 0 && a.verbose)
                std::fprintf(stderr,
                             "mpgmres: mixed-half: %lld nonzero entries rounded to 0 in the fp16 Arnoldi copy "
                             "(rows spanning more than fp16's range; %lld rows scaled)\n",
                             (long long)I.half_stats[1], (long long)I.half_stats[0]);
        } else {
            I.cast(I.val64.p, MPG_F64, I.val_inner_own.p, ty.VI, (int64_t)nz);
        }
        I.val_inner = I.val_inner_own.p;
    }

    // Jacobi<P>(A): fp64 original A for P = double (baseline), else the A
    // converted to float (types.hpp:393-431 on SparseMatrix<P>)
    // (max row sum all-reduced across ranks: ||A||_inf of the whole matrix)
    I.scal = DevMem(ctx, 64);
    if (a.prec == MPG_PREC_JACOBI) {
        I.diag = DevMem(ctx, (size_t)I.n * dsize(ty.P) + 16);
        double* rowmax = I.scal.as<double>() + 4;
        if (ty.P == MPG_F64) {
            check(mpg_jacobi_rowmax_f64(ctx, I.csr, I.val64.as<double>(), rowmax), "jacobi", ctx);
            if (comm) comm->allreduce_max(rowmax, 1, I.stream());
            check(mpg_jacobi_diag_f64(ctx, I.csr, I.val64.as<double>(), rowmax, I.diag.as<double>()), "jacobi", ctx);
        } else {
            DevMem f32(ctx, std::max<size_t>(nz, 1) * 4);
            I.cast(I.val64.p, MPG_F64, f32.p, MPG_F32, (int64_t)nz);
            check(mpg_jacobi_rowmax_f32(ctx, I.csr, f32.as<float>(), rowmax), "jacobi", ctx);
            if (comm) comm->allreduce_max(rowmax, 1, I.stream());
            check(mpg_jacobi_diag_f32(ctx, I.csr, f32.as<float>(), rowmax, I.diag.as<float>()), "jacobi", ctx);
            check(mpg_ctx_sync(ctx), "sync", ctx);
        }
    }

    // ILU(0) of the fp64 A in the preconditioner precision (gmres_perf_test.cpp:70-79, 140-149)
    if (ilu) check(mpg_ilu0_create(ctx, I.csr, I.val64.as<double>(), ty.P == MPG_F64 ? 0 : 1, &I.ilu), "ilu0", ctx);

    // b (outer type), x = 0 (outer type, with halo tail)
    DevMem b64(ctx, (size_t)I.n * 8 + 8);
    check(mpg_memcpy_h2d(ctx, b64.p, a.b, (size_t)I.n * 8), "h2d", ctx);
    if (ty.X == MPG_F64) {
        I.b = std::move(b64);
    } else {
        I.b = DevMem(ctx, (size_t)I.n * 4 + 8);
        I.cast(b64.p, MPG_F64, I.b.p, MPG_F32, I.n);
    }
    I.x = DevMem(ctx, (size_t)(I.front + I.n_ext) * dsize(ty.X) + 64);
    I.xp = static_cast<char*>(I.x.p) + (size_t)I.front * dsize(ty.X);

    // one-time norms of the drivers (gmres.cpp:51-58, 162-168)
    b_norm = I.nrm2(I.b.p, ty.X, I.n);
    {
        I.tmp_t = DevMem(ctx, (size_t)I.n * dsize(ty.T) + 64);
        I.cast(I.b.p, ty.X, I.tmp_t.p, ty.T, I.n);  // copy(b, w)
        if (ty.P != ty.T) {                             // typesafe_apply
            I.tmp_p = DevMem(ctx, (size_t)I.n * dsize(ty.P) + 64);
            I.cast(I.tmp_t.p, ty.T, I.tmp_p.p, ty.P, I.n);
        }
        void* wp = ty.P != ty.T ? I.tmp_p.p : I.tmp_t.p;
        if (a.prec == MPG_PREC_JACOBI) {
            if (ty.P == MPG_F64)
                check(mpg_gdmv_f64(ctx, I.n, 1.0, I.diag.as<double>(), (double*)wp, 0.0, (double*)wp), "gdmv", ctx);
            else
                check(mpg_gdmv_f32(ctx, I.n, 1.0f, I.diag.as<float>(), (float*)wp, 0.0f, (float*)wp), "gdmv", ctx);
        }
        if (I.ilu) I.solve_ilu(wp);
        if (ty.P != ty.T) I.cast(I.tmp_p.p, ty.P, I.tmp_t.p, ty.T, I.n);
        minvb_norm = I.nrm2(I.tmp_t.p, ty.T, I.n);
    }
    // ||A||_F of the matrix the driver was given (A_single in mixed mode)
    {
        const bool mixed = !rounded_outer;
        const void* av = mixed ? nullptr : I.val_outer;
        int at = ty.X;
        DevMem f32;
        if (mixed) {  // A_single values (fp32) even in mixed-half mode
            f32 = DevMem(ctx, std::max<size_t>(nz, 1) * 4);
            I.cast(I.val64.p, MPG_F64, f32.p, MPG_F32, (int64_t)nz);
            av = f32.p;
            at = MPG_F32;
        }
        a_norm = I.nrm2(av, at, (int64_t)nz);
    }

    mpg_arnoldi_desc d{};
    d.n = I.n;
    d.n_ext = I.n_ext;
    d.m = I.m;
    d.orth = I.orth;
    d.vec_type = ty.T;
    d.outer_type = ty.X;
    d.prec_type = ty.P;
    d.inner_val = ty.VI;
    d.jacobi = a.prec == MPG_PREC_JACOBI;
    d.A = I.csr;
    d.val_outer = I.val_outer;
    d.val_inner = I.val_inner;
    d.diag = d.jacobi ? I.diag.p : nullptr;
    d.b = I.b.p;
    d.x = I.xp;
    d.spmv_format = a.spmv_format;
    d.n_front = n_front;
    // rows all in range: the unscaled kernels (no exponent loads, same bits)
    d.inner_row_exp = I.half_stats[0] > 0 ? I.row_exp.as<int8_t>() : nullptr;
    check(mpg_arnoldi_create(ctx, &d, &I.arn), "mpg_arnoldi_create", ctx);
    // fp32 Arnoldi: the reference's fp32 accumulation class on request (arnoldi.h)
    if (a.accum) check(mpg_arnoldi_set_accum(I.arn, MPG_ACCUM_F32), "mpg_arnoldi_set_accum", ctx);
    // ranks all-reduce per-workgroup partials in place: same count on every rank
    // (MPG_UNIFORM_GROUPS=1 gives one GPU the ranks' partial counts: a P = 1
    // RCCL solve then has the single-GPU solve's bits, tests/test_dist_gpu.py)
    const char* uenv = std::getenv("MPG_UNIFORM_GROUPS");
    if (comm || (uenv && *uenv == '1')) check(mpg_arnoldi_uniform_groups(I.arn), "uniform groups", ctx);
    I.report_len = mpg_arnoldi_report_len(I.arn);
    for (double*& r : I.rep) hipck(hipHostMalloc((void**)&r, (size_t)I.report_len * sizeof(double), 0), "hipHostMalloc");
    I.report_host = I.rep[0];
    for (hipEvent_t& e : I.report_ev) hipck(hipEventCreateWithFlags(&e, hipEventDisableTiming), "event");
    const char* qenv = std::getenv("MPG_PIPELINE");  // 0: read each cycle's report before the next launch
    I.pipeline = !(qenv && *qenv == '0');
    if (I.pipeline) I.x_snap = DevMem(ctx, I.x.bytes);

    // convergence strategy (gmres_perf_test.cpp:185-196)
    const size_t mm = (size_t)a.rlen, mr = (size_t)a.max_restarts;
    if (a.rtol == 0) conv_ = std::make_unique<Convergence<double, void>>(a.tol, mm, mr);
    else if (a.repeat_iter) conv_ = std::make_unique<RepeatIteration_Convergence<double, void>>(a.tol, a.rtol, mm, mr);
    else if (I.orthloss) {
        auto lo = std::make_unique<LostOrthogonalityFused>(a.tol, a.rtol, mm, mr);
        lo->step_loss = [this](size_t k) { return orth_loss_step(k); };
        I.loss_S = DevMem(ctx, (size_t)(mm + 1) * (mm + 1) * dsize(ty.T));
        I.loss_u = DevMem(ctx, (size_t)(mm + 2) * dsize(ty.T));
        conv_ = std::move(lo);
    } else conv_ = std::make_unique<RelPrecRes_Convergence<double, void>>(a.tol, a.rtol, mm, mr);
    conv_->total_iters = 0;
    breakdown.stop = a.stop_on_breakdown != 0;

    const char* env = std::getenv("MPG_NO_GRAPH");
    I.use_graph = !(env && *env == '1') && (!comm || comm->capturable());
    // Givens(k-1) is folded into SpMV(k) by default (MPG_FOLD_GIVENS=0: its
    // own launch): every SpMV workgroup sums the 256 ||w||^2 partials of the
    // 1024-thread CGS update itself (+1.9 us per SpMV, -4.6 us Givens launch
    // and its boundary: 19.3k vs 18.7k it/s on BAND-10M). Experiments, off:
    // MPG_COMBINE=1 (one GPU, CGS/CGSR) does last-arriver combines in the dots
    // and CGS launches: 15.1k it/s (1024 tickets on one counter serialise).
    // One GPU, by default (MPG_CGS_PARTIALS=0: off): every CGS workgroup sums
    // the 256 dots partials per column itself (8 branch-free loads per lane,
    // one latency) instead of the reduce launch: 21.6k vs 21.1k it/s on
    // BAND-10M (tools/ab_bench.sh, 4 interleaved runs each).
    const char* cenv = std::getenv("MPG_COMBINE");
    I.combine = !comm && cenv && *cenv == '1' && I.orth != MPG_ORTH_MGS && I.m <= mpg_arnoldi_fold_max_m();
    const char* penv = std::getenv("MPG_CGS_PARTIALS");
    // (CGSR's first pass also emits the next dots: its in-launch form is the
    // older runtime-count kernel, slower than reduce + update; on only with =1)
    // (ranks: the dots' partials are all-reduced in place first, so the
    // update still sums them itself -- no reduce launch per step)
    I.cgs_partials = !I.combine && I.orth != MPG_ORTH_MGS &&
                     (I.orth == MPG_ORTH_CGSR ? (penv && *penv == '1') : !(penv && *penv == '0'));
    // MPG_FUSE_DOTS=1: the panel dots inside the SELL SpMV launch (SellDots)
    const char* denv = std::getenv("MPG_FUSE_DOTS");
    // (=2: required -- an error where the storage does not support it; tests)
    I.fuse_dots = I.cgs_partials && I.orth == MPG_ORTH_CGS && denv && (*denv == '1' || *denv == '2');
    I.fuse_dots_required = I.fuse_dots && *denv == '2';
    // MPG_FUSE_DOTS_K0=K: fuse only the steps with k + 1 <= K (the first
    // steps, whose per-row basis loads are few; VERDICT r3 item 5's policy)
    const char* kenv = std::getenv("MPG_FUSE_DOTS_K0");
    I.fuse_dots_k0 = kenv && *kenv ? std::max(0, std::min(32, std::atoi(kenv))) : 32;
    // MPG_FOLD_GIVENS: 0 never, 1 always (m permitting), unset: where it pays
    // (mpg_arnoldi_fold_pays: up to ~4k SpMV workgroups)
    const char* fenv = std::getenv("MPG_FOLD_GIVENS");
    bool fold_on = fenv && *fenv ? *fenv != '0' : mpg_arnoldi_fold_pays(I.arn) != 0;
    if (comm && !(fenv && *fenv)) {
        // ranks of one solve must run the same collective sequence (a folding
        // rank all-reduces the ||w||^2 partials with the halo, a non-folding
        // one reduces + all-reduces one sum after it): every rank's row block
        // and SELL layout differ, so the fold is taken only if it pays on
        // EVERY rank (all-reduce max of "does not pay")
        double* flag = I.scal.as<double>() + 6;
        const double no = fold_on ? 0.0 : 1.0;
        check(mpg_memcpy_h2d(ctx, flag, &no, sizeof no), "h2d", ctx);
        comm->allreduce_max(flag, 1, I.stream());
        double any_no = 0;
        check(mpg_memcpy_d2h(ctx, &any_no, flag, sizeof any_no), "d2h", ctx);
        fold_on = any_no == 0.0;
    }
    I.fold = !I.combine && fold_on && I.m <= mpg_arnoldi_fold_max_m();
    check(mpg_ctx_sync(ctx), "sync", ctx);
    setup_seconds = std::chrono::duration<double>(clk::now() - t0).count();
    prologue();
    read_report(4);
    if (I.ilu) check_ilu_fault(I.ilu);
}

FusedEngine::~FusedEngine() = default;

void FusedEngine::sync() { check(mpg_ctx_sync(p_->ctx), "sync", p_->ctx); }

void FusedEngine::prologue() {
    Impl& I = *p_;
    if (I.comm) I.comm->halo(I.xp, (int)dsize(I.ty.X), I.stream());
    timed(1, [&] { check(mpg_arnoldi_prologue(I.arn), "prologue", I.ctx); });
    check(mpg_arnoldi_prologue(I.arn), "prologue", I.ctx);
    if (I.ilu) {  // w = M(T(r)) outside the kernel, then ||w||^2 again
        I.apply_ilu(mpg_arnoldi_wprev_dev(I.arn, 0));
        check(mpg_arnoldi_prologue_wnorm(I.arn), "prologue wnorm", I.ctx);
    }
    if (!I.comm) {  // the 3 column sums inside the finish launch (same bits)
        check(mpg_arnoldi_prologue_finish_partials(I.arn), "prologue_finish", I.ctx);
        return;
    }
    check(mpg_arnoldi_reduce(I.arn, 3), "reduce", I.ctx);
    I.comm->allreduce_sum(mpg_arnoldi_sums_dev(I.arn), 3, I.stream());
    check(mpg_arnoldi_prologue_finish(I.arn), "prologue_finish", I.ctx);
}

// ranks: sum the last kernel's per-workgroup partials across ranks in place
// (bit-identical on every rank), for a consumer that sums them itself
void FusedEngine::allreduce_partials(int ncols) {
    Impl& I = *p_;
    // the last launch's partials, [column][workgroup] (uniform workgroup
    // counts on every rank: mpg_arnoldi_uniform_groups), summed in place
    I.comm->allreduce_sum(mpg_arnoldi_partials_dev(I.arn), (int64_t)ncols * mpg_arnoldi_partials_count(I.arn),
                          I.stream());
}

void FusedEngine::reduce(int nc) {
    Impl& I = *p_;
    check(mpg_arnoldi_reduce(I.arn, nc), "reduce", I.ctx);
    if (I.comm) I.comm->allreduce_sum(mpg_arnoldi_sums_dev(I.arn), nc, I.stream());
}

// ||w||^2: one GPU folds the partial sums into the Givens kernel; ranks of a
// partitioned solve reduce + all-reduce first
void FusedEngine::givens(int k) {
    Impl& I = *p_;
    if (I.comm) {
        reduce(1);
        check(mpg_arnoldi_givens(I.arn, k), "givens", I.ctx);
    } else {
        check(mpg_arnoldi_givens_partials(I.arn, k), "givens", I.ctx);
    }
}

// Arnoldi step k. fold: the Givens step k-1 rides in this step's SpMV
// launch (k >= 1) and step k's own Givens is left to step k+1 / the caller.
void FusedEngine::step(int k, bool fold) {
    Impl& I = *p_;
    // SpMV and panel dots in one launch (one GPU, CGS with in-launch sums)
    if (I.fuse_dots && !I.comm && !I.ilu && I.orth == MPG_ORTH_CGS && I.cgs_partials && !I.combine &&
        k + 1 <= I.fuse_dots_k0) {
        timed(0, [&] { check(mpg_arnoldi_spmv(I.arn, k), "spmv", I.ctx); });
        const int st = mpg_arnoldi_spmv_dots(I.arn, k, fold && k > 0 ? 2 : 0);
        timed_end(0);
        if (st == MPG_OK) {
            check(mpg_arnoldi_cgs_partials(I.arn, k), "cgs", I.ctx);
            if (!fold) givens(k);
            return;
        }
        if (st != MPG_ERR_UNSUPPORTED || I.fuse_dots_required) check(st, "spmv+dots", I.ctx);
        I.fuse_dots = false;  // not available for this storage: the separate launches below
    }
    if (fold && k > 0) {
        if (I.comm)  // the ||w||^2 partials' all-reduce and the w_prev halo in one RCCL group
            I.comm->allreduce_sum_and_halo(mpg_arnoldi_partials_dev(I.arn), mpg_arnoldi_partials_count(I.arn),
                                           mpg_arnoldi_wprev_dev(I.arn, k), mpg_arnoldi_vec_bytes(I.arn),
                                           I.stream());
        timed(0, [&] { check(mpg_arnoldi_spmv(I.arn, k), "spmv", I.ctx); });
        check(mpg_arnoldi_givens_partials_spmv(I.arn, k), "givens+spmv", I.ctx);
        dup(0, [&] { check(mpg_arnoldi_givens_partials_spmv(I.arn, k), "givens+spmv", I.ctx); });
        timed_end(0);
    } else {
        if (I.comm) I.comm->halo(mpg_arnoldi_wprev_dev(I.arn, k), mpg_arnoldi_vec_bytes(I.arn), I.stream());
        timed(0, [&] { check(mpg_arnoldi_spmv(I.arn, k), "spmv", I.ctx); });
        check(mpg_arnoldi_spmv(I.arn, k), "spmv", I.ctx);
        dup(0, [&] { check(mpg_arnoldi_spmv(I.arn, k), "spmv", I.ctx); });
        timed_end(0);
    }
    if (I.ilu) I.apply_ilu(mpg_arnoldi_wprev_dev(I.arn, k + 1));  // w = M(A v_k)
    if (I.orth == MPG_ORTH_MGS) {
        check(mpg_arnoldi_dots(I.arn, k), "dots", I.ctx);
        if (!I.comm) {  // one GPU: each update sums the previous launch's partials itself
            for (int j = 0; j <= k; ++j) check(mpg_arnoldi_mgs_partials(I.arn, k, j), "mgs", I.ctx);
        } else {  // ranks: all-reduce the 256 partials in place, then the same in-launch sums
            for (int j = 0; j <= k; ++j) {
                allreduce_partials(1);
                check(mpg_arnoldi_mgs_partials(I.arn, k, j), "mgs", I.ctx);
            }
        }
    } else {
        // MPG_CGS_PARTIALS=1 (one GPU, k+1 <= 32): the CGS update sums the dots
        // partials itself; MPG_COMBINE=1: the dots' last workgroup writes the
        // sums and the last CGS pass's last workgroup runs the Givens step
        // (one GPU, plain CGS: up to 128 columns -- GMRES(100) -- the wide
        // update sums the one-launch panel dots' partials itself)
        const bool small = k + 1 <= 32 || (!I.comm && I.orth == MPG_ORTH_CGS && k + 1 <= mpg_arnoldi_partials_max_cols());
        if (!I.comm && !I.combine && I.orth == MPG_ORTH_CGSR && k + 1 > 32 &&
            k + 1 <= mpg_arnoldi_partials_max_cols()) {
            // CGSR at GMRES(100): dots, pass 0, dots again on the updated w, pass 1
            for (int pass = 0; pass < 2; ++pass) {
                check(mpg_arnoldi_dots(I.arn, k), "dots", I.ctx);
                check(mpg_arnoldi_cgsr_wide_pass(I.arn, k, pass), "cgsr", I.ctx);
            }
            if (!fold) givens(k);
            return;
        }
        const int last_pass = I.orth == MPG_ORTH_CGSR ? 1 : 0;
        bool pass0_done = false;
        if (I.combine && k + 1 <= 32) {
            check(mpg_arnoldi_dots_sums(I.arn, k), "dots+sums", I.ctx);
        } else {
            timed(3, [&] { check(mpg_arnoldi_dots(I.arn, k), "dots", I.ctx); });
            check(mpg_arnoldi_dots(I.arn, k), "dots", I.ctx);
            dup(3, [&] { check(mpg_arnoldi_dots(I.arn, k), "dots", I.ctx); });
            timed_end(3);
            if (I.cgs_partials && small) {
                if (I.comm) allreduce_partials(k + 1);
                timed(2, [&] { check(mpg_arnoldi_cgs_partials(I.arn, k), "cgs", I.ctx); });
                check(mpg_arnoldi_cgs_partials(I.arn, k), "cgs", I.ctx);
                // (the in-launch sums read the dots' partials, which the first
                // update's own partials replaced: the duplicate re-runs the
                // dots first, and time_phase_dup takes their share back out)
                dup(2, [&] {
                    check(mpg_arnoldi_dots(I.arn, k), "dots", I.ctx);
                    check(mpg_arnoldi_cgs_partials(I.arn, k), "cgs", I.ctx);
                    ++I.dup_with_dots;
                });
                timed_end(2);
                pass0_done = true;
            } else {
                reduce(k + 1);
            }
        }
        if (last_pass == 1) {
            if (!pass0_done) check(mpg_arnoldi_cgs(I.arn, k, 0), "cgs", I.ctx);
            reduce(k + 1);
        } else if (pass0_done) {
            if (!fold) givens(k);
            return;
        }
        if (I.combine) {
            check(mpg_arnoldi_cgs_givens(I.arn, k, last_pass), "cgs+givens", I.ctx);
            return;
        }
        timed(2, [&] { check(mpg_arnoldi_cgs(I.arn, k, last_pass), "cgs", I.ctx); });
        check(mpg_arnoldi_cgs(I.arn, k, last_pass), "cgs", I.ctx);
        dup(2, [&] { check(mpg_arnoldi_cgs(I.arn, k, last_pass), "cgs", I.ctx); });
        timed_end(2);
    }
    if (!fold) givens(k);
}

// v_{k+1} = T(w * (1/h_{k+1,k})) into V(:,k+1) right after step k, as the
// reference's add_vector does (Orthogonalization.hpp:51-60); the next SpMV
// forms and stores the same value again. Only LostOrthogonality needs it
// early: it reads the basis column after the newest one.
void FusedEngine::store_next_basis(int k) {
    Impl& I = *p_;
    int64_t ld = 0;
    void* V = const_cast<void*>(mpg_arnoldi_basis_dev(I.arn, &ld));
    const void* inv = mpg_arnoldi_inv_dev(I.arn);
    const void* w = mpg_arnoldi_wprev_dev(I.arn, k + 1);
    const size_t off = (size_t)(k + 1) * (size_t)ld;
    if (I.ty.T == MPG_F64)
        check(mpg_scal_copy_dev_f64(I.ctx, I.n, (const double*)inv, (const double*)w, (double*)V + off), "v_k+1", I.ctx);
    else
        check(mpg_scal_copy_dev_f32(I.ctx, I.n, (const float*)inv, (const float*)w, (float*)V + off), "v_k+1", I.ctx);
}

// LostOrthogonality_Convergence::check body (IterUtil.hpp:206-216) for
// check(k): u = V(:,0:k+1)^T V(:,k+1); s_col = S(0:k+1,k+1) = u - S(0:k+1,
// 0:k+1) u; returns dot(s_col, s_col). V(:,k+1) is the column after the
// newest basis vector: what an earlier cycle left there, or zeros.
double FusedEngine::orth_loss_step(size_t kk) {
    Impl& I = *p_;
    const int64_t k = (int64_t)kk, ldS = I.m + 1;
    int64_t ld = 0;
    const void* V = mpg_arnoldi_basis_dev(I.arn, &ld);
    if (I.ty.T == MPG_F64) {
        const double* Vd = (const double*)V;
        double *u = I.loss_u.as<double>(), *S = I.loss_S.as<double>(), *scol = S + (k + 1) * ldS;
        check(mpg_gemv_f64(I.ctx, 1, I.n, k + 1, 1.0, Vd, ld, Vd + (k + 1) * ld, 0.0, u), "gemv", I.ctx);
        check(mpg_copy_f64f64(I.ctx, k + 1, u, scol), "copy", I.ctx);
        check(mpg_gemv_f64(I.ctx, 0, k + 1, k + 1, -1.0, S, ldS, u, 1.0, scol), "gemv", I.ctx);
        double d = 0;
        check(mpg_dot_f64_host(I.ctx, k + 1, scol, scol, &d), "dot", I.ctx);
        return d;
    }
    const float* Vf = (const float*)V;
    float *u = I.loss_u.as<float>(), *S = I.loss_S.as<float>(), *scol = S + (k + 1) * ldS;
    check(mpg_gemv_f32(I.ctx, 1, I.n, k + 1, 1.0f, Vf, ld, Vf + (k + 1) * ld, 0.0f, u), "gemv", I.ctx);
    check(mpg_copy_f32f32(I.ctx, k + 1, u, scol), "copy", I.ctx);
    check(mpg_gemv_f32(I.ctx, 0, k + 1, k + 1, -1.0f, S, ldS, u, 1.0f, scol), "gemv", I.ctx);
    float d = 0;
    check(mpg_dot_f32_host(I.ctx, k + 1, scol, scol, &d), "dot", I.ctx);
    return (double)d;
}

void FusedEngine::update(int k) { check(mpg_arnoldi_update(p_->arn, k), "update", p_->ctx); }

void FusedEngine::read_report(int count) {
    Impl& I = *p_;
    hipck(hipMemcpyAsync(I.report_host, mpg_arnoldi_report_dev(I.arn), (size_t)count * sizeof(double),
                         hipMemcpyDeviceToHost, I.stream()),
          "report d2h");
    if (I.comm && I.comm->async()) {
        hipck(hipEventRecord(I.report_ev[0], I.stream()), "event record");
        wait_event(I.report_ev[0], (int64_t)cycles.size(), "the step collectives (halo send/recv, all-reduces)");
    }
    hipck(hipStreamSynchronize(I.stream()), "report sync");
}

// Host wait for the device. With an asynchronous transport (RCCL) a peer
// that never arrives would hang the rank in hipEventSynchronize, and the
// driver's 8-GPU run would only end at its time limit with no message: poll
// instead, check the communicator's asynchronous error, and after
// MPG_COMM_TIMEOUT_S seconds (default 120) without completion abort the
// communicator and fail with the rank, the restart cycle and the collectives
// in flight named (MPG_ERR_RCCL).
void FusedEngine::wait_event(hipEvent_t ev, int64_t cycle, const char* what) {
    Impl& I = *p_;
    if (!I.comm || !I.comm->async()) {
        hipck(hipEventSynchronize(ev), "wait");
        return;
    }
    const char* env = std::getenv("MPG_COMM_TIMEOUT_S");
    const double limit = env && *env ? std::atof(env) : 120.0;
    const auto t0 = clk::now();
    for (int polls = 0;; ++polls) {
        const hipError_t q = hipEventQuery(ev);
        if (q == hipSuccess) return;
        if (q != hipErrorNotReady) hipck(q, "event query");
        const double waited = std::chrono::duration<double>(clk::now() - t0).count();
        std::string why = I.comm->async_error();
        if (why.empty() && waited > limit)
            why = "no progress for " + std::to_string(waited) + " s (MPG_COMM_TIMEOUT_S " + std::to_string(limit) + ")";
        if (!why.empty()) {
            // a grace period first: work that still completes was slow, not
            // hung, and is not torn down under running kernels (the
            // communicator stays intact); otherwise abort it
            bool done_late = false;
            const bool async_err = waited <= limit;
            if (!async_err) {
                const auto g0 = clk::now();
                while (std::chrono::duration<double>(clk::now() - g0).count() < 5.0)
                    if (hipEventQuery(ev) == hipSuccess) {
                        done_late = true;
                        break;
                    }
            }
            const std::string where = "rank " + std::to_string(I.comm->rank()) + " of " +
                                      std::to_string(I.comm->size()) + ": restart cycle " + std::to_string(cycle) +
                                      ", waiting for " + what + ": " + why;
            if (done_late) {
                // slow but healthy (e.g. a huge or time-shared solve): say so
                // and go on; only an async error or a real hang ends the solve
                // 
                std::fprintf(stderr, "mpgmres: warning: %s; it completed within the 5 s grace period, continuing\n",
                             where.c_str());
                return;
            }
            I.comm->abort();
            throw StatusError(MPG_ERR_RCCL, where + "; communicator aborted");
        }
        // spin for the first ~ms (a cycle is ~1 ms), then back off
        if (polls > 2000) std::this_thread::sleep_for(std::chrono::microseconds(100));
    }
}

// steps 0..m-1, solution update with k = m, next residual prologue
void FusedEngine::cycle_program() {
    Impl& I = *p_;
    if (I.pipeline)  // the cycle may run past a stop decision: keep the x it started from
        hipck(hipMemcpyAsync(I.x_snap.p, I.x.p, I.x.bytes, hipMemcpyDeviceToDevice, I.stream()), "x snapshot");
    const bool fold = I.fold;
    for (int k = 0; k < I.m; ++k) step(k, fold);
    if (fold) givens(I.m - 1);
    update(I.m);
    prologue();
}

// check_initial on the report of the last prologue (gmres.cpp:171-190)
bool FusedEngine::check_start(int64_t i) {
    Impl& I = *p_;
    const double* r = I.report_host;
    double r_norm = r[0], beta = r[1], x_norm = r[2];
    double normalization;
    if (I.ty.single_scalars) normalization = (double)((float)b_norm + (float)a_norm * (float)x_norm);
    else normalization = b_norm + a_norm * x_norm;
    cycles.push_back(CycleRecord{r_norm, normalization, beta, minvb_norm});
    restarts = i;
    breakdown.cycle(r_norm, beta, i);
    switch (conv_->check_initial(r_norm, normalization, beta, minvb_norm)) {
        case iteration_converged: {
            const double rel = I.ty.single_scalars ? (double)(float)((float)beta / (float)minvb_norm)
                             : I.ty.T == MPG_F64 ? beta / minvb_norm
                                                 : (double)((float)beta / minvb_norm);
            out() << "Found solution with rel prec res norm = " << rel << " when k = 0 and i = " << i << std::endl;
            out() << "  total iterations = " << conv_->total_iterations() << std::endl;
            status = MPG_RESULT_CONVERGED;
            return true;
        }
        case iteration_aborted:
            out() << "Aborting after " << conv_->total_iterations() << " iterations" << std::endl;
            status = MPG_RESULT_ABORTED;
            return true;
        default: return false;
    }
}

// capture the cycle program once; if the runtime refuses (e.g. a collective
// that cannot be captured) fall back to eager launches for good
void FusedEngine::ensure_graph() {
    Impl& I = *p_;
    if (!I.use_graph || I.graph_exec) return;
    hipck(hipStreamBeginCapture(I.stream(), hipStreamCaptureModeThreadLocal), "begin capture");
    bool ok = true;
    try {
        cycle_program();
    } catch (const std::exception& ex) {
        ok = false;
        std::fprintf(stderr, "mpgmres: cycle capture failed (%s); running eagerly\n", ex.what());
    }
    hipGraph_t g = nullptr;
    const hipError_t ec = hipStreamEndCapture(I.stream(), &g);
    if (ok && ec == hipSuccess && hipGraphInstantiate(&I.graph_exec, g, nullptr, nullptr, 0) == hipSuccess) {
        I.graph = g;
    } else {
        if (g) (void)hipGraphDestroy(g);
        (void)hipGetLastError();
        I.use_graph = false;
    }
}

// the base strategy's per-step bookkeeping for one cycle's report
void FusedEngine::record_steps(int64_t i) {
    Impl& I = *p_;
    for (int k = 0; k < I.m; ++k) {
        const double res = I.report_host[4 + k];
        step_res.push_back(res);
        step_cycle.push_back((int)i);
        breakdown.step(res, (int64_t)step_res.size() - 1, i, (size_t)k);
        conv_->check((size_t)k + 1, res, minvb_norm);  // base strategy: counts, restarts at m
    }
}

// Graph cycles with the host round trip hidden: cycle i+1 is launched before
// cycle i's report is read, so the GPU never waits for the host's
// check_initial (≈ 38 us per cycle on BAND-10M: the report copy, the
// stream synchronisation and the next launch). A cycle launched past a stop
// decision (converged or aborted at check_initial) is undone by restoring the
// x it started from (it cannot have changed anything else the result reads);
// no cycle is ever left in flight when run() returns.
int FusedEngine::run_pipelined(int max_cycles, bool& done) {
    Impl& I = *p_;
    int64_t i = (int64_t)cycles.size();
    if (check_start(i)) {
        done = true;
        return 0;
    }
    if (max_cycles <= 0) return 0;
    // one replay of the captured cycle, then its report into rep[p], marked by report_ev[p]
    auto launch = [&](int p) {
        hipck(hipGraphLaunch(I.graph_exec, I.stream()), "graph launch");
        hipck(hipMemcpyAsync(I.rep[p], mpg_arnoldi_report_dev(I.arn), (size_t)I.report_len * sizeof(double),
                             hipMemcpyDeviceToHost, I.stream()),
              "report d2h");
        hipck(hipEventRecord(I.report_ev[p], I.stream()), "event record");
    };
    // the buffer not holding the report check_start just read
    int p = I.report_host == I.rep[0] ? 1 : 0, ran = 0;
    launch(p);
    for (;;) {
        const bool more = ran + 1 < max_cycles;
        if (more) launch(p ^ 1);  // speculative: decided by this cycle's report
        wait_event(I.report_ev[p], i, "the step collectives (halo send/recv, all-reduces)");
        if (I.ilu) check_ilu_fault(I.ilu);  // every apply of this cycle is valid
        I.report_host = I.rep[p];
        record_steps(i);
        ++ran;
        ++i;
        if (!more) return ran;
        if (check_start(i)) {  // stop: undo the cycle launched past it
            done = true;
            sync();
            hipck(hipMemcpyAsync(I.x.p, I.x_snap.p, I.x.bytes, hipMemcpyDeviceToDevice, I.stream()), "x restore");
            sync();
            return ran;
        }
        p ^= 1;
    }
}

// --stop-on-breakdown: the first non-finite value ends the solve with
// MPG_ERR_BREAKDOWN (nothing left in flight: a pipelined cycle may be)
int FusedEngine::run(int max_cycles, bool& done) {
    if (measured)
        throw StatusError(MPG_ERR_UNSUPPORTED,
                          "the engine ran measurement launches (mpg_engine_time_*), which change its Krylov basis, "
                          "Hessenberg column and iterate; create a new engine to continue a solve");
    try {
        return run_cycles(max_cycles, done);
    } catch (const BreakdownError& e) {
        (void)hipStreamSynchronize(p_->stream());
        done = true;
        status = MPG_RESULT_ERROR;
        throw StatusError(MPG_ERR_BREAKDOWN, e.what());
    }
}

int FusedEngine::run_cycles(int max_cycles, bool& done) {
    Impl& I = *p_;
    done = false;
    int ran = 0;
    const bool stepwise = conv_->needs_arnoldi_residual();
    if (!stepwise) ensure_graph();
    if (!stepwise && I.use_graph && I.pipeline) return run_pipelined(max_cycles, done);
    for (; ran < max_cycles; ++ran) {
        const int64_t i = (int64_t)cycles.size();
        if (check_start(i)) {
            done = true;
            return ran;
        }
        if (!stepwise) {
            if (I.use_graph) hipck(hipGraphLaunch(I.graph_exec, I.stream()), "graph launch");
            else cycle_program();
            read_report(I.report_len);
            if (I.ilu) check_ilu_fault(I.ilu);
            record_steps(i);
            continue;
        }
        // adaptive restart strategies: one host read of |s(k+1)| per step
        for (int k = 0;; ++k) {
            step(k, false);
            if (I.orthloss) store_next_basis(k);
            read_report(4 + k + 1);
            if (I.ilu) check_ilu_fault(I.ilu);
            const double res = I.report_host[4 + k];
            step_res.push_back(res);
            step_cycle.push_back((int)i);
            breakdown.step(res, (int64_t)step_res.size() - 1, i, (size_t)k);
            const iteration_action act = conv_->check((size_t)k + 1, res, minvb_norm);
            if (act == iteration_converged) {
                update(k + 1);
                out() << "Found solution with rel prec res norm = " << res / minvb_norm << " when k = " << k + 1
                      << " and i = " << i << std::endl;
                out() << "  total iterations = " << conv_->total_iterations() << std::endl;
                status = MPG_RESULT_CONVERGED;
                inner_k = k + 1;
                done = true;
                sync();
                return ran + 1;
            }
            if (act == iteration_aborted) {
                out() << "Aborting after " << conv_->total_iterations() << " iterations" << std::endl;
                status = MPG_RESULT_ABORTED;
                done = true;
                return ran + 1;
            }
            if (act == iteration_restart) {
                update(k + 1);
                prologue();
                read_report(4);
                if (I.ilu) check_ilu_fault(I.ilu);
                break;
            }
        }
    }
    return ran;
}

void FusedEngine::finish_report(mpg_solve_result* r) {
    Impl& I = *p_;
    const int n = I.n;
    // x and b widened to fp64 (DoBaselineProblem copies x_type / b_type to double)
    DevMem x64m(I.ctx, (size_t)(I.front + I.n_ext) * 8 + 8), r64(I.ctx, (size_t)n * 8 + 8), b64(I.ctx, (size_t)n * 8 + 8);
    double* x64 = x64m.as<double>() + I.front;  // row 0
    I.cast(I.xp, I.ty.X, x64, MPG_F64, n);
    I.cast(I.b.p, I.ty.X, b64.p, MPG_F64, n);
    if (r->x_out) check(mpg_memcpy_d2h(I.ctx, r->x_out, x64, (size_t)n * 8), "d2h", I.ctx);
    if (I.comm) I.comm->halo(x64, 8, I.stream());
    check(mpg_memcpy_d2d(I.ctx, r64.p, b64.p, (size_t)n * 8), "d2d", I.ctx);
    check(mpg_csr_spmv_f64(I.ctx, I.csr, -1.0, I.val64.as<double>(), x64, 1.0, r64.as<double>()), "spmv", I.ctx);
    r->res_norm = std::sqrt(I.dot_acc(r64.p, r64.p, MPG_F64, n));
    if (I.args.x_true) {
        DevMem xt(I.ctx, (size_t)n * 8 + 8);
        check(mpg_memcpy_h2d(I.ctx, xt.p, I.args.x_true, (size_t)n * 8), "h2d", I.ctx);
        check(mpg_axpy_f64(I.ctx, n, -1.0, xt.as<double>(), x64), "axpy", I.ctx);
        r->err_norm = std::sqrt(I.dot_acc(x64, x64, MPG_F64, n));
    }
}

double FusedEngine::phase_bytes(int which) const {
    const Impl& I = *p_;
    const double n = I.n, z = (double)I.nnz, sT = (double)dsize(I.ty.T), sX = (double)dsize(I.ty.X);
    const double sV = (double)dsize(I.ty.VI), sP = (double)dsize(I.ty.P);
    const double jac = I.args.prec == MPG_PREC_JACOBI ? 1.0 : 0.0;
    if (which == 0) {
        // SURVEY §8(d) B_spmv, the same for every storage: CSR values + int32
        // columns + row pointers, x read once, y written (the SELL-64 copy
        // moves fewer bytes; profiles/ PMC traffic shows the actual ones),
        // plus the Jacobi diagonal when the preconditioner is fused in
        return z * (sV + 4) + (n + 1) * 4 + 2 * n * sT + jac * n * sP;
    }
    if (which == 1) return z * (sX + 4) + (n + 1) * 4 + 3 * n * sX + n * sT + jac * n * sP;
    if (which == 4) {
        // the bytes the Arnoldi SpMV's own storage moves per launch: SELL-64
        // slots (column offset + value), slice offsets and step bases, or CSR
        // values + int32 columns + row pointers; then w_prev read once, v_k
        // stored to V(:,k), w written, the Jacobi diagonal when fused
        int32_t fmt = 0, W = 0, cb = 0, win = 0;
        int64_t stored = 0;
        check(mpg_arnoldi_spmv_layout(I.arn, &fmt, &W, &cb, &stored, &win), "layout", I.ctx);
        const double vec = 3 * n * sT + jac * n * sP;
        if (fmt == 2 || fmt == 3) return (double)mpg_arnoldi_sell_matrix_bytes(I.arn) + vec;  // (3: node blocks)
        return z * (sV + 4) + (n + 1) * 4 + vec;
    }
    if (which == 3) {
        // panel dots, mean over k: V(:,0..k) and w read
        double cols = 0;
        for (int k = 0; k < I.m; ++k) cols += (I.orth == MPG_ORTH_MGS ? 1 : k + 1);
        return (cols / I.m + 1) * n * sT;
    }
    // CGS update at mean k: read V(:,0..k), read + write w
    return ((I.m - 1) / 2.0 + 1) * n * sT + 2 * n * sT;
}

mpg_arnoldi_t FusedEngine::arnoldi() const { return p_->arn; }
const int64_t* FusedEngine::half_stats() const { return p_->half_stats; }
bool FusedEngine::givens_folded() const { return p_->fold; }

// Device-event time of one phase kernel in its place in the cycle: `reps`
// restart cycles run eagerly in cycle order, and at every launch of phase
// `which` the plain form of that kernel is first replayed kTimedReplays
// times back to back between one event pair (amortising the dispatch
// latency an event pair around a single launch would include), then the
// cycle's own launch follows. Replays of the non-idempotent CGS update leave
// the engine's state meaningless: time_phase is for measurement only.
constexpr int kTimedReplays = 10;

double FusedEngine::time_phase(int which, int reps, bool inplace, std::vector<double>* per_launch) {
    measured = true;
    Impl& I = *p_;
    if (inplace && which != 0) throw std::invalid_argument("in-place timing covers the Arnoldi SpMV only");
    I.timed = which;
    I.timed_inplace = inplace;
    I.marks.clear();
    for (int r = 0; r < reps; ++r) cycle_program();
    I.timed = -1;
    I.timed_inplace = false;
    hipck(hipStreamSynchronize(I.stream()), "sync");
    float total_ms = 0;
    const size_t pairs = I.marks.size() / 2;
    for (size_t q = 0; q < pairs; ++q) {
        float ms = 0;
        hipck(hipEventElapsedTime(&ms, I.marks[2 * q], I.marks[2 * q + 1]), "elapsed");
        total_ms += ms;
        if (per_launch) per_launch->push_back(inplace ? ms : ms / kTimedReplays);
    }
    for (hipEvent_t e : I.marks) (void)hipEventDestroy(e);
    I.marks.clear();
    return pairs ? total_ms / (pairs * (inplace ? 1 : kTimedReplays)) : 0.0;
}

// replay mode: kTimedReplays plain launches between one event pair ahead of
// the site's own launch; in-place mode (SpMV): arm the kernel events that
// the site's own launch records (mpg_arnoldi_time_next_spmv)
// An event-record node spliced into the capture in progress on `st`: the
// node depends on the capture's current tail and becomes the new tail. Same
// place in the graph as hipEventRecordWithFlags(hipEventRecordExternal),
// which the HIP runtime bundled with PyTorch (ROCm 7.0) rejects inside a
// capture ("invalid argument").
static void capture_event_record(hipStream_t st, hipEvent_t ev) {
    hipStreamCaptureStatus status = hipStreamCaptureStatusNone;
    unsigned long long id = 0;
    hipGraph_t graph = nullptr;
    const hipGraphNode_t* deps = nullptr;
    size_t ndeps = 0;
    hipck(hipStreamGetCaptureInfo_v2(st, &status, &id, &graph, &deps, &ndeps), "capture info");
    if (status != hipStreamCaptureStatusActive || !graph) throw StatusError(MPG_ERR_HIP, "timing mark outside a capture");
    hipGraphNode_t node = nullptr;
    hipck(hipGraphAddEventRecordNode(&node, graph, deps, ndeps, ev), "event record node");
    hipck(hipStreamUpdateCaptureDependencies(st, &node, 1, hipStreamSetCaptureDependencies), "capture tail");
}

// time_phase_dup: the site's own launch once more, right behind it (the same
// kernel, arguments and queue position)
template <class F>
void FusedEngine::dup(int phase, F&& launch) {
    Impl& I = *p_;
    if (I.dup_phase != phase) return;
    launch();
    ++I.dup_count;
}

template <class F>
void FusedEngine::timed(int phase, F&& launch) {
    Impl& I = *p_;
    if (I.timed != phase) return;
    if (I.stamps) {
        // wave stamps of the site's own launch (disarmed again by timed_end,
        // so a site that launches another form stores nothing)
        if (I.stamp_q < I.stamp_max)
            check(mpg_arnoldi_stamp_next(I.arn, I.stamps + 2 * I.stamp_cap * I.stamp_q++, I.stamp_cap), "stamp",
                  I.ctx);
        return;
    }
    if (I.timed_graph) {
        // an external event node ahead of the site's own launch (its pair
        // follows the launch: timed_end)
        hipEvent_t e0;
        hipck(hipEventCreate(&e0), "event");
        I.marks.push_back(e0);
        capture_event_record(I.stream(), e0);
        return;
    }
    hipEvent_t e[2];
    for (auto& x : e) hipck(hipEventCreate(&x), "event");
    if (I.timed_inplace) {
        check(mpg_arnoldi_time_next_spmv(I.arn, e[0], e[1]), "time spmv", I.ctx);
    } else {
        hipck(hipEventRecord(e[0], I.stream()), "record");
        for (int r = 0; r < kTimedReplays; ++r) launch();
        hipck(hipEventRecord(e[1], I.stream()), "record");
    }
    I.marks.push_back(e[0]);
    I.marks.push_back(e[1]);
}

void FusedEngine::timed_end(int phase) {
    Impl& I = *p_;
    if (I.timed != phase) return;
    if (I.stamps) {
        check(mpg_arnoldi_stamp_next(I.arn, nullptr, 0), "stamp", I.ctx);
        return;
    }
    if (!I.timed_graph) return;
    hipEvent_t e1;
    hipck(hipEventCreate(&e1), "event");
    I.marks.push_back(e1);
    capture_event_record(I.stream(), e1);
}

// A phase kernel timed inside graph replays of the cycle (which: 0 the
// Arnoldi SpMV, 2 the CGS update, 3 the panel dots): the cycle is captured
// once more with an external event node on each side of every launch of
// that phase, and that graph is replayed `reps` times (each replay
// re-records the events; they are read after it). Measurement only, like
// time_phase: the replays run without the host's restart checks.
double FusedEngine::time_phase_graph(int which, int reps, std::vector<double>* per_launch) {
    measured = true;
    Impl& I = *p_;
    if (!I.use_graph) throw StatusError(MPG_ERR_UNSUPPORTED, "the cycle is not captured (MPG_NO_GRAPH / eager ranks)");
    if (which != 0 && which != 2 && which != 3) throw std::invalid_argument("phase: 0 spmv, 2 cgs update, 3 dots");
    I.timed = which;
    I.timed_graph = true;
    I.marks.clear();
    hipGraph_t g = nullptr;
    hipGraphExec_t ge = nullptr;
    double total = 0;
    size_t count = 0;
    auto cleanup = [&] {
        I.timed = -1;
        I.timed_graph = false;
        if (ge) (void)hipGraphExecDestroy(ge);
        if (g) (void)hipGraphDestroy(g);
        for (hipEvent_t e : I.marks) (void)hipEventDestroy(e);
        I.marks.clear();
    };
    try {
        hipck(hipStreamBeginCapture(I.stream(), hipStreamCaptureModeThreadLocal), "begin capture");
        try {
            cycle_program();
        } catch (...) {
            (void)hipStreamEndCapture(I.stream(), &g);
            throw;
        }
        hipck(hipStreamEndCapture(I.stream(), &g), "end capture");
        hipck(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0), "instantiate");
        const size_t pairs = I.marks.size() / 2;
        for (int r = 0; r < reps; ++r) {
            hipck(hipGraphLaunch(ge, I.stream()), "graph launch");
            hipck(hipStreamSynchronize(I.stream()), "sync");
            for (size_t q = 0; q < pairs; ++q) {
                float ms = 0;
                hipck(hipEventElapsedTime(&ms, I.marks[2 * q], I.marks[2 * q + 1]), "elapsed");
                total += ms;
                ++count;
                if (per_launch) per_launch->push_back(ms);
            }
        }
    } catch (...) {
        cleanup();
        (void)hipGetLastError();
        throw;
    }
    cleanup();
    return count ? total / count : 0.0;
}

// A phase kernel's own duration inside graph replays of the cycle (which: 0
// the Arnoldi SpMV, 2 the one-panel CGS update, 3 the one-panel dots): the
// cycle is captured once more (after a memset node clearing the slots) with
// every launch of that phase storing its waves' wall-clock stamps
// (mpg_arnoldi_stamp_next); a launch lasts max(end) - min(start) over its
// waves -- the kernel alone, with no event packet in the queue around it.
// Launches of another form at the phase's site (the panel kernels past 32
// columns) store nothing and are skipped. Measurement only, like
// time_phase_graph.
double FusedEngine::time_phase_stamps(int which, int reps, std::vector<double>* per_launch) {
    measured = true;
    Impl& I = *p_;
    if (!I.use_graph) throw StatusError(MPG_ERR_UNSUPPORTED, "the cycle is not captured (MPG_NO_GRAPH / eager ranks)");
    if (which != 0 && which != 2 && which != 3) throw std::invalid_argument("phase: 0 spmv, 2 cgs update, 3 dots");
    const int64_t cap = mpg_arnoldi_stamp_waves(I.arn);
    if (cap < 1) throw StatusError(MPG_ERR_HIP, "no SpMV waves");
    const int64_t slots = (int64_t)(I.m + 2);
    const size_t bytes = (size_t)(2 * cap * slots) * sizeof(unsigned long long);
    DevMem buf(I.ctx, bytes);
    int dev = 0, khz = 0;
    hipck(hipGetDevice(&dev), "device");
    hipck(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev), "wall clock rate");
    if (khz <= 0) throw StatusError(MPG_ERR_HIP, "no wall clock rate");
    std::vector<unsigned long long> host(bytes / sizeof(unsigned long long));
    hipGraph_t g = nullptr;
    hipGraphExec_t ge = nullptr;
    double total = 0;
    size_t count = 0;
    I.timed = which;
    I.stamps = buf.as<unsigned long long>();
    I.stamp_cap = cap;
    I.stamp_q = 0;
    I.stamp_max = slots;
    auto cleanup = [&] {
        I.timed = -1;
        I.stamps = nullptr;
        I.stamp_q = I.stamp_max = 0;
        if (ge) (void)hipGraphExecDestroy(ge);
        if (g) (void)hipGraphDestroy(g);
    };
    try {
        hipck(hipStreamBeginCapture(I.stream(), hipStreamCaptureModeThreadLocal), "begin capture");
        try {
            hipck(hipMemsetAsync(buf.p, 0, bytes, I.stream()), "clear stamps");
            cycle_program();
        } catch (...) {
            (void)hipStreamEndCapture(I.stream(), &g);
            throw;
        }
        hipck(hipStreamEndCapture(I.stream(), &g), "end capture");
        hipck(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0), "instantiate");
        const int64_t launches = I.stamp_q;
        for (int r = 0; r < reps; ++r) {
            hipck(hipGraphLaunch(ge, I.stream()), "graph launch");
            hipck(hipStreamSynchronize(I.stream()), "sync");
            hipck(hipMemcpy(host.data(), buf.p, bytes, hipMemcpyDeviceToHost), "read stamps");
            for (int64_t q = 0; q < launches; ++q) {
                const unsigned long long* st = host.data() + 2 * cap * q;
                unsigned long long t0 = ~0ull, t1 = 0;
                for (int64_t wv = 0; wv < cap; ++wv) {
                    if (st[2 * wv] && st[2 * wv] < t0) t0 = st[2 * wv];
                    if (st[2 * wv + 1] > t1) t1 = st[2 * wv + 1];
                }
                if (t0 == ~0ull || t1 <= t0) continue;  // another form ran at the site
                const double ms = (double)(t1 - t0) / (double)khz;
                total += ms;
                ++count;
                if (per_launch) per_launch->push_back(ms);
            }
        }
    } catch (...) {
        cleanup();
        (void)hipGetLastError();
        throw;
    }
    cleanup();
    if (!count) throw StatusError(MPG_ERR_UNSUPPORTED, "no launch of the phase stored stamps");
    return total / count;
}

// A phase kernel's share of the stream inside graph replays of the cycle
// (which: 0 the Arnoldi SpMV in the form each step runs, 2 the CGS update, 3
// the panel dots), from HIP events around whole replays: the cycle is
// captured twice, as the solve runs it and with every launch of that phase
// issued twice in a row, and the graphs are replayed alternately; the
// difference of the replay times over the number of added launches is what
// one launch adds to the cycle -- the kernel plus its dispatch and release,
// with no marker packet near it (what rocprofv3's kernel duration measures).
// The duplicates run on the state the first launch left: the SpMV and the
// dots rewrite the same outputs; a second CGS update subtracts V h once more
// (the basis stays normalised; an update that sums the dots' partials itself
// gets the dots re-run ahead of it, whose own share is measured and taken
// out). Measurement only, like time_phase_graph.
double FusedEngine::time_phase_dup(int which, int reps, int64_t* launches) {
    measured = true;
    Impl& I = *p_;
    if (!I.use_graph) throw StatusError(MPG_ERR_UNSUPPORTED, "the cycle is not captured (MPG_NO_GRAPH / eager ranks)");
    if (which != 0 && which != 2 && which != 3) throw std::invalid_argument("phase: 0 spmv, 2 cgs update, 3 dots");
    hipGraph_t g[2] = {nullptr, nullptr};
    hipGraphExec_t ge[2] = {nullptr, nullptr};
    hipEvent_t ev[2] = {nullptr, nullptr};
    auto cleanup = [&] {
        I.dup_phase = -1;
        for (int q = 0; q < 2; ++q) {
            if (ge[q]) (void)hipGraphExecDestroy(ge[q]);
            if (g[q]) (void)hipGraphDestroy(g[q]);
            if (ev[q]) (void)hipEventDestroy(ev[q]);
        }
    };
    std::vector<double> diff;
    int64_t added = 0, with_dots = 0;
    try {
        for (int q = 0; q < 2; ++q) {
            I.dup_phase = q ? which : -1;
            I.dup_count = 0;
            I.dup_with_dots = 0;
            hipck(hipStreamBeginCapture(I.stream(), hipStreamCaptureModeThreadLocal), "begin capture");
            try {
                cycle_program();
            } catch (...) {
                (void)hipStreamEndCapture(I.stream(), &g[q]);
                throw;
            }
            hipck(hipStreamEndCapture(I.stream(), &g[q]), "end capture");
            hipck(hipGraphInstantiate(&ge[q], g[q], nullptr, nullptr, 0), "instantiate");
            if (q) {
                added = I.dup_count;
                with_dots = I.dup_with_dots;
            }
        }
        I.dup_phase = -1;
        if (added < 1) throw StatusError(MPG_ERR_UNSUPPORTED, "the cycle has no launch of that phase");
        for (hipEvent_t& e : ev) hipck(hipEventCreate(&e), "event");
        for (int q = 0; q < 2; ++q) hipck(hipGraphLaunch(ge[q], I.stream()), "graph launch");  // warm
        hipck(hipStreamSynchronize(I.stream()), "sync");
        for (int r = 0; r < reps; ++r) {
            float ms[2] = {0, 0};
            for (int q = 0; q < 2; ++q) {
                hipck(hipEventRecord(ev[0], I.stream()), "record");
                hipck(hipGraphLaunch(ge[q], I.stream()), "graph launch");
                hipck(hipEventRecord(ev[1], I.stream()), "record");
                hipck(hipEventSynchronize(ev[1]), "sync");
                hipck(hipEventElapsedTime(&ms[q], ev[0], ev[1]), "elapsed");
            }
            diff.push_back((double)(ms[1] - ms[0]) / (double)added);
        }
    } catch (...) {
        cleanup();
        (void)hipGetLastError();
        throw;
    }
    cleanup();
    if (launches) *launches = added;
    std::sort(diff.begin(), diff.end());
    double ms = diff[diff.size() / 2];
    if (with_dots) ms -= time_phase_dup(3, reps) * (double)with_dots / (double)added;
    return ms;
}

// ---------------------------------------------------------------- mpg_solve (fused)
void fill_history(const FusedEngine& e, mpg_solve_result* r) {
    r->status = e.status;
    r->restarts = e.restarts;
    r->inner_k = e.inner_k;
    r->total_iters = (int64_t)e.total_iters();
    r->minvb_norm = e.minvb_norm;
    r->setup_seconds = e.setup_seconds;
    r->n_cycles = (int64_t)e.cycles.size();
    for (size_t c = 0; c < e.cycles.size() && (int64_t)c < r->cycle_cap; ++c) {
        if (r->cyc_r_norm) r->cyc_r_norm[c] = e.cycles[c].r_norm;
        if (r->cyc_normalization) r->cyc_normalization[c] = e.cycles[c].normalization;
        if (r->cyc_beta) r->cyc_beta[c] = e.cycles[c].beta;
    }
    r->nonfinite_steps = e.breakdown.steps;
    r->nonfinite_cycles = e.breakdown.cycles;
    r->first_nonfinite_step = e.breakdown.first_step;
    r->n_steps = (int64_t)e.step_res.size();
    for (size_t s = 0; s < e.step_res.size() && (int64_t)s < r->step_cap; ++s) {
        if (r->step_res) r->step_res[s] = e.step_res[s];
        if (r->step_cycle) r->step_cycle[s] = e.step_cycle[s];
    }
}

int solve_fused(const mpg_solve_args& a, mpg_solve_result* r) {
    mpg_ctx_t ctx = current_ctx();
    const char* banner = a.mode == MPG_MODE_MIXED || a.mode == MPG_MODE_MIXED_HALF ? "Doing Mixed Precision test"
                                                                                     : "Doing Baseline test";
    out() << banner << std::endl;
    FusedEngine e(ctx, a);
    auto t1 = clk::now();
    bool done = false;
    while (!done) e.run(1 << 20, done);
    e.sync();
    const double gmres_s = std::chrono::duration<double>(clk::now() - t1).count();
    fill_history(e, r);
    r->gmres_seconds = gmres_s;
    e.finish_report(r);
    out() << "  ilu took " << (float)r->setup_seconds << "s; gmres took " << (float)gmres_s << "s" << std::endl;
    out() << "  resNorm = " << r->res_norm << "; errNorm = " << r->err_norm << std::endl;
    return 0;
}

}  // namespace mpg

// ---------------------------------------------------------------- engine C-ABI

extern "C" {

int mpg_engine_create(const mpg_solve_args* a, mpg_engine_t* out, char* err, int errlen) {
    if (!a || !out) return MPG_ERR_ARG;
    *out = nullptr;
    auto* e = new mpg_engine();
    try {
        mpg::set_quiet(!a->verbose);
        mpg::check(mpg_ctx_create(a->device, &e->ctx), "mpg_ctx_create");
        mpg::ScopedContext scope(e->ctx);
        e->eng = std::make_unique<mpg::FusedEngine>(e->ctx, *a);
    } catch (const std::exception& ex) {
        if (err && errlen > 0) std::snprintf(err, (size_t)errlen, "%s", ex.what());
        mpg_engine_destroy(e);
        return MPG_ERR_ARG;
    }
    *out = e;
    return MPG_OK;
}

int mpg_engine_run(mpg_engine_t e, int max_cycles, int* done) {
    if (!e || !e->eng) return MPG_ERR_ARG;
    e->last_error.clear();
    try {
        mpg::ScopedContext scope(e->ctx);
        bool d = false;
        int ran = e->eng->run(max_cycles, d);
        if (done) *done = d ? 1 : 0;
        return ran;
    } catch (const mpg::StatusError& ex) {
        e->last_error = ex.what();
        return ex.status;
    } catch (const std::exception& ex) {
        e->last_error = ex.what();
        return MPG_ERR_HIP;
    }
}

const char* mpg_engine_last_error(mpg_engine_t e) { return e ? e->last_error.c_str() : ""; }

int mpg_engine_sync(mpg_engine_t e) {
    if (!e) return MPG_ERR_ARG;
    return mpg_ctx_sync(e->ctx);
}

int64_t mpg_engine_total_iters(mpg_engine_t e) { return e && e->eng ? (int64_t)e->eng->total_iters() : -1; }

int mpg_engine_time_phase(mpg_engine_t e, int which, int reps, double* avg_ms) {
    if (!e || !e->eng || !avg_ms || reps < 1 || which < 0 || which > 3) return MPG_ERR_ARG;
    try {
        mpg::ScopedContext scope(e->ctx);
        *avg_ms = e->eng->time_phase(which, reps);
        return MPG_OK;
    } catch (const std::exception&) {
        return MPG_ERR_HIP;
    }
}

int mpg_engine_time_spmv_incycle(mpg_engine_t e, int cycles, double* avg_ms, double* per_launch_ms, int cap) {
    if (!e || !e->eng || !avg_ms || cycles < 1 || cap < 0 || (cap && !per_launch_ms)) return MPG_ERR_ARG;
    try {
        mpg::ScopedContext scope(e->ctx);
        std::vector<double> t;
        *avg_ms = e->eng->time_phase(0, cycles, true, &t);
        for (size_t i = 0; i < t.size() && (int)i < cap; ++i) per_launch_ms[i] = t[i];
        return (int)t.size();
    } catch (const std::exception&) {
        return MPG_ERR_HIP;
    }
}

int mpg_engine_time_phase_dup(mpg_engine_t e, int which, int reps, double* avg_ms, int64_t* launches) {
    if (!e || !e->eng || !avg_ms || reps < 1 || (which != 0 && which != 2 && which != 3)) return MPG_ERR_ARG;
    e->last_error.clear();
    try {
        mpg::ScopedContext scope(e->ctx);
        *avg_ms = e->eng->time_phase_dup(which, reps, launches);
        return MPG_OK;
    } catch (const mpg::StatusError& ex) {
        e->last_error = ex.what();
        return ex.status;
    } catch (const std::exception& ex) {
        e->last_error = ex.what();
        return MPG_ERR_HIP;
    }
}

int mpg_engine_time_phase_stamps(mpg_engine_t e, int which, int reps, double* avg_ms, double* per_launch_ms,
                                 int cap) {
    if (!e || !e->eng || !avg_ms || reps < 1 || cap < 0 || (cap && !per_launch_ms) ||
        (which != 0 && which != 2 && which != 3))
        return MPG_ERR_ARG;
    e->last_error.clear();
    try {
        mpg::ScopedContext scope(e->ctx);
        std::vector<double> t;
        *avg_ms = e->eng->time_phase_stamps(which, reps, &t);
        for (size_t i = 0; i < t.size() && (int)i < cap; ++i) per_launch_ms[i] = t[i];
        return (int)t.size();
    } catch (const mpg::StatusError& ex) {
        e->last_error = ex.what();
        return ex.status;
    } catch (const std::exception& ex) {
        e->last_error = ex.what();
        return MPG_ERR_HIP;
    }
}

int mpg_engine_time_phase_graph(mpg_engine_t e, int which, int reps, double* avg_ms, double* per_launch_ms,
                                int cap) {
    if (!e || !e->eng || !avg_ms || reps < 1 || cap < 0 || (cap && !per_launch_ms) ||
        (which != 0 && which != 2 && which != 3))
        return MPG_ERR_ARG;
    e->last_error.clear();
    try {
        mpg::ScopedContext scope(e->ctx);
        std::vector<double> t;
        *avg_ms = e->eng->time_phase_graph(which, reps, &t);
        for (size_t i = 0; i < t.size() && (int)i < cap; ++i) per_launch_ms[i] = t[i];
        return (int)t.size();
    } catch (const mpg::StatusError& ex) {
        e->last_error = ex.what();
        return ex.status;
    } catch (const std::exception& ex) {
        e->last_error = ex.what();
        return MPG_ERR_HIP;
    }
}

int mpg_engine_report(mpg_engine_t e, mpg_solve_result* r) {
    if (!e || !e->eng || !r) return MPG_ERR_ARG;
    try {
        mpg::ScopedContext scope(e->ctx);
        e->eng->sync();
        mpg::fill_history(*e->eng, r);
        e->eng->finish_report(r);
        return MPG_OK;
    } catch (const mpg::StatusError& ex) {
        std::snprintf(r->message, sizeof r->message, "%s", ex.what());
        return ex.status;
    } catch (const std::exception& ex) {
        std::snprintf(r->message, sizeof r->message, "%s", ex.what());
        return MPG_ERR_HIP;
    }
}

double mpg_engine_phase_bytes(mpg_engine_t e, int which) {
    return e && e->eng ? e->eng->phase_bytes(which) : 0.0;
}

int mpg_engine_spmv_layout(mpg_engine_t e, int32_t* format, int32_t* vec_width, int32_t* col_bytes,
                           int64_t* stored, int32_t* window) {
    if (!e || !e->eng) return MPG_ERR_ARG;
    return mpg_arnoldi_spmv_layout(e->eng->arnoldi(), format, vec_width, col_bytes, stored, window);
}

int mpg_engine_sell_columns(mpg_engine_t e, int32_t* form, int64_t* csr_slices, int64_t* implicit_slices) {
    if (!e || !e->eng) return MPG_ERR_ARG;
    return mpg_arnoldi_sell_columns(e->eng->arnoldi(), form, csr_slices, implicit_slices);
}

int mpg_engine_accum(mpg_engine_t e) {
    if (!e || !e->eng) return MPG_ERR_ARG;
    return mpg_arnoldi_accum(e->eng->arnoldi());
}

int mpg_engine_prologue_format(mpg_engine_t e) {
    if (!e || !e->eng) return MPG_ERR_ARG;
    return mpg_arnoldi_prologue_format(e->eng->arnoldi());
}

int mpg_engine_givens_folded(mpg_engine_t e) {
    if (!e || !e->eng) return MPG_ERR_ARG;
    return e->eng->givens_folded() ? 1 : 0;
}

int mpg_engine_comm_ranks(mpg_engine_t e) {
    if (!e || !e->eng) return MPG_ERR_ARG;
    return e->comm ? e->comm->transport_ranks() : 1;
}

int64_t mpg_engine_sell_shared_slices(mpg_engine_t e) {
    if (!e || !e->eng) return MPG_ERR_ARG;
    return mpg_arnoldi_sell_shared_slices(e->eng->arnoldi());
}

int mpg_engine_sell_sigma(mpg_engine_t e) {
    if (!e || !e->eng) return MPG_ERR_ARG;
    return mpg_arnoldi_sell_sigma(e->eng->arnoldi());
}

int mpg_engine_slices_per_wave(mpg_engine_t e) {
    if (!e || !e->eng) return MPG_ERR_ARG;
    return mpg_arnoldi_slices_per_wave(e->eng->arnoldi());
}

int mpg_engine_half_stats(mpg_engine_t e, int64_t* stats) {
    if (!e || !e->eng || !stats) return MPG_ERR_ARG;
    for (int q = 0; q < 4; ++q) stats[q] = e->eng->half_stats()[q];
    return MPG_OK;
}

int mpg_engine_destroy(mpg_engine_t e) {
    if (!e) return MPG_OK;
    if (e->ctx) {
        {
            mpg::ScopedContext scope(e->ctx);
            e->eng.reset();
            e->comm.reset();
        }
        mpg_ctx_destroy(e->ctx);
    }
    delete e;
    return MPG_OK;
}

}  // extern "C"
