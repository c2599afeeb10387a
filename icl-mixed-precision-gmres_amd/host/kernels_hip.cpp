// `Hip` backend of the operator surface: explicit specialisations of every
// kernels.hpp template for Device = Hip, each a thin call into the C-ABI of
// libmpgmres_hip.so. Drop-in counterpart of kernels_mkl.cpp:73-352 and
// kernels_cuda.cpp:111-614 (same operators, same argument meaning).
//
// Host-value variants (`Type dot(x, y)`, `Type nrm2(x)`) synchronise the
// stream, like cuBLAS in host pointer mode; Scalar-result variants stay on
// the device (device pointer mode, kernels_cuda.cpp:142-150).
#include "types_hip.hpp"

#include <hip/hip_runtime_api.h>

#include <atomic>
#include <cstdlib>
#include <cstring>
#include <sstream>

#include "kernels.hpp"
#include "mpgmres/arnoldi.h"  // mpg_dtype_t
#include "mpgmres/solve.h"

namespace mpg {

namespace {
thread_local mpg_ctx_t tl_ctx = nullptr;
thread_local bool tl_owned = false;
// Device work this thread has issued through the surface: every operator
// takes its context from ctx_no_flush() (directly or through current_ctx()),
// which counts it, and a cycle program's graph replay counts itself
// (note_device_writes). The host-value nrm2 memo below is valid while the
// count has not moved.
thread_local uint64_t tl_writes = 0;

struct OwnedCtxReaper {
    ~OwnedCtxReaper() {
        // Process-exit path: the HIP runtime may already be torn down, so the
        // lazily created default context is intentionally leaked.
    }
};
}  // namespace

void check(int status, const char* what, mpg_ctx_t ctx) {
    if (status == MPG_OK) return;
    std::ostringstream os;
    os << "mpgmres: " << what << " failed: " << mpg_error_string(status);
    mpg_ctx_t c = ctx ? ctx : tl_ctx;
    if (c) {
        const char* e = mpg_ctx_last_error(c);
        if (e && *e) os << " (" << e << ")";
    }
    throw StatusError(status, os.str());
}

void check_ilu_fault(mpg_ilu_t ilu) {
    const int f = mpg_ilu_fault(ilu);
    if (f == 0) return;
    if (f < 0) check(MPG_ERR_HIP, "ILU fault word read");
    std::ostringstream os;
    os << "mpgmres: ILU triangular solve fault " << f << " (a row waited past its bound); the solve is invalid";
    throw StatusError(MPG_ERR_BREAKDOWN, os.str());
}

// A call that must read the device back cannot be part of a recorded cycle
// program: refuse it before it touches the stream (CycleProgram<Hip> then
// runs the steps eagerly).
void no_recording(const char* what) {
    if (tl_ctx && mpg_ctx_recording(tl_ctx))
        throw StatusError(MPG_ERR_UNSUPPORTED, std::string("mpgmres: ") + what + " cannot be recorded");
}

bool CycleProgram<Hip>::enabled() {
    const char* env = std::getenv("MPG_SURFACE_GRAPH");
    return !(env && *env == '0');
}

namespace {
std::atomic<int64_t> g_cycle_counts[3];
}
void CycleProgram<Hip>::count(int which) { g_cycle_counts[which].fetch_add(1, std::memory_order_relaxed); }

// MPG_SURFACE_SELL=0 keeps the operator surface's spmv on CSR
bool surface_sell_enabled() {
    const char* env = std::getenv("MPG_SURFACE_SELL");
    return !(env && *env == '0');
}
// MPG_SURFACE_NODE=0: never the node-block copy (SELL or CSR as before)
bool surface_node_enabled() {
    const char* env = std::getenv("MPG_SURFACE_NODE");
    return !(env && *env == '0');
}

// ---- scalar-op batching ----
// Consecutive scalar operators (rotg, rot, rot_vec, scalar copy/scal: the
// Givens step and the |s(k+1)| record of every Arnoldi step) are queued and
// issued as one mpg_scalar_program launch. Every other call reaches the
// device through current_ctx(), which issues the queue first, so the stream
// order of the calls is unchanged; so does every host read (to_host, fence).
// MPG_SURFACE_BATCH=0 issues each scalar call on its own.
namespace {
thread_local mpg_scalar_op tl_ops[MPG_SCALAR_PROGRAM_MAX];
thread_local int tl_nops = 0;
thread_local mpg_ctx_t tl_ops_ctx = nullptr;

bool batch_enabled() {
    const char* env = std::getenv("MPG_SURFACE_BATCH");
    return !(env && *env == '0');
}

mpg_ctx_t ctx_no_flush() {
    ++tl_writes;
    if (!tl_ctx) {
        const char* env = std::getenv("MPG_DEVICE");
        int dev = env ? std::atoi(env) : 0;
        check(mpg_ctx_create(dev, &tl_ctx), "mpg_ctx_create");
        tl_owned = true;
    }
    return tl_ctx;
}
}  // namespace

// ---- deferred stage 2 of reductions ----
// A reduction whose result goes to device memory (nrm2 / dot into a Scalar,
// gemv^T into a Vect with beta = 0) runs its stage 1 and leaves stage 2
// pending. If the very next call consumes that result (add_vector's
// scal_recip of the nrm2, MGS's naxpy of the dot, CGS's gemv of the gemv^T
// coefficients), it runs as one launch that sums the partials itself in
// stage 2's order (the same bits); any other call issues stage 2 first
// through current_ctx(). MPG_SURFACE_FUSE (bit mask below; 0: none) picks
// the pairs: MGS's dot -> naxpy is off by default, its 1024-thread consumer
// measured slower than stage 2 + naxpy (5.4k vs 5.7k it/s on BAND-10M).
namespace {
struct PendingReduction {
    int kind = 0;  // 0 none, 1 nrm2, 2 dot, 3 gemv^T
    bool f64 = false;
    mpg_ctx_t ctx = nullptr;
    int32_t nparts = 0;
    void* result = nullptr;
    int64_t cols = 0;    // gemv^T
    double alpha = 1.0;  // gemv^T
};
thread_local PendingReduction tl_red;

// MPG_SURFACE_FUSE: a bit mask of the fused pairs (1 nrm2 -> scal_recip,
// 2 dot -> naxpy, 4 gemv^T -> gemv, 8 gemv -> nrm2: the CGS update emits
// the ||w||^2 partials that the nrm2 of add_vector would compute, below;
// 16 scal_recip -> spmv: add_vector's normalisation rides the next SELL
// SpMV, below; 32 the host-value nrm2 memo, below; 64 the residual
// SpMV's input read with the next host nrm2, below); unset: kFuseDefault;
// 0: none
constexpr int kFuseDefault = 1 | 4 | 8 | 16 | 32 | 64;

// The ||y||^2 stage-1 partials a fused CGS gemv (mpg_gemv_n_from_t_nrm2_*)
// left in the context workspace: an nrm2 of exactly that y as the very
// next call takes them instead of launching its stage 1 (the same partials,
// bit for bit). Every other call reaches the device through current_ctx()
// (or queues a scalar op), which forgets them.
struct NormMemo {
    mpg_ctx_t ctx = nullptr;
    const void* y = nullptr;
    int64_t n = 0;
    bool f64 = false;
    int32_t nparts = 0;
};
thread_local NormMemo tl_norm;
int read_fuse_mask() {
    const char* env = std::getenv("MPG_SURFACE_FUSE");
    return env && *env ? std::atoi(env) & 0x7fffffff : kFuseDefault;
}
// read once when a ScopedContext opens (a solve), not on every call of the
// restart section, whose launches the host paces; -1: no scope open
thread_local int tl_fuse_mask = -1;
bool fuse_enabled(int bit) {
    const int mask = tl_fuse_mask >= 0 ? tl_fuse_mask : read_fuse_mask();
    return (mask & bit) != 0;
}
}  // namespace

// ---- add_vector's normalisation riding the next SpMV (round 5, bit 16) ----
// The CGS step of the reference (Orthogonalization.hpp:51-89, then
// gmres.cpp:213) is: gemv^T, gemv (w -= V h), nrm2(w) -> h(k+1,k),
// scal_recip -> V(:,k+1), Givens (scalar ops), spmv(A, V(:,k+1), w). The
// normalisation cannot ride that SpMV in place: the SpMV overwrites w while
// its other workgroups still gather w's neighbours. So the fused gemv writes
// w's new value to a scratch copy (the "redirect": w's value lives there),
// the nrm2 keeps its partials (NormMemo), the scal_recip is deferred, and the
// SpMV forms h, V(:,k+1) = T(1/h) w and A V(:,k+1) -> w in one launch
// (mpg_sell_spmv_norm_*, the same bits as the separate launches). Any other
// call through current_ctx() first issues what is deferred as the separate
// launches would have (scal_recip from the copy, then the copy back into
// w), so the semantics never change. tl_ride_score turns the redirect off on
// a context where the pattern keeps failing (CGSR's second pass reads w
// before the SpMV: two failures in a row switch it off; CGS fails only at the
// last step of a cycle). The score starts afresh in every ScopedContext
// (one per solve): a CGSR solve must not switch the ride off for the CGS
// solves that follow it on the same thread.
namespace {
struct Redirect {
    mpg_ctx_t ctx = nullptr;
    void* w = nullptr;  // the caller's w (nullptr: no redirect)
    void* s = nullptr;  // the scratch copy holding w's value
    int64_t n = 0;
    bool f64 = false;
};
thread_local Redirect tl_redir;
struct DeferredNorm {
    bool on = false;
    mpg_ctx_t ctx = nullptr;
    bool f64 = false;
    int32_t nparts = 0;
    void* h = nullptr;    // h(k+1,k)
    void* dst = nullptr;  // V(:,k+1)
    int64_t n = 0;
};
thread_local DeferredNorm tl_dnorm;
thread_local int tl_ride_score = 2;
struct Scratch {
    mpg_ctx_t ctx = nullptr;
    void* p = nullptr;
    size_t bytes = 0;
};
thread_local Scratch tl_scratch;
thread_local int64_t tl_ride_counts[3] = {0, 0, 0};  // redirects, rides, flushed
thread_local int64_t tl_spmv_counts[3] = {0, 0, 0};  // spmv calls on node blocks, SELL, CSR

// the scratch copy for w (kept per thread and context; never (re)allocated
// while the context's stream records a cycle program)
void* ride_scratch(mpg_ctx_t c, size_t bytes) {
    if (tl_scratch.p && tl_scratch.ctx == c && tl_scratch.bytes >= bytes) return tl_scratch.p;
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(static_cast<hipStream_t>(mpg_ctx_stream(c)), &cs) != hipSuccess ||
        cs != hipStreamCaptureStatusNone)
        return nullptr;
    if (tl_scratch.p) (void)mpg_free(tl_scratch.ctx == c ? c : nullptr, tl_scratch.p);
    tl_scratch = Scratch{};
    void* p = nullptr;
    if (mpg_malloc(c, bytes, &p) != MPG_OK) return nullptr;
    tl_scratch = Scratch{c, p, bytes};
    return p;
}
}  // namespace

// issue what the ride deferred, as the separate calls would have
void flush_ride() {
    if (tl_dnorm.on) {
        const DeferredNorm d = tl_dnorm;
        tl_dnorm.on = false;
        const int st = d.f64 ? mpg_scal_recip_nrm2_f64(d.ctx, d.nparts, (double*)d.h, d.n, (const double*)tl_redir.s,
                                                       (double*)d.dst)
                             : mpg_scal_recip_nrm2_f32(d.ctx, d.nparts, (float*)d.h, d.n, (const float*)tl_redir.s,
                                                       (float*)d.dst);
        check(st, "scal_recip (deferred)", d.ctx);
    }
    if (tl_redir.w) {
        const Redirect r = tl_redir;
        tl_redir.w = nullptr;
        const int st = r.f64 ? mpg_copy_f64f64(r.ctx, r.n, (const double*)r.s, (double*)r.w)
                             : mpg_copy_f32f32(r.ctx, r.n, (const float*)r.s, (float*)r.w);
        check(st, "copy (redirected w)", r.ctx);
        --tl_ride_score;
        ++tl_ride_counts[2];
    }
}

namespace {
bool ride_enabled() { return fuse_enabled(16) && tl_ride_score > 0; }
}  // namespace

void flush_pending_reduction() {
    if (!tl_red.kind) return;
    const PendingReduction r = tl_red;
    tl_red.kind = 0;
    int st = MPG_OK;
    if (r.kind == 1)
        st = r.f64 ? mpg_nrm2_finish_f64(r.ctx, r.nparts, (double*)r.result)
                   : mpg_nrm2_finish_f32(r.ctx, r.nparts, (float*)r.result);
    else if (r.kind == 2)
        st = r.f64 ? mpg_dot_finish_f64(r.ctx, r.nparts, (double*)r.result)
                   : mpg_dot_finish_f32(r.ctx, r.nparts, (float*)r.result);
    else
        st = r.f64 ? mpg_gemv_t_finish_f64(r.ctx, r.nparts, r.cols, r.alpha, 0.0, (double*)r.result)
                   : mpg_gemv_t_finish_f32(r.ctx, r.nparts, r.cols, (float)r.alpha, 0.f, (float*)r.result);
    check(st, "reduction stage 2", r.ctx);
}

void discard_pending_reduction() {
    tl_red.kind = 0;
    tl_norm.y = nullptr;
    tl_dnorm.on = false;
    tl_redir.w = nullptr;
}

// An elementwise call that writes none of the memo's y and runs no
// reduction (CGSR's axpy(1, corr, h) between its last gemv and the nrm2)
// keeps the memo: the partials in the workspace are still y's.
struct KeepNormMemo {
    NormMemo m;
    KeepNormMemo(const void* out, size_t bytes) : m(tl_norm) {
        const char* a = static_cast<const char*>(out);
        const char* y = static_cast<const char*>(m.y);
        if (m.y && a < y + m.n * (m.f64 ? 8 : 4) && y < a + bytes) m.y = nullptr;
    }
    void done() const { tl_norm = m; }
};

// the memo of the ||y||^2 partials, taken (cleared) when it is exactly y's
// on the current context and nothing is pending or queued; its nparts, or 0
static int32_t take_norm_memo(const void* y, int64_t n, bool f64) {
    const NormMemo m = tl_norm;
    tl_norm.y = nullptr;
    if (!m.y || m.y != y || m.n != n || m.f64 != f64 || m.ctx != tl_ctx || tl_red.kind || tl_nops) return 0;
    return m.nparts;
}

// the pending reduction of `kind` whose result is `result`, taken (cleared)
// when the caller will consume it; nullptr otherwise
static const PendingReduction* take_pending(int kind, bool f64, const void* result) {
    if (tl_red.kind != kind || tl_red.f64 != f64 || tl_red.result != result || tl_red.ctx != tl_ctx) return nullptr;
    static thread_local PendingReduction taken;
    taken = tl_red;
    tl_red.kind = 0;
    return &taken;
}

void flush_scalar_ops() {
    flush_ride();  // a queued program may read the h a deferred normalisation forms
    if (tl_nops == 0) return;
    const int n = tl_nops;
    tl_nops = 0;
    check(mpg_scalar_program(tl_ops_ctx, tl_ops, n), "scalar program", tl_ops_ctx);
}

void discard_scalar_ops() { tl_nops = 0; }

// true when queued (the caller issues the op itself otherwise)
bool queue_scalar_op(const mpg_scalar_op& op) {
    tl_norm.y = nullptr;
    if (!batch_enabled()) return false;
    if (tl_red.kind) flush_pending_reduction();
    mpg_ctx_t c = ctx_no_flush();
    if (tl_nops && tl_ops_ctx != c) flush_scalar_ops();
    tl_ops_ctx = c;
    tl_ops[tl_nops++] = op;
    if (tl_nops == MPG_SCALAR_PROGRAM_MAX) flush_scalar_ops();
    return true;
}

// The queued program for the SELL SpMV that comes next to carry in one
// extra workgroup of its launch (mpg_sell_spmv_prog_*): taken, emptying the
// queue, when it belongs to this context, no reduction stage is pending, and
// none of its operand cells overlaps the SpMV's x or y (so running it
// concurrently with the rows cannot change any value); otherwise the queue
// is issued as usual. MPG_SURFACE_RIDE=0: never taken. Returns the context.
mpg_ctx_t take_scalar_ops_for(const void* x, size_t xbytes, const void* y, size_t ybytes, mpg_scalar_op* ops,
                              int& nops) {
    nops = 0;
    const char* env = std::getenv("MPG_SURFACE_RIDE");
    bool ok = tl_nops > 0 && !tl_red.kind && tl_ops_ctx == ctx_no_flush() && !(env && *env == '0');
    auto clash = [&](const void* p, size_t bytes) {
        const char* a = static_cast<const char*>(p);
        const char* xa = static_cast<const char*>(x);
        const char* ya = static_cast<const char*>(y);
        return (a < xa + xbytes && xa < a + bytes) || (a < ya + ybytes && ya < a + bytes);
    };
    for (int i = 0; i < tl_nops && ok; ++i) {
        const mpg_scalar_op& o = tl_ops[i];
        const size_t es = o.f64 ? 8 : 4;
        for (int q = 0; q < 4 && ok; ++q) {
            if (!o.p[q]) continue;
            const size_t cells = o.op != MPG_SOP_ROT_VEC ? 1 : q == 0 ? (size_t)o.k + 1 : (size_t)o.k;
            ok = !clash(o.p[q], cells * es);
        }
    }
    if (!ok) return current_ctx();
    for (int i = 0; i < tl_nops; ++i) ops[i] = tl_ops[i];
    nops = tl_nops;
    tl_nops = 0;
    return tl_ops_ctx;
}

// add_vector's deferred normalisation and the next SpMV, on the SELL copy:
// when the SpMV is exactly spmv(A, V(:,k+1), w) for the deferred
// scal_recip's V(:,k+1) and the redirected w, take it (with the queued
// Givens program to ride workgroup 0 when none of its cells overlaps x or y;
// a program that would not ride makes everything issue separately). Returns
// true with the ride's context, nparts, h and the scratch copy.
bool take_ride(const void* x, const void* y, int64_t n, bool f64, mpg_scalar_op* ops, int& nops, mpg_ctx_t& c,
               int32_t& nparts, void*& h, const void*& w) {
    nops = 0;
    if (!tl_dnorm.on || !tl_redir.w || tl_dnorm.dst != x || tl_redir.w != y || tl_dnorm.n != n ||
        tl_redir.n != n || tl_dnorm.f64 != f64 || tl_redir.f64 != f64 || tl_dnorm.ctx != ctx_no_flush() ||
        tl_redir.ctx != tl_dnorm.ctx || tl_red.kind)
        return false;
    if (tl_nops) {
        mpg_ctx_t oc = take_scalar_ops_for(x, (size_t)n * (f64 ? 8 : 4), y, (size_t)n * (f64 ? 8 : 4), ops, nops);
        if (!nops || oc != tl_dnorm.ctx) return false;  // (current_ctx() issued everything: no ride)
    }
    c = tl_dnorm.ctx;
    nparts = tl_dnorm.nparts;
    h = tl_dnorm.h;
    w = tl_redir.s;
    tl_dnorm.on = false;
    tl_redir.w = nullptr;
    tl_ride_score = std::min(tl_ride_score + 1, 8);
    ++tl_ride_counts[1];
    return true;
}

// A node SpMV with more than kNodeNormRideGroups workgroups does not take
// add_vector's normalisation: every workgroup of the riding form re-sums the
// ||w||^2 partials and stores its rows of V(:,k+1), which at C4's size (71k
// workgroups) cost 342 us per launch against 296 us plain
// (profiles/r06_irr_pmc/), more than the separate scal_recip launch. The
// first such SpMV of a solve turns the redirect off for the rest of the
// scope, so the CGS gemv writes w itself again (no copy back).
constexpr int32_t kNodeNormRideGroups = 4096;
bool node_takes_norm_ride(mpg_node_t nd) {
    int32_t tiles = 0;
    if (mpg_node_layout(nd, nullptr, &tiles, nullptr, nullptr) != MPG_OK) return false;
    if ((tiles + 1) / 2 <= kNodeNormRideGroups) return true;
    tl_ride_score = 0;
    return false;
}

void note_device_writes() { ++tl_writes; }

// ---- host-value nrm2 memo (round 6, MPG_SURFACE_FUSE bit 32) ----
// The reference's restart section reads nrm2(w) to the host three times
// with nothing written in between when the preconditioner is the identity
// (r_norm, beta, first_vector's norm: gmres.cpp:176-196, Orthogonalization.hpp:
// 36-45), each a host round trip. A host-value nrm2 of the same vector on the
// same context, with no device work issued through the surface since the
// read and nothing deferred or queued, returns that read's value: the same
// deterministic sum of the same bits. Host-value reductions only read, so
// the context they take does not count as device work (read_ctx), unless
// taking it issued deferred work.
namespace {
struct HostNormMemo {
    const void* p = nullptr;
    int64_t n = 0;
    bool f64 = false;
    double v = 0;
    mpg_ctx_t ctx = nullptr;
    uint64_t token = 0;
};
thread_local HostNormMemo tl_hn[2];
thread_local int tl_hn_next = 0;
thread_local int64_t tl_hn_hits = 0;
bool nothing_deferred() { return !tl_dnorm.on && !tl_redir.w && tl_nops == 0 && tl_red.kind == 0; }
}  // namespace

bool host_norm_hit(const void* p, int64_t n, bool f64, double& v) {
    if (!fuse_enabled(32) || !tl_ctx || !nothing_deferred()) return false;
    for (const HostNormMemo& m : tl_hn)
        if (m.p == p && m.n == n && m.f64 == f64 && m.ctx == tl_ctx && m.token == tl_writes) {
            v = m.v;
            ++tl_hn_hits;
            return true;
        }
    return false;
}

void host_norm_store(const void* p, int64_t n, bool f64, double v) {
    tl_hn[tl_hn_next] = HostNormMemo{p, n, f64, v, tl_ctx, tl_writes};
    tl_hn_next ^= 1;
}

// ---- ||x|| read with ||w|| (round 6, MPG_SURFACE_FUSE bit 64) ----
// The restart section reads r_norm = ||w|| and, with nothing written in
// between when the preconditioner is the identity, x_norm = ||x|| of the x
// the residual SpMV (alpha -1, beta 1) has just read (gmres.cpp:173-196).
// That SpMV's input is remembered; the next host-value nrm2 that misses the
// memo reads both norms in one launch and one host round trip
// (mpg_nrm2_pair_host: each with the bits of its own read) and memoises
// both, so ||x|| is a memo hit when nothing was written since. Any surface
// deallocation forgets the remembered vector (it is never read after free).
namespace {
struct NormPrefetch {
    const void* p = nullptr;
    int64_t n = 0;
    bool f64 = false;
    mpg_ctx_t ctx = nullptr;
};
thread_local NormPrefetch tl_npf;
thread_local int64_t tl_npf_pairs = 0;
}  // namespace

void note_residual_spmv(const void* x, int64_t n, bool f64) {
    if (fuse_enabled(64) && fuse_enabled(32) && n > 0) tl_npf = NormPrefetch{x, n, f64, tl_ctx};
}
void forget_norm_prefetch() { tl_npf = NormPrefetch{}; }

mpg_ctx_t read_ctx();
bool host_norm_pair(const void* p, int64_t n, bool f64, double& v) {
    const NormPrefetch q = tl_npf;
    if (!q.p || q.p == p || q.n != n || !tl_ctx || q.ctx != tl_ctx || !fuse_enabled(64) || !fuse_enabled(32))
        return false;
    tl_npf = NormPrefetch{};
    double vq = 0;
    mpg_ctx_t c = read_ctx();
    const int st = mpg_nrm2_pair_host(c, n, f64 ? MPG_F64 : MPG_F32, p, q.f64 ? MPG_F64 : MPG_F32, q.p, &v, &vq);
    if (st == MPG_ERR_UNSUPPORTED) return false;
    check(st, "nrm2 (paired read)", c);
    host_norm_store(q.p, n, q.f64, vq);
    host_norm_store(p, n, f64, v);
    ++tl_npf_pairs;
    return true;
}

mpg_ctx_t current_ctx();
mpg_ctx_t read_ctx() {
    const bool deferred = !nothing_deferred();
    const uint64_t before = tl_writes;
    mpg_ctx_t c = current_ctx();
    if (!deferred) tl_writes = before;
    return c;
}

mpg_ctx_t current_ctx() {
    tl_norm.y = nullptr;
    flush_ride();
    if (tl_nops) flush_scalar_ops();
    if (tl_red.kind) flush_pending_reduction();
    return ctx_no_flush();
}

ScopedContext::ScopedContext(mpg_ctx_t ctx) : prev_(tl_ctx), prev_fuse_(tl_fuse_mask) {
    tl_norm.y = nullptr;
    flush_ride();
    if (tl_nops) flush_scalar_ops();
    if (tl_red.kind) flush_pending_reduction();
    tl_ctx = ctx;
    tl_ride_score = 2;  // (what the ride learned belongs to the previous scope's solve)
    tl_hn[0] = tl_hn[1] = HostNormMemo{};  // (so does the host-value nrm2 memo)
    tl_npf = NormPrefetch{};
    tl_fuse_mask = read_fuse_mask();
}
ScopedContext::~ScopedContext() {
    // the queue and a pending stage 2 belong to this scope's context; a
    // failure here has already been reported by the call that follows it,
    // or the scope is unwinding
    try {
        flush_ride();
    } catch (...) {
    }
    if (tl_nops) {
        const int n = tl_nops;
        tl_nops = 0;
        (void)mpg_scalar_program(tl_ops_ctx, tl_ops, n);
    }
    if (tl_red.kind) {
        try {
            flush_pending_reduction();
        } catch (...) {
        }
    }
    tl_ctx = prev_;
    tl_fuse_mask = prev_fuse_;
}

void build_transpose(CsrStructure& s) {
    if (s.transposed) return;
    mpg_ctx_t C = current_ctx();
    auto t = std::make_shared<CsrStructure>();
    t->m = s.n;
    t->n = s.m;
    t->nnz = s.nnz;
    const size_t ib = sizeof(int) * ((size_t)s.n + 1), jb = sizeof(int) * (size_t)s.nnz;
    t->row_map = device_alloc<Hip>(ib);
    t->inds = device_alloc<Hip>(jb ? jb : sizeof(int));
    auto perm = device_alloc<Hip>(jb ? jb : sizeof(int));
    check(mpg_csr_transpose(C, s.m, s.n, s.nnz, static_cast<const int32_t*>(s.row_map.get()),
                            static_cast<const int32_t*>(s.inds.get()), static_cast<int32_t*>(t->row_map.get()),
                            static_cast<int32_t*>(t->inds.get()), static_cast<int32_t*>(perm.get())),
          "mpg_csr_transpose", C);
    std::vector<int32_t> rp_host((size_t)s.n + 1);
    Hip::to_host(rp_host.data(), t->row_map.get(), ib);
    mpg_csr_t csr = nullptr;
    check(mpg_csr_create(C, t->m, t->n, t->nnz, rp_host.data(), static_cast<const int32_t*>(t->row_map.get()),
                         static_cast<const int32_t*>(t->inds.get()), &csr),
          "mpg_csr_create (transpose)", C);
    t->csr = std::shared_ptr<mpg_csr>(csr, [](mpg_csr* p) { mpg_csr_destroy(p); });
    s.perm = std::move(perm);
    s.transposed = std::move(t);
}

void gather_entries(const CsrStructure& s, const void* vals, void* out, size_t elem_bytes) {
    mpg_ctx_t C = current_ctx();
    const auto* perm = static_cast<const int32_t*>(s.perm.get());
    check(elem_bytes == 8 ? mpg_gather_b64(C, s.nnz, perm, vals, out) : mpg_gather_b32(C, s.nnz, perm, vals, out),
          "gather (transpose values)", C);
}

}  // namespace mpg

using mpg::check;
using mpg::current_ctx;

// ---------------- device tag ----------------
void* Hip::allocate(size_t bytes) {
    void* p = nullptr;
    check(mpg_malloc(current_ctx(), bytes, &p), "mpg_malloc");
    return p;
}
void Hip::deallocate(void* p) {
    mpg::forget_norm_prefetch();
    if (p) mpg_free(current_ctx(), p);
}
void Hip::to_host(void* dst, const void* src, size_t bytes) {
    check(mpg_memcpy_d2h(current_ctx(), dst, src, bytes), "mpg_memcpy_d2h");
}
void Hip::to_device(void* dst, const void* src, size_t bytes) {
    check(mpg_memcpy_h2d(current_ctx(), dst, src, bytes), "mpg_memcpy_h2d");
}
void Hip::fence() { check(mpg_ctx_sync(current_ctx()), "mpg_ctx_sync"); }

#define C current_ctx()

// ---------------- copy ----------------
template <> void copy<double, double, Hip>(Vect<double, Hip> x, Vect<double, Hip> y) {
    assert(x.n() == y.n());
    check(mpg_copy_f64f64(C, x.n(), x.data(), y.data()), "copy");
}
template <> void copy<float, float, Hip>(Vect<float, Hip> x, Vect<float, Hip> y) {
    assert(x.n() == y.n());
    check(mpg_copy_f32f32(C, x.n(), x.data(), y.data()), "copy");
}
template <> void copy<double, float, Hip>(Vect<double, Hip> x, Vect<float, Hip> y) {
    assert(x.n() == y.n());
    check(mpg_copy_f64f32(C, x.n(), x.data(), y.data()), "copy");
}
template <> void copy<float, double, Hip>(Vect<float, Hip> x, Vect<double, Hip> y) {
    assert(x.n() == y.n());
    check(mpg_copy_f32f64(C, x.n(), x.data(), y.data()), "copy");
}
template <> void copy<double, double, Hip>(Scalar<double, Hip> x, Scalar<double, Hip> y) {
    if (mpg::queue_scalar_op(mpg_scalar_op{MPG_SOP_COPY, 1, 0, 0, 0.0, {x.data(), y.data(), nullptr, nullptr}})) return;
    check(mpg_copy_f64f64(C, 1, x.data(), y.data()), "copy");
}
template <> void copy<float, float, Hip>(Scalar<float, Hip> x, Scalar<float, Hip> y) {
    if (mpg::queue_scalar_op(mpg_scalar_op{MPG_SOP_COPY, 0, 0, 0, 0.0, {x.data(), y.data(), nullptr, nullptr}})) return;
    check(mpg_copy_f32f32(C, 1, x.data(), y.data()), "copy");
}
template <> void copy<double, float, Hip>(Scalar<double, Hip> x, Scalar<float, Hip> y) {
    check(mpg_copy_f64f32(C, 1, x.data(), y.data()), "copy");
}
template <> void copy<float, double, Hip>(Scalar<float, Hip> x, Scalar<double, Hip> y) {
    check(mpg_copy_f32f64(C, 1, x.data(), y.data()), "copy");
}

// ---------------- reductions ----------------
template <> double dot<double, Hip>(Vect<double, Hip> x, Vect<double, Hip> y) {
    assert(x.n() == y.n());
    double r;
    check(mpg_dot_f64_host(mpg::read_ctx(), x.n(), x.data(), y.data(), &r), "dot");
    return r;
}
template <> float dot<float, Hip>(Vect<float, Hip> x, Vect<float, Hip> y) {
    assert(x.n() == y.n());
    float r;
    check(mpg_dot_f32_host(mpg::read_ctx(), x.n(), x.data(), y.data(), &r), "dot");
    return r;
}
template <> void dot<double, Hip>(Vect<double, Hip> x, Vect<double, Hip> y, Scalar<double, Hip> r) {
    assert(x.n() == y.n());
    if (mpg::fuse_enabled(2) && x.n() > 0) {
        mpg_ctx_t c = C;
        int32_t np = 0;
        check(mpg_dot_partials_f64(c, x.n(), x.data(), y.data(), &np), "dot");
        mpg::tl_red = mpg::PendingReduction{2, true, c, np, r.data()};
        return;
    }
    check(mpg_dot_f64(C, x.n(), x.data(), y.data(), r.data()), "dot");
}
template <> void dot<float, Hip>(Vect<float, Hip> x, Vect<float, Hip> y, Scalar<float, Hip> r) {
    assert(x.n() == y.n());
    if (mpg::fuse_enabled(2) && x.n() > 0) {
        mpg_ctx_t c = C;
        int32_t np = 0;
        check(mpg_dot_partials_f32(c, x.n(), x.data(), y.data(), &np), "dot");
        mpg::tl_red = mpg::PendingReduction{2, false, c, np, r.data()};
        return;
    }
    check(mpg_dot_f32(C, x.n(), x.data(), y.data(), r.data()), "dot");
}
template <> double nrm2<double, Hip>(Vect<double, Hip> x) {
    double r;
    if (mpg::host_norm_hit(x.data(), (int64_t)x.n(), true, r)) return r;
    if (mpg::host_norm_pair(x.data(), (int64_t)x.n(), true, r)) return r;
    check(mpg_nrm2_f64_host(mpg::read_ctx(), x.n(), x.data(), &r), "nrm2");
    mpg::host_norm_store(x.data(), (int64_t)x.n(), true, r);
    return r;
}
template <> float nrm2<float, Hip>(Vect<float, Hip> x) {
    double m;
    if (mpg::host_norm_hit(x.data(), (int64_t)x.n(), false, m)) return (float)m;
    if (mpg::host_norm_pair(x.data(), (int64_t)x.n(), false, m)) return (float)m;
    float r;
    check(mpg_nrm2_f32_host(mpg::read_ctx(), x.n(), x.data(), &r), "nrm2");
    mpg::host_norm_store(x.data(), (int64_t)x.n(), false, r);
    return r;
}
template <> void nrm2<double, Hip>(Vect<double, Hip> x, Scalar<double, Hip> r) {
    if (mpg::fuse_enabled(1) && x.n() > 0) {
        if (const int32_t np = mpg::take_norm_memo(x.data(), (int64_t)x.n(), true)) {
            // the partials the CGS gemv just emitted for this x: no stage 1
            mpg::tl_red = mpg::PendingReduction{1, true, mpg::tl_ctx, np, r.data()};
            return;
        }
        mpg_ctx_t c = C;
        int32_t np = 0;
        check(mpg_nrm2_partials_f64(c, x.n(), x.data(), &np), "nrm2");
        mpg::tl_red = mpg::PendingReduction{1, true, c, np, r.data()};
        return;
    }
    check(mpg_nrm2_f64(C, x.n(), x.data(), r.data()), "nrm2");
}
template <> void nrm2<float, Hip>(Vect<float, Hip> x, Scalar<float, Hip> r) {
    if (mpg::fuse_enabled(1) && x.n() > 0) {
        if (const int32_t np = mpg::take_norm_memo(x.data(), (int64_t)x.n(), false)) {
            // the partials the CGS gemv just emitted for this x: no stage 1
            mpg::tl_red = mpg::PendingReduction{1, false, mpg::tl_ctx, np, r.data()};
            return;
        }
        mpg_ctx_t c = C;
        int32_t np = 0;
        check(mpg_nrm2_partials_f32(c, x.n(), x.data(), &np), "nrm2");
        mpg::tl_red = mpg::PendingReduction{1, false, c, np, r.data()};
        return;
    }
    check(mpg_nrm2_f32(C, x.n(), x.data(), r.data()), "nrm2");
}

// ---------------- axpy ----------------
template <> void axpy<double, Hip>(double a, Vect<double, Hip> x, Vect<double, Hip> y) {
    assert(x.n() == y.n());
    const mpg::KeepNormMemo keep(y.data(), y.n() * sizeof(double));
    check(mpg_axpy_f64(C, x.n(), a, x.data(), y.data()), "axpy");
    keep.done();
}
template <> void axpy<float, Hip>(float a, Vect<float, Hip> x, Vect<float, Hip> y) {
    assert(x.n() == y.n());
    const mpg::KeepNormMemo keep(y.data(), y.n() * sizeof(float));
    check(mpg_axpy_f32(C, x.n(), a, x.data(), y.data()), "axpy");
    keep.done();
}
template <> void axpy<double, Hip>(Scalar<double, Hip> a, Vect<double, Hip> x, Vect<double, Hip> y) {
    assert(x.n() == y.n());
    check(mpg_axpy_dev_f64(C, x.n(), a.data(), x.data(), y.data()), "axpy");
}
template <> void axpy<float, Hip>(Scalar<float, Hip> a, Vect<float, Hip> x, Vect<float, Hip> y) {
    assert(x.n() == y.n());
    check(mpg_axpy_dev_f32(C, x.n(), a.data(), x.data(), y.data()), "axpy");
}
template <> void naxpy<double, Hip>(Scalar<double, Hip> a, Vect<double, Hip> x, Vect<double, Hip> y) {
    assert(x.n() == y.n());
    if (const auto* p = mpg::take_pending(2, true, a.data())) {
        check(mpg_naxpy_dot_f64(p->ctx, p->nparts, a.data(), x.n(), x.data(), y.data()), "naxpy (dot)", p->ctx);
        return;
    }
    check(mpg_naxpy_dev_f64(C, x.n(), a.data(), x.data(), y.data()), "naxpy");
}
template <> void naxpy<float, Hip>(Scalar<float, Hip> a, Vect<float, Hip> x, Vect<float, Hip> y) {
    assert(x.n() == y.n());
    if (const auto* p = mpg::take_pending(2, false, a.data())) {
        check(mpg_naxpy_dot_f32(p->ctx, p->nparts, a.data(), x.n(), x.data(), y.data()), "naxpy (dot)", p->ctx);
        return;
    }
    check(mpg_naxpy_dev_f32(C, x.n(), a.data(), x.data(), y.data()), "naxpy");
}

// ---------------- scal ----------------
template <> void scal<double, Hip>(double a, Vect<double, Hip> x) {
    check(mpg_scal_f64(C, x.n(), a, x.data()), "scal");
}
template <> void scal<float, Hip>(float a, Vect<float, Hip> x) {
    check(mpg_scal_f32(C, x.n(), a, x.data()), "scal");
}
template <> void scal<double, Hip>(double a, Vect<double, Hip> x, Vect<double, Hip> y) {
    assert(x.n() == y.n());
    check(mpg_scal_copy_f64(C, x.n(), a, x.data(), y.data()), "scal");
}
template <> void scal<float, Hip>(float a, Vect<float, Hip> x, Vect<float, Hip> y) {
    assert(x.n() == y.n());
    check(mpg_scal_copy_f32(C, x.n(), a, x.data(), y.data()), "scal");
}
template <> void scal<double, Hip>(Scalar<double, Hip> a, Vect<double, Hip> x, Vect<double, Hip> y) {
    assert(x.n() == y.n());
    check(mpg_scal_copy_dev_f64(C, x.n(), a.data(), x.data(), y.data()), "scal");
}
template <> void scal<float, Hip>(Scalar<float, Hip> a, Vect<float, Hip> x, Vect<float, Hip> y) {
    assert(x.n() == y.n());
    check(mpg_scal_copy_dev_f32(C, x.n(), a.data(), x.data(), y.data()), "scal");
}
template <> void scal<double, Hip>(double a, Scalar<double, Hip> x, Scalar<double, Hip> y) {
    if (mpg::queue_scalar_op(mpg_scalar_op{MPG_SOP_SCAL, 1, 0, 0, (double)a, {x.data(), y.data(), nullptr, nullptr}})) return;
    check(mpg_scal_scalar_f64(C, a, x.data(), y.data()), "scal");
}
template <> void scal<float, Hip>(float a, Scalar<float, Hip> x, Scalar<float, Hip> y) {
    if (mpg::queue_scalar_op(mpg_scalar_op{MPG_SOP_SCAL, 0, 0, 0, (double)a, {x.data(), y.data(), nullptr, nullptr}})) return;
    check(mpg_scal_scalar_f32(C, a, x.data(), y.data()), "scal");
}
template <> void scal<double, Hip>(Scalar<double, Hip> a, Scalar<double, Hip> x, Scalar<double, Hip> y) {
    if (mpg::queue_scalar_op(mpg_scalar_op{MPG_SOP_SCAL_DEV, 1, 0, 0, 0.0, {x.data(), y.data(), a.data(), nullptr}})) return;
    check(mpg_scal_scalar_dev_f64(C, a.data(), x.data(), y.data()), "scal");
}
template <> void scal<float, Hip>(Scalar<float, Hip> a, Scalar<float, Hip> x, Scalar<float, Hip> y) {
    if (mpg::queue_scalar_op(mpg_scalar_op{MPG_SOP_SCAL_DEV, 0, 0, 0, 0.0, {x.data(), y.data(), a.data(), nullptr}})) return;
    check(mpg_scal_scalar_dev_f32(C, a.data(), x.data(), y.data()), "scal");
}

template <> void scal_recip<double, Hip>(Scalar<double, Hip> a, Vect<double, Hip> x, Vect<double, Hip> y) {
    assert(x.n() == y.n());
    if (const auto* p = mpg::take_pending(1, true, a.data())) {
        // x's value in the redirect's copy: deferred to ride the next SpMV
        if (mpg::defer_norm(p->ctx, p->nparts, a.data(), x.data(), y.data(), (int64_t)x.n(), true)) return;
        check(mpg_scal_recip_nrm2_f64(p->ctx, p->nparts, a.data(), x.n(), x.data(), y.data()), "scal_recip (nrm2)",
              p->ctx);
        return;
    }
    check(mpg_scal_recip_copy_dev_f64(C, x.n(), a.data(), x.data(), y.data()), "scal_recip");
}
template <> void scal_recip<float, Hip>(Scalar<float, Hip> a, Vect<float, Hip> x, Vect<float, Hip> y) {
    assert(x.n() == y.n());
    if (const auto* p = mpg::take_pending(1, false, a.data())) {
        // x's value in the redirect's copy: deferred to ride the next SpMV
        if (mpg::defer_norm(p->ctx, p->nparts, a.data(), x.data(), y.data(), (int64_t)x.n(), false)) return;
        check(mpg_scal_recip_nrm2_f32(p->ctx, p->nparts, a.data(), x.n(), x.data(), y.data()), "scal_recip (nrm2)",
              p->ctx);
        return;
    }
    check(mpg_scal_recip_copy_dev_f32(C, x.n(), a.data(), x.data(), y.data()), "scal_recip");
}

namespace mpg {
// add_vector's scal_recip(h, w, V(:,k+1)) when w is redirected and its
// nrm2 partials are pending: recorded, to ride the next SpMV
bool defer_norm(mpg_ctx_t c, int32_t nparts, void* h, const void* x, void* y, int64_t n, bool f64) {
    if (!tl_redir.w || tl_redir.w != x || tl_redir.n != n || tl_redir.f64 != f64 || tl_redir.ctx != c ||
        tl_dnorm.on)
        return false;
    tl_dnorm = DeferredNorm{true, c, f64, nparts, h, y, n};
    return true;
}
// the fused CGS gemv's output buffer: the scratch copy (and the redirect
// recorded) when the ride is on, else y itself
void* redirect_target(mpg_ctx_t c, void* y, int64_t n, bool f64) {
    if (!ride_enabled() || tl_redir.w || tl_dnorm.on || n < 1) return y;
    void* sp = ride_scratch(c, (size_t)n * (f64 ? 8 : 4));
    return sp ? sp : y;
}
void set_redirect(mpg_ctx_t c, void* w, void* sp, int64_t n, bool f64) {
    tl_redir = Redirect{c, w, sp, n, f64};
    ++tl_ride_counts[0];
}
}  // namespace mpg

extern "C" int mpg_surface_host_norm_hits(int64_t* hits) {
    if (hits) *hits = mpg::tl_hn_hits;
    return MPG_OK;
}

extern "C" int mpg_surface_host_norm_pairs(int64_t* pairs) {
    if (pairs) *pairs = mpg::tl_npf_pairs;
    return MPG_OK;
}

extern "C" int mpg_surface_spmv_counts(int64_t* node, int64_t* sell, int64_t* csr) {
    if (node) *node = mpg::tl_spmv_counts[0];
    if (sell) *sell = mpg::tl_spmv_counts[1];
    if (csr) *csr = mpg::tl_spmv_counts[2];
    return MPG_OK;
}

extern "C" int mpg_surface_ride_counts(int64_t* redirects, int64_t* rides, int64_t* flushed) {
    if (redirects) *redirects = mpg::tl_ride_counts[0];
    if (rides) *rides = mpg::tl_ride_counts[1];
    if (flushed) *flushed = mpg::tl_ride_counts[2];
    return MPG_OK;
}

// ---------------- fill ----------------
template <> void fill_strided<double, Hip>(double* x, size_t r, size_t c, size_t ld, double v) {
    check(mpg_fill_f64(C, x, r, c, ld, v), "fill");
}
template <> void fill_strided<float, Hip>(float* x, size_t r, size_t c, size_t ld, float v) {
    check(mpg_fill_f32(C, x, r, c, ld, v), "fill");
}

// ---------------- Givens ----------------
template <> void rotg<double, Hip>(Scalar<double, Hip> a, Scalar<double, Hip> b, Scalar<double, Hip> c,
                                   Scalar<double, Hip> s) {
    if (mpg::queue_scalar_op(mpg_scalar_op{MPG_SOP_ROTG, 1, 0, 0, 0.0, {a.data(), b.data(), c.data(), s.data()}})) return;
    check(mpg_rotg_f64(C, a.data(), b.data(), c.data(), s.data()), "rotg");
}
template <> void rotg<float, Hip>(Scalar<float, Hip> a, Scalar<float, Hip> b, Scalar<float, Hip> c,
                                   Scalar<float, Hip> s) {
    if (mpg::queue_scalar_op(mpg_scalar_op{MPG_SOP_ROTG, 0, 0, 0, 0.0, {a.data(), b.data(), c.data(), s.data()}})) return;
    check(mpg_rotg_f32(C, a.data(), b.data(), c.data(), s.data()), "rotg");
}
template <> void rot<double, Hip>(Scalar<double, Hip> a, Scalar<double, Hip> b, Scalar<double, Hip> c,
                                  Scalar<double, Hip> s) {
    if (mpg::queue_scalar_op(mpg_scalar_op{MPG_SOP_ROT, 1, 0, 0, 0.0, {a.data(), b.data(), c.data(), s.data()}})) return;
    check(mpg_rot_f64(C, a.data(), b.data(), c.data(), s.data()), "rot");
}
template <> void rot<float, Hip>(Scalar<float, Hip> a, Scalar<float, Hip> b, Scalar<float, Hip> c,
                                  Scalar<float, Hip> s) {
    if (mpg::queue_scalar_op(mpg_scalar_op{MPG_SOP_ROT, 0, 0, 0, 0.0, {a.data(), b.data(), c.data(), s.data()}})) return;
    check(mpg_rot_f32(C, a.data(), b.data(), c.data(), s.data()), "rot");
}
template <> void rot<double, Hip>(Vect<double, Hip> a, Vect<double, Hip> c, Vect<double, Hip> s) {
    if (c.n() == 0) return;
    if (mpg::queue_scalar_op(mpg_scalar_op{MPG_SOP_ROT_VEC, 1, (int32_t)c.n(), 0, 0.0, {a.data(), nullptr, c.data(), s.data()}})) return;
    check(mpg_rot_vec_f64(C, (int)c.n(), a.data(), c.data(), s.data()), "rot");
}
template <> void rot<float, Hip>(Vect<float, Hip> a, Vect<float, Hip> c, Vect<float, Hip> s) {
    if (c.n() == 0) return;
    if (mpg::queue_scalar_op(mpg_scalar_op{MPG_SOP_ROT_VEC, 0, (int32_t)c.n(), 0, 0.0, {a.data(), nullptr, c.data(), s.data()}})) return;
    check(mpg_rot_vec_f32(C, (int)c.n(), a.data(), c.data(), s.data()), "rot");
}

// ---------------- BLAS-2 ----------------
template <> void gemv<double, Hip>(double alpha, MultiVect<double, Hip> A, Vect<double, Hip> x, double beta,
                                   Vect<double, Hip> y) {
    assert(A.ncols() == x.n() && A.nrows() == y.n());
    if (A.transposed() && beta == double(0) && mpg::fuse_enabled(4) && y.n() > 0 && y.n() <= 32) {
        // stage 1 now, stage 2 pending (CGS: the gemv that follows consumes it)
        mpg_ctx_t c = C;
        int32_t np = 0;
        const int st = mpg_gemv_t_partials_f64(c, A.nrows_base(), A.ncols_base(), A.data(), A.stride(), x.data(), &np);
        if (st == MPG_OK) {
            mpg::tl_red = mpg::PendingReduction{3, true, c, np, y.data(), (int64_t)y.n(), (double)alpha};
            return;
        }
        if (st != MPG_ERR_UNSUPPORTED) check(st, "gemv^T", c);
    }
    if (!A.transposed()) {
        if (const auto* p = mpg::take_pending(3, true, x.data())) {
            const bool emit = mpg::fuse_enabled(8) && mpg::fuse_enabled(1) && y.n() > 0;
            int32_t nnp = 0;
            // the ride (bit 16): w's new value into the scratch copy
            double* out = emit && A.nrows_base() == (int64_t)y.n()
                           ? static_cast<double*>(mpg::redirect_target(p->ctx, y.data(), (int64_t)y.n(), true))
                           : y.data();
            const int st = p->cols != (int64_t)x.n() ? MPG_ERR_UNSUPPORTED
                           : out != y.data()
                               ? mpg_gemv_n_from_t_nrm2_out_f64(p->ctx, A.nrows_base(), A.ncols_base(), alpha, A.data(),
                                                                  A.stride(), p->nparts, (double)p->alpha, x.data(), beta,
                                                                  y.data(), out, &nnp)
                           : emit ? mpg_gemv_n_from_t_nrm2_f64(p->ctx, A.nrows_base(), A.ncols_base(), alpha, A.data(),
                                                                 A.stride(), p->nparts, (double)p->alpha, x.data(), beta,
                                                                 y.data(), &nnp)
                                  : mpg_gemv_n_from_t_f64(p->ctx, A.nrows_base(), A.ncols_base(), alpha, A.data(),
                                                            A.stride(), p->nparts, (double)p->alpha, x.data(), beta, y.data());
            if (st == MPG_OK) {
                if (emit && A.nrows_base() == (int64_t)y.n())
                    mpg::tl_norm = mpg::NormMemo{p->ctx, y.data(), (int64_t)y.n(), true, nnp};
                if (out != y.data()) mpg::set_redirect(p->ctx, y.data(), out, (int64_t)y.n(), true);
                return;
            }
            if (st != MPG_ERR_UNSUPPORTED) check(st, "gemv (gemv^T)", p->ctx);
            mpg::tl_red = *p;  // not fusable here: issue its stage 2 first (below, through C)
        }
    }
    check(mpg_gemv_f64(C, A.transposed() ? 1 : 0, A.nrows_base(), A.ncols_base(), alpha, A.data(), A.stride(),
                       x.data(), beta, y.data()),
          "gemv");
}
template <> void gemv<float, Hip>(float alpha, MultiVect<float, Hip> A, Vect<float, Hip> x, float beta,
                                  Vect<float, Hip> y) {
    assert(A.ncols() == x.n() && A.nrows() == y.n());
    if (A.transposed() && beta == float(0) && mpg::fuse_enabled(4) && y.n() > 0 && y.n() <= 32) {
        // stage 1 now, stage 2 pending (CGS: the gemv that follows consumes it)
        mpg_ctx_t c = C;
        int32_t np = 0;
        const int st = mpg_gemv_t_partials_f32(c, A.nrows_base(), A.ncols_base(), A.data(), A.stride(), x.data(), &np);
        if (st == MPG_OK) {
            mpg::tl_red = mpg::PendingReduction{3, false, c, np, y.data(), (int64_t)y.n(), (double)alpha};
            return;
        }
        if (st != MPG_ERR_UNSUPPORTED) check(st, "gemv^T", c);
    }
    if (!A.transposed()) {
        if (const auto* p = mpg::take_pending(3, false, x.data())) {
            const bool emit = mpg::fuse_enabled(8) && mpg::fuse_enabled(1) && y.n() > 0;
            int32_t nnp = 0;
            // the ride (bit 16): w's new value into the scratch copy
            float* out = emit && A.nrows_base() == (int64_t)y.n()
                           ? static_cast<float*>(mpg::redirect_target(p->ctx, y.data(), (int64_t)y.n(), false))
                           : y.data();
            const int st = p->cols != (int64_t)x.n() ? MPG_ERR_UNSUPPORTED
                           : out != y.data()
                               ? mpg_gemv_n_from_t_nrm2_out_f32(p->ctx, A.nrows_base(), A.ncols_base(), alpha, A.data(),
                                                                  A.stride(), p->nparts, (float)p->alpha, x.data(), beta,
                                                                  y.data(), out, &nnp)
                           : emit ? mpg_gemv_n_from_t_nrm2_f32(p->ctx, A.nrows_base(), A.ncols_base(), alpha, A.data(),
                                                                 A.stride(), p->nparts, (float)p->alpha, x.data(), beta,
                                                                 y.data(), &nnp)
                                  : mpg_gemv_n_from_t_f32(p->ctx, A.nrows_base(), A.ncols_base(), alpha, A.data(),
                                                            A.stride(), p->nparts, (float)p->alpha, x.data(), beta, y.data());
            if (st == MPG_OK) {
                if (emit && A.nrows_base() == (int64_t)y.n())
                    mpg::tl_norm = mpg::NormMemo{p->ctx, y.data(), (int64_t)y.n(), false, nnp};
                if (out != y.data()) mpg::set_redirect(p->ctx, y.data(), out, (int64_t)y.n(), false);
                return;
            }
            if (st != MPG_ERR_UNSUPPORTED) check(st, "gemv (gemv^T)", p->ctx);
            mpg::tl_red = *p;  // not fusable here: issue its stage 2 first (below, through C)
        }
    }
    check(mpg_gemv_f32(C, A.transposed() ? 1 : 0, A.nrows_base(), A.ncols_base(), alpha, A.data(), A.stride(),
                       x.data(), beta, y.data()),
          "gemv");
}
template <> void trsv<double, Hip>(const char* upper, MultiVect<double, Hip> A, Vect<double, Hip> x) {
    assert(A.nrows() == A.ncols() && A.ncols() == x.n());
    check(mpg_trsv_f64(C, *upper == 'U', A.transposed() ? 1 : 0, A.ncols(), A.data(), A.stride(), x.data()),
          "trsv");
}
template <> void trsv<float, Hip>(const char* upper, MultiVect<float, Hip> A, Vect<float, Hip> x) {
    assert(A.nrows() == A.ncols() && A.ncols() == x.n());
    check(mpg_trsv_f32(C, *upper == 'U', A.transposed() ? 1 : 0, A.ncols(), A.data(), A.stride(), x.data()),
          "trsv");
}

template <> void gdmv<double, Hip>(double alpha, Vect<double, Hip> d, Vect<double, Hip> x, double beta,
                                   Vect<double, Hip> y) {
    assert(d.n() == x.n() && d.n() == y.n());
    check(mpg_gdmv_f64(C, d.n(), alpha, d.data(), x.data(), beta, y.data()), "gdmv");
}
template <> void gdmv<float, Hip>(float alpha, Vect<float, Hip> d, Vect<float, Hip> x, float beta,
                                  Vect<float, Hip> y) {
    assert(d.n() == x.n() && d.n() == y.n());
    check(mpg_gdmv_f32(C, d.n(), alpha, d.data(), x.data(), beta, y.data()), "gdmv");
}

// ---------------- sparse ----------------
// A transposed matrix runs the same CSR-adaptive kernel on A^T's own CSR
// (SparseMatrix::set_transpose); nrows()/ncols() stay A's, as in the
// reference, so the extents swap here.
template <> void spmv<double, Hip>(double alpha, SparseMatrix<double, Hip> A, Vect<double, Hip> x, double beta,
                                   Vect<double, Hip> y) {
    assert(A.is_transposed() ? ((size_t)A.nrows() == x.n() && (size_t)A.ncols() == y.n())
                             : ((size_t)A.ncols() == x.n() && (size_t)A.nrows() == y.n()));
    if (alpha == double(-1) && beta == double(1)) mpg::note_residual_spmv(x.data(), (int64_t)x.n(), true);
    mpg_node_t nd = A.node();
    mpg_sell_t s = nd ? nullptr : A.sell();
    if (nd || s) {
        // node blocks (round 6) or SELL-64: the same rides -- add_vector's
        // normalisation and the previous step's Givens program in this launch
        ++mpg::tl_spmv_counts[nd ? 0 : 1];
        mpg_scalar_op ops[MPG_SCALAR_PROGRAM_MAX];
        int nops = 0;
        mpg_ctx_t c = nullptr;
        int32_t np = 0;
        void* h = nullptr;
        const void* w = nullptr;
        if (beta == double(0) && x.n() == y.n() && (!nd || mpg::node_takes_norm_ride(nd)) &&
            mpg::take_ride(x.data(), y.data(), (int64_t)x.n(), true, ops, nops, c, np, h, w)) {
            check(nd ? mpg_node_spmv_norm_f64(c, nd, np, static_cast<double*>(h), static_cast<const double*>(w), x.data(),
                                               alpha, y.data(), ops, nops)
                     : mpg_sell_spmv_norm_f64(c, s, np, static_cast<double*>(h), static_cast<const double*>(w), x.data(),
                                               alpha, y.data(), ops, nops),
                  "spmv (normalising)", c);
            return;
        }
        // (a deferred normalisation this SpMV does not take is issued first: it
        // writes w's value back and V(:,k+1), which the SpMV may read)
        mpg::flush_ride();
        c = mpg::take_scalar_ops_for(x.data(), x.n() * 8, y.data(), y.n() * 8, ops, nops);
        if (nd)
            check(nops ? mpg_node_spmv_prog_f64(c, nd, alpha, x.data(), beta, y.data(), ops, nops)
                       : mpg_node_spmv_f64(c, nd, alpha, x.data(), beta, y.data()),
                  "spmv (node blocks)");
        else
            check(nops ? mpg_sell_spmv_prog_f64(c, s, alpha, x.data(), beta, y.data(), ops, nops)
                       : mpg_sell_spmv_f64(c, s, alpha, x.data(), beta, y.data()),
                  "spmv");
    } else {
        check(mpg_csr_spmv_f64(C, A.applied_csr(), alpha, A.applied_vals(), x.data(), beta, y.data()), "spmv");
        ++mpg::tl_spmv_counts[2];
    }
}
template <> void spmv<float, Hip>(float alpha, SparseMatrix<float, Hip> A, Vect<float, Hip> x, float beta,
                                  Vect<float, Hip> y) {
    assert(A.is_transposed() ? ((size_t)A.nrows() == x.n() && (size_t)A.ncols() == y.n())
                             : ((size_t)A.ncols() == x.n() && (size_t)A.nrows() == y.n()));
    if (alpha == float(-1) && beta == float(1)) mpg::note_residual_spmv(x.data(), (int64_t)x.n(), false);
    mpg_node_t nd = A.node();
    mpg_sell_t s = nd ? nullptr : A.sell();
    if (nd || s) {
        // node blocks (round 6) or SELL-64: the same rides -- add_vector's
        // normalisation and the previous step's Givens program in this launch
        ++mpg::tl_spmv_counts[nd ? 0 : 1];
        mpg_scalar_op ops[MPG_SCALAR_PROGRAM_MAX];
        int nops = 0;
        mpg_ctx_t c = nullptr;
        int32_t np = 0;
        void* h = nullptr;
        const void* w = nullptr;
        if (beta == float(0) && x.n() == y.n() && (!nd || mpg::node_takes_norm_ride(nd)) &&
            mpg::take_ride(x.data(), y.data(), (int64_t)x.n(), false, ops, nops, c, np, h, w)) {
            check(nd ? mpg_node_spmv_norm_f32(c, nd, np, static_cast<float*>(h), static_cast<const float*>(w), x.data(),
                                               alpha, y.data(), ops, nops)
                     : mpg_sell_spmv_norm_f32(c, s, np, static_cast<float*>(h), static_cast<const float*>(w), x.data(),
                                               alpha, y.data(), ops, nops),
                  "spmv (normalising)", c);
            return;
        }
        // (a deferred normalisation this SpMV does not take is issued first: it
        // writes w's value back and V(:,k+1), which the SpMV may read)
        mpg::flush_ride();
        c = mpg::take_scalar_ops_for(x.data(), x.n() * 4, y.data(), y.n() * 4, ops, nops);
        if (nd)
            check(nops ? mpg_node_spmv_prog_f32(c, nd, alpha, x.data(), beta, y.data(), ops, nops)
                       : mpg_node_spmv_f32(c, nd, alpha, x.data(), beta, y.data()),
                  "spmv (node blocks)");
        else
            check(nops ? mpg_sell_spmv_prog_f32(c, s, alpha, x.data(), beta, y.data(), ops, nops)
                       : mpg_sell_spmv_f32(c, s, alpha, x.data(), beta, y.data()),
                  "spmv");
    } else {
        check(mpg_csr_spmv_f32(C, A.applied_csr(), alpha, A.applied_vals(), x.data(), beta, y.data()), "spmv");
        ++mpg::tl_spmv_counts[2];
    }
}
template <> void jacobi_diag<double, Hip>(SparseMatrix<double, Hip> A, Vect<double, Hip> d) {
    check(mpg_jacobi_setup_f64(C, A.csr(), A.vals_data(), d.data()), "jacobi setup");
}
template <> void jacobi_diag<float, Hip>(SparseMatrix<float, Hip> A, Vect<float, Hip> d) {
    check(mpg_jacobi_setup_f32(C, A.csr(), A.vals_data(), d.data()), "jacobi setup");
}

// ---- ILU(0) / ILU-Jacobi (kernels_mkl.cpp:355-506, kernels_cuda.cpp:617-791) ----
namespace {
template <class T>
ILU<T, Hip> make_ilu(SparseMatrix<double, Hip> A, int type) {
    mpg_ilu_t h = nullptr;
    check(mpg_ilu0_create(C, A.csr(), A.vals_data(), type, &h), "ilu0");
    return ILU<T, Hip>(std::shared_ptr<mpg_ilu>(h, [](mpg_ilu* p) { mpg_ilu_destroy(p); }), A.nrows(), A.nnz());
}
}  // namespace
template <> ILU<double, Hip> ilu0<double, Hip>(SparseMatrix<double, Hip> A) { return make_ilu<double>(A, 0); }
template <> ILU<float, Hip> ilu0<float, Hip>(SparseMatrix<double, Hip> A) { return make_ilu<float>(A, 1); }
template <> void ilusv<double, Hip>(ILU<double, Hip> ilu, Vect<double, Hip> x) {
    mpg::no_recording("ilusv (its fault check reads the device)");
    check(mpg_ilu_solve(C, ilu.handle(), x.data()), "ilusv");
    // a level-scheduled solve can fault (a bounded wait expired): read the
    // sticky fault word before anything consumes x (the serial chain never waits)
    if (mpg_ilu_solve_mode(ilu.handle()) != 3) mpg::check_ilu_fault(ilu.handle());
}
template <> void ilusv<float, Hip>(ILU<float, Hip> ilu, Vect<float, Hip> x) {
    mpg::no_recording("ilusv (its fault check reads the device)");
    check(mpg_ilu_solve(C, ilu.handle(), x.data()), "ilusv");
    // a level-scheduled solve can fault (a bounded wait expired): read the
    // sticky fault word before anything consumes x (the serial chain never waits)
    if (mpg_ilu_solve_mode(ilu.handle()) != 3) mpg::check_ilu_fault(ilu.handle());
}
template <> void ilusv_jacobi<double, Hip>(ILU_Jacobi<double, Hip> ilu, Vect<double, Hip> x) {
    check(mpg_ilu_jacobi_solve(C, ilu.handle(), ilu.steps(), x.data()), "ilusv_jacobi");
}
template <> void ilusv_jacobi<float, Hip>(ILU_Jacobi<float, Hip> ilu, Vect<float, Hip> x) {
    check(mpg_ilu_jacobi_solve(C, ilu.handle(), ilu.steps(), x.data()), "ilusv_jacobi");
}

#undef C

extern "C" int mpg_cycle_program_counts(int64_t* recorded, int64_t* replayed, int64_t* voided) {
    if (recorded) *recorded = mpg::g_cycle_counts[0].load();
    if (replayed) *replayed = mpg::g_cycle_counts[1].load();
    if (voided) *voided = mpg::g_cycle_counts[2].load();
    return MPG_OK;
}
