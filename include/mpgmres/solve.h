/*
 * mpgmres solve C-ABI: one call = one restarted GMRES(m) solve of A x = b,
 * set up and reported the way the reference's perf-test driver does
 * (gmres_perf_test.cpp:53-182 DoBaselineProblem / DoMixedPrecisionProblem):
 * x0 = 0, timer around the GMRES call only, then resNorm = ||b - A x|| with
 * the original fp64 A and errNorm = ||x - x_true||.
 *
 * The same argument/result structs are used by the HIP path
 * (libmpgmres_host.so: mpg_solve) and by the CPU oracle under oracle/
 * (liboracle.so: oracle_solve), so parity tests can run both on one input.
 */
#ifndef MPGMRES_SOLVE_H
#define MPGMRES_SOLVE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* gmres_perf_test.cpp:31-36 test_mode_t, plus a new fp16-value mode */
typedef enum {
    MPG_MODE_MIXED = 0,       /* fp64 residual/update, fp32 Arnoldi (gmres_singleUpdate) */
    MPG_MODE_BASELINE = 1,    /* fp64 GMRES on double(float(A)) (gmres_baseline<d,d>) */
    MPG_MODE_SINGLE_PREC = 2, /* fp64 GMRES, fp32 preconditioner (gmres_baseline<d,f>) */
    MPG_MODE_SINGLE = 3,      /* fp32 GMRES (gmres_baseline<f,f>) */
    MPG_MODE_MIXED_HALF = 4   /* like MIXED, but the inner SpMV reads fp16 values (new) */
} mpg_mode_t;

/* gmres_perf_test.cpp:17-22 orth_t */
typedef enum { MPG_ORTH_CGS = 0, MPG_ORTH_MGS = 1, MPG_ORTH_CGSR = 2 } mpg_orth_t;

/* gmres_perf_test.cpp:24-29 prec_t (same numbering) */
typedef enum { MPG_PREC_ILU = 0, MPG_PREC_ILU_JACOBI = 1, MPG_PREC_JACOBI = 2, MPG_PREC_IDENTITY = 3 } mpg_prec_t;

typedef enum {
    MPG_ENGINE_SURFACE = 0,  /* generic driver over the kernels.hpp operator surface */
    MPG_ENGINE_FUSED = 1     /* fused Arnoldi kernels, device-side Givens, graph-captured cycles */
} mpg_engine_kind_t;

typedef enum { MPG_RESULT_CONVERGED = 1, MPG_RESULT_ABORTED = 3, MPG_RESULT_ERROR = -1 } mpg_result_status_t;

typedef struct {
    /* CSR matrix, 0-based int32 indices, fp64 values (host memory) */
    int32_t n;
    int64_t nnz;
    const int32_t* rowptr;
    const int32_t* col;
    const double* val;
    const double* b;       /* right-hand side (host, n) */
    const double* x_true;  /* for errNorm (host, n); may be NULL */
    int32_t mode, orth, prec, engine;
    int32_t rlen;          /* restart length m (--rlen) */
    double tol;            /* --tol */
    int64_t max_restarts;  /* --max-restarts */
    double rtol;           /* --rtol (0: base Convergence) */
    int32_t repeat_iter;   /* --repeat-iter */
    int32_t orthloss;      /* --orthloss */
    int32_t jacobi_steps;  /* --jacobi-steps */
    int32_t verbose;       /* print the reference's stdout lines */
    int32_t device;        /* HIP device (mpg_solve only) */
    int32_t threads;       /* host threads (oracle only; 0 = default) */
    int32_t spmv_format;   /* fused engine Arnoldi SpMV: 0 auto, 1 CSR row blocks, 2 SELL-64,
                              3 node blocks (3-dof nodes, 3 x 3 blocks) */
    int32_t half_unscaled; /* mode mixed-half: 0 = fp16 values scaled per row by powers of two where
                              a row's magnitude needs it (mpg_csr_half_values, capi.h); 1 = plain
                              cast: a value outside fp16's range fails the set-up (MPG_ERR_RANGE) */
    int32_t stop_on_breakdown; /* 1: stop at the first non-finite |s(k+1)| or restart residual and
                                  return MPG_ERR_BREAKDOWN (--stop-on-breakdown); 0: the reference's
                                  behaviour (Orthogonalization.hpp:56-59 divides unguarded and the
                                  restart loop runs on), the count is only reported */
    int32_t accum;         /* fp32 Arnoldi's accumulation class (MPG_ACCUM_F64 0 / MPG_ACCUM_F32 1,
                              arnoldi.h): 1 keeps every dot, norm, gemv and SpMV partial sum in fp32 --
                              the class of the reference's cblas_s* / mkl_sparse_s_mv (--accum f32);
                              fused engine only (the operator surface refuses it: MPG_ERR_UNSUPPORTED);
                              ignored by an fp64 Arnoldi and by the oracle */
} mpg_solve_args;

typedef struct {
    int32_t status;           /* mpg_result_status_t */
    int64_t restarts;         /* value of i when the solver returned */
    int64_t inner_k;          /* k when converged inside a cycle, else 0 */
    int64_t total_iters;
    double res_norm, err_norm;
    double gmres_seconds, setup_seconds;
    double minvb_norm;
    /* caller-provided outputs (may be NULL / zero capacity) */
    double* x_out;            /* n */
    int64_t cycle_cap;        /* capacity of the per-cycle arrays */
    int64_t n_cycles;         /* number of check_initial calls recorded */
    double* cyc_r_norm;       /* true residual norm at each restart */
    double* cyc_normalization;/* ||b|| + ||A||_F ||x|| */
    double* cyc_beta;         /* preconditioned residual norm */
    int64_t step_cap;
    int64_t n_steps;          /* number of check calls recorded */
    double* step_res;         /* |s(k+1)| per Arnoldi step */
    int32_t* step_cycle;      /* cycle index of each step */
    char message[256];        /* error text when status == MPG_RESULT_ERROR */
    /* breakdown report (not a reference decision: the solve runs as the
       reference's does unless args->stop_on_breakdown) */
    int64_t nonfinite_steps;  /* Arnoldi steps whose |s(k+1)| was NaN/Inf (h_{k+1,k} = 0 or
                                 non-finite makes the normalisation 1/h non-finite) */
    int64_t nonfinite_cycles; /* restarts whose true residual norm or beta was NaN/Inf */
    int64_t first_nonfinite_step; /* index of the first such step in the step history, -1: none */
} mpg_solve_result;

/* HIP path (libmpgmres_host.so). Returns 0 on success (result->status tells
 * converged/aborted), < 0 on error (result->message). */
int mpg_solve(const mpg_solve_args* args, mpg_solve_result* result);

/* ---- stepped access to the fused engine (benchmarks, multi-GPU ranks) ----
 * mpg_engine_create uploads the problem, builds the preconditioner, zeroes
 * x and runs the first residual prologue. mpg_engine_run advances the
 * restarted solve by up to `max_cycles` outer iterations exactly as
 * mpg_solve does (check_initial on the host once per cycle, graph-replayed
 * cycle on the device) and returns the number of cycles run; *done is set
 * when the solve converged or aborted. All timing is left to the caller. */
typedef struct mpg_engine* mpg_engine_t;
int mpg_engine_create(const mpg_solve_args* args, mpg_engine_t* out, char* err, int errlen);
int mpg_engine_run(mpg_engine_t e, int max_cycles, int* done);
/* the error text of the last mpg_engine_run that failed ("" otherwise) */
const char* mpg_engine_last_error(mpg_engine_t e);
int mpg_engine_sync(mpg_engine_t e);
int64_t mpg_engine_total_iters(mpg_engine_t e);
/* The solve so far as mpg_solve reports it: status, counts, the per-cycle
 * and per-step history, this rank's rows of x (result->x_out) and resNorm /
 * errNorm with the fp64 matrix (gmres_perf_test.cpp:104-117). Collective on a
 * row-partitioned engine (the norms are all-reduced). */
int mpg_engine_report(mpg_engine_t e, mpg_solve_result* result);
/* device-event timing of one phase kernel replayed `reps` times on the
 * engine's stream, back to back, averaged over the steps k = 0..m-1 of a
 * cycle (which: 0 = Arnoldi SpMV k_step_spmv, 1 = residual prologue,
 * 2 = CGS update, 3 = Gram-Schmidt panel dots) */
int mpg_engine_time_phase(mpg_engine_t e, int which, int reps, double* avg_ms);
/* the Arnoldi SpMV as it runs inside the cycle (Givens folded for k >= 1),
 * timed by each launch's own kernel events over `cycles` eager cycles:
 * returns the launch count (m per cycle), the mean in *avg_ms and up to
 * `cap` per-launch times in cycle order (measurement only: the cycles run
 * without the host's restart checks) */
int mpg_engine_time_spmv_incycle(mpg_engine_t e, int cycles, double* avg_ms, double* per_launch_ms, int cap);
/* a phase kernel's share of the stream inside graph replays of the cycle
 * (which: 0 the Arnoldi SpMV in the form each step runs, 2 the CGS update, 3
 * the panel dots): the cycle captured as the solve runs it and with every
 * launch of that phase issued twice in a row, replayed alternately `reps`
 * times between HIP events; *avg_ms = the median difference of the replay
 * times over the added launches (*launches, may be NULL) -- kernel plus
 * dispatch and release, as rocprofv3's kernel durations. MPG_ERR_UNSUPPORTED
 * when the engine runs eagerly. Measurement only. */
int mpg_engine_time_phase_dup(mpg_engine_t e, int which, int reps, double* avg_ms, int64_t* launches);
/* a phase kernel's own duration inside graph replays of the cycle (which: 2
 * the one-panel CGS update k_cgs_update_nc, 3 the one-panel dots k_dots_nc;
 * the SpMV stores no stamps): every launch of that phase in a captured cycle
 * stores its waves' wall-clock stamps (mpg_arnoldi_stamp_next), duration =
 * last wave end - first wave start; per-launch ms in cycle order, the launch
 * count returned (MPG_ERR_UNSUPPORTED when the engine runs eagerly or no
 * launch of the phase was a stamped form). Measurement only. */
int mpg_engine_time_phase_stamps(mpg_engine_t e, int which, int reps, double* avg_ms, double* per_launch_ms,
                                 int cap);
/* a phase kernel timed inside graph replays of the cycle (which: 0 the
 * Arnoldi SpMV, 2 the CGS update, 3 the panel dots): the cycle captured with
 * an event-record node on each side of every launch of that phase,
 * replayed `reps` times; per-launch times in cycle order (step k), the
 * launch count returned (m per replay for 0; MPG_ERR_UNSUPPORTED when the
 * engine runs eagerly). Measurement only, like the in-cycle timing above. */
int mpg_engine_time_phase_graph(mpg_engine_t e, int which, int reps, double* avg_ms, double* per_launch_ms,
                                int cap);
/* algorithmic bytes of one launch of phase `which` */
double mpg_engine_phase_bytes(mpg_engine_t e, int which);
/* storage of the engine's Arnoldi SpMV (mpg_arnoldi_spmv_layout) */
int mpg_engine_spmv_layout(mpg_engine_t e, int32_t* format, int32_t* vec_width, int32_t* col_bytes,
                           int64_t* stored, int32_t* window);
/* column form of the engine's SELL copy (mpg_arnoldi_sell_columns) */
int mpg_engine_sell_columns(mpg_engine_t e, int32_t* form, int64_t* csr_slices, int64_t* implicit_slices);
/* slices of the engine's SELL copy reading a shared column block (mpg_arnoldi_sell_shared_slices) */
int64_t mpg_engine_sell_shared_slices(mpg_engine_t e);
/* the engine's SELL-C-sigma window (mpg_arnoldi_sell_sigma; 0 unsorted) */
int mpg_engine_sell_sigma(mpg_engine_t e);
/* 1: the Givens step of step k-1 rides SpMV(k) (mpg_arnoldi_fold_pays); 0: its own launch */
int mpg_engine_givens_folded(mpg_engine_t e);
/* the accumulation class the engine's Arnoldi runs: MPG_ACCUM_F64 0 / MPG_ACCUM_F32 1 (arnoldi.h) */
int mpg_engine_accum(mpg_engine_t e);
/* the residual prologue's storage (mpg_arnoldi_prologue_format: 1 CSR, 2 SELL, 3 node blocks) */
int mpg_engine_prologue_format(mpg_engine_t e);
/* ranks of the engine's communicator as its transport reports them: 1 for a
 * single-GPU engine, ncclCommCount for an RCCL rank, the world size for the
 * host transport; < 0 on error */
int mpg_engine_comm_ranks(mpg_engine_t e);
/* slices per wave of the engine's SELL Arnoldi SpMV (mpg_arnoldi_slices_per_wave) */
int mpg_engine_slices_per_wave(mpg_engine_t e);
/* mode mixed-half: stats[4] of the fp16 cast (mpg_csr_half_values); zeros otherwise */
int mpg_engine_half_stats(mpg_engine_t e, int64_t* stats);
int mpg_engine_destroy(mpg_engine_t e);

/* process-wide counts of the operator-surface driver's cycle programs
 * (CycleProgram<Hip>, types_hip.hpp): cycles recorded into a graph, cycles
 * replayed from one, and recordings voided by a step that must read the
 * device (those cycles then run eagerly). Any pointer may be NULL. */
int mpg_cycle_program_counts(int64_t* recorded, int64_t* replayed, int64_t* voided);
/* the calling thread's counts of the operator surface's normalisation ride
 * (kernels_hip.cpp, MPG_SURFACE_FUSE bit 16): CGS updates that kept w's new
 * value apart, normalisations that rode the next SpMV, and those issued
 * separately instead (a call other than the SpMV came next). Any pointer
 * may be NULL. */
int mpg_surface_ride_counts(int64_t* redirects, int64_t* rides, int64_t* flushed);
/* The operator surface's spmv calls on this thread so far, by the storage
 * they ran on: node blocks (mpg_node_spmv_*), SELL-64, CSR. Pointers may be
 * NULL. */
int mpg_surface_spmv_counts(int64_t* node, int64_t* sell, int64_t* csr);
/* Host-value nrm2 calls of the operator surface on this thread answered from
 * the memo of the same vector's previous read (MPG_SURFACE_FUSE bit 32: no
 * device work issued through the surface in between, nothing deferred). */
int mpg_surface_host_norm_hits(int64_t* hits);
/* Host-value nrm2 calls of the operator surface on this thread that also
 * read the norm of the vector the preceding residual SpMV (alpha -1, beta 1)
 * took as input, in one launch (mpg_nrm2_pair_host; MPG_SURFACE_FUSE bit
 * 64): that vector's next host nrm2 is then a memo hit. */
int mpg_surface_host_norm_pairs(int64_t* pairs);

#ifdef __cplusplus
}
#endif
#endif /* MPGMRES_SOLVE_H */
