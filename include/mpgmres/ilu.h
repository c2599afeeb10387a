/*
 * mpgmres ILU(0) / ILU-Jacobi C-ABI (libmpgmres_hip.so) — the incomplete-LU
 * preconditioners of the reference on gfx950.
 *
 * Replaces:
 *   ilu0<T, Dev>(SparseMatrix<double, Dev>)   kernels.hpp:155-156; kernels_mkl.cpp:416-500;
 *                                             kernels_cuda.cpp:714-791 (csrilu02)
 *   ilusv<T, Dev>(ILU, Vect)                  kernels.hpp:168-169; kernels_mkl.cpp:355-384;
 *                                             kernels_cuda.cpp:617-711 (csrsv2, level policy)
 *   ilusv_jacobi<T, Dev>(ILU_Jacobi, Vect)    kernels.hpp:171-248; types.hpp:251-372
 *
 * Factorisation: the reference's ilu0_impl algorithm in fp64 (rows 1..n-1,
 * IKJ elimination by a sorted merge with the upper part of each pivot row,
 * pivots pushed to +-alpha, alpha = max_i sum_j |a_ij| * eps(T)), with the
 * pivot positions filled in (the MKL code allocates diag_inds and never
 * writes it, kernels_mkl.cpp:448). Factors are then rounded to T. One
 * wave64 per row, rows handed out in order by an atomic ticket, each row
 * waiting only on the rows it reads (sync-free): the same data-dependency
 * schedule cuSPARSE's level policy follows, with no host round trip.
 *
 * Triangular solves: unit-lower L then upper U, fp64 row sums rounded
 * once to T; x in, x out. Rows are level-scheduled and sync-free, with each
 * value its own ready flag (an internal buffer pre-filled with a NaN tag
 * the arithmetic never produces). Depth = the longest dependency chain of
 * the matrix (natural-order 3-D stencils: ~nx+ny+nz; banded matrices: n,
 * run by one workgroup serially — or use ILU-Jacobi).
 *
 * ILU-Jacobi: `steps` Jacobi sweeps per factor, every row independent
 * (ilusv_jacobi with the generic ilu_jacobi_mv, kernels.hpp:171-248).
 *
 * Types: 0 = fp64, 1 = fp32 (mpg_dtype_t of arnoldi.h). All calls are
 * stream-ordered on the context's stream; create synchronises once.
 */
#ifndef MPGMRES_ILU_H
#define MPGMRES_ILU_H

#include <stdint.h>

#include "mpgmres/capi.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct mpg_ilu* mpg_ilu_t;

/* ILU(0) of A (val64: device fp64 values in A's CSR order; every row needs
 * its diagonal entry and at most mpg_ilu_row_cap() entries). */
int mpg_ilu0_create(mpg_ctx_t ctx, mpg_csr_t A, const double* val64, int type, mpg_ilu_t* out);
int mpg_ilu_destroy(mpg_ilu_t ilu);
int mpg_ilu_row_cap(void);

/* x := U^-1 L^-1 x (device vector of the factor type, length n) */
int mpg_ilu_solve(mpg_ctx_t ctx, mpg_ilu_t ilu, void* x);
/* x := the ILU-Jacobi approximation of U^-1 L^-1 x with `steps` sweeps */
int mpg_ilu_jacobi_solve(mpg_ctx_t ctx, mpg_ilu_t ilu, int steps, void* x);

/* factors (device, CSR order, factor type), pivot positions (device int32,
 * n), and 1/u_ii (device, factor type): for tests and fused callers */
const void* mpg_ilu_values_dev(mpg_ilu_t ilu);
const int32_t* mpg_ilu_diag_dev(mpg_ilu_t ilu);
const void* mpg_ilu_dinv_dev(mpg_ilu_t ilu);
/* non-zero when a row waited past its bound (a scheduling fault; results
 * are then not valid). Synchronises. The word is sticky: every solve after
 * a fault keeps reporting it until mpg_ilu_clear_fault. The solve engines
 * read it at every restart-cycle boundary (fused) or after every apply
 * (operator surface) and fail the solve with MPG_ERR_BREAKDOWN. */
int mpg_ilu_fault(mpg_ilu_t ilu);
int mpg_ilu_clear_fault(mpg_ilu_t ilu);
/* per-wait bound of the level-scheduled triangular solves in ticks of the
 * 100 MHz real-time counter (0 = the default, ~2 s). Test hook: a tiny
 * bound makes any real wait fault. */
int mpg_ilu_set_wait_bound(mpg_ilu_t ilu, uint64_t ticks);
/* diagnostics: tickets drawn by the factor / L / U launches and the fault
 * word (1 = a bounded wait expired, 2 = a launch passed its deadline) */
int mpg_ilu_debug_state(mpg_ilu_t ilu, int32_t* out4);
/* how the triangular solves run: bit 0 set = L solved serially by one
 * workgroup (few rows per dependency level, e.g. banded), bit 1 = U; clear
 * bits use the level schedule. MPG_ILU_SERIAL=0 at create forces levels. */
int mpg_ilu_solve_mode(mpg_ilu_t ilu);

#ifdef __cplusplus
}
#endif
#endif /* MPGMRES_ILU_H */
