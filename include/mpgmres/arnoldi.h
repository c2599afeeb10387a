/*
 * mpgmres fused-Arnoldi C-ABI (libmpgmres_hip.so) — the performance form of
 * one restarted GMRES(m) cycle on gfx950, with no host synchronisation
 * inside a cycle.
 *
 * Replaces, for one restart cycle of gmres_singleUpdate / gmres_baseline
 * (gmres.cpp:160-242, 51-130), the per-operator calls of the reference
 * (spmv, M->apply, orth.add_vector, rot/rotg/rot, fence + s.access,
 * solution_update) by a short program of fused phase kernels:
 *
 *   prologue   r = b - A x (outer precision), w = M(T(r)), partial sums of
 *              ||T(r)||^2, ||w||^2, ||x||^2            (types.hpp:230-448, gmres.cpp:171-180)
 *   finish     r_norm, beta, x_norm -> report; 1/beta; s = [beta, 0, ...]
 *   spmv(k)    v_k = w_prev * (1/h_{k,k-1}) formed on the fly (written to V
 *              for local rows), w = M(A v_k), and per-workgroup partial dots
 *              <v_j, w> for j <= k (CGS / CGSR) or j = 0 (MGS)
 *              (Orthogonalization.hpp:56-59, 83-87, 99-105)
 *   cgs(k,p)   coefficients c = T(sums); w -= V c; partials of ||w||^2 (last
 *              pass) or of <v_j, w> (first CGSR pass)
 *   mgs(k,j)   h_jk = T(sum); w -= h_jk v_j; partial <v_{j+1}, w> or ||w||^2
 *   givens(k)  h_{k+1,k} = ||w||; 1/h for the next step; rotations on column
 *              k, rotg, rotation of s; |s(k+1)| -> report   (gmres.cpp:217-226)
 *   update(k)  y = H(0:k,0:k)^-1 s(0:k); x += V(:,0:k) y  (gmres.cpp:276-290)
 *
 * Every global reduction is two-stage: phase kernels write per-workgroup
 * partials (fp64 storage; fp32 values under MPG_ACCUM_F32, below),
 * mpg_arnoldi_reduce sums them in a fixed order into
 * `sums` (fp64). A row-partitioned multi-GPU caller all-reduces `sums`
 * across ranks between the two (mpg_arnoldi_sums_dev), and exchanges the
 * halo entries of w_prev / x (mpg_arnoldi_halo_*), before the consumers
 * read them — every rank then holds bit-identical scalars and takes the same
 * decisions.
 */
#ifndef MPGMRES_ARNOLDI_H
#define MPGMRES_ARNOLDI_H

#include <stdint.h>

#include "mpgmres/capi.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef enum { MPG_F64 = 0, MPG_F32 = 1, MPG_F16 = 2 } mpg_dtype_t;

typedef struct mpg_arnoldi* mpg_arnoldi_t;

typedef struct {
    int32_t n;             /* local rows */
    int32_t n_ext;         /* local rows + halo entries (== n on one GPU) */
    int32_t m;             /* restart length */
    int32_t orth;          /* 0 CGS, 1 MGS, 2 CGSR(2) — mpg_orth_t */
    int32_t vec_type;      /* T: Krylov basis, w, H, Givens (MPG_F64 | MPG_F32) */
    int32_t outer_type;    /* X: x, b, residual (MPG_F64 | MPG_F32) */
    int32_t prec_type;     /* P: preconditioner arithmetic (MPG_F64 | MPG_F32) */
    int32_t inner_val;     /* value type of the Arnoldi SpMV (MPG_F64 | MPG_F32 | MPG_F16) */
    int32_t jacobi;        /* 1: w = d∘w (gdmv), 0: identity */
    mpg_csr_t A;           /* analysed local CSR, columns in [-n_front, n_ext) */
    const void* val_outer; /* residual values, outer_type */
    const void* val_inner; /* Arnoldi values, inner_val */
    const void* diag;      /* Jacobi inverse diagonal (prec_type) or NULL */
    const void* b;         /* outer_type, n */
    void* x;               /* outer_type, row 0 of [-MPG_FRONT_PAD(n_front), n_ext) (halo filled by the caller) */
    int32_t spmv_format;   /* Arnoldi SpMV storage: 0 auto, 1 CSR row blocks, 2 sliced ELL (SELL-64),
                              3 node blocks (3-dof nodes, 3 x 3 blocks; node_tile.hpp) */
    int32_t n_front;       /* halo rows of lower ranks, local ids [-n_front, 0) (0 on one GPU) */
    const int8_t* inner_row_exp; /* inner_val MPG_F16: per-row exponents of the scaled fp16 copy
                                    (mpg_csr_half_values, capi.h), or NULL (unscaled) */
} mpg_arnoldi_desc;

/* Entries allocated in front of row 0 of every vector with a halo (x, the
 * w buffers): the lower halo rounded up to 64, plus the 64 rows the first
 * slice's LDS window reads below row 0 (vectors are passed as a pointer to
 * row 0; mpg_halo_n_front, dist.h). */
#define MPG_FRONT_PAD(n_front) ((n_front) > 0 ? ((n_front) + 63) / 64 * 64 + 64 : 0)

/* Allocates the basis V (n x (m+1), leading dimension padded to 256 B),
 * H, Givens state, two w buffers (n_ext), partials and the report block. */
int mpg_arnoldi_create(mpg_ctx_t ctx, const mpg_arnoldi_desc* desc, mpg_arnoldi_t* out);
int mpg_arnoldi_destroy(mpg_arnoldi_t a);

/* Storage the Arnoldi SpMV runs on: *format 1 = CSR row blocks (cuSPARSE
 * csrmv's input, types_cuda.hpp:53-60), 2 = SELL-64 copy made at create
 * (64-row slices, vec_width entries per lane load, col_bytes 4 = int32
 * columns or 2 = int16 offsets from the slice's first row); *stored = stored
 * entries including padding (nnz for CSR); *window = 1 when every slice's
 * columns lie within [row0 - 64, row0 + 128) and the SpMV reads v_k from an
 * LDS window instead of gathering from memory. Any output may be NULL. */
int mpg_arnoldi_spmv_layout(mpg_arnoldi_t a, int32_t* format, int32_t* vec_width, int32_t* col_bytes,
                            int64_t* stored, int32_t* window);
/* matrix bytes one SELL SpMV reads (0 without a SELL copy): every slot's
 * value, the columns of slots outside implicit slices (plus their shared
 * patterns), int64 slice offsets, the per-slice pattern indices and the
 * stepped form's (slice, step, element) bases */
int64_t mpg_arnoldi_sell_matrix_bytes(mpg_arnoldi_t a);
/* column form of the SELL copy as mpg_sell_columns (capi.h): -1 no copy,
 * 0 int32, 1 int16 slice-relative, 2 stepped int16; CSR-summed and implicit
 * slice counts. Any output may be NULL. */
int mpg_arnoldi_sell_columns(mpg_arnoldi_t a, int32_t* form, int64_t* csr_slices, int64_t* implicit_slices);
/* slices per wave of the SELL Arnoldi SpMV kernel: 0 no SELL copy, 1
 * k_step_sell, 2 k_step_sell2 (uniform int16 copies; MPG_SELL_PAIR=0: 1) */
int mpg_arnoldi_slices_per_wave(mpg_arnoldi_t a);
/* slices of the SELL copy that read another slice's column block (mpg_sell_shared_slices) */
int64_t mpg_arnoldi_sell_shared_slices(mpg_arnoldi_t a);
/* SELL-C-sigma: the window (rows) inside which the copy's rows were sorted by
 * length before slicing (rows of varying length, e.g. FEM-like matrices);
 * 0: slice s holds rows 64 s .. 64 s + 63 (MPG_SELL_SIGMA, sell_tile.hpp) */
int mpg_arnoldi_sell_sigma(mpg_arnoldi_t a);

int mpg_arnoldi_prologue(mpg_arnoldi_t a);              /* partials: 3 columns */
int mpg_arnoldi_prologue_finish(mpg_arnoldi_t a);
/* one GPU: mpg_arnoldi_reduce(a, 3) + mpg_arnoldi_prologue_finish in one
 * launch (the same column sums, the same bits) */
int mpg_arnoldi_prologue_finish_partials(mpg_arnoldi_t a);
/* recompute the ||w||^2 partials of the prologue (column 1) after the
 * caller preconditioned w (mpg_arnoldi_wprev_dev(a, 0)) itself — ILU */
int mpg_arnoldi_prologue_wnorm(mpg_arnoldi_t a);
int mpg_arnoldi_spmv(mpg_arnoldi_t a, int k);           /* w = M(A v_k), V(:,k) */
int mpg_arnoldi_dots(mpg_arnoldi_t a, int k);           /* partials: k+1 (CGS/CGSR) or 1 (MGS) */
int mpg_arnoldi_cgs(mpg_arnoldi_t a, int k, int pass);  /* pass 0: h; pass 1: CGSR correction */
/* one GPU, k+1 <= 32 (plain CGS: k+1 <= mpg_arnoldi_partials_max_cols()):
 * CGS pass 0 that sums the preceding mpg_arnoldi_dots partials itself
 * (every workgroup, same fixed order) — replaces mpg_arnoldi_reduce +
 * mpg_arnoldi_cgs(a, k, 0) */
int mpg_arnoldi_cgs_partials(mpg_arnoldi_t a, int k);
int mpg_arnoldi_partials_max_cols(void);
/* one GPU, CGSR(2) with 32 < k+1 <= mpg_arnoldi_partials_max_cols(): pass
 * `pass` (0: h(0:k,k), 1: the correction, Orthogonalization.hpp:109-136)
 * with its coefficients summed from the preceding mpg_arnoldi_dots partials
 * (the one-launch panel dots) and no next dots: the step is dots, pass 0,
 * dots, pass 1 -- four launches where the round-3 form needed one per 32
 * columns plus two reduces */
int mpg_arnoldi_cgsr_wide_pass(mpg_arnoldi_t a, int k, int pass);
int mpg_arnoldi_mgs(mpg_arnoldi_t a, int k, int j);
/* one GPU: MGS update j taking h_jk from the partials of the previous launch
 * (mpg_arnoldi_dots for j = 0, the previous update otherwise) — replaces
 * mpg_arnoldi_reduce + mpg_arnoldi_mgs */
int mpg_arnoldi_mgs_partials(mpg_arnoldi_t a, int k, int j);
int mpg_arnoldi_givens(mpg_arnoldi_t a, int k);
/* single-GPU form: the Givens kernel sums the ||w||^2 partials of the last
 * producer itself, saving one mpg_arnoldi_reduce launch per step */
int mpg_arnoldi_givens_partials(mpg_arnoldi_t a, int k);
/* Givens step k-1 folded into the SpMV launch of step k (1 <= k < m, m <=
 * mpg_arnoldi_fold_max_m()): every workgroup forms 1/h_{k,k-1} from the
 * ||w||^2 sum itself and workgroup 0 runs the rotation step — one launch
 * boundary fewer per Arnoldi step. _partials_ reads the last producer's
 * workgroup partials (one GPU), the other form sums[0] (after an all-reduce).
 * The last step's Givens (k = m-1) stays a separate mpg_arnoldi_givens*. */
int mpg_arnoldi_givens_spmv(mpg_arnoldi_t a, int k);
/* One-GPU combined forms (no separate reduce / Givens launch): the phase's
 * workgroup partials are written through to memory and the last workgroup
 * to finish sums them in a fixed order. dots_sums: panel dots for k+1 <= 32
 * columns straight into sums (replaces dots + reduce); cgs_givens: the last
 * CGS pass (pass 0 for CGS, 1 for CGSR) followed by the Givens step k
 * (replaces cgs + givens_partials; m <= mpg_arnoldi_fold_max_m()). */
int mpg_arnoldi_dots_sums(mpg_arnoldi_t a, int k);
int mpg_arnoldi_cgs_givens(mpg_arnoldi_t a, int k, int pass);
int mpg_arnoldi_givens_partials_spmv(mpg_arnoldi_t a, int k);
/* SpMV step k (fold as above: 0 plain, 1 from sums[0], 2 from the partials)
 * with the panel dots <v_j, w>, j <= k, formed in the same launch: replaces
 * spmv + dots ahead of mpg_arnoldi_cgs_partials (one GPU, CGS / CGSR,
 * k + 1 <= 32). MPG_ERR_UNSUPPORTED unless the SpMV runs on the SELL copy
 * with an fp32 basis, fp32 values, 16-bit columns and the v_k window. */
int mpg_arnoldi_spmv_dots(mpg_arnoldi_t a, int k, int fold);
int mpg_arnoldi_fold_max_m(void);
/* 1 when folding the Givens step into the SpMV pays at this size (the SpMV's
 * workgroups each sum the partials; past ~4k workgroups a separate Givens
 * launch costs less); the engine folds then unless MPG_FOLD_GIVENS says */
int mpg_arnoldi_fold_pays(mpg_arnoldi_t a);
int mpg_arnoldi_update(mpg_arnoldi_t a, int k);
/* sums[c] = sum over workgroups of partial column c, c < ncols */
int mpg_arnoldi_reduce(mpg_arnoldi_t a, int ncols);

/* Device pointers for a multi-GPU caller. */
double* mpg_arnoldi_sums_dev(mpg_arnoldi_t a);          /* fp64 [m + 4] */
void* mpg_arnoldi_wprev_dev(mpg_arnoldi_t a, int k);    /* input vector of step k, n_ext of T */
int mpg_arnoldi_vec_bytes(mpg_arnoldi_t a);             /* sizeof(T) */
/* report block (fp64, device): [0] r_norm [1] beta [2] x_norm [3] inv_beta
 * [4 + k] |s(k+1)| after step k */
const double* mpg_arnoldi_report_dev(mpg_arnoldi_t a);
int mpg_arnoldi_report_len(mpg_arnoldi_t a);
/* The Krylov basis (for tests): V column j of T, ld elements apart */
const void* mpg_arnoldi_basis_dev(mpg_arnoldi_t a, int64_t* ld);
const void* mpg_arnoldi_hessenberg_dev(mpg_arnoldi_t a);  /* (m+1) x m, column-major, T */
/* 1/h_{k+1,k} (T) written by the Givens step k for the next SpMV's
 * normalisation (Orthogonalization.hpp:56-59 reciprocal) */
const void* mpg_arnoldi_inv_dev(mpg_arnoldi_t a);
/* measurement: the next Arnoldi SpMV launch (any form: plain, Givens folded,
 * dots fused) records its own kernel start/stop on these hipEvent_t
 * (hipExtLaunchKernel events: the kernel alone, not the queue around it) */
int mpg_arnoldi_time_next_spmv(mpg_arnoldi_t a, void* start_event, void* stop_event);
/* measurement: the next stamped launch -- the one-panel dots (k_dots_nc) or
 * the one-panel CGS update (k_cgs_update_nc); not the SpMVs, whose occupancy
 * the stamp code would change -- stores, per wave q, the device wall clock
 * (wall_clock64, hipDeviceAttributeWallClockRate kHz) at the wave's start
 * to slots[2q] and at its end to slots[2q + 1] (device memory, 2 *
 * cap_waves entries; waves that exit early store no end). Nothing is stored
 * when the launch has more than cap_waves waves; slots = NULL disarms.
 * Usable inside a stream capture: the kernel's duration is max(end) -
 * min(start). */
int mpg_arnoldi_stamp_next(mpg_arnoldi_t a, unsigned long long* slots, int64_t cap_waves);
/* the most waves a stamped launch of this workspace has */
int64_t mpg_arnoldi_stamp_waves(mpg_arnoldi_t a);

/* Number of workgroups of the row-block phase kernels (partials per column). */
int mpg_arnoldi_num_groups(mpg_arnoldi_t a);

/* The per-workgroup fp64 partials the last phase kernel wrote, and their
 * count (columns x workgroups): a multi-GPU caller may all-reduce them in
 * place and let the next kernel sum them (mpg_arnoldi_givens_partials_spmv,
 * mpg_arnoldi_mgs_partials) instead of a reduce launch + a scalar
 * all-reduce. Every rank must then have the same partial count: call
 * mpg_arnoldi_uniform_groups once after create (the one-per-CU panel
 * kernels then always run 256 workgroups; those without rows write zeros). */
double* mpg_arnoldi_partials_dev(mpg_arnoldi_t a);
int mpg_arnoldi_partials_count(mpg_arnoldi_t a);
int mpg_arnoldi_uniform_groups(mpg_arnoldi_t a);

/* Accumulation class of an fp32 Arnoldi (vec_type MPG_F32), set once after
 * create, before the first cycle:
 *   MPG_ACCUM_F64 (default)  every dot, norm, gemv and SpMV row sum adds the
 *                            fp32 products in fp64 and rounds once;
 *   MPG_ACCUM_F32            every partial sum is an fp32 value: SpMV row
 *                            sums (products rounded to fp32, added in CSR
 *                            order), panel dots and the ||w||^2 partials
 *                            (fp32 fused multiply-adds per lane, fp32 wave /
 *                            workgroup trees), the partials' combines, the
 *                            CGS update's V c and the solution update's V y
 *                            -- the class of the reference's cblas_sdot /
 *                            snrm2 / sgemv and mkl_sparse_s_mv
 *                            (kernels_mkl.cpp:82,94,104,114,284,348) and of
 *                            its GPU backend's cublasSdot / Sgemv /
 *                            cusparseScsrmv (kernels_cuda.cpp:132,160,530,609).
 *                            The once-per-cycle prologue (the fp64 residual
 *                            and the norms of T(r), w and x) keeps fp64
 *                            sums; so does a multi-rank all-reduce of the
 *                            partials (ncclFloat64 sums of fp32 values).
 * An fp64 Arnoldi accumulates in fp64 whatever is asked (cblas_d*: the
 * reference's class); mpg_arnoldi_accum reports what runs. The panel dots
 * fused into the SpMV (mpg_arnoldi_spmv_dots) exist in fp64 only
 * (MPG_ERR_UNSUPPORTED under MPG_ACCUM_F32: the caller launches the dots). */
#define MPG_ACCUM_F64 0
#define MPG_ACCUM_F32 1
int mpg_arnoldi_set_accum(mpg_arnoldi_t a, int accum);
int mpg_arnoldi_accum(mpg_arnoldi_t a);

/* Storage the residual prologue runs on: 1 CSR row blocks, 2 the SELL copy
 * of the outer values, 3 node blocks (row sums on the node copy, then the
 * CSR prologue's epilogue and norm partials: its bits). */
int mpg_arnoldi_prologue_format(mpg_arnoldi_t a);

#ifdef __cplusplus
}
#endif
#endif /* MPGMRES_ARNOLDI_H */
