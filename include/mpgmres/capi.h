/*
 * mpgmres C-ABI — the drop-in boundary between host code and the hand-written
 * gfx950 HIP kernels of the mixed-precision GMRES hot path.
 *
 * Every entry point is `extern "C"`, takes plain pointers and sizes, and
 * returns an int status (0 = OK, < 0 = error; see mpg_status_t and
 * mpg_error_string). No torch types, no C++ types. Pointers named *_dev are
 * device (HBM) pointers; *_host are host pointers. All calls are ordered on
 * the context's HIP stream and are asynchronous unless the name ends in
 * `_host` (those synchronise the stream and return a value through host
 * memory — the equivalent of the reference's host-pointer-mode BLAS calls).
 *
 * Each family cites the reference interface it replaces (paths are relative
 * to the reference repository iamsonderr/icl-mixed-precision-gmres):
 *   kernels.hpp:9-169        operator surface (templates on <Type, Device>)
 *   kernels_mkl.cpp:73-352   MKL (host) specialisations — the semantics kept
 *   kernels_cuda.cpp:111-614 cuBLAS/cuSPARSE specialisations — replaced
 *   types.hpp:15-228         Scalar / Vect / MultiVect handles
 *   types_cuda.hpp:47-152    SparseMatrix<T, Cuda> (CSR, int32 indices)
 *   types.hpp:381-448        Jacobi preconditioner setup
 * The host-side C++ that binds these (types_hip.hpp / kernels_hip.cpp) lives
 * in icl-mixed-precision-gmres_amd/host/.
 */
#ifndef MPGMRES_CAPI_H
#define MPGMRES_CAPI_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum {
    MPG_OK = 0,
    MPG_ERR_HIP = -1,          /* a HIP runtime call failed */
    MPG_ERR_ARG = -2,          /* invalid argument (size mismatch, null, range) */
    MPG_ERR_ALLOC = -3,        /* device allocation failed */
    MPG_ERR_RCCL = -4,         /* an RCCL call failed */
    MPG_ERR_UNSUPPORTED = -5,  /* operation not supported for these arguments */
    MPG_ERR_BREAKDOWN = -6,    /* Arnoldi breakdown / non-finite value detected */
    MPG_ERR_RANGE = -7         /* a value does not fit the storage precision (fp16 values) */
} mpg_status_t;

typedef struct mpg_ctx* mpg_ctx_t;   /* one per (GPU, host thread) */
typedef struct mpg_csr* mpg_csr_t;   /* analysed CSR structure (row blocks) */
typedef struct mpg_sell* mpg_sell_t; /* SELL-64 copy of one CSR value array */
typedef struct mpg_node* mpg_node_t; /* node-block copy (3 x 3 blocks) of one CSR value array */

const char* mpg_error_string(int status);
/* Last HIP error text recorded in this context (for diagnostics). */
const char* mpg_ctx_last_error(mpg_ctx_t ctx);

/* ---- context / memory (replaces Kokkos::View allocation + deep_copy,
 *      types.hpp:15-228, and CudaLibSingleton, types_cuda.hpp:9-36) ---- */
int mpg_ctx_create(int device, mpg_ctx_t* out);
/* HIP devices visible to this process (hipGetDeviceCount; 0 when none) */
int mpg_device_count(void);
int mpg_ctx_destroy(mpg_ctx_t ctx);
/* Device::execution_space().fence() (gmres.cpp:113, 225) */
int mpg_ctx_sync(mpg_ctx_t ctx);
/* hipStream_t of the context, as an opaque pointer. */
void* mpg_ctx_stream(mpg_ctx_t ctx);
int mpg_ctx_device(mpg_ctx_t ctx);

/* ---- cycle programs: a run of asynchronous calls on the context's stream
 *      recorded once (HIP stream capture) and replayed as one graph launch.
 *      The operator-surface driver records its Arnoldi steps this way when
 *      they contain no host read (gmres.cpp:199-243 with the per-step reads
 *      deferred); the reference re-issues every call (no counterpart). ---- */
typedef struct mpg_graph* mpg_graph_t;
/* Start recording: every later call on ctx is recorded, not executed. A call
 * that must synchronise fails while recording (the recording is then void). */
int mpg_ctx_record_begin(mpg_ctx_t ctx);
/* Stop recording; on success *out is an executable program. On any failure
 * (a call inside was not recordable) *out = NULL, the status is an error and
 * nothing recorded has run. */
int mpg_ctx_record_end(mpg_ctx_t ctx, mpg_graph_t* out);
/* 1 while ctx is recording, else 0 */
int mpg_ctx_recording(mpg_ctx_t ctx);
/* Run a recorded program on ctx's stream (asynchronous). */
int mpg_graph_launch(mpg_ctx_t ctx, mpg_graph_t g);
int mpg_graph_destroy(mpg_graph_t g);
/* Zero-initialised device allocation (Kokkos views are zero-filled). */
int mpg_malloc(mpg_ctx_t ctx, size_t bytes, void** out_dev);
int mpg_free(mpg_ctx_t ctx, void* ptr_dev);
int mpg_memset(mpg_ctx_t ctx, void* ptr_dev, int value, size_t bytes);
int mpg_memcpy_h2d(mpg_ctx_t ctx, void* dst_dev, const void* src_host, size_t bytes);
int mpg_memcpy_d2h(mpg_ctx_t ctx, void* dst_host, const void* src_dev, size_t bytes);
int mpg_memcpy_d2d(mpg_ctx_t ctx, void* dst_dev, const void* src_dev, size_t bytes);

/* Measured HBM streaming rate (GB/s) of this GPU: kind 0 = float4 read
 * (bytes read), 1 = float4 copy (bytes read + written), on fresh buffers of
 * `bytes` (>= 1 MiB; use >= 1 GiB to stay clear of the Infinity Cache); the
 * best kernel time (hipExtLaunchKernel events) over a grid/unroll sweep with
 * `reps` launches each. No reference counterpart: the achievable peak
 * bench.py reports beside the 8 TB/s spec. */
int mpg_bw_probe(mpg_ctx_t ctx, int kind, size_t bytes, int reps, double* gbs_out);

/* ---- BLAS-1 (kernels.hpp:11-101; kernels_mkl.cpp:73-211) ----
 * Reductions accumulate in fp64 for both precisions and are deterministic
 * (fixed two-stage tree); *_dev variants leave the result in device memory
 * (cuBLAS device pointer mode, kernels_cuda.cpp:142-150). */
int mpg_dot_f64(mpg_ctx_t ctx, int64_t n, const double* x, const double* y, double* result_dev);
int mpg_dot_f32(mpg_ctx_t ctx, int64_t n, const float* x, const float* y, float* result_dev);
int mpg_dot_f64_host(mpg_ctx_t ctx, int64_t n, const double* x, const double* y, double* result_host);
int mpg_dot_f32_host(mpg_ctx_t ctx, int64_t n, const float* x, const float* y, float* result_host);
int mpg_nrm2_f64(mpg_ctx_t ctx, int64_t n, const double* x, double* result_dev);
int mpg_nrm2_f32(mpg_ctx_t ctx, int64_t n, const float* x, float* result_dev);
int mpg_nrm2_f64_host(mpg_ctx_t ctx, int64_t n, const double* x, double* result_host);
int mpg_nrm2_f32_host(mpg_ctx_t ctx, int64_t n, const float* x, float* result_host);
// ||a|| and ||b|| (each MPG_F32 or MPG_F64 of mpg_dtype_t, arnoldi.h; n rows, 16-B aligned) in one
// launch and one host read, each with the bits of its own mpg_nrm2_*_host
// (the operator surface's restart section: ||w|| with the ||x|| the
// reference's driver reads next, gmres.cpp:173-196); results widened to
// double. MPG_ERR_UNSUPPORTED: unaligned, or no pinned staging.
int mpg_nrm2_pair_host(mpg_ctx_t ctx, int64_t n, int type_a, const void* a, int type_b, const void* b,
                       double* norm_a_host, double* norm_b_host);
/* Split reductions (the operator surface defers stage 2 into the consumer
 * of the result; kernels_hip.cpp). *_partials runs stage 1 only: *nparts
 * fp64 partials in the context workspace, valid until the next reduction on
 * ctx. *_finish is stage 2 (the same result as the one-call form). The
 * consumers fold stage 2 in, every workgroup with stage 2's own order (same
 * bits), workgroup 0 storing the result:
 *   mpg_scal_recip_nrm2_*: h = ||x||, y = (1/h) x   (add_vector, Orthogonalization.hpp:51-60)
 *   mpg_naxpy_dot_*:       a = <x', y'>, y -= a x   (MGS_Kernel, Orthogonalization.hpp:91-107) */
int mpg_dot_partials_f64(mpg_ctx_t ctx, int64_t n, const double* x, const double* y, int32_t* nparts);
int mpg_dot_partials_f32(mpg_ctx_t ctx, int64_t n, const float* x, const float* y, int32_t* nparts);
int mpg_nrm2_partials_f64(mpg_ctx_t ctx, int64_t n, const double* x, int32_t* nparts);
int mpg_nrm2_partials_f32(mpg_ctx_t ctx, int64_t n, const float* x, int32_t* nparts);
int mpg_dot_finish_f64(mpg_ctx_t ctx, int32_t nparts, double* result_dev);
int mpg_dot_finish_f32(mpg_ctx_t ctx, int32_t nparts, float* result_dev);
int mpg_nrm2_finish_f64(mpg_ctx_t ctx, int32_t nparts, double* result_dev);
int mpg_nrm2_finish_f32(mpg_ctx_t ctx, int32_t nparts, float* result_dev);
int mpg_scal_recip_nrm2_f64(mpg_ctx_t ctx, int32_t nparts, double* h_dev, int64_t n, const double* x, double* y);
int mpg_scal_recip_nrm2_f32(mpg_ctx_t ctx, int32_t nparts, float* h_dev, int64_t n, const float* x, float* y);
int mpg_naxpy_dot_f64(mpg_ctx_t ctx, int32_t nparts, double* a_dev, int64_t n, const double* x, double* y);
int mpg_naxpy_dot_f32(mpg_ctx_t ctx, int32_t nparts, float* a_dev, int64_t n, const float* x, float* y);
/* the unrounded fp64 accumulator of <x, y> (one rank's share of a
 * distributed dot / squared norm, summed across ranks before rounding) */
int mpg_dot_acc_f64(mpg_ctx_t ctx, int64_t n, const double* x, const double* y, double* acc_dev);
int mpg_dot_acc_f32(mpg_ctx_t ctx, int64_t n, const float* x, const float* y, double* acc_dev);
/* y += alpha*x, alpha on host (kernels_mkl.cpp:118-128) */
int mpg_axpy_f64(mpg_ctx_t ctx, int64_t n, double alpha, const double* x, double* y);
int mpg_axpy_f32(mpg_ctx_t ctx, int64_t n, float alpha, const float* x, float* y);
/* y += alpha*x with alpha read from device memory (kernels_mkl.cpp:130-140) */
int mpg_axpy_dev_f64(mpg_ctx_t ctx, int64_t n, const double* alpha_dev, const double* x, double* y);
int mpg_axpy_dev_f32(mpg_ctx_t ctx, int64_t n, const float* alpha_dev, const float* x, float* y);
/* y -= alpha*x, alpha on device (naxpy, kernels_mkl.cpp:143-153) */
int mpg_naxpy_dev_f64(mpg_ctx_t ctx, int64_t n, const double* alpha_dev, const double* x, double* y);
int mpg_naxpy_dev_f32(mpg_ctx_t ctx, int64_t n, const float* alpha_dev, const float* x, float* y);
/* x *= alpha in place (kernels_mkl.cpp:155-163) */
int mpg_scal_f64(mpg_ctx_t ctx, int64_t n, double alpha, double* x);
int mpg_scal_f32(mpg_ctx_t ctx, int64_t n, float alpha, float* x);
/* y = alpha*x (copy then scal, kernels_mkl.cpp:165-191); alpha host or device */
int mpg_scal_copy_f64(mpg_ctx_t ctx, int64_t n, double alpha, const double* x, double* y);
int mpg_scal_copy_f32(mpg_ctx_t ctx, int64_t n, float alpha, const float* x, float* y);
int mpg_scal_copy_dev_f64(mpg_ctx_t ctx, int64_t n, const double* alpha_dev, const double* x, double* y);
int mpg_scal_copy_dev_f32(mpg_ctx_t ctx, int64_t n, const float* alpha_dev, const float* x, float* y);
/* y = (1/alpha)*x with the reciprocal formed on device in the vector's
 * precision — the sync-free form of `scal(1/h_final, w, v)`
 * (Orthogonalization.hpp:56-59). */
int mpg_scal_recip_copy_dev_f64(mpg_ctx_t ctx, int64_t n, const double* alpha_dev, const double* x, double* y);
int mpg_scal_recip_copy_dev_f32(mpg_ctx_t ctx, int64_t n, const float* alpha_dev, const float* x, float* y);
/* copy with cast (kernels.hpp:11-30). Suffix = <src><dst>. */
int mpg_copy_f64f64(mpg_ctx_t ctx, int64_t n, const double* x, double* y);
int mpg_copy_f32f32(mpg_ctx_t ctx, int64_t n, const float* x, float* y);
int mpg_copy_f64f32(mpg_ctx_t ctx, int64_t n, const double* x, float* y);
int mpg_copy_f32f64(mpg_ctx_t ctx, int64_t n, const float* x, double* y);
int mpg_copy_f64f16(mpg_ctx_t ctx, int64_t n, const double* x, uint16_t* y_half);
int mpg_copy_f32f16(mpg_ctx_t ctx, int64_t n, const float* x, uint16_t* y_half);
/* y[i] = x[idx[i]] for i < n, elements of 4 or 8 bytes (halo packing of a
 * row-partitioned vector before the neighbour exchange) */
int mpg_gather_b32(mpg_ctx_t ctx, int64_t n, const int32_t* idx, const void* x, void* y);
int mpg_gather_b64(mpg_ctx_t ctx, int64_t n, const int32_t* idx, const void* x, void* y);
/* fill (kernels.hpp:88-101): strided 2-D form covers Scalar/Vect/MultiVect */
int mpg_fill_f64(mpg_ctx_t ctx, double* x, int64_t rows, int64_t cols, int64_t ld, double value);
int mpg_fill_f32(mpg_ctx_t ctx, float* x, int64_t rows, int64_t cols, int64_t ld, float value);
/* y = beta*y + alpha*d∘x (gdmv, kernels.hpp:131-151; Jacobi::apply) */
int mpg_gdmv_f64(mpg_ctx_t ctx, int64_t n, double alpha, const double* d, const double* x, double beta, double* y);
int mpg_gdmv_f32(mpg_ctx_t ctx, int64_t n, float alpha, const float* d, const float* x, float beta, float* y);

/* ---- Givens (kernels_mkl.cpp:214-260; device-resident form of
 *      kernels_cuda.cpp:394-494) — all operands in device memory ---- */
/* BLAS rotg on (a,b) -> (r, c, s); b is then set to 0 (kernels_mkl.cpp:218) */
int mpg_rotg_f64(mpg_ctx_t ctx, double* a, double* b, double* c, double* s);
int mpg_rotg_f32(mpg_ctx_t ctx, float* a, float* b, float* c, float* s);
/* (a,b) <- (c a + s b, -s a + c b) on one pair (kernels_mkl.cpp:228-238) */
int mpg_rot_f64(mpg_ctx_t ctx, double* a, double* b, const double* c, const double* s);
int mpg_rot_f32(mpg_ctx_t ctx, float* a, float* b, const float* c, const float* s);
/* apply rotations j=0..k-1 to the column a[0..k] (kernels_mkl.cpp:240-260) */
int mpg_rot_vec_f64(mpg_ctx_t ctx, int k, double* a, const double* c, const double* s);
int mpg_rot_vec_f32(mpg_ctx_t ctx, int k, float* a, const float* c, const float* s);

/* ---- scalar programs: a short run of the scalar operators (rotg, rot,
 *      rot_vec, scalar copy and scal) executed in call order by one lane of
 *      ONE launch, with the arithmetic of the single-operator kernels above
 *      (bit-identical). The operator surface batches consecutive scalar calls
 *      into one program: on its own each is a dependent launch of ~4.6 us on
 *      gfx950, for a few flops (the Givens step gmres.cpp:217-222 is three). */
typedef enum {
    MPG_SOP_ROTG = 0,      /* rotg(p0=a, p1=b, p2=c, p3=s), then b := 0 */
    MPG_SOP_ROT = 1,       /* rot(p0=a, p1=b, p2=c, p3=s) */
    MPG_SOP_ROT_VEC = 2,   /* rot_vec(k, p0=a, p2=c, p3=s) */
    MPG_SOP_COPY = 3,      /* *p1 = *p0 (same precision) */
    MPG_SOP_SCAL = 4,      /* *p1 = alpha * *p0 */
    MPG_SOP_SCAL_DEV = 5   /* *p1 = *p2 * *p0 */
} mpg_scalar_opcode;
typedef struct {
    int32_t op;       /* mpg_scalar_opcode */
    int32_t f64;      /* 1: double operands, 0: float */
    int32_t k;        /* MPG_SOP_ROT_VEC: number of rotations */
    int32_t reserved;
    double alpha;     /* MPG_SOP_SCAL (rounded to the operand precision) */
    void* p[4];       /* device pointers */
} mpg_scalar_op;
#define MPG_SCALAR_PROGRAM_MAX 8
int mpg_scalar_program(mpg_ctx_t ctx, const mpg_scalar_op* ops, int count);
/* y[0] = alpha*x[0] (scalar scal, kernels_mkl.cpp:193-211) */
int mpg_scal_scalar_f64(mpg_ctx_t ctx, double alpha, const double* x, double* y);
int mpg_scal_scalar_f32(mpg_ctx_t ctx, float alpha, const float* x, float* y);
int mpg_scal_scalar_dev_f64(mpg_ctx_t ctx, const double* alpha_dev, const double* x, double* y);
int mpg_scal_scalar_dev_f32(mpg_ctx_t ctx, const float* alpha_dev, const float* x, float* y);

/* ---- BLAS-2 (kernels_mkl.cpp:264-321) — column-major, explicit lda ----
 * trans = 0: y = alpha*A x + beta*y   (A is rows x cols, x: cols, y: rows)
 * trans = 1: y = alpha*A^T x + beta*y (x: rows, y: cols)
 * The tall-skinny cases of the Arnoldi step (rows = n, cols <= m+1) are the
 * panel kernels of DESIGN.md §4. beta == 0 never reads y. */
int mpg_gemv_f64(mpg_ctx_t ctx, int trans, int64_t rows, int64_t cols, double alpha,
                 const double* A, int64_t lda, const double* x, double beta, double* y);
int mpg_gemv_f32(mpg_ctx_t ctx, int trans, int64_t rows, int64_t cols, float alpha,
                 const float* A, int64_t lda, const float* x, float beta, float* y);
/* gemv^T split the same way (<= 32 columns): stage 1, stage 2, and gemv (N)
 * with x = alpha_t * (the pending sums) formed in-launch and stored by
 * workgroup 0 (CGS_Kernel: h = V^T w, then w -= V h; MPG_ERR_UNSUPPORTED
 * unless A, lda and y allow the 16-B quad form) */
int mpg_gemv_t_partials_f64(mpg_ctx_t ctx, int64_t rows, int64_t cols, const double* A, int64_t lda, const double* x,
                            int32_t* nparts);
int mpg_gemv_t_partials_f32(mpg_ctx_t ctx, int64_t rows, int64_t cols, const float* A, int64_t lda, const float* x,
                            int32_t* nparts);
int mpg_gemv_t_finish_f64(mpg_ctx_t ctx, int32_t nparts, int64_t cols, double alpha, double beta, double* y);
int mpg_gemv_t_finish_f32(mpg_ctx_t ctx, int32_t nparts, int64_t cols, float alpha, float beta, float* y);
int mpg_gemv_n_from_t_f64(mpg_ctx_t ctx, int64_t rows, int64_t cols, double alpha, const double* A, int64_t lda,
                          int32_t nparts, double alpha_t, double* x, double beta, double* y);
int mpg_gemv_n_from_t_f32(mpg_ctx_t ctx, int64_t rows, int64_t cols, float alpha, const float* A, int64_t lda,
                          int32_t nparts, float alpha_t, float* x, float beta, float* y);
/* the same, and also the ||y||^2 partials of the y it wrote, exactly as
 * mpg_nrm2_partials_* of that y would leave them (*norm_nparts of them, in the
 * context workspace until the next reduction on ctx): the consumer of a
 * following nrm2(y) (mpg_nrm2_finish_*, mpg_scal_recip_nrm2_*) needs no
 * stage-1 launch (CGS: w -= V h, then h_{k+1,k} = ||w||, Orthogonalization.hpp:
 * 51-89). MPG_ERR_UNSUPPORTED as above, or for rows < 1. */
int mpg_gemv_n_from_t_nrm2_f64(mpg_ctx_t ctx, int64_t rows, int64_t cols, double alpha, const double* A, int64_t lda,
                               int32_t nparts, double alpha_t, double* x, double beta, double* y, int32_t* norm_nparts);
int mpg_gemv_n_from_t_nrm2_f32(mpg_ctx_t ctx, int64_t rows, int64_t cols, float alpha, const float* A, int64_t lda,
                               int32_t nparts, float alpha_t, float* x, float beta, float* y, int32_t* norm_nparts);
/* the same with the result written to y_out (16-B aligned, not overlapping y)
 * instead of y: y_out = alpha*T(A x) + beta*y (round 5: the operator surface
 * keeps w's new value apart until the normalisation that rides the next
 * SpMV has read it, mpg_sell_spmv_norm_*) */
int mpg_gemv_n_from_t_nrm2_out_f64(mpg_ctx_t ctx, int64_t rows, int64_t cols, double alpha, const double* A,
                                   int64_t lda, int32_t nparts, double alpha_t, double* x, double beta,
                                   const double* y, double* y_out, int32_t* norm_nparts);
int mpg_gemv_n_from_t_nrm2_out_f32(mpg_ctx_t ctx, int64_t rows, int64_t cols, float alpha, const float* A,
                                   int64_t lda, int32_t nparts, float alpha_t, float* x, float beta, const float* y,
                                   float* y_out, int32_t* norm_nparts);
/* triangular solve, non-unit diagonal, single workgroup (n <= 4096).
 * upper = 1 'U', 0 'L'; trans = 1 solves with A^T (kernels_mkl.cpp:291-321) */
int mpg_trsv_f64(mpg_ctx_t ctx, int upper, int trans, int64_t n, const double* A, int64_t lda, double* x);
int mpg_trsv_f32(mpg_ctx_t ctx, int upper, int trans, int64_t n, const float* A, int64_t lda, float* x);

/* ---- CSR SpMV (kernels_mkl.cpp:326-352; kernels_cuda.cpp:576-614) ----
 * rowptr/col are int32, 0-based, device pointers that must outlive the
 * handle. mpg_csr_create analyses the row lengths (CSR-adaptive row blocks:
 * short rows are streamed through LDS in nnz-chunks, long rows get a
 * workgroup each) from a HOST copy of rowptr. */
int mpg_csr_create(mpg_ctx_t ctx, int32_t rows, int32_t cols, int64_t nnz,
                   const int32_t* rowptr_host, const int32_t* rowptr_dev,
                   const int32_t* col_dev, mpg_csr_t* out);
int mpg_csr_destroy(mpg_csr_t csr);
int mpg_csr_num_blocks(mpg_csr_t csr);
/* y = alpha*A x + beta*y; vals/x/y in the named precision.
 * f16f32: half-precision values, fp32 x and y (low-precision cast path). */
int mpg_csr_spmv_f64(mpg_ctx_t ctx, mpg_csr_t A, double alpha, const double* vals,
                     const double* x, double beta, double* y);
int mpg_csr_spmv_f32(mpg_ctx_t ctx, mpg_csr_t A, float alpha, const float* vals,
                     const float* x, float beta, float* y);
int mpg_csr_spmv_f16f32(mpg_ctx_t ctx, mpg_csr_t A, float alpha, const uint16_t* vals_half,
                        const float* x, float beta, float* y);

/* ---- fp16 values for the mixed-half Arnoldi SpMV (BASELINE config 5; the
 * reference has no fp16 path). IEEE fp16 holds
 * magnitudes in [6.0e-8, 65504] only, so the copy is scaled per row by a
 * power of two: out[j] = half(float(vals[j] * 2^e_i)) for the entries j of
 * row i, with e_i = 0 when the row's largest finite |a_ij| lies in
 * [2^-2, 2^15) and otherwise e_i = 14 - floor(log2 max |a_ij|) (the row's
 * largest entry then lands in [2^14, 2^15)). A SpMV over the copy forms
 * the row sum in fp64 and multiplies it by 2^-e_i (exact) before rounding,
 * so rows with e_i = 0 keep the bits of the unscaled copy, and scaled rows
 * lose nothing to range (power-of-two scaling commutes with rounding in
 * the normal range). row_exp: int8 per row (may be NULL with scale == 0).
 * scale == 0: no scaling (e_i = 0). stats (host int64[4], may be NULL):
 * [0] rows with e_i != 0, [1] nonzero finite entries that round to 0,
 * [2] finite entries that round to +-Inf, [3] rows whose e_i does not fit
 * int8. Returns MPG_ERR_RANGE when [2] or [3] is nonzero, or when scale == 0
 * and [1] is nonzero (the copy is still written); synchronises. */
int mpg_csr_half_values(mpg_ctx_t ctx, mpg_csr_t A, const double* vals, int32_t scale, uint16_t* out_half,
                        int8_t* row_exp, int64_t* stats);
/* y = alpha * (2^-e_i * sum_j half(a_ij) x_j) + beta * y over that copy */
int mpg_csr_spmv_f16f32_scaled(mpg_ctx_t ctx, mpg_csr_t A, float alpha, const uint16_t* vals_half,
                               const int8_t* row_exp, const float* x, float beta, float* y);

/* ---- SELL-64 SpMV: the same y = alpha*A x + beta*y (kernels_mkl.cpp:326-352)
 * on a sliced-ELL copy (64-row slices padded to their longest row, int16
 * slice-relative columns when they fit). mpg_sell_create copies one value
 * array (vtype MPG_F64 | MPG_F32 | MPG_F16 raw half bits) of an analysed
 * CSR; format 0 = only when padding adds <= 20 % to the stored entries
 * (*out = NULL otherwise: keep mpg_csr_spmv), 2 = always. The copy owns all
 * the device memory it reads (a stepped copy's CSR-summed slices included):
 * A and vals may be destroyed or freed once it returns; it synchronises. The
 * spmv entry must match the copy's vtype (f64 / f32 / f16f32). */
int mpg_sell_create(mpg_ctx_t ctx, mpg_csr_t A, int32_t vtype, const void* vals, int32_t format,
                    mpg_sell_t* out);
int mpg_sell_destroy(mpg_sell_t A);
int mpg_sell_layout(mpg_sell_t A, int32_t* vec_width, int32_t* col_bytes, int64_t* stored, int32_t* window);
/* column form of the copy: 0 int32, 1 int16 slice-relative, 2 stepped int16
 * (per-(slice, step, element) bases; sell_tile.hpp); *csr_slices = slices
 * of a stepped copy summed from the CSR arrays (a spread beyond int16);
 * *implicit_slices = slices whose rows share one column pattern (no columns
 * read; MPG_SELL_IMPLICIT=0 disables them). Pointers may be NULL. */
int mpg_sell_columns(mpg_sell_t A, int32_t* form, int64_t* csr_slices, int64_t* implicit_slices);
/* slices of the copy that read another slice's column block: 2-byte column
 * blocks are stored once per distinct block (the interior slices of a
 * stencil with the same boundary pattern share one); -1 for NULL */
int64_t mpg_sell_shared_slices(mpg_sell_t A);
/* matrix bytes one SpMV over the copy reads (values, columns outside
 * implicit slices, slice offsets, pattern indices, stepped bases, a sorted
 * copy's row numbers); -1 for NULL */
int64_t mpg_sell_bytes(mpg_sell_t A);
int mpg_sell_spmv_f64(mpg_ctx_t ctx, mpg_sell_t A, double alpha, const double* x, double beta, double* y);
int mpg_sell_spmv_f32(mpg_ctx_t ctx, mpg_sell_t A, float alpha, const float* x, float beta, float* y);
int mpg_sell_spmv_f16f32(mpg_ctx_t ctx, mpg_sell_t A, float alpha, const float* x, float beta, float* y);

/* ---- node-block SpMV: the same y = alpha*A x + beta*y (kernels_mkl.cpp:
 * 326-352) on a copy for matrices of 3-dof nodes (rows 3r .. 3r + 2 made of
 * the same column triples c, c + 1, c + 2 in the same storage positions:
 * mpg_csr_node_dof, dist.h; or padded blocks, mpg_node_layout): one record
 * per 3 x 3 block, the block's first
 * column and its 9 values (4.44 B per fp32 nonzero against CSR's 8), the
 * CSR tile's fp64 products and row order -- the bits of mpg_csr_spmv.
 * mpg_node_create copies one value array (vtype MPG_F64 | MPG_F32) of an
 * analysed CSR. alt_bytes < 0: build whenever A has the structure; else only
 * when the copy streams fewer bytes than alt_bytes (the copy the caller
 * would otherwise run: mpg_sell_bytes, or the CSR arrays), or at most 10 %
 * more when x is larger than one XCD's 4 MB L2 (node_tile.hpp). *out = NULL
 * when it is not built. Owns its device memory; synchronises. */
int mpg_node_create(mpg_ctx_t ctx, mpg_csr_t A, int32_t vtype, const void* vals, int64_t alt_bytes,
                    mpg_node_t* out);
int mpg_node_destroy(mpg_node_t A);
/* blocks, tiles (runs of node rows of <= 256 blocks), the bytes one SpMV
 * reads and the zero slots of padded blocks (0: every block full). Padded
 * blocks: when some node row's three rows do not share one pattern (a
 * constrained dof's identity row, a dropped entry), the blocks are the
 * union of the rows' node columns c / 3 (rows sorted ascending, columns in
 * [0, cols), cols a multiple of 3) with zeros for the missing entries -- the
 * CSR sum's bits for finite x (+-0 products leave an fp64 sum started at +0
 * unchanged). Pointers may be NULL. */
int mpg_node_layout(mpg_node_t A, int64_t* blocks, int32_t* tiles, int64_t* bytes, int64_t* padded);
int mpg_node_spmv_f64(mpg_ctx_t ctx, mpg_node_t A, double alpha, const double* x, double beta, double* y);
int mpg_node_spmv_f32(mpg_ctx_t ctx, mpg_node_t A, float alpha, const float* x, float beta, float* y);
/* The node SpMV with the operator surface's rides (round 6), the forms of
 * mpg_sell_spmv_prog_* / mpg_sell_spmv_norm_* below on the node-block copy:
 * _prog runs a scalar program in one extra workgroup of the launch; _norm
 * forms h = T(sqrt(sum of the nparts ||w||^2 partials in the context
 * workspace)), v = T(T(1)/h * w) and y = alpha * T(A v) in one launch (A
 * square; w and y must not overlap) -- the bits of mpg_scal_recip_nrm2_*
 * followed by mpg_node_spmv_prog_* (Orthogonalization.hpp:51-60, then the
 * next step's spmv, gmres.cpp:213). */
int mpg_node_spmv_prog_f64(mpg_ctx_t ctx, mpg_node_t A, double alpha, const double* x, double beta, double* y,
                           const mpg_scalar_op* ops, int32_t nops);
int mpg_node_spmv_prog_f32(mpg_ctx_t ctx, mpg_node_t A, float alpha, const float* x, float beta, float* y,
                           const mpg_scalar_op* ops, int32_t nops);
int mpg_node_spmv_norm_f64(mpg_ctx_t ctx, mpg_node_t A, int32_t nparts, double* h, const double* w, double* v,
                           double alpha, double* y, const mpg_scalar_op* ops, int32_t nops);
int mpg_node_spmv_norm_f32(mpg_ctx_t ctx, mpg_node_t A, int32_t nparts, float* h, const float* w, float* v,
                           float alpha, float* y, const mpg_scalar_op* ops, int32_t nops);
/* The same SpMV with a scalar program (mpg_scalar_program) run by one extra
 * workgroup of the launch, concurrently with the rows: for a program whose
 * operands the SpMV neither reads nor writes (the caller checks). Replaces
 * the program's own launch before the next step's spmv (gmres.cpp:106-110
 * then 96-100 in the operator surface's order). nops = 0: plain SpMV. */
int mpg_sell_spmv_prog_f64(mpg_ctx_t ctx, mpg_sell_t A, double alpha, const double* x, double beta, double* y,
                           const mpg_scalar_op* ops, int32_t nops);
int mpg_sell_spmv_prog_f32(mpg_ctx_t ctx, mpg_sell_t A, float alpha, const float* x, float beta, float* y,
                           const mpg_scalar_op* ops, int32_t nops);
/* add_vector's normalisation riding the next Arnoldi SpMV (round 5; the
 * operator surface's CGS step, Orthogonalization.hpp:51-60 then the next
 * spmv(A, V(:,k+1), w), gmres.cpp:213). The context workspace holds the
 * nparts (<= 256) ||w||^2 stage-1 partials of w (mpg_gemv_n_from_t_nrm2_*'s);
 * in one launch: h = T(sqrt(sum)) (stored to *h, before the riding scalar
 * program runs), v = T(T(1)/h * w) for every row (scal_recip's two
 * roundings), y = alpha * T(A v). w and y must not overlap (y is the
 * caller's w, w a copy of it: mpg_gemv_n_from_t_nrm2_out_*); A square. The
 * same bits as mpg_scal_recip_nrm2_* followed by mpg_sell_spmv_prog_*. */
int mpg_sell_spmv_norm_f64(mpg_ctx_t ctx, mpg_sell_t A, int32_t nparts, double* h, const double* w, double* v,
                           double alpha, double* y, const mpg_scalar_op* ops, int32_t nops);
int mpg_sell_spmv_norm_f32(mpg_ctx_t ctx, mpg_sell_t A, int32_t nparts, float* h, const float* w, float* v,
                           float alpha, float* y, const mpg_scalar_op* ops, int32_t nops);

/* A^T as its own CSR (SparseMatrix::set_transpose, types_cuda.hpp:145-151;
 * cusparse?csrmv TRANSPOSE, kernels_cuda.cpp:588-596; condest.cpp:49-50).
 * Device outputs: rowptr_t[cols+1]; col_t[nnz] = the source rows; perm[nnz]
 * = the source entry of each transposed entry (values of any precision:
 * mpg_gather_b64/b32 with perm). Stable: a transposed row lists its entries
 * in increasing source row (source entry order for duplicates), so the
 * result is deterministic. Synchronises. */
int mpg_csr_transpose(mpg_ctx_t ctx, int32_t rows, int32_t cols, int64_t nnz, const int32_t* rowptr_dev,
                      const int32_t* col_dev, int32_t* rowptr_t_dev, int32_t* col_t_dev, int32_t* perm_dev);

/* ---- Jacobi preconditioner setup (types.hpp:393-431) ----
 * alpha = max_i sum_j |a_ij| (summed in the values' precision) *
 * FLT_EPSILON; d_i = 1 / boost(a_ii) where the diagonal entry is the first
 * entry of row i whose column >= i (types.hpp:422-425). */
int mpg_jacobi_setup_f64(mpg_ctx_t ctx, mpg_csr_t A, const double* vals, double* diag_out);
int mpg_jacobi_setup_f32(mpg_ctx_t ctx, mpg_csr_t A, const float* vals, float* diag_out);
/* the two halves, for a row-partitioned matrix whose max row sum is
 * all-reduced (max) between them; columns >= rows are halo entries */
int mpg_jacobi_rowmax_f64(mpg_ctx_t ctx, mpg_csr_t A, const double* vals, double* rowmax_dev);
int mpg_jacobi_rowmax_f32(mpg_ctx_t ctx, mpg_csr_t A, const float* vals, double* rowmax_dev);
int mpg_jacobi_diag_f64(mpg_ctx_t ctx, mpg_csr_t A, const double* vals, const double* rowmax_dev, double* diag_out);
int mpg_jacobi_diag_f32(mpg_ctx_t ctx, mpg_csr_t A, const float* vals, const double* rowmax_dev, float* diag_out);

#ifdef __cplusplus
}
#endif
#endif /* MPGMRES_CAPI_H */
