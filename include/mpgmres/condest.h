/*
 * mpgmres condition-number estimator C-ABI (libmpgmres_host.so): the
 * reference's offline `condest` tool (condest.cpp:36-179) on MI355X.
 *
 * sigma_max by power iteration (condest.cpp:153-164, klein_lu_bound(0.1,
 * 1e-12, n) steps, condest.cpp:28-31); sigma_min by LSQR on A x = A x_exact
 * with a random x_exact, keeping the smallest ||A d|| / ||d|| over the error
 * vectors d = x_exact - x_t (condest.cpp:34-150). Stopping rule, constants
 * and stdout lines as the reference (it runs only with --gpu; the CPU branch
 * prints "CPU not currently supported", condest.cpp:217-223).
 *
 * A^T u runs on an explicitly transposed CSR (mpg_csr_transpose), not a
 * scatter: the transposed product is deterministic.
 */
#ifndef MPGMRES_CONDEST_H
#define MPGMRES_CONDEST_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
    /* square CSR matrix, 0-based int32 indices, fp64 values (host memory) */
    int32_t n;
    int64_t nnz;
    const int32_t* rowptr;
    const int32_t* col;
    const double* val;
    int32_t rand_seed;   /* --rand (condest.cpp:185, default 42) */
    int64_t max_iters;   /* --max-iters (condest.cpp:187, default 100000) */
    int32_t verbose;     /* print the reference's stdout lines */
    int32_t device;      /* HIP device (mpg_condest only) */
    int32_t threads;     /* host threads (oracle only; 0 = default) */
} mpg_condest_args;

typedef struct {
    int32_t status;        /* 0 ok, < 0 error (message) */
    double sigma_max;      /* last power-iteration norm */
    double sigma_min;      /* smallest ||A d|| / ||d|| seen */
    double cond;           /* sigma_max / sigma_min */
    int64_t power_iters;   /* klein_lu_bound(0.1, 1e-12, n) */
    int64_t iters;         /* the `t` printed as "<t> iterations total" */
    int64_t finish_t;      /* t at which the stopping test fired (0: never) */
    int32_t stop_reason;   /* 0 ran to T, 1 ||d|| == 0, 2 ||A d|| is NaN */
    double seconds;        /* wall time of the estimator (after set-up) */
    char message[256];
} mpg_condest_result;

int mpg_condest(const mpg_condest_args* args, mpg_condest_result* result);

#ifdef __cplusplus
}
#endif
#endif /* MPGMRES_CONDEST_H */
