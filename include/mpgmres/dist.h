/*
 * mpgmres row-partitioned multi-GPU C-ABI (libmpgmres_host.so).
 *
 * The reference runs on one device only (no MPI/NCCL). Here the
 * CSR matrix is split into contiguous row blocks, one per rank (one process
 * and one GPU per rank). Each rank keeps its rows with columns remapped to
 * [0, n_local) for its own rows and [n_local, n_ext) for the "halo" entries
 * owned by other ranks. Per Arnoldi step a rank exchanges only those halo
 * entries with the ranks that own them (RCCL grouped send/recv over xGMI —
 * for a banded matrix a handful of values per neighbour) and all-reduces the
 * fp64 partial sums of the Gram-Schmidt dots and norms, so every rank holds
 * bit-identical H, Givens and convergence scalars and takes the same
 * decisions.
 *
 * Building the plan is transport-neutral and needs no GPU:
 *   mpg_halo_analyze        this rank's rows -> which rows it needs from whom
 *   (exchange the needs with any transport: torch.distributed, MPI, ...)
 *   mpg_halo_set_send       what each peer needs from this rank
 *   mpg_halo_local_cols     the remapped column array
 * then mpg_engine_create_dist builds the fused engine with an RCCL
 * communicator. mpg_solve_loopback runs P ranks as threads sharing one GPU
 * (device-to-device copies instead of RCCL) to test the partitioned path on
 * a single device.
 *
 * Reference correspondence (what each exchange distributes): the halo
 * exchange feeds the Arnoldi spmv (gmres.cpp:213, kernels_cuda.cpp:576-614)
 * and the residual spmv (gmres.cpp:174); the fp64 all-reduces carry the
 * CGS/CGSR gemv^T panels (Orthogonalization.hpp:83-87, 109-136), the MGS
 * dots (Orthogonalization.hpp:99-105), nrm2 (Orthogonalization.hpp:56) and
 * the restart norms (gmres.cpp:168-180); the Jacobi ||A||_inf boost
 * (types.hpp:404-430) is an all-reduce max.
 */
#ifndef MPGMRES_DIST_H
#define MPGMRES_DIST_H

#include <stdint.h>

#include "mpgmres/solve.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct mpg_halo* mpg_halo_t;

/* row_starts: nranks + 1 global row offsets; rowptr/col_global: this rank's
 * n_local rows with global column ids (sorted per row). */
int mpg_halo_analyze(int32_t rank, int32_t nranks, const int64_t* row_starts, int32_t n_local,
                     const int32_t* rowptr, const int32_t* col_global, mpg_halo_t* out);
/* Local numbering (columns and vector layout): own rows [0, n_local), halo
 * rows of lower ranks [-n_front, 0), halo rows of higher ranks
 * [n_local, n_ext); a vector with halo spans n_front + n_ext entries, its
 * row 0 at entry n_front. */
int32_t mpg_halo_n_ext(mpg_halo_t h);
int32_t mpg_halo_n_front(mpg_halo_t h);
/* local id of the first row received from `peer` (its rows are consecutive) */
int32_t mpg_halo_recv_pos(mpg_halo_t h, int32_t peer);
int32_t mpg_halo_recv_count(mpg_halo_t h, int32_t peer);
/* global ids (ascending) of the rows this rank needs from `peer` */
int mpg_halo_recv_rows(mpg_halo_t h, int32_t peer, int64_t* rows_out);
/* global ids of this rank's rows that `peer` needs (its recv list for us) */
int mpg_halo_set_send(mpg_halo_t h, int32_t peer, int32_t count, const int64_t* rows);
/* column array remapped to local ids (nnz entries) */
int mpg_halo_local_cols(mpg_halo_t h, int32_t* col_local_out);
void mpg_halo_free(mpg_halo_t h);

/* RCCL unique id (128 bytes) made by one rank and broadcast by the caller */
int mpg_rccl_unique_id(char* id_out, int len);

/* args: this rank's rows with GLOBAL column ids, local b and x_true; the
 * plan must have every peer's send list set. Collective over all ranks. */
int mpg_engine_create_dist(const mpg_solve_args* args, mpg_halo_t plan, const char* rccl_id, int32_t nranks,
                           int32_t rank, mpg_engine_t* out, char* err, int errlen);

/* Collectives over a caller-supplied host transport: ranks in separate
 * processes that may share one GPU (RCCL refuses that), e.g. driven by
 * torch.distributed over gloo (icl-mixed-precision-gmres_amd/transport.py).
 * Every rank calls the callbacks in the same order. Both return 0 on
 * success. allreduce: in-place sum (op 0) or max (op 1) of `count` doubles,
 * the same bits on every rank. exchange: for every peer q != rank, send
 * send_bytes[q] bytes from send[q] and receive recv_bytes[q] bytes into
 * recv[q] (zero sizes: nothing to move). */
typedef struct {
    void* user;
    int (*allreduce)(void* user, double* buf, int32_t count, int32_t op);
    int (*exchange)(void* user, void* const* send, const int64_t* send_bytes, void* const* recv,
                    const int64_t* recv_bytes);
} mpg_host_transport;

/* mpg_engine_create_dist with the host transport instead of RCCL (the
 * collectives stage through host memory; the cycle runs eagerly). */
int mpg_engine_create_dist_host(const mpg_solve_args* args, mpg_halo_t plan, const mpg_host_transport* transport,
                                int32_t nranks, int32_t rank, mpg_engine_t* out, char* err, int errlen);

/* Degrees of freedom per node of a CSR matrix: 3 when every node row (rows
 * 3r .. 3r + 2) is made of the same column triples c, c + 1, c + 2 in the
 * same storage positions (the node-block copy's condition, node_tile.hpp),
 * else 1. The nnz-balanced row split rounds its rank starts down to node
 * boundaries when it is 3, so every rank keeps whole nodes (and can take the
 * node-block copy). */
int32_t mpg_csr_node_dof(int32_t n, const int32_t* rowptr, const int32_t* col);

/* P ranks as threads on one device, rows split evenly by nnz (at node
 * boundaries, mpg_csr_node_dof); the result
 * (history, counts, norms, x gathered) matches mpg_solve's. */
int mpg_solve_loopback(const mpg_solve_args* args, int32_t nranks, mpg_solve_result* result);

/* What one rank's engine runs on (mpg_solve_loopback_ex): the Arnoldi SpMV
 * storage (mpg_arnoldi_spmv_layout / mpg_arnoldi_sell_columns), the local
 * numbering (dist.h above) and the fp16 cast's scaled rows. */
typedef struct {
    int32_t format;           /* 1 CSR row blocks, 2 SELL-64, 3 node blocks */
    int32_t col_form;         /* SELL columns: -1 none, 0 int32, 1 int16, 2 stepped int16 */
    int32_t vec_width;
    int32_t window;           /* 1: the SpMV reads v_k from the LDS window */
    int32_t n_local, n_front, n_ext;
    int32_t givens_folded;    /* 1: this rank folds the Givens step into the next SpMV (the
                                 same on every rank: decided collectively at create) */
    int64_t row0;             /* first global row */
    int64_t csr_slices, implicit_slices;
    int64_t half_rows_scaled; /* mixed-half: rows scaled by a power of two */
    int32_t device;           /* the HIP device the rank ran on */
    int32_t transport_ranks;  /* ranks its communicator reports (RCCL: ncclCommCount) */
} mpg_rank_layout;
/* mpg_solve_loopback, reporting each rank's layout (layouts: nranks entries, may be NULL) */
int mpg_solve_loopback_ex(const mpg_solve_args* args, int32_t nranks, mpg_solve_result* result,
                          mpg_rank_layout* layouts);

/* One process, `ngpus` ranks: rank q is a host thread on device devices[q]
 * (devices NULL: 0..ngpus-1), rows split evenly by nnz as in
 * mpg_solve_loopback, collectives over one RCCL clique made by
 * ncclCommInitAll (the CLI's --ngpus). The result matches
 * mpg_solve's (x gathered from every rank, history from rank 0). Fails with
 * MPG_ERR_ARG and a message when fewer devices are visible than requested or
 * a device is named twice (RCCL runs one rank per GPU), MPG_ERR_RCCL when the
 * clique cannot be made. layouts: ngpus entries, may be NULL. */
int mpg_solve_multi_gpu(const mpg_solve_args* args, int32_t ngpus, const int32_t* devices, mpg_solve_result* result,
                        mpg_rank_layout* layouts);

#ifdef __cplusplus
}
#endif
#endif /* MPGMRES_DIST_H */
