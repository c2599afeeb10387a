/*
 * Problem construction on the host (C-ABI): synthetic CSR generators, the
 * Matrix Market loader with the reference's semantics, the reference's
 * seeded random vector, and a plain fp64 host SpMV (b = A x_true).
 */
#ifndef MPGMRES_PROBLEMS_H
#define MPGMRES_PROBLEMS_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Host CSR, 0-based int32 indices, fp64 values; arrays malloc'd by the
 * library, released with mpg_host_csr_free. `nrows` rows of a matrix with
 * `ncols` columns (a row slice of a larger matrix keeps global columns). */
typedef struct {
    int32_t nrows, ncols;
    int64_t nnz;
    int32_t* rowptr;
    int32_t* col;
    double* val;
} mpg_host_csr;

void mpg_host_csr_free(mpg_host_csr* a);

/* Banded matrix of order n with column offsets -lo..+hi. Rows
 * [row_begin, row_end) are generated (global column ids). Off-diagonals are
 * -u with u in [0,1) from a counter-based hash of (seed, row, offset), so any
 * row slice is identical to the same rows of the whole matrix; the diagonal
 * is 1 + sum |off| (strict diagonal dominance). lo=5, hi=4, n=1e6 gives the
 * 9,999,975-nnz "BAND-10M" input of BASELINE.md. */
int mpg_gen_band(int64_t n, int32_t lo, int32_t hi, uint64_t seed, int64_t row_begin, int64_t row_end,
                 mpg_host_csr* out);

/* 7-point 3-D Laplacian on an nx*ny*nz grid, lexicographic order
 * (x fastest), diagonal 6, off-diagonals -1 (100^3: n = 1e6, nnz = 6,940,000). */
int mpg_gen_laplace3d(int32_t nx, int32_t ny, int32_t nz, mpg_host_csr* out);

/* 27-point 3-D stencil with `dof` unknowns per node (every unknown of a
 * node coupled to every unknown of its <= 27 neighbours), lexicographic
 * node order, symmetric off-diagonals -u (u from a counter-based hash of
 * the unordered pair), diagonal 1 + sum|off| (SPD, diagonally dominant).
 * The Queen_4147 stand-in of SURVEY §8(d): 111^3 nodes x 3 dof = 4,102,893
 * rows, ~3.2e8 nnz. */
int mpg_gen_stencil27(int32_t nx, int32_t ny, int32_t nz, int32_t dof, uint64_t seed, mpg_host_csr* out);

/* FEM-like irregular stand-in: the 27-point node coupling of
 * mpg_gen_stencil27 with each undirected node pair kept with probability
 * keep_pct / 100 (a hash of the pair, so the pattern is symmetric): rows of
 * dof x (1 + kept neighbours) entries, i.e. variable lengths (24..81 at dof 3
 * and most keep values). Values as mpg_gen_stencil27 (symmetric, diagonal
 * 1 + sum|off|). */
int mpg_gen_fem27(int32_t nx, int32_t ny, int32_t nz, int32_t dof, int32_t keep_pct, uint64_t seed,
                  mpg_host_csr* out);
/* perm[old] = new for nodes * dof unknowns: blocks of `block` consecutive
 * nodes placed in a seeded random order (mt19937_64), nodes shuffled within
 * each block, a node's dof kept together — a mesh-like ordering with local
 * runs and scattered neighbours (Queen_4147-like), not a uniform scatter. */
int mpg_perm_node_blocks(int64_t nodes, int32_t dof, int32_t block, uint64_t seed, int32_t* perm);
/* B = P A P^T (row perm[i] of B = row i of A, columns c -> perm[c], each row
 * sorted by column): the same spectrum under a symmetric renumbering. */
int mpg_csr_permute_sym(const mpg_host_csr* a, const int32_t* perm, mpg_host_csr* out);

/* One of the generators above from a CLI spec: "band:N[:LO:HI[:SEED]]"
 * (defaults 5, 4, 7), "laplace:NX[:NY:NZ]", "stencil27:NX[:DOF[:SEED]]"
 * (defaults 3, 11), "stencil27p:NX[:DOF[:SEED[:BLOCK[:PSEED]]]]" (stencil27
 * under mpg_perm_node_blocks; defaults block 64, pseed 5),
 * "fem27:NX[:DOF[:KEEP%[:SEED[:BLOCK[:PSEED]]]]]" (defaults 3, 70, 13, 0 =
 * natural order, 5). Returns 0, or -2 with a message in err. */
int mpg_gen_spec(const char* spec, mpg_host_csr* out, char* err, int errlen);

/* Matrix Market coordinate real|integer, general|symmetric, loaded as
 * LoadMatrix.hpp:17-154 does: an explicit diagonal slot in every row (0 if
 * the file has none; a diagonal entry in the file overwrites it), symmetric
 * entries mirrored, each row sorted by column with a stable sort.
 * Returns 0, or < 0 with a message in `err` (size errlen). */
int mpg_load_mtx(const char* path, mpg_host_csr* out, char* err, int errlen);

/* Dense Matrix Market vector (array or coordinate, column `col`), as
 * LoadVector (LoadMatrix.hpp:156-233). `out` must hold `n` entries. */
int mpg_load_mtx_vector(const char* path, int32_t col, double* out, int64_t n, char* err, int errlen);

/* gmres_perf_test.cpp:39-51: std::mt19937(seed) and
 * std::uniform_real_distribution<float>, one draw per entry, widened to double. */
int mpg_rand_vect(int64_t n, uint32_t seed, double* out);

/* y = A x, fp64, sequential row sums (host). */
int mpg_host_spmv(const mpg_host_csr* a, const double* x, double* y);

#ifdef __cplusplus
}
#endif
#endif /* MPGMRES_PROBLEMS_H */
