// CSR transpose on gfx950: the structure behind spmv with a transposed
// SparseMatrix (SparseMatrix::set_transpose, types_cuda.hpp:145-151, used by
// condest.cpp:49-50 and applied by cusparse?csrmv with
// CUSPARSE_OPERATION_TRANSPOSE, kernels_cuda.cpp:588-596).
//
// Instead of a scatter-with-atomics SpMV for A^T x (run-to-run different
// rounding), A^T is formed once as its own CSR: a stable LSD radix sort of
// the column indices carrying the entry index (rocPRIM), so the entries of
// each transposed row come in increasing source row, then the row starts by
// a boundary scan of the sorted keys. The values follow through `perm`
// (mpg_gather_b32/b64), so every precision of one matrix shares the
// structure. A^T x then runs on the ordinary CSR-adaptive SpMV.
#include <rocprim/device/device_radix_sort.hpp>

#include "internal.hpp"

namespace {

using namespace mpg;

__global__ void k_iota(int64_t n, int32_t* __restrict__ out) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        out[i] = (int32_t)i;
}

// source row of every entry (a wave per row, entries written coalesced)
__global__ void k_row_of_entry(int32_t rows, const int32_t* __restrict__ rowptr, int32_t* __restrict__ row_of) {
    const int lane = threadIdx.x & (kWave - 1);
    const int64_t waves = (int64_t)gridDim.x * (blockDim.x / kWave);
    for (int64_t r = blockIdx.x * (int64_t)(blockDim.x / kWave) + threadIdx.x / kWave; r < rows; r += waves)
        for (int32_t j = rowptr[r] + lane; j < rowptr[r + 1]; j += kWave) row_of[j] = (int32_t)r;
}

// rowptr_t[c] = first position of key >= c in the sorted keys: position t
// writes every c in (key[t-1], key[t]] (key[-1] = -1, key[nnz] = cols)
__global__ void k_key_bounds(int64_t nnz, int32_t cols, const uint32_t* __restrict__ key,
                             int32_t* __restrict__ rowptr_t) {
    for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t <= nnz; t += (int64_t)gridDim.x * blockDim.x) {
        const int64_t prev = t == 0 ? -1 : (int64_t)key[t - 1];
        const int64_t cur = t == nnz ? (int64_t)cols : (int64_t)key[t];
        for (int64_t c = prev + 1; c <= cur; ++c) rowptr_t[c] = (int32_t)t;
    }
}

// col_t[t] = source row of the entry moved to t
__global__ void k_perm_rows(int64_t nnz, const int32_t* __restrict__ perm, const int32_t* __restrict__ row_of,
                            int32_t* __restrict__ col_t) {
    for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < nnz; t += (int64_t)gridDim.x * blockDim.x)
        col_t[t] = row_of[perm[t]];
}

int key_bits(int32_t cols) {
    int b = 1;
    while (b < 31 && (int64_t(1) << b) < cols) ++b;
    return b;
}

}  // namespace

extern "C" int mpg_csr_transpose(mpg_ctx_t ctx, int32_t rows, int32_t cols, int64_t nnz, const int32_t* rowptr,
                                 const int32_t* col, int32_t* rowptr_t, int32_t* col_t, int32_t* perm) {
    if (!ctx || rows < 0 || cols < 0 || nnz < 0 || nnz > INT32_MAX || !rowptr || !rowptr_t) return MPG_ERR_ARG;
    if (nnz > 0 && (!col || !col_t || !perm)) return MPG_ERR_ARG;
    MPG_HIP(ctx, hipSetDevice(ctx->device));
    hipStream_t st = ctx->stream;
    if (nnz == 0) {
        MPG_HIP(ctx, hipMemsetAsync(rowptr_t, 0, sizeof(int32_t) * ((size_t)cols + 1), st));
        MPG_HIP(ctx, hipStreamSynchronize(st));
        return MPG_OK;
    }
    // scratch: iota values, sorted keys, row of every entry, radix temp
    int32_t* idx = nullptr;
    uint32_t* key_sorted = nullptr;
    int32_t* row_of = nullptr;
    void* temp = nullptr;
    size_t temp_bytes = 0;
    const int bits = key_bits(cols);
    int status = MPG_OK;
    auto fail = [&](hipError_t e, const char* what) {
        status = set_hip_error(ctx, e, what);
    };
    hipError_t e;
    if ((e = hipMalloc(&idx, sizeof(int32_t) * nnz)) != hipSuccess) fail(e, "hipMalloc");
    if (!status && (e = hipMalloc(&key_sorted, sizeof(uint32_t) * nnz)) != hipSuccess) fail(e, "hipMalloc");
    if (!status && (e = hipMalloc(&row_of, sizeof(int32_t) * nnz)) != hipSuccess) fail(e, "hipMalloc");
    if (!status && (e = rocprim::radix_sort_pairs(nullptr, temp_bytes, reinterpret_cast<const uint32_t*>(col),
                                                  key_sorted, idx, perm, (size_t)nnz, 0, bits, st)) != hipSuccess)
        fail(e, "rocprim::radix_sort_pairs (size)");
    if (!status && (e = hipMalloc(&temp, temp_bytes ? temp_bytes : 1)) != hipSuccess) fail(e, "hipMalloc");
    if (!status) {
        const int g = grid_for(nnz, 4);
        k_iota<<<g, kBlock, 0, st>>>(nnz, idx);
        k_row_of_entry<<<grid_for((int64_t)rows * kWave, 1, 4096), kBlock, 0, st>>>(rows, rowptr, row_of);
        if ((e = hipGetLastError()) != hipSuccess) fail(e, "kernel launch");
    }
    if (!status && (e = rocprim::radix_sort_pairs(temp, temp_bytes, reinterpret_cast<const uint32_t*>(col),
                                                  key_sorted, idx, perm, (size_t)nnz, 0, bits, st)) != hipSuccess)
        fail(e, "rocprim::radix_sort_pairs");
    if (!status) {
        const int g = grid_for(nnz + 1, 4);
        k_key_bounds<<<g, kBlock, 0, st>>>(nnz, cols, key_sorted, rowptr_t);
        k_perm_rows<<<g, kBlock, 0, st>>>(nnz, perm, row_of, col_t);
        if ((e = hipGetLastError()) != hipSuccess) fail(e, "kernel launch");
    }
    if (!status && (e = hipStreamSynchronize(st)) != hipSuccess) fail(e, "hipStreamSynchronize");
    (void)hipStreamSynchronize(st);  // scratch is freed only after the stream drained
    (void)hipFree(temp);
    (void)hipFree(row_of);
    (void)hipFree(key_sorted);
    (void)hipFree(idx);
    return status;
}
