"""ORACLE — test infrastructure only. Never imported by the product.

The reference's Matrix Market reading, run with the reference's own parser:
mm_read_banner / mm_read_mtx_crd_size from /root/reference/mmio.c compiled
as-is into oracle/_ref/libmmio_ref.so (oracle/Makefile), and the entry loop
of LoadMatrix.hpp:62-80 through libc's fscanf with its exact format. The CSR
assembly that follows in LoadMatrix.hpp:82-146 (a diagonal slot per row,
symmetric mirroring, then a per-row bubble sort on the column) is restated
here in Python. tests/test_mmio_ref.py compares mpg_load_mtx with it.
"""
import ctypes as C
from pathlib import Path

import numpy as np

LIB = Path(__file__).resolve().parent / "_ref" / "libmmio_ref.so"
# mmio.h:79-85
MM_PREMATURE_EOF, MM_NO_HEADER, MM_UNSUPPORTED_TYPE = 12, 14, 15

_libc = C.CDLL(None)
_libc.fopen.restype = C.c_void_p
_libc.fopen.argtypes = [C.c_char_p, C.c_char_p]
_libc.fclose.argtypes = [C.c_void_p]


def available() -> bool:
    return LIB.exists()


def _lib():
    lib = C.CDLL(str(LIB))
    lib.mm_read_banner.argtypes = [C.c_void_p, C.c_char_p]
    lib.mm_read_mtx_crd_size.argtypes = [C.c_void_p] + [C.POINTER(C.c_int)] * 3
    return lib


def load_matrix(path: str):
    """LoadMatrix<double>(file) (LoadMatrix.hpp:17-154): returns (M, N,
    rowptr, col, val) or raises ValueError with the reference's message."""
    lib = _lib()
    f = _libc.fopen(str(path).encode(), b"r")
    if not f:
        raise ValueError("Could not access file")
    try:
        code = C.create_string_buffer(4)
        err = lib.mm_read_banner(f, code)
        if err:
            raise ValueError({MM_PREMATURE_EOF: "Missing values in banner", MM_NO_HEADER: "Banner is missing",
                              MM_UNSUPPORTED_TYPE: "Unrecognized description"}.get(
                                  err, "Malformed banner with unknown error code"))
        M, N, nnz = C.c_int(), C.c_int(), C.c_int()
        if lib.mm_read_mtx_crd_size(f, C.byref(M), C.byref(N), C.byref(nnz)) != 0:
            raise ValueError("Malformed matrix size information")
        t = code.raw
        # mm_is_coordinate && (real || integer) && (general || symmetric)
        if not (t[1:2] == b"C" and t[2:3] in (b"R", b"I") and t[3:4] in (b"G", b"S")):
            raise ValueError("Unsupported matrix type")
        symmetric = t[3:4] == b"S"
        M, N, nnz = M.value, N.value, nnz.value
        I, J, V = np.empty(nnz, np.int64), np.empty(nnz, np.int64), np.empty(nnz)
        ii, jj, vv = C.c_int(), C.c_int(), C.c_double()
        for k in range(nnz):  # LoadMatrix.hpp:67-70, fscanf(in, "%d %d %lg\n", ...)
            _libc.fscanf(C.c_void_p(f), b"%d %d %lg\n", C.byref(ii), C.byref(jj), C.byref(vv))
            I[k], J[k], V[k] = ii.value - 1, jj.value - 1, vv.value
    finally:
        _libc.fclose(f)
    return (M, N) + assemble(N, I, J, V, symmetric)


def assemble(N, I, J, V, symmetric):
    """LoadMatrix.hpp:61-146: every row gets a diagonal slot first (value 0
    unless the file sets it; a repeated diagonal keeps the last), off-diagonal
    entries (and their mirrors) follow in file order, then each row is bubble
    sorted on the column (stable: equal columns keep file order)."""
    off = I != J
    counts = np.ones(N, np.int64)
    np.add.at(counts, I[off], 1)
    if symmetric:
        np.add.at(counts, J[off], 1)
    rowptr = np.zeros(N + 1, np.int64)
    rowptr[1:] = np.cumsum(counts)
    col = np.full(rowptr[-1], -1, np.int64)
    val = np.zeros(rowptr[-1])
    fill = np.ones(N, np.int64)
    col[rowptr[:-1]] = np.arange(N)
    for k in range(len(I)):
        r, c, v = int(I[k]), int(J[k]), V[k]
        if r == c:
            val[rowptr[r]] = v
            continue
        col[rowptr[r] + fill[r]], val[rowptr[r] + fill[r]] = c, v
        fill[r] += 1
        if symmetric:
            col[rowptr[c] + fill[c]], val[rowptr[c] + fill[c]] = r, v
            fill[c] += 1
    for r in range(N):  # the bubble sort is stable: a stable argsort gives the same order
        a, b = rowptr[r], rowptr[r + 1]
        order = np.argsort(col[a:b], kind="stable")
        col[a:b], val[a:b] = col[a:b][order], val[a:b][order]
    return rowptr, col, val


def load_vector(path: str, col: int = 0) -> np.ndarray:
    """LoadVector<double>(file, col) (LoadMatrix.hpp:156-233) with the
    reference's mmio.c banner/size readers and its fscanf formats."""
    lib = _lib()
    lib.mm_read_mtx_array_size.argtypes = [C.c_void_p] + [C.POINTER(C.c_int)] * 2
    f = _libc.fopen(str(path).encode(), b"r")
    if not f:
        raise ValueError("Could not access file")
    try:
        code = C.create_string_buffer(4)
        err = lib.mm_read_banner(f, code)
        if err:
            raise ValueError({MM_PREMATURE_EOF: "Missing values in banner", MM_NO_HEADER: "Banner is missing",
                              MM_UNSUPPORTED_TYPE: "Unrecognized description"}.get(
                                  err, "Malformed banner with unknown error code"))
        array = code.raw[1:2] == b"A"
        M, N, nnz = C.c_int(), C.c_int(), C.c_int()
        err = (lib.mm_read_mtx_array_size(f, C.byref(M), C.byref(N)) if array
               else lib.mm_read_mtx_crd_size(f, C.byref(M), C.byref(N), C.byref(nnz)))
        if err:
            raise ValueError("Malformed matrix size information")
        if col >= N.value:
            raise ValueError(f"Column {col} is too large for the {N.value} vectors")
        out = np.zeros(M.value)
        d = C.c_double()
        if array:  # LoadMatrix.hpp:197-209
            for _ in range(col * M.value):
                _libc.fscanf(C.c_void_p(f), b"%lf\n", C.byref(d))
            for j in range(M.value):
                _libc.fscanf(C.c_void_p(f), b"%lf\n", C.byref(d))
                out[j] = d.value
        else:  # LoadMatrix.hpp:210-222
            ii, jj = C.c_int(), C.c_int()
            for _ in range(nnz.value):
                _libc.fscanf(C.c_void_p(f), b"%d %d %lg\n", C.byref(ii), C.byref(jj), C.byref(d))
                if jj.value - 1 == col:
                    out[ii.value - 1] = d.value
    finally:
        _libc.fclose(f)
    return out
