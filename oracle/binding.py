"""ORACLE — test infrastructure only. ctypes binding of oracle/_build/liboracle.so."""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from pathlib import Path

import numpy as np

ORACLE_DIR = Path(__file__).resolve().parent
# MKL's conditional numerical reproducibility: one code branch on every host
# (read by MKL at its first call, so set before the library is used). Without
# it MKL picks its branch by CPU -- AVX-512 on the build container's Xeon, its
# generic branch on the GPU box's EPYC -- and the fp32 sums of a large solve
# differ between the two. COMPATIBLE is the branch MKL 2021.4 runs on the
# EPYC whatever is asked (a request for AVX2 there reports branch AUTO and
# gives COMPATIBLE's bits), so it is the one branch both hosts run: the
# oracle's results are bit-identical on the Xeon and the EPYC at 1, 4 and 8
# threads (tools/oracle_cnr.py, profiles/r05_oracle_cnr/). The CPU baseline in
# bench.py runs on it too -- the branch MKL already ran on the box.
os.environ.setdefault("MKL_CBWR", "COMPATIBLE")
# MPG_ORACLE_LIB: the ASan/UBSan build of the same sources (make -C oracle sanitize)
LIB = Path(os.environ["MPG_ORACLE_LIB"]) if os.environ.get("MPG_ORACLE_LIB") else ORACLE_DIR / "_build" / "liboracle.so"

_lib = None


def build() -> None:
    subprocess.run(["make", "-C", str(ORACLE_DIR)], check=True)


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        if not LIB.exists():
            build()
        _lib = C.CDLL(str(LIB))
        _lib.oracle_backend.restype = C.c_char_p
        _lib.oracle_max_threads.restype = C.c_int
        _lib.oracle_solve.restype = C.c_int
        _lib.oracle_force_loops.argtypes = [C.c_int]
        _lib.oracle_force_loops_mode.argtypes = [C.c_int]
        _lib.oracle_cbwr_branch.restype = C.c_int
        d, f, i, p = C.c_double, C.c_float, C.c_int, C.c_void_p
        _lib.oracle_spmv_f64.argtypes = [i, p, p, p, d, p, d, p]
        _lib.oracle_spmv_f32.argtypes = [i, p, p, p, f, p, f, p]
        _lib.oracle_dot_f64.argtypes = [i, p, p]
        _lib.oracle_dot_f64.restype = d
        _lib.oracle_dot_f32.argtypes = [i, p, p]
        _lib.oracle_dot_f32.restype = f
        _lib.oracle_nrm2_f64.argtypes = [i, p]
        _lib.oracle_nrm2_f64.restype = d
        _lib.oracle_nrm2_f32.argtypes = [i, p]
        _lib.oracle_nrm2_f32.restype = f
        _lib.oracle_gemv_f64.argtypes = [i, i, i, d, p, i, p, d, p]
        _lib.oracle_gemv_f32.argtypes = [i, i, i, f, p, i, p, f, p]
        _lib.oracle_trsv_upper_f64.argtypes = [i, p, i, p]
        _lib.oracle_trsv_upper_f32.argtypes = [i, p, i, p]
        _lib.oracle_rotg_f64.argtypes = [p, p, p, p]
        _lib.oracle_rotg_f32.argtypes = [p, p, p, p]
        _lib.oracle_jacobi_f64.argtypes = [i, p, p, p, p]
        _lib.oracle_jacobi_f32.argtypes = [i, p, p, p, p]
        _lib.oracle_condest.restype = C.c_int
        for t in ("f64", "f32"):
            getattr(_lib, f"oracle_ilu0_{t}").argtypes = [i, p, p, p, p, p]
            getattr(_lib, f"oracle_ilu_apply_{t}").argtypes = [i, p, p, p, i, i, p]
    return _lib


_DEFAULT_THREADS = None


def default_threads() -> int:
    """MKL's thread count when the oracle was first loaded (OMP_NUM_THREADS,
    else the host's), the count of every solve that names none."""
    global _DEFAULT_THREADS
    if _DEFAULT_THREADS is None:
        _DEFAULT_THREADS = max(1, int(lib().oracle_max_threads()))
    return _DEFAULT_THREADS


def cbwr() -> str:
    """The MKL code branch the oracle runs ("AVX2" when pinned; "auto" when
    MKL picks by CPU; "" without MKL)."""
    names = {1: "auto", 3: "COMPATIBLE", 4: "SSE2", 6: "SSSE3", 7: "SSE4_1", 8: "SSE4_2", 9: "AVX", 10: "AVX2",
             12: "AVX512", 14: "AVX512_E1"}
    b = lib().oracle_cbwr_branch()
    return "" if b < 0 else names.get(b, str(b))


def backend() -> str:
    return lib().oracle_backend().decode()


def _ptr(a: np.ndarray) -> int:
    return a.ctypes.data


# the loop kernels' summation of fp32 operands (oracle/cpu_blas.cpp): "loops"
# fp32 products summed in fp64 (rounded once); "seq32" every partial sum in
# fp32, one sequential chain (a scalar CPU BLAS's class and order);
# "pair32" fp32 partial sums in pairwise (tree) order over the long
# reductions (dots, norms, gemv^T) -- the order of a GPU reduction -- and in
# index order over a row of A and over a gemv row's basis columns
LOOP_MODES = {"loops": 0, "seq32": 1, "pair32": 2}


def solve(mpg, A, b, x_true=None, backend=None, **opts):
    """Run the oracle on the same mpg_solve_args the HIP path takes.
    backend="loops" runs this solve on the loop kernels even where MKL loaded
    (fp32 products summed in fp64 in index order -- the summation class of
    the HIP kernels, and the same on every machine; MKL's fp32 sgemv sums in
    fp32 in an order that depends on the CPU and its thread count)."""
    opts = dict(opts)
    opts.pop("engine", None)
    # MKL keeps the last thread count it was given: a solve without one runs
    # on the process's initial count, whatever ran before (tests' order)
    if not opts.get("threads"):
        opts["threads"] = default_threads()
    args, keep = mpg.make_args(A, b, x_true, **opts)
    fn = lib().oracle_solve
    fn.argtypes = [C.POINTER(type(args)), C.POINTER(mpg.SolveResult)]
    if backend not in (None, "mkl") + tuple(LOOP_MODES):
        raise ValueError(f"oracle backend {backend!r}")
    lib().oracle_force_loops_mode(LOOP_MODES.get(backend, -1))
    try:
        return mpg.run_solve(fn, args, A.nrows)
    finally:
        lib().oracle_force_loops_mode(-1)


def spmv(A, x: np.ndarray, alpha=1.0, beta=0.0, y=None, dtype=np.float64) -> np.ndarray:
    x = np.ascontiguousarray(x, dtype=dtype)
    y = np.zeros(A.nrows, dtype=dtype) if y is None else np.array(y, dtype=dtype)
    v = np.ascontiguousarray(A.val, dtype=dtype)
    fn = lib().oracle_spmv_f64 if dtype == np.float64 else lib().oracle_spmv_f32
    fn(A.nrows, _ptr(A.rowptr), _ptr(A.col), _ptr(v), alpha, _ptr(x), beta, _ptr(y))
    return y


def dot(x: np.ndarray, y: np.ndarray):
    if x.dtype == np.float64:
        return lib().oracle_dot_f64(len(x), _ptr(x), _ptr(y))
    return lib().oracle_dot_f32(len(x), _ptr(x), _ptr(y))


def nrm2(x: np.ndarray):
    if x.dtype == np.float64:
        return lib().oracle_nrm2_f64(len(x), _ptr(x))
    return lib().oracle_nrm2_f32(len(x), _ptr(x))


def gemv(trans: bool, A: np.ndarray, x: np.ndarray, alpha=1.0, beta=0.0, y=None) -> np.ndarray:
    """A given as a Fortran-ordered 2-D array (column-major, lda = rows)."""
    A = np.asfortranarray(A)
    rows, cols = A.shape
    out_len = cols if trans else rows
    y = np.zeros(out_len, dtype=A.dtype) if y is None else np.array(y, dtype=A.dtype)
    x = np.ascontiguousarray(x, dtype=A.dtype)
    fn = lib().oracle_gemv_f64 if A.dtype == np.float64 else lib().oracle_gemv_f32
    fn(int(trans), rows, cols, alpha, _ptr(A), rows, _ptr(x), beta, _ptr(y))
    return y


def trsv_upper(H: np.ndarray, y: np.ndarray) -> np.ndarray:
    H = np.asfortranarray(H)
    y = np.array(y, dtype=H.dtype)
    fn = lib().oracle_trsv_upper_f64 if H.dtype == np.float64 else lib().oracle_trsv_upper_f32
    fn(H.shape[0], _ptr(H), H.shape[0], _ptr(y))
    return y


def rotg(a, b, dtype=np.float64):
    v = np.array([a, b, 0, 0], dtype=dtype)
    fn = lib().oracle_rotg_f64 if dtype == np.float64 else lib().oracle_rotg_f32
    it = v.itemsize
    base = v.ctypes.data
    fn(base, base + it, base + 2 * it, base + 3 * it)
    return v  # r, 0, c, s


def jacobi(A, dtype=np.float64) -> np.ndarray:
    d = np.zeros(A.nrows, dtype=dtype)
    fn = lib().oracle_jacobi_f64 if dtype == np.float64 else lib().oracle_jacobi_f32
    fn(A.nrows, _ptr(A.rowptr), _ptr(A.col), _ptr(A.val), _ptr(d))
    return d


def ilu0(A, dtype=np.float64):
    """ILU(0) factors (CSR order) and diagonal positions of A (oracle ilu0)."""
    lu = np.zeros(A.nnz, dtype=dtype)
    di = np.zeros(A.nrows, dtype=np.int32)
    fn = lib().oracle_ilu0_f64 if dtype == np.float64 else lib().oracle_ilu0_f32
    if fn(A.nrows, _ptr(A.rowptr), _ptr(A.col), _ptr(np.ascontiguousarray(A.val, dtype=np.float64)), _ptr(lu),
          _ptr(di)):
        raise ValueError("oracle ilu0 failed")
    return lu, di


def ilu_apply(A, x: np.ndarray, kind="ilu", steps=1, dtype=np.float64) -> np.ndarray:
    """One preconditioner apply M^-1 x with M = ILU(0)(A) ("ilu": exact
    triangular solves; "ilu_jacobi": `steps` Jacobi sweeps per factor)."""
    kinds = {"ilu": 0, "ilu_jacobi": 1}
    x = np.array(x, dtype=dtype)
    fn = lib().oracle_ilu_apply_f64 if dtype == np.float64 else lib().oracle_ilu_apply_f32
    if fn(A.nrows, _ptr(A.rowptr), _ptr(A.col), _ptr(np.ascontiguousarray(A.val, dtype=np.float64)), kinds[kind],
          steps, _ptr(x)):
        raise ValueError("oracle ILU apply failed")
    return x


def condest(mpg, A, rand_seed: int = 42, max_iters: int = 100000, verbose: bool = False, threads: int = 0) -> dict:
    """The CPU restatement of condest.cpp:34-150 (oracle/cpu_condest.cpp);
    same argument/result structs as mpg.condest."""
    from importlib import import_module

    abi = import_module(mpg.__name__ + "._abi")
    a = abi.condest_args(A, rand_seed, max_iters, verbose, 0, threads)
    r = abi.CondestResult()
    if lib().oracle_condest(C.byref(a), C.byref(r)):
        raise RuntimeError(f"oracle_condest failed: {r.message.decode()}")
    return abi.condest_dict(r)
