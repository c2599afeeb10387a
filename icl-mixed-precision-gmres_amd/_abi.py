"""ctypes mirrors of the C-ABI structs in include/mpgmres/{solve,problems}.h.

Field order and types must match the headers exactly.
"""
import ctypes as C

MODES = {"mixed": 0, "baseline": 1, "single-prec": 2, "single": 3, "mixed-half": 4}
ORTHS = {"cgs": 0, "mgs": 1, "cgsr": 2}
PRECS = {"ilu": 0, "ilu_jacobi": 1, "jacobi": 2, "identity": 3}
ENGINES = {"surface": 0, "fused": 1}
SPMV_FORMATS = {"auto": 0, "csr": 1, "sell": 2, "node": 3}
ACCUMS = {"f64": 0, "f32": 1}  # mpg_solve_args.accum (MPG_ACCUM_F64 / MPG_ACCUM_F32, arnoldi.h)
STATUS = {1: "converged", 3: "aborted", -1: "error"}


class SolveArgs(C.Structure):
    _fields_ = [
        ("n", C.c_int32),
        ("nnz", C.c_int64),
        ("rowptr", C.POINTER(C.c_int32)),
        ("col", C.POINTER(C.c_int32)),
        ("val", C.POINTER(C.c_double)),
        ("b", C.POINTER(C.c_double)),
        ("x_true", C.POINTER(C.c_double)),
        ("mode", C.c_int32),
        ("orth", C.c_int32),
        ("prec", C.c_int32),
        ("engine", C.c_int32),
        ("rlen", C.c_int32),
        ("tol", C.c_double),
        ("max_restarts", C.c_int64),
        ("rtol", C.c_double),
        ("repeat_iter", C.c_int32),
        ("orthloss", C.c_int32),
        ("jacobi_steps", C.c_int32),
        ("verbose", C.c_int32),
        ("device", C.c_int32),
        ("threads", C.c_int32),
        ("spmv_format", C.c_int32),
        ("half_unscaled", C.c_int32),
        ("stop_on_breakdown", C.c_int32),
        ("accum", C.c_int32),
    ]


class SolveResult(C.Structure):
    _fields_ = [
        ("status", C.c_int32),
        ("restarts", C.c_int64),
        ("inner_k", C.c_int64),
        ("total_iters", C.c_int64),
        ("res_norm", C.c_double),
        ("err_norm", C.c_double),
        ("gmres_seconds", C.c_double),
        ("setup_seconds", C.c_double),
        ("minvb_norm", C.c_double),
        ("x_out", C.POINTER(C.c_double)),
        ("cycle_cap", C.c_int64),
        ("n_cycles", C.c_int64),
        ("cyc_r_norm", C.POINTER(C.c_double)),
        ("cyc_normalization", C.POINTER(C.c_double)),
        ("cyc_beta", C.POINTER(C.c_double)),
        ("step_cap", C.c_int64),
        ("n_steps", C.c_int64),
        ("step_res", C.POINTER(C.c_double)),
        ("step_cycle", C.POINTER(C.c_int32)),
        ("message", C.c_char * 256),
        ("nonfinite_steps", C.c_int64),
        ("nonfinite_cycles", C.c_int64),
        ("first_nonfinite_step", C.c_int64),
    ]


class HostCsr(C.Structure):
    _fields_ = [
        ("nrows", C.c_int32),
        ("ncols", C.c_int32),
        ("nnz", C.c_int64),
        ("rowptr", C.POINTER(C.c_int32)),
        ("col", C.POINTER(C.c_int32)),
        ("val", C.POINTER(C.c_double)),
    ]


class CondestArgs(C.Structure):  # include/mpgmres/condest.h
    _fields_ = [
        ("n", C.c_int32),
        ("nnz", C.c_int64),
        ("rowptr", C.POINTER(C.c_int32)),
        ("col", C.POINTER(C.c_int32)),
        ("val", C.POINTER(C.c_double)),
        ("rand_seed", C.c_int32),
        ("max_iters", C.c_int64),
        ("verbose", C.c_int32),
        ("device", C.c_int32),
        ("threads", C.c_int32),
    ]


class CondestResult(C.Structure):
    _fields_ = [
        ("status", C.c_int32),
        ("sigma_max", C.c_double),
        ("sigma_min", C.c_double),
        ("cond", C.c_double),
        ("power_iters", C.c_int64),
        ("iters", C.c_int64),
        ("finish_t", C.c_int64),
        ("stop_reason", C.c_int32),
        ("seconds", C.c_double),
        ("message", C.c_char * 256),
    ]


def condest_args(A, rand_seed: int = 42, max_iters: int = 100000, verbose: bool = False, device: int = 0,
                 threads: int = 0) -> CondestArgs:
    """Arguments for mpg_condest / oracle_condest; keeps references to A's
    arrays on the struct so they outlive the call."""
    a = CondestArgs()
    a.n, a.nnz = A.nrows, A.nnz
    a.rowptr = A.rowptr.ctypes.data_as(C.POINTER(C.c_int32))
    a.col = A.col.ctypes.data_as(C.POINTER(C.c_int32))
    a.val = A.val.ctypes.data_as(C.POINTER(C.c_double))
    a.rand_seed, a.max_iters, a.verbose, a.device, a.threads = rand_seed, max_iters, int(verbose), device, threads
    a._keep = A
    return a


def condest_dict(r: CondestResult) -> dict:
    return {k: getattr(r, k) for k, _ in CondestResult._fields_ if k != "message"}


class RankLayout(C.Structure):
    """mpg_rank_layout (dist.h): one rank's Arnoldi SpMV storage and numbering."""
    _fields_ = [
        ("format", C.c_int32),
        ("col_form", C.c_int32),
        ("vec_width", C.c_int32),
        ("window", C.c_int32),
        ("n_local", C.c_int32),
        ("n_front", C.c_int32),
        ("n_ext", C.c_int32),
        ("givens_folded", C.c_int32),
        ("row0", C.c_int64),
        ("csr_slices", C.c_int64),
        ("implicit_slices", C.c_int64),
        ("half_rows_scaled", C.c_int64),
        ("device", C.c_int32),
        ("transport_ranks", C.c_int32),
    ]
