"""mpgmres_amd — MI355X-native mixed-precision restarted GMRES hot path.

Python host mirror of the reference's solve interface (gmres_perf_test.cpp
flags / run_tests) over the C-ABI libraries built by this package:

  lib/libmpgmres_hip.so   gfx950 HIP kernels (include/mpgmres/capi.h)
  lib/libmpgmres_host.so  operator surface + drivers + solve C-ABI
                          (include/mpgmres/solve.h, problems.h)

There is no CPU fallback: if the HIP libraries are missing, every entry
point raises. The directory name is not a Python identifier, so load it with
`load_package()` from bench.py / tests (it registers as `mpgmres_amd`).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from dataclasses import dataclass, field
from pathlib import Path
from typing import Optional

import numpy as np

from ._abi import (ACCUMS, ENGINES, MODES, ORTHS, PRECS, SPMV_FORMATS, STATUS, CondestResult, HostCsr, RankLayout, SolveArgs, SolveResult,
                   condest_args, condest_dict)

PKG_DIR = Path(__file__).resolve().parent
REPO_DIR = PKG_DIR.parent
LIB_DIR = PKG_DIR / "lib"
HIP_LIB = LIB_DIR / "libmpgmres_hip.so"
HOST_LIB = LIB_DIR / "libmpgmres_host.so"
CLI = PKG_DIR / "bin" / "gmres_perf_test"


def build(jobs: int = 8) -> None:
    """Compile the HIP + host libraries for gfx950 (hipcc cross-compiles; no GPU needed)."""
    subprocess.run(["make", "-C", str(PKG_DIR), f"-j{jobs}"], check=True)


_libs: dict = {}
_runtime: dict = {}


def _torch_lib_dir() -> Optional[Path]:
    """torch/lib of an installed PyTorch, found without importing torch."""
    import importlib.util

    try:
        spec = importlib.util.find_spec("torch")
    except (ImportError, ValueError):
        return None
    if spec is None or not spec.submodule_search_locations:
        return None
    d = Path(list(spec.submodule_search_locations)[0]) / "lib"
    return d if (d / "libamdhip64.so").exists() else None


def _bind_hip_runtime() -> None:
    """Fix the process's HIP runtime, and PyTorch's place in it, before the
    package's libraries load and before anything initialises the GPU.

    The libraries need libamdhip64.so.7 and librccl.so.1 by soname; PyTorch
    bundles its own HIP runtime and RCCL and needs them by the file names
    libamdhip64.so / librccl.so. A process that loaded this package first,
    ran on the GPU, and imported torch afterwards aborted at exit with
    "double free or corruption" (SIGABRT; tools/exit_probe.py
    package_then_torch, profiles/r06_exit/) -- both with
    /opt/rocm's runtime bound (two HIP and HSA runtimes in one process) and
    with PyTorch's bound by file before the package: what the abort needs is
    PyTorch's libraries loaded after the HIP runtime initialised. Importing
    torch first never aborted (every bench and test process). So when
    PyTorch is installed the package imports it here, first: one runtime
    (PyTorch's), PyTorch's teardown in the order its own processes use.
    MPG_HIP_RUNTIME=system skips it and binds /opt/rocm's runtime (a
    process that will never import torch; the CLI's configuration)."""
    if _runtime:
        return
    choice = os.environ.get("MPG_HIP_RUNTIME", "auto")
    d = _torch_lib_dir() if choice in ("auto", "torch") else None
    if choice == "torch" and d is None:
        raise RuntimeError("MPG_HIP_RUNTIME=torch but no PyTorch installation with a HIP runtime was found")
    if d is not None:
        import torch  # noqa: F401  (first: see above)

        _runtime["hip"] = str(d / "libamdhip64.so")
    else:
        _runtime["hip"] = "system"


def hip_runtime() -> str:
    """The HIP runtime the package's libraries are bound to: the path of
    PyTorch's bundled libamdhip64.so, or "system" (/opt/rocm, by soname)."""
    _bind_hip_runtime()
    return _runtime["hip"]


def _lib(name: str) -> C.CDLL:
    if name in _libs:
        return _libs[name]
    _bind_hip_runtime()
    path = HIP_LIB if name == "hip" else HOST_LIB
    if name == "hip" and os.environ.get("MPG_HIP_LIB"):  # A/B of two kernel builds (tools/ab_bench.sh)
        path = Path(os.environ["MPG_HIP_LIB"])
    if name == "host" and os.environ.get("MPG_HOST_LIB"):  # the ASan/UBSan build (make sanitize)
        path = Path(os.environ["MPG_HOST_LIB"])
    if not path.exists():
        raise RuntimeError(f"{path} is missing: run build() (make -C {PKG_DIR}) — there is no CPU fallback")
    if name == "host":
        _lib("hip")
    lib = C.CDLL(str(path), mode=C.RTLD_GLOBAL)
    _libs[name] = lib
    if name == "host":
        _declare_host(lib)
    else:
        _declare_hip(lib)
    return lib


def hip_lib() -> C.CDLL:
    return _lib("hip")


def host_lib() -> C.CDLL:
    return _lib("host")


_P = C.c_void_p
_I64 = C.c_int64
_I32 = C.c_int32


def _declare_host(lib: C.CDLL) -> None:
    lib.mpg_solve.argtypes = [C.POINTER(SolveArgs), C.POINTER(SolveResult)]
    lib.mpg_solve.restype = C.c_int
    lib.mpg_gen_band.argtypes = [_I64, _I32, _I32, C.c_uint64, _I64, _I64, C.POINTER(HostCsr)]
    lib.mpg_gen_laplace3d.argtypes = [_I32, _I32, _I32, C.POINTER(HostCsr)]
    lib.mpg_gen_spec.argtypes = [C.c_char_p, C.POINTER(HostCsr), C.c_char_p, C.c_int]
    lib.mpg_condest.restype = C.c_int
    lib.mpg_gen_stencil27.argtypes = [_I32, _I32, _I32, _I32, C.c_uint64, C.POINTER(HostCsr)]
    lib.mpg_gen_fem27.argtypes = [_I32, _I32, _I32, _I32, _I32, C.c_uint64, C.POINTER(HostCsr)]
    lib.mpg_perm_node_blocks.argtypes = [C.c_int64, _I32, _I32, C.c_uint64, C.POINTER(C.c_int32)]
    lib.mpg_csr_permute_sym.argtypes = [C.POINTER(HostCsr), C.POINTER(C.c_int32), C.POINTER(HostCsr)]
    lib.mpg_load_mtx.argtypes = [C.c_char_p, C.POINTER(HostCsr), C.c_char_p, C.c_int]
    lib.mpg_load_mtx_vector.argtypes = [C.c_char_p, _I32, C.POINTER(C.c_double), _I64, C.c_char_p, C.c_int]
    lib.mpg_rand_vect.argtypes = [_I64, C.c_uint32, C.POINTER(C.c_double)]
    lib.mpg_host_spmv.argtypes = [C.POINTER(HostCsr), C.POINTER(C.c_double), C.POINTER(C.c_double)]
    lib.mpg_host_csr_free.argtypes = [C.POINTER(HostCsr)]
    lib.mpg_host_csr_free.restype = None
    lib.mpg_engine_create.argtypes = [C.POINTER(SolveArgs), C.POINTER(C.c_void_p), C.c_char_p, C.c_int]
    lib.mpg_cycle_program_counts.argtypes = [C.POINTER(_I64)] * 3
    lib.mpg_surface_ride_counts.argtypes = [C.POINTER(_I64)] * 3
    lib.mpg_surface_spmv_counts.argtypes = [C.POINTER(_I64)] * 3
    lib.mpg_surface_host_norm_hits.argtypes = [C.POINTER(_I64)]
    lib.mpg_surface_host_norm_pairs.argtypes = [C.POINTER(_I64)]
    lib.mpg_engine_report.argtypes = [C.c_void_p, C.POINTER(SolveResult)]
    lib.mpg_engine_run.argtypes = [C.c_void_p, C.c_int, C.POINTER(C.c_int)]
    lib.mpg_engine_sync.argtypes = [C.c_void_p]
    lib.mpg_engine_total_iters.argtypes = [C.c_void_p]
    lib.mpg_engine_total_iters.restype = C.c_int64
    lib.mpg_engine_time_phase.argtypes = [C.c_void_p, C.c_int, C.c_int, C.POINTER(C.c_double)]
    lib.mpg_engine_time_spmv_incycle.argtypes = [C.c_void_p, C.c_int, C.POINTER(C.c_double),
                                                 C.POINTER(C.c_double), C.c_int]
    lib.mpg_engine_time_phase_graph.argtypes = [C.c_void_p, C.c_int, C.c_int, C.POINTER(C.c_double),
                                                C.POINTER(C.c_double), C.c_int]
    lib.mpg_engine_time_phase_dup.argtypes = [C.c_void_p, C.c_int, C.c_int, C.POINTER(C.c_double),
                                              C.POINTER(C.c_int64)]
    lib.mpg_engine_time_phase_stamps.argtypes = [C.c_void_p, C.c_int, C.c_int, C.POINTER(C.c_double),
                                                 C.POINTER(C.c_double), C.c_int]
    lib.mpg_engine_last_error.argtypes = [C.c_void_p]
    lib.mpg_engine_last_error.restype = C.c_char_p
    lib.mpg_engine_phase_bytes.argtypes = [C.c_void_p, C.c_int]
    lib.mpg_engine_phase_bytes.restype = C.c_double
    lib.mpg_engine_destroy.argtypes = [C.c_void_p]
    lib.mpg_engine_spmv_layout.argtypes = [C.c_void_p, C.POINTER(C.c_int32), C.POINTER(C.c_int32),
                                           C.POINTER(C.c_int32), C.POINTER(C.c_int64), C.POINTER(C.c_int32)]
    P64 = C.POINTER(C.c_int64)
    P32 = C.POINTER(C.c_int32)
    lib.mpg_halo_analyze.argtypes = [_I32, _I32, P64, _I32, P32, P32, C.POINTER(C.c_void_p)]
    lib.mpg_csr_node_dof.argtypes = [_I32, P32, P32]
    lib.mpg_csr_node_dof.restype = _I32
    lib.mpg_halo_n_ext.argtypes = [C.c_void_p]
    lib.mpg_halo_n_ext.restype = _I32
    lib.mpg_halo_n_front.argtypes = [C.c_void_p]
    lib.mpg_halo_n_front.restype = _I32
    lib.mpg_halo_recv_pos.argtypes = [C.c_void_p, _I32]
    lib.mpg_halo_recv_pos.restype = _I32
    lib.mpg_halo_recv_count.argtypes = [C.c_void_p, _I32]
    lib.mpg_halo_recv_count.restype = _I32
    lib.mpg_halo_recv_rows.argtypes = [C.c_void_p, _I32, P64]
    lib.mpg_halo_set_send.argtypes = [C.c_void_p, _I32, _I32, P64]
    lib.mpg_halo_local_cols.argtypes = [C.c_void_p, P32]
    lib.mpg_halo_free.argtypes = [C.c_void_p]
    lib.mpg_halo_free.restype = None
    lib.mpg_rccl_unique_id.argtypes = [C.c_char_p, C.c_int]
    lib.mpg_engine_create_dist.argtypes = [C.POINTER(SolveArgs), C.c_void_p, C.c_char_p, _I32, _I32,
                                           C.POINTER(C.c_void_p), C.c_char_p, C.c_int]
    lib.mpg_solve_loopback.argtypes = [C.POINTER(SolveArgs), _I32, C.POINTER(SolveResult)]
    lib.mpg_solve_loopback_ex.argtypes = [C.POINTER(SolveArgs), _I32, C.POINTER(SolveResult), C.c_void_p]
    lib.mpg_solve_multi_gpu.argtypes = [C.POINTER(SolveArgs), _I32, C.c_void_p, C.POINTER(SolveResult), C.c_void_p]
    lib.mpg_engine_comm_ranks.argtypes = [C.c_void_p]
    lib.mpg_engine_sell_columns.argtypes = [C.c_void_p, C.POINTER(C.c_int32), C.POINTER(C.c_int64),
                                            C.POINTER(C.c_int64)]
    lib.mpg_engine_half_stats.argtypes = [C.c_void_p, C.POINTER(C.c_int64)]
    lib.mpg_engine_slices_per_wave.argtypes = [C.c_void_p]
    lib.mpg_engine_givens_folded.argtypes = [C.c_void_p]
    lib.mpg_engine_accum.argtypes = [C.c_void_p]
    lib.mpg_engine_prologue_format.argtypes = [C.c_void_p]
    lib.mpg_engine_sell_shared_slices.argtypes = [C.c_void_p]
    lib.mpg_engine_sell_shared_slices.restype = C.c_int64
    lib.mpg_engine_sell_sigma.argtypes = [C.c_void_p]


# (name, argtypes) for the kernel-level C-ABI, used by the per-kernel tests
_HIP_DECLS = {
    "mpg_error_string": ([C.c_int], C.c_char_p),
    "mpg_ctx_last_error": ([_P], C.c_char_p),
    "mpg_ctx_create": ([C.c_int, C.POINTER(_P)], C.c_int),
    "mpg_ctx_destroy": ([_P], C.c_int),
    "mpg_ctx_sync": ([_P], C.c_int),
    "mpg_ctx_stream": ([_P], _P),
    "mpg_malloc": ([_P, C.c_size_t, C.POINTER(_P)], C.c_int),
    "mpg_free": ([_P, _P], C.c_int),
    "mpg_memcpy_h2d": ([_P, _P, _P, C.c_size_t], C.c_int),
    "mpg_memcpy_d2h": ([_P, _P, _P, C.c_size_t], C.c_int),
    "mpg_csr_create": ([_P, _I32, _I32, _I64, _P, _P, _P, C.POINTER(_P)], C.c_int),
    "mpg_csr_transpose": ([_P, _I32, _I32, _I64, _P, _P, _P, _P, _P], C.c_int),
    "mpg_gather_b32": ([_P, _I64, _P, _P, _P], C.c_int),
    "mpg_gather_b64": ([_P, _I64, _P, _P, _P], C.c_int),
    "mpg_csr_destroy": ([_P], C.c_int),
    "mpg_csr_num_blocks": ([_P], C.c_int),
}
for _t, _ct in (("f64", C.c_double), ("f32", C.c_float)):
    _HIP_DECLS.update({
        f"mpg_dot_{_t}": ([_P, _I64, _P, _P, _P], C.c_int),
        f"mpg_nrm2_{_t}": ([_P, _I64, _P, _P], C.c_int),
        f"mpg_dot_{_t}_host": ([_P, _I64, _P, _P, _P], C.c_int),
        f"mpg_nrm2_{_t}_host": ([_P, _I64, _P, _P], C.c_int),
        f"mpg_axpy_{_t}": ([_P, _I64, _ct, _P, _P], C.c_int),
        f"mpg_axpy_dev_{_t}": ([_P, _I64, _P, _P, _P], C.c_int),
        f"mpg_naxpy_dev_{_t}": ([_P, _I64, _P, _P, _P], C.c_int),
        f"mpg_scal_{_t}": ([_P, _I64, _ct, _P], C.c_int),
        f"mpg_scal_copy_{_t}": ([_P, _I64, _ct, _P, _P], C.c_int),
        f"mpg_scal_copy_dev_{_t}": ([_P, _I64, _P, _P, _P], C.c_int),
        f"mpg_scal_recip_copy_dev_{_t}": ([_P, _I64, _P, _P, _P], C.c_int),
        f"mpg_fill_{_t}": ([_P, _P, _I64, _I64, _I64, _ct], C.c_int),
        f"mpg_gdmv_{_t}": ([_P, _I64, _ct, _P, _P, _ct, _P], C.c_int),
        f"mpg_rotg_{_t}": ([_P, _P, _P, _P, _P], C.c_int),
        f"mpg_rot_{_t}": ([_P, _P, _P, _P, _P], C.c_int),
        f"mpg_rot_vec_{_t}": ([_P, C.c_int, _P, _P, _P], C.c_int),
        f"mpg_scal_scalar_{_t}": ([_P, _ct, _P, _P], C.c_int),
        f"mpg_scal_scalar_dev_{_t}": ([_P, _P, _P, _P], C.c_int),
        f"mpg_gemv_{_t}": ([_P, C.c_int, _I64, _I64, _ct, _P, _I64, _P, _ct, _P], C.c_int),
        f"mpg_trsv_{_t}": ([_P, C.c_int, C.c_int, _I64, _P, _I64, _P], C.c_int),
        f"mpg_csr_spmv_{_t}": ([_P, _P, _ct, _P, _P, _ct, _P], C.c_int),
        f"mpg_jacobi_setup_{_t}": ([_P, _P, _P, _P], C.c_int),
    })
_HIP_DECLS.update({
    "mpg_csr_spmv_f16f32": ([_P, _P, C.c_float, _P, _P, C.c_float, _P], C.c_int),
    "mpg_csr_spmv_f16f32_scaled": ([_P, _P, C.c_float, _P, _P, _P, C.c_float, _P], C.c_int),
    "mpg_csr_half_values": ([_P, _P, _P, _I32, _P, _P, C.POINTER(_I64)], C.c_int),
    "mpg_sell_create": ([_P, _P, _I32, _P, _I32, C.POINTER(_P)], C.c_int),
    "mpg_sell_shared_slices": ([_P], C.c_int64),
    "mpg_sell_destroy": ([_P], C.c_int),
    "mpg_sell_layout": ([_P, C.POINTER(_I32), C.POINTER(_I32), C.POINTER(_I64), C.POINTER(_I32)], C.c_int),
    "mpg_sell_spmv_f64": ([_P, _P, C.c_double, _P, C.c_double, _P], C.c_int),
    "mpg_sell_spmv_f32": ([_P, _P, C.c_float, _P, C.c_float, _P], C.c_int),
    "mpg_sell_spmv_f16f32": ([_P, _P, C.c_float, _P, C.c_float, _P], C.c_int),
    "mpg_sell_spmv_prog_f64": ([_P, _P, C.c_double, _P, C.c_double, _P, _P, C.c_int32], C.c_int),
    "mpg_sell_spmv_prog_f32": ([_P, _P, C.c_float, _P, C.c_float, _P, _P, C.c_int32], C.c_int),
    "mpg_node_spmv_prog_f64": ([_P, _P, C.c_double, _P, C.c_double, _P, _P, C.c_int32], C.c_int),
    "mpg_node_spmv_prog_f32": ([_P, _P, C.c_float, _P, C.c_float, _P, _P, C.c_int32], C.c_int),
    "mpg_node_spmv_norm_f64": ([_P, _P, C.c_int32, _P, _P, _P, C.c_double, _P, _P, C.c_int32], C.c_int),
    "mpg_node_spmv_norm_f32": ([_P, _P, C.c_int32, _P, _P, _P, C.c_float, _P, _P, C.c_int32], C.c_int),
    "mpg_copy_f64f64": ([_P, _I64, _P, _P], C.c_int),
    "mpg_copy_f32f32": ([_P, _I64, _P, _P], C.c_int),
    "mpg_copy_f64f32": ([_P, _I64, _P, _P], C.c_int),
    "mpg_copy_f32f64": ([_P, _I64, _P, _P], C.c_int),
    "mpg_copy_f64f16": ([_P, _I64, _P, _P], C.c_int),
    "mpg_copy_f32f16": ([_P, _I64, _P, _P], C.c_int),
    "mpg_nrm2_pair_host": ([_P, _I64, C.c_int, _P, C.c_int, _P, C.POINTER(C.c_double), C.POINTER(C.c_double)],
                           C.c_int),
})


def _declare_hip(lib: C.CDLL) -> None:
    for name, (args, res) in _HIP_DECLS.items():
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = res


def exported_capi_symbols() -> list:
    """Every function the C-ABI headers declare (parsed from include/mpgmres/*.h)."""
    import re

    names = []
    for h in sorted((REPO_DIR / "include" / "mpgmres").glob("*.h")):
        txt = h.read_text()
        txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
        for m in re.finditer(r"^\s*(?:const\s+)?[A-Za-z_][\w\s\*]*?\b(mpg_\w+)\s*\(", txt, flags=re.M):
            names.append((h.name, m.group(1)))
    return names


# ---------------------------------------------------------------- problems
@dataclass
class Csr:
    """Host CSR (0-based int32 structure, fp64 values)."""
    nrows: int
    ncols: int
    rowptr: np.ndarray
    col: np.ndarray
    val: np.ndarray

    @property
    def nnz(self) -> int:
        return int(self.rowptr[-1])

    @property
    def n(self) -> int:
        return self.nrows

    def _c(self) -> HostCsr:
        h = HostCsr()
        h.nrows, h.ncols, h.nnz = self.nrows, self.ncols, self.nnz
        h.rowptr = self.rowptr.ctypes.data_as(C.POINTER(C.c_int32))
        h.col = self.col.ctypes.data_as(C.POINTER(C.c_int32))
        h.val = self.val.ctypes.data_as(C.POINTER(C.c_double))
        return h

    def to_scipy(self):
        import scipy.sparse as sp

        return sp.csr_matrix((self.val, self.col, self.rowptr), shape=(self.nrows, self.ncols))


def _take_csr(h: HostCsr) -> Csr:
    lib = host_lib()
    n, nnz = h.nrows, h.nnz
    rp = np.ctypeslib.as_array(h.rowptr, shape=(n + 1,)).copy()
    ci = np.ctypeslib.as_array(h.col, shape=(max(nnz, 1),))[:nnz].copy()
    va = np.ctypeslib.as_array(h.val, shape=(max(nnz, 1),))[:nnz].copy()
    out = Csr(n, h.ncols, rp, ci, va)
    lib.mpg_host_csr_free(C.byref(h))
    return out


def gen_band(n: int, lo: int = 5, hi: int = 4, seed: int = 7, row_begin: int = 0,
             row_end: Optional[int] = None) -> Csr:
    """Banded test matrix (BAND-10M at n=1e6); any row slice matches the whole."""
    h = HostCsr()
    st = host_lib().mpg_gen_band(n, lo, hi, seed, row_begin, n if row_end is None else row_end, C.byref(h))
    if st:
        raise ValueError(f"mpg_gen_band failed ({st})")
    return _take_csr(h)


def gen_laplace3d(nx: int, ny: Optional[int] = None, nz: Optional[int] = None) -> Csr:
    h = HostCsr()
    st = host_lib().mpg_gen_laplace3d(nx, ny or nx, nz or nx, C.byref(h))
    if st:
        raise ValueError(f"mpg_gen_laplace3d failed ({st})")
    return _take_csr(h)


def gen_stencil27(nx: int, dof: int = 3, seed: int = 11, ny: Optional[int] = None, nz: Optional[int] = None) -> Csr:
    """27-point 3-D stencil on nx x ny x nz nodes (cubic by default), `dof`
    unknowns per node (the Queen_4147 stand-in at nx = 111, dof = 3)."""
    h = HostCsr()
    st = host_lib().mpg_gen_stencil27(nx, ny or nx, nz or nx, dof, seed, C.byref(h))
    if st:
        raise ValueError(f"mpg_gen_stencil27 failed ({st})")
    return _take_csr(h)


def load_mtx_vector(path: str, n: int, col: int = 0) -> np.ndarray:
    """Column `col` of a Matrix Market array or coordinate file as a length-n
    vector (mpg_load_mtx_vector; the reference's LoadVector,
    LoadMatrix.hpp:156-233, behind --bpath)."""
    out = np.zeros(n, dtype=np.float64)
    err = C.create_string_buffer(256)
    if host_lib().mpg_load_mtx_vector(path.encode(), col, out.ctypes.data_as(C.POINTER(C.c_double)), n, err, 256):
        raise ValueError(err.value.decode())
    return out


def gen_fem27(nx: int, dof: int = 3, keep_pct: int = 70, seed: int = 13, ny: Optional[int] = None,
              nz: Optional[int] = None) -> Csr:
    """FEM-like irregular matrix: the 27-point node coupling with each node
    pair kept with probability keep_pct % (symmetric; rows of variable length)."""
    h = HostCsr()
    st = host_lib().mpg_gen_fem27(nx, ny or nx, nz or nx, dof, keep_pct, seed, C.byref(h))
    if st:
        raise ValueError(f"mpg_gen_fem27 failed ({st})")
    return _take_csr(h)


def perm_node_blocks(nodes: int, dof: int = 3, block: int = 64, seed: int = 5) -> np.ndarray:
    """perm[old] = new: node blocks in a seeded random order, nodes shuffled
    inside each block, dof kept together (mpg_perm_node_blocks)."""
    perm = np.zeros(nodes * dof, dtype=np.int32)
    if host_lib().mpg_perm_node_blocks(nodes, dof, block, seed, perm.ctypes.data_as(C.POINTER(C.c_int32))):
        raise ValueError("mpg_perm_node_blocks failed")
    return perm


def permute_sym(A: Csr, perm: np.ndarray) -> Csr:
    """P A P^T with row perm[i] = row i of A (mpg_csr_permute_sym)."""
    perm = np.ascontiguousarray(perm, dtype=np.int32)
    a, h = A._c(), HostCsr()
    if host_lib().mpg_csr_permute_sym(C.byref(a), perm.ctypes.data_as(C.POINTER(C.c_int32)), C.byref(h)):
        raise ValueError("mpg_csr_permute_sym failed (not a permutation?)")
    return _take_csr(h)


def gen_stencil27p(nx: int, dof: int = 3, seed: int = 11, block: int = 64, perm_seed: int = 5,
                   ny: Optional[int] = None, nz: Optional[int] = None) -> Csr:
    """The Queen_4147-like irregular stand-in: gen_stencil27 under a symmetric
    node-block permutation (same spectrum, scattered neighbours)."""
    A = gen_stencil27(nx, dof, seed, ny=ny, nz=nz)
    return permute_sym(A, perm_node_blocks(A.nrows // dof, dof, block, perm_seed))


def gen_spec(spec: str) -> Csr:
    """A generator by its CLI spec (mpg_gen_spec: band:..., laplace:..., stencil27:...)."""
    h = HostCsr()
    err = C.create_string_buffer(256)
    if host_lib().mpg_gen_spec(spec.encode(), C.byref(h), err, 256):
        raise ValueError(err.value.decode())
    return _take_csr(h)


def condest(A: Csr, rand_seed: int = 42, max_iters: int = 100000, verbose: bool = False, device: int = 0) -> dict:
    """Condition-number estimate of square A on the GPU (include/mpgmres/condest.h;
    the reference's condest.cpp:34-150): sigma_max, sigma_min, cond, iters, ..."""
    a = condest_args(A, rand_seed, max_iters, verbose, device)
    r = CondestResult()
    if host_lib().mpg_condest(C.byref(a), C.byref(r)):
        raise RuntimeError(f"mpg_condest failed: {r.message.decode()}")
    return condest_dict(r)


def load_mtx(path: str) -> Csr:
    h = HostCsr()
    err = C.create_string_buffer(256)
    if host_lib().mpg_load_mtx(str(path).encode(), C.byref(h), err, 256):
        raise ValueError(err.value.decode())
    return _take_csr(h)


def rand_vect(n: int, seed: int = 42) -> np.ndarray:
    """x_true of gmres_perf_test.cpp:39-51 (mt19937 + uniform_real_distribution<float>)."""
    out = np.empty(n, dtype=np.float64)
    host_lib().mpg_rand_vect(n, seed, out.ctypes.data_as(C.POINTER(C.c_double)))
    return out


def host_spmv(A: Csr, x: np.ndarray) -> np.ndarray:
    x = np.ascontiguousarray(x, dtype=np.float64)
    y = np.empty(A.nrows, dtype=np.float64)
    h = A._c()
    host_lib().mpg_host_spmv(C.byref(h), x.ctypes.data_as(C.POINTER(C.c_double)),
                             y.ctypes.data_as(C.POINTER(C.c_double)))
    return y


# ---------------------------------------------------------------- solve
@dataclass
class Result:
    status: str
    restarts: int
    inner_k: int
    total_iters: int
    res_norm: float
    err_norm: float
    gmres_seconds: float
    setup_seconds: float
    minvb_norm: float
    x: np.ndarray
    cyc_r_norm: np.ndarray
    cyc_normalization: np.ndarray
    cyc_beta: np.ndarray
    step_res: np.ndarray
    step_cycle: np.ndarray
    message: str = ""
    extra: dict = field(default_factory=dict)
    nonfinite_steps: int = 0       # Arnoldi steps with a NaN/Inf |s(k+1)| (breakdown report)
    nonfinite_cycles: int = 0      # restarts with a NaN/Inf true residual or beta
    first_nonfinite_step: int = -1

    @property
    def backward_error(self) -> np.ndarray:
        return self.cyc_r_norm / self.cyc_normalization


def make_args(A: Csr, b: np.ndarray, x_true: Optional[np.ndarray] = None, *, mode="mixed", orth="mgs",
              prec="identity", rlen=30, tol=1e-6, max_restarts=1_000_000, rtol=0.0, repeat_iter=False,
              orthloss=False, jacobi_steps=1, engine="fused", verbose=False, device=0, threads=0,
              spmv_format="auto", half_unscaled=False, stop_on_breakdown=False, accum="f64"):
    """Build mpg_solve_args (shared by mpg_solve and the CPU oracle).
    accum: the fp32 Arnoldi's accumulation class, "f64" (fp32 products
    summed in fp64, rounded once) or "f32" (every partial sum in fp32: the
    reference's cblas_s* / mkl_sparse_s_mv class; fused engine only)."""
    b = np.ascontiguousarray(b, dtype=np.float64)
    keep = [A.rowptr, A.col, A.val, b]
    a = SolveArgs()
    a.n, a.nnz = A.nrows, A.nnz
    a.rowptr = A.rowptr.ctypes.data_as(C.POINTER(C.c_int32))
    a.col = A.col.ctypes.data_as(C.POINTER(C.c_int32))
    a.val = A.val.ctypes.data_as(C.POINTER(C.c_double))
    a.b = b.ctypes.data_as(C.POINTER(C.c_double))
    if x_true is not None:
        x_true = np.ascontiguousarray(x_true, dtype=np.float64)
        keep.append(x_true)
        a.x_true = x_true.ctypes.data_as(C.POINTER(C.c_double))
    a.mode, a.orth, a.prec, a.engine = MODES[mode], ORTHS[orth], PRECS[prec], ENGINES[engine]
    a.rlen, a.tol, a.max_restarts, a.rtol = rlen, tol, max_restarts, rtol
    a.repeat_iter, a.orthloss, a.jacobi_steps = int(repeat_iter), int(orthloss), jacobi_steps
    a.verbose, a.device, a.threads = int(verbose), device, threads
    a.spmv_format = SPMV_FORMATS[spmv_format]
    a.half_unscaled = int(half_unscaled)
    a.stop_on_breakdown = int(stop_on_breakdown)
    a.accum = ACCUMS[accum]
    return a, keep


def run_solve(fn, args: SolveArgs, n: int, cycle_cap: int = 4096, step_cap: int = 1 << 17) -> Result:
    """Call an mpg_solve-shaped entry point and collect the result + history."""
    r = SolveResult()
    x = np.zeros(n, dtype=np.float64)
    cr, cn, cb = (np.zeros(cycle_cap) for _ in range(3))
    sr = np.zeros(step_cap)
    sc = np.zeros(step_cap, dtype=np.int32)
    dp = lambda a: a.ctypes.data_as(C.POINTER(C.c_double))  # noqa: E731
    r.x_out = dp(x)
    r.cycle_cap, r.cyc_r_norm, r.cyc_normalization, r.cyc_beta = cycle_cap, dp(cr), dp(cn), dp(cb)
    r.step_cap, r.step_res, r.step_cycle = step_cap, dp(sr), sc.ctypes.data_as(C.POINTER(C.c_int32))
    st = fn(C.byref(args), C.byref(r))
    msg = r.message.decode(errors="replace")
    if st != 0:
        raise RuntimeError(f"solve failed ({st}): {msg}")
    nc, ns = min(r.n_cycles, cycle_cap), min(r.n_steps, step_cap)
    return Result(STATUS.get(r.status, str(r.status)), r.restarts, r.inner_k, r.total_iters, r.res_norm,
                  r.err_norm, r.gmres_seconds, r.setup_seconds, r.minvb_norm, x, cr[:nc].copy(), cn[:nc].copy(),
                  cb[:nc].copy(), sr[:ns].copy(), sc[:ns].copy(), msg, nonfinite_steps=r.nonfinite_steps,
                  nonfinite_cycles=r.nonfinite_cycles, first_nonfinite_step=r.first_nonfinite_step)


def solve(A: Csr, b: np.ndarray, x_true: Optional[np.ndarray] = None, **opts) -> Result:
    """Restarted GMRES(m) on the MI355X (mpg_solve). Options as make_args."""
    args, keep = make_args(A, b, x_true, **opts)
    return run_solve(host_lib().mpg_solve, args, A.nrows)


def cycle_program_counts() -> dict:
    """Operator-surface cycle programs so far in this process
    (mpg_cycle_program_counts): recorded, replayed, voided."""
    v = [_I64() for _ in range(3)]
    host_lib().mpg_cycle_program_counts(*[C.byref(x) for x in v])
    return {"recorded": v[0].value, "replayed": v[1].value, "voided": v[2].value}


def surface_ride_counts() -> dict:
    """The calling thread's operator-surface normalisation rides so far
    (mpg_surface_ride_counts): CGS updates that redirected w, normalisations
    that rode the next SpMV, and those issued separately instead."""
    v = [_I64() for _ in range(3)]
    host_lib().mpg_surface_ride_counts(*[C.byref(x) for x in v])
    return {"redirects": v[0].value, "rides": v[1].value, "flushed": v[2].value}


def surface_host_norm_hits() -> int:
    """Host-value nrm2 calls of the operator surface on this thread answered
    from the previous read of the same, unwritten vector
    (mpg_surface_host_norm_hits)."""
    v = _I64()
    host_lib().mpg_surface_host_norm_hits(C.byref(v))
    return v.value


def surface_host_norm_pairs() -> int:
    """Host-value nrm2 calls of the operator surface on this thread that also
    read the residual SpMV's input vector's norm in the same launch
    (mpg_surface_host_norm_pairs)."""
    v = _I64()
    host_lib().mpg_surface_host_norm_pairs(C.byref(v))
    return v.value


def surface_spmv_counts() -> dict:
    """The operator surface's spmv calls on this thread so far by storage
    (mpg_surface_spmv_counts): node blocks, SELL-64, CSR."""
    v = [_I64() for _ in range(3)]
    host_lib().mpg_surface_spmv_counts(*[C.byref(x) for x in v])
    return {"node": v[0].value, "sell": v[1].value, "csr": v[2].value}


def row_slice(A: Csr, r0: int, r1: int) -> Csr:
    """Rows [r0, r1) of A with global column ids (one rank's share)."""
    base = int(A.rowptr[r0])
    rp = (A.rowptr[r0:r1 + 1] - base).astype(np.int32)
    end = int(A.rowptr[r1])
    return Csr(r1 - r0, A.ncols, rp, A.col[base:end].copy(), A.val[base:end].copy())


def node_dof(A: Csr) -> int:
    """3 when A is made of whole 3 x 3 node blocks (mpg_csr_node_dof), else 1."""
    rp = np.ascontiguousarray(A.rowptr, dtype=np.int32)
    col = np.ascontiguousarray(A.col, dtype=np.int32)
    return int(host_lib().mpg_csr_node_dof(A.nrows, rp.ctypes.data_as(C.POINTER(C.c_int32)),
                                           col.ctypes.data_as(C.POINTER(C.c_int32))))


def nnz_balanced_starts(A: Csr, nranks: int) -> np.ndarray:
    """Row offsets splitting A into nranks blocks of about equal nnz, rounded
    down to node boundaries when A has 3-dof node blocks (node_dof; as
    mpg_solve_loopback / mpg_solve_multi_gpu split)."""
    nnz = A.nnz
    al = node_dof(A)
    starts = [0]
    for q in range(1, nranks):
        r = int(np.searchsorted(A.rowptr, nnz * q // nranks, side="left"))
        starts.append(max(r // al * al, starts[-1]))
    starts.append(A.nrows)
    return np.array(starts, dtype=np.int64)


class HaloPlan:
    """Halo exchange plan of one rank (include/mpgmres/dist.h). Build with
    the rank's rows (global columns), exchange recv_rows() with the peers by
    any transport, then set_send() what each peer needs from this rank."""

    def __init__(self, rank: int, nranks: int, row_starts: np.ndarray, A_local: Csr):
        self._lib = host_lib()
        self.rank, self.nranks = rank, nranks
        self.row_starts = np.ascontiguousarray(row_starts, dtype=np.int64)
        self.A = A_local
        self._h = C.c_void_p()
        st = self._lib.mpg_halo_analyze(rank, nranks, self.row_starts.ctypes.data_as(C.POINTER(C.c_int64)),
                                        A_local.nrows, A_local.rowptr.ctypes.data_as(C.POINTER(C.c_int32)),
                                        A_local.col.ctypes.data_as(C.POINTER(C.c_int32)), C.byref(self._h))
        if st:
            raise ValueError(f"mpg_halo_analyze failed ({st})")

    @property
    def n_ext(self) -> int:
        """end of the local numbering: own rows [0, n), higher ranks' halo [n, n_ext)"""
        return int(self._lib.mpg_halo_n_ext(self._h))

    @property
    def n_front(self) -> int:
        """lower ranks' halo rows, local ids [-n_front, 0)"""
        return int(self._lib.mpg_halo_n_front(self._h))

    def recv_pos(self, peer: int) -> int:
        """local id of the first row received from `peer`"""
        return int(self._lib.mpg_halo_recv_pos(self._h, peer))

    def recv_rows(self, peer: int) -> np.ndarray:
        cnt = self._lib.mpg_halo_recv_count(self._h, peer)
        out = np.zeros(max(cnt, 1), dtype=np.int64)
        self._lib.mpg_halo_recv_rows(self._h, peer, out.ctypes.data_as(C.POINTER(C.c_int64)))
        return out[:cnt]

    def set_send(self, peer: int, rows) -> None:
        rows = np.ascontiguousarray(rows, dtype=np.int64)
        if self._lib.mpg_halo_set_send(self._h, peer, len(rows), rows.ctypes.data_as(C.POINTER(C.c_int64))):
            raise ValueError("mpg_halo_set_send: rows outside this rank's block")

    def local_cols(self) -> np.ndarray:
        out = np.zeros(max(self.A.nnz, 1), dtype=np.int32)
        self._lib.mpg_halo_local_cols(self._h, out.ctypes.data_as(C.POINTER(C.c_int32)))
        return out[:self.A.nnz]

    def close(self):
        if self._h:
            self._lib.mpg_halo_free(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def bw_probe(kind: str = "read", nbytes: int = 2 << 30, reps: int = 3, device: int = 0) -> float:
    """Measured HBM streaming rate in GB/s (mpg_bw_probe): "read" counts the
    bytes read by a float4 stream, "copy" read + written bytes."""
    lib = hip_lib()
    lib.mpg_bw_probe.argtypes = [C.c_void_p, C.c_int, C.c_size_t, C.c_int, C.POINTER(C.c_double)]
    ctx = C.c_void_p()
    if lib.mpg_ctx_create(device, C.byref(ctx)):
        raise RuntimeError("mpg_ctx_create failed")
    try:
        gbs = C.c_double()
        st = lib.mpg_bw_probe(ctx, {"read": 0, "copy": 1}[kind], nbytes, reps, C.byref(gbs))
        if st:
            raise RuntimeError(f"mpg_bw_probe failed ({st})")
        return gbs.value
    finally:
        lib.mpg_ctx_destroy(ctx)


def device_count() -> int:
    """HIP devices visible to this process (mpg_device_count), through the
    package's own HIP runtime (importing torch after the package would load
    a second one)."""
    lib = hip_lib()
    lib.mpg_device_count.argtypes = []
    return int(lib.mpg_device_count())


def rccl_unique_id() -> bytes:
    buf = C.create_string_buffer(128)
    if host_lib().mpg_rccl_unique_id(buf, 128):
        raise RuntimeError("ncclGetUniqueId failed")
    return buf.raw


def solve_loopback(A: Csr, b: np.ndarray, x_true: Optional[np.ndarray] = None, nranks: int = 2,
                   layouts: Optional[list] = None, **opts) -> Result:
    """The row-partitioned engine with `nranks` ranks as threads on one GPU.
    `layouts`: a list that receives one dict per rank (mpg_rank_layout)."""
    opts.pop("engine", None)
    args, keep = make_args(A, b, x_true, engine="fused", **opts)
    lib = host_lib()
    lay = (RankLayout * nranks)()
    res = run_solve(lambda a, r: lib.mpg_solve_loopback_ex(a, nranks, r, C.cast(lay, C.c_void_p)), args, A.nrows)
    _layout_dicts(lay, layouts)
    return res


def _layout_dicts(lay, layouts: Optional[list]):
    if layouts is None:
        return
    forms = {-1: "none", 0: "int32", 1: "int16", 2: "stepped"}
    for L in lay:
        d = {f: getattr(L, f) for f, _ in RankLayout._fields_}
        d["format"] = {1: "csr", 2: "sell", 3: "node"}.get(d["format"], d["format"])
        d["col_form"] = forms[d["col_form"]]
        layouts.append(d)


def solve_multi_gpu(A: Csr, b: np.ndarray, x_true: Optional[np.ndarray] = None, ngpus: int = 1,
                    devices: Optional[list] = None, layouts: Optional[list] = None, **opts) -> Result:
    """The row-partitioned engine in this process with `ngpus` ranks, rank q
    a host thread on devices[q] (default 0..ngpus-1), collectives over one
    RCCL clique (ncclCommInitAll; mpg_solve_multi_gpu, dist.h). Raises when
    fewer GPUs are visible than requested or a device is named twice."""
    opts.pop("engine", None)
    opts.pop("device", None)
    args, keep = make_args(A, b, x_true, engine="fused", **opts)
    lib = host_lib()
    lay = (RankLayout * ngpus)()
    devs = None
    if devices is not None:
        if len(devices) != ngpus:
            raise ValueError(f"{len(devices)} devices for {ngpus} ranks")
        devs = (C.c_int32 * ngpus)(*devices)
    res = run_solve(lambda a, r: lib.mpg_solve_multi_gpu(a, ngpus, C.cast(devs, C.c_void_p) if devs else None, r,
                                                         C.cast(lay, C.c_void_p)), args, A.nrows)
    _layout_dicts(lay, layouts)
    return res


class Engine:
    """Stepped fused engine (mpg_engine_*): set up once, then advance the
    restarted solve cycle by cycle — what bench.py times. Engine.distributed
    builds one rank of a row-partitioned solve over RCCL."""

    PHASES = {"spmv": 0, "prologue": 1, "cgs_update": 2, "dots": 3, "spmv_storage": 4}

    def __init__(self, A: Csr, b: np.ndarray, x_true: Optional[np.ndarray] = None, *, _dist=None, **opts):
        opts.pop("engine", None)
        self._args, self._keep = make_args(A, b, x_true, engine="fused", **opts)
        self._lib = host_lib()
        self._h = C.c_void_p()
        err = C.create_string_buffer(512)
        if _dist is None:
            st = self._lib.mpg_engine_create(C.byref(self._args), C.byref(self._h), err, 512)
        else:
            plan, link, nranks, rank = _dist
            self._plan = plan
            if isinstance(link, (bytes, bytearray)):
                st = self._lib.mpg_engine_create_dist(C.byref(self._args), plan._h, link, nranks, rank,
                                                      C.byref(self._h), err, 512)
            else:
                self._transport = link  # keeps the callbacks alive
                st = self._lib.mpg_engine_create_dist_host(C.byref(self._args), plan._h, C.byref(link.c), nranks,
                                                           rank, C.byref(self._h), err, 512)
        if st:
            raise RuntimeError(f"mpg_engine_create: {err.value.decode()}")

    @classmethod
    def distributed(cls, A_local: Csr, b_local, x_true_local, plan: HaloPlan, uid: bytes, nranks: int, rank: int,
                    **opts):
        return cls(A_local, b_local, x_true_local, _dist=(plan, uid, nranks, rank), **opts)

    @classmethod
    def distributed_host(cls, A_local: Csr, b_local, x_true_local, plan: HaloPlan, transport, nranks: int,
                         rank: int, **opts):
        """One rank of a row-partitioned solve whose collectives go through
        a host transport (transport.HostTransport over torch.distributed)
        instead of RCCL: ranks may share a GPU (mpg_engine_create_dist_host)."""
        return cls(A_local, b_local, x_true_local, _dist=(plan, transport, nranks, rank), **opts)

    def report(self, cycle_cap: int = 4096, step_cap: int = 1 << 17) -> Result:
        """The solve so far as mpg_solve reports it (mpg_engine_report): this
        rank's rows of x; collective on a row-partitioned engine."""
        n = self._args.n
        lib = self._lib
        return run_solve(lambda a, r: lib.mpg_engine_report(self._h, r), self._args, n, cycle_cap, step_cap)

    def run(self, cycles: int) -> tuple:
        done = C.c_int(0)
        ran = self._lib.mpg_engine_run(self._h, cycles, C.byref(done))
        if ran < 0:
            msg = self._lib.mpg_engine_last_error(self._h).decode(errors="replace")
            raise RuntimeError(f"mpg_engine_run failed ({ran}): {msg}")
        return ran, bool(done.value)

    def sync(self) -> None:
        if self._lib.mpg_engine_sync(self._h):
            raise RuntimeError("mpg_engine_sync failed")

    @property
    def total_iters(self) -> int:
        return int(self._lib.mpg_engine_total_iters(self._h))

    def time_phase(self, phase: str, reps: int = 20) -> float:
        ms = C.c_double()
        if self._lib.mpg_engine_time_phase(self._h, self.PHASES[phase], reps, C.byref(ms)):
            raise RuntimeError("mpg_engine_time_phase failed")
        return ms.value

    def time_spmv_incycle(self, cycles: int = 3) -> tuple:
        """(mean ms, per-launch ms in cycle order) of the Arnoldi SpMV as the
        cycle runs it (Givens folded for k >= 1), each launch timed by its own
        kernel events; measurement only (the cycles skip the restart checks)."""
        ms = C.c_double()
        cap = 4096
        per = (C.c_double * cap)()
        cnt = self._lib.mpg_engine_time_spmv_incycle(self._h, cycles, C.byref(ms), per, cap)
        if cnt < 0:
            raise RuntimeError(f"mpg_engine_time_spmv_incycle failed ({cnt})")
        return ms.value, [per[i] for i in range(min(cnt, cap))]

    def time_phase_graph(self, phase: str = "spmv", reps: int = 3) -> tuple:
        """(mean ms, per-launch ms in cycle order) of a phase kernel ("spmv",
        "cgs_update", "dots") inside graph replays of the cycle: external
        event nodes on each side of every launch of that phase
        (mpg_engine_time_phase_graph); measurement only."""
        ms = C.c_double()
        cap = 16384
        per = (C.c_double * cap)()
        which = {"spmv": 0, "cgs_update": 2, "dots": 3}[phase]
        cnt = self._lib.mpg_engine_time_phase_graph(self._h, which, reps, C.byref(ms), per, cap)
        if cnt < 0:
            msg = self._lib.mpg_engine_last_error(self._h).decode(errors="replace")
            raise RuntimeError(f"mpg_engine_time_phase_graph failed ({cnt}): {msg}")
        return ms.value, [per[i] for i in range(min(cnt, cap))]

    def time_phase_dup(self, phase: str = "spmv", reps: int = 5) -> tuple:
        """(ms, added launches): what one launch of a phase kernel ("spmv",
        "cgs_update", "dots") adds to a graph replay of the cycle -- the cycle
        captured as run and with that phase's launches doubled, replayed
        alternately between HIP events (mpg_engine_time_phase_dup); the
        stream-share figure rocprofv3 reports. Measurement only."""
        ms = C.c_double()
        n = C.c_int64()
        which = {"spmv": 0, "cgs_update": 2, "dots": 3}[phase]
        st = self._lib.mpg_engine_time_phase_dup(self._h, which, reps, C.byref(ms), C.byref(n))
        if st != 0:
            msg = self._lib.mpg_engine_last_error(self._h).decode(errors="replace")
            raise RuntimeError(f"mpg_engine_time_phase_dup failed ({st}): {msg}")
        return ms.value, int(n.value)

    def time_phase_stamps(self, phase: str = "spmv", reps: int = 3) -> tuple:
        """(mean ms, per-launch ms in cycle order) of a phase kernel ("spmv",
        "cgs_update", "dots") inside graph replays of the cycle, from its
        waves' wall-clock stamps (first wave start to last wave end;
        mpg_engine_time_phase_stamps); measurement only."""
        ms = C.c_double()
        cap = 16384
        per = (C.c_double * cap)()
        which = {"spmv": 0, "cgs_update": 2, "dots": 3}[phase]
        cnt = self._lib.mpg_engine_time_phase_stamps(self._h, which, reps, C.byref(ms), per, cap)
        if cnt < 0:
            msg = self._lib.mpg_engine_last_error(self._h).decode(errors="replace")
            raise RuntimeError(f"mpg_engine_time_phase_stamps failed ({cnt}): {msg}")
        return ms.value, [per[i] for i in range(min(cnt, cap))]

    def phase_bytes(self, phase: str) -> float:
        return float(self._lib.mpg_engine_phase_bytes(self._h, self.PHASES[phase]))

    def spmv_layout(self) -> dict:
        """Storage of the Arnoldi SpMV: {"format": "csr"|"sell", "vec_width",
        "col_bytes", "stored"} (mpg_engine_spmv_layout)."""
        f, w, cb, st, win = C.c_int32(), C.c_int32(), C.c_int32(), C.c_int64(), C.c_int32()
        if self._lib.mpg_engine_spmv_layout(self._h, C.byref(f), C.byref(w), C.byref(cb), C.byref(st), C.byref(win)):
            raise RuntimeError("mpg_engine_spmv_layout failed")
        return {"format": {1: "csr", 2: "sell", 3: "node"}[f.value], "vec_width": w.value, "col_bytes": cb.value,
                "stored": st.value, "window": bool(win.value),
                "slices_per_wave": int(self._lib.mpg_engine_slices_per_wave(self._h)),
                "givens_folded": bool(self._lib.mpg_engine_givens_folded(self._h) == 1),
                "accum": {0: "f64", 1: "f32"}[int(self._lib.mpg_engine_accum(self._h))],
                "prologue": {1: "csr", 2: "sell", 3: "node"}[int(self._lib.mpg_engine_prologue_format(self._h))]}

    def sell_columns(self) -> dict:
        """Column form of the Arnoldi SpMV's SELL copy (mpg_engine_sell_columns):
        {"form": "none"|"int32"|"int16"|"stepped", "csr_slices", "implicit_slices"}."""
        f, e, i = C.c_int32(), C.c_int64(), C.c_int64()
        if self._lib.mpg_engine_sell_columns(self._h, C.byref(f), C.byref(e), C.byref(i)):
            raise RuntimeError("mpg_engine_sell_columns failed")
        return {"form": {-1: "none", 0: "int32", 1: "int16", 2: "stepped"}[f.value], "csr_slices": e.value,
                "implicit_slices": i.value,
                "shared_slices": int(self._lib.mpg_engine_sell_shared_slices(self._h)),
                "sigma": int(self._lib.mpg_engine_sell_sigma(self._h))}

    def comm_ranks(self) -> int:
        """Ranks of the engine's communicator as its transport reports them
        (1 on one GPU; RCCL: ncclCommCount; mpg_engine_comm_ranks)."""
        return int(self._lib.mpg_engine_comm_ranks(self._h))

    def half_stats(self) -> dict:
        """mixed-half: what the fp16 cast did (mpg_engine_half_stats)."""
        st = (C.c_int64 * 4)()
        if self._lib.mpg_engine_half_stats(self._h, st):
            raise RuntimeError("mpg_engine_half_stats failed")
        return dict(zip(("rows_scaled", "flushed", "overflowed", "exp_out_of_range"), map(int, st)))

    def close(self) -> None:
        if self._h:
            self._lib.mpg_engine_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
