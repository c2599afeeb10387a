"""The C-ABI libraries load and export every symbol include/mpgmres/*.h
declares (CPU only: nothing here launches a kernel)."""
import ctypes as C

import pytest


def test_every_declared_symbol_is_exported(mpg):
    hip, host = mpg.hip_lib(), mpg.host_lib()
    declared = mpg.exported_capi_symbols()
    assert len(declared) > 60
    missing = []
    for header, name in declared:
        lib = hip if header in ("capi.h", "arnoldi.h", "ilu.h") else host
        try:
            getattr(lib, name)
        except AttributeError:
            missing.append((header, name))
    assert not missing, missing


def test_error_strings_and_arg_checks(mpg):
    hip = mpg.hip_lib()
    assert hip.mpg_error_string(0) == b"ok"
    assert b"argument" in hip.mpg_error_string(-2)
    # null context / out-pointer are rejected without touching a device
    assert hip.mpg_ctx_create(0, None) == -2
    assert hip.mpg_ctx_sync(None) == -2
    assert hip.mpg_dot_f64(None, 10, None, None, None) == -2


def test_solve_rejects_bad_args_without_gpu(mpg):
    import numpy as np

    A = mpg.gen_laplace3d(3)
    b = np.ones(A.nrows)
    with pytest.raises(RuntimeError, match="invalid solve arguments"):
        mpg.solve(A, b, rlen=0)
