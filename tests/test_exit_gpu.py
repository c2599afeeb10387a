"""Process exit. The exit-time "double free or corruption"
(SIGABRT) comes from PyTorch's libraries being loaded into a process whose
HIP runtime has already initialised: the package first, a GPU call, then
`import torch` (tools/exit_probe.py, profiles/r06_exit/). It aborts with
/opt/rocm's runtime bound (two HIP and HSA runtimes: PyTorch's libraries need
their bundled libamdhip64.so / librccl.so by file name, the package's
libraries /opt/rocm's by soname) and with PyTorch's own runtime bound by file
before the package; importing torch before the first GPU call never aborted.
The package loader therefore imports torch first when PyTorch is installed
(`_bind_hip_runtime` in __init__.py, mpg.hip_runtime()); MPG_HIP_RUNTIME=system
binds /opt/rocm's runtime for a process that never imports torch.

The GPU suite imports torch while collecting tests/test_dist_cpu.py, so every
check here runs in a fresh child process. Reference teardown order: the
reference destroys its library singleton in a Kokkos finalize hook
(types_cuda.hpp:26-29); this package holds no device state in static or
thread-local destructors (the surface's lazily created default context is
leaked on purpose, host/kernels_hip.cpp)."""
import os
import subprocess
import sys
from pathlib import Path

import pytest

pytestmark = pytest.mark.gpu

REPO = Path(__file__).resolve().parent.parent
GLIBC = ("double free", "corruption", "free(): invalid", "munmap_chunk", "Aborted")

LOAD = f"""
import sys, importlib.util, tempfile, os
import numpy as np
sys.path.insert(0, {str(REPO)!r})
d = {str(REPO / 'icl-mixed-precision-gmres_amd')!r}
spec = importlib.util.spec_from_file_location('mpgmres_amd', d + '/__init__.py', submodule_search_locations=[d])
mpg = importlib.util.module_from_spec(spec); sys.modules['mpgmres_amd'] = mpg; spec.loader.exec_module(mpg)
"""

CHILD = LOAD + """
A = mpg.gen_spec('laplace:10')
xt = mpg.rand_vect(A.nrows, 5)
b = mpg.host_spmv(A, xt)
p = os.path.join(tempfile.mkdtemp(), 'b.mtx')
open(p, 'w').write('%%MatrixMarket matrix array real general\\n' + f'{A.nrows} 1\\n' + ''.join(f'{v:.17g}\\n' for v in b))
assert np.array_equal(mpg.load_mtx_vector(p, A.nrows), b)
n = mpg.device_count()
f = mpg.solve(A, b, xt, engine='fused', mode='mixed', orth='cgs', prec='jacobi', rlen=30, tol=1e-9)
s = mpg.solve(A, b, xt, engine='surface', mode='mixed', orth='cgs', prec='jacobi', rlen=30, tol=1e-9)
m = mpg.solve_multi_gpu(A, b, xt, ngpus=1, mode='mixed', orth='cgs', prec='jacobi', rlen=30, tol=1e-9)
print('OK', n, f.total_iters, s.total_iters, m.total_iters, mpg.hip_runtime(), 'torch' in sys.modules)
"""

THEN_TORCH = CHILD + """
import torch
print('TORCH', torch.ones(4, device='cuda').sum().item())
"""


def _run(code, **env):
    e = {k: v for k, v in os.environ.items() if k not in ("LD_DEBUG", "MPG_HIP_RUNTIME")}
    e.update(env)
    return subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300, env=e)


def _ok_line(p):
    assert p.returncode == 0, (p.returncode, p.stdout[-2000:], p.stderr[-4000:])
    assert not any(g in p.stderr for g in GLIBC), p.stderr[-4000:]
    out = [ln for ln in p.stdout.splitlines() if ln.startswith("OK ")][-1].split()
    assert int(out[1]) >= 1
    assert min(int(v) for v in out[2:5]) > 0  # fused, surface and one-rank multi-GPU solves ran
    return out


def test_package_only_process_exits_cleanly():
    """device_count, the fused / surface / one-GPU multi solves and the
    Matrix Market vector loader in a process whose code never imports torch
    (the package does, first, when PyTorch is installed)."""
    out = _ok_line(_run(CHILD))
    assert out[5].endswith("torch/lib/libamdhip64.so") and out[6] == "True", out


def test_package_only_on_the_system_runtime_exits_cleanly():
    """The same calls bound to /opt/rocm's runtime (MPG_HIP_RUNTIME=system,
    the CLI's runtime)."""
    out = _ok_line(_run(CHILD, MPG_HIP_RUNTIME="system"))
    assert out[5] == "system" and out[6] == "False", out


def test_package_then_torch_exits_cleanly():
    """The order that aborted: the package first, torch afterwards."""
    p = _run(THEN_TORCH)
    out = _ok_line(p)
    assert out[5].endswith("torch/lib/libamdhip64.so"), out
    assert "TORCH 4.0" in p.stdout


def test_cli_tests_in_their_own_pytest_process():
    """tests/test_cli_gpu.py on its own (no torch imported at collection):
    the pytest process itself exits 0."""
    e = {k: v for k, v in os.environ.items() if k not in ("LD_DEBUG",)}
    p = subprocess.run([sys.executable, "-m", "pytest", str(REPO / "tests" / "test_cli_gpu.py"), "-q", "-x",
                        "-p", "no:cacheprovider", "--timeout", "120", "--timeout-method", "thread"],
                       capture_output=True, text=True, timeout=600, env=e, cwd=str(REPO))
    assert p.returncode == 0, (p.returncode, p.stdout[-3000:], p.stderr[-3000:])
    assert "12 passed" in p.stdout
    assert not any(g in p.stderr + p.stdout for g in GLIBC)
