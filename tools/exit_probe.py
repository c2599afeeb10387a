"""Process-exit probe: run the package's calls in fresh child
processes, without torch unless a variant names it, and record each child's
exit code and the tail of its stderr. A failing variant is run again with
LD_DEBUG=fini (glibc's list of the finalizers it calls, in order).
package_then_torch_system_runtime keeps /opt/rocm's runtime (MPG_HIP_RUNTIME=
system) and imports torch afterwards: the two-runtime exit abort, kept as the
evidence of the cause.

    python tools/exit_probe.py [--out gpurun_out/exit_probe.json] [variant ...]
"""
import argparse
import json
import os
import subprocess
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent

PRELUDE = f"""
import sys, importlib.util
sys.path.insert(0, {str(REPO)!r})
def load():
    d = {str(REPO / 'icl-mixed-precision-gmres_amd')!r}
    spec = importlib.util.spec_from_file_location('mpgmres_amd', d + '/__init__.py', submodule_search_locations=[d])
    m = importlib.util.module_from_spec(spec); sys.modules['mpgmres_amd'] = m; spec.loader.exec_module(m); return m
"""

VARIANTS = {
    "load": "mpg = load(); mpg.hip_lib(); mpg.host_lib()",
    "device_count": "mpg = load(); print(mpg.device_count())",
    "ctx": ("import ctypes as C\nmpg = load(); lib = mpg.hip_lib(); c = C.c_void_p()\n"
            "assert lib.mpg_ctx_create(0, C.byref(c)) == 0; assert lib.mpg_ctx_destroy(c) == 0"),
    "host_only": ("import numpy as np\nmpg = load(); A = mpg.gen_spec('laplace:10'); x = mpg.rand_vect(A.nrows, 5)\n"
                  "b = mpg.host_spmv(A, x)"),
    "solve_fused": ("import numpy as np\nmpg = load(); A = mpg.gen_spec('laplace:10'); xt = mpg.rand_vect(A.nrows, 5)\n"
                    "b = mpg.host_spmv(A, xt)\n"
                    "r = mpg.solve(A, b, xt, engine='fused', mode='mixed', orth='cgs', prec='jacobi', rlen=30, tol=1e-9)\n"
                    "print(r.total_iters)"),
    "solve_surface": ("import numpy as np\nmpg = load(); A = mpg.gen_spec('laplace:10'); xt = mpg.rand_vect(A.nrows, 5)\n"
                      "b = mpg.host_spmv(A, xt)\n"
                      "r = mpg.solve(A, b, xt, engine='surface', mode='mixed', orth='cgs', prec='jacobi', rlen=30, "
                      "tol=1e-9)\nprint(r.total_iters)"),
    "cli_sequence": ("import numpy as np, tempfile, os\nmpg = load(); A = mpg.gen_spec('laplace:10')\n"
                     "xt = mpg.rand_vect(A.nrows, 5); b = mpg.host_spmv(A, xt)\n"
                     "p = os.path.join(tempfile.mkdtemp(), 'b.mtx')\n"
                     "open(p, 'w').write('%%MatrixMarket matrix array real general\\n' + f'{A.nrows} 1\\n' + "
                     "''.join(f'{v:.17g}\\n' for v in b))\n"
                     "assert np.array_equal(mpg.load_mtx_vector(p, A.nrows), b)\n"
                     "r = mpg.solve(A, b, np.zeros(A.nrows), engine='fused', mode='mixed', orth='cgs', prec='jacobi', "
                     "rlen=30, tol=1e-9)\n"
                     "print(mpg.device_count() + 1, r.total_iters)"),
    "cli_sequence_torch_first": None,  # filled below: torch imported before the package
}
VARIANTS["cli_sequence_torch_first"] = "import torch\n" + VARIANTS["cli_sequence"]
# the package first, torch afterwards (torch then binds to the HIP runtime the
# package loaded: the same soname, libamdhip64.so.7)
VARIANTS["package_then_torch"] = VARIANTS["solve_fused"] + "\nimport torch\nprint(torch.ones(4, device='cuda').sum().item())"
# the cause without the package: torch's own runtime initialised through
# ctypes (a device count, an allocation), torch imported afterwards
VARIANTS["torch_runtime_init_then_torch"] = (
    "import ctypes as C, importlib.util, os\n"
    "d = os.path.join(list(importlib.util.find_spec('torch').submodule_search_locations)[0], 'lib')\n"
    "h = C.CDLL(os.path.join(d, 'libamdhip64.so'), mode=C.RTLD_GLOBAL)\n"
    "n = C.c_int(); assert h.hipGetDeviceCount(C.byref(n)) == 0\n"
    "p = C.c_void_p(); assert h.hipMalloc(C.byref(p), C.c_size_t(1 << 20)) == 0; assert h.hipFree(p) == 0\n"
    "import torch\nprint(torch.ones(4, device='cuda').sum().item())")
VARIANTS["package_then_torch_system_runtime"] = None  # run with MPG_HIP_RUNTIME=system: the two-runtime abort
VARIANTS["multi_gpu_one"] = ("import numpy as np\nmpg = load(); A = mpg.gen_spec('laplace:10'); xt = mpg.rand_vect(A.nrows, 5)\n"
                             "b = mpg.host_spmv(A, xt)\n"
                             "r = mpg.solve_multi_gpu(A, b, xt, ngpus=1, mode='mixed', orth='cgs', prec='jacobi', rlen=30, "
                             "tol=1e-9)\nprint(r.total_iters)")


def run(name, code, extra_env=None, timeout=120):
    env = dict(os.environ)
    env.update(extra_env or {})
    p = subprocess.run([sys.executable, "-c", PRELUDE + code], capture_output=True, text=True, timeout=timeout,
                       env=env)
    err = p.stderr
    return {"variant": name, "rc": p.returncode, "stdout": p.stdout[-400:], "stderr_tail": err[-6000:],
            "glibc_message": any(s in err for s in ("double free", "corruption", "free(): invalid")),
            "env": extra_env or {}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=str(REPO / "gpurun_out" / "exit_probe.json"))
    ap.add_argument("variants", nargs="*")
    a = ap.parse_args()
    names = a.variants or list(VARIANTS)
    out = []
    for n in names:
        if n == "package_then_torch_system_runtime":
            r = run(n, VARIANTS["package_then_torch"], {"MPG_HIP_RUNTIME": "system"})
            print(json.dumps({k: r[k] for k in ("variant", "rc", "glibc_message")}), flush=True)
            out.append(r)
            continue
        r = run(n, VARIANTS[n])
        print(json.dumps({k: r[k] for k in ("variant", "rc", "glibc_message")}), flush=True)
        out.append(r)
        if r["rc"] != 0:
            for env in ({"LD_DEBUG": "fini"},):
                rr = run(n, VARIANTS[n], env)
                print(json.dumps({k: rr[k] for k in ("variant", "rc", "glibc_message", "env")}), flush=True)
                out.append(rr)
    Path(a.out).parent.mkdir(parents=True, exist_ok=True)
    Path(a.out).write_text(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
