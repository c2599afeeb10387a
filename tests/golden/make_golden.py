"""Generate the golden fixtures of the GMRES path from the CPU oracle.

The reference repository holds no tests, fixtures or golden vectors for
this path and cannot be built here (Kokkos 3.1 and MKL headers are absent),
so the fixtures are produced by the oracle (oracle/cpu_gmres.cpp: the
reference's algorithm restated over the MKL 2021.4 runtime the image ships)
after it has been cross-checked against the independent NumPy restatement
(oracle/gmres_np.py; tests/test_oracle.py). Single MKL thread on MKL's
COMPATIBLE code branch (MKL_CBWR, which oracle/binding.py pins: conditional
numerical reproducibility), so the values are reproducible on the GPU box's
EPYC as on this Xeon, not only on this machine (round 5; the round-1..4
records came from MKL's default branch, AVX-512 on the build container).

Inputs are deterministic: lap10 (7-point Laplacian 10^3), band2000 (the
BAND generator, n=2000, offsets -5..+4, seed 7), convdiff32 (2-D upwind
convection-diffusion, 32^2, built below), x_true = rand_vect(n, 42),
b = A x_true. Each case records the per-restart true residual norms and
normalisations, the per-step Arnoldi residuals |s(k+1)|, iteration counts,
final resNorm/errNorm and a checksum of x.

Usage: python tests/golden/make_golden.py   (writes tests/golden/gmres_golden.json)
       python tests/golden/make_golden.py --m100   (GMRES(100) records: gmres_golden_m100.json)
"""
import json
import sys
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
REPO = HERE.parent.parent
sys.path.insert(0, str(REPO))

from tests.conftest import load_package  # noqa: E402


def convdiff(mpg, m=32, peclet=40.0):
    """-Δu + Pe·(u_x + u_y) on an m×m grid, first-order upwind, h = 1/(m+1)."""
    h = 1.0 / (m + 1)
    n = m * m
    rp, ci, va = [0], [], []
    for j in range(m):
        for i in range(m):
            row = []
            if j > 0:
                row.append((i + (j - 1) * m, -1.0 / h**2 - peclet / h))
            if i > 0:
                row.append((i - 1 + j * m, -1.0 / h**2 - peclet / h))
            row.append((i + j * m, 4.0 / h**2 + 2 * peclet / h))
            if i + 1 < m:
                row.append((i + 1 + j * m, -1.0 / h**2))
            if j + 1 < m:
                row.append((i + (j + 1) * m, -1.0 / h**2))
            for c, v in row:
                ci.append(c)
                va.append(v * h * h)  # scale to O(1) entries
            rp.append(len(ci))
    return mpg.Csr(n, n, np.array(rp, np.int32), np.array(ci, np.int32), np.array(va, np.float64))


def inputs(mpg):
    return {
        "lap10": mpg.gen_laplace3d(10),
        "band2000": mpg.gen_band(2000, 5, 4, seed=7),
        "convdiff32": convdiff(mpg),
    }


def checksum(A):
    return [float(A.val.sum()), int(A.col.astype(np.int64).sum()), int(A.nnz)]


CASES = []
for mat in ("lap10", "band2000", "convdiff32"):
    for mode in ("mixed", "baseline", "single-prec", "single"):
        for orth in ("cgs", "mgs", "cgsr"):
            for prec in ("identity", "jacobi"):
                for m in (10, 30):
                    tol = 1e-5 if mode == "single" else 1e-10
                    CASES.append(dict(matrix=mat, mode=mode, orth=orth, prec=prec, rlen=m, tol=tol, max_restarts=200))
# ILU(0) / ILU-Jacobi (3 sweeps per factor): SURVEY §8f #2
for mat in ("lap10", "band2000", "convdiff32"):
    for mode in ("mixed", "baseline", "single-prec", "single"):
        for prec in ("ilu", "ilu_jacobi"):
            tol = 1e-5 if mode == "single" else 1e-10
            CASES.append(dict(matrix=mat, mode=mode, orth="cgs", prec=prec, rlen=30, tol=tol, max_restarts=200,
                              jacobi_steps=3))


# GMRES(100), the restart length of every published reference number
# (automated.py:41, the notebook's timings at rlen '100'): identity / Jacobi
# x 4 modes x 3 orthogonalisations, in their own file (gmres_golden_m100.json)
CASES_M100 = []
for mat in ("lap10", "band2000", "convdiff32"):
    for mode in ("mixed", "baseline", "single-prec", "single"):
        for orth in ("cgs", "mgs", "cgsr"):
            for prec in ("identity", "jacobi"):
                tol = 1e-5 if mode == "single" else 1e-10
                CASES_M100.append(dict(matrix=mat, mode=mode, orth=orth, prec=prec, rlen=100, tol=tol,
                                       max_restarts=200))


def main():
    m100 = "--m100" in sys.argv
    cases, fname = (CASES_M100, "gmres_golden_m100.json") if m100 else (CASES, "gmres_golden.json")
    mpg = load_package()
    from oracle import binding

    mats = inputs(mpg)
    out = {"backend": binding.backend(), "mkl_cbwr": binding.cbwr(), "inputs": {}, "cases": []}
    for name, A in mats.items():
        xt = mpg.rand_vect(A.nrows, 42)
        b = mpg.host_spmv(A, xt)
        out["inputs"][name] = {"n": A.nrows, "checksum": checksum(A), "b_sum": float(b.sum())}
    for case in cases:
        A = mats[case["matrix"]]
        xt = mpg.rand_vect(A.nrows, 42)
        b = mpg.host_spmv(A, xt)
        opts = {k: v for k, v in case.items() if k != "matrix"}
        r = binding.solve(mpg, A, b, xt, threads=1, **opts)
        out["cases"].append(dict(
            case=case, status=r.status, restarts=int(r.restarts), total_iters=int(r.total_iters),
            res_norm=r.res_norm, err_norm=r.err_norm, minvb_norm=r.minvb_norm,
            cyc_r_norm=r.cyc_r_norm.tolist(), cyc_normalization=r.cyc_normalization.tolist(),
            cyc_beta=r.cyc_beta.tolist(), step_res=r.step_res.tolist(),
            x_sum=float(r.x.sum()), x_head=r.x[:16].tolist()))
    (HERE / fname).write_text(json.dumps(out, indent=0))
    print(f"wrote {len(out['cases'])} cases, backend {out['backend']}")


if __name__ == "__main__":
    main()
