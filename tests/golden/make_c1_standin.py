"""BASELINE config C1 (bcsstk17, fp64 GMRES(30), the kernels_mkl.cpp CPU
path) without the SuiteSparse file: a deterministic stand-in of the same
shape, written as a Matrix Market file and loaded through the reference's
loader semantics (LoadMatrix.hpp:17-154, our host/problems.cpp).

bcsstk17 is a real symmetric positive-definite stiffness matrix, n = 10,974,
stored as its lower triangle (219,812 entries; 428,650 after the symmetric
expansion, ~39 per row) with most entries within a few hundred of the
diagonal. The stand-in ("SPD banded n = 10,974, ~39 nnz/row"):
  * n = 10,974; 208,838 distinct strictly-lower entries (i, j) drawn
    uniformly from the band 1 <= i - j <= 400 (numpy PCG64, seed 17), so
    the lower triangle holds 219,812 entries with the diagonal and the
    expanded matrix 428,650, as bcsstk17;
  * off-diagonal values -u, u ~ U(0.1, 1);
  * diagonal a_ii = (1 + 1e-3) * sum_j |a_ij| over the expanded row, so the
    matrix is SPD (strict diagonal dominance) but not trivially conditioned
    (GMRES(30) needs several restarts).
The file is stored lower-triangle, column by column, as SuiteSparse ships
it ("coordinate real symmetric"), so loading it exercises the symmetric
mirror, the explicit diagonal and the per-row sort.

The .mtx (~9 MB) is not committed: tests regenerate it (bit-identically;
values are printed with 17 significant digits) and check it against the
checksums in tests/golden/c1_golden.json, which also holds the oracle's
records for the C1 solves (parity unpinned by reference data: the reference
ships no fixtures; the oracle is the MKL restatement, oracle/).

Usage: python tests/golden/make_c1_standin.py   (writes tests/golden/c1_golden.json)
"""
import json
import sys
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
REPO = HERE.parent.parent

N = 10_974
N_LOWER_OFFDIAG = 208_838
BAND = 400
SEED = 17
MARGIN = 1e-3

# the C1 solves recorded by the oracle: fp64 GMRES(30) as BASELINE C1, plus
# the mixed driver and MGS on the same matrix
CASES = [dict(mode=mode, orth=orth, prec=prec, rlen=30, tol=1e-10, max_restarts=400)
         for mode in ("baseline", "mixed") for orth in ("cgs", "mgs") for prec in ("identity", "jacobi")]


def lower_entries():
    """(rows, cols, vals) of the strictly-lower part, sorted column-major."""
    rng = np.random.Generator(np.random.PCG64(SEED))
    keys = set()
    rows, cols = [], []
    while len(rows) < N_LOWER_OFFDIAG:
        need = N_LOWER_OFFDIAG - len(rows)
        i = rng.integers(1, N, size=2 * need)
        d = rng.integers(1, BAND + 1, size=2 * need)
        for a, b in zip(i.tolist(), d.tolist()):
            j = a - b
            if j < 0 or (a, j) in keys:
                continue
            keys.add((a, j))
            rows.append(a)
            cols.append(j)
            if len(rows) == N_LOWER_OFFDIAG:
                break
    rows = np.array(rows, dtype=np.int64)
    cols = np.array(cols, dtype=np.int64)
    vals = -rng.uniform(0.1, 1.0, size=N_LOWER_OFFDIAG)
    order = np.lexsort((rows, cols))
    return rows[order], cols[order], vals[order]


def write_standin(path) -> dict:
    """Write the stand-in .mtx; returns its shape facts."""
    r, c, v = lower_entries()
    absrow = np.zeros(N)
    np.add.at(absrow, r, np.abs(v))
    np.add.at(absrow, c, np.abs(v))
    diag = (1.0 + MARGIN) * absrow
    # merge the diagonal into the column-major lower triangle (diagonal first in its column)
    rr = np.concatenate([r, np.arange(N)])
    cc = np.concatenate([c, np.arange(N)])
    vv = np.concatenate([v, diag])
    isdiag = np.concatenate([np.zeros(len(r), bool), np.ones(N, bool)])
    order = np.lexsort((rr, ~isdiag, cc))
    rr, cc, vv = rr[order], cc[order], vv[order]
    with open(path, "w") as f:
        f.write("%%MatrixMarket matrix coordinate real symmetric\n")
        f.write("% bcsstk17-shaped SPD banded stand-in (tests/golden/make_c1_standin.py)\n")
        f.write(f"{N} {N} {len(vv)}\n")
        f.write("".join(f"{a + 1} {b + 1} {x:.17g}\n" for a, b, x in zip(rr.tolist(), cc.tolist(), vv.tolist())))
    return {"n": N, "lower_entries": int(len(vv)), "expanded_nnz": int(2 * len(r) + N)}


def checksum(A):
    return [float(A.val.sum()), int(A.col.astype(np.int64).sum()), int(A.nnz),
            float(np.abs(A.val).max())]


def main():
    sys.path.insert(0, str(REPO))
    from tests.conftest import load_package
    from oracle import binding

    mpg = load_package()
    import tempfile

    with tempfile.TemporaryDirectory() as d:
        p = Path(d) / "bcsstk17_standin.mtx"
        shape = write_standin(p)
        A = mpg.load_mtx(str(p))
    xt = mpg.rand_vect(A.nrows, 42)
    b = mpg.host_spmv(A, xt)
    out = {"backend": binding.backend(), "shape": shape, "checksum": checksum(A), "b_sum": float(b.sum()),
           "cases": []}
    for case in CASES:
        r = binding.solve(mpg, A, b, xt, threads=1, **case)
        out["cases"].append(dict(
            case=dict(case, matrix="c1_standin"), status=r.status, restarts=int(r.restarts),
            total_iters=int(r.total_iters), res_norm=r.res_norm, err_norm=r.err_norm, minvb_norm=r.minvb_norm,
            cyc_r_norm=r.cyc_r_norm.tolist(), cyc_normalization=r.cyc_normalization.tolist(),
            cyc_beta=r.cyc_beta.tolist(), step_res=r.step_res.tolist(),
            x_sum=float(r.x.sum()), x_head=r.x[:16].tolist()))
        print(case, r.status, r.restarts, r.total_iters, flush=True)
    (HERE / "c1_golden.json").write_text(json.dumps(out, indent=0))
    print(f"wrote {len(out['cases'])} cases, backend {out['backend']}")


if __name__ == "__main__":
    main()
