"""BASELINE config C1 — bcsstk17 through the Matrix Market loader, fp64
GMRES(30) — on its stand-in (tests/golden/make_c1_standin.py: n = 10,974,
428,650 nnz after the symmetric expansion, SPD banded).

CPU (no GPU): the file regenerates bit-identically; the loader
(LoadMatrix.hpp:17-154 semantics) expands it to exactly the matrix SciPy's
independent Matrix Market reader gives, with sorted rows and an explicit
diagonal; the oracle's CPU path (the kernels_mkl.cpp restatement, the C1
path itself) reproduces the committed golden records.
GPU: both engines solve the loaded matrix and match the golden records
(tests/parity.py tolerances), and the CLI runs it with --Apath as the
reference harness does (gmres_perf_test.cpp:309-416)."""
import json
import subprocess
from pathlib import Path

import numpy as np
import pytest

from tests.golden.make_c1_standin import CASES, checksum, write_standin
from tests.parity import compare

GOLDEN = json.loads((Path(__file__).parent / "golden" / "c1_golden.json").read_text())


@pytest.fixture(scope="module")
def c1_path(tmp_path_factory):
    p = tmp_path_factory.mktemp("c1") / "bcsstk17_standin.mtx"
    shape = write_standin(p)
    assert shape == GOLDEN["shape"]
    return p


@pytest.fixture(scope="module")
def c1(mpg, c1_path):
    A = mpg.load_mtx(str(c1_path))
    xt = mpg.rand_vect(A.nrows, 42)
    return A, xt, mpg.host_spmv(A, xt)


def _id(rec):
    c = rec["case"]
    return f"{c['mode']}-{c['orth']}-{c['prec']}"


def test_c1_loader_matches_scipy(mpg, c1, c1_path):
    import scipy.io
    import scipy.sparse as sp

    A, _, b = c1
    assert A.nrows == 10_974 and A.nnz == 428_650
    assert checksum(A) == GOLDEN["checksum"]
    assert float(b.sum()) == GOLDEN["b_sum"]
    S = sp.csr_matrix(scipy.io.mmread(str(c1_path)))
    S.sort_indices()
    assert np.array_equal(A.rowptr, S.indptr) and np.array_equal(A.col, S.indices)
    assert np.array_equal(A.val, S.data)
    rows = np.repeat(np.arange(A.nrows), np.diff(A.rowptr))
    assert np.count_nonzero(A.col == rows) == A.nrows  # explicit diagonal in every row
    assert np.all(np.linalg.eigvalsh(S[:400, :400].toarray()) > 0)  # leading block SPD


@pytest.mark.parametrize("rec", GOLDEN["cases"], ids=_id)
def test_c1_cpu_path_reproduces_golden(mpg, oracle, c1, rec):
    """The CPU path of C1 (oracle = kernels_mkl.cpp restatement, 1 thread)."""
    A, xt, b = c1
    case = {k: v for k, v in rec["case"].items() if k != "matrix"}
    got = oracle.solve(mpg, A, b, xt, threads=1, **case)
    compare(rec, got, case["mode"], case["tol"], case["rlen"], "c1-cpu-" + _id(rec))
    assert got.total_iters == rec["total_iters"]


def test_c1_cases_cover_baseline_config():
    assert any(c["mode"] == "baseline" and c["rlen"] == 30 for c in CASES)


@pytest.mark.gpu
@pytest.mark.parametrize("engine", ["fused", "surface"])
@pytest.mark.parametrize("rec", GOLDEN["cases"], ids=_id)
def test_c1_gpu_matches_golden(mpg, c1, rec, engine):
    A, xt, b = c1
    case = {k: v for k, v in rec["case"].items() if k != "matrix"}
    got = mpg.solve(A, b, xt, engine=engine, **case)
    compare(rec, got, case["mode"], case["tol"], case["rlen"], f"c1-{engine}-{_id(rec)}")


@pytest.mark.gpu
def test_c1_cli_apath(mpg, c1_path):
    from tests.test_cli_gpu import SUMMARY

    rec = next(r for r in GOLDEN["cases"] if r["case"]["mode"] == "baseline" and r["case"]["orth"] == "mgs"
               and r["case"]["prec"] == "identity")
    out = subprocess.run([str(mpg.CLI), "--Apath", str(c1_path), "--rlen", "30", "--mode", "baseline", "--orth",
                          "mgs", "--prec", "identity", "--tol", "1e-10", "--gpu"],
                         capture_output=True, text=True, timeout=120, check=True).stdout
    m = SUMMARY.search(out)
    assert m, out
    assert int(m.group(3)) == rec["restarts"] and int(m.group(4)) == rec["total_iters"]
