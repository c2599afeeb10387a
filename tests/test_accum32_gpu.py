"""The reference's fp32 accumulation class (accum="f32",
mpg_arnoldi_set_accum, include/mpgmres/arnoldi.h).

The reference's mixed mode accumulates its fp32 Arnoldi in fp32:
cblas_sdot / snrm2 (kernels_mkl.cpp:82,94,104,114), cblas_sgemv (:284),
mkl_sparse_s_mv (:348); its GPU backend cublasSdot / Sgemv and
cusparseScsrmv (kernels_cuda.cpp:132,160,530,609). Under accum="f32" every
partial sum of the fused engine's fp32 Arnoldi is an fp32 value (SpMV row
sums, panel dots, norms, the CGS update's V c, the solution update's V y),
and parity is two-sided against fp32-accumulating evaluations only: every
cycle's backward error inside [min/3, 3 max] over the oracle's MKL runs at
1, 4 and 8 threads and its "pair32" loop mode -- the same fp32-accumulating
operations with the long reductions in pairwise (tree) order, the order of a
GPU reduction (tests/parity.py compare_mkl(extra=("pair32",))). The oracle's
fp64-summing loop kernels (the GPU's default class) are not in the envelope.
Measured on the CPU oracle (profiles/r06_accum/): within the fp32 class the
order sets plain CGS's loss of orthogonality -- BAND-300k m = 100 cycle-1
backward error: a single sequential fp32 chain 1.5e-7, MKL 6.0e-9, pairwise
fp32 4.5e-10 (GPU f32: 3.9e-10), fp64 sums 2.4e-10.
"""
import json
from pathlib import Path

import numpy as np
import pytest

from tests.golden.make_golden import inputs
from tests.parity import MKL_THREADS, compare, compare_mkl

pytestmark = pytest.mark.gpu

GOLDEN = Path(__file__).parent / "golden"


def _solve32(mpg, A, b, xt, **opts):
    return mpg.solve(A, b, xt, engine="fused", accum="f32", **opts)


def test_accum_is_what_runs(mpg):
    """The engine reports the class it runs: f32 for an fp32 Arnoldi on
    request, f64 otherwise (an fp64 Arnoldi is the reference's fp64 class)."""
    A = mpg.gen_band(50_000, 5, 4, seed=7)
    xt = mpg.rand_vect(A.nrows, 42)
    b = mpg.host_spmv(A, xt)
    for mode, accum, want in (("mixed", "f32", "f32"), ("mixed", "f64", "f64"), ("single", "f32", "f32"),
                              ("baseline", "f32", "f64"), ("mixed-half", "f32", "f32")):
        eng = mpg.Engine(A, b, xt, mode=mode, orth="cgs", prec="identity", rlen=30, tol=0.0, max_restarts=3,
                         accum=accum)
        lay = eng.spmv_layout()
        eng.close()
        assert lay["accum"] == want, (mode, accum, lay)


def test_surface_refuses_accum32(mpg):
    A = mpg.gen_band(2_000, 5, 4, seed=7)
    xt = mpg.rand_vect(A.nrows, 42)
    b = mpg.host_spmv(A, xt)
    with pytest.raises(RuntimeError, match="fused engine only"):
        mpg.solve(A, b, xt, engine="surface", mode="mixed", orth="cgs", rlen=30, tol=1e-8, accum="f32")


def test_accum32_changes_the_arithmetic(mpg):
    """f32 accumulation is a different arithmetic (not a relabelled f64 run):
    the step history differs in the last bits, and the solve still converges."""
    A = mpg.gen_band(200_000, 5, 4, seed=7)
    xt = mpg.rand_vect(A.nrows, 42)
    b = mpg.host_spmv(A, xt)
    opts = dict(mode="mixed", orth="cgs", prec="jacobi", rlen=30, tol=1e-10, max_restarts=50)
    r64 = mpg.solve(A, b, xt, engine="fused", **opts)
    r32 = _solve32(mpg, A, b, xt, **opts)
    assert r64.status == r32.status == "converged"
    assert not np.array_equal(r64.step_res, r32.step_res)


@pytest.mark.parametrize("which", ["stencil27p", "fem27"])
def test_accum32_storage_forms_same_bits(mpg, which):
    """The f32 class is one arithmetic in every storage form: products rounded
    to fp32 and added in CSR order on SELL, node blocks and CSR row blocks
    (mac / add_prod, internal.hpp), so the Arnoldi SpMVs give one another's
    bits. Node blocks and CSR agree over the whole solve; SELL over cycle 0
    (x0 = 0, so its residual is b in any order): from the first restart on,
    the fp64 residual prologue differs -- SELL's fp64 row sums contract to
    fused multiply-adds of fp64 products, the CSR tile adds the products it
    staged in LDS (the same in accum f64, tools/accum_forms_diag.py,
    profiles/r06_accum/forms.jsonl)."""
    if which == "stencil27p":
        A = mpg.gen_stencil27p(40, 3, ny=40, nz=8, block=64, perm_seed=5)
    else:
        A = mpg.gen_fem27(24, 3, keep_pct=70, seed=13)
    xt = mpg.rand_vect(A.nrows, 42)
    b = mpg.host_spmv(A, xt)
    opts = dict(mode="mixed", orth="cgs", prec="jacobi", rlen=30, tol=0.0, max_restarts=3)
    got = {f: _solve32(mpg, A, b, xt, spmv_format=f, **opts) for f in ("csr", "sell", "node")}
    np.testing.assert_array_equal(got["node"].step_res, got["csr"].step_res)
    np.testing.assert_array_equal(got["node"].x, got["csr"].x)
    np.testing.assert_array_equal(got["sell"].step_res[:30], got["csr"].step_res[:30])


_MKL = {}


@pytest.mark.parametrize("orth", ["cgs", "mgs", "cgsr"])
def test_band300k_m100_accum32_mkl_envelope(mpg, oracle, orth):
    """BAND-300k at m = 100, 2 cycles at tol = 0: where the fp64 class ran
    25x more accurate than MKL with CGS (cycle-1 backward error 2.4e-10 vs
    6.0e-9), the f32 class must land inside MKL's own envelope."""
    A = mpg.gen_band(300_000, 5, 4, seed=7)
    xt = mpg.rand_vect(A.nrows, 42)
    b = mpg.host_spmv(A, xt)
    opts = dict(mode="mixed", orth=orth, prec="jacobi", rlen=100, tol=0.0, max_restarts=2)
    got = _solve32(mpg, A, b, xt, **opts)
    runs = compare_mkl(oracle, mpg, A, b, xt, got, opts, f"band300k-{orth}-m100/f32",
                       runs=_MKL.setdefault(("band300k", orth), {}), extra=("pair32",))
    assert got.total_iters == runs[1].total_iters == 200


@pytest.mark.parametrize("orth", ["cgs", "cgsr"])
@pytest.mark.parametrize("which", ["stencil27p", "fem27p"])
def test_irregular_accum32_mkl_envelope(mpg, oracle, which, orth):
    from tests.test_irregular_gpu import _problem

    A, xt, b = _problem(mpg, which)
    opts = dict(mode="mixed", orth=orth, prec="jacobi", rlen=30, tol=1e-10, max_restarts=200)
    got = _solve32(mpg, A, b, xt, **opts)
    runs = compare_mkl(oracle, mpg, A, b, xt, got, opts, f"{which}-{orth}/f32",
                       runs=_MKL.setdefault((which, orth), {}), extra=("pair32",))
    assert runs[1].status == got.status == "converged"


@pytest.mark.parametrize("orth", ["cgs", "mgs", "cgsr"])
def test_lap1m_accum32_mkl_envelope(mpg, oracle, orth):
    """C3 (LAP-1M, fp32 inner + fp64 outer), 3 cycles at tol = 0."""
    A = mpg.gen_laplace3d(100)
    xt = mpg.rand_vect(A.nrows, 42)
    b = mpg.host_spmv(A, xt)
    opts = dict(mode="mixed", orth=orth, prec="identity", rlen=30, tol=0.0, max_restarts=3)
    got = _solve32(mpg, A, b, xt, **opts)
    runs = compare_mkl(oracle, mpg, A, b, xt, got, opts, f"lap1m-{orth}/f32",
                       runs=_MKL.setdefault(("lap1m", orth), {}), extra=("pair32",))
    assert got.total_iters == runs[1].total_iters == 90


@pytest.fixture(scope="module")
def mats(mpg):
    return inputs(mpg)


def _fp32_records(name):
    cases = json.loads((GOLDEN / name).read_text())["cases"]
    return [c for c in cases if c["case"]["mode"] in ("mixed", "single")]


def _case_id(c):
    k = c["case"]
    return f"{k['matrix']}-{k['mode']}-{k['orth']}-{k['prec']}-m{k['rlen']}"


_GOLDEN_ENV = {}


@pytest.mark.parametrize("rec", _fp32_records("gmres_golden.json") + _fp32_records("gmres_golden_m100.json"),
                         ids=_case_id)
def test_golden_accum32(mpg, oracle, mats, rec):
    """Every fp32-Arnoldi golden record (m = 10 / 30 / 100; made by the oracle
    on MKL's pinned branch at 1 thread) in the f32 class, its backward errors
    inside the envelope of the record, MKL live at 4 and 8 threads and the
    oracle's pair32 mode."""
    case = dict(rec["case"])
    A = mats[case.pop("matrix")]
    xt = mpg.rand_vect(A.nrows, 42)
    b = mpg.host_spmv(A, xt)
    got = _solve32(mpg, A, b, xt, **case)
    key = _case_id(rec)
    if key not in _GOLDEN_ENV:
        from types import SimpleNamespace

        g = SimpleNamespace(cyc_r_norm=rec["cyc_r_norm"], cyc_normalization=rec["cyc_normalization"],
                            restarts=rec["restarts"])
        _GOLDEN_ENV[key] = [g] + [oracle.solve(mpg, A, b, xt, backend="mkl", threads=t, **case)
                                  for t in MKL_THREADS if t != 1] + \
            [oracle.solve(mpg, A, b, xt, backend="pair32", threads=1, **case)]
    compare(rec, got, case["mode"], case["tol"], case["rlen"], key + "/f32", envelope=_GOLDEN_ENV[key])
