"""CPU checks of the oracle itself (no GPU).

The reference holds no tests or golden vectors for this path, so the oracle
is pinned by (1) the reference's own seeded input generator, whose first
values are known (mt19937(42) + uniform_real_distribution<float>,
gmres_perf_test.cpp:39-51), (2) agreement with an independent NumPy
restatement of the algorithm, and (3) the committed golden records it
produced (tolerances of tests/parity.py, since MKL's vector code paths differ
between host CPUs).
"""
import json
from pathlib import Path

import numpy as np
import pytest

from oracle import gmres_np
from tests.golden.make_golden import convdiff, inputs
from tests.parity import as_ref, compare

GOLDEN = json.loads((Path(__file__).parent / "golden" / "gmres_golden.json").read_text())


def test_rand_vect_matches_reference_sequence(mpg):
    x = mpg.rand_vect(5, 42)
    assert np.allclose(x, [0.37454012, 0.796543002, 0.95071429, 0.183434784, 0.731993914], rtol=0, atol=5e-9)
    # values are floats widened to double
    assert np.all(x.astype(np.float32).astype(np.float64) == x)


def test_backend_reported(oracle):
    assert oracle.backend() in ("mkl", "loops")


@pytest.mark.parametrize("mode", ["mixed", "baseline"])
def test_oracle_loops_backend_per_solve(mpg, oracle, mode):
    """backend="loops" (the summation class of the HIP kernels, used by the
    large live-oracle GPU tests) passes the parity rules against the default
    backend and leaves the default in place afterwards."""
    A = convdiff(mpg, 16)
    xt = mpg.rand_vect(A.nrows, 42)
    b = mpg.host_spmv(A, xt)
    opts = dict(mode=mode, orth="cgs", prec="jacobi", rlen=12, tol=1e-10, max_restarts=300)
    d = oracle.solve(mpg, A, b, xt, **opts)
    lp = oracle.solve(mpg, A, b, xt, backend="loops", **opts)
    compare(as_ref(d), lp, mode, 1e-10, 12, f"loops-vs-default {mode}")
    again = oracle.solve(mpg, A, b, xt, **opts)
    assert np.array_equal(again.step_res, d.step_res) and np.array_equal(again.x, d.x)
    with pytest.raises(ValueError):
        oracle.solve(mpg, A, b, xt, backend="blas", **opts)


@pytest.mark.parametrize("mode", ["mixed", "baseline", "single-prec", "single"])
@pytest.mark.parametrize("orth", ["cgs", "mgs", "cgsr"])
@pytest.mark.parametrize("prec", ["identity", "jacobi"])
def test_oracle_vs_numpy_restatement(mpg, oracle, mode, orth, prec):
    A = convdiff(mpg, 16)
    xt = mpg.rand_vect(A.nrows, 42)
    b = mpg.host_spmv(A, xt)
    tol = 1e-5 if mode == "single" else 1e-10
    r = oracle.solve(mpg, A, b, xt, mode=mode, orth=orth, prec=prec, rlen=12, tol=tol, max_restarts=300)
    q = gmres_np.solve(A, b, mode=mode, orth=orth, prec=prec, rlen=12, tol=tol, max_restarts=300)
    q["step_cycle"] = np.repeat(np.arange(len(q["cyc_r_norm"])), 12)[: len(q["step_res"])]
    # the NumPy run plays "got", the oracle record plays "ref"
    ns = type("R", (), {})()
    for k in ("status", "restarts", "total_iters", "step_res", "step_cycle", "cyc_r_norm", "cyc_normalization", "x"):
        setattr(ns, k, q[k])
    compare(as_ref(r), ns, mode, tol, 12, f"np-vs-oracle {mode}/{orth}/{prec}")


def test_oracle_reproduces_golden(mpg, oracle):
    mats = inputs(mpg)
    for name, meta in GOLDEN["inputs"].items():
        A = mats[name]
        assert A.nrows == meta["n"] and A.nnz == meta["checksum"][2]
        assert int(A.col.astype(np.int64).sum()) == meta["checksum"][1]
        assert abs(A.val.sum() - meta["checksum"][0]) <= 1e-9 * abs(meta["checksum"][0])
    for rec in GOLDEN["cases"][::5]:
        case = dict(rec["case"])
        A = mats[case.pop("matrix")]
        xt = mpg.rand_vect(A.nrows, 42)
        b = mpg.host_spmv(A, xt)
        r = oracle.solve(mpg, A, b, xt, threads=1, **case)
        compare(rec, r, case["mode"], case["tol"], case["rlen"], str(rec["case"]))


def test_oracle_reproduces_golden_bits(mpg, oracle):
    """Round 5: the records were made on MKL's pinned COMPATIBLE branch
    (MKL_CBWR, oracle/binding.py) at one thread, so the oracle reproduces
    them bit for bit -- here and on the GPU box's EPYC (tools/oracle_cnr.py
    --golden there: profiles/r05_oracle_cnr/)."""
    assert oracle.cbwr() == GOLDEN["mkl_cbwr"] == "COMPATIBLE"
    mats = inputs(mpg)
    for rec in GOLDEN["cases"][::7]:
        case = dict(rec["case"])
        A = mats[case.pop("matrix")]
        xt = mpg.rand_vect(A.nrows, 42)
        b = mpg.host_spmv(A, xt)
        r = oracle.solve(mpg, A, b, xt, threads=1, **case)
        assert r.step_res.tolist() == rec["step_res"] and r.x[:16].tolist() == rec["x_head"], rec["case"]
        assert r.cyc_r_norm.tolist() == rec["cyc_r_norm"] and r.total_iters == rec["total_iters"], rec["case"]


def test_oracle_abort_semantics(mpg, oracle):
    A = mpg.gen_laplace3d(8)
    xt = mpg.rand_vect(A.nrows, 42)
    b = mpg.host_spmv(A, xt)
    r = oracle.solve(mpg, A, b, xt, mode="mixed", orth="cgs", prec="identity", rlen=30, tol=0.0, max_restarts=2)
    assert r.status == "aborted" and r.total_iters == 60 and len(r.cyc_r_norm) == 3


def test_oracle_adaptive_restart_strategies(mpg, oracle):
    """RelPrecRes / RepeatIteration / LostOrthogonality (IterUtil.hpp:84-227) run and
    restart earlier than the fixed-length strategy."""
    A = convdiff(mpg, 24)
    xt = mpg.rand_vect(A.nrows, 42)
    b = mpg.host_spmv(A, xt)
    base = oracle.solve(mpg, A, b, xt, mode="mixed", orth="mgs", prec="identity", rlen=40, tol=1e-9)
    for extra in (dict(rtol=1e-3), dict(rtol=1e-3, repeat_iter=True), dict(rtol=1e-2, orthloss=True)):
        r = oracle.solve(mpg, A, b, xt, mode="mixed", orth="mgs", prec="identity", rlen=40, tol=1e-9, **extra)
        assert r.status == "converged"
        assert r.restarts >= base.restarts


# ---- ILU(0) / ILU-Jacobi (kernels_mkl.cpp:416-500 with diag_inds filled) ----

@pytest.mark.parametrize("dt", [np.float64, np.float32])
def test_oracle_ilu0_matches_numpy_restatement(mpg, oracle, dt):
    A = convdiff(mpg, 12)
    lu, di = oracle.ilu0(A, dt)
    lo, up = gmres_np.ilu0_factors(A, np.float64)
    full = (lo + up).toarray()
    got = np.zeros_like(full)
    for i in range(A.nrows):
        for k in range(A.rowptr[i], A.rowptr[i + 1]):
            got[i, A.col[k]] = lu[k]
        assert A.col[di[i]] == i
    np.testing.assert_allclose(got, full.astype(dt), rtol=2e-16 if dt == np.float64 else 0, atol=0)


@pytest.mark.parametrize("kind,steps", [("ilu", 1), ("ilu_jacobi", 1), ("ilu_jacobi", 3)])
@pytest.mark.parametrize("dt", [np.float64, np.float32])
def test_oracle_ilu_apply_matches_numpy(mpg, oracle, kind, steps, dt):
    A = convdiff(mpg, 12)
    x = mpg.rand_vect(A.nrows, 7).astype(dt)
    got = oracle.ilu_apply(A, x, kind, steps, dt)
    lo, up = gmres_np.ilu0_factors(A, dt)
    ref = gmres_np.ilu_apply(lo, up, x, dt, kind, steps)
    tol = 1e-12 if dt == np.float64 else 2e-5
    np.testing.assert_allclose(got, ref, rtol=tol, atol=tol * np.abs(ref).max())


def test_oracle_ilu_jacobi_tends_to_ilu(mpg, oracle):
    """Jacobi sweeps on a diagonally dominant factor converge to the exact
    triangular solves."""
    A = convdiff(mpg, 12)
    x = mpg.rand_vect(A.nrows, 7)
    exact = oracle.ilu_apply(A, x, "ilu")
    approx = oracle.ilu_apply(A, x, "ilu_jacobi", 60)
    np.testing.assert_allclose(approx, exact, rtol=1e-9, atol=1e-9 * np.abs(exact).max())


@pytest.mark.parametrize("mode", ["mixed", "baseline"])
@pytest.mark.parametrize("prec", ["ilu", "ilu_jacobi"])
def test_oracle_ilu_solve_vs_numpy_restatement(mpg, oracle, mode, prec):
    A = convdiff(mpg, 16)
    xt = mpg.rand_vect(A.nrows, 42)
    b = mpg.host_spmv(A, xt)
    # (one Jacobi sweep per factor stagnates on this convection-dominated
    # problem in both restatements; three converge)
    r = oracle.solve(mpg, A, b, xt, mode=mode, orth="cgs", prec=prec, rlen=12, tol=1e-10, max_restarts=300,
                     jacobi_steps=3)
    q = gmres_np.solve(A, b, mode=mode, orth="cgs", prec=prec, rlen=12, tol=1e-10, max_restarts=300,
                       jacobi_steps=3)
    assert r.status == "converged"
    q["step_cycle"] = np.repeat(np.arange(len(q["cyc_r_norm"])), 12)[: len(q["step_res"])]
    ns = type("R", (), {})()
    for k in ("status", "restarts", "total_iters", "step_res", "step_cycle", "cyc_r_norm", "cyc_normalization", "x"):
        setattr(ns, k, q[k])
    compare(as_ref(r), ns, mode, 1e-10, 12, f"np-vs-oracle {mode}/cgs/{prec}")
    # the preconditioner does its job: fewer restarts than without it
    r0 = oracle.solve(mpg, A, b, xt, mode=mode, orth="cgs", prec="identity", rlen=12, tol=1e-10, max_restarts=300)
    assert r.restarts < r0.restarts


@pytest.mark.parametrize("mode", ["baseline", "mixed"])
def test_parity_rejects_a_wrong_x(mpg, oracle, mode):
    """tests/parity.py's x checks bound the difference by the reference's own
    errNorm, not by the run under test's: a solution moved past that bound
    in one entry of the head, or evenly over the rest (only the sum sees it),
    fails the x check (the old bound, e_ref + e_got, could never fail: a
    moved x's own errNorm grows with the move); the run unmoved passes."""
    A = convdiff(mpg, 16)
    xt = mpg.rand_vect(A.nrows, 42)
    b = mpg.host_spmv(A, xt)
    r = oracle.solve(mpg, A, b, xt, mode=mode, orth="cgs", prec="jacobi", rlen=12, tol=1e-10, max_restarts=300)
    ref = as_ref(r)
    compare(ref, r, mode, 1e-10, 12, "unmoved")
    e_ref = float(r.err_norm)
    assert e_ref > 0
    # past the rounding allowance too (1e-12 / 1e-9 relative to max |x|)
    rt, w, ws = (1e-12, 0.25, 1.0) if mode == "baseline" else (1e-9, 0.5, 2.5)
    scale = float(np.max(np.abs(r.x[:16])))
    delta = 2 * (w * e_ref + rt * scale)
    delta_sum = 1.2 * (ws * e_ref + rt * max(abs(float(np.sum(r.x))), scale) / np.sqrt(A.nrows))
    for where in (0, 16):  # one entry of the checked head; every entry past it, evenly (only the sum sees it)
        bad = type("R", (), {})()
        for k in ("status", "restarts", "total_iters", "step_res", "step_cycle", "cyc_r_norm", "cyc_normalization",
                  "res_norm"):
            setattr(bad, k, getattr(r, k))
        bad.x = np.array(r.x)
        if where == 0:
            bad.x[0] += delta
        else:  # sum moved by sqrt(n) delta_sum, ||move||_2 ~ delta_sum
            bad.x[16:] += np.sqrt(A.nrows) * delta_sum / (A.nrows - 16)
        bad.err_norm = float(np.linalg.norm(bad.x - xt))
        with pytest.raises(AssertionError, match="x head|x sum"):
            compare(ref, bad, mode, 1e-10, 12, f"moved at {where}")


def test_oracle_fp32_summation_modes(mpg, oracle):
    """The oracle's fp32 summation modes (oracle/binding.py LOOP_MODES): on a
    small problem "pair32" and "seq32" reproduce numpy's fp32 arithmetic for
    a dot product (pairwise blocks of 8 / one chain), and the SpMV rounds each
    product to fp32 and adds in CSR order -- the GPU's f32 class
    (internal.hpp mac) -- in both modes."""
    g = np.random.default_rng(3)
    x = g.uniform(-1, 1, 1000).astype(np.float32)
    y = g.uniform(-1, 1, 1000).astype(np.float32)

    def seq(a, b):
        s = np.float32(0)
        for u, v in zip(a, b):
            s = np.float32(s + np.float32(u * v))
        return s

    def pair(a, b):
        if len(a) <= 8:
            return seq(a, b)
        h = len(a) // 2
        return np.float32(pair(a[:h], b[:h]) + pair(a[h:], b[h:]))

    A = mpg.gen_band(400, 5, 4, seed=7)
    xv = g.uniform(-1, 1, A.nrows).astype(np.float32)
    want = np.array([seq(A.val[A.rowptr[i]:A.rowptr[i + 1]].astype(np.float32),
                         xv[A.col[A.rowptr[i]:A.rowptr[i + 1]]]) for i in range(A.nrows)], dtype=np.float32)
    for mode, ref in (("seq32", seq), ("pair32", pair)):
        oracle.lib().oracle_force_loops_mode(oracle.LOOP_MODES[mode])
        try:
            got = oracle.dot(x, y)
            ys = oracle.spmv(A, xv, dtype=np.float32)
        finally:
            oracle.lib().oracle_force_loops_mode(-1)
        assert got == ref(x, y), (mode, got, ref(x, y))
        np.testing.assert_array_equal(ys, want)


def test_fp32_summation_order_sets_cgs_accuracy(mpg, oracle):
    """Why the GPU's fp32 class (accum="f32") is held to MKL plus the pairwise
    fp32 mode (tests/parity.py compare_mkl): within fp32 accumulation the
    ORDER sets how fast plain CGS loses orthogonality. BAND-300k, GMRES(100),
    2 cycles: cycle-1 backward error one sequential fp32 chain > MKL (SIMD
    chains) > pairwise fp32 >= fp64 sums (profiles/r06_accum/order.jsonl:
    1.5e-7, 6.0e-9, 4.5e-10, 2.4e-10)."""
    A = mpg.gen_band(300_000, 5, 4, seed=7)
    xt = mpg.rand_vect(A.nrows, 42)
    b = mpg.host_spmv(A, xt)
    opts = dict(mode="mixed", orth="cgs", prec="jacobi", rlen=100, tol=0.0, max_restarts=2)
    be = {m: oracle.solve(mpg, A, b, xt, backend=m, threads=1 if m == "mkl" else 0, **opts).backward_error[1]
          for m in ("seq32", "mkl", "pair32", "loops")}
    assert be["seq32"] > 5 * be["mkl"] > 25 * be["pair32"], be
    assert be["loops"] <= be["pair32"] <= 3 * be["loops"], be
