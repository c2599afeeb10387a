"""The measurement hooks bench.py's roofline rests on: the
Arnoldi SpMV's wave stamps inside graph replays of the cycle, the
event-record nodes around it, and eager kernel events. Stamps see the
kernel alone, so they must come out below the two event clocks, which add
the queue's packet latency; a solve after the measurement still matches one
without it."""
import numpy as np
import pytest

# bench.py runs the engine on PyTorch's HIP runtime; loaded at collection,
# before the package library, so the process holds one HIP runtime
torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def band(mpg):
    A = mpg.gen_band(200_000, 5, 4, seed=7)
    xt = mpg.rand_vect(A.nrows, 42)
    return A, xt, mpg.host_spmv(A, xt)


@pytest.mark.parametrize("fmt", ["auto", "csr"])
def test_spmv_stamps_in_graph(mpg, band, fmt):
    torch.cuda.synchronize()
    A, xt, b = band
    eng = mpg.Engine(A, b, xt, mode="mixed", orth="cgs", prec="identity", rlen=30, tol=0.0, max_restarts=20,
                     spmv_format=fmt)
    eng.run(2)
    eng.sync()
    s_ms, s_per = eng.time_phase_stamps("spmv", 2)
    g_ms, g_per = eng.time_phase_graph("spmv", 2)
    e_ms, e_per = eng.time_spmv_incycle(2)
    eng.close()
    assert len(s_per) == len(g_per) == 60 and len(e_per) == 60
    assert np.all(np.asarray(s_per) > 0) and np.all(np.isfinite(s_per))
    assert s_ms < g_ms and s_ms < 1.2 * e_ms, (s_ms, g_ms, e_ms)
    assert s_ms > 0.3 * e_ms, (s_ms, e_ms)


@pytest.mark.parametrize("rlen", [30, 100])
def test_phase_stamps(mpg, band, rlen):
    """The one-panel dots and CGS update store stamps; at m = 100 the sites
    past 32 columns run the panel kernels, which store none and are skipped."""
    A, xt, b = band
    eng = mpg.Engine(A, b, xt, mode="mixed", orth="cgs", prec="identity", rlen=rlen, tol=0.0, max_restarts=20)
    eng.run(1)
    eng.sync()
    out = {}
    for ph in ("dots", "cgs_update"):
        s_ms, s_per = eng.time_phase_stamps(ph, 2)
        g_ms, g_per = eng.time_phase_graph(ph, 2)
        out[ph] = (s_ms, g_ms, len(s_per), len(g_per))
    eng.close()
    for ph, (s_ms, g_ms, ns, ng) in out.items():
        assert ns == 2 * min(rlen, 32) and ng == 2 * rlen, (ph, ns, ng)
        assert 0 < s_ms < g_ms, (ph, s_ms, g_ms)


def test_solve_unchanged_after_measurement(mpg, band):
    A, xt, b = band
    opts = dict(mode="mixed", orth="cgs", prec="jacobi", rlen=30, tol=0.0, max_restarts=3)
    ref = mpg.solve(A, b, xt, engine="fused", **opts)
    eng = mpg.Engine(A, b, xt, **opts)
    eng.time_phase_stamps("spmv", 1)
    eng.close()
    got = mpg.solve(A, b, xt, engine="fused", **opts)
    assert np.array_equal(got.step_res, ref.step_res) and np.array_equal(got.x, ref.x)
