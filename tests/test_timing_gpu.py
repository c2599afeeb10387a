"""The measurement hooks bench.py's roofline rests on: what
one launch adds to a graph replay of the cycle (duplicate launches, HIP
events around whole replays), the dots' and CGS update's wave stamps, the
event-record nodes around a launch, and eager kernel events. These tests
assert structure only (launch counts, positive times, which kernels carry
stamps): the orderings between the clocks depend on dispatch overhead and
GPU sharing, so they are printed for the record, not asserted.
A measured engine refuses to continue its solve, and a solve after the
measurement still matches one without it."""
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
def test_spmv_dup_in_graph(mpg, band, fmt):
    """What one SpMV launch adds to a graph replay (kernel + dispatch) lies
    below the event-node clock (two marker packets per launch) and near the
    eager kernel events."""
    torch.cuda.synchronize()
    A, xt, b = band
    eng = mpg.Engine(A, b, xt, mode="mixed", orth="cgs", prec="identity", rlen=30, tol=0.0, max_restarts=20,
                     spmv_format=fmt)
    eng.run(2)
    eng.sync()
    d_ms, added = eng.time_phase_dup("spmv", 5)
    g_ms, g_per = eng.time_phase_graph("spmv", 2)
    e_ms, e_per = eng.time_spmv_incycle(2)
    with pytest.raises(RuntimeError):  # the SpMVs carry no stamp code
        eng.time_phase_stamps("spmv", 1)
    eng.close()
    assert added == 30 and len(g_per) == 60 and len(e_per) == 60
    assert d_ms > 0 and g_ms > 0 and e_ms > 0
    print(f"spmv {fmt}: dup {d_ms * 1e3:.2f} us, event nodes {g_ms * 1e3:.2f} us, eager events {e_ms * 1e3:.2f} us")


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
        d_ms, added = eng.time_phase_dup(ph, 3)
        out[ph] = (s_ms, g_ms, d_ms, len(s_per), len(g_per), added)
    eng.close()
    for ph, (s_ms, g_ms, d_ms, ns, ng, added) in out.items():
        assert ns == 2 * min(rlen, 32) and ng == 2 * rlen and added == rlen, (ph, ns, ng, added)
        assert s_ms > 0 and g_ms > 0, (ph, s_ms, g_ms)
        print(f"{ph} m={rlen}: stamps {s_ms * 1e3:.2f} us, dup {d_ms * 1e3:.2f} us, event nodes {g_ms * 1e3:.2f} us")


def test_solve_unchanged_after_measurement(mpg, band):
    A, xt, b = band
    opts = dict(mode="mixed", orth="cgs", prec="jacobi", rlen=30, tol=0.0, max_restarts=3)
    ref = mpg.solve(A, b, xt, engine="fused", **opts)
    eng = mpg.Engine(A, b, xt, **opts)
    eng.run(1)
    eng.time_phase_dup("spmv", 2)
    eng.time_phase_dup("cgs_update", 2)
    # the duplicated launches changed V, H and w: the engine will not go on
    with pytest.raises(RuntimeError, match="measurement launches"):
        eng.run(1)
    eng.close()
    got = mpg.solve(A, b, xt, engine="fused", **opts)
    assert np.array_equal(got.step_res, ref.step_res) and np.array_equal(got.x, ref.x)
