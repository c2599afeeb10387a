"""Irregular matrices (VERDICT r3 missing #2). Queen_4147 and bcsstk17 are
unstructured FEM matrices; every other GPU test input is a stencil or band,
where the SELL copy's implicit slices and shared / int16 column blocks
apply. Two stand-ins take the general path:
  * stencil27p: the C4 stencil (27-point, 3 dof) under a symmetric node-block
    permutation (mpg_perm_node_blocks: blocks of 64 nodes in random order,
    shuffled inside) -- the same spectrum, neighbours scattered over the
    whole matrix, so no slice has a common column pattern or a 16-bit span;
  * fem27: the 27-point coupling randomly thinned (each node pair kept with
    probability 70 %): rows of variable length, in natural and in permuted
    order.
Each solve is compared with the live oracle (kernels_mkl.cpp's path,
kernels_mkl.cpp:326-352 for the SpMV: MKL pinned to one code branch at fixed
thread counts, two-sided, tests/parity.py compare_mkl) on both engines, and
each asserts which Arnoldi SpMV form it ran (int32 SELL, CSR-adaptive row
blocks or node blocks: one record of a 3 x 3 block per column triple,
node_tile.hpp)."""
import os

import numpy as np
import pytest

from tests.parity import compare_mkl

pytestmark = pytest.mark.gpu


def _problem(mpg, which):
    if which == "stencil27p":  # C4's plane structure at 105 x 105 x 8 nodes, permuted
        A = mpg.gen_stencil27p(105, 3, ny=105, nz=8, block=64, perm_seed=5)
    elif which == "fem27":
        A = mpg.gen_fem27(30, 3, keep_pct=70, seed=13)
    else:
        A = mpg.gen_spec("fem27:30:3:70:13:32:5")
    xt = mpg.rand_vect(A.nrows, 42)
    return A, xt, mpg.host_spmv(A, xt)


@pytest.fixture(scope="module")
def problems(mpg):
    return {w: _problem(mpg, w) for w in ("stencil27p", "fem27", "fem27p")}


def _fmt(fmt, monkeypatch):
    """"sell-sigma": the SELL copy in SELL-C-sigma order (MPG_SELL_SIGMA=-1:
    rows sorted by length in windows of 1024; off by default, sell.hip)."""
    if fmt == "sell-sigma":
        monkeypatch.setenv("MPG_SELL_SIGMA", "-1")
        return "sell"
    monkeypatch.delenv("MPG_SELL_SIGMA", raising=False)
    return fmt


@pytest.mark.parametrize("fmt", ["auto", "sell", "csr", "sell-sigma"])
@pytest.mark.parametrize("which", ["stencil27p", "fem27", "fem27p"])
def test_irregular_layout(mpg, problems, which, fmt, monkeypatch):
    """What each storage choice runs: the permuted matrices never get 16-bit
    or implicit columns; auto keeps SELL only when padding adds <= 20 %, and
    takes the node-block copy (3-dof nodes, 3 x 3 blocks) whenever it is the
    smallest -- on all three stand-ins."""
    A, xt, b = problems[which]
    eng = mpg.Engine(A, b, xt, mode="mixed", orth="cgs", prec="jacobi", rlen=30, tol=0.0, max_restarts=2,
                     spmv_format=_fmt(fmt, monkeypatch))
    lay, cols = eng.spmv_layout(), eng.sell_columns()
    eng.close()
    assert (cols["sigma"] > 0) == (fmt == "sell-sigma"), (fmt, cols)
    if fmt == "sell-sigma":
        assert lay["format"] == "sell" and cols["form"] == "int32" and cols["implicit_slices"] == 0, cols
        return
    if fmt == "csr":
        assert lay["format"] == "csr" and cols["form"] == "none", (lay, cols)
        return
    if fmt == "auto":
        assert lay["format"] == "node" and lay["stored"] == A.nnz and cols["form"] == "none", (lay, cols)
        return
    if fmt == "sell":
        assert lay["format"] == "sell", lay
    if lay["format"] == "sell":
        if which != "fem27":
            assert cols["form"] == "int32" and cols["implicit_slices"] == 0, cols
        pad = lay["stored"] / A.nnz - 1.0
        assert fmt == "sell" or pad <= 0.20, (pad, lay)
    else:
        assert fmt == "auto" and cols["form"] == "none"


@pytest.mark.parametrize("engine,fmt", [("fused", "auto"), ("fused", "sell"), ("fused", "csr"), ("fused", "sell-sigma"),
                                        ("fused", "node"), ("surface", "auto"), ("surface", "sell-sigma")])
@pytest.mark.parametrize("mode,orth", [("mixed", "cgs"), ("baseline", "mgs"), ("mixed", "cgsr")])
@pytest.mark.parametrize("which", ["stencil27p", "fem27", "fem27p"])
def test_irregular_live_oracle(mpg, oracle, problems, which, mode, orth, engine, fmt, monkeypatch):
    A, xt, b = problems[which]
    opts = dict(mode=mode, orth=orth, prec="jacobi", rlen=30, tol=1e-10, max_restarts=200)
    got = mpg.solve(A, b, xt, engine=engine, spmv_format=_fmt(fmt, monkeypatch), **opts)
    label = f"{which}-{mode}-{orth}/{engine}-{fmt}"
    # the oracle runs once per (matrix, mode, orth), shared by every engine and storage
    runs = compare_mkl(oracle, mpg, A, b, xt, got, opts, label, runs=_ORACLE.setdefault((which, mode, orth), {}))
    assert runs[1].status == "converged"


_ORACLE = {}


@pytest.mark.parametrize("which", ["stencil27p", "fem27p"])
def test_irregular_spmv_forms_same_bits(mpg, problems, which):
    """The int32 SELL SpMV and the CSR row-block SpMV sum every row in CSR
    order in fp64: one Arnoldi cycle gives the same |s(k+1)| history to fp32
    rounding of the (differently ordered) fp64 residual prologue."""
    A, xt, b = problems[which]
    opts = dict(mode="mixed", orth="cgs", prec="identity", rlen=30, tol=0.0, max_restarts=1)
    s = mpg.solve(A, b, xt, engine="fused", spmv_format="sell", **opts)
    c = mpg.solve(A, b, xt, engine="fused", spmv_format="csr", **opts)
    np.testing.assert_allclose(s.step_res, c.step_res, rtol=1e-4)


@pytest.mark.parametrize("mode", ["1", "2", "3"])
@pytest.mark.parametrize("which", ["fem27", "fem27p"])
def test_csr_stream_modes_same_bits(mpg, which, mode, monkeypatch):
    """The Arnoldi CSR SpMV's stream options (MPG_CSR_MODE: bit 0
    non-temporal matrix loads, bit 1 row blocks in XCD order) load the same
    data into the same workgroup tiles: the same bits as the default."""
    A = mpg.gen_spec("fem27:44:3:70:13" if which == "fem27" else "fem27:44:3:70:13:64:5")
    xt = mpg.rand_vect(A.nrows, 42)
    b = mpg.host_spmv(A, xt)
    opts = dict(engine="fused", mode="mixed", orth="cgs", prec="jacobi", rlen=30, tol=0.0, max_restarts=2,
                spmv_format="csr")
    monkeypatch.setenv("MPG_CSR_MODE", "0")
    ref = mpg.solve(A, b, xt, **opts)
    monkeypatch.setenv("MPG_CSR_MODE", mode)
    got = mpg.solve(A, b, xt, **opts)
    assert np.array_equal(got.step_res, ref.step_res) and np.array_equal(got.x, ref.x)
    assert got.res_norm == ref.res_norm


def _node_problem(mpg, which):
    if which == "stencil27":  # C4's own structure (3 dof per node), small
        A = mpg.gen_stencil27(40, 3)
    elif which == "stencil27p":
        A = mpg.gen_stencil27p(48, 3, ny=48, nz=6, block=64, perm_seed=5)
    elif which == "fem27":
        A = mpg.gen_fem27(30, 3, keep_pct=70, seed=13)
    else:
        A = mpg.gen_spec("fem27:30:3:70:13:32:5")
    xt = mpg.rand_vect(A.nrows, 42)
    return A, xt, mpg.host_spmv(A, xt)


@pytest.mark.parametrize("mode,orth,prec", [("mixed", "cgs", "jacobi"), ("mixed", "cgsr", "identity"),
                                            ("baseline", "mgs", "jacobi"), ("single", "cgs", "jacobi"),
                                            ("mixed-half", "cgs", "jacobi")])
@pytest.mark.parametrize("which", ["stencil27", "stencil27p", "fem27", "fem27p"])
def test_node_blocks_same_bits_as_csr(mpg, which, mode, orth, prec):
    """The node-block SpMV (one record per 3 x 3 block: the block's first
    column and 9 values) forms the CSR tile's fp64 products and sums each row
    in CSR storage order: whole solves on either copy agree to the last bit,
    in every value type (fp32, fp64, scaled fp16 records)."""
    A, xt, b = _node_problem(mpg, which)
    opts = dict(engine="fused", mode=mode, orth=orth, prec=prec, rlen=30, tol=0.0, max_restarts=3)
    eng = mpg.Engine(A, b, xt, **{k: v for k, v in opts.items() if k != "engine"}, spmv_format="node")
    lay = eng.spmv_layout()
    eng.close()
    assert lay["format"] == "node" and lay["stored"] == A.nnz and lay["vec_width"] == 9, lay
    ref = mpg.solve(A, b, xt, spmv_format="csr", **opts)
    got = mpg.solve(A, b, xt, spmv_format="node", **opts)
    assert got.total_iters == ref.total_iters == 90
    assert np.array_equal(got.step_res, ref.step_res) and np.array_equal(got.x, ref.x)
    assert got.res_norm == ref.res_norm


@pytest.mark.parametrize("mode", ["mixed", "baseline", "mixed-half"])
@pytest.mark.parametrize("which", ["stencil27", "fem27p"])
def test_node_prologue_same_bits(mpg, monkeypatch, which, mode):
    """The residual prologue on node blocks (round 6; k_node_rowsums +
    k_prologue_rows: the node copy's fp64 row sums, then the CSR prologue's
    epilogue and norm partials with its own grid and lane-to-row map) gives
    the CSR prologue's bits: whole solves with it and with MPG_NODE_PROLOGUE=0
    agree to the last bit, and the layout reports which one ran."""
    A, xt, b = _node_problem(mpg, which)
    opts = dict(mode=mode, orth="cgs", prec="jacobi", rlen=30, tol=0.0, max_restarts=3, spmv_format="node")
    got = {}
    for env in ("1", "0"):
        monkeypatch.setenv("MPG_NODE_PROLOGUE", env)
        eng = mpg.Engine(A, b, xt, **opts)
        lay = eng.spmv_layout()
        eng.close()
        assert lay["format"] == "node" and lay["prologue"] == ("node" if env == "1" else "csr"), lay
        got[env] = mpg.solve(A, b, xt, engine="fused", **opts)
    assert got["1"].total_iters == got["0"].total_iters == 90
    assert np.array_equal(got["1"].step_res, got["0"].step_res) and np.array_equal(got["1"].x, got["0"].x)
    assert got["1"].res_norm == got["0"].res_norm


def test_node_blocks_refused(mpg, monkeypatch):
    """spmv_format="node" fails loudly where no node copy can be built (rows
    not a multiple of 3; exact blocks only, MPG_NODE_PAD=0, on a band and on
    fem27 under a row permutation that splits nodes), and auto never picks it
    on those two (the padded copy would stream more bytes)."""
    band = mpg.gen_band(30_000, 5, 4, seed=7)
    A = mpg.gen_fem27(12, 3, keep_pct=70, seed=13)
    rng = np.random.default_rng(3)
    split = mpg.permute_sym(A, rng.permutation(A.nrows).astype(np.int32))
    odd = mpg.gen_band(30_001, 5, 4, seed=7)
    opts = dict(mode="mixed", orth="cgs", prec="jacobi", rlen=30, tol=0.0, max_restarts=1)
    for M, pad in ((odd, None), (band, "0"), (split, "0")):
        if pad:
            monkeypatch.setenv("MPG_NODE_PAD", pad)
        else:
            monkeypatch.delenv("MPG_NODE_PAD", raising=False)
        xt = mpg.rand_vect(M.nrows, 42)
        b = mpg.host_spmv(M, xt)
        with pytest.raises((RuntimeError, ValueError)):
            mpg.Engine(M, b, xt, spmv_format="node", **opts).close()
    monkeypatch.delenv("MPG_NODE_PAD", raising=False)
    for M in (band, split):
        xt = mpg.rand_vect(M.nrows, 42)
        b = mpg.host_spmv(M, xt)
        eng = mpg.Engine(M, b, xt, **opts)
        assert eng.spmv_layout()["format"] != "node"
        eng.close()


@pytest.mark.parametrize("tpw", ["2", "4", "8", "0"])
@pytest.mark.parametrize("which", ["stencil27", "fem27p"])
def test_node_tile_walk_same_bits(mpg, which, tpw, monkeypatch):
    """MPG_NODE_TPW: each workgroup walks 2 / 4 / 8 (0: auto) consecutive tiles with the
    next tile's records in flight (node_tiles) -- the same tiles, products
    and row order as one tile per workgroup: the same bits."""
    A, xt, b = _node_problem(mpg, which)
    opts = dict(engine="fused", mode="mixed", orth="cgs", prec="jacobi", rlen=30, tol=0.0, max_restarts=3,
                spmv_format="node")
    monkeypatch.setenv("MPG_NODE_TPW", "1")
    ref = mpg.solve(A, b, xt, **opts)
    monkeypatch.setenv("MPG_NODE_TPW", tpw)
    got = mpg.solve(A, b, xt, **opts)
    assert np.array_equal(got.step_res, ref.step_res) and np.array_equal(got.x, ref.x)


@pytest.mark.parametrize("mode,orth", [("mixed", "cgs"), ("baseline", "mgs"), ("single", "cgsr")])
@pytest.mark.parametrize("which", ["stencil27p", "fem27", "fem27p"])
def test_surface_node_blocks_same_bits(mpg, which, mode, orth, monkeypatch):
    """The operator surface (kernels_hip.cpp spmv, the reference's
    kernels.hpp boundary) runs A's SpMV on the node-block copy when it
    streams fewer bytes than the SELL copy or the CSR arrays: whole solves
    give the bits of the same surface on CSR (MPG_SURFACE_NODE=0 and
    MPG_SURFACE_SELL=0; the SELL kernels fuse the fp64 multiply-add, so an
    fp64 matrix's SELL sums differ in the last bits), and the counts show
    which storage each ran on. (The natural-order stencil at this size keeps
    its SELL copy: 16-bit columns and implicit slices stream fewer bytes.)"""
    A, xt, b = _node_problem(mpg, which)
    opts = dict(engine="surface", mode=mode, orth=orth, prec="jacobi", rlen=30, tol=0.0, max_restarts=3)
    got = {}
    for env in ("", "0"):
        if env:
            monkeypatch.setenv("MPG_SURFACE_NODE", env)
            monkeypatch.setenv("MPG_SURFACE_SELL", env)
        else:
            monkeypatch.delenv("MPG_SURFACE_NODE", raising=False)
            monkeypatch.delenv("MPG_SURFACE_SELL", raising=False)
        before = mpg.surface_spmv_counts()
        got[env] = mpg.solve(A, b, xt, **opts)
        after = mpg.surface_spmv_counts()
        d = {k: after[k] - before[k] for k in after}
        if env:
            assert d["node"] == 0 and d["sell"] == 0 and d["csr"] > 0, d
        else:
            assert d["node"] > 0 and d["sell"] == 0, d
    ref, g = got["0"], got[""]
    assert g.total_iters == ref.total_iters == 90
    assert np.array_equal(g.step_res, ref.step_res) and np.array_equal(g.x, ref.x) and g.res_norm == ref.res_norm


@pytest.mark.parametrize("which", ["stencil27", "fem27p"])
def test_node_xcd_order_same_bits(mpg, which, monkeypatch):
    """MPG_NODE_XCD: the node SpMV's workgroups take their tiles in XCD order
    (auto on for scattered columns: fem27p) or in launch order -- the same
    tiles and sums, the same bits."""
    A, xt, b = _node_problem(mpg, which)
    opts = dict(engine="fused", mode="mixed", orth="cgs", prec="jacobi", rlen=30, tol=0.0, max_restarts=3,
                spmv_format="node")
    got = {}
    for v in ("0", "1"):
        monkeypatch.setenv("MPG_NODE_XCD", v)
        got[v] = mpg.solve(A, b, xt, **opts)
    assert np.array_equal(got["0"].step_res, got["1"].step_res) and np.array_equal(got["0"].x, got["1"].x)


def _constrained(mpg, A, every=7, drop=0.01, seed=3):
    """A with a constrained dof on every `every`-th node (row 3r + 1 replaced
    by its diagonal entry alone, as a Dirichlet condition leaves it) and a
    fraction `drop` of the other off-diagonal entries removed: node rows whose
    three rows no longer share one pattern."""
    g = np.random.default_rng(seed)
    rows, cols, vals = [], [], []
    for i in range(A.nrows):
        a, z = int(A.rowptr[i]), int(A.rowptr[i + 1])
        c, v = A.col[a:z], A.val[a:z]
        if (i // 3) % every == 0 and i % 3 == 1:
            keep = c == i
        else:
            keep = (c == i) | (g.random(z - a) >= drop)
        rows.append(np.full(int(keep.sum()), i)), cols.append(c[keep]), vals.append(v[keep])
    r, c, v = np.concatenate(rows), np.concatenate(cols), np.concatenate(vals)
    rp = np.zeros(A.nrows + 1, dtype=np.int32)
    np.add.at(rp, r + 1, 1)
    return mpg.Csr(A.nrows, A.ncols, np.cumsum(rp).astype(np.int32), c.astype(np.int32), v.astype(np.float64))


@pytest.mark.parametrize("mode,orth", [("mixed", "cgs"), ("baseline", "mgs"), ("mixed-half", "cgs")])
def test_node_padded_blocks_same_bits(mpg, mode, orth):
    """Padded node blocks (mpg_node_layout): node rows whose three rows do not
    share a pattern store the union of their node columns with zeros for the
    missing entries; each row still meets its entries in CSR order and the
    zero products leave its fp64 sum unchanged, so solves give the CSR bits.
    The exact-pattern check refuses this matrix (MPG_NODE_PAD=0)."""
    A = _constrained(mpg, mpg.gen_fem27(24, 3, keep_pct=70, seed=13))
    assert mpg.node_dof(A) == 1
    xt = mpg.rand_vect(A.nrows, 42)
    b = mpg.host_spmv(A, xt)
    opts = dict(engine="fused", mode=mode, orth=orth, prec="jacobi", rlen=30, tol=0.0, max_restarts=3)
    eng = mpg.Engine(A, b, xt, **{k: v for k, v in opts.items() if k != "engine"}, spmv_format="node")
    lay = eng.spmv_layout()
    eng.close()
    assert lay["format"] == "node" and A.nnz < lay["stored"] < 1.1 * A.nnz, lay
    ref = mpg.solve(A, b, xt, spmv_format="csr", **opts)
    got = mpg.solve(A, b, xt, spmv_format="node", **opts)
    assert got.total_iters == ref.total_iters == 90
    assert np.array_equal(got.step_res, ref.step_res) and np.array_equal(got.x, ref.x)
    os.environ["MPG_NODE_PAD"] = "0"
    try:
        with pytest.raises((RuntimeError, ValueError)):
            mpg.Engine(A, b, xt, **{k: v for k, v in opts.items() if k != "engine"}, spmv_format="node").close()
    finally:
        os.environ.pop("MPG_NODE_PAD", None)
