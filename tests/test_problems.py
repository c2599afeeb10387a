"""Host-side problem construction (CPU): generators, Matrix Market loader
semantics (LoadMatrix.hpp:17-154), the seeded vector, host SpMV."""
from pathlib import Path

import numpy as np
import pytest


def test_band_shape_and_dominance(mpg):
    A = mpg.gen_band(100_000, 5, 4, seed=7)
    assert A.nnz == 10 * 100_000 - 25  # BAND-10M at n=1e6 has 9,999,975
    S = A.to_scipy()
    d = S.diagonal()
    off = np.asarray(abs(S).sum(axis=1)).ravel() - d
    assert np.all(d == 1 + off) or np.allclose(d, 1 + off, rtol=1e-15)
    assert np.all(A.val[A.col != np.repeat(np.arange(A.nrows), np.diff(A.rowptr))] < 0)
    # rows sorted, in range
    for i in (0, 1, 50_000, 99_999):
        c = A.col[A.rowptr[i]:A.rowptr[i + 1]]
        assert np.all(np.diff(c) > 0) and c.min() >= 0 and c.max() < A.ncols


def test_band_row_slices_match_whole(mpg):
    A = mpg.gen_band(5000, 5, 4, seed=3)
    parts = [mpg.gen_band(5000, 5, 4, seed=3, row_begin=r0, row_end=r1) for r0, r1 in ((0, 1234), (1234, 5000))]
    assert parts[0].ncols == 5000
    assert np.array_equal(np.concatenate([parts[0].col, parts[1].col]), A.col)
    assert np.array_equal(np.concatenate([parts[0].val, parts[1].val]), A.val)


def test_laplace_counts(mpg):
    A = mpg.gen_laplace3d(10)
    assert A.nrows == 1000 and A.nnz == 7 * 1000 - 6 * 100
    S = A.to_scipy()
    assert (S - S.T).nnz == 0
    assert np.all(S.diagonal() == 6)
    # 100^3 count quoted in SURVEY §8d: 6,940,000
    assert 7 * 100**3 - 6 * 100**2 == 6_940_000


def test_mtx_loader_reference_semantics(mpg):
    A = mpg.load_mtx(str(Path(__file__).parent / "golden" / "small_quirks.mtx"))
    assert A.nrows == 6
    D = A.to_scipy().toarray()
    exp = np.zeros((6, 6))
    ent = [(0, 0, 4), (1, 0, -1), (1, 1, 6), (3, 1, -2), (2, 1, 1), (4, 4, 7), (5, 4, -3), (5, 0, 2), (3, 3, 3),
           (5, 5, 9)]
    for r, c, v in ent:
        exp[r, c] = v
        exp[c, r] = v
    assert np.array_equal(D, exp)
    # every row carries an explicit diagonal slot, even row 3 (index 2) which the file omits
    for i in range(6):
        cols = A.col[A.rowptr[i]:A.rowptr[i + 1]]
        assert i in cols and np.all(np.diff(cols) > 0)
    assert A.nnz == 6 + 2 * 5  # 6 diagonal slots + 5 mirrored off-diagonal pairs


def test_mtx_loader_errors(mpg, tmp_path):
    p = tmp_path / "bad.mtx"
    p.write_text("%%MatrixMarket matrix coordinate complex general\n2 2 1\n1 1 1.0 0.0\n")
    with pytest.raises(ValueError, match="Unsupported matrix type"):
        mpg.load_mtx(str(p))
    with pytest.raises(ValueError, match="Could not access file"):
        mpg.load_mtx(str(tmp_path / "missing.mtx"))
    p.write_text("not a banner\n")
    with pytest.raises(ValueError):
        mpg.load_mtx(str(p))


def test_host_spmv_matches_scipy(mpg):
    A = mpg.gen_band(20_000, 5, 4, seed=1)
    x = mpg.rand_vect(A.nrows, 42)
    assert np.allclose(mpg.host_spmv(A, x), A.to_scipy() @ x, rtol=1e-14, atol=1e-14)


def test_stencil27_counts_symmetry_dominance(mpg):
    """The Queen_4147 stand-in generator (27-point stencil, 3 dof/node)."""
    nx, dof = 7, 3
    A = mpg.gen_stencil27(nx, dof)
    assert A.nrows == nx**3 * dof
    # node-pair couplings: each dimension contributes (3 nx - 2) neighbour pairs per line
    assert A.nnz == (3 * nx - 2) ** 3 * dof * dof
    S = A.to_scipy()
    assert abs(S - S.T).max() == 0
    d = S.diagonal()
    off = np.asarray(abs(S).sum(axis=1)).ravel() - d
    assert np.allclose(d, 1 + off, rtol=1e-15)
    for i in (0, 17, A.nrows - 1):
        c = A.col[A.rowptr[i]:A.rowptr[i + 1]]
        assert np.all(np.diff(c) > 0)
    # Queen_4147 scale: 111^3 x 3 = 4,102,893 rows
    assert 111**3 * 3 == 4_102_893


def test_mtx_vector_loader_reference_semantics(mpg, tmp_path):
    """--bpath's LoadVector (LoadMatrix.hpp:156-233): an array file is read
    column-major (column `col` after skipping col * M values); a coordinate
    file fills the picked column's entries into zeros; a column past N and a
    missing file are errors."""
    p = tmp_path / "b.mtx"
    p.write_text("%%MatrixMarket matrix array real general\n% two right-hand sides\n3 2\n1.5\n-2\n3e-1\n"
                 "10\n20\n30\n")
    assert np.array_equal(mpg.load_mtx_vector(str(p), 3), [1.5, -2.0, 0.3])
    assert np.array_equal(mpg.load_mtx_vector(str(p), 3, col=1), [10.0, 20.0, 30.0])
    with pytest.raises(ValueError, match="Column 2 is too large for the 2 vectors"):
        mpg.load_mtx_vector(str(p), 3, col=2)
    q = tmp_path / "c.mtx"
    q.write_text("%%MatrixMarket matrix coordinate real general\n4 2 3\n2 1 7.25\n4 2 1.0\n4 1 -1\n")
    assert np.array_equal(mpg.load_mtx_vector(str(q), 4), [0.0, 7.25, 0.0, -1.0])
    assert np.array_equal(mpg.load_mtx_vector(str(q), 4, col=1), [0.0, 0.0, 0.0, 1.0])
    with pytest.raises(ValueError, match="Could not access file"):
        mpg.load_mtx_vector(str(tmp_path / "missing.mtx"), 4)
    with pytest.raises(ValueError, match="does not match"):
        mpg.load_mtx_vector(str(q), 5)


def test_mtx_loader_stops_on_a_text_size_line(mpg, tmp_path):
    """A size line with text in it: mmio.c's fscanf loop would spin forever
    (it never consumes a token that matches no %d); the loader reports it."""
    p = tmp_path / "t.mtx"
    p.write_text("%%MatrixMarket matrix coordinate real general\nthree by three\nno numbers here\n")
    with pytest.raises(ValueError, match="Malformed matrix size information"):
        mpg.load_mtx(str(p))


def test_node_block_permutation(mpg):
    """mpg_perm_node_blocks: a permutation; a node's dof stay together and in
    order; each block of `block` consecutive nodes lands on one run of
    consecutive new nodes (mesh-like locality), in a shuffled block order."""
    nodes, dof, block = 1000, 3, 64
    perm = mpg.perm_node_blocks(nodes, dof, block, seed=5)
    assert np.array_equal(np.sort(perm), np.arange(nodes * dof))
    p = perm.reshape(nodes, dof)
    assert np.all(p[:, 0] % dof == 0) and np.all(np.diff(p, axis=1) == 1)
    new_node = p[:, 0] // dof
    for q in range(0, nodes, block):
        run = np.sort(new_node[q:q + block])
        assert np.all(np.diff(run) == 1)
    assert not np.array_equal(new_node, np.arange(nodes))
    assert np.array_equal(perm, mpg.perm_node_blocks(nodes, dof, block, seed=5))


def test_permute_sym_matches_scipy(mpg):
    A = mpg.gen_stencil27(9, 3)
    perm = mpg.perm_node_blocks(A.nrows // 3, 3, 16, seed=7)
    B = mpg.permute_sym(A, perm)
    import scipy.sparse as sp

    P = sp.csr_matrix((np.ones(A.nrows), (perm, np.arange(A.nrows))), shape=(A.nrows, A.nrows))
    ref = (P @ A.to_scipy() @ P.T).tocsr()
    ref.sort_indices()
    Bs = B.to_scipy()
    assert np.array_equal(Bs.indptr, ref.indptr) and np.array_equal(Bs.indices, ref.indices)
    assert np.array_equal(Bs.data, ref.data)
    # same spectrum: the same multiset of values and a symmetric matrix
    assert np.array_equal(np.sort(B.val), np.sort(A.val)) and abs(Bs - Bs.T).max() == 0
    with pytest.raises(ValueError):
        mpg.permute_sym(A, np.zeros(A.nrows, np.int32))


def test_fem27_irregular_rows(mpg):
    """The FEM-like stand-in: symmetric, strictly diagonally dominant, each
    row dof x (1 + kept neighbours) long -- variable lengths -- with the
    explicit diagonal and sorted columns LoadMatrix.hpp guarantees."""
    A = mpg.gen_fem27(14, 3, keep_pct=70, seed=13)
    S = A.to_scipy()
    assert abs(S - S.T).max() == 0
    d = S.diagonal()
    assert np.all(d > abs(S).sum(axis=1).A1 - abs(d))
    rl = np.diff(A.rowptr)
    assert np.all(rl % 3 == 0) and rl.min() >= 3 and rl.max() <= 81 and len(np.unique(rl)) > 10
    assert 30 <= np.median(rl) <= 66
    for i in range(0, A.nrows, 97):
        c = A.col[A.rowptr[i]:A.rowptr[i + 1]]
        assert np.all(np.diff(c) > 0) and i in c
    full = mpg.gen_fem27(6, 2, keep_pct=100, seed=1)
    st = mpg.gen_stencil27(6, 2, seed=1)
    assert np.array_equal(full.rowptr, st.rowptr) and np.array_equal(full.col, st.col)


def test_irregular_specs(mpg):
    A = mpg.gen_spec("stencil27p:10:3:11:8:5")
    ref = mpg.gen_stencil27p(10, 3, seed=11, block=8, perm_seed=5)
    assert np.array_equal(A.col, ref.col) and np.array_equal(A.val, ref.val)
    F = mpg.gen_spec("fem27:8")
    G = mpg.gen_fem27(8, 3, 70, 13)
    assert np.array_equal(F.col, G.col) and np.array_equal(F.val, G.val)
    Fp = mpg.gen_spec("fem27:8:3:70:13:16:5")
    assert Fp.nnz == F.nnz and not np.array_equal(Fp.col, F.col)
