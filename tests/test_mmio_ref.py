"""The Matrix Market loader (mpg_load_mtx, LoadMatrix.hpp:17-154 semantics)
against the reference's own parser: /root/reference/mmio.c compiled as-is
into oracle/_ref/libmmio_ref.so (oracle/Makefile), the entry loop through
libc's fscanf with LoadMatrix.hpp:67's format, and the CSR assembly of
LoadMatrix.hpp:82-146 restated in oracle/mmio_ref.py. Banner and size
parsing, the accepted types, the error messages and the assembled CSR
(diagonal slots, symmetric mirroring, duplicates, column order) must all
agree exactly. Skipped where the reference tree is absent (the GPU box)."""
from pathlib import Path

import numpy as np
import pytest

from oracle import mmio_ref

pytestmark = pytest.mark.skipif(not mmio_ref.available(), reason="oracle/_ref/libmmio_ref.so not built")
GOLDEN = Path(__file__).parent / "golden"


def _same(mpg, path):
    M, N, rp, col, val = mmio_ref.load_matrix(str(path))
    A = mpg.load_mtx(str(path))
    assert (A.nrows, A.ncols) == (M, N)
    assert np.array_equal(A.rowptr, rp) and np.array_equal(A.col, col)
    assert np.array_equal(A.val, val)


def test_quirks_fixture_matches_reference_parser(mpg):
    _same(mpg, GOLDEN / "small_quirks.mtx")


def test_c1_standin_matches_reference_parser(mpg, tmp_path):
    from tests.golden.make_c1_standin import write_standin

    p = tmp_path / "c1.mtx"
    write_standin(p)
    _same(mpg, p)


@pytest.mark.parametrize("kind", ["real general", "integer general", "real symmetric"])
def test_random_files_match_reference_parser(mpg, tmp_path, kind):
    """Random coordinate files: unsorted entries, missing diagonals,
    duplicated off-diagonal entries, exponent and sign formats, comments."""
    g = np.random.default_rng(hash(kind) % 1000)
    n = 300
    lines = []
    for _ in range(2500):
        r, c = int(g.integers(1, n + 1)), int(g.integers(1, n + 1))
        if "symmetric" in kind and c > r:
            r, c = c, r
        v = int(g.integers(-9, 10)) if "integer" in kind else float(g.standard_normal() * 10.0 ** g.integers(-8, 8))
        lines.append(f"{r} {c} {v if 'integer' in kind else repr(v)}")
    lines += lines[:40]  # duplicates
    text = f"%%MatrixMarket matrix coordinate {kind}\n% comment line\n%\n{n} {n} {len(lines)}\n" + "\n".join(lines) + "\n"
    p = tmp_path / "r.mtx"
    p.write_text(text)
    _same(mpg, p)


@pytest.mark.parametrize("text", [
    "%%MatrixMarket matrix coordinate complex general\n2 2 1\n1 1 1.0 0.0\n",
    "%%MatrixMarket matrix array real general\n2 2\n1\n2\n3\n4\n",
    "%%MatrixMarket matrix coordinate real hermitian\n2 2 1\n1 1 1.0\n",
    "%%MatrixMarket matrix coordinate pattern general\n2 2 1\n1 1\n",
    "not a banner\n2 2 1\n1 1 1.0\n",
    "%%MatrixMarket matrix coordinate real\n2 2 1\n1 1 1.0\n",
    "%%MatrixMarket matrix coordinate real general\n% no size line\n",
    "%%MatrixMarket vector coordinate real general\n2 2 1\n1 1 1.0\n",
])
def test_rejections_match_reference_parser(mpg, tmp_path, text):
    p = tmp_path / "bad.mtx"
    p.write_text(text)
    with pytest.raises(ValueError) as ref:
        mmio_ref.load_matrix(str(p))
    with pytest.raises(ValueError) as ours:
        mpg.load_mtx(str(p))
    assert str(ours.value) == str(ref.value), (str(ours.value), str(ref.value))


@pytest.mark.parametrize("col", [0, 1])
def test_vector_loader_matches_reference_parser(mpg, tmp_path, col):
    """--bpath's LoadVector (LoadMatrix.hpp:156-233): array and coordinate
    files against the reference's mmio.c readers and fscanf formats."""
    g = np.random.default_rng(col)
    n = 200
    a = g.standard_normal((2, n)) * 10.0 ** g.integers(-6, 6, (2, n))
    pa = tmp_path / "a.mtx"
    pa.write_text("%%MatrixMarket matrix array real general\n% rhs\n" + f"{n} 2\n" +
                  "".join(f"{v!r}\n" for v in a.reshape(-1)))
    rows = g.choice(n, 50, replace=False)
    pc = tmp_path / "c.mtx"
    pc.write_text("%%MatrixMarket matrix coordinate real general\n" + f"{n} 2 100\n" +
                  "".join(f"{r + 1} {c + 1} {g.standard_normal()!r}\n" for c in (0, 1) for r in rows))
    for p in (pa, pc):
        ref = mmio_ref.load_vector(str(p), col)
        assert np.array_equal(mpg.load_mtx_vector(str(p), n, col), ref)
    with pytest.raises(ValueError) as ref_err:
        mmio_ref.load_vector(str(pa), 2)
    with pytest.raises(ValueError) as our_err:
        mpg.load_mtx_vector(str(pa), n, 2)
    assert str(our_err.value) == str(ref_err.value)
