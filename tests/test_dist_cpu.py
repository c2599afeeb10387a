"""Row-partitioned (multi-GPU) path on CPU: world_size-2 `gloo` ranks build
their halo plans with the C-ABI partitioner (include/mpgmres/dist.h, no GPU
needed), exchange their needs, then

  * a distributed SpMV with the halo exchange done over gloo must equal the
    rows of the global SpMV exactly (same per-row summation order), and
  * one distributed CGS Arnoldi cycle (partial dots + all-reduce, as the
    fused engine does with RCCL) must reproduce the Hessenberg matrix of the
    serial cycle to fp64 round-off.

The halo exchange and the all-reduces go through the product's host
transport (mpgmres_amd/transport.py), called through the C function
pointers exactly as host/dist.cpp's HostComm calls them; the GPU side of the
same engine over this transport is tests/test_dist_gpu.py's multi-process
test.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _exchange(plan, rank, world):
    needs = {q: plan.recv_rows(q).tolist() for q in range(world) if q != rank}
    got = [None] * world
    dist.all_gather_object(got, needs)
    sends = {}
    for q in range(world):
        if q != rank:
            rows = got[q].get(rank, [])
            plan.set_send(q, rows)
            sends[q] = np.asarray(rows, dtype=np.int64)
    return sends


def _halo(x_ext, n_loc, r0, plan, sends, rank, world, transport):
    """The halo exchange through the product's host transport
    (mpgmres_amd/transport.py), called through its C function pointer with
    the arguments host/dist.cpp's HostComm passes: per-peer send/recv
    buffers and byte counts."""
    import ctypes as C

    f = plan.n_front
    send_arrs = {q: np.ascontiguousarray(x_ext[f + sends[q] - r0]) for q in range(world) if q != rank and len(sends[q])}
    sizes = {q: 8 * len(plan.recv_rows(q)) for q in range(world) if q != rank}
    recv_arrs = {q: np.zeros(sizes[q] // 8) for q in sizes if sizes[q]}
    send = (C.c_void_p * world)(*[send_arrs[q].ctypes.data if q in send_arrs else None for q in range(world)])
    sb = (C.c_int64 * world)(*[send_arrs[q].nbytes if q in send_arrs else 0 for q in range(world)])
    recv = (C.c_void_p * world)(*[recv_arrs[q].ctypes.data if q in recv_arrs else None for q in range(world)])
    rb = (C.c_int64 * world)(*[sizes.get(q, 0) for q in range(world)])
    assert transport.c.exchange(None, send, sb, recv, rb) == 0, transport.error
    for q in range(world):
        if q != rank and sizes[q]:
            o = plan.n_front + plan.recv_pos(q)  # x_ext holds the front halo first
            x_ext[o:o + sizes[q] // 8] = recv_arrs[q]


def _allreduce(v, transport):
    """fp64 sum through the host transport's C callback (rank-order sum)."""
    import ctypes as C

    buf = np.array(v, dtype=np.float64)
    assert transport.c.allreduce(None, buf.ctypes.data_as(C.POINTER(C.c_double)), len(buf), 0) == 0, transport.error
    return buf


def _worker(rank, world, port, N, out_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from tests.conftest import load_package

        mpg = load_package()
        from mpgmres_amd.transport import HostTransport

        transport = HostTransport()
        A = mpg.gen_band(N, 5, 4, seed=3)
        starts = mpg.nnz_balanced_starts(A, world)
        r0, r1 = int(starts[rank]), int(starts[rank + 1])
        A_loc = mpg.row_slice(A, r0, r1)
        # the generator's row slice equals the slice of the whole matrix
        B = mpg.gen_band(N, 5, 4, seed=3, row_begin=r0, row_end=r1)
        assert np.array_equal(B.col, A_loc.col) and np.array_equal(B.val, A_loc.val)
        plan = mpg.HaloPlan(rank, world, starts, A_loc)
        sends = _exchange(plan, rank, world)
        # local numbering: lower ranks' halo at [-f, 0), own rows, higher
        # ranks' halo at [n_loc, n_ext); x_ext stores it from -f
        n_loc, n_ext, f = r1 - r0, plan.n_ext, plan.n_front
        assert (f > 0) == (rank > 0)
        cols = plan.local_cols() + f
        import scipy.sparse as sp

        S = sp.csr_matrix((A_loc.val, cols, A_loc.rowptr), shape=(n_loc, f + n_ext))
        S.has_sorted_indices = True  # keep the file's per-row order (= global order)
        x = mpg.rand_vect(N, 42)
        x_ext = np.zeros(f + n_ext)
        x_ext[f:f + n_loc] = x[r0:r1]
        _halo(x_ext, n_loc, r0, plan, sends, rank, world, transport)
        y = np.array([np.sum(A_loc.val[A_loc.rowptr[i]:A_loc.rowptr[i + 1]]
                             * x_ext[cols[A_loc.rowptr[i]:A_loc.rowptr[i + 1]]]) for i in range(n_loc)])
        full = mpg.host_spmv(A, x)[r0:r1]
        spmv_ok = bool(np.allclose(y, full, rtol=1e-15, atol=1e-15))

        # one CGS Arnoldi cycle, distributed like the fused engine
        m = 8
        V = np.zeros((n_loc, m + 1))
        H = np.zeros((m + 1, m))
        b = mpg.host_spmv(A, x)[r0:r1]
        beta = np.sqrt(_allreduce([b @ b], transport)[0])
        V[:, 0] = b / beta
        for k in range(m):
            v_ext = np.zeros(f + n_ext)
            v_ext[f:f + n_loc] = V[:, k]
            _halo(v_ext, n_loc, r0, plan, sends, rank, world, transport)
            w = S @ v_ext
            h = _allreduce(V[:, :k + 1].T @ w, transport)
            w = w - V[:, :k + 1] @ h
            H[:k + 1, k] = h
            H[k + 1, k] = np.sqrt(_allreduce([w @ w], transport)[0])
            V[:, k + 1] = w / H[k + 1, k]
        # max reduction and rank-order sums: the same bits on every rank
        import ctypes as C

        buf = np.array([float(rank), -float(rank), 1.0 / 3.0 * (rank + 1)])
        assert transport.c.allreduce(None, buf.ctypes.data_as(C.POINTER(C.c_double)), 3, 1) == 0
        mx = buf.copy()
        out_q.put((rank, spmv_ok, (H, mx)))
    except Exception as e:  # surface the failure in the parent
        out_q.put((rank, repr(e), None))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_partitioned_spmv_and_arnoldi_gloo(mpg, world):
    N = 3001
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, N, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    res.sort(key=lambda t: t[0])
    for rank, ok, H in res:
        assert ok is True, f"rank {rank}: {ok}"
    # serial reference cycle
    A = mpg.gen_band(N, 5, 4, seed=3)
    S = A.to_scipy()
    x = mpg.rand_vect(N, 42)
    b = S @ x
    m = 8
    V = np.zeros((N, m + 1))
    H = np.zeros((m + 1, m))
    V[:, 0] = b / np.linalg.norm(b)
    for k in range(m):
        w = S @ V[:, k]
        h = V[:, :k + 1].T @ w
        w = w - V[:, :k + 1] @ h
        H[:k + 1, k] = h
        H[k + 1, k] = np.linalg.norm(w)
        V[:, k + 1] = w / H[k + 1, k]
    for _, _, (Hd, mx) in res:
        assert np.allclose(Hd, H, rtol=1e-12, atol=1e-12)
        assert np.array_equal(mx, [world - 1.0, 0.0, world / 3.0])
    assert np.array_equal(res[0][2][0], res[1][2][0])  # every rank holds the same H


def test_halo_plan_single_process(mpg):
    """Plan bookkeeping: halo entries grouped by owner, local ids, send checks."""
    A = mpg.gen_band(1000, 5, 4, seed=1)
    starts = np.array([0, 300, 700, 1000])
    plans = [mpg.HaloPlan(r, 3, starts, mpg.row_slice(A, starts[r], starts[r + 1])) for r in range(3)]
    # middle rank needs 5 rows below and 4 above its block: the lower ones
    # get local ids -5..-1 (in front of its rows), the upper ones 400..403
    assert list(plans[1].recv_rows(0)) == list(range(295, 300))
    assert list(plans[1].recv_rows(2)) == list(range(700, 704))
    assert plans[1].n_front == 5 and plans[1].n_ext == 400 + 4
    assert plans[1].recv_pos(0) == -5 and plans[1].recv_pos(2) == 400
    assert plans[0].n_front == 0 and plans[0].recv_pos(1) == 300
    cols = plans[1].local_cols()
    assert cols.min() == -5 and cols.max() == 403
    # global column c of the block's rows maps to c - 300 for every c: banded
    # rows keep their offsets, so slices stay within int16 and the LDS window
    A1 = mpg.row_slice(A, 300, 700)
    assert np.array_equal(cols, A1.col - 300)
    with pytest.raises(ValueError):
        plans[1].set_send(0, [10])  # row 10 is not owned by rank 1


def test_node_dof_and_node_aligned_starts(mpg):
    """mpg_csr_node_dof: 3 on the 3-dof generators (27-point stencil, thinned
    FEM coupling, node-block permutation), 1 on a band, a 7-point Laplacian
    and fem27 under a row permutation that splits nodes; the nnz-balanced
    split then starts every rank on a node boundary."""
    A = mpg.gen_stencil27(20, 3)
    F = mpg.gen_fem27(10, 3, keep_pct=70, seed=13)
    Fp = mpg.gen_spec("fem27:10:3:70:13:32:5")
    split = mpg.permute_sym(F, np.random.default_rng(3).permutation(F.nrows).astype(np.int32))
    assert [mpg.node_dof(M) for M in (A, F, Fp)] == [3, 3, 3]
    assert [mpg.node_dof(M) for M in (mpg.gen_band(3000, 5, 4, seed=7), mpg.gen_laplace3d(9), split)] == [1, 1, 1]
    for M in (A, F, Fp):
        for P in (2, 3, 5, 8):
            st = mpg.nnz_balanced_starts(M, P)
            assert st[0] == 0 and st[-1] == M.nrows and np.all(np.diff(st) >= 0) and np.all(st % 3 == 0), (P, st)
            # still about nnz-balanced (within one node's rows of the target)
            for q in range(1, P):
                assert abs(int(M.rowptr[st[q]]) - M.nnz * q // P) <= 6 * 81, (q, st)
    B = mpg.gen_band(4000, 5, 4, seed=7)  # no nodes: the plain nnz split
    st = mpg.nnz_balanced_starts(B, 3)
    want = [0] + [int(np.searchsorted(B.rowptr, B.nnz * q // 3, side="left")) for q in (1, 2)] + [4000]
    assert np.array_equal(st, want) and any(v % 3 for v in want), (st, want)
