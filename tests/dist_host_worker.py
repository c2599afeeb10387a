"""One rank of a row-partitioned solve with the product's distributed
engine over the host transport (mpg_engine_create_dist_host + transport.py),
launched by tests/test_dist_gpu.py as

  python -m torch.distributed.run --nproc-per-node P --master-addr 127.0.0.1 \
      --master-port PORT tests/dist_host_worker.py OUT.npz MATRIX MODE ORTH PREC MAX_RESTARTS TOL [FORMAT]

MATRIX: N (BAND-N, gen_band(N, 5, 4, seed=7)) or stencil27:NX:NY:NZ (3 dof).
FORMAT: the Arnoldi SpMV storage (spmv_format; default auto).
Every rank uses device 0 (the ranks share the GPU; RCCL would refuse).
Rank 0 writes the gathered solution, its history and every rank's SpMV
layout (column form, CSR-summed slices, front halo) to OUT.npz.
"""
import os
import sys
from pathlib import Path

import numpy as np
import torch.distributed as dist

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO))


def matrix(mpg, spec: str):
    if spec.startswith("stencil27:"):
        nx, ny, nz = (int(v) for v in spec.split(":")[1:4])
        return mpg.gen_stencil27(nx, 3, ny=ny, nz=nz)
    return mpg.gen_band(int(spec), 5, 4, seed=7)


def main():
    out, spec, mode, orth, prec, max_restarts, tol = sys.argv[1:8]
    fmt = sys.argv[8] if len(sys.argv) > 8 else "auto"
    from __graft_entry__ import _load

    mpg = _load()
    from mpgmres_amd.transport import HostTransport

    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    A = matrix(mpg, spec)
    xt = mpg.rand_vect(A.nrows, 42)
    b = mpg.host_spmv(A, xt)
    starts = mpg.nnz_balanced_starts(A, world)
    r0, r1 = int(starts[rank]), int(starts[rank + 1])
    A_loc = mpg.row_slice(A, r0, r1)
    plan = mpg.HaloPlan(rank, world, starts, A_loc)
    needs = {q: plan.recv_rows(q).tolist() for q in range(world) if q != rank}
    got = [None] * world
    dist.all_gather_object(got, needs)
    for q in range(world):
        if q != rank:
            plan.set_send(q, got[q].get(rank, []))
    transport = HostTransport()
    opts = dict(mode=mode, orth=orth, prec=prec, rlen=30, tol=float(tol), max_restarts=int(max_restarts), device=0,
                spmv_format=fmt)
    eng = mpg.Engine.distributed_host(A_loc, b[r0:r1], xt[r0:r1], plan, transport, world, rank, **opts)
    cols = eng.sell_columns()
    mine = [{"csr": 0, "sell": 1, "node": 2}[eng.spmv_layout()["format"]],
            {"none": -1, "int32": 0, "int16": 1, "stepped": 2}[cols["form"]], cols["csr_slices"], plan.n_front]
    lays = [None] * world
    dist.all_gather_object(lays, mine)
    done = False
    while not done:
        _, done = eng.run(1 << 20)
    res = eng.report()
    eng.close()
    xs = [None] * world
    dist.all_gather_object(xs, res.x)
    if rank == 0:
        np.savez(out, x=np.concatenate(xs), step_res=res.step_res, cyc_r_norm=res.cyc_r_norm,
                 cyc_normalization=res.cyc_normalization, cyc_beta=res.cyc_beta,
                 counts=np.array([res.restarts, res.inner_k, res.total_iters]),
                 norms=np.array([res.res_norm, res.err_norm, res.minvb_norm]), status=np.array(res.status),
                 starts=starts, transport_error=np.array(transport.error or ""), layouts=np.array(lays))
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
