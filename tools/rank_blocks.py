"""The row blocks the 8-GPU run executes, timed one at a time on one GPU
(VERDICT r4 #4). For C4 (the Queen_4147 stand-in, stencil27:111 with 3 dof)
and C5 (BAND-100M with fp16 values), split over P ranks as
mpg_solve_loopback / bench.py lay them out (nnz-balanced for C4, equal rows
for C5), this builds rank q's local problem with its halo numbering
(HaloPlan: own rows, lower ranks' halo in front, higher ranks' after) and
runs that rank's fused engine alone on this GPU with a null communicator
(all-reduces leave the local partials, the halo exchange moves nothing):
the same kernels, launch shapes and storage the rank runs in the 8-GPU
solve, on a numerically different problem (halo entries stay 0), so the
per-kernel times are the rank's. Prints one JSON line per (config, rank):
the Arnoldi SpMV's layout, its in-cycle time (each launch's own events),
its storage bytes and fraction of 8 TB/s, and the dots / CGS update times.
  python tools/rank_blocks.py [--ranks 8] [--config c4 c5] [--which 0,big] [--format auto]
Run it under rocprofv3 --kernel-trace --stats for the kernel trace, or with
--pmc FETCH_SIZE / WRITE_SIZE (separate runs) for the traffic."""
import argparse
import ctypes as C
import json
import sys
import time
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO))
from tests.conftest import load_package  # noqa: E402

mpg = load_package()

ALLREDUCE_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(C.c_double), C.c_int32, C.c_int32)
EXCHANGE_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(C.c_void_p), C.POINTER(C.c_int64),
                          C.POINTER(C.c_void_p), C.POINTER(C.c_int64))


class _TransportC(C.Structure):
    _fields_ = [("user", C.c_void_p), ("allreduce", ALLREDUCE_FN), ("exchange", EXCHANGE_FN)]


class NullTransport:
    """mpg_host_transport that moves nothing: every rank's collectives are
    identities (timing of one rank's kernels only)."""

    def __init__(self):
        self._ar = ALLREDUCE_FN(lambda user, buf, count, op: 0)
        self._ex = EXCHANGE_FN(lambda user, send, sb, recv, rb: 0)
        self.c = _TransportC(None, self._ar, self._ex)
        self.error = None


def rows_of(A, r0, r1):
    """rows [r0, r1) of A with global columns"""
    a, z = int(A.rowptr[r0]), int(A.rowptr[r1])
    return mpg.Csr(r1 - r0, A.ncols, (A.rowptr[r0:r1 + 1] - a).astype(np.int32), A.col[a:z], A.val[a:z])


def config(name):
    if name == "c4":
        return mpg.gen_stencil27(111, 3), "mixed", "nnz"
    if name == "c5":
        return mpg.gen_band(10_000_000, 5, 4, seed=7), "mixed-half", "rows"
    raise ValueError(name)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", type=int, default=8)
    ap.add_argument("--config", nargs="+", default=["c4", "c5"])
    ap.add_argument("--which", default="0,big", help="ranks to time: numbers, 'big' (most nnz), 'last'")
    ap.add_argument("--cycles", type=int, default=2)
    ap.add_argument("--format", default="auto", help="the Arnoldi SpMV storage (spmv_format: auto, csr, sell, node)")
    a = ap.parse_args()
    P = a.ranks
    for cfg in a.config:
        t0 = time.time()
        A, mode, split = config(cfg)
        starts = (mpg.nnz_balanced_starts(A, P) if split == "nnz"
                  else np.array([A.nrows * q // P for q in range(P + 1)], dtype=np.int64))
        nnz_q = [int(A.rowptr[starts[q + 1]] - A.rowptr[starts[q]]) for q in range(P)]
        pick = []
        for w in a.which.split(","):
            q = int(np.argmax(nnz_q)) if w == "big" else P - 1 if w == "last" else int(w)
            if q not in pick:
                pick.append(q)
        xt = mpg.rand_vect(A.nrows, 42)
        print(f"[rank_blocks] {cfg}: n={A.nrows} nnz={A.nnz}, ranks' nnz {nnz_q}, built in {time.time() - t0:.1f}s",
              file=sys.stderr, flush=True)
        for q in pick:
            Aq = rows_of(A, int(starts[q]), int(starts[q + 1]))
            plan = mpg.HaloPlan(q, P, starts, Aq)
            for p in range(P):  # what every peer p needs from q (p's plan of its own rows)
                if p == q:
                    continue
                pp = mpg.HaloPlan(p, P, starts, rows_of(A, int(starts[p]), int(starts[p + 1])))
                plan.set_send(p, pp.recv_rows(q))
                pp.close()
            r0, r1 = int(starts[q]), int(starts[q + 1])
            bq = mpg.host_spmv(Aq, xt)  # (global columns: the rank's own b rows)
            opts = dict(mode=mode, orth="cgs", prec="identity", rlen=30, tol=0.0, max_restarts=100,
                        spmv_format=a.format)
            eng = mpg.Engine.distributed_host(Aq, bq, xt[r0:r1], plan, NullTransport(), P, q, **opts)
            try:
                eng.run(1)
                eng.sync()
                lay = dict(eng.spmv_layout(), **eng.sell_columns())
                ms, per = eng.time_spmv_incycle(a.cycles)

                def phase(ph):
                    try:
                        return round(eng.time_phase(ph, 5) * 1e3, 2)
                    except RuntimeError:  # (a phase the rank's step program does not launch on its own)
                        return None
                dots, upd = phase("dots"), phase("cgs_update")
                sb = eng.phase_bytes("spmv_storage")
                out = {"config": cfg, "rank": q, "ranks": P, "rows": r1 - r0, "nnz": nnz_q[q],
                       "n_front": plan.n_front, "n_ext": plan.n_ext, "layout": lay,
                       "spmv_us": round(ms * 1e3, 2), "spmv_launches": len(per),
                       "spmv_storage_mb": round(sb / 1e6, 2),
                       "spmv_storage_tbs": round(sb / (ms * 1e-3) / 1e12, 3),
                       "spmv_frac_8tbs": round(sb / (ms * 1e-3) / 8e12, 4),
                       "dots_us_mean_k": dots, "cgs_update_us_mean_k": upd,
                       "timing": "each SpMV launch's own kernel events over eager cycles (the rank's engine "
                                 "with a null communicator); dots / update: mpg_engine_time_phase"}
                print(json.dumps(out), flush=True)
            finally:
                eng.close()
                plan.close()
        del A


if __name__ == "__main__":
    main()
