"""Host transport for the row-partitioned engine (mpg_host_transport,
include/mpgmres/dist.h) over an initialised torch.distributed process group.

RCCL refuses two ranks on one GPU; this transport moves the same bytes
through host memory (gloo), so the product's distributed engine
(FusedEngine with a communicator, host/dist.cpp) runs as separate processes
sharing a device: the multi-rank rehearsal of bench.py and the multi-process
GPU tests. It is not the production transport (RCCL over xGMI is).

allreduce: every rank gathers all ranks' buffers and sums them in rank
order (q = 0, 1, ...), so every rank gets the same bits -- the order of the
single-process loopback communicator (mpg_solve_loopback), which makes the
two bit-comparable. exchange: one isend/irecv pair per peer.
"""
import ctypes as C

import numpy as np
import torch
import torch.distributed as dist

ALLREDUCE_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(C.c_double), C.c_int32, C.c_int32)
EXCHANGE_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(C.c_void_p), C.POINTER(C.c_int64),
                          C.POINTER(C.c_void_p), C.POINTER(C.c_int64))


class HostTransportC(C.Structure):
    """mirror of mpg_host_transport"""
    _fields_ = [("user", C.c_void_p), ("allreduce", ALLREDUCE_FN), ("exchange", EXCHANGE_FN)]


class HostTransport:
    def __init__(self, group=None):
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.error = None
        self._ar = ALLREDUCE_FN(self._allreduce)
        self._ex = EXCHANGE_FN(self._exchange)
        self.c = HostTransportC(None, self._ar, self._ex)

    # the reduction itself, on host arrays (also what the CPU tests call)
    def allreduce(self, buf: np.ndarray, op: int) -> None:
        t = torch.from_numpy(np.ascontiguousarray(buf, dtype=np.float64).copy())
        parts = [torch.empty_like(t) for _ in range(self.world)]
        dist.all_gather(parts, t, group=self.group)
        out = parts[0].numpy().copy()
        for p in parts[1:]:
            out = np.maximum(out, p.numpy()) if op else out + p.numpy()
        buf[:] = out

    def exchange(self, send: dict, recv_sizes: dict) -> dict:
        """send: {peer: bytes-like}, recv_sizes: {peer: nbytes} -> {peer: np.uint8 array}"""
        reqs, got = [], {}
        for q in range(self.world):
            if q == self.rank:
                continue
            if q in send and len(send[q]):
                src = torch.from_numpy(np.frombuffer(bytes(send[q]), dtype=np.uint8).copy())
                reqs.append(dist.isend(src, q, group=self.group))
            if recv_sizes.get(q, 0):
                buf = torch.empty(recv_sizes[q], dtype=torch.uint8)
                reqs.append(dist.irecv(buf, q, group=self.group))
                got[q] = buf
        for r in reqs:
            r.wait()
        return {q: b.numpy() for q, b in got.items()}

    # ctypes callbacks (errors are reported as a non-zero status; the C++
    # side raises, and the exception text is kept in self.error)
    def _allreduce(self, user, buf, count, op):
        try:
            self.allreduce(np.ctypeslib.as_array(buf, shape=(count,)), op)
            return 0
        except Exception as e:  # noqa: BLE001 -- must not unwind through C
            self.error = repr(e)
            return -1

    def _exchange(self, user, send, send_bytes, recv, recv_bytes):
        try:
            out = {q: C.string_at(send[q], send_bytes[q]) for q in range(self.world)
                   if q != self.rank and send_bytes[q] > 0}
            sizes = {q: int(recv_bytes[q]) for q in range(self.world) if q != self.rank and recv_bytes[q] > 0}
            got = self.exchange(out, sizes)
            for q, arr in got.items():
                C.memmove(recv[q], arr.ctypes.data, sizes[q])
            return 0
        except Exception as e:  # noqa: BLE001
            self.error = repr(e)
            return -1
