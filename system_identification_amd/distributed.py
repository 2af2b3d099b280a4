"""Multi-GPU normal equations: samples sharded over ranks, one all-reduce of the Gram.

One process per GPU (torch.distributed; backend "nccl" is RCCL over xGMI on ROCm).  Rank r owns the
contiguous samples ``[r·N/G, (r+1)·N/G)`` (filtering is done on the host first, so no halo), builds its
partial Gram on its own device, and a single ``all_reduce(SUM)`` of the (W+1)x(W+1) fp64 buffer gives
every rank the full normal equations.  The stacked Y panel, if requested, stays sharded.

The per-rank compute is a parameter (``build_partial``) so the same host logic runs with the HIP engine
on a GPU and, in the CPU test-suite, with a checker under the gloo backend.
"""
from __future__ import annotations

from typing import Callable

import numpy as np


def shard_range(N: int, rank: int, world: int) -> tuple:
    """Contiguous sample range of ``rank`` (sizes differ by at most one)."""
    if world < 1 or not (0 <= rank < world):
        raise ValueError("bad rank/world")
    return (N * rank) // world, (N * (rank + 1)) // world


def shard_channels(arrays, rank: int, world: int):
    """Slice channel-major (channels x N) arrays to this rank's samples."""
    N = np.asarray(arrays[0]).shape[-1]
    s0, s1 = shard_range(N, rank, world)
    return [np.ascontiguousarray(np.asarray(a)[..., s0:s1]) for a in arrays]


def pack_normal_equations(ne: dict):
    """(W+1)x(W+1) buffer [[G, g], [gᵀ, bᵀb]] and the row count (the engine's device Gram layout)."""
    G, g = np.asarray(ne["gram"]), np.asarray(ne["Atb"])
    W = G.shape[0]
    buf = np.empty((W + 1, W + 1))
    buf[:W, :W] = G
    buf[:W, W] = g
    buf[W, :W] = g
    buf[W, W] = ne["btb"]
    return buf, int(ne["num_rows"])


def unpack_normal_equations(buf, num_rows: int) -> dict:
    buf = np.asarray(buf)
    W = buf.shape[0] - 1
    return {"gram": buf[:W, :W].copy(), "Atb": buf[:W, W].copy(), "btb": float(buf[W, W]), "num_rows": int(num_rows)}


def pack_upper(buf, rows) -> np.ndarray:
    """The exchange format of SURVEY.md §8e (and of the device's sysid_allreduce_normal_equations): the upper
    triangle of the n x n buffer row by row (row i at i n - i (i - 1) / 2), then the row count: n (n + 1) / 2 + 1
    doubles (Spot n = W+1 = 155: 12,091; G1 n = 359: 64,621)."""
    buf = np.asarray(buf, dtype=np.float64)
    n = buf.shape[0]
    return np.concatenate([buf[np.triu_indices(n)], [float(rows)]])


def unpack_upper(x, n: int):
    """Inverse of pack_upper: the symmetric n x n buffer (both triangles from the packed one) and the row count."""
    x = np.asarray(x, dtype=np.float64)
    buf = np.empty((n, n))
    iu = np.triu_indices(n)
    buf[iu] = x[:-1]
    buf.T[iu] = x[:-1]
    return buf, x[-1]


def allreduce_normal_equations(ne: dict, device=None, group=None) -> dict:
    """Sum the per-rank normal equations over the process group: one collective of the packed upper triangle
    of [[G, g], [gᵀ, bᵀb]] plus the row count (pack_upper)."""
    import torch
    import torch.distributed as dist
    buf, rows = pack_normal_equations(ne)
    n = buf.shape[0]
    t = torch.from_numpy(pack_upper(buf, rows))
    if device is not None:
        t = t.to(device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    out, total = unpack_upper(t.cpu().numpy(), n)
    return unpack_normal_equations(out, int(round(total)))


def build_normal_equations_distributed(q, dq, ddq, tau, cnt, build_partial: Callable, rank: int, world: int,
                                       device=None, group=None) -> dict:
    """Shard (channel-major) inputs, build this rank's partial normal equations with ``build_partial``
    (e.g. ``SystemIdentification.build_normal_equations``), and all-reduce them."""
    parts = shard_channels([q, dq, ddq, tau, cnt], rank, world)
    ne = build_partial(*parts)
    if world == 1:
        return ne
    return allreduce_normal_equations(ne, device=device, group=group)


class RcclGramComm:
    """The C ABI's own exchange step (sysid_rccl_* / sysid_allreduce_gram): what a non-Python host would
    call between its per-rank sysid_build_device and the solver.  The 128-byte unique id is created on
    rank 0 and handed to the other ranks out of band (here: any callable, e.g. a torch.distributed or
    file broadcast)."""

    def __init__(self, engine, rank: int, world: int, share_id: Callable = None):
        import ctypes
        self.lib, self.engine = engine.lib, engine
        uid = ctypes.create_string_buffer(128)
        err = None
        if rank == 0 and self.lib.sysid_rccl_unique_id(uid) != 0:
            err = self.lib.sysid_rccl_last_error().decode()
        if world > 1:
            if share_id is None:
                raise ValueError("world > 1 needs share_id to distribute the RCCL unique id")
            # rank 0 shares an empty id when it has none, so that no rank is left waiting in comm_init
            got = bytes(share_id(b"" if err else uid.raw))
            if len(got) != 128:
                raise RuntimeError(err or "rank 0 could not create an RCCL unique id")
            uid = ctypes.create_string_buffer(got, 128)
        if err:
            raise RuntimeError(err)
        self._comm = ctypes.c_void_p()
        if self.lib.sysid_rccl_comm_init(ctypes.byref(self._comm), int(world), uid, int(rank), int(engine.device)) != 0:
            raise RuntimeError(self.lib.sysid_rccl_last_error().decode())

    def _check(self, t, n: int, what: str):
        """The C side trusts the buffer sizes: a float64 tensor of exactly n elements on the engine's device."""
        import torch
        if (not isinstance(t, torch.Tensor) or t.dtype != torch.float64 or t.device.type != "cuda"
                or t.device.index != self.engine.device or t.numel() != n or not t.is_contiguous()):
            raise ValueError(f"{what}: need a contiguous float64 tensor of {n} elements on cuda:{self.engine.device}, "
                             f"got {getattr(t, 'dtype', type(t))} {tuple(getattr(t, 'shape', ()))} on "
                             f"{getattr(t, 'device', None)}")

    def allreduce_gram(self, gram, stream=None):
        """In-place sum of a (W+1)x(W+1) float64 CUDA tensor over the ranks (stream-ordered)."""
        import ctypes
        import torch
        n = self.engine.w + 1
        self._check(gram, n * n, "gram")
        st = stream if stream is not None else torch.cuda.current_stream(self.engine.device).cuda_stream
        if self.lib.sysid_allreduce_gram(self.engine._h, ctypes.c_void_p(gram.data_ptr()), self._comm,
                                         ctypes.c_void_p(st)) != 0:
            raise RuntimeError(self.lib.sysid_rccl_last_error().decode())

    def exchange_buffer(self):
        """A device buffer for allreduce_normal_equations (sysid_exchange_bytes)."""
        import torch
        n = int(self.lib.sysid_exchange_bytes(self.engine._h)) // 8
        return torch.zeros(n, dtype=torch.float64, device=torch.device("cuda", self.engine.device))

    def allreduce_normal_equations(self, gram, rows: float, xbuf, stream=None):
        """The packed exchange: the upper triangle of the (W+1)x(W+1) Gram plus this rank's row
        count, (W+1)(W+2)/2 + 1 doubles in one all-reduce; the Gram is rewritten with the sums (both triangles) and
        xbuf[-1] holds the job's row count.  Stream-ordered."""
        import ctypes
        import torch
        n = self.engine.w + 1
        self._check(gram, n * n, "gram")
        self._check(xbuf, int(self.lib.sysid_exchange_bytes(self.engine._h)) // 8, "xbuf")
        st = stream if stream is not None else torch.cuda.current_stream(self.engine.device).cuda_stream
        if self.lib.sysid_allreduce_normal_equations(self.engine._h, ctypes.c_void_p(gram.data_ptr()),
                                                      ctypes.c_void_p(xbuf.data_ptr()), float(rows), self._comm,
                                                      ctypes.c_void_p(st)) != 0:
            raise RuntimeError(self.lib.sysid_rccl_last_error().decode())

    def close(self):
        if getattr(self, "_comm", None) and self._comm.value:
            self.lib.sysid_rccl_comm_destroy(self._comm)
            self._comm = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def make_gram_exchange(engine, rank: int, world: int, share_id: Callable, all_ok: Callable, comm_cls=None):
    """The multi-GPU exchange step bench.py runs (and a non-Python host would): the engine's own C-ABI RCCL
    communicator (RcclGramComm), or, when its set-up fails on ANY rank, no communicator, so that every rank falls
    back to the same torch.distributed all-reduce.  ``share_id(raw) -> bytes`` hands rank 0's 128-byte id to
    the others; ``all_ok(flag) -> bool`` is the minimum of a 0/1 flag over the ranks (a collective).  Returns
    (comm or None, a name for the JSON line)."""
    comm_cls = comm_cls or RcclGramComm
    comm, name = None, None
    try:
        comm = comm_cls(engine, rank, world, share_id=share_id)
        ok = 1
    except Exception as exc:  # noqa: BLE001 - the reason is reported
        comm, name, ok = None, f"torch.distributed.all_reduce (C-ABI RCCL init failed: {exc})", 0
    if not all_ok(ok) and comm is not None:
        comm.close()
        comm, name = None, "torch.distributed.all_reduce (C-ABI RCCL init failed on another rank)"
    if comm is not None:
        name = "sysid_allreduce_normal_equations (RCCL, C ABI, packed upper triangle + row count)"
    return comm, name
