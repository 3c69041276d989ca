"""RCCL communicator of the C ABI (include/enf.h: enf_comm_unique_id / enf_comm_init /
enf_allreduce_sum / enf_comm_destroy) for the data-parallel optimize_whitening step.

The reference has no distributed path (src/optimize_whitening.jl:25-45 is single-process); the
build's data-parallel training sums the (1 + P) unnormalised loss/gradient values
of every rank's minibatch share with one in-place RCCL all-reduce over xGMI. Calling RCCL through
libenf (rather than torch.distributed) puts the collective on the same HIP stream as the gradient
and update kernels, so a whole training epoch -- gradient, all-reduce, update -- can be captured as
one HIP graph and replayed (train.py optimize_whitening(graph=True)).
"""
from __future__ import annotations

import ctypes
from typing import Optional

import torch

from . import _lib

UNIQUE_ID_BYTES = _lib.UNIQUE_ID_BYTES


def unique_id() -> bytes:
    """A fresh RCCL unique id (rank 0 creates it and ships it to the other ranks out of band)."""
    buf = ctypes.create_string_buffer(UNIQUE_ID_BYTES)
    _lib.check(_lib.lib().enf_comm_unique_id(buf))
    return buf.raw


class EnfComm:
    """One rank of an RCCL communicator on the current HIP device."""

    def __init__(self, nranks: int, rank: int, uid: bytes):
        if len(uid) != UNIQUE_ID_BYTES:
            raise ValueError(f"unique id must be {UNIQUE_ID_BYTES} bytes")
        self.nranks, self.rank = int(nranks), int(rank)
        self._h = ctypes.c_void_p()
        _lib.check(_lib.lib().enf_comm_init(ctypes.byref(self._h), self.nranks, uid, self.rank))

    @classmethod
    def single(cls) -> "EnfComm":
        """A one-rank communicator (the all-reduce is the identity): tests and one-GPU graphs."""
        return cls(1, 0, unique_id())

    @classmethod
    def from_process_group(cls, group=None) -> "EnfComm":
        """Create the communicator of torch.distributed's (default) group: rank 0's unique id is
        broadcast over the group (gloo or nccl), then every rank initialises its RCCL rank."""
        import torch.distributed as dist

        world, rank = dist.get_world_size(group), dist.get_rank(group)
        obj = [unique_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=dist.get_global_rank(group, 0) if group is not None else 0, group=group)
        return cls(world, rank, obj[0])

    @property
    def handle(self) -> ctypes.c_void_p:
        """The enf_comm handle (for enf_whitening_step_dp)."""
        return self._h

    def allreduce_sum_(self, buf: torch.Tensor, stream: Optional[int] = None) -> torch.Tensor:
        """In-place sum over the ranks of a contiguous device tensor (fp32 / fp64), asynchronous on
        `stream` (default: torch's current stream of buf's device)."""
        if not buf.is_contiguous() or buf.dtype not in (torch.float32, torch.float64):
            raise ValueError("allreduce_sum_ needs a contiguous float32/float64 device tensor")
        if stream is None:
            stream = torch.cuda.current_stream(buf.device).cuda_stream
        dt = _lib.ENF_F64 if buf.dtype == torch.float64 else _lib.ENF_F32
        _lib.check(_lib.lib().enf_allreduce_sum(self._h, buf.data_ptr(), buf.numel(), dt, stream))
        return buf

    def close(self) -> None:
        if self._h:
            _lib.check(_lib.lib().enf_comm_destroy(self._h))
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
