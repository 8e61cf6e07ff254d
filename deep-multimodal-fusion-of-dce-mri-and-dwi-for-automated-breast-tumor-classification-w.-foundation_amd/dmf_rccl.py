"""A bare RCCL communicator for the data path's gradient all-reduce.

torch.distributed stays the rendezvous (ranks, barrier, the unique-id
broadcast, the gloo rehearsal); the gradient collectives of the captured
training step go straight to RCCL (``ncclAllReduce`` on a HIP stream):

  * they are plain stream work, so they capture into the step's hipGraph
    like any kernel (RCCL supports stream capture);
  * torch's NCCL process group would wrap each in a Work whose completion
    event its watchdog thread polls -- and polling an event recorded inside
    a capture fails (hipErrorCapturedEvent, measured on this stack), which
    takes the process down at random.

The library is the librccl.so torch itself loaded (same HIP runtime).
"""
from __future__ import annotations

import ctypes
import os

import torch

NCCL_FLOAT32 = 7
NCCL_SUM = 0


class _UniqueId(ctypes.Structure):
    _fields_ = [("internal", ctypes.c_char * 128)]


def _lib():
    here = os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so")
    path = here if os.path.exists(here) else "librccl.so"
    lib = ctypes.CDLL(path)
    lib.ncclGetUniqueId.argtypes = [ctypes.POINTER(_UniqueId)]
    lib.ncclCommInitRank.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_int, _UniqueId, ctypes.c_int]
    lib.ncclAllReduce.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int,
                                  ctypes.c_void_p, ctypes.c_void_p]
    lib.ncclCommDestroy.argtypes = [ctypes.c_void_p]
    lib.ncclCommCount.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int)]
    lib.ncclGetErrorString.argtypes = [ctypes.c_int]
    lib.ncclGetErrorString.restype = ctypes.c_char_p
    return lib


class RcclComm:
    """One RCCL communicator over the ranks of the default process group
    (``rank``/``world`` explicit so a 1-rank communicator works without one)."""

    def __init__(self, rank, world, device):
        self.lib = _lib()
        self.rank, self.world, self.device = rank, world, torch.device(device)
        uid = _UniqueId()
        if rank == 0:
            self._check(self.lib.ncclGetUniqueId(ctypes.byref(uid)), "ncclGetUniqueId")
        if world > 1:
            import torch.distributed as dist
            box = [bytes(uid.internal) if rank == 0 else None]
            dist.broadcast_object_list(box, src=0)
            ctypes.memmove(uid.internal, box[0], 128)
        self.comm = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            self._check(self.lib.ncclCommInitRank(ctypes.byref(self.comm), world, uid, rank), "ncclCommInitRank")

    def _check(self, rc, what):
        if rc != 0:
            raise RuntimeError(f"{what} failed: {self.lib.ncclGetErrorString(rc).decode()} ({rc})")

    def all_reduce_sum_(self, t):
        """In-place sum over ranks of a contiguous fp32 CUDA tensor, on the
        current HIP stream."""
        if t.dtype != torch.float32 or not t.is_cuda or not t.is_contiguous():
            raise ValueError("all_reduce_sum_: needs a contiguous float32 CUDA tensor")
        if t.numel() == 0:
            return t
        s = torch.cuda.current_stream(t.device).cuda_stream
        self._check(self.lib.ncclAllReduce(t.data_ptr(), t.data_ptr(), t.numel(), NCCL_FLOAT32, NCCL_SUM,
                                           self.comm, s), "ncclAllReduce")
        return t

    def count(self):
        """Ranks of the communicator as RCCL reports them (ncclCommCount)."""
        n = ctypes.c_int(0)
        self._check(self.lib.ncclCommCount(self.comm, ctypes.byref(n)), "ncclCommCount")
        return n.value

    def close(self):
        if self.comm:
            self.lib.ncclCommDestroy(self.comm)
            self.comm = ctypes.c_void_p()
