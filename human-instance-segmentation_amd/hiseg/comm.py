"""RCCL communicator owned by libhiseg for the collectives inside a training step (include/hiseg_comm.h).

Why not torch.distributed's ProcessGroupNCCL for those: its watchdog thread polls the end event of every
collective it issued (WorkNCCL::isCompleted -> hipEventQuery), and on ROCm that query fails with
hipErrorCapturedEvent while the stream the event was last recorded on is capturing.  The process group records
those events on its own communication stream, and a whole-step HIP graph capture that issues a collective pulls
that stream into the capture: if the watchdog has not yet retired the last eager collective when the capture
begins, its next poll aborts the process (round 5: rc 134 in test_graphed_ddp_step_rccl_world1_equals_eager).  A
sleep before each capture only narrowed that window.  Collectives on this communicator are plain enqueues on the
caller's stream (ncclAllReduce through libhiseg): no watchdog, no events, nothing polled from another thread, so a
capture cannot race anything.  The process group stays the rendezvous (it carries the RCCL unique id) and serves
the eager collectives (parameter / state broadcast), none of which is ever issued under capture.
"""
from __future__ import annotations

import ctypes
import os
from typing import Dict, Tuple

import torch
import torch.distributed as dist

from . import _lib

F32, F64 = 0, 1
SUM, AVG = 0, 1
_DTYPES = {torch.float32: F32, torch.float64: F64}
_cache: Dict[Tuple[int, int], "Communicator"] = {}


def _rccl_path() -> str:
    """The librccl torch itself loaded (one RCCL instance per process)."""
    p = os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so")
    return p if os.path.exists(p) else "librccl.so"


class Communicator:
    """An RCCL communicator over the ranks of ``process_group`` on ``device`` (collective construction)."""

    def __init__(self, process_group=None, device=None):
        if not dist.is_initialized():
            raise RuntimeError("hiseg.comm: torch.distributed is not initialised")
        device = torch.device(device if device is not None else "cuda")
        if device.type != "cuda":
            raise RuntimeError("hiseg.comm: an RCCL communicator needs a GPU device")
        self.device = torch.device("cuda", device.index if device.index is not None else torch.cuda.current_device())
        self.pg = process_group
        self.pg_obj = None
        self.world = dist.get_world_size(process_group)
        self.rank = dist.get_rank(process_group)
        L = _lib.lib()
        _lib.check(L.hiseg_comm_load(_rccl_path().encode()), "comm_load")
        uid = (ctypes.c_ubyte * 128)()
        if self.rank == 0:
            _lib.check(L.hiseg_comm_unique_id(uid), "comm_unique_id")
        t = torch.tensor(list(bytes(uid)), dtype=torch.uint8)
        if dist.get_backend(process_group) == "nccl":
            t = t.to(self.device)
        src = dist.get_global_rank(process_group, 0) if process_group is not None else 0
        dist.broadcast(t, src, group=process_group)
        uid = (ctypes.c_ubyte * 128)(*t.cpu().tolist())
        h = ctypes.c_void_p()
        _lib.check(L.hiseg_comm_init(ctypes.byref(h), self.world, uid, self.rank, self.device.index), "comm_init")
        self.handle = h.value

    def all_reduce_(self, t: torch.Tensor, op: int = SUM, stream=None) -> torch.Tensor:
        """In-place all-reduce of a contiguous f32 / f64 tensor on ``stream`` (default: the current stream)."""
        if t.dtype not in _DTYPES or not t.is_contiguous() or t.device != self.device:
            raise RuntimeError(f"hiseg.comm: all_reduce_ needs a contiguous f32/f64 tensor on {self.device}, got "
                               f"{t.dtype} {t.device} contiguous={t.is_contiguous()}")
        s = stream if stream is not None else torch.cuda.current_stream(self.device)
        _lib.check(_lib.lib().hiseg_comm_all_reduce(self.handle, t.data_ptr(), t.numel(), _DTYPES[t.dtype], op,
                                                    s.cuda_stream), "comm_all_reduce")
        return t

    def destroy(self):
        if self.handle:
            _lib.check(_lib.lib().hiseg_comm_destroy(self.handle), "comm_destroy")
            self.handle = None


def communicator(process_group=None, device=None) -> Communicator:
    """The process's communicator for (process_group, device), created on first use (collectively: every rank of
    the group must make its first call for a group together, as for any process-group collective)."""
    dev = torch.device(device if device is not None else "cuda")
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    pg = process_group if process_group is not None else dist.group.WORLD
    key = (id(pg), idx)   # the communicator holds ``pg``, so its id is not reused while the entry lives
    c = _cache.get(key)
    if c is None or c.handle is None or c.pg_obj is not pg:
        c = _cache[key] = Communicator(process_group, torch.device("cuda", idx))
        c.pg_obj = pg
    return c


def uses_rccl(process_group=None, t: torch.Tensor = None) -> bool:
    """True when collectives of ``process_group`` on ``t`` go through this communicator (an nccl group and a GPU
    tensor); gloo groups and CPU tensors stay on torch.distributed."""
    return (dist.is_initialized() and dist.get_backend(process_group) == "nccl"
            and (t is None or t.device.type == "cuda"))
