"""Data-parallel training of the hiseg ROI path: one process per GPU, gradient all-reduce over RCCL.

The reference trains on one device (train_advanced.py:680-762, no DDP); SURVEY §8e fixes the multi-GPU
semantics: every rank runs the full model on its own slice of the image batch (1..R ROIs per image),
BatchNorm statistics stay per rank (the reference has no SyncBN), and the only exchange is the average
of the parameter gradients before the optimiser step.

MI355X design: the gradients of all trainable parameters live in ONE flat f32 buffer (train_engine
.FlatParams), so the exchange is a few large contiguous RCCL all-reduces instead of one per tensor.  The
buffer is cut into buckets of ``bucket_mb`` at parameter boundaries.  The backward is a tape replayed in
reverse; the first step records, for every parameter, the last tape op that writes its gradient
(TrainState.grad is the only way a backward closure reaches a gradient pointer).  From the second step on,
each bucket's all-reduce is enqueued on a dedicated communication stream right after the tape op that
completes it (stream-ordered through an event), so RCCL traffic over xGMI overlaps the remaining backward
kernels; the compute stream waits for the communication stream once, at the end of the backward.  Parameter
order follows the forward, the backward runs it in reverse, so the tail buckets finish first.

xGMI is point-to-point (7 links x ~153 GB/s per GPU): a ring all-reduce of S bytes moves 2*(n-1)/n*S per
rank; 55 MB of B0-std gradients take ~0.7 ms on one ring, well under one backward conv of a 32-image step,
so the default buckets are large (25 MB: 2-3 buckets for B0, 10 for B7-ultra) to keep RCCL launches few.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Tuple

import torch
import torch.distributed as dist
import torch.nn as nn

from . import comm as _comm
from .streams import role_stream

_SYNC_KEY = "_hiseg_grad_sync"


class GradBucketSync:
    """Bucketed, backward-overlapped gradient averaging over a process group for one TrainState."""

    def __init__(self, process_group=None, bucket_mb: float = 25.0):
        self.pg = process_group
        self.bucket_bytes = int(bucket_mb * (1 << 20))
        self.world = dist.get_world_size(process_group)
        # RCCL averages in the collective (ReduceOp.AVG: a pre-multiply by 1/world, exact for power-of-two worlds);
        # gloo has no AVG, so there the bucket is summed and scaled by one extra kernel
        self.avg_in_collective = dist.get_backend(process_group) == "nccl"
        self.state = None
        self.buckets: List[Tuple[int, int]] = []          # [begin, end) element ranges of the flat grad
        self.bucket_params: List[List[int]] = []          # param ids per bucket
        self.last_op: Optional[Dict[int, int]] = None     # param id -> last backward op index (recorded)
        self.launch_after: Dict[int, List[int]] = {}      # op index -> buckets that become complete
        self.recording: Optional[Dict[int, int]] = None
        self.launched: List[int] = []                     # bucket launch order of the last backward
        self.comm_stream = None
        self.comm: Optional[_comm.Communicator] = None   # libhiseg's RCCL communicator (nccl groups, GPU grads)
        self.steps = 0

    # -- layout
    def attach(self, S):
        if self.state is S:
            return
        self.state = S
        flat = S.flat
        self.buckets, self.bucket_params = [], []
        begin, cur, ids = 0, 0, []
        for _, p in flat.named:
            off, k = flat.offsets[id(p)]
            if ids and (cur - begin) * 4 >= self.bucket_bytes:
                self.buckets.append((begin, cur))
                self.bucket_params.append(ids)
                begin, ids = cur, []
            ids.append(id(p))
            cur = off + k
        self.buckets.append((begin, cur))
        self.bucket_params.append(ids)
        self.last_op, self.launch_after = None, {}
        dev = flat.grad.device
        self.comm_stream = role_stream("comm", dev) if dev.type == "cuda" else None
        if self.comm is None and _comm.uses_rccl(self.pg, flat.grad):
            self.comm = _comm.communicator(self.pg, dev)

    # -- tape callbacks (train_engine.Tape.run_backward)
    def begin(self, n_ops: int):
        self.launched = []
        self.recording = {} if self.last_op is None else None
        for b in self.launch_after.get(-1, ()):   # buckets no backward op writes (already zeroed)
            self._launch(b)

    def record(self, p: nn.Parameter, op_index: Optional[int]):
        if self.recording is not None and op_index is not None:
            self.recording[id(p)] = max(op_index, self.recording.get(id(p), -1))

    def after_op(self, i: int):
        for b in self.launch_after.get(i, ()):
            self._launch(b)

    def end(self, n_ops: int):
        if self.recording is not None:   # first step: learn the schedule, reduce everything now
            self.last_op = self.recording
            self.recording = None
            self.launch_after = {}
            for b, ids in enumerate(self.bucket_params):
                ready = max((self.last_op.get(i, -1) for i in ids), default=-1)
                self.launch_after.setdefault(min(ready, n_ops - 1) if ready >= 0 else -1, []).append(b)
        for b in range(len(self.buckets)):
            if b not in self.launched:
                self._launch(b)
        if self.comm_stream is not None:
            torch.cuda.current_stream(self.comm_stream.device).wait_stream(self.comm_stream)
        self.steps += 1

    def _reduce(self, view: torch.Tensor):
        if self.comm is not None:   # RCCL through libhiseg: an enqueue on the current stream, nothing tracked
            self.comm.all_reduce_(view, _comm.AVG)
        elif self.avg_in_collective:
            dist.all_reduce(view, op=dist.ReduceOp.AVG, group=self.pg)
        else:
            dist.all_reduce(view, group=self.pg)
            view.mul_(1.0 / self.world)

    def _launch(self, b: int):
        begin, end = self.buckets[b]
        view = self.state.flat.grad[begin:end]
        if self.comm_stream is None:
            self._reduce(view)
        else:
            self.comm_stream.wait_stream(torch.cuda.current_stream(self.comm_stream.device))
            with torch.cuda.stream(self.comm_stream):
                self._reduce(view)
        self.launched.append(b)


def enable_grad_sync(model: nn.Module, process_group=None, bucket_mb: float = 25.0,
                     broadcast_from: Optional[int] = 0) -> GradBucketSync:
    """Make every hiseg training backward of `model` average its gradients over the process group.

    Parameters and buffers are broadcast from rank `broadcast_from` first (as torch DDP does at
    construction), so all replicas start identical."""
    if not dist.is_initialized():
        raise RuntimeError("hiseg.distributed: torch.distributed is not initialised")
    if broadcast_from is not None:
        with torch.no_grad():
            for t in list(model.parameters()) + list(model.buffers()):
                dist.broadcast(t.data, broadcast_from, group=process_group)
    sync = GradBucketSync(process_group, bucket_mb)
    p0 = next(iter(model.parameters()), None)
    if p0 is not None and _comm.uses_rccl(process_group, p0):   # collective: every rank is here together
        sync.comm = _comm.communicator(process_group, p0.device)
    model.__dict__[_SYNC_KEY] = sync
    return sync


def all_reduce_counts(counts: torch.Tensor, process_group=None) -> torch.Tensor:
    """Sum a count vector over the process group in place (float64; libhiseg's RCCL communicator on the GPU -- the
    step that calls this may be under graph capture -- gloo on the CPU)."""
    if _comm.uses_rccl(process_group, counts):
        _comm.communicator(process_group, counts.device).all_reduce_(counts, _comm.SUM)
    else:
        dist.all_reduce(counts, op=dist.ReduceOp.SUM, group=process_group)
    return counts


def sync_loss_class_weights(loss_fn: nn.Module, process_group=None) -> nn.Module:
    """Data-parallel semantics of the loss's dynamic class weights (hierarchical_segmentation.py:227-255,
    286-309): the reference derives them (and their EMA) from the class pixel counts of the whole batch, which
    under data parallelism is spread over the ranks.  With this, every rank's RefinedHierarchicalLoss
    all-reduces its 4 counts (bg, fg, target, non-target) before the EMA update, so all ranks carry the
    weights a single process would compute on the concatenated batch."""
    if not dist.is_initialized():
        raise RuntimeError("hiseg.distributed: torch.distributed is not initialised")
    if _comm.uses_rccl(process_group) and torch.cuda.is_available():
        _comm.communicator(process_group)   # collective creation here, where every rank calls together
    loss_fn.count_sync = lambda c: all_reduce_counts(c, process_group)
    return loss_fn


def broadcast_training_state(optimizer=None, loss_fn: Optional[nn.Module] = None, src: int = 0,
                             process_group=None) -> None:
    """Copy rank `src`'s FusedAdamW moments and per-parameter step counts and the loss's dynamic-weight EMA state
    to every rank (after enable_grad_sync broadcast the parameters): replicas that trained on their own before
    continue as one data-parallel trajectory, as torch DDP replicas built from one checkpoint would."""
    if not dist.is_initialized():
        raise RuntimeError("hiseg.distributed: torch.distributed is not initialised")
    with torch.no_grad():
        if optimizer is not None and getattr(optimizer, "exp_avg", None) is not None:
            # the flat layouts must match; the step-count segment table may not (ranks with different unfreeze
            # histories): broadcast the source's sizes first and re-size this rank's table to them
            o = optimizer
            meta = torch.tensor([o.exp_avg.numel(), o._nseg], dtype=torch.int64, device=o.exp_avg.device)
            dist.broadcast(meta, src, group=process_group)
            numel, nseg = (int(v) for v in meta.tolist())
            if numel != o.exp_avg.numel():
                raise RuntimeError(f"broadcast_training_state: this rank's optimizer covers {o.exp_avg.numel()} "
                                   f"parameters, rank {src}'s {numel}: the flat layouts differ")
            if nseg != o._nseg:
                o._seg_start = torch.empty(nseg + 1, dtype=o._seg_start.dtype, device=o._seg_start.device)
                o._steps = torch.empty(2 * nseg, dtype=o._steps.dtype, device=o._steps.device)
                o._nseg = nseg
            for t in (o.exp_avg, o.exp_avg_sq, o._seg_start, o._steps):
                dist.broadcast(t, src, group=process_group)
        st = getattr(loss_fn, "_state", None) if loss_fn is not None else None
        if st is not None:
            dist.broadcast(st, src, group=process_group)


def grad_sync_of(model: nn.Module) -> Optional[GradBucketSync]:
    return model.__dict__.get(_SYNC_KEY)


class DistributedDataParallel(nn.Module):
    """torch DDP-shaped wrapper: ``ddp = DistributedDataParallel(model); logits, aux = ddp(images, rois)``;
    ``ddp.module`` is the wrapped model (state_dict keys unchanged)."""

    def __init__(self, module: nn.Module, process_group=None, bucket_mb: float = 25.0):
        super().__init__()
        self.module = module
        self.sync = enable_grad_sync(module, process_group, bucket_mb)

    def forward(self, *args, **kwargs):
        return self.module(*args, **kwargs)
