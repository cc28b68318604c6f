"""Whole-step HIP graphs for training.

A training step on the hiseg path is ~1 000 kernel launches issued from Python (tape engine, ctypes
descriptors); on one MI355X the B0-std step's kernels take ~80 ms while issuing them takes longer, so the
GPU idles between launches.  GraphedStep captures one step -- forward, loss, backward and the optimizer --
into a HIP graph (torch.cuda.graph on the step's stream) and replays it: one launch per step.

Every piece of per-step state the kernels use lives on the device, so a replayed step is the next step:
the Dropout2d seed base (TrainState.begin_step), the loss's dynamic-weight EMA, FusedAdamW's step count and
skip counter (fixed slot, committed by the library).  Host-side values are frozen into the graph: the
inputs' addresses (the step must read the same input tensors, refilled in place between steps) and the shapes.
Schedule values are not host-side: FusedAdamW's learning rate (and decay factor) and UNetDistillationLoss's
temperature / weights live in small device buffers the kernels read at run time ("device-scalar owners").  An owner
used while a step is being captured registers with it (note_device_scalars); before every replay GraphedStep has
each owner write its current values (sync_device_scalars: a fill on the replay stream when they changed), so a
per-epoch LR or temperature schedule replays the same graph.  Only an owner's structural state (graph_key: e.g.
the distillation terms switched off) and an optimizer without device scalars (its learning rate) force a
re-capture.

The graph also holds raw pointers to the optimizer's buffers (moments, step counts, norm partials), the
model's flat parameters and its conv packing table.  Anything that re-allocates them -- a new optimizer
(the reference's pattern at progressive unfreezing), FusedAdamW re-binding to a new flat layout, a new
trainable set or compute dtype -- changes GraphedStep's fingerprint of that state; the next call then
drops the graph, runs ``eager`` steps again (the re-binding and re-packing happen there, for real) and
captures anew.

Data parallel (hiseg.distributed over RCCL): the bucketed gradient all-reduces are enqueued on the
communication stream during the backward and joined back before the optimizer, so stream capture records
them into the same graph (the RCCL kernels become graph nodes; the communicator was created by the eager
steps).  The first eager step of a GradBucketSync learns its launch schedule, the second uses it, the
capture records it.  Enabling the exchange after a capture changes the fingerprint (re-capture).  gloo
process groups cannot be captured (host-side reduction): keep such steps eager.
"""
from __future__ import annotations

import os
from typing import Callable, List, Optional

import torch

from .streams import role_stream

_capture_owners: Optional[List] = None


def note_device_scalars(owner) -> None:
    """Called by a device-scalar owner (``sync_device_scalars()`` / ``graph_key()``) whenever its kernels are
    enqueued: during a GraphedStep capture it joins that step's owners (synced before every replay)."""
    if _capture_owners is not None and all(o is not owner for o in _capture_owners):
        _capture_owners.append(owner)


class _CaptureOwners:
    def __enter__(self):
        global _capture_owners
        self.prev, _capture_owners = _capture_owners, []
        return _capture_owners

    def __exit__(self, *exc):
        global _capture_owners
        _capture_owners = self.prev
        return False


class GraphedStep:
    """``gs = GraphedStep(step_fn, optimizer_fn)``; every ``gs()`` runs exactly one training step and returns
    step_fn's outputs (for replays: the tensors captured, refreshed in place).

    The first ``eager`` calls (default 2: the first step creates the conv plans, the second builds the one
    packing table from them) run step_fn eagerly on a side stream -- host-to-device uploads, allocator
    warm-up, optimizer creation; torch.cuda.graph's warm-up rule -- the next call captures it and replays it
    once, later calls replay.  ``optimizer_fn`` returns the optimizer (or None): its learning rate is watched and
    its parameters' version counters are bumped after each replay (eval plans packed from the weights must
    see the update, as after an eager step)."""

    def __init__(self, step_fn: Callable, optimizer_fn: Optional[Callable] = None, eager: int = 2):
        self.fn, self.opt_fn, self.eager = step_fn, optimizer_fn, max(1, int(eager))
        self.calls = 0
        self.graph: Optional[torch.cuda.CUDAGraph] = None
        self.out = None
        self.lr = None
        self.captures = 0
        self.fp = None
        self.owners: List = []
        self.keys = None

    def _opt(self):
        return self.opt_fn() if self.opt_fn is not None else None

    def invalidate(self):
        """Drop the captured graph(s): the next call captures anew (after no further eager steps)."""
        self.graph = None
        if hasattr(self, "graphs"):
            self.graphs = None

    def _lr(self):
        """The host learning rates baked into a capture: none for an optimizer that keeps them on the device."""
        o = self._opt()
        if o is None or hasattr(o, "sync_device_scalars"):
            return None
        return tuple(g["lr"] for g in o.param_groups)

    def _keys(self):
        return tuple(o.graph_key() for o in self.owners)

    def _stale(self, captured) -> bool:
        return captured is None or self._lr() != self.lr or self._keys() != self.keys

    def _sync_owners(self):
        for o in self.owners:
            o.sync_device_scalars()

    def _fingerprint(self):
        """Identities / addresses of the device state a captured step reads and writes."""
        o = self._opt()
        if o is None:
            return None

        def ptr(t):
            return None if t is None else t.data_ptr()
        fp = [id(o), id(getattr(o, "_flat", None)), getattr(o, "_nseg", None)]
        fp += [ptr(getattr(o, k, None)) for k in ("exp_avg", "exp_avg_sq", "_steps", "_seg_start", "partial",
                                                  "_skipped", "last_norm")]
        model = getattr(o, "model", None)
        if model is not None:
            fp.append(tuple(id(p) for p in model.parameters() if p.requires_grad))
            for m in model.modules():
                S = m.__dict__.get("_hiseg_train")
                if S is not None:
                    fp += [id(m), id(S), id(S.flat), S.dtype, ptr(S.table), len(S.entries)]
                sync = m.__dict__.get("_hiseg_grad_sync")
                if sync is not None:   # a gradient exchange enabled after the capture must be captured too
                    fp += [id(sync), ptr(sync.state.flat.grad) if sync.state is not None else None]
        return tuple(fp)

    def __call__(self):
        self.calls += 1
        if self.graph is not None and self._fingerprint() != self.fp:
            # the optimizer or the model's flat layout / packing table was re-allocated since the capture
            self.graph, self.calls = None, 1
        if self.calls <= self.eager:
            s = role_stream("warm")   # the warm-up side stream (hiseg.streams: one per process, not per call)
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                out = self.fn()
            torch.cuda.current_stream().wait_stream(s)
            return out
        if self._stale(self.graph):
            self.graph = None
            torch.cuda.synchronize()
            before = self._fingerprint()
            g = torch.cuda.CUDAGraph()
            # thread-local capture: another thread's CUDA calls (a process group's watchdog, a data loader) are not
            # a capture error; the step itself issues no torch.distributed call (hiseg.comm)
            with _CaptureOwners() as owners:
                with torch.cuda.graph(g, stream=role_stream("capture"), capture_error_mode="thread_local"):
                    self.out = self.fn()
            self.owners, self.keys = owners, tuple(o.graph_key() for o in owners)
            self.fp = self._fingerprint()
            if self.fp != before:
                raise RuntimeError("GraphedStep: the step re-allocated optimizer / model state while it was being "
                                   "captured; run more eager steps first (GraphedStep(..., eager=N))")
            self.graph, self.lr = g, self._lr()
            self.captures += 1
        self._sync_owners()
        self.graph.replay()
        o = self._opt()
        bump = getattr(o, "_bump", None)
        if bump:
            torch.autograd.graph.increment_version(bump)
        return self.out


def _branch_priority() -> str:
    """HISEG_BRANCH_PRIO (read per call): "head" -- GraphedBranchStep replays its head and tail graphs on the
    high-priority stream; "branch" -- the branch graph there instead of the side stream; unset: neither (A/B)."""
    return os.environ.get("HISEG_BRANCH_PRIO", "")


class GraphedBranchStep(GraphedStep):
    """GraphedStep for a step that opens with two independent branches: ``branch_fn`` on the side stream (the frozen
    distillation teacher's forward), ``head_fn`` on the caller's stream beside it (the student's forward), then
    ``tail_fn`` once both are done (loss, backward, optimizer; it returns the step's outputs).  The functions pass
    values through the caller's closures.

    Why three graphs instead of one (round 5, profiles/r5_distill_branches.txt): a replayed graph's executor enqueues
    the whole node list of its launch queue -- the first-captured branch and everything after the join -- before the
    other branch's nodes (2.5 ms of host enqueue per distillation step against 0.5 ms here).  Here the branch graph
    is launched on the side stream first, the head graph on the caller's stream right after it, and the tail graph
    behind an event of the side stream.  Eager steps run the same functions on the same streams, so results equal a
    single-graph GraphedStep of the composed step bit for bit.

    ``handoff_fn`` given: the branch runs one step ahead (software pipelining; valid for a branch that reads no
    state the step updates -- the frozen, eval-mode teacher).  Call k launches the branch for step k+1, which then
    overlaps step k's head AND tail; the first call also runs the branch for step 0 first.  ``handoff_fn`` runs on
    the caller's stream at the start of every call, after the branch launched by the previous call has finished and
    before the next one starts: it moves the branch's result into the buffer the tail reads (e.g. ``t.copy_(t_next)``)
    and stages the branch's next input.  Same kernels on the same inputs: the results equal the unpipelined step's."""

    def __init__(self, branch_fn: Callable, head_fn: Callable, tail_fn: Callable,
                 optimizer_fn: Optional[Callable] = None, eager: int = 2, handoff_fn: Optional[Callable] = None):
        super().__init__(tail_fn, optimizer_fn, eager)
        self.branch_fn, self.head_fn, self.handoff_fn = branch_fn, head_fn, handoff_fn
        self.graphs = None
        self._ev = None
        self._primed = False

    def __call__(self):
        self.calls += 1
        if self.graphs is not None and self._fingerprint() != self.fp:
            self.graphs, self.calls = None, 1
        main = torch.cuda.current_stream()
        side = role_stream("teacher")
        if self._ev is None:
            self._ev = torch.cuda.Event()
        piped = self.handoff_fn is not None
        if piped:
            if not self._primed:   # the branch for the first step
                side.wait_stream(main)
                with torch.cuda.stream(side):
                    self.branch_fn()
                self._ev.record(side)
                self._primed = True
            main.wait_event(self._ev)
            self.handoff_fn()
        if self.calls <= self.eager:
            s = role_stream("warm")
            s.wait_stream(main)
            side.wait_stream(main)
            with torch.cuda.stream(side):
                self.branch_fn()
            self._ev.record(side)
            with torch.cuda.stream(s):
                self.head_fn()
                if not piped:
                    s.wait_stream(side)
                out = self.fn()
            main.wait_stream(s)
            return out
        if self._stale(self.graphs):
            self.graphs = None
            torch.cuda.synchronize()
            before = self._fingerprint()
            gb, gh, gt = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
            with _CaptureOwners() as owners:
                with torch.cuda.graph(gb, stream=side, capture_error_mode="thread_local"):
                    self.branch_fn()
                with torch.cuda.graph(gh, stream=role_stream("capture"), capture_error_mode="thread_local"):
                    self.head_fn()
                with torch.cuda.graph(gt, stream=role_stream("capture"), capture_error_mode="thread_local"):
                    self.out = self.fn()
            self.owners, self.keys = owners, tuple(o.graph_key() for o in owners)
            self.fp = self._fingerprint()
            if self.fp != before:
                raise RuntimeError("GraphedBranchStep: the step re-allocated optimizer / model state while it was "
                                   "being captured; run more eager steps first")
            self.graphs, self.lr = (gb, gh, gt), self._lr()
            self.captures += 1
        gb, gh, gt = self.graphs
        self._sync_owners()   # on the caller's stream: before the head / tail graphs that read them
        prio = _branch_priority()
        if prio == "branch":   # the branch replayed on the high-priority stream instead of the side stream
            side = role_stream("priority")
        side.wait_stream(main)   # the previous step's tail (or this step's handoff) is done with the branch buffers
        with torch.cuda.stream(side):
            gb.replay()
        self._ev.record(side)
        if prio == "head":
            # the head and tail -- the step's critical path -- replayed on the high-priority stream, the branch
            # filling what they leave (event-ordered with the caller's stream on both sides)
            hp = role_stream("priority")
            hp.wait_stream(main)
            with torch.cuda.stream(hp):
                gh.replay()
                if not piped:
                    hp.wait_event(self._ev)
                gt.replay()
            main.wait_stream(hp)
        else:
            gh.replay()
            if not piped:
                main.wait_event(self._ev)
            gt.replay()
        o = self._opt()
        bump = getattr(o, "_bump", None)
        if bump:
            torch.autograd.graph.increment_version(bump)
        return self.out

    def drain(self):
        """Wait (on the caller's stream) for the branch a pipelined step launched ahead."""
        if self._ev is not None:
            torch.cuda.current_stream().wait_event(self._ev)
