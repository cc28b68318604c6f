"""The process's side streams, one fixed set per device.

HIP binds a stream to a hardware queue when the stream first carries a command, at most GPU_MAX_HW_QUEUES (4 on
the MI355X boxes) queues per priority, and streams beyond that share a queue (the least-used one, AMD_LOG_LEVEL=3:
`acquireQueue` / `Selected queue refCount`).  Two streams on one in-order queue cannot overlap.  When every component
took the next stream of torch's pool, a process that had run the inference leg (UNet + head streams) and a train
leg (warm-up + capture streams) held five or more normal-priority streams, and the distillation step's teacher
branch shared a queue with the student's: 16.4 ms per replayed step instead of 8.9, its unfrozen form 32.5 instead of
16.2, in whatever order the bench legs ran (profiles/r5_leg_order.txt).  So the process uses at most four
normal-priority streams, each with a queue of its own whatever ran before:

* the caller's stream (the null stream; every graph is replayed there);
* ``side``: the one concurrent branch a step forks -- StreamPipelinedExport's UNet stream, DistillationUNetWrapper's
  teacher stream (one component at a time uses it; two users would only serialise, never reorder: every use is
  event-ordered);
* ``aux``: GraphedStep's eager warm-up steps and its capture stream (never concurrent with anything);
* ``comm``: GradBucketSync's all-reduces (world > 1 only).

plus ``head``, the high-priority stream of the inference head (its own priority level, so its own queue; also the
``priority`` role: GraphedBranchStep's head and tail with HISEG_BRANCH_PRIO=head, or its branch with =branch).  The
roles map onto those streams (``ROLE``); a stream is created on the first request for it, untouched (bound to a queue
on its first real command, so a process that never uses one never binds it)."""
from __future__ import annotations

from typing import Dict, Optional

import torch

ROLE = {"unet": "side", "teacher": "side", "warm": "aux", "capture": "aux", "comm": "comm", "head": "head",
        "head_normal": "head_normal", "priority": "head"}
_PRIORITY = {"head": -1}
_by_device: Dict[int, Dict[str, torch.cuda.Stream]] = {}


def role_stream(role: str, device: Optional[torch.device] = None) -> torch.cuda.Stream:
    """The stream serving ``role`` on ``device`` (default: the current CUDA device).  ``head_normal`` (the head of a
    StreamPipelinedExport built with head_priority=False) is a fifth normal-priority stream, outside the budget."""
    if role not in ROLE:
        raise ValueError(f"unknown stream role {role!r} (one of {tuple(ROLE)})")
    if device is None:
        idx = torch.cuda.current_device()
    else:
        device = torch.device(device)
        idx = device.index if device.index is not None else torch.cuda.current_device()
    tab = _by_device.setdefault(idx, {})
    name = ROLE[role]
    s = tab.get(name)
    if s is None:
        s = tab[name] = torch.cuda.Stream(device=idx, priority=_PRIORITY.get(name, 0))
    return s
