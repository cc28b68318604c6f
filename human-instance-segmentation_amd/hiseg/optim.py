"""Fused optimiser step on the flat parameter space of a hiseg model.

Replaces the reference's ``clip_grad_norm_(model.parameters(), 1.0)`` + ``torch.optim.AdamW(lr=1e-4,
weight_decay=0.01)`` pair (train_advanced.py:733-740, 1111-1143): two launches over the contiguous
parameter / gradient / moment buffers (gradient-norm partials, then clip + AdamW), no host sync.
Arithmetic follows torch.optim.AdamW (decoupled weight decay, bias-corrected moments, eps outside the
square root) and clip_grad_norm_ (coef = min(1, max_norm / (norm + 1e-6)), gradients scaled in place).
``torch.optim.AdamW`` over the same parameters keeps working too: they are ordinary nn.Parameters.
"""
from __future__ import annotations

import math
from collections.abc import MutableMapping
from typing import Optional

import torch

from . import _lib as L
from . import graphs as _graphs


def flat_params_of(model: torch.nn.Module):
    S = model.__dict__.get("_hiseg_train")
    if S is None:
        raise RuntimeError("hiseg optimiser: run one training forward first (it lays the parameters out flat)")
    return S.flat


class _LiveState(MutableMapping):
    """``optimizer.state`` of a FusedAdamW: a live view of its flat moment buffers keyed by parameter, in
    torch.optim.AdamW's per-parameter form (``step`` CPU tensor, ``exp_avg`` / ``exp_avg_sq`` views).  Assigning
    ``new_opt.state[p] = old_opt.state[p]`` copies the moments in -- the reference's optimizer-state transfer
    when progressive unfreezing builds a new optimizer (train_distillation_staged.py:1537-1550) works unchanged
    between two FusedAdamW instances."""

    def __init__(self, opt: "FusedAdamW"):
        self._opt = opt
        self._pending = {}

    def _off(self, p):
        o = self._opt
        o._ensure(required=False)
        if o._flat is None:
            return None
        for _, q, off in o._slots():
            if q is p:
                return off
        return None

    def __getitem__(self, p):
        o = self._opt
        off = self._off(p)
        t = 0 if off is None else o._param_steps().get(id(p), 0)
        if t == 0:      # torch.optim.AdamW: no state before the parameter's first step
            raise KeyError(p)
        k = p.numel()
        return {"step": torch.tensor(float(t)), "exp_avg": o.exp_avg[off:off + k].view(p.shape),
                "exp_avg_sq": o.exp_avg_sq[off:off + k].view(p.shape)}

    def __setitem__(self, p, ent):
        o = self._opt
        if o._flat is None:
            o._ensure(required=False)
        if o._flat is None:      # no training forward yet: applied once the flat layout exists
            self._pending[p] = ent
            return
        off = self._off(p)
        if off is None:
            raise KeyError("FusedAdamW.state: parameter is not optimised by this optimizer")
        k = p.numel()
        with torch.no_grad():
            o.exp_avg[off:off + k].copy_(ent["exp_avg"].reshape(-1))
            o.exp_avg_sq[off:off + k].copy_(ent["exp_avg_sq"].reshape(-1))
        steps = o._param_steps()
        steps[id(p)] = int(float(ent["step"]))
        o._set_steps(steps)

    def __delitem__(self, p):
        off = self._off(p)
        if off is None:
            raise KeyError(p)
        k = p.numel()
        self._opt.exp_avg[off:off + k].zero_()
        self._opt.exp_avg_sq[off:off + k].zero_()

    def __iter__(self):
        o = self._opt
        o._ensure(required=False)
        if o._flat is None:
            return iter(())
        steps = o._param_steps()
        return iter([q for _, q, _ in o._slots() if steps.get(id(q), 0) > 0])

    def __len__(self):
        return sum(1 for _ in self)

    def __bool__(self):
        return len(self) > 0

    def apply_pending(self):
        pend, self._pending = self._pending, {}
        for p, ent in pend.items():
            self[p] = ent


class FusedAdamW(torch.optim.Optimizer):
    """AdamW + optional global-norm clipping over a model's FlatParams (param_groups: one, as the reference).

    A ``torch.optim.Optimizer`` over the same parameter list as the reference's
    ``torch.optim.AdamW(model.parameters(), ...)`` (train_advanced.py:1111-1118), so torch's LR schedulers
    (CosineAnnealingLR, :1126-1131) drive its ``param_groups[0]['lr']`` and ``state_dict()`` /
    ``load_state_dict()`` use torch.optim.AdamW's layout (per-parameter ``step`` / ``exp_avg`` /
    ``exp_avg_sq`` keyed by the index in that list): optimizer states of reference checkpoints load here and
    vice versa (train_advanced.py:1226, 1592-1599).  The moments themselves live in two flat device buffers;
    ``optimizer.state`` is a live per-parameter view of them (_LiveState).

    Non-finite steps are skipped on the device, as the reference never applies them (GradScaler.step on the AMP
    path, train_advanced.py:751-762; the NaN loss / NaN gradient checks of the fp32 path, :814-832): when the
    gradient norm is NaN or Inf the parameters, gradients and moments stay untouched, the step count (kept on the
    device, so no host sync per step) does not advance and ``skipped_steps`` counts the skip.  Under
    hiseg.distributed the gradients are averaged over the ranks before the step, so a non-finite gradient on any
    rank makes every rank skip the same step.

    Inf-only gradients are skipped on purpose too, although the reference's fp32 path (train_advanced.py:815-832)
    checks only for NaN loss / NaN gradients and would apply such a step (clip_grad_norm_ turns it into NaN).

    Step counts are per parameter, as in torch.optim.AdamW: the device keeps one count per run of parameters
    that share it (segments of the flat layout, hiseg_adamw_step_segmented).  When the model's flat layout is
    rebuilt (a new trainable set after ``unfreeze_encoder_blocks``, a dtype change), the next ``zero_grad`` /
    ``step`` re-binds to the new buffers and carries every kept parameter's moments and step count over; a
    parameter new to the optimizer starts at step 0 with zero moments (the reference's new optimizer at
    progressive unfreezing, train_distillation_staged.py:1531-1552)."""

    def __init__(self, model: torch.nn.Module, lr: float = 1e-4, betas=(0.9, 0.999), eps: float = 1e-8,
                 weight_decay: float = 0.01, max_grad_norm: Optional[float] = 1.0, params=None):
        """``params`` (optional) restricts the step -- and the clipping norm -- to a subset of the trainable
        parameters that is contiguous in the flat layout, e.g. ``unet.decoder.parameters()`` of the
        distillation student (train_distillation_staged.py:1298-1305 optimises and clips the decoder only)."""
        self.model = model
        self._subset = None if params is None else [p for p in params]
        plist = list(model.parameters()) if self._subset is None else self._subset
        super().__init__(plist, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay, amsgrad=False,
                                     maximize=False, foreach=None, capturable=False, differentiable=False,
                                     fused=None, decoupled_weight_decay=True))
        self.state = _LiveState(self)
        self.betas, self.eps, self.weight_decay = betas, eps, weight_decay
        self.max_grad_norm = max_grad_norm
        self._flat = None
        self.exp_avg = self.exp_avg_sq = None
        self.partial = None
        self.last_norm: Optional[torch.Tensor] = None
        self._steps: Optional[torch.Tensor] = None     # device step counts [2][nseg] (hiseg_adamw_step_segmented)
        self._seg_start: Optional[torch.Tensor] = None  # int64 [nseg + 1] segment bounds in the moment buffers
        self._nseg = 0
        self._slot_list = None
        self._parity = 0
        self._host_steps = 0
        self._skipped: Optional[torch.Tensor] = None
        self._pending_state = None
        self._bump = None
        self._hyper: Optional[torch.Tensor] = None    # device f32 [lr, 1 - lr wd] (hiseg_adamw_step_segmented_dev)
        self._hyper_vals = None

    # ---------------------------------------------------------------- device scalars (hiseg.graphs)
    def sync_device_scalars(self):
        """Write the current learning rate and decay factor into the device buffer the step kernel reads, when they
        changed (a fill on the current stream: no host sync); GraphedStep calls this before every replay."""
        g0 = self.param_groups[0]
        lr = float(g0["lr"])
        vals = (lr, 1.0 - lr * float(g0["weight_decay"]))   # rounded to f32 by the fill, as by a c_float argument
        dev = self._flat.data.device if self._flat is not None else None
        if self._hyper is None or (dev is not None and self._hyper.device != dev):
            self._hyper = torch.empty(2, dtype=torch.float32, device=dev)
            self._hyper_vals = None
        if vals != self._hyper_vals:
            self._hyper[0].fill_(vals[0])
            self._hyper[1].fill_(vals[1])
            self._hyper_vals = vals

    def graph_key(self):
        return (self._hyper.data_ptr() if self._hyper is not None else None,)

    @property
    def lr(self) -> float:
        return self.param_groups[0]["lr"]

    @property
    def step_count(self) -> int:
        """Applied (not skipped) steps of the longest-trained parameter (torch.optim.AdamW's per-parameter
        ``step``: see ``param_steps``); reads the device counters (a host sync) once the buffers exist."""
        if self._steps is None:
            return self._host_steps
        n = self._nseg
        return int(self._steps[self._parity * n:(self._parity + 1) * n].max().item())

    @step_count.setter
    def step_count(self, v: int):
        if self._steps is None:
            self._host_steps = int(v)
        else:
            self._set_steps({id(p): int(v) for _, p, _ in self._slots()})

    def param_steps(self):
        """{parameter: step count} (torch.optim.AdamW's state[p]['step']) for every parameter with moments here."""
        steps = self._param_steps()
        return {p: steps.get(id(p), 0) for _, p, _ in self._slots()}

    def _param_steps(self):
        """{id(parameter): step} from the device segments (host sync)."""
        if self._steps is None:
            return {}
        n = self._nseg
        counts = self._steps[self._parity * n:(self._parity + 1) * n].tolist()
        bounds = self._seg_start.tolist()
        out = {}
        s = 0
        for _, p, off in sorted(self._slots(), key=lambda e: e[2]):
            while s + 1 < n and off >= bounds[s + 1]:
                s += 1
            out[id(p)] = int(counts[s])
        return out

    def _set_steps(self, steps):
        """Per-parameter step counts (dict id(p) -> t) -> device segments: maximal runs of the flat layout whose
        parameters share a count.  Rewrites the buffers in place when the segment count is unchanged."""
        bounds, counts = [0], []
        for _, p, off in sorted(self._slots(), key=lambda e: e[2]):
            t = int(steps.get(id(p), 0))
            if counts and counts[-1] == t:
                continue
            if counts:
                bounds.append(off)
            counts.append(t)
        if not counts:
            counts = [0]
        bounds.append(self._range[1] - self._range[0])
        if len(counts) > L.lib().hiseg_adamw_max_segments():
            raise ValueError(f"FusedAdamW: {len(counts)} distinct per-parameter step runs exceed the device table")
        dev = self._flat.data.device
        seg = torch.tensor(bounds, dtype=torch.int64)
        st = torch.tensor(counts + counts, dtype=torch.int32)
        if self._steps is not None and self._nseg == len(counts):
            self._seg_start.copy_(seg)
            self._steps.copy_(st)
        else:
            self._seg_start, self._steps = seg.to(dev), st.to(dev)
            self._nseg = len(counts)

    @property
    def skipped_steps(self) -> int:
        """Steps skipped because the gradient norm was not finite (host sync)."""
        return 0 if self._skipped is None else int(self._skipped.item())

    # ------------------------------------------------------------------------------------- flat layout
    def _ensure(self, required: bool = True):
        S = self.model.__dict__.get("_hiseg_train")
        if S is None:
            if self._flat is None and required:
                flat_params_of(self.model)   # raises with the message
            return
        f = S.flat
        if self._flat is None:
            self._bind(f, carried=None)
        elif f is not self._flat:
            self._rebind(f)

    def _range_of(self, f):
        if self._subset is None:
            return (0, f.numel)
        spans = sorted(f.offsets[id(p)] for p in self._subset if id(p) in f.offsets)
        if not spans:
            raise ValueError("FusedAdamW(params=...): none of the parameters is trainable in the flat layout")
        b, e = spans[0][0], spans[-1][0] + spans[-1][1]
        covered = sum(k for _, k in spans)
        if covered != e - b:
            raise ValueError("FusedAdamW(params=...): the parameters are not contiguous in the flat layout")
        return (b, e)

    def _bind(self, f, carried):
        first = carried is None
        host_steps = self._host_steps
        self._flat = f
        self._slot_list = None
        self._range = self._range_of(f)
        n = self._range[1] - self._range[0]
        dev = f.data.device
        self.exp_avg = torch.zeros(n, dtype=torch.float32, device=dev)
        self.exp_avg_sq = torch.zeros_like(self.exp_avg)
        self.partial = torch.empty(L.lib().hiseg_optim_blocks(), dtype=torch.float32, device=dev)
        self.last_norm = torch.zeros(1, dtype=torch.float32, device=dev)
        skipped = 0 if self._skipped is None else int(self._skipped.item())
        self._steps = self._seg_start = None
        self._parity = 0
        self._skipped = torch.full((1,), skipped, dtype=torch.int32, device=dev)
        self._bump = None
        steps = {}
        for _, p, off in self._slots():
            ent = None if first else carried.get(id(p))
            if ent is not None:
                k = p.numel()
                self.exp_avg[off:off + k].copy_(ent[0])
                self.exp_avg_sq[off:off + k].copy_(ent[1])
            steps[id(p)] = host_steps if first else (ent[2] if ent is not None else 0)
        self._set_steps(steps)
        if self._pending_state is not None:
            sd, self._pending_state = self._pending_state, None
            self._load_moments(sd)
        self.state.apply_pending()

    def _rebind(self, f):
        """The model re-laid its trainable parameters (new FlatParams): keep every parameter's moments."""
        carried = {}
        steps = self._param_steps()
        for _, p, off in self._slots():
            k = p.numel()
            carried[id(p)] = (self.exp_avg[off:off + k].clone(), self.exp_avg_sq[off:off + k].clone(),
                              steps.get(id(p), 0))
        self._bind(f, carried)

    def zero_grad(self, set_to_none: bool = False):
        self._ensure()
        self._flat.grad.zero_()
        self._flat.attach_grads()

    @torch.no_grad()
    def step(self, closure=None):
        """Returns the pre-clip total gradient norm as a device tensor (like clip_grad_norm_); a non-finite norm
        means the step was skipped (class docstring)."""
        if closure is not None:
            raise NotImplementedError("FusedAdamW.step: closures are not supported (the reference passes none)")
        self._ensure()
        f = self._flat
        f.prepare_backward()  # adopt any .grad tensors replaced since the backward
        lib = L.lib()
        g0 = self.param_groups[0]
        b1, b2 = g0["betas"]
        eps = g0["eps"]
        s = L.stream_ptr()
        clip = self.max_grad_norm is not None and self.max_grad_norm > 0
        b, e = self._range
        gp, dp = f.grad.data_ptr() + 4 * b, f.data.data_ptr() + 4 * b
        L.check(lib.hiseg_grad_norm_partials(gp, e - b, self.partial.data_ptr(), s), "grad_norm")
        # lr and 1 - lr wd come from the device buffer: a captured step follows the schedule without a re-capture
        if torch.cuda.is_current_stream_capturing():
            if self._hyper is None:
                raise RuntimeError("FusedAdamW: the first step cannot be captured (run it eagerly first)")
            _graphs.note_device_scalars(self)
        else:
            self.sync_device_scalars()
        L.check(lib.hiseg_adamw_step_segmented_dev(dp, gp, self.exp_avg.data_ptr(), self.exp_avg_sq.data_ptr(), e - b,
                                                   self._hyper.data_ptr(), float(b1), float(b2), 1.0 - float(b1),
                                                   1.0 - float(b2), float(eps), self.partial.data_ptr(),
                                                   float(self.max_grad_norm) if clip else 0.0,
                                                   self.last_norm.data_ptr(), self._seg_start.data_ptr(), self._nseg,
                                                   self._steps.data_ptr(), self._parity, self._skipped.data_ptr(), s),
                "adamw_step")
        # the count stays in slot _parity (the library commits it): no host-side state changes per step, so the
        # whole step can be captured into a HIP graph (hiseg.graphs.GraphedStep)
        # the kernel wrote the parameters in place: bump their versions so plans packed from them (eval
        # forward, frozen-layer caches keyed by tensor version) are rebuilt
        if self._bump is None:
            self._bump = [p for _, p, _ in self._slots()]
        torch.autograd.graph.increment_version(self._bump)
        return self.last_norm

    # ---------------------------------------------------------------- torch.optim.AdamW state layout
    def _slots(self):
        """(index in the optimizer's parameter list, parameter, flat offset relative to the moment buffers)
        for every parameter whose moments this optimiser keeps."""
        f = self._flat
        plist = self.param_groups[0]["params"]
        key = (id(f), tuple(id(p) for p in plist))   # the list can change in place (parameters swapped)
        if self._slot_list is not None and self._slot_list[0] == key:
            return self._slot_list[1]
        b, e = self._range
        out = []
        for i, p in enumerate(plist):
            if id(p) in f.offsets:
                off, k = f.offsets[id(p)]
                if b <= off and off + k <= e:
                    out.append((i, p, off - b))
        self._slot_list = (key, out)
        return out

    def state_dict(self):
        self._ensure()
        state = {}
        steps = self._param_steps()
        for i, p, off in self._slots():
            t = steps.get(id(p), 0)
            if t > 0:
                k = p.numel()
                state[i] = {"step": torch.tensor(float(t)),
                            "exp_avg": self.exp_avg[off:off + k].view(p.shape).clone(),
                            "exp_avg_sq": self.exp_avg_sq[off:off + k].view(p.shape).clone()}
        groups = []
        for g in self.param_groups:
            d = {k: v for k, v in g.items() if k != "params"}
            d["params"] = list(range(len(g["params"])))
            groups.append(d)
        return {"state": state, "param_groups": groups}

    def load_state_dict(self, sd):
        """Accepts torch.optim.AdamW's state_dict (reference checkpoints) or this optimiser's own."""
        if "state" not in sd:   # legacy flat layout of earlier hiseg versions
            sd = {"state": {}, "param_groups": sd["param_groups"], "_flat": sd}
        g = sd["param_groups"][0]
        if len(g.get("params", self.param_groups[0]["params"])) != len(self.param_groups[0]["params"]):
            raise ValueError("loaded state dict has a different number of parameters than this optimizer")
        for k, v in g.items():
            if k != "params":
                self.param_groups[0][k] = v
        self._ensure(required=False)
        if self._flat is None:   # no training forward yet: applied when the flat layout exists
            self._pending_state = sd
        else:
            self._load_moments(sd)

    def _load_moments(self, sd):
        if "_flat" in sd:
            old = sd["_flat"]
            self.step_count = int(old["step"])
            self.exp_avg.copy_(old["exp_avg"])
            self.exp_avg_sq.copy_(old["exp_avg_sq"])
            return
        self.exp_avg.zero_()
        self.exp_avg_sq.zero_()
        steps = {}
        st = sd["state"]
        for i, p, off in self._slots():
            ent = st.get(i, st.get(str(i)))
            if ent is None:
                steps[id(p)] = 0
                continue
            k = p.numel()
            self.exp_avg[off:off + k].copy_(ent["exp_avg"].reshape(-1))
            self.exp_avg_sq[off:off + k].copy_(ent["exp_avg_sq"].reshape(-1))
            steps[id(p)] = int(float(ent["step"]))
        self._set_steps(steps)


def cosine_lr(base_lr: float, epoch: int, total_epochs: int, min_lr: float = 1e-6) -> float:
    """CosineAnnealingLR(T_max=num_epochs, eta_min=min_lr) value at an epoch (train_advanced.py:1126-1131)."""
    return min_lr + (base_lr - min_lr) * 0.5 * (1 + math.cos(math.pi * epoch / total_epochs))
