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
from typing import Optional

import torch

from . import _lib as L


def flat_params_of(model: torch.nn.Module):
    S = model.__dict__.get("_hiseg_train")
    if S is None:
        raise RuntimeError("hiseg optimiser: run one training forward first (it lays the parameters out flat)")
    return S.flat


class FusedAdamW(torch.optim.Optimizer):
    """AdamW + optional global-norm clipping over a model's FlatParams (param_groups: one, as the reference).

    A ``torch.optim.Optimizer`` over the same parameter list as the reference's
    ``torch.optim.AdamW(model.parameters(), ...)`` (train_advanced.py:1111-1118), so torch's LR schedulers
    (CosineAnnealingLR, :1126-1131) drive its ``param_groups[0]['lr']`` and ``state_dict()`` /
    ``load_state_dict()`` use torch.optim.AdamW's layout (per-parameter ``step`` / ``exp_avg`` /
    ``exp_avg_sq`` keyed by the index in that list): optimizer states of reference checkpoints load here and
    vice versa (train_advanced.py:1226, 1592-1599).  The moments themselves live in two flat device buffers."""

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
        self.betas, self.eps, self.weight_decay = betas, eps, weight_decay
        self.max_grad_norm = max_grad_norm
        self.step_count = 0
        self._flat = None
        self.exp_avg = self.exp_avg_sq = None
        self.partial = None
        self.last_norm: Optional[torch.Tensor] = None
        self._pending_state = None
        self._bump = None

    @property
    def lr(self) -> float:
        return self.param_groups[0]["lr"]

    def _init(self):
        if self._flat is None:
            self._flat = flat_params_of(self.model)
            f = self._flat
            self._range = (0, f.numel)
            if self._subset is not None:
                spans = sorted(f.offsets[id(p)] for p in self._subset)
                b, e = spans[0][0], spans[-1][0] + spans[-1][1]
                covered = sum(k for _, k in spans)
                if covered != e - b:
                    raise ValueError("FusedAdamW(params=...): the parameters are not contiguous in the flat layout")
                self._range = (b, e)
            n = self._range[1] - self._range[0]
            self.exp_avg = torch.zeros(n, dtype=torch.float32, device=f.data.device)
            self.exp_avg_sq = torch.zeros_like(self.exp_avg)
            self.partial = torch.empty(L.lib().hiseg_optim_blocks(), dtype=torch.float32, device=f.data.device)
            self.last_norm = torch.zeros(1, dtype=torch.float32, device=f.data.device)
            if self._pending_state is not None:
                sd, self._pending_state = self._pending_state, None
                self._load_moments(sd)

    def zero_grad(self, set_to_none: bool = False):
        self._init()
        self._flat.grad.zero_()
        self._flat.attach_grads()

    @torch.no_grad()
    def step(self, closure=None):
        """Returns the pre-clip total gradient norm as a device tensor (like clip_grad_norm_)."""
        if closure is not None:
            raise NotImplementedError("FusedAdamW.step: closures are not supported (the reference passes none)")
        self._init()
        f = self._flat
        f.prepare_backward()  # adopt any .grad tensors replaced since the backward
        lib = L.lib()
        self.step_count += 1
        g0 = self.param_groups[0]
        lr = g0["lr"]
        b1, b2 = g0["betas"]
        eps, wd = g0["eps"], g0["weight_decay"]
        bc1, bc2 = 1.0 - b1 ** self.step_count, 1.0 - b2 ** self.step_count
        s = L.stream_ptr()
        clip = self.max_grad_norm is not None and self.max_grad_norm > 0
        b, e = self._range
        gp, dp = f.grad.data_ptr() + 4 * b, f.data.data_ptr() + 4 * b
        L.check(lib.hiseg_grad_norm_partials(gp, e - b, self.partial.data_ptr(), s), "grad_norm")
        L.check(lib.hiseg_adamw_step(dp, gp, self.exp_avg.data_ptr(),
                                     self.exp_avg_sq.data_ptr(), e - b, float(lr), float(b1), float(b2),
                                     float(eps), float(wd), float(bc1), float(bc2),
                                     self.partial.data_ptr(), float(self.max_grad_norm) if clip else 0.0,
                                     self.last_norm.data_ptr(), s), "adamw_step")
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
        b, e = self._range
        out = []
        for i, p in enumerate(self.param_groups[0]["params"]):
            if id(p) in f.offsets:
                off, k = f.offsets[id(p)]
                if b <= off and off + k <= e:
                    out.append((i, p, off - b))
        return out

    def state_dict(self):
        self._init()
        state = {}
        if self.step_count > 0:
            for i, p, off in self._slots():
                k = p.numel()
                state[i] = {"step": torch.tensor(float(self.step_count)),
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
        if self._flat is None and self.model.__dict__.get("_hiseg_train") is not None:
            self._init()
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
        steps = set()
        st = sd["state"]
        for i, p, off in self._slots():
            ent = st.get(i, st.get(str(i)))
            if ent is None:
                continue
            k = p.numel()
            self.exp_avg[off:off + k].copy_(ent["exp_avg"].reshape(-1))
            self.exp_avg_sq[off:off + k].copy_(ent["exp_avg_sq"].reshape(-1))
            steps.add(int(float(ent["step"])))
        if len(steps) > 1:
            raise ValueError(f"per-parameter AdamW steps differ ({sorted(steps)}); one step count is kept")
        self.step_count = steps.pop() if steps else 0


def cosine_lr(base_lr: float, epoch: int, total_epochs: int, min_lr: float = 1e-6) -> float:
    """CosineAnnealingLR(T_max=num_epochs, eta_min=min_lr) value at an epoch (train_advanced.py:1126-1131)."""
    return min_lr + (base_lr - min_lr) * 0.5 * (1 + math.cos(math.pi * epoch / total_epochs))
