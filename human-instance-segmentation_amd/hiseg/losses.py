"""RefinedHierarchicalLoss on libhiseg (advanced/hierarchical_segmentation_refinement.py:807-1068 over
advanced/hierarchical_segmentation.py:150-395 and losses.py:9-88).

Same constructor, same call ``loss_fn(pred, target, aux_outputs) -> (total, loss_dict)`` and the same
loss-dict keys as the reference.  The forward (targets rasterisation, dynamic class weights with their EMA,
every loss term, clamps) and the backward run as HIP kernels (include/hiseg_loss.h); the EMA state lives on
the device, so a step performs no host synchronisation.  ``loss_dict`` values are materialised lazily: the
first access copies the 15 device scalars to the host once (the reference calls ``.item()`` per term).
"""
from __future__ import annotations

import ctypes
from collections.abc import Mapping
from typing import Dict, Optional, Tuple

import numpy as np
import torch
import torch.nn as nn

from . import _lib as L

_OUT_KEYS = ["total_loss", "bg_fg_loss", "target_nontarget_loss", "final_loss", "consistency_loss", "dice_loss",
             "boundary_aware", "contour", "distance_transform", "aux_fg_accuracy", "aux_fg_iou", "bg_weight",
             "fg_weight", "target_weight", "nontarget_weight"]


class LazyLossDict(Mapping):
    """dict[str, float] view of the device loss outputs; one device->host copy on first access."""

    def __init__(self, out: torch.Tensor, keys, extra: Dict[str, float]):
        self._out, self._keys, self._extra = out, keys, extra
        self._vals: Optional[Dict[str, float]] = None

    def _materialise(self, host=None) -> Dict[str, float]:
        """``host``: the device values already copied (hiseg.metrics.evaluate_model copies every batch's
        values in one transfer at the end of the loop)."""
        if self._vals is None:
            if host is None:
                host = self._out.detach().cpu().tolist()
            v = {"bg_fg_loss": host[1], "target_nontarget_loss": host[2], "final_loss": host[3],
                 "consistency_loss": host[4], "total_loss": host[0], "ce_loss": host[3], "dice_loss": host[5],
                 "aux_fg_bg_loss": host[1], "aux_fg_accuracy": host[9], "aux_fg_iou": host[10],
                 "bg_weight": host[11], "fg_weight": host[12], "target_weight": host[13],
                 "nontarget_weight": host[14]}
            # total_loss of the reference's base dict is the base loss before the refinement terms
            v["total_loss"] = host[15] if len(host) > 15 else host[0]
            for k in self._keys:
                if k == "boundary_aware":
                    v[k] = host[6]
                elif k == "contour":
                    v[k] = host[7]
                elif k == "distance_transform":
                    v[k] = host[8]
            v.update(self._extra)
            self._vals = v
        return self._vals

    def __getitem__(self, k):
        return self._materialise()[k]

    def __iter__(self):
        return iter(self._materialise())

    def __len__(self):
        return len(self._materialise())

    def copy(self):
        return dict(self._materialise())


class _LossFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, handle, pred, bgfg, tn, cont, dist, target):
        lib = L.lib()
        cfg: L.LossCfg = handle["cfg"]
        N, _, H, W = pred.shape
        dev = pred.device
        ws = torch.empty(int(lib.hiseg_loss_ws(N, H, W)), dtype=torch.float32, device=dev)
        out = torch.empty(L.LOSS_NOUT + 1, dtype=torch.float32, device=dev)
        st = handle["state"]
        counts = None
        if handle.get("count_sync") is not None:   # data parallel: class weights from the counts of all ranks
            counts = torch.empty(4, dtype=torch.float64, device=dev)
            L.check(lib.hiseg_loss_fwd_begin(ctypes.byref(cfg), N, H, W, target.data_ptr(), ws.data_ptr(),
                                             counts.data_ptr(), L.stream_ptr()), "loss_fwd_begin")
            handle["count_sync"](counts)
        else:
            L.check(lib.hiseg_loss_fwd_begin(ctypes.byref(cfg), N, H, W, target.data_ptr(), ws.data_ptr(), None,
                                             L.stream_ptr()), "loss_fwd_begin")
        L.check(lib.hiseg_loss_fwd_end(ctypes.byref(cfg), N, H, W, pred.data_ptr(), bgfg.data_ptr(), tn.data_ptr(),
                                       cont.data_ptr() if cont is not None else None,
                                       dist.data_ptr() if dist is not None else None, target.data_ptr(),
                                       counts.data_ptr() if counts is not None else None, st.data_ptr(),
                                       ws.data_ptr(), out.data_ptr(), L.stream_ptr()), "loss_fwd")
        ctx.save_for_backward(pred, bgfg, tn, cont, dist, target, ws)
        ctx.cfg = cfg
        ctx.mark_non_differentiable(out)
        handle["out"] = out
        return out[0].clone(), out

    @staticmethod
    def backward(ctx, g_total, _g_out):
        lib = L.lib()
        pred, bgfg, tn, cont, dist, target, ws = ctx.saved_tensors
        N, _, H, W = pred.shape
        dp, db, dt = torch.empty_like(pred), torch.empty_like(bgfg), torch.empty_like(tn)
        dc = torch.empty_like(cont) if cont is not None else None
        dd = torch.empty_like(dist) if dist is not None else None
        g = g_total.contiguous().float()
        L.check(lib.hiseg_loss_bwd(ctypes.byref(ctx.cfg), N, H, W, pred.data_ptr(), bgfg.data_ptr(), tn.data_ptr(),
                                   cont.data_ptr() if cont is not None else None,
                                   dist.data_ptr() if dist is not None else None, target.data_ptr(), ws.data_ptr(),
                                   g.data_ptr(), dp.data_ptr(), db.data_ptr(), dt.data_ptr(),
                                   dc.data_ptr() if dc is not None else None,
                                   dd.data_ptr() if dd is not None else None, L.stream_ptr()), "loss_bwd")
        return None, dp, db, dt, dc, dd, None


class RefinedHierarchicalLoss(nn.Module):
    """Hierarchical loss with refinement terms (refinement.py:807-984); arguments as the reference."""

    def __init__(self, bg_weight: float = 1.5, fg_weight: float = 1.5, target_weight: float = 1.2,
                 consistency_weight: float = 0.3, use_dynamic_weights: bool = True, dice_weight: float = 1.0,
                 ce_weight: float = 1.0, active_contour_weight: float = 0.01, boundary_aware_weight: float = 0.01,
                 contour_loss_weight: float = 0.01, distance_loss_weight: float = 0.01,
                 use_active_contour_loss: bool = False, use_boundary_aware_loss: bool = False,
                 use_contour_detection: bool = False, use_distance_transform: bool = False,
                 base_mask_size: Tuple[int, int] = (64, 48), auto_adjust_contour_weight: bool = True):
        super().__init__()
        if use_active_contour_loss:
            raise NotImplementedError("active_contour_loss is not used by the measured configs (SURVEY.md §8a L1)")
        self.bg_weight, self.fg_weight, self.target_weight = bg_weight, fg_weight, target_weight
        self.consistency_weight, self.use_dynamic_weights = consistency_weight, use_dynamic_weights
        self.dice_weight, self.ce_weight = dice_weight, ce_weight
        self.boundary_aware_weight, self.contour_loss_weight = boundary_aware_weight, contour_loss_weight
        self.distance_loss_weight = distance_loss_weight
        self.use_boundary_aware_loss, self.use_contour_detection = use_boundary_aware_loss, use_contour_detection
        self.use_distance_transform = use_distance_transform
        self.base_mask_size = base_mask_size
        self.auto_adjust_contour_weight = auto_adjust_contour_weight
        self.base_resolution = base_mask_size[0] * base_mask_size[1]
        self._state: Optional[torch.Tensor] = None   # device EMA state (double[8])
        self.count_sync = None   # callable(counts double[4]) summing the class pixel counts over ranks, or None

    def _cfg(self, H: int, W: int, has_c: bool, has_d: bool) -> Tuple[L.LossCfg, Optional[float]]:
        c = L.LossCfg()
        c.bg_weight, c.fg_weight, c.target_weight = self.bg_weight, self.fg_weight, self.target_weight
        c.consistency_weight, c.dice_weight, c.ce_weight = self.consistency_weight, self.dice_weight, self.ce_weight
        c.boundary_aware_weight, c.distance_weight = self.boundary_aware_weight, self.distance_loss_weight
        adj = None
        if self.use_contour_detection and has_c:
            if self.auto_adjust_contour_weight:   # refinement.py:951-963
                adj = max(0.001, min(self.contour_loss_weight * float(np.sqrt(self.base_resolution / (H * W))), 0.5))
            else:
                adj = self.contour_loss_weight
        c.contour_weight = adj if adj is not None else 0.0
        c.use_dynamic_weights = int(self.use_dynamic_weights)
        c.use_boundary_aware = int(self.use_boundary_aware_loss)
        c.use_contour = int(adj is not None)
        c.use_distance = int(self.use_distance_transform and has_d)
        ew = max(1, int(np.sqrt(H * W / 3072) * 1.5))   # refinement.py:1018-1027
        c.contour_ks = 2 * ew - 1 if ew > 1 else 1
        return c, adj

    def forward(self, pred: torch.Tensor, target: torch.Tensor,
                aux_outputs: Optional[Dict[str, torch.Tensor]] = None):
        if not pred.is_cuda:
            raise RuntimeError("hiseg RefinedHierarchicalLoss runs on the GPU only (got a CPU tensor)")
        aux = aux_outputs or {}
        N, C, H, W = pred.shape
        assert C == 3 and tuple(target.shape) == (N, H, W)
        lib = L.lib()
        if self._state is None or self._state.device != pred.device:
            self._state = torch.empty(8, dtype=torch.float64, device=pred.device)
            L.check(lib.hiseg_loss_state_init(self._state.data_ptr(), L.stream_ptr()), "loss_state_init")
        cont = aux.get("contours") if self.use_contour_detection else None
        dist = aux.get("distance_map") if self.use_distance_transform else None
        cfg, adj = self._cfg(H, W, cont is not None, dist is not None)

        def f32(t):
            return None if t is None else t.float().contiguous()
        handle = {"cfg": cfg, "state": self._state, "count_sync": self.count_sync}
        total, out = _LossFunction.apply(handle, f32(pred), f32(aux["bg_fg_logits"]),
                                         f32(aux["target_nontarget_logits"]), f32(cont), f32(dist),
                                         target.to(device=pred.device, dtype=torch.int64).contiguous())
        keys = []
        if self.use_boundary_aware_loss:
            keys.append("boundary_aware")
        if adj is not None:
            keys.append("contour")
        if dist is not None:
            keys.append("distance_transform")
        extra = {"contour_weight": adj} if adj is not None else {}
        return total, LazyLossDict(out, keys, extra)
