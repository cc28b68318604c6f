"""B7 -> B0 UNet knowledge distillation on libhiseg (advanced/unet_decoder_distillation.py,
train_distillation_staged.py).

Same surface as the reference module: ``UNetDistillationLoss`` (temperature schedule, adaptive
distillation weight, ``forward(student, teacher, masks) -> (total, loss_dict)``), ``UNetDecoderOnly``,
``DistillationUNetWrapper`` (student + frozen teacher, progressive encoder unfreezing) and
``create_unet_distillation_model``.  The loss terms, reductions and the gradient run as HIP kernels
(include/hiseg_distill.h); the schedule state stays on the host exactly as in the reference (it is
updated once per epoch), and ``loss_dict`` is materialised lazily (one device->host copy on first
access instead of the reference's five ``.item()`` calls).  The reference's NaN/Inf fallbacks are
reproduced on the device (:560-568, :650-659): a non-finite total becomes the task loss, else the MSE
term, else a constant 1.0 without a gradient, and the backward differentiates the value returned;
NaN terms are reported as 0.0 in loss_dict.  Pinned to the reference by the non-finite golden cases
(tests/golden/distill_loss.npz: NaN / Inf teacher, NaN student, with and without targets).
"""
from __future__ import annotations

import ctypes
import math
import os
from collections.abc import Mapping
from typing import Dict, Optional, Tuple

import numpy as np
import torch
import torch.nn as nn

from . import _lib as L
from . import graphs as _graphs

_DICT_KEYS = ("total_loss", "kl_loss", "mse_loss", "bce_loss", "dice_loss")


class _LazyDict(Mapping):
    def __init__(self, out: torch.Tensor, keys):
        self._out, self._keys, self._vals = out, keys, None

    def _get(self):
        if self._vals is None:
            host = self._out.detach().cpu().tolist()
            self._vals = {k: float(host[i]) for i, k in enumerate(_DICT_KEYS) if k in self._keys}
        return self._vals

    def __getitem__(self, k):
        return self._get()[k]

    def __iter__(self):
        return iter(self._get())

    def __len__(self):
        return len(self._get())

    def get(self, k, default=None):
        return self._get().get(k, default)


class _DistillLossFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, cfg, student, teacher, target, dev_scalars=None):
        lib = L.lib()
        B, _, H, W = student.shape
        dev = student.device
        ws = torch.empty(int(lib.hiseg_distill_ws(B, H, W)), dtype=torch.float32, device=dev)
        out = torch.empty(L.DISTILL_NOUT, dtype=torch.float32, device=dev)
        L.check(lib.hiseg_distill_loss_fwd(ctypes.byref(cfg), B, H, W, student.data_ptr(), teacher.data_ptr(),
                                           target.data_ptr() if target is not None else None, ws.data_ptr(),
                                           out.data_ptr(), L.stream_ptr()), "distill_loss_fwd")
        ctx.cfg = cfg
        ctx.dev_scalars = dev_scalars   # cfg.dev_scalars points into it: alive until the backward ran
        ctx.save_for_backward(student, teacher, target, ws)
        ctx.mark_non_differentiable(out)
        return out[0].clone(), out

    @staticmethod
    def backward(ctx, g_total, _g_out):
        student, teacher, target, ws = ctx.saved_tensors
        B, _, H, W = student.shape
        ds = torch.empty_like(student)
        g = g_total.contiguous().float()
        L.check(L.lib().hiseg_distill_loss_bwd(ctypes.byref(ctx.cfg), B, H, W, student.data_ptr(), teacher.data_ptr(),
                                               target.data_ptr() if target is not None else None, ws.data_ptr(),
                                               g.data_ptr(), ds.data_ptr(), L.stream_ptr()), "distill_loss_bwd")
        return None, ds, None, None, None


class UNetDistillationLoss(nn.Module):
    """unet_decoder_distillation.py:338-663 (constructor arguments and state as the reference)."""

    def __init__(self, temperature: float = 3.0, alpha: float = 0.5, task_weight: float = 0.3,
                 use_feature_matching: bool = False, fg_ratio: float = 0.162, use_dice_loss: bool = True,
                 adaptive_distillation: bool = True):
        super().__init__()
        if use_feature_matching:
            raise NotImplementedError("feature matching is not used by the distillation configs (SURVEY §8a D2)")
        self.temperature = temperature
        self.initial_temperature = temperature
        self.alpha = alpha
        self.initial_alpha = alpha
        self.task_weight = task_weight
        self.initial_task_weight = task_weight
        self.use_feature_matching = use_feature_matching
        self.use_dice_loss = use_dice_loss
        self.adaptive_distillation = adaptive_distillation
        self.performance_ratio = 1.0
        self.distillation_eliminated = False
        self.pos_weight_value = float(np.sqrt((1.0 - fg_ratio) / fg_ratio))
        self._dev: Optional[torch.Tensor] = None   # device f32 [T, kl_weight, task_weight, pos_weight]
        self._dev_vals = None

    # -- schedules (host state, once per epoch: :366-469)
    def update_temperature(self, current_epoch: int, total_epochs: int, final_temperature: float = 1.0,
                           schedule_type: str = "linear") -> float:
        if total_epochs <= 1:
            self.temperature = final_temperature
            return self.temperature
        progress = current_epoch / (total_epochs - 1)
        if schedule_type == "linear":
            self.temperature = self.initial_temperature + (final_temperature - self.initial_temperature) * progress
        elif schedule_type == "cosine":
            f = 0.5 * (1 + math.cos(math.pi * progress))
            self.temperature = final_temperature + (self.initial_temperature - final_temperature) * f
        elif schedule_type == "exponential":
            rate = math.log(final_temperature / self.initial_temperature)
            self.temperature = self.initial_temperature * math.exp(rate * progress)
        return self.temperature

    def get_temperature(self) -> float:
        return self.temperature

    def update_distillation_weight(self, student_iou: float, teacher_iou: float, min_alpha: float = 0.0,
                                   amplification_factor: float = 20.0,
                                   zero_distillation_threshold: float = 0.03) -> float:
        if not self.adaptive_distillation:
            return self.alpha
        if self.distillation_eliminated:
            self.alpha, self.task_weight = 0.0, 1.0
            return self.alpha
        self.performance_ratio = student_iou / (teacher_iou + 1e-6)
        if self.performance_ratio > 1.0 + zero_distillation_threshold:
            self.alpha, self.task_weight = 0.0, 1.0
            self.distillation_eliminated = True
        elif self.performance_ratio > 1.0:
            diff = (self.performance_ratio - 1.0) * amplification_factor
            self.alpha = max(0.0, self.initial_alpha * np.exp(-diff))
            target = 1.0 - np.exp(-diff * 2)
            self.task_weight = min(1.0, self.initial_task_weight + (1.0 - self.initial_task_weight) * target)
        else:
            self.alpha, self.task_weight = self.initial_alpha, self.initial_task_weight
        return self.alpha

    # -- the reference's control flow (:510-663) reduced to the kernel configuration
    def _cfg(self, has_target: bool) -> L.DistillCfg:
        c = L.DistillCfg()
        disabled = ((self.adaptive_distillation and self.alpha == 0.0) or self.task_weight >= 0.99
                    or self.distillation_eliminated)
        in_total = not ((self.adaptive_distillation and self.alpha == 0.0) or self.task_weight >= 0.99)
        if self.adaptive_distillation and self.performance_ratio > 1.0:
            eff_alpha = self.alpha * max(0.1, 2.0 - self.performance_ratio)
        else:
            eff_alpha = self.alpha
        c.temperature = float(self.temperature)
        c.kl_weight = float(min(eff_alpha, 0.1))
        c.task_weight = float(self.task_weight)
        c.pos_weight = self.pos_weight_value
        c.distill_terms = int(not disabled)
        c.distill_in_total = int(in_total)
        c.use_dice = int(self.use_dice_loss)
        c.has_target = int(has_target)
        return c

    # ---------------------------------------------------------------- device scalars (hiseg.graphs)
    def sync_device_scalars(self, device=None):
        """Write the schedule values (temperature, effective KL weight, task weight, pos weight) into the device
        buffer the loss kernels read, when they changed; GraphedStep calls this before every replay, so the
        per-epoch temperature schedule (train_distillation_staged.py:1597-1610) replays one captured graph."""
        c = self._cfg(True)
        vals = (c.temperature, c.kl_weight, c.task_weight, c.pos_weight)   # already rounded to f32
        if self._dev is None or (device is not None and self._dev.device != torch.device(device)):
            self._dev = torch.empty(4, dtype=torch.float32, device=device)
            self._dev_vals = None
        if vals != self._dev_vals:
            for i, v in enumerate(vals):
                self._dev[i].fill_(v)
            self._dev_vals = vals
        return self._dev

    def graph_key(self):
        """What a captured step bakes in: which terms run and enter the total (structure, not values)."""
        c = self._cfg(True)
        return (c.distill_terms, c.distill_in_total, c.use_dice,
                self._dev.data_ptr() if self._dev is not None else None)

    def forward(self, student_output: torch.Tensor, teacher_output: torch.Tensor,
                target_masks: Optional[torch.Tensor] = None) -> Tuple[torch.Tensor, Dict[str, float]]:
        if not student_output.is_cuda:
            raise RuntimeError("hiseg UNetDistillationLoss runs on the GPU (libhiseg); got a CPU tensor")
        s = student_output.float().contiguous()
        t = teacher_output.detach().float().contiguous()
        y = target_masks.float().contiguous() if target_masks is not None else None
        if s.dim() != 4 or s.shape[1] != 1 or t.shape != s.shape or (y is not None and y.numel() != s.numel()):
            raise ValueError(f"distillation loss: student {tuple(s.shape)} teacher {tuple(t.shape)} "
                             f"target {None if y is None else tuple(y.shape)} (expect [B,1,H,W])")
        cfg = self._cfg(y is not None)
        if torch.cuda.is_current_stream_capturing():
            if self._dev is None or self._dev.device != s.device:
                raise RuntimeError("UNetDistillationLoss: the first call cannot be captured (run it eagerly first)")
            _graphs.note_device_scalars(self)
        else:
            self.sync_device_scalars(s.device)
        cfg.dev_scalars = self._dev.data_ptr()
        total, out = _DistillLossFn.apply(cfg, s, t, y, self._dev)
        return total, _LazyDict(out, _DICT_KEYS)

    def dice_loss(self, pred: torch.Tensor, target: torch.Tensor) -> torch.Tensor:
        """:471-508 (standalone helper; the forward computes it inside the fused kernels)."""
        c = self._cfg(True)
        c.distill_terms, c.distill_in_total, c.use_dice, c.task_weight = 0, 0, 1, 1.0
        s = pred.float().contiguous()
        _, out = _DistillLossFn.apply(c, s, torch.zeros_like(s), target.float().contiguous())
        return out[4]


# ======================================================================================= models
def _safe_state_dict(path: str) -> Dict[str, torch.Tensor]:
    """Checkpoint tensors through the non-executing loader (weights_only=True) and the reference's key
    handling (:173-195): 'state_dict' / 'model_state_dict' wrappers, 'model.' / 'unet.' prefixes."""
    ck = torch.load(path, map_location="cpu", weights_only=True)
    sd = ck.get("state_dict", ck.get("model_state_dict", ck)) if isinstance(ck, dict) else ck
    out = {}
    for k, v in sd.items():
        nk = k.replace("model.", "") if k.startswith("model.") else k
        nk = nk.replace("unet.", "") if nk.startswith("unet.") else nk
        if any(part in nk for part in ("encoder", "decoder", "segmentation_head")):
            out[nk] = v
    return out


class UNetDecoderOnly(nn.Module):
    """advanced/unet_decoder_distillation.py:17-82: the smp-UNet student (``self.unet``), encoder frozen on
    request.  Train mode runs the HIP training path (hiseg.effunet_train); eval runs the inference kernels."""

    def __init__(self, encoder_name: str = "timm-efficientnet-b0", encoder_weights: Optional[str] = None,
                 freeze_encoder: bool = True, freeze_decoder: bool = False):
        super().__init__()
        from .effunet import EfficientNetUnet
        if encoder_weights is not None:
            # the reference downloads ImageNet weights here (encoder_weights="imagenet"); no network on this
            # path -- load a checkpoint through student_pretrained_path / load_state_dict instead
            encoder_weights = None
        self.unet = EfficientNetUnet(encoder_name=encoder_name, classes=1, encoder_weights=encoder_weights)
        if freeze_encoder:
            for p in self.unet.encoder.parameters():
                p.requires_grad = False
        if freeze_decoder:
            for p in self.unet.decoder.parameters():
                p.requires_grad = False

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        from . import engine as EG
        if self.training:
            from .effunet_train import student_train_forward
            return student_train_forward(self, self.unet, x)
        with torch.no_grad():
            E = EG.Ctx(self.unet, EG._root_dtype(self), x.device)
            from .ops import Act
            return EG.effunet_forward(E, self.unet, Act.from_nchw(x.contiguous().float(), E.dtype))

    def get_decoder_parameters(self):
        return self.unet.decoder.parameters()

    @property
    def encoder(self):
        return self.unet.encoder


class _FrozenUnet(nn.Module):
    """Teacher smp.Unet in eval mode on the inference kernels (no gradients)."""

    def __init__(self, encoder_name: str):
        super().__init__()
        from .effunet import EfficientNetUnet
        self.unet = EfficientNetUnet(encoder_name=encoder_name, classes=1)

    @torch.no_grad()
    def forward(self, x: torch.Tensor) -> torch.Tensor:
        from . import engine as EG
        from .ops import Act
        E = EG.Ctx(self.unet, EG._root_dtype(self), x.device)
        return EG.effunet_forward(E, self.unet, Act.from_nchw(x.contiguous().float(), E.dtype))


class DistillationUNetWrapper(nn.Module):
    """advanced/unet_decoder_distillation.py:85-330: student + frozen teacher, progressive unfreezing."""

    def __init__(self, student_encoder: str = "timm-efficientnet-b0", teacher_encoder: str = "timm-efficientnet-b3",
                 teacher_checkpoint_path: Optional[str] = "ext_extractor/2020-09-23a.pth", freeze_teacher: bool = True,
                 progressive_unfreeze: bool = False, student_pretrained_path: Optional[str] = None):
        super().__init__()
        import os
        self.progressive_unfreeze = progressive_unfreeze
        self.student_encoder_name = student_encoder
        self.student = UNetDecoderOnly(encoder_name=student_encoder, freeze_encoder=progressive_unfreeze,
                                       freeze_decoder=False)
        if student_pretrained_path and os.path.exists(student_pretrained_path):
            ck = torch.load(student_pretrained_path, map_location="cpu", weights_only=True)
            sd = ck.get("model_state_dict", ck.get("state_dict", ck)) if isinstance(ck, dict) else ck
            self.student.load_state_dict(sd, strict=False)
        if teacher_checkpoint_path is not None and teacher_checkpoint_path != "":
            self.teacher = _FrozenUnet(teacher_encoder)
            if os.path.exists(teacher_checkpoint_path):
                self.teacher.unet.load_state_dict(_safe_state_dict(teacher_checkpoint_path), strict=False)
            if freeze_teacher:
                for p in self.teacher.parameters():
                    p.requires_grad = False
            self.teacher.eval()
        else:
            self.teacher = None
        if self.progressive_unfreeze:
            self._setup_encoder_blocks()

    def _setup_encoder_blocks(self):
        self.encoder_blocks = [(f"block_{i}", b) for i, b in enumerate(self.student.encoder.blocks)]

    def unfreeze_encoder_blocks(self, num_blocks: int, learning_rate_scale: float = 0.1):
        """:233-274 -- the deepest ``num_blocks`` encoder stages become trainable; returns their parameters."""
        if not self.progressive_unfreeze:
            return []
        for p in self.student.encoder.parameters():
            p.requires_grad = False
        params = []
        start = max(0, len(self.encoder_blocks) - num_blocks)
        for i in range(start, len(self.encoder_blocks)):
            for p in self.encoder_blocks[i][1].parameters():
                p.requires_grad = True
                params.append(p)
        return params

    def get_progressive_unfreeze_schedule(self, total_epochs: int, unfreeze_start_epoch: int = 10,
                                          unfreeze_rate: int = 5):
        """:276-302"""
        max_blocks = len(self.encoder_blocks) if hasattr(self, "encoder_blocks") else 7
        return {e: 0 if e < unfreeze_start_epoch else min(1 + (e - unfreeze_start_epoch) // unfreeze_rate, max_blocks)
                for e in range(total_epochs)}

    def train(self, mode: bool = True):
        super().train(mode)
        if self.teacher is not None:
            self.teacher.eval()   # the teacher always runs in eval mode (train_distillation_staged.py:270-271)
        return self

    # the frozen teacher's forward and the student's forward are independent until the loss: on a GPU the teacher
    # runs on a side stream beside the student (both are chains of small kernels that leave most CUs idle; forked
    # from and joined back into the caller's stream, so a captured HIP graph holds them as parallel branches).
    # Same kernels, same inputs: the results are the serial order's bit for bit.  HISEG_SERIAL_TEACHER=1: serial.
    concurrent_teacher = os.environ.get("HISEG_SERIAL_TEACHER", "0") != "1"

    def _side(self, device):
        from .streams import role_stream
        return role_stream("teacher", device)

    def forward(self, x: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
        if self.teacher is not None and x.is_cuda and self.concurrent_teacher:
            main = torch.cuda.current_stream(x.device)
            side = self._side(x.device)
            side.wait_stream(main)
            with torch.cuda.stream(side):
                t = self.teacher(x)
            s = self.student(x)
            main.wait_stream(side)
            t.record_stream(main)
            return s, t
        s = self.student(x)
        if self.teacher is not None:
            t = self.teacher(x)
        else:
            t = torch.zeros_like(s)
        return s, t


def create_unet_distillation_model(student_encoder: str = "timm-efficientnet-b0",
                                   teacher_encoder: str = "timm-efficientnet-b3",
                                   teacher_checkpoint: Optional[str] = "ext_extractor/2020-09-23a.pth",
                                   device: str = "cuda", progressive_unfreeze: bool = False,
                                   adaptive_distillation: bool = True, amplification_factor: float = 20.0,
                                   min_alpha: float = 0.001, student_pretrained_path: Optional[str] = None
                                   ) -> Tuple[nn.Module, nn.Module]:
    """:665-720 -- (wrapper, loss) with the reference's loss settings for distillation / pure fine-tuning."""
    model = DistillationUNetWrapper(student_encoder=student_encoder, teacher_encoder=teacher_encoder,
                                    teacher_checkpoint_path=teacher_checkpoint, freeze_teacher=True,
                                    progressive_unfreeze=progressive_unfreeze,
                                    student_pretrained_path=student_pretrained_path).to(device)
    if teacher_checkpoint is None or teacher_checkpoint == "":
        loss = UNetDistillationLoss(temperature=1.0, alpha=0.0, task_weight=1.0, use_dice_loss=True,
                                    adaptive_distillation=False)
    else:
        loss = UNetDistillationLoss(temperature=1.0, alpha=0.05, task_weight=0.7, use_dice_loss=True,
                                    adaptive_distillation=adaptive_distillation)
    return model, loss
