"""Training checkpoints in the reference's format (train_advanced.py:1592-1599 save, :1204-1246 resume).

A checkpoint is ``{'epoch', 'model_state_dict', 'optimizer_state_dict', 'scheduler_state_dict', 'best_miou',
'config'}``: the model keys are the reference's (hiseg keeps its module tree), the optimizer state is
torch.optim.AdamW's layout (hiseg.FusedAdamW reads and writes it), the scheduler state is the torch
scheduler's own.  So a run can resume from a reference checkpoint, and the reference can resume from a
hiseg one.  Files are read with the non-executing loader (``weights_only=True``), unlike the reference.
"""
from __future__ import annotations

import warnings
from typing import Optional, Tuple

import torch
import torch.nn as nn


def save_checkpoint(path: str, model: nn.Module, optimizer, epoch: int, best_miou: float = 0.0,
                    scheduler=None, config: Optional[dict] = None) -> dict:
    """train_advanced.py:1592-1599 (the dict it saves each epoch)."""
    # cloned: hiseg parameters are views into one flat training buffer
    ck = {"epoch": int(epoch), "model_state_dict": {k: v.detach().clone() for k, v in model.state_dict().items()},
          "optimizer_state_dict": optimizer.state_dict() if optimizer is not None else None,
          "scheduler_state_dict": scheduler.state_dict() if scheduler is not None else None,
          "best_miou": float(best_miou), "config": config if config is not None else {}}
    torch.save(ck, path)
    return ck


def _reseed_output_conv(model: nn.Module) -> None:
    # train_advanced.py:1230-1241: channel 0 = +u (background), channel 1 = -u, zero bias
    pu = getattr(model, "pretrained_unet", None)
    oc = getattr(pu, "output_conv", None)
    if oc is None:
        return
    with torch.no_grad():
        oc.weight.data[0, 0, 0, 0] = 1.0
        oc.weight.data[1, 0, 0, 0] = -1.0
        oc.bias.data.zero_()


def resume_from_checkpoint(path: str, model: nn.Module, optimizer=None, scheduler=None,
                           map_location="cpu") -> Tuple[int, float]:
    """train_advanced.py:1204-1246: strict load with a non-strict fallback, optimizer state, epoch + 1,
    best_miou, output_conv re-seed, scheduler state.  Returns (start_epoch, best_miou)."""
    ck = torch.load(path, map_location=map_location, weights_only=True)
    sd = ck["model_state_dict"]
    try:
        model.load_state_dict(sd)
    except RuntimeError as e:
        inc = model.load_state_dict(sd, strict=False)
        warnings.warn(f"strict load failed ({str(e).splitlines()[0]}); loaded with strict=False: "
                      f"{len(inc.missing_keys)} missing, {len(inc.unexpected_keys)} unexpected keys")
    if optimizer is not None and ck.get("optimizer_state_dict") is not None:
        optimizer.load_state_dict(ck["optimizer_state_dict"])
    start_epoch = int(ck["epoch"]) + 1
    best_miou = ck.get("best_miou", 0)
    _reseed_output_conv(model)
    if scheduler is not None and ck.get("scheduler_state_dict") is not None:
        scheduler.load_state_dict(ck["scheduler_state_dict"])
    return start_epoch, best_miou
