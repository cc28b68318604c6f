"""Shared helpers for the test-suite (test infrastructure only)."""
import json
import os

import numpy as np
import torch

from conftest import GOLDEN


def load(name):
    return np.load(os.path.join(GOLDEN, name + ".npz"))


def configs():
    with open(os.path.join(GOLDEN, "configs.json")) as f:
        return json.load(f)


def b0_kwargs():
    return dict(configs()["b0"]["model_kwargs"])


def hiseg_kwargs(kw):
    """create_rgb_hierarchical_model kwargs for hiseg (pretrained path left unresolved: no weight files)."""
    k = dict(kw)
    k["roi_size"] = tuple(k["roi_size"]) if isinstance(k["roi_size"], list) else k["roi_size"]
    k["mask_size"] = tuple(k["mask_size"]) if isinstance(k["mask_size"], list) else k["mask_size"]
    return k


def rel_err(a, b):
    a = torch.as_tensor(np.asarray(a)).double()
    b = torch.as_tensor(np.asarray(b)).double()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-12)).item()


def max_abs(a, b):
    a = torch.as_tensor(np.asarray(a)).double()
    b = torch.as_tensor(np.asarray(b)).double()
    return (a - b).abs().max().item()
