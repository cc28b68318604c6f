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


# normalisation / activation variants pinned by tests/golden/variants.npz (gen_golden.py variants)
VARIANTS = {"ln_gelu": ("layernorm2d", "gelu", 1.0), "bn_swish": ("batchnorm", "swish", 1.5),
            "ln_swish": ("layernorm2d", "swish", 0.75)}


def act_tag(act, beta):
    """The oracle's activation kind string (Swish's beta rides along as 'swish:<beta>')."""
    return f"swish:{float(beta)}" if act == "swish" and float(beta) != 1.0 else act


def variant_modules(norm, act, beta):
    """hiseg ResidualBlock(64), EnhancedUNet(64, 32, 3) and the small head of the variants fixture, filled."""
    import filler
    from hiseg.layers import EnhancedUNet, RefinedHierarchicalSegmentationHead, ResidualBlock
    blk = filler.fill_module(ResidualBlock(64, norm, 8, act, beta)).eval()
    unet = filler.fill_module(EnhancedUNet(64, 32, 3, norm, 8, act, beta)).eval()
    head = filler.fill_module(RefinedHierarchicalSegmentationHead(
        64, 64, 3, (32, 24), use_attention_module=True, use_contour_detection=True, use_distance_transform=True,
        normalization_type=norm, normalization_groups=8, activation_function=act, activation_beta=beta,
        hierarchical_base_channels=32, hierarchical_depth=3)).eval()
    return blk, unet, head


def small_head_cfg(norm, act, beta):
    return {"activation_function": act_tag(act, beta), "mask_hw": (32, 24), "roi_hw": (16, 12),
            "hierarchical_depth": 3, "use_attention_module": True, "use_contour_detection": True,
            "use_distance_transform": True}
