"""Building blocks of the ROI path with the reference's module tree and parameter names.

Each class holds standard torch parameters laid out exactly as the reference module of the
same name, so ``state_dict()`` keys, shapes and checkpoint files are interchangeable.  The
arithmetic never runs through these modules' own torch ops: forward passes are executed by
:mod:`hiseg.engine` on libhiseg kernels.  Reference citations are file:line in
PINTO0309/human-instance-segmentation.
"""
from __future__ import annotations

from typing import Tuple, Union

import torch
import torch.nn as nn


def _engine():
    from . import engine
    return engine


class LayerNorm2d(nn.Module):
    """Per-sample norm over (C, H, W) — src/human_edge_detection/model.py:18-38 (parameter layout only)."""

    def __init__(self, num_features: int, eps: float = 1e-5):
        super().__init__()
        self.weight = nn.Parameter(torch.ones(1, num_features, 1, 1))
        self.bias = nn.Parameter(torch.zeros(1, num_features, 1, 1))
        self.eps = eps


class Swish(nn.Module):
    """x * sigmoid(beta * x) — advanced/activation_utils.py (SwishInplace/Swish)."""

    def __init__(self, beta: float = 1.0):
        super().__init__()
        self.beta = beta


def make_norm(norm_type: str, channels: int, groups: int = 8) -> nn.Module:
    """advanced/normalization_comparison.py:159-206 (the two types the RGB path configs use)."""
    t = norm_type.lower()
    if t in ("batch", "batchnorm", "batchnorm2d"):
        return nn.BatchNorm2d(channels)
    if t in ("layer", "layernorm", "layernorm2d"):
        return LayerNorm2d(channels)
    raise NotImplementedError(f"normalization '{norm_type}' is outside the hiseg hot path (batchnorm, layernorm2d)")


def make_act(name: str, beta: float = 1.0) -> nn.Module:
    """advanced/activation_utils.py:71-101 and hierarchical_segmentation_unet.py:13-32."""
    n = name.lower()
    if n == "relu":
        return nn.ReLU(inplace=True)
    if n == "silu":
        return nn.SiLU(inplace=True)
    if n == "swish":
        return Swish(beta)
    if n == "gelu":
        return nn.GELU()
    raise ValueError(f"Unknown activation function: {name}")


def make_act_unet(name: str, beta: float = 1.0) -> nn.Module:
    """get_activation_function of hierarchical_segmentation_unet.py:13-32 (== rgb.py:21-40): 'swish' is
    nn.SiLU there -- beta is ignored -- unlike the refinement modules' get_activation (make_act)."""
    n = name.lower()
    if n == "relu":
        return nn.ReLU(inplace=True)
    if n in ("swish", "silu"):
        return nn.SiLU(inplace=True)
    if n == "gelu":
        return nn.GELU()
    raise ValueError(f"Unsupported activation function: {name}")


class ResidualBlock(nn.Module):
    """relu(bn2(conv2(relu(bn1(conv1 x)))) + x).

    ``two_acts=True`` mirrors the refinement-module variant (activation1/activation2,
    advanced/hierarchical_segmentation_refinement.py:31-55); ``False`` the UNet variant
    (single ``activation``, advanced/hierarchical_segmentation_unet.py:35-58).
    """

    def __init__(self, channels: int, norm: str = "batchnorm", groups: int = 8, act: str = "relu",
                 beta: float = 1.0, two_acts: bool = True):
        super().__init__()
        self.conv1 = nn.Conv2d(channels, channels, 3, padding=1)
        self.norm1 = make_norm(norm, channels, groups)
        self.conv2 = nn.Conv2d(channels, channels, 3, padding=1)
        self.norm2 = make_norm(norm, channels, groups)
        if two_acts:
            self.activation1 = make_act(act, beta)
            self.activation2 = make_act(act, beta)
        else:   # the UNet variant builds its activation with unet.py's factory (Swish -> SiLU)
            self.activation = make_act_unet(act, beta)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return _engine().residual_block_nchw(self, x)


class ChannelAttentionModule(nn.Module):
    """SE-style gate, advanced/attention_modules.py:10-64."""

    def __init__(self, in_channels: int, reduction_ratio: int = 8, min_channels: int = 8, act: str = "relu",
                 beta: float = 1.0):
        super().__init__()
        hidden = max(in_channels // reduction_ratio, min_channels)
        self.fc1 = nn.Conv2d(in_channels, hidden, 1, bias=False)
        self.activation = make_act(act, beta)
        self.fc2 = nn.Conv2d(hidden, in_channels, 1, bias=False)
        self.sigmoid = nn.Sigmoid()


class SpatialAttentionModule(nn.Module):
    """mean/max over channels -> kxk conv -> sigmoid gate, advanced/attention_modules.py:67-113."""

    def __init__(self, kernel_size: int = 7):
        super().__init__()
        assert kernel_size in (3, 5, 7)
        self.conv = nn.Conv2d(2, 1, kernel_size, padding=kernel_size // 2, bias=False)
        self.sigmoid = nn.Sigmoid()


class EnhancedUNet(nn.Module):
    """bg/fg U-Net of the hierarchical head, advanced/hierarchical_segmentation_unet.py:277-417."""

    def __init__(self, in_channels: int, base_channels: int = 64, depth: int = 4, norm: str = "batchnorm",
                 groups: int = 8, act: str = "relu", beta: float = 1.0):
        super().__init__()
        self.depth = depth
        self.activation_function = act
        self.activation_beta = beta
        ch = [in_channels] + [base_channels * (2 ** i) for i in range(depth)]

        def res(c):
            return ResidualBlock(c, norm, groups, act, beta, two_acts=False)

        self.encoders = nn.ModuleList()
        self.pools = nn.ModuleList()
        for i in range(depth):
            if i == 0:
                self.encoders.append(nn.Sequential(
                    nn.Conv2d(ch[0], ch[1], 3, padding=1), make_norm(norm, ch[1], groups), make_act_unet(act, beta),
                    res(ch[1]), res(ch[1])))
            else:
                self.encoders.append(nn.Sequential(
                    res(ch[i]), res(ch[i]), nn.Conv2d(ch[i], ch[i + 1], 3, padding=1),
                    make_norm(norm, ch[i + 1], groups), make_act_unet(act, beta)))
            if i < depth - 1:
                self.pools.append(nn.MaxPool2d(2))
        top = ch[-1]
        self.bottleneck = nn.Sequential(
            res(top), res(top), nn.Conv2d(top, top, 3, padding=1), make_norm(norm, top, groups), make_act_unet(act, beta),
            nn.Conv2d(top, top, 1), nn.Sigmoid())
        self.bottleneck_conv = nn.Conv2d(top, top, 3, padding=1)
        self.upconvs = nn.ModuleList()
        self.decoders = nn.ModuleList()
        for i in range(depth - 1, 0, -1):
            self.upconvs.append(nn.ConvTranspose2d(ch[i + 1], ch[i], 2, stride=2))
            self.decoders.append(nn.Sequential(
                nn.Conv2d(2 * ch[i], ch[i], 3, padding=1), make_norm(norm, ch[i], groups), make_act_unet(act, beta),
                res(ch[i]), res(ch[i])))
        self.final = nn.Sequential(
            nn.Conv2d(ch[1], ch[1] // 2, 3, padding=1), make_norm(norm, ch[1] // 2, groups), make_act_unet(act, beta),
            nn.Conv2d(ch[1] // 2, 2, 1))

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return _engine().enhanced_unet_nchw(self, x)


class ContourDetectionBranch(nn.Module):
    """advanced/hierarchical_segmentation_refinement.py:255-295."""

    def __init__(self, in_channels: int, contour_channels: int = 64, norm: str = "batchnorm", groups: int = 8,
                 act: str = "relu", beta: float = 1.0):
        super().__init__()
        self.contour_branch = nn.Sequential(
            nn.Conv2d(in_channels, contour_channels, 3, padding=1), make_norm(norm, contour_channels, groups),
            make_act(act, beta),
            nn.Conv2d(contour_channels, contour_channels, 3, padding=1), make_norm(norm, contour_channels, groups),
            make_act(act, beta),
            nn.Conv2d(contour_channels, 1, 1), nn.Sigmoid())


class DistanceTransformDecoder(nn.Module):
    """advanced/hierarchical_segmentation_refinement.py:298-344."""

    def __init__(self, in_channels: int, distance_channels: int = 128, norm: str = "batchnorm", groups: int = 8,
                 act: str = "relu", beta: float = 1.0):
        super().__init__()
        self.distance_head = nn.Sequential(
            nn.Conv2d(in_channels, distance_channels, 3, padding=1), make_norm(norm, distance_channels, groups),
            make_act(act, beta), ResidualBlock(distance_channels, norm, groups, act, beta),
            nn.Conv2d(distance_channels, 1, 1))
        self.threshold = nn.Parameter(torch.tensor(0.3))


def _hw(size: Union[int, Tuple[int, int]]) -> Tuple[int, int]:
    if isinstance(size, (tuple, list)):
        return int(size[0]), int(size[1])
    return int(size), int(size)


class ExtendedHierarchicalSegmentationHeadUNetV2(nn.Module):
    """Shared features -> bg/fg U-Net + gated target/non-target branch -> 3-class combine.

    advanced/hierarchical_segmentation_refinement.py:434-606.
    """

    def __init__(self, in_channels: int, mid_channels: int = 256, num_classes: int = 3,
                 mask_size: Union[int, Tuple[int, int]] = 56, dropout_rate: float = 0.1,
                 use_attention_module: bool = False, normalization_type: str = "layernorm2d",
                 normalization_groups: int = 8, activation_function: str = "relu", activation_beta: float = 1.0,
                 hierarchical_base_channels: int = 96, hierarchical_depth: int = 3):
        super().__init__()
        assert num_classes == 3, "Hierarchical model designed for 3 classes"
        self.num_classes = num_classes
        self.mask_size = mask_size
        self.mask_height, self.mask_width = _hw(mask_size)
        self.use_attention_module = use_attention_module
        norm, g, act, beta = normalization_type, normalization_groups, activation_function, activation_beta
        m = mid_channels
        half = m // 2
        self.shared_features = nn.Sequential(
            nn.Conv2d(in_channels, m, 3, padding=1), make_norm(norm, m, g), make_act(act, beta),
            nn.Dropout2d(dropout_rate), ResidualBlock(m, norm, g, act, beta), nn.Dropout2d(dropout_rate),
            ResidualBlock(m, norm, g, act, beta))
        self.bg_vs_fg_unet = EnhancedUNet(m, base_channels=hierarchical_base_channels, depth=hierarchical_depth,
                                          norm=norm, groups=g, act=act, beta=beta)
        self.upsample_bg_fg = nn.Sequential(
            nn.ConvTranspose2d(2, 32, 2, stride=2), make_norm(norm, 32, min(g, 32)), make_act(act, beta),
            nn.Conv2d(32, 2, 1))
        if use_attention_module:
            self.target_vs_nontarget_branch = nn.ModuleList([
                ResidualBlock(m, norm, g, act, beta), SpatialAttentionModule(7), nn.Dropout2d(dropout_rate),
                nn.ConvTranspose2d(m, half, 2, stride=2), make_norm(norm, half, min(g, half)), make_act(act, beta),
                ChannelAttentionModule(half, reduction_ratio=8, act=act, beta=beta), nn.Dropout2d(dropout_rate),
                ResidualBlock(half, norm, min(g, half), act, beta), nn.Conv2d(half, 2, 1)])
        else:
            self.target_vs_nontarget_branch = nn.Sequential(
                ResidualBlock(m, norm, g, act, beta), nn.Dropout2d(dropout_rate),
                nn.ConvTranspose2d(m, half, 2, stride=2), make_norm(norm, half, min(g, half)), make_act(act, beta),
                nn.Dropout2d(dropout_rate), ResidualBlock(half, norm, min(g, half), act, beta),
                nn.Conv2d(half, 2, 1))
        self.fg_gate = nn.Sequential(
            nn.Conv2d(2, m // 4, 1), make_act(act, beta), nn.Dropout2d(dropout_rate * 0.5),
            nn.Conv2d(m // 4, half, 1), make_act(act, beta), nn.Conv2d(half, m, 1), nn.Sigmoid())


class RefinedHierarchicalSegmentationHead(nn.Module):
    """advanced/hierarchical_segmentation_refinement.py:609-804 (contour + distance aux branches)."""

    def __init__(self, in_channels: int, mid_channels: int = 256, num_classes: int = 3,
                 mask_size: Union[int, Tuple[int, int]] = 56, use_attention_module: bool = False,
                 use_boundary_refinement: bool = False, use_progressive_upsampling: bool = False,
                 use_subpixel_conv: bool = False, use_contour_detection: bool = False,
                 use_distance_transform: bool = False, normalization_type: str = "layernorm2d",
                 normalization_groups: int = 8, activation_function: str = "relu", activation_beta: float = 1.0,
                 hierarchical_base_channels: int = 96, hierarchical_depth: int = 3):
        super().__init__()
        if use_boundary_refinement or use_progressive_upsampling or use_subpixel_conv:
            raise NotImplementedError(
                "boundary refinement / progressive upsampling / sub-pixel decoders are not used by the RGB "
                "hierarchical configs and are outside the hiseg hot path (SURVEY.md §8)")
        self.base_head = ExtendedHierarchicalSegmentationHeadUNetV2(
            in_channels, mid_channels, num_classes, mask_size, use_attention_module=use_attention_module,
            normalization_type=normalization_type, normalization_groups=normalization_groups,
            activation_function=activation_function, activation_beta=activation_beta,
            hierarchical_base_channels=hierarchical_base_channels, hierarchical_depth=hierarchical_depth)
        self.mask_size = mask_size
        self.mask_height, self.mask_width = _hw(mask_size)
        self.num_classes = num_classes
        self.use_boundary_refinement = False
        self.use_progressive_upsampling = False
        self.use_subpixel_conv = False
        self.use_contour_detection = use_contour_detection
        self.use_distance_transform = use_distance_transform
        args = dict(norm=normalization_type, groups=normalization_groups, act=activation_function,
                    beta=activation_beta)
        if use_contour_detection:
            self.contour_branch = ContourDetectionBranch(mid_channels, 64, **args)
        if use_distance_transform:
            self.distance_decoder = DistanceTransformDecoder(mid_channels, 128, **args)

    def forward(self, features: torch.Tensor):
        if self.training:
            raise NotImplementedError("hiseg executes the inference (eval-mode) forward; call .eval()")
        return _engine().head_nchw(self, features)
