"""EfficientNet-B0..B7 U-Net with the parameter layout of ``smp.Unet('timm-efficientnet-bX')``.

The reference builds this network through the third-party packages
segmentation_models_pytorch 0.5.0 + timm 1.0.19 (uv.lock:1496-1508,1683-1685) at
advanced/hierarchical_segmentation_unet.py:1770-1774; neither package is in this image, so
the architecture is restated from their published definitions:

* timm ``_gen_efficientnet`` arch string (stage: type, repeats, kernel, stride, expansion,
  out channels, SE 0.25), channel multiplier via make_divisible(., 8), depth multiplier via
  ceil, Swish activation, BatchNorm eps 1e-5, SE reduction from the block input channels;
  ``conv_head``/``bn2`` exist (smp only deletes the classifier).
* smp encoder taps: stem (stride 2), blocks[:2] (/4), blocks[2:3] (/8), blocks[3:5] (/16),
  blocks[5:] (/32);  UnetDecoder channels (256,128,64,32,16), nearest x2 upsample + skip
  concat + 2 x (conv3x3, BN, ReLU);  SegmentationHead conv3x3 -> classes.

Consistency checks against the reference itself (the only pins available):
encoder key counts B0 358 / B1 506 / B7 1198 (hierarchical_segmentation_unet.py:1815-1828
thresholds 400/540/700) and the decoder key pattern ``decoder.blocks.{i}.conv1.0.weight``
(export_peopleseg_onnx.py:111-124).  Numerical parity of this sub-network is unpinned.
"""
from __future__ import annotations

import math
from typing import List, Tuple

import torch.nn as nn

# stage: (block type, repeats, kernel, stride, expansion, out channels)
_ARCH = [
    ("ds", 1, 3, 1, 1, 16),
    ("ir", 2, 3, 2, 6, 24),
    ("ir", 2, 5, 2, 6, 40),
    ("ir", 3, 3, 2, 6, 80),
    ("ir", 3, 5, 1, 6, 112),
    ("ir", 4, 5, 2, 6, 192),
    ("ir", 1, 3, 1, 6, 320),
]
# (channel multiplier, depth multiplier)
_PARAMS = {
    "b0": (1.0, 1.0), "b1": (1.0, 1.1), "b2": (1.1, 1.2), "b3": (1.2, 1.4),
    "b4": (1.4, 1.8), "b5": (1.6, 2.2), "b6": (1.8, 2.6), "b7": (2.0, 3.1),
}
STAGE_IDXS = (2, 3, 5)
DECODER_CHANNELS = (256, 128, 64, 32, 16)


def make_divisible(v: float, divisor: int = 8, round_limit: float = 0.9) -> int:
    new_v = max(divisor, int(v + divisor / 2) // divisor * divisor)
    if new_v < round_limit * v:
        new_v += divisor
    return new_v


def variant_of(encoder_name: str) -> str:
    name = encoder_name.lower()
    for k in _PARAMS:
        if name.endswith(k):
            return k
    raise NotImplementedError(f"encoder '{encoder_name}' is not an EfficientNet-B0..B7 (hot path: timm-efficientnet-bX)")


class SqueezeExcite(nn.Module):
    def __init__(self, chs: int, rd: int):
        super().__init__()
        self.conv_reduce = nn.Conv2d(chs, rd, 1, bias=True)
        self.act1 = nn.SiLU(inplace=True)
        self.conv_expand = nn.Conv2d(rd, chs, 1, bias=True)
        self.gate = nn.Sigmoid()


class DepthwiseSeparableConv(nn.Module):
    def __init__(self, cin: int, cout: int, k: int, stride: int, se_rd: int):
        super().__init__()
        self.conv_dw = nn.Conv2d(cin, cin, k, stride, k // 2, groups=cin, bias=False)
        self.bn1 = nn.BatchNorm2d(cin)
        self.se = SqueezeExcite(cin, se_rd)
        self.conv_pw = nn.Conv2d(cin, cout, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(cout)
        self.kernel, self.stride = k, stride
        self.has_skip = stride == 1 and cin == cout


class InvertedResidual(nn.Module):
    def __init__(self, cin: int, cout: int, k: int, stride: int, exp: int, se_rd: int):
        super().__init__()
        mid = make_divisible(cin * exp)
        self.conv_pw = nn.Conv2d(cin, mid, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(mid)
        self.conv_dw = nn.Conv2d(mid, mid, k, stride, k // 2, groups=mid, bias=False)
        self.bn2 = nn.BatchNorm2d(mid)
        self.se = SqueezeExcite(mid, se_rd)
        self.conv_pwl = nn.Conv2d(mid, cout, 1, bias=False)
        self.bn3 = nn.BatchNorm2d(cout)
        self.kernel, self.stride = k, stride
        self.has_skip = stride == 1 and cin == cout


class EfficientNetEncoder(nn.Module):
    def __init__(self, variant: str):
        super().__init__()
        wm, dm = _PARAMS[variant]
        rc = lambda c: make_divisible(c * wm)  # noqa: E731
        stem = rc(32)
        self.conv_stem = nn.Conv2d(3, stem, 3, 2, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(stem)
        stages = []
        cin = stem
        for btype, reps, k, s, e, c in _ARCH:
            cout = rc(c)
            blocks = []
            for r in range(int(math.ceil(reps * dm))):
                stride = s if r == 0 else 1
                se_rd = max(1, int(round(cin * 0.25)))
                if btype == "ds":
                    blocks.append(DepthwiseSeparableConv(cin, cout, k, stride, se_rd))
                else:
                    blocks.append(InvertedResidual(cin, cout, k, stride, e, se_rd))
                cin = cout
            stages.append(nn.Sequential(*blocks))
        self.blocks = nn.Sequential(*stages)
        head = rc(1280)
        self.conv_head = nn.Conv2d(cin, head, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(head)
        chans = [3, stem]
        for lo, hi in ((0, STAGE_IDXS[0]), (STAGE_IDXS[0], STAGE_IDXS[1]), (STAGE_IDXS[1], STAGE_IDXS[2]),
                       (STAGE_IDXS[2], len(_ARCH))):
            chans.append(rc(_ARCH[hi - 1][5]))
        self.out_channels: Tuple[int, ...] = tuple(chans)


class Conv2dReLU(nn.Sequential):
    def __init__(self, cin: int, cout: int):
        super().__init__(nn.Conv2d(cin, cout, 3, padding=1, bias=False), nn.BatchNorm2d(cout), nn.ReLU(inplace=True))


class DecoderBlock(nn.Module):
    def __init__(self, cin: int, cskip: int, cout: int):
        super().__init__()
        self.conv1 = Conv2dReLU(cin + cskip, cout)
        self.attention1 = nn.Identity()
        self.conv2 = Conv2dReLU(cout, cout)
        self.attention2 = nn.Identity()
        self.in_channels, self.skip_channels, self.out_channels = cin, cskip, cout


class UnetDecoder(nn.Module):
    def __init__(self, encoder_channels: Tuple[int, ...], decoder_channels=DECODER_CHANNELS):
        super().__init__()
        enc = list(encoder_channels[1:])[::-1]
        head = enc[0]
        ins = [head] + list(decoder_channels[:-1])
        skips = enc[1:] + [0]
        self.center = nn.Identity()
        self.blocks = nn.ModuleList([DecoderBlock(i, s, o) for i, s, o in zip(ins, skips, decoder_channels)])


class EfficientNetUnet(nn.Module):
    """Stand-in for ``smp.Unet(encoder_name='timm-efficientnet-bX', classes=1, encoder_weights=None)``."""

    def __init__(self, encoder_name: str = "timm-efficientnet-b0", classes: int = 1, encoder_weights=None):
        super().__init__()
        if encoder_weights is not None:
            raise ValueError("pretrained encoder downloads are not available offline; load a checkpoint instead")
        self.encoder_name = encoder_name
        self.encoder = EfficientNetEncoder(variant_of(encoder_name))
        self.decoder = UnetDecoder(self.encoder.out_channels)
        self.segmentation_head = nn.Sequential(
            nn.Conv2d(DECODER_CHANNELS[-1], classes, 3, padding=1), nn.Identity(), nn.Identity())
        self.classes = classes

    def block_list(self) -> List[nn.Module]:
        return [b for stage in self.encoder.blocks for b in stage]
