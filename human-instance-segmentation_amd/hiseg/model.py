"""Drop-in model surface of the RGB hierarchical path.

Mirrors, module for module and parameter name for parameter name:
  * PreTrainedPeopleSegmentationUNet / ...Wrapper  (advanced/hierarchical_segmentation_unet.py:1708-1993)
  * DynamicRoIAlign                                (src/human_edge_detection/dynamic_roi_align.py:10-171)
  * HierarchicalRGBSegmentationModelWithFullImagePretrainedUNet and create_rgb_hierarchical_model
                                                   (advanced/hierarchical_segmentation_rgb.py:564-774, 925-1027)
Forward passes execute on libhiseg (hiseg.engine); CPU tensors are rejected.
"""
from __future__ import annotations

import os
from typing import Dict, Optional, Tuple, Union

import torch
import torch.nn as nn

from . import _lib as L
from . import engine
from . import export
from . import streams
from .effunet import EfficientNetUnet
from .layers import RefinedHierarchicalSegmentationHead, ResidualBlock, make_act_unet, make_norm


class DynamicRoIAlign(nn.Module):
    """Bilinear ROI crop with a per-call output size (dynamic_roi_align.py:10-171)."""

    def __init__(self, spatial_scale=(640, 640), sampling_ratio=-1, aligned=False):
        super().__init__()
        if isinstance(spatial_scale, (list, tuple)):
            assert len(spatial_scale) == 2, "spatial_scale tuple must have 2 elements (height, width)"
            self.spatial_scale_h, self.spatial_scale_w = spatial_scale
        else:
            self.spatial_scale_h = self.spatial_scale_w = spatial_scale
        self.spatial_scale = spatial_scale
        self.sampling_ratio = sampling_ratio  # unused, as in the reference (:37-38)
        self.aligned = aligned

    def forward(self, input_feature_map: torch.Tensor, rois: torch.Tensor, output_height, output_width):
        if export.tracing(input_feature_map, rois):
            return export.traced_roi_align(self, input_feature_map, rois, output_height, output_width)
        return engine.roi_align_nchw(self, input_feature_map, rois, output_height, output_width)


def _imagenet_or_half(path: str, mean, std):
    if mean is not None and std is not None:
        return list(mean), list(std)
    if any(v in path.lower() for v in ("b0", "b1", "b7")):
        return [0.485, 0.456, 0.406], [0.229, 0.224, 0.225]
    return [0.5, 0.5, 0.5], [0.5, 0.5, 0.5]


class PreTrainedPeopleSegmentationUNet(nn.Module):
    """Frozen full-image person UNet (hierarchical_segmentation_unet.py:1708-1916)."""

    def __init__(self, in_channels: int = 3, classes: int = 1,
                 pretrained_weights_path: str = "ext_extractor/2020-09-23a.pth", mean=None, std=None,
                 freeze_weights: bool = False, encoder_name: str = "timm-efficientnet-b3"):
        super().__init__()
        self.in_channels = in_channels
        self.classes = classes
        self.encoder_name = encoder_name
        # normalisation chosen by weights-path substring (:1744-1758)
        self.mean, self.std = _imagenet_or_half(pretrained_weights_path or "", mean, std)
        self.model = EfficientNetUnet(encoder_name=encoder_name, classes=classes, encoder_weights=None)
        if pretrained_weights_path and os.path.exists(pretrained_weights_path):
            load_pretrained_unet(self.model, pretrained_weights_path)
        if freeze_weights:
            for p in self.model.parameters():
                p.requires_grad = False
            self.model.eval()
            self._freeze_bn = True
        else:
            self._freeze_bn = False
        self.register_buffer("norm_mean", torch.tensor(self.mean).view(1, 3, 1, 1))
        self.register_buffer("norm_std", torch.tensor(self.std).view(1, 3, 1, 1))
        export.record_init(self, in_channels=in_channels, classes=classes, pretrained_weights_path="",
                           mean=list(self.mean), std=list(self.std), encoder_name=encoder_name)

    def train(self, mode: bool = True):
        super().train(mode)
        if getattr(self, "_freeze_bn", False):
            self.model.eval()
        return self

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if export.tracing(x):
            return export.traced_unet_logit(self, x)
        return engine.unet_logits_nchw(self, x)


def load_pretrained_unet(model: nn.Module, path: str) -> Tuple[list, list]:
    """Checkpoint loading of hierarchical_segmentation_unet.py:1781-1867 (prefix strip, strict=False).

    Unlike the reference (weights_only=False) the file is read with the non-executing loader.
    """
    ckpt = torch.load(path, map_location="cpu", weights_only=True)
    sd = ckpt
    if isinstance(ckpt, dict):
        for k in ("state_dict", "model_state_dict"):
            if k in ckpt:
                sd = ckpt[k]
                break
    first = next(iter(sd.keys()), "")
    prefix = "model." if first.startswith("model.") else ("unet." if first.startswith("unet.") else "")
    sd = {(k[len(prefix):] if prefix and k.startswith(prefix) else k): v for k, v in sd.items()}
    missing, unexpected = model.load_state_dict(sd, strict=False)
    return missing, unexpected


class PreTrainedPeopleSegmentationUNetWrapper(nn.Module):
    """UNet logit u -> trainable 1x1 conv 1->2 initialised [+1, -1] (hierarchical_segmentation_unet.py:1919-1993)."""

    def __init__(self, in_channels: int, base_channels: int = 64, depth: int = 4, groups=None,
                 normalization_type: str = "layernorm2d", normalization_groups: int = 8,
                 pretrained_weights_path: str = "ext_extractor/2020-09-23a.pth", freeze_weights: bool = False,
                 encoder_name: str = "timm-efficientnet-b3"):
        super().__init__()
        self.model = PreTrainedPeopleSegmentationUNet(in_channels=in_channels, classes=1,
                                                      pretrained_weights_path=pretrained_weights_path,
                                                      freeze_weights=freeze_weights, encoder_name=encoder_name)
        self.output_conv = nn.Conv2d(1, 2, kernel_size=1)
        with torch.no_grad():
            self.output_conv.weight.data[0, 0, 0, 0] = 1.0
            self.output_conv.weight.data[1, 0, 0, 0] = -1.0
            self.output_conv.bias.data.zero_()

    def forward(self, x: torch.Tensor):
        if export.tracing(x):
            return export.traced_unet_wrapper(self, x), []
        return engine.unet_two_channel_nchw(self, x), []


class HierarchicalRGBSegmentationModelWithFullImagePretrainedUNet(nn.Module):
    """Full-image UNet -> 2x RoIAlign -> RGB conv stack -> 258->256 combiner -> refined hierarchical head."""

    def __init__(self, roi_size: Union[int, Tuple[int, int]] = 28, mask_size: Union[int, Tuple[int, int]] = 56,
                 pretrained_weights_path: str = "ext_extractor/2020-09-23a.pth", use_attention_module: bool = False,
                 freeze_pretrained_weights: bool = False, use_boundary_refinement: bool = False,
                 use_progressive_upsampling: bool = False, use_subpixel_conv: bool = False,
                 use_contour_detection: bool = False, use_distance_transform: bool = False,
                 normalization_type: str = "layernorm2d", normalization_groups: int = 8,
                 activation_function: str = "relu", activation_beta: float = 1.0, **kwargs):
        super().__init__()
        base = kwargs.get("hierarchical_base_channels", 96)
        depth = kwargs.get("hierarchical_depth", 3)
        self.roi_size = (roi_size, roi_size) if isinstance(roi_size, int) else tuple(roi_size)
        self.mask_size = (mask_size, mask_size) if isinstance(mask_size, int) else tuple(mask_size)
        self.pretrained_unet = PreTrainedPeopleSegmentationUNetWrapper(
            in_channels=3, pretrained_weights_path=pretrained_weights_path, freeze_weights=freeze_pretrained_weights,
            encoder_name=kwargs.get("encoder_name", "timm-efficientnet-b3"))
        # training semantics: normalised ROIs x 640 (rgb.py:636-647); export sets (H, W)
        self.roi_align_mask = DynamicRoIAlign(spatial_scale=640.0, sampling_ratio=2, aligned=True)
        self.roi_align_rgb = DynamicRoIAlign(spatial_scale=640.0, sampling_ratio=2, aligned=True)
        fd = 256
        norm, g, act, beta = normalization_type, normalization_groups, activation_function, activation_beta
        self.rgb_feature_extractor = nn.Sequential(
            nn.Conv2d(3, 64, 3, padding=1), make_norm(norm, 64, min(g, 64)), make_act_unet(act, beta),
            ResidualBlock(64, norm, min(g, 64), act, beta),
            nn.Conv2d(64, 128, 3, padding=1), make_norm(norm, 128, min(g, 128)), make_act_unet(act, beta),
            ResidualBlock(128, norm, min(g, 128), act, beta),
            nn.Conv2d(128, 256, 3, padding=1), make_norm(norm, 256, min(g, 256)), make_act_unet(act, beta),
            ResidualBlock(256, norm, min(g, 256), act, beta),
            nn.Conv2d(256, fd, 1), make_norm(norm, fd, min(g, fd)), make_act_unet(act, beta))
        use_refinement = any([use_boundary_refinement, use_progressive_upsampling, use_subpixel_conv,
                              use_contour_detection, use_distance_transform])
        if not use_refinement:
            raise NotImplementedError(
                "PretrainedUNetGuidedSegmentationHead (no refinement flags) is not used by the measured configs; "
                "hiseg builds the RefinedHierarchicalSegmentationHead path (SURVEY.md §0 item 4)")
        self.feature_combiner = nn.Conv2d(fd + 2, fd, 1)
        ms = self.mask_size[0] if self.mask_size[0] == self.mask_size[1] else self.mask_size
        self.segmentation_head = RefinedHierarchicalSegmentationHead(
            in_channels=fd, mid_channels=256, num_classes=3, mask_size=ms, use_attention_module=use_attention_module,
            use_boundary_refinement=use_boundary_refinement, use_progressive_upsampling=use_progressive_upsampling,
            use_subpixel_conv=use_subpixel_conv, use_contour_detection=use_contour_detection,
            use_distance_transform=use_distance_transform, normalization_type=norm, normalization_groups=g,
            activation_function=act, activation_beta=beta, hierarchical_base_channels=base,
            hierarchical_depth=depth)
        # compute precision of the HIP path: f32 (parity with the reference) or bf16 (throughput)
        self.hiseg_dtype = torch.float32
        export.record_init(self, roi_size=list(self.roi_size), mask_size=list(self.mask_size),
                           pretrained_weights_path="", use_attention_module=use_attention_module,
                           use_boundary_refinement=use_boundary_refinement,
                           use_progressive_upsampling=use_progressive_upsampling, use_subpixel_conv=use_subpixel_conv,
                           use_contour_detection=use_contour_detection,
                           use_distance_transform=use_distance_transform, normalization_type=normalization_type,
                           normalization_groups=normalization_groups, activation_function=activation_function,
                           activation_beta=activation_beta, **kwargs)

    def forward(self, images: torch.Tensor, rois: torch.Tensor) -> Tuple[torch.Tensor, Dict[str, torch.Tensor]]:
        if self.training:  # train-mode BatchNorm / Dropout + hand-written backward (hiseg.train_engine)
            from . import train_engine
            return train_engine.train_forward(self, images, rois)
        if export.tracing(images, rois):
            return export.traced_rgb_model(self, images, rois, aux="full")
        return engine.rgb_model_forward(self, images, rois, aux="full")

    def infer(self, images: torch.Tensor, rois: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
        """Logits [N,3,mh,mw] and the UNet logit map u [B,1,H,W], no aux tensors (serving path)."""
        logits, aux = engine.rgb_model_forward(self, images, rois, aux="none")
        return logits, aux["unet_logit"]


class RGBHierarchicalExportWrapper(nn.Module):
    """The exported ONNX contract (export_onnx_advanced.py:353-420, export_hierarchical_instance_peopleseg_onnx.py
    :85-181): images [B,3,H,W] in [0,1], rois [N,5] -> instance_masks [N,1,mh,mw], binary_masks [B,1,H,W].

    ROIAlign scales are set to (H, W) as _adjust_roi_align_spatial_scale does (:80-98).  The reference runs the
    full-image UNet twice (once for binary_masks, once inside the model); both passes are the same deterministic
    function of the image, so it is computed once here.
    """

    def __init__(self, model: HierarchicalRGBSegmentationModelWithFullImagePretrainedUNet, image_size=None,
                 dilation_pixels: int = 0):
        super().__init__()
        self.model = model
        self.image_size = image_size
        self.dilation_pixels = dilation_pixels

    def forward(self, images: torch.Tensor, rois: torch.Tensor):
        H, W = images.shape[-2:] if self.image_size is None else self.image_size
        for m in (self.model.roi_align_mask, self.model.roi_align_rgb):
            m.spatial_scale = (H, W)
            m.spatial_scale_h, m.spatial_scale_w = H, W
        if export.tracing(images, rois):
            return export.traced_export(self, images, rois)
        return engine.export_forward(self.model, images, rois, self.dilation_pixels)


class StreamPipelinedExport:
    """Serving schedule of the exported contract on two HIP streams: the full-image UNet of batch k+1 (HBM /
    latency-bound depthwise, SE and narrow decoder kernels) runs on one stream while the ROI head of batch k
    (MFMA-bound 256-channel convs) runs on the other, so the two kernel classes share the CUs instead of
    alternating.  Every batch still runs the complete contract; results are identical to
    ``RGBHierarchicalExportWrapper(model)(images, rois)`` per batch (same kernels, same inputs).

    ``run(batches)`` takes an iterable of (images, rois) and returns [(instance_masks, binary_masks), ...],
    ready on the caller's current stream when it returns (the caller synchronises as usual).
    """

    def __init__(self, wrapper: "RGBHierarchicalExportWrapper", unet_cu_mask=None, head_priority: bool = True,
                 gate: bool = False, gate_min_gflop: float = 300.0):
        """``unet_cu_mask``: optional list of 32-bit words; the UNet stream then runs only on the CUs whose bits
        are set (hiseg_stream_create_cu_mask), leaving the rest to the head.  ``head_priority``: the head -- the
        critical path once the UNet got cheaper -- runs on a high-priority stream, so its workgroups are dispatched
        ahead of the UNet's when both wait for CUs (tools/pipeline_ab.py, profiles/r2_v11_schedule_ab2.txt: 19.0-19.3
        vs 19.5-19.7 ms per step on one box, 19.35-19.6 vs 19.8-20.0 on another)."""
        self.wrapper = wrapper
        self._raw_unet = None
        if unet_cu_mask is None:
            self.s_unet = streams.role_stream("unet")
        else:
            import ctypes
            words = (ctypes.c_uint * len(unet_cu_mask))(*[int(w) & 0xFFFFFFFF for w in unet_cu_mask])
            h = ctypes.c_void_p()
            L.check(L.lib().hiseg_stream_create_cu_mask(words, len(unet_cu_mask), ctypes.byref(h)),
                    "stream_create_cu_mask")
            self._raw_unet = h.value
            self.s_unet = torch.cuda.ExternalStream(h.value)
        self.s_head = streams.role_stream("head" if head_priority else "head_normal")
        self.gate = gate
        self.gate_min_flops = gate_min_gflop * 1e9
        self._windows = None   # learned: light conv launches of the head between its heavy ones (gate=True)

    def __del__(self):
        if getattr(self, "_raw_unet", None):
            try:
                torch.cuda.synchronize()
                L.lib().hiseg_stream_destroy(self._raw_unet)
            except Exception:
                pass

    def run(self, batches):
        if self.gate:
            return self._run_gated(list(batches))
        w = self.wrapper
        caller = torch.cuda.current_stream()
        self.s_unet.wait_stream(caller)
        self.s_head.wait_stream(caller)
        outs = []
        for images, rois in batches:
            H, W = images.shape[-2:] if w.image_size is None else w.image_size
            for m in (w.model.roi_align_mask, w.model.roi_align_rgb):
                m.spatial_scale = (H, W)
                m.spatial_scale_h, m.spatial_scale_w = H, W
            with torch.cuda.stream(self.s_unet):
                u, binary = engine.export_unet_phase(w.model, images)
                ready = torch.cuda.Event()
                ready.record(self.s_unet)
            with torch.cuda.stream(self.s_head):
                self.s_head.wait_event(ready)
                u.record_stream(self.s_head)
                inst = engine.export_head_phase(w.model, images, rois, u, w.dilation_pixels)
            outs.append((inst, binary))
        caller.wait_stream(self.s_unet)
        caller.wait_stream(self.s_head)
        for inst, binary in outs:
            inst.record_stream(caller)
            binary.record_stream(caller)
        return outs

    def _set_scale(self, images):
        w = self.wrapper
        H, W = images.shape[-2:] if w.image_size is None else w.image_size
        for m in (w.model.roi_align_mask, w.model.roi_align_rgb):
            m.spatial_scale = (H, W)
            m.spatial_scale_h, m.spatial_scale_w = H, W

    def _run_gated(self, batches):
        """gate=True: the UNet of batch k+1 is issued in chunks (one per encoder / decoder block) from inside the head
        of batch k, into the windows between the head's heavy convs (>= gate_min_gflop: the 256-channel 3x3 layers
        at the ROI grid), and each heavy conv first waits for the chunks issued so far -- so the MFMA-bound heavy convs
        run with the chip to themselves and the latency-bound UNet kernels share it with the head's light kernels.
        Chunks are spread over the windows in proportion to the light conv launches each window held in the first
        batch (learned once).  Same kernels on the same inputs as run(): identical results."""
        from . import ops
        w = self.wrapper
        caller = torch.cuda.current_stream()
        self.s_unet.wait_stream(caller)
        self.s_head.wait_stream(caller)
        outs = []
        if not batches:
            return outs
        self._set_scale(batches[0][0])
        with torch.cuda.stream(self.s_unet):
            u, binary = engine._drain(engine.export_unet_phase_iter(w.model, batches[0][0]))
        for k, (images, rois) in enumerate(batches):
            ready = torch.cuda.Event()
            ready.record(self.s_unet)
            nxt = None
            if k + 1 < len(batches):
                self._set_scale(batches[k + 1][0])
                nxt = engine.export_unet_phase_iter(w.model, batches[k + 1][0])
            self._set_scale(images)
            g = _HeadGate(self, nxt)
            with torch.cuda.stream(self.s_head):
                self.s_head.wait_event(ready)
                u.record_stream(self.s_head)
                ops.GATE = g
                try:
                    inst = engine.export_head_phase(w.model, images, rois, u, w.dilation_pixels)
                finally:
                    ops.GATE = None
            outs.append((inst, binary))
            if nxt is not None:
                u, binary = g.finish()
            if self._windows is None:
                self._windows = g.counts + [0]
        caller.wait_stream(self.s_unet)
        caller.wait_stream(self.s_head)
        for inst, binary in outs:
            inst.record_stream(caller)
            binary.record_stream(caller)
        return outs


class _HeadGate:
    """ops.GATE during one head phase of StreamPipelinedExport(gate=True): feeds the next batch's UNet chunks into
    the windows between heavy convs (see StreamPipelinedExport._run_gated)."""

    def __init__(self, runner: StreamPipelinedExport, gen):
        self.r, self.gen = runner, gen
        self.min_flops = runner.gate_min_flops
        self.counts = [0]            # light launches per window (window i ends at heavy conv i)
        self.window = 0
        self.done = gen is None
        self.result = None
        self.issued = 0
        self.last = None             # event after the latest chunk on the UNet stream
        w = runner._windows
        if w is not None and gen is not None:   # chunk budget per window, proportional to its light launches
            tot = max(sum(w), 1)
            self.share = [c / tot for c in w]
        else:
            self.share = None
        self._issue_window()         # window 0: the head's opening (RoIAlign, feature extractor, ...)

    def _chunks_for(self, i):
        if self.share is None:       # first batch: one chunk per window
            return 1
        # cumulative target after window i, against ~24 chunks of a B0 UNet (the rest drains after the head)
        return max(0, round(24 * sum(self.share[:i + 1])) - self.issued)

    def _issue(self, n):
        from . import ops
        if self.done or n <= 0:
            return
        s = self.r.s_unet
        prev, ops.GATE = ops.GATE, None
        try:
            with torch.cuda.stream(s):
                for _ in range(n):
                    try:
                        next(self.gen)
                        self.issued += 1
                    except StopIteration as e:
                        self.result = e.value
                        self.done = True
                        break
                self.last = torch.cuda.Event()
                self.last.record(s)
        finally:
            ops.GATE = prev

    def _issue_window(self):
        self._issue(self._chunks_for(self.window))

    def light(self):
        self.counts[-1] += 1

    def before(self):
        if self.last is not None:   # the chunks issued so far finish before the heavy conv starts
            torch.cuda.current_stream().wait_event(self.last)

    def after(self):
        self.window += 1
        self.counts.append(0)
        if self.done:
            return
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream())
        self.r.s_unet.wait_event(ev)
        self._issue_window()

    def finish(self):
        """Issue the rest of the UNet (after the head) and return (u, binary_masks) of the next batch."""
        while not self.done:
            self._issue(64)
        return self.result


def create_rgb_hierarchical_model(roi_size=28, mask_size=56, multi_scale: bool = False,
                                  activation_function: str = "relu", activation_beta: float = 1.0,
                                  normalization_type: str = "layernorm2d", normalization_groups: int = 8,
                                  **kwargs) -> nn.Module:
    """Factory of advanced/hierarchical_segmentation_rgb.py:925-1027 (full-image pretrained-UNet branch)."""
    use_attention_module = kwargs.pop("use_attention_module", False)
    flags = {k: kwargs.pop(k, False) for k in ("use_boundary_refinement", "use_progressive_upsampling",
                                               "use_subpixel_conv", "use_contour_detection", "use_distance_transform")}
    use_pretrained_unet = kwargs.pop("use_pretrained_unet", False)
    pretrained_weights_path = kwargs.pop("pretrained_weights_path", "")
    freeze = kwargs.pop("freeze_pretrained_weights", False)
    full_image = kwargs.pop("use_full_image_unet", False)
    kwargs.pop("roi_sizes", None)
    kwargs.pop("fusion_method", None)
    if multi_scale or not (use_pretrained_unet and full_image):
        raise NotImplementedError(
            "hiseg implements the full-image pretrained-UNet RGB hierarchical model (the BASELINE.json hot path); "
            "multi-scale / ROI-UNet / plain RGB variants are out of scope (SURVEY.md §2.1)")
    return HierarchicalRGBSegmentationModelWithFullImagePretrainedUNet(
        roi_size=roi_size, mask_size=mask_size, pretrained_weights_path=pretrained_weights_path,
        use_attention_module=use_attention_module, freeze_pretrained_weights=freeze,
        normalization_type=normalization_type, normalization_groups=normalization_groups,
        activation_function=activation_function, activation_beta=activation_beta, **flags, **kwargs)
