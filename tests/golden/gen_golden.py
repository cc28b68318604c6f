"""Generate golden input/output vectors by running the REFERENCE implementation on CPU.

Run in the build container only (the reference is at /root/reference and never leaves it):
    python tests/golden/gen_golden.py
Writes tests/golden/*.npz and configs.json.  The fixtures are data (inputs + expected outputs);
weights are not stored: both sides regenerate them with tests/golden/filler.py.

segmentation_models_pytorch (smp 0.5.0) is absent from this image, so the full model is built with
a stand-in ``segmentation_models_pytorch`` module whose ``Unet`` has no parameters and returns a
logit map injected by this script: the reference's own forward (normalize_input, output_conv,
both DynamicRoIAlign calls, rgb_feature_extractor, concat, feature_combiner, refined head) runs
unchanged with the UNet output as an input.  The EfficientNet-UNet itself stays parity-unpinned.
"""
import json
import os
import sys
import types

import numpy as np
import torch
import torch.nn as nn

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"
sys.path.insert(0, HERE)
sys.path.insert(0, REF)
import filler  # noqa: E402

torch.set_num_threads(os.cpu_count())
torch.manual_seed(0)


class _InjectedUnet(nn.Module):
    injected = None

    def __init__(self, encoder_name=None, classes=1, encoder_weights=None, **kw):
        super().__init__()

    def forward(self, x):
        return _InjectedUnet.injected


_smp = types.ModuleType("segmentation_models_pytorch")
_smp.Unet = _InjectedUnet
sys.modules["segmentation_models_pytorch"] = _smp

from src.human_edge_detection.dynamic_roi_align import DynamicRoIAlign  # noqa: E402
from src.human_edge_detection.advanced import hierarchical_segmentation_refinement as R  # noqa: E402
from src.human_edge_detection.advanced import hierarchical_segmentation_unet as U  # noqa: E402
from src.human_edge_detection.advanced.hierarchical_segmentation_rgb import create_rgb_hierarchical_model  # noqa: E402
from src.human_edge_detection.experiments.config_manager import ConfigManager  # noqa: E402

PRESETS = {
    "b0": "rgb_hierarchical_unet_v2_fullimage_pretrained_peopleseg_r64x48m128x96_disttrans_contdet_baware_from_B0",
    "b1": "rgb_hierarchical_unet_v2_fullimage_pretrained_peopleseg_r80x60m160x120_disttrans_contdet_baware_from_B1_enhanced",
    "b7": "rgb_hierarchical_unet_v2_fullimage_pretrained_peopleseg_r128x96m256x192_disttrans_contdet_baware_from_B7_enhanced",
    "distill": "rgb_hierarchical_unet_v2_distillation_b0_from_b7_temp_prog",
}


def model_kwargs(cfg):
    """The keyword arguments train_advanced.build_model (:123-162) passes for an RGB hierarchical config."""
    m = cfg.model
    enc = cfg.distillation.student_encoder if cfg.distillation.enabled else getattr(m, "encoder_name", "timm-efficientnet-b3")
    g = lambda k, d: getattr(m, k, d)  # noqa: E731
    return dict(
        roi_size=list(m.roi_size) if isinstance(m.roi_size, (list, tuple)) else m.roi_size,
        mask_size=list(m.mask_size) if isinstance(m.mask_size, (list, tuple)) else m.mask_size,
        multi_scale=False, use_attention_module=m.use_attention_module,
        use_boundary_refinement=g("use_boundary_refinement", False), use_progressive_upsampling=g("use_progressive_upsampling", False),
        use_subpixel_conv=g("use_subpixel_conv", False), use_contour_detection=g("use_contour_detection", False),
        use_distance_transform=g("use_distance_transform", False), normalization_type=g("normalization_type", "layernorm2d"),
        normalization_groups=g("normalization_groups", 8), activation_function=g("activation_function", "relu"),
        activation_beta=g("activation_beta", 1.0), use_pretrained_unet=g("use_pretrained_unet", False),
        pretrained_weights_path=g("pretrained_weights_path", ""), freeze_pretrained_weights=g("freeze_pretrained_weights", False),
        use_full_image_unet=g("use_full_image_unet", False), encoder_name=enc,
        hierarchical_base_channels=g("hierarchical_base_channels", 96), hierarchical_depth=g("hierarchical_depth", 3))


def tup(v):
    return tuple(v) if isinstance(v, list) else v


def save(name, **arrays):
    path = os.path.join(HERE, name + ".npz")
    np.savez_compressed(path, **{k: (v.detach().cpu().numpy() if torch.is_tensor(v) else np.asarray(v)) for k, v in arrays.items()})
    print(f"wrote {path} ({os.path.getsize(path) / 1024:.0f} KiB)")


def gen_roi_align():
    cases = {}
    feat = torch.from_numpy(filler.uniform(11, (2, 3, 24, 32)))
    rois = torch.tensor([[0, .10, .10, .40, .90], [1, .35, .15, .60, .95], [0, .0, .0, 1.0, 1.0],
                         [1, .70, .30, .95, .99], [0, .5, .5, .5, .5], [1, .9, .05, 1.0, .2]], dtype=torch.float32)
    for i, (oh, ow, scale, aligned) in enumerate([(16, 12, (24, 32), True), (7, 5, (24, 32), False), (1, 1, (24, 32), True),
                                                  (16, 12, 32, True), (9, 13, (24, 32), True)]):
        m = DynamicRoIAlign(spatial_scale=scale, sampling_ratio=2, aligned=aligned)
        out = m(feat, rois, oh, ow)
        cases[f"c{i}_out"] = out
        cases[f"c{i}_meta"] = np.array([oh, ow, scale[0] if isinstance(scale, tuple) else scale,
                                        scale[1] if isinstance(scale, tuple) else scale, int(aligned)], dtype=np.float32)
    feat2 = torch.from_numpy(filler.normal(12, (1, 2, 20, 20)))
    rois2 = torch.tensor([[0, .05, .05, .95, .95], [0, .2, .3, .4, .31]], dtype=torch.float32)
    out2 = DynamicRoIAlign(spatial_scale=20, aligned=True)(feat2, rois2, 6, 4)
    save("roi_align", feat=feat, rois=rois, feat2=feat2, rois2=rois2, out2=out2, **cases)


def gen_blocks():
    blk = filler.fill_module(R.ResidualBlock(64, "batchnorm", 8, "relu", 1.0)).eval()
    x = torch.from_numpy(filler.normal(21, (2, 64, 12, 10)))
    with torch.no_grad():
        y = blk(x)
    unet = filler.fill_module(U.EnhancedUNet(256, base_channels=64, depth=3, normalization_type="batchnorm",
                                             normalization_groups=8, activation_function="relu")).eval()
    xu = torch.from_numpy(filler.normal(22, (2, 256, 16, 12)))
    with torch.no_grad():
        yu = unet(xu)
    save("blocks", res_x=x, res_y=y, unet_x=xu, unet_y=yu)


def head_kwargs(kw):
    return dict(in_channels=256, mid_channels=256, num_classes=3,
                mask_size=tup(kw["mask_size"]) if tup(kw["mask_size"])[0] != tup(kw["mask_size"])[1] else tup(kw["mask_size"])[0],
                use_attention_module=kw["use_attention_module"], use_contour_detection=kw["use_contour_detection"],
                use_distance_transform=kw["use_distance_transform"], normalization_type=kw["normalization_type"],
                normalization_groups=kw["normalization_groups"], activation_function=kw["activation_function"],
                activation_beta=kw["activation_beta"], hierarchical_base_channels=kw["hierarchical_base_channels"],
                hierarchical_depth=kw["hierarchical_depth"])


def summarize(prefix, aux, out):
    for k, v in aux.items():
        if v.numel() > 400_000:  # large feature maps: per-channel means + a strided sample
            out[f"{prefix}{k}__chmean"] = v.mean(dim=(0, 2, 3))
            out[f"{prefix}{k}__sample"] = v.reshape(-1)[::997]
        else:
            out[f"{prefix}{k}"] = v


def gen_head(kw):
    head = filler.fill_module(R.RefinedHierarchicalSegmentationHead(**head_kwargs(kw))).eval()
    x = torch.from_numpy(filler.normal(31, (2, 256) + tuple(tup(kw["roi_size"]))))
    with torch.no_grad():
        logits, aux = head(x)
    out = {"logits": logits}  # input regenerated from filler.normal(31, ...) by the tests
    summarize("aux_", aux, out)
    save("head_b0", **out)


def build_ref_model(kw):
    kw = dict(kw)
    kw["roi_size"], kw["mask_size"] = tup(kw["roi_size"]), tup(kw["mask_size"])
    model = create_rgb_hierarchical_model(**kw)
    return filler.fill_module(model).eval()


def gen_model(kw):
    model = build_ref_model(kw)
    out = {}
    # (a) export-style scale (H, W) on a small image
    images = torch.from_numpy(filler.uniform(41, (2, 3, 96, 128)))
    u = torch.from_numpy(filler.normal(42, (2, 1, 96, 128)) * 2.0)
    rois = torch.tensor([[0, .10, .10, .40, .90], [1, .35, .15, .80, .95], [0, .55, .05, .95, .70]], dtype=torch.float32)
    for m in (model.roi_align_mask, model.roi_align_rgb):
        m.spatial_scale, m.spatial_scale_h, m.spatial_scale_w = (96, 128), 96, 128
    _InjectedUnet.injected = u
    with torch.no_grad():
        logits, aux = model(images, rois)
    out.update(images=images, u=u, rois=rois, logits=logits)
    summarize("aux_", aux, out)
    # (b) training semantics: scalar spatial_scale 640 on 640x640 inputs regenerated from seeds in the tests
    for m in (model.roi_align_mask, model.roi_align_rgb):
        m.spatial_scale, m.spatial_scale_h, m.spatial_scale_w = 640.0, 640.0, 640.0
    images640 = torch.from_numpy(filler.uniform(43, (1, 3, 640, 640)))
    u640 = torch.from_numpy(filler.normal(44, (1, 1, 640, 640)) * 2.0)
    rois640 = torch.from_numpy(filler.box_rois(45, 1, 2))
    _InjectedUnet.injected = u640
    with torch.no_grad():
        logits640, _ = model(images640, rois640)
    out.update(rois640=rois640, logits640=logits640)
    save("model_b0", **out)
    return model


def gen_configs():
    cfgs = {}
    for key, name in PRESETS.items():
        cfg = ConfigManager.get_config(name)
        cfgs[key] = {"name": name, "model_kwargs": model_kwargs(cfg), "config": cfg.to_dict()}
    path = os.path.join(HERE, "configs.json")
    with open(path, "w") as f:
        json.dump(cfgs, f, indent=1, default=str)
    print("wrote", path)
    return cfgs


def gen_state_keys(kw):
    model = build_ref_model(kw)
    keys = [k for k in model.state_dict().keys()]
    with open(os.path.join(HERE, "state_keys_b0_head.json"), "w") as f:
        json.dump(keys, f, indent=0)
    print("state keys", len(keys))


# Normalisation / activation variants of the factory (normalization_comparison.py:159-206,
# activation_utils.py:71-101): the presets all use batchnorm + relu; these pin layernorm2d, GELU and
# Swish(beta != 1) on the same modules.  `python tests/golden/gen_golden.py variants` -> variants.npz
VARIANTS = {"ln_gelu": ("layernorm2d", "gelu", 1.0), "bn_swish": ("batchnorm", "swish", 1.5),
            "ln_swish": ("layernorm2d", "swish", 0.75)}


def small_head_kwargs(norm, act, beta):
    return dict(in_channels=64, mid_channels=64, num_classes=3, mask_size=(32, 24), use_attention_module=True,
                use_contour_detection=True, use_distance_transform=True, normalization_type=norm,
                normalization_groups=8, activation_function=act, activation_beta=beta,
                hierarchical_base_channels=32, hierarchical_depth=3)


def gen_variants(kw):
    out = {}
    x = torch.from_numpy(filler.normal(61, (2, 64, 12, 10)))
    xu = torch.from_numpy(filler.normal(62, (2, 64, 16, 12)))
    xh = torch.from_numpy(filler.normal(63, (2, 64, 16, 12)))
    for key, (norm, act, beta) in VARIANTS.items():
        blk = filler.fill_module(R.ResidualBlock(64, norm, 8, act, beta)).eval()
        unet = filler.fill_module(U.EnhancedUNet(64, base_channels=32, depth=3, normalization_type=norm,
                                                 normalization_groups=8, activation_function=act,
                                                 activation_beta=beta)).eval()
        head = filler.fill_module(R.RefinedHierarchicalSegmentationHead(**small_head_kwargs(norm, act, beta))).eval()
        with torch.no_grad():
            out[f"{key}_res_y"] = blk(x)
            out[f"{key}_unet_y"] = unet(xu)
            logits, aux = head(xh)
        out[f"{key}_head_logits"] = logits
        summarize(f"{key}_head_aux_", aux, out)
    # the whole ROI path (rgb_feature_extractor, feature_combiner, full-size head) with layernorm2d + GELU
    mkw = dict(kw, normalization_type="layernorm2d", activation_function="gelu")
    model = build_ref_model(mkw)
    images = torch.from_numpy(filler.uniform(64, (2, 3, 96, 128)))
    u = torch.from_numpy(filler.normal(65, (2, 1, 96, 128)) * 2.0)
    rois = torch.tensor([[0, .10, .10, .40, .90], [1, .35, .15, .80, .95]], dtype=torch.float32)
    for m in (model.roi_align_mask, model.roi_align_rgb):
        m.spatial_scale, m.spatial_scale_h, m.spatial_scale_w = (96, 128), 96, 128
    _InjectedUnet.injected = u
    with torch.no_grad():
        logits, _ = model(images, rois)
    out.update(model_images=images, model_u=u, model_rois=rois, model_logits=logits)
    save("variants", **out)


def _import_export_script():
    """export_hierarchical_instance_peopleseg_onnx (reference root) for MaskDilationModule / ModelWithDilation.
    Its import chain (export_onnx_advanced, train_advanced) pulls in packages absent from this image -- onnx,
    onnxruntime, tensorboard, pycocotools, cv2, seaborn -- none of which the dilation path executes: they are
    stubbed as empty modules for the import only."""
    class _Stub(types.ModuleType):
        def __getattr__(self, k):
            if k.startswith("__"):
                raise AttributeError(k)
            return type(k, (), {"__init__": lambda s, *a, **kw: None})

    for name in ("onnx", "onnxruntime", "onnxsim", "pycocotools", "pycocotools.coco", "pycocotools.mask", "cv2",
                 "seaborn", "torch.utils.tensorboard"):
        if name not in sys.modules:
            m = _Stub(name)
            m.__path__ = []
            sys.modules[name] = m
    import export_hierarchical_instance_peopleseg_onnx as E  # noqa: E402
    return E


def gen_export(kw):
    """ModelWithDilation (export_hierarchical_instance_peopleseg_onnx.py:144-181) around the reference model at
    dilation 0 / 1 / 2, the instance masks of the export wrapper (export_onnx_advanced.py:358-362: argmax == 1)
    and its binary masks (:374-387: softmax of pretrained_unet(images), channel 0); MaskDilationModule alone on
    synthetic logits with larger radii."""
    E = _import_export_script()
    model = build_ref_model(kw)
    images = torch.from_numpy(filler.uniform(71, (2, 3, 96, 128)))
    u = torch.from_numpy(filler.normal(72, (2, 1, 96, 128)) * 2.0)
    rois = torch.from_numpy(filler.box_rois(73, 2, 3))
    for m in (model.roi_align_mask, model.roi_align_rgb):
        m.spatial_scale, m.spatial_scale_h, m.spatial_scale_w = (96, 128), 96, 128
    _InjectedUnet.injected = u
    out = dict(rois=rois)   # images / u are regenerated from the filler seeds by the tests
    with torch.no_grad():
        for d in (0, 1, 2):
            o = E.ModelWithDilation(model, d)(images, rois)
            masks = o[0] if isinstance(o, tuple) else o
            if d == 0:
                out["d0_logits"] = masks
            out[f"d{d}_instance"] = (torch.argmax(masks, dim=1, keepdim=True) == 1).to(torch.uint8)
        pu = model.pretrained_unet(images)
        pu = pu[0] if isinstance(pu, tuple) else pu
        out["binary"] = torch.softmax(pu, dim=1)[:, 0:1]
        z = torch.from_numpy(filler.normal(74, (3, 3, 20, 16)) * 3.0)
        out["syn_logits"] = z
        for d in (1, 2, 3):
            out[f"syn_d{d}"] = E.MaskDilationModule(d)(z)
    save("export", **out)


if __name__ == "__main__" and sys.argv[1:] == ["export"]:
    gen_export(gen_configs()["b0"]["model_kwargs"])
elif __name__ == "__main__" and sys.argv[1:] == ["variants"]:
    gen_variants(gen_configs()["b0"]["model_kwargs"])
elif __name__ == "__main__":
    cfgs = gen_configs()
    kw = cfgs["b0"]["model_kwargs"]
    gen_roi_align()
    gen_blocks()
    gen_state_keys(kw)
    gen_head(kw)
    gen_model(kw)
