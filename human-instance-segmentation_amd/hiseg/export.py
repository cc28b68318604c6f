"""Traceable surface of the hiseg modules: torch.library custom ops, fake (shape) kernels, ONNX symbolics.

The reference exports by calling ``torch.onnx.export`` on its nn.Modules (export_onnx_advanced.py:338-457,
export_hierarchical_instance_peopleseg_onnx.py:415-460): its wrapper calls ``model.pretrained_unet(images)`` and
``model(images, rois)`` and post-processes with plain torch ops.  hiseg's forwards run through ctypes, which no
tracer can see, so while a forward is being traced (torch.export / dynamo fake tensors, torch.jit.trace) each
module forward instead calls one custom op per reference module boundary:

  hiseg::unet_logit         PreTrainedPeopleSegmentationUNet.forward          (unet.py:1885-1916)   -> u [B,1,H,W]
  hiseg::output_conv        PreTrainedPeopleSegmentationUNetWrapper's 1->2 1x1 (unet.py:1976-1993)  -> [B,2,H,W]
  hiseg::dynamic_roi_align  DynamicRoIAlign.forward                           (dynamic_roi_align.py:56-171)
  hiseg::rgb_head           HierarchicalRGBSegmentationModelWithFullImagePretrainedUNet.forward after the UNet
                            (rgb.py:729-774): both RoIAligns, RGB extractor, combiner, refined head -> logits + aux
  hiseg::instance_masks     RGBHierarchicalWrapper._to_instance_masks (+ MaskDilationModule)
                            (export_onnx_advanced.py:360-364; export_hierarchical_instance_peopleseg_onnx.py:85-141)
  hiseg::binary_masks       softmax(output_conv(u))[:, 0:1]                   (export_onnx_advanced.py:374-387)

Every op's real kernel is the same libhiseg path the eager forward takes (there is no CPU kernel: a CPU call
fails like the eager forward does); its fake kernel only computes output shapes, so ``torch.export.export`` traces
a hiseg model on CPU, with symbolic batch and ROI counts.  Ops that carry a module take the module's state
(parameters + buffers, state_dict order) as a ``Tensor[]`` input -- the exported graph owns the weights -- plus a
JSON ``spec`` with the module's constructor arguments and the forward's non-tensor attributes (compute dtype,
RoIAlign scales, aux keys and their shape templates).  The real kernel rebuilds a parameter-free skeleton of the
module from the spec once per process and runs the engine on it with the passed tensors swapped in, so an
exported program runs after ``torch.export.save`` / ``load`` in a fresh process too.

ONNX: :func:`register_onnx_symbolics` maps each op for the TorchScript exporter (``torch.onnx.export(...,
dynamo=False, custom_opsets={"hiseg": 1})``).  dynamic_roi_align, output_conv, binary_masks and instance_masks
lower to standard ONNX ops (Gather / GridSample / Conv / Softmax / MaxPool / ArgMax ... -- the reference's own
decomposition, opset >= 16); unet_logit and rgb_head become nodes of the documented custom domain ``hiseg``
(inputs: the tensors, then the state; string attribute ``spec``), which a runtime implements with libhiseg
(INTEGRATION.md "Export").  The onnx package is not installed in this image, so the serialised model is not
checked here; tests/test_export.py runs each standard-op lowering through an eager ONNX-semantics interpreter
against the oracle instead.
"""
from __future__ import annotations

import json
import threading
import weakref
from typing import Dict, List, Sequence, Tuple

import torch
from torch import Tensor

from . import _lib as L

_DTYPES = {"f32": torch.float32, "bf16": torch.bfloat16}
_DTYPE_NAMES = {v: k for k, v in _DTYPES.items()}


# ------------------------------------------------------------------------------------ tracing detection
def tracing(*tensors) -> bool:
    """True while a tracer (dynamo / torch.export / torch.jit.trace) is running or the inputs are fake."""
    if torch.compiler.is_compiling() or torch.jit.is_tracing():
        return True
    from torch._subclasses.fake_tensor import is_fake
    return any(isinstance(t, Tensor) and is_fake(t) for t in tensors)


def record_init(module: torch.nn.Module, **kwargs) -> None:
    """Remember the constructor arguments a skeleton of ``module`` is rebuilt from (weights excluded)."""
    module.__dict__["_hiseg_init"] = (type(module).__name__, kwargs)


def _dtype_name(m: torch.nn.Module) -> str:
    return _DTYPE_NAMES[getattr(m, "hiseg_dtype", torch.float32)]


def _spec(module: torch.nn.Module, **extra) -> str:
    name, kwargs = module.__dict__["_hiseg_init"]
    return json.dumps({"cls": name, "init": kwargs, "dtype": _dtype_name(module), **extra}, sort_keys=True)


def _state(module: torch.nn.Module, skip: str = "") -> List[Tensor]:
    return [t for k, t in module.state_dict(keep_vars=True).items() if not (skip and k.startswith(skip))]


# ------------------------------------------------------------------------------------ skeletons (real kernels)
# spec key -> (skeleton module, its lock).  One skeleton serves every exported program of that architecture; the
# engine's plan cache on it (packed weights, folded BN tables: engine.Ctx, root.__dict__['_hiseg_plans']) is keyed
# by the (address, version) of the state tensors, which the plans themselves do not hold.  So the skeleton holds the
# state set it last ran with, and a call with another state set (a different exported program, or the same one
# reloaded) drops the plans first: addresses of a released program cannot come back under the same version and
# make another program's weights run.  The lock covers swap-in + run: two threads on one skeleton would otherwise
# overwrite each other's parameters mid-forward.
_SKELETONS: Dict[str, Tuple[torch.nn.Module, threading.Lock]] = {}
_SKELETON_LOCK = threading.Lock()


def _skeleton(spec: dict) -> Tuple[torch.nn.Module, threading.Lock]:
    key = json.dumps({k: spec[k] for k in ("cls", "init", "dtype")}, sort_keys=True)
    with _SKELETON_LOCK:
        ent = _SKELETONS.get(key)
        if ent is None:
            from . import model as M
            cls = {c.__name__: c for c in (M.PreTrainedPeopleSegmentationUNet,
                                           M.HierarchicalRGBSegmentationModelWithFullImagePretrainedUNet)}[spec["cls"]]
            with torch.device("meta"):
                m = cls(**spec["init"])
            m = m.to_empty(device="cpu").eval()   # storage is replaced by the op's state tensors on every call
            for mm in m.modules():
                mm.hiseg_dtype = _DTYPES[spec["dtype"]]
            ent = _SKELETONS[key] = (m, threading.Lock())
    return ent


def _run_on(spec: dict, state: Sequence[Tensor], skip: str, fn):
    m, lock = _skeleton(spec)
    names = [k for k in m.state_dict().keys() if not (skip and k.startswith(skip))]
    if len(names) != len(state):
        raise ValueError(f"hiseg export op: {len(state)} state tensors for a {spec['cls']} with {len(names)}")
    from torch.nn.utils.stateless import _reparametrize_module
    ident = tuple(t.data_ptr() for t in state)
    with lock:
        # The plans (packed weights) are keyed on the state's addresses.  Weak references tell whether the tensors
        # that owned them are still alive: if any died, the same address may now hold another program's weights, so
        # nothing carries over.  A released program's weights are not pinned by the skeleton.
        refs = m.__dict__.get("_hiseg_state_refs")
        same = (m.__dict__.get("_hiseg_state_ident") == ident and refs is not None
                and all(r() is not None for r in refs))
        if not same:
            m.__dict__.pop("_hiseg_plans", None)
            m.__dict__["_hiseg_state_ident"] = ident
            m.__dict__["_hiseg_state_refs"] = [weakref.ref(t) for t in state]
        with _reparametrize_module(m, dict(zip(names, state))):
            return fn(m)


def _shape(template, env: dict):
    return [env[d] if isinstance(d, str) else d for d in template]


# ------------------------------------------------------------------------------------ ops
@torch.library.custom_op("hiseg::unet_logit", mutates_args=())
def unet_logit(images: Tensor, state: List[Tensor], spec: str) -> Tensor:
    """PreTrainedPeopleSegmentationUNet.forward on libhiseg: images [B,3,H,W] -> u [B,1,H,W] f32."""
    from . import engine
    return _run_on(json.loads(spec), state, "", lambda m: engine.unet_logits_nchw(m, images))


@unet_logit.register_fake
def _(images, state, spec):
    B, _, H, W = images.shape
    return images.new_empty((B, 1, H, W), dtype=torch.float32)


@torch.library.custom_op("hiseg::output_conv", mutates_args=())
def output_conv(u: Tensor, weight: Tensor, bias: Tensor) -> Tensor:
    """The wrapper's trainable 1->2 1x1 conv (hiseg_output_conv_fwd): u [B,1,H,W] -> [B,2,H,W] f32."""
    engine_check(u, "output_conv")
    B, _, H, W = u.shape
    out = torch.empty(B, 2, H, W, dtype=torch.float32, device=u.device)
    w = weight.detach().float().reshape(2).contiguous()
    b = bias.detach().float().contiguous()
    L.check(L.lib().hiseg_output_conv_fwd(u.contiguous().data_ptr(), B, H, W, w.data_ptr(), b.data_ptr(),
                                          out.data_ptr(), L.stream_ptr()), "output_conv")
    return out


@output_conv.register_fake
def _(u, weight, bias):
    B, _, H, W = u.shape
    return u.new_empty((B, 2, H, W), dtype=torch.float32)


@torch.library.custom_op("hiseg::dynamic_roi_align", mutates_args=())
def dynamic_roi_align(feat: Tensor, rois: Tensor, output_height: int, output_width: int, scale_h: float,
                      scale_w: float, aligned: bool) -> Tensor:
    """DynamicRoIAlign.forward on libhiseg: feat [B,C,H,W], rois [N,5] -> [N,C,oh,ow] f32."""
    from . import ops
    engine_check(feat, "DynamicRoIAlign")
    feat = feat.contiguous().float()
    out = torch.empty(rois.shape[0], feat.shape[1], output_height, output_width, dtype=torch.float32,
                      device=feat.device)
    ops.roi_align(feat, rois.to(feat.device), output_height, output_width, scale_h, scale_w, aligned, nchw_out=out)
    return out


@dynamic_roi_align.register_fake
def _(feat, rois, output_height, output_width, scale_h, scale_w, aligned):
    return feat.new_empty((rois.shape[0], feat.shape[1], output_height, output_width), dtype=torch.float32)


@torch.library.custom_op("hiseg::rgb_head", mutates_args=())
def rgb_head(images: Tensor, u: Tensor, rois: Tensor, state: List[Tensor], spec: str) -> List[Tensor]:
    """The RGB hierarchical model's forward from the UNet logit u on: [logits, *aux in spec['outs'] order]."""
    from . import engine
    sp = json.loads(spec)

    def run(m):
        for mm in (m.roi_align_mask, m.roi_align_rgb):
            mm.spatial_scale_h, mm.spatial_scale_w = sp["scale_hw"]
        logits, aux = engine.rgb_model_forward(m, images, rois, aux=sp["aux"], unet_logit_override=u)
        aux["logits"] = logits
        return [aux[name] for name, _ in sp["outs"]]
    return _run_on(sp, state, UNET_PREFIX, run)


@rgb_head.register_fake
def _(images, u, rois, state, spec):
    sp = json.loads(spec)
    env = {"N": rois.shape[0], "B": images.shape[0], "H": images.shape[2], "W": images.shape[3]}
    return [images.new_empty(_shape(t, env), dtype=torch.float32) for _, t in sp["outs"]]


@torch.library.custom_op("hiseg::instance_masks", mutates_args=())
def instance_masks(logits: Tensor, dilation: int) -> Tensor:
    """argmax(logits) == 1 as float, after the optional mask dilation: [N,3,mh,mw] -> [N,1,mh,mw]."""
    from . import ops
    engine_check(logits, "instance_masks")
    return ops.instance_masks(logits.float(), dilation)


@instance_masks.register_fake
def _(logits, dilation):
    N, _, mh, mw = logits.shape
    return logits.new_empty((N, 1, mh, mw), dtype=torch.float32)


@torch.library.custom_op("hiseg::binary_masks", mutates_args=())
def binary_masks(u: Tensor, weight: Tensor, bias: Tensor) -> Tensor:
    """softmax(output_conv(u))[:, 0:1] (foreground probability): u [B,1,H,W] -> [B,1,H,W]."""
    from . import ops
    engine_check(u, "binary_masks")
    return ops.binary_masks(u.contiguous().float(), weight.detach().float().reshape(2).contiguous(),
                            bias.detach().float().contiguous())


@binary_masks.register_fake
def _(u, weight, bias):
    B, _, H, W = u.shape
    return u.new_empty((B, 1, H, W), dtype=torch.float32)


def engine_check(x: Tensor, what: str):
    if not x.is_cuda:
        raise RuntimeError(f"{what}: hiseg runs on the GPU only (got a CPU tensor); there is no CPU fallback")


# ------------------------------------------------------------------------------------ traced module forwards
UNET_PREFIX = "pretrained_unet.model."


def traced_unet_logit(pre: torch.nn.Module, images: Tensor) -> Tensor:
    return torch.ops.hiseg.unet_logit(images, _state(pre), _spec(pre))


def traced_unet_wrapper(wrapper: torch.nn.Module, images: Tensor) -> Tensor:
    u = traced_unet_logit(wrapper.model, images)
    return torch.ops.hiseg.output_conv(u, wrapper.output_conv.weight, wrapper.output_conv.bias)


def traced_roi_align(m: torch.nn.Module, feat: Tensor, rois: Tensor, oh: int, ow: int) -> Tensor:
    return torch.ops.hiseg.dynamic_roi_align(feat, rois, int(oh), int(ow), float(m.spatial_scale_h),
                                             float(m.spatial_scale_w), bool(m.aligned))


def rgb_out_templates(model: torch.nn.Module, aux: str) -> List[Tuple[str, list]]:
    """Output names and shapes (symbols N, B, H, W) of engine.rgb_model_forward for one aux mode."""
    (rh, rw), (mh, mw) = model.roi_size, model.mask_size
    outs = [("logits", ["N", 3, mh, mw])]
    if aux != "full":
        return outs
    head = model.segmentation_head
    m = head.base_head.shared_features[0].out_channels
    outs += [("bg_fg_logits", ["N", 2, mh, mw]), ("bg_fg_logits_low", ["N", 2, rh, rw]),
             ("target_nontarget_logits", ["N", 2, mh, mw]), ("fg_attention", ["N", m, rh, rw]),
             ("shared_features", ["N", m, rh, rw])]
    if head.use_contour_detection:
        outs.append(("contours", ["N", 1, mh, mw]))
    if head.use_distance_transform:
        outs += [("distance_mask", ["N", 1, mh, mw]), ("distance_map", ["N", 1, mh, mw])]
    outs += [("full_image_logits", ["B", 2, "H", "W"]), ("roi_features", ["N", 2, rh, rw]),
             ("roi_patches", ["N", 3, rh, rw])]
    return outs


def _head_spec(model: torch.nn.Module, aux: str) -> str:
    ma, mr = model.roi_align_mask, model.roi_align_rgb
    scales = [float(ma.spatial_scale_h), float(ma.spatial_scale_w)]
    if [float(mr.spatial_scale_h), float(mr.spatial_scale_w)] != scales or not (ma.aligned and mr.aligned):
        raise NotImplementedError("traced export needs both RoIAligns aligned=True with one spatial scale")
    return _spec(model, aux=aux, scale_hw=scales, outs=rgb_out_templates(model, aux))


def traced_rgb_model(model: torch.nn.Module, images: Tensor, rois: Tensor, aux: str = "full"):
    u = traced_unet_logit(model.pretrained_unet.model, images)
    outs = torch.ops.hiseg.rgb_head(images, u, rois, _state(model, UNET_PREFIX), _head_spec(model, aux))
    names = [n for n, _ in rgb_out_templates(model, aux)]
    d = dict(zip(names, outs))
    logits = d.pop("logits")
    if aux != "full":
        d["unet_logit"] = u
    return logits, d


def traced_export(wrapper: torch.nn.Module, images: Tensor, rois: Tensor):
    model = wrapper.model
    u = traced_unet_logit(model.pretrained_unet.model, images)
    oc = model.pretrained_unet.output_conv
    binary = torch.ops.hiseg.binary_masks(u, oc.weight, oc.bias)
    logits = torch.ops.hiseg.rgb_head(images, u, rois, _state(model, UNET_PREFIX), _head_spec(model, "none"))[0]
    return torch.ops.hiseg.instance_masks(logits, int(wrapper.dilation_pixels)), binary


# ------------------------------------------------------------------------------------ ONNX (TorchScript exporter)
def _onnx_roi_align(g, feat, rois, output_height, output_width, scale_h, scale_w, aligned):
    """dynamic_roi_align.py:77-169 in standard ONNX ops: Gather the ROI's image, build the bilinear sampling grid
    (linspace over the output size x the ROI extent, normalised for align_corners), GridSample (opset 16)."""
    oh, ow = int(output_height), int(output_width)

    def const(v, dtype=torch.float32):
        return g.op("Constant", value_t=torch.tensor(v, dtype=dtype))

    def col(i):                                             # rois[:, i] -> [N, 1, 1]
        c = g.op("Gather", rois, const(i, torch.int64), axis_i=1)
        return g.op("Unsqueeze", c, const([1, 2], torch.int64))
    bidx = g.op("Cast", g.op("Gather", rois, const(0, torch.int64), axis_i=1), to_i=7)   # INT64
    sel = g.op("Gather", feat, bidx, axis_i=0)
    x1 = g.op("Mul", col(1), const(float(scale_w)))
    y1 = g.op("Mul", col(2), const(float(scale_h)))
    x2 = g.op("Mul", col(3), const(float(scale_w)))
    y2 = g.op("Mul", col(4), const(float(scale_h)))
    lin_x = const(torch.linspace(0, 1, ow).view(1, 1, ow).tolist())
    lin_y = const(torch.linspace(0, 1, oh).view(1, oh, 1).tolist())
    fx = g.op("Add", x1, g.op("Mul", lin_x, g.op("Sub", x2, x1)))         # [N, 1, ow]
    fy = g.op("Add", y1, g.op("Mul", lin_y, g.op("Sub", y2, y1)))         # [N, oh, 1]
    shp = g.op("Cast", g.op("Shape", feat), to_i=1)                        # FLOAT
    W = g.op("Gather", shp, const(3, torch.int64), axis_i=0)
    H = g.op("Gather", shp, const(2, torch.int64), axis_i=0)
    if aligned:
        W = g.op("Sub", W, const(1.0))
        H = g.op("Sub", H, const(1.0))
    two, one = const(2.0), const(1.0)
    nx = g.op("Sub", g.op("Mul", g.op("Div", fx, W), two), one)
    ny = g.op("Sub", g.op("Mul", g.op("Div", fy, H), two), one)
    zeros = g.op("Mul", g.op("Add", nx, ny), const(0.0))                   # [N, oh, ow]
    nx = g.op("Unsqueeze", g.op("Add", nx, zeros), const([3], torch.int64))
    ny = g.op("Unsqueeze", g.op("Add", ny, zeros), const([3], torch.int64))
    grid = g.op("Concat", nx, ny, axis_i=3)                                # [N, oh, ow, 2]
    return g.op("GridSample", sel, grid, align_corners_i=int(bool(aligned)), mode_s="bilinear",
                padding_mode_s="zeros")


def _onnx_output_conv(g, u, weight, bias):
    return g.op("Conv", u, weight, bias, kernel_shape_i=[1, 1])


def _onnx_binary_masks(g, u, weight, bias):
    p = g.op("Softmax", _onnx_output_conv(g, u, weight, bias), axis_i=1)
    return g.op("Slice", p, g.op("Constant", value_t=torch.tensor([0])), g.op("Constant", value_t=torch.tensor([1])),
                g.op("Constant", value_t=torch.tensor([1])))


def _onnx_instance_masks(g, logits, dilation):
    """export_onnx_advanced.py:360-364 + the dilation module (export_hierarchical_instance_peopleseg_onnx.py:85-141)
    in standard ops: Softmax / MaxPool / Greater / Where, then ArgMax == 1."""
    d = int(dilation)

    def const(v, dtype=torch.float32):
        return g.op("Constant", value_t=torch.tensor(v, dtype=dtype))

    def sl(x, a, b):
        return g.op("Slice", x, const([a], torch.int64), const([b], torch.int64), const([1], torch.int64))
    if d > 0:
        probs = sl(g.op("Softmax", logits, axis_i=1), 1, 2)
        dil = g.op("MaxPool", probs, kernel_shape_i=[2 * d + 1, 2 * d + 1], pads_i=[d, d, d, d], strides_i=[1, 1])
        grow = g.op("Greater", g.op("Sub", dil, probs), const(0.1))
        c1 = sl(logits, 1, 2)
        c1 = g.op("Where", grow, g.op("Add", c1, const(2.0)), c1)
        logits = g.op("Concat", sl(logits, 0, 1), c1, sl(logits, 2, 3), axis_i=1)
    cls = g.op("ArgMax", logits, axis_i=1, keepdims_i=1)
    return g.op("Cast", g.op("Equal", cls, const(1, torch.int64)), to_i=1)


def _onnx_custom(name):
    def fn(g, *args):
        *tensors, state, spec = args
        from torch.onnx import symbolic_helper as sh
        spec_s = spec if isinstance(spec, str) else sh._maybe_get_const(spec, "s")
        return g.op(f"hiseg::{name}", *tensors, *sh._unpack_list(state), spec_s=spec_s)
    return fn


def _spec_of(spec):
    from torch.onnx import symbolic_helper as sh
    return json.loads(spec if isinstance(spec, str) else sh._maybe_get_const(spec, "s"))


def _named_state(sp: dict, state_values: Sequence, skip: str) -> Dict[str, object]:
    """state_dict name -> graph value of an op's state inputs (the skeleton of the spec gives the names)."""
    m, _ = _skeleton(sp)
    names = [k for k in m.state_dict().keys() if not (skip and k.startswith(skip))]
    if len(names) != len(state_values):
        raise ValueError(f"ONNX lowering: {len(state_values)} state inputs for a {sp['cls']} with {len(names)}")
    return dict(zip(names, state_values))


def onnx_unet_logit(g, images, state_values: Sequence, spec: dict):
    """hiseg::unet_logit in standard operators (onnx_graph.emit_unet_logit)."""
    from . import onnx_graph
    m, _ = _skeleton(spec)
    return onnx_graph.emit_unet_logit(g, m, _named_state(spec, state_values, ""), images)


def onnx_rgb_head(g, images, u, rois, state_values: Sequence, spec: dict) -> list:
    """hiseg::rgb_head in standard operators: the outputs named in the spec, in order (onnx_graph.emit_rgb_head)."""
    from . import onnx_graph
    m, _ = _skeleton(spec)
    return onnx_graph.emit_rgb_head(g, m, _named_state(spec, state_values, UNET_PREFIX), images, u, rois,
                                    spec["scale_hw"], [n for n, _ in spec["outs"]])


def _sym_unet_logit(g, images, state, spec):
    from torch.onnx import symbolic_helper as sh
    return onnx_unet_logit(g, images, sh._unpack_list(state), _spec_of(spec))


def _sym_rgb_head(g, images, u, rois, state, spec):
    from torch.onnx import symbolic_helper as sh
    outs = onnx_rgb_head(g, images, u, rois, sh._unpack_list(state), _spec_of(spec))
    return g.op("prim::ListConstruct", *outs)


def register_onnx_symbolics(opset: int = 17, custom_domain: bool = False) -> None:
    """Register the TorchScript-exporter lowering of every hiseg op (opset >= 16 for GridSample).  The composite
    UNet and head ops lower to standard operators (onnx_graph.py); ``custom_domain=True`` keeps them as single nodes
    of the ``hiseg`` domain instead (a runtime with a libhiseg custom-op library)."""
    from torch.onnx import symbolic_helper as sh
    reg = torch.onnx.register_custom_op_symbolic
    reg("hiseg::dynamic_roi_align", sh.parse_args("v", "v", "i", "i", "f", "f", "b")(_onnx_roi_align), opset)
    reg("hiseg::output_conv", sh.parse_args("v", "v", "v")(_onnx_output_conv), opset)
    reg("hiseg::binary_masks", sh.parse_args("v", "v", "v")(_onnx_binary_masks), opset)
    reg("hiseg::instance_masks", sh.parse_args("v", "i")(_onnx_instance_masks), opset)
    if custom_domain:
        reg("hiseg::unet_logit", _onnx_custom("PretrainedPeopleSegmentationUNet"), opset)
        reg("hiseg::rgb_head", _onnx_custom("RGBHierarchicalHead"), opset)
    else:
        reg("hiseg::unet_logit", _sym_unet_logit, opset)
        reg("hiseg::rgb_head", _sym_rgb_head, opset)


ONNX_LOWERINGS = {"dynamic_roi_align": _onnx_roi_align, "output_conv": _onnx_output_conv,
                  "binary_masks": _onnx_binary_masks, "instance_masks": _onnx_instance_masks,
                  "unet_logit": onnx_unet_logit, "rgb_head": onnx_rgb_head}
