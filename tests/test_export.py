"""Traceable export surface (hiseg.export): torch.export of the hiseg modules on CPU with fake tensors, the saved
program's round trip, and the standard-op ONNX lowerings run through an eager ONNX-semantics interpreter against
the oracle (the onnx package is absent here, so serialised ONNX is not checked).

Reference: export_onnx_advanced.py:338-457 (RGBHierarchicalWrapper: pretrained_unet(images) -> softmax[:, 0:1],
model(images, rois) -> argmax == 1), export_hierarchical_instance_peopleseg_onnx.py:85-141 (dilation),
dynamic_roi_align.py:56-171.
"""
import io

import numpy as np
import pytest
import torch
import torch.nn.functional as F

import filler
import hiseg
from hiseg import export as X
from helpers import b0_kwargs, hiseg_kwargs

HISEG_OPS = {"unet_logit", "output_conv", "dynamic_roi_align", "rgb_head", "instance_masks", "binary_masks"}


def _model(**over):
    kw = hiseg_kwargs(b0_kwargs())
    kw.update(over)
    torch.manual_seed(0)
    m = hiseg.create_rgb_hierarchical_model(**kw)
    filler.fill_module(m)
    return m.eval()


def _inputs(B=2, per_image=2, H=96, W=128):
    images = torch.from_numpy(filler.uniform(41, (B, 3, H, W)))
    rois = torch.from_numpy(filler.box_rois(42, B, per_image))
    return images, rois


def _hiseg_targets(ep):
    out = []
    for n in ep.graph.nodes:
        if n.op == "call_function" and str(n.target).startswith("hiseg."):
            out.append(str(n.target).split(".")[1])
    return out


def _dyn():
    b, n = torch.export.Dim("batch", min=1, max=64), torch.export.Dim("num_rois", min=1, max=4096)
    return {"images": {0: b}, "rois": {0: n}}


def test_export_contract_traces_on_cpu_with_symbolic_batch_and_rois():
    wrapper = hiseg.RGBHierarchicalExportWrapper(_model(), dilation_pixels=1).eval()
    images, rois = _inputs()
    ep = torch.export.export(wrapper, (images, rois), dynamic_shapes=_dyn())
    assert _hiseg_targets(ep) == ["unet_logit", "binary_masks", "rgb_head", "instance_masks"]
    inst, binary = [n for n in ep.graph.nodes if n.op == "output"][0].args[0]
    si, sb = inst.meta["val"].shape, binary.meta["val"].shape
    assert str(si[0]) != "4" and tuple(si[1:]) == (1, *wrapper.model.mask_size)   # symbolic N, the mask grid
    assert str(sb[0]) != "2" and tuple(sb[1:]) == (1, 96, 128)     # symbolic B, the image
    # the program owns the weights: every parameter and buffer of the model is lifted
    assert len(ep.state_dict) + len(ep.constants) >= len(list(wrapper.model.parameters()))


def test_export_model_forward_returns_reference_aux_dict():
    m = _model()
    images, rois = _inputs()
    ep = torch.export.export(m, (images, rois), dynamic_shapes=_dyn())
    assert _hiseg_targets(ep) == ["unet_logit", "rgb_head"]
    fake_out = [n for n in ep.graph.nodes if n.op == "output"][0].args[0]
    names = [n for n, _ in X.rgb_out_templates(m, "full")]
    assert len(fake_out) == len(names)
    shapes = {nm: tuple(int(d) if str(d).isdigit() else str(d) for d in node.meta["val"].shape)
              for nm, node in zip(names, fake_out)}
    assert shapes["logits"][1:] == (3, *m.mask_size)
    assert shapes["bg_fg_logits_low"][1:] == (2, *m.roi_size)
    assert shapes["full_image_logits"][1:] == (2, 96, 128)
    assert shapes["roi_patches"][1:] == (3, *m.roi_size)
    out_spec = ep.call_spec.out_spec                                 # (logits, {aux name: tensor})
    assert set(out_spec.child(1).context) == set(names) - {"logits"}


def test_export_submodules_of_the_reference_wrapper():
    """The reference's exporter calls model.pretrained_unet(images) and DynamicRoIAlign directly."""
    m = _model()
    images, rois = _inputs()
    ep = torch.export.export(m.pretrained_unet, (images,))
    assert _hiseg_targets(ep) == ["unet_logit", "output_conv"]
    ra = m.roi_align_rgb

    class Crop(torch.nn.Module):
        def forward(self, x, r):
            return ra(x, r, 16, 12)
    ep = torch.export.export(Crop(), (images, rois))
    assert _hiseg_targets(ep) == ["dynamic_roi_align"]


def test_exported_program_round_trips_through_save_and_load():
    wrapper = hiseg.RGBHierarchicalExportWrapper(_model()).eval()
    images, rois = _inputs()
    ep = torch.export.export(wrapper, (images, rois), dynamic_shapes=_dyn())
    buf = io.BytesIO()
    torch.export.save(ep, buf)
    buf.seek(0)
    ep2 = torch.export.load(buf)
    assert _hiseg_targets(ep2) == _hiseg_targets(ep)
    k1, k2 = sorted(ep.state_dict), sorted(ep2.state_dict)
    assert k1 == k2 and all(torch.equal(ep.state_dict[k], ep2.state_dict[k]) for k in k1)


def test_exported_program_has_no_cpu_fallback():
    wrapper = hiseg.RGBHierarchicalExportWrapper(_model()).eval()
    images, rois = _inputs()
    ep = torch.export.export(wrapper, (images, rois))
    with pytest.raises(RuntimeError, match="GPU only"):
        ep.module()(images, rois)


def test_skeleton_rebuilds_the_module_from_its_spec():
    import json
    m = _model(use_contour_detection=False)
    hiseg.set_compute_dtype(m, torch.bfloat16)
    sp = json.loads(X._head_spec(m, "full"))
    sk, _ = X._skeleton(sp)
    assert type(sk) is type(m) and sk.hiseg_dtype == torch.bfloat16
    assert list(sk.state_dict().keys()) == list(m.state_dict().keys())
    assert all(a.shape == b.shape for a, b in zip(sk.state_dict().values(), m.state_dict().values()))
    assert [n for n, _ in sp["outs"]] == [n for n, _ in X.rgb_out_templates(m, "full")]
    assert "contours" not in dict(sp["outs"])


def test_skeleton_plans_do_not_carry_over_between_state_sets():
    """one skeleton serves every exported program of an architecture; its engine plan cache must not
    survive a change of state set (a plan is keyed by the state tensors' addresses + versions, which a released
    program's tensors could hand to the next one).  Same state set: plans kept; another set: dropped.  ADVICE r4: the
    skeleton keeps only weak references to the set (a released program's weights are not pinned); a set whose
    tensors died is treated as another set even at the same addresses."""
    import json
    m = _model(use_contour_detection=False)
    sp = json.loads(X._head_spec(m, "full"))
    state_a = X._state(m, X.UNET_PREFIX)
    state_b = [t.detach().clone() for t in state_a]
    sk, _ = X._skeleton(sp)
    X._run_on(sp, state_a, X.UNET_PREFIX, lambda k: k.__dict__.__setitem__("_hiseg_plans", {"marker": 1}))
    assert X._run_on(sp, state_a, X.UNET_PREFIX, lambda k: k.__dict__.get("_hiseg_plans")) == {"marker": 1}
    assert X._run_on(sp, state_b, X.UNET_PREFIX, lambda k: k.__dict__.get("_hiseg_plans")) is None
    refs = sk.__dict__["_hiseg_state_refs"]
    assert len(refs) == len(state_b) and all(r() is b for r, b in zip(refs, state_b))
    assert "_hiseg_state_held" not in sk.__dict__
    X._run_on(sp, state_b, X.UNET_PREFIX, lambda k: k.__dict__.__setitem__("_hiseg_plans", {"marker": 2}))
    ptrs = [t.data_ptr() for t in state_b]
    state_c = [t.detach().clone() for t in state_b]
    del state_b, refs
    assert all(r() is None for r in sk.__dict__["_hiseg_state_refs"])   # not pinned by the skeleton
    # a new set (even one that reused the addresses) does not see the released set's plans
    assert X._run_on(sp, state_c, X.UNET_PREFIX, lambda k: k.__dict__.get("_hiseg_plans")) is None
    assert ptrs


# ------------------------------------------------------------------------------------ ONNX lowerings
class EagerOnnx:
    """Executes ONNX ops as they are emitted (ONNX operator semantics on torch CPU tensors)."""

    def op(self, name, *xs, **at):
        f = getattr(self, "_" + name)
        return f(*xs, **at)

    @staticmethod
    def _Constant(value_t):
        return value_t.clone()

    @staticmethod
    def _Gather(x, idx, axis_i=0):
        ax = axis_i % x.dim()
        flat = x.index_select(ax, idx.reshape(-1).long())
        return flat.reshape(x.shape[:ax] + idx.shape + x.shape[ax + 1:])

    @staticmethod
    def _Unsqueeze(x, axes):
        for a in sorted(int(v) for v in axes.reshape(-1)):
            x = x.unsqueeze(a)
        return x

    @staticmethod
    def _Cast(x, to_i):
        return x.to({1: torch.float32, 7: torch.int64}[to_i])

    _Mul = staticmethod(torch.mul)
    _Add = staticmethod(torch.add)
    _Sub = staticmethod(torch.sub)
    _Div = staticmethod(torch.div)
    _Greater = staticmethod(torch.gt)
    _Where = staticmethod(torch.where)
    _Equal = staticmethod(torch.eq)

    @staticmethod
    def _Shape(x):
        return torch.tensor(list(x.shape), dtype=torch.int64)

    @staticmethod
    def _Concat(*xs, axis_i):
        return torch.cat(xs, dim=axis_i)

    @staticmethod
    def _GridSample(x, grid, align_corners_i, mode_s, padding_mode_s):
        return F.grid_sample(x, grid, mode=mode_s, padding_mode=padding_mode_s, align_corners=bool(align_corners_i))

    @staticmethod
    def _Conv(x, w, b=None, kernel_shape_i=None, strides_i=(1, 1), pads_i=(0, 0, 0, 0), group_i=1, dilations_i=(1, 1)):
        assert pads_i[0] == pads_i[2] and pads_i[1] == pads_i[3]
        return F.conv2d(x, w, b, stride=tuple(strides_i), padding=(pads_i[0], pads_i[1]), groups=group_i,
                        dilation=tuple(dilations_i))

    @staticmethod
    def _ConvTranspose(x, w, b, kernel_shape_i, strides_i, pads_i):
        return F.conv_transpose2d(x, w, b, stride=tuple(strides_i))

    @staticmethod
    def _BatchNormalization(x, scale, bias, mean, var, epsilon_f):
        return F.batch_norm(x, mean, var, scale, bias, False, 0.0, epsilon_f)

    _Relu = staticmethod(torch.relu)
    _Sigmoid = staticmethod(torch.sigmoid)
    _Erf = staticmethod(torch.erf)
    _Sqrt = staticmethod(torch.sqrt)

    @staticmethod
    def _GlobalAveragePool(x):
        return x.mean(dim=(2, 3), keepdim=True)

    @staticmethod
    def _ReduceMean(x, axes_i, keepdims_i):
        return x.mean(dim=tuple(axes_i), keepdim=bool(keepdims_i))

    @staticmethod
    def _ReduceMax(x, axes_i=None, keepdims_i=1):
        if axes_i is None:
            return x.amax() if not keepdims_i else x.amax(dim=tuple(range(x.dim())), keepdim=True)
        return x.amax(dim=tuple(axes_i), keepdim=bool(keepdims_i))

    @staticmethod
    def _Resize(x, roi, scales, sizes=None, mode_s="nearest", coordinate_transformation_mode_s="half_pixel",
                nearest_mode_s="round_prefer_floor"):
        if mode_s == "nearest":
            assert coordinate_transformation_mode_s == "asymmetric" and nearest_mode_s == "floor"
            return F.interpolate(x, scale_factor=tuple(float(v) for v in scales[2:]), mode="nearest")
        assert mode_s == "linear" and coordinate_transformation_mode_s == "pytorch_half_pixel"
        return F.interpolate(x, size=tuple(int(v) for v in sizes[2:]), mode="bilinear", align_corners=False)

    @staticmethod
    def _Softmax(x, axis_i):
        return torch.softmax(x, dim=axis_i)

    @staticmethod
    def _Slice(x, starts, ends, axes=None, steps=None):
        if axes is None:
            axes = torch.arange(len(starts))
        idx = [slice(None)] * x.dim()
        for s, e, a in zip(starts.tolist(), ends.tolist(), axes.tolist()):
            idx[a] = slice(s, e)
        return x[tuple(idx)]

    @staticmethod
    def _MaxPool(x, kernel_shape_i, pads_i, strides_i):
        return F.max_pool2d(x, kernel_shape_i, stride=strides_i, padding=pads_i[:2])

    @staticmethod
    def _ArgMax(x, axis_i, keepdims_i):
        return torch.argmax(x, dim=axis_i, keepdim=bool(keepdims_i))


@pytest.mark.parametrize("aligned", [True, False])
@pytest.mark.parametrize("scale", [(96, 128), (640, 640)])
def test_onnx_roi_align_lowering_matches_oracle(aligned, scale):
    from oracle.roi_align import roi_align as oracle_roi_align
    feat = torch.from_numpy(filler.uniform(51, (2, 4, 24, 32)))
    rois = torch.from_numpy(filler.box_rois(52, 2, 3))
    rois[-1, 1:] = torch.tensor([-0.2, -0.1, 1.3, 1.1])                 # reaches past every border
    got = X._onnx_roi_align(EagerOnnx(), feat, rois, 7, 9, scale[0], scale[1], aligned)
    want = oracle_roi_align(feat.numpy(), rois.numpy(), 7, 9, scale[0], scale[1], aligned)
    np.testing.assert_allclose(got.numpy(), want, rtol=0, atol=2e-6)


def test_onnx_binary_and_output_conv_lowerings_match_oracle():
    from oracle import rgb_model as O
    u = torch.from_numpy(filler.uniform(53, (2, 1, 16, 24))) * 8 - 4
    w, b = torch.tensor([[[[1.25]]], [[[-0.75]]]]), torch.tensor([0.1, -0.2])
    sd = {"pretrained_unet.output_conv.weight": w, "pretrained_unet.output_conv.bias": b}
    got = X._onnx_binary_masks(EagerOnnx(), u, w, b)
    torch.testing.assert_close(got, O.binary_masks(sd, u), rtol=0, atol=0)
    torch.testing.assert_close(X._onnx_output_conv(EagerOnnx(), u, w, b), O.conv(sd, "pretrained_unet.output_conv", u))


@pytest.mark.parametrize("dilation", [0, 1, 2])
def test_onnx_instance_masks_lowering_matches_oracle(dilation):
    from oracle import rgb_model as O
    logits = torch.from_numpy(filler.uniform(54 + dilation, (3, 3, 20, 20))) * 6 - 3
    got = X._onnx_instance_masks(EagerOnnx(), logits, dilation)
    assert torch.equal(got, O.instance_masks(logits, dilation))


def test_onnx_symbolics_register():
    X.register_onnx_symbolics(17)


# ------------------------------------------------------------------------------------ standard-op UNet / head
def _filled_model(overrides=None, name="b0"):
    import hiseg
    from helpers import configs, hiseg_kwargs
    kw = hiseg_kwargs(dict(configs()[name]["model_kwargs"]))
    kw.update(overrides or {})
    return filler.fill_module(hiseg.create_rgb_hierarchical_model(**kw)).eval(), kw


def _rel(a, b):
    return ((a.double() - b.double()).abs().max() / b.double().abs().max().clamp_min(1e-12)).item()


@pytest.mark.parametrize("name", ["b0", "b1"])
def test_onnx_unet_logit_lowering_matches_oracle(name):
    """hiseg::unet_logit in standard ONNX operators (onnx_graph.emit_unet_logit: /255 guard, normalisation,
    EfficientNet encoder with SE, nearest x2 decoder, head) against the oracle's smp-UNet restatement, both the
    [0, 1] and the 8-bit input branch of normalize_input (unet.py:1885-1890)."""
    import json
    from oracle import rgb_model as O
    model, _ = _filled_model(name=name)
    pre = model.pretrained_unet.model
    sd = O.np_state(model)
    images = torch.from_numpy(filler.uniform(61, (2, 3, 64, 96)))
    for x in (images, images * 255.0):
        got = X.onnx_unet_logit(EagerOnnx(), x, X._state(pre), json.loads(X._spec(pre)))
        with torch.no_grad():
            want = O.pretrained_unet_logits(sd, x, name)
        assert got.shape == want.shape == (2, 1, 64, 96)
        assert _rel(got, want) < 1e-4


@pytest.mark.parametrize("case", ["b0", "b0_layernorm_gelu_noattn", "b1"])
def test_onnx_rgb_head_lowering_matches_oracle(case):
    """hiseg::rgb_head in standard ONNX operators (onnx_graph.emit_rgb_head: output conv, GridSample RoIAligns, RGB
    stack, combiner, refined head with every aux output) against the oracle, f32, 1e-4."""
    import json
    from oracle import rgb_model as O
    if case == "b0_layernorm_gelu_noattn":
        model, kw = _filled_model({"normalization_type": "layernorm2d", "activation_function": "gelu",
                                   "use_attention_module": False})
    else:
        model, kw = _filled_model(name=case)
    variant = "b1" if case == "b1" else "b0"
    sd = O.np_state(model)
    H, W = 64, 96
    for m in (model.roi_align_mask, model.roi_align_rgb):
        m.spatial_scale_h, m.spatial_scale_w = H, W
    images = torch.from_numpy(filler.uniform(62, (2, 3, H, W)))
    rois = torch.from_numpy(filler.box_rois(63, 2, 2))
    with torch.no_grad():
        u = O.pretrained_unet_logits(sd, images, variant)
        want, want_aux = O.rgb_model_from_unet(sd, images, rois, u, O.cfg_from_kwargs(kw), (H, W))
    spec = json.loads(X._head_spec(model, "full"))
    outs = X.onnx_rgb_head(EagerOnnx(), images, u, rois, X._state(model, X.UNET_PREFIX), spec)
    got = dict(zip([n for n, _ in spec["outs"]], outs))
    assert _rel(got["logits"], want) < 1e-4
    for k, v in want_aux.items():
        assert got[k].shape == v.shape, k
        assert _rel(got[k], v) < 1e-4, k


def test_onnx_symbolics_register_custom_domain_option():
    X.register_onnx_symbolics(17, custom_domain=True)
    X.register_onnx_symbolics(17)


def test_onnx_exported_contract_composition_matches_oracle():
    """The whole exported contract as the ONNX graph composes it (traced_export: unet_logit -> rgb_head(aux none) ->
    instance_masks with dilation 1, binary_masks), every node standard: instance masks equal the oracle's, binary
    masks at 1e-5 (export_onnx_advanced.py:353-420)."""
    import json
    from oracle import rgb_model as O
    model, kw = _filled_model()
    sd = O.np_state(model)
    H, W = 64, 96
    for m in (model.roi_align_mask, model.roi_align_rgb):
        m.spatial_scale_h, m.spatial_scale_w = H, W
    images = torch.from_numpy(filler.uniform(64, (2, 3, H, W)))
    rois = torch.from_numpy(filler.box_rois(65, 2, 3))
    g = EagerOnnx()
    pre, oc = model.pretrained_unet.model, model.pretrained_unet.output_conv
    u = X.onnx_unet_logit(g, images, X._state(pre), json.loads(X._spec(pre)))
    spec = json.loads(X._head_spec(model, "none"))
    logits = X.onnx_rgb_head(g, images, u, rois, X._state(model, X.UNET_PREFIX), spec)[0]
    inst = X._onnx_instance_masks(g, logits, 1)
    binary = X._onnx_binary_masks(g, u, oc.weight.detach(), oc.bias.detach())
    with torch.no_grad():
        ref, _, ref_u = O.rgb_model(sd, images, rois, O.cfg_from_kwargs(kw), (H, W), "b0")
    ref_inst = O.instance_masks(ref, 1)
    assert (inst != ref_inst).float().mean().item() < 1e-3   # argmax ties at 1e-6 logit differences only
    assert (binary - O.binary_masks(sd, ref_u)).abs().max().item() < 1e-5
