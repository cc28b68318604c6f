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
    program's tensors could hand to the next one).  Same state set: plans kept; another set: dropped, and the
    skeleton holds the set it runs with."""
    import json
    m = _model(use_contour_detection=False)
    sp = json.loads(X._head_spec(m, "full"))
    state_a = X._state(m, X.UNET_PREFIX)
    state_b = [t.detach().clone() for t in state_a]
    sk, _ = X._skeleton(sp)
    X._run_on(sp, state_a, X.UNET_PREFIX, lambda k: k.__dict__.__setitem__("_hiseg_plans", {"marker": 1}))
    assert X._run_on(sp, state_a, X.UNET_PREFIX, lambda k: k.__dict__.get("_hiseg_plans")) == {"marker": 1}
    assert X._run_on(sp, state_b, X.UNET_PREFIX, lambda k: k.__dict__.get("_hiseg_plans")) is None
    held = sk.__dict__["_hiseg_state_held"]
    assert len(held) == len(state_b) and all(a is b for a, b in zip(held, state_b))


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
    def _Conv(x, w, b, kernel_shape_i):
        return F.conv2d(x, w, b)

    @staticmethod
    def _Softmax(x, axis_i):
        return torch.softmax(x, dim=axis_i)

    @staticmethod
    def _Slice(x, starts, ends, axes, steps=None):
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
