"""GPU: a torch.export-ed hiseg program runs the same libhiseg kernels as the eager modules (bit-identical), at
batch / ROI counts other than the traced ones, and after torch.export.save / load with a cold skeleton cache."""
import io

import pytest
import torch

import filler
import hiseg
from hiseg import export as X
from helpers import b0_kwargs, hiseg_kwargs

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _model(dtype):
    torch.manual_seed(0)
    m = hiseg.create_rgb_hierarchical_model(**hiseg_kwargs(b0_kwargs()))
    filler.fill_module(m)
    hiseg.set_compute_dtype(m, dtype)
    return m.to(DEV).eval()


def _inputs(B, per_image, seed=61, H=96, W=128):
    images = torch.from_numpy(filler.uniform(seed, (B, 3, H, W))).to(DEV)
    rois = torch.from_numpy(filler.box_rois(seed + 1, B, per_image)).to(DEV)
    return images, rois


def _dyn():
    b, n = torch.export.Dim("batch", min=1, max=64), torch.export.Dim("num_rois", min=1, max=4096)
    return {"images": {0: b}, "rois": {0: n}}


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16], ids=["f32", "bf16"])
def test_exported_contract_equals_eager(dtype):
    wrapper = hiseg.RGBHierarchicalExportWrapper(_model(dtype), dilation_pixels=1).eval()
    ep = torch.export.export(wrapper, _inputs(2, 2), dynamic_shapes=_dyn())
    run = ep.module()
    for B, per in ((2, 2), (3, 5), (1, 1)):          # the traced sizes and two others
        images, rois = _inputs(B, per, seed=70 + B)
        with torch.no_grad():
            want = wrapper(images, rois)
            got = run(images, rois)
        torch.cuda.synchronize()
        for g, w in zip(got, want):
            assert g.shape == w.shape and torch.equal(g, w), (B, per)


def test_exported_model_forward_equals_eager():
    m = _model(torch.bfloat16)
    for mm in (m.roi_align_mask, m.roi_align_rgb):
        mm.spatial_scale_h, mm.spatial_scale_w = 96, 128
    images, rois = _inputs(2, 3)
    ep = torch.export.export(m, (images, rois), dynamic_shapes=_dyn())
    with torch.no_grad():
        logits, aux = m(images, rois)
        glog, gaux = ep.module()(images, rois)
    torch.cuda.synchronize()
    assert torch.equal(glog, logits)
    assert set(gaux) == set(aux)
    for k in aux:
        assert torch.equal(gaux[k], aux[k]), k


def test_exported_program_runs_after_save_load_with_cold_skeletons():
    wrapper = hiseg.RGBHierarchicalExportWrapper(_model(torch.bfloat16)).eval()
    images, rois = _inputs(2, 2)
    ep = torch.export.export(wrapper, (images, rois), dynamic_shapes=_dyn())
    buf = io.BytesIO()
    torch.export.save(ep, buf)
    buf.seek(0)
    X._SKELETONS.clear()
    ep2 = torch.export.load(buf)
    with torch.no_grad():
        want = wrapper(images, rois)
        got = ep2.module()(images, rois)
    torch.cuda.synchronize()
    for g, w in zip(got, want):
        assert torch.equal(g, w)


def test_exported_roi_align_and_unet_wrapper_equal_eager():
    m = _model(torch.float32)
    images, rois = _inputs(2, 3)
    ra = m.roi_align_rgb

    class Crop(torch.nn.Module):
        def forward(self, x, r):
            return ra(x, r, 16, 12)
    ep = torch.export.export(Crop(), (images, rois))
    assert torch.equal(ep.module()(images, rois), ra(images, rois, 16, 12))
    ep = torch.export.export(m.pretrained_unet, (images,))
    got, _ = ep.module()(images)
    want, _ = m.pretrained_unet(images)
    torch.cuda.synchronize()
    assert torch.equal(got, want)


def test_two_exported_programs_same_architecture_different_weights():
    """export program A, run it, drop it; export program B (same architecture, other weights), run it --
    B's outputs are B's eager outputs, not A's packed weights reused through the shared skeleton's plan cache."""
    import gc
    images, rois = _inputs(2, 2)
    outs = []
    for seed in (0, 1):
        m = hiseg.create_rgb_hierarchical_model(**hiseg_kwargs(b0_kwargs()))
        filler.fill_module(m, seed=100 + seed)
        hiseg.set_compute_dtype(m, torch.bfloat16)
        wrapper = hiseg.RGBHierarchicalExportWrapper(m.to(DEV).eval()).eval()
        ep = torch.export.export(wrapper, (images, rois), dynamic_shapes=_dyn())
        with torch.no_grad():
            want = wrapper(images, rois)
            got = ep.module()(images, rois)
        torch.cuda.synchronize()
        for g, w in zip(got, want):
            assert torch.equal(g, w), seed
        outs.append([t.clone() for t in got])
        del ep, wrapper, m, got, want
        gc.collect()
    assert not torch.equal(outs[0][1], outs[1][1])
