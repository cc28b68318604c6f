"""The C-ABI library loads and exports every entry point include/hiseg.h declares (no GPU calls)."""
import os
import re

from conftest import ROOT


def header_functions(names=None):
    """Entry points declared in include/*.h (every header by default)."""
    inc = os.path.join(ROOT, "include")
    names = names or sorted(f for f in os.listdir(inc) if f.endswith(".h"))
    out = set()
    for n in names:
        src = open(os.path.join(inc, n)).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        out |= set(re.findall(r"^\s*(?:int|long long|const char\*)\s+(hiseg_\w+)\s*\(", src, flags=re.M))
    return sorted(out)


def test_header_declares_the_hot_path():
    fns = header_functions(["hiseg.h"])
    for must in ("hiseg_roi_align_fwd", "hiseg_conv2d_fwd", "hiseg_hier_combine_fwd", "hiseg_dwconv_fwd",
                 "hiseg_se_gate_fwd", "hiseg_attn_spatial_fwd", "hiseg_instance_masks_fwd"):
        assert must in fns
    every = header_functions()
    for must in ("hiseg_conv2d_wgrad", "hiseg_loss_fwd", "hiseg_distill_loss_fwd", "hiseg_adamw_step",
                 "hiseg_seg_confusion"):
        assert must in every


def test_library_exports_every_declared_symbol():
    from hiseg import _lib as L
    lib = L.lib()
    for name in header_functions():
        assert hasattr(lib, name), name
    assert lib.hiseg_version() >= 100
    assert lib.hiseg_built_for_gfx950() == 1
    # every symbol has a ctypes signature in the binding
    assert set(header_functions()) <= set(L.EXPORTED)


def test_binding_struct_layouts_match_the_headers():
    """Every descriptor struct of the C ABI has the size the library was compiled with (hiseg_struct_sizes), so a
    field added to a header without its ctypes twin -- or in another place -- fails here, not as a silent misread
    on the GPU (round 5 appended fields to hiseg_conv2d_desc and hiseg_bn_bwd_desc)."""
    import ctypes
    from hiseg import _lib as L
    classes = [L.RoiAlignDesc, L.Conv2dDesc, L.WgradMap, L.PackEntry, L.BnApplyDesc, L.BnBwdDesc, L.LnBwdDesc,
               L.EwView, L.UbfDesc, L.UbfGrads, L.LossCfg, L.DistillCfg, L.RoiTargetDesc]
    out = (ctypes.c_longlong * len(classes))()
    n = L.lib().hiseg_struct_sizes(out, len(classes))
    assert n == len(classes)
    for cls, size in zip(classes, out):
        assert ctypes.sizeof(cls) == size, (cls.__name__, ctypes.sizeof(cls), size)


def test_invalid_descriptor_reports_an_error_without_touching_the_gpu():
    import ctypes
    from hiseg import _lib as L
    d = L.Conv2dDesc()
    d.dtype = 7  # unsupported
    st = L.lib().hiseg_conv2d_fwd(ctypes.byref(d), None)
    assert st == -3
    assert b"dtype" in L.lib().hiseg_last_error_string()


def test_product_path_refuses_cpu_tensors():
    import pytest
    import torch
    from hiseg import DynamicRoIAlign
    with pytest.raises(RuntimeError, match="GPU only"):
        DynamicRoIAlign(640, aligned=True)(torch.zeros(1, 1, 4, 4), torch.zeros(1, 5), 2, 2)


def test_release_library_refuses_diagnostic_conv_variants():
    """Timing-only (9, 19, 73, 75-77), s_memtime-stamp (18, 41, 59, 79) and experimental (10-45) conv variants
    exist only in a DIAG=1 build (Makefile): the release libhiseg.so refuses them before any launch, with
    HISEG_ERR_BAD_ARG (a stamp variant without its buffer once wrote to an illegal address)."""
    import ctypes
    from hiseg import _lib as L
    d = L.Conv2dDesc()
    d.dtype = d.out_dtype = 1  # bf16
    d.N, d.H, d.W, d.Ho, d.Wo = 1, 32, 32, 32, 32   # (> 256 pixels per image: the 3x3 split-K plan does not apply)
    d.KH, d.KW, d.stride, d.pad = 3, 3, 1, 1
    fake = 1 << 20
    with L.raw_pointers():   # never launched: the library refuses the variant first
        d.srcA, d.a_cstride, d.a_coff, d.Ca, d.a_up = fake, 256, 0, 256, 1
        d.weight, d.Cout, d.Cout_pad, d.K_pad = fake, 256, 256, 9 * 256
        d.scale, d.shift, d.act = fake, fake, 0
        d.out, d.o_cstride, d.o_coff = fake, 256, 0
    for v in (9, 10, 18, 19, 20, 30, 40, 41, 44, 59, 73, 75, 76, 77, 79, 142, -5):
        st = L.lib().hiseg_conv2d_fwd_variant(ctypes.byref(d), v, None)
        assert st == -1, v   # HISEG_ERR_BAD_ARG
        assert b"not a release variant" in L.lib().hiseg_last_error_string(), v
    # the split-K variant (99) is a release variant, refused before any launch where it does not apply (3x3, no
    # workspace)
    assert L.lib().hiseg_conv2d_fwd_variant(ctypes.byref(d), 99, None) == -1
    assert b"split-K" in L.lib().hiseg_last_error_string()
    assert L.lib().hiseg_conv2d_workspace_bytes(ctypes.byref(d)) == 0


def test_conv_splitk_workspace_plan_is_batch_invariant():
    """hiseg_conv2d_workspace_bytes (no GPU call): the split-K plan of a small-image, long-K SE-gated 1x1 layer
    depends on the layer and the per-image grid only -- bytes per image are the same for every batch size, so an
    image's outputs do not depend on the batch it runs in -- and layers outside the plan need no workspace."""
    import ctypes
    from hiseg import _lib as L

    def ws(N, H, W, Ca, Cout, gated=True, k=1):
        d = L.Conv2dDesc()
        d.dtype = d.out_dtype = 1
        d.N, d.H, d.W, d.Ho, d.Wo = N, H, W, H, W
        d.KH = d.KW = k
        d.stride, d.pad = 1, k // 2
        d.Ca, d.a_cstride, d.a_up = Ca, Ca, 1
        d.Cout, d.Cout_pad = Cout, (Cout + 15) // 16 * 16
        d.K_pad = (k * k * Ca + 63) // 64 * 64
        with L.raw_pointers():   # planning only, never launched
            d.srcA = d.weight = d.scale = d.shift = d.out = 1 << 20
            d.in_scale = (1 << 20) if gated else None
        return L.lib().hiseg_conv2d_workspace_bytes(ctypes.byref(d))

    for Ca, Cout, H, W in ((2304, 384, 20, 20), (960, 160, 40, 40), (1152, 192, 15, 20), (3840, 640, 20, 20)):
        nK = (Ca + 63) // 64
        sp = min(8, max(2, nK // 4))
        per_image = sp * H * W * ((Cout + 15) // 16 * 16) * 4
        for N in (1, 4, 32):
            assert ws(N, H, W, Ca, Cout) == N * per_image, (Ca, Cout, N)
    assert ws(4, 80, 80, 480, 80) == 0           # > 1600 pixels per image: unsplit
    assert ws(4, 20, 20, 384, 2304, gated=False) == 0   # ungated, short K: the LDS-DMA ring kernel
    assert ws(4, 20, 20, 288, 48) == 0           # the 10-k-step pointwise kernel takes it
    assert ws(4, 20, 20, 2304, 384, k=3) == 0    # 3x3 over 400-pixel images: never split
    for N in (1, 8):                              # 3x3 over <= 256-pixel images with K >= 1536: nK / 4 splits (<= 8)
        assert ws(N, 16, 12, 768, 768, gated=False, k=3) == N * 8 * 16 * 12 * 768 * 4
    assert ws(4, 16, 12, 64, 64, gated=False, k=3) == 0   # short K


def test_descriptor_holds_plain_tensors_and_activation_views():
    """A pointer field assigned a torch.Tensor stores its address and keeps it alive (torch.Tensor has a .t method,
    which must not be mistaken for an activation view's .t); an object that is neither raises; strict mode refuses
    raw addresses."""
    import pytest
    import torch
    from hiseg import _lib as L

    class View:
        def __init__(self, t):
            self.t = t

    d = L.Conv2dDesc()
    w = torch.zeros(8)
    d.weight = w
    assert d.weight == w.data_ptr() and d.held()["weight"] is w
    v = View(torch.zeros(4))
    d.out = v
    assert d.out == v.t.data_ptr() and d.held()["out"] is v
    c = d.copy()
    assert c.held()["weight"] is w and c.weight == w.data_ptr()
    d.weight = None
    assert "weight" not in d.held()
    with pytest.raises(TypeError):
        d.scale = "not a tensor"
    if L.STRICT_PTRS:
        with pytest.raises(TypeError):
            d.shift = 1 << 20
