"""ctypes binding of libhiseg.so (the C ABI declared in include/hiseg.h).

The library is loaded after ``import torch`` so that its ``libamdhip64.so.7`` dependency
resolves to the HIP runtime torch already loaded (one runtime, shared streams).  There is
no fallback: if the shared object is missing or was not built for gfx950, importing the
package's GPU path raises immediately.
"""
from __future__ import annotations

import contextlib
import ctypes
import os

import torch  # noqa: F401  (must precede the CDLL load: shares torch's HIP runtime)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("HISEG_LIB", os.path.join(_HERE, "libhiseg.so"))

HISEG_F32 = 0
HISEG_BF16 = 1
ACT_NONE, ACT_RELU, ACT_SIGMOID, ACT_SILU, ACT_GELU, ACT_SWISH = 0, 1, 2, 3, 4, 5


class ActCode(int):
    """An activation code (include/hiseg.h hiseg_act) that carries Swish's beta (act_beta fields)."""

    def __new__(cls, code: int, beta: float = 1.0):
        o = int.__new__(cls, code)
        o.beta = float(beta)
        return o

    def __repr__(self):
        return f"ActCode({int(self)}, beta={self.beta})"


def act_beta(act) -> float:
    """Swish beta of an activation code (1.0 for plain int codes)."""
    return float(getattr(act, "beta", 1.0))
LOSS_NOUT = 15  # include/hiseg_loss.h HISEG_LOSS_NOUT

c_int = ctypes.c_int
c_float = ctypes.c_float
c_void_p = ctypes.c_void_p
c_ll = ctypes.c_longlong

# Strict pointer mode (tests set HISEG_STRICT_PTRS=1): a descriptor pointer field may only be assigned a tensor /
# activation view (held by the descriptor) or None -- a raw integer address raises, so no descriptor can point at
# memory nothing keeps alive.
STRICT_PTRS = os.environ.get("HISEG_STRICT_PTRS", "0") == "1"


class Desc(ctypes.Structure):
    """A C-ABI descriptor that owns what it points at.

    Assigning a ``torch.Tensor`` or an activation view (anything with ``.t`` and ``.ptr()``, hiseg.ops.Act) to a
    pointer field stores its device address AND keeps the object alive for as long as the descriptor lives.  The
    training tape's backward closures capture descriptors built in the forward (the conv epilogue operands, a
    Dropout2d mask, the upsample/combine head's buffers) and launch kernels through them later; a tensor whose
    only reference was its address inside such a descriptor could be released after the forward and its block
    handed to another tensor by the caching allocator (round 3: fg_gate's Dropout2d mask).  Holding by
    construction makes that impossible; ``copy()`` carries the holds over to the copy."""

    _ptr_fields = frozenset()

    def __init_subclass__(cls, **kw):
        super().__init_subclass__(**kw)
        cls._ptr_fields = frozenset(n for n, t in cls.__dict__.get("_fields_", ()) if t is c_void_p)

    def __setattr__(self, name, value):
        if name in self._ptr_fields and value is not None and not isinstance(value, int):
            # (torch.Tensor has a .t method: test for a tensor before looking for an activation view's .t)
            t = value if isinstance(value, torch.Tensor) else getattr(value, "t", None)
            if not isinstance(t, torch.Tensor):
                raise TypeError(f"{type(self).__name__}.{name}: expected a tensor / activation view, got {type(value)}")
            self.__dict__.setdefault("_held", {})[name] = value
            value = t.data_ptr()
        elif name in self._ptr_fields:
            if STRICT_PTRS and value:
                raise TypeError(f"{type(self).__name__}.{name}: raw address assigned (strict pointer mode): pass the "
                                "tensor so the descriptor keeps it alive")
            held = self.__dict__.get("_held")
            if held is not None:
                held.pop(name, None)
        super().__setattr__(name, value)

    def held(self):
        """{field: object} of the pointer fields this descriptor keeps alive."""
        return dict(self.__dict__.get("_held", {}))

    def copy(self):
        c = type(self).from_buffer_copy(self)
        c.__dict__["_held"] = dict(self.__dict__.get("_held", {}))
        return c


@contextlib.contextmanager
def raw_pointers():
    """Allow raw integer addresses in descriptor pointer fields (tests that probe the C ABI's argument checks
    with descriptors that are never launched)."""
    global STRICT_PTRS
    old, STRICT_PTRS = STRICT_PTRS, False
    try:
        yield
    finally:
        STRICT_PTRS = old


class RoiAlignDesc(Desc):
    _fields_ = [
        ("feat", c_void_p), ("B", c_int), ("C", c_int), ("H", c_int), ("W", c_int),
        ("rois", c_void_p), ("N", c_int),
        ("oh", c_int), ("ow", c_int),
        ("scale_h", c_float), ("scale_w", c_float),
        ("aligned", c_int),
        ("aff_w", c_void_p), ("aff_b", c_void_p), ("n_aff", c_int),
        ("out", c_void_p), ("out_dtype", c_int), ("o_cstride", c_int), ("o_coff", c_int),
        ("o_nchw", c_int), ("zero_to", c_int),
    ]


class Conv2dDesc(Desc):
    _fields_ = [
        ("dtype", c_int), ("out_dtype", c_int),
        ("N", c_int), ("H", c_int), ("W", c_int),
        ("Ho", c_int), ("Wo", c_int),
        ("KH", c_int), ("KW", c_int), ("stride", c_int), ("pad", c_int),
        ("srcA", c_void_p), ("a_cstride", c_int), ("a_coff", c_int), ("Ca", c_int), ("a_up", c_int),
        ("srcB", c_void_p), ("b_cstride", c_int), ("b_coff", c_int), ("Cb", c_int),
        ("in_scale", c_void_p),
        ("weight", c_void_p), ("Cout", c_int), ("Cout_pad", c_int), ("K_pad", c_int),
        ("scale", c_void_p), ("shift", c_void_p),
        ("act", c_int),
        ("residual", c_void_p), ("r_cstride", c_int), ("r_coff", c_int),
        ("mul", c_void_p), ("m_cstride", c_int), ("m_coff", c_int),
        ("out", c_void_p), ("o_cstride", c_int), ("o_coff", c_int),
        ("out2", c_void_p), ("o2_cstride", c_int), ("o2_coff", c_int),
        ("convT", c_int),
        ("weight_frag", c_void_p),
        ("act_beta", c_float),
        ("workspace", c_void_p), ("workspace_bytes", ctypes.c_longlong),
        ("stats_partial", c_void_p),
        ("bnb_partial", c_void_p), ("bnb_z", c_void_p), ("bnb_z_cstride", c_int), ("bnb_z_coff", c_int),
        ("bnb_scale", c_void_p), ("bnb_shift", c_void_p), ("bnb_mean", c_void_p), ("bnb_invstd", c_void_p),
        ("bnb_act", c_int),
    ]


class WgradMap(Desc):
    _fields_ = [(n, c_int) for n in ("Cout", "KH", "KW", "ca", "ca_real", "cb", "cb_real", "convT", "Cg", "Kg",
                                     "want_bias")]


HISEG_PACK_FRAG = 8   # include/hiseg_train.h: pack mode flag, MFMA fragment order
HISEG_PACK_BIAS = 4   # pack mode: conv bias -> f32 epilogue shift


class PackEntry(Desc):
    _fields_ = [("src", c_void_p), ("dst", c_void_p), ("dtype", c_int), ("mode", c_int),
                ("Cout", c_int), ("Cin_real", c_int), ("KH", c_int), ("KW", c_int),
                ("ca", c_int), ("ca_real", c_int), ("cb", c_int), ("cb_real", c_int),
                ("rows", c_int), ("K_pad", c_int), ("cop", c_int), ("total", c_int)]


class BnApplyDesc(Desc):
    _fields_ = [("dtype", c_int), ("P", c_ll), ("HW", c_int), ("C", c_int),
                ("z", c_void_p), ("z_cstride", c_int), ("z_coff", c_int),
                ("scale", c_void_p), ("shift", c_void_p),
                ("residual", c_void_p), ("r_cstride", c_int), ("r_coff", c_int),
                ("act", c_int), ("chan_mul", c_void_p),
                ("y", c_void_p), ("y_cstride", c_int), ("y_coff", c_int),
                ("act_beta", c_float), ("per_sample", c_int)]


class BnBwdDesc(Desc):
    _fields_ = [("dtype", c_int), ("P", c_ll), ("HW", c_int), ("C", c_int),
                ("dy", c_void_p), ("dy_cstride", c_int), ("dy_coff", c_int),
                ("y", c_void_p), ("y_cstride", c_int), ("y_coff", c_int),
                ("z", c_void_p), ("z_cstride", c_int), ("z_coff", c_int),
                ("chan_mul", c_void_p), ("act", c_int),
                ("mean", c_void_p), ("invstd", c_void_p), ("gamma", c_void_p),
                ("partial", c_void_p),
                ("dgamma", c_void_p), ("dbeta", c_void_p), ("dconv_bias", c_void_p), ("accumulate_params", c_int),
                ("dz", c_void_p), ("dz_cstride", c_int), ("dz_coff", c_int),
                ("dres", c_void_p), ("dres_cstride", c_int), ("dres_coff", c_int), ("dres_accumulate", c_int),
                ("beta", c_void_p), ("fwd_scale", c_void_p), ("fwd_shift", c_void_p),
                ("act_beta", c_float), ("residual", c_void_p), ("r_cstride", c_int), ("r_coff", c_int),
                ("partial_splits", c_int)]


class LnBwdDesc(Desc):
    _fields_ = [("dtype", c_int), ("N", c_int), ("HW", c_int), ("C", c_int),
                ("dy", c_void_p), ("dy_cstride", c_int), ("dy_coff", c_int),
                ("z", c_void_p), ("z_cstride", c_int), ("z_coff", c_int),
                ("residual", c_void_p), ("r_cstride", c_int), ("r_coff", c_int),
                ("chan_mul", c_void_p), ("act", c_int), ("act_beta", c_float),
                ("mean", c_void_p), ("invstd", c_void_p), ("scale", c_void_p), ("shift", c_void_p),
                ("gamma", c_void_p),
                ("dgamma", c_void_p), ("dbeta", c_void_p), ("dconv_bias", c_void_p), ("accumulate_params", c_int),
                ("dz", c_void_p), ("dz_cstride", c_int), ("dz_coff", c_int),
                ("dres", c_void_p), ("dres_cstride", c_int), ("dres_coff", c_int), ("dres_accumulate", c_int),
                ("ws", c_void_p)]


class EwView(Desc):
    _fields_ = [("p", c_void_p), ("cstride", c_int), ("coff", c_int)]


class UbfDesc(Desc):
    _fields_ = [("dtype", c_int), ("low", c_void_p), ("N", c_int), ("h", c_int), ("w", c_int),
                ("ut_w", c_void_p), ("ut_b", c_void_p), ("gamma", c_void_p), ("beta", c_void_p),
                ("mean", c_void_p), ("invstd", c_void_p), ("scale", c_void_p), ("shift", c_void_p),
                ("u1_w", c_void_p), ("u1_b", c_void_p),
                ("tfeat", c_void_p), ("Ct", c_int), ("t_w", c_void_p), ("t_b", c_void_p),
                ("logits", c_void_p), ("bgfg", c_void_p), ("tn", c_void_p),
                ("act", c_int), ("act_beta", c_float), ("layernorm", c_int)]


class UbfGrads(Desc):
    _fields_ = [(n, c_void_p) for n in ("dut_w", "dut_b", "dgamma", "dbeta", "du1_w", "du1_b")]


class LossCfg(ctypes.Structure):
    _fields_ = [(n, c_float) for n in ("bg_weight", "fg_weight", "target_weight", "consistency_weight", "dice_weight",
                                       "ce_weight", "boundary_aware_weight", "contour_weight", "distance_weight")] + \
               [(n, c_int) for n in ("use_dynamic_weights", "use_boundary_aware", "use_contour", "use_distance",
                                     "contour_ks")]


class DistillCfg(ctypes.Structure):
    """include/hiseg_distill.h hiseg_distill_cfg"""
    _fields_ = [(n, c_float) for n in ("temperature", "kl_weight", "task_weight", "pos_weight")] + \
               [(n, c_int) for n in ("distill_terms", "distill_in_total", "use_dice", "has_target")] + \
               [("dev_scalars", c_void_p)]


DISTILL_NOUT = 5  # include/hiseg_distill.h HISEG_DISTILL_NOUT


class RoiTargetDesc(ctypes.Structure):
    """include/hiseg_data.h hiseg_roi_target_desc"""
    _fields_ = [("mask_offset", c_ll)] + [(n, c_int) for n in ("n_inst", "target", "h0", "w0", "x1", "y1", "x2",
                                                                 "y2", "img_w", "img_h")]


class HisegError(RuntimeError):
    """Raised when a libhiseg entry point returns a non-zero status."""


_lib = None
_load_error = None


def _declare(lib):
    P = c_void_p
    sigs = {
        "hiseg_version": ([], c_int),
        "hiseg_last_error_string": ([], ctypes.c_char_p),
        "hiseg_built_for_gfx950": ([], c_int),
        "hiseg_stream_create_cu_mask": ([ctypes.POINTER(ctypes.c_uint), c_int, ctypes.POINTER(c_void_p)], c_int),
        "hiseg_stream_destroy": ([P], c_int),
        "hiseg_comm_load": ([ctypes.c_char_p], c_int),
        "hiseg_comm_unique_id": ([P], c_int),
        "hiseg_comm_init": ([ctypes.POINTER(c_void_p), c_int, P, c_int, c_int], c_int),
        "hiseg_comm_all_reduce": ([P, P, c_ll, c_int, c_int, P], c_int),
        "hiseg_comm_destroy": ([P], c_int),
        "hiseg_roi_align_fwd": ([ctypes.POINTER(RoiAlignDesc), P], c_int),
        "hiseg_conv2d_fwd": ([ctypes.POINTER(Conv2dDesc), P], c_int),
        "hiseg_conv2d_fwd_variant": ([ctypes.POINTER(Conv2dDesc), c_int, P], c_int),
        "hiseg_conv2d_workspace_bytes": ([ctypes.POINTER(Conv2dDesc)], c_ll),
        "hiseg_maxpool2x2_fwd": ([c_int, P, c_int, c_int, c_int, c_int, P, P], c_int),
        "hiseg_attn_spatial_fwd": ([c_int, P, c_int, c_int, c_int, c_int, P, c_int, P, P, P, P], c_int),
        "hiseg_gap_splits": ([c_int], c_int),
        "hiseg_se_gate_fwd": ([c_int, P, c_int, c_int, c_int, P, P, c_int, P, P, c_int, c_float, P, P, P], c_int),
        "hiseg_channel_scale_fwd": ([c_int, P, c_int, c_int, c_int, P, P, P], c_int),
        "hiseg_dwconv_fwd": ([c_int, P, c_int, c_int, c_int, c_int, c_int, c_int, P, P, P, c_int, P,
                              c_int, c_int, P], c_int),
        "hiseg_dw_gap_tiles": ([c_int, c_int, c_int], c_int),
        "hiseg_dw_gap_parts": ([c_int, c_int, c_int, c_int, c_int, c_int, c_int], c_int),
        "hiseg_dwconv_gap_fwd": ([c_int, P, c_int, c_int, c_int, c_int, c_int, c_int, P, P, P, c_int, P,
                                  c_int, c_int, P, P], c_int),
        "hiseg_se_gate_partials_fwd": ([P, c_int, c_int, c_int, c_int, P, P, c_int, P, P, c_int, P, P], c_int),
        "hiseg_image_max_fwd": ([P, c_ll, P, P], c_int),
        "hiseg_input_norm_fwd": ([c_int, P, c_int, c_int, c_int, c_int, P, P, P, P, c_int, P], c_int),
        "hiseg_hier_combine_fwd": ([c_int, P, c_int, c_int, c_int, P, c_int, P, P, P, c_int, c_float, c_int, P, P,
                                    P, P, P, P, P, P], c_int),
        "hiseg_ubf_ln_tables": ([P, c_int, c_int, c_int, P, P, P, P, c_float, c_int, P, P, P, P, P], c_int),
        "hiseg_nhwc_to_nchw_fwd": ([c_int, P, c_int, c_int, c_int, c_int, c_int, c_int, P, P], c_int),
        "hiseg_nchw_to_nhwc_fwd": ([c_int, P, c_int, c_int, c_int, c_int, P, c_int, P], c_int),
        "hiseg_instance_masks_fwd": ([P, c_int, c_int, c_int, c_int, P, P], c_int),
        "hiseg_binary_masks_fwd": ([c_int, P, c_int, c_int, c_int, c_int, P, P, P, P], c_int),
        "hiseg_resize_bilinear_fwd": ([P, c_int, c_int, c_int, P, c_int, c_int, P], c_int),
        "hiseg_distance_mask_fwd": ([P, c_ll, P, P, P], c_int),
        "hiseg_output_conv_fwd": ([P, c_int, c_int, c_int, P, P, P, P], c_int),
        # ---- training (include/hiseg_train.h, hiseg_head_train.h, hiseg_loss.h)
        "hiseg_conv2d_wgrad_dims": ([ctypes.POINTER(Conv2dDesc), c_int, P, P, P], c_int),
        "hiseg_conv2d_wgrad": ([ctypes.POINTER(Conv2dDesc), P, c_int, c_int, c_int, P, c_int, P], c_int),
        "hiseg_wgrad_path_stats": ([ctypes.POINTER(c_ll), c_int], c_int),
        "hiseg_struct_sizes": ([ctypes.POINTER(c_ll), c_int], c_int),
        "hiseg_conv2d_stats_tiles": ([ctypes.POINTER(Conv2dDesc)], c_int),
        "hiseg_bn_finalize_n": ([P, c_int, c_int, c_ll, P, P, c_float, c_float, P, P, P, P, P, P, P], c_int),
        "hiseg_wgrad_last_path": ([], c_int),
        "hiseg_conv2d_wgrad_reduce": ([P, c_int, ctypes.POINTER(WgradMap), P, P, c_int, P], c_int),
        "hiseg_pack_weights": ([P, c_int, c_int, P], c_int),
        "hiseg_bn_partials": ([], c_int),
        "hiseg_bn_stats": ([c_int, P, c_ll, c_int, c_int, c_int, P, P], c_int),
        "hiseg_bn_finalize": ([P, c_int, c_ll, P, P, c_float, c_float, P, P, P, P, P, P, P], c_int),
        "hiseg_bn_apply": ([ctypes.POINTER(BnApplyDesc), P], c_int),
        "hiseg_bn_bwd": ([ctypes.POINTER(BnBwdDesc), P], c_int),
        "hiseg_dropout2d_mask": ([c_int, c_int, c_float, ctypes.c_ulonglong, P, P], c_int),
        "hiseg_dropout2d_mask_dev": ([c_int, c_int, c_float, P, ctypes.c_ulonglong, P, P], c_int),
        "hiseg_seed_advance": ([P, P], c_int),
        "hiseg_relu_bwd": ([c_int, c_ll, c_int, c_int, EwView, EwView, P, EwView, P], c_int),
        "hiseg_sigmoid_bwd": ([c_int, c_ll, c_int, EwView, EwView, EwView, P], c_int),
        "hiseg_gate_fwd": ([c_int, c_ll, c_int, EwView, EwView, EwView, P], c_int),
        "hiseg_gate_bwd": ([c_int, c_ll, c_int, EwView, EwView, EwView, EwView, c_int, EwView, P], c_int),
        "hiseg_add_inplace": ([c_int, c_ll, c_int, EwView, EwView, P], c_int),
        "hiseg_act_bwd_cvt": ([c_int, c_ll, c_int, EwView, EwView, c_int, EwView, c_int, P], c_int),
        "hiseg_act_bwd_pre": ([c_int, c_ll, c_int, EwView, EwView, c_int, c_float, EwView, c_int, P], c_int),
        "hiseg_ln_ws": ([c_int, c_int, c_int], c_ll),
        "hiseg_ln_fwd_stats": ([c_int, P, c_int, c_int, c_int, c_int, c_int, P, P, c_float, P, P, P, P, P, P],
                               c_int),
        "hiseg_ln_bwd": ([ctypes.POINTER(LnBwdDesc), P], c_int),
        "hiseg_maxpool2x2_bwd": ([c_int, P, c_int, c_int, c_int, c_int, P, P, c_int, P], c_int),
        "hiseg_resize_bilinear_bwd": ([P, c_int, c_int, c_int, c_int, c_int, P, P], c_int),
        "hiseg_upsample2x_bwd": ([c_int, c_ll, c_int, c_int, c_int, EwView, EwView, c_int, P], c_int),
        "hiseg_dw_train_fwd": ([c_int, P, c_int, c_int, c_int, c_int, c_int, c_int, P, P, c_int, c_int, P], c_int),
        "hiseg_dw_bwd_data": ([c_int, P, c_int, c_int, c_int, c_int, c_int, c_int, P, c_int, c_int, P, c_int, P],
                              c_int),
        "hiseg_dw_bwd_weight_ws": ([c_int, c_int, c_int, c_int, c_int, c_int], c_ll),
        "hiseg_dw_bwd_weight": ([c_int, P, P, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, P, P, P],
                                c_int),
        "hiseg_se_train_ws": ([c_int, c_int, c_int], c_ll),
        "hiseg_se_train_fwd": ([c_int, P, c_int, c_int, c_int, P, P, c_int, P, P, c_int, P, P, P, P, P, P], c_int),
        "hiseg_se_train_bwd": ([c_int, P, c_int, c_int, c_int, P, c_int, P, c_int, P, P, P, P, P, P, P, P, P, P, P],
                               c_int),
        "hiseg_attn_spatial_train_fwd": ([c_int, P, c_int, c_int, c_int, c_int, P, c_int, P, P, P, P, P, P], c_int),
        "hiseg_attn_spatial_ws": ([c_int, c_int, c_int, c_int], c_int),
        "hiseg_attn_spatial_bwd": ([c_int, P, c_int, c_int, c_int, c_int, P, c_int, P, P, P, P, P, P, P, P, P], c_int),
        "hiseg_attn_channel_ws": ([c_int, c_int, c_int], c_int),
        "hiseg_attn_channel_train_fwd": ([c_int, P, c_int, c_int, c_int, P, c_int, P, c_int, c_float, P, P, P, P, P,
                                          P, P], c_int),
        "hiseg_attn_channel_bwd": ([c_int, P, c_int, c_int, c_int, P, c_int, P, c_int, c_float, P, P, P, P, P, P, P,
                                    P, P, P], c_int),
        "hiseg_ubf_ws": ([c_int], c_int),
        "hiseg_ubf_train_fwd": ([ctypes.POINTER(UbfDesc), c_float, c_float, P, P, P, P], c_int),
        "hiseg_ubf_train_bwd": ([ctypes.POINTER(UbfDesc), P, P, P, P, P, P, P, ctypes.POINTER(UbfGrads), P], c_int),
        "hiseg_pw2_ws": ([c_int], c_int),
        "hiseg_pw2_bwd": ([c_int, P, c_ll, c_int, P, P, P, P, P, P, P], c_int),
        "hiseg_roi_align_ws": ([c_int], c_int),
        "hiseg_roi_align_bwd_affine": ([ctypes.POINTER(RoiAlignDesc), P, c_int, c_int, c_int, P, P, P, P], c_int),
        "hiseg_loss_state_init": ([P, P], c_int),
        "hiseg_loss_ws": ([c_int, c_int, c_int], c_ll),
        "hiseg_loss_fwd": ([ctypes.POINTER(LossCfg), c_int, c_int, c_int, P, P, P, P, P, P, P, P, P, P], c_int),
        "hiseg_loss_fwd_begin": ([ctypes.POINTER(LossCfg), c_int, c_int, c_int, P, P, P, P], c_int),
        "hiseg_loss_fwd_end": ([ctypes.POINTER(LossCfg), c_int, c_int, c_int, P, P, P, P, P, P, P, P, P, P, P],
                               c_int),
        "hiseg_loss_bwd": ([ctypes.POINTER(LossCfg), c_int, c_int, c_int, P, P, P, P, P, P, P, P, P, P, P, P, P, P],
                           c_int),
        "hiseg_distill_ws": ([c_int, c_int, c_int], c_ll),
        "hiseg_distill_loss_fwd": ([ctypes.POINTER(DistillCfg), c_int, c_int, c_int, P, P, P, P, P, P], c_int),
        "hiseg_distill_loss_bwd": ([ctypes.POINTER(DistillCfg), c_int, c_int, c_int, P, P, P, P, P, P, P], c_int),
        "hiseg_seg_confusion": ([P, c_int, P, P, c_int, c_int, c_ll, P, P], c_int),
        "hiseg_pil_bilinear_table": ([c_int, c_int, P, P, P], c_int),
        "hiseg_pil_resample_h": ([P, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, P, P, P, P], c_int),
        "hiseg_pil_resample_v": ([P, c_int, c_int, c_int, c_int, c_int, c_int, P, P, c_int, P, P], c_int),
        "hiseg_roi_targets": ([P, P, c_int, c_int, c_int, P, P], c_int),
        "hiseg_optim_blocks": ([], c_int),
        "hiseg_grad_norm_partials": ([P, c_ll, P, P], c_int),
        "hiseg_adamw_step": ([P, P, P, P, c_ll, c_float, c_float, c_float, c_float, c_float, c_float, c_float, P,
                              c_float, P, P], c_int),
        "hiseg_adamw_step_guarded": ([P, P, P, P, c_ll, c_float, c_float, c_float, c_float, c_float, P, c_float, P,
                                      P, c_int, P, P], c_int),
        "hiseg_adamw_max_segments": ([], c_int),
        "hiseg_debug_fill_lds": ([ctypes.c_uint, c_int, P], c_int),
        "hiseg_placement_stats": ([ctypes.POINTER(c_ll), ctypes.POINTER(c_ll), c_int], c_int),
        "hiseg_adamw_step_segmented": ([P, P, P, P, c_ll, c_float, c_float, c_float, c_float, c_float, c_float,
                                        c_float, P, c_float, P, P, c_int, P, c_int, P, P], c_int),
        "hiseg_adamw_step_segmented_dev": ([P, P, P, P, c_ll, P, c_float, c_float, c_float, c_float, c_float, P,
                                            c_float, P, P, c_int, P, c_int, P, P], c_int),
    }
    for name, (argtypes, restype) in sigs.items():
        fn = getattr(lib, name)
        fn.argtypes = argtypes
        fn.restype = restype
    return sigs.keys()


EXPORTED = None


def lib():
    """Return the loaded library, raising (never falling back) if it is unavailable."""
    global _lib, _load_error, EXPORTED
    if _lib is not None:
        return _lib
    if _load_error is not None:
        raise _load_error
    if not os.path.exists(LIB_PATH):
        _load_error = ImportError(
            f"libhiseg.so not found at {LIB_PATH}; build it with `make -C human-instance-segmentation_amd` "
            "or __graft_entry__.build()")
        raise _load_error
    try:
        handle = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
        EXPORTED = list(_declare(handle))
    except OSError as e:  # pragma: no cover - environment specific
        _load_error = ImportError(f"failed to load {LIB_PATH}: {e}")
        raise _load_error
    if handle.hiseg_built_for_gfx950() != 1:
        _load_error = ImportError("libhiseg.so was not built for gfx950")
        raise _load_error
    _lib = handle
    return _lib


def check(status: int, what: str) -> None:
    if status != 0:
        msg = lib().hiseg_last_error_string().decode(errors="replace")
        raise HisegError(f"{what} failed with status {status}: {msg}")


def placement_stats(reset: bool = False):
    """(declined, far): placement-dependent kernel choices since the last reset (include/hiseg.h)."""
    a, b = c_ll(), c_ll()
    check(lib().hiseg_placement_stats(ctypes.byref(a), ctypes.byref(b), int(reset)), "placement_stats")
    return a.value, b.value


WGRAD_PATHS = ("wide", "transposed_read", "generic_bf16", "f32", "halo")


def wgrad_path_stats(reset: bool = False) -> dict:
    """How many weight gradients each kernel computed since the last reset (include/hiseg_train.h):
    the wide tile, the transposed-read tile, the generic bf16 fallback, the f32 (parity) kernel, the halo tile."""
    c = (c_ll * 5)()
    check(lib().hiseg_wgrad_path_stats(c, int(reset)), "wgrad_path_stats")
    return dict(zip(WGRAD_PATHS, (int(v) for v in c)))


def stream_ptr(device=None) -> int:
    return torch.cuda.current_stream(device).cuda_stream
