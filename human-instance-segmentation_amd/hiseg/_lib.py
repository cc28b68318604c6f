"""ctypes binding of libhiseg.so (the C ABI declared in include/hiseg.h).

The library is loaded after ``import torch`` so that its ``libamdhip64.so.7`` dependency
resolves to the HIP runtime torch already loaded (one runtime, shared streams).  There is
no fallback: if the shared object is missing or was not built for gfx950, importing the
package's GPU path raises immediately.
"""
from __future__ import annotations

import ctypes
import os

import torch  # noqa: F401  (must precede the CDLL load: shares torch's HIP runtime)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("HISEG_LIB", os.path.join(_HERE, "libhiseg.so"))

HISEG_F32 = 0
HISEG_BF16 = 1
ACT_NONE, ACT_RELU, ACT_SIGMOID, ACT_SILU = 0, 1, 2, 3

c_int = ctypes.c_int
c_float = ctypes.c_float
c_void_p = ctypes.c_void_p
c_ll = ctypes.c_longlong


class RoiAlignDesc(ctypes.Structure):
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


class Conv2dDesc(ctypes.Structure):
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
    ]


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
        "hiseg_roi_align_fwd": ([ctypes.POINTER(RoiAlignDesc), P], c_int),
        "hiseg_conv2d_fwd": ([ctypes.POINTER(Conv2dDesc), P], c_int),
        "hiseg_conv2d_fwd_variant": ([ctypes.POINTER(Conv2dDesc), c_int, P], c_int),
        "hiseg_maxpool2x2_fwd": ([c_int, P, c_int, c_int, c_int, c_int, P, P], c_int),
        "hiseg_attn_spatial_fwd": ([c_int, P, c_int, c_int, c_int, c_int, P, c_int, P, P, P, P], c_int),
        "hiseg_gap_splits": ([c_int], c_int),
        "hiseg_se_gate_fwd": ([c_int, P, c_int, c_int, c_int, P, P, c_int, P, P, c_int, P, P, P], c_int),
        "hiseg_channel_scale_fwd": ([c_int, P, c_int, c_int, c_int, P, P, P], c_int),
        "hiseg_dwconv_fwd": ([c_int, P, c_int, c_int, c_int, c_int, c_int, c_int, P, P, P, c_int, P,
                              c_int, c_int, P], c_int),
        "hiseg_image_max_fwd": ([P, c_ll, P, P], c_int),
        "hiseg_input_norm_fwd": ([c_int, P, c_int, c_int, c_int, c_int, P, P, P, P, c_int, P], c_int),
        "hiseg_hier_combine_fwd": ([c_int, P, c_int, c_int, c_int, P, c_int, P, P, P, c_int, P, P, P, P,
                                    P, P, P, P], c_int),
        "hiseg_nhwc_to_nchw_fwd": ([c_int, P, c_int, c_int, c_int, c_int, c_int, c_int, P, P], c_int),
        "hiseg_nchw_to_nhwc_fwd": ([c_int, P, c_int, c_int, c_int, c_int, P, c_int, P], c_int),
        "hiseg_instance_masks_fwd": ([P, c_int, c_int, c_int, c_int, P, P], c_int),
        "hiseg_binary_masks_fwd": ([c_int, P, c_int, c_int, c_int, c_int, P, P, P, P], c_int),
        "hiseg_resize_bilinear_fwd": ([P, c_int, c_int, c_int, P, c_int, c_int, P], c_int),
        "hiseg_distance_mask_fwd": ([P, c_ll, P, P, P], c_int),
        "hiseg_output_conv_fwd": ([P, c_int, c_int, c_int, P, P, P, P], c_int),
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


def stream_ptr(device=None) -> int:
    return torch.cuda.current_stream(device).cuda_stream
