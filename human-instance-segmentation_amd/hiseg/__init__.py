"""hiseg — MI355X-native ROI-hierarchical instance segmentation.

Drop-in for the RGB hierarchical path of PINTO0309/human-instance-segmentation
(HierarchicalRGBSegmentationModelWithFullImagePretrainedUNet + RefinedHierarchicalSegmentationHead
on a full-image EfficientNet-UNet).  Module tree and state_dict keys follow the reference;
every forward runs on libhiseg (hand-written gfx950 HIP kernels, C ABI in include/hiseg.h).
"""
from .layers import (  # noqa: F401
    ChannelAttentionModule, ContourDetectionBranch, DistanceTransformDecoder, EnhancedUNet,
    ExtendedHierarchicalSegmentationHeadUNetV2, LayerNorm2d, RefinedHierarchicalSegmentationHead, ResidualBlock,
    SpatialAttentionModule)
from .effunet import EfficientNetUnet  # noqa: F401
from .model import (  # noqa: F401
    DynamicRoIAlign, HierarchicalRGBSegmentationModelWithFullImagePretrainedUNet, PreTrainedPeopleSegmentationUNet,
    PreTrainedPeopleSegmentationUNetWrapper, RGBHierarchicalExportWrapper, StreamPipelinedExport,
    create_rgb_hierarchical_model)

from .losses import RefinedHierarchicalLoss  # noqa: F401,E402
from .optim import FusedAdamW, cosine_lr  # noqa: F401,E402
from .graphs import GraphedStep, GraphedBranchStep  # noqa: F401,E402
from .checkpoint import resume_from_checkpoint, save_checkpoint  # noqa: F401,E402
from .data import GpuRoiBatchBuilder, resize_bilinear_pil  # noqa: F401,E402
from .metrics import (  # noqa: F401,E402
    SegmentationMetrics, calculate_confusion_matrix, calculate_detection_metrics, calculate_iou, evaluate_model,
)
from .distill import (  # noqa: F401,E402
    DistillationUNetWrapper, UNetDecoderOnly, UNetDistillationLoss, create_unet_distillation_model)

__version__ = "0.2.0"


def set_compute_dtype(model, dtype):
    """Select the HIP compute precision of a model: torch.float32 (parity) or torch.bfloat16 (throughput)."""
    import torch
    if dtype not in (torch.float32, torch.bfloat16):
        raise TypeError(dtype)
    for m in model.modules():
        m.hiseg_dtype = dtype
    return model
