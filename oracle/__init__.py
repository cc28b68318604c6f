"""CPU oracle of the ROI-hierarchical segmentation path — TEST INFRASTRUCTURE ONLY.

A float32 restatement of the reference algorithm (PINTO0309/human-instance-segmentation), used
only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg as the checker / CPU
baseline.  The product (hiseg, libhiseg.so) never imports it.

Pinning (see DESIGN.md "Oracle"):
  * roi_align, the refined hierarchical head, ResidualBlock, EnhancedUNet and the assembled
    model from UNet logits onward are pinned to golden vectors produced by running the
    reference itself in the build container (tests/golden/gen_golden.py);
  * the EfficientNet-UNet (third-party smp 0.5.0 + timm 1.0.19, absent from the image) is
    a restatement of their published definitions: PARITY UNPINNED for that sub-network
    (checked only for shapes and state_dict key counts against the reference's heuristics).
"""
