"""hiseg — MI355X-native ROI-hierarchical instance segmentation (drop-in for the RGB
hierarchical path of PINTO0309/human-instance-segmentation).  See DESIGN.md."""
__version__ = "0.1.0"
