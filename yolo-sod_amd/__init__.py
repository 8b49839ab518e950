"""yolosod_amd - MI355X (gfx950) native inference hot path of YOLO-SOD (quitedob/yolo-sod).

The package directory is ``yolo-sod_amd/``; it registers itself as the importable module ``yolosod_amd`` (see
``yolosod_import.py`` at the repository root).

Hot path (hand-written HIP, ``csrc/``, C ABI in ``include/yolosod_hip.h``): the MAFN operators SE / CBAM / CA /
A2_Attn / SwinBlock, the Detect decode and batched class-wise NMS. Backbone/neck convolutions stay PyTorch-ROCm.
"""
from . import _hip  # noqa: F401
from .nn.tasks import DetectionModel, build_model, parse_model, yaml_model_load  # noqa: F401
from .utils.ops import non_max_suppression, non_max_suppression_padded  # noqa: F401

__version__ = "0.1.0"
