"""MI355X-native Video-Depth-Anything clip forward (DINOv2 encoder + temporal DPT head).

Import as ``vda_amd`` (the repo-root shim ``vda_amd.py`` maps the hyphenated directory name).
Public API mirrors the reference: ``VideoDepthAnything`` (video_depth.py:35-65) plus
``build_model``; kernels live in ``libvda.so`` behind the C ABI of ``include/vda.h``.
"""
from .model import VideoDepthAnything, build_model, MODEL_CONFIGS, ENCODER_CFG  # noqa: F401
from ._lib import VDAUnavailable, VDAError, lib as _libvda  # noqa: F401

__all__ = ["VideoDepthAnything", "build_model", "MODEL_CONFIGS", "ENCODER_CFG", "VDAUnavailable", "VDAError"]
