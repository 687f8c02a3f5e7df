"""sds_amd -- MI355X-native image decode-and-augment path for snap-research/sds.

Drop-in for ``sds.transforms.presets.create_standard_image_pipeline``: baseline-JPEG decode,
centre crop, Pillow-exact resampling, hflip and CHW/normalise run as hand-written gfx950 HIP
kernels behind the C-ABI in ``include/sdsj.h`` (``sds_amd/lib/libsdsj.so``).
"""
from . import functional, presets
from .engine import ImageDecodeError, JpegEngine, UnsupportedImageError, get_engine, raise_for_status
from .presets import create_standard_image_pipeline

__all__ = ["create_standard_image_pipeline", "presets", "functional", "JpegEngine", "get_engine",
           "ImageDecodeError", "UnsupportedImageError", "raise_for_status"]
