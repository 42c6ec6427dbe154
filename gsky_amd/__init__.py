"""gsky_amd -- MI355X-native GSKY raster hot path.

warp (reprojection + NN/bilinear resampling) -> time-ordered nodata-aware
mosaic -> byte scaling -> palette/RGBA, and the drill zonal reduction, as
hand-written HIP kernels for gfx950 behind a C-ABI (include/gskyhip.h,
libgskyhip.so).  See DESIGN.md.
"""
from ._lib import GskyError, lib  # noqa: F401
from .raster import (FlexRaster, Mask, Palette, ScaleParams, band_math, compute_mask, encode_rgba,  # noqa: F401
                     gradient_rgba_palette, raster_merger_run, scale, scale_legacy)
from .tiles import GranuleSet, PipelinedBatch, RenderGraph, TileBatch, bbox_to_geot  # noqa: F401
from .service import WarpService  # noqa: F401

__version__ = "0.1.0"
