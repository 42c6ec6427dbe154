"""gsky_amd -- MI355X-native GSKY raster hot path.

warp (reprojection + NN/bilinear resampling) -> time-ordered nodata-aware
mosaic -> byte scaling -> palette/RGBA, and the drill zonal reduction, as
hand-written HIP kernels for gfx950 behind a C-ABI (include/gskyhip.h,
libgskyhip.so).  See DESIGN.md.

The public names are loaded on first use (PEP 562), so that processes which
only talk to the C-ABI -- warp workers forwarding to the per-node service,
gsky_amd.loadgen -- do not import torch.
"""
from ._lib import GskyError, lib  # noqa: F401

_LAZY = {
    "FlexRaster": "raster", "Mask": "raster", "Palette": "raster", "ScaleParams": "raster", "band_math": "raster",
    "compute_mask": "raster", "encode_rgba": "raster", "gradient_rgba_palette": "raster",
    "raster_merger_run": "raster", "scale": "raster", "scale_legacy": "raster",
    "GranuleSet": "tiles", "PipelinedBatch": "tiles", "RenderGraph": "tiles", "TileBatch": "tiles",
    "bbox_to_geot": "tiles", "WarpService": "service",
}

__version__ = "0.1.0"


def __getattr__(name):
    mod = _LAZY.get(name)
    if mod is None:
        raise AttributeError("module 'gsky_amd' has no attribute %r" % name)
    import importlib
    v = getattr(importlib.import_module("." + mod, __name__), name)
    globals()[name] = v
    return v


def __dir__():
    return sorted(list(globals()) + list(_LAZY))
