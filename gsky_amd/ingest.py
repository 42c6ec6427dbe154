"""Native granule ingest: GeoTIFF and netCDF classic
files decoded by libgskyhip.so (ingest.hip) -- the GDALOpenEx / GDALRasterIO step of the
worker (worker/gdalprocess/warp.go:89-118, drill.go:61-69, 142) -- into host
arrays (tests) or straight into HBM tensors (the product path), plus the
metadata GDAL reports for the file (size, type, geotransform, nodata, EPSG,
overviews)."""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass
from typing import List, Optional, Tuple

import numpy as np

from ._lib import BYTE, FLOAT32, FLOAT64, INT16, INT32, UINT16, UINT32, GskyError, RasterInfo, lib

NP_DTYPE = {BYTE: np.uint8, UINT16: np.uint16, INT16: np.int16, UINT32: np.uint32, INT32: np.int32,
            FLOAT32: np.float32, FLOAT64: np.float64}


@dataclass
class GeoTiffInfo:
    xsize: int
    ysize: int
    n_bands: int
    dtype: int
    signed_byte: bool
    block: Tuple[int, int]
    compression: int
    predictor: int
    planar: int
    epsg: int                 # -1: MODIS sinusoidal sphere, 0: unknown
    geot: Tuple[float, ...]
    nodata: Optional[float]   # None when GDAL_NODATA is absent
    overviews: List[Tuple[int, int]]

    @property
    def srs(self) -> str:
        return "MODIS" if self.epsg == -1 else ("EPSG:%d" % self.epsg if self.epsg > 0 else "")

    def np_dtype(self):
        return np.int8 if self.signed_byte else NP_DTYPE[self.dtype]

    def level_shape(self, level: int) -> Tuple[int, int]:
        return (self.ysize, self.xsize) if level == 0 else self.overviews[level - 1][::-1]


def is_netcdf(path: str) -> bool:
    """warp.go:89-101: "NETCDF:..." and "*.nc" go through the netCDF driver."""
    return path.startswith("NETCDF:") or path.endswith(".nc")


def info(path: str) -> GeoTiffInfo:
    r = RasterInfo()
    fn = lib().gskyhip_netcdf_info if is_netcdf(path) else lib().gskyhip_geotiff_info
    rc = fn(path.encode(), C.byref(r))
    if rc:
        raise GskyError(rc, "raster info (%s)" % path)
    return GeoTiffInfo(r.xsize, r.ysize, r.n_bands, r.dtype, bool(r.signed_byte), (r.block_x, r.block_y),
                       r.compression, r.predictor, r.planar, r.epsg, tuple(r.geot),
                       r.nodata if r.has_nodata else None,
                       [(r.ovr_xsize[k], r.ovr_ysize[k]) for k in range(r.n_ovr)])


def netcdf_srs(path: str, srs_cf: int = 0) -> str:
    """The dataset SRS GSKY_netCDF reports under the srs_cf open option
    (warp.go:95): "EPSG:<n>", a PROJ string, "" (none) or "?" (a CF grid
    mapping outside the supported projections)."""
    buf = C.create_string_buffer(1024)
    rc = lib().gskyhip_netcdf_srs(path.encode(), int(srs_cf), buf, len(buf))
    if rc:
        raise GskyError(rc, "netcdf_srs")
    return buf.value.decode()


def read_host(path: str, band: int = 1, level: int = 0) -> np.ndarray:
    """Band `band` (1-based) of `level` decoded on the host (no device work)."""
    inf = info(path)
    out = np.empty(inf.level_shape(level), inf.np_dtype())
    if is_netcdf(path):
        rc = lib().gskyhip_netcdf_read_host(path.encode(), band, out.ctypes.data, out.nbytes)
    else:
        rc = lib().gskyhip_geotiff_read_host(path.encode(), band, level, out.ctypes.data, out.nbytes)
    if rc:
        raise GskyError(rc, "gskyhip_geotiff_read_host(%s)" % path)
    return out


def read(path: str, band: int = 1, level: int = 0, device=None):
    """The same decoded into a new HBM tensor (host-thread decompression,
    one H2D copy, GPU block assembly)."""
    import torch
    inf = info(path)
    tdt = {np.uint8: torch.uint8, np.int8: torch.int8, np.int16: torch.int16, np.uint16: torch.int16,
           np.int32: torch.int32, np.uint32: torch.int32, np.float32: torch.float32,
           np.float64: torch.float64}[inf.np_dtype()]
    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    out = torch.empty(inf.level_shape(level), dtype=tdt, device=dev)
    stream = torch.cuda.current_stream(dev).cuda_stream
    if is_netcdf(path):
        rc = lib().gskyhip_netcdf_read(path.encode(), band, C.c_void_p(out.data_ptr()),
                                       out.numel() * out.element_size(), C.c_void_p(stream))
    else:
        rc = lib().gskyhip_geotiff_read(path.encode(), band, level, C.c_void_p(out.data_ptr()),
                                        out.numel() * out.element_size(), C.c_void_p(stream))
    if rc:
        raise GskyError(rc, "gskyhip_geotiff_read(%s)" % path)
    return out


def register(path: str, band: int = 1) -> None:
    """Decode every level of (path, band) into library-owned HBM and register
    it for warp_operation_fast (worker.warp_raster)."""
    fn = lib().gskyhip_register_netcdf if is_netcdf(path) else lib().gskyhip_register_geotiff
    rc = fn(path.encode(), band)
    if rc:
        raise GskyError(rc, "register (%s)" % path)
