"""Worker-side mirror of the gRPC `warp` and `extent` ops over the MI355X drop-in.

`warp_raster(GeoRPCGranule) -> Result` follows WarpRaster
(worker/gdalprocess/warp.go:489-584): it marshals the request into the C-ABI
call `warp_operation_fast` (exported by libgskyhip.so with the reference's
exact signature, warp.go:82), copies the malloc'd window back and frees it,
and maps the data type code to the RasterType name (warp.go:576-581).  The
granule behind `Path` must have been registered (HBM-resident) first:
`register_granule` replaces GDALOpenEx for this path.
`compute_reproject_extent(GeoRPCGranule) -> Result` follows
ComputeReprojectExtent (warp.go:433-487) over gskyhip_compute_reproject_extent.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field
from typing import List, Optional

import numpy as np
import torch

from . import _lib
from ._lib import check, lib
from .tiles import DTYPE_OF_TORCH, _to_device_bytes, parse_crs

GDAL_TYPES = {0: "Unkown", 1: "Byte", 2: "UInt16", 3: "Int16", 4: "UInt32", 5: "Int32", 6: "Float32",
              7: "Float64", 8: "CInt16", 9: "CInt32", 10: "CFloat32", 11: "CFloat64", 12: "TypeCount"}
NP_OF = {"Byte": np.uint8, "SignedByte": np.int8, "UInt16": np.uint16, "Int16": np.int16,
         "Float32": np.float32}

_REGISTERED = {}


@dataclass
class GeoRPCGranule:
    """gdalservice.GeoRPCGranule (worker/gdalservice/gdalservice.proto:7-26)."""
    operation: str = "warp"
    path: str = ""
    geometry: str = ""
    bands: List[int] = field(default_factory=lambda: [1])
    height: int = 0
    width: int = 0
    srcSRS: str = ""
    srcGeot: List[float] = field(default_factory=list)
    dstSRS: str = ""
    dstGeot: List[float] = field(default_factory=list)
    bandStrides: int = 0
    geoLocOpts: List[str] = field(default_factory=list)
    drillDecileCount: int = 0
    clipUpper: float = 0.0
    clipLower: float = 0.0
    sRSCf: int = 0
    pixelCount: int = 0
    vRT: str = ""


@dataclass
class Raster:
    """gdalservice.Raster (proto:28-33)."""
    data: bytes = b""
    noData: float = 0.0
    rasterType: str = ""
    bbox: List[int] = field(default_factory=list)


@dataclass
class Result:
    """gdalservice.Result (proto:77-85); error == "OK" on success."""
    raster: Optional[Raster] = None
    error: str = ""
    bytesRead: int = 0


def register_granule(path: str, band: int, data: torch.Tensor, geot, srs: str = "",
                     nodata: Optional[float] = None, overviews=(), signed_byte: bool = False,
                     block=(0, 0)) -> None:
    """Make an HBM-resident band visible to warp_operation_fast under (path, band).
    `block` = GDALGetBlockSize of the band ((0, 0): xsize x 1), for bytesRead."""
    d = data.contiguous()
    ovr = [o.contiguous() for o in overviews]
    g = _lib.Granule()
    g.block_x, g.block_y = block
    g.data = d.data_ptr()
    g.dtype = DTYPE_OF_TORCH[d.dtype]
    g.ysize, g.xsize = d.shape
    g.signed_byte = int(signed_byte or d.dtype == torch.int8)
    for k in range(6):
        g.geot[k] = geot[k]
    g.nodata = nodata if nodata is not None else -1e10
    g.has_nodata = int(nodata is not None)
    g.n_ovr = len(ovr)
    for k, o in enumerate(ovr):
        g.ovr_data[k] = o.data_ptr()
        g.ovr_ysize[k], g.ovr_xsize[k] = o.shape
    check(lib().gskyhip_register_granule(path.encode(), band, C.byref(g), srs.encode() if srs else None),
          "register")
    _REGISTERED[(path, band)] = (d, ovr, g, srs)  # keep the HBM buffers alive


def unregister_all() -> None:
    lib().gskyhip_unregister_all()
    _REGISTERED.clear()


def warp_raster(req: GeoRPCGranule) -> Result:
    """WarpRaster (warp.go:489-584) through the C-ABI drop-in."""
    L = lib()
    dst = req.dstSRS.encode() if req.dstSRS else None
    src = req.srcSRS.encode() if req.srcSRS else None
    src_gt = (C.c_double * 6)(*req.srcGeot) if req.srcGeot else None
    dst_gt = (C.c_double * 6)(*req.dstGeot)
    buf = C.c_void_p()
    size = C.c_int()
    bbox = (C.c_int * 4)()
    nod = C.c_double()
    dt = C.c_int()
    br = C.c_int()
    geo = None
    if req.geoLocOpts:   # NULL-terminated C strings (warp.go:514-526)
        geo = (C.c_char_p * (len(req.geoLocOpts) + 1))(*[o.encode() for o in req.geoLocOpts], None)
    rc = L.warp_operation_fast(req.path.encode(), src, src_gt, geo, dst, dst_gt, req.width, req.height,
                               req.bands[0], req.sRSCf, C.byref(buf), C.byref(size), bbox, C.byref(nod),
                               C.byref(dt), C.byref(br))
    if rc != 0:
        return Result(error="warp_operation() fail: %d" % rc)
    data = C.string_at(buf, size.value)
    C.CDLL(None).free(buf)                     # C.free(dstBufC), warp.go:574
    rtype = "SignedByte" if dt.value == 100 else GDAL_TYPES.get(dt.value, "Unkown")
    if req.srcGeot:
        req.srcGeot[:] = list(src_gt)          # warp.go:186-189 rescales the caller's srcGeot
    return Result(raster=Raster(data=data, noData=nod.value, rasterType=rtype, bbox=list(bbox)),
                  error="OK", bytesRead=br.value)


def raster_array(r: Raster) -> np.ndarray:
    """Result.Raster -> (h, w) array (what tile_grpc.go:228-241 reinterprets)."""
    return np.frombuffer(r.data, dtype=NP_OF[r.rasterType]).reshape(r.bbox[3], r.bbox[2])


def compute_reproject_extent(req: GeoRPCGranule) -> Result:
    """ComputeReprojectExtent (warp.go:433-487): the pixel counts of the
    request's bbox req.dstGeot[0..3] (xMin, yMin, xMax, yMax) at the
    resolution GDALSuggestedWarpOutput suggests for the dataset at req.path in
    req.dstSRS.  Result.Raster: two Go ints (int64, little endian)
    [nPixels, nLines], RasterType "Int", NoData 0."""
    ent = next((v for (p, _), v in sorted(_REGISTERED.items(), key=lambda kv: kv[0][1]) if p == req.path), None)
    if ent is None:   # GDALOpenEx failed
        return Result(error="Failed to open existing dataset: %s" % req.path)
    d, _, g, srs = ent
    try:
        crs = [parse_crs(srs)]
        dst_crs = -1
        if req.dstSRS:
            crs.append(parse_crs(req.dstSRS))
            dst_crs = 1
    except Exception:
        return Result(error="GDALCreateGenImgProjTransformer() failed")
    dev = d.device
    gc = _lib.Granule.from_buffer_copy(g)
    gc.crs = 0
    gran = _to_device_bytes(gc, dev)
    crs_t = _to_device_bytes((_lib.Crs * len(crs))(*crs), dev)
    bbox = torch.tensor([float(v) for v in req.dstGeot[:4]], dtype=torch.float64, device=dev)
    out = torch.zeros(2, dtype=torch.int32, device=dev)
    status = torch.zeros(1, dtype=torch.int32, device=dev)
    stream = C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    check(lib().gskyhip_compute_reproject_extent(C.c_void_p(gran.data_ptr()), 1, C.c_void_p(crs_t.data_ptr()),
                                                 len(crs), dst_crs, C.c_void_p(bbox.data_ptr()),
                                                 C.c_void_p(out.data_ptr()), C.c_void_p(status.data_ptr()),
                                                 stream), "compute_reproject_extent")
    if int(status.item()) != 0:
        return Result(error="GDALSuggestedWarpOutput() failed")
    data = np.asarray(out.cpu().numpy(), dtype="<i8").tobytes()   # []int{nPixels, nLines}
    return Result(raster=Raster(data=data, noData=0.0, rasterType="Int"), error="OK")
