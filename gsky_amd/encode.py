"""Output codecs over the C-ABI (include/gskyhip.h): EncodePNG's png.Encode
(utils/ogc_encoders.go:139) for batches of RGBA tiles rendered into HBM, and
the WCS GeoTIFF of EncodeGdalOpen / EncodeGdal (ogc_encoders.go:277-450)."""
from __future__ import annotations

import ctypes as C
import os
from typing import List, Optional, Sequence, Tuple

import numpy as np
import torch

from ._lib import check, lib


def encode_png(rgba: torch.Tensor, sizes: Optional[Sequence[Tuple[int, int]]] = None,
               n_threads: Optional[int] = None) -> List[bytes]:
    """PNG bytes of every tile of an RGBA batch (n_tiles, max_h, max_w, 4)
    uint8 on the device; sizes (width, height) per tile (default the full
    slot), e.g. TileBatch.tile_sizes."""
    if rgba.dim() != 4 or rgba.shape[-1] != 4 or rgba.dtype != torch.uint8 or not rgba.is_cuda:
        raise ValueError("encode_png: (n, H, W, 4) uint8 device tensor expected")
    rgba = rgba.contiguous()
    n, mh, mw, _ = rgba.shape
    if sizes is None:
        sizes = [(mw, mh)] * n
    wh = np.ascontiguousarray(np.asarray(sizes, np.int32).reshape(n, 2))
    L = lib()
    ws = torch.empty(max(1, int(L.gskyhip_png_workspace_size(n, mw, mh))), dtype=torch.uint8, device=rgba.device)
    cap = int(max(L.gskyhip_png_bound(int(w), int(h)) for w, h in wh)) if n else 0
    out = np.empty(max(1, n * cap), np.uint8)
    lens = np.zeros(max(1, n), np.int64)
    threads = n_threads or max(1, min(16, os.cpu_count() or 1))
    check(L.gskyhip_encode_png(C.c_void_p(rgba.data_ptr()), n, mw, mh, mw * mh * 4, mw * 4,
                               wh.ctypes.data_as(C.c_void_p), C.c_void_p(ws.data_ptr()), ws.numel(),
                               out.ctypes.data_as(C.c_void_p), cap, lens.ctypes.data_as(C.c_void_p), threads,
                               C.c_void_p(torch.cuda.current_stream().cuda_stream)), "encode_png")
    return [out[t * cap:t * cap + int(lens[t])].tobytes() for t in range(n)]


_TIFF_DTYPES = {torch.uint8: 1, torch.int8: 100, torch.int16: 3, torch.float32: 6}


def encode_geotiff(bands: Sequence[torch.Tensor], geot: Sequence[float], epsg: int,
                   nodata: Optional[Sequence[float]] = None, names: Optional[Sequence[str]] = None,
                   block: Tuple[int, int] = (1024, 256), uint16: bool = False) -> bytes:
    """GeoTIFF bytes of a coverage: `bands` (height, width) device tensors of
    one dtype (uint8, int8, int16 -- uint16 when `uint16`, the bits held in
    int16 --, float32), what EncodeGdal writes for format "geotiff" with
    the block size ows.go passes (1024 x 256)."""
    if not bands:
        raise ValueError("encode_geotiff: no bands")
    dt = bands[0].dtype
    if dt not in _TIFF_DTYPES or any(b.dtype != dt or b.shape != bands[0].shape or not b.is_cuda for b in bands):
        raise ValueError("encode_geotiff: bands must be device tensors of one shape and a GeoTIFF dtype")
    code = 2 if (uint16 and dt == torch.int16) else _TIFF_DTYPES[dt]
    h, w = int(bands[0].shape[0]), int(bands[0].shape[1])
    bands = [b.contiguous() for b in bands]
    n = len(bands)
    L = lib()
    bx, by = int(block[0]), int(block[1])
    ws = torch.empty(max(1, int(L.gskyhip_geotiff_workspace_size(w, h, n, code, bx, by))), dtype=torch.uint8,
                     device=bands[0].device)
    cap = int(L.gskyhip_geotiff_bound(w, h, n, code, bx, by))
    if cap <= 0:
        raise ValueError("encode_geotiff: bad size / block")
    out = np.empty(cap, np.uint8)
    size = C.c_int64(0)
    ptrs = (C.c_void_p * n)(*[b.data_ptr() for b in bands])   # EmptyTile bands: skipped by the writer
    gt = (C.c_double * 6)(*[float(v) for v in geot])
    nd = np.asarray(nodata, np.float64) if nodata is not None else None
    nm = (C.c_char_p * n)(*[s.encode() for s in names]) if names is not None else None
    check(L.gskyhip_encode_geotiff(ptrs, n, code, w, h, gt, int(epsg),
                                   nd.ctypes.data_as(C.c_void_p) if nd is not None else None, nm, bx, by,
                                   C.c_void_p(ws.data_ptr()), ws.numel(), out.ctypes.data_as(C.c_void_p), cap,
                                   C.byref(size), C.c_void_p(torch.cuda.current_stream().cuda_stream)),
          "encode_geotiff")
    return out[:size.value].tobytes()


def encode_netcdf(bands: Sequence[torch.Tensor], geot: Sequence[float], epsg: int,
                  nodata: Optional[Sequence[float]] = None, names: Optional[Sequence[str]] = None,
                  zlevel: int = 6, uint16: bool = False, threads: int = 16) -> bytes:
    """netCDF bytes of a coverage: what EncodeGdal writes for format
    "netcdf" with COMPRESS=DEFLATE, ZLEVEL=6 (utils/ogc_encoders.go:263-301):
    `bands` (height, width) device tensors of one dtype (uint8, int8, int16 --
    uint16 when `uint16`, the bits held in int16 --, float32)."""
    if not bands:
        raise ValueError("encode_netcdf: no bands")
    dt = bands[0].dtype
    if dt not in _TIFF_DTYPES or any(b.dtype != dt or b.shape != bands[0].shape or not b.is_cuda for b in bands):
        raise ValueError("encode_netcdf: bands must be device tensors of one shape and a supported dtype")
    code = 2 if (uint16 and dt == torch.int16) else _TIFF_DTYPES[dt]
    h, w = int(bands[0].shape[0]), int(bands[0].shape[1])
    bands = [b.contiguous() for b in bands]
    n = len(bands)
    L = lib()
    cap = int(L.gskyhip_netcdf_bound(w, h, n, code))
    if cap <= 0:
        raise ValueError("encode_netcdf: bad size / type")
    out = np.empty(cap, np.uint8)
    size = C.c_int64(0)
    ptrs = (C.c_void_p * n)(*[b.data_ptr() for b in bands])
    gt = (C.c_double * 6)(*[float(v) for v in geot])
    nd = np.asarray(nodata, np.float64) if nodata is not None else None
    nm = (C.c_char_p * n)(*[s.encode() for s in names]) if names is not None else None
    check(L.gskyhip_encode_netcdf(ptrs, n, code, w, h, gt, int(epsg),
                                  nd.ctypes.data_as(C.c_void_p) if nd is not None else None, nm, int(zlevel),
                                  int(threads), out.ctypes.data_as(C.c_void_p), cap, C.byref(size),
                                  C.c_void_p(torch.cuda.current_stream().cuda_stream)), "encode_netcdf")
    return out[:size.value].tobytes()


def encode_netcdf_host(bands: Sequence[np.ndarray], geot: Sequence[float], epsg: int,
                       nodata: Optional[Sequence[float]] = None, names: Optional[Sequence[str]] = None,
                       zlevel: int = 6, uint16: bool = False, threads: int = 4) -> bytes:
    """encode_netcdf of host numpy bands (gskyhip_encode_netcdf_host; no device)."""
    codes = {np.dtype(np.uint8): 1, np.dtype(np.int8): 100, np.dtype(np.int16): 3, np.dtype(np.float32): 6,
             np.dtype(np.uint16): 2}
    if not bands:
        raise ValueError("encode_netcdf_host: no bands")
    dt = np.dtype(bands[0].dtype)
    if dt not in codes or any(b.dtype != dt or b.shape != bands[0].shape for b in bands):
        raise ValueError("encode_netcdf_host: bands must be arrays of one shape and a supported dtype")
    code = codes[dt]
    h, w = int(bands[0].shape[0]), int(bands[0].shape[1])
    bands = [np.ascontiguousarray(b) for b in bands]
    n = len(bands)
    L = lib()
    cap = int(L.gskyhip_netcdf_bound(w, h, n, code))
    out = np.empty(cap, np.uint8)
    size = C.c_int64(0)
    ptrs = (C.c_void_p * n)(*[b.ctypes.data for b in bands])
    gt = (C.c_double * 6)(*[float(v) for v in geot])
    nd = np.asarray(nodata, np.float64) if nodata is not None else None
    nm = (C.c_char_p * n)(*[s.encode() for s in names]) if names is not None else None
    check(L.gskyhip_encode_netcdf_host(ptrs, n, code, w, h, gt, int(epsg),
                                       nd.ctypes.data_as(C.c_void_p) if nd is not None else None, nm, int(zlevel),
                                       int(threads), out.ctypes.data_as(C.c_void_p), cap, C.byref(size)),
          "encode_netcdf_host")
    return out[:size.value].tobytes()
