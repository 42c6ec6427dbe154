"""Host mirror of GSKY's raster operators over the MI355X kernels.

Names, argument meaning and error behaviour follow the reference operators
(chuc92man/gsky):

  ScaleParams, scale()          utils/raster_scaler.go:8-13, 30-346
  scale_legacy()                processor/tile_scaler.go:17-112
  Palette, gradient_rgba_palette()  utils/config.go:82-86, utils/palette.go:27-69
  encode_rgba()                 utils/ogc_encoders.go:82-134 (pixel loop; png.Encode excluded)
  Mask, compute_mask()          utils/config.go:73-80, processor/tile_merger.go:314-445
  FlexRaster, raster_merger_run()  processor/tile_types.go:95-106, tile_merger.go:447-503

Data live in HBM as torch tensors on a ROCm device; every pixel operation
runs in libgskyhip.so.  Nothing here computes pixels on the CPU.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch

from . import _lib
from ._lib import check, lib

TYPE_CODES = {"Byte": _lib.BYTE, "SignedByte": _lib.SIGNEDBYTE, "Int16": _lib.INT16,
              "UInt16": _lib.UINT16, "Float32": _lib.FLOAT32}
TYPE_NAMES = {v: k for k, v in TYPE_CODES.items()}
TORCH_OF = {"Byte": torch.uint8, "SignedByte": torch.int8, "Int16": torch.int16,
            "UInt16": torch.uint16, "Float32": torch.float32}


def type_of_tensor(t: torch.Tensor) -> str:
    return {torch.uint8: "Byte", torch.int8: "SignedByte", torch.int16: "Int16",
            torch.uint16: "UInt16", torch.float32: "Float32"}[t.dtype]


def _stream():
    return C.c_void_p(torch.cuda.current_stream().cuda_stream)


def _dev(t: torch.Tensor) -> torch.Tensor:
    if not t.is_cuda:
        raise ValueError("gsky_amd operators take HBM-resident (cuda) tensors")
    return t.contiguous()


# ---------------------------------------------------------------- scale
@dataclass
class ScaleParams:
    """utils.ScaleParams (raster_scaler.go:8-13)."""
    offset: float = 0.0
    scale: float = 0.0
    clip: float = 0.0
    colour_scale: int = 0

    def c(self) -> _lib.ScaleParams:
        return _lib.ScaleParams(float(self.offset), float(self.scale), float(self.clip),
                                int(self.colour_scale), 0)


def scale(rasters: Sequence[torch.Tensor], nodata: Sequence[float], params: ScaleParams,
          types: Optional[Sequence[str]] = None) -> List[torch.Tensor]:
    """utils.Scale (raster_scaler.go:334-346): one uint8 raster per input,
    0xFF = nodata.  Byte inputs are scaled in place, like the reference."""
    out = []
    sp = params.c()
    for i, r in enumerate(rasters):
        r = _dev(r)
        tname = types[i] if types else type_of_tensor(r)
        if tname not in TYPE_CODES:
            raise ValueError("Raster type not implemented")
        o = torch.empty(r.shape, dtype=torch.uint8, device=r.device)
        check(lib().gskyhip_scale(C.c_void_p(r.data_ptr()), TYPE_CODES[tname], r.numel(), float(nodata[i]),
                                  C.byref(sp), C.c_void_p(o.data_ptr()), _stream()), "Scale")
        out.append(o)
    return out


def scale_legacy(r: torch.Tensor, nodata: float, params: ScaleParams) -> torch.Tensor:
    """processor.RasterScaler.Run (tile_scaler.go:17-112; no callers in the reference)."""
    r = _dev(r)
    o = torch.empty(r.shape, dtype=torch.uint8, device=r.device)
    sp = params.c()
    check(lib().gskyhip_scale_legacy(C.c_void_p(r.data_ptr()), TYPE_CODES[type_of_tensor(r)], r.numel(),
                                     float(nodata), C.byref(sp), C.c_void_p(o.data_ptr()), _stream()),
          "RasterScaler")
    return o


# ---------------------------------------------------------------- palette / RGBA
@dataclass
class Palette:
    """utils.Palette (utils/config.go:82-86); colours are (R, G, B, A)."""
    colours: List[Sequence[int]]
    interpolate: bool = True
    name: str = ""


def gradient_rgba_palette(palette: Optional[Palette]) -> Optional[np.ndarray]:
    """GradientRGBAPalette (utils/palette.go:27-69): 256 x RGBA uint8."""
    if palette is None:
        return None
    col = np.ascontiguousarray(np.asarray(palette.colours, np.uint8).reshape(-1, 4))
    ramp = np.zeros((256, 4), np.uint8)
    check(lib().gskyhip_gradient_palette(col.ctypes.data_as(C.c_void_p), len(col), int(palette.interpolate),
                                         ramp.ctypes.data_as(C.c_void_p)), "GradientRGBAPalette")
    return ramp


def encode_rgba(bands: Sequence[torch.Tensor], palette: Optional[Palette] = None) -> torch.Tensor:
    """EncodePNG pixel loop (ogc_encoders.go:86-133): (H, W, 4) uint8 RGBA."""
    if len(bands) not in (1, 3):
        raise ValueError("Cannot encode other than 1 or 3 namespaces into a PNG: Received %d" % len(bands))
    bs = [_dev(b) for b in bands]
    h, w = bs[0].shape
    ramp = gradient_rgba_palette(palette) if (palette is not None and len(bs) == 1) else None
    ramp_d = torch.from_numpy(ramp).to(bs[0].device) if ramp is not None else None
    out = torch.empty((h, w, 4), dtype=torch.uint8, device=bs[0].device)
    arr = (C.c_void_p * len(bs))(*[b.data_ptr() for b in bs])
    check(lib().gskyhip_encode_rgba(arr, len(bs), w, h,
                                    C.c_void_p(ramp_d.data_ptr()) if ramp_d is not None else None,
                                    C.c_void_p(out.data_ptr()), _stream()), "EncodePNG")
    return out


# ---------------------------------------------------------------- masks / merge
@dataclass
class Mask:
    """utils.Mask (utils/config.go:73-80)."""
    id: str
    value: str = ""
    bit_tests: List[str] = field(default_factory=list)
    inclusive: bool = False

    def c(self, ns_slot: int) -> _lib.Mask:
        m = _lib.Mask()
        m.ns = ns_slot
        m.inclusive = int(self.inclusive)
        m.n_bit_tests = len(self.bit_tests)
        if len(self.bit_tests) > _lib.MAX_BIT_TESTS:
            raise ValueError("too many bit tests")
        m._keep = [s.encode() for s in self.bit_tests] + ([self.value.encode()] if self.value else [])
        m.value = self.value.encode() if self.value else None
        for i, s in enumerate(self.bit_tests):
            m.bit_tests[i] = s.encode()
        return m


def compute_mask(mask: Mask, data: torch.Tensor, rtype: Optional[str] = None) -> torch.Tensor:
    """ComputeMask (tile_merger.go:314-445) -> bool tensor."""
    d = _dev(data)
    rtype = rtype or type_of_tensor(d)
    if not mask.value:
        if not mask.bit_tests:
            raise ValueError("Please specify either mask.Value or mask.BitTests")
        if len(mask.bit_tests) % 2:
            raise ValueError("The entries in mask.BitTests must be in pairs")
    if rtype not in ("Byte", "SignedByte", "Int16", "UInt16"):
        raise ValueError("Type %s cannot contain a bit mask" % rtype)
    out = torch.empty(d.shape, dtype=torch.uint8, device=d.device)
    m = mask.c(0)
    check(lib().gskyhip_compute_mask(C.c_void_p(d.data_ptr()), TYPE_CODES[rtype], d.numel(), C.byref(m),
                                     C.c_void_p(out.data_ptr()), _stream()), "ComputeMask")
    return out.bool()


def fnv32a(s: str) -> int:
    b = s.encode()
    return lib().gskyhip_fnv32a(b, len(b))


@dataclass
class FlexRaster:
    """processor.FlexRaster (tile_types.go:95-106): one warped granule window."""
    data: torch.Tensor            # (DataHeight, DataWidth), HBM
    width: int
    height: int
    off_x: int
    off_y: int
    type: str
    nodata: float
    namespace: str
    timestamp: float
    polygon: str = ""


def raster_merger_run(rasters: Sequence[FlexRaster], namespaces: Sequence[str],
                      mask: Optional[Mask] = None) -> Dict[str, Optional[tuple]]:
    """RasterMerger.Run over one batch (tile_merger.go:447-503): returns
    {namespace: (canvas tensor, nodata)} (None for namespaces never merged)."""
    ns_list = list(namespaces)
    if mask is not None and mask.id not in ns_list:
        ns_list.append(mask.id)
    slot = {ns: i for i, ns in enumerate(ns_list)}
    arr = (_lib.FlexRasterC * max(1, len(rasters)))()
    keep = []
    for i, r in enumerate(rasters):
        if r.type not in TYPE_CODES:
            raise ValueError("MergeMaskedRaster hasn't been implemented for Raster type %s" % r.type)
        d = _dev(r.data)
        keep.append(d)
        arr[i].data = d.data_ptr()
        arr[i].data_h, arr[i].data_w = d.shape
        arr[i].width, arr[i].height = r.width, r.height
        arr[i].off_x, arr[i].off_y = r.off_x, r.off_y
        arr[i].dtype = TYPE_CODES[r.type]
        arr[i].ns = slot[r.namespace]
        arr[i].nodata = r.nodata
        arr[i].timestamp = r.timestamp
        arr[i].polygon_hash = fnv32a(r.polygon)
    width = rasters[0].width if rasters else 0
    height = rasters[0].height if rasters else 0
    dev = keep[0].device if keep else torch.device("cuda")
    canv = [torch.empty(width * height * 4, dtype=torch.uint8, device=dev) for _ in ns_list]
    cptr = (C.c_void_p * len(ns_list))(*[c.data_ptr() for c in canv])
    created = (C.c_int32 * len(ns_list))()
    dtypes = (C.c_int32 * len(ns_list))()
    nod = (C.c_double * len(ns_list))()
    m = mask.c(slot[mask.id]) if mask is not None else None
    check(lib().gskyhip_merge_rasters(arr, len(rasters), C.byref(m) if m is not None else None, cptr,
                                      len(ns_list), created, dtypes, nod, _stream()), "RasterMerger")
    out = {}
    for k, ns in enumerate(ns_list):
        if not created[k]:
            out[ns] = None
            continue
        tname = TYPE_NAMES[dtypes[k]]
        nbytes = {"Byte": 1, "SignedByte": 1, "Int16": 2, "UInt16": 2, "Float32": 4}[tname]
        t = canv[k][: width * height * nbytes].view(TORCH_OF[tname]).reshape(height, width)
        out[ns] = (t, nod[k])
    return out


# ---------------------------------------------------------------- band-math
def band_math(expr: str, variables: Sequence[tuple], out_nodata: float) -> torch.Tensor:
    """Band-math of RasterMerger.Run (tile_merger.go:654-731) for one
    expression over one axis: `variables` = [(name, canvas tensor, nodata)]
    (typed canvases of the merged namespaces, all the same shape), result a
    float32 tensor of that shape.  Pixels where any variable is its nodata,
    and non-finite results, are `out_nodata` (the first namespace's nodata).
    Raises GskyError(-1) on a parse error or unknown variable."""
    if not variables:
        raise ValueError("band_math needs the axis variables")
    if len(variables) > 8:
        raise ValueError("at most 8 variables per axis (GSKYHIP_BANDMATH_MAX_VARS)")
    shape = variables[0][1].shape
    ts = [_dev(v[1]) for v in variables]
    if any(t.shape != shape for t in ts):
        raise ValueError("variables must share one canvas shape")
    out = torch.empty(shape, dtype=torch.float32, device=ts[0].device)
    names = (C.c_char_p * len(ts))(*[v[0].encode() for v in variables])
    ptrs = (C.c_void_p * len(ts))(*[t.data_ptr() for t in ts])
    dts = np.array([TYPE_CODES[type_of_tensor(t)] for t in ts], np.int32)
    nds = np.array([float(v[2]) for v in variables], np.float64)
    check(lib().gskyhip_band_math(expr.encode(), names, ptrs, dts.ctypes.data_as(C.c_void_p),
                                  nds.ctypes.data_as(C.c_void_p), len(ts), int(out.numel()), float(out_nodata),
                                  C.c_void_p(out.data_ptr()), _stream()), "bandExpr %r" % expr)
    return out
