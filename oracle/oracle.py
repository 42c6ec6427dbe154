"""ctypes binding of the CPU oracle (oracle/gsky_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py as the checker.  The product (gsky_amd/) never
imports this module.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liboracle.so")

BYTE, UINT16, INT16, UINT32, INT32, FLOAT32, FLOAT64, SIGNEDBYTE = 1, 2, 3, 4, 5, 6, 7, 100
NP_OF = {BYTE: np.uint8, UINT16: np.uint16, INT16: np.int16, UINT32: np.uint32,
         INT32: np.int32, FLOAT32: np.float32, FLOAT64: np.float64, SIGNEDBYTE: np.int8}
CODE_OF = {np.dtype(v): k for k, v in NP_OF.items() if k != SIGNEDBYTE}
CODE_OF[np.dtype(np.int8)] = SIGNEDBYTE
MAX_OVR = 12


def build(force: bool = False) -> str:
    src = os.path.join(_HERE, "gsky_oracle.c")
    if force or not os.path.exists(_LIB_PATH) or os.path.getmtime(_LIB_PATH) < os.path.getmtime(src):
        subprocess.check_call(["make", "-s", "-C", _HERE])
    return _LIB_PATH


class Crs(C.Structure):
    _fields_ = [("kind", C.c_int32), ("_pad", C.c_int32)] + [
        (n, C.c_double) for n in ("a", "ra", "es", "e", "one_es", "lam0", "phi0", "phi1",
                                  "phi2", "x0", "y0", "k0", "n", "c", "dd", "rho0", "ec",
                                  "tm_qn", "tm_zb")] + [
        (n, C.c_double * 6) for n in ("tm_cgb", "tm_cbg", "tm_utg", "tm_gtu")]


class Granule(C.Structure):
    _fields_ = [("data", C.c_void_p), ("dtype", C.c_int32), ("xsize", C.c_int32),
                ("ysize", C.c_int32), ("signed_byte", C.c_int32), ("geot", C.c_double * 6),
                ("nodata", C.c_double), ("n_ovr", C.c_int32), ("_pad", C.c_int32),
                ("ovr_data", C.c_void_p * MAX_OVR), ("ovr_xsize", C.c_int32 * MAX_OVR),
                ("ovr_ysize", C.c_int32 * MAX_OVR), ("block_x", C.c_int32), ("block_y", C.c_int32)]


class GeoLoc(C.Structure):
    _fields_ = [("gx", C.c_void_p), ("gy", C.c_void_p), ("nx", C.c_int), ("ny", C.c_int),
                ("has_nodata", C.c_int), ("nodata_x", C.c_double), ("pixel_offset", C.c_double),
                ("line_offset", C.c_double), ("pixel_step", C.c_double), ("line_step", C.c_double),
                ("bmx", C.c_void_p), ("bmy", C.c_void_p), ("bw", C.c_int), ("bh", C.c_int),
                ("bgt", C.c_double * 6)]


class FlexRaster(C.Structure):
    _fields_ = [("data", C.c_void_p), ("data_w", C.c_int32), ("data_h", C.c_int32),
                ("width", C.c_int32), ("height", C.c_int32), ("off_x", C.c_int32),
                ("off_y", C.c_int32), ("dtype", C.c_int32), ("ns", C.c_int32),
                ("nodata", C.c_double), ("timestamp", C.c_double),
                ("polygon_hash", C.c_uint32), ("_pad", C.c_int32)]


class Canvas(C.Structure):
    _fields_ = [("data", C.c_void_p), ("created", C.c_int32), ("dtype", C.c_int32),
                ("nodata", C.c_double), ("timestamp", C.c_double)]


class Tile(C.Structure):
    _fields_ = [("dst_geot", C.c_double * 6), ("width", C.c_int32), ("height", C.c_int32),
                ("pair_begin", C.c_int32), ("pair_end", C.c_int32)]


class ScaleParams(C.Structure):
    _fields_ = [("offset", C.c_double), ("scale", C.c_double), ("clip", C.c_double),
                ("colour_scale", C.c_int32), ("_pad", C.c_int32)]


_lib = None


def lib():
    global _lib
    if _lib is None:
        _lib = C.CDLL(build())
        L = _lib
        vp, i32, i64, d = C.c_void_p, C.c_int32, C.c_int64, C.c_double
        L.oracle_scale.argtypes = [vp, C.c_int, i64, d, d, d, d, C.c_int, vp]
        L.oracle_scale_legacy.argtypes = [vp, C.c_int, i64, d, d, d, d, vp]
        L.oracle_gradient_palette.argtypes = [vp, C.c_int, C.c_int, vp]
        L.oracle_encode_rgba.argtypes = [vp, C.c_int, C.c_int, C.c_int, vp, vp]
        L.oracle_fnv32a.argtypes = [C.c_char_p, C.c_size_t]
        L.oracle_fnv32a.restype = C.c_uint32
        L.oracle_compute_mask.argtypes = [vp, C.c_int, i64, C.c_char_p, vp, C.c_int, vp]
        L.oracle_merge_batch.argtypes = [vp, C.c_int, C.c_int, C.c_char_p, vp, C.c_int,
                                         C.c_int, vp, C.c_int]
        L.oracle_crs_init.argtypes = [vp, C.c_char_p]
        L.oracle_crs_transform.argtypes = [vp, vp, C.POINTER(d), C.POINTER(d)]
        L.oracle_warp.argtypes = [vp, vp, vp, vp, C.c_int, C.c_int, C.c_int, vp,
                                  C.POINTER(C.c_int), vp, C.POINTER(d), C.POINTER(C.c_int),
                                  C.POINTER(C.c_int)]
        L.oracle_warp_geoloc.argtypes = [vp, vp, vp, vp, C.c_int, C.c_int, C.c_int, vp, vp,
                                         C.POINTER(C.c_int), vp, C.POINTER(d), C.POINTER(C.c_int),
                                         C.POINTER(C.c_int)]
        L.oracle_geoloc_init.argtypes = [vp, vp, C.c_int, C.c_int, vp, C.c_int, C.c_int, C.c_int, d, d, d, d, d]
        L.oracle_geoloc_free.argtypes = [vp]
        L.oracle_suggested_warp_output.argtypes = [vp, vp, vp, vp, vp, vp, C.POINTER(C.c_int),
                                                   C.POINTER(C.c_int), vp]
        L.oracle_approx_row.argtypes = [vp, vp, vp, vp, C.c_int, vp, vp, vp]
        L.oracle_render_tiles.argtypes = [vp, vp, vp, vp, vp, C.c_int, vp, vp, C.c_int, vp,
                                          C.c_int, C.c_int, C.c_char_p, C.c_int, C.c_int, vp,
                                          vp, vp, C.c_int]
        L.oracle_render_tiles2.argtypes = [vp, vp, vp, vp, vp, C.c_int, vp, vp, C.c_int, vp,
                                           C.c_int, C.c_int, C.c_char_p, C.c_int, C.c_int, vp,
                                           vp, vp, C.c_int, C.c_int, vp, vp, C.c_int]
        L.oracle_drill_read_data.argtypes = [vp, C.c_int, C.c_int, C.c_int, vp, C.c_float,
                                             C.c_float, C.c_float, C.c_int, C.c_int, vp, vp]
        L.oracle_drill_merge.argtypes = [vp, vp, C.c_int, C.c_int, vp]
        L.oracle_drill_descriptor.argtypes = [C.c_char_p, vp, vp, C.c_int, C.c_int, vp, C.POINTER(C.c_void_p)]
        L.or_go_f64_u8.argtypes = [d]
        L.or_go_f64_u8.restype = C.c_uint8
        L.or_go_f64_i16.argtypes = [d]
        L.or_go_f64_i16.restype = C.c_int16
    return _lib


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(C.c_void_p)


def dtype_code(a: np.ndarray, signed_byte: bool = False) -> int:
    if a.dtype == np.int8 or signed_byte:
        return SIGNEDBYTE
    return CODE_OF[a.dtype]


# ---------------------------------------------------------------- scale / palette
def scale(data: np.ndarray, nodata: float, offset: float, scale_: float, clip: float,
          colour_scale: int = 0) -> np.ndarray:
    """utils.scale (raster_scaler.go:30-332).  Byte input is scaled in place
    by the reference; here a copy is scaled so the caller's array is kept."""
    d = np.ascontiguousarray(data).copy()
    out = np.zeros(d.size, np.uint8)
    rc = lib().oracle_scale(_ptr(d), dtype_code(d), d.size, nodata, offset, scale_, clip,
                            colour_scale, _ptr(out))
    if rc:
        raise ValueError("Raster type not implemented")
    return out.reshape(data.shape)


def scale_legacy(data, nodata, offset, scale_, clip):
    d = np.ascontiguousarray(data).copy()
    out = np.zeros(d.size, np.uint8)
    if lib().oracle_scale_legacy(_ptr(d), dtype_code(d), d.size, nodata, offset, scale_, clip, _ptr(out)):
        raise ValueError("Raster type not implemented")
    return out.reshape(data.shape)


def gradient_palette(colours, interpolate: bool) -> np.ndarray:
    c = np.ascontiguousarray(np.asarray(colours, np.uint8).reshape(-1, 4))
    ramp = np.zeros((256, 4), np.uint8)
    if lib().oracle_gradient_palette(_ptr(c), len(c), int(bool(interpolate)), _ptr(ramp)):
        raise ValueError("bad palette")
    return ramp


def encode_rgba(bands, w, h, ramp=None) -> np.ndarray:
    bs = [np.ascontiguousarray(b, np.uint8).reshape(-1) for b in bands]
    arr = (C.c_void_p * len(bs))(*[b.ctypes.data for b in bs])
    out = np.zeros((h, w, 4), np.uint8)
    rp = _ptr(np.ascontiguousarray(ramp, np.uint8)) if ramp is not None else None
    if lib().oracle_encode_rgba(arr, len(bs), w, h, rp, _ptr(out)):
        raise ValueError("Cannot encode other than 1 or 3 namespaces")
    return out


def fnv32a(s: str) -> int:
    b = s.encode()
    return lib().oracle_fnv32a(b, len(b))


def compute_mask(data: np.ndarray, value=None, bit_tests=(), signed_byte=False) -> np.ndarray:
    d = np.ascontiguousarray(data)
    out = np.zeros(d.size, np.uint8)
    bt = [s.encode() for s in bit_tests]
    arr = (C.c_char_p * max(1, len(bt)))(*bt) if bt else None
    rc = lib().oracle_compute_mask(_ptr(d), dtype_code(d, signed_byte), d.size,
                                   value.encode() if value else None,
                                   C.cast(arr, C.c_void_p) if arr else None, len(bt), _ptr(out))
    if rc:
        raise ValueError("ComputeMask error %d" % rc)
    return out.reshape(data.shape).astype(bool)


def merge_batch(rasters, n_ns, width, height, mask_ns=-1, mask_value=None, bit_tests=(),
                mask_inclusive=False):
    """RasterMerger.Run over one batch.  rasters: list of dicts with keys
    data (2-D window array), off_x, off_y, nodata, timestamp, polygon_hash, ns
    and optional signed_byte.  Returns list of (canvas array or None, nodata)."""
    keep = []
    fr = (FlexRaster * max(1, len(rasters)))()
    for i, r in enumerate(rasters):
        d = np.ascontiguousarray(r["data"])
        keep.append(d)
        fr[i].data = d.ctypes.data
        fr[i].data_h, fr[i].data_w = d.shape
        fr[i].width, fr[i].height = width, height
        fr[i].off_x, fr[i].off_y = r["off_x"], r["off_y"]
        fr[i].dtype = dtype_code(d, r.get("signed_byte", False))
        fr[i].ns = r["ns"]
        fr[i].nodata = r["nodata"]
        fr[i].timestamp = r["timestamp"]
        fr[i].polygon_hash = r["polygon_hash"]
    bufs = [np.zeros(width * height * 8, np.uint8) for _ in range(n_ns)]
    cv = (Canvas * n_ns)()
    for k in range(n_ns):
        cv[k].data = bufs[k].ctypes.data
    bt = [s.encode() for s in bit_tests]
    arr = (C.c_char_p * max(1, len(bt)))(*bt) if bt else None
    rc = lib().oracle_merge_batch(fr, len(rasters), mask_ns,
                                  mask_value.encode() if mask_value else None,
                                  C.cast(arr, C.c_void_p) if arr else None, len(bt),
                                  int(mask_inclusive), cv, n_ns)
    if rc:
        raise ValueError("merge error %d" % rc)
    out = []
    for k in range(n_ns):
        if not cv[k].created:
            out.append((None, None))
            continue
        dt = NP_OF[cv[k].dtype]
        a = bufs[k].view(dt)[: width * height].reshape(height, width).copy()
        out.append((a, cv[k].nodata))
    return out


# ---------------------------------------------------------------- projections / warp
def crs(spec: str) -> Crs:
    c = Crs()
    if lib().oracle_crs_init(C.byref(c), spec.encode()):
        raise ValueError("unsupported CRS %r" % spec)
    return c


def crs_transform(src: Crs, dst: Crs, x: float, y: float):
    xx, yy = C.c_double(x), C.c_double(y)
    ok = lib().oracle_crs_transform(C.byref(src), C.byref(dst), C.byref(xx), C.byref(yy))
    return (xx.value, yy.value) if ok else None


def make_granule(data: np.ndarray, geot, nodata=-1e10, overviews=(), signed_byte=False, block=(0, 0)):
    g = Granule()
    g.block_x, g.block_y = block
    d = np.ascontiguousarray(data)
    g.data = d.ctypes.data
    g.dtype = dtype_code(d, signed_byte)
    if d.dtype == np.int8:
        g.dtype = BYTE
        signed_byte = True
    g.signed_byte = int(signed_byte)
    g.ysize, g.xsize = d.shape
    for i in range(6):
        g.geot[i] = geot[i]
    g.nodata = nodata
    keep = [d]
    g.n_ovr = len(overviews)
    for i, o in enumerate(overviews):
        o = np.ascontiguousarray(o, d.dtype)
        keep.append(o)
        g.ovr_data[i] = o.ctypes.data
        g.ovr_ysize[i], g.ovr_xsize[i] = o.shape
    g._keep = keep
    return g


def warp(g: Granule, src: Crs, dst, dst_geot, w, h, resample=0):
    """warp_operation_fast restated; returns (window array, bbox, nodata, dtype)."""
    buf = C.c_void_p()
    size = C.c_int()
    bbox = np.zeros(4, np.int32)
    nd = C.c_double()
    dt = C.c_int()
    br = C.c_int()
    gt = np.ascontiguousarray(dst_geot, np.float64)
    rc = lib().oracle_warp(C.byref(g), C.byref(src), C.byref(dst) if dst is not None else None,
                           _ptr(gt), w, h, resample, C.byref(buf), C.byref(size), _ptr(bbox),
                           C.byref(nd), C.byref(dt), C.byref(br))
    if rc:
        raise RuntimeError("warp_operation() fail: %d" % rc)
    npdt = NP_OF[dt.value]
    arr = np.frombuffer(C.string_at(buf, size.value), dtype=npdt).copy()
    C.CDLL(None).free(buf)
    arr = arr.reshape(int(bbox[3]), int(bbox[2]))
    warp.bytes_read = br.value        # warp.go:347 of the last call
    return arr, bbox.copy(), nd.value, dt.value


def geoloc(x_band: np.ndarray, y_band: np.ndarray, nodata_x=None, pixel_offset=0.0, line_offset=0.0,
           pixel_step=1.0, line_step=1.0) -> GeoLoc:
    """GDALCreateGeoLocTransformer restated (oracle_geoloc_init): the X / Y
    bands (2-D, or both one row: a regular grid) and the GeoLocOpts numbers
    (tile_grpc.go:338-350).  Freed with the returned object."""
    gl = GeoLoc()
    xb = np.ascontiguousarray(x_band, np.float64)
    yb = np.ascontiguousarray(y_band, np.float64)
    xb2, yb2 = xb.reshape(-1, xb.shape[-1]), yb.reshape(-1, yb.shape[-1])
    rc = lib().oracle_geoloc_init(C.byref(gl), _ptr(xb2), xb2.shape[1], xb2.shape[0], _ptr(yb2), yb2.shape[1],
                                  yb2.shape[0], int(nodata_x is not None),
                                  float(nodata_x if nodata_x is not None else 0.0), pixel_offset, line_offset,
                                  pixel_step, line_step)
    if rc:
        raise RuntimeError("GDALCreateGeoLocTransformer failed")
    gl._lib = lib()
    return gl


def free_geoloc(gl: GeoLoc) -> None:
    lib().oracle_geoloc_free(C.byref(gl))


def warp_geoloc(g: Granule, src: Crs, dst, dst_geot, w, h, gl: GeoLoc, resample=0):
    """warp_operation_fast with GeoLocOpts (warp.go:128-141, 158)."""
    buf = C.c_void_p()
    size = C.c_int()
    bbox = np.zeros(4, np.int32)
    nd = C.c_double()
    dt = C.c_int()
    br = C.c_int()
    gt = np.ascontiguousarray(dst_geot, np.float64)
    rc = lib().oracle_warp_geoloc(C.byref(g), C.byref(src), C.byref(dst) if dst is not None else None,
                                  _ptr(gt), w, h, resample, C.byref(gl), C.byref(buf), C.byref(size), _ptr(bbox),
                                  C.byref(nd), C.byref(dt), C.byref(br))
    if rc:
        raise RuntimeError("warp_operation() fail: %d" % rc)
    arr = np.frombuffer(C.string_at(buf, size.value), dtype=NP_OF[dt.value]).copy()
    C.CDLL(None).free(buf)
    warp_geoloc.bytes_read = br.value
    return arr.reshape(int(bbox[3]), int(bbox[2])), bbox.copy(), nd.value, dt.value


def suggested_warp_output(g: Granule, src: Crs, dst: Crs, dst_geot):
    gt = np.ascontiguousarray(dst_geot, np.float64)
    out = np.zeros(6)
    ext = np.zeros(4)
    np_, nl = C.c_int(), C.c_int()
    rc = lib().oracle_suggested_warp_output(C.byref(g), C.byref(src), C.byref(dst), None,
                                            _ptr(gt), _ptr(out), C.byref(np_), C.byref(nl),
                                            _ptr(ext))
    return rc, out, np_.value, nl.value, ext


def compute_reproject_extent(g: Granule, src: Crs, dst: Crs, dst_bbox):
    """ComputeReprojectExtent (worker/gdalprocess/warp.go:433-487): the
    GenImgProj transformer of the dataset to dst (no destination dataset, so
    destination coordinates are georeferenced: identity geotransform),
    GDALSuggestedWarpOutput (= SuggestedWarpOutput2, nOptions 0), then
    nPixels = int((xMax - xMin + xRes/2) / xRes), nLines likewise, with
    (xMin, yMin, xMax, yMax) = dst_bbox (the request's DstGeot[0..3]).
    Returns (nPixels, nLines), or None where the reference answers
    "GDALSuggestedWarpOutput() failed"."""
    rc, gt, _, _, _ = suggested_warp_output(g, src, dst, [0.0, 1.0, 0.0, 0.0, 0.0, 1.0])
    if rc != 0:
        return None
    x_res, y_res = float(gt[1]), abs(float(gt[5]))
    x_min, y_min, x_max, y_max = (float(v) for v in dst_bbox[:4])
    return int((x_max - x_min + x_res / 2.0) / x_res), int((y_max - y_min + y_res / 2.0) / y_res)


def render_tiles(granules, src_crs, ts, ph, ns, dst, tiles_geot, width, height, pairs,
                 scale_params, ramp=None, n_ns=1, mask_ns=-1, mask_value=None,
                 mask_inclusive=False, resample=0, n_threads=1, sizes=None, canvas=False):
    """CPU baseline of the whole tile path.  pairs: list (per tile) of granule
    index lists; sizes: optional per-tile (w, h) (default width x height).
    Returns (n_tiles, max_h, max_w, 4) uint8 RGBA (tile t in [t, :h, :w]);
    with canvas=True also the typed merged canvases (n_tiles, n_out,
    max_h*max_w*4 bytes, row stride max_w) and their created flags (n_tiles, 3)."""
    ng = len(granules)
    garr = (Granule * ng)(*granules)
    carr = (Crs * ng)(*src_crs)
    ts = np.ascontiguousarray(ts, np.float64)
    ph = np.ascontiguousarray(ph, np.uint32)
    nsa = np.ascontiguousarray(ns, np.int32)
    nt = len(tiles_geot)
    sizes = list(sizes) if sizes is not None else [(width, height)] * nt
    max_w = max([w for w, _ in sizes] + [1])
    max_h = max([h for _, h in sizes] + [1])
    tarr = (Tile * max(1, nt))()
    flat = []
    for i in range(nt):
        for k in range(6):
            tarr[i].dst_geot[k] = tiles_geot[i][k]
        tarr[i].width, tarr[i].height = sizes[i]
        tarr[i].pair_begin = len(flat)
        flat.extend(pairs[i])
        tarr[i].pair_end = len(flat)
    pg = np.ascontiguousarray(flat if flat else [0], np.int32)
    sp = ScaleParams(*scale_params[:3], int(scale_params[3]) if len(scale_params) > 3 else 0, 0)
    out = np.zeros((nt, max_h, max_w, 4), np.uint8)
    n_out = n_ns - (1 if mask_ns >= 0 else 0)
    cv = np.zeros((nt, n_out, max_h * max_w * 4), np.uint8) if canvas else None
    created = np.zeros((nt, 3), np.int32) if canvas else None
    rp = _ptr(np.ascontiguousarray(ramp, np.uint8)) if ramp is not None else None
    rc = lib().oracle_render_tiles2(garr, carr, _ptr(ts), _ptr(ph), _ptr(nsa), ng, C.byref(dst),
                                    tarr, nt, _ptr(pg), resample, mask_ns,
                                    mask_value.encode() if mask_value else None,
                                    int(mask_inclusive), n_ns, C.byref(sp), rp, _ptr(out), max_w, max_h,
                                    _ptr(cv) if canvas else None, _ptr(created) if canvas else None,
                                    n_threads)
    if rc:
        raise RuntimeError("render error %d" % rc)
    return (out, cv, created) if canvas else out


def drill_read_data(data, mask, nodata, clip_lower, clip_upper, pixel_count=0, band_strides=1):
    d = np.ascontiguousarray(data, np.float32)
    nb, cy, cx = d.shape
    m = np.ascontiguousarray(mask, np.uint8)
    cap = nb * max(1, band_strides) + 4
    v = np.zeros(cap)
    c = np.zeros(cap, np.int32)
    n = lib().oracle_drill_read_data(_ptr(d), nb, cx, cy, _ptr(m), nodata, clip_lower,
                                     clip_upper, pixel_count, band_strides, _ptr(v), _ptr(c))
    return v[:n].copy(), c[:n].copy()


def compute_deciles(values, mask, nodata, decile_count):
    """computeDeciles (worker/gdalprocess/drill.go:229-273) of one band, a
    pure-Python restatement (small cases): the in-mask (255), non-nodata
    values (no clipping) in row-major order, sorted ascending; step =
    len // (dc + 1); step > 0: buf[(i+1)*step], or the float32 mean with the
    next value when len % (dc + 1) == 0; otherwise each value repeated by its
    padding count.  Returns float32 (dc,), or None where the reference
    indexes past the slice (Go panics)."""
    v = np.asarray(values, np.float32).reshape(-1)
    m = np.asarray(mask, np.uint8).reshape(-1)
    nd = np.float32(nodata)
    buf = sorted(float(x) for x, k in zip(v, m) if k == 255 and np.float32(x) != nd)
    buf = [np.float32(x) for x in buf]
    dc = int(decile_count)
    out = np.zeros(dc, np.float32)
    step = len(buf) // (dc + 1)
    if step > 0:
        even = len(buf) % (dc + 1) == 0
        for i in range(dc):
            j = (i + 1) * step
            de = buf[j]
            if even:
                if j + 1 >= len(buf):
                    return None
                de = np.float32((buf[j] + buf[j + 1]) / np.float32(2.0))
            out[i] = de
    else:
        pad = {}
        for i in range(dc):
            k = i % len(buf)
            pad[k] = pad.get(k, 0) + 1
        idx = 0
        for i in range(len(buf)):
            for _ in range(pad.get(i, 0)):
                out[idx] = buf[i]
                idx += 1
    return out


def _go_round(x: float) -> float:   # math.Round: half away from zero
    import math
    return math.copysign(math.floor(abs(x) + 0.5), x)


def drill_read_data_full(data, mask, nodata, clip_lower, clip_upper, pixel_count=0, band_strides=1,
                         decile_count=0, bands=None):
    """readData (worker/gdalprocess/drill.go:90-227) with deciles and
    bandStrides, a pure-Python restatement over one polygon window: data
    (n_bands, h, w) float32, bands 1-based (default all).  Per group
    [ibBgn, ibEnd) the bound bands bands[ibBgn], bands[ibEnd-1] (one band when
    bandStrides is 1, the same band twice for a 1-band group), their mean /
    count (drill_read_data) and deciles (compute_deciles; zeros with Count 0
    where the total is 0), appended as rows [mean, d1..dk]; for bandStrides > 2
    bandStrides - 2 rows interpolated in every column in between, Count
    math.Round((c0 + c1) / 2).  Returns (values (rows, nCols) float64,
    counts int32), or None where computeDeciles panics."""
    d = np.asarray(data, np.float32)
    blist = list(bands) if bands is not None else list(range(1, d.shape[0] + 1))
    strides = band_strides if band_strides > 0 else 1
    nc = 1 + int(decile_count)
    vals, cnts = [], []
    for ib in range(0, len(blist), strides):
        ie = min(ib + strides, len(blist))
        read = [blist[ib], blist[ie - 1]] if strides > 1 else [blist[ib]]
        bound = []
        for b in read:
            mv, mc = drill_read_data(d[b - 1:b], mask, nodata, clip_lower, clip_upper, pixel_count, 1)
            row_v, row_c = [float(mv[0])], [int(mc[0])]
            if decile_count > 0:
                if mc[0] > 0:
                    dec = compute_deciles(d[b - 1], mask, nodata, decile_count)
                    if dec is None:
                        return None
                    row_v += [float(x) for x in dec]
                    row_c += [1] * decile_count
                else:
                    row_v += [0.0] * decile_count
                    row_c += [0] * decile_count
            bound.append((row_v, row_c))
        vals.append(bound[0][0])
        cnts.append(bound[0][1])
        if strides > 2 and len(bound) > 1:
            beta = [(bound[1][0][ic] - bound[0][0][ic]) / float(strides - 1) for ic in range(nc)]
            count = [_go_round(float(bound[0][1][ic] + bound[1][1][ic]) / 2.0) for ic in range(nc)]
            for ip in range(1, strides - 1):
                vals.append([bound[0][0][ic] + float(ip) * beta[ic] for ic in range(nc)])
                cnts.append([int(count[ic]) for ic in range(nc)])
        if len(bound) > 1:
            vals.append(bound[1][0])
            cnts.append(bound[1][1])
    return np.array(vals, np.float64).reshape(-1, nc), np.array(cnts, np.int32).reshape(-1, nc)


def go_png_rows(rgba):
    """What Go 1.12 image/png's writeImage hands zlib for EncodePNG's
    *image.RGBA canvas (utils/ogc_encoders.go:82-139), a numpy restatement:
    (opaque, bytes).  opaque: every alpha 0xff (image.RGBA.Opaque) -> RGB rows,
    else NRGBA rows (color.NRGBAModel of each premultiplied pixel, 16-bit
    arithmetic, uint8() wrap).  Each row = [filter type][residuals] with the
    filter of writer.go filter(): sums of |int8| residuals of Up, Paeth, None,
    Sub, Average in that order, the first strictly smaller wins."""
    px = np.asarray(rgba, np.uint8)
    h, w, _ = px.shape
    opaque = bool((px[..., 3] == 0xFF).all())
    if opaque:
        img = px[..., :3].astype(np.int64)
    else:
        a = px[..., 3].astype(np.int64)
        a16 = a | (a << 8)
        img = np.zeros((h, w, 4), np.int64)
        for c in range(3):
            v16 = px[..., c].astype(np.int64)
            v16 = v16 | (v16 << 8)
            conv = ((v16 * 0xFFFF) // np.maximum(a16, 1)) >> 8
            img[..., c] = np.where(a == 0xFF, px[..., c], np.where(a == 0, 0, conv & 0xFF))
        img[..., 3] = a
    bpp = 3 if opaque else 4
    rows = img.reshape(h, w * bpp)
    out = bytearray()
    prev = np.zeros(w * bpp, np.int64)

    def abs8(d):
        d = d & 0xFF
        return np.where(d < 128, d, 256 - d).sum()

    def paeth(a, b, c):
        pa = b - c
        pb = a - c
        pc = np.abs(pa + pb)
        pa, pb = np.abs(pa), np.abs(pb)
        return np.where((pa <= pb) & (pa <= pc), a, np.where(pb <= pc, b, c))

    for y in range(h):
        cur = rows[y]
        left = np.concatenate([np.zeros(bpp, np.int64), cur[:-bpp]])
        ul = np.concatenate([np.zeros(bpp, np.int64), prev[:-bpp]])
        cand = {2: cur - prev,
                4: np.concatenate([cur[:bpp] - prev[:bpp], cur[bpp:] - paeth(left, prev, ul)[bpp:]]),
                0: cur,
                1: cur - left,
                3: np.concatenate([cur[:bpp] - prev[:bpp] // 2, cur[bpp:] - (left[bpp:] + prev[bpp:]) // 2])}
        best, ft = None, 2
        for f in (2, 4, 0, 1, 3):
            sm = abs8(cand[f])
            if best is None or sm < best:
                best, ft = sm, f
        out.append(ft)
        out += (cand[ft] & 0xFF).astype(np.uint8).tobytes()
        prev = cur
    return opaque, bytes(out)


def band_math(expr, variables, out_nodata):
    """Band-math of RasterMerger.Run (processor/tile_merger.go:654-731) for
    one expression over one axis, a pure-Python restatement: variables =
    [(name, array, nodata)] converted to float32; the grammar of
    gskyhip_band_math (a govaluate subset) evaluated with numpy float32
    element-wise arithmetic and constants rounded to float32; pixels where
    any variable is its nodata, and non-finite results, -> out_nodata; a
    constant expression fills every valid pixel.  (The govaluate fork is
    absent from /root/reference: parity with it is unpinned.)"""
    import re
    toks = re.findall(r"\d+\.\d*(?:[eE][-+]?\d+)?|\.\d+(?:[eE][-+]?\d+)?|\d+(?:[eE][-+]?\d+)?|"
                      r"[A-Za-z_][A-Za-z0-9_.]*|\*\*|&&|\|\||==|!=|<=|>=|[-+*/%<>!?:()]", expr)
    if "".join(toks) != re.sub(r"\s+", "", expr):
        raise ValueError("bad token in %r" % expr)
    env = {n: np.asarray(a).astype(np.float32) for n, a, _ in variables}
    f32 = np.float32
    pos = [0]
    used = [False]

    def peek():
        return toks[pos[0]] if pos[0] < len(toks) else None

    def take(t=None):
        tok = peek()
        if t is not None and tok != t:
            raise ValueError("expected %r in %r" % (t, expr))
        pos[0] += 1
        return tok

    def b(x):
        return np.where(x, f32(1), f32(0))

    def ternary():
        c = logic_or()
        if peek() == "?":
            take("?")
            a = ternary()
            take(":")
            bb = ternary()
            return np.where(c != 0, a, bb).astype(f32)
        return c

    def logic_or():
        v = logic_and()
        while peek() == "||":
            take()
            w = logic_and()
            v = b((v != 0) | (w != 0))
        return v

    def logic_and():
        v = equality()
        while peek() == "&&":
            take()
            w = equality()
            v = b((v != 0) & (w != 0))
        return v

    def equality():
        v = relation()
        while peek() in ("==", "!="):
            op = take()
            w = relation()
            v = b(v == w) if op == "==" else b(v != w)
        return v

    def relation():
        v = additive()
        while peek() in ("<", "<=", ">", ">="):
            op = take()
            w = additive()
            v = b({"<": v < w, "<=": v <= w, ">": v > w, ">=": v >= w}[op])
        return v

    def additive():
        v = multiplicative()
        while peek() in ("+", "-"):
            op = take()
            w = multiplicative()
            v = (v + w) if op == "+" else (v - w)
        return v

    def multiplicative():
        v = power()
        while peek() in ("*", "/", "%"):
            op = take()
            w = power()
            with np.errstate(all="ignore"):
                v = v * w if op == "*" else (v / w if op == "/" else np.fmod(v, w))
        return v

    def power():
        v = unary()
        if peek() == "**":
            take()
            w = power()
            with np.errstate(all="ignore"):
                v = np.power(v, w)
        return v

    def unary():
        if peek() == "-":
            take()
            return -unary()
        if peek() == "+":
            take()
            return unary()
        if peek() == "!":
            take()
            return b(unary() == 0)
        return primary()

    def primary():
        tok = take()
        if tok == "(":
            v = ternary()
            take(")")
            return v
        if tok is not None and (tok[0].isdigit() or tok[0] == "."):
            return f32(float(tok))
        if tok in env:
            used[0] = True
            return env[tok]
        raise ValueError("No parameter %r found." % tok)

    with np.errstate(all="ignore"):
        res = ternary()
    if pos[0] != len(toks):
        raise ValueError("trailing tokens in %r" % expr)
    shape = np.asarray(variables[0][1]).shape
    valid = np.ones(shape, bool)
    for n, a, nd in variables:
        valid &= np.asarray(a).astype(np.float32).astype(np.float64) != float(nd)
    res = np.broadcast_to(np.asarray(res, np.float32), shape)
    if used[0]:
        res = np.where(np.isfinite(res), res, f32(out_nodata))
    return np.where(valid, res, f32(out_nodata)).astype(np.float32)


def drill_merge(values, counts):
    v = np.ascontiguousarray(values, np.float64)
    c = np.ascontiguousarray(counts, np.int32)
    nf, nd = v.shape
    out = np.zeros(nd)
    lib().oracle_drill_merge(_ptr(v), _ptr(c), nf, nd, _ptr(out))
    return out


def drill_descriptor(geometry_json: str, ds_srs, geot, xsize: int, ysize: int):
    """getDrillFileDescriptor + createMask restated: ((offX, offY, countX,
    countY), mask uint8 (countY, countX), 255 inside) or raises ValueError."""
    c = crs(ds_srs) if ds_srs else None
    gt = np.ascontiguousarray(geot, np.float64)
    win = np.zeros(4, np.int32)
    mp = C.c_void_p()
    rc = lib().oracle_drill_descriptor(geometry_json.encode(), C.byref(c) if c is not None else None, _ptr(gt),
                                       xsize, ysize, _ptr(win), C.byref(mp))
    if rc:
        raise ValueError("drill descriptor error %d" % rc)
    n = int(win[2]) * int(win[3])
    m = np.frombuffer(C.string_at(mp, n), np.uint8).reshape(int(win[3]), int(win[2])).copy()
    C.CDLL(None).free(mp)
    return tuple(int(v) for v in win), m
