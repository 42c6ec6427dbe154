"""ctypes binding of libgskyhip.so (include/gskyhip.h).

The shared library is the product: hand-written HIP kernels for gfx950 plus a
C-ABI.  This module only loads it and mirrors its structs; there is no CPU
fallback.  A missing library raises immediately.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# GSKYHIP_LIB=ab selects the A/B build (make -C gsky_amd/csrc ab: the same
# kernels plus the experiment knobs it reads from the environment); tools and
# A/B scripts only -- the product library reads no knob.
# GSKYHIP_LIB=<name> (other than "ab") loads libgskyhip_<name>.so: a kept
# earlier build, for A/B timing against the current one.
_SEL = os.environ.get("GSKYHIP_LIB", "")
LIB_PATH = os.path.join(_HERE, "libgskyhip_%s.so" % _SEL if _SEL and _SEL != "default" else "libgskyhip.so")

# GDALDataType codes (warp.go:428-431) + 100 = SignedByte (warp.go:354-359)
BYTE, UINT16, INT16, UINT32, INT32, FLOAT32, FLOAT64, SIGNEDBYTE = 1, 2, 3, 4, 5, 6, 7, 100
CRS_LONGLAT, CRS_WEBMERC, CRS_AEA, CRS_SINU = 0, 1, 2, 3
RESAMPLE_NEAREST, RESAMPLE_BILINEAR = 0, 1
# value-type hint bits of gskyhip_render_tiles_typed
VT_BIT = {BYTE: 1, SIGNEDBYTE: 2, INT16: 4, UINT16: 8, FLOAT32: 16}
MAX_OVR = 12
MAX_BIT_TESTS = 8

ERRORS = {0: "OK", -1: "bad argument", -2: "raster type not implemented", -3: "HIP runtime error",
          -4: "unsupported CRS", -5: "bad mask", -6: "no HIP device", -7: "index out of range",
          -8: "GDALSuggestedWarpOutput() failed", -9: "warp service unreachable",
          1: "open failed", 2: "band failed", 3: "transformer failed"}


class GskyError(RuntimeError):
    def __init__(self, code: int, what: str = ""):
        self.code = code
        super().__init__("%s: %s (%d)" % (what or "gskyhip", ERRORS.get(code, "error"), code))


class Crs(C.Structure):
    _fields_ = [("kind", C.c_int32), ("_pad", C.c_int32)] + [
        (n, C.c_double) for n in ("a", "ra", "es", "e", "one_es", "lam0", "phi0", "phi1", "phi2",
                                  "x0", "y0", "k0", "n", "c", "dd", "rho0", "ec", "tm_qn", "tm_zb")] + [
        (n, C.c_double * 6) for n in ("tm_cgb", "tm_cbg", "tm_utg", "tm_gtu")]


class Granule(C.Structure):
    _fields_ = [("data", C.c_void_p), ("dtype", C.c_int32), ("xsize", C.c_int32), ("ysize", C.c_int32),
                ("signed_byte", C.c_int32), ("geot", C.c_double * 6), ("nodata", C.c_double),
                ("has_nodata", C.c_int32), ("crs", C.c_int32), ("n_ovr", C.c_int32), ("ns", C.c_int32),
                ("ovr_data", C.c_void_p * MAX_OVR), ("ovr_xsize", C.c_int32 * MAX_OVR),
                ("ovr_ysize", C.c_int32 * MAX_OVR), ("timestamp", C.c_double),
                ("polygon_hash", C.c_uint32), ("block_x", C.c_int32), ("block_y", C.c_int32),
                ("geoloc", C.c_int32)]


class Tile(C.Structure):
    _fields_ = [("dst_geot", C.c_double * 6), ("width", C.c_int32), ("height", C.c_int32),
                ("pair_begin", C.c_int32), ("pair_end", C.c_int32)]


class ScaleParams(C.Structure):
    _fields_ = [("offset", C.c_double), ("scale", C.c_double), ("clip", C.c_double),
                ("colour_scale", C.c_int32), ("_pad", C.c_int32)]


class Mask(C.Structure):
    _fields_ = [("ns", C.c_int32), ("inclusive", C.c_int32), ("n_bit_tests", C.c_int32),
                ("_pad", C.c_int32), ("value", C.c_char_p), ("bit_tests", C.c_char_p * MAX_BIT_TESTS)]


class RasterInfo(C.Structure):
    _fields_ = [(n, C.c_int32) for n in ("xsize", "ysize", "n_bands", "dtype", "signed_byte", "block_x", "block_y",
                                         "compression", "predictor", "planar", "epsg", "has_nodata", "n_ovr",
                                         "_pad")] + [
        ("geot", C.c_double * 6), ("nodata", C.c_double), ("ovr_xsize", C.c_int32 * MAX_OVR),
        ("ovr_ysize", C.c_int32 * MAX_OVR)]


class FlexRasterC(C.Structure):
    _fields_ = [("data", C.c_void_p), ("data_w", C.c_int32), ("data_h", C.c_int32), ("width", C.c_int32),
                ("height", C.c_int32), ("off_x", C.c_int32), ("off_y", C.c_int32), ("dtype", C.c_int32),
                ("ns", C.c_int32), ("nodata", C.c_double), ("timestamp", C.c_double),
                ("polygon_hash", C.c_uint32), ("_pad", C.c_int32)]


# every symbol include/gskyhip.h declares (checked by tests/test_abi.py)
EXPORTS = [
    "gskyhip_crs_from_srs", "gskyhip_crs_transform", "gskyhip_register_granule", "gskyhip_unregister_all", "warp_operation_fast",
    "gskyhip_render_workspace_size", "gskyhip_render_tiles", "gskyhip_render_tiles_phase",
    "gskyhip_render_tiles_typed", "gskyhip_render_coverage", "gskyhip_warp_windows",
    "gskyhip_merge_rasters", "gskyhip_scale", "gskyhip_scale_legacy", "gskyhip_gradient_palette",
    "gskyhip_encode_rgba", "gskyhip_compute_mask", "gskyhip_drill_rows", "gskyhip_drill",
    "gskyhip_drill_workspace_size", "gskyhip_drill_batch", "gskyhip_drill_descriptors",
    "gskyhip_drill_merge", "gskyhip_fnv32a", "gskyhip_version", "gskyhip_device_count",
    "gskyhip_render_status",
    "gskyhip_render_tile_info", "gskyhip_render_pair_info", "gskyhip_render_touched", "gskyhip_compute_reproject_extent",
    "gskyhip_service_run", "gskyhip_service_register_granule", "gskyhip_service_unregister_all",
    "gskyhip_service_stats", "gskyhip_service_stats_n", "gskyhip_service_shutdown", "gskyhip_drill_deciles_workspace_size",
    "gskyhip_drill_deciles", "gskyhip_band_math", "gskyhip_drill_descriptors_device", "gskyhip_drill_masks_device", "gskyhip_drill_masks_device_packed", "gskyhip_parse_numbers",
    "gskyhip_drill_read_data_workspace_size", "gskyhip_drill_read_data",
    "gskyhip_png_workspace_size", "gskyhip_png_bound", "gskyhip_encode_png",
    "gskyhip_geotiff_workspace_size", "gskyhip_geotiff_bound", "gskyhip_encode_geotiff",
    "gskyhip_netcdf_bound", "gskyhip_encode_netcdf", "gskyhip_encode_netcdf_host",
    "gskyhip_geotiff_info", "gskyhip_geotiff_read_host", "gskyhip_geotiff_read", "gskyhip_register_geotiff",
    "gskyhip_netcdf_info", "gskyhip_netcdf_srs", "gskyhip_netcdf_read_host", "gskyhip_netcdf_read", "gskyhip_register_netcdf",
]

_lib = None


def lib() -> C.CDLL:
    """Load libgskyhip.so (raises if it was not built: no fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError("libgskyhip.so not built: run __graft_entry__.build() (%s)" % LIB_PATH)
    L = C.CDLL(LIB_PATH)
    vp, i32, i64, d = C.c_void_p, C.c_int32, C.c_int64, C.c_double
    ci = C.c_int
    L.gskyhip_crs_from_srs.argtypes = [C.c_char_p, C.POINTER(Crs)]
    L.gskyhip_crs_transform.argtypes = [C.POINTER(Crs), C.POINTER(Crs), C.c_int, C.c_void_p, C.c_void_p,
                                        C.c_void_p]
    L.gskyhip_register_granule.argtypes = [C.c_char_p, ci, C.POINTER(Granule), C.c_char_p]
    L.gskyhip_geotiff_info.argtypes = [C.c_char_p, C.POINTER(RasterInfo)]
    L.gskyhip_geotiff_read_host.argtypes = [C.c_char_p, ci, ci, vp, i64]
    L.gskyhip_geotiff_read.argtypes = [C.c_char_p, ci, ci, vp, i64, vp]
    L.gskyhip_register_geotiff.argtypes = [C.c_char_p, ci]
    L.gskyhip_netcdf_info.argtypes = [C.c_char_p, C.POINTER(RasterInfo)]
    if hasattr(L, "gskyhip_netcdf_srs"):
        L.gskyhip_netcdf_srs.argtypes = [C.c_char_p, ci, C.c_char_p, ci]
    L.gskyhip_netcdf_read_host.argtypes = [C.c_char_p, ci, vp, i64]
    L.gskyhip_netcdf_read.argtypes = [C.c_char_p, ci, vp, i64, vp]
    L.gskyhip_register_netcdf.argtypes = [C.c_char_p, ci]
    L.warp_operation_fast.argtypes = [C.c_char_p, C.c_char_p, C.POINTER(d), vp, C.c_char_p, C.POINTER(d),
                                      ci, ci, ci, ci, C.POINTER(vp), C.POINTER(ci), C.POINTER(ci),
                                      C.POINTER(d), C.POINTER(ci), C.POINTER(ci)]
    L.gskyhip_render_workspace_size.argtypes = [ci, ci, ci]
    L.gskyhip_render_workspace_size.restype = i64
    L.gskyhip_render_tiles.argtypes = [vp, ci, vp, ci, ci, vp, ci, vp, ci, ci, ci, C.POINTER(i32), ci,
                                       C.POINTER(Mask), ci, C.POINTER(ScaleParams), vp, vp, vp, vp, i64, vp]
    L.gskyhip_render_tiles_phase.argtypes = [ci] + L.gskyhip_render_tiles.argtypes
    L.gskyhip_render_tiles_typed.argtypes = [ci, C.c_uint32] + L.gskyhip_render_tiles.argtypes
    L.gskyhip_render_coverage.argtypes = [ci, C.c_uint32, vp, ci, vp, ci, ci, vp, ci, vp, ci, ci, ci, ci,
                                          C.POINTER(ScaleParams), vp, i64, vp, vp, i64, vp]
    L.gskyhip_warp_windows.argtypes = [vp, ci, vp, ci, ci, vp, ci, vp, ci, ci, ci, ci, vp, vp, vp, vp, i64,
                                       vp, i64, vp]
    L.gskyhip_render_status.argtypes = [vp, ci, ci, ci, vp]
    L.gskyhip_compute_reproject_extent.argtypes = [vp, ci, vp, ci, ci, vp, vp, vp, vp]
    L.gskyhip_service_run.argtypes = [C.c_char_p, ci, ci]
    L.gskyhip_service_register_granule.argtypes = [C.c_char_p, C.c_char_p, ci, C.POINTER(Granule), vp,
                                                   C.POINTER(vp), C.c_char_p]
    L.gskyhip_service_unregister_all.argtypes = [C.c_char_p]
    L.gskyhip_service_stats.argtypes = [C.c_char_p, C.POINTER(i64)]
    if hasattr(L, "gskyhip_service_stats_n"):
        L.gskyhip_service_stats_n.argtypes = [C.c_char_p, C.POINTER(i64), C.c_int]
    L.gskyhip_service_shutdown.argtypes = [C.c_char_p]
    L.gskyhip_render_tile_info.argtypes = [vp, ci, ci, ci, vp, vp, vp]
    L.gskyhip_render_pair_info.argtypes = [vp, ci, ci, ci, vp, vp]
    if hasattr(L, "gskyhip_render_touched"):   # (an older A/B library for timing comparisons lacks it)
        L.gskyhip_render_touched.argtypes = [vp, ci, ci, ci, vp, vp]
    L.gskyhip_merge_rasters.argtypes = [C.POINTER(FlexRasterC), ci, C.POINTER(Mask), C.POINTER(vp), ci,
                                        C.POINTER(i32), C.POINTER(i32), C.POINTER(d), vp]
    L.gskyhip_scale.argtypes = [vp, ci, i64, d, C.POINTER(ScaleParams), vp, vp]
    L.gskyhip_scale_legacy.argtypes = [vp, ci, i64, d, C.POINTER(ScaleParams), vp, vp]
    L.gskyhip_gradient_palette.argtypes = [vp, ci, ci, vp]
    L.gskyhip_encode_rgba.argtypes = [C.POINTER(vp), ci, ci, ci, vp, vp, vp]
    L.gskyhip_compute_mask.argtypes = [vp, ci, i64, C.POINTER(Mask), vp, vp]
    L.gskyhip_drill_rows.argtypes = [ci, ci]
    L.gskyhip_drill.argtypes = [vp, ci, ci, ci, ci, vp, vp, vp, ci, C.c_float, C.c_float, C.c_float, ci, ci,
                                vp, vp, vp]
    L.gskyhip_drill_workspace_size.argtypes = [ci, i64, ci, ci, ci]
    L.gskyhip_drill_workspace_size.restype = i64
    L.gskyhip_drill_batch.argtypes = [vp, ci, ci, ci, ci, vp, vp, vp, ci, i64, vp, ci, C.c_float, C.c_float,
                                      C.c_float, ci, ci, ci, vp, vp, vp, i64, vp]
    L.gskyhip_drill_descriptors.argtypes = [C.POINTER(C.c_char_p), ci, C.c_char_p, C.POINTER(d), ci, ci, vp, vp,
                                            C.POINTER(i64), vp, vp]
    L.gskyhip_drill_merge.argtypes = [vp, vp, ci, ci, vp, vp]
    L.gskyhip_drill_descriptors_device.argtypes = [C.POINTER(C.c_char_p), ci, C.c_char_p, C.POINTER(d), ci, ci,
                                                   vp, vp, C.POINTER(i64), vp, vp, vp]
    if hasattr(L, "gskyhip_parse_numbers"):
        L.gskyhip_parse_numbers.argtypes = [C.c_char_p, ci, C.c_void_p, C.c_void_p]
    if hasattr(L, "gskyhip_drill_masks_device_packed"):
        L.gskyhip_drill_masks_device_packed.argtypes = [C.c_char_p, i64, ci, C.c_char_p, C.POINTER(d), ci, ci, vp,
                                                        vp, C.POINTER(i64), vp, vp, C.POINTER(vp), vp, vp]
    if hasattr(L, "gskyhip_drill_masks_device"):   # absent from kept earlier builds (GSKYHIP_LIB=<name>)
        L.gskyhip_drill_masks_device.argtypes = [C.POINTER(C.c_char_p), ci, C.c_char_p, C.POINTER(d), ci, ci, vp,
                                                 vp, C.POINTER(i64), vp, vp, C.POINTER(vp), vp, vp]
    L.gskyhip_band_math.argtypes = [C.c_char_p, C.POINTER(C.c_char_p), C.POINTER(vp), vp, vp, ci, i64, d,
                                    vp, vp]
    L.gskyhip_drill_deciles_workspace_size.argtypes = [ci, i64, ci]
    L.gskyhip_drill_deciles_workspace_size.restype = i64
    L.gskyhip_drill_deciles.argtypes = [vp, ci, ci, ci, ci, vp, vp, vp, ci, i64, vp, ci, C.c_float, ci, ci, vp, vp,
                                        vp, vp, i64, vp]
    L.gskyhip_drill_read_data_workspace_size.argtypes = [ci, i64, ci, ci, ci, ci]
    L.gskyhip_drill_read_data_workspace_size.restype = i64
    L.gskyhip_drill_read_data.argtypes = [vp, ci, ci, ci, ci, vp, vp, vp, ci, i64, vp, ci, C.c_float, C.c_float,
                                          C.c_float, ci, ci, ci, ci, vp, vp, vp, vp, i64, vp]
    L.gskyhip_png_workspace_size.argtypes = [ci, ci, ci]
    L.gskyhip_png_workspace_size.restype = i64
    L.gskyhip_png_bound.argtypes = [ci, ci]
    L.gskyhip_png_bound.restype = i64
    L.gskyhip_encode_png.argtypes = [vp, ci, ci, ci, i64, i64, vp, vp, i64, vp, i64, vp, ci, vp]
    L.gskyhip_geotiff_workspace_size.argtypes = [ci, ci, ci, ci, ci, ci]
    L.gskyhip_geotiff_workspace_size.restype = i64
    L.gskyhip_geotiff_bound.argtypes = [ci, ci, ci, ci, ci, ci]
    L.gskyhip_geotiff_bound.restype = i64
    L.gskyhip_encode_geotiff.argtypes = [C.POINTER(vp), ci, ci, ci, ci, C.POINTER(d), ci, vp,
                                         C.POINTER(C.c_char_p), ci, ci, vp, i64, vp, i64, C.POINTER(i64), vp]
    if hasattr(L, "gskyhip_encode_netcdf"):   # (an older A/B library for timing comparisons lacks it)
        L.gskyhip_netcdf_bound.argtypes = [ci, ci, ci, ci]
        L.gskyhip_netcdf_bound.restype = i64
        L.gskyhip_encode_netcdf.argtypes = [C.POINTER(vp), ci, ci, ci, ci, C.POINTER(d), ci, vp,
                                            C.POINTER(C.c_char_p), ci, ci, vp, i64, C.POINTER(i64), vp]
        L.gskyhip_encode_netcdf_host.argtypes = [C.POINTER(vp), ci, ci, ci, ci, C.POINTER(d), ci, vp,
                                                 C.POINTER(C.c_char_p), ci, ci, vp, i64, C.POINTER(i64)]
    L.gskyhip_fnv32a.argtypes = [C.c_char_p, i64]
    L.gskyhip_fnv32a.restype = C.c_uint32
    L.gskyhip_version.restype = C.c_char_p
    _lib = L
    return L


def check(code: int, what: str = "") -> None:
    if code != 0:
        raise GskyError(code, what)
