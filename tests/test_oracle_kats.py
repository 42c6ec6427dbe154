"""CPU tests: pin the oracle against the reference's own known answers.

- utils/raster_scaler_test.go:18-151 (TestScale): 18 cases, transcribed
  (the reference's utils test binary does not build: ogc_encoders_test.go:77).
- Hand-derived KATs from reading the reference: palette ramp,
  merge order, Go conversion wrap, mask parsing.
Everything else the oracle restates (GDAL/PROJ semantics) is "parity
unpinned" and is checked here only for internal consistency properties.
"""
import math

import numpy as np
import pytest

# (dtype, input, (offset, scale, clip), expected) -- raster_scaler_test.go
SCALE_KATS = []
for dt, line in ((np.uint8, 18), (np.int16, 47), (np.uint16, 82), (np.float32, 111)):
    SCALE_KATS += [
        (dt, [1, 2], (1, 1, 1000), [2, 3]),
        (dt, [1, 2], (0, 0, 2), [127, 254]),
        (dt, [1, 2], (3, 2, 1000), [8, 10]),
        (dt, [1, 2], (3, 2, 2), [4, 4]),
    ]
SCALE_KATS += [
    (np.int16, [-100, -200], (3, 2, 2), [0, 0]),      # raster_scaler_test.go:75-79
    (np.float32, [-100, -200], (3, 2, 2), [0, 0]),    # raster_scaler_test.go:139-143
]


def test_scale_kat_count():
    assert len(SCALE_KATS) == 18


@pytest.mark.parametrize("dt,data,sp,exp", SCALE_KATS)
def test_scale_reference_kats(oracle, dt, data, sp, exp):
    out = oracle.scale(np.array(data, dt), 0.0, sp[0], sp[1], sp[2])
    assert out.tolist() == exp


def test_go_conversion_quirks(oracle):
    L = oracle.lib()
    assert L.or_go_f64_u8(300.0) == 44
    assert L.or_go_f64_u8(1000.0) == 232
    assert L.or_go_f64_i16(-1e10) == 0          # CVTTSD2SL -> 0x80000000
    assert L.or_go_f64_u8(float("nan")) == 0


def test_scale_byte_clip_wrap(oracle):
    # Byte, Clip=1000 -> clip = uint8(1000) = 232: values stay <= 232
    d = np.array([250, 10, 0], np.uint8)
    out = oracle.scale(d, 0.0, 0.0, 1.0, 1000.0)
    assert out.tolist() == [232, 10, 0xFF]


def test_scale_nodata_and_auto(oracle):
    # nodata -> 0xFF; auto mode with pixel 0 nodata: min/max start at 0
    d = np.array([-9999, 100, 200], np.float32)
    out = oracle.scale(d, -9999.0, 0, 0, 0)
    # min=0 (init), max=200: scale = 254/200
    assert out.tolist() == [255, int(np.float32(100) * np.float32(254.0 / 200.0)), 254]
    # pixel 0 valid: min = 50
    d2 = np.array([50, 100, 200], np.int16)
    out2 = oracle.scale(d2, -9999.0, 0, 0, 0)
    assert out2[0] == 0 and out2[2] == 254


def test_scale_log(oracle):
    d = np.array([1.0, 10.0, 100.0, 0.0, -1.0], np.float32)
    out = oracle.scale(d, -9999.0, 0, 1.0, 2.0, colour_scale=1)
    # log10: 0, 1, 2 -> *1 -> clip 2; log10(0) = -inf and log10(-1) = NaN -> nodata
    assert out.tolist() == [0, 1, 2, 255, 255]


def test_palette_kat(oracle):
    # docker/gsky_config.json:26-31, interpolate
    ramp = oracle.gradient_palette([(0, 100, 0, 255), (255, 255, 0, 255), (160, 82, 45, 255)], True)
    assert ramp[0].tolist() == [0, 100, 0, 255]
    assert ramp[127].tolist() == [253, 253, 0, 255]
    assert ramp[128].tolist() == [255, 255, 0, 255]
    assert ramp[255].tolist() == [161, 84, 44, 255]


def test_palette_stepped_and_alpha(oracle):
    ramp = oracle.gradient_palette([(1, 2, 3, 10), (4, 5, 6, 20), (7, 8, 9, 30)], False)
    assert ramp[0].tolist() == [1, 2, 3, 10] and ramp[85].tolist() == [1, 2, 3, 10]
    assert ramp[86].tolist() == [4, 5, 6, 20] and ramp[255].tolist() == [7, 8, 9, 30]
    ramp2 = oracle.gradient_palette([(0, 0, 0, 7), (255, 255, 255, 99)], True)
    assert (ramp2[:, 3] == 7).all()         # alpha of the lower colour (palette.go:22)


def test_encode_rgba(oracle):
    b = np.array([[0, 255], [7, 128]], np.uint8)
    rgba = oracle.encode_rgba([b], 2, 2)
    assert rgba[0, 0].tolist() == [0, 0, 0, 255]
    assert rgba[0, 1].tolist() == [0, 0, 0, 0]
    assert rgba[1, 0].tolist() == [7, 7, 7, 255]
    r = np.array([[255, 1]], np.uint8)
    g = np.array([[255, 255]], np.uint8)
    bl = np.array([[255, 255]], np.uint8)
    rgba3 = oracle.encode_rgba([r, g, bl], 2, 1)
    assert rgba3[0, 0].tolist() == [0, 0, 0, 0] and rgba3[0, 1].tolist() == [1, 255, 255, 255]


def test_fnv32a(oracle):
    assert oracle.fnv32a("") == 0x811C9DC5
    assert oracle.fnv32a("a") == 0xE40C292C
    assert oracle.fnv32a("foobar") == 0xBF9CF968


def _raster(v, ts, ns=0, off=(0, 0), nodata=0.0, ph=0):
    v = np.asarray(v)
    if v.dtype == np.int64:
        v = v.astype(np.int16)
    return dict(data=v, off_x=off[0], off_y=off[1], nodata=nodata, timestamp=ts,
                polygon_hash=ph, ns=ns)


def test_merge_order_kat(oracle):
    # A(ts=1), B(ts=3), C(ts=2) in one batch; a pixel valid in A
    # and C only.  geoStamps sort descending: B, C, A.  B overwrites (ts 3),
    # C (2 < 3) fills holes only, A (1 < 3) fills holes only -> C's value.
    A = _raster([[10]], 1.0)
    B = _raster([[0]], 3.0)
    Cr = _raster([[30]], 2.0)
    (cv, nd), = oracle.merge_batch([A, B, Cr], 1, 1, 1)
    assert int(cv[0, 0]) == 30
    # same stamps but hash differences change the order: A stamp highest
    A2 = _raster([[10]], 1.0, ph=100)
    (cv2, _), = oracle.merge_batch([A2, B, Cr], 1, 1, 1)
    # order A2(101), B(3), C(2): A2 overwrites (1 >= 0), B's pixel is nodata
    # (but canvas ts -> 3), C fills holes only -> A2's value stays
    assert int(cv2[0, 0]) == 10


def test_merge_mask(oracle):
    data = _raster(np.array([[1, 2], [3, 4]], np.int16), 5.0, ns=0, nodata=-1)
    qa = _raster(np.array([[1, 0], [0, 1]], np.uint8), 5.0, ns=1, nodata=255)
    out = oracle.merge_batch([data, qa], 2, 2, 2, mask_ns=1, mask_value="00000001")
    cv, nd = out[0]
    assert cv.tolist() == [[-1, 2], [3, -1]]
    assert out[1] == (None, None)   # non-inclusive mask layer is not merged


def test_compute_mask_parse(oracle):
    d = np.array([0, 1, 2, 3, 255], np.uint8)
    assert oracle.compute_mask(d, "10").tolist() == [False, False, True, True, True]
    # bit tests: (v & 0b11) == 0b01
    assert oracle.compute_mask(d, None, ["11", "01"]).tolist() == [False, True, False, False, False]
    # Int16 Value goes through ParseInt(.., 2, 16): "1000000000000000" is out
    # of range and clamps to 32767 (Go strconv), so both values are masked ...
    s = np.array([-1, 1], np.int16)
    assert oracle.compute_mask(s, "1000000000000000").tolist() == [True, True]
    # ... and with "-1" (all bits) a negative AND result is not masked
    # (tile_merger.go:391: (val & maskValue) > 0 on int16)
    assert oracle.compute_mask(s, "-1").tolist() == [False, True]
    with pytest.raises(ValueError):
        oracle.compute_mask(d, None, ["11"])


def test_drill_kat(oracle):
    data = np.array([[[1, 2], [3, -9999]], [[4, 5], [6, 7]]], np.float32)
    mask = np.array([[255, 255], [0, 255]], np.uint8)
    v, c = oracle.drill_read_data(data, mask, -9999.0, -1e30, 1e30)
    assert c.tolist() == [2, 3]
    assert v[0] == np.float32(1.5) and v[1] == float(np.float32(16.0) / np.float32(3.0))
    # clip filter and pixel_count mode
    v2, c2 = oracle.drill_read_data(data, mask, -9999.0, 4.5, 1e30, pixel_count=1)
    assert c2.tolist() == [2, 3] and v2[0] == 0.0 and v2[1] == float(np.float32(2) / np.float32(3))
    # bandStrides 3 over 4 bands: group 0 -> b0, interp, b2; the short last
    # group still reads {b3, b3} and interpolates bandStrides-2 rows (drill.go:134-218)
    d4 = np.stack([data[0], data[1], data[1], data[0]])
    v3, c3 = oracle.drill_read_data(d4, mask, -9999.0, -1e30, 1e30, band_strides=3)
    assert len(v3) == 6 and v3[3] == v3[4] == v3[5]


def test_drill_merge(oracle):
    v = np.array([[1.0, np.nan], [3.0, 2.0]])
    c = np.array([[1, 0], [3, 2]], np.int32)
    out = oracle.drill_merge(v, c)
    assert out[0] == pytest.approx(2.5) and out[1] == pytest.approx(2.0)


def test_projection_round_trips(oracle):
    wgs, wm, aea, sinu = (oracle.crs(s) for s in ("EPSG:4326", "EPSG:3857", "EPSG:3577", "MODIS"))
    for lon, lat in [(132.0, -25.0), (149.13, -35.28), (115.86, -31.95), (140.0, -10.0)]:
        for c in (wm, aea, sinu):
            x, y = oracle.crs_transform(wgs, c, lon, lat)
            lo, la = oracle.crs_transform(c, wgs, x, y)
            assert lo == pytest.approx(lon, abs=1e-9) and la == pytest.approx(lat, abs=1e-9)
    # EPSG:3577 central meridian maps to x = 0
    x, y = oracle.crs_transform(wgs, aea, 132.0, -25.0)
    assert abs(x) < 1e-6
    # web mercator: x = a * lon
    x, y = oracle.crs_transform(wgs, wm, 90.0, 0.0)
    assert x == pytest.approx(6378137.0 * math.pi / 2) and abs(y) < 1e-6


def test_approx_row_error_bound(oracle):
    """GDALApproxTransform keeps every point within the error bound (0.125
    source px at the split test) -- internal consistency of the restatement."""
    wm, aea = oracle.crs("EPSG:3857"), oracle.crs("EPSG:3577")
    src_gt = np.array([1400000.0, 25.0, 0.0, -3800000.0, 0.0, -25.0])
    dst_gt = np.array([16394750.0, 14.0, 0.0, -3972760.0, 0.0, -14.0])
    n = 512
    x = np.arange(n) + 0.5
    y = np.full(n, 100.5)
    ok = np.zeros(n, np.int32)
    xa, ya = x.copy(), y.copy()
    import ctypes
    oracle.lib().oracle_approx_row(ctypes.byref(aea), ctypes.byref(wm), src_gt.ctypes.data, dst_gt.ctypes.data,
                                   n, xa.ctypes.data, ya.ctypes.data, ok.ctypes.data)
    assert ok.all()
    # exact transforms
    ex = []
    for i in range(0, n, 37):
        X = dst_gt[0] + x[i] * dst_gt[1]
        Y = dst_gt[3] + y[i] * dst_gt[5]
        sx, sy = oracle.crs_transform(wm, aea, X, Y)
        ex.append((i, (sx - src_gt[0]) / 25.0, (sy - src_gt[3]) / -25.0))
    for i, sx, sy in ex:
        assert abs(xa[i] - sx) + abs(ya[i] - sy) < 0.25


def test_compute_reproject_extent_kat(oracle):
    """ComputeReprojectExtent (warp.go:433-487) by hand: with no
    reprojection GDALSuggestedWarpOutput keeps the source pixel size along
    the diagonal, 0.1 deg for a 3600 x 1800 global lon/lat grid, so a
    10 x 5 deg request is int((10 + 0.05) / 0.1) = 100 x 50 pixels; a
    Web Mercator request of the same granule gets the Mercator pixel size of
    the diagonal (about 2 x 0.1 deg of equatorial metres, the Mercator
    stretch of the polar edge samples), and an empty request one pixel."""
    wgs, wm = oracle.crs("EPSG:4326"), oracle.crs("EPSG:3857")
    g = oracle.make_granule(np.zeros((1800, 3600), np.float32), [-180.0, 0.1, 0.0, 90.0, 0.0, -0.1])
    assert oracle.compute_reproject_extent(g, wgs, wgs, [0.0, 0.0, 10.0, 5.0]) == (100, 50)
    assert oracle.compute_reproject_extent(g, wgs, wgs, [0.0, 0.0, 0.0, 0.0]) == (0, 0)
    rc, gt, npx, nln, _ = oracle.suggested_warp_output(g, wgs, wgs, [0.0, 1.0, 0.0, 0.0, 0.0, 1.0])
    assert rc == 0 and gt[1] == pytest.approx(0.1, rel=1e-12) and gt[5] == pytest.approx(-0.1, rel=1e-12)
    assert (npx, nln) == (3600, 1800)
    # a granule that stays clear of the poles reprojects without failures
    g2 = oracle.make_granule(np.zeros((500, 600), np.float32), [110.0, 0.05, 0.0, -10.0, 0.0, -0.05])
    rc, gt, npx, nln, _ = oracle.suggested_warp_output(g2, wgs, wm, [0.0, 1.0, 0.0, 0.0, 0.0, 1.0])
    assert rc == 0 and gt[1] > 0 and gt[5] < 0
    bb = [12245143.98, -4865942.28, 15584728.71, -1118889.97]
    px, ln = oracle.compute_reproject_extent(g2, wgs, wm, bb)
    assert px == int((bb[2] - bb[0] + gt[1] / 2.0) / gt[1]) and ln == int((bb[3] - bb[1] - gt[5] / 2.0) / -gt[5])


def test_compute_deciles_kats(oracle):
    """computeDeciles (drill.go:229-273) by hand: the three branches."""
    m = np.full(12, 255, np.uint8)
    v = np.array([5, 1, 9, 3, 7, 11, 2, 8, 4, 10, 6, 12], np.float32)
    # len 12, dc 3: step 3, 12 % 4 == 0 -> means of sorted[3,4], [6,7], [9,10]
    assert oracle.compute_deciles(v, m, -1.0, 3).tolist() == [4.5, 7.5, 10.5]
    # len 12, dc 4: step 2, 12 % 5 != 0 -> sorted[2], [4], [6], [8]
    assert oracle.compute_deciles(v, m, -1.0, 4).tolist() == [3.0, 5.0, 7.0, 9.0]
    # nodata (1) and masked-out pixels do not count: len 2 < dc + 1 = 5, padding {0: 2, 1: 2}
    m2 = m.copy()
    m2[3:] = 0
    assert oracle.compute_deciles(v, m2, 1.0, 4).tolist() == [5.0, 5.0, 9.0, 9.0]
    # len 2 (values 5, 9 after dropping nodata 1), dc 3: padding {0: 2, 1: 1} -> 5, 5, 9
    assert oracle.compute_deciles(v, m2, 1.0, 3).tolist() == [5.0, 5.0, 9.0]
    # len == dc + 1 with step 1: buf[len] is read -> the reference panics
    assert oracle.compute_deciles(v[:4], m[:4], -1.0, 3) is None


def test_band_math_kats(oracle):
    """Band-math (tile_merger.go:654-731) by hand: NDVI, nodata of ANY axis
    variable masks the pixel (used or not), non-finite -> nodata, a constant
    expression fills every valid pixel, ternary / comparisons as 1.0 / 0.0."""
    nir = np.array([3, 2, 1, -9999, 5], np.float32)
    red = np.array([1, 2, 0, 4, 7], np.float32)
    qa = np.array([0, 0, 0, 0, 255], np.uint8)
    vs = [("nir", nir, -9999.0), ("red", red, -9999.0), ("qa", qa, 255.0)]
    got = oracle.band_math("(nir - red) / (nir + red)", vs, -9999.0)
    assert got.tolist() == [0.5, 0.0, 1.0, -9999.0, -9999.0]
    assert oracle.band_math("nir / (red - red)", vs, -1.0).tolist() == [-1.0, -1.0, -1.0, -1.0, -1.0]
    assert oracle.band_math("2.5", vs, -1.0).tolist() == [2.5, 2.5, 2.5, -1.0, -1.0]
    assert oracle.band_math("nir > red ? nir : 0 - red", vs, -1.0).tolist() == [3.0, -2.0, 1.0, -1.0, -1.0]
    assert oracle.band_math("!(nir == 2) && red < 3", vs, -1.0).tolist() == [1.0, 0.0, 1.0, -1.0, -1.0]
    with pytest.raises(ValueError):
        oracle.band_math("nir + swir", vs, -1.0)


def test_read_data_full_means_match_c_oracle(oracle):
    """The pure-Python readData restatement with bandStrides (drill.go:128-219)
    gives the C oracle's mean / count rows bit for bit, including the
    reference's extra rows for a short last group (10 bands, stride 3 -> 12
    rows)."""
    rng = np.random.default_rng(3)
    d = (rng.random((10, 7, 9)) * 0.3).astype(np.float32)
    d[rng.random(d.shape) < 0.1] = -9999.0
    m = np.where(rng.random((7, 9)) < 0.7, 255, 0).astype(np.uint8)
    for strides in (1, 2, 3, 4, 11):
        for pc, lo, hi in ((0, -1e30, 1e30), (1, 0.05, 0.2)):
            v, c = oracle.drill_read_data_full(d, m, -9999.0, lo, hi, pc, strides, 0)
            ev, ec = oracle.drill_read_data(d, m, -9999.0, lo, hi, pc, strides)
            assert np.array_equal(v[:, 0].view(np.uint64), ev.view(np.uint64)) and np.array_equal(c[:, 0], ec)
    v, _ = oracle.drill_read_data_full(d, m, -9999.0, -1e30, 1e30, 0, 3, 0)
    assert v.shape[0] == 12
