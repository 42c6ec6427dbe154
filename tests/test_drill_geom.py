"""Drill request geometry (A16): polygon -> window -> ALL_TOUCHED mask,
worker/gdalprocess/drill.go:363-423 (getDrillFileDescriptor) and 275-327
(createMask).  The product's host implementation (libgskyhip.so,
gskyhip_drill_descriptors) against the oracle's independent C restatement on
the same GeoJSON, plus hand-derived known answers.  GDAL/GEOS are absent, so
parity with a running reference is unpinned; these tests pin the
product to the restatement bit for bit.  The product's rasterizer (scanline
fill as per-edge parity toggles, drill_geom.cpp) is a different algorithm from
the oracle's (GDAL's sorted intersection spans); they agree on every polygon
below, including the reference's own WPS acceptance geometries
(tests/golden/wps_polygons.json.gz: 32 local-government areas of 359-16,922
vertices, extracted from acceptance_tests/polygon_requests/*.xml)."""
import gzip
import json
import os

import numpy as np
import pytest

from gsky_amd import drill, synth

GT4326 = [130.0, 0.01, 0.0, -20.0, 0.0, -0.01]
WPS_DATASETS = [("EPSG:4326", [112.0, 0.01, 0.0, -9.0, 0.0, -0.01], 4300, 3500),
                ("EPSG:4326", [112.0, 0.0025, 0.0, -9.0, 0.0, -0.0025], 17200, 14000),
                ("EPSG:3577", [-2000000.0, 250.0, 0.0, -1000000.0, 0.0, -250.0], 16000, 16000)]


def wps_polygons():
    """{request file: GeoJSON geometry} of the reference's WPS acceptance requests."""
    p = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "wps_polygons.json.gz")
    with gzip.open(p, "rt", encoding="utf-8") as f:
        return json.load(f)


def feature(rings, multi=False):
    coords = [[[list(p) for p in r] for r in rings]] if multi else [[list(p) for p in r] for r in rings]
    return json.dumps({"type": "Feature", "properties": {},
                       "geometry": {"type": "MultiPolygon" if multi else "Polygon", "coordinates": coords}})


def close(pts):
    pts = [tuple(p) for p in pts]
    return pts + [pts[0]]


def stars(n, gt, size, seed):
    rng = np.random.default_rng(seed)
    out = []
    for p in range(n):
        r = rng.uniform(3, 60)
        cx, cy = rng.uniform(-20, size + 20), rng.uniform(-20, size + 20)   # some cross the file edge
        pix = synth.star_polygon(cx, cy, r, k=int(rng.integers(3, 13)), seed=p)
        lon = gt[0] + pix[:, 0] * gt[1]
        lat = gt[3] + pix[:, 1] * gt[5]
        out.append(feature([close(np.stack([lon, lat], 1))]))
    return out


def test_descriptor_known_answers(oracle):
    # a square over pixels 10.25 .. 12.75: offsets truncate and count = int(max) - off (drill.go:404-407)
    x0, y0 = 130 + 0.1025, -20 - 0.1025
    sq = feature([close([(x0, y0), (x0 + 0.025, y0), (x0 + 0.025, y0 - 0.025), (x0, y0 - 0.025)])])
    win, off, buf, st = drill.drill_descriptors([sq], "EPSG:4326", GT4326, 2048, 2048)
    assert st.tolist() == [0] and win[0].tolist() == [10, 10, 2, 2]
    assert buf[:4].tolist() == [255] * 4
    # a polygon entirely outside the file: no window (the reference's
    # indexer never sends such a file; here it is reported per polygon)
    far = feature([close([(100, 10), (101, 10), (101, 11), (100, 11)])])
    win, off, buf, st = drill.drill_descriptors([far, sq], "EPSG:4326", GT4326, 2048, 2048)
    assert st[0] != 0 and win[0].tolist() == [0, 0, 0, 0] and st[1] == 0
    # thin diagonal: ALL_TOUCHED burns every pixel the edges cross
    tri = feature([close([(130.0005, -20.0005), (130.0595, -20.0295), (130.0005, -20.0015)])])
    win, off, buf, st = drill.drill_descriptors([tri], "EPSG:4326", GT4326, 2048, 2048)
    m = buf[off[0]:off[0] + win[0][2] * win[0][3]].reshape(win[0][3], win[0][2])
    ew, em = oracle.drill_descriptor(tri, "EPSG:4326", GT4326, 2048, 2048)
    assert tuple(win[0]) == ew and np.array_equal(m, em)
    assert (m == 255).sum() >= win[0][2]      # at least one pixel per column along the long edge


@pytest.mark.parametrize("srs,seed", [("EPSG:4326", 1), ("EPSG:4326", 2), ("EPSG:3577", 3), ("EPSG:28355", 4),
                                      ("EPSG:3112", 5), ("EPSG:3031", 6)])
def test_descriptor_matches_oracle(oracle, srs, seed):
    if srs == "EPSG:4326":
        gt, size = GT4326, 2048
        geoms = stars(120, gt, size, seed)
    elif srs in ("EPSG:28355", "EPSG:3112"):   # MGA zone 55 / GA Lambert: polygons around lon 145.5, lat -36.5
        gt, size = ([230000.0, 100.0, 0.0, 6080000.0, 0.0, -100.0] if srs == "EPSG:28355"
                    else [880000.0, 150.0, 0.0, -3990000.0, 0.0, -150.0]), 2400
        rng = np.random.default_rng(seed)
        geoms = []
        for p in range(60):
            lon0, lat0 = rng.uniform(144.2, 146.8), rng.uniform(-37.8, -35.6)
            pts = synth.star_polygon(lon0, lat0, rng.uniform(0.02, 0.3), k=9, seed=p)
            geoms.append(feature([close(pts)]))
    elif srs == "EPSG:3031":   # Antarctic polar stereographic: polygons off the Peninsula
        gt, size = [-2500000.0, 150.0, 0.0, 1500000.0, 0.0, -150.0], 2400
        rng = np.random.default_rng(seed)
        geoms = []
        for p in range(60):
            lon0, lat0 = rng.uniform(-61.5, -59.3), rng.uniform(-66.8, -65.0)
            pts = synth.star_polygon(lon0, lat0, rng.uniform(0.02, 0.3), k=9, seed=p)
            geoms.append(feature([close(pts)]))
    else:   # Albers dataset: polygons in lon/lat around lon 132, lat -27
        gt, size = [-300000.0, 250.0, 0.0, -2800000.0, 0.0, -250.0], 2400
        rng = np.random.default_rng(seed)
        geoms = []
        for p in range(60):
            lon0, lat0 = rng.uniform(128.5, 135.0), rng.uniform(-31.5, -25.0)
            r = rng.uniform(0.05, 0.6)
            pts = synth.star_polygon(lon0, lat0, r, k=9, seed=p)
            geoms.append(feature([close(pts)]))
    win, off, buf, st = drill.drill_descriptors(geoms, srs, gt, size, size)
    n_ok = 0
    for i, g in enumerate(geoms):
        try:
            ew, em = oracle.drill_descriptor(g, srs, gt, size, size)
        except ValueError:
            assert st[i] != 0, i
            continue
        assert st[i] == 0 and tuple(win[i]) == ew, (i, win[i], ew)
        m = buf[off[i]:off[i] + ew[2] * ew[3]].reshape(ew[3], ew[2])
        assert np.array_equal(m, em), i
        n_ok += 1
    assert n_ok > len(geoms) // 2


def test_descriptor_multipolygon_with_hole(oracle):
    outer = close([(130.1, -20.1), (130.5, -20.1), (130.5, -20.5), (130.1, -20.5)])
    hole = close([(130.2, -20.2), (130.4, -20.2), (130.4, -20.4), (130.2, -20.4)])
    other = close([(130.6, -20.6), (130.7, -20.6), (130.65, -20.7)])
    g = feature([[outer, hole], [other]][0], multi=False)
    mp = json.dumps({"type": "MultiPolygon", "coordinates": [[[list(p) for p in outer], [list(p) for p in hole]],
                                                             [[list(p) for p in other]]]})
    for geom in (g, mp):
        win, off, buf, st = drill.drill_descriptors([geom], "EPSG:4326", GT4326, 2048, 2048)
        ew, em = oracle.drill_descriptor(geom, "EPSG:4326", GT4326, 2048, 2048)
        assert st[0] == 0 and tuple(win[0]) == ew
        m = buf[off[0]:off[0] + ew[2] * ew[3]].reshape(ew[3], ew[2])
        assert np.array_equal(m, em)
        assert m[25, 25] == 0 and m[5, 5] == 255      # the hole is not burnt, the ring is


@pytest.mark.parametrize("ds", range(len(WPS_DATASETS)))
def test_wps_acceptance_polygons_match_oracle(oracle, ds):
    """The reference's 32 WPS polygons (+ its sample polygon payload; the
    point payload is not a polygon and is refused): windows and ALL_TOUCHED
    masks equal the oracle's, on a 0.01 and a 0.0025 degree EPSG:4326 grid
    and a 250 m Albers grid over Australia."""
    srs, gt, xs, ys = WPS_DATASETS[ds]
    polys = wps_polygons()
    names = sorted(polys)
    geoms = [polys[k] for k in names]
    win, off, buf, st = drill.drill_descriptors(geoms, srs, gt, xs, ys)
    n_ok = 0
    for i, g in enumerate(geoms):
        try:
            ew, em = oracle.drill_descriptor(g, srs, gt, xs, ys)
        except ValueError:
            assert st[i] != 0, names[i]
            continue
        assert st[i] == 0 and tuple(win[i]) == ew, (names[i], win[i], ew)
        m = buf[off[i]:off[i] + ew[2] * ew[3]].reshape(ew[3], ew[2])
        assert np.array_equal(m, em), names[i]
        n_ok += 1
    assert n_ok >= 32
    assert st[names.index("point_drill.payload")] != 0


def test_descriptor_bad_geometry():
    win, off, buf, st = drill.drill_descriptors(['{"type": "Point", "coordinates": [1, 2]}', "nonsense"],
                                                "EPSG:4326", GT4326, 2048, 2048)
    assert (st != 0).all() and (win == 0).all()


@pytest.mark.gpu
@pytest.mark.parametrize("srs,seed", [("EPSG:4326", 5), ("EPSG:3577", 6)])
def test_descriptor_masks_on_gpu(oracle, srs, seed):
    """The ALL_TOUCHED masks burnt on the GPU (gskyhip_drill_descriptors_device:
    one workgroup per polygon, edges then scanlines) are the host rasterizer's
    masks byte for byte, and the oracle's; the windows / offsets / status are
    the host call's.  Includes polygons crossing the file edge, a multipolygon
    with a hole and a 90-vertex ring."""
    import torch
    if srs == "EPSG:4326":
        gt, size = GT4326, 2048
        geoms = stars(150, gt, size, seed)
        outer = close([(130.1, -20.1), (130.5, -20.1), (130.5, -20.5), (130.1, -20.5)])
        hole = close([(130.2, -20.2), (130.4, -20.2), (130.4, -20.4), (130.2, -20.4)])
        geoms.append(json.dumps({"type": "MultiPolygon", "coordinates": [[[list(p) for p in outer],
                                                                          [list(p) for p in hole]]]}))
        ang = np.linspace(0, 2 * np.pi, 90, endpoint=False)
        rad = 0.2 + 0.05 * np.sin(ang * 7)
        geoms.append(feature([close(np.stack([130.9 + rad * np.cos(ang), -20.9 + rad * np.sin(ang)], 1))]))
    else:
        gt, size = [-300000.0, 250.0, 0.0, -2800000.0, 0.0, -250.0], 2400
        rng = np.random.default_rng(seed)
        geoms = []
        for p in range(60):
            lon0, lat0 = rng.uniform(128.5, 135.0), rng.uniform(-31.5, -25.0)
            geoms.append(feature([close(synth.star_polygon(lon0, lat0, rng.uniform(0.05, 0.6), k=9, seed=p))]))
    win, off, buf, st = drill.drill_descriptors(geoms, srs, gt, size, size)
    mb, st2 = drill.drill_dataset(geoms, srs, gt, size, size, device="cuda", rasterize="gpu")
    torch.cuda.synchronize()
    assert np.array_equal(st, st2)
    assert np.array_equal(mb.win.cpu().numpy(), win) and np.array_equal(mb.mask_off.cpu().numpy(), off)
    gm = mb.masks.cpu().numpy()
    assert gm.size == buf.size and np.array_equal(gm, buf)
    n_ok = 0
    for i, g in enumerate(geoms):
        if st[i] != 0:
            continue
        ew, em = oracle.drill_descriptor(g, srs, gt, size, size)
        assert np.array_equal(gm[off[i]:off[i] + ew[2] * ew[3]].reshape(ew[3], ew[2]), em), i
        n_ok += 1
    assert n_ok > len(geoms) // 2


@pytest.mark.gpu
@pytest.mark.parametrize("ds", range(len(WPS_DATASETS)))
def test_wps_acceptance_polygons_on_gpu(oracle, ds):
    """The reference's WPS polygons (up to 16,922 vertices) rasterized on the
    GPU -- no vertex or intersection bound, no host fallback -- equal the
    host call's and the oracle's windows and masks byte for byte, issued on a
    non-default stream."""
    import torch
    srs, gt, xs, ys = WPS_DATASETS[ds]
    polys = wps_polygons()
    names = sorted(polys)
    geoms = [polys[k] for k in names]
    win, off, buf, st = drill.drill_descriptors(geoms, srs, gt, xs, ys)
    side = torch.cuda.Stream()
    with torch.cuda.stream(side):
        mb, st2 = drill.drill_dataset(geoms, srs, gt, xs, ys, device="cuda", rasterize="gpu")
        gm = mb.masks.cpu().numpy()
    torch.cuda.synchronize()
    assert np.array_equal(st, st2)
    assert np.array_equal(mb.win.cpu().numpy(), win) and np.array_equal(mb.mask_off.cpu().numpy(), off)
    assert gm.size == buf.size and np.array_equal(gm, buf)
    n_ok = 0
    for i, g in enumerate(geoms):
        if st[i] != 0:
            continue
        ew, em = oracle.drill_descriptor(g, srs, gt, xs, ys)
        assert np.array_equal(gm[off[i]:off[i] + ew[2] * ew[3]].reshape(ew[3], ew[2]), em), names[i]
        n_ok += 1
    assert n_ok >= 32


def test_geojson_number_parser_matches_float():
    """The descriptor step's decimal parser (drill_geom.cpp fast_decimal:
    64x128-bit reciprocal products, exact division near halfway, strtod past
    19 digits) returns what Python's float() (correctly rounded) returns, bit
    for bit, on GeoJSON-style coordinates, integers, exponents and long
    mantissas."""
    import ctypes as C

    from gsky_amd._lib import lib
    rng = np.random.default_rng(11)
    strs = []
    for _ in range(60000):
        nd = int(rng.integers(1, 22))
        d = "".join(map(str, rng.integers(0, 10, nd)))
        pt = int(rng.integers(0, nd + 1))
        s = ("-" if rng.random() < 0.5 else "") + d[:pt] + "." + d[pt:]
        if pt == 0:
            s = s.replace(".", "0.", 1)
        if rng.random() < 0.25:
            s += "e%d" % int(rng.integers(-25, 26))
        strs.append(s)
    # round-trip reprs of doubles (17 significant digits) and halfway-adjacent ones
    for v in rng.standard_normal(20000) * 10.0 ** rng.integers(-8, 9, 20000):
        strs.append(repr(float(v)))
        strs.append("%.17e" % v)
    strs += ["0", "-0.0", "1e19", "9007199254740993", "9007199254740993.0", "0.1", "123456789012345678",
             "1.7976931348623157e308", "4.9e-324", "18446744073709551615", "0.30000000000000004"]
    buf = b"\0".join(s.encode() for s in strs) + b"\0"
    out = np.zeros(len(strs), np.float64)
    used = np.zeros(len(strs), np.int32)
    assert lib().gskyhip_parse_numbers(buf, len(strs), out.ctypes.data_as(C.c_void_p),
                                       used.ctypes.data_as(C.c_void_p)) == 0
    exp = np.array([float(s) for s in strs])
    assert (used == np.array([len(s) for s in strs])).all()
    bad = np.nonzero(out.view(np.uint64) != exp.view(np.uint64))[0]
    assert bad.size == 0, [(strs[i], out[i], exp[i]) for i in bad[:5]]
