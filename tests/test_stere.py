"""Polar stereographic (WGS 84 / Antarctic Polar Stereographic EPSG:3031,
NSIDC Sea Ice Polar Stereographic North EPSG:3413, EPSG:3976, UPS North /
South EPSG:32661 / 32761, +proj=stere at a pole, +proj=ups, WKT1
Polar_Stereographic, CF polar_stereographic): PROJ 6's ellipsoidal stere in
its polar aspects, checked without the oracle against

* Snyder's worked example (Map Projections: A Working Manual, USGS PP 1395,
  p. 317: International ellipsoid, true scale at 71 S, central meridian
  100 W; 75 S 150 E -> x = -1,540,033.6 m, y = -560,526.4 m);
* Snyder's equations 21-33..21-36 written here in numpy over grids;
* the scale factor: 1 along the true-scale parallel, k0 at the pole (UPS
  0.994), measured from the transform by finite differences;
* round trips (the inverse iterates to 1e-10 rad).

The oracle restatement (the warp parity tests' checker) must set up the same
constants and agree to a few ulps; GPU warps from a polar stereographic
granule are in tests/test_gpu_parity.py."""
import math

import numpy as np
import pytest

from gsky_amd import _lib
from gsky_amd.tiles import crs_transform, parse_crs

WGS84 = (6378137.0, 298.257223563)
INTL = (6378388.0, 297.0)


def snyder_polar(lon, lat, ell, lat_ts, lon0, south, k0=1.0, x0=0.0, y0=0.0):
    """Snyder 21-33..21-36 (ellipsoid, polar aspects), degrees in, metres out;
    the south pole by his sign flips of phi, lambda, lambda0 and phi_c."""
    a, rf = ell
    f = 1.0 / rf
    e = math.sqrt(2 * f - f * f)
    sg = -1.0 if south else 1.0
    phi = sg * np.radians(np.asarray(lat, float))
    dl = sg * np.radians(np.asarray(lon, float) - lon0)

    def t(p):
        s = np.sin(p)
        return np.tan(np.pi / 4 - p / 2) / ((1 - e * s) / (1 + e * s)) ** (e / 2)

    if lat_ts is None or abs(abs(lat_ts) - 90) < 1e-12:
        rho = 2 * a * k0 * t(phi) / math.sqrt((1 + e) ** (1 + e) * (1 - e) ** (1 - e))
    else:
        pc = math.radians(abs(lat_ts))
        mc = math.cos(pc) / math.sqrt(1 - e * e * math.sin(pc) ** 2)
        rho = a * mc * t(phi) / t(pc)
    return x0 + sg * rho * np.sin(dl), y0 - sg * rho * np.cos(dl)


def test_snyder_worked_example():
    spec = "+proj=stere +lat_0=-90 +lat_ts=-71 +lon_0=-100 +a=6378388 +rf=297"
    geo = "+proj=longlat +a=6378388 +rf=297"
    x, y, ok = crs_transform(geo, spec, [150.0], [-75.0])
    assert ok.all() and abs(x[0] + 1540033.6) < 0.05 and abs(y[0] + 560526.4) < 0.05, (x, y)
    lo, la, ok = crs_transform(spec, geo, x, y)
    assert ok.all() and abs(lo[0] - 150.0) < 1e-10 and abs(la[0] + 75.0) < 1e-10


@pytest.mark.parametrize("spec,ell,lat_ts,lon0,south,k0,x0,box", [
    ("EPSG:3031", WGS84, -71.0, 0.0, True, 1.0, 0.0, (-180, 180, -89.99, -45)),
    ("EPSG:3976", WGS84, -70.0, 0.0, True, 1.0, 0.0, (-180, 180, -89.99, -45)),
    ("EPSG:3413", WGS84, 70.0, -45.0, False, 1.0, 0.0, (-180, 180, 45, 89.99)),
    ("EPSG:32661", WGS84, None, 0.0, False, 0.994, 2e6, (-180, 180, 60, 90)),
    ("EPSG:32761", WGS84, None, 0.0, True, 0.994, 2e6, (-180, 180, -90, -60)),
    ("+proj=stere +lat_0=-90 +lat_ts=-71 +lon_0=-100 +a=6378388 +rf=297", INTL, -71.0, -100.0, True, 1.0, 0.0,
     (-180, 180, -89, -50)),
    ("+proj=stere +lat_0=90 +lon_0=10 +k_0=0.97 +x_0=300000 +ellps=GRS80", (6378137.0, 298.257222101), None, 10.0,
     False, 0.97, 3e5, (-180, 180, 50, 89.9)),
])
def test_stere_matches_snyder(spec, ell, lat_ts, lon0, south, k0, x0, box):
    rng = np.random.default_rng(13)
    lon = rng.uniform(box[0], box[1], 3000)
    lat = rng.uniform(box[2], box[3], 3000)
    geo = "+proj=longlat +a=%.17g +rf=%.17g" % ell
    x, y, ok = crs_transform(geo, spec, lon, lat)
    assert ok.all()
    y0 = 2e6 if spec.startswith("EPSG:32") else 0.0
    ex, ey = snyder_polar(lon, lat, ell, lat_ts, lon0, south, k0, x0, y0)
    assert np.abs(x - ex).max() < 1e-6 and np.abs(y - ey).max() < 1e-6, (np.abs(x - ex).max(), np.abs(y - ey).max())
    lo, la, ok = crs_transform(spec, geo, x, y)
    assert ok.all()
    dl = np.abs((lo - lon + 180) % 360 - 180)
    assert dl[np.abs(lat) < 89.9].max() < 1e-9 and np.abs(la - lat).max() < 1e-9


@pytest.mark.parametrize("spec,lat_k,k_expect", [
    ("EPSG:3031", -71.0, 1.0), ("EPSG:3413", 70.0, 1.0), ("EPSG:3976", -70.0, 1.0),
    ("EPSG:32661", 89.9999, 0.994), ("EPSG:32761", -89.9999, 0.994)])
def test_scale_factor(spec, lat_k, k_expect):
    """Parallels are circles about the pole, so k = rho / (a m(phi)), rho the
    plane distance from the pole's image and a m = a cos(phi) / sqrt(1 - e^2
    sin^2 phi) the parallel's radius on the ellipsoid: 1 on the true-scale
    parallel, k0 at the pole."""
    a, rf = WGS84
    f = 1 / rf
    e2 = 2 * f - f * f
    pole = 90.0 if lat_k > 0 else -90.0
    x, y, ok = crs_transform("EPSG:4326", spec, [30.0, 0.0], [lat_k, pole])
    assert ok.all()
    phi = math.radians(lat_k)
    k = math.hypot(x[0] - x[1], y[0] - y[1]) / (a * math.cos(phi) / math.sqrt(1 - e2 * math.sin(phi) ** 2))
    assert abs(k - k_expect) < 1e-9, k


def test_pole_and_origin():
    for code, pole in ((32661, 90.0), (32761, -90.0)):
        x, y, ok = crs_transform("EPSG:4326", "EPSG:%d" % code, [0.0, 123.0], [pole, pole])
        assert ok.all() and np.all(x == 2000000.0) and np.all(y == 2000000.0)
        lo, la, ok = crs_transform("EPSG:%d" % code, "EPSG:4326", [2000000.0], [2000000.0])
        assert ok.all() and lo[0] == 0.0 and la[0] == pole
    # EPSG:3031: the prime meridian runs up the +y axis, 90 E along +x
    x, y, ok = crs_transform("EPSG:4326", "EPSG:3031", [0.0, 90.0], [-71.0, -71.0])
    assert ok.all() and abs(x[0]) < 1e-9 and y[0] > 0 and x[1] > 0 and abs(y[1]) < 1e-6


def _fields_equal(a, b):
    for f, _ in _lib.Crs._fields_:
        va, vb = getattr(a, f), getattr(b, f)
        assert (list(va) == list(vb)) if hasattr(va, "__len__") else va == vb, f


def test_stere_srs_forms():
    wkt = ('PROJCS["WGS 84 / Antarctic Polar Stereographic",GEOGCS["WGS 84",DATUM["WGS_1984",'
           'SPHEROID["WGS 84",6378137,298.257223563]],PRIMEM["Greenwich",0],UNIT["degree",0.0174532925199433]],'
           'PROJECTION["Polar_Stereographic"],PARAMETER["latitude_of_origin",-71],PARAMETER["central_meridian",0],'
           'PARAMETER["scale_factor",1],PARAMETER["false_easting",0],PARAMETER["false_northing",0],UNIT["metre",1]]')
    _fields_equal(parse_crs(wkt), parse_crs("EPSG:3031"))
    _fields_equal(parse_crs("+proj=stere +lat_0=-90 +lat_ts=-71 +lon_0=0 +datum=WGS84"), parse_crs("EPSG:3031"))
    _fields_equal(parse_crs("+proj=stere +lat_0=90 +lat_ts=70 +lon_0=-45 +ellps=WGS84"), parse_crs("EPSG:3413"))
    _fields_equal(parse_crs("+proj=ups +ellps=WGS84"), parse_crs("EPSG:32661"))
    _fields_equal(parse_crs("+proj=ups +south +ellps=WGS84"), parse_crs("EPSG:32761"))
    _fields_equal(parse_crs("+proj=stere +lat_0=90 +lat_ts=90 +lon_0=0 +k=0.994 +x_0=2000000 +y_0=2000000 "
                            "+datum=WGS84"), parse_crs("EPSG:32661"))
    ups_wkt = wkt.replace('"latitude_of_origin",-71', '"latitude_of_origin",90').replace(
        '"scale_factor",1', '"scale_factor",0.994').replace('"false_easting",0', '"false_easting",2000000').replace(
        '"false_northing",0', '"false_northing",2000000')
    _fields_equal(parse_crs(ups_wkt), parse_crs("EPSG:32661"))
    for bad in ("+proj=stere +lat_0=45 +lon_0=10 +ellps=WGS84",       # oblique: not carried
                "+proj=stere +lat_0=90 +R=6371000"):                  # spherical: not carried
        with pytest.raises(Exception):
            parse_crs(bad)


def test_oracle_stere_is_the_product_transform(oracle):
    rng = np.random.default_rng(7)
    for srs, box in (("EPSG:3031", (-180, 180, -89.9, -50)), ("EPSG:3413", (-180, 180, 50, 89.9)),
                     ("EPSG:32761", (-180, 180, -90, -60)),
                     ("+proj=stere +lat_0=90 +lon_0=10 +k_0=0.97 +ellps=GRS80", (-180, 180, 50, 89.9))):
        c, o = parse_crs(srs), oracle.crs(srs)
        for f in ("kind", "a", "es", "lam0", "phi0", "phi1", "k0", "c", "x0", "y0"):
            assert getattr(c, f) == getattr(o, f), (srs, f)
        lon, lat = rng.uniform(box[0], box[1], 300), rng.uniform(box[2], box[3], 300)
        x, y, ok = crs_transform("EPSG:4326", srs, lon, lat)
        lo, la, ok2 = crs_transform(srs, "EPSG:4326", x, y)
        src, dst = oracle.crs("EPSG:4326"), oracle.crs(srs)
        for i in range(lon.size):
            r = oracle.crs_transform(src, dst, float(lon[i]), float(lat[i]))
            assert ok[i] and abs(r[0] - x[i]) <= 4e-9 and abs(r[1] - y[i]) <= 4e-9, (srs, i)
            r = oracle.crs_transform(dst, src, float(x[i]), float(y[i]))
            assert ok2[i] and abs(r[0] - lo[i]) <= 1e-12 and abs(r[1] - la[i]) <= 1e-12, (srs, i)
