"""Transverse Mercator (UTM, GDA94 / GDA2020 MGA, +proj=tmerc): the exact
ellipsoidal algorithm PROJ 6 runs for tmerc / utm (Poder / Engsager), checked
without the oracle against

* a published known-answer point: Flinders Peak, GDA94 -> MGA zone 55
  (Geocentric Datum of Australia Technical Manual, the worked example:
  37 57 03.72030 S, 144 25 29.52440 E -> E 273 741.297, N 5 796 489.777);
* an independent restatement of the same mathematics in another form --
  Karney (2011), "Transverse Mercator with an accuracy of a few nanometers":
  conformal latitude through tau' = sinh(asinh(tan phi) - e atanh(e sin phi)),
  then the Krueger alpha series; no Gaussian-latitude series, no Clenshaw;
* round trips forward -> inverse.

The C-ABI host transform (gskyhip_crs_transform) runs the functions the
kernels run (gsky_device.h crs_inverse / crs_forward).  The oracle restatement
(the warp parity tests' checker) must set up the same constants and agree to
a few ulps; the GPU warps from UTM granules are in tests/test_warp_exact.py
and tests/test_gpu_parity.py."""
import ctypes as C
import math

import numpy as np
import pytest

from gsky_amd import _lib
from gsky_amd.tiles import parse_crs

GRS80 = (6378137.0, 298.257222101)
WGS84 = (6378137.0, 298.257223563)


def transform(src: str, dst: str, x, y):
    a, b = parse_crs(src), parse_crs(dst)
    x = np.array(x, dtype=np.float64).ravel().copy()
    y = np.array(y, dtype=np.float64).ravel().copy()
    ok = np.zeros(x.size, np.int32)
    assert _lib.lib().gskyhip_crs_transform(C.byref(a), C.byref(b), x.size, x.ctypes.data, y.ctypes.data,
                                            ok.ctypes.data) == 0
    return x, y, ok.astype(bool)


def karney(lon, lat, lon0, k0, x0, y0, ell, lat0=0.0):
    """Karney 2011 eq. (7)-(11), (35): (lon, lat) degrees -> (E, N)."""
    a, rf = ell
    f = 1 / rf
    n = f / (2 - f)
    e = math.sqrt(f * (2 - f))
    A = a / (1 + n) * (1 + n ** 2 / 4 + n ** 4 / 64 + n ** 6 / 256)
    al = [0.0,
          n / 2 - 2 * n ** 2 / 3 + 5 * n ** 3 / 16 + 41 * n ** 4 / 180 - 127 * n ** 5 / 288 + 7891 * n ** 6 / 37800,
          13 * n ** 2 / 48 - 3 * n ** 3 / 5 + 557 * n ** 4 / 1440 + 281 * n ** 5 / 630 - 1983433 * n ** 6 / 1935360,
          61 * n ** 3 / 240 - 103 * n ** 4 / 140 + 15061 * n ** 5 / 26880 + 167603 * n ** 6 / 181440,
          49561 * n ** 4 / 161280 - 179 * n ** 5 / 168 + 6601661 * n ** 6 / 7257600,
          34729 * n ** 5 / 80640 - 3418889 * n ** 6 / 1995840,
          212378941 * n ** 6 / 319334400]

    def xi_eta(lon, lat):
        phi, lam = np.radians(lat), np.radians(lon - lon0)
        t = np.sinh(np.arcsinh(np.tan(phi)) - e * np.arctanh(e * np.sin(phi)))
        xi_, eta_ = np.arctan2(t, np.cos(lam)), np.arctanh(np.sin(lam) / np.sqrt(1 + t * t))
        xi = xi_ + sum(al[j] * np.sin(2 * j * xi_) * np.cosh(2 * j * eta_) for j in range(1, 7))
        eta = eta_ + sum(al[j] * np.cos(2 * j * xi_) * np.sinh(2 * j * eta_) for j in range(1, 7))
        return xi, eta

    xi, eta = xi_eta(np.asarray(lon, float), np.asarray(lat, float))
    xi0, _ = xi_eta(np.array(lon0, float), np.array(lat0, float))
    return x0 + k0 * A * eta, y0 + k0 * A * (xi - xi0)


def test_flinders_peak_mga55():
    lat = -(37 + 57 / 60 + 3.72030 / 3600)
    lon = 144 + 25 / 60 + 29.52440 / 3600
    x, y, ok = transform("EPSG:4283", "EPSG:28355", [lon], [lat])
    assert ok.all()
    assert abs(x[0] - 273741.297) < 0.001 and abs(y[0] - 5796489.777) < 0.001, (x, y)
    lo, la, ok = transform("EPSG:28355", "EPSG:4283", x, y)
    assert ok.all()
    assert abs(lo[0] - lon) < 1e-10 and abs(la[0] - lat) < 1e-10
    # GDA2020 MGA zone 55 shares the projection (GRS80, no datum shift here)
    x2, y2, _ = transform("EPSG:4283", "EPSG:7855", [lon], [lat])
    assert x2[0] == x[0] and y2[0] == y[0]


@pytest.mark.parametrize("srs,lon0,k0,x0,y0,ell,lat0,south", [
    ("EPSG:28355", 147.0, 0.9996, 500000.0, 10000000.0, GRS80, 0.0, True),
    ("EPSG:28350", 117.0, 0.9996, 500000.0, 10000000.0, GRS80, 0.0, True),
    ("EPSG:7856", 153.0, 0.9996, 500000.0, 10000000.0, GRS80, 0.0, True),
    ("EPSG:32633", 15.0, 0.9996, 500000.0, 0.0, WGS84, 0.0, False),
    ("EPSG:32701", -177.0, 0.9996, 500000.0, 10000000.0, WGS84, 0.0, True),
    ("+proj=utm +zone=60 +ellps=WGS84", 177.0, 0.9996, 500000.0, 0.0, WGS84, 0.0, False),
    ("+proj=utm +zone=54 +south +ellps=GRS80", 141.0, 0.9996, 500000.0, 10000000.0, GRS80, 0.0, True),
    ("+proj=tmerc +lat_0=-28 +lon_0=153 +k=0.99999 +x_0=50000 +y_0=100000 +ellps=GRS80",
     153.0, 0.99999, 50000.0, 100000.0, GRS80, -28.0, True),
    ("+proj=tmerc +lat_0=49 +lon_0=-2 +k_0=0.9996012717 +x_0=400000 +y_0=-100000 +a=6377563.396 +rf=299.3249646",
     -2.0, 0.9996012717, 400000.0, -100000.0, (6377563.396, 299.3249646), 49.0, False),
])
def test_tmerc_matches_an_independent_krueger_restatement(srs, lon0, k0, x0, y0, ell, lat0, south):
    rng = np.random.default_rng(7)
    lon = lon0 + rng.uniform(-6.0, 6.0, 4000)
    lat = (-1 if south else 1) * rng.uniform(0.0, 80.0, 4000)
    geo = "+proj=longlat +a=%.17g +rf=%.17g" % ell
    x, y, ok = transform(geo, srs, lon, lat)
    assert ok.all()
    ex, ey = karney(lon, lat, lon0, k0, x0, y0, ell, lat0)
    assert np.abs(x - ex).max() < 1e-6 and np.abs(y - ey).max() < 1e-6, (np.abs(x - ex).max(), np.abs(y - ey).max())
    lo, la, ok = transform(srs, geo, x, y)
    assert ok.all()
    dlon = (lo - lon + 180.0) % 360.0 - 180.0
    assert np.abs(dlon).max() < 1e-9 and np.abs(la - lat).max() < 1e-9


def test_tmerc_far_from_the_meridian():
    """Beyond 150 degrees of spherical easting the algorithm gives up
    (HUGE_VAL in PROJ): the transform reports failure."""
    x, y, ok = transform("EPSG:4326", "EPSG:32633", [15.0, 100.0, 15.0 + 89.0], [10.0, 0.0, 0.5])
    assert ok[0] and not ok[1]
    _, _, ok = transform("EPSG:32633", "EPSG:4326", [500000.0 + 3.0e7], [0.0])
    assert not ok[0]


def test_tmerc_srs_forms():
    from gsky_amd.tiles import parse_crs as P
    for spec in ("EPSG:32601", "EPSG:32660", "EPSG:32701", "EPSG:32760", "EPSG:28348", "EPSG:28358", "EPSG:7846",
                 "EPSG:7859", "+proj=utm +zone=33 +datum=WGS84", "+proj=etmerc +lon_0=9 +ellps=GRS80"):
        assert P(spec).kind == 4, spec
    wkt = ('PROJCS["GDA94 / MGA zone 55",GEOGCS["GDA94",DATUM["Geocentric_Datum_of_Australia_1994",'
           'SPHEROID["GRS 1980",6378137,298.257222101,AUTHORITY["EPSG","7019"]],AUTHORITY["EPSG","6283"]],'
           'PRIMEM["Greenwich",0],UNIT["degree",0.0174532925199433],AUTHORITY["EPSG","4283"]],'
           'PROJECTION["Transverse_Mercator"],PARAMETER["latitude_of_origin",0],PARAMETER["central_meridian",147],'
           'PARAMETER["scale_factor",0.9996],PARAMETER["false_easting",500000],'
           'PARAMETER["false_northing",10000000],UNIT["metre",1],AUTHORITY["EPSG","28355"]]')
    a, b = P(wkt), P("EPSG:28355")
    for f, _ in _lib.Crs._fields_:
        va, vb = getattr(a, f), getattr(b, f)
        assert (list(va) == list(vb)) if hasattr(va, "__len__") else va == vb, f
    # without the authority the parameters still define it
    c = P(wkt.replace(',AUTHORITY["EPSG","28355"]]', "]"))
    assert c.kind == 4 and c.lam0 == b.lam0 and c.y0 == b.y0 and c.tm_zb == b.tm_zb
    for bad in ("EPSG:32600", "EPSG:32662", "EPSG:28347", "+proj=utm +ellps=GRS80", "+proj=utm +zone=61",
                "+proj=tmerc +R=6371000", "+proj=tmerc +approx +ellps=GRS80"):
        with pytest.raises(Exception):
            P(bad)


def test_oracle_tmerc_is_the_product_transform(oracle):
    """The warp parity tests' checker sets up the same constants bit for bit
    and transforms to within a few ulps of the host transform (the two
    libraries are built by different compilers, whose libm call choices --
    sincos, inlined hypot -- may round the last bit differently)."""
    rng = np.random.default_rng(3)
    for srs, lon0 in (("EPSG:28355", 147.0), ("EPSG:32633", 15.0), ("EPSG:32760", 177.0)):
        c, o = parse_crs(srs), oracle.crs(srs)
        for f, _ in oracle.Crs._fields_:
            vo, vc = getattr(o, f), getattr(c, f)
            assert (list(vo) == list(vc)) if hasattr(vo, "__len__") else vo == vc, (srs, f)
        lon = lon0 + rng.uniform(-5, 5, 300)
        lat = rng.uniform(-60, 60, 300)
        x, y, ok = transform("EPSG:4326", srs, lon, lat)
        src, dst = oracle.crs("EPSG:4326"), oracle.crs(srs)
        for i in range(lon.size):
            r = oracle.crs_transform(src, dst, float(lon[i]), float(lat[i]))
            assert ok[i] and abs(r[0] - x[i]) <= 4e-9 and abs(r[1] - y[i]) <= 4e-9, (srs, i, r, x[i], y[i])
