"""Lambert Conformal Conic (GDA94 / GDA2020 Geoscience Australia Lambert,
+proj=lcc 1SP / 2SP, WKT1 Lambert_Conformal_Conic_1SP / _2SP): PROJ 6's
ellipsoidal lcc, checked without the oracle against

* Snyder's worked example (Map Projections: A Working Manual, USGS PP 1395,
  p. 296: Clarke 1866, standard parallels 33 / 45 N, origin 23 N 96 W;
  35 N 75 W -> x = 1,894,410.9 m, y = 1,564,649.5 m);
* Snyder's equations 15-1..15-11 written here in numpy (F, t, m as he
  states them, not PROJ's arrangement), over grids for several cones;
* round trips (the inverse iterates pj_phi2 to 1e-10 rad).

The oracle restatement (the warp parity tests' checker) must set up the same
constants and agree to a few ulps; GPU warps from GA Lambert granules are in
tests/test_gpu_parity.py and tests/test_warp_exact.py."""
import math

import numpy as np
import pytest

from gsky_amd import _lib
from gsky_amd.tiles import crs_transform, parse_crs

GRS80 = (6378137.0, 298.257222101)
CLARKE1866 = (6378206.4, 294.978698213898)


def snyder_lcc(lon, lat, ell, lat1, lat2, lat0, lon0, x0=0.0, y0=0.0, k0=1.0):
    """Snyder 15-1..15-11 (ellipsoid), degrees in, metres out."""
    a, rf = ell
    f = 1.0 / rf
    e = math.sqrt(2 * f - f * f)

    def t(phi):
        s = np.sin(phi)
        return np.tan(np.pi / 4 - phi / 2) / ((1 - e * s) / (1 + e * s)) ** (e / 2)

    def m(phi):
        return np.cos(phi) / np.sqrt(1 - e * e * np.sin(phi) ** 2)

    p1, p2, p0 = (math.radians(v) for v in (lat1, lat2, lat0))
    n = math.sin(p1) if abs(p1 - p2) < 1e-12 else (math.log(m(p1)) - math.log(m(p2))) / (
        math.log(t(p1)) - math.log(t(p2)))
    F = m(p1) / (n * t(p1) ** n)
    rho0 = a * k0 * F * t(p0) ** n
    phi = np.radians(np.asarray(lat, float))
    rho = a * k0 * F * t(phi) ** n
    th = n * np.radians(np.asarray(lon, float) - lon0)
    return x0 + rho * np.sin(th), y0 + rho0 - rho * np.cos(th)


def test_snyder_worked_example():
    spec = "+proj=lcc +lat_1=33 +lat_2=45 +lat_0=23 +lon_0=-96 +a=6378206.4 +rf=294.978698213898"
    geo = "+proj=longlat +a=6378206.4 +rf=294.978698213898"
    x, y, ok = crs_transform(geo, spec, [-75.0], [35.0])
    assert ok.all() and abs(x[0] - 1894410.9) < 0.05 and abs(y[0] - 1564649.5) < 0.05, (x, y)
    lo, la, ok = crs_transform(spec, geo, x, y)
    assert ok.all() and abs(lo[0] + 75.0) < 1e-10 and abs(la[0] - 35.0) < 1e-10


@pytest.mark.parametrize("spec,ell,lat1,lat2,lat0,lon0,x0,y0,k0,box", [
    ("EPSG:3112", GRS80, -18.0, -36.0, 0.0, 134.0, 0.0, 0.0, 1.0, (112, 154, -44, -10)),
    ("EPSG:7845", GRS80, -18.0, -36.0, 0.0, 134.0, 0.0, 0.0, 1.0, (112, 154, -44, -10)),
    ("+proj=lcc +lat_1=33 +lat_2=45 +lat_0=23 +lon_0=-96 +x_0=1000000 +y_0=500000 +ellps=WGS84",
     (6378137.0, 298.257223563), 33.0, 45.0, 23.0, -96.0, 1e6, 5e5, 1.0, (-125, -67, 20, 50)),
    ("+proj=lcc +lat_1=-30 +lat_0=-30 +lon_0=140 +k_0=0.9995 +ellps=GRS80", GRS80, -30.0, -30.0, -30.0, 140.0,
     0.0, 0.0, 0.9995, (125, 155, -40, -20)),
    ("+proj=lcc +lat_1=49 +lon_0=10 +ellps=GRS80", GRS80, 49.0, 49.0, 49.0, 10.0, 0.0, 0.0, 1.0, (0, 20, 40, 58)),
])
def test_lcc_matches_snyder(spec, ell, lat1, lat2, lat0, lon0, x0, y0, k0, box):
    rng = np.random.default_rng(11)
    lon = rng.uniform(box[0], box[1], 3000)
    lat = rng.uniform(box[2], box[3], 3000)
    geo = "+proj=longlat +a=%.17g +rf=%.17g" % ell
    x, y, ok = crs_transform(geo, spec, lon, lat)
    assert ok.all()
    ex, ey = snyder_lcc(lon, lat, ell, lat1, lat2, lat0, lon0, x0, y0, k0)
    assert np.abs(x - ex).max() < 1e-6 and np.abs(y - ey).max() < 1e-6, (np.abs(x - ex).max(), np.abs(y - ey).max())
    lo, la, ok = crs_transform(spec, geo, x, y)
    assert ok.all()
    assert np.abs(lo - lon).max() < 1e-9 and np.abs(la - lat).max() < 1e-9


def test_lcc_srs_forms():
    wkt2 = ('PROJCS["GDA94 / Geoscience Australia Lambert",GEOGCS["GDA94",DATUM["Geocentric_Datum_of_Australia_1994",'
            'SPHEROID["GRS 1980",6378137,298.257222101]],PRIMEM["Greenwich",0],UNIT["degree",0.0174532925199433]],'
            'PROJECTION["Lambert_Conformal_Conic_2SP"],PARAMETER["standard_parallel_1",-18],'
            'PARAMETER["standard_parallel_2",-36],PARAMETER["latitude_of_origin",0],PARAMETER["central_meridian",134],'
            'PARAMETER["false_easting",0],PARAMETER["false_northing",0],UNIT["metre",1],AUTHORITY["EPSG","3112"]]')
    a, b = parse_crs(wkt2), parse_crs("EPSG:3112")
    for f, _ in _lib.Crs._fields_:
        va, vb = getattr(a, f), getattr(b, f)
        assert (list(va) == list(vb)) if hasattr(va, "__len__") else va == vb, f
    c = parse_crs(wkt2.replace(',AUTHORITY["EPSG","3112"]]', "]"))
    assert c.kind == 5 and (c.n, c.c, c.rho0) == (b.n, b.c, b.rho0)
    wkt1 = ('PROJCS["x",GEOGCS["GRS80",DATUM["d",SPHEROID["GRS 1980",6378137,298.257222101]]],'
            'PROJECTION["Lambert_Conformal_Conic_1SP"],PARAMETER["latitude_of_origin",-30],'
            'PARAMETER["central_meridian",140],PARAMETER["scale_factor",0.9995],PARAMETER["false_easting",0],'
            'PARAMETER["false_northing",0],UNIT["metre",1]]')
    d = parse_crs(wkt1)
    e = parse_crs("+proj=lcc +lat_1=-30 +lat_0=-30 +lon_0=140 +k_0=0.9995 +ellps=GRS80")
    assert d.kind == e.kind == 5 and (d.n, d.c, d.rho0, d.k0) == (e.n, e.c, e.rho0, e.k0)
    for bad in ("+proj=lcc +lat_1=30 +lat_2=40 +R=6371000", "+proj=lcc +lat_1=30 +lat_2=-30 +ellps=GRS80"):
        with pytest.raises(Exception):
            parse_crs(bad)


def test_oracle_lcc_is_the_product_transform(oracle):
    rng = np.random.default_rng(5)
    for srs, box in (("EPSG:3112", (112, 154, -44, -10)),
                     ("+proj=lcc +lat_1=33 +lat_2=45 +lat_0=23 +lon_0=-96 +ellps=WGS84", (-125, -67, 20, 50))):
        c, o = parse_crs(srs), oracle.crs(srs)
        for f in ("kind", "a", "es", "lam0", "phi0", "phi1", "phi2", "k0", "n", "c", "rho0"):
            assert getattr(c, f) == getattr(o, f), (srs, f)
        lon, lat = rng.uniform(box[0], box[1], 300), rng.uniform(box[2], box[3], 300)
        x, y, ok = crs_transform("EPSG:4326", srs, lon, lat)
        src, dst = oracle.crs("EPSG:4326"), oracle.crs(srs)
        for i in range(lon.size):
            r = oracle.crs_transform(src, dst, float(lon[i]), float(lat[i]))
            assert ok[i] and abs(r[0] - x[i]) <= 4e-9 and abs(r[1] - y[i]) <= 4e-9, (srs, i)
