"""Geolocation-array warps (warp.go:52-67, 128-141, 158): requests whose
GeoLocOpts name X / Y datasets (tile_grpc.go:338-350) warp through GDAL
3.0.1's geolocation transformer (forward by interpolating the arrays, inverse
through a backmap) instead of the source geotransform, and never use
overviews.

Parity unpinned: GDAL's gdalgeoloc.cpp is not in /root/reference and GDAL is
absent, so the product (gsky_device.h geoloc_*, host.cpp geoloc_backmap) is
checked against oracle/'s independent restatement of the same published
algorithm, and both against the synthetic swath's own analytic geometry."""
import numpy as np
import pytest

from oracle import oracle as O


def swath(nx=160, ny=120, step=2):
    """A curved swath: geolocation arrays at every `step`-th pixel of a
    (ny*step) x (nx*step) raster, lon/lat bent and sheared like a polar
    orbiter's scan lines."""
    i = np.arange(nx, dtype=np.float64)[None, :]
    j = np.arange(ny, dtype=np.float64)[:, None]
    lon = 130.0 + 0.05 * i + 0.012 * j + 1.5e-4 * (i - nx / 2) ** 2 * 0.1
    lat = -20.0 - 0.045 * j + 0.01 * i - 2.0e-5 * (i - nx / 2) ** 2
    return lon, lat


def raster(ny, nx, seed=5):
    rng = np.random.default_rng(seed)
    d = rng.integers(0, 10000, (ny, nx)).astype(np.int16)
    d[rng.random((ny, nx)) < 0.02] = -999
    return d


def test_oracle_geoloc_backmap_size():
    """The backmap has ~1.3 cells per geolocation sample over the points'
    extent, origin half a cell outside it (GeoLocGenerateBackMap)."""
    lon, lat = swath()
    gl = O.geoloc(lon, lat, pixel_step=2.0, line_step=2.0)
    ext = (lon.max() - lon.min()) * (lat.max() - lat.min())
    ps = np.sqrt(ext / (lon.size * 1.3))
    assert gl.bgt[1] == pytest.approx(ps) and gl.bgt[5] == pytest.approx(-ps)
    assert gl.bw == int(np.ceil((lon.max() - lon.min()) / ps) + 1)
    assert gl.bh == int(np.ceil((lat.max() - lat.min()) / ps) + 1)
    assert gl.bgt[0] == pytest.approx(lon.min() - ps / 2) and gl.bgt[3] == pytest.approx(lat.max() + ps / 2)
    O.free_geoloc(gl)


def test_oracle_geoloc_regular_grid():
    """One-row X and Y bands form a regular grid (GeoLocLoadFullData)."""
    lon = 120.0 + 0.1 * np.arange(50)
    lat = -10.0 - 0.1 * np.arange(40)
    gl = O.geoloc(lon[None, :], lat[None, :])
    assert (gl.nx, gl.ny) == (50, 40)
    O.free_geoloc(gl)


def test_oracle_geoloc_warp_matches_geometry():
    """Warping a raster whose value encodes its own (pixel, line) through
    the oracle's geolocation transformer lands every output pixel within a
    couple of source pixels of where the analytic swath geometry puts it."""
    lon, lat = swath(80, 60, 2)
    ny, nx = 120, 160
    code = (np.arange(ny)[:, None] * nx + np.arange(nx)[None, :]).astype(np.float32)
    g = O.make_granule(code, (0, 1, 0, 0, 0, 1))
    gl = O.geoloc(lon, lat, pixel_step=2.0, line_step=2.0)
    src, dst = O.crs("EPSG:4326"), O.crs("EPSG:4326")
    W = H = 64
    gt = (131.0, 0.03, 0.0, -21.0, 0.0, -0.03)
    arr, bbox, nd, dt = O.warp_geoloc(g, src, dst, gt, W, H, gl)
    assert bbox[2] > 0 and bbox[3] > 0
    ok = arr != np.float32(-1e10)
    assert ok.mean() > 0.5
    # where the output pixel's source pixel came from, the forward geometry
    # (bilinear in the arrays) must map back near the output pixel centre
    yy, xx = np.nonzero(ok)
    v = arr[yy, xx].astype(np.int64)
    sl, sp = v // nx, v % nx
    gi, gj = sp / 2.0, sl / 2.0
    i0, j0 = np.floor(gi).astype(int).clip(0, 78), np.floor(gj).astype(int).clip(0, 58)
    fx, fy = gi - i0, gj - j0
    X = (1 - fy) * (lon[j0, i0] + fx * (lon[j0, i0 + 1] - lon[j0, i0])) + \
        fy * (lon[j0 + 1, i0] + fx * (lon[j0 + 1, i0 + 1] - lon[j0 + 1, i0]))
    Y = (1 - fy) * (lat[j0, i0] + fx * (lat[j0, i0 + 1] - lat[j0, i0])) + \
        fy * (lat[j0 + 1, i0] + fx * (lat[j0 + 1, i0 + 1] - lat[j0 + 1, i0]))
    cx = gt[0] + (xx + bbox[0] + 0.5) * gt[1]
    cy = gt[3] + (yy + bbox[1] + 0.5) * gt[5]
    # inside the swath (a geolocation sample within half its spacing; the
    # backmap's hole filling extrapolates edge pixels a few cells beyond it)
    near = np.hypot(cx[:, None] - lon.ravel()[None, :], cy[:, None] - lat.ravel()[None, :]).min(axis=1) < 0.025
    assert near.mean() > 0.5
    # one source pixel is ~0.025 deg, a backmap cell ~0.04 deg
    assert np.percentile(np.hypot(X - cx, Y - cy)[near], 99) < 0.06
    O.free_geoloc(gl)


def test_oracle_geoloc_missing_fields_fail():
    """GDALCreateGeoLocTransformer with a degenerate extent fails (3)."""
    with pytest.raises(RuntimeError):
        O.geoloc(np.zeros((4, 4)), np.zeros((4, 4)))


@pytest.mark.gpu
def test_gpu_geoloc_drop_in_matches_oracle():
    """warp_operation_fast with GeoLocOpts: the swath's X / Y bands
    registered as their own datasets, several EPSG:3857 and EPSG:4326 tiles
    over and around the swath, bit-identical to the oracle's restatement
    (windows, values, nodata fill); overviews registered with the band are
    ignored (warp.go:158); incomplete options fail with 3."""
    import torch

    from gsky_amd import worker
    from gsky_amd.tiles import bbox_to_geot
    lon, lat = swath()
    ny, nx = 240, 320
    data = raster(ny, nx)
    worker.unregister_all()
    worker.register_granule("swath.nc", 1, torch.from_numpy(data).cuda(), (0, 1, 0, 0, 0, 1), "EPSG:4326", -999.0,
                            overviews=[torch.from_numpy(data[::2, ::2].copy()).cuda()])
    worker.register_granule("lon", 1, torch.from_numpy(lon).cuda(), (0, 1, 0, 0, 0, 1))
    worker.register_granule("lat", 1, torch.from_numpy(lat).cuda(), (0, 1, 0, 0, 0, 1))
    opts = ["X_DATASET=lon", "Y_DATASET=lat", "X_BAND=1", "Y_BAND=1", "LINE_OFFSET=0", "PIXEL_OFFSET=0",
            "LINE_STEP=2", "PIXEL_STEP=2"]
    gl = O.geoloc(lon, lat, pixel_step=2.0, line_step=2.0)
    g = O.make_granule(data, (0, 1, 0, 0, 0, 1), nodata=-999.0)
    src = O.crs("EPSG:4326")
    cases = [("EPSG:4326", (131.0, -24.0, 135.0, -20.5), 256),
             ("EPSG:4326", (129.0, -27.0, 141.0, -18.0), 128),
             ("EPSG:4326", (133.5, -22.5, 134.0, -22.0), 64)]
    for (b0, b1, b2, b3) in [(131.0, -24.0, 135.0, -20.5)]:
        x0, y0 = O.crs_transform(src, O.crs("EPSG:3857"), b0, b1)
        x1, y1 = O.crs_transform(src, O.crs("EPSG:3857"), b2, b3)
        cases.append(("EPSG:3857", (x0, y0, x1, y1), 256))
    n_same = n_all = 0
    for srs, bbox, px in cases:
        gt = bbox_to_geot(px, px, bbox)
        r = worker.warp_raster(worker.GeoRPCGranule(path="swath.nc", bands=[1], width=px, height=px, dstSRS=srs,
                                                    dstGeot=gt, geoLocOpts=opts))
        assert r.error == "OK", (srs, bbox, r.error)
        got = worker.raster_array(r.raster)
        exp, ebbox, end, edt = O.warp_geoloc(g, src, O.crs(srs), gt, px, px, gl)
        assert list(r.raster.bbox) == list(ebbox), (srs, bbox)
        assert got.shape == exp.shape
        n_same += int((got == exp).sum())
        n_all += exp.size
        assert (got != -999).any(), "nothing warped"
    assert n_same == n_all, "%d of %d pixels differ" % (n_all - n_same, n_all)
    bad = worker.warp_raster(worker.GeoRPCGranule(path="swath.nc", bands=[1], width=64, height=64,
                                                  dstSRS="EPSG:4326", dstGeot=bbox_to_geot(64, 64, cases[2][1]),
                                                  geoLocOpts=opts[:3]))
    assert bad.error == "warp_operation() fail: 3"
    O.free_geoloc(gl)
    worker.unregister_all()
    torch.cuda.synchronize()
