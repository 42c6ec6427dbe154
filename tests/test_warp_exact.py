"""Independent check of the warp (no oracle involved): the source pixel the
MI355X path picked for every window pixel, against an exact fp64 transform of
the pixel centre written here from the published formulas -- EPSG:3857
inverse (spherical Mercator), then the source CRS forward: EPSG:3577 Albers
equal area on GRS80 for a C2-shaped batch (Snyder, Map Projections -- A
Working Manual, 14-1..14-12; phi1 -18, phi2 -36, phi0 0, lambda0 132),
EPSG:4326 longitude / latitude for the reference's acceptance tiles (C1 /
C3's pair), the MODIS sinusoidal sphere (R 6371007.181, Snyder 30-1) for C5's
tiles, GDA94 / MGA zone 55 Transverse Mercator (Karney 2011's form,
tests/test_tmerc.py) for UTM granules, Snyder's Lambert Conformal Conic
equations (tests/test_lcc.py) for GA Lambert granules and his polar
stereographic equations (tests/test_stere.py) for Antarctic granules.  The
reference warps through
GDAL's approximate transformer with a 0.125-pixel error bound
(warp.go:219); so for every pixel the picked cell [i, i+1) x [j, j+1) must
reach within 0.125 px of the exact coordinate, and only pixels whose exact
coordinate lies within 0.125 px of a cell edge may pick a different cell
than the exact truncation.  The granules hold their own pixel index as
float32 (exact below 2^24), so each window value names the picked pixel."""
import math

import numpy as np
import pytest

from gsky_amd import synth

from .helpers import gpu_batch

pytestmark = pytest.mark.gpu

A, INV_F = 6378137.0, 298.257222101          # GRS80
E2 = (2 - 1 / INV_F) / INV_F
E = math.sqrt(E2)


def _q(phi):
    s = np.sin(phi)
    return (1 - E2) * (s / (1 - E2 * s * s) - (1 / (2 * E)) * np.log((1 - E * s) / (1 + E * s)))


def _m(phi):
    s = np.sin(phi)
    return np.cos(phi) / np.sqrt(1 - E2 * s * s)


P1, P2, P0, L0 = (math.radians(v) for v in (-18.0, -36.0, 0.0, 132.0))
N = (_m(P1) ** 2 - _m(P2) ** 2) / (_q(P2) - _q(P1))
CC = _m(P1) ** 2 + N * _q(P1)
RHO0 = A * np.sqrt(CC - N * _q(P0)) / N


def albers(lon, lat):
    rho = A * np.sqrt(CC - N * _q(lat)) / N
    th = N * (lon - L0)
    return rho * np.sin(th), RHO0 - rho * np.cos(th)


def merc_inv(x, y):
    R = 6378137.0
    return x / R, np.arctan(np.sinh(y / R))


def _check_picks(cfg, gpu, src_fwd):
    """Every window pixel of cfg's (tile, granule) pairs against the exact
    transform; src_fwd(lon, lat) (radians) -> source CRS coordinates."""
    for g in cfg.granules:   # each granule holds its pixel index
        ny, nx = g.data.shape
        assert nx * ny < 1 << 24
        g.data = np.arange(nx * ny, dtype=np.float32).reshape(ny, nx)
        g.nodata = -1.0
        g.overviews = []
    b = gpu_batch(cfg, gpu)
    wins = b.warp_windows()
    p = 0
    n_px = n_diff = 0
    worst = 0.0
    for t, ((bb, w, h), ks) in enumerate(zip(cfg.tiles, cfg.pairs)):
        gt_t = [bb[0], (bb[2] - bb[0]) / w, 0.0, bb[3], 0.0, -(bb[3] - bb[1]) / h]
        for k in ks:
            arr, (xoff, yoff, ww, hh), tname, nd = wins[p]
            p += 1
            assert tname == "Float32"
            v = arr.cpu().numpy().astype(np.int64)
            g = cfg.granules[k]
            ny, nx = g.data.shape
            jj, ii = np.mgrid[0:hh, 0:ww]
            X = gt_t[0] + (xoff + ii + 0.5) * gt_t[1]
            Y = gt_t[3] + (yoff + jj + 0.5) * gt_t[5]
            lon, lat = merc_inv(X, Y)
            ax, ay = src_fwd(lon, lat)
            sx = (ax - g.geot[0]) / g.geot[1]
            sy = (ay - g.geot[3]) / g.geot[5]
            ok = v >= 0                                 # picked pixels (nodata = outside)
            px, py = v % nx, v // nx
            # the cell reaches within 0.125 px of the exact coordinate on both axes
            dx = np.maximum(np.maximum(px - sx, sx - (px + 1)), 0.0)
            dy = np.maximum(np.maximum(py - sy, sy - (py + 1)), 0.0)
            if ok.any():
                worst = max(worst, float(np.maximum(dx, dy)[ok].max()))
            tx, ty = np.floor(sx + 1e-10).astype(np.int64), np.floor(sy + 1e-10).astype(np.int64)
            diff = ok & ((px != tx) | (py != ty))
            near = np.minimum(np.abs(sx - np.round(sx)), np.abs(sy - np.round(sy))) <= 0.125
            assert not (diff & ~near).any(), (t, k)
            n_px += int(ok.sum())
            n_diff += int(diff.sum())
    return n_px, n_diff, worst


def test_warp_longlat_within_the_approximation_bound(gpu):
    """EPSG:4326 -> EPSG:3857 (C1 / C3's pair) on 60 of the reference's
    acceptance GetMap tiles (tests/golden/acpt_bboxes.json) over six
    overlapping longitude / latitude granules."""
    import json
    import os
    reqs = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "acpt_bboxes.json")))
    cfg = synth.config_acpt(reqs)
    keep = list(range(0, len(cfg.tiles), max(1, len(cfg.tiles) // 60)))[:60]
    cfg.tiles = [cfg.tiles[i] for i in keep]
    cfg.pairs = [cfg.pairs[i] for i in keep]
    n_px, n_diff, worst = _check_picks(cfg, gpu, lambda lon, lat: (np.degrees(lon), np.degrees(lat)))
    assert n_px > 500_000, n_px
    assert worst <= 0.125 + 1e-6, worst
    print("longlat warp vs exact: %d px, %d (%.4f %%) another cell, worst %.4f px"
          % (n_px, n_diff, 100.0 * n_diff / n_px, worst))
    assert n_diff / n_px < 0.15


def test_warp_sinusoidal_within_the_approximation_bound(gpu):
    """MODIS sinusoidal -> EPSG:3857 (C5's pair) on C5's z4 / z5 tiles
    (data granules only, level 0: the overview choice is the oracle's
    parity test's subject)."""
    cfg = synth.config_c5(scale=0.05, dates=1)
    data = [i for i, g in enumerate(cfg.granules) if g.namespace == ""]
    remap = {old: new for new, old in enumerate(data)}
    cfg.granules = [cfg.granules[i] for i in data]
    cfg.pairs = [[remap[k] for k in ks if k in remap] for ks in cfg.pairs]
    cfg.mask = None
    cfg.tiles, cfg.pairs = cfg.tiles[::4], cfg.pairs[::4]
    R = synth.SINU_R
    n_px, n_diff, worst = _check_picks(cfg, gpu, lambda lon, lat: (R * lon * np.cos(lat), R * lat))
    assert n_px > 500_000, n_px
    assert worst <= 0.125 + 1e-6, worst
    print("sinusoidal warp vs exact: %d px, %d (%.4f %%) another cell, worst %.4f px"
          % (n_px, n_diff, 100.0 * n_diff / n_px, worst))
    assert n_diff / n_px < 0.15


def test_warp_within_the_approximation_bound(gpu):
    import torch
    cfg = synth.config_c2(scale=0.25, tiles_per_side=8, tile_px=256)
    for g in cfg.granules:   # each granule holds its pixel index
        ny, nx = g.data.shape
        g.data = np.arange(nx * ny, dtype=np.float32).reshape(ny, nx)
        g.nodata = -1.0
    b = gpu_batch(cfg, gpu)
    wins = b.warp_windows()
    p = 0
    n_px = n_diff = 0
    worst = 0.0
    for t, ((bb, w, h), ks) in enumerate(zip(cfg.tiles, cfg.pairs)):
        gt_t = [bb[0], (bb[2] - bb[0]) / w, 0.0, bb[3], 0.0, -(bb[3] - bb[1]) / h]
        for k in ks:
            arr, (xoff, yoff, ww, hh), tname, nd = wins[p]
            p += 1
            assert tname == "Float32"
            v = arr.cpu().numpy().astype(np.int64)
            g = cfg.granules[k]
            ny, nx = g.data.shape
            jj, ii = np.mgrid[0:hh, 0:ww]
            X = gt_t[0] + (xoff + ii + 0.5) * gt_t[1]
            Y = gt_t[3] + (yoff + jj + 0.5) * gt_t[5]
            lon, lat = merc_inv(X, Y)
            ax, ay = albers(lon, lat)
            sx = (ax - g.geot[0]) / g.geot[1]
            sy = (ay - g.geot[3]) / g.geot[5]
            ok = v >= 0                                 # picked pixels (nodata = outside)
            px, py = v % nx, v // nx
            # the cell reaches within 0.125 px of the exact coordinate on both axes
            dx = np.maximum(np.maximum(px - sx, sx - (px + 1)), 0.0)
            dy = np.maximum(np.maximum(py - sy, sy - (py + 1)), 0.0)
            if ok.any():
                worst = max(worst, float(np.maximum(dx, dy)[ok].max()))
            tx, ty = np.floor(sx + 1e-10).astype(np.int64), np.floor(sy + 1e-10).astype(np.int64)
            diff = ok & ((px != tx) | (py != ty))
            near = np.minimum(np.abs(sx - np.round(sx)), np.abs(sy - np.round(sy))) <= 0.125
            assert not (diff & ~near).any(), (t, k)
            n_px += int(ok.sum())
            n_diff += int(diff.sum())
    assert n_px > 1_000_000
    assert worst <= 0.125 + 1e-6, worst
    print("warp vs exact transform: %d px, %d (%.4f %%) pick another cell than the exact truncation, "
          "worst cell distance %.4f px" % (n_px, n_diff, 100.0 * n_diff / n_px, worst))
    # measured on MI355X: 5.3 % of 3.56 M pixels pick the neighbouring cell,
    # every one within 0.125 px of a cell edge (asserted above); the share is
    # the approximation's error band over the cell size, bounded here loosely
    assert n_diff / n_px < 0.15


def test_warp_utm_within_the_approximation_bound(gpu):
    """GDA94 / MGA zone 55 -> EPSG:3857: the exact transform is Karney's form
    of the Krueger series (tests/test_tmerc.py), not the product's."""
    from .test_tmerc import GRS80, karney
    cfg = synth.config_utm(scale=0.25, tiles_per_side=8, tile_px=256)
    n_px, n_diff, worst = _check_picks(
        cfg, gpu, lambda lon, lat: karney(np.degrees(lon), np.degrees(lat), 147.0, 0.9996, 500000.0, 10000000.0,
                                          GRS80))
    assert n_px > 500_000, n_px
    assert worst <= 0.125 + 1e-6, worst
    print("utm warp vs exact: %d px, %d (%.4f %%) another cell, worst %.4f px"
          % (n_px, n_diff, 100.0 * n_diff / n_px, worst))
    assert n_diff / n_px < 0.15


def test_warp_lambert_within_the_approximation_bound(gpu):
    """GDA94 / Geoscience Australia Lambert (EPSG:3112) -> EPSG:3857: the exact
    transform is Snyder's equations (tests/test_lcc.py), not the product's."""
    from .test_lcc import GRS80 as G, snyder_lcc
    cfg = synth.config_lambert(scale=0.25, tiles_per_side=8, tile_px=256)
    n_px, n_diff, worst = _check_picks(
        cfg, gpu, lambda lon, lat: snyder_lcc(np.degrees(lon), np.degrees(lat), G, -18.0, -36.0, 0.0, 134.0))
    assert n_px > 500_000, n_px
    assert worst <= 0.125 + 1e-6, worst
    print("lambert warp vs exact: %d px, %d (%.4f %%) another cell, worst %.4f px"
          % (n_px, n_diff, 100.0 * n_diff / n_px, worst))
    assert n_diff / n_px < 0.15


def test_warp_polar_within_the_approximation_bound(gpu):
    """WGS 84 / Antarctic Polar Stereographic (EPSG:3031) -> EPSG:3857: the
    exact transform is Snyder's polar equations (tests/test_stere.py)."""
    from .test_stere import WGS84, snyder_polar
    cfg = synth.config_polar(scale=0.25, tiles_per_side=8, tile_px=256)
    n_px, n_diff, worst = _check_picks(
        cfg, gpu, lambda lon, lat: snyder_polar(np.degrees(lon), np.degrees(lat), WGS84, -71.0, 0.0, True))
    assert n_px > 500_000, n_px
    assert worst <= 0.125 + 1e-6, worst
    print("polar stereographic warp vs exact: %d px, %d (%.4f %%) another cell, worst %.4f px"
          % (n_px, n_diff, 100.0 * n_diff / n_px, worst))
    assert n_diff / n_px < 0.15
