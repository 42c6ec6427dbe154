"""Synthetic workloads of BASELINE.json's configs.

There is no network and no NCI data, so every granule is generated from a
splitmix64 stream (per-granule seed 0x6A5D0000 + k) with the shapes, CRSs,
nodata patterns and timestamps the survey fixes.  Each generator takes a
`scale` so tests can run the same geometry at sizes the CPU oracle finishes in
seconds; scale=1 is the full benchmark size.
"""
from __future__ import annotations

import json
import math
import os
from concurrent.futures import ThreadPoolExecutor
from dataclasses import dataclass, field
from typing import List, Optional, Tuple

import numpy as np

SEED0 = 0x6A5D0000
PALETTE_GSKY = [(0, 100, 0, 255), (255, 255, 0, 255), (160, 82, 45, 255)]  # docker/gsky_config.json:26-31
WEBMERC_A = 6378137.0


def splitmix64(x: np.ndarray) -> np.ndarray:
    """splitmix64 finaliser over uint64 counters (vectorised)."""
    with np.errstate(over="ignore"):
        z = (x + np.uint64(0x9E3779B97F4A7C15)).astype(np.uint64)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def uniform01(h: np.ndarray) -> np.ndarray:
    return (h >> np.uint64(11)).astype(np.float64) * (1.0 / 9007199254740992.0)


def _pmap(fn, items):
    """Map over granules / bands on a thread pool (numpy releases the GIL in
    its ufuncs); results in input order, bit-identical to a serial loop."""
    items = list(items)
    workers = max(1, min(16, os.cpu_count() or 1, len(items)))
    if workers == 1:
        return [fn(x) for x in items]
    with ThreadPoolExecutor(workers) as ex:
        return list(ex.map(fn, items))


# ---------------------------------------------------------------- projections for setup only
# (tile grids and indexer footprints; the warp itself runs in libgskyhip.so)
def merc_fwd(lon, lat):
    lon = np.radians(lon)
    lat = np.radians(lat)
    return WEBMERC_A * lon, WEBMERC_A * np.log(np.tan(np.pi / 4 + lat / 2))


def merc_inv(x, y):
    return np.degrees(x / WEBMERC_A), np.degrees(np.pi / 2 - 2 * np.arctan(np.exp(-y / WEBMERC_A)))


class _Aea:
    """EPSG:3577 (GRS80, lat1 -18, lat2 -36, lon0 132) for setup geometry."""

    def __init__(self):
        a, rf = 6378137.0, 298.257222101
        f = 1 / rf
        self.a, self.es = a, 2 * f - f * f
        self.e = math.sqrt(self.es)
        self.lam0 = math.radians(132.0)
        p1, p2 = math.radians(-18.0), math.radians(-36.0)
        m = lambda p: math.cos(p) / math.sqrt(1 - self.es * math.sin(p) ** 2)
        q = self.q
        self.n = (m(p1) ** 2 - m(p2) ** 2) / (q(math.sin(p2)) - q(math.sin(p1)))
        self.c = m(p1) ** 2 + self.n * q(math.sin(p1))
        self.rho0 = math.sqrt(self.c) / self.n

    def q(self, s):
        e, es = self.e, self.es
        return (1 - es) * (s / (1 - es * s * s) - (0.5 / e) * np.log((1 - e * s) / (1 + e * s)))

    def inv(self, x, y):
        x = np.asarray(x, float) / self.a
        y = self.rho0 - np.asarray(y, float) / self.a
        rho = np.hypot(x, y)
        if self.n < 0:
            rho, x, y = -rho, -x, -y
        qv = (self.c - (rho * self.n) ** 2) / self.n
        phi = np.arcsin(qv / 2)
        for _ in range(10):
            s = np.sin(phi)
            con = self.e * s
            com = 1 - con * con
            phi = phi + 0.5 * com * com / np.cos(phi) * (
                qv / (1 - self.es) - s / com + 0.5 / self.e * np.log((1 - con) / (1 + con)))
        lam = np.arctan2(x, y) / self.n + self.lam0
        return np.degrees(lam), np.degrees(phi)


AEA = _Aea()
SINU_R = 6371007.181


def sinu_inv(x, y):
    lat = y / SINU_R
    return np.degrees(x / (SINU_R * np.cos(lat))), np.degrees(lat)


# ---------------------------------------------------------------- containers
@dataclass
class SynthGranule:
    data: np.ndarray
    geot: List[float]
    srs: str
    nodata: Optional[float]
    timestamp: float = 0.0
    polygon: str = ""
    namespace: str = ""
    overviews: List[np.ndarray] = field(default_factory=list)


@dataclass
class SynthConfig:
    name: str
    granules: List[SynthGranule]
    dst_srs: str
    tiles: List[Tuple[Tuple[float, float, float, float], int, int]]
    pairs: List[List[int]]
    namespaces: List[str]
    scale: Tuple[float, float, float, int]   # offset, scale, clip, colour_scale
    palette: Optional[list]
    resample: int = 0
    mask: Optional[dict] = None
    bbox: Optional[Tuple[float, float, float, float]] = None   # whole coverage (C3)
    out_w: int = 0
    out_h: int = 0

    @property
    def out_pixels(self) -> int:
        return sum(w * h for (_, w, h) in self.tiles)

    def index_chunk(self, bbox) -> List[int]:
        """The indexer's granule list for one request bbox (MAS intersects)."""
        fps = getattr(self, "_fps", None)
        if fps is None:
            fps = self._fps = [_footprint_merc(g) for g in self.granules]
        return [k for k, f in enumerate(fps) if f[0] < bbox[2] and f[2] > bbox[0] and f[1] < bbox[3] and f[3] > bbox[1]]


def _footprint_merc(g: SynthGranule, n=16):
    """Granule footprint (edge samples) in EPSG:3857 -> bbox."""
    h, w = g.data.shape
    gt = g.geot
    t = np.linspace(0.0, 1.0, n)
    px = np.concatenate([t * w, t * w, np.zeros(n), np.full(n, w)])
    py = np.concatenate([np.zeros(n), np.full(n, h), t * h, t * h])
    X = gt[0] + px * gt[1] + py * gt[2]
    Y = gt[3] + px * gt[4] + py * gt[5]
    if g.srs == "EPSG:3577":
        lon, lat = AEA.inv(X, Y)
    elif g.srs == "EPSG:4326":
        lon, lat = X, np.clip(Y, -85.05, 85.05)
    elif g.srs.upper() in ("MODIS", "SR-ORG:6842") or "+proj=sinu" in g.srs:
        lon, lat = sinu_inv(X, Y)
        lon = np.clip(lon, -180, 180)
    else:   # any other SRS the library parses (UTM / MGA zones): its host transform
        from .tiles import crs_transform
        lon, lat, _ = crs_transform(g.srs, "EPSG:4326", X, Y)
    mx, my = merc_fwd(lon, lat)
    return mx.min(), my.min(), mx.max(), my.max()


def _index_pairs(cfg_granules, tiles):
    """The indexer's granule list per tile (MAS intersects; bbox test)."""
    fps = [_footprint_merc(g) for g in cfg_granules]
    pairs = []
    for (bb, _, _) in tiles:
        lst = []
        for k, f in enumerate(fps):
            if f[0] < bb[2] and f[2] > bb[0] and f[1] < bb[3] and f[3] > bb[1]:
                lst.append(k)
        pairs.append(lst)
    return pairs


def _grid_tiles(bbox, n_x, n_y, px):
    tw = (bbox[2] - bbox[0]) / n_x
    th = (bbox[3] - bbox[1]) / n_y
    tiles = []
    for j in range(n_y):
        for i in range(n_x):
            x0 = bbox[0] + i * tw
            y1 = bbox[3] - j * th
            tiles.append(((x0, y1 - th, x0 + tw, y1), px, px))
    return tiles


# ---------------------------------------------------------------- C1
C1_BBOX = (15028131.257091936, -7514065.628545966, 17532819.79994059, -5009377.085697312)


def config_c1(scale: float = 1.0) -> SynthConfig:
    """Single 256x256 EPSG:3857 GetMap tile from one EPSG:4326 float32 granule."""
    W, H = int(round(3600 * scale)), int(round(1800 * scale))
    res = 360.0 / W
    k = 0
    idx = np.arange(W * H, dtype=np.uint64).reshape(H, W) + np.uint64((SEED0 + k) << 32)
    hh = splitmix64(idx)
    lon = -180 + res * (np.arange(W) + 0.5)
    lat = 90 - res * (np.arange(H) + 0.5)
    v = 500 + 400 * np.sin(np.pi * lon[None, :] / 45) * np.cos(np.pi * lat[:, None] / 30)
    v = v + (uniform01(hh) * 10 - 5)
    nod = uniform01(splitmix64(hh)) < 0.01
    v = v.astype(np.float32)
    v[nod] = -9999.0
    g = SynthGranule(v, [-180.0, res, 0.0, 90.0, 0.0, -res], "EPSG:4326", -9999.0, 1577836800.0,
                     "POLYGON ((-180 -90,-180 90,180 90,180 -90,-180 -90))")
    tiles = [(C1_BBOX, 256, 256)]
    return SynthConfig("C1", [g], "EPSG:3857", tiles, [[0]], [""], (0.0, 0.0, 1000.0, 0), None)


def config_acpt(requests, res: float = 0.02) -> SynthConfig:
    """The reference's acceptance GetMap requests (tests/golden/acpt_bboxes.json:
    500 EPSG:3857 256^2 tiles over Australia) over six overlapping synthetic
    EPSG:4326 float32 granules (3 x 2, 20 x 19 degrees at `res`, one day
    apart, nodata at 1 %), nearest, clip 1000 scale, the docker palette: the
    indexer's granule lists from the footprints."""
    def make(k):
        j, i = divmod(k, 3)
        x0, y0 = 100.0 + 19.0 * i, -10.0 - 17.0 * j
        nx, ny = int(round(20.0 / res)), int(round(19.0 / res))
        idx = np.arange(nx * ny, dtype=np.uint64).reshape(ny, nx) + np.uint64((SEED0 + 0xAC00 + k) << 32)
        hh = splitmix64(idx)
        lon = x0 + res * (np.arange(nx) + 0.5)
        lat = y0 - res * (np.arange(ny) + 0.5)
        v = 500 + 400 * np.sin(np.pi * lon[None, :] / 7) * np.cos(np.pi * lat[:, None] / 5) + (uniform01(hh) * 10 - 5)
        v = v.astype(np.float32)
        v[uniform01(splitmix64(hh)) < 0.01] = -9999.0
        poly = "POLYGON ((%g %g,%g %g,%g %g,%g %g,%g %g))" % (x0, y0, x0 + 20, y0, x0 + 20, y0 - 19, x0, y0 - 19, x0, y0)
        return SynthGranule(v, [x0, res, 0.0, y0, 0.0, -res], "EPSG:4326", -9999.0, 1577836800.0 + 86400.0 * k,
                            poly)
    granules = _pmap(make, range(6))
    tiles = [((r[0], r[1], r[2], r[3]), int(r[4]), int(r[5])) for r in requests]
    cfg = SynthConfig("ACPT", granules, "EPSG:3857", tiles, [], [""], (0.0, 0.0, 1000.0, 0), PALETTE_GSKY)
    cfg.pairs = [cfg.index_chunk(bb) for (bb, _, _) in tiles]
    return cfg


# ---------------------------------------------------------------- C2
def config_c2(scale: float = 1.0, tiles_per_side: int = 64, tile_px: int = 512, grid: int = 4) -> SynthConfig:
    """Batch of EPSG:3857 tiles from `grid`^2 Albers EPSG:3577 int16 granules
    (full size: 16 x 4000^2 at 25 m, 64 x 64 tiles of 512^2)."""
    n = int(round(4000 * scale))
    psize = 100000.0 / n        # a granule always spans 100 km
    def make(k):
        j, i = divmod(k, grid)
        x0 = 1400000.0 + 95000.0 * i
        y0 = -3800000.0 - 95000.0 * j
        idx = np.arange(n * n, dtype=np.uint64).reshape(n, n) + np.uint64((SEED0 + k) << 32)
        v = (splitmix64(idx) % np.uint64(10000)).astype(np.int16)
        nb = (n + 63) // 64
        bidx = np.arange(nb * nb, dtype=np.uint64) + np.uint64(((SEED0 + k) << 32) | 0xB10C0000)
        blk = (uniform01(splitmix64(bidx)) < 0.1).reshape(nb, nb)
        mask = np.repeat(np.repeat(blk, 64, 0), 64, 1)[:n, :n]
        v[mask] = -999
        poly = "POLYGON ((%.1f %.1f,%.1f %.1f,%.1f %.1f,%.1f %.1f,%.1f %.1f))" % (
            x0, y0, x0 + 100000, y0, x0 + 100000, y0 - 100000, x0, y0 - 100000, x0, y0)
        return SynthGranule(v, [x0, psize, 0.0, y0, 0.0, -psize], "EPSG:3577", -999.0,
                            1577836800.0 + 86400.0 * k, poly)

    granules = _pmap(make, range(grid * grid))
    # union bbox forward-projected to EPSG:3857
    ux0, uy1 = 1400000.0, -3800000.0
    ux1 = 1400000.0 + 95000.0 * (grid - 1) + 100000.0
    uy0 = -3800000.0 - 95000.0 * (grid - 1) - 100000.0
    t = np.linspace(0, 1, 64)
    X = np.concatenate([ux0 + t * (ux1 - ux0)] * 2 + [np.full(64, ux0), np.full(64, ux1)])
    Y = np.concatenate([np.full(64, uy0), np.full(64, uy1)] + [uy0 + t * (uy1 - uy0)] * 2)
    lon, lat = AEA.inv(X, Y)
    mx, my = merc_fwd(lon, lat)
    bbox = (float(np.floor(mx.min())), float(np.floor(my.min())), float(np.ceil(mx.max())),
            float(np.ceil(my.max())))
    tiles = _grid_tiles(bbox, tiles_per_side, tiles_per_side, tile_px)
    pairs = _index_pairs(granules, tiles)
    return SynthConfig("C2", granules, "EPSG:3857", tiles, pairs, [""], (0.0, 0.0, 10000.0, 0), PALETTE_GSKY)


# ---------------------------------------------------------------- UTM (widening)
def config_utm(scale: float = 1.0, tiles_per_side: int = 16, tile_px: int = 256, grid: int = 2,
               srs: str = "EPSG:28355", origin=(250000.0, 5900000.0)) -> SynthConfig:
    """C2's shape from projected granules of another family: `grid`^2 int16
    granules of GDA94 / MGA zone 55 (default; 4000^2 at 25 m at full size,
    100 km each, 5 km overlaps, over Victoria around 144-147 E) -- or any
    `srs` with the union's top-left corner at `origin` (config_lambert) --
    EPSG:3857 tiles over their union, nearest, the C2 scale and palette."""
    n = int(round(4000 * scale))
    psize = 100000.0 / n
    def make(k):
        j, i = divmod(k, grid)
        x0 = origin[0] + 95000.0 * i
        y0 = origin[1] - 95000.0 * j
        idx = np.arange(n * n, dtype=np.uint64).reshape(n, n) + np.uint64((SEED0 + 0x7A00 + k) << 32)
        v = (splitmix64(idx) % np.uint64(10000)).astype(np.int16)
        v[uniform01(splitmix64(idx)) < 0.02] = -999
        poly = "POLYGON ((%.1f %.1f,%.1f %.1f,%.1f %.1f,%.1f %.1f,%.1f %.1f))" % (
            x0, y0, x0 + 100000, y0, x0 + 100000, y0 - 100000, x0, y0 - 100000, x0, y0)
        return SynthGranule(v, [x0, psize, 0.0, y0, 0.0, -psize], srs, -999.0, 1577836800.0 + 86400.0 * k, poly)

    granules = [make(k) for k in range(grid * grid)]
    from .tiles import crs_transform
    ux0, uy1 = origin
    ux1, uy0 = ux0 + 95000.0 * (grid - 1) + 100000.0, uy1 - 95000.0 * (grid - 1) - 100000.0
    t = np.linspace(0, 1, 64)
    X = np.concatenate([ux0 + t * (ux1 - ux0)] * 2 + [np.full(64, ux0), np.full(64, ux1)])
    Y = np.concatenate([np.full(64, uy0), np.full(64, uy1)] + [uy0 + t * (uy1 - uy0)] * 2)
    lon, lat, _ = crs_transform(srs, "EPSG:4326", X, Y)
    mx, my = merc_fwd(lon, lat)
    bbox = (float(np.floor(mx.min())), float(np.floor(my.min())), float(np.ceil(mx.max())),
            float(np.ceil(my.max())))
    tiles = _grid_tiles(bbox, tiles_per_side, tiles_per_side, tile_px)
    pairs = _index_pairs(granules, tiles)
    return SynthConfig("UTM", granules, "EPSG:3857", tiles, pairs, [""], (0.0, 0.0, 10000.0, 0), PALETTE_GSKY)


def config_lambert(scale: float = 1.0, tiles_per_side: int = 16, tile_px: int = 256, grid: int = 2) -> SynthConfig:
    """config_utm's shape from GDA94 / Geoscience Australia Lambert (EPSG:3112)
    granules around Sydney (x 1.40-1.60 Mm, y -3.82 to -4.02 Mm)."""
    cfg = config_utm(scale, tiles_per_side, tile_px, grid, srs="EPSG:3112", origin=(1400000.0, -3820000.0))
    cfg.name = "LCC"
    return cfg


def config_polar(scale: float = 1.0, tiles_per_side: int = 16, tile_px: int = 256, grid: int = 2,
                 srs: str = "EPSG:3031", origin=(-2400000.0, 1400000.0)) -> SynthConfig:
    """config_utm's shape from polar stereographic granules: WGS 84 / Antarctic
    Polar Stereographic (EPSG:3031) off the Antarctic Peninsula by default
    (about 66-68 S, 58-62 W), or NSIDC North (EPSG:3413, origin (-200000,
    -2000000): western Greenland)."""
    cfg = config_utm(scale, tiles_per_side, tile_px, grid, srs=srs, origin=origin)
    cfg.name = "STERE"
    return cfg


def subset(cfg: SynthConfig, tile_ids) -> SynthConfig:
    """The same config restricted to some tiles (for bounded CPU samples)."""
    tiles = [cfg.tiles[i] for i in tile_ids]
    pairs = [cfg.pairs[i] for i in tile_ids]
    return SynthConfig(cfg.name, cfg.granules, cfg.dst_srs, tiles, pairs, cfg.namespaces, cfg.scale,
                       cfg.palette, cfg.resample, cfg.mask, cfg.bbox, cfg.out_w, cfg.out_h)


def mpix(cfg: SynthConfig) -> float:
    return cfg.out_pixels / 1e6


# ---------------------------------------------------------------- C3
def config_c3(scale: float = 1.0, chunk_px: int = 1024, grid: int = 8, out_px: int = 16384,
              out_h: Optional[int] = None) -> SynthConfig:
    """WCS GetCoverage: EPSG:4326 float32 granules (8x8 over lon 112..154,
    lat -44..-10, 2048^2 each at full size) -> EPSG:3857 float32 bilinear
    mosaic of out_px^2, split in chunk_px^2 chunks (utils/config.go:55-56)."""
    n = max(8, int(round(2048 * scale)))
    lon0, lon1, lat0, lat1 = 112.0, 154.0, -44.0, -10.0
    gw, gh = (lon1 - lon0) / grid, (lat1 - lat0) / grid
    def make(k):
        j, i = divmod(k, grid)
        x0, y0 = lon0 + i * gw, lat1 - j * gh
        rx, ry = gw / n, gh / n
        lon = x0 + rx * (np.arange(n) + 0.5)
        lat = y0 - ry * (np.arange(n) + 0.5)
        idx = np.arange(n * n, dtype=np.uint64).reshape(n, n) + np.uint64((SEED0 + k) << 32)
        hh = splitmix64(idx)
        v = 200.0 + 50.0 * np.sin(lon[None, :] / 3.0) * np.cos(lat[:, None] / 2.0) + uniform01(hh)
        v = v.astype(np.float32)
        v[uniform01(splitmix64(hh)) < 0.01] = -9999.0
        poly = "POLYGON ((%g %g,%g %g,%g %g,%g %g,%g %g))" % (x0, y0, x0 + gw, y0, x0 + gw, y0 - gh, x0,
                                                              y0 - gh, x0, y0)
        return SynthGranule(v, [x0, rx, 0.0, y0, 0.0, -ry], "EPSG:4326", -9999.0, 1577836800.0, poly)

    granules = _pmap(make, range(grid * grid))
    mx0, my0 = merc_fwd(lon0, lat0)
    mx1, my1 = merc_fwd(lon1, lat1)
    bbox = (float(mx0), float(my0), float(mx1), float(my1))
    from .coverage import chunk_requests   # the reference's chunking, ows.go:817-831
    out_h = out_px if out_h is None else out_h
    chunks = chunk_requests(bbox, out_px, out_h, chunk_px, chunk_px)
    tiles = [(c.bbox, c.width, c.height) for c in chunks]
    cfg = SynthConfig("C3", granules, "EPSG:3857", tiles, [], [""], (0.0, 1.0, 0.0, 0), None, resample=1,
                      bbox=bbox, out_w=out_px, out_h=out_h)
    cfg.pairs = [cfg.index_chunk(bb) for (bb, _, _) in tiles]
    return cfg


# ---------------------------------------------------------------- C5
MODIS_T = 1111950.5197665
MODIS_X0, MODIS_Y0 = -20015109.354, 10007554.677


def _webmerc_tile_bbox(z, x, y):
    n = 2 ** z
    span = 2 * math.pi * WEBMERC_A
    x0 = -math.pi * WEBMERC_A + x * span / n
    y1 = math.pi * WEBMERC_A - y * span / n
    return (x0, y1 - span / n, x0 + span / n, y1)


def config_c5(scale: float = 1.0, dates: int = 4, h_range=(25, 33), v_range=(8, 16), zooms=((4, 11, 8, 4), (5, 22, 16, 8)),
              tile_px: int = 512) -> SynthConfig:
    """Zoomed-out MODIS sinusoidal -> EPSG:3857 overview tiles: int16 data +
    uint8 QA granules (mask value "00000001", not inclusive), overview
    pyramids /2 down to 75^2 at full size, grey byte scaling (clip 10000)."""
    n = max(16, int(round(2400 * scale)))
    px = MODIS_T / n
    keys = [(d, v, h) for d in range(dates) for v in range(*v_range) for h in range(*h_range)]

    def make(item):
        k, (d, v, h) = item
        x0 = MODIS_X0 + h * MODIS_T
        y0 = MODIS_Y0 - v * MODIS_T
        idx = np.arange(n * n, dtype=np.uint64).reshape(n, n) + np.uint64((SEED0 + k) << 32)
        hh = splitmix64(idx)
        data = (hh % np.uint64(10000)).astype(np.int16)
        nb = (n + 31) // 32
        bidx = np.arange(nb * nb, dtype=np.uint64) + np.uint64(((SEED0 + k) << 32) | 0x0A000000)
        blk = (uniform01(splitmix64(bidx)) < 0.15).reshape(nb, nb)
        qa = np.repeat(np.repeat(blk, 32, 0), 32, 1)[:n, :n].astype(np.uint8)
        qa |= (((hh >> np.uint64(20)) & np.uint64(0x7E)).astype(np.uint8))  # other bits noise
        ovr_d, ovr_q = [], []
        lvl = 1
        while n // (2 ** lvl) >= max(4, int(round(75 * scale))):
            s = 2 ** lvl
            ovr_d.append(np.ascontiguousarray(data[::s, ::s][: n // s, : n // s]))
            ovr_q.append(np.ascontiguousarray(qa[::s, ::s][: n // s, : n // s]))
            lvl += 1
        poly = "MODIS h%02dv%02d" % (h, v)
        ts = 1577836800.0 + 8 * 86400.0 * d
        gt = [x0, px, 0.0, y0, 0.0, -px]
        return (SynthGranule(data, gt, "MODIS", -28672.0, ts, poly, "", ovr_d),
                SynthGranule(qa, gt, "MODIS", 255.0, ts, poly, "qa", ovr_q))

    granules = [g for pair in _pmap(make, enumerate(keys)) for g in pair]
    tiles = []
    for (z, x0t, y0t, cnt) in zooms:
        for yy in range(y0t, y0t + cnt):
            for xx in range(x0t, x0t + cnt):
                tiles.append((_webmerc_tile_bbox(z, xx, yy), tile_px, tile_px))
    pairs = _index_pairs(granules, tiles)
    return SynthConfig("C5", granules, "EPSG:3857", tiles, pairs, [""], (0.0, 0.0, 10000.0, 0), None,
                       mask=dict(id="qa", value="00000001", inclusive=False))


# ---------------------------------------------------------------- C4 drill
def star_polygon(cx, cy, r, k=12, seed=0):
    rng = np.random.default_rng(seed)
    ang = np.linspace(0, 2 * np.pi, 2 * k, endpoint=False) + rng.uniform(0, np.pi / k)
    rad = np.where(np.arange(2 * k) % 2 == 0, r, r * 0.5)
    return np.stack([cx + rad * np.cos(ang), cy + rad * np.sin(ang)], 1)


def _point_in_poly(px, py, poly):
    inside = np.zeros(px.shape, bool)
    n = len(poly)
    for i in range(n):
        x1, y1 = poly[i]
        x2, y2 = poly[(i + 1) % n]
        cond = ((y1 > py) != (y2 > py)) & (px < (x2 - x1) * (py - y1) / (y2 - y1 + 1e-300) + x1)
        inside ^= cond
    return inside


def drill_mask(poly: np.ndarray, x0: int, y0: int, w: int, h: int) -> np.ndarray:
    yy, xx = np.mgrid[0:h, 0:w]
    cx = x0 + xx + 0.5
    cy = y0 + yy + 0.5
    m = _point_in_poly(cx, cy, poly)
    # ALL_TOUCHED: also pixels an edge passes through (sampled along edges)
    n = len(poly)
    for i in range(n):
        a, b = poly[i], poly[(i + 1) % n]
        L = int(np.ceil(np.hypot(*(b - a)) * 4)) + 2
        t = np.linspace(0, 1, L)
        ex = np.floor(a[0] + t * (b[0] - a[0])).astype(int) - x0
        ey = np.floor(a[1] + t * (b[1] - a[1])).astype(int) - y0
        ok = (ex >= 0) & (ex < w) & (ey >= 0) & (ey < h)
        m[ey[ok], ex[ok]] = True
    return np.where(m, 255, 0).astype(np.uint8)


@dataclass
class DrillConfig:
    bands: np.ndarray            # (n_bands, ysize, xsize) float32 (host)
    nodata: float
    windows: List[Tuple[int, int, int, int]]
    masks: List[np.ndarray]
    geometries: Optional[List[str]] = None   # the polygons as WGS84 GeoJSON (C4_GT grid)
    geot: Optional[List[float]] = None


C4_GT = [130.0, 0.01, 0.0, -20.0, 0.0, -0.01]   # EPSG:4326, 0.01 deg, origin (130, -20)


def c4_band(t: int, size: int, n_bands: int = 365) -> np.ndarray:
    """Slice t of the C4 time stack: 0.2 + 0.1 sin(2 pi t / 365) +
    U(0, 0.05) per (pixel, slice), nodata -9999 at 5 % of the (pixel, slice)
    cells, float32.  One splitmix64 draw per cell: its top 53 bits give the
    uniform, its low 16 bits the nodata test."""
    base = np.float32(0.2 + 0.1 * math.sin(2 * math.pi * t / 365.0))
    idx = np.arange(size * size, dtype=np.uint64) + np.uint64((SEED0 + 0x4C4) << 32) + \
        np.uint64(t) * np.uint64(size * size)
    u = splitmix64(idx)
    v = (uniform01(u) * 0.05).astype(np.float32) + base
    v[(u & np.uint64(0xFFFF)) < np.uint64(3277)] = np.float32(-9999.0)   # 3277 / 65536 = 5.0 %
    return v.reshape(size, size)


def pixel_polygon_geojson(poly: np.ndarray, gt: Sequence[float]) -> str:
    """A closed GeoJSON Polygon of pixel-space vertices mapped through `gt`."""
    lon = gt[0] + poly[:, 0] * gt[1]
    lat = gt[3] + poly[:, 1] * gt[5]
    ring = [[float(a), float(b)] for a, b in zip(lon, lat)]
    ring.append(ring[0])
    return json.dumps({"type": "Feature", "properties": {},
                       "geometry": {"type": "Polygon", "coordinates": [ring]}})


def c4_polygons(size: int = 2048, n_polys: int = 1000, rmin=10.0, rmax=100.0, seed: int = 4):
    """The C4 star polygons: (test-generator windows, masks, GeoJSON on C4_GT)."""
    rng = np.random.default_rng(seed)
    wins, masks, geoms = [], [], []
    for p in range(n_polys):
        r = rng.uniform(rmin, rmax)
        cx, cy = rng.uniform(r, size - r), rng.uniform(r, size - r)
        poly = star_polygon(cx, cy, r, seed=p)
        xmin, ymin = np.floor(poly.min(0)).astype(int)
        xmax, ymax = np.floor(poly.max(0)).astype(int)
        xmin, ymin = max(0, xmin), max(0, ymin)
        w = min(size, xmax + 1) - xmin
        h = min(size, ymax + 1) - ymin
        wins.append((int(xmin), int(ymin), int(w), int(h)))
        masks.append(drill_mask(poly, xmin, ymin, w, h))
        geoms.append(pixel_polygon_geojson(poly, C4_GT))
    return wins, masks, geoms


def config_c4(n_bands: int = 365, size: int = 2048, n_polys: int = 1000, rmin=10.0, rmax=100.0,
              seed: int = 4) -> DrillConfig:
    """WPS drill: n_bands daily float32 slices of size^2 (c4_band) + star
    polygons (12 points, radius U[rmin, rmax] px, centres uniform over the
    grid) as GeoJSON on C4_GT; windows / masks here are the test generator's
    (point-in-polygon + sampled edges) -- the product's ALL_TOUCHED masks come
    from drill.drill_dataset(cfg.geometries, ...)."""
    bands = np.empty((n_bands, size, size), np.float32)

    def fill(b):
        bands[b] = c4_band(b, size, n_bands)

    _pmap(fill, range(n_bands))
    wins, masks, geoms = c4_polygons(size, n_polys, rmin, rmax, seed)
    return DrillConfig(bands, -9999.0, wins, masks, geoms, list(C4_GT))
