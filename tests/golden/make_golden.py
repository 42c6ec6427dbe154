#!/usr/bin/env python3
"""Generates the committed golden fixtures under tests/golden/ (TEST
INFRASTRUCTURE: the expected outputs come from the CPU oracle, oracle/).

Each fixture is a small .npz (no pickles) holding the case parameters, a
checksum of the synthetic inputs (synth.py, splitmix64) so that
a drift of the input generator is detected instead of silently re-baselined,
and the oracle's expected output.  The inputs themselves are regenerated from
synth.py (deterministic), which keeps the fixtures a few hundred KB.

  python tests/golden/make_golden.py        # rewrites every fixture

Cases (the reference paths they pin):
  render_c1  -- warp_operation_fast (warp.go:82-382) 4326->3857 f32 + Scale
                (raster_scaler.go:334) grey RGBA (ogc_encoders.go:82-134)
  render_c2  -- 16 Albers int16 granules, time-ordered merge
                (tile_merger.go:281-312), palette (palette.go:27)
  render_c5  -- MODIS sinusoidal, overviews (warp.go:156-198), QA mask
                (tile_merger.go:314-445)
  drill_c4   -- readData mean/count (drill.go:90-227)
  scale_kats -- Scale over every type with auto mode (raster_scaler.go:30-346)
"""
from __future__ import annotations

import hashlib
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

from gsky_amd import synth  # noqa: E402

RENDER_CASES = {
    "render_c1": lambda: synth.config_c1(scale=0.25),
    "render_c2": lambda: synth.config_c2(scale=0.05, tiles_per_side=3, tile_px=96),
    "render_c5": lambda: synth.config_c5(scale=0.05, dates=2, zooms=((4, 11, 8, 2),), tile_px=96),
}
DRILL_CASE = dict(n_bands=9, size=96, n_polys=6, rmin=3, rmax=20)
SCALE_PARAMS = [(0, 0, 0), (0, 0, 1000), (1, 1, 1000), (3, 2, 2), (-5, 0.5, 300), (0, 3.5, 0)]
SCALE_TYPES = ["uint8", "int8", "int16", "uint16", "float32"]


def input_digest(cfg) -> str:
    h = hashlib.sha256()
    for g in cfg.granules:
        h.update(np.ascontiguousarray(g.data).tobytes())
        h.update(np.asarray(g.geot, dtype=np.float64).tobytes())
        for o in g.overviews:
            h.update(np.ascontiguousarray(o).tobytes())
    for (bb, w, hh) in cfg.tiles:
        h.update(np.asarray(list(bb) + [w, hh], dtype=np.float64).tobytes())
    return h.hexdigest()


def drill_digest(dc) -> str:
    h = hashlib.sha256(dc.bands.tobytes())
    for m in dc.masks:
        h.update(m.tobytes())
    h.update(np.asarray(dc.windows, dtype=np.int64).tobytes())
    return h.hexdigest()


def scale_input(tname: str, n: int = 4099):
    rng = np.random.default_rng(1234 + SCALE_TYPES.index(tname))
    if tname == "float32":
        v = rng.normal(300, 400, n).astype(np.float32)
        v[rng.random(n) < 0.05] = -9999.0
        return v, -9999.0
    info = np.iinfo(np.dtype(tname))
    v = rng.integers(info.min, int(info.max) + 1, n).astype(tname)
    return v, float(v[17])


def expected_render(O, cfg):
    from tests.helpers import oracle_render
    return oracle_render(O, cfg, n_threads=4)


def expected_drill(O, dc):
    vals, cnts = [], []
    for p, (x0, y0, w, h) in enumerate(dc.windows):
        v, c = O.drill_read_data(dc.bands[:, y0:y0 + h, x0:x0 + w], dc.masks[p], dc.nodata, -1e30, 1e30, 0, 1)
        vals.append(v)
        cnts.append(c)
    return np.stack(vals), np.stack(cnts)


def main():
    from oracle import oracle as O
    O.lib()
    for name, mk in RENDER_CASES.items():
        cfg = mk()
        exp = expected_render(O, cfg)
        np.savez_compressed(os.path.join(HERE, name + ".npz"), expected=exp,
                            digest=np.array(input_digest(cfg)))
        print(name, exp.shape, "valid px %.3f" % (exp[..., 3] > 0).mean())
    dc = synth.config_c4(**DRILL_CASE)
    v, c = expected_drill(O, dc)
    np.savez_compressed(os.path.join(HERE, "drill_c4.npz"), values=v, counts=c, digest=np.array(drill_digest(dc)))
    print("drill_c4", v.shape)
    out = {}
    for t in SCALE_TYPES:
        d, nd = scale_input(t)
        for k, sp in enumerate(SCALE_PARAMS):
            out["%s_%d" % (t, k)] = O.scale(d, nd, *sp)
    np.savez_compressed(os.path.join(HERE, "scale_kats.npz"), **out)
    print("scale_kats", len(out))


if __name__ == "__main__":
    main()
