"""GPU parity of the band-kernel variants on ragged batches: small C2 (int16,
palette) batches whose tiles have mixed sizes (ragged last 64-column slot,
partial 512-column blocks, tiles narrower than one slot) and a C5 batch
(masks, overviews, two zoom levels), rendered by the product library and --
in one child process per setting -- by the A/B build (libgskyhip_ab.so, the
only build that reads GSKYHIP_* knobs) with every shape forced: rows per wave
1 / 4 / 8, the single-entry prefetch path on and off, masked stacks at one or
four rows per wave.  The small batches never reach the size thresholds
that pick those shapes in production, so without the knobs these code paths
would only run in the full-size tests.  Measurements: profiles/r03*_ab_*.jsonl."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from gsky_amd import synth

from .helpers import gpu_batch, oracle_render

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _mixed_c2():
    cfg = synth.config_c2(scale=0.1, tiles_per_side=4, tile_px=256)
    sizes = [(256, 256), (200, 256), (77, 130), (256, 255), (9, 5), (129, 64)]
    cfg.tiles = [(bb, *sizes[i % len(sizes)]) for i, (bb, _, _) in enumerate(cfg.tiles)]
    return cfg


def _c5():
    return synth.config_c5(scale=0.05, dates=2, zooms=((4, 11, 8, 2), (5, 22, 16, 3)), tile_px=128)


def _differing_tiles(cfg, got, exp):
    return [t for t, (_, w, h) in enumerate(cfg.tiles) if not np.array_equal(got[t, :h, :w], exp[t, :h, :w])]


@pytest.fixture(scope="module")
def cases(oracle):
    import gsky_amd
    out = []
    for name, cfg, pal in [("c2", _mixed_c2(), True), ("c5", _c5(), False)]:
        b = gpu_batch(cfg)
        sp = gsky_amd.ScaleParams(*cfg.scale)
        p = gsky_amd.Palette(cfg.palette, True) if pal and cfg.palette else None
        out.append((name, cfg, b, sp, p, oracle_render(oracle, cfg)))
    return out


def test_band_kernels_match_oracle(cases):
    for name, cfg, b, sp, pal, exp in cases:
        got = b.render(sp, pal).cpu().numpy()
        assert b.status() == 0
        assert _differing_tiles(cfg, got, exp) == [], name


CHILD = r"""
import json, sys
import numpy as np
sys.path.insert(0, %(root)r)
import gsky_amd
from gsky_amd import synth
from oracle import oracle as O
from tests.helpers import gpu_batch, oracle_render
from tests.test_gpu_variants import _mixed_c2, _c5, _differing_tiles
res = {}
for name, cfg, pal in [("c2", _mixed_c2(), True), ("c5", _c5(), False)]:
    b = gpu_batch(cfg)
    p = gsky_amd.Palette(cfg.palette, True) if pal and cfg.palette else None
    got = b.render(gsky_amd.ScaleParams(*cfg.scale), p).cpu().numpy()
    res[name] = {"status": b.status(), "differ": _differing_tiles(cfg, got, oracle_render(O, cfg))}
print(json.dumps(res))
"""


@pytest.mark.parametrize("knobs", [
    {"GSKYHIP_NN_RPW": "1"}, {"GSKYHIP_NN_RPW": "4"},
    {"GSKYHIP_NN_RPW": "8", "GSKYHIP_NN_ONE": "1"}, {"GSKYHIP_NN_RPW": "8", "GSKYHIP_NN_ONE": "0"},
    {"GSKYHIP_NN_MASK_RPW": "1"}, {"GSKYHIP_NN_MASK_RPW": "4"},
])
def test_ab_build_variants_match_oracle(knobs):
    lib = os.path.join(ROOT, "gsky_amd", "libgskyhip_ab.so")
    if not os.path.exists(lib):
        pytest.skip("A/B build not present (make -C gsky_amd/csrc ab)")
    env = dict(os.environ, GSKYHIP_LIB="ab", **knobs)
    p = subprocess.run([sys.executable, "-c", CHILD % {"root": ROOT}], env=env, capture_output=True, text=True,
                       timeout=240, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-3000:]
    res = json.loads(p.stdout.strip().splitlines()[-1])
    for name, r in res.items():
        assert r["status"] == 0 and r["differ"] == [], (knobs, name, r)
