"""GPU parity of the typed band kernels on ragged batches: small C2 (int16,
palette) batches whose tiles have mixed sizes (ragged last 64-column slot,
partial 512-column blocks, tiles narrower than one slot) and a C5 batch
(masks, overviews, two zoom levels).  Round 3 removed the round-2 A/B
variants of the band kernels from the library; their measurements stay in
profiles/r02*_ab_*.jsonl.
"""
import numpy as np
import pytest

from gsky_amd import synth

from .helpers import gpu_batch, oracle_render

pytestmark = pytest.mark.gpu


def _mixed_c2():
    cfg = synth.config_c2(scale=0.1, tiles_per_side=4, tile_px=256)
    sizes = [(256, 256), (200, 256), (77, 130), (256, 255), (9, 5), (129, 64)]
    cfg.tiles = [(bb, *sizes[i % len(sizes)]) for i, (bb, _, _) in enumerate(cfg.tiles)]
    return cfg


@pytest.fixture(scope="module")
def cases(oracle):
    import gsky_amd
    out = []
    for name, cfg, pal in [("c2", _mixed_c2(), True),
                           ("c5", synth.config_c5(scale=0.05, dates=2, zooms=((4, 11, 8, 2), (5, 22, 16, 3)),
                                                  tile_px=128), False)]:
        b = gpu_batch(cfg)
        sp = gsky_amd.ScaleParams(*cfg.scale)
        p = gsky_amd.Palette(cfg.palette, True) if pal and cfg.palette else None
        out.append((name, cfg, b, sp, p, oracle_render(oracle, cfg)))
    return out


def test_band_kernels_match_oracle(cases):
    for name, cfg, b, sp, pal, exp in cases:
        got = b.render(sp, pal).cpu().numpy()
        assert b.status() == 0
        for t, (_, w, h) in enumerate(cfg.tiles):
            assert np.array_equal(got[t, :h, :w], exp[t, :h, :w]), (name, t)
