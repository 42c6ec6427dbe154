"""HIP-graph replay of a render (gsky_amd.RenderGraph): the captured launch
sequence gives the eager render's RGBA bit for bit, and after
TileBatch.set_tiles() (new requests of the same shape) the replay renders the
new tiles exactly as the oracle does."""
import numpy as np
import pytest

from gsky_amd import synth

from .helpers import gpu_batch, oracle_render

pytestmark = pytest.mark.gpu


def _shifted(cfg, dx_px, dy_px):
    """The same tiles moved by a fraction of a pixel (same granule lists)."""
    tiles = []
    for (x0, y0, x1, y1), w, h in cfg.tiles:
        rx, ry = (x1 - x0) / w, (y1 - y0) / h
        tiles.append(((x0 + dx_px * rx, y0 + dy_px * ry, x1 + dx_px * rx, y1 + dy_px * ry), w, h))
    return tiles


def test_graph_replay_matches_eager_and_oracle(oracle):
    import torch

    import gsky_amd
    cfg = synth.config_c2(scale=0.1, tiles_per_side=3, tile_px=128)
    b = gpu_batch(cfg)
    sp, pal = gsky_amd.ScaleParams(*cfg.scale), gsky_amd.Palette(cfg.palette, True)
    eager = b.render(sp, pal).clone()
    rg = b.graph(sp, pal)
    rg.out.fill_(7)   # the replay must write every pixel
    got = rg.replay()
    torch.cuda.synchronize()
    assert b.status() == 0
    assert torch.equal(got, eager)
    assert np.array_equal(got.cpu().numpy(), oracle_render(oracle, cfg))
    # new requests of the same shape: descriptors updated in HBM, graph replayed
    for dx, dy in [(0.37, -0.21), (5.5, 3.25)]:
        cfg.tiles = _shifted(cfg, dx, dy)
        b.set_tiles(cfg.tiles)
        got = rg.replay()
        torch.cuda.synchronize()
        assert b.status() == 0
        exp = oracle_render(oracle, cfg)
        assert np.array_equal(got.cpu().numpy(), exp), (dx, dy)
        assert (exp[..., 3] > 0).mean() > 0.2


def test_set_tiles_rejects_other_shapes():
    import gsky_amd
    cfg = synth.config_c2(scale=0.05, tiles_per_side=2, tile_px=64)
    b = gpu_batch(cfg)
    with pytest.raises(ValueError):
        b.set_tiles(cfg.tiles[:-1])
    with pytest.raises(ValueError):
        b.set_tiles([(bb, w + 1, h) for (bb, w, h) in cfg.tiles])
    assert isinstance(b.graph(gsky_amd.ScaleParams(*cfg.scale)), gsky_amd.RenderGraph)
