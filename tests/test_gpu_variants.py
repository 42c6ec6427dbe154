"""GPU parity of the band-kernel variants behind the A/B knobs (render_lds.hip
reads them at every launch): each lane layout, occupancy build, Scale LUT and
the bilinear shapes must stay bit-identical to the oracle, so that the
measurements in profiles/r02z*_ab_*.jsonl compare equal work and a knob can
become the default without a new parity argument.  Small C2 (int16, palette),
C5 (masks, overviews) and C3 (bilinear float canvas) batches, mixed tile
sizes for the strided layouts' column bounds.
"""
import os

import numpy as np
import pytest

from gsky_amd import synth

from .helpers import gpu_batch, oracle_render

pytestmark = pytest.mark.gpu

KNOBS = ("GSKYHIP_NN_SHAPE", "GSKYHIP_NN_STRIDE", "GSKYHIP_NN_LUT", "GSKYHIP_NN_GEN", "GSKYHIP_NN_RPW",
         "GSKYHIP_BIL_KERNEL")

# (label, environment): the defaults first, then the round's A/B variants
NN_VARIANTS = [
    ("default", {}),
    ("4x2_consecutive", {"GSKYHIP_NN_SHAPE": "3", "GSKYHIP_NN_STRIDE": "0"}),
    ("4x2_strided", {"GSKYHIP_NN_SHAPE": "3", "GSKYHIP_NN_STRIDE": "1"}),
    ("4x1_w8_mask4x2", {"GSKYHIP_NN_SHAPE": "4", "GSKYHIP_NN_STRIDE": "1"}),
    ("4x2_strided_lut", {"GSKYHIP_NN_SHAPE": "3", "GSKYHIP_NN_STRIDE": "1", "GSKYHIP_NN_LUT": "1"}),
    ("4x2_strided_cached_stores", {"GSKYHIP_NN_SHAPE": "3", "GSKYHIP_NN_STRIDE": "2"}),
    ("4x2_lds_out", {"GSKYHIP_NN_SHAPE": "3", "GSKYHIP_NN_STRIDE": "4"}),
    ("4x4_strided", {"GSKYHIP_NN_SHAPE": "0", "GSKYHIP_NN_STRIDE": "1"}),
    ("8x2_strided", {"GSKYHIP_NN_SHAPE": "2", "GSKYHIP_NN_STRIDE": "1"}),
    ("4x2_strided_rpw8", {"GSKYHIP_NN_SHAPE": "3", "GSKYHIP_NN_STRIDE": "1", "GSKYHIP_NN_RPW": "8"}),
    ("gen3", {"GSKYHIP_NN_GEN": "3"}),
]


class _env:
    def __init__(self, env):
        self.env = env

    def __enter__(self):
        self.saved = {k: os.environ.get(k) for k in KNOBS}
        for k in KNOBS:
            os.environ.pop(k, None)
        os.environ.update(self.env)

    def __exit__(self, *exc):
        for k, v in self.saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


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


@pytest.mark.parametrize("label,env", NN_VARIANTS, ids=[v[0] for v in NN_VARIANTS])
def test_nn_variant_matches_oracle(cases, label, env):
    with _env(env):
        for name, cfg, b, sp, pal, exp in cases:
            got = b.render(sp, pal).cpu().numpy()
            assert b.status() == 0
            for t, (_, w, h) in enumerate(cfg.tiles):
                assert np.array_equal(got[t, :h, :w], exp[t, :h, :w]), (label, name, t)


@pytest.mark.parametrize("k", ["1", "2", "3", "4", "5", "6"])
def test_bilinear_variant_matches_default(oracle, k):
    """Every render_bil_kernel shape gives the default's float canvas bit for
    bit (the default itself is held to the oracle by test_gpu_parity /
    test_gpu_full)."""
    import torch

    import gsky_amd
    cfg = synth.config_c3(scale=0.05, chunk_px=96, out_px=288, grid=3)
    b = gpu_batch(cfg)
    sp = gsky_amd.ScaleParams(*cfg.scale)
    outs = []
    for env in ({}, {"GSKYHIP_BIL_KERNEL": k}):
        with _env(env):
            _, cv = b.render(sp, resample=1, canvas=True)
            torch.cuda.synchronize()
            assert b.status() == 0
            outs.append(cv.clone())
    assert torch.equal(outs[0], outs[1])
    assert (outs[0] != 0).any()
