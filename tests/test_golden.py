"""Golden fixtures (tests/golden/, made by tests/golden/make_golden.py).

CPU: the synthetic inputs still hash to the digests the fixtures were made
from, and the oracle still reproduces every fixture bit for bit.
GPU: the MI355X path (libgskyhip.so through its C-ABI) against the same
fixtures -- render 100 % identical RGBA pixels (the bar is 1.0, stricter than
BASELINE.json north_star's 99.99 %), drill and scale bit-exact.
"""
import os

import numpy as np
import pytest

from gsky_amd import synth
from tests.golden import make_golden as G

from .helpers import gpu_batch, identity

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
NN_IDENTITY = 1.0   # every golden case is 100 % identical


def _load(name):
    return np.load(os.path.join(HERE, name + ".npz"), allow_pickle=False)


@pytest.mark.parametrize("name", sorted(G.RENDER_CASES))
def test_golden_render_oracle(oracle, name):
    f = _load(name)
    cfg = G.RENDER_CASES[name]()
    assert str(f["digest"]) == G.input_digest(cfg), "synthetic inputs drifted from the fixture"
    assert np.array_equal(G.expected_render(oracle, cfg), f["expected"])


def test_golden_drill_oracle(oracle):
    f = _load("drill_c4")
    dc = synth.config_c4(**G.DRILL_CASE)
    assert str(f["digest"]) == G.drill_digest(dc)
    v, c = G.expected_drill(oracle, dc)
    assert np.array_equal(v.view(np.uint64), f["values"].view(np.uint64))
    assert np.array_equal(c, f["counts"])


def test_golden_scale_oracle(oracle):
    f = _load("scale_kats")
    for t in G.SCALE_TYPES:
        d, nd = G.scale_input(t)
        for k, sp in enumerate(G.SCALE_PARAMS):
            assert np.array_equal(oracle.scale(d, nd, *sp), f["%s_%d" % (t, k)]), (t, sp)


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(G.RENDER_CASES))
def test_golden_render_gpu(gpu, name):
    import gsky_amd
    f = _load(name)
    cfg = G.RENDER_CASES[name]()
    b = gpu_batch(cfg, gpu)
    pal = gsky_amd.Palette(cfg.palette, True) if cfg.palette else None
    got = b.render(gsky_amd.ScaleParams(*cfg.scale), pal).cpu().numpy()
    assert b.status() == 0
    assert identity(got, f["expected"]) >= NN_IDENTITY


@pytest.mark.gpu
def test_golden_drill_gpu(gpu):
    import torch

    from gsky_amd import drill
    f = _load("drill_c4")
    dc = synth.config_c4(**G.DRILL_CASE)
    st = drill.DrillStack(torch.from_numpy(dc.bands), dc.nodata, gpu)
    win, off, masks = drill.pack_masks(dc.windows, dc.masks, gpu)
    vals, cnts = drill.read_data(st, win, off, masks, -1e30, 1e30, 0, 1)
    assert np.array_equal(cnts.cpu().numpy(), f["counts"])
    assert np.array_equal(vals.cpu().numpy().view(np.uint64), f["values"].view(np.uint64))


@pytest.mark.gpu
def test_golden_scale_gpu(gpu):
    import torch

    import gsky_amd
    f = _load("scale_kats")
    for t in G.SCALE_TYPES:
        d, nd = G.scale_input(t)
        for k, sp in enumerate(G.SCALE_PARAMS):
            got = gsky_amd.scale([torch.from_numpy(d).to(gpu)], [nd], gsky_amd.ScaleParams(*sp),
                                 ["SignedByte"] if t == "int8" else None)[0]
            assert np.array_equal(got.cpu().numpy(), f["%s_%d" % (t, k)]), (t, sp)
