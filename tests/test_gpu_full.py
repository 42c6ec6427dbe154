"""Full-size parity: every BASELINE.json config at its benchmark size, MI355X
path (libgskyhip.so) against the CPU oracle on the same synthetic inputs.

Bars (north_star):
  C2, C5 (NN warp + time-ordered merge + masks + scale + palette/grey):
      100 % of RGBA pixels identical -- no pixel is excepted;
  C3 (bilinear, typed float canvas): identical nodata mask and EVERY valid
      pixel within 1e-4 relative;
  C4 (drill through the product: GeoJSON polygons -> windows + ALL_TOUCHED
      masks rasterized on the GPU -> readData): windows and masks identical to
      the oracle's, counts identical and means bit-exact for all 1000
      polygons x 365 slices (reference order), deciles of a 100-polygon sample
      equal as float32.
Comparisons of the big outputs run on the GPU (the oracle's arrays are
uploaded), so a 4.3 GB RGBA batch compares in well under a second.
"""
import os
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

from gsky_amd import synth

from .helpers import gpu_batch, oracle_render

pytestmark = pytest.mark.gpu

THREADS = max(1, min(16, os.cpu_count() or 1))   # the box's CPU share is 16 cores


def _mismatch_report(got, exp, limit=8):
    """(count of differing RGBA pixels, first few as (tile, row, col, got, exp))."""
    import torch
    g = torch.as_tensor(got, device="cuda")
    e = torch.from_numpy(exp).to("cuda")
    bad = (g != e).any(dim=-1)
    n = int(bad.sum().item())
    first = []
    if n:
        idx = torch.nonzero(bad)[:limit].cpu().numpy()
        for t, r, c in idx:
            first.append((int(t), int(r), int(c), got[t, r, c].tolist() if isinstance(got, np.ndarray)
                          else g[t, r, c].tolist(), exp[t, r, c].tolist()))
    return n, first


def test_c2_full_identical(gpu, oracle):
    """C2: 4096 x 512^2 tiles from 16 EPSG:3577 int16 4000^2 granules."""
    import gsky_amd
    cfg = synth.config_c2()
    b = gpu_batch(cfg)
    got = b.render(gsky_amd.ScaleParams(*cfg.scale), gsky_amd.Palette(cfg.palette, True))
    assert b.status() == 0
    exp = oracle_render(oracle, cfg, n_threads=THREADS)
    assert got.shape == exp.shape == (4096, 512, 512, 4)
    n, first = _mismatch_report(got, exp)
    assert n == 0, "C2: %d of %d pixels differ, e.g. %s" % (n, exp.shape[0] * 512 * 512, first)
    assert (exp[..., 3] > 0).mean() > 0.5


def test_c2_full_pipelined_identical(gpu, oracle):
    """C2 as bench.py times it: 4 chunks on 2 streams (PipelinedBatch) --
    every RGBA pixel identical to the oracle, like the one-batch path."""
    import gsky_amd
    cfg = synth.config_c2()
    b = gpu_batch(cfg, chunks=4)
    got = b.render(gsky_amd.ScaleParams(*cfg.scale), gsky_amd.Palette(cfg.palette, True))
    assert b.status() == 0
    exp = oracle_render(oracle, cfg, n_threads=THREADS)
    n, first = _mismatch_report(got, exp)
    assert n == 0, "C2 pipelined: %d pixels differ, e.g. %s" % (n, first)


def test_c5_full_identical(gpu, oracle):
    """C5: 80 x 512^2 overview tiles over 256 MODIS granules + QA masks."""
    import gsky_amd
    cfg = synth.config_c5()
    b = gpu_batch(cfg)
    got = b.render(gsky_amd.ScaleParams(*cfg.scale))
    assert b.status() == 0
    exp = oracle_render(oracle, cfg, n_threads=THREADS)
    n, first = _mismatch_report(got, exp)
    assert n == 0, "C5: %d pixels differ, e.g. %s" % (n, first)
    assert (exp[..., 3] > 0).mean() > 0.1


def test_c3_full_bilinear_canvas(gpu, oracle):
    """C3 at N=1: the whole 16384^2 float32 bilinear coverage (256 chunks of
    1024^2 from 64 EPSG:4326 2048^2 granules) against the oracle's canvases."""
    import torch

    from gsky_amd import coverage
    cfg = synth.config_c3()
    full, _ = coverage.render_coverage(cfg, cfg.out_w, cfg.out_h, device=gpu)
    _, cv, created = oracle_render(oracle, cfg, n_threads=THREADS, canvas=True)
    assert created[:, 0].all()
    chunks = coverage.chunk_requests(cfg.bbox, cfg.out_w, cfg.out_h)
    mh = max(c.height for c in chunks)
    mw = max(c.width for c in chunks)
    canv = [torch.from_numpy(cv[i, 0].view(np.float32).reshape(mh, mw)[:c.height, :c.width])
            for i, c in enumerate(chunks)]
    exp = coverage.place_chunks(canv, chunks, 0, cfg.out_h, cfg.out_w, device=gpu)
    del cv, canv
    nod_e, nod_g = exp == -9999.0, full == -9999.0
    assert torch.equal(nod_e, nod_g), "nodata masks differ at %d pixels" % int((nod_e != nod_g).sum())
    v = ~nod_e
    assert v.float().mean().item() > 0.5
    e64, g64 = exp[v].double(), full[v].double()
    rel = ((g64 - e64).abs() / e64.abs().clamp_min(1e-30)).max().item()
    assert rel <= 1e-4, rel


def _drill_oracle(oracle, dc, clip, pc, strides):
    def one(p):
        x0, y0, w, h = dc.windows[p]
        sub = np.ascontiguousarray(dc.bands[:, y0:y0 + h, x0:x0 + w])
        return oracle.drill_read_data(sub, dc.masks[p], dc.nodata, clip[0], clip[1], pc, strides)
    with ThreadPoolExecutor(THREADS) as ex:
        return list(ex.map(one, range(len(dc.windows))))


@pytest.fixture(scope="module")
def c4(gpu, oracle):
    """The C4 stack and polygons, the product's windows / masks for the GeoJSON
    polygons (GPU rasterizer), checked against the oracle's descriptors; the
    config's windows / masks are replaced by the product's."""
    from gsky_amd import drill
    dc = synth.config_c4()
    size = dc.bands.shape[1]
    mb, st = drill.drill_dataset(dc.geometries, "EPSG:4326", dc.geot, size, size, device=gpu)
    assert (st == 0).all()
    win, off, buf = mb.win.cpu().numpy(), mb.mask_off.cpu().numpy(), mb.masks.cpu().numpy()

    def one(p):
        ew, em = oracle.drill_descriptor(dc.geometries[p], "EPSG:4326", dc.geot, size, size)
        w, h = int(win[p][2]), int(win[p][3])
        return tuple(win[p]) == ew and np.array_equal(buf[off[p]:off[p] + w * h].reshape(h, w), em)
    with ThreadPoolExecutor(THREADS) as ex:
        same = list(ex.map(one, range(len(dc.geometries))))
    assert all(same), "product windows / masks differ from the oracle for %d polygons" % same.count(False)
    dc.windows = [tuple(int(v) for v in w) for w in win]
    dc.masks = [buf[off[p]:off[p] + w * h].reshape(h, w) for p, (_, _, w, h) in enumerate(dc.windows)]
    dc.mb = mb
    return dc


def test_c4_full_drill_bit_exact(gpu, oracle, c4):
    """C4: 1000 polygons x 365 daily float32 slices, mean mode, clip
    +-MaxFloat32 (ows.go:1373-1381), reference summation order, over the
    product's masks."""
    import torch

    from gsky_amd import drill
    clip = (-3.4028234663852886e38, 3.4028234663852886e38)
    st = drill.DrillStack(torch.from_numpy(c4.bands), c4.nodata, gpu)
    vals, cnts = drill.read_data(st, c4.mb, clip[0], clip[1], 0, 1)
    vals, cnts = vals.cpu().numpy(), cnts.cpu().numpy()
    del st
    exp = _drill_oracle(oracle, c4, clip, 0, 1)
    bad = [p for p, (ev, ec) in enumerate(exp)
           if not (np.array_equal(cnts[p], ec) and np.array_equal(vals[p].view(np.uint64), ev.view(np.uint64)))]
    assert not bad, "C4: %d polygons differ (first %s)" % (len(bad), bad[:5])
    assert sum(int(ec.sum()) for _, ec in exp) > 1e8


def test_c4_full_deciles_sample(gpu, oracle, c4):
    """readData with decileCount 9 over all 1000 polygons x 365 slices on the
    GPU (radix selection); 100 polygons checked against numpy's sort of the
    same in-mask, non-nodata values (the oracle's computeDeciles picks)."""
    import torch

    from gsky_amd import drill
    clip = (-3.4028234663852886e38, 3.4028234663852886e38)
    st = drill.DrillStack(torch.from_numpy(c4.bands), c4.nodata, gpu)
    vals, cnts = drill.read_data(st, c4.mb, clip[0], clip[1], decile_count=9)
    vals, cnts = vals.cpu().numpy(), cnts.cpu().numpy()
    del st
    nd = np.float32(c4.nodata)

    def one(p):
        x0, y0, w, h = c4.windows[p]
        sub = c4.bands[:, y0:y0 + h, x0:x0 + w].reshape(c4.bands.shape[0], -1)
        m = c4.masks[p].reshape(-1) == 255
        for b in range(c4.bands.shape[0]):
            v = sub[b][m]
            v = np.sort(v[v != nd])
            if cnts[p, b, 0] == 0:
                if vals[p, b, 1:].any():
                    return False
                continue
            step = len(v) // 10
            exp = np.zeros(9, np.float32)
            if step > 0:
                even = len(v) % 10 == 0
                for i in range(9):
                    j = (i + 1) * step
                    exp[i] = np.float32((v[j] + v[j + 1]) / np.float32(2.0)) if even else v[j]
            else:
                exp = oracle.compute_deciles(sub[b], m.astype(np.uint8) * 255, c4.nodata, 9)
            if not np.array_equal(vals[p, b, 1:].astype(np.float32), exp):
                return False
        return True
    with ThreadPoolExecutor(THREADS) as ex:
        ok = list(ex.map(one, range(0, len(c4.windows), 10)))
    assert all(ok), "deciles differ for %d of %d sampled polygons" % (ok.count(False), len(ok))


def test_c4_full_drill_wave_split(gpu, oracle, c4):
    """C4 in the wave-split mode: counts exact, means within 1e-5 relative."""
    import torch

    from gsky_amd import drill
    clip = (-3.4028234663852886e38, 3.4028234663852886e38)
    st = drill.DrillStack(torch.from_numpy(c4.bands), c4.nodata, gpu)
    vals, cnts = drill.read_data(st, c4.mb, clip[0], clip[1], mode=drill.WAVE_SPLIT)
    vals, cnts = vals.cpu().numpy(), cnts.cpu().numpy()
    del st
    exp = _drill_oracle(oracle, c4, clip, 0, 1)
    worst = 0.0
    for p, (ev, ec) in enumerate(exp):
        assert np.array_equal(cnts[p], ec), p
        ok = ec > 0
        if ok.any():
            worst = max(worst, float((np.abs(vals[p][ok] - ev[ok]) / np.abs(ev[ok])).max()))
    assert worst <= 1e-5, worst
