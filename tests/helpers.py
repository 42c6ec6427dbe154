"""Shared test helpers: feed one synthetic config to both the oracle (CPU
checker) and the MI355X path, and compare."""
from __future__ import annotations

import numpy as np

from gsky_amd import synth
from gsky_amd.tiles import bbox_to_geot


def oracle_inputs(O, cfg: synth.SynthConfig):
    gr, crs, ts, ph, ns = [], [], [], [], []
    slots = list(cfg.namespaces)
    if cfg.mask and cfg.mask["id"] not in slots:
        slots.append(cfg.mask["id"])
    for g in cfg.granules:
        gr.append(O.make_granule(g.data, g.geot, g.nodata if g.nodata is not None else -1e10, g.overviews))
        crs.append(O.crs(g.srs))
        ts.append(g.timestamp)
        ph.append(O.fnv32a(g.polygon))
        ns.append(slots.index(g.namespace))
    geots = [bbox_to_geot(w, h, bb) for (bb, w, h) in cfg.tiles]
    mask_ns = slots.index(cfg.mask["id"]) if cfg.mask else -1
    return gr, crs, ts, ph, ns, geots, slots, mask_ns


def oracle_render(O, cfg: synth.SynthConfig, tile_ids=None, n_threads=8, canvas=False):
    """The oracle's rendering of a synth config: RGBA (n_tiles, max_h, max_w, 4),
    with canvas=True also (typed canvases, created flags)."""
    sub = synth.subset(cfg, tile_ids) if tile_ids is not None else cfg
    gr, crs, ts, ph, ns, geots, slots, mask_ns = oracle_inputs(O, sub)
    ramp = O.gradient_palette(sub.palette, True) if sub.palette else None
    return O.render_tiles(gr, crs, ts, ph, ns, O.crs(sub.dst_srs), geots, 0, 0, sub.pairs, sub.scale, ramp=ramp,
                          n_ns=len(slots), mask_ns=mask_ns,
                          mask_value=sub.mask["value"] if sub.mask else None,
                          mask_inclusive=bool(sub.mask["inclusive"]) if sub.mask else False,
                          resample=sub.resample, n_threads=n_threads,
                          sizes=[(w, h) for (_, w, h) in sub.tiles], canvas=canvas)


def gpu_batch(cfg: synth.SynthConfig, device="cuda", chunks: int = 0):
    """The config's tiles as one TileBatch, or (chunks > 0) a PipelinedBatch
    of that many chunks."""
    import torch

    from gsky_amd import GranuleSet, Mask, PipelinedBatch, TileBatch
    gs = GranuleSet(device)
    for g in cfg.granules:
        gs.add(torch.from_numpy(np.ascontiguousarray(g.data)), g.geot, g.srs, g.nodata,
               [torch.from_numpy(np.ascontiguousarray(o)) for o in g.overviews], g.timestamp, g.polygon,
               g.namespace)
    mask = Mask(cfg.mask["id"], cfg.mask.get("value", ""), cfg.mask.get("bit_tests", []),
                cfg.mask.get("inclusive", False)) if cfg.mask else None
    if chunks > 0:
        return PipelinedBatch(gs, cfg.dst_srs, cfg.tiles, cfg.pairs, cfg.namespaces, mask, n_chunks=chunks)
    return TileBatch(gs, cfg.dst_srs, cfg.tiles, cfg.pairs, cfg.namespaces, mask)


def identity(a: np.ndarray, b: np.ndarray) -> float:
    """Fraction of identical pixels (RGBA compared per pixel)."""
    if a.shape != b.shape:
        return 0.0
    if a.ndim >= 3 and a.shape[-1] == 4:
        eq = (a == b).all(axis=-1)
    else:
        eq = (a == b) | (np.isnan(a.astype(np.float64)) & np.isnan(b.astype(np.float64)))
    return float(eq.mean())
