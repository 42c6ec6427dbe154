"""WCS GetCoverage over several MI355X (BASELINE.json configs[2]).

The reference splits a large coverage into chunk requests of at most
1024x1024 (utils/config.go:55-56, ows.go:815-833), fans them out over HTTP to
other gsky-ows instances and merges the returned GeoTIFFs through temporary
files (ows.go:930-995, 1094-1150).  Here the chunks are partitioned into
contiguous row bands, one per rank (one process per GPU); each rank renders its
band's chunks as typed canvases with the batched tile path (no RGBA,
TileBatch.render(rgba=False)) and the bands are gathered to rank 0 with
torch.distributed -- RCCL over xGMI on the GPU box, gloo in the CPU tests.
That gather is the only data-path collective of the whole hot path.
"""
from __future__ import annotations

from typing import Callable, List, Optional, Sequence, Tuple

import torch


def chunk_grid(bbox: Sequence[float], width: int, height: int, chunk: int = 1024):
    """Row-major chunk bboxes of a width x height coverage (ows.go:815-833:
    xRes/yRes from the request, chunks of at most `chunk` pixels a side)."""
    nx = (width + chunk - 1) // chunk
    ny = (height + chunk - 1) // chunk
    xres = (bbox[2] - bbox[0]) / width
    yres = (bbox[3] - bbox[1]) / height
    out = []
    for j in range(ny):
        for i in range(nx):
            w = min(chunk, width - i * chunk)
            h = min(chunk, height - j * chunk)
            x0 = bbox[0] + i * chunk * xres
            y1 = bbox[3] - j * chunk * yres
            out.append(((x0, y1 - h * yres, x0 + w * xres, y1), w, h))
    return out, nx, ny


def band_of_rank(n_chunk_rows: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous chunk rows [start, end) served by `rank` (balanced within one
    row when world does not divide n_chunk_rows)."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError("bad rank/world")
    base, extra = divmod(n_chunk_rows, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def assemble_band(chunks: torch.Tensor, n_rows: int, nx: int, chunk_h: int, chunk_w: int,
                  width: Optional[int] = None) -> torch.Tensor:
    """(n_rows*nx, chunk_h, chunk_w) chunk canvases, row-major -> one
    (n_rows*chunk_h, width) row band."""
    b = chunks.reshape(n_rows, nx, chunk_h, chunk_w).permute(0, 2, 1, 3).reshape(n_rows * chunk_h, nx * chunk_w)
    return b[:, :width] if width is not None else b


def gather_coverage(band: torch.Tensor, band_rows: Sequence[Tuple[int, int]], chunk_h: int, height: int,
                    group=None) -> Optional[torch.Tensor]:
    """Gathers every rank's row band to rank 0 and returns the full coverage
    there (None elsewhere).  Bands are padded to the largest band so one
    fixed-size gather serves uneven partitions."""
    import torch.distributed as dist
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    max_rows = max(e - s for s, e in band_rows) * chunk_h
    pad = torch.zeros((max_rows, band.shape[1]), dtype=band.dtype, device=band.device)
    pad[: band.shape[0]] = band
    bufs = [torch.empty_like(pad) for _ in range(world)] if rank == 0 else None
    dist.gather(pad, bufs, dst=0, group=group)
    if rank != 0:
        return None
    parts = []
    for r, (s, e) in enumerate(band_rows):
        parts.append(bufs[r][: (e - s) * chunk_h])
    return torch.cat(parts, 0)[:height]


def render_band_gpu(cfg, rows: Tuple[int, int], nx: int, device) -> torch.Tensor:
    """Renders chunk rows [rows) of a synth-style coverage config (tiles =
    row-major chunks, one namespace, Float32 canvas) on `device`."""
    from . import ScaleParams
    from .tiles import GranuleSet, TileBatch
    import numpy as np
    s, e = rows
    ids = list(range(s * nx, e * nx))
    gs = GranuleSet(device)
    for g in cfg.granules:
        gs.add(torch.from_numpy(np.ascontiguousarray(g.data)), g.geot, g.srs, g.nodata, [], g.timestamp,
               g.polygon, g.namespace)
    tb = TileBatch(gs, cfg.dst_srs, [cfg.tiles[i] for i in ids], [cfg.pairs[i] for i in ids], cfg.namespaces)
    cv = tb.render(ScaleParams(*cfg.scale), resample=cfg.resample, rgba=False)
    ch, cw = tb.max_h, tb.max_w
    chunks = cv[:, 0, : ch * cw * 4].contiguous().view(torch.float32).reshape(len(ids), ch, cw)
    return assemble_band(chunks, e - s, nx, ch, cw)


def render_coverage(cfg, nx: int, ny: int, renderer: Callable = render_band_gpu, device=None,
                    group=None) -> Tuple[Optional[torch.Tensor], List[Tuple[int, int]]]:
    """The whole multi-rank GetCoverage: partition, render own band, gather."""
    import torch.distributed as dist
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    bands = [band_of_rank(ny, r, world) for r in range(world)]
    band = renderer(cfg, bands[rank], nx, device)
    chunk_h = cfg.tiles[0][2]
    if world == 1:
        return band, bands
    return gather_coverage(band, bands, chunk_h, ny * chunk_h, group), bands
