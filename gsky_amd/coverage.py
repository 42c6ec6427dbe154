"""WCS GetCoverage over several MI355X (BASELINE.json configs[2]).

The reference splits a large coverage into chunk requests of at most
WcsMaxTileWidth x WcsMaxTileHeight (1024 x 1024 by default,
utils/config.go:55-56; chunking at ows.go:815-833), fans them out over HTTP
to other gsky-ows instances and merges the returned GeoTIFFs through temporary
files (ows.go:930-995, 1094-1150).  Here the chunk list is built exactly as
ows.go:817-831 does (south to north, west to east, `int(.5 + extent/res)`
sizes, image offset `(x, Height - y - tileYSize)`), the chunk rows are
partitioned into contiguous bands, one per rank (one process per GPU), each
rank uploads only the granules its chunks intersect and renders its chunks as
typed canvases with the batched tile path (no RGBA: TileBatch.render(rgba=False),
FusionUnscale of ows.go:728), and the bands are gathered to rank 0 with
torch.distributed -- RCCL over xGMI on the GPU box, gloo in the CPU tests.
That gather is the only data-path collective of the whole hot path.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Callable, List, Optional, Sequence, Tuple


@dataclass
class Chunk:
    """One GeoTileRequest of the chunked coverage (ows.go:822-830)."""
    bbox: Tuple[float, float, float, float]
    width: int
    height: int
    off_x: int          # image column of the chunk's west edge
    off_y: int          # image row of the chunk's north edge
    row: int            # chunk row in list order (0 = southernmost)


def chunk_requests(bbox: Sequence[float], width: int, height: int, max_x: int = 1024,
                   max_y: int = 1024) -> List[Chunk]:
    """The reference's chunk list (ows.go:817-831), in its order."""
    x_res = (bbox[2] - bbox[0]) / float(width)
    y_res = (bbox[3] - bbox[1]) / float(height)
    out = []
    for row, y in enumerate(range(0, height, max_y)):
        for x in range(0, width, max_x):
            y_min = bbox[1] + float(y) * y_res
            y_max = min(bbox[1] + float(y + max_y) * y_res, bbox[3])
            x_min = bbox[0] + float(x) * x_res
            x_max = min(bbox[0] + float(x + max_x) * x_res, bbox[2])
            tw = int(.5 + (x_max - x_min) / x_res)
            th = int(.5 + (y_max - y_min) / y_res)
            out.append(Chunk((x_min, y_min, x_max, y_max), tw, th, x, height - y - th, row))
    return out


def n_chunk_rows(chunks: Sequence[Chunk]) -> int:
    return 1 + max(c.row for c in chunks) if chunks else 0


def band_of_rank(n_rows: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous chunk rows [start, end) served by `rank` (balanced within one
    row when world does not divide n_rows; empty when world > n_rows)."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError("bad rank/world")
    base, extra = divmod(n_rows, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def band_extent(chunks: Sequence[Chunk], rows: Tuple[int, int]) -> Tuple[int, int]:
    """Image rows [top, bottom) covered by chunk rows [rows) (empty -> (0, 0))."""
    sel = [c for c in chunks if rows[0] <= c.row < rows[1]]
    if not sel:
        return 0, 0
    return min(c.off_y for c in sel), max(c.off_y + c.height for c in sel)


def place_chunks(canvases, chunks: Sequence[Chunk], top: int, n_rows: int, width: int, dtype=None,
                 device=None):
    """Writes each chunk canvas (its own height x width) at its image offset
    into one (n_rows, width) band whose first row is image row `top`."""
    import torch
    band = torch.empty((n_rows, width), dtype=dtype or torch.float32, device=device)
    for cv, c in zip(canvases, chunks):
        band[c.off_y - top: c.off_y - top + c.height, c.off_x: c.off_x + c.width] = cv
    return band


def gather_coverage(band, extents: Sequence[Tuple[int, int]], height: int, width: int, group=None, out=None):
    """Gathers every rank's row band to rank 0 and returns the full
    (height, width) coverage there (None elsewhere): rank 0 receives each
    band straight into its rows of the coverage (point-to-point receives of
    exactly that band's size, RCCL over xGMI on a node: no padded buffers,
    no copy afterwards; the WCS reference instead merges per-node GeoTIFF
    files over HTTP, ows.go:930-995, 1094-1150).  `out`: a preallocated
    coverage on rank 0; when rank 0's own band is already a view of its rows
    (rendered in place) it is not copied either.  A gloo group with device
    tensors stages through host memory (tests; gloo has no device p2p)."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    via_host = band.is_cuda and dist.get_backend(group) == "gloo"
    if rank != 0:
        # posted through batch_isend_irecv like rank 0's receives: under
        # NCCL/RCCL a batched P2P that is the group's first collective must be
        # entered by every rank
        t, b = extents[rank]
        if b > t:
            src = band[: b - t].contiguous()
            if via_host:
                src = src.cpu()
            for w in dist.batch_isend_irecv([dist.P2POp(dist.isend, src, 0, group)]):
                w.wait()
        return None
    full = out if out is not None else torch.empty((height, width), dtype=band.dtype, device=band.device)
    t0, b0 = extents[0]
    if b0 > t0 and band.data_ptr() != full[t0].data_ptr():
        full[t0:b0] = band[: b0 - t0]
    ops, staged = [], []
    for r in range(1, world):
        t, b = extents[r]
        if b <= t:
            continue
        if via_host:
            h = torch.empty((b - t, width), dtype=band.dtype)
            staged.append((h, t, b))
            ops.append(dist.P2POp(dist.irecv, h, r, group))
        else:
            ops.append(dist.P2POp(dist.irecv, full[t:b], r, group))
    if ops:
        for w in dist.batch_isend_irecv(ops):
            w.wait()
    for h, t, b in staged:
        full[t:b] = h.to(full.device)
    return full


def render_band_gpu(cfg, chunks: Sequence[Chunk], rows: Tuple[int, int], width: int, device, out=None):
    """Renders the chunks of chunk rows [rows) of a synth-style coverage config
    on `device` (one namespace, Float32 canvases, cfg.resample) and returns the
    (band rows, width) band.  Only granules intersecting the band's chunks are
    uploaded.  `out`: a (band rows, width) float32 view to render into -- rank
    0 passes its rows of the coverage, so its band is never copied."""
    import numpy as np
    import torch

    from . import ScaleParams
    from .tiles import GranuleSet, TileBatch
    top, bottom = band_extent(chunks, rows)
    sel = [c for c in chunks if rows[0] <= c.row < rows[1]]
    if not sel:
        return torch.zeros((0, width), dtype=torch.float32, device=device)
    pairs = [cfg.index_chunk(c.bbox) for c in sel]
    used = sorted({g for p in pairs for g in p})
    remap = {g: i for i, g in enumerate(used)}
    gs = GranuleSet(device)
    for g in used:
        gr = cfg.granules[g]
        gs.add(torch.from_numpy(np.ascontiguousarray(gr.data)), gr.geot, gr.srs, gr.nodata, [], gr.timestamp,
               gr.polygon, gr.namespace)
    tiles = [(c.bbox, c.width, c.height) for c in sel]
    tb = TileBatch(gs, cfg.dst_srs, tiles, [[remap[g] for g in p] for p in pairs], cfg.namespaces)
    band = out if out is not None else torch.empty((bottom - top, width), dtype=torch.float32, device=device)
    if tuple(band.shape) != (bottom - top, width) or band.dtype != torch.float32 or not band.is_contiguous():
        raise ValueError("render_band_gpu: out must be a contiguous (%d, %d) float32 band" % (bottom - top, width))
    # every chunk is rendered straight into the band at its offset (no assembly copy)
    tb.render_coverage(ScaleParams(*cfg.scale), band, band_offsets(sel, top, width), resample=cfg.resample)
    return band


def band_offsets(chunks: Sequence[Chunk], top: int, width: int) -> List[int]:
    """Flat element offset of each chunk's top-left in a band whose first row
    is image row `top` and whose rows are `width` elements."""
    return [(c.off_y - top) * width + c.off_x for c in chunks]


def render_coverage(cfg, width: int, height: int, renderer: Callable = render_band_gpu, device=None,
                    group=None, max_x: int = 1024, max_y: int = 1024):
    """The whole multi-rank GetCoverage: chunk, partition, render own band,
    gather.  Returns (coverage on rank 0 / None elsewhere, band extents)."""
    import torch.distributed as dist
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    chunks = chunk_requests(cfg.bbox, width, height, max_x, max_y)
    nrows = n_chunk_rows(chunks)
    rows = [band_of_rank(nrows, r, world) for r in range(world)]
    extents = [band_extent(chunks, rw) for rw in rows]
    if world > 1 and rank == 0 and renderer is render_band_gpu:
        # rank 0 renders its band in place inside the coverage (no copy)
        import torch
        full = torch.empty((height, width), dtype=torch.float32, device=device)
        t0, b0 = extents[0]
        band = renderer(cfg, chunks, rows[rank], width, device, out=full[t0:b0])
        return gather_coverage(band, extents, height, width, group, out=full), extents
    band = renderer(cfg, chunks, rows[rank], width, device)
    if world == 1:
        return band, extents
    return gather_coverage(band, extents, height, width, group), extents
