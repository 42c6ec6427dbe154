"""Multi-GPU partitions of the hot path: one process per GPU,
torch.distributed (RCCL over xGMI on the node, gloo in the CPU tests).

* GetMap tile batches (C2/C5): tiles are independent requests
  (tile_grpc.go:96-258 serves each on its own), so a batch is cut into
  contiguous blocks of tiles -- neighbouring tiles share granules -- balanced
  by the work of each tile (`tile_cost`: the RGBA slot every tile writes plus
  one gather pass per granule under it, so the empty tiles at the edge of a
  union bbox weigh less than the covered ones), and each rank uploads only
  the granules its block touches (`sub_config`).  No data-path collective:
  every rank's RGBA tiles are its own responses.
* Drill (C4): polygons are independent (drill.go:90-158 reads each file's
  window per polygon); they are dealt largest-first round-robin so the ranks'
  pixel counts balance.  `gather_drill` returns every polygon's result to
  rank 0 when one requester wants them all (the OWS drill response).
* WCS coverage (C3): chunk rows, gsky_amd/coverage.py.
"""
from __future__ import annotations

from typing import List, Optional, Sequence


def tile_blocks(n: int, rank: int, world: int, weights: Optional[Sequence[float]] = None) -> List[int]:
    """Contiguous block of tile indices of `rank`.  Without weights the
    sizes differ by at most 1; with per-tile weights tile i goes to the rank
    whose share [r, r+1) * total / world holds the midpoint of i's weight
    interval, so blocks stay contiguous and their weights balance to within
    one tile."""
    if weights is None:
        base, extra = divmod(n, world)
        s = rank * base + min(rank, extra)
        return list(range(s, s + base + (1 if rank < extra else 0)))
    if len(weights) != n:
        raise ValueError("tile_blocks: %d weights for %d tiles" % (len(weights), n))
    total = float(sum(weights))
    if total <= 0.0:
        return tile_blocks(n, rank, world)
    out, acc = [], 0.0
    for i, w in enumerate(weights):
        owner = min(world - 1, int((acc + 0.5 * float(w)) * world / total))
        if owner == rank:
            out.append(i)
        acc += float(w)
    return out


def tile_cost(pairs: Sequence[Sequence[int]]) -> List[float]:
    """Relative render work of each tile: 1 for its RGBA slot (written even
    when no granule covers it) + 1 per granule pair merged into it."""
    return [1.0 + len(p) for p in pairs]


def sub_config(cfg, ids: Sequence[int]):
    """The synth config restricted to tiles `ids`, with only the granules
    those tiles touch (pair indices remapped): what a rank uploads."""
    from . import synth
    used = sorted({g for i in ids for g in cfg.pairs[i]})
    remap = {g: k for k, g in enumerate(used)}
    return synth.SynthConfig(cfg.name, [cfg.granules[g] for g in used], cfg.dst_srs, [cfg.tiles[i] for i in ids],
                             [[remap[g] for g in cfg.pairs[i]] for i in ids], cfg.namespaces, cfg.scale,
                             cfg.palette, cfg.resample, cfg.mask, cfg.bbox, cfg.out_w, cfg.out_h)


def drill_assignment(pixel_counts: Sequence[int], rank: int, world: int) -> List[int]:
    """Polygons of `rank`: sorted by in-mask pixel count, largest first (ties
    by index), dealt round-robin."""
    order = sorted(range(len(pixel_counts)), key=lambda p: (-int(pixel_counts[p]), p))
    return order[rank::world]


def gather_drill(values, counts, mine: Sequence[int], n_polys: int, group=None):
    """Rank 0 receives every polygon's (values, counts) rows in polygon order
    (tensors of shape (len(mine), n_bands)); other ranks get None.  The one
    collective of the drill path, after the timed reduction."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    n_bands = values.shape[1]
    per = max(1, max(len(range(r, n_polys, world)) for r in range(world)))   # largest share
    pad_v = torch.zeros((per, n_bands), dtype=values.dtype, device=values.device)
    pad_c = torch.zeros((per, n_bands), dtype=counts.dtype, device=counts.device)
    idx = torch.full((per,), -1, dtype=torch.int64, device=values.device)
    k = len(mine)
    pad_v[:k] = values
    pad_c[:k] = counts
    idx[:k] = torch.tensor(list(mine), dtype=torch.int64, device=values.device)
    if rank == 0:
        bv = [torch.empty_like(pad_v) for _ in range(world)]
        bc = [torch.empty_like(pad_c) for _ in range(world)]
        bi = [torch.empty_like(idx) for _ in range(world)]
    else:
        bv = bc = bi = None
    dist.gather(pad_v, bv, dst=0, group=group)
    dist.gather(pad_c, bc, dst=0, group=group)
    dist.gather(idx, bi, dst=0, group=group)
    if rank != 0:
        return None
    out_v = torch.zeros((n_polys, n_bands), dtype=values.dtype, device=values.device)
    out_c = torch.zeros((n_polys, n_bands), dtype=counts.dtype, device=counts.device)
    for r in range(world):
        ok = bi[r] >= 0
        out_v[bi[r][ok]] = bv[r][ok]
        out_c[bi[r][ok]] = bc[r][ok]
    return out_v, out_c


def shard_of(n: int, rank: int, world: int, kind: str = "tiles", weights: Optional[Sequence[int]] = None):
    """Indices of `rank` for a partition kind: "tiles" (contiguous blocks) or
    "drill" (largest-first round-robin by `weights`)."""
    if kind == "tiles":
        return tile_blocks(n, rank, world)
    if kind == "drill":
        return drill_assignment(weights if weights is not None else [1] * n, rank, world)
    raise ValueError("unknown partition kind %r" % kind)
