"""Multi-rank partitions of the GetMap batch and the drill (gsky_amd/partition.py),
world size 2 over gloo on CPU (RCCL over xGMI on the node).

CPU tests check the HIP-free planning every rank runs: each tile and polygon
is owned by exactly one rank, tile blocks are contiguous and balanced by
tile work (1 + granule pairs), a rank's sub-configuration keeps exactly the
granules its tiles touch with the pair lists remapped, and gather_drill
returns every polygon's row to rank 0.  The GPU test renders the blocks with
the HIP path in two processes on one device and compares the union with the
single-process render.  Rank timing on several GPUs is measured only by the
driver's 8-GPU runs (SCALE_r*.json)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from gsky_amd import partition, synth


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _tile_cfg():
    return synth.config_c2(scale=0.05, tiles_per_side=4, tile_px=64, grid=4)


def _drill_cfg():
    return synth.config_c4(n_bands=6, size=160, n_polys=24, rmin=3.0, rmax=30.0)


def _tile_plan(cfg, rank, world):
    """What a rank plans before it touches a device: its weighted tile block
    and the sub-configuration it uploads."""
    ids = partition.tile_blocks(len(cfg.tiles), rank, world, partition.tile_cost(cfg.pairs))
    sub = partition.sub_config(cfg, ids)
    gidx = [next(k for k, g in enumerate(cfg.granules) if g is sg) for sg in sub.granules]
    remapped = [[gidx[j] for j in sub.pairs[t]] for t in range(len(ids))]
    touched = sorted({g for i in ids for g in cfg.pairs[i]})
    return ids, sub, gidx, remapped == [list(cfg.pairs[i]) for i in ids] and gidx == touched


def _tile_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        cfg = _tile_cfg()
        ids, sub, gidx, ok = _tile_plan(cfg, rank, world)
        parts = [None] * world
        dist.all_gather_object(parts, (ids, gidx, ok, sum(partition.tile_cost(sub.pairs))))
        if rank == 0:
            q.put(parts)
    finally:
        dist.destroy_process_group()


def _tile_worker_gpu(rank, world, port, q):
    """The same plan, then the rank's block rendered by the HIP path on cuda:0."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import gsky_amd
        from tests.helpers import gpu_batch
        cfg = _tile_cfg()
        ids, sub, _, ok = _tile_plan(cfg, rank, world)
        rgba = None
        if ids:
            b = gpu_batch(sub, "cuda:0")
            rgba = b.render(gsky_amd.ScaleParams(*sub.scale), gsky_amd.Palette(sub.palette, True)).cpu().numpy()
            assert b.status() == 0
        parts = [None] * world
        dist.all_gather_object(parts, (ids, rgba, ok))
        if rank == 0:
            q.put(parts)
    finally:
        dist.destroy_process_group()


def _drill_worker(rank, world, port, q):
    """Largest-first polygon shares, then gather_drill of per-polygon rows
    that encode (polygon, band) so the gathered order is checkable."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        dc = _drill_cfg()
        inside = [int(m.sum()) for m in dc.masks]
        mine = partition.drill_assignment(inside, rank, world)
        nb = dc.bands.shape[0]
        v = torch.tensor([[p + b / 1000.0 for b in range(nb)] for p in mine], dtype=torch.float64).reshape(-1, nb)
        c = torch.tensor([[p * 10 + b for b in range(nb)] for p in mine], dtype=torch.int64).reshape(-1, nb)
        out = partition.gather_drill(v, c, mine, len(dc.masks))
        if rank == 0:
            q.put((out[0].numpy(), out[1].numpy(), [partition.drill_assignment(inside, r, world)
                                                    for r in range(world)]))
    finally:
        dist.destroy_process_group()


def _run(target, world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = q.get(timeout=240)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    return res


def test_tile_blocks_cover_once():
    for n in (0, 1, 7, 64, 4096):
        for w in (1, 2, 3, 8):
            ids = [partition.tile_blocks(n, r, w) for r in range(w)]
            flat = [i for b in ids for i in b]
            assert flat == list(range(n))
            assert max(map(len, ids)) - min(map(len, ids)) <= 1


def test_drill_assignment_balanced():
    rng = np.random.default_rng(0)
    counts = rng.integers(1, 10000, 1000)
    for w in (2, 4, 8):
        parts = [partition.drill_assignment(counts, r, w) for r in range(w)]
        assert sorted(i for p in parts for i in p) == list(range(1000))
        loads = [int(counts[p].sum()) for p in parts]
        assert max(loads) - min(loads) <= int(counts.max())   # round-robin of a sorted list


def test_tile_blocks_weighted():
    rng = np.random.default_rng(1)
    for n in (1, 5, 64, 4096):
        wts = [1.0 + int(k) for k in rng.integers(0, 4, n)]
        for w in (1, 2, 3, 8):
            ids = [partition.tile_blocks(n, r, w, wts) for r in range(w)]
            flat = [i for b in ids for i in b]
            assert flat == list(range(n))                                  # contiguous, each once
            loads = [sum(wts[i] for i in b) for b in ids]
            if n >= 8 * w:
                assert max(loads) - min(loads) <= 2 * max(wts)


def test_c2_blocks_balanced_by_pairs():
    cfg = synth.config_c2()
    cost = partition.tile_cost(cfg.pairs)
    for w in (2, 4, 8):
        loads = [sum(cost[i] for i in partition.tile_blocks(len(cfg.tiles), r, w, cost)) for r in range(w)]
        assert max(loads) - min(loads) <= 2 * max(cost), loads


def test_tile_partition_gloo():
    """Two ranks plan their weighted tile blocks and sub-configurations: every
    tile once, in order, exactly the touched granules per rank, pair lists
    remapped consistently, loads balanced."""
    world = 2
    parts = _run(_tile_worker, world)
    cfg = _tile_cfg()
    ids = [i for p in parts for i in p[0]]
    assert ids == list(range(len(cfg.tiles)))
    assert all(p[2] for p in parts)
    assert all(len(p[1]) < len(cfg.granules) for p in parts)   # a strict subset here
    loads = [p[3] for p in parts]
    assert max(loads) - min(loads) <= 2 * max(partition.tile_cost(cfg.pairs))


@pytest.mark.gpu
def test_tile_partition_gpu_ranks():
    """Two processes on one device render their blocks through the HIP path;
    the concatenation equals the single-process render bit for bit."""
    import gsky_amd
    from tests.helpers import gpu_batch
    world = 2
    parts = _run(_tile_worker_gpu, world)
    cfg = _tile_cfg()
    b = gpu_batch(cfg, "cuda:0")
    full = b.render(gsky_amd.ScaleParams(*cfg.scale), gsky_amd.Palette(cfg.palette, True)).cpu().numpy()
    assert [i for p in parts for i in p[0]] == list(range(len(cfg.tiles)))
    got = np.concatenate([p[1] for p in parts if p[0]], axis=0)
    assert np.array_equal(got, full)
    assert all(p[2] for p in parts)
    assert (full[..., 3] > 0).mean() > 0.3


def test_drill_partition_gloo():
    """Two ranks gather their largest-first polygon shares: rank 0 holds every
    polygon's row in polygon order."""
    world = 2
    vals, cnts, assign = _run(_drill_worker, world)
    dc = _drill_cfg()
    nb = dc.bands.shape[0]
    assert sorted(i for a in assign for i in a) == list(range(len(dc.masks)))
    for p in range(len(dc.masks)):
        assert np.array_equal(cnts[p], np.array([p * 10 + b for b in range(nb)])), p
        assert np.array_equal(vals[p], np.array([p + b / 1000.0 for b in range(nb)])), p
