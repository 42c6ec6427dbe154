"""Multi-rank partitions of the GetMap batch and the drill (gsky_amd/partition.py),
world size 2 over gloo on CPU (RCCL over xGMI on the node): every tile and
polygon is owned by exactly one rank, a rank's sub-configuration keeps only
the granules its tiles touch, and the union of the ranks' results -- here
the CPU oracle's, the checker (tests may run it) -- equals the single-rank
result bit for bit.  The GPU ranks run the same partition in bench.py."""
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


def _tile_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import oracle as O
        from tests.helpers import oracle_render
        cfg = _tile_cfg()
        ids = partition.tile_blocks(len(cfg.tiles), rank, world)
        sub = partition.sub_config(cfg, ids)
        used = {id(g) for g in sub.granules}
        touched = {id(cfg.granules[g]) for i in ids for g in cfg.pairs[i]}
        rgba = oracle_render(O, sub, n_threads=2) if ids else np.zeros((0, 64, 64, 4), np.uint8)
        parts = [None] * world
        dist.all_gather_object(parts, (ids, rgba, used == touched, len(sub.granules)))
        if rank == 0:
            q.put(parts)
    finally:
        dist.destroy_process_group()


def _drill_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import oracle as O
        dc = _drill_cfg()
        clip = (-3.4028234663852886e38, 3.4028234663852886e38)
        inside = [int(m.sum()) for m in dc.masks]
        mine = partition.drill_assignment(inside, rank, world)
        vals, cnts = [], []
        for p in mine:
            x0, y0, w, h = dc.windows[p]
            ev, ec = O.drill_read_data(np.ascontiguousarray(dc.bands[:, y0:y0 + h, x0:x0 + w]), dc.masks[p],
                                       dc.nodata, clip[0], clip[1], 0, 1)
            vals.append(ev)
            cnts.append(ec)
        nb = dc.bands.shape[0]
        v = torch.tensor(np.array(vals).reshape(len(mine), -1)[:, :nb], dtype=torch.float64)
        c = torch.tensor(np.array(cnts).reshape(len(mine), -1)[:, :nb], dtype=torch.int64)
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


def test_tile_partition_gloo(oracle):
    """Two ranks render their tile blocks from their own granule subsets; the
    concatenation is the single-rank batch."""
    from tests.helpers import oracle_render
    world = 2
    parts = _run(_tile_worker, world)
    cfg = _tile_cfg()
    full = oracle_render(oracle, cfg, n_threads=2)
    ids = [i for p in parts for i in p[0]]
    assert ids == list(range(len(cfg.tiles)))
    got = np.concatenate([p[1] for p in parts if len(p[0])], axis=0)
    assert np.array_equal(got, full)
    assert all(p[2] for p in parts)                       # exactly the touched granules uploaded
    assert all(p[3] < len(cfg.granules) for p in parts)   # ... a strict subset here
    assert (full[..., 3] > 0).mean() > 0.3


def test_drill_partition_gloo(oracle):
    """Two ranks reduce their largest-first share of the polygons; the
    gathered rows equal the single-rank reduction."""
    world = 2
    vals, cnts, assign = _run(_drill_worker, world)
    dc = _drill_cfg()
    clip = (-3.4028234663852886e38, 3.4028234663852886e38)
    nb = dc.bands.shape[0]
    assert sorted(i for a in assign for i in a) == list(range(len(dc.masks)))
    for p in range(len(dc.masks)):
        x0, y0, w, h = dc.windows[p]
        ev, ec = oracle.drill_read_data(np.ascontiguousarray(dc.bands[:, y0:y0 + h, x0:x0 + w]), dc.masks[p],
                                        dc.nodata, clip[0], clip[1], 0, 1)
        assert np.array_equal(cnts[p], np.asarray(ec)[:nb]), p
        assert np.array_equal(vals[p].view(np.uint64), np.asarray(ev, np.float64)[:nb].view(np.uint64)), p
    assert cnts.sum() > 0
