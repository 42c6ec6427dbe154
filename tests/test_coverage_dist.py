"""WCS coverage sharding (gsky_amd/coverage.py) with world_size 2 over gloo
on CPU: row-band partition of the chunk grid, per-rank band assembly, and
the gather to rank 0 (RCCL over xGMI on the GPU box).  The per-rank renderer
is a deterministic stand-in so that the exchange logic is checked exactly."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from gsky_amd import coverage


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


CH, CW, NX, NY = 8, 6, 3, 5


class _Cfg:
    tiles = [((0, 0, 1, 1), CW, CH)] * (NX * NY)


def _truth():
    return np.arange(NY * CH * NX * CW, dtype=np.float32).reshape(NY * CH, NX * CW)


def _renderer(cfg, rows, nx, device):
    s, e = rows
    full = _truth()
    # chunks row-major as TileBatch renders them, then assembled
    chunks = []
    for j in range(s, e):
        for i in range(nx):
            chunks.append(full[j * CH:(j + 1) * CH, i * CW:(i + 1) * CW])
    if not chunks:
        return torch.zeros((0, nx * CW))
    return coverage.assemble_band(torch.from_numpy(np.stack(chunks)), e - s, nx, CH, CW)


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        full, bands = coverage.render_coverage(_Cfg(), NX, NY, renderer=_renderer)
        if rank == 0:
            q.put((full.numpy(), bands))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_coverage_gather_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    full, bands = q.get(timeout=120)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    assert np.array_equal(full, _truth())
    assert bands[0][0] == 0 and bands[-1][1] == NY
    assert all(bands[i][1] == bands[i + 1][0] for i in range(len(bands) - 1))


def test_band_partition():
    for n in range(1, 20):
        for w in range(1, 9):
            b = [coverage.band_of_rank(n, r, w) for r in range(w)]
            assert b[0][0] == 0 and b[-1][1] == n
            sizes = [e - s for s, e in b]
            assert max(sizes) - min(sizes) <= 1


def test_chunk_grid_covers_request():
    bb = (0.0, 0.0, 3000.0, 2500.0)
    tiles, nx, ny = coverage.chunk_grid(bb, 3000, 2500, 1024)
    assert (nx, ny) == (3, 3) and len(tiles) == 9
    assert sum(w * h for _, w, h in tiles) == 3000 * 2500
    assert tiles[0][0][0] == 0.0 and tiles[0][0][3] == 2500.0
    assert abs(tiles[-1][0][2] - 3000.0) < 1e-9 and abs(tiles[-1][0][1]) < 1e-9


@pytest.mark.gpu
def test_coverage_band_gpu_matches_oracle(gpu, oracle):
    """World-size-1 GetCoverage on the GPU: the assembled float32 coverage,
    byte-scaled, against the oracle's rendered chunks (bilinear bar)."""
    from gsky_amd import synth
    from tests.helpers import oracle_render
    cfg = synth.config_c3(scale=0.05, chunk_px=96, out_px=288, grid=3)
    cfg.scale = (0.0, 1.0, 255.0, 0)
    nx = ny = 3
    full, bands = coverage.render_coverage(cfg, nx, ny, device=gpu)
    assert full.shape == (ny * 96, nx * 96) and bands == [(0, 3)]
    exp = oracle_render(oracle, cfg)                       # (9, 96, 96, 4) RGBA
    exp_full = exp.reshape(ny, nx, 96, 96, 4).transpose(0, 2, 1, 3, 4).reshape(ny * 96, nx * 96, 4)
    v = full.cpu().numpy()
    valid = exp_full[..., 3] > 0
    grey = np.clip(v, 0, 255).astype(np.uint8)
    agree = (grey[valid] == exp_full[..., 0][valid]).mean()
    assert agree >= 0.999
