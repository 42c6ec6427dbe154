"""WCS coverage sharding (gsky_amd/coverage.py): the reference's chunk list
(ows.go:817-831), the row-band partition, per-rank placement by chunk offset
and the gather to rank 0, over gloo on CPU at world sizes 2 and 3 (RCCL over
xGMI on the GPU box).  The per-rank renderer is a deterministic stand-in
(chunks cut from a known image at their offsets) so that the exchange logic
is checked exactly, including sizes that are not chunk multiples and ranks
whose band is empty."""
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


class _Cfg:
    def __init__(self, w, h):
        self.bbox = (1000.0, -500.0, 1000.0 + 3.0 * w, -500.0 + 2.0 * h)
        self.w, self.h = w, h


def _truth(w, h):
    return np.arange(w * h, dtype=np.float32).reshape(h, w)


def _renderer(cfg, chunks, rows, width, device):
    full = torch.from_numpy(_truth(cfg.w, cfg.h))
    sel = [c for c in chunks if rows[0] <= c.row < rows[1]]
    if not sel:
        return torch.zeros((0, width))
    top, bottom = coverage.band_extent(chunks, rows)
    canv = [full[c.off_y:c.off_y + c.height, c.off_x:c.off_x + c.width].clone() for c in sel]
    return coverage.place_chunks(canv, sel, top, bottom - top, width)


def _worker(rank, world, port, q, w, h, ch):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        full, ext = coverage.render_coverage(_Cfg(w, h), w, h, renderer=_renderer, max_x=ch, max_y=ch)
        if rank == 0:
            q.put((full.numpy(), ext))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,w,h,ch", [(2, 250, 200, 96), (3, 250, 200, 96), (2, 288, 288, 96),
                                          (3, 70, 90, 96)])
def test_coverage_gather_gloo(world, w, h, ch):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, w, h, ch)) for r in range(world)]
    for p in procs:
        p.start()
    full, ext = q.get(timeout=120)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    assert full.shape == (h, w)
    assert np.array_equal(full, _truth(w, h))
    nonempty = [e for e in ext if e[1] > e[0]]
    assert sum(b - t for t, b in nonempty) == h
    if h <= ch:
        assert len(nonempty) == 1          # world > chunk rows: the other bands are empty


def test_band_partition():
    for n in range(0, 20):
        for w in range(1, 9):
            b = [coverage.band_of_rank(n, r, w) for r in range(w)]
            assert b[0][0] == 0 and b[-1][1] == n
            sizes = [e - s for s, e in b]
            assert max(sizes) - min(sizes) <= 1


def test_chunk_requests_match_reference():
    """ows.go:817-831: rows from the south edge up, the partial chunk at the
    north edge, int(.5 + extent/res) sizes, image offset (x, H - y - h)."""
    bb = (0.0, 0.0, 3000.0, 2500.0)
    ch = coverage.chunk_requests(bb, 3000, 2500, 1024, 1024)
    assert len(ch) == 9
    assert [c.height for c in ch[::3]] == [1024, 1024, 452]
    assert [c.off_y for c in ch[::3]] == [1476, 452, 0]
    assert [c.width for c in ch[:3]] == [1024, 1024, 952]
    assert ch[0].bbox == (0.0, 0.0, 1024.0, 1024.0)
    assert ch[-1].bbox[2] == 3000.0 and ch[-1].bbox[3] == 2500.0
    cover = np.zeros((2500, 3000), np.int32)
    for c in ch:
        cover[c.off_y:c.off_y + c.height, c.off_x:c.off_x + c.width] += 1
    assert (cover == 1).all()


@pytest.mark.gpu
@pytest.mark.parametrize("w,h", [(288, 288), (250, 200)])
def test_coverage_band_gpu_matches_oracle(gpu, oracle, w, h):
    """World-size-1 GetCoverage on the GPU against the oracle's typed float
    canvases: identical nodata mask, every valid pixel within 1e-4 relative."""
    from gsky_amd import synth
    from tests.helpers import oracle_render
    cfg = synth.config_c3(scale=0.05, chunk_px=96, out_px=w, out_h=h, grid=3)
    full, ext = coverage.render_coverage(cfg, w, h, device=gpu, max_x=96, max_y=96)
    assert full.shape == (h, w)
    _, cv, created = oracle_render(oracle, cfg, canvas=True)
    chunks = coverage.chunk_requests(cfg.bbox, w, h, 96, 96)
    mh = max(c.height for c in chunks)
    mw = max(c.width for c in chunks)
    canv = [torch.from_numpy(cv[i, 0].view(np.float32).reshape(mh, mw)[:c.height, :c.width].copy())
            for i, c in enumerate(chunks)]
    exp = coverage.place_chunks(canv, chunks, 0, h, w).numpy()
    got = full.cpu().numpy()
    assert created[:, 0].all()
    nod_e, nod_g = exp == -9999.0, got == -9999.0
    assert np.array_equal(nod_e, nod_g)
    v = ~nod_e
    assert v.mean() > 0.5
    rel = np.abs(got[v].astype(np.float64) - exp[v]) / np.maximum(np.abs(exp[v].astype(np.float64)), 1e-30)
    assert rel.max() <= 1e-4, rel.max()


def _gpu_worker(rank, world, port, q, w, h, ch):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from gsky_amd import synth
        torch.cuda.set_device(0)
        cfg = synth.config_c3(scale=0.05, chunk_px=ch, out_px=w, out_h=h, grid=3)
        full, ext = coverage.render_coverage(cfg, w, h, device=torch.device("cuda", 0), max_x=ch, max_y=ch)
        torch.cuda.synchronize()
        q.put((rank, full.cpu().numpy() if rank == 0 else None, ext))
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 3])
def test_coverage_hip_ranks_match_single_process(world):
    """The multi-rank GetCoverage through the HIP path: `world` processes on
    the one device each render their row band with the product kernels and
    gather it to rank 0 (exact-size point-to-point receives into the
    coverage; gloo stages the device bands through host memory), and rank 0's
    coverage equals the single-process render bit for bit."""
    from gsky_amd import synth
    w, h, ch = 250, 300, 96
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gpu_worker, args=(r, world, port, q, w, h, ch)) for r in range(world)]
    for p in procs:
        p.start()
    got = {}
    for _ in range(world):
        r, arr, ext = q.get(timeout=240)
        got[r] = (arr, ext)
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    cfg = synth.config_c3(scale=0.05, chunk_px=ch, out_px=w, out_h=h, grid=3)
    one, _ = coverage.render_coverage(cfg, w, h, device=torch.device("cuda", 0), max_x=ch, max_y=ch)
    full, ext = got[0]
    assert sum(b - t for t, b in ext) == h and len([e for e in ext if e[1] > e[0]]) == world
    assert np.array_equal(full, one.cpu().numpy())
