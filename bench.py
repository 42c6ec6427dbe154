#!/usr/bin/env python3
"""Benchmark of the MI355X GSKY raster hot path (BASELINE.json metric).

Workload (N=1): BASELINE.json configs[1] = C2: a batch of 4096 512x512
EPSG:3857 GetMap tiles from 16 Albers EPSG:3577 int16 4000x4000 granules,
nearest-neighbour, time-ordered merge + byte scale + palette.
A step = one pass of the whole batch: planning kernels (windows, merge order,
approximate-transformer rows) + the fused warp/merge/scale/palette kernel,
granules already resident in HBM.

Multi-GPU: one process per GPU (torch.distributed, RCCL); every rank serves
its own C2 batch (tiles are independent requests, no data-path collective):
weak scaling, value = all ranks' output pixels / max-over-ranks time.

Extra fields: roofline of the dominant kernel (render, HIP events on the
launch stream), cpu_baseline (the CPU oracle, rank 0, N=1, bounded sample),
p50_tile_ms (C1 single-tile latency).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import gsky_amd  # noqa: E402
from gsky_amd import GranuleSet, Mask, Palette, ScaleParams, TileBatch, synth  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def build_batch(cfg, device):
    gs = GranuleSet(device)
    for g in cfg.granules:
        gs.add(torch.from_numpy(np.ascontiguousarray(g.data)), g.geot, g.srs, g.nodata,
               [torch.from_numpy(np.ascontiguousarray(o)) for o in g.overviews], g.timestamp, g.polygon,
               g.namespace)
    mask = Mask(cfg.mask["id"], cfg.mask.get("value", ""), cfg.mask.get("bit_tests", []),
                cfg.mask.get("inclusive", False)) if cfg.mask else None
    return TileBatch(gs, cfg.dst_srs, cfg.tiles, cfg.pairs, cfg.namespaces, mask)


def algorithmic_bytes(cfg) -> int:
    """Unique source bytes touched (every granule pixel lies under the tile
    set) + RGBA output bytes."""
    src = sum(g.data.nbytes for g in cfg.granules)
    return src + cfg.out_pixels * 4


def cpu_baseline(cfg, n_tiles: int, threads: int):
    from oracle import oracle as O
    from tests.helpers import oracle_render
    ids = np.linspace(0, len(cfg.tiles) - 1, n_tiles).round().astype(int).tolist()
    sub = synth.subset(cfg, ids)
    oracle_render(O, synth.subset(cfg, ids[:2]), n_threads=threads)  # warm
    t0 = time.perf_counter()
    oracle_render(O, sub, n_threads=threads)
    dt = time.perf_counter() - t0
    return sub.out_pixels / dt / 1e6, dt


def c1_latency(device, reps: int = 50):
    cfg = synth.config_c1()
    b = build_batch(cfg, device)
    sp = ScaleParams(*cfg.scale)
    for _ in range(5):
        b.render(sp)
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        b.render(sp)
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t0) * 1e3)
    return float(np.median(ts))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--scale", type=float, default=1.0, help="granule size scale (1 = 4000^2)")
    ap.add_argument("--tiles", type=int, default=64, help="tiles per side (64 -> 4096 tiles)")
    ap.add_argument("--cpu-tiles", type=int, default=4096, help="CPU baseline sample (tiles)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-c1", action="store_true")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    device = torch.device("cuda", torch.cuda.current_device())

    cfg = synth.config_c2(scale=args.scale, tiles_per_side=args.tiles, tile_px=512)
    batch = build_batch(cfg, device)
    sp = ScaleParams(*cfg.scale)
    pal = Palette(cfg.palette, True)

    for _ in range(args.warmup):
        batch.render(sp, pal)
    torch.cuda.synchronize()
    if batch.status() != 0:
        raise RuntimeError("render status %d" % batch.status())

    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        batch.render(sp, pal)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    dt = time.perf_counter() - t0
    if dist:
        t = torch.tensor([dt], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    ms_per_step = dt / args.steps * 1e3
    total_px = cfg.out_pixels * world * args.steps
    value = total_px / dt / 1e6

    # dominant kernel: the fused render (phase 2), HIP events on its stream
    stream = torch.cuda.current_stream()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    plan_ms, render_ms = [], []
    for _ in range(max(3, args.steps)):
        ev[0].record(stream)
        batch.render(sp, pal, phase=1)
        ev[1].record(stream)
        batch.render(sp, pal, phase=2)
        ev[2].record(stream)
        torch.cuda.synchronize()
        plan_ms.append(ev[0].elapsed_time(ev[1]))
        render_ms.append(ev[1].elapsed_time(ev[2]))
    t_render = float(np.mean(render_ms)) / 1e3
    abytes = algorithmic_bytes(cfg)
    achieved = abytes / t_render / 1e9
    traffic = None
    pmc = os.path.join(ROOT, "profiles", "pmc_render_c2.json")
    if os.path.exists(pmc) and args.scale == 1.0 and args.tiles == 64:
        try:
            traffic = json.load(open(pmc)).get("hbm_bytes_per_launch")
        except Exception:
            traffic = None

    out = {
        "metric": "reprojected+merged output Mpix/s (whole node) at 1/2/4/8 MI355X; p50 tile ms",
        "value": round(value, 1),
        "unit": "Mpix/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "int16",
        "data": "synthetic (splitmix64 granules, SURVEY.md 8d)",
        "config": {"workload": "C2: %d x %dx%d EPSG:3857 tiles from %d EPSG:3577 int16 %dx%d granules, nearest, "
                               "time-ordered merge + scale + palette" % (
                                   len(cfg.tiles), 512, 512, len(cfg.granules), cfg.granules[0].data.shape[1],
                                   cfg.granules[0].data.shape[0]),
                   "tiles_per_step_per_gpu": len(cfg.tiles), "pairs": batch.n_pairs,
                   "parallelism": "tile batches per GPU, %d rank(s)" % world},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                     "kernel": "render_fast_kernel (+ render_general, phase 2)",
                     "kernel_ms": round(t_render * 1e3, 4), "plan_ms": round(float(np.mean(plan_ms)), 4),
                     "algorithmic_bytes_per_launch": abytes},
    }
    if rank == 0 and world == 1:
        if not args.no_c1:
            out["p50_tile_ms"] = round(c1_latency(device), 4)
            out["p50_tile_config"] = "C1: one 256x256 EPSG:3857 tile from a 3600x1800 EPSG:4326 f32 granule"
        if not args.no_cpu:
            threads = min(16, os.cpu_count() or 1)
            v, secs = cpu_baseline(cfg, args.cpu_tiles, threads)
            out["cpu_baseline"] = {"value": round(v, 2), "unit": "Mpix/s", "cores": threads, "kind": "port",
                                   "sample": "%d C2 tiles (512x512) rendered by oracle/ (C restatement of "
                                             "warp_operation_fast + merge + Scale + palette), %d threads, "
                                             "%.2f s wall" % (args.cpu_tiles, threads, secs)}
    if rank == 0:
        print(json.dumps(out))
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
