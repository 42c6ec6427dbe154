#!/usr/bin/env python3
"""Benchmark of the MI355X GSKY raster hot path (BASELINE.json metric).

Headline (`value`): BASELINE.json configs[1] = C2, a batch of 4096 512x512
EPSG:3857 GetMap tiles from 16 Albers EPSG:3577 int16 4000x4000 granules,
nearest-neighbour, time-ordered merge + byte scale + palette.
A step = one pass of the whole batch: planning kernels (windows, merge order,
approximate-transformer rows) + the fused warp/merge/scale/palette kernel,
granules already resident in HBM.

Multi-GPU: one process per GPU (torch.distributed, RCCL).  The C2 request
stream is partitioned -- rank r renders a contiguous block of the 4096 tiles
(independent requests, contiguous spatial blocks for granule
locality) and uploads only the granules its tiles touch; no data-path
collective.  Total work is fixed as N grows: "scaling": "strong", `value` =
all 4096 tiles' output pixels / max-over-ranks time.

The same line carries the other BASELINE configs under "configs" (each timed
the same way: warmup, barrier + synchronize, K steps, max over ranks):
  C1  single 256^2 tile: GPU p50/p99 latency, CPU (oracle) p50/p99 beside it;
  C3  WCS 16384^2 float32 bilinear coverage, chunk rows sharded over ranks,
      RCCL gather to rank 0 (the only collective of the path);
  C4  drill 1000 polygons x 365 slices, reference-order (bit-exact) and
      wave-split modes, polygons dealt largest-first round-robin to ranks;
  C5  80 MODIS overview tiles with QA masks: tiles/s and p50 tile latency.
`roofline` is the dominant kernel of C2 (HIP events on its launch stream);
`cpu_baseline` the oracle (C restatement, test infrastructure) on the box's
host cores, rank 0, N=1 only.
"""
from __future__ import annotations

import argparse
import gc
import hashlib
import json
import os
import socket
import subprocess
import sys
import time
import traceback

ROOT = os.path.dirname(os.path.abspath(__file__))


def _launch_ranks(n: int) -> int:
    """`bench.py --gpus N` started without a launcher (no WORLD_SIZE in the
    environment): start N rank processes of this script -- before anything
    here has imported torch or touched a GPU, and as children (never exec) --
    each with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT, wait
    for them, relay rank 0's JSON line and fail if any rank fails (the others
    are then terminated, so none waits forever at a barrier)."""
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env,
                                      stdout=subprocess.PIPE if r == 0 else subprocess.DEVNULL))
    import threading
    out0 = []
    reader = threading.Thread(target=lambda: out0.append(procs[0].stdout.read()), daemon=True)
    reader.start()
    failed = 0
    live = set(range(n))
    while live:
        for r in sorted(live):
            rc = procs[r].poll()
            if rc is None:
                continue
            live.discard(r)
            if rc != 0 and not failed:
                failed = rc
                for q in live:
                    procs[q].terminate()
        time.sleep(0.05)
    reader.join()
    out0 = b"".join(out0)
    sys.stdout.write(out0.decode())
    sys.stdout.flush()
    return failed


if __name__ == "__main__" and "WORLD_SIZE" not in os.environ:
    _pre = argparse.ArgumentParser(add_help=False)
    _pre.add_argument("--gpus", type=int, default=1)
    _n = _pre.parse_known_args()[0].gpus
    if _n > 1:
        sys.exit(_launch_ranks(_n))

import numpy as np  # noqa: E402
import torch  # noqa: E402

sys.path.insert(0, ROOT)

import gsky_amd  # noqa: E402
from gsky_amd import GranuleSet, Mask, Palette, PipelinedBatch, ScaleParams, TileBatch, partition, synth  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
METRIC = "reprojected+merged output Mpix/s (whole node) at 1/2/4/8 MI355X; p50 tile ms"
CLIP = (-3.4028234663852886e38, 3.4028234663852886e38)   # ows.go:1373-1381


# ---------------------------------------------------------------- plumbing
class Ctx:
    """Rank context: one process per GPU (RANK / LOCAL_RANK / WORLD_SIZE from
    the launcher or from _launch_ranks), RCCL ("nccl") process group; the
    CPU dry run (tests) uses gloo and no device."""

    def __init__(self, dry_run: bool = False):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local = int(os.environ.get("LOCAL_RANK", "0"))
        self.dry = dry_run
        self.dist = None
        if self.world > 1:
            import torch.distributed as dist
            if dry_run:
                dist.init_process_group("gloo")
            else:
                torch.cuda.set_device(self.local)
                dist.init_process_group("nccl", device_id=torch.device("cuda", self.local))
            self.dist = dist
        elif not dry_run:
            torch.cuda.set_device(0)
        self.device = torch.device("cpu") if dry_run else torch.device("cuda", torch.cuda.current_device())

    def sync(self):
        if not self.dry:
            torch.cuda.synchronize()

    def barrier(self):
        if self.dist:
            self.dist.barrier()

    def max_over_ranks(self, x: float) -> float:
        if not self.dist:
            return x
        t = torch.tensor([x], dtype=torch.float64, device=self.device)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def ranks_seen(self):
        """Every rank's index, gathered (proves the N processes joined)."""
        if not self.dist:
            return [self.rank]
        t = torch.tensor([self.rank], dtype=torch.int64, device=self.device)
        out = [torch.zeros_like(t) for _ in range(self.world)]
        self.dist.all_gather(out, t)
        return [int(x.item()) for x in out]

    def timed(self, step, steps: int, warmup: int) -> float:
        """W untimed steps, then K steps bracketed by barrier + synchronize;
        returns the max-over-ranks seconds of the K steps.  Each timed step is
        also bracketed by HIP events on the current (launch) stream, so an
        outlier step is recorded (self.step_stats: min / median / max ms of
        this rank's steps) instead of averaged away."""
        for _ in range(warmup):
            step()
        self.sync()
        self.barrier()
        self.sync()
        # no collector pause inside the timed region: the steps only launch
        # (host-side stalls there stretch the wall time while the per-step
        # device times stay normal -- round 5's one-off 16.8 ms C5 step)
        gc.collect()
        gc.disable()
        evs = None
        if not self.dry:
            s = torch.cuda.current_stream()
            evs = [torch.cuda.Event(enable_timing=True) for _ in range(steps + 1)]
        t0 = time.perf_counter()
        if evs:
            evs[0].record(s)
        for k in range(steps):
            step()
            if evs:
                evs[k + 1].record(s)
        self.sync()
        self.barrier()
        wall = time.perf_counter() - t0
        gc.enable()
        dt = self.max_over_ranks(wall)
        if evs and steps > 0:
            ms = [evs[k].elapsed_time(evs[k + 1]) for k in range(steps)]
            self.step_stats = {"min": round(float(np.min(ms)), 4), "median": round(float(np.median(ms)), 4),
                               "max": round(float(np.max(ms)), 4)}
        else:
            self.step_stats = None
        return dt


def event_ms(fn, reps: int = 10) -> float:
    """Mean device time of fn() on the current stream (HIP events)."""
    s = torch.cuda.current_stream()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ts = []
    for _ in range(reps):
        ev[0].record(s)
        fn()
        ev[1].record(s)
        torch.cuda.synchronize()
        ts.append(ev[0].elapsed_time(ev[1]))
    return float(np.mean(ts))


block_part = partition.tile_blocks     # contiguous tile blocks (gsky_amd/partition.py)
sub_config = partition.sub_config      # a rank uploads only the granules its tiles touch


def build_granules(cfg, device):
    """The config's granules uploaded once (HBM-resident for every batch)."""
    gs = GranuleSet(device)
    for g in cfg.granules:
        gs.add(torch.from_numpy(np.ascontiguousarray(g.data)), g.geot, g.srs, g.nodata,
               [torch.from_numpy(np.ascontiguousarray(o)) for o in g.overviews], g.timestamp, g.polygon,
               g.namespace)
    return gs


def build_batch(cfg, device, chunks: int = 0, gs=None, ids=None):
    """A TileBatch (or PipelinedBatch) of the config's tiles -- or of tiles
    `ids` only -- over `gs` (uploaded here when not given)."""
    gs = gs if gs is not None else build_granules(cfg, device)
    mask = Mask(cfg.mask["id"], cfg.mask.get("value", ""), cfg.mask.get("bit_tests", []),
                cfg.mask.get("inclusive", False)) if cfg.mask else None
    tiles = cfg.tiles if ids is None else [cfg.tiles[i] for i in ids]
    pairs = cfg.pairs if ids is None else [cfg.pairs[i] for i in ids]
    if chunks > 1:
        return PipelinedBatch(gs, cfg.dst_srs, tiles, pairs, cfg.namespaces, mask, n_chunks=chunks)
    return TileBatch(gs, cfg.dst_srs, tiles, pairs, cfg.namespaces, mask)


def tile_latency(ctx, cfg, gs, sp, pal, ids, reps):
    """Host wall time of one-tile requests (plan + render + synchronize; the
    reference serves every GetMap tile as its own request, ows.go:257-524),
    granules resident: list of ms."""
    lat = []
    for i in ids:
        one = build_batch(cfg, ctx.device, gs=gs, ids=[i])
        for _ in range(3):
            one.render(sp, pal)
        torch.cuda.synchronize()
        for _ in range(reps):
            t0 = time.perf_counter()
            one.render(sp, pal)
            torch.cuda.synchronize()
            lat.append((time.perf_counter() - t0) * 1e3)
        del one
    return lat


def host_cores():
    """Cores this process may use: the cgroup CPU quota (the GPU box grants a
    16-core share of a larger machine) or the affinity mask."""
    n = len(os.sched_getaffinity(0))
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            n = min(n, max(1, int(int(q) // int(p))))
    except Exception:
        pass
    return n


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except Exception:
        pass
    return "unknown"


def lib_sha():
    h = hashlib.sha256()
    with open(os.path.join(ROOT, "gsky_amd", "libgskyhip.so"), "rb") as f:
        h.update(f.read())
    return h.hexdigest()[:16]


def pmc_traffic(name: str):
    """HBM bytes per launch from a committed PMC pass of THIS library build
    (profiles/pmc_<name>.json records the lib hash it was measured on)."""
    p = os.path.join(ROOT, "profiles", "pmc_%s.json" % name)
    try:
        d = json.load(open(p))
        if d.get("lib_sha16") == lib_sha():
            return d.get("hbm_bytes_per_launch")
    except Exception:
        pass
    return None


def oracle_render(O, cfg, threads):
    from tests.helpers import oracle_render as orr
    return orr(O, cfg, n_threads=threads)


# ---------------------------------------------------------------- C2 (headline)
def run_c2(ctx: Ctx, args):
    full = synth.config_c2()
    ids = block_part(len(full.tiles), ctx.rank, ctx.world, partition.tile_cost(full.pairs))
    cfg = sub_config(full, ids)
    gs = build_granules(cfg, ctx.device)
    batch = build_batch(cfg, ctx.device, gs=gs)
    sp, pal = ScaleParams(*cfg.scale), Palette(cfg.palette, True)
    # the timed step: the batch in chunks on two streams, so each chunk's
    # planning kernels run under the previous chunk's render (PipelinedBatch)
    step_batch = build_batch(cfg, ctx.device, chunks=args.c2_chunks, gs=gs) if args.c2_chunks > 1 else batch
    for bb in (batch, step_batch):
        bb.render(sp, pal)
        torch.cuda.synchronize()
        if bb.status() != 0:
            raise RuntimeError("render status %d" % bb.status())
    dt = ctx.timed(lambda: step_batch.render(sp, pal), args.steps, args.warmup)
    total_px = full.out_pixels * args.steps
    plan_ms = event_ms(lambda: batch.render(sp, pal, phase=1), max(3, args.steps))
    render_ms = event_ms(lambda: batch.render(sp, pal, phase=2), max(3, args.steps))
    # algorithmic bytes of rank 0's launch: the distinct
    # source elements its tiles' windows pick (gskyhip_render_touched; at
    # N=1 nearly all of the 0.512 GB) + RGBA out
    src, src_lines = batch.touched_bytes()
    abytes = int(src + cfg.out_pixels * 4)
    achieved = abytes / (render_ms / 1e3) / 1e9
    # p50 GetMap tile latency: tiles the index gives at least one granule
    # (evenly spaced over those of the rank's block), each as its own
    # request; tiles with no granule (transparent, no planning) apart
    covered = [i for i in range(len(ids)) if cfg.pairs[i]]
    empty = [i for i in range(len(ids)) if not cfg.pairs[i]]
    lat_ids = [covered[k] for k in range(0, len(covered), max(1, len(covered) // args.c2_lat_tiles))][
        : args.c2_lat_tiles]
    lat = tile_latency(ctx, cfg, gs, sp, pal, lat_ids, args.c2_lat_reps) if lat_ids else [float("nan")]
    emp_ids = [empty[k] for k in range(0, len(empty), max(1, len(empty) // 8))][:8]
    lat_e = tile_latency(ctx, cfg, gs, sp, pal, emp_ids, args.c2_lat_reps) if emp_ids else [float("nan")]
    out = {
        "value": round(total_px / dt / 1e6, 1), "ms_per_step": round(dt / args.steps * 1e3, 4),
        "step_ms": ctx.step_stats,
        "p50_tile_ms": round(float(np.percentile(lat, 50)), 4),
        "p99_tile_ms": round(float(np.percentile(lat, 99)), 4),
        "p50_timing": "C2 one-tile GetMap requests over tiles with >= 1 granule (%d of the %d such tiles, evenly "
                      "spaced, x %d reps, rank 0): host wall of plan + render + synchronize, granules resident in "
                      "HBM" % (len(lat_ids), len(covered), args.c2_lat_reps),
        "p50_empty_tile_ms": round(float(np.percentile(lat_e, 50)), 4),
        "empty_tiles": "%d of the %d tiles have no granule (transparent RGBA, no pair planning); %d timed"
                       % (len(empty), len(ids), len(emp_ids)),
        "config": {"workload": "C2: %d x 512x512 EPSG:3857 tiles from %d EPSG:3577 int16 4000x4000 granules, "
                               "nearest, time-ordered merge + scale + palette" % (len(full.tiles), len(full.granules)),
                   "tiles_per_step": len(full.tiles), "tiles_per_rank": len(ids), "pairs_rank0": batch.n_pairs,
                   "parallelism": "tile blocks over %d rank(s) (contiguous, balanced by 1 + pairs per tile, "
                                  "granules per rank)" % ctx.world,
                   "pipeline": "%d chunks on 2 HIP streams (plan of chunk k+1 under render of chunk k)"
                               % args.c2_chunks if args.c2_chunks > 1 else "one batch, one stream"},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": pmc_traffic("render_c2")
                     if ctx.world == 1 else None,
                     "kernel": "render_nn_kernel<int16> + render_general_kernel (phase 2, one batch, rank 0)",
                     "kernel_ms": round(render_ms, 4), "plan_ms": round(plan_ms, 4),
                     "algorithmic_bytes_per_launch": abytes, "source_bytes": int(src),
                     "source_line_bytes": int(src_lines),
                     "bytes": "distinct source elements the tiles' windows pick (gskyhip_render_touched) x 2 B "
                              "+ 4 B RGBA per output pixel; source_line_bytes: the 128-B lines holding them",
                     "lib_sha16": lib_sha()},
    }
    if ctx.rank == 0 and args.png_tiles > 0:
        # EncodePNG's png.Encode (ogc_encoders.go:139) of rendered C2 tiles:
        # colour type + Go's filter rows and the deflate (LZ77 + per-tile Huffman codes) on the GPU, PNG framing on host threads
        from gsky_amd.encode import encode_png
        rgba = batch.render(sp, pal)
        sample = [covered[k] for k in range(0, len(covered), max(1, len(covered) // args.png_tiles))][
            : args.png_tiles]
        sub = rgba[torch.tensor(sample, device=rgba.device)].contiguous()
        sizes = [batch.tile_sizes[i] for i in sample]
        threads = host_cores()
        encode_png(sub[:2], sizes[:2], n_threads=threads)                   # warm
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        pngs = encode_png(sub, sizes, n_threads=threads)
        pt = time.perf_counter() - t0
        raw = sum(w * h * 4 for w, h in sizes)
        # fixed Huffman codes only (round 4's first GPU deflate) on the same tiles
        os.environ["GSKYHIP_PNG_FIXED"] = "1"
        try:
            t0 = time.perf_counter()
            fp = encode_png(sub, sizes, n_threads=threads)
            ft = time.perf_counter() - t0
        finally:
            del os.environ["GSKYHIP_PNG_FIXED"]
        # the round-3 path beside it: zlib level 6 on the host threads
        zs = sub[: max(2, len(sample) // 4)]
        os.environ["GSKYHIP_PNG_ZLIB"] = "1"
        try:
            t0 = time.perf_counter()
            zp = encode_png(zs, sizes[: zs.shape[0]], n_threads=threads)
            zt = time.perf_counter() - t0
        finally:
            del os.environ["GSKYHIP_PNG_ZLIB"]
        out["png"] = {"tiles": len(sample), "threads": threads, "tiles_per_s": round(len(sample) / pt, 1),
                      "rgba_MB_per_s": round(raw / pt / 1e6, 1), "png_bytes_mean": int(np.mean([len(b) for b in pngs])),
                      "projected_batch_s": round(len(ids) / (len(sample) / pt), 3),
                      "fixed_codes": {"tiles_per_s": round(len(sample) / ft, 1),
                                      "png_bytes_mean": int(np.mean([len(b) for b in fp]))},
                      "zlib_host": {"tiles": int(zs.shape[0]), "tiles_per_s": round(zs.shape[0] / zt, 1),
                                    "png_bytes_mean": int(np.mean([len(b) for b in zp])),
                                    "same_tiles_gpu_bytes_mean": int(np.mean([len(b) for b in pngs[: zs.shape[0]]]))},
                      "timing": "gskyhip_encode_png of %d covered C2 tiles already rendered in HBM: GPU colour-type "
                                "+ filter pass, GPU deflate (LZ77 at run / pixel / row / diagonal distances with one-step lazy matching, tokens searched once; per-tile dynamic Huffman codes or the fixed ones where "
                                "shorter) + IDAT CRC-32, PNG framing on "
                                "%d host threads, host wall; zlib_host = the same tiles through host zlib level 6"
                                % (len(sample), threads)}
        del sub, rgba
    if ctx.rank == 0 and ctx.world == 1 and not args.no_cpu:
        from oracle import oracle as O
        cores = host_cores()
        oracle_render(O, synth.subset(full, [0, 1]), cores)                 # warm
        runs = []
        for _ in range(args.cpu_runs):
            t0 = time.perf_counter()
            oracle_render(O, full, cores)
            runs.append(time.perf_counter() - t0)
        one = synth.subset(full, list(range(0, 4096, 16)))                   # 256 tiles
        t0 = time.perf_counter()
        oracle_render(O, one, 1)
        t1 = time.perf_counter() - t0
        med = float(np.median(runs))
        out["cpu_baseline"] = {
            "value": round(full.out_pixels / med / 1e6, 2), "unit": "Mpix/s", "cores": cores, "kind": "port",
            "one_core_value": round(one.out_pixels / t1 / 1e6, 2),
            "cpu": cpu_model(), "runs_s": [round(r, 3) for r in runs],
            "sample": "all 4096 C2 tiles rendered by oracle/ (C restatement of warp_operation_fast + merge + "
                      "Scale + palette) on %d threads = the box's CPU share (cgroup quota), median of %d runs; "
                      "1-core figure on 256 tiles" % (cores, args.cpu_runs)}
    del batch, step_batch, gs
    return out


# ---------------------------------------------------------------- C1
def run_c1(ctx: Ctx, args):
    cfg = synth.config_c1()
    b = build_batch(cfg, ctx.device)
    sp = ScaleParams(*cfg.scale)
    for _ in range(10):
        b.render(sp)
    torch.cuda.synchronize()
    ts = []
    for _ in range(args.c1_reps):
        t0 = time.perf_counter()
        b.render(sp)
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t0) * 1e3)
    # the same request served from a captured HIP graph (RenderGraph): tile
    # descriptor upload + one replay + synchronize per request
    rg = b.graph(sp)
    gts = []
    for _ in range(args.c1_reps):
        t0 = time.perf_counter()
        b.set_tiles(cfg.tiles)
        rg.replay()
        torch.cuda.synchronize()
        gts.append((time.perf_counter() - t0) * 1e3)
    # the replay alone (the same request again, no descriptor upload): what
    # the graph costs beside the upload (verdict r4: graph slower than eager)
    rts = []
    for _ in range(args.c1_reps):
        t0 = time.perf_counter()
        rg.replay()
        torch.cuda.synchronize()
        rts.append((time.perf_counter() - t0) * 1e3)
    ups = []
    for _ in range(args.c1_reps):
        t0 = time.perf_counter()
        b.set_tiles(cfg.tiles)
        torch.cuda.synchronize()
        ups.append((time.perf_counter() - t0) * 1e3)
    out = {"workload": "C1: one 256x256 EPSG:3857 tile from a 3600x1800 EPSG:4326 f32 granule, nearest, scale",
           "p50_tile_ms": round(float(np.percentile(ts, 50)), 4), "p99_tile_ms": round(float(np.percentile(ts, 99)), 4),
           "reps": args.c1_reps, "timing": "host wall per call incl. launch + synchronize",
           "p50_tile_ms_graph": round(float(np.percentile(gts, 50)), 4),
           "p99_tile_ms_graph": round(float(np.percentile(gts, 99)), 4),
           "graph_timing": "host wall per request: tile descriptor upload + HIP graph replay + synchronize",
           "p50_graph_replay_only_ms": round(float(np.percentile(rts, 50)), 4),
           "p50_descriptor_upload_ms": round(float(np.percentile(ups, 50)), 4)}
    if ctx.rank == 0 and ctx.world == 1 and not args.no_cpu:
        from oracle import oracle as O
        cts = []
        for _ in range(args.c1_cpu_reps):
            t0 = time.perf_counter()
            oracle_render(O, cfg, 1)
            cts.append((time.perf_counter() - t0) * 1e3)
        out["cpu_p50_tile_ms"] = round(float(np.percentile(cts, 50)), 4)
        out["cpu_p99_tile_ms"] = round(float(np.percentile(cts, 99)), 4)
        out["cpu"] = "oracle/, 1 thread (one gsky-gdal-process equivalent), %d reps" % args.c1_cpu_reps
    return out


# ---------------------------------------------------------------- C3
def run_c3(ctx: Ctx, args):
    from gsky_amd import coverage
    cfg = synth.config_c3()
    W, H = cfg.out_w, cfg.out_h
    chunks = coverage.chunk_requests(cfg.bbox, W, H)
    nrows = coverage.n_chunk_rows(chunks)
    rows = [coverage.band_of_rank(nrows, r, ctx.world) for r in range(ctx.world)]
    extents = [coverage.band_extent(chunks, rw) for rw in rows]
    sel = [c for c in chunks if rows[ctx.rank][0] <= c.row < rows[ctx.rank][1]]
    sub = synth.SynthConfig("C3", cfg.granules, cfg.dst_srs, [(c.bbox, c.width, c.height) for c in sel],
                            [cfg.index_chunk(c.bbox) for c in sel], cfg.namespaces, cfg.scale, None, cfg.resample)
    sub = sub_config(sub, list(range(len(sel))))
    b = build_batch(sub, ctx.device)
    sp = ScaleParams(*cfg.scale)
    top, bottom = extents[ctx.rank]

    # rank 0 renders its band in place, as rows of the coverage the others'
    # bands are received into (no assembly copy)
    full = torch.empty((H, W), dtype=torch.float32, device=ctx.device) if ctx.rank == 0 and ctx.world > 1 else None
    band = full[top:bottom] if full is not None else torch.empty((bottom - top, W), dtype=torch.float32,
                                                                   device=ctx.device)
    offs = torch.tensor(coverage.band_offsets(sel, top, W), dtype=torch.int64, device=ctx.device)

    def render():   # chunks straight into the band at their offsets (gskyhip_render_coverage)
        return b.render_coverage(sp, band, offs, resample=cfg.resample)

    def step():
        render()
        if ctx.world > 1:
            coverage.gather_coverage(band, extents, H, W, out=full)
        return band

    dt = ctx.timed(step, args.c3_steps, 1)
    # roofline of the band kernel alone (phase 2, planning already in the
    # workspace), as for C2; planning timed beside it
    plan_ms = event_ms(lambda: b.render_coverage(sp, band, offs, resample=cfg.resample, phase=1), 3)
    render_ms = event_ms(lambda: b.render_coverage(sp, band, offs, resample=cfg.resample, phase=2), 3)
    gather_ms = None
    if ctx.world > 1:
        band = step()
        torch.cuda.synchronize()
        gather_ms = ctx.max_over_ranks(event_ms(lambda: coverage.gather_coverage(band, extents, H, W, out=full), 3))
    src = sum(cfg.granules[0].data.nbytes for _ in sub.granules)
    abytes = src + sub.out_pixels * 4
    ach = abytes / (render_ms / 1e3) / 1e9
    out = {"workload": "C3: WCS GetCoverage %dx%d float32 bilinear EPSG:4326->3857 mosaic from %d granules, "
                       "%d chunks of <=1024^2 (ows.go:817-831)" % (W, H, len(cfg.granules), len(chunks)),
           "value": round(W * H * args.c3_steps / dt / 1e6, 1), "unit": "Mpix/s", "ms_per_step": round(dt / args.c3_steps * 1e3, 3),
           "step_ms": ctx.step_stats,
           "step": "render own chunk rows straight into the band" + (" + RCCL gather to rank 0"
                                                                      if ctx.world > 1 else ""),
           "chunk_rows_rank0": rows[0], "gather_ms": round(gather_ms, 3) if gather_ms is not None else None,
           "roofline": {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": round(ach / HBM_PEAK_GBS, 4),
                        "kernel": "render_bil_kernel + render_general_kernel (phase 2, rank 0)",
                        "kernel_ms": round(render_ms, 4), "plan_ms": round(plan_ms, 4),
                        "algorithmic_bytes_per_launch": int(abytes),
                        "traffic": pmc_traffic("bil_c3")}}
    if ctx.rank == 0 and ctx.world == 1 and not args.no_cpu:
        from oracle import oracle as O
        ids = list(range(0, len(chunks), max(1, len(chunks) // 16)))[:16]
        cs = synth.subset(cfg, ids)
        cores = host_cores()
        t0 = time.perf_counter()
        oracle_render(O, cs, cores)
        ct = time.perf_counter() - t0
        out["cpu_baseline"] = {"value": round(cs.out_pixels / ct / 1e6, 2), "unit": "Mpix/s", "cores": cores,
                               "kind": "port", "sample": "%d of the %d chunks by oracle/ (bilinear warp + merge), "
                                                         "%d threads" % (len(ids), len(chunks), cores)}
    del b
    return out


# ---------------------------------------------------------------- C4
def c4_stack(n_bands, size, device):
    """The C4 time stack built in HBM, time-innermost, slice by slice from
    synth.c4_band (per-(pixel, slice) U(0, 0.05) noise and 5 % nodata,
    SURVEY 8d)."""
    from gsky_amd import drill
    ts = (n_bands + 31) // 32 * 32   # 128-byte aligned pixel rows (gsky_amd.drill.DrillStack)
    st = torch.zeros((size, size, ts), dtype=torch.float32, device=device)
    for t0 in range(0, n_bands, 16):
        bs = synth._pmap(lambda t: synth.c4_band(t, size, n_bands), range(t0, min(n_bands, t0 + 16)))
        for k, b in enumerate(bs):
            st[:, :, t0 + k] = torch.from_numpy(b).to(device)
    return drill.DrillStack.from_time_innermost(st, n_bands, -9999.0)


def run_c4(ctx: Ctx, args):
    """C4 through the product: GeoJSON polygons -> getDrillFileDescriptor
    windows + ALL_TOUCHED masks on the GPU (gskyhip_drill_descriptors_device)
    -> readData (compaction + reduction) over the HBM time stack."""
    from gsky_amd import drill
    size, n_bands = 2048, 365
    _, _, geoms = synth.c4_polygons(size, 1000)
    wins, _ = drill.drill_windows(geoms, "EPSG:4326", synth.C4_GT, size, size)
    area = [int(w[2]) * int(w[3]) for w in wins]
    mine = partition.drill_assignment(area, ctx.rank, ctx.world)   # largest window first, round-robin
    my_geoms = [geoms[p] for p in mine]
    st = c4_stack(n_bands, size, ctx.device)

    def describe():
        return drill.drill_dataset(my_geoms, "EPSG:4326", synth.C4_GT, size, size, ctx.device)
    mb, status = describe()
    torch.cuda.synchronize()
    if (status != 0).any():
        raise RuntimeError("C4 descriptors: %d polygons failed" % int((status != 0).sum()))
    dts = []
    for _ in range(5):
        t0 = time.perf_counter()
        describe()
        torch.cuda.synchronize()
        dts.append((time.perf_counter() - t0) * 1e3)
    inside = int((mb.masks == 255).sum().item())
    px = int(sum(int(w[2]) * int(w[3]) for w in mb.win.cpu().numpy()))
    res = {}
    for name, mode in (("reference_order", drill.REFERENCE_ORDER), ("wave_split", drill.WAVE_SPLIT)):
        dt = ctx.timed(lambda: drill.read_data(st, mb, *CLIP, mode=mode), args.steps, args.warmup)
        k_ms = event_ms(lambda: drill.read_data(st, mb, *CLIP, mode=mode), 5)
        abytes = inside * n_bands * 4 + px
        ach = abytes / (k_ms / 1e3) / 1e9
        res[name] = {"value": round(len(geoms) * n_bands * args.steps / dt, 1), "unit": "polygon-slices/s",
                     "ms_per_step": round(dt / args.steps * 1e3, 4), "step_ms": ctx.step_stats,
                     "roofline": {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                  "frac": round(ach / HBM_PEAK_GBS, 4), "kernel_ms": round(k_ms, 4),
                                  "kernel": "drill compaction + %s reduction (rank 0)" % name,
                                  "algorithmic_bytes_per_launch": int(abytes)}}
    # decileCount = 9 (drill.go:229-273): radix selection of the picks per (polygon, slice)
    if not args.no_deciles:
        dt_dec = ctx.timed(lambda: drill.read_data(st, mb, *CLIP, decile_count=9), 3, 1)
        k_dec = event_ms(lambda: drill.read_data(st, mb, *CLIP, decile_count=9), 3)
        # algorithmic bytes: the mean pass (in-mask values + mask bytes) + its
        # band-major write of the in-mask values + the select's read of that copy
        vals = inside * n_bands * 4
        dbytes = 3 * vals + px
        dach = dbytes / (k_dec / 1e3) / 1e9
        res["deciles"] = {"value": round(len(mine) * n_bands * 3 / dt_dec, 1), "unit": "polygon-slices/s",
                          "ms_per_step": round(dt_dec / 3 * 1e3, 3), "step_ms": ctx.step_stats,
                          "decile_count": 9,
                          "step": "readData with decileCount 9: mean pass writing the band-major rows + radix select "
                                  "(rank 0)",
                          "roofline": {"bound": "hbm", "achieved": round(dach, 1), "peak": HBM_PEAK_GBS,
                                       "unit": "GB/s", "frac": round(dach / HBM_PEAK_GBS, 4),
                                       "kernel_ms": round(k_dec, 4),
                                       "kernel": "drill compaction + mean with band-major write + decile select (rank 0)",
                                       "algorithmic_bytes_per_launch": int(dbytes),
                                       "bytes": "mean pass (in-mask values + mask) + its band-major write + the "
                                                "select's read of the in-mask values"}}
    out = {"workload": "C4: WPS drill zonal mean, 1000 star polygons (GeoJSON, EPSG:4326) x 365 daily f32 slices "
                       "of 2048^2, product windows + ALL_TOUCHED masks on the GPU, clip +-MaxFloat32",
           "polygons_rank0": len(mine), "in_mask_px_rank0": inside,
           "descriptors_ms": round(float(np.median(dts)), 3),
           "descriptors_timing": "host geometry (parse, envelope, window) + GPU rasterization of rank 0's "
                                 "polygons, median of 5", **res}
    if ctx.rank == 0 and ctx.world == 1 and not args.no_cpu:
        from concurrent.futures import ThreadPoolExecutor

        from oracle import oracle as O
        wn = mb.win.cpu().numpy()
        offs = mb.mask_off.cpu().numpy()
        mk = mb.masks.cpu().numpy()
        order = sorted(range(len(mine)), key=lambda p: -int(wn[p][2]) * int(wn[p][3]))
        ids = order[:: max(1, len(order) // args.c4_cpu_polys)][: args.c4_cpu_polys]
        subs, msk = {}, {}
        for p in ids:
            x0, y0, w, h = (int(v) for v in wn[p])
            subs[p] = st.stack[y0:y0 + h, x0:x0 + w, :n_bands].permute(2, 0, 1).contiguous().cpu().numpy()
            msk[p] = mk[offs[p]:offs[p] + w * h].reshape(h, w)
        cores = host_cores()

        def one(p):
            return O.drill_read_data(subs[p], msk[p], -9999.0, CLIP[0], CLIP[1], 0, 1)
        t0 = time.perf_counter()
        with ThreadPoolExecutor(cores) as ex:
            list(ex.map(one, ids))
        ct = time.perf_counter() - t0
        out["cpu_baseline"] = {"value": round(len(ids) * n_bands / ct, 1), "unit": "polygon-slices/s",
                               "cores": cores, "kind": "port",
                               "sample": "%d polygons (every %d-th by window size) x %d slices, oracle readData on "
                                         "the product masks, %d threads"
                                         % (len(ids), max(1, len(order) // args.c4_cpu_polys), n_bands, cores)}
    del st
    return out


# ---------------------------------------------------------------- C5
def run_c5(ctx: Ctx, args):
    full = synth.config_c5()
    ids = block_part(len(full.tiles), ctx.rank, ctx.world, partition.tile_cost(full.pairs))
    cfg = sub_config(full, ids)
    gs = build_granules(cfg, ctx.device)
    b = build_batch(cfg, ctx.device, gs=gs)
    sp = ScaleParams(*cfg.scale)
    steps = args.c5_steps or args.steps
    dt = ctx.timed(lambda: b.render(sp), steps, args.warmup)
    plan_ms = event_ms(lambda: b.render(sp, phase=1), max(3, args.steps))
    render_ms = event_ms(lambda: b.render(sp, phase=2), max(3, args.steps))
    # algorithmic bytes of the render launch: the distinct
    # source elements every pair's window pixels pick at the picked level,
    # data and QA rasters alike (gskyhip_render_touched), x element bytes,
    # + 4 B RGBA per output pixel; the 128-B lines holding them beside it
    src, src_lines = b.touched_bytes()
    abytes = int(src + cfg.out_pixels * 4)
    achieved = abytes / (render_ms / 1e3) / 1e9
    # p50 single-tile latency: each sampled tile as its own request
    lat = tile_latency(ctx, cfg, gs, sp, None, list(range(0, len(cfg.tiles), max(1, len(cfg.tiles) // 8))), 10)
    out = {"workload": "C5: 80 512x512 EPSG:3857 overview tiles (z4+z5) from 256 MODIS sinusoidal int16 granules + "
                       "256 QA mask granules with overview pyramids, mask 00000001, grey scaling",
           "tiles_per_s": round(len(full.tiles) * steps / dt, 1),
           "value": round(full.out_pixels * steps / dt / 1e6, 1), "unit": "Mpix/s",
           "ms_per_step": round(dt / steps * 1e3, 4), "steps": steps, "step_ms": ctx.step_stats,
           "p50_tile_ms": round(float(np.percentile(lat, 50)), 4),
           "p50_timing": "host wall of a one-tile request (plan + render + synchronize), rank 0",
           "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": round(achieved / HBM_PEAK_GBS, 4),
                        "traffic": pmc_traffic("render_c5") if ctx.world == 1 else None,
                        "kernel": "render_nn_kernel<int16, mask> + render_general_kernel (phase 2, rank 0)",
                        "kernel_ms": round(render_ms, 4), "plan_ms": round(plan_ms, 4),
                        "algorithmic_bytes_per_launch": abytes, "source_bytes": int(src),
                        "source_line_bytes": int(src_lines),
                        "bytes": "distinct source elements picked by every pair's window pixels (data and QA, "
                                 "picked overview level; gskyhip_render_touched) x element size, + 4 B RGBA per "
                                 "output pixel; source_line_bytes: the 128-B lines holding them", "lib_sha16": lib_sha()}}
    if ctx.rank == 0 and ctx.world == 1 and not args.no_cpu:
        from oracle import oracle as O
        cores = host_cores()
        t0 = time.perf_counter()
        oracle_render(O, full, cores)
        ct = time.perf_counter() - t0
        out["cpu_baseline"] = {"value": round(len(full.tiles) / ct, 2), "unit": "tiles/s", "cores": cores,
                               "kind": "port", "sample": "all 80 tiles by oracle/, %d threads" % cores}
    del b, gs
    return out


# ---------------------------------------------------------------- the per-node warp service
def run_service(ctx: Ctx, args):
    """The path GSKY calls: N worker processes (gsky-rpc's gsky-gdal-process
    pool, grpc-server/main.go:58) each sending C2 (tile, granule) warp
    requests through warp_operation_fast -> Unix socket -> gskyhipd, which
    batches across workers (service.cpp); the window bytes come back to the
    worker in host memory as warp.go:573-574 expects.  Beside it the oracle's
    warp_operation_fast on one thread per worker (the reference's CPU path)."""
    from concurrent.futures import ThreadPoolExecutor

    from gsky_amd import WarpService
    from gsky_amd.loadgen import service_load
    from gsky_amd.tiles import bbox_to_geot
    cfg = synth.config_c2()
    sock = "/tmp/gskyhip-bench-%d.sock" % os.getpid()
    svc = WarpService(sock, max_batch=64, window_us=args.svc_window_us)
    out = {"workload": "C2 (tile, granule) warp requests, 512x512 EPSG:3857 windows from 16 EPSG:3577 int16 "
                       "4000x4000 granules resident in the daemon's HBM; %d distinct requests dealt round-robin to "
                       "the workers, each worker one request at a time, cycling through its share: %d untimed "
                       "requests per worker, then %.1f s timed (steady state)" %
                       (args.svc_jobs, args.svc_warmup, args.svc_seconds),
           "daemon": "gskyhipd max_batch 64, window %d us (only while a batch is on the GPU), two batches in "
                     "flight, windows written by the GPU into each worker's shared reply arena" % args.svc_window_us}
    try:
        for k, g in enumerate(cfg.granules):
            svc.register_granule("/g/data/c2/g%d.tif" % k, 1, g.data, g.geot, "EPSG:3577", g.nodata, block=(256, 256))
        pairs = [(k, bb, w, h) for (bb, w, h), ks in zip(cfg.tiles, cfg.pairs) for k in ks]
        step = max(1, len(pairs) // args.svc_jobs)
        sel = pairs[::step][: args.svc_jobs]
        jobs = [("/g/data/c2/g%d.tif" % k, 1, list(bbox_to_geot(w, h, bb)), w, h, "EPSG:3857") for k, bb, w, h in sel]
        for n in (16, 64):
            s0 = svc.stats()
            r = service_load(sock, jobs, n, seconds=args.svc_seconds, warmup=args.svc_warmup)
            s1 = svc.stats()
            r["mean_batch"] = round((s1["requests"] - s0["requests"]) / max(1, s1["batches"] - s0["batches"]), 2)
            r["max_batch"] = s1["max_batch"]
            nb, nr = max(1, s1["batches"] - s0["batches"]), max(1, s1["requests"] - s0["requests"])
            r["daemon_dispatch_ms_mean"] = round((s1["batch_s"] - s0["batch_s"]) * 1e3 / nb, 3)
            r["daemon_resident_ms_mean"] = round((s1["resident_s"] - s0["resident_s"]) * 1e3 / nr, 3)
            r["daemon_batch_phases_ms_mean"] = {k: round((s1[k + "_s"] - s0[k + "_s"]) * 1e3 / nb, 3)
                                                for k in ("launch", "gpu_wait", "readback")}
            r["replies_in_place"] = s1["in_place"] - s0["in_place"]
            r["replies_copied"] = s1["copied"] - s0["copied"]
            out["workers_%d" % n] = r
    finally:
        svc.shutdown()
    if not args.no_cpu:
        from oracle import oracle as O
        cores = host_cores()
        aea, wm = O.crs("EPSG:3577"), O.crs("EPSG:3857")
        ogs = [O.make_granule(g.data, g.geot, g.nodata, block=(256, 256)) for g in cfg.granules]
        sub = sel[:: max(1, len(sel) // 256)]

        def one(job):
            k, bb, w, h = job
            O.warp(ogs[k], aea, wm, list(bbox_to_geot(w, h, bb)), w, h)
        with ThreadPoolExecutor(cores) as ex:
            list(ex.map(one, sub[:cores]))          # warm
            t0 = time.perf_counter()
            list(ex.map(one, sub))
            ct = time.perf_counter() - t0
        out["cpu_baseline"] = {"value": round(len(sub) / ct, 1), "unit": "requests/s", "cores": cores,
                               "kind": "port", "sample": "%d of the requests, oracle warp_operation_fast, one "
                                                         "thread per worker (%d)" % (len(sub), cores)}
    return out


def run_dry(ctx: Ctx, args):
    """CPU dry run of the launch / timing contract (tests): a trivial step per
    rank over gloo, timed like the real ones."""
    if ctx.rank == args.dry_fail_rank:
        raise SystemExit(3)   # a failing rank: the launcher must fail and stop the others
    x = torch.zeros(1 << 16)
    dt = ctx.timed(lambda: x.add_(1.0), args.steps, args.warmup)
    return {"value": round(ctx.world * (1 << 16) * args.steps / dt / 1e6, 3),
            "ms_per_step": round(dt / args.steps * 1e3, 4), "dry_run": True, "ranks": ctx.ranks_seen(),
            "config": {"workload": "dry run: 65536-element add per rank (launcher test)"}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--only", default="c2,c1,c3,c4,c5,svc", help="comma list of configs (c2 is the headline)")
    ap.add_argument("--svc-jobs", type=int, default=1024, help="service leg: C2 (tile, granule) requests per run")
    ap.add_argument("--svc-window-us", type=int, default=0,
                    help="service leg: gskyhipd batching window (taken only while a batch is on the GPU)")
    ap.add_argument("--svc-seconds", type=float, default=2.0, help="service leg: timed seconds per worker count")
    ap.add_argument("--svc-warmup", type=int, default=8, help="service leg: untimed requests per worker")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-c1", action="store_true", help="(compat) drop C1")
    ap.add_argument("--cpu-runs", type=int, default=5)
    ap.add_argument("--c1-reps", type=int, default=1000)
    ap.add_argument("--c1-cpu-reps", type=int, default=200)
    ap.add_argument("--c2-chunks", type=int, default=1, help="C2 step: tile chunks pipelined on 2 streams (1: one batch; measured no gain, profiles/r02o_*)")
    ap.add_argument("--c3-steps", type=int, default=3)
    ap.add_argument("--c5-steps", type=int, default=50,
                    help="C5 timed steps (0: --steps); a 0.33 ms step would carry the timed region's ~0.8 ms of "
                         "start / end latency at 10 steps")
    ap.add_argument("--c4-cpu-polys", type=int, default=160)
    ap.add_argument("--no-deciles", action="store_true", help="C4: skip the decileCount=9 line")
    ap.add_argument("--c2-lat-tiles", type=int, default=32, help="C2 p50: one-tile requests over this many tiles")
    ap.add_argument("--c2-lat-reps", type=int, default=10)
    ap.add_argument("--png-tiles", type=int, default=256, help="C2: PNG-encode this many rendered tiles (0: skip)")
    ap.add_argument("--dry-run", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--dry-fail-rank", type=int, default=-1, help=argparse.SUPPRESS)
    args = ap.parse_args()
    only = [s.strip().lower() for s in args.only.split(",") if s.strip()]
    if args.no_c1 and "c1" in only:
        only.remove("c1")
    ctx = Ctx(dry_run=args.dry_run)
    if ctx.world != args.gpus and ctx.rank == 0:
        print("bench.py: --gpus %d but WORLD_SIZE %d: reporting the %d ranks that joined" %
              (args.gpus, ctx.world, ctx.world), file=sys.stderr)
    out = {"metric": METRIC, "value": None, "unit": "Mpix/s", "n_gpus": ctx.world, "ranks_seen": None,
           "steps": args.steps, "warmup": args.warmup, "ms_per_step": None, "higher_is_better": True,
           "scaling": "strong", "vs_baseline": None, "dtype": "int16",
           "data": "synthetic (splitmix64 granules, SURVEY.md 8d)"}
    out["ranks_seen"] = len(ctx.ranks_seen())
    if args.dry_run:
        out.update(run_dry(ctx, args))
        only = []
    if "c2" in only:
        out.update(run_c2(ctx, args))
    configs = {}

    def settle():
        # between legs, outside every timed region: the previous leg's host
        # arrays and cached device blocks released, so a leg's timing never
        # overlaps the host's reclaim of the last one's (a C5 step once read
        # 13-17 ms instead of 0.6 after C4's CPU baseline freed its copies)
        gc.collect()
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
        time.sleep(0.2)
    for name, fn in (("C1", run_c1), ("C3", run_c3), ("C4", run_c4), ("C5", run_c5), ("service", run_service)):
        if name.lower() in only or (name == "service" and "svc" in only):
            settle()
        if name == "service":
            if "svc" not in only or ctx.world > 1:
                continue
            try:
                configs[name] = fn(ctx, args)
            except Exception as ex:   # noqa: BLE001
                traceback.print_exc()
                configs[name] = {"error": "%s: %s" % (type(ex).__name__, ex)}
            continue
        if name.lower() not in only:
            continue
        try:
            configs[name] = fn(ctx, args)
        except Exception as ex:   # an auxiliary config must not lose the headline line
            configs[name] = {"error": "%s: %s" % (type(ex).__name__, ex)}
            if ctx.rank == 0:
                traceback.print_exc()
        torch.cuda.empty_cache()
    if configs:
        out["configs"] = configs
    if ctx.rank == 0:
        print(json.dumps(out), flush=True)
    if ctx.dist:
        ctx.dist.destroy_process_group()


if __name__ == "__main__":
    main()
