#!/usr/bin/env python3
"""C4 measurement (BASELINE.json configs[3]): WPS drill zonal
mean over 1000 star polygons x 365 daily float32 slices of a 2048^2 EPSG:4326
grid, on one MI355X.  Prints one JSON line.

The stack is built directly in HBM in the time-innermost layout
([y][x][t_stride], synthetic: base(t) + noise(y, x) * (1 + (t mod 7)/100),
5 % nodata); polygons and ALL_TOUCHED masks come from
gsky_amd.synth.  Timed region: gskyhip_drill over all 1000 polygons (HIP
events on the launch stream).  Unit = polygon x time slice.
Algorithmic bytes = in-mask pixels x 365 x 4 B (masked-out window pixels are
never read) + 1 B of mask per window pixel.  cpu_baseline: the oracle (readData restatement, 1 thread) on a sample
of polygons, which is also checked bit for bit against the GPU result.

  python tools/bench_drill.py [--polys 1000] [--bands 365] [--size 2048]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from gsky_amd import drill, synth  # noqa: E402

HBM_PEAK_GBS = 8000.0


def build_stack(n_bands, size, device):
    idx = np.arange(size * size, dtype=np.uint64) + np.uint64(synth.SEED0 << 32)
    noise = (synth.uniform01(synth.splitmix64(idx)) * 0.05).astype(np.float32).reshape(size, size)
    nod = synth.uniform01(synth.splitmix64(idx + np.uint64(1 << 40))).reshape(size, size) < 0.05
    t = torch.arange(n_bands, dtype=torch.float64, device=device)
    base = (0.2 + 0.1 * torch.sin(2 * np.pi * t / 365.0)).float()
    fac = (1.0 + (t % 7) * 0.01).float()
    ts = (n_bands + 31) // 32 * 32   # 128-byte aligned pixel rows (gsky_amd.drill.DrillStack)
    st = torch.zeros((size, size, ts), dtype=torch.float32, device=device)
    nz = torch.from_numpy(noise).to(device)
    for y0 in range(0, size, 256):   # bounded temporaries
        st[y0:y0 + 256, :, :n_bands] = base + nz[y0:y0 + 256, :, None] * fac
    st[torch.from_numpy(nod).to(device)] = -9999.0
    return drill.DrillStack.from_time_innermost(st, n_bands, -9999.0)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--polys", type=int, default=1000)
    ap.add_argument("--bands", type=int, default=365)
    ap.add_argument("--size", type=int, default=2048)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--cpu-polys", type=int, default=40)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    geo = synth.config_c4(n_bands=1, size=args.size, n_polys=args.polys)
    st = build_stack(args.bands, args.size, dev)
    win, off, masks = drill.pack_masks(geo.windows, geo.masks, dev)
    clip = (-3.4028234663852886e38, 3.4028234663852886e38)   # ows.go:1373-1381
    for _ in range(args.warmup):
        drill.read_data(st, win, off, masks, *clip)
    torch.cuda.synchronize()
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record(s)
    for _ in range(args.steps):
        vals, cnts = drill.read_data(st, win, off, masks, *clip)
    e1.record(s)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / args.steps
    k_s = e0.elapsed_time(e1) / 1e3 / args.steps
    px = sum(w * h for (_, _, w, h) in geo.windows)
    inside = int(sum(int((m == 255).sum()) for m in geo.masks))
    # unique bytes a launch must move: the time vectors of in-mask pixels
    # (masked-out window pixels are never read) + every window mask byte
    abytes = inside * args.bands * 4 + px
    units = args.polys * args.bands

    # CPU baseline + bit-exact spot check on a polygon sample
    from oracle import oracle as O
    ids = np.linspace(0, args.polys - 1, min(args.cpu_polys, args.polys)).round().astype(int)
    subs = []
    for p in ids:
        x0, y0, w, h = geo.windows[p]
        subs.append(st.stack[y0:y0 + h, x0:x0 + w, :args.bands].permute(2, 0, 1).contiguous().cpu().numpy())
    gv, gc = vals.cpu().numpy(), cnts.cpu().numpy()
    c0 = time.perf_counter()
    exact = True
    for k, p in enumerate(ids):
        ev, ec = O.drill_read_data(subs[k], geo.masks[p], -9999.0, clip[0], clip[1], 0, 1)
        exact &= bool(np.array_equal(ec, gc[p]) and np.array_equal(ev.view(np.uint64), gv[p].view(np.uint64)))
    cdt = time.perf_counter() - c0
    out = {
        "metric": "drill zonal mean polygon-slices/s (C4)", "value": round(units / k_s, 1),
        "unit": "polygon-slices/s", "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(k_s * 1e3, 4), "wall_ms_per_step": round(wall * 1e3, 4), "higher_is_better": True,
        "dtype": "f32", "data": "synthetic (SURVEY.md 8d C4; stack built in HBM, time-innermost)",
        "config": {"workload": "C4: %d star polygons x %d daily f32 slices of %d^2, mean, ALL_TOUCHED masks"
                               % (args.polys, args.bands, args.size), "window_pixels": px, "in_mask_pixels": inside},
        "roofline": {"bound": "hbm", "achieved": round(abytes / k_s / 1e9, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(abytes / k_s / 1e9 / HBM_PEAK_GBS, 4), "kernel": "drill_kernel",
                     "algorithmic_bytes_per_launch": abytes},
        "cpu_baseline": {"value": round(len(ids) * args.bands / cdt, 1), "unit": "polygon-slices/s", "cores": 1,
                         "kind": "port", "sample": "%d polygons x %d slices, oracle readData, 1 thread"
                                                   % (len(ids), args.bands)},
        "spot_check_bit_exact": exact,
    }
    print(json.dumps(out))
    if not exact:
        sys.exit(1)


if __name__ == "__main__":
    main()
