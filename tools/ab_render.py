#!/usr/bin/env python3
"""Timing of the render phase of one config (phase-2 kernels only, HIP events
on the launch stream): the typed band kernels (default) or, with --generic,
the general kernels.  One JSON line.  With GSKYHIP_LIB=ab (the -DGSKYHIP_AB
build, gsky_amd/libgskyhip_ab.so) the A/B knobs of that build apply.
Used for rocprofv3 / PMC passes of the dominant kernel and to compare
variants; bench.py is the contract."""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import gsky_amd  # noqa: E402
from gsky_amd import synth  # noqa: E402
from tests.helpers import gpu_batch  # noqa: E402


def time_render(b, sp, pal, reps, resample=0):
    s = torch.cuda.current_stream()
    b.render(sp, pal, phase=1, resample=resample)
    for _ in range(3):
        b.render(sp, pal, phase=2, resample=resample)
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ts = []
    for _ in range(reps):
        ev[0].record(s)
        b.render(sp, pal, phase=2, resample=resample)
        ev[1].record(s)
        torch.cuda.synchronize()
        ts.append(ev[0].elapsed_time(ev[1]))
    return float(np.median(ts)), float(np.min(ts))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--config", default="c2", choices=["c2", "c5"])
    ap.add_argument("--generic", action="store_true", help="force the general kernels")
    ap.add_argument("--oracle", action="store_true", help="also count RGBA pixels differing from the oracle")
    ap.add_argument("--label", default="", help="label of the line (A/B knob settings)")
    args = ap.parse_args()
    cfg = synth.config_c2() if args.config == "c2" else synth.config_c5()
    b = gpu_batch(cfg)
    b.typed = not args.generic
    sp = gsky_amd.ScaleParams(*cfg.scale)
    pal = gsky_amd.Palette(cfg.palette, True) if cfg.palette else None
    med, mn = time_render(b, sp, pal, args.reps)
    rec = {"label": args.label, "config": args.config, "kernels": "generic" if args.generic else "typed",
           "lib": os.environ.get("GSKYHIP_LIB", "default"),
           "render_ms_median": round(med, 4), "render_ms_min": round(mn, 4)}
    if args.oracle:
        from oracle import oracle as O
        from tests.helpers import oracle_render
        exp = torch.from_numpy(oracle_render(O, cfg, n_threads=16)).to("cuda")
        out = b.render(sp, pal)
        torch.cuda.synchronize()
        rec["differ_from_oracle"] = int((out != exp).any(dim=-1).sum().item())
    print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
