#!/usr/bin/env python3
"""Where C2's band-kernel time goes, by tile class (round 6, VERDICT r05 item
2's model): the tiles of the C2 batch grouped by their number of granule
pairs (0 = no granule, 1 = one stack entry, 2-4 = seams between overlapping
granules); each class repeated to a full 4096-tile batch and timed alone
(phase 2, HIP events on the launch stream).  Prints one JSON line per class
plus the full batch, and the class-weighted prediction of the full batch."""
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
from tools.ab_render import time_render  # noqa: E402


def main():
    cfg = synth.config_c2()
    sp = gsky_amd.ScaleParams(*cfg.scale)
    pal = gsky_amd.Palette(cfg.palette, True)
    n_all = len(cfg.tiles)
    b = gpu_batch(cfg)
    full, _ = time_render(b, sp, pal, 10)
    info = b.tile_info()
    ents = info[:, 3]
    del b
    torch.cuda.empty_cache()
    print(json.dumps({"class": "all", "tiles": n_all, "render_ms": round(full, 4)}), flush=True)
    pred = 0.0
    tiles0, pairs0 = cfg.tiles, cfg.pairs
    for ne in sorted(set(int(e) for e in ents)):
        idx = [i for i in range(n_all) if int(ents[i]) == ne]
        rep = [idx[k % len(idx)] for k in range(n_all)]
        cfg.tiles = [tiles0[i] for i in rep]
        cfg.pairs = [pairs0[i] for i in rep]
        b = gpu_batch(cfg)
        ms, _ = time_render(b, sp, pal, 10)
        del b
        torch.cuda.empty_cache()
        pred += ms * len(idx) / n_all
        print(json.dumps({"class": "entries=%d" % ne, "tiles": len(idx), "render_ms_4096": round(ms, 4),
                          "share_ms": round(ms * len(idx) / n_all, 4)}), flush=True)
    cfg.tiles, cfg.pairs = tiles0, pairs0
    print(json.dumps({"class": "predicted_all", "render_ms": round(pred, 4)}), flush=True)


if __name__ == "__main__":
    main()
