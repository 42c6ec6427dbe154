#!/usr/bin/env python3
"""C3 (WCS 16384^2 float32 bilinear coverage, N=1) render time of the
current library (GSKYHIP_LIB=ab: the A/B build),
HIP events on the launch stream over the whole coverage launch (plan +
bilinear band kernel), with --oracle the nodata-mask identity and the largest
relative difference of the valid pixels against oracle/.  One JSON line."""
import argparse
import hashlib
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from gsky_amd import GranuleSet, ScaleParams, TileBatch, coverage, synth  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--oracle", action="store_true")
    ap.add_argument("--label", default="")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    cfg = synth.config_c3()
    chunks = coverage.chunk_requests(cfg.bbox, cfg.out_w, cfg.out_h)
    pairs = [cfg.index_chunk(c.bbox) for c in chunks]
    gs = GranuleSet(dev)
    for g in cfg.granules:
        gs.add(torch.from_numpy(np.ascontiguousarray(g.data)), g.geot, g.srs, g.nodata, [], g.timestamp,
               g.polygon, g.namespace)
    tb = TileBatch(gs, cfg.dst_srs, [(c.bbox, c.width, c.height) for c in chunks], pairs, cfg.namespaces)
    offs = torch.tensor(coverage.band_offsets(chunks, 0, cfg.out_w), dtype=torch.int64, device=dev)
    band = torch.empty((cfg.out_h, cfg.out_w), dtype=torch.float32, device=dev)
    sp = ScaleParams(*cfg.scale)

    def run(phase=0):
        return tb.render_coverage(sp, band, offs, resample=cfg.resample, phase=phase)
    run()
    torch.cuda.synchronize()
    s = torch.cuda.current_stream()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    res = {}
    for name, ph in (("total", 0), ("render", 2)):
        ts = []
        for _ in range(args.reps):
            ev[0].record(s)
            run(ph)
            ev[1].record(s)
            torch.cuda.synchronize()
            ts.append(ev[0].elapsed_time(ev[1]))
        res[name + "_ms_median"] = round(float(np.median(ts)), 4)
        res[name + "_ms_min"] = round(float(np.min(ts)), 4)
    rec = {"label": args.label, "config": "c3", "lib": os.environ.get("GSKYHIP_LIB", "default"),
           "variant": os.environ.get("GSKYHIP_BIL_REUSE", ""), **res}
    run()
    torch.cuda.synchronize()
    rec["canvas_sha16"] = hashlib.sha256(band.cpu().numpy().tobytes()).hexdigest()[:16]   # bit identity across variants
    if args.oracle:
        from oracle import oracle as O
        from tests.helpers import oracle_render
        run()
        torch.cuda.synchronize()
        _, cv, _ = oracle_render(O, cfg, n_threads=16, canvas=True)
        mh = max(c.height for c in chunks)
        mw = max(c.width for c in chunks)
        canv = [torch.from_numpy(cv[i, 0].view(np.float32).reshape(mh, mw)[:c.height, :c.width])
                for i, c in enumerate(chunks)]
        exp = coverage.place_chunks(canv, chunks, 0, cfg.out_h, cfg.out_w, device=dev)
        nod_e, nod_g = exp == -9999.0, band == -9999.0
        v = ~nod_e
        e64, g64 = exp[v].double(), band[v].double()
        rec["nodata_mask_differs"] = int((nod_e != nod_g).sum().item())
        rec["max_rel_diff"] = float(((g64 - e64).abs() / e64.abs().clamp_min(1e-30)).max().item())
        rec["bit_identical_frac"] = float((g64 == e64).double().mean().item())
    print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
