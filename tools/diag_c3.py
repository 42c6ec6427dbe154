"""C3 diagnostic: the whole bilinear coverage through the typed band kernel
and through the generic kernels (TileBatch.typed = False), compared bit for
bit; prints per-chunk mismatch counts and the first differing pixels.
Usage: python tools/diag_c3.py [--scale S]"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    from gsky_amd import ScaleParams, coverage, synth
    from gsky_amd.tiles import GranuleSet, TileBatch
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=float, default=1.0)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    cfg = synth.config_c3(scale=args.scale)
    chunks = coverage.chunk_requests(cfg.bbox, cfg.out_w, cfg.out_h)
    pairs = [cfg.index_chunk(c.bbox) for c in chunks]
    used = sorted({g for p in pairs for g in p})
    remap = {g: i for i, g in enumerate(used)}
    gs = GranuleSet(dev)
    import numpy as np
    for g in used:
        gr = cfg.granules[g]
        gs.add(torch.from_numpy(np.ascontiguousarray(gr.data)), gr.geot, gr.srs, gr.nodata, [], gr.timestamp,
               gr.polygon, gr.namespace)
    tiles = [(c.bbox, c.width, c.height) for c in chunks]
    tb = TileBatch(gs, cfg.dst_srs, tiles, [[remap[g] for g in p] for p in pairs], cfg.namespaces)
    offs = coverage.band_offsets(chunks, 0, cfg.out_w)
    outs = {}
    for typed in (True, False):
        tb.typed = typed
        band = torch.full((cfg.out_h, cfg.out_w), float("nan"), dtype=torch.float32, device=dev)
        tb.render_coverage(ScaleParams(*cfg.scale), band, offs, resample=cfg.resample)
        torch.cuda.synchronize()
        outs[typed] = band
    for typed in (True, False):   # render-only (phase 2) time of each path
        tb.typed = typed
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        tb.render_coverage(ScaleParams(*cfg.scale), outs[typed], offs, resample=cfg.resample, phase=2)
        ev[0].record()
        for _ in range(5):
            tb.render_coverage(ScaleParams(*cfg.scale), outs[typed], offs, resample=cfg.resample, phase=2)
        ev[1].record()
        torch.cuda.synchronize()
        print(json.dumps({"typed": typed, "render_ms": round(ev[0].elapsed_time(ev[1]) / 5, 4)}))
    info = tb.tile_info()
    print(json.dumps({"tiles": int(len(info)), "complex": int(info[:, 1].sum()),
                      "vt": sorted(set(int(v) for v in info[:, 2])), "counters": tb.plan_counters,
                      "n_pairs": int(sum(len(p) for p in pairs))}))
    a, b = outs[True], outs[False]
    same = (a.view(torch.int32) == b.view(torch.int32))
    print(json.dumps({"pixels": a.numel(), "differ": int((~same).sum().item()),
                      "nan_typed": int(torch.isnan(a).sum().item()), "nan_generic": int(torch.isnan(b).sum().item())}))
    rep = []
    for i, c in enumerate(chunks):
        sa = same[c.off_y:c.off_y + c.height, c.off_x:c.off_x + c.width]
        n = int((~sa).sum().item())
        if n:
            idx = torch.nonzero(~sa)[:4].cpu().tolist()
            ex = [(r, x, float(a[c.off_y + r, c.off_x + x]), float(b[c.off_y + r, c.off_x + x])) for r, x in idx]
            rep.append({"chunk": i, "w": c.width, "h": c.height, "n_pairs": len(pairs[i]), "differ": n, "first": ex})
    print(json.dumps({"chunks_differing": len(rep)}))
    for r in rep[:40]:
        print(json.dumps(r))


if __name__ == "__main__":
    main()
