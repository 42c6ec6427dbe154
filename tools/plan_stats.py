"""Plan statistics of the benchmark configs: tiles on the typed band kernel vs
the general kernel, rows split by the approximation recursion, leaf pool
use, and the render time of the typed and generic paths (phase 2).
Usage: python tools/plan_stats.py [c2 c5 ...]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import numpy as np
    import torch

    import gsky_amd
    from gsky_amd import synth
    from tests.helpers import gpu_batch
    names = sys.argv[1:] or ["c2", "c5", "c3"]
    for name in names:
        cfg = getattr(synth, "config_" + name)()
        if name == "c3":   # the WCS chunks of the coverage as one tile batch
            from gsky_amd import coverage
            chunks = coverage.chunk_requests(cfg.bbox, cfg.out_w, cfg.out_h)
            cfg.tiles = [(c.bbox, c.width, c.height) for c in chunks]
            cfg.pairs = [cfg.index_chunk(c.bbox) for c in chunks]
        b = gpu_batch(cfg, "cuda")
        sp = gsky_amd.ScaleParams(*cfg.scale)
        pal = gsky_amd.Palette(cfg.palette, True) if cfg.palette else None
        b.render(sp, pal, resample=cfg.resample)
        torch.cuda.synchronize()
        info = b.tile_info()
        out = {"config": name, "tiles": int(len(info)), "pairs": b.n_pairs, "complex_tiles": int(info[:, 1].sum()),
               "value_types": sorted(set(int(v) for v in info[:, 2])), "entries_mean": float(info[:, 3].mean()),
               "entries_max": int(info[:, 3].max()), **b.plan_counters}
        for typed in (True, False):
            b.typed = typed
            b.render(sp, pal, resample=cfg.resample, phase=2)
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            ev[0].record()
            for _ in range(10):
                b.render(sp, pal, resample=cfg.resample, phase=2)
            ev[1].record()
            torch.cuda.synchronize()
            out["render_ms_typed" if typed else "render_ms_generic"] = round(ev[0].elapsed_time(ev[1]) / 10, 4)
        b.typed = True
        ref = b.render(sp, pal, resample=cfg.resample).clone()
        for sep in ("1", "0"):   # planning time (phase 1) with and without the separable transform
            os.environ["GSKYHIP_PLAN_SEP"] = sep
            b.render(sp, pal, resample=cfg.resample, phase=1)
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            ev[0].record()
            for _ in range(10):
                b.render(sp, pal, resample=cfg.resample, phase=1)
            ev[1].record()
            torch.cuda.synchronize()
            out["plan_ms_sep" + sep] = round(ev[0].elapsed_time(ev[1]) / 10, 4)
            out["identical_sep" + sep] = bool(torch.equal(b.render(sp, pal, resample=cfg.resample), ref))
        os.environ["GSKYHIP_PLAN_SEP"] = "1"
        print(json.dumps(out), flush=True)
        del b
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
