#!/usr/bin/env python3
"""A/B timing of the C2 render phase (phase-2 kernels only, HIP events on the
launch stream) for the kernel variants: the NN band kernel (render_nn.h) in
its lane shapes, the first band kernel (render_lds.h: LDS-staged source
windows, HBM gathers, fixed point, LUT) and the generic kernel.
One JSON line per variant.  Used to pick defaults; bench.py is the contract."""
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


def time_render(b, sp, pal, reps):
    s = torch.cuda.current_stream()
    b.render(sp, pal, phase=1)
    for _ in range(3):
        b.render(sp, pal, phase=2)
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ts = []
    for _ in range(reps):
        ev[0].record(s)
        b.render(sp, pal, phase=2)
        ev[1].record(s)
        torch.cuda.synchronize()
        ts.append(ev[0].elapsed_time(ev[1]))
    return float(np.median(ts)), float(np.min(ts))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--config", default="c2")
    ap.add_argument("--variant", default="", help="run only this variant (for rocprofv3 passes)")
    ap.add_argument("--probes", action="store_true", help="timing-only probes: no gathers / no stores")
    ap.add_argument("--oracle", action="store_true", help="also count RGBA pixels differing from the oracle")
    ap.add_argument("--stride", action="store_true", help="lane-pixel layout variants (GSKYHIP_NN_STRIDE / NN_LUT)")
    ap.add_argument("--all-layouts", action="store_true", help="with --stride: every layout variant")
    args = ap.parse_args()
    cfg = synth.config_c2() if args.config == "c2" else synth.config_c5()
    b = gpu_batch(cfg)
    sp = gsky_amd.ScaleParams(*cfg.scale)
    pal = gsky_amd.Palette(cfg.palette, True) if cfg.palette else None
    ref = None
    exp = None
    if args.oracle:
        from oracle import oracle as O
        from tests.helpers import oracle_render
        exp = torch.from_numpy(oracle_render(O, cfg, n_threads=16)).to("cuda")
    # (name, typed, LDS_STAGE, LDS_FLAGS, NN_KERNEL, NN_SHAPE[, NN_XCD, NN_PROBE, NN_GEN, NN_WPE, NN_EXPRESS, NN_WIDE, NN_RPW])
    variants = [("nn_4x2_rpw16", True, "0", "0", "1", "3", "0", "0", "2", "0", "1", "0", "16"),
                ("nn_4x2_rpw8", True, "0", "0", "1", "3", "0", "0", "2", "0", "1", "0", "8"),
                ("nn3w_4x1", True, "0", "0", "1", "4", "0", "0", "3", "0", "1", "1"),
                ("nn3w_4x2", True, "0", "0", "1", "3", "0", "0", "3", "0", "1", "1"),
                ("nn3w_4x1_nox", True, "0", "0", "1", "4", "0", "0", "3", "0", "0", "1"),
                ("nn3_4x2", True, "0", "0", "1", "3", "0", "0", "3"), ("nn3_4x4", True, "0", "0", "1", "0", "0", "0", "3"),
                ("nn3_8x1", True, "0", "0", "1", "1", "0", "0", "3"), ("nn3_4x1", True, "0", "0", "1", "4", "0", "0", "3"),
                ("nn3_4x2_w6", True, "0", "0", "1", "3", "0", "0", "3", "6"),
                ("nn3_4x2_nox", True, "0", "0", "1", "3", "0", "0", "3", "0", "0"),
                ("nn3_4x1_nox", True, "0", "0", "1", "4", "0", "0", "3", "0", "0"),
                ("nn_4x2", True, "0", "0", "1", "3"), ("nn_4x4", True, "0", "0", "1", "0"), ("nn_8x1", True, "0", "0", "1", "1"),
                ("nn_8x2", True, "0", "0", "1", "2"),
                ("generic", False, "1", "0", "0", "0")]
    if args.probes:   # timing-only probes of the default NN kernel (images are wrong by design)
        variants = [("nn_4x2", True, "0", "0", "1", "3")] + [
            ("probe_%s" % p, True, "0", "0", "1", "3", "0", p) for p in ("1", "2", "3", "4")]
        variants = [v + ({"GSKYHIP_NN_STRIDE": "1"},) for v in variants]
    if args.stride:   # trailing dict: extra environment of the variant
        variants = [("nn_4x2", True, "0", "0", "1", "3"),
                    ("nn_4x2_s", True, "0", "0", "1", "3", {"GSKYHIP_NN_STRIDE": "1"}),
                    ("nn_4x1_s_w8", True, "0", "0", "1", "4", {"GSKYHIP_NN_STRIDE": "1"}),
                    ("nn_4x1_s_w8_mask4x1", True, "0", "0", "1", "5", {"GSKYHIP_NN_STRIDE": "1"}),
                    ("nn_4x1_s_w8_again", True, "0", "0", "1", "4", {"GSKYHIP_NN_STRIDE": "1"}),
                    ("nn_4x1_s_w8_mask4x1_again", True, "0", "0", "1", "5", {"GSKYHIP_NN_STRIDE": "1"})]
        if args.all_layouts:   # the round's other layout variants (profiles/r02z7_ab_*.jsonl)
            variants += [("nn_8x1_s", True, "0", "0", "1", "1", {"GSKYHIP_NN_STRIDE": "1"}),
                         ("nn_8x2_s", True, "0", "0", "1", "2", {"GSKYHIP_NN_STRIDE": "1"}),
                         ("nn_4x2_s_lut", True, "0", "0", "1", "3",
                          {"GSKYHIP_NN_STRIDE": "1", "GSKYHIP_NN_LUT": "1"}),
                         ("nn_4x4_s", True, "0", "0", "1", "0", {"GSKYHIP_NN_STRIDE": "1"}),
                         ("nn_4x2_s_plain", True, "0", "0", "1", "3", {"GSKYHIP_NN_STRIDE": "2"}),
                         ("nn_4x2_s_ldsout", True, "0", "0", "1", "3", {"GSKYHIP_NN_STRIDE": "4"}),
                         ("nn_4x2_s_w8", True, "0", "0", "1", "3", {"GSKYHIP_NN_STRIDE": "5"}),
                         ("nn_4x2_s_rpw8", True, "0", "0", "1", "3", "0", "0", "2", "0", "1", "0", "8",
                          {"GSKYHIP_NN_STRIDE": "1"})]
    for name, typed, stage, flags, nnk, shape, *extra in variants:
        if args.variant and name != args.variant:
            continue
        env = extra.pop() if extra and isinstance(extra[-1], dict) else {}
        for k in ("GSKYHIP_NN_STRIDE", "GSKYHIP_NN_LUT"):
            os.environ[k] = env.get(k, "0")
        xcd = extra[:1]
        os.environ["GSKYHIP_LDS_STAGE"] = stage
        os.environ["GSKYHIP_LDS_FLAGS"] = flags
        os.environ["GSKYHIP_NN_KERNEL"] = nnk
        os.environ["GSKYHIP_NN_SHAPE"] = shape
        os.environ["GSKYHIP_NN_XCD"] = xcd[0] if xcd else "0"
        os.environ["GSKYHIP_NN_PROBE"] = extra[1] if len(extra) > 1 else "0"
        os.environ["GSKYHIP_NN_GEN"] = extra[2] if len(extra) > 2 else "2"
        os.environ["GSKYHIP_NN_WPE"] = extra[3] if len(extra) > 3 else "0"
        os.environ["GSKYHIP_NN_EXPRESS"] = extra[4] if len(extra) > 4 else "1"
        os.environ["GSKYHIP_NN_WIDE"] = extra[5] if len(extra) > 5 else "0"
        os.environ["GSKYHIP_NN_RPW"] = extra[6] if len(extra) > 6 else "4"
        b.typed = typed
        med, mn = time_render(b, sp, pal, args.reps)
        out = b.render(sp, pal).clone()
        torch.cuda.synchronize()
        same = True if ref is None else bool(torch.equal(out, ref))
        ref = out if ref is None else ref
        rec = {"variant": name, "config": args.config, "render_ms_median": round(med, 4),
               "render_ms_min": round(mn, 4), "identical_to_first": same}
        if exp is not None:
            rec["differ_from_oracle"] = int((out != exp).any(dim=-1).sum().item())
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
