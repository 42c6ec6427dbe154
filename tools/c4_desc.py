#!/usr/bin/env python3
"""Breakdown of C4's descriptor step (bench.py run_c4 `descriptors_ms`) for
1000 star polygons on a 2048^2 EPSG:4326 grid: Python string marshalling,
the host describe alone (parse, envelope, window: gskyhip_drill_descriptors_device
with no mask buffer), and the whole drill_dataset (+ GPU rasterization and
the MaskBatch upload).  Medians of `--reps`.  One JSON line; the host thread
count follows GSKYHIP_DRILL_THREADS."""
import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from gsky_amd import drill, synth  # noqa: E402


def med(f, reps):
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        f()
        ts.append((time.perf_counter() - t0) * 1e3)
    return round(float(np.median(ts)), 3)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--label", default="")
    args = ap.parse_args()
    size = 2048
    _, _, geoms = synth.c4_polygons(size, 1000)
    gt = synth.C4_GT
    dev = torch.device("cuda")

    def marshal():
        return (C.c_char_p * len(geoms))(*[g.encode() for g in geoms])

    def whole():
        drill.drill_dataset(geoms, "EPSG:4326", gt, size, size, dev)
        torch.cuda.synchronize()
    whole()
    from gsky_amd._lib import lib
    arr = marshal()
    gta = (C.c_double * 6)(*gt)
    n = len(geoms)
    win = np.zeros((n, 4), np.int32)
    off = np.zeros(n, np.int64)
    st = np.zeros(n, np.int32)
    total = C.c_int64()

    def c_call():   # the host describe alone, strings already marshalled
        lib().gskyhip_drill_descriptors_device(arr, n, b"EPSG:4326", gta, size, size,
                                               win.ctypes.data_as(C.c_void_p), off.ctypes.data_as(C.c_void_p),
                                               C.byref(total), None, st.ctypes.data_as(C.c_void_p), None)
    out = {"label": args.label, "threads_env": os.environ.get("GSKYHIP_DRILL_THREADS", "16"),
           "c_call_ms": med(c_call, args.reps),
           "polygons": len(geoms), "geojson_bytes": sum(len(g) for g in geoms),
           "marshal_ms": med(marshal, args.reps),
           "windows_ms": med(lambda: drill.drill_windows(geoms, "EPSG:4326", gt, size, size), args.reps),
           "drill_dataset_ms": med(whole, args.reps)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
