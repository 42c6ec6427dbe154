#!/usr/bin/env python3
"""Soak test of the per-node warp service: the C2 request mix through
gskyhipd from 64 client processes for several consecutive segments, with
the daemon's resident memory and the request / error counts after each --
a long-running daemon must neither leak (arenas, registered host memory,
batch state) nor drop requests.  One JSON line per segment, then a summary.

usage: python tools/soak_service.py [--segments 6] [--seconds 20] [--workers 64]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from gsky_amd import WarpService, synth  # noqa: E402
from gsky_amd.loadgen import service_load  # noqa: E402
from gsky_amd.tiles import bbox_to_geot  # noqa: E402


def rss_kib(pid: int) -> int:
    with open("/proc/%d/status" % pid) as f:
        for line in f:
            if line.startswith("VmRSS:"):
                return int(line.split()[1])
    return -1


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--segments", type=int, default=6)
    ap.add_argument("--seconds", type=float, default=20.0)
    ap.add_argument("--workers", type=int, default=64)
    ap.add_argument("--jobs", type=int, default=1024)
    args = ap.parse_args()
    cfg = synth.config_c2()
    sock = "/tmp/gskyhip-soak-%d.sock" % os.getpid()
    svc = WarpService(sock, max_batch=64, window_us=0)
    try:
        for k, g in enumerate(cfg.granules):
            svc.register_granule("/g/data/c2/g%d.tif" % k, 1, g.data, g.geot, "EPSG:3577", g.nodata, block=(256, 256))
        pairs = [(k, bb, w, h) for (bb, w, h), ks in zip(cfg.tiles, cfg.pairs) for k in ks]
        sel = pairs[:: max(1, len(pairs) // args.jobs)][: args.jobs]
        jobs = [("/g/data/c2/g%d.tif" % k, 1, list(bbox_to_geot(w, h, bb)), w, h, "EPSG:3857") for k, bb, w, h in sel]
        rss = []
        total_req = total_err = 0
        for s in range(args.segments):
            r = service_load(sock, jobs, args.workers, seconds=args.seconds, warmup=4 if s == 0 else 0)
            st = svc.stats()
            rss.append(rss_kib(svc.proc.pid))
            total_req += r["requests"]
            total_err += r["errors"]
            print(json.dumps({"segment": s, "requests_per_s": r["requests_per_s"], "p99_ms": r["p99_ms"],
                              "errors": r["errors"], "daemon_requests": st["requests"],
                              "daemon_rss_kib": rss[-1]}), flush=True)
        growth = rss[-1] - rss[1] if len(rss) > 1 else 0
        print(json.dumps({"soak": "service", "workers": args.workers, "segments": args.segments,
                          "seconds_per_segment": args.seconds, "requests": total_req, "errors": total_err,
                          "daemon_rss_kib": rss, "rss_growth_after_first_segment_kib": growth}), flush=True)
        ok = total_err == 0 and growth < 64 * 1024
    finally:
        svc.shutdown()
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
