"""Load generator for the per-node warp service: the path a GSKY deployment
actually calls.  N worker processes stand in for gsky-rpc's N single-threaded
gsky-gdal-process workers (grpc-server/main.go:58, worker/gdalprocess/
process.go:108-160); each sends its share of warp requests, one at a time,
through the unchanged `warp_operation_fast` C-ABI with GSKYHIP_SERVICE set, so
every request travels over the Unix socket to gskyhipd, which batches what
arrives from all workers (service.cpp).  The workers import only ctypes and
the library (no torch, no HIP context).

    res = service_load(sock, jobs, n_workers=16)
    res -> {"requests", "wall_s", "requests_per_s", "p50_ms", "p99_ms", ...}

A job is (path, band, dst_geot[6], width, height, dst_srs)."""
from __future__ import annotations

import ctypes as C
import os
import time
from typing import List, Sequence, Tuple

Job = Tuple[str, int, Sequence[float], int, int, str]


def _client(sock: str, jobs: List[Job], ready, go, q) -> None:
    os.environ["GSKYHIP_SERVICE"] = sock
    from gsky_amd._lib import lib
    L = lib()
    libc = C.CDLL(None)
    buf, size, nd, dt, br = C.c_void_p(), C.c_int(), C.c_double(), C.c_int(), C.c_int()
    bbox = (C.c_int * 4)()
    lat, errs, nbytes = [], 0, 0
    ready.put(os.getpid())
    go.wait()                       # all workers start together, once every one has imported
    for path, band, gt, w, h, srs in jobs:
        g = (C.c_double * 6)(*gt)
        t0 = time.perf_counter()
        rc = L.warp_operation_fast(path.encode(), None, None, None, srs.encode(), g, w, h, band, 0, C.byref(buf),
                                   C.byref(size), bbox, C.byref(nd), C.byref(dt), C.byref(br))
        lat.append(time.perf_counter() - t0)
        if rc == 0:
            nbytes += size.value
            libc.free(buf)
        else:
            errs += 1
    q.put((lat, errs, nbytes))


def service_load(sock: str, jobs: Sequence[Job], n_workers: int, timeout: float = 600.0) -> dict:
    """Runs `jobs` through the service with `n_workers` client processes
    (jobs dealt round-robin); returns throughput and per-request latency."""
    import multiprocessing as mp

    import numpy as np
    ctx = mp.get_context("spawn")
    q, ready, go = ctx.Queue(), ctx.Queue(), ctx.Event()
    procs = [ctx.Process(target=_client, args=(sock, list(jobs[r::n_workers]), ready, go, q))
             for r in range(n_workers)]
    for p in procs:
        p.start()
    for _ in procs:                 # every client has imported the library
        ready.get(timeout=timeout)
    t0 = time.perf_counter()
    go.set()
    res = [q.get(timeout=timeout) for _ in procs]
    wall = time.perf_counter() - t0
    for p in procs:
        p.join(60)
    lat = np.concatenate([np.asarray(r[0], np.float64) for r in res]) * 1e3
    return {"workers": n_workers, "requests": int(lat.size), "errors": int(sum(r[1] for r in res)),
            "wall_s": round(wall, 3), "requests_per_s": round(lat.size / wall, 1),
            "p50_ms": round(float(np.percentile(lat, 50)), 3), "p99_ms": round(float(np.percentile(lat, 99)), 3),
            "window_bytes": int(sum(r[2] for r in res))}
