"""Load generator for the per-node warp service: the path a GSKY deployment
actually calls.  N worker processes stand in for gsky-rpc's N single-threaded
gsky-gdal-process workers (grpc-server/main.go:58, worker/gdalprocess/
process.go:108-160); each sends its share of warp requests, one at a time,
through the unchanged `warp_operation_fast` C-ABI with GSKYHIP_SERVICE set, so
every request travels over the Unix socket to gskyhipd, which batches what
arrives from all workers (service.cpp).  The workers import only ctypes and
the library (no torch, no HIP context).

    res = service_load(sock, jobs, n_workers=16, seconds=2.0, warmup=8)
    res -> {"requests", "wall_s", "requests_per_s", "p50_ms", "p99_ms", ...}

A job is (path, band, dst_geot[6], width, height, dst_srs)."""
from __future__ import annotations

import ctypes as C
import os
import time
from typing import List, Sequence, Tuple

Job = Tuple[str, int, Sequence[float], int, int, str]


def _client(sock: str, jobs: List[Job], warmup: int, ready, go, t_win, q) -> None:
    os.environ["GSKYHIP_SERVICE"] = sock
    from gsky_amd._lib import lib
    L = lib()
    libc = C.CDLL(None)
    buf, size, nd, dt, br = C.c_void_p(), C.c_int(), C.c_double(), C.c_int(), C.c_int()
    bbox = (C.c_int * 4)()
    args = [(path.encode(), (C.c_double * 6)(*gt), w, h, band, srs.encode()) for path, band, gt, w, h, srs in jobs]

    def one(a):
        rc = L.warp_operation_fast(a[0], None, None, None, a[5], a[1], a[2], a[3], a[4], 0, C.byref(buf),
                                   C.byref(size), bbox, C.byref(nd), C.byref(dt), C.byref(br))
        n = 0
        if rc == 0:
            n = size.value
            libc.free(buf)
        return rc, n

    for k in range(warmup):         # untimed: connection, arena, daemon thread, first batches
        one(args[k % len(args)])
    ready.put(os.getpid())
    go.wait()                       # all workers start together, once every one has imported and warmed up
    t_start, t_end = t_win[0], t_win[1]
    while time.perf_counter() < t_start:
        pass
    lat, errs, nbytes = [], 0, 0
    k = 0
    last = t_start
    while True:
        if t_end > 0:
            if time.perf_counter() >= t_end:
                break
        elif k >= len(args):
            break
        t0 = time.perf_counter()
        rc, n = one(args[k % len(args)])
        last = time.perf_counter()
        lat.append(last - t0)
        k += 1
        if rc == 0:
            nbytes += n
        else:
            errs += 1
    q.put((lat, errs, nbytes, last))


def service_load(sock: str, jobs: Sequence[Job], n_workers: int, seconds: float = 0.0, warmup: int = 0,
                 timeout: float = 600.0) -> dict:
    """Runs `jobs` through the service with `n_workers` client processes (jobs
    dealt round-robin).  seconds == 0: every job once.  seconds > 0: steady
    state -- each worker first sends `warmup` untimed requests, then all
    start together and each cycles through its share, one request at a time,
    for `seconds`.  Returns throughput (timed requests / the time from the
    common start to the last answer) and per-request latency over the timed
    requests only."""
    import multiprocessing as mp

    import numpy as np
    ctx = mp.get_context("spawn")
    q, ready, go = ctx.Queue(), ctx.Queue(), ctx.Event()
    t_win = ctx.Array("d", 2)
    procs = [ctx.Process(target=_client, args=(sock, list(jobs[r::n_workers]), warmup, ready, go, t_win, q))
             for r in range(n_workers)]
    for p in procs:
        p.start()
    for _ in procs:                 # every client has imported the library and warmed up
        ready.get(timeout=timeout)
    t0 = time.perf_counter() + 0.05
    t_win[0] = t0
    t_win[1] = t0 + seconds if seconds > 0 else 0.0
    go.set()
    res = [q.get(timeout=timeout) for _ in procs]
    wall = max(r[3] for r in res) - t0
    for p in procs:
        p.join(60)
    lat = np.concatenate([np.asarray(r[0], np.float64) for r in res]) * 1e3
    return {"workers": n_workers, "requests": int(lat.size), "errors": int(sum(r[1] for r in res)),
            "warmup_per_worker": warmup, "wall_s": round(wall, 3), "requests_per_s": round(lat.size / wall, 1),
            "p50_ms": round(float(np.percentile(lat, 50)), 3), "p99_ms": round(float(np.percentile(lat, 99)), 3),
            "window_bytes": int(sum(r[2] for r in res))}
