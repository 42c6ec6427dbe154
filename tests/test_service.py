"""Per-node GPU warp service (gskyhipd; include/gskyhip.h, gsky_amd/service.py).

N worker processes -- the reference's gsky-gdal-process pool (pool.go:19-74,
process.go:108-160, grpc-server/main.go:58) -- call the unchanged
warp_operation_fast C-ABI with GSKYHIP_SERVICE set and never open the GPU; one
daemon per GPU batches their requests.

CPU tests (no GPU): the socket protocol, the batching queue and the
reference's early returns across processes, a client dying mid-message, an
unreachable service.  GPU test: 8 workers x their (tile, granule) warps of a
C2 batch against the oracle (bit-exact windows, bbox, nodata, bytesRead),
batches larger than one request, and a worker SIGKILLed mid-stream.
"""
import multiprocessing as mp
import os
import signal
import socket
import tempfile
import time

import pytest

from gsky_amd import synth


def _sock_path():
    return os.path.join(tempfile.mkdtemp(prefix="gskyhip-"), "svc.sock")


def _unknown_paths(sock, n, q):
    os.environ["GSKYHIP_SERVICE"] = sock
    from gsky_amd import worker as W
    out = []
    for i in range(n):
        r = W.warp_raster(W.GeoRPCGranule(path="/nope/%d.tif" % i, bands=[1], width=8, height=8,
                                          dstSRS="EPSG:3857", dstGeot=[0.0, 1.0, 0.0, 0.0, 0.0, -1.0]))
        out.append(r.error)
    q.put(out)


def test_service_protocol_and_batching_queue():
    from gsky_amd import WarpService
    sock = _sock_path()
    svc = WarpService(sock, max_batch=16, window_us=2000)
    try:
        ctx = mp.get_context("spawn")
        q = ctx.Queue()
        procs = [ctx.Process(target=_unknown_paths, args=(sock, 8, q)) for _ in range(4)]
        for p in procs:
            p.start()
        errs = [e for _ in procs for e in q.get(timeout=120)]
        for p in procs:
            p.join(60)
            assert p.exitcode == 0
        # GDALOpenEx fails for an unregistered path: warp.go:103-105 -> "fail: 1"
        assert errs == ["warp_operation() fail: 1"] * 32
        st = svc.stats()
        assert st["requests"] == 32 and 1 <= st["batches"] <= 32 and st["max_batch"] >= 1
        # a client that dies in the middle of a message does not take the daemon down
        c = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
        c.connect(sock)
        c.send(b"GSKY\x01\x00")
        c.close()
        q2 = ctx.Queue()
        p = ctx.Process(target=_unknown_paths, args=(sock, 1, q2))
        p.start()
        assert q2.get(timeout=60) == ["warp_operation() fail: 1"]
        p.join(60)
        assert svc.stats()["requests"] == 33
    finally:
        assert svc.shutdown() == 0
    assert not os.path.exists(sock)


def test_loadgen_counts_and_timing():
    """gsky_amd.loadgen (bench.py's service leg): every job answered once,
    failures counted, the clock started only after every client imported
    the library; the daemon's stats carry the batch / residence timers."""
    from gsky_amd import WarpService
    from gsky_amd.loadgen import service_load
    sock = _sock_path()
    svc = WarpService(sock, max_batch=16, window_us=500)
    try:
        jobs = [("/nope/%d.tif" % i, 1, [0.0, 1.0, 0.0, 0.0, 0.0, -1.0], 8, 8, "EPSG:3857") for i in range(40)]
        s0 = svc.stats()
        r = service_load(sock, jobs, 4)
        s1 = svc.stats()
        assert r["requests"] == 40 and r["errors"] == 40 and r["workers"] == 4
        assert r["wall_s"] > 0 and r["requests_per_s"] > 0 and r["p99_ms"] >= r["p50_ms"] > 0
        assert s1["requests"] - s0["requests"] == 40
        assert s1["batch_s"] >= s0["batch_s"] and s1["resident_s"] > s0["resident_s"]
        # steady state: 3 untimed requests per worker, then a timed window
        r = service_load(sock, jobs, 4, seconds=0.5, warmup=3)
        s2 = svc.stats()
        assert r["requests"] > 0 and r["errors"] == r["requests"] and r["warmup_per_worker"] == 3
        assert s2["requests"] - s1["requests"] == r["requests"] + 4 * 3
        assert 0.5 <= r["wall_s"] < 5.0
    finally:
        assert svc.shutdown() == 0


def _spin_unknown(sock):
    os.environ["GSKYHIP_SERVICE"] = sock
    from gsky_amd import worker as W
    while True:
        W.warp_raster(W.GeoRPCGranule(path="/nope.tif", bands=[1], width=8, height=8, dstSRS="EPSG:3857",
                                      dstGeot=[0.0, 1.0, 0.0, 0.0, 0.0, -1.0]))


def test_service_bad_headers_do_not_kill_the_daemon():
    """A header announcing a payload far above what its op may carry (a stats
    request of 1 TiB, a warp request of 64 GiB) or an unknown op closes that
    connection only: no allocation, no std::terminate, the daemon keeps
    answering."""
    import struct

    from gsky_amd import WarpService
    sock = _sock_path()
    svc = WarpService(sock, max_batch=4, window_us=100)
    try:
        for op, n in ((4, 1 << 40), (1, 1 << 36), (2, 1 << 50), (99, 8)):
            c = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
            c.connect(sock)
            c.sendall(struct.pack("<IIQ", 0x594B5347, op, n) + (b"\0" * n if n <= 64 else b""))
            c.settimeout(10)
            assert c.recv(16) == b""   # the daemon hung up
            c.close()
        assert svc.proc.poll() is None
        assert svc.stats()["requests"] == 0
    finally:
        assert svc.shutdown() == 0


def test_service_shutdown_under_load():
    """Shutdown while workers keep sending warps: the daemon stops within a
    few seconds (no request is queued behind a stopped batcher), and workers
    then see the service as unreachable."""
    from gsky_amd import WarpService
    sock = _sock_path()
    svc = WarpService(sock, max_batch=8, window_us=500)
    ctx = mp.get_context("spawn")
    procs = [ctx.Process(target=_spin_unknown, args=(sock,)) for _ in range(4)]
    try:
        for p in procs:
            p.start()
        t0 = time.time()
        while svc.stats()["requests"] < 20 and time.time() - t0 < 120:
            time.sleep(0.2)
        assert svc.stats()["requests"] >= 20
        t0 = time.time()
        assert svc.shutdown(timeout=30.0) == 0
        assert time.time() - t0 < 15.0
    finally:
        for p in procs:
            p.kill()
            p.join(30)


def test_service_unreachable():
    """No daemon behind GSKYHIP_SERVICE: the drop-in reports the failure (the
    OWS retries an errored request, process.go:147-150)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_unknown_paths, args=(_sock_path(), 1, q))
    p.start()
    assert q.get(timeout=60) == ["warp_operation() fail: -9"]
    p.join(60)


# ---------------------------------------------------------------- GPU
def _warp_jobs(sock, wid, jobs, q, go=None):
    """A worker process: warp_raster over the service for its (tile, granule)
    jobs (all workers start together when `go` is given)."""
    os.environ["GSKYHIP_SERVICE"] = sock
    from gsky_amd import worker as W
    if go is not None:
        go.wait(120)
    res = []
    for (k, gt, w, h) in jobs:
        r = W.warp_raster(W.GeoRPCGranule(path="/g/data/c2/g%d.tif" % k, bands=[1], width=w, height=h,
                                          dstSRS="EPSG:3857", dstGeot=list(gt)))
        res.append((r.error, r.raster.data if r.raster else b"", r.raster.bbox if r.raster else [],
                    r.raster.noData if r.raster else 0.0, r.raster.rasterType if r.raster else "", r.bytesRead))
    q.put((wid, res))


def _spin(sock, job):
    os.environ["GSKYHIP_SERVICE"] = sock
    from gsky_amd import worker as W
    k, gt, w, h = job
    while True:
        W.warp_raster(W.GeoRPCGranule(path="/g/data/c2/g%d.tif" % k, bands=[1], width=w, height=h,
                                      dstSRS="EPSG:3857", dstGeot=list(gt)))


@pytest.mark.gpu
@pytest.mark.parametrize("direct", [1, 0])
def test_service_workers_share_one_gpu(oracle, direct):
    """8 worker processes (no HIP context of their own) warp every (tile,
    granule) pair of a C2 batch through one gskyhipd: each window bit-exact
    against the oracle, requests batched across workers, a SIGKILLed worker
    leaving the daemon serving.  direct=1: the warp kernel writes every
    window into the worker's registered reply arena; direct=0
    (GSKYHIP_SVC_DIRECT=0): staged in HBM, read back and copied."""
    from gsky_amd import WarpService
    from gsky_amd.tiles import bbox_to_geot
    cfg = synth.config_c2(scale=0.1, tiles_per_side=4, tile_px=256)
    sock = _sock_path()
    svc = WarpService(sock, max_batch=64, window_us=2000, env={"GSKYHIP_SVC_DIRECT": str(direct)})
    try:
        for k, g in enumerate(cfg.granules):
            svc.register_granule("/g/data/c2/g%d.tif" % k, 1, g.data, g.geot, "EPSG:3577", g.nodata,
                                 block=(128, 64))
        assert svc.stats()["granules"] == len(cfg.granules)
        jobs = [(k, bbox_to_geot(w, h, bb), w, h) for (bb, w, h), ks in zip(cfg.tiles, cfg.pairs) for k in ks]
        ctx = mp.get_context("spawn")
        q, go = ctx.Queue(), ctx.Event()
        n_workers = 8
        procs = [ctx.Process(target=_warp_jobs, args=(sock, r, jobs[r::n_workers], q, go)) for r in range(n_workers)]
        for p in procs:
            p.start()
        time.sleep(5.0)   # every worker imported and waiting: their requests meet in the daemon's queue
        go.set()
        got = dict(q.get(timeout=300) for _ in procs)
        for p in procs:
            p.join(60)
            assert p.exitcode == 0
        aea, wm = oracle.crs("EPSG:3577"), oracle.crs("EPSG:3857")
        n_checked = 0
        for r in range(n_workers):
            for (k, gt, w, h), (err, data, bbox, nd, rtype, br) in zip(jobs[r::n_workers], got[r]):
                g = cfg.granules[k]
                og = oracle.make_granule(g.data, g.geot, g.nodata, block=(128, 64))
                arr, ebbox, end, _ = oracle.warp(og, aea, wm, list(gt), w, h)
                assert err == "OK" and bbox == list(ebbox), (k, gt, err)
                assert data == arr.tobytes() and nd == end and rtype == "Int16", (k, gt)
                assert br == oracle.warp.bytes_read, (k, gt)               # warp.go:347
                n_checked += 1
        assert n_checked == len(jobs)
        st = svc.stats()
        assert st["requests"] == len(jobs) and st["max_batch"] > 1 and st["batches"] < len(jobs), st
        n_ok = st["in_place"] + st["copied"]
        assert n_ok == len(jobs), st
        assert st["in_place"] == (len(jobs) if direct else 0), st
        # a worker SIGKILLed while its requests are in flight (gdal-process is killed after 120 s,
        # gdal-process/main.go:57-68): the daemon keeps serving
        p = ctx.Process(target=_spin, args=(sock, jobs[0]))
        p.start()
        time.sleep(3.0)
        os.kill(p.pid, signal.SIGKILL)
        p.join(30)
        q2 = ctx.Queue()
        p2 = ctx.Process(target=_warp_jobs, args=(sock, 0, jobs[:3], q2))
        p2.start()
        _, again = q2.get(timeout=120)
        p2.join(60)
        assert [e for e, *_ in again] == ["OK"] * 3
        assert svc.stats()["requests"] > st["requests"] + 3
    finally:
        assert svc.shutdown() == 0


def _warp_loop(sock, wid, jobs, rounds, q, go):
    """A worker process: its jobs `rounds` times over (all workers start on `go`)."""
    os.environ["GSKYHIP_SERVICE"] = sock
    from gsky_amd import worker as W
    go.wait(120)
    res = []
    for _ in range(rounds):
        for (k, gt, w, h) in jobs:
            r = W.warp_raster(W.GeoRPCGranule(path="/g/data/c2/g%d.tif" % k, bands=[1], width=w, height=h,
                                              dstSRS="EPSG:3857", dstGeot=list(gt)))
            res.append((r.error, r.raster.data if r.raster else b""))
    q.put((wid, res))


@pytest.mark.gpu
def test_service_register_while_batches_in_flight(oracle):
    """with a batching window (window_us > 0) a registration that
    arrives while batches are in flight must not run beside a newly launched
    batch -- a granule refresh frees the old upload.  6 workers warp in a
    loop while the granules are registered again and again; every window
    stays bit-exact against the oracle."""
    from gsky_amd import WarpService
    from gsky_amd.tiles import bbox_to_geot
    cfg = synth.config_c2(scale=0.1, tiles_per_side=4, tile_px=256)
    sock = _sock_path()
    svc = WarpService(sock, max_batch=16, window_us=300)
    try:
        def reg_all():
            for k, g in enumerate(cfg.granules):
                svc.register_granule("/g/data/c2/g%d.tif" % k, 1, g.data, g.geot, "EPSG:3577", g.nodata,
                                     block=(128, 64))
        reg_all()
        jobs = [(k, bbox_to_geot(w, h, bb), w, h) for (bb, w, h), ks in zip(cfg.tiles, cfg.pairs) for k in ks]
        ctx = mp.get_context("spawn")
        q, go = ctx.Queue(), ctx.Event()
        n_workers, rounds = 6, 6
        procs = [ctx.Process(target=_warp_loop, args=(sock, r, jobs[r::n_workers], rounds, q, go))
                 for r in range(n_workers)]
        for p in procs:
            p.start()
        time.sleep(5.0)
        go.set()
        n_reg = 0
        t_end = time.time() + 60
        while n_reg < 12 and time.time() < t_end:   # refreshes while the workers' batches run
            reg_all()
            n_reg += 1
        got = dict(q.get(timeout=300) for _ in procs)
        for p in procs:
            p.join(60)
            assert p.exitcode == 0
        aea, wm = oracle.crs("EPSG:3577"), oracle.crs("EPSG:3857")
        want = {}
        for (k, gt, w, h) in jobs:
            g = cfg.granules[k]
            arr, _, _, _ = oracle.warp(oracle.make_granule(g.data, g.geot, g.nodata, block=(128, 64)), aea, wm,
                                       list(gt), w, h)
            want[(k, tuple(gt))] = arr.tobytes()
        for r in range(n_workers):
            mine = jobs[r::n_workers] * rounds
            assert len(got[r]) == len(mine)
            for (k, gt, w, h), (err, data) in zip(mine, got[r]):
                assert err == "OK" and data == want[(k, tuple(gt))], (k, gt, err)
        assert n_reg >= 1 and svc.stats()["granules"] == len(cfg.granules)
    finally:
        assert svc.shutdown() == 0
