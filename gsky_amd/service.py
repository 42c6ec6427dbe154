"""Per-node GPU warp service (include/gskyhip.h "per-node warp service").

The reference serves `warp` from N = NumCPU single-threaded gsky-gdal-process
workers per node, spawned, fed and recycled by processor/pool.go:19-74 and
process.go:108-160 (grpc-server/main.go:58).  On MI355X one daemon per GPU
(`gskyhipd`, built next to libgskyhip.so) owns the HIP context and the
HBM-resident granules; workers keep calling the unchanged
`warp_operation_fast` C-ABI (gsky_amd.worker.warp_raster here, the cgo shim of
INTEGRATION.md in Go) with GSKYHIP_SERVICE=<socket> in their environment, so
they forward each request over a Unix socket and never open the GPU.  The
daemon batches the requests of all workers that arrive within its window into
one plan + warp launch set, keeps two batches in flight, and has the GPU
write each window straight into the worker's shared reply arena.

    svc = WarpService("/tmp/gskyhip-0.sock")        # starts gskyhipd
    svc.register_granule("NETCDF:/g/x.nc:v", 1, array, geot, "EPSG:3577", -999.0)
    env = svc.env()                                  # give to each worker process
    ...
    svc.shutdown()
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
import time
from typing import Dict, Optional, Sequence

import numpy as np

from . import _lib
from ._lib import check, lib

# GSKYHIP_DAEMON: another daemon binary (tools: gskyhipd_ab, on the A/B build)
DAEMON = os.environ.get("GSKYHIP_DAEMON") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "gskyhipd")

_NP_DTYPE = {np.dtype(np.uint8): _lib.BYTE, np.dtype(np.int8): _lib.BYTE, np.dtype(np.int16): _lib.INT16,
             np.dtype(np.uint16): _lib.UINT16, np.dtype(np.float32): _lib.FLOAT32}


class WarpService:
    """Handle on one gskyhipd daemon (start=True launches it as a child)."""

    def __init__(self, socket_path: str, max_batch: int = 64, window_us: int = 0, start: bool = True,
                 device: Optional[int] = None, timeout: float = 60.0, env: Optional[Dict[str, str]] = None):
        self.socket_path = socket_path
        self.proc = None
        if start:
            if not os.path.exists(DAEMON):
                raise FileNotFoundError("gskyhipd not built: run __graft_entry__.build() (%s)" % DAEMON)
            env_extra = dict(env or {})
            env = denv = dict(os.environ)
            env.pop("GSKYHIP_SERVICE", None)
            if device is not None:
                env["HIP_VISIBLE_DEVICES"] = str(device)
            denv.update(env_extra)
            self.proc = subprocess.Popen([DAEMON, socket_path, str(int(max_batch)), str(int(window_us))], env=denv)
            t0 = time.time()
            while True:
                if os.path.exists(socket_path):
                    try:
                        self.stats()
                        break
                    except RuntimeError:
                        pass
                if self.proc.poll() is not None:
                    raise RuntimeError("gskyhipd exited with %d" % self.proc.returncode)
                if time.time() - t0 > timeout:
                    self.proc.kill()
                    raise TimeoutError("gskyhipd did not come up on %s" % socket_path)
                time.sleep(0.05)

    def env(self) -> Dict[str, str]:
        """Environment entries that route a worker's warp_operation_fast here."""
        return {"GSKYHIP_SERVICE": self.socket_path}

    def register_granule(self, path: str, band: int, data: np.ndarray, geot: Sequence[float], srs: str = "",
                         nodata: Optional[float] = None, overviews: Sequence[np.ndarray] = (),
                         signed_byte: bool = False, block=(0, 0)) -> None:
        """Uploads a band (and its overviews) into the daemon's HBM under
        (path, band): the daemon-side GDALOpenEx of warp.go:89-101."""
        d = np.ascontiguousarray(data)
        ovr = [np.ascontiguousarray(o, dtype=d.dtype) for o in overviews]
        g = _lib.Granule()
        g.dtype = _NP_DTYPE[d.dtype]
        g.ysize, g.xsize = d.shape
        g.signed_byte = int(signed_byte or d.dtype == np.int8)
        for k in range(6):
            g.geot[k] = geot[k]
        g.nodata = nodata if nodata is not None else -1e10
        g.has_nodata = int(nodata is not None)
        g.n_ovr = len(ovr)
        for k, o in enumerate(ovr):
            g.ovr_ysize[k], g.ovr_xsize[k] = o.shape
        g.block_x, g.block_y = block
        optrs = (C.c_void_p * max(1, len(ovr)))(*[o.ctypes.data for o in ovr])
        check(lib().gskyhip_service_register_granule(self.socket_path.encode(), path.encode(), int(band),
                                                     C.byref(g), C.c_void_p(d.ctypes.data), optrs,
                                                     srs.encode() if srs else None), "service register")

    def unregister_all(self) -> None:
        check(lib().gskyhip_service_unregister_all(self.socket_path.encode()), "service unregister")

    def stats(self) -> Dict[str, int]:
        st = (C.c_int64 * 11)()
        check(lib().gskyhip_service_stats_n(self.socket_path.encode(), st, 11), "service stats")
        return {"requests": st[0], "batches": st[1], "max_batch": st[2], "granules": st[3],
                "batch_s": st[4] * 1e-9, "resident_s": st[5] * 1e-9, "launch_s": st[6] * 1e-9,
                "gpu_wait_s": st[7] * 1e-9, "readback_s": st[8] * 1e-9, "in_place": st[9], "copied": st[10]}

    def shutdown(self, timeout: float = 60.0) -> Optional[int]:
        """Stops the daemon; returns its exit code when this handle started it."""
        try:
            lib().gskyhip_service_shutdown(self.socket_path.encode())
        finally:
            if self.proc is not None:
                try:
                    return self.proc.wait(timeout)
                except subprocess.TimeoutExpired:
                    self.proc.kill()
                    return self.proc.wait()
        return None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.shutdown()
