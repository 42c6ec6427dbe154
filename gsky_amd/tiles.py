"""Batched WMS GetMap path on MI355X.

Replaces, for a whole batch of output tiles at once, the per-tile chain of the
reference: gRPC warp fan-out (processor/tile_grpc.go:200-289) ->
warp_operation_fast (worker/gdalprocess/warp.go:82-382) -> RasterMerger
(processor/tile_merger.go:447-738) -> utils.Scale (utils/raster_scaler.go:334)
-> EncodePNG RGBA fill (utils/ogc_encoders.go:82-134).

Granules are HBM-resident (GranuleSet); a TileBatch uploads its descriptor
tables once and `render()` is then one asynchronous launch sequence on the
current torch stream (capturable in a HIP graph).
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass
from typing import List, Optional, Sequence, Tuple

import numpy as np
import torch

from . import _lib
from ._lib import check, lib
from .raster import TYPE_CODES, TYPE_NAMES, TORCH_OF, Mask, Palette, ScaleParams, fnv32a, gradient_rgba_palette

DTYPE_OF_TORCH = {torch.uint8: _lib.BYTE, torch.int8: _lib.BYTE, torch.int16: _lib.INT16,
                  torch.uint16: _lib.UINT16, torch.float32: _lib.FLOAT32, torch.int32: _lib.INT32,
                  torch.float64: _lib.FLOAT64}


def bbox_to_geot(width: int, height: int, bbox: Sequence[float]) -> List[float]:
    """BBox2Geot (processor/tile_grpc.go:380-382)."""
    return [bbox[0], (bbox[2] - bbox[0]) / float(width), 0.0, bbox[3], 0.0, (bbox[1] - bbox[3]) / float(height)]


def parse_crs(srs: str) -> _lib.Crs:
    c = _lib.Crs()
    check(lib().gskyhip_crs_from_srs(srs.encode(), C.byref(c)), "SRS %r" % srs)
    return c


def crs_transform(src_srs: str, dst_srs: str, x, y):
    """Points from one SRS to another on the host, through the functions the
    kernels run (gskyhip_crs_transform; OGRCoordinateTransformation's place in
    the warp, warp.go:130).  Returns (x, y, ok) float64 / bool arrays."""
    a, b = parse_crs(src_srs), parse_crs(dst_srs)
    xs = np.array(x, dtype=np.float64).ravel().copy()
    ys = np.array(y, dtype=np.float64).ravel().copy()
    if xs.size != ys.size:
        raise ValueError("crs_transform: x and y differ in length")
    ok = np.zeros(xs.size, np.int32)
    check(lib().gskyhip_crs_transform(C.byref(a), C.byref(b), xs.size, xs.ctypes.data, ys.ctypes.data,
                                      ok.ctypes.data), "crs_transform")
    return xs, ys, ok.astype(bool)


def _to_device_bytes(obj, device) -> torch.Tensor:
    raw = np.frombuffer(bytes(obj), dtype=np.uint8).copy()
    return torch.from_numpy(raw).to(device)


@dataclass
class GranuleInfo:
    data: torch.Tensor
    overviews: List[torch.Tensor]
    geot: List[float]
    srs: str
    nodata: Optional[float]
    timestamp: float
    polygon: str
    namespace: str
    signed_byte: bool


class GranuleSet:
    """HBM-resident granules: the stand-in for the GDAL datasets the worker
    opens (warp.go:89-101).  Overviews are finest first (GDALGetOverview)."""

    def __init__(self, device=None):
        self.device = torch.device(device or "cuda")
        self.items: List[GranuleInfo] = []

    def add(self, data: torch.Tensor, geot: Sequence[float], srs: str, nodata: Optional[float] = None,
            overviews: Sequence[torch.Tensor] = (), timestamp: float = 0.0, polygon: str = "",
            namespace: str = "", signed_byte: bool = False) -> int:
        if data.dim() != 2:
            raise ValueError("granule data must be 2-D (ysize, xsize)")
        if len(overviews) > _lib.MAX_OVR:
            raise ValueError("too many overviews")
        d = data.to(self.device).contiguous()
        ovr = [o.to(self.device).contiguous() for o in overviews]
        self.items.append(GranuleInfo(d, ovr, list(geot), srs, nodata, float(timestamp), polygon, namespace,
                                      signed_byte or data.dtype == torch.int8))
        return len(self.items) - 1

    def __len__(self):
        return len(self.items)


class TileBatch:
    """A batch of GetMap tiles over a GranuleSet.

    tiles: list of (bbox [minx, miny, maxx, maxy] in dst_srs, width, height).
    pairs: per tile, the granule indices the indexer returned (MAS order).
    namespaces: ConfigPayLoad.NameSpaces (rendered order: 1 -> palette/grey,
    3 -> RGB); granules of `mask.id` form the mask layer."""

    def __init__(self, granules: GranuleSet, dst_srs: Optional[str], tiles, pairs: Sequence[Sequence[int]],
                 namespaces: Sequence[str] = ("",), mask: Optional[Mask] = None,
                 slot: Optional[Tuple[int, int]] = None):
        if len(tiles) != len(pairs):
            raise ValueError("one granule list per tile")
        self.granules = granules
        self.device = granules.device
        self.namespaces = list(namespaces)
        self.mask = mask
        slots = list(self.namespaces)
        if mask is not None and mask.id not in slots:
            slots.append(mask.id)
        if len(slots) > 4:
            raise ValueError("at most 4 namespace slots per batch")
        self.slots = slots
        # CRS table: distinct SRS strings, destination last
        specs = []
        for g in granules.items:
            if g.srs not in specs:
                specs.append(g.srs)
        crs_list = [parse_crs(s) for s in specs]
        self.dst_crs = -1
        if dst_srs:
            crs_list.append(parse_crs(dst_srs))
            self.dst_crs = len(crs_list) - 1
        self.n_crs = len(crs_list)
        self._crs = _to_device_bytes((_lib.Crs * len(crs_list))(*crs_list), self.device)
        # granule table
        n = len(granules.items)
        garr = (_lib.Granule * max(1, n))()
        for i, g in enumerate(granules.items):
            c = garr[i]
            c.data = g.data.data_ptr()
            c.dtype = DTYPE_OF_TORCH[g.data.dtype]
            c.ysize, c.xsize = g.data.shape
            c.signed_byte = int(g.signed_byte)
            for k in range(6):
                c.geot[k] = g.geot[k]
            c.nodata = g.nodata if g.nodata is not None else -1e10
            c.has_nodata = int(g.nodata is not None)
            c.crs = specs.index(g.srs)
            c.n_ovr = len(g.overviews)
            for k, o in enumerate(g.overviews):
                c.ovr_data[k] = o.data_ptr()
                c.ovr_ysize[k], c.ovr_xsize[k] = o.shape
            c.timestamp = g.timestamp
            c.polygon_hash = fnv32a(g.polygon)
            c.ns = slots.index(g.namespace) if g.namespace in slots else 3
        self.n_granules = n
        self._gran = _to_device_bytes(garr, self.device)
        # value types the stack entries warp to (warp.go:232-243, 354-359);
        # a non-inclusive mask layer is not merged, so it does not count
        vts = 0
        for g in granules.items:
            if mask is not None and g.namespace == mask.id and not mask.inclusive:
                continue
            dt = DTYPE_OF_TORCH[g.data.dtype]
            if dt not in (_lib.BYTE, _lib.INT16, _lib.UINT16, _lib.FLOAT32):
                dt = _lib.FLOAT32
            if dt == _lib.BYTE and g.signed_byte:
                dt = _lib.SIGNEDBYTE
            vts |= _lib.VT_BIT[dt]
        self.value_types = vts
        # tiles + pairs (CSR)
        flat: List[int] = []
        tarr = (_lib.Tile * max(1, len(tiles)))()
        self.max_w = 1
        self.max_h = 1
        for i, (bbox, w, h) in enumerate(tiles):
            gt = bbox_to_geot(w, h, bbox)
            for k in range(6):
                tarr[i].dst_geot[k] = gt[k]
            tarr[i].width, tarr[i].height = w, h
            tarr[i].pair_begin = len(flat)
            flat.extend(int(p) for p in pairs[i])
            tarr[i].pair_end = len(flat)
            self.max_w = max(self.max_w, w)
            self.max_h = max(self.max_h, h)
        if slot is not None:   # a fixed (max_w, max_h) tile slot, e.g. a chunk of a PipelinedBatch
            if slot[0] < self.max_w or slot[1] < self.max_h:
                raise ValueError("tile larger than the slot")
            self.max_w, self.max_h = int(slot[0]), int(slot[1])
        self.n_tiles = len(tiles)
        self.n_pairs = len(flat)
        self.tile_sizes = [(w, h) for (_, w, h) in tiles]
        self._tarr = tarr
        self._tiles = _to_device_bytes(tarr, self.device)
        self._pairs = torch.tensor(flat if flat else [0], dtype=torch.int32, device=self.device)
        ws = lib().gskyhip_render_workspace_size(self.n_tiles, self.n_pairs, self.max_h)
        self._ws = torch.empty(int(ws), dtype=torch.uint8, device=self.device)
        self._mask_c = mask.c(slots.index(mask.id)) if mask is not None else None
        self.typed = True   # pass the value-type hint (False: force the generic kernels)

    # ------------------------------------------------------------------ render
    def render(self, params: ScaleParams, palette: Optional[Palette] = None, resample: int = 0,
               out: Optional[torch.Tensor] = None, canvas: bool = False, phase: int = 0, rgba: bool = True):
        """Warp + merge + scale + RGBA for every tile.  Returns the RGBA
        tensor (n_tiles, H, W, 4); with canvas=True also the typed canvases
        (n_tiles, n_out, H*W*4 bytes).  rgba=False renders canvases only (WCS).
        phase 1 / 2 run the planning / render kernels alone (same arguments)."""
        n_out = len(self.namespaces)
        if n_out not in (1, 3):
            raise ValueError("Cannot encode other than 1 or 3 namespaces into a PNG: Received %d" % n_out)
        if rgba and out is None:
            out = self._out if getattr(self, "_out", None) is not None else None
            if out is None:
                out = torch.empty((self.n_tiles, self.max_h, self.max_w, 4), dtype=torch.uint8,
                                  device=self.device)
                self._out = out
        autom = rgba and params.offset == 0 and params.scale == 0 and params.clip == 0
        cv = None
        if canvas or autom or not rgba:
            cv = getattr(self, "_cv", None)
            if cv is None:
                cv = torch.empty((self.n_tiles, n_out, self.max_h * self.max_w * 4), dtype=torch.uint8,
                                 device=self.device)
                self._cv = cv
        if not hasattr(self, "_ramp_key") or self._ramp_key != id(palette):
            ramp = gradient_rgba_palette(palette) if (palette is not None and n_out == 1) else None
            self._ramp = torch.from_numpy(ramp).to(self.device) if ramp is not None else None
            self._ramp_key = id(palette)
        # the call's arguments, built once per distinct request shape (a
        # one-tile GetMap is latency-bound: building ~25 ctypes objects per
        # call cost as much host time as the planning kernel takes on the GPU)
        stream = torch.cuda.current_stream().cuda_stream
        key = (phase, self.typed, out.data_ptr() if rgba else 0, cv.data_ptr() if cv is not None else 0,
               self._ramp.data_ptr() if self._ramp is not None else 0, resample, params.offset, params.scale,
               params.clip, params.colour_scale, stream, self._ws.data_ptr())
        cache = self.__dict__.setdefault("_call_cache", {})
        args = cache.get(key)
        if args is None:
            out_ns = (C.c_int32 * 3)(*[self.slots.index(ns) for ns in self.namespaces] + [0] * (3 - n_out))
            sp = params.c()
            args = (phase, self.value_types if self.typed else 0, self._gran.data_ptr(), self.n_granules,
                    self._crs.data_ptr(), self.n_crs, self.dst_crs, self._tiles.data_ptr(), self.n_tiles,
                    self._pairs.data_ptr(), self.n_pairs, self.max_w, self.max_h, out_ns, n_out,
                    C.byref(self._mask_c) if self._mask_c is not None else None, resample, C.byref(sp),
                    self._ramp.data_ptr() if self._ramp is not None else None,
                    out.data_ptr() if rgba else None, cv.data_ptr() if cv is not None else None,
                    self._ws.data_ptr(), self._ws.numel(), stream)
            if len(cache) > 64:
                cache.clear()
            cache[key] = args = (args, sp, out_ns)   # the structs the byrefs point at stay alive with them
        check(lib().gskyhip_render_tiles_typed(*args[0]), "render_tiles")
        if not rgba:
            return cv
        return (out, cv) if canvas else out

    # ------------------------------------------------------------------ graphs
    def set_tiles(self, tiles) -> None:
        """New requests of the same shape: every tile's (bbox, width, height)
        is replaced, its granule list (CSR) kept.  The descriptors go to HBM on
        the current stream (pinned host buffer, asynchronous), ahead of the
        next render or graph replay."""
        if len(tiles) != self.n_tiles:
            raise ValueError("set_tiles: %d tiles for a batch of %d" % (len(tiles), self.n_tiles))
        for i, (bbox, w, h) in enumerate(tiles):
            if w > self.max_w or h > self.max_h:
                raise ValueError("set_tiles: tile %d larger than the batch slot" % i)
            gt = bbox_to_geot(w, h, bbox)
            for k in range(6):
                self._tarr[i].dst_geot[k] = gt[k]
            self._tarr[i].width, self._tarr[i].height = w, h
        self.tile_sizes = [(w, h) for (_, w, h) in tiles]
        host = getattr(self, "_tiles_pinned", None)
        if host is None:
            host = torch.empty(self._tiles.numel(), dtype=torch.uint8).pin_memory()
            self._tiles_pinned = host
        else:
            torch.cuda.current_stream().synchronize()   # the previous upload has left the buffer
        host.numpy()[:] = np.frombuffer(bytes(self._tarr), dtype=np.uint8)
        self._tiles.copy_(host, non_blocking=True)

    def graph(self, params: ScaleParams, palette: Optional[Palette] = None, resample: int = 0) -> "RenderGraph":
        """The batch's render (planning + band kernels, RGBA out) captured as
        one HIP graph (see RenderGraph)."""
        return RenderGraph(self, params, palette, resample)

    def render_coverage(self, params: ScaleParams, out: torch.Tensor, offsets, resample: int = 0,
                        phase: int = 0) -> torch.Tensor:
        """WCS GetCoverage: every tile's typed canvas of the first namespace
        written straight into `out` (a 2-D tensor of the canvas type) with
        tile t's top-left at flat element offset offsets[t]
        (gskyhip_render_coverage; no per-tile slots, no assembly copy)."""
        if out.dim() != 2:
            raise ValueError("coverage must be 2-D")
        offs = offsets if isinstance(offsets, torch.Tensor) else torch.tensor(list(offsets), dtype=torch.int64)
        offs = offs.to(self.device, torch.int64).contiguous()
        self._cov_offs = offs
        sp = params.c()
        stream = C.c_void_p(torch.cuda.current_stream().cuda_stream)
        check(lib().gskyhip_render_coverage(
            phase, self.value_types if self.typed else 0, C.c_void_p(self._gran.data_ptr()), self.n_granules,
            C.c_void_p(self._crs.data_ptr()), self.n_crs, self.dst_crs, C.c_void_p(self._tiles.data_ptr()),
            self.n_tiles, C.c_void_p(self._pairs.data_ptr()), self.n_pairs, self.max_w, self.max_h, resample,
            C.byref(sp), C.c_void_p(offs.data_ptr()), out.shape[1], C.c_void_p(out.data_ptr()),
            C.c_void_p(self._ws.data_ptr()), self._ws.numel(), stream), "render_coverage")
        return out

    def status(self) -> int:
        """TilePlan status of the last call (synchronous): 0 or an error code."""
        stream = C.c_void_p(torch.cuda.current_stream().cuda_stream)
        return lib().gskyhip_render_status(C.c_void_p(self._ws.data_ptr()), self.n_tiles, self.n_pairs,
                                           self.max_h, stream)

    def tile_info(self):
        """Per tile (status, complex, value type, merged entries) of the last
        plan (gskyhip_render_tile_info), an int32 numpy array (n_tiles, 4);
        also sets self.plan_counters (leaf pool, split rows, complex tiles)."""
        import numpy as np
        info = np.zeros((max(1, self.n_tiles), 4), dtype=np.int32)
        cnt = np.zeros(3, dtype=np.int32)
        stream = C.c_void_p(torch.cuda.current_stream().cuda_stream)
        check(lib().gskyhip_render_tile_info(C.c_void_p(self._ws.data_ptr()), self.n_tiles, self.n_pairs, self.max_h,
                                             info.ctypes.data_as(C.c_void_p), cnt.ctypes.data_as(C.c_void_p),
                                             stream), "render_tile_info")
        self.plan_counters = {"pool_leaves": int(cnt[0]), "split_rows": int(cnt[1]), "complex_tiles": int(cnt[2])}
        return info[: self.n_tiles]

    def pair_info(self):
        """Per pair of the last plan (gskyhip_render_pair_info): int32 numpy
        array (n_pairs, 8) = granule, picked level width / height, element
        bytes, source footprint x0, y0, x1, y1 at that level."""
        out = np.zeros((max(1, self.n_pairs), 8), dtype=np.int32)
        stream = C.c_void_p(torch.cuda.current_stream().cuda_stream)
        check(lib().gskyhip_render_pair_info(C.c_void_p(self._ws.data_ptr()), self.n_tiles, self.n_pairs, self.max_h,
                                             out.ctypes.data_as(C.c_void_p), stream), "render_pair_info")
        return out[: self.n_pairs]

    def touched_bytes(self):
        """Algorithmic source bytes of the last plan (gskyhip_render_touched):
        (distinct source elements x element bytes, distinct 128-byte lines x
        128) over every pair's window pixels at the picked levels."""
        out = np.zeros(2, dtype=np.int64)
        stream = C.c_void_p(torch.cuda.current_stream().cuda_stream)
        check(lib().gskyhip_render_touched(C.c_void_p(self._ws.data_ptr()), self.n_tiles, self.n_pairs, self.max_h,
                                           out.ctypes.data_as(C.c_void_p), stream), "render_touched")
        return int(out[0]), int(out[1])

    def canvas_view(self, cv: torch.Tensor, tile: int, k: int, type_name: str) -> torch.Tensor:
        nb = {"Byte": 1, "SignedByte": 1, "Int16": 2, "UInt16": 2, "Float32": 4}[type_name]
        return cv[tile, k, : self.max_w * self.max_h * nb].view(TORCH_OF[type_name]).reshape(self.max_h,
                                                                                              self.max_w)

    # ------------------------------------------------------------------ windows
    def warp_windows(self, resample: int = 0):
        """The FlexRasters of tile_grpc.go:228-241: per pair
        (window tensor, bbox [xoff, yoff, w, h], type name, nodata)."""
        npairs = self.n_pairs
        bbox = torch.zeros((max(1, npairs), 4), dtype=torch.int32, device=self.device)
        dt = torch.zeros(max(1, npairs), dtype=torch.int32, device=self.device)
        nd = torch.zeros(max(1, npairs), dtype=torch.float64, device=self.device)
        stride = self.max_w * self.max_h * 4
        win = torch.empty((max(1, npairs), stride), dtype=torch.uint8, device=self.device)
        stream = C.c_void_p(torch.cuda.current_stream().cuda_stream)
        check(lib().gskyhip_warp_windows(
            C.c_void_p(self._gran.data_ptr()), self.n_granules, C.c_void_p(self._crs.data_ptr()), self.n_crs,
            self.dst_crs, C.c_void_p(self._tiles.data_ptr()), self.n_tiles, C.c_void_p(self._pairs.data_ptr()),
            npairs, self.max_w, self.max_h, resample, C.c_void_p(bbox.data_ptr()), C.c_void_p(dt.data_ptr()),
            C.c_void_p(nd.data_ptr()), C.c_void_p(win.data_ptr()), stride, C.c_void_p(self._ws.data_ptr()),
            self._ws.numel(), stream), "warp_windows")
        bb = bbox.cpu().numpy()
        dts = dt.cpu().numpy()
        nds = nd.cpu().numpy()
        out = []
        for p in range(npairs):
            tname = TYPE_NAMES[int(dts[p])]
            w, h = int(bb[p, 2]), int(bb[p, 3])
            nb = {"Byte": 1, "SignedByte": 1, "Int16": 2, "UInt16": 2, "Float32": 4}[tname]
            t = win[p, : w * h * nb].view(TORCH_OF[tname]).reshape(h, w)
            out.append((t, bb[p].tolist(), tname, float(nds[p])))
        return out


class RenderGraph:
    """One TileBatch.render() captured as a HIP graph: the ~10 planning and
    band-kernel launches of a request replay with one host call, which is
    what bounds the latency of a single small tile (BASELINE C1).  Every
    kernel reads the tile, pair and granule descriptors from HBM when it
    runs, so a new request of the same shape (tile count, pair lists, slot
    size) is served by TileBatch.set_tiles() followed by replay(); the
    result lands in the same RGBA tensor."""

    def __init__(self, batch: TileBatch, params: ScaleParams, palette: Optional[Palette], resample: int):
        self.batch = batch
        batch.render(params, palette, resample)   # loads the kernels, allocates the output and the ramp
        torch.cuda.synchronize()
        self._graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self._graph):
            self.out = batch.render(params, palette, resample)
        torch.cuda.synchronize()

    def replay(self) -> torch.Tensor:
        self._graph.replay()
        return self.out


class PipelinedBatch:
    """A GetMap batch cut into contiguous chunks of tiles, each its own
    TileBatch (own workspace), issued round-robin on `n_streams` HIP streams:
    the planning kernels of chunk k+1 (latency-bound fp64 transforms, few
    waves) run while the render kernel of chunk k streams RGBA.  Tiles are
    independent requests (tile_grpc.go:96-258), so the RGBA is identical to
    one TileBatch over all tiles; every chunk uses the batch's tile slot, so
    the output layout is the same (n_tiles, max_h, max_w, 4) tensor."""

    def __init__(self, granules: GranuleSet, dst_srs: Optional[str], tiles, pairs: Sequence[Sequence[int]],
                 namespaces: Sequence[str] = ("",), mask: Optional[Mask] = None, n_chunks: int = 4,
                 n_streams: int = 2):
        if len(tiles) != len(pairs):
            raise ValueError("one granule list per tile")
        n = len(tiles)
        n_chunks = max(1, min(int(n_chunks), n)) if n else 1
        self.device = granules.device
        self.max_w = max([w for (_, w, _) in tiles] + [1])
        self.max_h = max([h for (_, _, h) in tiles] + [1])
        self.n_tiles = n
        bounds = [n * k // n_chunks for k in range(n_chunks + 1)]
        self.chunks = [(b0, b1, TileBatch(granules, dst_srs, tiles[b0:b1], pairs[b0:b1], namespaces, mask,
                                          slot=(self.max_w, self.max_h)))
                       for b0, b1 in zip(bounds[:-1], bounds[1:]) if b1 > b0]
        self.n_pairs = sum(c[2].n_pairs for c in self.chunks)
        self.streams = [torch.cuda.Stream(device=self.device) for _ in range(max(1, int(n_streams)))]
        self._out = None

    def render(self, params: ScaleParams, palette: Optional[Palette] = None, resample: int = 0,
               out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """RGBA of every tile, (n_tiles, max_h, max_w, 4); ordered after the
        work already queued on the current stream, and the current stream
        waits for every chunk."""
        if out is None:
            if self._out is None:
                self._out = torch.empty((self.n_tiles, self.max_h, self.max_w, 4), dtype=torch.uint8,
                                        device=self.device)
            out = self._out
        cur = torch.cuda.current_stream(self.device)
        for s in self.streams:
            s.wait_stream(cur)
        for k, (b0, b1, tb) in enumerate(self.chunks):
            with torch.cuda.stream(self.streams[k % len(self.streams)]):
                tb.render(params, palette, resample, out=out[b0:b1])
        for s in self.streams:
            cur.wait_stream(s)
        return out

    def status(self) -> int:
        """First non-zero planning status of any chunk (0: all tiles rendered)."""
        for _, _, tb in self.chunks:
            st = tb.status()
            if st != 0:
                return st
        return 0
