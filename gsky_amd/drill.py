"""WPS drill (zonal statistics) on MI355X.

`DrillStack` holds a time stack resident in HBM in the time-innermost layout
([y][x][t], t padded to a multiple of 32: 128-byte aligned pixel rows).  `read_data` runs readData
(worker/gdalprocess/drill.go:90-227) for a batch of polygon windows at once;
`drill_merge` is the DrillMerger per-date weighted mean
(processor/drill_merger.go:79-93).
"""
from __future__ import annotations

import ctypes as C
from typing import List, Optional, Sequence, Tuple

import numpy as np
import torch

from ._lib import check, lib


def _stream():
    return C.c_void_p(torch.cuda.current_stream().cuda_stream)


_WS = {}


def _workspace(dev, nbytes: int) -> torch.Tensor:
    """The drill workspace of (device, stream), grown as needed and kept:
    readData with deciles needs gigabytes of it, and a fresh allocation per
    request costs more than the kernels (calls on one stream are ordered, so
    they can share it)."""
    key = (str(dev), torch.cuda.current_stream(dev).cuda_stream)
    t = _WS.get(key)
    if t is None or t.numel() < nbytes:
        _WS.pop(key, None)
        t = torch.empty(max(1, int(nbytes)), dtype=torch.uint8, device=dev)
        _WS[key] = t
    return t


class DrillStack:
    """Float32 time stack (n_bands, ysize, xsize) -> HBM [y][x][t_stride]."""

    def __init__(self, bands: torch.Tensor, nodata: float, device=None):
        if bands.dim() != 3:
            raise ValueError("stack must be (n_bands, ysize, xsize)")
        nb, ys, xs = bands.shape
        self.n_bands, self.ysize, self.xsize = nb, ys, xs
        # many slices: 128-byte pixel rows, so a 32-slice group never straddles
        # an extra line; few slices: 16 bytes (padding to 32 would multiply a
        # 1-band stack's HBM by 32)
        self.t_stride = (nb + 31) // 32 * 32 if nb > 16 else (nb + 3) // 4 * 4
        dev = torch.device(device or "cuda")
        st = torch.zeros((ys, xs, self.t_stride), dtype=torch.float32, device=dev)
        st[:, :, :nb] = bands.to(dev, torch.float32).permute(1, 2, 0)
        self.stack = st
        self.nodata = float(nodata)

    @classmethod
    def from_time_innermost(cls, stack: torch.Tensor, n_bands: int, nodata: float):
        """Wrap an already laid out (ysize, xsize, t_stride) float32 tensor."""
        self = cls.__new__(cls)
        self.ysize, self.xsize, self.t_stride = stack.shape
        self.n_bands = n_bands
        self.stack = stack.contiguous()
        self.nodata = float(nodata)
        return self


class MaskBatch:
    """Per-polygon window masks packed for the GPU: `win` (n, 4) int32
    {off_x, off_y, count_x, count_y}, `mask_off` (n,) int64 byte offsets
    (16-byte aligned, in polygon order, non-overlapping) and `masks` (uint8,
    255 = inside).  Iterates as (win, mask_off, masks) for round-1 callers."""

    def __init__(self, win, mask_off, masks):
        self.win, self.mask_off, self.masks = win, mask_off, masks
        self.n = int(win.shape[0])
        self.mask_bytes = int(masks.numel())

    def __iter__(self):
        return iter((self.win, self.mask_off, self.masks))


def pack_masks(windows: Sequence[Tuple[int, int, int, int]], masks: Sequence[np.ndarray], device=None) -> MaskBatch:
    """Concatenate per-polygon window masks (count_y, count_x; 255 = inside),
    16-byte aligned, into HBM."""
    offs = []
    total = 0
    for m in masks:
        offs.append(total)
        total += (m.size + 15) // 16 * 16
    buf = np.zeros(max(16, total), np.uint8)
    for o, m in zip(offs, masks):
        buf[o:o + m.size] = np.ascontiguousarray(m, np.uint8).reshape(-1)
    dev = torch.device(device or "cuda")
    win = torch.tensor(np.asarray(windows, np.int32).reshape(-1, 4), device=dev)
    off = torch.tensor(np.asarray(offs, np.int64), device=dev)
    return MaskBatch(win, off, torch.from_numpy(buf).to(dev))


def drill_descriptors(geometries: Sequence[str], dataset_srs: Optional[str], geot: Sequence[float], xsize: int,
                      ysize: int):
    """getDrillFileDescriptor + createMask (drill.go:363-423, 275-327) for a
    batch of GeoJSON geometries against one dataset: (windows (n, 4) int32,
    mask_off (n,) int64, masks uint8 host buffer, status (n,) int32)."""
    n = len(geometries)
    arr = (C.c_char_p * max(1, n))(*[g.encode() for g in geometries])
    gt = (C.c_double * 6)(*geot)
    win = np.zeros((max(1, n), 4), np.int32)
    off = np.zeros(max(1, n), np.int64)
    st = np.zeros(max(1, n), np.int32)
    total = C.c_int64()
    srs = dataset_srs.encode() if dataset_srs else None
    L = lib()
    check(L.gskyhip_drill_descriptors(arr, n, srs, gt, xsize, ysize, win.ctypes.data_as(C.c_void_p),
                                      off.ctypes.data_as(C.c_void_p), C.byref(total), None,
                                      st.ctypes.data_as(C.c_void_p)), "drill_descriptors")
    buf = np.zeros(int(total.value), np.uint8)
    check(L.gskyhip_drill_descriptors(arr, n, srs, gt, xsize, ysize, win.ctypes.data_as(C.c_void_p),
                                      off.ctypes.data_as(C.c_void_p), C.byref(total),
                                      buf.ctypes.data_as(C.c_void_p), st.ctypes.data_as(C.c_void_p)),
          "drill_descriptors")
    return win[:n], off[:n], buf, st[:n]


def drill_windows(geometries: Sequence[str], dataset_srs: Optional[str], geot: Sequence[float], xsize: int,
                  ysize: int) -> Tuple[np.ndarray, np.ndarray]:
    """The windows (n, 4) and status (n,) of getDrillFileDescriptor
    (drill.go:363-423) without rasterizing a mask (host only)."""
    n = len(geometries)
    arr = (C.c_char_p * max(1, n))(*[g.encode() for g in geometries])
    gt = (C.c_double * 6)(*geot)
    win = np.zeros((max(1, n), 4), np.int32)
    off = np.zeros(max(1, n), np.int64)
    st = np.zeros(max(1, n), np.int32)
    total = C.c_int64()
    check(lib().gskyhip_drill_descriptors_device(arr, n, dataset_srs.encode() if dataset_srs else None, gt, xsize,
                                                 ysize, win.ctypes.data_as(C.c_void_p),
                                                 off.ctypes.data_as(C.c_void_p), C.byref(total), None,
                                                 st.ctypes.data_as(C.c_void_p), None), "drill_windows")
    return win[:n], st[:n]


def drill_dataset(geometries: Sequence[str], dataset_srs: Optional[str], geot: Sequence[float], xsize: int,
                  ysize: int, device=None, rasterize: str = "gpu") -> Tuple["MaskBatch", np.ndarray]:
    """DrillDataset's geometry step for a batch of requests: the windows and
    ALL_TOUCHED masks as a MaskBatch in HBM, plus the per-polygon status (0
    ok; a polygon that misses the file gets an empty window).  rasterize
    "gpu" burns the masks on the device (gskyhip_drill_descriptors_device),
    "host" rasterizes on the CPU and uploads them."""
    dev = torch.device(device or "cuda")
    if rasterize == "host":
        win, off, buf, st = drill_descriptors(geometries, dataset_srs, geot, xsize, ysize)
        return MaskBatch(torch.from_numpy(win.copy()).to(dev), torch.from_numpy(off.copy()).to(dev),
                         torch.from_numpy(buf).to(dev)), st
    n = len(geometries)
    packed = ("\0".join(geometries) + "\0").encode()   # one buffer, no per-string objects
    gt = (C.c_double * 6)(*geot)
    # windows and mask offsets written by the library straight into pinned
    # memory, then one asynchronous upload (no pageable copies, no wait)
    m = max(1, n)
    pin = _pinned_meta(24 * m)
    hb = pin.numpy()
    win = hb[:16 * m].view(np.int32).reshape(m, 4)
    off = hb[16 * m:24 * m].view(np.int64)
    st = np.zeros(m, np.int32)
    total = C.c_int64()
    srs = dataset_srs.encode() if dataset_srs else None
    L = lib()
    # one pass: the library describes every polygon once and asks for the
    # mask buffer through the callback (a torch tensor kept here)
    held = []

    def alloc(_ctx, nbytes):
        t = torch.empty(int(nbytes), dtype=torch.uint8, device=dev)
        held.append(t)
        return t.data_ptr()
    cb = _ALLOC_FN(alloc)
    mptr = C.c_void_p()
    check(L.gskyhip_drill_masks_device_packed(packed, len(packed), n, srs, gt, xsize, ysize,
                                              win.ctypes.data_as(C.c_void_p), off.ctypes.data_as(C.c_void_p),
                                              C.byref(total), cb, None, C.byref(mptr), st.ctypes.data_as(C.c_void_p),
                                              _stream()), "drill_masks_device")
    masks = held[0]
    meta = torch.empty(24 * m, dtype=torch.uint8, device=dev)
    meta.copy_(pin[:24 * m], non_blocking=True)
    _META_EVENT[0] = torch.cuda.Event()
    _META_EVENT[0].record()
    mb = MaskBatch(meta[:16 * n].view(torch.int32).view(n, 4), meta[16 * m:16 * m + 8 * n].view(torch.int64), masks)
    return mb, st[:n]


_META_PIN: List[torch.Tensor] = []
_META_EVENT: List[Optional[torch.cuda.Event]] = [None]


def _pinned_meta(nbytes: int) -> torch.Tensor:
    """A pinned host buffer of at least nbytes for drill_dataset's windows
    and offsets, reused across calls once the previous upload from it is
    done."""
    if _META_EVENT[0] is not None:
        _META_EVENT[0].synchronize()
    if not _META_PIN or _META_PIN[0].numel() < nbytes:
        _META_PIN[:] = [torch.empty(max(nbytes, 1 << 16), dtype=torch.uint8).pin_memory()]
    return _META_PIN[0]


_ALLOC_FN = C.CFUNCTYPE(C.c_void_p, C.c_void_p, C.c_int64)


REFERENCE_ORDER, WAVE_SPLIT = 0, 1


def read_data(stack: DrillStack, win, mask_off=None, masks=None, clip_lower: float = -3.4028234663852886e38,
              clip_upper: float = 3.4028234663852886e38, pixel_count: int = 0, band_strides: int = 1,
              decile_count: int = 0, bands: Optional[Sequence[int]] = None, mode: int = REFERENCE_ORDER):
    """readData (drill.go:90-227) for every polygon window -> (values f64,
    counts i32), each (n_polys, rows) with rows = len(TimeSeries) / nCols of
    drill.go:225.  `win` is a MaskBatch (or the round-1 (win, mask_off,
    masks) tensors); `bands` the reference's 1-based band list (default all);
    mode REFERENCE_ORDER is bit-exact, WAVE_SPLIT within 1e-5 relative.
    decile_count > 0: values / counts (n_polys, rows, 1 + decile_count),
    each row [mean, decile 1..k] as the reference's TimeSeries (drill.go:
    172-214: Count 1 per decile, zeros with Count 0 where the band total is
    0, interpolated rows for bandStrides > 2); see read_data_deciles."""
    mb = win if isinstance(win, MaskBatch) else MaskBatch(win, mask_off, masks)
    if decile_count:
        return read_data_deciles(stack, mb, clip_lower, clip_upper, pixel_count, band_strides, decile_count, bands,
                                 mode)
    n_polys = mb.n
    blist = None if bands is None else np.ascontiguousarray(bands, np.int32)
    n_list = stack.n_bands if blist is None else len(blist)
    rows = lib().gskyhip_drill_rows(n_list, band_strides)
    dev = stack.stack.device
    vals = torch.empty((n_polys, rows), dtype=torch.float64, device=dev)
    cnts = torch.empty((n_polys, rows), dtype=torch.int32, device=dev)
    ws_bytes = lib().gskyhip_drill_workspace_size(n_polys, mb.mask_bytes, n_list, band_strides, mode)
    ws = _workspace(dev, int(ws_bytes))
    check(lib().gskyhip_drill_batch(C.c_void_p(stack.stack.data_ptr()), stack.xsize, stack.ysize, stack.n_bands,
                                    stack.t_stride, C.c_void_p(mb.win.data_ptr()), C.c_void_p(mb.mask_off.data_ptr()),
                                    C.c_void_p(mb.masks.data_ptr()), n_polys, mb.mask_bytes,
                                    blist.ctypes.data_as(C.c_void_p) if blist is not None else None, n_list,
                                    stack.nodata, clip_lower, clip_upper, pixel_count, band_strides, mode,
                                    C.c_void_p(vals.data_ptr()), C.c_void_p(cnts.data_ptr()),
                                    C.c_void_p(ws.data_ptr()), ws.numel(), _stream()), "drill")
    return vals, cnts


def read_data_deciles(stack: DrillStack, mb: "MaskBatch", clip_lower: float, clip_upper: float, pixel_count: int,
                      band_strides: int, decile_count: int, bands: Optional[Sequence[int]] = None,
                      mode: int = REFERENCE_ORDER):
    """readData with decileCount > 0 and any bandStrides in one call
    (gskyhip_drill_read_data): the read bands' means, their deciles by radix
    selection, the TimeSeries rows.  Raises GskyError(-7) where the reference's
    computeDeciles would panic (drill.go:247-253)."""
    n_polys = mb.n
    blist = None if bands is None else np.ascontiguousarray(bands, np.int32)
    n_list = stack.n_bands if blist is None else len(blist)
    rows = lib().gskyhip_drill_rows(n_list, band_strides)
    dev = stack.stack.device
    nc = 1 + decile_count
    vals = torch.empty((n_polys, rows, nc), dtype=torch.float64, device=dev)
    cnts = torch.empty((n_polys, rows, nc), dtype=torch.int32, device=dev)
    st = torch.empty(n_polys, dtype=torch.int32, device=dev)
    ws_bytes = lib().gskyhip_drill_read_data_workspace_size(n_polys, mb.mask_bytes, n_list, band_strides,
                                                            decile_count, mode)
    if ws_bytes < 0:
        raise ValueError("readData workspace out of range")
    ws = _workspace(dev, int(ws_bytes))
    check(lib().gskyhip_drill_read_data(C.c_void_p(stack.stack.data_ptr()), stack.xsize, stack.ysize,
                                        stack.n_bands, stack.t_stride, C.c_void_p(mb.win.data_ptr()),
                                        C.c_void_p(mb.mask_off.data_ptr()), C.c_void_p(mb.masks.data_ptr()),
                                        n_polys, mb.mask_bytes,
                                        blist.ctypes.data_as(C.c_void_p) if blist is not None else None, n_list,
                                        stack.nodata, clip_lower, clip_upper, pixel_count, band_strides,
                                        decile_count, mode, C.c_void_p(vals.data_ptr()), C.c_void_p(cnts.data_ptr()),
                                        C.c_void_p(st.data_ptr()), C.c_void_p(ws.data_ptr()), ws.numel(),
                                        _stream()), "drill_read_data")
    if bool((st == -7).any()):
        from ._lib import GskyError
        raise GskyError(-7, "computeDeciles indexes past the values (the reference panics)")
    return vals, cnts


def compute_deciles(stack: DrillStack, mb: "MaskBatch", totals: torch.Tensor, decile_count: int,
                    bands: Optional[Sequence[int]] = None, band_chunk: int = 0):
    """computeDeciles (drill.go:229-273) of every polygon and band:
    (deciles float32 (n_polys, n_list, decile_count), status int32 (n_polys,
    n_list): 0, 1 = band total 0, -7 = the reference would panic).  `totals`:
    the mean pass's counts (n_polys, n_list)."""
    n_polys = mb.n
    blist = None if bands is None else np.ascontiguousarray(bands, np.int32)
    n_list = stack.n_bands if blist is None else len(blist)
    dev = stack.stack.device
    if band_chunk <= 0:   # bound the segment buffer (mask_bytes x chunk values) to 4 GiB
        band_chunk = int(max(1, min(n_list, (1 << 30) // max(1, mb.mask_bytes))))
    ws_bytes = lib().gskyhip_drill_deciles_workspace_size(n_polys, mb.mask_bytes, band_chunk)
    if ws_bytes < 0:
        raise ValueError("deciles workspace: mask_bytes x band_chunk must stay below 2^31")
    ws = _workspace(dev, int(ws_bytes))
    out = torch.empty((n_polys, n_list, decile_count), dtype=torch.float32, device=dev)
    st = torch.empty((n_polys, n_list), dtype=torch.int32, device=dev)
    tot = totals.to(dev, torch.int32).contiguous()
    check(lib().gskyhip_drill_deciles(C.c_void_p(stack.stack.data_ptr()), stack.xsize, stack.ysize, stack.n_bands,
                                      stack.t_stride, C.c_void_p(mb.win.data_ptr()),
                                      C.c_void_p(mb.mask_off.data_ptr()), C.c_void_p(mb.masks.data_ptr()), n_polys,
                                      mb.mask_bytes, blist.ctypes.data_as(C.c_void_p) if blist is not None else None,
                                      n_list, stack.nodata, decile_count, band_chunk, C.c_void_p(tot.data_ptr()),
                                      C.c_void_p(out.data_ptr()), C.c_void_p(st.data_ptr()),
                                      C.c_void_p(ws.data_ptr()), ws.numel(), _stream()), "drill_deciles")
    return out, st


def drill_merge(values: torch.Tensor, counts: torch.Tensor) -> torch.Tensor:
    """Per-date weighted mean over files (drill_merger.go:79-93); NaN = no value."""
    v = values.contiguous()
    c = counts.contiguous()
    nf, nd = v.shape
    out = torch.empty(nd, dtype=torch.float64, device=v.device)
    check(lib().gskyhip_drill_merge(C.c_void_p(v.data_ptr()), C.c_void_p(c.data_ptr()), nf, nd,
                                    C.c_void_p(out.data_ptr()), _stream()), "drill_merge")
    return out
