"""WPS drill (zonal statistics) on MI355X.

`DrillStack` holds a time stack resident in HBM in the time-innermost layout
([y][x][t], t padded to a multiple of 4).  `read_data` runs readData
(worker/gdalprocess/drill.go:90-227) for a batch of polygon windows at once;
`drill_merge` is the DrillMerger per-date weighted mean
(processor/drill_merger.go:79-93).
"""
from __future__ import annotations

import ctypes as C
from typing import List, Sequence, Tuple

import numpy as np
import torch

from ._lib import check, lib


def _stream():
    return C.c_void_p(torch.cuda.current_stream().cuda_stream)


class DrillStack:
    """Float32 time stack (n_bands, ysize, xsize) -> HBM [y][x][t_stride]."""

    def __init__(self, bands: torch.Tensor, nodata: float, device=None):
        if bands.dim() != 3:
            raise ValueError("stack must be (n_bands, ysize, xsize)")
        nb, ys, xs = bands.shape
        self.n_bands, self.ysize, self.xsize = nb, ys, xs
        self.t_stride = (nb + 3) // 4 * 4
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


def pack_masks(windows: Sequence[Tuple[int, int, int, int]], masks: Sequence[np.ndarray], device=None):
    """Concatenate per-polygon window masks (count_y, count_x; 255 = inside),
    16-byte aligned, into HBM.  Returns (win tensor, mask_off tensor, masks tensor)."""
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
    return win, off, torch.from_numpy(buf).to(dev)


def read_data(stack: DrillStack, win: torch.Tensor, mask_off: torch.Tensor, masks: torch.Tensor,
              clip_lower: float, clip_upper: float, pixel_count: int = 0, band_strides: int = 1,
              decile_count: int = 0):
    """readData for every polygon window -> (values f64, counts i32), each
    (n_polys, rows) with rows = len(TimeSeries) / nCols of drill.go:225."""
    if decile_count:
        raise NotImplementedError("drill deciles (drill.go:229-273) are SURVEY 8f 'next'")
    n_polys = win.shape[0]
    rows = lib().gskyhip_drill_rows(stack.n_bands, band_strides)
    vals = torch.empty((n_polys, rows), dtype=torch.float64, device=stack.stack.device)
    cnts = torch.empty((n_polys, rows), dtype=torch.int32, device=stack.stack.device)
    check(lib().gskyhip_drill(C.c_void_p(stack.stack.data_ptr()), stack.xsize, stack.ysize, stack.n_bands,
                              stack.t_stride, C.c_void_p(win.data_ptr()), C.c_void_p(mask_off.data_ptr()),
                              C.c_void_p(masks.data_ptr()), n_polys, stack.nodata, clip_lower, clip_upper,
                              pixel_count, band_strides, C.c_void_p(vals.data_ptr()),
                              C.c_void_p(cnts.data_ptr()), _stream()), "drill")
    return vals, cnts


def drill_merge(values: torch.Tensor, counts: torch.Tensor) -> torch.Tensor:
    """Per-date weighted mean over files (drill_merger.go:79-93); NaN = no value."""
    v = values.contiguous()
    c = counts.contiguous()
    nf, nd = v.shape
    out = torch.empty(nd, dtype=torch.float64, device=v.device)
    check(lib().gskyhip_drill_merge(C.c_void_p(v.data_ptr()), C.c_void_p(c.data_ptr()), nf, nd,
                                    C.c_void_p(out.data_ptr()), _stream()), "drill_merge")
    return out
