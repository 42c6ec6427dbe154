"""EncodePNG's png.Encode (utils/ogc_encoders.go:139, Go 1.12 image/png) on
the GPU path (gskyhip_encode_png): PNG structure (signature, IHDR colour type
RGB for opaque tiles / RGBA otherwise, IDAT chunks of 32768 bytes but the
last, IEND, CRCs), and the decompressed IDAT stream equal byte for byte to
the oracle's restatement of Go's writeImage (NRGBA conversion, per-row filter
choice).  The deflate bytes are the GPU deflate's (encode.hip), neither
zlib's nor Go's compress/flate (parity unpinned); every stream is inflated by
zlib and PIL decodes every PNG to the expected pixels."""
import io
import struct
import zlib

import numpy as np
import pytest

from gsky_amd import synth

from .helpers import gpu_batch

pytestmark = pytest.mark.gpu


def _chunks(png):
    assert png[:8] == b"\x89PNG\r\n\x1a\n"
    p, out = 8, []
    while p < len(png):
        n, = struct.unpack(">I", png[p:p + 4])
        typ = png[p + 4:p + 8]
        data = png[p + 8:p + 8 + n]
        crc, = struct.unpack(">I", png[p + 8 + n:p + 12 + n])
        assert crc == zlib.crc32(typ + data) & 0xFFFFFFFF
        out.append((typ, data))
        p += 12 + n
    return out


def _check(png, rgba, oracle):
    from PIL import Image
    ch = _chunks(png)
    assert ch[0][0] == b"IHDR" and ch[-1] == (b"IEND", b"")
    w, h, depth, ctype = struct.unpack(">IIBB", ch[0][1][:10])
    assert (w, h, depth) == (rgba.shape[1], rgba.shape[0], 8)
    idat = [d for t, d in ch if t == b"IDAT"]
    assert all(len(d) == 32768 for d in idat[:-1]) and 0 < len(idat[-1]) <= 32768
    opaque, rows = oracle.go_png_rows(rgba)
    assert ctype == (2 if opaque else 6)
    assert zlib.decompress(b"".join(idat)) == rows
    im = np.asarray(Image.open(io.BytesIO(png)))
    if opaque:
        assert np.array_equal(im, rgba[..., :3])
    else:
        nz = rgba[..., 3] > 0
        assert np.array_equal(im[..., 3], rgba[..., 3])
        assert np.array_equal(im[nz & (rgba[..., 3] == 255)], rgba[nz & (rgba[..., 3] == 255)])
    return opaque


def test_png_of_rendered_tiles(gpu, oracle):
    """Palette tiles of a C2 batch, mixed sizes (transparent pixels where no
    granule or the palette's 0xFF index: RGBA; the opaque RGB case is
    test_png_nrgba_conversion_and_filters' tile 1)."""
    import gsky_amd
    from gsky_amd.encode import encode_png
    cfg = synth.config_c2(scale=0.1, tiles_per_side=3, tile_px=200)
    cfg.tiles = [(bb, w - 17 * (i % 3), h - 9 * (i % 2)) for i, (bb, w, h) in enumerate(cfg.tiles)]
    b = gpu_batch(cfg, gpu)
    rgba = b.render(gsky_amd.ScaleParams(*cfg.scale), gsky_amd.Palette(cfg.palette, True))
    sizes = [(w, h) for (_, w, h) in cfg.tiles]
    pngs = encode_png(rgba, sizes)
    host = rgba.cpu().numpy()
    kinds = set()
    for t, (w, h) in enumerate(sizes):
        kinds.add(_check(pngs[t], np.ascontiguousarray(host[t, :h, :w]), oracle))
    assert False in kinds


def test_png_nrgba_conversion_and_filters(gpu, oracle):
    """Every filter type on synthetic RGBA, alpha < 255 with colour > alpha
    (Go's un-premultiplication wraps in uint8), alpha 0 with colour bytes."""
    import torch

    from gsky_amd.encode import encode_png
    rng = np.random.default_rng(5)
    h, w = 67, 131
    t0 = rng.integers(0, 256, (h, w, 4), dtype=np.uint8)                       # noise: None / Sub rows
    gy, gx = np.mgrid[0:h, 0:w]
    t1 = np.stack([(gx * 3) % 256, (gy * 5) % 256, (gx + gy) % 256, np.full((h, w), 255)], -1).astype(np.uint8)
    t2 = t1.copy()
    t2[..., 3] = np.where((gx // 8 + gy // 8) % 3 == 0, 0, np.where((gx + gy) % 5 == 0, 77, 255))
    t3 = np.repeat(np.repeat(rng.integers(0, 256, (h // 4 + 1, w // 4 + 1, 4), dtype=np.uint8), 4, 0), 4, 1)[:h, :w]
    tiles = np.stack([t0, t1, t2, t3])
    pngs = encode_png(torch.from_numpy(tiles).to(gpu))
    fts = set()
    for t in range(4):
        assert _check(pngs[t], tiles[t], oracle) == (t == 1)
        _, rows = oracle.go_png_rows(tiles[t])
        n = len(rows) // h
        fts |= {rows[y * n] for y in range(h)}
    assert len(fts) >= 4, fts
