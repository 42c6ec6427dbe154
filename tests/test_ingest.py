"""Native granule ingest (gsky_amd/csrc/ingest.hip): the
GeoTIFF decoder against files written by an independent TIFF implementation
(Pillow's libtiff: every compression it writes, predictors 2 and 3, chunky
RGB) and against the layouts Pillow cannot write, made by the small TIFF
writer below (tiles with edge tiles, BigTIFF, big-endian, planar bands,
int16 / int8 / float64 samples, predictor 2 on 16-bit samples, GeoTIFF
georeferencing, GDAL_NODATA, reduced-resolution IFDs as overviews); the
netCDF classic decoder against files written by scipy.io.netcdf_file (an
independent netCDF-3 writer): variables, time bands, record dimensions,
the driver's geotransform and bottom-up rule, grid mappings.  CPU
tests decode on the host (gskyhip_geotiff_read_host, no device work); the
GPU tests decode into HBM and warp a registered file through
warp_operation_fast against the same array registered directly."""
import os
import struct
import zlib

import numpy as np
import pytest

from gsky_amd import ingest

PIL = pytest.importorskip("PIL.Image")


# ---------------------------------------------------------------- a small TIFF writer
def _packbits(b: bytes) -> bytes:
    out, i = bytearray(), 0
    while i < len(b):
        j = i
        while j + 1 < len(b) and b[j + 1] == b[i] and j - i < 127:
            j += 1
        if j > i:
            out += bytes([(257 - (j - i + 1)) & 0xFF, b[i]])
            i = j + 1
        else:
            k = i
            while k < len(b) and k - i < 128 and not (k + 1 < len(b) and b[k + 1] == b[k]):
                k += 1
            k = max(k, i + 1)
            out += bytes([k - i - 1]) + b[i:k]
            i = k
    return bytes(out)


def _predict(block: np.ndarray, predictor: int) -> np.ndarray:
    """block (rows, cols, samples) -> the bytes the predictor stores."""
    if predictor == 2:
        d = block.copy()
        d[:, 1:] = block[:, 1:] - block[:, :-1]   # wraps in the sample type
        return d
    return block


def write_tiff(path, planes, tile=None, rows_per_strip=None, compression=1, predictor=1, big=False, be=False,
               planar=2, geo=None, nodata=None, overviews=()):
    """planes: list of 2-D arrays (bands) of one dtype; overviews: list of
    lists of planes written as reduced-resolution IFDs after the first."""
    bo = ">" if be else "<"
    dt = planes[0].dtype
    fmt = {"u": 1, "i": 2, "f": 3}[dt.kind]
    out = bytearray(b"MM" if be else b"II")
    out += struct.pack(bo + "H", 43 if big else 42)
    if big:
        out += struct.pack(bo + "HHQ", 8, 0, 0)
    else:
        out += struct.pack(bo + "I", 0)
    first_ptr = 8 if big else 4
    prev_next_ptr = first_ptr
    levels = [planes] + [list(o) for o in overviews]
    for lvl, bands in enumerate(levels):
        h, w = bands[0].shape
        nb = len(bands)
        if tile:
            tw, th = tile
            across, down = -(-w // tw), -(-h // th)
        else:
            tw, th = w, rows_per_strip or h
            across, down = 1, -(-h // th)
        chunks = []
        arr = np.stack(bands, -1).astype(dt.newbyteorder(">" if be else "<"))
        groups = [[b] for b in range(nb)] if planar == 2 else [list(range(nb))]
        for grp in groups:
            for by in range(down):
                for bx in range(across):
                    if tile:
                        blk = np.zeros((th, tw, len(grp)), arr.dtype)
                        src = arr[by * th:(by + 1) * th, bx * tw:(bx + 1) * tw][..., grp]
                        blk[:src.shape[0], :src.shape[1]] = src
                    else:
                        blk = arr[by * th:(by + 1) * th][..., grp]
                    raw = _predict(blk, predictor).tobytes()
                    chunks.append(zlib.compress(raw) if compression == 8 else
                                  _packbits(raw) if compression == 32773 else raw)
        offs = []
        for c in chunks:
            offs.append(len(out))
            out += c
            if len(out) % 2:
                out += b"\0"
        ents = []   # (tag, type, values)
        ents.append((254, 4, [1 if lvl else 0]))
        ents.append((256, 4, [w]))
        ents.append((257, 4, [h]))
        ents.append((258, 3, [dt.itemsize * 8] * nb))
        ents.append((259, 3, [compression]))
        ents.append((262, 3, [1]))
        if not tile:
            ents.append((273, 16 if big else 4, offs))
        ents.append((277, 3, [nb]))
        if not tile:
            ents.append((278, 4, [th]))
            ents.append((279, 16 if big else 4, [len(c) for c in chunks]))
        ents.append((284, 3, [planar]))
        if predictor != 1:
            ents.append((317, 3, [predictor]))
        if tile:
            ents.append((322, 3, [tw]))
            ents.append((323, 3, [th]))
            ents.append((324, 16 if big else 4, offs))
            ents.append((325, 16 if big else 4, [len(c) for c in chunks]))
        ents.append((339, 3, [fmt] * nb))
        if geo and lvl == 0:
            for tag, typ, vals in geo:
                ents.append((tag, typ, vals))
        if nodata is not None and lvl == 0:
            ents.append((42113, 2, nodata))
        ents.sort()
        ifd_off = len(out)
        out[prev_next_ptr:prev_next_ptr + (8 if big else 4)] = struct.pack(bo + ("Q" if big else "I"), ifd_off)
        esz, inl = (20, 8) if big else (12, 4)
        body = bytearray(struct.pack(bo + ("Q" if big else "H"), len(ents)))
        extra = bytearray()
        extra_base = ifd_off + len(body) + esz * len(ents) + (8 if big else 4)
        tcode = {2: "s", 3: "H", 4: "I", 12: "d", 16: "Q"}
        tsize = {2: 1, 3: 2, 4: 4, 12: 8, 16: 8}
        for tag, typ, vals in ents:
            if typ == 2:
                data = vals.encode() + b"\0"
                cnt = len(data)
            else:
                data = struct.pack(bo + "%d%s" % (len(vals), tcode[typ]), *vals)
                cnt = len(vals)
            ent = struct.pack(bo + ("HHQ" if big else "HHI"), tag, typ, cnt)
            if len(data) <= inl:
                ent += data + b"\0" * (inl - len(data))
            else:
                ent += struct.pack(bo + ("Q" if big else "I"), extra_base + len(extra))
                extra += data
                if len(extra) % 2:
                    extra += b"\0"
            body += ent
        prev_next_ptr = ifd_off + len(body)
        body += b"\0" * (8 if big else 4)
        out += body + extra
    with open(path, "wb") as f:
        f.write(bytes(out))


def geokeys(model=1, raster=1, keys=()):
    """GeoKeyDirectory: (key, value) SHORT keys after GTModelType / GTRasterType."""
    ks = [(1024, model), (1025, raster)] + list(keys)
    vals = [1, 1, 0, len(ks)]
    for k, v in ks:
        vals += [k, 0, 1, v]
    return (34735, 3, vals)


# ---------------------------------------------------------------- Pillow-written files
@pytest.mark.parametrize("comp", ["raw", "tiff_deflate", "tiff_lzw", "packbits"])
@pytest.mark.parametrize("mode", ["L", "I;16", "I", "F"])
def test_pillow_compressions(tmp_path, comp, mode):
    rng = np.random.default_rng(len(comp) * 7 + len(mode))
    a = {"L": lambda: rng.integers(0, 256, (97, 131)).astype(np.uint8),
         "I;16": lambda: rng.integers(0, 65536, (97, 131)).astype(np.uint16),
         "I": lambda: rng.integers(-2**31, 2**31 - 1, (97, 131)).astype(np.int32),
         "F": lambda: rng.standard_normal((97, 131)).astype(np.float32)}[mode]()
    a[5:9, 10:50] = a[5, 10]   # runs for PackBits / LZW
    p = str(tmp_path / "a.tif")
    PIL.fromarray(a).save(p, compression=comp)
    inf = ingest.info(p)
    assert (inf.xsize, inf.ysize, inf.n_bands) == (131, 97, 1)
    assert np.array_equal(ingest.read_host(p), a)


@pytest.mark.parametrize("pred", [2, 3])
def test_pillow_float_predictors(tmp_path, pred):
    f = np.random.default_rng(pred).standard_normal((61, 203)).astype(np.float32)
    p = str(tmp_path / "f.tif")
    PIL.fromarray(f).save(p, compression="tiff_deflate", tiffinfo={317: pred})
    assert ingest.info(p).predictor == pred
    assert np.array_equal(ingest.read_host(p), f)


def test_pillow_uint16_predictor2_and_rgb(tmp_path):
    a = np.random.default_rng(5).integers(0, 65536, (40, 300)).astype(np.uint16)
    p = str(tmp_path / "u.tif")
    PIL.fromarray(a).save(p, compression="tiff_lzw", tiffinfo={317: 2})
    assert np.array_equal(ingest.read_host(p), a)
    rgb = np.random.default_rng(6).integers(0, 256, (50, 61, 3)).astype(np.uint8)
    p = str(tmp_path / "rgb.tif")
    PIL.fromarray(rgb).save(p, compression="tiff_deflate")
    inf = ingest.info(p)
    assert inf.n_bands == 3 and inf.planar == 1
    for b in range(3):
        assert np.array_equal(ingest.read_host(p, b + 1), rgb[..., b])


# ---------------------------------------------------------------- layouts Pillow cannot write
@pytest.mark.parametrize("big,be", [(False, False), (True, False), (False, True), (True, True)])
@pytest.mark.parametrize("comp,pred", [(1, 1), (8, 2), (32773, 1), (8, 1)])
def test_tiled_planar_int16(tmp_path, big, be, comp, pred):
    rng = np.random.default_rng(comp + pred + 2 * big + be)
    b1 = rng.integers(-32768, 32767, (150, 210)).astype(np.int16)
    b2 = (b1 // 3).astype(np.int16)
    p = str(tmp_path / "t.tif")
    write_tiff(p, [b1, b2], tile=(64, 48), compression=comp, predictor=pred, big=big, be=be, planar=2)
    inf = ingest.info(p)
    assert (inf.xsize, inf.ysize, inf.n_bands, inf.block) == (210, 150, 2, (64, 48))
    assert inf.dtype == 3 and not inf.signed_byte
    assert np.array_equal(ingest.read_host(p, 1), b1)
    assert np.array_equal(ingest.read_host(p, 2), b2)


@pytest.mark.parametrize("dt", [np.int8, np.uint8, np.float64, np.uint32])
def test_strips_chunky_types(tmp_path, dt):
    rng = np.random.default_rng(11)
    bands = [(rng.standard_normal((77, 45)) * 100).astype(dt) for _ in range(3)]
    p = str(tmp_path / "s.tif")
    write_tiff(p, bands, rows_per_strip=10, compression=8, planar=1)
    inf = ingest.info(p)
    assert inf.signed_byte == (dt == np.int8)
    for k in range(3):
        got = ingest.read_host(p, k + 1)
        assert np.array_equal(got.view(dt) if got.dtype != dt else got, bands[k]), k


def test_geotiff_georeferencing(tmp_path):
    """GDAL's reading of the GeoTIFF tags: tiepoint + pixel scale ->
    geotransform, PixelIsPoint shifted by half a pixel, ModelTransformation,
    EPSG from the GeoKeys (projected, geographic, MODIS sinusoidal),
    GDAL_NODATA, -1e10 when absent (warp.go:246), overview sizes."""
    a = np.arange(40 * 30, dtype=np.int16).reshape(30, 40)
    ov = [a[::2, ::2].copy()], [a[::4, ::4].copy()]
    p = str(tmp_path / "g.tif")
    geo = [(33550, 12, [25.0, 25.0, 0.0]), (33922, 12, [0.0, 0.0, 0.0, 1400000.0, -3800000.0, 0.0]),
           geokeys(1, 1, [(3072, 3577)])]
    write_tiff(p, [a], tile=(16, 16), geo=geo, nodata="-999", overviews=ov)
    inf = ingest.info(p)
    assert inf.geot == (1400000.0, 25.0, 0.0, -3800000.0, 0.0, -25.0)
    assert inf.epsg == 3577 and inf.srs == "EPSG:3577" and inf.nodata == -999.0
    assert inf.overviews == [(20, 15), (10, 8)]
    assert np.array_equal(ingest.read_host(p, 1, 1), a[::2, ::2])
    assert np.array_equal(ingest.read_host(p, 1, 2), a[::4, ::4])
    # PixelIsPoint, geographic CRS, no nodata
    p2 = str(tmp_path / "g2.tif")
    write_tiff(p2, [a], geo=[(33550, 12, [0.5, 0.5, 0.0]), (33922, 12, [0, 0, 0, 112.0, -10.0, 0]),
                             geokeys(2, 2, [(2048, 4326)])])
    inf = ingest.info(p2)
    assert inf.geot == (111.75, 0.5, 0.0, -9.75, 0.0, -0.5) and inf.epsg == 4326 and inf.nodata is None
    # ModelTransformation (rotated grid) and a user-defined sinusoidal on the MODIS sphere
    p3 = str(tmp_path / "g3.tif")
    mt = [463.3, 0.1, 0.0, -20015109.354, 0.2, -463.3, 0.0, 10007554.677, 0, 0, 0, 0, 0, 0, 0, 1]
    keys = geokeys(1, 1, [(3072, 32767), (3075, 24)])
    keys = (keys[0], keys[1], keys[2][:3] + [keys[2][3] + 1] + keys[2][4:] + [2057, 34736, 1, 0])
    write_tiff(p3, [a], geo=[(34264, 12, mt), keys, (34736, 12, [6371007.181])])
    inf = ingest.info(p3)
    assert inf.geot == (-20015109.354, 463.3, 0.1, 10007554.677, 0.2, -463.3) and inf.srs == "MODIS"


def test_missing_file_and_band(tmp_path):
    from gsky_amd import GskyError
    with pytest.raises(GskyError) as e:
        ingest.info(str(tmp_path / "none.tif"))
    assert e.value.code == 1                     # open failed (warp.go:103-110)
    p = str(tmp_path / "one.tif")
    write_tiff(p, [np.zeros((4, 4), np.uint8)])
    with pytest.raises(GskyError) as e:
        ingest.read_host(p, 2)
    assert e.value.code == 2                     # band failed (warp.go:111-118)


# ---------------------------------------------------------------- GPU: into HBM, through the drop-in
@pytest.mark.gpu
def test_gpu_read_matches_host(tmp_path):
    import torch
    rng = np.random.default_rng(3)
    a = rng.integers(-20000, 20000, (1000, 1300)).astype(np.int16)
    p = str(tmp_path / "big.tif")
    write_tiff(p, [a, (a // 2).astype(np.int16)], tile=(256, 256), compression=8, predictor=2, big=True)
    for band, exp in ((1, a), (2, a // 2)):
        got = ingest.read(p, band).cpu().numpy()
        assert got.dtype == np.int16 and np.array_equal(got, exp)
    f = rng.standard_normal((333, 517)).astype(np.float32)
    p2 = str(tmp_path / "f.tif")
    PIL.fromarray(f).save(p2, compression="tiff_lzw", tiffinfo={317: 3})
    assert np.array_equal(ingest.read(p2).cpu().numpy(), f)
    torch.cuda.synchronize()


@pytest.mark.gpu
def test_gpu_drop_in_opens_geotiff(tmp_path):
    """warp_operation_fast on an unregistered *.tif path decodes it the way
    GDALOpenEx would (warp.go:89-101) and warps it bit-identically to the
    same array registered by hand."""
    import torch

    from gsky_amd import synth, worker
    from gsky_amd.tiles import bbox_to_geot
    cfg = synth.config_c2(scale=0.05, tiles_per_side=2, tile_px=128)
    g = cfg.granules[0]
    p = str(tmp_path / "granule.tif")
    geo = [(33550, 12, [g.geot[1], -g.geot[5], 0.0]), (33922, 12, [0, 0, 0, g.geot[0], g.geot[3], 0]),
           geokeys(1, 1, [(3072, 3577)])]
    write_tiff(p, [g.data], tile=(64, 64), compression=8, predictor=2, geo=geo, nodata="%g" % g.nodata)
    worker.unregister_all()
    worker.register_granule("hand", 1, torch.from_numpy(g.data).cuda(), g.geot, "EPSG:3577", g.nodata)
    bbox, w, h = cfg.tiles[0]
    req = dict(bands=[1], width=w, height=h, dstSRS="EPSG:3857", dstGeot=bbox_to_geot(w, h, bbox))
    a = worker.warp_raster(worker.GeoRPCGranule(path="hand", **req))
    b = worker.warp_raster(worker.GeoRPCGranule(path=p, **req))
    assert a.error == "OK" and b.error == "OK", (a.error, b.error)
    assert np.array_equal(worker.raster_array(a.raster), worker.raster_array(b.raster))
    assert a.raster.bbox == b.raster.bbox and b.raster.noData == g.nodata
    assert worker.warp_raster(worker.GeoRPCGranule(path=str(tmp_path / "absent.tif"), **req)).error == \
        "warp_operation() fail: 1"
    assert worker.warp_raster(worker.GeoRPCGranule(path=p, **dict(req, bands=[2]))).error == \
        "warp_operation() fail: 2"
    worker.unregister_all()


# ---------------------------------------------------------------- netCDF classic (scipy's writer)
def _write_nc(path, var, data, x, y, xname="lon", yname="lat", fill=None, version=1, attrs=None, time=None,
              record=False):
    from scipy.io import netcdf_file
    with netcdf_file(path, "w", version=version) as f:
        if time is not None:
            f.createDimension("time", None if record else len(time))
        f.createDimension(yname, len(y))
        f.createDimension(xname, len(x))
        vx = f.createVariable(xname, "f8", (xname,))
        vx[:] = x
        vy = f.createVariable(yname, "f8", (yname,))
        vy[:] = y
        dims = ((("time",) if time is not None else ()) + (yname, xname))
        v = f.createVariable(var, data.dtype.char, dims)
        if fill is not None:
            v._FillValue = data.dtype.type(fill)
        for k, val in (attrs or {}).items():
            setattr(v, k, val)
        v[:] = data


@pytest.mark.parametrize("version", [1, 2])
@pytest.mark.parametrize("dt", [np.int16, np.float32, np.int8, np.float64, np.int32])
def test_netcdf_variable_and_geotransform(tmp_path, version, dt):
    """Latitude increasing (bottom-up): rows come back north first and the
    geotransform is the driver's (netcdfdataset.cpp:3504-3655)."""
    rng = np.random.default_rng(int(np.dtype(dt).itemsize) + version)
    ny, nx = 37, 52
    data = (rng.standard_normal((ny, nx)) * 50).astype(dt)
    lon = 112.0 + 0.25 * np.arange(nx)
    lat = -44.0 + 0.2 * np.arange(ny)      # increasing -> bBottomUp
    p = str(tmp_path / "v.nc")
    _write_nc(p, "ndvi", data, lon, lat, fill=-99, version=version)
    inf = ingest.info(p)
    assert (inf.xsize, inf.ysize, inf.n_bands) == (nx, ny, 1)
    assert inf.epsg == 4326 and inf.nodata == -99.0
    assert inf.signed_byte == (dt == np.int8)
    dx, dy = (lon[-1] - lon[0]) / (nx - 1), (lat[0] - lat[-1]) / (ny - 1)
    exp_gt = (lon[0] - dx / 2, dx, 0.0, lat[-1] - dy / 2, 0.0, dy)
    assert np.allclose(inf.geot, exp_gt, rtol=0, atol=1e-12)
    got = ingest.read_host(p)
    assert np.array_equal(got.view(dt) if got.dtype != dt else got, data[::-1])
    assert np.array_equal(ingest.read_host("NETCDF:%s:ndvi" % p).view(got.dtype), got)


@pytest.mark.parametrize("record", [False, True])
def test_netcdf_time_bands(tmp_path, record):
    """3-D (time, y, x): band_query = the time index (warp.go:89-101); y
    decreasing keeps file row order; a record (unlimited) time dimension
    interleaves the bands with the other record variables."""
    rng = np.random.default_rng(9)
    nt, ny, nx = 5, 20, 30
    data = rng.integers(-1000, 1000, (nt, ny, nx)).astype(np.int16)
    lat = 10.0 - 0.5 * np.arange(ny)
    p = str(tmp_path / "t.nc")
    _write_nc(p, "sm", data, np.arange(nx) * 1.0, lat, time=np.arange(nt), record=record)
    inf = ingest.info(p)
    # no _FillValue / missing_value: the driver's NCDFGetDefaultNoDataValue
    # (netcdfdataset.cpp:420-430, 10182-10225), NC_FILL_SHORT for a short
    assert inf.n_bands == nt and inf.nodata == -32767.0
    for b in range(nt):
        assert np.array_equal(ingest.read_host(p, b + 1), data[b]), b
    from gsky_amd import GskyError
    with pytest.raises(GskyError):
        ingest.read_host(p, nt + 1)


def test_netcdf_projected_grid_mapping(tmp_path):
    from scipy.io import netcdf_file
    p = str(tmp_path / "albers.nc")
    data = np.arange(12 * 9, dtype=np.float32).reshape(12, 9)
    x = 1400012.5 + 25.0 * np.arange(9)
    y = -3800012.5 - 25.0 * np.arange(12)
    with netcdf_file(p, "w") as f:
        f.createDimension("y", 12)
        f.createDimension("x", 9)
        f.createVariable("x", "f8", ("x",))[:] = x
        f.createVariable("y", "f8", ("y",))[:] = y
        crs = f.createVariable("crs", "i", ())
        crs.spatial_ref = 'PROJCS["GDA94 / Australian Albers",AUTHORITY["EPSG","3577"]]'
        v = f.createVariable("band", "f", ("y", "x"))
        v.grid_mapping = "crs"
        v[:] = data
    inf = ingest.info(p)
    assert inf.epsg == 3577 and inf.geot == (1400000.0, 25.0, 0.0, -3800000.0, 0.0, -25.0)
    assert np.array_equal(ingest.read_host("NETCDF:%s:band" % p), data)


def _write_albers_nc(path, data, x, y, wkt=None, cf=None):
    """A projected netCDF grid whose grid mapping carries a GDAL WKT
    (spatial_ref) and / or CF grid-mapping attributes."""
    from scipy.io import netcdf_file
    ny, nx = data.shape
    with netcdf_file(path, "w") as f:
        f.createDimension("y", ny)
        f.createDimension("x", nx)
        f.createVariable("x", "f8", ("x",))[:] = x
        f.createVariable("y", "f8", ("y",))[:] = y
        crs = f.createVariable("crs", "i", ())
        if wkt:
            crs.spatial_ref = wkt
        for k, val in (cf or {}).items():
            setattr(crs, k, val)
        v = f.createVariable("band", data.dtype.char, ("y", "x"))
        v.grid_mapping = "crs"
        v._FillValue = data.dtype.type(-999)
        v[:] = data


ALBERS_CF = {"grid_mapping_name": "albers_conical_equal_area", "standard_parallel": np.array([-18.0, -36.0]),
             "longitude_of_central_meridian": np.array([132.0]), "latitude_of_projection_origin": np.array([0.0]),
             "false_easting": np.array([0.0]), "false_northing": np.array([0.0]),
             "semi_major_axis": np.array([6378137.0]), "inverse_flattening": np.array([298.257222101])}


UTM55_CF = {"grid_mapping_name": "transverse_mercator", "scale_factor_at_central_meridian": np.array([0.9996]),
            "longitude_of_central_meridian": np.array([147.0]), "latitude_of_projection_origin": np.array([0.0]),
            "false_easting": np.array([500000.0]), "false_northing": np.array([10000000.0]),
            "semi_major_axis": np.array([6378137.0]), "inverse_flattening": np.array([298.257222101])}


GALCC_CF = {"grid_mapping_name": "lambert_conformal_conic", "standard_parallel": np.array([-18.0, -36.0]),
            "longitude_of_central_meridian": np.array([134.0]), "latitude_of_projection_origin": np.array([0.0]),
            "false_easting": np.array([0.0]), "false_northing": np.array([0.0]),
            "semi_major_axis": np.array([6378137.0]), "inverse_flattening": np.array([298.257222101])}


PSN_CF = {"grid_mapping_name": "polar_stereographic", "latitude_of_projection_origin": np.array([90.0]),
          "standard_parallel": np.array([70.0]), "straight_vertical_longitude_from_pole": np.array([-45.0]),
          "false_easting": np.array([0.0]), "false_northing": np.array([0.0]),
          "semi_major_axis": np.array([6378137.0]), "inverse_flattening": np.array([298.257223563])}


def test_netcdf_srs_cf_option(tmp_path):
    """srs_cf (warp.go:95 -> netcdfdataset.cpp:7023-7025, 3666): without it
    the GDAL WKT's EPSG code wins; with it only the CF grid mapping counts.
    No grid mapping on lon / lat axes: EPSG:4326 either way; an unsupported
    CF mapping is "?"."""
    data = np.zeros((4, 5), np.int16)
    x, y = 1400012.5 + 25.0 * np.arange(5), -3800012.5 - 25.0 * np.arange(4)
    p = str(tmp_path / "a.nc")
    wkt = 'PROJCS["GDA94 / Australian Albers",AUTHORITY["EPSG","3577"]]'
    cf = dict(ALBERS_CF, longitude_of_central_meridian=np.array([131.0]))
    _write_albers_nc(p, data, x, y, wkt=wkt, cf=cf)
    assert ingest.netcdf_srs(p, 0) == "EPSG:3577"
    got = ingest.netcdf_srs(p, 1)
    assert got.startswith("+proj=aea ") and "+lon_0=131 " in got and "+lat_1=-18 " in got and "+lat_2=-36 " in got
    assert "+a=6378137 +rf=298.25722210100002" in got
    p2 = str(tmp_path / "b.nc")
    _write_albers_nc(p2, data, x, y, cf=cf)          # CF only: both options agree
    assert ingest.netcdf_srs(p2, 0) == ingest.netcdf_srs(p2, 1) == got
    p3 = str(tmp_path / "c.nc")
    _write_albers_nc(p3, data, x, y, wkt=wkt, cf={"grid_mapping_name": "rotated_latitude_longitude"})
    assert ingest.netcdf_srs(p3, 0) == "EPSG:3577" and ingest.netcdf_srs(p3, 1) == "?"
    p4 = str(tmp_path / "d.nc")
    _write_albers_nc(p4, data, x, y, cf={"grid_mapping_name": "sinusoidal", "longitude_of_central_meridian": np.array([0.0]),
                                         "earth_radius": np.array([6371007.181])})
    s4 = ingest.netcdf_srs(p4, 1)
    assert s4.startswith("+proj=sinu +lon_0=0 +x_0=0 +y_0=0 +R=") and float(s4.split("+R=")[1]) == 6371007.181
    p5 = str(tmp_path / "e.nc")
    _write_nc(p5, "v", data, np.arange(5.0), np.arange(4.0))
    assert ingest.netcdf_srs(p5, 0) == ingest.netcdf_srs(p5, 1) == "EPSG:4326"
    # transverse_mercator: a UTM zone's parameters as +proj=utm, others as tmerc
    p6 = str(tmp_path / "f.nc")
    _write_albers_nc(p6, data, x, y, cf=UTM55_CF)
    assert ingest.netcdf_srs(p6, 1) == "+proj=utm +zone=55 +south +a=6378137 +rf=298.25722210100002"
    p7 = str(tmp_path / "g.nc")
    _write_albers_nc(p7, data, x, y, cf=dict(UTM55_CF, scale_factor_at_central_meridian=np.array([0.99994]),
                                             false_northing=np.array([5000000.0])))
    s7 = ingest.netcdf_srs(p7, 1)
    assert s7.startswith("+proj=tmerc +lat_0=0 +lon_0=147 +k_0=0.99994") and "+y_0=5000000 " in s7
    from gsky_amd.tiles import parse_crs
    assert parse_crs(s7).kind == 4 and parse_crs(ingest.netcdf_srs(p6, 1)).kind == 4
    # lambert_conformal_conic: two standard parallels (GA Lambert), or one (the tangent cone)
    p8 = str(tmp_path / "h.nc")
    _write_albers_nc(p8, data, x, y, cf=GALCC_CF)
    s8 = ingest.netcdf_srs(p8, 1)
    assert s8.startswith("+proj=lcc +lat_1=-18 +lat_2=-36 +lat_0=0 +lon_0=134 ")
    c8, e3112 = parse_crs(s8), parse_crs("EPSG:3112")
    assert c8.kind == 5 and (c8.n, c8.c, c8.rho0) == (e3112.n, e3112.c, e3112.rho0)
    p9 = str(tmp_path / "i.nc")
    _write_albers_nc(p9, data, x, y, cf=dict(GALCC_CF, standard_parallel=np.array([-30.0])))
    assert ingest.netcdf_srs(p9, 1).startswith("+proj=lcc +lat_1=-30 +lat_0=0 +lon_0=134 +k_0=1 ")
    # polar_stereographic: the polar aspects, by standard parallel or scale at the pole
    p10 = str(tmp_path / "j.nc")
    _write_albers_nc(p10, data, x, y, cf=PSN_CF)
    s10 = ingest.netcdf_srs(p10, 1)
    assert s10 == "+proj=stere +lat_0=90 +lat_ts=70 +lon_0=-45 +x_0=0 +y_0=0 +a=6378137 +rf=298.25722356300003"
    c10, e3413 = parse_crs(s10), parse_crs("EPSG:3413")
    assert c10.kind == 6 and all(getattr(c10, f) == getattr(e3413, f) for f in ("phi0", "phi1", "lam0", "c", "k0"))
    p11 = str(tmp_path / "k.nc")
    ups = {k: v for k, v in PSN_CF.items() if k != "standard_parallel"}
    ups.update(scale_factor_at_projection_origin=np.array([0.994]), straight_vertical_longitude_from_pole=np.array([0.0]),
               false_easting=np.array([2000000.0]), false_northing=np.array([2000000.0]))
    _write_albers_nc(p11, data, x, y, cf=ups)
    c11, e32661 = parse_crs(ingest.netcdf_srs(p11, 1)), parse_crs("EPSG:32661")
    assert c11.kind == 6 and all(getattr(c11, f) == getattr(e32661, f) for f in ("phi0", "phi1", "lam0", "c", "k0", "x0"))
    p12 = str(tmp_path / "l.nc")
    _write_albers_nc(p12, data, x, y, cf=dict(PSN_CF, latitude_of_projection_origin=np.array([60.0])))
    assert ingest.netcdf_srs(p12, 1) == "?"            # oblique stereographic: not carried


@pytest.mark.gpu
def test_gpu_netcdf_srs_cf_drop_in(tmp_path):
    """warp_operation_fast with srsCf: the granule whose GDAL WKT says
    EPSG:3577 but whose CF mapping has its central meridian at 131 E warps
    as EPSG:3577 without srsCf and through the CF Albers with it -- each
    bit-identical to the oracle with that SRS; an unsupported CF mapping is
    an error (GSKYHIP_E_CRS), not a silent WGS84."""
    import torch

    from gsky_amd import worker
    from gsky_amd.tiles import bbox_to_geot
    from oracle import oracle as O
    rng = np.random.default_rng(21)
    ny, nx = 300, 400
    data = rng.integers(0, 10000, (ny, nx)).astype(np.int16)
    x = 1000012.5 + 25.0 * np.arange(nx)
    y = -2500012.5 - 25.0 * np.arange(ny)
    wkt = 'PROJCS["GDA94 / Australian Albers",AUTHORITY["EPSG","3577"]]'
    p = str(tmp_path / "g.nc")
    _write_albers_nc(p, data, x, y, wkt=wkt, cf=dict(ALBERS_CF, longitude_of_central_meridian=np.array([131.99])))
    gt = (1000000.0, 25.0, 0.0, -2500000.0, 0.0, -25.0)
    g = O.make_granule(data, gt, -999.0)
    wm = O.crs("EPSG:3857")
    x0, y0 = O.crs_transform(O.crs("EPSG:3577"), wm, 1001000.0, -2507000.0)
    x1, y1 = O.crs_transform(O.crs("EPSG:3577"), wm, 1009000.0, -2501000.0)
    dgt = bbox_to_geot(256, 256, (x0, y0, x1, y1))
    worker.unregister_all()
    outs = {}
    for cf in (0, 1):
        r = worker.warp_raster(worker.GeoRPCGranule(path=p, bands=[1], width=256, height=256, dstSRS="EPSG:3857",
                                                    dstGeot=dgt, sRSCf=cf))
        assert r.error == "OK", (cf, r.error)
        src = O.crs(ingest.netcdf_srs(p, cf))
        exp, ebbox, end, edt = O.warp(g, src, wm, dgt, 256, 256)
        got = worker.raster_array(r.raster)
        assert list(r.raster.bbox) == list(ebbox), cf
        assert np.array_equal(got, exp), (cf, int((got != exp).sum()))
        outs[cf] = got
    assert not np.array_equal(outs[0], outs[1])      # the 0.01 degree meridian shift moves the picks
    p2 = str(tmp_path / "h.nc")
    _write_albers_nc(p2, data, x, y, wkt=wkt, cf={"grid_mapping_name": "rotated_latitude_longitude"})
    ok = worker.warp_raster(worker.GeoRPCGranule(path=p2, bands=[1], width=64, height=64, dstSRS="EPSG:3857",
                                                 dstGeot=dgt, sRSCf=0))
    bad = worker.warp_raster(worker.GeoRPCGranule(path=p2, bands=[1], width=64, height=64, dstSRS="EPSG:3857",
                                                  dstGeot=dgt, sRSCf=1))
    assert ok.error == "OK" and bad.error.startswith("warp_operation() fail: -"), (ok.error, bad.error)
    worker.unregister_all()
    torch.cuda.synchronize()


@pytest.mark.gpu
def test_gpu_netcdf_cf_transverse_mercator(tmp_path):
    """A netCDF granule in GDA94 / MGA zone 55 known only by its CF
    transverse_mercator grid mapping warps to EPSG:3857 bit-identically to
    the oracle through EPSG:28355."""
    import torch

    from gsky_amd import worker
    from gsky_amd.tiles import bbox_to_geot
    from oracle import oracle as O
    rng = np.random.default_rng(22)
    ny, nx = 300, 400
    data = rng.integers(0, 10000, (ny, nx)).astype(np.int16)
    x = 300012.5 + 25.0 * np.arange(nx)
    y = 5850000.0 - 12.5 - 25.0 * np.arange(ny)
    p = str(tmp_path / "utm.nc")
    _write_albers_nc(p, data, x, y, cf=UTM55_CF)
    gt = (300000.0, 25.0, 0.0, 5850000.0, 0.0, -25.0)
    g = O.make_granule(data, gt, -999.0)
    wm = O.crs("EPSG:3857")
    x0, y0 = O.crs_transform(O.crs("EPSG:28355"), wm, 301000.0, 5843000.0)
    x1, y1 = O.crs_transform(O.crs("EPSG:28355"), wm, 309000.0, 5849000.0)
    dgt = bbox_to_geot(256, 256, (x0, y0, x1, y1))
    worker.unregister_all()
    try:
        r = worker.warp_raster(worker.GeoRPCGranule(path=p, bands=[1], width=256, height=256, dstSRS="EPSG:3857",
                                                    dstGeot=dgt, sRSCf=1))
        assert r.error == "OK", r.error
        exp, ebbox, end, edt = O.warp(g, O.crs("EPSG:28355"), wm, dgt, 256, 256)
        got = worker.raster_array(r.raster)
        assert list(r.raster.bbox) == list(ebbox)
        assert np.array_equal(got, exp), int((got != exp).sum())
        assert (got != -999).mean() > 0.5
    finally:
        worker.unregister_all()
        torch.cuda.synchronize()


@pytest.mark.parametrize("dt,exp", [(np.int16, -32767.0), (np.int32, -2147483647.0),
                                    (np.float32, float(np.float32(9.9692099683868690e+36))),
                                    (np.float64, 9.9692099683868690e+36), (np.int8, 0.0)])
def test_netcdf_default_nodata(tmp_path, dt, exp):
    """A variable without _FillValue / missing_value still gets the driver's
    default fill value as its nodata (netcdfdataset.cpp:420-430, 558)."""
    p = str(tmp_path / "d.nc")
    _write_nc(p, "v", np.zeros((4, 6), dt), np.arange(6) * 1.0, -np.arange(4) * 1.0)
    assert ingest.info(p).nodata == exp


@pytest.mark.parametrize("attrs,gdal,signed,nodata", [
    ({}, False, True, -1.0),                                   # netCDF bytes are signed
    ({"_Unsigned": b"true"}, False, False, 255.0),             # _Unsigned, nodata + 256
    ({"_Unsigned": b"FALSE"}, False, True, -1.0),
    ({"valid_range": np.array([0, 255], np.int16)}, False, False, 255.0),
    ({"valid_range": np.array([-128, 127], np.int16), "_Unsigned": b"true"}, False, True, -1.0),
    ({}, True, False, 255.0),                                  # a GDAL-written file: unsigned
    ({"valid_range": np.array([-128, 127], np.int16)}, True, True, 255.0),
])
def test_netcdf_byte_signedness(tmp_path, attrs, gdal, signed, nodata):
    """NC_BYTE signedness and nodata as netCDFRasterBand decides them
    (netcdfdataset.cpp:466-541): signed unless the file was written by GDAL
    (a "GDAL" global attribute >= 1.9, 2498-2518, 8879-8919); valid_range
    {0,255} / {-128,127} decides when present, else _Unsigned; an unsigned
    band's negative nodata gets +256 (once the signedness is known -- the
    GDAL-file rule's own +256 stays when valid_range later says signed)."""
    from scipy.io import netcdf_file
    p = str(tmp_path / "b.nc")
    with netcdf_file(p, "w") as f:
        if gdal:
            f.GDAL = b"GDAL 3.0.1, released 2019/06/28"
        f.createDimension("lat", 3)
        f.createDimension("lon", 4)
        f.createVariable("lon", "f8", ("lon",))[:] = np.arange(4) * 1.0
        f.createVariable("lat", "f8", ("lat",))[:] = -np.arange(3) * 1.0
        v = f.createVariable("v", "b", ("lat", "lon"))
        v._FillValue = np.int8(-1)
        for k, val in attrs.items():
            setattr(v, k, val)
        v[:] = np.zeros((3, 4), np.int8)
    inf = ingest.info(p)
    assert inf.signed_byte == signed and inf.nodata == nodata


def _tiff_le(entries, extra=b""):
    """A minimal little-endian classic TIFF: one IFD of (tag, type, count,
    value-or-offset) entries at offset 8, then `extra`."""
    import struct
    ifd = struct.pack("<H", len(entries))
    for tag, typ, cnt, val in entries:
        ifd += struct.pack("<HHII", tag, typ, cnt, val)
    ifd += struct.pack("<I", 0)
    return b"II*\x00" + struct.pack("<I", 8) + ifd + extra


@pytest.mark.parametrize("name,entries", [
    ("count0", [(256, 3, 0, 0), (257, 3, 1, 4), (258, 3, 1, 8), (273, 4, 1, 200), (279, 4, 1, 16)]),
    ("huge_count", [(256, 3, 1, 4), (257, 3, 1, 4), (258, 3, 1, 8), (273, 4, 0x40000000, 8), (279, 4, 1, 16)]),
    ("huge_dims", [(256, 4, 1, 0xFFFFFFF0), (257, 4, 1, 0xFFFFFFF0), (258, 3, 1, 64), (273, 4, 1, 8),
                   (279, 4, 1, 16)]),
    ("huge_tile", [(256, 3, 1, 4), (257, 3, 1, 4), (258, 3, 1, 32), (322, 4, 1, 1 << 20), (323, 4, 1, 1 << 20),
                   (324, 4, 1, 8), (325, 4, 1, 16)]),
    ("offset_past_end", [(256, 3, 1, 4), (257, 3, 1, 4), (258, 3, 1, 8), (273, 4, 1, 1 << 30), (279, 4, 1, 16)]),
    ("bits_odd", [(256, 3, 1, 4), (257, 3, 1, 4), (258, 3, 1, 12), (273, 4, 1, 8), (279, 4, 1, 16)]),
])
def test_malformed_tiff_is_an_error_not_a_crash(tmp_path, name, entries):
    """Malformed headers come back as error codes through the C ABI: a tag
    with no value, counts or sizes that would overflow or exhaust memory,
    strips past the end of the file, unsupported sample sizes."""
    from gsky_amd import GskyError
    p = str(tmp_path / (name + ".tif"))
    with open(p, "wb") as f:
        f.write(_tiff_le(entries, b"\x00" * 64))
    with pytest.raises(GskyError):
        ingest.read_host(p)


@pytest.mark.gpu
def test_gpu_drop_in_unsupported_encoding_is_an_error(tmp_path):
    """A file the reader cannot decode (JPEG compression) is reported as an
    error by warp_operation_fast, not as an empty "open failed" tile; a
    missing file stays rc 1 (warp.go:103-110)."""
    from gsky_amd import worker
    from gsky_amd.tiles import bbox_to_geot
    import struct
    p = str(tmp_path / "jpeg.tif")
    geo = struct.pack("<3d", 1.0, 1.0, 0.0) + struct.pack("<6d", 0, 0, 0, 130.0, -20.0, 0)
    n_ent = 9
    data_off = 8 + 2 + 12 * n_ent + 4
    entries = [(256, 3, 1, 16), (257, 3, 1, 16), (258, 3, 1, 8), (259, 3, 1, 7), (273, 4, 1, data_off + len(geo)),
               (277, 3, 1, 1), (279, 4, 1, 256), (33550, 12, 3, data_off), (33922, 12, 6, data_off + 24)]
    with open(p, "wb") as f:
        f.write(_tiff_le(entries, geo + b"\x00" * 256))
    worker.unregister_all()
    req = dict(bands=[1], width=64, height=64, dstSRS="EPSG:4326",
               dstGeot=bbox_to_geot(64, 64, (130.0, -36.0, 146.0, -20.0)))
    r = worker.warp_raster(worker.GeoRPCGranule(path=p, **req))
    assert r.error == "warp_operation() fail: -2", r.error
    r = worker.warp_raster(worker.GeoRPCGranule(path=str(tmp_path / "none.tif"), **req))
    assert r.error == "warp_operation() fail: 1", r.error
    worker.unregister_all()


def test_truncated_netcdf_is_an_error(tmp_path):
    from gsky_amd import GskyError
    p = str(tmp_path / "ok.nc")
    _write_nc(p, "v", np.arange(24, dtype=np.int16).reshape(4, 6), np.arange(6) * 1.0, -np.arange(4) * 1.0)
    raw = open(p, "rb").read()
    for cut in (9, 40, 80, len(raw) // 2):
        q = str(tmp_path / ("cut%d.nc" % cut))
        open(q, "wb").write(raw[:cut])
        with pytest.raises(GskyError):
            ingest.read_host(q)


@pytest.mark.gpu
def test_gpu_netcdf_read_and_drop_in(tmp_path):
    """NETCDF:file:var bands decoded into HBM (byte order fixed on the GPU)
    and opened by warp_operation_fast itself: bit-identical to the same band
    registered by hand."""
    import torch

    from gsky_amd import worker
    from gsky_amd.tiles import bbox_to_geot
    rng = np.random.default_rng(4)
    nt, ny, nx = 3, 400, 600
    data = rng.integers(0, 10000, (nt, ny, nx)).astype(np.int16)
    lon = 130.0 + 0.01 * (np.arange(nx) + 0.5)
    lat = -20.0 - 0.01 * (np.arange(ny) + 0.5)
    p = str(tmp_path / "g.nc")
    _write_nc(p, "v", data, lon, lat, fill=-1, time=np.arange(nt))
    for b in range(nt):
        assert np.array_equal(ingest.read("NETCDF:%s:v" % p, b + 1).cpu().numpy(), data[b])
    inf = ingest.info(p)
    worker.unregister_all()
    worker.register_granule("hand", 2, torch.from_numpy(data[1]).cuda(), inf.geot, "EPSG:4326", -1.0)
    bbox = (14471533.8, -2504688.5, 14526000.0, -2450000.0)
    req = dict(bands=[2], width=256, height=256, dstSRS="EPSG:3857", dstGeot=bbox_to_geot(256, 256, bbox))
    a = worker.warp_raster(worker.GeoRPCGranule(path="hand", **req))
    b = worker.warp_raster(worker.GeoRPCGranule(path="NETCDF:%s:v" % p, **req))
    assert a.error == "OK" and b.error == "OK", (a.error, b.error)
    assert np.array_equal(worker.raster_array(a.raster), worker.raster_array(b.raster))
    assert a.raster.bbox == b.raster.bbox
    worker.unregister_all()
    torch.cuda.synchronize()
