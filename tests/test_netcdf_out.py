"""The WCS netCDF output (gskyhip_encode_netcdf[_host], nc4write.cpp):
EncodeGdalOpen / EncodeGdal for format "netcdf" with COMPRESS=DEFLATE,
ZLEVEL=6 (utils/ogc_encoders.go:263-301).  No netCDF or HDF5 library is in
the image, so GDAL's own file cannot be compared byte for byte (parity
unpinned): the files are read back through the product's independent
reader (hdf5.cpp + ingest.hip, itself checked against scipy-written classic
files and the spec-restated writer of tests/h5write.py) -- samples bit-exact
per band and dtype, geotransform, nodata, SRS (EPSG from spatial_ref and the
CF grid mapping alone) -- and checked structurally: HDF5 signature and
superblock checksum, the NC4C marker, the global Conventions, one row per
deflated chunk, and the zlib level of the chunks."""
import struct
import zlib

import numpy as np
import pytest

from gsky_amd import encode, ingest
from gsky_amd._lib import GskyError

from .h5write import lookup3


def _write(tmp_path, name, data_bytes):
    p = str(tmp_path / name)
    with open(p, "wb") as f:
        f.write(data_bytes)
    return p


def _bands(dt, n=2, h=37, w=53, seed=3):
    rng = np.random.default_rng(seed)
    if np.dtype(dt).kind == "f":
        return [rng.normal(size=(h, w)).astype(dt) * 100 for _ in range(n)]
    info = np.iinfo(dt)
    return [rng.integers(info.min, info.max, size=(h, w), endpoint=True).astype(dt) for _ in range(n)]


@pytest.mark.parametrize("dt", [np.uint8, np.int8, np.int16, np.uint16, np.float32])
def test_netcdf_roundtrip_dtypes(tmp_path, dt):
    bands = _bands(dt)
    gt = [1400000.0, 25.0, 0.0, -3800000.0, 0.0, -25.0]
    nd = [float(np.asarray(bands[0]).ravel()[7]), 0.0]
    blob = encode.encode_netcdf_host(bands, gt, 3577, nodata=nd, names=["ls8", "qa"], zlevel=6)
    p = _write(tmp_path, "cov.nc", blob)
    for k, b in enumerate(bands):
        vp = "NETCDF:%s:Band%d" % (p, k + 1)
        inf = ingest.info(vp)
        assert (inf.xsize, inf.ysize) == (b.shape[1], b.shape[0])
        assert np.allclose(inf.geot, gt, rtol=0, atol=1e-9)
        got = ingest.read_host(vp, 1)
        want = b.astype(np.int32) if dt == np.uint16 else b   # UInt16 widens to NC_INT in the classic model
        if dt == np.uint16:
            assert got.dtype.itemsize == 4 or got.dtype == np.float32
            assert np.array_equal(got.astype(np.int64), want.astype(np.int64))
        else:
            # NC_BYTE reads back as Byte under the driver's rules (ingest.hip:
            # netcdfdataset.cpp:386-559): the same bits
            assert got.dtype.itemsize == np.dtype(dt).itemsize
            assert np.array_equal(got.view(np.uint8), np.ascontiguousarray(want).view(np.uint8))
        exp_nd = np.asarray(nd[k], dt).astype(np.float64) if dt != np.float32 else float(np.float32(nd[k]))
        assert inf.nodata == pytest.approx(float(exp_nd))
        assert ingest.netcdf_srs(vp, 0) == "EPSG:3577"


@pytest.mark.parametrize("epsg,gt,cf", [
    (4326, [112.0, 0.01, 0.0, -10.0, 0.0, -0.01], "+proj=longlat"),
    (3857, [15028131.0, 611.5, 0.0, -1000000.0, 0.0, -611.5], None),
    (3577, [1400000.0, 25.0, 0.0, -3800000.0, 0.0, -25.0], "+proj=aea"),
    (28355, [250000.0, 25.0, 0.0, 5900000.0, 0.0, -25.0], "+proj=utm +zone=55 +south"),
    (3112, [-2000000.0, 1000.0, 0.0, -1000000.0, 0.0, -1000.0], "+proj=lcc"),
    (3031, [-3000000.0, 1000.0, 0.0, 3000000.0, 0.0, -1000.0], "+proj=stere"),
])
def test_netcdf_srs_and_grid(tmp_path, epsg, gt, cf):
    """The SRS reads back as its EPSG code (spatial_ref) and, from the CF grid
    mapping alone (srs_cf), as the same projection; the geotransform from
    the bottom-up coordinate variables equals the coverage's."""
    b = _bands(np.float32, n=1, h=20, w=30)
    p = _write(tmp_path, "c.nc", encode.encode_netcdf_host(b, gt, epsg, nodata=[-9999.0], names=["v"]))
    inf = ingest.info(p)
    assert np.allclose(inf.geot, gt, rtol=1e-12, atol=1e-9 * max(abs(g) for g in gt))
    assert ingest.netcdf_srs(p, 0) == "EPSG:%d" % epsg
    cfs = ingest.netcdf_srs(p, 1)
    if cf is None:
        assert cfs in ("?", "")    # CF "mercator": outside the warp's CF families (the EPSG route serves it)
    elif epsg == 4326:
        assert cfs.startswith("+proj=longlat") or cfs == "EPSG:4326"
    else:
        assert cfs.startswith(cf), cfs
    assert np.array_equal(ingest.read_host(p, 1), b[0])


def test_netcdf_structure(tmp_path):
    """HDF5 signature and superblock-2 checksum, netCDF-4 classic marker and
    CF conventions, one deflated chunk per row at the requested level."""
    h, w = 16, 40
    b = [np.arange(h * w, dtype=np.int16).reshape(h, w)]
    blob = encode.encode_netcdf_host(b, [0.0, 1.0, 0.0, 16.0, 0.0, -1.0], 4326, nodata=[-1.0], names=["v"],
                                     zlevel=6)
    assert blob[:8] == b"\x89HDF\r\n\x1a\n" and blob[8] == 2
    assert struct.unpack("<I", blob[44:48])[0] == lookup3(blob[:44])
    assert struct.unpack("<Q", blob[28:36])[0] == len(blob)   # end-of-file address
    for s in (b"_nc3_strict", b"Conventions", b"CF-1.5", b"DIMENSION_LIST", b"_Netcdf4Dimid", b"grid_mapping",
              b"spatial_ref", b"GeoTransform", b"Band1", b"lat", b"lon"):
        assert s in blob, s
    # each row a zlib stream at level 6 (FLEVEL bits of the header: 2 = default), shuffled int16
    n_streams, at = 0, 0
    while True:
        at = blob.find(b"\x78\x9c", at)
        if at < 0:
            break
        try:
            d = zlib.decompressobj()
            raw = d.decompress(blob[at:at + 4 * w + 64])
            if len(raw) == 2 * w:
                n_streams += 1
        except zlib.error:
            pass
        at += 2
    assert n_streams == h


def test_netcdf_empty_tile_and_errors(tmp_path):
    """An "EmptyTile" band is skipped as EncodeGdal skips it (no _FillValue,
    no long_name, zero samples); bad arguments are errors, not crashes."""
    b = _bands(np.int16, n=2, h=8, w=8)
    p = _write(tmp_path, "e.nc", encode.encode_netcdf_host(b, [0, 1, 0, 8, 0, -1], 4326, nodata=[-5.0, -6.0],
                                                            names=["ok", "EmptyTile_1"]))
    inf = ingest.info("NETCDF:%s:Band2" % p)
    assert np.array_equal(ingest.read_host("NETCDF:%s:Band2" % p, 1), np.zeros((8, 8), np.int16))
    assert ingest.info("NETCDF:%s:Band1" % p).nodata == -5.0
    assert inf.nodata is None or inf.nodata != -6.0
    with pytest.raises(GskyError):
        encode.encode_netcdf_host(b, [0, 1, 0, 8, 0, -1], 4326, zlevel=12)


@pytest.mark.gpu
def test_netcdf_from_hbm_matches_host_path(tmp_path, gpu):
    """gskyhip_encode_netcdf from HBM bands writes the same file as the host
    path, and it reads back bit-exact (a WCS coverage canvas shape)."""
    import torch
    b = _bands(np.float32, n=2, h=300, w=257)
    dev = [torch.from_numpy(x).to(gpu) for x in b]
    gt = [112.0, 0.01, 0.0, -10.0, 0.0, -0.01]
    blob_d = encode.encode_netcdf(dev, gt, 4326, nodata=[-9999.0, -9999.0], names=["a", "b"])
    blob_h = encode.encode_netcdf_host(b, gt, 4326, nodata=[-9999.0, -9999.0], names=["a", "b"])
    assert blob_d == blob_h
    p = _write(tmp_path, "d.nc", blob_d)
    for k in range(2):
        assert np.array_equal(ingest.read_host("NETCDF:%s:Band%d" % (p, k + 1), 1), b[k])
