"""CPU tests of the C-ABI library: it loads, exports every symbol the header
declares, and its host-side parts (SRS parsing, palette, FNV) agree with the
oracle.  No kernel is launched here."""
import ctypes
import os
import re

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _header_functions():
    src = open(os.path.join(ROOT, "include", "gskyhip.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = re.findall(r"^\s*(?:const\s+)?[a-z_0-9]+\s*\*?\s*([a-z_0-9]+)\s*\(", src, flags=re.M)
    return sorted(set(n for n in names if n not in ("if", "return")))


@pytest.fixture(scope="module")
def L():
    from gsky_amd import _lib
    return _lib.lib()


def test_header_exports(L):
    from gsky_amd import _lib
    fns = _header_functions()
    assert "warp_operation_fast" in fns and "gskyhip_render_tiles" in fns
    assert sorted(_lib.EXPORTS) == fns
    for f in fns:
        assert hasattr(L, f), f


def test_version(L):
    assert b"gfx950" in L.gskyhip_version()


def test_struct_sizes():
    from gsky_amd import _lib
    # layouts must match include/gskyhip.h (checked by a C compile below)
    assert ctypes.sizeof(_lib.Granule) % 8 == 0
    assert ctypes.sizeof(_lib.Tile) == 64


def test_crs_parsing_matches_oracle(L, oracle):
    from gsky_amd import _lib
    wkt_3857 = ('PROJCS["WGS 84 / Pseudo-Mercator",GEOGCS["WGS 84",DATUM["WGS_1984",SPHEROID["WGS 84",6378137,'
                '298.257223563,AUTHORITY["EPSG","7030"]],AUTHORITY["EPSG","6326"]],PRIMEM["Greenwich",0],'
                'UNIT["degree",0.0174532925199433],AUTHORITY["EPSG","4326"]],PROJECTION["Mercator_1SP"],'
                'PARAMETER["scale_factor",1],UNIT["metre",1],AUTHORITY["EPSG","3857"]]')
    cases = [("EPSG:4326", "EPSG:4326"), ("EPSG:3857", "EPSG:3857"), ("EPSG:3577", "EPSG:3577"),
             ("MODIS", "MODIS"), (wkt_3857, "EPSG:3857"),
             ("+proj=aea +lat_1=-18 +lat_2=-36 +lat_0=0 +lon_0=132 +x_0=0 +y_0=0 +ellps=GRS80", "EPSG:3577"),
             ("+proj=sinu +lon_0=0 +x_0=0 +y_0=0 +R=6371007.181 +units=m", "MODIS")]
    for spec, ref in cases:
        c = _lib.Crs()
        assert L.gskyhip_crs_from_srs(spec.encode(), ctypes.byref(c)) == 0, spec
        o = oracle.crs(ref)
        for f in ("kind", "a", "es", "lam0", "phi1", "phi2", "n", "c", "dd", "rho0", "ec"):
            assert getattr(c, f) == getattr(o, f), (spec, f)
    c = _lib.Crs()
    assert L.gskyhip_crs_from_srs(b"EPSG:9999", ctypes.byref(c)) == -4


def test_palette_matches_oracle(L, oracle):
    import gsky_amd
    rng = np.random.default_rng(1)
    for n in (2, 3, 4, 9, 256, 300):
        cols = rng.integers(0, 256, (n, 4)).astype(np.uint8)
        for interp in (True, False):
            if interp and n > 257:   # sectionLength 0: the reference panics (palette.go:12)
                with pytest.raises(Exception):
                    gsky_amd.gradient_rgba_palette(gsky_amd.Palette(cols.tolist(), interp))
                with pytest.raises(ValueError):
                    oracle.gradient_palette(cols, interp)
                continue
            got = gsky_amd.gradient_rgba_palette(gsky_amd.Palette(cols.tolist(), interp))
            assert np.array_equal(got, oracle.gradient_palette(cols, interp))


def test_fnv_matches_oracle(L, oracle):
    for s in ["", "a", "POLYGON ((1 2,3 4))", "MODIS h25v08" * 10]:
        b = s.encode()
        assert L.gskyhip_fnv32a(b, len(b)) == oracle.fnv32a(s)


def test_header_compiles_as_c(tmp_path):
    src = tmp_path / "t.c"
    src.write_text('#include "gskyhip.h"\n#include <stddef.h>\n'
                   '_Static_assert(sizeof(gskyhip_tile) == 64, "tile");\n'
                   '_Static_assert(offsetof(gskyhip_granule, geot) == 24, "geot");\n'
                   'int main(void){return 0;}\n')
    import subprocess
    subprocess.check_call(["gcc", "-std=c11", "-I", os.path.join(ROOT, "include"), "-c", str(src), "-o",
                           str(tmp_path / "t.o")])
