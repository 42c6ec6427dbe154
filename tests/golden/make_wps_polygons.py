"""Extract the drill geometries of the reference's WPS acceptance requests
(acceptance_tests/polygon_requests/*.xml and *.payload of chuc92man/gsky:
32 Australian local-government areas plus the two sample payloads) into
tests/golden/wps_polygons.json.gz: {file name: GeoJSON text of the
wps:ComplexData geometry input}, unchanged.  Data only (the requests' inputs);
run in the build container, where /root/reference exists:

    python tests/golden/make_wps_polygons.py [/root/reference]
"""
import glob
import gzip
import json
import os
import re
import sys

HERE = os.path.dirname(os.path.abspath(__file__))


def main():
    ref = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
    out = {}
    for p in sorted(glob.glob(os.path.join(ref, "acceptance_tests", "polygon_requests", "*"))):
        txt = open(p, encoding="utf-8").read()
        m = re.search(r"<ows:Identifier>geometry</ows:Identifier>.*?<wps:ComplexData[^>]*>(.*?)</wps:ComplexData>",
                      txt, re.S)
        if not m:
            continue
        geo = m.group(1).strip()
        json.loads(geo)   # must be valid GeoJSON text
        out[os.path.basename(p)] = geo
    with gzip.open(os.path.join(HERE, "wps_polygons.json.gz"), "wt", encoding="utf-8") as f:
        json.dump(out, f)
    print("%d geometries" % len(out))


if __name__ == "__main__":
    main()
