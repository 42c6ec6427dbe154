"""Extract the 500 WMS GetMap requests of the reference's acceptance test
(acceptance_tests/acpt_url.tpl of chuc92man/gsky: EPSG:3857 bbox, width,
height; 179 distinct 256x256 tiles at zooms 6-9 over Australia) into
tests/golden/acpt_bboxes.json as [[minx, miny, maxx, maxy, width, height],
...] in file order.  Data only; run in the build container:

    python tests/golden/make_acpt_bboxes.py [/root/reference]
"""
import json
import os
import re
import sys

HERE = os.path.dirname(os.path.abspath(__file__))


def main():
    ref = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
    out = []
    for line in open(os.path.join(ref, "acceptance_tests", "acpt_url.tpl")):
        if "bbox=" not in line:
            continue
        bb = [float(v) for v in re.search(r"bbox=([^&\s]*)", line).group(1).split("%%2C")]
        w = int(re.search(r"width=(\d+)", line).group(1))
        h = int(re.search(r"height=(\d+)", line).group(1))
        out.append(bb + [w, h])
    json.dump(out, open(os.path.join(HERE, "acpt_bboxes.json"), "w"))
    print("%d requests" % len(out))


if __name__ == "__main__":
    main()
