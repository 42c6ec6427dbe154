"""OGR_G_Buffer(g, 0, 30) of the drill request geometry (drill.go:364-367):
GEOS 3.7.2's zero-distance buffer before the polygon is reprojected,
intersected with the file and rasterized ALL_TOUCHED.  GEOS is absent here,
so parity is unpinned; these tests pin the product
(gsky_amd/csrc/repair.cpp) to

* known answers: the repaired polygon rasterizes exactly like the polygon the
  buffer is known to produce, drawn explicitly -- a bow-tie keeps the lobe of
  its highest vertex's orientation (CGAlgorithms::isCCW), overlapping or
  nested polygons become their union, a hole outside its shell and a
  zero-area spike vanish, a doubly wound ring is its single ring;
* the oracle's separate restatement (oracle/gsky_oracle.c rings_buffer0) on
  random self-intersecting rings;
* the identity on valid polygons (the WPS acceptance polygons keep their
  masks, tests/test_drill_geom.py).
"""
import json

import numpy as np
import pytest

from gsky_amd import drill

GT = [0.0, 0.25, 0.0, 8.0, 0.0, -0.25]     # 32 x 32 pixels over [0, 8] x [0, 8] (lon / lat)
SIZE = 32


def poly(*rings):
    return json.dumps({"type": "Polygon", "coordinates": [[list(map(float, p)) for p in r] for r in rings]})


def multi(*polys):
    return json.dumps({"type": "MultiPolygon",
                       "coordinates": [[[list(map(float, p)) for p in r] for r in rs] for rs in polys]})


def ring(*pts):
    return list(pts) + [pts[0]]


def mask(g, oracle=None):
    win, off, buf, st = drill.drill_descriptors([g], "EPSG:4326", GT, SIZE, SIZE)
    assert st[0] == 0
    w = tuple(int(v) for v in win[0])
    m = buf[off[0]:off[0] + w[2] * w[3]].reshape(w[3], w[2])
    if oracle is not None:
        ew, em = oracle.drill_descriptor(g, "EPSG:4326", GT, SIZE, SIZE)
        assert w == ew and np.array_equal(m, em)
    full = np.zeros((SIZE, SIZE), np.uint8)
    full[w[1]:w[1] + w[3], w[0]:w[0] + w[2]] = m
    return full, w


def same_as(g, explicit, oracle):
    a, wa = mask(g, oracle)
    b, wb = mask(explicit, oracle)
    assert wa == wb and np.array_equal(a, b)
    return a


@pytest.mark.parametrize("g,kept", [
    # highest vertex (6.5, 6.5) first; its turn is clockwise -> the right lobe (clockwise) survives
    (poly(ring((1.5, 1.5), (6.5, 6.5), (6.5, 1.5), (1.5, 6.5))),
     poly(ring((4, 4), (6.5, 6.5), (6.5, 1.5)))),
    # mirrored: the highest vertex turns counter-clockwise -> the counter-clockwise (left) lobe
    (poly(ring((6.5, 1.5), (1.5, 6.5), (1.5, 1.5), (6.5, 6.5))),
     poly(ring((4, 4), (1.5, 6.5), (1.5, 1.5)))),
])
def test_bowtie_keeps_one_lobe(oracle, g, kept):
    m = same_as(g, kept, oracle)
    # as drawn, GDAL's even-odd fill would burn both lobes
    assert m[:, :12].sum() == 0 or m[:, 20:].sum() == 0


def test_union_of_overlapping_and_nested_polygons(oracle):
    a = ring((1, 1), (5, 1), (5, 5), (1, 5))
    b = ring((3, 3), (7, 3), (7, 7), (3, 7))
    union = ring((1, 1), (5, 1), (5, 3), (7, 3), (7, 7), (3, 7), (3, 5), (1, 5))
    m = same_as(multi([a], [b]), poly(union), oracle)
    assert m[(8 - 4) * 4, 4 * 4] == 255            # the overlap (4, 4) burnt (even-odd would leave it out)
    outer, inner = ring((1, 1), (7, 1), (7, 7), (1, 7)), ring((3, 3), (5, 3), (5, 5), (3, 5))
    same_as(multi([outer], [inner]), poly(outer), oracle)          # nested shells: the outer one
    same_as(multi([outer], [list(reversed(inner))]), poly(outer), oracle)


def test_hole_outside_its_shell_vanishes(oracle):
    shell, hole = ring((1, 1), (4, 1), (4, 4), (1, 4)), ring((5, 5), (7, 5), (7, 7), (5, 7))
    m = same_as(poly(shell, hole), poly(shell), oracle)
    assert m[:10, 20:].sum() == 0


def test_spike_and_double_winding(oracle):
    sq = [(1, 1), (5, 1), (5, 5), (1, 5)]
    spike = ring((1, 1), (5, 1), (5, 3), (7.3, 3), (5, 3), (5, 5), (1, 5))
    m = same_as(poly(spike), poly(ring(*sq)), oracle)
    assert m[:, 21:].sum() == 0                     # as drawn, ALL_TOUCHED would burn the spike
    twice = sq + sq + [sq[0]]
    same_as(poly(twice), poly(ring(*sq)), oracle)
    # orientation does not matter for a valid ring
    same_as(poly(ring(*reversed(sq))), poly(ring(*sq)), oracle)


def test_hole_touching_and_crossing(oracle):
    shell = ring((1, 1), (7, 1), (7, 7), (1, 7))
    # a hole crossing the shell's right side: shell minus the hole's inside part
    hole = ring((5, 3), (7.5, 3), (7.5, 5), (5, 5))
    same_as(poly(shell, hole), poly(ring((1, 1), (7, 1), (7, 3), (5, 3), (5, 5), (7, 5), (7, 7), (1, 7))), oracle)


def test_empty_buffer_keeps_the_rings_as_drawn(oracle):
    flat = poly(ring((1, 1), (6, 6), (1, 1.0), (6, 6)))      # zero area: GEOS returns empty, the clone is used
    m, _ = mask(flat, oracle)
    assert m.sum() > 0                               # the line is still burnt ALL_TOUCHED


def test_random_self_intersecting_rings_match_oracle(oracle):
    rng = np.random.default_rng(3)
    geoms = []
    for k in range(60):
        n = int(rng.integers(4, 14))
        pts = [(float(x), float(y)) for x, y in rng.uniform(0.3, 7.7, (n, 2))]
        rs = [ring(*pts)]
        if k % 3 == 0:
            rs.append(ring(*[(float(x), float(y)) for x, y in rng.uniform(0.3, 7.7, (5, 2))]))
        geoms.append(poly(*rs) if k % 2 else multi(rs[:1], *([rs[1:]] if len(rs) > 1 else [])))
    win, off, buf, st = drill.drill_descriptors(geoms, "EPSG:4326", GT, SIZE, SIZE)
    for i, g in enumerate(geoms):
        ew, em = oracle.drill_descriptor(g, "EPSG:4326", GT, SIZE, SIZE)
        assert st[i] == 0 and tuple(win[i]) == ew, i
        assert np.array_equal(buf[off[i]:off[i] + ew[2] * ew[3]].reshape(ew[3], ew[2]), em), i


@pytest.mark.gpu
def test_repaired_masks_on_gpu(oracle):
    """The GPU rasterizer burns the repaired rings: the same masks as the host
    call and the oracle."""
    import torch
    rng = np.random.default_rng(4)
    geoms = [poly(ring((1.5, 1.5), (6.5, 6.5), (6.5, 1.5), (1.5, 6.5))),
             multi([ring((1, 1), (5, 1), (5, 5), (1, 5))], [ring((3, 3), (7, 3), (7, 7), (3, 7))]),
             poly(ring((1, 1), (5, 1), (5, 3), (7.3, 3), (5, 3), (5, 5), (1, 5)))]
    for k in range(40):
        geoms.append(poly(ring(*[(float(x), float(y)) for x, y in rng.uniform(0.3, 7.7, (int(rng.integers(4, 12)), 2))])))
    win, off, buf, st = drill.drill_descriptors(geoms, "EPSG:4326", GT, SIZE, SIZE)
    mb, st2 = drill.drill_dataset(geoms, "EPSG:4326", GT, SIZE, SIZE, device="cuda", rasterize="gpu")
    torch.cuda.synchronize()
    assert np.array_equal(st, st2) and np.array_equal(mb.win.cpu().numpy(), win)
    gm = mb.masks.cpu().numpy()
    assert np.array_equal(gm, buf)
    for i, g in enumerate(geoms):
        ew, em = oracle.drill_descriptor(g, "EPSG:4326", GT, SIZE, SIZE)
        assert np.array_equal(gm[off[i]:off[i] + ew[2] * ew[3]].reshape(ew[3], ew[2]), em), i


def test_degenerate_lattice_rings_match_oracle(oracle):
    """Rings on a half-unit lattice -- collinear overlaps, vertices on edges,
    many edges through one node, segments crossing several collinear copies
    -- and wide sets (ray casts turned across the short side): the product's
    noding, depths and ring chaining agree with the oracle's exactly."""
    rng = np.random.default_rng(12)
    geoms = []
    for k in range(80):
        n = int(rng.integers(4, 70))
        pts = np.round(rng.uniform(0.3, 7.7, (n, 2)) * 2) / 2
        if k % 3 == 0:
            pts[:, 1] = pts[:, 1] * 0.3 + 3
        geoms.append(poly(ring(*[(float(x), float(y)) for x, y in pts])))
    win, off, buf, st = drill.drill_descriptors(geoms, "EPSG:4326", GT, SIZE, SIZE)
    for i, g in enumerate(geoms):
        ew, em = oracle.drill_descriptor(g, "EPSG:4326", GT, SIZE, SIZE)
        assert st[i] == 0 and tuple(win[i]) == ew, i
        assert np.array_equal(buf[off[i]:off[i] + ew[2] * ew[3]].reshape(ew[3], ew[2]), em), i


def test_zigzag_self_crossing_is_fast_and_matches_oracle(oracle):
    """A ring of 1,500 teeth crossed by its own return stroke (~3,000
    crossings, every edge spanning the whole height): noded and cast in well
    under a second, equal to the oracle."""
    import time
    n = 1500
    pts = [(0.3 + 7.4 * i / n, 3.0 + (1.0 if i % 2 else 0.0)) for i in range(n)]
    pts += [(0.3 + 7.4 * (i + 0.5) / n, 3.0 + (0.0 if i % 2 else 1.0)) for i in reversed(range(n))]
    g = poly(ring(*pts))
    t = time.time()
    win, off, buf, st = drill.drill_descriptors([g], "EPSG:4326", GT, SIZE, SIZE)
    assert time.time() - t < 1.0 and st[0] == 0
    ew, em = oracle.drill_descriptor(g, "EPSG:4326", GT, SIZE, SIZE)
    assert tuple(win[0]) == ew and np.array_equal(buf[off[0]:off[0] + ew[2] * ew[3]].reshape(ew[3], ew[2]), em)
