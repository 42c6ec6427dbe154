// drill_geom.cpp -- the drill request geometry -> window + ALL_TOUCHED mask
// (worker/gdalprocess/drill.go:363-423 getDrillFileDescriptor, 275-327
// createMask) for a batch of polygons against one dataset, host side of
// gskyhip_drill_descriptors (include/gskyhip.h).
//
// The reference goes through OGR/GEOS/GDAL:
//   OGR_G_Buffer(g, 0, 30)        taken as the identity: for a valid simple
//                                 polygon GEOS buffer(0) keeps the vertex set
//                                 (ring start / orientation may change, which
//                                 the rasterizer below does not depend on,
//                                 except for edges lying exactly on a pixel-
//                                 centre line);
//   OGR_G_Transform WGS84 -> SRS  the same PROJ formulas the warp uses
//                                 (gsky_device.h crs_forward), traditional
//                                 lon/lat order (drill.go:376);
//   envelopePolygon               the file corners through the geotransform,
//                                 printed with Go "%f" (6 decimals) into WKT;
//   OGR_G_Intersection + envelope the envelope of polygon n file envelope:
//                                 vertices inside, edge/side crossings and
//                                 file corners inside the polygon;
//   GDALRasterizeGeometries       GDAL 3.0.1 alg/llrasterize.cpp with
//     ALL_TOUCHED=TRUE            ALL_TOUCHED: GDALdllImageLineAllTouched over
//                                 every ring, then GDALdllImageFilledPolygon
//                                 (pixel-centre scanlines, even-odd), burn 255.
// Parity is pinned to oracle/ (an independent C restatement), not to a
// running GDAL (absent here).
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include <hip/hip_runtime.h>

#include "../../include/gskyhip.h"
#include "gsky_device.h"

namespace gsky {
namespace {

struct Rings {
  std::vector<double> x, y;
  std::vector<int> part;   // points per ring
};

// ---------------------------------------------------------------- GeoJSON
struct Parser {
  const char *p;
  bool ok = true;
  void ws() {
    while (*p == ' ' || *p == '\n' || *p == '\t' || *p == '\r') p++;
  }
  // nested coordinate arrays; rings start at `ring_depth`
  void coords(int depth, int ring_depth, Rings &r) {
    ws();
    if (*p != '[') { ok = false; return; }
    p++;
    if (depth == ring_depth) r.part.push_back(0);
    if (depth == ring_depth + 1) {   // [x, y(, z)]
      double v[2];
      for (int k = 0; k < 2; k++) {
        ws();
        char *e;
        v[k] = std::strtod(p, &e);
        if (e == p) { ok = false; return; }
        p = e;
        ws();
        if (k == 0) {
          if (*p != ',') { ok = false; return; }
          p++;
        }
      }
      while (*p == ',') {   // z ignored
        p++;
        char *e;
        std::strtod(p, &e);
        if (e == p) { ok = false; return; }
        p = e;
        ws();
      }
      if (*p != ']') { ok = false; return; }
      p++;
      r.x.push_back(v[0]);
      r.y.push_back(v[1]);
      r.part.back()++;
      return;
    }
    ws();
    if (*p == ']') { p++; return; }
    for (;;) {
      coords(depth + 1, ring_depth, r);
      if (!ok) return;
      ws();
      if (*p == ',') { p++; continue; }
      if (*p == ']') { p++; return; }
      ok = false;
      return;
    }
  }
};

// The geometry of a GeoJSON Feature (drill.go:35-42 re-marshals feat.Geometry)
// or a bare Polygon / MultiPolygon.
bool parse_geometry(const char *js, Rings &r) {
  if (!js) return false;
  const char *g = std::strstr(js, "\"geometry\"");
  const char *base = g ? g : js;
  const bool multi = std::strstr(base, "\"MultiPolygon\"") != nullptr;
  if (!multi && !std::strstr(base, "\"Polygon\"")) return false;
  const char *c = std::strstr(base, "\"coordinates\"");
  if (!c || !(c = std::strchr(c, ':'))) return false;
  Parser ps{c + 1};
  ps.coords(0, multi ? 2 : 1, r);
  return ps.ok && !r.part.empty();
}

bool inside_rings(const Rings &r, double px, double py) {   // even-odd over every ring
  bool in = false;
  size_t off = 0;
  for (int n : r.part) {
    for (int i = 0, j = n - 1; i < n; j = i++) {
      const double xi = r.x[off + i], yi = r.y[off + i], xj = r.x[off + j], yj = r.y[off + j];
      if ((yi > py) != (yj > py) && px < (xj - xi) * (py - yi) / (yj - yi) + xi) in = !in;
    }
    off += n;
  }
  return in;
}

// Envelope of the polygon intersected with [x0,x1] x [y0,y1]; false if empty.
bool clip_envelope(const Rings &r, double x0, double y0, double x1, double y1, double env[4]) {
  double mnx = HUGE_VAL, mny = HUGE_VAL, mxx = -HUGE_VAL, mxy = -HUGE_VAL;
  bool any = false;
  auto add = [&](double px, double py) {
    any = true;
    mnx = std::min(mnx, px); mxx = std::max(mxx, px);
    mny = std::min(mny, py); mxy = std::max(mxy, py);
  };
  size_t off = 0;
  for (int n : r.part) {
    for (int i = 0; i < n; i++) {
      const double ax = r.x[off + i], ay = r.y[off + i];
      if (ax >= x0 && ax <= x1 && ay >= y0 && ay <= y1) add(ax, ay);
      const int j = (i + 1) % n;
      const double bx = r.x[off + j], by = r.y[off + j];
      for (double X : {x0, x1})   // crossings of the vertical sides
        if ((ax - X) * (bx - X) <= 0 && ax != bx) {
          const double y = ay + (X - ax) * (by - ay) / (bx - ax);
          if (y >= y0 && y <= y1) add(X, y);
        }
      for (double Y : {y0, y1})   // crossings of the horizontal sides
        if ((ay - Y) * (by - Y) <= 0 && ay != by) {
          const double x = ax + (Y - ay) * (bx - ax) / (by - ay);
          if (x >= x0 && x <= x1) add(x, Y);
        }
    }
    off += n;
  }
  const double cx[4] = {x0, x1, x1, x0}, cy[4] = {y0, y0, y1, y1};
  for (int k = 0; k < 4; k++)
    if (inside_rings(r, cx[k], cy[k])) add(cx[k], cy[k]);
  if (!any) return false;
  env[0] = mnx; env[1] = mny; env[2] = mxx; env[3] = mxy;
  return true;
}

double go_f6(double v) {   // fmt.Sprintf("%f") parsed back by OGR
  char buf[64];
  std::snprintf(buf, sizeof(buf), "%.6f", v);
  return std::strtod(buf, nullptr);
}

// ---------------------------------------------------------------- rasterizer
struct Canvas {
  uint8_t *m;
  int w, h;
  void point(int x, int y) const {
    if (x >= 0 && x < w && y >= 0 && y < h) m[(int64_t)y * w + x] = 255;
  }
  void span(int y, int xs, int xe) const {   // gvBurnScanline
    if (xs > xe) return;
    xs = std::max(xs, 0);
    xe = std::min(xe, w - 1);
    for (int x = xs; x <= xe; x++) point(x, y);
  }
};

// GDALdllImageFilledPolygon (GDAL 3.0.1).
void fill_polygon(const Rings &r, const Canvas &cv) {
  const int n = (int)r.x.size();
  if (r.part.empty() || n == 0) return;
  double dminy = r.y[0], dmaxy = r.y[0];
  for (int i = 1; i < n; i++) { dminy = std::min(dminy, r.y[i]); dmaxy = std::max(dmaxy, r.y[i]); }
  const int miny = std::max((int)dminy, 0), maxy = std::min((int)dmaxy, cv.h - 1);
  const int minx = 0, maxx = cv.w - 1;
  std::vector<int> ints;
  for (int y = miny; y <= maxy; y++) {
    ints.clear();
    const double dy = y + 0.5;
    int partoffset = 0, part = 0;
    for (int i = 0; i < n; i++) {
      if (i == partoffset + r.part[part]) { partoffset += r.part[part]; part++; }
      const int ind1 = (i == partoffset) ? partoffset + r.part[part] - 1 : i - 1;
      const int ind2 = (i == partoffset) ? partoffset : i;
      double dy1 = r.y[ind1], dy2 = r.y[ind2], dx1, dx2;
      if ((dy1 < dy && dy2 < dy) || (dy1 > dy && dy2 > dy)) continue;
      if (dy1 < dy2) {
        dx1 = r.x[ind1]; dx2 = r.x[ind2];
      } else if (dy1 > dy2) {
        std::swap(dy1, dy2);
        dx1 = r.x[ind2]; dx2 = r.x[ind1];
      } else {   // horizontal: bottom edges filled on their own, top edges skipped
        if (r.x[ind1] > r.x[ind2]) {
          const int h1 = (int)std::floor(r.x[ind2] + 0.5), h2 = (int)std::floor(r.x[ind1] + 0.5);
          if (h1 > maxx || h2 <= minx) continue;
          cv.span(y, h1, h2 - 1);
        }
        continue;
      }
      if (dy < dy2 && dy >= dy1) ints.push_back((int)std::floor((dy - dy1) * (dx2 - dx1) / (dy2 - dy1) + dx1 + 0.5));
    }
    std::sort(ints.begin(), ints.end());
    for (size_t i = 0; i + 1 < ints.size(); i += 2)
      if (ints[i] <= maxx && ints[i + 1] > minx) cv.span(y, ints[i], ints[i + 1] - 1);
  }
}

// GDALdllImageLineAllTouched (GDAL 3.0.1), burn value only.
void touch_lines(const Rings &r, const Canvas &cv) {
  const int w = cv.w, h = cv.h;
  size_t n0 = 0;
  for (int np : r.part) {
    for (int j = 1; j < np; j++) {
      double x = r.x[n0 + j - 1], y = r.y[n0 + j - 1], xe = r.x[n0 + j], ye = r.y[n0 + j];
      if ((y < 0.0 && ye < 0.0) || (y > h && ye > h) || (x < 0.0 && xe < 0.0) || (x > w && xe > w)) continue;
      if (x > xe) { std::swap(x, xe); std::swap(y, ye); }
      if (std::floor(x) == std::floor(xe) || std::fabs(x - xe) < .01) {   // vertical
        if (ye < y) std::swap(y, ye);
        const int ix = (int)std::floor(xe);
        if (ix < 0 || ix >= w) continue;
        const int iy0 = std::max((int)std::floor(y), 0), iy1 = std::min((int)std::floor(ye), h - 1);
        for (int iy = iy0; iy <= iy1; iy++) cv.point(ix, iy);
        continue;
      }
      if (std::floor(y) == std::floor(ye) || std::fabs(y - ye) < .01) {   // horizontal
        const int iy = (int)std::floor(y);
        if (iy < 0 || iy >= h) continue;
        const int ix0 = std::max((int)std::floor(x), 0), ix1 = std::min((int)std::floor(xe), w - 1);
        for (int ix = ix0; ix <= ix1; ix++) cv.point(ix, iy);
        continue;
      }
      const double slope = (ye - y) / (xe - x);   // general, left to right
      if (xe > w) { ye -= (xe - w) * slope; xe = w; }
      if (x < 0.0) { y += (0.0 - x) * slope; x = 0.0; }
      if (ye > y) {
        if (y < 0.0) { x += (0.0 - y) / slope; y = 0.0; }
        if (ye >= h) { xe += (ye - h) / slope; ye = h; }
      } else {
        if (y >= h) { x += (h - y) / slope; y = h; }
        if (ye < 0.0) { xe -= (ye - 0) / slope; ye = 0.0; }
      }
      while (x >= 0.0 && x < xe) {
        const int ix = (int)std::floor(x), iy = (int)std::floor(y);
        if (iy >= 0 && iy < h) cv.point(ix, iy);
        double sx = std::floor(x + 1.0) - x;
        double sy = sx * slope;
        if ((int)std::floor(y + sy) == iy) {
          x += sx; y += sy;
        } else if (slope < 0) {
          sy = iy - y;
          if (sy > -0.000000001) sy = -0.000000001;
          sx = sy / slope;
          x += sx; y += sy;
        } else {
          sy = (iy + 1) - y;
          if (sy < 0.000000001) sy = 0.000000001;
          sx = sy / slope;
          x += sx; y += sy;
        }
      }
    }
    n0 += np;
  }
}

struct Descriptor {
  int32_t win[4] = {0, 0, 0, 0};
  int status = 0;
  Rings pix;   // rings in the window's pixel space (mask rasterization)
};

// getDrillFileDescriptor (drill.go:363-423) up to the mask's pixel rings.
Descriptor describe(const char *geometry, const gskyhip_crs *crs, const double gt[6], int xsize, int ysize) {
  Descriptor d;
  Rings r;
  if (!parse_geometry(geometry, r)) { d.status = GSKYHIP_E_ARG; return d; }
  if (crs) {   // WGS84 lon/lat -> dataset SRS, the warp's transform (identity for the same CRS)
    gskyhip_crs wgs;
    gskyhip_crs_from_srs("EPSG:4326", &wgs);
    if (!crs_same(wgs, *crs))
      for (size_t i = 0; i < r.x.size(); i++) {
        double lam, phi, X, Y;
        if (!crs_inverse(wgs, r.x[i], r.y[i], lam, phi) || !crs_forward(*crs, lam, phi, X, Y)) {
          d.status = GSKYHIP_E_CRS;
          return d;
        }
        r.x[i] = X;
        r.y[i] = Y;
      }
  }
  const double ulX = go_f6(gt[0] + 0 * gt[1] + 0 * gt[2]), ulY = go_f6(gt[3] + 0 * gt[4] + 0 * gt[5]);
  const double lrX = go_f6(gt[0] + xsize * gt[1] + ysize * gt[2]);
  const double lrY = go_f6(gt[3] + xsize * gt[4] + ysize * gt[5]);
  double env[4];
  if (!clip_envelope(r, std::min(ulX, lrX), std::min(ulY, lrY), std::max(ulX, lrX), std::max(ulY, lrY), env)) {
    d.status = GSKYHIP_E_RANGE;   // the polygon misses the file
    return d;
  }
  double igt[6];
  inv_geot(gt, igt);
  const double omx = igt[0] + env[0] * igt[1] + env[1] * igt[2], omy = igt[3] + env[0] * igt[4] + env[1] * igt[5];
  const double oMx = igt[0] + env[2] * igt[1] + env[3] * igt[2], oMy = igt[3] + env[2] * igt[4] + env[3] * igt[5];
  int32_t offX = go_cvtt32(std::fmin(omx, oMx)), offY = go_cvtt32(std::fmin(omy, oMy));
  int32_t cX = go_cvtt32(std::fmax(omx, oMx)) - offX, cY = go_cvtt32(std::fmax(omy, oMy)) - offY;
  if (cX == 0) cX++;
  if (cY == 0) cY++;
  if (offX < 0) offX = 0;
  if (offY < 0) offY = 0;
  d.win[0] = offX; d.win[1] = offY; d.win[2] = cX; d.win[3] = cY;
  if (cX <= 0 || cY <= 0) { d.status = GSKYHIP_E_RANGE; return d; }
  // createMask (drill.go:294-308): the MEM raster's geotransform is the
  // dataset's shifted by the window offset (rotation terms kept as they are)
  double mgt[6], migt[6];
  std::memcpy(mgt, gt, sizeof(mgt));
  mgt[0] += mgt[1] * (double)offX;
  mgt[3] += mgt[5] * (double)offY;
  inv_geot(mgt, migt);
  d.pix = std::move(r);
  for (size_t i = 0; i < d.pix.x.size(); i++) {
    const double X = d.pix.x[i], Y = d.pix.y[i];
    d.pix.x[i] = migt[0] + X * migt[1] + Y * migt[2];
    d.pix.y[i] = migt[3] + X * migt[4] + Y * migt[5];
  }
  return d;
}

// ---------------------------------------------------------------- GPU rasterizer
// The same two passes on the GPU, one workgroup per polygon, straight into
// the device mask buffer (no host mask, no copy): touch_edge_kernel gives each
// thread one edge of the rings (GDALdllImageLineAllTouched, the expressions of
// touch_lines()), fill_rows_kernel one scanline (GDALdllImageFilledPolygon,
// the expressions of fill_polygon(): intersections collected, insertion-
// sorted, spans burned).  Both only ever write 255, so the thread order and
// overlapping writes do not matter; the region is zeroed first.  Polygons
// with more than kMaxInts edges (more intersections than a thread keeps) are
// rasterized on the host instead.
constexpr int kMaxInts = 64;

struct PolyDev {
  int64_t mask_off;
  int32_t w, h;
  int32_t v0, nv;      // vertex range in vx / vy
  int32_t p0, np;      // ring range in parts (points per ring)
};

__device__ __forceinline__ void dpoint(uint8_t *m, int w, int h, int x, int y) {
  if (x >= 0 && x < w && y >= 0 && y < h) m[(int64_t)y * w + x] = 255;
}

__global__ __launch_bounds__(256) void touch_edge_kernel(const PolyDev *polys, const double *vx, const double *vy,
                                                         const int32_t *parts, uint8_t *masks) {
  const PolyDev P = polys[blockIdx.x];
  uint8_t *m = masks + P.mask_off;
  const int w = P.w, h = P.h;
  for (int k = threadIdx.x; k < P.nv; k += blockDim.x) {
    // edge (k-1, k) of its ring; the first point of a ring starts no edge
    int start = 0, r = 0;
    while (r < P.np && k >= start + parts[P.p0 + r]) { start += parts[P.p0 + r]; r++; }
    if (r >= P.np || k == start) continue;
    double x = vx[P.v0 + k - 1], y = vy[P.v0 + k - 1], xe = vx[P.v0 + k], ye = vy[P.v0 + k];
    if ((y < 0.0 && ye < 0.0) || (y > h && ye > h) || (x < 0.0 && xe < 0.0) || (x > w && xe > w)) continue;
    if (x > xe) { double t = x; x = xe; xe = t; t = y; y = ye; ye = t; }
    if (floor(x) == floor(xe) || fabs(x - xe) < .01) {   // vertical
      if (ye < y) { const double t = y; y = ye; ye = t; }
      const int ix = (int)floor(xe);
      if (ix < 0 || ix >= w) continue;
      const int iy0 = max((int)floor(y), 0), iy1 = min((int)floor(ye), h - 1);
      for (int iy = iy0; iy <= iy1; iy++) dpoint(m, w, h, ix, iy);
      continue;
    }
    if (floor(y) == floor(ye) || fabs(y - ye) < .01) {   // horizontal
      const int iy = (int)floor(y);
      if (iy < 0 || iy >= h) continue;
      const int ix0 = max((int)floor(x), 0), ix1 = min((int)floor(xe), w - 1);
      for (int ix = ix0; ix <= ix1; ix++) dpoint(m, w, h, ix, iy);
      continue;
    }
    const double slope = (ye - y) / (xe - x);   // general, left to right
    if (xe > w) { ye -= (xe - w) * slope; xe = w; }
    if (x < 0.0) { y += (0.0 - x) * slope; x = 0.0; }
    if (ye > y) {
      if (y < 0.0) { x += (0.0 - y) / slope; y = 0.0; }
      if (ye >= h) { xe += (ye - h) / slope; ye = h; }
    } else {
      if (y >= h) { x += (h - y) / slope; y = h; }
      if (ye < 0.0) { xe -= (ye - 0) / slope; ye = 0.0; }
    }
    while (x >= 0.0 && x < xe) {
      const int ix = (int)floor(x), iy = (int)floor(y);
      if (iy >= 0 && iy < h) dpoint(m, w, h, ix, iy);
      double sx = floor(x + 1.0) - x;
      double sy = sx * slope;
      if ((int)floor(y + sy) == iy) {
        x += sx; y += sy;
      } else if (slope < 0) {
        sy = iy - y;
        if (sy > -0.000000001) sy = -0.000000001;
        sx = sy / slope;
        x += sx; y += sy;
      } else {
        sy = (iy + 1) - y;
        if (sy < 0.000000001) sy = 0.000000001;
        sx = sy / slope;
        x += sx; y += sy;
      }
    }
  }
}

__global__ __launch_bounds__(256) void fill_rows_kernel(const PolyDev *polys, const double *vx, const double *vy,
                                                        const int32_t *parts, uint8_t *masks) {
  const PolyDev P = polys[blockIdx.x];
  uint8_t *m = masks + P.mask_off;
  const int w = P.w, h = P.h, n = P.nv;
  if (P.np <= 0 || n == 0) return;
  const double *X = vx + P.v0, *Y = vy + P.v0;
  const int32_t *part = parts + P.p0;
  double dminy = Y[0], dmaxy = Y[0];
  for (int i = 1; i < n; i++) { dminy = fmin(dminy, Y[i]); dmaxy = fmax(dmaxy, Y[i]); }
  const int miny = max((int)dminy, 0), maxy = min((int)dmaxy, h - 1);
  const int minx = 0, maxx = w - 1;
  int ints[kMaxInts];
  for (int y = miny + (int)threadIdx.x; y <= maxy; y += blockDim.x) {
    int ni = 0;
    const double dy = y + 0.5;
    int partoffset = 0, pi = 0;
    for (int i = 0; i < n; i++) {
      if (i == partoffset + part[pi]) { partoffset += part[pi]; pi++; }
      const int ind1 = (i == partoffset) ? partoffset + part[pi] - 1 : i - 1;
      const int ind2 = (i == partoffset) ? partoffset : i;
      double dy1 = Y[ind1], dy2 = Y[ind2], dx1, dx2;
      if ((dy1 < dy && dy2 < dy) || (dy1 > dy && dy2 > dy)) continue;
      if (dy1 < dy2) {
        dx1 = X[ind1]; dx2 = X[ind2];
      } else if (dy1 > dy2) {
        const double t = dy1; dy1 = dy2; dy2 = t;
        dx1 = X[ind2]; dx2 = X[ind1];
      } else {   // horizontal: bottom edges filled on their own, top edges skipped
        if (X[ind1] > X[ind2]) {
          const int h1 = (int)floor(X[ind2] + 0.5), h2 = (int)floor(X[ind1] + 0.5);
          if (h1 > maxx || h2 <= minx) continue;
          for (int xx = max(h1, 0); xx <= min(h2 - 1, w - 1); xx++) dpoint(m, w, h, xx, y);
        }
        continue;
      }
      if (dy < dy2 && dy >= dy1 && ni < kMaxInts)
        ints[ni++] = (int)floor((dy - dy1) * (dx2 - dx1) / (dy2 - dy1) + dx1 + 0.5);
    }
    for (int a = 1; a < ni; a++) {   // insertion sort (a few intersections per row)
      const int v = ints[a];
      int b = a - 1;
      while (b >= 0 && ints[b] > v) { ints[b + 1] = ints[b]; b--; }
      ints[b + 1] = v;
    }
    for (int i = 0; i + 1 < ni; i += 2)
      if (ints[i] <= maxx && ints[i + 1] > minx)
        for (int xx = max(ints[i], 0); xx <= min(ints[i + 1] - 1, w - 1); xx++) dpoint(m, w, h, xx, y);
  }
}

}  // namespace
}  // namespace gsky

using namespace gsky;

// Windows on the host, ALL_TOUCHED masks rasterized on the GPU into masks_dev.
extern "C" int gskyhip_drill_descriptors_device(const char *const *geometries, int n, const char *dataset_srs,
                                                const double *geot, int xsize, int ysize, int32_t *win_out,
                                                int64_t *mask_off_out, int64_t *mask_bytes_out, uint8_t *masks_dev,
                                                int32_t *status_out, void *stream) {
  if (n < 0 || !geot || !win_out || !mask_off_out || !mask_bytes_out || !status_out) return GSKYHIP_E_ARG;
  gskyhip_crs crs;
  const gskyhip_crs *pc = nullptr;
  if (dataset_srs && *dataset_srs) {
    if (gskyhip_crs_from_srs(dataset_srs, &crs)) return GSKYHIP_E_CRS;
    pc = &crs;
  }
  std::vector<PolyDev> polys;
  std::vector<double> vx, vy;
  std::vector<int32_t> parts;
  std::vector<std::pair<int64_t, std::vector<uint8_t>>> host_masks;   // polygons too complex for a thread
  int64_t off = 0;
  for (int i = 0; i < n; i++) {
    Descriptor d = describe(geometries[i], pc, geot, xsize, ysize);
    status_out[i] = d.status;
    const int64_t bytes = d.status == 0 ? (int64_t)d.win[2] * d.win[3] : 0;
    for (int k = 0; k < 4; k++) win_out[4 * i + k] = d.status == 0 ? d.win[k] : 0;
    mask_off_out[i] = off;
    if (masks_dev && bytes > 0) {
      if ((int)d.pix.x.size() > kMaxInts) {
        std::vector<uint8_t> hm((size_t)bytes, 0);
        Canvas cv{hm.data(), d.win[2], d.win[3]};
        touch_lines(d.pix, cv);
        fill_polygon(d.pix, cv);
        host_masks.emplace_back(off, std::move(hm));
      } else {
        PolyDev P;
        P.mask_off = off;
        P.w = d.win[2];
        P.h = d.win[3];
        P.v0 = (int32_t)vx.size();
        P.nv = (int32_t)d.pix.x.size();
        P.p0 = (int32_t)parts.size();
        P.np = (int32_t)d.pix.part.size();
        vx.insert(vx.end(), d.pix.x.begin(), d.pix.x.end());
        vy.insert(vy.end(), d.pix.y.begin(), d.pix.y.end());
        parts.insert(parts.end(), d.pix.part.begin(), d.pix.part.end());
        polys.push_back(P);
      }
    }
    off += (bytes + 15) / 16 * 16;   // 16-byte aligned regions, polygon order
  }
  *mask_bytes_out = off > 0 ? off : 16;
  if (!masks_dev) return 0;
  hipStream_t s = (hipStream_t)stream;
  if (hipMemsetAsync(masks_dev, 0, (size_t)*mask_bytes_out, s) != hipSuccess) return GSKYHIP_E_HIP;
  if (!polys.empty()) {
    // one staging allocation: polygons | x | y | parts
    const size_t b0 = polys.size() * sizeof(PolyDev), b1 = vx.size() * 8, b2 = parts.size() * 4;
    char *dev = nullptr;
    if (hipMalloc(&dev, b0 + 2 * b1 + b2) != hipSuccess) return GSKYHIP_E_HIP;
    std::vector<char> host(b0 + 2 * b1 + b2);
    std::memcpy(host.data(), polys.data(), b0);
    std::memcpy(host.data() + b0, vx.data(), b1);
    std::memcpy(host.data() + b0 + b1, vy.data(), b1);
    std::memcpy(host.data() + b0 + 2 * b1, parts.data(), b2);
    int rc = 0;
    if (hipMemcpyAsync(dev, host.data(), host.size(), hipMemcpyHostToDevice, s) != hipSuccess) rc = GSKYHIP_E_HIP;
    const PolyDev *dp = (const PolyDev *)dev;
    const double *dx = (const double *)(dev + b0), *dy = (const double *)(dev + b0 + b1);
    const int32_t *dpart = (const int32_t *)(dev + b0 + 2 * b1);
    if (!rc) {
      hipLaunchKernelGGL(touch_edge_kernel, dim3((unsigned)polys.size()), dim3(256), 0, s, dp, dx, dy, dpart,
                         masks_dev);
      hipLaunchKernelGGL(fill_rows_kernel, dim3((unsigned)polys.size()), dim3(256), 0, s, dp, dx, dy, dpart,
                         masks_dev);
      if (hipGetLastError() != hipSuccess) rc = GSKYHIP_E_HIP;
    }
    // the staging buffers must outlive the kernels
    if (hipStreamSynchronize(s) != hipSuccess && !rc) rc = GSKYHIP_E_HIP;
    (void)hipFree(dev);
    if (rc) return rc;
  }
  for (auto &hm : host_masks)
    if (hipMemcpy(masks_dev + hm.first, hm.second.data(), hm.second.size(), hipMemcpyHostToDevice) != hipSuccess)
      return GSKYHIP_E_HIP;
  return 0;
}

extern "C" int gskyhip_drill_descriptors(const char *const *geometries, int n, const char *dataset_srs,
                                         const double *geot, int xsize, int ysize, int32_t *win_out,
                                         int64_t *mask_off_out, int64_t *mask_bytes_out, uint8_t *masks_out,
                                         int32_t *status_out) {
  if (n < 0 || !geot || !win_out || !mask_off_out || !mask_bytes_out || !status_out) return GSKYHIP_E_ARG;
  gskyhip_crs crs;
  const gskyhip_crs *pc = nullptr;
  if (dataset_srs && *dataset_srs) {
    if (gskyhip_crs_from_srs(dataset_srs, &crs)) return GSKYHIP_E_CRS;
    pc = &crs;
  }
  int64_t off = 0;
  for (int i = 0; i < n; i++) {
    Descriptor d = describe(geometries[i], pc, geot, xsize, ysize);
    status_out[i] = d.status;
    const int64_t bytes = d.status == 0 ? (int64_t)d.win[2] * d.win[3] : 0;
    for (int k = 0; k < 4; k++) win_out[4 * i + k] = d.status == 0 ? d.win[k] : 0;
    mask_off_out[i] = off;
    if (masks_out && bytes > 0) {
      Canvas cv{masks_out + off, d.win[2], d.win[3]};
      std::memset(cv.m, 0, (size_t)bytes);
      touch_lines(d.pix, cv);    // ALL_TOUCHED: every pixel an edge passes through
      fill_polygon(d.pix, cv);   // plus every pixel centre inside
    }
    off += (bytes + 15) / 16 * 16;   // 16-byte aligned regions, polygon order
  }
  *mask_bytes_out = off > 0 ? off : 16;
  return 0;
}
