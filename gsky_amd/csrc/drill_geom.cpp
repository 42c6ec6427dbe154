// drill_geom.cpp -- the drill request geometry -> window + ALL_TOUCHED mask
// (worker/gdalprocess/drill.go:363-423 getDrillFileDescriptor, 275-327
// createMask) for a batch of polygons against one dataset, host side of
// gskyhip_drill_descriptors (include/gskyhip.h).
//
// The reference goes through OGR/GEOS/GDAL:
//   OGR_G_Buffer(g, 0, 30)        GEOS 3.7.2's zero-distance buffer
//                                 (repair.cpp): a valid polygon keeps its
//                                 vertices (rings turned interior-right);
//                                 self-intersecting, multiply-wound,
//                                 overlapping or inside-out rings become the
//                                 region of depth >= 1;
//   OGR_G_Transform WGS84 -> SRS  the same PROJ formulas the warp uses
//                                 (gsky_device.h crs_forward), traditional
//                                 lon/lat order (drill.go:376);
//   envelopePolygon               the file corners through the geotransform,
//                                 printed with Go "%f" (6 decimals) into WKT;
//   OGR_G_Intersection + envelope the envelope of polygon n file envelope:
//                                 vertices inside, edge/side crossings and
//                                 file corners inside the polygon;
//   GDALRasterizeGeometries       GDAL 3.0.1 alg/llrasterize.cpp (MIT
//     ALL_TOUCHED=TRUE            licence, (c) Frank Warmerdam and GDAL
//                                 contributors): ALL_TOUCHED burns every pixel
//                                 GDALdllImageLineAllTouched steps through on
//                                 every ring (its DDA expressions are restated
//                                 in touch_edge(), bit-exactness needs them),
//                                 then GDALdllImageFilledPolygon's pixel-centre
//                                 scanline fill, burn 255.
// The scanline fill is NOT GDAL's per-row sort of intersections: every edge
// computes GDAL's intersection abscissa on each pixel-centre line it crosses
// (the same expression and half-open rule) and toggles one bit of a per-row
// parity bitmap; a pixel is inside iff an odd number of intersections lie at
// or left of it, which is exactly what burning the spans between sorted
// intersection pairs gives (rings are closed, so every line crosses an even
// number of edges).  This is edge-parallel with no bound on vertices or
// intersections per row, and the same functions run on the host
// (gskyhip_drill_descriptors) and on the GPU (..._device).  Parity is pinned
// to oracle/ (a separate C restatement that sorts intersections the way GDAL
// does), not to a running GDAL (absent here).
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include <hip/hip_runtime.h>
#include <unistd.h>

#include "../../include/gskyhip.h"
#include "gsky_device.h"
#include "repair.h"

namespace gsky {
namespace {

struct Rings {
  std::vector<double> x, y;
  std::vector<int> part;   // points per ring
  std::vector<int> poly;   // polygon of each ring (its first ring is the shell)
};

// ---------------------------------------------------------------- GeoJSON
// A decimal number, correctly rounded to double (what strtod returns) for
// up to 19 significant digits and a decimal exponent in [-19, 19]; false (the
// caller uses strtod) otherwise.  GeoJSON coordinates are 15-18 digit
// decimals, where glibc's strtod takes its multi-precision path.
//
// m * 10^-k (k > 0): the 64-bit normalized m times a 128-bit truncated
// reciprocal R_k = floor(2^(127+b_k) / 10^k) in [2^127, 2^128) gives the
// quotient's leading 128 bits to within 2 units of the last; the 53-bit
// rounding is decided from them unless the bits below the mantissa sit
// within that error of the halfway point, which goes to an exact 128-bit
// division.  m * 10^k (k >= 0) is an exact 128-bit product.
struct Recip {
  uint64_t hi[20], lo[20];
  int b[20];
  Recip() {
    uint64_t p = 1;
    for (int k = 1; k < 20; k++) {
      p *= 10;   // 10^k < 2^64
      int bk = 0;
      while (bk < 64 && (((unsigned __int128)1 << bk) < p)) bk++;
      b[k] = bk;
      // floor(2^(127+bk) / p) by shift-subtract over the numerator's bits
      unsigned __int128 q = 0, rem = 0;
      for (int bit = 127 + bk; bit >= 0; bit--) {
        rem = (rem << 1) | (bit == 127 + bk ? 1u : 0u);
        q <<= 1;
        if (rem >= p) { rem -= p; q |= 1; }
      }
      hi[k] = (uint64_t)(q >> 64);
      lo[k] = (uint64_t)q;
    }
  }
};
const Recip &recip() {
  static const Recip r;
  return r;
}

inline double from_mant(uint64_t mant, int e) {   // mant in [2^52, 2^53], value mant * 2^e, normal range
  if (mant >> 53) { mant >>= 1; e++; }
  const uint64_t bits = ((uint64_t)(e + 52 + 1023) << 52) | (mant & ((1ull << 52) - 1));
  double v;
  std::memcpy(&v, &bits, 8);
  return v;
}

// exact m / 10^k by one 128-bit division (the rare near-halfway case)
double div_exact(uint64_t m, uint64_t den) {
  unsigned __int128 num = m;
  const int lz = 64 + __builtin_clzll(m);
  const int sh = lz - 1;
  num <<= sh;
  const unsigned __int128 q = num / den, r = num % den;
  const int qlz = (q >> 64) ? __builtin_clzll((uint64_t)(q >> 64)) : 64 + __builtin_clzll((uint64_t)q);
  const int drop = (128 - qlz) - 53;
  unsigned __int128 mant = q >> drop;
  const unsigned __int128 rem = q & (((unsigned __int128)1 << drop) - 1), half = (unsigned __int128)1 << (drop - 1);
  if (rem > half || (rem == half && (r != 0 || (mant & 1)))) mant++;   // round half to even, r: sticky
  return std::ldexp((double)(uint64_t)mant, drop - sh);
}

bool fast_decimal(const char *p, const char **end, double *out) {
  const char *s = p;
  bool neg = false;
  if (*s == '-' || *s == '+') { neg = *s == '-'; s++; }
  uint64_t m = 0;
  int nd = 0, dexp = 0;
  bool lost = false;   // a nonzero digit past the 19th
  const char *d0 = s;
  while (*s >= '0' && *s <= '9') {
    if (nd < 19) { m = m * 10 + (uint64_t)(*s - '0'); if (m) nd++; }
    else { dexp++; lost |= *s != '0'; }
    s++;
  }
  const char *digits_end = s;
  if (*s == '.') {
    s++;
    while (*s >= '0' && *s <= '9') {
      if (nd < 19) { m = m * 10 + (uint64_t)(*s - '0'); if (m) nd++; dexp--; }
      else lost |= *s != '0';
      s++;
    }
  }
  if (digits_end == d0 && s == d0 + 1) return false;   // "." alone
  if (s == d0) return false;
  if (*s == 'e' || *s == 'E') {
    const char *e = s + 1;
    bool en = false;
    if (*e == '-' || *e == '+') { en = *e == '-'; e++; }
    if (!(*e >= '0' && *e <= '9')) return false;
    int ev = 0;
    while (*e >= '0' && *e <= '9') { if (ev < 10000) ev = ev * 10 + (*e - '0'); e++; }
    dexp += en ? -ev : ev;
    s = e;
  }
  if (lost || dexp < -19 || dexp > 19) return false;
  *end = s;
  if (m == 0) { *out = neg ? -0.0 : 0.0; return true; }
  static const uint64_t p10[20] = {1ull, 10ull, 100ull, 1000ull, 10000ull, 100000ull, 1000000ull, 10000000ull,
                                   100000000ull, 1000000000ull, 10000000000ull, 100000000000ull, 1000000000000ull,
                                   10000000000000ull, 100000000000000ull, 1000000000000000ull,
                                   10000000000000000ull, 100000000000000000ull, 1000000000000000000ull,
                                   10000000000000000000ull};
  double v;
  if (dexp >= 0) {   // exact integer m * 10^dexp < 2^128
    const unsigned __int128 num = (unsigned __int128)m * p10[dexp];
    const uint64_t nh = (uint64_t)(num >> 64);
    const int lz = nh ? __builtin_clzll(nh) : 64 + __builtin_clzll((uint64_t)num);
    const int drop = 128 - lz - 53;
    if (drop <= 0) {
      v = (double)(uint64_t)num;   // < 2^53: exact
    } else {
      uint64_t mant = (uint64_t)(num >> drop);
      const unsigned __int128 rem = num & (((unsigned __int128)1 << drop) - 1), half = (unsigned __int128)1 << (drop - 1);
      if (rem > half || (rem == half && (mant & 1))) mant++;
      v = from_mant(mant, drop);
    }
  } else {
    const int k = -dexp;
    const Recip &R = recip();
    const int lz = __builtin_clzll(m);
    const uint64_t M = m << lz;
    const unsigned __int128 ph = (unsigned __int128)M * R.hi[k], pl = (unsigned __int128)M * R.lo[k];
    const unsigned __int128 mid = (ph & 0xFFFFFFFFFFFFFFFFull) + (pl >> 64);
    const uint64_t U = (uint64_t)mid;
    const uint64_t T = (uint64_t)(ph >> 64) + (uint64_t)(mid >> 64);
    const int drop = 11 - __builtin_clzll(T);   // 11 or 10: T's top bit is 63 or 62
    const uint64_t half = 1ull << (drop - 1), rT = T & ((1ull << drop) - 1);
    uint64_t mant = T >> drop;
    // the exact product exceeds (T, U) by less than 2 units of U
    if ((rT == half && U < 4) || (rT == half - 1 && U >= ~3ull)) {
      v = div_exact(m, p10[k]);
    } else {
      if (rT >= half) mant++;
      v = from_mant(mant, drop + 1 - lz - R.b[k]);
    }
  }
  *out = neg ? -v : v;
  return true;
}

double parse_number(const char *p, char **end) {
  double v;
  const char *e;
  if (fast_decimal(p, &e, &v)) { *end = (char *)e; return v; }
  return std::strtod(p, end);
}

struct Parser {
  const char *p;
  bool ok = true;
  int npoly = 0;
  void ws() {
    while (*p == ' ' || *p == '\n' || *p == '\t' || *p == '\r') p++;
  }
  // nested coordinate arrays; rings start at `ring_depth`
  void coords(int depth, int ring_depth, Rings &r) {
    ws();
    if (*p != '[') { ok = false; return; }
    p++;
    if (depth == ring_depth - 1) npoly++;
    if (depth == ring_depth) {
      r.part.push_back(0);
      r.poly.push_back(npoly);
    }
    if (depth == ring_depth + 1) {   // [x, y(, z)]
      double v[2];
      for (int k = 0; k < 2; k++) {
        ws();
        char *e;
        v[k] = parse_number(p, &e);
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
        parse_number(p, &e);
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
  // the geometry's "type" value (one short scan: it precedes the coordinates
  // in every GeoJSON writer); anything else -> a search of the whole text
  int kind = -1;   // 1 MultiPolygon, 0 Polygon
  if (const char *t = std::strstr(base, "\"type\"")) {
    t += 6;
    while (*t == ' ' || *t == '\n' || *t == '\t' || *t == '\r') t++;
    if (*t == ':') {
      t++;
      while (*t == ' ' || *t == '\n' || *t == '\t' || *t == '\r') t++;
      if (std::strncmp(t, "\"MultiPolygon\"", 14) == 0) kind = 1;
      else if (std::strncmp(t, "\"Polygon\"", 9) == 0) kind = 0;
    }
  }
  if (kind < 0) {
    kind = std::strstr(base, "\"MultiPolygon\"") != nullptr ? 1 : 0;
    if (!kind && !std::strstr(base, "\"Polygon\"")) return false;
  }
  const bool multi = kind == 1;
  const char *c = std::strstr(base, "\"coordinates\"");
  if (!c || !(c = std::strchr(c, ':'))) return false;
  Parser ps{c + 1};
  const size_t guess = std::strlen(c) / 24 + 4;   // ~2 numbers of ~12+ characters per vertex
  r.x.reserve(guess);
  r.y.reserve(guess);
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
// Per-polygon rasterization state: the window canvas and its parity bitmap
// (one bit per pixel of the rows [miny, maxy] of GDALdllImageFilledPolygon).
struct RasterJob {
  uint8_t *m;          // mask, h rows x w bytes
  uint32_t *bits;      // parity bitmap, (maxy - miny + 1) rows x wpr words
  int32_t w, h;
  int32_t miny, maxy;  // scanline range of the fill (clamped to the canvas)
  int32_t wpr;         // words per bitmap row
};

__host__ __device__ inline void burn(const RasterJob &J, int x, int y) {
  if (x >= 0 && x < J.w && y >= 0 && y < J.h) J.m[(int64_t)y * J.w + x] = 255;
}

__host__ __device__ inline void toggle(const RasterJob &J, int y, int x) {
  uint32_t *word = J.bits + (int64_t)(y - J.miny) * J.wpr + (x >> 5);
#ifdef __HIP_DEVICE_COMPILE__
  atomicXor(word, 1u << (x & 31));
#else
  *word ^= 1u << (x & 31);
#endif
}

// Scanline range of GDALdllImageFilledPolygon over every vertex of the rings.
inline void fill_rows(const double *Y, int n, int h, int32_t &miny, int32_t &maxy) {
  double dminy = Y[0], dmaxy = Y[0];
  for (int i = 1; i < n; i++) { dminy = std::min(dminy, Y[i]); dmaxy = std::max(dmaxy, Y[i]); }
  miny = std::max((int)dminy, 0);
  maxy = std::min((int)dmaxy, h - 1);
}

// Edge (ind1 -> ind2) of GDALdllImageFilledPolygon: on every pixel-centre
// line y + 0.5 it crosses (half-open [dy1, dy2)), GDAL's intersection
// abscissa toggles the parity bit at max(x, 0) when x <= w - 1 (an
// intersection right of the canvas never counts); a horizontal edge lying on
// a pixel-centre line burns its span when it is a bottom edge (x1 > x2).
__host__ __device__ inline void scan_edge(const RasterJob &J, double dx1, double dy1, double dx2, double dy2) {
  const int minx = 0, maxx = J.w - 1;
  if (dy1 == dy2) {
    if (!(dx1 > dx2)) return;   // top edges skipped
    const int y = (int)floor(dy1);
    if (y < J.miny || y > J.maxy || (double)y + 0.5 != dy1) return;
    const int h1 = (int)floor(dx2 + 0.5), h2 = (int)floor(dx1 + 0.5);
    if (h1 > maxx || h2 <= minx) return;
    for (int x = h1 > 0 ? h1 : 0; x <= (h2 - 1 < J.w - 1 ? h2 - 1 : J.w - 1); x++) burn(J, x, y);
    return;
  }
  if (dy1 > dy2) {
    double t = dy1; dy1 = dy2; dy2 = t;
    t = dx1; dx1 = dx2; dx2 = t;
  }
  // rows whose centre can lie in [dy1, dy2); the test below is GDAL's, exactly
  const double f0 = floor(dy1 - 0.5) - 1.0, f1 = floor(dy2 - 0.5) + 1.0;
  const int y0 = f0 > (double)J.miny ? (int)f0 : J.miny;
  const int y1 = f1 < (double)J.maxy ? (int)f1 : J.maxy;
  for (int y = y0; y <= y1; y++) {
    const double dy = y + 0.5;
    if (!(dy < dy2 && dy >= dy1)) continue;
    const int x = (int)floor((dy - dy1) * (dx2 - dx1) / (dy2 - dy1) + dx1 + 0.5);
    if (x <= maxx) toggle(J, y, x > minx ? x : minx);
  }
}

// Row y of the fill: prefix parity over the row's bits, burn the odd pixels.
__host__ __device__ inline void burn_row(const RasterJob &J, int y) {
  const uint32_t *row = J.bits + (int64_t)(y - J.miny) * J.wpr;
  uint32_t carry = 0;
  for (int k = 0; k < J.wpr; k++) {
    uint32_t p = row[k];
    p ^= p << 1; p ^= p << 2; p ^= p << 4; p ^= p << 8; p ^= p << 16;   // prefix xor within the word
    p ^= carry;
    carry = (p >> 31) ? 0xFFFFFFFFu : 0u;
    while (p) {
      const int b = __builtin_ctz(p);
      burn(J, 32 * k + b, y);
      p &= p - 1;
    }
  }
}

// GDALdllImageLineAllTouched (GDAL 3.0.1) for the segment (x, y) -> (xe, ye),
// burn value only.
__host__ __device__ inline void touch_edge(const RasterJob &J, double x, double y, double xe, double ye) {
  const int w = J.w, h = J.h;
  if ((y < 0.0 && ye < 0.0) || (y > h && ye > h) || (x < 0.0 && xe < 0.0) || (x > w && xe > w)) return;
  if (x > xe) {
    double t = x; x = xe; xe = t;
    t = y; y = ye; ye = t;
  }
  if (floor(x) == floor(xe) || fabs(x - xe) < .01) {   // vertical
    if (ye < y) { const double t = y; y = ye; ye = t; }
    const int ix = (int)floor(xe);
    if (ix < 0 || ix >= w) return;
    const int iy0 = (int)floor(y) > 0 ? (int)floor(y) : 0;
    const int iy1 = (int)floor(ye) < h - 1 ? (int)floor(ye) : h - 1;
    for (int iy = iy0; iy <= iy1; iy++) burn(J, ix, iy);
    return;
  }
  if (floor(y) == floor(ye) || fabs(y - ye) < .01) {   // horizontal
    const int iy = (int)floor(y);
    if (iy < 0 || iy >= h) return;
    const int ix0 = (int)floor(x) > 0 ? (int)floor(x) : 0;
    const int ix1 = (int)floor(xe) < w - 1 ? (int)floor(xe) : w - 1;
    for (int ix = ix0; ix <= ix1; ix++) burn(J, ix, iy);
    return;
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
    if (iy >= 0 && iy < h) burn(J, ix, iy);
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

// Edge k of a polygon's rings, k in [0, n): (ind1, ind2) of
// GDALdllImageFilledPolygon (the closing edge last -> first of its ring for
// the ring's first point) and, unless k starts its ring, the segment k-1 -> k
// that GDALdllImageLineAllTouched draws.
__host__ __device__ inline void edge_of(const int32_t *part, int np, int k, int &ind1, int &ind2, bool &draw) {
  int start = 0, r = 0;
  while (r < np && k >= start + part[r]) { start += part[r]; r++; }
  if (r >= np) { ind1 = ind2 = k; draw = false; return; }
  draw = k != start;
  ind1 = draw ? k - 1 : start + part[r] - 1;
  ind2 = k;
}

struct Descriptor {
  int32_t win[4] = {0, 0, 0, 0};
  int status = 0;
  Rings pix;   // rings in the window's pixel space (mask rasterization)
};

// What every polygon of one call shares: the CRS pair, the file envelope
// (its corners printed with Go "%f" into WKT, drill.go:386-393) and the
// inverse geotransform -- computed once per call, not per polygon.
struct DescribeCtx {
  const gskyhip_crs *crs = nullptr;   // dataset SRS, or NULL (no reprojection)
  gskyhip_crs wgs;
  bool reproject = false;
  double box[4];                      // file envelope: min x, min y, max x, max y
  double igt[6];
  const double *gt = nullptr;
};

DescribeCtx make_ctx(const gskyhip_crs *crs, const double gt[6], int xsize, int ysize) {
  DescribeCtx c;
  c.crs = crs;
  c.gt = gt;
  if (crs) {
    gskyhip_crs_from_srs("EPSG:4326", &c.wgs);
    c.reproject = !crs_same(c.wgs, *crs);
  }
  const double ulX = go_f6(gt[0] + 0 * gt[1] + 0 * gt[2]), ulY = go_f6(gt[3] + 0 * gt[4] + 0 * gt[5]);
  const double lrX = go_f6(gt[0] + xsize * gt[1] + ysize * gt[2]);
  const double lrY = go_f6(gt[3] + xsize * gt[4] + ysize * gt[5]);
  c.box[0] = std::min(ulX, lrX); c.box[1] = std::min(ulY, lrY);
  c.box[2] = std::max(ulX, lrX); c.box[3] = std::max(ulY, lrY);
  inv_geot(gt, c.igt);
  return c;
}

// getDrillFileDescriptor (drill.go:363-423) up to the mask's pixel rings,
// into `d` (its ring vectors keep their capacity from earlier calls).
void describe(const char *geometry, const DescribeCtx &c, Descriptor &d) {
  d.status = 0;
  for (int k = 0; k < 4; k++) d.win[k] = 0;
  Rings &r = d.pix;
  r.x.clear();
  r.y.clear();
  r.part.clear();
  r.poly.clear();
  if (!parse_geometry(geometry, r)) { d.status = GSKYHIP_E_ARG; return; }
  buffer0_rings(r.x, r.y, r.part, r.poly);   // OGR_G_Buffer(g, 0, 30); empty -> the rings as drawn
  if (c.reproject)   // WGS84 lon/lat -> dataset SRS, the warp's transform
    for (size_t i = 0; i < r.x.size(); i++) {
      double lam, phi, X, Y;
      if (!crs_inverse(c.wgs, r.x[i], r.y[i], lam, phi) || !crs_forward(*c.crs, lam, phi, X, Y)) {
        d.status = GSKYHIP_E_CRS;
        return;
      }
      r.x[i] = X;
      r.y[i] = Y;
    }
  double env[4];
  if (!clip_envelope(r, c.box[0], c.box[1], c.box[2], c.box[3], env)) {
    d.status = GSKYHIP_E_RANGE;   // the polygon misses the file
    return;
  }
  const double *igt = c.igt;
  const double omx = igt[0] + env[0] * igt[1] + env[1] * igt[2], omy = igt[3] + env[0] * igt[4] + env[1] * igt[5];
  const double oMx = igt[0] + env[2] * igt[1] + env[3] * igt[2], oMy = igt[3] + env[2] * igt[4] + env[3] * igt[5];
  int32_t offX = go_cvtt32(std::fmin(omx, oMx)), offY = go_cvtt32(std::fmin(omy, oMy));
  int32_t cX = go_cvtt32(std::fmax(omx, oMx)) - offX, cY = go_cvtt32(std::fmax(omy, oMy)) - offY;
  if (cX == 0) cX++;
  if (cY == 0) cY++;
  if (offX < 0) offX = 0;
  if (offY < 0) offY = 0;
  d.win[0] = offX; d.win[1] = offY; d.win[2] = cX; d.win[3] = cY;
  if (cX <= 0 || cY <= 0) { d.status = GSKYHIP_E_RANGE; return; }
  // createMask (drill.go:294-308): the MEM raster's geotransform is the
  // dataset's shifted by the window offset (rotation terms kept as they are)
  double mgt[6], migt[6];
  std::memcpy(mgt, c.gt, sizeof(mgt));
  mgt[0] += mgt[1] * (double)offX;
  mgt[3] += mgt[5] * (double)offY;
  inv_geot(mgt, migt);
  for (size_t i = 0; i < r.x.size(); i++) {
    const double X = r.x[i], Y = r.y[i];
    r.x[i] = migt[0] + X * migt[1] + Y * migt[2];
    r.y[i] = migt[3] + X * migt[4] + Y * migt[5];
  }
}

// A persistent pool of host threads for describe_all: created once (again
// in a forked child, whose copy has no threads), woken per call through a
// generation counter; the caller works too and waits until every worker has
// left the job.  Thread creation per call cost 300 us of a 0.5 ms describe
// (16 threads, r04r); a wake costs a few microseconds.
struct DescribePool {
  std::mutex mu;
  std::condition_variable cv_go, cv_done;
  uint64_t gen = 0;
  int busy = 0;                       // workers inside the current job
  int n_workers = 0;
  pid_t pid = 0;
  std::function<void()> job;
  std::mutex call_mu;                 // one describe_all at a time (the storage below is shared)
  std::vector<Descriptor> store;      // descriptors of the last call, capacity kept

  void worker(uint64_t seen) {
    for (;;) {
      std::function<void()> f;
      {
        std::unique_lock<std::mutex> lk(mu);
        cv_go.wait(lk, [&] { return gen != seen; });
        seen = gen;
        f = job;
      }
      if (f) f();
      {
        std::lock_guard<std::mutex> lk(mu);
        if (--busy == 0) cv_done.notify_all();
      }
    }
  }
  // run f on the caller and up to `want` workers; returns once all are done
  void run(int want, const std::function<void()> &f) {
    if (pid != getpid()) {   // first use, or a forked child: (re)start the workers
      pid = getpid();
      n_workers = 0;
    }
    while (n_workers < want) {
      uint64_t g;
      {
        std::lock_guard<std::mutex> lk(mu);
        g = gen;
      }
      std::thread(&DescribePool::worker, this, g).detach();
      n_workers++;
    }
    if (n_workers == 0) { f(); return; }
    {
      std::lock_guard<std::mutex> lk(mu);
      job = f;
      busy = n_workers;
      gen++;
    }
    cv_go.notify_all();
    f();
    std::unique_lock<std::mutex> lk(mu);
    cv_done.wait(lk, [&] { return busy == 0; });
    job = nullptr;
  }
};
DescribePool &describe_pool() {
  static DescribePool *p = new DescribePool();   // never destroyed: its threads are detached
  return *p;
}

// describe() of every polygon on the pool (polygons are independent; the
// reference describes one per gRPC call, drill_grpc.go:127-158).  The result
// lives in the pool's storage; the caller holds `lk` (DescribePool::call_mu)
// while it uses it.
std::vector<Descriptor> &describe_all(const char *const *geometries, int n, const DescribeCtx &c,
                                      std::unique_lock<std::mutex> &lk) {
  DescribePool &P = describe_pool();
  lk = std::unique_lock<std::mutex>(P.call_mu);
  std::vector<Descriptor> &out = P.store;
  if ((int)out.size() < n) out.resize((size_t)n);
  static const int cap = [] {   // GSKYHIP_DRILL_THREADS: at most this many (default 16)
    const char *e = std::getenv("GSKYHIP_DRILL_THREADS");
    const int v = e ? std::atoi(e) : 16;
    return std::max(1, std::min(64, v));
  }();
  const int hw = (int)std::max(1u, std::thread::hardware_concurrency());
  const int nth = std::min(std::min(cap, hw), std::max(1, n / 32));
  std::atomic<int> next(0);
  auto work = [&]() {
    for (int i = next.fetch_add(8); i < n; i = next.fetch_add(8))
      for (int k = i; k < std::min(n, i + 8); k++) {
        try {
          describe(geometries[k], c, out[k]);
        } catch (...) {   // bad_alloc of a huge ring: that polygon fails, not the process
          out[k].pix = Rings();
          out[k].status = GSKYHIP_E_ARG;
        }
      }
  };
  static const bool trace = std::getenv("GSKYHIP_DRILL_TRACE") != nullptr;
  const auto t0 = std::chrono::steady_clock::now();
  P.run(nth - 1, work);
  if (trace) {
    const auto t1 = std::chrono::steady_clock::now();
    std::fprintf(stderr, "describe_all n=%d threads=%d us=%.1f\n", n, nth,
                 std::chrono::duration<double, std::micro>(t1 - t0).count());
  }
  return out;
}

// ---------------------------------------------------------------- GPU rasterizer
// The same passes on the GPU, straight into the device mask buffer: one
// workgroup per polygon, a thread per edge for the ALL_TOUCHED lines and the
// parity toggles (atomic XOR), then a thread per scanline for the burn.  Both
// only ever write 255, so thread order and overlapping writes do not matter;
// masks and bitmaps are zeroed first.  No bound on vertices or intersections.
struct PolyDev {
  int64_t mask_off;
  int64_t bits_off;    // first parity word
  int32_t w, h;
  int32_t v0, nv;      // vertex range in vx / vy
  int32_t p0, np;      // ring range in parts (points per ring)
  int32_t miny, maxy, wpr, _pad;
};

__device__ inline RasterJob job_of(const PolyDev &P, uint8_t *masks, uint32_t *bits) {
  RasterJob J;
  J.m = masks + P.mask_off;
  J.bits = bits + P.bits_off;
  J.w = P.w; J.h = P.h; J.miny = P.miny; J.maxy = P.maxy; J.wpr = P.wpr;
  return J;
}

__global__ __launch_bounds__(256) void edges_kernel(const PolyDev *polys, const double *vx, const double *vy,
                                                    const int32_t *parts, uint8_t *masks, uint32_t *bits) {
  const PolyDev P = polys[blockIdx.x];
  const RasterJob J = job_of(P, masks, bits);
  const double *X = vx + P.v0, *Y = vy + P.v0;
  for (int k = threadIdx.x; k < P.nv; k += blockDim.x) {
    int ind1, ind2;
    bool draw;
    edge_of(parts + P.p0, P.np, k, ind1, ind2, draw);
    if (draw) touch_edge(J, X[k - 1], Y[k - 1], X[k], Y[k]);
    if (ind1 != ind2 || draw) scan_edge(J, X[ind1], Y[ind1], X[ind2], Y[ind2]);
  }
}

__global__ __launch_bounds__(256) void burn_rows_kernel(const PolyDev *polys, uint8_t *masks, uint32_t *bits) {
  const PolyDev P = polys[blockIdx.x];
  const RasterJob J = job_of(P, masks, bits);
  for (int y = P.miny + (int)threadIdx.x; y <= P.maxy; y += blockDim.x) burn_row(J, y);
}

// Host rasterization of one window (gskyhip_drill_descriptors): the same
// functions, edges then rows.
void rasterize_host(const Rings &r, uint8_t *m, int w, int h) {
  const int n = (int)r.x.size();
  if (r.part.empty() || n == 0) return;
  RasterJob J;
  J.m = m; J.w = w; J.h = h;
  fill_rows(r.y.data(), n, h, J.miny, J.maxy);
  J.wpr = (w + 31) / 32;
  std::vector<uint32_t> bits(J.maxy >= J.miny ? (size_t)(J.maxy - J.miny + 1) * J.wpr : 0, 0u);
  J.bits = bits.data();
  for (int k = 0; k < n; k++) {
    int ind1, ind2;
    bool draw;
    edge_of(r.part.data(), (int)r.part.size(), k, ind1, ind2, draw);
    if (draw) touch_edge(J, r.x[k - 1], r.y[k - 1], r.x[k], r.y[k]);
    if (J.maxy >= J.miny) scan_edge(J, r.x[ind1], r.y[ind1], r.x[ind2], r.y[ind2]);
  }
  for (int y = J.miny; y <= J.maxy; y++) burn_row(J, y);
}

// Persistent staging of the GPU rasterizer (polygons | x | y | parts |
// parity bitmaps): grown, never freed per call; one call at a time uses it
// (the call synchronizes its stream before releasing the lock).
struct Staging {
  std::mutex mu;
  char *dev = nullptr;
  size_t dev_cap = 0;
  char *host = nullptr;   // pinned
  size_t host_cap = 0;
};
Staging &staging() {
  static Staging st;
  return st;
}

// Windows, mask offsets and statuses of described polygons (16-byte aligned
// mask regions in polygon order); returns the mask buffer size.
int64_t layout(const std::vector<Descriptor> &ds, int n, int32_t *win_out, int64_t *mask_off_out,
               int32_t *status_out) {
  int64_t off = 0;
  for (size_t i = 0; i < (size_t)n; i++) {
    const Descriptor &d = ds[i];
    status_out[i] = d.status;
    const int64_t bytes = d.status == 0 ? (int64_t)d.win[2] * d.win[3] : 0;
    for (int k = 0; k < 4; k++) win_out[4 * i + k] = d.status == 0 ? d.win[k] : 0;
    mask_off_out[i] = off;
    off += (bytes + 15) / 16 * 16;
  }
  return off > 0 ? off : 16;
}

// ALL_TOUCHED masks of described polygons rasterized on the GPU into
// masks_dev (zeroed first), on `s`.
int rasterize_device(const std::vector<Descriptor> &ds, int n, const int64_t *mask_off, uint8_t *masks_dev,
                     int64_t mask_bytes, hipStream_t s) {
  if (hipMemsetAsync(masks_dev, 0, (size_t)mask_bytes, s) != hipSuccess) return GSKYHIP_E_HIP;
  std::vector<PolyDev> polys;
  size_t nv = 0, npart = 0;
  for (int di = 0; di < n; di++) {
    const Descriptor &d = ds[di];
    if (d.status == 0 && !d.pix.x.empty()) { nv += d.pix.x.size(); npart += d.pix.part.size(); }
  }
  polys.reserve((size_t)n);
  int64_t words = 0;
  int32_t v0 = 0, p0 = 0;
  for (size_t i = 0; i < (size_t)n; i++) {
    const Descriptor &d = ds[i];
    if (d.status != 0 || d.pix.x.empty() || (int64_t)d.win[2] * d.win[3] <= 0) continue;
    PolyDev P;
    P.mask_off = mask_off[i];
    P.w = d.win[2];
    P.h = d.win[3];
    P.v0 = v0;
    P.nv = (int32_t)d.pix.x.size();
    P.p0 = p0;
    P.np = (int32_t)d.pix.part.size();
    fill_rows(d.pix.y.data(), P.nv, P.h, P.miny, P.maxy);
    P.wpr = (P.w + 31) / 32;
    P._pad = 0;
    P.bits_off = words;
    if (P.maxy >= P.miny) words += (int64_t)(P.maxy - P.miny + 1) * P.wpr;
    else P.maxy = P.miny - 1;   // no scanline: only the ALL_TOUCHED lines
    v0 += P.nv;
    p0 += P.np;
    polys.push_back(P);
  }
  if (polys.empty()) return 0;
  const size_t b0 = (polys.size() * sizeof(PolyDev) + 15) / 16 * 16, b1 = nv * 8, b2 = (npart * 4 + 15) / 16 * 16;
  const size_t b3 = (size_t)std::max<int64_t>(words, 1) * 4;
  const size_t hbytes = b0 + 2 * b1 + b2;
  Staging &st = staging();
  std::lock_guard<std::mutex> lk(st.mu);
  if (st.dev_cap < hbytes + b3) {
    if (st.dev) (void)hipFree(st.dev);
    st.dev = nullptr;
    st.dev_cap = 0;
    if (hipMalloc(&st.dev, (hbytes + b3) * 5 / 4) != hipSuccess) return GSKYHIP_E_HIP;
    st.dev_cap = (hbytes + b3) * 5 / 4;
  }
  if (st.host_cap < hbytes) {
    if (st.host) (void)hipHostFree(st.host);
    st.host = nullptr;
    st.host_cap = 0;
    if (hipHostMalloc((void **)&st.host, hbytes * 5 / 4, hipHostMallocDefault) != hipSuccess) return GSKYHIP_E_HIP;
    st.host_cap = hbytes * 5 / 4;
  }
  char *h = st.host;
  std::memcpy(h, polys.data(), polys.size() * sizeof(PolyDev));
  double *hx = (double *)(h + b0), *hy = (double *)(h + b0 + b1);
  int32_t *hp = (int32_t *)(h + b0 + 2 * b1);
  for (int di = 0; di < n; di++) {
    const Descriptor &d = ds[di];
    if (d.status != 0 || d.pix.x.empty() || (int64_t)d.win[2] * d.win[3] <= 0) continue;
    std::memcpy(hx, d.pix.x.data(), d.pix.x.size() * 8); hx += d.pix.x.size();
    std::memcpy(hy, d.pix.y.data(), d.pix.y.size() * 8); hy += d.pix.y.size();
    std::memcpy(hp, d.pix.part.data(), d.pix.part.size() * 4); hp += d.pix.part.size();
  }
  char *dev = st.dev;
  int rc = 0;
  uint32_t *bits = (uint32_t *)(dev + hbytes);
  if (hipMemcpyAsync(dev, h, hbytes, hipMemcpyHostToDevice, s) != hipSuccess) rc = GSKYHIP_E_HIP;
  if (!rc && hipMemsetAsync(bits, 0, b3, s) != hipSuccess) rc = GSKYHIP_E_HIP;
  const PolyDev *dp = (const PolyDev *)dev;
  const double *dx = (const double *)(dev + b0), *dy = (const double *)(dev + b0 + b1);
  const int32_t *dpart = (const int32_t *)(dev + b0 + 2 * b1);
  if (!rc) {
    hipLaunchKernelGGL(edges_kernel, dim3((unsigned)polys.size()), dim3(256), 0, s, dp, dx, dy, dpart, masks_dev,
                       bits);
    hipLaunchKernelGGL(burn_rows_kernel, dim3((unsigned)polys.size()), dim3(256), 0, s, dp, masks_dev, bits);
    if (hipGetLastError() != hipSuccess) rc = GSKYHIP_E_HIP;
  }
  // the staging buffers are reused by the next call: the work must be done
  if (hipStreamSynchronize(s) != hipSuccess && !rc) rc = GSKYHIP_E_HIP;
  return rc;
}

int ctx_of(const char *dataset_srs, gskyhip_crs &crs, const gskyhip_crs *&pc) {
  pc = nullptr;
  if (dataset_srs && *dataset_srs) {
    if (gskyhip_crs_from_srs(dataset_srs, &crs)) return GSKYHIP_E_CRS;
    pc = &crs;
  }
  return 0;
}

}  // namespace
}  // namespace gsky

using namespace gsky;

// The GeoJSON number parser on n NUL-separated strings packed in `text` (test
// hook: checked against strtod / Python float by tests/test_drill_geom.py);
// consumed[i] = characters parsed.
extern "C" int gskyhip_parse_numbers(const char *text, int n, double *out, int32_t *consumed) {
  if (!text || n < 0 || !out || !consumed) return GSKYHIP_E_ARG;
  for (int i = 0; i < n; i++) {
    char *e;
    out[i] = parse_number(text, &e);
    consumed[i] = (int32_t)(e - text);
    text += std::strlen(text) + 1;
  }
  return 0;
}

// Windows on the host, ALL_TOUCHED masks rasterized on the GPU into masks_dev
// (every polygon, any vertex count), all on `stream`.  masks_dev == NULL:
// windows, offsets and the buffer size only.
extern "C" int gskyhip_drill_descriptors_device(const char *const *geometries, int n, const char *dataset_srs,
                                                const double *geot, int xsize, int ysize, int32_t *win_out,
                                                int64_t *mask_off_out, int64_t *mask_bytes_out, uint8_t *masks_dev,
                                                int32_t *status_out, void *stream) {
  if (n < 0 || !geot || !win_out || !mask_off_out || !mask_bytes_out || !status_out) return GSKYHIP_E_ARG;
  try {
    gskyhip_crs crs;
    const gskyhip_crs *pc;
    if (ctx_of(dataset_srs, crs, pc)) return GSKYHIP_E_CRS;
    std::unique_lock<std::mutex> lk;
    std::vector<Descriptor> &ds = describe_all(geometries, n, make_ctx(pc, geot, xsize, ysize), lk);
    *mask_bytes_out = layout(ds, n, win_out, mask_off_out, status_out);
    if (!masks_dev) return 0;
    return rasterize_device(ds, n, mask_off_out, masks_dev, *mask_bytes_out, (hipStream_t)stream);
  } catch (...) {
    return GSKYHIP_E_ARG;
  }
}

// The same in one pass: the polygons are described once, then alloc(ctx,
// bytes) supplies the device mask buffer of the size that needs.
extern "C" int gskyhip_drill_masks_device(const char *const *geometries, int n, const char *dataset_srs,
                                          const double *geot, int xsize, int ysize, int32_t *win_out,
                                          int64_t *mask_off_out, int64_t *mask_bytes_out, gskyhip_alloc_fn alloc,
                                          void *alloc_ctx, uint8_t **masks_dev_out, int32_t *status_out,
                                          void *stream) {
  if (n < 0 || !geot || !win_out || !mask_off_out || !mask_bytes_out || !status_out || !alloc || !masks_dev_out)
    return GSKYHIP_E_ARG;
  try {
    gskyhip_crs crs;
    const gskyhip_crs *pc;
    if (ctx_of(dataset_srs, crs, pc)) return GSKYHIP_E_CRS;
    std::unique_lock<std::mutex> lk;
    std::vector<Descriptor> &ds = describe_all(geometries, n, make_ctx(pc, geot, xsize, ysize), lk);
    *mask_bytes_out = layout(ds, n, win_out, mask_off_out, status_out);
    uint8_t *m = (uint8_t *)alloc(alloc_ctx, *mask_bytes_out);
    *masks_dev_out = m;
    if (!m) return GSKYHIP_E_HIP;
    return rasterize_device(ds, n, mask_off_out, m, *mask_bytes_out, (hipStream_t)stream);
  } catch (...) {
    return GSKYHIP_E_ARG;
  }
}

// The same with the n geometries packed NUL-separated in one buffer (a
// caller with the strings in one allocation -- Python's one join + encode --
// builds no pointer array).
extern "C" int gskyhip_drill_masks_device_packed(const char *packed, int64_t packed_bytes, int n,
                                                 const char *dataset_srs, const double *geot, int xsize, int ysize,
                                                 int32_t *win_out, int64_t *mask_off_out, int64_t *mask_bytes_out,
                                                 gskyhip_alloc_fn alloc, void *alloc_ctx, uint8_t **masks_dev_out,
                                                 int32_t *status_out, void *stream) {
  if (n < 0 || !packed || packed_bytes < 0) return GSKYHIP_E_ARG;
  try {
    std::vector<const char *> ptr((size_t)std::max(1, n));
    const char *p = packed, *end = packed + packed_bytes;
    for (int i = 0; i < n; i++) {
      if (p >= end) return GSKYHIP_E_ARG;
      ptr[(size_t)i] = p;
      const void *z = std::memchr(p, 0, (size_t)(end - p));
      if (!z) return GSKYHIP_E_ARG;   // every string NUL-terminated inside the buffer
      p = (const char *)z + 1;
    }
    return gskyhip_drill_masks_device(ptr.data(), n, dataset_srs, geot, xsize, ysize, win_out, mask_off_out,
                                      mask_bytes_out, alloc, alloc_ctx, masks_dev_out, status_out, stream);
  } catch (...) {
    return GSKYHIP_E_ARG;
  }
}

extern "C" int gskyhip_drill_descriptors(const char *const *geometries, int n, const char *dataset_srs,
                                         const double *geot, int xsize, int ysize, int32_t *win_out,
                                         int64_t *mask_off_out, int64_t *mask_bytes_out, uint8_t *masks_out,
                                         int32_t *status_out) {
  if (n < 0 || !geot || !win_out || !mask_off_out || !mask_bytes_out || !status_out) return GSKYHIP_E_ARG;
  try {
    gskyhip_crs crs;
    const gskyhip_crs *pc;
    if (ctx_of(dataset_srs, crs, pc)) return GSKYHIP_E_CRS;
    std::unique_lock<std::mutex> lk;
    std::vector<Descriptor> &ds = describe_all(geometries, n, make_ctx(pc, geot, xsize, ysize), lk);
    *mask_bytes_out = layout(ds, n, win_out, mask_off_out, status_out);
    if (masks_out)
      for (int i = 0; i < n; i++) {
        const Descriptor &d = ds[i];
        const int64_t bytes = d.status == 0 ? (int64_t)d.win[2] * d.win[3] : 0;
        if (bytes <= 0) continue;
        std::memset(masks_out + mask_off_out[i], 0, (size_t)bytes);
        rasterize_host(d.pix, masks_out + mask_off_out[i], d.win[2], d.win[3]);   // ALL_TOUCHED lines + fill
      }
    return 0;
  } catch (...) {
    return GSKYHIP_E_ARG;
  }
}
