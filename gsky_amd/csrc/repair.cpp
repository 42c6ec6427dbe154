// repair.cpp -- OGR_G_Buffer(g, 0, 30) (worker/gdalprocess/drill.go:364-367)
// of the drill request geometry, as GEOS 3.7.2 (the reference's pin,
// docker/build_deps.sh:90) computes a zero-distance buffer of a Polygon /
// MultiPolygon:
//
//   OffsetCurveSetBuilder::addPolygon  each ring, repeated points removed, is
//                                      its own offset curve at distance 0;
//                                      a shell of < 3 points drops its
//                                      polygon, a ring of < 4 points is
//                                      skipped;
//   addPolygonRing                     the ring's sides are labelled from its
//                                      orientation (CGAlgorithms::isCCW: the
//                                      turn at the first highest vertex):
//                                      shell interior / hole exterior on the
//                                      right of a clockwise ring, swapped for
//                                      a counter-clockwise one;
//   BufferBuilder                      the curves noded against each other
//                                      (every crossing, touch and collinear
//                                      overlap splits the segments), equal
//                                      edges merged with their depth deltas
//                                      summed, depths propagated from the
//                                      outside (0), and the result is the
//                                      region of depth >= 1: the boundary
//                                      edges with depth >= 1 on their right
//                                      and <= 0 on their left, as rings with
//                                      the interior on their right.
//
// The depth of a point is thus the sum over the curves of their winding
// numbers, each signed by its ring's role and isCCW; the implementation
// computes it directly, per noded edge, by a ray cast over the edges of its
// horizontal band; candidate crossings come from a sweep in x.  A valid polygon (no crossings, overlaps or touches; every ring
// between depths 0 and 1) comes back with its vertices unchanged, reversed
// where its interior was on the left.  The results the rasterizer sees differ
// from the rings as drawn for self-intersecting or multiply-wound rings (a
// bow-tie keeps only the lobe of its highest vertex's orientation), holes
// outside their shell, nested or overlapping polygons (unioned), and
// zero-area spikes (removed).  A geometry with more than 2^16 self-crossings
// is left as drawn.  Parity unpinned beyond the oracle's separate
// restatement: GEOS is absent from this image.
#include "repair.h"

#include <algorithm>
#include <cmath>
#include <cstdint>

namespace gsky {
namespace {

struct Pt {
  double x, y;
};
inline bool same(const Pt &a, const Pt &b) { return a.x == b.x && a.y == b.y; }
inline bool before(const Pt &a, const Pt &b) { return a.x < b.x || (a.x == b.x && a.y < b.y); }

// sign of (b - a) x (c - a), exact: the double evaluation when it clears its
// error bound, else the products and differences in double-double
// (CGAlgorithmsDD::orientationIndex's role)
struct DD {
  double hi, lo;
};
inline DD two_diff(double a, double b) {
  const double s = a - b, bb = s - a;
  return {s, (a - (s - bb)) - (b + bb)};
}
inline DD dd_mul(DD a, DD b) {
  const double p = a.hi * b.hi;
  const double e = std::fma(a.hi, b.hi, -p) + (a.hi * b.lo + a.lo * b.hi);
  const double s = p + e;
  return {s, e - (s - p)};
}
inline DD dd_sub(DD a, DD b) {
  const double s = a.hi - b.hi, bb = s - a.hi;
  const double e = ((a.hi - (s - bb)) - (b.hi + bb)) + a.lo - b.lo;
  const double r = s + e;
  return {r, e - (r - s)};
}
int orient(const Pt &a, const Pt &b, const Pt &c) {
  if (same(c, a) || same(c, b)) return 0;
  const double l = (b.x - a.x) * (c.y - a.y), r = (b.y - a.y) * (c.x - a.x);
  const double det = l - r, bound = 1e-15 * (std::fabs(l) + std::fabs(r));
  if (det > bound) return 1;
  if (det < -bound) return -1;
  if (l == 0 && r == 0) return 0;   // c on a vertex, or a degenerate segment
  const DD d = dd_sub(dd_mul(two_diff(b.x, a.x), two_diff(c.y, a.y)), dd_mul(two_diff(b.y, a.y), two_diff(c.x, a.x)));
  const double v = d.hi + d.lo;
  return (v > 0) - (v < 0);
}

// CGAlgorithms::isCCW (GEOS 3.7) of a closed ring of n >= 4 points
bool is_ccw(const Pt *p, int n) {
  const int npts = n - 1;
  int hi = 0;
  for (int i = 1; i <= npts; i++)
    if (p[i].y > p[hi].y) hi = i;
  int ip = hi;
  do {
    if (--ip < 0) ip = npts;
  } while (same(p[ip], p[hi]) && ip != hi);
  int in = hi;
  do {
    in = (in + 1) % npts;
  } while (same(p[in], p[hi]) && in != hi);
  if (same(p[ip], p[hi]) || same(p[in], p[hi]) || same(p[ip], p[in])) return false;
  const int d = orient(p[ip], p[hi], p[in]);
  return d == 0 ? p[ip].x > p[in].x : d > 0;
}

// a ring crossing itself more often than this (a hostile request, not a
// boundary) is left as drawn rather than noded without bound
constexpr size_t kMaxCrossings = size_t(1) << 16;   // per geometry

struct Seg {
  Pt a, b;
  int q;      // depth(left) - depth(right)
  int ring;   // curve it came from (-1 after merging)
};

// Horizontal bands over the segments' y-ranges (CSR), for ray casts: a
// segment is listed in every band its y-range meets.
struct Bands {
  double y0 = 0, sy = 1;
  int n = 1;
  std::vector<int> start, ids;
  int band(double y) const {
    const double v = (y - y0) / sy;
    return !(v > 0) ? 0 : v >= n - 1 ? n - 1 : (int)v;   // NaN (non-finite input) -> band 0
  }
  void build(const std::vector<Seg> &s) {
    const size_t m = s.size();
    double y1 = -HUGE_VAL;
    y0 = HUGE_VAL;
    for (const Seg &e : s) {
      y0 = std::min(y0, std::min(e.a.y, e.b.y));
      y1 = std::max(y1, std::max(e.a.y, e.b.y));
    }
    n = std::max(1, std::min(4096, 2 * (int)std::sqrt((double)m)));
    sy = y1 > y0 ? (y1 - y0) / n : 1.0;
    start.assign((size_t)n + 1, 0);
    for (int pass = 0; pass < 2; pass++) {
      for (size_t k = 0; k < m; k++) {
        const int lo = band(std::min(s[k].a.y, s[k].b.y)), hi = band(std::max(s[k].a.y, s[k].b.y));
        for (int j = lo; j <= hi; j++) {
          if (pass == 0) start[j + 1]++;
          else ids[start[j]++] = (int)k;
        }
      }
      if (pass == 0) {
        for (int j = 0; j < n; j++) start[j + 1] += start[j];
        ids.resize(start.back());
      } else {
        for (int j = n; j > 0; j--) start[j] = start[j - 1];
        start[0] = 0;
      }
    }
  }
};

// winding number contribution of a -> b (weight q) at p (Sunday's half-open
// rule: a point on a vertex's height counts as just above it)
inline int winding(const Seg &e, const Pt &p) {
  if (e.a.y <= p.y) {
    if (e.b.y > p.y && orient(e.a, e.b, p) > 0) return e.q;
  } else if (e.b.y <= p.y && orient(e.a, e.b, p) < 0) {
    return -e.q;
  }
  return 0;
}

// Depth just right of segment k (at its midpoint): the winding sum of the
// other segments -- those of the midpoint's band, or all of them for a small
// set -- plus k's own share.  A set wider than tall is cast in a frame turned
// by -90 degrees ((x, y) -> (y, -x), exact), so the rays run across its short
// side; the winding numbers are the same.
struct Depth {
  const std::vector<Seg> &s;
  Bands b;
  const bool banded;
  Depth(const std::vector<Seg> &s0, std::vector<Seg> &turned) : s(pick(s0, turned)), banded(s.size() >= 48) {
    if (banded) b.build(s);
  }
  static const std::vector<Seg> &pick(const std::vector<Seg> &s0, std::vector<Seg> &turned) {
    if (s0.size() < 48) return s0;
    double x0 = HUGE_VAL, x1 = -HUGE_VAL, y0 = HUGE_VAL, y1 = -HUGE_VAL;
    for (const Seg &e : s0) {
      x0 = std::min(x0, std::min(e.a.x, e.b.x)); x1 = std::max(x1, std::max(e.a.x, e.b.x));
      y0 = std::min(y0, std::min(e.a.y, e.b.y)); y1 = std::max(y1, std::max(e.a.y, e.b.y));
    }
    if (!(x1 - x0 > y1 - y0)) return s0;
    turned.resize(s0.size());
    for (size_t k = 0; k < s0.size(); k++) {
      const Seg &e = s0[k];
      turned[k] = {{e.a.y, -e.a.x}, {e.b.y, -e.b.x}, e.q, e.ring};
    }
    return turned;
  }
  int right_of(size_t k) const {
    const Seg &e = s[k];
    const Pt m{0.5 * (e.a.x + e.b.x), 0.5 * (e.a.y + e.b.y)};
    int d = 0;
    if (banded) {
      const int j = b.band(m.y);
      for (int t = b.start[j]; t < b.start[j + 1]; t++)
        if ((size_t)b.ids[t] != k) d += winding(s[b.ids[t]], m);
    } else {
      for (size_t t = 0; t < s.size(); t++)
        if (t != k) d += winding(s[t], m);
    }
    if (e.a.y == e.b.y)
      return e.a.x < e.b.x ? d - e.q : d;
    return e.b.y < e.a.y ? d - e.q : d;
  }
};

// p strictly inside segment a-b, given orient(a, b, p) == 0
inline bool strictly_inside(const Pt &a, const Pt &b, const Pt &p) {
  if (same(p, a) || same(p, b)) return false;
  return std::min(a.x, b.x) <= p.x && p.x <= std::max(a.x, b.x) && std::min(a.y, b.y) <= p.y &&
         p.y <= std::max(a.y, b.y);
}

}  // namespace

bool buffer0_rings(std::vector<double> &X, std::vector<double> &Y, std::vector<int> &part,
                   const std::vector<int> &poly) {
  // per-thread scratch (the descriptors run on a thread pool, a polygon per
  // call): grown, never freed, so a valid polygon allocates nothing
  thread_local std::vector<std::vector<Pt>> curves_s;
  thread_local std::vector<int> curve_q_s, order_s;
  thread_local std::vector<Seg> segs_s;
  thread_local std::vector<std::vector<Pt>> splits_s;
  std::vector<int> &curve_q = curve_q_s, &order = order_s;
  std::vector<Seg> &segs = segs_s;
  curve_q.clear();
  segs.clear();
  size_t ncurves = 0;
  // ---- the offset curves: rings without repeated points, closed
  {
    size_t off = 0;
    bool skip_poly = false;
    for (size_t r = 0; r < part.size(); off += part[r], r++) {
      const bool shell = r == 0 || poly[r] != poly[r - 1];
      if (curves_s.size() <= ncurves) curves_s.resize(ncurves + 1);
      std::vector<Pt> &c = curves_s[ncurves];
      c.clear();
      for (int i = 0; i < part[r]; i++) {
        const Pt p{X[off + i], Y[off + i]};
        if (c.empty() || !same(c.back(), p)) c.push_back(p);
      }
      if (shell) skip_poly = c.size() < 3;
      if (skip_poly) continue;
      if (!c.empty() && !same(c.front(), c.back())) c.push_back(c.front());
      if (c.size() < 4) continue;
      const int q = (shell ? 1 : -1) * (is_ccw(c.data(), (int)c.size()) ? 1 : -1);
      const int id = (int)ncurves;
      for (size_t i = 0; i + 1 < c.size(); i++) segs.push_back({c[i], c[i + 1], q, id});
      ncurves++;
      curve_q.push_back(q);
    }
  }
  const std::vector<std::vector<Pt>> &curves = curves_s;
  if (segs.empty()) return false;

  // ---- noding: split points of every segment, candidate pairs from a sweep
  // over the segments sorted by their least x
  const size_t M = segs.size();
  order.resize(M);
  for (size_t k = 0; k < M; k++) order[k] = (int)k;
  auto xlo = [&](int k) { return std::min(segs[k].a.x, segs[k].b.x); };
  std::sort(order.begin(), order.end(), [&](int u, int v) { return xlo(u) < xlo(v); });
  if (splits_s.size() < M) splits_s.resize(M);
  for (size_t k = 0; k < M; k++) splits_s[k].clear();
  std::vector<std::vector<Pt>> &splits = splits_s;
  bool any_split = false, overlap = false, touch = false;
  size_t crossings = 0;
  for (size_t u = 0; u < M; u++) {
    const int i0 = order[u];
    const double xhi = std::max(segs[i0].a.x, segs[i0].b.x);
    for (size_t v = u + 1; v < M && xlo(order[v]) <= xhi; v++) {
      const int i = std::min(i0, order[v]), j = std::max(i0, order[v]);
      const Seg &s = segs[i], &t = segs[j];
      if (std::max(s.a.y, s.b.y) < std::min(t.a.y, t.b.y) || std::max(t.a.y, t.b.y) < std::min(s.a.y, s.b.y))
        continue;
      const int o3 = orient(s.a, s.b, t.a), o4 = orient(s.a, s.b, t.b);
      if (o3 * o4 > 0) continue;   // t wholly on one side of s: no contact
      const int o1 = orient(t.a, t.b, s.a), o2 = orient(t.a, t.b, s.b);
      if (o1 * o2 > 0) continue;
      if (o1 == 0 && o2 == 0 && o3 == 0 && o4 == 0) {   // collinear
        const bool xs = std::fabs(s.b.x - s.a.x) >= std::fabs(s.b.y - s.a.y);
        const double s0 = xs ? std::min(s.a.x, s.b.x) : std::min(s.a.y, s.b.y);
        const double s1 = xs ? std::max(s.a.x, s.b.x) : std::max(s.a.y, s.b.y);
        const double t0 = xs ? std::min(t.a.x, t.b.x) : std::min(t.a.y, t.b.y);
        const double t1 = xs ? std::max(t.a.x, t.b.x) : std::max(t.a.y, t.b.y);
        if (std::min(s1, t1) > std::max(s0, t0)) overlap = true;
        for (const Pt &p : {t.a, t.b})
          if (strictly_inside(s.a, s.b, p)) { splits[i].push_back(p); any_split = true; }
        for (const Pt &p : {s.a, s.b})
          if (strictly_inside(t.a, t.b, p)) { splits[j].push_back(p); any_split = true; }
        continue;
      }
      if (o1 * o2 < 0 && o3 * o4 < 0) {   // proper crossing: one point for both
        // computed from the two segments in a canonical order and direction,
        // so every copy of a segment (a spike, a shared boundary) meets a
        // third one at the same point
        Pt sa = s.a, sb = s.b, ta = t.a, tb = t.b;
        if (before(sb, sa)) std::swap(sa, sb);
        if (before(tb, ta)) std::swap(ta, tb);
        if (before(ta, sa) || (same(ta, sa) && before(tb, sb))) { std::swap(sa, ta); std::swap(sb, tb); }
        const double dx = sb.x - sa.x, dy = sb.y - sa.y, ex = tb.x - ta.x, ey = tb.y - ta.y;
        const double den = dx * ey - dy * ex;
        const double k = ((ta.x - sa.x) * ey - (ta.y - sa.y) * ex) / den;
        Pt p{sa.x + k * dx, sa.y + k * dy};
        // keep it within both segments' envelopes (LineIntersector's guard)
        p.x = std::min(std::max(p.x, std::max(std::min(s.a.x, s.b.x), std::min(t.a.x, t.b.x))),
                       std::min(std::max(s.a.x, s.b.x), std::max(t.a.x, t.b.x)));
        p.y = std::min(std::max(p.y, std::max(std::min(s.a.y, s.b.y), std::min(t.a.y, t.b.y))),
                       std::min(std::max(s.a.y, s.b.y), std::max(t.a.y, t.b.y)));
        splits[i].push_back(p);
        splits[j].push_back(p);
        any_split = true;
        if (++crossings > kMaxCrossings) return false;
        continue;
      }
      // touches: an endpoint on the other segment's interior splits it
      if (o3 == 0 && strictly_inside(s.a, s.b, t.a)) { splits[i].push_back(t.a); any_split = true; }
      if (o4 == 0 && strictly_inside(s.a, s.b, t.b)) { splits[i].push_back(t.b); any_split = true; }
      if (o1 == 0 && strictly_inside(t.a, t.b, s.a)) { splits[j].push_back(s.a); any_split = true; }
      if (o2 == 0 && strictly_inside(t.a, t.b, s.b)) { splits[j].push_back(s.b); any_split = true; }
      // shared endpoints of segments that do not follow each other on a ring
      const int L = s.ring == t.ring ? (int)curves[s.ring].size() - 1 : 0;
      if ((same(s.a, t.a) || same(s.a, t.b) || same(s.b, t.a) || same(s.b, t.b)) &&
          !(s.ring == t.ring && (std::abs(i - j) == 1 || std::abs(i - j) == L - 1)))
        touch = true;
    }
  }

  // ---- a valid polygon: vertices kept, each ring turned interior-right
  if (!any_split && !overlap && !touch) {
    thread_local std::vector<Seg> turned_s;
    const Depth dep(segs, turned_s);
    std::vector<int> first(ncurves, -1);
    for (size_t k = 0; k < segs.size(); k++)
      if (first[segs[k].ring] < 0) first[segs[k].ring] = (int)k;
    bool valid = true;
    std::vector<bool> flip(ncurves);
    for (size_t c = 0; c < ncurves && valid; c++) {
      const int dr = dep.right_of(first[c]), dl = dr + curve_q[c];
      valid = (dr == 1 && dl == 0) || (dr == 0 && dl == 1);
      flip[c] = dl == 1;
    }
    if (valid) {
      X.clear(); Y.clear(); part.clear();
      for (size_t c = 0; c < ncurves; c++) {
        const std::vector<Pt> &v = curves[c];
        for (size_t i = 0; i < v.size(); i++) {
          const Pt &p = flip[c] ? v[v.size() - 1 - i] : v[i];
          X.push_back(p.x);
          Y.push_back(p.y);
        }
        part.push_back((int)v.size());
      }
      return true;
    }
  }

  // ---- noded edges, equal ones merged (canonical direction: lower point first)
  std::vector<Seg> edges;
  edges.reserve(segs.size() * 2);
  for (size_t k = 0; k < segs.size(); k++) {
    const Seg &s = segs[k];
    std::vector<Pt> &sp = splits[k];
    const double dx = s.b.x - s.a.x, dy = s.b.y - s.a.y;
    std::sort(sp.begin(), sp.end(), [&](const Pt &p, const Pt &q) {
      const double u = (p.x - s.a.x) * dx + (p.y - s.a.y) * dy, v = (q.x - s.a.x) * dx + (q.y - s.a.y) * dy;
      return u < v || (u == v && before(p, q));
    });
    Pt prev = s.a;
    auto emit = [&](const Pt &p) {
      if (same(p, prev)) return;
      if (before(prev, p)) edges.push_back({prev, p, s.q, -1});
      else edges.push_back({p, prev, -s.q, -1});
      prev = p;
    };
    for (const Pt &p : sp) emit(p);
    emit(s.b);
  }
  std::sort(edges.begin(), edges.end(), [](const Seg &u, const Seg &v) {
    return before(u.a, v.a) || (same(u.a, v.a) && before(u.b, v.b));
  });
  std::vector<Seg> uniq;
  for (const Seg &e : edges) {
    if (!uniq.empty() && same(uniq.back().a, e.a) && same(uniq.back().b, e.b)) uniq.back().q += e.q;
    else uniq.push_back(e);
  }
  uniq.erase(std::remove_if(uniq.begin(), uniq.end(), [](const Seg &e) { return e.q == 0; }), uniq.end());
  if (uniq.empty()) return false;

  // ---- result edges: depth >= 1 on the right, <= 0 on the left
  thread_local std::vector<Seg> turned_u;
  const Depth dep(uniq, turned_u);
  std::vector<Seg> res;
  for (size_t k = 0; k < uniq.size(); k++) {
    const int dr = dep.right_of(k), dl = dr + uniq[k].q;
    if (dr >= 1 && dl <= 0) res.push_back({uniq[k].a, uniq[k].b, 0, 0});
    else if (dl >= 1 && dr <= 0) res.push_back({uniq[k].b, uniq[k].a, 0, 0});
  }
  if (res.empty()) return false;

  // ---- rings: from each unused edge in order, follow the first unused edge
  // out of the current end (in the same order) until back at the start
  thread_local std::vector<int> by_start_s;
  std::vector<int> &by_start = by_start_s;
  by_start.resize(res.size());
  for (size_t k = 0; k < res.size(); k++) by_start[k] = (int)k;
  std::stable_sort(by_start.begin(), by_start.end(), [&](int u, int v) { return before(res[u].a, res[v].a); });
  std::vector<char> used(res.size(), 0);
  auto next_from = [&](const Pt &p) -> int {
    size_t lo = 0, hi = by_start.size();
    while (lo < hi) {
      const size_t mid = (lo + hi) / 2;
      if (before(res[by_start[mid]].a, p)) lo = mid + 1;
      else hi = mid;
    }
    for (size_t k = lo; k < by_start.size() && same(res[by_start[k]].a, p); k++)
      if (!used[by_start[k]]) return by_start[k];
    return -1;
  };
  X.clear(); Y.clear(); part.clear();
  for (size_t s0 = 0; s0 < res.size(); s0++) {
    if (used[s0]) continue;
    const Pt start = res[s0].a;
    int n = 1;
    X.push_back(start.x);
    Y.push_back(start.y);
    for (int cur = (int)s0; cur >= 0;) {
      used[cur] = 1;
      const Pt b = res[cur].b;
      X.push_back(b.x);
      Y.push_back(b.y);
      n++;
      if (same(b, start)) break;
      cur = next_from(b);
      if (cur < 0) {   // not closed (degenerate noding): close it as drawn
        X.push_back(start.x);
        Y.push_back(start.y);
        n++;
      }
    }
    part.push_back(n);
  }
  return true;
}

}  // namespace gsky
