// render.hip -- batched GetMap hot path on gfx950.
//
// Pipeline for a batch of tiles (one launch each, all async on one stream):
//   plan_pairs_kernel   one wavefront per (tile, granule) pair: the window of
//                       warp.go:154-217 (GDALSuggestedWarpOutput2 edge sampling
//                       in 64 lanes) and the overview pick of warp.go:156-198.
//   plan_tiles_kernel   one thread per tile: merge order of ProcessRasterStack
//                       (tile_merger.go:281-312), maskMap links, fill/overwrite
//                       mode of MergeMaskedRaster (tile_merger.go:47).
//   plan_rows_kernel    one thread per window row, workgroups per pair: GDALApproxTransform
//                       (max error 0.125) reduced to row records / leaves.
//   render_kernel       one lane per 4 output pixels: gather (NN or bilinear)
//                       from HBM-resident granules, ordered nodata/mask fold,
//                       utils.Scale, palette/RGBA fill, 16-byte stores.
// No intermediate FlexRaster ever reaches HBM on the fused path.
#include "gsky_device.h"
#include "render.h"
#include "stages.h"
#include "render_common.h"
#include <algorithm>
#include <map>
#include <vector>
#include <cstdlib>
#include <type_traits>

namespace gsky {

// Everything the planning kernels need per call.
struct PlanArgs {
  const gskyhip_granule *granules;
  const gskyhip_crs *crs;
  int n_crs;
  int dst_crs;                 // -1: no reprojection (warp.go:143-148)
  const gskyhip_tile *tiles;
  int n_tiles;
  const int32_t *pair_granule;
  int n_pairs;
  int pair_tile_max;           // scratch sizes
  int max_h, max_w;            // tile slot of the batch (rgba / canvas layout)
  int mask_ns;
  int mask_inclusive;
  PairPlan *pairs;
  Xform *xforms;
  TilePlan *tplans;
  int32_t *order;              // n_pairs: per tile, stack entries in merge order
  int32_t *pair_tile;          // n_pairs: owning tile of each pair
  RowRec *rows;                // n_pairs * max_h
  RowFix *rowfix;              // n_pairs * max_h: fixed-point form of `inside` LINEAR rows
  Leaf *pool;
  int32_t *counters;           // [0] pool, [1] split rows, [2] complex tiles
  int pool_cap;
  int64_t *split_list;         // (pair * max_h + row) of rows that need the recursion
  int32_t *complex_list;       // tiles that need exact per-pixel transforms
  EntryD *entries;             // n_pairs render descriptors
  SepCol *sepcols;             // 3 per pair: column parts of the separable transform
  int sep;                     // 1: plan_rows uses the separable transform where it applies
  int n_granules;
  struct GEdge *gedge;         // per granule: SuggestedWarpOutput2 edge samples in dst georef (or NULL)
  const GeoLocD *geolocs;      // granule.geoloc k > 0: entry k - 1 (device), or NULL
  int resample;                // GSKYHIP_RESAMPLE_* of the call (the rows' fixed forms)
  int small;                   // 1: plan_pairs finds each pair's tile itself, plan_small_kernel plans the rest
};

// The 84 edge samples of GDALSuggestedWarpOutput2 taken through the
// transformer up to destination GEOREFERENCED coordinates.  They depend on
// the granule (source geotransform + CRS) and the batch's destination CRS
// only, not on the tile, so plan_prologue_kernel computes them once per
// granule and every pair of that granule applies just its tile's inverse
// geotransform -- the last step of xform_point(), the same operations, so
// the samples are bit-identical to the per-pair transform (C2: ~300 pairs
// share each granule's PROJ work).  n_fail > 0 sends the pairs of that
// granule back to the per-pair path (which then samples the 21 x 21 grid).
struct GEdge {
  double x[4 * 21], y[4 * 21];
  int32_t n_fail;
  int32_t _pad;
};

// ---------------------------------------------------------------- pair ownership
// Pair p's tile: the last one whose CSR range starts at or before it (tiles'
// pair ranges are consecutive and ascending).
__device__ __forceinline__ int owning_tile(const gskyhip_tile *tiles, int n_tiles, int p) {
  int lo = 0, hi = n_tiles - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (tiles[mid].pair_begin <= p) lo = mid; else hi = mid - 1;
  }
  while (lo > 0 && tiles[lo].pair_end <= p) lo--;   // empty tiles sharing a begin
  if (!(p >= tiles[lo].pair_begin && p < tiles[lo].pair_end)) {   // not CSR-ordered: scan
    lo = -1;
    for (int t = 0; t < n_tiles; t++)
      if (p >= tiles[t].pair_begin && p < tiles[t].pair_end) lo = t;
  }
  return lo;   // -1: no tile references the pair
}

// ---------------------------------------------------------------- wave helpers
__device__ __forceinline__ double wave_min(double v) {
  for (int o = 32; o > 0; o >>= 1) v = fmin(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ double wave_max(double v) {
  for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o, 64));
  return v;
}

// xform_point behind a call: the planning wave runs it from six sites, and
// inlining every copy of the projection math costs the kernel its occupancy.
__device__ __noinline__ bool xform_point_nl(const Xform &t, bool dst_to_src, double &x, double &y) {
  return xform_point(t, dst_to_src, x, y);
}

// GDALSuggestedWarpOutput2_MustAdjustFor{Right,Bottom}Border, lanes 0..20.
__device__ bool must_adjust(const Xform &t, const double *ext, int np, int nl, double psx,
                            double psy, bool right, int lane) {
  bool bad = false;
  if (lane < 21) {
    // the reference accumulates dfRatio += 0.05 (clamped to 1.0 past 0.99
    // for the sample points, unclamped for the expected values)
    double r1 = 0.0, r2 = 0.0;
    for (int k = 0; k < lane; k++) {
      r1 += 0.05;
      r2 += 0.05;
    }
    if (r1 > 0.99) r1 = 1.0;
    double ax, ay;
    if (right) { ax = ext[2]; ay = ext[3] - psy * r1 * nl; }
    else { ax = ext[0] + psx * r1 * np; ay = ext[1]; }
    bool ok1 = xform_point_nl(t, true, ax, ay);
    bool ok2 = ok1 ? xform_point_nl(t, false, ax, ay) : false;
    double ex = right ? ext[2] : ext[0] + psx * r2 * np;
    double ey = right ? ext[3] - psy * r2 * nl : ext[1];
    bad = !ok1 || !ok2 || fabs(ax - ex) > psx || fabs(ay - ey) > psy;
  }
  unsigned long long b = __ballot(bad);
  return __popcll(b) == 21;
}

// Both border tests at once (lanes 0..20: right border with er / psxr / psyr,
// lanes 32..52: bottom border with eb / psxb / psyb) -- the same per-lane
// expressions as must_adjust().  Bit 0: right must adjust, bit 1: bottom.
__device__ int must_adjust2(const Xform &t, const double *er, double psxr, double psyr, const double *eb,
                            double psxb, double psyb, int np, int nl, int lane) {
  const bool right = lane < 32;
  const int j = lane & 31;
  bool bad = false;
  if (j < 21) {
    double r1 = 0.0, r2 = 0.0;
    for (int k = 0; k < j; k++) {
      r1 += 0.05;
      r2 += 0.05;
    }
    if (r1 > 0.99) r1 = 1.0;
    const double *ext = right ? er : eb;
    const double psx = right ? psxr : psxb, psy = right ? psyr : psyb;
    double ax, ay;
    if (right) { ax = ext[2]; ay = ext[3] - psy * r1 * nl; }
    else { ax = ext[0] + psx * r1 * np; ay = ext[1]; }
    bool ok1 = xform_point_nl(t, true, ax, ay);
    bool ok2 = ok1 ? xform_point_nl(t, false, ax, ay) : false;
    double ex = right ? ext[2] : ext[0] + psx * r2 * np;
    double ey = right ? ext[3] - psy * r2 * nl : ext[1];
    bad = !ok1 || !ok2 || fabs(ax - ex) > psx || fabs(ay - ey) > psy;
  }
  const unsigned long long b = __ballot(bad);
  return (__popcll(b & 0x1FFFFFull) == 21 ? 1 : 0) | (__popcll((b >> 32) & 0x1FFFFFull) == 21 ? 2 : 0);
}

constexpr int kSteps = 20;
constexpr int kSmallBatchPairs = 512;   // plan_pairs_kernel<256> up to this many pairs
constexpr int kSmallBatchTiles = 8, kSmallBatchPlanPairs = 32;   // plan_small_kernel batches
constexpr int64_t kSmallBatchPlanRows = 2048;                      // pairs x tile rows it plans
constexpr int kFusedPlanPairs = 2;   // ... that plan their pairs in the same launch
constexpr int kGrid = (kSteps + 1) * (kSteps + 1);

// First half of xform_point_nl(t, false, ...): source pixel -> destination
// georeferenced coordinates (the same expressions and order).
__device__ __forceinline__ bool src_to_dst_georef(const Xform &t, double x, double y, double &X, double &Y) {
  const double *g1 = t.src_gt;
  if (t.gl) {
    X = x; Y = y;
    if (!geoloc_forward(*t.gl, X, Y)) return false;
  } else {
    X = g1[0] + x * g1[1] + y * g1[2];
    Y = g1[3] + x * g1[4] + y * g1[5];
  }
  if (t.reproject) {
    double lam, phi;
    if (!crs_inverse(t.src, X, Y, lam, phi)) return false;
    if (!crs_forward(t.dst, lam, phi, X, Y)) return false;
  }
  return true;
}

// Planning prologue, 128-thread workgroups: the first n_edge_blocks take a
// granule each, a thread per edge sample (its GEdge, see PlanArgs); the rest
// a pair each per thread (its owning tile).  Workgroup 0 also zeroes the
// plan counters (no separate memset launch: the later planning kernels are
// ordered after this one on the stream).
__global__ __launch_bounds__(128) void plan_prologue_kernel(PlanArgs a, int n_edge_blocks) {
  const int lane = threadIdx.x;
  if (blockIdx.x == 0 && lane < 64) a.counters[lane] = 0;
  if ((int)blockIdx.x >= n_edge_blocks) {
    const int p = ((int)blockIdx.x - n_edge_blocks) * 128 + lane;
    if (p < a.n_pairs) a.pair_tile[p] = owning_tile(a.tiles, a.n_tiles, p);
    return;
  }
  const int g = blockIdx.x;
  if (g >= a.n_granules) return;
  const gskyhip_granule &gr = a.granules[g];
  Xform t;
  t.src = a.crs[gr.crs];
  t.gl = (gr.geoloc > 0 && a.geolocs) ? a.geolocs + (gr.geoloc - 1) : nullptr;
  t.reproject = 0;
  if (a.dst_crs >= 0) {
    t.dst = a.crs[a.dst_crs];
    t.reproject = crs_same(t.src, t.dst) ? 0 : 1;
  } else {
    t.dst = t.src;
  }
  for (int k = 0; k < 6; k++) t.src_gt[k] = gr.geot[k];
  const int nInX = gr.xsize, nInY = gr.ysize;
  const double dfStep = 1.0 / kSteps;
  GEdge &E = a.gedge[g];
  int fail = 0;
  for (int k = lane; k < 4 * (kSteps + 1); k += 128) {
    const int i = k >> 2, e = k & 3;
    const double r = (i == kSteps) ? 1.0 : i * dfStep;
    double x, y;
    if (e == 0) { x = r * nInX; y = 0.0; }
    else if (e == 1) { x = r * nInX; y = nInY; }
    else if (e == 2) { x = 0.0; y = r * nInY; }
    else { x = nInX; y = r * nInY; }
    double X = 0.0, Y = 0.0;
    const bool ok = src_to_dst_georef(t, x, y, X, Y);
    E.x[k] = X;
    E.y[k] = Y;
    fail += ok ? 0 : 1;
  }
  fail = __syncthreads_count(fail);
  if (lane == 0) E.n_fail = fail;
}

// GDALSuggestedWarpOutput2 (gdaltransformer.cpp 3.0.1, nOptions = 0) of the
// transformer t over an nInX x nInY source, by one wavefront: 21 samples on
// each source edge (the full 21 x 21 grid when an edge point fails), the
// pixel size from the diagonal, then the right / bottom border adjustment.
// sx / sy / sok: LDS scratch of kGrid entries.  Returns 0 (CE_None) or 1;
// ext (dst extent), psx / psy (pixel size), nPixels / nLines on success.
__device__ int suggested_warp_output2(const Xform &t, int nInX, int nInY, int lane, double *sx, double *sy,
                                      int *sok, double ext[4], double &psx, double &psy, int &nPixels,
                                      int &nLines, const GEdge *ge = nullptr) {
  const double dfStep = 1.0 / kSteps;
  int ns = 4 * (kSteps + 1);
  if (ge && ge->n_fail == 0) {   // shared georeferenced samples: only this tile's inverse geotransform
    const double *g2 = t.dst_igt;
    for (int k = lane; k < ns; k += 64) {
      const double X = ge->x[k], Y = ge->y[k];
      sx[k] = g2[0] + X * g2[1] + Y * g2[2];
      sy[k] = g2[3] + X * g2[4] + Y * g2[5];
      sok[k] = 1;
    }
  } else for (int k = lane; k < ns; k += 64) {
    int i = k >> 2, e = k & 3;
    double r = (i == kSteps) ? 1.0 : i * dfStep;
    double x, y;
    if (e == 0) { x = r * nInX; y = 0.0; }
    else if (e == 1) { x = r * nInX; y = nInY; }
    else if (e == 2) { x = 0.0; y = r * nInY; }
    else { x = nInX; y = r * nInY; }
    int ok = xform_point_nl(t, false, x, y);
    sx[k] = x; sy[k] = y; sok[k] = ok;
  }
  __syncthreads();
  int failed = 0;
  for (int k = lane; k < ns; k += 64) failed += sok[k] ? 0 : 1;
  for (int o = 32; o > 0; o >>= 1) failed += __shfl_xor(failed, o, 64);
  if (failed > 0) {  // full grid of the source raster
    __syncthreads();
    ns = kGrid;
    for (int k = lane; k < ns; k += 64) {
      int iy = k / (kSteps + 1), ix = k % (kSteps + 1);
      double ry = (iy == kSteps) ? 1.0 : iy * dfStep;
      double rx = (ix == kSteps) ? 1.0 : ix * dfStep;
      double x = rx * nInX, y = ry * nInY;
      int ok = xform_point_nl(t, false, x, y);
      sx[k] = x; sy[k] = y; sok[k] = ok;
    }
    __syncthreads();
  }
  double mnx = INFINITY, mny = INFINITY, mxx = -INFINITY, mxy = -INFINITY;
  int got = 0;
  for (int k = lane; k < ns; k += 64) {
    if (!sok[k]) continue;
    got = 1;
    mnx = fmin(mnx, sx[k]); mny = fmin(mny, sy[k]);
    mxx = fmax(mxx, sx[k]); mxy = fmax(mxy, sy[k]);
  }
  mnx = wave_min(mnx); mny = wave_min(mny); mxx = wave_max(mxx); mxy = wave_max(mxy);
  got = __ballot(got) != 0ull;

  int err = 1;
  ext[0] = ext[1] = ext[2] = ext[3] = 0.0;
  psx = 0.0; psy = 0.0;
  nPixels = 0; nLines = 0;
  if (got) {
    double dX = 0, dY = 0;
    if (sok[0] && sok[ns - 1]) { dX = sx[ns - 1] - sx[0]; dY = sy[ns - 1] - sy[0]; }
    if (dX == 0.0 || dY == 0.0) { dX = mxx - mnx; dY = mxy - mny; }
    const double diag = sqrt(dX * dX + dY * dY);
    const double ps = diag / sqrt((double)nInX * nInX + (double)nInY * nInY);
    const double dfPixels = (mxx - mnx) / ps;
    const double dfLines = (mxy - mny) / ps;
    if (dfPixels <= 2147483646.0 && dfLines <= 2147483646.0) {
      err = 0;
      nPixels = (int)(dfPixels + 0.5);
      nLines = (int)(dfLines + 0.5);
      psx = ps; psy = ps;
      const double ratios[5] = {0.000, 0.001, 0.010, 0.100, 1.000};
      // first trial of both borders in one pass of the wave: the bottom test
      // assumes the right border keeps psx (trial 0 leaves it unchanged:
      // psx - psx * 0 / nPixels == psx), which holds whenever the right test
      // passes at trial 0 -- the common case; otherwise the reference's
      // sequential loops run from where the speculation stopped
      int kx0 = 0, ky0 = 0;
      bool xdone = false, ydone = false;
      {
        const double tryx = psx - psx * ratios[0] / nPixels;
        const double tryy = psy - psy * ratios[0] / nLines;
        const double er[4] = {mnx, mxy - nLines * psy, mnx + nPixels * tryx, mxy};
        const double eb[4] = {mnx, mxy - nLines * tryy, mnx + nPixels * tryx, mxy};
        const int adj = must_adjust2(t, er, tryx, psy, eb, tryx, tryy, nPixels, nLines, lane);
        kx0 = 1;
        if (!(adj & 1)) {
          psx = tryx;
          xdone = true;
          ky0 = 1;
          if (!(adj & 2)) { psy = tryy; ydone = true; }
        }
      }
      for (int k = kx0; k < 5 && !xdone; k++) {
        const double tryx = psx - psx * ratios[k] / nPixels;
        double e[4] = {mnx, mxy - nLines * psy, mnx + nPixels * tryx, mxy};
        if (!must_adjust(t, e, nPixels, nLines, tryx, psy, true, lane)) { psx = tryx; break; }
      }
      for (int k = ky0; k < 5 && !ydone; k++) {
        const double tryy = psy - psy * ratios[k] / nLines;
        double e[4] = {mnx, mxy - nLines * tryy, mnx + nPixels * psx, mxy};
        if (!must_adjust(t, e, nPixels, nLines, psx, tryy, false, lane)) { psy = tryy; break; }
      }
      ext[0] = mnx;
      ext[1] = mxy - nLines * psy;
      ext[2] = mnx + nPixels * psx;
      ext[3] = mxy;
    }
  }
  return err;
}

// One border-test sample j of GDALSuggestedWarpOutput2_MustAdjustFor{Right,
// Bottom}Border: the per-lane expressions of must_adjust().
// INL: the transforms inlined (workgroup planning of small batches, where a
// call's register save / restore through scratch sits on the latency path).
template <bool INL = false>
__device__ bool border_bad(const Xform &t, const double *ext, int np, int nl, double psx, double psy, bool right,
                           int j) {
  double r1 = 0.0, r2 = 0.0;
  for (int k = 0; k < j; k++) {
    r1 += 0.05;
    r2 += 0.05;
  }
  if (r1 > 0.99) r1 = 1.0;
  double ax, ay;
  if (right) { ax = ext[2]; ay = ext[3] - psy * r1 * nl; }
  else { ax = ext[0] + psx * r1 * np; ay = ext[1]; }
  bool ok1, ok2;
  if constexpr (INL) {
    ok1 = xform_point(t, true, ax, ay);
    ok2 = ok1 ? xform_point(t, false, ax, ay) : false;
  } else {
    ok1 = xform_point_nl(t, true, ax, ay);
    ok2 = ok1 ? xform_point_nl(t, false, ax, ay) : false;
  }
  const double ex = right ? ext[2] : ext[0] + psx * r2 * np;
  const double ey = right ? ext[3] - psy * r2 * nl : ext[1];
  return !ok1 || !ok2 || fabs(ax - ex) > psx || fabs(ay - ey) > psy;
}

#ifdef GSKYHIP_AB
// phase stamps of plan_pair<256> inside plan_small_kernel (GSKYHIP_PLAN_STAMPS)
__device__ __forceinline__ void pstamp(uint64_t *ps, int i) { if (ps && threadIdx.x == 0) ps[i] = wall_clock64(); }
#define PSTAMP(ps, i) pstamp(ps, i)
#else
#define PSTAMP(ps, i) ((void)0)
#endif

// suggested_warp_output2() by a workgroup of NT threads (small batches, where
// the planning chain is latency-bound): the 21 x 21 grid in kGrid / NT rounds
// instead of kGrid / 64, and the border trials side by side -- the five right
// trials plus the bottom trial 0 (valid when the right border keeps trial 0)
// in one pass, the remaining bottom trials in a second; the reference takes
// the first trial that passes, which is what each pass picks.  Same
// expressions per sample, so the same results.
template <int NT>
__device__ int suggested_warp_output2_blk(const Xform &t, int nInX, int nInY, double *sx, double *sy, int *sok,
                                          double ext[4], double &psx, double &psy, int &nPixels, int &nLines,
                                          const GEdge *ge, uint64_t *stp = nullptr) {
  constexpr int kW = NT / 64;
  __shared__ double s_red[4][kW];
  __shared__ int s_cnt[8];
  const int tid = threadIdx.x, w = tid >> 6;
  const double dfStep = 1.0 / kSteps;
  int ns = 4 * (kSteps + 1);
  if (ge && ge->n_fail == 0) {
    const double *g2 = t.dst_igt;
    for (int k = tid; k < ns; k += NT) {
      const double X = ge->x[k], Y = ge->y[k];
      sx[k] = g2[0] + X * g2[1] + Y * g2[2];
      sy[k] = g2[3] + X * g2[4] + Y * g2[5];
      sok[k] = 1;
    }
  }
  // the grid point (ix, iy) of the 21 x 21 fallback, source pixel coordinates
  auto grid_xy = [&](int ix, int iy, double &x, double &y) {
    const double ry = (iy == kSteps) ? 1.0 : iy * dfStep;
    const double rx = (ix == kSteps) ? 1.0 : ix * dfStep;
    x = rx * nInX; y = ry * nInY;
  };
  constexpr int kEdge = 4 * (kSteps + 1), kInner = (kSteps - 1) * (kSteps - 1);
  constexpr bool kSpec = NT >= kEdge;   // one edge sample per thread: the rest speculate on the grid
  double gx = 0.0, gy = 0.0;            // this thread's edge sample / speculative interior point
  int gok = 0;
  if (!(ge && ge->n_fail == 0)) {
    if constexpr (kSpec) {
      if (tid < kEdge) {
        const int i = tid >> 2, e = tid & 3;
        const double r = (i == kSteps) ? 1.0 : i * dfStep;
        double x, y;
        if (e == 0) { x = r * nInX; y = 0.0; }
        else if (e == 1) { x = r * nInX; y = nInY; }
        else if (e == 2) { x = 0.0; y = r * nInY; }
        else { x = nInX; y = r * nInY; }
        gok = xform_point(t, false, x, y);
        gx = x; gy = y;
        sx[tid] = x; sy[tid] = y; sok[tid] = gok;
      } else if (tid - kEdge < kInner) {   // interior point j of the grid, in case an edge sample fails
        const int j = tid - kEdge;
        double x, y;
        grid_xy(1 + j % (kSteps - 1), 1 + j / (kSteps - 1), x, y);
        gok = xform_point(t, false, x, y);
        gx = x; gy = y;
      }
    } else {
      for (int k = tid; k < ns; k += NT) {
        const int i = k >> 2, e = k & 3;
        const double r = (i == kSteps) ? 1.0 : i * dfStep;
        double x, y;
        if (e == 0) { x = r * nInX; y = 0.0; }
        else if (e == 1) { x = r * nInX; y = nInY; }
        else if (e == 2) { x = 0.0; y = r * nInY; }
        else { x = nInX; y = r * nInY; }
        const int ok = xform_point(t, false, x, y);
        sx[k] = x; sy[k] = y; sok[k] = ok;
      }
    }
  }
  __syncthreads();
  PSTAMP(stp, 2);
  int failed = 0;
  for (int k = tid; k < ns; k += NT) failed |= sok[k] ? 0 : 1;
  if (__syncthreads_or(failed)) {   // full grid of the source raster
    if constexpr (kSpec) {
      // the edge samples are the grid's boundary points (the same expressions
      // of the same coordinates), the first interior points were speculated:
      // place both, transform the remaining interior points
      if (tid < kEdge) {
        const int i = tid >> 2, e = tid & 3;
        const int g = e == 0 ? i : e == 1 ? kSteps * (kSteps + 1) + i : e == 2 ? i * (kSteps + 1)
                                                                                  : i * (kSteps + 1) + kSteps;
        sx[g] = gx; sy[g] = gy; sok[g] = gok;   // corners: two equal writes
      } else if (tid - kEdge < kInner) {
        const int j = tid - kEdge;
        const int g = (1 + j / (kSteps - 1)) * (kSteps + 1) + 1 + j % (kSteps - 1);
        sx[g] = gx; sy[g] = gy; sok[g] = gok;
      }
      for (int j = NT - kEdge + tid; j < kInner; j += NT) {
        double x, y;
        const int ix = 1 + j % (kSteps - 1), iy = 1 + j / (kSteps - 1);
        grid_xy(ix, iy, x, y);
        const int ok = xform_point(t, false, x, y);
        const int g = iy * (kSteps + 1) + ix;
        sx[g] = x; sy[g] = y; sok[g] = ok;
      }
    } else {
      for (int k = tid; k < kGrid; k += NT) {
        const int iy = k / (kSteps + 1), ix = k % (kSteps + 1);
        double x, y;
        grid_xy(ix, iy, x, y);
        const int ok = xform_point(t, false, x, y);
        sx[k] = x; sy[k] = y; sok[k] = ok;
      }
    }
    ns = kGrid;
    __syncthreads();
  }
  double mnx = INFINITY, mny = INFINITY, mxx = -INFINITY, mxy = -INFINITY;
  int got = 0;
  for (int k = tid; k < ns; k += NT) {
    if (!sok[k]) continue;
    got = 1;
    mnx = fmin(mnx, sx[k]); mny = fmin(mny, sy[k]);
    mxx = fmax(mxx, sx[k]); mxy = fmax(mxy, sy[k]);
  }
  mnx = wave_min(mnx); mny = wave_min(mny); mxx = wave_max(mxx); mxy = wave_max(mxy);
  if ((tid & 63) == 0) { s_red[0][w] = mnx; s_red[1][w] = mny; s_red[2][w] = mxx; s_red[3][w] = mxy; }
  got = __syncthreads_or(got);
  for (int i = 0; i < kW; i++) {
    mnx = fmin(mnx, s_red[0][i]); mny = fmin(mny, s_red[1][i]);
    mxx = fmax(mxx, s_red[2][i]); mxy = fmax(mxy, s_red[3][i]);
  }
  int err = 1;
  ext[0] = ext[1] = ext[2] = ext[3] = 0.0;
  psx = 0.0; psy = 0.0;
  nPixels = 0; nLines = 0;
  if (!got) return err;
  double dX = 0, dY = 0;
  if (sok[0] && sok[ns - 1]) { dX = sx[ns - 1] - sx[0]; dY = sy[ns - 1] - sy[0]; }
  if (dX == 0.0 || dY == 0.0) { dX = mxx - mnx; dY = mxy - mny; }
  const double diag = sqrt(dX * dX + dY * dY);
  const double ps = diag / sqrt((double)nInX * nInX + (double)nInY * nInY);
  const double dfPixels = (mxx - mnx) / ps;
  const double dfLines = (mxy - mny) / ps;
  if (!(dfPixels <= 2147483646.0 && dfLines <= 2147483646.0)) return err;
  err = 0;
  nPixels = (int)(dfPixels + 0.5);
  nLines = (int)(dfLines + 0.5);
  psx = ps; psy = ps;
  const double ratios[5] = {0.000, 0.001, 0.010, 0.100, 1.000};
  // pass A: right trials 0..4 (tests 0..4), bottom trial 0 under right trial 0 (test 5)
  if (tid < 8) s_cnt[tid] = 0;
  __syncthreads();
  PSTAMP(stp, 3);
  const double tryx0 = psx - psx * ratios[0] / nPixels;
  const double tryy0 = psy - psy * ratios[0] / nLines;
  if (tid < 6 * 21) {
    const int id = tid / 21, j = tid % 21;
    bool bad;
    if (id < 5) {
      const double tryx = psx - psx * ratios[id] / nPixels;
      const double e[4] = {mnx, mxy - nLines * psy, mnx + nPixels * tryx, mxy};
      bad = border_bad<true>(t, e, nPixels, nLines, tryx, psy, true, j);
    } else {
      const double e[4] = {mnx, mxy - nLines * tryy0, mnx + nPixels * tryx0, mxy};
      bad = border_bad<true>(t, e, nPixels, nLines, tryx0, tryy0, false, j);
    }
    if (bad) atomicAdd(&s_cnt[id], 1);
  }
  __syncthreads();
  PSTAMP(stp, 4);
  int kx = -1;
  for (int k = 0; k < 5; k++)
    if (s_cnt[k] != 21) { kx = k; break; }
  if (kx >= 0) psx = psx - psx * ratios[kx] / nPixels;
  int ky0 = 0;
  bool ydone = false;
  if (kx == 0) {
    ky0 = 1;
    if (s_cnt[5] != 21) { psy = tryy0; ydone = true; }
  }
  if (!ydone) {   // pass B: bottom trials ky0..4 under the final psx
    __syncthreads();
    if (tid < 8) s_cnt[tid] = 0;
    __syncthreads();
    if (tid < (5 - ky0) * 21) {
      const int k = ky0 + tid / 21, j = tid % 21;
      const double tryy = psy - psy * ratios[k] / nLines;
      const double e[4] = {mnx, mxy - nLines * tryy, mnx + nPixels * psx, mxy};
      if (border_bad<true>(t, e, nPixels, nLines, psx, tryy, false, j)) atomicAdd(&s_cnt[k], 1);
    }
    __syncthreads();
    for (int k = ky0; k < 5; k++)
      if (s_cnt[k] != 21) { psy = psy - psy * ratios[k] / nLines; break; }
  }
  ext[0] = mnx;
  ext[1] = mxy - nLines * psy;
  ext[2] = mnx + nPixels * psx;
  ext[3] = mxy;
  return err;
}

// Plan of pair p by one workgroup of NT threads (sx / sy / sok: LDS scratch
// of kGrid entries, ts: the transformer in LDS).
template <int NT>
__device__ void plan_pair(const PlanArgs &a, int p, double *sx, double *sy, int *sok, Xform &ts,
                          uint64_t *ps = nullptr) {
  const int lane = threadIdx.x;
  PSTAMP(ps, 0);
  const int t_idx = a.small ? owning_tile(a.tiles, a.n_tiles, p) : a.pair_tile[p];
  if (t_idx < 0) {   // unreferenced pair: an empty plan nothing reads
    if (lane == 0) {
      PairPlan z = {};
      z.tile = -1;
      z.mask_pair = -1;
      a.pairs[p] = z;
    }
    return;
  }
  const gskyhip_tile &tile = a.tiles[t_idx];
  const int gi = a.pair_granule[p];
  const gskyhip_granule &g = a.granules[gi];
  Xform &xf = a.xforms[p];
  PairPlan &pp = a.pairs[p];

  // ---- transformer (warp.go:120-148), kept in LDS: the wave-uniform state
  // would otherwise live in scratch (xform_point selects its geotransforms
  // through pointers) or cost ~130 VGPRs
  Xform &t = ts;
  {   // set up by the lanes side by side (round 3 had lane 0 copy ~90 words
      // and invert both geotransforms in series): work item w < 2 kCw is a
      // word of the two CRS records, then 6 + 6 geotransform words, the two
      // inverses (from global) and the reprojection flag / geolocation arrays
    static_assert(sizeof(gskyhip_crs) % 8 == 0, "crs words");
    constexpr int kCw = (int)(sizeof(gskyhip_crs) / 8);   // 43 words
    const int dsti = a.dst_crs >= 0 ? a.dst_crs : g.crs;
    for (int w = lane; w < 2 * kCw + 15; w += NT) {
      if (w < kCw) {
        ((uint64_t *)&t.src)[w] = ((const uint64_t *)&a.crs[g.crs])[w];
      } else if (w < 2 * kCw) {
        ((uint64_t *)&t.dst)[w - kCw] = ((const uint64_t *)&a.crs[dsti])[w - kCw];
      } else if (w < 2 * kCw + 6) {
        t.src_gt[w - 2 * kCw] = g.geot[w - 2 * kCw];
      } else if (w < 2 * kCw + 12) {
        t.dst_gt[w - 2 * kCw - 6] = tile.dst_geot[w - 2 * kCw - 6];
      } else if (w == 2 * kCw + 12) {
        double gt[6];
        for (int k = 0; k < 6; k++) gt[k] = g.geot[k];
        inv_geot(gt, t.src_igt);
      } else if (w == 2 * kCw + 13) {
        double gt[6];
        for (int k = 0; k < 6; k++) gt[k] = tile.dst_geot[k];
        inv_geot(gt, t.dst_igt);
      } else if (w == 2 * kCw + 14) {
        t.gl = (g.geoloc > 0 && a.geolocs) ? a.geolocs + (g.geoloc - 1) : nullptr;
        t.reproject = a.dst_crs >= 0 ? (crs_same(a.crs[g.crs], a.crs[a.dst_crs]) ? 0 : 1) : 0;
      }
    }
  }
  __syncthreads();
  PSTAMP(ps, 1);

  // ---- GDALSuggestedWarpOutput2 (warp.go:154)
  const int nInX = g.xsize, nInY = g.ysize;
  double ext[4], psx, psy;
  int nPixels, nLines;
  int err;
  if constexpr (NT == 64)
    err = suggested_warp_output2(t, nInX, nInY, lane, sx, sy, sok, ext, psx, psy, nPixels, nLines,
                                 a.gedge ? a.gedge + gi : nullptr);
  else
    err = suggested_warp_output2_blk<NT>(t, nInX, nInY, sx, sy, sok, ext, psx, psy, nPixels, nLines,
                                         a.gedge ? a.gedge + gi : nullptr, ps);
  PSTAMP(ps, 5);
  if (lane != 0) return;

  // ---- overview pick (warp.go:156-198)
  const void *band = g.data;
  int bandX = g.xsize, bandY = g.ysize;
  if (!t.gl && err == 0 && g.n_ovr > 0) {   // never with geolocation arrays (warp.go:158)
    const double targetRatio = 1.0 / psx;
    if (targetRatio > 1.0) {
      int iOvr = -1;
      for (; iOvr < g.n_ovr - 1; iOvr++) {
        double ovrRatio = 1.0;
        if (iOvr >= 0) ovrRatio = (double)nInX / g.ovr_xsize[iOvr];
        const double nextOvrRatio = (double)nInX / g.ovr_xsize[iOvr + 1];
        if (ovrRatio < targetRatio && nextOvrRatio > targetRatio) break;
        const double diff = ovrRatio - targetRatio;
        if (diff > -1e-1 && diff < 1e-1) break;
      }
      if (iOvr >= 0) {
        band = g.ovr_data[iOvr];
        bandX = g.ovr_xsize[iOvr];
        bandY = g.ovr_ysize[iOvr];
        t.src_gt[1] *= nInX / (double)bandX;
        t.src_gt[2] *= nInX / (double)bandX;
        t.src_gt[4] *= nInY / (double)bandY;
        t.src_gt[5] *= nInY / (double)bandY;
        inv_geot(t.src_gt, t.src_igt);
      }
    }
  }

  // ---- window (warp.go:200-217; roundCoord 69-80)
  auto round_coord = [](double c, int maxExtent) {
    int r;
    if (c < 0) r = 0;
    else {
      r = (int)(c + 1e-10);
      if (r > maxExtent - 1) r = maxExtent - 1;
    }
    return r;
  };
  int xoff = 0, yoff = 0, w = tile.width, h = tile.height;
  const bool fits = tile.width > 0 && tile.height > 0 && tile.width <= a.max_w && tile.height <= a.max_h;
  if (!fits) { w = 0; h = 0; err = 1; }
  if (err == 0) {
    const int minX = round_coord(ext[0], w), minY = round_coord(ext[1], h);
    const int maxX = round_coord(ext[2] + 0.5, w), maxY = round_coord(ext[3] + 0.5, h);
    xoff = minX; yoff = minY;
    w = maxX - minX + 1;
    h = maxY - minY + 1;
  }

  xf = t;
  for (int k = 0; k < 6; k++) { pp.src_gt[k] = t.src_gt[k]; pp.src_igt[k] = t.src_igt[k]; }
  pp.band = band;
  pp.band_x = bandX; pp.band_y = bandY;
  pp.xoff = xoff; pp.yoff = yoff; pp.w = w; pp.h = h;
  pp.granule = gi; pp.tile = t_idx;
  pp.src_dtype = g.dtype;
  const bool supported = g.dtype == GSKYHIP_BYTE || g.dtype == GSKYHIP_INT16 ||
                         g.dtype == GSKYHIP_UINT16 || g.dtype == GSKYHIP_FLOAT32;
  int odt = supported ? g.dtype : GSKYHIP_FLOAT32;
  pp.signed_byte = (odt == GSKYHIP_BYTE && g.signed_byte) ? 1 : 0;
  if (pp.signed_byte) odt = GSKYHIP_SIGNEDBYTE;
  pp.out_dtype = odt;
  pp.ns = g.ns;
  pp.is_mask = (a.mask_ns >= 0 && g.ns == a.mask_ns) ? 1 : 0;
  pp.in_stack = (!pp.is_mask || a.mask_inclusive) ? 1 : 0;
  pp.fill_mode = 0;
  pp.mask_pair = -1;
  pp.status = fits ? 0 : GSKYHIP_E_ARG;
  pp.nodata = g.nodata;
  pp.has_nodata = g.has_nodata;
  pp.fill = gdal_copy_to(g.nodata, odt);
  pp.ts = g.timestamp;
  pp.stamp = g.timestamp + (double)g.polygon_hash;
}

// One workgroup of NT threads per pair: NT = 64 (one wavefront) for batches
// that fill the GPU, NT = 256 for small, latency-bound batches.
template <int NT>
__global__ __launch_bounds__(NT) void plan_pairs_kernel(PlanArgs a) {
  if ((int)blockIdx.x >= a.n_pairs) return;
  __shared__ double sx[kGrid], sy[kGrid];
  __shared__ int sok[kGrid];
  __shared__ Xform ts;
  plan_pair<NT>(a, blockIdx.x, sx, sy, sok, ts);
}

// ---------------------------------------------------------------- extent op
// ComputeReprojectExtent (worker/gdalprocess/warp.go:433-487), one wavefront
// per granule: GDALCreateGenImgProjTransformer(src, dst SRS, no dst dataset)
// maps source pixels to destination georeferenced coordinates (identity
// destination geotransform), GDALSuggestedWarpOutput = SuggestedWarpOutput2
// with nOptions 0, then the request's pixel counts for its bbox
// (xMin, yMin, xMax, yMax) = DstGeot[0..3] at the suggested resolution:
//   nPixels = int((xMax - xMin + xRes/2) / xRes), nLines likewise.
__global__ __launch_bounds__(64) void extent_kernel(const gskyhip_granule *granules, int n, const gskyhip_crs *crs,
                                                    int dst_crs, const double *bbox, int32_t *out, int32_t *status) {
  const int i = blockIdx.x;
  const int lane = threadIdx.x;
  if (i >= n) return;
  __shared__ double sx[kGrid], sy[kGrid];
  __shared__ int sok[kGrid];
  const gskyhip_granule &g = granules[i];
  Xform t;
  t.src = crs[g.crs];
  t.gl = nullptr;   // ComputeReprojectExtent: no geolocation arrays (warp.go:433-487)
  t.reproject = 0;
  if (dst_crs >= 0) {
    t.dst = crs[dst_crs];
    t.reproject = crs_same(t.src, t.dst) ? 0 : 1;
  } else {
    t.dst = t.src;
  }
  const double ident[6] = {0.0, 1.0, 0.0, 0.0, 0.0, 1.0};
  for (int k = 0; k < 6; k++) { t.src_gt[k] = g.geot[k]; t.dst_gt[k] = ident[k]; }
  inv_geot(t.src_gt, t.src_igt);
  inv_geot(t.dst_gt, t.dst_igt);
  double ext[4], psx, psy;
  int nPixels, nLines;
  const int err = suggested_warp_output2(t, g.xsize, g.ysize, lane, sx, sy, sok, ext, psx, psy, nPixels, nLines);
  if (lane != 0) return;
  if (err) {
    out[2 * i] = 0; out[2 * i + 1] = 0;
    status[i] = GSKYHIP_E_XFORM;   // "GDALSuggestedWarpOutput() failed"
    return;
  }
  const double xRes = psx, yRes = fabs(-psy);   // padfGeoTransformOut[1], |padfGeoTransformOut[5]|
  const double *bb = bbox + 4 * i;
  out[2 * i] = (int32_t)go_cvtt64((bb[2] - bb[0] + xRes / 2.0) / xRes);
  out[2 * i + 1] = (int32_t)go_cvtt64((bb[3] - bb[1] + yRes / 2.0) / yRes);
  status[i] = 0;
}

int launch_extent(const gskyhip_granule *granules, int n, const gskyhip_crs *crs, int dst_crs, const double *bbox,
                  int32_t *out, int32_t *status, hipStream_t s) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(extent_kernel, dim3((unsigned)n), dim3(64), 0, s, granules, n, crs, dst_crs, bbox, out, status);
  return hipGetLastError() == hipSuccess ? 0 : GSKYHIP_E_HIP;
}

// ---------------------------------------------------------------- merge order
// Entry descriptor of pair p (render kernels) and its value-type vote: the
// typed band kernels need one value type, no GDALCopyWords promotion and a
// band addressable with 32-bit offsets.  Returns -1 (not merged), 0 (no) or
// the value type.
__device__ __forceinline__ int write_entry(const PlanArgs &a, int p) {
  const PairPlan &pp = a.pairs[p];
  EntryD d;
  d.band = pp.band;
  d.band_x = pp.band_x; d.band_y = pp.band_y;
  d.xoff = pp.xoff; d.yoff = pp.yoff; d.w = pp.w; d.h = pp.h;
  d.ns = pp.ns; d.fill_mode = pp.fill_mode; d.mask_pair = pp.mask_pair; d.src_dtype = pp.src_dtype;
  d.out_dtype = pp.out_dtype; d.has_nodata = pp.has_nodata;
  d.nd = go_conv_to(pp.nodata, pp.out_dtype);
  d.fill = pp.fill;
  d.nodata64 = pp.nodata;
  d.row_base = (int64_t)p * a.max_h;
  a.entries[p] = d;
  if (!pp.in_stack) return -1;
  const bool same = pp.src_dtype == pp.out_dtype ||
                    (pp.src_dtype == GSKYHIP_BYTE && pp.out_dtype == GSKYHIP_SIGNEDBYTE);
  const bool small = pp.band_x < (1 << 24) && pp.band_y < (1 << 24) &&
                     (int64_t)pp.band_x * pp.band_y * type_size(pp.src_dtype) < 2147483648LL;
  return (same && small) ? pp.out_dtype : 0;
}

// Mirrors RasterMerger.Run for the tile's batch, one thread (tiles with more
// than kWavePairs pairs; plan_tiles_kernel below is the wave-parallel form).
__device__ void plan_tile_serial(const PlanArgs &a, int t) {
  const gskyhip_tile &tile = a.tiles[t];
  TilePlan tp;
  tp.n_entries = 0;
  tp.status = 0;
  tp.complex = 0;
  tp.vt = 0;
  tp.e0 = -1;
  tp._pad = 0;
  double canvas_ts[4];
  for (int k = 0; k < 4; k++) { tp.created[k] = 0; tp.dtype[k] = 0; tp.nodata[k] = 0; canvas_ts[k] = 0; }
  const int b = tile.pair_begin, e = tile.pair_end;
  int32_t *ord = a.order + b;
  if (tile.width <= 0 || tile.height <= 0 || tile.width > a.max_w || tile.height > a.max_h) {
    tp.status = GSKYHIP_E_ARG;   // outside the batch's max_h x max_w slot
    tp.complex = 1;              // no render kernel touches it
    a.tplans[t] = tp;
    return;
  }
  // stack entries; stable insertion sort by geoStamp descending (keys sorted
  // descending, rasters of one key in arrival order: tile_merger.go:286-290)
  int n = 0;
  for (int p = b; p < e; p++) {
    if (!a.pairs[p].in_stack) continue;
    const double s = a.pairs[p].stamp;
    int j = n;
    while (j > 0 && a.pairs[ord[j - 1]].stamp < s) { ord[j] = ord[j - 1]; j--; }
    ord[j] = p;
    n++;
  }
  tp.n_entries = n;
  tp.e0 = n > 0 ? ord[0] : -1;
  for (int k = 0; k < n; k++) {
    PairPlan &pp = a.pairs[ord[k]];
    // maskMap[geoStamp]: the last mask raster of that key (tile_merger.go:478-484)
    int mp = -1;
    for (int q = b; q < e; q++)
      if (a.pairs[q].is_mask && a.pairs[q].stamp == pp.stamp) mp = q;
    pp.mask_pair = mp;
    if (mp >= 0) {
      const PairPlan &mq = a.pairs[mp];
      const int mdt = mq.out_dtype;
      if (!(mdt == GSKYHIP_SIGNEDBYTE || mdt == GSKYHIP_BYTE || mdt == GSKYHIP_INT16 || mdt == GSKYHIP_UINT16))
        tp.status = GSKYHIP_E_MASK;       // "Type %s cannot contain a bit mask"
      else if ((long)pp.w * pp.h > (long)mq.w * mq.h)
        tp.status = GSKYHIP_E_RANGE;      // mask[iSrc] out of range: Go panics
    }
    const int ns = pp.ns;
    if (ns < 0 || ns >= 4) { tp.status = GSKYHIP_E_RANGE; continue; }
    if (!tp.created[ns]) {  // tile_merger.go:291-297
      tp.created[ns] = 1;
      tp.dtype[ns] = pp.out_dtype;
      tp.nodata[ns] = pp.nodata;
      canvas_ts[ns] = 0;
    } else if (tp.dtype[ns] != pp.out_dtype) {
      tp.status = GSKYHIP_E_TYPE;  // the reference would reinterpret the canvas bytes
    }
    pp.fill_mode = pp.ts < canvas_ts[ns] ? 1 : 0;  // tile_merger.go:47
    if (!pp.fill_mode) canvas_ts[ns] = pp.ts;
  }
  // render descriptors of every pair of the tile (mask pairs included)
  int vt = -1;
  for (int p = b; p < e; p++) {
    const int v = write_entry(a, p);
    if (v == 0) vt = 0;
    else if (v > 0 && vt < 0) vt = v;
    else if (v > 0 && vt != v) vt = 0;
  }
  tp.vt = vt < 0 ? 0 : vt;
  // mixed types or promotion: the general kernel renders the tile; a tile
  // with no entry at all is written (transparent / zero canvas) by whichever
  // band kernel the batch launches (n_entries == 0 passes their type test)
  if (n > 0 && tp.vt == 0) {
    tp.complex = 1;
    const int k = atomicAdd(&a.counters[2], 1);
    a.complex_list[k] = t;
  }
  a.tplans[t] = tp;
}


constexpr int kWavePairs = 256;   // pairs per tile the wave-parallel merge planner holds in registers
constexpr int kTileSlots = kWavePairs / 64;

// One wavefront per tile: RasterMerger.Run's merge order (tile_merger.go:281-312:
// stable sort by geoStamp descending), maskMap links (478-484), canvas
// creation and the fill / overwrite mode of MergeMaskedRaster (47), as data-
// parallel passes over the tile's pairs instead of the serial walk:
//   rank(p)   = #{q: stamp_q > stamp_p} + #{q < p: stamp_q == stamp_p}
//   fill(k)   = ts_k < max(0, max{ts_j: j before k in the order, same ns})
//   status    = the last error in merge order (the serial walk's last write).
// Lane l holds pairs l, l + 64, ... in registers; each pass walks the tile's
// pairs q in index order, q's values read out of its lane (v_readlane), and
// every lane updates its own pairs -- no memory access inside the passes
// (round 6: the LDS form's dependent loads took 70 us for C5's 128-pair
// tiles).
__device__ __forceinline__ double readlane_d(double v, int l) {
  const uint64_t u = (uint64_t)__double_as_longlong(v);
  const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)u, l), hi = __builtin_amdgcn_readlane((uint32_t)(u >> 32), l);
  return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}

// Synchronisation of the 64 lanes of one wavefront: its global accesses are
// performed in program order, so this only keeps the compiler from moving
// memory operations across it.
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// The per-wave partials of the passes when NW waves share a tile (wave w
// walks the pairs q = w, w + NW, ... of each register slot).
template <int NW>
struct TileRed {
  int32_t rk[NW][kWavePairs], mp[NW][kWavePairs], fk[NW][kWavePairs], fdt[NW][kWavePairs];
  double cts[NW][kWavePairs];
};

template <int NW>
__device__ __forceinline__ void plan_tile_waves(const PlanArgs &a, int t, int w, int lane, TileRed<NW> *red) {
  const gskyhip_tile &tile = a.tiles[t];
  const int b = tile.pair_begin, e = tile.pair_end, np = e - b;
  const bool bad_size = tile.width <= 0 || tile.height <= 0 || tile.width > a.max_w || tile.height > a.max_h;
  if (np > kWavePairs || bad_size) {
    if (w == 0 && lane == 0) plan_tile_serial(a, t);
    return;
  }
  const int S = (np + 63) >> 6;   // register slots in use
  double st[kTileSlots], tsv[kTileSlots];
  int inf[kTileSlots];            // in_stack | is_mask << 1 | (ns + 1) << 2 | out_dtype << 8
#pragma unroll
  for (int j = 0; j < kTileSlots; j++) {
    const int i = 64 * j + lane;
    st[j] = 0.0; tsv[j] = 0.0; inf[j] = 0;
    if (j < S && i < np) {
      const PairPlan &pp = a.pairs[b + i];
      st[j] = pp.stamp;
      tsv[j] = pp.ts;
      inf[j] = (pp.in_stack ? 1 : 0) | (pp.is_mask ? 2 : 0) | ((pp.ns + 1) << 2) | (pp.out_dtype << 8);
    }
  }
  // pass 1: merge rank and maskMap link (the last mask pair of the same key)
  int rk[kTileSlots], mpi[kTileSlots];
#pragma unroll
  for (int j = 0; j < kTileSlots; j++) { rk[j] = 0; mpi[j] = -1; }
#pragma unroll
  for (int jq = 0; jq < kTileSlots; jq++) {
    if (jq >= S) break;
    const int nq = min(64, np - 64 * jq);
#pragma unroll 1
    for (int l = w; l < nq; l += NW) {
      const double sq = readlane_d(st[jq], l);
      const int iq = __builtin_amdgcn_readlane(inf[jq], l);
      const int q = 64 * jq + l;
#pragma unroll
      for (int j = 0; j < kTileSlots; j++) {
        if (j >= S) break;
        const int i = 64 * j + lane;
        rk[j] += ((iq & 1) && (sq > st[j] || (q < i && sq == st[j]))) ? 1 : 0;
        mpi[j] = ((iq & 2) && sq == st[j]) ? q : mpi[j];
      }
    }
  }
  if constexpr (NW > 1) {   // the waves' partial counts and last links, summed / maxed
#pragma unroll
    for (int j = 0; j < kTileSlots; j++) {
      red->rk[w][64 * j + lane] = rk[j];
      red->mp[w][64 * j + lane] = mpi[j];
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kTileSlots; j++) {
      int sr = 0, sm = -1;
#pragma unroll
      for (int v = 0; v < NW; v++) { sr += red->rk[v][64 * j + lane]; sm = max(sm, red->mp[v][64 * j + lane]); }
      rk[j] = sr;
      mpi[j] = sm;
    }
  }
  int n_local = 0;
#pragma unroll
  for (int j = 0; j < kTileSlots; j++) {
    const int i = 64 * j + lane;
    const bool in = j < S && i < np && (inf[j] & 1);
    if (in && w == 0) a.order[b + rk[j]] = b + i;
    rk[j] = in ? rk[j] : -1;
    n_local += in ? 1 : 0;
  }
  for (int o = 32; o > 0; o >>= 1) n_local += __shfl_xor(n_local, o, 64);
  const int n = n_local;
  // pass 2: the canvas timestamp before each entry (running max of its
  // namespace's earlier entries, from 0) and its namespace's first entry
  double cts[kTileSlots];
  int fk[kTileSlots], fdt[kTileSlots];
#pragma unroll
  for (int j = 0; j < kTileSlots; j++) { cts[j] = 0.0; fk[j] = 0x7FFFFFFF; fdt[j] = 0; }
#pragma unroll
  for (int jq = 0; jq < kTileSlots; jq++) {
    if (jq >= S) break;
    const int nq = min(64, np - 64 * jq);
#pragma unroll 1
    for (int l = w; l < nq; l += NW) {
      const int kq = __builtin_amdgcn_readlane(rk[jq], l);
      if (kq < 0) continue;
      const int iq = __builtin_amdgcn_readlane(inf[jq], l);
      const double tq = readlane_d(tsv[jq], l);
#pragma unroll
      for (int j = 0; j < kTileSlots; j++) {
        if (j >= S) break;
        const bool same = ((iq ^ inf[j]) & (63 << 2)) == 0;
        if (same && kq < rk[j]) cts[j] = fmax(cts[j], tq);
        if (same && kq < fk[j]) { fk[j] = kq; fdt[j] = iq >> 8; }
      }
    }
  }
  if constexpr (NW > 1) {   // the waves' partial canvas timestamps and first entries; wave 0 goes on
#pragma unroll
    for (int j = 0; j < kTileSlots; j++) {
      red->cts[w][64 * j + lane] = cts[j];
      red->fk[w][64 * j + lane] = fk[j];
      red->fdt[w][64 * j + lane] = fdt[j];
    }
    __syncthreads();
    if (w != 0) return;
#pragma unroll
    for (int j = 0; j < kTileSlots; j++) {
      for (int v = 1; v < NW; v++) {
        cts[j] = fmax(cts[j], red->cts[v][64 * j + lane]);
        const int k2 = red->fk[v][64 * j + lane];
        if (k2 < fk[j]) { fk[j] = k2; fdt[j] = red->fdt[v][64 * j + lane]; }
      }
    }
  }
  // per merged entry: maskMap link, fill mode, error
  int err_k = -1, err_code = 0;                  // this lane's last error (largest merge position)
  int first_k[4] = {0x7FFFFFFF, 0x7FFFFFFF, 0x7FFFFFFF, 0x7FFFFFFF};
#pragma unroll
  for (int j = 0; j < kTileSlots; j++) {
    const int k = rk[j];
    if (j >= S || k < 0) continue;
    const int i = 64 * j + lane;
    PairPlan &pp = a.pairs[b + i];
    const int mp = mpi[j] >= 0 ? b + mpi[j] : -1;
    pp.mask_pair = mp;
    int st_code = 0;
    if (mp >= 0) {
      const PairPlan &mq = a.pairs[mp];
      const int mdt = mq.out_dtype;
      if (!(mdt == GSKYHIP_SIGNEDBYTE || mdt == GSKYHIP_BYTE || mdt == GSKYHIP_INT16 || mdt == GSKYHIP_UINT16))
        st_code = GSKYHIP_E_MASK;
      else if ((long)pp.w * pp.h > (long)mq.w * mq.h)
        st_code = GSKYHIP_E_RANGE;
    }
    const int ns = ((inf[j] >> 2) & 63) - 1;
    int fill = 0;
    if (ns < 0 || ns >= 4) {
      st_code = GSKYHIP_E_RANGE;
    } else {
      first_k[ns] = min(first_k[ns], k);
      fill = tsv[j] < cts[j] ? 1 : 0;
      if (fk[j] < k && fdt[j] != (inf[j] >> 8)) st_code = GSKYHIP_E_TYPE;
    }
    pp.fill_mode = fill;
    if (st_code && k > err_k) { err_k = k; err_code = st_code; }
  }
  // wave reductions: last error, first entry of each namespace
  for (int o = 32; o > 0; o >>= 1) {
    const int ok_ = __shfl_xor(err_k, o, 64), oc = __shfl_xor(err_code, o, 64);
    if (ok_ > err_k) { err_k = ok_; err_code = oc; }
#pragma unroll
    for (int s2 = 0; s2 < 4; s2++) first_k[s2] = min(first_k[s2], __shfl_xor(first_k[s2], o, 64));
  }
  wave_sync();   // fill_mode / mask_pair of every pair written (same workgroup)
  // render descriptors of every pair (mask pairs included) + value-type vote
  int vmin = 0x7FFFFFFF, vmax = -1;
  bool vzero = false;
  for (int i = lane; i < np; i += 64) {
    const int v = write_entry(a, b + i);
    if (v == 0) vzero = true;
    if (v > 0) { vmin = min(vmin, v); vmax = max(vmax, v); }
  }
  for (int o = 32; o > 0; o >>= 1) {
    vmin = min(vmin, __shfl_xor(vmin, o, 64));
    vmax = max(vmax, __shfl_xor(vmax, o, 64));
  }
  vzero = __ballot(vzero) != 0ull;
  if (lane != 0) return;
  TilePlan tp;
  tp.n_entries = n;
  tp.status = err_code;
  tp.complex = 0;
  tp.e0 = n > 0 ? a.order[b] : -1;
  tp._pad = 0;
  for (int s2 = 0; s2 < 4; s2++) {
    tp.created[s2] = first_k[s2] != 0x7FFFFFFF ? 1 : 0;
    tp.dtype[s2] = 0;
    tp.nodata[s2] = 0;
    if (tp.created[s2]) {
      const PairPlan &pf = a.pairs[a.order[b + first_k[s2]]];
      tp.dtype[s2] = pf.out_dtype;
      tp.nodata[s2] = pf.nodata;
    }
  }
  tp.vt = (vzero || vmax < 0 || vmin != vmax) ? 0 : vmax;
  if (n > 0 && tp.vt == 0) {   // as above: empty tiles go to the band kernel
    tp.complex = 1;
    const int k = atomicAdd(&a.counters[2], 1);
    a.complex_list[k] = t;
  }
  a.tplans[t] = tp;
}

__global__ __launch_bounds__(64) void plan_tiles_kernel(PlanArgs a) {
  const int t = blockIdx.x;
  if (t >= a.n_tiles) return;
  plan_tile_waves<1>(a, t, 0, threadIdx.x, nullptr);
}

// Tiles of many pairs (C5's overview tiles: 34 on average, up to 128): the
// passes of a tile spread over 4 waves (70 -> 37 -> ~20 us on C5; one wave
// per tile stays for batches of few pairs per tile, C2's 1.2).
constexpr int kTiles4MinPairsPerTile = 8;
__global__ __launch_bounds__(256) void plan_tiles4_kernel(PlanArgs a) {
  const int t = blockIdx.x;
  if (t >= a.n_tiles) return;
  __shared__ TileRed<4> red;
  plan_tile_waves<4>(a, t, threadIdx.x >> 6, threadIdx.x & 63, &red);
}

// ---------------------------------------------------------------- row plans
__device__ __forceinline__ void flag_complex(const PlanArgs &a, int tile) {
  if (atomicOr(&a.tplans[tile].complex, 1) == 0) {
    const int k = atomicAdd(&a.counters[2], 1);
    a.complex_list[k] = tile;
  }
}

__device__ __forceinline__ void push_split(const PlanArgs &a, int p, int row) {
  const int k = atomicAdd(&a.counters[1], 1);
  a.split_list[k] = (int64_t)p * a.max_h + row;
}

__device__ __forceinline__ Leaf pending_leaf(int p, int row, int i) {
  Leaf L;
  L.xs0 = 0.0; L.ys0 = 0.0; L.dX = (double)p; L.dY = (double)row;
  L.start = i; L.kind = LEAF_PENDING;
  return L;
}

// Column parts of the separable transform (gsky_device.h) at the three
// columns every row record transforms: first, middle, last.
__device__ __forceinline__ void plan_col(const PlanArgs &a, int64_t gid) {
  const int p = (int)(gid / 3), k = (int)(gid % 3);
  if (p >= a.n_pairs) return;
  const PairPlan &pp = a.pairs[p];
  const Xform &t = a.xforms[p];
  if (!sep_possible(t) || pp.w <= 5 || pp.h <= 0) return;
  const int n = pp.w, nMiddle = (n - 1) / 2;
  const int col = k == 0 ? 0 : (k == 1 ? nMiddle : n - 1);
  a.sepcols[3 * (int64_t)p + k] = sep_col(t, col + 0.5 + pp.xoff, 0.5 + pp.yoff);
}

__global__ __launch_bounds__(256) void plan_cols_kernel(PlanArgs a) {
  plan_col(a, (int64_t)blockIdx.x * blockDim.x + threadIdx.x);
}

// Light pass, one thread per (pair, window row): the three exact points of
// GDALApproxTransform (first / middle / last) and its error test.  Rows whose
// middle error exceeds 0.125 go to the split list (plan_split_kernel).
__device__ __forceinline__ void plan_row(const PlanArgs &a, int p, const PairPlan &pp, const Xform &t, int row) {
  RowRec rec;
  rec.nleaf = 1; rec.pool_off = 0; rec.inside = 0;
  for (int k = 0; k < 6; k++) rec.v[k] = 0;
  const int n = pp.w;
  const int nMiddle = (n - 1) / 2;
  const double yrow = row + 0.5 + pp.yoff;
  // GDALApproxTransform preconditions: y constant, x distinct, nPoints > 5;
  // otherwise every pixel is transformed exactly: the split pass turns the row
  // into per-pixel leaves (plan_exact_kernel) so the tile stays simple
  if (n <= 0) {
    rec.kind = ROW_LINEAR;   // empty window: no pixel reads the record
  } else if (n <= 5) {
    rec.kind = ROW_EXACT;
    push_split(a, p, row);
  } else {
    double xs[3] = {0 + 0.5 + pp.xoff, nMiddle + 0.5 + pp.xoff, (n - 1) + 0.5 + pp.xoff};
    double ys[3] = {yrow, yrow, yrow};
    bool ok0, ok1, ok2;
    if (a.sep && sep_possible(t)) {   // per-column parts from plan_cols_kernel, one row part
      const SepCol *sc = a.sepcols + 3 * (int64_t)p;
      const SepRow sr = sep_row(t, xs[0], yrow);
      double ox, oy;
      ok0 = sep_point(t, sc[0], sr, ox, oy);
      if (ok0) { xs[0] = ox; ys[0] = oy; }
      ok1 = sep_point(t, sc[1], sr, ox, oy);
      if (ok1) { xs[1] = ox; ys[1] = oy; }
      ok2 = sep_point(t, sc[2], sr, ox, oy);
      if (ok2) { xs[2] = ox; ys[2] = oy; }
    } else {
      ok0 = xform_point(t, true, xs[0], ys[0]);
      ok1 = xform_point(t, true, xs[1], ys[1]);
      ok2 = xform_point(t, true, xs[2], ys[2]);
    }
    if (!(ok0 && ok1 && ok2)) {
      rec.kind = ROW_EXACT;
      push_split(a, p, row);
    } else {
      const double x0 = 0 + 0.5 + pp.xoff, xl = (n - 1) + 0.5 + pp.xoff, xm = nMiddle + 0.5 + pp.xoff;
      const double dX = (xs[2] - xs[0]) / (xl - x0);
      const double dY = (ys[2] - ys[0]) / (xl - x0);
      const double dfError = fabs((xs[0] + dX * (xm - x0)) - xs[1]) + fabs((ys[0] + dY * (xm - x0)) - ys[1]);
      if (dfError <= kMaxErr) {
        rec.kind = ROW_LINEAR;
        rec.v[0] = xs[0]; rec.v[1] = ys[0]; rec.v[2] = dX; rec.v[3] = dY;
        rec.inside = linear_row_inside(rec, n, pp.band_x, pp.band_y) ? 1 : 0;
        rec.v[4] = __longlong_as_double(rec.inside ? span_bits(0, n) : linear_row_span(rec, n, pp.band_x, pp.band_y));
      } else {
        rec.kind = ROW_DESCEND;  // provisional: root SME kept for the split pass
        rec.v[0] = xs[0]; rec.v[1] = ys[0]; rec.v[2] = xs[1];
        rec.v[3] = ys[1]; rec.v[4] = xs[2]; rec.v[5] = ys[2];
        push_split(a, p, row);
      }
    }
  }
  a.rows[(long)p * a.max_h + row] = rec;
  a.rowfix[(long)p * a.max_h + row] = row_fix(rec, n, a.resample != GSKYHIP_RESAMPLE_BILINEAR);
}

// Workgroups of one pair (blockIdx.x: pair, blockIdx.y: 256-row chunk): the
// pair's plan and transformer are wave-uniform, so their fields arrive
// through scalar loads rather than per-lane gathers.
__global__ __launch_bounds__(256) void plan_rows_kernel(PlanArgs a) {
  const int p = blockIdx.x;
  const int row = blockIdx.y * blockDim.x + threadIdx.x;
  if (p >= a.n_pairs) return;
  const PairPlan &pp = a.pairs[p];
  if (row >= pp.h) return;
  plan_row(a, p, pp, a.xforms[p], row);
}

struct Node {
  int lo, n;
  double xs[3], ys[3];
  int exact_leaf;  // 1: emit an exact leaf for [lo, lo+n)
};

// GDALApproxTransformInternal recursion (3.0.1) of one row, emitting ordered
// leaves into `out` (capacity kMaxLeavesLocal).  -1 on overflow.
__device__ __noinline__ int approx_leaves(const Xform &t, int xoff, double yrow, int n0, const double *v,
                                          Leaf *out) {
  Node stack[14];
  int sp = 0, nl = 0;
  Node cur;
  cur.lo = 0; cur.n = n0; cur.exact_leaf = 0;
  cur.xs[0] = v[0]; cur.ys[0] = v[1]; cur.xs[1] = v[2]; cur.ys[1] = v[3]; cur.xs[2] = v[4]; cur.ys[2] = v[5];
  auto xpos = [&](int idx) { return idx + 0.5 + xoff; };
  for (;;) {
    if (cur.exact_leaf) {
      if (nl >= kMaxLeavesLocal) return -1;
      out[nl].start = cur.lo; out[nl].kind = 1;
      out[nl].xs0 = out[nl].ys0 = out[nl].dX = out[nl].dY = 0;
      nl++;
    } else {
      const int lo = cur.lo, n = cur.n;
      const int nMiddle = (n - 1) / 2;
      const double x0 = xpos(lo), xl = xpos(lo + n - 1), xm = xpos(lo + nMiddle);
      const double dX = (cur.xs[2] - cur.xs[0]) / (xl - x0);
      const double dY = (cur.ys[2] - cur.ys[0]) / (xl - x0);
      const double dfError = fabs((cur.xs[0] + dX * (xm - x0)) - cur.xs[1]) +
                             fabs((cur.ys[0] + dY * (xm - x0)) - cur.ys[1]);
      if (dfError <= kMaxErr) {
        if (nl >= kMaxLeavesLocal) return -1;
        out[nl].start = lo; out[nl].kind = 0;
        out[nl].xs0 = cur.xs[0]; out[nl].ys0 = cur.ys[0]; out[nl].dX = dX; out[nl].dY = dY;
        nl++;
      } else {
        const int i0 = lo + (nMiddle - 1) / 2, i1 = lo + nMiddle - 1, i2 = lo + nMiddle + (n - nMiddle - 1) / 2;
        double mx[3] = {xpos(i0), xpos(i1), xpos(i2)};
        double my[3] = {yrow, yrow, yrow};
        const bool base1 = nMiddle <= 5 || x0 == mx[1] || x0 == mx[0];
        const bool base2 = n - nMiddle <= 5 || xm == xl || xm == mx[2];
        bool ok = false;
        if (!base1 && !base2) {
          ok = xform_point(t, true, mx[0], my[0]);
          ok = xform_point(t, true, mx[1], my[1]) && ok;
          ok = xform_point(t, true, mx[2], my[2]) && ok;
        } else if (!base1) {
          ok = xform_point(t, true, mx[0], my[0]);
          ok = xform_point(t, true, mx[1], my[1]) && ok;
        } else if (!base2) {
          ok = xform_point(t, true, mx[2], my[2]);
        }
        if (!ok) {  // the whole node is transformed exactly
          if (nl >= kMaxLeavesLocal) return -1;
          out[nl].start = lo; out[nl].kind = 1;
          out[nl].xs0 = out[nl].ys0 = out[nl].dX = out[nl].dY = 0;
          nl++;
        } else {
          if (sp >= 14) return -1;
          Node &h2 = stack[sp++];  // second half deferred, first half next
          h2.lo = lo + nMiddle; h2.n = n - nMiddle;
          h2.exact_leaf = base2 ? 1 : 0;
          h2.xs[0] = cur.xs[1]; h2.ys[0] = cur.ys[1];
          h2.xs[1] = mx[2]; h2.ys[1] = my[2];
          h2.xs[2] = cur.xs[2]; h2.ys[2] = cur.ys[2];
          Node h1;
          h1.lo = lo; h1.n = nMiddle;
          h1.exact_leaf = base1 ? 1 : 0;
          h1.xs[0] = cur.xs[0]; h1.ys[0] = cur.ys[0];
          h1.xs[1] = mx[0]; h1.ys[1] = my[0];
          h1.xs[2] = mx[1]; h1.ys[2] = my[1];
          cur = h1;
          continue;
        }
      }
    }
    if (sp == 0) break;
    cur = stack[--sp];
  }
  return nl;
}

// Split pass over the rows the light pass could not interpolate in one
// piece.  DESCEND rows: the approximation recursion's leaves into the pool,
// every EXACT piece expanded into per-pixel pending leaves; EXACT rows: one
// pending leaf per pixel.  The row becomes ROW_POOL; on pool overflow it keeps
// its kind and the tile goes to the general kernel.
__device__ void plan_split_one(const PlanArgs &a, int k) {
  {
    const int64_t key = a.split_list[k];
    const int p = (int)(key / a.max_h), row = (int)(key % a.max_h);
    const PairPlan &pp = a.pairs[p];
    RowRec &rec = a.rows[key];
    if (rec.kind == ROW_EXACT) {
      const int n = pp.w;
      const int off = atomicAdd(&a.counters[0], n);
      if (off + n > a.pool_cap) { flag_complex(a, pp.tile); return; }
      for (int j = 0; j < n; j++) a.pool[off + j] = pending_leaf(p, row, j);
      rec.kind = ROW_POOL;
      rec.nleaf = n;
      rec.pool_off = off;
      return;
    }
    const double yrow = row + 0.5 + pp.yoff;
    Leaf local[kMaxLeavesLocal];
    const int nl = approx_leaves(a.xforms[p], pp.xoff, yrow, pp.w, rec.v, local);
    int total = 0;
    for (int j = 0; j < nl; j++)
      total += local[j].kind == LEAF_LINEAR ? 1 : (j + 1 < nl ? local[j + 1].start : pp.w) - local[j].start;
    int off = -1;
    if (nl > 0) {
      off = atomicAdd(&a.counters[0], total);
      if (off + total > a.pool_cap) off = -1;
    }
    if (off < 0) { flag_complex(a, pp.tile); return; }   // stays ROW_DESCEND
    int m = off;
    for (int j = 0; j < nl; j++) {
      if (local[j].kind == LEAF_LINEAR) {
        a.pool[m++] = local[j];
      } else {
        const int end = j + 1 < nl ? local[j + 1].start : pp.w;
        for (int i = local[j].start; i < end; i++) a.pool[m++] = pending_leaf(p, row, i);
      }
    }
    rec.kind = ROW_POOL;
    rec.nleaf = total;
    rec.pool_off = off;
  }
}

__global__ __launch_bounds__(64) void plan_split_kernel(PlanArgs a) {
  const int nsplit = a.counters[1];
  for (int k = blockIdx.x * blockDim.x + threadIdx.x; k < nsplit; k += gridDim.x * blockDim.x) plan_split_one(a, k);
}

// Exact points of the pending leaves (GDALGenImgProjTransform per pixel, the
// expressions of exact_coords()), one thread per pool entry.
__device__ __forceinline__ void plan_exact_one(const PlanArgs &a, int k) {
  {
    Leaf L = a.pool[k];
    if (L.kind != LEAF_PENDING) return;
    const int p = (int)L.dX, row = (int)L.dY;
    if (p < 0 || p >= a.n_pairs || row < 0 || row >= a.max_h) return;   // stale slot of an abandoned reservation
    const PairPlan &pp = a.pairs[p];
    double sx, sy;
    const bool ok = exact_coords(a.xforms[p], pp.xoff, pp.yoff, L.start, row, sx, sy);
    L.xs0 = sx; L.ys0 = sy; L.dX = 0.0; L.dY = 0.0;
    L.kind = ok ? LEAF_LINEAR : LEAF_FAILED;
    a.pool[k] = L;
  }
}

__global__ __launch_bounds__(256) void plan_exact_kernel(PlanArgs a) {
  const int used = min(a.counters[0], a.pool_cap);
  for (int k = blockIdx.x * blockDim.x + threadIdx.x; k < used; k += gridDim.x * blockDim.x) plan_exact_one(a, k);
}

// Small batches (C1: one tile), where every planning kernel is a few us of
// dispatch for a few us of work: plan_tiles, plan_cols, plan_rows,
// plan_split and plan_exact as the phases of ONE workgroup (waves take tiles,
// threads take columns, rows, split rows and pending leaves; a workgroup
// barrier between phases).  The same device bodies as the separate kernels,
// so the same plan.  Also zeroes the counters (the prologue does not run).
__global__ __launch_bounds__(256) void plan_small_kernel(PlanArgs a) {
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
#ifdef GSKYHIP_AB
  // phase time stamps (GSKYHIP_PLAN_STAMPS): 100 MHz wall clock into counters[40 + i]
  uint64_t st[8], st_pair[6] = {0, 0, 0, 0, 0, 0};
  int ns = 0;
  auto stamp = [&]() { if (ns < 8) st[ns++] = wall_clock64(); };
#else
  auto stamp = [&]() {};
#endif
  stamp();
  if (a.small == 2) {   // the pairs too (one or two): the whole plan is this one launch
    __shared__ double sx[kGrid], sy[kGrid];
    __shared__ int sok[kGrid];
    __shared__ Xform ts;
#ifdef GSKYHIP_AB
    __shared__ uint64_t s_ps[8];
    uint64_t *ps = s_ps;
#else
    uint64_t *ps = nullptr;
#endif
    for (int p = 0; p < a.n_pairs; p++) {
      plan_pair<256>(a, p, sx, sy, sok, ts, p == 0 ? ps : nullptr);
      __syncthreads();
    }
#ifdef GSKYHIP_AB
    if (tid == 0) for (int i = 1; i < 6; i++) st_pair[i] = s_ps[i] - s_ps[i - 1];
#endif
  }
  stamp();
  if (tid < 64) a.counters[tid] = 0;
  __syncthreads();
  for (int t = wave; t < a.n_tiles; t += 4) plan_tile_waves<1>(a, t, 0, lane, nullptr);
  __syncthreads();
  stamp();
  if (a.sep)
    for (int64_t g = tid; g < 3 * (int64_t)a.n_pairs; g += 256) plan_col(a, g);
  __syncthreads();
  stamp();
  for (int64_t i = tid; i < (int64_t)a.n_pairs * a.max_h; i += 256) {
    const int p = (int)(i / a.max_h), row = (int)(i % a.max_h);
    const PairPlan &pp = a.pairs[p];
    if (row < pp.h) plan_row(a, p, pp, a.xforms[p], row);
  }
  __syncthreads();
  stamp();
  const int nsplit = a.counters[1];
  for (int k = tid; k < nsplit; k += 256) plan_split_one(a, k);
  __syncthreads();
  stamp();
  const int used = min(a.counters[0], a.pool_cap);
  for (int k = tid; k < used; k += 256) plan_exact_one(a, k);
  __syncthreads();
  stamp();
#ifdef GSKYHIP_AB
  if (tid == 0) {
    for (int i = 1; i < ns; i++) a.counters[40 + i] = (int32_t)(st[i] - st[i - 1]);
    for (int i = 1; i < 6; i++) a.counters[50 + i] = (int32_t)st_pair[i];
  }
#endif
}

}  // namespace gsky

#include "render_generic.h"

namespace gsky {


// Scale + RGBA from typed canvases (auto-scale second pass).
__global__ __launch_bounds__(256) void canvas_rgba_kernel(RenderArgs a) {
  __shared__ uint32_t s_ramp[256];
  const int tid = threadIdx.x;
  if (a.ramp) s_ramp[tid] = a.ramp[tid];
  __syncthreads();
  const int bands_per_tile = (a.max_h + a.rows_per_block - 1) / a.rows_per_block;
  const int t = blockIdx.x / bands_per_tile;
  const int band0 = (blockIdx.x % bands_per_tile) * a.rows_per_block;
  if (t >= a.n_tiles) return;
  const gskyhip_tile tile = a.tiles[t];
  const TilePlan tp = a.tplans[t];
  if (tp.status == GSKYHIP_E_ARG) return;   // tile outside the slot: never written
  const int W = tile.width, H = tile.height, n_out = a.n_out;
  ScaleK sk[3];
  bool all_created = true;
  for (int s = 0; s < n_out; s++) {
    const int ns = a.out_ns[s];
    all_created = all_created && tp.created[ns];
    if (!tp.created[ns]) continue;
    float mn = 0.0f, mx = 0.0f;
    if (a.autom) auto_minmax(a.minmax[t * 3 + s], mn, mx);
    sk[s] = make_scale(tp.dtype[ns], tp.nodata[ns], a.sp, a.autom != 0, mn, mx);
  }
  for (int r = band0; r < band0 + a.rows_per_block && r < H; r++) {
    for (int x = tid; x < W; x += 256) {
      const long idx = (long)r * a.max_w + x;
      uint8_t b[3] = {0xFF, 0xFF, 0xFF};
      if (all_created) {
        for (int s = 0; s < n_out; s++) {
          const int dt = tp.dtype[a.out_ns[s]];
          const uint8_t *cb = a.canvas + t * a.canvas_tile_stride + s * a.canvas_ns_stride;
          Val v;
          switch (dt) {
            case GSKYHIP_SIGNEDBYTE: v.i = ((const int8_t *)cb)[idx]; break;
            case GSKYHIP_BYTE: v.i = cb[idx]; break;
            case GSKYHIP_INT16: v.i = ((const int16_t *)cb)[idx]; break;
            case GSKYHIP_UINT16: v.i = ((const uint16_t *)cb)[idx]; break;
            default: v.u = ((const uint32_t *)cb)[idx]; break;
          }
          b[s] = scale_px(sk[s], v);
        }
      }
      uint32_t o = 0;
      if (all_created) {
        if (n_out == 1) {
          if (b[0] != 0xFF) o = a.ramp ? s_ramp[b[0]] : (0xFF000000u | ((uint32_t)b[0] << 16) | ((uint32_t)b[0] << 8) | b[0]);
        } else if (b[0] != 0xFF || b[1] != 0xFF || b[2] != 0xFF) {
          o = 0xFF000000u | ((uint32_t)b[2] << 16) | ((uint32_t)b[1] << 8) | b[0];
        }
      }
      ((uint32_t *)(a.rgba + (long)t * a.max_h * a.max_w * 4))[idx] = o;
    }
  }
}

__global__ void minmax_init_kernel(MinMax *m, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  m[i].mn = fenc(INFINITY);
  m[i].mx = fenc(-INFINITY);
  m[i].p0_valid = 0;
  m[i].p0 = 0.0f;
}

// Warped window of each pair (the FlexRaster data of tile_grpc.go:228-241).
template <int RES>
__global__ __launch_bounds__(256) void warp_window_kernel(const PairPlan *pairs, const Xform *xforms,
                                                          const RowRec *rows, const Leaf *pool, int max_h,
                                                          int max_w, int n_pairs, uint8_t *out, long stride) {
  const long gid = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long per = (long)max_h * max_w;
  const int p = (int)(gid / per);
  if (p >= n_pairs) return;
  const PairPlan &pp = pairs[p];
  const long k = gid % per;
  const int row = (int)(k / max_w), i = (int)(k % max_w);
  if (row >= pp.h || i >= pp.w) return;
  const RowRec &rr = rows[(long)p * max_h + row];
  const Val v = warped_value<true, RES>(pp, rr, pool, xforms + p, i, row);
  const int dsz = type_size(pp.out_dtype);
  uint8_t *o = out + p * stride;
  const long idx = (long)row * pp.w + i;
  if (dsz == 1) o[idx] = (uint8_t)v.i;
  else if (dsz == 2) ((uint16_t *)o)[idx] = (uint16_t)v.i;
  else ((uint32_t *)o)[idx] = v.u;
}

// bytesRead of the drop-in (warp.go:278-347), pair 0: per window pixel the
// reference's two tests -- the cache heuristic's x test (success, dx >= 0,
// iSrcX < srcXSize; no dy test) and the full gather test -- plus the set of
// source blocks that valid pixels touch.
// warp.go:281-347 bytesRead of every (single-pair) request of a warp batch,
// blockIdx.y = job = pair: per valid pixel the source x (xsrc, for the
// cache decision), the first valid pixel, the valid count and the touched
// block bits.  The counters are reduced per workgroup (ballots, one atomic
// each) and the bits per wave (a lane ORs its block only where it differs
// from the previous lane's), so neighbouring pixels do not serialize on one
// address.
__global__ __launch_bounds__(256) void block_stats_init_kernel(const BlockStatsJob *jobs, char *scratch,
                                                               int32_t *stats) {
  const BlockStatsJob J = jobs[blockIdx.x];
  uint32_t *bits = (uint32_t *)(scratch + J.bits_off);
  for (int k = threadIdx.x; k < J.n_words; k += blockDim.x) bits[k] = 0u;
  if (threadIdx.x == 0) {
    int32_t *st = stats + 4 * blockIdx.x;
    st[0] = 0x7FFFFFFF; st[1] = 0; st[2] = 0; st[3] = 0;
  }
}

__global__ __launch_bounds__(256) void block_stats_kernel(const PairPlan *pairs, const Xform *xforms,
                                                          const RowRec *rows, const Leaf *pool, int max_h,
                                                          const BlockStatsJob *jobs, char *scratch, int32_t *stats) {
  const int job = blockIdx.y;
  const PairPlan &pp = pairs[job];
  const BlockStatsJob J = jobs[job];
  int32_t *xsrc = (int32_t *)(scratch + J.xsrc_off);
  uint32_t *bits = (uint32_t *)(scratch + J.bits_off);
  const long gid = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long n = (long)pp.w * pp.h;
  bool valid = false;
  int ix = 0, iy = 0;
  if (gid < n) {
    const int row = (int)(gid / pp.w), i = (int)(gid % pp.w);
    double sx, sy;
    const bool ok = src_coords<true>(rows[(int64_t)job * max_h + row], pool, xforms + job, pp.xoff, pp.yoff, pp.w, i,
                                     row, sx, sy);
    int xs = -1;
    if (ok && !(sx < 0)) {
      const double ax = sx + 1.0e-10;
      if (ax < 2147483647.0) {
        ix = (int)ax;
        if (ix < pp.band_x) xs = ix;
      }
    }
    if (xs >= 0 && !(sy < 0)) {
      const double ay = sy + 1.0e-10;
      if (ay < 2147483647.0) {
        iy = (int)ay;
        valid = iy < pp.band_y;
      }
    }
    xsrc[gid] = xs;
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const unsigned long long bal = __ballot(valid);
  __shared__ int s_first[4], s_count[4];
  if (lane == 0) {
    s_first[wave] = bal ? (int)(gid + __ffsll((long long)bal) - 1) : 0x7FFFFFFF;
    s_count[wave] = __popcll(bal);
  }
  int bx = J.bx;
  if (bx <= 0) bx = pp.band_x;        // default block: one scanline of the chosen level
  const int nxb = (pp.band_x + bx - 1) / bx;
  const long long blk = valid ? (long long)(ix / bx) + (long long)(iy / J.by) * nxb : -1;
  const long long prev = __shfl_up(blk, 1, 64);
  if (valid && (lane == 0 || prev != blk)) atomicOr(&bits[blk >> 5], 1u << (blk & 31));
  __syncthreads();
  if (threadIdx.x == 0) {
    int first = s_first[0], count = s_count[0];
    for (int w = 1; w < 4; w++) { first = min(first, s_first[w]); count += s_count[w]; }
    if (count > 0) {
      atomicMin(&stats[4 * job], first);
      atomicAdd(&stats[4 * job + 1], count);
    }
  }
}

// warp.go:281-313 (the cache decision at the first valid pixel) and 347, a
// workgroup (one thread) per job.
__global__ void block_stats_resolve_kernel(const PairPlan *pairs, const BlockStatsJob *jobs, const char *scratch,
                                           int32_t *stats_all) {
  if (threadIdx.x != 0) return;
  const int job = blockIdx.x;
  const PairPlan &pp = pairs[job];
  const BlockStatsJob J = jobs[job];
  const int32_t *xsrc = (const int32_t *)(scratch + J.xsrc_off);
  const uint32_t *bits = (const uint32_t *)(scratch + J.bits_off);
  int32_t *stats = stats_all + 4 * job;
  int bx = J.bx;
  if (bx <= 0) bx = pp.band_x;
  const int i0 = stats[0];
  if (i0 == 0x7FFFFFFF) { stats[2] = 0; return; }
  const int r0 = i0 / pp.w, c0 = i0 % pp.w;
  const int prev = xsrc[i0];
  int curr = -1;
  for (int c = c0 + 1; c < pp.w; c++) {
    const int v = xsrc[(long)r0 * pp.w + c];
    if (v >= 0) { curr = v; break; }
  }
  if (curr < prev) curr = prev;
  const int stride = curr - prev;
  const bool cache = stride >= 0 && stride < bx;
  long nread = 0;
  if (cache) {
    for (int k = 0; k < J.n_words; k++) nread += __popc(bits[k]);
  } else {
    nread = stats[1];   // one GDALReadBlock per valid pixel (warp.go:319-322)
  }
  // C int arithmetic of warp.go:347 (wraps like the reference's 32-bit int)
  const long long b = (long long)bx * J.by * type_size(pp.src_dtype) * nread;
  stats[2] = (int32_t)(uint32_t)(unsigned long long)b;
}

// One window pixel of a job: its value (warped_value's rules, warp.go:271-344)
// and the bytesRead inputs (block_stats_kernel's, warp.go:281-347).
template <int RES>
__device__ __forceinline__ Val warp_job_pixel(const PairPlan &pp, const RowRec &rr, const Leaf *pool, const Xform *xf,
                                              int i, int row, int &xs, bool &valid, int &ix, int &iy) {
  double sx, sy;
  const bool ok = src_coords<true>(rr, pool, xf, pp.xoff, pp.yoff, pp.w, i, row, sx, sy);
  // bytesRead: the cache heuristic's x test and the full gather test
  xs = -1;
  valid = false;
  ix = 0;
  iy = 0;
  if (ok && !(sx < 0)) {
    const double ax = sx + 1.0e-10;
    if (ax < 2147483647.0) {
      ix = (int)ax;
      if (ix < pp.band_x) xs = ix;
    }
  }
  if (xs >= 0 && !(sy < 0)) {
    const double ay = sy + 1.0e-10;
    if (ay < 2147483647.0) {
      iy = (int)ay;
      valid = iy < pp.band_y;
    }
  }
  // the window value, exactly as warped_value<true, RES>
  Val v = pp.fill;
  if (ok) {
    if (RES == GSKYHIP_RESAMPLE_BILINEAR) {
      v = bilinear_value(pp, sx, sy);
    } else if (!(sx < 0 || sy < 0)) {
      const double ax = sx + 1.0e-10, ay = sy + 1.0e-10;
      if (!(ax >= 2147483647.0 || ay >= 2147483647.0)) {
        const int jx = (int)ax, jy = (int)ay;
        if (jx < pp.band_x && jy < pp.band_y) {
          v = load_val(pp.band, pp.src_dtype, (long)jy * pp.band_x + jx);
          if (pp.out_dtype == GSKYHIP_SIGNEDBYTE) v.i = (int32_t)(int8_t)(uint8_t)v.i;
        }
      }
    }
  }
  return v;
}

// The per-node service's warp batch (warp_batch_launch, host.cpp): for every
// request (job = pair) its window values AND its bytesRead inputs from ONE
// source-coordinate evaluation per pixel -- round 4 ran warp_window_kernel
// and block_stats_kernel, each deriving the same coordinates again.  The
// window goes straight to the job's destination `outs[job]`: a device staging
// slot, or the requesting worker's shared reply arena (host memory registered
// with HIP, written over PCIe: no read-back copy).  PX pixels per thread
// (consecutive in the packed window): with PX = 4 a thread's values leave in
// one store of 4 * element bytes (wider writes over PCIe).
template <int RES, int PX = 1>
__global__ __launch_bounds__(256) void warp_job_kernel(const PairPlan *pairs, const Xform *xforms,
                                                       const RowRec *rows, const Leaf *pool, int max_h,
                                                       const BlockStatsJob *jobs, char *scratch, int32_t *stats,
                                                       uint8_t *const *outs) {
  const int job = blockIdx.y;
  const PairPlan &pp = pairs[job];
  const BlockStatsJob J = jobs[job];
  int32_t *xsrc = (int32_t *)(scratch + J.xsrc_off);
  uint32_t *bits = (uint32_t *)(scratch + J.bits_off);
  const long gid = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long n = (long)pp.w * pp.h;
  const long p0 = gid * PX;
  int bx = J.bx;
  if (bx <= 0) bx = pp.band_x;
  const int nxb = (pp.band_x + bx - 1) / bx;
  const int dsz = type_size(pp.out_dtype);
  uint8_t *o = outs[job];
  int first = 0x7FFFFFFF, count = 0;
  long long blk[PX];
  Val v[PX];
#pragma unroll
  for (int q = 0; q < PX; q++) {
    blk[q] = -1;
    v[q].u = 0;
    const long p = p0 + q;
    if (p >= n) continue;
    const int row = (int)(p / pp.w), i = (int)(p % pp.w);
    int xs, ix, iy;
    bool valid;
    v[q] = warp_job_pixel<RES>(pp, rows[(int64_t)job * max_h + row], pool, xforms + job, i, row, xs, valid, ix, iy);
    xsrc[p] = xs;
    if (valid) {
      first = min(first, (int)p);
      count++;
      blk[q] = (long long)(ix / bx) + (long long)(iy / J.by) * nxb;
    }
  }
  const int wbytes = PX * dsz;   // the thread's window bytes
  if (PX > 1 && p0 + PX <= n && ((uintptr_t)(o + p0 * dsz) & ((wbytes < 16 ? wbytes : 16) - 1)) == 0) {
    // packed into 32-bit words, stored 4, 8 or 16 bytes at a time
    uint32_t w[PX];
#pragma unroll
    for (int k = 0; k < PX; k++) {
      if (dsz == 1)
        w[k] = k < PX / 4 ? (v[4 * k].u & 0xFFu) | (v[4 * k + 1].u & 0xFFu) << 8 | (v[4 * k + 2].u & 0xFFu) << 16 |
                                v[4 * k + 3].u << 24
                          : 0u;
      else if (dsz == 2)
        w[k] = k < PX / 2 ? (v[2 * k].u & 0xFFFFu) | v[2 * k + 1].u << 16 : 0u;
      else
        w[k] = v[k].u;
    }
    uint8_t *d = o + p0 * dsz;
    if (wbytes == 4) {
      *(uint32_t *)d = w[0];
    } else if (wbytes == 8) {
      *(uint2 *)d = make_uint2(w[0], w[1]);
    } else {
#pragma unroll
      for (int k = 0; k + 3 < PX; k += 4)
        if (4 * k < wbytes) *(uint4 *)(d + 4 * k) = make_uint4(w[k], w[k + 1], w[k + 2], w[k + 3]);
    }
  } else {
#pragma unroll
    for (int q = 0; q < PX; q++) {
      const long p = p0 + q;
      if (p >= n) continue;
      if (dsz == 1) o[p] = (uint8_t)v[q].i;
      else if (dsz == 2) ((uint16_t *)o)[p] = (uint16_t)v[q].i;
      else ((uint32_t *)o)[p] = v[q].u;
    }
  }
  // touched blocks: a pixel ORs its block's bit where it differs from the
  // pixel before it (the previous lane's last pixel for the first)
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  long long prev = __shfl_up(blk[PX - 1], 1, 64);
  if (lane == 0) prev = -2;
#pragma unroll
  for (int q = 0; q < PX; q++) {
    if (blk[q] >= 0 && blk[q] != prev) atomicOr(&bits[blk[q] >> 5], 1u << (blk[q] & 31));
    prev = blk[q];
  }
  // first valid pixel and valid count: per wave, then per workgroup
  for (int sft = 32; sft > 0; sft >>= 1) {
    first = min(first, __shfl_xor(first, sft, 64));
    count += __shfl_xor(count, sft, 64);
  }
  __shared__ int s_first[4], s_count[4];
  if (lane == 0) {
    s_first[wave] = first;
    s_count[wave] = count;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int f = s_first[0], c = s_count[0];
    for (int w = 1; w < 4; w++) { f = min(f, s_first[w]); c += s_count[w]; }
    if (c > 0) {
      atomicMin(&stats[4 * job], f);
      atomicAdd(&stats[4 * job + 1], c);
    }
  }
}

// bytesRead (block_stats_resolve_kernel's rules) and the job's reply record
// (bbox, dtype, nodata, overview-rescaled geotransform): one thread per job.
__global__ void warp_job_resolve_kernel(const PairPlan *pairs, const BlockStatsJob *jobs, const char *scratch,
                                        int32_t *stats_all, int n_jobs, WarpResult *res) {
  const int job = blockIdx.x * blockDim.x + threadIdx.x;
  if (job >= n_jobs) return;
  const PairPlan &pp = pairs[job];
  const BlockStatsJob J = jobs[job];
  const int32_t *xsrc = (const int32_t *)(scratch + J.xsrc_off);
  const uint32_t *bits = (const uint32_t *)(scratch + J.bits_off);
  int32_t *stats = stats_all + 4 * job;
  int bx = J.bx;
  if (bx <= 0) bx = pp.band_x;
  const int i0 = stats[0];
  int32_t br = 0;
  if (i0 != 0x7FFFFFFF) {
    const int r0 = i0 / pp.w, c0 = i0 % pp.w;
    const int prev = xsrc[i0];
    int curr = -1;
    for (int c = c0 + 1; c < pp.w; c++) {
      const int v = xsrc[(long)r0 * pp.w + c];
      if (v >= 0) { curr = v; break; }
    }
    if (curr < prev) curr = prev;
    const int stride = curr - prev;
    const bool cache = stride >= 0 && stride < bx;
    long nread = 0;
    if (cache) {
      for (int k = 0; k < J.n_words; k++) nread += __popc(bits[k]);
    } else {
      nread = stats[1];
    }
    const long long b = (long long)bx * J.by * type_size(pp.src_dtype) * nread;
    br = (int32_t)(uint32_t)(unsigned long long)b;
  }
  WarpResult &r = res[job];
  r.bbox[0] = pp.xoff; r.bbox[1] = pp.yoff; r.bbox[2] = pp.w; r.bbox[3] = pp.h;
  r.dtype = pp.out_dtype;
  r.bytes_read = br;
  r.nodata = pp.nodata;
  for (int k = 0; k < 6; k++) r.src_gt[k] = pp.src_gt[k];
}

// Source footprint of every planned pair (gskyhip_render_pair_info, an
// observability hook for the algorithmic bytes of a batch): the picked
// level, its element size and the bounding box of the source pixels the
// pair's LINEAR rows and linear leaves sample (first and last pixel of each
// row or leaf: the interpolation is linear along a row), clamped to the
// level.  One thread per pair.
__global__ void pair_footprint_kernel(const PairPlan *pairs, const RowRec *rows, const Leaf *pool, int n_pairs,
                                      int max_h, int32_t *out) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n_pairs) return;
  const PairPlan &pp = pairs[p];
  double x0 = INFINITY, y0 = INFINITY, x1 = -INFINITY, y1 = -INFINITY;
  auto take = [&](double xs, double ys, double dx, double dy, int n) {
    const double xe = xs + dx * (n - 1), ye = ys + dy * (n - 1);
    x0 = fmin(x0, fmin(xs, xe)); x1 = fmax(x1, fmax(xs, xe));
    y0 = fmin(y0, fmin(ys, ye)); y1 = fmax(y1, fmax(ys, ye));
  };
  for (int r = 0; r < pp.h && pp.w > 0; r++) {
    const RowRec &rr = rows[(int64_t)p * max_h + r];
    if (rr.kind == ROW_LINEAR) {
      take(rr.v[0], rr.v[1], rr.v[2], rr.v[3], pp.w);
    } else if (rr.kind == ROW_POOL) {
      const Leaf *lv = pool + rr.pool_off;
      for (int k = 0; k < rr.nleaf; k++) {
        const Leaf &L = lv[k];
        if (L.kind != LEAF_LINEAR) continue;
        const int end = k + 1 < rr.nleaf ? lv[k + 1].start : pp.w;
        if (end > L.start) take(L.xs0, L.ys0, L.dX, L.dY, end - L.start);
      }
    }
  }
  int32_t *o = out + 8 * p;
  o[0] = pp.granule; o[1] = pp.band_x; o[2] = pp.band_y; o[3] = type_size(pp.src_dtype);
  if (x0 <= x1 && y0 <= y1) {
    o[4] = (int32_t)fmax(0.0, fmin((double)pp.band_x, floor(x0)));
    o[5] = (int32_t)fmax(0.0, fmin((double)pp.band_y, floor(y0)));
    o[6] = (int32_t)fmax(0.0, fmin((double)pp.band_x, floor(x1) + 1.0));
    o[7] = (int32_t)fmax(0.0, fmin((double)pp.band_y, floor(y1) + 1.0));
  } else {
    o[4] = o[5] = o[6] = o[7] = 0;
  }
}

// Source elements and 128-byte lines the pairs of a planned batch touch
// (gskyhip_render_touched: the algorithmic bytes of a batch, SURVEY.md 8(d)
// "unique source bytes touched ... at the chosen overview level"): every
// window pixel of every pair -- data and mask rasters alike, as GDAL reads
// each granule's window -- picks its source element by the nearest-neighbour
// rule of warp.go:271-300 (lin_coords + truncation + bounds); the element and
// its line are set in per-level bitmaps (base[p]: bit offsets of pair p's
// level in the element / line maps).  ROW_LINEAR and ROW_POOL rows (what the
// band kernels render); rows computed exactly at render time are not counted.
// Block = (pair, 4 rows), 256 threads over the window columns.
__global__ void pair_touch_kernel(const PairPlan *pairs, const RowRec *rows, const Leaf *pool, int max_h,
                                  const int64_t *base, uint32_t *ebits, uint32_t *lbits) {
  const int p = blockIdx.x;
  const PairPlan &pp = pairs[p];
  const int64_t eb = base[2 * p], lb = base[2 * p + 1];
  if (eb < 0 || pp.w <= 0) return;
  const int es = type_size(pp.src_dtype);
  for (int r = blockIdx.y * 4; r < min(pp.h, (int)blockIdx.y * 4 + 4); r++) {
    const RowRec &rr = rows[(int64_t)p * max_h + r];
    if (rr.kind != ROW_LINEAR && rr.kind != ROW_POOL) continue;
    for (int ic = threadIdx.x; ic < pp.w; ic += blockDim.x) {
      double sx, sy;
      if (!lin_coords(rr, pool, ic, sx, sy) || sx < 0.0 || sy < 0.0) continue;
      const double ax = sx + 1.0e-10, ay = sy + 1.0e-10;
      if (ax >= (double)pp.band_x || ay >= (double)pp.band_y) continue;
      const int64_t idx = (int64_t)(int)ay * pp.band_x + (int)ax;
      const int64_t e = eb + idx, l = lb + idx * es / 128;
      atomicOr(&ebits[e >> 5], 1u << (e & 31));
      atomicOr(&lbits[l >> 5], 1u << (l & 31));
    }
  }
}

__global__ void popcount_kernel(const uint32_t *bits, int64_t n_words, const int64_t *word_es, int n_seg,
                                unsigned long long *out) {
  // word_es: n_seg x (first word, element bytes) of each level's segment
  unsigned long long acc = 0;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n_words; i += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t w = bits[i];
    if (!w) continue;
    int lo = 0, hi = n_seg - 1;   // the segment holding word i
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (word_es[2 * mid] <= i) lo = mid; else hi = mid - 1;
    }
    acc += (unsigned long long)__popc(w) * (unsigned long long)word_es[2 * lo + 1];
  }
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
  if ((threadIdx.x & 63) == 0 && acc) atomicAdd(out, acc);
}

__global__ void pair_meta_kernel(const PairPlan *pairs, int n_pairs, int32_t *bbox, int32_t *dtype, double *nodata) {
  int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n_pairs) return;
  const PairPlan &pp = pairs[p];
  bbox[4 * p] = pp.xoff; bbox[4 * p + 1] = pp.yoff; bbox[4 * p + 2] = pp.w; bbox[4 * p + 3] = pp.h;
  dtype[p] = pp.out_dtype;
  nodata[p] = pp.nodata;
}

}  // namespace gsky

// ======================================================================== host
namespace gsky {

static inline int64_t align256(int64_t x) { return (x + 255) & ~(int64_t)255; }

struct Carve {
  PairPlan *pairs; Xform *xforms; TilePlan *tplans; int32_t *order; int32_t *pair_tile;
  RowRec *rows; RowFix *rowfix; Leaf *pool; int32_t *counters; MinMax *minmax; int64_t *split_list; int32_t *complex_list;
  EntryD *entries;
  SepCol *sepcols;
  int pool_cap;
  int64_t total;
};

// Workspace layout; PairPlan[] first and TilePlan[] third are relied upon by
// host.cpp (drop-in geotransform read-back, gskyhip_render_status).
static Carve carve(void *base, int n_tiles, int n_pairs, int max_h) {
  Carve c;
  int64_t off = 0;
  auto take = [&](int64_t bytes) { int64_t o = off; off = align256(off + bytes); return o; };
  const int np = n_pairs > 0 ? n_pairs : 1, nt = n_tiles > 0 ? n_tiles : 1;
  c.pool_cap = (int)std::min<int64_t>((int64_t)np * max_h / 2 + 4096, 64 << 20);
  const int64_t o_pairs = take(sizeof(PairPlan) * (int64_t)np);
  const int64_t o_xf = take(sizeof(Xform) * (int64_t)np);
  const int64_t o_tp = take(sizeof(TilePlan) * (int64_t)nt);
  const int64_t o_ord = take(sizeof(int32_t) * (int64_t)np);
  const int64_t o_pt = take(sizeof(int32_t) * (int64_t)np);
  const int64_t o_rows = take(sizeof(RowRec) * (int64_t)np * max_h);
  const int64_t o_rfix = take(sizeof(RowFix) * (int64_t)np * max_h);
  const int64_t o_pool = take(sizeof(Leaf) * (int64_t)c.pool_cap);
  const int64_t o_cnt = take(256);
  const int64_t o_mm = take(sizeof(MinMax) * (int64_t)nt * 3);
  const int64_t o_split = take(sizeof(int64_t) * (int64_t)np * max_h);
  const int64_t o_cl = take(sizeof(int32_t) * (int64_t)nt);
  const int64_t o_ent = take(sizeof(EntryD) * (int64_t)np);
  const int64_t o_sep = take(sizeof(SepCol) * 3 * (int64_t)np);
  c.total = off;
  char *b = (char *)base;
  c.pairs = (PairPlan *)(b + o_pairs);
  c.xforms = (Xform *)(b + o_xf);
  c.tplans = (TilePlan *)(b + o_tp);
  c.order = (int32_t *)(b + o_ord);
  c.pair_tile = (int32_t *)(b + o_pt);
  c.rows = (RowRec *)(b + o_rows);
  c.rowfix = (RowFix *)(b + o_rfix);
  c.pool = (Leaf *)(b + o_pool);
  c.counters = (int32_t *)(b + o_cnt);
  c.minmax = (MinMax *)(b + o_mm);
  c.split_list = (int64_t *)(b + o_split);
  c.complex_list = (int32_t *)(b + o_cl);
  c.entries = (EntryD *)(b + o_ent);
  c.sepcols = (SepCol *)(b + o_sep);
  return c;
}

int64_t render_counters_offset(int n_tiles, int n_pairs, int max_h) {
  return (int64_t)((char *)carve(nullptr, n_tiles, n_pairs, max_h).counters - (char *)nullptr);
}

int64_t render_workspace_size(int n_tiles, int n_pairs, int max_h) {
  return carve(nullptr, n_tiles, n_pairs, max_h).total;
}

static int plan_all(const RenderCall &rc, Carve &cv) {
  if (rc.n_tiles <= 0) return 0;
  if (!rc.workspace || rc.workspace_bytes < render_workspace_size(rc.n_tiles, rc.n_pairs, rc.max_h))
    return GSKYHIP_E_ARG;
  cv = carve(rc.workspace, rc.n_tiles, rc.n_pairs, rc.max_h);
  PlanArgs a;
  a.granules = rc.granules; a.crs = rc.crs; a.n_crs = rc.n_crs; a.dst_crs = rc.dst_crs;
  a.tiles = rc.tiles; a.n_tiles = rc.n_tiles; a.pair_granule = rc.pair_granule; a.n_pairs = rc.n_pairs;
  a.pair_tile_max = 0; a.max_h = rc.max_h; a.max_w = rc.max_w; a.mask_ns = rc.mask_ns; a.mask_inclusive = rc.mask_inclusive;
  a.pairs = cv.pairs; a.xforms = cv.xforms; a.tplans = cv.tplans; a.order = cv.order;
  a.pair_tile = cv.pair_tile; a.rows = cv.rows; a.rowfix = cv.rowfix; a.pool = cv.pool; a.counters = cv.counters;
  a.pool_cap = cv.pool_cap; a.split_list = cv.split_list; a.complex_list = cv.complex_list;
  a.entries = cv.entries;
  a.sepcols = cv.sepcols;
  a.geolocs = rc.geolocs;
  a.resample = rc.resample;
  a.sep = 1;   // separable row transform (plan_cols_kernel); 0 = three full transforms per row
#ifdef GSKYHIP_AB
  if (const char *sep = getenv("GSKYHIP_PLAN_SEP")) a.sep = atoi(sep);
#endif
  hipStream_t s = rc.stream;
  // per-granule edge samples, staged in the split-list region (plan_rows
  // writes that list only after plan_pairs has read the table), in one launch
  // with the pairs' owning tiles
  a.n_granules = rc.n_granules;
  a.gedge = nullptr;
  // small batches: pairs (a workgroup each, own edge samples and owning
  // tile), then every later planning step in one workgroup -- 2 launches
  // (and few rows to plan: the one workgroup plans every pair's rows, so a
  // tile over many granules goes faster through the multi-launch planner,
  // profiles/r04al_ab_plan_small_c5_c1.txt)
  bool small = rc.n_tiles <= kSmallBatchTiles && rc.n_pairs > 0 && rc.n_pairs <= kSmallBatchPlanPairs &&
               (int64_t)rc.n_pairs * rc.max_h <= kSmallBatchPlanRows;
#ifdef GSKYHIP_AB
  if (const char *sm = getenv("GSKYHIP_PLAN_SMALL")) small = small && atoi(sm) != 0;
#endif
  a.small = small ? (rc.n_pairs <= kFusedPlanPairs ? 2 : 1) : 0;
  if (small) {
    if (a.small == 1) hipLaunchKernelGGL(plan_pairs_kernel<256>, dim3(rc.n_pairs), dim3(256), 0, s, a);
    hipLaunchKernelGGL(plan_small_kernel, dim3(1), dim3(256), 0, s, a);
#ifdef GSKYHIP_AB
    if (getenv("GSKYHIP_PLAN_STAMPS")) {   // phase times of plan_small_kernel, 10 ns ticks
      int32_t st[16] = {0};
      hipStreamSynchronize(s);
      hipMemcpy(st, a.counters + 40, sizeof(st), hipMemcpyDeviceToHost);
      fprintf(stderr, "plan_small_stamps_us pairs=%.2f tiles=%.2f cols=%.2f rows=%.2f split=%.2f exact=%.2f"
              " | pair: setup=%.2f edges=%.2f extent=%.2f borderA=%.2f rest=%.2f\n",
              st[1] * 0.01, st[2] * 0.01, st[3] * 0.01, st[4] * 0.01, st[5] * 0.01, st[6] * 0.01,
              st[11] * 0.01, st[12] * 0.01, st[13] * 0.01, st[14] * 0.01, st[15] * 0.01);
    }
#endif
    return hipGetLastError() == hipSuccess ? 0 : GSKYHIP_E_HIP;
  }
  bool ge_on = true;   // per-granule edge table; false = per-pair edge transforms
#ifdef GSKYHIP_AB
  if (const char *ge_env = getenv("GSKYHIP_GRANULE_EDGES")) ge_on = atoi(ge_env) != 0;
#endif
  if (ge_on && rc.n_granules > 0 && rc.n_pairs > 0 &&
      (int64_t)sizeof(GEdge) * rc.n_granules <= (int64_t)sizeof(int64_t) * rc.n_pairs * rc.max_h)
    a.gedge = (GEdge *)cv.split_list;
  const int n_edge_blocks = a.gedge ? rc.n_granules : 0;
  hipLaunchKernelGGL(plan_prologue_kernel, dim3(std::max(1, n_edge_blocks + (rc.n_pairs + 127) / 128)), dim3(128),
                     0, s, a, n_edge_blocks);
  // small batches (C1: one pair) are latency-bound: a workgroup per pair
  int small_pairs = kSmallBatchPairs;
#ifdef GSKYHIP_AB
  if (const char *sp = getenv("GSKYHIP_PAIRS_SMALL")) small_pairs = atoi(sp);
#endif
  if (rc.n_pairs > 0 && rc.n_pairs <= small_pairs)
    hipLaunchKernelGGL(plan_pairs_kernel<256>, dim3(rc.n_pairs), dim3(256), 0, s, a);
  else if (rc.n_pairs > 0)
    hipLaunchKernelGGL(plan_pairs_kernel<64>, dim3(rc.n_pairs), dim3(64), 0, s, a);
  if (rc.n_pairs >= kTiles4MinPairsPerTile * rc.n_tiles)
    hipLaunchKernelGGL(plan_tiles4_kernel, dim3(rc.n_tiles), dim3(256), 0, s, a);
  else
    hipLaunchKernelGGL(plan_tiles_kernel, dim3(rc.n_tiles), dim3(64), 0, s, a);
  if (rc.n_pairs > 0) {
    if (a.sep)
      hipLaunchKernelGGL(plan_cols_kernel, dim3((unsigned)((3 * (int64_t)rc.n_pairs + 255) / 256)), dim3(256), 0, s,
                         a);
    hipLaunchKernelGGL(plan_rows_kernel, dim3(rc.n_pairs, (rc.max_h + 255) / 256), dim3(256), 0, s, a);
    hipLaunchKernelGGL(plan_split_kernel, dim3(1024), dim3(64), 0, s, a);
    hipLaunchKernelGGL(plan_exact_kernel, dim3(512), dim3(256), 0, s, a);
  }
  return hipGetLastError() == hipSuccess ? 0 : GSKYHIP_E_HIP;
}

// One value type for the whole batch (bit mask of GSKYHIP_VT_*): the typed
// LDS band kernel, else 0.
static int single_value_type(uint32_t vt) {
  switch (vt) {
    case GSKYHIP_VT_BYTE: return GSKYHIP_BYTE;
    case GSKYHIP_VT_SIGNEDBYTE: return GSKYHIP_SIGNEDBYTE;
    case GSKYHIP_VT_INT16: return GSKYHIP_INT16;
    case GSKYHIP_VT_UINT16: return GSKYHIP_UINT16;
    case GSKYHIP_VT_FLOAT32: return GSKYHIP_FLOAT32;
    default: return 0;
  }
}

int launch_render(const RenderCall &rc, const int32_t *out_ns, int n_out, const gskyhip_scale_params &sp,
                  const uint8_t *ramp, uint8_t *rgba_out, void *canvas_out, int phase) {
  if (n_out != 1 && n_out != 3) return GSKYHIP_E_ARG;  // ogc_encoders.go:135-136
  for (int k = 0; k < n_out; k++) if (out_ns[k] < 0 || out_ns[k] >= 4) return GSKYHIP_E_ARG;
  if (rc.resample != GSKYHIP_RESAMPLE_NEAREST && rc.resample != GSKYHIP_RESAMPLE_BILINEAR) return GSKYHIP_E_ARG;
  // rgba_out == NULL: canvases only (WCS GetCoverage, FusionUnscale, ows.go:728)
  const bool autom = rgba_out && sp.offset == 0.0 && sp.scale == 0.0 && sp.clip == 0.0;
  if ((autom || !rgba_out) && !canvas_out) return GSKYHIP_E_ARG;
  if (rc.n_tiles <= 0) return 0;
  Carve cv;
  if (phase != 2) {  // 0: plan + render, 1: plan only, 2: render only (plan done)
    int rcode = plan_all(rc, cv);
    if (rcode || phase == 1) return rcode;
  } else {
    if (!rc.workspace || rc.workspace_bytes < render_workspace_size(rc.n_tiles, rc.n_pairs, rc.max_h))
      return GSKYHIP_E_ARG;
    cv = carve(rc.workspace, rc.n_tiles, rc.n_pairs, rc.max_h);
  }
  RenderArgs a;
  a.pairs = cv.pairs; a.xforms = cv.xforms; a.tplans = cv.tplans; a.order = cv.order;
  a.tiles = rc.tiles; a.rows = cv.rows; a.rowfix = cv.rowfix; a.pool = cv.pool; a.counters = cv.counters;
  a.complex_list = cv.complex_list; a.max_h = rc.max_h; a.max_w = rc.max_w;
  a.n_tiles = rc.n_tiles; a.rows_per_block = 16; a.n_out = n_out;
  for (int k = 0; k < 3; k++) a.out_ns[k] = k < n_out ? out_ns[k] : -1;
  for (int k = 0; k < 4; k++) a.mask[k] = rc.mask_specs[k];
  a.sp = sp;
  a.autom = autom ? 1 : 0;
  a.ramp = (const uint32_t *)ramp;
  a.rgba = rgba_out;
  a.canvas = (uint8_t *)canvas_out;
  a.canvas_ns_stride = (long)rc.max_w * rc.max_h * 4;
  a.canvas_tile_stride = a.canvas_ns_stride * n_out;
  a.minmax = cv.minmax;
  a.entries = cv.entries;
  a.lds_mode = 0;
  a.cov_offsets = rc.cov_offsets;
  a.cov_stride = rc.cov_stride;
  const int bands = (rc.max_h + a.rows_per_block - 1) / a.rows_per_block;
  const dim3 grid((unsigned)(rc.n_tiles * bands));
  hipStream_t s = rc.stream;
  const bool mask = rc.mask_ns >= 0;
  if (autom) {
    hipLaunchKernelGGL(minmax_init_kernel, dim3((rc.n_tiles * 3 + 255) / 256), dim3(256), 0, s, cv.minmax,
                       rc.n_tiles * 3);
    a.write_rgba = 0;
  } else {
    a.write_rgba = rgba_out ? 1 : 0;
  }
  // One value type, one namespace, no auto-scale: the typed band kernel, for
  // RGBA output (GetMap) or typed canvases only (GetCoverage); complex tiles
  // (exact transforms, type promotion) still go to render_general_kernel.
  const int vt = single_value_type(rc.value_types);
  const bool bil = rc.resample == GSKYHIP_RESAMPLE_BILINEAR;
  int lds_mode = -1;
  if (vt && n_out == 1 && !autom) {
    if (a.write_rgba && !canvas_out) lds_mode = bil ? kBilinear : 0;
    else if (!rgba_out && canvas_out) lds_mode = kCanvas | (bil ? kBilinear : 0);
  }
  if (lds_mode >= 0) {
    a.lds_mode = lds_mode;
    const int n_items = rc.n_tiles * ((rc.max_h + kLdsBandRows - 1) / kLdsBandRows) * ((rc.max_w + 511) / 512);
    launch_band_kernels(a, vt, mask, n_items, s);
    dispatch_render_1(a, rc.resample, mask, grid, true, s);
  } else if (n_out == 1) {
    dispatch_render_1(a, rc.resample, mask, grid, false, s);
  } else {
    dispatch_render_3(a, rc.resample, mask, grid, false, s);
  }
  if (autom) {
    a.write_rgba = 1;
    hipLaunchKernelGGL(canvas_rgba_kernel, grid, dim3(256), 0, s, a);
  }
  return hipGetLastError() == hipSuccess ? 0 : GSKYHIP_E_HIP;
}

int launch_block_stats_batch(const RenderCall &rc, const BlockStatsJob *jobs, int n_jobs, int64_t max_px,
                             void *scratch, int32_t *stats) {
  if (n_jobs <= 0) return 0;
  const Carve cv = carve(rc.workspace, rc.n_tiles, rc.n_pairs, rc.max_h);
  hipStream_t s = rc.stream;
  hipLaunchKernelGGL(block_stats_init_kernel, dim3(n_jobs), dim3(256), 0, s, jobs, (char *)scratch, stats);
  if (max_px > 0)
    hipLaunchKernelGGL(block_stats_kernel, dim3((unsigned)((max_px + 255) / 256), n_jobs), dim3(256), 0, s, cv.pairs,
                       cv.xforms, cv.rows, cv.pool, rc.max_h, jobs, (char *)scratch, stats);
  hipLaunchKernelGGL(block_stats_resolve_kernel, dim3(n_jobs), dim3(64), 0, s, cv.pairs, jobs,
                     (const char *)scratch, stats);
  return hipGetLastError() == hipSuccess ? 0 : GSKYHIP_E_HIP;
}

int launch_pair_footprint(void *workspace, int n_tiles, int n_pairs, int max_h, int32_t *out, hipStream_t s) {
  if (n_pairs <= 0) return 0;
  const Carve cv = carve(workspace, n_tiles, n_pairs, max_h);
  hipLaunchKernelGGL(pair_footprint_kernel, dim3((n_pairs + 63) / 64), dim3(64), 0, s, cv.pairs, cv.rows, cv.pool,
                     n_pairs, max_h, out);
  return hipGetLastError() == hipSuccess ? 0 : GSKYHIP_E_HIP;
}

int launch_pair_touched(void *workspace, int n_tiles, int n_pairs, int max_h, int64_t *out2, hipStream_t s) {
  out2[0] = out2[1] = 0;
  if (n_pairs <= 0) return 0;
  const Carve cv = carve(workspace, n_tiles, n_pairs, max_h);
  std::vector<PairPlan> hp(n_pairs);
  if (hipMemcpyAsync(hp.data(), cv.pairs, sizeof(PairPlan) * n_pairs, hipMemcpyDeviceToHost, s) != hipSuccess ||
      hipStreamSynchronize(s) != hipSuccess)
    return GSKYHIP_E_HIP;
  // one element map and one line map per distinct level (band pointer), 32-bit aligned segments
  struct Seg { int64_t ebit, lbit; };
  std::map<const void *, Seg> segs;
  std::vector<int64_t> base(2 * (size_t)n_pairs, -1), ew, lw;   // ew / lw: (first word, bytes per bit)
  int64_t ebits = 0, lbits = 0;
  for (int p = 0; p < n_pairs; p++) {
    const PairPlan &pp = hp[p];
    if (!pp.band || pp.w <= 0 || pp.h <= 0 || pp.band_x <= 0 || pp.band_y <= 0) continue;
    auto it = segs.find(pp.band);
    if (it == segs.end()) {
      const int es = type_size(pp.src_dtype);
      const int64_t n = (int64_t)pp.band_x * pp.band_y, nl = (n * es + 127) / 128;
      ew.push_back(ebits / 32); ew.push_back(es);
      lw.push_back(lbits / 32); lw.push_back(128);
      it = segs.emplace(pp.band, Seg{ebits, lbits}).first;
      ebits += (n + 31) / 32 * 32;
      lbits += (nl + 31) / 32 * 32;
    }
    base[2 * p] = it->second.ebit;
    base[2 * p + 1] = it->second.lbit;
  }
  if (segs.empty()) return 0;
  const int64_t ew_words = ebits / 32, lw_words = lbits / 32;
  const size_t bytes = (size_t)(ew_words + lw_words) * 4 + base.size() * 8 + (ew.size() + lw.size()) * 8 + 16;
  char *dev = nullptr;
  if (hipMalloc((void **)&dev, bytes) != hipSuccess) return GSKYHIP_E_HIP;
  uint32_t *eb = (uint32_t *)dev, *lb = eb + ew_words;
  int64_t *dbase = (int64_t *)(lb + lw_words + ((ew_words + lw_words) & 1));
  int64_t *dew = dbase + base.size(), *dlw = dew + ew.size();
  unsigned long long *cnt = (unsigned long long *)(dlw + lw.size());
  int rc = 0;
  if (hipMemsetAsync(dev, 0, (size_t)(ew_words + lw_words) * 4, s) != hipSuccess ||
      hipMemsetAsync(cnt, 0, 16, s) != hipSuccess ||
      hipMemcpyAsync(dbase, base.data(), base.size() * 8, hipMemcpyHostToDevice, s) != hipSuccess ||
      hipMemcpyAsync(dew, ew.data(), ew.size() * 8, hipMemcpyHostToDevice, s) != hipSuccess ||
      hipMemcpyAsync(dlw, lw.data(), lw.size() * 8, hipMemcpyHostToDevice, s) != hipSuccess)
    rc = GSKYHIP_E_HIP;
  if (!rc) {
    hipLaunchKernelGGL(pair_touch_kernel, dim3((unsigned)n_pairs, (unsigned)((max_h + 3) / 4)), dim3(256), 0, s,
                       cv.pairs, cv.rows, cv.pool, max_h, dbase, eb, lb);
    hipLaunchKernelGGL(popcount_kernel, dim3(1024), dim3(256), 0, s, eb, ew_words, dew, (int)(ew.size() / 2), cnt);
    hipLaunchKernelGGL(popcount_kernel, dim3(1024), dim3(256), 0, s, lb, lw_words, dlw, (int)(lw.size() / 2), cnt + 1);
    unsigned long long h[2] = {0, 0};
    if (hipGetLastError() != hipSuccess || hipMemcpyAsync(h, cnt, 16, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
      rc = GSKYHIP_E_HIP;
    out2[0] = (int64_t)h[0];
    out2[1] = (int64_t)h[1];
  }
  (void)hipFree(dev);
  return rc;
}

int launch_warp_jobs(const RenderCall &rc, const BlockStatsJob *jobs, int64_t max_px, void *scratch,
                     int32_t *stats, uint8_t *const *outs, WarpResult *results) {
  Carve cv;
  int rcode = plan_all(rc, cv);
  if (rcode || rc.n_pairs <= 0) return rcode;
  hipStream_t s = rc.stream;
  const int n = rc.n_pairs;
  hipLaunchKernelGGL(block_stats_init_kernel, dim3(n), dim3(256), 0, s, jobs, (char *)scratch, stats);
  if (max_px > 0) {
    // eight pixels per thread, 8-32 bytes in one or two stores (service leg,
    // 16 / 64 workers: 1 px 32.3k / 48.4k req/s, 4 px 42.1-43.4k / 61.3-66.2k,
    // 8 px 44.8k / 62.7-63.4k; profiles/r05f_svc.txt, r05g_svc.txt);
    // GSKYHIP_SVC_PX=1/4 selects the others
    static const int env_px = [] {
      const char *e = getenv("GSKYHIP_SVC_PX");
      const int v = e ? atoi(e) : 8;
      return v == 1 || v == 4 ? v : 8;
    }();
    const int px = rc.resample == GSKYHIP_RESAMPLE_BILINEAR ? 1 : env_px;
    const dim3 grid((unsigned)((max_px + 256 * px - 1) / (256 * px)), n);
    if (rc.resample == GSKYHIP_RESAMPLE_BILINEAR)
      hipLaunchKernelGGL(warp_job_kernel<GSKYHIP_RESAMPLE_BILINEAR>, grid, dim3(256), 0, s, cv.pairs, cv.xforms,
                         cv.rows, cv.pool, rc.max_h, jobs, (char *)scratch, stats, outs);
    else if (px == 4)
      hipLaunchKernelGGL((warp_job_kernel<GSKYHIP_RESAMPLE_NEAREST, 4>), grid, dim3(256), 0, s, cv.pairs, cv.xforms,
                         cv.rows, cv.pool, rc.max_h, jobs, (char *)scratch, stats, outs);
    else if (px == 8)
      hipLaunchKernelGGL((warp_job_kernel<GSKYHIP_RESAMPLE_NEAREST, 8>), grid, dim3(256), 0, s, cv.pairs, cv.xforms,
                         cv.rows, cv.pool, rc.max_h, jobs, (char *)scratch, stats, outs);
    else
      hipLaunchKernelGGL(warp_job_kernel<GSKYHIP_RESAMPLE_NEAREST>, grid, dim3(256), 0, s, cv.pairs, cv.xforms,
                         cv.rows, cv.pool, rc.max_h, jobs, (char *)scratch, stats, outs);
  }
  hipLaunchKernelGGL(warp_job_resolve_kernel, dim3((n + 63) / 64), dim3(64), 0, s, cv.pairs, jobs,
                     (const char *)scratch, stats, n, results);
  return hipGetLastError() == hipSuccess ? 0 : GSKYHIP_E_HIP;
}

int launch_warp_windows(const RenderCall &rc, int32_t *bbox_out, int32_t *dtype_out, double *nodata_out,
                        void *win_out, int64_t win_stride) {
  Carve cv;
  int rcode = plan_all(rc, cv);
  if (rcode || rc.n_pairs <= 0) return rcode;
  hipStream_t s = rc.stream;
  hipLaunchKernelGGL(pair_meta_kernel, dim3((rc.n_pairs + 255) / 256), dim3(256), 0, s, cv.pairs, rc.n_pairs,
                     bbox_out, dtype_out, nodata_out);
  const int64_t nthreads = (int64_t)rc.n_pairs * rc.max_h * rc.max_w;
  const dim3 grid((unsigned)((nthreads + 255) / 256));
  if (rc.resample == GSKYHIP_RESAMPLE_BILINEAR)
    hipLaunchKernelGGL(warp_window_kernel<GSKYHIP_RESAMPLE_BILINEAR>, grid, dim3(256), 0, s, cv.pairs, cv.xforms,
                       cv.rows, cv.pool, rc.max_h, rc.max_w, rc.n_pairs, (uint8_t *)win_out, (long)win_stride);
  else
    hipLaunchKernelGGL(warp_window_kernel<GSKYHIP_RESAMPLE_NEAREST>, grid, dim3(256), 0, s, cv.pairs, cv.xforms,
                       cv.rows, cv.pool, rc.max_h, rc.max_w, rc.n_pairs, (uint8_t *)win_out, (long)win_stride);
  return hipGetLastError() == hipSuccess ? 0 : GSKYHIP_E_HIP;
}

}  // namespace gsky
