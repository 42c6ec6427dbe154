// render_bil.h -- bilinear band kernel for float32 typed canvases (WCS
// GetCoverage, BASELINE C3), shaped like render_nn_kernel (render_nn.h):
//
//   * a wave owns RPW consecutive rows of a 512-column block; a lane the 8
//     pixels lane, lane + 64, ..., lane + 448 of each row, so one row of one
//     entry is a single scalar chain (order -> descriptor -> row record) for
//     all 512 columns, and every tap load and canvas store instruction covers
//     64 consecutive output columns;
//   * per pixel GWKBilinearResample4Sample (GDAL 3.0.1): the fp64 source
//     coordinate of the row record, the 2x2 taps at floor(s - 0.5) with the
//     reference's -1 edge rule, taps outside the band or equal to the band's
//     nodata dropped and the weights renormalised (accDiv), no sample below
//     accDiv 1e-5; the four taps arrive as two 8-byte buffer loads (x and
//     x + 1 of the two source rows), issued for 4 pixels before the first
//     wait; taps outside the band read 0 through the buffer range check and
//     are dropped by their validity flag;
//   * W = float (default): tap selection and fractions from the same fp64
//     coordinates, weights and sums in fp32 -- on C3 71 % of pixels
//     bit-identical to GDAL's fp64 expressions, the rest within 1.6e-7
//     relative (north_star's bar: 1e-4), 17 % faster (render 0.94 vs
//     1.13 ms, profiles/r03b_ab_c3.jsonl);
//     W = double (A/B build, GSKYHIP_BIL_F32=0): the weights and sums in
//     fp64, the expressions of bil_sample() (render_lds.h);
//   * the fp64 division runs only for pixels whose accDiv is not exactly 1
//     (a tap dropped): the others take accR as it is.
#pragma once
#include "render_nn.h"

namespace gsky {


// The sample of one pixel whose 2x2 taps are all inside the band (t0: x and
// x + 1 of the upper source row, t1 of the lower; rx / ry the weights of x
// and y) and its fold into the canvas value c: the four weights sum to 1
// within fp32 rounding, so the sample is accR unless a tap holds nodata
// (then the taps are dropped and the weights renormalised: bil_sample's
// rule).  The dropped-tap sums are formed for every pixel (a few selects);
// only their division sits behind a branch.  NaN nodata: the fp64 path.
template <typename WT>
__device__ __forceinline__ void bil_fold4(u32x2 t0, u32x2 t1, WT rx, WT ry, int ic, int lim, float nd, float ndf,
                                          bool hnd, float fillv, bool fill_mode, float &c) {
  const float tv[4] = {__uint_as_float(t0.x), __uint_as_float(t0.y), __uint_as_float(t1.x), __uint_as_float(t1.y)};
  const WT one = (WT)1.0;
  const WT wx[2] = {rx, one - rx}, wy[2] = {ry, one - ry};
  WT accR = (WT)0.0, aR = (WT)0.0, aD = (WT)0.0;
  bool anynd = false;
#pragma unroll
  for (int kk = 0; kk < 4; kk++) {
    const WT w = wx[kk & 1] * wy[kk >> 1];
    const WT p = (WT)tv[kk] * w;
    const bool isnd = hnd & (tv[kk] == ndf);
    accR += p;
    aR += isnd ? (WT)0.0 : p;
    aD += isnd ? (WT)0.0 : w;
    anynd = anynd | isnd;
  }
  float v = (float)accR;
  if (anynd) {
    v = fillv;
    if (aD == (WT)1.0) v = (float)aR;
    else if (aD >= (WT)0.00001) v = (float)(aR / aD);
  }
  const bool take = ((unsigned)ic < (unsigned)lim) & (v != nd) & (!fill_mode | (c == nd));
  c = take ? v : c;
}

// Typed float canvas row (tile_merger.go:562-652), at the chunk's place in
// the coverage: 8 non-temporal stores per lane, each covering 64 columns.
__device__ __forceinline__ void bil_store(const RenderArgs &a, int t, int r, int xl, int lane, bool full, int ncols,
                                          const float (&c)[kNnPx]) {
  const int64_t eo = a.cov_offsets ? a.cov_offsets[t] + (int64_t)r * a.cov_stride + xl : (int64_t)r * a.max_w + xl;
  float *cdst = (float *)(a.cov_offsets ? a.canvas : a.canvas + t * a.canvas_tile_stride) + eo;
  if (full) {
#pragma unroll
    for (int q = 0; q < kNnPx; q++) __builtin_nontemporal_store(__float_as_uint(c[q]), (GPTR(uint32_t))(cdst + 64 * q));
  } else {
#pragma unroll
    for (int q = 0; q < kNnPx; q++)
      if (64 * q + lane < ncols) __builtin_nontemporal_store(__float_as_uint(c[q]), (GPTR(uint32_t))(cdst + 64 * q));
  }
}

// Separable rows (EPSG:4326 -> 3857: the source x depends on the
// destination column only, the source y on the row only).  A wave (rows r0 ..
// r0 + nrows - 1 of the block's columns) is eligible when exactly one entry
// reaches those rows and columns, it covers every one of the rows, the rows
// are LINEAR with the same (xs0, dX) and dY == 0 -- bit for bit, as plan_row
// writes them from the shared column parts -- the band's nodata is exact in
// float32, and every sampled pixel's 2x2 taps lie inside the band (no -1 edge
// rule, no tap outside).  Then each lane's x taps and weights serve all the
// wave's rows and a row's y tap and weight are one uniform value.  Wave-uniform.
struct BilSep {
  int entry;
  double xs0, dX;
};
#ifdef GSKYHIP_AB
// A/B build, GSKYHIP_BIL_SEPSTAT=1: waves reaching each eligibility test
// (0 checked, 1 one entry, 2 rows covered, 3 rows same / in band, 4 taps in band)
__device__ unsigned long long g_bil_sep_stat[8];
#define SEPSTAT(i) do { if (stat && __lane_id() == 0) atomicAdd(&g_bil_sep_stat[i], 1ull); } while (0)
#else
#define SEPSTAT(i) ((void)0)
#endif
template <typename WT>
__device__ __forceinline__ bool bil_sep_eligible(const EntryD *__restrict__ ents, const int32_t *__restrict__ ord,
                                                 int n_entries, const RowRec *__restrict__ rows, int ns_out, int r0,
                                                 int nrows, int xb, int ncols, int W, int xl, BilSep &sp,
                                                 bool stat = false) {
  SEPSTAT(0);
  int found = -1, n_touch = 0;
  for (int k = 0; k < n_entries; k++) {
    const int ek = ord[k];
    const EntryD &e = ents[ek];
    if (e.ns != ns_out || e.w <= 0) continue;
    if (r0 + nrows <= e.yoff || r0 >= e.yoff + e.h) continue;   // no row of the wave in the entry's window
    const int lim = max(0, min(e.w, W - e.xoff));
    const int c0 = e.xoff - xb, c1 = e.xoff + lim - xb;
    if (c1 <= 0 || c0 >= ncols) continue;                        // no column of the block
    n_touch++;
    found = ek;
  }
  if (n_touch != 1) return false;
  SEPSTAT(1);
  const EntryD &e = ents[found];
  const double nd64 = e.nodata64;
  const bool nd_f32 = e.has_nodata == 0 || nd64 != nd64 || (double)(float)nd64 == nd64;
  if (!nd_f32 || r0 < e.yoff || r0 + nrows > e.yoff + e.h) return false;
  SEPSTAT(2);
  const RowRec *rr0 = rows + e.row_base + (r0 - e.yoff);
  const double xs0 = uni64d(rr0->v[0]), dX = uni64d(rr0->v[2]);
  const int ic0 = xl - e.xoff;
  bool ok = true;
  for (int j = 0; j < nrows; j++) {
    const RowRec *rj = rr0 + j;
    const double sy = uni64d(rj->v[1]) + uni64d(rj->v[3]) * (double)ic0;
    const int iy = (int)floor(sy - 0.5);
    ok = ok & (__builtin_amdgcn_readfirstlane(rj->kind) == ROW_LINEAR) & (uni64d(rj->v[0]) == xs0) &
         (uni64d(rj->v[2]) == dX) & (uni64d(rj->v[3]) == 0.0) & ((unsigned)iy < (unsigned)(e.band_y - 1));
  }
  if (!ok) return false;
  SEPSTAT(3);
  const int lim = max(0, min(e.w, W - e.xoff));
  bool xin = true;
#pragma unroll
  for (int q = 0; q < kNnPx; q++) {
    const int ic = ic0 + 64 * q;
    const double sx = xs0 + dX * (double)ic;
    const int ix = (int)floor(sx - 0.5);
    xin = xin & (((unsigned)ic >= (unsigned)lim) | ((unsigned)ix < (unsigned)(e.band_x - 1)));
  }
  if (!__all(xin)) return false;
  SEPSTAT(4);
  sp.entry = found;
  sp.xs0 = xs0;
  sp.dX = dX;
  return true;
}

// The waves render_bil_kernel leaves to it (bil_sep_eligible): per lane the
// pixels' x tap offsets and weights once for all the wave's rows, per row one
// uniform y tap and weight, the next row's taps in flight while a row is
// folded and stored (HP == 0), or 8 pixels a lane with HP pixels' taps in
// flight and 8 stores a row; the same expressions as render_bil_kernel's
// all-inside path, so the same values.
template <typename WT, int RPW, int HP, int WPS>
__global__ __launch_bounds__(256, WPS) void render_bil_sep_kernel(RenderArgs a, const EntryD *__restrict__ ents,
                                                                const int32_t *__restrict__ order,
                                                                const RowRec *__restrict__ rows,
                                                                const TilePlan *__restrict__ tplans,
                                                                const gskyhip_tile *__restrict__ tiles, int n_items) {
  constexpr int kRowsBlk = 4 * RPW;
  int item = blockIdx.x;
  if (a.ab_xcd == 2) {   // A/B: XCD x (blockIdx % 8) takes the x-th contiguous eighth of the items
    const int per = (n_items + 7) >> 3;
    item = (int)(blockIdx.x & 7) * per + (int)(blockIdx.x >> 3);
  }
  if (item >= n_items) return;
  const int bands_per_tile = (a.max_h + kRowsBlk - 1) / kRowsBlk;
  const int col_blocks = (a.max_w + kBandCols - 1) / kBandCols;
  const int t = item / (bands_per_tile * col_blocks);
  const int in_tile = item - t * bands_per_tile * col_blocks;
  const TilePlan &tp = tplans[t];
  if (tp.complex || tp.n_entries <= 0 || tp.vt != GSKYHIP_FLOAT32) return;
  const gskyhip_tile &tile = tiles[t];
  const int W = tile.width, H = tile.height;
  const int band0 = (in_tile / col_blocks) * kRowsBlk;
  const int xb = (in_tile % col_blocks) * kBandCols;
  if (band0 >= H || xb >= W) return;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int r0 = band0 + wave * RPW;
  if (r0 >= H) return;
  const int ns_out = a.out_ns[0];
  const int32_t *ord = order + tile.pair_begin;
  const int ncols = min(kBandCols, W - xb);
  const bool full = ncols == kBandCols;
  const int xl = xb + lane;
  const int nrows = min(RPW, H - r0);
  BilSep sp;
  if (!bil_sep_eligible<WT>(ents, ord, tp.n_entries, rows, ns_out, r0, nrows, xb, ncols, W, xl, sp,
                           a.ab_mode == 0x5E9)) return;
  const float cnod = go_conv_to(tp.nodata[ns_out], tp.dtype[ns_out]).f;
  const EntryD &e = ents[sp.entry];
  const int bx = e.band_x, by = e.band_y;
  const int lim = max(0, min(e.w, W - e.xoff));
  const int ic0 = xl - e.xoff;
  const RowRec *rr0 = rows + e.row_base + (r0 - e.yoff);
  if constexpr (HP == 0) {   // pipelined halves
  const double nd64 = e.nodata64;
  const float nd = e.nd.f, fillv = e.fill.f, ndf = (float)nd64;
  const bool hnd = e.has_nodata != 0, nd_nan = nd64 != nd64;
  const bool take_any = (e.fill_mode == 0) | (cnod == nd);   // one entry: the canvas holds its nodata
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void *)uniform_ptr(e.band), (short)0,
                                                                      (int)((int64_t)bx * by * 4), 0x00020000);
  // each row's y tap (byte offset of its upper source row) and weight: uniform
  uint32_t ybase[RPW];
  WT ryv[RPW];
#pragma unroll
  for (int j = 0; j < RPW; j++) {
    const RowRec *rj = rr0 + (j < nrows ? j : 0);
    const double sy = uni64d(rj->v[1]) + uni64d(rj->v[3]) * (double)ic0;
    const int iy = (int)floor(sy - 0.5);
    ryv[j] = (WT)(1.5 - (sy - (double)iy));
    ybase[j] = (uint32_t)(iy * bx) * 4u;
  }
  const int64_t eo0 = a.cov_offsets ? a.cov_offsets[t] + (int64_t)r0 * a.cov_stride + xl : (int64_t)r0 * a.max_w + xl;
  const int64_t row_stride = a.cov_offsets ? a.cov_stride : a.max_w;
  float *cbase = (float *)(a.cov_offsets ? a.canvas : a.canvas + t * a.canvas_tile_stride) + eo0;
  // the block's 512 columns in two halves of 4 pixels per lane, each half
  // down all the rows with the next row's taps loaded while this row's are
  // folded and stored (so a row's loads never wait on the stores before them)
#pragma unroll 1
  for (int hh = 0; hh < kNnPx; hh += 4) {
    // per lane and pixel: the x tap's byte offset (past the buffer for a pixel
    // outside the window: its loads read 0 and it is not taken), the x weight
    uint32_t xo[4];
    WT rxv[4];
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const int ic = ic0 + 64 * (hh + q);
      const double sx = sp.xs0 + sp.dX * (double)ic;
      const int ix = (int)floor(sx - 0.5);
      rxv[q] = (WT)(1.5 - (sx - (double)ix));
      xo[q] = (unsigned)ic < (unsigned)lim ? (uint32_t)ix * 4u : 0x80000000u;
    }
    u32x2 ta[2][4], tb[2][4];
    auto issue = [&](int j, u32x2 (&A)[4], u32x2 (&B)[4]) {
      const uint32_t b0 = ybase[j], b1 = b0 + (uint32_t)bx * 4u;
#pragma unroll
      for (int q = 0; q < 4; q++) {
        A[q] = __builtin_amdgcn_raw_buffer_load_b64(rs, b0 + xo[q], 0, 0);
        B[q] = __builtin_amdgcn_raw_buffer_load_b64(rs, b1 + xo[q], 0, 0);
      }
    };
    issue(0, ta[0], tb[0]);
#pragma unroll
    for (int j = 0; j < RPW; j++) {
      if (j >= nrows) break;
      if (j + 1 < nrows) issue(j + 1, ta[(j + 1) & 1], tb[(j + 1) & 1]);
      const WT one = (WT)1.0;
      const WT wy[2] = {ryv[j], one - ryv[j]};
      float *cdst = cbase + (int64_t)j * row_stride;
#pragma unroll
      for (int q = 0; q < 4; q++) {
        const u32x2 t0 = ta[j & 1][q], t1 = tb[j & 1][q];
        const float tv[4] = {__uint_as_float(t0.x), __uint_as_float(t0.y), __uint_as_float(t1.x),
                             __uint_as_float(t1.y)};
        const WT wx[2] = {rxv[q], one - rxv[q]};
        WT accR = (WT)0.0;
        bool anynd = false;
#pragma unroll
        for (int kk = 0; kk < 4; kk++) {
          accR += (WT)tv[kk] * (wx[kk & 1] * wy[kk >> 1]);
          anynd = anynd | (nd_nan ? (tv[kk] != tv[kk]) : (tv[kk] == ndf));
        }
        anynd = anynd & hnd;
        float v = (float)accR;
        if (anynd) {   // drop the nodata taps and renormalise (bil_sample's rule)
          WT aR = (WT)0.0, aD = (WT)0.0;
#pragma unroll
          for (int kk = 0; kk < 4; kk++) {
            const WT w = wx[kk & 1] * wy[kk >> 1];
            const bool use = !(nd_nan ? (tv[kk] != tv[kk]) : (tv[kk] == ndf));
            aD += use ? w : (WT)0.0;
            aR += use ? (WT)tv[kk] * w : (WT)0.0;
          }
          v = fillv;
          if (aD == (WT)1.0) v = (float)aR;
          else if (aD >= (WT)0.00001) v = (float)(aR / aD);
        }
        const bool take = (xo[q] != 0x80000000u) & (v != nd) & take_any;
        const float o = take ? v : cnod;
        if (full || 64 * (hh + q) + lane < ncols)
          __builtin_nontemporal_store(__float_as_uint(o), (GPTR(uint32_t))(cdst + 64 * (hh + q)));
      }
      __builtin_amdgcn_sched_barrier(0);   // rows stay in order: two rows' taps live, not all of them
    }
  }
  } else {   // 8 pixels a lane, HP taps in flight, 8 stores a row
  // per lane and pixel: the x tap's byte offset (past the buffer for a pixel
  // outside the window: its loads read 0 and it is not taken), the x weight
  uint32_t xo[kNnPx];
  WT rxv[kNnPx];
#pragma unroll
  for (int q = 0; q < kNnPx; q++) {
    const int ic = ic0 + 64 * q;
    const double sx = sp.xs0 + sp.dX * (double)ic;
    const int ix = (int)floor(sx - 0.5);
    rxv[q] = (WT)(1.5 - (sx - (double)ix));
    xo[q] = (unsigned)ic < (unsigned)lim ? (uint32_t)ix * 4u : 0x80000000u;
  }
  const double nd64 = e.nodata64;
  const float nd = e.nd.f, fillv = e.fill.f, ndf = (float)nd64;
  const bool hnd = e.has_nodata != 0, nd_nan = nd64 != nd64;
  const bool take_any = (e.fill_mode == 0) | (cnod == nd);   // one entry: the canvas holds its nodata
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void *)uniform_ptr(e.band), (short)0,
                                                                      (int)((int64_t)bx * by * 4), 0x00020000);
#pragma unroll 1
  for (int j = 0; j < nrows; j++) {
    const RowRec *rj = rr0 + j;
    const double sy = uni64d(rj->v[1]) + uni64d(rj->v[3]) * (double)ic0;
    const int iy = (int)floor(sy - 0.5);
    const WT ry = (WT)(1.5 - (sy - (double)iy));
    const WT one = (WT)1.0;
    const WT wy[2] = {ry, one - ry};
    const uint32_t base0 = (uint32_t)(iy * bx) * 4u, base1 = base0 + (uint32_t)bx * 4u;
    float c[kNnPx];
#pragma unroll
    for (int h = 0; h < kNnPx; h += HP) {
      u32x2 t0[HP], t1[HP];
#pragma unroll
      for (int q = 0; q < HP; q++) {
        t0[q] = __builtin_amdgcn_raw_buffer_load_b64(rs, base0 + xo[h + q], 0, 0);
        t1[q] = __builtin_amdgcn_raw_buffer_load_b64(rs, base1 + xo[h + q], 0, 0);
      }
#pragma unroll
      for (int q = 0; q < HP; q++) {
        const float tv[4] = {__uint_as_float(t0[q].x), __uint_as_float(t0[q].y), __uint_as_float(t1[q].x),
                             __uint_as_float(t1[q].y)};
        const WT wx[2] = {rxv[h + q], one - rxv[h + q]};
        WT accR = (WT)0.0;
        bool anynd = false;
#pragma unroll
        for (int kk = 0; kk < 4; kk++) {
          accR += (WT)tv[kk] * (wx[kk & 1] * wy[kk >> 1]);
          anynd = anynd | (nd_nan ? (tv[kk] != tv[kk]) : (tv[kk] == ndf));
        }
        anynd = anynd & hnd;
        float v = (float)accR;
        if (anynd) {   // drop the nodata taps and renormalise (bil_sample's rule)
          WT aR = (WT)0.0, aD = (WT)0.0;
#pragma unroll
          for (int kk = 0; kk < 4; kk++) {
            const WT w = wx[kk & 1] * wy[kk >> 1];
            const bool use = !(nd_nan ? (tv[kk] != tv[kk]) : (tv[kk] == ndf));
            aD += use ? w : (WT)0.0;
            aR += use ? (WT)tv[kk] * w : (WT)0.0;
          }
          v = fillv;
          if (aD == (WT)1.0) v = (float)aR;
          else if (aD >= (WT)0.00001) v = (float)(aR / aD);
        }
        const bool take = (xo[h + q] != 0x80000000u) & (v != nd) & take_any;
        c[h + q] = take ? v : cnod;
      }
    }
    bil_store(a, t, r0 + j, xl, lane, full, ncols, c);
  }
  }
}

// HP: pixels whose taps are in flight together; WPS: waves per SIMD the
// register budget is sized for.
template <typename WT, int RPW, int HP, int WPS, bool FIX = true, bool SEP = true>
__global__ __launch_bounds__(256, WPS) void render_bil_kernel(RenderArgs a, const EntryD *__restrict__ ents,
                                                            const int32_t *__restrict__ order,
                                                            const RowRec *__restrict__ rows,
                                                            const RowFix *__restrict__ rowfix,
                                                            const Leaf *__restrict__ pool,
                                                            const TilePlan *__restrict__ tplans,
                                                            const gskyhip_tile *__restrict__ tiles, int n_items) {
  constexpr int kRowsBlk = 4 * RPW;
  const int item = blockIdx.x;
  if (item >= n_items) return;
  const int bands_per_tile = (a.max_h + kRowsBlk - 1) / kRowsBlk;
  const int col_blocks = (a.max_w + kBandCols - 1) / kBandCols;
  const int t = item / (bands_per_tile * col_blocks);
  const int in_tile = item - t * bands_per_tile * col_blocks;
  const TilePlan &tp = tplans[t];
  if (tp.complex || (tp.n_entries > 0 && tp.vt != GSKYHIP_FLOAT32)) return;   // empty tiles: written here
  const gskyhip_tile &tile = tiles[t];
  const int W = tile.width, H = tile.height;
  const int band0 = (in_tile / col_blocks) * kRowsBlk;
  const int xb = (in_tile % col_blocks) * kBandCols;
  if (band0 >= H || xb >= W) return;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int r0 = band0 + wave * RPW;
  if (r0 >= H) return;

  const int ns_out = a.out_ns[0];
  const float cnod = go_conv_to(tp.nodata[ns_out], tp.dtype[ns_out]).f;
  const int32_t *ord = order + tile.pair_begin;
  const int n_entries = tp.n_entries;
  const int ncols = min(kBandCols, W - xb);
  const bool full = ncols == kBandCols;
  const int xl = xb + lane;

  // waves whose rows are separable run in render_bil_sep_kernel
  if (SEP && n_entries > 0) {
    BilSep sp;
    if (bil_sep_eligible<WT>(ents, ord, n_entries, rows, ns_out, r0, min(RPW, H - r0), xb, ncols, W, xl, sp)) return;
  }

#pragma unroll 1
  for (int j = 0; j < RPW; j++) {
    const int r = r0 + j;
    if (r >= H) break;
    float c[kNnPx];
#pragma unroll
    for (int q = 0; q < kNnPx; q++) c[q] = cnod;

#pragma unroll 1
    for (int k = 0; k < n_entries; k++) {
      const EntryD &e = ents[ord[k]];
      const int eyoff = e.yoff, eh = e.h, exoff = e.xoff, ew = e.w;
      if (e.ns != ns_out || ew <= 0) continue;
      const int ir = r - eyoff;
      if (ir < 0 || ir >= eh) continue;
      const int lim = max(0, min(ew, W - exoff));
      const int c0 = exoff - xb, c1 = exoff + lim - xb;
      if (c1 <= 0 || c0 >= ncols) continue;
      const RowRec *rr = rows + e.row_base + ir;
      const int kind = __builtin_amdgcn_readfirstlane(rr->kind);
      const int bx = e.band_x, by = e.band_y;
      const float nd = e.nd.f, fillv = e.fill.f;
      const bool fill_mode = e.fill_mode != 0;
      const bool hnd = e.has_nodata != 0;
      const double nd64 = e.nodata64;
      const bool nd_nan = nd64 != nd64;
      const int ic0 = xl - exoff;
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
          (void *)uniform_ptr(e.band), (short)0, (int)((int64_t)bx * by * 4), 0x00020000);
      // one pixel: tap addresses + fractions (prep), then the sample and the fold (finish)
      auto prep = [&](int q, double sx, double sy, bool ok, WT &rx, WT &ry, uint32_t &valid, u32x2 &t0, u32x2 &t1) {
        const double fx = floor(sx - 0.5), fy = floor(sy - 0.5);
        const int iSrcX = (int)fx, iSrcY = (int)fy;
        double drx = 1.5 - (sx - (double)iSrcX), dry = 1.5 - (sy - (double)iSrcY);
        const int lx = iSrcX == -1 ? 0 : iSrcX, ly = iSrcY == -1 ? 0 : iSrcY;
        drx = iSrcX == -1 ? 1.0 : drx;
        dry = iSrcY == -1 ? 1.0 : dry;
        rx = (WT)drx;
        ry = (WT)dry;
        const uint32_t x0in = (unsigned)lx < (unsigned)bx, x1in = (unsigned)(lx + 1) < (unsigned)bx;
        const uint32_t y0in = (unsigned)ly < (unsigned)by, y1in = (unsigned)(ly + 1) < (unsigned)by;
        // bit k: tap k (x + (k & 1), y + (k >> 1)) inside the band; bit 4: a sample is taken
        valid = ok ? ((x0in & y0in) | ((x1in & y0in) << 1) | ((x0in & y1in) << 2) | ((x1in & y1in) << 3) | 16u) : 0u;
        // no sample: an offset past the band (< 2 GiB) reads 0 without a fetch
        const uint32_t o0 = ok ? (uint32_t)(ly * bx + lx) * 4u : 0x80000000u;
        const uint32_t o1 = ok ? o0 + (uint32_t)bx * 4u : 0x80000000u;
        t0 = __builtin_amdgcn_raw_buffer_load_b64(rs, o0, 0, 0);
        t1 = __builtin_amdgcn_raw_buffer_load_b64(rs, o1, 0, 0);
      };
      auto finish = [&](int q, WT rx, WT ry, uint32_t valid, u32x2 t0, u32x2 t1) {
        const float tv[4] = {__uint_as_float(t0.x), __uint_as_float(t0.y), __uint_as_float(t1.x),
                             __uint_as_float(t1.y)};
        const WT one = (WT)1.0;
        const WT wx[2] = {rx, one - rx}, wy[2] = {ry, one - ry};
        WT accR = (WT)0.0, accDiv = (WT)0.0;
#pragma unroll
        for (int kk = 0; kk < 4; kk++) {
          const WT w = wx[kk & 1] * wy[kk >> 1];
          const double d = (double)tv[kk];
          // bitwise, not short-circuit: no per-pixel exec-mask branches
          const bool isnd = (d == nd64) | (nd_nan & (d != d));
          const bool use = (((valid >> kk) & 1u) != 0u) & !(hnd & isnd);
          accDiv += use ? w : (WT)0.0;
          accR += use ? (WT)d * w : (WT)0.0;
        }
        float v = fillv;
        if (valid & 16u) {
          if (accDiv == (WT)1.0) v = (float)accR;
          else if (accDiv >= (WT)0.00001) v = (float)(accR / accDiv);
        }
        const int ic = ic0 + 64 * q;
        const bool take = ((unsigned)ic < (unsigned)lim) & (v != nd) & (!fill_mode | (c[q] == nd));
        c[q] = take ? v : c[q];
      };
      // the nodata test of a tap in float32 (exact: the band's nodata is a float32 value or NaN)
      const bool nd_f32 = !hnd || nd_nan || (double)(float)nd64 == nd64;
      const float ndf = (float)nd64;
      bool fixed_done = false;
      if (FIX && kind == ROW_LINEAR && nd_f32 && !nd_nan) {
        // the row's fixed-point form (RowFix): s - 0.5 as 32.32 integers --
        // the tap is the integer part, the fraction gives the weight
        // (rx = 1.5 - (s - floor(s - 0.5)) = 1 - frac), two 64-bit adds per
        // axis and pixel instead of the fp64 coordinate, floor and weight
        // expressions.  Rows where some sampled pixel is within kFixMargin of
        // a tap boundary, or has a tap outside the band, take the fp64 code.
        const RowFix *fp = rowfix + e.row_base + ir;
        const int64_t fx0 = uni64(fp->x0);
        if (fx0 != kFixNone) {
          const int64_t fy0 = uni64(fp->y0), fdx = uni64(fp->dx), fdy = uni64(fp->dy);
          const uint64_t X0 = (uint64_t)(fx0 + (int64_t)ic0 * fdx) - 0x80000000ull;
          const uint64_t Y0 = (uint64_t)(fy0 + (int64_t)ic0 * fdy) - 0x80000000ull;
          const uint64_t SX = (uint64_t)fdx << 6, SY = (uint64_t)fdy << 6;
          uint32_t amin = 0xFFFFFFFFu;
          bool allin = true;
          {
            uint64_t X = X0, Y = Y0;
#pragma unroll
            for (int q = 0; q < kNnPx; q++) {
              const bool inw = (unsigned)(ic0 + 64 * q) < (unsigned)lim;
              const int ix = (int)(int32_t)(X >> 32), iy = (int)(int32_t)(Y >> 32);
              const uint32_t am = min((uint32_t)X + kFixMargin, (uint32_t)Y + kFixMargin);
              amin = inw ? min(amin, am) : amin;
              allin = allin & (!inw | (((unsigned)ix < (unsigned)(bx - 1)) & ((unsigned)iy < (unsigned)(by - 1))));
              X += SX;
              Y += SY;
            }
          }
          if (__builtin_amdgcn_ballot_w64(amin < 2u * kFixMargin) == 0 && __all(allin)) {
            uint64_t X = X0, Y = Y0;
            // recomputed, not carried over from the test pass (kept live, its
            // 8 pixels' coordinates spill at 8 waves per SIMD)
            asm volatile("" : "+v"(X), "+v"(Y));
#pragma unroll
            for (int h = 0; h < kNnPx; h += HP) {
              u32x2 t0[HP], t1[HP];
              WT rx[HP], ry[HP];
#pragma unroll
              for (int q = 0; q < HP; q++) {
                const int ic = ic0 + 64 * (h + q);
                const bool ok = (unsigned)ic < (unsigned)lim;
                const uint32_t ix = (uint32_t)(X >> 32), iy = (uint32_t)(Y >> 32);
                rx[q] = (WT)1.0 - (WT)((float)(uint32_t)X * 2.3283064365386963e-10f);   // 2^-32
                ry[q] = (WT)1.0 - (WT)((float)(uint32_t)Y * 2.3283064365386963e-10f);
                const uint32_t o0 = ok ? (iy * (uint32_t)bx + ix) * 4u : 0x80000000u;
                const uint32_t o1 = ok ? o0 + (uint32_t)bx * 4u : 0x80000000u;
                t0[q] = __builtin_amdgcn_raw_buffer_load_b64(rs, o0, 0, 0);
                t1[q] = __builtin_amdgcn_raw_buffer_load_b64(rs, o1, 0, 0);
                X += SX;
                Y += SY;
              }
#pragma unroll
              for (int q = 0; q < HP; q++) bil_fold4(t0[q], t1[q], rx[q], ry[q], ic0 + 64 * (h + q), lim, nd, ndf,
                                                     hnd, fillv, fill_mode, c[h + q]);
            }
            fixed_done = true;
          }
        }
      }
      if (fixed_done) {
      } else if (kind == ROW_LINEAR) {   // HP pixels' taps in flight
        const double xs0 = rr->v[0], ys0 = rr->v[1], dX = rr->v[2], dY = rr->v[3];
#pragma unroll
        for (int h = 0; h < kNnPx; h += HP) {
          int ixv[HP], iyv[HP];
          WT rx[HP], ry[HP];
          bool allin = true;
#pragma unroll
          for (int q = 0; q < HP; q++) {
            const int ic = ic0 + 64 * (h + q);
            const double dist = (double)ic;
            const double sx = xs0 + dX * dist, sy = ys0 + dY * dist;
            ixv[q] = (int)floor(sx - 0.5);
            iyv[q] = (int)floor(sy - 0.5);
            rx[q] = (WT)(1.5 - (sx - (double)ixv[q]));
            ry[q] = (WT)(1.5 - (sy - (double)iyv[q]));
            allin = allin & (((unsigned)ic >= (unsigned)lim) |
                             (((unsigned)ixv[q] < (unsigned)(bx - 1)) & ((unsigned)iyv[q] < (unsigned)(by - 1))));
          }
          if (nd_f32 && __all(allin)) {
            // every sampled pixel of the wave has its 2x2 taps inside the band:
            // no -1 edge rule, no tap outside; the weights of four valid taps
            // sum to 1 within fp32 rounding, so the sample is accR unless a
            // tap holds nodata (then the general renormalisation)
            u32x2 t0[HP], t1[HP];
#pragma unroll
            for (int q = 0; q < HP; q++) {
              const int ic = ic0 + 64 * (h + q);
              const bool ok = (unsigned)ic < (unsigned)lim;
              const uint32_t o0 = ok ? (uint32_t)(iyv[q] * bx + ixv[q]) * 4u : 0x80000000u;
              const uint32_t o1 = ok ? o0 + (uint32_t)bx * 4u : 0x80000000u;
              t0[q] = __builtin_amdgcn_raw_buffer_load_b64(rs, o0, 0, 0);
              t1[q] = __builtin_amdgcn_raw_buffer_load_b64(rs, o1, 0, 0);
            }
#pragma unroll
            for (int q = 0; q < HP; q++) {
              const float tv[4] = {__uint_as_float(t0[q].x), __uint_as_float(t0[q].y), __uint_as_float(t1[q].x),
                                   __uint_as_float(t1[q].y)};
              const WT one = (WT)1.0;
              const WT wx[2] = {rx[q], one - rx[q]}, wy[2] = {ry[q], one - ry[q]};
              WT accR = (WT)0.0;
              bool anynd = false;
#pragma unroll
              for (int kk = 0; kk < 4; kk++) {
                accR += (WT)tv[kk] * (wx[kk & 1] * wy[kk >> 1]);
                anynd = anynd | (nd_nan ? (tv[kk] != tv[kk]) : (tv[kk] == ndf));
              }
              anynd = anynd & hnd;
              float v = (float)accR;
              if (anynd) {   // drop the nodata taps and renormalise (bil_sample's rule)
                WT aR = (WT)0.0, aD = (WT)0.0;
#pragma unroll
                for (int kk = 0; kk < 4; kk++) {
                  const WT w = wx[kk & 1] * wy[kk >> 1];
                  const bool use = !(nd_nan ? (tv[kk] != tv[kk]) : (tv[kk] == ndf));
                  aD += use ? w : (WT)0.0;
                  aR += use ? (WT)tv[kk] * w : (WT)0.0;
                }
                v = fillv;
                if (aD == (WT)1.0) v = (float)aR;
                else if (aD >= (WT)0.00001) v = (float)(aR / aD);
              }
              const int ic = ic0 + 64 * (h + q);
              const bool take = ((unsigned)ic < (unsigned)lim) & (v != nd) & (!fill_mode | (c[h + q] == nd));
              c[h + q] = take ? v : c[h + q];
            }
          } else {   // the reference's per-tap rules (coordinates recomputed)
            uint32_t valid[HP];
            u32x2 t0[HP], t1[HP];
#pragma unroll
            for (int q = 0; q < HP; q++) {
              const int ic = ic0 + 64 * (h + q);
              const double dist = (double)ic;
              prep(h + q, xs0 + dX * dist, ys0 + dY * dist, (unsigned)ic < (unsigned)lim, rx[q], ry[q], valid[q],
                   t0[q], t1[q]);
            }
#pragma unroll
            for (int q = 0; q < HP; q++) finish(h + q, rx[q], ry[q], valid[q], t0[q], t1[q]);
          }
        }
      } else {   // POOL: linear leaves, per-pixel exact points, failed pixels; one pixel at a time
#pragma unroll
        for (int q = 0; q < kNnPx; q++) {
          const int ic = ic0 + 64 * q;
          bool ok = (unsigned)ic < (unsigned)lim;
          double sx = 0.0, sy = 0.0;
          ok = ok && lin_coords(*rr, pool, ok ? ic : 0, sx, sy);
          WT rx, ry;
          uint32_t valid;
          u32x2 t0, t1;
          prep(q, sx, sy, ok, rx, ry, valid, t0, t1);
          finish(q, rx, ry, valid, t0, t1);
        }
      }
    }

    bil_store(a, t, r, xl, lane, full, ncols, c);
  }
}

// Bilinear float canvases (no mask layer): fp32 weights, 4 rows per wave,
// 4 pixels' taps in flight at 8 waves per SIMD; the A/B build also has the
// fp64 weights (GSKYHIP_BIL_F32=0: 6 waves per SIMD, or 8 with 2 pixels in
// flight, GSKYHIP_BIL_HP=2) and 8 rows per wave (GSKYHIP_BIL_RPW=8).
template <typename WT, int RPW, int HP, int WPS, bool FIX = true, bool SEP = true, int SHP = 4, int SWPS = 8>
void launch_bil_v(const RenderArgs &a, hipStream_t s) {
  const int items = a.n_tiles * ((a.max_h + 4 * RPW - 1) / (4 * RPW)) * ((a.max_w + kBandCols - 1) / kBandCols);
  const int grid = a.ab_xcd == 2 ? (items + 7) / 8 * 8 : items;
  hipLaunchKernelGGL((render_bil_kernel<WT, RPW, HP, WPS, FIX, SEP>), dim3((unsigned)grid), dim3(256), 0, s, a,
                     a.entries, a.order, a.rows, a.rowfix, a.pool, a.tplans, a.tiles, items);
  if (SEP)
    hipLaunchKernelGGL((render_bil_sep_kernel<WT, RPW, SHP, SWPS>), dim3((unsigned)items), dim3(256), 0, s, a,
                       a.entries, a.order, a.rows, a.tplans, a.tiles, items);
#ifdef GSKYHIP_AB
  if (SEP && a.ab_mode == 0x5E9) {   // counts of the sep kernel's checks (both kernels count: / 2)
    unsigned long long st[8];
    hipStreamSynchronize(s);
    hipMemcpyFromSymbol(st, HIP_SYMBOL(g_bil_sep_stat), sizeof(st));
    fprintf(stderr, "bil_sep_stat waves=%llu one_entry=%llu rows_covered=%llu rows_same=%llu taps_in=%llu\n",
            st[0] / 2, st[1] / 2, st[2] / 2, st[3] / 2, st[4] / 2);
    unsigned long long z[8] = {0};
    hipMemcpyToSymbol(HIP_SYMBOL(g_bil_sep_stat), z, sizeof(z));
  }
#endif
}

void launch_bil(const RenderArgs &a, int n_items, hipStream_t s) {
  (void)n_items;
#ifdef GSKYHIP_AB
  const char *f = getenv("GSKYHIP_BIL_F32");
  const char *rp = getenv("GSKYHIP_BIL_RPW");
  const char *hp = getenv("GSKYHIP_BIL_HP");
  const char *sp = getenv("GSKYHIP_BIL_SEP");   // 0: no separable-row reuse (round 4's kernel)
  const bool f32 = !f || atoi(f) != 0;
  const int rpw = rp ? atoi(rp) : 4;
  const int hpx = hp ? atoi(hp) : 4;
  const bool sep = !sp || atoi(sp) != 0;
  const char *fx = getenv("GSKYHIP_BIL_FIX");   // 1: the fixed-point LINEAR rows
  if (fx && atoi(fx) == 1) { launch_bil_v<float, 4, 4, 8, true>(a, s); return; }
  if (f32) {
    if (!sep) launch_bil_v<float, 4, 4, 8, false, false>(a, s);
    else if (hpx == 8) launch_bil_v<float, 4, 4, 8, false, true, 8, 6>(a, s);
    else if (hpx == 0) launch_bil_v<float, 4, 4, 8, false, true, 0, 8>(a, s);
    else if (hpx == 10) launch_bil_v<float, 4, 4, 8, false, true, 0, 6>(a, s);
    else if (rpw == 8) launch_bil_v<float, 8, 4, 8, false>(a, s);
    else if (rpw == 16) launch_bil_v<float, 16, 4, 8, false>(a, s);
    else launch_bil_v<float, 4, 4, 8, false>(a, s);
  } else if (hpx == 2) {
    launch_bil_v<double, 4, 2, 8, false>(a, s);
  } else {
    if (rpw == 8) launch_bil_v<double, 8, 4, 6, false>(a, s); else launch_bil_v<double, 4, 4, 6, false>(a, s);
  }
  return;
#endif
  // the fp64 row code: the fixed-point LINEAR rows cut VALU but measured
  // slower on C3 (profiles/r04b_ab_c2c5.jsonl: 0.93 vs 0.82 ms); so did the
  // separable-row kernel (72 % of C3's waves eligible, 0.86-0.93 vs 0.81 ms
  // total, profiles/r05b_ab_c3.jsonl): no separable split in the product
  launch_bil_v<float, 4, 4, 8, false, false>(a, s);
}

}  // namespace gsky
