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

// HP: pixels whose taps are in flight together; WPS: waves per SIMD the
// register budget is sized for.
template <typename WT, int RPW, int HP, int WPS, bool SEP = false>
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

  // Single-entry tiles, separable rows (round 6): a LINEAR row with dY == 0
  // samples one source row pair (iy, iy + 1) at every pixel, at the same
  // columns on every row with the same (xs0, dX) bits -- C3's EPSG:4326 ->
  // 3857 chunks at 1:1 -- so the next row down (iy + 1, iy + 2) finds its
  // upper taps already in registers: one 8-byte tap load per pixel instead
  // of two.  Same coordinates, addresses and fold as the fast path below.
  bool sp_have = false;
  int sp_iy = 0;
  double sp_xs0 = 0.0, sp_dX = 0.0;
  u32x2 sp_t1[kNnPx];
#pragma unroll 1
  for (int j = 0; j < RPW; j++) {
    const int r = r0 + j;
    if (r >= H) break;
    float c[kNnPx];
#pragma unroll
    for (int q = 0; q < kNnPx; q++) c[q] = cnod;

    if constexpr (SEP) {
      bool done = false;
      if (n_entries == 1) {
        const EntryD &e = ents[ord[0]];
        const int ir = r - e.yoff, ew = e.w, exoff = e.xoff;
        const int lim = max(0, min(ew, W - exoff));
        const int c0 = exoff - xb, c1 = exoff + lim - xb;
        const double nd64 = e.nodata64;
        const bool hnd = e.has_nodata != 0, nd_nan = nd64 != nd64;
        // a NaN nodata takes the per-entry path (bil_fold4 compares taps with ==)
        const bool nd_f32 = !hnd || (!nd_nan && (double)(float)nd64 == nd64);
        if (e.ns == ns_out && ew > 0 && ir >= 0 && ir < e.h && c1 > 0 && c0 < ncols && nd_f32) {
          const RowRec *rr = rows + e.row_base + ir;
          const int kind = __builtin_amdgcn_readfirstlane(rr->kind);
          const double xs0 = uni64d(rr->v[0]), ys0 = uni64d(rr->v[1]), dX = uni64d(rr->v[2]), dY = uni64d(rr->v[3]);
          const int bx = e.band_x, by = e.band_y;
          if (kind == ROW_LINEAR && dY == 0.0) {
            const int ic0 = xl - exoff;
            const int iy = (int)floor(ys0 - 0.5);   // sy == ys0 at every pixel (dY * dist is a signed zero)
            const WT ry = (WT)(1.5 - (ys0 - (double)iy));
            int ixv[kNnPx];
            WT rx[kNnPx];
            bool allin = (unsigned)iy < (unsigned)(by - 1);
#pragma unroll
            for (int q = 0; q < kNnPx; q++) {
              const int ic = ic0 + 64 * q;
              const double sx = xs0 + dX * (double)ic;
              ixv[q] = (int)floor(sx - 0.5);
              rx[q] = (WT)(1.5 - (sx - (double)ixv[q]));
              allin = allin & (((unsigned)ic >= (unsigned)lim) | ((unsigned)ixv[q] < (unsigned)(bx - 1)));
            }
            if (__all(allin)) {
              const bool reuse = sp_have & (iy == sp_iy + 1) & (__double_as_longlong(xs0) == __double_as_longlong(sp_xs0)) &
                                 (__double_as_longlong(dX) == __double_as_longlong(sp_dX));
              const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
                  (void *)uniform_ptr(e.band), (short)0, (int)((int64_t)bx * by * 4), 0x00020000);
              const float nd = e.nd.f, fillv = e.fill.f;
              const bool fill_mode = e.fill_mode != 0;
              const float ndf = (float)nd64;
              // HP pixels' taps in flight at a time (the register peak of the fast path)
#pragma unroll
              for (int h = 0; h < kNnPx; h += HP) {
                u32x2 t0[HP], t1[HP];
#pragma unroll
                for (int q = 0; q < HP; q++) {
                  const int ic = ic0 + 64 * (h + q);
                  const bool ok = (unsigned)ic < (unsigned)lim;
                  const uint32_t o0 = ok ? (uint32_t)(iy * bx + ixv[h + q]) * 4u : 0x80000000u;
                  const uint32_t o1 = ok ? o0 + (uint32_t)bx * 4u : 0x80000000u;
                  if (reuse) t0[q] = sp_t1[h + q];
                  else t0[q] = __builtin_amdgcn_raw_buffer_load_b64(rs, o0, 0, 0);
                  t1[q] = __builtin_amdgcn_raw_buffer_load_b64(rs, o1, 0, 0);
                }
#pragma unroll
                for (int q = 0; q < HP; q++) {
                  bil_fold4<WT>(t0[q], t1[q], rx[h + q], ry, ic0 + 64 * (h + q), lim, nd, ndf, hnd, fillv, fill_mode,
                                c[h + q]);
                  sp_t1[h + q] = t1[q];
                }
              }
              sp_have = true;
              sp_iy = iy;
              sp_xs0 = xs0;
              sp_dX = dX;
              done = true;
            }
          }
        }
      }
      if (done) {
        bil_store(a, t, r, xl, lane, full, ncols, c);
        continue;
      }
      sp_have = false;
    }

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
      if (kind == ROW_LINEAR) {   // HP pixels' taps in flight
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
// 4 pixels' taps in flight at 8 waves per SIMD.  Measured and not kept
// (DESIGN.md 5): fp64 weights, 8 / 16 rows per wave, the fixed-point LINEAR
// rows (profiles/r04b_ab_c2c5.jsonl: 0.93 vs 0.82 ms) and the separable-row
// kernel (72 % of C3's waves eligible, 0.86-0.93 vs 0.81 ms total,
// profiles/r05b_ab_c3.jsonl).
void launch_bil(const RenderArgs &a, int n_items, hipStream_t s) {
  (void)n_items;
  const int items = a.n_tiles * ((a.max_h + 15) / 16) * ((a.max_w + kBandCols - 1) / kBandCols);
  int sep = 6;
#ifdef GSKYHIP_AB
  if (const char *e = getenv("GSKYHIP_BIL_REUSE")) sep = atoi(e);   // 0: round 5's kernel; 8: reuse at 8 waves / SIMD
#endif
  if (sep == 6)
    hipLaunchKernelGGL((render_bil_kernel<float, 4, 4, 6, true>), dim3((unsigned)items), dim3(256), 0, s, a,
                       a.entries, a.order, a.rows, a.rowfix, a.pool, a.tplans, a.tiles, items);
  else if (sep)
    hipLaunchKernelGGL((render_bil_kernel<float, 4, 4, 8, true>), dim3((unsigned)items), dim3(256), 0, s, a,
                       a.entries, a.order, a.rows, a.rowfix, a.pool, a.tplans, a.tiles, items);
  else
    hipLaunchKernelGGL((render_bil_kernel<float, 4, 4, 8>), dim3((unsigned)items), dim3(256), 0, s, a, a.entries,
                       a.order, a.rows, a.rowfix, a.pool, a.tplans, a.tiles, items);
}

}  // namespace gsky
