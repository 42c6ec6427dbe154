// render_generic.h -- per-pixel sampling (descend/exact/approx coordinates,
// GWKBilinear, typed loads) and the generic render kernels (any value type,
// RGB or single namespace, auto-scale, complex tiles).  Included by render.hip
// (window / bytesRead kernels use the sampling helpers) and instantiated in
// render_generic1.hip / render_generic3.hip so the NOUT=1 and NOUT=3 kernel
// families compile as separate translation units.
#pragma once
#include "gsky_device.h"
#include "render.h"
#include "stages.h"
#include "render_common.h"
#include <type_traits>

namespace gsky {

// ---------------------------------------------------------------- sampling
// Load one source value as a Val of the pair's output dtype (warp.go:339-343).
__device__ __forceinline__ Val load_val(const void *band, int src_dtype, long idx) {
  Val o;
  switch (src_dtype) {
    case GSKYHIP_BYTE: o.i = ((const uint8_t *)band)[idx]; break;
    case GSKYHIP_INT16: o.i = ((const int16_t *)band)[idx]; break;
    case GSKYHIP_UINT16: o.i = ((const uint16_t *)band)[idx]; break;
    case GSKYHIP_FLOAT32: o.f = ((const float *)band)[idx]; break;
    case GSKYHIP_INT32: o = gdal_copy_to((double)((const int32_t *)band)[idx], GSKYHIP_FLOAT32); break;
    case GSKYHIP_UINT32: o = gdal_copy_to((double)((const uint32_t *)band)[idx], GSKYHIP_FLOAT32); break;
    case GSKYHIP_FLOAT64: o = gdal_copy_to(((const double *)band)[idx], GSKYHIP_FLOAT32); break;
    default: o.u = 0; break;
  }
  return o;
}
__device__ __forceinline__ double load_dbl(const void *band, int src_dtype, long idx, int signed_byte) {
  switch (src_dtype) {
    case GSKYHIP_BYTE: return signed_byte ? (double)((const int8_t *)band)[idx] : (double)((const uint8_t *)band)[idx];
    case GSKYHIP_INT16: return ((const int16_t *)band)[idx];
    case GSKYHIP_UINT16: return ((const uint16_t *)band)[idx];
    case GSKYHIP_FLOAT32: return ((const float *)band)[idx];
    case GSKYHIP_INT32: return ((const int32_t *)band)[idx];
    case GSKYHIP_UINT32: return ((const uint32_t *)band)[idx];
    case GSKYHIP_FLOAT64: return ((const double *)band)[idx];
    default: return 0;
  }
}

// GWKBilinearResample4Sample semantics (SURVEY 8a parity targets).
__device__ __noinline__ Val bilinear_value(const PairPlan &pp, double sx, double sy) {
  int iSrcX = (int)floor(sx - 0.5);
  int iSrcY = (int)floor(sy - 0.5);
  double rX = 1.5 - (sx - iSrcX);
  double rY = 1.5 - (sy - iSrcY);
  if (iSrcX == -1) { iSrcX = 0; rX = 1; }
  if (iSrcY == -1) { iSrcY = 0; rY = 1; }
  double accR = 0.0, accDiv = 0.0;
  const int xs4[4] = {iSrcX, iSrcX + 1, iSrcX, iSrcX + 1};
  const int ys4[4] = {iSrcY, iSrcY, iSrcY + 1, iSrcY + 1};
  const double w4[4] = {rX * rY, (1.0 - rX) * rY, rX * (1.0 - rY), (1.0 - rX) * (1.0 - rY)};
#pragma unroll
  for (int k = 0; k < 4; k++) {
    if (xs4[k] < 0 || xs4[k] >= pp.band_x || ys4[k] < 0 || ys4[k] >= pp.band_y) continue;
    const double v = load_dbl(pp.band, pp.src_dtype, (long)ys4[k] * pp.band_x + xs4[k], pp.signed_byte);
    if (pp.has_nodata && (v == pp.nodata || (pp.nodata != pp.nodata && v != v))) continue;
    accDiv += w4[k];
    accR += v * w4[k];
  }
  double r;
  if (accDiv == 1.0) r = accR;
  else if (accDiv < 0.00001) return pp.fill;
  else r = accR / accDiv;
  if (pp.out_dtype == GSKYHIP_FLOAT32) { Val o; o.f = (float)r; return o; }
  return gdal_copy_to(floor(r + 0.5), pp.out_dtype);
}

// Warped value of window pixel (i,row) of a pair: the source value or the
// window's nodata fill (warp.go:246-247, 271-344).
template <bool GENERAL, int RES>
__device__ __forceinline__ Val warped_value(const PairPlan &pp, const RowRec &rr, const Leaf *pool,
                                            const Xform *xf, int i, int row) {
  double sx, sy;
  const bool ok = src_coords<GENERAL>(rr, pool, xf, pp.xoff, pp.yoff, pp.w, i, row, sx, sy);
  if (!ok) return pp.fill;
  if (RES == GSKYHIP_RESAMPLE_BILINEAR) return bilinear_value(pp, sx, sy);
  if (sx < 0 || sy < 0) return pp.fill;
  const double ax = sx + 1.0e-10, ay = sy + 1.0e-10;
  if (ax >= 2147483647.0 || ay >= 2147483647.0) return pp.fill;
  const int ix = (int)ax, iy = (int)ay;
  if (ix >= pp.band_x || iy >= pp.band_y) return pp.fill;
  Val v = load_val(pp.band, pp.src_dtype, (long)iy * pp.band_x + ix);
  if (pp.out_dtype == GSKYHIP_SIGNEDBYTE) v.i = (int32_t)(int8_t)(uint8_t)v.i;
  return v;
}

// Mask bit for data pair `pp` at its window pixel (ic, ir): mask[iSrc] with
// iSrc the data window's linear index (tile_merger.go:53/64), read from the
// warped mask raster of the same geoStamp.
template <bool GENERAL, int RES>
__device__ __forceinline__ bool mask_at(const RenderArgs &a, const PairPlan &pp, int ic, int ir) {
  const int mp = pp.mask_pair;
  const PairPlan &mq = a.pairs[mp];
  const long iSrc = (long)ir * pp.w + ic;
  const int mx = (int)(iSrc % mq.w), my = (int)(iSrc / mq.w);
  if (my >= mq.h) return false;  // Go would panic; plan_tiles flags it
  const int slot = mask_slot(mq.out_dtype);
  if (slot < 0) return false;    // flagged in plan_tiles (not a bit-mask type)
  const RowRec &mr = a.rows[(long)mp * a.max_h + my];
  Val v = warped_value<GENERAL, RES>(mq, mr, a.pool, a.xforms + mp, mx, my);
  return mask_bit(a.mask[slot], mq.out_dtype, v.i);
}

// Fused warp + merge (+ scale + palette) of a band of rows of one tile: each
// wave walks rows, each lane 4 consecutive pixels of a 256-pixel chunk.
template <int NOUT, int RES, bool MASK, bool GENERAL>
__device__ __forceinline__ void render_band(const RenderArgs &a, int t, int band0, const uint32_t *s_ramp) {
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const gskyhip_tile &tile = a.tiles[t];
  const TilePlan &tp = a.tplans[t];
  const int W = tile.width, H = tile.height;
  const int32_t *ord = a.order + tile.pair_begin;
  const int n_entries = tp.n_entries;

  Val cnod[NOUT];
  bool cfloat[NOUT];
  ScaleK sk[NOUT];
  bool all_created = true;
#pragma unroll
  for (int s = 0; s < NOUT; s++) {
    const int ns = a.out_ns[s];
    all_created = all_created && tp.created[ns] != 0;
    cfloat[s] = tp.dtype[ns] == GSKYHIP_FLOAT32;
    cnod[s] = go_conv_to(tp.nodata[ns], tp.dtype[ns]);
    sk[s] = make_scale(tp.dtype[ns], tp.nodata[ns], a.sp, false, 0.f, 0.f);
  }
  for (int r = band0 + wave; r < band0 + a.rows_per_block && r < H; r += 4) {
    for (int cx = 0; cx < W; cx += 256) {
      const int x0 = cx + lane * 4;
      Val c[NOUT][4];
#pragma unroll
      for (int s = 0; s < NOUT; s++)
#pragma unroll
        for (int q = 0; q < 4; q++) c[s][q] = cnod[s];
      for (int e = 0; e < n_entries; e++) {
        const int p = ord[e];
        const PairPlan &pp = a.pairs[p];
        if (r < pp.yoff || r >= pp.yoff + pp.h) continue;
        if (cx + 256 <= pp.xoff || cx >= pp.xoff + pp.w) continue;
        int s = -1;
#pragma unroll
        for (int k = 0; k < NOUT; k++) if (a.out_ns[k] == pp.ns) s = k;
        if (s < 0) continue;  // merged into a canvas that is not rendered
        const int ir = r - pp.yoff;
        const RowRec &rr = a.rows[(long)p * a.max_h + ir];
        const Val nd = go_conv_to(pp.nodata, pp.out_dtype);
        const bool isf = pp.out_dtype == GSKYHIP_FLOAT32;
        const bool fill = pp.fill_mode != 0;
#pragma unroll
        for (int q = 0; q < 4; q++) {
          const int ic = x0 + q - pp.xoff;
          if (x0 + q >= W || ic < 0 || ic >= pp.w) continue;
          const Val v = warped_value<GENERAL, RES>(pp, rr, a.pool, a.xforms + p, ic, ir);
          if (val_eq(v, nd, isf)) continue;
          if (MASK && pp.mask_pair >= 0 && mask_at<GENERAL, RES>(a, pp, ic, ir)) continue;
#pragma unroll
          for (int k = 0; k < NOUT; k++) {
            if (k != s) continue;
            if (fill && !val_eq(c[k][q], nd, isf)) continue;
            c[k][q] = v;
          }
        }
      }
      const bool active = x0 < W;   // inactive lanes still join the wave reduction below
      // typed canvases (tile_merger.go:562-652) and the auto-scale reduction
      if (a.canvas && active) {
#pragma unroll
        for (int s = 0; s < NOUT; s++) {
          const int dsz = type_size(tp.dtype[a.out_ns[s]]);
          uint8_t *cb = a.cov_offsets ? a.canvas : a.canvas + t * a.canvas_tile_stride + s * a.canvas_ns_stride;
          const long row0 = a.cov_offsets ? a.cov_offsets[t] + (long)r * a.cov_stride : (long)r * a.max_w;
          for (int q = 0; q < 4 && x0 + q < W; q++) {
            const long idx = row0 + x0 + q;
            if (dsz == 1) cb[idx] = (uint8_t)c[s][q].i;
            else if (dsz == 2) ((uint16_t *)cb)[idx] = (uint16_t)c[s][q].i;
            else ((uint32_t *)cb)[idx] = c[s][q].u;
          }
        }
      }
      if (!a.write_rgba) {
        if (a.autom) {
#pragma unroll
          for (int s = 0; s < NOUT; s++) {
            const int ns = a.out_ns[s];
            float mn = INFINITY, mx = -INFINITY;
            for (int q = 0; q < 4 && x0 + q < W; q++) {
              const Val v = c[s][q];
              if (val_eq(v, cnod[s], cfloat[s])) continue;
              float f = cfloat[s] ? v.f : (float)v.i;
              if (cfloat[s] && a.sp.colour_scale > 0 && !normalise_f(f, a.sp.colour_scale, tp.nodata[ns])) continue;
              if (r == 0 && x0 + q == 0) {
                a.minmax[t * 3 + s].p0_valid = 1;
                a.minmax[t * 3 + s].p0 = f;
              }
              if (f == f) { mn = fminf(mn, f); mx = fmaxf(mx, f); }
            }
            int32_t emn = fenc(mn), emx = fenc(mx);
            for (int o = 32; o > 0; o >>= 1) {
              emn = min(emn, __shfl_xor(emn, o, 64));
              emx = max(emx, __shfl_xor(emx, o, 64));
            }
            if (lane == 0) {
              if (emn != fenc(INFINITY)) atomicMin(&a.minmax[t * 3 + s].mn, emn);
              if (emx != fenc(-INFINITY)) atomicMax(&a.minmax[t * 3 + s].mx, emx);
            }
          }
        }
        continue;
      }
      if (!active) continue;
      // utils.Scale + EncodePNG pixel loop
      uint32_t px[4];
#pragma unroll
      for (int q = 0; q < 4; q++) {
        uint32_t o = 0;
        if (all_created) {
          if (NOUT == 1) {
            const uint8_t b = scale_px(sk[0], c[0][q]);
            if (b != 0xFF) o = a.ramp ? s_ramp[b] : (0xFF000000u | ((uint32_t)b << 16) | ((uint32_t)b << 8) | b);
          } else {
            const uint8_t rr = scale_px(sk[0], c[0][q]);
            const uint8_t gg = scale_px(sk[NOUT > 1 ? 1 : 0], c[NOUT > 1 ? 1 : 0][q]);
            const uint8_t bb = scale_px(sk[NOUT > 2 ? 2 : 0], c[NOUT > 2 ? 2 : 0][q]);
            if (rr != 0xFF || gg != 0xFF || bb != 0xFF)
              o = 0xFF000000u | ((uint32_t)bb << 16) | ((uint32_t)gg << 8) | rr;
          }
        }
        px[q] = o;
      }
      uint8_t *dst = a.rgba + (((long)t * a.max_h + r) * a.max_w + x0) * 4;
      if (x0 + 3 < W && ((((uintptr_t)dst) & 15) == 0)) {
        *(uint4 *)dst = make_uint4(px[0], px[1], px[2], px[3]);
      } else {
        for (int q = 0; q < 4 && x0 + q < W; q++) ((uint32_t *)dst)[q] = px[q];
      }
    }
  }
}

// Branch-free NN sample of window pixel (sx, sy): the source value, or the
// window fill when the pixel is outside the window or maps off the source
// (warp.go:271-344).  One unconditional gather (index 0 when invalid).
template <typename T>
__device__ __forceinline__ typename VOf<T>::type nn_px(const EntryD &e, double sx, double sy, bool in,
                                                       typename VOf<T>::type fillv) {
  const double ax = sx + 1.0e-10, ay = sy + 1.0e-10;
  const int ix = __double2int_rz(ax), iy = __double2int_rz(ay);
  const bool ok = in && !(sx < 0) && !(sy < 0) && ax < 2147483647.0 && ay < 2147483647.0 && ix < e.band_x &&
                  iy < e.band_y;
  const long idx = ok ? (long)iy * e.band_x + ix : 0;
  const typename VOf<T>::type raw = (typename VOf<T>::type)((const GPTR(T))e.band)[idx];
  return ok ? raw : fillv;
}

// One wave owns a 4-row x 256-pixel block (4 x 4 pixels per lane): each
// entry descriptor and row record is loaded once (scalar) per block.
template <int NOUT, int RES, bool MASK, typename T>
__device__ __forceinline__ void render_fast_t(const RenderArgs &a, const EntryD *__restrict__ ents,
                                              const int32_t *__restrict__ order, const RowRec *__restrict__ rows,
                                              const Leaf *__restrict__ pool, const gskyhip_tile &tile,
                                              const TilePlan &tp, int t, int band0, const uint32_t *s_ramp) {
  using V = typename VOf<T>::type;
  // wave index in an SGPR: rows, row records and window tests become scalar
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int W = tile.width, H = tile.height;
  const int r0 = band0 + wave * 4;
  if (r0 >= H) return;
  const int32_t *ord = order + tile.pair_begin;
  const int n_entries = tp.n_entries;
  V cnod[NOUT];
  ScaleK sk[NOUT];
  bool all_created = true;
#pragma unroll
  for (int s = 0; s < NOUT; s++) {
    const int ns = a.out_ns[s];
    all_created = all_created && tp.created[ns] != 0;
    cnod[s] = as_v<T>(go_conv_to(tp.nodata[ns], tp.dtype[ns]));
    sk[s] = make_scale(tp.dtype[ns], tp.nodata[ns], a.sp, false, 0.f, 0.f);
  }
  const bool has_ramp = a.ramp != nullptr;
  uint8_t *rgba_tile = a.rgba + (long)t * a.max_h * a.max_w * 4;
  for (int cx = 0; cx < W; cx += 256) {
    const int x0 = cx + lane * 4;
    V c[NOUT][4][4];
#pragma unroll
    for (int s = 0; s < NOUT; s++)
#pragma unroll
      for (int j = 0; j < 4; j++)
#pragma unroll
        for (int q = 0; q < 4; q++) c[s][j][q] = cnod[s];
    for (int k = 0; k < n_entries; k++) {
      const EntryD e = ents[ord[k]];
      if (r0 + 3 < e.yoff || r0 >= e.yoff + e.h) continue;
      if (cx + 256 <= e.xoff || cx >= e.xoff + e.w) continue;
      int slot = -1;
#pragma unroll
      for (int s = 0; s < NOUT; s++) if (a.out_ns[s] == e.ns) slot = s;
      if (slot < 0) continue;
      const V nd = as_v<T>(e.nd), fillv = as_v<T>(e.fill);
#pragma unroll
      for (int j = 0; j < 4; j++) {
        const int ir = r0 + j - e.yoff;
        if (r0 + j >= H || ir < 0 || ir >= e.h) continue;
        const RowRec &rr = rows[e.row_base + ir];
        // wave-uniform row kind: LINEAR rows (the common case) take a straight
        // 4-pixel body whose gathers issue back to back; the source
        // coordinates are the same fp64 expressions as lin_coords().
        double sxq[4], syq[4];
        bool okq[4] = {true, true, true, true};   // false: failed exact transform (window fill)
        const int ic0 = x0 - e.xoff;
        if (rr.kind == ROW_LINEAR) {
          const double xs0 = rr.v[0], ys0 = rr.v[1], dX = rr.v[2], dY = rr.v[3];
          const double d0 = (double)ic0;
#pragma unroll
          for (int q = 0; q < 4; q++) {
            const double dist = d0 + (double)q;   // exact: small integers
            syq[q] = ys0 + dY * dist;
            sxq[q] = xs0 + dX * dist;
          }
        } else {
#pragma unroll
          for (int q = 0; q < 4; q++) {
            const int ic = ic0 + q;
            okq[q] = lin_coords(rr, pool, ((unsigned)ic < (unsigned)e.w) ? ic : 0, sxq[q], syq[q]);
          }
        }
#pragma unroll
        for (int q = 0; q < 4; q++) {
          const int ic = ic0 + q;
          const bool in = (unsigned)ic < (unsigned)e.w && x0 + q < W;
          const double sx = sxq[q], sy = syq[q];
          V v;
          if (RES == GSKYHIP_RESAMPLE_BILINEAR) {
            v = fillv;
            V got;
            if (in && okq[q] && bil_fetch<T>(e, sx, sy, got)) v = got;
          } else {
            v = nn_px<T>(e, sx, sy, in && okq[q], fillv);
          }
          bool take = in && (v != nd);
          if (MASK && e.mask_pair >= 0) take = take && !mask_fast<RES>(ents, rows, pool, a.mask, e, ic, ir);
#pragma unroll
          for (int s = 0; s < NOUT; s++) {
            if (s != slot) continue;
            const bool t2 = take && (!e.fill_mode || c[s][j][q] == nd);
            c[s][j][q] = t2 ? v : c[s][j][q];
          }
        }
      }
    }
    if (x0 >= W) continue;
#pragma unroll
    for (int j = 0; j < 4; j++) {
      const int r = r0 + j;
      if (r >= H) break;
      if (a.canvas) {
#pragma unroll
        for (int s = 0; s < NOUT; s++) {
          T *cb = (T *)(a.cov_offsets ? a.canvas : a.canvas + t * a.canvas_tile_stride + s * a.canvas_ns_stride);
          const long row0 = a.cov_offsets ? a.cov_offsets[t] + (long)r * a.cov_stride : (long)r * a.max_w;
#pragma unroll
          for (int q = 0; q < 4; q++)
            if (x0 + q < W) cb[row0 + x0 + q] = (T)c[s][j][q];
        }
      }
      if (!a.write_rgba) continue;
      uint32_t px[4];
#pragma unroll
      for (int q = 0; q < 4; q++) {
        uint32_t o;
        if (NOUT == 1) {
          const uint32_t b = scale_t<T>(sk[0], c[0][j][q]);
          const uint32_t col = has_ramp ? s_ramp[b & 0xFFu] : (0xFF000000u | (b << 16) | (b << 8) | b);
          o = (b == 0xFFu) ? 0u : col;
        } else {
          const uint32_t rr8 = scale_t<T>(sk[0], c[0][j][q]);
          const uint32_t gg8 = scale_t<T>(sk[NOUT > 1 ? 1 : 0], c[NOUT > 1 ? 1 : 0][j][q]);
          const uint32_t bb8 = scale_t<T>(sk[NOUT > 2 ? 2 : 0], c[NOUT > 2 ? 2 : 0][j][q]);
          o = (rr8 != 0xFFu || gg8 != 0xFFu || bb8 != 0xFFu) ? (0xFF000000u | (bb8 << 16) | (gg8 << 8) | rr8) : 0u;
        }
        px[q] = all_created ? o : 0u;
      }
      uint8_t *dst = rgba_tile + ((long)r * a.max_w + x0) * 4;
      if (x0 + 3 < W && ((((uintptr_t)dst) & 15) == 0)) {
        u32x4 v4 = {px[0], px[1], px[2], px[3]};
        // streaming output, never re-read: non-temporal, keeps L2 for source rows
        __builtin_nontemporal_store(v4, (GPTR(u32x4))dst);
      } else {
#pragma unroll
        for (int q = 0; q < 4; q++)
          if (x0 + q < W) ((uint32_t *)dst)[q] = px[q];
      }
    }
  }
}

// Simple tiles (every row LINEAR / linear leaves, one value type).
// Grid n_tiles * bands; complex tiles go to render_general_kernel.
template <int NOUT, int RES, bool MASK>
__global__ __launch_bounds__(256) void render_fast_kernel(RenderArgs a, const EntryD *__restrict__ ents,
                                                          const int32_t *__restrict__ order,
                                                          const RowRec *__restrict__ rows,
                                                          const Leaf *__restrict__ pool,
                                                          const TilePlan *__restrict__ tplans,
                                                          const gskyhip_tile *__restrict__ tiles) {
  __shared__ uint32_t s_ramp[256];
  if (a.ramp) s_ramp[threadIdx.x] = a.ramp[threadIdx.x];
  __syncthreads();
  const int bands_per_tile = (a.max_h + a.rows_per_block - 1) / a.rows_per_block;
  const int t = blockIdx.x / bands_per_tile;
  if (t >= a.n_tiles) return;
  const TilePlan &tp = tplans[t];
  if (tp.complex) return;
  const gskyhip_tile &tile = tiles[t];
  const int band0 = (blockIdx.x % bands_per_tile) * a.rows_per_block;
  switch (tp.vt) {
    case GSKYHIP_INT16: render_fast_t<NOUT, RES, MASK, int16_t>(a, ents, order, rows, pool, tile, tp, t, band0, s_ramp); break;
    case GSKYHIP_UINT16: render_fast_t<NOUT, RES, MASK, uint16_t>(a, ents, order, rows, pool, tile, tp, t, band0, s_ramp); break;
    case GSKYHIP_FLOAT32: render_fast_t<NOUT, RES, MASK, float>(a, ents, order, rows, pool, tile, tp, t, band0, s_ramp); break;
    case GSKYHIP_SIGNEDBYTE: render_fast_t<NOUT, RES, MASK, int8_t>(a, ents, order, rows, pool, tile, tp, t, band0, s_ramp); break;
    default: render_fast_t<NOUT, RES, MASK, uint8_t>(a, ents, order, rows, pool, tile, tp, t, band0, s_ramp); break;
  }
}

// Auto-scale pass 1 over simple tiles: typed canvases + per-tile min/max
// (raster_scaler.go:47-78) with the generic body.
template <int NOUT, int RES, bool MASK>
__global__ __launch_bounds__(256) void render_auto_kernel(RenderArgs a) {
  __shared__ uint32_t s_ramp[256];
  if (a.ramp) s_ramp[threadIdx.x] = a.ramp[threadIdx.x];
  __syncthreads();
  const int bands_per_tile = (a.max_h + a.rows_per_block - 1) / a.rows_per_block;
  const int t = blockIdx.x / bands_per_tile;
  if (t >= a.n_tiles || a.tplans[t].complex) return;
  render_band<NOUT, RES, MASK, false>(a, t, (blockIdx.x % bands_per_tile) * a.rows_per_block, s_ramp);
}

// Complex tiles (exact points, recursion leftovers), from the device list.
template <int NOUT, int RES, bool MASK>
__global__ __launch_bounds__(256) void render_general_kernel(RenderArgs a) {
  __shared__ uint32_t s_ramp[256];
  const int bands_per_tile = (a.max_h + a.rows_per_block - 1) / a.rows_per_block;
  const int items = a.counters[2] * bands_per_tile;
  if ((int)blockIdx.x >= items) return;   // no complex tile for this block (the common case)
  if (a.ramp) s_ramp[threadIdx.x] = a.ramp[threadIdx.x];
  __syncthreads();
  for (int it = blockIdx.x; it < items; it += gridDim.x) {
    const int t = a.complex_list[it / bands_per_tile];
    render_band<NOUT, RES, MASK, true>(a, t, (it % bands_per_tile) * a.rows_per_block, s_ramp);
  }
}

template <int NOUT, int RES, bool MASK>
static void launch_render_kernels(const RenderArgs &a, dim3 grid, bool general_only, hipStream_t s) {
  if (!general_only) {
    if (a.autom && !a.write_rgba)
      hipLaunchKernelGGL((render_auto_kernel<NOUT, RES, MASK>), grid, dim3(256), 0, s, a);
    else
      hipLaunchKernelGGL((render_fast_kernel<NOUT, RES, MASK>), grid, dim3(256), 0, s, a, a.entries, a.order,
                         a.rows, a.pool, a.tplans, a.tiles);
  }
  // a grid no larger than the batch's (tile, band) items: small requests (C1)
  // dispatch a few blocks, not 512
  const int bpt = (a.max_h + a.rows_per_block - 1) / a.rows_per_block;
  const int gen_grid = (int)std::max<int64_t>(1, std::min<int64_t>(512, (int64_t)a.n_tiles * bpt));
  hipLaunchKernelGGL((render_general_kernel<NOUT, RES, MASK>), dim3(gen_grid), dim3(256), 0, s, a);
}

template <int NOUT>
static void dispatch_render_t(const RenderArgs &a, int resample, bool mask, dim3 grid, bool general_only,
                              hipStream_t s) {
  if (resample == GSKYHIP_RESAMPLE_BILINEAR) {
    if (mask) launch_render_kernels<NOUT, GSKYHIP_RESAMPLE_BILINEAR, true>(a, grid, general_only, s);
    else launch_render_kernels<NOUT, GSKYHIP_RESAMPLE_BILINEAR, false>(a, grid, general_only, s);
  } else {
    if (mask) launch_render_kernels<NOUT, GSKYHIP_RESAMPLE_NEAREST, true>(a, grid, general_only, s);
    else launch_render_kernels<NOUT, GSKYHIP_RESAMPLE_NEAREST, false>(a, grid, general_only, s);
  }
}

}  // namespace gsky
