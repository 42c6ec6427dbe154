// render_bil.h -- bilinear band kernel for float32 typed canvases (WCS
// GetCoverage, BASELINE C3), shaped like render_nn_kernel (render_nn.h):
//
//   * a wave owns 4 consecutive rows of a 16-row band and a 512-column
//     block, walks the tile's entries in merge order with scalar loads and
//     folds R rows x LPX pixels per lane at once;
//   * per pixel the GWKBilinearResample4Sample expressions of bil_sample()
//     (render_lds.h) -- same fp64 operations in the same order, so the
//     values are bit-identical to the first band kernel's -- but the four
//     taps arrive as two 8-byte buffer loads (the x and x+1 taps of the two
//     source rows), issued for all R x LPX pixels before the first wait.
//     The first band kernel sampled pixel by pixel under a branch, one tap
//     round trip after the other (profiles/r02j_kernel_stats_c3.csv: 2.1 ms);
//   * taps outside the band read 0 through the buffer range check and are
//     dropped by their validity flag, as bil_sample() `continue`s; skipped
//     taps add +0.0, which leaves the non-negative sums bit-identical.
#pragma once
#include "render_nn.h"

namespace gsky {

typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

// One pixel of GWKBilinearResample4Sample from its two tap pairs (t0: row
// iSrcY, x and x+1; t1: row iSrcY + 1).  false: accDiv < 1e-5 (no sample).
__device__ __forceinline__ bool bil_combine(double sx, double sy, int iSrcX, int iSrcY, int bx, int by,
                                            float t00, float t01, float t10, float t11, bool hnd, double nd64,
                                            float &out) {
  double rX = 1.5 - (sx - iSrcX);
  double rY = 1.5 - (sy - iSrcY);
  int x0 = iSrcX, y0 = iSrcY;
  if (x0 == -1) { x0 = 0; rX = 1; }
  if (y0 == -1) { y0 = 0; rY = 1; }
  const float tv[4] = {t00, t01, t10, t11};
  double accR = 0.0, accDiv = 0.0;
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const int xx = x0 + (k & 1), yy = y0 + (k >> 1);
    const double w = ((k & 1) ? (1.0 - rX) : rX) * ((k >> 1) ? (1.0 - rY) : rY);
    const double d = (double)tv[k];
    const bool use = xx >= 0 && xx < bx && yy >= 0 && yy < by &&
                     !(hnd && (d == nd64 || (nd64 != nd64 && d != d)));
    accDiv += use ? w : 0.0;
    accR += use ? d * w : 0.0;
  }
  double r;
  if (accDiv == 1.0) r = accR;
  else if (accDiv < 0.00001) return false;
  else r = accR / accDiv;
  out = (float)r;
  return true;
}

template <int LPX, int R, int S, int W8>
__global__ __launch_bounds__(256, W8 ? 8 : 1) void render_bil_kernel(RenderArgs a, const EntryD *__restrict__ ents,
                                                         const int32_t *__restrict__ order,
                                                         const RowRec *__restrict__ rows,
                                                         const Leaf *__restrict__ pool,
                                                         const TilePlan *__restrict__ tplans,
                                                         const gskyhip_tile *__restrict__ tiles, int n_items) {
  constexpr int kCols = 64 * LPX;   // S: column step between a lane's pixels (1 or 64, render_nn.h)
  const int item = blockIdx.x;
  if (item >= n_items) return;
  const int bands_per_tile = (a.max_h + kBandRows - 1) / kBandRows;
  const int col_blocks = (a.max_w + kBandCols - 1) / kBandCols;
  const int t = item / (bands_per_tile * col_blocks);
  const int in_tile = item - t * bands_per_tile * col_blocks;
  const TilePlan &tp = tplans[t];
  if (tp.complex || (tp.n_entries > 0 && tp.vt != GSKYHIP_FLOAT32)) return;   // empty tiles: written here
  const gskyhip_tile &tile = tiles[t];
  const int W = tile.width, H = tile.height;
  const int band0 = (in_tile / col_blocks) * kBandRows;
  const int xb = (in_tile % col_blocks) * kBandCols;
  if (band0 >= H || xb >= W) return;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int r0 = band0 + wave * 4;
  if (r0 >= H) return;

  const int ns_out = a.out_ns[0];
  const float cnod = go_conv_to(tp.nodata[ns_out], tp.dtype[ns_out]).f;
  const int32_t *ord = order + tile.pair_begin;
  const int n_entries = tp.n_entries;
  const int xend = min(xb + kBandCols, W);

#pragma unroll 1
  for (int cx = xb; cx < xend; cx += kCols) {
    const int x0 = cx + (S == 1 ? lane * LPX : lane);
#pragma unroll 1
    for (int j = 0; j < 4; j += R) {
      const int rb = r0 + j;
      if (rb >= H) break;
      float c[R][LPX];
#pragma unroll
      for (int i = 0; i < R; i++)
#pragma unroll
        for (int q = 0; q < LPX; q++) c[i][q] = cnod;

#pragma unroll 1
      for (int k = 0; k < n_entries; k++) {
        const EntryD &e = ents[ord[k]];
        const int eyoff = e.yoff, eh = e.h, exoff = e.xoff, ew = e.w;
        if (e.ns != ns_out || ew <= 0) continue;
        if (rb + R <= eyoff || rb >= eyoff + eh) continue;
        if (cx + kCols <= exoff || cx >= exoff + ew) continue;
        const int bx = e.band_x, by = e.band_y;
        const float nd = e.nd.f, fillv = e.fill.f;
        const bool fill_mode = e.fill_mode != 0;
        const bool hnd = e.has_nodata != 0;
        const double nd64 = e.nodata64;
        const int ic0 = x0 - exoff;
        const int lim = max(0, min(ew, W - exoff));
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            (void *)uniform_ptr(e.band), (short)0, (int)((int64_t)bx * by * 4), 0x00020000);
        double sxv[R][LPX], syv[R][LPX];
        bool okc[R][LPX];
        u32x2 t0[R][LPX], t1[R][LPX];
        // coordinates and the two tap-pair loads of every pixel first
#pragma unroll
        for (int i = 0; i < R; i++) {
          const int ir = rb + i - eyoff;
          const bool row_in = ir >= 0 && ir < eh && rb + i < H;
          const RowRec *rr = rows + e.row_base + (row_in ? ir : 0);
          const int kind = __builtin_amdgcn_readfirstlane(rr->kind);
#pragma unroll
          for (int q = 0; q < LPX; q++) {
            const int ic = ic0 + q * S;
            const bool in = row_in && (unsigned)ic < (unsigned)lim;
            double sx = 0.0, sy = 0.0;
            bool ok = in;
            if (kind == ROW_LINEAR) {
              const double dist = (double)ic0 + (double)(q * S);
              sy = rr->v[1] + rr->v[3] * dist;
              sx = rr->v[0] + rr->v[2] * dist;
            } else {   // POOL: linear leaves, per-pixel exact points, failed pixels
              ok = ok && lin_coords(*rr, pool, in ? ic : 0, sx, sy);
            }
            const int iSrcX = (int)floor(sx - 0.5), iSrcY = (int)floor(sy - 0.5);
            const int lx = iSrcX == -1 ? 0 : iSrcX, ly = iSrcY == -1 ? 0 : iSrcY;
            // no sample: an offset past the band (< 2 GiB) reads 0 without a fetch
            const uint32_t o0 = ok ? (uint32_t)(ly * bx + lx) * 4u : 0x80000000u;
            const uint32_t o1 = ok ? o0 + (uint32_t)bx * 4u : 0x80000000u;
            sxv[i][q] = sx; syv[i][q] = sy; okc[i][q] = ok;
            t0[i][q] = __builtin_amdgcn_raw_buffer_load_b64(rs, o0, 0, 0);
            t1[i][q] = __builtin_amdgcn_raw_buffer_load_b64(rs, o1, 0, 0);
          }
        }
        // GWKBilinearResample4Sample + ordered fold (tile_merger.go:47-120)
#pragma unroll
        for (int i = 0; i < R; i++) {
#pragma unroll
          for (int q = 0; q < LPX; q++) {
            const double sx = sxv[i][q], sy = syv[i][q];
            float v = fillv, got;
            if (okc[i][q] && bil_combine(sx, sy, (int)floor(sx - 0.5), (int)floor(sy - 0.5), bx, by,
                                         __uint_as_float(t0[i][q].x), __uint_as_float(t0[i][q].y),
                                         __uint_as_float(t1[i][q].x), __uint_as_float(t1[i][q].y), hnd, nd64,
                                         got))
              v = got;
            const int ir = rb + i - eyoff;
            const bool in = ir >= 0 && ir < eh && rb + i < H && (unsigned)(ic0 + q * S) < (unsigned)lim;
            const bool take = in & (v != nd) & (!fill_mode | (c[i][q] == nd));
            c[i][q] = take ? v : c[i][q];
          }
        }
      }

      // typed float canvas (tile_merger.go:562-652), at the chunk's place in the coverage
#pragma unroll
      for (int i = 0; i < R; i++) {
        const int r = rb + i;
        if (r >= H || x0 >= W) continue;
        const int64_t eo = a.cov_offsets ? a.cov_offsets[t] + (int64_t)r * a.cov_stride + x0
                                         : (int64_t)r * a.max_w + x0;
        float *cdst = (float *)(a.cov_offsets ? a.canvas : a.canvas + t * a.canvas_tile_stride) + eo;
        if constexpr (S > 1) {   // 64 lanes x 4 B contiguous per store
#pragma unroll
          for (int q = 0; q < LPX; q++)
            if (x0 + q * S < W) __builtin_nontemporal_store(__float_as_uint(c[i][q]), (GPTR(uint32_t))(cdst + q * S));
        } else if (x0 + LPX <= W && (((uintptr_t)cdst) & 15) == 0 && LPX % 4 == 0) {
#pragma unroll
          for (int h = 0; h < LPX / 4; h++) {
            u32x4 v4 = {__float_as_uint(c[i][4 * h]), __float_as_uint(c[i][4 * h + 1]),
                        __float_as_uint(c[i][4 * h + 2]), __float_as_uint(c[i][4 * h + 3])};
            __builtin_nontemporal_store(v4, (GPTR(u32x4))(cdst + 4 * h));
          }
        } else {
#pragma unroll
          for (int q = 0; q < LPX; q++)
            if (x0 + q < W) cdst[q] = c[i][q];
        }
      }
    }
  }
}

// Bilinear float canvases (no mask layer): 4 pixels per lane 64 columns
// apart, one row at a time (the fastest of the round-2 lane shapes: C3
// 1.31-1.34 ms against 1.35-1.49 ms for 4 x 1 / 4 x 2 / 2 x 2 / 8 x 1
// consecutive and 2.30 ms for render_lds_kernel, profiles/r02r_*, r02z6_*).
void launch_bil(const RenderArgs &a, int n_items, hipStream_t s) {
  hipLaunchKernelGGL((render_bil_kernel<4, 1, 64, 0>), dim3((unsigned)n_items), dim3(256), 0, s, a, a.entries,
                     a.order, a.rows, a.pool, a.tplans, a.tiles, n_items);
}

}  // namespace gsky
