// render_nn.h -- the nearest-neighbour band kernel, second generation.
//
// Same work as render_lds_kernel's NN path (render_lds.h) -- every stack entry
// of the tile shares value type T, every row LINEAR or POOL(linear leaves),
// one rendered namespace, RGBA or typed canvas out -- shaped for memory-level
// parallelism instead of LDS tables:
//   * no entry tables and no barriers (after the palette load): every wave
//     walks the tile's entries in merge order with scalar loads, like the
//     generic kernel, and skips entries outside its rows / columns;
//   * a wave owns 4 consecutive rows of a 16-row band and a 512-column block;
//     it folds R rows at once, so R x LPX gathers per lane are in flight
//     before the first wait (R = 1 folds one row at a time);
//   * source coordinates by the reference's fp64 expressions (lin_coords(),
//     nn_px()); POOL rows walk their leaves incrementally -- exact rows and
//     exact pieces arrive as per-pixel leaves materialised by the planner
//     (plan_exact_kernel), so no transformer code runs here; 32.32 fixed
//     point (render_lds.h) is an A/B flag (kFixed);
//   * the gather is a raw buffer load whose offset is the element index times
//     sizeof(T): the "no pixel" index 0xFFFFFFFF lands past the buffer end, so
//     the hardware returns 0 without a fetch and no select is needed before
//     the load.  The planner sends tiles whose bands exceed 2 GiB or 2^24
//     pixels on a side to the general kernel (plan_tiles_kernel).
#pragma once
#include "render_lds.h"

namespace gsky {

constexpr uint32_t kNoPx = 0xFFFFFFFFu;

// Element index of each of the lane's LPX pixels on a LINEAR row, 32.32
// fixed point.  false (wave-uniform): some valid pixel of the wave sits
// inside the guard band around an integer, take the fp64 expressions.
template <int LPX>
__device__ __forceinline__ bool nn_index_fixed(double xs0, double ys0, double dX, double dY, int ic0, int ew,
                                               int lim, int bx, int by, uint32_t *idx) {
  const double xe = xs0 + dX * (double)ew, ye = ys0 + dY * (double)ew;
  const bool fits = fabs(xs0) < 1048576.0 && fabs(ys0) < 1048576.0 && fabs(xe) < 1048576.0 &&
                    fabs(ye) < 1048576.0 && ew < 65536;
  if (!fits) return false;
  const int64_t Dx = to_fix(dX), Dy = to_fix(dY);
  int64_t fx = to_fix(xs0 + 1.0e-10) + (int64_t)ic0 * Dx;
  int64_t fy = to_fix(ys0 + 1.0e-10) + (int64_t)ic0 * Dy;
  const uint32_t G = 4u * (uint32_t)(ew + 16) + 64u;   // guard, in 2^-32 px (render_lds.h)
  bool bad = false;
#pragma unroll
  for (int q = 0; q < LPX; q++) {
    const uint32_t lx = (uint32_t)fx, ly = (uint32_t)fy;
    const uint32_t ux = (uint32_t)(fx >> 32), uy = (uint32_t)(fy >> 32);
    const bool in = (unsigned)(ic0 + q) < (unsigned)lim;
    bad = bad || (in && (min(lx + G, ly + G) < 2u * G));
    const bool ok = in && ux < (uint32_t)bx && uy < (uint32_t)by;
    const uint32_t e = __umul24(uy, (uint32_t)bx) + ux;
    idx[q] = ok ? e : kNoPx;
    fx += Dx;
    fy += Dy;
  }
  return __ballot(bad) == 0ull;
}

// nn_px() of source coordinates (sx, sy): the element index, or kNoPx where
// the reference's window fill applies.
__device__ __forceinline__ uint32_t nn_index_sxy(double sx, double sy, bool ok, int bx, int by) {
  const int ix = __double2int_rz(sx + 1.0e-10), iy = __double2int_rz(sy + 1.0e-10);
  ok = ok && (sx >= 0.0) && (sy >= 0.0) && ix < bx && iy < by;
  return ok ? __umul24((uint32_t)iy, (uint32_t)bx) + (uint32_t)ix : kNoPx;
}

// Element indices of the lane's LPX pixels on a window row of an entry
// (lin_coords() + nn_px(), bit for bit).
template <int LPX, bool FIXED>
__device__ __forceinline__ void nn_row_index(const RowRec *__restrict__ rr, const Leaf *__restrict__ pool, int ic0,
                                             int ew, int lim, int bx, int by, uint32_t *idx) {
  const int kind = __builtin_amdgcn_readfirstlane(rr->kind);
  if (kind == ROW_LINEAR) {
    const double xs0 = rr->v[0], ys0 = rr->v[1], dX = rr->v[2], dY = rr->v[3];
    if (FIXED && nn_index_fixed<LPX>(xs0, ys0, dX, dY, ic0, ew, lim, bx, by, idx)) return;
#pragma unroll
    for (int q = 0; q < LPX; q++) {
      const bool in = (unsigned)(ic0 + q) < (unsigned)lim;
      const double dist = (double)ic0 + (double)q;
      idx[q] = nn_index_sxy(xs0 + dX * dist, ys0 + dY * dist, in, bx, by);
    }
    return;
  }
  // POOL (the only other kind in a simple tile): the lane's pixels are
  // consecutive, so the leaf (the last one starting at or before the pixel,
  // lin_coords()) only ever moves forward
  const int nleaf = __builtin_amdgcn_readfirstlane(rr->nleaf);
  const Leaf *lv = pool + __builtin_amdgcn_readfirstlane(rr->pool_off);
  const int icf = ic0 > 0 ? ic0 : 0;
  int l = leaf_of(lv, nleaf, icf);
  int nxt = l + 1 < nleaf ? lv[l + 1].start : 0x7FFFFFFF;
#pragma unroll
  for (int q = 0; q < LPX; q++) {
    const int ic = ic0 + q;
    const bool in = (unsigned)ic < (unsigned)lim;
    if (in && ic >= nxt) {
      while (l + 1 < nleaf && lv[l + 1].start <= ic) l++;
      nxt = l + 1 < nleaf ? lv[l + 1].start : 0x7FFFFFFF;
    }
    const Leaf &L = lv[l];
    const double dist = (double)(ic - L.start);
    idx[q] = nn_index_sxy(L.xs0 + L.dX * dist, L.ys0 + L.dY * dist, in && L.kind != LEAF_FAILED, bx, by);
  }
}

template <typename T, bool MASK, int LPX, int R, int FLAGS>
__global__ __launch_bounds__(256) void render_nn_kernel(RenderArgs a, const EntryD *__restrict__ ents,
                                                        const int32_t *__restrict__ order,
                                                        const RowRec *__restrict__ rows,
                                                        const Leaf *__restrict__ pool,
                                                        const TilePlan *__restrict__ tplans,
                                                        const gskyhip_tile *__restrict__ tiles, int n_items,
                                                        int per_xcd) {
  using V = typename VOf<T>::type;
  constexpr int kCols = 64 * LPX;   // columns of one wave pass
  __shared__ uint32_t s_ramp[256];

  // linear item order, or XCD-aware (per_xcd > 0: blocks b, b+8, ... share an
  // XCD and its L2) -- linear measured faster: neighbouring tiles on every XCD
  // share source rows through the MALL
  const int item = per_xcd > 0 ? (blockIdx.x & 7) * per_xcd + (blockIdx.x >> 3) : (int)blockIdx.x;
  if (item >= n_items) return;
  const int bands_per_tile = (a.max_h + kBandRows - 1) / kBandRows;
  const int col_blocks = (a.max_w + kBandCols - 1) / kBandCols;
  const int t = item / (bands_per_tile * col_blocks);
  const int in_tile = item - t * bands_per_tile * col_blocks;
  const TilePlan &tp = tplans[t];
  if (tp.complex || tp.vt != vt_code<T>()) return;
  const gskyhip_tile &tile = tiles[t];
  const int W = tile.width, H = tile.height;
  const int band0 = (in_tile / col_blocks) * kBandRows;
  const int xb = (in_tile % col_blocks) * kBandCols;
  if (band0 >= H || xb >= W) return;
  const int tid = threadIdx.x;
  if (a.ramp) s_ramp[tid] = a.ramp[tid];
  __syncthreads();
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const int r0 = band0 + wave * 4;
  if (r0 >= H) return;

  const int ns_out = a.out_ns[0];
  const bool created = tp.created[ns_out] != 0;
  const V cnod = as_v<T>(go_conv_to(tp.nodata[ns_out], tp.dtype[ns_out]));
  const int32_t *ord = order + tile.pair_begin;
  const int n_entries = a.nn_probe == 2 ? 0 : tp.n_entries;   // timing probe 2: stores only
  const ScaleK sk = make_scale(tp.dtype[ns_out], tp.nodata[ns_out], a.sp, false, 0.f, 0.f);
  const bool has_ramp = a.ramp != nullptr;
  uint8_t *rgba_tile = a.rgba + (int64_t)t * a.max_h * a.max_w * 4;
  const int xend = min(xb + kBandCols, W);

#pragma unroll 1
  for (int cx = xb; cx < xend; cx += kCols) {
    const int x0 = cx + lane * LPX;
#pragma unroll 1
    for (int j = 0; j < 4; j += R) {
      const int rb = r0 + j;
      if (rb >= H) break;
      V c[R][LPX];
#pragma unroll
      for (int i = 0; i < R; i++)
#pragma unroll
        for (int q = 0; q < LPX; q++) c[i][q] = cnod;

#pragma unroll 1
      for (int k = 0; k < n_entries; k++) {
        const int p = ord[k];
        const EntryD &e = ents[p];
        const int eyoff = e.yoff, eh = e.h, exoff = e.xoff, ew = e.w;
        if (e.ns != ns_out || ew <= 0) continue;
        if (rb + R <= eyoff || rb >= eyoff + eh) continue;
        if (cx + kCols <= exoff || cx >= exoff + ew) continue;
        const int bx = e.band_x, by = e.band_y;
        const V nd = as_v<T>(e.nd), fillv = as_v<T>(e.fill);
        const int fill_mode = e.fill_mode;
        const int64_t row_base = e.row_base;
        const int ic0 = x0 - exoff;
        const int lim = max(0, min(ew, W - exoff));   // pixel in the entry and the tile: (unsigned)ic < lim
        // timing probe 1 (A/B only): a zero-record descriptor, gathers read 0 without traffic
        const int nrec = a.nn_probe == 1 ? 0 : (int)((int64_t)bx * by * (int64_t)sizeof(T));
        const __amdgpu_buffer_rsrc_t rs =
            __builtin_amdgcn_make_buffer_rsrc((void *)uniform_ptr(e.band), (short)0, nrec, 0x00020000);
        uint32_t idx[R][LPX];
        V vv[R][LPX];
        // coordinates and gathers of all R rows first: R x LPX loads in flight
#pragma unroll
        for (int i = 0; i < R; i++) {
          const int ir = rb + i - eyoff;
          if (ir < 0 || ir >= eh || rb + i >= H) {
#pragma unroll
            for (int q = 0; q < LPX; q++) idx[i][q] = kNoPx;
          } else {
            nn_row_index<LPX, (FLAGS & kFixed) != 0>(rows + row_base + ir, pool, ic0, ew, lim, bx, by, idx[i]);
          }
#pragma unroll
          for (int q = 0; q < LPX; q++) vv[i][q] = buf_load<T>(rs, idx[i][q] * (uint32_t)sizeof(T));
        }
        // ordered fold (tile_merger.go:47-120)
#pragma unroll
        for (int i = 0; i < R; i++) {
          const int ir = rb + i - eyoff;
#pragma unroll
          for (int q = 0; q < LPX; q++) {
            const bool in = (unsigned)(ic0 + q) < (unsigned)lim && ir >= 0 && ir < eh;
            const V v = idx[i][q] != kNoPx ? vv[i][q] : fillv;
            bool take = in && (v != nd);
            if (MASK && e.mask_pair >= 0) {
              if (take) take = !mask_fast<GSKYHIP_RESAMPLE_NEAREST>(ents, rows, pool, a.mask, e, ic0 + q, ir);
            }
            const bool t2 = take && (!fill_mode || c[i][q] == nd);
            c[i][q] = t2 ? v : c[i][q];
          }
        }
      }

      // output: typed canvas (WCS) or utils.Scale + palette / grey RGBA
#pragma unroll
      for (int i = 0; i < R; i++) {
        const int r = rb + i;
        if (r >= H || x0 >= W) continue;
        if (a.nn_probe == 3) continue;   // timing probe 3: no stores
        if constexpr ((FLAGS & kCanvas) != 0) {
          const int64_t eo = a.cov_offsets ? a.cov_offsets[t] + (int64_t)r * a.cov_stride + x0
                                           : (int64_t)r * a.max_w + x0;
          T *cdst = (T *)(a.cov_offsets ? a.canvas : a.canvas + t * a.canvas_tile_stride) + eo;
          T tv[LPX];
#pragma unroll
          for (int q = 0; q < LPX; q++) tv[q] = (T)c[i][q];
          constexpr int kBytes = (int)sizeof(T) * LPX;
          if (x0 + LPX <= W && (((uintptr_t)cdst) & (kBytes >= 16 ? 15 : kBytes - 1)) == 0) {
            if constexpr (kBytes % 16 == 0) {
#pragma unroll
              for (int h = 0; h < kBytes / 16; h++) {
                u32x4 v4;
                __builtin_memcpy(&v4, (const char *)tv + 16 * h, 16);
                __builtin_nontemporal_store(v4, (GPTR(u32x4))((char *)cdst + 16 * h));
              }
            } else if constexpr (kBytes == 8) {
              uint64_t v2;
              __builtin_memcpy(&v2, tv, 8);
              *(uint64_t *)cdst = v2;
            } else {
              uint32_t v1;
              __builtin_memcpy(&v1, tv, 4);
              *(uint32_t *)cdst = v1;
            }
          } else {
#pragma unroll
            for (int q = 0; q < LPX; q++)
              if (x0 + q < W) cdst[q] = tv[q];
          }
        } else {
          uint32_t px[LPX];
#pragma unroll
          for (int q = 0; q < LPX; q++) {
            const uint32_t bb = scale_t<T>(sk, c[i][q]);
            const uint32_t col = has_ramp ? s_ramp[bb & 0xFFu] : (0xFF000000u | (bb << 16) | (bb << 8) | bb);
            px[q] = (created && bb != 0xFFu) ? col : 0u;
          }
          uint8_t *dst = rgba_tile + ((int64_t)r * a.max_w + x0) * 4;
          if (x0 + LPX <= W && ((((uintptr_t)dst) & 15) == 0)) {
#pragma unroll
            for (int h = 0; h < LPX / 4; h++) {
              u32x4 v4 = {px[4 * h], px[4 * h + 1], px[4 * h + 2], px[4 * h + 3]};
              __builtin_nontemporal_store(v4, (GPTR(u32x4))(dst + 16 * h));
            }
          } else {
#pragma unroll
            for (int q = 0; q < LPX; q++)
              if (x0 + q < W) ((uint32_t *)dst)[q] = px[q];
          }
        }
      }
    }
  }
}

// NN band kernel launch for value type T: lanes shape (LPX pixels x R rows)
// from RenderArgs.nn_shape (0: 4 x 4, 1: 8 x 1, 2: 8 x 2, 3: 4 x 2, the
// default: fastest on C2 and C5, profiles/r02h_ab_*.jsonl), 32.32
// fixed point when lds_flags has kFixed, XCD-aware order when nn_xcd
// (A/B knobs GSKYHIP_NN_SHAPE, GSKYHIP_LDS_FLAGS, GSKYHIP_NN_XCD).
template <typename T>
void launch_nn_t(const RenderArgs &a, bool mask, int n_items, hipStream_t s) {
  const int per_xcd = a.nn_xcd ? (n_items + 7) / 8 : 0;
  const dim3 grid(a.nn_xcd ? (unsigned)per_xcd * 8 : (unsigned)n_items);
#define GSKY_NN_LAUNCH(M, L, RR, F)                                                                              \
  hipLaunchKernelGGL((render_nn_kernel<T, M, L, RR, F>), grid, dim3(256), 0, s, a, a.entries, a.order, a.rows, \
                     a.pool, a.tplans, a.tiles, n_items, per_xcd)
  const bool canvas = (a.lds_mode & kCanvas) != 0;
  const bool fixed = (a.lds_flags & kFixed) != 0;
  if (mask) {
    if (canvas) GSKY_NN_LAUNCH(true, 4, 2, kCanvas); else GSKY_NN_LAUNCH(true, 4, 2, 0);
  } else if (fixed) {
    if (canvas) GSKY_NN_LAUNCH(false, 4, 4, kCanvas | kFixed); else GSKY_NN_LAUNCH(false, 4, 4, kFixed);
  } else if (a.nn_shape == 1) {
    if (canvas) GSKY_NN_LAUNCH(false, 8, 1, kCanvas); else GSKY_NN_LAUNCH(false, 8, 1, 0);
  } else if (a.nn_shape == 2) {
    if (canvas) GSKY_NN_LAUNCH(false, 8, 2, kCanvas); else GSKY_NN_LAUNCH(false, 8, 2, 0);
  } else if (a.nn_shape == 3) {
    if (canvas) GSKY_NN_LAUNCH(false, 4, 2, kCanvas); else GSKY_NN_LAUNCH(false, 4, 2, 0);
  } else {
    if (canvas) GSKY_NN_LAUNCH(false, 4, 4, kCanvas); else GSKY_NN_LAUNCH(false, 4, 4, 0);
  }
#undef GSKY_NN_LAUNCH
}

// Band kernel of one call: the NN kernel above (RenderArgs.nn_kernel, the
// default) or render_lds_kernel (bilinear, LDS staging, A/B variants).
template <typename T>
void launch_band_t(const RenderArgs &a, bool mask, int n_items, hipStream_t s) {
  if (a.nn_kernel && !(a.lds_mode & kBilinear) && !a.lds_stage)
    launch_nn_t<T>(a, mask, n_items, s);
  else
    launch_lds_t<T>(a, mask, n_items, s);
}

}  // namespace gsky
