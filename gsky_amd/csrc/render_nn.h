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
constexpr int kExpress = 16;   // render_nn2_kernel: single-entry express path (A/B knob GSKYHIP_NN_EXPRESS)
constexpr int kWide = 32;      // render_nn2_kernel: 16-B source-row loads for 16-bit values (GSKYHIP_NN_WIDE)
constexpr int kClampLut = 64;  // render_nn_kernel: Scale through the clamped-value LUT (GSKYHIP_NN_LUT)
constexpr int kStrided = 128;  // render_nn_kernel: lane pixels 64 columns apart (GSKYHIP_NN_STRIDE)
constexpr int kPlainStore = 256;   // render_nn_kernel, strided: cached instead of non-temporal RGBA stores (A/B)
constexpr int kLdsOut = 1024;      // render_nn_kernel, strided RGBA: rows collected in LDS, stored when the wave ends
constexpr int kWaves8 = 2048;      // render_nn_kernel: compiled for 8 waves per SIMD (<= 64 VGPRs) (A/B)
constexpr int kClampLutCap = 16384;   // LUT bytes in LDS: clip values 0 .. 16383

// utils.Scale of an integer canvas (scale_t) is, past the nodata test and
// the wrap + clamp of value + offset to [0, clip], a function of the clamped
// value alone: lut8[v] = go_u8_f32((float)v * sc) for v in [0, clip].  One
// launch builds it for the call's scale parameters; render_nn_kernel copies
// it to LDS and replaces the per-pixel convert / multiply / range test with
// one byte read (the palette entry 255 doubles as the transparent pixel).
template <typename T>
__global__ void clamp_lut_kernel(RenderArgs a, uint8_t *lut8, int n) {
  const int v = blockIdx.x * blockDim.x + threadIdx.x;
  if (v >= n) return;
  const ScaleK sk = make_scale(vt_code<T>(), 0.0, a.sp, false, 0.f, 0.f);
  lut8[v] = (uint8_t)go_u8_f32((float)v * sk.sc);
}

// Entries of that LUT for value type T under the call's scale parameters
// (clip in the canvas type, as make_scale() converts it), or 0 when it does
// not fit in LDS.
template <typename T>
__host__ __device__ inline int clamp_lut_size(const RenderArgs &a) {
  if constexpr (std::is_same<T, float>::value) return 0;
  else {
    const int clp = go_conv_to(a.sp.clip, vt_code<T>()).i;
    const int n = (clp > 0 ? clp : 0) + 1;
    return n <= kClampLutCap ? n : 0;
  }
}

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
// S: column stride between the lane's pixels (1: consecutive, 64: the
// wave's lanes cover 64 consecutive columns per pixel slot).
template <int LPX, bool FIXED, int S = 1>
__device__ __forceinline__ void nn_row_index(const RowRec *__restrict__ rr, const Leaf *__restrict__ pool, int ic0,
                                             int ew, int lim, int bx, int by, uint32_t *idx) {
  const int kind = __builtin_amdgcn_readfirstlane(rr->kind);
  if (kind == ROW_LINEAR) {
    const double xs0 = rr->v[0], ys0 = rr->v[1], dX = rr->v[2], dY = rr->v[3];
    if constexpr (S == 1) {
      if (FIXED && nn_index_fixed<LPX>(xs0, ys0, dX, dY, ic0, ew, lim, bx, by, idx)) return;
    }
#pragma unroll
    for (int q = 0; q < LPX; q++) {
      const bool in = (unsigned)(ic0 + q * S) < (unsigned)lim;
      const double dist = (double)ic0 + (double)(q * S);
      idx[q] = nn_index_sxy(xs0 + dX * dist, ys0 + dY * dist, in, bx, by);
    }
    return;
  }
  // POOL (the only other kind in a simple tile): the lane's pixels ascend,
  // so the leaf (the last one starting at or before the pixel, lin_coords())
  // only ever moves forward
  const int nleaf = __builtin_amdgcn_readfirstlane(rr->nleaf);
  const Leaf *lv = pool + __builtin_amdgcn_readfirstlane(rr->pool_off);
  const int icf = ic0 > 0 ? ic0 : 0;
  int l = leaf_of(lv, nleaf, icf);
  int nxt = l + 1 < nleaf ? lv[l + 1].start : 0x7FFFFFFF;
#pragma unroll
  for (int q = 0; q < LPX; q++) {
    const int ic = ic0 + q * S;
    if (S > 1 && ic >= nxt) {   // 64 columns on: search again rather than walk
      l = leaf_of(lv, nleaf, ic > 0 ? ic : 0);
      nxt = l + 1 < nleaf ? lv[l + 1].start : 0x7FFFFFFF;
    }
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

template <typename T, bool MASK, int LPX, int R, int FLAGS, int RPW = 4>
__global__ __launch_bounds__(256, (FLAGS & kWaves8) != 0 ? 8 : 1) void render_nn_kernel(RenderArgs a, const EntryD *__restrict__ ents,
                                                        const int32_t *__restrict__ order,
                                                        const RowRec *__restrict__ rows,
                                                        const Leaf *__restrict__ pool,
                                                        const TilePlan *__restrict__ tplans,
                                                        const gskyhip_tile *__restrict__ tiles, int n_items,
                                                        int per_xcd) {
  using V = typename VOf<T>::type;
  constexpr int kCols = 64 * LPX;   // columns of one wave pass
  constexpr bool kLutOut = (FLAGS & kClampLut) != 0 && (FLAGS & kCanvas) == 0 && !std::is_same<T, float>::value;
  // S: column step between a lane's pixels.  1: LPX consecutive pixels (one
  // 16-B store); 64: each pixel slot of the wave covers 64 consecutive
  // columns, so one gather instruction touches about half the source lines
  constexpr int S = (FLAGS & kStrided) != 0 ? 64 : 1;
  __shared__ uint32_t s_ramp[256];
  __shared__ __attribute__((aligned(16))) uint8_t s_lut[kLutOut ? kClampLutCap : 16];
  // kOutLds: the wave's RGBA rows wait in LDS and leave in one burst of
  // 16-B stores at the end.  vmcnt counts loads and stores in issue order,
  // so a store issued between two entry iterations makes the next gathers'
  // wait drain it too; with the stores last, the gather chain never waits
  // for the write stream
  constexpr bool kOutLds = (FLAGS & kLdsOut) != 0 && S > 1 && (FLAGS & kCanvas) == 0;
  __shared__ __attribute__((aligned(16))) uint32_t s_out[kOutLds ? 4 * RPW * kBandCols : 4];

  // linear item order, or XCD-aware (per_xcd > 0: blocks b, b+8, ... share an
  // XCD and its L2) -- linear measured faster: neighbouring tiles on every XCD
  // share source rows through the MALL
  const int item = per_xcd > 0 ? (blockIdx.x & 7) * per_xcd + (blockIdx.x >> 3) : (int)blockIdx.x;
  if (item >= n_items) return;
  constexpr int kRowsPerBlock = 4 * RPW;   // RPW rows per wave (A/B knob nn_rpw; 4 = kBandRows)
  const int bands_per_tile = (a.max_h + kRowsPerBlock - 1) / kRowsPerBlock;
  const int col_blocks = (a.max_w + kBandCols - 1) / kBandCols;
  const int t = item / (bands_per_tile * col_blocks);
  const int in_tile = item - t * bands_per_tile * col_blocks;
  const TilePlan &tp = tplans[t];
  if (tp.complex || (tp.n_entries > 0 && tp.vt != vt_code<T>())) return;   // empty tiles: written here
  const gskyhip_tile &tile = tiles[t];
  const int W = tile.width, H = tile.height;
  const int band0 = (in_tile / col_blocks) * kRowsPerBlock;
  const int xb = (in_tile % col_blocks) * kBandCols;
  if (band0 >= H || xb >= W) return;
  const int tid = threadIdx.x;
  const int ns_out = a.out_ns[0];
  // clamped-value LUT: only for canvases of T's own type (empty tiles may carry another)
  const bool use_lut = kLutOut && tp.dtype[ns_out] == vt_code<T>();
  int lut_n = 0;
  if constexpr (kLutOut) {
    if (use_lut) {
      const uint32_t g = (uint32_t)tid;
      s_ramp[tid] = tid == 255 ? 0u : (a.ramp ? a.ramp[tid] : (0xFF000000u | (g << 16) | (g << 8) | g));
      lut_n = clamp_lut_size<T>(a);
      const int n16 = (lut_n + 15) >> 4;
      for (int i = tid; i < n16; i += 256)
        reinterpret_cast<u32x4 *>(s_lut)[i] = reinterpret_cast<const u32x4 *>(a.lut)[i];
    } else if (a.ramp) {
      s_ramp[tid] = a.ramp[tid];
    }
  } else if (a.ramp) {
    s_ramp[tid] = a.ramp[tid];
  }
  __syncthreads();
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const int r0 = band0 + wave * RPW;
  if (r0 >= H) return;

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
    const int x0 = cx + (S == 1 ? lane * LPX : lane);
#pragma unroll 1
    for (int j = 0; j < RPW; j += R) {
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
            nn_row_index<LPX, (FLAGS & kFixed) != 0, S>(rows + row_base + ir, pool, ic0, ew, lim, bx, by, idx[i]);
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
            const bool in = (unsigned)(ic0 + q * S) < (unsigned)lim && ir >= 0 && ir < eh;
            const V v = idx[i][q] != kNoPx ? vv[i][q] : fillv;
            bool take = in && (v != nd);
            if (MASK && e.mask_pair >= 0) {
              if (take) take = !mask_fast<GSKYHIP_RESAMPLE_NEAREST>(ents, rows, pool, a.mask, e, ic0 + q * S, ir);
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
          if constexpr (S > 1) {
#pragma unroll
            for (int q = 0; q < LPX; q++)
              if (x0 + q * S < W) cdst[q * S] = tv[q];
          } else if (x0 + LPX <= W && (((uintptr_t)cdst) & (kBytes >= 16 ? 15 : kBytes - 1)) == 0) {
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
          if (kLutOut && use_lut) {   // scale_t(): nodata test, wrap + clamp, then the LUT byte
#pragma unroll
            for (int q = 0; q < LPX; q++) {
              int32_t value = c[i][q] + sk.off.i;
              if constexpr (std::is_same<T, int8_t>::value) value = (int8_t)value;
              else if constexpr (std::is_same<T, uint8_t>::value) value = (uint8_t)value;
              else if constexpr (std::is_same<T, int16_t>::value) value = (int16_t)value;
              else value = (uint16_t)value;
              value = max(min(value, sk.clp.i), 0);
              const uint32_t col = s_ramp[s_lut[value]];
              px[q] = (created && c[i][q] != sk.noData.i) ? col : 0u;
            }
          } else if (a.nn_probe == 4) {   // timing probe 4: no Scale / palette (raw values out)
#pragma unroll
            for (int q = 0; q < LPX; q++) px[q] = (uint32_t)c[i][q];
          } else {
#pragma unroll
            for (int q = 0; q < LPX; q++) {
              const uint32_t bb = scale_t<T>(sk, c[i][q]);
              const uint32_t col = has_ramp ? s_ramp[bb & 0xFFu] : (0xFF000000u | (bb << 16) | (bb << 8) | bb);
              px[q] = (created && bb != 0xFFu) ? col : 0u;
            }
          }
          uint8_t *dst = rgba_tile + ((int64_t)r * a.max_w + x0) * 4;
          if constexpr (kOutLds) {
            uint32_t *so = s_out + (wave * RPW + j + i) * kBandCols + (cx - xb) + lane;
#pragma unroll
            for (int q = 0; q < LPX; q++) so[q * S] = px[q];
          } else if constexpr (S > 1) {   // 64 lanes x 4 B contiguous per store
#pragma unroll
            for (int q = 0; q < LPX; q++)
              if (x0 + q * S < W) {
                if constexpr ((FLAGS & kPlainStore) != 0) *(GPTR(uint32_t))(dst + 4 * q * S) = px[q];
                else __builtin_nontemporal_store(px[q], (GPTR(uint32_t))(dst + 4 * q * S));
              }
          } else if (x0 + LPX <= W && ((((uintptr_t)dst) & 15) == 0)) {
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
  if constexpr (kOutLds) {
    if (a.nn_probe == 3) return;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const int ncols = xend - xb;
    const int c0 = lane * 8;   // a lane's 8 columns of each row: two 16-B stores
#pragma unroll 1
    for (int jj = 0; jj < RPW; jj++) {
      const int r = r0 + jj;
      if (r >= H) break;
      const uint32_t *src = s_out + (wave * RPW + jj) * kBandCols + c0;
      uint8_t *d = rgba_tile + ((int64_t)r * a.max_w + xb + c0) * 4;
      if (c0 + 8 <= ncols && (((uintptr_t)d) & 15) == 0) {
        const u32x4 v0 = *(const u32x4 *)src, v1 = *(const u32x4 *)(src + 4);
        __builtin_nontemporal_store(v0, (GPTR(u32x4))d);
        __builtin_nontemporal_store(v1, (GPTR(u32x4))(d + 16));
      } else {
#pragma unroll
        for (int q = 0; q < 8; q++)
          if (c0 + q < ncols) __builtin_nontemporal_store(src[q], (GPTR(uint32_t))(d + 4 * q));
      }
    }
  }
}

// ---------------------------------------------------------------- third generation
// render_nn2_kernel: the work of render_nn_kernel (no-mask tiles) with the
// VALU per pixel cut down -- the kernel above measured VALU-issue bound
// (profiles/pmc_render_nn_c2_r02h.json: ~42 VALU lane-ops per output pixel,
// SIMDs 61 % VALU-busy):
//   * rows the planner marked `inside` (every window pixel's NN source pixel
//     lies in the band, RowRec.inside) skip the per-pixel sign / size tests,
//     the "no pixel" index and the window-fill select: truncate, index, load;
//   * 8/16-bit values travel through the fold as zero-extended bit patterns
//     (the fold only compares and selects), sign-extended once at the output;
//   * the output is branch-free: utils.Scale in the canvas type, Go's
//     uint8(float32) range test only when float32(clip) * scale can reach
//     2^31 (wave-uniform), and the palette / grey ramp in LDS with the
//     EncodePNG transparency rule baked in (entry 255 and uncreated canvases
//     are 0), so one LDS read per pixel replaces the select chain.
// Rows that are not `inside` (window edges, POOL rows) take the exact
// expressions of nn_row_index() with the fill select, as before.
template <typename T> struct POf { using type = uint32_t; };
template <> struct POf<float> { using type = float; };

template <typename T>
__device__ __forceinline__ typename POf<T>::type to_pat(Val x) {
  if constexpr (std::is_same<T, float>::value) return x.f;
  else return (uint32_t)x.i & (sizeof(T) == 1 ? 0xFFu : 0xFFFFu);
}

template <typename T>
__device__ __forceinline__ typename POf<T>::type buf_load_pat(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  if constexpr (sizeof(T) == 1) return (uint32_t)__builtin_amdgcn_raw_buffer_load_b8(r, off, 0, 0);
  else if constexpr (sizeof(T) == 2) return (uint32_t)__builtin_amdgcn_raw_buffer_load_b16(r, off, 0, 0);
  else return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0));
}

// utils.Scale of an integer canvas value given as its bit pattern (the
// arithmetic of scale_t(): value += offset wrapping in T, clip, clamp at 0,
// float32 multiply, Go uint8(float32)); 0xFF for the canvas nodata.
template <typename T, bool SAFE>
__device__ __forceinline__ uint32_t scale_pat(uint32_t c, uint32_t nd_pat, int32_t off, int32_t clp, float sc) {
  int32_t value = (int32_t)(c + (uint32_t)off);
  if constexpr (std::is_same<T, int8_t>::value) value = (int8_t)value;
  else if constexpr (std::is_same<T, uint8_t>::value) value = (uint8_t)value;
  else if constexpr (std::is_same<T, int16_t>::value) value = (int16_t)value;
  else value = (uint16_t)value;
  value = max(min(value, clp), 0);
  const float f = (float)value * sc;
  const uint32_t b = SAFE ? ((uint32_t)(int32_t)f & 0xFFu) : go_u8_f32(f);   // SAFE: 0 <= f < 2^31
  return c == nd_pat ? 0xFFu : b;
}

// NN gathers of a lane's LPX consecutive pixels on an `inside` LINEAR row of
// a 16-bit band with one 16-byte load per source row the pixels touch: at
// the ~2x upsampling of C2 four destination pixels fall on 2-3 source pixels
// of 1-2 rows, so 1-2 wide loads replace 4 two-byte gathers (the gather
// instruction count is what the kernel issues most).  The indices are the
// reference's fp64 expressions (lin_coords() + nn_px()); the coordinates are
// monotone along the row, so the end pixels bound the span.  A lane whose
// pixels span more than 7 elements or 2 rows, or reach the band's last 8
// elements, gathers per pixel as before.  Values come back zero-extended
// (the fold's bit patterns).
template <int LPX>
__device__ __forceinline__ void wide_gather16(__amdgpu_buffer_rsrc_t rs, const RowRec *rr, int ic0, int bx,
                                              uint32_t nel, uint32_t *v) {
  const double xs0 = rr->v[0], ys0 = rr->v[1], dX = rr->v[2], dY = rr->v[3];
  int ix[LPX], iy[LPX];
#pragma unroll
  for (int q = 0; q < LPX; q++) {
    const double dist = (double)(ic0 + q);
    ix[q] = __double2int_rz(xs0 + dX * dist + 1.0e-10);
    iy[q] = __double2int_rz(ys0 + dY * dist + 1.0e-10);
  }
  const int xa = min(ix[0], ix[LPX - 1]), xz = max(ix[0], ix[LPX - 1]);
  const int ya = min(iy[0], iy[LPX - 1]), yz = max(iy[0], iy[LPX - 1]);
  const bool wide = xa >= 0 && ya >= 0 && xz - xa <= 6 && yz - ya <= 1 &&
                    (uint64_t)(ya + 1) * (uint32_t)bx + (uint32_t)xa + 8u <= (uint64_t)nel;
  if (wide) {
    const uint32_t e0 = __umul24((uint32_t)ya, (uint32_t)bx) + (uint32_t)xa;
    const uint32_t s0 = e0 & 1u;
    const u32x4 w0 = __builtin_amdgcn_raw_buffer_load_b128(rs, (e0 & ~1u) * 2u, 0, 0);
    u32x4 w1 = w0;
    uint32_t s1 = s0;
    if (yz != ya) {
      const uint32_t e1 = e0 + (uint32_t)bx;
      s1 = e1 & 1u;
      w1 = __builtin_amdgcn_raw_buffer_load_b128(rs, (e1 & ~1u) * 2u, 0, 0);
    }
#pragma unroll
    for (int q = 0; q < LPX; q++) {
      const bool r1 = iy[q] != ya;
      const uint32_t k = (r1 ? s1 : s0) + (uint32_t)(ix[q] - xa);
      const uint32_t d0 = r1 ? w1.x : w0.x, d1 = r1 ? w1.y : w0.y;
      const uint32_t d2 = r1 ? w1.z : w0.z, d3 = r1 ? w1.w : w0.w;
      const uint32_t d = k < 4u ? (k < 2u ? d0 : d1) : (k < 6u ? d2 : d3);
      v[q] = (d >> ((k & 1u) * 16u)) & 0xFFFFu;
    }
  } else {
#pragma unroll
    for (int q = 0; q < LPX; q++)
      v[q] = (uint32_t)__builtin_amdgcn_raw_buffer_load_b16(
          rs, (__umul24((uint32_t)iy[q], (uint32_t)bx) + (uint32_t)ix[q]) * 2u, 0, 0);
  }
}

template <typename T, int LPX, int R, int FLAGS, int WPE>
__global__ __launch_bounds__(256, WPE) void render_nn2_kernel(RenderArgs a, const EntryD *__restrict__ ents,
                                                         const int32_t *__restrict__ order,
                                                         const RowRec *__restrict__ rows,
                                                         const Leaf *__restrict__ pool,
                                                         const TilePlan *__restrict__ tplans,
                                                         const gskyhip_tile *__restrict__ tiles, int n_items) {
  using P = typename POf<T>::type;
  constexpr bool kInt = !std::is_same<T, float>::value;
  constexpr bool kCv = (FLAGS & kCanvas) != 0;
  constexpr bool kWide16 = (FLAGS & kWide) != 0 && sizeof(T) == 2;
  constexpr int kCols = 64 * LPX;
  __shared__ uint32_t s_tab[256];

  const int item = blockIdx.x;
  if (item >= n_items) return;
  const int bands_per_tile = (a.max_h + kBandRows - 1) / kBandRows;
  const int col_blocks = (a.max_w + kBandCols - 1) / kBandCols;
  const int t = item / (bands_per_tile * col_blocks);
  const int in_tile = item - t * bands_per_tile * col_blocks;
  const TilePlan &tp = tplans[t];
  if (tp.complex || (tp.n_entries > 0 && tp.vt != vt_code<T>())) return;   // empty tiles: written here
  const gskyhip_tile &tile = tiles[t];
  const int W = tile.width, H = tile.height;
  const int band0 = (in_tile / col_blocks) * kBandRows;
  const int xb = (in_tile % col_blocks) * kBandCols;
  if (band0 >= H || xb >= W) return;
  const int tid = threadIdx.x;
  const int ns_out = a.out_ns[0];
  const bool created = tp.created[ns_out] != 0;
  if constexpr (!kCv) {   // EncodePNG: utils.Scale 0xFF and uncreated canvases are transparent
    const uint32_t col = a.ramp ? a.ramp[tid] : (0xFF000000u | ((uint32_t)tid * 0x10101u));
    s_tab[tid] = (created && tid != 255) ? col : 0u;
    __syncthreads();
  }
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const int r0 = band0 + wave * 4;
  if (r0 >= H) return;

  const P cnod = to_pat<T>(go_conv_to(tp.nodata[ns_out], tp.dtype[ns_out]));
  const int32_t *ord = order + tile.pair_begin;
  const int n_entries = tp.n_entries;
  const ScaleK sk = make_scale(tp.dtype[ns_out], tp.nodata[ns_out], a.sp, false, 0.f, 0.f);
  const bool safe = !kInt || (float)max(sk.clp.i, 0) * sk.sc < 2147483648.0f;   // NaN -> false
  uint8_t *rgba_tile = a.rgba + (int64_t)t * a.max_h * a.max_w * 4;
  const int xend = min(xb + kBandCols, W);

  // output of the lane's LPX pixels of row r from x0: typed canvas (WCS) or
  // utils.Scale + palette / grey RGBA
  auto emit = [&](int r, int x0, const P *cv) {
    if (r >= H || x0 >= W) return;
    if constexpr (kCv) {
      const int64_t eo = a.cov_offsets ? a.cov_offsets[t] + (int64_t)r * a.cov_stride + x0
                                       : (int64_t)r * a.max_w + x0;
      T *cdst = (T *)(a.cov_offsets ? a.canvas : a.canvas + t * a.canvas_tile_stride) + eo;
      T tv[LPX];
#pragma unroll
      for (int q = 0; q < LPX; q++) {
        if constexpr (kInt) tv[q] = (T)cv[q]; else tv[q] = cv[q];
      }
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
      if constexpr (kInt) {
        const uint32_t ndp = to_pat<T>(sk.noData);
        if (safe) {
#pragma unroll
          for (int q = 0; q < LPX; q++) px[q] = s_tab[scale_pat<T, true>(cv[q], ndp, sk.off.i, sk.clp.i, sk.sc)];
        } else {
#pragma unroll
          for (int q = 0; q < LPX; q++) px[q] = s_tab[scale_pat<T, false>(cv[q], ndp, sk.off.i, sk.clp.i, sk.sc)];
        }
      } else {
#pragma unroll
        for (int q = 0; q < LPX; q++) px[q] = s_tab[scale_t<T>(sk, cv[q]) & 0xFFu];
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
  };

  // Express path (wave-uniform): the tile has one entry, it covers the
  // wave's 4 rows, every one of them `inside`, and the block is at most two
  // passes wide.  All 2 x 4 x LPX gathers of the wave are issued before the
  // first wait: one scalar chain and one gather round trip per wave instead
  // of one per (pass, row) -- the general loops below are latency-bound.
  if (n_entries == 1 && r0 + 4 <= H && xend - xb <= 2 * kCols && (FLAGS & kExpress)) {
    const EntryD &e = ents[ord[0]];
    const int eyoff = e.yoff, exoff = e.xoff, ew = e.w;
    bool ok = e.ns == ns_out && ew > 0 && r0 >= eyoff && r0 + 4 <= eyoff + e.h;
    const RowRec *rr = rows + e.row_base + (r0 - eyoff);
#pragma unroll
    for (int i = 0; i < 4; i++)
      ok = ok && __builtin_amdgcn_readfirstlane(rr[i].kind) == ROW_LINEAR &&
           __builtin_amdgcn_readfirstlane(rr[i].inside) != 0;
    if (ok) {
      const int bx = e.band_x, by = e.band_y;
      const P nd = to_pat<T>(e.nd);
      const bool allow = e.fill_mode == 0 || cnod == nd;   // fill mode: only onto canvas nodata
      const int lim = allow ? max(0, min(ew, W - exoff)) : 0;
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
          (void *)uniform_ptr(e.band), (short)0, (int)((int64_t)bx * by * (int64_t)sizeof(T)), 0x00020000);
      const bool two = xend - xb > kCols;
      P vv[2][4][LPX];
#pragma unroll
      for (int pp = 0; pp < 2; pp++) {
        if (pp == 1 && !two) break;
        const int ic0 = xb + pp * kCols + lane * LPX - exoff;
#pragma unroll
        for (int i = 0; i < 4; i++) {
          if constexpr (kWide16) {
            wide_gather16<LPX>(rs, rr + i, ic0, bx, (uint32_t)bx * (uint32_t)by, vv[pp][i]);
            continue;
          }
          const double xs0 = rr[i].v[0], ys0 = rr[i].v[1], dX = rr[i].v[2], dY = rr[i].v[3];
#pragma unroll
          for (int q = 0; q < LPX; q++) {
            const double dist = (double)(ic0 + q);
            const int ix = __double2int_rz(xs0 + dX * dist + 1.0e-10);
            const int iy = __double2int_rz(ys0 + dY * dist + 1.0e-10);
            vv[pp][i][q] = buf_load_pat<T>(rs, (__umul24((uint32_t)iy, (uint32_t)bx) + (uint32_t)ix) * (uint32_t)sizeof(T));
          }
        }
      }
      // one entry: the fold is "take the value unless nodata or outside the window"
#pragma unroll
      for (int pp = 0; pp < 2; pp++) {
        if (pp == 1 && !two) break;
        const int x0 = xb + pp * kCols + lane * LPX;
        const int ic0 = x0 - exoff;
#pragma unroll
        for (int i = 0; i < 4; i++) {
          P cv[LPX];
#pragma unroll
          for (int q = 0; q < LPX; q++)
            cv[q] = (((unsigned)(ic0 + q) < (unsigned)lim) & (vv[pp][i][q] != nd)) ? vv[pp][i][q] : cnod;
          emit(r0 + i, x0, cv);
        }
      }
      return;
    }
  }

#pragma unroll 1
  for (int cx = xb; cx < xend; cx += kCols) {
    const int x0 = cx + lane * LPX;
#pragma unroll 1
    for (int j = 0; j < 4; j += R) {
      const int rb = r0 + j;
      if (rb >= H) break;
      P c[R][LPX];
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
        const P nd = to_pat<T>(e.nd), fillv = to_pat<T>(e.fill);
        const bool fill_mode = e.fill_mode != 0;
        const RowRec *rrow = rows + e.row_base;
        const int ic0 = x0 - exoff;
        const int lim = max(0, min(ew, W - exoff));
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            (void *)uniform_ptr(e.band), (short)0, (int)((int64_t)bx * by * (int64_t)sizeof(T)), 0x00020000);
        bool inq[LPX];
#pragma unroll
        for (int q = 0; q < LPX; q++) inq[q] = (unsigned)(ic0 + q) < (unsigned)lim;
        // row state (wave-uniform): 0 no pixel, 1 inside (fast), 2 exact tests
        int st[R];
        bool all_fast = true;
#pragma unroll
        for (int i = 0; i < R; i++) {
          const int ir = rb + i - eyoff;
          if (ir < 0 || ir >= eh || rb + i >= H) {
            st[i] = 0;
          } else {
            const RowRec *rr = rrow + ir;
            const bool in = __builtin_amdgcn_readfirstlane(rr->kind) == ROW_LINEAR &&
                            __builtin_amdgcn_readfirstlane(rr->inside) != 0;
            st[i] = in ? 1 : 2;
            all_fast = all_fast && in;
          }
        }
        P vv[R][LPX];
        if (all_fast) {
          // every row inside (or empty): truncate, index, load -- nothing else
#pragma unroll
          for (int i = 0; i < R; i++) {
            if (st[i] == 0) continue;
            const RowRec *rr = rrow + (rb + i - eyoff);
            if constexpr (kWide16) {
              wide_gather16<LPX>(rs, rr, ic0, bx, (uint32_t)bx * (uint32_t)by, vv[i]);
              continue;
            }
            const double xs0 = rr->v[0], ys0 = rr->v[1], dX = rr->v[2], dY = rr->v[3];
#pragma unroll
            for (int q = 0; q < LPX; q++) {
              const double dist = (double)(ic0 + q);
              const int ix = __double2int_rz(xs0 + dX * dist + 1.0e-10);
              const int iy = __double2int_rz(ys0 + dY * dist + 1.0e-10);
              vv[i][q] = buf_load_pat<T>(rs, (__umul24((uint32_t)iy, (uint32_t)bx) + (uint32_t)ix) * (uint32_t)sizeof(T));
            }
          }
          // ordered fold (tile_merger.go:47-120); bitwise &, not &&: a short
          // circuit lets the compiler sink a gather under a branch
          if (!fill_mode) {
#pragma unroll
            for (int i = 0; i < R; i++) {
              if (st[i] == 0) continue;
#pragma unroll
              for (int q = 0; q < LPX; q++) c[i][q] = (inq[q] & (vv[i][q] != nd)) ? vv[i][q] : c[i][q];
            }
          } else {
#pragma unroll
            for (int i = 0; i < R; i++) {
              if (st[i] == 0) continue;
#pragma unroll
              for (int q = 0; q < LPX; q++)
                c[i][q] = (inq[q] & (vv[i][q] != nd) & (c[i][q] == nd)) ? vv[i][q] : c[i][q];
            }
          }
        } else {
          // some row needs the exact tests: one row at a time (keeps the
          // register peak of the R-row fast path)
#pragma unroll
          for (int i = 0; i < R; i++) {
            if (st[i] == 0) continue;
            uint32_t idx[LPX];
            P v1[LPX];
            nn_row_index<LPX, false>(rrow + (rb + i - eyoff), pool, ic0, ew, lim, bx, by, idx);
#pragma unroll
            for (int q = 0; q < LPX; q++) v1[q] = buf_load_pat<T>(rs, idx[q] * (uint32_t)sizeof(T));
#pragma unroll
            for (int q = 0; q < LPX; q++) {
              const P v = idx[q] != kNoPx ? v1[q] : fillv;
              const bool take = inq[q] & (v != nd) & (!fill_mode | (c[i][q] == nd));
              c[i][q] = take ? v : c[i][q];
            }
          }
        }
      }

#pragma unroll
      for (int i = 0; i < R; i++) emit(rb + i, x0, c[i]);
    }
  }
}

// NN band kernel launch for value type T: lanes shape (LPX pixels x R rows)
// from RenderArgs.nn_shape (0: 4 x 4, 1: 8 x 1, 2: 8 x 2, 3: 4 x 2 (the
// round-2 default until r02z10), 4: 4 x 1 compiled for 8 waves per SIMD,
// 5: the same for the masked kernel too (the default)), lane pixels 64
// columns apart when nn_stride (default; typed canvases use 4 x 2), 32.32
// fixed point when
// lds_flags has kFixed, XCD-aware order when nn_xcd (A/B knobs
// GSKYHIP_NN_SHAPE, GSKYHIP_NN_STRIDE, GSKYHIP_LDS_FLAGS, GSKYHIP_NN_XCD;
// profiles/r02h_ab_*.jsonl, r02z*_ab_*.jsonl).
template <typename T>
void launch_nn_t(const RenderArgs &a, bool mask, int n_items, hipStream_t s) {
  const int per_xcd = a.nn_xcd ? (n_items + 7) / 8 : 0;
  const dim3 grid(a.nn_xcd ? (unsigned)per_xcd * 8 : (unsigned)n_items);
#define GSKY_NN_LAUNCH(M, L, RR, F)                                                                              \
  hipLaunchKernelGGL((render_nn_kernel<T, M, L, RR, F>), grid, dim3(256), 0, s, a, a.entries, a.order, a.rows, \
                     a.pool, a.tplans, a.tiles, n_items, per_xcd)
  const bool canvas = (a.lds_mode & kCanvas) != 0;
  const bool fixed = (a.lds_flags & kFixed) != 0;
  if (!mask && !fixed && a.nn_gen >= 3 && a.nn_probe == 0) {   // third generation (A/B)
#define GSKY_NN2_LAUNCH(L, RR, F, WP)                                                                          \
  hipLaunchKernelGGL((render_nn2_kernel<T, L, RR, F, WP>), dim3((unsigned)n_items), dim3(256), 0, s, a,      \
                     a.entries, a.order, a.rows, a.pool, a.tplans, a.tiles, n_items)
#define GSKY_NN2_SHAPE(L, RR, WP) \
  do { if (canvas) GSKY_NN2_LAUNCH(L, RR, kCanvas, WP); else GSKY_NN2_LAUNCH(L, RR, 0, WP); } while (0)
#define GSKY_NN2_SHAPE_X(L, RR, WP)                                                  \
  do {                                                                               \
    if (a.nn_express && a.nn_wide) {                                                 \
      if (canvas) GSKY_NN2_LAUNCH(L, RR, kCanvas | kExpress | kWide, WP);            \
      else GSKY_NN2_LAUNCH(L, RR, kExpress | kWide, WP);                             \
    } else if (a.nn_wide) {                                                          \
      if (canvas) GSKY_NN2_LAUNCH(L, RR, kCanvas | kWide, WP);                       \
      else GSKY_NN2_LAUNCH(L, RR, kWide, WP);                                        \
    } else if (a.nn_express) {                                                       \
      if (canvas) GSKY_NN2_LAUNCH(L, RR, kCanvas | kExpress, WP);                    \
      else GSKY_NN2_LAUNCH(L, RR, kExpress, WP);                                     \
    } else GSKY_NN2_SHAPE(L, RR, WP);                                                \
  } while (0)
    // A/B knobs: nn_shape (0: 4 x 4, 1: 8 x 1, 4: 4 x 1, else 4 x 2), nn_wpe (minimum waves per SIMD the
    // compiler must fit: 0 = free, 6, 8), nn_express (single-entry express path, default on)
    if (a.nn_shape == 0) GSKY_NN2_SHAPE(4, 4, 1);
    else if (a.nn_shape == 1) GSKY_NN2_SHAPE(8, 1, 1);
    else if (a.nn_shape == 4) GSKY_NN2_SHAPE_X(4, 1, 1);
    else {
      if (a.nn_wpe == 6) GSKY_NN2_SHAPE(4, 2, 6);
      else GSKY_NN2_SHAPE_X(4, 2, 1);
    }
#undef GSKY_NN2_SHAPE_X
#undef GSKY_NN2_SHAPE
#undef GSKY_NN2_LAUNCH
    return;
  }
  // Scale through the clamped-value LUT (RGBA out, integer T, default shape)
  const int lut_n = (a.nn_lut && !canvas && !fixed && a.lut && a.nn_probe == 0 &&
                     (mask || (a.nn_shape == 3 && a.nn_rpw <= 4))) ? clamp_lut_size<T>(a) : 0;
  if (lut_n > 0)
    hipLaunchKernelGGL(clamp_lut_kernel<T>, dim3((lut_n + 255) / 256), dim3(256), 0, s, a, (uint8_t *)a.lut, lut_n);
  if (mask && a.nn_stride && a.nn_shape == 5 && !canvas) {   // default: masked 4 x 1 at 8 waves per SIMD
    GSKY_NN_LAUNCH(true, 4, 1, kStrided | kWaves8);
  } else if (mask && a.nn_stride) {
    if (canvas) GSKY_NN_LAUNCH(true, 4, 2, kCanvas | kStrided);
    else if (lut_n > 0) GSKY_NN_LAUNCH(true, 4, 2, kClampLut | kStrided);
    else GSKY_NN_LAUNCH(true, 4, 2, kStrided);
  } else if (mask) {
    if (canvas) GSKY_NN_LAUNCH(true, 4, 2, kCanvas);
    else if (lut_n > 0) GSKY_NN_LAUNCH(true, 4, 2, kClampLut);
    else GSKY_NN_LAUNCH(true, 4, 2, 0);
  } else if (fixed) {
    if (canvas) GSKY_NN_LAUNCH(false, 4, 4, kCanvas | kFixed); else GSKY_NN_LAUNCH(false, 4, 4, kFixed);
  } else if (a.nn_shape == 1 && a.nn_stride) {
    if (canvas) GSKY_NN_LAUNCH(false, 8, 1, kCanvas | kStrided); else GSKY_NN_LAUNCH(false, 8, 1, kStrided);
  } else if (a.nn_shape == 1) {
    if (canvas) GSKY_NN_LAUNCH(false, 8, 1, kCanvas); else GSKY_NN_LAUNCH(false, 8, 1, 0);
  } else if (a.nn_shape == 2 && a.nn_stride) {
    if (canvas) GSKY_NN_LAUNCH(false, 8, 2, kCanvas | kStrided); else GSKY_NN_LAUNCH(false, 8, 2, kStrided);
  } else if (a.nn_shape == 2) {
    if (canvas) GSKY_NN_LAUNCH(false, 8, 2, kCanvas); else GSKY_NN_LAUNCH(false, 8, 2, 0);
  } else if (a.nn_shape == 3 && a.nn_rpw > 4) {   // A/B: 8 or 16 rows per wave, fewer and longer waves
    const int rows_blk = 4 * (a.nn_rpw >= 16 ? 16 : 8);
    const int items = a.n_tiles * ((a.max_h + rows_blk - 1) / rows_blk) * ((a.max_w + kBandCols - 1) / kBandCols);
    const dim3 g2((unsigned)items);
    if (a.nn_stride && !canvas) {
      if (a.nn_rpw >= 16)
        hipLaunchKernelGGL((render_nn_kernel<T, false, 4, 2, kStrided, 16>), g2, dim3(256), 0, s, a, a.entries,
                           a.order, a.rows, a.pool, a.tplans, a.tiles, items, 0);
      else
        hipLaunchKernelGGL((render_nn_kernel<T, false, 4, 2, kStrided, 8>), g2, dim3(256), 0, s, a, a.entries,
                           a.order, a.rows, a.pool, a.tplans, a.tiles, items, 0);
    } else if (a.nn_rpw >= 16) {
      if (canvas) hipLaunchKernelGGL((render_nn_kernel<T, false, 4, 2, kCanvas, 16>), g2, dim3(256), 0, s, a,
                                     a.entries, a.order, a.rows, a.pool, a.tplans, a.tiles, items, 0);
      else hipLaunchKernelGGL((render_nn_kernel<T, false, 4, 2, 0, 16>), g2, dim3(256), 0, s, a, a.entries, a.order,
                              a.rows, a.pool, a.tplans, a.tiles, items, 0);
    } else {
      if (canvas) hipLaunchKernelGGL((render_nn_kernel<T, false, 4, 2, kCanvas, 8>), g2, dim3(256), 0, s, a,
                                     a.entries, a.order, a.rows, a.pool, a.tplans, a.tiles, items, 0);
      else hipLaunchKernelGGL((render_nn_kernel<T, false, 4, 2, 0, 8>), g2, dim3(256), 0, s, a, a.entries, a.order,
                              a.rows, a.pool, a.tplans, a.tiles, items, 0);
    }
  } else if (a.nn_shape == 3 && a.nn_stride == 2 && !canvas) {   // A/B: cached stores
    GSKY_NN_LAUNCH(false, 4, 2, kStrided | kPlainStore);
  } else if (a.nn_shape == 3 && a.nn_stride == 4 && !canvas) {   // A/B: rows through LDS, stores at the end
    GSKY_NN_LAUNCH(false, 4, 2, kStrided | kLdsOut);
  } else if (a.nn_shape == 3 && a.nn_stride == 5 && !canvas) {   // A/B: 8 waves per SIMD
    GSKY_NN_LAUNCH(false, 4, 2, kStrided | kWaves8);
  } else if ((a.nn_shape == 4 || a.nn_shape == 5) && a.nn_stride) {   // default: 4 x 1 strided, 8 waves / SIMD
    if (canvas) GSKY_NN_LAUNCH(false, 4, 2, kCanvas | kStrided);
    else GSKY_NN_LAUNCH(false, 4, 1, kStrided | kWaves8);
  } else if (a.nn_shape == 0 && a.nn_stride) {
    if (canvas) GSKY_NN_LAUNCH(false, 4, 4, kCanvas | kStrided); else GSKY_NN_LAUNCH(false, 4, 4, kStrided);
  } else if (a.nn_shape == 3 && a.nn_stride) {
    if (canvas) GSKY_NN_LAUNCH(false, 4, 2, kCanvas | kStrided);
    else if (lut_n > 0) GSKY_NN_LAUNCH(false, 4, 2, kClampLut | kStrided);
    else GSKY_NN_LAUNCH(false, 4, 2, kStrided);
  } else if (a.nn_shape == 3) {
    if (canvas) GSKY_NN_LAUNCH(false, 4, 2, kCanvas);
    else if (lut_n > 0) GSKY_NN_LAUNCH(false, 4, 2, kClampLut);
    else GSKY_NN_LAUNCH(false, 4, 2, 0);
  } else {
    if (canvas) GSKY_NN_LAUNCH(false, 4, 4, kCanvas); else GSKY_NN_LAUNCH(false, 4, 4, 0);
  }
#undef GSKY_NN_LAUNCH
}

// Band kernel of one call: the NN kernel above (RenderArgs.nn_kernel, the
// default) or render_lds_kernel (bilinear, LDS staging, A/B variants).
template <int LPX, int R, int S, int W8>
__global__ void render_bil_kernel(RenderArgs a, const EntryD *__restrict__ ents, const int32_t *__restrict__ order,
                                  const RowRec *__restrict__ rows, const Leaf *__restrict__ pool,
                                  const TilePlan *__restrict__ tplans, const gskyhip_tile *__restrict__ tiles,
                                  int n_items);
void launch_bil(const RenderArgs &a, int n_items, hipStream_t s);   // render_bil.h, render_lds_f32.hip

template <typename T>
void launch_band_t(const RenderArgs &a, bool mask, int n_items, hipStream_t s) {
  if constexpr (std::is_same<T, float>::value) {   // bilinear float canvases (C3): render_bil_kernel
    if (a.bil_kernel && !mask && (a.lds_mode & kBilinear) && (a.lds_mode & kCanvas) && !a.lds_stage) {
      launch_bil(a, n_items, s);
      return;
    }
  }
  if (a.nn_kernel && !(a.lds_mode & kBilinear) && !a.lds_stage)
    launch_nn_t<T>(a, mask, n_items, s);
  else
    launch_lds_t<T>(a, mask, n_items, s);
}

}  // namespace gsky
