// render_nn_stage.h -- the nearest-neighbour band kernel with the source
// staged in LDS (large RGBA GetMap batches, BASELINE C2).
//
// Same work and the same expressions as render_nn_kernel (render_nn.h):
// per output pixel the fp64 source coordinate of the row record (the GDAL
// approximate transformer, warp.go:269), the truncation of warp.go:271-300,
// the ordered nodata fold of MergeMaskedRaster (tile_merger.go:38-225),
// utils.Scale and the palette of EncodePNG -- but the source pixels come from
// LDS instead of one 2-byte gather per pixel:
//   * block = 64 tile rows x 256 columns (4 waves x 16 rows; a lane the 4
//     pixels lane, lane + 64, lane + 128, lane + 192 of a row), a footprint
//     close to square in the source (~32 x 125 source pixels for C2's 2x
//     upsampling) so its bounding box stays small under rotation;
//   * set-up: wave k takes entry k, lane l block row l: from the row records
//     the first and last source pixel of the row's window columns (the
//     truncations are monotone in the column, render_common linear_row_inside)
//     -> the entry's source bounding box; an entry whose block rows are all
//     LINEAR and `inside` and whose box fits the remaining LDS budget is
//     staged: its box rows copied HBM -> LDS by all 256 threads with 4-byte
//     loads (each instruction 256 contiguous bytes);
//   * then every row folds its entries in ProcessRasterStack order, staged
//     entries from LDS (ds_read of the pixel's source value), the others by
//     the gather path of render_nn_kernel (nn_entry_row).
// Per block this replaces 64 x 4 gather instructions by ~12 coalesced loads;
// the gathers' per-instruction address processing, not HBM bytes, bounded
// render_nn_kernel.
#pragma once
#include "render_nn.h"

namespace gsky {

constexpr int kStCols = 256;              // columns per block
constexpr int kStRowsW = 16;              // rows per wave
constexpr int kStRowsBlk = 4 * kStRowsW;  // rows per block
constexpr int kStPx = 4;                  // pixels per lane per row, 64 columns apart
constexpr int kStBytes = 16384;           // staging LDS per block (8 blocks per CU with the table)
constexpr int kStMaxEnt = 8;              // entries a block can stage
constexpr int kStLoads = 16;              // staging loads in flight per thread per entry

struct StageEnt {
  int32_t ixmin, ixmax, iymin, iymax;   // source box of the entry's block pixels
  int32_t bad, any;                     // a block row not LINEAR+inside / some block pixel in the window
  int32_t staged, base;                 // staged: LDS byte of source pixel (0, 0) is base (may be < 0)
  int32_t pitch, x0b, nrows, lds_off;   // box: bytes per LDS row, first byte in a source row, rows, LDS byte
};

template <typename T>
__device__ __forceinline__ typename VOf<T>::type lds_val(const uint8_t *s, int byte) {
  using V = typename VOf<T>::type;
  const T v = *(const T *)(s + byte);
  if constexpr (std::is_same<T, float>::value) return v;
  else return (V)v;
}

template <typename T>
__global__ __launch_bounds__(256, 8) void render_nn_stage_kernel(RenderArgs a, const EntryD *__restrict__ ents,
                                                                 const int32_t *__restrict__ order,
                                                                 const RowRec *__restrict__ rows,
                                                                 const Leaf *__restrict__ pool,
                                                                 const TilePlan *__restrict__ tplans,
                                                                 const gskyhip_tile *__restrict__ tiles,
                                                                 int n_items) {
  using V = typename VOf<T>::type;
  __shared__ uint32_t s_tab[256];
  __shared__ __attribute__((aligned(16))) uint8_t s_src[kStBytes];
  __shared__ StageEnt s_ent[kStMaxEnt];

  const int item = blockIdx.x;
  if (item >= n_items) return;
  const int bands_per_tile = (a.max_h + kStRowsBlk - 1) / kStRowsBlk;
  const int col_blocks = (a.max_w + kStCols - 1) / kStCols;
  const int t = item / (bands_per_tile * col_blocks);
  const int in_tile = item - t * bands_per_tile * col_blocks;
  const TilePlan &tp = tplans[t];
  if (tp.complex || (tp.n_entries > 0 && tp.vt != vt_code<T>())) return;   // empty tiles: written elsewhere
  const gskyhip_tile &tile = tiles[t];
  const int W = tile.width, H = tile.height;
  const int band0 = (in_tile / col_blocks) * kStRowsBlk;
  const int xb = (in_tile % col_blocks) * kStCols;
  if (band0 >= H || xb >= W) return;
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const int ns_out = a.out_ns[0];
  const bool created = tp.created[ns_out] != 0;
  {
    const uint32_t col = a.ramp ? a.ramp[tid] : (0xFF000000u | ((uint32_t)tid * 0x10101u));
    s_tab[tid] = (created && tid != 255) ? col : 0u;
  }
  const int32_t *ord = order + tile.pair_begin;
  const int n_entries = tp.n_entries;
  const int n_st = min(n_entries, kStMaxEnt);
  const int ncols = min(kStCols, W - xb);

  // ---- set-up: the source box of each entry over the block's pixels
  for (int k = wave; k < n_st; k += 4) {
    const EntryD &e = ents[ord[k]];
    const int eyoff = e.yoff, eh = e.h, exoff = e.xoff, ew = e.w;
    const int lim = max(0, min(ew, W - exoff));
    const int c0 = exoff - xb, c1 = exoff + lim - xb;
    const bool rel = e.ns == ns_out && ew > 0 && c1 > 0 && c0 < ncols;
    const int r = band0 + lane, ir = r - eyoff;
    const bool has = rel && r < H && ir >= 0 && ir < eh;
    int ixa = 0x7FFFFFFF, ixb = -1, iya = 0x7FFFFFFF, iyb = -1, bad = 0;
    if (has) {
      const RowRec &rr = rows[e.row_base + ir];
      if (rr.kind != ROW_LINEAR || !rr.inside) {
        bad = 1;
      } else {
        const double xs0 = rr.v[0], ys0 = rr.v[1], dX = rr.v[2], dY = rr.v[3];
        const double da = (double)(xb + max(c0, 0) - exoff), db = (double)(xb + min(c1, ncols) - 1 - exoff);
        const int x1 = __double2int_rz(xs0 + dX * da + 1.0e-10), y1 = __double2int_rz(ys0 + dY * da + 1.0e-10);
        const int x2 = __double2int_rz(xs0 + dX * db + 1.0e-10), y2 = __double2int_rz(ys0 + dY * db + 1.0e-10);
        ixa = min(x1, x2); ixb = max(x1, x2); iya = min(y1, y2); iyb = max(y1, y2);
      }
    }
    int any = has ? 1 : 0;
#pragma unroll
    for (int sh = 32; sh > 0; sh >>= 1) {
      ixa = min(ixa, __shfl_xor(ixa, sh)); ixb = max(ixb, __shfl_xor(ixb, sh));
      iya = min(iya, __shfl_xor(iya, sh)); iyb = max(iyb, __shfl_xor(iyb, sh));
      bad |= __shfl_xor(bad, sh); any |= __shfl_xor(any, sh);
    }
    if (lane == 0) {
      StageEnt &S = s_ent[k];
      S.ixmin = ixa; S.ixmax = ixb; S.iymin = iya; S.iymax = iyb; S.bad = bad; S.any = any;
    }
  }
  __syncthreads();
  if (tid == 0) {   // LDS budget, in stack order
    int off = 0;
    for (int k = 0; k < n_st; k++) {
      StageEnt &S = s_ent[k];
      S.staged = 0;
      if (!S.any || S.bad) continue;
      const EntryD &e = ents[ord[k]];
      if (((int64_t)e.band_x * (int64_t)sizeof(T)) % 4 != 0) continue;   // rows must start on 4-byte boundaries
      const int x0b = (S.ixmin * (int)sizeof(T)) & ~3;
      const int pitch = (((S.ixmax + 1) * (int)sizeof(T) - x0b) + 3) & ~3;
      const int nrows = S.iymax - S.iymin + 1;
      if (pitch > 1024 || off + pitch * nrows > kStBytes) continue;
      S.staged = 1; S.x0b = x0b; S.pitch = pitch; S.nrows = nrows; S.lds_off = off;
      S.base = off - S.iymin * pitch - x0b;
      off += pitch * nrows;
    }
  }
  __syncthreads();
  // ---- staging: box rows HBM -> LDS, 4-byte loads, kStLoads in flight per thread
  for (int k = 0; k < n_st; k++) {
    if (!s_ent[k].staged) continue;
    const EntryD &e = ents[ord[k]];
    const int pitch = s_ent[k].pitch, nrows = s_ent[k].nrows, x0b = s_ent[k].x0b, iy0 = s_ent[k].iymin;
    const int lds_off = s_ent[k].lds_off;
    const int nw = pitch >> 2;                    // words per box row (<= 256)
    const int per = 256 / nw;                     // box rows per pass
    const int rr0 = tid / nw, cc = tid - rr0 * nw;
    const uint32_t rowb = (uint32_t)e.band_x * (uint32_t)sizeof(T);
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        (void *)uniform_ptr(e.band), (short)0, (int)((int64_t)e.band_x * e.band_y * (int64_t)sizeof(T)), 0x00020000);
    if (rr0 < per) {
      for (int rb = rr0; rb < nrows; rb += per * kStLoads) {
        uint32_t w[kStLoads];
#pragma unroll
        for (int u = 0; u < kStLoads; u++) {
          const int rr = rb + u * per;
          // rows past the box read from its first row (a valid address), stored nowhere
          const uint32_t src = (uint32_t)(iy0 + (rr < nrows ? rr : 0)) * rowb + (uint32_t)x0b + 4u * cc;
          w[u] = __builtin_amdgcn_raw_buffer_load_b32(rs, src, 0, 0);
        }
#pragma unroll
        for (int u = 0; u < kStLoads; u++) {
          const int rr = rb + u * per;
          if (rr < nrows) *(uint32_t *)(s_src + lds_off + rr * pitch + 4 * cc) = w[u];
        }
      }
    }
  }
  __syncthreads();

  // ---- rows: the ordered fold, Scale, palette, RGBA stores
  const int r0 = band0 + wave * kStRowsW;
  if (r0 >= H) return;
  const V cnod = as_v<T>(go_conv_to(tp.nodata[ns_out], tp.dtype[ns_out]));
  const ScaleK sk = make_scale(tp.dtype[ns_out], tp.nodata[ns_out], a.sp, false, 0.f, 0.f);
  const bool safe = !std::is_same<T, float>::value && (float)max(sk.clp.i, 0) * sk.sc < 2147483648.0f;
  const bool full = ncols == kStCols;
  const int xl = xb + lane;
  uint32_t *rgba_lane = (uint32_t *)(a.rgba + (((int64_t)t * a.max_h) * a.max_w + xl) * 4);
#pragma unroll 1
  for (int j = 0; j < kStRowsW; j++) {
    const int r = r0 + j;
    if (r >= H) break;
    V c[kStPx];
#pragma unroll
    for (int q = 0; q < kStPx; q++) c[q] = cnod;
#pragma unroll 1
    for (int k = 0; k < n_entries; k++) {
      const EntryD &e = ents[ord[k]];
      if (k >= n_st || !s_ent[k].staged) {
        nn_entry_row<T, false, kStPx>(a, ents, e, rows, a.rowfix, pool, ns_out, r, xb, xl, W, ncols, c);
        continue;
      }
      const int eyoff = e.yoff, eh = e.h, exoff = e.xoff, ew = e.w;
      if (e.ns != ns_out || ew <= 0) continue;
      const int ir = r - eyoff;
      if (ir < 0 || ir >= eh) continue;
      const int lim = max(0, min(ew, W - exoff));
      const int c0 = exoff - xb, c1 = exoff + lim - xb;
      if (c1 <= 0 || c0 >= ncols) continue;
      const RowRec *rr = rows + e.row_base + ir;   // LINEAR and inside (set-up)
      const double xs0 = rr->v[0], ys0 = rr->v[1], dX = rr->v[2], dY = rr->v[3];
      const int base = s_ent[k].base, pitch = s_ent[k].pitch;
      const V nd = as_v<T>(e.nd);
      const bool fill_mode = e.fill_mode != 0;
      const int ic0 = xl - exoff;
      V vv[kStPx];
#pragma unroll
      for (int q = 0; q < kStPx; q++) {
        const int ic = ic0 + 64 * q;
        const double dist = (double)ic;
        const int ix = __double2int_rz(xs0 + dX * dist + 1.0e-10);
        const int iy = __double2int_rz(ys0 + dY * dist + 1.0e-10);
        const bool in = (unsigned)ic < (unsigned)lim;
        vv[q] = lds_val<T>(s_src, in ? base + iy * pitch + ix * (int)sizeof(T) : 0);
      }
      if (c0 <= 0 && c1 >= ncols) {   // the window covers the block's columns
        if (!fill_mode) {
#pragma unroll
          for (int q = 0; q < kStPx; q++) c[q] = (vv[q] != nd) ? vv[q] : c[q];
        } else {
#pragma unroll
          for (int q = 0; q < kStPx; q++) c[q] = (c[q] == nd) ? vv[q] : c[q];
        }
      } else {
#pragma unroll
        for (int q = 0; q < kStPx; q++) {
          const bool in = (unsigned)(ic0 + 64 * q) < (unsigned)lim;
          const bool take = in && (vv[q] != nd) && (!fill_mode || c[q] == nd);
          c[q] = take ? vv[q] : c[q];
        }
      }
    }
    uint32_t px[kStPx];
    nn_rgba<T, kStPx>(sk, safe, s_tab, c, px);
    uint32_t *dst = rgba_lane + (int64_t)r * a.max_w;
    if (full) {
#pragma unroll
      for (int q = 0; q < kStPx; q++) __builtin_nontemporal_store(px[q], (GPTR(uint32_t))(dst + 64 * q));
    } else {
#pragma unroll
      for (int q = 0; q < kStPx; q++)
        if (64 * q + lane < ncols) __builtin_nontemporal_store(px[q], (GPTR(uint32_t))(dst + 64 * q));
    }
  }
}

template <typename T>
void launch_nn_stage(const RenderArgs &a, hipStream_t s) {
  const int items = a.n_tiles * ((a.max_h + kStRowsBlk - 1) / kStRowsBlk) * ((a.max_w + kStCols - 1) / kStCols);
  hipLaunchKernelGGL((render_nn_stage_kernel<T>), dim3((unsigned)items), dim3(256), 0, s, a, a.entries, a.order,
                     a.rows, a.pool, a.tplans, a.tiles, items);
}

}  // namespace gsky
