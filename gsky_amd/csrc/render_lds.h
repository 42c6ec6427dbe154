// render_lds.h -- shared pieces of the typed band kernels and the general
// bilinear band kernel.
//
// The typed band kernels serve the common GetMap / GetCoverage case: every
// stack entry of the tile shares value type T, every row LINEAR or
// POOL(linear leaves), one rendered namespace.  A 256-thread block owns a band
// of kBandRows tile rows and a kBandCols-column block.  Nearest neighbour goes
// to render_nn_kernel (render_nn.h), bilinear float canvases to
// render_bil_kernel (render_bil.h); what is left -- bilinear RGBA tiles,
// bilinear integer canvases and bilinear stacks with a mask layer -- runs
// render_lds_kernel below: wave w folds rows w, w+4, w+8, w+12 of the band,
// each lane 8 consecutive pixels, over the band's entries listed in LDS
// (kBandEnt per pass; a band with more parks its partial canvas in its own
// output slot between passes).
//
// Instantiated once per value type in render_lds_<type>.hip (separate
// translation units build in parallel); launched by launch_render
// (render.hip) when the batch has one value type, one namespace and no
// auto-scale.
#pragma once
#include "render_common.h"

namespace gsky {

constexpr int kBandRows = kLdsBandRows;
constexpr int kBandEnt = 16;            // entries per pass over the band (render_lds_kernel)
constexpr int kLanePx = 8;              // pixels per lane per row
constexpr int kBandCols = 64 * kLanePx;  // columns per block

struct BandEnt {
  const void *band;
  int32_t band_x, band_y;
  int32_t xoff, yoff, w, h;
  int32_t fill_mode, mask_pair;
  Val nd, fillv;                        // merge nodata / window fill, as Val bits
  int32_t pair;
  int32_t has_nodata, out_dtype;        // bilinear: nodata taps are dropped (GWKBilinearResample4Sample)
  double nodata64;
};

template <typename T> __host__ __device__ constexpr int vt_code();
template <> __host__ __device__ constexpr int vt_code<uint8_t>() { return GSKYHIP_BYTE; }
template <> __host__ __device__ constexpr int vt_code<int8_t>() { return GSKYHIP_SIGNEDBYTE; }
template <> __host__ __device__ constexpr int vt_code<int16_t>() { return GSKYHIP_INT16; }
template <> __host__ __device__ constexpr int vt_code<uint16_t>() { return GSKYHIP_UINT16; }
template <> __host__ __device__ constexpr int vt_code<float>() { return GSKYHIP_FLOAT32; }

__device__ __forceinline__ const void *uniform_ptr(const void *p) {
  const uint64_t v = (uint64_t)p;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
  return (const void *)(((uint64_t)hi << 32) | lo);
}

// One raw buffer load of a T (range-checked: out of range reads 0, no fetch).
template <typename T>
__device__ __forceinline__ typename VOf<T>::type buf_load(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  using V = typename VOf<T>::type;
  if constexpr (sizeof(T) == 1) {
    const uint8_t b = __builtin_amdgcn_raw_buffer_load_b8(r, off, 0, 0);
    return std::is_signed<T>::value ? (V)(int8_t)b : (V)b;
  } else if constexpr (sizeof(T) == 2) {
    const uint16_t h = __builtin_amdgcn_raw_buffer_load_b16(r, off, 0, 0);
    return std::is_signed<T>::value ? (V)(int16_t)h : (V)h;
  } else {
    const uint32_t w = __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0);
    return __builtin_bit_cast(V, w);
  }
}

// buf_load of a 1- or 2-byte T through the aligned dword that holds it (the
// buffer's num_records rounded up to 4: a dword never straddles a page, so
// the read past the band's last byte stays inside its page).  A gather of
// dwords retires faster than one of 16-bit halves where lanes share a dword
// (tools/calib/gather_rate.hip: 8.3 vs 13.4 CU cycles per instruction with
// C2's 2x upsampling); the value is the same.
template <typename T>
__device__ __forceinline__ typename VOf<T>::type buf_load_w(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  using V = typename VOf<T>::type;
  if constexpr (sizeof(T) >= 4) {
    return buf_load<T>(r, off);
  } else {
    const uint32_t w = __builtin_amdgcn_raw_buffer_load_b32(r, off & ~3u, 0, 0) >> ((off & 3u) * 8u);
    if constexpr (sizeof(T) == 1) return std::is_signed<T>::value ? (V)(int8_t)w : (V)(uint8_t)w;
    else return std::is_signed<T>::value ? (V)(int16_t)w : (V)(uint16_t)w;
  }
}

// GWKBilinearResample4Sample semantics of bil_fetch() (render_common.h), the
// same fp64 expressions, for the band kernel: false -> window fill.
template <typename T>
__device__ __forceinline__ bool bil_sample(const T *band, int bx, int by, bool has_nodata, double nodata64,
                                           int out_dtype, double sx, double sy, typename VOf<T>::type &v) {
  int iSrcX = (int)floor(sx - 0.5);
  int iSrcY = (int)floor(sy - 0.5);
  double rX = 1.5 - (sx - iSrcX);
  double rY = 1.5 - (sy - iSrcY);
  if (iSrcX == -1) { iSrcX = 0; rX = 1; }
  if (iSrcY == -1) { iSrcY = 0; rY = 1; }
  double accR = 0.0, accDiv = 0.0;
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const int xx = iSrcX + (k & 1), yy = iSrcY + (k >> 1);
    const double w = ((k & 1) ? (1.0 - rX) : rX) * ((k >> 1) ? (1.0 - rY) : rY);
    if (xx < 0 || xx >= bx || yy < 0 || yy >= by) continue;
    const double d = (double)((const GPTR(T))band)[(int64_t)yy * bx + xx];
    if (has_nodata && (d == nodata64 || (nodata64 != nodata64 && d != d))) continue;
    accDiv += w;
    accR += d * w;
  }
  double r;
  if (accDiv == 1.0) r = accR;
  else if (accDiv < 0.00001) return false;
  else r = accR / accDiv;
  if constexpr (std::is_same<T, float>::value) v = (float)r;
  else v = gdal_copy_to(floor(r + 0.5), out_dtype).i;
  return true;
}

// Bilinear band kernel (FLAGS: kBilinear, plus kCanvas for typed canvas output).
template <typename T, bool MASK, int FLAGS>
__global__ __launch_bounds__(256) void render_lds_kernel(RenderArgs a, const EntryD *__restrict__ ents,
                                                         const int32_t *__restrict__ order,
                                                         const RowRec *__restrict__ rows,
                                                         const Leaf *__restrict__ pool,
                                                         const TilePlan *__restrict__ tplans,
                                                         const gskyhip_tile *__restrict__ tiles, int n_items) {
  static_assert((FLAGS & kBilinear) != 0, "render_lds_kernel is the bilinear band kernel");
  using V = typename VOf<T>::type;
  __shared__ uint32_t s_ramp[256];
  __shared__ BandEnt s_ent[kBandEnt];
  __shared__ int32_t s_n, s_next;

  // item = (tile, 16-row band, 512-column block); column blocks innermost
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
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  if (a.ramp) s_ramp[tid] = a.ramp[tid];

  const int ns_out = a.out_ns[0];
  const bool created = tp.created[ns_out] != 0;
  const V cnod = as_v<T>(go_conv_to(tp.nodata[ns_out], tp.dtype[ns_out]));
  const int32_t *ord = order + tile.pair_begin;
  const int n_entries = tp.n_entries;
  const int x0 = xb + lane * kLanePx;
  const ScaleK sk = make_scale(tp.dtype[ns_out], tp.nodata[ns_out], a.sp, false, 0.f, 0.f);
  const bool has_ramp = a.ramp != nullptr;
  uint8_t *rgba_tile = a.rgba + (int64_t)t * a.max_h * a.max_w * 4;

  int e0 = 0;
  do {
    __syncthreads();   // previous pass done with the LDS tables
    if (wave == 0) {   // 64 entries examined at once, hits compacted by ballot
      const int k = e0 + lane;
      bool hit = false;
      int p = -1;
      if (k < n_entries) {
        p = ord[k];
        const EntryD &e = ents[p];
        hit = e.ns == ns_out && e.w > 0 && e.yoff < band0 + kBandRows && e.yoff + e.h > band0 &&
              e.xoff < xb + kBandCols && e.xoff + e.w > xb;
      }
      const unsigned long long m = __ballot(hit);
      const int pos = __popcll(m & ((1ull << lane) - 1ull));
      if (hit && pos < kBandEnt) {
        const EntryD &e = ents[p];
        BandEnt &b = s_ent[pos];
        b.band = e.band; b.band_x = e.band_x; b.band_y = e.band_y;
        b.xoff = e.xoff; b.yoff = e.yoff; b.w = e.w; b.h = e.h;
        b.fill_mode = e.fill_mode; b.mask_pair = e.mask_pair;
        b.nd = e.nd; b.fillv = e.fill;
        b.has_nodata = e.has_nodata; b.out_dtype = e.out_dtype; b.nodata64 = e.nodata64;
        b.pair = p;
      }
      if (lane == 0) {
        const int cnt = __popcll(m);
        int nxt = e0 + 64;
        if (cnt > kBandEnt) {   // resume at the first hit that did not fit
          unsigned long long mm = m;
          for (int i = 0; i < kBandEnt; i++) mm &= mm - 1ull;
          nxt = e0 + __ffsll(mm) - 1;
        }
        s_n = cnt < kBandEnt ? cnt : kBandEnt;
        s_next = nxt < n_entries ? nxt : n_entries;
      }
    }
    __syncthreads();
    const int nb = s_n;
    const int next_e0 = s_next;

    // fold: wave owns rows wave, wave+4, wave+8, wave+12 of the band
    const bool first = e0 == 0, last = next_e0 >= n_entries;
#pragma unroll 1
    for (int j = 0; j < 4; j++) {
      const int rr = wave + 4 * j;
      const int r = band0 + rr;
      if (r >= H || x0 >= W) break;
      uint8_t *dst = rgba_tile + ((int64_t)r * a.max_w + x0) * 4;
      T *cdst = nullptr;   // canvas mode: the typed canvas row of this lane
      if constexpr ((FLAGS & kCanvas) != 0) {
        const int64_t e = a.cov_offsets ? a.cov_offsets[t] + (int64_t)r * a.cov_stride + x0
                                        : (int64_t)r * a.max_w + x0;
        cdst = (T *)(a.cov_offsets ? a.canvas : a.canvas + t * a.canvas_tile_stride) + e;
      }
      V c[kLanePx];
      if (first) {
#pragma unroll
        for (int q = 0; q < kLanePx; q++) c[q] = cnod;
      } else if constexpr ((FLAGS & kCanvas) != 0) {
#pragma unroll
        for (int q = 0; q < kLanePx; q++) c[q] = (x0 + q < W) ? (V)cdst[q] : cnod;
      } else {
#pragma unroll
        for (int q = 0; q < kLanePx; q++) c[q] = (x0 + q < W) ? ((const V *)dst)[q] : cnod;
      }
      for (int k = 0; k < nb; k++) {
        const BandEnt &b = s_ent[k];
        const int yoff = __builtin_amdgcn_readfirstlane(b.yoff);
        const int eh = __builtin_amdgcn_readfirstlane(b.h);
        const int ir = r - yoff;
        if (ir < 0 || ir >= eh) continue;
        const int pair = __builtin_amdgcn_readfirstlane(b.pair);
        const int ew = __builtin_amdgcn_readfirstlane(b.w);
        const int bx = __builtin_amdgcn_readfirstlane(b.band_x);
        const int by = __builtin_amdgcn_readfirstlane(b.band_y);
        const T *bandp = (const T *)uniform_ptr(b.band);
        const V nd = as_v<T>(b.nd), fillv = as_v<T>(b.fillv);
        const int fill_mode = __builtin_amdgcn_readfirstlane(b.fill_mode);
        const int ic0 = x0 - __builtin_amdgcn_readfirstlane(b.xoff);
        const RowRec &R = rows[(int64_t)pair * a.max_h + ir];   // wave-uniform: scalar loads
        const double xs0 = R.v[0], ys0 = R.v[1], dX = R.v[2], dY = R.v[3];
        const int kind = __builtin_amdgcn_readfirstlane(R.kind);
        const bool hnd = b.has_nodata != 0;
        const double nd64 = b.nodata64;
        const int odt = b.out_dtype;
#pragma unroll
        for (int q = 0; q < kLanePx; q++) {
          const int ic = ic0 + q;
          const bool in = (unsigned)ic < (unsigned)ew && x0 + q < W;
          double sx, sy;
          bool okc = true;
          if (kind == ROW_LINEAR) {
            const double dist = (double)ic0 + (double)q;
            sy = ys0 + dY * dist;
            sx = xs0 + dX * dist;
          } else {   // POOL: linear leaves, per-pixel exact points, failed pixels
            okc = lin_coords(R, pool, in ? ic : 0, sx, sy);
          }
          V v = fillv, got;
          if (in && okc && bil_sample<T>(bandp, bx, by, hnd, nd64, odt, sx, sy, got)) v = got;
          bool take = in && (v != nd);
          if (MASK && b.mask_pair >= 0) {
            if (take) take = !mask_fast<GSKYHIP_RESAMPLE_BILINEAR>(ents, rows, pool, a.mask, ents[pair], ic, ir);
          }
          const bool t2 = take && (!fill_mode || c[q] == nd);
          c[q] = t2 ? v : c[q];
        }
      }
      if constexpr ((FLAGS & kCanvas) != 0) {   // typed canvas (tile_merger.go:562-652): T stores
#pragma unroll
        for (int q = 0; q < kLanePx; q++)
          if (x0 + q < W) cdst[q] = (T)c[q];
        continue;
      }
      if (!last) {   // partial canvas parked in the slot (raw values), re-read next pass
#pragma unroll
        for (int q = 0; q < kLanePx; q++)
          if (x0 + q < W) ((V *)dst)[q] = c[q];
        continue;
      }
      // utils.Scale + palette / grey
      uint32_t pxo[kLanePx];
#pragma unroll
      for (int q = 0; q < kLanePx; q++) {
        const uint32_t bb = scale_t<T>(sk, c[q]);
        const uint32_t col = has_ramp ? s_ramp[bb & 0xFFu] : (0xFF000000u | (bb << 16) | (bb << 8) | bb);
        pxo[q] = (created && bb != 0xFFu) ? col : 0u;
      }
      if (x0 + kLanePx <= W && ((((uintptr_t)dst) & 15) == 0)) {
        u32x4 v0 = {pxo[0], pxo[1], pxo[2], pxo[3]};
        u32x4 v1 = {pxo[4], pxo[5], pxo[6], pxo[7]};
        __builtin_nontemporal_store(v0, (GPTR(u32x4))dst);
        __builtin_nontemporal_store(v1, (GPTR(u32x4))(dst + 16));
      } else {
#pragma unroll
        for (int q = 0; q < kLanePx; q++)
          if (x0 + q < W) ((uint32_t *)dst)[q] = pxo[q];
      }
    }
    e0 = next_e0;
  } while (e0 < n_entries);
}

template <typename T>
void launch_lds_t(const RenderArgs &a, bool mask, int n_items, hipStream_t s) {
#define GSKY_LDS_LAUNCH(M, F)                                                                                  \
  hipLaunchKernelGGL((render_lds_kernel<T, M, F>), dim3((unsigned)n_items), dim3(256), 0, s, a, a.entries, \
                     a.order, a.rows, a.pool, a.tplans, a.tiles, n_items)
  const bool canvas = (a.lds_mode & kCanvas) != 0;
  if (mask) {
    if (canvas) GSKY_LDS_LAUNCH(true, kBilinear | kCanvas); else GSKY_LDS_LAUNCH(true, kBilinear);
  } else {
    if (canvas) GSKY_LDS_LAUNCH(false, kBilinear | kCanvas); else GSKY_LDS_LAUNCH(false, kBilinear);
  }
#undef GSKY_LDS_LAUNCH
}

void launch_band_i16(const RenderArgs &a, bool mask, int n_items, hipStream_t s);
void launch_band_u16(const RenderArgs &a, bool mask, int n_items, hipStream_t s);
void launch_band_f32(const RenderArgs &a, bool mask, int n_items, hipStream_t s);
void launch_band_i8(const RenderArgs &a, bool mask, int n_items, hipStream_t s);
void launch_band_u8(const RenderArgs &a, bool mask, int n_items, hipStream_t s);

}  // namespace gsky
