// render_lds.h -- the typed band kernel of the batched GetMap path.
//
// The common GetMap case -- every stack entry of the tile shares value type T,
// nearest neighbour, every row LINEAR or POOL(linear leaves), one rendered
// namespace, RGBA out -- runs as one lean kernel per T (no value-type switch,
// no SGPR spills).  A 256-thread block owns a band of kBandRows tile rows (all
// columns); wave w folds rows w, w+4, w+8, w+12, each lane 8 consecutive
// pixels (two 16-B RGBA stores).  Items go to blocks in linear order: all
// XCDs then work on neighbouring tiles and share source rows through the
// MALL, measured faster than XCD-contiguous runs (profiles/r02g_ab_*.jsonl).
//
// STAGE = true additionally stages, per band, in LDS:
//   * the row records of the band's entries,
//   * each entry's SOURCE WINDOW under the band: the exact extremes of the
//     truncated source column / row over every row (the fp64 coordinate is
//     monotone along a linear leaf, so they sit at the leaf end points) give
//     a rectangle that is loaded once with dword loads all issued before the
//     first wait; the per-pixel gathers then read LDS.
// STAGE = false gathers straight from HBM with scalar row-record loads.
// Both are bit-identical to lin_coords()/nn_px(): the per-pixel fp64
// coordinate expressions are the same.
//
// Instantiated once per value type in render_lds_<type>.hip (separate
// translation units build in parallel); launched by launch_render
// (render.hip) when the batch has one value type, one NN namespace and RGBA
// output.
#pragma once
#include "render_common.h"

namespace gsky {

constexpr int kBandRows = kLdsBandRows;
constexpr int kBandEnt = 16;            // entries per pass over the band
constexpr int kStageBytes = 24 * 1024;  // LDS for source windows per block
constexpr int kLanePx = 8;              // pixels per lane per row
constexpr int kBandCols = 64 * kLanePx;  // columns per block (one wave row)
constexpr int kStageDw = 8;             // staging dwords per thread per round (in flight together)

struct BandEnt {
  const void *band;
  int32_t band_x, band_y;
  int32_t xoff, yoff, w, h;
  int32_t fill_mode, mask_pair;
  Val nd, fillv;                        // merge nodata / window fill, as Val bits
  int32_t sx0, sy0, sh, pitch_dw;       // staged rectangle: origin (sx0 dword-aligned), rows, dwords per row
  int32_t soff;                         // LDS byte offset of the rectangle, -1: gather from HBM
  int32_t pair;
  int32_t has_nodata, out_dtype;        // bilinear: nodata taps are dropped (GWKBilinearResample4Sample)
  double nodata64;
};
struct BandRow {
  double xs0, ys0, dX, dY;
  int32_t kind, nleaf, pool_off, _pad;
};

template <typename T> __host__ __device__ constexpr int vt_code();
template <> __host__ __device__ constexpr int vt_code<uint8_t>() { return GSKYHIP_BYTE; }
template <> __host__ __device__ constexpr int vt_code<int8_t>() { return GSKYHIP_SIGNEDBYTE; }
template <> __host__ __device__ constexpr int vt_code<int16_t>() { return GSKYHIP_INT16; }
template <> __host__ __device__ constexpr int vt_code<uint16_t>() { return GSKYHIP_UINT16; }
template <> __host__ __device__ constexpr int vt_code<float>() { return GSKYHIP_FLOAT32; }

// Exact truncated source index at distance `dist` along a linear piece (the
// expressions of lin_coords() / nn_px()); -1 when the coordinate is negative.
__device__ __forceinline__ int piece_index(double s0, double d, int dist) {
  const double v = s0 + d * (double)dist;
  const int idx = __double2int_rz(v + 1.0e-10);   // saturates: >= 2^31 -> INT_MAX, like the >= size test
  return (v >= 0.0) ? idx : -1;
}

// v (|v| < 2^30) as signed 32.32 fixed point, truncated: error < 2^-32.
__device__ __forceinline__ int64_t to_fix(double v) {
  const double f = floor(v);
  const uint32_t lo = (uint32_t)((v - f) * 4294967296.0);   // v - f is exact
  return (int64_t)(((uint64_t)(uint32_t)(int32_t)f << 32) | lo);
}

__device__ __forceinline__ const void *uniform_ptr(const void *p) {
  const uint64_t v = (uint64_t)p;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
  return (const void *)(((uint64_t)hi << 32) | lo);
}

// Scale + palette (or grey) of every value of an integer canvas type T,
// with the nodata rule left out (tested per pixel): lut[v & mask] is the
// RGBA the EncodePNG loop writes for canvas value v (0 where utils.Scale
// yields 0xFF).  Float32 canvases keep the arithmetic path.
template <typename T>
__global__ void scale_lut_kernel(RenderArgs a, const uint32_t *ramp, uint32_t *lut, int n) {
  const int v = blockIdx.x * blockDim.x + threadIdx.x;
  if (v >= n) return;
  using V = typename VOf<T>::type;
  ScaleK sk = make_scale(vt_code<T>(), 0.0, a.sp, false, 0.f, 0.f);
  sk.noData.i = INT32_MIN;            // never equal to a sign/zero-extended 8/16-bit value
  const V c = (V)(T)(uint32_t)v;      // the bits of v as a T
  const uint32_t bb = scale_t<T>(sk, c);
  const uint32_t col = ramp ? ramp[bb & 0xFFu] : (0xFF000000u | (bb << 16) | (bb << 8) | bb);
  lut[v] = bb != 0xFFu ? col : 0u;
}

// FLAGS: bit 0 fixed-point source coordinates, bit 1 Scale+palette LUT
// (A/B knob GSKYHIP_LDS_FLAGS; every combination is bit-identical), bit 2
// bilinear resampling, bit 3 typed canvas output (WCS) instead of RGBA.
constexpr int kFixed = 1, kLut = 2;   // kBilinear = 4, kCanvas = 8: render_common.h

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

template <typename T, bool MASK, bool STAGE, int FLAGS>
__global__ __launch_bounds__(256) void render_lds_kernel(RenderArgs a, const EntryD *__restrict__ ents,
                                                         const int32_t *__restrict__ order,
                                                         const RowRec *__restrict__ rows,
                                                         const Leaf *__restrict__ pool,
                                                         const TilePlan *__restrict__ tplans,
                                                         const gskyhip_tile *__restrict__ tiles, int n_items,
                                                         int per_xcd) {
  using V = typename VOf<T>::type;
  __shared__ uint32_t s_ramp[256];
  __shared__ BandEnt s_ent[kBandEnt];
  __shared__ BandRow s_row[STAGE ? kBandEnt : 1][STAGE ? kBandRows : 1];
  __shared__ int32_t s_ext[kBandEnt][4];     // min x, max x, min y, max y of the source indices
  __shared__ int32_t s_nost[STAGE ? kBandEnt : 1];   // entry has exact rows: not staged
  __shared__ int32_t s_n, s_next;
  __shared__ __attribute__((aligned(16))) uint32_t s_stage[STAGE ? kStageBytes / 4 : 1];

  // item = (tile, 16-row band, 512-column block); column blocks innermost;
  // XCD-aware order when per_xcd > 0 (A/B: linear order measured faster)
  const int item = per_xcd > 0 ? (blockIdx.x & 7) * per_xcd + (blockIdx.x >> 3) : (int)blockIdx.x;
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
  const GPTR(const uint32_t) lut = (GPTR(const uint32_t))a.lut;

  // entries in merge order, kBandEnt band-intersecting ones per pass; a band
  // with more (rare) parks its partial canvas in its own RGBA slot between passes
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
        b.soff = -1;
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
    if (STAGE && tid < kBandEnt * 4) s_ext[tid >> 2][tid & 3] = (tid & 1) ? -1 : 0x7FFFFFFF;
    if (STAGE && tid < kBandEnt) s_nost[tid] = 0;
    __syncthreads();
    const int nb = s_n;
    const int next_e0 = s_next;

    if (STAGE) {
      // row records + exact source-index extremes, one thread per (entry, row)
      {
        const int k = tid >> 4, rr = tid & 15;
        const int r = band0 + rr;
        if (k < nb && r < H) {
          const BandEnt &b = s_ent[k];
          const int ir = r - b.yoff;
          if (ir >= 0 && ir < b.h) {
            const RowRec &R = rows[(int64_t)b.pair * a.max_h + ir];
            BandRow o;
            o.xs0 = R.v[0]; o.ys0 = R.v[1]; o.dX = R.v[2]; o.dY = R.v[3];
            o.kind = R.kind; o.nleaf = R.nleaf; o.pool_off = R.pool_off; o._pad = 0;
            s_row[k][rr] = o;
            int mnx = 0x7FFFFFFF, mxx = -1, mny = 0x7FFFFFFF, mxy = -1;
            const int nl = R.kind == ROW_LINEAR ? 1 : R.kind == ROW_POOL ? R.nleaf : 0;
                      if (nl == 0) s_nost[k] = 1;   // exact / descend row: gather this entry from HBM
            for (int l = 0; l < nl; l++) {
              double xs0 = o.xs0, ys0 = o.ys0, dX = o.dX, dY = o.dY;
              int st = 0, en = b.w - 1;
              if (R.kind != ROW_LINEAR) {
                const Leaf &L = pool[R.pool_off + l];
                if (L.kind != 0) s_nost[k] = 1;
                xs0 = L.xs0; ys0 = L.ys0; dX = L.dX; dY = L.dY; st = L.start;
                en = (l + 1 < nl) ? pool[R.pool_off + l + 1].start - 1 : b.w - 1;
              }
              const int ia = piece_index(xs0, dX, 0), ib = piece_index(xs0, dX, en - st);
              const int ja = piece_index(ys0, dY, 0), jb = piece_index(ys0, dY, en - st);
              mnx = min(mnx, min(ia, ib)); mxx = max(mxx, max(ia, ib));
              mny = min(mny, min(ja, jb)); mxy = max(mxy, max(ja, jb));
            }
            atomicMin(&s_ext[k][0], max(mnx, 0));
            atomicMax(&s_ext[k][1], min(mxx, b.band_x - 1));
            atomicMin(&s_ext[k][2], max(mny, 0));
            atomicMax(&s_ext[k][3], min(mxy, b.band_y - 1));
          }
        }
      }
      __syncthreads();
      if (tid == 0) {   // LDS allocation of the source rectangles, merge order
        int used = 0;
        for (int k = 0; k < nb; k++) {
          BandEnt &b = s_ent[k];
          b.soff = -1;
          const int sh = s_ext[k][3] - s_ext[k][2] + 1;
          const bool dw_rows = ((uintptr_t)b.band & 3) == 0 && ((int64_t)b.band_x * sizeof(T)) % 4 == 0;
          if (s_nost[k] || s_ext[k][1] < s_ext[k][0] || sh <= 0 || !dw_rows) continue;
          const int dw0 = (int)(((int64_t)s_ext[k][0] * sizeof(T)) >> 2);
          const int dw1 = (int)((((int64_t)s_ext[k][1] + 1) * sizeof(T) + 3) >> 2);
          const int pitch = dw1 - dw0;
          const int bytes = pitch * sh * 4;
          if (used + bytes > kStageBytes) continue;
          b.sx0 = (int)((int64_t)dw0 * 4 / sizeof(T));
          b.sy0 = s_ext[k][2];
          b.sh = sh;
          b.pitch_dw = pitch;
          b.soff = used;
          used += bytes;
        }
      }
      __syncthreads();
      // staging: kStageDw dword loads per thread issued together, then stored
      for (int k = 0; k < nb; k++) {
        const BandEnt &b = s_ent[k];
        if (b.soff < 0) continue;
        const uint32_t *src = (const uint32_t *)b.band;
        const int64_t row_dw = (int64_t)b.band_x * sizeof(T) / 4;
        const int64_t col_dw = (int64_t)b.sx0 * sizeof(T) / 4;
        const int total = b.sh * b.pitch_dw;
        uint32_t *dst = s_stage + (b.soff >> 2);
        for (int d0 = 0; d0 < total; d0 += 256 * kStageDw) {
          uint32_t v[kStageDw];
#pragma unroll
          for (int m = 0; m < kStageDw; m++) {
            const int d = d0 + m * 256 + tid;
            const int rr = d / b.pitch_dw, cc = d - rr * b.pitch_dw;
            v[m] = d < total ? src[(int64_t)(b.sy0 + rr) * row_dw + col_dw + cc] : 0u;
          }
#pragma unroll
          for (int m = 0; m < kStageDw; m++) {
            const int d = d0 + m * 256 + tid;
            if (d < total) dst[d] = v[m];
          }
        }
      }
      __syncthreads();
    }

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
        const int soff = __builtin_amdgcn_readfirstlane(b.soff);
        const int ic0 = x0 - __builtin_amdgcn_readfirstlane(b.xoff);
        double xs0, ys0, dX, dY;
        int kind, nleaf, pool_off;
        if (STAGE) {
          const BandRow &R = s_row[k][rr];
          xs0 = R.xs0; ys0 = R.ys0; dX = R.dX; dY = R.dY;
          kind = R.kind; nleaf = R.nleaf; pool_off = R.pool_off;
        } else {
          const RowRec &R = rows[(int64_t)pair * a.max_h + ir];   // wave-uniform: scalar loads
          xs0 = R.v[0]; ys0 = R.v[1]; dX = R.v[2]; dY = R.v[3];
          kind = R.kind; nleaf = R.nleaf; pool_off = R.pool_off;
        }
        kind = __builtin_amdgcn_readfirstlane(kind);
        if constexpr ((FLAGS & kBilinear) != 0) {   // bilinear: exact fp64 coordinates, 4 taps
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
              okc = lin_coords(rows[(int64_t)pair * a.max_h + ir], pool, in ? ic : 0, sx, sy);
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
          continue;
        }
        // source index of each of the lane's pixels: (ux, uy) and validity
        uint32_t ux[kLanePx], uy[kLanePx];
        bool ok[kLanePx];
        bool exact = kind != ROW_LINEAR || !(FLAGS & kFixed);
        if (!exact) {
          // 32.32 fixed point: fx(i) = (xs0 + 1e-10 + dX * i) * 2^32, stepped per
          // pixel.  Off by at most (|i| + 8) * 2^-32 plus a few fp64 ulps from the
          // reference's ax = (xs0 + dX * i) + 1e-10, so away from the guard band
          // around an integer its floor is the reference's (int)ax exactly; a
          // pixel inside the band sends the wave to the fp64 expressions.
          const double xe = xs0 + dX * (double)ew, ye = ys0 + dY * (double)ew;
          const bool fits = fabs(xs0) < 1048576.0 && fabs(ys0) < 1048576.0 && fabs(xe) < 1048576.0 &&
                            fabs(ye) < 1048576.0 && ew < 65536;
          if (!fits) {
            exact = true;
          } else {
            const int64_t Dx = to_fix(dX), Dy = to_fix(dY);
            int64_t fx = to_fix(xs0 + 1.0e-10) + (int64_t)ic0 * Dx;
            int64_t fy = to_fix(ys0 + 1.0e-10) + (int64_t)ic0 * Dy;
            const uint32_t G = 4u * (uint32_t)(ew + 16) + 64u;   // guard, in 2^-32 px
            bool bad = false;
#pragma unroll
            for (int q = 0; q < kLanePx; q++) {
              const uint32_t lx = (uint32_t)fx, ly = (uint32_t)fy;
              ux[q] = (uint32_t)(fx >> 32);
              uy[q] = (uint32_t)(fy >> 32);
              const int ic = ic0 + q;
              const bool in = (unsigned)ic < (unsigned)ew && x0 + q < W;
              bad = bad || (in && (lx + G < 2u * G || ly + G < 2u * G));
              ok[q] = in && ux[q] < (uint32_t)bx && uy[q] < (uint32_t)by;
              fx += Dx;
              fy += Dy;
            }
            exact = __ballot(bad) != 0ull;
          }
        }
        if (exact) {   // the reference's fp64 expressions (lin_coords() / nn_px())
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
              okc = lin_coords(rows[(int64_t)pair * a.max_h + ir], pool, in ? ic : 0, sx, sy);
            }
            const int ix = __double2int_rz(sx + 1.0e-10), iy = __double2int_rz(sy + 1.0e-10);
            ux[q] = (uint32_t)ix;
            uy[q] = (uint32_t)iy;
            ok[q] = in && okc && (sx >= 0.0) && (sy >= 0.0) && ix < bx && iy < by;
          }
        }
        // gather, branch-free: a raw buffer load per pixel with the range check
        // in hardware; an invalid pixel gets an out-of-range offset (no fetch)
        V vv[kLanePx];
        const int64_t nbytes = (int64_t)bx * by * (int64_t)sizeof(T);
        if (STAGE && soff >= 0) {
          const uint8_t *sbase = (const uint8_t *)s_stage + soff;
          const int sx0 = b.sx0, sy0 = b.sy0, pitch_b = b.pitch_dw * 4;
#pragma unroll
          for (int q = 0; q < kLanePx; q++) {
            const int lofs = ok[q] ? ((int)uy[q] - sy0) * pitch_b + ((int)ux[q] - sx0) * (int)sizeof(T) : 0;
            vv[q] = (V)(*(const T *)(sbase + lofs));
          }
        } else if (nbytes < 2147483648LL && bx < (1 << 24) && by < (1 << 24)) {
          const __amdgpu_buffer_rsrc_t rs =
              __builtin_amdgcn_make_buffer_rsrc((void *)bandp, (short)0, (int)nbytes, 0x00020000);
#pragma unroll
          for (int q = 0; q < kLanePx; q++) {
            const uint32_t off = ok[q] ? (__umul24(uy[q], (uint32_t)bx) + ux[q]) * (uint32_t)sizeof(T) : 0x80000000u;
            vv[q] = buf_load<T>(rs, off);
          }
        } else {
#pragma unroll
          for (int q = 0; q < kLanePx; q++) {
            const int64_t idx = ok[q] ? (int64_t)uy[q] * bx + ux[q] : 0;
            vv[q] = (V)((const GPTR(T))bandp)[idx];
          }
        }
#pragma unroll
        for (int q = 0; q < kLanePx; q++) {
          const int ic = ic0 + q;
          const V v = ok[q] ? vv[q] : fillv;
          const bool in = (unsigned)ic < (unsigned)ew && x0 + q < W;
          bool take = in && (v != nd);
          if (MASK && b.mask_pair >= 0) {
            if (take) take = !mask_fast<GSKYHIP_RESAMPLE_NEAREST>(ents, rows, pool, a.mask, ents[pair], ic, ir);
          }
          const bool t2 = take && (!fill_mode || c[q] == nd);
          c[q] = t2 ? v : c[q];
        }
      }
      if constexpr ((FLAGS & kCanvas) != 0) {   // typed canvas (tile_merger.go:562-652): T stores
        T tv[kLanePx];
#pragma unroll
        for (int q = 0; q < kLanePx; q++) tv[q] = (T)c[q];
        if (x0 + kLanePx <= W && (((uintptr_t)cdst) & (sizeof(T) * kLanePx >= 16 ? 15 : sizeof(T) * kLanePx - 1)) == 0) {
          if constexpr (sizeof(T) == 4) {
            u32x4 v0, v1;
            __builtin_memcpy(&v0, tv, 16);
            __builtin_memcpy(&v1, tv + 4, 16);
            __builtin_nontemporal_store(v0, (GPTR(u32x4))cdst);
            __builtin_nontemporal_store(v1, (GPTR(u32x4))(cdst + 4));
          } else if constexpr (sizeof(T) == 2) {
            u32x4 v0;
            __builtin_memcpy(&v0, tv, 16);
            __builtin_nontemporal_store(v0, (GPTR(u32x4))cdst);
          } else {
            uint64_t v0;
            __builtin_memcpy(&v0, tv, 8);
            *(uint64_t *)cdst = v0;
          }
        } else {
#pragma unroll
          for (int q = 0; q < kLanePx; q++)
            if (x0 + q < W) cdst[q] = tv[q];
        }
        continue;
      }
      if (!last) {   // partial canvas parked in the slot (raw values), re-read next pass
#pragma unroll
        for (int q = 0; q < kLanePx; q++)
          if (x0 + q < W) ((V *)dst)[q] = c[q];
        continue;
      }
      // utils.Scale + palette / grey: the per-launch LUT for integer canvases
      uint32_t pxo[kLanePx];
#pragma unroll
      for (int q = 0; q < kLanePx; q++) {
        if constexpr (std::is_same<T, float>::value || !(FLAGS & kLut)) {
          const uint32_t bb = scale_t<T>(sk, c[q]);
          const uint32_t col = has_ramp ? s_ramp[bb & 0xFFu] : (0xFF000000u | (bb << 16) | (bb << 8) | bb);
          pxo[q] = (created && bb != 0xFFu) ? col : 0u;
        } else {
          const uint32_t col = lut[(uint32_t)c[q] & (sizeof(T) == 1 ? 0xFFu : 0xFFFFu)];
          pxo[q] = (created && c[q] != cnod) ? col : 0u;
        }
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
  const int per_xcd = a.nn_xcd ? (n_items + 7) / 8 : 0;
  const dim3 grid(a.nn_xcd ? (unsigned)per_xcd * 8 : (unsigned)n_items);
#define GSKY_LDS_LAUNCH(M, S, F)                                                                                   \
  hipLaunchKernelGGL((render_lds_kernel<T, M, S, F>), grid, dim3(256), 0, s, a, a.entries, a.order, a.rows, a.pool, \
                     a.tplans, a.tiles, n_items, per_xcd)
  if (!std::is_same<T, float>::value && (a.lds_flags & kLut) && !(a.lds_mode & (kBilinear | kCanvas))) {
    const int n = sizeof(T) == 1 ? 256 : 65536;   // Scale + palette LUT of the launch
    hipLaunchKernelGGL(scale_lut_kernel<T>, dim3((n + 255) / 256), dim3(256), 0, s, a, (const uint32_t *)a.ramp,
                       a.lut, n);
  }
  const bool stage = a.lds_stage != 0;
  const int fl = a.lds_flags;
  if (a.lds_mode & (kBilinear | kCanvas)) {   // bilinear and / or typed canvas output
    switch ((a.lds_mode & (kBilinear | kCanvas)) | (mask ? 16 : 0)) {
      case kBilinear: GSKY_LDS_LAUNCH(false, false, kBilinear); break;
      case kCanvas: GSKY_LDS_LAUNCH(false, false, kCanvas); break;
      case kBilinear | kCanvas: GSKY_LDS_LAUNCH(false, false, kBilinear | kCanvas); break;
      case 16 | kBilinear: GSKY_LDS_LAUNCH(true, false, kBilinear); break;
      case 16 | kCanvas: GSKY_LDS_LAUNCH(true, false, kCanvas); break;
      default: GSKY_LDS_LAUNCH(true, false, kBilinear | kCanvas); break;
    }
    return;
  }
  if (mask) {
    if (stage) GSKY_LDS_LAUNCH(true, true, 0); else GSKY_LDS_LAUNCH(true, false, 0);
  } else if (stage) {
    GSKY_LDS_LAUNCH(false, true, 0);
  } else if (fl == 1) {
    GSKY_LDS_LAUNCH(false, false, 1);
  } else if (fl == 2) {
    GSKY_LDS_LAUNCH(false, false, 2);
  } else if (fl == 3) {
    GSKY_LDS_LAUNCH(false, false, 3);
  } else {
    GSKY_LDS_LAUNCH(false, false, 0);
  }
#undef GSKY_LDS_LAUNCH
}

void launch_lds_i16(const RenderArgs &a, bool mask, int n_items, hipStream_t s);
void launch_lds_u16(const RenderArgs &a, bool mask, int n_items, hipStream_t s);
void launch_lds_f32(const RenderArgs &a, bool mask, int n_items, hipStream_t s);
void launch_lds_i8(const RenderArgs &a, bool mask, int n_items, hipStream_t s);
void launch_lds_u8(const RenderArgs &a, bool mask, int n_items, hipStream_t s);

}  // namespace gsky
