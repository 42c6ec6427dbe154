// render_nn.h -- the nearest-neighbour band kernel (GetMap C1 / C2 / C5 and
// nearest-neighbour GetCoverage).
//
// Work of one launch: every (tile, 16-row band, 512-column block) item of the
// simple tiles of a batch whose stack entries share value type T.  Per output
// pixel: the reference's fp64 source coordinate of the window pixel
// (lin_coords(): the GDAL approximate transformer's row interpolation,
// warp.go:269), the truncation and bounds test of warp.go:271-300 (nn_px()),
// one gather, the ordered nodata / mask / timestamp fold of MergeMaskedRaster
// (tile_merger.go:38-225) over the tile's entries in ProcessRasterStack order,
// then utils.Scale (raster_scaler.go:30-332) and the palette / grey RGBA of
// EncodePNG (ogc_encoders.go:94-133) -- or the typed canvas of GetCoverage.
//
// Shape (round 3; the round-2 kernel issued ~40 SALU + ~47 VALU wave
// instructions per 64-pixel slot, profiles/pmc_render_c2.json):
//   * a wave owns kNnRows consecutive rows of the block; a lane the 8 pixels
//     lane, lane + 64, ..., lane + 448 of each row, so every gather and every
//     RGBA store instruction covers 64 consecutive output columns, and one
//     row of one entry is a single scalar chain (order -> descriptor -> row
//     record) for all 512 columns;
//   * an entry whose window covers every column of the block on a row the
//     planner marked `inside` (RowRec.inside: every window pixel's source
//     pixel lies in the band) takes the fast body: truncate, index, load, and
//     a fold that is one compare + one select -- (v != nd) ? v : c, or in fill
//     mode (c == nd) ? v : c, which is "v != nd && c == nd" without the
//     second compare -- so no lane-mask logic lands on the scalar unit;
//   * everything else (window edges inside the block, POOL rows with their
//     leaves, failed transforms, entries carrying a mask layer) takes the
//     general body with the per-pixel tests of the reference;
//   * output: Scale in the canvas type, the uint8(float32) range test only
//     when clip * scale can reach 2^31 (wave-uniform), and one LDS read of a
//     256-entry table that has EncodePNG's transparency rule baked in (entry
//     255 and canvases never created are 0); 8 non-temporal 4-B stores per
//     lane and row, each 256 contiguous bytes per wave.
// Every body computes the reference's expressions, so all of them agree bit
// for bit with oracle/ (tests/test_gpu_parity.py, tests/test_gpu_full.py).
#pragma once
#ifdef GSKYHIP_AB
#include <cstdlib>
#endif
#include "render_lds.h"

namespace gsky {

constexpr uint32_t kNoPx = 0xFFFFFFFFu;
constexpr int kNnRows = 4;   // rows per wave (a block: 4 waves x 4 rows = kBandRows)
constexpr int kNnPx = 8;     // pixels per lane per row, 64 columns apart

// a wave-uniform 64-bit value in scalar registers
__device__ __forceinline__ int64_t uni64(int64_t v) {
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v), hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
  return (int64_t)(((uint64_t)hi << 32) | lo);
}

__device__ __forceinline__ double uni64d(double v) {
  return __longlong_as_double(uni64(__double_as_longlong(v)));
}

// nn_px() of source coordinates (sx, sy): the element index, or kNoPx where
// the reference's window fill applies.
__device__ __forceinline__ uint32_t nn_index_sxy(double sx, double sy, bool ok, int bx, int by) {
  const int ix = __double2int_rz(sx + 1.0e-10), iy = __double2int_rz(sy + 1.0e-10);
  ok = ok && (sx >= 0.0) && (sy >= 0.0) && ix < bx && iy < by;
  return ok ? __umul24((uint32_t)iy, (uint32_t)bx) + (uint32_t)ix : kNoPx;
}

// utils.Scale of an integer canvas value (scale_t(): nodata -> 0xFF, value +=
// offset wrapping in T, clamp to [0, clip], float32 multiply, Go uint8 of the
// float32).  SAFE: 0 <= value * sc < 2^31 holds for every clamped value.
template <typename T, bool SAFE>
__device__ __forceinline__ uint32_t scale_int(const ScaleK &k, int32_t c) {
  int32_t value = c + k.off.i;
  if constexpr (std::is_same<T, int8_t>::value) value = (int8_t)value;
  else if constexpr (std::is_same<T, uint8_t>::value) value = (uint8_t)value;
  else if constexpr (std::is_same<T, int16_t>::value) value = (int16_t)value;
  else value = (uint16_t)value;
  value = max(min(value, k.clp.i), 0);   // raster_scaler.go: clip first, then 0 (clip < 0 gives 0)
  const float f = (float)value * k.sc;
  const uint32_t b = SAFE ? ((uint32_t)(int32_t)f & 0xFFu) : go_u8_f32(f);
  return c == k.noData.i ? 0xFFu : b;
}

// The fold of one `inside` LINEAR row whose window edge falls inside the
// block: the fast body plus the window test (pixels outside the window read
// nothing and fold nothing; fill mode takes v where c is nodata, which equals
// the general rule's "v != nd && c == nd" because v == nd == c leaves c
// unchanged).  Halves of 4 pixels keep the register peak of the fast body.
template <typename T, int NPX>
__device__ __forceinline__ void nn_partial_row(__amdgpu_buffer_rsrc_t rs, double xs0, double ys0, double dX, double dY,
                                               int ic0, int lim, int bx, typename VOf<T>::type nd, bool fill_mode,
                                               int c0, int c1, typename VOf<T>::type (&c)[NPX]) {
  using V = typename VOf<T>::type;
#pragma unroll
  for (int h = 0; h < NPX; h += 4) {
    uint32_t off[4];
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const int ic = ic0 + 64 * (h + q);
      const double dist = (double)ic;
      const int ix = __double2int_rz(xs0 + dX * dist + 1.0e-10);
      const int iy = __double2int_rz(ys0 + dY * dist + 1.0e-10);
      off[q] = (unsigned)ic < (unsigned)lim ? (__umul24((uint32_t)iy, (uint32_t)bx) + (uint32_t)ix) * (uint32_t)sizeof(T)
                                            : 0x80000000u;
    }
    V vv[4];
#pragma unroll
    for (int q = 0; q < 4; q++) vv[q] = buf_load<T>(rs, off[q]);
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const bool inw = (unsigned)(ic0 + 64 * (h + q)) < (unsigned)lim;
      c[h + q] = (inw & (fill_mode ? (c[h + q] == nd) : (vv[q] != nd))) ? vv[q] : c[h + q];
    }
  }
}

// The fold of one `inside` LINEAR row from its fixed-point form (RowFix,
// gsky_device.h): per pixel two 64-bit integer adds per axis in place of the
// fp64 multiply, two adds and the conversion of each axis.  The source pixel
// is the integer part wherever the fraction is at least kFixMargin from an
// integer -- there it equals the truncation of the reference's fp64
// expression; if any pixel of the wave's row is closer (about 1 row in 250),
// nothing is folded and false sends the row to the fp64 bodies.
// PART: the window edge falls inside the block (pixels outside the window
// read nothing and fold nothing).
template <typename T, int NPX, bool PART, bool WIDE = false>
__device__ __forceinline__ bool nn_fix_row(__amdgpu_buffer_rsrc_t rs, int64_t fx0, int64_t fy0, int64_t fdx,
                                           int64_t fdy, int ic0, int lim, int bx, typename VOf<T>::type nd,
                                           bool fill_mode, typename VOf<T>::type (&c)[NPX]) {
  using V = typename VOf<T>::type;
  uint64_t X = (uint64_t)(fx0 + (int64_t)ic0 * fdx), Y = (uint64_t)(fy0 + (int64_t)ic0 * fdy);
  const uint64_t SX = (uint64_t)fdx << 6, SY = (uint64_t)fdy << 6;   // 64 columns
  uint32_t amin = 0xFFFFFFFFu;
  uint32_t off[NPX];
#pragma unroll
  for (int q = 0; q < NPX; q++) {
    const uint32_t ix = (uint32_t)(X >> 32), iy = (uint32_t)(Y >> 32);
    uint32_t a = min((uint32_t)X + kFixMargin, (uint32_t)Y + kFixMargin);
    off[q] = (__umul24(iy, (uint32_t)bx) + ix) * (uint32_t)sizeof(T);
    if constexpr (PART) {
      const bool inw = (unsigned)(ic0 + 64 * q) < (unsigned)lim;
      off[q] = inw ? off[q] : 0x80000000u;
      a = inw ? a : 0xFFFFFFFFu;
    }
    amin = min(amin, a);
    // keep the offset here: sunk below the test, it would hold every X, Y
    // (32 VGPRs) live across it and spill at 8 waves per SIMD
    asm volatile("" : "+v"(off[q]));
    X += SX;
    Y += SY;
  }
  // the test comes before the loads: a load left unconsumed on the fallback
  // path would make the compiler drain vmcnt -- the previous row's RGBA
  // stores included -- before the next use of its register
  if (__builtin_amdgcn_ballot_w64(amin < 2u * kFixMargin) != 0) return false;
  V vv[NPX];
#pragma unroll
  for (int q = 0; q < NPX; q++) vv[q] = WIDE ? buf_load_w<T>(rs, off[q]) : buf_load<T>(rs, off[q]);
  if (!fill_mode) {
#pragma unroll
    for (int q = 0; q < NPX; q++) {
      bool take = vv[q] != nd;
      if constexpr (PART) take = take & ((unsigned)(ic0 + 64 * q) < (unsigned)lim);
      c[q] = take ? vv[q] : c[q];
    }
  } else {
#pragma unroll
    for (int q = 0; q < NPX; q++) {
      bool take = c[q] == nd;
      if constexpr (PART) take = take & ((unsigned)(ic0 + 64 * q) < (unsigned)lim);
      c[q] = take ? vv[q] : c[q];
    }
  }
  return true;
}

// nn_fix_row's cover case for 2-byte T with a lane owning column PAIRS
// (A/B, GSKYHIP_NN_PAIR=1): the lane's pixels are columns icp + 128 q + k
// (k = 0, 1) -> c[2 q + k], so one aligned dword gather serves both pixels of
// a pair whenever their source pixels share it (C2: ~70 % of pairs; the
// rest take a second, lane-masked gather) and the RGBA leaves as 8-byte
// stores: half the 64-lane gather and store instructions, whose per-quad L1
// work bounds the row-major body.  Same fixed-point values,
// margin test and fold as nn_fix_row: the same result bit for bit.
template <typename T, int NPX>
__device__ __forceinline__ bool nn_fix_row_pair(__amdgpu_buffer_rsrc_t rs, int64_t fx0, int64_t fy0, int64_t fdx,
                                                int64_t fdy, int icp, int bx, typename VOf<T>::type nd,
                                                bool fill_mode, typename VOf<T>::type (&c)[NPX]) {
  static_assert(sizeof(T) == 2 && NPX % 2 == 0, "pairs of 16-bit pixels");
  using V = typename VOf<T>::type;
  constexpr int NQ = NPX / 2;
  uint64_t X = (uint64_t)(fx0 + (int64_t)icp * fdx), Y = (uint64_t)(fy0 + (int64_t)icp * fdy);
  const uint64_t SX = (uint64_t)fdx << 7, SY = (uint64_t)fdy << 7;   // 128 columns
  uint32_t amin = 0xFFFFFFFFu;
  uint32_t e0[NQ], e1[NQ];
#pragma unroll
  for (int q = 0; q < NQ; q++) {
    const uint64_t X1 = X + (uint64_t)fdx, Y1 = Y + (uint64_t)fdy;
    e0[q] = __umul24((uint32_t)(Y >> 32), (uint32_t)bx) + (uint32_t)(X >> 32);
    e1[q] = __umul24((uint32_t)(Y1 >> 32), (uint32_t)bx) + (uint32_t)(X1 >> 32);
    amin = min(amin, min(min((uint32_t)X + kFixMargin, (uint32_t)Y + kFixMargin),
                         min((uint32_t)X1 + kFixMargin, (uint32_t)Y1 + kFixMargin)));
    asm volatile("" : "+v"(e0[q]), "+v"(e1[q]));
    X += SX;
    Y += SY;
  }
  if (__builtin_amdgcn_ballot_w64(amin < 2u * kFixMargin) != 0) return false;
  uint32_t w0[NQ], w1[NQ];
#pragma unroll
  for (int q = 0; q < NQ; q++) w0[q] = __builtin_amdgcn_raw_buffer_load_b32(rs, (e0[q] * 2u) & ~3u, 0, 0);
#pragma unroll
  for (int q = 0; q < NQ; q++) {
    w1[q] = w0[q];
    if ((e1[q] ^ e0[q]) > 1u) w1[q] = __builtin_amdgcn_raw_buffer_load_b32(rs, (e1[q] * 2u) & ~3u, 0, 0);
  }
#pragma unroll
  for (int q = 0; q < NQ; q++) {
    const uint32_t h0 = (w0[q] >> ((e0[q] & 1u) * 16u)) & 0xFFFFu, h1 = (w1[q] >> ((e1[q] & 1u) * 16u)) & 0xFFFFu;
    const V v0 = std::is_signed<T>::value ? (V)(int16_t)h0 : (V)h0;
    const V v1 = std::is_signed<T>::value ? (V)(int16_t)h1 : (V)h1;
    if (!fill_mode) {
      c[2 * q] = v0 != nd ? v0 : c[2 * q];
      c[2 * q + 1] = v1 != nd ? v1 : c[2 * q + 1];
    } else {
      c[2 * q] = c[2 * q] == nd ? v0 : c[2 * q];
      c[2 * q + 1] = c[2 * q + 1] == nd ? v1 : c[2 * q + 1];
    }
  }
  return true;
}

// The fold of one `inside` LINEAR row covering the block (nn_fix_row's cover
// case) with cooperative loads instead of per-lane gathers: for each of the
// lane's 8 pixels the wave's 64 consecutive output columns read a source run
// of at most 2 rows and 32 * (4 / sizeof(T)) - 2 columns; lanes 0-31 load
// that run of the upper row and lanes 32-63 of the lower as consecutive
// dwords (one coalesced load instruction), and every lane picks its value
// with ds_bpermute.  The same source pixels as the gathers (the fixed-point
// indices), so the same result bit for bit.  false: ambiguous (nothing
// folded, the fp64 bodies follow) -- or, with nothing loaded yet, a run that
// does not fit, where the per-lane gathers are used.  A/B (GSKYHIP_NN_COOP).
template <typename T, int NPX>
__device__ __forceinline__ bool nn_fix_row_coop(__amdgpu_buffer_rsrc_t rs, int64_t fx0, int64_t fy0, int64_t fdx,
                                                int64_t fdy, int ic0, int lim, int bx, typename VOf<T>::type nd,
                                                bool fill_mode, typename VOf<T>::type (&c)[NPX], int lane) {
  using V = typename VOf<T>::type;
  constexpr int K = 4 / (int)sizeof(T);   // elements per dword
  uint64_t X = (uint64_t)(fx0 + (int64_t)ic0 * fdx), Y = (uint64_t)(fy0 + (int64_t)ic0 * fdy);
  const uint64_t SX = (uint64_t)fdx << 6, SY = (uint64_t)fdy << 6;
  uint32_t amin = 0xFFFFFFFFu;
  int ix[NPX], iy[NPX];
#pragma unroll
  for (int q = 0; q < NPX; q++) {
    ix[q] = (int)(uint32_t)(X >> 32);
    iy[q] = (int)(uint32_t)(Y >> 32);
    amin = min(amin, min((uint32_t)X + kFixMargin, (uint32_t)Y + kFixMargin));
    X += SX;
    Y += SY;
  }
  if (__builtin_amdgcn_ballot_w64(amin < 2u * kFixMargin) != 0) return false;
  // per pixel slot: the run's rows and columns (monotone in the column: the
  // end lanes hold the extremes)
  int base0[NPX], base1[NPX], r0s[NPX];
  bool fits = true;
#pragma unroll
  for (int q = 0; q < NPX; q++) {
    const int xa = __builtin_amdgcn_readlane(ix[q], 0), xb2 = __builtin_amdgcn_readlane(ix[q], 63);
    const int ya = __builtin_amdgcn_readlane(iy[q], 0), yb = __builtin_amdgcn_readlane(iy[q], 63);
    const int lo = min(xa, xb2), hi = max(xa, xb2), r0 = min(ya, yb), r1 = max(ya, yb);
    fits = fits & (hi - lo <= 32 * K - 2 * K) & (r1 - r0 <= 1);
    const int e0 = r0 * bx + lo, e1 = (r0 + 1) * bx + lo;
    base0[q] = e0 & ~(K - 1);
    base1[q] = e1 & ~(K - 1);
    r0s[q] = r0;
  }
  V vv[NPX];
  if (fits) {
    uint32_t w[NPX];
#pragma unroll
    for (int q = 0; q < NPX; q++) {
      const int mybase = lane < 32 ? base0[q] : base1[q];
      w[q] = __builtin_amdgcn_raw_buffer_load_b32(rs, (uint32_t)(mybase / K + (lane & 31)) * 4u, 0, 0);
    }
#pragma unroll
    for (int q = 0; q < NPX; q++) {
      const bool upper = iy[q] == r0s[q];
      const int rel = iy[q] * bx + ix[q] - (upper ? base0[q] : base1[q]);
      const int src = (upper ? 0 : 32) + rel / K;
      const uint32_t got = (uint32_t)__builtin_amdgcn_ds_bpermute(src * 4, (int)w[q]);
      const uint32_t sh = (uint32_t)(rel % K) * 8u * (uint32_t)sizeof(T);
      if constexpr (sizeof(T) == 4) {
        vv[q] = __builtin_bit_cast(V, got);
      } else if constexpr (sizeof(T) == 2) {
        const uint32_t h = (got >> sh) & 0xFFFFu;
        vv[q] = std::is_signed<T>::value ? (V)(int16_t)h : (V)h;
      } else {
        const uint32_t b = (got >> sh) & 0xFFu;
        vv[q] = std::is_signed<T>::value ? (V)(int8_t)b : (V)b;
      }
    }
  } else {
#pragma unroll
    for (int q = 0; q < NPX; q++)
      vv[q] = buf_load<T>(rs, (__umul24((uint32_t)iy[q], (uint32_t)bx) + (uint32_t)ix[q]) * (uint32_t)sizeof(T));
  }
  if (!fill_mode) {
#pragma unroll
    for (int q = 0; q < NPX; q++) c[q] = (vv[q] != nd) ? vv[q] : c[q];
  } else {
#pragma unroll
    for (int q = 0; q < NPX; q++) c[q] = (c[q] == nd) ? vv[q] : c[q];
  }
  return true;
}

// A/B (GSKYHIP_NN_MASKB=1; 0.526 vs 0.494 ms on C5, profiles/r05o_c5.jsonl):
// the general body for an entry carrying a mask layer (C5's QA stacks), all
// NPX pixels at once: every data index and every mask index first, then all
// 2 x NPX gathers in flight together, then the fold -- mask_fast() per pixel
// inside the fold chained the mask entry's descriptor, row record and gather
// behind each taken pixel (4 dependent memory latencies per half row).  The
// same expressions as the general body + mask_fast(): the same result.
template <typename T, int NPX>
__device__ __forceinline__ void nn_masked_row(const RenderArgs &a, const EntryD *__restrict__ ents, const EntryD &e,
                                              const RowRec *__restrict__ rows, const Leaf *__restrict__ pool,
                                              __amdgpu_buffer_rsrc_t rs, const RowRec *rr, int kind, int ic0, int lim,
                                              int bx, int by, typename VOf<T>::type nd, bool fill_mode, int ir,
                                              typename VOf<T>::type (&c)[NPX]) {
  using V = typename VOf<T>::type;
  constexpr uint32_t kMaskOff = 0xFFFFFFFEu;   // mask row past the mask's height: not masked
  const EntryD &m = ents[e.mask_pair];
  const int ew = e.w, mw = m.w, mh = m.h, mbx = m.band_x, mby = m.band_y, mdt = m.out_dtype;
  const int msz = type_size(mdt);
  const int slot = mask_slot(mdt);
  const int32_t mfill = m.fill.i;
  const __amdgpu_buffer_rsrc_t mrs = __builtin_amdgcn_make_buffer_rsrc(
      (void *)uniform_ptr(m.band), (short)0, (int)((int64_t)mbx * mby * (int64_t)msz), 0x00020000);
  uint32_t idx[NPX], midx[NPX];
  if (kind == ROW_LINEAR) {
    const double xs0 = rr->v[0], ys0 = rr->v[1], dX = rr->v[2], dY = rr->v[3];
#pragma unroll
    for (int q = 0; q < NPX; q++) {
      const int ic = ic0 + 64 * q;
      const double dist = (double)ic;
      idx[q] = nn_index_sxy(xs0 + dX * dist, ys0 + dY * dist, (unsigned)ic < (unsigned)lim, bx, by);
    }
  } else {   // POOL: the leaf of each pixel
    const int nleaf = __builtin_amdgcn_readfirstlane(rr->nleaf);
    const Leaf *lv = pool + __builtin_amdgcn_readfirstlane(rr->pool_off);
#pragma unroll 1
    for (int q = 0; q < NPX; q++) {
      const int ic = ic0 + 64 * q;
      const bool in = (unsigned)ic < (unsigned)lim;
      const Leaf &L = lv[leaf_of(lv, nleaf, in ? ic : 0)];
      const double dist = (double)(ic - L.start);
      idx[q] = nn_index_sxy(L.xs0 + L.dX * dist, L.ys0 + L.dY * dist, in && L.kind != LEAF_FAILED, bx, by);
    }
  }
  // mask_fast(): the mask window index of data pixel (ic, ir) -- the same
  // index when the widths agree, else through the row-major data index
  if (mw == ew) {
    if (ir >= mh) {
#pragma unroll
      for (int q = 0; q < NPX; q++) midx[q] = kMaskOff;
    } else {
      const RowRec *mr = rows + m.row_base + ir;
#pragma unroll
      for (int q = 0; q < NPX; q++) {
        const int ic = ic0 + 64 * q;
        double sx, sy;
        const bool ok = lin_coords(*mr, pool, (unsigned)ic < (unsigned)lim ? ic : 0, sx, sy);
        midx[q] = ok ? nn_index_sxy(sx, sy, true, mbx, mby) : kNoPx;
      }
    }
  } else {
#pragma unroll 1
    for (int q = 0; q < NPX; q++) {
      const int ic = ic0 + 64 * q;
      midx[q] = kMaskOff;
      if ((unsigned)ic < (unsigned)lim) {
        const long iSrc = (long)ir * ew + ic;
        const int mx = (int)(iSrc % mw), my = (int)(iSrc / mw);
        if (my < mh) {
          double sx, sy;
          midx[q] = lin_coords(rows[m.row_base + my], pool, mx, sx, sy) ? nn_index_sxy(sx, sy, true, mbx, mby) : kNoPx;
        }
      }
    }
  }
  V vv[NPX];
  uint32_t mraw[NPX];
#pragma unroll
  for (int q = 0; q < NPX; q++) vv[q] = buf_load<T>(rs, idx[q] * (uint32_t)sizeof(T));
  if (msz == 1) {
#pragma unroll
    for (int q = 0; q < NPX; q++) mraw[q] = __builtin_amdgcn_raw_buffer_load_b8(mrs, midx[q], 0, 0);
  } else {
#pragma unroll
    for (int q = 0; q < NPX; q++) mraw[q] = __builtin_amdgcn_raw_buffer_load_b16(mrs, midx[q] * 2u, 0, 0);
  }
  const V fillv = as_v<T>(e.fill);
#pragma unroll
  for (int q = 0; q < NPX; q++) {
    const int ic = ic0 + 64 * q;
    const V v = idx[q] != kNoPx ? vv[q] : fillv;
    int32_t mv;
    switch (mdt) {   // nn_fetch<mask type>'s value
      case GSKYHIP_SIGNEDBYTE: mv = (int32_t)(int8_t)(uint8_t)mraw[q]; break;
      case GSKYHIP_INT16: mv = (int32_t)(int16_t)(uint16_t)mraw[q]; break;
      case GSKYHIP_BYTE: mv = (int32_t)(uint8_t)mraw[q]; break;
      default: mv = (int32_t)(uint16_t)mraw[q]; break;
    }
    if (midx[q] == kNoPx) mv = mfill;
    const bool mk = midx[q] != kMaskOff && slot >= 0 && mask_bit(a.mask[slot], mdt, mv);
    const bool take = (unsigned)ic < (unsigned)lim && (v != nd) && !mk;
    const bool t2 = take && (!fill_mode || c[q] == nd);
    c[q] = t2 ? v : c[q];
  }
}

// One stack entry e of the ordered fold of tile row r (MergeMaskedRaster,
// tile_merger.go:38-225): c[q] is the canvas value of the lane's pixel q
// (tile column xl + 64 q).
// PARTIAL: with the window-edge body for `inside` rows (the single-entry path
// of render_nn_kernel has its own and passes false).
template <typename T, bool MASK, int NPX = kNnPx, bool PARTIAL = true, bool FIX = true>
__device__ __forceinline__ void nn_entry_row(const RenderArgs &a, const EntryD *__restrict__ ents, const EntryD &e,
                                             const RowRec *__restrict__ rows, const RowFix *__restrict__ rowfix,
                                             const Leaf *__restrict__ pool,
                                             int ns_out, int r, int xb, int xl, int W, int ncols,
                                             typename VOf<T>::type (&c)[NPX]) {
  using V = typename VOf<T>::type;
  const int eyoff = e.yoff, eh = e.h, exoff = e.xoff, ew = e.w;
  if (e.ns != ns_out || ew <= 0) return;
  const int ir = r - eyoff;
  if (ir < 0 || ir >= eh) return;
  const int lim = max(0, min(ew, W - exoff));   // window pixel in the tile: (unsigned)ic < lim
  const int c0 = exoff - xb, c1 = exoff + lim - xb;   // the entry's columns of the block: [c0, c1)
  if (c1 <= 0 || c0 >= ncols) return;
  const int bx = e.band_x, by = e.band_y;
  const V nd = as_v<T>(e.nd);
  const bool fill_mode = e.fill_mode != 0;
  const int ic0 = xl - exoff;   // window column of the lane's pixel 0
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
      (void *)uniform_ptr(e.band), (short)0, (int)((int64_t)bx * by * (int64_t)sizeof(T)), 0x00020000);
  const bool masked = MASK && e.mask_pair >= 0;
  if (FIX && !masked) {   // fixed-point form of an `inside` LINEAR row
    const RowFix *fp = rowfix + e.row_base + ir;
    const int64_t fx0 = uni64(fp->x0);
    if (fx0 != kFixNone) {
      const int64_t fy0 = uni64(fp->y0), fdx = uni64(fp->dx), fdy = uni64(fp->dy);
      const bool done = (c0 <= 0 && c1 >= ncols)
                            ? nn_fix_row<T, NPX, false>(rs, fx0, fy0, fdx, fdy, ic0, lim, bx, nd, fill_mode, c)
                            : nn_fix_row<T, NPX, true>(rs, fx0, fy0, fdx, fdy, ic0, lim, bx, nd, fill_mode, c);
      if (done) return;
    }
  }
  const RowRec *rr = rows + e.row_base + ir;
  const int kind = __builtin_amdgcn_readfirstlane(rr->kind);
  const int inside = __builtin_amdgcn_readfirstlane(rr->inside);
  if (kind == ROW_LINEAR && inside && c0 <= 0 && c1 >= ncols && !masked) {
    // fast body: every pixel of the block is in the window and its source
    // pixel in the band -- lin_coords() + nn_px() reduce to the truncations
    const double xs0 = rr->v[0], ys0 = rr->v[1], dX = rr->v[2], dY = rr->v[3];
    uint32_t off[NPX];
#pragma unroll
    for (int q = 0; q < NPX; q++) {
      const double dist = (double)(ic0 + 64 * q);
      const int ix = __double2int_rz(xs0 + dX * dist + 1.0e-10);
      const int iy = __double2int_rz(ys0 + dY * dist + 1.0e-10);
      off[q] = (__umul24((uint32_t)iy, (uint32_t)bx) + (uint32_t)ix) * (uint32_t)sizeof(T);
    }
    V vv[NPX];
#pragma unroll
    for (int q = 0; q < NPX; q++) vv[q] = buf_load<T>(rs, off[q]);
    if (!fill_mode) {
#pragma unroll
      for (int q = 0; q < NPX; q++) c[q] = (vv[q] != nd) ? vv[q] : c[q];
    } else {
#pragma unroll
      for (int q = 0; q < NPX; q++) c[q] = (c[q] == nd) ? vv[q] : c[q];
    }
    return;
  }
  if (PARTIAL && kind == ROW_LINEAR && inside && !masked) {
    // window edge inside the block on an `inside` row: the fast body plus the
    // window test (pixels outside the window read nothing and fold nothing;
    // fill mode takes v where c is nodata, which equals the general rule's
    // "v != nd && c == nd" because v == nd == c leaves c unchanged)
    nn_partial_row<T, NPX>(rs, rr->v[0], rr->v[1], rr->v[2], rr->v[3], ic0, lim, bx, nd, fill_mode, c0, c1, c);
    return;
  }
#ifdef GSKYHIP_AB
  if constexpr (MASK) {
    if (masked && a.nn_maskb) {   // A/B (GSKYHIP_NN_MASKB=1): measured slower on C5, 0.526 vs 0.494 ms
      nn_masked_row<T, NPX>(a, ents, e, rows, pool, rs, rr, kind, ic0, lim, bx, by, nd, fill_mode, ir, c);
      return;
    }
  }
#endif
  // general body: POOL rows, rows not inside the band, mask layer;
  // two halves of 4 pixels (4 gathers in flight) keep the register peak
  // of the fast body
  const V fillv = as_v<T>(e.fill);
#pragma unroll
  for (int h = 0; h < NPX; h += 4) {
    uint32_t idx[4];
    if (kind == ROW_LINEAR) {
      const double xs0 = rr->v[0], ys0 = rr->v[1], dX = rr->v[2], dY = rr->v[3];
#pragma unroll
      for (int q = 0; q < 4; q++) {
        const int ic = ic0 + 64 * (h + q);
        const double dist = (double)ic;
        idx[q] = nn_index_sxy(xs0 + dX * dist, ys0 + dY * dist, (unsigned)ic < (unsigned)lim, bx, by);
      }
    } else {   // POOL (the only other kind of a simple tile): the leaf of each pixel
      const int nleaf = __builtin_amdgcn_readfirstlane(rr->nleaf);
      const Leaf *lv = pool + __builtin_amdgcn_readfirstlane(rr->pool_off);
#pragma unroll 1
      for (int q = 0; q < 4; q++) {
        const int ic = ic0 + 64 * (h + q);
        const bool in = (unsigned)ic < (unsigned)lim;
        const Leaf &L = lv[leaf_of(lv, nleaf, in ? ic : 0)];
        const double dist = (double)(ic - L.start);
        idx[q] = nn_index_sxy(L.xs0 + L.dX * dist, L.ys0 + L.dY * dist, in && L.kind != LEAF_FAILED, bx, by);
      }
    }
    V vv[4];
#pragma unroll
    for (int q = 0; q < 4; q++) vv[q] = buf_load<T>(rs, idx[q] * (uint32_t)sizeof(T));
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const int ic = ic0 + 64 * (h + q);
      const V v = idx[q] != kNoPx ? vv[q] : fillv;
      bool take = (unsigned)ic < (unsigned)lim && (v != nd);
      if (masked) {
        if (take) take = !mask_fast<GSKYHIP_RESAMPLE_NEAREST>(ents, rows, pool, a.mask, e, ic, ir);
      }
      const bool t2 = take && (!fill_mode || c[h + q] == nd);
      c[h + q] = t2 ? v : c[h + q];
    }
  }
}

// The ordered fold of tile row r over the tile's entries in ProcessRasterStack
// order; c[] arrives holding the canvas nodata.
template <typename T, bool MASK>
__device__ __forceinline__ void nn_fold_row(const RenderArgs &a, const EntryD *__restrict__ ents,
                                            const int32_t *__restrict__ ord, int n_entries,
                                            const RowRec *__restrict__ rows, const RowFix *__restrict__ rowfix,
                                            const Leaf *__restrict__ pool,
                                            int ns_out, int r, int xb, int xl, int W, int ncols,
                                            typename VOf<T>::type (&c)[kNnPx]) {
  // FIX off: in a stack the RowFix load is one more dependent latency per
  // entry row before the row record's (C5 0.47 vs 0.435 ms with it,
  // profiles/r04i_ab.jsonl); the fixed-point rows serve the single-entry path
#pragma unroll 1
  for (int k = 0; k < n_entries; k++)
    nn_entry_row<T, MASK, kNnPx, true, false>(a, ents, ents[ord[k]], rows, rowfix, pool, ns_out, r, xb, xl, W, ncols,
                                              c);
}

// utils.Scale + palette / grey of the lane's 8 canvas values (EncodePNG's
// pixel loop through the LDS table s_tab).
template <typename T, int NPX = kNnPx>
__device__ __forceinline__ void nn_rgba(const ScaleK &sk, bool safe, const uint32_t *s_tab,
                                        const typename VOf<T>::type (&c)[NPX], uint32_t (&px)[NPX]) {
  if constexpr (!std::is_same<T, float>::value) {
    if (safe) {
#pragma unroll
      for (int q = 0; q < NPX; q++) px[q] = s_tab[scale_int<T, true>(sk, c[q])];
    } else {
#pragma unroll
      for (int q = 0; q < NPX; q++) px[q] = s_tab[scale_int<T, false>(sk, c[q])];
    }
  } else {
#pragma unroll
    for (int q = 0; q < NPX; q++) px[q] = s_tab[scale_t<T>(sk, c[q]) & 0xFFu];
  }
}

// RPW: rows per wave (a block of 4 waves covers 4 * RPW rows of a 512-column
// block).  Rows are processed one after the other; a row's RGBA stores are
// issued before the next row's gathers (deferring them behind those gathers
// measured 0.6 % slower on C2 and C5, profiles/r03b_ab_nn.jsonl).
// ONE (RGBA, no mask layer): tiles with a single stack entry -- most GetMap
// tiles -- keep the entry's descriptor in scalar registers for all the
// wave's rows and fetch the next row's record while the current row is
// gathered, so no row waits for its record.
template <typename T, bool MASK, bool CANVAS, int RPW, bool ONE = false, bool STAGE = false, bool COOP = false,
          bool WIDE = false>
__global__ __launch_bounds__(256, MASK ? 1 : 8) void render_nn_kernel(RenderArgs a, const EntryD *__restrict__ ents,
                                                                      const int32_t *__restrict__ order,
                                                                      const RowRec *__restrict__ rows,
                                                                      const RowFix *__restrict__ rowfix,
                                                                      const Leaf *__restrict__ pool,
                                                                      const TilePlan *__restrict__ tplans,
                                                                      const gskyhip_tile *__restrict__ tiles,
                                                                      int n_items) {
  using V = typename VOf<T>::type;
  constexpr int kRowsBlk = 4 * RPW;
  __shared__ uint32_t s_tab[256];
  // STAGE (A/B): a row's 512 RGBA words go through the wave's LDS row so
  // they leave as two 16-B-per-lane stores (1 KB contiguous each) instead of
  // eight 4-B ones
  __shared__ __attribute__((aligned(16))) uint32_t s_stage[STAGE ? 4 : 1][STAGE ? kBandCols : 4];

  const int bands_per_tile = (a.max_h + kRowsBlk - 1) / kRowsBlk;
  const int col_blocks = (a.max_w + kBandCols - 1) / kBandCols;
  int item = blockIdx.x;
#ifdef GSKYHIP_AB
  if (a.ab_xcd == 1) {   // A/B: every block of a tile on one XCD (blockIdx % 8), tiles dealt round-robin over the XCDs
    const int per = bands_per_tile * col_blocks;
    const int xcd = blockIdx.x & 7, slot = blockIdx.x >> 3;
    item = ((slot / per) * 8 + xcd) * per + slot % per;
  } else if (a.ab_xcd == 2) {   // A/B: XCD x takes the x-th contiguous eighth of the items (a strip of tiles)
    const int per = (n_items + 7) >> 3;
    item = (int)(blockIdx.x & 7) * per + (int)(blockIdx.x >> 3);
  }
#endif
  if (item >= n_items) return;
  const int t = item / (bands_per_tile * col_blocks);
  const int in_tile = item - t * bands_per_tile * col_blocks;
  // the block's per-tile values in one round of scalar loads, and the
  // palette word in flight beside them, before the first branch on any of
  // them (each dependent load round costs a memory latency per workgroup)
  const int tid = threadIdx.x;
  const int ns_out = a.out_ns[0];
  const TilePlan *tpp = tplans + t;
  const int tp_complex = tpp->complex, n_entries = tpp->n_entries, tp_vt = tpp->vt;
  const bool created = tpp->created[ns_out] != 0;
  const int tp_dtype = tpp->dtype[ns_out];
  const double tp_nodata = tpp->nodata[ns_out];
  const int e0 = tpp->e0;
  const int W = tiles[t].width, H = tiles[t].height, pair_begin = tiles[t].pair_begin;
  uint32_t col = 0;
  if constexpr (!CANVAS) col = a.ramp ? a.ramp[tid] : (0xFF000000u | ((uint32_t)tid * 0x10101u));
  const int band0 = (in_tile / col_blocks) * kRowsBlk;
  const int xb = (in_tile % col_blocks) * kBandCols;
  // every value above loaded before the first branch (asm: the compiler
  // would sink the ones used later past it, one more latency each)
  asm volatile("" ::"s"((int)created), "s"(tp_dtype), "s"(__double_as_longlong(tp_nodata)), "s"(e0));
  // empty tiles: written here; bitwise, so that no branch splits the loads
  if ((tp_complex != 0) | ((n_entries > 0) & (tp_vt != vt_code<T>())) | (band0 >= H) | (xb >= W)) return;
  // ONE: the single entry's descriptor, loaded in the round after the tile's
  // (its index is the tile plan's e0) and before the palette barrier
  const EntryD *e1 = ents + max(e0, 0);
  int e1_yoff = 0, e1_h = 0, e1_xoff = 0, e1_w = 0, e1_ns = 0, e1_bx = 0, e1_by = 0, e1_fill = 0;
  uint32_t e1_nd = 0;
  const void *e1_band = nullptr;
  int64_t e1_row_base = 0;
  if constexpr (ONE && !MASK && !CANVAS) {
    e1_yoff = e1->yoff; e1_h = e1->h; e1_xoff = e1->xoff; e1_w = e1->w; e1_ns = e1->ns;
    e1_bx = e1->band_x; e1_by = e1->band_y; e1_fill = e1->fill_mode; e1_nd = e1->nd.u;
    e1_band = e1->band; e1_row_base = e1->row_base;
    asm volatile("" ::"s"(e1_yoff), "s"(e1_h), "s"(e1_xoff), "s"(e1_w), "s"(e1_ns), "s"(e1_bx), "s"(e1_by),
                 "s"(e1_fill), "s"(e1_nd), "s"(e1_band), "s"(e1_row_base));
  }
  if constexpr (!CANVAS) {   // EncodePNG: utils.Scale 0xFF and canvases never created are transparent
    s_tab[tid] = (created && tid != 255) ? col : 0u;
    __syncthreads();
  }
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const int r0 = band0 + wave * RPW;
  if (r0 >= H) return;

  const V cnod = as_v<T>(go_conv_to(tp_nodata, tp_dtype));
  const int32_t *ord = order + pair_begin;
  const ScaleK sk = make_scale(tp_dtype, tp_nodata, a.sp, false, 0.f, 0.f);
  const bool safe = !std::is_same<T, float>::value && (float)max(sk.clp.i, 0) * sk.sc < 2147483648.0f;
  const int ncols = min(kBandCols, W - xb);     // columns of the block inside the tile
  const bool full = ncols == kBandCols;
  const int xl = xb + lane;                     // tile column of the lane's pixel 0
  uint32_t *rgba_lane = (uint32_t *)(a.rgba + (((int64_t)t * a.max_h) * a.max_w + xl) * 4);

  auto rgba = [&](const V (&c)[kNnPx], uint32_t (&px)[kNnPx]) {
#ifdef GSKYHIP_AB
    if (a.ab_mode == 3) {   // A/B: Scale without the palette's LDS lookup
#pragma unroll
      for (int q = 0; q < kNnPx; q++) px[q] = 0xFF000000u | scale_int<T, false>(sk, c[q]) * 0x10101u;
      return;
    }
    if (a.ab_mode == 4) {   // A/B: neither Scale nor palette
#pragma unroll
      for (int q = 0; q < kNnPx; q++) px[q] = (uint32_t)c[q];
      return;
    }
#endif
    nn_rgba<T>(sk, safe, s_tab, c, px);
  };

  // RGBA stores of row r
  auto store_row = [&](int r, const uint32_t *px, bool full_known = false) {
    uint32_t *dst = rgba_lane + (int64_t)r * a.max_w;
    if constexpr (STAGE && !CANVAS) {
      if (full && (a.max_w & 3) == 0) {
        uint32_t *row = s_stage[wave];
#pragma unroll
        for (int q = 0; q < kNnPx; q++) row[lane + 64 * q] = px[q];
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const u32x4 v0 = *(const u32x4 *)&row[4 * lane], v1 = *(const u32x4 *)&row[256 + 4 * lane];
        uint32_t *d0 = dst - lane;   // the block's first column of row r
        __builtin_nontemporal_store(v0, (GPTR(u32x4))(d0 + 4 * lane));
        __builtin_nontemporal_store(v1, (GPTR(u32x4))(d0 + 256 + 4 * lane));
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        return;
      }
    }
    auto st = [&](uint32_t *p, uint32_t v) {
#ifdef GSKYHIP_AB
      // A/B: the store's L2 policy (nt / plain keep the line in the XCD's
      // L2; sc1 / sc0 sc1 drop it, MI355X_MICROARCH.md)
      if (a.st_pol == 1) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); return; }
      if (a.st_pol == 2) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM); return; }
      if (a.st_pol == 3) { *p = v; return; }
#endif
      __builtin_nontemporal_store(v, (GPTR(uint32_t))p);
    };
#ifdef GSKYHIP_AB
    if (a.ab_mode == 2) {   // A/B: no stores (the values stay live)
#pragma unroll
      for (int q = 0; q < kNnPx; q++)
        if (px[q] == 0x9E3779B9u) st(dst + 64 * q, px[q]);
      return;
    }
#endif
    if (full_known || full) {
#pragma unroll
      for (int q = 0; q < kNnPx; q++) st(dst + 64 * q, px[q]);
    } else {
#pragma unroll
      for (int q = 0; q < kNnPx; q++)
        if (64 * q + lane < ncols) st(dst + 64 * q, px[q]);
    }
  };

  if constexpr (ONE && !MASK && !CANVAS) {
    if (n_entries == 1) {
      const EntryD &e = *e1;   // the fp64 fallback rows read the rest of it
      const int eyoff = e1_yoff, eh = e1_h, exoff = e1_xoff, ew = e1_w;
      const int lim = max(0, min(ew, W - exoff));
      const int c0 = exoff - xb, c1 = exoff + lim - xb;
      const bool cols_ok = e1_ns == ns_out && ew > 0 && c1 > 0 && c0 < ncols;
      const bool cover = c0 <= 0 && c1 >= ncols;
      const int bx = e1_bx, by = e1_by;
      Val ndv;
      ndv.u = e1_nd;
      const V nd = as_v<T>(ndv);
      const bool fill_mode = e1_fill != 0;
      const int ic0 = xl - exoff;
      bool pair_on = false;   // A/B: nn_fix_row_pair (column pairs, 8-byte stores)
#ifdef GSKYHIP_AB
      pair_on = a.nn_pair != 0 && (a.max_w & 1) == 0;
#endif
      // WIDE / pairs: the band's last dword whole (buf_load_w; a dword never
      // straddles a page)
      const int64_t band_bytes = (int64_t)bx * by * (int64_t)sizeof(T);
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
          (void *)uniform_ptr(e1_band), (short)0,
          (int)((WIDE || pair_on) ? (band_bytes + 3) & ~(int64_t)3 : band_bytes), 0x00020000);
      const RowFix *fbase = rowfix + e1_row_base;
      // the row's fixed-point form, or fk = -1 outside the window / 0 none
      auto fetch = [&](int ir, int64_t (&f)[4], int &fk) {
        if (ir < 0 || ir >= eh) { fk = -1; return; }
        const RowFix *p = fbase + ir;
        f[0] = uni64(p->x0); f[1] = uni64(p->y0); f[2] = uni64(p->dx); f[3] = uni64(p->dy);
        fk = f[0] != kFixNone ? 1 : 0;
      };
      int64_t cf[4] = {0, 0, 0, 0}, nf[4] = {0, 0, 0, 0};
      int cfk = -1, nfk = -1;
      // rows left to the fp64 bodies (no fixed form, or a pixel near a
      // truncation boundary): done in a second loop, so that loop's loads do
      // not reach the register and wait-count state of this one
      uint32_t redo = 0;
      // VFETCH: the RowFix records of all RPW rows in one coalesced vector
      // load (lane 4j + k: field k of row j), read out per row with
      // v_readlane -- one memory latency per wave instead of one per row
      // (the scalar fetch of the next row is still in flight when a row's
      // stores are issued)
      bool vfetch = RPW <= 16;
#ifdef GSKYHIP_AB
      vfetch = vfetch && a.ab_vfetch;
#endif
      int64_t fv = kFixNone;
      if (vfetch) {
        const int jj = lane >> 2, kk = lane & 3, ir = r0 - eyoff + jj;
        if (cols_ok && lane < 4 * RPW && ir >= 0 && ir < eh)
          fv = __builtin_nontemporal_load((const int64_t *)(fbase + ir) + kk);
      } else if (cols_ok) {
        fetch(r0 - eyoff, cf, cfk);
      }
      // the row loop, once for blocks whose every row the entry's window
      // covers in a full-width block (CF: the fast fold and unconditional
      // stores as straight-line code -- merged with the window-edge and
      // ragged-block forms, the compiler predicated every pixel on spilled
      // per-pixel masks) and once for the rest
      auto row_loop = [&](auto cf_tag) {
        constexpr bool CF = decltype(cf_tag)::value;
#pragma unroll 1
        for (int j = 0; j < RPW; j++) {
          const int r = r0 + j;
          if (r >= H) break;
          if (vfetch) {
            const int ir = r - eyoff;
            if (!cols_ok || ir < 0 || ir >= eh) {
              cfk = -1;
            } else {
#pragma unroll
              for (int k = 0; k < 4; k++) {
                const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)fv, 4 * j + k);
                const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)((uint64_t)fv >> 32), 4 * j + k);
                cf[k] = (int64_t)(((uint64_t)hi << 32) | lo);
              }
              cfk = cf[0] != kFixNone ? 1 : 0;
            }
          } else if (cols_ok && j + 1 < RPW) {
            fetch(r + 1 - eyoff, nf, nfk);   // next row's record, in flight now
          }
          V c[kNnPx];
#pragma unroll
          for (int q = 0; q < kNnPx; q++) c[q] = cnod;
          bool done = cfk < 0;
          bool paired = false;
#ifdef GSKYHIP_AB
          if (a.ab_mode == 1) done = true;   // A/B: no gathers
          else if (a.ab_mode == 8 && cfk == 1) {
            // A/B lower bound: the same number of gathers, fold, Scale,
            // palette and stores, with near-free index math -- an unrotated
            // 0.47 source px per output px pattern from the row's first pixel
            const uint32_t ix0 = (uint32_t)(cf[0] >> 32), iy0 = (uint32_t)(cf[1] >> 32);
            const uint32_t rb = (__umul24(iy0, (uint32_t)bx) + ix0) * (uint32_t)sizeof(T);
            V vv[kNnPx];
#pragma unroll
            for (int q = 0; q < kNnPx; q++)
              vv[q] = buf_load<T>(rs, rb + (((uint32_t)(lane + 64 * q) * 15u) >> 5) * (uint32_t)sizeof(T));
#pragma unroll
            for (int q = 0; q < kNnPx; q++) c[q] = vv[q] != nd ? vv[q] : c[q];
            done = true;
          } else
#endif
          if (cfk == 1) {
            if constexpr (CF && sizeof(T) == 2 && !WIDE) {
              if (pair_on) {
                done = nn_fix_row_pair<T, kNnPx>(rs, cf[0], cf[1], cf[2], cf[3], ic0 + lane, bx, nd, fill_mode, c);
                paired = true;
              } else {
                done = nn_fix_row<T, kNnPx, false, WIDE>(rs, cf[0], cf[1], cf[2], cf[3], ic0, lim, bx, nd, fill_mode,
                                                         c);
              }
            } else if constexpr (CF)
              done = nn_fix_row<T, kNnPx, false, WIDE>(rs, cf[0], cf[1], cf[2], cf[3], ic0, lim, bx, nd, fill_mode, c);
            else
              done = cover ? (COOP ? nn_fix_row_coop<T, kNnPx>(rs, cf[0], cf[1], cf[2], cf[3], ic0, lim, bx, nd,
                                                               fill_mode, c, lane)
                                   : nn_fix_row<T, kNnPx, false, WIDE>(rs, cf[0], cf[1], cf[2], cf[3], ic0, lim, bx, nd,
                                                                       fill_mode, c))
                           : nn_fix_row<T, kNnPx, true, WIDE>(rs, cf[0], cf[1], cf[2], cf[3], ic0, lim, bx, nd,
                                                              fill_mode, c);
          }
          if (done) {
            uint32_t px[kNnPx];
            rgba(c, px);
            if (paired) {   // columns 2 lane + 128 q + {0, 1}: 8-byte stores
              uint32_t *d = rgba_lane - lane + (int64_t)r * a.max_w + 2 * lane;
#pragma unroll
              for (int q = 0; q < kNnPx / 2; q++)
                __builtin_nontemporal_store(u32x2{px[2 * q], px[2 * q + 1]}, (GPTR(u32x2))(d + 128 * q));
            } else {
              store_row(r, px, CF);
            }
          } else {
            redo |= 1u << j;
          }
          if (!vfetch) {
#pragma unroll
            for (int k = 0; k < 4; k++) cf[k] = nf[k];
            cfk = nfk;
          }
        }
      };
      bool cf_on = cover && full && !COOP;
#ifdef GSKYHIP_AB
      if (a.ab_mode == 7) cf_on = false;   // A/B: one merged row loop (round 4)
#endif
      // COLG (A/B build, GSKYHIP_NN_COLG=1; measured slower): the block's 8
      // rows x 512 columns in column-group-major order -- for each 64-column
      // group the wave's RPW rows back to back, so the RPW gathers in flight
      // read the few source lines under that group.  Row-major, L1 -> L2
      // reads are 7x the unique source bytes (32 waves per CU evict a wave's
      // lines before its next row); this order halves them (57.4 M -> 31.5 M
      // requests) and still runs 1.64 vs 1.57 ms: the texture data unit stays
      // busy ~97 % of the kernel at ~21 L1 accesses per 64-lane gather
      // (profiles/r05j_pmc_c2_l1.json, r05k_*).  The same fixed-point values
      // and margin test as nn_fix_row, the same fp64 redo of a row with an
      // ambiguous pixel: the same result bit for bit (0 px differ on C2, C5).
      bool colg_done = false;
#ifdef GSKYHIP_AB
      if constexpr (RPW == kNnPx && !COOP && !WIDE) {
        bool colg = a.nn_colg && cf_on && vfetch && r0 + RPW <= H && r0 - eyoff >= 0 && r0 + RPW - eyoff <= eh;
        if (colg) {
          const bool missing = lane < 4 * RPW && (lane & 3) == 0 && fv == kFixNone;
          colg = __builtin_amdgcn_ballot_w64(missing) == 0;
        }
        if (colg) {
          colg_done = true;
          uint32_t amb = 0;   // per lane: bit j = row j has an ambiguous pixel
          uint32_t *const dst0 = rgba_lane + (int64_t)r0 * a.max_w;
#pragma unroll 1
          for (int g = 0; g < kNnPx; g++) {
            // the row records come by scalar loads each group (held across the
            // loop they would be 64 SGPRs)
            int jb = r0 - eyoff;
            asm volatile("" : "+s"(jb));   // (the index, not the pointer: that keeps its address space)
            const RowFix *rb = fbase + jb;
            const uint32_t ic = (uint32_t)(ic0 + 64 * g);
            uint32_t off[RPW];
#pragma unroll
            for (int j = 0; j < RPW; j++) {
              const uint64_t x0 = (uint64_t)uni64(rb[j].x0), y0 = (uint64_t)uni64(rb[j].y0);
              const uint64_t dx = (uint64_t)uni64(rb[j].dx), dy = (uint64_t)uni64(rb[j].dy);
              const uint64_t X = x0 + (uint64_t)ic * dx, Y = y0 + (uint64_t)ic * dy;
              const uint32_t m = min((uint32_t)X + kFixMargin, (uint32_t)Y + kFixMargin);
              amb |= (m < 2u * kFixMargin ? 1u : 0u) << j;
              off[j] = (__umul24((uint32_t)(Y >> 32), (uint32_t)bx) + (uint32_t)(X >> 32)) * (uint32_t)sizeof(T);
            }
            V vv[RPW];
#pragma unroll
            for (int j = 0; j < RPW; j++) vv[j] = buf_load<T>(rs, off[j]);
            V c[RPW];
            if (!fill_mode) {
#pragma unroll
              for (int j = 0; j < RPW; j++) c[j] = vv[j] != nd ? vv[j] : cnod;
            } else {
              const bool take = cnod == nd;
#pragma unroll
              for (int j = 0; j < RPW; j++) c[j] = take ? vv[j] : cnod;
            }
            uint32_t px[RPW];
            rgba(c, px);
#pragma unroll
            for (int j = 0; j < RPW; j++)
              __builtin_nontemporal_store(px[j], (GPTR(uint32_t))(dst0 + (int64_t)j * a.max_w + 64 * g));
          }
#pragma unroll
          for (int j = 0; j < RPW; j++)
            if (__builtin_amdgcn_ballot_w64((amb >> j) & 1u) != 0) redo |= 1u << j;
        }
      }
#endif
      if (!colg_done) {
        if (cf_on) row_loop(std::true_type{});
        else row_loop(std::false_type{});
      }
#pragma unroll 1
      while (redo) {
        const int j = __builtin_ctz(redo);
        redo &= redo - 1;
        const int r = r0 + j;
        V c[kNnPx];
#pragma unroll
        for (int q = 0; q < kNnPx; q++) c[q] = cnod;
        nn_entry_row<T, false, kNnPx, true, false>(a, ents, e, rows, rowfix, pool, ns_out, r, xb, xl, W, ncols, c);
        uint32_t px[kNnPx];
        rgba(c, px);
        store_row(r, px);
      }
      return;
    }
  }
#pragma unroll 1
  for (int j = 0; j < RPW; j++) {
    const int r = r0 + j;
    if (r >= H) break;
    V c[kNnPx];
#pragma unroll
    for (int q = 0; q < kNnPx; q++) c[q] = cnod;
    nn_fold_row<T, MASK>(a, ents, ord, n_entries, rows, rowfix, pool, ns_out, r, xb, xl, W, ncols, c);

    // output: typed canvas (WCS) or utils.Scale + palette / grey RGBA
    if constexpr (CANVAS) {
      const int64_t eo = a.cov_offsets ? a.cov_offsets[t] + (int64_t)r * a.cov_stride + xl
                                       : (int64_t)r * a.max_w + xl;
      T *cdst = (T *)(a.cov_offsets ? a.canvas : a.canvas + t * a.canvas_tile_stride) + eo;
#pragma unroll
      for (int q = 0; q < kNnPx; q++)
        if (full || 64 * q + lane < ncols) __builtin_nontemporal_store((T)c[q], (GPTR(T))(cdst + 64 * q));
    } else {
      uint32_t px[kNnPx];
      rgba(c, px);
      store_row(r, px);
    }
  }
}

// Rows per wave of the NN band kernel: 8 when the batch has work for every
// CU many times over (C2: 1.473 vs 1.506 ms), else 4 (C5, 80 tiles: 0.66 vs
// 0.86 ms at 8 -- too few blocks); profiles/r03b_ab_nn.jsonl.  Masked and
// canvas batches keep 4 (measured on C5 only).  A/B build: GSKYHIP_NN_RPW.
constexpr int kNnRpw8MinItems = 32768;
constexpr int kNnRpw1MaxItems = 256;   // below one workgroup per CU at 4 rows per wave
constexpr int kNnMaskRpw1Items = 16384;   // masked stacks: one row per wave below this many workgroups

template <typename T, bool M, bool C, int RPW, bool ONE = false, bool STAGE = false, bool COOP = false,
          bool WIDE = false>
void launch_nn_v(const RenderArgs &a, hipStream_t s) {
  const int items = a.n_tiles * ((a.max_h + 4 * RPW - 1) / (4 * RPW)) * ((a.max_w + kBandCols - 1) / kBandCols);
  // the XCD order (A/B) maps blocks over whole groups of 8 tiles: round the grid up
  const int per = ((a.max_h + 4 * RPW - 1) / (4 * RPW)) * ((a.max_w + kBandCols - 1) / kBandCols);
  const int grid = a.ab_xcd == 1 ? (a.n_tiles + 7) / 8 * 8 * per : a.ab_xcd == 2 ? (items + 7) / 8 * 8 : items;
  hipLaunchKernelGGL((render_nn_kernel<T, M, C, RPW, ONE, STAGE, COOP, WIDE>), dim3((unsigned)grid), dim3(256), 0, s, a, a.entries,
                     a.order, a.rows, a.rowfix, a.pool, a.tplans, a.tiles, items);
}

// render_nn_stage.h (included by the per-type translation units)
template <typename T> void launch_nn_stage(const RenderArgs &a, hipStream_t s);

// NN band kernel launch for value type T (RGBA or typed canvas, with or
// without a mask layer).
template <typename T>
void launch_nn_t(const RenderArgs &a, bool mask, hipStream_t s) {
  const bool canvas = (a.lds_mode & kCanvas) != 0;
  const int64_t items8 = (int64_t)a.n_tiles * ((a.max_h + 31) / 32) * ((a.max_w + kBandCols - 1) / kBandCols);
  bool rpw8 = items8 >= kNnRpw8MinItems;
  // small batches (C1: one 256^2 tile = 16 blocks at 4 rows per wave) are
  // latency-bound: one row per wave, 4x the workgroups
  const int64_t items4 = (int64_t)a.n_tiles * ((a.max_h + 15) / 16) * ((a.max_w + kBandCols - 1) / kBandCols);
  bool rpw1 = items4 < kNnRpw1MaxItems;
  // single-entry tiles through the prefetching path (C2: 1.445 vs 1.470 ms,
  // profiles/r03f_ab_c2.jsonl)
  bool one = true;
#ifdef GSKYHIP_AB
  // large RGBA batches through the LDS-staged kernel (render_nn_stage.h): 7 %
  // slower on C2 (1.54 vs 1.44 ms, profiles/r03j_ab_c2_staged.jsonl)
  bool staged = false;
  if (const char *rp = getenv("GSKYHIP_NN_RPW")) {
    rpw8 = atoi(rp) == 8; rpw1 = atoi(rp) == 1;
    if (atoi(rp) == 16 && !mask && !canvas && one) { launch_nn_v<T, false, false, 16, true>(a, s); return; }
  }
  if (const char *on = getenv("GSKYHIP_NN_ONE")) one = atoi(on) != 0;
  if (const char *sg = getenv("GSKYHIP_NN_STAGED")) staged = atoi(sg) != 0;
  if (const char *st = getenv("GSKYHIP_NN_STAGE")) {
    if (!mask && !canvas && rpw8 && atoi(st) == 1) {
      if (one) launch_nn_v<T, false, false, 8, true, true>(a, s);
      else launch_nn_v<T, false, false, 8, false, true>(a, s);
      return;
    }
  }
#endif
  if (mask) {
    // stacks with a mask layer (C5: ~17 entries and a mask raster per tile)
    // are latency-bound per wave row: below kNnMaskRpw1Items workgroups, one
    // row per wave (4x the waves in flight)
    bool m1 = items4 < kNnMaskRpw1Items;
#ifdef GSKYHIP_AB
    if (const char *rp = getenv("GSKYHIP_NN_MASK_RPW")) m1 = atoi(rp) == 1;
#endif
    if (canvas) launch_nn_v<T, true, true, 4>(a, s);
    else if (m1) launch_nn_v<T, true, false, 1>(a, s);
    else launch_nn_v<T, true, false, 4>(a, s);
  } else if (canvas) {
    launch_nn_v<T, false, true, 4>(a, s);
#ifdef GSKYHIP_AB
  } else if (rpw8 && staged) {
    launch_nn_stage<T>(a, s);
#endif
  } else if (rpw8) {
#ifdef GSKYHIP_AB
    if (const char *co = getenv("GSKYHIP_NN_COOP")) {
      if (one && atoi(co) != 0) { launch_nn_v<T, false, false, 8, true, false, true>(a, s); return; }
    }
    if (const char *wd = getenv("GSKYHIP_NN_WIDE")) {
      if (one && atoi(wd) != 0) { launch_nn_v<T, false, false, 8, true, false, false, true>(a, s); return; }
    }
#endif
    if (one) launch_nn_v<T, false, false, 8, true>(a, s);
    else launch_nn_v<T, false, false, 8>(a, s);
  } else if (rpw1) {
    launch_nn_v<T, false, false, 1>(a, s);
  } else {
    launch_nn_v<T, false, false, 4>(a, s);
  }
}

void launch_bil(const RenderArgs &a, int n_items, hipStream_t s);   // render_bil.h, render_lds_f32.hip

// Band kernel of one call: bilinear float canvases without a mask layer ->
// render_bil_kernel; other bilinear work -> render_lds_kernel; nearest
// neighbour -> render_nn_kernel.
template <typename T>
void launch_band_t(const RenderArgs &a, bool mask, int n_items, hipStream_t s) {
  if ((a.lds_mode & kBilinear) != 0) {
    if constexpr (std::is_same<T, float>::value) {
      if (!mask && (a.lds_mode & kCanvas)) {
        launch_bil(a, n_items, s);
        return;
      }
    }
    launch_lds_t<T>(a, mask, n_items, s);
    return;
  }
  launch_nn_t<T>(a, mask, s);
}

}  // namespace gsky
