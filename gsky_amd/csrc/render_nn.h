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
//     leaves, failed transforms) takes the general body with the per-pixel
//     tests of the reference;
//   * stacks (round 6): an entry in fill mode whose block row holds no pixel
//     its nodata could fill is skipped before its row record is read; an
//     entry with a mask layer whose mask row picks the same source element
//     (C5's QA granules) gathers data and mask from one index, a 64-column
//     slot only where some lane can still change; masked stacks prefetch
//     every entry's descriptor, row record and mask row in one round of
//     vector loads (nn_fold_row_stack) instead of the serial scalar chain;
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
// The window is [wlo, whi) (wlo 0 and whi the window width, or a row's
// in-band span).
template <typename T, int NPX>
__device__ __forceinline__ void nn_partial_row(__amdgpu_buffer_rsrc_t rs, double xs0, double ys0, double dX, double dY,
                                               int ic0, int wlo, int whi, int bx, typename VOf<T>::type nd,
                                               bool fill_mode, typename VOf<T>::type (&c)[NPX]) {
  using V = typename VOf<T>::type;
  const unsigned wn = (unsigned)(whi - wlo);
#pragma unroll
  for (int h = 0; h < NPX; h += 4) {
    uint32_t off[4];
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const int ic = ic0 + 64 * (h + q);
      const double dist = (double)ic;
      const int ix = __double2int_rz(xs0 + dX * dist + 1.0e-10);
      const int iy = __double2int_rz(ys0 + dY * dist + 1.0e-10);
      off[q] = (unsigned)(ic - wlo) < wn ? (__umul24((uint32_t)iy, (uint32_t)bx) + (uint32_t)ix) * (uint32_t)sizeof(T)
                                         : 0x80000000u;
    }
    V vv[4];
#pragma unroll
    for (int q = 0; q < 4; q++) vv[q] = buf_load<T>(rs, off[q]);
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const bool inw = (unsigned)(ic0 + 64 * (h + q) - wlo) < wn;
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
template <typename T, int NPX, bool PART>
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
  for (int q = 0; q < NPX; q++) vv[q] = buf_load<T>(rs, off[q]);
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

// The fold of one LINEAR row of an entry carrying a mask layer whose mask row
// picks the same source element (C5's QA stacks: the QA granule shares the
// data granule's grid, picked level and window, so the planner gives both
// pairs the same row record): each window pixel's element index once, the
// data and mask gathers from it side by side, and only for 64-column slots
// where some lane can still change -- in fill mode (tile_merger.go:47-58) a
// pixel whose canvas no longer holds this raster's nodata can take nothing,
// so a slot with no such lane issues neither gather.  The same rule per
// pixel as the general body + mask_fast(): in window, v != nodata, not
// masked (ComputeMask, tile_merger.go:314-445), and in fill mode canvas ==
// nodata; a pixel whose element is outside the band takes the window fill
// and the mask's fill (warp.go:246-247), as nn_fetch() does.
template <typename T, int NPX, bool M8>
__device__ __forceinline__ void nn_masked_same_row(const MaskSpecS &ms, int mdt, int32_t mfill,
                                                   __amdgpu_buffer_rsrc_t rs, __amdgpu_buffer_rsrc_t mrs,
                                                   double xs0, double ys0, double dX, double dY, int ic0, int lim,
                                                   int bx, int by, typename VOf<T>::type nd,
                                                   typename VOf<T>::type fillv, bool fill_mode,
                                                   typename VOf<T>::type (&c)[NPX]) {
  using V = typename VOf<T>::type;
#pragma unroll
  for (int h = 0; h < NPX; h += 4) {
    uint32_t idx[4];
    bool need[4];
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const int ic = ic0 + 64 * (h + q);
      const double dist = (double)ic;
      const bool inw = (unsigned)ic < (unsigned)lim;
      idx[q] = nn_index_sxy(xs0 + dX * dist, ys0 + dY * dist, inw, bx, by);
      need[q] = inw & (!fill_mode | (c[h + q] == nd));
    }
    V vv[4];
    uint32_t mraw[4];
#pragma unroll
    for (int q = 0; q < 4; q++) {
      vv[q] = 0;
      mraw[q] = 0;
      if (__builtin_amdgcn_ballot_w64(need[q]) != 0) {
        // kNoPx reads nothing: its offset is past every band (range-checked)
        vv[q] = buf_load<T>(rs, idx[q] * (uint32_t)sizeof(T));
        mraw[q] = M8 ? (uint32_t)__builtin_amdgcn_raw_buffer_load_b8(mrs, idx[q], 0, 0)
                     : (uint32_t)__builtin_amdgcn_raw_buffer_load_b16(mrs, idx[q] * 2u, 0, 0);
      }
    }
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const bool hit = idx[q] != kNoPx;
      const V v = hit ? vv[q] : fillv;
      // nn_fetch<mask type>'s value; the pixel's take rule bitwise (a
      // short-circuit && put an exec-mask branch around each pixel's test)
      const int32_t mv = hit ? mask_typed(mdt, (int32_t)mraw[q]) : mfill;
      const bool take = need[q] & (v != nd) & !mask_bit(ms, mdt, mv);
      c[h + q] = take ? v : c[h + q];
    }
  }
}

// One stack entry's render descriptor (EntryD) and its row record (RowRec)
// for one tile row, as wave-uniform values: loaded from memory by
// nn_entry_row(), or read out of a wave's prefetched lanes by
// nn_fold_row_stack().
struct EntryU {
  const void *band;
  int64_t row_base;
  int bx, by, xoff, yoff, w, h, ns, fill_mode, mask_pair;
  uint32_t nd, fill;
};
struct RowU {
  double v[4];
  int kind, inside, nleaf, pool_off;
};
// the mask pair of a masked entry on this row: its window width / height,
// level size, type, fill, band and the row record's kind + LINEAR values
struct MaskU {
  const void *band;
  double v[4];
  int w, h, bx, by, dt, kind;
  int32_t fill;
  int same;   // -1: test v / w / h / bx / by / kind here; 0 / 1: tested where the mask row was read
};

// Where nn_entry_core() takes the row's fixed-point form and record from:
// RowMem reads them from memory at first use (scalar loads of a uniform
// pointer: the fixed-point form first, the record only for the fp64 bodies),
// RowVal holds values read out of a prefetched lane.
struct RowMem {
  const RowRec *rr;
  const RowFix *fp;   // nullptr: no fixed-point form
  __device__ __forceinline__ bool fix(int64_t (&f)[4]) const {
    if (!fp) return false;
    f[0] = uni64(fp->x0);
    if (f[0] == kFixNone) return false;
    f[1] = uni64(fp->y0); f[2] = uni64(fp->dx); f[3] = uni64(fp->dy);
    return true;
  }
  __device__ __forceinline__ int kind() const { return __builtin_amdgcn_readfirstlane(rr->kind); }
  __device__ __forceinline__ int inside() const { return __builtin_amdgcn_readfirstlane(rr->inside); }
  __device__ __forceinline__ int nleaf() const { return __builtin_amdgcn_readfirstlane(rr->nleaf); }
  __device__ __forceinline__ int pool_off() const { return __builtin_amdgcn_readfirstlane(rr->pool_off); }
  __device__ __forceinline__ double v(int k) const { return rr->v[k]; }
  __device__ __forceinline__ int64_t span() const { return uni64(__double_as_longlong(rr->v[4])); }
};
struct RowVal {
  RowU ru;
  RowFix fx;
  __device__ __forceinline__ bool fix(int64_t (&f)[4]) const {
    f[0] = fx.x0; f[1] = fx.y0; f[2] = fx.dx; f[3] = fx.dy;
    return fx.x0 != kFixNone;
  }
  __device__ __forceinline__ int kind() const { return ru.kind; }
  __device__ __forceinline__ int inside() const { return ru.inside; }
  __device__ __forceinline__ int nleaf() const { return ru.nleaf; }
  __device__ __forceinline__ int pool_off() const { return ru.pool_off; }
  __device__ __forceinline__ double v(int k) const { return ru.v[k]; }
  // the prefetching fold drops empty spans from its walk; no span here
  __device__ __forceinline__ int64_t span() const { return kSpanNone; }
};

__device__ __forceinline__ EntryU entry_u(const EntryD &e) {
  EntryU u;
  u.band = uniform_ptr(e.band);
  u.row_base = uni64(e.row_base);
  u.bx = e.band_x; u.by = e.band_y; u.xoff = e.xoff; u.yoff = e.yoff; u.w = e.w; u.h = e.h;
  u.ns = e.ns; u.fill_mode = e.fill_mode; u.mask_pair = e.mask_pair; u.nd = e.nd.u; u.fill = e.fill.u;
  return u;
}

// One stack entry of the ordered fold of tile row r (MergeMaskedRaster,
// tile_merger.go:38-225): c[q] is the canvas value of the lane's pixel q
// (tile column xl + 64 q).  fix: the row's 32.32 fixed-point form (RowFix,
// x0 == kFixNone: none); mu: the mask pair's row when the entry is masked and
// the mask row was prefetched (else mask_fast() reads it per pixel).
template <typename T, bool MASK, int NPX, typename RS, bool SKIP = true>
__device__ __forceinline__ void nn_entry_core(const RenderArgs &a, const EntryD *__restrict__ ents,
                                              const RowRec *__restrict__ rows, const Leaf *__restrict__ pool,
                                              const EntryU &e, const RS &ru, const MaskU *mu,
                                              int r, int xb, int xl, int W, int ncols,
                                              typename VOf<T>::type (&c)[NPX]) {
  using V = typename VOf<T>::type;
  const int ir = r - e.yoff, ew = e.w;
  const int lim = max(0, min(ew, W - e.xoff));   // window pixel in the tile: (unsigned)ic < lim
  const int c0 = e.xoff - xb, c1 = e.xoff + lim - xb;   // the entry's columns of the block: [c0, c1)
  const int bx = e.bx, by = e.by;
  Val ndv;
  ndv.u = e.nd;
  const V nd = as_v<T>(ndv);
  const bool fill_mode = e.fill_mode != 0;
  const int ic0 = xl - e.xoff;   // window column of the lane's pixel 0
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
      (void *)e.band, (short)0, (int)((int64_t)bx * by * (int64_t)sizeof(T)), 0x00020000);
  const bool masked = MASK && e.mask_pair >= 0;
  // fill mode: only pixels whose canvas still holds this raster's nodata can
  // change (tile_merger.go:47-58); a row of the block with none skips the
  // entry's gathers (a NaN nodata never compares equal: such an entry never
  // fills, as in the reference)
  if (SKIP && fill_mode) {
    bool any = false;
#pragma unroll
    for (int q = 0; q < NPX; q++) any |= c[q] == nd;
    if (__builtin_amdgcn_ballot_w64(any) == 0) return;
  }
  const bool cover = c0 <= 0 && c1 >= ncols;
  int64_t f[4];
  if (!masked && ru.fix(f)) {   // fixed-point form of an `inside` LINEAR row
    const bool done = cover ? nn_fix_row<T, NPX, false>(rs, f[0], f[1], f[2], f[3], ic0, lim, bx, nd, fill_mode, c)
                            : nn_fix_row<T, NPX, true>(rs, f[0], f[1], f[2], f[3], ic0, lim, bx, nd, fill_mode, c);
    if (done) return;
  }
  const int kind = ru.kind();
  const int inside = ru.inside();
  if (kind == ROW_LINEAR && inside && cover && !masked) {
    // fast body: every pixel of the block is in the window and its source
    // pixel in the band -- lin_coords() + nn_px() reduce to the truncations
    const double xs0 = ru.v(0), ys0 = ru.v(1), dX = ru.v(2), dY = ru.v(3);
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
  if (kind == ROW_LINEAR && inside && !masked) {
    // window edge inside the block on an `inside` row: the fast body plus the
    // window test (pixels outside the window read nothing and fold nothing;
    // fill mode takes v where c is nodata, which equals the general rule's
    // "v != nd && c == nd" because v == nd == c leaves c unchanged)
    nn_partial_row<T, NPX>(rs, ru.v(0), ru.v(1), ru.v(2), ru.v(3), ic0, 0, lim, bx, nd, fill_mode, c);
    return;
  }
  if (kind == ROW_LINEAR && !masked && e.fill == e.nd && !(nd != nd)) {
    // a row leaving the band (granule seams, bounding-box window corners):
    // outside its in-band span every pixel takes the window fill, which is
    // the nodata here and folds nothing (v == nd in either mode; a NaN
    // nodata would fold), so the row is a window edge row over the span
    const int64_t sp = ru.span();
    if (sp != kSpanNone) {
      const int lo = (int)(uint32_t)sp, hi = min((int)(sp >> 32), lim);
      const int s0 = e.xoff + lo - xb, s1 = e.xoff + hi - xb;   // the span's columns of the block
      if (hi <= lo || s1 <= 0 || s0 >= ncols) return;
      nn_partial_row<T, NPX>(rs, ru.v(0), ru.v(1), ru.v(2), ru.v(3), ic0, lo, hi, bx, nd, fill_mode, c);
      return;
    }
  }
  Val fv;
  fv.u = e.fill;
  const V fillv = as_v<T>(fv);
  if constexpr (MASK) {
    if (masked && kind == ROW_LINEAR) {
      // the mask pair's row: the same element index when it has the data
      // row's width, level size and row record (bit for bit)
      MaskU m;
      if (mu) {
        m = *mu;
      } else {
        const EntryD &me = ents[e.mask_pair];
        m.w = me.w; m.h = me.h; m.bx = me.band_x; m.by = me.band_y; m.dt = me.out_dtype; m.fill = me.fill.i;
        m.band = uniform_ptr(me.band);
        m.kind = -1;
        m.same = -1;
        if (ir < m.h) {
          const RowRec &mr = rows[uni64(me.row_base) + ir];
          m.kind = __builtin_amdgcn_readfirstlane(mr.kind);
#pragma unroll
          for (int k = 0; k < 4; k++) m.v[k] = uni64d(mr.v[k]);
        }
      }
      const int slot = mask_slot(m.dt);
      const bool same = m.same >= 0 ? m.same != 0
                                    : m.w == ew && ir < m.h && m.bx == bx && m.by == by && m.kind == ROW_LINEAR &&
                                          __double_as_longlong(m.v[0]) == __double_as_longlong(ru.v(0)) &&
                                          __double_as_longlong(m.v[1]) == __double_as_longlong(ru.v(1)) &&
                                          __double_as_longlong(m.v[2]) == __double_as_longlong(ru.v(2)) &&
                                          __double_as_longlong(m.v[3]) == __double_as_longlong(ru.v(3));
      if (same && slot >= 0) {
        const __amdgpu_buffer_rsrc_t mrs = __builtin_amdgcn_make_buffer_rsrc(
            (void *)m.band, (short)0, (int)((int64_t)m.bx * m.by * (int64_t)type_size(m.dt)), 0x00020000);
        // the mask's element width chosen once per entry row (per pixel, the
        // compiler branched on the type around every mask gather)
        if (m.dt == GSKYHIP_BYTE || m.dt == GSKYHIP_SIGNEDBYTE)
          nn_masked_same_row<T, NPX, true>(a.mask[slot], m.dt, m.fill, rs, mrs, ru.v(0), ru.v(1), ru.v(2), ru.v(3), ic0,
                                           lim, bx, by, nd, fillv, fill_mode, c);
        else
          nn_masked_same_row<T, NPX, false>(a.mask[slot], m.dt, m.fill, rs, mrs, ru.v(0), ru.v(1), ru.v(2), ru.v(3), ic0,
                                            lim, bx, by, nd, fillv, fill_mode, c);
        return;
      }
    }
  }
  // general body: POOL rows, rows not inside the band, mask layer;
  // two halves of 4 pixels (4 gathers in flight) keep the register peak
  // of the fast body
#pragma unroll
  for (int h = 0; h < NPX; h += 4) {
    uint32_t idx[4];
    if (kind == ROW_LINEAR) {
      const double xs0 = ru.v(0), ys0 = ru.v(1), dX = ru.v(2), dY = ru.v(3);
#pragma unroll
      for (int q = 0; q < 4; q++) {
        const int ic = ic0 + 64 * (h + q);
        const double dist = (double)ic;
        idx[q] = nn_index_sxy(xs0 + dX * dist, ys0 + dY * dist, (unsigned)ic < (unsigned)lim, bx, by);
      }
    } else {   // POOL (the only other kind of a simple tile): the leaf of each pixel
      const int nleaf = ru.nleaf();
      const Leaf *lv = pool + ru.pool_off();
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
        if (take) take = !mask_fast_pair<GSKYHIP_RESAMPLE_NEAREST>(ents, rows, pool, a.mask, e.mask_pair, ew, ic, ir);
      }
      const bool t2 = take && (!fill_mode || c[h + q] == nd);
      c[h + q] = t2 ? v : c[h + q];
    }
  }
}

// nn_entry_core() of entry e on tile row r, its descriptor and row records
// read from memory (the single-entry path's fp64 redo rows).
template <typename T, bool MASK, int NPX = kNnPx, bool SKIP = true>
__device__ __forceinline__ void nn_entry_row(const RenderArgs &a, const EntryD *__restrict__ ents, const EntryD &e,
                                             const RowRec *__restrict__ rows, const RowFix *__restrict__ rowfix,
                                             const Leaf *__restrict__ pool, bool use_fix,
                                             int ns_out, int r, int xb, int xl, int W, int ncols,
                                             typename VOf<T>::type (&c)[NPX]) {
  const EntryU u = entry_u(e);
  if (u.ns != ns_out || u.w <= 0) return;
  const int ir = r - u.yoff;
  if (ir < 0 || ir >= u.h) return;
  const int lim = max(0, min(u.w, W - u.xoff));
  const int c0 = u.xoff - xb, c1 = u.xoff + lim - xb;
  if (c1 <= 0 || c0 >= ncols) return;
  RowMem rm;
  rm.rr = rows + u.row_base + ir;
  rm.fp = use_fix ? rowfix + u.row_base + ir : nullptr;
  nn_entry_core<T, MASK, NPX, RowMem, SKIP>(a, ents, rows, pool, u, rm, nullptr, r, xb, xl, W, ncols, c);
}

// The ordered fold of tile row r over the tile's entries in
// ProcessRasterStack order (tile_merger.go:281-312); c[] arrives holding the
// canvas nodata.  Entries are taken 64 at a time, lane j holding entry
// k0 + j: one round of vector loads reads every entry's window and, for the
// entries that touch this row of the block, the row record, the fixed-point
// form and (masked stacks) the mask pair's descriptor and row -- the
// dependent scalar chain order -> descriptor -> row -> mask -> mask row of
// the serial walk costs four memory latencies per entry; here about four per
// 64 entries.  The fold then walks the active entries in order, each one's
// values read out of its lane.
template <typename T, bool MASK>
__device__ __forceinline__ void nn_fold_row_stack(const RenderArgs &a, const EntryD *__restrict__ ents,
                                                  const int32_t *__restrict__ ord, int n_entries,
                                                  const RowRec *__restrict__ rows, const RowFix *__restrict__ rowfix,
                                                  const Leaf *__restrict__ pool, int ns_out, int r, int xb, int xl,
                                                  int W, int ncols, int lane, typename VOf<T>::type (&c)[kNnPx]) {
#pragma unroll 1
  for (int k0 = 0; k0 < n_entries; k0 += 64) {
    const bool has = k0 + lane < n_entries;
    const int p = has ? ord[k0 + lane] : 0;
    const EntryD &E = ents[p];
    const int yoff = E.yoff, eh = E.h, xoff = E.xoff, ew = E.w, ens = E.ns;
    const int ir = r - yoff;
    const int lim = max(0, min(ew, W - xoff));
    const int c0 = xoff - xb, c1 = xoff + lim - xb;
    const bool act = has & (ens == ns_out) & (ew > 0) & (ir >= 0) & (ir < eh) & (c1 > 0) & (c0 < ncols);
    uint64_t am = __builtin_amdgcn_ballot_w64(act);
    if (am == 0) continue;
    // the active lanes' descriptors, row records (and mask rows), in flight together
    const int64_t rb = act ? E.row_base + ir : 0;
    const RowRec &R = rows[rb];
    const double v0 = R.v[0], v1 = R.v[1], v2 = R.v[2], v3 = R.v[3];
    const int kind = R.kind, inside = R.inside, nleaf = R.nleaf, pool_off = R.pool_off;
    const void *band = E.band;
    const int bx = E.band_x, by = E.band_y, fill_mode = E.fill_mode, mask_pair = E.mask_pair;
    const uint32_t nd = E.nd.u, fill = E.fill.u;
    {
      // a LINEAR row whose in-band span misses the block's columns folds
      // nothing when the window fill is the (non-NaN) nodata: off the walk
      const int64_t sp = __double_as_longlong(R.v[4]);
      const int slo = (int)(uint32_t)sp, shi = min((int)(sp >> 32), lim);
      Val ndv;
      ndv.u = nd;
      const typename VOf<T>::type ndt = as_v<T>(ndv);
      const bool empty = (kind == ROW_LINEAR) & (inside == 0) & (fill == nd) & (ndt == ndt) & (sp != kSpanNone) &
                         ((shi <= slo) | (xoff + shi - xb <= 0) | (xoff + slo - xb >= ncols));
      am &= __builtin_amdgcn_ballot_w64(!empty);
    }
    int64_t fx0 = kFixNone, fy0 = 0, fdx = 0, fdy = 0;
    int mdt = 0;
    int32_t mfill = 0;
    const void *mband = nullptr;
    uint64_t msame = 0;   // entries whose mask row picks the data row's elements (nn_masked_same_row)
    if constexpr (!MASK) {
      const RowFix &F = rowfix[rb];
      fx0 = act ? F.x0 : kFixNone; fy0 = F.y0; fdx = F.dx; fdy = F.dy;
    } else {
      // the mask pair's descriptor and row, tested here against the data
      // row in each lane: only the result, the mask's type, fill and band
      // stay live through the fold (the mask row's values held across it
      // took the kernel to 87 VGPRs, 5 waves per SIMD)
      const bool mk = act & (mask_pair >= 0);
      const EntryD &M = ents[mk ? mask_pair : p];
      const int mw = M.w, mh = M.h, mbx = M.band_x, mby = M.band_y;
      mdt = M.out_dtype; mfill = M.fill.i; mband = M.band;
      const bool mrow = mk & (ir < mh);
      const RowRec &MR = rows[mrow ? M.row_base + ir : 0];
      const bool same = mrow & (mw == ew) & (mbx == bx) & (mby == by) & (MR.kind == ROW_LINEAR) &
                        (__double_as_longlong(MR.v[0]) == __double_as_longlong(v0)) &
                        (__double_as_longlong(MR.v[1]) == __double_as_longlong(v1)) &
                        (__double_as_longlong(MR.v[2]) == __double_as_longlong(v2)) &
                        (__double_as_longlong(MR.v[3]) == __double_as_longlong(v3));
      msame = __builtin_amdgcn_ballot_w64(same);
    }
    auto rl = [](int v, int j) { return __builtin_amdgcn_readlane(v, j); };
    auto rl64 = [](int64_t v, int j) {
      const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)v, j);
      const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)((uint64_t)v >> 32), j);
      return (int64_t)(((uint64_t)hi << 32) | lo);
    };
    auto rld = [&](double v, int j) { return __longlong_as_double(rl64(__double_as_longlong(v), j)); };
    auto rlp = [&](const void *v, int j) { return (const void *)rl64((int64_t)(uintptr_t)v, j); };
#pragma unroll 1
    while (am) {
      const int j = __builtin_ctzll(am);
      am &= am - 1;
      EntryU u;
      u.band = rlp(band, j); u.row_base = 0;
      u.bx = rl(bx, j); u.by = rl(by, j); u.xoff = rl(xoff, j); u.yoff = rl(yoff, j); u.w = rl(ew, j);
      u.h = rl(eh, j); u.ns = ns_out; u.fill_mode = rl(fill_mode, j); u.mask_pair = rl(mask_pair, j);
      u.nd = (uint32_t)rl((int)nd, j); u.fill = (uint32_t)rl((int)fill, j);
      RowVal rv;
      rv.ru.v[0] = rld(v0, j); rv.ru.v[1] = rld(v1, j); rv.ru.v[2] = rld(v2, j); rv.ru.v[3] = rld(v3, j);
      rv.ru.kind = rl(kind, j); rv.ru.inside = rl(inside, j); rv.ru.nleaf = rl(nleaf, j);
      rv.ru.pool_off = rl(pool_off, j);
      rv.fx.x0 = rl64(fx0, j); rv.fx.y0 = rl64(fy0, j); rv.fx.dx = rl64(fdx, j); rv.fx.dy = rl64(fdy, j);
      if constexpr (MASK) {
        MaskU m;
        m.band = rlp(mband, j); m.bx = u.bx; m.by = u.by; m.dt = rl(mdt, j); m.fill = rl(mfill, j);
        m.same = (int)((msame >> j) & 1ull);
        m.w = 0; m.h = 0; m.kind = -1;
        m.v[0] = m.v[1] = m.v[2] = m.v[3] = 0.0;
        nn_entry_core<T, MASK, kNnPx>(a, ents, rows, pool, u, rv, &m, r, xb, xl, W, ncols, c);
      } else {
        nn_entry_core<T, MASK, kNnPx>(a, ents, rows, pool, u, rv, nullptr, r, xb, xl, W, ncols, c);
      }
    }
  }
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
// wave's rows and take all RPW rows' fixed-point forms in one vector load,
// so no row waits for its record.  Tiles with more entries (or a mask layer)
// fold through nn_fold_row_stack().
// MW (masked stacks): waves per SIMD the kernel is compiled for (0: as the
// registers fall, 87 VGPRs = 5 for C5's int16 kernel).
template <typename T, bool MASK, bool CANVAS, int RPW, bool ONE = false, int MW = 0>
__global__ __launch_bounds__(256, MASK ? (MW > 0 ? MW : 1) : 8) void render_nn_kernel(RenderArgs a, const EntryD *__restrict__ ents,
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

  const int bands_per_tile = (a.max_h + kRowsBlk - 1) / kRowsBlk;
  const int col_blocks = (a.max_w + kBandCols - 1) / kBandCols;
  const int item = blockIdx.x;
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

  // RGBA stores of row r
  auto store_row = [&](int r, const uint32_t *px, bool full_known = false) {
    uint32_t *dst = rgba_lane + (int64_t)r * a.max_w;
    if (full_known || full) {
#pragma unroll
      for (int q = 0; q < kNnPx; q++) __builtin_nontemporal_store(px[q], (GPTR(uint32_t))(dst + 64 * q));
    } else {
#pragma unroll
      for (int q = 0; q < kNnPx; q++)
        if (64 * q + lane < ncols) __builtin_nontemporal_store(px[q], (GPTR(uint32_t))(dst + 64 * q));
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
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
          (void *)uniform_ptr(e1_band), (short)0, (int)((int64_t)bx * by * (int64_t)sizeof(T)), 0x00020000);
      const RowFix *fbase = rowfix + e1_row_base;
      // the RowFix records of all RPW rows in one coalesced vector load
      // (lane 4j + k: field k of row j), read out per row with v_readlane --
      // one memory latency per wave instead of one per row
      static_assert(RPW <= 16, "4 RowFix fields of each row in one lane group");
      int64_t fv = kFixNone;
      {
        const int jj = lane >> 2, kk = lane & 3, ir = r0 - eyoff + jj;
        if (cols_ok && lane < 4 * RPW && ir >= 0 && ir < eh)
          fv = __builtin_nontemporal_load((const int64_t *)(fbase + ir) + kk);
      }
      // rows left to the fp64 bodies (no fixed form, or a pixel near a
      // truncation boundary): done in a second loop, so that loop's loads do
      // not reach the register and wait-count state of this one
      uint32_t redo = 0;
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
          const int ir = r - eyoff;
          int64_t cf[4] = {0, 0, 0, 0};
          int cfk = -1;   // -1: outside the window, 0: no fixed form, 1: fixed form
          if (cols_ok && ir >= 0 && ir < eh) {
#pragma unroll
            for (int k = 0; k < 4; k++) {
              const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)fv, 4 * j + k);
              const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)((uint64_t)fv >> 32), 4 * j + k);
              cf[k] = (int64_t)(((uint64_t)hi << 32) | lo);
            }
            cfk = cf[0] != kFixNone ? 1 : 0;
          }
          V c[kNnPx];
#pragma unroll
          for (int q = 0; q < kNnPx; q++) c[q] = cnod;
          bool done = cfk < 0;
          if (cfk == 1) {
            if constexpr (CF)
              done = nn_fix_row<T, kNnPx, false>(rs, cf[0], cf[1], cf[2], cf[3], ic0, lim, bx, nd, fill_mode, c);
            else
              done = cover ? nn_fix_row<T, kNnPx, false>(rs, cf[0], cf[1], cf[2], cf[3], ic0, lim, bx, nd, fill_mode, c)
                           : nn_fix_row<T, kNnPx, true>(rs, cf[0], cf[1], cf[2], cf[3], ic0, lim, bx, nd, fill_mode, c);
          }
          if (done) {
            uint32_t px[kNnPx];
            nn_rgba<T>(sk, safe, s_tab, c, px);
            store_row(r, px, CF);
          } else {
            redo |= 1u << j;
          }
        }
      };
      if (cover && full) row_loop(std::true_type{});
      else row_loop(std::false_type{});
#pragma unroll 1
      while (redo) {
        const int j = __builtin_ctz(redo);
        redo &= redo - 1;
        const int r = r0 + j;
        V c[kNnPx];
#pragma unroll
        for (int q = 0; q < kNnPx; q++) c[q] = cnod;
        nn_entry_row<T, false, kNnPx, false>(a, ents, e, rows, rowfix, pool, false, ns_out, r, xb, xl, W, ncols, c);
        uint32_t px[kNnPx];
        nn_rgba<T>(sk, safe, s_tab, c, px);
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
    if constexpr (MASK) {
      nn_fold_row_stack<T, true>(a, ents, ord, n_entries, rows, rowfix, pool, ns_out, r, xb, xl, W, ncols, lane, c);
    } else {
      // entries without a mask layer (C2's granule seams: 2-4 entries) one
      // after the other: the prefetched fold's per-lane descriptors would
      // not fit the 64 VGPRs of this kernel at 8 waves per SIMD
      // (the fixed-point rows here too: 1.50 vs 1.48 ms on C2, one more
      // dependent load per entry row, profiles/r06i_render.jsonl)
#pragma unroll 1
      for (int k = 0; k < n_entries; k++)
        nn_entry_row<T, false, kNnPx>(a, ents, ents[ord[k]], rows, rowfix, pool, false, ns_out, r, xb, xl, W, ncols,
                                      c);
    }

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
      nn_rgba<T>(sk, safe, s_tab, c, px);
      store_row(r, px);
    }
  }
}

// Rows per wave of the NN band kernel: 8 when the batch has work for every
// CU many times over (C2: 1.473 vs 1.506 ms), else 4 (C5, 80 tiles: 0.66 vs
// 0.86 ms at 8 -- too few blocks); profiles/r03b_ab_nn.jsonl.  Masked and
// canvas batches keep 4 (measured on C5 only).
constexpr int kNnRpw8MinItems = 32768;
constexpr int kNnRpw1MaxItems = 256;   // below one workgroup per CU at 4 rows per wave
constexpr int kNnMaskRpw1Items = 16384;   // masked stacks: one row per wave below this many workgroups

template <typename T, bool M, bool C, int RPW, bool ONE = false, int MW = 0>
void launch_nn_v(const RenderArgs &a, hipStream_t s) {
  const int items = a.n_tiles * ((a.max_h + 4 * RPW - 1) / (4 * RPW)) * ((a.max_w + kBandCols - 1) / kBandCols);
  hipLaunchKernelGGL((render_nn_kernel<T, M, C, RPW, ONE, MW>), dim3((unsigned)items), dim3(256), 0, s, a, a.entries,
                     a.order, a.rows, a.rowfix, a.pool, a.tplans, a.tiles, items);
}

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
  bool m1 = items4 < kNnMaskRpw1Items;
  // masked one-row kernel compiled for 7 waves per SIMD (71 VGPRs): C5 band
  // kernel 0.270 ms vs 0.281 at the 6 its registers fall to and 0.277 at 8
  // (15 VGPRs spilled), profiles/r06y_c5.jsonl; A/B: 0 (as the registers
  // fall) or 8
  int mw = 7;
  bool one = true;
#ifdef GSKYHIP_AB
  // shape forcing for tests/test_gpu_variants.py: small test batches never
  // reach the thresholds that pick these shapes in production
  if (const char *rp = getenv("GSKYHIP_NN_RPW")) { rpw8 = atoi(rp) == 8; rpw1 = atoi(rp) == 1; }
  if (const char *on = getenv("GSKYHIP_NN_ONE")) one = atoi(on) != 0;
  if (const char *mr = getenv("GSKYHIP_NN_MASK_RPW")) m1 = atoi(mr) == 1;
  if (const char *mv = getenv("GSKYHIP_NN_MASK_WPE")) mw = atoi(mv);
#endif
  if (mask) {
    // stacks with a mask layer (C5: ~17 entries and a mask raster per tile)
    // are latency-bound per wave row: below kNnMaskRpw1Items workgroups, one
    // row per wave (4x the waves in flight)
    if (canvas) launch_nn_v<T, true, true, 4>(a, s);
    else if (m1 && mw == 8) launch_nn_v<T, true, false, 1, false, 8>(a, s);
    else if (m1 && mw == 0) launch_nn_v<T, true, false, 1>(a, s);
    else if (m1) launch_nn_v<T, true, false, 1, false, 7>(a, s);
    else launch_nn_v<T, true, false, 4>(a, s);
  } else if (canvas) {
    launch_nn_v<T, false, true, 4>(a, s);
  } else if (rpw8) {
    // single-entry tiles through the prefetching path (C2: 1.445 vs 1.470 ms,
    // profiles/r03f_ab_c2.jsonl)
    if (one) launch_nn_v<T, false, false, 8, true>(a, s);
    else launch_nn_v<T, false, false, 8>(a, s);
  } else if (rpw1) {
    launch_nn_v<T, false, false, 1>(a, s);
  } else {
    launch_nn_v<T, false, false, 4>(a, s);
  }
}

void launch_bil(const RenderArgs &a, int n_items, hipStream_t s);   // render_bil.h, band_f32.hip

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
