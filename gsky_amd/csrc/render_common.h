// render_common.h -- device-side pieces shared by the render kernels
// (render.hip: planning + generic kernels; render_lds.hip: the typed
// LDS-staged band kernel): ComputeMask bit tests, utils.Scale constants and
// conversions, the render argument block and the typed fast-path helpers.
#pragma once
#include <type_traits>

#include "gsky_device.h"
#include "stages.h"

namespace gsky {

// ---------------------------------------------------------------- ComputeMask
// mask spec per mask-raster dtype: 0 SignedByte, 1 Byte, 2 Int16, 3 UInt16
__device__ __forceinline__ int mask_slot(int dtype) {
  switch (dtype) {
    case GSKYHIP_SIGNEDBYTE: return 0;
    case GSKYHIP_BYTE: return 1;
    case GSKYHIP_INT16: return 2;
    case GSKYHIP_UINT16: return 3;
    default: return -1;
  }
}

// A mask raster's value as its type reads it (tile_merger.go's int8 / uint8 /
// int16 / uint16 views of the masked bits): sign or zero extension of the low
// 8 or 16 bits, without a branch on the (wave-uniform) type.
__device__ __forceinline__ int32_t mask_typed(int dtype, int32_t a) {
  const int sh = (dtype == GSKYHIP_SIGNEDBYTE || dtype == GSKYHIP_BYTE) ? 24 : 16;
  const bool sgn = dtype == GSKYHIP_SIGNEDBYTE || dtype == GSKYHIP_INT16;
  const uint32_t u = (uint32_t)a << sh;
  return sgn ? ((int32_t)u >> sh) : (int32_t)(u >> sh);
}

// ComputeMask (tile_merger.go:314-445) of one mask value: value & mask > 0, or
// any bit test (value & filter == want).  Branch-free over the tests (no
// early exit), so a wave's lanes never diverge inside it -- with `return
// true` per lane the compiler built exec-mask branches around every pixel.
__device__ __forceinline__ bool mask_bit(const MaskSpecS &m, int dtype, int32_t v) {
  if (m.has_value) return mask_typed(dtype, v & m.value) > 0;
  bool hit = false;
  for (int j = 0; j < m.n_tests; j++) hit |= mask_typed(dtype, v & m.filt[j]) == mask_typed(dtype, m.want[j]);
  return hit;
}

// ---------------------------------------------------------------- scale
// utils.scale (raster_scaler.go:30-332) constants of one canvas.
struct ScaleK {
  int32_t dtype;
  int32_t colour_scale;
  Val noData, off, clp;  // in the canvas type
  float sc;
  double nodata64;
};

// Go math.Log / Log2 / Log10 (Go 1.12, same op sequence as the amd64 asm).
static __device__ __noinline__ double go_log(double x) {
  const double Ln2Hi = 6.93147180369123816490e-01, Ln2Lo = 1.90821492927058770002e-10;
  const double L1 = 6.666666666666735130e-01, L2 = 3.999999999940941908e-01, L3 = 2.857142874366239149e-01,
               L4 = 2.222219843214978396e-01, L5 = 1.818357216161805012e-01, L6 = 1.531383769920937332e-01,
               L7 = 1.479819860511658591e-01;
  if (x != x || x == INFINITY) return x;
  if (x < 0) return NAN;
  if (x == 0) return -INFINITY;
  int ki;
  double f1 = frexp(x, &ki);
  if (f1 < 1.41421356237309504880168872420969808 / 2) { f1 *= 2; ki--; }
  double f = f1 - 1;
  double k = (double)ki;
  double s = f / (2 + f);
  double s2 = s * s;
  double s4 = s2 * s2;
  double t1 = s2 * (L1 + s4 * (L3 + s4 * (L5 + s4 * L7)));
  double t2 = s4 * (L2 + s4 * (L4 + s4 * L6));
  double R = t1 + t2;
  double hfsq = 0.5 * f * f;
  return k * Ln2Hi - ((hfsq - (s * (hfsq + R) + k * Ln2Lo)) - f);
}
static __device__ __noinline__ double go_log10(double x) {
  int e;
  double frac = frexp(x, &e);
  double l2;
  if (frac == 0.5) l2 = (double)(e - 1);
  else l2 = go_log(frac) * (1.0 / 0.693147180559945309417232121458176568) + (double)e;
  return l2 * 0.301029995663981195213738894724493026768189881462108541310;
}

// normalise() (raster_scaler.go:15-28); returns false when the value maps to nodata
__device__ __forceinline__ bool normalise_f(float &value, int colour_scale, double nodata64) {
  double d = (double)value;
  if (!(d == nodata64)) {
    if (colour_scale == 1) d = go_log10(d);
    if (isinf(d) || d != d) d = nodata64;
  }
  if (d == nodata64) return false;
  value = (float)d;
  return true;
}

__device__ __forceinline__ uint8_t scale_px(const ScaleK &k, Val v) {
  if (k.dtype == GSKYHIP_FLOAT32) {
    float value = v.f;
    if (value == k.noData.f) return 0xFF;
    if (k.colour_scale > 0 && !normalise_f(value, k.colour_scale, k.nodata64)) return 0xFF;
    value += k.off.f;
    if (value > k.clp.f) value = k.clp.f;
    if (value < 0.0f) value = 0.0f;
    return go_f32_u8(value * k.sc);
  }
  int32_t value = v.i;
  if (value == k.noData.i) return 0xFF;
  switch (k.dtype) {  // value += offset in the raster's own type (wraps)
    case GSKYHIP_SIGNEDBYTE: value = (int8_t)(value + k.off.i); break;
    case GSKYHIP_BYTE: value = (uint8_t)(value + k.off.i); break;
    case GSKYHIP_INT16: value = (int16_t)(value + k.off.i); break;
    default: value = (uint16_t)(value + k.off.i); break;
  }
  if (value > k.clp.i) value = k.clp.i;
  if (value < 0) value = 0;
  return go_f32_u8((float)value * k.sc);
}

// Scale constants of a canvas; auto mode takes min/max from the fold pass
// (raster_scaler.go:47-78 and its typed siblings).
__device__ inline ScaleK make_scale(int dtype, double nodata, const gskyhip_scale_params &sp, bool autom,
                                    float minVal, float maxVal) {
  ScaleK k;
  k.dtype = dtype;
  k.colour_scale = sp.colour_scale;
  k.nodata64 = nodata;
  float sc = (float)sp.scale;
  if (sc <= 0.0f) sc = (sp.clip <= 0.0) ? 1.0f : (float)(254.0f / (float)sp.clip);
  k.noData = go_conv_to(nodata, dtype);
  if (dtype == GSKYHIP_FLOAT32) {
    k.off.f = (float)sp.offset;
    k.clp.f = (float)sp.clip;
    if (autom) {
      if (minVal == maxVal) maxVal += 0.1f;
      sc = 254.0f / (maxVal - minVal);
      k.off.f = -minVal;
      k.clp.f = maxVal + k.off.f;
    }
  } else {
    k.off = go_conv_to(sp.offset, dtype);
    k.clp = go_conv_to(sp.clip, dtype);
    if (autom) {
      if (minVal == maxVal) maxVal += 0.1f;
      sc = 254.0f / (maxVal - minVal);
      const float dfOffset = -minVal;
      k.off = go_conv_to((double)dfOffset, dtype);
      k.clp = go_conv_to((double)(maxVal + dfOffset), dtype);
    }
  }
  k.sc = sc;
  return k;
}

// ordered-int encoding of float for atomic min/max
__device__ __forceinline__ int32_t fenc(float f) {
  int32_t i = __float_as_int(f);
  return i ^ ((i >> 31) & 0x7FFFFFFF);
}
__device__ __forceinline__ float fdec(int32_t i) { return __int_as_float(i ^ ((i >> 31) & 0x7FFFFFFF)); }

// Per (tile, out ns) auto-scale reduction state.
struct MinMax {
  int32_t mn, mx;      // fenc, over valid non-NaN values
  int32_t p0_valid;    // pixel 0 valid (not nodata, and log-normalisable)
  float p0;            // its (normalised) value
};

__device__ __forceinline__ void auto_minmax(const MinMax &m, float &mn, float &mx) {
  // min/max start at 0 unless pixel 0 is valid (raster_scaler.go:55-58)
  if (m.p0_valid) {
    if (m.p0 != m.p0) { mn = m.p0; mx = m.p0; }
    else { mn = fdec(m.mn); mx = fdec(m.mx); }
  } else {
    mn = fminf(0.0f, fdec(m.mn));
    mx = fmaxf(0.0f, fdec(m.mx));
  }
}

struct RenderArgs {
  const PairPlan *pairs;
  const Xform *xforms;
  const TilePlan *tplans;
  const int32_t *order;
  const gskyhip_tile *tiles;
  const RowRec *rows;
  const RowFix *rowfix;  // fixed-point form of `inside` LINEAR rows (render_nn.h)
  const Leaf *pool;
  const int32_t *counters;
  const int32_t *complex_list;
  int max_h, max_w;     // tile slot: rgba / canvas row stride is max_w
  int n_tiles;
  int rows_per_block;
  int n_out;
  int32_t out_ns[3];
  MaskSpecS mask[4];
  gskyhip_scale_params sp;
  int autom;
  const uint32_t *ramp;  // 256 packed RGBA or NULL
  uint8_t *rgba;
  uint8_t *canvas;       // optional typed canvases
  long canvas_tile_stride, canvas_ns_stride;
  MinMax *minmax;        // n_tiles * 3
  int write_rgba;
  const EntryD *entries;
  int lds_mode;          // typed band kernels: kBilinear | kCanvas bits of the call
  const int64_t *cov_offsets;  // canvas mode: per tile element offset into one image (NULL: slots)
  int64_t cov_stride;          // ... and that image's row stride (elements)
};

// ---------------------------------------------------------------- typed fast path
// Every entry of a simple tile shares one value type T (vt) and needs no
// GDALCopyWords promotion, every row is LINEAR or POOL with linear leaves,
// so a pixel is: two fp64 affine evaluations, truncation, one typed gather,
// a branch-free ordered fold, the scale and the palette lookup.
#define GPTR(T) __attribute__((address_space(1))) T *
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
template <typename T> struct VOf { using type = int32_t; };
template <> struct VOf<float> { using type = float; };

template <typename T>
__device__ __forceinline__ typename VOf<T>::type as_v(Val x) {
  if constexpr (std::is_same<T, float>::value) return x.f; else return x.i;
}

// Go uint8(f) of a float32 (CVTTSS2SL, low byte): NaN / out of range -> 0.
__device__ __forceinline__ uint32_t go_u8_f32(float f) {
  return (f > -2147483648.0f && f < 2147483648.0f) ? ((uint32_t)(int32_t)f & 0xFFu) : 0u;
}

template <typename T>
__device__ __forceinline__ uint32_t scale_t(const ScaleK &k, typename VOf<T>::type c) {
  if constexpr (std::is_same<T, float>::value) {
    Val v; v.f = c;
    return scale_px(k, v);   // float32: normalise / log path stays exact and general
  } else {
    if (c == k.noData.i) return 0xFFu;
    int32_t value = c + k.off.i;
    if constexpr (std::is_same<T, int8_t>::value) value = (int8_t)value;
    else if constexpr (std::is_same<T, uint8_t>::value) value = (uint8_t)value;
    else if constexpr (std::is_same<T, int16_t>::value) value = (int16_t)value;
    else value = (uint16_t)value;
    value = min(value, k.clp.i);
    value = max(value, 0);
    return go_u8_f32((float)value * k.sc);
  }
}

// The leaf of window pixel i: the last one starting at or before i (leaf 0
// starts at 0; starts strictly increase), by binary search -- rows of
// per-pixel leaves can hold a leaf per window column.
__device__ __forceinline__ int leaf_of(const Leaf *__restrict__ lv, int nleaf, int i) {
  int lo = 0, hi = nleaf - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (lv[mid].start <= i) lo = mid; else hi = mid - 1;
  }
  return lo;
}

// Source coordinates of window pixel i of a LINEAR / POOL row (simple tiles:
// leaves linear, or per-pixel exact points with dX = dY = 0, or LEAF_FAILED).
// false: the exact transform of the pixel failed (window fill).
__device__ __forceinline__ bool lin_coords(const RowRec &rr, const Leaf *__restrict__ pool, int i, double &sx,
                                           double &sy) {
  double xs0 = rr.v[0], ys0 = rr.v[1], dX = rr.v[2], dY = rr.v[3];
  int start = 0;
  bool ok = true;
  if (rr.kind == ROW_POOL) {
    const Leaf *lv = pool + rr.pool_off;
    const int k = leaf_of(lv, rr.nleaf, i);
    xs0 = lv[k].xs0; ys0 = lv[k].ys0; dX = lv[k].dX; dY = lv[k].dY; start = lv[k].start;
    ok = lv[k].kind != LEAF_FAILED;
  }
  const double dist = (double)(i - start);
  sy = ys0 + dY * dist;
  sx = xs0 + dX * dist;
  return ok;
}

// NN gather of one window pixel in type T; returns false -> window fill.
template <typename T>
__device__ __forceinline__ bool nn_fetch(const EntryD &e, double sx, double sy, typename VOf<T>::type &v) {
  if (sx < 0 || sy < 0) return false;
  const double ax = sx + 1.0e-10, ay = sy + 1.0e-10;
  if (ax >= 2147483647.0 || ay >= 2147483647.0) return false;
  const int ix = (int)ax, iy = (int)ay;
  if (ix >= e.band_x || iy >= e.band_y) return false;
  v = (typename VOf<T>::type)((const T *)e.band)[(long)iy * e.band_x + ix];
  return true;
}

template <typename T>
__device__ __forceinline__ bool bil_fetch(const EntryD &e, double sx, double sy, typename VOf<T>::type &v) {
  int iSrcX = (int)floor(sx - 0.5);
  int iSrcY = (int)floor(sy - 0.5);
  double rX = 1.5 - (sx - iSrcX);
  double rY = 1.5 - (sy - iSrcY);
  if (iSrcX == -1) { iSrcX = 0; rX = 1; }
  if (iSrcY == -1) { iSrcY = 0; rY = 1; }
  double accR = 0.0, accDiv = 0.0;
  const T *band = (const T *)e.band;
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const int xx = iSrcX + (k & 1), yy = iSrcY + (k >> 1);
    const double w = ((k & 1) ? (1.0 - rX) : rX) * ((k >> 1) ? (1.0 - rY) : rY);
    if (xx < 0 || xx >= e.band_x || yy < 0 || yy >= e.band_y) continue;
    const double d = (double)band[(long)yy * e.band_x + xx];
    if (e.has_nodata && (d == e.nodata64 || (e.nodata64 != e.nodata64 && d != d))) continue;
    accDiv += w;
    accR += d * w;
  }
  double r;
  if (accDiv == 1.0) r = accR;
  else if (accDiv < 0.00001) return false;
  else r = accR / accDiv;
  if constexpr (std::is_same<T, float>::value) v = (float)r;
  else v = gdal_copy_to(floor(r + 0.5), e.out_dtype).i;
  return true;
}

// Full per-pixel path (exact points, descend): only complex tiles and the
// drop-in window kernel run it.
__device__ __noinline__ bool descend_coords(const Xform &t, int xoff, double yrow, int n0, const double *v,
                                            int i, double &sx, double &sy) {
  int lo = 0, n = n0;
  double xs[3] = {v[0], v[2], v[4]}, ys[3] = {v[1], v[3], v[5]};
  auto xpos = [&](int idx) { return idx + 0.5 + xoff; };
  for (;;) {
    const int nMiddle = (n - 1) / 2;
    const double x0 = xpos(lo), xl = xpos(lo + n - 1), xm = xpos(lo + nMiddle);
    const double dX = (xs[2] - xs[0]) / (xl - x0);
    const double dY = (ys[2] - ys[0]) / (xl - x0);
    const double dfError = fabs((xs[0] + dX * (xm - x0)) - xs[1]) + fabs((ys[0] + dY * (xm - x0)) - ys[1]);
    if (dfError <= kMaxErr) {
      const double dist = xpos(i) - x0;
      sy = ys[0] + dY * dist;
      sx = xs[0] + dX * dist;
      return true;
    }
    const int i0 = lo + (nMiddle - 1) / 2, i1 = lo + nMiddle - 1, i2 = lo + nMiddle + (n - nMiddle - 1) / 2;
    double mx[3] = {xpos(i0), xpos(i1), xpos(i2)};
    double my[3] = {yrow, yrow, yrow};
    const bool base1 = nMiddle <= 5 || x0 == mx[1] || x0 == mx[0];
    const bool base2 = n - nMiddle <= 5 || xm == xl || xm == mx[2];
    bool ok = false;
    if (!base1 && !base2) {
      ok = xform_point(t, true, mx[0], my[0]);
      ok = xform_point(t, true, mx[1], my[1]) && ok;
      ok = xform_point(t, true, mx[2], my[2]) && ok;
    } else if (!base1) {
      ok = xform_point(t, true, mx[0], my[0]);
      ok = xform_point(t, true, mx[1], my[1]) && ok;
    } else if (!base2) {
      ok = xform_point(t, true, mx[2], my[2]);
    }
    const bool first = (i - lo) < nMiddle;
    if (!ok || (first && base1) || (!first && base2)) {
      sx = xpos(i); sy = yrow;
      return xform_point(t, true, sx, sy);
    }
    if (first) {
      n = nMiddle;
      xs[1] = mx[0]; ys[1] = my[0]; xs[2] = mx[1]; ys[2] = my[1];
    } else {
      xs[0] = xs[1]; ys[0] = ys[1];
      xs[1] = mx[2]; ys[1] = my[2];
      lo = lo + nMiddle;
      n = n - nMiddle;
    }
  }
}

__device__ __noinline__ bool exact_coords(const Xform &t, int xoff, int yoff, int i, int row, double &sx,
                                          double &sy) {
  sx = i + 0.5 + xoff;
  sy = row + 0.5 + yoff;
  return xform_point(t, true, sx, sy);
}

// Source coordinates of window pixel (i, row).  GENERAL=false: the row is
// LINEAR or POOL with linear leaves only (simple tiles).
template <bool GENERAL>
__device__ __forceinline__ bool src_coords(const RowRec &rr, const Leaf *pool, const Xform *xf, int xoff,
                                           int yoff, int w, int i, int row, double &sx, double &sy) {
  if (rr.kind == ROW_LINEAR) {
    const double dist = (double)i;
    sy = rr.v[1] + rr.v[3] * dist;
    sx = rr.v[0] + rr.v[2] * dist;
    return true;
  }
  if (rr.kind == ROW_POOL) {
    const Leaf *lv = pool + rr.pool_off;
    const Leaf &L = lv[leaf_of(lv, rr.nleaf, i)];
    if (L.kind == LEAF_FAILED) return false;
    if (!GENERAL || L.kind == LEAF_LINEAR) {
      const double dist = (double)(i - L.start);
      sy = L.ys0 + L.dY * dist;
      sx = L.xs0 + L.dX * dist;
      return true;
    }
  }
  if (GENERAL) {
    if (rr.kind == ROW_DESCEND) return descend_coords(*xf, xoff, row + 0.5 + yoff, w, rr.v, i, sx, sy);
    return exact_coords(*xf, xoff, yoff, i, row, sx, sy);
  }
  return false;
}

// Mask raster value (its own dtype, NN) for data window index (ic, ir) of an
// entry of window width ew whose mask pair is mask_pair.
template <int RES>
__device__ __forceinline__ bool mask_fast_pair(const EntryD *__restrict__ ents, const RowRec *__restrict__ rows,
                                               const Leaf *__restrict__ pool, const MaskSpecS *ms, int mask_pair,
                                               int ew, int ic, int ir) {
  const EntryD &m = ents[mask_pair];
  int mx = ic, my = ir;
  if (m.w != ew) {
    const long iSrc = (long)ir * ew + ic;
    mx = (int)(iSrc % m.w);
    my = (int)(iSrc / m.w);
  }
  if (my >= m.h) return false;
  double sx, sy;
  int32_t v = 0;
  bool ok = false;
  if (lin_coords(rows[m.row_base + my], pool, mx, sx, sy)) {   // false: failed transform -> fill
    switch (m.out_dtype) {
      case GSKYHIP_BYTE: ok = nn_fetch<uint8_t>(m, sx, sy, v); break;
      case GSKYHIP_SIGNEDBYTE: ok = nn_fetch<int8_t>(m, sx, sy, v); break;
      case GSKYHIP_INT16: ok = nn_fetch<int16_t>(m, sx, sy, v); break;
      default: ok = nn_fetch<uint16_t>(m, sx, sy, v); break;
    }
  }
  if (!ok) v = m.fill.i;
  const int slot = mask_slot(m.out_dtype);
  return slot >= 0 && mask_bit(ms[slot], m.out_dtype, v);
}

template <int RES>
__device__ __forceinline__ bool mask_fast(const EntryD *__restrict__ ents, const RowRec *__restrict__ rows,
                                          const Leaf *__restrict__ pool, const MaskSpecS *ms, const EntryD &e,
                                          int ic, int ir) {
  return mask_fast_pair<RES>(ents, rows, pool, ms, e.mask_pair, e.w, ic, ir);
}

constexpr int kLdsBandRows = 16;   // rows per block of render_lds_kernel
constexpr int kBilinear = 4, kCanvas = 8;   // render_lds_kernel modes (RenderArgs.lds_mode)

// The typed band kernels (render_lds.hip) for value type `vt`.
void launch_band_kernels(const RenderArgs &a, int vt, bool mask, int n_items, hipStream_t s);
// Generic kernels (render_generic{1,3}.hip); general_only: complex tiles only.
void dispatch_render_1(const RenderArgs &a, int resample, bool mask, dim3 grid, bool general_only, hipStream_t s);
void dispatch_render_3(const RenderArgs &a, int resample, bool mask, dim3 grid, bool general_only, hipStream_t s);

}  // namespace gsky
