// gsky_device.h -- device-side building blocks of the MI355X raster hot path.
//
// Projection math restates PROJ 6.1.1 (merc/webmerc, aea, gn_sinu, tmerc, lcc, polar stere and the
// pj_fwd / pj_inv wrappers) and GDAL 3.0.1's GenImgProj transformer; numeric
// conversions restate Go 1.12 on amd64.  All of it
// is compiled with -ffp-contract=off so every double expression rounds once
// per operation, as in the reference's SSE2 code.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/gskyhip.h"

namespace gsky {

constexpr double kHalfPi = 1.57079632679489661923;
constexpr double kPi = 3.14159265358979323846;
constexpr double kTwoPi = 6.2831853071795864769;
constexpr double kFortPi = 0.78539816339744830962;
constexpr double kD2R = 0.017453292519943295769236907684886;
constexpr double kR2D = 1.0 / 0.017453292519943295769236907684886;
constexpr double kMaxErr = 0.125;   // GDALCreateApproxTransformer(.., 0.125), warp.go:219

// ---------------------------------------------------------------- Go conversions
__host__ __device__ inline int32_t go_cvtt32(double x) {
  // CVTTSD2SL: NaN / out of range -> 0x80000000
  if (!(x > -2147483649.0 && x < 2147483648.0)) return INT32_MIN;
  return (int32_t)x;
}
__host__ __device__ inline int64_t go_cvtt64(double x) {
  // CVTTSD2SQ (Go int(float64) on amd64): NaN / out of range -> 0x8000000000000000
  if (!(x >= -9223372036854775808.0 && x < 9223372036854775808.0)) return INT64_MIN;
  return (int64_t)x;
}
__host__ __device__ inline int8_t go_i8(double v) { return (int8_t)(uint8_t)(uint32_t)go_cvtt32(v); }
__host__ __device__ inline uint8_t go_u8(double v) { return (uint8_t)(uint32_t)go_cvtt32(v); }
__host__ __device__ inline int16_t go_i16(double v) { return (int16_t)(uint16_t)(uint32_t)go_cvtt32(v); }
__host__ __device__ inline uint16_t go_u16(double v) { return (uint16_t)(uint32_t)go_cvtt32(v); }
__host__ __device__ inline uint8_t go_f32_u8(float v) { return go_u8((double)v); }

// GDALCopyWord(double -> integer T): round half away from zero, saturate, NaN->0.
__host__ __device__ inline double gdal_round_clamp(double v, double lo, double hi) {
  if (v != v) return 0.0;
  double r = v >= 0.0 ? v + 0.5 : v - 0.5;
  if (r > hi) r = hi;
  if (r < lo) r = lo;
  return trunc(r);
}

__host__ __device__ inline int type_size(int dtype) {
  switch (dtype) {
    case GSKYHIP_BYTE: case GSKYHIP_SIGNEDBYTE: return 1;
    case GSKYHIP_UINT16: case GSKYHIP_INT16: return 2;
    case GSKYHIP_UINT32: case GSKYHIP_INT32: case GSKYHIP_FLOAT32: return 4;
    case GSKYHIP_FLOAT64: return 8;
    default: return 0;
  }
}

// A raster value carried through the fold as raw bits of its output type.
// Integer types are sign/zero-extended into `i`; float32 lives in `f`.
struct Val {
  union { int32_t i; float f; uint32_t u; };
};

// GDALCopyWords(nodata double -> output dtype), returned as a Val.
__host__ __device__ inline Val gdal_copy_to(double v, int dtype) {
  Val o; o.u = 0;
  switch (dtype) {
    case GSKYHIP_BYTE: o.i = (int32_t)(uint8_t)gdal_round_clamp(v, 0, 255); break;
    // a SignedByte band is a GDT_Byte band: GDALCopyWords clamps to [0,255];
    // the merge then reads those bits as int8 (tile_merger.go:40-46).
    case GSKYHIP_SIGNEDBYTE: o.i = (int32_t)(int8_t)(uint8_t)gdal_round_clamp(v, 0, 255); break;
    case GSKYHIP_UINT16: o.i = (int32_t)(uint16_t)gdal_round_clamp(v, 0, 65535); break;
    case GSKYHIP_INT16: o.i = (int32_t)(int16_t)gdal_round_clamp(v, -32768, 32767); break;
    case GSKYHIP_FLOAT32: {
      float f;
      if (v == INFINITY || v == -INFINITY) f = (float)v;
      else if (v > 3.402823466e+38) f = 3.402823466e+38f;
      else if (v < -3.402823466e+38) f = -3.402823466e+38f;
      else f = (float)v;
      o.f = f;
      break;
    }
    default: break;
  }
  return o;
}

// Go T(nodata) of the merge (tile_merger.go:46,80,117,155,193) as a Val of the
// canvas type.  SignedByte values are kept as int8 sign-extended.
__host__ __device__ inline Val go_conv_to(double v, int dtype) {
  Val o; o.u = 0;
  switch (dtype) {
    case GSKYHIP_SIGNEDBYTE: o.i = go_i8(v); break;
    case GSKYHIP_BYTE: o.i = go_u8(v); break;
    case GSKYHIP_INT16: o.i = go_i16(v); break;
    case GSKYHIP_UINT16: o.i = go_u16(v); break;
    case GSKYHIP_FLOAT32: o.f = (float)v; break;
    default: break;
  }
  return o;
}

// Value equality in the canvas type (float compare for Float32: NaN != NaN).
__device__ __forceinline__ bool val_eq(Val a, Val b, bool is_float) {
  return is_float ? (a.f == b.f) : (a.i == b.i);
}

// ---------------------------------------------------------------- projections
__host__ __device__ inline double adjlon(double lon) {
  if (fabs(lon) < kPi + 1e-12) return lon;
  lon += kPi;
  lon -= kTwoPi * floor(lon / kTwoPi);
  lon -= kPi;
  return lon;
}

__host__ __device__ inline double qsfn(double sinphi, double e, double one_es) {
  if (e >= 1.0e-7) {
    double con = e * sinphi;
    double div1 = 1.0 - con * con;
    double div2 = 1.0 + con;
    if (div1 == 0.0 || div2 == 0.0) return HUGE_VAL;
    return one_es * (sinphi / div1 - (.5 / e) * log((1. - con) / div2));
  }
  return sinphi + sinphi;
}

__host__ __device__ inline double aea_phi1(double qs, double Te, double Tone_es) {
  double Phi = asin(.5 * qs);
  if (Te < 1.0e-7) return Phi;
  int i = 15;
  double dphi;
  do {
    double sinpi = sin(Phi), cospi = cos(Phi);
    double con = Te * sinpi;
    double com = 1. - con * con;
    dphi = .5 * com * com / cospi *
           (qs / Tone_es - sinpi / com + .5 / Te * log((1. - con) / (1. + con)));
    Phi += dphi;
  } while (fabs(dphi) > 1.0e-10 && --i);
  return i ? Phi : HUGE_VAL;
}

// Transverse Mercator, ellipsoidal: the Poder / Engsager algorithm that
// PROJ 6 runs for +proj=tmerc and +proj=utm (tmerc.cpp exact_e_fwd /
// exact_e_inv / setup_exact, [ext]: not in /root/reference; restated from the
// published algorithm -- Engsager & Poder, ICC 2007; Krueger series to n^6 as
// in Karney 2011 -- parity unpinned beyond the known-answer points of
// tests/test_tmerc.py).  Gaussian <-> geodetic latitude: a real Clenshaw sum
// of sin(2k B); spherical <-> ellipsoidal N, E: a complex one.
__host__ __device__ inline double tm_gatg(const double *p1, int len, double B) {
  const double cos_2B = 2 * cos(2 * B);
  const double *p = p1 + len;
  double h = 0, h1 = *--p, h2 = 0;
  while (p - p1) {
    h = -h2 + cos_2B * h1 + *--p;
    h2 = h1;
    h1 = h;
  }
  return B + h * sin(2 * B);
}

__host__ __device__ inline double tm_clens(const double *a, int size, double arg_r) {
  const double *p = a + size;
  const double r = 2 * cos(arg_r);
  double hr1 = 0, hr = *--p, hr2;
  for (; a - p;) {
    hr2 = hr1;
    hr1 = hr;
    hr = -hr2 + r * hr1 + *--p;
  }
  return sin(arg_r) * hr;
}

__host__ __device__ inline double tm_clenS(const double *a, int size, double arg_r, double arg_i, double *R,
                                           double *I) {
  const double *p = a + size;
  const double sin_arg_r = sin(arg_r), cos_arg_r = cos(arg_r);
  const double sinh_arg_i = sinh(arg_i), cosh_arg_i = cosh(arg_i);
  double r = 2 * cos_arg_r * cosh_arg_i;
  double i = -2 * sin_arg_r * sinh_arg_i;
  double hi1 = 0, hr1 = 0, hi = 0, hr = *--p, hr2, hi2;
  for (; a - p;) {
    hr2 = hr1;
    hi2 = hi1;
    hr1 = hr;
    hi1 = hi;
    hr = -hr2 + r * hr1 - i * hi1 + *--p;
    hi = -hi2 + i * hr1 + r * hi1;
  }
  r = sin_arg_r * cosh_arg_i;
  i = cos_arg_r * sinh_arg_i;
  *R = r * hr - i * hi;
  *I = r * hi + i * hr;
  return *R;
}

constexpr double kTmMaxCe = 2.623395162778;   // 150 degrees of spherical easting

// (lam, phi) -> normalised (E, N) (before pj_fwd's a * x + x0).  Not inlined:
// inlined, its transcendental chain raised the register peak of every kernel
// carrying the projection switch (plan_small 350 -> 360 VGPRs, plan_pairs<256>
// 198 -> 230); called, only the tmerc path pays for it.
__host__ __device__ inline __attribute__((noinline)) bool tm_fwd(const gskyhip_crs &c, double lam, double phi, double &xn, double &yn) {
  double Cn = tm_gatg(c.tm_cbg, 6, phi);   // ellipsoidal -> Gaussian latitude
  const double sin_Cn = sin(Cn), cos_Cn = cos(Cn), sin_Ce = sin(lam), cos_Ce = cos(lam);
  Cn = atan2(sin_Cn, cos_Ce * cos_Cn);     // Gaussian -> complementary spherical
  double Ce = atan2(sin_Ce * cos_Cn, hypot(sin_Cn, cos_Cn * cos_Ce));
  Ce = asinh(tan(Ce));
  double dCn, dCe;
  Cn += tm_clenS(c.tm_gtu, 6, 2 * Cn, 2 * Ce, &dCn, &dCe);
  Ce += dCe;
  if (!(fabs(Ce) <= kTmMaxCe)) return false;
  yn = c.tm_qn * Cn + c.tm_zb;
  xn = c.tm_qn * Ce;
  return true;
}

// normalised (E, N) -> (lam, phi) (after pj_inv's (x - x0) / a).
__host__ __device__ inline __attribute__((noinline)) bool tm_inv(const gskyhip_crs &c, double xn, double yn, double &lam, double &phi) {
  double Cn = (yn - c.tm_zb) / c.tm_qn, Ce = xn / c.tm_qn;
  if (!(fabs(Ce) <= kTmMaxCe)) return false;
  double dCn, dCe;
  Cn += tm_clenS(c.tm_utg, 6, 2 * Cn, 2 * Ce, &dCn, &dCe);
  Ce += dCe;
  Ce = atan(sinh(Ce));
  const double sin_Cn = sin(Cn), cos_Cn = cos(Cn), sin_Ce = sin(Ce), cos_Ce = cos(Ce);
  Ce = atan2(sin_Ce, cos_Ce * cos_Cn);
  Cn = atan2(sin_Cn * cos_Ce, hypot(sin_Ce, cos_Ce * cos_Cn));
  phi = tm_gatg(c.tm_cgb, 6, Cn);
  lam = Ce;
  return true;
}

// Lambert Conformal Conic, ellipsoidal (PROJ 6.1.1 lcc.cpp e_forward /
// e_inverse with pj_tsfn / pj_phi2, [ext]; restated from the published
// algorithm -- Snyder, Map Projections: A Working Manual, 15-1..15-11 --
// pinned by Snyder's worked example in tests/test_lcc.py).  Out of line for
// the same register reason as tm_fwd.
// The transcendental calls of lcc / stere out of line: inlined, the
// scheduler overlapped their bodies and took lcc_inv / stere_inv to 248 VGPRs,
// which the planners that may call them inherit (same functions, same bits).
__host__ __device__ inline __attribute__((noinline)) double ext_pow(double a, double b) { return pow(a, b); }
__host__ __device__ inline __attribute__((noinline)) double ext_atan(double a) { return atan(a); }
__host__ __device__ inline __attribute__((noinline)) double ext_tan(double a) { return tan(a); }
__host__ __device__ inline __attribute__((noinline)) double ext_sin(double a) { return sin(a); }

__host__ __device__ inline double lcc_tsfn(double phi, double sinphi, double e) {
  sinphi *= e;
  return ext_tan(.5 * (kHalfPi - phi)) / ext_pow((1. - sinphi) / (1. + sinphi), .5 * e);
}

__host__ __device__ inline __attribute__((noinline)) bool lcc_fwd(const gskyhip_crs &c, double lam, double phi,
                                                                   double &xn, double &yn) {
  double rho;
  if (fabs(fabs(phi) - kHalfPi) < 1.e-10) {
    if (phi * c.n <= 0.) return false;
    rho = 0.;
  } else {
    rho = c.c * ext_pow(lcc_tsfn(phi, ext_sin(phi), c.e), c.n);
  }
  lam *= c.n;
  xn = c.k0 * (rho * ext_sin(lam));
  yn = c.k0 * (c.rho0 - rho * cos(lam));
  return true;
}

__host__ __device__ inline __attribute__((noinline)) bool lcc_inv(const gskyhip_crs &c, double xn, double yn,
                                                                   double &lam, double &phi) {
  xn /= c.k0;
  yn /= c.k0;
  yn = c.rho0 - yn;
  double rho = hypot(xn, yn);
  if (rho != 0.) {
    if (c.n < 0.) { rho = -rho; xn = -xn; yn = -yn; }
    const double ts = ext_pow(rho / c.c, 1. / c.n);   // pj_phi2
    const double eccnth = .5 * c.e;
    double Phi = kHalfPi - 2. * ext_atan(ts), dphi;
    int i = 15;
    do {
      const double con = c.e * ext_sin(Phi);
      dphi = kHalfPi - 2. * ext_atan(ts * ext_pow((1. - con) / (1. + con), eccnth)) - Phi;
      Phi += dphi;
    } while (fabs(dphi) > 1.0e-10 && --i);
    if (i <= 0) return false;
    phi = Phi;
    lam = atan2(xn, yn) / c.n;
  } else {
    lam = 0.;
    phi = c.n > 0. ? kHalfPi : -kHalfPi;
  }
  return true;
}

// Polar stereographic, ellipsoidal (PROJ 6.1.1 stere.cpp e_forward /
// e_inverse, N_POLE / S_POLE modes, [ext]; Snyder 21-33..21-39, pinned by
// Snyder's worked example in tests/test_stere.py): akm1 in c.c, the pole by
// the sign of phi0.
__host__ __device__ inline __attribute__((noinline)) bool stere_fwd(const gskyhip_crs &c, double lam, double phi,
                                                                     double &xn, double &yn) {
  double coslam = cos(lam);
  const double sinlam = ext_sin(lam);
  double sinphi = ext_sin(phi);
  if (c.phi0 < 0) {   // S_POLE
    phi = -phi;
    coslam = -coslam;
    sinphi = -sinphi;
  }
  double x = c.c * lcc_tsfn(phi, sinphi, c.e);
  yn = -x * coslam;
  xn = x * sinlam;
  return true;
}

__host__ __device__ inline __attribute__((noinline)) bool stere_inv(const gskyhip_crs &c, double xn, double yn,
                                                                     double &lam, double &phi) {
  const double rho = hypot(xn, yn);
  if (c.phi0 >= 0) yn = -yn;   // N_POLE
  const double tp = -rho / c.c, halfpi = -kHalfPi, halfe = -.5 * c.e;
  double phi_l = kHalfPi - 2. * ext_atan(tp);
#pragma unroll 1
  for (int i = 8; i--; phi_l = phi) {
    const double sinphi = c.e * ext_sin(phi_l);
    phi = 2. * ext_atan(tp * ext_pow((1. + sinphi) / (1. - sinphi), halfe)) - halfpi;
    if (fabs(phi_l - phi) < 1.e-10) {
      if (c.phi0 < 0) phi = -phi;
      lam = (xn == 0. && yn == 0.) ? 0. : atan2(xn, yn);
      return true;
    }
  }
  return false;
}

// pj_inv: CRS coordinates -> (lam, phi) in radians.
__host__ __device__ inline bool crs_inverse(const gskyhip_crs &c, double x, double y, double &lam, double &phi) {
  if (x == HUGE_VAL || y == HUGE_VAL) return false;
  if (c.kind == GSKYHIP_CRS_LONGLAT) {  // +proj=unitconvert deg -> rad
    lam = x * kD2R;
    phi = y * kD2R;
    return true;
  }
  double xn = (x * 1.0 - c.x0) * c.ra;
  double yn = (y * 1.0 - c.y0) * c.ra;
  double l, p;
  if (c.kind == GSKYHIP_CRS_WEBMERC) {  // merc.cpp s_inverse
    p = kHalfPi - 2. * atan(exp(-yn / c.k0));
    l = xn / c.k0;
  } else if (c.kind == GSKYHIP_CRS_AEA) {  // aea.cpp e_inverse
    yn = c.rho0 - yn;
    double rho = hypot(xn, yn);
    if (rho != 0.0) {
      if (c.n < 0.) { rho = -rho; xn = -xn; yn = -yn; }
      p = rho / c.dd;
      if (c.es > 0.) {
        p = (c.c - p * p) / c.n;
        if (fabs(c.ec - fabs(p)) > 1e-7) {
          p = aea_phi1(p, c.e, c.one_es);
          if (p == HUGE_VAL) return false;
        } else {
          p = p < 0. ? -kHalfPi : kHalfPi;
        }
      } else {
        p = (c.c - p * p) / (c.n + c.n);
        if (fabs(p) <= 1.) p = asin(p);
        else p = p < 0. ? -kHalfPi : kHalfPi;
      }
      l = atan2(xn, yn) / c.n;
    } else {
      l = 0.;
      p = c.n > 0. ? kHalfPi : -kHalfPi;
    }
  } else if (c.kind == GSKYHIP_CRS_SINU) {  // gn_sinu.cpp s_inverse (m=0, n=1)
    p = yn;
    l = xn / cos(yn);
  } else if (c.kind == GSKYHIP_CRS_TMERC) {  // tmerc.cpp exact_e_inv
    if (!tm_inv(c, xn, yn, l, p)) return false;
  } else if (c.kind == GSKYHIP_CRS_LCC) {  // lcc.cpp e_inverse
    if (!lcc_inv(c, xn, yn, l, p)) return false;
  } else if (c.kind == GSKYHIP_CRS_STERE_POLAR) {  // stere.cpp e_inverse (polar)
    if (!stere_inv(c, xn, yn, l, p)) return false;
  } else {
    return false;
  }
  if (l == HUGE_VAL || p == HUGE_VAL || l != l || p != p) return false;
  l = l + c.lam0;
  lam = adjlon(l);
  phi = p;
  return true;
}

// pj_fwd: (lam, phi) radians -> CRS coordinates.
__host__ __device__ inline bool crs_forward(const gskyhip_crs &c, double lam, double phi, double &x, double &y) {
  if (c.kind == GSKYHIP_CRS_LONGLAT) {  // +proj=unitconvert rad -> deg
    x = lam * kR2D;
    y = phi * kR2D;
    return true;
  }
  double t = (phi < 0 ? -phi : phi) - kHalfPi;
  if (t > 1e-12 || lam > 10 || lam < -10) return false;
  if (phi > kHalfPi) phi = kHalfPi;
  if (phi < -kHalfPi) phi = -kHalfPi;
  lam = lam - c.lam0;
  lam = adjlon(lam);
  double xn, yn;
  if (c.kind == GSKYHIP_CRS_WEBMERC) {  // merc.cpp s_forward
    if (fabs(fabs(phi) - kHalfPi) <= 1.e-10) return false;
    xn = c.k0 * lam;
    yn = c.k0 * log(tan(kFortPi + .5 * phi));
  } else if (c.kind == GSKYHIP_CRS_AEA) {  // aea.cpp e_forward
    double rho = c.c - (c.es > 0. ? c.n * qsfn(sin(phi), c.e, c.one_es) : (c.n + c.n) * sin(phi));
    if (rho < 0.) return false;
    rho = c.dd * sqrt(rho);
    lam *= c.n;
    xn = rho * sin(lam);
    yn = c.rho0 - rho * cos(lam);
  } else if (c.kind == GSKYHIP_CRS_SINU) {  // gn_sinu.cpp s_forward (m=0, n=1)
    xn = lam * cos(phi);
    yn = phi;
  } else if (c.kind == GSKYHIP_CRS_TMERC) {  // tmerc.cpp exact_e_fwd
    if (!tm_fwd(c, lam, phi, xn, yn)) return false;
  } else if (c.kind == GSKYHIP_CRS_LCC) {  // lcc.cpp e_forward
    if (!lcc_fwd(c, lam, phi, xn, yn)) return false;
  } else if (c.kind == GSKYHIP_CRS_STERE_POLAR) {  // stere.cpp e_forward (polar)
    if (!stere_fwd(c, lam, phi, xn, yn)) return false;
  } else {
    return false;
  }
  if (xn != xn || yn != yn || fabs(xn) == HUGE_VAL || fabs(yn) == HUGE_VAL) return false;
  x = 1.0 * (c.a * xn + c.x0);
  y = 1.0 * (c.a * yn + c.y0);
  return true;
}

// ---------------------------------------------------------------- geolocation arrays
// GDAL 3.0.1's geolocation-array transformer (alg/gdalgeoloc.cpp, [ext]: not
// in /root/reference; restated from its published algorithm, parity
// unpinned), selected by warp.go:128-141 when the request carries GeoLocOpts
// (tile_grpc.go:338-350: X_DATASET / Y_DATASET / X_BAND / Y_BAND /
// PIXEL_OFFSET / LINE_OFFSET / PIXEL_STEP / LINE_STEP).  The source side of
// the GenImgProj transformer is then this instead of the source geotransform
// (createGeoLocTransformer, warp.go:52-67):
//   forward  (source pixel/line -> georeferenced): bilinear interpolation of
//            the geolocation arrays at ((x - PIXEL_OFFSET) / PIXEL_STEP,
//            (y - LINE_OFFSET) / LINE_STEP), the nearest grid square
//            extended beyond the arrays, nodata corners dropping to the
//            edge / corner rules;
//   inverse  (georeferenced -> source pixel/line): the backmap (a regular
//            grid over the arrays' extent, ~1.3 cells per geolocation sample,
//            built by bilinear splatting, averaging and three hole-filling
//            passes -- host.cpp geoloc_backmap), bilinearly interpolated
//            where its four cells are set, else its nearest cell.
struct GeoLocD {
  const double *gx, *gy;       // geolocation arrays, ny rows x nx (device)
  const float *bmx, *bmy;      // backmap, bm_h rows x bm_w: source pixel / line (< 0: none)
  int32_t nx, ny, bm_w, bm_h;
  int32_t has_nodata, _pad;
  double nodata_x;             // GDALGetRasterNoDataValue of the X band
  double pixel_offset, line_offset, pixel_step, line_step;
  double bm_gt[6];             // backmap geotransform (north up)
};

__host__ __device__ inline bool geoloc_forward(const GeoLocD &g, double &x, double &y) {
  if (x == HUGE_VAL || y == HUGE_VAL) return false;
  const double px = (x - g.pixel_offset) / g.pixel_step;
  const double ln = (y - g.line_offset) / g.line_step;
  int ix = go_cvtt32(px), iy = go_cvtt32(ln);   // static_cast<int> on x86: out of range -> INT_MIN
  ix = ix < 0 ? 0 : ix;
  ix = ix > g.nx - 1 ? g.nx - 1 : ix;
  iy = iy < 0 ? 0 : iy;
  iy = iy > g.ny - 1 ? g.ny - 1 : iy;
  const int64_t o = (int64_t)iy * g.nx + ix;
  const double *gx = g.gx + o, *gy = g.gy + o;
  const double nd = g.nodata_x;
  if (g.has_nodata && gx[0] == nd) return false;
  const double fx = px - ix, fy = ln - iy;
  if (ix + 1 < g.nx && iy + 1 < g.ny &&
      (!g.has_nodata || (gx[1] != nd && gx[g.nx] != nd && gx[g.nx + 1] != nd))) {
    x = (1 - fy) * (gx[0] + fx * (gx[1] - gx[0])) + fy * (gx[g.nx] + fx * (gx[g.nx + 1] - gx[g.nx]));
    y = (1 - fy) * (gy[0] + fx * (gy[1] - gy[0])) + fy * (gy[g.nx] + fx * (gy[g.nx + 1] - gy[g.nx]));
  } else if (ix + 1 < g.nx && (!g.has_nodata || gx[1] != nd)) {
    x = gx[0] + fx * (gx[1] - gx[0]);
    y = gy[0] + fx * (gy[1] - gy[0]);
  } else if (iy + 1 < g.ny && (!g.has_nodata || gx[g.nx] != nd)) {
    x = gx[0] + fy * (gx[g.nx] - gx[0]);
    y = gy[0] + fy * (gy[g.nx] - gy[0]);
  } else {
    x = gx[0];
    y = gy[0];
  }
  return true;
}

__host__ __device__ inline bool geoloc_inverse(const GeoLocD &g, double &x, double &y) {
  if (x == HUGE_VAL || y == HUGE_VAL) return false;
  const double bx = (x - g.bm_gt[0]) / g.bm_gt[1] - 0.5;
  const double by = (y - g.bm_gt[3]) / g.bm_gt[5] - 0.5;
  if (!(bx > -0.5 && by > -0.5 && bx < g.bm_w - 0.5 && by < g.bm_h - 0.5)) return false;   // NaN too
  const int ix = (int)floor(bx), iy = (int)floor(by);
  const int64_t w = g.bm_w;
  if (ix >= 0 && iy >= 0 && ix + 1 < g.bm_w && iy + 1 < g.bm_h) {
    const int64_t o = iy * w + ix;
    const float *mx = g.bmx + o, *my = g.bmy + o;
    if (mx[0] >= 0 && mx[1] >= 0 && mx[w] >= 0 && mx[w + 1] >= 0) {
      const double fx = bx - ix, fy = by - iy;
      x = (1 - fx) * (1 - fy) * mx[0] + fx * (1 - fy) * mx[1] + (1 - fx) * fy * mx[w] + fx * fy * mx[w + 1];
      y = (1 - fx) * (1 - fy) * my[0] + fx * (1 - fy) * my[1] + (1 - fx) * fy * my[w] + fx * fy * my[w + 1];
      return true;
    }
  }
  const int nx = (int)floor(bx + 0.5), ny = (int)floor(by + 0.5);   // nearest cell (in range by the test above)
  const int64_t o = (int64_t)ny * w + nx;
  if (g.bmx[o] < 0) return false;
  x = g.bmx[o];
  y = g.bmy[o];
  return true;
}

// GenImgProj transformer state of one (tile, granule) pair.  gl: a
// geolocation-array source transformer in place of src_gt (warp.go:128-141).
struct Xform {
  gskyhip_crs src, dst;
  double src_gt[6], src_igt[6], dst_gt[6], dst_igt[6];
  int reproject;
  const GeoLocD *gl;   // set at every construction (NULL: the source geotransform)
};

__host__ __device__ inline void inv_geot(const double *gt, double *o) {  // GDALInvGeoTransform
  if (gt[2] == 0.0 && gt[4] == 0.0 && gt[1] != 0.0 && gt[5] != 0.0) {
    o[0] = -gt[0] / gt[1];
    o[1] = 1.0 / gt[1];
    o[2] = 0.0;
    o[3] = -gt[3] / gt[5];
    o[4] = 0.0;
    o[5] = 1.0 / gt[5];
    return;
  }
  double det = gt[1] * gt[5] - gt[2] * gt[4];
  double inv_det = 1.0 / det;
  o[0] = (gt[2] * gt[3] - gt[0] * gt[5]) * inv_det;
  o[3] = (-gt[1] * gt[3] + gt[0] * gt[4]) * inv_det;
  o[1] = gt[5] * inv_det;
  o[4] = -gt[4] * inv_det;
  o[2] = -gt[2] * inv_det;
  o[5] = gt[1] * inv_det;
}

__host__ __device__ inline bool crs_same(const gskyhip_crs &a, const gskyhip_crs &b) {
  return a.kind == b.kind && a.a == b.a && a.es == b.es && a.lam0 == b.lam0 && a.phi0 == b.phi0 &&
         a.phi1 == b.phi1 && a.phi2 == b.phi2 && a.x0 == b.x0 && a.y0 == b.y0 && a.k0 == b.k0;
}

// GDALGenImgProjTransform for one point; dst_to_src selects the direction.
__device__ inline bool xform_point(const Xform &t, bool dst_to_src, double &x, double &y) {
  const double *g1 = dst_to_src ? t.dst_gt : t.src_gt;
  const double *g2 = dst_to_src ? t.src_igt : t.dst_igt;
  double X, Y;
  if (!dst_to_src && t.gl) {   // geolocation arrays: source pixel/line -> georeferenced
    X = x; Y = y;
    if (!geoloc_forward(*t.gl, X, Y)) return false;
  } else {
    X = g1[0] + x * g1[1] + y * g1[2];
    Y = g1[3] + x * g1[4] + y * g1[5];
  }
  if (t.reproject) {
    double lam, phi;
    if (dst_to_src) {
      if (!crs_inverse(t.dst, X, Y, lam, phi)) return false;
      if (!crs_forward(t.src, lam, phi, X, Y)) return false;
    } else {
      if (!crs_inverse(t.src, X, Y, lam, phi)) return false;
      if (!crs_forward(t.dst, lam, phi, X, Y)) return false;
    }
  }
  if (dst_to_src && t.gl) {    // georeferenced -> source pixel/line through the backmap
    x = X; y = Y;
    return geoloc_inverse(*t.gl, x, y);
  }
  x = g2[0] + X * g2[1] + Y * g2[2];
  y = g2[3] + X * g2[4] + Y * g2[5];
  return true;
}

// ---------------------------------------------------------------- separable transform
// dst -> src of a north-up destination geotransform (gt[2] = gt[4] = 0) and
// a cylindrical destination CRS (Web Mercator, lon/lat): X and lambda depend
// on the pixel column only, Y and phi on the row only.  The points of a row
// record (planning) then share per-column parts (SepCol, once per pair) and
// a per-row part (SepRow, once per row); sep_point() combines them with the
// expressions and operation order of xform_point(t, true, ...) -- bit for
// bit: the dropped y*gt[2] / x*gt[4] terms are signed zeros for the positive
// pixel coordinates used, and adding a zero leaves every other value alone.
struct SepCol { double lam, sl, cl; int32_t ok, _pad; };
struct SepRow { double phi, r1, r2; int32_t ok, _pad; };

__host__ __device__ inline bool sep_possible(const Xform &t) {
  const int dk = t.dst.kind, sk = t.src.kind;
  return t.reproject && !t.gl && t.dst_gt[2] == 0.0 && t.dst_gt[4] == 0.0 &&
         (dk == GSKYHIP_CRS_WEBMERC || dk == GSKYHIP_CRS_LONGLAT) &&
         (sk == GSKYHIP_CRS_WEBMERC || sk == GSKYHIP_CRS_LONGLAT || sk == GSKYHIP_CRS_AEA ||
          sk == GSKYHIP_CRS_SINU);
}

// Column part at pixel column x (y_any: any positive pixel row).
__host__ __device__ inline SepCol sep_col(const Xform &t, double x, double y_any) {
  SepCol c;
  c.sl = c.cl = 0.0;
  c._pad = 0;
  const double *g1 = t.dst_gt;
  const double X = g1[0] + x * g1[1] + y_any * g1[2];
  bool ok = !(X == HUGE_VAL);
  double lam;
  const gskyhip_crs &d = t.dst, &s = t.src;
  if (d.kind == GSKYHIP_CRS_LONGLAT) {        // crs_inverse, unitconvert
    lam = X * kD2R;
  } else {                                    // crs_inverse, merc s_inverse
    const double xn = (X * 1.0 - d.x0) * d.ra;
    double l = xn / d.k0;
    if (l == HUGE_VAL || l != l) ok = false;
    l = l + d.lam0;
    lam = adjlon(l);
  }
  if (s.kind == GSKYHIP_CRS_LONGLAT) {        // crs_forward, unitconvert
    c.sl = lam * kR2D;
  } else {
    if (lam > 10 || lam < -10) ok = false;
    lam = lam - s.lam0;
    lam = adjlon(lam);
    if (s.kind == GSKYHIP_CRS_WEBMERC) {
      c.sl = s.k0 * lam;
    } else if (s.kind == GSKYHIP_CRS_AEA) {
      lam *= s.n;
      c.sl = sin(lam);
      c.cl = cos(lam);
    } else {                                  // SINU: xn = lam * cos(phi)
      c.sl = lam;
    }
  }
  c.lam = lam;
  c.ok = ok ? 1 : 0;
  return c;
}

// Row part at pixel row y (x_any: any positive pixel column).
__host__ __device__ inline SepRow sep_row(const Xform &t, double x_any, double y) {
  SepRow r;
  r.r1 = r.r2 = 0.0;
  r._pad = 0;
  const double *g1 = t.dst_gt;
  const double Y = g1[3] + x_any * g1[4] + y * g1[5];
  bool ok = !(Y == HUGE_VAL);
  double phi;
  const gskyhip_crs &d = t.dst, &s = t.src;
  if (d.kind == GSKYHIP_CRS_LONGLAT) {
    phi = Y * kD2R;
  } else {
    const double yn = (Y * 1.0 - d.y0) * d.ra;
    const double p = kHalfPi - 2. * atan(exp(-yn / d.k0));
    if (p == HUGE_VAL || p != p) ok = false;
    phi = p;
  }
  if (s.kind == GSKYHIP_CRS_LONGLAT) {
    r.r1 = phi * kR2D;
  } else {
    const double tt = (phi < 0 ? -phi : phi) - kHalfPi;
    if (tt > 1e-12) ok = false;
    if (phi > kHalfPi) phi = kHalfPi;
    if (phi < -kHalfPi) phi = -kHalfPi;
    if (s.kind == GSKYHIP_CRS_WEBMERC) {
      if (fabs(fabs(phi) - kHalfPi) <= 1.e-10) ok = false;
      r.r1 = s.k0 * log(tan(kFortPi + .5 * phi));
    } else if (s.kind == GSKYHIP_CRS_AEA) {
      double rho = s.c - (s.es > 0. ? s.n * qsfn(sin(phi), s.e, s.one_es) : (s.n + s.n) * sin(phi));
      if (rho < 0.) ok = false;
      r.r1 = s.dd * sqrt(rho);
    } else {                                  // SINU
      r.r1 = cos(phi);
      r.r2 = phi;
    }
  }
  r.phi = phi;
  r.ok = ok ? 1 : 0;
  return r;
}

// xform_point(t, true, x, y) of the pixel at (column part c, row part r).
__host__ __device__ inline bool sep_point(const Xform &t, const SepCol &c, const SepRow &r, double &x, double &y) {
  if (!c.ok || !r.ok) return false;
  const gskyhip_crs &s = t.src;
  double X, Y;
  if (s.kind == GSKYHIP_CRS_LONGLAT) {
    X = c.sl;
    Y = r.r1;
  } else {
    double xn, yn;
    if (s.kind == GSKYHIP_CRS_WEBMERC) {
      xn = c.sl;
      yn = r.r1;
    } else if (s.kind == GSKYHIP_CRS_AEA) {
      xn = r.r1 * c.sl;
      yn = s.rho0 - r.r1 * c.cl;
    } else {
      xn = c.sl * r.r1;
      yn = r.r2;
    }
    if (xn != xn || yn != yn || fabs(xn) == HUGE_VAL || fabs(yn) == HUGE_VAL) return false;
    X = 1.0 * (s.a * xn + s.x0);
    Y = 1.0 * (s.a * yn + s.y0);
  }
  const double *g2 = t.src_igt;
  x = g2[0] + X * g2[1] + Y * g2[2];
  y = g2[3] + X * g2[4] + Y * g2[5];
  return true;
}

// ---------------------------------------------------------------- plans
// Per (tile, granule) pair, produced by the planning kernels.
struct PairPlan {
  double src_gt[6];       // overview-rescaled source geotransform (warp.go:186-189)
  double src_igt[6];
  const void *band;       // chosen level (warp.go:181-183)
  int32_t band_x, band_y;
  int32_t xoff, yoff, w, h;  // window (warp.go:200-217)
  int32_t granule, tile;
  int32_t src_dtype;      // GDAL type of the level
  int32_t out_dtype;      // after warp.go:236-243 promotion (SignedByte kept as Byte here)
  int32_t ns;             // namespace slot
  int32_t is_mask;        // raster of the mask layer
  int32_t in_stack;       // merged into a canvas (not a non-inclusive mask)
  int32_t fill_mode;      // 1: r.TimeStamp < canvas.TimeStamp (tile_merger.go:47)
  int32_t mask_pair;      // pair whose mask applies (maskMap[geoStamp]) or -1
  int32_t status;         // 0 ok, else error code
  double nodata;          // Raster.NoData (warp.go:246)
  Val fill;               // GDALCopyWords(nodata -> out_dtype), warp.go:247
  int32_t signed_byte;
  double stamp;           // TimeStamp + fnv32a(Polygon), tile_merger.go:473-475
  double ts;              // TimeStamp
  int32_t has_nodata;
  int32_t _pad;
};

struct TilePlan {
  int32_t n_entries;          // pairs merged (in order[] slots)
  int32_t status;
  int32_t complex;            // some row needs exact transforms at render time
  int32_t vt;                 // common value type of every entry (0: mixed -> general kernel)
  int32_t created[4];
  int32_t dtype[4];
  double nodata[4];           // canvas NoData (first raster of the ns)
  int32_t e0;                 // first merge entry (order[pair_begin]), -1 when none
  int32_t _pad;
};

// Render-time descriptor of one pair (indexed by pair), written by
// plan_tiles_kernel: everything the fused kernel reads per (row, pair).
struct EntryD {
  const void *band;
  int32_t band_x, band_y;
  int32_t xoff, yoff, w, h;
  int32_t ns, fill_mode, mask_pair, src_dtype;
  int32_t out_dtype, has_nodata;
  Val nd, fill;               // Go T(r.NoData) of the merge; GDALCopyWords window fill
  double nodata64;
  int64_t row_base;           // pair * max_h (index of row 0 in the row records)
};

// Row record of the approximate transformer for one window row.
enum RowKind : int32_t { ROW_LINEAR = 0, ROW_EXACT = 1, ROW_POOL = 2, ROW_DESCEND = 3 };
struct RowRec {
  double v[6];   // LINEAR: xs0, ys0, dX, dY ; DESCEND: xs0, ys0, xs1, ys1, xs2, ys2
  int32_t kind, nleaf, pool_off;
  int32_t inside;   // LINEAR: 1 when every window pixel's NN source pixel is inside the band
};

// NN source pixel of window pixel `dist` of a LINEAR row (the expressions of
// lin_coords() + nn_px()): false where the reference's window fill applies.
__device__ __forceinline__ bool linear_nn_px(const RowRec &r, int dist, int bx, int by) {
  const double sx = r.v[0] + r.v[2] * (double)dist, sy = r.v[1] + r.v[3] * (double)dist;
  const int ix = __double2int_rz(sx + 1.0e-10), iy = __double2int_rz(sy + 1.0e-10);
  return sx >= 0.0 && sy >= 0.0 && ix < bx && iy < by;
}

// RowRec.inside: fl(a + fl(b * d)) and the truncation after + 1e-10 are
// monotone in d, so every pixel of the row [0, n) is inside when both end
// pixels are.  The NN band kernel then drops the per-pixel range tests and
// the window fill select (render_nn.h).
__device__ __forceinline__ bool linear_row_inside(const RowRec &r, int n, int bx, int by) {
  return n > 0 && linear_nn_px(r, 0, bx, by) && linear_nn_px(r, n - 1, bx, by);
}

// The in-band span of a LINEAR row (round 6): the window pixels [lo, hi) whose
// NN source pixel lies in the band -- every other pixel of the row takes the
// window fill.  Kept in RowRec.v[4] as the bits lo | hi << 32 (v[4..5] only
// carry DESCEND rows' points); kSpanNone: not computed.  Each of the four
// tests of linear_nn_px() (sx >= 0, trunc(sx + 1e-10) < bx, same in y) is
// monotone in d (the argument of linear_row_inside()), so the pixels passing
// them form one interval: lo is the first pixel passing the tests that turn
// true as d grows, hi the first one after it failing a test that turns false.
// The NN band kernel folds such a row of a multi-entry tile like a window
// edge row over the span, and drops the row outright when the span is empty
// (the window fill equal to the nodata, render_nn.h).
constexpr int64_t kSpanNone = -1;
__device__ __forceinline__ int64_t span_bits(int lo, int hi) {
  return (int64_t)(uint32_t)lo | ((int64_t)(uint32_t)hi << 32);
}
__device__ __forceinline__ int64_t linear_row_span(const RowRec &r, int n, int bx, int by) {
  if (n <= 0) return span_bits(0, 0);
  if (!(isfinite(r.v[0]) && isfinite(r.v[1]) && isfinite(r.v[2]) && isfinite(r.v[3]))) return kSpanNone;
  const bool xup = r.v[2] >= 0.0, yup = r.v[3] >= 0.0;
  // rising tests: true from some d on; falling: true up to some d
  auto tests = [&](int d, bool &rise, bool &fall) {
    const double sx = r.v[0] + r.v[2] * (double)d, sy = r.v[1] + r.v[3] * (double)d;
    const int ix = __double2int_rz(sx + 1.0e-10), iy = __double2int_rz(sy + 1.0e-10);
    const bool x0 = sx >= 0.0, x1 = ix < bx, y0 = sy >= 0.0, y1 = iy < by;
    rise = (xup ? x0 : x1) && (yup ? y0 : y1);
    fall = (xup ? x1 : x0) && (yup ? y1 : y0);
  };
  bool rs, fl;
  int a = 0, b = n;   // lo: first d in [0, n) with the rising tests true (n: none)
  while (a < b) {
    const int m = (a + b) >> 1;
    tests(m, rs, fl);
    if (rs) b = m; else a = m + 1;
  }
  const int lo = a;
  b = n;              // hi: first d in [lo, n) with a falling test false (n: none)
  while (a < b) {
    const int m = (a + b) >> 1;
    tests(m, rs, fl);
    if (!fl) b = m; else a = m + 1;
  }
  return lo < a ? span_bits(lo, a) : span_bits(0, 0);
}
// 32.32 fixed-point form of an `inside` LINEAR row (round 4), written beside
// the RowRec by plan_row: x0 = round(xs0 * 2^32), dx = round(dX * 2^32), same
// for y.  Window pixel d's fixed coordinate x0 + d * dx is within
// 2^-33 * (d + 1) of the real xs0 + dX * d, and the reference's
// fl(fl(xs0 + fl(dX * d)) + 1e-10) is within 1e-10 + a few ulps of it (every
// coordinate < 2^20, so an ulp is <= 2^-32): with d < kFixMaxW the two differ
// by < 2^-20.  Wherever the fixed value's fraction is at least kFixMargin
// (2^-19) away from an integer, both truncate to the same source pixel, so the
// NN band kernel takes the integer part of the fixed value and falls back to
// the fp64 expressions only for a row where some pixel is closer than that
// (render_nn.h nn_fix_row).  x0 == kFixNone: no fixed form (not LINEAR +
// inside, coordinates too large, window too wide).
struct RowFix {
  int64_t x0, y0, dx, dy;
};
constexpr int64_t kFixNone = (int64_t)0x8000000000000000ull;
constexpr int kFixMaxW = 4096;
constexpr uint32_t kFixMargin = 1u << 13;   // 2^-19 in units of 2^-32

__device__ __forceinline__ bool fix_range_ok(double v0, double dv, int n) {
  const double lim = 1048576.0;   // 2^20
  const double v1 = v0 + dv * (double)n;
  return fabs(v0) < lim && fabs(v1) < lim && fabs(dv) < 1024.0;
}

// need_inside: the NN kernel's rows (their fixed form is used only where
// every source pixel lies in the band); the bilinear kernel takes any LINEAR row.
__device__ __forceinline__ RowFix row_fix(const RowRec &r, int n, bool need_inside) {
  RowFix f;
  f.x0 = kFixNone; f.y0 = 0; f.dx = 0; f.dy = 0;
  if (r.kind == ROW_LINEAR && (r.inside || !need_inside) && n > 0 && n <= kFixMaxW && fix_range_ok(r.v[0], r.v[2], n) &&
      fix_range_ok(r.v[1], r.v[3], n)) {
    const double s = 4294967296.0;   // scaling by 2^32 is exact
    f.x0 = __double2ll_rn(r.v[0] * s);
    f.y0 = __double2ll_rn(r.v[1] * s);
    f.dx = __double2ll_rn(r.v[2] * s);
    f.dy = __double2ll_rn(r.v[3] * s);
  }
  return f;
}

struct Leaf {
  double xs0, ys0, dX, dY;
  int32_t start, kind;   // LeafKind
};
// LINEAR: xs0 + dX * (i - start); one pixel's exact point is a LINEAR leaf
// with dX = dY = 0.  EXACT: [start, next start) transformed per pixel at
// render time (complex tiles only).  FAILED: the pixel's exact transform
// failed (window fill).  PENDING: planning-internal, pixel `start` of pair
// (int)dX, window row (int)dY awaiting plan_exact_kernel.
enum LeafKind : int32_t { LEAF_LINEAR = 0, LEAF_EXACT = 1, LEAF_FAILED = 2, LEAF_PENDING = 3 };

constexpr int kMaxLeavesLocal = 16;

}  // namespace gsky
