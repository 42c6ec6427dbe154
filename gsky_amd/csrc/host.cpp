// host.cpp -- C-ABI of libgskyhip.so (include/gskyhip.h).
//
// Host side of the MI355X path: SRS parsing, Go strconv mask parsing, the
// (path, band) -> HBM granule registry behind the warp_operation_fast
// drop-in, and the launch sequences.  All pixel work runs in the HIP kernels
// of render.hip / stages.hip / drill.hip; nothing here falls back to the CPU.
#include <hip/hip_runtime.h>
#include <sys/stat.h>

#include <atomic>
#include <chrono>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/gskyhip.h"
#include "drill.h"
#include "gsky_device.h"
#include "ingest.h"
#include "render.h"
#include "stages.h"
#include "service.h"
#include "warp_batch.h"

using namespace gsky;

namespace {

// ---------------------------------------------------------------- SRS parsing
constexpr double kD2R_h = 0.017453292519943295769236907684886;

void set_ellps(gskyhip_crs *c, double a, double rf) {
  c->a = a;
  c->ra = 1.0 / a;
  if (rf == 0.0) c->es = 0.0;
  else { double f = 1.0 / rf; c->es = 2 * f - f * f; }
  c->e = std::sqrt(c->es);
  c->one_es = 1.0 - c->es;
}

double h_qsfn(double sinphi, double e, double one_es) {
  if (e >= 1.0e-7) {
    double con = e * sinphi;
    double div1 = 1.0 - con * con;
    double div2 = 1.0 + con;
    if (div1 == 0.0 || div2 == 0.0) return HUGE_VAL;
    return one_es * (sinphi / div1 - (.5 / e) * std::log((1. - con) / div2));
  }
  return sinphi + sinphi;
}

// aea.cpp setup() of PROJ 6.1.1
int aea_setup(gskyhip_crs *c) {
  const double phi1 = c->phi1, phi2 = c->phi2;
  if (std::fabs(phi1 + phi2) < 1e-10) return GSKYHIP_E_CRS;
  double sinphi = std::sin(phi1), cosphi = std::cos(phi1);
  c->n = sinphi;
  const bool secant = std::fabs(phi1 - phi2) >= 1e-10;
  if (c->es > 0.) {
    const double m1 = cosphi / std::sqrt(1. - c->es * sinphi * sinphi);
    const double ml1 = h_qsfn(sinphi, c->e, c->one_es);
    if (secant) {
      const double s2 = std::sin(phi2), c2 = std::cos(phi2);
      const double m2 = c2 / std::sqrt(1. - c->es * s2 * s2);
      const double ml2 = h_qsfn(s2, c->e, c->one_es);
      if (ml2 == ml1) return GSKYHIP_E_CRS;
      c->n = (m1 * m1 - m2 * m2) / (ml2 - ml1);
    }
    c->ec = 1. - .5 * c->one_es * std::log((1. - c->e) / (1. + c->e)) / c->e;
    c->c = m1 * m1 + c->n * ml1;
    c->dd = 1. / c->n;
    c->rho0 = c->dd * std::sqrt(c->c - c->n * h_qsfn(std::sin(c->phi0), c->e, c->one_es));
  } else {
    if (secant) c->n = .5 * (c->n + std::sin(phi2));
    const double n2 = c->n + c->n;
    c->c = cosphi * cosphi + n2 * sinphi;
    c->dd = 1. / c->n;
    c->rho0 = c->dd * std::sqrt(c->c - n2 * std::sin(c->phi0));
  }
  return 0;
}

// tmerc.cpp setup_exact() of PROJ 6.1.1 (the Poder / Engsager series,
// gsky_device.h tm_fwd / tm_inv): third flattening n, the 6th-order series
// coefficients, the normalised meridian quadrant Qn and the northing of the
// origin latitude Zb.  Ellipsoids only (the spherical tmerc is not carried).
int tmerc_setup(gskyhip_crs *c) {
  if (!(c->es > 0)) return GSKYHIP_E_CRS;
  c->kind = GSKYHIP_CRS_TMERC;
  const double f = c->es / (1 + std::sqrt(1 - c->es));
  const double n = f / (2 - f);
  double np = n;
  double *cgb = c->tm_cgb, *cbg = c->tm_cbg, *utg = c->tm_utg, *gtu = c->tm_gtu;
  cgb[0] = n * (2 + n * (-2 / 3.0 + n * (-2 + n * (116 / 45.0 + n * (26 / 45.0 + n * (-2854 / 675.0))))));
  cbg[0] = n * (-2 + n * (2 / 3.0 + n * (4 / 3.0 + n * (-82 / 45.0 + n * (32 / 45.0 + n * (4642 / 4725.0))))));
  np *= n;
  cgb[1] = np * (7 / 3.0 + n * (-8 / 5.0 + n * (-227 / 45.0 + n * (2704 / 315.0 + n * (2323 / 945.0)))));
  cbg[1] = np * (5 / 3.0 + n * (-16 / 15.0 + n * (-13 / 9.0 + n * (904 / 315.0 + n * (-1522 / 945.0)))));
  np *= n;
  cgb[2] = np * (56 / 15.0 + n * (-136 / 35.0 + n * (-1262 / 105.0 + n * (73814 / 2835.0))));
  cbg[2] = np * (-26 / 15.0 + n * (34 / 21.0 + n * (8 / 5.0 + n * (-12686 / 2835.0))));
  np *= n;
  cgb[3] = np * (4279 / 630.0 + n * (-332 / 35.0 + n * (-399572 / 14175.0)));
  cbg[3] = np * (1237 / 630.0 + n * (-12 / 5.0 + n * (-24832 / 14175.0)));
  np *= n;
  cgb[4] = np * (4174 / 315.0 + n * (-144838 / 6237.0));
  cbg[4] = np * (-734 / 315.0 + n * (109598 / 31185.0));
  np *= n;
  cgb[5] = np * (601676 / 22275.0);
  cbg[5] = np * (444337 / 155925.0);
  np = n * n;
  c->tm_qn = c->k0 / (1 + n) * (1 + np * (1 / 4.0 + np * (1 / 64.0 + np / 256.0)));
  utg[0] = n * (-0.5 + n * (2 / 3.0 + n * (-37 / 96.0 + n * (1 / 360.0 + n * (81 / 512.0 + n * (-96199 / 604800.0))))));
  gtu[0] = n * (0.5 + n * (-2 / 3.0 + n * (5 / 16.0 + n * (41 / 180.0 + n * (-127 / 288.0 + n * (7891 / 37800.0))))));
  utg[1] = np * (-1 / 48.0 + n * (-1 / 15.0 + n * (437 / 1440.0 + n * (-46 / 105.0 + n * (1118711 / 3870720.0)))));
  gtu[1] = np * (13 / 48.0 + n * (-3 / 5.0 + n * (557 / 1440.0 + n * (281 / 630.0 + n * (-1983433 / 1935360.0)))));
  np *= n;
  utg[2] = np * (-17 / 480.0 + n * (37 / 840.0 + n * (209 / 4480.0 + n * (-5569 / 90720.0))));
  gtu[2] = np * (61 / 240.0 + n * (-103 / 140.0 + n * (15061 / 26880.0 + n * (167603 / 181440.0))));
  np *= n;
  utg[3] = np * (-4397 / 161280.0 + n * (11 / 504.0 + n * (830251 / 7257600.0)));
  gtu[3] = np * (49561 / 161280.0 + n * (-179 / 168.0 + n * (6601661 / 7257600.0)));
  np *= n;
  utg[4] = np * (-4583 / 161280.0 + n * (108847 / 3991680.0));
  gtu[4] = np * (34729 / 80640.0 + n * (-3418889 / 1995840.0));
  np *= n;
  utg[5] = np * (-20648693 / 638668800.0);
  gtu[5] = np * (212378941 / 319334400.0);
  const double Z = tm_gatg(cbg, 6, c->phi0);   // Gaussian latitude of the origin
  c->tm_zb = -c->tm_qn * (Z + tm_clens(gtu, 6, 2 * Z));
  return 0;
}

// lcc.cpp setup() of PROJ 6.1.1 for an ellipsoid (pj_msfn / pj_tsfn): the
// cone constant n (one standard parallel: its sine; two: the secant form),
// c and rho0.  phi1 / phi2 / phi0 / k0 set by the caller.
int lcc_setup(gskyhip_crs *c) {
  if (!(c->es > 0)) return GSKYHIP_E_CRS;   // the spherical lcc is not carried
  c->kind = GSKYHIP_CRS_LCC;
  const double phi1 = c->phi1, phi2 = c->phi2;
  if (std::fabs(phi1 + phi2) < 1e-10) return GSKYHIP_E_CRS;
  double sinphi = std::sin(phi1);
  const double cosphi = std::cos(phi1);
  c->n = sinphi;
  const bool secant = std::fabs(phi1 - phi2) >= 1e-10;
  auto msfn = [&](double s, double co) { return co / std::sqrt(1. - c->es * s * s); };
  const double m1 = msfn(sinphi, cosphi);
  const double ml1 = lcc_tsfn(phi1, sinphi, c->e);
  if (secant) {
    sinphi = std::sin(phi2);
    c->n = std::log(m1 / msfn(sinphi, std::cos(phi2)));
    c->n /= std::log(ml1 / lcc_tsfn(phi2, sinphi, c->e));
  }
  c->c = c->rho0 = m1 * std::pow(ml1, -c->n) / c->n;
  c->rho0 *= (std::fabs(std::fabs(c->phi0) - kHalfPi) < 1e-10) ? 0.
                                                                : std::pow(lcc_tsfn(c->phi0, std::sin(c->phi0), c->e), c->n);
  return 0;
}

// stere.cpp setup() of PROJ 6.1.1, polar aspects on an ellipsoid: phi0 =
// +-pi/2 picks the pole, |lat_ts| the true-scale parallel (pi/2: k0 at the
// pole); akm1 into c->c.
int stere_polar_setup(gskyhip_crs *c, double phi0, bool has_ts, double lat_ts) {
  if (!(c->es > 0)) return GSKYHIP_E_CRS;   // the spherical stere is not carried
  if (std::fabs(std::fabs(phi0) - kHalfPi) >= 1e-10) return GSKYHIP_E_CRS;   // oblique / equatorial: not carried
  c->kind = GSKYHIP_CRS_STERE_POLAR;
  c->phi0 = phi0 < 0 ? -kHalfPi : kHalfPi;
  const double phits = std::fabs(has_ts ? lat_ts : kHalfPi);
  c->phi1 = phits;
  const double e = c->e;
  if (std::fabs(phits - kHalfPi) < 1e-10) {
    c->c = 2. * c->k0 / std::sqrt(std::pow(1 + e, 1 + e) * std::pow(1 - e, 1 - e));
  } else {
    double t = std::sin(phits);
    c->c = std::cos(phits) / lcc_tsfn(phits, t, e);
    t *= e;
    c->c /= std::sqrt(1. - t * t);
  }
  return 0;
}

// utm.cpp setup: zone -> central meridian, k0 0.9996, false easting 500 km,
// false northing 10,000 km in the south.
int utm_setup(gskyhip_crs *c, int zone, bool south) {
  if (zone < 1 || zone > 60) return GSKYHIP_E_CRS;
  c->lam0 = (zone - 0.5) * (kPi / 30.0) - kPi;   // PROJ: (zone - .5) * M_PI / 30. - M_PI
  c->phi0 = 0.0;
  c->k0 = 0.9996;
  c->x0 = 500000.0;
  c->y0 = south ? 10000000.0 : 0.0;
  return tmerc_setup(c);
}

double proj_param(const std::string &s, const char *key, double dflt, bool *found = nullptr) {
  const std::string k = std::string(key) + "=";
  size_t pos = 0;
  while ((pos = s.find(k, pos)) != std::string::npos) {
    if (pos == 0 || s[pos - 1] == ' ' || s[pos - 1] == '+') {
      if (found) *found = true;
      return std::strtod(s.c_str() + pos + k.size(), nullptr);
    }
    pos += k.size();
  }
  if (found) *found = false;
  return dflt;
}

int crs_epsg(int code, gskyhip_crs *c) {
  std::memset(c, 0, sizeof(*c));
  c->k0 = 1.0;
  switch (code) {
    case 4326: c->kind = GSKYHIP_CRS_LONGLAT; set_ellps(c, 6378137.0, 298.257223563); return 0;
    case 4283: c->kind = GSKYHIP_CRS_LONGLAT; set_ellps(c, 6378137.0, 298.257222101); return 0;
    case 3857: case 900913: c->kind = GSKYHIP_CRS_WEBMERC; set_ellps(c, 6378137.0, 0.0); return 0;
    case 3577:
      c->kind = GSKYHIP_CRS_AEA;
      set_ellps(c, 6378137.0, 298.257222101);
      c->lam0 = 132.0 * kD2R_h; c->phi0 = 0.0; c->phi1 = -18.0 * kD2R_h; c->phi2 = -36.0 * kD2R_h;
      return aea_setup(c);
    default: break;
  }
  // Transverse Mercator zones: WGS 84 / UTM north (326zz) and south (327zz),
  // GDA94 / MGA (283zz, zones 48-58) and GDA2020 / MGA (78zz, zones 46-59);
  // both GDA datums on GRS80, taken without a datum shift like EPSG:3577
  if (code >= 32601 && code <= 32660) { set_ellps(c, 6378137.0, 298.257223563); return utm_setup(c, code - 32600, false); }
  if (code >= 32701 && code <= 32760) { set_ellps(c, 6378137.0, 298.257223563); return utm_setup(c, code - 32700, true); }
  if (code >= 28348 && code <= 28358) { set_ellps(c, 6378137.0, 298.257222101); return utm_setup(c, code - 28300, true); }
  if (code >= 7846 && code <= 7859) { set_ellps(c, 6378137.0, 298.257222101); return utm_setup(c, code - 7800, true); }
  if (code == 3031 || code == 3413 || code == 3976) {   // WGS 84 polar stereographic (Antarctic, NSIDC)
    set_ellps(c, 6378137.0, 298.257223563);
    c->lam0 = (code == 3413 ? -45.0 : 0.0) * kD2R_h;
    const double ts = code == 3031 ? -71.0 : code == 3413 ? 70.0 : -70.0;
    return stere_polar_setup(c, (ts < 0 ? -90.0 : 90.0) * kD2R_h, true, ts * kD2R_h);
  }
  if (code == 32661 || code == 32761) {   // WGS 84 / UPS North / South
    set_ellps(c, 6378137.0, 298.257223563);
    c->k0 = 0.994; c->x0 = 2000000.0; c->y0 = 2000000.0;
    return stere_polar_setup(c, (code == 32661 ? 90.0 : -90.0) * kD2R_h, false, 0.0);
  }
  if (code == 3112 || code == 7845) {   // GDA94 / GDA2020 Geoscience Australia Lambert
    set_ellps(c, 6378137.0, 298.257222101);
    c->phi1 = -18.0 * kD2R_h; c->phi2 = -36.0 * kD2R_h; c->phi0 = 0.0; c->lam0 = 134.0 * kD2R_h;
    return lcc_setup(c);
  }
  return GSKYHIP_E_CRS;
}

int crs_proj4(const std::string &s, gskyhip_crs *c) {
  std::memset(c, 0, sizeof(*c));
  c->k0 = 1.0;
  bool has_a = false;
  double a = proj_param(s, "+a", 0, &has_a);
  double R = proj_param(s, "+R", 0);
  double rf = proj_param(s, "+rf", 0);
  if (s.find("+ellps=GRS80") != std::string::npos) { a = 6378137.0; rf = 298.257222101; has_a = true; }
  else if (s.find("+ellps=WGS84") != std::string::npos || s.find("+datum=WGS84") != std::string::npos) {
    a = 6378137.0; rf = 298.257223563; has_a = true;
  }
  if (R > 0) { a = R; rf = 0; has_a = true; }
  if (!has_a) { a = 6378137.0; rf = 298.257223563; }
  c->lam0 = proj_param(s, "+lon_0", 0) * kD2R_h;
  c->phi0 = proj_param(s, "+lat_0", 0) * kD2R_h;
  c->x0 = proj_param(s, "+x_0", 0);
  c->y0 = proj_param(s, "+y_0", 0);
  if (s.find("+proj=longlat") != std::string::npos || s.find("+proj=latlong") != std::string::npos) {
    c->kind = GSKYHIP_CRS_LONGLAT; set_ellps(c, a, rf); return 0;
  }
  if (s.find("+proj=webmerc") != std::string::npos || (s.find("+proj=merc") != std::string::npos && R > 0)) {
    c->kind = GSKYHIP_CRS_WEBMERC; set_ellps(c, a, 0.0); return 0;
  }
  if (s.find("+proj=aea") != std::string::npos) {
    c->kind = GSKYHIP_CRS_AEA; set_ellps(c, a, rf);
    c->phi1 = proj_param(s, "+lat_1", 0) * kD2R_h;
    c->phi2 = proj_param(s, "+lat_2", 0) * kD2R_h;
    return aea_setup(c);
  }
  if (s.find("+proj=sinu") != std::string::npos) {
    c->kind = GSKYHIP_CRS_SINU; set_ellps(c, a, rf);
    return c->es == 0 ? 0 : GSKYHIP_E_CRS;  // only the spherical form (MODIS)
  }
  if (s.find("+proj=utm") != std::string::npos) {
    set_ellps(c, a, rf);
    bool has_zone = false;
    const double zone = proj_param(s, "+zone", 0, &has_zone);
    if (!has_zone || zone != std::floor(zone)) return GSKYHIP_E_CRS;   // PROJ guesses from lon_0: not carried
    return utm_setup(c, (int)zone, s.find("+south") != std::string::npos);
  }
  if (s.find("+proj=ups") != std::string::npos) {   // ups: stere at a pole, k0 0.994, false E / N 2000 km
    set_ellps(c, a, rf);
    c->k0 = 0.994; c->x0 = 2000000.0; c->y0 = 2000000.0; c->lam0 = 0.0;
    return stere_polar_setup(c, (s.find("+south") != std::string::npos ? -90.0 : 90.0) * kD2R_h, false, 0.0);
  }
  if (s.find("+proj=stere ") != std::string::npos ||
      (s.size() >= 11 && s.compare(s.size() - 11, 11, "+proj=stere") == 0)) {
    set_ellps(c, a, rf);
    bool has_ts = false, has_k = false;
    const double ts = proj_param(s, "+lat_ts", 0, &has_ts) * kD2R_h;
    c->k0 = proj_param(s, "+k_0", 1.0, &has_k);
    if (!has_k) c->k0 = proj_param(s, "+k", 1.0);
    return stere_polar_setup(c, c->phi0, has_ts, ts);
  }
  if (s.find("+proj=lcc") != std::string::npos) {   // lcc.cpp: one parallel -> the tangent cone at it
    set_ellps(c, a, rf);
    bool has_l1 = false, has_l2 = false, has_l0 = false, has_k = false;
    c->phi1 = proj_param(s, "+lat_1", 0, &has_l1) * kD2R_h;
    c->phi2 = proj_param(s, "+lat_2", 0, &has_l2) * kD2R_h;
    proj_param(s, "+lat_0", 0, &has_l0);
    if (!has_l2) {
      c->phi2 = c->phi1;
      if (!has_l0) c->phi0 = c->phi1;
    }
    c->k0 = proj_param(s, "+k_0", 1.0, &has_k);
    if (!has_k) c->k0 = proj_param(s, "+k", 1.0);
    return lcc_setup(c);
  }
  if (s.find("+proj=tmerc") != std::string::npos || s.find("+proj=etmerc") != std::string::npos) {
    if (s.find("+approx") != std::string::npos) return GSKYHIP_E_CRS;   // Evenden / Snyder series: not carried
    set_ellps(c, a, rf);
    bool has_k = false;
    c->k0 = proj_param(s, "+k_0", 1.0, &has_k);
    if (!has_k) c->k0 = proj_param(s, "+k", 1.0);
    return tmerc_setup(c);
  }
  return GSKYHIP_E_CRS;
}

int parse_srs(const char *srs, gskyhip_crs *c) {
  if (!srs) return GSKYHIP_E_CRS;
  std::string s(srs);
  auto ieq = [](const std::string &a, const char *b) { return strcasecmp(a.c_str(), b) == 0; };
  if (ieq(s, "MODIS") || ieq(s, "SR-ORG:6842")) return crs_proj4("+proj=sinu +R=6371007.181", c);
  if (s.size() > 5 && strncasecmp(s.c_str(), "EPSG:", 5) == 0) return crs_epsg(std::atoi(s.c_str() + 5), c);
  if (s.find("+proj=") != std::string::npos) return crs_proj4(s, c);
  // WKT: a Sinusoidal / Lambert Conformal Conic / Transverse Mercator projection, else the top-level (last) EPSG
  // authority
  if (s.find("PROJECTION[\"Sinusoidal\"]") != std::string::npos) {
    size_t p = s.find("SPHEROID[");
    double a = 6371007.181;
    if (p != std::string::npos) {
      size_t q = s.find(',', p);
      if (q != std::string::npos) a = std::strtod(s.c_str() + q + 1, nullptr);
    }
    char buf[96];
    std::snprintf(buf, sizeof(buf), "+proj=sinu +R=%.17g", a);
    return crs_proj4(buf, c);
  }
  if (s.find("PROJECTION[\"Polar_Stereographic\"]") != std::string::npos) {   // WKT1 (GDAL): latitude_of_origin = lat_ts
    auto param = [&](const char *name, double dflt) {
      const std::string k = std::string("PARAMETER[\"") + name + "\",";
      const size_t p = s.find(k);
      return p == std::string::npos ? dflt : std::strtod(s.c_str() + p + k.size(), nullptr);
    };
    double a = 6378137.0, rf = 298.257223563;
    const size_t p = s.find("SPHEROID[");
    if (p != std::string::npos) {
      const size_t q = s.find(',', p);
      if (q != std::string::npos) {
        char *end = nullptr;
        a = std::strtod(s.c_str() + q + 1, &end);
        if (end && *end == ',') rf = std::strtod(end + 1, nullptr);
      }
    }
    std::memset(c, 0, sizeof(*c));
    set_ellps(c, a, rf);
    const double ts = param("latitude_of_origin", 90.0);
    c->lam0 = param("central_meridian", 0) * kD2R_h;
    c->k0 = param("scale_factor", 1.0);
    c->x0 = param("false_easting", 0);
    c->y0 = param("false_northing", 0);
    return stere_polar_setup(c, (ts < 0 ? -90.0 : 90.0) * kD2R_h, std::fabs(std::fabs(ts) - 90.0) > 1e-12,
                             ts * kD2R_h);
  }
  const bool lcc2 = s.find("PROJECTION[\"Lambert_Conformal_Conic_2SP\"]") != std::string::npos;
  const bool lcc1 = s.find("PROJECTION[\"Lambert_Conformal_Conic_1SP\"]") != std::string::npos;
  if (lcc1 || lcc2) {   // WKT1 Lambert Conformal Conic: its parameters
    auto param = [&](const char *name, double dflt) {
      const std::string k = std::string("PARAMETER[\"") + name + "\",";
      const size_t p = s.find(k);
      return p == std::string::npos ? dflt : std::strtod(s.c_str() + p + k.size(), nullptr);
    };
    double a = 6378137.0, rf = 298.257223563;
    const size_t p = s.find("SPHEROID[");
    if (p != std::string::npos) {
      const size_t q = s.find(',', p);
      if (q != std::string::npos) {
        char *end = nullptr;
        a = std::strtod(s.c_str() + q + 1, &end);
        if (end && *end == ',') rf = std::strtod(end + 1, nullptr);
      }
    }
    std::memset(c, 0, sizeof(*c));
    set_ellps(c, a, rf);
    c->phi0 = param("latitude_of_origin", 0) * kD2R_h;
    c->lam0 = param("central_meridian", 0) * kD2R_h;
    c->x0 = param("false_easting", 0);
    c->y0 = param("false_northing", 0);
    if (lcc2) {
      c->k0 = 1.0;
      c->phi1 = param("standard_parallel_1", 0) * kD2R_h;
      c->phi2 = param("standard_parallel_2", 0) * kD2R_h;
    } else {
      c->k0 = param("scale_factor", 1.0);
      c->phi1 = c->phi2 = c->phi0;
    }
    return lcc_setup(c);
  }
  if (s.find("PROJECTION[\"Transverse_Mercator\"]") != std::string::npos) {   // WKT1 TM: its parameters
    auto param = [&](const char *name, double dflt) {
      const std::string k = std::string("PARAMETER[\"") + name + "\",";
      const size_t p = s.find(k);
      return p == std::string::npos ? dflt : std::strtod(s.c_str() + p + k.size(), nullptr);
    };
    double a = 6378137.0, rf = 298.257223563;
    const size_t p = s.find("SPHEROID[");
    if (p != std::string::npos) {
      const size_t q = s.find(',', p);
      if (q != std::string::npos) {
        char *end = nullptr;
        a = std::strtod(s.c_str() + q + 1, &end);
        if (end && *end == ',') rf = std::strtod(end + 1, nullptr);
      }
    }
    std::memset(c, 0, sizeof(*c));
    set_ellps(c, a, rf);
    const double lat0 = param("latitude_of_origin", 0), cm = param("central_meridian", 0);
    c->k0 = param("scale_factor", 1.0);
    c->x0 = param("false_easting", 0);
    c->y0 = param("false_northing", 0);
    // a UTM zone's parameters become +proj=utm in PROJ 6 (Conversion's
    // isUTM when exporting the PROJ string): the zone's own central meridian
    const double zone = (cm + 183.0) / 6.0;
    if (lat0 == 0 && c->k0 == 0.9996 && c->x0 == 500000.0 && (c->y0 == 0 || c->y0 == 10000000.0) &&
        zone == std::floor(zone) && zone >= 1 && zone <= 60)
      return utm_setup(c, (int)zone, c->y0 != 0);
    c->phi0 = lat0 * kD2R_h;
    c->lam0 = cm * kD2R_h;
    return tmerc_setup(c);
  }
  size_t pos = s.rfind("AUTHORITY[\"EPSG\",\"");
  if (pos != std::string::npos) return crs_epsg(std::atoi(s.c_str() + pos + 18), c);
  pos = s.rfind("ID[\"EPSG\",");
  if (pos != std::string::npos) return crs_epsg(std::atoi(s.c_str() + pos + 10), c);
  return GSKYHIP_E_CRS;
}

// ---------------------------------------------------------------- Go strconv (base 2)
uint64_t go_parse_uint2(const char *s, int bits, bool *syntax = nullptr) {
  const uint64_t maxVal = (bits >= 64) ? UINT64_MAX : ((1ull << bits) - 1);
  if (syntax) *syntax = false;
  if (!s || !*s) { if (syntax) *syntax = true; return 0; }
  uint64_t n = 0;
  for (const char *p = s; *p; p++) {
    const char c = *p;
    int d;
    if (c >= '0' && c <= '9') d = c - '0';
    else if ((c | 0x20) >= 'a' && (c | 0x20) <= 'z') d = (c | 0x20) - 'a' + 10;
    else { if (syntax) *syntax = true; return 0; }
    if (d >= 2) { if (syntax) *syntax = true; return 0; }
    if (n >= UINT64_MAX / 2 + 1) return maxVal;
    n *= 2;
    const uint64_t n1 = n + (uint64_t)d;
    if (n1 < n || n1 > maxVal) return maxVal;
    n = n1;
  }
  return n;
}
int64_t go_parse_int2(const char *s, int bits) {
  if (!s || !*s) return 0;
  bool neg = false;
  if (*s == '+') s++;
  else if (*s == '-') { neg = true; s++; }
  bool syntax = false;
  const uint64_t un = go_parse_uint2(s, bits, &syntax);
  if (syntax) return 0;
  const uint64_t cutoff = 1ull << (bits - 1);
  if (!neg && un >= cutoff) return (int64_t)(cutoff - 1);
  if (neg && un > cutoff) return -(int64_t)cutoff;
  return neg ? -(int64_t)un : (int64_t)un;
}

// Mask specs for the four mask-raster types (tile_merger.go:328-439).
int build_mask_specs(const gskyhip_mask *m, MaskSpecS out[4]) {
  std::memset(out, 0, sizeof(MaskSpecS) * 4);
  if (!m || m->ns < 0) return 0;
  const bool has_value = m->value && *m->value;
  if (!has_value) {
    if (m->n_bit_tests == 0 || m->n_bit_tests % 2 != 0) return GSKYHIP_E_MASK;
  }
  if (m->n_bit_tests > GSKYHIP_MAX_BIT_TESTS) return GSKYHIP_E_ARG;
  const int dts[4] = {GSKYHIP_SIGNEDBYTE, GSKYHIP_BYTE, GSKYHIP_INT16, GSKYHIP_UINT16};
  for (int k = 0; k < 4; k++) {
    MaskSpecS &o = out[k];
    const int dt = dts[k];
    const int bits = (dt == GSKYHIP_INT16 || dt == GSKYHIP_UINT16) ? 16 : 8;
    o.has_value = has_value ? 1 : 0;
    if (has_value) {
      switch (dt) {
        case GSKYHIP_SIGNEDBYTE: o.value = (int8_t)go_parse_uint2(m->value, 8); break;
        case GSKYHIP_BYTE: o.value = (uint8_t)go_parse_uint2(m->value, 8); break;
        case GSKYHIP_INT16: o.value = (int16_t)go_parse_int2(m->value, 16); break;
        default: o.value = (uint16_t)go_parse_uint2(m->value, 16); break;
      }
    } else {
      o.n_tests = m->n_bit_tests / 2;
      for (int j = 0; j < o.n_tests; j++) {
        const int64_t f = go_parse_int2(m->bit_tests[2 * j], bits);
        const int64_t v = go_parse_int2(m->bit_tests[2 * j + 1], bits);
        switch (dt) {
          case GSKYHIP_SIGNEDBYTE: o.filt[j] = (int8_t)f; o.want[j] = (int8_t)v; break;
          case GSKYHIP_BYTE: o.filt[j] = (uint8_t)f; o.want[j] = (uint8_t)v; break;
          case GSKYHIP_INT16: o.filt[j] = (int16_t)f; o.want[j] = (int16_t)v; break;
          default: o.filt[j] = (uint16_t)f; o.want[j] = (uint16_t)v; break;
        }
      }
    }
  }
  return 0;
}

int mask_slot_h(int dtype) {
  switch (dtype) {
    case GSKYHIP_SIGNEDBYTE: return 0;
    case GSKYHIP_BYTE: return 1;
    case GSKYHIP_INT16: return 2;
    case GSKYHIP_UINT16: return 3;
    default: return -1;
  }
}

// ---------------------------------------------------------------- drop-in state
struct Registered {
  gskyhip_granule g;
  gskyhip_crs crs;
  bool has_crs;
  // netCDF: the SRS under srs_cf=yes (netcdfdataset.cpp:3666), and whether
  // either SRS is a projection the warp cannot represent (-> GSKYHIP_E_CRS)
  gskyhip_crs crs_cf;
  bool has_crs_cf = false, bad_crs = false, bad_crs_cf = false;
  std::vector<void *> owned;   // HBM the library allocated for it (ingested files)
  int64_t bytes = 0;           // ... and its size
  uint64_t last_use = 0;       // DropIn::tick of the last batch that used it
  int64_t mtime_ns = 0, fsize = -1;   // the file as ingested (fsize < 0: registered by the caller)
  bool stamped = false;                // the stamp could be taken: re-read the file when it changes
  Registered() { std::memset(&g, 0, sizeof(g)); }
  Registered(const Registered &) = delete;
  Registered &operator=(const Registered &) = delete;
  // The registry and every warp batch in flight that reads the granule hold
  // it (shared_ptr): its HBM is freed when the last of them lets go, so a
  // re-ingest, an eviction or unregister_all never frees what a launched
  // batch still reads.
  ~Registered() {
    for (void *p : owned) (void)hipFree(p);
  }
};
using RegPtr = std::shared_ptr<Registered>;

struct DropIn {
  std::mutex mu;
  std::map<std::pair<std::string, int>, RegPtr> reg;
  uint64_t tick = 0;     // one per warp batch (LRU order of the ingest cache)
  std::map<std::string, std::shared_ptr<struct GeoLocEntry>> geolocs;   // by GeoLocOpts (geoloc_entry)
};
DropIn &dropin() {
  static DropIn *d = new DropIn();   // never destroyed: its entries would call HIP at process exit
  return *d;
}

// HBM the ingested (library-owned) granules may hold before the least
// recently used ones are released: GSKYHIP_INGEST_CACHE_MB, default 32 GiB
// (of 288 GB per MI355X).  Caller-registered granules are never evicted.
int64_t ingest_cache_cap() {
  static const int64_t cap = [] {
    const char *e = std::getenv("GSKYHIP_INGEST_CACHE_MB");
    const long long mb = e ? std::atoll(e) : 32768;
    return (int64_t)(mb > 0 ? mb : 32768) << 20;
  }();
  return cap;
}

// Make room for `need` more bytes of ingested granules: drop the least
// recently used ones that no batch holds (in flight, or being assembled:
// last_use == d.tick).
void evict_for(DropIn &d, int64_t need) {
  const int64_t cap = ingest_cache_cap();
  for (;;) {
    int64_t held = 0;
    auto victim = d.reg.end();
    for (auto it = d.reg.begin(); it != d.reg.end(); ++it) {
      const Registered &R = *it->second;
      held += R.bytes;
      if (R.bytes > 0 && R.last_use < d.tick && it->second.use_count() == 1 &&
          (victim == d.reg.end() || R.last_use < victim->second->last_use))
        victim = it;
    }
    if (held + need <= cap || victim == d.reg.end()) return;   // fits, or nothing evictable: exceed the cap
    d.reg.erase(victim);
  }
}

// mtime (ns) and size of a file; false if it cannot be stat'ed
bool file_stamp(const std::string &path, int64_t &mtime_ns, int64_t &size) {
  std::string f = path;
  if (f.compare(0, 7, "NETCDF:") == 0) {   // NETCDF:file:var / NETCDF:"file":var
    f = f.substr(7);
    if (!f.empty() && f[0] == '"') {
      const size_t q = f.find('"', 1);
      f = q == std::string::npos ? f.substr(1) : f.substr(1, q - 1);
    } else {
      const size_t c = f.rfind(':');
      if (c != std::string::npos) f = f.substr(0, c);
    }
  }
  struct stat st;
  if (stat(f.c_str(), &st) != 0) return false;
  mtime_ns = (int64_t)st.st_mtim.tv_sec * 1000000000 + st.st_mtim.tv_nsec;
  size = (int64_t)st.st_size;
  return true;
}

bool have_gpu() {
  int n = 0;
  return hipGetDeviceCount(&n) == hipSuccess && n > 0;
}

// GDALOpenEx + GDALGetRasterBand of a GeoTIFF (warp.go:89-118) for the
// registry: every level of band `band` decoded into HBM the library owns
// (ingest.hip), registered under (path, band) with the file's SRS.  Returns
// 0, 1 (open failed), 2 (no such band) or GSKYHIP_E_*.  d.mu held.
int ingest_geotiff_locked(DropIn &d, const std::string &path, int band) {
  gskyhip_raster_info info;
  int rc = gskyhip_geotiff_info(path.c_str(), &info);
  if (rc) return rc;
  if (band < 1 || band > info.n_bands) return 2;
  if (!have_gpu()) return GSKYHIP_E_NOGPU;
  RegPtr rp = std::make_shared<Registered>();
  Registered &r = *rp;
  const int ts = type_size(info.dtype);
  if (ts <= 0) return GSKYHIP_E_TYPE;
  int64_t total = 0;
  for (int lv = 0; lv <= info.n_ovr; lv++)
    total += (int64_t)(lv ? info.ovr_xsize[lv - 1] : info.xsize) * (lv ? info.ovr_ysize[lv - 1] : info.ysize) * ts;
  d.reg.erase({path, band});   // a batch still holding the old entry keeps it alive
  evict_for(d, total);
  r.bytes = total;
  r.last_use = d.tick;
  r.stamped = file_stamp(path, r.mtime_ns, r.fsize);
  if (!r.stamped) r.fsize = 0;
  for (int lv = 0; lv <= info.n_ovr; lv++) {
    const int64_t xs = lv ? info.ovr_xsize[lv - 1] : info.xsize, ys = lv ? info.ovr_ysize[lv - 1] : info.ysize;
    void *p = nullptr;
    if (hipMalloc(&p, (size_t)(xs * ys * ts)) != hipSuccess) return GSKYHIP_E_HIP;
    r.owned.push_back(p);
    if ((rc = gskyhip_geotiff_read(path.c_str(), band, lv, p, xs * ys * ts, nullptr))) return rc;
  }
  gskyhip_granule &g = r.g;
  g.data = r.owned[0];
  g.dtype = info.dtype; g.xsize = info.xsize; g.ysize = info.ysize; g.signed_byte = info.signed_byte;
  for (int k = 0; k < 6; k++) g.geot[k] = info.geot[k];
  g.nodata = info.nodata; g.has_nodata = info.has_nodata;
  g.n_ovr = info.n_ovr;
  for (int k = 0; k < info.n_ovr; k++) {
    g.ovr_data[k] = r.owned[k + 1]; g.ovr_xsize[k] = info.ovr_xsize[k]; g.ovr_ysize[k] = info.ovr_ysize[k];
  }
  g.block_x = info.block_x; g.block_y = info.block_y;
  r.has_crs = false;
  char srs[32] = {0};
  if (info.epsg > 0) std::snprintf(srs, sizeof(srs), "EPSG:%d", info.epsg);
  else if (info.epsg == -1) std::snprintf(srs, sizeof(srs), "MODIS");
  if (srs[0] && parse_srs(srs, &r.crs) == 0) r.has_crs = true;
  d.reg[{path, band}] = std::move(rp);
  return 0;
}

// The same for a netCDF classic variable band (band_query semantics,
// warp.go:89-101: the band is registered under (path, band)).
int ingest_netcdf_locked(DropIn &d, const std::string &path, int band) {
  gskyhip_raster_info info;
  std::string srs_no, srs_cf;
  int rc = netcdf_info_srs(path.c_str(), &info, &srs_no, &srs_cf);
  if (rc) return rc;
  if (band < 1 || band > info.n_bands) return 1;   // band_query past the variable: the open fails
  if (!have_gpu()) return GSKYHIP_E_NOGPU;
  const int ts = type_size(info.dtype);
  if (ts <= 0) return GSKYHIP_E_TYPE;
  RegPtr rp = std::make_shared<Registered>();
  Registered &r = *rp;
  void *p = nullptr;
  const int64_t bytes = (int64_t)info.xsize * info.ysize * ts;
  d.reg.erase({path, band});   // a batch still holding the old entry keeps it alive
  evict_for(d, bytes);
  r.bytes = bytes;
  r.last_use = d.tick;
  r.stamped = file_stamp(path, r.mtime_ns, r.fsize);
  if (!r.stamped) r.fsize = 0;
  if (hipMalloc(&p, (size_t)bytes) != hipSuccess) return GSKYHIP_E_HIP;
  r.owned.push_back(p);
  if ((rc = gskyhip_netcdf_read(path.c_str(), band, p, bytes, nullptr))) return rc;
  gskyhip_granule &g = r.g;
  g.data = p;
  g.dtype = info.dtype; g.xsize = info.xsize; g.ysize = info.ysize; g.signed_byte = info.signed_byte;
  for (int k = 0; k < 6; k++) g.geot[k] = info.geot[k];
  g.nodata = info.nodata; g.has_nodata = info.has_nodata;
  g.block_x = info.block_x; g.block_y = info.block_y;
  // "" -> no SRS (the warp takes WGS84, warp.go:107-112); "?" or one the
  // warp cannot parse -> the request fails with GSKYHIP_E_CRS
  auto set_crs = [](const std::string &srs, gskyhip_crs &c, bool &has, bool &bad) {
    has = false;
    bad = false;
    if (srs.empty()) return;
    if (srs != "?" && parse_srs(srs.c_str(), &c) == 0) has = true;
    else bad = true;
  };
  set_crs(srs_no, r.crs, r.has_crs, r.bad_crs);
  set_crs(srs_cf, r.crs_cf, r.has_crs_cf, r.bad_crs_cf);
  d.reg[{path, band}] = std::move(rp);
  return 0;
}

// ---------------------------------------------------------------- geolocation arrays
// GDALCreateGeoLocTransformer (GDAL 3.0.1 alg/gdalgeoloc.cpp [ext], called by
// createGeoLocTransformer, warp.go:52-67) for the drop-in: the X / Y bands
// named by GeoLocOpts (registered, or opened like any source file), read as
// double (GeoLocLoadFullData: a 1-row X and a 1-row Y band form a regular
// grid), then the backmap (GeoLocGenerateBackMap), kept in HBM and cached by
// the option strings.  Parity unpinned (GDAL is absent; oracle/ restates the
// same algorithm independently).
struct GeoLocEntry {
  GeoLocD d;
  std::vector<void *> owned;
  RegPtr x_src, y_src;   // the X / Y datasets it was built from: rebuilt when either is re-read
  GeoLocEntry() { std::memset(&d, 0, sizeof(d)); }
  GeoLocEntry(const GeoLocEntry &) = delete;
  GeoLocEntry &operator=(const GeoLocEntry &) = delete;
  ~GeoLocEntry() {
    for (void *p : owned) (void)hipFree(p);
  }
};
using GeoLocPtr = std::shared_ptr<GeoLocEntry>;

int ingest_geotiff_locked(DropIn &d, const std::string &path, int band);
int ingest_netcdf_locked(DropIn &d, const std::string &path, int band);
bool is_geotiff_path(const std::string &p);

bool is_netcdf_path(const std::string &p) {
  return p.compare(0, 7, "NETCDF:") == 0 || (p.size() >= 3 && p.compare(p.size() - 3, 3, ".nc") == 0);
}

// The registry entry of (path, band) as GDALOpenEx would see it now: an
// ingested file that changed on disk is dropped and read again (never an
// entry this batch already uses: last_use == d.tick); an unregistered
// GeoTIFF / netCDF path is opened and ingested.  *irc: the ingest's code (0,
// 1 no such file, 2 no such band, GSKYHIP_E_*), or 0 when nothing was read.
RegPtr lookup_dataset(DropIn &d, const std::string &path, int band, int *irc) {
  *irc = 0;
  auto it = d.reg.find({path, band});
  if (it != d.reg.end() && it->second->fsize >= 0 && it->second->stamped && it->second->last_use != d.tick) {
    int64_t mt = 0, sz = 0;
    if (!file_stamp(path, mt, sz) || mt != it->second->mtime_ns || sz != it->second->fsize) {
      d.reg.erase(it);   // batches in flight keep their reference
      it = d.reg.end();
    }
  }
  const bool nc = is_netcdf_path(path);
  if (it == d.reg.end() && (nc || is_geotiff_path(path))) {
    *irc = nc ? ingest_netcdf_locked(d, path, band) : ingest_geotiff_locked(d, path, band);
    if (*irc == 0) it = d.reg.find({path, band});
  }
  if (it == d.reg.end()) return RegPtr();
  it->second->last_use = d.tick;
  return it->second;
}

bool band_as_double(const Registered &R, std::vector<double> &out) {
  const gskyhip_granule &g = R.g;
  const int ts = type_size(g.dtype);
  if (ts <= 0 || !g.data) return false;
  const size_t n = (size_t)g.xsize * g.ysize;
  std::vector<uint8_t> raw(n * ts);
  if (hipMemcpy(raw.data(), g.data, raw.size(), hipMemcpyDeviceToHost) != hipSuccess) return false;
  out.resize(n);
  for (size_t i = 0; i < n; i++) {
    const uint8_t *p = raw.data() + i * ts;
    switch (g.dtype) {
      case GSKYHIP_BYTE: out[i] = g.signed_byte ? (double)(int8_t)p[0] : (double)p[0]; break;
      case GSKYHIP_INT16: { int16_t v; std::memcpy(&v, p, 2); out[i] = v; break; }
      case GSKYHIP_UINT16: { uint16_t v; std::memcpy(&v, p, 2); out[i] = v; break; }
      case GSKYHIP_INT32: { int32_t v; std::memcpy(&v, p, 4); out[i] = v; break; }
      case GSKYHIP_UINT32: { uint32_t v; std::memcpy(&v, p, 4); out[i] = v; break; }
      case GSKYHIP_FLOAT32: { float v; std::memcpy(&v, p, 4); out[i] = v; break; }
      default: { double v; std::memcpy(&v, p, 8); out[i] = v; break; }
    }
  }
  return true;
}

// GeoLocGenerateBackMap: extent of the valid geolocation points, a grid of
// ~1.3 cells per point, every point splatted bilinearly into its 4 cells
// (source pixel / line weighted), cells with weight > 0.25 averaged (the
// others -1), then 3 passes filling holes from their set 4-neighbours (a cell
// filled in pass k is used from pass k+1 on).
bool geoloc_backmap(const std::vector<double> &gx, const std::vector<double> &gy, int nx, int ny, bool has_nd,
                    double nd, double pix_off, double line_off, double pix_step, double line_step,
                    std::vector<float> &bmx, std::vector<float> &bmy, int &bw, int &bh, double gt[6]) {
  const int nMaxIter = 3;
  double minX = 0, maxX = 0, minY = 0, maxY = 0;
  bool init = false;
  for (int64_t i = (int64_t)nx * ny - 1; i >= 0; i--) {
    if (has_nd && gx[i] == nd) continue;
    if (init) {
      minX = std::min(minX, gx[i]); maxX = std::max(maxX, gx[i]);
      minY = std::min(minY, gy[i]); maxY = std::max(maxY, gy[i]);
    } else {
      init = true;
      minX = maxX = gx[i];
      minY = maxY = gy[i];
    }
  }
  const double target = (double)nx * ny * 1.3;
  const double ps = std::sqrt((maxX - minX) * (maxY - minY) / target);
  if (!(ps > 0.0) || !std::isfinite(ps)) return false;
  const double fw = std::ceil((maxX - minX) / ps) + 1, fh = std::ceil((maxY - minY) / ps) + 1;
  if (!(fw > 0 && fw < 65536.0 * 64) || !(fh > 0 && fh < 65536.0 * 64) || fw * fh > 4.0e9) return false;
  bw = (int)fw;
  bh = (int)fh;
  minX -= ps / 2.0;
  maxY += ps / 2.0;
  gt[0] = minX; gt[1] = ps; gt[2] = 0.0; gt[3] = maxY; gt[4] = 0.0; gt[5] = -ps;
  const size_t nbm = (size_t)bw * bh;
  bmx.assign(nbm, 0.0f);
  bmy.assign(nbm, 0.0f);
  std::vector<float> wgt(nbm, 0.0f);
  for (int iY = 0; iY < ny; iY++)
    for (int iX = 0; iX < nx; iX++) {
      const size_t o = (size_t)iX + (size_t)iY * nx;
      if (has_nd && gx[o] == nd) continue;
      const double dBMX = (gx[o] - minX) / ps - 0.5;
      const double dBMY = (maxY - gy[o]) / ps - 0.5;
      const int iBMX = (int)std::floor(dBMX), iBMY = (int)std::floor(dBMY);
      const double fx = dBMX - iBMX, fy = dBMY - iBMY;
      const double sp = iX * pix_step + pix_off, sl = iY * line_step + line_off;
      for (int k = 0; k < 4; k++) {
        const int cx = iBMX + (k & 1), cy = iBMY + (k >> 1);
        if (cx < 0 || cx >= bw || cy < 0 || cy >= bh) continue;
        const double w = ((k & 1) ? fx : 1.0 - fx) * ((k >> 1) ? fy : 1.0 - fy);
        const size_t c = (size_t)cx + (size_t)cy * bw;
        bmx[c] += (float)(sp * w);
        bmy[c] += (float)(sl * w);
        wgt[c] += (float)w;
      }
    }
  for (size_t i = 0; i < nbm; i++) {
    if (wgt[i] > 0.25f) {
      bmx[i] /= wgt[i];
      bmy[i] /= wgt[i];
      wgt[i] = (float)(nMaxIter + 1);
    } else {
      bmx[i] = -1.0f;
      bmy[i] = -1.0f;
      wgt[i] = 0.0f;
    }
  }
  for (int iter = 0; iter < nMaxIter; iter++) {
    size_t valid = 0;
    const int mark = nMaxIter - iter;
    for (int y = 0; y < bh; y++)
      for (int x = 0; x < bw; x++) {
        const size_t c = (size_t)x + (size_t)y * bw;
        if (bmx[c] >= 0) { valid++; continue; }
        int n = 0;
        double sx = 0.0, sy = 0.0;
        auto take = [&](size_t j) { if (wgt[j] > mark) { sx += bmx[j]; sy += bmy[j]; n++; } };
        if (x > 0) take(c - 1);
        if (x + 1 < bw) take(c + 1);
        if (y > 0) take(c - bw);
        if (y + 1 < bh) take(c + bw);
        if (n > 0) {
          bmx[c] = (float)(sx / n);
          bmy[c] = (float)(sy / n);
          wgt[c] = (float)mark;
        }
      }
    if (valid == nbm) break;
  }
  return true;
}

// The transformer of one GeoLocOpts list (cached while its X / Y datasets
// are unchanged), or NULL (the reference's GDALCreateGeoLocTransformer
// failure: warp_operation_fast returns 3).
GeoLocPtr geoloc_entry(DropIn &d, const std::vector<std::string> &opts) {
  std::string key;
  for (const std::string &o : opts) key += o + '\n';
  std::map<std::string, std::string> kv;
  for (const std::string &o : opts) {
    const size_t e = o.find('=');
    if (e != std::string::npos) kv[o.substr(0, e)] = o.substr(e + 1);   // CSLFetchNameValue: KEY=VALUE
  }
  for (const char *k : {"PIXEL_OFFSET", "LINE_OFFSET", "PIXEL_STEP", "LINE_STEP", "X_BAND", "Y_BAND",
                        "X_DATASET", "Y_DATASET"})
    if (!kv.count(k)) return nullptr;   // "Missing some geolocation fields"
  int irc = 0;
  const RegPtr X = lookup_dataset(d, kv["X_DATASET"], std::atoi(kv["X_BAND"].c_str()), &irc);
  const RegPtr Y = lookup_dataset(d, kv["Y_DATASET"], std::atoi(kv["Y_BAND"].c_str()), &irc);
  if (!X || !Y) return nullptr;
  auto hit = d.geolocs.find(key);
  if (hit != d.geolocs.end()) {
    if (hit->second->x_src == X && hit->second->y_src == Y) return hit->second;
    d.geolocs.erase(hit);   // a dataset was re-read: build the transformer again
  }
  std::vector<double> ax, ay;
  if (!band_as_double(*X, ax) || !band_as_double(*Y, ay)) return nullptr;
  // GeoLocLoadFullData: a regular grid when both bands are one row
  const bool regular = X->g.ysize == 1 && Y->g.ysize == 1;
  const int nx = X->g.xsize, ny = regular ? Y->g.xsize : X->g.ysize;
  if (!regular && (Y->g.xsize != nx || Y->g.ysize != ny)) return nullptr;
  std::vector<double> gx((size_t)nx * ny), gy((size_t)nx * ny);
  for (int j = 0; j < ny; j++)
    for (int i = 0; i < nx; i++) {
      const size_t o = (size_t)j * nx + i;
      gx[o] = regular ? ax[i] : ax[o];
      gy[o] = regular ? ay[j] : ay[o];
    }
  GeoLocPtr e = std::make_shared<GeoLocEntry>();
  e->x_src = X;
  e->y_src = Y;
  GeoLocD &g = e->d;
  g.nx = nx; g.ny = ny;
  g.has_nodata = X->g.has_nodata ? 1 : 0;
  g.nodata_x = X->g.nodata;
  g.pixel_offset = std::atof(kv["PIXEL_OFFSET"].c_str());   // CPLAtof
  g.line_offset = std::atof(kv["LINE_OFFSET"].c_str());
  g.pixel_step = std::atof(kv["PIXEL_STEP"].c_str());
  g.line_step = std::atof(kv["LINE_STEP"].c_str());
  std::vector<float> bmx, bmy;
  int bw = 0, bh = 0;
  if (!geoloc_backmap(gx, gy, nx, ny, g.has_nodata != 0, g.nodata_x, g.pixel_offset, g.line_offset, g.pixel_step,
                      g.line_step, bmx, bmy, bw, bh, g.bm_gt))
    return nullptr;
  g.bm_w = bw; g.bm_h = bh;
  auto up = [&](const void *src, size_t bytes) -> void * {
    void *p = nullptr;
    if (hipMalloc(&p, bytes) != hipSuccess) return nullptr;
    e->owned.push_back(p);
    if (hipMemcpy(p, src, bytes, hipMemcpyHostToDevice) != hipSuccess) return nullptr;
    return p;
  };
  g.gx = (const double *)up(gx.data(), gx.size() * 8);
  g.gy = (const double *)up(gy.data(), gy.size() * 8);
  g.bmx = (const float *)up(bmx.data(), bmx.size() * 4);
  g.bmy = (const float *)up(bmy.data(), bmy.size() * 4);
  if (!g.gx || !g.gy || !g.bmx || !g.bmy) return nullptr;
  d.geolocs[key] = e;
  return e;
}

bool is_geotiff_path(const std::string &p) {
  auto ends = [&](const char *suf) {
    const size_t n = std::strlen(suf);
    if (p.size() < n) return false;
    for (size_t i = 0; i < n; i++)
      if (std::tolower((unsigned char)p[p.size() - n + i]) != suf[i]) return false;
    return true;
  };
  return ends(".tif") || ends(".tiff");
}

}  // namespace

// ======================================================================== C-ABI
extern "C" {

int gskyhip_crs_from_srs(const char *srs, gskyhip_crs *out) { return parse_srs(srs, out); }

int gskyhip_crs_transform(const gskyhip_crs *src, const gskyhip_crs *dst, int n, double *x, double *y,
                          int32_t *ok) {
  if (!src || !dst || n < 0 || (n > 0 && (!x || !y || !ok))) return GSKYHIP_E_ARG;
  for (int i = 0; i < n; i++) {
    double lam, phi;
    ok[i] = crs_inverse(*src, x[i], y[i], lam, phi) && crs_forward(*dst, lam, phi, x[i], y[i]) ? 1 : 0;
  }
  return 0;
}

uint32_t gskyhip_fnv32a(const char *s, int64_t n) {
  uint32_t h = 2166136261u;  // Go hash/fnv New32a (tile_merger.go:473-475)
  for (int64_t i = 0; i < n; i++) {
    h ^= (uint8_t)s[i];
    h *= 16777619u;
  }
  return h;
}

const char *gskyhip_version(void) { return "gskyhip 0.1 gfx950"; }

int gskyhip_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

int gskyhip_register_granule(const char *path, int band, const gskyhip_granule *g, const char *srs) {
  if (!path || !g || !g->data || g->xsize <= 0 || g->ysize <= 0 || type_size(g->dtype) <= 0) return GSKYHIP_E_ARG;
  if (g->n_ovr < 0 || g->n_ovr > GSKYHIP_MAX_OVR) return GSKYHIP_E_ARG;
  for (int k = 0; k < g->n_ovr; k++)
    if (!g->ovr_data[k] || g->ovr_xsize[k] <= 0 || g->ovr_ysize[k] <= 0) return GSKYHIP_E_ARG;
  RegPtr r = std::make_shared<Registered>();
  r->g = *g;
  r->has_crs = false;
  if (srs && *srs) {
    if (parse_srs(srs, &r->crs)) return GSKYHIP_E_CRS;
    r->has_crs = true;
  }
  DropIn &d = dropin();
  std::lock_guard<std::mutex> lk(d.mu);
  d.reg[{std::string(path), band}] = std::move(r);
  return 0;
}

int gskyhip_unregister_all(void) {
  DropIn &d = dropin();
  std::lock_guard<std::mutex> lk(d.mu);
  d.reg.clear();       // HBM of ingested granules is freed once no batch in flight holds it
  d.geolocs.clear();
  return 0;
}

int gskyhip_register_geotiff(const char *path, int band) {
  if (!path) return GSKYHIP_E_ARG;
  DropIn &d = dropin();
  std::lock_guard<std::mutex> lk(d.mu);
  return ingest_geotiff_locked(d, path, band);
}

int gskyhip_register_netcdf(const char *path, int band) {
  if (!path) return GSKYHIP_E_ARG;
  DropIn &d = dropin();
  std::lock_guard<std::mutex> lk(d.mu);
  return ingest_netcdf_locked(d, path, band);
}

}  // extern "C"

// ---------------------------------------------------------------- warp batches
namespace gsky {

// warp.go:82-382 for n requests at once: per request the registry lookup and
// the reference's early returns (open / band / transformer failures), then
// every request with the same destination SRS planned and warped in one set
// of launches (one tile + one pair each), the window and bytesRead of every
// request in one pass, one read-back of the reply records.  Split in
// launch / finish so the service keeps two batches in flight (service.cpp).
namespace {
std::atomic<int64_t> g_wb_ns[4];
int64_t now_ns() {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}
int64_t a256(int64_t v) { return (v + 255) & ~(int64_t)255; }
}  // namespace

void warp_batch_timers(int64_t out[4]) {
  for (int k = 0; k < 4; k++) out[k] = g_wb_ns[k].load();
}

// One batch's device, upload and read-back buffers, stream and completion
// event.  A slot carries one batch at a time; the buffers grow and are kept.
struct WarpSlot {
  hipStream_t stream = nullptr;
  hipEvent_t ev = nullptr;
  char *dev = nullptr;   // per group: header | results | stats | workspace | staged windows | scratch
  size_t dev_bytes = 0;
  char *up = nullptr;    // pinned: the groups' headers
  size_t up_bytes = 0;
  char *pin = nullptr;   // pinned: reply records, then staged windows
  size_t pin_bytes = 0;
  struct Job {
    int req;
    int err;                       // a launch failure of its group (GSKYHIP_E_*), else 0
    int64_t res_pin;               // reply record in `pin`
    int64_t win_dev, win_pin;      // staged window: device / pinned offsets (-1: written in place)
    int64_t stride;
  };
  std::vector<Job> jobs;
  std::vector<RegPtr> hold;        // granules the batch reads (freed only after it finished)
  std::vector<GeoLocPtr> hold_gl;
  WarpResp *out = nullptr;
  bool inflight = false;
};

WarpSlot *warp_slot_create() { return new WarpSlot(); }

void warp_slot_destroy(WarpSlot *s) {
  if (!s) return;
  warp_batch_finish(*s);
  if (s->dev) (void)hipFree(s->dev);
  if (s->up) (void)hipHostFree(s->up);
  if (s->pin) (void)hipHostFree(s->pin);
  if (s->ev) (void)hipEventDestroy(s->ev);
  if (s->stream) (void)hipStreamDestroy(s->stream);
  delete s;
}

namespace {
template <typename T> bool grow_dev(T *&p, size_t &have, size_t need) {
  if (have >= need) return true;
  if (p) (void)hipFree(p);
  p = nullptr;
  have = 0;
  if (hipMalloc((void **)&p, need) != hipSuccess) return false;
  have = need;
  return true;
}
bool grow_pin(char *&p, size_t &have, size_t need) {
  if (have >= need) return true;
  if (p) (void)hipHostFree(p);
  p = nullptr;
  have = 0;
  if (hipHostMalloc((void **)&p, need, hipHostMallocDefault) != hipSuccess) return false;
  have = need;
  return true;
}
}  // namespace

void warp_batch_launch(WarpSlot &S, const WarpReq *reqs, int n, WarpResp *out, uint8_t *const *direct,
                       const int64_t *direct_cap) {
  const int64_t t0 = now_ns();
  g_wb_ns[3]++;
  S.jobs.clear();
  S.out = out;
  S.inflight = false;
  DropIn &d = dropin();
  std::lock_guard<std::mutex> lk(d.mu);
  d.tick++;
  struct Item { int req; gskyhip_granule g; gskyhip_crs src; int bx, by; const GeoLocEntry *gl; };
  std::map<std::pair<int, std::string>, std::vector<Item>> groups;   // (has dst, dst srs) -> items
  for (int i = 0; i < n; i++) {
    const WarpReq &q = reqs[i];
    WarpResp &r = out[i];
    r = WarpResp();
    // warp.go:89-101: "NETCDF:..." and "*.nc" are opened through GSKY_netCDF
    // with band_query=<band>, which exposes that band as band 1; any other
    // path is opened whole and GDALGetRasterBand(band) may fail (114-118).
    const bool netcdf = is_netcdf_path(q.path);
    int irc = 0;
    const RegPtr RP = lookup_dataset(d, q.path, q.band, &irc);
    if (irc == 2) { r.rc = 2; continue; }
    if (irc < 0) { r.rc = irc; continue; }   // HBM exhausted, unsupported encoding, ...: an error, not "open failed"
    if (!RP) {   // (irc 1: no such file) a path registered with other bands is an open dataset without this band
      bool path_known = false;
      for (const auto &kv : d.reg) if (kv.first.first == q.path) { path_known = true; break; }
      r.rc = (netcdf || !path_known) ? 1 : 2;                         // open failed / band failed
      continue;
    }
    const Registered &R = *RP;
    if (!R.g.data) { r.rc = 2; continue; }                             // band failed
    if (q.width <= 0 || q.height <= 0) { r.rc = GSKYHIP_E_ARG; continue; }
    Item it2;
    it2.req = i;
    it2.gl = nullptr;
    if (q.geoloc) {   // warp.go:134-140: createGeoLocTransformer, 3 when it fails
      GeoLocPtr gl = geoloc_entry(d, q.geoloc_opts);
      if (!gl) { r.rc = 3; continue; }
      it2.gl = gl.get();
      S.hold_gl.push_back(std::move(gl));
    }
    // the dataset SRS: GSKY_netCDF opened with srs_cf=yes takes the CF
    // grid mapping only (warp.go:95, netcdfdataset.cpp:3666)
    const bool cf = netcdf && q.srs_cf > 0 && R.fsize >= 0;
    const bool has_crs = cf ? R.has_crs_cf : R.has_crs, bad_crs = cf ? R.bad_crs_cf : R.bad_crs;
    if (q.has_src_srs) {
      if (parse_srs(q.src_srs.c_str(), &it2.src)) { r.rc = 3; continue; }
    } else if (bad_crs) {
      r.rc = GSKYHIP_E_CRS;                                            // a projection outside the four families
      continue;
    } else if (has_crs) {
      it2.src = cf ? R.crs_cf : R.crs;
    } else {
      crs_epsg(4326, &it2.src);                                        // warp.go:107-112
    }
    if (q.has_dst_srs) {
      gskyhip_crs tmp;
      if (parse_srs(q.dst_srs.c_str(), &tmp)) { r.rc = 3; continue; }
    }
    it2.g = R.g;
    it2.g.ns = 0;
    if (q.has_src_gt) std::memcpy(it2.g.geot, q.src_gt, sizeof(it2.g.geot));
    it2.bx = R.g.block_x > 0 ? R.g.block_x : 0;                      // 0: one scanline of the chosen level
    it2.by = R.g.block_y > 0 ? R.g.block_y : 1;
    S.hold.push_back(RP);
    groups[{q.has_dst_srs, q.has_dst_srs ? q.dst_srs : std::string()}].push_back(it2);
  }
  if (groups.empty()) { g_wb_ns[0] += now_ns() - t0; return; }
  auto fail_all = [&](int code) {
    for (auto &kv : groups) for (const Item &it : kv.second) out[it.req].rc = code;
  };
  if (!have_gpu()) { fail_all(GSKYHIP_E_NOGPU); return; }
  if ((!S.stream && hipStreamCreateWithFlags(&S.stream, hipStreamNonBlocking) != hipSuccess) ||
      (!S.ev && hipEventCreateWithFlags(&S.ev, hipEventDisableTiming) != hipSuccess)) {
    fail_all(GSKYHIP_E_HIP);
    return;
  }
  // ---- layout of every group in the slot's three buffers
  // device group: granules | geolocation transformers | crs (m sources + dst) | tiles | pairs
  //               | block-stats jobs | window destinations (uploaded up to here) | reply records
  //               | stats | workspace | staged windows | block-stats scratch
  struct Lay {
    const std::vector<Item> *items;
    const std::string *dst;
    int has_dst, m, max_w, max_h, n_staged;
    int64_t o_gl, o_crs, o_tiles, o_pairs, o_jobs, o_outs, o_res, o_stats, o_ws, ws, stride, o_win, o_scr, max_px;
    int64_t dev_base, up_base, pin_res, pin_win;
    std::vector<BlockStatsJob> jobs;
    std::vector<char> staged;
  };
  std::vector<Lay> lays;
  int64_t dev_total = 0, up_total = 0, pin_total = 0;
  for (auto &kv : groups) {
    Lay L;
    L.items = &kv.second;
    L.has_dst = kv.first.first;
    L.dst = &kv.first.second;
    const std::vector<Item> &items = kv.second;
    const int m = L.m = (int)items.size();
    L.max_w = 1; L.max_h = 1; L.max_px = 0; L.n_staged = 0;
    int64_t st_bytes = 0;
    std::vector<int64_t> n_words(m);
    L.jobs.resize(m);
    L.staged.assign(m, 0);
    for (int k = 0; k < m; k++) {
      const WarpReq &q = reqs[items[k].req];
      L.max_w = std::max(L.max_w, q.width);
      L.max_h = std::max(L.max_h, q.height);
      const gskyhip_granule &g = items[k].g;
      const int bx0 = items[k].bx > 0 ? items[k].bx : g.xsize;
      const int64_t nblocks = ((int64_t)(g.xsize + bx0 - 1) / bx0) * ((g.ysize + items[k].by - 1) / items[k].by);
      n_words[k] = (nblocks + 31) / 32;
      const int64_t px = (int64_t)q.width * q.height;
      L.max_px = std::max(L.max_px, px);
      BlockStatsJob &J = L.jobs[k];
      J.bx = items[k].bx; J.by = items[k].by; J.n_words = (int32_t)n_words[k]; J._pad = 0;
      J.xsrc_off = st_bytes;                     // xsrc of every job, then every job's bitmap
      st_bytes += a256(px * 4);
      const int i = items[k].req;
      // a window is written in place when the caller gave a destination big
      // enough for any value type (8 bytes per pixel)
      const bool in_place = direct && direct[i] && direct_cap && direct_cap[i] >= px * 8;
      if (!in_place) { L.staged[k] = 1; L.n_staged++; }
    }
    for (int k = 0; k < m; k++) {
      L.jobs[k].bits_off = st_bytes;
      st_bytes += a256(n_words[k] * 4);
    }
    L.o_gl = a256((int64_t)m * sizeof(gskyhip_granule));
    L.o_crs = L.o_gl + a256((int64_t)m * sizeof(GeoLocD));
    L.o_tiles = L.o_crs + a256((int64_t)(m + 1) * sizeof(gskyhip_crs));
    L.o_pairs = L.o_tiles + a256((int64_t)m * sizeof(gskyhip_tile));
    L.o_jobs = L.o_pairs + a256((int64_t)m * 4);
    L.o_outs = L.o_jobs + a256((int64_t)m * sizeof(BlockStatsJob));
    L.o_res = L.o_outs + a256((int64_t)m * sizeof(void *));
    L.o_stats = L.o_res + a256((int64_t)m * sizeof(WarpResult));
    L.o_ws = L.o_stats + a256((int64_t)m * 16);
    L.ws = render_workspace_size(m, m, L.max_h);
    L.stride = a256((int64_t)L.max_w * L.max_h * 8);
    L.o_win = L.o_ws + a256(L.ws);
    L.o_scr = L.o_win + L.stride * L.n_staged;
    L.dev_base = dev_total;
    dev_total += a256(L.o_scr + st_bytes);
    L.up_base = up_total;
    up_total += a256(L.o_res);
    L.pin_res = pin_total;
    pin_total += a256((int64_t)m * sizeof(WarpResult));
    L.pin_win = pin_total;
    pin_total += L.stride * L.n_staged;
    lays.push_back(std::move(L));
  }
  if (!grow_dev(S.dev, S.dev_bytes, (size_t)dev_total) || !grow_pin(S.up, S.up_bytes, (size_t)up_total) ||
      !grow_pin(S.pin, S.pin_bytes, (size_t)pin_total)) {
    fail_all(GSKYHIP_E_HIP);
    return;
  }
  // ---- headers, launches, reply read-back
  for (Lay &L : lays) {
    const std::vector<Item> &items = *L.items;
    const int m = L.m;
    char *base = S.dev + L.dev_base;
    char *hdr = S.up + L.up_base;
    std::memset(hdr, 0, (size_t)L.o_res);
    gskyhip_granule *hg = (gskyhip_granule *)hdr;
    gskyhip_crs *hc = (gskyhip_crs *)(hdr + L.o_crs);
    gskyhip_tile *ht = (gskyhip_tile *)(hdr + L.o_tiles);
    int32_t *hp = (int32_t *)(hdr + L.o_pairs);
    uint8_t **houts = (uint8_t **)(hdr + L.o_outs);
    int dst_crs = -1;
    if (L.has_dst) {
      parse_srs(L.dst->c_str(), &hc[m]);
      dst_crs = m;
    }
    std::memcpy(hdr + L.o_jobs, L.jobs.data(), (size_t)m * sizeof(BlockStatsJob));
    GeoLocD *hgl = (GeoLocD *)(hdr + L.o_gl);
    bool any_gl = false;
    int si = 0;
    for (int k = 0; k < m; k++) {
      const WarpReq &q = reqs[items[k].req];
      hg[k] = items[k].g;
      hg[k].crs = k;
      hg[k].geoloc = 0;
      if (items[k].gl) {
        hgl[k] = items[k].gl->d;
        hg[k].geoloc = k + 1;
        any_gl = true;
      }
      hc[k] = items[k].src;
      std::memcpy(ht[k].dst_geot, q.dst_gt, sizeof(ht[k].dst_geot));
      ht[k].width = q.width;
      ht[k].height = q.height;
      ht[k].pair_begin = k;
      ht[k].pair_end = k + 1;
      hp[k] = k;
      WarpSlot::Job J;
      J.req = items[k].req;
      J.err = 0;
      J.res_pin = L.pin_res + (int64_t)k * sizeof(WarpResult);
      J.stride = L.stride;
      if (L.staged[k]) {
        J.win_dev = L.dev_base + L.o_win + L.stride * si;
        J.win_pin = L.pin_win + L.stride * si;
        si++;
        houts[k] = (uint8_t *)(S.dev + J.win_dev);
      } else {
        J.win_dev = J.win_pin = -1;
        houts[k] = direct[J.req];
      }
      S.jobs.push_back(J);
    }
    const size_t first_job = S.jobs.size() - (size_t)m;
    auto fail = [&](int code) { for (size_t j = first_job; j < S.jobs.size(); j++) S.jobs[j].err = code; };
    if (hipMemcpyAsync(base, hdr, (size_t)L.o_res, hipMemcpyHostToDevice, S.stream) != hipSuccess) {
      fail(GSKYHIP_E_HIP);
      continue;
    }
    MaskSpecS ms[4];
    std::memset(ms, 0, sizeof(ms));
    RenderCall rc;
    rc.granules = (const gskyhip_granule *)base; rc.n_granules = m;
    rc.crs = (const gskyhip_crs *)(base + L.o_crs); rc.n_crs = m + 1; rc.dst_crs = dst_crs;
    rc.tiles = (const gskyhip_tile *)(base + L.o_tiles); rc.n_tiles = m;
    rc.pair_granule = (const int32_t *)(base + L.o_pairs); rc.n_pairs = m;
    rc.max_w = L.max_w; rc.max_h = L.max_h;
    rc.mask_ns = -1; rc.mask_inclusive = 0; rc.mask_specs = ms;
    rc.resample = GSKYHIP_RESAMPLE_NEAREST;
    rc.value_types = 0;
    rc.cov_offsets = nullptr;
    rc.cov_stride = 0;
    rc.workspace = base + L.o_ws; rc.workspace_bytes = L.ws;
    rc.stream = S.stream;
    rc.geolocs = any_gl ? (const GeoLocD *)(base + L.o_gl) : nullptr;
    int code = launch_warp_jobs(rc, (const BlockStatsJob *)(base + L.o_jobs), L.max_px, base + L.o_scr,
                                (int32_t *)(base + L.o_stats), (uint8_t *const *)(base + L.o_outs),
                                (WarpResult *)(base + L.o_res));
    if (!code && hipMemcpyAsync(S.pin + L.pin_res, base + L.o_res, (size_t)m * sizeof(WarpResult),
                                hipMemcpyDeviceToHost, S.stream) != hipSuccess)
      code = GSKYHIP_E_HIP;
    if (code) fail(code);
  }
  if (hipEventRecord(S.ev, S.stream) != hipSuccess) {
    for (WarpSlot::Job &J : S.jobs) J.err = GSKYHIP_E_HIP;
    (void)hipStreamSynchronize(S.stream);
  }
  S.inflight = true;
  g_wb_ns[0] += now_ns() - t0;
}

void warp_batch_finish(WarpSlot &S) {
  if (!S.inflight) {
    if (!S.hold.empty() || !S.hold_gl.empty()) {
      std::lock_guard<std::mutex> lk(dropin().mu);
      S.hold.clear();
      S.hold_gl.clear();
    }
    return;
  }
  const int64_t t0 = now_ns();
  const bool ok = hipEventSynchronize(S.ev) == hipSuccess;
  const int64_t t1 = now_ns();
  g_wb_ns[1] += t1 - t0;
  bool copy_ok = true;
  std::vector<int64_t> staged(S.jobs.size(), 0);   // staged window bytes to take per job
  int n_copies = 0;
  for (size_t j = 0; j < S.jobs.size(); j++) {
    const WarpSlot::Job &J = S.jobs[j];
    WarpResp &r = S.out[J.req];
    if (J.err || !ok) { r.rc = J.err ? J.err : GSKYHIP_E_HIP; continue; }
    WarpResult w;
    std::memcpy(&w, S.pin + J.res_pin, sizeof(w));
    for (int k = 0; k < 4; k++) r.bbox[k] = w.bbox[k];
    r.dtype = w.dtype;
    r.nodata = w.nodata;
    r.bytes_read = w.bytes_read;
    std::memcpy(r.src_gt, w.src_gt, sizeof(r.src_gt));
    const int64_t bytes = std::min<int64_t>(std::max<int64_t>((int64_t)w.bbox[2] * w.bbox[3] * type_size(w.dtype), 0),
                                            J.stride);
    if (J.win_dev < 0) {
      r.in_place = bytes;   // already in the caller's destination
    } else if (bytes > 0) {
      if (hipMemcpyAsync(S.pin + J.win_pin, S.dev + J.win_dev, (size_t)bytes, hipMemcpyDeviceToHost, S.stream) !=
          hipSuccess)
        copy_ok = false;
      staged[j] = bytes;
      n_copies++;
    }
  }
  if (n_copies && (!copy_ok || hipStreamSynchronize(S.stream) != hipSuccess)) copy_ok = false;
  for (size_t j = 0; j < S.jobs.size(); j++) {
    if (!staged[j]) continue;
    const WarpSlot::Job &J = S.jobs[j];
    WarpResp &r = S.out[J.req];
    if (!copy_ok) { r.rc = GSKYHIP_E_HIP; continue; }
    r.data.assign(S.pin + J.win_pin, S.pin + J.win_pin + staged[j]);
  }
  {
    std::lock_guard<std::mutex> lk(dropin().mu);
    S.hold.clear();
    S.hold_gl.clear();
  }
  S.inflight = false;
  g_wb_ns[2] += now_ns() - t1;
}

void warp_batch(const WarpReq *reqs, int n, WarpResp *out) {
  static std::mutex mu;
  static WarpSlot *slot = new WarpSlot();   // never destroyed: no HIP calls at process exit
  std::lock_guard<std::mutex> lk(mu);
  warp_batch_launch(*slot, reqs, n, out, nullptr, nullptr);
  warp_batch_finish(*slot);
}

}  // namespace gsky

extern "C" {

// warp.go:82 drop-in: one request through warp_batch -- in this process, or
// forwarded to the per-node service when GSKYHIP_SERVICE names its socket
// (service.cpp; the worker process then never touches the GPU).  The window
// comes back in malloc'd host memory the caller frees (warp.go:573-574).
int warp_operation_fast(const char *srcFilePath, char *srcProjRef, double *srcGeot,
                        const char **geoLocOpts, const char *dstProjRef, double *dstGeot,
                        int dstXImageSize, int dstYImageSize, int band, int srsCf, void **dstBuf,
                        int *dstBufSize, int *dstBbox, double *noData, int *dType, int *bytesRead) {
  *bytesRead = 0;
  if (!srcFilePath) return 1;
  if (!dstGeot) return GSKYHIP_E_ARG;
  WarpReq q;
  q.path = srcFilePath;
  q.band = band;
  q.has_src_srs = srcProjRef ? 1 : 0;
  if (srcProjRef) q.src_srs = srcProjRef;
  q.has_src_gt = srcGeot ? 1 : 0;
  if (srcGeot) std::memcpy(q.src_gt, srcGeot, sizeof(q.src_gt));
  q.geoloc = geoLocOpts ? 1 : 0;
  if (geoLocOpts)   // NULL-terminated (warp.go:514-526)
    for (int k = 0; geoLocOpts[k] && k < 64; k++) q.geoloc_opts.push_back(geoLocOpts[k]);
  q.has_dst_srs = dstProjRef ? 1 : 0;
  if (dstProjRef) q.dst_srs = dstProjRef;
  std::memcpy(q.dst_gt, dstGeot, sizeof(q.dst_gt));
  q.width = dstXImageSize;
  q.height = dstYImageSize;
  q.srs_cf = srsCf;
  WarpResp r;
  const char *svc = std::getenv("GSKYHIP_SERVICE");
  if (svc && *svc) {   // the window arrives straight in the malloc'd buffer
    void *mb = nullptr;
    size_t ml = 0;
    const int e = service_warp(svc, q, r, &mb, &ml);
    if (e) return e;
    if (r.rc) { std::free(mb); return r.rc; }
    *dstBuf = mb;
    *dstBufSize = (int)ml;
  } else {
    warp_batch(&q, 1, &r);
    if (r.rc) return r.rc;
    *dstBufSize = (int)r.data.size();
    *dstBuf = std::malloc(r.data.empty() ? 1 : r.data.size());
    if (!*dstBuf) return GSKYHIP_E_ARG;
    if (!r.data.empty()) std::memcpy(*dstBuf, r.data.data(), r.data.size());
  }
  for (int k = 0; k < 4; k++) dstBbox[k] = r.bbox[k];
  *noData = r.nodata;
  *dType = r.dtype;
  *bytesRead = r.bytes_read;
  if (srcGeot) std::memcpy(srcGeot, r.src_gt, sizeof(r.src_gt));
  return 0;
}

int64_t gskyhip_render_workspace_size(int n_tiles, int n_pairs, int max_tile_height) {
  return render_workspace_size(n_tiles, n_pairs, max_tile_height);
}

int gskyhip_render_tiles_phase(int phase, const gskyhip_granule *granules, int n_granules,
                               const gskyhip_crs *crs_table, int n_crs, int dst_crs, const gskyhip_tile *tiles,
                               int n_tiles, const int32_t *pair_granule, int n_pairs, int max_tile_width,
                               int max_tile_height, const int32_t *out_ns, int n_out_ns, const gskyhip_mask *mask,
                               int resample, const gskyhip_scale_params *sp, const uint8_t *ramp,
                               uint8_t *rgba_out, void *canvas_out, void *workspace, int64_t workspace_bytes,
                               void *stream) {
  return gskyhip_render_tiles_typed(phase, 0u, granules, n_granules, crs_table, n_crs, dst_crs, tiles, n_tiles,
                                    pair_granule, n_pairs, max_tile_width, max_tile_height, out_ns, n_out_ns, mask,
                                    resample, sp, ramp, rgba_out, canvas_out, workspace, workspace_bytes, stream);
}

static int render_call(int phase, uint32_t value_types, const gskyhip_granule *granules, int n_granules,
                       const gskyhip_crs *crs_table, int n_crs, int dst_crs, const gskyhip_tile *tiles,
                       int n_tiles, const int32_t *pair_granule, int n_pairs, int max_tile_width,
                       int max_tile_height, const int32_t *out_ns, int n_out_ns, const gskyhip_mask *mask,
                       int resample, const gskyhip_scale_params *sp, const uint8_t *ramp, uint8_t *rgba_out,
                       void *canvas_out, const int64_t *cov_offsets, int64_t cov_stride, void *workspace,
                       int64_t workspace_bytes, void *stream);

int gskyhip_render_coverage(int phase, uint32_t value_types, const gskyhip_granule *granules, int n_granules,
                            const gskyhip_crs *crs_table, int n_crs, int dst_crs, const gskyhip_tile *tiles,
                            int n_tiles, const int32_t *pair_granule, int n_pairs, int max_tile_width,
                            int max_tile_height, int resample, const gskyhip_scale_params *sp,
                            const int64_t *tile_offsets, int64_t row_stride, void *coverage_out, void *workspace,
                            int64_t workspace_bytes, void *stream) {
  if (!tile_offsets || !coverage_out || row_stride < max_tile_width) return GSKYHIP_E_ARG;
  const int32_t out_ns[1] = {0};
  return render_call(phase, value_types, granules, n_granules, crs_table, n_crs, dst_crs, tiles, n_tiles,
                     pair_granule, n_pairs, max_tile_width, max_tile_height, out_ns, 1, nullptr, resample, sp,
                     nullptr, nullptr, coverage_out, tile_offsets, row_stride, workspace, workspace_bytes, stream);
}

int gskyhip_render_tiles_typed(int phase, uint32_t value_types, const gskyhip_granule *granules,
                               int n_granules, const gskyhip_crs *crs_table, int n_crs, int dst_crs,
                               const gskyhip_tile *tiles, int n_tiles, const int32_t *pair_granule, int n_pairs,
                               int max_tile_width, int max_tile_height, const int32_t *out_ns, int n_out_ns,
                               const gskyhip_mask *mask, int resample, const gskyhip_scale_params *sp,
                               const uint8_t *ramp, uint8_t *rgba_out, void *canvas_out, void *workspace,
                               int64_t workspace_bytes, void *stream) {
  return render_call(phase, value_types, granules, n_granules, crs_table, n_crs, dst_crs, tiles, n_tiles,
                     pair_granule, n_pairs, max_tile_width, max_tile_height, out_ns, n_out_ns, mask, resample, sp,
                     ramp, rgba_out, canvas_out, nullptr, 0, workspace, workspace_bytes, stream);
}

static int render_call(int phase, uint32_t value_types, const gskyhip_granule *granules, int n_granules,
                       const gskyhip_crs *crs_table, int n_crs, int dst_crs, const gskyhip_tile *tiles,
                       int n_tiles, const int32_t *pair_granule, int n_pairs, int max_tile_width,
                       int max_tile_height, const int32_t *out_ns, int n_out_ns, const gskyhip_mask *mask,
                       int resample, const gskyhip_scale_params *sp, const uint8_t *ramp, uint8_t *rgba_out,
                       void *canvas_out, const int64_t *cov_offsets, int64_t cov_stride, void *workspace,
                       int64_t workspace_bytes, void *stream) {
  if (!sp || !out_ns || n_tiles < 0 || n_pairs < 0 || phase < 0 || phase > 2) return GSKYHIP_E_ARG;
  MaskSpecS ms[4];
  int r = build_mask_specs(mask, ms);
  if (r) return r;
  RenderCall rc;
  rc.granules = granules; rc.n_granules = n_granules;
  rc.crs = crs_table; rc.n_crs = n_crs; rc.dst_crs = dst_crs;
  rc.tiles = tiles; rc.n_tiles = n_tiles;
  rc.pair_granule = pair_granule; rc.n_pairs = n_pairs;
  rc.max_w = max_tile_width; rc.max_h = max_tile_height;
  rc.mask_ns = mask ? mask->ns : -1;
  rc.mask_inclusive = mask ? mask->inclusive : 0;
  rc.mask_specs = ms;
  rc.resample = resample;
  rc.value_types = value_types;
  rc.cov_offsets = cov_offsets;
  rc.cov_stride = cov_stride;
  rc.workspace = workspace; rc.workspace_bytes = workspace_bytes;
  rc.stream = (hipStream_t)stream;
  return launch_render(rc, out_ns, n_out_ns, *sp, ramp, rgba_out, canvas_out, phase);
}

int gskyhip_render_tiles(const gskyhip_granule *granules, int n_granules, const gskyhip_crs *crs_table,
                         int n_crs, int dst_crs, const gskyhip_tile *tiles, int n_tiles,
                         const int32_t *pair_granule, int n_pairs, int max_tile_width, int max_tile_height,
                         const int32_t *out_ns, int n_out_ns, const gskyhip_mask *mask, int resample,
                         const gskyhip_scale_params *sp, const uint8_t *ramp, uint8_t *rgba_out,
                         void *canvas_out, void *workspace, int64_t workspace_bytes, void *stream) {
  return gskyhip_render_tiles_phase(0, granules, n_granules, crs_table, n_crs, dst_crs, tiles, n_tiles,
                                    pair_granule, n_pairs, max_tile_width, max_tile_height, out_ns, n_out_ns,
                                    mask, resample, sp, ramp, rgba_out, canvas_out, workspace, workspace_bytes,
                                    stream);
}

int gskyhip_render_status(void *workspace, int n_tiles, int n_pairs, int max_tile_height, void *stream) {
  // TilePlan array position: after PairPlan[n_pairs] and Xform[n_pairs]
  auto al = [](int64_t x) { return (x + 255) & ~(int64_t)255; };
  const int np = n_pairs > 0 ? n_pairs : 1;
  const int64_t off = al(sizeof(PairPlan) * (int64_t)np) + al(sizeof(Xform) * (int64_t)np);
  (void)max_tile_height;
  std::vector<TilePlan> tp((size_t)(n_tiles > 0 ? n_tiles : 0));
  if (n_tiles <= 0) return 0;
  if (hipMemcpyAsync(tp.data(), (char *)workspace + off, sizeof(TilePlan) * n_tiles, hipMemcpyDeviceToHost,
                     (hipStream_t)stream) != hipSuccess)
    return GSKYHIP_E_HIP;
  if (hipStreamSynchronize((hipStream_t)stream) != hipSuccess) return GSKYHIP_E_HIP;
  for (const auto &t : tp)
    if (t.status) return t.status;
  return 0;
}

int gskyhip_render_tile_info(void *workspace, int n_tiles, int n_pairs, int max_tile_height, int32_t *info_out,
                             int32_t *counters_out, void *stream) {
  if (n_tiles < 0 || n_pairs < 0 || (n_tiles > 0 && (!workspace || !info_out))) return GSKYHIP_E_ARG;
  auto al = [](int64_t x) { return (x + 255) & ~(int64_t)255; };
  const int np = n_pairs > 0 ? n_pairs : 1;
  const int64_t off = al(sizeof(PairPlan) * (int64_t)np) + al(sizeof(Xform) * (int64_t)np);
  if (n_tiles == 0) return 0;
  if (counters_out) {
    const int64_t c_off = gsky::render_counters_offset(n_tiles, n_pairs, max_tile_height);
    if (hipMemcpyAsync(counters_out, (char *)workspace + c_off, 3 * sizeof(int32_t), hipMemcpyDeviceToHost,
                       (hipStream_t)stream) != hipSuccess)
      return GSKYHIP_E_HIP;
  }
  std::vector<TilePlan> tp((size_t)n_tiles);
  if (hipMemcpyAsync(tp.data(), (char *)workspace + off, sizeof(TilePlan) * n_tiles, hipMemcpyDeviceToHost,
                     (hipStream_t)stream) != hipSuccess)
    return GSKYHIP_E_HIP;
  if (hipStreamSynchronize((hipStream_t)stream) != hipSuccess) return GSKYHIP_E_HIP;
  for (int t = 0; t < n_tiles; t++) {
    info_out[4 * t] = tp[t].status;
    info_out[4 * t + 1] = tp[t].complex;
    info_out[4 * t + 2] = tp[t].vt;
    info_out[4 * t + 3] = tp[t].n_entries;
  }
  return 0;
}

int gskyhip_render_touched(void *workspace, int n_tiles, int n_pairs, int max_tile_height, int64_t *bytes_out,
                           void *stream) {
  if (n_tiles < 0 || n_pairs < 0 || !bytes_out || (n_pairs > 0 && !workspace)) return GSKYHIP_E_ARG;
  return launch_pair_touched(workspace, n_tiles, n_pairs, max_tile_height, bytes_out, (hipStream_t)stream);
}

int gskyhip_render_pair_info(void *workspace, int n_tiles, int n_pairs, int max_tile_height, int32_t *info_out,
                             void *stream) {
  if (n_tiles < 0 || n_pairs < 0 || (n_pairs > 0 && (!workspace || !info_out))) return GSKYHIP_E_ARG;
  if (n_pairs == 0) return 0;
  int32_t *dev = nullptr;
  if (hipMalloc((void **)&dev, (size_t)n_pairs * 8 * sizeof(int32_t)) != hipSuccess) return GSKYHIP_E_HIP;
  hipStream_t s = (hipStream_t)stream;
  int rc = launch_pair_footprint(workspace, n_tiles, n_pairs, max_tile_height, dev, s);
  if (!rc && (hipMemcpyAsync(info_out, dev, (size_t)n_pairs * 8 * sizeof(int32_t), hipMemcpyDeviceToHost, s) !=
                  hipSuccess ||
              hipStreamSynchronize(s) != hipSuccess))
    rc = GSKYHIP_E_HIP;
  (void)hipFree(dev);
  return rc;
}

int gskyhip_warp_windows(const gskyhip_granule *granules, int n_granules, const gskyhip_crs *crs_table,
                         int n_crs, int dst_crs, const gskyhip_tile *tiles, int n_tiles,
                         const int32_t *pair_granule, int n_pairs, int max_tile_width, int max_tile_height,
                         int resample, int32_t *bbox_out, int32_t *dtype_out, double *nodata_out,
                         void *win_out, int64_t win_stride, void *workspace, int64_t workspace_bytes,
                         void *stream) {
  MaskSpecS ms[4];
  std::memset(ms, 0, sizeof(ms));
  RenderCall rc;
  rc.granules = granules; rc.n_granules = n_granules;
  rc.crs = crs_table; rc.n_crs = n_crs; rc.dst_crs = dst_crs;
  rc.tiles = tiles; rc.n_tiles = n_tiles;
  rc.pair_granule = pair_granule; rc.n_pairs = n_pairs;
  rc.max_w = max_tile_width; rc.max_h = max_tile_height;
  rc.mask_ns = -1; rc.mask_inclusive = 0; rc.mask_specs = ms;
  rc.resample = resample;
  rc.value_types = 0;
  rc.cov_offsets = nullptr;
  rc.cov_stride = 0;
  rc.workspace = workspace; rc.workspace_bytes = workspace_bytes;
  rc.stream = (hipStream_t)stream;
  if (win_stride < (int64_t)max_tile_width * max_tile_height * 4) return GSKYHIP_E_ARG;
  return launch_warp_windows(rc, bbox_out, dtype_out, nodata_out, win_out, win_stride);
}

// ComputeReprojectExtent (warp.go:433-487), batched: one wavefront per granule.
int gskyhip_compute_reproject_extent(const gskyhip_granule *granules, int n, const gskyhip_crs *crs_table,
                                     int n_crs, int dst_crs, const double *dst_bbox, int32_t *out,
                                     int32_t *status, void *stream) {
  if (n < 0 || n_crs <= 0 || dst_crs >= n_crs || (n > 0 && (!granules || !crs_table || !dst_bbox || !out || !status)))
    return GSKYHIP_E_ARG;
  return launch_extent(granules, n, crs_table, dst_crs, dst_bbox, out, status, (hipStream_t)stream);
}

int64_t gskyhip_drill_deciles_workspace_size(int n_polys, int64_t mask_bytes, int band_chunk) {
  return drill_deciles_workspace_size(n_polys, mask_bytes, band_chunk);
}

// computeDeciles (drill.go:229-273) for a polygon batch: segmented GPU sort.
int gskyhip_drill_deciles(const float *stack, int xsize, int ysize, int n_bands, int t_stride, const int32_t *win,
                          const int64_t *mask_off, const uint8_t *masks, int n_polys, int64_t mask_bytes,
                          const int32_t *bands, int n_list, float nodata, int decile_count, int band_chunk,
                          const int32_t *totals, float *out, int32_t *status, void *workspace,
                          int64_t workspace_bytes, void *stream) {
  if (!stack || !win || !mask_off || !masks || !totals || !out || !status) return GSKYHIP_E_ARG;
  DecileCall c;
  c.stack = stack; c.xsize = xsize; c.ysize = ysize; c.n_bands = n_bands; c.t_stride = t_stride;
  c.win = win; c.mask_off = mask_off; c.masks = masks; c.n_polys = n_polys; c.mask_bytes = mask_bytes;
  c.bands = bands; c.n_list = n_list; c.nodata = nodata; c.decile_count = decile_count;
  c.band_chunk = band_chunk; c.totals = totals; c.out = out; c.status = status;
  c.workspace = workspace; c.workspace_bytes = workspace_bytes; c.stream = (hipStream_t)stream;
  return launch_drill_deciles(c);
}

int64_t gskyhip_drill_read_data_workspace_size(int n_polys, int64_t mask_bytes, int n_list, int band_strides,
                                               int decile_count, int mode) {
  return drill_read_data_workspace_size(n_polys, mask_bytes, n_list, band_strides, decile_count, mode);
}

int gskyhip_drill_read_data(const float *stack, int xsize, int ysize, int n_bands, int t_stride, const int32_t *win,
                            const int64_t *mask_off, const uint8_t *masks, int n_polys, int64_t mask_bytes,
                            const int32_t *bands, int n_list, float nodata, float clip_lower, float clip_upper,
                            int pixel_count, int band_strides, int decile_count, int mode, double *out_value,
                            int32_t *out_count, int32_t *status, void *workspace, int64_t workspace_bytes,
                            void *stream) {
  if (!stack || !win || !mask_off || !masks || !out_value || !out_count || !status) return GSKYHIP_E_ARG;
  if (mode != 0 && mode != 1) return GSKYHIP_E_ARG;
  ReadDataCall c;
  c.stack = stack; c.xsize = xsize; c.ysize = ysize; c.n_bands = n_bands; c.t_stride = t_stride;
  c.win = win; c.mask_off = mask_off; c.masks = masks; c.n_polys = n_polys; c.mask_bytes = mask_bytes;
  c.bands = bands; c.n_list = n_list; c.nodata = nodata; c.lo = clip_lower; c.hi = clip_upper;
  c.pixel_count = pixel_count; c.band_strides = band_strides; c.decile_count = decile_count; c.mode = mode;
  c.out_value = out_value; c.out_count = out_count; c.status = status;
  c.workspace = workspace; c.workspace_bytes = workspace_bytes; c.stream = (hipStream_t)stream;
  return launch_drill_read_data(c);
}

// RasterMerger.Run for one batch over warped FlexRasters (tile_merger.go:447-503).
int gskyhip_merge_rasters(const gskyhip_flex_raster *rasters, int n, const gskyhip_mask *mask,
                          void *const *canvases, int n_ns, int32_t *created, int32_t *dtype, double *nodata,
                          void *stream) {
  MaskSpecS ms[4];
  int r = build_mask_specs(mask, ms);
  if (r) return r;
  const int mask_ns = mask ? mask->ns : -1;
  const bool inclusive = mask && mask->inclusive;
  hipStream_t s = (hipStream_t)stream;
  std::vector<double> stamp(n);
  std::vector<int> keys;
  std::vector<char> in_stack(n, 0);
  for (int i = 0; i < n; i++) {
    stamp[i] = rasters[i].timestamp + (double)rasters[i].polygon_hash;   // 473-475
    if (mask_ns >= 0 && rasters[i].ns == mask_ns) {
      if (mask_slot_h(rasters[i].dtype) < 0) return GSKYHIP_E_MASK;      // 440-442
      if (!inclusive) continue;                                          // 485-487
    }
    in_stack[i] = 1;
  }
  // stable order: geoStamp descending, arrival order within a key (281-290)
  std::vector<int> order;
  for (int i = 0; i < n; i++) if (in_stack[i]) order.push_back(i);
  for (size_t a = 1; a < order.size(); a++) {
    const int v = order[a];
    size_t j = a;
    while (j > 0 && stamp[order[j - 1]] < stamp[v]) { order[j] = order[j - 1]; j--; }
    order[j] = v;
  }
  for (int k = 0; k < n_ns; k++) { created[k] = 0; dtype[k] = 0; nodata[k] = 0; }
  std::vector<std::vector<FlexEntry>> per_ns(n_ns);
  std::vector<double> canvas_ts(n_ns, 0.0);
  int width = 0, height = 0;
  for (int idx : order) {
    const gskyhip_flex_raster &fr = rasters[idx];
    if (fr.ns < 0 || fr.ns >= n_ns) return GSKYHIP_E_RANGE;
    width = fr.width; height = fr.height;
    if (!created[fr.ns]) {                                               // 291-297
      created[fr.ns] = 1;
      dtype[fr.ns] = fr.dtype;
      nodata[fr.ns] = fr.nodata;
      canvas_ts[fr.ns] = 0;
    } else if (dtype[fr.ns] != fr.dtype) {
      return GSKYHIP_E_TYPE;
    }
    FlexEntry e;
    std::memset(&e, 0, sizeof(e));
    e.data = fr.data;
    e.data_w = fr.data_w; e.data_h = fr.data_h; e.off_x = fr.off_x; e.off_y = fr.off_y;
    e.dtype = fr.dtype;
    e.nodata = fr.nodata;
    e.fill_mode = fr.timestamp < canvas_ts[fr.ns] ? 1 : 0;              // 47
    if (!e.fill_mode) canvas_ts[fr.ns] = fr.timestamp;
    for (int q = 0; q < n; q++) {                                        // maskMap[geoStamp]
      if (mask_ns >= 0 && rasters[q].ns == mask_ns && stamp[q] == stamp[idx]) {
        e.mask_data = rasters[q].data;
        e.mask_dtype = rasters[q].dtype;
        e.mask_len = (int64_t)rasters[q].data_w * rasters[q].data_h;
      }
    }
    if (e.mask_data && (int64_t)e.data_w * e.data_h > e.mask_len) return GSKYHIP_E_RANGE;
    per_ns[fr.ns].push_back(e);
  }
  for (int k = 0; k < n_ns; k++) {
    if (!created[k]) continue;
    const int slot = mask_slot_h(per_ns[k].empty() ? 0 : per_ns[k][0].mask_dtype);
    const MaskSpecS &m = ms[slot < 0 ? 0 : slot];
    // all mask rasters of one layer share a dtype; pick its spec
    MaskSpecS mm = m;
    for (const auto &e : per_ns[k]) {
      if (e.mask_data) { int sl = mask_slot_h(e.mask_dtype); if (sl >= 0) mm = ms[sl]; break; }
    }
    r = launch_merge_fold(per_ns[k].data(), (int)per_ns[k].size(), width, height, dtype[k], nodata[k], mm,
                          canvases[k], s);
    if (r) return r;
  }
  if (hipStreamSynchronize(s) != hipSuccess) return GSKYHIP_E_HIP;
  return 0;
}

int gskyhip_scale(void *data, int dtype, int64_t n, double nodata, const gskyhip_scale_params *sp,
                  uint8_t *out, void *stream) {
  if (!sp) return GSKYHIP_E_ARG;
  return launch_scale(data, dtype, n, nodata, *sp, out, (hipStream_t)stream);
}

int gskyhip_scale_legacy(void *data, int dtype, int64_t n, double nodata, const gskyhip_scale_params *sp,
                         uint8_t *out, void *stream) {
  if (!sp) return GSKYHIP_E_ARG;
  return launch_scale_legacy(data, dtype, n, nodata, *sp, out, (hipStream_t)stream);
}

// GradientRGBAPalette (utils/palette.go:27-69); 256 entries, host only.
int gskyhip_gradient_palette(const uint8_t *colours, int n, int interpolate, uint8_t *ramp) {
  auto interp = [](uint8_t a, uint8_t b, long i, long section) {
    const long q = (i * ((long)b - (long)a)) / section;   // Go int, truncating division
    return (uint8_t)(a + (uint8_t)q);                      // uint8 wrap
  };
  if (interpolate) {
    if (n < 2) return GSKYHIP_E_ARG;
    const int bins = n - 1, section = 256 / bins, bonus = 256 - section * bins;
    if (section == 0) return GSKYHIP_E_ARG;  // Go: integer divide by zero panic (palette.go:12)
    int index = 0;
    for (int s = 0; s < bins; s++) {
      const uint8_t *a = colours + 4 * s, *b = colours + 4 * (s + 1);
      const int cnt = section + (s < bonus ? 1 : 0);
      for (int i = 0; i < cnt; i++, index++) {
        uint8_t *o = ramp + 4 * index;
        o[0] = interp(a[0], b[0], i, section);
        o[1] = interp(a[1], b[1], i, section);
        o[2] = interp(a[2], b[2], i, section);
        o[3] = a[3];
      }
    }
  } else {
    if (n < 1) return GSKYHIP_E_ARG;
    const int bins = n, section = 256 / bins, bonus = 256 - section * bins;
    int index = 0;
    for (int s = 0; s < bins; s++) {
      const int cnt = section + (s < bonus ? 1 : 0);
      for (int i = 0; i < cnt; i++, index++) std::memcpy(ramp + 4 * index, colours + 4 * s, 4);
    }
  }
  return 0;
}

int gskyhip_encode_rgba(const uint8_t *const *bands, int nbands, int w, int h, const uint8_t *ramp,
                        uint8_t *rgba, void *stream) {
  if (nbands != 1 && nbands != 3) return GSKYHIP_E_ARG;
  return launch_encode_rgba(bands[0], nbands == 3 ? bands[1] : nullptr, nbands == 3 ? bands[2] : nullptr,
                            nbands, (int64_t)w * h, ramp, rgba, (hipStream_t)stream);
}

int gskyhip_compute_mask(const void *data, int dtype, int64_t n, const gskyhip_mask *mask, uint8_t *out,
                         void *stream) {
  gskyhip_mask m = mask ? *mask : gskyhip_mask{};
  m.ns = 0;
  MaskSpecS ms[4];
  int r = build_mask_specs(&m, ms);
  if (r) return r;
  const int slot = mask_slot_h(dtype);
  if (slot < 0) return GSKYHIP_E_MASK;
  return launch_compute_mask(data, dtype, n, ms[slot], out, (hipStream_t)stream);
}

int gskyhip_drill_rows(int n_bands, int band_strides) { return drill_rows_per_poly(n_bands, band_strides); }

int64_t gskyhip_drill_workspace_size(int n_polys, int64_t mask_bytes, int n_list, int band_strides, int mode) {
  return drill_workspace_size(n_polys, mask_bytes, n_list, band_strides, mode);
}

int gskyhip_drill_batch(const float *stack, int xsize, int ysize, int n_bands, int t_stride, const int32_t *win,
                        const int64_t *mask_off, const uint8_t *masks, int n_polys, int64_t mask_bytes,
                        const int32_t *bands, int n_list, float nodata, float clip_lower, float clip_upper,
                        int pixel_count, int band_strides, int mode, double *out_value, int32_t *out_count,
                        void *workspace, int64_t workspace_bytes, void *stream) {
  DrillCall c;
  c.stack = stack; c.xsize = xsize; c.ysize = ysize; c.n_bands = n_bands; c.t_stride = t_stride;
  c.win = win; c.mask_off = mask_off; c.masks = masks; c.n_polys = n_polys; c.mask_bytes = mask_bytes;
  c.bands = bands; c.n_list = n_list; c.nodata = nodata; c.lo = clip_lower; c.hi = clip_upper;
  c.pixel_count = pixel_count; c.band_strides = band_strides; c.mode = mode;
  c.out_value = out_value; c.out_count = out_count;
  c.workspace = workspace; c.workspace_bytes = workspace_bytes; c.stream = (hipStream_t)stream;
  return launch_drill_batch(c);
}

// Round-1 entry point: sizes the workspace from the windows (synchronous
// read-back) and runs the reference-order batch over bands 1..n_bands.
int gskyhip_drill(const float *stack, int xsize, int ysize, int n_bands, int t_stride, const int32_t *win,
                  const int64_t *mask_off, const uint8_t *masks, int n_polys, float nodata, float clip_lower,
                  float clip_upper, int pixel_count, int band_strides, double *out_value, int32_t *out_count,
                  void *stream) {
  if (n_polys <= 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  std::vector<int32_t> w(4 * (size_t)n_polys);
  std::vector<int64_t> off((size_t)n_polys);
  if (hipMemcpyAsync(w.data(), win, w.size() * 4, hipMemcpyDeviceToHost, s) != hipSuccess ||
      hipMemcpyAsync(off.data(), mask_off, off.size() * 8, hipMemcpyDeviceToHost, s) != hipSuccess ||
      hipStreamSynchronize(s) != hipSuccess)
    return GSKYHIP_E_HIP;
  int64_t mask_bytes = 0;
  for (int p = 0; p < n_polys; p++)
    mask_bytes = std::max<int64_t>(mask_bytes, off[p] + (int64_t)std::max(0, w[4 * p + 2]) * std::max(0, w[4 * p + 3]));
  const int64_t ws = drill_workspace_size(n_polys, mask_bytes, n_bands, band_strides, 0);
  void *buf = nullptr;
  if (hipMallocAsync(&buf, (size_t)ws, s) != hipSuccess) return GSKYHIP_E_HIP;
  const int r = gskyhip_drill_batch(stack, xsize, ysize, n_bands, t_stride, win, mask_off, masks, n_polys,
                                    mask_bytes, nullptr, n_bands, nodata, clip_lower, clip_upper, pixel_count,
                                    band_strides, 0, out_value, out_count, buf, ws, stream);
  if (hipFreeAsync(buf, s) != hipSuccess) return GSKYHIP_E_HIP;
  return r;
}

int gskyhip_drill_merge(const double *values, const int32_t *counts, int n_files, int n_dates, double *out,
                        void *stream) {
  return launch_drill_merge(values, counts, n_files, n_dates, out, (hipStream_t)stream);
}

}  // extern "C"
