// nc4write.cpp -- EncodeGdalOpen / EncodeGdal for format "netcdf"
// (utils/ogc_encoders.go:263-301 creation options COMPRESS=DEFLATE,
// ZLEVEL=6; ows.go:1172 serves it): a WCS coverage held in HBM written as the
// netCDF file GDAL 3.0.1's netCDF driver creates for those options -- the
// classic data model in an HDF5 container (GDAL switches FORMAT to NC4C when
// DEFLATE is asked for), one 2-D variable per band ("Band1", ...; long_name =
// the namespace, as EncodeGdal sets it; _FillValue = the band nodata;
// grid_mapping = "crs"), chunks of one row (GDAL's default chunking),
// shuffle + deflate at ZLEVEL, rows stored bottom-up with increasing y
// coordinates (GDAL's WRITE_BOTTOMUP default), the coordinate variables at
// pixel centres (x / y for projected SRSs, lon / lat for geographic ones),
// the "crs" grid mapping variable with the CF attributes of the SRS, a WKT
// naming the EPSG code (spatial_ref) and GeoTransform, and the global
// Conventions / GDAL / history attributes.
//
// The HDF5 structures are written from the HDF5 file format specification
// 3.0 (the layout netCDF-C 4.x gives a netCDF-4 classic file): superblock 2,
// version-2 object headers with lookup3 checksums, compact links in the root
// group, compact attributes, every dimension a dimension-scale dataset
// (CLASS / NAME / _Netcdf4Dimid), each variable's DIMENSION_LIST a
// variable-length sequence of object references in a global heap, chunked
// layouts (v3) indexed by a version-1 B-tree.  No HDF5 or netCDF library is
// in the image: the files are checked by the product's own reader (hdf5.cpp,
// ingest.hip) and structurally (tests/test_netcdf_out.py) -- parity with
// GDAL's bytes unpinned.  The compression runs on host threads (zlib), one
// chunk (row) at a time, after one device-to-host copy of each band.
#include <hip/hip_runtime.h>
#include <zlib.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../../include/gskyhip.h"

namespace gsky {
namespace {

constexpr uint64_t kUndef = 0xFFFFFFFFFFFFFFFFull;

// H5_checksum_lookup3 (Bob Jenkins' hashlittle, little-endian words).
uint32_t lookup3(const uint8_t *k, size_t length, uint32_t initval = 0) {
  auto rot = [](uint32_t x, int r) { return (x << r) | (x >> (32 - r)); };
  uint32_t a, b, c;
  a = b = c = 0xdeadbeefu + (uint32_t)length + initval;
  auto rd = [&](size_t i) {
    uint32_t v = 0;
    for (int q = 0; q < 4; q++) v |= (uint32_t)k[i + q] << (8 * q);
    return v;
  };
  size_t i = 0;
  while (length - i > 12) {
    a += rd(i); b += rd(i + 4); c += rd(i + 8);
    a -= c; a ^= rot(c, 4); c += b;
    b -= a; b ^= rot(a, 6); a += c;
    c -= b; c ^= rot(b, 8); b += a;
    a -= c; a ^= rot(c, 16); c += b;
    b -= a; b ^= rot(a, 19); a += c;
    c -= b; c ^= rot(b, 4); b += a;
    i += 12;
  }
  if (length - i == 0) return c;
  uint8_t tail[12] = {0};
  std::memcpy(tail, k + i, length - i);
  auto rt = [&](int j) {
    uint32_t v = 0;
    for (int q = 0; q < 4; q++) v |= (uint32_t)tail[j + q] << (8 * q);
    return v;
  };
  a += rt(0); b += rt(4); c += rt(8);
  c ^= b; c -= rot(b, 14);
  a ^= c; a -= rot(c, 11);
  b ^= a; b -= rot(a, 25);
  c ^= b; c -= rot(b, 16);
  a ^= c; a -= rot(c, 4);
  b ^= a; b -= rot(a, 14);
  c ^= b; c -= rot(b, 24);
  return c;
}

// A little-endian byte string.
struct Bytes {
  std::vector<uint8_t> b;
  Bytes &u8(uint32_t v) { b.push_back((uint8_t)v); return *this; }
  Bytes &u16(uint32_t v) { for (int q = 0; q < 2; q++) b.push_back((uint8_t)(v >> (8 * q))); return *this; }
  Bytes &u32(uint32_t v) { for (int q = 0; q < 4; q++) b.push_back((uint8_t)(v >> (8 * q))); return *this; }
  Bytes &u64(uint64_t v) { for (int q = 0; q < 8; q++) b.push_back((uint8_t)(v >> (8 * q))); return *this; }
  Bytes &raw(const void *p, size_t n) { b.insert(b.end(), (const uint8_t *)p, (const uint8_t *)p + n); return *this; }
  Bytes &str(const std::string &s) { return raw(s.data(), s.size()); }
  Bytes &add(const Bytes &o) { return raw(o.b.data(), o.b.size()); }
  Bytes &zero(size_t n) { b.insert(b.end(), n, 0); return *this; }
  size_t size() const { return b.size(); }
};

// The file image: objects appended 8-byte aligned.
struct Img {
  std::vector<uint8_t> b;
  uint64_t alloc(const Bytes &d) { return alloc(d.b.data(), d.b.size()); }
  uint64_t alloc(const void *p, size_t n) {
    b.resize((b.size() + 7) & ~(size_t)7, 0);
    const uint64_t at = b.size();
    b.insert(b.end(), (const uint8_t *)p, (const uint8_t *)p + n);
    return at;
  }
  uint64_t reserve(size_t n) {
    b.resize((b.size() + 7) & ~(size_t)7, 0);
    const uint64_t at = b.size();
    b.resize(b.size() + n, 0);
    return at;
  }
  void put(uint64_t at, const Bytes &d) { std::memcpy(&b[at], d.b.data(), d.b.size()); }
};

// ---------------------------------------------------------------- datatypes / dataspaces (IV.A.2.b, d)
// kind: 'i' signed, 'u' unsigned, 'f' float; little-endian
Bytes dtype_num(char kind, int size) {
  Bytes d;
  if (kind == 'f') {
    d.u8(0x11).u8(0x20).u8(size == 4 ? 31 : 63).u8(0).u32(size);
    if (size == 4) d.u16(0).u16(32).u8(23).u8(8).u8(0).u8(23).u32(127);
    else d.u16(0).u16(64).u8(52).u8(11).u8(0).u8(52).u32(1023);
  } else {
    d.u8(0x10).u8(kind == 'i' ? 0x08 : 0x00).u8(0).u8(0).u32(size).u16(0).u16(8 * size);
  }
  return d;
}

Bytes dtype_str(size_t n) {   // fixed-length, null-terminated ASCII
  Bytes d;
  d.u8(0x13).u8(0x00).u8(0).u8(0).u32((uint32_t)std::max<size_t>(1, n));
  return d;
}

Bytes dtype_vlen_ref() {   // variable-length sequence of object references (DIMENSION_LIST)
  Bytes base;
  base.u8(0x17).u8(0x00).u8(0).u8(0).u32(8);
  Bytes d;
  d.u8(0x19).u8(0x00).u8(0x00).u8(0).u32(16).add(base);
  return d;
}

Bytes dspace(const std::vector<uint64_t> &dims) {   // version 2; rank 0: scalar
  Bytes d;
  d.u8(2).u8((uint32_t)dims.size()).u8(0).u8(dims.empty() ? 0 : 1);
  for (uint64_t x : dims) d.u64(x);
  return d;
}

// ---------------------------------------------------------------- attributes (IV.A.2.m, version 3)
struct Att {
  std::string name;
  Bytes dt, ds, data;
};

Att att_str(const std::string &name, const std::string &v) {
  Att a{name, dtype_str(v.size()), dspace({}), {}};
  a.data.str(v.empty() ? std::string(1, '\0') : v);
  return a;
}

Att att_f64(const std::string &name, const std::vector<double> &v) {
  Att a{name, dtype_num('f', 8), dspace(v.size() == 1 ? std::vector<uint64_t>{} : std::vector<uint64_t>{v.size()}), {}};
  for (double x : v) a.data.raw(&x, 8);
  return a;
}

Att att_i32(const std::string &name, int32_t v) {
  Att a{name, dtype_num('i', 4), dspace({}), {}};
  a.data.raw(&v, 4);
  return a;
}

Att att_typed(const std::string &name, char kind, int size, const void *v) {   // scalar of the variable's type
  Att a{name, dtype_num(kind, size), dspace({}), {}};
  a.data.raw(v, size);
  return a;
}

Bytes att_msg(const Att &a) {
  Bytes m;
  const std::string nb = a.name + std::string(1, '\0');
  m.u8(3).u8(0).u16((uint32_t)nb.size()).u16((uint32_t)a.dt.size()).u16((uint32_t)a.ds.size()).u8(0);
  m.str(nb).add(a.dt).add(a.ds).add(a.data);
  return m;
}

// ---------------------------------------------------------------- object headers (IV.A.1.b, version 2)
uint64_t ohdr(Img &img, const std::vector<std::pair<int, Bytes>> &msgs) {
  Bytes body;
  for (const auto &m : msgs) body.u8((uint32_t)m.first).u16((uint32_t)m.second.size()).u8(0).add(m.second);
  Bytes h;
  h.str("OHDR").u8(2).u8(0x02).u32((uint32_t)body.size()).add(body);   // flags: 4-byte chunk-0 size
  h.u32(lookup3(h.b.data(), h.size()));
  return img.alloc(h);
}

// ---------------------------------------------------------------- chunk index: version-1 B-tree (III.A.1)
constexpr int kBtreeK = 32;   // default chunk B-tree K: nodes hold up to 2K = 64 children

struct ChunkRec { uint64_t row, addr, size; };

// Key of a chunk of (rows x cols) starting at (row, 0): stored size, filter
// mask, offsets (rank + 1: the element dimension 0).
void chunk_key(Bytes &b, uint64_t size, uint64_t row) {
  b.u32((uint32_t)size).u32(0).u64(row).u64(0).u64(0);
}

uint64_t chunk_btree(Img &img, const std::vector<ChunkRec> &chunks, uint64_t n_rows) {
  // level 0: leaves over the chunks; each level above: nodes over the nodes below
  struct Node { uint64_t addr, first_row; };
  auto node = [&](int level, const std::vector<std::pair<uint64_t, uint64_t>> &kids,   // (first row, addr)
                  const std::vector<uint64_t> &sizes) {
    Bytes b;
    b.str("TREE").u8(1).u8((uint32_t)level).u16((uint32_t)kids.size()).u64(kUndef).u64(kUndef);
    for (size_t i = 0; i < kids.size(); i++) {
      chunk_key(b, sizes[i], kids[i].first);
      b.u64(kids[i].second);
    }
    chunk_key(b, 0, n_rows);   // the final key: past the last chunk
    const size_t full = 24 + 2 * kBtreeK * (32 + 8) + 32;
    b.zero(full > b.size() ? full - b.size() : 0);
    return img.alloc(b);
  };
  std::vector<Node> level;
  for (size_t i = 0; i < chunks.size(); i += 2 * kBtreeK) {
    std::vector<std::pair<uint64_t, uint64_t>> kids;
    std::vector<uint64_t> sizes;
    for (size_t j = i; j < std::min(chunks.size(), i + 2 * kBtreeK); j++) {
      kids.push_back({chunks[j].row, chunks[j].addr});
      sizes.push_back(chunks[j].size);
    }
    level.push_back({node(0, kids, sizes), chunks[i].row});
  }
  int lv = 0;
  while (level.size() > 1) {
    lv++;
    std::vector<Node> up;
    for (size_t i = 0; i < level.size(); i += 2 * kBtreeK) {
      std::vector<std::pair<uint64_t, uint64_t>> kids;
      std::vector<uint64_t> sizes;
      for (size_t j = i; j < std::min(level.size(), i + 2 * kBtreeK); j++) {
        kids.push_back({level[j].first_row, level[j].addr});
        sizes.push_back(0);
      }
      up.push_back({node(lv, kids, sizes), level[i].first_row});
    }
    level.swap(up);
  }
  return level.empty() ? kUndef : level[0].addr;
}

// ---------------------------------------------------------------- CRS
// CF grid-mapping attributes of the SRS of `epsg` (CF-1.x Appendix F), the
// family set the warp supports; false when the code is outside it.
bool cf_mapping(int epsg, std::vector<Att> &atts, bool &geographic) {
  char srs[32];
  std::snprintf(srs, sizeof(srs), "EPSG:%d", epsg);
  gskyhip_crs c;
  geographic = false;
  if (epsg <= 0 || gskyhip_crs_from_srs(srs, &c) != 0) return false;
  const double rad = 180.0 / M_PI;
  auto ellps = [&]() {
    if (c.es == 0.0) {
      atts.push_back(att_f64("earth_radius", {c.a}));
    } else {
      atts.push_back(att_f64("semi_major_axis", {c.a}));
      const double f = 1.0 - std::sqrt(1.0 - c.es);
      atts.push_back(att_f64("inverse_flattening", {1.0 / f}));
    }
  };
  switch (c.kind) {
    case GSKYHIP_CRS_LONGLAT:
      geographic = true;
      atts.push_back(att_str("grid_mapping_name", "latitude_longitude"));
      ellps();
      atts.push_back(att_f64("longitude_of_prime_meridian", {0.0}));
      return true;
    case GSKYHIP_CRS_WEBMERC:
      atts.push_back(att_str("grid_mapping_name", "mercator"));
      atts.push_back(att_f64("standard_parallel", {0.0}));
      atts.push_back(att_f64("longitude_of_projection_origin", {0.0}));
      atts.push_back(att_f64("false_easting", {0.0}));
      atts.push_back(att_f64("false_northing", {0.0}));
      atts.push_back(att_f64("earth_radius", {c.a}));
      return true;
    case GSKYHIP_CRS_AEA:
      atts.push_back(att_str("grid_mapping_name", "albers_conical_equal_area"));
      atts.push_back(att_f64("standard_parallel", {c.phi1 * rad, c.phi2 * rad}));
      atts.push_back(att_f64("latitude_of_projection_origin", {c.phi0 * rad}));
      atts.push_back(att_f64("longitude_of_central_meridian", {c.lam0 * rad}));
      atts.push_back(att_f64("false_easting", {c.x0}));
      atts.push_back(att_f64("false_northing", {c.y0}));
      ellps();
      return true;
    case GSKYHIP_CRS_SINU:
      atts.push_back(att_str("grid_mapping_name", "sinusoidal"));
      atts.push_back(att_f64("longitude_of_central_meridian", {c.lam0 * rad}));
      atts.push_back(att_f64("false_easting", {c.x0}));
      atts.push_back(att_f64("false_northing", {c.y0}));
      atts.push_back(att_f64("earth_radius", {c.a}));
      return true;
    case GSKYHIP_CRS_TMERC:
      atts.push_back(att_str("grid_mapping_name", "transverse_mercator"));
      atts.push_back(att_f64("longitude_of_central_meridian", {c.lam0 * rad}));
      atts.push_back(att_f64("latitude_of_projection_origin", {c.phi0 * rad}));
      atts.push_back(att_f64("scale_factor_at_central_meridian", {c.k0}));
      atts.push_back(att_f64("false_easting", {c.x0}));
      atts.push_back(att_f64("false_northing", {c.y0}));
      ellps();
      return true;
    case GSKYHIP_CRS_LCC:
      atts.push_back(att_str("grid_mapping_name", "lambert_conformal_conic"));
      atts.push_back(att_f64("standard_parallel", {c.phi1 * rad, c.phi2 * rad}));
      atts.push_back(att_f64("latitude_of_projection_origin", {c.phi0 * rad}));
      atts.push_back(att_f64("longitude_of_central_meridian", {c.lam0 * rad}));
      atts.push_back(att_f64("false_easting", {c.x0}));
      atts.push_back(att_f64("false_northing", {c.y0}));
      ellps();
      return true;
    case GSKYHIP_CRS_STERE_POLAR:
      atts.push_back(att_str("grid_mapping_name", "polar_stereographic"));
      atts.push_back(att_f64("latitude_of_projection_origin", {c.phi0 > 0 ? 90.0 : -90.0}));
      atts.push_back(att_f64("straight_vertical_longitude_from_pole", {c.lam0 * rad}));
      atts.push_back(att_f64("standard_parallel", {(c.phi0 > 0 ? 1.0 : -1.0) * c.phi1 * rad}));
      atts.push_back(att_f64("false_easting", {c.x0}));
      atts.push_back(att_f64("false_northing", {c.y0}));
      ellps();
      return true;
    default:
      return false;
  }
}

// The netCDF classic type of a GSKYHIP dtype in an NC4C file (GDAL's netCDF
// CreateLL: Byte -> NC_BYTE + _Unsigned "true", SIGNEDBYTE -> NC_BYTE, Int16
// -> NC_SHORT, UInt16 -> NC_INT (no unsigned types in the classic model),
// Float32 -> NC_FLOAT): kind / size in the file.
bool nc_type_of(int dtype, char &kind, int &size, bool &unsigned_att) {
  unsigned_att = false;
  switch (dtype) {
    case GSKYHIP_BYTE: kind = 'i'; size = 1; unsigned_att = true; return true;
    case GSKYHIP_SIGNEDBYTE: kind = 'i'; size = 1; return true;
    case GSKYHIP_INT16: kind = 'i'; size = 2; return true;
    case GSKYHIP_UINT16: kind = 'i'; size = 4; return true;
    case GSKYHIP_FLOAT32: kind = 'f'; size = 4; return true;
    default: return false;
  }
}

int src_size(int dtype) {
  switch (dtype) {
    case GSKYHIP_BYTE: case GSKYHIP_SIGNEDBYTE: return 1;
    case GSKYHIP_INT16: case GSKYHIP_UINT16: return 2;
    case GSKYHIP_FLOAT32: return 4;
    default: return 0;
  }
}

bool is_empty_tile(const char *name) { return name && std::strncmp(name, "EmptyTile", 9) == 0; }

}  // namespace
}  // namespace gsky

using namespace gsky;

extern "C" int64_t gskyhip_netcdf_bound(int width, int height, int n_bands, int dtype) {
  char kind;
  int es;
  bool us;
  if (width <= 0 || height <= 0 || n_bands <= 0 || !nc_type_of(dtype, kind, es, us)) return -1;
  const int64_t row = (int64_t)width * es;
  const int64_t zrow = (int64_t)compressBound((uLong)row) + 16;
  const int64_t btree_nodes = (height + 63) / 64 * 2 + 8;
  return (int64_t)n_bands * ((int64_t)height * zrow + btree_nodes * (24 + 64 * 40 + 32 + 8) + 8192) +
         ((int64_t)width + height) * 8 + 65536 + 16384;
}

// The file from host bands (each height x width of dtype, row-major; NULL or
// an "EmptyTile" name: a skipped band of zeros).
static int encode_netcdf_host(const void *const *bands, int n_bands, int dtype, int width, int height,
                              const double *geot, int epsg, const double *nodata, const char *const *names, int zlevel,
                              int n_threads, uint8_t *out, int64_t capacity, int64_t *size) {
  char kind;
  int es;
  bool unsigned_att;
  if (!bands || n_bands <= 0 || width <= 0 || height <= 0 || !geot || !out || !size || zlevel < 0 || zlevel > 9 ||
      !nc_type_of(dtype, kind, es, unsigned_att))
    return GSKYHIP_E_ARG;
  const int ss = src_size(dtype);
  // ---- the bands widened to the file type (UInt16 -> int32)
  const int64_t npx = (int64_t)width * height;
  std::vector<std::vector<uint8_t>> host(n_bands);
  for (int k = 0; k < n_bands; k++) {
    host[k].assign((size_t)(npx * es), 0);
    const bool empty = names && is_empty_tile(names[k]);
    if (empty || !bands[k]) {   // EncodeGdal skips the band: its samples stay the dataset fill (0)
      continue;
    }
    const uint8_t *raw = (const uint8_t *)bands[k];
    if (dtype == GSKYHIP_UINT16) {
      for (int64_t i = 0; i < npx; i++) {
        uint16_t v;
        std::memcpy(&v, &raw[(size_t)i * 2], 2);
        const int32_t w = v;
        std::memcpy(&host[k][(size_t)i * 4], &w, 4);
      }
    } else {
      std::memcpy(host[k].data(), raw, (size_t)(npx * ss));
    }
  }
  std::vector<Att> crs_atts;
  bool geographic = false;
  const bool have_crs = cf_mapping(epsg, crs_atts, geographic);

  Img img;
  img.reserve(48);   // superblock 2
  // the global heap collection of the DIMENSION_LIST references (written last)
  const size_t gheap_size = 4096 + (size_t)n_bands * 64;
  const uint64_t gheap_at = img.reserve(gheap_size);
  std::vector<Bytes> gobjs;
  auto gheap_add = [&](const Bytes &o) {
    gobjs.push_back(o);
    return (uint32_t)gobjs.size();
  };
  std::vector<std::pair<std::string, uint64_t>> links;
  // ---- dimensions: y / x (lat / lon for a geographic SRS), coordinates at
  // pixel centres, y increasing (rows stored bottom-up)
  const std::string xn = geographic ? "lon" : "x", yn = geographic ? "lat" : "y";
  uint64_t dim_addr[2];
  for (int d = 0; d < 2; d++) {   // 0: y, 1: x
    const bool isy = d == 0;
    const int n = isy ? height : width;
    std::vector<double> cv(n);
    for (int i = 0; i < n; i++)
      cv[i] = isy ? geot[3] + ((double)(height - 1 - i) + 0.5) * geot[5] : geot[0] + ((double)i + 0.5) * geot[1];
    Bytes data;
    data.raw(cv.data(), cv.size() * 8);
    const uint64_t data_at = img.alloc(data);
    std::vector<std::pair<int, Bytes>> msgs;
    msgs.push_back({0x01, dspace({(uint64_t)n})});
    msgs.push_back({0x03, dtype_num('f', 8)});
    Bytes fv;   // fill value v3: allocation early, write time "if set", defined: NC_FILL_DOUBLE
    const double fd = 9.9692099683868690e+36;
    fv.u8(3).u8(1 | (2 << 2) | 0x20).u32(8).raw(&fd, 8);
    msgs.push_back({0x05, fv});
    Bytes lay;
    lay.u8(3).u8(1).u64(data_at).u64(data.size());
    msgs.push_back({0x08, lay});
    std::vector<Att> atts;
    atts.push_back(att_str("CLASS", "DIMENSION_SCALE"));
    atts.push_back(att_str("NAME", isy ? yn : xn));
    atts.push_back(att_i32("_Netcdf4Dimid", d));
    if (geographic) {
      atts.push_back(att_str("standard_name", isy ? "latitude" : "longitude"));
      atts.push_back(att_str("long_name", isy ? "latitude" : "longitude"));
      atts.push_back(att_str("units", isy ? "degrees_north" : "degrees_east"));
    } else {
      atts.push_back(att_str("standard_name", isy ? "projection_y_coordinate" : "projection_x_coordinate"));
      atts.push_back(att_str("long_name", isy ? "y coordinate of projection" : "x coordinate of projection"));
      atts.push_back(att_str("units", "m"));
    }
    for (const Att &a : atts) msgs.push_back({0x0C, att_msg(a)});
    dim_addr[d] = ohdr(img, msgs);
    links.push_back({isy ? yn : xn, dim_addr[d]});
  }
  // ---- the grid mapping variable (scalar int, never written)
  if (have_crs) {
    std::vector<std::pair<int, Bytes>> msgs;
    msgs.push_back({0x01, dspace({})});
    msgs.push_back({0x03, dtype_num('i', 4)});
    Bytes fv;
    const int32_t fi = -2147483647;   // NC_FILL_INT
    fv.u8(3).u8(1 | (2 << 2) | 0x20).u32(4).raw(&fi, 4);
    msgs.push_back({0x05, fv});
    Bytes lay;
    lay.u8(3).u8(1).u64(kUndef).u64(4);   // contiguous, not allocated: reads as the fill
    msgs.push_back({0x08, lay});
    char wkt[160], gts[256];
    std::snprintf(wkt, sizeof(wkt), "%s[\"EPSG:%d\",AUTHORITY[\"EPSG\",\"%d\"]]", geographic ? "GEOGCS" : "PROJCS", epsg,
                  epsg);
    std::snprintf(gts, sizeof(gts), "%.17g %.17g %.17g %.17g %.17g %.17g", geot[0], geot[1], geot[2], geot[3], geot[4],
                  geot[5]);
    crs_atts.push_back(att_str("spatial_ref", wkt));
    crs_atts.push_back(att_str("crs_wkt", wkt));
    crs_atts.push_back(att_str("GeoTransform", gts));
    for (const Att &a : crs_atts) msgs.push_back({0x0C, att_msg(a)});
    links.push_back({"crs", ohdr(img, msgs)});
  }
  // ---- the bands: chunks of one row, shuffle + deflate, bottom-up
  const size_t row_bytes = (size_t)width * es;
  for (int k = 0; k < n_bands; k++) {
    const bool empty = names && is_empty_tile(names[k]);
    // compress the rows on host threads (file row j = image row height - 1 - j)
    std::vector<std::vector<uint8_t>> z((size_t)height);
    std::atomic<int> next{0};
    std::atomic<int> fail{0};
    auto work = [&]() {
      std::vector<uint8_t> shuf(row_bytes);
      for (;;) {
        const int j = next.fetch_add(1);
        if (j >= height) break;
        const uint8_t *src = host[k].data() + (size_t)(height - 1 - j) * row_bytes;
        for (int b = 0; b < es; b++)   // shuffle: byte b of every element, then byte b + 1
          for (int i = 0; i < width; i++) shuf[(size_t)b * width + i] = src[(size_t)i * es + b];
        uLongf zl = compressBound((uLong)row_bytes);
        z[j].resize(zl);
        if (compress2(z[j].data(), &zl, shuf.data(), (uLong)row_bytes, zlevel) != Z_OK) fail = 1;
        z[j].resize(zl);
      }
    };
    const int nt = std::max(1, std::min(n_threads > 0 ? n_threads : 1, 64));
    std::vector<std::thread> th;
    for (int t = 1; t < nt; t++) th.emplace_back(work);
    work();
    for (auto &t : th) t.join();
    if (fail) return GSKYHIP_E_HIP;
    std::vector<ChunkRec> chunks((size_t)height);
    for (int j = 0; j < height; j++) {
      chunks[j].row = (uint64_t)j;
      chunks[j].addr = img.alloc(z[j].data(), z[j].size());
      chunks[j].size = z[j].size();
      std::vector<uint8_t>().swap(z[j]);
    }
    const uint64_t btree = chunk_btree(img, chunks, (uint64_t)height);
    std::vector<std::pair<int, Bytes>> msgs;
    msgs.push_back({0x01, dspace({(uint64_t)height, (uint64_t)width})});
    msgs.push_back({0x03, dtype_num(kind, es)});
    // the fill value: the band nodata in the file type (netCDF-C sets the
    // dataset fill property to _FillValue)
    uint8_t fvb[8] = {0};
    const bool has_nd = nodata && !empty;
    const double nd = has_nd ? nodata[k] : 0.0;
    if (kind == 'f') { const float f = (float)nd; std::memcpy(fvb, &f, 4); }
    else if (es == 1) { const int8_t v = (int8_t)(int32_t)(uint32_t)(int64_t)nd; std::memcpy(fvb, &v, 1); }
    else if (es == 2) { const int16_t v = (int16_t)(int64_t)nd; std::memcpy(fvb, &v, 2); }
    else { const int32_t v = (int32_t)(int64_t)nd; std::memcpy(fvb, &v, 4); }
    if (has_nd) {
      Bytes fv;
      fv.u8(3).u8(2 | (2 << 2) | 0x20).u32(es).raw(fvb, es);   // allocation incremental, write if set, defined
      msgs.push_back({0x05, fv});
    }
    Bytes lay;   // layout v3 chunked: rank + 1 dims (the last: element size)
    lay.u8(3).u8(2).u8(3).u64(btree).u32(1).u32((uint32_t)width).u32((uint32_t)es);
    msgs.push_back({0x08, lay});
    Bytes fl;   // filter pipeline v1: shuffle (element size), deflate (level)
    fl.u8(1).u8(2).zero(6);
    fl.u16(2).u16(0).u16(1).u16(1).u32(es).u32(0);
    fl.u16(1).u16(0).u16(1).u16(1).u32((uint32_t)zlevel).u32(0);
    msgs.push_back({0x0B, fl});
    std::vector<Att> atts;
    // DIMENSION_LIST: for each dimension one object reference in the global heap
    Att dl{"DIMENSION_LIST", dtype_vlen_ref(), dspace({2}), {}};
    for (int d = 0; d < 2; d++) {
      Bytes ref;
      ref.u64(dim_addr[d]);
      const uint32_t idx = gheap_add(ref);
      dl.data.u32(1).u64(gheap_at).u32(idx);
    }
    atts.push_back(dl);
    if (has_nd) atts.push_back(att_typed("_FillValue", kind, es, fvb));
    if (unsigned_att) atts.push_back(att_str("_Unsigned", "true"));
    if (names && names[k] && !empty) atts.push_back(att_str("long_name", names[k]));
    if (have_crs) atts.push_back(att_str("grid_mapping", "crs"));
    for (const Att &a : atts) msgs.push_back({0x0C, att_msg(a)});
    links.push_back({"Band" + std::to_string(k + 1), ohdr(img, msgs)});
  }
  // ---- the root group: link info, group info, links, global attributes
  std::vector<std::pair<int, Bytes>> msgs;
  Bytes li;
  li.u8(0).u8(0).u64(kUndef).u64(kUndef);
  msgs.push_back({0x02, li});
  Bytes gi;
  gi.u8(0).u8(0);
  msgs.push_back({0x0A, gi});
  for (const auto &l : links) {
    Bytes m;
    m.u8(1).u8(0).u8((uint32_t)l.first.size()).str(l.first).u64(l.second);
    msgs.push_back({0x06, m});
  }
  std::vector<Att> gatts;
  gatts.push_back(att_str("Conventions", "CF-1.5"));
  gatts.push_back(att_str("GDAL", "GDAL 3.0.1 netCDF driver layout (gskyhip_encode_netcdf)"));
  gatts.push_back(att_str("history", "EncodeGdal format=netcdf COMPRESS=DEFLATE ZLEVEL=" + std::to_string(zlevel)));
  gatts.push_back(att_i32("_nc3_strict", 1));
  for (const Att &a : gatts) msgs.push_back({0x0C, att_msg(a)});
  const uint64_t root = ohdr(img, msgs);
  // ---- the global heap collection (III.E)
  {
    Bytes body;
    for (size_t i = 0; i < gobjs.size(); i++) {
      body.u16((uint32_t)(i + 1)).u16(1).u32(0).u64(gobjs[i].size()).add(gobjs[i]);
      body.zero((8 - gobjs[i].size() % 8) % 8);
    }
    if (16 + body.size() + 16 > gheap_size) return GSKYHIP_E_ARG;
    const uint64_t free_sz = gheap_size - 16 - body.size();
    body.u16(0).u16(0).u32(0).u64(free_sz);
    Bytes g;
    g.str("GCOL").u8(1).zero(3).u64(gheap_size).add(body);
    g.zero(gheap_size - g.size());
    img.put(gheap_at, g);
  }
  // ---- superblock 2
  const uint64_t eof = img.b.size();
  Bytes sb;
  sb.raw("\x89HDF\r\n\x1a\n", 8).u8(2).u8(8).u8(8).u8(0).u64(0).u64(kUndef).u64(eof).u64(root);
  sb.u32(lookup3(sb.b.data(), sb.size()));
  img.put(0, sb);
  if ((int64_t)img.b.size() > capacity) return GSKYHIP_E_ARG;
  std::memcpy(out, img.b.data(), img.b.size());
  *size = (int64_t)img.b.size();
  return 0;
}

extern "C" int gskyhip_encode_netcdf_host(const void *const *bands, int n_bands, int dtype, int width, int height,
                                          const double *geot, int epsg, const double *nodata,
                                          const char *const *names, int zlevel, int n_threads, uint8_t *out,
                                          int64_t capacity, int64_t *size) {
  return encode_netcdf_host(bands, n_bands, dtype, width, height, geot, epsg, nodata, names, zlevel, n_threads, out,
                            capacity, size);
}

extern "C" int gskyhip_encode_netcdf(const void *const *bands, int n_bands, int dtype, int width, int height,
                                     const double *geot, int epsg, const double *nodata, const char *const *names,
                                     int zlevel, int n_threads, uint8_t *out, int64_t capacity, int64_t *size,
                                     void *stream) {
  const int ss = src_size(dtype);
  if (!bands || n_bands <= 0 || width <= 0 || height <= 0 || ss <= 0) return GSKYHIP_E_ARG;
  hipStream_t s = (hipStream_t)stream;
  const size_t nb = (size_t)width * height * ss;
  std::vector<std::vector<uint8_t>> host(n_bands);
  std::vector<const void *> ptrs(n_bands, nullptr);
  for (int k = 0; k < n_bands; k++) {
    if (!bands[k] || (names && is_empty_tile(names[k]))) continue;
    host[k].resize(nb);
    if (hipMemcpyAsync(host[k].data(), bands[k], nb, hipMemcpyDeviceToHost, s) != hipSuccess) return GSKYHIP_E_HIP;
    ptrs[k] = host[k].data();
  }
  if (hipStreamSynchronize(s) != hipSuccess) return GSKYHIP_E_HIP;
  return encode_netcdf_host(ptrs.data(), n_bands, dtype, width, height, geot, epsg, nodata, names, zlevel, n_threads,
                            out, capacity, size);
}
