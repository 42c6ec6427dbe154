// ingest.hip -- native granule ingest: GeoTIFF files
// decoded into HBM, the step GDALOpenEx + GDALRasterIO take in the worker
// (worker/gdalprocess/warp.go:89-101, drill.go:61-69, 142) before the warp.
//
// Reader: classic TIFF and BigTIFF, little or big endian; striped or tiled;
// chunky or planar; 8/16/32/64-bit unsigned, signed and float samples;
// compression none (1), LZW (5), Deflate (8, 32946) and PackBits (32773);
// predictor 1 (none), 2 (horizontal differencing) and 3 (floating point).
// Georeferencing as GDAL's GTiff driver reads it: ModelTransformation, or
// ModelTiepoint + ModelPixelScale (PixelIsPoint shifted by half a pixel),
// EPSG from ProjectedCSTypeGeoKey / GeographicTypeGeoKey (user-defined
// sinusoidal on the MODIS sphere -> "MODIS"), nodata from GDAL_NODATA
// (42113), internal overviews from the reduced-resolution IFDs in file
// order (GDALGetOverview order).
//
// netCDF classic (CDF-1, CDF-2 64-bit offsets, CDF-5 64-bit data), the
// format the GSKY_netCDF driver opens with nc_open (libs/gdal/frmts/
// gsky_netcdf/netcdfdataset.cpp): "NETCDF:file:var" or a file with one data
// variable; the band is the index along the leading dimension of a 3-D
// variable (band_query, netcdfdataset.cpp:6994-7021, warp.go:89-101); the
// geotransform from the 1-D coordinate variables as the driver computes it
// (netcdfdataset.cpp:3504-3655: actual_range when present, y reversed when
// increasing -- bBottomUp, rows then read south-up so row 0 is the north);
// nodata from _FillValue / missing_value / the type default and NC_BYTE
// signedness as netCDFRasterBand sets them; EPSG:4326 for lon / lat axes,
// else an EPSG from the grid mapping's crs_wkt / spatial_ref AUTHORITY.
// netCDF-4 (HDF5) files: the HDF5 subset of hdf5.h (host parse, chunks
// inflated / unshuffled on host threads), mapped to the same variables,
// dimensions and attributes netCDF-C reports.
//
// Device path: the band's blocks are decompressed and un-predicted by host
// threads (zlib / LZW / PackBits are byte-serial), staged block-major in
// pinned memory, copied to HBM in one transfer and placed row-major by
// assemble_kernel (a thread per output element; edge blocks clipped).
#include <hip/hip_runtime.h>
#include <zlib.h>

#include <algorithm>
#include <map>
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../../include/gskyhip.h"
#include "hdf5.h"

namespace gsky {
namespace {

struct Ifd {
  int64_t width = 0, height = 0;
  int bits = 0, spp = 1, fmt = 1, compression = 1, predictor = 1, planar = 1;
  int64_t block_w = 0, block_h = 0;   // tile size, or width x RowsPerStrip
  bool tiled = false;
  int subfile = 0;
  std::vector<uint64_t> offsets, counts;
  std::vector<double> scale, tiepoint, transform;
  std::vector<uint16_t> geokeys;
  std::vector<double> geodoubles;
  std::string nodata;
};

struct Tiff {
  std::vector<uint8_t> buf;   // the whole file (memory of a granule band is read whole anyway)
  bool be = false, big = false;
  std::vector<Ifd> ifds;

  uint16_t u16(uint64_t o) const {
    uint16_t v;
    std::memcpy(&v, &buf[o], 2);
    return be ? (uint16_t)((v >> 8) | (v << 8)) : v;
  }
  uint32_t u32(uint64_t o) const {
    uint32_t v;
    std::memcpy(&v, &buf[o], 4);
    return be ? __builtin_bswap32(v) : v;
  }
  uint64_t u64(uint64_t o) const {
    uint64_t v;
    std::memcpy(&v, &buf[o], 8);
    return be ? __builtin_bswap64(v) : v;
  }
  double f64(uint64_t o) const {
    const uint64_t v = u64(o);
    double d;
    std::memcpy(&d, &v, 8);
    return d;
  }
};

int type_bytes(int t) {
  switch (t) {
    case 1: case 2: case 6: case 7: return 1;
    case 3: case 8: return 2;
    case 4: case 9: case 11: case 13: return 4;
    case 5: case 10: case 12: case 16: case 17: case 18: return 8;
    default: return 0;
  }
}

// Parse every IFD; false on a malformed file.
bool parse(Tiff &t) {
  const std::vector<uint8_t> &b = t.buf;
  if (b.size() < 16) return false;
  if (b[0] == 'I' && b[1] == 'I') t.be = false;
  else if (b[0] == 'M' && b[1] == 'M') t.be = true;
  else return false;
  const uint16_t magic = t.u16(2);
  if (magic == 42) t.big = false;
  else if (magic == 43 && t.u16(4) == 8) t.big = true;
  else return false;
  uint64_t off = t.big ? t.u64(8) : t.u32(4);
  for (int guard = 0; off && guard < 64; guard++) {
    const uint64_t esz = t.big ? 20 : 12, hdr = t.big ? 8 : 2;
    if (off + hdr > b.size()) return false;
    const uint64_t n = t.big ? t.u64(off) : t.u16(off);
    if (off + hdr + n * esz + (t.big ? 8 : 4) > b.size()) return false;
    Ifd d;
    for (uint64_t i = 0; i < n; i++) {
      const uint64_t e = off + hdr + i * esz;
      const int tag = t.u16(e), typ = t.u16(e + 2);
      const uint64_t cnt = t.big ? t.u64(e + 4) : t.u32(e + 4);
      const int tb = type_bytes(typ);
      if (tb == 0 || cnt == 0) continue;   // unknown type; a tag with no value is ignored
      if (cnt > b.size() / (uint64_t)tb) return false;   // before the multiplication can overflow
      const uint64_t inl = t.big ? 8 : 4;
      const uint64_t voff = e + (t.big ? 12 : 8);
      const uint64_t data = (uint64_t)tb * cnt <= inl ? voff : (t.big ? t.u64(voff) : t.u32(voff));
      if (data > b.size() || (uint64_t)tb * cnt > b.size() - data) return false;
      auto ints = [&]() {
        std::vector<uint64_t> v(cnt);
        for (uint64_t k = 0; k < cnt; k++) {
          const uint64_t p = data + k * tb;
          v[k] = tb == 1 ? b[p] : tb == 2 ? t.u16(p) : tb == 4 ? t.u32(p) : t.u64(p);
        }
        return v;
      };
      auto dbls = [&]() {
        std::vector<double> v(cnt);
        if (typ == 12) {
          for (uint64_t k = 0; k < cnt; k++) v[k] = t.f64(data + 8 * k);
        } else {
          const std::vector<uint64_t> iv = ints();
          for (uint64_t k = 0; k < cnt; k++) v[k] = (double)iv[k];
        }
        return v;
      };
      switch (tag) {
        case 254: d.subfile = (int)ints()[0]; break;
        case 256: d.width = (int64_t)ints()[0]; break;
        case 257: d.height = (int64_t)ints()[0]; break;
        case 258: d.bits = (int)ints()[0]; break;
        case 259: d.compression = (int)ints()[0]; break;
        case 273: case 324: d.offsets = ints(); d.tiled = d.tiled || tag == 324; break;
        case 277: d.spp = (int)ints()[0]; break;
        case 278: d.block_h = (int64_t)ints()[0]; break;
        case 279: case 325: d.counts = ints(); break;
        case 284: d.planar = (int)ints()[0]; break;
        case 317: d.predictor = (int)ints()[0]; break;
        case 322: d.block_w = (int64_t)ints()[0]; break;
        case 323: d.block_h = (int64_t)ints()[0]; break;
        case 339: d.fmt = (int)ints()[0]; break;
        case 33550: d.scale = dbls(); break;
        case 33922: d.tiepoint = dbls(); break;
        case 34264: d.transform = dbls(); break;
        case 34735: { auto v = ints(); d.geokeys.assign(v.begin(), v.end()); break; }
        case 34736: d.geodoubles = dbls(); break;
        case 42113: d.nodata.assign((const char *)&b[data], (size_t)cnt); break;
        default: break;
      }
    }
    if (!d.tiled) {
      d.block_w = d.width;
      if (d.block_h <= 0 || d.block_h > d.height) d.block_h = d.height;
    }
    if (d.width <= 0 || d.height <= 0 || d.block_w <= 0 || d.block_h <= 0 || d.offsets.empty() ||
        d.offsets.size() != d.counts.size())
      return false;
    // sizes a corrupt file could make absurd (every decoder buffer is sized
    // from these): a raster side <= 2^24, a sample of 1-64 bits, <= 64
    // samples, one decoded block <= 1 GiB
    if (d.width > (1 << 24) || d.height > (1 << 24) || d.block_w > (1 << 24) || d.block_h > (1 << 24) ||
        d.bits <= 0 || d.bits > 64 || d.spp <= 0 || d.spp > 64 ||
        (uint64_t)d.block_w * (uint64_t)d.block_h * (uint64_t)d.spp * (uint64_t)((d.bits + 7) / 8) > (1ull << 30))
      return false;
    t.ifds.push_back(std::move(d));
    off = t.big ? t.u64(off + hdr + n * esz) : t.u32(off + hdr + n * esz);
  }
  return !t.ifds.empty();
}

bool read_file(const char *path, std::vector<uint8_t> &out) {
  FILE *f = std::fopen(path, "rb");
  if (!f) return false;
  std::fseek(f, 0, SEEK_END);
  const long n = std::ftell(f);
  std::fseek(f, 0, SEEK_SET);
  out.resize(n > 0 ? (size_t)n : 0);
  const bool ok = n > 0 && std::fread(out.data(), 1, (size_t)n, f) == (size_t)n;
  std::fclose(f);
  return ok;
}

int dtype_of(const Ifd &d, int &signed_byte) {
  signed_byte = 0;
  if (d.fmt == 3) return d.bits == 32 ? GSKYHIP_FLOAT32 : d.bits == 64 ? GSKYHIP_FLOAT64 : 0;
  const bool sgn = d.fmt == 2;
  switch (d.bits) {
    case 8: signed_byte = sgn ? 1 : 0; return GSKYHIP_BYTE;
    case 16: return sgn ? GSKYHIP_INT16 : GSKYHIP_UINT16;
    case 32: return sgn ? GSKYHIP_INT32 : GSKYHIP_UINT32;
    default: return 0;
  }
}

// TIFF LZW (MSB-first codes, the code width grows one code early).
bool lzw_decode(const uint8_t *in, size_t n, uint8_t *out, size_t cap) {
  std::vector<uint32_t> prefix(4096), first(4096);
  std::vector<uint8_t> suffix(4096);
  std::vector<uint16_t> len(4096);
  for (int i = 0; i < 256; i++) { suffix[i] = (uint8_t)i; len[i] = 1; prefix[i] = 0xFFFF; first[i] = i; }
  size_t op = 0;
  uint64_t bitbuf = 0;
  int bits = 0, width = 9, next = 258;
  int old = -1;
  size_t ip = 0;
  std::vector<uint8_t> tmp(4096);
  auto emit = [&](int code) -> bool {
    const int l = len[code];
    if (op + l > cap) return false;
    int c = code;
    for (int k = l - 1; k >= 0; k--) { out[op + k] = suffix[c]; c = (int)prefix[c]; }
    op += l;
    return true;
  };
  for (;;) {
    while (bits < width) {
      if (ip >= n) return op == cap;
      bitbuf = (bitbuf << 8) | in[ip++];
      bits += 8;
    }
    const int code = (int)((bitbuf >> (bits - width)) & ((1u << width) - 1));
    bits -= width;
    if (code == 257) break;   // EOI
    if (code == 256) {        // clear
      width = 9; next = 258; old = -1;
      continue;
    }
    if (old < 0) {
      if (code > 255 || !emit(code)) return false;
      old = code;
      continue;
    }
    if (code < next) {
      if (!emit(code)) return false;
      if (next < 4096) { prefix[next] = old; suffix[next] = (uint8_t)first[code]; len[next] = len[old] + 1;
                         first[next] = first[old]; next++; }
    } else if (code == next && next < 4096) {
      prefix[next] = old; suffix[next] = (uint8_t)first[old]; len[next] = len[old] + 1; first[next] = first[old];
      next++;
      if (!emit(code)) return false;
    } else {
      return false;
    }
    old = code;
    if (next + 1 >= (1 << width) && width < 12) width++;
  }
  return op == cap;
}

bool packbits_decode(const uint8_t *in, size_t n, uint8_t *out, size_t cap) {
  size_t ip = 0, op = 0;
  while (ip < n && op < cap) {
    const int8_t h = (int8_t)in[ip++];
    if (h >= 0) {
      const size_t l = (size_t)h + 1;
      if (ip + l > n || op + l > cap) return false;
      std::memcpy(out + op, in + ip, l);
      ip += l; op += l;
    } else if (h != -128) {
      const size_t l = (size_t)(1 - h);
      if (ip >= n || op + l > cap) return false;
      std::memset(out + op, in[ip++], l);
      op += l;
    }
  }
  return op == cap;
}

// Decode one block into `out` (block_w x rows x spp samples of `bytes`, the
// block's own layout): decompression, byte order, predictor.
bool decode_block(const Tiff &t, const Ifd &d, size_t bi, int64_t rows, int samples, uint8_t *out) {
  const int bytes = d.bits / 8;
  const size_t row_bytes = (size_t)d.block_w * samples * bytes;
  const size_t cap = row_bytes * rows;
  const uint64_t off = d.offsets[bi], cnt = d.counts[bi];
  if (off + cnt > t.buf.size()) return false;
  const uint8_t *in = &t.buf[off];
  bool ok;
  switch (d.compression) {
    case 1: ok = cnt >= cap; if (ok) std::memcpy(out, in, cap); break;
    case 8: case 32946: { uLongf dl = (uLongf)cap; ok = uncompress(out, &dl, in, (uLong)cnt) == Z_OK && dl == cap;
                          if (!ok) {   // a block may carry more rows than the image has (strips): accept a short tail
                            std::vector<uint8_t> big(cap + row_bytes * d.block_h);
                            uLongf dl2 = (uLongf)big.size();
                            const int z = uncompress(big.data(), &dl2, in, (uLong)cnt);
                            ok = (z == Z_OK) && dl2 >= cap;
                            if (ok) std::memcpy(out, big.data(), cap);
                          }
                          break; }
    case 5: ok = lzw_decode(in, cnt, out, cap); break;
    case 32773: ok = packbits_decode(in, cnt, out, cap); break;
    default: return false;
  }
  if (!ok) return false;
  if (t.be && bytes > 1 && d.predictor != 3) {   // to host (little endian) order
    for (size_t i = 0; i < cap; i += bytes) std::reverse(out + i, out + i + bytes);
  }
  if (d.predictor == 2) {   // horizontal differencing per sample
    for (int64_t r = 0; r < rows; r++) {
      uint8_t *row = out + r * row_bytes;
      const int64_t n = d.block_w * samples;
      if (bytes == 1) { for (int64_t i = samples; i < n; i++) row[i] = (uint8_t)(row[i] + row[i - samples]); }
      else if (bytes == 2) { uint16_t *v = (uint16_t *)row; for (int64_t i = samples; i < n; i++) v[i] = (uint16_t)(v[i] + v[i - samples]); }
      else if (bytes == 4) { uint32_t *v = (uint32_t *)row; for (int64_t i = samples; i < n; i++) v[i] += v[i - samples]; }
      else { uint64_t *v = (uint64_t *)row; for (int64_t i = samples; i < n; i++) v[i] += v[i - samples]; }
    }
  } else if (d.predictor == 3) {   // floating point: byte differencing, then byte planes (MSB first)
    std::vector<uint8_t> tmp(row_bytes);
    const int64_t n = d.block_w * samples;
    for (int64_t r = 0; r < rows; r++) {
      uint8_t *row = out + r * row_bytes;
      for (size_t i = samples; i < row_bytes; i++) row[i] = (uint8_t)(row[i] + row[i - samples]);
      for (int64_t i = 0; i < n; i++)
        for (int k = 0; k < bytes; k++) tmp[i * bytes + k] = row[(size_t)(bytes - 1 - k) * n + i];
      std::memcpy(row, tmp.data(), row_bytes);
    }
  }
  return true;
}

struct Layout {
  int64_t bw, bh, across, down;   // block size, blocks per row / column
  int samples;                    // samples per pixel inside a block (chunky: spp, planar: 1)
  size_t block_bytes;             // staged block: bw x bh of ONE sample
};

Layout layout_of(const Ifd &d) {
  Layout L;
  L.bw = d.block_w; L.bh = d.block_h;
  L.across = (d.width + L.bw - 1) / L.bw;
  L.down = (d.height + L.bh - 1) / L.bh;
  L.samples = d.planar == 2 ? 1 : d.spp;
  L.block_bytes = (size_t)L.bw * L.bh * (d.bits / 8);
  return L;
}

// Decode every block of band `band` (0-based sample) into `stage`
// (block-major, each block bw x bh of one sample); host threads.
bool decode_band(const Tiff &t, const Ifd &d, int band, uint8_t *stage) {
  const Layout L = layout_of(d);
  const int64_t nblk = L.across * L.down;
  const int64_t plane0 = d.planar == 2 ? (int64_t)band * nblk : 0;
  if ((int64_t)d.offsets.size() < plane0 + nblk) return false;
  const int bytes = d.bits / 8;
  std::atomic<int64_t> next(0);
  std::atomic<bool> ok(true);
  const unsigned nth = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  auto work = [&]() {
   try {   // an exception may not leave a std::thread (std::terminate)
    std::vector<uint8_t> blk((size_t)L.bw * L.bh * L.samples * bytes);
    for (int64_t i = next++; i < nblk && ok; i = next++) {
      // strips: the last one holds only the image's remaining rows
      const int64_t rows = d.tiled ? L.bh : std::min<int64_t>(L.bh, d.height - (i / L.across) * L.bh);
      if (!decode_block(t, d, (size_t)(plane0 + i), rows, L.samples, blk.data())) { ok = false; break; }
      uint8_t *dst = stage + (size_t)i * L.block_bytes;
      if (L.samples == 1) {
        std::memcpy(dst, blk.data(), (size_t)L.bw * rows * bytes);
      } else {
        for (int64_t k = 0; k < L.bw * rows; k++)
          std::memcpy(dst + k * bytes, blk.data() + ((size_t)k * L.samples + band) * bytes, bytes);
      }
    }
   } catch (...) {
    ok = false;
   }
  };
  std::vector<std::thread> th;
  for (unsigned k = 1; k < std::min<unsigned>(nth, (unsigned)std::max<int64_t>(1, nblk)); k++) th.emplace_back(work);
  work();
  for (auto &x : th) x.join();
  return ok;
}

// Output element (x, y) <- staged block (y / bh) * across + x / bw.
template <typename W>
__global__ __launch_bounds__(256) void assemble_kernel(const W *__restrict__ stage, W *__restrict__ out, int64_t width,
                                                       int64_t height, int64_t bw, int64_t bh, int64_t across) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= width * height) return;
  const int64_t y = i / width, x = i - y * width;
  const int64_t by = y / bh, bx = x / bw;
  out[i] = stage[((by * across + bx) * bh + (y - by * bh)) * bw + (x - bx * bw)];
}

void assemble_host(const uint8_t *stage, uint8_t *out, const Ifd &d) {
  const Layout L = layout_of(d);
  const int bytes = d.bits / 8;
  for (int64_t y = 0; y < d.height; y++) {
    const int64_t by = y / L.bh;
    for (int64_t bx = 0; bx < L.across; bx++) {
      const int64_t x0 = bx * L.bw, n = std::min(L.bw, d.width - x0);
      std::memcpy(out + ((size_t)y * d.width + x0) * bytes,
                  stage + (((size_t)(by * L.across + bx) * L.bh + (y - by * L.bh)) * L.bw) * bytes, (size_t)n * bytes);
    }
  }
}

// GeoKey value (SHORT, inline) or 0.
int geokey(const Ifd &d, int key) {
  const auto &g = d.geokeys;
  if (g.size() < 4) return 0;
  const int n = g[3];
  for (int i = 0; i < n && 4 + 4 * i + 3 < (int)g.size(); i++)
    if (g[4 + 4 * i] == key && g[4 + 4 * i + 1] == 0) return g[4 + 4 * i + 3];
  return 0;
}

double geodouble(const Ifd &d, int key, double dflt) {
  const auto &g = d.geokeys;
  if (g.size() < 4) return dflt;
  const int n = g[3];
  for (int i = 0; i < n && 4 + 4 * i + 3 < (int)g.size(); i++)
    if (g[4 + 4 * i] == key && g[4 + 4 * i + 1] == 34736 && g[4 + 4 * i + 3] < (int)d.geodoubles.size())
      return d.geodoubles[g[4 + 4 * i + 3]];
  return dflt;
}

// Full-resolution IFD and its reduced-resolution ones (NewSubfileType bit 0).
void levels(const Tiff &t, std::vector<int> &out) {
  out.clear();
  int base = -1;
  for (int i = 0; i < (int)t.ifds.size(); i++)
    if (!(t.ifds[i].subfile & 1)) { base = i; break; }
  if (base < 0) return;
  out.push_back(base);
  for (int i = 0; i < (int)t.ifds.size(); i++)
    if (i != base && (t.ifds[i].subfile & 1) && t.ifds[i].spp == t.ifds[base].spp &&
        t.ifds[i].bits == t.ifds[base].bits && (int)out.size() <= GSKYHIP_MAX_OVR)
      out.push_back(i);
}

int fill_info(const Tiff &t, gskyhip_raster_info *info) {
  std::vector<int> lv;
  levels(t, lv);
  if (lv.empty()) return GSKYHIP_E_ARG;
  const Ifd &d = t.ifds[lv[0]];
  std::memset(info, 0, sizeof(*info));
  int sb = 0;
  info->dtype = dtype_of(d, sb);
  if (!info->dtype) return GSKYHIP_E_TYPE;
  info->signed_byte = sb;
  info->xsize = (int32_t)d.width; info->ysize = (int32_t)d.height; info->n_bands = d.spp;
  info->block_x = (int32_t)d.block_w; info->block_y = (int32_t)d.block_h;
  info->compression = d.compression; info->predictor = d.predictor; info->planar = d.planar;
  double *g = info->geot;
  g[0] = 0; g[1] = 1; g[2] = 0; g[3] = 0; g[4] = 0; g[5] = 1;   // GDAL's default geotransform
  if (d.transform.size() >= 16) {
    const auto &m = d.transform;
    g[0] = m[3]; g[1] = m[0]; g[2] = m[1]; g[3] = m[7]; g[4] = m[4]; g[5] = m[5];
  } else if (d.scale.size() >= 2 && d.tiepoint.size() >= 6) {
    const auto &tp = d.tiepoint;
    g[1] = d.scale[0]; g[5] = -d.scale[1];
    g[0] = tp[3] - tp[0] * g[1];
    g[3] = tp[4] - tp[1] * g[5];
    if (geokey(d, 1025) == 2) { g[0] -= 0.5 * g[1]; g[3] -= 0.5 * g[5]; }   // RasterPixelIsPoint
  }
  int epsg = geokey(d, 3072);
  if (!epsg || epsg == 32767) {
    if (geokey(d, 3075) == 24 &&
        std::fabs(geodouble(d, 2057, geodouble(d, 2058, 0.0)) - 6371007.181) < 1e-3)   // CT_Sinusoidal, MODIS sphere
      epsg = -1;
    else if (!epsg)
      epsg = geokey(d, 2048);
  }
  info->epsg = epsg == 32767 ? 0 : epsg;
  info->has_nodata = 0;
  info->nodata = -1e10;   // GDALGetRasterNoDataValue when unset (warp.go:246)
  if (!d.nodata.empty()) {
    std::string s(d.nodata.c_str());
    char *end = nullptr;
    const double v = std::strtod(s.c_str(), &end);
    if (end != s.c_str()) { info->nodata = v; info->has_nodata = 1; }
  }
  info->n_ovr = (int32_t)lv.size() - 1;
  for (int k = 1; k < (int)lv.size(); k++) {
    info->ovr_xsize[k - 1] = (int32_t)t.ifds[lv[k]].width;
    info->ovr_ysize[k - 1] = (int32_t)t.ifds[lv[k]].height;
  }
  return 0;
}

int open_level(const char *path, int band, int level, Tiff &t, const Ifd *&d) {
  if (!path) return GSKYHIP_E_ARG;
  if (!read_file(path, t.buf)) return 1;   // the reference's "open failed" (warp.go:103-110)
  if (!parse(t)) return GSKYHIP_E_TYPE;
  std::vector<int> lv;
  levels(t, lv);
  if (lv.empty() || level < 0 || level >= (int)lv.size()) return GSKYHIP_E_RANGE;
  d = &t.ifds[lv[level]];
  if (band < 1 || band > d->spp) return 2;   // band failed (warp.go:111-118)
  int sb;
  if (!dtype_of(*d, sb) || (d->bits % 8) != 0) return GSKYHIP_E_TYPE;
  return 0;
}

}  // namespace
}  // namespace gsky

using namespace gsky;

static int geotiff_info_impl(const char *path, gskyhip_raster_info *info) {
  if (!path || !info) return GSKYHIP_E_ARG;
  Tiff t;
  if (!read_file(path, t.buf)) return 1;
  if (!parse(t)) return GSKYHIP_E_TYPE;
  return fill_info(t, info);
}

extern "C" int gskyhip_geotiff_info(const char *path, gskyhip_raster_info *info) {
  try {
    return geotiff_info_impl(path, info);
  } catch (...) {   // a malformed file (bad_alloc of a size it declares): never through the C ABI
    return GSKYHIP_E_TYPE;
  }
}

static int geotiff_read_host_impl(const char *path, int band, int level, void *out, int64_t out_bytes) {
  Tiff t;
  const Ifd *d = nullptr;
  int rc = open_level(path, band, level, t, d);
  if (rc) return rc;
  const int64_t need = d->width * d->height * (d->bits / 8);
  if (!out || out_bytes < need) return GSKYHIP_E_ARG;
  const Layout L = layout_of(*d);
  std::vector<uint8_t> stage((size_t)(L.across * L.down) * L.block_bytes);
  if (!decode_band(t, *d, band - 1, stage.data())) return GSKYHIP_E_TYPE;
  assemble_host(stage.data(), (uint8_t *)out, *d);
  return 0;
}

extern "C" int gskyhip_geotiff_read_host(const char *path, int band, int level, void *out, int64_t out_bytes) {
  try {
    return geotiff_read_host_impl(path, band, level, out, out_bytes);
  } catch (...) {   // a malformed file (bad_alloc of a size it declares): never through the C ABI
    return GSKYHIP_E_TYPE;
  }
}

static int geotiff_read_impl(const char *path, int band, int level, void *dev_out, int64_t out_bytes,
                                    void *stream) {
  Tiff t;
  const Ifd *d = nullptr;
  int rc = open_level(path, band, level, t, d);
  if (rc) return rc;
  const int bytes = d->bits / 8;
  const int64_t n = d->width * d->height;
  if (!dev_out || out_bytes < n * bytes) return GSKYHIP_E_ARG;
  const Layout L = layout_of(*d);
  const size_t stage_bytes = (size_t)(L.across * L.down) * L.block_bytes;
  void *host = nullptr, *dev = nullptr;
  if (hipHostMalloc(&host, stage_bytes, hipHostMallocDefault) != hipSuccess) return GSKYHIP_E_HIP;
  if (!decode_band(t, *d, band - 1, (uint8_t *)host)) { hipHostFree(host); return GSKYHIP_E_TYPE; }
  hipStream_t s = (hipStream_t)stream;
  rc = 0;
  if (hipMallocAsync(&dev, stage_bytes, s) != hipSuccess) rc = GSKYHIP_E_HIP;
  if (!rc && hipMemcpyAsync(dev, host, stage_bytes, hipMemcpyHostToDevice, s) != hipSuccess) rc = GSKYHIP_E_HIP;
  if (!rc) {
    const dim3 grid((unsigned)((n + 255) / 256)), blk(256);
    switch (bytes) {
      case 1: hipLaunchKernelGGL(assemble_kernel<uint8_t>, grid, blk, 0, s, (const uint8_t *)dev, (uint8_t *)dev_out, d->width, d->height, L.bw, L.bh, L.across); break;
      case 2: hipLaunchKernelGGL(assemble_kernel<uint16_t>, grid, blk, 0, s, (const uint16_t *)dev, (uint16_t *)dev_out, d->width, d->height, L.bw, L.bh, L.across); break;
      case 4: hipLaunchKernelGGL(assemble_kernel<uint32_t>, grid, blk, 0, s, (const uint32_t *)dev, (uint32_t *)dev_out, d->width, d->height, L.bw, L.bh, L.across); break;
      default: hipLaunchKernelGGL(assemble_kernel<uint64_t>, grid, blk, 0, s, (const uint64_t *)dev, (uint64_t *)dev_out, d->width, d->height, L.bw, L.bh, L.across); break;
    }
    if (hipGetLastError() != hipSuccess) rc = GSKYHIP_E_HIP;
  }
  if (dev) hipFreeAsync(dev, s);
  // the pinned staging buffer is released once the copy has completed
  if (hipStreamSynchronize(s) != hipSuccess && !rc) rc = GSKYHIP_E_HIP;
  hipHostFree(host);
  return rc;
}

extern "C" int gskyhip_geotiff_read(const char *path, int band, int level, void *dev_out, int64_t out_bytes,
                                    void *stream) {
  try {
    return geotiff_read_impl(path, band, level, dev_out, out_bytes, stream);
  } catch (...) {   // a malformed file (bad_alloc of a size it declares): never through the C ABI
    return GSKYHIP_E_TYPE;
  }
}

// ======================================================================== netCDF classic
namespace gsky {
namespace {

struct NcAtt { std::string name; int type = 0; std::vector<double> num; std::string text; };
struct NcVar {
  std::string name;
  std::vector<int> dims;
  std::vector<NcAtt> atts;
  int type = 0;
  uint64_t vsize = 0, begin = 0;
  bool record = false;
  int h5v = -1;          // netCDF-4: the HDF5 dataset (Nc::h5.vars index)
};
struct Nc {
  std::vector<uint8_t> buf;
  int version = 1;       // 1, 2, 5: classic; 4: netCDF-4 (HDF5)
  h5::File h5;
  uint64_t numrecs = 0, recsize = 0;
  std::vector<std::pair<std::string, uint64_t>> dims;
  int rec_dim = -1;
  std::vector<NcAtt> gatts;
  std::vector<NcVar> vars;
};

int nc_type_size(int t) {
  switch (t) {
    case 1: case 2: case 7: return 1;   // byte, char, ubyte
    case 3: case 8: return 2;           // short, ushort
    case 4: case 5: case 9: return 4;   // int, float, uint
    case 6: case 10: case 11: return 8; // double, int64, uint64
    default: return 0;
  }
}

struct NcCursor {
  const std::vector<uint8_t> &b;
  size_t p;
  bool ok = true;
  uint32_t u32() {
    if (p + 4 > b.size()) { ok = false; return 0; }
    const uint32_t v = ((uint32_t)b[p] << 24) | ((uint32_t)b[p + 1] << 16) | ((uint32_t)b[p + 2] << 8) | b[p + 3];
    p += 4;
    return v;
  }
  uint64_t u64() { const uint64_t hi = u32(); return (hi << 32) | u32(); }
  std::string name(int ver) {
    const uint64_t n = ver == 5 ? u64() : u32();
    if (!ok || p + n > b.size()) { ok = false; return ""; }
    std::string s((const char *)&b[p], (size_t)n);
    p += (n + 3) & ~(uint64_t)3;
    return s;
  }
};

double nc_value(const uint8_t *q, int type) {
  uint64_t v = 0;
  const int n = nc_type_size(type);
  for (int k = 0; k < n; k++) v = (v << 8) | q[k];
  switch (type) {
    case 1: return (double)(int8_t)v;
    case 7: return (double)(uint8_t)v;
    case 3: return (double)(int16_t)v;
    case 8: return (double)(uint16_t)v;
    case 4: return (double)(int32_t)v;
    case 9: return (double)(uint32_t)v;
    case 10: return (double)(int64_t)v;
    case 11: return (double)v;
    case 5: { uint32_t u = (uint32_t)v; float f; std::memcpy(&f, &u, 4); return f; }
    case 6: { double d; std::memcpy(&d, &v, 8); return d; }
    default: return 0.0;
  }
}

bool nc_atts(NcCursor &c, int ver, std::vector<NcAtt> &out) {
  const uint32_t tag = c.u32();
  const uint64_t n = ver == 5 ? c.u64() : c.u32();
  if (tag == 0 && n == 0) return c.ok;
  if (tag != 0x0C) return false;
  for (uint64_t i = 0; i < n && c.ok; i++) {
    NcAtt a;
    a.name = c.name(ver);
    a.type = (int)c.u32();
    const uint64_t cnt = ver == 5 ? c.u64() : c.u32();
    const int ts = nc_type_size(a.type);
    if (!ts || c.p + cnt * ts > c.b.size()) return false;
    if (a.type == 2) a.text.assign((const char *)&c.b[c.p], (size_t)cnt);
    else for (uint64_t k = 0; k < cnt; k++) a.num.push_back(nc_value(&c.b[c.p + k * ts], a.type));
    c.p += (cnt * ts + 3) & ~(uint64_t)3;
    out.push_back(std::move(a));
  }
  return c.ok;
}

// netCDF-4: the HDF5 datasets of the root group as netCDF-C presents them
// (nc4hdf.c / nc4file.c of netCDF-C 4.x [ext]): dimension scales are the
// dimensions (ordered by _Netcdf4Dimid when every scale has one), a
// variable's dimensions are its DIMENSION_LIST references, a dimension
// without a coordinate variable is not a variable, the bookkeeping
// attributes are hidden.
bool nc_from_h5(Nc &f) {
  f.h5.buf.swap(f.buf);
  if (!h5::open(f.h5)) return false;
  f.version = 4;
  const auto &hv = f.h5.vars;
  std::vector<int> scales;
  for (int i = 0; i < (int)hv.size(); i++)
    if (hv[i].is_scale && hv[i].shape.size() == 1) scales.push_back(i);
  auto dimid = [&](int i) {
    for (const h5::Att &a : hv[i].atts)
      if (a.name == "_Netcdf4Dimid" && !a.num.empty()) return (int)a.num[0];
    return -1;
  };
  bool all_ids = !scales.empty();
  for (int i : scales) all_ids = all_ids && dimid(i) >= 0;
  if (all_ids) std::stable_sort(scales.begin(), scales.end(), [&](int a, int b) { return dimid(a) < dimid(b); });
  std::map<uint64_t, int> by_ohdr;
  for (int i : scales) {
    by_ohdr[hv[i].ohdr] = (int)f.dims.size();
    f.dims.emplace_back(hv[i].name, hv[i].shape[0]);
  }
  auto hidden = [](const std::string &n) {
    return n == "DIMENSION_LIST" || n == "REFERENCE_LIST" || n == "CLASS" || n == "NAME" || n == "_Netcdf4Dimid" ||
           n == "_Netcdf4Coordinates" || n == "_nc3_strict" || n == "_NCProperties" || n == "_IsNetcdf4";
  };
  auto conv = [&](const std::vector<h5::Att> &in, std::vector<NcAtt> &out) {
    for (const h5::Att &a : in) {
      if (hidden(a.name) || a.nctype == 0) continue;
      NcAtt n;
      n.name = a.name;
      n.type = a.nctype;
      n.num = a.num;
      n.text = a.text;
      out.push_back(std::move(n));
    }
  };
  conv(f.h5.gatts, f.gatts);
  for (int i = 0; i < (int)hv.size(); i++) {
    const h5::Var &h = hv[i];
    if (h.pure_dim || h.nctype == 0) continue;
    NcVar v;
    v.name = h.name;
    v.type = h.nctype;
    v.h5v = i;
    if (!h.dim_refs.empty()) {
      if (h.dim_refs.size() != h.shape.size()) return false;
      for (uint64_t ref : h.dim_refs) {
        auto it = by_ohdr.find(ref);
        if (it == by_ohdr.end()) return false;
        v.dims.push_back(it->second);
      }
    } else if (h.is_scale) {
      v.dims.push_back(by_ohdr[h.ohdr]);
    } else {   // anonymous dimensions (a plain HDF5 dataset): phony_dim_k as netCDF-C names them
      for (uint64_t n : h.shape) {
        v.dims.push_back((int)f.dims.size());
        f.dims.emplace_back("phony_dim_" + std::to_string(f.dims.size()), n);
      }
    }
    for (size_t k = 0; k < v.dims.size(); k++)
      if (f.dims[v.dims[k]].second != h.shape[k]) return false;
    conv(h.atts, v.atts);
    f.vars.push_back(std::move(v));
  }
  return true;
}

bool nc_parse(Nc &f) {
  if (h5::is_hdf5(f.buf)) return nc_from_h5(f);
  const std::vector<uint8_t> &b = f.buf;
  if (b.size() < 8 || b[0] != 'C' || b[1] != 'D' || b[2] != 'F') return false;
  f.version = b[3];
  if (f.version != 1 && f.version != 2 && f.version != 5) return false;
  NcCursor c{b, 4};
  const int ver = f.version;
  f.numrecs = ver == 5 ? c.u64() : c.u32();
  uint32_t tag = c.u32();
  uint64_t n = ver == 5 ? c.u64() : c.u32();
  if (tag == 0x0A) {
    if (n > b.size()) return false;
    for (uint64_t i = 0; i < n && c.ok; i++) {
      std::string nm = c.name(ver);
      const uint64_t len = ver == 5 ? c.u64() : c.u32();
      if (len == 0) f.rec_dim = (int)i;
      f.dims.emplace_back(nm, len);
    }
  } else if (tag != 0 || n != 0) {
    return false;
  }
  if (!nc_atts(c, ver, f.gatts)) return false;
  tag = c.u32();
  n = ver == 5 ? c.u64() : c.u32();
  if (tag != 0x0B && !(tag == 0 && n == 0)) return false;
  if (n > b.size()) return false;
  for (uint64_t i = 0; i < n && c.ok; i++) {
    NcVar v;
    v.name = c.name(ver);
    const uint64_t nd = ver == 5 ? c.u64() : c.u32();
    if (nd > 64) return false;   // a corrupt count: NC_MAX_VAR_DIMS is 1024, a raster has <= 3
    for (uint64_t k = 0; k < nd && c.ok; k++) v.dims.push_back((int)(ver == 5 ? c.u64() : c.u32()));
    if (!nc_atts(c, ver, v.atts)) return false;
    v.type = (int)c.u32();
    v.vsize = ver == 5 ? c.u64() : c.u32();
    v.begin = ver == 1 ? c.u32() : c.u64();
    for (int d : v.dims) if (d < 0 || d >= (int)f.dims.size()) return false;
    v.record = !v.dims.empty() && v.dims[0] == f.rec_dim;
    f.vars.push_back(std::move(v));
  }
  if (!c.ok) return false;
  int nrec = 0;
  for (const NcVar &v : f.vars) if (v.record) { f.recsize += v.vsize; nrec++; }
  if (nrec == 1) {   // one record variable: records are not padded to 4 bytes
    for (const NcVar &v : f.vars)
      if (v.record) {
        uint64_t e = nc_type_size(v.type);
        for (size_t k = 1; k < v.dims.size(); k++) e *= f.dims[v.dims[k]].second;
        f.recsize = e;
      }
  }
  return true;
}

const NcAtt *nc_att(const std::vector<NcAtt> &atts, const char *name) {
  for (const NcAtt &a : atts) if (a.name == name) return &a;
  return nullptr;
}

// Element i of a non-record variable as a double (coordinate values).
bool nc_elem(const Nc &f, const NcVar &v, uint64_t i, double &out) {
  const int ts = nc_type_size(v.type);
  if (!ts) return false;
  if (v.h5v >= 0) {
    const h5::Var &h = f.h5.vars[v.h5v];
    uint8_t e[8];
    if (!h5::read(f.h5, h, i, 1, e)) return false;
    uint8_t be[8];
    for (int k = 0; k < ts; k++) be[k] = h.big_endian ? e[k] : e[ts - 1 - k];   // nc_value reads big-endian
    out = nc_value(be, v.type);
    return true;
  }
  if (v.record || v.begin + (i + 1) * ts > f.buf.size()) return false;
  out = nc_value(&f.buf[v.begin + i * ts], v.type);
  return true;
}

// "NETCDF:file:var" / "NETCDF:\"file\":var" / "file" -> file, var
void nc_split(const char *path, std::string &file, std::string &var) {
  std::string p(path);
  var.clear();
  if (p.compare(0, 7, "NETCDF:") == 0) {
    p = p.substr(7);
    if (!p.empty() && p[0] == '"') {
      const size_t q = p.find('"', 1);
      file = p.substr(1, q == std::string::npos ? std::string::npos : q - 1);
      if (q != std::string::npos && q + 2 <= p.size()) var = p.substr(q + 2);
      return;
    }
    const size_t k = p.rfind(':');
    if (k != std::string::npos) { file = p.substr(0, k); var = p.substr(k + 1); return; }
  }
  file = p;
}

struct NcRaster {
  Nc f;
  const NcVar *v = nullptr;
  int64_t nx = 0, ny = 0, nb = 1;
  bool bottom_up = false;
};

int nc_open_raster(const char *path, NcRaster &r) {
  std::string file, var;
  nc_split(path, file, var);
  if (!read_file(file.c_str(), r.f.buf)) return 1;
  if (!nc_parse(r.f)) return GSKYHIP_E_TYPE;
  auto is_coord = [&](const NcVar &v) { return v.dims.size() == 1 && r.f.dims[v.dims[0]].first == v.name; };
  const NcVar *pick = nullptr;
  int n_data = 0;
  for (const NcVar &v : r.f.vars) {
    if (!var.empty()) { if (v.name == var) pick = &v; continue; }
    if (v.dims.size() >= 2 && !is_coord(v)) { n_data++; if (!pick) pick = &v; }
  }
  if (!pick || (var.empty() && n_data != 1)) return 1;   // no such variable / subdatasets only
  if (pick->dims.size() < 2 || pick->dims.size() > 3 || !nc_type_size(pick->type)) return GSKYHIP_E_TYPE;
  r.v = pick;
  const auto dimlen = [&](int d) { return d == r.f.rec_dim ? (int64_t)r.f.numrecs : (int64_t)r.f.dims[d].second; };
  const size_t nd = pick->dims.size();
  r.nx = dimlen(pick->dims[nd - 1]);
  r.ny = dimlen(pick->dims[nd - 2]);
  r.nb = nd == 3 ? dimlen(pick->dims[0]) : 1;
  if (r.nx <= 0 || r.ny <= 0 || r.nb <= 0) return GSKYHIP_E_ARG;
  // bBottomUp from the y coordinate variable (netcdfdataset.cpp:3271)
  const std::string &ydim = r.f.dims[pick->dims[nd - 2]].first;
  for (const NcVar &cv : r.f.vars)
    if (cv.name == ydim && cv.dims.size() == 1 && r.ny >= 2 && !cv.record) {
      double y0, y1;
      if (nc_elem(r.f, cv, 0, y0) && nc_elem(r.f, cv, 1, y1)) r.bottom_up = y0 <= y1;
    }
  return 0;
}

// bIsGdalFile of the driver (netcdfdataset.cpp:2498-2518): a global "GDAL"
// attribute of version >= 1.9 (NCDFIsGDALVersionGTE, 8879-8919), or
// spatial_ref + GeoTransform on the variable's grid_mapping variable.
bool nc_is_gdal_file(const Nc &f, const NcVar &v) {
  auto ieq_prefix = [](const std::string &s, const char *p) {
    size_t n = std::strlen(p);
    if (s.size() < n) return false;
    for (size_t i = 0; i < n; i++) if (std::tolower((unsigned char)s[i]) != std::tolower((unsigned char)p[i])) return false;
    return true;
  };
  if (const NcAtt *g = nc_att(f.gatts, "GDAL")) {
    const std::string ver(g->text.c_str());
    if (ieq_prefix(ver, "GDAL ")) {
      int vn = 0;
      if (ieq_prefix(ver, "GDAL 2.0dev, released 2011/12/29") && ver.size() == 32) vn = 1100000;
      else if (ieq_prefix(ver, "GDAL 1.9dev")) vn = 1900;
      else if (ieq_prefix(ver, "GDAL 1.8dev")) vn = 1800;
      else {
        int t[4] = {0, 0, 0, 0};
        const char *c = ver.c_str() + 5;
        for (int k = 0; k < 4 && *c; k++) {   // CSLTokenizeString2(".", 0) + atoi, clamped to [0, 99]
          t[k] = std::max(0, std::min(99, std::atoi(c)));
          const char *d = std::strchr(c, '.');
          if (!d) break;
          c = d + 1;
        }
        vn = (t[0] > 1 || t[1] >= 10) ? t[0] * 1000000 + t[1] * 10000 + t[2] * 100
                                      : t[0] * 1000 + t[1] * 100 + t[2] * 10 + t[3];
      }
      if (1900 <= vn) return true;
    }
  }
  if (const NcAtt *gm = nc_att(v.atts, "grid_mapping"))
    for (const NcVar &m : f.vars)
      if (m.name == std::string(gm->text.c_str()) && nc_att(m.atts, "spatial_ref") && nc_att(m.atts, "GeoTransform"))
        return true;
  return false;
}

// Data type, signedness and nodata of a variable as netCDFRasterBand sets
// them (netcdfdataset.cpp:386-559): nodata from _FillValue, else
// missing_value, else NCDFGetDefaultNoDataValue (10182-10225) -- always set;
// NC_BYTE is PIXELTYPE=SIGNEDBYTE unless the file was written by GDAL,
// valid_range {0,255} / {-128,127} decides when present, else _Unsigned; an
// unsigned byte's negative nodata gets +256.
int nc_dtype(const Nc &f, const NcVar &v, int &signed_byte, double &nodata) {
  signed_byte = 0;
  const NcAtt *fv = nc_att(v.atts, "_FillValue");
  if (!fv) fv = nc_att(v.atts, "missing_value");
  if (fv && !fv->num.empty()) {
    nodata = fv->num[0];
  } else {
    switch (v.type) {
      case 3: nodata = -32767.0; break;                  // NC_FILL_SHORT
      case 4: nodata = -2147483647.0; break;             // NC_FILL_INT
      case 5: nodata = (double)9.9692099683868690e+36f; break;   // NC_FILL_FLOAT
      case 6: nodata = 9.9692099683868690e+36; break;    // NC_FILL_DOUBLE
      case 8: nodata = 65535.0; break;                   // NC_FILL_USHORT
      case 9: nodata = 4294967295.0; break;              // NC_FILL_UINT
      default: nodata = 0.0; break;                      // bytes, chars
    }
  }
  switch (v.type) {
    case 1: {   // NC_BYTE
      bool sgn = !nc_is_gdal_file(f, v);
      if (!sgn && nodata < 0) nodata += 256;
      const NcAtt *vr = nc_att(v.atts, "valid_range");
      if (vr && vr->num.size() == 2) {   // HONOUR_VALID_RANGE defaults to true; nc_get_att_int
        const int lo = (int)vr->num[0], hi = (int)vr->num[1];
        if (lo == 0 && hi == 255) {
          sgn = false;
          if (nodata < 0) nodata += 256;
        } else if (lo == -128 && hi == 127) {
          sgn = true;
        }
      } else {
        if (const NcAtt *u = nc_att(v.atts, "_Unsigned")) {
          std::string t(u->text.c_str());
          for (auto &ch : t) ch = (char)std::tolower((unsigned char)ch);
          if (t == "true") sgn = false;
          else if (t == "false") sgn = true;
        }
        if (!sgn && nodata < 0) nodata += 256;
      }
      signed_byte = sgn ? 1 : 0;
      return GSKYHIP_BYTE;
    }
    case 7: return GSKYHIP_BYTE;
    case 3: return GSKYHIP_INT16;
    case 8: return GSKYHIP_UINT16;
    case 4: return GSKYHIP_INT32;
    case 9: return GSKYHIP_UINT32;
    case 5: return GSKYHIP_FLOAT32;
    case 6: return GSKYHIP_FLOAT64;
    default: return 0;
  }
}

int nc_epsg(const Nc &f, const NcVar &v) {
  const NcAtt *gm = nc_att(v.atts, "grid_mapping");
  if (gm)
    for (const NcVar &m : f.vars)
      if (m.name == std::string(gm->text.c_str()))   // text attributes may carry a NUL
        for (const char *k : {"crs_wkt", "spatial_ref"}) {
          const NcAtt *w = nc_att(m.atts, k);
          if (!w) continue;
          const size_t a = w->text.rfind("AUTHORITY[\"EPSG\",\"");
          if (a != std::string::npos) return std::atoi(w->text.c_str() + a + 18);
        }
  const size_t nd = v.dims.size();
  const std::string &xn = f.dims[v.dims[nd - 1]].first, &yn = f.dims[v.dims[nd - 2]].first;
  auto low = [](std::string s) { for (auto &ch : s) ch = (char)std::tolower((unsigned char)ch); return s; };
  const std::string x = low(xn), y = low(yn);
  if ((x == "lon" || x == "longitude" || x == "x") && (y == "lat" || y == "latitude" || y == "y") &&
      (x != "x" || y != "y"))
    return 4326;
  return 0;
}

// The SRS of the variable's CF grid mapping (grid_mapping_name and its
// parameters, CF-1.x Appendix F, as GSKY_netCDF's SetProjectionFromVar reads
// them), as a PROJ string of the projection families the warp supports;
// "" without a grid mapping (lon / lat axes: EPSG:4326, else none -- the
// warp then takes WGS84, warp.go:107-112), "?" for a mapping it cannot
// represent.  Parity unpinned (netCDF-C / GDAL are absent).
std::string nc_cf_srs(const Nc &f, const NcVar &v) {
  auto num = [](const NcVar &m, const char *k, int i, double dflt) {
    const NcAtt *a = nc_att(m.atts, k);
    return (a && (int)a->num.size() > i) ? a->num[i] : dflt;
  };
  auto has = [](const NcVar &m, const char *k) {
    const NcAtt *a = nc_att(m.atts, k);
    return a && !a->num.empty();
  };
  if (const NcAtt *gm = nc_att(v.atts, "grid_mapping"))
    for (const NcVar &m : f.vars) {
      if (m.name != std::string(gm->text.c_str())) continue;
      const NcAtt *gn = nc_att(m.atts, "grid_mapping_name");
      if (!gn) break;
      std::string name(gn->text.c_str());
      for (auto &ch : name) ch = (char)std::tolower((unsigned char)ch);
      // the ellipsoid: earth_radius, else semi_major_axis with
      // inverse_flattening or semi_minor_axis (a sphere without either),
      // else WGS84
      char ell[96];
      bool sphere = false;
      if (has(m, "earth_radius")) {
        std::snprintf(ell, sizeof(ell), "+R=%.17g", num(m, "earth_radius", 0, 0));
        sphere = true;
      } else if (has(m, "semi_major_axis")) {
        const double a = num(m, "semi_major_axis", 0, 0);
        double rf = num(m, "inverse_flattening", 0, 0);
        if (rf == 0 && has(m, "semi_minor_axis")) {
          const double b = num(m, "semi_minor_axis", 0, a);
          rf = a != b ? a / (a - b) : 0;
        }
        if (rf > 0) std::snprintf(ell, sizeof(ell), "+a=%.17g +rf=%.17g", a, rf);
        else { std::snprintf(ell, sizeof(ell), "+R=%.17g", a); sphere = true; }
      } else {
        std::snprintf(ell, sizeof(ell), "+ellps=WGS84");
      }
      const double fe = num(m, "false_easting", 0, 0), fn = num(m, "false_northing", 0, 0);
      char buf[384];
      if (name == "latitude_longitude") {
        std::snprintf(buf, sizeof(buf), "+proj=longlat %s", ell);
        return buf;
      }
      if (name == "albers_conical_equal_area") {
        const NcAtt *sp = nc_att(m.atts, "standard_parallel");
        if (!sp || sp->num.empty()) return "?";
        const double p1 = sp->num[0], p2 = sp->num.size() > 1 ? sp->num[1] : sp->num[0];
        std::snprintf(buf, sizeof(buf), "+proj=aea +lat_1=%.17g +lat_2=%.17g +lat_0=%.17g +lon_0=%.17g +x_0=%.17g "
                      "+y_0=%.17g %s", p1, p2, num(m, "latitude_of_projection_origin", 0, 0),
                      num(m, "longitude_of_central_meridian", 0, 0), fe, fn, ell);
        return buf;
      }
      if (name == "lambert_conformal_conic" && !sphere) {   // ellipsoidal only (as the warp's lcc)
        const NcAtt *sp = nc_att(m.atts, "standard_parallel");
        if (!sp || sp->num.empty()) return "?";
        const double lat0 = num(m, "latitude_of_projection_origin", 0, 0);
        const double cm = num(m, "longitude_of_central_meridian", 0, 0);
        if (sp->num.size() > 1)
          std::snprintf(buf, sizeof(buf), "+proj=lcc +lat_1=%.17g +lat_2=%.17g +lat_0=%.17g +lon_0=%.17g +x_0=%.17g "
                        "+y_0=%.17g %s", sp->num[0], sp->num[1], lat0, cm, fe, fn, ell);
        else   // one standard parallel: the tangent cone (LCC 1SP)
          std::snprintf(buf, sizeof(buf), "+proj=lcc +lat_1=%.17g +lat_0=%.17g +lon_0=%.17g +k_0=%.17g +x_0=%.17g "
                        "+y_0=%.17g %s", sp->num[0], lat0, cm, num(m, "scale_factor_at_projection_origin", 0, 1.0),
                        fe, fn, ell);
        return buf;
      }
      if (name == "transverse_mercator" && !sphere) {   // ellipsoidal only (as the warp's tmerc)
        const double k0 = num(m, "scale_factor_at_central_meridian", 0, 1.0);
        const double cm = num(m, "longitude_of_central_meridian", 0, 0);
        const double lat0 = num(m, "latitude_of_projection_origin", 0, 0);
        // a UTM zone's parameters: +proj=utm, as PROJ 6 exports the conversion
        const double zone = (cm + 183.0) / 6.0;
        if (lat0 == 0 && k0 == 0.9996 && fe == 500000.0 && (fn == 0 || fn == 10000000.0) && zone == std::floor(zone) &&
            zone >= 1 && zone <= 60)
          std::snprintf(buf, sizeof(buf), "+proj=utm +zone=%d%s %s", (int)zone, fn != 0 ? " +south" : "", ell);
        else
          std::snprintf(buf, sizeof(buf), "+proj=tmerc +lat_0=%.17g +lon_0=%.17g +k_0=%.17g +x_0=%.17g +y_0=%.17g %s",
                        lat0, cm, k0, fe, fn, ell);
        return buf;
      }
      if (name == "polar_stereographic" && !sphere && has(m, "latitude_of_projection_origin")) {
        // polar aspects only (as the warp's stere): the pole, then the
        // true-scale parallel or the scale at the pole
        const double lat0 = num(m, "latitude_of_projection_origin", 0, 0);
        if (lat0 != 90.0 && lat0 != -90.0) return "?";
        const double cm = num(m, "straight_vertical_longitude_from_pole", 0, 0);
        if (has(m, "standard_parallel"))
          std::snprintf(buf, sizeof(buf), "+proj=stere +lat_0=%.17g +lat_ts=%.17g +lon_0=%.17g +x_0=%.17g +y_0=%.17g %s",
                        lat0, num(m, "standard_parallel", 0, lat0), cm, fe, fn, ell);
        else
          std::snprintf(buf, sizeof(buf), "+proj=stere +lat_0=%.17g +lon_0=%.17g +k_0=%.17g +x_0=%.17g +y_0=%.17g %s",
                        lat0, cm, num(m, "scale_factor_at_projection_origin", 0, 1.0), fe, fn, ell);
        return buf;
      }
      if (name == "sinusoidal" && sphere) {
        std::snprintf(buf, sizeof(buf), "+proj=sinu +lon_0=%.17g +x_0=%.17g +y_0=%.17g %s",
                      num(m, "longitude_of_central_meridian", 0, num(m, "longitude_of_projection_origin", 0, 0)),
                      fe, fn, ell);
        return buf;
      }
      return "?";
    }
  const size_t nd = v.dims.size();
  auto low = [](std::string s) { for (auto &ch : s) ch = (char)std::tolower((unsigned char)ch); return s; };
  const std::string x = low(f.dims[v.dims[nd - 1]].first), y = low(f.dims[v.dims[nd - 2]].first);
  if ((x == "lon" || x == "longitude" || x == "x") && (y == "lat" || y == "latitude" || y == "y") &&
      (x != "x" || y != "y"))
    return "EPSG:4326";
  return "";
}

// The dataset SRS for the srs_cf open option (netcdfdataset.cpp:7023-7025,
// 3661-3720): srs_cf=no -- the GDAL-written WKT (spatial_ref / crs_wkt) of
// the grid mapping wins when it names an EPSG code, else the CF mapping;
// srs_cf=yes -- the CF mapping only.
std::string nc_srs(const Nc &f, const NcVar &v, bool srs_cf) {
  if (!srs_cf)
    if (const NcAtt *gm = nc_att(v.atts, "grid_mapping"))
      for (const NcVar &m : f.vars)
        if (m.name == std::string(gm->text.c_str()))
          for (const char *k : {"crs_wkt", "spatial_ref"}) {
            const NcAtt *w = nc_att(m.atts, k);
            if (!w) continue;
            const size_t a = w->text.rfind("AUTHORITY[\"EPSG\",\"");
            if (a != std::string::npos) return "EPSG:" + std::to_string(std::atoi(w->text.c_str() + a + 18));
          }
  return nc_cf_srs(f, v);
}

int nc_fill_info(const NcRaster &r, gskyhip_raster_info *info) {
  std::memset(info, 0, sizeof(*info));
  const NcVar &v = *r.v;
  int sb = 0;
  double nodata = 0.0;
  info->dtype = nc_dtype(r.f, v, sb, nodata);
  if (!info->dtype) return GSKYHIP_E_TYPE;
  info->signed_byte = sb;
  info->xsize = (int32_t)r.nx; info->ysize = (int32_t)r.ny; info->n_bands = (int32_t)r.nb;
  info->block_x = (int32_t)r.nx; info->block_y = 1;
  info->compression = 1; info->predictor = 1; info->planar = 2;
  double *g = info->geot;
  g[0] = 0; g[1] = 1; g[2] = 0; g[3] = 0; g[4] = 0; g[5] = 1;
  const size_t nd = v.dims.size();
  const Nc &f = r.f;
  auto coord = [&](const std::string &dn, int64_t n, double mm[2]) {
    for (const NcVar &cv : f.vars)
      if (cv.name == dn && cv.dims.size() == 1 && !cv.record) {
        if (n < 2) return false;
        const NcAtt *ar = nc_att(cv.atts, "actual_range");
        if (ar && ar->num.size() >= 2) { mm[0] = ar->num[0]; mm[1] = ar->num[1]; }
        else if (!nc_elem(f, cv, 0, mm[0]) || !nc_elem(f, cv, (uint64_t)n - 1, mm[1])) return false;
        const NcAtt *ao = nc_att(cv.atts, "add_offset"), *sf = nc_att(cv.atts, "scale_factor");
        if (ao && sf && !ao->num.empty() && !sf->num.empty()) {
          mm[0] = ao->num[0] + mm[0] * sf->num[0];
          mm[1] = ao->num[0] + mm[1] * sf->num[0];
        }
        return true;
      }
    return false;
  };
  double xm[2], ym[2];
  if (coord(f.dims[v.dims[nd - 1]].first, r.nx, xm) && coord(f.dims[v.dims[nd - 2]].first, r.ny, ym)) {
    int node_offset = 0;
    const NcAtt *no = nc_att(f.gatts, "node_offset");
    if (no && !no->num.empty()) node_offset = (int)no->num[0];
    if (ym[0] > ym[1]) std::swap(ym[0], ym[1]);   // netcdfdataset.cpp:3549-3555
    g[0] = xm[0];
    g[1] = (xm[1] - xm[0]) / (r.nx + (node_offset - 1));
    g[3] = ym[1];
    g[5] = (ym[0] - ym[1]) / (r.ny + (node_offset - 1));
    if (!node_offset) { g[0] -= g[1] / 2; g[3] -= g[5] / 2; }
  }
  info->epsg = nc_epsg(f, v);
  info->nodata = nodata;   // netCDFRasterBand::SetNoDataValue, always (netcdfdataset.cpp:558)
  info->has_nodata = 1;
  return 0;
}

// Byte offset of row y (file order) of band b.
uint64_t nc_row_offset(const NcRaster &r, int64_t b, int64_t y) {
  const int ts = nc_type_size(r.v->type);
  const uint64_t row = (uint64_t)r.nx * ts;
  if (r.v->record) return r.v->begin + (uint64_t)b * r.f.recsize + (uint64_t)y * row;
  return r.v->begin + ((uint64_t)b * r.ny + y) * row;
}

// Band rows into host `out` (big-endian file order -> host order; rows
// south-up when the y axis increases).
bool nc_read_rows(const NcRaster &r, int64_t b, uint8_t *out, bool swap) {
  const int ts = nc_type_size(r.v->type);
  const uint64_t row = (uint64_t)r.nx * ts;
  if (r.v->h5v >= 0) {   // netCDF-4: the band's plane from its chunks (file byte order)
    const h5::Var &h = r.f.h5.vars[r.v->h5v];
    const uint64_t plane = (uint64_t)r.nx * r.ny;
    if (!h5::read(r.f.h5, h, (uint64_t)b * plane, plane, out)) return false;
    if (r.bottom_up) {
      std::vector<uint8_t> tmp(row);
      for (int64_t y = 0; y < r.ny / 2; y++) {
        uint8_t *a = out + (uint64_t)y * row, *c = out + (uint64_t)(r.ny - 1 - y) * row;
        std::memcpy(tmp.data(), a, row);
        std::memcpy(a, c, row);
        std::memcpy(c, tmp.data(), row);
      }
    }
    if (swap && h.big_endian && ts > 1)
      for (uint64_t i = 0; i < plane * ts; i += ts) std::reverse(out + i, out + i + ts);
    return true;
  }
  for (int64_t y = 0; y < r.ny; y++) {
    const uint64_t o = nc_row_offset(r, b, r.bottom_up ? r.ny - 1 - y : y);
    if (o + row > r.f.buf.size()) return false;
    uint8_t *d = out + (uint64_t)y * row;
    std::memcpy(d, &r.f.buf[o], row);
    if (swap && ts > 1)
      for (uint64_t i = 0; i < row; i += ts) std::reverse(d + i, d + i + ts);
  }
  return true;
}

template <typename W>
__global__ __launch_bounds__(256) void byteswap_kernel(W *__restrict__ v, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  W x = v[i], y = 0;
#pragma unroll
  for (int k = 0; k < (int)sizeof(W); k++) y = (W)((y << 8) | ((x >> (8 * k)) & 0xFF));
  v[i] = y;
}

}  // namespace
}  // namespace gsky

static int netcdf_info_impl(const char *path, gskyhip_raster_info *info) {
  if (!path || !info) return GSKYHIP_E_ARG;
  NcRaster r;
  const int rc = nc_open_raster(path, r);
  return rc ? rc : nc_fill_info(r, info);
}

extern "C" int gskyhip_netcdf_info(const char *path, gskyhip_raster_info *info) {
  try {
    return netcdf_info_impl(path, info);
  } catch (...) {   // a malformed file (bad_alloc of a size it declares): never through the C ABI
    return GSKYHIP_E_TYPE;
  }
}

static int netcdf_read_host_impl(const char *path, int band, void *out, int64_t out_bytes) {
  NcRaster r;
  int rc = nc_open_raster(path, r);
  if (rc) return rc;
  if (band < 1 || band > r.nb) return 2;
  const int64_t need = r.nx * r.ny * nc_type_size(r.v->type);
  if (!out || out_bytes < need) return GSKYHIP_E_ARG;
  return nc_read_rows(r, band - 1, (uint8_t *)out, true) ? 0 : GSKYHIP_E_ARG;
}

namespace gsky {
int netcdf_info_srs(const char *path, gskyhip_raster_info *info, std::string *srs_no, std::string *srs_cf) {
  try {
    if (!path || !info) return GSKYHIP_E_ARG;
    NcRaster r;
    int rc = nc_open_raster(path, r);
    if (!rc) rc = nc_fill_info(r, info);
    if (rc) return rc;
    if (srs_no) *srs_no = nc_srs(r.f, *r.v, false);
    if (srs_cf) *srs_cf = nc_srs(r.f, *r.v, true);
    return 0;
  } catch (...) {
    return GSKYHIP_E_TYPE;
  }
}
}  // namespace gsky

static int netcdf_srs_impl(const char *path, int srs_cf, char *out, int cap) {
  if (!path || !out || cap <= 0) return GSKYHIP_E_ARG;
  NcRaster r;
  const int rc = nc_open_raster(path, r);
  if (rc) return rc;
  const std::string srs = nc_srs(r.f, *r.v, srs_cf > 0);
  if ((int)srs.size() >= cap) return GSKYHIP_E_ARG;
  std::memcpy(out, srs.c_str(), srs.size() + 1);
  return 0;
}

extern "C" int gskyhip_netcdf_srs(const char *path, int srs_cf, char *out, int cap) {
  try {
    return netcdf_srs_impl(path, srs_cf, out, cap);
  } catch (...) {
    return GSKYHIP_E_TYPE;
  }
}

extern "C" int gskyhip_netcdf_read_host(const char *path, int band, void *out, int64_t out_bytes) {
  try {
    return netcdf_read_host_impl(path, band, out, out_bytes);
  } catch (...) {   // a malformed file (bad_alloc of a size it declares): never through the C ABI
    return GSKYHIP_E_TYPE;
  }
}

static int netcdf_read_impl(const char *path, int band, void *dev_out, int64_t out_bytes, void *stream) {
  NcRaster r;
  int rc = nc_open_raster(path, r);
  if (rc) return rc;
  if (band < 1 || band > r.nb) return 2;
  const int ts = nc_type_size(r.v->type);
  const int64_t n = r.nx * r.ny;
  if (!dev_out || out_bytes < n * ts) return GSKYHIP_E_ARG;
  void *host = nullptr;
  if (hipHostMalloc(&host, (size_t)(n * ts), hipHostMallocDefault) != hipSuccess) return GSKYHIP_E_HIP;
  if (!nc_read_rows(r, band - 1, (uint8_t *)host, false)) { hipHostFree(host); return GSKYHIP_E_ARG; }
  hipStream_t s = (hipStream_t)stream;
  rc = hipMemcpyAsync(dev_out, host, (size_t)(n * ts), hipMemcpyHostToDevice, s) == hipSuccess ? 0 : GSKYHIP_E_HIP;
  const bool file_be = r.v->h5v < 0 || r.f.h5.vars[r.v->h5v].big_endian;   // classic: always big-endian
  if (!rc && ts > 1 && file_be) {   // big-endian file order -> device order on the GPU
    const dim3 grid((unsigned)((n + 255) / 256)), blk(256);
    if (ts == 2) hipLaunchKernelGGL(byteswap_kernel<uint16_t>, grid, blk, 0, s, (uint16_t *)dev_out, n);
    else if (ts == 4) hipLaunchKernelGGL(byteswap_kernel<uint32_t>, grid, blk, 0, s, (uint32_t *)dev_out, n);
    else hipLaunchKernelGGL(byteswap_kernel<uint64_t>, grid, blk, 0, s, (uint64_t *)dev_out, n);
    if (hipGetLastError() != hipSuccess) rc = GSKYHIP_E_HIP;
  }
  if (hipStreamSynchronize(s) != hipSuccess && !rc) rc = GSKYHIP_E_HIP;
  hipHostFree(host);
  return rc;
}

extern "C" int gskyhip_netcdf_read(const char *path, int band, void *dev_out, int64_t out_bytes, void *stream) {
  try {
    return netcdf_read_impl(path, band, dev_out, out_bytes, stream);
  } catch (...) {   // a malformed file (bad_alloc of a size it declares): never through the C ABI
    return GSKYHIP_E_TYPE;
  }
}
