// hdf5.cpp -- the HDF5 / netCDF-4 subset of hdf5.h.  Host code: parsing the
// file structure is pointer chasing over a few kilobytes of metadata; the
// band's bytes go to HBM through the same path as the classic netCDF reader
// (ingest.hip).  Format structures follow the HDF5 file format specification
// version 3.0 (section numbers in the comments); parity unpinned.
#include "hdf5.h"

#include <zlib.h>

#include <algorithm>
#include <cstring>
#include <functional>
#include <map>

namespace gsky {
namespace h5 {
namespace {

constexpr uint64_t kUndef = ~(uint64_t)0;

// Little-endian field reader over the file image; every read bounds-checked
// (a truncated or corrupt file fails the open, it never reads past the end).
struct Rd {
  const File &f;
  bool ok = true;
  uint64_t u(uint64_t p, int n) {
    if (n <= 0 || n > 8 || p > f.buf.size() || f.buf.size() - p < (uint64_t)n) { ok = false; return 0; }
    uint64_t v = 0;
    for (int k = n - 1; k >= 0; k--) v = (v << 8) | f.buf[p + k];
    return v;
  }
  uint64_t addr(uint64_t p) {
    const uint64_t a = u(p, f.off_size);
    if (f.off_size < 8 && a == ((uint64_t)1 << (8 * f.off_size)) - 1) return kUndef;
    return a == kUndef ? kUndef : a + f.base;
  }
  uint64_t len(uint64_t p) { return u(p, f.len_size); }
  bool sig(uint64_t p, const char *s) {
    if (p > f.buf.size() || f.buf.size() - p < 4) { ok = false; return false; }
    return std::memcmp(&f.buf[p], s, 4) == 0;
  }
  bool has(uint64_t p, uint64_t n) { return p <= f.buf.size() && f.buf.size() - p >= n; }
};

// Nodes one tree walk may visit: a corrupt or crafted index (children that
// point back into the tree) fails the open instead of running for ever.
constexpr uint64_t kMaxNodes = 1u << 16;

int bytes_for(uint64_t x) {   // H5VM_limit_enc_size: (log2(x) / 8) + 1
  int l = 0;
  while (x >>= 1) l++;
  return l / 8 + 1;
}
int log2_of(uint64_t x) {
  int l = 0;
  while (x > 1) { x >>= 1; l++; }
  return l;
}

// ---------------------------------------------------------------- datatypes (IV.A.2.d)
struct DType {
  int cls = -1, size = 0;
  bool sign = false, be = false;
  int vlen_kind = -1;              // class 9: 0 sequence, 1 string
  std::vector<DType> base;         // class 9: the element type
  int nctype() const {
    if (cls == 0) {
      switch (size) {
        case 1: return sign ? 1 : 7;
        case 2: return sign ? 3 : 8;
        case 4: return sign ? 4 : 9;
        case 8: return sign ? 10 : 11;
      }
      return 0;
    }
    if (cls == 1) return size == 4 ? 5 : size == 8 ? 6 : 0;
    if (cls == 3 || (cls == 9 && vlen_kind == 1)) return 2;
    return 0;
  }
};

bool parse_dtype(Rd &r, uint64_t p, uint64_t end, DType &t) {
  if (!r.has(p, 8) || p + 8 > end) return false;
  const uint8_t b0 = (uint8_t)r.u(p, 1);
  t.cls = b0 & 0x0F;
  const uint32_t bf = (uint32_t)r.u(p + 1, 3);
  t.size = (int)r.u(p + 4, 4);
  switch (t.cls) {
    case 0: t.be = bf & 1; t.sign = (bf >> 3) & 1; return r.ok;
    case 1: t.be = bf & 1; t.sign = true; return r.ok;
    case 3: return r.ok;
    case 7: return r.ok;   // reference: bf & 0xF == 0 object (an address)
    case 9: {
      t.vlen_kind = bf & 0x0F;
      DType b;
      if (!parse_dtype(r, p + 8, end, b)) return false;
      t.base.push_back(b);
      return r.ok;
    }
    default: return r.ok;   // compound / enum / array / ...: kept, values not decoded
  }
}

// ---------------------------------------------------------------- dataspace (IV.A.2.b)
bool parse_dspace(Rd &r, uint64_t p, std::vector<uint64_t> &dims, uint64_t &n) {
  const int ver = (int)r.u(p, 1), rank = (int)r.u(p + 1, 1);
  dims.clear();
  uint64_t q;
  bool null_space = false;
  if (ver == 1) q = p + 8;
  else if (ver == 2) { q = p + 4; null_space = r.u(p + 3, 1) == 2; }
  else return false;
  for (int k = 0; k < rank; k++) dims.push_back(r.len(q + (uint64_t)k * r.f.len_size));
  n = null_space ? 0 : 1;
  for (uint64_t d : dims) n *= d;
  return r.ok;
}

double num_at(Rd &r, uint64_t p, const DType &t) {
  const uint64_t raw = r.u(p, t.size);
  uint64_t v = raw;
  if (t.be) {   // byte-swap the little-endian read
    v = 0;
    for (int k = 0; k < t.size; k++) v = (v << 8) | ((raw >> (8 * k)) & 0xFF);
  }
  if (t.cls == 1) {
    if (t.size == 4) { uint32_t u = (uint32_t)v; float x; std::memcpy(&x, &u, 4); return x; }
    double x; std::memcpy(&x, &v, 8); return x;
  }
  if (t.sign) {
    const int sh = 64 - 8 * t.size;
    return (double)((int64_t)(v << sh) >> sh);
  }
  return (double)v;
}

// ---------------------------------------------------------------- global heap (III.E)
bool gheap_object(Rd &r, uint64_t coll, uint32_t index, uint64_t &at, uint64_t &size) {
  if (coll == kUndef || !r.sig(coll, "GCOL")) return false;
  const uint64_t csize = r.len(coll + 8);
  uint64_t p = coll + 8 + r.f.len_size;
  const uint64_t end = coll + csize;
  while (r.ok && p + 8 + r.f.len_size <= end) {
    const uint32_t idx = (uint32_t)r.u(p, 2);
    const uint64_t sz = r.len(p + 8);
    if (idx == 0) break;   // free space
    const uint64_t data = p + 8 + r.f.len_size;
    if (idx == index) { at = data; size = sz; return r.has(data, sz); }
    p = data + ((sz + 7) & ~(uint64_t)7);
  }
  return false;
}

// ---------------------------------------------------------------- attributes (IV.A.2.m)
bool parse_attr(Rd &r, uint64_t p, uint64_t size, Att &a, std::vector<uint64_t> *refs) {
  const int ver = (int)r.u(p, 1);
  const int flags = (int)r.u(p + 1, 1);
  const uint64_t nlen = r.u(p + 2, 2), tlen = r.u(p + 4, 2), slen = r.u(p + 6, 2);
  if (flags & 3) return false;   // shared datatype / dataspace: not in netCDF-4 attributes
  uint64_t q = p + 8;
  auto pad = [&](uint64_t n) { return ver == 1 ? (n + 7) & ~(uint64_t)7 : n; };
  if (ver == 3) q++;   // name character set
  else if (ver != 1 && ver != 2) return false;
  if (!r.has(q, nlen)) return false;
  a.name.assign((const char *)&r.f.buf[q], (size_t)nlen);
  while (!a.name.empty() && a.name.back() == '\0') a.name.pop_back();
  q += pad(nlen);
  DType t;
  if (!parse_dtype(r, q, q + tlen, t)) return false;
  q += pad(tlen);
  std::vector<uint64_t> dims;
  uint64_t n = 0;
  if (!parse_dspace(r, q, dims, n)) return false;
  q += pad(slen);
  if (n > (1u << 24) || (t.size > 0 && !r.has(q, n * (uint64_t)t.size))) return false;
  a.nctype = t.nctype();
  if (t.cls == 0 || t.cls == 1) {
    for (uint64_t i = 0; i < n; i++) a.num.push_back(num_at(r, q + i * t.size, t));
  } else if (t.cls == 3) {
    a.text.assign((const char *)&r.f.buf[q], (size_t)(n * t.size));
  } else if (t.cls == 9) {
    // element: sequence length (4), global heap collection (O), object index (4)
    for (uint64_t i = 0; i < n; i++) {
      const uint64_t e = q + i * t.size;
      const uint64_t cnt = r.u(e, 4);
      const uint64_t coll = r.addr(e + 4);
      const uint32_t idx = (uint32_t)r.u(e + 4 + r.f.off_size, 4);
      uint64_t at = 0, sz = 0;
      if (cnt == 0) { if (t.vlen_kind == 1 && i) a.text += ','; continue; }
      if (!gheap_object(r, coll, idx, at, sz)) return false;
      if (t.vlen_kind == 1) {
        if (i) a.text += ',';
        a.text.append((const char *)&r.f.buf[at], (size_t)sz);
      } else if (!t.base.empty() && t.base[0].cls == 7 && refs) {   // DIMENSION_LIST: object references
        refs->push_back(r.addr(at));                                  // the first reference of each element
      } else if (!t.base.empty() && (t.base[0].cls == 0 || t.base[0].cls == 1)) {
        for (uint64_t k = 0; k < cnt && (k + 1) * t.base[0].size <= sz; k++)
          a.num.push_back(num_at(r, at + k * t.base[0].size, t.base[0]));
      }
    }
  }
  (void)size;
  return r.ok;
}

// ---------------------------------------------------------------- v2 B-trees (III.A.2)
// Every record of the tree (depth-first), as file offsets.
bool btree2_records(Rd &r, uint64_t hdr, std::vector<uint64_t> &recs, uint32_t &rsize) {
  if (hdr == kUndef) return true;
  if (!r.sig(hdr, "BTHD")) return false;
  const uint64_t node_size = r.u(hdr + 6, 4);
  rsize = (uint32_t)r.u(hdr + 10, 2);
  const int depth = (int)r.u(hdr + 12, 2);
  const uint64_t root = r.addr(hdr + 16);
  const uint64_t root_n = r.u(hdr + 16 + r.f.off_size, 2);
  if (!r.ok || rsize == 0 || node_size < 16 || depth > 16) return false;
  // per depth: records a node holds at most and the widths of a child pointer's counts
  std::vector<uint64_t> max_nrec(depth + 1), cum_max(depth + 1);
  std::vector<int> nrec_sz(depth + 1), cum_sz(depth + 1);
  max_nrec[0] = (node_size - 10) / rsize;
  nrec_sz[0] = bytes_for(max_nrec[0]);
  cum_max[0] = max_nrec[0];
  cum_sz[0] = nrec_sz[0];
  for (int d = 1; d <= depth; d++) {
    const uint64_t ptr = (uint64_t)r.f.off_size + nrec_sz[0] + (d > 1 ? cum_sz[d - 1] : 0);
    max_nrec[d] = (node_size - 10 - ptr) / (rsize + ptr);
    nrec_sz[d] = bytes_for(max_nrec[d]);
    cum_max[d] = (max_nrec[d] + 1) * cum_max[d - 1] + max_nrec[d];
    cum_sz[d] = bytes_for(cum_max[d]);
  }
  uint64_t visited = 0;   // nodes of this walk (a crafted tree can point back into itself)
  std::function<bool(uint64_t, uint64_t, int)> walk = [&](uint64_t node, uint64_t n, int d) -> bool {
    if (recs.size() > (1u << 20) || ++visited > kMaxNodes) return false;
    if (d == 0) {
      if (!r.sig(node, "BTLF")) return false;
      for (uint64_t i = 0; i < n; i++) recs.push_back(node + 6 + i * rsize);
      return r.ok;
    }
    if (!r.sig(node, "BTIN")) return false;
    uint64_t p = node + 6 + n * rsize;
    const int ps = r.f.off_size + nrec_sz[0] + (d > 1 ? cum_sz[d - 1] : 0);
    for (uint64_t i = 0; i <= n; i++) {
      const uint64_t child = r.addr(p + i * ps);
      const uint64_t cn = r.u(p + i * ps + r.f.off_size, nrec_sz[0]);
      if (!walk(child, cn, d - 1)) return false;
      if (i < n) recs.push_back(node + 6 + i * rsize);
    }
    return r.ok;
  };
  return root == kUndef || walk(root, root_n, depth);
}

// ---------------------------------------------------------------- fractal heaps (III.G)
struct FHeap {
  uint64_t hdr = kUndef;
  int id_len = 0, width = 0, max_heap_bits = 0, cur_rows = 0;
  uint64_t start_block = 0, max_dblock = 0, max_obj = 0, root = kUndef;
  bool checksummed = false, filtered = false;
  int off_sz = 0, len_sz = 0, max_drows = 0;
};

bool fheap_open(Rd &r, uint64_t a, FHeap &h) {
  if (!r.sig(a, "FRHP")) return false;
  h.hdr = a;
  h.id_len = (int)r.u(a + 5, 2);
  h.filtered = r.u(a + 7, 2) != 0;
  h.checksummed = (r.u(a + 9, 1) & 2) != 0;
  h.max_obj = r.u(a + 10, 4);
  const int O = r.f.off_size, L = r.f.len_size;
  uint64_t p = a + 14 + L + O + L + O + 8 * (uint64_t)L;   // through "number of tiny objects"
  h.width = (int)r.u(p, 2);
  h.start_block = r.len(p + 2);
  h.max_dblock = r.len(p + 2 + L);
  h.max_heap_bits = (int)r.u(p + 2 + 2 * L, 2);
  h.root = r.addr(p + 2 + 2 * L + 4);
  h.cur_rows = (int)r.u(p + 2 + 2 * L + 4 + O, 2);
  if (!r.ok || h.width <= 0 || h.start_block == 0 || h.max_dblock < h.start_block || h.filtered) return false;
  h.off_sz = (h.max_heap_bits + 7) / 8;
  h.len_sz = std::min((log2_of(h.max_dblock) + 7) / 8, log2_of(h.max_obj) / 8 + 1);
  h.max_drows = log2_of(h.max_dblock) - log2_of(h.start_block) + 2;
  return true;
}

uint64_t row_block(const FHeap &h, int row) {
  return row == 0 ? h.start_block : h.start_block << (row - 1);
}

// File offset of the managed object at heap offset `off` (kUndef if absent).
uint64_t fheap_locate(Rd &r, const FHeap &h, uint64_t off) {
  if (h.root == kUndef) return kUndef;
  if (h.cur_rows == 0) return h.root + off;   // the root is a direct block at heap offset 0
  int visited = 0;
  std::function<uint64_t(uint64_t, uint64_t, int)> find = [&](uint64_t ib, uint64_t ib_off, int nrows) -> uint64_t {
    if (++visited > 64 || !r.sig(ib, "FHIB")) return kUndef;
    const uint64_t ents = ib + 5 + r.f.off_size + h.off_sz;
    const int nd = std::min(nrows, h.max_drows) * h.width;
    uint64_t pos = ib_off;
    for (int row = 0; row < nrows; row++) {
      const uint64_t bs = row_block(h, row);
      for (int c = 0; c < h.width; c++, pos += bs) {
        if (off >= pos + bs) continue;
        const int e = row * h.width + c;
        if (row < h.max_drows) {
          const uint64_t db = r.addr(ents + (uint64_t)e * r.f.off_size);
          return db == kUndef ? kUndef : db + (off - pos);
        }
        const uint64_t child = r.addr(ents + (uint64_t)nd * r.f.off_size + (uint64_t)(e - nd) * r.f.off_size);
        if (child == kUndef) return kUndef;
        const int child_rows = log2_of(bs) - log2_of(h.start_block * (uint64_t)h.width) + 1;
        return find(child, pos, child_rows);
      }
    }
    return kUndef;
  };
  return find(h.root, 0, h.cur_rows);
}

// The object a heap ID names: file offset + length (managed or tiny).
bool fheap_object(Rd &r, const FHeap &h, uint64_t id, uint64_t &at, uint64_t &len) {
  const int b0 = (int)r.u(id, 1);
  const int type = (b0 >> 4) & 3;
  if (type == 2) {   // tiny: the data is in the ID
    len = (uint64_t)(b0 & 0x0F) + 1;
    at = id + 1;
    return r.ok;
  }
  if (type != 0) return false;   // huge objects: not in netCDF-4 metadata
  const uint64_t off = r.u(id + 1, h.off_sz);
  len = r.u(id + 1 + h.off_sz, h.len_sz);
  at = fheap_locate(r, h, off);
  return r.ok && at != kUndef && r.has(at, len);
}

// ---------------------------------------------------------------- object headers (IV.A)
// Calls f(type, data offset, size) for every message, continuations followed.
bool for_messages(Rd &r, uint64_t oh, const std::function<bool(int, uint64_t, uint64_t)> &f) {
  struct Blk { uint64_t p, end; };
  std::vector<Blk> todo;
  bool v2 = false;
  if (r.sig(oh, "OHDR")) {
    v2 = true;
    const int flags = (int)r.u(oh + 5, 1);
    uint64_t p = oh + 6;
    if (flags & 0x20) p += 16;
    if (flags & 0x10) p += 4;
    const int nb = 1 << (flags & 3);
    const uint64_t size = r.u(p, nb);
    p += nb;
    todo.push_back({p, p + size});
    int guard = 0;
    for (size_t k = 0; k < todo.size() && r.ok; k++) {
      if (++guard > 4096) return false;
      uint64_t q = todo[k].p;
      const uint64_t end = todo[k].end;
      const int mh = 4 + ((flags & 0x04) ? 2 : 0);
      while (q + mh <= end && r.ok) {
        const int type = (int)r.u(q, 1);
        const uint64_t sz = r.u(q + 1, 2);
        const int mflags = (int)r.u(q + 3, 1);
        const uint64_t data = q + mh;
        if (data + sz > end) break;
        if (type == 0x10) {   // continuation: "OCHK", messages, checksum
          const uint64_t co = r.addr(data), cl = r.len(data + r.f.off_size);
          if (co == kUndef || !r.sig(co, "OCHK") || cl < 8) return false;
          todo.push_back({co + 4, co + cl - 4});
        } else if (type != 0 && !(mflags & 0x02)) {
          if (!f(type, data, sz)) return false;
        }
        q = data + sz;
      }
    }
  } else {
    if (r.u(oh, 1) != 1) return false;
    const uint64_t nmsgs = r.u(oh + 2, 2);
    const uint64_t hsize = r.u(oh + 8, 4);
    todo.push_back({oh + 16, oh + 16 + hsize});
    uint64_t seen = 0;
    for (size_t k = 0; k < todo.size() && r.ok && seen < nmsgs; k++) {
      if (k > 4096) return false;
      uint64_t q = todo[k].p;
      const uint64_t end = todo[k].end;
      while (q + 8 <= end && r.ok && seen < nmsgs) {
        const int type = (int)r.u(q, 2);
        const uint64_t sz = r.u(q + 2, 2);
        const int mflags = (int)r.u(q + 4, 1);
        const uint64_t data = q + 8;
        if (data + sz > end) break;
        seen++;
        if (type == 0x10) {
          const uint64_t co = r.addr(data), cl = r.len(data + r.f.off_size);
          if (co == kUndef) return false;
          todo.push_back({co, co + cl});
        } else if (type != 0 && !(mflags & 0x02)) {
          if (!f(type, data, sz)) return false;
        }
        q = data + sz;
      }
    }
  }
  (void)v2;
  return r.ok;
}

// ---------------------------------------------------------------- groups (IV.A.2.g/h/i, III.A.1, III.C, III.D)
struct Link { std::string name; uint64_t addr; };

bool parse_link(Rd &r, uint64_t p, uint64_t sz, Link &l) {
  if (r.u(p, 1) != 1) return false;
  const int flags = (int)r.u(p + 1, 1);
  uint64_t q = p + 2;
  int ltype = 0;
  if (flags & 0x08) { ltype = (int)r.u(q, 1); q++; }
  if (flags & 0x04) q += 8;
  if (flags & 0x10) q++;
  const int nl = 1 << (flags & 3);
  const uint64_t n = r.u(q, nl);
  q += nl;
  if (!r.has(q, n) || q + n > p + sz) return false;
  l.name.assign((const char *)&r.f.buf[q], (size_t)n);
  q += n;
  l.addr = ltype == 0 ? r.addr(q) : kUndef;   // soft / external links: not followed
  return r.ok;
}

bool symbol_table_links(Rd &r, uint64_t btree, uint64_t heap, std::vector<Link> &out) {
  if (!r.sig(heap, "HEAP")) return false;
  const uint64_t hdata = r.addr(heap + 8 + 2 * (uint64_t)r.f.len_size);
  const uint64_t hsize = r.len(heap + 8);
  const int O = r.f.off_size, L = r.f.len_size;
  uint64_t visited = 0;
  std::function<bool(uint64_t, int)> walk = [&](uint64_t node, int guard) -> bool {
    if (guard > 32 || ++visited > kMaxNodes || !r.sig(node, "TREE") || r.u(node + 4, 1) != 0) return false;
    const int level = (int)r.u(node + 5, 1);
    const uint64_t n = r.u(node + 6, 2);
    const uint64_t kc = node + 8 + 2 * (uint64_t)O;   // key0, child0, key1, ...
    for (uint64_t i = 0; i < n; i++) {
      const uint64_t child = r.addr(kc + L + i * (uint64_t)(L + O));
      if (level > 0) {
        if (!walk(child, guard + 1)) return false;
        continue;
      }
      if (!r.sig(child, "SNOD")) return false;
      const uint64_t ns = r.u(child + 6, 2);
      const uint64_t ent = child + 8;
      const uint64_t esz = 2 * (uint64_t)O + 24;
      for (uint64_t k = 0; k < ns; k++) {
        const uint64_t e = ent + k * esz;
        const uint64_t noff = r.u(e, O);
        Link l;
        l.addr = r.addr(e + O);
        if (noff >= hsize || !r.has(hdata + noff, 1)) return false;
        const char *s = (const char *)&r.f.buf[hdata + noff];
        l.name.assign(s, strnlen(s, (size_t)(hsize - noff)));
        out.push_back(l);
      }
    }
    return r.ok;
  };
  return walk(btree, 0);
}

// Links of the group whose object header is at oh.
bool group_links(Rd &r, uint64_t oh, std::vector<Link> &out) {
  uint64_t st_btree = kUndef, st_heap = kUndef, li_heap = kUndef, li_name = kUndef;
  bool ok = for_messages(r, oh, [&](int type, uint64_t p, uint64_t sz) {
    if (type == 0x11) { st_btree = r.addr(p); st_heap = r.addr(p + r.f.off_size); }
    else if (type == 0x06) { Link l; if (parse_link(r, p, sz, l)) out.push_back(l); }
    else if (type == 0x02) {
      const int flags = (int)r.u(p + 1, 1);
      const uint64_t q = p + 2 + ((flags & 1) ? 8 : 0);
      li_heap = r.addr(q);
      li_name = r.addr(q + r.f.off_size);
    }
    return true;
  });
  if (!ok) return false;
  if (st_btree != kUndef && !symbol_table_links(r, st_btree, st_heap, out)) return false;
  if (li_heap != kUndef && li_name != kUndef) {   // dense link storage
    FHeap h;
    if (!fheap_open(r, li_heap, h)) return false;
    std::vector<uint64_t> recs;
    uint32_t rsize = 0;
    if (!btree2_records(r, li_name, recs, rsize)) return false;
    for (uint64_t rec : recs) {   // type 5 record: name hash (4), heap ID
      uint64_t at = 0, len = 0;
      if (!fheap_object(r, h, rec + 4, at, len)) return false;
      Link l;
      if (!parse_link(r, at, len, l)) return false;
      out.push_back(l);
    }
  }
  return r.ok;
}

// ---------------------------------------------------------------- objects
struct Obj {
  bool dataset = false;
  std::vector<uint64_t> dims;
  DType type;
  int layout_ver = 0, layout = -1;
  uint64_t addr = kUndef, size = 0;
  std::vector<uint8_t> compact;
  std::vector<uint64_t> chunk;
  int index_type = 0;
  uint64_t single_size = 0;
  uint32_t single_mask = 0;
  int fa_bits = 0;
  bool single_filtered = false;
  std::vector<Filter> filters;
  std::vector<Att> atts;
  std::vector<uint8_t> fill;   // fill-value message's value (empty: none defined)
  std::vector<uint64_t> dim_refs;
};

bool parse_filters(Rd &r, uint64_t p, std::vector<Filter> &out) {
  const int ver = (int)r.u(p, 1), n = (int)r.u(p + 1, 1);
  uint64_t q = ver == 1 ? p + 8 : p + 2;
  if (ver != 1 && ver != 2) return false;
  for (int i = 0; i < n && r.ok; i++) {
    Filter f;
    f.id = (int)r.u(q, 2);
    uint64_t nlen = 0;
    if (ver == 1 || f.id >= 256) { nlen = r.u(q + 2, 2); q += 2; }
    const uint64_t ncd = r.u(q + 4, 2);
    q += 6;
    q += ver == 1 ? (nlen + 7) & ~(uint64_t)7 : nlen;
    for (uint64_t k = 0; k < ncd; k++) f.cd.push_back((uint32_t)r.u(q + 4 * k, 4));
    q += 4 * ncd;
    if (ver == 1 && (ncd & 1)) q += 4;
    out.push_back(f);
  }
  return r.ok;
}

bool parse_layout(Rd &r, uint64_t p, uint64_t sz, Obj &o) {
  const int ver = (int)r.u(p, 1);
  o.layout_ver = ver;
  const int O = r.f.off_size;
  if (ver == 3 || ver == 4) {
    o.layout = (int)r.u(p + 1, 1);
    if (o.layout == 0) {
      const uint64_t n = r.u(p + 2, 2);
      if (!r.has(p + 4, n)) return false;
      o.compact.assign(r.f.buf.begin() + (p + 4), r.f.buf.begin() + (p + 4 + n));
    } else if (o.layout == 1) {
      o.addr = r.addr(p + 2);
      o.size = r.len(p + 2 + O);
    } else if (o.layout == 2 && ver == 3) {
      const int nd = (int)r.u(p + 2, 1);
      o.addr = r.addr(p + 3);
      for (int k = 0; k + 1 < nd; k++) o.chunk.push_back(r.u(p + 3 + O + 4 * (uint64_t)k, 4));
      o.index_type = 0;
    } else if (o.layout == 2) {
      const int flags = (int)r.u(p + 2, 1), nd = (int)r.u(p + 3, 1), el = (int)r.u(p + 4, 1);
      uint64_t q = p + 5;
      for (int k = 0; k < nd; k++, q += el)
        if (k + 1 < nd) o.chunk.push_back(r.u(q, el));
      o.index_type = (int)r.u(q, 1);
      q++;
      if (o.index_type == 1) {
        if (flags & 2) {
          o.single_filtered = true;
          o.single_size = r.len(q);
          o.single_mask = (uint32_t)r.u(q + r.f.len_size, 4);
          q += r.f.len_size + 4;
        }
      } else if (o.index_type == 3) {
        o.fa_bits = (int)r.u(q, 1);
        q++;
      } else if (o.index_type != 2) {
        return false;   // extensible array / v2 B-tree chunk indexes: not in this subset
      }
      o.addr = r.addr(q);
    } else {
      return false;
    }
    (void)sz;
    return r.ok;
  }
  if (ver == 1 || ver == 2) {
    const int nd = (int)r.u(p + 1, 1);
    o.layout = (int)r.u(p + 2, 1);
    uint64_t q = p + 8;
    if (o.layout != 0) { o.addr = r.addr(q); q += O; }
    std::vector<uint64_t> d;
    for (int k = 0; k < nd; k++) d.push_back(r.u(q + 4 * (uint64_t)k, 4));
    q += 4 * (uint64_t)nd;
    if (o.layout == 2) { o.chunk.assign(d.begin(), d.end() - 1); o.index_type = 0; }
    else if (o.layout == 1) { o.size = 0; }
    else {
      const uint64_t n = r.u(q, 4);
      if (!r.has(q + 4, n)) return false;
      o.compact.assign(r.f.buf.begin() + (q + 4), r.f.buf.begin() + (q + 4 + n));
    }
    return r.ok;
  }
  return false;
}

bool parse_object(Rd &r, uint64_t oh, Obj &o) {
  uint64_t ai_heap = kUndef, ai_name = kUndef;
  bool ok = for_messages(r, oh, [&](int type, uint64_t p, uint64_t sz) {
    switch (type) {
      case 0x01: { uint64_t n; if (!parse_dspace(r, p, o.dims, n)) return false; break; }
      case 0x03: if (!parse_dtype(r, p, p + sz, o.type)) return false; break;
      case 0x08: o.dataset = true; if (!parse_layout(r, p, sz, o)) return false; break;
      case 0x0B: if (!parse_filters(r, p, o.filters)) return false; break;
      case 0x04: {   // old fill value: size, value
        const uint64_t n = r.u(p, 4);
        if (n > 0 && n <= 16 && n + 4 <= sz && r.has(p + 4, n)) o.fill.assign(r.f.buf.begin() + (p + 4), r.f.buf.begin() + (p + 4 + n));
        break;
      }
      case 0x05: {   // fill value (IV.A.2.f): v1/v2 allocation / write time bytes + "defined"; v3 flags
        const int ver = (int)r.u(p, 1);
        uint64_t q = 0;
        bool defined = false;
        if (ver == 1 || ver == 2) {
          defined = r.u(p + 3, 1) != 0;
          q = p + 4;
          if (ver == 1) defined = true;   // v1: size (+ value) always present
        } else if (ver == 3) {
          defined = (r.u(p + 1, 1) & 0x20) != 0;
          q = p + 2;
        }
        if (defined && q + 4 <= p + sz) {
          const uint64_t n = r.u(q, 4);
          if (n > 0 && n <= 16 && q + 4 + n <= p + sz && r.has(q + 4, n))
            o.fill.assign(r.f.buf.begin() + (q + 4), r.f.buf.begin() + (q + 4 + n));
          else if (n == 0) o.fill.clear();
        }
        break;
      }
      case 0x0C: {
        Att a;
        std::vector<uint64_t> refs;
        if (parse_attr(r, p, sz, a, &refs)) {
          if (a.name == "DIMENSION_LIST") o.dim_refs = refs;
          o.atts.push_back(a);
        }
        break;
      }
      case 0x15: {   // attribute info: dense attributes
        const int flags = (int)r.u(p + 1, 1);
        const uint64_t q = p + 2 + ((flags & 1) ? 2 : 0);
        ai_heap = r.addr(q);
        ai_name = r.addr(q + r.f.off_size);
        break;
      }
      default: break;
    }
    return true;
  });
  if (!ok) return false;
  if (ai_heap != kUndef && ai_name != kUndef) {
    FHeap h;
    if (!fheap_open(r, ai_heap, h)) return false;
    std::vector<uint64_t> recs;
    uint32_t rsize = 0;
    if (!btree2_records(r, ai_name, recs, rsize)) return false;
    for (uint64_t rec : recs) {   // type 8 record: heap ID (8), flags (1), creation order (4), hash (4)
      uint64_t at = 0, len = 0;
      if (!fheap_object(r, h, rec, at, len)) return false;
      Att a;
      std::vector<uint64_t> refs;
      if (parse_attr(r, at, len, a, &refs)) {
        if (a.name == "DIMENSION_LIST") o.dim_refs = refs;
        o.atts.push_back(a);
      }
    }
  }
  return r.ok;
}

// ---------------------------------------------------------------- chunks (III.A.1, VII.B filters)
struct ChunkRef { uint64_t addr, size; uint32_t mask; };

bool chunk_index_v1(Rd &r, uint64_t node, int rank, std::map<std::vector<uint64_t>, ChunkRef> &out, int guard,
                    uint64_t &visited) {
  if (guard > 32 || ++visited > kMaxNodes || !r.sig(node, "TREE") || r.u(node + 4, 1) != 1) return false;
  const int level = (int)r.u(node + 5, 1);
  const uint64_t n = r.u(node + 6, 2);
  const int O = r.f.off_size;
  const uint64_t ksz = 8 + 8 * (uint64_t)(rank + 1);
  uint64_t q = node + 8 + 2 * (uint64_t)O;
  for (uint64_t i = 0; i < n && r.ok; i++) {
    const uint64_t key = q + i * (ksz + O);
    const uint64_t child = r.addr(key + ksz);
    if (level > 0) {
      if (!chunk_index_v1(r, child, rank, out, guard + 1, visited)) return false;
      continue;
    }
    ChunkRef c;
    c.size = r.u(key, 4);
    c.mask = (uint32_t)r.u(key + 4, 4);
    c.addr = child;
    std::vector<uint64_t> off(rank);
    for (int k = 0; k < rank; k++) off[k] = r.u(key + 8 + 8 * (uint64_t)k, 8);
    out[off] = c;
  }
  return r.ok;
}

bool unfilter(const Var &v, const std::vector<uint8_t> &in, uint32_t mask, uint64_t want, std::vector<uint8_t> &out) {
  std::vector<uint8_t> cur = in, nxt;
  for (int i = (int)v.filters.size() - 1; i >= 0; i--) {
    if (mask & (1u << i)) continue;
    const Filter &f = v.filters[i];
    if (f.id == 1) {   // deflate (the stream may hold more than the chunk: a checksum filter ran first)
      nxt.assign(want + 64, 0);
      z_stream z;
      std::memset(&z, 0, sizeof(z));
      if (inflateInit(&z) != Z_OK) return false;
      z.next_in = cur.data();
      z.avail_in = (uInt)cur.size();
      int rc = Z_OK;
      for (;;) {
        z.next_out = nxt.data() + z.total_out;
        z.avail_out = (uInt)(nxt.size() - z.total_out);
        rc = inflate(&z, Z_NO_FLUSH);
        if (rc == Z_STREAM_END || (rc != Z_OK && rc != Z_BUF_ERROR)) break;
        if (z.avail_out == 0 && nxt.size() < 2 * want + (1u << 20)) { nxt.resize(nxt.size() * 2); continue; }
        if (z.avail_in == 0 || z.avail_out != 0) break;   // input exhausted, or no progress
        break;
      }
      const uint64_t got = z.total_out;
      inflateEnd(&z);
      if (rc != Z_STREAM_END) return false;
      nxt.resize(got);
      cur.swap(nxt);
    } else if (f.id == 2) {   // shuffle: byte k of every element, then byte k + 1 ...
      const uint64_t es = f.cd.empty() ? (uint64_t)v.esize : f.cd[0];
      if (es > 1) {
        const uint64_t ne = cur.size() / es;
        nxt.assign(cur.size(), 0);
        for (uint64_t b = 0; b < es; b++)
          for (uint64_t e = 0; e < ne; e++) nxt[e * es + b] = cur[b * ne + e];
        for (uint64_t t = ne * es; t < cur.size(); t++) nxt[t] = cur[t];   // leftover bytes stay
        cur.swap(nxt);
      }
    } else if (f.id == 3) {   // fletcher32: a 4-byte checksum at the end
      if (cur.size() < 4) return false;
      cur.resize(cur.size() - 4);
    } else {
      return false;   // szip and third-party filters: not in this subset
    }
  }
  if (cur.size() < want) return false;
  cur.resize(want);
  out.swap(cur);
  return true;
}

// Fill bytes of one element, file order: the dataset's fill-value message
// (what HDF5 returns for storage never written, and what netCDF-C reads back),
// else the _FillValue attribute, else netCDF-C's NC_FILL_* default of the
// type (netcdf.h), which netCDF-C stores in that message itself.
std::vector<uint8_t> fill_bytes(const Var &v) {
  if ((int)v.fill_msg.size() == v.esize && v.esize > 0) return v.fill_msg;
  std::vector<uint8_t> b(v.esize, 0);
  bool have = false;
  double x = 0.0;
  for (const Att &a : v.atts)
    if (a.name == "_FillValue" && !a.num.empty()) { x = a.num[0]; have = true; }
  uint64_t u = 0;
  if (have) {
    if (v.nctype == 5) { float f = (float)x; uint32_t w; std::memcpy(&w, &f, 4); u = w; }
    else if (v.nctype == 6) std::memcpy(&u, &x, 8);
    else if (v.nctype == 1 || v.nctype == 3 || v.nctype == 4 || v.nctype == 10) u = (uint64_t)(int64_t)x;
    else u = (uint64_t)x;
  } else {
    switch (v.nctype) {
      case 1: u = (uint64_t)(int64_t)-127; break;                   // NC_FILL_BYTE
      case 3: u = (uint64_t)(int64_t)-32767; break;                 // NC_FILL_SHORT
      case 4: u = (uint64_t)(int64_t)-2147483647; break;            // NC_FILL_INT
      case 5: { float f = 9.9692099683868690e+36f; uint32_t w; std::memcpy(&w, &f, 4); u = w; break; }
      case 6: { double d = 9.9692099683868690e+36; std::memcpy(&u, &d, 8); break; }
      case 7: u = 255u; break;                                      // NC_FILL_UBYTE
      case 8: u = 65535u; break;                                    // NC_FILL_USHORT
      case 9: u = 4294967295u; break;                               // NC_FILL_UINT
      case 10: u = (uint64_t)(int64_t)-9223372036854775806LL; break;  // NC_FILL_INT64
      case 11: u = 18446744073709551614ull; break;                  // NC_FILL_UINT64
      default: u = 0; break;                                        // NC_FILL_CHAR
    }
  }
  for (int k = 0; k < v.esize && k < 8; k++) b[v.big_endian ? v.esize - 1 - k : k] = (uint8_t)(u >> (8 * k));
  return b;
}

}  // namespace

bool is_hdf5(const std::vector<uint8_t> &buf) {
  static const uint8_t sig[8] = {0x89, 'H', 'D', 'F', '\r', '\n', 0x1a, '\n'};
  for (uint64_t at = 0; at + 8 <= buf.size(); at = at ? at * 2 : 512)
    if (std::memcmp(&buf[at], sig, 8) == 0) return true;
  return false;
}

bool open(File &f) {
  static const uint8_t sig[8] = {0x89, 'H', 'D', 'F', '\r', '\n', 0x1a, '\n'};
  uint64_t sb = kUndef;
  for (uint64_t at = 0; at + 8 <= f.buf.size(); at = at ? at * 2 : 512)
    if (std::memcmp(&f.buf[at], sig, 8) == 0) { sb = at; break; }
  if (sb == kUndef) { f.err = "no HDF5 signature"; return false; }
  Rd r{f};
  const int ver = (int)r.u(sb + 8, 1);
  uint64_t root = kUndef;
  if (ver == 0 || ver == 1) {
    f.off_size = (int)r.u(sb + 13, 1);
    f.len_size = (int)r.u(sb + 14, 1);
    const uint64_t p = sb + 24 + (ver == 1 ? 4 : 0);
    if (f.off_size != 4 && f.off_size != 8) { f.err = "offset size"; return false; }
    f.base = r.u(p, f.off_size);
    root = r.addr(p + 4 * (uint64_t)f.off_size + f.off_size);   // root symbol table entry: object header
  } else if (ver == 2 || ver == 3) {
    f.off_size = (int)r.u(sb + 9, 1);
    f.len_size = (int)r.u(sb + 10, 1);
    if (f.off_size != 4 && f.off_size != 8) { f.err = "offset size"; return false; }
    f.base = r.u(sb + 12, f.off_size);
    root = r.addr(sb + 12 + 3 * (uint64_t)f.off_size);
  } else {
    f.err = "superblock version";
    return false;
  }
  if (!r.ok || root == kUndef) { f.err = "truncated superblock"; return false; }
  std::vector<Link> links;
  if (!group_links(r, root, links)) { f.err = "root group"; return false; }
  Obj ro;
  if (!parse_object(r, root, ro)) { f.err = "root attributes"; return false; }
  f.gatts = ro.atts;
  for (const Link &l : links) {
    if (l.addr == kUndef) continue;
    Obj o;
    if (!parse_object(r, l.addr, o)) { f.err = "object " + l.name; return false; }
    if (!o.dataset) continue;   // subgroups: not read
    Var v;
    v.name = l.name;
    v.ohdr = l.addr;
    v.shape = o.dims;
    v.nctype = o.type.nctype();
    v.esize = o.type.size;
    v.big_endian = o.type.be;
    v.atts = o.atts;
    v.dim_refs = o.dim_refs;
    for (const Att &a : o.atts) {
      if (a.name == "CLASS" && a.text.compare(0, 15, "DIMENSION_SCALE") == 0) v.is_scale = true;
      if (a.name == "NAME" && a.text.compare(0, 45, "This is a netCDF dimension but not a netCDF v") == 0)
        v.pure_dim = true;
    }
    v.layout = o.layout;
    v.addr = o.addr;
    v.size = o.size;
    v.compact = o.compact;
    v.chunk = o.chunk;
    v.index_type = o.layout == 2 ? o.index_type : -1;
    v.single_size = o.single_filtered ? o.single_size : 0;
    v.single_mask = o.single_mask;
    v.fa_page_bits = o.fa_bits;
    v.filters = o.filters;
    if ((int)o.fill.size() == v.esize) v.fill_msg = o.fill;
    if (v.layout == 2 && v.chunk.size() != v.shape.size()) { f.err = "chunk rank of " + l.name; return false; }
    f.vars.push_back(std::move(v));
  }
  return true;
}

bool read(const File &f, const Var &v, uint64_t start, uint64_t count, uint8_t *out) {
  Rd r{f};
  const int rank = (int)v.shape.size();
  const uint64_t es = (uint64_t)v.esize;
  uint64_t total = 1;
  for (uint64_t d : v.shape) total *= d;
  if (es == 0 || start > total || count > total - start) return false;
  if (count == 0) return true;
  if (v.layout == 0 || v.layout == 1) {   // row-major in the file
    if (v.layout == 0) {
      if ((start + count) * es > v.compact.size()) return false;
      std::memcpy(out, v.compact.data() + start * es, count * es);
      return true;
    }
    if (v.addr == kUndef) {   // never written: the fill value
      const std::vector<uint8_t> fb = fill_bytes(v);
      for (uint64_t i = 0; i < count; i++) std::memcpy(out + i * es, fb.data(), es);
      return true;
    }
    if (!r.has(v.addr + start * es, count * es)) return false;
    std::memcpy(out, &f.buf[v.addr + start * es], count * es);
    return true;
  }
  if (v.layout != 2 || rank == 0) return false;
  // the box [lo, hi) the linear range covers: whole trailing dimensions
  std::vector<uint64_t> lo(rank, 0), hi(v.shape);
  uint64_t trail = 1;
  for (int k = 1; k < rank; k++) trail *= v.shape[k];
  if (start % trail || count % trail) return false;
  lo[0] = start / trail;
  hi[0] = (start + count) / trail;
  // chunk index
  std::map<std::vector<uint64_t>, ChunkRef> idx;
  uint64_t cbytes = es;
  for (uint64_t c : v.chunk) cbytes *= c;
  std::vector<uint64_t> nchunks(rank);
  uint64_t total_chunks = 1;
  for (int k = 0; k < rank; k++) {
    if (v.chunk[k] == 0) return false;
    nchunks[k] = (v.shape[k] + v.chunk[k] - 1) / v.chunk[k];
    total_chunks *= nchunks[k];
    if (total_chunks > ((uint64_t)1 << 32)) return false;   // a corrupt shape / chunk size
  }
  auto linear_chunk = [&](const std::vector<uint64_t> &off) {
    uint64_t li = 0;
    for (int k = 0; k < rank; k++) li = li * nchunks[k] + off[k] / v.chunk[k];
    return li;
  };
  std::vector<ChunkRef> by_linear;   // implicit / fixed array: by linear chunk index
  if (v.index_type == 0) {
    uint64_t visited = 0;
    if (v.addr != kUndef && !chunk_index_v1(r, v.addr, rank, idx, 0, visited)) return false;
  } else if (v.index_type == 1) {
    if (v.addr != kUndef) {
      ChunkRef c{v.addr, v.single_size ? v.single_size : cbytes, v.single_mask};
      idx[std::vector<uint64_t>(rank, 0)] = c;
    }
  } else if (v.index_type == 2) {
    for (uint64_t i = 0; i < total_chunks; i++) by_linear.push_back({v.addr + i * cbytes, cbytes, 0});
  } else if (v.index_type == 3) {   // fixed array header "FAHD" -> data block "FADB" (unpaged)
    if (!r.sig(v.addr, "FAHD")) return false;
    const int client = (int)r.u(v.addr + 5, 1), esz = (int)r.u(v.addr + 6, 1), bits = (int)r.u(v.addr + 7, 1);
    const uint64_t nent = r.len(v.addr + 8);
    const uint64_t db = r.addr(v.addr + 8 + f.len_size);
    if (nent > ((uint64_t)1 << bits) || !r.sig(db, "FADB")) return false;   // paged data blocks: not covered
    const uint64_t e0 = db + 6 + f.off_size;
    for (uint64_t i = 0; i < nent; i++) {
      const uint64_t e = e0 + i * esz;
      ChunkRef c{r.addr(e), cbytes, 0};
      if (client == 1) {
        const int csz = esz - f.off_size - 4;
        c.size = r.u(e + f.off_size, csz);
        c.mask = (uint32_t)r.u(e + f.off_size + csz, 4);
      }
      by_linear.push_back(c);
    }
  } else {
    return false;
  }
  if (!r.ok) return false;
  const std::vector<uint8_t> fb = fill_bytes(v);
  // every chunk meeting the box
  std::vector<uint64_t> c0(rank), c1(rank), cc(rank);
  for (int k = 0; k < rank; k++) {
    c0[k] = lo[k] / v.chunk[k];
    c1[k] = (hi[k] + v.chunk[k] - 1) / v.chunk[k];
    cc[k] = c0[k];
  }
  std::vector<uint64_t> box(rank);
  for (int k = 0; k < rank; k++) box[k] = hi[k] - lo[k];
  std::vector<uint8_t> raw, data;
  for (;;) {
    std::vector<uint64_t> off(rank);
    for (int k = 0; k < rank; k++) off[k] = cc[k] * v.chunk[k];
    const ChunkRef *c = nullptr;
    ChunkRef tmp;
    if (!by_linear.empty()) {
      const uint64_t li = linear_chunk(off);
      if (li < by_linear.size()) { tmp = by_linear[li]; c = &tmp; }
    } else {
      auto it = idx.find(off);
      if (it != idx.end()) c = &it->second;
    }
    bool have = c && c->addr != kUndef;
    if (have) {
      if (!r.has(c->addr, c->size)) return false;
      raw.assign(f.buf.begin() + c->addr, f.buf.begin() + (c->addr + c->size));
      if (v.filters.empty()) {
        if (raw.size() < cbytes) return false;
        data.swap(raw);
      } else if (!unfilter(v, raw, c->mask, cbytes, data)) {
        return false;
      }
    }
    // copy the intersection of this chunk with the box, row by row along the last dimension
    std::vector<uint64_t> a(rank), b(rank);
    for (int k = 0; k < rank; k++) {
      a[k] = std::max(lo[k], off[k]);
      b[k] = std::min(hi[k], off[k] + v.chunk[k]);
    }
    std::vector<uint64_t> it(a);
    const uint64_t run = b[rank - 1] - a[rank - 1];
    for (;;) {
      uint64_t co = 0, bo = 0;   // element offsets in the chunk / in the box
      for (int k = 0; k < rank; k++) {
        co = co * v.chunk[k] + (it[k] - off[k]);
        bo = bo * box[k] + (it[k] - lo[k]);
      }
      uint8_t *dst = out + bo * es;
      if (have) std::memcpy(dst, data.data() + co * es, run * es);
      else for (uint64_t i = 0; i < run; i++) std::memcpy(dst + i * es, fb.data(), es);
      int k = rank - 2;
      for (; k >= 0; k--) {
        if (++it[k] < b[k]) break;
        it[k] = a[k];
      }
      if (k < 0) break;
    }
    int k = rank - 1;
    for (; k >= 0; k--) {
      if (++cc[k] < c1[k]) break;
      cc[k] = c0[k];
    }
    if (k < 0) break;
  }
  return true;
}

}  // namespace h5
}  // namespace gsky
