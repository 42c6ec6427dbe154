// hdf5.h -- the HDF5 subset netCDF-4 files use, read on the host for the
// granule ingest (ingest.hip), as GSKY_netCDF opens them through netCDF-C
// (libs/gdal/frmts/gsky_netcdf/netcdfdataset.cpp:8711-8870; warp.go:89-101
// routes every NETCDF: / *.nc path there).  Restated from the published
// HDF5 file format specification (version 3.0); no HDF5 library is in the
// image, so the reader is checked against the test suite's own writer
// (tests/h5write.py) -- parity unpinned.
//
// Covered: superblock versions 0-3; object headers v1 and v2 (continuation
// blocks); old-style groups (symbol table: v1 B-tree of SNOD nodes + local
// heap) and new-style groups (link messages, compact or dense: fractal heap +
// v2 B-tree name index); attributes compact or dense; datatypes fixed-point,
// floating-point (either byte order), fixed-length strings, variable-length
// strings and sequences (global heap), object references; dataspaces v1/v2;
// data layouts v3 (compact, contiguous, chunked with a v1 B-tree) and v4
// (compact, contiguous, chunked: single chunk, implicit, fixed array);
// filters deflate (1), shuffle (2), fletcher32 (3).  netCDF-4 on top: each
// dataset is a variable, dimension scales are the dimensions (their link
// names, their sizes), a variable's dimensions come from its DIMENSION_LIST
// references, the root group's attributes are the global attributes.
#pragma once
#include <stdint.h>

#include <string>
#include <vector>

namespace gsky {
namespace h5 {

struct Att {
  std::string name;
  int nctype = 0;            // netCDF type code (1 byte .. 11 uint64; 2 char for strings)
  std::vector<double> num;   // numeric values
  std::string text;          // string values (vlen strings joined by ',')
};

struct Filter {
  int id = 0;
  std::vector<uint32_t> cd;  // client data
};

struct Var {
  std::string name;
  uint64_t ohdr = 0;                 // object header address (dimension-scale references point here)
  std::vector<uint64_t> shape;
  int nctype = 0;                    // element type as a netCDF type code
  int esize = 0;                     // element bytes
  bool big_endian = false;
  std::vector<Att> atts;
  std::vector<uint64_t> dim_refs;    // DIMENSION_LIST: object header address per dimension
  bool is_scale = false;             // CLASS = "DIMENSION_SCALE"
  bool pure_dim = false;             // a dimension without a variable (netCDF-4's NAME marker)
  // storage
  int layout = -1;                   // 0 compact, 1 contiguous, 2 chunked
  uint64_t addr = 0, size = 0;       // contiguous: address / bytes; chunked: index address
  std::vector<uint8_t> compact;      // compact data
  std::vector<uint64_t> chunk;       // chunk dimensions (rank entries)
  int index_type = 1;                // chunked: 0 v1 B-tree, 1 single chunk, 2 implicit, 3 fixed array
  uint64_t single_size = 0;          // single filtered chunk: stored bytes
  uint32_t single_mask = 0;
  int fa_page_bits = 0;
  std::vector<Filter> filters;
  // the fill-value message (0x05, or the old 0x04) when it defines a value:
  // one element in the file's byte order; netCDF-C writes its NC_FILL_*
  // default there for variables without _FillValue
  std::vector<uint8_t> fill_msg;
};

struct File {
  std::vector<uint8_t> buf;
  int off_size = 8, len_size = 8;
  uint64_t base = 0;
  std::vector<Var> vars;
  std::vector<Att> gatts;
  std::string err;
};

// Parse the file in f.buf (a netCDF-4 / HDF5 file: signature at 0, 512,
// 1024, ...).  False with f.err set on anything outside the subset.
bool open(File &f);

// True if buf starts (at a superblock search offset) with the HDF5 signature.
bool is_hdf5(const std::vector<uint8_t> &buf);

// Elements [start, start + count) in row-major order of variable v into out
// (count * v.esize bytes, the file's byte order); false on a read error.
bool read(const File &f, const Var &v, uint64_t start, uint64_t count, uint8_t *out);

}  // namespace h5
}  // namespace gsky
