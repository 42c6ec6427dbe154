// drill.h -- host launchers of drill.hip.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <vector>

namespace gsky {

// One batched readData call (worker/gdalprocess/drill.go:90-227) over a
// time-innermost stack; see gskyhip_drill_batch in include/gskyhip.h.
struct DrillCall {
  const float *stack;
  int xsize, ysize, n_bands, t_stride;
  const int32_t *win;          // dev: n_polys x {off_x, off_y, count_x, count_y}
  const int64_t *mask_off;     // dev: byte offset of each polygon's mask
  const uint8_t *masks;        // dev
  int n_polys;
  int64_t mask_bytes;          // size of masks (bounds the compacted pixel lists)
  const int32_t *bands;        // HOST band list (1-based) or NULL = 1..n_bands
  int n_list;
  float nodata, lo, hi;
  int pixel_count, band_strides, mode;
  double *out_value;
  int32_t *out_count;
  void *workspace;
  int64_t workspace_bytes;
  hipStream_t stream;
  // readData with deciles in reference order (mode 0): the mean pass also
  // writes every in-mask value band-major -- polygon p's rows start at
  // emit_chunk_base[p] * 64 * n_sel, one row of count[p] values (padded to
  // 64) per read band -- and each (polygon, band)'s smallest / largest order
  // key and count of non-nodata values (emit_stats[p * n_sel + j])
  float *emit_vals = nullptr;
  int32_t *emit_chunk_base = nullptr;
  uint4 *emit_stats = nullptr;
};

// Order-preserving 32-bit key of a float (the deciles' radix selection).
__device__ __forceinline__ uint32_t order_key(float f) {
  const uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

// computeDeciles (drill.go:229-273) for a batch of polygons: see
// gskyhip_drill_deciles in include/gskyhip.h.
struct DecileCall {
  const float *stack;
  int xsize, ysize, n_bands, t_stride;
  const int32_t *win;
  const int64_t *mask_off;
  const uint8_t *masks;
  int n_polys;
  int64_t mask_bytes;
  const int32_t *bands;        // HOST band list (1-based) or NULL = 1..n_bands
  int n_list;
  float nodata;
  int decile_count, band_chunk;
  const int32_t *totals;       // dev n_polys x n_list: the mean pass's totals (drill.go:172-191)
  float *out;                  // dev n_polys x n_list x decile_count
  int32_t *status;             // dev n_polys x n_list
  void *workspace;
  int64_t workspace_bytes;
  hipStream_t stream;
};

// readData complete (drill.go:90-227): mean / pixel count, decileCount >= 0,
// bandStrides >= 1 -- see gskyhip_drill_read_data in include/gskyhip.h.
struct ReadDataCall {
  const float *stack;
  int xsize, ysize, n_bands, t_stride;
  const int32_t *win;
  const int64_t *mask_off;
  const uint8_t *masks;
  int n_polys;
  int64_t mask_bytes;
  const int32_t *bands;        // HOST band list (1-based) or NULL = 1..n_bands
  int n_list;
  float nodata, lo, hi;
  int pixel_count, band_strides, decile_count, mode;
  double *out_value;           // dev n_polys x rows x (1 + decile_count)
  int32_t *out_count;
  int32_t *status;             // dev n_polys: 0, or GSKYHIP_E_RANGE (the reference panics)
  void *workspace;
  int64_t workspace_bytes;
  hipStream_t stream;
};
int64_t drill_read_data_workspace_size(int n_polys, int64_t mask_bytes, int n_list, int band_strides,
                                       int decile_count, int mode);
int launch_drill_read_data(const ReadDataCall &c);

__global__ __launch_bounds__(256) void drill_compact_kernel(const int32_t *__restrict__ win,
                                                            const int64_t *__restrict__ mask_off,
                                                            const uint8_t *__restrict__ masks, int n_polys,
                                                            int xsize, int ysize, int32_t *__restrict__ idx,
                                                            int32_t *__restrict__ count);
int64_t drill_deciles_workspace_size(int n_polys, int64_t mask_bytes, int band_chunk);
int launch_drill_deciles(const DecileCall &c);
// The fused path (DrillCall::emit_*): 64-pixel chunk offsets per polygon, and
// the selection over the mean pass's band-major rows and key ranges.
void launch_decile_chunk_scan(const int32_t *count, int n_polys, int32_t *chunk_base, hipStream_t s);
int launch_decile_select_fused(const float *vals, const int32_t *chunk_base, const int32_t *count,
                               const int32_t *totals, int n_polys, int n_sel, int decile_count, float nodata,
                               const uint4 *stats, float *out, int32_t *status, hipStream_t s);

int drill_rows_per_poly(int n_list, int band_strides);
int64_t drill_workspace_size(int n_polys, int64_t mask_bytes, int n_list, int band_strides, int mode);
int launch_drill_batch(const DrillCall &c);
int launch_drill_merge(const double *values, const int32_t *counts, int n_files, int n_dates, double *out,
                       hipStream_t stream);

}  // namespace gsky
