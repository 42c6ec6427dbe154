// drill_deciles.hip -- computeDeciles (worker/gdalprocess/drill.go:229-273)
// for a batch of polygons over the HBM-resident time stack, as a segmented
// GPU sort.
//
// Per (polygon, band) the reference collects the in-mask, non-nodata values
// (no clipping), sorts them ascending and reads decileCount order statistics:
// step = len / (dc + 1); if step > 0, decile i = buf[(i+1)*step], or the
// float32 mean of it and its successor when len % (dc + 1) == 0; otherwise
// the values are repeated in order to fill dc slots.  It runs only where the
// band's mean-pass total is > 0 (drill.go:179-191).
//
// Pipeline per chunk of bands (all asynchronous, workspace from the caller):
//   drill_compact_kernel (drill.hip)  in-mask pixels of each window, compacted
//   decile_count_kernel   one wave per (polygon, 64 bands of the chunk): the
//                         non-nodata values of each segment
//   hipcub ExclusiveSum   segment offsets
//   decile_gather_kernel  the segment values, contiguous
//   hipcub SegmentedSort  ascending float keys per segment (radix)
//   decile_pick_kernel    one thread per segment: the reference's picks
// Sorting floats by key bits orders -0.0 before +0.0 where Go's sort may
// leave them in either order; the picked values are then equal as float32
// (NaN-free stacks; with NaNs the reference's order is implementation-defined).
#include <hipcub/hipcub.hpp>

#include <vector>

#include "drill.h"
#include "gsky_device.h"

namespace gsky {

namespace {

constexpr int kDUnroll = 16;

// one wave per (polygon, group of 64 bands of the chunk); lane = band
__global__ __launch_bounds__(64) void decile_count_kernel(const float *__restrict__ stack, int t_stride,
                                                          const int32_t *__restrict__ idx,
                                                          const int64_t *__restrict__ mask_off,
                                                          const int32_t *__restrict__ count,
                                                          const int32_t *__restrict__ tsel, int n_chunk,
                                                          int n_groups, float nodata, int32_t *__restrict__ cnt) {
  const int p = blockIdx.x / n_groups;
  const int j = (blockIdx.x % n_groups) * 64 + threadIdx.x;
  const bool active = j < n_chunk;
  const float *base = stack + (active ? tsel[j] : 0);
  const int32_t *ip = idx + mask_off[p];
  const int n = count[p];
  int32_t c = 0;
  int k = 0;
  for (; k + kDUnroll <= n; k += kDUnroll) {
    float v[kDUnroll];
#pragma unroll
    for (int q = 0; q < kDUnroll; q++) v[q] = base[(int64_t)ip[k + q] * t_stride];
#pragma unroll
    for (int q = 0; q < kDUnroll; q++) c += v[q] != nodata ? 1 : 0;
  }
  for (; k < n; k++) c += base[(int64_t)ip[k] * t_stride] != nodata ? 1 : 0;
  if (active) cnt[(int64_t)p * n_chunk + j] = c;
}

__global__ __launch_bounds__(64) void decile_gather_kernel(const float *__restrict__ stack, int t_stride,
                                                           const int32_t *__restrict__ idx,
                                                           const int64_t *__restrict__ mask_off,
                                                           const int32_t *__restrict__ count,
                                                           const int32_t *__restrict__ tsel, int n_chunk,
                                                           int n_groups, float nodata, const int32_t *__restrict__ off,
                                                           float *__restrict__ vals) {
  const int p = blockIdx.x / n_groups;
  const int j = (blockIdx.x % n_groups) * 64 + threadIdx.x;
  if (j >= n_chunk) return;
  const float *base = stack + tsel[j];
  const int32_t *ip = idx + mask_off[p];
  const int n = count[p];
  float *out = vals + off[(int64_t)p * n_chunk + j];
  int w = 0;
  int k = 0;
  for (; k + kDUnroll <= n; k += kDUnroll) {
    float v[kDUnroll];
#pragma unroll
    for (int q = 0; q < kDUnroll; q++) v[q] = base[(int64_t)ip[k + q] * t_stride];
#pragma unroll
    for (int q = 0; q < kDUnroll; q++)
      if (v[q] != nodata) out[w++] = v[q];
  }
  for (; k < n; k++) {
    const float v = base[(int64_t)ip[k] * t_stride];
    if (v != nodata) out[w++] = v;
  }
}

// computeDeciles on a sorted segment; status 0, 1 (band total 0: zeros, Count
// 0 in the reference's TimeSeries) or GSKYHIP_E_RANGE (the reference indexes
// buf[len] and panics: len == dc + 1... with len % (dc + 1) == 0 and step 1).
__global__ void decile_pick_kernel(const float *__restrict__ sorted, const int32_t *__restrict__ off,
                                   const int32_t *__restrict__ totals, int n_polys, int n_chunk, int b0, int n_list,
                                   int dc, float *__restrict__ out, int32_t *__restrict__ status) {
  const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= (int64_t)n_polys * n_chunk) return;
  const int p = (int)(s / n_chunk), j = (int)(s % n_chunk);
  const int64_t o = (int64_t)p * n_list + b0 + j;
  float *dst = out + o * dc;
  if (totals[o] <= 0) {   // drill.go:186-190
    for (int i = 0; i < dc; i++) dst[i] = 0.f;
    status[o] = 1;
    return;
  }
  const float *buf = sorted + off[s];
  const int len = off[s + 1] - off[s];
  status[o] = 0;
  if (len <= 0) {   // total > 0 implies a non-nodata value; keep the slot defined anyway
    for (int i = 0; i < dc; i++) dst[i] = 0.f;
    return;
  }
  const int step = len / (dc + 1);
  if (step > 0) {
    const bool isEven = len % (dc + 1) == 0;
    for (int i = 0; i < dc; i++) {
      const int iStep = (i + 1) * step;
      float de = buf[iStep];
      if (isEven) {
        if (iStep + 1 >= len) { status[o] = GSKYHIP_E_RANGE; de = 0.f; }
        else de = (buf[iStep] + buf[iStep + 1]) / 2.0f;
      }
      dst[i] = de;
    }
  } else {
    // padding[i % len]++ for i < dc, then each value repeated padding times, in order
    int idx = 0;
    for (int i = 0; i < len && idx < dc; i++) {
      const int pad = dc / len + (i < dc % len ? 1 : 0);
      for (int q = 0; q < pad && idx < dc; q++) dst[idx++] = buf[i];
    }
  }
}

inline int64_t al256(int64_t x) { return (x + 255) & ~(int64_t)255; }

struct DecWs {
  int32_t *idx, *count, *cnt, *off, *tsel;
  float *vals, *sorted;
  void *scan_tmp, *sort_tmp;
  size_t scan_bytes, sort_bytes;
  int64_t total;
};

DecWs decile_carve(void *base, int n_polys, int64_t mask_bytes, int chunk) {
  DecWs w;
  const int64_t n_seg = (int64_t)n_polys * chunk;
  const int64_t cap = mask_bytes * chunk;
  w.scan_bytes = 0;
  hipcub::DeviceScan::ExclusiveSum(nullptr, w.scan_bytes, (const int32_t *)nullptr, (int32_t *)nullptr,
                                   (int)(n_seg + 1));
  w.sort_bytes = 0;
  hipcub::DeviceSegmentedSort::SortKeys(nullptr, w.sort_bytes, (const float *)nullptr, (float *)nullptr,
                                        (int)cap, (int)n_seg, (const int32_t *)nullptr, (const int32_t *)nullptr);
  char *b = (char *)base;
  int64_t o = 0;
  auto take = [&](int64_t bytes) { char *p = b ? b + o : nullptr; o += al256(bytes); return p; };
  w.idx = (int32_t *)take(mask_bytes * 4);
  w.count = (int32_t *)take((int64_t)n_polys * 4);
  w.cnt = (int32_t *)take((n_seg + 1) * 4);
  w.off = (int32_t *)take((n_seg + 1) * 4);
  w.tsel = (int32_t *)take((int64_t)chunk * 4);
  w.vals = (float *)take(cap * 4);
  w.sorted = (float *)take(cap * 4);
  w.scan_tmp = take((int64_t)w.scan_bytes);
  w.sort_tmp = take((int64_t)w.sort_bytes);
  w.total = o;
  return w;
}

}  // namespace

int64_t drill_deciles_workspace_size(int n_polys, int64_t mask_bytes, int band_chunk) {
  if (n_polys <= 0 || band_chunk <= 0 || mask_bytes < 0) return 0;
  if (mask_bytes * band_chunk >= 2147483647LL || (int64_t)n_polys * band_chunk >= 2147483647LL) return -1;
  return decile_carve(nullptr, n_polys, mask_bytes, band_chunk).total;
}

int launch_drill_deciles(const DecileCall &c) {
  const int n_list = c.bands ? c.n_list : c.n_bands;
  if (c.n_polys <= 0 || n_list <= 0) return 0;
  if (c.decile_count <= 0 || c.band_chunk <= 0) return GSKYHIP_E_ARG;
  if (c.t_stride < c.n_bands || (int64_t)c.xsize * c.ysize >= 2147483647LL) return GSKYHIP_E_ARG;
  const int64_t need = drill_deciles_workspace_size(c.n_polys, c.mask_bytes, c.band_chunk);
  if (need < 0 || !c.workspace || c.workspace_bytes < need) return GSKYHIP_E_ARG;
  std::vector<int32_t> sel(n_list);
  for (int i = 0; i < n_list; i++) {
    const int b = c.bands ? c.bands[i] : i + 1;
    if (b < 1 || b > c.n_bands) return GSKYHIP_E_RANGE;
    sel[i] = b - 1;
  }
  DecWs w = decile_carve(c.workspace, c.n_polys, c.mask_bytes, c.band_chunk);
  hipStream_t s = c.stream;
  hipLaunchKernelGGL(drill_compact_kernel, dim3(c.n_polys), dim3(256), 0, s, c.win, c.mask_off, c.masks, c.n_polys,
                     c.xsize, c.ysize, w.idx, w.count);
  for (int b0 = 0; b0 < n_list; b0 += c.band_chunk) {
    const int n_chunk = std::min(c.band_chunk, n_list - b0);
    const int n_groups = (n_chunk + 63) / 64;
    const int64_t n_seg = (int64_t)c.n_polys * n_chunk;
    if (hipMemcpyAsync(w.tsel, sel.data() + b0, sizeof(int32_t) * n_chunk, hipMemcpyHostToDevice, s) != hipSuccess)
      return GSKYHIP_E_HIP;
    if (hipMemsetAsync(w.cnt + n_seg, 0, sizeof(int32_t), s) != hipSuccess) return GSKYHIP_E_HIP;
    const dim3 grid((unsigned)((int64_t)c.n_polys * n_groups));
    hipLaunchKernelGGL(decile_count_kernel, grid, dim3(64), 0, s, c.stack, c.t_stride, w.idx, c.mask_off, w.count,
                       w.tsel, n_chunk, n_groups, c.nodata, w.cnt);
    size_t sb = w.scan_bytes;
    if (hipcub::DeviceScan::ExclusiveSum(w.scan_tmp, sb, w.cnt, w.off, (int)(n_seg + 1), s) != hipSuccess)
      return GSKYHIP_E_HIP;
    hipLaunchKernelGGL(decile_gather_kernel, grid, dim3(64), 0, s, c.stack, c.t_stride, w.idx, c.mask_off, w.count,
                       w.tsel, n_chunk, n_groups, c.nodata, w.off, w.vals);
    // the item count is on the device; sort the capacity bound's worth of
    // segments by their own offsets (items past the last offset are untouched)
    size_t tb = w.sort_bytes;
    if (hipcub::DeviceSegmentedSort::SortKeys(w.sort_tmp, tb, w.vals, w.sorted,
                                              (int)(c.mask_bytes * n_chunk), (int)n_seg, w.off, w.off + 1,
                                              s) != hipSuccess)
      return GSKYHIP_E_HIP;
    hipLaunchKernelGGL(decile_pick_kernel, dim3((unsigned)((n_seg + 255) / 256)), dim3(256), 0, s, w.sorted, w.off,
                       c.totals, c.n_polys, n_chunk, b0, n_list, c.decile_count, c.out, c.status);
  }
  return hipGetLastError() == hipSuccess ? 0 : GSKYHIP_E_HIP;
}

}  // namespace gsky
