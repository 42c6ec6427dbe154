// drill.hip -- WPS drill zonal reduction (worker/gdalprocess/drill.go:90-227)
// over an HBM-resident time stack, for a batch of polygons.
//
// Layout: time-innermost [y][x][t] with t padded to t_stride, so one pixel's
// time vector is contiguous and a wave-instruction that reads 64 consecutive
// slices of one pixel moves 256 contiguous bytes.
//
// Pipeline (all asynchronous on one stream, workspace from the caller):
//   drill_compact_kernel   one block per polygon: the in-mask pixels of its
//                          window (mask byte 255, inside the stack) compacted
//                          to global pixel indices in row-major order -- the
//                          order of the reference's `for i < bandSize` loop --
//                          so the reduction never touches masked-out pixels.
//   hipcub radix sort      polygons by in-mask pixel count, largest first: the
//                          longest sequential walks start first.
//   drill_sum_kernel       mode 0 (reference order): one wave per (polygon,
//                          64 selected bands); lane j keeps a sequential
//                          float32 sum over the compacted pixels in order, so
//                          the means are bit-exact (drill.go:153-177).
//   drill_seg_kernel       mode 1 (wave split): the compacted list is cut in
//   + drill_combine_kernel segments of kSeg pixels, one wave per (segment,
//                          64 bands) keeps a float32 partial, partials are
//                          combined in float64 in segment order (deterministic);
//                          the largest polygon no longer bounds the launch.
//                          Within 1e-5 relative of the reference order.
//   drill_rows_kernel      bandStrides rows (drill.go:128-219).
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <vector>

#include "drill.h"
#include "gsky_device.h"

namespace gsky {

constexpr int kSeg = 1024;      // pixels per segment in the wave-split mode
constexpr int kUnroll = 16;     // pixel loads in flight per lane

// ---------------------------------------------------------------- compaction
__global__ __launch_bounds__(256) void drill_compact_kernel(const int32_t *__restrict__ win,
                                                            const int64_t *__restrict__ mask_off,
                                                            const uint8_t *__restrict__ masks, int n_polys,
                                                            int xsize, int ysize, int32_t *__restrict__ idx,
                                                            int32_t *__restrict__ count) {
  const int p = blockIdx.x;
  if (p >= n_polys) return;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int offX = win[4 * p], offY = win[4 * p + 1], cx = win[4 * p + 2], cy = win[4 * p + 3];
  const uint8_t *m = masks + mask_off[p];
  int32_t *out = idx + mask_off[p];
  __shared__ int s_wave[4];
  const int64_t npx = (cx > 0 && cy > 0) ? (int64_t)cx * cy : 0;
  int base = 0;
  for (int64_t i0 = 0; i0 < npx; i0 += 256) {
    const int64_t i = i0 + tid;
    bool in = false;
    int32_t pix = 0;
    if (i < npx) {
      const int iy = (int)(i / cx), ix = (int)(i - (int64_t)iy * cx);
      const int gx = offX + ix, gy = offY + iy;
      // a window reaching past the stack reads nothing there (the reference
      // clamps its window to the raster in getDrillFileDescriptor)
      in = m[i] == 255 && gx >= 0 && gx < xsize && gy >= 0 && gy < ysize;
      pix = gy * xsize + gx;
    }
    const unsigned long long b = __ballot(in);
    const int pos = __popcll(b & ((1ull << lane) - 1ull));
    if (lane == 0) s_wave[wave] = __popcll(b);
    __syncthreads();
    int wbase = base;
    for (int w = 0; w < wave; w++) wbase += s_wave[w];
    if (in) out[wbase + pos] = pix;
    base += s_wave[0] + s_wave[1] + s_wave[2] + s_wave[3];
    __syncthreads();
  }
  if (tid == 0) count[p] = base;
}

__global__ void iota_kernel(int32_t *v, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) v[i] = i;
}

// ---------------------------------------------------------------- per-pixel rule
// drill.go:154-169 for one value.
template <bool PC>
__device__ __forceinline__ void drill_acc(float val, float nodata, float lo, float hi, float &sum, int32_t &total) {
  if (val != nodata) {
    if (PC) total++;
    if (!(val < lo || val > hi)) {
      if (PC) {
        sum += 1.0f;
      } else {
        sum += val;
        total++;
      }
    }
  }
}

// Sequential walk of compacted pixels [k0, k1) for the lane's band.
template <bool PC>
__device__ __forceinline__ void drill_walk(const float *__restrict__ base, int t_stride,
                                           const int32_t *__restrict__ ip, int k0, int k1, float nodata, float lo,
                                           float hi, float &sum, int32_t &total) {
  int k = k0;
  for (; k + kUnroll <= k1; k += kUnroll) {
    float v[kUnroll];
#pragma unroll
    for (int q = 0; q < kUnroll; q++) v[q] = base[(int64_t)ip[k + q] * t_stride];
#pragma unroll
    for (int q = 0; q < kUnroll; q++) drill_acc<PC>(v[q], nodata, lo, hi, sum, total);
  }
  for (; k < k1; k++) drill_acc<PC>(base[(int64_t)ip[k] * t_stride], nodata, lo, hi, sum, total);
}

// The same walk for readData with deciles (DrillCall::emit_*): each lane
// also keeps its band's smallest / largest order key and count of
// non-nodata values, and the wave writes the values band-major: 32 pixels x
// 64 bands through an LDS tile, then two band rows of 128 contiguous bytes
// per store instruction (rows are 256-byte aligned and padded to 64 values,
// so the last block's padding lanes may write; per-lane 16-byte stores
// straight from the walk ran at a third of the rate, r04af).
__device__ __forceinline__ void wave_lds_fence() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <bool PC>
__device__ __forceinline__ void drill_walk_emit(const float *__restrict__ base, int t_stride,
                                                const int32_t *__restrict__ ip, int n, float nodata, float lo,
                                                float hi, float &sum, int32_t &total, float *__restrict__ rows,
                                                int64_t npad, int nb, float *T, uint32_t &ka, uint32_t &ko,
                                                int32_t &valid) {
  constexpr int kB = 32, kP = 65;
  const int lane = threadIdx.x & 63, px = lane & 31, hb = lane >> 5;
  for (int k0 = 0; k0 < n; k0 += kB) {
    float v[kB];
#pragma unroll
    for (int q = 0; q < kB; q++) v[q] = base[(int64_t)ip[min(k0 + q, n - 1)] * t_stride];
#pragma unroll
    for (int q = 0; q < kB; q++) {
      if (k0 + q < n) {   // uniform
        drill_acc<PC>(v[q], nodata, lo, hi, sum, total);
        const uint32_t key = order_key(v[q]);
        if (v[q] != nodata) { ka = min(ka, key); ko = max(ko, key); valid++; }
      }
      T[q * kP + lane] = v[q];
    }
    wave_lds_fence();
#pragma unroll 4
    for (int i = 0; i < 32; i++) {
      const int jj = 2 * i + hb;
      if (jj < nb) rows[(int64_t)jj * npad + k0 + px] = T[px * kP + jj];
    }
    wave_lds_fence();
  }
}

// Mode 0, reference order: one wave per (polygon, group of 64 selected bands),
// polygons largest first.
template <bool PC, bool EMIT = false>
__global__ __launch_bounds__(64) void drill_sum_kernel(const float *__restrict__ stack, int t_stride,
                                                       const int32_t *__restrict__ idx,
                                                       const int64_t *__restrict__ mask_off,
                                                       const int32_t *__restrict__ count,
                                                       const int32_t *__restrict__ order,
                                                       const int32_t *__restrict__ tsel, int n_sel, int n_groups,
                                                       float nodata, float lo, float hi,
                                                       double *__restrict__ band_value,
                                                       int32_t *__restrict__ band_count,
                                                       float *__restrict__ emit_vals,
                                                       const int32_t *__restrict__ emit_cb,
                                                       uint4 *__restrict__ emit_stats) {
  const int item = blockIdx.x;
  const int p = order[item / n_groups];
  const int j = (item % n_groups) * 64 + threadIdx.x;
  const bool active = j < n_sel;
  const int t = active ? tsel[j] : 0;
  float sum = 0.f;
  int32_t total = 0;
  if constexpr (EMIT) {
    __shared__ float T[32 * 65];
    const int n = count[p];
    const int64_t npad = (int64_t)(n + 63) / 64 * 64;
    const int g0 = (item % n_groups) * 64;
    float *rows = emit_vals + (int64_t)emit_cb[p] * 64 * n_sel + (int64_t)g0 * npad;
    uint32_t ka = 0xFFFFFFFFu, ko = 0u;
    int32_t valid = 0;
    drill_walk_emit<PC>(stack + t, t_stride, idx + mask_off[p], n, nodata, lo, hi, sum, total, rows, npad,
                        min(64, n_sel - g0), T, ka, ko, valid);
    if (active) emit_stats[(int64_t)p * n_sel + j] = make_uint4(ka, ko, (uint32_t)valid, 0u);
  } else {
    drill_walk<PC>(stack + t, t_stride, idx + mask_off[p], 0, count[p], nodata, lo, hi, sum, total);
  }
  if (!active) return;
  const int64_t o = (int64_t)p * n_sel + j;
  band_value[o] = total > 0 ? (double)(sum / (float)total) : 0.0;   // drill.go:172-177
  band_count[o] = total;
}

// Mode 0 without deciles: the reference-order walk with U pixel loads in
// flight per lane, in a kernel of its own (69 VGPRs at U = 32: 7 waves per
// SIMD; drill_sum_kernel's walk at 32 needs 86).  r04ap: 2.21 -> 1.99 ms per
// C4 step against drill_sum_kernel at 16.
template <bool PC, int U>
__global__ __launch_bounds__(64) void drill_sum_u_kernel(const float *__restrict__ stack, int t_stride,
                                                         const int32_t *__restrict__ idx,
                                                         const int64_t *__restrict__ mask_off,
                                                         const int32_t *__restrict__ count,
                                                         const int32_t *__restrict__ order,
                                                         const int32_t *__restrict__ tsel, int n_sel, int n_groups,
                                                         float nodata, float lo, float hi,
                                                         double *__restrict__ band_value,
                                                         int32_t *__restrict__ band_count) {
  const int item = blockIdx.x;
  const int p = order[item / n_groups];
  const int j = (item % n_groups) * 64 + threadIdx.x;
  const bool active = j < n_sel;
  const float *base = stack + (active ? tsel[j] : 0);
  const int32_t *ip = idx + mask_off[p];
  const int n = count[p];
  float sum = 0.f;
  int32_t total = 0;
  int k = 0;
  for (; k + U <= n; k += U) {
    float v[U];
#pragma unroll
    for (int q = 0; q < U; q++) v[q] = base[(int64_t)ip[k + q] * t_stride];
#pragma unroll
    for (int q = 0; q < U; q++) drill_acc<PC>(v[q], nodata, lo, hi, sum, total);
  }
  for (; k < n; k++) drill_acc<PC>(base[(int64_t)ip[k] * t_stride], nodata, lo, hi, sum, total);
  if (!active) return;
  const int64_t o = (int64_t)p * n_sel + j;
  band_value[o] = total > 0 ? (double)(sum / (float)total) : 0.0;
  band_count[o] = total;
}

// ---------------------------------------------------------------- wave split
// Exclusive scan of segments per polygon (one block; n_polys is modest).
__global__ __launch_bounds__(1024) void drill_seg_scan_kernel(const int32_t *__restrict__ count, int n_polys,
                                                              int32_t *__restrict__ seg_base) {
  __shared__ int32_t s_sum[1024];
  const int tid = threadIdx.x;
  int carry = 0;
  for (int c0 = 0; c0 < n_polys; c0 += 1024) {
    const int i = c0 + tid;
    const int v = i < n_polys ? (count[i] + kSeg - 1) / kSeg : 0;
    s_sum[tid] = v;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) {   // Hillis-Steele inclusive scan
      const int add = tid >= o ? s_sum[tid - o] : 0;
      __syncthreads();
      s_sum[tid] += add;
      __syncthreads();
    }
    if (i < n_polys) seg_base[i] = carry + s_sum[tid] - v;
    const int tot = s_sum[1023];
    __syncthreads();
    carry += tot;
  }
  if (tid == 0) seg_base[n_polys] = carry;
}

template <bool PC>
__global__ __launch_bounds__(64) void drill_seg_kernel(const float *__restrict__ stack, int t_stride,
                                                       const int32_t *__restrict__ idx,
                                                       const int64_t *__restrict__ mask_off,
                                                       const int32_t *__restrict__ count,
                                                       const int32_t *__restrict__ seg_base, int n_polys,
                                                       const int32_t *__restrict__ tsel, int n_sel, int n_groups,
                                                       float nodata, float lo, float hi,
                                                       float *__restrict__ part_sum,
                                                       int32_t *__restrict__ part_total) {
  const int seg = blockIdx.x / n_groups;
  if (seg >= seg_base[n_polys]) return;
  int lo_p = 0, hi_p = n_polys - 1;   // polygon owning segment `seg`
  while (lo_p < hi_p) {
    const int mid = (lo_p + hi_p + 1) >> 1;
    if (seg_base[mid] <= seg) lo_p = mid; else hi_p = mid - 1;
  }
  const int p = lo_p;
  const int s = seg - seg_base[p];
  const int j = (blockIdx.x % n_groups) * 64 + threadIdx.x;
  const bool active = j < n_sel;
  const int t = active ? tsel[j] : 0;
  const int k0 = s * kSeg, k1 = min(count[p], k0 + kSeg);
  float sum = 0.f;
  int32_t total = 0;
  drill_walk<PC>(stack + t, t_stride, idx + mask_off[p], k0, k1, nodata, lo, hi, sum, total);
  if (!active) return;
  part_sum[(int64_t)seg * n_sel + j] = sum;
  part_total[(int64_t)seg * n_sel + j] = total;
}

__global__ void drill_combine_kernel(const float *__restrict__ part_sum, const int32_t *__restrict__ part_total,
                                     const int32_t *__restrict__ seg_base, int n_polys, int n_sel,
                                     double *__restrict__ band_value, int32_t *__restrict__ band_count) {
  const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= (int64_t)n_polys * n_sel) return;
  const int p = (int)(gid / n_sel), j = (int)(gid % n_sel);
  double sum = 0.0;
  int32_t total = 0;
  for (int s = seg_base[p]; s < seg_base[p + 1]; s++) {
    sum += (double)part_sum[(int64_t)s * n_sel + j];
    total += part_total[(int64_t)s * n_sel + j];
  }
  band_value[gid] = total > 0 ? (double)((float)sum / (float)total) : 0.0;
  band_count[gid] = total;
}

// ---------------------------------------------------------------- bandStrides rows
// drill.go:128-219 from the per-read-band results: for band_strides == 1 the
// read list is the band list; otherwise read j = 2g is band[ibBgn] and
// j = 2g + 1 band[ibEnd - 1] of group g.
__global__ void drill_rows_kernel(const double *band_value, const int32_t *band_count, int n_polys, int n_list,
                                  int n_sel, int band_strides, int rows_per_poly, double *out_value,
                                  int32_t *out_count) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n_polys) return;
  const double *bv = band_value + (int64_t)p * n_sel;
  const int32_t *bc = band_count + (int64_t)p * n_sel;
  double *ov = out_value + (int64_t)p * rows_per_poly;
  int32_t *oc = out_count + (int64_t)p * rows_per_poly;
  int nrow = 0, g = 0;
  for (int ibBgn = 0; ibBgn < n_list; ibBgn += band_strides, g++) {
    const int j0 = 2 * g, j1 = 2 * g + 1;
    ov[nrow] = bv[j0]; oc[nrow] = bc[j0]; nrow++;
    if (band_strides > 2) {
      const double beta = (bv[j1] - bv[j0]) / (double)(band_strides - 1);
      const double cnt = round((double)(bc[j0] + bc[j1]) / 2.0);  // math.Round: half away from zero
      for (int ip = 1; ip < band_strides - 1; ip++) {
        ov[nrow] = bv[j0] + (double)ip * beta;
        oc[nrow] = (int32_t)cnt;
        nrow++;
      }
    }
    ov[nrow] = bv[j1]; oc[nrow] = bc[j1]; nrow++;
  }
}

// readData's TimeSeries with deciles (drill.go:150-219): nCols = 1 + dc
// columns per row -- the mean / count, then decile i with Count 1 (zeros
// with Count 0 where the band total is 0) -- and for bandStrides > 2 every
// column interpolated between the two bound bands of the group, counts
// math.Round((c0 + c1) / 2).  status[p]: GSKYHIP_E_RANGE if computeDeciles
// would have panicked on any read band of the polygon.
// One thread per (polygon, TimeSeries row): grid (row blocks, polygons).
// Row k of polygon p for bandStrides <= 1 is read band k; otherwise group g =
// k / R (R = max(2, bandStrides) rows: the first bound band, the
// interpolated columns, the last bound band).  status[p] (zeroed by the
// caller) receives the smallest error code of the polygon's deciles.
__global__ __launch_bounds__(128) void drill_timeseries_kernel(const double *band_value, const int32_t *band_count,
                                                               const float *dec, const int32_t *dec_status,
                                                               int n_polys, int n_list, int n_sel, int band_strides,
                                                               int dc, int rows_per_poly, double *out_value,
                                                               int32_t *out_count, int32_t *status) {
  const int p = blockIdx.y;
  const int row = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n_polys) return;
  int st = 0;
  if (row < rows_per_poly) {
    const int nc = 1 + dc;
    const double *bv = band_value + (int64_t)p * n_sel;
    const int32_t *bc = band_count + (int64_t)p * n_sel;
    double *ov = out_value + ((int64_t)p * rows_per_poly + row) * nc;
    int32_t *oc = out_count + ((int64_t)p * rows_per_poly + row) * nc;
    auto cell = [&](int j, int ic, double &v, int32_t &c) {
      if (ic == 0) { v = bv[j]; c = bc[j]; return; }
      const int64_t sj = (int64_t)p * n_sel + j;
      const int ds = dec_status[sj];
      if (ds == 0) { v = (double)dec[sj * dc + ic - 1]; c = 1; }
      else { v = 0.0; c = 0; if (ds != 1) st = min(st, ds); }
    };
    int j = row, ip = 0, R = 1;
    if (band_strides > 1) {
      R = band_strides > 2 ? band_strides : 2;
      const int g = row / R, k = row - g * R;
      j = k == 0 ? 2 * g : (k == R - 1 ? 2 * g + 1 : -1);
      ip = k;
    }
    if (j >= 0) {
      for (int ic = 0; ic < nc; ic++) cell(j, ic, ov[ic], oc[ic]);
    } else {   // interpolated column between the group's bound bands (drill.go:197-214)
      const int g = row / R;
      for (int ic = 0; ic < nc; ic++) {
        double v0, v1;
        int32_t c0, c1;
        cell(2 * g, ic, v0, c0);
        cell(2 * g + 1, ic, v1, c1);
        const double beta = (v1 - v0) / (double)(band_strides - 1);
        ov[ic] = v0 + (double)ip * beta;
        oc[ic] = (int32_t)round((double)(c0 + c1) / 2.0);   // math.Round: half away from zero
      }
    }
  }
  if (st) atomicMin(&status[p], st);
}

// DrillMerger weighted mean (drill_merger.go:79-93).
__global__ void drill_merge_kernel(const double *values, const int32_t *counts, int n_files, int n_dates,
                                   double *out) {
  const int d = blockIdx.x * blockDim.x + threadIdx.x;
  if (d >= n_dates) return;
  double total = 0.0;
  long count = 0;
  for (int f = 0; f < n_files; f++) {
    const double v = values[(long)f * n_dates + d];
    if (v == v) {
      total += v * (double)counts[(long)f * n_dates + d];
      count += counts[(long)f * n_dates + d];
    }
  }
  out[d] = (total == total && count > 0) ? total / (double)count : __longlong_as_double(0x7ff8000000000000LL);
}

// ======================================================================== host
int drill_rows_per_poly(int n_list, int band_strides) {
  if (band_strides <= 0) band_strides = 1;
  int nrow = 0;
  for (int ibBgn = 0; ibBgn < n_list; ibBgn += band_strides) {
    nrow++;
    if (band_strides > 2) nrow += band_strides - 2;
    if (band_strides > 1) nrow++;
  }
  return nrow;
}

static inline int64_t al256(int64_t x) { return (x + 255) & ~(int64_t)255; }

// Number of read bands (drill.go:134-137) for a band list of n_list.
static int read_count(int n_list, int band_strides) {
  if (band_strides <= 1) return n_list;
  return 2 * ((n_list + band_strides - 1) / band_strides);
}

static size_t sort_temp_bytes(int n_polys) {
  size_t bytes = 0;
  hipcub::DeviceRadixSort::SortPairsDescending(nullptr, bytes, (const int32_t *)nullptr, (int32_t *)nullptr,
                                               (const int32_t *)nullptr, (int32_t *)nullptr, n_polys);
  return bytes;
}

struct DrillWs {
  int32_t *idx, *count, *order, *keys_out, *ids, *tsel, *seg_base, *part_total;
  float *part_sum;
  double *band_value;
  int32_t *band_count;
  void *sort_tmp;
  size_t sort_bytes;
  int64_t total;
};

static DrillWs drill_carve(void *base, int n_polys, int64_t mask_bytes, int n_list, int band_strides, int mode) {
  DrillWs w;
  const int np = n_polys > 0 ? n_polys : 1;
  const int n_sel = read_count(n_list, band_strides);
  const int64_t n_seg_max = mask_bytes / kSeg + np;
  int64_t off = 0;
  auto take = [&](int64_t bytes) { const int64_t o = off; off = al256(off + bytes); return o; };
  const int64_t o_idx = take(4 * (mask_bytes > 0 ? mask_bytes : 1));
  const int64_t o_cnt = take(4 * (int64_t)np);
  const int64_t o_ord = take(4 * (int64_t)np);
  const int64_t o_ko = take(4 * (int64_t)np);
  const int64_t o_ids = take(4 * (int64_t)np);
  const int64_t o_tsel = take(4 * (int64_t)(n_sel > 0 ? n_sel : 1));
  const int64_t o_seg = take(4 * ((int64_t)np + 1));
  const bool split = mode == 1;
  const int64_t o_ps = take(split ? 4 * n_seg_max * n_sel : 0);
  const int64_t o_pt = take(split ? 4 * n_seg_max * n_sel : 0);
  const bool direct = band_strides <= 1;
  const int64_t o_bv = take(direct ? 0 : 8 * (int64_t)np * n_sel);
  const int64_t o_bc = take(direct ? 0 : 4 * (int64_t)np * n_sel);
  w.sort_bytes = sort_temp_bytes(np);
  const int64_t o_tmp = take((int64_t)w.sort_bytes);
  w.total = off;
  char *b = (char *)base;
  w.idx = (int32_t *)(b + o_idx); w.count = (int32_t *)(b + o_cnt); w.order = (int32_t *)(b + o_ord);
  w.keys_out = (int32_t *)(b + o_ko); w.ids = (int32_t *)(b + o_ids); w.tsel = (int32_t *)(b + o_tsel);
  w.seg_base = (int32_t *)(b + o_seg); w.part_sum = (float *)(b + o_ps); w.part_total = (int32_t *)(b + o_pt);
  w.band_value = (double *)(b + o_bv); w.band_count = (int32_t *)(b + o_bc); w.sort_tmp = b + o_tmp;
  return w;
}

int64_t drill_workspace_size(int n_polys, int64_t mask_bytes, int n_list, int band_strides, int mode) {
  if (band_strides <= 0) band_strides = 1;
  return drill_carve(nullptr, n_polys, mask_bytes, n_list, band_strides, mode).total;
}

int launch_drill_batch(const DrillCall &c) {
  const int band_strides = c.band_strides <= 0 ? 1 : c.band_strides;
  const int n_list = c.bands ? c.n_list : c.n_bands;
  if (c.n_polys <= 0 || n_list <= 0) return 0;
  if (c.mode != 0 && c.mode != 1) return GSKYHIP_E_ARG;
  if (c.t_stride < c.n_bands || (int64_t)c.xsize * c.ysize >= 2147483647LL) return GSKYHIP_E_ARG;
  if (!c.workspace ||
      c.workspace_bytes < drill_workspace_size(c.n_polys, c.mask_bytes, n_list, band_strides, c.mode))
    return GSKYHIP_E_ARG;
  DrillWs w = drill_carve(c.workspace, c.n_polys, c.mask_bytes, n_list, band_strides, c.mode);
  hipStream_t s = c.stream;
  // read list (drill.go:128-137): bands are 1-based GDAL band numbers
  const int n_sel = read_count(n_list, band_strides);
  std::vector<int32_t> tsel;
  tsel.reserve(n_sel);
  for (int ibBgn = 0; ibBgn < n_list; ibBgn += band_strides) {
    int ibEnd = ibBgn + band_strides;
    if (ibEnd > n_list) ibEnd = n_list;
    const int b0 = c.bands ? c.bands[ibBgn] : ibBgn + 1;
    const int b1 = c.bands ? c.bands[ibEnd - 1] : ibEnd;
    if (b0 < 1 || b0 > c.n_bands || b1 < 1 || b1 > c.n_bands) return GSKYHIP_E_RANGE;
    tsel.push_back(b0 - 1);
    if (band_strides > 1) tsel.push_back(b1 - 1);
  }
  if (hipMemcpyAsync(w.tsel, tsel.data(), sizeof(int32_t) * n_sel, hipMemcpyHostToDevice, s) != hipSuccess)
    return GSKYHIP_E_HIP;
  hipLaunchKernelGGL(drill_compact_kernel, dim3(c.n_polys), dim3(256), 0, s, c.win, c.mask_off, c.masks, c.n_polys,
                     c.xsize, c.ysize, w.idx, w.count);
  const bool direct = band_strides <= 1;
  double *bv = direct ? c.out_value : w.band_value;
  int32_t *bc = direct ? c.out_count : w.band_count;
  const int n_groups = (n_sel + 63) / 64;
  const bool pc = c.pixel_count != 0;
  if (c.mode == 0) {
    hipLaunchKernelGGL(iota_kernel, dim3((c.n_polys + 255) / 256), dim3(256), 0, s, w.ids, c.n_polys);
    size_t bytes = w.sort_bytes;
    if (hipcub::DeviceRadixSort::SortPairsDescending(w.sort_tmp, bytes, w.count, w.keys_out, w.ids, w.order,
                                                     c.n_polys, 0, 32, s) != hipSuccess)
      return GSKYHIP_E_HIP;
    const dim3 grid((unsigned)((int64_t)c.n_polys * n_groups));
    const bool emit = c.emit_vals != nullptr;
    if (emit) launch_decile_chunk_scan(w.count, c.n_polys, c.emit_chunk_base, s);
    auto *kf = emit ? (pc ? drill_sum_kernel<true, true> : drill_sum_kernel<false, true>)
                    : (pc ? drill_sum_kernel<true, false> : drill_sum_kernel<false, false>);
    bool walk32 = !emit;
#ifdef GSKYHIP_AB
    if (const char *ue = getenv("GSKYHIP_DRILL_U")) walk32 = walk32 && atoi(ue) != 16;   // 16: drill_sum_kernel
#endif
    if (walk32)
      hipLaunchKernelGGL((pc ? drill_sum_u_kernel<true, 32> : drill_sum_u_kernel<false, 32>), grid, dim3(64), 0, s,
                         c.stack, c.t_stride, w.idx, c.mask_off, w.count, w.order, w.tsel, n_sel, n_groups, c.nodata,
                         c.lo, c.hi, bv, bc);
    else
      hipLaunchKernelGGL(kf, grid, dim3(64), 0, s, c.stack, c.t_stride, w.idx, c.mask_off, w.count, w.order, w.tsel,
                         n_sel, n_groups, c.nodata, c.lo, c.hi, bv, bc, c.emit_vals, c.emit_chunk_base, c.emit_stats);
  } else {
    hipLaunchKernelGGL(drill_seg_scan_kernel, dim3(1), dim3(1024), 0, s, w.count, c.n_polys, w.seg_base);
    const int64_t n_seg_max = c.mask_bytes / kSeg + c.n_polys;
    const dim3 grid((unsigned)(n_seg_max * n_groups));
    if (pc)
      hipLaunchKernelGGL(drill_seg_kernel<true>, grid, dim3(64), 0, s, c.stack, c.t_stride, w.idx, c.mask_off,
                         w.count, w.seg_base, c.n_polys, w.tsel, n_sel, n_groups, c.nodata, c.lo, c.hi, w.part_sum,
                         w.part_total);
    else
      hipLaunchKernelGGL(drill_seg_kernel<false>, grid, dim3(64), 0, s, c.stack, c.t_stride, w.idx, c.mask_off,
                         w.count, w.seg_base, c.n_polys, w.tsel, n_sel, n_groups, c.nodata, c.lo, c.hi, w.part_sum,
                         w.part_total);
    const int64_t n_out = (int64_t)c.n_polys * n_sel;
    hipLaunchKernelGGL(drill_combine_kernel, dim3((unsigned)((n_out + 255) / 256)), dim3(256), 0, s, w.part_sum,
                       w.part_total, w.seg_base, c.n_polys, n_sel, bv, bc);
  }
  if (!direct) {
    const int rows = drill_rows_per_poly(n_list, band_strides);
    hipLaunchKernelGGL(drill_rows_kernel, dim3((c.n_polys + 127) / 128), dim3(128), 0, s, bv, bc, c.n_polys,
                       n_list, n_sel, band_strides, rows, c.out_value, c.out_count);
  }
  return hipGetLastError() == hipSuccess ? 0 : GSKYHIP_E_HIP;
}

// ---- readData complete: the read bands' means (stride 1 over the read list),
// their deciles, then the TimeSeries rows.
struct ReadWs {
  int32_t *sel_dummy;
  double *bv;
  int32_t *bc, *dst;
  float *dec;
  void *mean_ws, *dec_ws;
  int64_t mean_bytes, dec_bytes, total;
  int chunk;
  bool fused;   // mode 0 with deciles: the mean pass writes the band-major rows (DrillCall::emit_*)
  float *f_vals;
  int32_t *f_cb;
  uint4 *f_stats;
};

static ReadWs read_carve(void *base, int n_polys, int64_t mask_bytes, int n_list, int band_strides, int dc,
                         int mode) {
  ReadWs w;
  const int n_sel = read_count(n_list, band_strides <= 0 ? 1 : band_strides);
  const int np = n_polys > 0 ? n_polys : 1;
  int ws_log2 = 30;   // the deciles' band-major segment buffer: <= 2^ws_log2 values
#ifdef GSKYHIP_AB
  if (const char *e = getenv("GSKYHIP_DEC_WS_LOG2")) ws_log2 = std::max(20, std::min(34, atoi(e)));
#endif
  w.chunk = (int)std::max<int64_t>(1, std::min<int64_t>(n_sel, (1LL << ws_log2) / std::max<int64_t>(1, mask_bytes)));
  w.mean_bytes = drill_workspace_size(np, mask_bytes, n_sel, 1, mode);
  // fused: every read band's rows at once, up to 2^33 values (32 GB of the 288)
  int fused_log2 = 33;
#ifdef GSKYHIP_AB
  if (const char *e = getenv("GSKYHIP_DEC_FUSED_LOG2")) fused_log2 = std::max(0, std::min(36, atoi(e)));
#endif
  const int64_t f_vals = (mask_bytes + 64 * (int64_t)np) * n_sel;
  w.fused = mode == 0 && dc > 0 && fused_log2 > 0 && f_vals <= (1LL << fused_log2);
  int64_t f_cb = 0, f_st = 0, f_end = 0;
  if (w.fused) {
    f_cb = al256(4 * f_vals);
    f_st = f_cb + al256(4 * (mask_bytes / 64 + np + 1));
    f_end = f_st + al256(16 * (int64_t)np * n_sel);
  }
  w.dec_bytes = dc <= 0 ? 0 : w.fused ? f_end : drill_deciles_workspace_size(np, mask_bytes, w.chunk);
  int64_t off = 0;
  auto take = [&](int64_t bytes) { const int64_t o = off; off = al256(off + (bytes > 0 ? bytes : 0)); return o; };
  const int64_t o_bv = take(8 * (int64_t)np * n_sel);
  const int64_t o_bc = take(4 * (int64_t)np * n_sel);
  const int64_t o_dst = take(dc > 0 ? 4 * (int64_t)np * n_sel : 0);
  const int64_t o_dec = take(dc > 0 ? 4 * (int64_t)np * n_sel * dc : 0);
  const int64_t o_mw = take(w.mean_bytes);
  const int64_t o_dw = take(w.dec_bytes);
  w.total = (w.dec_bytes < 0) ? -1 : off;
  char *b = (char *)base;
  w.sel_dummy = nullptr;
  w.bv = (double *)(b + o_bv); w.bc = (int32_t *)(b + o_bc); w.dst = (int32_t *)(b + o_dst);
  w.dec = (float *)(b + o_dec); w.mean_ws = b + o_mw; w.dec_ws = b + o_dw;
  w.f_vals = w.fused ? (float *)(b + o_dw) : nullptr;
  w.f_cb = w.fused ? (int32_t *)(b + o_dw + f_cb) : nullptr;
  w.f_stats = w.fused ? (uint4 *)(b + o_dw + f_st) : nullptr;
  return w;
}

int64_t drill_read_data_workspace_size(int n_polys, int64_t mask_bytes, int n_list, int band_strides,
                                       int decile_count, int mode) {
  if (n_polys <= 0 || n_list <= 0) return 0;
  return read_carve(nullptr, n_polys, mask_bytes, n_list, band_strides, decile_count, mode).total;
}

int launch_drill_read_data(const ReadDataCall &c) {
  const int band_strides = c.band_strides <= 0 ? 1 : c.band_strides;
  const int n_list = c.bands ? c.n_list : c.n_bands;
  if (c.n_polys <= 0 || n_list <= 0) return 0;
  if (c.decile_count < 0) return GSKYHIP_E_ARG;
  const int64_t need = drill_read_data_workspace_size(c.n_polys, c.mask_bytes, n_list, band_strides,
                                                      c.decile_count, c.mode);
  if (need < 0 || !c.workspace || c.workspace_bytes < need) return GSKYHIP_E_ARG;
  ReadWs w = read_carve(c.workspace, c.n_polys, c.mask_bytes, n_list, band_strides, c.decile_count, c.mode);
  // the read list (drill.go:128-137) as 1-based bands, stride 1
  std::vector<int32_t> sel;
  for (int ibBgn = 0; ibBgn < n_list; ibBgn += band_strides) {
    const int ibEnd = std::min(ibBgn + band_strides, n_list);
    sel.push_back(c.bands ? c.bands[ibBgn] : ibBgn + 1);
    if (band_strides > 1) sel.push_back(c.bands ? c.bands[ibEnd - 1] : ibEnd);
  }
  const int n_sel = (int)sel.size();
  DrillCall m;
  m.stack = c.stack; m.xsize = c.xsize; m.ysize = c.ysize; m.n_bands = c.n_bands; m.t_stride = c.t_stride;
  m.win = c.win; m.mask_off = c.mask_off; m.masks = c.masks; m.n_polys = c.n_polys; m.mask_bytes = c.mask_bytes;
  m.bands = sel.data(); m.n_list = n_sel; m.nodata = c.nodata; m.lo = c.lo; m.hi = c.hi;
  m.pixel_count = c.pixel_count; m.band_strides = 1; m.mode = c.mode;
  m.out_value = w.bv; m.out_count = w.bc; m.workspace = w.mean_ws; m.workspace_bytes = w.mean_bytes;
  m.stream = c.stream;
  if (w.fused) { m.emit_vals = w.f_vals; m.emit_chunk_base = w.f_cb; m.emit_stats = w.f_stats; }
  int rc = launch_drill_batch(m);
  if (rc) return rc;
  if (c.decile_count > 0 && w.fused) {
    const DrillWs mw = drill_carve(w.mean_ws, c.n_polys, c.mask_bytes, n_sel, 1, c.mode);
    if ((rc = launch_decile_select_fused(w.f_vals, w.f_cb, mw.count, w.bc, c.n_polys, n_sel, c.decile_count,
                                         c.nodata, w.f_stats, w.dec, w.dst, c.stream)))
      return rc;
  } else if (c.decile_count > 0) {
    DecileCall d;
    d.stack = c.stack; d.xsize = c.xsize; d.ysize = c.ysize; d.n_bands = c.n_bands; d.t_stride = c.t_stride;
    d.win = c.win; d.mask_off = c.mask_off; d.masks = c.masks; d.n_polys = c.n_polys; d.mask_bytes = c.mask_bytes;
    d.bands = sel.data(); d.n_list = n_sel; d.nodata = c.nodata; d.decile_count = c.decile_count;
    d.band_chunk = w.chunk; d.totals = w.bc; d.out = w.dec; d.status = w.dst;
    d.workspace = w.dec_ws; d.workspace_bytes = w.dec_bytes; d.stream = c.stream;
    if ((rc = launch_drill_deciles(d))) return rc;
  }
  const int rows = drill_rows_per_poly(n_list, band_strides);
  if (hipMemsetAsync(c.status, 0, sizeof(int32_t) * (size_t)c.n_polys, c.stream) != hipSuccess) return GSKYHIP_E_HIP;
  hipLaunchKernelGGL(drill_timeseries_kernel, dim3((rows + 127) / 128, c.n_polys), dim3(128), 0, c.stream, w.bv,
                     w.bc, w.dec, w.dst, c.n_polys, n_list, n_sel, band_strides, c.decile_count, rows, c.out_value,
                     c.out_count, c.status);
  return hipGetLastError() == hipSuccess ? 0 : GSKYHIP_E_HIP;
}

int launch_drill_merge(const double *values, const int32_t *counts, int n_files, int n_dates, double *out,
                       hipStream_t stream) {
  if (n_dates <= 0) return 0;
  hipLaunchKernelGGL(drill_merge_kernel, dim3((n_dates + 255) / 256), dim3(256), 0, stream, values, counts,
                     n_files, n_dates, out);
  return hipGetLastError() == hipSuccess ? 0 : GSKYHIP_E_HIP;
}

}  // namespace gsky
