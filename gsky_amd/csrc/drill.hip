// drill.hip -- WPS drill zonal reduction (worker/gdalprocess/drill.go:90-227)
// over an HBM-resident time stack.
//
// Layout: time-innermost [y][x][t] with t padded to t_stride (multiple of 4),
// so one pixel's time vector is a contiguous run of 16-byte words.  Lane l of
// a polygon's block owns bands 4l..4l+3 and walks the polygon window in the
// reference's row-major pixel order, keeping four sequential float32 sums:
// the additions happen in exactly the order of drill.go:153-170, so means are
// bit-exact, while every wave-instruction still moves 1 KiB contiguous.
#include "gsky_device.h"
#include "drill.h"

namespace gsky {

constexpr int kDrillBatch = 32;

// One time slice per lane (n_bands lanes per polygon): each wave-instruction
// reads 256 contiguous bytes of a pixel's time vector.  The polygon window is
// walked as its flattened row-major pixel sequence -- the reference order of
// drill.go:153-170 -- in batches of 32 pixels; the batch's 32 mask bytes are
// two 16-B words (masks are 16-B aligned and padded, pack_masks) fetched one
// batch ahead, so each batch costs one memory round trip, and every lane
// issues its 32 loads branch-free.  Lane sums stay sequential float32, so the
// means are bit-exact.
__global__ __launch_bounds__(128) void drill_kernel(const float *__restrict__ stack, int xsize, int ysize,
                                                    int n_bands, int t_stride,
                                                    const int32_t *__restrict__ win,
                                                    const int64_t *__restrict__ mask_off,
                                                    const uint8_t *__restrict__ masks, int n_polys,
                                                    float nodata, float lo, float hi, int pixel_count,
                                                    double *__restrict__ band_value,
                                                    int32_t *__restrict__ band_count) {
  const int p = blockIdx.x;
  if (p >= n_polys) return;
  const int t0 = blockIdx.y * blockDim.x + threadIdx.x;
  const int offX = win[4 * p], offY = win[4 * p + 1], cx = win[4 * p + 2], cy = win[4 * p + 3];
  const uint8_t *m = masks + mask_off[p];
  const bool active = t0 < n_bands;
  const long npx = (long)cx * cy;
  float sum = 0.f;
  int32_t total = 0;
  const float *base = stack + t0;
  const uint4 zero4 = make_uint4(0u, 0u, 0u, 0u);
  uint4 mw0 = npx > 0 ? *(const uint4 *)m : zero4;
  uint4 mw1 = npx > 16 ? *(const uint4 *)(m + 16) : zero4;
  int iy = 0, ix = 0;
  for (long i0 = 0; i0 < npx; i0 += kDrillBatch) {
    const uint4 nw0 = (i0 + 32 < npx) ? *(const uint4 *)(m + i0 + 32) : zero4;
    const uint4 nw1 = (i0 + 48 < npx) ? *(const uint4 *)(m + i0 + 48) : zero4;
    const uint32_t mw[8] = {mw0.x, mw0.y, mw0.z, mw0.w, mw1.x, mw1.y, mw1.z, mw1.w};
    float x[kDrillBatch];
    bool use[kDrillBatch];
    long rowbase = ((long)(offY + iy) * xsize + offX) * t_stride;
#pragma unroll
    for (int k = 0; k < kDrillBatch; k++) {
      use[k] = (i0 + k < npx) && ((mw[k >> 2] >> (8 * (k & 3))) & 0xFFu) == 0xFFu;
      const bool ok = use[k] && active;
      const float *src = base + rowbase + (long)ix * t_stride;
      const float v = *(ok ? src : stack);
      x[k] = ok ? v : 0.f;
      if (++ix == cx) {
        ix = 0;
        iy++;
        rowbase = ((long)(offY + iy) * xsize + offX) * t_stride;
      }
    }
#pragma unroll
    for (int k = 0; k < kDrillBatch; k++) {
      if (!use[k]) continue;
      const float val = x[k];
      if (val == nodata) continue;
      if (pixel_count != 0) total++;
      if (val < lo || val > hi) continue;
      if (pixel_count == 0) {
        sum += val;
        total++;
      } else {
        sum += 1.0f;
      }
    }
    mw0 = nw0;
    mw1 = nw1;
  }
  (void)ysize;
  if (!active) return;
  const long o = (long)p * n_bands + t0;
  if (total > 0) {
    band_value[o] = (double)(sum / (float)total);  // drill.go:172-174
    band_count[o] = total;
  } else {
    band_value[o] = 0.0;
    band_count[o] = 0;
  }
}

// bandStrides output rows (drill.go:128-219) from per-band results.
__global__ void drill_rows_kernel(const double *band_value, const int32_t *band_count, int n_polys,
                                  int n_bands, int band_strides, int rows_per_poly, double *out_value,
                                  int32_t *out_count) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n_polys) return;
  const double *bv = band_value + (long)p * n_bands;
  const int32_t *bc = band_count + (long)p * n_bands;
  double *ov = out_value + (long)p * rows_per_poly;
  int32_t *oc = out_count + (long)p * rows_per_poly;
  int nrow = 0;
  for (int ibBgn = 0; ibBgn < n_bands; ibBgn += band_strides) {
    int ibEnd = ibBgn + band_strides;
    if (ibEnd > n_bands) ibEnd = n_bands;
    const int b0 = ibBgn, b1 = ibEnd - 1;
    const int eff = band_strides == 1 ? 1 : 2;
    ov[nrow] = bv[b0]; oc[nrow] = bc[b0]; nrow++;
    if (band_strides > 2 && eff > 1) {
      const double beta = (bv[b1] - bv[b0]) / (double)(band_strides - 1);
      const double cnt = round((double)(bc[b0] + bc[b1]) / 2.0);  // math.Round: half away from zero
      for (int ip = 1; ip < band_strides - 1; ip++) {
        ov[nrow] = bv[b0] + (double)ip * beta;
        oc[nrow] = (int32_t)cnt;
        nrow++;
      }
    }
    if (eff > 1) { ov[nrow] = bv[b1]; oc[nrow] = bc[b1]; nrow++; }
  }
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

int drill_rows_per_poly(int n_bands, int band_strides) {
  if (band_strides <= 0) band_strides = 1;
  int nrow = 0;
  for (int ibBgn = 0; ibBgn < n_bands; ibBgn += band_strides) {
    nrow++;
    if (band_strides > 2) nrow += band_strides - 2;
    if (band_strides > 1) nrow++;
  }
  return nrow;
}

int launch_drill(const float *stack, int xsize, int ysize, int n_bands, int t_stride, const int32_t *win,
                 const int64_t *mask_off, const uint8_t *masks, int n_polys, float nodata, float lo,
                 float hi, int pixel_count, int band_strides, double *out_value, int32_t *out_count,
                 hipStream_t stream) {
  if (band_strides <= 0) band_strides = 1;
  if (n_polys <= 0) return 0;
  if (t_stride % 4 != 0 || t_stride < n_bands) return GSKYHIP_E_ARG;
  if (((uintptr_t)masks & 15u) != 0) return GSKYHIP_E_ARG;   // 16-B mask words
  double *bv = out_value;
  int32_t *bc = out_count;
  const bool direct = band_strides == 1;
  if (!direct) {
    if (hipMallocAsync((void **)&bv, sizeof(double) * (size_t)n_polys * n_bands, stream) != hipSuccess)
      return GSKYHIP_E_HIP;
    if (hipMallocAsync((void **)&bc, sizeof(int32_t) * (size_t)n_polys * n_bands, stream) != hipSuccess)
      return GSKYHIP_E_HIP;
  }
  // one time slice per lane: n_bands lanes per polygon (C4: 3 x 2 waves)
  dim3 grid(n_polys, (n_bands + 127) / 128);
  hipLaunchKernelGGL(drill_kernel, grid, dim3(128), 0, stream, stack, xsize, ysize, n_bands, t_stride,
                     win, mask_off, masks, n_polys, nodata, lo, hi, pixel_count, bv, bc);
  if (!direct) {
    const int rows = drill_rows_per_poly(n_bands, band_strides);
    hipLaunchKernelGGL(drill_rows_kernel, dim3((n_polys + 127) / 128), dim3(128), 0, stream, bv, bc,
                       n_polys, n_bands, band_strides, rows, out_value, out_count);
    hipFreeAsync(bv, stream);
    hipFreeAsync(bc, stream);
  }
  return hipGetLastError() == hipSuccess ? 0 : GSKYHIP_E_HIP;
}

int launch_drill_merge(const double *values, const int32_t *counts, int n_files, int n_dates, double *out,
                       hipStream_t stream) {
  if (n_dates <= 0) return 0;
  hipLaunchKernelGGL(drill_merge_kernel, dim3((n_dates + 255) / 256), dim3(256), 0, stream, values,
                     counts, n_files, n_dates, out);
  return hipGetLastError() == hipSuccess ? 0 : GSKYHIP_E_HIP;
}

}  // namespace gsky
