// drill.h -- host launchers of drill.hip.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace gsky {
int drill_rows_per_poly(int n_bands, int band_strides);
int launch_drill(const float *stack, int xsize, int ysize, int n_bands, int t_stride, const int32_t *win,
                 const int64_t *mask_off, const uint8_t *masks, int n_polys, float nodata, float lo,
                 float hi, int pixel_count, int band_strides, double *out_value, int32_t *out_count,
                 hipStream_t stream);
int launch_drill_merge(const double *values, const int32_t *counts, int n_files, int n_dates, double *out,
                       hipStream_t stream);
}  // namespace gsky
