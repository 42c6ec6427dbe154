// stages.h -- shared host/device structs of the standalone stage kernels.
#pragma once
#include "gsky_device.h"

namespace gsky {

// Go strconv-parsed mask spec for one mask raster dtype (tile_merger.go:332-431).
struct MaskSpecS {
  int32_t has_value;
  int32_t n_tests;
  int32_t value;
  int32_t filt[GSKYHIP_MAX_BIT_TESTS / 2 + 1];
  int32_t want[GSKYHIP_MAX_BIT_TESTS / 2 + 1];
};

// One merge entry in ProcessRasterStack order.
struct FlexEntry {
  const void *data;
  int32_t data_w, data_h, off_x, off_y;
  int32_t dtype, fill_mode;
  double nodata;
  const void *mask_data;   // data of the mask raster (maskMap[geoStamp]) or NULL
  int32_t mask_dtype, _pad;
  int64_t mask_len;
};

// Scale constants (raster_scaler.go:30-78).
struct ScaleC {
  int32_t dtype;
  int32_t colour_scale;
  Val noData, off, clp;
  float sc;
  double nodata64;
};

__global__ void merge_fold_kernel(const FlexEntry *e, int n, int width, int height, int canvas_dtype,
                                  double canvas_nodata, MaskSpecS ms, void *canvas);
__global__ void compute_mask_kernel(const void *data, int dtype, long n, MaskSpecS ms, uint8_t *out);
__global__ void scale_minmax_kernel(const void *data, int dtype, long n, double nodata,
                                    int colour_scale, int32_t *mm);
__global__ void scale_finalize_kernel(ScaleC *k, const int32_t *mm, int autom);
__global__ void scale_apply_kernel(void *data, int dtype, long n, const ScaleC *kp, uint8_t *out,
                                   int inplace_byte);
__global__ void scale_legacy_kernel(void *data, int dtype, long n, double nodata, double offset,
                                    double scale, double clip, uint8_t *out);
__global__ void encode_rgba_kernel(const uint8_t *b0, const uint8_t *b1, const uint8_t *b2,
                                   int nbands, long npx, const uint32_t *ramp, uint32_t *rgba);

}  // namespace gsky

namespace gsky {
// host launchers (stages.hip)
int launch_merge_fold(const FlexEntry *entries_host, int n, int width, int height, int canvas_dtype,
                      double canvas_nodata, const MaskSpecS &ms, void *canvas, hipStream_t s);
int launch_compute_mask(const void *data, int dtype, int64_t n, const MaskSpecS &ms, uint8_t *out,
                        hipStream_t s);
int launch_scale(void *data, int dtype, int64_t n, double nodata, const gskyhip_scale_params &sp,
                 uint8_t *out, hipStream_t s);
int launch_scale_legacy(void *data, int dtype, int64_t n, double nodata, const gskyhip_scale_params &sp,
                        uint8_t *out, hipStream_t s);
int launch_encode_rgba(const uint8_t *b0, const uint8_t *b1, const uint8_t *b2, int nbands, int64_t npx,
                       const uint8_t *ramp, uint8_t *rgba, hipStream_t s);
ScaleC host_scale_consts(int dtype, double nodata, const gskyhip_scale_params &sp);
}  // namespace gsky
