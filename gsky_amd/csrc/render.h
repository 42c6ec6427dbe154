// render.h -- host launchers of render.hip (batched GetMap path).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/gskyhip.h"

namespace gsky {

struct MaskSpecS;

int64_t render_counters_offset(int n_tiles, int n_pairs, int max_h);   // plan counters in the workspace
int64_t render_workspace_size(int n_tiles, int n_pairs, int max_h);

// Shared planning: pairs, tiles, rows.  Returns 0 or an error.
struct RenderCall {
  const gskyhip_granule *granules; int n_granules;
  const gskyhip_crs *crs; int n_crs; int dst_crs;
  const gskyhip_tile *tiles; int n_tiles;
  const int32_t *pair_granule; int n_pairs;
  int max_w, max_h;
  int mask_ns, mask_inclusive;
  const MaskSpecS *mask_specs;  // 4 entries (host)
  int resample;
  uint32_t value_types;         // GSKYHIP_VT_* of the stack entries (0 = unknown)
  const int64_t *cov_offsets;   // canvases placed in one image: per tile element offset (dev) or NULL
  int64_t cov_stride;           // that image's row stride in elements
  void *workspace; int64_t workspace_bytes;
  hipStream_t stream;
  const GeoLocD *geolocs = nullptr;   // geolocation transformers of the granules (dev), or NULL
};

int launch_render(const RenderCall &c, const int32_t *out_ns, int n_out, const gskyhip_scale_params &sp,
                  const uint8_t *ramp, uint8_t *rgba_out, void *canvas_out, int phase);
int launch_extent(const gskyhip_granule *granules, int n, const gskyhip_crs *crs, int dst_crs, const double *bbox,
                  int32_t *out, int32_t *status, hipStream_t s);
int launch_warp_windows(const RenderCall &c, int32_t *bbox_out, int32_t *dtype_out, double *nodata_out,
                        void *win_out, int64_t win_stride);
// bytesRead of the drop-in (pair `pair` of a planned call): stats[2] receives it.
int64_t block_stats_scratch_bytes(int64_t n_px, int64_t n_words);
int launch_block_stats(const RenderCall &c, int pair, int bx, int by, void *scratch, int64_t n_px,
                       int64_t n_words, int32_t *stats);

}  // namespace gsky
