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
// bytesRead of the drop-in for the pairs of a planned call, job k = pair k
// (one request each): stats[4k + 2] receives it.  `jobs` (device) give each
// job's block size, its bitmap words and its xsrc / bitmap regions (byte
// offsets into `scratch`, 4-byte aligned, xsrc max_px words); max_px bounds
// every pair's window (w * h).
struct BlockStatsJob {
  int32_t bx, by, n_words, _pad;
  int64_t xsrc_off, bits_off;
};
int launch_block_stats_batch(const RenderCall &c, const BlockStatsJob *jobs, int n_jobs, int64_t max_px,
                             void *scratch, int32_t *stats);

// Per pair of a planned batch: granule, picked level (x, y), element bytes,
// source footprint [x0, y0, x1, y1) at that level (8 int32 per pair, device).
int launch_pair_footprint(void *workspace, int n_tiles, int n_pairs, int max_h, int32_t *out, hipStream_t s);
int launch_pair_touched(void *workspace, int n_tiles, int n_pairs, int max_h, int64_t *out2, hipStream_t s);

// One reply of a warp batch (warp_operation_fast's outputs but the window).
struct WarpResult {
  int32_t bbox[4];
  int32_t dtype, bytes_read;
  double nodata;
  double src_gt[6];
};
// The service's warp batch: plan, then per job (= pair, one request each)
// the window into outs[job] (device addresses: staging or registered host
// memory) with its bytesRead inputs in the same pass, then results[job].
// max_px bounds every pair's window (w * h).  3 launches after planning.
int launch_warp_jobs(const RenderCall &c, const BlockStatsJob *jobs, int64_t max_px, void *scratch,
                     int32_t *stats, uint8_t *const *outs, WarpResult *results);

}  // namespace gsky
