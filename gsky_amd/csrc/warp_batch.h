// warp_batch.h -- warp_operation_fast (worker/gdalprocess/warp.go:82-382) as
// a batch: n independent requests (each one (tile, granule) pair) planned and
// warped in ONE set of launches.  The C-ABI drop-in calls it with n = 1; the
// per-node service (service.cpp) with every request that arrived from the N
// worker processes within its batching window.
#pragma once
#include <stdint.h>

#include <string>
#include <vector>

namespace gsky {

// One warp_operation_fast call, by value (the strings and geotransforms the
// caller owns are copied).
struct WarpReq {
  std::string path;
  int32_t band = 1;
  int32_t has_src_srs = 0, has_src_gt = 0, geoloc = 0, has_dst_srs = 0;
  std::string src_srs, dst_srs;
  double src_gt[6] = {0, 0, 0, 0, 0, 0};
  double dst_gt[6] = {0, 0, 0, 0, 0, 0};
  int32_t width = 0, height = 0, srs_cf = 0;
  std::vector<std::string> geoloc_opts;   // GeoLocOpts "KEY=VALUE" strings (geoloc != 0)
};

// Its outputs: return code (0, 1 open failed, 2 band failed, 3 transformer
// failed, or a GSKYHIP_E_* code), window bbox / nodata / dtype / bytesRead,
// the overview-rescaled source geotransform (warp.go:186-189) and the window
// bytes (bbox[2] x bbox[3] values of dtype).
struct WarpResp {
  int32_t rc = 0;
  int32_t bbox[4] = {0, 0, 0, 0};
  double nodata = 0;
  int32_t dtype = 0;
  int32_t bytes_read = 0;
  double src_gt[6] = {0, 0, 0, 0, 0, 0};
  std::vector<char> data;
  int64_t in_place = -1;   // >= 0: the window (this many bytes) was written to the caller's destination
};

// Runs the batch against this process's granule registry (HBM-resident,
// gskyhip_register_granule) and waits for it.  Thread-safe (one batch at a
// time).
void warp_batch(const WarpReq *reqs, int n, WarpResp *out);

// The same in two halves, for a caller that keeps several batches in flight
// (the service, service.cpp): a slot holds one batch's buffers, stream and
// completion event.  warp_batch_launch does the registry lookups (requests
// that fail early get their rc at once), uploads the headers and queues every
// launch and the reply read-back on the slot's stream without waiting;
// warp_batch_finish waits for the slot and fills `out` (the array given to
// launch, which must live until then).  Request i's window is written to
// direct[i] -- a device-visible address with direct_cap[i] >= width * height
// * 8 bytes, e.g. host memory registered with HIP -- and out[i].in_place set;
// without one it lands in out[i].data.  The granules a batch reads stay
// allocated until its finish.  Different slots may be in flight together.
struct WarpSlot;
WarpSlot *warp_slot_create();
void warp_slot_destroy(WarpSlot *s);   // finishes a batch still in flight
void warp_batch_launch(WarpSlot &s, const WarpReq *reqs, int n, WarpResp *out, uint8_t *const *direct,
                       const int64_t *direct_cap);
void warp_batch_finish(WarpSlot &s);

// Nanoseconds this process spent in warp batches by phase, summed over calls:
// [0] launch (registry, SRS parsing, headers, launches queued), [1] waiting
// for the GPU in finish, [2] staged window read-back into the responses and
// release, [3] batches.
void warp_batch_timers(int64_t out[4]);

}  // namespace gsky
