// service.h -- the per-node GPU warp service (SURVEY.md 8b "preferred
// design", 8f row 1).
//
// The reference serves warps from N = NumCPU single-threaded gsky-gdal-process
// workers per node (grpc-server/main.go:58; gdal-process/main.go:115-123),
// each killed after 120 s or max_tasks (gdal-process/main.go:57-68,
// process.go:154-158).  N processes each opening a HIP context on the same GPU
// would multiply contexts and serialise on the device; instead one daemon per
// GPU (gskyhipd, gskyhip_service_run) owns the context, the HBM-resident
// granules and the streams.  Workers keep calling warp_operation_fast; with
// GSKYHIP_SERVICE=<socket> set, the drop-in forwards the request over a Unix
// socket and never touches the GPU, so a SIGKILLed worker leaves no device
// state behind.  The daemon batches the warps that arrive within its window
// from all workers into one plan + warp launch set (warp_batch.h).
//
// Wire: every message is [u32 magic 'GSKY'][u32 op][u64 payload bytes][payload];
// the reply to each request has the same framing.
#pragma once
#include <stdint.h>

#include "warp_batch.h"

namespace gsky {

constexpr uint32_t kSvcMagic = 0x594B5347u;   // "GSKY"
// SVC_WARP_SHM: a warp whose window comes back in the worker's reply arena
// (a sealed memfd passed with SCM_RIGHTS on the first request of a
// connection, or when it grows); SVC_WARP carries the window in the socket.
enum SvcOp : uint32_t {
  SVC_WARP = 1, SVC_REGISTER = 2, SVC_UNREGISTER_ALL = 3, SVC_STATS = 4, SVC_SHUTDOWN = 5, SVC_WARP_SHM = 6
};

// Forward one request to the service at `sock`; 0, or GSKYHIP_E_SERVICE when
// the service cannot be reached (the worker reports the failure and the OWS
// retries, process.go:147-150).  The thread keeps its connection for the next
// request (a fresh one after fork or a broken pipe).  With `mbuf`, the window
// bytes are received straight into malloc'd memory (*mbuf, *mlen; the caller
// frees it, as warp.go:573-574 frees the worker's buffer) and r.data stays
// empty.
int service_warp(const char *sock, const WarpReq &q, WarpResp &r, void **mbuf = nullptr, size_t *mlen = nullptr);

}  // namespace gsky
