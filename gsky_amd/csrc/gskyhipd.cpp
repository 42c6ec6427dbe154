// gskyhipd -- the per-node GPU warp service (one per GPU; pick it with
// HIP_VISIBLE_DEVICES).  usage: gskyhipd <socket> [max_batch=64] [window_us=0]
// Workers reach it through GSKYHIP_SERVICE=<socket> (include/gskyhip.h).
#include <cstdio>
#include <cstdlib>

#include "../../include/gskyhip.h"

int main(int argc, char **argv) {
  if (argc < 2) {
    std::fprintf(stderr, "usage: %s <socket> [max_batch] [window_us]\n", argv[0]);
    return 2;
  }
  const int max_batch = argc > 2 ? std::atoi(argv[2]) : 64;
  const int window_us = argc > 3 ? std::atoi(argv[3]) : 0;
  const int rc = gskyhip_service_run(argv[1], max_batch, window_us);
  if (rc) std::fprintf(stderr, "gskyhipd: %s: error %d\n", argv[1], rc);
  return rc ? 1 : 0;
}
