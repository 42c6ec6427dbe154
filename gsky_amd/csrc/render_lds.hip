// render_lds.hip -- dispatch of the typed LDS-staged band kernels.
#include <cstdlib>

#include "render_lds.h"

namespace gsky {

void launch_lds_kernels(const RenderArgs &a0, int vt, bool mask, int n_items, hipStream_t s) {
  // GSKYHIP_LDS_STAGE=1 stages the source windows in LDS; the default gathers
  // from HBM, measured faster on C2 and C5 (profiles/r02_ab_*.jsonl).  Results
  // are identical either way.
  RenderArgs a = a0;
  const char *st = getenv("GSKYHIP_LDS_STAGE");
  a.lds_stage = st ? atoi(st) : 0;
  const char *fl = getenv("GSKYHIP_LDS_FLAGS");
  a.lds_flags = fl ? atoi(fl) : 0;
  switch (vt) {
    case GSKYHIP_INT16: launch_lds_i16(a, mask, n_items, s); break;
    case GSKYHIP_UINT16: launch_lds_u16(a, mask, n_items, s); break;
    case GSKYHIP_FLOAT32: launch_lds_f32(a, mask, n_items, s); break;
    case GSKYHIP_SIGNEDBYTE: launch_lds_i8(a, mask, n_items, s); break;
    default: launch_lds_u8(a, mask, n_items, s); break;
  }
}

}  // namespace gsky
