// render_lds_u16.hip -- render_lds_kernel<uint16_t> (one TU per value type).
#include "render_lds.h"

namespace gsky {
void launch_lds_u16(const RenderArgs &a, bool mask, int n_items, hipStream_t s) {
  launch_lds_t<uint16_t>(a, mask, n_items, s);
}
}  // namespace gsky
