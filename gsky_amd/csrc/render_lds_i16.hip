// render_lds_i16.hip -- render_lds_kernel<int16_t> (one TU per value type).
#include "render_lds.h"

namespace gsky {
void launch_lds_i16(const RenderArgs &a, bool mask, int n_items, hipStream_t s) {
  launch_lds_t<int16_t>(a, mask, n_items, s);
}
}  // namespace gsky
