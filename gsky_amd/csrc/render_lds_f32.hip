// render_lds_f32.hip -- render_lds_kernel<float> (one TU per value type).
#include "render_lds.h"

namespace gsky {
void launch_lds_f32(const RenderArgs &a, bool mask, int n_items, hipStream_t s) {
  launch_lds_t<float>(a, mask, n_items, s);
}
}  // namespace gsky
