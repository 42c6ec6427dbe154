// render_lds_u8.hip -- band kernels of uint8_t (one TU per value type).
#include "render_nn_stage.h"

namespace gsky {
void launch_lds_u8(const RenderArgs &a, bool mask, int n_items, hipStream_t s) {
  launch_band_t<uint8_t>(a, mask, n_items, s);
}
}  // namespace gsky
